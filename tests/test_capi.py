"""The C ABI from plain C (no PyTorch, no C++): tests/capi/capi_lightgcn.c compiles against
include/gnnrec.h with gcc here (the header is valid C and self-contained), and on the GPU it
runs the builders and the propagation through hipMalloc'd buffers, bit-identical to the
oracle."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
LIBDIR = ROOT / "gnn-recommendations_amd" / "lib"


def _compile(out: Path) -> None:
    gcc = shutil.which("gcc")
    if gcc is None or not Path("/opt/rocm/include/hip/hip_runtime_api.h").exists():
        pytest.skip("gcc or the ROCm headers are missing")
    if not (LIBDIR / "libgnnrec.so").exists():
        pytest.skip("libgnnrec.so not built")
    cmd = [gcc, "-std=c11", "-O2", "-ffp-contract=off", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
           "-I/opt/rocm/include", f"-I{ROOT / 'include'}", str(ROOT / "tests/capi/capi_lightgcn.c"),
           str(ROOT / "oracle/oracle.c"), f"-L{LIBDIR}", "-lgnnrec", "-L/opt/rocm/lib",
           "-lamdhip64", "-lm", f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath,/opt/rocm/lib",
           "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_capi_client_compiles_as_c(tmp_path):
    _compile(tmp_path / "capi")


@pytest.mark.gpu
def test_capi_client_runs_bit_exact(tmp_path, cuda):
    exe = tmp_path / "capi"
    _compile(exe)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK:" in r.stdout
