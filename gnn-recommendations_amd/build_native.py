"""Build libgnnrec.so (HIP kernels for gfx950 + native host code) in-tree.

    python gnn-recommendations_amd/build_native.py [--force] [-v]

Objects are compiled in parallel with hipcc and linked into ``lib/libgnnrec.so`` next to
this file, so the library travels with the repository snapshot to the GPU box. A source
is rebuilt only when it (or a header) is newer than its object.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent
CSRC = PKG_ROOT / "csrc"
INCLUDE = PKG_ROOT.parent / "include"
BUILD = PKG_ROOT / "build"
LIB = PKG_ROOT / "lib" / "libgnnrec.so"
VENDOR_SRC = PKG_ROOT / "vendor" / "rocsparse_spmm.cpp"
VENDOR_LIB = PKG_ROOT / "lib" / "libgnnrec_vendor.so"

ARCH = "gfx950"
# fp-contract off: every FMA in the kernels is an explicit fmaf, nothing else may fuse
# (bit-exact parity with the reference CPU path depends on it).
CFLAGS = [
    "-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-ffp-contract=off",
    "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wall", "-Wno-unused-function",
    # compressed code-object bundles (the HIP runtime inflates them at load): the library
    # goes from 9.4 to ~3.5 MB, which every GPU-box push carries
    "--offload-compress",
]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libgnnrec)")


def sources() -> list[Path]:
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.cpp")))


def _headers() -> list[Path]:
    return sorted(list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h")))


def _stale(obj: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> Path:
    hipcc = _hipcc()
    BUILD.mkdir(parents=True, exist_ok=True)
    LIB.parent.mkdir(parents=True, exist_ok=True)
    hdrs = _headers()
    jobs = []
    objs = []
    for src in sources():
        obj = BUILD / (src.name + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs):
            jobs.append([hipcc, *CFLAGS, "-c", str(src), "-o", str(obj)])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r

    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            list(ex.map(run, jobs))
    if force or jobs or _stale(LIB, objs):
        tmp = LIB.with_suffix(".so.tmp")
        run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs),
             "-lpthread"])
        os.replace(tmp, LIB)
    try:
        build_vendor(force=force, verbose=verbose)
    except Exception as e:  # the comparator is bench-only; the product library is built
        print(f"build_native: rocSPARSE comparator not built ({e}); bench.py records it as "
              "unavailable", file=sys.stderr)
    return LIB


def build_vendor(force: bool = False, verbose: bool = False) -> Path:
    """lib/libgnnrec_vendor.so: bench.py's rocSPARSE comparator (vendor/rocsparse_spmm.cpp).
    Host code only, linked against librocsparse; never loaded by the product path."""
    src = VENDOR_SRC
    if not (force or _stale(VENDOR_LIB, [src])):
        return VENDOR_LIB
    tmp = VENDOR_LIB.with_suffix(".so.tmp")
    cmd = [_hipcc(), "-O2", "-fPIC", "-std=c++17", "-shared", "-Wall", str(src), "-o", str(tmp),
           "-L/opt/rocm/lib", "-lrocsparse", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, VENDOR_LIB)
    return VENDOR_LIB


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    print(build(force=a.force, verbose=a.verbose))
    return 0


if __name__ == "__main__":
    sys.exit(main())
