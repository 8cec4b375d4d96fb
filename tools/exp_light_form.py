"""The row-parallel chain's two forms on large operands (the CSR path, column-ordered hop
off): K = 3 LightGCN propagation at d = 64 with GNNREC_CSR_LIGHT_LATENCY (16 lanes x float4
per row, the next step's indices one step ahead) against _THROUGHPUT (a wave per row), on
uniform 1M x 1M graphs of several average degrees and the power-law 2M x 2M operand. Output
hashes must agree between the forms.

    python tools/exp_light_form.py
"""
import hashlib
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT), str(ROOT / "tools")]
import bench  # noqa: E402
from bench_configs import powerlaw_graph  # noqa: E402
from src.ops import _lib  # noqa: E402
from src.ops import functional as F  # noqa: E402

dev = torch.device("cuda", 0)
F.TILED_HOP = False


def ms_of(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(3):
        s.record()
        for _ in range(reps):
            out = fn()
        e.record()
        e.synchronize()
        best.append(s.elapsed_time(e) / reps)
    return sorted(best)[1], out


graphs = [(f"uniform_1Mx1M_{p // 1_000_000}M", lambda p=p: bench.build_graph(1_000_000, 1_000_000, p, 0, 16))
          for p in (10_000_000, 25_000_000, 50_000_000, 100_000_000)]
graphs.append(("powerlaw_2Mx2M_50M", lambda: powerlaw_graph(2_000_000, 2_000_000, 50_000_000, 0.9, 0)))
for name, make in graphs:
    g = make().to(dev)
    x = torch.randn(g.shape[1], 64, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
    rec = {"graph": name, "n_rows": g.n_rows, "nnz": g.nnz, "avg_degree": g.nnz / g.n_rows,
           "max_degree": g.max_degree()}
    hashes = set()
    for form, fl in (("throughput", _lib.CSR_LIGHT_THROUGHPUT), ("latency", _lib.CSR_LIGHT_LATENCY)):
        F.CSR_FLAGS = fl
        t, (out, _) = ms_of(lambda: F.lightgcn_forward(g, x, 3))
        rec[f"{form}_ms"] = t
        hashes.add(hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16])
    F.CSR_FLAGS = 0
    rec["same_bits"] = len(hashes) == 1
    print(json.dumps(rec), flush=True)
    del g, x, out
    torch.cuda.empty_cache()
