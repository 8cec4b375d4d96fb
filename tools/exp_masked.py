"""Sparse-input hops on G100M: dense vs masked (zero-row mask + activity mask), for the
backward of a BPR batch (2048 users + 2048 positives + 2048 negatives non-zero)."""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
import bench  # noqa: E402
from src.ops import _lib, functional as F  # noqa: E402


def t_ms(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


dev = torch.device("cuda", 0)
g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
n = g.shape[0]
gen = torch.Generator(device=dev).manual_seed(0)
grad = torch.zeros(n, 64, device=dev)
rows = torch.cat([torch.randint(0, 1_000_000, (2048,), device=dev, generator=gen),
                  1_000_000 + torch.randint(0, 1_000_000, (4096,), device=dev, generator=gen)])
grad[rows] = torch.randn(rows.numel(), 64, device=dev, generator=gen)
h1 = torch.empty_like(grad)
F.spmm_into(g, grad, h1)
res = {"hop1_input_nonzero_rows": int(F.row_nonzero(grad).sum()),
       "hop2_input_nonzero_rows": int(F.row_nonzero(h1).sum())}
y = torch.empty_like(grad)


def masked(x):
    xm = F.row_nonzero(x)
    ya = torch.empty(n, dtype=torch.uint8, device=dev)
    _lib.check(_lib.lib().gnnrec_mark_active_rows(_lib.ptr(g.row_ptr), _lib.ptr(g.col), n,
                                                  _lib.ptr(xm), n, _lib.ptr(ya),
                                                  _lib.stream_of(dev)), "mark")
    F.spmm_into(g, x, y, x_mask=xm, y_active=ya)


for name, x in (("hop1", grad), ("hop2", h1)):
    res[f"{name}_dense_ms"] = t_ms(lambda: F.spmm_into(g, x, y))
    res[f"{name}_masked_ms"] = t_ms(lambda: masked(x))
    res[f"{name}_masked_no_active_ms"] = t_ms(lambda: F.spmm_into(g, x, y, x_mask=F.row_nonzero(x)))
out = torch.empty_like(grad)
res["backward_masked1_ms"] = t_ms(lambda: F.lightgcn_backward(g, grad, 3, masked_hops=1))
res["backward_masked2_ms"] = t_ms(lambda: F.lightgcn_backward(g, grad, 3, masked_hops=2))
res["backward_dense_ms"] = t_ms(lambda: F.lightgcn_backward(g, grad, 3, masked_hops=0))
print(json.dumps(res))
