"""Why is the G100M d = 64 hop slower inside config 3 (NGCF + GAS) than alone? The same hop
(column-ordered, factored plan, x a column block of a [N, 256] table, compact output) is
timed with HIP events after different preceding kernels on the same stream:
  none  hop after hop (the LightGCN pattern)
  tf    hop after the NGCF+GAS streaming transform (the config-3 pattern)
  mm    hop after a dense fp32 GEMM of about the transform's length (matrix cores busy)
  copy  hop after a 512 MB device copy (HBM busy, no matrix cores)
  idle  hop after ~0.5 ms of an idle GPU (torch.cuda._sleep)
One JSON line per pattern: median / min hop ms over 12 timed hops."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
import bench  # noqa: E402
from src.ops import _lib  # noqa: E402
from src.ops import functional as F  # noqa: E402
from src.ops._lib import check, ptr  # noqa: E402

dev = torch.device("cuda", 0)
gen = torch.Generator(dev).manual_seed(0)
g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
n, d = g.shape[0], 64
T = torch.randn(n, 4 * d, device=dev, generator=gen) * 0.1
x, y = T[:, :d], T[:, d:2 * d]
work = torch.empty(n, d, device=dev)
W1, W2 = (torch.randn(d, d, device=dev, generator=gen) * 0.1 for _ in range(2))
b1, b2 = torch.zeros(d, device=dev), torch.zeros(d, device=dev)
blocks = torch.randn(d // 8, 8, 8, device=dev, generator=gen)
perm = torch.randperm(d, device=dev, generator=gen).to(torch.int32)
A = torch.randn(2048, 4096, device=dev, generator=gen)
B = torch.randn(4096, 4096, device=dev, generator=gen)
C = torch.empty(2048, 4096, device=dev)
src = torch.randn(n, d, device=dev, generator=gen)
dst = torch.empty(n, d, device=dev)
plan = F.tiled_plan_for(g, x)
assert plan is not None
L = _lib.lib()
st = _lib.stream_of(dev)


def hop():
    F.spmm_tiled_into(g, x, work, plan)


def tf():
    check(L.gnnrec_ngcf_transform_f32(n, ptr(work), d, ptr(x), x.stride(0), ptr(y), y.stride(0),
                                      d, ptr(W1), ptr(b1), ptr(W2), ptr(b2), 0.2, ptr(blocks),
                                      ptr(perm), 8, st), "transform")


def mm():
    torch.mm(A, B, out=C)


def copy():
    dst.copy_(src)


def idle():
    torch.cuda._sleep(1_000_000)


def ev_ms(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    fn()
    e.record()
    return s, e


pre = {"none": None, "tf": tf, "mm": mm, "copy": copy, "idle": idle}
for _ in range(3):
    hop()
for name, fn in pre.items():
    hops, others = [], []
    for it in range(14):
        if fn is not None:
            others.append(ev_ms(fn))
        hops.append(ev_ms(hop))
    torch.cuda.synchronize()
    hm = [s.elapsed_time(e) for s, e in hops[2:]]
    om = [s.elapsed_time(e) for s, e in others[2:]]
    print(json.dumps({"pattern": name, "hop_ms_median": float(np.median(hm)),
                      "hop_ms_min": float(np.min(hm)),
                      "preceding_ms_median": float(np.median(om)) if om else None,
                      "hop_ms": hm}), flush=True)
