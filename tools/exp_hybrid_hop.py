"""Power-law LightGCN hop: would a hybrid (column-ordered kernel on the rows of at most
TILED_MAX_DEGREE neighbours, the hubs on the heavy-row kernel, in the same hop) beat the CSR
path the whole operand takes today (one row above 4,096 sends every row to it,
functional.tiled_plan_for)? VERDICT r05 item 6; tools/exp_heavy_tiled.py's method: the rows
are cut out by degree as their own CSR (same columns, same x), and each part is timed alone.

    (a) today: F.spmm_into on the whole operand (CSR path: row-parallel + heavy-row kernels)
    (b) the light part (degree <= --cut) as its own operand: the column-ordered kernel
    (c) the hub part (degree > --cut): the heavy-row kernel (every row above the threshold)
    hybrid estimate = (b) + (c), launched back to back (no scatter of the compact outputs,
    so a lower bound of what a built hybrid would cost by the output-row scatter)

    python tools/exp_hybrid_hop.py [--shape 2000000 2000000 50000000] [--cut 4096]
"""
import argparse
import hashlib
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT), str(ROOT / "tools")]
from bench_configs import powerlaw_graph  # noqa: E402
from src.ops import CsrGraph  # noqa: E402
from src.ops import functional as F  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", type=int, nargs=3, default=[2_000_000, 2_000_000, 50_000_000])
ap.add_argument("--cut", type=int, default=F.TILED_MAX_DEGREE)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
dev = torch.device("cuda", 0)
g = powerlaw_graph(*a.shape, 0.9, 0, 16, device=dev)
deg = g.row_ptr[1:] - g.row_ptr[:-1]


def sub_of(keep):
    rows = torch.nonzero(keep).flatten()
    cnt = deg[rows]
    rp = torch.zeros(rows.numel() + 1, dtype=torch.int64, device=dev)
    rp[1:] = torch.cumsum(cnt, 0)
    nnz = int(rp[-1])
    off = torch.repeat_interleave(g.row_ptr[rows] - rp[:-1], cnt)
    idx = torch.arange(nnz, device=dev, dtype=torch.int64) + off
    return rows, CsrGraph(rp, g.col[idx].contiguous(), g.val[idx].contiguous(),
                          (rows.numel(), g.shape[1]))


def ms_of(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(5):
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        out.append(s.elapsed_time(e) / reps)
    return sorted(out)[2]


def sha(t):
    return hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()[:16]


light_rows, light = sub_of(deg <= a.cut)
hub_rows, hubs = sub_of(deg > a.cut)
info = dict(shape=a.shape, nnz=g.nnz, max_degree=int(deg.max()), cut=a.cut,
            light_rows=light.n_rows, light_nnz=light.nnz, hub_rows=hubs.n_rows, hub_nnz=hubs.nnz)
print(json.dumps({"case": "operand", **info}), flush=True)
for d in (64, 128):
    x = F.hop_table(g.shape[1], d, device=dev)
    x.copy_(torch.randn(g.shape[1], d, device=dev,
                        generator=torch.Generator(device=dev).manual_seed(d)) * 0.1)
    y = torch.empty(g.n_rows, d, device=dev)
    yl = torch.empty(light.n_rows, d, device=dev)
    yh = torch.empty(hubs.n_rows, d, device=dev)
    t_full = ms_of(lambda: F.spmm_into(g, x, y), a.reps)
    plan = F.tiled_plan_for(light, x, outputs=(yl,))
    t_light = ms_of(lambda: F.spmm_into(light, x, yl), a.reps)
    t_light_csr = None
    F.TILED_HOP = False
    t_light_csr = ms_of(lambda: F.spmm_into(light, x, yl), a.reps)
    F.TILED_HOP = True
    t_hubs = ms_of(lambda: F.spmm_into(hubs, x, yh, heavy_threshold=min(a.cut, 128)), a.reps)
    # the parts equal the whole operand's rows, bit for bit
    F.spmm_into(light, x, yl)
    F.spmm_into(hubs, x, yh, heavy_threshold=min(a.cut, 128))
    F.spmm_into(g, x, y)
    torch.cuda.synchronize()
    same = bool(torch.equal(y[light_rows], yl)) and bool(torch.equal(y[hub_rows], yh))
    print(json.dumps({"case": "hop", "d": d, "full_csr_ms": t_full,
                      "light_tiled_ms": t_light, "light_is_tiled": plan is not None,
                      "light_csr_ms": t_light_csr, "hubs_heavy_ms": t_hubs,
                      "hybrid_estimate_ms": t_light + t_hubs,
                      "hybrid_vs_full": (t_light + t_hubs) / t_full, "parts_bit_equal": same,
                      "sha_full": sha(y), **info}), flush=True)
    del x, y, yl, yh
    light._plans.clear()
    torch.cuda.empty_cache()
