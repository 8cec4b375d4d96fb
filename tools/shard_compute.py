"""Compute side of the N-GPU LightGCN curve, measured on ONE GPU.

For N in --ns and each rank layout bench.py times at N > 1 — the default grid (F = gcd(N, d/32)
feature groups x R = N/F destination-row shards) and the north star's F = 1 (N row shards) —
this builds every row shard r of the layout in a world-1 process, exactly as rank r's
RankGrid does (CsrGraph.shard: nnz-balanced rows, columns remapped into the padded gather
layout; a d/F-wide padded x table), and times bench.py's step on it with the per-hop exchange
replaced by nothing: the same lightgcn_propagate_dist schedule (deferred layer mean), the same
column-ordered plans, and the overlap-chunk / reserve_cus candidates bench.py tries. What it
reports is each shard's hop-chain time, its max over the shards (what an exchange-free N-GPU
step would cost), and the N = 1 hop / N beside it. Not a scaling run: no RCCL, no xGMI.

    python tools/shard_compute.py [--ns 2 4 8] [--dim 64] [--steps 5] > profiles/r06/shard_compute.jsonl
"""
import argparse
import json
import math
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
import bench  # noqa: E402
from src.ops import functional as F  # noqa: E402
from src.ops.distributed import DistributedGraph, lightgcn_propagate_dist, make_work  # noqa: E402


def emit(**kw):
    print(json.dumps(kw), flush=True)


def shard_dg(full, r, R, device):
    """Rank r's DistributedGraph of an R-way row sharding, built without a process group:
    CsrGraph.shard does the layout; the exchange is a no-op (every gathered table keeps the
    values it has — the kernels' time does not depend on them)."""
    dg = DistributedGraph.__new__(DistributedGraph)
    dg.rank, dg.world, dg.group = r, R, None
    dg.ranks = list(range(R))
    dg.device = torch.device(device)
    dg.shard = full.shard(r, R).to(dg.device)
    info = dg.shard.shard_info
    dg.bounds, dg.rows_pad = info.bounds, info.rows_pad
    dg.row_begin, dg.row_end = info.row_begin, info.row_end
    dg.n_local = dg.row_end - dg.row_begin
    dg.n_global = full.shape[0]
    dg.needs = torch.ones((R, R), dtype=torch.bool)
    dg.exchange_mode = "p2p"
    dg.exchange = lambda out, piece: None
    dg.post_chunk = lambda out, piece, c0, c1: []
    dg.finish = lambda pending: None
    return dg


def time_chain(dg, x_pad, K, chunks, reserve, steps):
    timer = bench.HopTimer()
    work = make_work(dg, x_pad.shape[1], x_pad.device)

    def step():
        return lightgcn_propagate_dist(dg, x_pad, K, hop_fn=timer.hop, work=work,
                                       overlap_chunks=chunks, reserve_cus=reserve,
                                       placed_output=True)
    step()
    torch.cuda.synchronize()
    timer.reset(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ms_step = (time.perf_counter() - t0) / steps * 1e3
    durs = timer.durations_ms()
    timer.reset(False)
    return ms_step, float(np.sum(durs)) / (steps * K)


def main():
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--ns", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    full = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, bench.host_threads())
    assert full.nnz == bench.G100M_NNZ
    N, d, K = full.shape[0], a.dim, a.layers
    torch.manual_seed(0)
    x0 = torch.randn(N, d, dtype=torch.float32) * 0.1

    # N = 1: the headline step itself (one shard = the whole operand)
    dg1 = shard_dg(full, 0, 1, device)
    x1 = dg1.pad_table(x0, hop_layout=True)
    ms1, hop1 = time_chain(dg1, x1, K, 1, 0, a.steps)
    emit(n=1, layout="F1xR1", rank=0, nnz=dg1.shard.nnz, rows=dg1.n_local, d_loc=d,
         chunks=1, reserve_cus=0, ms_per_step=ms1, compute_ms_per_hop=hop1,
         tiled=F.tiled_plan_for(dg1.shard, x1) is not None)
    del dg1, x1
    summary = []
    for n in a.ns:
        f_def = math.gcd(n, d // 32) if d % 32 == 0 else 1
        for fg in sorted({f_def, 1}, reverse=True):
            R = n // fg
            d_loc = d // fg
            cands = [(1, 0)] if R == 1 else [(1, 0), (4, 0), (8, 0), (4, 16), (8, 16)]
            worst = {}
            for r in range(R):
                dg = shard_dg(full, r, R, device)
                xs = torch.randn(R * dg.rows_pad, d_loc, device=device,
                                 generator=torch.Generator(device=device).manual_seed(r)) * 0.1
                xs = dg.pad_table(x0[:, :d_loc].contiguous(), hop_layout=True) if R == 1 else xs
                tiled = F.tiled_plan_for(dg.shard, xs) is not None
                for chunks, reserve in cands:
                    ms, hop = time_chain(dg, xs, K, chunks, reserve, a.steps)
                    emit(n=n, layout=f"F{fg}xR{R}", rank=r, nnz=dg.shard.nnz, rows=dg.n_local,
                         d_loc=d_loc, chunks=chunks, reserve_cus=reserve, ms_per_step=ms,
                         compute_ms_per_hop=hop, tiled=tiled)
                    key = (chunks, reserve)
                    worst[key] = max(worst.get(key, (0.0, 0.0)), (hop, ms))
                dg.shard._plans.clear()
                del dg, xs
                torch.cuda.empty_cache()
            for (chunks, reserve), (hop, ms) in sorted(worst.items()):
                row = dict(n=n, layout=f"F{fg}xR{R}", chunks=chunks, reserve_cus=reserve,
                           max_compute_ms_per_hop=hop, max_ms_per_step=ms,
                           n1_hop_over_n=hop1 / n, ratio_to_ideal=hop / (hop1 / n),
                           exchange_free_edges_per_s=K * full.nnz / (ms * 1e-3))
                summary.append(row)
                emit(summary=True, **row)
    return 0


if __name__ == "__main__":
    sys.exit(main())
