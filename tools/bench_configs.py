"""Secondary benchmarks: the BASELINE.json configs other than the headline.

    python tools/bench_configs.py [--configs 2 3 4 5] [--steps 10] [--g1b]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P tools/bench_configs.py --gpus N --configs 3 4 5

  2  ML-1M-shaped LightGCN K=3 d=64 (synthetic 6040 x 3706, 1M ratings -> reference
     preprocessing), model-class forward (1 GPU only)
  3  G100M NGCF K=3 d=64 + GAS after every layer (NGCFGroupShuffle: hop + streaming MFMA
     transform per layer), eval forward
  4  G100M LightGCN K=3 d=128 (the 8-GPU config; dst-row shards at N > 1)
  6  G100M LightGCN K=3 d=64 BPR training step (1 GPU): batch 2048 from the
     device sampler, full propagation forward + fused backward (same propagation over A^T),
     the reference's [B, B] BPR loss, clip_grad_norm_, Adam
  7  G100M operand construction: CsrGraph.from_interactions_device (pairs
     resident in HBM -> normalised CSR in HBM) vs the native host builder (1 GPU)
  8  full-catalogue scoring + seen mask + top-20 (1 GPU): 16 384 G100M users x
     1M items, d = 64, ~100 seen items per user; MFMA fp32 (exact k-ordered chain) TFLOP/s
  9  G100M LightGCN K=3 d=64 BPR training step, row-sharded (src/training/distributed.py):
     any N; the embedding table and its Adam state split by destination rows
  5  power-law bipartite graph, GAT d=64 4 heads K=3: by default a 2M x 2M, 50M-pair slice;
     --g1b: the full 10M x 10M, 1B-pair configuration (Zipf exponent 0.9, seed 0, every node
     degree >= 1)

N > 1: one process per GPU; every rank builds the same graph and model (same seeds), keeps
its destination-row shard and runs the sharded forward of src/ops/distributed.py (per layer:
local kernels, then one exchange of the rows its neighbours read). Time = max over ranks.
--verify compares every rank's rows with a single-device forward of the whole graph
(bit-exact for LightGCN and NGCF; GAT's projections are library GEMMs over a different
number of rows, so it is held to 1e-5).

Each config prints one JSON line: ms per forward and edges/s (= layers * nnz / t).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gnn-recommendations_amd"))
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from src.data.dataset import RecommendationDataset  # noqa: E402
from src.models import GAT, LightGCN, NGCFGroupShuffle  # noqa: E402
from src.ops import CsrGraph  # noqa: E402
from src.ops.distributed import (DistributedGraph, gat_forward_dist,  # noqa: E402
                                 lightgcn_propagate_dist, make_work, ngcf_forward_dist)


def progress(msg: str) -> None:
    """Phase line with host RSS and device memory (stderr, line-buffered): a run that dies
    leaves the phase it died in."""
    try:
        import psutil
        rss = psutil.Process().memory_info().rss / 2**30
    except Exception:  # noqa: BLE001
        rss = float("nan")
    dev = torch.cuda.memory_allocated() / 2**30 if torch.cuda.is_available() else 0.0
    print(f"[bench_configs {time.strftime('%H:%M:%S')}] {msg} | host RSS {rss:.1f} GiB, "
          f"device {dev:.1f} GiB", file=sys.stderr, flush=True)


def zipf_ids(rng, n: int, count: int, a: float, chunk: int = 1 << 26) -> np.ndarray:
    """`count` ids in [0, n) with P(k) ~ (k+1)^-a (inverse CDF of the continuous power law on
    [1, n+1), vectorised in chunks; rng.choice over 10M categories would take minutes)."""
    out = np.empty(count, dtype=np.int64)
    e = 1.0 - a
    top = (n + 1.0) ** e - 1.0
    for s in range(0, count, chunk):
        u = rng.random(min(chunk, count - s))
        k = np.floor((u * top + 1.0) ** (1.0 / e)) - 1.0
        out[s:s + u.size] = np.minimum(k, n - 1).astype(np.int64)
    return out


def powerlaw_graph(n_users, n_items, n_pairs, a, seed, threads=16, device=None):
    """device: build the operand in HBM (CsrGraph.from_interactions_device, bit-identical to
    the host builder) and keep only the pair arrays on the host — the host builder's sort
    buffers for 1B pairs are tens of GB of host memory."""
    rng = np.random.default_rng(seed)
    u = zipf_ids(rng, n_users, n_pairs, a)
    i = zipf_ids(rng, n_items, n_pairs, a)
    # min degree >= 1 (the reference's dense GAT turns an isolated node into all-NaN)
    u = np.concatenate([u, np.arange(n_users), rng.integers(0, n_users, n_items)])
    i = np.concatenate([i, rng.integers(0, n_items, n_users), np.arange(n_items)])
    progress(f"{u.size} pairs sampled")
    if device is not None:
        return CsrGraph.from_interactions_device(u, i, n_users, n_items, binary=True,
                                                 device=device)
    return CsrGraph.from_interactions(u, i, n_users, n_items, binary=True, n_threads=threads)


def config3_model(device):
    """Config 3's model: NGCF K=3 d=64 + GAS (8x8 blocks) after every layer, seed 0, eval."""
    torch.manual_seed(0)
    return NGCFGroupShuffle(1_000_000, 1_000_000, 64, [64, 64, 64], 0.1, 0.01, 8, 0.3).to(device).eval()


def config5_model(shape, device):
    """Config 5's model: GAT d=64, 4 heads, K=3 (concat layers, head-averaged last), seed 0."""
    torch.manual_seed(0)
    return GAT(shape[0], shape[1], 64, 3, 4, 0.1, 0.2, 0.1).to(device).eval()


def _close(got, ref, rtol=1e-4, atol=1e-6) -> dict:
    """The governing check, elementwise |diff| <= atol + rtol |ref| (`within_tolerance`, with
    its atol / rtol in the record), and the north star's bar beside it: embeddings within 1e-4
    (absolute, fp32)."""
    err = (got - ref).abs()
    mx = float(err.max())
    return {"max_abs_diff": mx, "max_abs_ref": float(ref.abs().max()), "atol": atol,
            "rtol": rtol, "within_tolerance": bool((err <= atol + rtol * ref.abs()).all()),
            "within_north_star_1e-4": mx <= 1e-4}


def hop_roofline(n_rows, nnz, d, ms, K=3, extra_per_row=0, what="") -> dict:
    """K hops at SURVEY §8(d)'s bytes (bench.hop_bytes_alg: CSR, x read once, y written once)
    plus extra_per_row bytes per layer (config 3: the transform's n and x rows in, its output
    row out), against 8 TB/s: the same model as the headline's roofline."""
    algo = K * (bench.hop_bytes_alg(nnz, n_rows, n_rows, d) + extra_per_row * n_rows)
    gbps = algo / (ms * 1e-3) / 1e9
    return {"roofline": {"bound": "hbm", "algorithmic_bytes": algo, "achieved": gbps,
                         "peak": 8000.0, "unit": "GB/s", "frac": gbps / 8000.0,
                         "bytes_model": "K x SURVEY 8(d) B_hop" + what}}


def gat_cost(n_rows, nnz, ms) -> dict:
    """Config 5's forward against the HBM roofline and the request model.
    Compulsory bytes per forward (GAT d=64, 4 heads, K=3, layer mean fused into the epilogues):
    per layer the CSR (8 B row_ptr per row, 4 B col per edge); layers 1-2 the projection (x in,
    h out: 256 + 256 B per row), one read of the gathered h table (256), y out (256), the layer
    mean accumulator (written at layer 1, read + written at 2: 256 / 512); layer 3 one read of
    the gathered x table (256), the per-head aggregates z out and back into the head-mean GEMM
    (1 024 + 1 024), the accumulator read and the mean out (256 + 256). The request model: a
    neighbour's 256-B row is two 128-B lines per layer, priced at the random-miss cost of
    §3.1c (15.4 ps per line, the 65 G lines/s probe rate) with no L2 hits."""
    per_row = 3 * 8 + (256 + 256 + 256 + 256 + 256) + (256 + 256 + 256 + 256 + 512) \
        + (256 + 1024 + 1024 + 256 + 256)
    algo = n_rows * per_row + 3 * 4 * nnz
    lines = 3 * 2 * nnz
    gbps = algo / (ms * 1e-3) / 1e9
    return {"roofline": {"bound": "hbm", "algorithmic_bytes": algo, "achieved": gbps,
                         "peak": 8000.0, "unit": "GB/s", "frac": gbps / 8000.0,
                         "bytes_model": "per row 5 656 B (3 layers' tables, projections, "
                                        "aggregates, mean accumulator) + 12 B per edge"},
            "request_model": {"gathered_lines": lines, "G_lines_per_s": lines / (ms * 1e-3) / 1e9,
                              "all_miss_ms": lines * 15.4e-9, "frac": lines * 15.4e-9 / ms,
                              "what": "2 x 128-B lines per neighbour per layer at 15.4 ps each "
                                      "(no L2 hits) / the measured forward"}}


def torch_csr(g, device):
    """The operand as a torch CSR tensor on the device (ATen's ROCm sparse path)."""
    return torch.sparse_csr_tensor(g.row_ptr.to(device), g.col.to(device).long(),
                                   g.val.to(device), g.shape)


def verify_config3(g, m, table, device) -> dict:
    """Every layer of the native NGCF + GAS forward ([N, 4d] = cat(x0..x3)) against the
    reference's own composition in plain PyTorch fp32 on the same device and layer input:
    torch.sparse.mm (hipSPARSE), the two nn.Linear, LeakyReLU (ngcf.py:69-84), then
    (x @ blockdiag(expm))[:, perm] (group_shuffle_layer.py:88-94)."""
    A = torch_csr(g, device)
    d = m.embedding_dim
    res = {"reference": "torch fp32 on the device: torch.sparse.mm + nn.Linear + LeakyReLU + "
                        "dense block-diagonal GAS, per layer on the native layer input"}
    for k, (layer, gs) in enumerate(zip(m.layers, m.gs_layers)):
        x = table[:, k * d:(k + 1) * d].contiguous()
        n = torch.sparse.mm(A, x)
        o = layer.activation(layer.W1(n) + layer.W2(x * n))
        ref = (o @ gs._build_orthogonal_matrix())[:, gs.perm]
        res[f"layer{k + 1}"] = _close(table[:, (k + 1) * d:(k + 2) * d], ref)
        del x, n, o, ref
    del A
    res["all_within_tolerance"] = all(v["within_tolerance"] for k, v in res.items()
                                      if k.startswith("layer"))
    return res


def _edge_softmax_layer(rows, col, x, layer, n, chunk_heads=1):
    """One GATLayer forward as a sparse restatement of the reference's dense masked softmax
    (gat.py:99-149) in plain PyTorch: per head h = W_h x, e = LeakyReLU(h a_self [row] +
    h a_neigh [col]), softmax over each row's edges (scatter amax / exp / index_add), the
    weighted sum of h[col]; concat or head mean, then ELU."""
    outs = []
    for i in range(layer.n_heads):
        h = x @ layer.W[i].weight.t()
        ss = (h @ layer.a_self[i])[:, 0]
        sn = (h @ layer.a_neigh[i])[:, 0]
        e = torch.nn.functional.leaky_relu(ss[rows] + sn[col], layer.alpha)
        mx = torch.full((n,), float("-inf"), device=x.device).scatter_reduce(0, rows, e, "amax")
        p = torch.exp(e - mx[rows])
        s = torch.zeros(n, device=x.device).index_add_(0, rows, p)
        agg = torch.zeros(n, h.shape[1], device=x.device).index_add_(0, rows, p[:, None] * h[col])
        outs.append(agg / s[:, None])
        del h, e, p, agg
    out = torch.cat(outs, dim=1) if layer.concat_heads else torch.stack(outs).mean(0)
    return torch.nn.functional.elu(out)


def verify_config5(g, m, mine, device) -> dict:
    """The native GAT forward's layer mean against the reference composition (sparse
    restatement of gat.py:99-149 + gat.py:258-297) in plain PyTorch fp32 on the device."""
    rp = g.row_ptr.to(device)
    n = g.shape[0]
    rows = torch.repeat_interleave(torch.arange(n, device=device), rp[1:] - rp[:-1])
    col = g.col.to(device).long()
    x = m._initial_table()
    acc = x.clone()
    for layer in m.layers:
        x = _edge_softmax_layer(rows, col, x, layer, n)
        acc += x
    ref = acc / float(len(m.layers) + 1)
    res = {"reference": "torch fp32 on the device: per-head edge softmax (scatter amax/exp/"
                        "index_add) over the CSR pattern, ELU, layer mean"}
    # atol 1e-5 + rtol 1e-4: the tolerance of the sampled-row oracle check (oracle/gat_sample.py)
    # — both sides are fp32 softmax chains in different orders, over three layers
    res.update(_close(mine, ref, atol=1e-5))
    return res


def timed(fn, steps, warmup, world, device):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = torch.tensor([(time.perf_counter() - t0) / steps * 1e3], dtype=torch.float64,
                     device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()), out


def rank_max(v, world, device):
    t = torch.tensor([float(v)], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def check(mine, ref, exact, world, device):
    diff = float((mine - ref).abs().max()) if mine.numel() else 0.0
    ok = torch.equal(mine, ref) if exact else diff <= 1e-5
    flag = torch.tensor([1 if ok else 0], device=device)
    if world > 1:
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return {"bit_exact" if exact else "within_1e-5": bool(flag.item()), "max_abs_diff": diff}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--configs", nargs="+", type=int, default=[2, 3, 4, 5])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--g1b", action="store_true", help="config 5 at full size (10M x 10M, 1B pairs)")
    ap.add_argument("--c5-shape", type=int, nargs=3, default=None, metavar=("USERS", "ITEMS", "PAIRS"),
                    help="config 5 at another size (operand built on the device)")
    ap.add_argument("--host-build", action="store_true",
                    help="config 5 --g1b / --c5-shape: build the operand on the host (the form "
                         "round 2's G1B run completed with; profiles/r03/g1b_box_loss_record.md)")
    ap.add_argument("--verify", action="store_true")
    ap.add_argument("--no-ref-check", action="store_true",
                    help="N = 1: skip the per-config check against the reference's composition "
                         "in plain PyTorch on the device (configs 3 and 5-slice)")
    ap.add_argument("--topk-splits", type=int, nargs="*", default=[],
                    help="config 8: item-range splits timed besides 1 and the default")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    a = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    torch.cuda.set_device(device)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
    threads = max(1, bench.host_threads() // world)
    out = []

    def emit(rec):
        rec["n_gpus"] = world
        if rank == 0:
            print(json.dumps(rec), flush=True)
        out.append(rec)

    with torch.no_grad():
        if 2 in a.configs and world == 1:
            ds = RecommendationDataset.synthetic_movielens(6040, 3706, 1_000_209, seed=1, name="ml-1m")
            g = ds.get_graph(device)
            torch.manual_seed(0)
            m = LightGCN(ds.n_users, ds.n_items, 64, 3, 0.1).to(device).eval()
            t, _ = timed(lambda: m(g), a.steps * 10, a.warmup, 1, device)
            emit({"config": 2, "workload": "ML-1M-shaped LightGCN K=3 d=64 forward",
                  "nnz": g.nnz, "n_nodes": g.shape[0], "ms": t,
                  "edges_per_s": 3 * g.nnz / (t * 1e-3), **hop_roofline(g.shape[0], g.nnz, 64, t)})
        g100 = None
        if 3 in a.configs or 4 in a.configs or 9 in a.configs or (6 in a.configs and world == 1):
            g100 = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, threads)
        if 3 in a.configs:
            m = config3_model(device)
            dg = DistributedGraph(g100, rank, world, device)
            x0p = dg.pad_table(m._initial_table())
            t, mine = timed(lambda: ngcf_forward_dist(dg, m, x0p), a.steps, a.warmup, world, device)
            rec = {"config": 3, "workload": "G100M NGCF K=3 d=64 + GAS (hop + streaming MFMA "
                   "transform per layer)", "nnz": g100.nnz, "ms": t,
                   "edges_per_s": 3 * g100.nnz / (t * 1e-3),
                   "mfma_flops_per_s": 3 * 2 * 2_000_000 * 128 * 64 / (t * 1e-3),
                   "exchange": dg.exchange_mode if world > 1 else None,
                   **hop_roofline(2_000_000, g100.nnz, 64, t, extra_per_row=3 * 256,
                                  what=" + 768 B per row per layer (transform: n, x in; out)")}
            if a.verify:
                g1 = g100.to(device)
                u, i = m(g1)
                rec["verify"] = check(mine, torch.cat([u, i])[dg.row_begin:dg.row_end], True,
                                      world, device)
                del g1, u, i
            if world == 1 and not a.no_ref_check:
                rec["verify_vs_torch_reference"] = verify_config3(g100, m, mine, device)
            emit(rec)
            del m, dg, x0p, mine
        if 4 in a.configs:
            torch.manual_seed(0)
            m = LightGCN(1_000_000, 1_000_000, 128, 3, 0.1).to(device).eval()
            dg = DistributedGraph(g100, rank, world, device)
            x0p = dg.pad_table(m._initial_table())
            work = make_work(dg, 128, device)
            t, mine = timed(lambda: lightgcn_propagate_dist(dg, x0p, 3, work=work),
                            a.steps, a.warmup, world, device)
            rec = {"config": 4, "workload": "G100M LightGCN K=3 d=128, dst-row shards",
                   "nnz": g100.nnz, "ms": t, "edges_per_s": 3 * g100.nnz / (t * 1e-3),
                   "exchange": dg.exchange_mode if world > 1 else None,
                   **hop_roofline(2_000_000, g100.nnz, 128, t)}
            if a.verify:
                g1 = g100.to(device)
                u, i = m(g1)
                rec["verify"] = check(mine, torch.cat([u, i])[dg.row_begin:dg.row_end], True,
                                      world, device)
                del g1, u, i
            emit(rec)
            del m, dg, x0p, work, mine
        if 9 in a.configs:
            from src.training import lightgcn_train_step_dist, make_adam
            torch.manual_seed(0)
            m = LightGCN(1_000_000, 1_000_000, 64, 3, 0.1)
            dg = DistributedGraph(g100, rank, world, device)
            x0 = m._initial_table().detach()
            emb = torch.nn.Parameter(x0[dg.row_begin:dg.row_end].to(device).clone())
            del m, x0
            opt = make_adam([emb], 1e-3, 1e-4, device)
            gen = torch.Generator().manual_seed(0)      # the same batches on every rank

            def step9():
                bu = torch.randint(0, 1_000_000, (2048,), generator=gen)
                bp = torch.randint(0, 1_000_000, (2048,), generator=gen)
                bn = torch.randint(0, 1_000_000, (2048, 1), generator=gen)
                return lightgcn_train_step_dist(dg, emb, 3, 1_000_000, bu, bp, bn, opt)
            with torch.enable_grad():
                t, loss = timed(step9, a.steps, a.warmup, world, device)
            emit({"config": 9, "workload": "G100M LightGCN K=3 d=64 BPR train step, row-sharded "
                  "(batch 2048, fwd + bwd propagation with per-hop exchanges, sharded Adam)",
                  "nnz": g100.nnz, "ms": t, "equiv_edges_per_s": 2 * 3 * g100.nnz / (t * 1e-3),
                  "loss": float(loss), "exchange": dg.exchange_mode if world > 1 else None})
            del dg, emb, opt
        if 6 in a.configs and world == 1:
            from src.training import BPRLoss, DeviceSampler, make_adam, train_step
            torch.manual_seed(0)
            m = LightGCN(1_000_000, 1_000_000, 64, 3, 0.1).to(device).train()
            g1 = g100.to(device)
            rp = g100.row_ptr.numpy()
            users = np.repeat(np.arange(1_000_000), np.diff(rp[:1_000_001]))
            items = g100.col.numpy()[:rp[1_000_000]] - 1_000_000
            samp = DeviceSampler(users, items, 1_000_000, 2048, 1, device, seed=0)
            opt = make_adam(m.parameters(), 1e-3, 1e-4, device)
            loss_fn = BPRLoss()
            res = {}
            for subset in (True, False):
                with torch.enable_grad():
                    res[subset] = timed(lambda: train_step(m, g1, *samp(), opt, loss_fn, 1.0,
                                                           row_subset=subset),
                                        a.steps, a.warmup, 1, device)
            t, loss = res[True]
            # equiv_edges_per_s: the 2*K*nnz edge messages of the reference's full forward +
            # backward, per step time (the row-subset forward skips most of the forward's)
            emit({"config": 6, "workload": "G100M LightGCN K=3 d=64 BPR train step (batch 2048, "
                  "row-subset fwd + masked bwd propagation, Adam)", "nnz": g1.nnz, "ms": t,
                  "ms_full_forward": res[False][0],
                  "equiv_edges_per_s": 2 * 3 * g1.nnz / (t * 1e-3), "loss": float(loss)})
            del m, g1, opt, samp
        if 8 in a.configs and world == 1:
            from src.ops import score_topk
            from src.ops.functional import topk_splits
            ni, dd = 1_000_000, 64
            for nb in (16384, 2048):
                gen = torch.Generator(device=device).manual_seed(0)
                U = torch.randn(nb, dd, device=device, generator=gen) * 0.1
                V = torch.randn(ni, dd, device=device, generator=gen) * 0.1
                seen = torch.sort(torch.randint(0, ni, (nb, 100), device=device, generator=gen), 1).values
                seen_ptr = torch.arange(0, nb * 100 + 1, 100, dtype=torch.int64)
                seen_col = seen.flatten().to(torch.int32).cpu()
                res = {}
                for ns in sorted({1, topk_splits(nb, ni, dd, 20)} | set(a.topk_splits)):
                    f = lambda: score_topk(U, V, 20, seen_ptr, seen_col, n_split=ns)
                    t, _ = timed(f, max(2, a.steps // 5), 1, 1, device)
                    res[ns] = t
                ns = min(res, key=res.get)
                t = res[ns]
                flops = 2.0 * nb * ni * dd
                emit({"config": 8, "workload": f"score + mask + top-20: {nb} users x {ni} items, d={dd}",
                      "ms": t, "n_split": ns, "ms_by_split": res,
                      "tflops": flops / (t * 1e-3) / 1e12, "mfma_f32_peak_tflops": 157.3,
                      "frac": flops / (t * 1e-3) / 157.3e12, "users_per_s": nb / (t * 1e-3)})
        if 7 in a.configs and world == 1:
            rng = np.random.default_rng(0)
            u = rng.integers(0, 1_000_000, 100_000_000, dtype=np.int64)
            i = rng.integers(0, 1_000_000, 100_000_000, dtype=np.int64)
            ud, idv = torch.from_numpy(u).to(device), torch.from_numpy(i).to(device)
            ts = []
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                gd = CsrGraph.from_interactions_device(ud, idv, 1_000_000, 1_000_000,
                                                       binary=True, device=device)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
                if len(ts) < 3:
                    del gd
            t0 = time.perf_counter()
            gh = CsrGraph.from_interactions(u, i, 1_000_000, 1_000_000, binary=True,
                                            n_threads=threads)
            th = time.perf_counter() - t0
            same = (gd.nnz == gh.nnz and torch.equal(gd.col.cpu(), gh.col)
                    and torch.equal(gd.val.cpu().view(torch.int32), gh.val.view(torch.int32))
                    and torch.equal(gd.row_ptr.cpu(), gh.row_ptr))
            emit({"config": 7, "workload": "G100M operand build (100M pairs -> normalised CSR)",
                  "nnz": gd.nnz, "device_s": float(np.median(ts)), "host_s": th,
                  "host_threads": threads, "bit_identical": bool(same)})
            del gd, gh, ud, idv
        del g100
        torch.cuda.empty_cache()
        if 5 in a.configs:
            t0 = time.time()
            big = a.g1b or a.c5_shape is not None
            shape = (tuple(a.c5_shape) if a.c5_shape else
                     (10_000_000, 10_000_000, 1_000_000_000) if a.g1b else (2_000_000, 2_000_000, 50_000_000))
            progress(f"config 5: sampling {shape}")
            g = powerlaw_graph(*shape, 0.9, 0, threads,
                               device=device if big and not a.host_build else None)
            build_s = time.time() - t0
            progress(f"operand built: {g.nnz} nnz in {build_s:.1f} s")
            deg = (g.row_ptr[1:] - g.row_ptr[:-1]).cpu().numpy()
            m = config5_model(shape, device)
            dg = DistributedGraph(g, rank, world, device)
            x0p = dg.pad_table(m._initial_table())
            progress("shard + x0 ready; first forward")
            gat_forward_dist(dg, m, x0p)
            torch.cuda.synchronize()
            progress("first forward done; timing")
            t, mine = timed(lambda: gat_forward_dist(dg, m, x0p), a.steps, a.warmup, world, device)
            progress(f"timed: {t:.2f} ms per forward")
            rec = {"config": 5, "workload": f"power-law {shape[0]}x{shape[1]} ({shape[2]} pairs, "
                   f"Zipf 0.9, seed 0) GAT d=64 4 heads K=3 forward", "nnz": g.nnz,
                   "max_degree": int(deg.max()), "median_degree": float(np.median(deg)),
                   "ms": t, "edges_per_s": 3 * g.nnz / (t * 1e-3), "graph_build_s": build_s,
                   "shard_nnz_max": int(rank_max(dg.shard.nnz, world, device)),
                   "exchange": dg.exchange_mode if world > 1 else None}
            rec.update(gat_cost(shape[0] + shape[1], g.nnz, t))
            if a.verify:
                del x0p
                g1 = g.to(device)
                u, i = m(g1)
                rec["verify"] = check(mine, torch.cat([u, i])[dg.row_begin:dg.row_end], False,
                                      world, device)
                del g1, u, i
            if world == 1 and not big and not a.no_ref_check:
                rec["verify_vs_torch_reference"] = verify_config5(g, m, mine, device)
            if world == 1 and big and not a.no_ref_check:
                # too large for the whole-graph references: the sampled-row oracle check
                # (oracle/gat_sample.py) at the 64 heaviest rows + 4096 per degree decile
                from oracle.gat_sample import check_forward, sample_rows
                rows = sample_rows(deg, n_heavy=64, per_decile=4096, seed=0)
                progress(f"sampled-row oracle check: {rows.size} rows")
                t1 = time.time()
                gd = g if g.row_ptr.is_cuda else g.to(device)
                rec["verify"] = check_forward(m, gd, mine, rows)
                rec["verify"]["seconds"] = time.time() - t1
                progress(f"check done: all_within_tolerance={rec['verify']['all_within_tolerance']}")
                del gd
            emit(rec)
    if world > 1:
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
