"""Sharded forwards with the NATIVE kernels: two ranks sharing the one MI355X over gloo
(host-staged exchange; RCCL refuses two ranks on one GPU). Every rank's rows must equal the
single-device forward of the whole graph: bit for bit for LightGCN and NGCF+GAS (each kernel
computes a row from that row's inputs only), within 1e-5 for GAT (its projections are
library GEMMs over a different number of rows)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _graph():
    from src.ops import CsrGraph
    rng = np.random.default_rng(11)
    nu, ni, n = 3000, 2000, 60000
    u = rng.integers(0, nu, n)
    i = np.minimum(rng.zipf(1.6, n) - 1, ni - 1)  # skewed items: some heavy rows
    u = np.concatenate([u, np.arange(nu), rng.integers(0, nu, ni)])
    i = np.concatenate([i, rng.integers(0, ni, nu), np.arange(ni)])
    return CsrGraph.from_interactions(u, i, nu, ni, binary=True), nu, ni


def _model(kind, nu, ni, dev):
    from src.models import GAT, LightGCN, NGCFGroupShuffle
    torch.manual_seed(7)
    if kind in ("lightgcn", "train", "lightgcn_tiled", "lightgcn_grid_tiled"):
        m = LightGCN(nu, ni, 64, 3, 0.1)
    elif kind == "lightgcn_d128_tiled":
        m = LightGCN(nu, ni, 128, 3, 0.1)
    elif kind == "lightgcn_k4_tiled":
        m = LightGCN(nu, ni, 64, 4, 0.1)
    elif kind == "ngcf_gs":
        m = NGCFGroupShuffle(nu, ni, 64, [64, 64, 64], 0.1, 0.1, 8, 0.3)
    else:
        m = GAT(nu, ni, 64, 3, 4, 0.1, 0.2, 0.1)
    return m.to(dev).eval()


def _worker(rank, world, port, kind, exchange, q):
    try:
        _work(rank, world, port, kind, exchange, q)
    except BaseException as e:   # report instead of leaving the parent waiting on the queue
        import traceback
        q.put((rank, None, traceback.format_exc(), None))
        raise


def _work(rank, world, port, kind, exchange, q):
    import sys
    from conftest import PKG, ROOT
    sys.path[:0] = [str(ROOT), str(PKG)]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from src.ops.distributed import (DistributedGraph, gat_forward_dist,
                                         lightgcn_propagate_dist, ngcf_forward_dist)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        if kind.endswith("_tiled"):   # the small test graph through the column-ordered kernel
            from src.ops import functional as F
            F.TILED_MIN_ROWS, F.TILED_MIN_TABLE_BYTES = 0, 0
        full, nu, ni = _graph()
        m = _model(kind, nu, ni, dev)
        with torch.no_grad():
            dg = DistributedGraph(full, rank, world, dev, exchange=exchange)
            x0p = dg.pad_table(m._initial_table())
            if kind == "train":   # one BPR step on the shard, then the updated rows
                from src.training import lightgcn_train_step_dist
                emb = torch.nn.Parameter(dg.local_slice(x0p).clone())
                opt = torch.optim.Adam([emb], lr=1e-2)
                gen = torch.Generator().manual_seed(3)
                bu = torch.randint(0, nu, (256,), generator=gen)
                bp = torch.randint(0, ni, (256,), generator=gen)
                bn = torch.randint(0, ni, (256, 1), generator=gen)
                with torch.enable_grad():
                    lightgcn_train_step_dist(dg, emb, 3, nu, bu, bp, bn, opt)
                mine = emb.detach()
                one = DistributedGraph(full, 0, 1, dev)
                emb1 = torch.nn.Parameter(m._initial_table().clone())
                opt1 = torch.optim.Adam([emb1], lr=1e-2)
                with torch.enable_grad():
                    lightgcn_train_step_dist(one, emb1, 3, nu, bu, bp, bn, opt1)
                q.put((rank, mine.cpu().numpy(), emb1.detach()[dg.row_begin:dg.row_end].cpu().numpy(),
                       dg.exchange_mode))
                return
            if kind == "lightgcn_grid_tiled":
                # 2 feature groups x 1 row shard: each rank propagates 32 of the 64 columns of
                # every row, no exchange; gathered back to the full table
                from src.ops import functional as F
                from src.ops.distributed import RankGrid, lightgcn_propagate_grid
                grid = RankGrid(full, rank, world, dev, 64)
                assert (grid.F, grid.R) == (2, 1)
                xc = grid.x0_table(m._initial_table())
                assert xc.shape[1] == 32 and F.tiled_plan_for(grid.dg.shard, xc) is not None
                mine = lightgcn_propagate_grid(grid, xc, 3, gather_output=True)
                u, i = m(full.to(dev))
                ref = torch.cat([u, i])
                q.put((rank, mine.cpu().numpy(), ref.cpu().numpy(), "none"))
                return
            if kind == "lightgcn":
                mine = lightgcn_propagate_dist(dg, x0p, 3, overlap_chunks=3)
            elif kind == "lightgcn_k4_tiled":
                # deferred layer mean at K = 4: hop 3 reads its input rows (prev) from one
                # exchange piece and writes its output into another (no aliasing)
                from src.ops import functional as F
                assert F.tiled_plan_for(dg.shard, x0p) is not None
                mine = lightgcn_propagate_dist(dg, x0p, 4)
            elif kind.endswith("_tiled"):
                from src.ops import functional as F
                for c0, c1 in dg.chunk_bounds(3):   # every overlap chunk runs the tiled kernel
                    if min(c1, dg.n_local) > c0:
                        assert F.tiled_plan_for(dg.shard.row_slice(c0, min(c1, dg.n_local)),
                                                x0p) is not None
                mine = lightgcn_propagate_dist(dg, x0p, 3, overlap_chunks=3)
                # chunks sized to leave 16 CUs to the exchange: one pass of <= cus - 16 blocks,
                # the same bits
                cus = torch.cuda.get_device_properties(dev).multi_processor_count
                sl = dg.shard.row_slice(0, min(dg.chunk_bounds(3)[0][1], dg.n_local))
                assert F.tiled_plan_for(sl, x0p, reserve_cus=16)["n_blocks"] <= cus - 16
                again = lightgcn_propagate_dist(dg, x0p, 3, overlap_chunks=3, reserve_cus=16)
                assert torch.equal(again, mine), "reserve_cus changed the result"
            elif kind == "ngcf_gs":
                mine = ngcf_forward_dist(dg, m, x0p)
            else:
                mine = gat_forward_dist(dg, m, x0p)
            u, i = m(full.to(dev))
            ref = torch.cat([u, i])[dg.row_begin:dg.row_end]
            q.put((rank, mine.cpu().numpy(), ref.cpu().numpy(), dg.exchange_mode))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,exchange", [("lightgcn", "p2p"), ("lightgcn", "allgather"),
                                           ("lightgcn_tiled", "p2p"),
                                           ("lightgcn_grid_tiled", "auto"),
                                           ("lightgcn_d128_tiled", "p2p"),
                                           ("lightgcn_k4_tiled", "p2p"),
                                           ("ngcf_gs", "auto"), ("gat", "auto"),
                                           ("train", "auto")])
def test_two_ranks_native_match_single_device(cuda, kind, exchange):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, kind, exchange, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for rank, mine, ref, _ in res:
        assert mine is not None, f"rank {rank} failed:\n{ref}"
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, mine, ref, mode in res:
        assert mine.shape == ref.shape and mine.shape[0] > 0
        assert np.isfinite(mine).all()
        if kind in ("gat", "train"):   # train: the clip norm is summed across ranks
            np.testing.assert_allclose(mine, ref, rtol=0, atol=1e-5)
        else:
            np.testing.assert_array_equal(mine.view(np.uint32), ref.view(np.uint32))
