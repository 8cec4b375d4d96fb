"""Multi-rank propagation logic on CPU ranks over gloo (world_size 2 and 3).

The partition, padded all-gather layout and fused layer-mean bookkeeping of
src/ops/distributed.py run exactly as on the GPUs; only the local hop is the oracle's CPU
restatement instead of the HIP kernel (injected through `hop_fn`). The result must be
bit-identical to the single-device oracle propagation.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from conftest import golden_csr, load_golden

from src.ops import CsrGraph
from src.ops._lib import EPI_ACC_ADD, EPI_ACC_DIV, EPI_ACC_INIT, EPI_ACC_X, EPI_NO_Y
from src.ops.distributed import (DistributedGraph, RankGrid, feature_groups_for,
                                 lightgcn_propagate_dist, lightgcn_propagate_grid)


def _overlap(a, b) -> bool:
    """Do two row-major tables share any byte of storage?"""
    if a is None or b is None or a.numel() == 0 or b.numel() == 0:
        return False
    def span(t):
        lo = t.data_ptr()
        return lo, lo + ((t.shape[0] - 1) * t.stride(0) + t.shape[-1]) * t.element_size()
    (a0, a1), (b0, b1) = span(a), span(b)
    return a0 < b1 and b0 < a1


def cpu_hop(adj, x, y, *, epi, self_rows, acc, acc_div, prev=None):
    """CPU stand-in for gnnrec_spmm_tiled_f32 (oracle SpMM + the same epilogue order:
    acc = (((self | acc) [+ acc on INIT|ADD]) [+ prev on ACC_X]) + y [/ div]). It computes
    before it writes, so it also asserts the kernel's __restrict__ contract: y shares no rows
    with the gathered table x nor with the ACC_X rows prev."""
    assert not _overlap(y, x), "a hop writes rows it gathers"
    assert not (epi & EPI_ACC_X and _overlap(y, prev)), "a hop writes its ACC_X rows"
    yy = oracle.spmm(adj.row_ptr.numpy(), adj.col.numpy(), adj.val.numpy(), x.numpy())
    if epi & (EPI_ACC_INIT | EPI_ACC_ADD):
        b = (self_rows if epi & EPI_ACC_INIT else acc).numpy().copy()
        if epi & EPI_ACC_INIT and epi & EPI_ACC_ADD:
            b = b + acc.numpy()
        if epi & EPI_ACC_X:
            b = b + (prev if prev is not None else x[:adj.n_rows]).numpy()
        b = b + yy
        if epi & EPI_ACC_DIV:
            b = b / np.float32(acc_div)
    if not (epi & EPI_NO_Y):
        y.copy_(torch.from_numpy(yy))
    if epi & (EPI_ACC_INIT | EPI_ACC_ADD):
        acc.copy_(torch.from_numpy(b.astype(np.float32)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, K, balance, q, exchange="auto", chunks=1, deferred=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rp, col, val, nu, ni = golden_csr("g_small")
        full = CsrGraph(torch.from_numpy(rp), torch.from_numpy(col), torch.from_numpy(val),
                        (rp.size - 1, rp.size - 1), nu, ni, True)
        torch.manual_seed(5)
        x0 = torch.randn(full.shape[0], 32) * 0.1
        dg = DistributedGraph(full, rank, world, "cpu", balance=balance, exchange=exchange)
        xp = dg.pad_table(x0)
        local = lightgcn_propagate_dist(dg, xp, K, hop_fn=cpu_hop, overlap_chunks=chunks,
                                        deferred=deferred)
        whole = lightgcn_propagate_dist(dg, xp, K, hop_fn=cpu_hop, gather_output=True,
                                        overlap_chunks=chunks, deferred=deferred)
        if rank == 0:
            ref = oracle.lightgcn(rp, col, val, x0.numpy(), K)
            q.put((whole.numpy(), ref, local.numpy(), ref[dg.row_begin:dg.row_end],
                   dg.exchange_mode, dg.needs.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,K,balance,exchange,chunks,deferred", [
    (2, 3, "nnz", "auto", 1, False), (3, 2, "rows", "auto", 1, False),
    (2, 1, "nnz", "allgather", 1, False), (4, 3, "nnz", "auto", 1, False),
    (4, 2, "nnz", "allgather", 1, False), (4, 3, "nnz", "p2p", 3, False),
    (3, 3, "rows", "p2p", 4, False),
    # the deferred layer mean on shards (y1 parked in the output rows, hop 3's previous layer
    # from the rank's own exchange piece): 2/3/4 ranks, both exchanges, chunked, K = 2, 3, 4
    (2, 3, "nnz", "auto", 1, True), (4, 3, "nnz", "p2p", 3, True),
    (3, 3, "rows", "allgather", 1, True), (4, 2, "nnz", "auto", 2, True),
    (3, 4, "nnz", "p2p", 1, True), (1, 3, "nnz", "auto", 1, True),
    (2, 4, "nnz", "p2p", 1, True), (4, 5, "nnz", "allgather", 1, True)])
def test_sharded_propagation_matches_single_device(world, K, balance, exchange, chunks,
                                                   deferred):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, K, balance, q, exchange, chunks,
                                               deferred))
             for r in range(world)]
    for p in procs:
        p.start()
    whole, ref, local, ref_local, mode, needs = q.get(timeout=120)
    if exchange == "auto" and world == 4:
        # bipartite graph, nnz-balanced: users on ranks 0-1, items on 2-3 -> point-to-point
        assert mode == "p2p" and not needs.all()
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(whole.view(np.uint32), ref.view(np.uint32))
    np.testing.assert_array_equal(local.view(np.uint32), ref_local.view(np.uint32))


def _grid_worker(rank, world, port, K, d, F, exchange, deferred, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rp, col, val, nu, ni = golden_csr("g_small")
        full = CsrGraph(torch.from_numpy(rp), torch.from_numpy(col), torch.from_numpy(val),
                        (rp.size - 1, rp.size - 1), nu, ni, True)
        torch.manual_seed(6)
        x0 = torch.randn(full.shape[0], d) * 0.1
        grid = RankGrid(full, rank, world, "cpu", d, F, exchange=exchange)
        xc = grid.x0_table(x0)
        local = lightgcn_propagate_grid(grid, xc, K, hop_fn=cpu_hop, deferred=deferred)
        whole = lightgcn_propagate_grid(grid, xc, K, hop_fn=cpu_hop, gather_output=True,
                                        deferred=deferred)
        ref = oracle.lightgcn(rp, col, val, x0.numpy(), K)
        c0, c1 = grid.cols
        dg = grid.dg
        q.put((rank, grid.F, grid.R, grid.f, grid.r, whole.numpy(), ref,
               local.numpy(), ref[dg.row_begin:dg.row_end, c0:c1], dg.recv_rows()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,K,d,F,exchange,deferred", [
    (2, 3, 64, None, "auto", False),       # F = 2: no exchange at all
    (4, 3, 64, None, "auto", True),        # 2 feature groups x 2 row shards (p2p in group)
    (4, 2, 64, 2, "allgather", False),
    (4, 3, 128, None, "auto", True),       # F = 4
    (4, 3, 64, 1, "auto", True),           # plain row shards through the grid
    (3, 3, 96, 3, "auto", False),
    # the driver's 8-GPU layouts (bench.py): headline d = 64 -> 2 feature groups x 4 row
    # shards, config 4 d = 128 -> 4 x 2, and the north star's 1-D row shards (F = 1), with
    # both exchanges and the deferred layer mean
    (8, 3, 64, None, "p2p", True), (8, 3, 64, None, "allgather", True),
    (8, 3, 128, None, "p2p", True), (8, 3, 128, None, "allgather", True),
    (8, 3, 64, 1, "p2p", True), (8, 3, 64, 1, "allgather", True)])
def test_rank_grid_matches_single_device(world, K, d, F, exchange, deferred):
    """Feature groups x row shards: every rank's column block of its rows, and the gathered
    [N, d] table, bit-identical to the single-device oracle propagation."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grid_worker, args=(r, world, port, K, d, F, exchange, deferred,
                                                    q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_F = feature_groups_for(world, d, F)
    cells = set()
    for rank, gF, gR, f, r, whole, ref, local, ref_local, recv in res:
        assert (gF, gR) == (want_F, world // want_F) and rank == r * gF + f
        cells.add((f, r))
        np.testing.assert_array_equal(whole.view(np.uint32), ref.view(np.uint32))
        np.testing.assert_array_equal(local.view(np.uint32), ref_local.view(np.uint32))
        if gR == 1:
            assert recv == 0
    assert len(cells) == world


def test_feature_groups_for():
    assert feature_groups_for(2, 64) == 2 and feature_groups_for(8, 64) == 2
    assert feature_groups_for(8, 128) == 4 and feature_groups_for(3, 64) == 1
    assert feature_groups_for(4, 48) == 1            # d % 32 != 0: one group
    assert feature_groups_for(4, 128, 2) == 2
    with pytest.raises(ValueError):
        feature_groups_for(4, 64, 4)                 # only 2 slices
    with pytest.raises(ValueError):
        feature_groups_for(6, 128, 4)                # does not divide the world


def test_partition_bounds_balance_nnz():
    rp = np.array([0, 10, 10, 11, 30, 31, 32, 40], dtype=np.int64)
    b = CsrGraph.partition_bounds(rp, 2)
    assert b[0] == 0 and b[-1] == 7
    loads = [rp[b[i + 1]] - rp[b[i]] for i in range(2)]
    assert max(loads) <= 30
    assert CsrGraph.partition_bounds(rp, 7, "rows") == tuple(range(8))


# ---- sharded NGCF(+GAS) and GAT forwards (row-local epilogues on the shard) ----------------
def cpu_ngcf_layer(shard, x_in, x_self, layer, gs, out):
    """CPU stand-in for gnnrec_spmm_ngcf_f32 on a shard: the reference layer's own ops."""
    n = torch.sparse.mm(shard.to_torch_sparse_coo(), x_in)
    o = layer.activation(layer.W1(n) + layer.W2(x_self * n))
    out.copy_(gs(o) if gs is not None else o)


def cpu_gat_layer(shard, feat, s_self, s_neigh, layer, *, apply_elu, epi, self_rows, acc,
                  acc_div):
    """CPU stand-in for GATLayer.native_forward: edge softmax over the shard's CSR pattern."""
    n, H = shard.n_rows, layer.n_heads
    shared = layer.shares_input()
    o = layer.in_dim if shared else layer.out_dim
    rp = shard.row_ptr
    rows = torch.repeat_interleave(torch.arange(n), rp[1:] - rp[:-1])
    col = shard.col.long()
    e = torch.nn.functional.leaky_relu(s_self[rows] + s_neigh[col], layer.alpha)
    m = torch.full((n, H), float("-inf")).scatter_reduce(0, rows[:, None].expand(-1, H), e,
                                                         "amax")
    p = torch.exp(e - m[rows])
    s = torch.zeros(n, H).index_add_(0, rows, p)
    g = feat[col].unsqueeze(1).expand(-1, H, -1) if shared else feat.view(-1, H, o)[col]
    agg = torch.zeros(n, H, o).index_add_(0, rows, p[..., None] * g)
    agg = agg / s[..., None]
    if shared:
        out = agg.reshape(n, H * o) @ layer.head_mean_weight()
    else:
        out = agg.reshape(n, H * o) if layer.concat_heads else agg.mean(1)
    if apply_elu:
        out = torch.nn.functional.elu(out)
    if epi & EPI_ACC_INIT:
        acc.copy_(self_rows + out)
    else:
        acc.add_(out)
    if epi & EPI_ACC_DIV:
        acc.div_(acc_div)
    return out


def _make_model(kind, nu, ni):
    from src.models import GAT, NGCFGroupShuffle
    torch.manual_seed(3)
    if kind == "ngcf_gs":
        m = NGCFGroupShuffle(nu, ni, 32, [32, 32, 32], 0.0, 0.1, 8, 0.3)
    else:
        m = GAT(nu, ni, 32, 3, 4, 0.0, 0.2, 0.1)
    return m.eval()


def _model_worker(rank, world, port, kind, q):
    from src.ops.distributed import gat_forward_dist, ngcf_forward_dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rp, col, val, nu, ni = golden_csr("g_small")
        full = CsrGraph(torch.from_numpy(rp), torch.from_numpy(col), torch.from_numpy(val),
                        (rp.size - 1, rp.size - 1), nu, ni, True)
        m = _make_model(kind, nu, ni)
        with torch.no_grad():
            x0 = m._initial_table()
            dg = DistributedGraph(full, rank, world, "cpu")
            fwd, fn = ((ngcf_forward_dist, cpu_ngcf_layer) if kind == "ngcf_gs"
                       else (gat_forward_dist, cpu_gat_layer))
            whole = fwd(dg, m, dg.pad_table(x0), layer_fn=fn, gather_output=True)
            if rank == 0:
                one = DistributedGraph(full, 0, 1, "cpu")
                single = fwd(one, m, one.pad_table(x0), layer_fn=fn)
                u, i = m(full.to_torch_sparse_coo())      # the reference path of the model
                q.put((whole.numpy(), single.numpy(), torch.cat([u, i]).numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,world", [("ngcf_gs", 2), ("ngcf_gs", 3), ("gat", 2), ("gat", 4)])
def test_sharded_model_forward_matches_single_device(kind, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_model_worker, args=(r, world, port, kind, q))
             for r in range(world)]
    for p in procs:
        p.start()
    whole, single, ref = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert whole.shape == single.shape == ref.shape
    # shard bookkeeping: same per-row computation on every rank -> same numbers as one device
    np.testing.assert_allclose(whole, single, rtol=0, atol=1e-6)
    # and the stand-in layers reproduce the model's own (reference) forward
    np.testing.assert_allclose(single, ref, rtol=0, atol=2e-6)


# ---- row-sharded BPR training step (§8e training + §8f1) ---------------------------------
def _train_worker(rank, world, port, q):
    from src.models import LightGCN
    from src.ops.distributed import gather_rows
    from src.training import lightgcn_train_step_dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        f = load_golden("bpr_train_K3_d64")
        rp, col, val, nu, ni = golden_csr("g_small")
        full = CsrGraph(torch.from_numpy(rp), torch.from_numpy(col), torch.from_numpy(val),
                        (rp.size - 1, rp.size - 1), nu, ni, True)
        torch.manual_seed(56)
        m = LightGCN(nu, ni, embedding_dim=64, n_layers=3, init_scale=0.1)
        x0 = torch.cat([m.user_embedding.weight, m.item_embedding.weight]).detach()
        dg = DistributedGraph(full, rank, world, "cpu")
        emb = torch.nn.Parameter(x0[dg.row_begin:dg.row_end].clone())
        opt = torch.optim.Adam([emb], lr=1e-2, weight_decay=1e-4)
        losses = []
        for b in range(3):
            args = [torch.from_numpy(f[k][b]) for k in ("users", "pos", "neg")]
            losses.append(float(lightgcn_train_step_dist(dg, emb, 3, nu, *args, opt,
                                                         hop_fn=cpu_hop)))
        table = gather_rows(dg, emb.detach())
        if rank == 0:
            q.put((np.array(losses), table[:nu].numpy(), table[nu:].numpy()))
    finally:
        if world > 1:
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_training_matches_reference_trainer(world):
    """Three Adam steps of the row-sharded step reproduce the reference trainer's golden
    (tests/golden/bpr_train_K3_d64.npz, made by running its own code) at every world size."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    losses, uw, iw = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    f = load_golden("bpr_train_K3_d64")
    np.testing.assert_allclose(losses, f["losses"], rtol=1e-6)
    np.testing.assert_allclose(uw, f["user_w"], atol=1e-6)
    np.testing.assert_allclose(iw, f["item_w"], atol=1e-6)
