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
from conftest import golden_csr

from src.ops import CsrGraph
from src.ops._lib import EPI_ACC_ADD, EPI_ACC_DIV, EPI_ACC_INIT, EPI_NO_Y
from src.ops.distributed import DistributedGraph, lightgcn_propagate_dist


def cpu_hop(adj, x, y, *, epi, self_rows, acc, acc_div):
    """CPU stand-in for gnnrec_spmm_csr_f32 (oracle SpMM + the same epilogue order)."""
    yy = oracle.spmm(adj.row_ptr.numpy(), adj.col.numpy(), adj.val.numpy(), x.numpy())
    if not (epi & EPI_NO_Y):
        y.copy_(torch.from_numpy(yy))
    if epi & (EPI_ACC_INIT | EPI_ACC_ADD):
        b = (self_rows if epi & EPI_ACC_INIT else acc).numpy() + yy
        if epi & EPI_ACC_DIV:
            b = b / np.float32(acc_div)
        acc.copy_(torch.from_numpy(b.astype(np.float32)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, K, balance, q, exchange="auto", chunks=1):
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
        local = lightgcn_propagate_dist(dg, xp, K, hop_fn=cpu_hop, overlap_chunks=chunks)
        whole = lightgcn_propagate_dist(dg, xp, K, hop_fn=cpu_hop, gather_output=True,
                                        overlap_chunks=chunks)
        if rank == 0:
            ref = oracle.lightgcn(rp, col, val, x0.numpy(), K)
            q.put((whole.numpy(), ref, local.numpy(), ref[dg.row_begin:dg.row_end],
                   dg.exchange_mode, dg.needs.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,K,balance,exchange,chunks", [
    (2, 3, "nnz", "auto", 1), (3, 2, "rows", "auto", 1), (2, 1, "nnz", "allgather", 1),
    (4, 3, "nnz", "auto", 1), (4, 2, "nnz", "allgather", 1), (4, 3, "nnz", "p2p", 3),
    (3, 3, "rows", "p2p", 4)])
def test_sharded_propagation_matches_single_device(world, K, balance, exchange, chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, K, balance, q, exchange, chunks))
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


def test_partition_bounds_balance_nnz():
    rp = np.array([0, 10, 10, 11, 30, 31, 32, 40], dtype=np.int64)
    b = CsrGraph.partition_bounds(rp, 2)
    assert b[0] == 0 and b[-1] == 7
    loads = [rp[b[i + 1]] - rp[b[i]] for i in range(2)]
    assert max(loads) <= 30
    assert CsrGraph.partition_bounds(rp, 7, "rows") == tuple(range(8))
