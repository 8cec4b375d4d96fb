"""bench.py's multi-rank bookkeeping on CPU ranks over gloo.

The driver runs `bench.py --gpus N` with no flags, so at N > 1 the line must check itself:
`--verify` defaults on, every rank compares its block with a single-device propagation and
the flags are MIN-reduced into `all_ranks_bit_exact`. The exchange forms are probed in
lock-step before any timed collective (the pre-flight). Here the single-device reference is
the CPU oracle and the sharded result comes from lightgcn_propagate_grid with the oracle as
the local hop (tests/test_distributed.py's stand-in), so everything but the HIP kernel runs.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
import oracle
from conftest import golden_csr
from test_distributed import cpu_hop

from src.ops import CsrGraph
from src.ops.distributed import RankGrid, lightgcn_propagate_grid


def test_verify_defaults_on_for_several_ranks():
    assert bench.resolve_verify(None, 2) is True
    assert bench.resolve_verify(None, 8) is True
    assert bench.resolve_verify(None, 1) is False
    assert bench.resolve_verify(False, 8) is False      # --no-verify
    assert bench.resolve_verify(True, 1) is True        # --verify


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_reference(full, x0, K, device):
    rp, col, val = full.row_ptr.numpy(), full.col.numpy(), full.val.numpy()
    return torch.from_numpy(oracle.lightgcn(rp, col, val, x0.numpy(), K))


def _worker(rank, world, port, fg, corrupt, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rp, col, val, nu, ni = golden_csr("g_small")
        full = CsrGraph(torch.from_numpy(rp), torch.from_numpy(col), torch.from_numpy(val),
                        (rp.size - 1, rp.size - 1), nu, ni, True)
        torch.manual_seed(3)
        x0 = torch.randn(full.shape[0], 64) * 0.1
        grid = RankGrid(full, rank, world, "cpu", 64, fg)
        xc = grid.x0_table(x0)
        # the pre-flight: both exchange forms on a small piece, every rank in lock-step
        probed = []
        if grid.dg.world > 1:
            for mode in ("allgather", "p2p"):
                bench.probe_exchange(grid.dg, mode, xc)
                probed.append(mode)
        out = lightgcn_propagate_grid(grid, xc, 3, hop_fn=cpu_hop, deferred=True)
        if corrupt and rank == world - 1:
            out = out.clone()
            out.view(-1)[0] += 1.0
        check = bench.verify(grid.dg, full, x0, 3, out, torch.device("cpu"), grid.cols, world,
                             reference_fn=_oracle_reference)
        q.put((rank, check, probed, grid.dg.exchange_mode, grid.dg.rows_pad))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fg,corrupt", [(2, 1, False), (2, 2, False), (2, 1, True),
                                              (4, 2, False)])
def test_multi_rank_line_carries_all_ranks_bit_exact(world, fg, corrupt):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fg, corrupt, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, check, probed, mode, rows_pad in res:
        assert "all_ranks_bit_exact" in check
        assert check["all_ranks_bit_exact"] is (not corrupt)
        assert check["bit_exact_vs_single_device"] is (not (corrupt and rank == world - 1))
        if world // fg > 1:
            assert probed == ["allgather", "p2p"]
        # the probe leaves the layout as it found it
        assert mode in ("allgather", "p2p") and rows_pad > 8
