"""Multi-GPU propagation: destination-row shards + one all-gather per hop.

One process per GPU (torchrun / torch.distributed.run), backend "nccl" = RCCL over xGMI.

Partition: destination rows are split into `world` contiguous ranges balanced by nnz
(CsrGraph.partition_bounds). Rank p owns rows [b_p, b_{p+1}) of A with its CSR rebased and
its columns remapped into the *padded* all-gather layout, where global row r of rank q sits
at q*rows_pad + (r - b_q). Every rank holds the full replicated input table in that layout
([world*rows_pad, d]) and produces only its own rows.

Per hop:  Y_p = A[R_p, :] X            (local HIP SpMM, fused layer-mean epilogue)
          X' = exchange(Y_p)           (RCCL, equal-size pieces of rows_pad rows)
The exchange sends a rank's piece only to the ranks whose shard references it. For a
general graph every pair is needed and it is one all_gather_into_tensor. For the bipartite
user-item graph a user shard references only item rows and vice versa, so the pieces go as
direct point-to-point transfers (batched isend/irecv: one xGMI link per peer, all links in
parallel) and each rank receives only the opposite side: (P/2)/(P-1) of the all-gather
bytes (4/7 at 8 GPUs).
The last hop needs no gather: the layer mean stays row-sharded (scoring can be sharded by
user range); `gather_output=True` returns the full table.

The local hop is injectable (`hop_fn`, default: the native gnnrec_spmm_csr_f32 wrapper) so
the partition / gather / epilogue bookkeeping is testable on CPU ranks over gloo with the
oracle as the local hop (tests/test_distributed.py).

Feature groups (RankGrid): propagation is independent per feature column (y[:, f] = A x[:, f]
with the same fmaf chain for every f), and the column-ordered kernel already runs a hop as
d/32 independent 32-feature slices. So the ranks form a grid of F feature groups x R row
shards (rank = r * F + f): rank (r, f) propagates columns [f d/F, (f+1) d/F) of its row
shard, and the per-hop exchange runs only among the R ranks of its feature group, with 1/F
of the row bytes. At F = world (d = 64: two GPUs) no hop exchanges anything. Every edge
still costs one 128-B line per 32-feature slice on exactly one rank, so the per-rank kernel
work is 1/world of the hop either way; the exchanged bytes per rank drop from
(world-1)/world to (R-1)/R/F of the table.
"""
from __future__ import annotations

import math
from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist

from ._lib import EPI_ACC_ADD, EPI_ACC_DIV, EPI_ACC_INIT, EPI_ACC_X, EPI_NO_Y
from .graph import CsrGraph

HopFn = Callable[..., None]


def _native_hop(adj, x, y, *, epi, self_rows, acc, acc_div, x_mask=None, y_active=None,
                meet_us=None, reserve_cus=0, prev=None):
    from .functional import spmm_into
    spmm_into(adj, x, y, epi=epi, self_rows=self_rows, acc=acc, acc_div=acc_div,
              x_mask=x_mask, y_active=y_active, meet_us=meet_us, reserve_cus=reserve_cus,
              prev=prev)


class DistributedGraph:
    """This rank's shard of the operand plus the padded layout helpers."""

    def __init__(self, full: CsrGraph, rank: int, world: int, device,
                 balance: str = "nnz", group=None, exchange: str = "auto",
                 ranks: Optional[list] = None):
        """rank / world: this rank's index among the `group` ranks that shard the rows;
        ranks: their global ranks (point-to-point peers), default 0 .. world-1."""
        self.rank, self.world, self.group = rank, world, group
        self.ranks = list(ranks) if ranks is not None else list(range(world))
        if len(self.ranks) != world:
            raise ValueError("ranks must list the global rank of every row shard")
        self.device = torch.device(device)
        self.shard = full.shard(rank, world, balance).to(self.device)
        info = self.shard.shard_info
        self.bounds = info.bounds
        self.rows_pad = info.rows_pad
        self.row_begin, self.row_end = info.row_begin, info.row_end
        self.n_local = self.row_end - self.row_begin
        self.n_global = full.shape[0]
        self.needs = self._needs_matrix()
        if exchange == "auto":
            exchange = "allgather" if bool(self.needs.all()) else "p2p"
        if exchange not in ("allgather", "p2p"):
            raise ValueError(f"unknown exchange: {exchange}")
        self.exchange_mode = exchange

    def _needs_matrix(self) -> torch.Tensor:
        """needs[p, q]: rank p's shard references rows owned by rank q (all ranks agree)."""
        mine = torch.zeros(self.world, dtype=torch.int32)
        if self.shard.nnz:
            owners = torch.unique(self.shard.col.to(torch.int64) // self.rows_pad).cpu()
            mine[owners] = 1
        if self.world == 1:
            return mine.view(1, 1).bool()
        backend = dist.get_backend(self.group)
        t = mine.to(self.device) if backend != "gloo" else mine
        allm = torch.empty((self.world, self.world), dtype=torch.int32, device=t.device)
        dist.all_gather_into_tensor(allm.view(-1), t, group=self.group)
        return allm.cpu().bool()

    def recv_rows(self) -> int:
        if self.exchange_mode == "allgather":
            return (self.world - 1) * self.rows_pad
        return int(sum(self.rows_pad for q in range(self.world)
                       if q != self.rank and self.needs[self.rank, q]))

    # ---- layout ----------------------------------------------------------------------------
    def padded_index(self) -> np.ndarray:
        """Position of every global row in the padded layout."""
        b = np.asarray(self.bounds)
        r = np.arange(self.n_global)
        owner = np.searchsorted(b, r, side="right") - 1
        return owner * self.rows_pad + (r - b[owner])

    def pad_table(self, x: torch.Tensor, hop_layout: bool = False) -> torch.Tensor:
        """[N, d] global table -> [world*rows_pad, d] padded table on this rank's device.
        hop_layout (one rank, fp32): a functional.hop_table view, placed for the hops that
        gather from it (a gathered table of several ranks stays compact: RCCL writes it)."""
        if hop_layout and self.world == 1 and x.dtype == torch.float32:
            from .functional import hop_table
            out = hop_table(self.rows_pad, x.shape[1], device=self.device, zero=True)
        else:
            out = torch.zeros((self.world * self.rows_pad, x.shape[1]), dtype=x.dtype,
                              device=self.device)
        idx = torch.from_numpy(self.padded_index()).to(self.device)
        out[idx] = x.to(self.device)
        return out

    def unpad_table(self, xp: torch.Tensor) -> torch.Tensor:
        idx = torch.from_numpy(self.padded_index()).to(xp.device)
        return xp[idx]

    def local_slice(self, xp: torch.Tensor) -> torch.Tensor:
        o = self.rank * self.rows_pad
        return xp[o:o + self.n_local]

    # ---- communication ---------------------------------------------------------------------
    def exchange(self, out: torch.Tensor, piece: torch.Tensor) -> None:
        """Deliver every rank's piece to the ranks that reference it (see module doc)."""
        if self.world == 1 or self.exchange_mode == "allgather":
            return self.all_gather(out, piece)
        rp, me = self.rows_pad, self.rank
        staged = out.is_cuda and dist.get_backend(self.group) == "gloo"  # 1-GPU test harness
        src = piece.cpu() if staged else piece
        ops, landing = [], []
        for q in range(self.world):
            if q == me:
                continue
            if self.needs[q, me]:
                ops.append(dist.P2POp(dist.isend, src, self.ranks[q], self.group))
            if self.needs[me, q]:
                dst = out[q * rp:(q + 1) * rp]
                buf = torch.empty(dst.shape, dtype=dst.dtype) if staged else dst
                ops.append(dist.P2POp(dist.irecv, buf, self.ranks[q], self.group))
                landing.append((dst, buf))
        if self.needs[me, me]:
            out[me * rp:(me + 1) * rp].copy_(piece)
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        if staged:
            for dst, buf in landing:
                dst.copy_(buf)

    def chunk_bounds(self, chunks: int):
        """Row boundaries of the overlap chunks inside a rows_pad piece (multiples of 4)."""
        step = -(-self.rows_pad // chunks)
        step = -(-step // 4) * 4
        b = list(range(0, self.rows_pad, step)) + [self.rows_pad]
        return list(zip(b[:-1], b[1:]))

    def post_chunk(self, out: torch.Tensor, piece: torch.Tensor, c0: int, c1: int) -> list:
        """Start the point-to-point exchange of rows [c0, c1) of every piece (async)."""
        rp, me = self.rows_pad, self.rank
        staged = out.is_cuda and dist.get_backend(self.group) == "gloo"
        src = piece[c0:c1].cpu() if staged else piece[c0:c1]
        ops, landing = [], []
        for q in range(self.world):
            if q == me:
                continue
            if self.needs[q, me]:
                ops.append(dist.P2POp(dist.isend, src, self.ranks[q], self.group))
            if self.needs[me, q]:
                dst = out[q * rp + c0:q * rp + c1]
                buf = torch.empty(dst.shape, dtype=dst.dtype) if staged else dst
                ops.append(dist.P2POp(dist.irecv, buf, self.ranks[q], self.group))
                if staged:
                    landing.append((dst, buf))
        if self.needs[me, me]:
            out[me * rp + c0:me * rp + c1].copy_(piece[c0:c1])
        reqs = dist.batch_isend_irecv(ops) if ops else []
        return [(reqs, landing)]

    @staticmethod
    def finish(pending: list) -> None:
        for reqs, landing in pending:
            for r in reqs:
                r.wait()
            for dst, buf in landing:
                dst.copy_(buf)

    def all_gather(self, out: torch.Tensor, piece: torch.Tensor) -> None:
        if self.world == 1:
            out.copy_(piece)
        elif out.is_cuda and dist.get_backend(self.group) == "gloo":
            # test harness only (several ranks sharing one GPU): stage through the host
            host = torch.empty(out.shape, dtype=out.dtype)
            dist.all_gather_into_tensor(host, piece.cpu(), group=self.group)
            out.copy_(host)
        else:
            dist.all_gather_into_tensor(out, piece, group=self.group)


def feature_groups_for(world: int, d: int, requested: Optional[int] = None) -> int:
    """F of the rank grid: `requested` if it divides both world and the d/32 feature slices,
    else (None) the largest such divisor, gcd(world, d/32); 1 when d % 32 != 0."""
    slices = d // 32 if d % 32 == 0 else 1
    if requested is None:
        return math.gcd(world, slices)
    F = int(requested)
    if F < 1 or world % F or slices % F:
        raise ValueError(f"feature_groups={F} must divide the world ({world}) and the "
                         f"{slices} 32-feature slices of d={d}")
    return F


class RankGrid:
    """F feature groups x R row shards (module doc): rank = r * F + f owns columns
    `cols` of the rows of row shard r. `dg` is the row-shard DistributedGraph over the R
    ranks of feature group f (its exchange runs in that process group); `col_group` joins
    the F ranks of row shard r (gather_features). Every rank of the job must construct the
    grid (process groups are created collectively, in the same order everywhere)."""

    def __init__(self, full: CsrGraph, rank: int, world: int, device, d: int,
                 feature_groups: Optional[int] = None, balance: str = "nnz",
                 exchange: str = "auto"):
        F = feature_groups_for(world, d, feature_groups)
        R = world // F
        self.F, self.R, self.d = F, R, d
        self.f, self.r = rank % F, rank // F
        self.cols = (self.f * d // F, (self.f + 1) * d // F)
        row_group, self.col_group = None, None
        if world > 1 and F > 1:
            for f in range(F):
                g = dist.new_group([r * F + f for r in range(R)])
                if f == self.f:
                    row_group = g
            for r in range(R):
                g = dist.new_group([r * F + f for f in range(F)])
                if r == self.r:
                    self.col_group = g
        self.dg = DistributedGraph(full, self.r, R, device, balance, group=row_group,
                                   exchange=exchange,
                                   ranks=[r * F + self.f for r in range(R)])

    def x0_table(self, x0: torch.Tensor) -> torch.Tensor:
        """This rank's columns of the [N, d] initial table in the row shards' padded layout."""
        c0, c1 = self.cols
        return self.dg.pad_table(x0[:, c0:c1].contiguous(), hop_layout=True)

    def gather_features(self, local: torch.Tensor) -> torch.Tensor:
        """[n, d/F] column block of this rank -> [n, d] rows of its row shard (all F column
        blocks of the same rows, from the ranks of its row shard)."""
        if self.F == 1:
            return local
        local = local.contiguous()
        staged = local.is_cuda and dist.get_backend(self.col_group) == "gloo"
        src = local.cpu() if staged else local
        parts = [torch.empty_like(src) for _ in range(self.F)]
        dist.all_gather(parts, src, group=self.col_group)
        return torch.cat(parts, dim=1).to(local.device)


def lightgcn_propagate_grid(grid: RankGrid, x0_cols: torch.Tensor, n_layers: int,
                            **kw) -> torch.Tensor:
    """lightgcn_propagate_dist on the rank grid: x0_cols = grid.x0_table(x0). Returns this
    rank's [rows of its shard, d/F] block of mean(x0..xK); gather_output=True: the full
    [N, d] table on every rank."""
    gather = kw.pop("gather_output", False)
    out = lightgcn_propagate_dist(grid.dg, x0_cols, n_layers, gather_output=gather, **kw)
    return grid.gather_features(out) if gather else out


def lightgcn_propagate_dist(dg: DistributedGraph, x0_pad: torch.Tensor, n_layers: int, *,
                            gather_output: bool = False, hop_fn: Optional[HopFn] = None,
                            work: Optional[tuple] = None, overlap_chunks: int = 1,
                            masks: Optional[Callable] = None,
                            reserve_cus: int = 0,
                            deferred: Optional[bool] = None,
                            placed_output: bool = False) -> torch.Tensor:
    """LightGCN propagation over a row-sharded operand.

    x0_pad: [world*rows_pad, d] padded initial table (identical on every rank).
    Returns this rank's rows of mean(x0..xK) ([n_local, d]), or the full [N, d] table when
    gather_output, as a contiguous tensor. On one rank the deferred schedule forms the mean
    in a placed table (functional.hop_table: row stride > d, twice the compact bytes);
    placed_output=True returns that row-major strided view itself instead of a compact copy
    (bench.py's timed step: the same values, without the extra 4*d*N-byte copy).
    `work` (from `make_work`) holds reusable hop buffers. With world == 1
    the hop outputs feed the next hop directly (no gather, no copy).
    overlap_chunks > 1 (point-to-point exchange only): the hop runs in that many row chunks
    and each chunk's transfer is posted as soon as its kernel is queued, so the exchange of
    chunk c overlaps the SpMM of chunk c+1. Each chunk is a cached row view of the shard with
    its own column-ordered plan (spmm_into picks the tiled kernel for chunks of at least
    TILED_MIN_ROWS rows), launched without the pass-start meeting (RCCL kernels share the
    device while it runs).
    masks(k, x_in) -> (x_mask [padded rows], y_active [n_local]) or None: the sparse-input /
    row-subset options of the native hop (spmm_into) for hop k.
    reserve_cus (overlapped chunks): a chunk's column-ordered kernel is sized for that many
    fewer CUs than the device has (one pass of cus - reserve_cus workgroups), so the
    exchange's RCCL kernels find free CUs while it runs (the kernel takes a CU's whole LDS).
    deferred: the deferred layer mean (_propagate_deferred); None = whenever the native hop
    runs the shard on the column-ordered kernel (the only one with its epilogue); True forces
    it for an injected hop_fn that implements that epilogue (CPU tests).
    """
    hop = hop_fn or _native_hop
    # the native hop's pass-start meeting must not wait on workgroups that share the device
    # with concurrent RCCL kernels (overlapped chunks)
    # (a wrapper of the native hop — e.g. bench.py's timer — says so by a `native_hop` attribute)
    native = hop is _native_hop or getattr(hop, "native_hop", False)
    chunk_kw = {"meet_us": 0, "reserve_cus": int(reserve_cus)} if native else {}

    def mkw(k, x_in):
        m = masks(k, x_in) if masks is not None else None
        return {} if m is None else {"x_mask": m[0], "y_active": m[1]}

    d = x0_pad.shape[1]
    if work is None:
        work = make_work(dg, d, x0_pad.device)
    Y, Xa, Xb = work
    self_rows = dg.local_slice(x0_pad)
    from .functional import tiled_plan_for
    chunked = overlap_chunks > 1 and dg.world > 1 and dg.exchange_mode == "p2p"
    # the deferred layer mean (functional.lightgcn_hop_schedule): its flag hop (the last at
    # K <= 3) runs on the column-ordered kernel over the whole shard, never in chunks
    if deferred is None:
        deferred = native and tiled_plan_for(dg.shard, x0_pad) is not None
    if deferred and n_layers >= 2 and (n_layers <= 3 or not chunked):
        out = _propagate_deferred(dg, x0_pad, n_layers, hop, mkw, work, self_rows, chunked,
                                  overlap_chunks, chunk_kw, masks, gather_output)
        return out if placed_output else out.contiguous()
    acc = torch.empty((dg.n_local, d), dtype=torch.float32, device=x0_pad.device)
    if n_layers == 0:
        acc.copy_(self_rows)
    x_in = x0_pad
    for k in range(1, n_layers + 1):
        last = k == n_layers
        epi = EPI_ACC_INIT if k == 1 else EPI_ACC_ADD
        if last:
            epi |= EPI_ACC_DIV | EPI_NO_Y
        if dg.world == 1:  # ping-pong the hop outputs themselves
            y = None if last else (Xa if x_in is not Xa else Xb)
            hop(dg.shard, x_in, None if last else y[:dg.n_local], epi=epi, self_rows=self_rows,
                acc=acc, acc_div=float(n_layers + 1), **mkw(k, x_in))
            x_in = y
            continue
        if last or not chunked:
            hop(dg.shard, x_in, None if last else Y[:dg.n_local], epi=epi, self_rows=self_rows,
                acc=acc, acc_div=float(n_layers + 1), **mkw(k, x_in))
            if not last:
                x_next = Xa if x_in is not Xa else Xb
                dg.exchange(x_next, Y)
                x_in = x_next
            continue
        x_next = Xa if x_in is not Xa else Xb
        pending = []
        m = masks(k, x_in) if masks is not None else None
        for c0, c1 in dg.chunk_bounds(overlap_chunks):
            r1 = min(c1, dg.n_local)
            if r1 > c0:
                kw = {} if m is None else {"x_mask": m[0],
                                           "y_active": None if m[1] is None else m[1][c0:r1]}
                hop(dg.shard.row_slice(c0, r1), x_in, Y[c0:r1], epi=epi,
                    self_rows=self_rows[c0:r1], acc=acc[c0:r1], acc_div=float(n_layers + 1),
                    **kw, **chunk_kw)
            pending += dg.post_chunk(x_next, Y, c0, c1)
        dg.finish(pending)
        x_in = x_next
    if not gather_output:
        return acc
    if dg.world == 1:
        return acc
    Y[:dg.n_local].copy_(acc)
    full = torch.empty_like(x0_pad)
    dg.all_gather(full, Y)
    return dg.unpad_table(full)


def _propagate_deferred(dg, x0_pad, K, hop, mkw, work, self_rows, chunked, overlap_chunks,
                        chunk_kw, masks, gather_output):
    """lightgcn_propagate_dist with the deferred layer mean (functional.lightgcn_hop_schedule,
    deferred=True) on any number of ranks: hop 1 parks y1 in the output rows, the mean is
    formed once on hop 3 from x0, the parked y1 and the previous layer's own rows
    (EPI_ACC_X with an explicit `prev`: on a shard they live in this rank's exchange piece,
    not in the gathered table) — 6 instead of 8 epilogue row transfers per K=3 step, the same
    additions in the same order as the eager schedule, so the same bits.
    Buffers per schedule name: the rank's PIECE (rows_pad rows: what its hop writes and sends)
    and the GATHERED table (world * rows_pad rows: what the next hop reads). One device: they
    are the same buffer and nothing is exchanged. A mask that `masks` returns for a hop whose
    epilogue only the column-ordered kernel has (ACC_X, ACC_INIT|ACC_ADD) is dropped: a dense
    hop gives the same bits (a skipped zero row adds fmaf(v, 0, acc) = acc)."""
    from .functional import lightgcn_hop_schedule
    Y, Xa, Xb = work
    n, d, dev = dg.n_local, x0_pad.shape[1], x0_pad.device
    if dg.world == 1:
        # y1 is gathered by hop 2 straight from the output rows: pad them to the table's rows
        # and place them like a hop table (the result is then a row-major strided view)
        from .functional import hop_table
        acc_piece = hop_table(Xa.shape[0], d, device=dev)
        acc_piece[n:].zero_()
        piece = {"acc": acc_piece, "a": Xa, "b": Xb}
        gath = dict(piece)
    else:
        acc_piece = torch.zeros((dg.rows_pad, d), dtype=torch.float32, device=dev)
        # K >= 4: hop 3 reads its own input rows ("b", EPI_ACC_X's prev) while it writes "a";
        # the kernel takes prev and y as __restrict__, so the two get separate pieces
        piece = {"acc": acc_piece, "a": Y,
                 "b": Y if K <= 3 else torch.zeros_like(Y)}
        gath = {}
    acc = acc_piece[:n]
    sched = lightgcn_hop_schedule(K, deferred=True)
    readers = {k: xn for k, (xn, _, _) in enumerate(sched, start=1)}
    for k, (xn, yn, epi) in enumerate(sched, start=1):
        x_in = x0_pad if xn == "x0" else gath[xn]
        kw = mkw(k, x_in)
        if kw and (epi & EPI_ACC_X or (epi & EPI_ACC_INIT and epi & EPI_ACC_ADD)):
            kw = {}                                  # tiled-only epilogue: dense, same bits
        prev = piece[xn][:n] if (epi & EPI_ACC_X) else None
        y = piece[yn] if yn is not None else None
        needed = yn is not None and any(readers.get(j) == yn for j in range(k + 1, K + 1))
        common = dict(epi=epi, acc_div=float(K + 1))
        if dg.world == 1 or not needed:
            hop(dg.shard, x_in, None if y is None else y[:n], self_rows=self_rows, acc=acc,
                prev=prev, **common, **kw)
            continue
        target = Xa if x_in is not Xa else Xb        # never the table this hop reads
        if not chunked:
            hop(dg.shard, x_in, y[:n], self_rows=self_rows, acc=acc, prev=prev, **common, **kw)
            dg.exchange(target, y)
        else:
            pending = []
            m = masks(k, x_in) if (masks is not None and kw) else None
            for c0, c1 in dg.chunk_bounds(overlap_chunks):
                r1 = min(c1, n)
                if r1 > c0:
                    ckw = {} if m is None else {"x_mask": m[0],
                                                "y_active": None if m[1] is None else m[1][c0:r1]}
                    hop(dg.shard.row_slice(c0, r1), x_in, y[c0:r1], self_rows=self_rows[c0:r1],
                        acc=acc[c0:r1], prev=None if prev is None else prev[c0:r1], **common,
                        **ckw, **chunk_kw)
                pending += dg.post_chunk(target, y, c0, c1)
            dg.finish(pending)
        gath[yn] = target
    if not gather_output or dg.world == 1:
        return acc
    Y[:n].copy_(acc)
    full = torch.empty_like(x0_pad)
    dg.all_gather(full, Y)
    return dg.unpad_table(full)


def gather_rows(dg: DistributedGraph, local: torch.Tensor) -> torch.Tensor:
    """Collect every rank's [n_local, w] rows into the full [N, w] table (global row order)."""
    if dg.world == 1:
        return local
    w = local.shape[1]
    piece = torch.zeros((dg.rows_pad, w), dtype=local.dtype, device=local.device)
    piece[:dg.n_local].copy_(local)
    full = torch.empty((dg.world * dg.rows_pad, w), dtype=local.dtype, device=local.device)
    dg.all_gather(full, piece)
    return dg.unpad_table(full)


def _exchanged(dg: DistributedGraph, local: torch.Tensor) -> torch.Tensor:
    """This rank's [n_local, w] rows -> the padded gather table [world*rows_pad, w] holding
    every row this rank's shard references plus its own rows (one exchange)."""
    if dg.world == 1:
        return local
    piece = torch.zeros((dg.rows_pad, local.shape[1]), dtype=local.dtype, device=local.device)
    piece[:dg.n_local].copy_(local)
    table = torch.zeros((dg.world * dg.rows_pad, local.shape[1]), dtype=local.dtype,
                        device=local.device)
    dg.exchange(table, piece)
    dg.local_slice(table).copy_(local)   # own rows too (the point-to-point form skips them
    return table                         # when the shard does not reference them)


def _native_ngcf_layer(shard, x_in, x_self, layer, gs, out):
    from .functional import ngcf_layer
    blocks, perm = (gs.blocks(), gs.perm) if gs is not None else (None, None)
    ngcf_layer(shard, x_in, layer.W1.weight, layer.W1.bias, layer.W2.weight, layer.W2.bias,
               layer.activation.negative_slope, x_self=x_self, gas_blocks=blocks,
               gas_perm=perm, fused=layer.single_kernel, out=out)


def ngcf_forward_dist(dg: DistributedGraph, model, x0_pad: torch.Tensor, *,
                      gather_output: bool = False, layer_fn: Optional[Callable] = None
                      ) -> torch.Tensor:
    """NGCF / NGCFGroupShuffle eval forward over a row-sharded operand (SURVEY §8e step 2:
    the row-local epilogue runs on the shard). Per layer: the local hop + both Linear layers
    + LeakyReLU (+ GAS) with x_self = this rank's own rows of the layer input
    (gnnrec_spmm_ngcf_f32), then one exchange of the layer output. All parameters are
    replicated. Returns this rank's rows of cat(x0, x1, ..., xK) (ngcf.py:186), or the
    full table when gather_output. Bit-identical to the single-device forward (every kernel
    computes a row from that row's inputs only)."""
    layer_fn = layer_fn or _native_ngcf_layer
    gs_layers = list(getattr(model, "gs_layers", [None] * len(model.layers)))
    n = dg.n_local
    x_local = dg.local_slice(x0_pad)
    widths = [x_local.shape[1]] + [layer.W1.out_features for layer in model.layers]
    # every layer writes its column block of the final cat(x0, ..., xK) table directly
    # (placed so that the blocks the hops gather avoid the slow line offset, gather_table)
    from .functional import gather_table
    local = gather_table(n, sum(widths), sum(widths[:-1]), device=x0_pad.device)
    local[:, :widths[0]].copy_(x_local)
    c0 = widths[0]
    x_in = x0_pad
    for k, (layer, gs) in enumerate(zip(model.layers, gs_layers)):
        y = local[:, c0:c0 + widths[k + 1]]
        layer_fn(dg.shard, x_in, x_local, layer, gs, y)
        x_local = y
        c0 += widths[k + 1]
        if k + 1 < len(model.layers):
            x_in = _exchanged(dg, y)
    return gather_rows(dg, local) if gather_output else local


def _native_gat_layer(shard, feat, s_self, s_neigh, layer, *, apply_elu, epi, self_rows, acc,
                      acc_div):
    return layer.native_forward(shard, feat, s_self, s_neigh, apply_elu=apply_elu, epi=epi,
                                self_rows=self_rows, acc=acc, acc_div=acc_div)


def gat_forward_dist(dg: DistributedGraph, model, x0_pad: torch.Tensor, *,
                     gather_output: bool = False, layer_fn: Optional[Callable] = None
                     ) -> torch.Tensor:
    """GAT eval forward over a row-sharded operand (SURVEY §8e "GAT: all-gather h and the
    per-node attention scalars instead"). Per layer each rank computes the per-node values
    of its own rows only (GATLayer.native_inputs: h = x W^T for all heads, or x itself for the
    head-averaged layer, plus s_self and s_neigh), exchanges that table and s_neigh (the
    values a neighbour reads), and runs the sparse edge-softmax aggregation over its shard
    with ELU and the layer mean fused (gnnrec_gat_aggregate_f32 + heavy-row split). Returns
    this rank's rows of the layer mean (or the full table)."""
    layer_fn = layer_fn or _native_gat_layer
    x_local = dg.local_slice(x0_pad)
    acc = torch.empty_like(x_local)
    L = len(model.layers)
    for k, layer in enumerate(model.layers, start=1):
        epi = EPI_ACC_INIT if k == 1 else EPI_ACC_ADD
        if k == L:
            epi |= EPI_ACC_DIV | EPI_NO_Y   # only the layer mean is read after it
        if layer_fn is _native_gat_layer and layer.att_ok():
            # scores from the rows: only the gathered table travels (no score columns), and
            # the destination rows' own scores come from this rank's rows of it
            feat = layer.native_rows(x_local)
            x_local = layer.native_forward_att(dg.shard, _exchanged(dg, feat), feat,
                                               apply_elu=True, epi=epi, self_rows=x_local,
                                               acc=acc, acc_div=float(L + 1))
            continue
        feat, ss, sn = layer.native_inputs(x_local)
        # scores travel as their (strided) projection columns: no compaction copy, and on one
        # device the kernel reads them next to the gathered rows
        featp, snp = _exchanged(dg, feat), _exchanged(dg, sn)
        x_local = layer_fn(dg.shard, featp, ss, snp, layer, apply_elu=True, epi=epi,
                           self_rows=x_local, acc=acc, acc_div=float(L + 1))
    return gather_rows(dg, acc) if gather_output else acc


def make_work(dg: DistributedGraph, d: int, device) -> tuple:
    """Hop buffers: Y [rows_pad, d] (zero padded tail) and two [world*rows_pad, d] tables."""
    rows = dg.world * dg.rows_pad
    # world == 1 ping-pongs Xa/Xb directly, so Y is a placeholder, and the hops gather from
    # Xa/Xb themselves: functional.hop_table's placement (several ranks: RCCL writes them)
    Y = torch.zeros((dg.rows_pad if dg.world > 1 else 1, d), dtype=torch.float32, device=device)
    if dg.world == 1:
        from .functional import hop_table
        return (Y, hop_table(rows, d, device=device, zero=True),
                hop_table(rows, d, device=device, zero=True))
    return (Y, torch.zeros((rows, d), dtype=torch.float32, device=device),
            torch.zeros((rows, d), dtype=torch.float32, device=device))
