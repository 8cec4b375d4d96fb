"""CsrGraph: the device-resident graph operand of the propagation kernels.

The reference keeps the normalised adjacency as a scipy COO matrix, re-wraps it into an
uncoalesced int64 ``torch.sparse_coo_tensor`` on every ``get_torch_adjacency()`` call
(data/dataset.py:472-491, data/graph_builder.py:147-174) and copies it host->device every
epoch (training/trainer.py:233-234). Here the operand is built once, natively, as CSR over
destination rows and stays resident in HBM:

    row_ptr  int64 [n_rows + 1]  absolute offsets
    col      int32 [nnz]         ascending inside each row (what makes SpMM bit-exact)
    val      fp32  [nnz]         fl32(fl32(dis[r] * a_rc) * dis[c]), as scipy computes it

That is 8 B per nonzero instead of the reference's 20 B (two int64 indices + fp32 value).
A CsrGraph quacks like the reference's adjacency where the models look at it
(``.is_sparse``, ``.shape``, ``.size()``, ``.device``, ``.to()``), so it can be passed
wherever ``adj_matrix`` is expected.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Tuple

import numpy as np
import torch

from . import _lib

# where a device-resident graph's column-ordered plan is built ("device" | "host"; the same
# arrays either way)
TILED_PLANNER = "device"
# gnnrec_tiled_plan_device error words: 1 negative column (the host planner's EINVAL),
# 2 scratch too small, 3 a run (one row's slots in one step) longer than 32 767, 4 count / emit
# disagree
_DEVICE_PLAN_ERRORS = {1: ValueError}
# slots of one step (a panel of a block) the device planner's scratch is sized for first
TILED_PLAN_STEP_CAP = 32768
# longest row tiled_plan() accepts: a row's slots are merged into streams by one lane, so a
# power-law operand's hub rows make planning serial (config 5's 5M x 5M rows of degree
# 2 049-65 536: 24 s; with its 1.48M-degree row: not done in 5 minutes,
# profiles/r05/c12_heavy_tiled.jsonl). The SpMM itself never plans rows past
# functional.TILED_MAX_DEGREE = 4 096 (they take the CSR kernel). 32 767 also bounds a run
# (one row's slots in one step), which the device planner keeps in 16 bits.
TILED_PLAN_MAX_DEGREE = 32767
# factored plans (gnnrec_tiled_plan_factor, DESIGN.md §3.1c "plan values"): a device graph's
# plan carries 1-byte column classes instead of fp32 values whenever every value is
# fl(dis_r * dis_c) with dis from the row counts and at most TILED_MAX_CLASSES distinct dis
TILED_FACTOR = True


class _ScratchTooSmall(Exception):
    pass


def _np(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy()


def inv_sqrt_degrees(deg: np.ndarray, normalization: str = "symmetric") -> np.ndarray:
    """Degree scaling exactly as graph_builder.py:111-131 (numpy float32 power)."""
    deg = np.maximum(np.asarray(deg, dtype=np.float32), np.float32(1.0))
    if normalization == "symmetric":
        d = np.power(deg, np.float32(-0.5))
    elif normalization == "row":
        d = np.power(deg, np.float32(-1.0))
    else:
        raise ValueError(f"unknown normalization: {normalization}")
    d[np.isinf(d)] = 0.0
    return d.astype(np.float32, copy=False)


@dataclass
class ShardInfo:
    """Destination-row shard of a partitioned graph (multi-GPU)."""
    rank: int
    world: int
    row_begin: int          # first global row owned by this shard
    row_end: int            # one past the last
    rows_pad: int           # rows per rank in the padded all-gather layout
    bounds: Tuple[int, ...]  # row boundaries of every rank (len world+1)


@dataclass
class CsrGraph:
    row_ptr: torch.Tensor
    col: torch.Tensor
    val: torch.Tensor
    shape: Tuple[int, int]
    n_users: Optional[int] = None
    n_items: Optional[int] = None
    symmetric: bool = False
    shard_info: Optional[ShardInfo] = None
    _transpose: Optional["CsrGraph"] = field(default=None, repr=False)
    _plans: dict = field(default_factory=dict, repr=False)

    # ---- reference-adjacency look-alike -------------------------------------------
    is_sparse = True

    @property
    def device(self) -> torch.device:
        return self.val.device

    @property
    def nnz(self) -> int:
        return int(self.col.numel())

    @property
    def n_rows(self) -> int:
        return int(self.row_ptr.numel() - 1)

    def size(self, dim: Optional[int] = None):
        s = torch.Size(self.shape)
        return s if dim is None else s[dim]

    def _nonzero_count(self) -> int:
        return self.nnz

    def to(self, device, non_blocking: bool = False) -> "CsrGraph":
        device = torch.device(device)
        if device == self.device:
            return self
        g = CsrGraph(self.row_ptr.to(device, non_blocking=non_blocking),
                     self.col.to(device, non_blocking=non_blocking),
                     self.val.to(device, non_blocking=non_blocking), self.shape, self.n_users,
                     self.n_items, self.symmetric, self.shard_info)
        f = self._plans.get("degree_factors")
        if f is not None:   # a shard's factors come from its full graph (shard())
            g._plans["degree_factors"] = tuple(t.to(device) for t in f)
        if "pattern_sym" in self._plans:
            g._plans["pattern_sym"] = self._plans["pattern_sym"]
        return g

    def pattern_symmetric(self) -> bool:
        """The sparsity pattern equals its transpose's (values ignored; cached): True without
        a check for the interaction graphs the builders make (both directions stored,
        graph_builder.py:52-61), else compared with t() once. The native GAT backward walks
        a node's row as the list of rows that aggregate it, which needs this."""
        if "pattern_sym" not in self._plans:
            if self.shard_info is not None or self.shape[0] != self.shape[1]:
                v = False
            elif self.symmetric:
                v = True
            else:
                tt = self.t()
                v = bool(torch.equal(tt.row_ptr.cpu(), self.row_ptr.cpu())
                         and torch.equal(tt.col.cpu(), self.col.cpu()))
            self._plans["pattern_sym"] = v
        return self._plans["pattern_sym"]

    def cuda(self, device=None) -> "CsrGraph":
        return self.to(torch.device("cuda") if device is None else torch.device("cuda", device)
                       if isinstance(device, int) else device)

    def cpu(self) -> "CsrGraph":
        return self.to("cpu")

    def validate(self) -> None:
        """Host-side structural checks (the kernels trust the operand)."""
        rp = _np(self.row_ptr)
        col = _np(self.col)
        if rp.shape[0] != self.shape[0] + 1 and self.shard_info is None:
            raise ValueError("row_ptr length must be n_rows + 1")
        if np.any(np.diff(rp) < 0):
            raise ValueError("row_ptr must be non-decreasing")
        if rp[-1] - rp[0] != col.shape[0] or self.val.numel() != col.shape[0]:
            raise ValueError("row_ptr span, col and val sizes disagree")
        if col.size and (col.min() < 0 or col.max() >= self.shape[1]):
            raise ValueError("column index out of range")
        rows = np.repeat(np.arange(rp.shape[0] - 1), np.diff(rp))
        bad = (np.diff(col.astype(np.int64)) <= 0) & (rows[1:] == rows[:-1])
        if np.any(bad):
            raise ValueError("columns must be strictly ascending within each row")

    # ---- construction ---------------------------------------------------------------
    @classmethod
    def from_interactions(cls, users, items, n_users: int, n_items: int,
                          normalization: str = "symmetric", self_loop: bool = False,
                          n_threads: int = 0, device="cpu", binary: bool = False) -> "CsrGraph":
        """Native equivalent of build_bipartite_graph + normalize_adjacency_matrix
        (graph_builder.py:16-144) for interaction lists; identical values and order.
        Duplicate pairs are summed like the reference (weight 2) unless `binary`."""
        u = np.ascontiguousarray(np.asarray(users, dtype=np.int64))
        i = np.ascontiguousarray(np.asarray(items, dtype=np.int64))
        if u.shape != i.shape:
            raise ValueError("users and items must have the same length")
        N = int(n_users) + int(n_items)
        cap = 2 * u.shape[0] + (N if self_loop else 0)
        row_ptr = np.empty(N + 1, np.int64)
        col = np.empty(max(cap, 1), np.int32)
        cnt = np.empty(max(cap, 1), np.float32)
        deg = np.empty(max(N, 1), np.float32)
        nnz = np.zeros(1, np.int64)
        L = _lib.lib()
        _lib.check(L.gnnrec_build_bipartite_csr(
            u.ctypes.data, i.ctypes.data, u.shape[0], int(n_users), int(n_items),
            (1 if self_loop else 0) | (2 if binary else 0),
            row_ptr.ctypes.data, col.ctypes.data, cnt.ctypes.data, deg.ctypes.data,
            nnz.ctypes.data, int(n_threads)), "build_bipartite_csr")
        nnz = int(nnz[0])
        col, cnt, deg = col[:nnz], cnt[:nnz], deg[:N]
        if normalization == "none":
            val = cnt
        else:
            dis = inv_sqrt_degrees(deg, normalization)
            val = np.empty(max(nnz, 1), np.float32)[:nnz]
            _lib.check(L.gnnrec_normalize_values(
                row_ptr.ctypes.data, col.ctypes.data, cnt.ctypes.data, N, dis.ctypes.data,
                0 if normalization == "symmetric" else 1, val.ctypes.data, int(n_threads)),
                "normalize_values")
        # D^-1/2 A D^-1/2 is symmetric in exact arithmetic; its fp32 values fl(fl(dis_r a) dis_c)
        # are bitwise symmetric only when every multiplicity a is a power of two (then
        # fl(dis_r a) is exact and the two products commute) — otherwise A^T is built
        # explicitly for backward (t()), as torch.sparse.mm's autograd transposes the stored
        # values.
        sym = normalization == "none" or (normalization == "symmetric" and bool(
            nnz == 0 or np.all(np.frexp(cnt)[0] == 0.5)))
        g = cls(torch.from_numpy(row_ptr), torch.from_numpy(col), torch.from_numpy(val), (N, N),
                int(n_users), int(n_items), symmetric=sym)
        g._plans["pattern_sym"] = True      # both directions of every pair are stored
        return g.to(device)

    @classmethod
    def from_interactions_device(cls, users, items, n_users: int, n_items: int,
                                 normalization: str = "symmetric", self_loop: bool = False,
                                 binary: bool = False, device="cuda") -> "CsrGraph":
        """from_interactions built in HBM: sort-based CSR construction and the
        value products run on the GPU (gnnrec_build_bipartite_csr_device /
        gnnrec_normalize_values_device); only the N degrees make a host round trip for the
        numpy float32 power of graph_builder.py:119. Bit-identical to from_interactions."""
        dev = torch.device(device)
        if dev.type != "cuda":
            raise ValueError("from_interactions_device needs a ROCm device")
        u = torch.as_tensor(users, dtype=torch.int64).to(dev).contiguous()
        i = torch.as_tensor(items, dtype=torch.int64).to(dev).contiguous()
        if u.shape != i.shape or u.dim() != 1:
            raise ValueError("users and items must be 1-D and of the same length")
        N = int(n_users) + int(n_items)
        P = u.numel()
        cap = max(2 * P + (N if self_loop else 0), 1)
        flags = (1 if self_loop else 0) | (2 if binary else 0)
        L = _lib.lib()
        stream = _lib.stream_of(dev)
        row_ptr = torch.empty(N + 1, dtype=torch.int64, device=dev)
        col = torch.empty(cap, dtype=torch.int32, device=dev)
        cnt = torch.empty(cap, dtype=torch.float32, device=dev)
        deg = torch.empty(max(N, 1), dtype=torch.float32, device=dev)
        nbytes = _lib.C.c_size_t(0)
        nnz = _lib.C.c_int64(0)
        args = [_lib.ptr(u), _lib.ptr(i), P, int(n_users), int(n_items), flags,
                _lib.ptr(row_ptr), _lib.ptr(col), _lib.ptr(cnt), _lib.ptr(deg)]
        _lib.check(L.gnnrec_build_bipartite_csr_device(*args, _lib.C.addressof(nnz), None,
                                                        _lib.C.addressof(nbytes), stream),
                   "build_bipartite_csr_device")
        work = torch.empty(max(int(nbytes.value), 1), dtype=torch.uint8, device=dev)
        _lib.check(L.gnnrec_build_bipartite_csr_device(*args, _lib.C.addressof(nnz),
                                                        _lib.ptr(work), _lib.C.addressof(nbytes),
                                                        stream), "build_bipartite_csr_device")
        del work
        nz = int(nnz.value)
        col, cnt = col[:nz], cnt[:nz]
        if normalization == "none" or nz == 0:
            val = cnt
        else:
            dis = torch.from_numpy(inv_sqrt_degrees(deg[:N].cpu().numpy(), normalization)).to(dev)
            val = torch.empty(max(nz, 1), dtype=torch.float32, device=dev)[:nz]
            _lib.check(L.gnnrec_normalize_values_device(
                _lib.ptr(row_ptr), _lib.ptr(col), _lib.ptr(cnt), N, _lib.ptr(dis),
                0 if normalization == "symmetric" else 1, _lib.ptr(val), stream),
                "normalize_values_device")
        sym = normalization == "none" or (normalization == "symmetric" and bool(
            nz == 0 or torch.all(torch.frexp(cnt).mantissa == 0.5)))   # as from_interactions
        g = cls(row_ptr, col.clone(), val.clone(), (N, N), int(n_users), int(n_items),
                symmetric=sym)
        g._plans["pattern_sym"] = True      # both directions of every pair are stored
        return g

    @classmethod
    def from_scipy(cls, adj, n_users: Optional[int] = None, n_items: Optional[int] = None,
                   symmetric: Optional[bool] = None, device="cpu") -> "CsrGraph":
        """From any scipy sparse matrix (e.g. the reference's norm_adj_matrix)."""
        import scipy.sparse as sp
        csr = sp.csr_matrix(adj, dtype=np.float32, copy=True)
        csr.sum_duplicates()
        csr.sort_indices()
        if csr.shape[1] >= 2 ** 31:
            raise ValueError("more than 2^31 columns")
        if symmetric is None:
            symmetric = csr.shape[0] == csr.shape[1] and (abs(csr - csr.T) > 0).nnz == 0
        g = cls(torch.from_numpy(csr.indptr.astype(np.int64)),
                torch.from_numpy(csr.indices.astype(np.int32)),
                torch.from_numpy(csr.data.astype(np.float32)), tuple(csr.shape), n_users,
                n_items, bool(symmetric))
        return g.to(device)

    @classmethod
    def from_torch_sparse(cls, adj: torch.Tensor, symmetric: Optional[bool] = None,
                          n_users: Optional[int] = None,
                          n_items: Optional[int] = None) -> "CsrGraph":
        """From a torch COO/CSR tensor, on its own device (coalesced: duplicates summed)."""
        if adj.layout == torch.sparse_csr:
            crow, colv, val = adj.crow_indices(), adj.col_indices(), adj.values()
            n_rows = adj.shape[0]
        else:
            a = adj.coalesce()
            idx, val = a.indices(), a.values()
            n_rows = a.shape[0]
            crow = torch.zeros(n_rows + 1, dtype=torch.int64, device=idx.device)
            crow[1:] = torch.cumsum(torch.bincount(idx[0], minlength=n_rows), 0)
            colv = idx[1]
        g = cls(crow.to(torch.int64).contiguous(), colv.to(torch.int32).contiguous(),
                val.to(torch.float32).contiguous(), tuple(adj.shape), n_users, n_items,
                bool(symmetric) if symmetric is not None else False)
        if symmetric is None:
            g.symmetric = g.is_symmetric()
        return g

    # ---- conversion -------------------------------------------------------------------
    def to_scipy(self):
        import scipy.sparse as sp
        rp = _np(self.row_ptr)
        return sp.csr_matrix((_np(self.val), _np(self.col).astype(np.int64), rp - rp[0]),
                             shape=(rp.shape[0] - 1, self.shape[1]))

    def to_torch_sparse_coo(self) -> torch.Tensor:
        """The reference's operand layout (graph_builder.py:163-172), uncoalesced flag."""
        rp = self.row_ptr
        counts = (rp[1:] - rp[:-1])
        rows = torch.repeat_interleave(torch.arange(counts.numel(), device=rp.device), counts)
        idx = torch.stack([rows, self.col.to(torch.int64)])
        return torch.sparse_coo_tensor(idx, self.val, (counts.numel(), self.shape[1]))

    def is_symmetric(self) -> bool:
        if self.shape[0] != self.shape[1] or self.shard_info is not None:
            return False
        s = self.to_scipy()
        return (abs(s - s.T) > 0).nnz == 0

    def t(self) -> "CsrGraph":
        """A^T as a CsrGraph (cached); A itself when the operand is symmetric."""
        if self.symmetric:
            return self
        if self._transpose is None:
            st = self.to_scipy().T.tocsr()
            st.sort_indices()
            self._transpose = CsrGraph.from_scipy(st, self.n_items, self.n_users, False,
                                                  device=self.device)
            self._transpose._transpose = self
        return self._transpose

    # ---- multi-GPU partition -----------------------------------------------
    @staticmethod
    def partition_bounds(row_ptr: np.ndarray, world: int, balance: str = "nnz") -> Tuple[int, ...]:
        """Contiguous destination-row ranges, balanced by nnz (default) or by rows."""
        n = row_ptr.shape[0] - 1
        if balance == "rows":
            b = [min(n, (n * p + world - 1) // world) for p in range(world + 1)]
        else:
            total = row_ptr[-1] - row_ptr[0]
            targets = row_ptr[0] + (total * np.arange(world + 1)) // max(world, 1)
            b = list(np.searchsorted(row_ptr, targets, side="left").clip(0, n))
            b[0], b[-1] = 0, n
            for p in range(1, world + 1):
                b[p] = max(b[p], b[p - 1])
        return tuple(int(v) for v in b)

    def shard(self, rank: int, world: int, balance: str = "nnz") -> "CsrGraph":
        """Rows [b_rank, b_rank+1) with columns remapped into the padded all-gather layout
        (global row r of rank p lives at p*rows_pad + (r - b_p))."""
        rp = _np(self.row_ptr)
        bounds = self.partition_bounds(rp, world, balance)
        rows_pad = max(bounds[p + 1] - bounds[p] for p in range(world))
        rows_pad = max(1, (rows_pad + 3) // 4 * 4)
        lo, hi = bounds[rank], bounds[rank + 1]
        k0, k1 = int(rp[lo]), int(rp[hi])
        if world == 1:  # identity layout: nothing to remap
            col_t, val_t, rp_t = self.col, self.val, self.row_ptr
        else:
            col = _np(self.col)[k0:k1].astype(np.int64)
            owner = np.searchsorted(np.asarray(bounds), col, side="right") - 1
            col = owner * rows_pad + (col - np.asarray(bounds)[owner])
            col_t = torch.from_numpy(col.astype(np.int32))
            val_t = self.val.detach().cpu()[k0:k1].clone()
            rp_t = torch.from_numpy(rp[lo:hi + 1] - k0)
        g = CsrGraph(rp_t, col_t, val_t, (hi - lo, rows_pad * world),
                     self.n_users, self.n_items, False,
                     ShardInfo(rank, world, lo, hi, rows_pad, bounds))
        f = self.degree_factors() if world > 1 else None
        if f is not None:
            # the full graph's factors in the shard's layout: its rows, and the column classes
            # moved to the padded gather layout (padding columns are never referenced)
            rowf, cc, table = (t.cpu() for t in f)
            pad = torch.zeros(rows_pad * world, dtype=torch.uint8)
            for q in range(world):
                pad[q * rows_pad:q * rows_pad + bounds[q + 1] - bounds[q]] = \
                    cc[bounds[q]:bounds[q + 1]]
            g._plans["degree_factors"] = (rowf[lo:hi].clone(), pad, table)
        return g.to(self.device)

    def row_slice(self, r0: int, r1: int) -> "CsrGraph":
        """View of rows [r0, r1) (row_ptr keeps absolute offsets: no copy of col/val). Cached,
        so per-view plans (heavy rows) are computed once."""
        key = ("slice", r0, r1)
        if key not in self._plans:
            v = CsrGraph(self.row_ptr[r0:r1 + 1], self.col, self.val,
                         (r1 - r0, self.shape[1]), self.n_users, self.n_items,
                         False, self.shard_info)
            f = self.degree_factors()
            v._plans["degree_factors"] = None if f is None else (f[0][r0:r1], f[1], f[2])
            self._plans[key] = v
        return self._plans[key]

    def heavy_rows(self, threshold: int) -> Optional[torch.Tensor]:
        """int64 ids of the rows with more than `threshold` neighbours on this device, longest
        first (they start first and finish last), or None (cached): the SpMM's
        workgroup-per-row bucket."""
        key = ("heavy_rows", threshold)
        if key not in self._plans:
            deg = self.row_ptr[1:] - self.row_ptr[:-1]
            rows = torch.nonzero(deg > threshold).flatten().to(torch.int64)
            rows = rows[torch.argsort(deg[rows], descending=True, stable=True)]
            self._plans[key] = rows.contiguous() if rows.numel() else None
        return self._plans[key]

    def heavy_rows_longer(self, threshold: int, length: int) -> int:
        """How many of heavy_rows(threshold) have more than `length` neighbours (a prefix of
        that longest-first list; cached): the rows the SpMM runs as feature slices."""
        key = ("heavy_rows_longer", threshold, length)
        if key not in self._plans:
            rows = self.heavy_rows(threshold)
            if rows is None:
                self._plans[key] = 0
            else:
                deg = self.row_ptr[rows + 1] - self.row_ptr[rows]
                self._plans[key] = int((deg > length).sum())
        return self._plans[key]

    def light_avg_degree(self, threshold: int) -> float:
        """Mean neighbours of the rows not in heavy_rows(threshold) (cached): picks the
        row-parallel chain's form on large operands (functional.light_form_flag)."""
        key = ("light_avg_degree", threshold)
        if key not in self._plans:
            rows = self.heavy_rows(threshold) if threshold > 0 else None
            heavy_nnz, n_heavy = 0, 0
            if rows is not None:
                heavy_nnz = int((self.row_ptr[rows + 1] - self.row_ptr[rows]).sum())
                n_heavy = rows.numel()
            self._plans[key] = (self.nnz - heavy_nnz) / max(self.n_rows - n_heavy, 1)
        return self._plans[key]

    def row_stats(self, block_rows: int = 0) -> Tuple[int, int]:
        """(longest row, most edges in a block of block_rows consecutive rows): on a device
        graph one gnnrec_csr_row_stats launch and an 16-B read (no torch kernels, whose first
        launches in a fresh process cost ~0.1 s each to load), on the host numpy."""
        if self.n_rows == 0:
            return 0, 0
        if self.device.type == "cuda":
            out = torch.empty(2, dtype=torch.int64, device=self.device)
            _lib.check(_lib.lib().gnnrec_csr_row_stats(_lib.ptr(self.row_ptr), self.n_rows,
                                                       int(block_rows), _lib.ptr(out),
                                                       _lib.stream_of(self.device)),
                       "gnnrec_csr_row_stats")
            a, b = out.cpu().tolist()
            return int(a), int(b)
        rp = self.row_ptr.numpy()
        mb = 0
        if block_rows > 0:
            starts = np.arange(0, self.n_rows, block_rows)
            mb = int((rp[np.minimum(starts + block_rows, self.n_rows)] - rp[starts]).max())
        return int(np.diff(rp).max()), mb

    def max_degree(self) -> int:
        """Longest row (cached; one device read the first time)."""
        if "max_degree" not in self._plans:
            self._plans["max_degree"] = self.row_stats()[0]
        return self._plans["max_degree"]

    def tiled_plan(self, rows_per_block: int = 1117, panel: int = 49152,
                   sub_panel: int = 4096, planner: Optional[str] = None) -> dict:
        """Column-ordered re-layout of this operand for gnnrec_spmm_tiled_f32 (DESIGN.md
        §3.1c), cached; one plan serves every x table (any d that is a multiple of 32, any row
        stride up to TILED_MAX_LDX, any size). planner: "device" builds it in HBM from the
        device CSR (gnnrec_tiled_plan_device, the default for a graph on a GPU), "host" on the
        host from the CSR (gnnrec_tiled_plan_build/emit) and uploads it; both give the same
        arrays bit for bit (tests/test_tiled_plan_gpu.py). Defaults from the G100M sweeps
        (profiles/r02/tiled_sweep.jsonl, profiles/r03/sweep_R_*.jsonl): 1117 rows per block
        fill the LDS with 32-feature accumulators in 14 full passes, 48K-column panels
        (steps: a workgroup barrier each, which keeps its waves on nearby columns), each
        stream's slots in ascending 4K-column sub-panels inside a step (0: no sub-panel
        order)."""
        key = ("tiled", int(rows_per_block), int(panel), int(sub_panel))
        if key not in self._plans:
            if self.max_degree() > TILED_PLAN_MAX_DEGREE:
                raise ValueError(
                    f"tiled_plan: a row of {self.max_degree()} neighbours (> "
                    f"TILED_PLAN_MAX_DEGREE = {TILED_PLAN_MAX_DEGREE}); rows that long are "
                    "planned serially — the SpMM runs such operands on the CSR kernel")
            import time
            cuda = self.device.type == "cuda"

            def now():
                if cuda:
                    torch.cuda.synchronize(self.device)
                return time.perf_counter()
            if planner is None:
                planner = TILED_PLANNER if cuda else "host"
            t0 = now()
            if planner == "device":
                plan = self._tiled_plan_device(int(rows_per_block), int(panel), int(sub_panel))
            elif planner == "host":
                plan = self._tiled_plan_host(int(rows_per_block), int(panel), int(sub_panel))
            else:
                raise ValueError(f"unknown planner {planner!r}")
            plan.update(rows_per_block=int(rows_per_block),
                        panel=min(int(panel), _lib.TILED_MAX_PANEL), sub_panel=int(sub_panel),
                        n_slots=plan["n_chunks"] * _lib.TILED_CHUNK,
                        sync=torch.zeros(_lib.TILED_SYNC_WORDS, dtype=torch.int32,
                                         device=self.device))
            t1 = now()
            build_s = {"planner": planner, "plan_s": t1 - t0}
            if "planner_phases" in plan:
                build_s["planner_phases"] = plan.pop("planner_phases")
            if (TILED_FACTOR and cuda
                    and int(rows_per_block) <= _lib.TILED_MAX_ROWS_FACTORED):
                self.degree_factors()
                t2 = now()
                factored = self._factor_plan(plan)
                t3 = now()
                build_s.update(degree_factors_s=t2 - t1, factor_check_s=t3 - t2,
                               factored=bool(factored))
            if cuda and _lib.lib().gnnrec_tiled_plan_quad():
                t4 = now()
                self._quad_plan(plan)
                build_s["quad_layout_s"] = now() - t4
            # phase times of this build (each phase synchronised): bench.py reports them
            plan["build_s"] = build_s
            self._plans[key] = plan
        return self._plans[key]

    def degree_factors(self):
        """(row_factor [n_rows], col_class uint8 [n_cols], class_table [n_classes]) on this
        device, or None (cached): the symmetric normalisation's dis = float32(deg)^-0.5 exactly
        as inv_sqrt_degrees (graph_builder.py:111-131) with deg = the row's stored-entry
        count (a binary interaction graph), when the operand is square and dis takes at most
        TILED_MAX_CLASSES distinct values. A guess: gnnrec_tiled_plan_factor checks every
        value against it bit for bit before a plan drops its values."""
        if "degree_factors" not in self._plans:
            out = None
            n, m = self.shape
            info = self.shard_info
            # node-indexed columns: a square operand, or the identity layout of one shard
            # (columns padded to a multiple of 4); shards of several ranks get theirs from
            # their full graph (shard())
            node_cols = (n == m and info is None) or (info is not None and info.world == 1
                                                      and m >= n)
            if node_cols and self.row_ptr.numel() == n + 1 and self.nnz > 0:
                # dis per DISTINCT degree on the host (numpy float32 power, as before), spread to
                # the rows on the operand's device: the rows' degrees never leave it
                dev = self.device
                udeg, inv = torch.unique(self.row_ptr[1:] - self.row_ptr[:-1], sorted=True,
                                         return_inverse=True)
                dis_u = inv_sqrt_degrees(udeg.cpu().numpy().astype(np.float32), "symmetric")
                table = np.unique(dis_u)
                if table.size <= _lib.TILED_MAX_CLASSES:
                    cls_u = torch.from_numpy(np.searchsorted(table, dis_u).astype(np.uint8)).to(dev)
                    cls = torch.zeros(m, dtype=torch.uint8, device=dev)
                    cls[:n] = cls_u[inv]
                    out = (torch.from_numpy(dis_u).to(dev)[inv].contiguous(), cls,
                           torch.from_numpy(table).to(dev))
            self._plans["degree_factors"] = out
        return self._plans["degree_factors"]

    def _factor_plan(self, plan: dict) -> bool:
        """Replace the plan's fp32 values by 1-byte column classes when every real slot's value
        is fl(row_factor[r] * class_table[class]) bit for bit (gnnrec_tiled_plan_factor);
        otherwise the plan keeps its values. Returns whether it was factored."""
        f = self.degree_factors()
        if f is None:
            return False
        rowf, col_class, table = f
        L = _lib.lib()
        dev = self.device
        cls = torch.zeros(plan["slot"].numel(), dtype=torch.uint8, device=dev)
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.check(L.gnnrec_tiled_plan_factor(
            _lib.ptr(plan["slot"]), _lib.ptr(plan["val"]), _lib.ptr(plan["hdr"]),
            _lib.ptr(plan["wave_ptr"]), plan["n_blocks"], plan["rows_per_block"], self.n_rows,
            self.shape[1], _lib.ptr(rowf), _lib.ptr(col_class), _lib.ptr(table), table.numel(),
            _lib.ptr(cls), _lib.ptr(bad), _lib.stream_of(dev)), "gnnrec_tiled_plan_factor")
        if int(bad):
            return False
        del plan["val"]
        plan.update(cls=cls, row_factor=rowf, class_table=table, n_classes=int(table.numel()))
        return True

    @staticmethod
    def _quad_plan(plan: dict) -> None:
        """The quad-interleaved layout the kernel reads (ABI 9, gnnrec_tiled_plan_quad):
        gnnrec_tiled_plan_quad_offsets pads every wave's chunk range to a multiple of 4,
        gnnrec_tiled_plan_quad_layout moves the chunks there (empty chunks after them and in
        TILED_QUAD_TAIL tail chunks) and interleaves the slot words and class bytes / values
        of 4 chunks per lane. Headers stay chunk-major."""
        L = _lib.lib()
        ptr = _lib.ptr
        CH = _lib.TILED_CHUNK
        wp = plan["wave_ptr"]
        dev = wp.device
        stream = _lib.stream_of(dev)
        n_waves = wp.numel() - 1
        wq = torch.empty_like(wp)
        _lib.check(L.gnnrec_tiled_plan_quad_offsets(ptr(wp), n_waves, ptr(wq), stream),
                   "gnnrec_tiled_plan_quad_offsets")
        total = int(wq[-1])
        alloc = total + _lib.TILED_QUAD_TAIL
        fact = "cls" in plan
        slot = torch.empty(alloc * CH, dtype=torch.int32, device=dev)
        hdr = torch.empty(alloc * _lib.TILED_HDR_WORDS, dtype=torch.int32, device=dev)
        cls = torch.empty(alloc * CH, dtype=torch.uint8, device=dev) if fact else None
        val = None if fact else torch.empty(alloc * CH, dtype=torch.float32, device=dev)
        _lib.check(L.gnnrec_tiled_plan_quad_layout(
            ptr(wp), ptr(wq), n_waves, total, int(plan["rows_per_block"]), ptr(plan["slot"]),
            ptr(plan.get("val")), ptr(plan["cls"]) if fact else 0, ptr(plan["hdr"]),
            ptr(slot), ptr(val), ptr(cls), ptr(hdr), stream), "gnnrec_tiled_plan_quad_layout")
        plan.update(slot=slot, hdr=hdr, wave_ptr=wq, n_chunks=total, n_slots=total * CH,
                    layout="quad")
        if fact:
            plan["cls"] = cls
        else:
            plan["val"] = val

    def _tiled_plan_host(self, R: int, panel: int, sub_panel: int) -> dict:
        import ctypes as C
        L = _lib.lib()
        rp = np.ascontiguousarray(_np(self.row_ptr), dtype=np.int64)
        col = np.ascontiguousarray(_np(self.col), dtype=np.int32)
        val = np.ascontiguousarray(_np(self.val), dtype=np.float32)
        h, n_chunks, n_blocks = C.c_void_p(), C.c_int64(), C.c_int64()
        _lib.check(L.gnnrec_tiled_plan_build(rp.ctypes.data, col.ctypes.data, val.ctypes.data,
                                             self.n_rows, R, panel, sub_panel, 0, C.byref(h),
                                             C.byref(n_chunks), C.byref(n_blocks)),
                   "gnnrec_tiled_plan_build")
        nb = n_blocks.value
        chunks = n_chunks.value + _lib.TILED_TAIL          # + tail chunks (prefetch)
        slot = np.empty(chunks * _lib.TILED_CHUNK, np.uint32)
        v = np.empty(chunks * _lib.TILED_CHUNK, np.float32)
        hdr = np.empty(chunks * _lib.TILED_HDR_WORDS, np.uint32)
        wave_ptr = np.empty(nb * _lib.TILED_WAVES + 1, np.int64)
        n_steps = np.empty(max(nb, 1), np.int32)
        try:
            _lib.check(L.gnnrec_tiled_plan_emit(h, slot.ctypes.data, v.ctypes.data,
                                                hdr.ctypes.data, wave_ptr.ctypes.data,
                                                n_steps.ctypes.data),
                       "gnnrec_tiled_plan_emit")
        finally:
            L.gnnrec_tiled_plan_free(h)
        dev = self.device
        return dict(slot=torch.from_numpy(slot.view(np.int32)).to(dev),
                    val=torch.from_numpy(v).to(dev),
                    hdr=torch.from_numpy(hdr.view(np.int32)).to(dev),
                    wave_ptr=torch.from_numpy(wave_ptr).to(dev),
                    n_steps=torch.from_numpy(n_steps).to(dev),
                    n_blocks=nb, n_chunks=n_chunks.value)

    def _tiled_plan_device(self, R: int, panel: int, sub_panel: int) -> dict:
        """gnnrec_tiled_plan_device: a counting pass, the chunk offsets by a device cumsum,
        the emitting pass (device reads: the chunk total and the error word). The scratch is
        sized for steps of up to `cap` slots — a step is one panel of one block, far smaller
        than the block — so every block can have its own workgroup; a step beyond it fails
        the pass (error 2) and the pass is re-run with the block bound."""
        dev = self.device
        if dev.type != "cuda":
            raise ValueError("the device planner needs the graph on a ROCm device")
        import time
        t0 = time.perf_counter()
        n, W = self.n_rows, _lib.TILED_WAVES
        nb = -(-n // R)
        max_nnz = self.row_stats(R)[1] if nb else 0
        if max_nnz >= (1 << 31) - 1:
            raise ValueError("tiled plan: a block holds more than 2^31 edges")
        cap = min(max_nnz, TILED_PLAN_STEP_CAP)
        prologue = time.perf_counter() - t0
        try:
            plan = self._tiled_plan_device_pass(R, panel, sub_panel, nb, cap)
        except _ScratchTooSmall:
            plan = self._tiled_plan_device_pass(R, panel, sub_panel, nb, max_nnz)
        plan["planner_phases"]["block_sizes_s"] = prologue
        return plan

    def _tiled_plan_device_pass(self, R, panel, sub_panel, nb, cap) -> dict:
        dev = self.device
        L = _lib.lib()
        n, W = self.n_rows, _lib.TILED_WAVES
        import time
        t_alloc = time.perf_counter()
        per_wg = 8 * L.gnnrec_tiled_plan_device_scratch_words(cap, 1)
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        # one 64-lane workgroup per block (23 KB of LDS: 7 per CU), scratch at most ~4 GB
        wg = max(1, min(nb, 7 * cus, (4 << 30) // max(per_wg, 1)))
        scratch = torch.empty(max(1, L.gnnrec_tiled_plan_device_scratch_words(cap, wg)),
                              dtype=torch.int64, device=dev)
        chunks = torch.zeros(max(1, nb * W), dtype=torch.int64, device=dev)
        n_steps = torch.zeros(max(nb, 1), dtype=torch.int32, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        stream = _lib.stream_of(dev)
        ptr = _lib.ptr
        args = (ptr(self.row_ptr), ptr(self.col), ptr(self.val), n, R, panel, sub_panel, cap,
                ptr(scratch), wg)

        def failed(what, code):
            if code == 2:
                raise _ScratchTooSmall()
            raise _DEVICE_PLAN_ERRORS.get(code, RuntimeError)(
                f"gnnrec_tiled_plan_device ({what}) failed: error {code}")

        torch.cuda.synchronize(dev)
        t_count = time.perf_counter()
        _lib.check(L.gnnrec_tiled_plan_device(*args, ptr(chunks), ptr(n_steps), None, None, None,
                                              None, ptr(err), stream),
                   "gnnrec_tiled_plan_device (count)")
        wave_ptr = torch.zeros(nb * W + 1, dtype=torch.int64, device=dev)
        torch.cumsum(chunks[:nb * W], 0, out=wave_ptr[1:])
        n_chunks, code = int(wave_ptr[-1]), int(err)
        if code:
            failed("count", code)
        t_emit_alloc = time.perf_counter()
        total = n_chunks + _lib.TILED_TAIL
        slot = torch.empty(total * _lib.TILED_CHUNK, dtype=torch.int32, device=dev)
        v = torch.empty(total * _lib.TILED_CHUNK, dtype=torch.float32, device=dev)
        hdr = torch.empty(total * _lib.TILED_HDR_WORDS, dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)
        t_emit = time.perf_counter()
        _lib.check(L.gnnrec_tiled_plan_device(*args, None, None, ptr(wave_ptr), ptr(slot), ptr(v),
                                              ptr(hdr), ptr(err), stream),
                   "gnnrec_tiled_plan_device (emit)")
        code = int(err)
        if code:
            failed("emit", code)
        t_end = time.perf_counter()
        del scratch
        # sub-phases of the planner (bench.py's operand_prep_s): the scratch / count arrays'
        # allocation, the count pass (+ cumsum, chunk total read back), the plan arrays'
        # allocation, the emit pass (and, from _tiled_plan_device, the block sizes before them)
        phases = dict(scratch_alloc_s=t_count - t_alloc, count_s=t_emit_alloc - t_count,
                      arrays_alloc_s=t_emit - t_emit_alloc, emit_s=t_end - t_emit)
        return dict(slot=slot, val=v, hdr=hdr, wave_ptr=wave_ptr, n_steps=n_steps,
                    n_blocks=nb, n_chunks=n_chunks, planner_phases=phases)

    def heavy_plan(self, threshold: int, seg_len: int):
        """Degree buckets for the skew-tolerant kernels (cached): rows with more than
        `threshold` neighbours, each cut into ceil(degree / seg_len) segments of EQUAL length
        (degree-aware: a row of degree D gets segments of D / ceil(D / seg_len) edges, one
        edge apart at most, instead of full segments and a short last one that would leave
        its wave's other lanes waiting). Returns None when there are none, else
        dict(heavy_rows, heavy_seg_ptr, seg_row, seg_beg, seg_end) on this device."""
        key = ("heavy", threshold, seg_len)
        if key not in self._plans:
            rp = self.row_ptr
            deg = rp[1:] - rp[:-1]
            heavy = torch.nonzero(deg > threshold).flatten()
            if heavy.numel() == 0:
                self._plans[key] = None
            else:
                dh = deg[heavy]
                nseg = (dh + seg_len - 1) // seg_len
                seg_ptr = torch.zeros(heavy.numel() + 1, dtype=torch.int64, device=rp.device)
                seg_ptr[1:] = torch.cumsum(nseg, 0)
                seg_row = torch.repeat_interleave(heavy, nseg)
                j = torch.arange(int(seg_ptr[-1]), device=rp.device) - torch.repeat_interleave(
                    seg_ptr[:-1], nseg)
                D = torch.repeat_interleave(dh, nseg)
                n = torch.repeat_interleave(nseg, nseg)
                start = rp[seg_row]
                seg_beg = start + (j * D) // n
                seg_end = start + ((j + 1) * D) // n
                self._plans[key] = dict(heavy_rows=heavy.contiguous(), heavy_seg_ptr=seg_ptr,
                                        seg_row=seg_row.contiguous(), seg_beg=seg_beg.contiguous(),
                                        seg_end=seg_end.contiguous())
        return self._plans[key]

    def heavy_plan_by_column(self, threshold: int, seg_len: int):
        """heavy_plan with the segment arrays sorted by each segment's first column (stable;
        cached), plus seg_pos: the sorted position of each segment of the row-grouped
        numbering heavy_seg_ptr refers to (gnnrec_gat_heavy_att_f32). Segments of different
        heavy rows over the same columns then run together and share gathered lines in L2."""
        key = ("heavy_col", threshold, seg_len)
        if key not in self._plans:
            base = self.heavy_plan(threshold, seg_len)
            if base is None:
                self._plans[key] = None
            else:
                first = self.col[base["seg_beg"]].to(torch.int64)
                order = torch.sort(first, stable=True).indices
                pos = torch.empty_like(order)
                pos[order] = torch.arange(order.numel(), device=order.device)
                self._plans[key] = dict(
                    heavy_rows=base["heavy_rows"], heavy_seg_ptr=base["heavy_seg_ptr"],
                    seg_row=base["seg_row"][order].contiguous(),
                    seg_beg=base["seg_beg"][order].contiguous(),
                    seg_end=base["seg_end"][order].contiguous(), seg_pos=pos.contiguous())
        return self._plans[key]

    def heavy_plan_panels(self, threshold: int, seg_len: int, panel: int, min_per_panel: int):
        """heavy_plan_by_column with the heaviest rows cut at column-panel boundaries: a heavy
        row with at least `min_per_panel` edges per `panel`-column panel on average gets one
        segment per (panel, seg_len edges) run instead of equal-length segments, so the
        segments of every such row over one panel start in that panel and — sorted by first
        column — run together while that panel's gathered lines sit in L2 (cached). The other
        heavy rows keep heavy_plan's equal-length cut. Same output layout as
        heavy_plan_by_column."""
        key = ("heavy_pan", threshold, seg_len, panel, min_per_panel)
        if key not in self._plans:
            base = self.heavy_plan(threshold, seg_len)
            if base is None:
                self._plans[key] = None
                return None
            rp, col = self.row_ptr, self.col
            dev = rp.device
            heavy = base["heavy_rows"]
            deg = rp[heavy + 1] - rp[heavy]
            n_panels = max(1, -(-self.shape[1] // panel))
            cut = deg >= min_per_panel * n_panels
            # equal-length segments of the other heavy rows (heavy_plan's, row by row)
            keep_seg = ~cut[torch.repeat_interleave(torch.arange(heavy.numel(), device=dev),
                                                    base["heavy_seg_ptr"][1:] -
                                                    base["heavy_seg_ptr"][:-1])]
            segs = [(base["seg_row"][keep_seg], base["seg_beg"][keep_seg],
                     base["seg_end"][keep_seg])]
            rows = heavy[cut]
            if rows.numel():
                beg, end = rp[rows], rp[rows + 1]
                lens = end - beg
                total = int(lens.sum())
                start = torch.zeros(rows.numel() + 1, dtype=torch.int64, device=dev)
                start[1:] = torch.cumsum(lens, 0)
                e = torch.repeat_interleave(beg - start[:-1], lens, output_size=total) + \
                    torch.arange(total, device=dev)                   # edge ids, row by row
                rid = torch.repeat_interleave(rows, lens, output_size=total)
                pan = col[e].to(torch.int64) // panel
                first = torch.ones(total, dtype=torch.bool, device=dev)
                first[1:] = (rid[1:] != rid[:-1]) | (pan[1:] != pan[:-1])
                run = torch.cumsum(first.to(torch.int64), 0) - 1
                run_start = torch.nonzero(first).flatten()
                brk = first | ((torch.arange(total, device=dev) - run_start[run]) % seg_len == 0)
                bpos = torch.nonzero(brk).flatten()
                nxt = torch.empty_like(bpos)
                nxt[:-1] = bpos[1:]
                nxt[-1] = total
                segs.append((rid[bpos], e[bpos], e[nxt - 1] + 1))
                del e, rid, pan, first, run, run_start, brk
            seg_row = torch.cat([t[0] for t in segs])
            seg_beg = torch.cat([t[1] for t in segs])
            seg_end = torch.cat([t[2] for t in segs])
            # row-grouped numbering for the merge (heavy rows ascending, segments by position)
            grp = torch.sort(seg_beg, stable=True).indices          # CSR order = row order
            seg_row, seg_beg, seg_end = seg_row[grp], seg_beg[grp], seg_end[grp]
            counts = torch.zeros(heavy.numel(), dtype=torch.int64, device=dev)
            counts.index_add_(0, torch.searchsorted(heavy, seg_row),
                              torch.ones_like(seg_row))
            seg_ptr = torch.zeros(heavy.numel() + 1, dtype=torch.int64, device=dev)
            seg_ptr[1:] = torch.cumsum(counts, 0)
            order = torch.sort(col[seg_beg].to(torch.int64), stable=True).indices
            pos = torch.empty_like(order)
            pos[order] = torch.arange(order.numel(), device=dev)
            self._plans[key] = dict(
                heavy_rows=heavy, heavy_seg_ptr=seg_ptr, seg_row=seg_row[order].contiguous(),
                seg_beg=seg_beg[order].contiguous(), seg_end=seg_end[order].contiguous(),
                seg_pos=pos.contiguous(), n_cut_rows=int(cut.sum()))
        return self._plans[key]

    def __repr__(self) -> str:  # keep it short: the tensors are huge
        return (f"CsrGraph(shape={self.shape}, nnz={self.nnz}, device={self.device}, "
                f"symmetric={self.symmetric}, shard={self.shard_info})")
