"""Torch-facing ops over libgnnrec (device tensors only; no fallback path).

Every function here takes a :class:`CsrGraph` on a ROCm device and fp32 row-major tables on
the same device, launches on torch's current stream, and raises if the native library is
unavailable. Autograd: the SpMM and the fused LightGCN propagation are differentiable
(backward = the same kernel over A^T, which is A itself for the symmetric normalisation,
SURVEY §2.1); the fused NGCF / GAS / OrthogonalBundle kernels are inference kernels and the
models use them only when no gradient is required.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch

from . import _lib
from ._lib import EPI_ACC_ADD, EPI_ACC_DIV, EPI_ACC_INIT, EPI_ACC_X, EPI_NO_Y, check, ptr
from .graph import CsrGraph


def _require_device(adj: CsrGraph, *tensors: torch.Tensor) -> None:
    if adj.device.type != "cuda":
        raise ValueError(f"libgnnrec ops need the operand on a ROCm device, got {adj.device}")
    for t in tensors:
        if t is None:
            continue
        if t.device != adj.device:
            raise ValueError(f"tensor on {t.device}, operand on {adj.device}")
        if t.dtype != torch.float32:
            raise TypeError(f"expected float32, got {t.dtype}")
        if t.dim() != 2 or t.stride(1) != 1:
            raise ValueError("expected a 2-D row-major table (stride(1) == 1)")


def _rowmajor(t: torch.Tensor) -> torch.Tensor:
    return t if (t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 4 == 0) else t.contiguous()


def _csr_args(adj: CsrGraph):
    return ptr(adj.row_ptr), ptr(adj.col), ptr(adj.val), adj.n_rows


# Rows longer than this go to the workgroup-per-row kernel (bit-exact, LDS-pipelined gather);
# 0 disables the split. Sweep (tools/exp_heavy.py, profiles/r01/heavy_split_sweep.jsonl):
# ML-1M-shaped LightGCN K=3 0.90 ms unsplit -> 0.30 ms at 128, power-law 2M x 2M 123 -> 29 ms;
# uniform graphs (G100M, max degree ~150) have no rows above it.
# Heavy-row knobs of the CSR hop (gnnrec_spmm_csr_heavy_f32), None = by operand (heavy_knobs):
# rows longer than SPMM_HEAVY_THRESHOLD run one workgroup per row, and of those the rows longer
# than SPMM_SLICE_LEN as feature slices (workgroups of d/4 or 32 features, chosen in the kernel
# by operand size; 0 = none). Round-6 sweeps, every output bit-identical
# (profiles/r06/config2_knobs_sweep_*.jsonl, powerlaw_knobs_sweep.jsonl):
#   small operands (<= 65 536 rows, e.g. ML-1M): threshold 128, slices above 1024 — config 2
#     0.246 -> 0.191 ms per forward (threshold 256 unsliced: 0.215); with the light rows fused
#     into the heavy launch (unmasked hops, d = 32 / 64 / 128): threshold 256, slices above
#     2048 — K = 3 propagation 0.17 -> 0.114 ms (profiles/r06/csr_fused_*.jsonl);
#   large: threshold 256 (d <= 64) / 512 (d >= 128), slices above 4096 — power-law 2M x 2M
#     K=3 d=64 18.98 -> 15.6 ms (slices above 1024, throughput-form light rows), 12.9 ms with
#     the latency-form light rows (light_form_flag) and slices above 4096 (13.2 at 1024,
#     profiles/r06/powerlaw_knobs_sweep_latency.jsonl); d=128 36.4 -> 24.0 ms; G100M's CSR path
#     (no row above ~200) 21.1 ms at 256 against 21.4 at 128.
SPMM_HEAVY_THRESHOLD = None
SPMM_SLICE_LEN = None
SMALL_OPERAND_ROWS = 65536          # gnnrec_spmm_csr_heavy_f32's own small-operand bound
# CSR_FLAGS: _lib.CSR_FORK (the heavy rows on a side stream beside the row-parallel kernel:
# measured slower, the cross-stream join costs ~17 us per hop, profiles/r06/config2_trace/)
# and the row-parallel chain's form (CSR_LIGHT_*; 0 = by operand size).
CSR_FLAGS = 0
# The row-parallel chain's form on large operands (the library picks the latency form by
# itself up to SMALL_OPERAND_ROWS rows): the latency form (16 lanes x float4 per row, d = 64)
# when the light rows average at most LIGHT_LATENCY_MAX_AVG neighbours, else the throughput
# form (a wave per row). tools/exp_light_form.py, profiles/r06/light_form.jsonl (K = 3, d = 64,
# ms throughput / latency): uniform 2M rows of avg degree 10: 3.50 / 2.64; 25: 5.75 / 6.05;
# 50: 10.8 / 11.8; 100: 21.2 / 22.9; power-law 2M x 2M (light rows avg 19): 15.0 / 13.2.
LIGHT_LATENCY_MAX_AVG = 22.0


def light_form_flag(adj: CsrGraph, heavy_threshold: int) -> int:
    """CSR_FLAGS plus _lib.CSR_LIGHT_LATENCY for a large operand whose light rows are short
    (LIGHT_LATENCY_MAX_AVG), unless CSR_FLAGS already names a form."""
    fl = int(CSR_FLAGS)
    if fl & (_lib.CSR_LIGHT_LATENCY | _lib.CSR_LIGHT_THROUGHPUT) or adj.n_rows <= SMALL_OPERAND_ROWS:
        return fl
    if adj.light_avg_degree(max(int(heavy_threshold), 0)) <= LIGHT_LATENCY_MAX_AVG:
        fl |= _lib.CSR_LIGHT_LATENCY
    return fl


def heavy_knobs(n_rows: int, d: int, masked: bool = False) -> Tuple[int, int]:
    """(heavy threshold, slice length) for a CSR hop over n_rows destination rows at width d
    (the module's SPMM_* settings when not None). masked: the hop has x_mask / y_active (the
    library then keeps its light rows a launch of their own, even on small operands)."""
    small = n_rows <= SMALL_OPERAND_ROWS
    fused = small and not masked and d in (32, 64, 128) and not (CSR_FLAGS & (
        _lib.CSR_FORK | _lib.CSR_TWO_LAUNCHES | _lib.CSR_LIGHT_THROUGHPUT))
    ht = SPMM_HEAVY_THRESHOLD if SPMM_HEAVY_THRESHOLD is not None else (
        256 if fused else 128 if small else (256 if d <= 64 else 512))
    sl = SPMM_SLICE_LEN if SPMM_SLICE_LEN is not None else (
        2048 if fused else 1024 if small else 4096)
    return ht, sl


# Column-ordered hop (gnnrec_spmm_tiled_f32): the same bits, used for any d
# that is a multiple of 32 when the operand has at least TILED_MIN_ROWS rows, the gathered
# table is larger than the chip's L2s together (TILED_MIN_TABLE_BYTES; below that the
# row-parallel gathers hit L2 anyway) and no row is longer than TILED_MAX_DEGREE (a long row's
# panel run stays on one slot stream and would hold its step). Crossover on G100M row slices
# (profiles/r02/exp_chunks.jsonl, d = 64): 31K rows CSR 0.124 vs tiled 0.140 ms, 62.5K rows
# 0.232 vs 0.208, 250K 0.88 vs 0.62. Masked / row-subset hops keep the CSR kernel. Rows per
# block are evened out so every pass of the persistent grid is full (G100M: 14 passes of 1117
# rows — 7 per 32-feature slice at d = 64 — not 6 of 1279 plus a tail pass).
TILED_HOP = True
TILED_MIN_ROWS = 49152
TILED_MIN_TABLE_BYTES = 32 << 20
TILED_MAX_DEGREE = 4096
TILED_MAX_ROWS = _lib.TILED_MAX_ROWS
TILED_MAX_LDX = _lib.TILED_MAX_LDX
TILED_BALANCE_PASSES = True
# bound of the pass-start meeting of an XCD group's workgroups (µs; 0 = no meeting: use when
# other kernels share the device, e.g. a concurrent exchange)
TILED_MEET_US = 200


def _tiled_rows_per_block(n_rows: int, device, reserve_cus: int = 0) -> int:
    """Rows per block so every pass of the persistent grid is full. reserve_cus > 0: size a
    single-pass operand for cus - reserve_cus blocks, so the launch grid (one workgroup per
    block, at most one per CU) leaves that many CUs free for kernels that run beside it
    (the exchange of overlapped multi-GPU chunks)."""
    if not TILED_BALANCE_PASSES:
        return TILED_MAX_ROWS
    cus = torch.cuda.get_device_properties(device).multi_processor_count
    if 0 < reserve_cus < cus:
        eff = cus - int(reserve_cus)
        if n_rows <= eff * TILED_MAX_ROWS:
            return max(1, -(-n_rows // eff))
    passes = max(1, -(-n_rows // (cus * TILED_MAX_ROWS)))
    return min(TILED_MAX_ROWS, -(-n_rows // (passes * cus)))


def _tiled_views_ok(*tables) -> bool:
    """The column-ordered kernel moves 16 B per lane: 16-B aligned rows (ld % 4 == 0)."""
    return all(t is None or (t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0) for t in tables)


_TILED_OK: dict = {}


def _tiled_supported(device, rows_per_block: int) -> bool:
    """Whether `device` grants the column-ordered kernel its LDS (gnnrec_spmm_tiled_supported,
    cached per device and block size)."""
    key = (torch.device(device).index or 0, int(rows_per_block))
    if key not in _TILED_OK:
        _TILED_OK[key] = bool(_lib.lib().gnnrec_spmm_tiled_supported(*key))
    return _TILED_OK[key]


# Gathering from a table whose rows are a multiple of 1 KB apart, the hop runs ~40 % slower
# on a 32-feature slice whose 128-B lines start at byte 384 of a 1-KB window than at any
# other line offset (G100M d = 32: 2.33 ms against 1.66-1.76 ms; d = 64 blocks covering that
# line 3.99-4.06 ms against 3.31-3.36 ms; tools/exp_hop_offset2.py,
# profiles/r04/exp_hop_line_offset.jsonl). Config 3's [N, 4d] concat table put layer 2's
# input block exactly there. Tables this package allocates for its own gathered blocks are
# placed so that none of their lines does.
SLOW_GATHER_LINE = 384


def gather_table_shift(addr: int, width: int, gathered_cols: int, esz: int = 4):
    """Elements to skip from a buffer at byte address `addr` so that rows of `width` elements
    whose columns [0, gathered_cols) are gathered keep every 128-B line of those columns off
    SLOW_GATHER_LINE of a 1-KB window; None when there is nothing to choose (rows not a
    multiple of 1 KB apart, `addr` not 128-B aligned, or the columns cover every offset)."""
    if (width * esz) % 1024 or addr % 128:
        return None
    lines = range(0, -(-gathered_cols * esz // 128) * 128, 128)
    good = [s for s in range(0, 1024, 128)
            if all((s + o) % 1024 != SLOW_GATHER_LINE for o in lines)]
    if not good:
        return None
    return min((s - addr) % 1024 for s in good) // esz


def gather_table(n_rows: int, width: int, gathered_cols: int, *, dtype=torch.float32,
                 device=None) -> torch.Tensor:
    """torch.empty((n_rows, width)) — a contiguous row-major tensor, possibly at a storage
    offset — whose columns [0, gathered_cols) are hop inputs, placed by gather_table_shift."""
    esz = torch.empty((), dtype=dtype).element_size()
    if (width * esz) % 1024 or n_rows == 0:
        return torch.empty((n_rows, width), dtype=dtype, device=device)
    buf = torch.empty(n_rows * width + 1024 // esz, dtype=dtype, device=device)
    start = gather_table_shift(buf.data_ptr(), width, gathered_cols, esz) or 0
    return buf[start:start + n_rows * width].view(n_rows, width)


# Row stride of the tables the propagation gathers from, by width (floats -> (ld, start byte
# of the 1-KB window)): compact rows put one line in eight at SLOW_GATHER_LINE; 256-B / 512-B
# rows starting 1-KB aligned (d = 32 / 64), or 1-KB rows starting at byte 512 (d = 128), keep
# every line off it. G100M LightGCN K = 3 on the bench path, same bits
# (profiles/r04/exp_hop_tables.jsonl): d = 64 10.29 -> 9.88 ms, d = 32 5.08 -> 4.95 ms,
# d = 128 20.70-20.81 -> 20.52 ms.
HOP_TABLE_LAYOUT = {32: (64, 0), 64: (128, 0), 128: (256, 512)}


def hop_table(n_rows: int, d: int, *, device=None, zero: bool = False,
              layout: Optional[Tuple[int, int]] = None) -> torch.Tensor:
    """A [n_rows, d] fp32 table for hops to gather from: a row-major view (row stride ld >= d,
    16-B aligned rows) of a wider buffer placed per HOP_TABLE_LAYOUT (or `layout` = (ld,
    start byte mod 1 KB)); a compact tensor for other widths. zero: the d columns are zeroed
    (the padding columns are never read)."""
    ld, start = layout if layout is not None else HOP_TABLE_LAYOUT.get(d, (d, None))
    if layout is None and start is not None and not _placed_tables_fit(n_rows, d, ld, device):
        start = None
    if start is None or n_rows == 0:
        mk = torch.zeros if zero else torch.empty
        return mk((n_rows, d), dtype=torch.float32, device=device)
    if ld < d or ld % 4 or start % 128:
        raise ValueError(f"hop_table layout ({ld}, {start}) for d = {d}")
    buf = torch.empty(n_rows * ld + 256, dtype=torch.float32, device=device)
    s = ((start - buf.data_ptr()) % 1024) // 4
    t = buf[s:s + n_rows * ld].view(n_rows, ld)[:, :d]
    if zero:
        t.zero_()
    return t


# The placed tables cost ld / d times the compact bytes (2x at d = 32 / 64 / 128). They are
# used only while that extra space is a small part of the device's free memory, and never with
# GNNREC_HOP_TABLE_LAYOUT=0 (compact tables everywhere; same bits, the hop is ~4 % slower).
HOP_TABLE_MAX_EXTRA_FRACTION = 0.25


_PLACED_FIT: dict = {}


def _placed_tables_fit(n_rows: int, d: int, ld: int, device) -> bool:
    """Decided once per (device, n_rows, d, ld) and cached, so a layer's tables keep one
    layout from call to call and the hot path makes no device-memory query."""
    if os.environ.get("GNNREC_HOP_TABLE_LAYOUT", "1") == "0":
        return False
    dev = torch.device(device) if device is not None else None
    if dev is None or dev.type != "cuda" or n_rows == 0:
        return True
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), n_rows, d, ld)
    if key not in _PLACED_FIT:
        extra = n_rows * (ld - d) * 4
        free, _ = torch.cuda.mem_get_info(dev)
        cached = torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
        _PLACED_FIT[key] = extra <= HOP_TABLE_MAX_EXTRA_FRACTION * (free + max(0, cached))
    return _PLACED_FIT[key]


def tiled_plan_for(adj: CsrGraph, x: torch.Tensor, x_mask=None, y_active=None,
                   reserve_cus: int = 0, outputs=()):
    """The column-ordered plan spmm_into would use for (adj, x) (and the `outputs` tables
    it writes or reads row-wise), or None (CSR kernel). A device that cannot grant the
    kernel's LDS (rows per block + 1 accumulator rows of 128 B) keeps the CSR kernel."""
    if (not TILED_HOP or x_mask is not None or y_active is not None or x.shape[1] % 32
            or adj.n_rows < max(TILED_MIN_ROWS, 1) or adj.nnz == 0
            or x.stride(0) > TILED_MAX_LDX or not _tiled_views_ok(x, *outputs)
            or x.shape[0] * x.shape[1] * 4 < TILED_MIN_TABLE_BYTES
            or adj.max_degree() > TILED_MAX_DEGREE):
        return None
    R = _tiled_rows_per_block(adj.n_rows, x.device, reserve_cus)
    if not _tiled_supported(x.device, R):
        return None
    return adj.tiled_plan(rows_per_block=R)


def _heavy_args(adj: CsrGraph, x: torch.Tensor, heavy_threshold: int,
                slice_len: Optional[int] = None, masked: bool = False):
    """(heavy_rows ptr, n_heavy, threshold, n_sliced) for the split launch, or the no-split
    tuple. n_sliced: how many of the (longest-first) heavy rows are longer than slice_len
    (None: heavy_knobs; 0: none)."""
    d = x.shape[1]
    if (heavy_threshold <= 0 or d % 4 or d < 16 or d > 256 or x.stride(0) % 4
            or x.data_ptr() % 16):
        return None, 0, 0, 0
    rows = adj.heavy_rows(heavy_threshold)
    if rows is None:
        return None, 0, 0, 0
    sl = heavy_knobs(adj.n_rows, d, masked)[1] if slice_len is None else slice_len
    n_sliced = adj.heavy_rows_longer(heavy_threshold, sl) if sl > 0 else 0
    return ptr(rows), rows.numel(), int(heavy_threshold), n_sliced


# ---- raw launches (no autograd) ---------------------------------------------------------
def spmm_into(adj: CsrGraph, x: torch.Tensor, y: Optional[torch.Tensor], *, epi: int = 0,
              self_rows: Optional[torch.Tensor] = None, acc: Optional[torch.Tensor] = None,
              acc_div: float = 1.0, heavy_threshold: Optional[int] = None,
              x_mask: Optional[torch.Tensor] = None,
              y_active: Optional[torch.Tensor] = None, meet_us: Optional[int] = None,
              reserve_cus: int = 0, prev: Optional[torch.Tensor] = None) -> None:
    """y = A x with an optional fused layer-mean epilogue (gnnrec_spmm_csr_heavy_f32: rows
    longer than `heavy_threshold` run on the workgroup-per-row kernel; rows of x whose
    `x_mask` byte is 0 are all-zero and are not gathered — same bits; destination rows whose
    `y_active` byte is 0 are not computed — y is +0 there, or the true value). `meet_us`: the
    column-ordered kernel's pass-start meeting bound (None: TILED_MEET_US); `reserve_cus`: its
    single-pass grid leaves that many CUs free (_tiled_rows_per_block); `prev`: the ACC_X
    rows (column-ordered kernel only; default x's own rows)."""
    _require_device(adj, x, y, self_rows, acc, prev)
    if x_mask is not None and (x_mask.dtype != torch.uint8 or x_mask.device != x.device
                               or x_mask.numel() < adj.shape[1]):
        raise ValueError("x_mask must be a uint8 tensor on x's device with a byte per row")
    d = x.shape[1]
    if x.shape[0] < adj.shape[1]:
        raise ValueError(f"x has {x.shape[0]} rows, operand has {adj.shape[1]} columns")
    L = _lib.lib()
    masked = x_mask is not None or y_active is not None
    ht = heavy_knobs(adj.n_rows, d, masked)[0] if heavy_threshold is None else heavy_threshold
    if y_active is not None and (y_active.dtype != torch.uint8 or y_active.device != x.device
                                 or y_active.numel() < adj.n_rows):
        raise ValueError("y_active must be a uint8 tensor on x's device with a byte per "
                         "destination row")
    plan = tiled_plan_for(adj, x, x_mask, y_active, reserve_cus,
                          outputs=(y, self_rows if epi & EPI_ACC_INIT else None,
                                   acc if epi & (EPI_ACC_INIT | EPI_ACC_ADD) else None,
                                   prev if epi & EPI_ACC_X else None))
    if plan is not None:
        spmm_tiled_into(adj, x, y, plan, epi=epi, self_rows=self_rows, acc=acc, acc_div=acc_div,
                        meet_us=meet_us, prev=prev)
        return
    check(L.gnnrec_spmm_csr_heavy_f32(*_csr_args(adj), ptr(x), x.stride(0), ptr(x_mask),
                                      ptr(y_active), ptr(y), y.stride(0) if y is not None else d, d,
                                      epi, ptr(self_rows),
                                      self_rows.stride(0) if self_rows is not None else d,
                                      ptr(acc), acc.stride(0) if acc is not None else d,
                                      float(acc_div), *_heavy_args(adj, x, ht, masked=masked),
                                      light_form_flag(adj, ht), _lib.stream_of(adj.device)),
          "gnnrec_spmm_csr_heavy_f32")


def spmm_tiled_into(adj: CsrGraph, x: torch.Tensor, y: Optional[torch.Tensor], plan: dict, *,
                    epi: int = 0, self_rows: Optional[torch.Tensor] = None,
                    acc: Optional[torch.Tensor] = None, acc_div: float = 1.0,
                    meet_us: Optional[int] = None, prev: Optional[torch.Tensor] = None) -> None:
    """spmm_into through the column-ordered kernel with an explicit plan (adj.tiled_plan());
    same results, bit for bit. The plan's sync words make
    concurrent launches of one plan on different streams unsafe. `prev`: the ACC_X rows
    ([n_rows, >= d]; None: x's own rows)."""
    _require_device(adj, x, y, self_rows, acc, prev)
    d = x.shape[1]
    if bool(_lib.lib().gnnrec_tiled_plan_quad()) != (plan.get("layout") == "quad"):
        raise ValueError("spmm_tiled_into: the plan's layout does not match the kernel's "
                         "(gnnrec_tiled_plan_quad); build it with CsrGraph.tiled_plan()")
    check(_lib.lib().gnnrec_spmm_tiled_f32(
        ptr(plan["slot"]), ptr(plan.get("val")), ptr(plan.get("cls")),
        ptr(plan.get("row_factor")), ptr(plan.get("class_table")), int(plan.get("n_classes", 0)),
        ptr(plan["hdr"]), ptr(plan["wave_ptr"]), ptr(plan["n_steps"]), plan["n_blocks"],
        plan["rows_per_block"],
        ptr(x), x.shape[0], x.stride(0), ptr(y), y.stride(0) if y is not None else d, adj.n_rows,
        d, epi, ptr(self_rows), self_rows.stride(0) if self_rows is not None else d, ptr(acc),
        acc.stride(0) if acc is not None else d, float(acc_div), ptr(prev),
        prev.stride(0) if prev is not None else d, ptr(plan["sync"]),
        int(TILED_MEET_US if meet_us is None else meet_us),
        _lib.stream_of(adj.device)), "gnnrec_spmm_tiled_f32")


def row_nonzero(x: torch.Tensor) -> torch.Tensor:
    """uint8 [rows]: 1 where the row of x holds any non-zero (NaN included)."""
    x = _rowmajor(x)
    m = torch.empty(x.shape[0], dtype=torch.uint8, device=x.device)
    check(_lib.lib().gnnrec_row_nonzero_f32(ptr(x), x.stride(0), x.shape[0], x.shape[1], ptr(m),
                                            _lib.stream_of(x.device)), "gnnrec_row_nonzero_f32")
    return m


# Row-sparse input hop (gnnrec_spmm_sparse_src_f32): used for the training backward's first
# hop when its sources' stored entries are at most this fraction of the operand's
SPARSE_SRC_MAX_FRAC = 0.05


class SparseSrc:
    """A hop input that is zero outside `rows` (int64, ascending) whose rows of the forward
    operand hold `pairs` entries: the hop runs as gnnrec_spmm_sparse_src_f32."""

    def __init__(self, fwd: CsrGraph, rows: torch.Tensor, pairs: int):
        self.fwd, self.rows, self.pairs = fwd, rows, int(pairs)


def sparse_sources(fwd: CsrGraph, x: torch.Tensor, max_frac: float = SPARSE_SRC_MAX_FRAC):
    """SparseSrc for a hop over fwd^T of x when x's non-zero rows (NaN included) hold at most
    `max_frac` of fwd's entries, else None (two small device reads)."""
    rows = torch.nonzero(row_nonzero(x)).flatten()
    if rows.numel() == 0:
        return SparseSrc(fwd, rows, 0)
    rp = fwd.row_ptr
    pairs = int((rp[rows + 1] - rp[rows]).sum())
    return SparseSrc(fwd, rows, pairs) if pairs <= max_frac * max(fwd.nnz, 1) else None


def spmm_sparse_src_into(src: SparseSrc, x: torch.Tensor, y: torch.Tensor) -> None:
    """y = fwd^T x for an x that is zero outside src.rows: every output row a source reaches
    gets the dense hop's bits, the others are zeroed here."""
    fwd = src.fwd
    _require_device(fwd, x, y)
    y.zero_()
    if src.pairs == 0:
        return
    L = _lib.lib()
    nbytes = _lib.C.c_size_t(0)
    args = (ptr(fwd.row_ptr), ptr(fwd.col), ptr(fwd.val), fwd.n_rows, fwd.shape[1],
            ptr(src.rows), src.rows.numel(), src.pairs, ptr(x), x.stride(0), ptr(y), y.stride(0),
            x.shape[1])
    stream = _lib.stream_of(fwd.device)
    check(L.gnnrec_spmm_sparse_src_f32(*args, None, _lib.C.addressof(nbytes), stream),
          "gnnrec_spmm_sparse_src_f32 (size)")
    work = torch.empty(max(int(nbytes.value), 1), dtype=torch.uint8, device=x.device)
    check(L.gnnrec_spmm_sparse_src_f32(*args, ptr(work), _lib.C.addressof(nbytes), stream),
          "gnnrec_spmm_sparse_src_f32")


def mark_rows(row_ptr: torch.Tensor, col: torch.Tensor, marked: torch.Tensor,
              n_out: int) -> torch.Tensor:
    """uint8 [n_out]: 1 at every column listed in a marked row of (row_ptr, col)
    (gnnrec_mark_active_rows)."""
    m = torch.empty(n_out, dtype=torch.uint8, device=marked.device)
    check(_lib.lib().gnnrec_mark_active_rows(ptr(row_ptr), ptr(col), row_ptr.numel() - 1,
                                             ptr(marked), n_out, ptr(m),
                                             _lib.stream_of(marked.device)),
          "gnnrec_mark_active_rows")
    return m


def lightgcn_hop_schedule(K: int, deferred: bool) -> list:
    """The K hop launches of LightGCN propagation with the layer mean in their epilogues:
    per hop (x, y, epi), x / y naming a buffer — "x0", "acc" (the output), "a", "b" (hop
    buffers) or None (no y store).

    Eager (any kernel): hop 1 acc = x0 + y1, then acc += yk, / (K+1) on the last hop — 8 row
    transfers of the epilogue per K=3 forward (x0 read, y1/y2 written, acc written 3x and
    read 2x). Deferred (column-ordered kernel only, EPI_ACC_X and INIT|ADD): hops 1 and 2 store
    their output only — y1 parked in the acc rows — and hop 3 forms ((x0 + y1) + y2) + y3
    reading x0, acc (y1) and its own input rows (y2): 6 transfers at K=3, 4 instead of 5 at K=2
    (x0 + y1 read on hop 2, y1 being hop 2's input). The additions and their order are the
    eager schedule's, so the bits are too. No hop gathers from the rows it writes."""
    if K <= 0:
        return []
    if not deferred or K == 1:
        sched = []
        x = "x0"
        for k in range(1, K + 1):
            last = k == K
            epi = (EPI_ACC_INIT if k == 1 else EPI_ACC_ADD) | ((EPI_ACC_DIV | EPI_NO_Y) if last else 0)
            y = None if last else ("a" if k & 1 else "b")
            sched.append((x, y, epi))
            x = y
        return sched
    if K == 2:
        return [("x0", "a", 0), ("a", None, EPI_ACC_INIT | EPI_ACC_X | EPI_ACC_DIV | EPI_NO_Y)]
    sched = [("x0", "acc", 0), ("acc", "b", 0)]
    x = "b"
    for k in range(3, K + 1):
        last = k == K
        epi = (EPI_ACC_INIT | EPI_ACC_ADD | EPI_ACC_X) if k == 3 else EPI_ACC_ADD
        if last:
            epi |= EPI_ACC_DIV | EPI_NO_Y
        y = None if last else ("a" if x == "b" else "b")
        sched.append((x, y, epi))
        x = y
    return sched


def _lightgcn_hops(op: CsrGraph, x0: torch.Tensor, K: int, masks,
                   deferred: bool = False) -> torch.Tensor:
    """mean(x0, op x0, ..., op^K x0) as K spmm_into launches with the layer mean in their
    epilogues (lightgcn_hop_schedule; eager: the launch and rounding order of
    gnnrec_lightgcn_split_f32). `masks(k, x_in)` gives hop k's (x_mask, y_active), either
    None. deferred: the column-ordered kernel's schedule (the caller checks that spmm_into
    takes that kernel for (op, x0) and that no hop is masked)."""
    out = torch.empty_like(x0)
    if K == 0:
        out.copy_(x0)
        return out
    bufs = {"x0": x0, "acc": out, None: None}
    for k, (xn, yn, epi) in enumerate(lightgcn_hop_schedule(K, deferred), start=1):
        for name in (xn, yn):
            if name not in bufs:   # scratch hop outputs: placed tables (hop_table) when tiled
                bufs[name] = (hop_table(x0.shape[0], x0.shape[1], device=x0.device) if deferred
                              else torch.empty_like(x0))
        xm, ya = masks(k, bufs[xn])
        if isinstance(xm, SparseSrc) and epi == 0:
            spmm_sparse_src_into(xm, bufs[xn], bufs[yn])
            continue
        if isinstance(xm, SparseSrc):
            xm = None
        spmm_into(op, bufs[xn], bufs[yn], epi=epi, self_rows=x0, acc=out,
                  acc_div=float(K + 1), x_mask=xm, y_active=ya)
    return out


def lightgcn_backward(adj: CsrGraph, g: torch.Tensor, n_layers: int,
                      masked_hops: Optional[int] = None, active_hops: int = 1) -> torch.Tensor:
    """d/dx0 of mean_k A^k x0 applied to g: mean_k (A^T)^k g — the same launches and epilogue
    order as lightgcn_forward over A^T (so the same bits). The BPR gradient touches a few
    thousand rows, so the first `masked_hops` hops skip the all-zero rows of their input, and
    the first `active_hops` also skip the output rows no non-zero row reaches. G100M, batch
    2048 (tools/exp_masked.py): hop 1 1.9 ms masked+active vs 7.0 dense (row-parallel); hop 2
    (a quarter of the rows live) 5.9 ms masked, 6.0 + 0.4 (marking) masked+active, but 4.2 ms
    dense through the column-ordered kernel. Default: only hop 1 masked where that kernel
    takes the operand (and then the deferred layer mean), K-1 hops otherwise (a skipped row
    adds fmaf(v, 0, acc) = acc: the same bits as the dense hop, which is the reference's own
    arithmetic)."""
    at = adj.t()
    g = g.contiguous()
    _require_device(at, g)
    K = int(n_layers)
    tiled = tiled_plan_for(at, g) is not None
    if masked_hops is None:
        masked_hops = 1 if tiled else K - 1
    # the deferred layer mean (lightgcn_hop_schedule) when the hop carrying its tiled-only
    # epilogue (hop 2 at K = 2, hop 3 otherwise) is a dense column-ordered hop: a masked hop
    # before it stores its y as the eager one does (+0 on skipped rows), so the same bits
    deferred = tiled and K >= 2 and masked_hops < (2 if K == 2 else 3)

    def masks(k, x_in):
        if k > masked_hops:
            return None, None
        if k == 1 and deferred and SPARSE_SRC_MAX_FRAC > 0:
            # hop 1 of the deferred schedule stores y only: the row-sparse input hop when the
            # gradient's rows are few (same bits)
            src = sparse_sources(adj, x_in)
            if src is not None:
                return src, None
        xm = row_nonzero(x_in)
        # rows of A^T that reach a non-zero row: listed by (A^T)^T = A's rows
        ya = mark_rows(adj.row_ptr, adj.col, xm, at.n_rows) if k <= active_hops else None
        return xm, ya

    return _lightgcn_hops(at, g, K, masks, deferred=deferred)


def lightgcn_forward_rows(adj: CsrGraph, x0: torch.Tensor, n_layers: int, need: torch.Tensor,
                          restricted_hops: int = 2) -> torch.Tensor:
    """lightgcn_forward's output at the rows where `need` (uint8 [N]) is 1, with the same
    bits; the other rows are NOT defined. For a training batch: the BPR loss reads ~6K of 2M
    output rows, so hop K computes only those (R_K = need) and hop k < K only what hop k+1
    reads plus the needed rows (R_k = need | columns of R_{k+1}) — for the last
    `restricted_hops` hops; earlier hops reach nearly every row and run dense."""
    x0 = x0.contiguous()
    _require_device(adj, x0)
    n = x0.shape[0]
    if adj.n_rows != n or adj.shape[1] != n:
        raise ValueError("LightGCN propagation needs a square operand matching x0")
    if need.dtype != torch.uint8 or need.numel() != n or need.device != x0.device:
        raise ValueError("need must be a uint8 tensor with a byte per row on x0's device")
    K = int(n_layers)
    rows = {K: need}
    for k in range(K - 1, max(K - restricted_hops, 0), -1):
        rows[k] = mark_rows(adj.row_ptr, adj.col, rows[k + 1], n).bitwise_or_(need)
    return _lightgcn_hops(adj, x0, K, lambda k, _x: (None, rows.get(k)))


def spmm_forward(adj: CsrGraph, x: torch.Tensor) -> torch.Tensor:
    x = _rowmajor(x)
    y = torch.empty((adj.n_rows, x.shape[1]), dtype=torch.float32, device=x.device)
    spmm_into(adj, x, y)
    return y


def lightgcn_forward(adj: CsrGraph, x0: torch.Tensor, n_layers: int,
                     return_layers: bool = False, heavy_threshold: Optional[int] = None
                     ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """out = mean(x0, A x0, ..., A^K x0); optionally the K hop outputs [K, N, d]."""
    x0 = x0.contiguous()
    _require_device(adj, x0)
    n, d = x0.shape
    if adj.n_rows != n or adj.shape[1] != n:
        raise ValueError("LightGCN propagation needs a square operand matching x0")
    if not return_layers and tiled_plan_for(adj, x0) is not None:
        # per-hop launches of the column-ordered kernel, same epilogue order and bits
        return _lightgcn_hops(adj, x0, int(n_layers), lambda k, x_in: (None, None),
                              deferred=True), None
    out = torch.empty_like(x0)
    layers = work0 = work1 = None
    if return_layers:
        layers = torch.empty((n_layers, n, d), dtype=torch.float32, device=x0.device)
    elif n_layers > 1:
        work0 = torch.empty_like(x0)
        work1 = torch.empty_like(x0)
    elif n_layers == 1:
        work0 = work1 = torch.empty_like(x0)
    L = _lib.lib()
    ht = heavy_knobs(n, d)[0] if heavy_threshold is None else heavy_threshold
    check(L.gnnrec_lightgcn_heavy_f32(*_csr_args(adj), ptr(x0), d, int(n_layers), ptr(work0),
                                      ptr(work1), ptr(layers), ptr(out), d,
                                      *_heavy_args(adj, x0, ht), light_form_flag(adj, ht),
                                      _lib.stream_of(adj.device)),
          "gnnrec_lightgcn_heavy_f32")
    return out, layers


# ---- autograd: through the registered torch.library ops (src/ops/library.py) --------------
def spmm(adj: CsrGraph, x: torch.Tensor) -> torch.Tensor:
    """Drop-in for torch.sparse.mm(adj_matrix, x) with a CsrGraph operand (bit-exact):
    torch.ops.gnnrec.spmm, differentiable (backward = the same kernel over A^T)."""
    from . import library
    library.register(adj)
    return torch.ops.gnnrec.spmm(adj.row_ptr, adj.col, adj.val, x, adj.shape[1])


def lightgcn_propagate(adj: CsrGraph, x0: torch.Tensor, n_layers: int,
                       need: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused K-hop LightGCN propagation + layer mean (lightgcn.py:76-95), differentiable:
    torch.ops.gnnrec.lightgcn_propagate (backward = mean_k (A^T)^k g, its first hops skipping
    the all-zero rows of the sparse incoming gradient). With `need` (uint8 [N]) only those
    output rows are defined (lightgcn_forward_rows); the gradient must then be zero
    elsewhere, as it is when only those rows are read."""
    from . import library
    library.register(adj)
    return torch.ops.gnnrec.lightgcn_propagate(adj.row_ptr, adj.col, adj.val, x0, adj.shape[1],
                                               int(n_layers), need)


# ---- fused inference kernels ----------------------------------------------------------
def gas(x: torch.Tensor, blocks: torch.Tensor, perm: torch.Tensor) -> torch.Tensor:
    """GroupShuffleLayer forward: (x @ blockdiag(blocks))[:, perm] (gnnrec_gas_f32)."""
    x = _rowmajor(x)
    nb, bs, _ = blocks.shape
    d = x.shape[1]
    if nb * bs != d:
        raise ValueError("blocks do not tile the feature dimension")
    if x.device.type != "cuda":
        raise ValueError("gas needs a ROCm device tensor")
    y = torch.empty_like(x, memory_format=torch.contiguous_format)
    b = blocks.detach().to(x.device, torch.float32).contiguous()
    p = perm.to(x.device, torch.int32).contiguous()
    check(_lib.lib().gnnrec_gas_f32(ptr(x), x.stride(0), x.shape[0], d, bs, ptr(b), ptr(p),
                                    ptr(y), d, _lib.stream_of(x.device)), "gnnrec_gas_f32")
    return y


def spmm_gas(adj: CsrGraph, x: torch.Tensor, blocks: torch.Tensor,
             perm: torch.Tensor) -> torch.Tensor:
    """GAS(A x) in one kernel."""
    x = _rowmajor(x)
    _require_device(adj, x)
    nb, bs, _ = blocks.shape
    d = x.shape[1]
    y = torch.empty((adj.n_rows, d), dtype=torch.float32, device=x.device)
    b = blocks.detach().to(x.device, torch.float32).contiguous()
    p = perm.to(x.device, torch.int32).contiguous()
    check(_lib.lib().gnnrec_spmm_gas_f32(*_csr_args(adj), ptr(x), x.stride(0), ptr(y), d, d, bs,
                                         ptr(b), ptr(p), _lib.stream_of(adj.device)),
          "gnnrec_spmm_gas_f32")
    return y


def ngcf_layer(adj: CsrGraph, x: torch.Tensor, W1: torch.Tensor, b1: torch.Tensor,
               W2: torch.Tensor, b2: torch.Tensor, slope: float = 0.2,
               x_self: Optional[torch.Tensor] = None,
               gas_blocks: Optional[torch.Tensor] = None,
               gas_perm: Optional[torch.Tensor] = None, fused: bool = False,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """NGCFLayer.forward in eval mode (ngcf.py:69-84), optionally followed by GAS.
    fused=False (default): hop into a scratch table + streaming MFMA transform (faster on
    gather-bound graphs); fused=True: one kernel. x_self: the destination rows' own x (the
    rows of x by default; a rank's local rows when x is a sharded gather table)."""
    x = _rowmajor(x)
    if x_self is None:
        x_self = x
    _require_device(adj, x, x_self)
    d = x.shape[1]
    if W1.shape != (d, d) or W2.shape != (d, d):
        raise NotImplementedError("fused NGCF kernel needs square d x d Linear layers")
    if out is None:
        y = torch.empty((adj.n_rows, d), dtype=torch.float32, device=x.device)
    else:
        y = out
        if y.shape != (adj.n_rows, d) or y.stride(1) != 1 or y.stride(0) % 4:
            raise ValueError("out must be a row-major [n_rows, d] view with ld % 4 == 0")
        _require_device(adj, y)
    dev = x.device
    w1 = W1.detach().to(dev, torch.float32).contiguous()
    w2 = W2.detach().to(dev, torch.float32).contiguous()
    bb1 = b1.detach().to(dev, torch.float32).contiguous()
    bb2 = b2.detach().to(dev, torch.float32).contiguous()
    gb = gp = None
    bs = 0
    if gas_blocks is not None:
        gb = gas_blocks.detach().to(dev, torch.float32).contiguous()
        gp = gas_perm.to(dev, torch.int32).contiguous()
        bs = gb.shape[1]
    stream = _lib.stream_of(adj.device)
    if fused:
        check(_lib.lib().gnnrec_spmm_ngcf_f32(*_csr_args(adj), ptr(x), x.stride(0), ptr(x_self),
                                              x_self.stride(0), ptr(y), y.stride(0), d, ptr(w1),
                                              ptr(bb1), ptr(w2), ptr(bb2), float(slope), ptr(gb),
                                              ptr(gp), bs, None, stream), "gnnrec_spmm_ngcf_f32")
        return y
    # split form: the hop (heavy-row aware) into a scratch table, then the streaming transform
    work = torch.empty((adj.n_rows, d), dtype=torch.float32, device=x.device)
    spmm_into(adj, x, work)
    check(_lib.lib().gnnrec_ngcf_transform_f32(adj.n_rows, ptr(work), d, ptr(x_self),
                                               x_self.stride(0), ptr(y), y.stride(0), d, ptr(w1),
                                               ptr(bb1), ptr(w2), ptr(bb2), float(slope), ptr(gb),
                                               ptr(gp), bs, stream), "gnnrec_ngcf_transform_f32")
    return y


def dense_layer(adj: CsrGraph, x: torch.Tensor, M: torch.Tensor, c_out: float,
                resid: Optional[torch.Tensor], c_res: float, *, y: Optional[torch.Tensor] = None,
                acc: Optional[torch.Tensor] = None, acc_mode: int = 0, w_out: float = 0.0,
                w_res: float = 0.0, store_y: bool = True,
                fused: bool = False) -> Optional[torch.Tensor]:
    """c_out * ((A x) @ M) + c_res * resid, with the optional fused layer sum into `acc`."""
    x = _rowmajor(x)
    resid = _rowmajor(resid) if resid is not None else None
    _require_device(adj, x, resid, acc)
    d = x.shape[1]
    if store_y and y is None:
        y = torch.empty((adj.n_rows, d), dtype=torch.float32, device=x.device)
    m = M.detach().to(x.device, torch.float32).contiguous()
    tail = (ptr(y if store_y else None), y.stride(0) if store_y else d, d, ptr(m), float(c_out),
            ptr(resid), resid.stride(0) if resid is not None else d, float(c_res), ptr(acc),
            acc.stride(0) if acc is not None else d, int(acc_mode), float(w_out), float(w_res))
    stream = _lib.stream_of(adj.device)
    if fused:
        check(_lib.lib().gnnrec_spmm_dense_f32(*_csr_args(adj), ptr(x), x.stride(0), *tail, None,
                                               stream), "gnnrec_spmm_dense_f32")
    else:  # split form: heavy-row aware hop into a scratch table, then the transform
        work = torch.empty((adj.n_rows, d), dtype=torch.float32, device=x.device)
        spmm_into(adj, x, work)
        check(_lib.lib().gnnrec_dense_transform_f32(adj.n_rows, ptr(work), d, *tail, stream),
              "gnnrec_dense_transform_f32")
    return y if store_y else None


# GAT heavy-row split: rows with more than the threshold's neighbours run as segments of at
# most `segment` edges (partials merged per row). By operand (gat_knobs): large operands
# (G1B / 5M x 5M, request-bound) 2048 / 1024; small ones (<= SMALL_OPERAND_ROWS rows, e.g. the
# reference's ML-1M configs) are latency-bound on their longest per-row chains: 64 / 32 —
# the ML-1M-shaped GAT forward 1.09 -> 0.28-0.29 ms, outputs within 2.1e-9 of the unsplit
# kernels' (tools/exp_gat_small.py, profiles/r06/gat_small_knobs.jsonl). An int here forces it.
GAT_HEAVY_THRESHOLD: Optional[int] = None
GAT_SEGMENT: Optional[int] = None
GAT_LARGE_KNOBS = (2048, 1024)
GAT_SMALL_KNOBS = (64, 32)


def gat_knobs(n_rows: int) -> Tuple[int, int]:
    """(heavy threshold, segment length) of the GAT forward split for an operand of n_rows
    destination rows (GAT_HEAVY_THRESHOLD / GAT_SEGMENT when set)."""
    base = GAT_SMALL_KNOBS if n_rows <= SMALL_OPERAND_ROWS else GAT_LARGE_KNOBS
    return (GAT_HEAVY_THRESHOLD if GAT_HEAVY_THRESHOLD is not None else base[0],
            GAT_SEGMENT if GAT_SEGMENT is not None else base[1])


def gat_aggregate(adj: CsrGraph, h: torch.Tensor, s_self: torch.Tensor, s_neigh: torch.Tensor,
                  heads: int, o_dim: int, slope: float = 0.2, mean_heads: bool = False,
                  apply_elu: bool = False, *, out: Optional[torch.Tensor] = None, epi: int = 0,
                  self_rows: Optional[torch.Tensor] = None, acc: Optional[torch.Tensor] = None,
                  acc_div: float = 1.0, heavy_threshold: Optional[int] = None,
                  shared_rows: bool = False) -> Optional[torch.Tensor]:
    """Sparse edge-softmax aggregation of one GAT layer, all heads (gnnrec_gat_aggregate_f32),
    with rows longer than `heavy_threshold` split into segments (gnnrec_gat_heavy_f32).
    shared_rows: `h` is ONE [N, o_dim] table every head aggregates (head_stride 0), e.g. the
    layer input x when W_h is applied after the aggregation. heavy_threshold None:
    gat_knobs at call time; 0: no split."""
    knob_threshold, segment = gat_knobs(adj.n_rows)
    if heavy_threshold is None:
        heavy_threshold = knob_threshold
    h = _rowmajor(h)
    # score tables are read in place with their row strides (e.g. columns of the projection
    # output); only a column-strided view is compacted
    s_self = s_self if s_self.stride(1) == 1 else s_self.contiguous()
    s_neigh = s_neigh if s_neigh.stride(1) == 1 else s_neigh.contiguous()
    _require_device(adj, h, self_rows, acc)
    if h.shape[1] < (o_dim if shared_rows else heads * o_dim):
        raise ValueError("h is narrower than the aggregated rows")
    head_stride = 0 if shared_rows else o_dim
    width = o_dim if mean_heads else heads * o_dim
    if out is None and not (epi & EPI_NO_Y):
        out = torch.empty((adj.n_rows, width), dtype=torch.float32, device=h.device)
    plan = adj.heavy_plan(heavy_threshold, segment) if heavy_threshold > 0 else None
    common = (ptr(h), h.stride(0), head_stride, ptr(s_self), ptr(s_neigh), s_self.stride(0),
              s_neigh.stride(0), int(heads),
              int(o_dim), float(slope), int(mean_heads), int(apply_elu), ptr(out),
              out.stride(0) if out is not None else width, int(epi), ptr(self_rows),
              self_rows.stride(0) if self_rows is not None else width, ptr(acc),
              acc.stride(0) if acc is not None else width, float(acc_div))
    L = _lib.lib()
    stream = _lib.stream_of(adj.device)
    check(L.gnnrec_gat_aggregate_f32(ptr(adj.row_ptr), ptr(adj.col), adj.n_rows, *common,
                                     int(heavy_threshold if plan is not None else 0), stream),
          "gnnrec_gat_aggregate_f32")
    if plan is not None:
        n_seg = plan["seg_row"].numel()
        work = torch.empty(n_seg * (heads * o_dim + 2 * heads) + 4, dtype=torch.float32,
                           device=h.device)
        check(L.gnnrec_gat_heavy_f32(ptr(adj.col), ptr(plan["seg_row"]), ptr(plan["seg_beg"]),
                                     ptr(plan["seg_end"]), n_seg, ptr(plan["heavy_rows"]),
                                     ptr(plan["heavy_seg_ptr"]), plan["heavy_rows"].numel(),
                                     ptr(work), *common, stream), "gnnrec_gat_heavy_f32")
    return out


# Heavy-row segments of the scores-from-rows kernels: "column" runs them sorted by their first
# column (CsrGraph.heavy_plan_by_column), "row" in row order; GAT_XCD_ORDER gives each XCD a
# contiguous eighth of that list.
GAT_SEGMENT_ORDER = os.environ.get("GNNREC_GAT_SEGMENT_ORDER", "panel")
GAT_XCD_ORDER = os.environ.get("GNNREC_GAT_XCD_ORDER", "1") != "0"
# "panel" (the default): the heaviest rows (>= GAT_PANEL_MIN_EDGES edges per GAT_PANEL-column
# panel on average) are cut at panel boundaries (CsrGraph.heavy_plan_panels), the others as
# "column"; G1B 179.8 -> 176.7 ms, 5M x 5M 54.0 -> 53.6 ms (profiles/r05/c9_g1b_plans.jsonl,
# c5_gat_panels.jsonl)
GAT_PANEL = int(os.environ.get("GNNREC_GAT_PANEL", "8192"))
GAT_PANEL_MIN_EDGES = int(os.environ.get("GNNREC_GAT_PANEL_MIN_EDGES", "256"))


def gat_att_supported(o_dim: int) -> bool:
    """o_dim the ATT kernels take (a head's score dot spans o_dim / 4 <= 16 lanes)."""
    q = o_dim // 4
    return o_dim % 4 == 0 and 1 <= q <= 16 and (q & (q - 1)) == 0


def gat_aggregate_att(adj: CsrGraph, h: torch.Tensor, hself: torch.Tensor, att: torch.Tensor,
                      heads: int, o_dim: int, slope: float = 0.2, mean_heads: bool = False,
                      apply_elu: bool = False, *, out: Optional[torch.Tensor] = None,
                      epi: int = 0, self_rows: Optional[torch.Tensor] = None,
                      acc: Optional[torch.Tensor] = None, acc_div: float = 1.0,
                      heavy_threshold: Optional[int] = None,
                      shared_rows: bool = False) -> Optional[torch.Tensor]:
    """gat_aggregate with the attention scores formed in the kernel from the rows it reads
    (gnnrec_gat_aggregate_att_f32 / gnnrec_gat_heavy_att_f32): att [2, heads, o_dim] holds
    the self and neighbour attention vectors (shared_rows: the row vectors W_h^T a_h acting on
    the shared o_dim-wide row); hself: the destination rows' own rows of h's layout (row r of
    adj -> hself[r]). No score tables are read: a neighbour costs its feature row only."""
    knob_threshold, segment = gat_knobs(adj.n_rows)
    if heavy_threshold is None:
        heavy_threshold = knob_threshold
    if not gat_att_supported(o_dim):
        raise ValueError(f"gat_aggregate_att: o_dim = {o_dim} unsupported")
    h, hself = _rowmajor(h), _rowmajor(hself)
    att = att.to(device=h.device, dtype=torch.float32).contiguous()
    if att.numel() != 2 * heads * o_dim:
        raise ValueError("att must hold [2, heads, o_dim] floats")
    _require_device(adj, h, hself, self_rows, acc)
    row_w = o_dim if shared_rows else heads * o_dim
    if (h.shape[1] < row_w or hself.shape[1] < row_w or hself.shape[0] < adj.n_rows):
        raise ValueError("h / hself too small for the aggregated rows")
    head_stride = 0 if shared_rows else o_dim
    width = o_dim if mean_heads else heads * o_dim
    if out is None and not (epi & EPI_NO_Y):
        out = torch.empty((adj.n_rows, width), dtype=torch.float32, device=h.device)
    plan = None
    if heavy_threshold > 0:
        if GAT_SEGMENT_ORDER == "panel":
            plan = adj.heavy_plan_panels(heavy_threshold, segment, GAT_PANEL,
                                         GAT_PANEL_MIN_EDGES)
        elif GAT_SEGMENT_ORDER == "column":
            plan = adj.heavy_plan_by_column(heavy_threshold, segment)
        else:
            plan = adj.heavy_plan(heavy_threshold, segment)
    common = (ptr(h), h.stride(0), head_stride, ptr(hself), hself.stride(0), ptr(att),
              int(heads), int(o_dim), float(slope), int(mean_heads), int(apply_elu), ptr(out),
              out.stride(0) if out is not None else width, int(epi), ptr(self_rows),
              self_rows.stride(0) if self_rows is not None else width, ptr(acc),
              acc.stride(0) if acc is not None else width, float(acc_div))
    L = _lib.lib()
    stream = _lib.stream_of(adj.device)
    check(L.gnnrec_gat_aggregate_att_f32(ptr(adj.row_ptr), ptr(adj.col), adj.n_rows, *common,
                                         int(heavy_threshold if plan is not None else 0), stream),
          "gnnrec_gat_aggregate_att_f32")
    if plan is not None:
        n_seg = plan["seg_row"].numel()
        work = torch.empty(n_seg * (heads * o_dim + 2 * heads) + 4, dtype=torch.float32,
                           device=h.device)
        check(L.gnnrec_gat_heavy_att_f32(ptr(adj.col), ptr(plan["seg_row"]),
                                         ptr(plan["seg_beg"]), ptr(plan["seg_end"]), n_seg,
                                         ptr(plan["heavy_rows"]), ptr(plan["heavy_seg_ptr"]),
                                         plan["heavy_rows"].numel(), ptr(work), *common,
                                         ptr(plan.get("seg_pos")), int(GAT_XCD_ORDER), stream),
              "gnnrec_gat_heavy_att_f32")
    return out


# ---- GAT training (gnnrec_gat_train_forward_f32 / _backward_f32, csrc/gat_train.hip) ---------
def gat_train_supported(adj: CsrGraph, heads: int, o_dim: int) -> bool:
    """The native differentiable GAT aggregation applies: a square operand with a symmetric
    pattern on a ROCm device (its backward walks the columns as rows), heads * o_dim in
    {16 .. 256} and o_dim / 4 a power of two."""
    q = o_dim // 4
    return (isinstance(adj, CsrGraph) and adj.device.type == "cuda"
            and o_dim % 4 == 0 and q >= 1 and (q & (q - 1)) == 0
            and heads * o_dim in (16, 32, 64, 128, 256) and adj.pattern_symmetric())


# GAT training's heavy-row split (gnnrec_gat_train_*_split_f32): rows longer than the threshold
# are cut into segments of at most GAT_TRAIN_SEGMENT edges (CsrGraph.heavy_plan), their partial
# sums merged per row. 0 disables it (every row one lane group: a 4e5-neighbour hub then takes
# the whole step, profiles/r06/gat_train_*).
# By operand (gat_train_knobs): 2048 / 1024 on large operands; 128 / 64 up to
# SMALL_OPERAND_ROWS rows, where the per-row chains set the time — the ML-1M-shaped GAT training
# step (forward + backward, attention dropout) 10.8 -> 3.1 ms, loss and gradients equal to
# fp32 reassociation (tools/exp_gat_train.py --ml1m, profiles/r06/gat_train_ml1m_knobs.jsonl).
# An int here forces it.
GAT_TRAIN_HEAVY_THRESHOLD: Optional[int] = None
GAT_TRAIN_SEGMENT: Optional[int] = None
GAT_TRAIN_LARGE_KNOBS = (2048, 1024)
GAT_TRAIN_SMALL_KNOBS = (128, 64)


def gat_train_knobs(n_rows: int) -> Tuple[int, int]:
    """(heavy threshold, segment length) of the GAT training split for n_rows destination rows
    (GAT_TRAIN_HEAVY_THRESHOLD / GAT_TRAIN_SEGMENT when set)."""
    base = GAT_TRAIN_SMALL_KNOBS if n_rows <= SMALL_OPERAND_ROWS else GAT_TRAIN_LARGE_KNOBS
    return (GAT_TRAIN_HEAVY_THRESHOLD if GAT_TRAIN_HEAVY_THRESHOLD is not None else base[0],
            GAT_TRAIN_SEGMENT if GAT_TRAIN_SEGMENT is not None else base[1])


def _gat_train_split_args(adj: CsrGraph, F: int, heads: int, device):
    """(max_row_len, seg_row, seg_beg, seg_end, n_seg, heavy_rows, heavy_seg_ptr, n_heavy,
    work) for the split launches, or the no-split tuple; work is returned separately to keep
    it alive."""
    threshold, segment = gat_train_knobs(adj.n_rows)
    plan = adj.heavy_plan(threshold, segment) if threshold > 0 else None
    if plan is None:
        return (0, None, None, None, 0, None, None, 0, None), None
    n_seg = plan["seg_row"].numel()
    work = torch.empty(n_seg * (F + 2 * heads) + 4, dtype=torch.float32, device=device)
    return (int(threshold), ptr(plan["seg_row"]), ptr(plan["seg_beg"]),
            ptr(plan["seg_end"]), n_seg, ptr(plan["heavy_rows"]), ptr(plan["heavy_seg_ptr"]),
            plan["heavy_rows"].numel(), ptr(work)), work


class _GatTrainAggregate(torch.autograd.Function):
    """out[:, q*o:(q+1)*o] = dropout(softmax_j(LeakyReLU(s_self[r,q] + s_neigh[j,q]))) @ h_q —
    one GATLayer's per-head aggregation (gat.py:113-141) with its backward in two native passes;
    h, s_self and s_neigh are the differentiable inputs (the projections stay in autograd).
    Rows above gat_train_knobs' threshold run as merged segments in all three passes; the forward
    keeps the softmax statistics for the backward."""

    @staticmethod
    def forward(ctx, h, s_self, s_neigh, adj, heads, o_dim, slope, drop_p, seed):
        h, s_self, s_neigh = h.contiguous(), s_self.contiguous(), s_neigh.contiguous()
        n = adj.n_rows
        out = torch.empty((n, heads * o_dim), dtype=torch.float32, device=h.device)
        stats = torch.empty(n * heads * 4 + 4, dtype=torch.float32, device=h.device)
        split, work = _gat_train_split_args(adj, heads * o_dim, heads, h.device)
        check(_lib.lib().gnnrec_gat_train_forward_split_f32(
            ptr(adj.row_ptr), ptr(adj.col), n, ptr(h), h.stride(0), ptr(s_self), ptr(s_neigh),
            s_self.stride(0), int(heads), int(o_dim), float(slope), float(drop_p), int(seed),
            ptr(out), out.stride(0), ptr(stats), *split, _lib.stream_of(adj.device)),
            "gnnrec_gat_train_forward_split_f32")
        ctx.save_for_backward(h, s_self, s_neigh, out, stats)
        ctx.cfg = (adj, int(heads), int(o_dim), float(slope), float(drop_p), int(seed))
        return out

    @staticmethod
    def backward(ctx, dout):
        h, s_self, s_neigh, out, stats = ctx.saved_tensors
        adj, heads, o_dim, slope, drop_p, seed = ctx.cfg
        dout = dout.contiguous()
        n = adj.n_rows
        dh = torch.empty_like(h)
        d_self = torch.empty_like(s_self)
        d_neigh = torch.empty_like(s_neigh)
        split, work = _gat_train_split_args(adj, heads * o_dim, heads, h.device)
        check(_lib.lib().gnnrec_gat_train_backward_split_f32(
            ptr(adj.row_ptr), ptr(adj.col), n, ptr(h), h.stride(0), ptr(s_self), ptr(s_neigh),
            s_self.stride(0), heads, o_dim, slope, drop_p, seed, ptr(out), out.stride(0),
            ptr(dout), dout.stride(0), ptr(stats), ptr(dh), dh.stride(0), ptr(d_self),
            ptr(d_neigh), *split, _lib.stream_of(adj.device)),
            "gnnrec_gat_train_backward_split_f32")
        return dh, d_self, d_neigh, None, None, None, None, None, None


def gat_aggregate_train(adj: CsrGraph, h: torch.Tensor, s_self: torch.Tensor,
                        s_neigh: torch.Tensor, heads: int, o_dim: int, slope: float = 0.2,
                        drop_p: float = 0.0, seed: int = 0) -> torch.Tensor:
    """Differentiable per-head GAT aggregation on the native kernels: h [N, heads*o_dim]
    (head-major), s_self / s_neigh [N, heads]; attention dropout drop_p with a counter-based
    mask of `seed` (regenerated by the backward). Returns [N, heads*o_dim] (heads
    concatenated)."""
    if not gat_train_supported(adj, heads, o_dim):
        raise ValueError("gat_aggregate_train: needs a symmetric square CsrGraph on a ROCm "
                         "device, heads*o_dim in {16..256}, o_dim/4 a power of two")
    _require_device(adj, h, s_self, s_neigh)
    if h.shape != (adj.n_rows, heads * o_dim) or s_self.shape != (adj.n_rows, heads) \
            or s_neigh.shape != (adj.n_rows, heads):
        raise ValueError("gat_aggregate_train: h [N, heads*o_dim], s_self / s_neigh [N, heads]")
    return _GatTrainAggregate.apply(h.float(), s_self.float(), s_neigh.float(), adj, heads,
                                    o_dim, slope, drop_p, seed & 0xFFFFFFFF)


# ---- Linear layers whose weight gradient reduces over every row (training) -----------------
# nn.Linear's weight gradient dW = dY^T X is a [out, in] product with an N-long reduction: one
# library GEMM gives it one or two output tiles that each walk all N rows (64 x 64 over 2M rows
# 2.93 ms). Cut into row chunks as one batched GEMM plus a sum over the chunks it is 0.23 ms,
# and closer to the float64 value (tools/exp_linear_dw.py, profiles/r06/linear_dw.jsonl:
# 9 746 rows 0.073 -> 0.054 ms, 200K 0.40 -> 0.058 ms). Forward and input gradient are
# nn.Linear's own ops. Below SMALL_OPERAND_ROWS rows the autograd Function's own overhead
# outweighs the GEMM it saves (ML-1M-shaped NGCF step 2.1 -> 3.2 ms with it), so those keep
# nn.Linear; config 5's 2M x 2M GAT training step 222.8 -> 176.9 ms
# (profiles/r06/gat_train_slice_linear_rows.jsonl, same loss and gradient sums).
LINEAR_SPLIT_K_MIN_ROWS = 65536


def _dw_split_k(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dy^T x ([out, in]) as chunked partial products summed over the chunks."""
    n = dy.shape[0]
    chunk = max(256, (n // 512) // 64 * 64)
    c = n // chunk
    w = torch.bmm(dy[:c * chunk].view(c, chunk, -1).transpose(1, 2),
                  x[:c * chunk].view(c, chunk, -1)).sum(0)
    if c * chunk < n:
        w = w + dy[c * chunk:].t() @ x[c * chunk:]
    return w


class _LinearRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return torch.nn.functional.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = (dy2 @ weight).view(x.shape)
        if ctx.needs_input_grad[1]:
            dw = (_dw_split_k(dy2, x2) if dy2.shape[0] >= LINEAR_SPLIT_K_MIN_ROWS
                  else dy2.t() @ x2)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy2.sum(0)
        return dx, dw, db


def linear_rows(x: torch.Tensor, layer: torch.nn.Linear) -> torch.Tensor:
    """layer(x) with the weight gradient reduced over row chunks (_dw_split_k) on a ROCm
    device when x has at least LINEAR_SPLIT_K_MIN_ROWS rows and autograd needs it; the
    forward is nn.Linear's. Otherwise layer(x) itself."""
    if not (x.is_cuda and torch.is_grad_enabled() and layer.weight.requires_grad
            and x.reshape(-1, x.shape[-1]).shape[0] >= LINEAR_SPLIT_K_MIN_ROWS):
        return layer(x)
    return _LinearRows.apply(x, layer.weight, layer.bias)


def rows_gemm_supported(k: int, p: int) -> bool:
    """(k, p) shapes gnnrec_rows_gemm_f32 has an instance for (csrc/dense_epi.hip)."""
    return k in (64, 128, 256) and p % 4 == 0 and 0 < p <= (80 if k == 64 else 64)


def _rows_view_ok(t: torch.Tensor) -> bool:
    return t.dim() == 2 and t.stride(-1) == 1 and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0


def rows_gemm(x: torch.Tensor, B: torch.Tensor, out: Optional[torch.Tensor] = None, *,
              apply_elu: bool = False, epi: int = 0, self_rows: Optional[torch.Tensor] = None,
              acc: Optional[torch.Tensor] = None, acc_div: float = 1.0) -> Optional[torch.Tensor]:
    """x [n, k] @ B [k, p] on the matrix cores (gnnrec_rows_gemm_f32): the tall-skinny GAT
    projections, streamed at HBM rate instead of hipBLASLt's 1-3 TB/s, with GAT's epilogue
    optionally fused (ELU, then the layer-mean accumulator acc = (self_rows | acc) + y
    [/ acc_div], as gat_aggregate). fp32 (tolerance-equal to torch.matmul). Native only: a
    shape the kernel has no instance for (rows_gemm_supported), a tensor off x's device or a
    misaligned view raises — the caller decides what runs instead (GATLayer._project)."""
    if x.dim() != 2 or B.dim() != 2:
        raise ValueError("rows_gemm: x and B must be 2-D")
    n, k = x.shape
    p = B.shape[1]
    no_y = bool(epi & EPI_NO_Y)
    if B.shape[0] != k:
        raise ValueError(f"rows_gemm: B has {B.shape[0]} rows, x has {k} columns")
    if not x.is_cuda:
        raise ValueError("rows_gemm needs x on a ROCm device")
    rows = [t for t in (out, self_rows, acc) if t is not None]
    for t in [B] + rows:
        if t.device != x.device:
            raise ValueError(f"rows_gemm: tensor on {t.device}, x on {x.device}")
    for t in [x, B] + rows:
        if t.dtype != torch.float32:
            raise TypeError(f"rows_gemm: expected float32, got {t.dtype}")
    for t, w in ((out, p), (self_rows, p), (acc, p)):
        if t is not None and (t.shape[0] != n or t.shape[1] < w):
            raise ValueError("rows_gemm: out / self_rows / acc must be [n, >= p]")
    if epi & EPI_ACC_INIT and self_rows is None or epi & (EPI_ACC_INIT | EPI_ACC_ADD) and acc is None:
        raise ValueError("rows_gemm: the ACC epilogue needs acc (and self_rows for ACC_INIT)")
    if not rows_gemm_supported(k, p):
        raise NotImplementedError(f"rows_gemm: no kernel instance for k={k}, p={p} "
                                  "(k 64: p <= 80; k 128/256: p <= 64; p % 4 == 0)")
    if not all(_rows_view_ok(t) for t in [x] + rows):
        raise ValueError("rows_gemm: x / out / self_rows / acc must be row-major views with "
                         "ld % 4 == 0 and 16-B aligned rows")
    Bc = B.contiguous()
    if out is None and not no_y:
        out = torch.empty((n, p), dtype=torch.float32, device=x.device)
    y = None if no_y else out
    check(_lib.lib().gnnrec_rows_gemm_f32(
        n, ptr(x), x.stride(0), k, ptr(Bc), p, ptr(y), y.stride(0) if y is not None else p,
        int(apply_elu), int(epi), ptr(self_rows),
        self_rows.stride(0) if self_rows is not None else p, ptr(acc),
        acc.stride(0) if acc is not None else p, float(acc_div), _lib.stream_of(x.device)),
        "gnnrec_rows_gemm_f32")
    return y


def score_topk(user_emb: torch.Tensor, item_emb: torch.Tensor, k: int,
               seen_ptr: Optional[torch.Tensor] = None,
               seen_col: Optional[torch.Tensor] = None,
               n_split: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Top-k items per user by score = sequential-fmaf dot product, seen items excluded,
    order (score desc, item index asc) (gnnrec_score_topk_f32; evaluator.py:96-105).
    seen_ptr [B+1] int64 / seen_col int32: per-user sorted seen item lists (CSR)."""
    u = _rowmajor(user_emb)
    v = _rowmajor(item_emb)
    if not (u.is_cuda and v.is_cuda and u.device == v.device):
        raise ValueError("score_topk needs both tables on the same ROCm device")
    if u.dtype != torch.float32 or v.dtype != torch.float32:
        raise TypeError("score_topk needs float32 tables")
    B, d = u.shape
    dp = next((w for w in (16, 32, 64, 128, 256) if w >= d), None)
    if dp is None:
        raise NotImplementedError(f"score_topk: d={d} > 256")
    if dp != d:  # zero columns leave every fmaf chain unchanged
        u = torch.nn.functional.pad(u, (0, dp - d))
        v = torch.nn.functional.pad(v, (0, dp - d))
        d = dp
    idx = torch.empty((B, k), dtype=torch.int64, device=u.device)
    sc = torch.empty((B, k), dtype=torch.float32, device=u.device)
    if seen_ptr is not None:
        seen_ptr = seen_ptr.to(u.device, torch.int64).contiguous()
        seen_col = seen_col.to(u.device, torch.int32).contiguous()
    n_split = topk_splits(B, v.shape[0], d, k) if n_split is None else int(n_split)
    wi = ws = None
    if n_split > 1:
        wi = torch.empty((B, n_split, k), dtype=torch.int64, device=u.device)
        ws = torch.empty((B, n_split, k), dtype=torch.float32, device=u.device)
    check(_lib.lib().gnnrec_score_topk_split_f32(ptr(u), u.stride(0), B, ptr(v), v.stride(0),
                                                 v.shape[0], d, ptr(seen_ptr), ptr(seen_col),
                                                 int(k), n_split, ptr(wi), ptr(ws), ptr(idx),
                                                 ptr(sc), _lib.stream_of(u.device)),
          "gnnrec_score_topk_split_f32")
    return idx, sc


def topk_splits(n_users: int, n_items: int, d: int, k: int = 20,
                target_wg: Optional[int] = None) -> int:
    """Item ranges for gnnrec_score_topk_split_f32: enough workgroups to fill the 256 CUs in
    one round — 512 of 128 users for d <= 64 and k <= 64 (two per CU: 68 KB LDS, 240
    registers per lane; csrc/topk.hip launch_topk), else 1024 of 64 — each range at least 16
    tiles long. Measured (profiles/r02/config8_uf2_splits.jsonl): 16K users 35.7 ms at 512
    workgroups vs 43.6 at 1024; 2K users 10.5 ms at 512 vs 16.8 at 1024."""
    two = d <= 64 and k <= 64
    upb = 128 if two else 64
    target_wg = target_wg or (512 if two else 1024)
    wg = max(1, -(-n_users // upb))
    tile = 64 if d <= 128 else 32
    return int(max(1, min(-(-target_wg // wg), n_items // (16 * tile), 65535)))
