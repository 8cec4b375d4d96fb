// Column-ordered ("tiled") SpMM hop for any d % 32 == 0 (gnnrec_spmm_tiled_f32).
//
// Same arithmetic as spmm_vec_kernel — replaces torch.sparse.mm(adj, x) of the reference
// (baselines/lightgcn.py:88,178) with y[r] = fmaf chain over the row's neighbours in ascending
// column order from +0 — but a different schedule. The row-parallel hop gathers every
// neighbour row from beyond L2 (G100M: 16x the compulsory bytes). Here one persistent
// 1024-thread workgroup per CU owns R destination rows per pass with fp32 accumulators in
// LDS, and its 16 waves walk the rows' edges PANEL BY PANEL in ascending source column
// (a step = one panel; a workgroup barrier between steps, so a row may move to another wave
// from one step to the next without reordering its chain). The workgroups of a blockIdx % 8
// group (one XCD under round-robin placement — speed only, never correctness) meet at every
// pass start (bounded counter wait), so they sweep the same panels together and a gathered
// source row is reused from the XCD's L2 by the group's other rows.
//
// Feature slices: a pass computes ONE 32-feature slice of its block's rows (a gather = one
// 128-B line of a source row; the LDS row = 128 B), so R is twice what whole 64-feature rows
// allow and an XCD group's pass covers twice the rows, touching each gathered line for more of
// them (G100M: 14 passes x 1117 rows x 2 slices instead of 14 x 559 x 1). A d-wide hop is d/32
// sweeps of the same plan; the work items are (slice, block) pairs, slice-major.
//
// The two 32-lane halves of a wave take two slot streams (lane = half * 32 + feature). A chunk
// holds 16 slots per half. Every lane loads ITS slot's word (column offset from the chunk's
// panel base | local row), value and one word of the chunk header once per chunk (lane l:
// slot (l / 32, l % 16)), and step t broadcasts slot t of each half to that half with DPP
// row_newbcast:t (a 16-lane row reads its lane t), fused into the address add where the
// compiler can; the header words (v_readlane) carry the step barriers, the chain mask (slot t
// continues slot t-1's row in the same half: take the register value, not LDS) and the panel
// base the chunk's buffer resource starts at. Pipeline per wave: chunk c+2's slot loads,
// chunk c+1's gathers and chunk c's LDS read-fmaf-write in flight together. What bounds it:
// the per-CU L1 miss path (one L2 request per gathered 128-B line).
#include <algorithm>
#include <atomic>
#include <mutex>
#include <new>
#include <thread>
#include <utility>
#include <vector>

#include "common.h"

namespace gnnrec {

constexpr int kTiledWaves = GNNREC_TILED_WAVES;
constexpr int kTiledChunk = GNNREC_TILED_CHUNK;   // slots per chunk (both halves)
constexpr int kHalf = kTiledChunk / 2;            // slots per half = steps per chunk
constexpr int kTiledTail = GNNREC_TILED_TAIL;
constexpr int kSlice = 32;                        // features per pass
constexpr int kRowBits = 11;
constexpr int kRowMask = (1 << kRowBits) - 1;
constexpr int kMaxPanel = 1 << 20;                // columns per panel (slot word: 21 bits)
constexpr int kMaxRowBytes = GNNREC_TILED_MAX_LDX * 4;   // keeps the lane offset 32-bit
constexpr int kGroup = 8;                         // steps whose reads precede their writes
#ifndef GNNREC_TILED_EPI_BATCH
#define GNNREC_TILED_EPI_BATCH 20
#endif
constexpr int kEpiBatch = GNNREC_TILED_EPI_BATCH;   // epilogue rows per half-wave, loads in flight
#ifndef GNNREC_TILED_EPI_PRELOAD
#define GNNREC_TILED_EPI_PRELOAD 1   // the first batch's base rows loaded before the pass-end barriers
#endif
// epilogue stores non-temporal (aux bit 1, nt): the rows are read again only by the next
// launch; 12.62 -> 12.56 ms per step (profiles/r02/exp_epi_store_policy.jsonl; sc1 write-through, 12.60)
constexpr int kEpiStoreAux = 2;
#ifndef GNNREC_TILED_EPI_BATCH3
#define GNNREC_TILED_EPI_BATCH3 10
#endif
constexpr int kEpiBatch3 = GNNREC_TILED_EPI_BATCH3;   // the same with 2-3 base inputs per row
static_assert(kHalf == 16, "a half-chunk is one DPP row of 16 lanes");
static_assert(kHalf == 2 * kGroup, "a half-chunk is applied as two groups");
static_assert(GNNREC_TILED_MAX_ROWS < kRowMask, "row field is 11 bits (row R = scratch)");
static_assert((GNNREC_TILED_MAX_ROWS + 1) * kSlice * 4 <= 160 * 1024, "LDS");
static_assert((int64_t)kMaxPanel * kMaxRowBytes <= ((int64_t)1 << 32), "32-bit lane offsets");

// ---- device -----------------------------------------------------------------------------
#ifdef GNNREC_TILED_TRACE
// Diagnostic build only (tools/trace_tiled.py): wave 0 of each workgroup stamps wall_clock64
// at every pass start and step barrier into g_tiled_trace[blockIdx][event].
constexpr int kTraceEvents = 1024;
__device__ unsigned long long* g_tiled_trace;
#define GNNREC_TILED_STAMP(ev)                                                    \
  do {                                                                            \
    if (threadIdx.x == 0 && g_tiled_trace && (ev) < kTraceEvents)                 \
      g_tiled_trace[(size_t)blockIdx.x * kTraceEvents + (ev)] = wall_clock64();   \
    ++(ev);                                                                       \
  } while (0)
#else
#define GNNREC_TILED_STAMP(ev) ((void)0)
#endif

struct TiledSlots {   // this lane's slot of the chunk: (half, lane % 16)
  uint32_t o;         // byte offset of the source row from the chunk's panel base
  float v;
  uint32_t r;         // byte offset of the destination row's accumulator in LDS
  uint32_t h;         // word (lane % 4) of the chunk header
};

template <int T>
__device__ __forceinline__ uint32_t bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x150 + T, 0xF, 0xF, true);
}
template <int T>
__device__ __forceinline__ float bcastf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               0x150 + T, 0xF, 0xF, true));
}

// Slot word: (column - chunk's panel base) << kRowBits | local row. The chunk header {step
// barriers before the chunk, chain mask, panel base column, 0} is loaded with the slots as a
// vector load (lane l: word l % 4) and read back with v_readlane: a scalar load would share
// lgkmcnt with the LDS chain and stall it.
__device__ __forceinline__ void tiled_slots(const uint32_t* __restrict__ ss,
                                            const float* __restrict__ sv,
                                            const uint32_t* __restrict__ hdr, int64_t c,
                                            int my_slot, int lane, uint32_t row_bytes,
                                            TiledSlots& m) {
  const int64_t i = c * kTiledChunk + my_slot;
  const uint32_t wd = ss[i];
  m.o = __umul24(wd >> kRowBits, row_bytes);
  m.v = sv[i];
  m.r = (wd & kRowMask) * (kSlice * 4);
  m.h = hdr[4 * c + (lane & 3)];
}

template <int W>
__device__ __forceinline__ uint32_t hdr_word(const TiledSlots& m) {
  return (uint32_t)__builtin_amdgcn_readlane((int)m.h, W);
}

// The gathers of a chunk read through a buffer whose base is its panel's first source row, so
// lane offsets stay 32-bit for any table size.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t chunk_rsrc(const char* xs, uint64_t xs_bytes,
                                                             uint32_t base, uint32_t row_bytes) {
  const uint64_t off = (uint64_t)base * row_bytes;
  const uint64_t left = off < xs_bytes ? xs_bytes - off : 0;
  const uint32_t n = left > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)left;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(xs) + off, 0, (int)n, 0x00020000);
}

// Rows [r0, r0 + rows) of a row-major fp32 table (row stride ld), from column slice * 32: the
// range ends right after the last row's slice, so offsets of later rows are out of range.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const float* p, int64_t r0,
                                                            int64_t ld, int slice, int rows) {
  const float* b = p ? p + r0 * ld + (int64_t)slice * kSlice : p;
  const uint32_t n = p ? (uint32_t)(rows - 1) * (uint32_t)ld * 4u + kSlice * 4u : 0u;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(b), 0, (int)n, 0x00020000);
}

template <int... T>
__device__ __forceinline__ void tiled_gather(std::integer_sequence<int, T...>,
                                             __amdgpu_buffer_rsrc_t xr, uint32_t f4,
                                             const TiledSlots& m, float (&x)[kHalf]) {
  ((x[T] = __builtin_bit_cast(
        float, __builtin_amdgcn_raw_buffer_load_b32(xr, bcast<T>(m.o) + f4, 0, 0))),
   ...);
}

// lane-wise select on a wave-uniform 64-bit lane mask held in SGPRs (no compare per lane)
__device__ __forceinline__ float select_lanes(float if0, float if1, uint64_t mask) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if0), "v"(if1), "s"(mask));
  return r;
}

template <int T>
__device__ __forceinline__ uint64_t chain_lanes(uint32_t cm) {
  // slot T of half 0 (lanes 0-31): bit T; of half 1 (lanes 32-63): bit 16 + T
  const uint32_t lo = 0u - ((cm >> T) & 1u), hi = 0u - ((cm >> (16 + T)) & 1u);
  return ((uint64_t)hi << 32) | lo;
}

// Steps G .. G+7 of a chunk: 8 accumulator reads, 8 chained fmaf, 8 writes. A chunk is
// applied as two such groups, so a row may appear in both groups of a piece: the second
// group's reads follow the first group's writes in the wave's LDS order (and a slot at step 8
// chaining on step 7 selects the value step 7 just wrote).
template <int G, int... T>
__device__ __forceinline__ void tiled_apply8(std::integer_sequence<int, T...>, char* base,
                                             uint32_t f4, const TiledSlots& m,
                                             const float (&x)[kHalf], uint32_t cm,
                                             float& prev) {
  uint32_t a[sizeof...(T)];
  ((a[T] = bcast<G + T>(m.r) + f4), ...);
  float av[sizeof...(T)];
  ((av[T] = *reinterpret_cast<float*>(base + a[T])), ...);
  // slot t continuing slot t-1's row (same half) chains on its register value
  ((av[T] = __builtin_fmaf(bcastf<G + T>(m.v), x[G + T],
                           G + T > 0 ? select_lanes(av[T], T > 0 ? av[T > 0 ? T - 1 : 0] : prev,
                                                    chain_lanes<G + T>(cm))
                                     : av[T])),
   ...);
  ((*reinterpret_cast<float*>(base + a[T]) = av[T]), ...);
  prev = av[sizeof...(T) - 1];
}

__device__ __forceinline__ void tiled_apply(float* acc, uint32_t f4, const TiledSlots& m,
                                            const float (&x)[kHalf], uint32_t cm) {
  constexpr auto k8 = std::make_integer_sequence<int, kGroup>{};
  char* base = reinterpret_cast<char*>(acc);
  float prev = 0.f;
  tiled_apply8<0>(k8, base, f4, m, x, cm, prev);
  tiled_apply8<kGroup>(k8, base, f4, m, x, cm, prev);
}

// Pass-end epilogue of one half-wave: its rows i = rl + 32q of the block (rl = 2 * wave +
// half), B at a time with every load of a batch issued before the first use. All offsets are
// 32-bit rows of buffers based at the block's first row whose ranges end at the last valid
// row: loads past it return 0 and stores are dropped, so there is no branch (a branch around
// a load makes the compiler wait for it in place). A null ry: no y output.
// NB base inputs (the layer-mean terms before this hop, in layer order): acc_out =
// (((b0 [+ b1]) [+ b2]) + y) [/ div] — b0 = x0 (ACC_INIT) or the running sum (ACC_ADD);
// INIT|ADD: b0 = x0, b1 = the acc rows (an earlier layer parked there); ACC_X: the hop's
// input row x[r] (the previous layer) last. NB = 0: y only.
template <int NB, int B, class Wait>
__device__ __forceinline__ void tiled_epilogue(const float* acc, int R, int rl, uint32_t f4,
                                               __amdgpu_buffer_rsrc_t ry, uint32_t ly,
                                               __amdgpu_buffer_rsrc_t rb0, uint32_t lb0,
                                               __amdgpu_buffer_rsrc_t rb1, uint32_t lb1,
                                               __amdgpu_buffer_rsrc_t rb2, uint32_t lb2,
                                               __amdgpu_buffer_rsrc_t ra, uint32_t la,
                                               bool div, float acc_div, Wait wait) {
  constexpr int kStride = 2 * kTiledWaves;
  const __amdgpu_buffer_rsrc_t rb[3] = {rb0, rb1, rb2};
  const uint32_t lb[3] = {lb0, lb1, lb2};
  float base[NB > 0 ? NB : 1][B];
  // the base rows of batch i0 (global, independent of the pass: the first batch is loaded
  // before the pass-end barriers, so its latency hides behind the block's slowest wave)
  auto load_base = [&](int i0) {
    // per-row offsets advance by a stride; the opaque copy keeps the compiler from hoisting
    // B x 3 of them out of the persistent loop (they would spill)
    uint32_t ob[3];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      ob[j] = (uint32_t)i0 * lb[j] + f4;
      asm volatile("" : "+v"(ob[j]));
    }
#pragma unroll
    for (int q = 0; q < B; ++q)
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        base[j][q] =
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb[j], ob[j], 0, 0));
        ob[j] += kStride * lb[j];
      }
  };
  int i0 = rl;
  if (GNNREC_TILED_EPI_PRELOAD) load_base(i0);
  wait();
  // the first batch runs even when rl is past the block's rows: its LDS reads stay inside
  // (row R is the scratch row) and its stores fall outside the buffer ranges
  for (;;) {
    if (!GNNREC_TILED_EPI_PRELOAD) load_base(i0);
    uint32_t ol = (uint32_t)i0;
    asm volatile("" : "+v"(ol));
    float a[B];
#pragma unroll
    for (int q = 0; q < B; ++q) {
      a[q] = acc[min(ol, (uint32_t)R) * kSlice + (f4 >> 2)];
      ol += kStride;
    }
    uint32_t oy = (uint32_t)i0 * ly + f4, oa = (uint32_t)i0 * la + f4;
    asm volatile("" : "+v"(oy), "+v"(oa));
#pragma unroll
    for (int q = 0; q < B; ++q) {
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, a[q]), ry, oy, 0, kEpiStoreAux);
      oy += kStride * ly;
      if (NB > 0) {
        float bsum = base[0][q];
#pragma unroll
        for (int j = 1; j < NB; ++j) bsum = bsum + base[j][q];
        bsum = bsum + a[q];
        if (div) bsum = bsum / acc_div;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, bsum), ra, oa, 0, kEpiStoreAux);
        oa += kStride * la;
      }
    }
    i0 += kStride * B;
    if (i0 - (rl & 1) >= R) break;
    if (GNNREC_TILED_EPI_PRELOAD) load_base(i0);
  }
}

__global__ __launch_bounds__(kTiledWaves * 64) void tiled_hop_kernel(
    const uint32_t* __restrict__ ss, const float* __restrict__ sv,
    const uint32_t* __restrict__ hdr, const int64_t* __restrict__ wptr,
    const int32_t* __restrict__ nsteps, int n_blocks, int nb_pad, int n_items, int R,
    const float* __restrict__ x, uint64_t x_bytes, uint32_t row_bytes,
    float* __restrict__ y, int64_t ldy, int64_t n_rows, int epi, const float* __restrict__ self,
    int64_t ld_self, float* __restrict__ accg, int64_t ld_acc, float acc_div,
    unsigned* __restrict__ sync, unsigned meet_ticks) {
  extern __shared__ float acc[];  // [(R+1)][32]: row R is the padding slots' scratch row
  constexpr auto kSeq = std::make_integer_sequence<int, kHalf>{};
  const int lane = threadIdx.x & 63;
  const int half = lane >> 5;
  const int f = lane & 31;
  const uint32_t f4 = (uint32_t)f * 4;
  const int my_slot = half * kHalf + (lane & 15);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  unsigned* ctr = sync + (blockIdx.x % 8) * 32;   // the group's counter, own 128-B line
  const long long G = gridDim.x / 8 + ((blockIdx.x % 8) < (gridDim.x % 8) ? 1 : 0);
  long long pass = 0;
#ifdef GNNREC_TILED_TRACE
  int ev = 0;
#endif
  for (int item = blockIdx.x; item < n_items; item += gridDim.x, ++pass) {
    if (threadIdx.x == 0 && pass > 0 && meet_ticks > 0) {
      // pass start: report the finished pass, wait (bounded) for the group's others
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long t0 = wall_clock64();
      while ((long long)__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                 G * pass &&
             wall_clock64() - t0 < meet_ticks)
        __builtin_amdgcn_s_sleep(2);
    }
    const int slice = item / nb_pad, blk = item - slice * nb_pad;
    if (blk >= n_blocks) continue;   // padding item (uniform over the workgroup)
    for (int i = threadIdx.x; i < (R + 1) * kSlice; i += kTiledWaves * 64) acc[i] = 0.f;
    __syncthreads();
    GNNREC_TILED_STAMP(ev);
    const uint32_t soff = (uint32_t)slice * kSlice * 4;
    const char* xs = reinterpret_cast<const char*>(x) + soff;
    const uint64_t xs_bytes = x_bytes - soff;
    const int64_t s = (int64_t)blk * kTiledWaves + w;
    const int64_t b = wptr[s], e = wptr[s + 1];
    int cur = 0;
    if (b < e) {
      // slot loads (and headers) two chunks ahead, gathers one chunk ahead of the LDS chain (a
      // third chunk of gathers in flight measured the same: profiles/r02/tiled_depth3.jsonl)
      TiledSlots M0, M1, M2;
      float X0[kHalf], X1[kHalf];
      int64_t c = b;
      tiled_slots(ss, sv, hdr, c, my_slot, lane, row_bytes, M0);
      tiled_slots(ss, sv, hdr, c + 1, my_slot, lane, row_bytes, M1);
      tiled_gather(kSeq, chunk_rsrc(xs, xs_bytes, hdr_word<2>(M0), row_bytes), f4, M0, X0);
#define GNNREC_TILED_STAGE(MLOAD, MG, XG, MA, XA)                                     \
  {                                                                                   \
    tiled_slots(ss, sv, hdr, c + 2, my_slot, lane, row_bytes, MLOAD);                 \
    tiled_gather(kSeq, chunk_rsrc(xs, xs_bytes, hdr_word<2>(MG), row_bytes), f4, MG, XG); \
    const int bar = (int)hdr_word<0>(MA);                                             \
    for (int i = 0; i < bar; ++i) {                                                   \
      __syncthreads();                                                                \
      GNNREC_TILED_STAMP(ev);                                                         \
    }                                                                                 \
    cur += bar;                                                                       \
    tiled_apply(acc, f4, MA, XA, hdr_word<1>(MA));                                    \
    if (++c >= e) break;                                                              \
  }
      for (;;) {
        GNNREC_TILED_STAGE(M2, M1, X1, M0, X0)
        GNNREC_TILED_STAGE(M0, M2, X0, M1, X1)
        GNNREC_TILED_STAGE(M1, M0, X1, M2, X0)
        GNNREC_TILED_STAGE(M2, M1, X0, M0, X1)
        GNNREC_TILED_STAGE(M0, M2, X1, M1, X0)
        GNNREC_TILED_STAGE(M1, M0, X0, M2, X1)
      }
#undef GNNREC_TILED_STAGE
    }
    const int ns = nsteps[blk];
    auto wait = [&]() {
      for (int i = cur; i < ns; ++i) {  // this wave's remaining steps + the last
        __syncthreads();
        GNNREC_TILED_STAMP(ev);
      }
    };
    // epilogue: half-wave h of wave w owns rows i = 2w + h + 32q (see tiled_epilogue)
    const int64_t r0 = (int64_t)blk * R;
    const int nv = (int)min((int64_t)R, n_rows - r0);
    const int rl = 2 * w + half;
    const __amdgpu_buffer_rsrc_t ry = rows_rsrc((epi & GNNREC_EPI_NO_Y) ? nullptr : y, r0, ldy,
                                                slice, nv);
    // base inputs in layer order: x0 (INIT), the acc rows (ADD), the input rows (ACC_X)
    const bool init = (epi & GNNREC_EPI_ACC_INIT) != 0, add = (epi & GNNREC_EPI_ACC_ADD) != 0,
               xin = (epi & GNNREC_EPI_ACC_X) != 0;
    const int nb = (int)init + (int)add + (int)xin;
    const __amdgpu_buffer_rsrc_t rs = rows_rsrc(init ? self : nullptr, r0, ld_self, slice, nv);
    const __amdgpu_buffer_rsrc_t racc = rows_rsrc(nb ? accg : nullptr, r0, ld_acc, slice, nv);
    const __amdgpu_buffer_rsrc_t rx = rows_rsrc(xin ? x : nullptr, r0, row_bytes / 4, slice, nv);
    const uint32_t ls = (uint32_t)ld_self * 4, la = (uint32_t)ld_acc * 4, ly = (uint32_t)ldy * 4;
    const __amdgpu_buffer_rsrc_t rb0 = init ? rs : racc, rb1 = (init && add) ? racc : rx;
    const uint32_t lb0 = init ? ls : la, lb1 = (init && add) ? la : row_bytes;
    const bool div = (epi & GNNREC_EPI_ACC_DIV) != 0;
#define GNNREC_TILED_EPI(NB, B, DIV) \
  tiled_epilogue<NB, B>(acc, R, rl, f4, ry, ly, rb0, lb0, rb1, lb1, rx, row_bytes, racc, la, DIV, \
                        acc_div, wait)
    if (nb == 0)
      GNNREC_TILED_EPI(0, kEpiBatch, false);
    else if (nb == 1)
      GNNREC_TILED_EPI(1, kEpiBatch, div);
    else if (nb == 2)
      GNNREC_TILED_EPI(2, kEpiBatch3, div);
    else
      GNNREC_TILED_EPI(3, kEpiBatch3, div);
#undef GNNREC_TILED_EPI
    __syncthreads();
  }
  // finished: never hold the group back again
  if (threadIdx.x == 0 && meet_ticks > 0)
    __hip_atomic_fetch_add(ctr, 1u << 24, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#ifdef GNNREC_TILED_TRACE
extern "C" int gnnrec_debug_tiled_trace(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_tiled_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : -2;
}
#endif

// ---- host plan builder --------------------------------------------------------------------
namespace {

constexpr int kVirt = 2 * kTiledWaves;   // slot streams per block: (wave, half)

struct Run {
  int32_t p, row;   // panel, local row
  int64_t k;        // first edge (absolute index into col/val)
  int32_t n;        // edges of the row in this panel
};

struct BlockPlan {
  std::vector<uint32_t> slot[kTiledWaves];
  std::vector<float> val[kTiledWaves];
  std::vector<uint32_t> hdr[kTiledWaves];   // 4 words per chunk
  int32_t nsteps = 0;
};

struct TiledPlan {
  int64_t n_blocks = 0;
  std::vector<BlockPlan> blocks;
};

struct Slot {
  const Run* run;   // nullptr: padding
  int32_t t;        // edge of the run
};

// One stream's slots of a step cut into groups of kGroup (two groups = its half of a chunk):
// slots in ascending column sub-panel, rows in order inside one (a row's edges keep their
// column order); a row appears in a group only as ONE run of consecutive slots (the kernel
// reads a group's accumulators before it writes any) — a slot that would repeat a row
// non-adjacently is deferred, with the rest of that row, to a later group (per-row order
// kept). Padded to a multiple of kHalf.
void half_chunks(const std::vector<const Run*>& runs, const int32_t* col, int sub_panel,
                 std::vector<Slot>& seq) {
  std::vector<Slot> pending, deferred;
  std::vector<int> in_chunk, blocked;
  seq.clear();
  for (const Run* e : runs)
    for (int t = 0; t < e->n; ++t) pending.push_back({e, t});
  if (sub_panel > 0)
    std::stable_sort(pending.begin(), pending.end(), [&](const Slot& a, const Slot& c) {
      const int32_t ka = col[a.run->k + a.t] / sub_panel, kc = col[c.run->k + c.t] / sub_panel;
      return ka != kc ? ka < kc : a.run->row < c.run->row;
    });
  while (!pending.empty()) {
    deferred.clear();
    in_chunk.clear();
    blocked.clear();
    int n = 0, last = -1;
    const size_t start = seq.size();
    for (size_t q = 0; q < pending.size(); ++q) {
      const Slot& sl = pending[q];
      if (n == kGroup) {   // group full: the rest keeps its order for the next ones
        deferred.insert(deferred.end(), pending.begin() + q, pending.end());
        break;
      }
      const int r = sl.run->row;
      const bool is_blocked = std::find(blocked.begin(), blocked.end(), r) != blocked.end();
      const bool seen = std::find(in_chunk.begin(), in_chunk.end(), r) != in_chunk.end();
      if (is_blocked || (seen && r != last)) {
        if (seen && r != last && !is_blocked) blocked.push_back(r);
        deferred.push_back(sl);
        continue;
      }
      seq.push_back(sl);
      if (!seen) in_chunk.push_back(r);
      last = r;
      ++n;
    }
    while (seq.size() - start < (size_t)kGroup) seq.push_back({nullptr, 0});
    pending.swap(deferred);
  }
  while (seq.size() % kHalf) seq.push_back({nullptr, 0});
}

void build_block(const int64_t* rp, const int32_t* col, const float* val, int64_t n_rows,
                 int R, int panel, int sub_panel, int64_t b, BlockPlan& out) {
  const int64_t r0 = b * R, r1 = std::min<int64_t>(n_rows, r0 + R);
  std::vector<Run> runs;
  for (int64_t r = r0; r < r1; ++r) {
    int64_t k = rp[r];
    const int64_t e = rp[r + 1];
    while (k < e) {
      const int32_t p = col[k] / panel;
      int64_t j = k;
      while (j < e && col[j] / panel == p) ++j;
      runs.push_back({p, (int32_t)(r - r0), k, (int32_t)(j - k)});
      k = j;
    }
  }
  std::stable_sort(runs.begin(), runs.end(), [](const Run& a, const Run& c) { return a.p < c.p; });
  int32_t cur[kTiledWaves] = {};    // step of each wave's last emitted chunk
  int64_t load[kVirt];
  std::vector<const Run*> wl[kVirt];
  std::vector<const Run*> g;
  std::vector<Slot> hs[2];
  int32_t step = 0;
  size_t i = 0;
  while (i < runs.size()) {
    size_t j = i;
    while (j < runs.size() && runs[j].p == runs[i].p) ++j;
    // LPT over the (wave, half) streams: longest run first onto the least loaded
    g.clear();
    for (size_t q = i; q < j; ++q) g.push_back(&runs[q]);
    std::stable_sort(g.begin(), g.end(), [](const Run* a, const Run* c) { return a->n > c->n; });
    for (int v = 0; v < kVirt; ++v) {
      load[v] = 0;
      wl[v].clear();
    }
    for (const Run* e : g) {
      int v = 0;
      for (int q = 1; q < kVirt; ++q)
        if (load[q] < load[v]) v = q;
      load[v] += e->n;
      wl[v].push_back(e);
    }
    const uint32_t base = (uint32_t)runs[i].p * (uint32_t)panel;   // the step's first column
    for (int w = 0; w < kTiledWaves; ++w) {
      if (wl[2 * w].empty() && wl[2 * w + 1].empty()) continue;
      for (int h = 0; h < 2; ++h) half_chunks(wl[2 * w + h], col, sub_panel, hs[h]);
      const size_t n = std::max(hs[0].size(), hs[1].size());
      for (int h = 0; h < 2; ++h) hs[h].resize(n, Slot{nullptr, 0});
      uint32_t bar = (uint32_t)(step - cur[w]);
      for (size_t c = 0; c < n; c += kHalf) {
        // padding slots gather a line the chunk fetches anyway (its first real slot's)
        uint32_t x0 = 0;
        for (int q = 0; q < kTiledChunk; ++q) {
          const Slot& sl = hs[q / kHalf][c + q % kHalf];
          if (sl.run) {
            x0 = (uint32_t)col[sl.run->k + sl.t] - base;
            break;
          }
        }
        uint32_t cmask = 0;
        for (int h = 0; h < 2; ++h)
          for (int t = 0; t < kHalf; ++t) {
            const Slot& sl = hs[h][c + t];
            if (!sl.run) {
              out.slot[w].push_back(x0 << kRowBits | (uint32_t)R);
              out.val[w].push_back(0.f);
              continue;
            }
            const int64_t k = sl.run->k + sl.t;
            if (t > 0 && hs[h][c + t - 1].run == sl.run) cmask |= 1u << (16 * h + t);
            out.slot[w].push_back(((uint32_t)col[k] - base) << kRowBits | (uint32_t)sl.run->row);
            out.val[w].push_back(val[k]);
          }
        out.hdr[w].insert(out.hdr[w].end(), {bar, cmask, base, 0u});
        bar = 0;
      }
      cur[w] = step;
    }
    ++step;
    i = j;
  }
  out.nsteps = step;
}

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_tiled_plan_build(const int64_t* row_ptr, const int32_t* col,
                                       const float* val, int64_t n_rows, int32_t rows_per_block,
                                       int32_t panel, int32_t sub_panel, int32_t n_threads,
                                       void** plan, int64_t* n_chunks, int64_t* n_blocks) {
  GNNREC_REQUIRE(row_ptr && plan && n_chunks && n_blocks && n_rows >= 0, "tiled_plan: bad args");
  GNNREC_REQUIRE(rows_per_block >= 1 && rows_per_block <= GNNREC_TILED_MAX_ROWS,
                 "tiled_plan: rows_per_block must be in [1, %d]", GNNREC_TILED_MAX_ROWS);
  GNNREC_REQUIRE(panel >= 1 && sub_panel >= 0, "tiled_plan: bad panel / sub_panel");
  panel = std::min(panel, kMaxPanel);   // a slot word holds 20 bits of column offset
  const int64_t nnz = n_rows > 0 ? row_ptr[n_rows] - row_ptr[0] : 0;
  GNNREC_REQUIRE(nnz == 0 || (col && val), "tiled_plan: null col/val");
  auto* pl = new (std::nothrow) TiledPlan;
  GNNREC_REQUIRE(pl != nullptr, "tiled_plan: out of host memory");
  pl->n_blocks = (n_rows + rows_per_block - 1) / rows_per_block;
  pl->blocks.resize(pl->n_blocks);
  int t = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
  t = std::max(1, std::min<int>(t, (int)std::max<int64_t>(1, pl->n_blocks)));
  std::atomic<int64_t> next{0};
  std::atomic<bool> bad_col{false};
  auto worker = [&] {
    for (int64_t b; (b = next.fetch_add(1)) < pl->n_blocks;) {
      const int64_t r0 = b * rows_per_block, r1 = std::min<int64_t>(n_rows, r0 + rows_per_block);
      for (int64_t k = row_ptr[r0]; k < row_ptr[r1]; ++k)
        if (col[k] < 0) bad_col = true;
      if (bad_col) continue;
      build_block(row_ptr, col, val, n_rows, rows_per_block, panel, sub_panel, b, pl->blocks[b]);
    }
  };
  std::vector<std::thread> pool;
  for (int i = 1; i < t; ++i) pool.emplace_back(worker);
  worker();
  for (auto& th : pool) th.join();
  if (bad_col) {
    delete pl;
    set_error("tiled_plan: negative column index");
    return GNNREC_EINVAL;
  }
  int64_t tot = 0;
  for (const auto& bp : pl->blocks)
    for (int w = 0; w < kTiledWaves; ++w) tot += (int64_t)bp.hdr[w].size() / 4;
  *n_chunks = tot;
  *n_blocks = pl->n_blocks;
  *plan = pl;
  return GNNREC_OK;
}

extern "C" int gnnrec_tiled_plan_emit(void* plan, uint32_t* slot, float* val, uint32_t* hdr,
                                      int64_t* wave_ptr, int32_t* n_steps) {
  GNNREC_REQUIRE(plan && slot && val && hdr && wave_ptr && n_steps, "tiled_emit: null pointer");
  auto* pl = static_cast<TiledPlan*>(plan);
  const int64_t nb = pl->n_blocks;
  wave_ptr[0] = 0;
  for (int64_t b = 0; b < nb; ++b)
    for (int w = 0; w < kTiledWaves; ++w)
      wave_ptr[b * kTiledWaves + w + 1] =
          wave_ptr[b * kTiledWaves + w] + (int64_t)pl->blocks[b].hdr[w].size() / 4;
  for (int64_t b = 0; b < nb; ++b) {
    const BlockPlan& bp = pl->blocks[b];
    n_steps[b] = bp.nsteps;
    for (int w = 0; w < kTiledWaves; ++w) {
      const int64_t c = wave_ptr[b * kTiledWaves + w];
      std::copy(bp.slot[w].begin(), bp.slot[w].end(), slot + c * kTiledChunk);
      std::copy(bp.val[w].begin(), bp.val[w].end(), val + c * kTiledChunk);
      std::copy(bp.hdr[w].begin(), bp.hdr[w].end(), hdr + 4 * c);
    }
  }
  // tail chunks for the last prefetches: harmless slots (row 0 of x, row field all ones)
  const int64_t end = wave_ptr[nb * kTiledWaves];
  for (int64_t s = end * kTiledChunk; s < (end + kTiledTail) * kTiledChunk; ++s) {
    slot[s] = (uint32_t)kRowMask;
    val[s] = 0.f;
  }
  for (int64_t s = 4 * end; s < 4 * (end + kTiledTail); ++s) hdr[s] = 0;
  return GNNREC_OK;
}

extern "C" int gnnrec_tiled_plan_free(void* plan) {
  delete static_cast<TiledPlan*>(plan);
  return GNNREC_OK;
}

namespace {
// The kernel may take all 160 KB of LDS: the attribute is set once per device, and a failure
// is reported (not ignored) so the caller can fall back to the row-parallel hop.
int tiled_lds_attribute(int dev) {
  static std::mutex mu;
  static std::vector<int> done;   // 0 unset, 1 ok, -1 failed
  std::lock_guard<std::mutex> lock(mu);
  if ((int)done.size() <= dev) done.resize(dev + 1, 0);
  if (done[dev] == 0) {
    const hipError_t e = hipFuncSetAttribute((const void*)tiled_hop_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             160 * 1024);
    done[dev] = e == hipSuccess ? 1 : -1;
    if (e != hipSuccess) (void)hipGetLastError();
  }
  return done[dev];
}
}  // namespace

extern "C" int gnnrec_spmm_tiled_f32(const uint32_t* slot, const float* val,
                                     const uint32_t* hdr, const int64_t* wave_ptr,
                                     const int32_t* n_steps, int64_t n_blocks,
                                     int32_t rows_per_block, const float* x, int64_t x_rows,
                                     int64_t ldx, float* y, int64_t ldy, int64_t n_rows, int32_t d,
                                     int32_t epi, const float* self, int64_t ld_self, float* acc,
                                     int64_t ld_acc, float acc_div, uint32_t* sync,
                                     int32_t meet_us, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(d > 0 && d % kSlice == 0, "spmm_tiled: d must be a multiple of 32 (got %d)",
                 (int)d);
  GNNREC_REQUIRE(rows_per_block >= 1 && rows_per_block <= GNNREC_TILED_MAX_ROWS,
                 "spmm_tiled: bad rows_per_block");
  GNNREC_REQUIRE(n_rows >= 0 && n_blocks == (n_rows + rows_per_block - 1) / rows_per_block,
                 "spmm_tiled: n_blocks does not match n_rows / rows_per_block");
  GNNREC_REQUIRE(ldx >= d && x_rows >= 0 && ldx * 4 <= kMaxRowBytes,
                 "spmm_tiled: need d <= ldx <= %d", kMaxRowBytes / 4);
  GNNREC_REQUIRE((epi & GNNREC_EPI_NO_Y) || (y && ldy >= d), "spmm_tiled: null y or ldy < d");
  GNNREC_REQUIRE(!(epi & GNNREC_EPI_ACC_INIT) || (self && ld_self >= d),
                 "spmm_tiled: ACC_INIT needs self");
  GNNREC_REQUIRE(!(epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)) || (acc && ld_acc >= d),
                 "spmm_tiled: ACC needs acc");
  GNNREC_REQUIRE(!(epi & GNNREC_EPI_ACC_X) ||
                     ((epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)) && x_rows >= n_rows),
                 "spmm_tiled: ACC_X needs ACC_INIT or ACC_ADD and a square operand");
  GNNREC_REQUIRE(!(epi & GNNREC_EPI_ACC_DIV) || (epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)),
                 "spmm_tiled: ACC_DIV needs ACC_INIT or ACC_ADD");
  GNNREC_REQUIRE(meet_us >= 0 && meet_us <= 100000, "spmm_tiled: meet_us must be in [0, 1e5]");
  constexpr int64_t kMaxLd = ((int64_t)1 << 32) / (4 * 4096);   // epilogue row offsets: 32-bit
  GNNREC_REQUIRE(ldy <= kMaxLd && ld_self <= kMaxLd && ld_acc <= kMaxLd,
                 "spmm_tiled: output / self / acc row strides must be <= %lld",
                 (long long)kMaxLd);
  if (n_rows == 0) return GNNREC_OK;
  GNNREC_REQUIRE(slot && val && hdr && wave_ptr && n_steps && x && sync,
                 "spmm_tiled: null pointer");
  hipStream_t s = as_hip(stream);
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  const size_t lds = (size_t)(rows_per_block + 1) * kSlice * sizeof(float);
  if (lds > 64 * 1024 && tiled_lds_attribute(dev) < 0) {
    set_error("spmm_tiled: the device refused %zu bytes of dynamic LDS", lds);
    return GNNREC_EHIP;
  }
  const int64_t grid = std::min<int64_t>(cus, n_blocks);
  const int64_t nb_pad = ceil_div(n_blocks, grid) * grid;   // every slice starts a pass
  const int64_t n_items = (int64_t)(d / kSlice) * nb_pad;
  GNNREC_REQUIRE(n_items < INT32_MAX, "spmm_tiled: too many blocks");
  if (hipMemsetAsync(sync, 0, GNNREC_TILED_SYNC_WORDS * sizeof(uint32_t), s) != hipSuccess)
    return check_launch("spmm_tiled (sync reset)");
  hipLaunchKernelGGL(tiled_hop_kernel, dim3((unsigned)grid), dim3(kTiledWaves * 64), lds, s,
                     slot, val, hdr, wave_ptr, n_steps,
                     (int)n_blocks, (int)nb_pad, (int)n_items, (int)rows_per_block, x,
                     (uint64_t)(x_rows * ldx * 4), (uint32_t)(ldx * 4), y, ldy,
                     n_rows, epi, self, ld_self, acc, ld_acc, acc_div, sync,
                     (unsigned)meet_us * 100u /* wall_clock64 runs at 100 MHz */);
  return check_launch("spmm_tiled");
}
