// Column-ordered ("tiled") SpMM hop for any d % 32 == 0 (gnnrec_spmm_tiled_f32).
//
// Same arithmetic as spmm_vec_kernel — replaces torch.sparse.mm(adj, x) of the reference
// (baselines/lightgcn.py:88,178) with y[r] = fmaf chain over the row's neighbours in ascending
// column order from +0 — but a different schedule. The row-parallel hop gathers every
// neighbour row from beyond L2 (G100M: 16x the compulsory bytes). Here one persistent
// 512-thread workgroup per CU owns R destination rows per pass with fp32 accumulators in
// LDS, and its 8 waves walk the rows' edges PANEL BY PANEL in ascending source column
// (a step = one panel; a workgroup barrier between steps, so a row may move to another slot
// stream from one step to the next without reordering its chain). The workgroups of a
// blockIdx % 8 group (one XCD under round-robin placement — speed only, never correctness)
// meet at every pass start (bounded counter wait), so they sweep the same panels together and
// a gathered source row is reused from the XCD's L2 by the group's other rows.
//
// Feature slices: a pass computes ONE 32-feature slice of its block's rows (a gather = one
// 128-B line of a source row; the LDS row = 128 B), so an XCD group's pass covers 35.7K rows
// (G100M: 14 passes x 1117 rows x 2 slices). A d-wide hop is d/32 sweeps of the same plan; the
// work items are (slice, block) pairs, slice-major.
//
// Plan v3 (round 3): 16 bytes per lane. A wave runs EIGHT slot streams, one per 8-lane group
// (lane = 8 g + q; lane q of group g owns features 4q .. 4q+3 of the slice), so one gather
// instruction fetches eight 128-B lines with one buffer_load_dwordx4 per lane and one LDS
// accumulator update is one ds_read_b128 / 4 fmaf / ds_write_b128 per lane. The per-CU L2->CU
// rate of random 128-B lines is 2.2x higher in this form than with one dword per lane and two
// lines per instruction (tools/gather_probe2.hip: 117 vs 53 GB/s per CU from L2;
// profiles/r03/gather_probe2.jsonl) — the round-2 kernel's floor. A chunk is 8 steps x 8
// streams = 64 slots, one per lane (lane 8 g + t holds slot t of stream g); step t hands slot
// t of every stream to its group with two DPP row_newbcast moves under bank masks (lanes 0-7
// of a 16-lane row read row lane t, lanes 8-15 read row lane 8 + t). The chunk header
// {step barriers, chain mask lo, hi, panel base} comes back by v_readlane: bit 8 g + t of the
// 64-bit chain mask = slot t of stream g continues slot t-1's row (take the register value);
// SALU spreads the step's bits to lane masks. A chunk is applied as two groups of 4 steps
// (reads of a group precede its writes; a row is at most one run of slots per group and
// stream). Pipeline per wave: chunk c+5's slot loads, chunk c+2's 8 gathers and chunk c's LDS
// chain in flight (plan ring kPlanAhead = 5, gather ring kGatherAhead = 2).
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
constexpr int kGroups = GNNREC_TILED_GROUPS;      // slot streams per wave (8 lanes each)
constexpr int kSteps = GNNREC_TILED_STEPS;        // steps per chunk
constexpr int kTiledChunk = GNNREC_TILED_CHUNK;   // slots per chunk (one per lane)
constexpr int kTiledTail = GNNREC_TILED_TAIL;
constexpr int kSlice = 32;                        // features per gathered line
constexpr int kRowBytes = kSlice * 4;             // one gathered line
#ifndef GNNREC_TILED_SPW
#define GNNREC_TILED_SPW 1
#endif
// Slices per plan walk (experiment builds, DESIGN.md §3.1c "one plan walk"): SPW = 2 walks the
// plan once for two adjacent 32-feature slices — every slot gathers two 128-B lines and the
// LDS accumulator rows are 256 B, so a block holds half the rows.
constexpr int kSPW = GNNREC_TILED_SPW;
constexpr int kAccBytes = kRowBytes * kSPW;       // one LDS accumulator row
static_assert(kSPW == 1 || kSPW == 2, "1 or 2 slices per plan walk");
constexpr int kRowBits = 11;
constexpr int kRowMask = (1 << kRowBits) - 1;
constexpr int kMaxPanel = 1 << 20;                // columns per panel (slot word: 21 bits)
constexpr int kMaxRowBytes = GNNREC_TILED_MAX_LDX * 4;   // keeps the lane offset 32-bit
#ifndef GNNREC_TILED_NOCHAIN
#define GNNREC_TILED_NOCHAIN 0
#endif
// NOCHAIN: a row appears at most once per chunk of a stream, so all 8 reads of a chunk precede
// its writes and no slot chains on a register value
constexpr bool kNoChain = GNNREC_TILED_NOCHAIN != 0;
#ifndef GNNREC_TILED_APPLY
#define GNNREC_TILED_APPLY 4
#endif
constexpr int kApply = GNNREC_TILED_APPLY;        // steps whose reads precede their writes
#ifndef GNNREC_TILED_PLAN_AHEAD
#define GNNREC_TILED_PLAN_AHEAD 5
#endif
#ifndef GNNREC_TILED_GATHER_AHEAD
#define GNNREC_TILED_GATHER_AHEAD 2
#endif
constexpr int kPlanAhead = GNNREC_TILED_PLAN_AHEAD;       // slot loads, chunks ahead of the apply
constexpr int kGatherAhead = GNNREC_TILED_GATHER_AHEAD;   // gathers, chunks ahead of the apply
constexpr int kMRing = kPlanAhead + 1;
constexpr int kXRing = kGatherAhead + 1;
constexpr int ring_gcd(int a, int b) { return b ? ring_gcd(b, a % b) : a; }
constexpr int kRingUnroll = kMRing / ring_gcd(kMRing, kXRing) * kXRing;
static_assert(kPlanAhead > kGatherAhead && kGatherAhead >= 1, "pipeline order");
static_assert(kPlanAhead <= GNNREC_TILED_TAIL, "tail chunks cover the last prefetches");
#ifndef GNNREC_TILED_EPI_BATCH
#define GNNREC_TILED_EPI_BATCH 5
#endif
constexpr int kEpiBatch = GNNREC_TILED_EPI_BATCH;   // epilogue rows per group, loads in flight
#ifndef GNNREC_TILED_EPI_BATCH3
#define GNNREC_TILED_EPI_BATCH3 3
#endif
constexpr int kEpiBatch3 = GNNREC_TILED_EPI_BATCH3;   // the same with 2-3 base inputs per row
#ifndef GNNREC_TILED_EPI_PRELOAD
#define GNNREC_TILED_EPI_PRELOAD 1   // the first batch's base rows loaded before the pass-end barriers
#endif
// epilogue stores non-temporal (aux bit 1, nt): the rows are read again only by the next
// launch (round 2: 12.62 -> 12.56 ms per step, profiles/r02/exp_epi_store_policy.jsonl)
constexpr int kEpiStoreAux = 2;
static_assert(kTiledChunk == kGroups * kSteps && kTiledChunk == 64, "one slot per lane");
static_assert(kGroups == 8 && kSteps == 8, "a stream is 8 lanes: half a 16-lane DPP row");
static_assert(kSteps == 2 * kApply || kSteps == kApply, "a chunk is one or two apply groups");
static_assert(GNNREC_TILED_MAX_ROWS < kRowMask, "row field is 11 bits (row R = scratch)");
static_assert(kSPW > 1 || (GNNREC_TILED_MAX_ROWS + 1) * kRowBytes <= 160 * 1024, "LDS");
static_assert((int64_t)kMaxPanel * kMaxRowBytes <= ((int64_t)1 << 32), "32-bit lane offsets");

typedef float f4 __attribute__((ext_vector_type(4)));

// Diagnostic builds only (tools/build_variant.sh, results wrong): bit 0 skips the LDS
// accumulator reads and writes (registers instead), bit 1 replaces the gathers by a constant,
// bit 2 skips the step barriers, bit 3 reads every chunk's slot words and values from the
// plan's first 64 chunks (cache-resident plan stream; headers unchanged), bit 4 replaces the
// DPP broadcasts by the lane's own value, bit 5 skips the main loop (passes and epilogues),
// bit 6 drops a factored plan's class load (every slot class 0: the cost of one plan-load
// instruction per chunk).
#ifndef GNNREC_TILED_EXP
#define GNNREC_TILED_EXP 0
#endif

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

struct TiledSlots {   // this lane's slot of the chunk: stream lane / 8, step lane % 8
  uint32_t w;         // slot word: (column - panel base) << kRowBits | local row
  float v;            // the slot's value (a factored plan: formed at the gather stage)
  uint32_t h;         // word (lane % 4) of the chunk header (quad layout: lane % 16 of the quad's)
  uint32_t c;         // a factored plan: the slot's column class
  int hl = 0;         // quad layout: the chunk's first header lane (4 k)
};

#ifndef GNNREC_TILED_QUAD
#define GNNREC_TILED_QUAD 1
#endif
// Quad plan layout (ABI 9, DESIGN.md §3.1c "plan-load instructions"): the plan streams are
// interleaved per 4 chunks — lane l's slot words of chunks 4q .. 4q+3 are one 16-B load, their
// class bytes one dword (values one 16-B load), the 4 chunk headers one dword per lane
// (lane % 16) — so a wave issues 3 plan loads per 4 chunks instead of 12 (G100M hop 3.54 ->
// 3.41 ms, profiles/r04/ab_quad_plan.jsonl). Every wave's chunk range starts on a quad: the
// layout step (gnnrec_tiled_plan_quad_layout) pads ranges to multiples of 4 with empty chunks.
// GNNREC_TILED_QUAD=0 builds read the planners' chunk-major arrays directly.
constexpr bool kQuad = GNNREC_TILED_QUAD != 0;
struct TiledQuad {
  uint4 w;
  uint32_t c;   // factored: 4 class bytes (byte k: chunk 4q + k)
  float4 v;     // explicit values
  uint32_t h;   // header word lane % 16 of the quad (chunk k: lanes 4k .. 4k+3)
};

// Factored plans (ABI 8, DESIGN.md §3.1c "plan values"): every value of the operand is
// fl(row_factor[r] * class_table[k]) for its column's class k (the symmetric normalisation:
// fl(dis_r * dis_c), graph_builder.py:119-126), so a slot carries a 1-byte class instead of
// its 4-byte value. The block's row factors and the class table sit in LDS after the
// accumulator rows; the value is formed once per chunk per lane — the same fp32 product the
// operand's builder stored, so the same bits.
constexpr int kMaxClasses = GNNREC_TILED_MAX_CLASSES;
static_assert(kSPW > 1 || GNNREC_TILED_MAX_ROWS_FACTORED * (kRowBytes + 4) + kRowBytes + 4 +
                      kMaxClasses * 4 <= 160 * 1024, "LDS of a factored plan");

// Slot t of every stream to the stream's 8 lanes: within a 16-lane DPP row, lanes 0-7 (stream
// 2k) take row lane t, lanes 8-15 (stream 2k+1) row lane 8 + t.
template <int T>
__device__ __forceinline__ uint32_t gbcast(uint32_t v) {
  if (GNNREC_TILED_EXP & 16) return v ^ (T << 4);
  // lanes 8-15 of the first move are left undefined: the second writes them
  const int a = __builtin_amdgcn_mov_dpp((int)v, 0x150 + T, 0xF, 0x3, false);
  return (uint32_t)__builtin_amdgcn_update_dpp(a, (int)v, 0x158 + T, 0xF, 0xC, false);
}
template <int T>
__device__ __forceinline__ float gbcastf(float v) {
  return __builtin_bit_cast(float, gbcast<T>(__builtin_bit_cast(uint32_t, v)));
}

// The chunk header {step barriers before the chunk, chain mask lo, chain mask hi, panel base
// column} is loaded with the slots as a vector load (lane l: word l % 4) and read back with
// v_readlane: a scalar load would share lgkmcnt with the LDS chain and stall it.
// chunk c of the plan: this lane's slot word and value, and header word lane % 4 (three
// coalesced vector loads; same-box A/B: separate 128-B-aligned arrays beat one interleaved
// 528-B chunk stream by 4 %, profiles/r03/ab_interleaved_plan_vs_separate_fixed_range.txt)
template <bool FACT>
__device__ __forceinline__ void tiled_slots(const uint32_t* __restrict__ ss,
                                            const float* __restrict__ sv,
                                            const uint8_t* __restrict__ sc,
                                            const uint32_t* __restrict__ hdr, int64_t c, int lane,
                                            TiledSlots& m) {
  if (GNNREC_TILED_EXP & 8) c &= 63;
  const int64_t i = c * kTiledChunk + lane;
  m.w = ss[i];   // default policy: nt plan loads measured 1 % slower (exp_plan_nt.jsonl)
  if constexpr (FACT)
    m.c = (GNNREC_TILED_EXP & 64) ? 0u : sc[i];
  else
    m.v = sv[i];
  m.h = hdr[4 * c + (lane & 3)];
}

// a factored plan's slot value (rows past the block's, e.g. of prefetched chunks beyond the
// wave's range, read the scratch row's 0 factor)
template <bool FACT>
__device__ __forceinline__ void slot_value(TiledSlots& m, const float* rfl, const float* ctl,
                                           uint32_t R) {
  if constexpr (FACT) m.v = __fmul_rn(rfl[min(m.w & kRowMask, R)], ctl[m.c]);
}

template <int W>
__device__ __forceinline__ uint32_t hdr_word(const TiledSlots& m) {
  return (uint32_t)__builtin_amdgcn_readlane((int)m.h, W + m.hl);
}

template <bool FACT>
__device__ __forceinline__ void tiled_quad(const uint32_t* __restrict__ ss,
                                           const float* __restrict__ sv,
                                           const uint8_t* __restrict__ sc,
                                           const uint32_t* __restrict__ hdr, int64_t q, int lane,
                                           TiledQuad& Q) {
  const int64_t i = q * kTiledChunk + lane;
  Q.w = reinterpret_cast<const uint4*>(ss)[i];
  if constexpr (FACT)
    Q.c = reinterpret_cast<const uint32_t*>(sc)[i];
  else
    Q.v = reinterpret_cast<const float4*>(sv)[i];
  Q.h = hdr[16 * q + (lane & 15)];
}

template <int K, bool FACT>
__device__ __forceinline__ TiledSlots quad_chunk(const TiledQuad& Q) {
  TiledSlots m;
  m.w = K == 0 ? Q.w.x : K == 1 ? Q.w.y : K == 2 ? Q.w.z : Q.w.w;
  if constexpr (FACT)
    m.c = (Q.c >> (8 * K)) & 255u;
  else
    m.v = K == 0 ? Q.v.x : K == 1 ? Q.v.y : K == 2 ? Q.v.z : Q.v.w;
  m.h = Q.h;
  m.hl = 4 * K;
  return m;
}

// The gathers of a chunk read through a buffer whose base is its panel's first source row, so
// lane offsets stay 32-bit for any table size; its range ends at the table's last byte. (A
// form in 32-bit row units was 5 % slower on the G100M hop: profiles/r03/bisect.jsonl.)
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
  const float* b = p ? p + r0 * ld + (int64_t)slice * kSlice * kSPW : p;
  const uint32_t n = p ? (uint32_t)(rows - 1) * (uint32_t)ld * 4u + kAccBytes : 0u;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(b), 0, (int)n, 0x00020000);
}

__device__ __forceinline__ f4 load4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
#ifndef GNNREC_TILED_EPI_LOAD_AUX
#define GNNREC_TILED_EPI_LOAD_AUX 2   // nt: hop 3 3.92 -> 3.87 ms (profiles/r03/exp_epi_load_policy.jsonl)
#endif
// the epilogue's base rows, read once per hop: non-temporal (aux 2), so they do not evict the
// gathered lines the next pass reuses from L2
__device__ __forceinline__ f4 load4_base(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0,
                                                                      GNNREC_TILED_EPI_LOAD_AUX));
}
__device__ __forceinline__ void store4(f4 v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b128(
      __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), r, off, 0,
      kEpiStoreAux);
}

template <int... T>
__device__ __forceinline__ void tiled_gather(std::integer_sequence<int, T...>,
                                             __amdgpu_buffer_rsrc_t xr, uint32_t q16,
                                             uint32_t row_bytes, const TiledSlots& m,
                                             f4 (&x)[kSteps][kSPW]) {
  const uint32_t o = __umul24(m.w >> kRowBits, row_bytes);   // this lane's slot's source row
  if constexpr (GNNREC_TILED_EXP & 2) {
    ((x[T][0] = f4{__builtin_bit_cast(float, gbcast<T>(o)), 1.f, 1.f, 1.f}), ...);
    if constexpr (kSPW > 1) ((x[T][kSPW - 1] = x[T][0]), ...);
  } else if constexpr (kSPW == 1) {
    ((x[T][0] = load4(xr, gbcast<T>(o) + q16)), ...);
  } else {
    uint32_t ot[sizeof...(T)];
    ((ot[T] = gbcast<T>(o) + q16), ...);
    ((x[T][0] = load4(xr, ot[T]), x[T][1] = load4(xr, ot[T] + kRowBytes)), ...);
  }
}

// lane-wise select on a wave-uniform 64-bit lane mask held in SGPRs (no compare per lane)
__device__ __forceinline__ float select_lanes(float if0, float if1, uint64_t mask) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if0), "v"(if1), "s"(mask));
  return r;
}
__device__ __forceinline__ f4 select4(f4 if0, f4 if1, uint64_t mask) {
  f4 r;
  r.x = select_lanes(if0.x, if1.x, mask);
  r.y = select_lanes(if0.y, if1.y, mask);
  r.z = select_lanes(if0.z, if1.z, mask);
  r.w = select_lanes(if0.w, if1.w, mask);
  return r;
}

// lanes of the streams whose slot T continues slot T-1's row: bit 8 g + T of cm -> byte g
template <int T>
__device__ __forceinline__ uint64_t chain_lanes(uint64_t cm) {
  uint64_t m = (cm >> T) & 0x0101010101010101ull;
  m |= m << 1;
  m |= m << 2;
  m |= m << 4;
  return m;
}

__device__ __forceinline__ f4 fma4(float v, f4 x, f4 a) {
  f4 r;
  r.x = __builtin_fmaf(v, x.x, a.x);
  r.y = __builtin_fmaf(v, x.y, a.y);
  r.z = __builtin_fmaf(v, x.z, a.z);
  r.w = __builtin_fmaf(v, x.w, a.w);
  return r;
}

// Steps G .. G+3 of a chunk: 4 accumulator reads, 4 chained fmaf, 4 writes (per lane: 16 B
// of a row each). A chunk is applied as two such groups, so a row may appear in both groups
// of a stream: the second group's reads follow the first group's writes in the wave's LDS
// order (and a slot at step 4 chaining on step 3 selects the value step 3 just wrote).
template <bool CHAIN, int G, int S, int... T>
__device__ __forceinline__ void tiled_apply4(std::integer_sequence<int, T...>, char* base,
                                             uint32_t q16, uint32_t r, const TiledSlots& m,
                                             const f4 (&x)[kSteps][kSPW], uint64_t cm, f4& prev) {
  uint32_t a[sizeof...(T)];
  ((a[T] = gbcast<G + T>(r) + q16 + S * kRowBytes), ...);
  f4 av[sizeof...(T)];
  if constexpr (GNNREC_TILED_EXP & 1)
    ((av[T] = f4{__builtin_bit_cast(float, a[T]), 0.f, 0.f, 0.f}), ...);
  else
    ((av[T] = *reinterpret_cast<const f4*>(base + a[T])), ...);
  if constexpr (CHAIN) {
    // slot t continuing slot t-1's row (same stream) chains on its register value
    ((av[T] = fma4(gbcastf<G + T>(m.v), x[G + T][S],
                   G + T > 0 ? select4(av[T], T > 0 ? av[T > 0 ? T - 1 : 0] : prev,
                                       chain_lanes<G + T>(cm))
                             : av[T])),
     ...);
  } else {
    ((av[T] = fma4(gbcastf<G + T>(m.v), x[G + T][S], av[T])), ...);
  }
  if constexpr (GNNREC_TILED_EXP & 1)
    prev = prev + ((av[T]) + ...);
  else
    ((*reinterpret_cast<f4*>(base + a[T]) = av[T]), ...);
  prev = (GNNREC_TILED_EXP & 1) ? prev : av[sizeof...(T) - 1];
}

template <bool CHAIN>
__device__ __forceinline__ void tiled_apply(float* acc, uint32_t q16, const TiledSlots& m,
                                            const f4 (&x)[kSteps][kSPW], uint64_t cm, f4& sink) {
  constexpr auto k4 = std::make_integer_sequence<int, kApply>{};
  char* base = reinterpret_cast<char*>(acc);
  const uint32_t r = (m.w & kRowMask) * kAccBytes;   // this lane's slot's accumulator row
  // the slices of a walk are independent chains over the same slots
  {
    f4 prev = (GNNREC_TILED_EXP & 1) ? sink : f4{0.f, 0.f, 0.f, 0.f};
    tiled_apply4<CHAIN, 0, 0>(k4, base, q16, r, m, x, cm, prev);
    if constexpr (kApply < kSteps) tiled_apply4<CHAIN, kApply, 0>(k4, base, q16, r, m, x, cm, prev);
    if (GNNREC_TILED_EXP & 1) sink = prev;
  }
  if constexpr (kSPW > 1) {
    f4 prev = {0.f, 0.f, 0.f, 0.f};
    tiled_apply4<CHAIN, 0, 1>(k4, base, q16, r, m, x, cm, prev);
    if constexpr (kApply < kSteps) tiled_apply4<CHAIN, kApply, 1>(k4, base, q16, r, m, x, cm, prev);
  }
}

// Pass-end epilogue of one 8-lane group: its rows i = rl + 128 j of the block (rl = 8 * wave
// + group), B at a time with every load of a batch issued before the first use; lane q moves
// 16 B of each row. All offsets are 32-bit rows of buffers based at the block's first row
// whose ranges end at the last valid row: loads past it return 0 and stores are dropped, so
// there is no branch (a branch around a load makes the compiler wait for it in place). A null
// ry: no y output.
// NB base inputs (the layer-mean terms before this hop, in layer order): acc_out =
// (((b0 [+ b1]) [+ b2]) + y) [/ div] — b0 = x0 (ACC_INIT) or the running sum (ACC_ADD);
// INIT|ADD: b0 = x0, b1 = the acc rows (an earlier layer parked there); ACC_X: the hop's
// input row (the previous layer) last. NB = 0: y only.
template <int NB, int B, class Wait>
__device__ __forceinline__ void tiled_epilogue(const float* acc, int R, int rl, uint32_t q16,
                                               __amdgpu_buffer_rsrc_t ry, uint32_t ly,
                                               __amdgpu_buffer_rsrc_t rb0, uint32_t lb0,
                                               __amdgpu_buffer_rsrc_t rb1, uint32_t lb1,
                                               __amdgpu_buffer_rsrc_t rb2, uint32_t lb2,
                                               __amdgpu_buffer_rsrc_t ra, uint32_t la,
                                               bool div, float acc_div, Wait wait) {
  constexpr int kStride = kGroups * kTiledWaves;
  const __amdgpu_buffer_rsrc_t rb[3] = {rb0, rb1, rb2};
  const uint32_t lb[3] = {lb0, lb1, lb2};
  f4 base[NB > 0 ? NB : 1][B][kSPW];
  // the base rows of batch i0 (global, independent of the pass: the first batch is loaded
  // before the pass-end barriers, so its latency hides behind the block's slowest wave)
  auto load_base = [&](int i0) {
    // per-row offsets advance by a stride; the opaque copy keeps the compiler from hoisting
    // B x 3 of them out of the persistent loop (they would spill)
    uint32_t ob[3];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      ob[j] = (uint32_t)i0 * lb[j] + q16;
      asm volatile("" : "+v"(ob[j]));
    }
#pragma unroll
    for (int q = 0; q < B; ++q)
#pragma unroll
      for (int j = 0; j < NB; ++j) {
#pragma unroll
        for (int sl = 0; sl < kSPW; ++sl) base[j][q][sl] = load4_base(rb[j], ob[j] + sl * kRowBytes);
        ob[j] += kStride * lb[j];
      }
  };
  int i0 = rl;
  if (GNNREC_TILED_EPI_PRELOAD) load_base(i0);
  wait();
  // the first batch runs even when rl is past the block's rows: its LDS reads stay inside
  // (row R is the scratch row) and its stores fall outside the buffer ranges
  const char* lds = reinterpret_cast<const char*>(acc);
  for (;;) {
    if (!GNNREC_TILED_EPI_PRELOAD) load_base(i0);
    uint32_t ol = (uint32_t)i0;
    asm volatile("" : "+v"(ol));
    f4 a[B][kSPW];
#pragma unroll
    for (int q = 0; q < B; ++q) {
#pragma unroll
      for (int sl = 0; sl < kSPW; ++sl)
        a[q][sl] = *reinterpret_cast<const f4*>(lds + min(ol, (uint32_t)R) * kAccBytes +
                                                sl * kRowBytes + q16);
      ol += kStride;
    }
    uint32_t oy = (uint32_t)i0 * ly + q16, oa = (uint32_t)i0 * la + q16;
    asm volatile("" : "+v"(oy), "+v"(oa));
#pragma unroll
    for (int q = 0; q < B; ++q) {
#pragma unroll
      for (int sl = 0; sl < kSPW; ++sl) {
        store4(a[q][sl], ry, oy + sl * kRowBytes);
        if (NB > 0) {
          f4 bsum = base[0][q][sl];
#pragma unroll
          for (int j = 1; j < NB; ++j) bsum = bsum + base[j][q][sl];
          bsum = bsum + a[q][sl];
          if (div) bsum = bsum / acc_div;
          store4(bsum, ra, oa + sl * kRowBytes);
        }
      }
      oy += kStride * ly;
      if (NB > 0) oa += kStride * la;
    }
    i0 += kStride * B;
    if (i0 - (rl & (kGroups - 1)) >= R) break;   // wave-uniform: the wave's first row
    if (GNNREC_TILED_EPI_PRELOAD) load_base(i0);
  }
}

template <class F, int... J>
__device__ __forceinline__ void for_seq(std::integer_sequence<int, J...>, F&& f) {
  (f(std::integral_constant<int, J>{}), ...);
}

// the main loop unrolled over one turn of the pipeline rings (compile-time ring indices)
template <class F, int... I>
__device__ __forceinline__ void run_ring(std::integer_sequence<int, I...>, F&& stage) {
  for (;;)
    if ((stage(std::integral_constant<int, I>{}) || ...)) break;
}

template <bool FACT>
__global__ __launch_bounds__(kTiledWaves * 64) void tiled_hop_kernel(
    const uint32_t* __restrict__ ss, const float* __restrict__ sv,
    const uint8_t* __restrict__ sc, const float* __restrict__ rowf,
    const float* __restrict__ ctab, int n_classes, const uint32_t* __restrict__ hdr, const int64_t* __restrict__ wptr,
    const int32_t* __restrict__ nsteps, int n_blocks, int nb_pad, int n_items, int R,
    const float* __restrict__ x, uint32_t x_rows32, uint32_t row_bytes,
    float* __restrict__ y, uint32_t ldy4, int n_rows, int epi, const float* __restrict__ self,
    uint32_t ls4, float* __restrict__ accg, uint32_t la4, float acc_div,
    const float* __restrict__ prev, uint32_t lp4, unsigned* __restrict__ sync,
    unsigned meet_ticks) {
  extern __shared__ f4 acc4[];   // [(R+1)][32] floats: row R is the padding slots' scratch row
  float* acc = reinterpret_cast<float*>(acc4);
  // factored plans: the block's row factors [R+1] (row R: 0) and the class table [kMaxClasses]
  float* rfl = acc + (R + 1) * kSlice * kSPW;
  float* ctl = rfl + (R + 1);
  if constexpr (FACT)
    for (int i = threadIdx.x; i < kMaxClasses; i += kTiledWaves * 64)
      ctl[i] = i < n_classes ? ctab[i] : 0.f;   // read after the first pass-start barrier
  constexpr auto kSeq = std::make_integer_sequence<int, kSteps>{};
  const int lane = threadIdx.x & 63;
  const uint32_t q16 = (uint32_t)(lane & 7) * 16;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  unsigned* ctr = sync + (blockIdx.x % 8) * 32;   // the group's counter, own 128-B line
  const int G = gridDim.x / 8 + ((blockIdx.x % 8) < (gridDim.x % 8) ? 1 : 0);
  int pass = 0;
#ifdef GNNREC_TILED_TRACE
  int ev = 0;
#endif
  for (int item = blockIdx.x; item < n_items; item += gridDim.x, ++pass) {
    if (threadIdx.x == 0 && pass > 0 && meet_ticks > 0) {
      // pass start: report the finished pass, wait (bounded) for the group's others
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long t0 = wall_clock64();
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                 (unsigned)(G * pass) &&
             wall_clock64() - t0 < meet_ticks)
        __builtin_amdgcn_s_sleep(2);
    }
    const int slice = item / nb_pad, blk = item - slice * nb_pad;
    if (blk >= n_blocks) continue;   // padding item (uniform over the workgroup)
    {
      const f4 z = {0.f, 0.f, 0.f, 0.f};
      for (int i = threadIdx.x; i < (R + 1) * (kSlice * kSPW / 4); i += kTiledWaves * 64) acc4[i] = z;
      if constexpr (FACT) {
        const int r0 = blk * R;
        for (int i = threadIdx.x; i <= R; i += kTiledWaves * 64)
          rfl[i] = (i < R && r0 + i < n_rows) ? rowf[r0 + i] : 0.f;
      }
    }
    __syncthreads();
    GNNREC_TILED_STAMP(ev);
    const uint32_t soff = (uint32_t)slice * kAccBytes;
    const char* xs = reinterpret_cast<const char*>(x) + soff;
    const uint64_t xs_bytes = (uint64_t)x_rows32 * row_bytes - soff;
    const int64_t s = (int64_t)blk * kTiledWaves + w;
    const int64_t b = wptr[s], e = (GNNREC_TILED_EXP & 32) ? b : wptr[s + 1];
    int cur = 0;
    f4 sink = {0.f, 0.f, 0.f, 0.f};   // diagnostic builds only (GNNREC_TILED_EXP & 1)
    if (kQuad && b < e && (b & 3)) {
      // a chunk-major plan passed to a quad build: the quads would straddle waves' ranges.
      // Flag it (the caller checks GNNREC_TILED_SYNC_ERR_WORD after the launch) and skip the
      // chunks; the block's epilogue still stores, so the launch's rows are undefined.
      if (lane == 0)
        __hip_atomic_fetch_or(sync + GNNREC_TILED_SYNC_ERR_WORD, 1u, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
    } else if (kQuad && b < e) {
      // quad layout: a ring of 3 quads (12 chunks) and kGatherAhead + 1 gathered chunks; stage
      // c (c % 4 == 0) loads quad c / 4 + 2, every stage gathers chunk c + kGatherAhead and
      // applies chunk c (wave ranges start on a quad, so c % 4 is the unrolled stage's)
      TiledQuad QR[3];
      f4 X[kXRing][kSteps][kSPW];
      float V[kXRing];
      const int nc = (int)(e - b);
      const int64_t q0 = b / 4;
      int c = 0;
      tiled_quad<FACT>(ss, sv, sc, hdr, q0, lane, QR[0]);
      tiled_quad<FACT>(ss, sv, sc, hdr, q0 + 1, lane, QR[1]);
      auto gather_j = [&](auto jc) {
        constexpr int J = decltype(jc)::value;
        TiledSlots mg = quad_chunk<J % 4, FACT>(QR[(J / 4) % 3]);
        tiled_gather(kSeq, chunk_rsrc(xs, xs_bytes, hdr_word<3>(mg), row_bytes), q16,
                     row_bytes, mg, X[J % kXRing]);
        slot_value<FACT>(mg, rfl, ctl, (uint32_t)R);
        V[J % kXRing] = mg.v;
      };
      for_seq(std::make_integer_sequence<int, kGatherAhead>{}, gather_j);
      auto stage = [&](auto ic) -> bool {
        constexpr int I = decltype(ic)::value;
        if constexpr (I % 4 == 0)
          tiled_quad<FACT>(ss, sv, sc, hdr, q0 + c / 4 + 2, lane, QR[(I / 4 + 2) % 3]);
        gather_j(std::integral_constant<int, I + kGatherAhead>{});
        TiledSlots ma = quad_chunk<I % 4, FACT>(QR[(I / 4) % 3]);
        ma.v = V[I % kXRing];
        const int bar = (int)hdr_word<0>(ma);
        for (int i = 0; i < bar; ++i) {
          if (!(GNNREC_TILED_EXP & 4)) __syncthreads();
          GNNREC_TILED_STAMP(ev);
        }
        cur += bar;
        const uint64_t cm =
            kNoChain ? 0 : (uint64_t)hdr_word<1>(ma) | ((uint64_t)hdr_word<2>(ma) << 32);
        if (!kNoChain && cm)
          tiled_apply<true>(acc, q16, ma, X[I % kXRing], cm, sink);
        else
          tiled_apply<false>(acc, q16, ma, X[I % kXRing], 0, sink);
        return ++c >= nc;
      };
      static_assert(12 % kXRing == 0, "quad ring: 12 stages cover the gather ring");
      // stage 4k loads quad k + 2, so at stage I the ring holds the chunks up to
      // 4 (I / 4) + 11: the chunk I + kGatherAhead it gathers is loaded for kGatherAhead <= 8
      static_assert(kGatherAhead <= 8, "quad ring: gathers at most 8 chunks ahead");
      run_ring(std::make_integer_sequence<int, 12>{}, stage);
    } else if (b < e) {
      // a ring of kPlanAhead + 1 slot sets and kGatherAhead + 1 gathered chunks: stage c loads
      // chunk c + kPlanAhead's slots, gathers chunk c + kGatherAhead and applies chunk c
      TiledSlots M[kMRing];
      f4 X[kXRing][kSteps][kSPW];
      const int nc = (int)(e - b);   // this wave's chunks of the pass
      int c = 0;
#pragma unroll
      for (int j = 0; j < kPlanAhead; ++j) tiled_slots<FACT>(ss, sv, sc, hdr, b + c + j, lane, M[j]);
#pragma unroll
      for (int j = 0; j < kGatherAhead; ++j) {
        tiled_gather(kSeq, chunk_rsrc(xs, xs_bytes, hdr_word<3>(M[j]), row_bytes), q16,
                     row_bytes, M[j], X[j]);
        slot_value<FACT>(M[j], rfl, ctl, (uint32_t)R);
      }
      auto stage = [&](auto ic) -> bool {
        constexpr int I = decltype(ic)::value;
        tiled_slots<FACT>(ss, sv, sc, hdr, b + c + kPlanAhead, lane, M[(I + kPlanAhead) % kMRing]);
        {
          TiledSlots& mg = M[(I + kGatherAhead) % kMRing];
          tiled_gather(kSeq, chunk_rsrc(xs, xs_bytes, hdr_word<3>(mg), row_bytes), q16,
                       row_bytes, mg, X[(I + kGatherAhead) % kXRing]);
          slot_value<FACT>(mg, rfl, ctl, (uint32_t)R);
        }
        const TiledSlots& ma = M[I % kMRing];
        const int bar = (int)hdr_word<0>(ma);
        for (int i = 0; i < bar; ++i) {
          if (!(GNNREC_TILED_EXP & 4)) __syncthreads();
          GNNREC_TILED_STAMP(ev);
        }
        cur += bar;
        const uint64_t cm =
            kNoChain ? 0 : (uint64_t)hdr_word<1>(ma) | ((uint64_t)hdr_word<2>(ma) << 32);
        if (!kNoChain && cm)
          tiled_apply<true>(acc, q16, ma, X[I % kXRing], cm, sink);
        else
          tiled_apply<false>(acc, q16, ma, X[I % kXRing], 0, sink);
        return ++c >= nc;
      };
      run_ring(std::make_integer_sequence<int, kRingUnroll>{}, stage);
    }
    if (GNNREC_TILED_EXP & 1) *reinterpret_cast<f4*>(reinterpret_cast<char*>(acc) + R * kAccBytes + q16) = sink;
    const int ns = nsteps[blk];
    auto wait = [&]() {
      for (int i = cur; i < ns; ++i) {  // this wave's remaining steps + the last
        __syncthreads();
        GNNREC_TILED_STAMP(ev);
      }
    };
    // epilogue: group g of wave w owns rows i = 8w + g + 128j (see tiled_epilogue)
    const int r0 = blk * R;
    const int nv = min(R, n_rows - r0);
    const int rl = kGroups * w + (lane >> 3);
    const __amdgpu_buffer_rsrc_t ry = rows_rsrc((epi & GNNREC_EPI_NO_Y) ? nullptr : y, r0,
                                                ldy4 / 4, slice, nv);
    // base inputs in layer order: x0 (INIT), the acc rows (ADD), the previous layer (ACC_X:
    // `prev`, by default the hop's own input rows)
    const bool init = (epi & GNNREC_EPI_ACC_INIT) != 0, add = (epi & GNNREC_EPI_ACC_ADD) != 0,
               xin = (epi & GNNREC_EPI_ACC_X) != 0;
    const int nb = (int)init + (int)add + (int)xin;
    const __amdgpu_buffer_rsrc_t rs = rows_rsrc(init ? self : nullptr, r0, ls4 / 4, slice, nv);
    const __amdgpu_buffer_rsrc_t racc = rows_rsrc(nb ? accg : nullptr, r0, la4 / 4, slice, nv);
    const __amdgpu_buffer_rsrc_t rx = rows_rsrc(xin ? prev : nullptr, r0, lp4 / 4, slice, nv);
    const uint32_t ls = ls4, la = la4, ly = ldy4;
    const __amdgpu_buffer_rsrc_t rb0 = init ? rs : racc, rb1 = (init && add) ? racc : rx;
    const uint32_t lb0 = init ? ls : la, lb1 = (init && add) ? la : lp4;
    const bool div = (epi & GNNREC_EPI_ACC_DIV) != 0;
#define GNNREC_TILED_EPI(NB, B, DIV) \
  tiled_epilogue<NB, B>(acc, R, rl, q16, ry, ly, rb0, lb0, rb1, lb1, rx, lp4, racc, la, DIV, \
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

constexpr int kVirt = kGroups * kTiledWaves;   // slot streams per block: (wave, group)

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

// One stream's slots of a step cut into groups of kApply (the kernel reads a group's
// accumulators before it writes any): slots in ascending column sub-panel, rows in order
// inside one (a row's edges keep their column order); a row appears in a group only as ONE
// run of consecutive slots — a slot that would repeat a row non-adjacently is deferred, with
// the rest of that row, to a later group (per-row order kept). Padded to a multiple of kSteps.
void stream_slots(const std::vector<const Run*>& runs, const int32_t* col, int sub_panel,
                  std::vector<Slot>& seq) {
  std::vector<Slot> pending, deferred;
  std::vector<int> in_group, blocked;
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
    in_group.clear();
    blocked.clear();
    int n = 0, last = -1;
    const size_t start = seq.size();
    for (size_t q = 0; q < pending.size(); ++q) {
      const Slot& sl = pending[q];
      if (n == kApply) {   // group full: the rest keeps its order for the next ones
        deferred.insert(deferred.end(), pending.begin() + q, pending.end());
        break;
      }
      const int r = sl.run->row;
      const bool is_blocked = std::find(blocked.begin(), blocked.end(), r) != blocked.end();
      const bool seen = std::find(in_group.begin(), in_group.end(), r) != in_group.end();
      // a repeat of the group's row: deferred unless it continues the run (chain), and
      // always without chains
      const bool repeat = seen && (kNoChain || r != last);
      if (is_blocked || repeat) {
        if (repeat && !is_blocked) blocked.push_back(r);
        deferred.push_back(sl);
        continue;
      }
      seq.push_back(sl);
      if (!seen) in_group.push_back(r);
      last = r;
      ++n;
    }
    if (!deferred.empty())   // only the stream's last group may end short
      while (seq.size() - start < (size_t)kApply) seq.push_back({nullptr, 0});
    pending.swap(deferred);
  }
  while (seq.size() % kSteps) seq.push_back({nullptr, 0});
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
  std::vector<Slot> hs[kGroups];
  int32_t step = 0;
  size_t i = 0;
  while (i < runs.size()) {
    size_t j = i;
    while (j < runs.size() && runs[j].p == runs[i].p) ++j;
    // LPT over the (wave, group) streams: longest run first onto the least loaded
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
      bool any = false;
      for (int q = 0; q < kGroups; ++q) any |= !wl[kGroups * w + q].empty();
      if (!any) continue;
      size_t n = 0;
      for (int q = 0; q < kGroups; ++q) {
        stream_slots(wl[kGroups * w + q], col, sub_panel, hs[q]);
        n = std::max(n, hs[q].size());
      }
      for (int q = 0; q < kGroups; ++q) hs[q].resize(n, Slot{nullptr, 0});
      uint32_t bar = (uint32_t)(step - cur[w]);
      for (size_t c = 0; c < n; c += kSteps) {
        // padding slots gather a line the chunk fetches anyway (its first real slot's)
        uint32_t x0 = 0;
        for (int q = 0; q < kTiledChunk; ++q) {
          const Slot& sl = hs[q / kSteps][c + q % kSteps];
          if (sl.run) {
            x0 = (uint32_t)col[sl.run->k + sl.t] - base;
            break;
          }
        }
        uint64_t cmask = 0;
        for (int q = 0; q < kGroups; ++q)       // lane 8 q + t: slot t of stream q
          for (int t = 0; t < kSteps; ++t) {
            const Slot& sl = hs[q][c + t];
            if (!sl.run) {
              out.slot[w].push_back(x0 << kRowBits | (uint32_t)R);
              out.val[w].push_back(0.f);
              continue;
            }
            const int64_t k = sl.run->k + sl.t;
            if (t > 0 && hs[q][c + t - 1].run == sl.run) cmask |= 1ull << (kSteps * q + t);
            out.slot[w].push_back(((uint32_t)col[k] - base) << kRowBits | (uint32_t)sl.run->row);
            out.val[w].push_back(val[k]);
          }
        out.hdr[w].insert(out.hdr[w].end(),
                          {bar, (uint32_t)cmask, (uint32_t)(cmask >> 32), base});
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
  // tail chunks for the last prefetches: harmless slots (row 0 of x, the scratch-row field)
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
    hipError_t e = hipFuncSetAttribute((const void*)tiled_hop_kernel<false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)tiled_hop_kernel<true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    done[dev] = e == hipSuccess ? 1 : -1;
    if (e != hipSuccess) (void)hipGetLastError();
  }
  return done[dev];
}
}  // namespace

extern "C" int gnnrec_tiled_plan_quad(void) { return kQuad ? 1 : 0; }

namespace gnnrec {
namespace {
// wave_ptr_out = exclusive scan of each wave's chunk count rounded up to a multiple of 4: one
// workgroup, each thread a contiguous run of waves
__global__ __launch_bounds__(1024) void quad_offsets_kernel(const int64_t* __restrict__ wp,
                                                            int64_t n_waves,
                                                            int64_t* __restrict__ out) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int64_t per = (n_waves + 1023) / 1024;
  const int64_t s0 = min(n_waves, t * per), s1 = min(n_waves, s0 + per);
  int64_t sum = 0;
  for (int64_t s = s0; s < s1; ++s) sum += (wp[s + 1] - wp[s] + 3) / 4 * 4;
  part[t] = sum;
  __syncthreads();
  if (t == 0) {
    int64_t run = 0;
    for (int i = 0; i < 1024; ++i) {
      const int64_t v = part[i];
      part[i] = run;
      run += v;
    }
    out[0] = 0;
  }
  __syncthreads();
  int64_t run = part[t];
  for (int64_t s = s0; s < s1; ++s) {
    run += (wp[s + 1] - wp[s] + 3) / 4 * 4;
    out[s + 1] = run;
  }
}

// one 64-lane workgroup per output chunk j: the chunk-major plan's chunk at the same position
// of its wave's range, or an empty chunk (padding to the quad, or one of the 16 tail chunks)
template <bool FACT>
__global__ __launch_bounds__(64) void quad_layout_kernel(
    const int64_t* __restrict__ wp, const int64_t* __restrict__ wq, int64_t n_waves,
    int64_t total, uint32_t pad_word, const uint32_t* __restrict__ slot,
    const float* __restrict__ val, const uint8_t* __restrict__ cls,
    const uint32_t* __restrict__ hdr, uint32_t* __restrict__ slot_out,
    float* __restrict__ val_out, uint8_t* __restrict__ cls_out, uint32_t* __restrict__ hdr_out) {
  const int64_t j = blockIdx.x;
  const int l = threadIdx.x;
  int64_t src = -1;
  if (j < total) {
    int64_t lo = 0, hi = n_waves;   // the wave s with wq[s] <= j < wq[s + 1]
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) / 2;
      if (wq[mid] <= j) lo = mid; else hi = mid;
    }
    const int64_t off = j - wq[lo];
    if (off < wp[lo + 1] - wp[lo]) src = wp[lo] + off;
  }
  const int64_t o = (j / 4) * (4 * kTiledChunk) + 4 * l + (j % 4);
  slot_out[o] = src >= 0 ? slot[src * kTiledChunk + l] : pad_word;
  if constexpr (FACT)
    cls_out[o] = src >= 0 ? cls[src * kTiledChunk + l] : (uint8_t)0;
  else
    val_out[o] = src >= 0 ? val[src * kTiledChunk + l] : 0.f;
  if (l < 4) hdr_out[4 * j + l] = src >= 0 ? hdr[4 * src + l] : 0u;
}
}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_tiled_plan_quad_offsets(const int64_t* wave_ptr, int64_t n_waves,
                                              int64_t* wave_ptr_out, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(wave_ptr && wave_ptr_out && n_waves >= 0, "tiled_quad_offsets: bad args");
  hipLaunchKernelGGL(quad_offsets_kernel, dim3(1), dim3(1024), 0, as_hip(stream), wave_ptr,
                     n_waves, wave_ptr_out);
  return check_launch("tiled_quad_offsets");
}

extern "C" int gnnrec_tiled_plan_quad_layout(const int64_t* wave_ptr, const int64_t* wave_ptr_out,
                                             int64_t n_waves, int64_t total_chunks,
                                             int32_t rows_per_block, const uint32_t* slot,
                                             const float* val, const uint8_t* slot_class,
                                             const uint32_t* hdr, uint32_t* slot_out,
                                             float* val_out, uint8_t* class_out,
                                             uint32_t* hdr_out, gnnrec_stream_t stream) {
  const bool fact = slot_class != nullptr;
  GNNREC_REQUIRE(wave_ptr && wave_ptr_out && slot && hdr && slot_out && hdr_out &&
                     (fact ? class_out != nullptr : (val && val_out)) && n_waves >= 0 &&
                     total_chunks >= 0 && total_chunks % 4 == 0 && rows_per_block >= 1 &&
                     rows_per_block <= GNNREC_TILED_MAX_ROWS,
                 "tiled_quad_layout: bad args (total_chunks = wave_ptr_out[n_waves], a multiple "
                 "of 4)");
  const int64_t chunks = total_chunks + GNNREC_TILED_QUAD_TAIL;
  GNNREC_REQUIRE(chunks < INT32_MAX, "tiled_quad_layout: too many chunks");
  hipStream_t s = as_hip(stream);
  if (fact)
    hipLaunchKernelGGL(quad_layout_kernel<true>, dim3((unsigned)chunks), dim3(64), 0, s, wave_ptr,
                       wave_ptr_out, n_waves, total_chunks, (uint32_t)rows_per_block, slot, val,
                       slot_class, hdr, slot_out, val_out, class_out, hdr_out);
  else
    hipLaunchKernelGGL(quad_layout_kernel<false>, dim3((unsigned)chunks), dim3(64), 0, s,
                       wave_ptr, wave_ptr_out, n_waves, total_chunks, (uint32_t)rows_per_block,
                       slot, val, slot_class, hdr, slot_out, val_out, class_out, hdr_out);
  return check_launch("tiled_quad_layout");
}

extern "C" int gnnrec_spmm_tiled_supported(int32_t device, int32_t rows_per_block) {
  if (rows_per_block < 1 || rows_per_block > GNNREC_TILED_MAX_ROWS) return 0;
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return 0;
  if (device != cur && hipSetDevice(device) != hipSuccess) return 0;
  const size_t lds = (size_t)(rows_per_block + 1) * kAccBytes;
  const int ok = lds <= 160 * 1024 && (lds <= 64 * 1024 || tiled_lds_attribute(device) > 0);
  if (device != cur) (void)hipSetDevice(cur);
  return ok;
}

extern "C" int gnnrec_spmm_tiled_f32(const uint32_t* slot, const float* val,
                                     const uint8_t* slot_class, const float* row_factor,
                                     const float* class_table, int32_t n_classes,
                                     const uint32_t* hdr, const int64_t* wave_ptr,
                                     const int32_t* n_steps, int64_t n_blocks,
                                     int32_t rows_per_block, const float* x, int64_t x_rows,
                                     int64_t ldx, float* y, int64_t ldy, int64_t n_rows, int32_t d,
                                     int32_t epi, const float* self, int64_t ld_self, float* acc,
                                     int64_t ld_acc, float acc_div, const float* prev,
                                     int64_t ld_prev, uint32_t* sync, int32_t meet_us,
                                     gnnrec_stream_t stream) {
  GNNREC_REQUIRE(d > 0 && d % (kSlice * kSPW) == 0,
                 "spmm_tiled: d must be a multiple of %d (got %d)", kSlice * kSPW, (int)d);
  GNNREC_REQUIRE(rows_per_block >= 1 && rows_per_block <= GNNREC_TILED_MAX_ROWS,
                 "spmm_tiled: bad rows_per_block");
  GNNREC_REQUIRE(n_rows >= 0 && n_blocks == (n_rows + rows_per_block - 1) / rows_per_block,
                 "spmm_tiled: n_blocks does not match n_rows / rows_per_block");
  GNNREC_REQUIRE(ldx >= d && ldx % 4 == 0 && x_rows >= 0 && ldx * 4 <= kMaxRowBytes,
                 "spmm_tiled: need d <= ldx <= %d and ldx %% 4 == 0", kMaxRowBytes / 4);
  GNNREC_REQUIRE((epi & GNNREC_EPI_NO_Y) || (y && ldy >= d && ldy % 4 == 0),
                 "spmm_tiled: null y or ldy < d or ldy %% 4 != 0");
  GNNREC_REQUIRE(!(epi & GNNREC_EPI_ACC_INIT) || (self && ld_self >= d && ld_self % 4 == 0),
                 "spmm_tiled: ACC_INIT needs self (ld %% 4 == 0)");
  GNNREC_REQUIRE(!(epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)) ||
                     (acc && ld_acc >= d && ld_acc % 4 == 0),
                 "spmm_tiled: ACC needs acc (ld %% 4 == 0)");
  if (prev == nullptr) {   // ACC_X default: the hop's own input rows
    prev = x;
    ld_prev = ldx;
    GNNREC_REQUIRE(!(epi & GNNREC_EPI_ACC_X) || x_rows >= n_rows,
                   "spmm_tiled: ACC_X without prev needs a square operand");
  }
  GNNREC_REQUIRE(!(epi & GNNREC_EPI_ACC_X) || (epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)),
                 "spmm_tiled: ACC_X needs ACC_INIT or ACC_ADD");
  GNNREC_REQUIRE(!(epi & GNNREC_EPI_ACC_X) || (ld_prev >= d && ld_prev % 4 == 0 &&
                                               aligned16(prev)),
                 "spmm_tiled: ACC_X rows must be 16-B aligned with ld %% 4 == 0, ld >= d");
  GNNREC_REQUIRE(!(epi & GNNREC_EPI_ACC_DIV) || (epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)),
                 "spmm_tiled: ACC_DIV needs ACC_INIT or ACC_ADD");
  GNNREC_REQUIRE(meet_us >= 0 && meet_us <= 100000, "spmm_tiled: meet_us must be in [0, 1e5]");
  const bool fact = slot_class != nullptr;
  GNNREC_REQUIRE(!fact || (row_factor && class_table && n_classes >= 1 &&
                           n_classes <= kMaxClasses &&
                           rows_per_block <= GNNREC_TILED_MAX_ROWS_FACTORED),
                 "spmm_tiled: a factored plan needs row_factor, class_table, 1 <= n_classes <= "
                 "%d and rows_per_block <= %d", kMaxClasses, GNNREC_TILED_MAX_ROWS_FACTORED);
  constexpr int64_t kMaxLd = ((int64_t)1 << 32) / (4 * 4096);   // epilogue row offsets: 32-bit
  GNNREC_REQUIRE(ldy <= kMaxLd && ld_self <= kMaxLd && ld_acc <= kMaxLd && ld_prev <= kMaxLd,
                 "spmm_tiled: output / self / acc row strides must be <= %lld",
                 (long long)kMaxLd);
  if (n_rows == 0) return GNNREC_OK;
  GNNREC_REQUIRE(slot && (val || fact) && hdr && wave_ptr && n_steps && x && sync,
                 "spmm_tiled: null pointer");
  GNNREC_REQUIRE(aligned16(x) && ((epi & GNNREC_EPI_NO_Y) || aligned16(y)) &&
                     (!(epi & GNNREC_EPI_ACC_INIT) || aligned16(self)) &&
                     (!(epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)) || aligned16(acc)),
                 "spmm_tiled: x / y / self / acc must be 16-B aligned");
  hipStream_t s = as_hip(stream);
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  const size_t lds = (size_t)(rows_per_block + 1) * kAccBytes +
                     (fact ? (size_t)(rows_per_block + 1) * 4 + kMaxClasses * 4 : 0);
  GNNREC_REQUIRE(lds <= 160 * 1024, "spmm_tiled: %d rows per block need %zu B of LDS (> 160 KB)",
                 (int)rows_per_block, lds);
  if (lds > 64 * 1024 && tiled_lds_attribute(dev) < 0) {
    set_error("spmm_tiled: the device refused %zu bytes of dynamic LDS", lds);
    return GNNREC_EHIP;
  }
  const int64_t grid = std::min<int64_t>(cus, n_blocks);
  const int64_t nb_pad = ceil_div(n_blocks, grid) * grid;   // every slice starts a pass
  const int64_t n_items = (int64_t)(d / (kSlice * kSPW)) * nb_pad;
  GNNREC_REQUIRE(n_items < INT32_MAX && n_rows < INT32_MAX && x_rows < INT32_MAX,
                 "spmm_tiled: too many blocks / rows");
  if (hipMemsetAsync(sync, 0, GNNREC_TILED_SYNC_WORDS * sizeof(uint32_t), s) != hipSuccess)
    return check_launch("spmm_tiled (sync reset)");
  hipLaunchKernelGGL(fact ? tiled_hop_kernel<true> : tiled_hop_kernel<false>, dim3((unsigned)grid),
                     dim3(kTiledWaves * 64), lds, s, slot, val, slot_class, row_factor,
                     class_table, (int)n_classes, hdr, wave_ptr, n_steps,
                     (int)n_blocks, (int)nb_pad, (int)n_items, (int)rows_per_block, x,
                     (uint32_t)x_rows, (uint32_t)(ldx * 4), y, (uint32_t)(ldy * 4),
                     (int)n_rows, epi, self, (uint32_t)(ld_self * 4), acc, (uint32_t)(ld_acc * 4),
                     acc_div, prev, (uint32_t)(ld_prev * 4), sync,
                     (unsigned)meet_us * 100u /* wall_clock64 runs at 100 MHz */);
  return check_launch("spmm_tiled");
}

// ---- factored plans (ABI 8) ----------------------------------------------------------------
namespace gnnrec {
namespace {
// One workgroup per (block, wave) run of chunks: each real slot's class is its column's class,
// and its value must be fl(row_factor[row] * class_table[class]) bit for bit — any slot that
// is not counts one mismatch (the caller then keeps the explicit values). Padding slots
// (row field = rows_per_block) get class 0; their products land in the scratch row.
__global__ __launch_bounds__(256) void tiled_factor_kernel(
    const uint32_t* __restrict__ slot, const float* __restrict__ val,
    const uint32_t* __restrict__ hdr, const int64_t* __restrict__ wave_ptr, int R,
    int64_t n_rows, int64_t n_cols, const float* __restrict__ rowf,
    const uint8_t* __restrict__ col_class, const float* __restrict__ ctab, int n_classes,
    uint8_t* __restrict__ cls, unsigned* __restrict__ bad) {
  const int64_t s = blockIdx.x;
  const int64_t blk = s / kTiledWaves;
  const int64_t e = wave_ptr[s + 1] * kTiledChunk;
  unsigned miss = 0;
  for (int64_t i = wave_ptr[s] * kTiledChunk + threadIdx.x; i < e; i += blockDim.x) {
    const uint32_t w = slot[i];
    const uint32_t row = w & kRowMask;
    uint8_t k = 0;
    if (row < (uint32_t)R) {
      const int64_t col = (int64_t)hdr[4 * (i / kTiledChunk) + 3] + (w >> kRowBits);
      const int64_t r = blk * R + row;
      bool ok = col < n_cols && r < n_rows;
      if (ok) {
        k = col_class[col];
        ok = k < n_classes &&
             __float_as_uint(__fmul_rn(rowf[r], ctab[k])) == __float_as_uint(val[i]);
      }
      miss += ok ? 0u : 1u;
    }
    cls[i] = k;
  }
  if (miss) atomicAdd(bad, miss);
}
}  // namespace
}  // namespace gnnrec

extern "C" int gnnrec_tiled_plan_factor(const uint32_t* slot, const float* val,
                                        const uint32_t* hdr, const int64_t* wave_ptr,
                                        int64_t n_blocks, int32_t rows_per_block, int64_t n_rows,
                                        int64_t n_cols, const float* row_factor,
                                        const uint8_t* col_class, const float* class_table,
                                        int32_t n_classes, uint8_t* slot_class,
                                        uint32_t* mismatches, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_blocks >= 0 && rows_per_block >= 1 &&
                     rows_per_block <= GNNREC_TILED_MAX_ROWS && n_rows >= 0 && n_cols >= 0,
                 "tiled_factor: bad sizes");
  GNNREC_REQUIRE(n_classes >= 1 && n_classes <= kMaxClasses,
                 "tiled_factor: n_classes must be in [1, %d]", kMaxClasses);
  if (n_blocks == 0) return GNNREC_OK;
  GNNREC_REQUIRE(slot && val && hdr && wave_ptr && row_factor && col_class && class_table &&
                     slot_class && mismatches,
                 "tiled_factor: null pointer");
  const int64_t segs = n_blocks * kTiledWaves;
  GNNREC_REQUIRE(segs < INT32_MAX, "tiled_factor: too many blocks");
  hipLaunchKernelGGL(tiled_factor_kernel, dim3((unsigned)segs), dim3(256), 0, as_hip(stream),
                     slot, val, hdr, wave_ptr, (int)rows_per_block, n_rows, n_cols, row_factor,
                     col_class, class_table, (int)n_classes, slot_class, mismatches);
  return check_launch("tiled_factor");
}
