// Normalised-adjacency SpMM over a CSR destination-row operand, gfx950 (MI355X).
//
// Replaces torch.sparse.mm(adj, x) of the reference (baselines/lightgcn.py:88,178,
// baselines/ngcf.py:70, orthogonal_bundle/model.py:172,184,333,344). The reference CPU kernel
// (ATen sparse addmm on the row-sorted COO) computes, per destination row r and feature f,
//     y[r,f] = fmaf(val_k, x[col_k, f], y[r,f])  for k over the row in ascending column order,
// starting from +0.0f. That order is reproduced exactly here, so results are bit-identical.
//
// Row mapping and load pipelining: see gather.h.
#include <mutex>

#include "gather.h"

// LDS steps (4 neighbours each) the heavy-row consumer keeps in flight ahead of its chain
#ifndef GNNREC_HEAVY_AHEAD
#define GNNREC_HEAVY_AHEAD 4
#endif

namespace gnnrec {

// Trace builds only (tools/exp_heavy_trace.py): wave-0-lane timestamps (wall_clock64, 100 MHz,
// then clock64, core cycles) of the first kHeavyTraceBlocks heavy workgroups,
// [2][block][wave][event]
#ifdef GNNREC_HEAVY_TRACE
constexpr int kHeavyTraceBlocks = 8, kHeavyTraceEvents = 64;
__device__ unsigned long long* g_heavy_trace;
#define GNNREC_HEAVY_STAMP(ev)                                                                  \
  do {                                                                                          \
    if (blockIdx.x < kHeavyTraceBlocks && (threadIdx.x & 63) == 0 && (ev) < kHeavyTraceEvents) \
    {                                                                                           \
      const int64_t i_ = (blockIdx.x * (kHeavyThreads / 64) + (threadIdx.x >> 6)) *            \
                             kHeavyTraceEvents + (ev);                                          \
      g_heavy_trace[i_] = wall_clock64();                                                       \
      g_heavy_trace[i_ + kHeavyTraceBlocks * (kHeavyThreads / 64) * kHeavyTraceEvents] =        \
          clock64();                                                                            \
    }                                                                                           \
    ++(ev);                                                                                     \
  } while (0)
#else
#define GNNREC_HEAVY_STAMP(ev) ((void)0)
#endif

// MASKED: skip the neighbours whose input row is all-zero (xmask). ACTIVE: rows with
// y_active[r] == 0 are not computed (written as +0 with the epilogue applied) — for rows
// whose value nobody reads, or that no non-zero input row reaches.
// LAT: the latency form of the chain (gather_row_pipe; small operands, see gather.h).
template <int D, bool MASKED = false, bool ACTIVE = false, bool LAT = false>
__global__ __launch_bounds__(kBlock) void spmm_vec_kernel(
    Csr A, const float* __restrict__ x, int64_t ldx, float* __restrict__ y, int64_t ldy,
    int epi, const float* __restrict__ self, int64_t ld_self, float* __restrict__ acc,
    int64_t ld_acc, float acc_div, int64_t skip_len, const uint8_t* __restrict__ xmask,
    const uint8_t* __restrict__ y_active) {
  constexpr int VEC = LAT ? SpmmLatCfg<D>::VEC : SpmmCfg<D>::VEC;
  constexpr int CH = SpmmCfg<D>::CH;
  constexpr int GROUP = D / VEC;
  constexpr int RPW = 64 / GROUP;
  const int lane = threadIdx.x & 63;
  const int gl = lane % GROUP;
  const int64_t r =
      ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * RPW + lane / GROUP;
  if (r >= A.n_rows) return;  // the whole group leaves together
  const int64_t beg = A.row_ptr[r], end = A.row_ptr[r + 1];
  if (skip_len > 0 && end - beg > skip_len) return;  // a heavy row: spmm_heavy_kernel's
  VecF<VEC> a;
  if (ACTIVE && y_active[r] == 0) {
    // no neighbour of this row is non-zero (or the row is not needed): the chain would add
    // only +-0 terms to +0
#pragma unroll
    for (int q = 0; q < VEC; ++q) a.v[q] = 0.f;
  } else if constexpr (LAT && !MASKED) {
    a = gather_row_pipe<VEC, GROUP, SpmmLatCfg<D>::CH>(A.col, A.val, beg, end, x, ldx, gl);
  } else {
    a = gather_row_v<VEC, GROUP, CH, false, MASKED>(A.col, A.val, beg, end, x, ldx, gl, xmask);
  }
  if (!(epi & GNNREC_EPI_NO_Y)) stv<VEC>(y + r * ldy + VEC * gl, a);
  acc_epilogue_v<VEC>(epi, a, self + r * ld_self + VEC * gl, acc + r * ld_acc + VEC * gl, acc_div);
}

// Any-d fallback: one wave per row, lanes stride the features (same k order per feature).
__global__ __launch_bounds__(kBlock) void spmm_generic_kernel(
    Csr A, const float* __restrict__ x, int64_t ldx, float* __restrict__ y, int64_t ldy,
    int d, int epi, const float* __restrict__ self, int64_t ld_self, float* __restrict__ acc,
    int64_t ld_acc, float acc_div, int64_t skip_len) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (r >= A.n_rows) return;
  const int64_t beg = A.row_ptr[r], end = A.row_ptr[r + 1];
  if (skip_len > 0 && end - beg > skip_len) return;
  for (int f = lane; f < d; f += 64) {
    float a = 0.f;
    for (int64_t k = beg; k < end; ++k) a = __builtin_fmaf(A.val[k], x[(int64_t)A.col[k] * ldx + f], a);
    if (!(epi & GNNREC_EPI_NO_Y)) y[r * ldy + f] = a;
    if (epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)) {
      float b = (epi & GNNREC_EPI_ACC_INIT) ? self[r * ld_self + f] : acc[r * ld_acc + f];
      b = b + a;
      if (epi & GNNREC_EPI_ACC_DIV) b = b / acc_div;
      acc[r * ld_acc + f] = b;
    }
  }
}

// Heavy rows (one workgroup of kHeavyThreads per listed row). The bit-exact order makes a row
// one sequential fmaf chain per feature, so a long row cannot be split; what is parallelised
// is the GATHER. Wave 0 is the consumer and does nothing but the chain; waves 1..7 (the
// loaders) fetch the neighbour rows chunk by chunk into an LDS double buffer. Software
// pipeline, round c: the loaders issue the row gathers of chunk c+2 (whose columns arrived in
// round c-1) and the (col, val) loads of chunk c+3, then park chunk c+1 (gathered in round
// c-1) in the free buffer, while wave 0 consumes chunk c; one barrier per round.
//
// The parked chunk is stored FEATURE-major, [d][S] with S = chk + 2 (S/2 odd): consumer lane f
// reads neighbours j, j+1 of its feature with one conflict-free ds_read_b64 (two per 4
// neighbours, plus one 16-B broadcast read of their 4 values), so the consumer issues ~1.75
// instructions per neighbour around its dependent fmaf instead of a ds_read_b32 each.
// Workgroup geometry (experiment builds may halve both: 2 workgroups per CU)
#ifndef GNNREC_HEAVY_THREADS
#define GNNREC_HEAVY_THREADS 512
#endif
#ifndef GNNREC_HEAVY_BUF
#define GNNREC_HEAVY_BUF 16384
#endif
constexpr int kHeavyThreads = GNNREC_HEAVY_THREADS;
constexpr int kHeavyLoaders = kHeavyThreads - 64;       // waves 1..7
constexpr int kHeavyBufFloats = GNNREC_HEAVY_BUF;        // per LDS buffer (64 KB)
constexpr int kHeavyMinD = 16;
constexpr int kHeavyMaxChunk = kHeavyBufFloats / kHeavyMinD;          // vals per buffer
constexpr int kHeavyPieces = (kHeavyBufFloats / 4 + kHeavyLoaders - 1) / kHeavyLoaders;  // 10
constexpr int kHeavyVals = (kHeavyMaxChunk + kHeavyLoaders - 1) / kHeavyLoaders;         // 3
constexpr int kHeavyPad = 64;   // floats past the value buffers: the consumer's read-ahead
constexpr size_t kHeavyLds = 2 * kHeavyBufFloats * sizeof(float) +
                             2 * kHeavyMaxChunk * sizeof(float) + kHeavyPad * sizeof(float);

// Neighbours per chunk (a multiple of 4) for a row width d: chk + 2 <= 16384 / d.
__host__ __device__ constexpr int heavy_chunk(int d) { return ((kHeavyBufFloats / d - 2) / 4) * 4; }
// ... for the 16-neighbour-group consumer: a multiple of 16 with chk + 4 <= 16384 / d
__host__ __device__ constexpr int heavy_chunk_grp(int d) { return ((kHeavyBufFloats / d - 4) / 16) * 16; }

// 1: the narrow-slice instances (d = 16 / 32 per workgroup, the sliced longest rows) consume in
// 16-neighbour groups with the values broadcast by DPP (see heavy_row's consume)
#ifndef GNNREC_HEAVY_GROUPS
#define GNNREC_HEAVY_GROUPS 1
#endif
// diagnostic builds (timing only, results wrong): 1 = no consumer chain, 2 = no row gathers,
// 4 = loaders idle (the consumer chains whatever the buffers hold), 16 = the group consumer's
// chain without its LDS reads
#ifndef GNNREC_HEAVY_DIAG
#define GNNREC_HEAVY_DIAG 0
#endif
// groups of 16 neighbours the group consumer keeps in flight (LDS reads ahead of its chain)
#ifndef GNNREC_HEAVY_GRP_AHEAD
#define GNNREC_HEAVY_GRP_AHEAD 2
#endif
// 1: the group consumer's fmafs as v_fmac_f32_dpp (inline asm), 0: DPP move + v_fmac
#ifndef GNNREC_HEAVY_DPP_FMAC
#define GNNREC_HEAVY_DPP_FMAC 1
#endif

template <int T>
__device__ __forceinline__ float lane_bcast16(float v) {   // DPP row_newbcast: lane T of each 16
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               0x150 + T, 0xF, 0xF, true));
}

struct HeavyCols {        // (col, val) of one chunk, as this loader thread needs them
  int c[kHeavyPieces];
  float v[kHeavyVals];
};
struct HeavyStage {       // one chunk's gathered rows + vals in flight in registers
  float4 x[kHeavyPieces];
  float v[kHeavyVals];
};

// Which chunk slot (j = neighbour, part = float4 of its row) loader piece p fills. The plain
// order (j = p / q4) gives a 32-lane store group two neighbours x all 16 parts at d = 64, and
// the feature-major park then lands those 32 dwords on 8 banks (4-way: every ds_write_b32 at
// twice its cycles, 40 of them per loader thread per round). Swizzled, a 64-piece block holds
// rpb = 64 / q4 neighbours with j fastest, so a group spans 8 parts x 4 neighbours = 16 banks
// at d = 64 (2-way: free for ds_write_b32) and 32 banks at d = 32. A wave's load instruction
// still covers the same rpb whole rows. Needs q4 | 64 (d = 16, 32, 64, 128, 256).
#ifndef GNNREC_HEAVY_SWIZZLE
#define GNNREC_HEAVY_SWIZZLE 1
#endif
template <int DC>
__device__ __forceinline__ void heavy_piece(int p, int q4, int& j, int& part) {
  const bool swz = GNNREC_HEAVY_SWIZZLE && (DC ? (64 % (DC / 4) == 0) : (64 % q4 == 0));
  if (swz) {
    const int rpb = 64 / q4;
    j = (p >> 6) * rpb + (p & 63) % rpb;
    part = (p & 63) / rpb;
  } else {
    j = p / q4;
    part = p - j * q4;
  }
}

// One heavy row r (or a feature slice of it: x / y / self / acc already offset to the slice,
// d = its width) on the whole workgroup. F: features per consumer lane (d <= 64 F); DC: d as a
// compile-time constant (0 = runtime d).
template <int F, int DC>
__device__ __forceinline__ void heavy_row(
    const Csr& A, int64_t r, const float* __restrict__ x, int64_t ldx, float* __restrict__ y,
    int64_t ldy, int d_rt, int epi, const float* __restrict__ self, int64_t ld_self,
    float* __restrict__ acc, int64_t ld_acc, float acc_div) {
  const int d = DC ? DC : d_rt;
  extern __shared__ float4 heavy_lds4[];
  float* buf = reinterpret_cast<float*>(heavy_lds4);     // [2][kHeavyBufFloats]: [d][S] each
  float* vbuf = buf + 2 * kHeavyBufFloats;               // [2][kHeavyMaxChunk]
  const int tid = threadIdx.x, lane = tid & 63;
  const bool consumer = tid < 64;
  const int lt = tid - 64;                               // loader thread index
  const int64_t beg = A.row_ptr[r], end = A.row_ptr[r + 1];
  const int q4 = d >> 2;                                 // float4 per neighbour row
  // the 16-neighbour-group consumer (narrow slices, see consume): chunks of 16k neighbours and
  // a feature stride S = 4 x odd, so a lane's 4 neighbours are one aligned conflict-free
  // ds_read_b128; otherwise S = chk + 2 (S/2 odd) for the ds_read_b64 pairs
  constexpr bool kGrp = GNNREC_HEAVY_GROUPS && F == 1 && (DC == 16 || DC == 32);
  const int chk = kGrp ? heavy_chunk_grp(d) : heavy_chunk(d);   // neighbours per chunk
  const int S = kGrp ? chk + 4 : chk + 2;                       // LDS row stride of a feature
  const int64_t n_chunks = (end - beg + chk - 1) / chk;

  auto load_cols = [&](int64_t c, HeavyCols& hc) {
    const int64_t k0 = beg + c * chk;
#pragma unroll
    for (int i = 0; i < kHeavyPieces; ++i) {
      int j, part;
      heavy_piece<DC>(lt + i * kHeavyLoaders, q4, j, part);
      const int64_t k = k0 + j;
      hc.c[i] = (c < n_chunks && j < chk && k < end) ? A.col[k] : -1;
    }
#pragma unroll
    for (int i = 0; i < kHeavyVals; ++i) {
      const int j = lt + i * kHeavyLoaders;
      const int64_t k = k0 + j;
      hc.v[i] = (c < n_chunks && j < chk && k < end) ? A.val[k] : 0.f;
    }
  };
  auto gather = [&](const HeavyCols& hc, HeavyStage& st) {
#pragma unroll
    for (int i = 0; i < kHeavyPieces; ++i) {
      int j, part;
      heavy_piece<DC>(lt + i * kHeavyLoaders, q4, j, part);
      if (GNNREC_HEAVY_DIAG & 2) {   // diagnostic builds only: no row gathers (wrong results)
        st.x[i] = make_float4(__int_as_float(hc.c[i]), 0.f, 0.f, 0.f);
        continue;
      }
      st.x[i] = hc.c[i] >= 0
                    ? *reinterpret_cast<const float4*>(x + (int64_t)hc.c[i] * ldx + 4 * part)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < kHeavyVals; ++i) st.v[i] = hc.v[i];
  };
  auto park = [&](const HeavyStage& st, int b) {
    float* dst = buf + b * kHeavyBufFloats;
#pragma unroll
    for (int i = 0; i < kHeavyPieces; ++i) {
      int j, part;
      heavy_piece<DC>(lt + i * kHeavyLoaders, q4, j, part);
      if (j < chk) {
        const int f0 = 4 * part;
        dst[(f0 + 0) * S + j] = st.x[i].x;
        dst[(f0 + 1) * S + j] = st.x[i].y;
        dst[(f0 + 2) * S + j] = st.x[i].z;
        dst[(f0 + 3) * S + j] = st.x[i].w;
      }
    }
#pragma unroll
    for (int i = 0; i < kHeavyVals; ++i) {
      const int j = lt + i * kHeavyLoaders;
      if (j < chk) vbuf[b * kHeavyMaxChunk + j] = st.v[i];
    }
  };

  float a[F];
#pragma unroll
  for (int f = 0; f < F; ++f) a[f] = 0.f;
  // consumer lanes: feature lane + 64 f, clamped into the row so no lane is masked off (a
  // clamped lane computes a duplicate it never stores) and the LDS reads need no branches
  int fo[F];
#pragma unroll
  for (int f = 0; f < F; ++f) fo[f] = min(lane + 64 * f, d - 1) * S;
  // One step = 4 neighbours: their values (one broadcast float4) and, per feature, two
  // float2 reads of the feature-major chunk; then the 4 ordered fmafs per feature.
  struct Step {
    float4 v;
    float2 x[F][2];
  };
  auto fetch = [&](const float* xb, const float* vb, int j, Step& st) {
    st.v = *reinterpret_cast<const float4*>(vb + j);
#pragma unroll
    for (int f = 0; f < F; ++f) {
      st.x[f][0] = *reinterpret_cast<const float2*>(xb + fo[f] + j);
      st.x[f][1] = *reinterpret_cast<const float2*>(xb + fo[f] + j + 2);
    }
  };
  auto apply = [&](const Step& st) {
#pragma unroll
    for (int f = 0; f < F; ++f) a[f] = __builtin_fmaf(st.v.x, st.x[f][0].x, a[f]);
#pragma unroll
    for (int f = 0; f < F; ++f) a[f] = __builtin_fmaf(st.v.y, st.x[f][0].y, a[f]);
#pragma unroll
    for (int f = 0; f < F; ++f) a[f] = __builtin_fmaf(st.v.z, st.x[f][1].x, a[f]);
#pragma unroll
    for (int f = 0; f < F; ++f) a[f] = __builtin_fmaf(st.v.w, st.x[f][1].y, a[f]);
  };
#ifdef GNNREC_HEAVY_TRACE
  int ev = 0;
#endif
  auto consume = [&](int64_t c) {
    if (GNNREC_HEAVY_DIAG & 1) return;   // diagnostic builds only: no chain (wrong results)
    const float* xb = buf + (c & 1) * kHeavyBufFloats;
    const float* vb = vbuf + (c & 1) * kHeavyMaxChunk;
    const int m = (int)min<int64_t>(chk, end - (beg + c * chk));
    const int steps = m >> 2;
    if constexpr (kGrp) {
      // Narrow slices (the longest rows' chains, d = 16 / 32 features per workgroup): the chain
      // is the time, and the step form below waited on its LDS reads (2 per 4 neighbours, at
      // most 15 outstanding: lgkmcnt) — 16-18 cycles per neighbour against the ≈ 6 of a bare
      // dependent v_fma_f32 chain (tools/fma_latency.hip). Here a group of 16 neighbours is ONE
      // ds_read_b32 of their values (lane l of each 16-lane row reads value j + l % 16; DPP
      // row_newbcast hands value j + t to every lane) and 4 aligned ds_read_b128 of the lane's
      // feature, two groups in flight. The fmafs are the row's, in its order: the same bits.
      struct Grp {
        float v;
        float4 x[4];
      };
      auto fetch_g = [&](int j, Grp& g) {
        if (GNNREC_HEAVY_DIAG & 16) {   // diagnostic builds only: no LDS reads (wrong results)
          g.v = __int_as_float(j + lane);
#pragma unroll
          for (int q = 0; q < 4; ++q) g.x[q] = make_float4(g.v, g.v, g.v, g.v);
          return;
        }
        g.v = vb[j + (lane & 15)];
#pragma unroll
        for (int q = 0; q < 4; ++q) g.x[q] = *reinterpret_cast<const float4*>(xb + fo[0] + j + 4 * q);
      };
      auto apply_g = [&](const Grp& g) {
#if GNNREC_HEAVY_DPP_FMAC
        // one v_fmac_f32_dpp per neighbour (the compiler does not fold a DPP move into a MAC)
#define GNNREC_F1(X, T)                                                                      \
  asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:" #T " row_mask:0xf bank_mask:0xf"  \
               " bound_ctrl:1"                                                             \
               : "+v"(a[0])                                                                \
               : "v"(g.v), "v"(X));
#define GNNREC_G4(Q, T0, T1, T2, T3) \
  GNNREC_F1(g.x[Q].x, T0) GNNREC_F1(g.x[Q].y, T1) GNNREC_F1(g.x[Q].z, T2) GNNREC_F1(g.x[Q].w, T3)
        GNNREC_G4(0, 0, 1, 2, 3) GNNREC_G4(1, 4, 5, 6, 7) GNNREC_G4(2, 8, 9, 10, 11)
        GNNREC_G4(3, 12, 13, 14, 15)
#undef GNNREC_G4
#undef GNNREC_F1
#else
#define GNNREC_G4(Q, T0)                                                  \
  a[0] = __builtin_fmaf(lane_bcast16<T0 + 0>(g.v), g.x[Q].x, a[0]);      \
  a[0] = __builtin_fmaf(lane_bcast16<T0 + 1>(g.v), g.x[Q].y, a[0]);      \
  a[0] = __builtin_fmaf(lane_bcast16<T0 + 2>(g.v), g.x[Q].z, a[0]);      \
  a[0] = __builtin_fmaf(lane_bcast16<T0 + 3>(g.v), g.x[Q].w, a[0]);
        GNNREC_G4(0, 0) GNNREC_G4(1, 4) GNNREC_G4(2, 8) GNNREC_G4(3, 12)
#undef GNNREC_G4
#endif
      };
      // GA groups in flight (register sets); the read-ahead past the chunk stays inside the
      // allocation for GA <= 3 (feature rows: chk + 4 + 16 (GA - 1) <= S + 16 (GA - 1) floats
      // of a 16 384-float buffer; values: into kHeavyPad) and is never applied
      constexpr int GA = GNNREC_HEAVY_GRP_AHEAD;
      static_assert(GA >= 1 && GA <= 3, "group consumer: 1..3 groups in flight");
      const int groups = m >> 4;
      Grp g[GA];
#pragma unroll
      for (int i = 0; i < GA; ++i) fetch_g(16 * i, g[i]);
      int q = 0;
      for (; q + GA <= groups; q += GA) {
#pragma unroll
        for (int i = 0; i < GA; ++i) {
          apply_g(g[i]);
          fetch_g(16 * (q + i + GA), g[i]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int i = 0; i < GA; ++i)
        if (q + i < groups) apply_g(g[i]);
      for (int j = groups * 16; j < m; ++j) a[0] = __builtin_fmaf(vb[j], xb[fo[0] + j], a[0]);
      return;
    } else if constexpr (F == 1 && DC != 0) {
      // d = 32 / 64: P register sets, the LDS reads of steps q+1 .. q+P-1 in flight while step
      // q's chain runs. The read-ahead is not clamped to the chunk: reads past it stay inside
      // the allocation (the next buffer, the value buffers, kHeavyPad) and are never applied,
      // so a step costs no index arithmetic; a scheduling barrier per step keeps each fetch P
      // steps ahead of its use (unpinned, the compiler regrouped the fetches of P steps and
      // then waited on them). The wider and runtime-d instances spilled with it, and the
      // d = 128 one ran slower in this form: they keep two sets below.
      constexpr int P = GNNREC_HEAVY_AHEAD;
      Step s[P];
#pragma unroll
      for (int i = 0; i < P; ++i) fetch(xb, vb, 4 * i, s[i]);
      int q = 0;
      for (; q + P <= steps; q += P) {
#pragma unroll
        for (int i = 0; i < P; ++i) {
          apply(s[i]);
          fetch(xb, vb, 4 * (q + i + P), s[i]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int i = 0; i < P; ++i)
        if (q + i < steps) apply(s[i]);
    } else {
      // two register sets: the reads of step q+1 are in flight while step q's chain runs
      Step s0, s1;
      if (steps > 0) fetch(xb, vb, 0, s0);
      int q = 0;
      for (; q + 2 <= steps; q += 2) {
        fetch(xb, vb, 4 * (q + 1), s1);
        apply(s0);
        fetch(xb, vb, 4 * min(q + 2, steps - 1), s0);
        apply(s1);
      }
      if (q < steps) apply(s0);
    }
    for (int j = steps * 4; j < m; ++j) {
      const float v = vb[j];
#pragma unroll
      for (int f = 0; f < F; ++f) a[f] = __builtin_fmaf(v, xb[fo[f] + j], a[f]);
    }
  };

  // prologue (loaders): chunk 0 parked, chunk 1 gathering, columns of chunk 2 loading
  HeavyCols ca, cb;
  HeavyStage sa, sb;
  GNNREC_HEAVY_STAMP(ev);
  if (!consumer && !(GNNREC_HEAVY_DIAG & 4)) {
    load_cols(0, ca);
    gather(ca, sa);
    load_cols(1, cb);
    park(sa, 0);
    gather(cb, sb);
    load_cols(2, ca);
  }
  GNNREC_HEAVY_STAMP(ev);
  __syncthreads();
  GNNREC_HEAVY_STAMP(ev);
  // round c: loaders gather c+2, load the columns of c+3, park c+1; wave 0 consumes c.
  // Unrolled by two so the register sets alternate statically.
  auto round = [&](int64_t c, HeavyCols& cols_c2, HeavyCols& cols_c3, HeavyStage& st_c1,
                   HeavyStage& st_c2) {
    if (consumer) {
      consume(c);
    } else if (!(GNNREC_HEAVY_DIAG & 4)) {   // diagnostic builds: 4 = idle loaders
      gather(cols_c2, st_c2);                // columns of c+2 arrived during round c-1
      load_cols(c + 3, cols_c3);
      if (c + 1 < n_chunks) park(st_c1, (int)((c + 1) & 1));
    }
    GNNREC_HEAVY_STAMP(ev);
    __syncthreads();
    GNNREC_HEAVY_STAMP(ev);
  };
  for (int64_t c = 0; c < n_chunks; c += 2) {
    round(c, ca, cb, sb, sa);                // c+1 in sb, c+2 -> sa, cols c+2 in ca, c+3 -> cb
    if (c + 1 < n_chunks) round(c + 1, cb, ca, sa, sb);
  }
  if (!consumer) return;
  GNNREC_HEAVY_STAMP(ev);
#pragma unroll
  for (int f = 0; f < F; ++f) {
    const int col_f = lane + 64 * f;
    if (col_f >= d) continue;
    if (!(epi & GNNREC_EPI_NO_Y)) y[r * ldy + col_f] = a[f];
    if (epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)) {
      float b = (epi & GNNREC_EPI_ACC_INIT) ? self[r * ld_self + col_f] : acc[r * ld_acc + col_f];
      b = b + a[f];
      if (epi & GNNREC_EPI_ACC_DIV) b = b / acc_div;
      acc[r * ld_acc + col_f] = b;
    }
  }
}

// The heavy-row launch: block b < n_sliced * SLICES runs feature slice b % SLICES (d / SLICES
// features, instance <SF, SDC>) of row rows[b / SLICES]; the other blocks run whole rows
// rows[n_sliced ..] (instance <F, DC>). rows is longest first, so the sliced rows are the
// longest: each slice gathers 1/SLICES of every neighbour row, so its loaders fill a chunk of
// SLICES x the neighbours per round and the row's chain finishes in fewer rounds. Every slice
// still applies its features' fmafs in the row's order: the same bits.
//
// Fused light rows (small operands, d = 32 / 64 / 128): blocks b >= n_heavy_blocks run the
// row-parallel kernel's latency form over rows [(b - n_heavy_blocks) R, ... + R) (R rows per
// block at GROUP lanes per row), skipping the heavy rows (longer than light_skip) exactly as
// spmm_vec_kernel<D, false, false, true> does. They are dispatched after the heavy blocks, so
// they fill the CUs the shorter heavy rows free while the longest chains run: one launch per
// hop instead of two back-to-back (config 2: the light rows' ~15 us per hop ran after the
// heavy rows' ~40 us). Same fmaf chains: the same bits.
template <int D>
__device__ __forceinline__ void light_rows_block(
    const Csr& A, int64_t lb, int64_t light_skip, const float* __restrict__ x, int64_t ldx,
    float* __restrict__ y, int64_t ldy, int epi, const float* __restrict__ self, int64_t ld_self,
    float* __restrict__ acc, int64_t ld_acc, float acc_div) {
  constexpr int VEC = SpmmLatCfg<D>::VEC, GROUP = D / VEC, RPW = 64 / GROUP;
  const int lane = threadIdx.x & 63, gl = lane % GROUP;
  const int64_t r = (lb * (kHeavyThreads / 64) + (threadIdx.x >> 6)) * RPW + lane / GROUP;
  if (r >= A.n_rows) return;   // the whole row group leaves together
  const int64_t beg = A.row_ptr[r], end = A.row_ptr[r + 1];
  if (end - beg > light_skip) return;   // a heavy row: one of this launch's heavy blocks
  const VecF<VEC> a = gather_row_pipe<VEC, GROUP, SpmmLatCfg<D>::CH>(A.col, A.val, beg, end, x, ldx, gl);
  if (!(epi & GNNREC_EPI_NO_Y)) stv<VEC>(y + r * ldy + VEC * gl, a);
  acc_epilogue_v<VEC>(epi, a, self + r * ld_self + VEC * gl, acc + r * ld_acc + VEC * gl, acc_div);
}
template <int D> constexpr int kLightRowsPerBlock =
    (64 / (D / SpmmLatCfg<D>::VEC)) * (kHeavyThreads / 64);

template <int F, int DC, int SLICES, int SF, int SDC>
__global__ __launch_bounds__(kHeavyThreads) void spmm_heavy_kernel(
    Csr A, const int64_t* __restrict__ rows, int64_t n_sliced, int64_t heavy_first,
    int64_t n_light_blocks, int64_t light_skip, const float* __restrict__ x,
    int64_t ldx, float* __restrict__ y, int64_t ldy, int d_rt, int epi,
    const float* __restrict__ self, int64_t ld_self, float* __restrict__ acc, int64_t ld_acc,
    float acc_div) {
  int64_t b = blockIdx.x;
  if constexpr (DC == 32 || DC == 64 || DC == 128) {
    // dispatch order: heavy blocks [0, heavy_first), the light blocks, the other heavy blocks
    if (n_light_blocks > 0 && b >= heavy_first) {
      if (b < heavy_first + n_light_blocks) {
        light_rows_block<DC>(A, b - heavy_first, light_skip, x, ldx, y, ldy, epi, self, ld_self,
                             acc, ld_acc, acc_div);
        return;
      }
      b -= n_light_blocks;
    }
  }
  if constexpr (SLICES > 1) {
    static_assert(DC > 0 && SDC * SLICES == DC, "sliced instance: SDC = DC / SLICES");
    if (b < n_sliced * SLICES) {
      const int64_t r = rows[b / SLICES];
      const int f0 = (int)(b % SLICES) * SDC;
      // (y / self / acc are null when the epilogue does not use them)
      heavy_row<SF, SDC>(A, r, x + f0, ldx, y ? y + f0 : nullptr, ldy, SDC, epi,
                         self ? self + f0 : nullptr, ld_self, acc ? acc + f0 : nullptr, ld_acc,
                         acc_div);
      return;
    }
    b -= n_sliced * (SLICES - 1);
  }
  heavy_row<F, DC>(A, rows[b], x, ldx, y, ldy, d_rt, epi, self, ld_self, acc, ld_acc, acc_div);
}

// mask[r] = 1 if row r of x has any element != 0 (NaN counts as non-zero), for the masked hop.
__global__ __launch_bounds__(kBlock) void row_nonzero_kernel(const float* __restrict__ x,
                                                             int64_t ldx, int64_t n_rows, int d,
                                                             uint8_t* __restrict__ mask) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; r < n_rows;
       r += ((int64_t)gridDim.x * kBlock) >> 6) {
    bool nz = false;
    for (int f = lane; f < d; f += 64) nz |= !(x[r * ldx + f] == 0.f);
    const unsigned long long b = __ballot(nz);
    if (lane == 0) mask[r] = b != 0 ? 1 : 0;
  }
}

// y_active[r] = 1 for every destination row r with a neighbour c whose x row is non-zero,
// scattered from the non-zero sources through the TRANSPOSE's rows (row c lists every r with
// A[r, c] != 0); y_active must be zeroed first. Benign races: every writer stores 1.
__global__ __launch_bounds__(kBlock) void mark_active_kernel(const int64_t* __restrict__ rp_t,
                                                             const int32_t* __restrict__ col_t,
                                                             int64_t n_src,
                                                             const uint8_t* __restrict__ x_nonzero,
                                                             uint8_t* __restrict__ y_active) {
  const int lane = threadIdx.x & 63;
  for (int64_t c = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; c < n_src;
       c += ((int64_t)gridDim.x * kBlock) >> 6) {
    if (!x_nonzero[c]) continue;
    for (int64_t k = rp_t[c] + lane; k < rp_t[c + 1]; k += 64) y_active[col_t[k]] = 1;
  }
}

// MODE 0: standalone GAS of x rows. MODE 1: GAS(A x) (fused hop epilogue).
template <int D, int MODE>
__global__ __launch_bounds__(kBlock) void gas_kernel(Csr A, const float* __restrict__ x,
                                                     int64_t ldx, float* __restrict__ y,
                                                     int64_t ldy, int bs,
                                                     const float* __restrict__ blocks,
                                                     const int32_t* __restrict__ perm) {
  constexpr int GROUP = D / 4;
  constexpr int RPW = 64 / GROUP;
  constexpr int ROWS = RPW * (kBlock / 64);
  __shared__ float w_lds[D * 32];         // d/bs blocks of bs*bs (bs <= 32)
  __shared__ float z_lds[ROWS][D + 4];
  const int lane = threadIdx.x & 63;
  const int gl = lane % GROUP;
  const int slot = (threadIdx.x >> 6) * RPW + lane / GROUP;
  for (int i = threadIdx.x; i < D * bs; i += kBlock) w_lds[i] = blocks[i];
  int pj[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) pj[q] = perm[4 * gl + q];
  const int64_t r = (int64_t)blockIdx.x * ROWS + slot;
  const bool valid = r < A.n_rows;
  float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  if (valid) {
    if (MODE == 0) {
      z = ld4(x + r * ldx + 4 * gl);
    } else {
      z = gather_row<GROUP>(A.col, A.val, A.row_ptr[r], A.row_ptr[r + 1], x, ldx, gl);
    }
  }
  st4(&z_lds[slot][4 * gl], z);
  __syncthreads();
  if (valid) st4(y + r * ldy + 4 * gl, gas_row<D>(&z_lds[slot][0], w_lds, bs, pj));
}

}  // namespace gnnrec

using namespace gnnrec;

namespace {

template <int D>
void launch_spmm_vec4(const Csr& A, const float* x, int64_t ldx, float* y, int64_t ldy, int epi,
                      const float* self, int64_t ld_self, float* acc, int64_t ld_acc,
                      float acc_div, int64_t skip, const uint8_t* xmask, const uint8_t* y_active,
                      bool lat, hipStream_t s) {
  // rows per workgroup of each form (the latency form may map a row to fewer lanes)
  constexpr int RPB = (64 / (D / SpmmCfg<D>::VEC)) * (kBlock / 64);
  constexpr int RPB_LAT = (64 / (D / SpmmLatCfg<D>::VEC)) * (kBlock / 64);
  // the masked kernels have no latency form
  const bool use_lat = lat && SpmmLatCfg<D>::OK && !xmask;
  const int64_t grid = ceil_div(A.n_rows, use_lat ? RPB_LAT : RPB);
#define GNNREC_VEC(M, AC, LT)                                                                      \
  hipLaunchKernelGGL((spmm_vec_kernel<D, M, AC, LT>), dim3((unsigned)grid), dim3(kBlock), 0, s, A, \
                     x, ldx, y, ldy, epi, self, ld_self, acc, ld_acc, acc_div, skip, xmask,       \
                     y_active)
  if (xmask && y_active) GNNREC_VEC(true, true, false);
  else if (xmask) GNNREC_VEC(true, false, false);
  else if (y_active && use_lat) GNNREC_VEC(false, true, SpmmLatCfg<D>::OK);
  else if (y_active) GNNREC_VEC(false, true, false);
  else if (use_lat) GNNREC_VEC(false, false, SpmmLatCfg<D>::OK);
  else GNNREC_VEC(false, false, false);
#undef GNNREC_VEC
}

bool vec4_ok(int d, const float* x, int64_t ldx, const float* y, int64_t ldy, int epi,
             const float* self, int64_t ld_self, const float* acc, int64_t ld_acc) {
  if (!(d == 8 || d == 16 || d == 32 || d == 64 || d == 128 || d == 256)) return false;
  if (!aligned16(x) || (ldx & 3)) return false;
  if (!(epi & GNNREC_EPI_NO_Y) && (!aligned16(y) || (ldy & 3))) return false;
  if ((epi & GNNREC_EPI_ACC_INIT) && (!aligned16(self) || (ld_self & 3))) return false;
  if ((epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)) && (!aligned16(acc) || (ld_acc & 3)))
    return false;
  return true;
}

// Rows at most this many: the row-parallel kernel runs the latency form of the chain (gather.h
// gather_row_pipe) unless a GNNREC_CSR_LIGHT_* flag says otherwise.
constexpr int64_t kLatencyMaxRows = 65536;

// The side stream a GNNREC_CSR_FORK launch runs its heavy rows on (one per device, created on
// first use, the device's highest priority so its workgroups are dispatched before the
// row-parallel kernel's), with the fork / join events. The mutex also keeps one caller's
// record-wait-launch-record-wait sequence whole.
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};
std::mutex g_side_mu;
SideStream g_side[64];

int side_stream(hipStream_t caller, SideStream** out) {
  // the side stream lives on the caller's stream's device (the null stream: the current one)
  hipDevice_t dev = 0;
  int cur = 0;
  if (hipStreamGetDevice(caller, &dev) != hipSuccess || dev < 0 || dev >= 64 ||
      hipGetDevice(&cur) != hipSuccess) {
    set_error("spmm: no device for the heavy-row side stream");
    return GNNREC_EHIP;
  }
  if (cur != dev) {
    set_error("spmm: GNNREC_CSR_FORK needs the caller's stream on the current device");
    return GNNREC_EINVAL;
  }
  SideStream& ss = g_side[dev];
  if (!ss.s) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
        hipStreamCreateWithPriority(&ss.s, hipStreamNonBlocking, greatest) != hipSuccess ||
        hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ss.join, hipEventDisableTiming) != hipSuccess) {
      set_error("spmm: creating the heavy-row side stream failed");
      return GNNREC_EHIP;
    }
  }
  *out = &ss;
  return GNNREC_OK;
}

// Feature slices of a sliced heavy row: narrow (16 features) at d = 32 and on small operands
// at d = 64, where the rows' chains are latency-bound and a 64-B slice of a neighbour row
// costs nothing extra (config 2: 4 slices 0.188 ms vs 2 slices 0.192 ms); otherwise whole
// 128-B lines (32 features: d = 64 -> 2 slices, 128 -> 4) or 64 features at d = 256, since a
// half-line slice doubles a bandwidth-bound row's line requests (power-law 2M x 2M, d = 64:
// 4 slices 21.9 ms vs 19.0 ms unsliced, profiles/r06/).
int heavy_slices(int d, bool small) {
  if (d == 32) return 2;
  if (d == 64) return small ? 4 : 2;
  return 4;   // d = 128 (32-wide), 256 (64-wide)
}

// light_skip > 0: the launch also runs the light rows (rows of at most light_skip neighbours,
// d = 32 / 64 / 128 only) as blocks after the heavy ones (see light_rows_block)
int launch_heavy(const Csr& A, const int64_t* heavy_rows, int64_t n_heavy, int64_t n_sliced,
                 const float* x, int64_t ldx, float* y, int64_t ldy, int d, int epi,
                 const float* self, int64_t ld_self, float* acc, int64_t ld_acc, float acc_div,
                 bool small, int64_t light_skip, hipStream_t s) {
  const int slices = heavy_slices(d, small);
  const int64_t heavy_blocks = n_heavy + n_sliced * (slices - 1);   // a block per slice
  int64_t light_blocks = 0;
  if (light_skip > 0) {
    const int rpb = d == 32 ? kLightRowsPerBlock<32> : d == 64 ? kLightRowsPerBlock<64>
                                                               : kLightRowsPerBlock<128>;
    light_blocks = ceil_div(A.n_rows, (int64_t)rpb);
  }
  const int64_t blocks = heavy_blocks + light_blocks;
  GNNREC_REQUIRE(blocks < (int64_t)INT32_MAX, "spmm: too many heavy rows");
  // dispatch order: the sliced (longest) rows' blocks, then the light blocks, then the other
  // heavy rows (config 2, threshold 256: 0.124 ms per K = 3 propagation against 0.144 with
  // every heavy block first and 0.141 with the light blocks first, profiles/r06/)
  const int64_t heavy_first = n_sliced * slices;
  const dim3 grid((unsigned)blocks), block(kHeavyThreads);
#define GNNREC_HEAVY(F, DC, SL, SF, SDC)                                                          \
  hipLaunchKernelGGL((spmm_heavy_kernel<F, DC, SL, SF, SDC>), grid, block, kHeavyLds, s, A,      \
                     heavy_rows, n_sliced, heavy_first, light_blocks, light_skip, x, ldx, y, ldy, \
                     d, epi,                                                                      \
                     self, ld_self, acc, ld_acc, acc_div)
  switch (d) {
    case 32: GNNREC_HEAVY(1, 32, 2, 1, 16); break;
    case 64:
      if (slices == 4) GNNREC_HEAVY(1, 64, 4, 1, 16);
      else GNNREC_HEAVY(1, 64, 2, 1, 32);
      break;
    case 128: GNNREC_HEAVY(2, 128, 4, 1, 32); break;
    case 256: GNNREC_HEAVY(4, 256, 4, 1, 64); break;
    default:
      if (d <= 64) GNNREC_HEAVY(1, 0, 1, 1, 0);
      else if (d <= 128) GNNREC_HEAVY(2, 0, 1, 1, 0);
      else GNNREC_HEAVY(4, 0, 1, 1, 0);
  }
#undef GNNREC_HEAVY
  return check_launch("spmm_heavy");
}

}  // namespace

#ifdef GNNREC_HEAVY_TRACE
extern "C" int gnnrec_debug_heavy_trace(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_heavy_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : -2;
}
#endif

extern "C" int gnnrec_spmm_csr_heavy_f32(const int64_t* row_ptr, const int32_t* col,
                                         const float* val, int64_t n_rows, const float* x,
                                         int64_t ldx, const uint8_t* x_nonzero,
                                         const uint8_t* y_active, float* y, int64_t ldy,
                                         int32_t d, int32_t epi, const float* self,
                                         int64_t ld_self, float* acc, int64_t ld_acc,
                                         float acc_div, const int64_t* heavy_rows,
                                         int64_t n_heavy, int64_t heavy_threshold,
                                         int64_t n_sliced, int32_t flags,
                                         gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_rows >= 0 && d >= 1, "spmm: bad sizes n_rows=%lld d=%d", (long long)n_rows, d);
  if (n_rows == 0) return GNNREC_OK;
  GNNREC_REQUIRE(row_ptr && x, "spmm: null row_ptr/x");
  GNNREC_REQUIRE(ldx >= d, "spmm: ldx < d");
  GNNREC_REQUIRE((epi & GNNREC_EPI_NO_Y) || (y && ldy >= d), "spmm: null y or ldy < d");
  GNNREC_REQUIRE(!(epi & GNNREC_EPI_ACC_INIT) || (self && ld_self >= d), "spmm: ACC_INIT needs self");
  GNNREC_REQUIRE(!(epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)) || (acc && ld_acc >= d),
                 "spmm: ACC needs acc");
  GNNREC_REQUIRE(!(epi & GNNREC_EPI_ACC_DIV) || (epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)),
                 "spmm: ACC_DIV without ACC_INIT/ACC_ADD");
  if ((epi & GNNREC_EPI_ACC_X) ||
      ((epi & GNNREC_EPI_ACC_INIT) && (epi & GNNREC_EPI_ACC_ADD))) {
    set_error("spmm: ACC_X and ACC_INIT|ACC_ADD are epilogues of gnnrec_spmm_tiled_f32 only");
    return GNNREC_EUNSUPPORTED;
  }
  GNNREC_REQUIRE(heavy_threshold >= 0 && n_heavy >= 0, "spmm: negative heavy_threshold/n_heavy");
  GNNREC_REQUIRE(n_sliced >= 0 && n_sliced <= n_heavy, "spmm: n_sliced must be in [0, n_heavy]");
  GNNREC_REQUIRE((flags & ~(GNNREC_CSR_FORK | GNNREC_CSR_LIGHT_LATENCY |
                            GNNREC_CSR_LIGHT_THROUGHPUT | GNNREC_CSR_TWO_LAUNCHES)) == 0 &&
                     (flags & (GNNREC_CSR_LIGHT_LATENCY | GNNREC_CSR_LIGHT_THROUGHPUT)) !=
                         (GNNREC_CSR_LIGHT_LATENCY | GNNREC_CSR_LIGHT_THROUGHPUT),
                 "spmm: bad flags 0x%x", flags);
  const bool split = heavy_threshold > 0;
  if (split) {
    GNNREC_REQUIRE(n_heavy == 0 || heavy_rows, "spmm: null heavy_rows");
    GNNREC_REQUIRE(d % 4 == 0 && d >= kHeavyMinD && d <= 256 && aligned16(x) && !(ldx & 3),
                   "spmm: the heavy-row path needs d %% 4 == 0, 16 <= d <= 256 and a 16-B "
                   "aligned x with ldx %% 4 == 0");
  }
  // feature slices only where the instance has them (d = 32, 64, 128, 256)
  if (!(d == 32 || d == 64 || d == 128 || d == 256)) n_sliced = 0;
  const bool heavy = split && n_heavy > 0;
  const Csr A{row_ptr, col, val, n_rows};
  hipStream_t s = as_hip(stream);
  const int64_t skip = split ? heavy_threshold : 0;
  // a small operand (its rows cannot fill the chip): latency-bound chains
  const bool small = n_rows <= kLatencyMaxRows;
  const bool lat = (flags & GNNREC_CSR_LIGHT_LATENCY) ||
                   (!(flags & GNNREC_CSR_LIGHT_THROUGHPUT) && !x_nonzero && small);
  auto light = [&]() -> int {
    const uint8_t* xm = x_nonzero;
    if (vec4_ok(d, x, ldx, y, ldy, epi, self, ld_self, acc, ld_acc)) {
      switch (d) {
        case 8: launch_spmm_vec4<8>(A, x, ldx, y, ldy, epi, self, ld_self, acc, ld_acc, acc_div, skip, xm, y_active, lat, s); break;
        case 16: launch_spmm_vec4<16>(A, x, ldx, y, ldy, epi, self, ld_self, acc, ld_acc, acc_div, skip, xm, y_active, lat, s); break;
        case 32: launch_spmm_vec4<32>(A, x, ldx, y, ldy, epi, self, ld_self, acc, ld_acc, acc_div, skip, xm, y_active, lat, s); break;
        case 64: launch_spmm_vec4<64>(A, x, ldx, y, ldy, epi, self, ld_self, acc, ld_acc, acc_div, skip, xm, y_active, lat, s); break;
        case 128: launch_spmm_vec4<128>(A, x, ldx, y, ldy, epi, self, ld_self, acc, ld_acc, acc_div, skip, xm, y_active, lat, s); break;
        default: launch_spmm_vec4<256>(A, x, ldx, y, ldy, epi, self, ld_self, acc, ld_acc, acc_div, skip, xm, y_active, lat, s); break;
      }
    } else {
      const int64_t grid = ceil_div(n_rows, kBlock / 64);
      hipLaunchKernelGGL(spmm_generic_kernel, dim3((unsigned)grid), dim3(kBlock), 0, s, A, x, ldx,
                         y, ldy, d, epi, self, ld_self, acc, ld_acc, acc_div, skip);
    }
    return check_launch("spmm");
  };
  if (!heavy) return light();
  // small operands: the light rows as blocks of the heavy launch (one launch per hop), where
  // the light kernel would run its latency form anyway
  const bool fused = !(flags & (GNNREC_CSR_FORK | GNNREC_CSR_TWO_LAUNCHES)) && lat && small &&
                     !x_nonzero && !y_active && (d == 32 || d == 64 || d == 128) &&
                     vec4_ok(d, x, ldx, y, ldy, epi, self, ld_self, acc, ld_acc);
  if (fused)
    return launch_heavy(A, heavy_rows, n_heavy, n_sliced, x, ldx, y, ldy, d, epi, self, ld_self,
                        acc, ld_acc, acc_div, small, heavy_threshold, s);
  if (!(flags & GNNREC_CSR_FORK)) {
    if (int rc = light()) return rc;
    return launch_heavy(A, heavy_rows, n_heavy, n_sliced, x, ldx, y, ldy, d, epi, self, ld_self,
                        acc, ld_acc, acc_div, small, 0, s);
  }
  // Fork / join: the heavy rows (disjoint from the row-parallel kernel's rows) go first, on the
  // high-priority side stream, so their workgroups — the longest chains — start first and the
  // row-parallel rows fill the CUs as the shorter heavy rows retire.
  std::lock_guard<std::mutex> lock(g_side_mu);
  SideStream* ss = nullptr;
  if (int rc = side_stream(s, &ss)) return rc;
  if (hipEventRecord(ss->fork, s) != hipSuccess || hipStreamWaitEvent(ss->s, ss->fork, 0) != hipSuccess)
    return check_launch("spmm: fork");
  int rc = launch_heavy(A, heavy_rows, n_heavy, n_sliced, x, ldx, y, ldy, d, epi, self, ld_self,
                        acc, ld_acc, acc_div, small, 0, ss->s);
  const int rc_light = rc == GNNREC_OK ? light() : rc;
  // join even after a failed launch, so the caller's stream never runs ahead of the side's
  if (hipEventRecord(ss->join, ss->s) != hipSuccess || hipStreamWaitEvent(s, ss->join, 0) != hipSuccess)
    return check_launch("spmm: join");
  return rc != GNNREC_OK ? rc : rc_light;
}

extern "C" int gnnrec_spmm_csr_masked_f32(const int64_t* row_ptr, const int32_t* col,
                                          const float* val, int64_t n_rows, const float* x,
                                          int64_t ldx, const uint8_t* x_nonzero,
                                          const uint8_t* y_active, float* y,
                                          int64_t ldy, int32_t d, int32_t epi, const float* self,
                                          int64_t ld_self, float* acc, int64_t ld_acc,
                                          float acc_div, const int64_t* heavy_rows,
                                          int64_t n_heavy, int64_t heavy_threshold,
                                          gnnrec_stream_t stream) {
  return gnnrec_spmm_csr_heavy_f32(row_ptr, col, val, n_rows, x, ldx, x_nonzero, y_active, y, ldy,
                                   d, epi, self, ld_self, acc, ld_acc, acc_div, heavy_rows,
                                   n_heavy, heavy_threshold, 0, 0, stream);
}

extern "C" int gnnrec_row_nonzero_f32(const float* x, int64_t ldx, int64_t n_rows, int32_t d,
                                      uint8_t* mask, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_rows >= 0 && d >= 1 && ldx >= d, "row_nonzero: bad sizes");
  if (n_rows == 0) return GNNREC_OK;
  GNNREC_REQUIRE(x && mask, "row_nonzero: null pointer");
  const int64_t g = ceil_div(n_rows, kBlock / 64);
  hipLaunchKernelGGL(row_nonzero_kernel, dim3((unsigned)(g < 65536 ? g : 65536)), dim3(kBlock), 0,
                     as_hip(stream), x, ldx, n_rows, (int)d, mask);
  return check_launch("row_nonzero");
}

extern "C" int gnnrec_mark_active_rows(const int64_t* row_ptr_t, const int32_t* col_t,
                                       int64_t n_src, const uint8_t* x_nonzero, int64_t n_dst,
                                       uint8_t* y_active, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_src >= 0 && n_dst >= 0, "mark_active_rows: bad sizes");
  GNNREC_REQUIRE(y_active && (n_src == 0 || (row_ptr_t && col_t && x_nonzero)),
                 "mark_active_rows: null pointer");
  hipStream_t s = as_hip(stream);
  if (n_dst > 0 && hipMemsetAsync(y_active, 0, (size_t)n_dst, s) != hipSuccess)
    return check_launch("mark_active_rows: memset");
  if (n_src == 0) return GNNREC_OK;
  const int64_t g = ceil_div(n_src, kBlock / 64);
  hipLaunchKernelGGL(mark_active_kernel, dim3((unsigned)(g < 65536 ? g : 65536)), dim3(kBlock), 0,
                     s, row_ptr_t, col_t, n_src, x_nonzero, y_active);
  return check_launch("mark_active_rows");
}

extern "C" int gnnrec_spmm_csr_split_f32(const int64_t* row_ptr, const int32_t* col,
                                         const float* val, int64_t n_rows, const float* x,
                                         int64_t ldx, float* y, int64_t ldy, int32_t d, int32_t epi,
                                         const float* self, int64_t ld_self, float* acc,
                                         int64_t ld_acc, float acc_div, const int64_t* heavy_rows,
                                         int64_t n_heavy, int64_t heavy_threshold,
                                         gnnrec_stream_t stream) {
  return gnnrec_spmm_csr_masked_f32(row_ptr, col, val, n_rows, x, ldx, nullptr, nullptr, y, ldy, d, epi,
                                    self, ld_self, acc, ld_acc, acc_div, heavy_rows, n_heavy,
                                    heavy_threshold, stream);
}

extern "C" int gnnrec_spmm_csr_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                                   int64_t n_rows, const float* x, int64_t ldx, float* y,
                                   int64_t ldy, int32_t d, int32_t epi, const float* self,
                                   int64_t ld_self, float* acc, int64_t ld_acc, float acc_div,
                                   gnnrec_stream_t stream) {
  return gnnrec_spmm_csr_split_f32(row_ptr, col, val, n_rows, x, ldx, y, ldy, d, epi, self,
                                   ld_self, acc, ld_acc, acc_div, nullptr, 0, 0, stream);
}

extern "C" int gnnrec_lightgcn_heavy_f32(const int64_t* row_ptr, const int32_t* col,
                                         const float* val, int64_t n_rows, const float* x0,
                                         int32_t d, int32_t n_layers, float* work0, float* work1,
                                         float* layers, float* out, int64_t ld_out,
                                         const int64_t* heavy_rows, int64_t n_heavy,
                                         int64_t heavy_threshold, int64_t n_sliced,
                                         int32_t flags, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_layers >= 0 && d >= 1 && n_rows >= 0, "lightgcn: bad sizes");
  GNNREC_REQUIRE(x0 && out && ld_out >= d, "lightgcn: null x0/out");
  GNNREC_REQUIRE(layers || n_layers <= 1 || (work0 && work1), "lightgcn: need work0/work1 or layers");
  if (n_rows == 0) return GNNREC_OK;
  hipStream_t s = as_hip(stream);
  if (n_layers == 0) {  // mean of a single layer is the layer itself
    if (hipMemcpy2DAsync(out, ld_out * sizeof(float), x0, d * sizeof(float), d * sizeof(float),
                         n_rows, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return check_launch("lightgcn copy");
    return GNNREC_OK;
  }
  const float* in = x0;
  for (int k = 1; k <= n_layers; ++k) {
    float* yk = layers ? layers + (int64_t)(k - 1) * n_rows * d : ((k & 1) ? work0 : work1);
    int epi = (k == 1) ? GNNREC_EPI_ACC_INIT : GNNREC_EPI_ACC_ADD;
    if (k == n_layers) {
      epi |= GNNREC_EPI_ACC_DIV;
      if (!layers) epi |= GNNREC_EPI_NO_Y;
    }
    const int rc = gnnrec_spmm_csr_heavy_f32(row_ptr, col, val, n_rows, in, d, nullptr, nullptr, yk,
                                             d, d, epi, x0, d, out, ld_out, (float)(n_layers + 1),
                                             heavy_rows, n_heavy, heavy_threshold, n_sliced, flags,
                                             stream);
    if (rc != GNNREC_OK) return rc;
    in = yk;
  }
  return GNNREC_OK;
}

extern "C" int gnnrec_lightgcn_split_f32(const int64_t* row_ptr, const int32_t* col,
                                         const float* val, int64_t n_rows, const float* x0,
                                         int32_t d, int32_t n_layers, float* work0, float* work1,
                                         float* layers, float* out, int64_t ld_out,
                                         const int64_t* heavy_rows, int64_t n_heavy,
                                         int64_t heavy_threshold, gnnrec_stream_t stream) {
  return gnnrec_lightgcn_heavy_f32(row_ptr, col, val, n_rows, x0, d, n_layers, work0, work1,
                                   layers, out, ld_out, heavy_rows, n_heavy, heavy_threshold, 0, 0,
                                   stream);
}

extern "C" int gnnrec_lightgcn_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                                   int64_t n_rows, const float* x0, int32_t d, int32_t n_layers,
                                   float* work0, float* work1, float* layers, float* out,
                                   int64_t ld_out, gnnrec_stream_t stream) {
  return gnnrec_lightgcn_split_f32(row_ptr, col, val, n_rows, x0, d, n_layers, work0, work1,
                                   layers, out, ld_out, nullptr, 0, 0, stream);
}

namespace {
template <int D, int MODE>
void launch_gas(const Csr& A, const float* x, int64_t ldx, float* y, int64_t ldy, int bs,
                const float* blocks, const int32_t* perm, hipStream_t s) {
  constexpr int ROWS = (64 / (D / 4)) * (kBlock / 64);
  hipLaunchKernelGGL((gas_kernel<D, MODE>), dim3((unsigned)ceil_div(A.n_rows, ROWS)), dim3(kBlock),
                     0, s, A, x, ldx, y, ldy, bs, blocks, perm);
}

template <int MODE>
int gas_dispatch(const Csr& A, const float* x, int64_t ldx, float* y, int64_t ldy, int d, int bs,
                 const float* blocks, const int32_t* perm, hipStream_t s) {
  GNNREC_REQUIRE(bs >= 1 && bs <= 32 && d % bs == 0, "gas: block size %d must divide d=%d and be <= 32", bs, d);
  GNNREC_REQUIRE(aligned16(x) && aligned16(y) && !(ldx & 3) && !(ldy & 3), "gas: x/y must be 16-B aligned with ld %% 4 == 0");
  GNNREC_REQUIRE(blocks && perm, "gas: null blocks/perm");
  switch (d) {
    case 16: launch_gas<16, MODE>(A, x, ldx, y, ldy, bs, blocks, perm, s); break;
    case 32: launch_gas<32, MODE>(A, x, ldx, y, ldy, bs, blocks, perm, s); break;
    case 64: launch_gas<64, MODE>(A, x, ldx, y, ldy, bs, blocks, perm, s); break;
    case 128: launch_gas<128, MODE>(A, x, ldx, y, ldy, bs, blocks, perm, s); break;
    default: set_error("gas: d=%d unsupported (16, 32, 64, 128)", d); return GNNREC_EUNSUPPORTED;
  }
  return check_launch("gas");
}
}  // namespace

extern "C" int gnnrec_gas_f32(const float* x, int64_t ldx, int64_t n_rows, int32_t d, int32_t bs,
                              const float* blocks, const int32_t* perm, float* y, int64_t ldy,
                              gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_rows >= 0 && x && y && ldx >= d && ldy >= d, "gas: bad args");
  if (n_rows == 0) return GNNREC_OK;
  const Csr A{nullptr, nullptr, nullptr, n_rows};
  return gas_dispatch<0>(A, x, ldx, y, ldy, d, bs, blocks, perm, as_hip(stream));
}

extern "C" int gnnrec_spmm_gas_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                                   int64_t n_rows, const float* x, int64_t ldx, float* y,
                                   int64_t ldy, int32_t d, int32_t bs, const float* blocks,
                                   const int32_t* perm, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_rows >= 0 && row_ptr && x && y && ldx >= d && ldy >= d, "spmm_gas: bad args");
  if (n_rows == 0) return GNNREC_OK;
  const Csr A{row_ptr, col, val, n_rows};
  return gas_dispatch<1>(A, x, ldx, y, ldy, d, bs, blocks, perm, as_hip(stream));
}
