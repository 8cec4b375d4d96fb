// Diagnostic variants of spmm_heavy_kernel (NOT part of libgnnrec): MODE 0 full, 1 no
// consumer chain, 2 no loads, 3 no park. Generated from csrc/spmm.hip's heavy-row section.
#include "../gnn-recommendations_amd/csrc/gather.h"
namespace gnnrec {
constexpr int kHeavyThreads = 512;
constexpr int kHeavyLoaders = kHeavyThreads - 64;       // waves 1..7
constexpr int kHeavyBufFloats = 16384;                   // per LDS buffer (64 KB)
constexpr int kHeavyMinD = 16;
constexpr int kHeavyMaxChunk = kHeavyBufFloats / kHeavyMinD;          // vals per buffer
constexpr int kHeavyPieces = (kHeavyBufFloats / 4 + kHeavyLoaders - 1) / kHeavyLoaders;  // 10
constexpr int kHeavyVals = (kHeavyMaxChunk + kHeavyLoaders - 1) / kHeavyLoaders;         // 3
constexpr size_t kHeavyLds = 2 * kHeavyBufFloats * sizeof(float) +
                             2 * kHeavyMaxChunk * sizeof(float);

// Neighbours per chunk (a multiple of 4) for a row width d: chk + 2 <= 16384 / d.
__host__ __device__ constexpr int heavy_chunk(int d) { return ((kHeavyBufFloats / d - 2) / 4) * 4; }

struct HeavyCols {        // (col, val) of one chunk, as this loader thread needs them
  int c[kHeavyPieces];
  float v[kHeavyVals];
};
struct HeavyStage {       // one chunk's gathered rows + vals in flight in registers
  float4 x[kHeavyPieces];
  float v[kHeavyVals];
};

// F: features per consumer lane (d <= 64 F); DC: d as a compile-time constant (0 = runtime d).
template <int F, int DC, int MODE>
__global__ __launch_bounds__(kHeavyThreads) void xheavy(
    Csr A, const int64_t* __restrict__ rows, const float* __restrict__ x, int64_t ldx,
    float* __restrict__ y, int64_t ldy, int d_rt, int epi, const float* __restrict__ self,
    int64_t ld_self, float* __restrict__ acc, int64_t ld_acc, float acc_div) {
  const int d = DC ? DC : d_rt;
  extern __shared__ float4 heavy_lds4[];
  float* buf = reinterpret_cast<float*>(heavy_lds4);     // [2][kHeavyBufFloats]: [d][S] each
  float* vbuf = buf + 2 * kHeavyBufFloats;               // [2][kHeavyMaxChunk]
  const int tid = threadIdx.x, lane = tid & 63;
  const bool consumer = tid < 64;
  const int lt = tid - 64;                               // loader thread index
  const int64_t r = rows[blockIdx.x];
  const int64_t beg = A.row_ptr[r], end = A.row_ptr[r + 1];
  const int q4 = d >> 2;                                 // float4 per neighbour row
  const int chk = heavy_chunk(d);                        // neighbours per chunk
  const int S = chk + 2;                                 // LDS row stride of a feature
  const int npieces = chk * q4;
  const int64_t n_chunks = (end - beg + chk - 1) / chk;

  auto load_cols = [&](int64_t c, HeavyCols& hc) {
    const int64_t k0 = beg + c * chk;
#pragma unroll
    for (int i = 0; i < kHeavyPieces; ++i) {
      const int p = lt + i * kHeavyLoaders;
      const int64_t k = k0 + p / q4;
      hc.c[i] = (c < n_chunks && p < npieces && k < end) ? A.col[k] : -1;
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
      const int p = lt + i * kHeavyLoaders, part = p - (p / q4) * q4;
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
      const int p = lt + i * kHeavyLoaders;
      if (p < npieces) {
        const int j = p / q4, f0 = 4 * (p - j * q4);
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
  auto consume = [&](int64_t c) {
    const float* xb = buf + (c & 1) * kHeavyBufFloats;
    const float* vb = vbuf + (c & 1) * kHeavyMaxChunk;
    const int m = (int)min<int64_t>(chk, end - (beg + c * chk));
    const int steps = m >> 2;
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
    for (int j = steps * 4; j < m; ++j) {
      const float v = vb[j];
#pragma unroll
      for (int f = 0; f < F; ++f) a[f] = __builtin_fmaf(v, xb[fo[f] + j], a[f]);
    }
  };

  // prologue (loaders): chunk 0 parked, chunk 1 gathering, columns of chunk 2 loading
  HeavyCols ca, cb;
  HeavyStage sa, sb;
  if (!consumer) {
    load_cols(0, ca);
    gather(ca, sa);
    load_cols(1, cb);
    park(sa, 0);
    gather(cb, sb);
    load_cols(2, ca);
  }
  __syncthreads();
  // round c: loaders gather c+2, load the columns of c+3, park c+1; wave 0 consumes c.
  // Unrolled by two so the register sets alternate statically.
  auto round = [&](int64_t c, HeavyCols& cols_c2, HeavyCols& cols_c3, HeavyStage& st_c1,
                   HeavyStage& st_c2) {
    if (consumer) {
      if (MODE != 1) consume(c);
    } else {
      if (MODE != 2) gather(cols_c2, st_c2);
      if (MODE != 2) load_cols(c + 3, cols_c3);
      if (MODE != 3 && c + 1 < n_chunks) park(st_c1, (int)((c + 1) & 1));
    }
    __syncthreads();
  };
  for (int64_t c = 0; c < n_chunks; c += 2) {
    round(c, ca, cb, sb, sa);                // c+1 in sb, c+2 -> sa, cols c+2 in ca, c+3 -> cb
    if (c + 1 < n_chunks) round(c + 1, cb, ca, sa, sb);
  }
  if (!consumer) return;
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

}  // namespace gnnrec
using namespace gnnrec;

template <int MODE>
static void launch(Csr A, const int64_t* rows, int64_t n, const float* x, float* y, hipStream_t st) {
  hipLaunchKernelGGL((xheavy<1, 64, MODE>), dim3((unsigned)n), dim3(kHeavyThreads), kHeavyLds, st,
                     A, rows, x, 64, y, 64, 64, 0, nullptr, 0, nullptr, 0, 1.f);
}

extern "C" int xheavy_run(int mode, const int64_t* rp, const int32_t* col, const float* val,
                          const int64_t* rows, int64_t n, const float* x, float* y,
                          hipStream_t st) {
  const Csr A{rp, col, val, 0};
  if (mode == 0) launch<0>(A, rows, n, x, y, st);
  else if (mode == 1) launch<1>(A, rows, n, x, y, st);
  else if (mode == 2) launch<2>(A, rows, n, x, y, st);
  else launch<3>(A, rows, n, x, y, st);
  return (int)hipGetLastError();
}
