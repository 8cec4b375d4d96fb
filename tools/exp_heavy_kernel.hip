// Diagnostic variants of spmm_heavy_kernel (NOT part of libgnnrec).
#include "../gnn-recommendations_amd/csrc/gather.h"
namespace gnnrec {
constexpr int kHeavyThreads = 512;
constexpr int kHeavyChunkFloats = 16384;                 // per LDS buffer
constexpr int kHeavyPieces = kHeavyChunkFloats / 4 / kHeavyThreads;  // float4 per thread
constexpr int kHeavyMinD = 16;
constexpr int kHeavyMaxChunkRows = kHeavyChunkFloats / kHeavyMinD;   // 1024
constexpr int kHeavyVals = kHeavyMaxChunkRows / kHeavyThreads;       // vals per thread
constexpr size_t kHeavyLds = 2 * kHeavyChunkFloats * sizeof(float) +
                             2 * kHeavyMaxChunkRows * sizeof(float);

struct HeavyCols {        // (col, val) of one chunk, as this thread needs them
  int c[kHeavyPieces];
  float v[kHeavyVals];
};
struct HeavyStage {       // one chunk's gathered rows + vals in flight in registers
  float4 x[kHeavyPieces];
  float v[kHeavyVals];
};

// F: features per consumer lane (d <= 64 F); DC: d as a compile-time constant (0 = runtime d),
// which turns the consumer's LDS addressing into immediate offsets.
template <int F, int DC, int MODE>
__global__ __launch_bounds__(kHeavyThreads) void xheavy(
    Csr A, const int64_t* __restrict__ rows, const float* __restrict__ x, int64_t ldx,
    float* __restrict__ y, int64_t ldy, int d_rt, int epi, const float* __restrict__ self,
    int64_t ld_self, float* __restrict__ acc, int64_t ld_acc, float acc_div) {
  const int d = DC ? DC : d_rt;
  constexpr int STEP = 16 / F;                           // neighbours per consumer step
  extern __shared__ float4 heavy_lds4[];
  float* buf = reinterpret_cast<float*>(heavy_lds4);     // [2][kHeavyChunkFloats]
  float* vbuf = buf + 2 * kHeavyChunkFloats;             // [2][kHeavyMaxChunkRows]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r = rows[blockIdx.x];
  const int64_t beg = A.row_ptr[r], end = A.row_ptr[r + 1];
  const int q4 = d >> 2;                                 // float4 per neighbour row
  const int chk = kHeavyChunkFloats / d;                 // neighbours per chunk (<= 4096)
  const int64_t n_chunks = (end - beg + chk - 1) / chk;

  auto load_cols = [&](int64_t c, HeavyCols& hc) {
    const int64_t k0 = beg + c * chk;
#pragma unroll
    for (int i = 0; i < kHeavyPieces; ++i) {
      const int j = (tid + i * kHeavyThreads) / q4;
      const int64_t k = k0 + j;
      hc.c[i] = (c < n_chunks && j < chk && k < end) ? A.col[k] : -1;
    }
#pragma unroll
    for (int i = 0; i < kHeavyVals; ++i) {
      const int j = tid + i * kHeavyThreads;
      const int64_t k = k0 + j;
      hc.v[i] = (c < n_chunks && j < chk && k < end) ? A.val[k] : 0.f;
    }
  };
  auto gather = [&](const HeavyCols& hc, HeavyStage& st) {
#pragma unroll
    for (int i = 0; i < kHeavyPieces; ++i) {
      const int p = tid + i * kHeavyThreads, part = p - (p / q4) * q4;
      st.x[i] = hc.c[i] >= 0
                    ? *reinterpret_cast<const float4*>(x + (int64_t)hc.c[i] * ldx + 4 * part)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < kHeavyVals; ++i) st.v[i] = hc.v[i];
  };
  auto park = [&](const HeavyStage& st, int b) {
    float4* dst = reinterpret_cast<float4*>(buf + b * kHeavyChunkFloats);
#pragma unroll
    for (int i = 0; i < kHeavyPieces; ++i) {
      const int p = tid + i * kHeavyThreads;
      if (p / q4 < chk) dst[p] = st.x[i];
    }
#pragma unroll
    for (int i = 0; i < kHeavyVals; ++i) {
      const int j = tid + i * kHeavyThreads;
      if (j < chk) vbuf[b * kHeavyMaxChunkRows + j] = st.v[i];
    }
  };

  float a[F];
#pragma unroll
  for (int f = 0; f < F; ++f) a[f] = 0.f;
  // consumer lanes: feature lane + 64 f, clamped into the row so no lane is masked off (a
  // clamped lane computes a duplicate it never stores) and the LDS reads need no branches
  int fcol[F];
#pragma unroll
  for (int f = 0; f < F; ++f) fcol[f] = min(lane + 64 * f, d - 1);
  // One step = the LDS reads of STEP neighbours, then their ordered FMAs. The chain itself
  // (one dependent fmaf per neighbour) bounds the consumer.
  struct Step {
    float v[STEP];
    float x[STEP][F];
  };
  auto fetch = [&](const float* xb, const float* vb, int j, Step& st) {
#pragma unroll
    for (int t = 0; t < STEP; t += 4) {   // vals: one 16-B broadcast read per 4 neighbours
      const float4 v4 = *reinterpret_cast<const float4*>(vb + j + t);
      st.v[t] = v4.x; st.v[t + 1] = v4.y; st.v[t + 2] = v4.z; st.v[t + 3] = v4.w;
    }
#pragma unroll
    for (int t = 0; t < STEP; ++t)
#pragma unroll
      for (int f = 0; f < F; ++f) st.x[t][f] = xb[(j + t) * d + fcol[f]];
  };
  auto apply = [&](const Step& st) {
#pragma unroll
    for (int t = 0; t < STEP; ++t)
#pragma unroll
      for (int f = 0; f < F; ++f) a[f] = __builtin_fmaf(st.v[t], st.x[t][f], a[f]);
  };
  auto consume = [&](int64_t c) {
    const float* xb = buf + (c & 1) * kHeavyChunkFloats;
    const float* vb = vbuf + (c & 1) * kHeavyMaxChunkRows;
    const int m = (int)min<int64_t>(chk, end - (beg + c * chk));
    const int steps = m / STEP;
    for (int q = 0; q < steps; ++q) {   // (a two-set software pipeline measured 6 % slower)
      Step s0;
      fetch(xb, vb, q * STEP, s0);
      apply(s0);
    }
    for (int j = steps * STEP; j < m; ++j) {
      const float v = vb[j];
#pragma unroll
      for (int f = 0; f < F; ++f) a[f] = __builtin_fmaf(v, xb[j * d + fcol[f]], a[f]);
    }
  };

  // prologue: chunk 0 parked, chunk 1 gathering, columns of chunk 2 loading
  HeavyCols ca, cb;
  HeavyStage sa, sb;
  load_cols(0, ca);
  gather(ca, sa);
  load_cols(1, cb);
  park(sa, 0);
  gather(cb, sb);
  load_cols(2, ca);
  __syncthreads();
  // round c: columns of c+3 -> gather of c+2 -> consume c -> park c+1 -> barrier.
  // Unrolled by two so the register sets alternate statically.
  auto round = [&](int64_t c, HeavyCols& cols_c2, HeavyCols& cols_c3, HeavyStage& st_c1,
                   HeavyStage& st_c2) {
    if (MODE != 2) gather(cols_c2, st_c2);                  // columns of c+2 arrived during round c-1
    if (MODE != 2) load_cols(c + 3, cols_c3);
    if (wave == 0 && MODE != 1) consume(c);
    if (MODE != 3 && c + 1 < n_chunks) park(st_c1, (int)((c + 1) & 1));
    __syncthreads();
  };
  for (int64_t c = 0; c < n_chunks; c += 2) {
    round(c, ca, cb, sb, sa);                // c+1 in sb, c+2 -> sa, cols c+2 in ca, c+3 -> cb
    if (c + 1 < n_chunks) round(c + 1, cb, ca, sa, sb);
  }
  if (wave != 0) return;
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
extern "C" int xheavy_run(int mode, const int64_t* rp, const int32_t* col, const float* val,
                          const int64_t* rows, int64_t n_rows_list, const float* x, float* y,
                          hipStream_t s) {
  Csr A{rp, col, val, 0};
  const dim3 g((unsigned)n_rows_list), b(kHeavyThreads);
#define L(M) hipLaunchKernelGGL((xheavy<1, 64, M>), g, b, kHeavyLds, s, A, rows, x, (int64_t)64, y, \
                               (int64_t)64, 64, 0, nullptr, (int64_t)64, nullptr, (int64_t)64, 1.f)
  switch (mode) { case 0: L(0); break; case 1: L(1); break; case 2: L(2); break; case 3: L(3); break;
                  default: return -1; }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
