// GAT training path (SURVEY §8 f1 for GAT): the sparse edge-softmax aggregation with attention
// dropout, and its backward — so GATLayer trains on the native operand instead of the
// reference's dense [N, N] masked softmax (baselines/gat.py:99-141; trained through
// trainer.py:251-276, loss.backward() at :270).
//
// Per head (o_dim features), destination row r with neighbours j (CSR pattern):
//   z_rj = s_self[r] + s_neigh[j],  e_rj = LeakyReLU(z_rj),  alpha_rj = softmax_j(e_rj)
//   out_r = sum_j alpha_rj * keep_rj / (1 - p) * h_j          (F.dropout on the weights)
// keep_rj: a Bernoulli(1 - p) draw from a counter-based hash of (seed, r, j, head), the same in
// the forward and both backward passes (no mask is stored).
// Backward, given g_r = dL/dout_r:
//   da_rj = keep_rj / (1 - p) * (g_r . h_j),   c_r = sum_j alpha_rj da_rj = g_r . out_r
//   dz_rj = alpha_rj (da_rj - c_r) * (z_rj > 0 ? 1 : slope)
//   d s_self[r] = sum_j dz_rj                                   (row pass, CSR rows)
//   d h_j = sum_{r: j in N(r)} alpha_rj keep_rj / (1 - p) g_r,  d s_neigh[j] = sum_r dz_rj
//                                                               (column pass)
// The column pass walks row j of the SAME CSR: the pattern must be symmetric (the reference's
// normalised bipartite adjacency is, graph_builder.py:52-61); the caller checks it.
// Softmax statistics (max, sum in base 2, c_r) come from the row pass and are read per edge by
// the column pass from a [n_rows][heads][4] table (one 64-B line per row at 4 heads).
// fp32 throughout; tolerance-level against the reference's dense autograd (the reference's own
// softmax and mm sum in other orders).
#include <math.h>

#include "gather.h"

namespace gnnrec {
namespace {

constexpr float kLog2eT = 1.4426950408889634f;
constexpr int kTrainChunk = 8;

struct GatTrain {
  const int64_t* row_ptr;
  const int32_t* col;
  int64_t n_rows;
  const float* h;
  int64_t ldh;          // h[j, head, :] = h + j * ldh + head * o_dim
  const float* s_self;  // [n, heads] row stride ld_s
  const float* s_neigh;
  int64_t ld_s;
  int heads, o_dim;
  float slope;
  float drop_p;   // attention dropout probability (0: none)
  uint32_t seed;
  float* out;     // forward: [n, heads * o_dim] (ldo)
  int64_t ldo;
  const float* dout;   // backward: dL/dout (lddo)
  int64_t lddo;
  float* stats;        // [n][heads][4]: max (base-2 logits), sum, c, unused
  float* dh;           // [n, heads * o_dim] (lddh)
  int64_t lddh;
  float* d_self;       // [n, heads]
  float* d_neigh;      // [n, heads]
};

// keep multiplier of edge (r <- j), head q: 0 or 1 / (1 - p)
__device__ __forceinline__ float drop_keep(const GatTrain& p, int64_t r, int64_t j, int q) {
  if (p.drop_p <= 0.f) return 1.f;
  uint32_t x = p.seed ^ (uint32_t)(r * 0x9E3779B1u) ^ (uint32_t)((uint64_t)r >> 32) * 0x7FEB352Du;
  x ^= (uint32_t)(j * 0x85EBCA77u) + (uint32_t)((uint64_t)j >> 32) * 0x846CA68Bu;
  x ^= (uint32_t)q * 0xC2B2AE3Du;
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  const float u = (float)(x >> 8) * (1.0f / 16777216.0f);   // [0, 1)
  return u >= p.drop_p ? 1.f / (1.f - p.drop_p) : 0.f;
}

__device__ __forceinline__ float logit2(float z, float slope) {
  return (z > 0.f ? z : z * slope) * kLog2eT;
}

// sum over the hl lanes of a head (aligned group inside the row's GROUP lanes)
template <int GROUP>
__device__ __forceinline__ float head_sum(float v, int hl) {
  for (int d = 1; d < hl; d <<= 1) v += __shfl_xor(v, d, GROUP);
  return v;
}

__device__ __forceinline__ float dot4t(const float4& a, const float4& b) {
  return __builtin_fmaf(a.w, b.w, __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x)));
}

// Forward with attention dropout: online max / sum in base 2 over blocks of kTrainChunk
// neighbours; the sum of the weights (softmax denominator) takes every neighbour, the weighted
// row sum only the kept ones, scaled.
template <int F>
__global__ __launch_bounds__(kBlock) void gat_train_fwd_kernel(GatTrain p) {
  constexpr int GROUP = F / 4;
  constexpr int RPW = 64 / GROUP;
  const int lane = threadIdx.x & 63;
  const int gl = lane % GROUP;
  const int64_t r = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * RPW + lane / GROUP;
  if (r >= p.n_rows) return;
  const int hl = p.o_dim / 4, head = gl / hl, fo = 4 * (gl - head * hl);
  const int64_t beg = p.row_ptr[r], end = p.row_ptr[r + 1];
  const float ss = p.s_self[r * p.ld_s + head];
  float m = -INFINITY, l = 0.f;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t k0 = beg; k0 < end; k0 += kTrainChunk) {
    int cj[kTrainChunk];
    float E[kTrainChunk];
    float4 xv[kTrainChunk];
#pragma unroll
    for (int t = 0; t < kTrainChunk; ++t) {
      const int64_t k = k0 + t < end ? k0 + t : end - 1;
      cj[t] = p.col[k];
      xv[t] = ld4(p.h + (int64_t)cj[t] * p.ldh + head * p.o_dim + fo);
      E[t] = k0 + t < end ? logit2(ss + p.s_neigh[(int64_t)cj[t] * p.ld_s + head], p.slope) : -INFINITY;
    }
    float bm = E[0];
#pragma unroll
    for (int t = 1; t < kTrainChunk; ++t) bm = fmaxf(bm, E[t]);
    const float mn = fmaxf(m, bm);
    const float sc = __builtin_amdgcn_exp2f(m - mn);
    l *= sc;
    a = make_float4(a.x * sc, a.y * sc, a.z * sc, a.w * sc);
#pragma unroll
    for (int t = 0; t < kTrainChunk; ++t) {
      const float pe = __builtin_amdgcn_exp2f(E[t] - mn);
      l += pe;
      const float w = k0 + t < end ? pe * drop_keep(p, r, cj[t], head) : 0.f;
      a = fma4(w, xv[t], a);
    }
    m = mn;
  }
  // an empty row: 0 / 0 = NaN, like the reference's all -inf softmax row
  st4(p.out + r * p.ldo + head * p.o_dim + fo, make_float4(a.x / l, a.y / l, a.z / l, a.w / l));
}

// Backward, row pass: softmax statistics, c_r = g_r . out_r and d s_self[r].
template <int F>
__global__ __launch_bounds__(kBlock) void gat_train_bwd_rows_kernel(GatTrain p) {
  constexpr int GROUP = F / 4;
  constexpr int RPW = 64 / GROUP;
  const int lane = threadIdx.x & 63;
  const int gl = lane % GROUP;
  const int64_t r = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * RPW + lane / GROUP;
  if (r >= p.n_rows) return;
  const int hl = p.o_dim / 4, head = gl / hl, fo = 4 * (gl - head * hl);
  const int64_t beg = p.row_ptr[r], end = p.row_ptr[r + 1];
  const float ss = p.s_self[r * p.ld_s + head];
  // pass 1: max and sum of the base-2 logits
  float m = -INFINITY, l = 0.f;
  for (int64_t k = beg; k < end; ++k) {
    const float e = logit2(ss + p.s_neigh[(int64_t)p.col[k] * p.ld_s + head], p.slope);
    const float mn = fmaxf(m, e);
    l = l * __builtin_amdgcn_exp2f(m - mn) + __builtin_amdgcn_exp2f(e - mn);
    m = mn;
  }
  const float4 g = ld4(p.dout + r * p.lddo + head * p.o_dim + fo);
  const float c = head_sum<GROUP>(dot4t(g, ld4(p.out + r * p.ldo + head * p.o_dim + fo)), hl);
  const float inv_l = 1.f / l;
  // pass 2: d s_self
  float dss = 0.f;
  for (int64_t k0 = beg; k0 < end; k0 += kTrainChunk) {
    int cj[kTrainChunk];
    float4 xv[kTrainChunk];
    float z[kTrainChunk];
#pragma unroll
    for (int t = 0; t < kTrainChunk; ++t) {
      const int64_t k = k0 + t < end ? k0 + t : end - 1;
      cj[t] = p.col[k];
      xv[t] = ld4(p.h + (int64_t)cj[t] * p.ldh + head * p.o_dim + fo);
      z[t] = ss + p.s_neigh[(int64_t)cj[t] * p.ld_s + head];
    }
#pragma unroll
    for (int t = 0; t < kTrainChunk; ++t) {
      const float da = drop_keep(p, r, cj[t], head) * head_sum<GROUP>(dot4t(g, xv[t]), hl);
      const float alpha = __builtin_amdgcn_exp2f(logit2(z[t], p.slope) - m) * inv_l;
      const float dz = alpha * (da - c) * (z[t] > 0.f ? 1.f : p.slope);
      dss += k0 + t < end ? dz : 0.f;
    }
  }
  if (fo == 0) {
    p.d_self[r * p.heads + head] = end > beg ? dss : 0.f;
    float* st = p.stats + (r * p.heads + head) * 4;
    st[0] = m;
    st[1] = l;
    st[2] = c;
    st[3] = 0.f;
  }
}

// Backward, column pass over the symmetric pattern: node j's row lists the rows r that
// aggregate j. d h_j and d s_neigh[j].
template <int F>
__global__ __launch_bounds__(kBlock) void gat_train_bwd_cols_kernel(GatTrain p) {
  constexpr int GROUP = F / 4;
  constexpr int RPW = 64 / GROUP;
  const int lane = threadIdx.x & 63;
  const int gl = lane % GROUP;
  const int64_t j = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * RPW + lane / GROUP;
  if (j >= p.n_rows) return;
  const int hl = p.o_dim / 4, head = gl / hl, fo = 4 * (gl - head * hl);
  const int64_t beg = p.row_ptr[j], end = p.row_ptr[j + 1];
  const float sn = p.s_neigh[j * p.ld_s + head];
  const float4 hj = ld4(p.h + j * p.ldh + head * p.o_dim + fo);
  float4 dh = make_float4(0.f, 0.f, 0.f, 0.f);
  float dsn = 0.f;
  for (int64_t k0 = beg; k0 < end; k0 += kTrainChunk) {
    int ri[kTrainChunk];
    float4 g[kTrainChunk];
    float4 st[kTrainChunk];
    float ssr[kTrainChunk];
#pragma unroll
    for (int t = 0; t < kTrainChunk; ++t) {
      const int64_t k = k0 + t < end ? k0 + t : end - 1;
      ri[t] = p.col[k];
      g[t] = ld4(p.dout + (int64_t)ri[t] * p.lddo + head * p.o_dim + fo);
      st[t] = ld4(p.stats + ((int64_t)ri[t] * p.heads + head) * 4);
      ssr[t] = p.s_self[(int64_t)ri[t] * p.ld_s + head];
    }
#pragma unroll
    for (int t = 0; t < kTrainChunk; ++t) {
      const float z = ssr[t] + sn;
      const float alpha = __builtin_amdgcn_exp2f(logit2(z, p.slope) - st[t].x) / st[t].y;
      const float keep = drop_keep(p, ri[t], j, head);
      const float da = keep * head_sum<GROUP>(dot4t(g[t], hj), hl);
      const float dz = alpha * (da - st[t].z) * (z > 0.f ? 1.f : p.slope);
      const float w = k0 + t < end ? alpha * keep : 0.f;
      dh = fma4(w, g[t], dh);
      dsn += k0 + t < end ? dz : 0.f;
    }
  }
  st4(p.dh + j * p.lddh + head * p.o_dim + fo, dh);
  if (fo == 0) p.d_neigh[j * p.heads + head] = dsn;
}

int check_train(const GatTrain& p, bool bwd) {
  GNNREC_REQUIRE(p.n_rows >= 0 && p.heads >= 1 && p.o_dim >= 4 && p.o_dim % 4 == 0,
                 "gat_train: bad sizes");
  const int F = p.heads * p.o_dim;
  GNNREC_REQUIRE(F == 16 || F == 32 || F == 64 || F == 128 || F == 256,
                 "gat_train: heads*o_dim = %d unsupported (16..256, power of two)", F);
  GNNREC_REQUIRE((p.o_dim / 4 & (p.o_dim / 4 - 1)) == 0, "gat_train: o_dim / 4 must be a power of two");
  GNNREC_REQUIRE(p.drop_p >= 0.f && p.drop_p < 1.f, "gat_train: dropout p must be in [0, 1)");
  GNNREC_REQUIRE(p.row_ptr && p.col && p.h && p.s_self && p.s_neigh && p.out && aligned16(p.h) &&
                     aligned16(p.out) && !(p.ldh & 3) && !(p.ldo & 3) && p.ldh >= F && p.ldo >= F &&
                     p.ld_s >= p.heads,
                 "gat_train: null or misaligned operand");
  if (bwd)
    GNNREC_REQUIRE(p.dout && p.stats && p.dh && p.d_self && p.d_neigh && aligned16(p.dout) &&
                       aligned16(p.stats) && aligned16(p.dh) && !(p.lddo & 3) && !(p.lddh & 3) &&
                       p.lddo >= F && p.lddh >= F,
                   "gat_train_backward: null or misaligned gradient buffer");
  return GNNREC_OK;
}

template <template <int> class K>
int launch_f(const GatTrain& p, hipStream_t s) {
  const int F = p.heads * p.o_dim;
  auto grid = [&](int f) { return dim3((unsigned)ceil_div(p.n_rows, (64 / (f / 4)) * (kBlock / 64))); };
  switch (F) {
    case 16: hipLaunchKernelGGL(K<16>::fn(), grid(16), dim3(kBlock), 0, s, p); break;
    case 32: hipLaunchKernelGGL(K<32>::fn(), grid(32), dim3(kBlock), 0, s, p); break;
    case 64: hipLaunchKernelGGL(K<64>::fn(), grid(64), dim3(kBlock), 0, s, p); break;
    case 128: hipLaunchKernelGGL(K<128>::fn(), grid(128), dim3(kBlock), 0, s, p); break;
    default: hipLaunchKernelGGL(K<256>::fn(), grid(256), dim3(kBlock), 0, s, p); break;
  }
  return GNNREC_OK;
}

template <int F> struct FwdK { static auto fn() { return gat_train_fwd_kernel<F>; } };
template <int F> struct RowsK { static auto fn() { return gat_train_bwd_rows_kernel<F>; } };
template <int F> struct ColsK { static auto fn() { return gat_train_bwd_cols_kernel<F>; } };

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_gat_train_forward_f32(const int64_t* row_ptr, const int32_t* col,
                                            int64_t n_rows, const float* h, int64_t ldh,
                                            const float* s_self, const float* s_neigh, int64_t ld_s,
                                            int32_t heads, int32_t o_dim, float slope,
                                            float drop_p, uint32_t seed, float* out, int64_t ldo,
                                            gnnrec_stream_t stream) {
  GatTrain p{row_ptr, col, n_rows, h, ldh, s_self, s_neigh, ld_s, heads, o_dim, slope, drop_p,
             seed, out, ldo, nullptr, 0, nullptr, nullptr, 0, nullptr, nullptr};
  if (int st = check_train(p, false)) return st;
  if (n_rows == 0) return GNNREC_OK;
  launch_f<FwdK>(p, as_hip(stream));
  return check_launch("gat_train_forward");
}

extern "C" int gnnrec_gat_train_backward_f32(const int64_t* row_ptr, const int32_t* col,
                                             int64_t n_rows, const float* h, int64_t ldh,
                                             const float* s_self, const float* s_neigh,
                                             int64_t ld_s, int32_t heads, int32_t o_dim,
                                             float slope, float drop_p, uint32_t seed,
                                             const float* out, int64_t ldo, const float* dout,
                                             int64_t lddo, float* stats, float* dh, int64_t lddh,
                                             float* d_self, float* d_neigh,
                                             gnnrec_stream_t stream) {
  GatTrain p{row_ptr, col, n_rows, h, ldh, s_self, s_neigh, ld_s, heads, o_dim, slope, drop_p,
             seed, const_cast<float*>(out), ldo, dout, lddo, stats, dh, lddh, d_self, d_neigh};
  if (int st = check_train(p, true)) return st;
  if (n_rows == 0) return GNNREC_OK;
  hipStream_t s = as_hip(stream);
  launch_f<RowsK>(p, s);
  if (int st = check_launch("gat_train_backward (rows)")) return st;
  launch_f<ColsK>(p, s);
  return check_launch("gat_train_backward (columns)");
}
