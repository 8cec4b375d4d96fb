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
  int64_t max_row_len; // rows longer than this run the split path (0: none)
  int stats_in;        // backward: stats' (max, sum) come from the forward (no recount pass)
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

// Rows longer than GatTrain::max_row_len (power-law hubs: one of config 5's rows has 4e5
// neighbours, which one lane group would walk serially, 2.4 s per training step on the 2M x 2M
// slice) are left to the split path: their edges are cut into segments (CsrGraph.heavy_plan),
// each segment's partial sums computed by one lane group, then merged per row in segment order
// (deterministic). The same row-range device functions serve both paths.
struct TrainSplit {
  const int64_t* seg_row;
  const int64_t* seg_beg;
  const int64_t* seg_end;
  int64_t n_seg;
  const int64_t* heavy_rows;
  const int64_t* heavy_seg_ptr;   // [n_heavy + 1]: segments of heavy row i, row-grouped
  int64_t n_heavy;
  float* work;                    // n_seg * (F + 2 heads) floats
};

template <int F>
struct Lanes {                     // a lane's row group / head / feature offset
  static constexpr int GROUP = F / 4;
  static constexpr int RPW = 64 / GROUP;
  int gl, head, fo;
  int64_t item;                    // row (or segment, or heavy-row index) of the lane group
  __device__ Lanes(int o_dim) {
    const int lane = threadIdx.x & 63;
    gl = lane % GROUP;
    const int hl = o_dim / 4;
    head = gl / hl;
    fo = 4 * (gl - head * hl);
    item = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * RPW + lane / GROUP;
  }
};

__device__ __forceinline__ bool is_heavy(const GatTrain& p, int64_t beg, int64_t end) {
  return p.max_row_len > 0 && end - beg > p.max_row_len;
}

// Forward over the edges [beg, end) of row r (one head's lanes): online max / sum in base 2 over
// blocks of kTrainChunk neighbours; the sum of the weights (softmax denominator) takes every
// neighbour, the weighted row sum only the kept ones, scaled.
__device__ __forceinline__ void fwd_range(const GatTrain& p, int64_t r, int64_t beg, int64_t end,
                                          int head, int fo, float& m, float& l, float4& a) {
  const float ss = p.s_self[r * p.ld_s + head];
  m = -INFINITY;
  l = 0.f;
  a = make_float4(0.f, 0.f, 0.f, 0.f);
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
}

__device__ __forceinline__ void store_stats(const GatTrain& p, int64_t r, int head, float m,
                                            float l) {
  float* st = p.stats + (r * p.heads + head) * 4;
  st[0] = m;
  st[1] = l;
}

template <int F>
__global__ __launch_bounds__(kBlock) void gat_train_fwd_kernel(GatTrain p) {
  const Lanes<F> L(p.o_dim);
  const int64_t r = L.item;
  if (r >= p.n_rows) return;
  const int64_t beg = p.row_ptr[r], end = p.row_ptr[r + 1];
  if (is_heavy(p, beg, end)) return;   // the split path's
  float m, l;
  float4 a;
  fwd_range(p, r, beg, end, L.head, L.fo, m, l, a);
  // an empty row: 0 / 0 = NaN, like the reference's all -inf softmax row
  st4(p.out + r * p.ldo + L.head * p.o_dim + L.fo, make_float4(a.x / l, a.y / l, a.z / l, a.w / l));
  if (p.stats && L.fo == 0) store_stats(p, r, L.head, m, l);
}

// heavy rows, forward pass 1: a segment's (m, l, sum_j w_j h_j) -> work
template <int F>
__global__ __launch_bounds__(kBlock) void gat_train_fwd_part_kernel(GatTrain p, TrainSplit sp) {
  const Lanes<F> L(p.o_dim);
  const int64_t s = L.item;
  if (s >= sp.n_seg) return;
  float m, l;
  float4 a;
  fwd_range(p, sp.seg_row[s], sp.seg_beg[s], sp.seg_end[s], L.head, L.fo, m, l, a);
  st4(sp.work + s * F + L.head * p.o_dim + L.fo, a);
  if (L.fo == 0) {
    float* ml = sp.work + sp.n_seg * F + (s * p.heads + L.head) * 2;
    ml[0] = m;
    ml[1] = l;
  }
}

// heavy rows, forward pass 2: merge the row's segments in order (max-rescaled), normalise
template <int F>
__global__ __launch_bounds__(kBlock) void gat_train_fwd_merge_kernel(GatTrain p, TrainSplit sp) {
  const Lanes<F> L(p.o_dim);
  const int64_t i = L.item;
  if (i >= sp.n_heavy) return;
  const int64_t r = sp.heavy_rows[i], s0 = sp.heavy_seg_ptr[i], s1 = sp.heavy_seg_ptr[i + 1];
  const float* ml = sp.work + sp.n_seg * F;
  float M = -INFINITY;
  for (int64_t s = s0; s < s1; ++s) M = fmaxf(M, ml[(s * p.heads + L.head) * 2]);
  float l = 0.f;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t s = s0; s < s1; ++s) {
    const float w = __builtin_amdgcn_exp2f(ml[(s * p.heads + L.head) * 2] - M);
    l = __builtin_fmaf(w, ml[(s * p.heads + L.head) * 2 + 1], l);
    a = fma4(w, ld4(sp.work + s * F + L.head * p.o_dim + L.fo), a);
  }
  st4(p.out + r * p.ldo + L.head * p.o_dim + L.fo, make_float4(a.x / l, a.y / l, a.z / l, a.w / l));
  if (p.stats && L.fo == 0) store_stats(p, r, L.head, M, l);
}

// Backward, row pass over the edges [beg, end) of row r: sum_j dz_rj (the d s_self part).
template <int GROUP>
__device__ __forceinline__ float rows_dss(const GatTrain& p, int64_t r, int64_t beg, int64_t end,
                                          int head, int fo, int hl, float m, float inv_l,
                                          float c, const float4& g) {
  const float ss = p.s_self[r * p.ld_s + head];
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
  return dss;
}

// c_r = g_r . out_r for one head (every lane of the head gets it) and the lane's g_r slice
template <int GROUP>
__device__ __forceinline__ float row_c(const GatTrain& p, int64_t r, int head, int fo, int hl,
                                       float4& g) {
  g = ld4(p.dout + r * p.lddo + head * p.o_dim + fo);
  return head_sum<GROUP>(dot4t(g, ld4(p.out + r * p.ldo + head * p.o_dim + fo)), hl);
}

// Backward, row pass: softmax statistics (from the forward's when stats_in, else recomputed),
// c_r = g_r . out_r and d s_self[r].
template <int F>
__global__ __launch_bounds__(kBlock) void gat_train_bwd_rows_kernel(GatTrain p) {
  constexpr int GROUP = F / 4;
  const Lanes<F> L(p.o_dim);
  const int64_t r = L.item;
  if (r >= p.n_rows) return;
  const int hl = p.o_dim / 4, head = L.head, fo = L.fo;
  const int64_t beg = p.row_ptr[r], end = p.row_ptr[r + 1];
  if (is_heavy(p, beg, end)) return;
  float m, l;
  if (p.stats_in) {
    const float* st = p.stats + (r * p.heads + head) * 4;
    m = st[0];
    l = st[1];
  } else {
    // pass 1: max and sum of the base-2 logits
    const float ss = p.s_self[r * p.ld_s + head];
    m = -INFINITY;
    l = 0.f;
    for (int64_t k = beg; k < end; ++k) {
      const float e = logit2(ss + p.s_neigh[(int64_t)p.col[k] * p.ld_s + head], p.slope);
      const float mn = fmaxf(m, e);
      l = l * __builtin_amdgcn_exp2f(m - mn) + __builtin_amdgcn_exp2f(e - mn);
      m = mn;
    }
  }
  float4 g;
  const float c = row_c<GROUP>(p, r, head, fo, hl, g);
  const float dss = rows_dss<GROUP>(p, r, beg, end, head, fo, hl, m, 1.f / l, c, g);
  if (fo == 0) {
    p.d_self[r * p.heads + head] = end > beg ? dss : 0.f;
    float* st = p.stats + (r * p.heads + head) * 4;
    st[0] = m;
    st[1] = l;
    st[2] = c;
    st[3] = 0.f;
  }
}

// heavy rows, backward row pass 1: a segment's partial d s_self (statistics from the forward)
template <int F>
__global__ __launch_bounds__(kBlock) void gat_train_bwd_rows_part_kernel(GatTrain p, TrainSplit sp) {
  constexpr int GROUP = F / 4;
  const Lanes<F> L(p.o_dim);
  const int64_t s = L.item;
  if (s >= sp.n_seg) return;
  const int hl = p.o_dim / 4;
  const int64_t r = sp.seg_row[s];
  const float* st = p.stats + (r * p.heads + L.head) * 4;
  float4 g;
  const float c = row_c<GROUP>(p, r, L.head, L.fo, hl, g);
  const float dss = rows_dss<GROUP>(p, r, sp.seg_beg[s], sp.seg_end[s], L.head, L.fo, hl, st[0],
                                    1.f / st[1], c, g);
  if (L.fo == 0) sp.work[s * p.heads + L.head] = dss;
}

// heavy rows, backward row pass 2: the row's partials summed in segment order, c_r
template <int F>
__global__ __launch_bounds__(kBlock) void gat_train_bwd_rows_merge_kernel(GatTrain p, TrainSplit sp) {
  constexpr int GROUP = F / 4;
  const Lanes<F> L(p.o_dim);
  const int64_t i = L.item;
  if (i >= sp.n_heavy) return;
  const int hl = p.o_dim / 4;
  const int64_t r = sp.heavy_rows[i];
  float4 g;
  const float c = row_c<GROUP>(p, r, L.head, L.fo, hl, g);
  float dss = 0.f;
  for (int64_t s = sp.heavy_seg_ptr[i]; s < sp.heavy_seg_ptr[i + 1]; ++s)
    dss += sp.work[s * p.heads + L.head];
  if (L.fo == 0) {
    p.d_self[r * p.heads + L.head] = dss;
    float* st = p.stats + (r * p.heads + L.head) * 4;
    st[2] = c;
    st[3] = 0.f;
  }
}

// Backward, column pass over the edges [beg, end) of node j's row (the rows r that aggregate
// j, the pattern being symmetric): the partial d h_j and d s_neigh[j].
template <int GROUP>
__device__ __forceinline__ void cols_range(const GatTrain& p, int64_t j, int64_t beg, int64_t end,
                                           int head, int fo, int hl, float4& dh, float& dsn) {
  const float sn = p.s_neigh[j * p.ld_s + head];
  const float4 hj = ld4(p.h + j * p.ldh + head * p.o_dim + fo);
  dh = make_float4(0.f, 0.f, 0.f, 0.f);
  dsn = 0.f;
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
}

template <int F>
__global__ __launch_bounds__(kBlock) void gat_train_bwd_cols_kernel(GatTrain p) {
  constexpr int GROUP = F / 4;
  const Lanes<F> L(p.o_dim);
  const int64_t j = L.item;
  if (j >= p.n_rows) return;
  const int64_t beg = p.row_ptr[j], end = p.row_ptr[j + 1];
  if (is_heavy(p, beg, end)) return;
  float4 dh;
  float dsn;
  cols_range<GROUP>(p, j, beg, end, L.head, L.fo, p.o_dim / 4, dh, dsn);
  st4(p.dh + j * p.lddh + L.head * p.o_dim + L.fo, dh);
  if (L.fo == 0) p.d_neigh[j * p.heads + L.head] = dsn;
}

template <int F>
__global__ __launch_bounds__(kBlock) void gat_train_bwd_cols_part_kernel(GatTrain p, TrainSplit sp) {
  constexpr int GROUP = F / 4;
  const Lanes<F> L(p.o_dim);
  const int64_t s = L.item;
  if (s >= sp.n_seg) return;
  float4 dh;
  float dsn;
  cols_range<GROUP>(p, sp.seg_row[s], sp.seg_beg[s], sp.seg_end[s], L.head, L.fo, p.o_dim / 4, dh,
                    dsn);
  st4(sp.work + s * F + L.head * p.o_dim + L.fo, dh);
  if (L.fo == 0) sp.work[sp.n_seg * F + s * p.heads + L.head] = dsn;
}

template <int F>
__global__ __launch_bounds__(kBlock) void gat_train_bwd_cols_merge_kernel(GatTrain p, TrainSplit sp) {
  const Lanes<F> L(p.o_dim);
  const int64_t i = L.item;
  if (i >= sp.n_heavy) return;
  const int64_t j = sp.heavy_rows[i];
  float4 dh = make_float4(0.f, 0.f, 0.f, 0.f);
  float dsn = 0.f;
  for (int64_t s = sp.heavy_seg_ptr[i]; s < sp.heavy_seg_ptr[i + 1]; ++s) {
    const float4 v = ld4(sp.work + s * F + L.head * p.o_dim + L.fo);
    dh = make_float4(dh.x + v.x, dh.y + v.y, dh.z + v.z, dh.w + v.w);
    dsn += sp.work[sp.n_seg * F + s * p.heads + L.head];
  }
  st4(p.dh + j * p.lddh + L.head * p.o_dim + L.fo, dh);
  if (L.fo == 0) p.d_neigh[j * p.heads + L.head] = dsn;
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

// grid of lane groups over `items` (rows, segments or heavy rows) for width F
inline dim3 grid_for(int64_t items, int F) {
  return dim3((unsigned)ceil_div(items, (64 / (F / 4)) * (kBlock / 64)));
}

#define GNNREC_GAT_TRAIN_LAUNCH(KERNEL, ITEMS, ...)                                               \
  do {                                                                                          \
    const int F_ = p.heads * p.o_dim;                                                           \
    switch (F_) {                                                                               \
      case 16: hipLaunchKernelGGL(KERNEL<16>, grid_for(ITEMS, 16), dim3(kBlock), 0, s, __VA_ARGS__); break;  \
      case 32: hipLaunchKernelGGL(KERNEL<32>, grid_for(ITEMS, 32), dim3(kBlock), 0, s, __VA_ARGS__); break;  \
      case 64: hipLaunchKernelGGL(KERNEL<64>, grid_for(ITEMS, 64), dim3(kBlock), 0, s, __VA_ARGS__); break;  \
      case 128: hipLaunchKernelGGL(KERNEL<128>, grid_for(ITEMS, 128), dim3(kBlock), 0, s, __VA_ARGS__); break; \
      default: hipLaunchKernelGGL(KERNEL<256>, grid_for(ITEMS, 256), dim3(kBlock), 0, s, __VA_ARGS__); break; \
    }                                                                                           \
  } while (0)

int check_split(const GatTrain& p, const TrainSplit& sp) {
  GNNREC_REQUIRE(p.max_row_len >= 0 && sp.n_seg >= 0 && sp.n_heavy >= 0,
                 "gat_train: negative max_row_len / n_seg / n_heavy");
  if (p.max_row_len > 0 && sp.n_heavy > 0)
    GNNREC_REQUIRE(sp.seg_row && sp.seg_beg && sp.seg_end && sp.heavy_rows && sp.heavy_seg_ptr &&
                       sp.work && aligned16(sp.work) && sp.n_seg >= sp.n_heavy,
                   "gat_train: the split path needs the segment plan and a 16-B aligned work "
                   "buffer of n_seg * (heads * o_dim + 2 heads) floats");
  return GNNREC_OK;
}

int train_forward(const GatTrain& p, const TrainSplit& sp, hipStream_t s) {
  GNNREC_GAT_TRAIN_LAUNCH(gat_train_fwd_kernel, p.n_rows, p);
  if (int st = check_launch("gat_train_forward")) return st;
  if (p.max_row_len > 0 && sp.n_heavy > 0) {
    GNNREC_GAT_TRAIN_LAUNCH(gat_train_fwd_part_kernel, sp.n_seg, p, sp);
    if (int st = check_launch("gat_train_forward (segments)")) return st;
    GNNREC_GAT_TRAIN_LAUNCH(gat_train_fwd_merge_kernel, sp.n_heavy, p, sp);
    return check_launch("gat_train_forward (merge)");
  }
  return GNNREC_OK;
}

int train_backward(const GatTrain& p, const TrainSplit& sp, hipStream_t s) {
  const bool split = p.max_row_len > 0 && sp.n_heavy > 0;
  GNNREC_GAT_TRAIN_LAUNCH(gat_train_bwd_rows_kernel, p.n_rows, p);
  if (int st = check_launch("gat_train_backward (rows)")) return st;
  if (split) {
    GNNREC_GAT_TRAIN_LAUNCH(gat_train_bwd_rows_part_kernel, sp.n_seg, p, sp);
    if (int st = check_launch("gat_train_backward (row segments)")) return st;
    GNNREC_GAT_TRAIN_LAUNCH(gat_train_bwd_rows_merge_kernel, sp.n_heavy, p, sp);
    if (int st = check_launch("gat_train_backward (row merge)")) return st;
  }
  GNNREC_GAT_TRAIN_LAUNCH(gat_train_bwd_cols_kernel, p.n_rows, p);
  if (int st = check_launch("gat_train_backward (columns)")) return st;
  if (split) {
    GNNREC_GAT_TRAIN_LAUNCH(gat_train_bwd_cols_part_kernel, sp.n_seg, p, sp);
    if (int st = check_launch("gat_train_backward (column segments)")) return st;
    GNNREC_GAT_TRAIN_LAUNCH(gat_train_bwd_cols_merge_kernel, sp.n_heavy, p, sp);
    return check_launch("gat_train_backward (column merge)");
  }
  return GNNREC_OK;
}

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_gat_train_forward_split_f32(
    const int64_t* row_ptr, const int32_t* col, int64_t n_rows, const float* h, int64_t ldh,
    const float* s_self, const float* s_neigh, int64_t ld_s, int32_t heads, int32_t o_dim,
    float slope, float drop_p, uint32_t seed, float* out, int64_t ldo, float* stats,
    int64_t max_row_len, const int64_t* seg_row, const int64_t* seg_beg, const int64_t* seg_end,
    int64_t n_seg, const int64_t* heavy_rows, const int64_t* heavy_seg_ptr, int64_t n_heavy,
    float* work, gnnrec_stream_t stream) {
  GatTrain p{row_ptr, col, n_rows, h, ldh, s_self, s_neigh, ld_s, heads, o_dim, slope, drop_p,
             seed, out, ldo, nullptr, 0, stats, nullptr, 0, nullptr, nullptr, max_row_len, 0};
  const TrainSplit sp{seg_row, seg_beg, seg_end, n_seg, heavy_rows, heavy_seg_ptr, n_heavy, work};
  if (int st = check_train(p, false)) return st;
  if (int st = check_split(p, sp)) return st;
  GNNREC_REQUIRE(!stats || aligned16(stats), "gat_train_forward: stats must be 16-B aligned");
  if (n_rows == 0) return GNNREC_OK;
  return train_forward(p, sp, as_hip(stream));
}

extern "C" int gnnrec_gat_train_forward_f32(const int64_t* row_ptr, const int32_t* col,
                                            int64_t n_rows, const float* h, int64_t ldh,
                                            const float* s_self, const float* s_neigh, int64_t ld_s,
                                            int32_t heads, int32_t o_dim, float slope,
                                            float drop_p, uint32_t seed, float* out, int64_t ldo,
                                            gnnrec_stream_t stream) {
  return gnnrec_gat_train_forward_split_f32(row_ptr, col, n_rows, h, ldh, s_self, s_neigh, ld_s,
                                            heads, o_dim, slope, drop_p, seed, out, ldo, nullptr,
                                            0, nullptr, nullptr, nullptr, 0, nullptr, nullptr, 0,
                                            nullptr, stream);
}

extern "C" int gnnrec_gat_train_backward_split_f32(
    const int64_t* row_ptr, const int32_t* col, int64_t n_rows, const float* h, int64_t ldh,
    const float* s_self, const float* s_neigh, int64_t ld_s, int32_t heads, int32_t o_dim,
    float slope, float drop_p, uint32_t seed, const float* out, int64_t ldo, const float* dout,
    int64_t lddo, float* stats, float* dh, int64_t lddh, float* d_self, float* d_neigh,
    int64_t max_row_len, const int64_t* seg_row, const int64_t* seg_beg, const int64_t* seg_end,
    int64_t n_seg, const int64_t* heavy_rows, const int64_t* heavy_seg_ptr, int64_t n_heavy,
    float* work, gnnrec_stream_t stream) {
  GatTrain p{row_ptr, col, n_rows, h, ldh, s_self, s_neigh, ld_s, heads, o_dim, slope, drop_p,
             seed, const_cast<float*>(out), ldo, dout, lddo, stats, dh, lddh, d_self, d_neigh,
             max_row_len, 1};
  const TrainSplit sp{seg_row, seg_beg, seg_end, n_seg, heavy_rows, heavy_seg_ptr, n_heavy, work};
  if (int st = check_train(p, true)) return st;
  if (int st = check_split(p, sp)) return st;
  if (n_rows == 0) return GNNREC_OK;
  return train_backward(p, sp, as_hip(stream));
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
             seed, const_cast<float*>(out), ldo, dout, lddo, stats, dh, lddh, d_self, d_neigh, 0,
             0};
  const TrainSplit sp{nullptr, nullptr, nullptr, 0, nullptr, nullptr, 0, nullptr};
  if (int st = check_train(p, true)) return st;
  if (n_rows == 0) return GNNREC_OK;
  return train_backward(p, sp, as_hip(stream));
}
