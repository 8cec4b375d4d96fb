// GAT sparse edge-softmax aggregation (BASELINE config 5), gfx950.
//
// Replaces GATLayer.forward's dense path (baselines/gat.py:99-149): the reference builds an
// [N, N] score matrix per head, masks non-edges with -inf, row-softmaxes and multiplies by
// h — O(N^2) memory, infeasible past N ~ 2e4. Here each destination row walks its CSR
// neighbours once: e_j = LeakyReLU(s_self[r,h] + s_neigh[j,h]) with an online max / sum
// (flash-style rescaling), accumulating p_j * h[j] for every head at the same time.
// Row mapping as the SpMM (gather.h): F = heads*o_dim features per row, GROUP = F/4 lanes
// per row, 4 features (one head) per lane; a neighbour costs one F*4-byte row gather plus
// one 4-byte score gather per lane. With head_stride = 0 every head aggregates the same
// o_dim-wide row (the layer input x itself): the last, head-averaged layer then gathers x
// once per neighbour instead of the 4x wider h, and W_h is applied after the aggregation
// (sum_j a_hj W_h x_j = W_h sum_j a_hj x_j).
// Fused epilogue: mean over heads (last layer, gat.py:149), F.elu (gat.py:283) and the
// layer-mean accumulator (gat.py:287-288, GNNREC_EPI_* flags).
#include <math.h>

#include <type_traits>
#include <utility>

#include "gather.h"

namespace gnnrec {

struct GatParams {
  Csr A;
  const float* h;
  int64_t ldh;
  int64_t head_stride;  // h[j] of head q starts at h + j*ldh + q*head_stride (o_dim: [N, H*o]
                        // head-major; 0: every head reads the same o_dim-wide row)
  const float* s_self;
  const float* s_neigh;
  int64_t ld_ss, ld_sn;  // row strides of s_self / s_neigh (>= heads)
  int heads, o_dim;
  float slope;
  int mean_heads, apply_elu;
  float* out;
  int64_t ldo;
  int epi;
  const float* self;
  int64_t ld_self;
  float* acc;
  int64_t ld_acc;
  float acc_div;
  int64_t max_row_len;  // rows longer than this are left to the split path (0: none)
  // attention vectors (ATT kernels): att[0][h][o_dim] (self), att[1][h][o_dim] (neighbour):
  // s_self[r, h] = att[0][h] . row_r,h and s_neigh[j, h] = att[1][h] . row_j,h from the rows
  // the kernel reads anyway (s_self / s_neigh / ld_* unused)
  const float* att;
  const float* hself;   // ATT: destination row r's own row (hself + r * ld_hself, head_stride)
  int64_t ld_hself;
};

// Softmax normalisation a / l of one head's features: one correctly rounded reciprocal, then
// products — an IEEE division per feature cost ~10 instructions each, 160 per row in the
// shared-row kernel (4 heads x 4 features per lane). Within an ulp of a / l (fp32 tolerance,
// as the reference's own softmax); every kernel normalises through here, so the head-major,
// shared-row and heavy-row paths keep equal bits. l = 0 (an empty row): 0 * inf = NaN, as 0 / 0.
__device__ __forceinline__ float4 gat_norm(const float4& a, float l) {
  const float r = 1.f / l;
  return make_float4(a.x * r, a.y * r, a.z * r, a.w * r);
}

// Softmax normalisation + head mean + ELU + store + layer-mean epilogue of one row.
template <int GROUP>
__device__ __forceinline__ void gat_finish(const GatParams& p, int64_t r, float4 o, int gl) {
  const int hl = p.o_dim / 4;
  int owner_lanes = GROUP;
  if (p.mean_heads) {  // mean over heads: lanes fg, fg+hl, ... hold the same features
    const int fg = gl % hl;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int q = 0; q < p.heads; ++q) {
      const int src = fg + q * hl;
      const float4 t = make_float4(__shfl(o.x, src, GROUP), __shfl(o.y, src, GROUP),
                                   __shfl(o.z, src, GROUP), __shfl(o.w, src, GROUP));
      s = q == 0 ? t : make_float4(s.x + t.x, s.y + t.y, s.z + t.z, s.w + t.w);
    }
    const float H = (float)p.heads;
    o = make_float4(s.x / H, s.y / H, s.z / H, s.w / H);
    owner_lanes = hl;
  }
  if (gl >= owner_lanes) return;
  if (p.apply_elu) {
    o.x = o.x > 0.f ? o.x : expm1f(o.x);
    o.y = o.y > 0.f ? o.y : expm1f(o.y);
    o.z = o.z > 0.f ? o.z : expm1f(o.z);
    o.w = o.w > 0.f ? o.w : expm1f(o.w);
  }
  if (!(p.epi & GNNREC_EPI_NO_Y)) st4(p.out + r * p.ldo + 4 * gl, o);
  acc_epilogue(p.epi, o, p.self + r * p.ld_self + 4 * gl, p.acc + r * p.ld_acc + 4 * gl, p.acc_div);
}

// Online softmax in blocks of kSoftBlock neighbours, base 2: E_j = LeakyReLU(s_self + s_neigh[j])
// * log2(e); per block the running max moves once (m' = max(m, max_j E_j)), the sums are
// rescaled once by 2^(m - m'), and each neighbour costs ONE v_exp_f32 (2^(E_j - m')) and its
// fmaf. softmax = sum_j 2^(E_j - m) h_j / sum_j 2^(E_j - m) is the reference's
// exp(e_j - max) / sum (gat.py:135-141) reassociated — fp32 tolerance, as the reference's
// own dense softmax. Neighbours past the row end get E = -inf (p = 0: the sums are unchanged,
// no branch). Every kernel below uses the same blocks from the row's (or segment's) first
// neighbour, so the shared-row and the head-major kernels agree bit for bit.
// The ATT kernels keep the score dots in registers: cap them at 128 VGPRs, 4 waves per SIMD
// like the score-table kernels (uncapped they take 132-176 and drop to 2-3 waves)
#ifndef GAT_ATT_WAVES
#define GAT_ATT_WAVES 4
#endif
#ifndef GAT_ATT_CHUNK
#define GAT_ATT_CHUNK 16
#endif
// a neighbour row's float4 (plain policy: non-temporal cold-row gathers were measured slower in
// every form)
__device__ __forceinline__ float4 ld4_src(const float* p, int) { return ld4(p); }
#ifndef GAT_MAIN_PIPE
#define GAT_MAIN_PIPE 0
#endif
#define GAT_OCCUPANCY(ATT) __attribute__((amdgpu_waves_per_eu((ATT) ? GAT_ATT_WAVES : 1)))
#ifndef GAT_SHARED_WAVES
#define GAT_SHARED_WAVES GAT_ATT_WAVES
#endif
#define GAT_SHARED_OCCUPANCY(ATT) __attribute__((amdgpu_waves_per_eu((ATT) ? GAT_SHARED_WAVES : 1)))

constexpr int kSoftBlock = 8;
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ float gat_exp2(float v) { return __builtin_amdgcn_exp2f(v); }

__device__ __forceinline__ float gat_logit2(float ss, float sn, float slope, bool valid) {
  float e = ss + sn;
  e = e > 0.f ? e : e * slope;
  return valid ? e * kLog2e : -INFINITY;
}

// ---- scores from the gathered rows (ATT kernels) -------------------------------------------
// s_neigh[j, h] = a_h . row_j,h is a dot product of a row the kernel gathers for the weighted
// sum anyway, so it is formed in registers instead of gathered: 2 instead of 3 128-B lines per
// neighbour of a 256-B row (the score table's line was a third random request per edge). The
// dot of a head spans its hl = o_dim / 4 lanes (4 features each); the lane sums reduce with DPP
// moves inside the aligned hl-lane group, in an order that gives every lane the same bits.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               CTRL, 0xF, 0xF, false));
}
constexpr int kDppRowMirror = 0x140, kDppHalfMirror = 0x141, kDppXor2 = 0x4E, kDppXor1 = 0xB1,
              kDppRor8 = 0x128;

// sum over the aligned group of HL lanes (HL in {1, 2, 4, 8, 16}), in every lane of it
template <int HL>
__device__ __forceinline__ float group_sum(float v) {
  static_assert(HL >= 1 && HL <= 16 && (HL & (HL - 1)) == 0, "group of 1..16 lanes");
  if constexpr (HL >= 16) v += dpp_f<kDppRowMirror>(v);   // lane i + lane 15 - i
  if constexpr (HL >= 8) v += dpp_f<kDppHalfMirror>(v);   // lane i + lane 7 - i (8-lane halves)
  if constexpr (HL >= 4) v += dpp_f<kDppXor2>(v);
  if constexpr (HL >= 2) v += dpp_f<kDppXor1>(v);
  return v;
}

__device__ __forceinline__ float dot4(const float4& a, const float4& b) {
  return __builtin_fmaf(a.w, b.w, __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x)));
}

// One softmax block of one head: logits E[0..kSoftBlock), rows xv[0..kSoftBlock).
__device__ __forceinline__ void gat_block(const float (&E)[kSoftBlock], const float4* xv,
                                          float& m, float& l, float4& a) {
  float bm = E[0];
#pragma unroll
  for (int t = 1; t < kSoftBlock; ++t) bm = fmaxf(bm, E[t]);
  const float mn = fmaxf(m, bm);
  const float sc = gat_exp2(m - mn);   // m = -inf on the first block: sc = 0
  l *= sc;
  a = make_float4(a.x * sc, a.y * sc, a.z * sc, a.w * sc);
#pragma unroll
  for (int t = 0; t < kSoftBlock; ++t) {
    const float pe = gat_exp2(E[t] - mn);
    l += pe;
    a = fma4(pe, xv[t], a);
  }
  m = mn;
}

// Row c of a table: base + c * ld floats as ONE v_mad_u64_u32 (c >= 0, ld * 4 < 2^32): the
// int64 product took 5 VALU instructions per gathered row (sign extension, two 32-bit
// multiplies, a 64-bit multiply-add, an add) before its pointer add
__device__ __forceinline__ const float* row_at(const float* base, int c, uint32_t ld_bytes) {
  return reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) +
                                        (uint64_t)(uint32_t)c * ld_bytes);
}

// Lane T of each 16-lane DPP row to every lane of the row (row_newbcast): a neighbour's column
// index to its row group without an LDS permute (__shfl compiles to ds_bpermute, and the 16
// of them sat between the index load and the row gathers, each behind an LDS wait)
template <int T>
__device__ __forceinline__ int row_bcast_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x150 + T, 0xF, 0xF, true);
}
template <int... T>
__device__ __forceinline__ void bcast_cols16(std::integer_sequence<int, T...>, int cm,
                                             int (&c)[sizeof...(T)]) {
  ((c[T] = row_bcast_i<T % 16>(cm)), ...);
}
// rows cm@lane T (T < 16) of a 16-lane row group: one float4 per lane each. The index moves by
// __shfl here: the DPP form held the 8 indices in registers and pushed the 128-VGPR shared-row
// kernels from 2 to 10 spilled registers
template <int... T>
__device__ __forceinline__ void gather_rows16(std::integer_sequence<int, T...>, int cm,
                                              const float* base, uint32_t ld_bytes,
                                              float4 (&dst)[sizeof...(T)]) {
  ((dst[T] = ld4(row_at(base, __shfl(cm, T, 16), ld_bytes))), ...);
}

// Online-softmax accumulation of neighbours [beg, end) of row r (head of this lane); m is in
// the base-2 logit domain.
// HL: lanes per head (o_dim / 4) as a compile-time constant for the ATT kernels (0: runtime)
template <int GROUP, bool ATT, int HL = 0>
__device__ __forceinline__ void gat_accumulate(const GatParams& p, int64_t r, int64_t beg,
                                               int64_t end, int gl, float& m, float& l,
                                               float4& a) {
  static_assert(kChunk % kSoftBlock == 0, "a gather step holds whole softmax blocks");
  static_assert(!ATT || (HL >= 1 && HL <= GROUP), "ATT needs the lanes per head");
  const int hl = HL > 0 ? HL : p.o_dim / 4;
  const int head = gl / hl;
  const int fo = 4 * (gl - head * hl);   // this lane's features of its head's row
  float ss;
  float4 an = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (ATT) {
    const float4 as = ld4(p.att + head * p.o_dim + fo);
    an = ld4(p.att + (p.heads + head) * p.o_dim + fo);
    ss = group_sum<(HL > 0 ? HL : 1)>(dot4(ld4(p.hself + r * p.ld_hself + head * p.head_stride + fo), as));
  } else {
    ss = p.s_self[r * p.ld_ss + head];
  }
  // neighbours per gather step: the score-table kernels keep kChunk rows in flight per lane;
  // the ATT kernels hold each row until its score is reduced, so they gather GAT_ATT_CHUNK at
  // a time and win the occupancy back
  constexpr int CH = ATT ? GAT_ATT_CHUNK : kChunk;
  static_assert(CH % kSoftBlock == 0, "a gather step holds whole softmax blocks");
  constexpr int PER = (GROUP >= CH) ? 1 : CH / GROUP;
  auto load_chunk = [&](int64_t k0, float4 (&dst)[CH], float (&snd)[CH]) {
    int cm[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      int64_t k = k0 + gl + (int64_t)q * GROUP;
      k = k < end ? k : end - 1;
      cm[q] = p.A.col[k];
    }
    int cs[CH];
    if constexpr (GROUP == 16 && PER == 1) {
      bcast_cols16(std::make_integer_sequence<int, CH>{}, cm[0], cs);
    } else {
#pragma unroll
      for (int t = 0; t < CH; ++t) cs[t] = __shfl(cm[t / GROUP < PER ? t / GROUP : 0], t % GROUP, GROUP);
    }
    const float* hb = p.h + head * p.head_stride + fo;
    const uint32_t ldb = (uint32_t)(p.ldh * 4);
#pragma unroll
    for (int t = 0; t < CH; ++t) {
      const int c = cs[t];
      dst[t] = ld4_src(row_at(hb, c, ldb), c);
      if constexpr (!ATT) snd[t] = p.s_neigh[(int64_t)c * p.ld_sn + head];
    }
  };
  // ATT + GAT_MAIN_PIPE: the next chunk's rows are in flight while this chunk is reduced
  constexpr bool kPipe = ATT && GAT_MAIN_PIPE;
  float4 xv[CH];
  float sn[CH];
  if constexpr (kPipe) load_chunk(beg, xv, sn);
  for (int64_t k0 = beg; k0 < end; k0 += CH) {
    float4 xn[CH];
    float snn[CH];
    if constexpr (kPipe) {
      if (k0 + CH < end) load_chunk(k0 + CH, xn, snn);
    } else {
      load_chunk(k0, xv, sn);
    }
    if constexpr (ATT) {
#pragma unroll
      for (int t = 0; t < CH; ++t) sn[t] = group_sum<(HL > 0 ? HL : 1)>(dot4(xv[t], an));
    }
#pragma unroll
    for (int b = 0; b < CH / kSoftBlock; ++b) {
      if (k0 + b * kSoftBlock >= end) break;
      float E[kSoftBlock];
#pragma unroll
      for (int t = 0; t < kSoftBlock; ++t)
        E[t] = gat_logit2(ss, sn[b * kSoftBlock + t], p.slope, k0 + b * kSoftBlock + t < end);
      gat_block(E, xv + b * kSoftBlock, m, l, a);
    }
    if constexpr (kPipe) {
#pragma unroll
      for (int t = 0; t < CH; ++t) xv[t] = xn[t];
    }
  }
}

template <int F, bool ATT, int HL = 0>
__global__ __launch_bounds__(kBlock) GAT_OCCUPANCY(ATT) void gat_kernel(GatParams p) {
  constexpr int GROUP = F / 4;
  constexpr int RPW = 64 / GROUP;
  const int lane = threadIdx.x & 63;
  const int gl = lane % GROUP;
  const int64_t r = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * RPW + lane / GROUP;
  if (r >= p.A.n_rows) return;
  const int64_t beg = p.A.row_ptr[r], end = p.A.row_ptr[r + 1];
  if (p.max_row_len > 0 && end - beg > p.max_row_len) return;  // heavy row: split path
  float m = -INFINITY, l = 0.f;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  gat_accumulate<GROUP, ATT, HL>(p, r, beg, end, gl, m, l, a);
  // softmax normalisation (l = 0 for an empty row -> 0/0 = NaN, like the reference)
  gat_finish<GROUP>(p, r, gat_norm(a, l), gl);
}

template <int T>
__device__ __forceinline__ float row_bcast(float v) {   // DPP row_newbcast: lane T of each 16
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               0x150 + T, 0xF, 0xF, true));
}

// One block of 8 neighbours for a 16-lane row group with 4 heads: lane gl computes the logits
// and weights of ONE neighbour (gl & 7) for TWO heads (2 (gl >> 3), +1) instead of every lane
// computing all 32, and the weights reach the other lanes by DPP row broadcasts. Every value
// is produced by the same operations on the same inputs as gat_block's, and each lane applies
// them in gat_block's order, so the results are bit-identical to the generic path.
template <int... T>
__device__ __forceinline__ void gat_apply16(std::integer_sequence<int, T...>, float pa, float pb,
                                            const float4 (&xv)[8], float (&l)[4],
                                            float4 (&a)[4]) {
  // neighbour t = T: head 0/1 weights from lane t, head 2/3 weights from lane t + 8
  ((l[0] += row_bcast<T>(pa), a[0] = fma4(row_bcast<T>(pa), xv[T], a[0]),
    l[1] += row_bcast<T>(pb), a[1] = fma4(row_bcast<T>(pb), xv[T], a[1]),
    l[2] += row_bcast<T + 8>(pa), a[2] = fma4(row_bcast<T + 8>(pa), xv[T], a[2]),
    l[3] += row_bcast<T + 8>(pb), a[3] = fma4(row_bcast<T + 8>(pb), xv[T], a[3])), ...);
}

// ATT form of the shared-row scores: every lane holds 4 of the 64 features of the 8 neighbour
// rows, so s_neigh[t, h] = v_h . x_t is 16 lanes' partial dots; a reduce-scatter over the
// 16-lane row group (DPP: lanes L / L^8 exchange head pairs, then the 8-lane halves split the
// neighbours 4 / 2 / 1) leaves lane gl exactly the two sums it turns into logits below:
// neighbour gl & 7, heads 2 (gl >> 3) and 2 (gl >> 3) + 1.
#ifndef GAT_ATT_LDS
#define GAT_ATT_LDS 1
#endif
#ifndef GAT_SHARED_PIPE
#define GAT_SHARED_PIPE 0
#endif
// an: the 4 heads' neighbour vectors, this lane's float4 of each (registers: an[h]; LDS:
// an[h * 16 + gl])
template <class AN>
__device__ __forceinline__ float4 an_of(const AN& an, int h, int gl) {
  if constexpr (std::is_pointer_v<AN>) return an[h * 16 + gl];   // AN = float4[4]: no decay
  else return an[h];
}

template <class AN>
__device__ __forceinline__ void shared_scores16(const float4 (&xv)[8], const AN& an,
                                                int gl, float& sa, float& sb) {
  const bool hi = gl >= 8, b2 = gl & 4, b1 = gl & 2, b0 = gl & 1;
  float T[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {   // one head of each pair per pass: 16 partial dots live, not 32
    float Q[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float mine = dot4(xv[t], an_of(an, j, gl)), other = dot4(xv[t], an_of(an, 2 + j, gl));
      Q[t] = (hi ? other : mine) + dpp_f<kDppRor8>(hi ? mine : other);   // lanes L, L^8
    }
    float R[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)           // lanes t, 7 - t: neighbours 4 b2 + k
      R[k] = (b2 ? Q[4 + k] : Q[k]) + dpp_f<kDppHalfMirror>(b2 ? Q[k] : Q[4 + k]);
    float S[2];
#pragma unroll
    for (int k = 0; k < 2; ++k)           // lanes t, t^2: neighbours ... + 2 b1 + k
      S[k] = (b1 ? R[2 + k] : R[k]) + dpp_f<kDppXor2>(b1 ? R[k] : R[2 + k]);
    T[j] = (b0 ? S[1] : S[0]) + dpp_f<kDppXor1>(b0 ? S[0] : S[1]);   // lanes t, t^1: neighbour t
  }
  sa = T[0];   // neighbour gl & 7, head 2 hi
  sb = T[1];   // head 2 hi + 1
}

template <bool ATT>
__device__ __forceinline__ void gat_shared_rows16(const GatParams& p, int64_t r, int64_t beg,
                                                  int64_t end, int gl, const float (&ss)[4],
                                                  float (&m)[4], float (&l)[4],
                                                  float4 (&a)[4]) {
  const int tl = gl & 7;
  const bool hi = gl >= 8;                       // heads 2, 3 (else 0, 1)
  const float ssa = hi ? ss[2] : ss[0], ssb = hi ? ss[3] : ss[1];
#if GAT_ATT_LDS
  // the neighbour vectors parked in LDS instead of 16 VGPRs: every lane writes the 4 float4 it
  // reads back itself (all row groups write the same values), so no barrier is needed
  __shared__ float4 s_an[4 * 16];
  if constexpr (ATT) {
#pragma unroll
    for (int h = 0; h < 4; ++h) s_an[h * 16 + gl] = ld4(p.att + (4 + h) * 64 + 4 * gl);
  }
  const float4* an = s_an;
#else
  float4 an[4];
  if constexpr (ATT) {
#pragma unroll
    for (int h = 0; h < 4; ++h) an[h] = ld4(p.att + (4 + h) * 64 + 4 * gl);
  }
#endif
  auto load_block = [&](int64_t k0, float4 (&dst)[8]) {
    int64_t k = k0 + gl;
    k = k < end ? k : end - 1;
    const int cm = p.A.col[k];
    gather_rows16(std::make_integer_sequence<int, 8>{}, cm, p.h + 4 * gl, (uint32_t)(p.ldh * 4), dst);
  };
  // ATT + GAT_SHARED_PIPE: the next block's rows are in flight while this block's scores,
  // reduce-scatter and weighted sums run (the ATT form has twice the VALU work per
  // neighbour of the score-table form, so without it the loads wait behind the compute)
  constexpr bool kPipe = ATT && GAT_SHARED_PIPE;
  float4 xv[8];
  if constexpr (kPipe) load_block(beg, xv);
  for (int64_t k0 = beg; k0 < end; k0 += 8) {
    float4 xn[8];
    if constexpr (kPipe) {
      if (k0 + 8 < end) load_block(k0 + 8, xn);
    } else {
      load_block(k0, xv);
    }
    int cm = 0;
    if constexpr (!ATT) {
      int64_t k = k0 + gl;
      k = k < end ? k : end - 1;
      cm = p.A.col[k];
    }
    float sna, snb;
    if constexpr (ATT) {
      shared_scores16(xv, an, gl, sna, snb);
    } else {
      const int co = __shfl(cm, tl, 16);
      const float4 s4 = ld4(p.s_neigh + (int64_t)co * p.ld_sn);
      sna = hi ? s4.z : s4.x;
      snb = hi ? s4.w : s4.y;
    }
    const bool valid = k0 + tl < end;
    const float ea = gat_logit2(ssa, sna, p.slope, valid);
    const float eb = gat_logit2(ssb, snb, p.slope, valid);
    float ma = ea, mb = eb;   // block max per head over the 8 lanes of the half-row
#pragma unroll
    for (int d = 1; d < 8; d <<= 1) {
      ma = fmaxf(ma, __shfl_xor(ma, d, 8));
      mb = fmaxf(mb, __shfl_xor(mb, d, 8));
    }
    const float bm[4] = {row_bcast<0>(ma), row_bcast<0>(mb), row_bcast<8>(ma), row_bcast<8>(mb)};
    float mn[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      mn[h] = fmaxf(m[h], bm[h]);
      const float sc = gat_exp2(m[h] - mn[h]);
      l[h] *= sc;
      a[h] = make_float4(a[h].x * sc, a[h].y * sc, a[h].z * sc, a[h].w * sc);
      m[h] = mn[h];
    }
    const float pa = gat_exp2(ea - (hi ? mn[2] : mn[0]));
    const float pb = gat_exp2(eb - (hi ? mn[3] : mn[1]));
    gat_apply16(std::make_integer_sequence<int, 8>{}, pa, pb, xv, l, a);
    if constexpr (kPipe) {
#pragma unroll
      for (int t = 0; t < 8; ++t) xv[t] = xn[t];
    }
  }
}

// Shared-row mode (head_stride 0, no epilogue: the caller applies W_h afterwards): every
// head aggregates the same O-wide row, so a row is owned by O/4 lanes that each load ONE
// float4 of x per neighbour and keep H heads' online-softmax state for it (the generic
// kernel would spread the heads over H times as many lanes that all load the same bytes).
// Per (row, head, feature) the arithmetic is the generic kernel's, step for step.
// Neighbours [beg, end) of row r in shared-row mode (the online-softmax state of H heads).
template <int O, int H, int CH, bool ATT>
__device__ __forceinline__ void gat_shared_range(const GatParams& p, int64_t r, int64_t beg,
                                                 int64_t end, int gl, const float (&ss)[H],
                                                 float (&m)[H], float (&l)[H], float4 (&a)[H]) {
  constexpr int GROUP = O / 4;
  static_assert(CH == kSoftBlock, "one softmax block per gather step (same blocks as gat_kernel)");
  static_assert(!ATT || (GROUP == 16 && H == 4 && CH == 8), "ATT: the 16-lane, 4-head form");
  if constexpr (GROUP == 16 && H == 4 && CH == 8) {
    gat_shared_rows16<ATT>(p, r, beg, end, gl, ss, m, l, a);
  } else {
  for (int64_t k0 = beg; k0 < end; k0 += CH) {
    constexpr int PER = (GROUP >= CH) ? 1 : CH / GROUP;
    int cm[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      int64_t k = k0 + gl + (int64_t)q * GROUP;
      k = k < end ? k : end - 1;
      cm[q] = p.A.col[k];
    }
    float4 xv[CH];
    float sn[CH][H];
#pragma unroll
    for (int t = 0; t < CH; ++t) {
      const int c = __shfl(cm[t / GROUP < PER ? t / GROUP : 0], t % GROUP, GROUP);
      xv[t] = ld4(row_at(p.h + 4 * gl, c, (uint32_t)(p.ldh * 4)));
      if constexpr (H == 4) {
        const float4 s4 = ld4(p.s_neigh + (int64_t)c * p.ld_sn);
        sn[t][0] = s4.x; sn[t][1] = s4.y; sn[t][2] = s4.z; sn[t][3] = s4.w;
      } else {
#pragma unroll
        for (int h = 0; h < H; ++h) sn[t][h] = p.s_neigh[(int64_t)c * p.ld_sn + h];
      }
    }
#pragma unroll
    for (int h = 0; h < H; ++h) {
      float E[CH];
#pragma unroll
      for (int t = 0; t < CH; ++t) E[t] = gat_logit2(ss[h], sn[t][h], p.slope, k0 + t < end);
      gat_block(E, xv, m[h], l[h], a[h]);
    }
  }
  }
}

// the H self scores of row r for the shared-row kernels: from s_self, or (ATT) as dots of the
// row's own x with att[0][h] over the 16 lanes (every lane gets the same bits)
template <int O, int H, bool ATT>
__device__ __forceinline__ void shared_self_scores(const GatParams& p, int64_t r, int gl,
                                                   float (&ss)[H]) {
  if constexpr (ATT) {
    const float4 xr = ld4(p.hself + r * p.ld_hself + 4 * gl);
#pragma unroll
    for (int h = 0; h < H; ++h) ss[h] = group_sum<O / 4>(dot4(xr, ld4(p.att + h * O + 4 * gl)));
  } else {
#pragma unroll
    for (int h = 0; h < H; ++h) ss[h] = p.s_self[r * p.ld_ss + h];
  }
}

template <int O, int H, int CH, bool ATT>
__global__ __launch_bounds__(kBlock) GAT_SHARED_OCCUPANCY(ATT) void gat_shared_kernel(GatParams p) {
  constexpr int GROUP = O / 4;
  constexpr int RPW = 64 / GROUP;
  const int lane = threadIdx.x & 63;
  const int gl = lane % GROUP;
  const int64_t r = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * RPW + lane / GROUP;
  if (r >= p.A.n_rows) return;
  const int64_t beg = p.A.row_ptr[r], end = p.A.row_ptr[r + 1];
  if (p.max_row_len > 0 && end - beg > p.max_row_len) return;  // heavy row: split path
  float ss[H], m[H], l[H];
  float4 a[H];
  shared_self_scores<O, H, ATT>(p, r, gl, ss);
#pragma unroll
  for (int h = 0; h < H; ++h) {
    m[h] = -INFINITY;
    l[h] = 0.f;
    a[h] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  gat_shared_range<O, H, CH, ATT>(p, r, beg, end, gl, ss, m, l, a);
#pragma unroll
  for (int h = 0; h < H; ++h)
    st4(p.out + r * p.ldo + h * O + 4 * gl,
        gat_norm(a[h], l[h]));
}

// Heavy rows, pass 1: one row group per segment -> partial (acc[F], m[H], l[H]).
struct GatSplit {
  const int64_t* seg_row;
  const int64_t* seg_beg;
  const int64_t* seg_end;
  int64_t n_seg;
  const int64_t* heavy_rows;
  const int64_t* heavy_seg_ptr;
  int64_t n_heavy;
  float* work;  // [n_seg][F] acc | [n_seg][H] m | [n_seg][H] l
  // ATT entry point (ABI 10): the segment arrays may be in any order (e.g. sorted by their
  // first column, so that segments of different heavy rows over the same columns run
  // together and share the gathered lines in L2); seg_pos[j] = position of the j-th segment
  // in heavy_seg_ptr's row-grouped numbering (NULL: identity)
  const int64_t* seg_pos;
  int xcd_blocks;   // > 0: grid padded to 8 * xcd_blocks; XCD x runs logical blocks
                    // [x * xcd_blocks, (x + 1) * xcd_blocks): a contiguous stretch of segments
};

// logical block of a partial kernel (blocks are dealt round-robin to the 8 XCDs)
__device__ __forceinline__ int64_t split_block(const GatSplit& sp) {
  const int64_t b = blockIdx.x;
  return sp.xcd_blocks > 0 ? (b % 8) * sp.xcd_blocks + b / 8 : b;
}

template <int F, bool ATT, int HL = 0>
__global__ __launch_bounds__(kBlock) GAT_OCCUPANCY(ATT) void gat_partial_kernel(GatParams p, GatSplit sp) {
  constexpr int GROUP = F / 4;
  constexpr int RPW = 64 / GROUP;
  const int lane = threadIdx.x & 63;
  const int gl = lane % GROUP;
  const int64_t sg = (split_block(sp) * (kBlock / 64) + (threadIdx.x >> 6)) * RPW + lane / GROUP;
  if (sg >= sp.n_seg) return;
  float m = -INFINITY, l = 0.f;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  gat_accumulate<GROUP, ATT, HL>(p, sp.seg_row[sg], sp.seg_beg[sg], sp.seg_end[sg], gl, m, l, a);
  st4(sp.work + sg * F + 4 * gl, a);
  const int hl = p.o_dim / 4;
  if (gl % hl == 0) {
    float* ml = sp.work + sp.n_seg * F;
    ml[sg * p.heads + gl / hl] = m;
    ml[sp.n_seg * p.heads + sg * p.heads + gl / hl] = l;
  }
}

// Heavy rows, pass 1 in shared-row mode: O/4 lanes per segment load each neighbour's x row
// ONCE for all H heads (gat_partial_kernel<H*O> would load it H times, one head per lane
// group); the partials have gat_partial_kernel's layout, so gat_merge_kernel<H*O> finishes.
template <int O, int H, int CH, bool ATT>
__global__ __launch_bounds__(kBlock) GAT_SHARED_OCCUPANCY(ATT) void gat_shared_partial_kernel(GatParams p, GatSplit sp) {
  constexpr int GROUP = O / 4;
  constexpr int RPW = 64 / GROUP;
  const int lane = threadIdx.x & 63;
  const int gl = lane % GROUP;
  const int64_t sg = (split_block(sp) * (kBlock / 64) + (threadIdx.x >> 6)) * RPW + lane / GROUP;
  if (sg >= sp.n_seg) return;
  const int64_t r = sp.seg_row[sg];
  float ss[H], m[H], l[H];
  float4 a[H];
  shared_self_scores<O, H, ATT>(p, r, gl, ss);
#pragma unroll
  for (int h = 0; h < H; ++h) {
    m[h] = -INFINITY;
    l[h] = 0.f;
    a[h] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  gat_shared_range<O, H, CH, ATT>(p, r, sp.seg_beg[sg], sp.seg_end[sg], gl, ss, m, l, a);
  float* ml = sp.work + sp.n_seg * (H * O);
#pragma unroll
  for (int h = 0; h < H; ++h) {
    st4(sp.work + sg * (H * O) + h * O + 4 * gl, a[h]);
    if (gl == 0) {
      ml[sg * H + h] = m[h];
      ml[sp.n_seg * H + sg * H + h] = l[h];
    }
  }
}

// Heavy rows, pass 2: merge the segments of each heavy row (max-rescaled sums), finish. One
// workgroup per heavy row: its NG = 256 / GROUP row groups each merge a strided subset of
// the row's segments, then group 0 merges the NG partials (the longest power-law rows have
// hundreds of segments; one group walking them all was the serial tail of the launch).
template <int F>
__global__ __launch_bounds__(kBlock) void gat_merge_kernel(GatParams p, GatSplit sp) {
  constexpr int GROUP = F / 4;
  constexpr int NG = kBlock / GROUP;
  __shared__ float s_m[NG][GROUP], s_l[NG][GROUP];
  __shared__ float4 s_a[NG][GROUP];
  const int64_t h = blockIdx.x;
  const int g = threadIdx.x / GROUP, gl = threadIdx.x % GROUP;
  const int hl = p.o_dim / 4, head = gl / hl;
  const float* mm = sp.work + sp.n_seg * F;
  const float* ll = mm + sp.n_seg * p.heads;
  const int64_t s0 = sp.heavy_seg_ptr[h], s1 = sp.heavy_seg_ptr[h + 1];
  float M = -INFINITY;
  for (int64_t j = s0 + g; j < s1; j += NG) {
    const int64_t s = sp.seg_pos ? sp.seg_pos[j] : j;
    M = fmaxf(M, mm[s * p.heads + head]);
  }
  float L = 0.f;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t j = s0 + g; j < s1; j += NG) {
    const int64_t s = sp.seg_pos ? sp.seg_pos[j] : j;
    const float w = gat_exp2(mm[s * p.heads + head] - M);   // base-2 maxima (gat_block)
    const float4 t = ld4(sp.work + s * F + 4 * gl);
    L = __builtin_fmaf(ll[s * p.heads + head], w, L);
    a = make_float4(__builtin_fmaf(t.x, w, a.x), __builtin_fmaf(t.y, w, a.y),
                    __builtin_fmaf(t.z, w, a.z), __builtin_fmaf(t.w, w, a.w));
  }
  s_m[g][gl] = M;
  s_l[g][gl] = L;
  s_a[g][gl] = a;
  __syncthreads();
  if (g != 0) return;
  M = -INFINITY;
#pragma unroll
  for (int q = 0; q < NG; ++q) M = fmaxf(M, s_m[q][gl]);
  L = 0.f;
  a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    // a group without segments holds (-inf, 0, 0): weight 0
    const float w = s_m[q][gl] == -INFINITY ? 0.f : gat_exp2(s_m[q][gl] - M);
    const float4 t = s_a[q][gl];
    L = __builtin_fmaf(s_l[q][gl], w, L);
    a = make_float4(__builtin_fmaf(t.x, w, a.x), __builtin_fmaf(t.y, w, a.y),
                    __builtin_fmaf(t.z, w, a.z), __builtin_fmaf(t.w, w, a.w));
  }
  gat_finish<GROUP>(p, sp.heavy_rows[h], gat_norm(a, L), gl);
}

}  // namespace gnnrec

using namespace gnnrec;

namespace {

// f(integral_constant<F>, integral_constant<HL>) for the instantiated (F, HL) pair of the ATT
// kernels: F = heads * o_dim in {16 .. 256}, HL = o_dim / 4 in {1 .. 16}, HL <= F / 4
template <int FF, class Fn>
void for_hl_f(int hl, Fn&& f) {
  auto one = [&](auto hc) {
    if constexpr (decltype(hc)::value <= FF / 4)
      if (hl == decltype(hc)::value) f(std::integral_constant<int, FF>{}, hc);
  };
  one(std::integral_constant<int, 1>{});
  one(std::integral_constant<int, 2>{});
  one(std::integral_constant<int, 4>{});
  one(std::integral_constant<int, 8>{});
  one(std::integral_constant<int, 16>{});
}

template <class Fn>
void for_hl(int F, int hl, Fn&& f) {
  switch (F) {
    case 16: for_hl_f<16>(hl, f); break;
    case 32: for_hl_f<32>(hl, f); break;
    case 64: for_hl_f<64>(hl, f); break;
    case 128: for_hl_f<128>(hl, f); break;
    case 256: for_hl_f<256>(hl, f); break;
    default: break;
  }
}

// checks shared by both score forms; fills the epilogue part of GatParams
int gat_check_common(int64_t n_rows, int32_t heads, int32_t o_dim, const float* hfeat, int64_t ldh,
                     int64_t head_stride, int32_t mean_heads, float* out, int64_t ldo, int32_t epi,
                     const float* self, int64_t ld_self, float* acc, int64_t ld_acc) {
  GNNREC_REQUIRE(n_rows >= 0 && heads >= 1 && o_dim >= 4 && o_dim % 4 == 0, "gat: bad sizes");
  const int F = heads * o_dim;
  const int width = mean_heads ? o_dim : F;
  GNNREC_REQUIRE(head_stride >= 0 && !(head_stride & 3), "gat: head_stride must be >= 0 and %% 4 == 0");
  GNNREC_REQUIRE(hfeat && aligned16(hfeat) && !(ldh & 3) && ldh >= (heads - 1) * head_stride + o_dim &&
                     ldh < ((int64_t)1 << 30),
                 "gat: hfeat must be 16-B aligned, ld %% 4 == 0, (heads-1)*head_stride + o_dim <= ld "
                 "< 2^30 (row offsets are formed as 32-bit ld bytes x column)");
  GNNREC_REQUIRE((epi & GNNREC_EPI_NO_Y) || (out && aligned16(out) && !(ldo & 3) && ldo >= width),
                 "gat: bad out");
  GNNREC_REQUIRE(!(epi & GNNREC_EPI_ACC_INIT) || (self && aligned16(self) && !(ld_self & 3) && ld_self >= width),
                 "gat: ACC_INIT needs 16-B aligned self rows");
  GNNREC_REQUIRE(!(epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)) ||
                     (acc && aligned16(acc) && !(ld_acc & 3) && ld_acc >= width),
                 "gat: ACC needs 16-B aligned acc");
  return GNNREC_OK;
}

// ATT form: scores from the rows (o_dim <= 64: a head's dot spans at most a 16-lane DPP row)
int gat_check_att(const float* att, const float* hself, int64_t ld_hself, int64_t ldh,
                  int32_t o_dim, int32_t heads, int64_t head_stride) {
  GNNREC_REQUIRE(att && aligned16(att), "gat_att: att must be a 16-B aligned [2][heads][o_dim] array");
  GNNREC_REQUIRE(hself && aligned16(hself) && !(ld_hself & 3),
                 "gat_att: hself must be 16-B aligned with ld %% 4 == 0");
  GNNREC_REQUIRE(o_dim <= 64 && ((o_dim / 4) & (o_dim / 4 - 1)) == 0,
                 "gat_att: o_dim must be 4, 8, 16, 32 or 64 (got %d)", (int)o_dim);
  // the kernels read hself[r * ld_hself + h * head_stride + o] for h < heads, o < o_dim
  GNNREC_REQUIRE(ld_hself >= (int64_t)(heads - 1) * head_stride + o_dim,
                 "gat_att: ld_hself %lld < (heads - 1) * head_stride + o_dim", (long long)ld_hself);
  (void)ldh;
  return GNNREC_OK;
}

template <bool ATT>
int gat_aggregate_launch(const GatParams& p, int64_t n_rows, int heads, int o_dim, int mean_heads,
                         int apply_elu, int epi, const float* s_neigh, int64_t ld_sn,
                         hipStream_t s) {
  const int F = heads * o_dim;
  auto grid = [&](int f) { return dim3((unsigned)ceil_div(n_rows, (64 / (f / 4)) * (kBlock / 64))); };
  const bool shared_fast = p.head_stride == 0 && heads == 4 && !mean_heads && !apply_elu && epi == 0 &&
                           (ATT ? o_dim == 64
                                : ((o_dim == 16 || o_dim == 32 || o_dim == 64) && aligned16(s_neigh) &&
                                   !(ld_sn & 3))) &&
                           aligned16(p.out);
  if (shared_fast) {
    if constexpr (ATT) {
      hipLaunchKernelGGL((gat_shared_kernel<64, 4, 8, true>), grid(64), dim3(kBlock), 0, s, p);
    } else {
      switch (o_dim) {
        case 16: hipLaunchKernelGGL((gat_shared_kernel<16, 4, 8, false>), grid(16), dim3(kBlock), 0, s, p); break;
        case 32: hipLaunchKernelGGL((gat_shared_kernel<32, 4, 8, false>), grid(32), dim3(kBlock), 0, s, p); break;
        default: hipLaunchKernelGGL((gat_shared_kernel<64, 4, 8, false>), grid(64), dim3(kBlock), 0, s, p); break;
      }
    }
    return check_launch("gat_aggregate (shared rows)");
  }
  if constexpr (ATT) {
    const int hl = o_dim / 4;
    bool ok = false;
    for_hl(F, hl, [&](auto fc, auto hc) {
      constexpr int FF = decltype(fc)::value, HH = decltype(hc)::value;
      hipLaunchKernelGGL((gat_kernel<FF, true, HH>), grid(FF), dim3(kBlock), 0, s, p);
      ok = true;
    });
    if (!ok) {
      set_error("gat_att: heads*o_dim = %d with o_dim = %d unsupported", F, o_dim);
      return GNNREC_EUNSUPPORTED;
    }
    return check_launch("gat_aggregate_att");
  }
  switch (F) {
    case 16: hipLaunchKernelGGL((gat_kernel<16, false>), grid(16), dim3(kBlock), 0, s, p); break;
    case 32: hipLaunchKernelGGL((gat_kernel<32, false>), grid(32), dim3(kBlock), 0, s, p); break;
    case 64: hipLaunchKernelGGL((gat_kernel<64, false>), grid(64), dim3(kBlock), 0, s, p); break;
    case 128: hipLaunchKernelGGL((gat_kernel<128, false>), grid(128), dim3(kBlock), 0, s, p); break;
    case 256: hipLaunchKernelGGL((gat_kernel<256, false>), grid(256), dim3(kBlock), 0, s, p); break;
    default: set_error("gat: heads*o_dim = %d unsupported (16..256, power of two)", F); return GNNREC_EUNSUPPORTED;
  }
  return check_launch("gat_aggregate");
}

template <bool ATT>
int gat_heavy_launch(const GatParams& p, const GatSplit& sp, int heads, int o_dim,
                     const float* s_neigh, int64_t ld_sn, hipStream_t s) {
  const int F = heads * o_dim;
  auto g = [&](int64_t n, int f) {
    const int64_t nb = ceil_div(n, (64 / (f / 4)) * (kBlock / 64));
    return dim3((unsigned)(sp.xcd_blocks > 0 ? 8 * ceil_div(nb, 8) : nb));
  };
  const bool shared = p.head_stride == 0 && heads == 4 &&
                      (ATT ? o_dim == 64
                           : ((o_dim == 16 || o_dim == 32 || o_dim == 64) && aligned16(s_neigh) &&
                              !(ld_sn & 3)));
  if (shared) {
    // shared rows: one x load per neighbour for the 4 heads, then the generic merge
    if constexpr (ATT) {
      hipLaunchKernelGGL((gat_shared_partial_kernel<64, 4, 8, true>), g(sp.n_seg, 64), dim3(kBlock), 0, s, p, sp);
      hipLaunchKernelGGL(gat_merge_kernel<256>, dim3((unsigned)sp.n_heavy), dim3(kBlock), 0, s, p, sp);
    } else {
      switch (o_dim) {
#define GAT_SHARED_HEAVY(OO)                                                                        \
  case OO:                                                                                          \
    hipLaunchKernelGGL((gat_shared_partial_kernel<OO, 4, 8, false>), g(sp.n_seg, OO), dim3(kBlock), 0, \
                       s, p, sp);                                                                   \
    hipLaunchKernelGGL(gat_merge_kernel<4 * OO>, dim3((unsigned)sp.n_heavy), dim3(kBlock), 0, s, p, sp); \
    break;
        GAT_SHARED_HEAVY(16) GAT_SHARED_HEAVY(32) GAT_SHARED_HEAVY(64)
#undef GAT_SHARED_HEAVY
      }
    }
    return check_launch("gat_heavy (shared rows)");
  }
  if constexpr (ATT) {
    bool ok = false;
    for_hl(F, o_dim / 4, [&](auto fc, auto hc) {
      constexpr int FF = decltype(fc)::value, HH = decltype(hc)::value;
      hipLaunchKernelGGL((gat_partial_kernel<FF, true, HH>), g(sp.n_seg, FF), dim3(kBlock), 0, s, p, sp);
      hipLaunchKernelGGL(gat_merge_kernel<FF>, dim3((unsigned)sp.n_heavy), dim3(kBlock), 0, s, p, sp);
      ok = true;
    });
    if (!ok) {
      set_error("gat_heavy_att: heads*o_dim = %d with o_dim = %d unsupported", F, o_dim);
      return GNNREC_EUNSUPPORTED;
    }
    return check_launch("gat_heavy_att");
  }
  switch (F) {
#define GAT_HEAVY(FF)                                                                               \
  case FF:                                                                                          \
    hipLaunchKernelGGL((gat_partial_kernel<FF, false>), g(sp.n_seg, FF), dim3(kBlock), 0, s, p, sp); \
    hipLaunchKernelGGL(gat_merge_kernel<FF>, dim3((unsigned)sp.n_heavy), dim3(kBlock), 0, s, p, sp); \
    break;
    GAT_HEAVY(16) GAT_HEAVY(32) GAT_HEAVY(64) GAT_HEAVY(128) GAT_HEAVY(256)
#undef GAT_HEAVY
    default: set_error("gat_heavy: heads*o_dim = %d unsupported", F); return GNNREC_EUNSUPPORTED;
  }
  return check_launch("gat_heavy");
}

}  // namespace

extern "C" int gnnrec_gat_aggregate_f32(const int64_t* row_ptr, const int32_t* col, int64_t n_rows,
                                        const float* hfeat, int64_t ldh, int64_t head_stride,
                                        const float* s_self, const float* s_neigh, int64_t ld_ss,
                                        int64_t ld_sn, int32_t heads,
                                        int32_t o_dim,
                                        float slope, int32_t mean_heads, int32_t apply_elu,
                                        float* out, int64_t ldo, int32_t epi, const float* self,
                                        int64_t ld_self, float* acc, int64_t ld_acc, float acc_div,
                                        int64_t max_row_len, gnnrec_stream_t stream) {
  if (int st = gat_check_common(n_rows, heads, o_dim, hfeat, ldh, head_stride, mean_heads, out, ldo,
                                epi, self, ld_self, acc, ld_acc))
    return st;
  if (n_rows == 0) return GNNREC_OK;
  GNNREC_REQUIRE(row_ptr && col && s_self && s_neigh, "gat: null operand");
  GNNREC_REQUIRE(ld_ss >= heads && ld_sn >= heads, "gat: score row strides must be >= heads");
  GatParams p{Csr{row_ptr, col, nullptr, n_rows}, hfeat, ldh, head_stride, s_self, s_neigh, ld_ss, ld_sn, heads, o_dim, slope,
              mean_heads, apply_elu, out, ldo, epi, self, ld_self, acc, ld_acc, acc_div, max_row_len,
              nullptr, nullptr, 0};
  return gat_aggregate_launch<false>(p, n_rows, heads, o_dim, mean_heads, apply_elu, epi, s_neigh,
                                     ld_sn, as_hip(stream));
}

extern "C" int gnnrec_gat_aggregate_att_f32(const int64_t* row_ptr, const int32_t* col,
                                            int64_t n_rows, const float* hfeat, int64_t ldh,
                                            int64_t head_stride, const float* hself,
                                            int64_t ld_hself, const float* att, int32_t heads,
                                            int32_t o_dim, float slope, int32_t mean_heads,
                                            int32_t apply_elu, float* out, int64_t ldo, int32_t epi,
                                            const float* self, int64_t ld_self, float* acc,
                                            int64_t ld_acc, float acc_div, int64_t max_row_len,
                                            gnnrec_stream_t stream) {
  if (int st = gat_check_common(n_rows, heads, o_dim, hfeat, ldh, head_stride, mean_heads, out, ldo,
                                epi, self, ld_self, acc, ld_acc))
    return st;
  if (n_rows == 0) return GNNREC_OK;
  GNNREC_REQUIRE(row_ptr && col, "gat_att: null operand");
  if (int st = gat_check_att(att, hself, ld_hself, ldh, o_dim, heads, head_stride)) return st;
  GatParams p{Csr{row_ptr, col, nullptr, n_rows}, hfeat, ldh, head_stride, nullptr, nullptr, 0, 0, heads, o_dim, slope,
              mean_heads, apply_elu, out, ldo, epi, self, ld_self, acc, ld_acc, acc_div, max_row_len,
              att, hself, ld_hself};
  return gat_aggregate_launch<true>(p, n_rows, heads, o_dim, mean_heads, apply_elu, epi, nullptr, 0,
                                    as_hip(stream));
}

extern "C" int gnnrec_gat_heavy_f32(const int32_t* col, const int64_t* seg_row,
                                    const int64_t* seg_beg, const int64_t* seg_end, int64_t n_seg,
                                    const int64_t* heavy_rows, const int64_t* heavy_seg_ptr,
                                    int64_t n_heavy, float* work, const float* hfeat, int64_t ldh,
                                    int64_t head_stride, const float* s_self, const float* s_neigh,
                                    int64_t ld_ss, int64_t ld_sn, int32_t heads,
                                    int32_t o_dim, float slope, int32_t mean_heads,
                                    int32_t apply_elu, float* out, int64_t ldo, int32_t epi,
                                    const float* self, int64_t ld_self, float* acc, int64_t ld_acc,
                                    float acc_div, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_seg >= 0 && n_heavy >= 0 && heads >= 1 && o_dim >= 4 && o_dim % 4 == 0,
                 "gat_heavy: bad sizes");
  if (n_heavy == 0) return GNNREC_OK;
  GNNREC_REQUIRE(col && seg_row && seg_beg && seg_end && heavy_rows && heavy_seg_ptr && work &&
                     hfeat && s_self && s_neigh && aligned16(work) && aligned16(hfeat) && !(ldh & 3) &&
                     ldh < ((int64_t)1 << 30) && head_stride >= 0 && !(head_stride & 3),
                 "gat_heavy: null or misaligned operand (or ld >= 2^30)");
  GNNREC_REQUIRE(ld_ss >= heads && ld_sn >= heads, "gat_heavy: score row strides must be >= heads");
  GatParams p{Csr{nullptr, col, nullptr, 0}, hfeat, ldh, head_stride, s_self, s_neigh, ld_ss, ld_sn, heads, o_dim, slope,
              mean_heads, apply_elu, out, ldo, epi, self, ld_self, acc, ld_acc, acc_div, 0,
              nullptr, nullptr, 0};
  GatSplit sp{seg_row, seg_beg, seg_end, n_seg, heavy_rows, heavy_seg_ptr, n_heavy, work,
              nullptr, 0};
  return gat_heavy_launch<false>(p, sp, heads, o_dim, s_neigh, ld_sn, as_hip(stream));
}

extern "C" int gnnrec_gat_heavy_att_f32(const int32_t* col, const int64_t* seg_row,
                                        const int64_t* seg_beg, const int64_t* seg_end,
                                        int64_t n_seg, const int64_t* heavy_rows,
                                        const int64_t* heavy_seg_ptr, int64_t n_heavy, float* work,
                                        const float* hfeat, int64_t ldh, int64_t head_stride,
                                        const float* hself, int64_t ld_hself, const float* att,
                                        int32_t heads, int32_t o_dim, float slope,
                                        int32_t mean_heads, int32_t apply_elu, float* out,
                                        int64_t ldo, int32_t epi, const float* self,
                                        int64_t ld_self, float* acc, int64_t ld_acc, float acc_div,
                                        const int64_t* seg_pos, int32_t xcd_order,
                                        gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_seg >= 0 && n_heavy >= 0 && heads >= 1 && o_dim >= 4 && o_dim % 4 == 0,
                 "gat_heavy_att: bad sizes");
  if (n_heavy == 0) return GNNREC_OK;
  GNNREC_REQUIRE(col && seg_row && seg_beg && seg_end && heavy_rows && heavy_seg_ptr && work &&
                     hfeat && aligned16(work) && aligned16(hfeat) && !(ldh & 3) &&
                     ldh < ((int64_t)1 << 30) && head_stride >= 0 && !(head_stride & 3),
                 "gat_heavy_att: null or misaligned operand (or ld >= 2^30)");
  if (int st = gat_check_att(att, hself, ld_hself, ldh, o_dim, heads, head_stride)) return st;
  GatParams p{Csr{nullptr, col, nullptr, 0}, hfeat, ldh, head_stride, nullptr, nullptr, 0, 0, heads, o_dim, slope,
              mean_heads, apply_elu, out, ldo, epi, self, ld_self, acc, ld_acc, acc_div, 0,
              att, hself, ld_hself};
  // xcd_blocks: logical blocks per XCD of the partial kernel's grid (16 segment lanes groups
  // per block at o_dim <= 64 rows of 64 floats; the kernel derives its own geometry)
  int64_t xb = 0;
  if (xcd_order) {
    const int f = (head_stride == 0 && heads == 4 && o_dim == 64) ? 64 : heads * o_dim;
    xb = ceil_div(ceil_div(n_seg, (64 / (f / 4)) * (kBlock / 64)), 8);
  }
  GatSplit sp{seg_row, seg_beg, seg_end, n_seg, heavy_rows, heavy_seg_ptr, n_heavy, work,
              seg_pos, (int)xb};
  return gat_heavy_launch<true>(p, sp, heads, o_dim, nullptr, 0, as_hip(stream));
}
