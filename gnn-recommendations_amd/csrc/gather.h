// Device building blocks shared by the SpMM-family kernels (spmm.hip, dense_epi.hip):
// the sequential-order CSR row gather and the GAS row transform.
//
// Mapping (d = 4*GROUP): a destination row is owned by GROUP consecutive lanes of a 64-wide
// wavefront, each lane owning 4 consecutive features (one float4). A wave therefore carries
// 64/GROUP rows (d=64: 16 lanes/row, 4 rows/wave) and every neighbour gather is one coalesced
// 4*d-byte row read issued as global_load_dwordx4 by the row's lanes. Neighbour (col,val)
// pairs are fetched cooperatively, kChunk per step, and broadcast inside the group with
// __shfl; the kChunk row gathers of a step are all issued before the first FMA, so kChunk
// independent 16-B loads per lane are in flight. FMAs are applied in k order per lane, so
// splitting the loads never changes the arithmetic (bit-exact with the reference).
#pragma once

#include "common.h"

namespace gnnrec {

constexpr int kBlock = 256;  // 4 waves per workgroup
constexpr int kChunk = 16;   // neighbours per gather step

__device__ __forceinline__ float4 fma4(float v, const float4& x, const float4& a) {
  return make_float4(__builtin_fmaf(v, x.x, a.x), __builtin_fmaf(v, x.y, a.y),
                     __builtin_fmaf(v, x.z, a.z), __builtin_fmaf(v, x.w, a.w));
}

__device__ __forceinline__ float4 ld4(const float* p) {
  return *reinterpret_cast<const float4*>(p);
}
__device__ __forceinline__ void st4(float* p, const float4& v) {
  *reinterpret_cast<float4*>(p) = v;
}

// One gather step of CH neighbours [k0, k0+CH) of a row ending at `end`. TAIL selects the
// FMA of out-of-row slots away (their loads are clamped to the row's last element).
template <int GROUP, bool TAIL, int CH = kChunk>
__device__ __forceinline__ void gather_step(const int32_t* __restrict__ col,
                                            const float* __restrict__ val, int64_t k0,
                                            int64_t end, const float* __restrict__ x,
                                            int64_t ldx, int gl, float4& a) {
  constexpr int PER = (GROUP >= CH) ? 1 : CH / GROUP;  // pairs loaded per lane
  int cm[PER];
  float vm[PER];
#pragma unroll
  for (int m = 0; m < PER; ++m) {
    int64_t k = k0 + gl + (int64_t)m * GROUP;
    if (TAIL) k = k < end ? k : end - 1;
    if (GROUP >= CH && gl >= CH) k = k0;  // idle lanes: any in-row address
    cm[m] = col[k];
    vm[m] = val[k];
  }
  float4 xv[CH];
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    const int c = __shfl(cm[t / GROUP < PER ? t / GROUP : 0], t % GROUP, GROUP);
    xv[t] = ld4(x + (int64_t)c * ldx + 4 * gl);
  }
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    const float v = __shfl(vm[t / GROUP < PER ? t / GROUP : 0], t % GROUP, GROUP);
    const float4 n = fma4(v, xv[t], a);
    if (TAIL) {
      const bool ok = (k0 + t) < end;
      a.x = ok ? n.x : a.x;
      a.y = ok ? n.y : a.y;
      a.z = ok ? n.z : a.z;
      a.w = ok ? n.w : a.w;
    } else {
      a = n;
    }
  }
}

// Sequential-order row reduction: returns the lane's float4 slice of (A x)[r].
template <int GROUP, int CH = kChunk>
__device__ __forceinline__ float4 gather_row(const int32_t* __restrict__ col,
                                             const float* __restrict__ val, int64_t beg,
                                             int64_t end, const float* __restrict__ x,
                                             int64_t ldx, int gl) {
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  int64_t k0 = beg;
  for (; k0 + CH <= end; k0 += CH) gather_step<GROUP, false, CH>(col, val, k0, end, x, ldx, gl, a);
  if (k0 < end) gather_step<GROUP, true, CH>(col, val, k0, end, x, ldx, gl, a);
  return a;
}

// ---- VEC-generic form (VEC = 1, 2 or 4 features per lane, GROUP = d / VEC lanes per row) --
template <int N>
struct VecF {
  float v[N];
};

template <int N>
__device__ __forceinline__ VecF<N> ldv(const float* p) {
  VecF<N> r;
  if constexpr (N == 4) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    r.v[0] = t.x; r.v[1] = t.y; r.v[2] = t.z; r.v[3] = t.w;
  } else if constexpr (N == 2) {
    const float2 t = *reinterpret_cast<const float2*>(p);
    r.v[0] = t.x; r.v[1] = t.y;
  } else {
    r.v[0] = *p;
  }
  return r;
}

template <int N>
__device__ __forceinline__ void stv(float* p, const VecF<N>& a) {
  if constexpr (N == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(a.v[0], a.v[1], a.v[2], a.v[3]);
  } else if constexpr (N == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(a.v[0], a.v[1]);
  } else {
    *p = a.v[0];
  }
}

// xmask (optional): one byte per source row, 0 = the row is all zeros. Such a row is not
// gathered and contributes 0: fmaf(v, +-0, acc) == acc for the finite operand values and the
// accumulator that starts at +0, so the result is the same bits (sparse inputs, e.g. the
// BPR gradient entering the backward propagation, skip almost every gather).
template <int VEC, int GROUP, bool TAIL, int CH, bool NT = false, bool MASKED = false>
__device__ __forceinline__ void gather_step_v(const int32_t* __restrict__ col,
                                              const float* __restrict__ val, int64_t k0,
                                              int64_t end, const float* __restrict__ x,
                                              int64_t ldx, int gl, VecF<VEC>& a,
                                              const uint8_t* __restrict__ xmask = nullptr) {
  constexpr int PER = (GROUP >= CH) ? 1 : CH / GROUP;
  int cm[PER];
  float vm[PER];
#pragma unroll
  for (int m = 0; m < PER; ++m) {
    int64_t k = k0 + gl + (int64_t)m * GROUP;
    if (TAIL) k = k < end ? k : end - 1;
    if (GROUP >= CH && gl >= CH) k = k0;
    if (NT) {
      cm[m] = __builtin_nontemporal_load(col + k);
      vm[m] = __builtin_nontemporal_load(val + k);
    } else {
      cm[m] = col[k];
      vm[m] = val[k];
    }
  }
  VecF<VEC> xv[CH];
  int cc[CH];
#pragma unroll
  for (int t = 0; t < CH; ++t) cc[t] = __shfl(cm[t / GROUP < PER ? t / GROUP : 0], t % GROUP, GROUP);
  if constexpr (MASKED) {
    // all CH mask bytes in flight together, then only the non-zero rows are gathered
    uint8_t mk[CH];
#pragma unroll
    for (int t = 0; t < CH; ++t) mk[t] = xmask[cc[t]];
#pragma unroll
    for (int t = 0; t < CH; ++t) {
      if (mk[t]) {
        xv[t] = ldv<VEC>(x + (int64_t)cc[t] * ldx + VEC * gl);
      } else {
#pragma unroll
        for (int q = 0; q < VEC; ++q) xv[t].v[q] = 0.f;
      }
    }
  } else {
#pragma unroll
    for (int t = 0; t < CH; ++t) xv[t] = ldv<VEC>(x + (int64_t)cc[t] * ldx + VEC * gl);
  }
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    const float v = __shfl(vm[t / GROUP < PER ? t / GROUP : 0], t % GROUP, GROUP);
    const bool ok = !TAIL || (k0 + t) < end;
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      const float n = __builtin_fmaf(v, xv[t].v[q], a.v[q]);
      a.v[q] = ok ? n : a.v[q];
    }
  }
}

template <int VEC, int GROUP, int CH, bool NT = false, bool MASKED = false>
__device__ __forceinline__ VecF<VEC> gather_row_v(const int32_t* __restrict__ col,
                                                  const float* __restrict__ val, int64_t beg,
                                                  int64_t end, const float* __restrict__ x,
                                                  int64_t ldx, int gl,
                                                  const uint8_t* __restrict__ xmask = nullptr) {
  VecF<VEC> a;
#pragma unroll
  for (int q = 0; q < VEC; ++q) a.v[q] = 0.f;
  int64_t k0 = beg;
  for (; k0 + CH <= end; k0 += CH)
    gather_step_v<VEC, GROUP, false, CH, NT, MASKED>(col, val, k0, end, x, ldx, gl, a, xmask);
  if (k0 < end)
    gather_step_v<VEC, GROUP, true, CH, NT, MASKED>(col, val, k0, end, x, ldx, gl, a, xmask);
  return a;
}

// Latency form of the same chain, for operands too small to fill the chip with rows (ML-1M:
// 9.4K row-parallel rows, one wave each): the next step's (col, val) are loaded before this
// step's row gathers, so a step waits for one memory latency (the gathers) instead of two
// (indices, then rows), and a step carries CH (>= the throughput form's) gathers. Same fmaf
// order, same bits. PER == 1 only (GROUP >= CH: lanes gl < CH hold the step's indices).
template <int VEC, int GROUP, bool TAIL, int CH>
__device__ __forceinline__ void gather_apply_v(int cm, float vm, int64_t k0, int64_t end,
                                               const float* __restrict__ x, int64_t ldx, int gl,
                                               VecF<VEC>& a) {
  VecF<VEC> xv[CH];
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    const int c = __shfl(cm, t, GROUP);
    xv[t] = ldv<VEC>(x + (int64_t)c * ldx + VEC * gl);
  }
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    const float v = __shfl(vm, t, GROUP);
    const bool ok = !TAIL || (k0 + t) < end;
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      const float n = __builtin_fmaf(v, xv[t].v[q], a.v[q]);
      a.v[q] = ok ? n : a.v[q];
    }
  }
}

template <int VEC, int GROUP, int CH>
__device__ __forceinline__ VecF<VEC> gather_row_pipe(const int32_t* __restrict__ col,
                                                     const float* __restrict__ val, int64_t beg,
                                                     int64_t end, const float* __restrict__ x,
                                                     int64_t ldx, int gl) {
  static_assert(GROUP >= CH, "one index per lane per step");
  VecF<VEC> a;
#pragma unroll
  for (int q = 0; q < VEC; ++q) a.v[q] = 0.f;
  if (beg >= end) return a;
  // step k0's index of lane gl (lanes past CH repeat k0's), clamped into the row: always a
  // valid entry, so the loads need no branch (a branch made the compiler wait on them)
  auto load_cv = [&](int64_t k0, int& c, float& v) {
    int64_t k = gl < CH ? k0 + gl : k0;
    k = k < end ? k : end - 1;
    c = col[k];
    v = val[k];
  };
  int cm;
  float vm;
  load_cv(beg, cm, vm);
  int64_t k0 = beg;
  for (; k0 + CH <= end; k0 += CH) {
    int cn;
    float vn;
    load_cv(k0 + CH, cn, vn);
    gather_apply_v<VEC, GROUP, false, CH>(cm, vm, k0, end, x, ldx, gl, a);
    cm = cn;
    vm = vn;
  }
  if (k0 < end) gather_apply_v<VEC, GROUP, true, CH>(cm, vm, k0, end, x, ldx, gl, a);
  return a;
}

template <int VEC>
__device__ __forceinline__ void acc_epilogue_v(int epi, const VecF<VEC>& y, const float* self_row,
                                               float* acc_row, float acc_div) {
  if (!(epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD))) return;
  VecF<VEC> b = (epi & GNNREC_EPI_ACC_INIT) ? ldv<VEC>(self_row) : ldv<VEC>(acc_row);
#pragma unroll
  for (int q = 0; q < VEC; ++q) {
    b.v[q] = b.v[q] + y.v[q];
    if (epi & GNNREC_EPI_ACC_DIV) b.v[q] = b.v[q] / acc_div;
  }
  stv<VEC>(acc_row, b);
}

// Lane mapping per d, from the G100M sweep (tools/exp_prod.py, profiles/r01/): VEC features
// per lane, GROUP = d / VEC lanes per row, CH neighbours in flight per step.
template <int D> struct SpmmCfg { static constexpr int VEC = 4, CH = 16; };
template <> struct SpmmCfg<32> { static constexpr int VEC = 2, CH = 16; };
template <> struct SpmmCfg<64> { static constexpr int VEC = 1, CH = 8; };   // wave per row
template <> struct SpmmCfg<128> { static constexpr int VEC = 2, CH = 16; };  // wave per row

// Latency form (gather_row_pipe) per d: VEC features per lane (the throughput form's unless
// GNNREC_LAT_VEC64 sets d = 64's) and CH gathers per step.
#ifndef GNNREC_LAT_CH
#define GNNREC_LAT_CH 16
#endif
#ifndef GNNREC_LAT_VEC64
#define GNNREC_LAT_VEC64 4
#endif
// d = 128 takes 8 gathers per step (a wave per row, 2 features per lane): the power-law
// 2M x 2M K = 3 propagation 24.0 -> 22.6 ms against 16 (the throughput form's count, which
// made the two forms the same), config 2 unchanged (profiles/r06/light_chunk_ab.jsonl)
#ifndef GNNREC_LAT_CH128
#define GNNREC_LAT_CH128 8
#endif
template <int D> struct SpmmLatCfg {
  static constexpr bool OK = (D == 32 || D == 64 || D == 128);
  static constexpr int VEC = D == 64 ? GNNREC_LAT_VEC64 : SpmmCfg<D>::VEC;
  static constexpr int GROUP = D / VEC;
  static constexpr int CH_WANT = D == 128 ? GNNREC_LAT_CH128 : GNNREC_LAT_CH;
  static constexpr int CH = CH_WANT < GROUP ? CH_WANT : GROUP;
};

// ---- GAS (block-diagonal orthogonal transform + column shuffle) -----------------------
// y[r, j] = sum_{c<bs} z[r, bs*b + c] * W_b[c, e],  perm[j] = bs*b + e  (sequential fmaf in c).
// The row z is parked in LDS so every lane can read the bs inputs of its 4 outputs.
template <int D>
__device__ __forceinline__ float4 gas_row(const float* zrow_lds, const float* w_lds, int bs,
                                          const int (&pj)[4]) {
  float o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int b = pj[q] / bs, e = pj[q] - b * bs;
    const float* z = zrow_lds + b * bs;
    const float* w = w_lds + (b * bs) * bs + e;
    float s = 0.f;
    for (int c = 0; c < bs; ++c) s = __builtin_fmaf(z[c], w[c * bs], s);
    o[q] = s;
  }
  return make_float4(o[0], o[1], o[2], o[3]);
}

// VEC-output form: outputs j = VEC*gl + q, q < VEC (pj holds perm[VEC*gl + q]).
template <int VEC>
__device__ __forceinline__ VecF<VEC> gas_row_v(const float* zrow_lds, const float* w_lds, int bs,
                                               const int (&pj)[VEC]) {
  VecF<VEC> o;
#pragma unroll
  for (int q = 0; q < VEC; ++q) {
    const int b = pj[q] / bs, e = pj[q] - b * bs;
    const float* z = zrow_lds + b * bs;
    const float* w = w_lds + (b * bs) * bs + e;
    float s = 0.f;
    for (int c = 0; c < bs; ++c) s = __builtin_fmaf(z[c], w[c * bs], s);
    o.v[q] = s;
  }
  return o;
}

// LightGCN layer-mean epilogue (see GNNREC_EPI_* in gnnrec.h).
__device__ __forceinline__ void acc_epilogue(int epi, const float4& y, const float* self_row,
                                             float* acc_row, float acc_div) {
  if (!(epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD))) return;
  float4 b = (epi & GNNREC_EPI_ACC_INIT) ? ld4(self_row) : ld4(acc_row);
  b.x = b.x + y.x;
  b.y = b.y + y.y;
  b.z = b.z + y.z;
  b.w = b.w + y.w;
  if (epi & GNNREC_EPI_ACC_DIV) {
    b.x = b.x / acc_div;
    b.y = b.y / acc_div;
    b.z = b.z / acc_div;
    b.w = b.w / acc_div;
  }
  st4(acc_row, b);
}

}  // namespace gnnrec
