// Experimental SpMM variants for tools/exp_sweep.py (NOT part of libgnnrec): used to find
// what bounds the hop kernel on MI355X (gather working set, chunk depth, lane mapping).
#include "../gnn-recommendations_amd/csrc/gather.h"

using namespace gnnrec;

template <int CH, bool NT_COLVAL>
__global__ __launch_bounds__(256) void k_group16(Csr A, const float* __restrict__ x, float* __restrict__ y) {
  const int lane = threadIdx.x & 63, gl = lane % 16;
  const int64_t r = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + lane / 16;
  if (r >= A.n_rows) return;
  const float4 a = gather_row<16, CH>(A.col, A.val, A.row_ptr[r], A.row_ptr[r + 1], x, 64, gl);
  st4(y + r * 64 + 4 * gl, a);
}

// one row per wave, one feature per lane (d = 64)
__global__ __launch_bounds__(256) void k_wave_row(Csr A, const float* __restrict__ x, float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= A.n_rows) return;
  const int64_t beg = A.row_ptr[r], end = A.row_ptr[r + 1];
  float a = 0.f;
  for (int64_t k0 = beg; k0 < end; k0 += 16) {
    int64_t k = k0 + (lane & 15);
    k = k < end ? k : end - 1;
    const int c = A.col[k];
    const float v = A.val[k];
    float xv[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) xv[t] = x[(int64_t)__shfl(c, t, 64) * 64 + lane];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const float n = __builtin_fmaf(__shfl(v, t, 64), xv[t], a);
      a = (k0 + t < end) ? n : a;
    }
  }
  y[r * 64 + lane] = a;
}

// CSR stream only (no gathers): the col/val/row_ptr streaming floor
__global__ __launch_bounds__(256) void k_stream(Csr A, const float* __restrict__ x, float* __restrict__ y) {
  const int lane = threadIdx.x & 63, gl = lane % 16;
  const int64_t r = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + lane / 16;
  if (r >= A.n_rows) return;
  const int64_t beg = A.row_ptr[r], end = A.row_ptr[r + 1];
  float s = 0.f;
  for (int64_t k = beg + gl; k < end; k += 16) s += A.val[k] + (float)A.col[k];
  y[r * 64 + 4 * gl] = s;
}

// gathers with non-temporal x loads
__global__ __launch_bounds__(256) void k_nt(Csr A, const float* __restrict__ x, float* __restrict__ y) {
  const int lane = threadIdx.x & 63, gl = lane % 16;
  const int64_t r = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + lane / 16;
  if (r >= A.n_rows) return;
  const int64_t beg = A.row_ptr[r], end = A.row_ptr[r + 1];
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t k0 = beg; k0 < end; k0 += 16) {
    int64_t k = k0 + gl;
    k = k < end ? k : end - 1;
    const int c = A.col[k];
    const float v = A.val[k];
    float4 xv[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const float* p = x + (int64_t)__shfl(c, t, 16) * 64 + 4 * gl;
      xv[t] = make_float4(__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1),
                          __builtin_nontemporal_load(p + 2), __builtin_nontemporal_load(p + 3));
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const float4 n = fma4(__shfl(v, t, 16), xv[t], a);
      if (k0 + t < end) a = n;
    }
  }
  st4(y + r * 64 + 4 * gl, a);
}


// one row per wave, CH-deep
template <int CH>
__global__ __launch_bounds__(256) void k_wave_row_ch(Csr A, const float* __restrict__ x, float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= A.n_rows) return;
  const int64_t beg = A.row_ptr[r], end = A.row_ptr[r + 1];
  float a = 0.f;
  for (int64_t k0 = beg; k0 < end; k0 += CH) {
    int64_t k = k0 + (lane % CH);
    k = k < end ? k : end - 1;
    const int c = A.col[k];
    const float v = A.val[k];
    float xv[CH];
#pragma unroll
    for (int t = 0; t < CH; ++t) xv[t] = x[(int64_t)__shfl(c, t, 64) * 64 + lane];
#pragma unroll
    for (int t = 0; t < CH; ++t) {
      const float n = __builtin_fmaf(__shfl(v, t, 64), xv[t], a);
      a = (k0 + t < end) ? n : a;
    }
  }
  y[r * 64 + lane] = a;
}

// 32 lanes per row, float2 per lane (d = 64), 2 rows per wave
__global__ __launch_bounds__(256) void k_group32(Csr A, const float* __restrict__ x, float* __restrict__ y) {
  const int lane = threadIdx.x & 63, gl = lane % 32;
  const int64_t r = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + lane / 32;
  if (r >= A.n_rows) return;
  const int64_t beg = A.row_ptr[r], end = A.row_ptr[r + 1];
  float2 a = make_float2(0.f, 0.f);
  for (int64_t k0 = beg; k0 < end; k0 += 16) {
    int64_t k = k0 + (gl & 15);
    k = k < end ? k : end - 1;
    const int c = A.col[k];
    const float v = A.val[k];
    float2 xv[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) xv[t] = *reinterpret_cast<const float2*>(x + (int64_t)__shfl(c, t, 32) * 64 + 2 * gl);
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const float vv = __shfl(v, t, 32);
      const float2 n = make_float2(__builtin_fmaf(vv, xv[t].x, a.x), __builtin_fmaf(vv, xv[t].y, a.y));
      if (k0 + t < end) a = n;
    }
  }
  *reinterpret_cast<float2*>(y + r * 64 + 2 * gl) = a;
}

// group16 over a row permutation (degree-sorted order)
__global__ __launch_bounds__(256) void k_group16_perm(Csr A, const int32_t* __restrict__ order, const float* __restrict__ x, float* __restrict__ y) {
  const int lane = threadIdx.x & 63, gl = lane % 16;
  const int64_t i = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + lane / 16;
  if (i >= A.n_rows) return;
  const int64_t r = order[i];
  const float4 a = gather_row<16, 16>(A.col, A.val, A.row_ptr[r], A.row_ptr[r + 1], x, 64, gl);
  st4(y + r * 64 + 4 * gl, a);
}

// d = 128: 32 lanes x float4, 2 rows per wave
__global__ __launch_bounds__(256) void k_d128(Csr A, const float* __restrict__ x, float* __restrict__ y) {
  const int lane = threadIdx.x & 63, gl = lane % 32;
  const int64_t r = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + lane / 32;
  if (r >= A.n_rows) return;
  const float4 a = gather_row<32, 16>(A.col, A.val, A.row_ptr[r], A.row_ptr[r + 1], x, 128, gl);
  st4(y + r * 128 + 4 * gl, a);
}

extern "C" int exp_spmm2(int variant, const int64_t* rp, const int32_t* col, const float* val,
                         int64_t n_rows, const int32_t* order, const float* x, float* y, hipStream_t s) {
  Csr A{rp, col, val, n_rows};
  const unsigned g16 = (unsigned)((n_rows + 15) / 16), gw = (unsigned)((n_rows + 3) / 4),
                 g32 = (unsigned)((n_rows + 7) / 8);
  switch (variant) {
    case 6: hipLaunchKernelGGL(k_wave_row_ch<32>, dim3(gw), dim3(256), 0, s, A, x, y); break;
    case 7: hipLaunchKernelGGL(k_group32, dim3(g32), dim3(256), 0, s, A, x, y); break;
    case 8: hipLaunchKernelGGL(k_group16_perm, dim3(g16), dim3(256), 0, s, A, order, x, y); break;
    case 9: hipLaunchKernelGGL(k_d128, dim3(g32), dim3(256), 0, s, A, x, y); break;
    case 10: hipLaunchKernelGGL(k_wave_row_ch<8>, dim3(gw), dim3(256), 0, s, A, x, y); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int exp_spmm(int variant, const int64_t* rp, const int32_t* col, const float* val,
                        int64_t n_rows, const float* x, float* y, hipStream_t s) {
  Csr A{rp, col, val, n_rows};
  const unsigned g16 = (unsigned)((n_rows + 15) / 16), gw = (unsigned)((n_rows + 3) / 4);
  switch (variant) {
    case 0: hipLaunchKernelGGL((k_group16<16, true>), dim3(g16), dim3(256), 0, s, A, x, y); break;
    case 1: hipLaunchKernelGGL((k_group16<32, true>), dim3(g16), dim3(256), 0, s, A, x, y); break;
    case 2: hipLaunchKernelGGL((k_group16<8, true>), dim3(g16), dim3(256), 0, s, A, x, y); break;
    case 3: hipLaunchKernelGGL(k_wave_row, dim3(gw), dim3(256), 0, s, A, x, y); break;
    case 4: hipLaunchKernelGGL(k_stream, dim3(g16), dim3(256), 0, s, A, x, y); break;
    case 5: hipLaunchKernelGGL(k_nt, dim3(g16), dim3(256), 0, s, A, x, y); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <int D, int VEC, int CH, bool NT = true>
__global__ __launch_bounds__(256) void k_prod(Csr A, const float* __restrict__ x, float* __restrict__ y) {
  constexpr int GROUP = D / VEC, RPW = 64 / GROUP;
  const int lane = threadIdx.x & 63, gl = lane % GROUP;
  const int64_t r = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / GROUP;
  if (r >= A.n_rows) return;
  const VecF<VEC> a = gather_row_v<VEC, GROUP, CH, NT>(A.col, A.val, A.row_ptr[r], A.row_ptr[r + 1], x, D, gl);
  stv<VEC>(y + r * D + VEC * gl, a);
}

template <int D, int VEC, int CH, bool NT = true>
static void lp(Csr A, const float* x, float* y, hipStream_t s) {
  constexpr int RPB = 4 * (64 / (D / VEC));
  hipLaunchKernelGGL((k_prod<D, VEC, CH, NT>), dim3((unsigned)((A.n_rows + RPB - 1) / RPB)), dim3(256), 0, s, A, x, y);
}

extern "C" int exp_prod(int d, int vec, int ch, const int64_t* rp, const int32_t* col, const float* val,
                        int64_t n_rows, const float* x, float* y, hipStream_t s) {
  Csr A{rp, col, val, n_rows};
#define CASE(D, V, C) if (d == D && vec == V && ch == C) { lp<D, V, C>(A, x, y, s); return hipGetLastError() == hipSuccess ? 0 : -2; }
  CASE(32, 1, 8) CASE(32, 1, 16) CASE(32, 2, 8) CASE(32, 2, 16) CASE(32, 4, 8) CASE(32, 4, 16)
  CASE(64, 1, 8) CASE(64, 1, 16) CASE(64, 2, 8) CASE(64, 2, 16) CASE(64, 4, 8) CASE(64, 4, 16) CASE(64, 1, 4) CASE(64, 2, 4)
  CASE(128, 2, 8) CASE(128, 2, 16) CASE(128, 4, 8) CASE(128, 4, 16) CASE(128, 2, 4)
#undef CASE
#define CASEP(D, V, C) if (d == D && vec == V && ch == C + 1000) { lp<D, V, C, false>(A, x, y, s); return hipGetLastError() == hipSuccess ? 0 : -2; }
  CASEP(64, 1, 8) CASEP(64, 1, 16) CASEP(64, 2, 8) CASEP(64, 2, 16) CASEP(64, 4, 16) CASEP(128, 2, 16) CASEP(128, 4, 16) CASEP(32, 2, 16)
#undef CASEP
  return -1;
}
