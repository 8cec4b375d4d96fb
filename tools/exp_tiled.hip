// Experiment (NOT part of libgnnrec): column-ordered SpMM hop with on-chip accumulators.
//
// Idea: the row-parallel hop gathers every neighbour row from beyond L2 (16x the compulsory
// bytes on G100M). Here a persistent workgroup per CU owns R destination rows per pass with
// their accumulators in LDS; each wave owns a subset of those rows and walks its edges in
// ascending COLUMN order (ties by row), so all waves of an XCD sweep the source table together
// and a gathered row is reused from L2 by the other rows of the XCD that read it. Per row the
// edges are still applied in ascending column order from +0 -> same bits as the CSR kernel.
//
// Stream layout (built by tools/exp_tiled.py): per (block, wave) a run of chunks of CH edges
// (plus CH padding entries after the last stream so a prefetch past the end is harmless):
//   col int32, val f32, meta uint16 = local row (11 bits) | (prev slot + 1) << 11
// prev slot = the latest earlier slot of the same chunk with the same row (its new value is
// the chain input instead of the LDS value). Padding slots: row = R (scratch), val = 0.
#include <hip/hip_runtime.h>
#include <cstdint>

#ifndef EXP_NW
#define EXP_NW 16
#endif
constexpr int NW = EXP_NW;  // waves per workgroup
constexpr int CH = 16;

template <int MODE>
struct Chunk {
  int c[CH];
  float v[CH];
  uint32_t m[CH / 2];
  float x[CH];
};

template <int D, int MODE>
__device__ __forceinline__ void fetch(const int32_t* __restrict__ scol,
                                      const float* __restrict__ sval,
                                      const uint32_t* __restrict__ smeta, int64_t c,
                                      const float* __restrict__ x, int lane, Chunk<MODE>& k) {
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    k.c[t] = scol[c + t];
    k.v[t] = sval[c + t];
  }
#pragma unroll
  for (int t = 0; t < CH / 2; ++t) k.m[t] = smeta[c / 2 + t];
  if (MODE == 3) {
#pragma unroll
    for (int t = 0; t < CH; ++t) k.x[t] = k.v[t];
  } else {
#pragma unroll
    for (int t = 0; t < CH; ++t) k.x[t] = x[(int64_t)k.c[t] * D + lane];
  }
}

template <int D, int MODE>
__device__ __forceinline__ void apply(float* acc, int lane, const Chunk<MODE>& k) {
  if (MODE == 2) {  // no LDS: one register chain
    float a = acc[lane];
#pragma unroll
    for (int t = 0; t < CH; ++t) a = __builtin_fmaf(k.v[t], k.x[t], a);
    acc[lane] = a;
    return;
  }
  int mm[CH];
#pragma unroll
  for (int t = 0; t < CH; ++t) mm[t] = (t & 1) ? (k.m[t / 2] >> 16) : (k.m[t / 2] & 0xffff);
  float av[CH];
#pragma unroll
  for (int t = 0; t < CH; ++t) av[t] = acc[(mm[t] & 2047) * D + lane];
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    float base = av[t];
    if (MODE == 0 || MODE == 3) {
      const int pv = mm[t] >> 11;
      if (t > 0 && pv) {
#pragma unroll
        for (int q = 0; q < t; ++q) base = (pv == q + 1) ? av[q] : base;
      }
    }
    av[t] = __builtin_fmaf(k.v[t], k.x[t], base);
  }
#pragma unroll
  for (int t = 0; t < CH; ++t) acc[(mm[t] & 2047) * D + lane] = av[t];
}

// MODE 0: chunks may repeat a row (select chain); MODE 1: rows distinct inside a chunk;
// diagnostics: MODE 2 = no LDS accumulators (one register chain), MODE 3 = no gathers.
template <int D, int MODE>
__global__ __launch_bounds__(NW * 64) void tiled_hop(
    const int32_t* __restrict__ scol, const float* __restrict__ sval,
    const uint32_t* __restrict__ smeta, const int64_t* __restrict__ sptr,  // [blocks*NW+1]
    const float* __restrict__ x, float* __restrict__ y, int64_t n_rows, int R, int n_blocks) {
  extern __shared__ float acc[];  // [(R+1)][D]
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int blk = blockIdx.x; blk < n_blocks; blk += gridDim.x) {
    for (int i = threadIdx.x; i < (R + 1) * D; i += NW * 64) acc[i] = 0.f;
    __syncthreads();
    const int64_t s = (int64_t)blk * NW + w;
    const int64_t b = sptr[s], e = sptr[s + 1];
    if (b < e) {
      Chunk<MODE> A, B;
      int64_t c = b;
      fetch<D>(scol, sval, smeta, c, x, lane, A);
      for (;;) {
        fetch<D>(scol, sval, smeta, c + CH, x, lane, B);
        apply<D>(acc, lane, A);
        c += CH;
        if (c >= e) break;
        fetch<D>(scol, sval, smeta, c + CH, x, lane, A);
        apply<D>(acc, lane, B);
        c += CH;
        if (c >= e) break;
      }
    }
    __syncthreads();
    const int64_t r0 = (int64_t)blk * R;
    for (int i = w; i < R; i += NW) {
      const int64_t r = r0 + i;
      if (r < n_rows) y[r * D + lane] = acc[i * D + lane];
    }
    __syncthreads();
  }
}

extern "C" int exp_tiled_hop(int mode, const int32_t* scol, const float* sval,
                             const uint32_t* smeta, const int64_t* sptr, const float* x, float* y,
                             int64_t n_rows, int R, int n_blocks, int grid, hipStream_t st) {
  const size_t lds = (size_t)(R + 1) * 64 * sizeof(float);
  auto k = mode == 0 ? tiled_hop<64, 0> : mode == 1 ? tiled_hop<64, 1>
          : mode == 2 ? tiled_hop<64, 2> : tiled_hop<64, 3>;
  if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                          160 * 1024) != hipSuccess)
    return -1;
  hipLaunchKernelGGL(k, dim3(grid), dim3(NW * 64), lds, st, scol, sval, smeta, sptr, x, y,
                     n_rows, R, n_blocks);
  return (int)hipGetLastError();
}

// ---- v2: panel-stepped streams (tools/exp_tiled_build.cpp) --------------------------------
// Slots: xoff uint32 (byte offset of the source row in x), val f32, meta u16 = row | bar<<10.
// Rows inside a chunk are distinct (no chain); bar (slot 0) = barriers before the chunk.
struct Chunk2 {
  uint32_t o[CH];
  float v[CH];
  uint32_t m[CH / 2];
  float x[CH];
};

template <int GMODE>
__device__ __forceinline__ void fetch2(const uint32_t* __restrict__ sx,
                                       const float* __restrict__ sv,
                                       const uint32_t* __restrict__ sm, int64_t c,
                                       __amdgpu_buffer_rsrc_t xr, int lane, Chunk2& k) {
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    k.o[t] = sx[c + t];
    k.v[t] = sv[c + t];
  }
#pragma unroll
  for (int t = 0; t < CH / 2; ++t) k.m[t] = sm[c / 2 + t];
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    if (GMODE == 1) {
      k.x[t] = k.v[t];
    } else {
      k.x[t] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(xr, lane * 4, k.o[t], 0));
    }
  }
}

struct Pace {
  unsigned* ctr;   // this workgroup's group counter (own 128-B line)
  unsigned target_per_step;  // workgroups in the group
  int gs;          // steps this workgroup has completed (all passes)
  int slack;
};

// Pacing (speed only, never correctness): before a step barrier, wave 0 reports the finished
// step to its XCD group's counter and waits (bounded) until the group's average is within
// `slack` steps, so the group's workgroups sweep the same source panel together.
__device__ __forceinline__ void pace_step(Pace& p, int w, int lane) {
  ++p.gs;
  if (p.ctr && w == 0) {
    if (lane == 0) {
      __hip_atomic_fetch_add(p.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const long long need = (long long)p.target_per_step * (p.gs - p.slack);
      const unsigned long long t0 = wall_clock64();
      while ((long long)__hip_atomic_load(p.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need &&
             wall_clock64() - t0 < 2000) {  // 100 MHz clock: <= 20 us
        __builtin_amdgcn_s_sleep(2);
      }
    }
  }
}

template <int GMODE>
__device__ __forceinline__ void apply2(float* acc, int lane, const Chunk2& k, int& cur, Pace& pc,
                                       int w) {
  const int bar = (k.m[0] >> 10) & 31;
  for (int i = 0; i < bar; ++i) {
    pace_step(pc, w, lane);
    __syncthreads();
  }
  cur += bar;
  int rr[CH];
#pragma unroll
  for (int t = 0; t < CH; ++t) rr[t] = ((t & 1) ? (k.m[t / 2] >> 16) : k.m[t / 2]) & 1023;
  float av[CH];
#pragma unroll
  for (int t = 0; t < CH; ++t) av[t] = acc[rr[t] * 64 + lane];
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    float base = av[t];
    if (t > 0) {
      const bool chain = ((t & 1) ? (k.m[t / 2] >> 31) : (k.m[t / 2] >> 15)) & 1;
      base = chain ? av[t - 1] : base;
    }
    av[t] = __builtin_fmaf(k.v[t], k.x[t], base);
  }
#pragma unroll
  for (int t = 0; t < CH; ++t) acc[rr[t] * 64 + lane] = av[t];
}

// GMODE 0: real; 1: no gathers (diagnostic). ADDTID: acc stores by ds_write_addtid_b32.
// With a counter, wave NW-1 is a pacer (no edges): before each step barrier it waits (bounded)
// until its XCD group's workgroups are within `slack` steps, and reports each finished step.
template <int GMODE, bool ADDTID>
__device__ __forceinline__ void apply3(float* acc, int lane, const Chunk2& k, int& cur) {
  const int bar = (k.m[0] >> 10) & 31;
  for (int i = 0; i < bar; ++i) __syncthreads();
  cur += bar;
  int rr[CH];
#pragma unroll
  for (int t = 0; t < CH; ++t) rr[t] = ((t & 1) ? (k.m[t / 2] >> 16) : k.m[t / 2]) & 1023;
  float av[CH];
#pragma unroll
  for (int t = 0; t < CH; ++t) av[t] = acc[rr[t] * 64 + lane];
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    float base = av[t];
    if (t > 0) {
      const bool chain = ((t & 1) ? (k.m[t / 2] >> 31) : (k.m[t / 2] >> 15)) & 1;
      base = chain ? av[t - 1] : base;
    }
    av[t] = __builtin_fmaf(k.v[t], k.x[t], base);
  }
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    if (ADDTID) {
      asm volatile("s_mov_b32 m0, %0\n\tds_write_addtid_b32 %1" ::"s"(rr[t] * 256), "v"(av[t])
                   : "memory");
    } else {
      acc[rr[t] * 64 + lane] = av[t];
    }
  }
}

template <int GMODE, bool ADDTID>
__global__ __launch_bounds__(NW * 64) void stepped_hop(
    const uint32_t* __restrict__ sx, const float* __restrict__ sv,
    const uint32_t* __restrict__ sm, const int64_t* __restrict__ wptr,
    const int32_t* __restrict__ nsteps, const float* __restrict__ x, int64_t x_bytes,
    float* __restrict__ y, int64_t n_rows, int R, int n_blocks, unsigned* ctr, int slack) {
  extern __shared__ float acc[];  // [(R+1)][64]
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // slack < 0: no pacer wave; instead the workgroups of a blockIdx%8 group meet at every
  // block (pass) start (counter barrier, bounded wait)
  const bool pass_sync = ctr && slack < 0;
  const int nwc = (ctr && !pass_sync) ? NW - 1 : NW;  // waves carrying edges
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0, (int)x_bytes, 0x00020000);
  if (pass_sync) {
    unsigned* c = ctr + (blockIdx.x % 8) * 32;
    const long long G = gridDim.x / 8 + ((blockIdx.x % 8) < (gridDim.x % 8) ? 1 : 0);
    long long p = 0;
    for (int blk = blockIdx.x; blk < n_blocks; blk += gridDim.x, ++p) {
      if (threadIdx.x == 0 && p > 0) {
        __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long t0 = wall_clock64();
        while ((long long)__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                   G * p && wall_clock64() - t0 < 20000)   // <= 200 us
          __builtin_amdgcn_s_sleep(2);
      }
      for (int i = threadIdx.x; i < (R + 1) * 64; i += NW * 64) acc[i] = 0.f;
      __syncthreads();  // B0
      const int64_t s = (int64_t)blk * NW + w;
      const int64_t b = wptr[s], e = wptr[s + 1];
      int cur = 0;
      if (b < e) {
        Chunk2 A, B;
        int64_t cc = b;
        fetch2<GMODE>(sx, sv, sm, cc, xr, lane, A);
        for (;;) {
          fetch2<GMODE>(sx, sv, sm, cc + CH, xr, lane, B);
          apply3<GMODE, ADDTID>(acc, lane, A, cur);
          cc += CH;
          if (cc >= e) break;
          fetch2<GMODE>(sx, sv, sm, cc + CH, xr, lane, A);
          apply3<GMODE, ADDTID>(acc, lane, B, cur);
          cc += CH;
          if (cc >= e) break;
        }
      }
      const int ns = nsteps[blk];
      for (int i = cur; i < ns; ++i) __syncthreads();
      const int64_t r0 = (int64_t)blk * R;
      for (int i = w; i < R; i += NW) {
        const int64_t r = r0 + i;
        if (r < n_rows) y[r * 64 + lane] = acc[i * 64 + lane];
      }
      __syncthreads();  // B_end
    }
    if (threadIdx.x == 0)
      __hip_atomic_fetch_add(c, 1u << 24, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (w == nwc) {  // pacer
    unsigned* c = ctr + (blockIdx.x % 8) * 32;
    const long long G = gridDim.x / 8 + ((blockIdx.x % 8) < (gridDim.x % 8) ? 1 : 0);
    long long gs = 0;
    for (int blk = blockIdx.x; blk < n_blocks; blk += gridDim.x) {
      __syncthreads();  // B0
      const int ns = nsteps[blk];
      for (int s = 0; s < ns; ++s) {
        if (lane == 0) {
          const long long need = G * (gs - slack);
          const unsigned long long t0 = wall_clock64();
          while ((long long)__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                     need && wall_clock64() - t0 < 2000)
            __builtin_amdgcn_s_sleep(1);
        }
        __syncthreads();
        ++gs;
        if (lane == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();  // B_end
    }
    if (lane == 0) __hip_atomic_fetch_add(c, 1u << 24, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  for (int blk = blockIdx.x; blk < n_blocks; blk += gridDim.x) {
    for (int i = threadIdx.x; i < (R + 1) * 64; i += nwc * 64) acc[i] = 0.f;
    __syncthreads();  // B0
    const int64_t s = (int64_t)blk * nwc + w;
    const int64_t b = wptr[s], e = wptr[s + 1];
    int cur = 0;
    if (b < e) {
      Chunk2 A, B;
      int64_t c = b;
      fetch2<GMODE>(sx, sv, sm, c, xr, lane, A);
      for (;;) {
        fetch2<GMODE>(sx, sv, sm, c + CH, xr, lane, B);
        apply3<GMODE, ADDTID>(acc, lane, A, cur);
        c += CH;
        if (c >= e) break;
        fetch2<GMODE>(sx, sv, sm, c + CH, xr, lane, A);
        apply3<GMODE, ADDTID>(acc, lane, B, cur);
        c += CH;
        if (c >= e) break;
      }
    }
    const int ns = nsteps[blk];
    for (int i = cur; i < ns; ++i) __syncthreads();  // remaining step barriers + final
    const int64_t r0 = (int64_t)blk * R;
    for (int i = w; i < R; i += nwc) {
      const int64_t r = r0 + i;
      if (r < n_rows) y[r * 64 + lane] = acc[i * 64 + lane];
    }
    __syncthreads();  // B_end
  }
}

extern "C" int exp_stepped_hop(int mode, const uint32_t* sx, const float* sv, const uint32_t* sm,
                               const int64_t* wptr, const int32_t* nsteps, const float* x,
                               int64_t x_bytes, float* y, int64_t n_rows, int R, int n_blocks,
                               int grid, unsigned* ctr, int slack, hipStream_t st) {
  const size_t lds = (size_t)(R + 1) * 64 * sizeof(float);
  auto k = mode == 1 ? stepped_hop<1, false> : mode == 2 ? stepped_hop<0, true>
                                              : stepped_hop<0, false>;
  if (ctr) hipMemsetAsync(ctr, 0, 8 * 128, st);
  if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                          160 * 1024) != hipSuccess)
    return -1;
  hipLaunchKernelGGL(k, dim3(grid), dim3(NW * 64), lds, st, sx, sv, sm, wptr, nsteps, x, x_bytes,
                     y, n_rows, R, n_blocks, ctr, slack);
  return (int)hipGetLastError();
}
