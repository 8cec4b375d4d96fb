// Dependent fp32 FMA chain latency on gfx950, one wave: cycles per fmaf of a chain of N
// dependent v_fma_f32 (the heavy-row consumer's per-neighbour floor), for 1, 2
// and 4 interleaved independent chains per lane, and with a ds_read_b32 feeding each fmaf.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/fma_latency.hip -o tools/bin/fma_latency
#include <hip/hip_runtime.h>
#include <cstdio>

// 32 steps per loop iteration (unrolled: the loop's scalar overhead spread over 32 fmafs per
// chain), CHAINS independent accumulators interleaved
template <int CHAINS>
__global__ void chain_kernel(const float* __restrict__ in, float* out, long long* cyc, int n) {
  float a[CHAINS];
  for (int c = 0; c < CHAINS; ++c) a[c] = in[threadIdx.x + c];
  const float v = in[64 + threadIdx.x], x = in[128 + threadIdx.x];
  const long long t0 = clock64();
  for (int i = 0; i < n; i += 32) {
#pragma unroll
    for (int u = 0; u < 32; ++u) {
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) a[c] = __builtin_fmaf(v, a[c], x);
    }
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int c = 0; c < CHAINS; ++c) s += a[c];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// v_fmac_f32_dpp row_newbcast chain (the group consumer's instruction), and a chain whose
// multiplier is an SGPR (a value broadcast without DPP)
#define DPP1(T) asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:" #T " row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a) : "v"(v), "v"(x));
__global__ void dpp_chain_kernel(const float* __restrict__ in, float* out, long long* cyc, int n) {
  float a = in[threadIdx.x];
  const float v = in[64 + threadIdx.x], x = in[128 + threadIdx.x];
  const long long t0 = clock64();
  for (int i = 0; i < n; i += 16) {
    DPP1(0) DPP1(1) DPP1(2) DPP1(3) DPP1(4) DPP1(5) DPP1(6) DPP1(7)
    DPP1(8) DPP1(9) DPP1(10) DPP1(11) DPP1(12) DPP1(13) DPP1(14) DPP1(15)
  }
  const long long t1 = clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
#undef DPP1

__global__ void sgpr_chain_kernel(const float* __restrict__ in, float* out, long long* cyc, int n) {
  float a = in[threadIdx.x];
  const float x = in[128 + threadIdx.x];
  float s[16];
  for (int t = 0; t < 16; ++t)
    s[t] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, in[64 + t])));
  const long long t0 = clock64();
  for (int i = 0; i < n; i += 16) {
#pragma unroll
    for (int t = 0; t < 16; ++t) a = __builtin_fmaf(s[t], x, a);
  }
  const long long t1 = clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// The heavy-row consumer's inner loop in isolation (one wave, lane = feature of a 16-feature
// slice, a chunk of 1008 neighbours parked feature-major with stride S = 1012, the values in
// their own array): cycles per neighbour of
//   MODE 0: 16-neighbour groups, one ds_read_b32 of values + DPP row_newbcast v_fmac (shipped)
//   MODE 1: NB-neighbour groups, values as broadcast ds_read_b128 (every lane the same
//           address), features as aligned ds_read_b128, plain v_fmac_f32
template <int MODE, int NB, int GA>
__global__ void consumer_kernel(const float* __restrict__ in, float* out, long long* cyc, int reps) {
  constexpr int CHK = 1008, S = 1012;
  __shared__ float xb[16 * S];
  __shared__ float vb[CHK + 64];
  for (int i = threadIdx.x; i < 16 * S; i += 64) xb[i] = in[i & 4095] * 0.5f;
  for (int i = threadIdx.x; i < CHK + 64; i += 64) vb[i] = in[(i + 7) & 4095] * 0.25f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int fo = (lane & 15) * S;
  float a = 0.f;
  const long long t0 = clock64();
  for (int rep = 0; rep < reps; ++rep) {
    if constexpr (MODE == 0) {
      struct G { float v; float4 x[4]; };
      auto fetch = [&](int j, G& g) {
        g.v = vb[j + (lane & 15)];
#pragma unroll
        for (int q = 0; q < 4; ++q) g.x[q] = *reinterpret_cast<const float4*>(xb + fo + j + 4 * q);
      };
#define F1(X, T) asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:" #T " row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a) : "v"(g.v), "v"(X));
#define G4(Q, T0, T1, T2, T3) F1(g.x[Q].x, T0) F1(g.x[Q].y, T1) F1(g.x[Q].z, T2) F1(g.x[Q].w, T3)
      auto apply = [&](const G& g) { G4(0, 0, 1, 2, 3) G4(1, 4, 5, 6, 7) G4(2, 8, 9, 10, 11) G4(3, 12, 13, 14, 15) };
#undef G4
#undef F1
      G g[GA];
      for (int i = 0; i < GA; ++i) fetch(16 * i, g[i]);
      for (int q = 0; q + GA <= CHK / 16; q += GA) {
#pragma unroll
        for (int i = 0; i < GA; ++i) {
          apply(g[i]);
          fetch(16 * (q + i + GA), g[i]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else {
      constexpr int NQ = NB / 4;
      struct G { float4 v[NQ]; float4 x[NQ]; };
      auto fetch = [&](int j, G& g) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          g.v[q] = *reinterpret_cast<const float4*>(vb + j + 4 * q);
          g.x[q] = *reinterpret_cast<const float4*>(xb + fo + j + 4 * q);
        }
      };
      auto apply = [&](const G& g) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          a = __builtin_fmaf(g.v[q].x, g.x[q].x, a);
          a = __builtin_fmaf(g.v[q].y, g.x[q].y, a);
          a = __builtin_fmaf(g.v[q].z, g.x[q].z, a);
          a = __builtin_fmaf(g.v[q].w, g.x[q].w, a);
        }
      };
      G g[GA];
      for (int i = 0; i < GA; ++i) fetch(NB * i, g[i]);
      for (int q = 0; q + GA <= CHK / NB; q += GA) {
#pragma unroll
        for (int i = 0; i < GA; ++i) {
          apply(g[i]);
          fetch(NB * (q + i + GA), g[i]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  }
  const long long t1 = clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// The broadcast consumer (8-neighbour groups, 3 in flight) in the heavy kernel's environment:
// dynamic LDS laid out as the kernel's (two 64-KB feature buffers, then the value buffers),
// reading buffer BUF; THREADS 64 or 512 (the other waves wait at a barrier, or with PARK
// write the other buffer feature-major, as the loaders park, for PARK rounds first)
template <int BUF, int THREADS, int PARK>
__global__ __launch_bounds__(512) void consumer_env_kernel(const float* __restrict__ in, float* out,
                                                           long long* cyc, int reps) {
  constexpr int CHK = 1008, S = 1012;
  extern __shared__ float lds[];
  float* xb = lds + BUF * 16384;
  float* vb = lds + 2 * 16384 + BUF * 1024;
  for (int i = threadIdx.x; i < 2 * 16384 + 2 * 1024 + 64; i += THREADS) lds[i] = in[i & 4095] * 0.5f;
  __syncthreads();
  if (threadIdx.x >= 64) {
    float* ob = lds + (1 - BUF) * 16384;
    const int lt = threadIdx.x - 64;
    for (int r = 0; r < PARK; ++r)
      for (int i = 0; i < 10; ++i) {
        const int p = lt + i * (THREADS - 64), j = p % CHK, f = (p / CHK) & 3;
        ob[(4 * f + 0) * S + j] = in[p & 4095];
        ob[(4 * f + 1) * S + j] = in[(p + 1) & 4095];
        ob[(4 * f + 2) * S + j] = in[(p + 2) & 4095];
        ob[(4 * f + 3) * S + j] = in[(p + 3) & 4095];
      }
    __syncthreads();
    return;
  }
  const int lane = threadIdx.x & 63;
  const int fo = min(lane, 15) * S;
  float a = 0.f;
  const long long t0 = clock64(), w0 = wall_clock64();
  for (int rep = 0; rep < reps; ++rep) {
    struct G { float4 v[2]; float4 x[2]; };
    auto fetch = [&](int j, G& g) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        g.v[q] = *reinterpret_cast<const float4*>(vb + j + 4 * q);
        g.x[q] = *reinterpret_cast<const float4*>(xb + fo + j + 4 * q);
      }
    };
    auto apply = [&](const G& g) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        a = __builtin_fmaf(g.v[q].x, g.x[q].x, a);
        a = __builtin_fmaf(g.v[q].y, g.x[q].y, a);
        a = __builtin_fmaf(g.v[q].z, g.x[q].z, a);
        a = __builtin_fmaf(g.v[q].w, g.x[q].w, a);
      }
    };
    G g[3];
    for (int i = 0; i < 3; ++i) fetch(8 * i, g[i]);
    for (int q = 0; q + 3 <= CHK / 8; q += 3) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        apply(g[i]);
        fetch(8 * (q + i + 3), g[i]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  const long long t1 = clock64(), w1 = wall_clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = w1 - w0;
  }
  __syncthreads();
}

// values through v_readlane_b32 into an SGPR, then v_fmac with the SGPR operand
__global__ void readlane_chain_kernel(const float* __restrict__ in, float* out, long long* cyc, int n) {
  float a = in[threadIdx.x];
  const float x = in[128 + threadIdx.x];
  const int vv = __builtin_bit_cast(int, in[64 + threadIdx.x]);
  const long long t0 = clock64();
  for (int i = 0; i < n; i += 16) {
#pragma unroll
    for (int t = 0; t < 16; ++t)
      a = __builtin_fmaf(__builtin_bit_cast(float, __builtin_amdgcn_readlane(vv, t + (i & 32))), x, a);
  }
  const long long t1 = clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// the group consumer with its values through v_readlane (one ds_read_b32 of 64 values per 64
// neighbours) and its features as 4 aligned ds_read_b128 per 16; kernel-like LDS layout
__global__ __launch_bounds__(64) void consumer_readlane_kernel(const float* __restrict__ in, float* out,
                                                               long long* cyc, int reps) {
  constexpr int CHK = 1008, S = 1012;
  extern __shared__ float lds[];
  float* xb = lds;
  float* vb = lds + 2 * 16384;
  for (int i = threadIdx.x; i < 2 * 16384 + 2 * 1024 + 64; i += 64) lds[i] = in[i & 4095] * 0.5f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int fo = min(lane, 15) * S;
  float a = 0.f;
  const long long t0 = clock64(), w0 = wall_clock64();
  for (int rep = 0; rep < reps; ++rep) {
    for (int j0 = 0; j0 + 64 <= CHK; j0 += 64) {
      const int vv = __builtin_bit_cast(int, vb[j0 + lane]);
      float4 x[2][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) x[0][q] = *reinterpret_cast<const float4*>(xb + fo + j0 + 4 * q);
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        if (gq < 3) {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            x[(gq + 1) & 1][q] = *reinterpret_cast<const float4*>(xb + fo + j0 + 16 * (gq + 1) + 4 * q);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 xv = x[gq & 1][q];
          a = __builtin_fmaf(__builtin_bit_cast(float, __builtin_amdgcn_readlane(vv, 16 * gq + 4 * q + 0)), xv.x, a);
          a = __builtin_fmaf(__builtin_bit_cast(float, __builtin_amdgcn_readlane(vv, 16 * gq + 4 * q + 1)), xv.y, a);
          a = __builtin_fmaf(__builtin_bit_cast(float, __builtin_amdgcn_readlane(vv, 16 * gq + 4 * q + 2)), xv.z, a);
          a = __builtin_fmaf(__builtin_bit_cast(float, __builtin_amdgcn_readlane(vv, 16 * gq + 4 * q + 3)), xv.w, a);
        }
      }
    }
  }
  const long long t1 = clock64(), w1 = wall_clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = w1 - w0;
  }
}

// values as SGPR operands straight from global memory (s_load, uniform addresses) and the
// features from LDS (kernel-like layout): 2 groups of 16 neighbours per batch, the next batch's
// s_loads and ds_reads issued before this batch's chain; PF: also touch the values PF batches
// ahead with one s_load_dword (warming the scalar cache)
template <int PF>
__global__ __launch_bounds__(64) void consumer_sgpr_kernel(const float* __restrict__ in,
                                                           const float* __restrict__ vals,
                                                           float* out, long long* cyc, int reps) {
  constexpr int CHK = 1008, S = 1012, NB = 32;
  extern __shared__ float lds[];
  float* xb = lds;
  for (int i = threadIdx.x; i < 2 * 16384; i += 64) lds[i] = in[i & 4095] * 0.5f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int fo = min(lane, 15) * S;
  float a = 0.f;
  unsigned sink = 0;
  const long long t0 = clock64(), w0 = wall_clock64();
  for (int rep = 0; rep < reps; ++rep) {
    const float* vr = vals + (rep & 7) * 1024;
    float vc[NB];
    float4 xc[NB / 4];
#pragma unroll
    for (int t = 0; t < NB; ++t) vc[t] = vr[t];
#pragma unroll
    for (int q = 0; q < NB / 4; ++q) xc[q] = *reinterpret_cast<const float4*>(xb + fo + 4 * q);
    for (int j0 = 0; j0 + NB <= CHK; j0 += NB) {
      float vn[NB];
      float4 xn[NB / 4];
#pragma unroll
      for (int t = 0; t < NB; ++t) vn[t] = vr[j0 + NB + t];
#pragma unroll
      for (int q = 0; q < NB / 4; ++q) xn[q] = *reinterpret_cast<const float4*>(xb + fo + j0 + NB + 4 * q);
      if (PF) sink += __builtin_bit_cast(unsigned, vr[j0 + PF * NB]);
#pragma unroll
      for (int q = 0; q < NB / 4; ++q) {
        a = __builtin_fmaf(vc[4 * q + 0], xc[q].x, a);
        a = __builtin_fmaf(vc[4 * q + 1], xc[q].y, a);
        a = __builtin_fmaf(vc[4 * q + 2], xc[q].z, a);
        a = __builtin_fmaf(vc[4 * q + 3], xc[q].w, a);
      }
#pragma unroll
      for (int t = 0; t < NB; ++t) vc[t] = vn[t];
#pragma unroll
      for (int q = 0; q < NB / 4; ++q) xc[q] = xn[q];
    }
  }
  const long long t1 = clock64(), w1 = wall_clock64();
  out[threadIdx.x] = a + (sink == 12345u ? 1.f : 0.f);
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = w1 - w0;
  }
}

// core clock against the 100 MHz wall clock (cycles figures -> ns)
__global__ void clock_rate_kernel(long long* cyc, int n) {
  const long long c0 = clock64(), w0 = wall_clock64();
  float a = 1.f;
  for (int i = 0; i < n; ++i) a = __builtin_fmaf(a, 0.999999f, 1e-7f);
  const long long c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) {
    cyc[0] = c1 - c0;
    cyc[1] = w1 - w0;
    cyc[2] = a > 1e30f;
  }
}

// the consumer's shape: per step 4 neighbours, values read from LDS (broadcast), features from
// LDS (two b64 reads), 4 dependent fmafs on ONE accumulator; LDS reads issued P steps ahead
__global__ void lds_chain_kernel(const float* __restrict__ in, float* out, long long* cyc, int n) {
  __shared__ float buf[4096];
  __shared__ float vals[1024];
  for (int i = threadIdx.x; i < 4096; i += 64) buf[i] = in[i & 255] * 0.5f;
  for (int i = threadIdx.x; i < 1024; i += 64) vals[i] = in[(i + 7) & 255] * 0.25f;
  __syncthreads();
  float a = 0.f;
  const int fo = threadIdx.x * 16;
  const long long t0 = clock64();
  for (int rep = 0; rep < n; ++rep) {
    for (int j = 0; j < 1024; j += 4) {
      const float4 v = *reinterpret_cast<const float4*>(vals + j);
      const float2 x0 = *reinterpret_cast<const float2*>(buf + ((fo + j) & 4095));
      const float2 x1 = *reinterpret_cast<const float2*>(buf + ((fo + j + 2) & 4095));
      a = __builtin_fmaf(v.x, x0.x, a);
      a = __builtin_fmaf(v.y, x0.y, a);
      a = __builtin_fmaf(v.z, x1.x, a);
      a = __builtin_fmaf(v.w, x1.y, a);
    }
  }
  const long long t1 = clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  float *in, *out;
  long long* cyc;
  hipMalloc(&in, 4096 * sizeof(float));
  hipMalloc(&out, 64 * sizeof(float));
  hipMalloc(&cyc, 4 * sizeof(long long));
  float h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = 0.999f + 1e-6f * (i % 17);
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  const int n = 1 << 16;
  long long c = 0;
  auto run = [&](auto kern, const char* name, long long fmas) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, in, out, cyc, n);
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, in, out, cyc, n);
    hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("{\"case\": \"%s\", \"cycles\": %lld, \"cycles_per_fmaf_per_chain\": %.3f}\n", name, c,
           (double)c / (double)fmas);
  };
  run(chain_kernel<1>, "chain1", (long long)n);
  run(chain_kernel<2>, "chain2", (long long)n);
  run(chain_kernel<4>, "chain4", (long long)n);
  run(chain_kernel<8>, "chain8", (long long)n);
  run(dpp_chain_kernel, "dpp_fmac_chain", (long long)n);
  run(sgpr_chain_kernel, "sgpr_fmac_chain", (long long)n);
  run(readlane_chain_kernel, "readlane_fmac_chain", (long long)n);
  {
    long long cw[3];
    hipLaunchKernelGGL(clock_rate_kernel, dim3(1), dim3(64), 0, 0, cyc, 1 << 22);
    hipLaunchKernelGGL(clock_rate_kernel, dim3(1), dim3(64), 0, 0, cyc, 1 << 22);
    hipMemcpy(cw, cyc, sizeof(cw), hipMemcpyDeviceToHost);
    printf("{\"case\": \"clock\", \"core_cycles\": %lld, \"wall_ticks_100mhz\": %lld, \"core_ghz\": %.3f}\n",
           cw[0], cw[1], (double)cw[0] / (double)cw[1] / 10.0);
  }
  {
    auto cons = [&](auto kern, const char* name) {
      const int r = 32;
      hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, in, out, cyc, r);
      hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, in, out, cyc, r);
      hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
      printf("{\"case\": \"%s\", \"cycles_per_neighbour\": %.3f}\n", name, (double)c / (r * 1008.0));
    };
    cons(consumer_kernel<0, 16, 2>, "consumer_dpp_g16_ga2");
    cons(consumer_kernel<0, 16, 3>, "consumer_dpp_g16_ga3");
    cons(consumer_kernel<1, 8, 3>, "consumer_bcast_g8_ga3");
    cons(consumer_kernel<1, 8, 2>, "consumer_bcast_g8_ga2");
    cons(consumer_kernel<1, 4, 4>, "consumer_bcast_g4_ga4");
    cons(consumer_kernel<1, 16, 1>, "consumer_bcast_g16_ga1");
    const size_t lds = (2 * 16384 + 2 * 1024 + 64) * sizeof(float);
    auto env = [&](auto kern, int threads, const char* name) {
      hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      const int r = 32;
      hipLaunchKernelGGL(kern, dim3(1), dim3(threads), lds, 0, in, out, cyc, r);
      hipLaunchKernelGGL(kern, dim3(1), dim3(threads), lds, 0, in, out, cyc, r);
      long long cw[2];
      hipMemcpy(cw, cyc, sizeof(cw), hipMemcpyDeviceToHost);
      printf("{\"case\": \"%s\", \"cycles_per_neighbour\": %.3f, \"ns_per_neighbour\": %.3f, \"err\": \"%s\"}\n",
             name, (double)cw[0] / (r * 1008.0), 10.0 * (double)cw[1] / (r * 1008.0),
             hipGetErrorString(hipGetLastError()));
    };
    env(consumer_readlane_kernel, 64, "env_readlane_1wave");
    {
      float* vals;
      hipMalloc(&vals, 8 * 1024 * sizeof(float) + 4096);
      hipMemcpy(vals, h, 4096 * sizeof(float), hipMemcpyHostToDevice);
      hipMemcpy(vals + 4096, h, 4096 * sizeof(float), hipMemcpyHostToDevice);
      auto sg = [&](auto kern, const char* name) {
        hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        const int r = 32;
        hipLaunchKernelGGL(kern, dim3(1), dim3(64), lds, 0, in, vals, out, cyc, r);
        hipLaunchKernelGGL(kern, dim3(1), dim3(64), lds, 0, in, vals, out, cyc, r);
        long long cw[2];
        hipMemcpy(cw, cyc, sizeof(cw), hipMemcpyDeviceToHost);
        printf("{\"case\": \"%s\", \"cycles_per_neighbour\": %.3f, \"ns_per_neighbour\": %.3f, \"err\": \"%s\"}\n",
               name, (double)cw[0] / (r * 1008.0), 10.0 * (double)cw[1] / (r * 1008.0),
               hipGetErrorString(hipGetLastError()));
      };
      sg(consumer_sgpr_kernel<0>, "sgpr_values_nopf");
      sg(consumer_sgpr_kernel<4>, "sgpr_values_pf4");
      sg(consumer_sgpr_kernel<8>, "sgpr_values_pf8");
    }
    env(consumer_env_kernel<0, 64, 0>, 64, "env_buf0_1wave");
    env(consumer_env_kernel<1, 64, 0>, 64, "env_buf1_1wave");
    env(consumer_env_kernel<0, 512, 0>, 512, "env_buf0_8waves_idle");
    env(consumer_env_kernel<1, 512, 0>, 512, "env_buf1_8waves_idle");
    env(consumer_env_kernel<0, 512, 4>, 512, "env_buf0_8waves_park4");
    env(consumer_env_kernel<0, 512, 32>, 512, "env_buf0_8waves_park32");
  }
  const int reps = 64;
  hipLaunchKernelGGL(lds_chain_kernel, dim3(1), dim3(64), 0, 0, in, out, cyc, reps);
  hipLaunchKernelGGL(lds_chain_kernel, dim3(1), dim3(64), 0, 0, in, out, cyc, reps);
  hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  printf("{\"case\": \"lds_chain\", \"cycles\": %lld, \"cycles_per_neighbour\": %.3f}\n", c,
         (double)c / (double)(reps * 1024));
  return 0;
}
