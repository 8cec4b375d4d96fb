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
  hipMalloc(&cyc, sizeof(long long));
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
  const int reps = 64;
  hipLaunchKernelGGL(lds_chain_kernel, dim3(1), dim3(64), 0, 0, in, out, cyc, reps);
  hipLaunchKernelGGL(lds_chain_kernel, dim3(1), dim3(64), 0, 0, in, out, cyc, reps);
  hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  printf("{\"case\": \"lds_chain\", \"cycles\": %lld, \"cycles_per_neighbour\": %.3f}\n", c,
         (double)c / (double)(reps * 1024));
  return 0;
}
