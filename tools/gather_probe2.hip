// Gather-rate probe v2 (not product code): per-CU rate of random 128-B line gathers by load
// width. A wave instruction gathers 64 lanes x W bytes = 64*W/128 random 128-B lines (W = 4: 2
// lines, the tiled hop's raw_buffer_load_b32 form; W = 8: 4 lines; W = 16: 8 lines), through a
// buffer resource with 32-bit offsets as the hop does. Each wave keeps two batches of DEPTH
// instructions in flight (batch b+1 issued before batch b is consumed), 16 waves per CU, one
// 1024-thread workgroup per CU. Tables: power-of-two sizes so the line index is a mask.
//   hipcc --offload-arch=gfx950 -O3 tools/gather_probe2.hip -o tools/_var/gather_probe2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);        \
      return 1;                                                               \
    }                                                                         \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}

template <int W>
struct Vec;
template <>
struct Vec<4> {
  using T = float;
  __device__ static T load(__amdgpu_buffer_rsrc_t r, uint32_t o) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, o, 0, 0));
  }
  __device__ static float sum(T v) { return v; }
};
template <>
struct Vec<8> {
  using T = float __attribute__((ext_vector_type(2)));
  __device__ static T load(__amdgpu_buffer_rsrc_t r, uint32_t o) {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, o, 0, 0));
  }
  __device__ static float sum(T v) { return v.x + v.y; }
};
template <>
struct Vec<16> {
  using T = float __attribute__((ext_vector_type(4)));
  __device__ static T load(__amdgpu_buffer_rsrc_t r, uint32_t o) {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0));
  }
  __device__ static float sum(T v) { return (v.x + v.y) + (v.z + v.w); }
};

template <int W, int DEPTH>
__global__ __launch_bounds__(1024) void probe(const float* __restrict__ t, uint32_t line_mask,
                                              int iters, uint32_t seed, float* out) {
  constexpr int kLanesPerLine = 128 / W;
  using V = Vec<W>;
  const int lane = threadIdx.x & 63;
  const uint32_t grp = (uint32_t)(lane / kLanesPerLine);
  const uint32_t inl = (uint32_t)(lane % kLanesPerLine) * W;
  const uint32_t wid = blockIdx.x * 16 + (threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(t), 0, 0x7FFFFFFF, 0x00020000);
  uint32_t ctr = mix(seed ^ (wid * 0x9E3779B9u)) + grp * 0x632BE5ABu;
  float acc = 0.f;
  typename V::T a[DEPTH], b[DEPTH];
#pragma unroll
  for (int k = 0; k < DEPTH; ++k) a[k] = V::load(r, (mix(ctr + k * 977u) & line_mask) * 128u + inl);
  ctr += DEPTH * 977u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < DEPTH; ++k)
      b[k] = V::load(r, (mix(ctr + k * 977u) & line_mask) * 128u + inl);
    ctr += DEPTH * 977u;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) acc += V::sum(a[k]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < DEPTH; ++k)
      a[k] = V::load(r, (mix(ctr + k * 977u) & line_mask) * 128u + inl);
    ctr += DEPTH * 977u;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) acc += V::sum(b[k]);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (acc == 12345.f) out[0] = acc;
}

template <int W, int DEPTH>
int run(const float* t, size_t table_bytes, float* out, int cus) {
  const uint32_t lines = (uint32_t)(table_bytes / 128);
  constexpr int kLinesPerInstr = 64 * W / 128;
  // about 16 GB of lines per timed launch
  const double target = 16e9;
  const double per_iter = (double)cus * 16 * 2 * DEPTH * kLinesPerInstr * 128.0;
  const int iters = (int)(target / per_iter) + 1;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((probe<W, DEPTH>), dim3(cus), dim3(1024), 0, 0, t, lines - 1, 4, 1u, out);
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL((probe<W, DEPTH>), dim3(cus), dim3(1024), 0, 0, t, lines - 1, iters, 7u, out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double bytes = per_iter * iters;
  printf("{\"load_bytes\": %d, \"lines_per_instr\": %d, \"depth\": %d, \"table_MB\": %.1f, "
         "\"ms\": %.3f, \"TBps\": %.2f, \"GBps_per_CU\": %.1f}\n",
         W, kLinesPerInstr, DEPTH, table_bytes / 1e6, ms, bytes / ms / 1e9, bytes / ms / 1e6 / cus);
  fflush(stdout);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return 0;
}

int main(int argc, char** argv) {
  int cus = 256;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t max_bytes = (size_t)1 << 29;
  float* t;
  float* out;
  CHECK(hipMalloc(&t, max_bytes));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(t, 0, max_bytes));
  // optional argument: one table size in MiB (PMC runs), else the three of the sweep
  const size_t only = argc > 1 ? (size_t)atoi(argv[1]) << 20 : 0;
  for (size_t tb : {(size_t)2 << 20, (size_t)32 << 20, (size_t)512 << 20}) {
    if (only && tb != only) continue;
    if (run<4, 8>(t, tb, out, cus)) return 1;
    if (run<4, 16>(t, tb, out, cus)) return 1;
    if (run<8, 8>(t, tb, out, cus)) return 1;
    if (run<8, 16>(t, tb, out, cus)) return 1;
    if (run<16, 2>(t, tb, out, cus)) return 1;
    if (run<16, 4>(t, tb, out, cus)) return 1;
    if (run<16, 8>(t, tb, out, cus)) return 1;
  }
  return 0;
}
