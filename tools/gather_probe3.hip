// Gather-rate probe v3 (not product code): per-CU rate of random SECTOR gathers of S bytes
// (S = 128: whole lines, as the tiled hop; 64 / 32: half / quarter lines) with 16-B lanes,
// S / 16 lanes per sector, 64 * 16 / S random sectors per wave instruction, through a buffer
// resource with 32-bit offsets. Two batches of DEPTH instructions in flight per wave, 16 waves
// per CU. Question: is the beyond-L2 path limited by requests (a 64-B sector costs a 128-B
// line's slot) or by bytes?
//   hipcc --offload-arch=gfx950 -O3 tools/gather_probe3.hip -o tools/_var/gather_probe3
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

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ f4 ld(__amdgpu_buffer_rsrc_t r, uint32_t o) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0));
}

template <int S, int DEPTH>
__global__ __launch_bounds__(1024) void probe(const float* __restrict__ t, uint32_t sec_mask,
                                              int iters, uint32_t seed, float* out) {
  constexpr int kLanes = S / 16;
  const int lane = threadIdx.x & 63;
  const uint32_t grp = (uint32_t)(lane / kLanes);
  const uint32_t inl = (uint32_t)(lane % kLanes) * 16;
  const uint32_t wid = blockIdx.x * 16 + (threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(t), 0, 0x7FFFFFFF, 0x00020000);
  uint32_t ctr = mix(seed ^ (wid * 0x9E3779B9u)) + grp * 0x632BE5ABu;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  f4 a[DEPTH], b[DEPTH];
#pragma unroll
  for (int k = 0; k < DEPTH; ++k) a[k] = ld(r, (mix(ctr + k * 977u) & sec_mask) * S + inl);
  ctr += DEPTH * 977u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) b[k] = ld(r, (mix(ctr + k * 977u) & sec_mask) * S + inl);
    ctr += DEPTH * 977u;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) acc += a[k];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) a[k] = ld(r, (mix(ctr + k * 977u) & sec_mask) * S + inl);
    ctr += DEPTH * 977u;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < DEPTH; ++k) acc += b[k];
    __builtin_amdgcn_sched_barrier(0);
  }
  if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[0] = acc.x;
}

template <int S, int DEPTH>
int run(const float* t, size_t table_bytes, float* out, int cus) {
  const uint32_t secs = (uint32_t)(table_bytes / S);
  const double per_iter = (double)cus * 16 * 2 * DEPTH * 64 * 16.0;   // useful bytes
  const int iters = (int)(16e9 / per_iter) + 1;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((probe<S, DEPTH>), dim3(cus), dim3(1024), 0, 0, t, secs - 1, 4, 1u, out);
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL((probe<S, DEPTH>), dim3(cus), dim3(1024), 0, 0, t, secs - 1, iters, 7u, out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double bytes = per_iter * iters;
  printf("{\"sector_bytes\": %d, \"sectors_per_instr\": %d, \"depth\": %d, \"table_MB\": %.1f, "
         "\"ms\": %.3f, \"useful_TBps\": %.2f, \"GBps_per_CU\": %.1f, \"Gsectors_per_s\": %.1f}\n",
         S, 64 * 16 / S, DEPTH, table_bytes / 1e6, ms, bytes / ms / 1e9,
         bytes / ms / 1e6 / cus, bytes / S / ms / 1e6);
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
  const size_t only = argc > 1 ? (size_t)atoi(argv[1]) << 20 : 0;
  for (size_t tb : {(size_t)2 << 20, (size_t)32 << 20, (size_t)512 << 20}) {
    if (only && tb != only) continue;
    if (run<128, 4>(t, tb, out, cus)) return 1;
    if (run<64, 4>(t, tb, out, cus)) return 1;
    if (run<32, 4>(t, tb, out, cus)) return 1;
    if (run<128, 8>(t, tb, out, cus)) return 1;
    if (run<64, 8>(t, tb, out, cus)) return 1;
  }
  return 0;
}
