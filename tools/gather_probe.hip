// Gather-rate probe (not product code): how fast can a CU pull random fixed-size segments of
// a table through L2, by segment size? Each wave instruction gathers 64 lanes x 4 B as
// 64/SEG_LANES segments of SEG_LANES*4 bytes at random segment-aligned offsets; 16 loads in
// flight per wave; 16 waves per CU. Prints GB/s for each (segment size, table size).
//   hipcc --offload-arch=gfx950 -O3 tools/gather_probe.hip -o /tmp/gather_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);        \
      return 1;                                                               \
    }                                                                         \
  } while (0)

template <int SEG_LANES>
__global__ __launch_bounds__(1024) void probe(const float* __restrict__ t, unsigned n_seg,
                                              int iters, unsigned seed, float* out) {
  const int lane = threadIdx.x & 63;
  const int seg = lane / SEG_LANES, f = lane % SEG_LANES;
  unsigned s = seed * 2654435761u + blockIdx.x * 97u + (threadIdx.x >> 6) * 131u;
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      s = s * 1664525u + 1013904223u;
      // wave-uniform random base, one random segment per lane group
      unsigned r = (s ^ (unsigned)(seg * 0x9E3779B9u)) * 2246822519u;
      unsigned idx = (r >> 7) % n_seg;
      v[k] = t[(size_t)idx * SEG_LANES + f];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += v[k];
  }
  if (acc == 12345.f) out[0] = acc;
}

template <int SEG>
int run(const float* t, size_t table_bytes, float* out, int iters) {
  const unsigned n_seg = (unsigned)(table_bytes / (SEG * 4));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(probe<SEG>, dim3(256), dim3(1024), 0, 0, t, n_seg, 1, 1u, out);
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(probe<SEG>, dim3(256), dim3(1024), 0, 0, t, n_seg, iters, 7u, out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double bytes = 256.0 * 1024 * iters * 16 * 4;   // every lane loads 4 B
  printf("{\"segment_bytes\": %d, \"table_MB\": %.1f, \"ms\": %.3f, \"GBps\": %.1f}\n", SEG * 4,
         table_bytes / 1e6, ms, bytes / ms / 1e6);
  return 0;
}

int main() {
  const size_t max_bytes = (size_t)1 << 30;
  float* t;
  float* out;
  CHECK(hipMalloc(&t, max_bytes));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(t, 0, max_bytes));
  for (size_t tb : {(size_t)1 << 20, (size_t)256 << 20, (size_t)1 << 30}) {
    if (run<8>(t, tb, out, 200)) return 1;    // 32-B segments
    if (run<16>(t, tb, out, 200)) return 1;   // 64-B
    if (run<32>(t, tb, out, 200)) return 1;   // 128-B
    if (run<64>(t, tb, out, 200)) return 1;   // 256-B
  }
  return 0;
}
