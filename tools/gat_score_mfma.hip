// GAT layer 3's shared-row scores, VALU vs matrix cores, one wave:
// cycles per block of 8 neighbours x 4 destination rows (a wave's work per softmax block).
//  VALU: the kernel's form (csrc/gat.hip shared_scores16): each lane holds 4 of the 64 features
//        of the 8 neighbour rows, 8 x 4 partial dot4s, reduce-scatter over the 16-lane group by
//        DPP — 2 passes of 8 x (2 dot4 + 1 DPP add) + 7 DPP adds.
//  MFMA: the same [32 x 64] x [64 x 4 -> padded 16] product as v_mfma_f32_16x16x4_f32 (2 M tiles
//        x 16 K steps = 32 MFMAs), the operands already in MFMA fragment layout — a lower bound
//        for the matrix-core form (it also needs the rows transposed through LDS).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/gat_score_mfma.hip -o gat_score_mfma
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float dot4(float4 a, float4 b) {
  return __builtin_fmaf(a.w, b.w, __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x)));
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, true));
}
constexpr int kRor8 = 0x128, kHalfMirror = 0x141, kXor2 = 0x4E /* quad perm 2,3,0,1 */,
              kXor1 = 0xB1 /* quad perm 1,0,3,2 */;

__global__ void valu_kernel(const float* __restrict__ in, float* out, long long* cyc, int blocks) {
  const int gl = threadIdx.x & 15;
  float4 xv[8], an[4];
  for (int t = 0; t < 8; ++t) xv[t] = make_float4(in[t * 64 + (threadIdx.x & 63)], in[t * 64 + (threadIdx.x & 63) + 1],
                                                  in[t * 64 + (threadIdx.x & 63) + 2], in[t * 64 + (threadIdx.x & 63) + 3]);
  for (int h = 0; h < 4; ++h) an[h] = make_float4(in[600 + h], in[601 + h], in[602 + h], in[603 + h]);
  const bool hi = gl >= 8, b2 = gl & 4, b1 = gl & 2, b0 = gl & 1;
  float acc = 0.f;
  const long long t0 = clock64();
  for (int b = 0; b < blocks; ++b) {
    float T[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float Q[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const float mine = dot4(xv[t], an[j]), other = dot4(xv[t], an[2 + j]);
        Q[t] = (hi ? other : mine) + dpp_f<kRor8>(hi ? mine : other);
      }
      float R[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) R[k] = (b2 ? Q[4 + k] : Q[k]) + dpp_f<kHalfMirror>(b2 ? Q[k] : Q[4 + k]);
      float S[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) S[k] = (b1 ? R[2 + k] : R[k]) + dpp_f<kXor2>(b1 ? R[k] : R[2 + k]);
      T[j] = (b0 ? S[1] : S[0]) + dpp_f<kXor1>(b0 ? S[0] : S[1]);
    }
    acc += T[0] * T[1];
    // perturb the inputs so the blocks are not folded together
#pragma unroll
    for (int t = 0; t < 8; ++t) xv[t].x += acc * 1e-30f;
  }
  const long long t1 = clock64();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void mfma_kernel(const float* __restrict__ in, float* out, long long* cyc, int blocks) {
  float a[2][16], bb[16];
  for (int k = 0; k < 16; ++k) {
    a[0][k] = in[k * 64 + (threadIdx.x & 63)];
    a[1][k] = in[1024 + k * 64 + (threadIdx.x & 63)];
    bb[k] = in[2048 + k * 64 + (threadIdx.x & 63)];
  }
  f4v c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
  const long long t0 = clock64();
  for (int b = 0; b < blocks; ++b) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0][k], bb[k], c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1][k], bb[k], c1, 0, 0, 0);
    }
    a[0][0] += c0.x * 1e-30f;   // a dependence between blocks, as the kernel's next block
  }
  const long long t1 = clock64();
  out[threadIdx.x] = c0.x + c0.y + c1.z + c1.w;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  float *in, *out;
  long long* cyc;
  (void)hipMalloc(&in, 8192 * sizeof(float));
  (void)hipMalloc(&out, 1024 * sizeof(float));
  (void)hipMalloc(&cyc, sizeof(long long));
  static float h[8192];
  for (int i = 0; i < 8192; ++i) h[i] = 0.01f * (float)((i * 37) % 101) - 0.5f;
  (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  const int blocks = 4096;
  long long c = 0;
  // threads 64: one wave (latency); 1024: 4 waves per SIMD as the kernel runs (the issue
  // rate: a SIMD's cycles per block = wave 0's cycles / 4)
  auto run = [&](auto kern, const char* name, int threads) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(threads), 0, 0, in, out, cyc, blocks);
    hipLaunchKernelGGL(kern, dim3(1), dim3(threads), 0, 0, in, out, cyc, blocks);
    (void)hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"simd_cycles_per_block\": %.1f}\n",
           name, threads / 256 ? threads / 256 : 1, (double)c / blocks / (threads >= 256 ? threads / 256 : 1));
  };
  for (int threads : {64, 1024}) {
    run(valu_kernel, "valu_shared_scores16", threads);
    run(mfma_kernel, "mfma_16x16x4f32_x32_lower_bound", threads);
  }
  return 0;
}
