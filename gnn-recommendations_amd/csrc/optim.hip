// Adam update for the embedding tables, gfx950 (the reference's optimizer is
// torch.optim.Adam with L2 weight decay, trainer.py:59-63). The tables are 128M parameters
// at G100M d=64: the update is a pure stream over param, grad and the two moments (16 B read
// + 12 B written per parameter), so it is HBM-bound — one pass, 16-B accesses, no launch per
// chunk (the multi-tensor loop issues 28-75 per step).
//
// Per element, in the order torch's single-tensor Adam applies them:
//   g  = grad * scale                      (scale: clip_grad_norm_'s coefficient, optional)
//   g  = g + wd * p                        (weight_decay != 0)
//   m  = m + (1 - b1) * (g - m)            (exp_avg.lerp_(g, 1 - b1), weight < 0.5 branch)
//   v  = v * b2 + (1 - b2) * g * g         (exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2))
//   p  = p - step_size * m / (sqrt(v) / bc2_sqrt + eps)
#include "common.h"

namespace gnnrec {

constexpr int kAdamBlock = 256;

struct AdamArgs {
  float step_size, b1, b2, omb1, omb2, bc2_sqrt, eps, wd;
};

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, float scale,
                                         const AdamArgs& a) {
  g = g * scale;
  if (a.wd != 0.f) g = g + a.wd * p;
  m = m + a.omb1 * (g - m);
  v = v * a.b2 + (a.omb2 * g) * g;
  const float denom = __builtin_sqrtf(v) / a.bc2_sqrt + a.eps;
  p = p + (-a.step_size) * (m / denom);
}

__global__ __launch_bounds__(kAdamBlock) void adam_kernel(float* __restrict__ p,
                                                          const float* __restrict__ g,
                                                          float* __restrict__ m,
                                                          float* __restrict__ v, int64_t n,
                                                          const float* __restrict__ scale_ptr,
                                                          AdamArgs a) {
  const float scale = scale_ptr ? *scale_ptr : 1.f;
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * kAdamBlock;
  for (int64_t i = (int64_t)blockIdx.x * kAdamBlock + threadIdx.x; i < n4; i += stride) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    const float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    adam_one(pp.x, gg.x, mm.x, vv.x, scale, a);
    adam_one(pp.y, gg.y, mm.y, vv.y, scale, a);
    adam_one(pp.z, gg.z, mm.z, vv.z, scale, a);
    adam_one(pp.w, gg.w, mm.w, vv.w, scale, a);
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * kAdamBlock + threadIdx.x; i < n; i += stride)
    adam_one(p[i], g[i], m[i], v[i], scale, a);
}

}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_adam_step_f32(float* param, const float* grad, float* exp_avg,
                                    float* exp_avg_sq, int64_t n, float step_size, double beta1,
                                    double beta2, float bias_correction2_sqrt, float eps,
                                    float weight_decay, const float* grad_scale,
                                    gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n >= 0, "adam: negative size");
  if (n == 0) return GNNREC_OK;
  GNNREC_REQUIRE(param && grad && exp_avg && exp_avg_sq, "adam: null pointer");
  GNNREC_REQUIRE(aligned16(param) && aligned16(grad) && aligned16(exp_avg) && aligned16(exp_avg_sq),
                 "adam: tensors must be 16-B aligned");
  GNNREC_REQUIRE(bias_correction2_sqrt > 0.f, "adam: bias_correction2_sqrt must be > 0");
  // 1 - beta in double, then rounded (as torch's Python-scalar arithmetic does: 1 - 0.999f
  // would be 1.3e-5 off)
  const AdamArgs a{step_size,         (float)beta1,          (float)beta2, (float)(1.0 - beta1),
                   (float)(1.0 - beta2), bias_correction2_sqrt, eps,          weight_decay};
  const int64_t want = ceil_div(ceil_div(n, 4), kAdamBlock);
  const unsigned grid = (unsigned)(want < 8192 ? want : 8192);
  hipLaunchKernelGGL(adam_kernel, dim3(grid), dim3(kAdamBlock), 0, as_hip(stream), param, grad,
                     exp_avg, exp_avg_sq, n, grad_scale, a);
  return check_launch("adam");
}
