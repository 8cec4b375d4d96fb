// Hop with a row-sparse input: y = A^T x where x is zero outside a short list of rows
// (gnnrec_spmm_sparse_src_f32). The training backward's first hop takes the BPR
// gradient, which touches the 3B rows of a batch (trainer.py:199-281 differentiating
// lightgcn.py:88's torch.sparse.mm): a few thousand of 2M rows. The row-parallel masked hop
// walks every neighbour of every output row a source reaches (G100M: ~60M neighbour tests for
// ~600K reached rows); here the sources' own rows of A are scattered instead — one
// (output row, source) pair per stored entry, ~0.6M pairs — sorted by (output row, source),
// and every reached output row runs ONE fmaf chain from +0 over its sources in ascending
// order. That is the dense hop's chain with its zero terms left out (fmaf(v, 0, acc) = acc
// for a finite acc), so the bits of y = A^T x through any other hop kernel. Rows no source
// reaches are left to the caller (it zeroes y first).
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace gnnrec {
namespace {

constexpr uint64_t kPadKey = ~0ull;

int bits_for(int64_t v) {
  int b = 1;
  while (b < 63 && (v >> b) != 0) ++b;
  return b;
}
size_t align_up(size_t v) { return (v + 255) & ~size_t(255); }

__device__ __forceinline__ int64_t src_degree(const int64_t* rp, const int64_t* src, int64_t i) {
  const int64_t c = src[i];
  return rp[c + 1] - rp[c];
}

__global__ __launch_bounds__(256) void src_degrees_kernel(const int64_t* __restrict__ rp,
                                                          const int64_t* __restrict__ src,
                                                          int64_t n_src, int64_t* __restrict__ deg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_src) deg[i] = src_degree(rp, src, i);
}

// one wave per source row: its entries become keys (output row << 32 | source index) with
// the value; pairs past the scan's total (the caller's bound) are padding keys
__global__ __launch_bounds__(256) void scatter_pairs_kernel(
    const int64_t* __restrict__ rp, const int32_t* __restrict__ col, const float* __restrict__ val,
    const int64_t* __restrict__ src, int64_t n_src, const int64_t* __restrict__ off,
    int64_t max_pairs, uint64_t* __restrict__ keys, float* __restrict__ vals,
    int* __restrict__ overflow) {
  const int lane = threadIdx.x & 63;
  for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n_src;
       i += (int64_t)gridDim.x * 4) {
    const int64_t c = src[i], k0 = rp[c], k1 = rp[c + 1], o = off[i];
    if (o + (k1 - k0) > max_pairs) {   // the caller's bound is short: reported, nothing written
      if (lane == 0) *overflow = 1;
      continue;
    }
    for (int64_t k = k0 + lane; k < k1; k += 64) {
      keys[o + (k - k0)] = ((uint64_t)(uint32_t)col[k] << 32) | (uint64_t)i;
      vals[o + (k - k0)] = val[k];
    }
  }
  // padding: the entries past the total
  const int64_t total = off[n_src];
  for (int64_t e = total + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < max_pairs;
       e += (int64_t)gridDim.x * blockDim.x) {
    keys[e] = kPadKey;
    vals[e] = 0.f;
  }
}

// a 16-lane group per sorted pair that starts an output row: the row's chain over its
// sources (ascending: the sort order), lane q owning features 4q .. 4q+3 (+64 per round)
__global__ __launch_bounds__(256) void source_chain_kernel(
    const uint64_t* __restrict__ keys, const float* __restrict__ vals, int64_t n_pairs,
    const int64_t* __restrict__ src, const float* __restrict__ x, int64_t ldx,
    float* __restrict__ y, int64_t ldy, int d, const int* __restrict__ overflow) {
  const int64_t e = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int q = threadIdx.x & 15;
  // a short bound left some key slots unwritten (scatter_pairs_kernel, same stream, already
  // finished): their garbage would index x and y, so nothing is computed and y stays as it was
  if (e >= n_pairs || *overflow) return;
  const uint64_t key = keys[e];
  if (key == kPadKey) return;
  const uint32_t r = (uint32_t)(key >> 32);
  if (e > 0 && (uint32_t)(keys[e - 1] >> 32) == r) return;   // not the row's first pair
  for (int f0 = 4 * q; f0 < d; f0 += 64) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t j = e; j < n_pairs; ++j) {
      const uint64_t kj = keys[j];
      if (kj == kPadKey || (uint32_t)(kj >> 32) != r) break;
      const float v = vals[j];
      const float4 xv =
          *reinterpret_cast<const float4*>(x + src[(uint32_t)kj] * ldx + f0);
      acc.x = __builtin_fmaf(v, xv.x, acc.x);
      acc.y = __builtin_fmaf(v, xv.y, acc.y);
      acc.z = __builtin_fmaf(v, xv.z, acc.z);
      acc.w = __builtin_fmaf(v, xv.w, acc.w);
    }
    *reinterpret_cast<float4*>(y + (int64_t)r * ldy + f0) = acc;
  }
}

struct Layout {
  size_t keys_in, keys_out, vals_in, vals_out, deg, off, flag, tmp, total;
};

Layout layout(int64_t n_src, int64_t max_pairs, size_t sort_tmp, size_t scan_tmp) {
  Layout l;
  const size_t P = (size_t)(max_pairs > 0 ? max_pairs : 1);
  const size_t S = (size_t)(n_src > 0 ? n_src : 1);
  l.keys_in = 0;
  l.keys_out = l.keys_in + align_up(P * 8);
  l.vals_in = l.keys_out + align_up(P * 8);
  l.vals_out = l.vals_in + align_up(P * 4);
  l.deg = l.vals_out + align_up(P * 4);
  l.off = l.deg + align_up((S + 1) * 8);
  l.flag = l.off + align_up((S + 1) * 8);
  l.tmp = l.flag + 256;
  l.total = l.tmp + align_up(sort_tmp > scan_tmp ? sort_tmp : scan_tmp);
  return l;
}

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_spmm_sparse_src_f32(const int64_t* row_ptr, const int32_t* col,
                                          const float* val, int64_t n_rows, int64_t n_cols,
                                          const int64_t* src_rows, int64_t n_src,
                                          int64_t max_pairs, const float* x, int64_t ldx,
                                          float* y, int64_t ldy, int32_t d, void* workspace,
                                          size_t* workspace_bytes, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(workspace_bytes, "sparse_src: null workspace_bytes");
  GNNREC_REQUIRE(n_rows >= 0 && n_cols >= 0 && n_src >= 0 && n_src <= n_rows && max_pairs >= 0,
                 "sparse_src: bad sizes");
  GNNREC_REQUIRE(n_cols < ((int64_t)1 << 32) - 1 && n_src < ((int64_t)1 << 32) &&
                     max_pairs < (int64_t)INT32_MAX,
                 "sparse_src: n_cols, n_src and max_pairs must fit the 32-bit key halves / "
                 "item counts");
  GNNREC_REQUIRE(d > 0 && d % 4 == 0 && ldx >= d && ldy >= d && ldx % 4 == 0 && ldy % 4 == 0,
                 "sparse_src: need d %% 4 == 0 and 16-B rows (ld %% 4 == 0, ld >= d)");
  hipStream_t s = as_hip(stream);
  const int end_bit = 32 + bits_for(n_cols > 0 ? n_cols - 1 : 0);
  size_t sort_tmp = 0, scan_tmp = 0;
  const int P = (int)(max_pairs > 0 ? max_pairs : 1);
  hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (const uint64_t*)nullptr,
                                     (uint64_t*)nullptr, (const float*)nullptr, (float*)nullptr, P,
                                     0, end_bit, s);
  hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, (const int64_t*)nullptr, (int64_t*)nullptr,
                                   (int)(n_src + 1), s);
  const Layout l = layout(n_src, max_pairs, sort_tmp, scan_tmp);
  if (workspace == nullptr) {
    *workspace_bytes = l.total;
    return GNNREC_OK;
  }
  GNNREC_REQUIRE(*workspace_bytes >= l.total, "sparse_src: workspace too small (%zu < %zu)",
                 *workspace_bytes, l.total);
  if (n_src == 0 || max_pairs == 0) return GNNREC_OK;
  GNNREC_REQUIRE(row_ptr && col && val && src_rows && x && y, "sparse_src: null pointer");
  GNNREC_REQUIRE(aligned16(x) && aligned16(y), "sparse_src: x / y must be 16-B aligned");
  char* w = static_cast<char*>(workspace);
  uint64_t* keys_in = reinterpret_cast<uint64_t*>(w + l.keys_in);
  uint64_t* keys_out = reinterpret_cast<uint64_t*>(w + l.keys_out);
  float* vals_in = reinterpret_cast<float*>(w + l.vals_in);
  float* vals_out = reinterpret_cast<float*>(w + l.vals_out);
  int64_t* deg = reinterpret_cast<int64_t*>(w + l.deg);
  int64_t* off = reinterpret_cast<int64_t*>(w + l.off);
  int* flag = reinterpret_cast<int*>(w + l.flag);
  void* tmp = w + l.tmp;
  // off[i] = the degrees before source i, off[n_src] = the total (a zero degree appended)
  if (hipMemsetAsync(flag, 0, sizeof(int), s) != hipSuccess ||
      hipMemsetAsync(deg + n_src, 0, sizeof(int64_t), s) != hipSuccess)
    return check_launch("sparse_src: memset");
  hipLaunchKernelGGL(src_degrees_kernel, dim3((unsigned)ceil_div(n_src, 256)), dim3(256), 0, s,
                     row_ptr, src_rows, n_src, deg);
  size_t t = scan_tmp;
  if (hipcub::DeviceScan::ExclusiveSum(tmp, t, deg, off, (int)(n_src + 1), s) != hipSuccess)
    return check_launch("sparse_src: scan");
  const int64_t blocks = std::max<int64_t>(ceil_div(n_src, 4), 1);
  hipLaunchKernelGGL(scatter_pairs_kernel, dim3((unsigned)std::min<int64_t>(blocks, 1 << 16)),
                     dim3(256), 0, s, row_ptr, col, val, src_rows, n_src, off, max_pairs, keys_in,
                     vals_in, flag);
  if (int rc = check_launch("sparse_src: scatter")) return rc;
  t = sort_tmp;
  if (hipcub::DeviceRadixSort::SortPairs(tmp, t, keys_in, keys_out, vals_in, vals_out, P, 0,
                                         end_bit, s) != hipSuccess)
    return check_launch("sparse_src: sort");
  hipLaunchKernelGGL(source_chain_kernel, dim3((unsigned)ceil_div(max_pairs, 16)), dim3(256), 0,
                     s, keys_out, vals_out, max_pairs, src_rows, x, ldx, y, ldy, (int)d, flag);
  if (int rc = check_launch("sparse_src: chain")) return rc;
  int h_flag = 0;
  hipMemcpyAsync(&h_flag, flag, sizeof(int), hipMemcpyDeviceToHost, s);
  if (hipStreamSynchronize(s) != hipSuccess) return check_launch("sparse_src: sync");
  if (h_flag) {
    set_error("sparse_src: the sources hold more than max_pairs = %lld entries",
              (long long)max_pairs);
    return GNNREC_EINVAL;
  }
  return GNNREC_OK;
}
