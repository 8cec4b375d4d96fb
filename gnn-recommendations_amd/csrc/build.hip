// On-device operand construction (reference data/graph_builder.py:16-144):
// bipartite interaction pairs -> CSR of the symmetric adjacency -> D^-1/2 A D^-1/2 values,
// without leaving HBM. Output identical to gnnrec_build_bipartite_csr (host.cpp) and hence
// to the reference's scipy operand.
//
//   1. expand: every pair (u, i) becomes two 64-bit keys row<<32 | col, (u, U+i) and (U+i, u),
//      plus (r, r) per node with self loops;
//   2. radix-sort the keys (rocPRIM via hipCUB, only the bits the node count needs);
//   3. run-length encode: unique keys = the nonzeros in CSR order (columns ascending inside
//      each row, exactly the host builder's order); run lengths = multiplicities;
//   4. row_ptr by a boundary scan of the unique keys; degrees = fp32 row sums of the weights,
//      which are small integers, so they are the row lengths of the sorted (weighted) or the
//      unique (binary) key array — exact below 2^24;
//   5. values: val = fl32(fl32(dis[r] * a) * dis[c]) (gnnrec_normalize_values_device), with
//      dis = deg^-1/2 computed by the caller exactly as graph_builder.py:119 (numpy float32
//      power on the host: N floats each way).
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace gnnrec {

__global__ void expand_pairs_kernel(const int64_t* __restrict__ users,
                                    const int64_t* __restrict__ items, int64_t n_pairs,
                                    int64_t n_users, int64_t n_items, int self_loop,
                                    uint64_t* __restrict__ keys, int* __restrict__ bad) {
  const int64_t N = n_users + n_items;
  const int64_t total = 2 * n_pairs + (self_loop ? N : 0);
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    if (t < 2 * n_pairs) {
      const int64_t e = t >> 1;
      const int64_t u = users[e], i = items[e];
      if (u < 0 || u >= n_users || i < 0 || i >= n_items) {
        atomicMin(bad, (int)min<int64_t>(e, INT32_MAX - 1));
        keys[t] = 0;
        continue;
      }
      const uint64_t ri = (uint64_t)(n_users + i);
      keys[t] = (t & 1) ? (ri << 32 | (uint64_t)u) : ((uint64_t)u << 32 | ri);
    } else {
      const uint64_t r = (uint64_t)(t - 2 * n_pairs);
      keys[t] = r << 32 | r;
    }
  }
}

// row_ptr[r] = first position in `keys` (sorted, length n) whose row is >= r; rows 0..N.
__global__ void row_bounds_kernel(const uint64_t* __restrict__ keys, int64_t n, int64_t N,
                                  int64_t* __restrict__ row_ptr) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k <= n;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = k < n ? (int64_t)(keys[k] >> 32) : N;
    const int64_t prev = k > 0 ? (int64_t)(keys[k - 1] >> 32) : -1;
    for (int64_t rr = prev + 1; rr <= r; ++rr) row_ptr[rr] = k;
  }
}

__global__ void split_keys_kernel(const uint64_t* __restrict__ uniq, const int* __restrict__ runs,
                                  int64_t nnz, int binary, int32_t* __restrict__ col,
                                  float* __restrict__ cnt) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nnz;
       k += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = uniq[k];
    col[k] = (int32_t)(key & 0xffffffffu);
    const bool self = (key >> 32) == (key & 0xffffffffu);
    cnt[k] = (binary || self) ? 1.f : (float)runs[k];
  }
}

__global__ void degrees_kernel(const int64_t* __restrict__ bounds, int64_t N,
                               float* __restrict__ deg) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < N;
       r += (int64_t)gridDim.x * blockDim.x)
    deg[r] = (float)(bounds[r + 1] - bounds[r]);
}

__global__ void normalize_kernel(const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
                                 const float* __restrict__ cnt, int64_t n_rows,
                                 const float* __restrict__ dis, int mode, float* __restrict__ val) {
  // one wave per row, lanes stride the row (rows of any length, coalesced)
  const int lane = threadIdx.x & 63;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n_rows;
       r += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const float dr = dis[r];
    for (int64_t k = row_ptr[r] + lane; k < row_ptr[r + 1]; k += 64) {
      const float t = dr * cnt[k];                 // fp-contract off: two roundings
      val[k] = mode == 0 ? t * dis[col[k]] : t;
    }
  }
}

static unsigned grid_for(int64_t n, int per_block = 256) {
  const int64_t g = ceil_div(n > 0 ? n : 1, per_block);
  return (unsigned)(g < 65536 ? g : 65536);
}

static int bits_for(int64_t v) {
  int b = 1;
  while ((int64_t(1) << b) <= v) ++b;
  return b;
}

static size_t align_up(size_t v) { return (v + 255) & ~size_t(255); }

}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_build_bipartite_csr_device(const int64_t* users, const int64_t* items,
                                                 int64_t n_pairs, int64_t n_users, int64_t n_items,
                                                 int32_t flags, int64_t* row_ptr, int32_t* col,
                                                 float* cnt, float* deg, int64_t* nnz_out,
                                                 void* workspace, size_t* workspace_bytes,
                                                 gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_pairs >= 0 && n_users >= 0 && n_items >= 0, "build_device: negative sizes");
  GNNREC_REQUIRE(n_users + n_items < (int64_t)INT32_MAX, "build_device: N must fit int32 columns");
  GNNREC_REQUIRE(workspace_bytes, "build_device: null workspace_bytes");
  GNNREC_REQUIRE((flags & ~(GNNREC_BUILD_SELF_LOOP | GNNREC_BUILD_BINARY)) == 0,
                 "build_device: bad flags");
  const bool self_loop = flags & GNNREC_BUILD_SELF_LOOP, binary = flags & GNNREC_BUILD_BINARY;
  const int64_t N = n_users + n_items;
  const int64_t M = 2 * n_pairs + (self_loop ? N : 0);
  GNNREC_REQUIRE(M < (int64_t)INT32_MAX, "build_device: 2*pairs (+N) must fit int32 (hipCUB item counts)");
  const int end_bit = 32 + bits_for(N > 0 ? N - 1 : 0);
  hipStream_t s = as_hip(stream);

  // workspace: keys_in (reused for the unique keys) | keys_out | runs | bounds | num_runs |
  // bad | cub temp
  size_t sort_tmp = 0, rle_tmp = 0;
  hipcub::DeviceRadixSort::SortKeys(nullptr, sort_tmp, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                    (int)M, 0, end_bit, s);
  hipcub::DeviceRunLengthEncode::Encode(nullptr, rle_tmp, (const uint64_t*)nullptr,
                                        (uint64_t*)nullptr, (int*)nullptr, (int*)nullptr, (int)M, s);
  const size_t Mk = (size_t)(M > 0 ? M : 1);
  const size_t off_keys_out = align_up(Mk * 8), off_runs = off_keys_out + align_up(Mk * 8),
               off_bounds = off_runs + align_up(Mk * 4),
               off_num = off_bounds + align_up((size_t)(N + 1) * 8), off_bad = off_num + 256,
               off_tmp = off_bad + 256;
  const size_t tmp = sort_tmp > rle_tmp ? sort_tmp : rle_tmp;
  const size_t need = off_tmp + align_up(tmp);
  if (workspace == nullptr) {
    *workspace_bytes = need;
    return GNNREC_OK;
  }
  GNNREC_REQUIRE(*workspace_bytes >= need, "build_device: workspace too small (%zu < %zu)",
                 *workspace_bytes, need);
  GNNREC_REQUIRE(row_ptr && nnz_out && deg && (M == 0 || (col && cnt)), "build_device: null output");
  GNNREC_REQUIRE(n_pairs == 0 || (users && items), "build_device: null input");
  char* w = static_cast<char*>(workspace);
  uint64_t* keys_in = reinterpret_cast<uint64_t*>(w);
  uint64_t* keys_out = reinterpret_cast<uint64_t*>(w + off_keys_out);
  uint64_t* uniq = keys_in;  // free once sorted
  int* runs = reinterpret_cast<int*>(w + off_runs);
  int64_t* bounds = reinterpret_cast<int64_t*>(w + off_bounds);
  int* num_runs = reinterpret_cast<int*>(w + off_num);
  int* bad = reinterpret_cast<int*>(w + off_bad);
  void* cub_tmp = w + off_tmp;

  const int init_bad = INT32_MAX;
  if (hipMemcpyAsync(bad, &init_bad, sizeof(int), hipMemcpyHostToDevice, s) != hipSuccess)
    return check_launch("build_device: memcpy");
  if (M > 0)
    hipLaunchKernelGGL(expand_pairs_kernel, dim3(grid_for(M)), dim3(256), 0, s, users, items,
                       n_pairs, n_users, n_items, (int)self_loop, keys_in, bad);
  if (int rc = check_launch("expand_pairs_kernel")) return rc;
  int h_bad = INT32_MAX;
  hipMemcpyAsync(&h_bad, bad, sizeof(int), hipMemcpyDeviceToHost, s);
  if (hipStreamSynchronize(s) != hipSuccess) return check_launch("build_device: sync");
  if (h_bad != INT32_MAX) {
    set_error("build_device: pair %d out of range", h_bad);
    return GNNREC_EINVAL;
  }
  size_t t1 = sort_tmp, t2 = rle_tmp;
  int nnz = 0;
  if (M > 0) {
    if (hipcub::DeviceRadixSort::SortKeys(cub_tmp, t1, keys_in, keys_out, (int)M, 0, end_bit, s) !=
        hipSuccess)
      return check_launch("build_device: radix sort");
    if (hipcub::DeviceRunLengthEncode::Encode(cub_tmp, t2, keys_out, uniq, runs, num_runs, (int)M, s) !=
        hipSuccess)
      return check_launch("build_device: run-length encode");
    hipMemcpyAsync(&nnz, num_runs, sizeof(int), hipMemcpyDeviceToHost, s);
    if (hipStreamSynchronize(s) != hipSuccess) return check_launch("build_device: sync");
  }
  // CSR structure from the unique keys; degrees from the weighted (sorted) or unique keys.
  hipLaunchKernelGGL(row_bounds_kernel, dim3(grid_for(nnz + 1)), dim3(256), 0, s, uniq,
                     (int64_t)nnz, N, row_ptr);
  if (!binary)
    hipLaunchKernelGGL(row_bounds_kernel, dim3(grid_for(M + 1)), dim3(256), 0, s, keys_out, M, N,
                       bounds);
  hipLaunchKernelGGL(degrees_kernel, dim3(grid_for(N)), dim3(256), 0, s,
                     binary ? (const int64_t*)row_ptr : (const int64_t*)bounds, N, deg);
  if (nnz > 0)
    hipLaunchKernelGGL(split_keys_kernel, dim3(grid_for(nnz)), dim3(256), 0, s, uniq, runs,
                       (int64_t)nnz, (int)binary, col, cnt);
  if (int rc = check_launch("build_device: csr kernels")) return rc;
  if (hipStreamSynchronize(s) != hipSuccess) return check_launch("build_device: sync");
  *nnz_out = nnz;
  return GNNREC_OK;
}

extern "C" int gnnrec_normalize_values_device(const int64_t* row_ptr, const int32_t* col,
                                              const float* cnt, int64_t n_rows, const float* dis,
                                              int32_t mode, float* val, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(row_ptr && col && cnt && dis && val && n_rows >= 0, "normalize_device: bad args");
  GNNREC_REQUIRE(mode == 0 || mode == 1, "normalize_device: mode must be 0 or 1");
  if (n_rows == 0) return GNNREC_OK;
  hipLaunchKernelGGL(normalize_kernel, dim3(grid_for(n_rows * 64)), dim3(256), 0, as_hip(stream),
                     row_ptr, col, cnt, n_rows, dis, (int)mode, val);
  return check_launch("normalize_kernel");
}
