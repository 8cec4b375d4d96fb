// Host-side part of libgnnrec: ABI identity/error plumbing and the native operand builder
// (data/graph_builder.py:16-144 of the reference: bipartite COO -> CSR -> D^-1/2 A D^-1/2).
//
// The reference builds the operand with scipy (coo_matrix, tocsr, sparse products: 28 s at
// 2e8 nnz). Here it is a counting sort by user (O(pairs)), an in-row sort + duplicate merge,
// and a transpose for the item rows that emits users already ascending; values are one fp32
// product chain per nonzero, identical to scipy's (see gnnrec_normalize_values).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "common.h"

namespace gnnrec {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: HIP error %d (%s)", what, (int)e, hipGetErrorString(e));
    return GNNREC_EHIP;
  }
  return GNNREC_OK;
}

// Static partition of [0, n) over worker threads.
template <class F>
static void parallel_for(int64_t n, int n_threads, F&& f) {
  int t = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
  if (t < 1) t = 1;
  if (n < 1 << 14) t = 1;
  if (t == 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> pool;
  const int64_t step = (n + t - 1) / t;
  for (int i = 0; i < t; ++i) {
    const int64_t lo = i * step, hi = std::min<int64_t>(n, lo + step);
    if (lo >= hi) break;
    pool.emplace_back([&f, lo, hi] { f(lo, hi); });
  }
  for (auto& th : pool) th.join();
}

}  // namespace gnnrec

using namespace gnnrec;

extern "C" const char* gnnrec_version(void) { return "gnnrec-mi355x 0.1.0 (gfx950)"; }
extern "C" int gnnrec_abi_version(void) { return GNNREC_ABI_VERSION; }
extern "C" const char* gnnrec_last_error(void) { return g_last_error.c_str(); }

extern "C" int gnnrec_build_bipartite_csr(const int64_t* users, const int64_t* items,
                                          int64_t n_pairs, int64_t n_users, int64_t n_items,
                                          int32_t flags, int64_t* row_ptr, int32_t* col,
                                          float* cnt, float* deg, int64_t* nnz_out,
                                          int32_t n_threads) {
  GNNREC_REQUIRE(n_pairs >= 0 && n_users >= 0 && n_items >= 0, "build: negative sizes");
  GNNREC_REQUIRE(n_users + n_items < (int64_t)INT32_MAX, "build: N must fit int32 columns");
  GNNREC_REQUIRE(row_ptr && col && cnt && deg && nnz_out, "build: null output");
  GNNREC_REQUIRE(n_pairs == 0 || (users && items), "build: null input");
  GNNREC_REQUIRE((flags & ~(GNNREC_BUILD_SELF_LOOP | GNNREC_BUILD_BINARY)) == 0, "build: bad flags");
  const bool self_loop = flags & GNNREC_BUILD_SELF_LOOP;
  const float dup_w = (flags & GNNREC_BUILD_BINARY) ? 0.f : 1.f;
  const int64_t N = n_users + n_items;
  // Range check + counting sort of the pairs by user.
  std::vector<int64_t> ustart(n_users + 1, 0);
  for (int64_t e = 0; e < n_pairs; ++e) {
    const int64_t u = users[e], i = items[e];
    if (u < 0 || u >= n_users || i < 0 || i >= n_items) {
      set_error("build: pair %lld = (%lld, %lld) out of range", (long long)e, (long long)u,
                (long long)i);
      return GNNREC_EINVAL;
    }
    ustart[u + 1]++;
  }
  for (int64_t u = 0; u < n_users; ++u) ustart[u + 1] += ustart[u];
  std::vector<int32_t> bucket(n_pairs > 0 ? n_pairs : 1);
  {
    std::vector<int64_t> fill(ustart.begin(), ustart.end() - 1);
    for (int64_t e = 0; e < n_pairs; ++e) bucket[fill[users[e]]++] = (int32_t)items[e];
  }
  // Sort each user's items, merge duplicates (multiplicity), count unique per user.
  std::vector<int32_t> ucnt_unique(n_users, 0);
  std::vector<float> mult(n_pairs > 0 ? n_pairs : 1, 0.f);
  parallel_for(n_users, n_threads, [&](int64_t lo, int64_t hi) {
    for (int64_t u = lo; u < hi; ++u) {
      int32_t* b = bucket.data() + ustart[u];
      const int64_t m = ustart[u + 1] - ustart[u];
      std::sort(b, b + m);
      int64_t w = 0;
      for (int64_t k = 0; k < m; ++k) {
        if (w > 0 && b[w - 1] == b[k]) {
          mult[ustart[u] + w - 1] += dup_w;
        } else {
          b[w] = b[k];
          mult[ustart[u] + w] = 1.f;
          ++w;
        }
      }
      ucnt_unique[u] = (int32_t)w;
    }
  });
  // Row sizes: user rows = unique items (+1 self); item rows = unique users (+1 self).
  const int sl = self_loop ? 1 : 0;
  std::vector<int64_t> icount(n_items, 0);
  for (int64_t u = 0; u < n_users; ++u)
    for (int64_t k = 0; k < ucnt_unique[u]; ++k) icount[bucket[ustart[u] + k]]++;
  row_ptr[0] = 0;
  for (int64_t u = 0; u < n_users; ++u) row_ptr[u + 1] = row_ptr[u] + ucnt_unique[u] + sl;
  for (int64_t i = 0; i < n_items; ++i) row_ptr[n_users + i + 1] = row_ptr[n_users + i] + icount[i] + sl;
  const int64_t nnz = row_ptr[N];
  // User rows: [self] then items (global col = n_users + item), ascending.
  parallel_for(n_users, n_threads, [&](int64_t lo, int64_t hi) {
    for (int64_t u = lo; u < hi; ++u) {
      int64_t o = row_ptr[u];
      if (sl) { col[o] = (int32_t)u; cnt[o] = 1.f; ++o; }
      for (int64_t k = 0; k < ucnt_unique[u]; ++k, ++o) {
        col[o] = (int32_t)(n_users + bucket[ustart[u] + k]);
        cnt[o] = mult[ustart[u] + k];
      }
    }
  });
  // Item rows: users in ascending order (users visited ascending), then [self].
  {
    std::vector<int64_t> fill(n_items);
    for (int64_t i = 0; i < n_items; ++i) fill[i] = row_ptr[n_users + i];
    for (int64_t u = 0; u < n_users; ++u) {
      for (int64_t k = 0; k < ucnt_unique[u]; ++k) {
        const int32_t i = bucket[ustart[u] + k];
        const int64_t o = fill[i]++;
        col[o] = (int32_t)u;
        cnt[o] = mult[ustart[u] + k];
      }
    }
    if (sl)
      for (int64_t i = 0; i < n_items; ++i) {
        col[fill[i]] = (int32_t)(n_users + i);
        cnt[fill[i]] = 1.f;
      }
  }
  // Degrees = fp32 row sums of A (graph_builder.py:111); counts are small integers, exact.
  parallel_for(N, n_threads, [&](int64_t lo, int64_t hi) {
    for (int64_t r = lo; r < hi; ++r) {
      float s = 0.f;
      for (int64_t k = row_ptr[r]; k < row_ptr[r + 1]; ++k) s += cnt[k];
      deg[r] = s;
    }
  });
  *nnz_out = nnz;
  return GNNREC_OK;
}

extern "C" int gnnrec_normalize_values(const int64_t* row_ptr, const int32_t* col, const float* cnt,
                                       int64_t n_rows, const float* dis, int32_t mode, float* val,
                                       int32_t n_threads) {
  GNNREC_REQUIRE(row_ptr && col && cnt && dis && val && n_rows >= 0, "normalize: bad args");
  GNNREC_REQUIRE(mode == 0 || mode == 1, "normalize: mode must be 0 (symmetric) or 1 (row)");
  parallel_for(n_rows, n_threads, [&](int64_t lo, int64_t hi) {
    for (int64_t r = lo; r < hi; ++r) {
      const float dr = dis[r];
      for (int64_t k = row_ptr[r]; k < row_ptr[r + 1]; ++k) {
        // scipy: (D @ A) first -> fl(dis[r] * a), then (DA) @ D -> fl(. * dis[c]).
        volatile float t = dr * cnt[k];
        val[k] = mode == 0 ? t * dis[col[k]] : t;
      }
    }
  });
  return GNNREC_OK;
}
