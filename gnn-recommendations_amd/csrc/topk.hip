// Scoring GEMM + seen-item mask + per-user top-K (evaluator.py:96-105, trainer.py:327-336).
//
// The reference computes scores = U[b] @ I^T with MKL sgemm, sets the train/valid items of
// each user to -inf in a Python loop, calls torch.topk (tie order unspecified) and copies
// the indices to the host. Here one kernel does all of it on the device:
//   * scores on the matrix cores: v_mfma_f32_16x16x4_f32 is an exact k-ordered fmaf chain,
//     and the k-steps are issued in ascending k, so score[b,i] is bit-identical to
//     `acc = 0; for f in 0..d-1: acc = fmaf(u[b,f], v[i,f], acc)` (the oracle's definition);
//   * a per-user top-K list lives in LDS as a heap rooted at its worst entry under the fixed
//     order (score desc, item index asc); a candidate enters only if it beats the root, so
//     after the first tiles a tile costs one register compare per score and one ballot;
//   * seen items are masked lazily: only a candidate that would enter the list is looked up,
//     through a per-user cursor into its sorted seen list that only moves forward (the
//     candidates of a user arrive in ascending item order), and, if seen, re-scored as -inf.
// Workgroup = 4 waves = 64 * UF users (16 * UF per wave: UF user fragments share every B
// fragment a wave reads, UF MFMA chains per item block); item tiles of 64 rows are staged in
// LDS ([64][d+2]: d+2 == 2 mod 32 makes the B-fragment reads conflict-free) and reused by the
// four waves.
#include <math.h>

#include "gather.h"

namespace gnnrec {

typedef float floatx4_t __attribute__((ext_vector_type(4)));

struct TopkParams {
  const float* u;
  int64_t ldu;
  int64_t nb;
  const float* v;
  int64_t ldv;
  int64_t n_items;
  const int64_t* seen_ptr;
  const int32_t* seen_col;
  int k;
  int64_t* out_idx;
  float* out_score;
  int n_split;           // item ranges (blockIdx.y); > 1: partial lists go to out_* with
                         // row stride n_split*k at offset split*k, merged by topk_merge_kernel
};

// a strictly precedes b in the output order
__device__ __forceinline__ bool better(float sa, int ia, float sb, int ib) {
  return sa > sb || (sa == sb && ia < ib);
}


// One user's list is a binary heap over KM slots whose root is the list's WORST entry under
// the output order (score desc, item asc). Replacing the root by a better candidate and
// sifting it down keeps that invariant in log2(KM) steps of one lane (the previous design
// re-scanned the whole list with wave shuffles after every insertion).
template <int KM>
__device__ __forceinline__ void heap_replace_root(float* hs, int* hi, float cs, int ci) {
  int pos = 0;
  while (true) {
    const int l = 2 * pos + 1, r = l + 1;
    if (l >= KM) break;
    int w = l;                        // the worse child
    float wsc = hs[l];
    int wit = hi[l];
    if (r < KM) {
      const float rs = hs[r];
      const int ri = hi[r];
      if (better(wsc, wit, rs, ri)) { w = r; wsc = rs; wit = ri; }
    }
    if (!better(cs, ci, wsc, wit)) break;  // the worse child is not worse than the candidate
    hs[pos] = wsc;
    hi[pos] = wit;
    pos = w;
  }
  hs[pos] = cs;
  hi[pos] = ci;
}

template <int D, int KM, int UF>
__global__ __launch_bounds__(kBlock) void score_topk_kernel(TopkParams p) {
  constexpr int STEPS = D / 4;
  constexpr int TI = D <= 128 ? 64 : 32;  // items per LDS tile
  constexpr int LDV = D + 2;
  constexpr int UPW = 16 * UF;  // users per wave
  constexpr int UPB = 4 * UPW;  // users per workgroup
  static_assert(UF * 4 * (TI / 16) <= 32, "candidate mask bits");
  constexpr int PIECES = TI * (D / 4) / kBlock;  // float4 per thread per tile
  __shared__ __attribute__((aligned(16))) float v_lds[2][TI * LDV];
  __shared__ float l_score[UPB][KM];
  __shared__ int l_item[UPB][KM];
  __shared__ int64_t s_cur[UPB];   // per user: cursor into its sorted seen list ...
  __shared__ int s_val[UPB];       // ... and the item there (INT_MAX when exhausted)

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i16 = lane & 15, k4 = lane >> 4;
  const int64_t ub = (int64_t)blockIdx.x * UPB;
  const int wu = UPW * wave;   // this wave's first user in the workgroup
  // this workgroup's item range (a multiple of TI, so tiles never straddle two ranges)
  const int64_t per = ((p.n_items + p.n_split - 1) / p.n_split + TI - 1) / TI * TI;
  const int64_t i_beg = (int64_t)blockIdx.y * per;
  const int64_t i_end = min<int64_t>(p.n_items, i_beg + per);
  // A fragments: this wave's 16 * UF users, k = 4s + k4 (ascending k per MFMA chain)
  float af[UF][STEPS];
#pragma unroll
  for (int f = 0; f < UF; ++f) {
    const int64_t user = ub + wu + 16 * f + i16;
#pragma unroll
    for (int s = 0; s < STEPS; ++s)
      af[f][s] = user < p.nb ? p.u[user * p.ldu + 4 * s + k4] : 0.f;
  }
  for (int e = threadIdx.x; e < UPB * KM; e += kBlock) {
    l_score[e / KM][e % KM] = -INFINITY;
    l_item[e / KM][e % KM] = INT_MAX;  // sentinel: loses to every real item
  }
  // A user's candidates reach its list in ascending item order (tiles ascend, and inside a
  // tile nt then i16 ascend), so the seen test is a cursor that only moves forward: set it
  // to the first seen item >= this workgroup's range start.
  for (int e = threadIdx.x; e < UPB; e += kBlock) {
    int64_t lo = 0, hi = 0;
    if (p.seen_ptr && ub + e < p.nb) {
      lo = p.seen_ptr[ub + e];
      hi = p.seen_ptr[ub + e + 1];
      const int64_t last = hi;
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (p.seen_col[mid] < i_beg) lo = mid + 1; else hi = mid;
      }
      hi = last;
    }
    s_cur[e] = lo;
    s_val[e] = lo < hi ? p.seen_col[lo] : INT_MAX;
  }

  // item tiles are double-buffered: the global loads of tile t+1 are in flight while the
  // MFMAs and the list updates of tile t run
  float4 stage[PIECES];
  auto load_tile = [&](int64_t t0) {
#pragma unroll
    for (int q = 0; q < PIECES; ++q) {
      const int e = threadIdx.x + q * kBlock, r = e / (D / 4), c4 = e % (D / 4);
      const int64_t item = t0 + r;
      stage[q] = item < i_end ? ld4(p.v + item * p.ldv + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto park_tile = [&](int b) {
#pragma unroll
    for (int q = 0; q < PIECES; ++q) {
      const int e = threadIdx.x + q * kBlock, r = e / (D / 4), c4 = e % (D / 4);
      float* dst = &v_lds[b][r * LDV + 4 * c4];
      dst[0] = stage[q].x; dst[1] = stage[q].y; dst[2] = stage[q].z; dst[3] = stage[q].w;
    }
  };
  if (i_beg < i_end) load_tile(i_beg);
  int buf = 0;
  for (int64_t t0 = i_beg; t0 < i_end; t0 += TI, buf ^= 1) {
    park_tile(buf);
    __syncthreads();
    if (t0 + TI < i_end) load_tile(t0 + TI);
    // all B fragments of the tile first (LDS latency paid once), then the MFMAs with the
    // TI/16 independent accumulator chains interleaved; each chain still runs k ascending
    floatx4_t acc[UF][TI / 16];
    float bf[TI / 16][STEPS];
#pragma unroll
    for (int nt = 0; nt < TI / 16; ++nt) {
      const float* brow = &v_lds[buf][(16 * nt + i16) * LDV + k4];
#pragma unroll
      for (int s = 0; s < STEPS; ++s) bf[nt][s] = brow[4 * s];
#pragma unroll
      for (int f = 0; f < UF; ++f) acc[f][nt] = floatx4_t{0.f, 0.f, 0.f, 0.f};
    }
    __builtin_amdgcn_sched_barrier(0);  // keep every LDS read ahead of the MFMA stream
#pragma unroll
    for (int s = 0; s < STEPS; ++s)
#pragma unroll
      for (int nt = 0; nt < TI / 16; ++nt)
#pragma unroll
        for (int f = 0; f < UF; ++f)
          acc[f][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[f][s], bf[nt][s], acc[f][nt], 0,
                                                            0, 0);
    // candidates: lane holds users wu + 16*f + 4*k4 + q (q = reg) x items t0 + 16*nt + i16.
    // Fast filter against register copies of the users' current worst entries (a list's
    // worst only rises, so a score that fails the copy fails the list); the wave leaves the
    // tile after one ballot unless some lane has a candidate.
    float ws[UF][4];
    int wi[UF][4];
    unsigned cmask = 0;   // bit (f * TI/16 + nt) * 4 + q: (item, user) passes the filter
#pragma unroll
    for (int f = 0; f < UF; ++f)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        ws[f][q] = l_score[wu + 16 * f + 4 * k4 + q][0];   // heap roots = current worst
        wi[f][q] = l_item[wu + 16 * f + 4 * k4 + q][0];
      }
#pragma unroll
    for (int f = 0; f < UF; ++f)
#pragma unroll
      for (int nt = 0; nt < TI / 16; ++nt)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float sc = acc[f][nt][q];
          if (sc != sc) sc = -INFINITY;  // NaN scores rank last
          acc[f][nt][q] = sc;
          const int64_t item64 = t0 + 16 * nt + i16;
          // >= : a superset of better() (ties are settled by the leader's exact check)
          if (sc >= ws[f][q] && item64 < i_end && ub + wu + 16 * f + 4 * k4 + q < p.nb &&
              (sc > ws[f][q] || (int)item64 < wi[f][q]))
            cmask |= 1u << ((f * (TI / 16) + nt) * 4 + q);
        }
    if (__ballot(cmask != 0) == 0) continue;
#pragma unroll
    for (int f = 0; f < UF; ++f)
#pragma unroll
    for (int nt = 0; nt < TI / 16; ++nt) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ul = wu + 16 * f + 4 * k4 + q;
        const int64_t user = ub + ul;
        const int64_t item64 = t0 + 16 * nt + i16;
        const float s = acc[f][nt][q];
        const int item = (int)item64;
        // (the leader re-checks each candidate against the heap root, which only rises)
        const unsigned long long m = __ballot((cmask >> ((f * (TI / 16) + nt) * 4 + q)) & 1u);
        if (m == 0) continue;
        // the 16 lanes of group k4 share user ul; group leader (i16 == 0) inserts the group's
        // candidates into that user's heap one by one — the four groups work in parallel
        unsigned grp = (unsigned)(m >> (16 * k4)) & 0xffffu;
        while (__ballot(grp != 0)) {
          const bool has = grp != 0;
          const int src = has ? __ffs(grp) - 1 : 0;
          grp &= grp - 1;
          const int src_lane = 16 * k4 + src;
          float cs = __shfl(s, src_lane, 64);
          const int ci = __shfl(item, src_lane, 64);
          if (i16 == 0 && has && better(cs, ci, l_score[ul][0], l_item[ul][0])) {
            // the seen lookup (a binary search in HBM) only for a candidate that would enter;
            // a masked item scores -inf and still enters if the root is an empty slot
            int64_t cur = s_cur[ul];
            int sv = s_val[ul];
            if (sv < ci) {
              const int64_t end = p.seen_ptr[user + 1];
              do {
                ++cur;
                sv = cur < end ? p.seen_col[cur] : INT_MAX;
              } while (sv < ci);
              s_cur[ul] = cur;
              s_val[ul] = sv;
            }
            if (sv == ci) cs = -INFINITY;
            if (better(cs, ci, l_score[ul][0], l_item[ul][0]))
              heap_replace_root<KM>(&l_score[ul][0], &l_item[ul][0], cs, ci);
          }
          __builtin_amdgcn_s_waitcnt(0xc07f);
          __builtin_amdgcn_wave_barrier();
        }
      }
    }
  }
  __syncthreads();
  // emit each user's list sorted by (score desc, item asc): rank by counting
  for (int ul = wu; ul < wu + UPW; ++ul) {
    const int64_t user = ub + ul;
    if (user >= p.nb) break;
    for (int e = lane; e < KM; e += 64) {
      const float s = l_score[ul][e];
      const int i = l_item[ul][e];
      int rank = 0;
      for (int f = 0; f < KM; ++f) {  // identical sentinels are ordered by slot
        const float sf = l_score[ul][f];
        const int jf = l_item[ul][f];
        rank += (better(sf, jf, s, i) || (sf == s && jf == i && f < e)) ? 1 : 0;
      }
      if (rank < p.k) {
        const int64_t o = user * ((int64_t)p.n_split * p.k) + (int64_t)blockIdx.y * p.k + rank;
        p.out_idx[o] = i == INT_MAX ? -1 : (int64_t)i;
        p.out_score[o] = s;
      }
    }
  }
}


// Merge the n_split partial lists of each user (one wave per user): rank every candidate
// by counting the candidates that precede it under (score desc, item asc; -1 = empty slot
// last, empty slots ordered by position) and keep ranks < k. Exact: each partial list is the
// exact top-k of its item range.
__global__ __launch_bounds__(kBlock) void topk_merge_kernel(const int64_t* __restrict__ pidx,
                                                            const float* __restrict__ pscore,
                                                            int64_t nb, int n_split, int k,
                                                            int64_t* __restrict__ out_idx,
                                                            float* __restrict__ out_score) {
  const int lane = threadIdx.x & 63;
  const int64_t user = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (user >= nb) return;
  const int C = n_split * k;
  const int64_t* ci = pidx + user * C;
  const float* cs = pscore + user * C;
  for (int e = lane; e < C; e += 64) {
    const float s = cs[e];
    const int64_t i = ci[e];
    const int64_t ie = i < 0 ? INT64_MAX : i;
    int rank = 0;
    for (int f = 0; f < C; ++f) {
      const float sf = cs[f];
      const int64_t jf = ci[f] < 0 ? INT64_MAX : ci[f];
      rank += (sf > s || (sf == s && (jf < ie || (jf == ie && f < e)))) ? 1 : 0;
    }
    if (rank < k) {
      out_idx[user * k + rank] = i;
      out_score[user * k + rank] = s;
    }
  }
}

}  // namespace gnnrec

using namespace gnnrec;

namespace {
// Two user fragments per wave where the A fragments and the lists fit (d <= 64, k <= 64).
template <int D, int KM>
void launch_topk(const TopkParams& p, hipStream_t s) {
  constexpr int UF = (D <= 64 && KM <= 64) ? 2 : 1;
  hipLaunchKernelGGL((score_topk_kernel<D, KM, UF>),
                     dim3((unsigned)ceil_div(p.nb, 64 * UF), (unsigned)p.n_split), dim3(kBlock), 0,
                     s, p);
}
template <int D>
int dispatch_k(const TopkParams& p, hipStream_t s) {
  if (p.k <= 32) launch_topk<D, 32>(p, s);
  else if (p.k <= 64) launch_topk<D, 64>(p, s);
  else launch_topk<D, 128>(p, s);
  return check_launch("score_topk");
}
}  // namespace

extern "C" int gnnrec_score_topk_split_f32(const float* u, int64_t ldu, int64_t n_users_batch,
                                           const float* v, int64_t ldv, int64_t n_items, int32_t d,
                                           const int64_t* seen_ptr, const int32_t* seen_col,
                                           int32_t k, int32_t n_split, int64_t* work_idx,
                                           float* work_score, int64_t* out_idx, float* out_score,
                                           gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_users_batch >= 0 && n_items >= 0 && k >= 1 && k <= 128, "score_topk: need 1 <= k <= 128");
  GNNREC_REQUIRE(n_split >= 1 && n_split <= 65535, "score_topk: n_split must be in [1, 65535]");
  if (n_users_batch == 0) return GNNREC_OK;
  GNNREC_REQUIRE(n_items < (int64_t)INT32_MAX, "score_topk: n_items must fit int32");
  GNNREC_REQUIRE(u && v && out_idx && out_score, "score_topk: null operand");
  GNNREC_REQUIRE(n_split == 1 || (work_idx && work_score), "score_topk: n_split > 1 needs work buffers");
  GNNREC_REQUIRE(ldu >= d && ldv >= d && aligned16(v) && !(ldv & 3), "score_topk: v must be 16-B aligned rows");
  GNNREC_REQUIRE(!seen_ptr || seen_col || n_users_batch == 0, "score_topk: seen_ptr without seen_col");
  const bool split = n_split > 1;
  const TopkParams p{u, ldu, n_users_batch, v, ldv, n_items, seen_ptr, seen_col, k,
                     split ? work_idx : out_idx, split ? work_score : out_score, n_split};
  hipStream_t s = as_hip(stream);
  int rc;
  switch (d) {
    case 16: rc = dispatch_k<16>(p, s); break;
    case 32: rc = dispatch_k<32>(p, s); break;
    case 64: rc = dispatch_k<64>(p, s); break;
    case 128: rc = dispatch_k<128>(p, s); break;
    case 256: rc = dispatch_k<256>(p, s); break;
    default: set_error("score_topk: d=%d unsupported (16, 32, 64, 128, 256)", d); return GNNREC_EUNSUPPORTED;
  }
  if (rc != GNNREC_OK || !split) return rc;
  hipLaunchKernelGGL(topk_merge_kernel, dim3((unsigned)ceil_div(n_users_batch, kBlock / 64)),
                     dim3(kBlock), 0, s, work_idx, work_score, n_users_batch, n_split, k, out_idx,
                     out_score);
  return check_launch("topk_merge");
}

extern "C" int gnnrec_score_topk_f32(const float* u, int64_t ldu, int64_t n_users_batch,
                                     const float* v, int64_t ldv, int64_t n_items, int32_t d,
                                     const int64_t* seen_ptr, const int32_t* seen_col, int32_t k,
                                     int64_t* out_idx, float* out_score, gnnrec_stream_t stream) {
  return gnnrec_score_topk_split_f32(u, ldu, n_users_batch, v, ldv, n_items, d, seen_ptr, seen_col,
                                     k, 1, nullptr, nullptr, out_idx, out_score, stream);
}
