// Column-ordered ("tiled") SpMM hop for d = 64 (gnnrec_spmm_tiled_f32).
//
// Same arithmetic as spmm_vec_kernel — replaces torch.sparse.mm(adj, x) of the reference
// (baselines/lightgcn.py:88,178) with y[r] = fmaf chain over the row's neighbours in ascending
// column order from +0 — but a different schedule. The row-parallel hop gathers every
// neighbour row from beyond L2 (G100M: 16x the compulsory bytes). Here one persistent
// 1024-thread workgroup per CU owns R destination rows per pass with fp32 accumulators in
// LDS, and its 16 waves walk the rows' edges PANEL BY PANEL in ascending source column
// (a step = one panel; a workgroup barrier between steps, so a row may move to another wave
// from one step to the next without reordering its chain). The workgroups of a blockIdx % 8
// group (one XCD under round-robin placement — speed only, never correctness) meet at every
// pass start (bounded counter wait), so they sweep the same panels together and a gathered
// source row is reused from the XCD's L2 by the group's other rows: L2 hit rate 12 % -> 32 %.
//
// Plan (host, gnnrec_tiled_plan_build): per (block, wave) a run of chunks of kChunk slots
//   xoff u32 = byte offset of the source row, val f32,
//   meta u16 = local row (10 bits) | barriers before the chunk (5 bits, slot 0) << 10
//              | "continues the previous slot's row" << 15.
// Inside a step a wave's rows are laid back to back, each a run in column order; a slot that
// continues a run inside the same chunk takes the previous slot's register value instead of
// the LDS accumulator (which that slot only writes at the chunk's end). Unused slots are
// dummies: row R (a scratch row), val 0, xoff of the chunk's first slot.
#include <algorithm>
#include <atomic>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "common.h"

namespace gnnrec {

constexpr int kTiledWaves = GNNREC_TILED_WAVES;
constexpr int kTiledChunk = GNNREC_TILED_CHUNK;
constexpr int kTiledD = 64;
constexpr int kTiledMaxBar = 31;
static_assert(GNNREC_TILED_MAX_ROWS < 1023, "row field is 10 bits (row R = scratch)");
static_assert((GNNREC_TILED_MAX_ROWS + 1) * kTiledD * 4 <= 160 * 1024, "LDS");

// ---- device -----------------------------------------------------------------------------
struct TiledChunk {
  uint32_t o[kTiledChunk];
  float v[kTiledChunk];
  uint32_t m[kTiledChunk / 2];
  float x[kTiledChunk];
};

// Slot metadata by scalar loads (the chunk offset is wave-uniform), then the chunk's 16 row
// gathers (64 lanes x 4 B each) by buffer loads with the row offset in soffset.
__device__ __forceinline__ void tiled_fetch(const uint32_t* __restrict__ sx,
                                            const float* __restrict__ sv,
                                            const uint32_t* __restrict__ sm, int64_t c,
                                            __amdgpu_buffer_rsrc_t xr, int lane, TiledChunk& k) {
#pragma unroll
  for (int t = 0; t < kTiledChunk; ++t) {
    k.o[t] = sx[c + t];
    k.v[t] = sv[c + t];
  }
#pragma unroll
  for (int t = 0; t < kTiledChunk / 2; ++t) k.m[t] = sm[c / 2 + t];
#pragma unroll
  for (int t = 0; t < kTiledChunk; ++t)
    k.x[t] = __builtin_bit_cast(float,
                                __builtin_amdgcn_raw_buffer_load_b32(xr, lane * 4, k.o[t], 0));
}

__device__ __forceinline__ void tiled_apply(float* acc, int lane, const TiledChunk& k,
                                            int& cur) {
  const int bar = (k.m[0] >> 10) & kTiledMaxBar;
  for (int i = 0; i < bar; ++i) __syncthreads();   // step boundaries before this chunk
  cur += bar;
  int rr[kTiledChunk];
#pragma unroll
  for (int t = 0; t < kTiledChunk; ++t)
    rr[t] = ((t & 1) ? (k.m[t / 2] >> 16) : k.m[t / 2]) & 1023;
  float av[kTiledChunk];
#pragma unroll
  for (int t = 0; t < kTiledChunk; ++t) av[t] = acc[rr[t] * kTiledD + lane];
#pragma unroll
  for (int t = 0; t < kTiledChunk; ++t) {
    float base = av[t];
    if (t > 0) {
      const bool chain = ((t & 1) ? (k.m[t / 2] >> 31) : (k.m[t / 2] >> 15)) & 1;
      base = chain ? av[t - 1] : base;
    }
    av[t] = __builtin_fmaf(k.v[t], k.x[t], base);
  }
#pragma unroll
  for (int t = 0; t < kTiledChunk; ++t) acc[rr[t] * kTiledD + lane] = av[t];
}

__global__ __launch_bounds__(kTiledWaves * 64) void tiled_hop_kernel(
    const uint32_t* __restrict__ sx, const float* __restrict__ sv,
    const uint32_t* __restrict__ sm, const int64_t* __restrict__ wptr,
    const int32_t* __restrict__ nsteps, int n_blocks, int R, const float* __restrict__ x,
    uint32_t x_bytes, float* __restrict__ y, int64_t ldy, int64_t n_rows, int epi,
    const float* __restrict__ self, int64_t ld_self, float* __restrict__ accg, int64_t ld_acc,
    float acc_div, unsigned* __restrict__ sync) {
  extern __shared__ float acc[];  // [(R+1)][64]: row R is the dummies' scratch row
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0, (int)x_bytes, 0x00020000);
  unsigned* ctr = sync + (blockIdx.x % 8) * 32;   // the group's counter, own 128-B line
  const long long G = gridDim.x / 8 + ((blockIdx.x % 8) < (gridDim.x % 8) ? 1 : 0);
  long long pass = 0;
  for (int blk = blockIdx.x; blk < n_blocks; blk += gridDim.x, ++pass) {
    if (threadIdx.x == 0 && pass > 0) {
      // pass start: report the finished pass, wait (<= 200 us) for the group's others
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long t0 = wall_clock64();
      while ((long long)__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                 G * pass &&
             wall_clock64() - t0 < 20000)
        __builtin_amdgcn_s_sleep(2);
    }
    for (int i = threadIdx.x; i < (R + 1) * kTiledD; i += kTiledWaves * 64) acc[i] = 0.f;
    __syncthreads();
    const int64_t s = (int64_t)blk * kTiledWaves + w;
    const int64_t b = wptr[s], e = wptr[s + 1];
    int cur = 0;
    if (b < e) {
      // two chunk register sets: the next chunk's gathers fly while this one's chain runs
      TiledChunk A, B;
      int64_t c = b;
      tiled_fetch(sx, sv, sm, c, xr, lane, A);
      for (;;) {
        tiled_fetch(sx, sv, sm, c + kTiledChunk, xr, lane, B);
        tiled_apply(acc, lane, A, cur);
        c += kTiledChunk;
        if (c >= e) break;
        tiled_fetch(sx, sv, sm, c + kTiledChunk, xr, lane, A);
        tiled_apply(acc, lane, B, cur);
        c += kTiledChunk;
        if (c >= e) break;
      }
    }
    const int ns = nsteps[blk];
    for (int i = cur; i < ns; ++i) __syncthreads();  // this wave's remaining steps + the last
    const int64_t r0 = (int64_t)blk * R;
    for (int i = w; i < R; i += kTiledWaves) {
      const int64_t r = r0 + i;
      if (r >= n_rows) break;
      const float a = acc[i * kTiledD + lane];
      if (!(epi & GNNREC_EPI_NO_Y)) y[r * ldy + lane] = a;
      if (epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)) {
        float bsum = (epi & GNNREC_EPI_ACC_INIT) ? self[r * ld_self + lane] : accg[r * ld_acc + lane];
        bsum = bsum + a;
        if (epi & GNNREC_EPI_ACC_DIV) bsum = bsum / acc_div;
        accg[r * ld_acc + lane] = bsum;
      }
    }
    __syncthreads();
  }
  // finished: never hold the group back again
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1u << 24, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- host plan builder --------------------------------------------------------------------
namespace {

struct Run {
  int32_t p, row;   // panel, local row
  int64_t k;        // first edge (absolute index into col/val)
  int32_t n;        // edges of the row in this panel
};

struct BlockPlan {
  std::vector<uint32_t> xoff[kTiledWaves];
  std::vector<float> val[kTiledWaves];
  std::vector<uint16_t> meta[kTiledWaves];
  int32_t nsteps = 0;
};

struct TiledPlan {
  int64_t n_blocks = 0;
  std::vector<BlockPlan> blocks;
};

void push_slot(BlockPlan& bp, int w, uint32_t xo, float v, uint16_t m) {
  bp.xoff[w].push_back(xo);
  bp.val[w].push_back(v);
  bp.meta[w].push_back(m);
}

struct Slot {
  const Run* run;   // nullptr: dummy
  int32_t t;        // edge of the run
};

void build_block(const int64_t* rp, const int32_t* col, const float* val, int64_t n_rows,
                 int R, int panel, int sub_panel, int64_t row_bytes, int64_t b, BlockPlan& out) {
  std::vector<Slot> slots, seq, pending, deferred;
  std::vector<int> in_chunk, blocked;
  const int64_t r0 = b * R, r1 = std::min<int64_t>(n_rows, r0 + R);
  std::vector<Run> runs;
  for (int64_t r = r0; r < r1; ++r) {
    int64_t k = rp[r];
    const int64_t e = rp[r + 1];
    while (k < e) {
      const int32_t p = col[k] / panel;
      int64_t j = k;
      while (j < e && col[j] / panel == p) ++j;
      runs.push_back({p, (int32_t)(r - r0), k, (int32_t)(j - k)});
      k = j;
    }
  }
  std::stable_sort(runs.begin(), runs.end(), [](const Run& a, const Run& c) { return a.p < c.p; });
  int32_t cur[kTiledWaves] = {};    // step of each wave's last emitted chunk
  int64_t load[kTiledWaves];
  std::vector<const Run*> wl[kTiledWaves];
  std::vector<const Run*> g;
  int32_t step = 0;
  size_t i = 0;
  while (i < runs.size()) {
    size_t j = i;
    while (j < runs.size() && runs[j].p == runs[i].p) ++j;
    // LPT: longest run first onto the least loaded wave
    g.clear();
    for (size_t q = i; q < j; ++q) g.push_back(&runs[q]);
    std::stable_sort(g.begin(), g.end(), [](const Run* a, const Run* c) { return a->n > c->n; });
    for (int w = 0; w < kTiledWaves; ++w) {
      load[w] = 0;
      wl[w].clear();
    }
    for (const Run* e : g) {
      int w = 0;
      for (int q = 1; q < kTiledWaves; ++q)
        if (load[q] < load[w]) w = q;
      load[w] += e->n;
      wl[w].push_back(e);
    }
    for (int w = 0; w < kTiledWaves; ++w) {
      if (wl[w].empty()) continue;
      // the wave's slots in ascending column sub-panel, rows in order inside one (a row's
      // edges keep their column order): the group's waves sweep the panel together
      slots.clear();
      for (const Run* e : wl[w])
        for (int t = 0; t < e->n; ++t) slots.push_back({e, t});
      if (sub_panel > 0)
        std::stable_sort(slots.begin(), slots.end(), [&](const Slot& a, const Slot& c) {
          const int32_t ka = col[a.run->k + a.t] / sub_panel, kc = col[c.run->k + c.t] / sub_panel;
          return ka != kc ? ka < kc : a.run->row < c.run->row;
        });
      // chunks: a row appears in a chunk only as one run of consecutive slots (the kernel reads
      // every accumulator at the chunk start); a slot that would repeat a row non-adjacently is
      // deferred to a later chunk with the rest of that row (per-row order kept)
      seq.clear();
      pending.swap(slots);
      while (!pending.empty()) {
        deferred.clear();
        in_chunk.clear();
        blocked.clear();
        int n = 0, last = -1;
        const size_t start = seq.size();
        for (size_t q = 0; q < pending.size(); ++q) {
          const Slot& sl = pending[q];
          if (n == kTiledChunk) {   // chunk full: the rest keeps its order for the next ones
            deferred.insert(deferred.end(), pending.begin() + q, pending.end());
            break;
          }
          const int r = sl.run->row;
          const bool is_blocked = std::find(blocked.begin(), blocked.end(), r) != blocked.end();
          const bool seen = std::find(in_chunk.begin(), in_chunk.end(), r) != in_chunk.end();
          if (is_blocked || (seen && r != last)) {
            if (seen && r != last && !is_blocked) blocked.push_back(r);
            deferred.push_back(sl);
            continue;
          }
          seq.push_back(sl);
          if (!seen) in_chunk.push_back(r);
          last = r;
          ++n;
        }
        while (seq.size() - start < (size_t)kTiledChunk) seq.push_back({nullptr, 0});
        pending.swap(deferred);
      }
      int32_t bar = step - cur[w];
      for (size_t c = 0; c < seq.size(); c += kTiledChunk) {
        while (bar > kTiledMaxBar) {   // more barriers than the field holds: an empty chunk
          for (int s = 0; s < kTiledChunk; ++s)
            push_slot(out, w, 0u, 0.f, (uint16_t)(R | (s == 0 ? kTiledMaxBar << 10 : 0)));
          bar -= kTiledMaxBar;
        }
        const uint32_t x0 = (uint32_t)(col[seq[c].run->k + seq[c].t] * row_bytes);
        for (int s = 0; s < kTiledChunk; ++s) {
          const Slot& sl = seq[c + s];
          const int bits = s == 0 ? bar << 10 : 0;
          if (!sl.run) {            // dummy: scratch row, value 0, an already-fetched row
            push_slot(out, w, x0, 0.f, (uint16_t)(R | bits));
            continue;
          }
          const int64_t k = sl.run->k + sl.t;
          const int chain = (s > 0 && seq[c + s - 1].run == sl.run) ? 1 : 0;
          push_slot(out, w, (uint32_t)(col[k] * row_bytes), val[k],
                    (uint16_t)(sl.run->row | bits | (chain << 15)));
        }
        bar = 0;
      }
      cur[w] = step;
    }
    ++step;
    i = j;
  }
  out.nsteps = step;
}

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_tiled_plan_build(const int64_t* row_ptr, const int32_t* col,
                                       const float* val, int64_t n_rows, int32_t rows_per_block,
                                       int32_t panel, int32_t sub_panel, int64_t row_bytes,
                                       int32_t n_threads, void** plan, int64_t* n_slots,
                                       int64_t* n_blocks) {
  GNNREC_REQUIRE(row_ptr && plan && n_slots && n_blocks && n_rows >= 0, "tiled_plan: bad args");
  GNNREC_REQUIRE(rows_per_block >= 1 && rows_per_block <= GNNREC_TILED_MAX_ROWS,
                 "tiled_plan: rows_per_block must be in [1, %d]", GNNREC_TILED_MAX_ROWS);
  GNNREC_REQUIRE(panel >= 1 && sub_panel >= 0 && row_bytes > 0,
                 "tiled_plan: bad panel / sub_panel / row_bytes");
  const int64_t nnz = n_rows > 0 ? row_ptr[n_rows] - row_ptr[0] : 0;
  GNNREC_REQUIRE(nnz == 0 || (col && val), "tiled_plan: null col/val");
  auto* pl = new (std::nothrow) TiledPlan;
  GNNREC_REQUIRE(pl != nullptr, "tiled_plan: out of host memory");
  pl->n_blocks = (n_rows + rows_per_block - 1) / rows_per_block;
  pl->blocks.resize(pl->n_blocks);
  int t = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
  t = std::max(1, std::min<int>(t, (int)std::max<int64_t>(1, pl->n_blocks)));
  std::atomic<int64_t> next{0};
  std::atomic<bool> bad_col{false};
  auto worker = [&] {
    for (int64_t b; (b = next.fetch_add(1)) < pl->n_blocks;) {
      const int64_t r0 = b * rows_per_block, r1 = std::min<int64_t>(n_rows, r0 + rows_per_block);
      for (int64_t k = row_ptr[r0]; k < row_ptr[r1]; ++k)
        if (col[k] < 0 || (int64_t)col[k] * row_bytes + row_bytes > (int64_t)UINT32_MAX)
          bad_col = true;
      build_block(row_ptr, col, val, n_rows, rows_per_block, panel, sub_panel, row_bytes, b,
                  pl->blocks[b]);
    }
  };
  std::vector<std::thread> pool;
  for (int i = 1; i < t; ++i) pool.emplace_back(worker);
  worker();
  for (auto& th : pool) th.join();
  if (bad_col) {
    delete pl;
    set_error("tiled_plan: a source row lies beyond 4 GB of the table (col * row_bytes)");
    return GNNREC_EINVAL;
  }
  int64_t tot = 0;
  for (const auto& bp : pl->blocks)
    for (int w = 0; w < kTiledWaves; ++w) tot += (int64_t)bp.xoff[w].size();
  *n_slots = tot;
  *n_blocks = pl->n_blocks;
  *plan = pl;
  return GNNREC_OK;
}

extern "C" int gnnrec_tiled_plan_emit(void* plan, uint32_t* xoff, float* val, uint16_t* meta,
                                      int64_t* wave_ptr, int32_t* n_steps) {
  GNNREC_REQUIRE(plan && xoff && val && meta && wave_ptr && n_steps, "tiled_emit: null pointer");
  auto* pl = static_cast<TiledPlan*>(plan);
  const int64_t nb = pl->n_blocks;
  wave_ptr[0] = 0;
  for (int64_t b = 0; b < nb; ++b)
    for (int w = 0; w < kTiledWaves; ++w)
      wave_ptr[b * kTiledWaves + w + 1] =
          wave_ptr[b * kTiledWaves + w] + (int64_t)pl->blocks[b].xoff[w].size();
  for (int64_t b = 0; b < nb; ++b) {
    const BlockPlan& bp = pl->blocks[b];
    n_steps[b] = bp.nsteps;
    for (int w = 0; w < kTiledWaves; ++w) {
      const int64_t o = wave_ptr[b * kTiledWaves + w];
      std::copy(bp.xoff[w].begin(), bp.xoff[w].end(), xoff + o);
      std::copy(bp.val[w].begin(), bp.val[w].end(), val + o);
      std::copy(bp.meta[w].begin(), bp.meta[w].end(), meta + o);
    }
  }
  // tail chunk for the last prefetch: harmless slots (row 0 of x, scratch row)
  const int64_t end = wave_ptr[nb * kTiledWaves];
  const uint16_t scratch = (uint16_t)(nb > 0 ? 1023 : 0);
  for (int s = 0; s < kTiledChunk; ++s) {
    xoff[end + s] = 0;
    val[end + s] = 0.f;
    meta[end + s] = scratch;
  }
  return GNNREC_OK;
}

extern "C" int gnnrec_tiled_plan_free(void* plan) {
  delete static_cast<TiledPlan*>(plan);
  return GNNREC_OK;
}

extern "C" int gnnrec_spmm_tiled_f32(const uint32_t* xoff, const float* val, const uint16_t* meta,
                                     const int64_t* wave_ptr, const int32_t* n_steps,
                                     int64_t n_blocks, int32_t rows_per_block, const float* x,
                                     int64_t x_rows, int64_t ldx, float* y, int64_t ldy,
                                     int64_t n_rows, int32_t d, int32_t epi, const float* self,
                                     int64_t ld_self, float* acc, int64_t ld_acc, float acc_div,
                                     uint32_t* sync, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(d == kTiledD, "spmm_tiled: d must be 64 (got %d)", (int)d);
  GNNREC_REQUIRE(rows_per_block >= 1 && rows_per_block <= GNNREC_TILED_MAX_ROWS,
                 "spmm_tiled: bad rows_per_block");
  GNNREC_REQUIRE(n_rows >= 0 && n_blocks == (n_rows + rows_per_block - 1) / rows_per_block,
                 "spmm_tiled: n_blocks does not match n_rows / rows_per_block");
  GNNREC_REQUIRE(ldx >= d && x_rows >= 0 && x_rows * ldx * 4 < ((int64_t)1 << 32),
                 "spmm_tiled: the x table must be under 4 GB with ldx >= 64");
  GNNREC_REQUIRE((epi & GNNREC_EPI_NO_Y) || (y && ldy >= d), "spmm_tiled: null y or ldy < d");
  GNNREC_REQUIRE(!(epi & GNNREC_EPI_ACC_INIT) || (self && ld_self >= d),
                 "spmm_tiled: ACC_INIT needs self");
  GNNREC_REQUIRE(!(epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)) || (acc && ld_acc >= d),
                 "spmm_tiled: ACC needs acc");
  if (n_rows == 0) return GNNREC_OK;
  GNNREC_REQUIRE(xoff && val && meta && wave_ptr && n_steps && x && sync,
                 "spmm_tiled: null pointer");
  GNNREC_REQUIRE(n_blocks < INT32_MAX, "spmm_tiled: too many blocks");
  hipStream_t s = as_hip(stream);
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  const size_t lds = (size_t)(rows_per_block + 1) * kTiledD * sizeof(float);
  static std::once_flag lds_attr;   // per-process: the kernel may take all 160 KB of LDS
  std::call_once(lds_attr, [] {
    (void)hipFuncSetAttribute((const void*)tiled_hop_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  });
  if (hipMemsetAsync(sync, 0, GNNREC_TILED_SYNC_WORDS * sizeof(uint32_t), s) != hipSuccess)
    return check_launch("spmm_tiled (sync reset)");
  const int grid = (int)std::min<int64_t>(cus, n_blocks);
  hipLaunchKernelGGL(tiled_hop_kernel, dim3(grid), dim3(kTiledWaves * 64), lds, s, xoff, val,
                     reinterpret_cast<const uint32_t*>(meta), wave_ptr, n_steps, (int)n_blocks,
                     (int)rows_per_block, x, (uint32_t)(x_rows * ldx * 4), y, ldy, n_rows, epi,
                     self, ld_self, acc, ld_acc, acc_div, sync);
  return check_launch("spmm_tiled");
}
