// Device planner of the column-ordered hop (gnnrec_tiled_plan_device).
//
// Builds, in HBM, exactly the arrays the host planner (tiled.hip: build_block /
// stream_slots / gnnrec_tiled_plan_emit) writes — same slots, values, headers, wave_ptr and
// n_steps, bit for bit (tests/test_tiled_plan_gpu.py) — so a device-resident operand is
// re-laid out without a host round trip (G100M: 2.0 s on 16 host threads).
//
// One 64-lane workgroup per block at a time (a persistent grid walks the blocks); lane v is
// slot stream v of the block (GNNREC_TILED_WAVES x GNNREC_TILED_GROUPS = 64 streams). Per
// step (one source-column panel that holds edges of the block):
//   1. the step's panel: the smallest panel any row's cursor points into (wave min);
//   2. one run per row with edges in it (its consecutive edges in the panel);
//   3. LPT: runs by length descending, then row (a bitonic sort of 32-bit keys in LDS), each
//      onto the first least-loaded stream (a wave min of load << 6 | lane per run);
//   4. per stream (lane): its slots in (column sub-panel, row, edge) order — a merge of its
//      runs sorted by row — then cut into groups of 4 with the host's one-run rule
//      (deferred repeats, padding), into per-workgroup scratch;
//   5. per wave of the block: chunks of 8 steps x 8 streams, header and chain mask (two
//      ballots), written at the offsets a counting pass of the same kernel produced.
// Scratch per workgroup: 6 * cap + 512 words (slot lists, their ping-pong copy and the padded
// sequences, at most 4 entries per slot + 7) for steps of at most `cap` slots (error 2, and
// the caller retries with a larger cap, beyond).
#include <climits>

#include "common.h"

namespace gnnrec {
namespace {

constexpr int kPW = GNNREC_TILED_WAVES;
constexpr int kPG = GNNREC_TILED_GROUPS;
constexpr int kPS = GNNREC_TILED_STEPS;
constexpr int kPV = kPW * kPG;                    // slot streams per block
constexpr int kPA = 4;                            // slots per apply group (GNNREC_TILED_APPLY)
constexpr int kPRowBits = 11;
constexpr uint32_t kPRowMask = (1u << kPRowBits) - 1;
constexpr int kPMaxRows = GNNREC_TILED_MAX_ROWS + 1;
constexpr int kPKeys = 2048;                      // >= rows per block, a power of two
constexpr int kPNMax = (1 << 21) - 1;             // run length field of a sort key
// a run (one row's slots in one step) is kept in 16 bits in LDS: 23 040 B of LDS per
// workgroup, 7 workgroups per CU, so G100M's 1 791 blocks are planned in one round (6 per CU
// and 32-bit lengths left 255 blocks for a second round). Longer runs fail the plan (error 3).
constexpr int kPLenMax = 32767;
static_assert(kPLenMax <= kPNMax, "run length within the key field");
constexpr int kPMaxPanel = 1 << 20;
constexpr uint64_t kPPad = ~0ull;
static_assert(kPV == 64, "one lane per slot stream");
static_assert(kPS == 2 * kPA && GNNREC_TILED_CHUNK == kPG * kPS, "chunk = 8 steps x 8 streams");
static_assert(kPKeys >= kPMaxRows, "one key per row");
#if defined(GNNREC_TILED_APPLY) && GNNREC_TILED_APPLY != 4
#error "the device planner implements the default apply group of 4 slots"
#endif
#if defined(GNNREC_TILED_NOCHAIN) && GNNREC_TILED_NOCHAIN
#error "the device planner implements the chained plan"
#endif

struct PlanArgs {
  const int64_t* rp;
  const int32_t* col;
  const float* val;
  int64_t n_rows;
  int R, panel, sub;
  int64_t n_blocks;
  uint64_t* scratch;
  int64_t cap;          // max slots of a step (slot-list region of one workgroup)
  int64_t* chunks;      // count pass: chunks per (block, wave)
  int32_t* nsteps;      // count pass: steps per block
  const int64_t* wave_ptr;   // emit pass: chunk offsets
  uint32_t* slot;
  float* vout;
  uint32_t* hdr;
  int32_t* err;
};

__device__ __forceinline__ uint64_t shfl64(uint64_t x, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)x, src);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(x >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_min64(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, o);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), o);
    const uint64_t y = ((uint64_t)hi << 32) | lo;
    x = y < x ? y : x;
  }
  return x;
}

// a 64-lane reduction by DPP inside each 16-lane row (xor 1, xor 2, half-row and row
// mirrors), then the 4 rows by v_readlane: no LDS round trips (every lane must be active)
template <class Op>
__device__ __forceinline__ int wave_reduce_dpp(int x, Op op) {
  x = op(x, __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false));    // quad_perm [1,0,3,2]
  x = op(x, __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false));    // quad_perm [2,3,0,1]
  x = op(x, __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false));   // row_half_mirror
  x = op(x, __builtin_amdgcn_mov_dpp(x, 0x140, 0xF, 0xF, false));   // row_mirror
  return op(op(__builtin_amdgcn_readlane(x, 0), __builtin_amdgcn_readlane(x, 16)),
            op(__builtin_amdgcn_readlane(x, 32), __builtin_amdgcn_readlane(x, 48)));
}

__device__ __forceinline__ int wave_min32(int x) {
  return wave_reduce_dpp(x, [](int a, int b) { return min(a, b); });
}

__device__ __forceinline__ int wave_max32(int x) {
  return wave_reduce_dpp(x, [](int a, int b) { return max(a, b); });
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
  return (uint32_t)wave_reduce_dpp((int)x, [](int a, int b) {
    return (int)min((uint32_t)a, (uint32_t)b);
  });
}

__device__ __forceinline__ void fail(int32_t* err, int code) {
  __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool failed(const int32_t* err) {
  return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

// ascending bitonic sort of s[0, n) (n a power of two) by one wave
__device__ void bitonic64(uint32_t* s, int n, int lane) {
  for (int k = 2; k <= n; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = lane; i < n; i += 64) {
        const int l = i ^ j;
        if (l > i) {
          const uint32_t x = s[i], y = s[l];
          if ((x > y) == ((i & k) == 0)) {
            s[i] = y;
            s[l] = x;
          }
        }
      }
      __syncthreads();
    }
}

__global__ __launch_bounds__(64) void tiled_plan_kernel(PlanArgs a, int emit) {
  __shared__ int32_t s_pos[kPMaxRows], s_end[kPMaxRows];
  __shared__ int16_t s_len[kPMaxRows];
  __shared__ uint32_t s_key[kPKeys];
  __shared__ uint8_t s_asg[kPKeys];
  const int lane = threadIdx.x;
  uint64_t* const A = a.scratch + (int64_t)blockIdx.x * (6 * a.cap + 512);
  uint64_t* const A2 = A + a.cap;
  uint64_t* const B = A2 + a.cap;
  for (int64_t b = blockIdx.x; b < a.n_blocks; b += gridDim.x) {
    if (failed(a.err)) return;
    const int64_t r0 = b * a.R, r1 = min(a.n_rows, r0 + a.R);
    const int nr = (int)(r1 - r0);
    const int64_t kb = a.rp[r0];
    const int32_t* col = a.col + kb;   // the block's edges, relative offsets
    const float* val = a.val + kb;
    const int64_t nnzb = a.rp[r1] - kb;
    if (nnzb >= INT32_MAX) {
      if (lane == 0) fail(a.err, 2);
      return;
    }
    for (int i = lane; i < nr; i += 64) {
      s_pos[i] = (int32_t)(a.rp[r0 + i] - kb);
      s_end[i] = (int32_t)(a.rp[r0 + i + 1] - kb);
    }
    bool bad = false;
    for (int64_t k = lane; k < nnzb; k += 64) bad |= col[k] < 0;
    if (__ballot(bad)) {
      if (lane == 0) fail(a.err, 1);
      return;
    }
    __syncthreads();
    int32_t curw = 0;                                    // lane w < 8: step of wave w's last chunk
    int64_t pw = (emit && lane < kPW) ? a.wave_ptr[b * kPW + lane] : 0;   // its next chunk
    int64_t cntw = 0;
    int step = 0;
    for (;;) {
      // 1. the step's panel
      int pm = INT_MAX;
      for (int i = lane; i < nr; i += 64)
        if (s_pos[i] < s_end[i]) pm = min(pm, col[s_pos[i]] / a.panel);
      pm = wave_min32(pm);
      if (pm == INT_MAX) break;
      const uint32_t base = (uint32_t)pm * (uint32_t)a.panel;
      // 2. runs, as LPT sort keys (length descending, then row)
      int nk = 0;
      bool too_long = false;
      for (int i0 = 0; i0 < nr; i0 += 64) {
        const int i = i0 + lane;
        int n = 0;
        if (i < nr) {
          const int32_t k = s_pos[i], e = s_end[i];
          while (k + n < e && col[k + n] / a.panel == pm) ++n;
          s_len[i] = (int16_t)min(n, kPLenMax);
          too_long |= n > kPLenMax;
        }
        const uint64_t m = __ballot(n > 0);
        if (n > 0)
          s_key[nk + __popcll(m & ((1ull << lane) - 1))] =
              ((uint32_t)(kPNMax - min(n, kPNMax)) << kPRowBits) | (uint32_t)i;
        nk += __popcll(m);
      }
      if (__ballot(too_long)) {
        if (lane == 0) fail(a.err, 3);
        return;
      }
      int np2 = 1;
      while (np2 < nk) np2 <<= 1;
      for (int i = nk + lane; i < np2; i += 64) s_key[i] = 0xFFFFFFFFu;
      __syncthreads();
      bitonic64(s_key, np2, lane);
      // 3. LPT onto the first least-loaded stream
      uint32_t load = 0;
      for (int idx = 0; idx < nk; ++idx) {
        const uint32_t key = s_key[idx];
        const int n = kPNMax - (int)(key >> kPRowBits);
        // loads below 2^26 (nnzb bounds them): one 32-bit DPP min of load << 6 | lane
        const int v = nnzb < (1 << 26)
                          ? (int)(wave_min_u32((load << 6) | (uint32_t)lane) & 63)
                          : (int)(wave_min64(((uint64_t)load << 6) | (uint32_t)lane) & 63);
        if (lane == v) {
          load += (uint32_t)n;
          s_asg[idx] = (uint8_t)v;
        }
      }
      __syncthreads();
      // 4. this stream's slots: A[aoff, aoff + load) in (sub-panel, row, edge) order
      int aoff = (int)load;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(aoff, o);
        if (lane >= o) aoff += y;
      }
      aoff -= (int)load;
      // the step's slots must fit the scratch regions (sized for a step, not a block: the
      // caller retries with a larger cap when this fails)
      if (__shfl(aoff + (int)load, 63) > a.cap) {
        if (lane == 0) fail(a.err, 2);
        return;
      }
      uint64_t* const Rn = A2 + aoff;   // the stream's runs {edge << 32 | n << 11 | row}
      uint64_t* const S = A + aoff;
      int nrun = 0;
      for (int idx = 0; idx < nk; ++idx)
        if (s_asg[idx] == lane) {
          const uint32_t key = s_key[idx];
          const int i = (int)(key & kPRowMask);
          const uint32_t n = (uint32_t)(kPNMax - (int)(key >> kPRowBits));
          Rn[nrun++] = ((uint64_t)(uint32_t)s_pos[i] << 32) | ((uint64_t)n << kPRowBits) | (uint32_t)i;
        }
      int ns = 0;
      if (a.sub > 0) {
        for (int x = 1; x < nrun; ++x) {   // runs by row (one run per row and step)
          const uint64_t e = Rn[x];
          int y = x - 1;
          while (y >= 0 && (Rn[y] & kPRowMask) > (e & kPRowMask)) {
            Rn[y + 1] = Rn[y];
            --y;
          }
          Rn[y + 1] = e;
        }
        int left = (int)load;
        while (left > 0) {
          int smin = INT_MAX;
          for (int x = 0; x < nrun; ++x) {
            const uint64_t e = Rn[x];
            if ((e >> kPRowBits) & kPNMax) smin = min(smin, col[(int32_t)(e >> 32)] / a.sub);
          }
          for (int x = 0; x < nrun; ++x) {
            const uint64_t e = Rn[x];
            int32_t k = (int32_t)(e >> 32);
            uint32_t n = (uint32_t)((e >> kPRowBits) & kPNMax);
            const uint32_t row = (uint32_t)(e & kPRowMask);
            while (n > 0 && col[k] / a.sub == smin) {
              S[ns++] = ((uint64_t)(uint32_t)k << kPRowBits) | row;
              ++k;
              --n;
              --left;
            }
            Rn[x] = ((uint64_t)(uint32_t)k << 32) | ((uint64_t)n << kPRowBits) | row;
          }
        }
      } else {
        for (int x = 0; x < nrun; ++x) {
          const uint64_t e = Rn[x];
          const int32_t k = (int32_t)(e >> 32);
          const uint32_t n = (uint32_t)((e >> kPRowBits) & kPNMax);
          for (uint32_t t = 0; t < n; ++t)
            S[ns++] = ((uint64_t)(uint32_t)(k + (int32_t)t) << kPRowBits) | (e & kPRowMask);
        }
      }
      // groups of kPA: a row once per group as one run, repeats deferred; padded
      const int64_t boff = 4 * (int64_t)aoff + 8 * lane;
      uint64_t* const O = B + boff;
      int L = 0;
      uint64_t* src = S;
      uint64_t* dst = A2 + aoff;
      int m = ns;
      while (m > 0) {
        int n = 0, last = -1, nin = 0, nbl = 0, dc = 0;
        int ing[kPA], blk[kPA];
        for (int q = 0; q < m; ++q) {
          const uint64_t sl = src[q];
          if (n == kPA) {
            for (int z = q; z < m; ++z) dst[dc++] = src[z];
            break;
          }
          const int r = (int)(sl & kPRowMask);
          bool isb = false, seen = false;
          for (int z = 0; z < nbl; ++z) isb |= blk[z] == r;
          for (int z = 0; z < nin; ++z) seen |= ing[z] == r;
          const bool rep = seen && r != last;
          if (isb || rep) {
            if (rep && !isb) blk[nbl++] = r;
            dst[dc++] = sl;
            continue;
          }
          O[L++] = sl;
          if (!seen) ing[nin++] = r;
          last = r;
          ++n;
        }
        if (dc > 0)
          for (; n < kPA; ++n) O[L++] = kPPad;
        uint64_t* t = src;
        src = dst;
        dst = t;
        m = dc;
      }
      while (L % kPS) O[L++] = kPPad;
      // 5. chunks of each wave of the block
      const int q = lane >> 3, t = lane & 7;
      for (int w = 0; w < kPW; ++w) {
        int nw = (q == w) ? L : 0;   // lanes 8w .. 8w+7 hold the wave's streams' lengths
        nw = wave_max32(nw);
        if (nw == 0) continue;       // no slot of this wave in the step: no chunk, no barrier
        const int nc = nw / kPS;
        if (!emit) {
          if (lane == w) cntw += nc;
        } else {
          const int64_t P = (int64_t)shfl64((uint64_t)pw, w);
          if (P + nc > a.wave_ptr[b * kPW + w + 1]) {   // the counting pass disagrees
            if (lane == 0) fail(a.err, 4);
            return;
          }
          const uint32_t bar = (uint32_t)(step - __shfl(curw, w));
          const int v = kPG * w + (lane >> 3);   // stream of this lane's slot (lane = 8 g + t)
          const int Lq = __shfl(L, v);
          const int64_t bq = (int64_t)shfl64((uint64_t)boff, v);
          for (int c = 0; c < nc; ++c) {
            const int idx = c * kPS + t;
            const uint64_t e = idx < Lq ? B[bq + idx] : kPPad;
            const bool real = e != kPPad;
            const uint64_t rm = __ballot(real);
            uint32_t x0 = 0;
            const uint64_t ef = shfl64(e, rm ? __ffsll((long long)rm) - 1 : 0);
            if (rm) x0 = (uint32_t)col[(int32_t)(ef >> kPRowBits)] - base;
            const uint64_t ep = (t > 0 && idx - 1 < Lq) ? B[bq + idx - 1] : kPPad;
            const uint64_t cm =
                __ballot(t > 0 && real && ep != kPPad && (ep & kPRowMask) == (e & kPRowMask));
            uint32_t word;
            float vv;
            if (real) {
              const int32_t k = (int32_t)(e >> kPRowBits);
              word = (((uint32_t)col[k] - base) << kPRowBits) | (uint32_t)(e & kPRowMask);
              vv = val[k];
            } else {
              word = (x0 << kPRowBits) | (uint32_t)a.R;
              vv = 0.f;
            }
            const int64_t o = (P + c) * GNNREC_TILED_CHUNK + lane;
            a.slot[o] = word;
            a.vout[o] = vv;
            if (lane < GNNREC_TILED_HDR_WORDS)
              a.hdr[(P + c) * GNNREC_TILED_HDR_WORDS + lane] =
                  lane == 0 ? (c == 0 ? bar : 0u)
                            : lane == 1 ? (uint32_t)cm : lane == 2 ? (uint32_t)(cm >> 32) : base;
          }
          if (lane == w) pw += nc;
        }
        if (lane == w) curw = step;
      }
      for (int i = lane; i < nr; i += 64) s_pos[i] += s_len[i];
      __syncthreads();
      ++step;
    }
    if (!emit) {
      if (lane < kPW) a.chunks[b * kPW + lane] = cntw;
      if (lane == 0) a.nsteps[b] = step;
    }
    __syncthreads();
  }
}

// the tail chunks after the last block's (read by the kernel's last prefetches)
__global__ __launch_bounds__(256) void tiled_plan_tail_kernel(const int64_t* end_chunk,
                                                              uint32_t* slot, float* vout,
                                                              uint32_t* hdr) {
  const int64_t e = *end_chunk;
  const int i = threadIdx.x;
  for (int s = i; s < GNNREC_TILED_TAIL * GNNREC_TILED_CHUNK; s += blockDim.x) {
    slot[e * GNNREC_TILED_CHUNK + s] = kPRowMask;
    vout[e * GNNREC_TILED_CHUNK + s] = 0.f;
  }
  if (i < GNNREC_TILED_TAIL * GNNREC_TILED_HDR_WORDS) hdr[e * GNNREC_TILED_HDR_WORDS + i] = 0u;
}

// Row statistics of a device CSR in one workgroup: out[0] = the longest row, out[1] = the most
// edges of any block of `block_rows` consecutive rows (0 when block_rows <= 0). One kernel of
// this library instead of a chain of torch reductions: in a fresh process every torch kernel's
// first launch loads its code object, which cost the plan build ≈ 0.2 s (profiles/r06/).
__global__ __launch_bounds__(1024) void csr_row_stats_kernel(const int64_t* __restrict__ row_ptr,
                                                             int64_t n_rows, int64_t block_rows,
                                                             int64_t* __restrict__ out) {
  __shared__ int64_t red[2][1024 / 64];
  int64_t mrow = 0, mblk = 0;
  for (int64_t r = threadIdx.x; r < n_rows; r += blockDim.x)
    mrow = max(mrow, row_ptr[r + 1] - row_ptr[r]);
  if (block_rows > 0) {
    const int64_t nb = (n_rows + block_rows - 1) / block_rows;
    for (int64_t b = threadIdx.x; b < nb; b += blockDim.x) {
      const int64_t e = min(n_rows, (b + 1) * block_rows);
      mblk = max(mblk, row_ptr[e] - row_ptr[b * block_rows]);
    }
  }
  for (int d = 32; d >= 1; d >>= 1) {
    mrow = max(mrow, __shfl_xor(mrow, d, 64));
    mblk = max(mblk, __shfl_xor(mblk, d, 64));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = mrow;
    red[1][w] = mblk;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    int64_t m = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) m = max(m, red[threadIdx.x][i]);
    out[threadIdx.x] = m;
  }
}

}  // namespace
}  // namespace gnnrec

using namespace gnnrec;

extern "C" int gnnrec_csr_row_stats(const int64_t* row_ptr, int64_t n_rows, int64_t block_rows,
                                    int64_t* out, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(row_ptr && out && n_rows >= 0, "csr_row_stats: bad args");
  hipLaunchKernelGGL(csr_row_stats_kernel, dim3(1), dim3(1024), 0, as_hip(stream), row_ptr,
                     n_rows, block_rows, out);
  return check_launch("csr_row_stats");
}

extern "C" int64_t gnnrec_tiled_plan_device_scratch_words(int64_t max_block_nnz,
                                                         int32_t workgroups) {
  return (int64_t)workgroups * (6 * max_block_nnz + 512);
}

extern "C" int gnnrec_tiled_plan_device(const int64_t* row_ptr, const int32_t* col,
                                        const float* val, int64_t n_rows, int32_t rows_per_block,
                                        int32_t panel, int32_t sub_panel, int64_t max_block_nnz,
                                        uint64_t* scratch, int32_t workgroups, int64_t* chunks,
                                        int32_t* n_steps, const int64_t* wave_ptr, uint32_t* slot,
                                        float* val_out, uint32_t* hdr, int32_t* err,
                                        gnnrec_stream_t stream) {
  GNNREC_REQUIRE(row_ptr && err && n_rows >= 0, "tiled_plan_device: bad args");
  GNNREC_REQUIRE(rows_per_block >= 1 && rows_per_block <= GNNREC_TILED_MAX_ROWS,
                 "tiled_plan_device: rows_per_block must be in [1, %d]", GNNREC_TILED_MAX_ROWS);
  GNNREC_REQUIRE(panel >= 1 && sub_panel >= 0, "tiled_plan_device: bad panel / sub_panel");
  GNNREC_REQUIRE(max_block_nnz >= 0 && max_block_nnz < INT32_MAX,
                 "tiled_plan_device: a block's edges must fit 31 bits (max_block_nnz)");
  GNNREC_REQUIRE(workgroups >= 1 && scratch, "tiled_plan_device: scratch / workgroups");
  const bool emit = wave_ptr != nullptr;
  GNNREC_REQUIRE(emit ? (slot && val_out && hdr) : (chunks && n_steps),
                 "tiled_plan_device: count pass needs chunks + n_steps, emit pass wave_ptr + "
                 "slot / val / hdr");
  const int64_t nb = (n_rows + rows_per_block - 1) / rows_per_block;
  PlanArgs a{row_ptr, col, val, n_rows, rows_per_block, std::min(panel, kPMaxPanel), sub_panel,
             nb, scratch, max_block_nnz, chunks, n_steps, wave_ptr, slot, val_out, hdr, err};
  hipStream_t s = as_hip(stream);
  if (nb > 0) {
    GNNREC_REQUIRE(col && val, "tiled_plan_device: null col / val");
    const int grid = (int)std::min<int64_t>(nb, workgroups);
    hipLaunchKernelGGL(tiled_plan_kernel, dim3(grid), dim3(64), 0, s, a, emit ? 1 : 0);
    if (int rc = check_launch("tiled_plan_device")) return rc;
  }
  if (emit) {
    hipLaunchKernelGGL(tiled_plan_tail_kernel, dim3(1), dim3(256), 0, s,
                       wave_ptr + nb * GNNREC_TILED_WAVES, slot, val_out, hdr);
    return check_launch("tiled_plan_device (tail)");
  }
  return GNNREC_OK;
}
