// SpMM hop fused with a dense d x d transform on the matrix cores (gfx950 MFMA, f32 in /
// f32 accumulate: v_mfma_f32_16x16x4_f32, an exact fmaf chain).
//
//   MODE 0, NGCF (baselines/ngcf.py:69-84, eval mode):
//       n = A x;  out = LeakyReLU((n @ W1^T + b1) + ((x_self*n) @ W2^T + b2))  [then GAS]
//   MODE 1, OrthogonalBundle (orthogonal_bundle/model.py:171-195 + :204-207):
//       out = c_out * ((A x) @ M) + c_res * resid;   acc (+)= w * out   (layer sum)
//
// These are true small-GEMM contractions (K = 2d or d, N = d per row), so they go to MFMA,
// unlike GAS's 8x8 blocks (VALU, gather.h). A workgroup (4 waves) owns a tile of TR rows:
//   phase 1  the rows are gathered (gather.h, bit-exact order) into an LDS A-tile [TR][K],
//   phase 2  each wave multiplies it by its 16-column slab of W, kept in VGPRs for the
//            whole persistent loop (B fragments: K/4 floats per lane per slab),
//   phase 3  the row-owning lanes apply bias/activation/GAS/residual/layer-sum from an LDS
//            output tile and store whole rows (float4, coalesced).
// MFMA 16x16x4 f32 lane maps (cdna_hip_programming.md §3): A[i=l&15][k=l>>4],
// B[k=l>>4][j=l&15], C/D: col = l&15, row = 4*(l>>4) + reg.
#include <algorithm>
#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "gather.h"

namespace gnnrec {

typedef float floatx4 __attribute__((ext_vector_type(4)));

struct DenseParams {
  Csr A;
  const float* x;
  int64_t ldx;
  const float* x_self;  // MODE 0: input rows of the destinations
  int64_t ld_self;
  float* y;
  int64_t ldy;
  // MODE 0
  const float* W1;
  const float* b1;
  const float* W2;
  const float* b2;
  float slope;
  const float* gas_blocks;
  const int32_t* gas_perm;
  int gas_bs;
  // MODE 1
  const float* M;
  float c_out, c_res;
  const float* resid;
  int64_t ld_resid;
  float* acc;
  int64_t ld_acc;
  int acc_mode;
  float w_out, w_res;
};

// MFMA contraction order of the dense transforms: step s of a chain (s < K/4) contracts
// k = 16 (s / 4) + 4 g + (s % 4) in lane group g = lane >> 4. With that order a lane's A
// operands for steps 4t .. 4t+3 are the row's columns 16t + 4g .. +3 — ONE float4 — so the
// streaming transform feeds the matrix cores from registers (the rows_gemm form), and its B
// fragments for those four steps are one ds_read_b128. spmm_mfma_kernel (the fused form)
// contracts in the same order, so the split and the fused layers keep equal bits.
__device__ __forceinline__ constexpr int mfma_k(int s, int g) { return 16 * (s >> 2) + 4 * g + (s & 3); }

// GATHER = true: the A rows are gathered here (fused hop). GATHER = false: p.x already holds
// the hop output n = A x (rows read straight, float4 per lane) and only the transform runs.
template <int D, int MODE, int NW, bool GATHER>
__global__ __launch_bounds__(64 * NW) void spmm_mfma_kernel(DenseParams p) {
  constexpr int NTH = 64 * NW;
  // gather mapping of the plain hop (SpmmCfg, gather.h): VEC features per lane
  constexpr int VEC = GATHER ? SpmmCfg<D>::VEC : 4, CH = SpmmCfg<D>::CH;
  constexpr int GROUP = D / VEC;
  constexpr int RPW = 64 / GROUP;
  constexpr int PASS_ROWS = RPW * NW;
  constexpr int TR = PASS_ROWS > 4 * NW ? PASS_ROWS : 4 * NW;  // rows per tile (16 per 4 waves)
  constexpr int PASSES = TR / PASS_ROWS;
  constexpr int KD = MODE == 0 ? 2 * D : D;  // contraction length
  constexpr int LDA = KD + 2;                // == 2 mod 32: conflict-free A-fragment reads
  constexpr int LDB = D + 16;                // == 16 mod 32: conflict-free B-fragment reads
  constexpr bool B_LDS = KD * LDB * 4 <= 48 * 1024;
  constexpr int MT = TR / 16, NT = D / 16, TILES = MT * NT;
  constexpr int TPW = (TILES + NW - 1) / NW;  // MFMA output tiles per wave
  constexpr int STEPS = KD / 4;
  __shared__ __attribute__((aligned(16))) float a_lds[TR * LDA];
  __shared__ __attribute__((aligned(16))) float o_lds[TR][D + 4];
  __shared__ __attribute__((aligned(16))) float b_lds[B_LDS ? KD * LDB : 4];
  __shared__ __attribute__((aligned(16))) float w_gas[MODE == 0 ? D * 32 : 4];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int gl = lane % GROUP;
  const int i16 = lane & 15, k4 = lane >> 4;

  // B = [W1^T ; W2^T] (MODE 0) or M (MODE 1), K-major: B[k][j]
  auto bval = [&](int k, int j) -> float {
    if (MODE == 0) return k < D ? p.W1[j * D + k] : p.W2[j * D + (k - D)];
    return p.M[k * D + j];
  };
  float bf[B_LDS ? 1 : TPW][B_LDS ? 1 : STEPS];
  if constexpr (B_LDS) {
    for (int e = threadIdx.x; e < KD * D; e += NTH) b_lds[(e / D) * LDB + e % D] = bval(e / D, e % D);
  } else {
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int t = wave + NW * i;
      const int j = 16 * ((t < TILES ? t : 0) % NT) + i16;
#pragma unroll
      for (int s = 0; s < STEPS; ++s) bf[i][s] = bval(mfma_k(s, k4), j);
    }
  }
  float bias1[TPW], bias2[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = wave + NW * i;
    const int j = 16 * ((t < TILES ? t : 0) % NT) + i16;
    bias1[i] = MODE == 0 ? p.b1[j] : 0.f;
    bias2[i] = MODE == 0 ? p.b2[j] : 0.f;
  }
  const bool gas = MODE == 0 && p.gas_blocks != nullptr;
  int pj[VEC];
#pragma unroll
  for (int q = 0; q < VEC; ++q) pj[q] = 0;
  // GAS on the matrix cores when each wave owns one output tile (d <= 64): out = o @ G with
  // G[k][j] = blockdiag(blocks)[k][perm[j]], the B fragments (D/4 per lane) in VGPRs. The
  // MFMA chain runs over all k in order; the off-block terms are fmaf(o, +0, acc) == acc, so
  // the bits equal gas_row_v's 8-term chain (o is a finite LeakyReLU output).
  constexpr bool GAS_MFMA = MODE == 0 && TPW == 1 && TILES == NW && D <= 64;
  float gf[GAS_MFMA ? D / 4 : 1];
  if (gas) {
    for (int i = threadIdx.x; i < D * p.gas_bs; i += NTH) w_gas[i] = p.gas_blocks[i];
#pragma unroll
    for (int q = 0; q < VEC; ++q) pj[q] = p.gas_perm[VEC * gl + q];
    if constexpr (GAS_MFMA) {
      const int bs = p.gas_bs;
      const int c = p.gas_perm[16 * (wave % NT) + i16];   // output column j -> z column c
      const int b = c / bs, e = c - b * bs;
#pragma unroll
      for (int st = 0; st < D / 4; ++st) {
        const int k = 4 * st + k4;
        gf[st] = (k / bs == b) ? p.gas_blocks[(int64_t)(b * bs + (k - b * bs)) * bs + e] : 0.f;
      }
    }
  }
  __syncthreads();

  const int64_t n_tiles = ceil_div(p.A.n_rows, TR);
  // GATHER = false streams rows: the next tile's rows are loaded into registers while this
  // tile multiplies and stores (one tile in flight per workgroup doubles the bytes in flight)
  VecF<VEC> pre_n[GATHER ? 1 : PASSES], pre_x[GATHER ? 1 : PASSES];
  auto load_rows = [&](int64_t tile, VecF<VEC>* n, VecF<VEC>* xs) {
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
      const int64_t r = tile * TR + ps * PASS_ROWS + wave * RPW + lane / GROUP;
#pragma unroll
      for (int q = 0; q < VEC; ++q) n[ps].v[q] = xs[ps].v[q] = 0.f;
      if (tile < n_tiles && r < p.A.n_rows) {
        n[ps] = ldv<VEC>(p.x + r * p.ldx + VEC * gl);
        if (MODE == 0) xs[ps] = ldv<VEC>(p.x_self + r * p.ld_self + VEC * gl);
      }
    }
  };
  if constexpr (!GATHER) load_rows(blockIdx.x, pre_n, pre_x);
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t row0 = tile * TR;
    // ---- phase 1: gather rows into the A tile
    VecF<VEC> cur_n[GATHER ? 1 : PASSES], cur_x[GATHER ? 1 : PASSES];
    if constexpr (!GATHER) {
#pragma unroll
      for (int ps = 0; ps < PASSES; ++ps) {
        cur_n[ps] = pre_n[ps];
        cur_x[ps] = pre_x[ps];
      }
      load_rows(tile + gridDim.x, pre_n, pre_x);
    }
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
      const int slot = ps * PASS_ROWS + wave * RPW + lane / GROUP;
      const int64_t r = row0 + slot;
      VecF<VEC> n, xs;
#pragma unroll
      for (int q = 0; q < VEC; ++q) n.v[q] = xs.v[q] = 0.f;
      if constexpr (GATHER) {
        if (r < p.A.n_rows) {
          n = gather_row_v<VEC, GROUP, CH>(p.A.col, p.A.val, p.A.row_ptr[r], p.A.row_ptr[r + 1],
                                           p.x, p.ldx, gl);
          if (MODE == 0) xs = ldv<VEC>(p.x_self + r * p.ld_self + VEC * gl);
        }
      } else {
        n = cur_n[ps];
        xs = cur_x[ps];
      }
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        a_lds[slot * LDA + VEC * gl + q] = n.v[q];
        if (MODE == 0) a_lds[slot * LDA + D + VEC * gl + q] = xs.v[q] * n.v[q];
      }
    }
    __syncthreads();
    // ---- phase 2: MFMA
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int t = wave + NW * i;
      if (t < TILES) {
        const int mt = t / NT, nt = t % NT;
        floatx4 c1 = {0.f, 0.f, 0.f, 0.f}, c2 = {0.f, 0.f, 0.f, 0.f};
        const float* arow = &a_lds[(16 * mt + i16) * LDA];
        const float* bcol = &b_lds[16 * nt + i16];
#pragma unroll
        for (int s = 0; s < STEPS; ++s) {
          const float a = arow[mfma_k(s, k4)];   // the streaming transform's k order
          float b;
          if constexpr (B_LDS) b = bcol[mfma_k(s, k4) * LDB]; else b = bf[i][s];
          if (MODE == 0 && s >= STEPS / 2)
            c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
          else
            c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
        }
        const int j = 16 * nt + i16;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v;
          if (MODE == 0) {
            v = (c1[q] + bias1[i]) + (c2[q] + bias2[i]);
            v = v > 0.f ? v : v * p.slope;
          } else {
            v = c1[q];
          }
          o_lds[16 * mt + 4 * k4 + q][j] = v;
        }
      }
    }
    __syncthreads();
    if constexpr (GAS_MFMA) {
      if (gas) {  // phase 2b: o_tile @ G on MFMA, written back over o_tile
        const int mt = wave / NT, nt = wave % NT;
        floatx4 c = {0.f, 0.f, 0.f, 0.f};
        const float* arow = &o_lds[16 * mt + i16][k4];
#pragma unroll
        for (int st = 0; st < D / 4; ++st)
          c = __builtin_amdgcn_mfma_f32_16x16x4f32(arow[4 * st], gf[st], c, 0, 0, 0);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) o_lds[16 * mt + 4 * k4 + q][16 * nt + i16] = c[q];
        __syncthreads();
      }
    }
    // ---- phase 3: row epilogue + coalesced store
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
      const int slot = ps * PASS_ROWS + wave * RPW + lane / GROUP;
      const int64_t r = row0 + slot;
      if (r >= p.A.n_rows) continue;
      VecF<VEC> o;
      if (MODE == 0) {
        if (gas && !GAS_MFMA) {
          o = gas_row_v<VEC>(&o_lds[slot][0], w_gas, p.gas_bs, pj);
        } else {
#pragma unroll
          for (int q = 0; q < VEC; ++q) o.v[q] = o_lds[slot][VEC * gl + q];
        }
      } else {
        VecF<VEC> rs;
        if (p.resid) rs = ldv<VEC>(p.resid + r * p.ld_resid + VEC * gl);
#pragma unroll
        for (int q = 0; q < VEC; ++q) {
          const float t = o_lds[slot][VEC * gl + q];
          o.v[q] = p.resid ? p.c_out * t + p.c_res * rs.v[q] : p.c_out * t;
        }
        if (p.acc_mode) {
          float* ar = p.acc + r * p.ld_acc + VEC * gl;
          VecF<VEC> base;
          if (p.acc_mode == 1) {
#pragma unroll
            for (int q = 0; q < VEC; ++q) base.v[q] = p.w_res * rs.v[q];
          } else {
            base = ldv<VEC>(ar);
          }
#pragma unroll
          for (int q = 0; q < VEC; ++q) base.v[q] = base.v[q] + p.w_out * o.v[q];
          stv<VEC>(ar, base);
        }
      }
      if (p.y) stv<VEC>(p.y + r * p.ldy + VEC * gl, o);
    }
  }
}

// Streaming transform for d = 64 (the split form's second kernel; n = A x is already in HBM):
// every wave owns 16-row tiles on its own — no workgroup barrier inside the loop. Lane
// (i16, g) holds row i16's columns 16t + 4g .. +3 (t < 4) of n and x in registers, forms
// x (.) n there, and runs the 16x16x4 f32 MFMA chains of all four 16-column output tiles
// (c1: n @ W1^T, c2: (x (.) n) @ W2^T — the reference's two Linear layers, kept apart for
// (c1 + b1) + (c2 + b2)) with B read from LDS as one float4 per 4 steps; bias, LeakyReLU and
// the GAS product (VALU for 8x8 blocks, else on the matrix cores) run from a private o tile,
// and whole rows are stored (float4). The next tile's rows are in flight in registers.
// Diagnostic builds only (results wrong, timing only): bit 0 skips the MFMAs (accumulators stay
// 0), bit 1 skips the GAS product (the o tile is stored as is), bit 2 replaces the row loads by
// register constants (no HBM reads).
#ifndef GNNREC_TRANSFORM_EXP
#define GNNREC_TRANSFORM_EXP 0
#endif
// the next tile's rows in flight in registers during this tile's MFMAs (1), or loaded at the
// tile start (0: 32 fewer VGPRs, e.g. for 16 waves per workgroup)
#ifndef GNNREC_TRANSFORM_PREFETCH
#define GNNREC_TRANSFORM_PREFETCH 1
#endif
constexpr bool kTransformPrefetch = GNNREC_TRANSFORM_PREFETCH != 0;
#ifndef GNNREC_TRANSFORM_GAS_DPP
#define GNNREC_TRANSFORM_GAS_DPP 0
#endif
// Lanes 0-7 of each 16-lane DPP row take row lane T, lanes 8-15 row lane 8 + T (two DPP
// row_newbcast moves under bank masks): one 8-column GAS block's value c to its 8 lanes.
template <int T>
__device__ __forceinline__ float half_bcast(float v) {
  const int a = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x150 + T, 0xF, 0x3, false);
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(a, __builtin_bit_cast(int, v), 0x158 + T, 0xF, 0xC, false));
}
// z = sum_c o[c] W[c][e] of one 8x8 GAS block in the MFMA output layout (lane i16 = 8 h + e
// holds column 8 b + e of the block's row): fmaf over c ascending from +0, oracle_gas's order
template <int... C>
__device__ __forceinline__ float gas_dpp8(std::integer_sequence<int, C...>, float v,
                                          const float (&w)[8]) {
  float z = 0.f;
  ((z = __builtin_fmaf(half_bcast<C>(v), w[C], z)), ...);
  return z;
}

template <int MODE, int NW, bool GASV>
__global__ __launch_bounds__(64 * NW) void transform64_kernel(DenseParams p) {
  constexpr int D = 64;
  constexpr int NP = MODE == 0 ? 2 : 1;   // contraction parts: n (W1) [, x (.) n (W2)]
  constexpr int LDO = D + 4;
  constexpr int LDB = D + 16;             // dense GAS matrix (non-8x8 blocks), as before
  // B fragments: [part][t][nt][lane][q] = B_part[k = 16t + 4(lane>>4) + q][j = 16nt + (lane&15)]
  __shared__ __attribute__((aligned(16))) float b_lds[NP * 4 * 4 * 64 * 4];
  __shared__ __attribute__((aligned(16))) float g_lds[MODE == 0 && !GASV ? D * LDB : 4];
  __shared__ __attribute__((aligned(16))) float t_lds[NW][16 * LDO];
  constexpr int kVbs = 8;
  __shared__ __attribute__((aligned(16))) float wv_lds[MODE == 0 && GASV ? D * kVbs : 4];
  __shared__ int inv_lds[MODE == 0 && GASV ? D : 1];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i16 = lane & 15, k4 = lane >> 4;
  float* ot = t_lds[wave];
  for (int e = threadIdx.x; e < NP * 4096; e += 64 * NW) {
    const int q = e & 3, l = (e >> 2) & 63, nt = (e >> 8) & 3, t = (e >> 10) & 3, part = e >> 12;
    const int k = 16 * t + 4 * (l >> 4) + q, j = 16 * nt + (l & 15);
    float v;
    if (MODE == 0) v = part == 0 ? p.W1[j * D + k] : p.W2[j * D + k];
    else v = p.M[k * D + j];
    b_lds[e] = v;
  }
  const bool gas = MODE == 0 && p.gas_blocks != nullptr;
  // 8x8 blocks: the GAS product runs on the VALU, 8 fmaf per output in the oracle's order
  // (oracle_gas: c ascending from +0), instead of as a dense 64x64 MFMA product that spends 7/8
  // of its work on zeros (profiles/r02/config3_transform_mfma_pmc.json: 24M MFMA per launch,
  // 8M of them GAS). GASV instances are launched for 8x8 blocks only.
  constexpr bool gas_valu = GASV;
  if (gas_valu) {
    for (int e = threadIdx.x; e < D * kVbs; e += 64 * NW) wv_lds[e] = p.gas_blocks[e];
    for (int j = threadIdx.x; j < D; j += 64 * NW) inv_lds[p.gas_perm[j]] = j;
  } else if (gas && !GASV) {   // G[k][j] = blockdiag(blocks)[k][perm[j]]
    const int bs = p.gas_bs;
    for (int e = threadIdx.x; e < D * D; e += 64 * NW) {
      const int k = e / D, j = e % D;
      const int c = p.gas_perm[j];
      const int b = c / bs, col = c - b * bs;
      g_lds[k * LDB + j] =
          (k / bs == b) ? p.gas_blocks[(int64_t)(b * bs + (k - b * bs)) * bs + col] : 0.f;
    }
  }
  float bias1[4], bias2[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    bias1[nt] = MODE == 0 ? p.b1[16 * nt + i16] : 0.f;
    bias2[nt] = MODE == 0 ? p.b2[16 * nt + i16] : 0.f;
  }
  // GAS in registers (GNNREC_TRANSFORM_GAS_DPP): lane i16 = 8 h + e of output tile nt holds
  // column 8 (2 nt + h) + e, so it needs W_{2nt+h}[c][e] for c < 8 (32 weights, constant)
  // and the output column of its block column, inv[16 nt + i16]
  constexpr bool gas_dpp = MODE == 0 && GASV && GNNREC_TRANSFORM_GAS_DPP;
  float wg[gas_dpp ? 4 : 1][8];
  int invc[4];
  if (gas_dpp) {
    const int h = i16 >> 3, e = i16 & 7;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int c = 0; c < 8; ++c) wg[nt][c] = p.gas_blocks[((2 * nt + h) * kVbs + c) * kVbs + e];
  }
  __syncthreads();
  if (gas_dpp) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) invc[nt] = inv_lds[16 * nt + i16];
  }

  const int64_t n_tiles = ceil_div(p.A.n_rows, 16);
  const int64_t stride = (int64_t)gridDim.x * NW;
  // A operands: lane (i16, k4) loads row i16's float4 at columns 16t + 4 k4 (t < 4)
  float4 pn[4], px[4];
  // MODE 0: rows past the end (the last tile's tail, the prefetch past the last tile) load the
  // last row instead — no row is ever stored from them — and the unconditional loads keep the
  // prefetch in flight: behind a branch the compiler waited for them right after issuing them
  // (config 3's transform 364 -> 356 us, profiles/r05/c15_*). MODE 1 keeps the branch (the
  // unconditional form ran 5 % slower there).
  auto load = [&](int64_t tile) {
    if constexpr (MODE == 0) {
      const int64_t r = std::min<int64_t>(tile * 16 + i16, p.A.n_rows - 1);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (GNNREC_TRANSFORM_EXP & 4) {
          pn[t] = make_float4((float)r, 1.f, 2.f, (float)t);
          px[t] = pn[t];
        } else {
          pn[t] = *reinterpret_cast<const float4*>(p.x + r * p.ldx + 16 * t + 4 * k4);
          px[t] = *reinterpret_cast<const float4*>(p.x_self + r * p.ld_self + 16 * t + 4 * k4);
        }
      }
    } else {
      const int64_t r = tile * 16 + i16;
      const bool ok = tile < n_tiles && r < p.A.n_rows;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        pn[t] = px[t] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (GNNREC_TRANSFORM_EXP & 4) {
          pn[t] = make_float4((float)r, 1.f, 2.f, (float)t);
          px[t] = pn[t];
        } else if (ok) {
          pn[t] = *reinterpret_cast<const float4*>(p.x + r * p.ldx + 16 * t + 4 * k4);
        }
      }
    }
  };
  // output rows: lane covers rows 4 it + (lane >> 4), columns 4 (lane & 15) .. +3, it = 0..3
  const int lr = lane >> 4, lc = 4 * (lane & 15);
  int64_t tile = (int64_t)blockIdx.x * NW + wave;
  if (kTransformPrefetch) load(tile);
  for (; tile < n_tiles; tile += stride) {
    if (!kTransformPrefetch) load(tile);
    float an[4][4], ax[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      an[t][0] = pn[t].x; an[t][1] = pn[t].y; an[t][2] = pn[t].z; an[t][3] = pn[t].w;
      if (MODE == 0) {
        ax[t][0] = px[t].x * pn[t].x; ax[t][1] = px[t].y * pn[t].y;
        ax[t][2] = px[t].z * pn[t].z; ax[t][3] = px[t].w * pn[t].w;
      }
    }
    float4 rs[4];   // MODE 1 residual rows (loaded with the tile, used at the store)
    if (MODE == 1 && p.resid) {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int64_t r = tile * 16 + 4 * it + lr;
        rs[it] = r < p.A.n_rows ? *reinterpret_cast<const float4*>(p.resid + r * p.ld_resid + lc)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    if (kTransformPrefetch) load(tile + stride);
    floatx4 c1[4], c2[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) c1[nt] = c2[nt] = floatx4{0.f, 0.f, 0.f, 0.f};
    // B in half-groups h = (t, part): the 4 float4 (one per nt) of 4 MFMA steps of one
    // contraction part, double-buffered so half-group h + 1's LDS reads fly under h's 16
    // MFMAs; inside h the MFMAs cycle over the 4 output tiles (independent accumulators, no
    // dependent back-to-back issue); every chain keeps its (t, q) order
    const float4* bl = reinterpret_cast<const float4*>(b_lds) + lane;
    constexpr int NH = 4 * NP;   // half-groups: h = t * NP + part
    float4 bc[4], bn[4];
    auto load_b = [&](int h, float4 (&bb)[4]) {
      const int t = h / NP, part = h % NP;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) bb[nt] = bl[((part * 4 + t) * 4 + nt) * 64];
    };
    load_b(0, bc);
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int t = h / NP, part = h % NP;
      if (h + 1 < NH) load_b(h + 1, bn);
      __builtin_amdgcn_sched_barrier(0);   // the next half-group's reads issue first
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float a = part == 0 ? an[t][q] : ax[t][q];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const float bq = q == 0 ? bc[nt].x : q == 1 ? bc[nt].y : q == 2 ? bc[nt].z : bc[nt].w;
          if (GNNREC_TRANSFORM_EXP & 1)
            c1[nt][q] += a * bq;   // keeps the operands live without the matrix cores
          else if (part == 0)
            c1[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bq, c1[nt], 0, 0, 0);
          else
            c2[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bq, c2[nt], 0, 0, 0);
        }
      }
      if (h + 1 < NH) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) bc[nt] = bn[nt];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // o tile (rows 4 k4 + q, column 16 nt + i16); with gas_dpp the GAS outputs go straight
    // to their permuted columns
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v;
        if (MODE == 0) {
          v = (c1[nt][q] + bias1[nt]) + (c2[nt][q] + bias2[nt]);
          v = v > 0.f ? v : v * p.slope;
        } else {
          v = c1[nt][q];
        }
        if (gas_dpp)
          ot[(4 * k4 + q) * LDO + invc[nt]] = gas_dpp8(std::make_integer_sequence<int, 8>{}, v, wg[nt]);
        else
          ot[(4 * k4 + q) * LDO + 16 * nt + i16] = v;
      }
    if (gas_valu && !gas_dpp && !(GNNREC_TRANSFORM_EXP & 2)) {
      // lane (i16, k4): z = GAS of row i16's columns 16 k4 .. 16 k4 + 15 (two 8-blocks), then
      // z[t] to column inv[16 k4 + t] of the same row; the wave's LDS operations run in order,
      // so every lane's reads of the row precede the scattered writes
      float ov[16], z[16];
      const float* orow = ot + i16 * LDO + 16 * k4;
#pragma unroll
      for (int t4 = 0; t4 < 4; ++t4) {
        const float4 v = *reinterpret_cast<const float4*>(orow + 4 * t4);
        ov[4 * t4] = v.x; ov[4 * t4 + 1] = v.y; ov[4 * t4 + 2] = v.z; ov[4 * t4 + 3] = v.w;
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float* W = wv_lds + (16 * k4 + kVbs * h) * kVbs;   // block 2 k4 + h
#pragma unroll
        for (int e = 0; e < kVbs; ++e) z[kVbs * h + e] = 0.f;
#pragma unroll
        for (int c = 0; c < kVbs; ++c) {
          const float4 w0 = *reinterpret_cast<const float4*>(W + c * kVbs);
          const float4 w1 = *reinterpret_cast<const float4*>(W + c * kVbs + 4);
          const float wc[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
          const float x = ov[kVbs * h + c];
#pragma unroll
          for (int e = 0; e < kVbs; ++e) z[kVbs * h + e] = __builtin_fmaf(x, wc[e], z[kVbs * h + e]);
        }
      }
      float* wrow = ot + i16 * LDO;
#pragma unroll
      for (int t = 0; t < 16; ++t) wrow[inv_lds[16 * k4 + t]] = z[t];
    } else if (gas && !GASV) {   // out = o @ G on the matrix cores, k ascending (== gas_row_v's chain)
      floatx4 cg[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) cg[nt] = floatx4{0.f, 0.f, 0.f, 0.f};
      const float* orow = ot + i16 * LDO + k4;
#pragma unroll
      for (int st = 0; st < D / 4; ++st) {
        const float a = orow[4 * st];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          cg[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(
              a, g_lds[(4 * st + k4) * LDB + 16 * nt + i16], cg[nt], 0, 0, 0);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int q = 0; q < 4; ++q) ot[(4 * k4 + q) * LDO + 16 * nt + i16] = cg[nt][q];
    }
    // whole rows out
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int row = 4 * it + lr;
      const int64_t r = tile * 16 + row;
      if (r >= p.A.n_rows) continue;
      const float* orow = ot + row * LDO + lc;
      float o[4] = {orow[0], orow[1], orow[2], orow[3]};
      if (MODE == 1) {
        const float rv[4] = {rs[it].x, rs[it].y, rs[it].z, rs[it].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = p.resid ? p.c_out * o[q] + p.c_res * rv[q] : p.c_out * o[q];
        if (p.acc_mode) {
          float* ar = p.acc + r * p.ld_acc + lc;
          float bse[4];
          if (p.acc_mode == 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) bse[q] = p.w_res * rv[q];
          } else {
            const float4 t = *reinterpret_cast<const float4*>(ar);
            bse[0] = t.x; bse[1] = t.y; bse[2] = t.z; bse[3] = t.w;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) bse[q] = bse[q] + p.w_out * o[q];
          *reinterpret_cast<float4*>(ar) = make_float4(bse[0], bse[1], bse[2], bse[3]);
        }
      }
      if (p.y) *reinterpret_cast<float4*>(p.y + r * p.ldy + lc) = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
}

// Streaming row GEMM y[r, :P] = x[r, :K] @ B[K, P] for tall-skinny operands (GAT's fused
// projection [N, 64] x [64, H*o + 2H] and head-mean [N, H*in] x [H*in, o]; hipBLASLt ran these
// at 1-3 TB/s). Every wave owns 16-row tiles on its own (no barrier in the loop) and feeds the
// A operand of v_mfma_f32_16x16x4f32 straight from registers: lane (i, g) = (lane & 15,
// lane >> 4) loads row i's float4 at columns 16 t + 4 g (t < K/16: the 4 lanes of a row read
// 64 contiguous bytes per instruction), and MFMA step 4 t + q contracts k = 16 t + 4 g + q
// (a permutation of the k order; GAT is an fp32-tolerance path). B sits in LDS for the launch:
// for K >= 128 (MFMA-bound) as MFMA fragments — [t][nt][lane][q] = B[16 t + 4 g + q][16 nt + i],
// a lane's B operands of 4 steps in one ds_read_b128, double-buffered per t (K = 256: 1.79 ->
// 1.70 ms per 5M rows, same bits, profiles/r05/c13_rows_gemm.jsonl); for K = 64 (HBM-bound) as
// rows [K][PN + 4] read per MFMA, which keeps the instances within 128 VGPRs (the fragment form
// took P = 72 from 0.72 to 0.84 ms). NT 16-column output tiles, the o tile goes through a small
// private LDS tile so whole rows are stored, and the next tile's rows are in flight in
// registers meanwhile.
struct RowsGemmEpi {   // optional epilogue of gnnrec_rows_gemm_f32 (GAT's last layer)
  int apply_elu;
  int epi;             // GNNREC_EPI_ACC_* flags, as gnnrec_gat_aggregate_f32
  const float* self;
  int64_t ld_self;
  float* acc;
  int64_t ld_acc;
  float acc_div;
};

template <int K, int NT, int NW>
__global__ __launch_bounds__(64 * NW) void rows_gemm_kernel(int64_t n_rows, const float* __restrict__ x,
                                                            int64_t ldx, const float* __restrict__ B,
                                                            int P, float* __restrict__ y, int64_t ldy,
                                                            RowsGemmEpi ep) {
  constexpr int PN = NT * 16;
  constexpr int LDB = PN + 4;
  constexpr int LDO = PN + 4;
  constexpr int T = K / 16;            // float4 per lane per tile
  constexpr bool kFrag = K >= 128;     // B as fragments [T][NT][64][4] (else rows [K][LDB])
  static_assert(K % 16 == 0 && NT >= 1, "rows_gemm: K % 16 == 0");
  // dynamic LDS (rows_gemm_lds): B, then NW o tiles [16][LDO]
  extern __shared__ __attribute__((aligned(16))) float rg_lds[];
  float* b_lds = rg_lds;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i16 = lane & 15, g = lane >> 4;
  for (int e = threadIdx.x; e < K * PN; e += 64 * NW) {
    if constexpr (kFrag) {
      const int q = e & 3, l = (e >> 2) & 63, tn = e >> 8;
      const int k = 16 * (tn / NT) + 4 * (l >> 4) + q, j = 16 * (tn % NT) + (l & 15);
      b_lds[e] = j < P ? B[(int64_t)k * P + j] : 0.f;
    } else {
      const int k = e / PN, j = e % PN;
      b_lds[k * LDB + j] = j < P ? B[(int64_t)k * P + j] : 0.f;
    }
  }
  __syncthreads();
  float* ot = rg_lds + K * (kFrag ? PN : LDB) + wave * 16 * LDO;
  const int64_t n_tiles = ceil_div(n_rows, 16);
  const int64_t stride = (int64_t)gridDim.x * NW;
  float4 pa[T], pn[T];
  // K >= 128: rows past the end load the last row (never stored), and the unconditional loads
  // keep the prefetch in flight (as transform64_kernel's; behind a branch the compiler waited for
  // them right after issuing them). K = 64 keeps the branch: unconditional, its NT = 2 / 4
  // instances compile to partially overlapping MFMA accumulators (tests/test_native_host.py).
  auto load = [&](int64_t tile, float4 (&v)[T]) {
    if constexpr (kFrag) {
      const float* xr = x + std::min<int64_t>(tile * 16 + i16, n_rows - 1) * ldx + 4 * g;
#pragma unroll
      for (int t = 0; t < T; ++t) v[t] = *reinterpret_cast<const float4*>(xr + 16 * t);
    } else {
      const int64_t r = tile * 16 + i16;
      const bool ok = tile < n_tiles && r < n_rows;
      const float* xr = x + (ok ? r : 0) * ldx + 4 * g;
#pragma unroll
      for (int t = 0; t < T; ++t)
        v[t] = ok ? *reinterpret_cast<const float4*>(xr + 16 * t) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  int64_t tile = (int64_t)blockIdx.x * NW + wave;
  load(tile, pa);
  const int P4 = P / 4;
  const float4* bl = reinterpret_cast<const float4*>(b_lds) + lane;
  const float* brow = b_lds + (4 * g) * LDB + i16;
  for (; tile < n_tiles; tile += stride) {
    load(tile + stride, pn);
    floatx4 c[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) c[nt] = floatx4{0.f, 0.f, 0.f, 0.f};
    // fully unrolled (a rolled k loop made the compiler rotate the accumulators through
    // partially overlapping AGPR ranges, v_mfma a[10:13], ..., a[12:15]: wrong on gfx950)
    if constexpr (kFrag) {
      // the B fragments of step group t + 1 are read while group t's MFMAs run
      float4 bc[NT], bn[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bc[nt] = bl[nt * 64];
#pragma unroll
      for (int t = 0; t < T; ++t) {
        if (t + 1 < T) {
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) bn[nt] = bl[((t + 1) * NT + nt) * 64];
        }
        __builtin_amdgcn_sched_barrier(0);
        const float av[4] = {pa[t].x, pa[t].y, pa[t].z, pa[t].w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) {
            const float bq = q == 0 ? bc[nt].x : q == 1 ? bc[nt].y : q == 2 ? bc[nt].z : bc[nt].w;
            c[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q], bq, c[nt], 0, 0, 0);
          }
        if (t + 1 < T) {
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) bc[nt] = bn[nt];
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const float av[4] = {pa[t].x, pa[t].y, pa[t].z, pa[t].w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            c[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                av[q], brow[(16 * t + q) * LDB + 16 * nt], c[nt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int q = 0; q < 4; ++q) ot[(4 * g + q) * LDO + 16 * nt + i16] = c[nt][q];
    // whole rows out; the accumulator rows (ACC epilogue) are all loaded before the first use
    constexpr int MAXIT = (16 * PN / 4 + 63) / 64;
    const bool has_acc = (ep.epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)) != 0;
    const bool init = (ep.epi & GNNREC_EPI_ACC_INIT) != 0;
    float4 bse[MAXIT];
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      const int e = lane + 64 * it;
      const int row = e / P4, c4 = e - row * P4;
      const int64_t r = tile * 16 + row;
      bse[it] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (has_acc && e < 16 * P4 && r < n_rows)
        bse[it] = init ? ld4(ep.self + r * ep.ld_self + 4 * c4) : ld4(ep.acc + r * ep.ld_acc + 4 * c4);
    }
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      const int e = lane + 64 * it;
      const int row = e / P4, c4 = e - row * P4;
      const int64_t r = tile * 16 + row;
      if (e < 16 * P4 && r < n_rows) {
        const float* o = ot + row * LDO + 4 * c4;
        float4 v = make_float4(o[0], o[1], o[2], o[3]);
        if (ep.apply_elu) {   // F.elu (gat.py:283), as gat_finish
          v.x = v.x > 0.f ? v.x : expm1f(v.x);
          v.y = v.y > 0.f ? v.y : expm1f(v.y);
          v.z = v.z > 0.f ? v.z : expm1f(v.z);
          v.w = v.w > 0.f ? v.w : expm1f(v.w);
        }
        if (y) *reinterpret_cast<float4*>(y + r * ldy + 4 * c4) = v;
        if (has_acc) {   // acc_epilogue's order: (base + y) [/ div]
          float4 b = bse[it];
          b.x = b.x + v.x; b.y = b.y + v.y; b.z = b.z + v.z; b.w = b.w + v.w;
          if (ep.epi & GNNREC_EPI_ACC_DIV) {
            b.x = b.x / ep.acc_div; b.y = b.y / ep.acc_div;
            b.z = b.z / ep.acc_div; b.w = b.w / ep.acc_div;
          }
          st4(ep.acc + r * ep.ld_acc + 4 * c4, b);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < T; ++t) pa[t] = pn[t];
  }
}

}  // namespace gnnrec

using namespace gnnrec;

namespace {

// Two forms (measured on G100M, tools/bench_configs.py config 3):
//  * split (default when the caller passes a workspace): the plain hop kernel writes
//    n = A x at full gather efficiency, then this kernel streams n (and x) rows through the
//    MFMA transform: ~1 GB more HBM traffic per layer but the gather keeps the hop's
//    occupancy;
//  * fused (no workspace): gather + MFMA in one kernel.
// Waves per workgroup: 8 for d <= 64 (weights in LDS), 4 for d = 128 (weights in VGPRs).
#ifndef GNNREC_TRANSFORM_GASV_WAVES
#define GNNREC_TRANSFORM_GASV_WAVES 12
#endif
template <int MODE, bool GATHER>
int launch_dense(const DenseParams& p, int d, hipStream_t s) {
  if (!GATHER && d == 64) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    auto go64 = [&](auto kern, int nw) {
      const int64_t tiles = ceil_div(p.A.n_rows, 16 * nw);
      const unsigned grid = (unsigned)std::min<int64_t>(tiles, (int64_t)cus);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * nw), 0, s, p);
    };
    if (MODE == 0 && p.gas_blocks && p.gas_bs == 8)
      go64(transform64_kernel<MODE, GNNREC_TRANSFORM_GASV_WAVES, true>,
           GNNREC_TRANSFORM_GASV_WAVES);
    else
      go64(transform64_kernel<MODE, 8, false>, 8);
    return check_launch(MODE == 0 ? "ngcf_transform" : "dense_transform");
  }
  auto go = [&](auto kern, int nw) {
    const int64_t tiles = ceil_div(p.A.n_rows, 4 * nw);
    const unsigned grid = (unsigned)(tiles < 2048 ? tiles : 2048);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * nw), 0, s, p);
  };
  switch (d) {
    case 32: go(spmm_mfma_kernel<32, MODE, 8, GATHER>, 8); break;
    case 64: go(spmm_mfma_kernel<64, MODE, 8, GATHER>, 8); break;
    case 128: go(spmm_mfma_kernel<128, MODE, 4, GATHER>, 4); break;
    default: set_error("dense epilogue: d=%d unsupported (32, 64, 128)", d); return GNNREC_EUNSUPPORTED;
  }
  return check_launch(MODE == 0 ? "spmm_ngcf" : "spmm_dense");
}

// Runs the hop into `work` (n_rows x d) and the transform over it, or the fused kernel.
template <int MODE>
int run_dense(DenseParams p, int d, float* work, hipStream_t s) {
  if (!work) return launch_dense<MODE, true>(p, d, s);
  const int rc = gnnrec_spmm_csr_f32(p.A.row_ptr, p.A.col, p.A.val, p.A.n_rows, p.x, p.ldx, work,
                                     d, d, 0, nullptr, d, nullptr, d, 1.f,
                                     reinterpret_cast<gnnrec_stream_t>(s));
  if (rc != GNNREC_OK) return rc;
  p.x = work;
  p.ldx = d;
  return launch_dense<MODE, false>(p, d, s);
}

bool rows_ok(const float* p, int64_t ld) { return p && aligned16(p) && !(ld & 3); }  // float4 rows

}  // namespace

extern "C" int gnnrec_spmm_ngcf_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                                    int64_t n_rows, const float* x, int64_t ldx,
                                    const float* x_self, int64_t ld_self, float* y, int64_t ldy,
                                    int32_t d, const float* W1, const float* b1, const float* W2,
                                    const float* b2, float slope, const float* gas_blocks,
                                    const int32_t* gas_perm, int32_t gas_bs, float* work,
                                    gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_rows >= 0, "spmm_ngcf: n_rows < 0");
  if (n_rows == 0) return GNNREC_OK;
  GNNREC_REQUIRE(row_ptr && col && val && W1 && b1 && W2 && b2, "spmm_ngcf: null operand");
  GNNREC_REQUIRE(ldx >= d && ld_self >= d && ldy >= d, "spmm_ngcf: leading dimension < d");
  GNNREC_REQUIRE(rows_ok(x, ldx) && rows_ok(x_self, ld_self) && rows_ok(y, ldy),
                 "spmm_ngcf: x/x_self/y must be 16-B aligned with ld %% 4 == 0");
  if (gas_blocks) {
    GNNREC_REQUIRE(gas_perm && gas_bs >= 1 && gas_bs <= 32 && d % gas_bs == 0,
                   "spmm_ngcf: bad GAS block size %d", gas_bs);
  }
  DenseParams p{};
  p.A = Csr{row_ptr, col, val, n_rows};
  p.x = x; p.ldx = ldx; p.x_self = x_self; p.ld_self = ld_self; p.y = y; p.ldy = ldy;
  p.W1 = W1; p.b1 = b1; p.W2 = W2; p.b2 = b2; p.slope = slope;
  p.gas_blocks = gas_blocks; p.gas_perm = gas_perm; p.gas_bs = gas_bs;
  GNNREC_REQUIRE(!work || aligned16(work), "spmm_ngcf: work must be 16-B aligned");
  return run_dense<0>(p, d, work, as_hip(stream));
}

extern "C" int gnnrec_spmm_dense_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                                     int64_t n_rows, const float* x, int64_t ldx, float* y,
                                     int64_t ldy, int32_t d, const float* M, float c_out,
                                     const float* resid, int64_t ld_resid, float c_res, float* acc,
                                     int64_t ld_acc, int32_t acc_mode, float w_out, float w_res,
                                     float* work, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_rows >= 0, "spmm_dense: n_rows < 0");
  if (n_rows == 0) return GNNREC_OK;
  GNNREC_REQUIRE(row_ptr && col && val && M, "spmm_dense: null operand");
  GNNREC_REQUIRE(acc_mode >= 0 && acc_mode <= 2, "spmm_dense: acc_mode must be 0, 1 or 2");
  GNNREC_REQUIRE(y || acc_mode, "spmm_dense: nothing to write (y == NULL and acc_mode == 0)");
  GNNREC_REQUIRE(rows_ok(x, ldx) && ldx >= d, "spmm_dense: x must be 16-B aligned, ld %% 4 == 0, ld >= d");
  GNNREC_REQUIRE(resid ? (rows_ok(resid, ld_resid) && ld_resid >= d) : acc_mode != 1,
                 "spmm_dense: resid must be 16-B aligned with ld >= d (required by acc_mode 1)");
  GNNREC_REQUIRE(!y || (rows_ok(y, ldy) && ldy >= d), "spmm_dense: bad y");
  GNNREC_REQUIRE(!acc_mode || (rows_ok(acc, ld_acc) && ld_acc >= d), "spmm_dense: bad acc");
  DenseParams p{};
  p.A = Csr{row_ptr, col, val, n_rows};
  p.x = x; p.ldx = ldx; p.y = y; p.ldy = ldy;
  p.M = M; p.c_out = c_out; p.c_res = c_res; p.resid = resid; p.ld_resid = ld_resid;
  p.acc = acc; p.ld_acc = ld_acc; p.acc_mode = acc_mode; p.w_out = w_out; p.w_res = w_res;
  GNNREC_REQUIRE(!work || aligned16(work), "spmm_dense: work must be 16-B aligned");
  return run_dense<1>(p, d, work, as_hip(stream));
}

// Transform-only forms: the caller already holds n = A x (e.g. from gnnrec_spmm_csr_split_f32,
// whose heavy-row kernel keeps power-law operands fast); the streaming MFMA kernel applies
// the rest exactly as the split form of the two calls above.
extern "C" int gnnrec_ngcf_transform_f32(int64_t n_rows, const float* n, int64_t ldn,
                                         const float* x_self, int64_t ld_self, float* y,
                                         int64_t ldy, int32_t d, const float* W1, const float* b1,
                                         const float* W2, const float* b2, float slope,
                                         const float* gas_blocks, const int32_t* gas_perm,
                                         int32_t gas_bs, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_rows >= 0, "ngcf_transform: n_rows < 0");
  if (n_rows == 0) return GNNREC_OK;
  GNNREC_REQUIRE(W1 && b1 && W2 && b2, "ngcf_transform: null weights");
  GNNREC_REQUIRE(ldn >= d && ld_self >= d && ldy >= d, "ngcf_transform: leading dimension < d");
  GNNREC_REQUIRE(rows_ok(n, ldn) && rows_ok(x_self, ld_self) && rows_ok(y, ldy),
                 "ngcf_transform: n/x_self/y must be 16-B aligned with ld %% 4 == 0");
  if (gas_blocks) {
    GNNREC_REQUIRE(gas_perm && gas_bs >= 1 && gas_bs <= 32 && d % gas_bs == 0,
                   "ngcf_transform: bad GAS block size %d", gas_bs);
  }
  DenseParams p{};
  p.A = Csr{nullptr, nullptr, nullptr, n_rows};
  p.x = n; p.ldx = ldn; p.x_self = x_self; p.ld_self = ld_self; p.y = y; p.ldy = ldy;
  p.W1 = W1; p.b1 = b1; p.W2 = W2; p.b2 = b2; p.slope = slope;
  p.gas_blocks = gas_blocks; p.gas_perm = gas_perm; p.gas_bs = gas_bs;
  return launch_dense<0, false>(p, d, as_hip(stream));
}

extern "C" int gnnrec_dense_transform_f32(int64_t n_rows, const float* n, int64_t ldn, float* y,
                                          int64_t ldy, int32_t d, const float* M, float c_out,
                                          const float* resid, int64_t ld_resid, float c_res,
                                          float* acc, int64_t ld_acc, int32_t acc_mode,
                                          float w_out, float w_res, gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_rows >= 0, "dense_transform: n_rows < 0");
  if (n_rows == 0) return GNNREC_OK;
  GNNREC_REQUIRE(M, "dense_transform: null M");
  GNNREC_REQUIRE(acc_mode >= 0 && acc_mode <= 2, "dense_transform: acc_mode must be 0, 1 or 2");
  GNNREC_REQUIRE(y || acc_mode, "dense_transform: nothing to write");
  GNNREC_REQUIRE(rows_ok(n, ldn) && ldn >= d, "dense_transform: n must be 16-B aligned, ld %% 4 == 0, ld >= d");
  GNNREC_REQUIRE(resid ? (rows_ok(resid, ld_resid) && ld_resid >= d) : acc_mode != 1,
                 "dense_transform: resid must be 16-B aligned with ld >= d (required by acc_mode 1)");
  GNNREC_REQUIRE(!y || (rows_ok(y, ldy) && ldy >= d), "dense_transform: bad y");
  GNNREC_REQUIRE(!acc_mode || (rows_ok(acc, ld_acc) && ld_acc >= d), "dense_transform: bad acc");
  DenseParams p{};
  p.A = Csr{nullptr, nullptr, nullptr, n_rows};
  p.x = n; p.ldx = ldn; p.y = y; p.ldy = ldy;
  p.M = M; p.c_out = c_out; p.c_res = c_res; p.resid = resid; p.ld_resid = ld_resid;
  p.acc = acc; p.ld_acc = ld_acc; p.acc_mode = acc_mode; p.w_out = w_out; p.w_res = w_res;
  return launch_dense<1, false>(p, d, as_hip(stream));
}

namespace {
template <int K, int NT, int NW>
constexpr size_t rows_gemm_lds() {
  constexpr int PN = NT * 16;
  return sizeof(float) * ((size_t)K * (K >= 128 ? PN : PN + 4) + (size_t)NW * 16 * (PN + 4));
}

// Dynamic LDS past 64 KB needs the kernel attribute, set once per (kernel, device); a
// refusal is reported, not ignored.
bool big_lds_ok(const void* kern, int dev, size_t bytes) {
  static std::mutex mu;
  static std::vector<std::pair<std::pair<const void*, int>, int>> done;
  std::lock_guard<std::mutex> lock(mu);
  for (auto& e : done)
    if (e.first.first == kern && e.first.second == dev) return e.second > 0;
  const bool ok = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)bytes) == hipSuccess;
  if (!ok) (void)hipGetLastError();
  done.push_back({{kern, dev}, ok ? 1 : -1});
  return ok;
}
}  // namespace

// y[r, :p] = x[r, :k] @ B[k, p] (B row-major [k][p]) on the matrix cores, fp32 in / fp32
// accumulate, k ascending per output. k in {64, 128, 256}, p % 4 == 0, p <= 80 (k = 64),
// 64 (k = 128, 256); x and y rows 16-B aligned.
extern "C" int gnnrec_rows_gemm_f32(int64_t n_rows, const float* x, int64_t ldx, int32_t k,
                                    const float* B, int32_t p, float* y, int64_t ldy,
                                    int32_t apply_elu, int32_t epi, const float* self,
                                    int64_t ld_self, float* acc, int64_t ld_acc, float acc_div,
                                    gnnrec_stream_t stream) {
  GNNREC_REQUIRE(n_rows >= 0 && k > 0 && p > 0 && p % 4 == 0, "rows_gemm: bad sizes");
  if (n_rows == 0) return GNNREC_OK;
  const bool has_acc = (epi & (GNNREC_EPI_ACC_INIT | GNNREC_EPI_ACC_ADD)) != 0;
  GNNREC_REQUIRE(B && rows_ok(x, ldx) && ldx >= k && (y ? rows_ok(y, ldy) && ldy >= p : has_acc),
                 "rows_gemm: x/y must be 16-B aligned with ld %% 4 == 0 and ld >= k / p");
  GNNREC_REQUIRE(!has_acc || (rows_ok(acc, ld_acc) && ld_acc >= p),
                 "rows_gemm: ACC needs 16-B aligned acc rows");
  GNNREC_REQUIRE(!(epi & GNNREC_EPI_ACC_INIT) || (rows_ok(self, ld_self) && ld_self >= p),
                 "rows_gemm: ACC_INIT needs 16-B aligned self rows");
  const RowsGemmEpi ep{apply_elu, has_acc ? epi : 0, self, ld_self, acc, ld_acc, acc_div};
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  hipStream_t s = as_hip(stream);
  auto go = [&](auto kern, auto kk, auto ntc, auto nwc, int per_cu) -> int {
    constexpr int K = decltype(kk)::value, NT = decltype(ntc)::value, NW = decltype(nwc)::value;
    const size_t lds = rows_gemm_lds<K, NT, NW>();
    if (lds > 64 * 1024 && !big_lds_ok((const void*)kern, dev, lds)) {
      set_error("rows_gemm: the device refused %zu bytes of dynamic LDS", lds);
      return GNNREC_EHIP;
    }
    const int64_t tiles = ceil_div(n_rows, 16 * NW);
    const unsigned grid = (unsigned)std::min<int64_t>(tiles, (int64_t)cus * per_cu);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * NW), lds, s, n_rows, x, ldx, B, (int)p, y,
                       ldy, ep);
    return check_launch("rows_gemm");
  };
  using I = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I4 = std::integral_constant<int, 4>;
  using I5 = std::integral_constant<int, 5>;
  using I8 = std::integral_constant<int, 8>;
  using K64 = std::integral_constant<int, 64>;
  using K128 = std::integral_constant<int, 128>;
  using K256 = std::integral_constant<int, 256>;
  const int nt = (p + 15) / 16;
  if (k == 64) {
    switch (nt) {
      case 1: return go(rows_gemm_kernel<64, 1, 8>, K64{}, I{}, I8{}, 2);
      case 2: return go(rows_gemm_kernel<64, 2, 8>, K64{}, I2{}, I8{}, 2);
      // three 16-column tiles run as four: the NT = 3 instance compiles to a partially
      // overlapping MFMA accumulator (tests/test_native_host.py guards the ISA)
      case 3:
      case 4: return go(rows_gemm_kernel<64, 4, 8>, K64{}, I4{}, I8{}, 2);
      case 5: return go(rows_gemm_kernel<64, 5, 8>, K64{}, I5{}, I8{}, 2);
      default: break;
    }
  } else if (k == 128 && nt <= 4) {
    return go(rows_gemm_kernel<128, 4, 8>, K128{}, I4{}, I8{}, 1);
  } else if (k == 256 && nt <= 4) {
    return go(rows_gemm_kernel<256, 4, 8>, K256{}, I4{}, I8{}, 1);
  }
  set_error("rows_gemm: (k=%d, p=%d) unsupported (k 64: p <= 80; k 128/256: p <= 64)", (int)k,
            (int)p);
  return GNNREC_EUNSUPPORTED;
}
