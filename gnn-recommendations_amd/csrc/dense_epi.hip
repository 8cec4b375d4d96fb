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

template <int D, int MODE>
__global__ __launch_bounds__(kBlock) void spmm_mfma_kernel(DenseParams p) {
  constexpr int GROUP = D / 4;
  constexpr int RPW = 64 / GROUP;
  constexpr int PASS_ROWS = RPW * (kBlock / 64);
  constexpr int TR = PASS_ROWS > 16 ? PASS_ROWS : 16;  // rows per tile
  constexpr int PASSES = TR / PASS_ROWS;
  constexpr int KD = MODE == 0 ? 2 * D : D;  // contraction length
  constexpr int LDA = KD + 2;                // == 2 mod 32: conflict-free ds_read_b32 A reads
  constexpr int MT = TR / 16, NT = D / 16, TILES = MT * NT;
  constexpr int TPW = (TILES + 3) / 4;  // MFMA output tiles per wave
  constexpr int STEPS = KD / 4;
  __shared__ __attribute__((aligned(16))) float a_lds[TR * LDA];
  __shared__ __attribute__((aligned(16))) float o_lds[TR][D + 4];
  __shared__ __attribute__((aligned(16))) float w_gas[MODE == 0 ? D * 32 : 4];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int gl = lane % GROUP;
  const int i16 = lane & 15, k4 = lane >> 4;

  // Weight slabs -> VGPRs, once per workgroup.
  float bf[TPW][STEPS];
  float bias1[TPW], bias2[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = wave + 4 * i;
    const int j = 16 * ((t < TILES ? t : 0) % NT) + i16;
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      const int k = 4 * s + k4;
      if (MODE == 0)
        bf[i][s] = k < D ? p.W1[j * D + k] : p.W2[j * D + (k - D)];
      else
        bf[i][s] = p.M[k * D + j];
    }
    if (MODE == 0) {
      bias1[i] = p.b1[j];
      bias2[i] = p.b2[j];
    }
  }
  const bool gas = MODE == 0 && p.gas_blocks != nullptr;
  int pj[4] = {0, 0, 0, 0};
  if (gas) {
    for (int i = threadIdx.x; i < D * p.gas_bs; i += kBlock) w_gas[i] = p.gas_blocks[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) pj[q] = p.gas_perm[4 * gl + q];
  }

  const int64_t n_tiles = ceil_div(p.A.n_rows, TR);
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t row0 = tile * TR;
    // ---- phase 1: gather rows into the A tile
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
      const int slot = ps * PASS_ROWS + wave * RPW + lane / GROUP;
      const int64_t r = row0 + slot;
      float4 n = make_float4(0.f, 0.f, 0.f, 0.f), xs = n;
      if (r < p.A.n_rows) {
        n = gather_row<GROUP>(p.A.col, p.A.val, p.A.row_ptr[r], p.A.row_ptr[r + 1], p.x, p.ldx, gl);
        if (MODE == 0) xs = ld4(p.x_self + r * p.ld_self + 4 * gl);
      }
      float2* a2 = reinterpret_cast<float2*>(&a_lds[slot * LDA + 4 * gl]);
      a2[0] = make_float2(n.x, n.y);
      a2[1] = make_float2(n.z, n.w);
      if (MODE == 0) {
        float2* i2 = reinterpret_cast<float2*>(&a_lds[slot * LDA + D + 4 * gl]);
        i2[0] = make_float2(xs.x * n.x, xs.y * n.y);
        i2[1] = make_float2(xs.z * n.z, xs.w * n.w);
      }
    }
    __syncthreads();
    // ---- phase 2: MFMA
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int t = wave + 4 * i;
      if (t < TILES) {
        const int mt = t / NT, nt = t % NT;
        floatx4 c1 = {0.f, 0.f, 0.f, 0.f}, c2 = {0.f, 0.f, 0.f, 0.f};
        const float* arow = &a_lds[(16 * mt + i16) * LDA + k4];
#pragma unroll
        for (int s = 0; s < STEPS; ++s) {
          const float a = arow[4 * s];
          if (MODE == 0 && s >= STEPS / 2)
            c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bf[i][s], c2, 0, 0, 0);
          else
            c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bf[i][s], c1, 0, 0, 0);
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
    // ---- phase 3: row epilogue + coalesced store
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
      const int slot = ps * PASS_ROWS + wave * RPW + lane / GROUP;
      const int64_t r = row0 + slot;
      if (r >= p.A.n_rows) continue;
      float4 o;
      if (MODE == 0) {
        o = gas ? gas_row<D>(&o_lds[slot][0], w_gas, p.gas_bs, pj) : ld4(&o_lds[slot][4 * gl]);
      } else {
        const float4 t = ld4(&o_lds[slot][4 * gl]);
        const float4 rs = p.resid ? ld4(p.resid + r * p.ld_resid + 4 * gl)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
        if (p.resid)
          o = make_float4(p.c_out * t.x + p.c_res * rs.x, p.c_out * t.y + p.c_res * rs.y,
                          p.c_out * t.z + p.c_res * rs.z, p.c_out * t.w + p.c_res * rs.w);
        else
          o = make_float4(p.c_out * t.x, p.c_out * t.y, p.c_out * t.z, p.c_out * t.w);
        if (p.acc_mode) {
          float* ar = p.acc + r * p.ld_acc + 4 * gl;
          const float4 base =
              p.acc_mode == 1
                  ? make_float4(p.w_res * rs.x, p.w_res * rs.y, p.w_res * rs.z, p.w_res * rs.w)
                  : ld4(ar);
          st4(ar, make_float4(base.x + p.w_out * o.x, base.y + p.w_out * o.y,
                              base.z + p.w_out * o.z, base.w + p.w_out * o.w));
        }
      }
      if (p.y) st4(p.y + r * p.ldy + 4 * gl, o);
    }
  }
}

}  // namespace gnnrec

using namespace gnnrec;

namespace {

template <int MODE>
int launch_dense(const DenseParams& p, int d, hipStream_t s) {
  const int tr = (d == 32) ? 32 : 16;
  const int64_t tiles = ceil_div(p.A.n_rows, tr);
  const unsigned grid = (unsigned)(tiles < 2048 ? tiles : 2048);
  switch (d) {
    case 32: hipLaunchKernelGGL((spmm_mfma_kernel<32, MODE>), dim3(grid), dim3(kBlock), 0, s, p); break;
    case 64: hipLaunchKernelGGL((spmm_mfma_kernel<64, MODE>), dim3(grid), dim3(kBlock), 0, s, p); break;
    case 128: hipLaunchKernelGGL((spmm_mfma_kernel<128, MODE>), dim3(grid), dim3(kBlock), 0, s, p); break;
    default: set_error("dense epilogue: d=%d unsupported (32, 64, 128)", d); return GNNREC_EUNSUPPORTED;
  }
  return check_launch(MODE == 0 ? "spmm_ngcf" : "spmm_dense");
}

bool rows_ok(const float* p, int64_t ld) { return p && aligned16(p) && !(ld & 3); }

}  // namespace

extern "C" int gnnrec_spmm_ngcf_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                                    int64_t n_rows, const float* x, int64_t ldx,
                                    const float* x_self, int64_t ld_self, float* y, int64_t ldy,
                                    int32_t d, const float* W1, const float* b1, const float* W2,
                                    const float* b2, float slope, const float* gas_blocks,
                                    const int32_t* gas_perm, int32_t gas_bs,
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
  return launch_dense<0>(p, d, as_hip(stream));
}

extern "C" int gnnrec_spmm_dense_f32(const int64_t* row_ptr, const int32_t* col, const float* val,
                                     int64_t n_rows, const float* x, int64_t ldx, float* y,
                                     int64_t ldy, int32_t d, const float* M, float c_out,
                                     const float* resid, int64_t ld_resid, float c_res, float* acc,
                                     int64_t ld_acc, int32_t acc_mode, float w_out, float w_res,
                                     gnnrec_stream_t stream) {
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
  return launch_dense<1>(p, d, as_hip(stream));
}
