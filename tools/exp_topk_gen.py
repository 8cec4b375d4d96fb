"""Generate tools/exp_topk_kernel.hip: diagnostic variants of score_topk_kernel (MODE 0 full,
1 no candidate pass, 2 no MFMA (scores = 0 -> candidate pass on ties), 3 no tile loads).
Not part of the product."""
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
src = (ROOT / "gnn-recommendations_amd/csrc/topk.hip").read_text()
start = src.index("typedef float floatx4_t")
end = src.index("// Merge the n_split partial lists")
body = src[start:end]
body = body.replace("template <int D, int KM>\n__global__ __launch_bounds__(kBlock) void score_topk_kernel(TopkParams p) {",
                    "template <int D, int KM, int MODE>\n__global__ __launch_bounds__(kBlock) void xtopk(TopkParams p) {")
body = body.replace("        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], bf[nt][s], acc[nt], 0, 0, 0);",
                    "        if (MODE != 2) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], bf[nt][s], acc[nt], 0, 0, 0);")
body = body.replace("    if (t0 + TI < i_end) load_tile(t0 + TI);", "    if (MODE != 3 && t0 + TI < i_end) load_tile(t0 + TI);")
body = body.replace("    // candidates: lane holds users", "    if (MODE == 1) { if (acc[0][0] == 12345.f) p.out_score[0] = acc[1][1] + acc[2][2] + acc[3][3]; continue; }\n    // candidates: lane holds users")
assert body.count("MODE") >= 4
out = ('// Diagnostic variants of score_topk_kernel (NOT part of libgnnrec).\n#include <math.h>\n'
       '#include "../gnn-recommendations_amd/csrc/gather.h"\nnamespace gnnrec {\n' + body +
       '''}  // namespace gnnrec
using namespace gnnrec;
extern "C" int xtopk_run(int mode, const float* u, int64_t nb, const float* v, int64_t ni,
                         const int64_t* sp, const int32_t* sc, int64_t* oi, float* os, int n_split,
                         hipStream_t s) {
  TopkParams p{u, 64, nb, v, 64, ni, sp, sc, 20, oi, os, n_split};
  const dim3 g((unsigned)((nb + 63) / 64), (unsigned)n_split), b(kBlock);
  switch (mode) {
    case 0: hipLaunchKernelGGL((xtopk<64, 32, 0>), g, b, 0, s, p); break;
    case 1: hipLaunchKernelGGL((xtopk<64, 32, 1>), g, b, 0, s, p); break;
    case 2: hipLaunchKernelGGL((xtopk<64, 32, 2>), g, b, 0, s, p); break;
    case 3: hipLaunchKernelGGL((xtopk<64, 32, 3>), g, b, 0, s, p); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
''')
(ROOT / "tools/exp_topk_kernel.hip").write_text(out)
