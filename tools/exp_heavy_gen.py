"""Generate tools/exp_heavy_kernel.hip: diagnostic variants of spmm_heavy_kernel (MODE 0 full,
1 no consume, 2 no loads, 3 no park) copied from csrc/spmm.hip. Not part of the product."""
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
src = (ROOT / "gnn-recommendations_amd/csrc/spmm.hip").read_text()
start = src.index("constexpr int kHeavyThreads")
end = src.index("// MODE 0: standalone GAS of x rows.")
body = src[start:end]
body = body.replace("template <int F, int DC>\n"
                    "__global__ __launch_bounds__(kHeavyThreads) void spmm_heavy_kernel(",
                    "template <int F, int DC, int MODE>\n__global__ __launch_bounds__(kHeavyThreads) void xheavy(")
body = body.replace("    if (wave == 0) consume(c);", "    if (wave == 0 && MODE != 1) consume(c);")
body = body.replace("    load_cols(c + 3, cols_c3);", "    if (MODE != 2) load_cols(c + 3, cols_c3);")
body = body.replace("    gather(cols_c2, st_c2);", "    if (MODE != 2) gather(cols_c2, st_c2);")
body = body.replace("    if (c + 1 < n_chunks) park(st_c1,", "    if (MODE != 3 && c + 1 < n_chunks) park(st_c1,")
assert "xheavy" in body and "MODE != 1" in body and "MODE != 2" in body and "MODE != 3" in body
out = ('// Diagnostic variants of spmm_heavy_kernel (NOT part of libgnnrec).\n'
       '#include "../gnn-recommendations_amd/csrc/gather.h"\nnamespace gnnrec {\n' + body +
       '''}  // namespace gnnrec
using namespace gnnrec;
extern "C" int xheavy_run(int mode, const int64_t* rp, const int32_t* col, const float* val,
                          const int64_t* rows, int64_t n_rows_list, const float* x, float* y,
                          hipStream_t s) {
  Csr A{rp, col, val, 0};
  const dim3 g((unsigned)n_rows_list), b(kHeavyThreads);
#define L(M) hipLaunchKernelGGL((xheavy<1, 64, M>), g, b, kHeavyLds, s, A, rows, x, (int64_t)64, y, \\
                               (int64_t)64, 64, 0, nullptr, (int64_t)64, nullptr, (int64_t)64, 1.f)
  switch (mode) { case 0: L(0); break; case 1: L(1); break; case 2: L(2); break; case 3: L(3); break;
                  default: return -1; }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
''')
(ROOT / "tools/exp_heavy_kernel.hip").write_text(out)
