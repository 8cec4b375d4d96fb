"""Time the top-K kernel's parts (tools/exp_topk_kernel.hip): 16384 users x 1M items, d=64."""
import ctypes as C
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
lib = C.CDLL(str(ROOT / "tools" / "exp_topk_kernel.so"))
lib.xtopk_run.argtypes = [C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p,
                          C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
dev = torch.device("cuda", 0)
nb, ni = 16384, 1_000_000
U = torch.randn(nb, 64, device=dev) * 0.1
V = torch.randn(ni, 64, device=dev) * 0.1
oi = torch.empty(nb * 4 * 20, dtype=torch.int64, device=dev)
os_ = torch.empty(nb * 4 * 20, device=dev)
st = torch.cuda.current_stream().cuda_stream
res = {}
for ns in (1, 4):
    for mode, name in [(0, "full"), (1, "no_candidates"), (2, "no_mfma"), (3, "no_loads")]:
        f = lambda: lib.xtopk_run(mode, U.data_ptr(), nb, V.data_ptr(), ni, None, None,
                                  oi.data_ptr(), os_.data_ptr(), ns, st)
        assert f() == 0
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(3):
            f()
        e.record()
        e.synchronize()
        res[f"split{ns}_{name}_ms"] = s.elapsed_time(e) / 3
print(json.dumps(res))
