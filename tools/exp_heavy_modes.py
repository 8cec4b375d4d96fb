"""Time the heavy-row kernel's parts (tools/exp_heavy_kernel.hip) on the longest ML-1M rows."""
import ctypes as C
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
from src.data.dataset import RecommendationDataset  # noqa: E402

lib = C.CDLL(str(ROOT / "tools" / "exp_heavy_kernel.so"))
lib.xheavy_run.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                           C.c_void_p, C.c_void_p, C.c_void_p]
dev = torch.device("cuda", 0)
ds = RecommendationDataset.synthetic_movielens(6040, 3706, 1_000_209, seed=1, name="ml-1m")
g = ds.get_graph(dev)
x = torch.randn(g.shape[0], 64, device=dev) * 0.1
y = torch.empty_like(x)
deg = g.row_ptr[1:] - g.row_ptr[:-1]
res = {}
for name, rows in {"longest": torch.argmax(deg).view(1),
                   "gt128": torch.nonzero(deg > 128).flatten()}.items():
    rows = rows.to(torch.int64).contiguous()
    st = torch.cuda.current_stream().cuda_stream
    for mode, mname in [(0, "full"), (1, "no_consume"), (2, "no_loads"), (3, "no_park")]:
        f = lambda: lib.xheavy_run(mode, g.row_ptr.data_ptr(), g.col.data_ptr(), g.val.data_ptr(),
                                   rows.data_ptr(), rows.numel(), x.data_ptr(), y.data_ptr(), st)
        for _ in range(3):
            assert f() == 0
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            f()
        e.record()
        e.synchronize()
        res[f"{name}_{mname}_us"] = s.elapsed_time(e) / 20 * 1e3
    res[f"{name}_rows"] = rows.numel()
res["max_deg"] = int(deg.max())
print(json.dumps(res))
