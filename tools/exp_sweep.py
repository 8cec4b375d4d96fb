"""Diagnostics for the SpMM hop on MI355X (not part of the product).

Times experimental kernel variants (tools/exp_spmm.hip) on G100M and a working-set sweep:
the same 200M-nnz operand with columns folded into the first W rows (col % W), which shows
how the gather rate depends on where the gathered table lives (L2 / Infinity Cache / HBM).
"""
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gnn-recommendations_amd"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

lib = C.CDLL(str(ROOT / "tools" / "exp_spmm.so"))
lib.exp_spmm.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p,
                         C.c_void_p, C.c_void_p]


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts))


def main():
    dev = torch.device("cuda", 0)
    g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16)
    rp = g.row_ptr.to(dev)
    col_h = g.col.numpy()
    col = g.col.to(dev)
    val = g.val.to(dev)
    N = g.shape[0]
    x = torch.randn(N, 64, device=dev) * 0.1
    y = torch.empty_like(x)
    st = torch.cuda.current_stream().cuda_stream
    res = {}

    def run(v, c):
        rc = lib.exp_spmm(v, rp.data_ptr(), c.data_ptr(), val.data_ptr(), N, x.data_ptr(),
                          y.data_ptr(), st)
        assert rc == 0, rc

    names = {0: "group16_ch16", 1: "group16_ch32", 2: "group16_ch8", 3: "wave_per_row",
             4: "stream_only", 5: "nt_x_loads"}
    for v, name in names.items():
        res[name] = timeit(lambda: run(v, col))
        print(name, res[name], flush=True)
    lib.exp_spmm2.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    deg = np.diff(g.row_ptr.numpy())
    order = torch.from_numpy(np.argsort(-deg, kind="stable").astype(np.int32)).to(dev)
    x128 = torch.randn(N, 128, device=dev) * 0.1
    y128 = torch.empty_like(x128)

    def run2(v, xx=x, yy=y):
        rc = lib.exp_spmm2(v, rp.data_ptr(), col.data_ptr(), val.data_ptr(), N, order.data_ptr(),
                           xx.data_ptr(), yy.data_ptr(), st)
        assert rc == 0, rc

    for v, name in {6: "wave_row_ch32", 7: "group32_float2", 8: "group16_degree_sorted",
                    10: "wave_row_ch8"}.items():
        res[name] = timeit(lambda: run2(v))
        print(name, res[name], flush=True)
    res["d128_group32"] = timeit(lambda: run2(9, x128, y128))
    print("d128_group32", res["d128_group32"], flush=True)
    if "--quick" in sys.argv:
        print(json.dumps(res))
        return
    sweep = {}
    for W in [1024, 4096, 16384, 65536, 262144, 524288, 1_000_000, 2_000_000]:
        cw = torch.from_numpy((col_h % W).astype(np.int32)).to(dev)
        sweep[W] = timeit(lambda: run(0, cw))
        print("W", W, "table MB", W * 256 / 1e6, "ms", sweep[W], flush=True)
        del cw
    # half-table sweep keeping the bipartite structure: user rows only
    res["sweep"] = sweep
    print(json.dumps(res))


if __name__ == "__main__":
    main()
