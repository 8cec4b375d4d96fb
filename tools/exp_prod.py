"""Sweep the VEC-generic SpMM form (gather.h gather_row_v) over VEC x CH x d on G100M."""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gnn-recommendations_amd"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from tools.exp_sweep import timeit  # noqa: E402

lib = C.CDLL(str(ROOT / "tools" / "exp_spmm.so"))
lib.exp_prod.argtypes = [C.c_int] * 3 + [C.c_void_p] * 3 + [C.c_int64] + [C.c_void_p] * 3


def main():
    dev = torch.device("cuda", 0)
    g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16)
    rp, col, val = g.row_ptr.to(dev), g.col.to(dev), g.val.to(dev)
    N = g.shape[0]
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    lib.exp_spmm.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p,
                             C.c_void_p, C.c_void_p]
    lib.exp_spmm2.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    x = torch.randn(N, 64, device=dev) * 0.1
    y = torch.empty_like(x)
    for rep in range(2):
        for v in (3, 0):
            t = timeit(lambda: lib.exp_spmm(v, rp.data_ptr(), col.data_ptr(), val.data_ptr(), N,
                                            x.data_ptr(), y.data_ptr(), st), reps=7)
            res[f"exp{v}_r{rep}"] = t
            print("exp", v, t, flush=True)
        t = timeit(lambda: lib.exp_spmm2(10, rp.data_ptr(), col.data_ptr(), val.data_ptr(), N, 0,
                                         x.data_ptr(), y.data_ptr(), st), reps=7)
        res[f"wave_row_ch8_r{rep}"] = t
        print("wave_row_ch8", t, flush=True)
    for d, combos in {64: [(1, 8), (1, 1008), (1, 16), (1, 1016), (2, 16), (2, 1016), (2, 8), (2, 1008), (4, 16), (4, 1016)],
                      32: [(2, 16), (2, 1016)],
                      128: [(2, 16), (2, 1016), (4, 16), (4, 1016)]}.items():
        x = torch.randn(N, d, device=dev) * 0.1
        y = torch.empty_like(x)
        for vec, ch in combos:
            def run():
                assert lib.exp_prod(d, vec, ch, rp.data_ptr(), col.data_ptr(), val.data_ptr(), N,
                                    x.data_ptr(), y.data_ptr(), st) == 0
            t = timeit(run, reps=7)
            res[f"d{d}_v{vec}_c{ch}"] = t
            print(d, vec, ch, t, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
