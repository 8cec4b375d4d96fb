"""gnnrec_rows_gemm_f32 alone (GAT's projections K = 64 and head mean K = 256) for one libgnnrec
build (GNNREC_LIB): ms per launch, TFLOP/s, GB/s, output hash (bit-identity across builds) and
max |diff| against torch fp32. One JSON line per shape.

    GNNREC_LIB=tools/var/x.so python tools/exp_rows_gemm.py --tag x
"""
import argparse
import hashlib
import json
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
from src.ops import functional as F  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tag", required=True)
ap.add_argument("--rows", type=int, default=5_000_000)
a = ap.parse_args()
dev = torch.device("cuda", 0)
for K, P in ((64, 64), (64, 72), (128, 64), (256, 64)):
    g = torch.Generator(device=dev).manual_seed(K + P)
    x = torch.randn(a.rows, K, device=dev, generator=g)
    B = torch.randn(K, P, device=dev, generator=g) * 0.1
    y = torch.empty(a.rows, P, device=dev)
    F.rows_gemm(x, B, out=y)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        F.rows_gemm(x, B, out=y)
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / 20
    print(json.dumps({"tag": a.tag, "lib": os.environ.get("GNNREC_LIB", "default"), "K": K, "P": P,
                      "rows": a.rows, "ms": ms, "TFLOPs": 2 * a.rows * K * P / ms / 1e9,
                      "GBps": a.rows * (K + P) * 4 / ms / 1e6,
                      "max_abs_diff_vs_torch": float((y - x @ B).abs().max()),
                      "y_sha256": hashlib.sha256(y.cpu().numpy().tobytes()).hexdigest()[:16]}),
          flush=True)
    del x, y
