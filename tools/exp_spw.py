"""A/B of the column-ordered hop's plan walks at d = 128 (BASELINE config 4 width, G100M):
the shipped kernel walks the plan once per 32-feature slice (4 walks per hop, R = 1117 rows
per block); a GNNREC_TILED_SPW=2 build walks it once per PAIR of slices (2 walks, 256-B LDS
rows, R <= 600). Run once per library (GNNREC_LIB=...), same graph and x0:

    python tools/exp_spw.py --max-rows 1279 > a.json
    GNNREC_LIB=tools/bin/libgnnrec_spw2.so python tools/exp_spw.py --max-rows 600 > b.json

Prints ms per K=3 propagation (HIP events per hop), the plan's rows per block and chunks,
and a SHA-256 of the output bits (equal hashes = bit-identical results)."""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gnn-recommendations_amd"))
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from src.ops import functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-rows", type=int, default=1279)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    F.TILED_MAX_ROWS = a.max_rows
    t0 = time.perf_counter()
    g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
    torch.manual_seed(0)
    x0 = (torch.randn(g.shape[0], a.dim) * 0.1).to(dev)
    plan = F.tiled_plan_for(g, x0)
    assert plan is not None
    torch.cuda.synchronize()
    print(f"[exp_spw] graph + plan {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
    for _ in range(2):
        out, _ = F.lightgcn_forward(g, x0, 3)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(a.steps)]
    for s, e in ev:
        s.record()
        out, _ = F.lightgcn_forward(g, x0, 3)
        e.record()
    torch.cuda.synchronize()
    ms = [s.elapsed_time(e) for s, e in ev]
    print(json.dumps({
        "lib": os.environ.get("GNNREC_LIB", "default"), "dim": a.dim,
        "rows_per_block": int(plan["rows_per_block"]),
        "n_chunks": int(plan["n_chunks"]),
        "ms_per_step_median": float(np.median(ms)), "ms_samples": ms,
        "out_sha256": hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()}), flush=True)


if __name__ == "__main__":
    main()
