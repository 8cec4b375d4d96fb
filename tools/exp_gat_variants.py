"""Config-5 forward time for one libgnnrec build (GNNREC_LIB) and GAT switches (env), for
same-box A/Bs of the GAT kernels: prints one JSON line tagged with --tag.

    GNNREC_LIB=tools/var/x.so python tools/exp_gat_variants.py --tag x [--shape U I PAIRS]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT), str(ROOT / "tools")]
from bench_configs import config5_model, powerlaw_graph  # noqa: E402
from src.ops.distributed import DistributedGraph, gat_forward_dist  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tag", required=True)
ap.add_argument("--shape", type=int, nargs=3, default=[5_000_000, 5_000_000, 250_000_000])
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--plans", nargs="*", default=[],
                help="heavy-segment plans timed in this one process (same graph): 'column', "
                     "'row' or 'panel:<columns>:<min edges per panel>'")
ap.add_argument("--splits", nargs="*", default=[],
                help="heavy-row threshold / segment length pairs timed in this one process: "
                     "'<threshold>:<segment>' (default plan order)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
g = powerlaw_graph(*a.shape, 0.9, 0, 16, device=dev)
m = config5_model(tuple(a.shape[:2]), dev)
dg = DistributedGraph(g, 0, 1, dev)
x0 = dg.pad_table(m._initial_table())
from src.ops import functional as F  # noqa: E402


def run(tag):
    with torch.no_grad():
        out = gat_forward_dist(dg, m, x0)
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = gat_forward_dist(dg, m, x0)
            e.record()
            torch.cuda.synchronize()
            ms.append(s.elapsed_time(e))
    sig = float(out.double().abs().sum())
    print(json.dumps({"tag": tag, "lib": os.environ.get("GNNREC_LIB", "default"),
                      "env": {k: v for k, v in os.environ.items() if k.startswith("GNNREC_GAT")},
                      "plan": [F.GAT_SEGMENT_ORDER, F.GAT_PANEL, F.GAT_PANEL_MIN_EDGES],
                      "split": [F.GAT_HEAVY_THRESHOLD, F.GAT_SEGMENT],
                      "shape": a.shape, "nnz": g.nnz, "ms_median": float(np.median(ms)),
                      "ms": ms, "abs_sum": sig, "time": time.strftime("%H:%M:%S")}), flush=True)


if not a.plans and not a.splits:
    run(a.tag)
for spec in a.splits:
    F.GAT_HEAVY_THRESHOLD, F.GAT_SEGMENT = (int(v) for v in spec.split(":"))
    run(f"{a.tag}_split{spec}")
for spec in a.plans:
    parts = spec.split(":")
    F.GAT_SEGMENT_ORDER = parts[0]
    if parts[0] == "panel":
        F.GAT_PANEL, F.GAT_PANEL_MIN_EDGES = int(parts[1]), int(parts[2])
    run(f"{a.tag}_{spec}")
