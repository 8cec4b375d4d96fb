"""The CSR hop kernels (spmm_vec_kernel + spmm_heavy_kernel) for one libgnnrec build
(GNNREC_LIB): config 2 (ML-1M-shaped LightGCN K=3 d=64, the model's forward and the
propagation at several heavy-row thresholds) and, with --g100m, the G100M K=3 propagation on
the CSR path (tiled hop off), with --powerlaw the power-law 2M x 2M propagation (rows up to
400K neighbours: the heavy-row kernel). ms per call and an output hash (bit-identity across builds).

    GNNREC_LIB=tools/ab/base.so python tools/exp_csr_hop.py --tag base [--g100m]
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
import bench  # noqa: E402
from src.data.dataset import RecommendationDataset  # noqa: E402
from src.models import LightGCN  # noqa: E402
from src.ops import functional as F  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tag", required=True)
ap.add_argument("--g100m", action="store_true")
ap.add_argument("--powerlaw", action="store_true",
                help="also the power-law 2M x 2M graph (50M pairs, Zipf 0.9) at d = 64 and 128")
a = ap.parse_args()
dev = torch.device("cuda", 0)
lib = os.environ.get("GNNREC_LIB", "default")


def ms_of(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(5):
        s.record()
        for _ in range(reps):
            out = fn()
        e.record()
        e.synchronize()
        best.append(s.elapsed_time(e) / reps)
    return sorted(best)[2], out


def sha(t):
    return hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()[:16]


def emit(**kw):
    print(json.dumps({"tag": a.tag, "lib": lib, **kw}), flush=True)


with torch.no_grad():
    ds = RecommendationDataset.synthetic_movielens(6040, 3706, 1_000_209, seed=1, name="ml-1m")
    g = ds.get_graph(dev)
    torch.manual_seed(0)
    m = LightGCN(ds.n_users, ds.n_items, 64, 3, 0.1).to(dev).eval()
    t, (u, i) = ms_of(lambda: m(g), 100)
    emit(case="config2_model_forward", ms=t, sha=sha(torch.cat([u, i])))
    x0 = m._initial_table().contiguous()
    for ht in (256, 512, 1024, 4096, 0):
        t, (out, _) = ms_of(lambda: F.lightgcn_forward(g, x0, 3, heavy_threshold=ht), 100)
        emit(case="config2_propagate", heavy_threshold=ht, ms=t, sha=sha(out))
    if a.g100m:
        g100 = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
        x = torch.randn(2_000_000, 64, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
        F.TILED_HOP = False
        t, (out, _) = ms_of(lambda: F.lightgcn_forward(g100, x, 3), 2)
        emit(case="g100m_csr_propagate", ms=t, sha=sha(out))
    if a.powerlaw:
        sys.path.insert(0, str(ROOT / "tools"))
        from bench_configs import powerlaw_graph
        gp = powerlaw_graph(2_000_000, 2_000_000, 50_000_000, 0.9, 0).to(dev)
        for d in (64, 128):
            x = torch.randn(4_000_000, d, device=dev, generator=torch.Generator(device=dev).manual_seed(d))
            t, (out, _) = ms_of(lambda: F.lightgcn_forward(gp, x, 3), 2)
            emit(case=f"powerlaw2m_propagate_d{d}", ms=t, sha=sha(out))
            del x, out
