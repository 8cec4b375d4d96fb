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
ap.add_argument("--sweep", action="store_true",
                help="config 2 over the round-6 CSR knobs (light form, fork, slices, threshold)")
ap.add_argument("--one", default=None, metavar="FLAGS:SLICE:HT[,...]",
                help="only config 2's propagation at these knob settings, 200 calls each "
                     "(for a kernel trace)")
ap.add_argument("--powerlaw", action="store_true",
                help="also the power-law 2M x 2M graph (50M pairs, Zipf 0.9) at d = 64 and 128")
ap.add_argument("--flags", type=int, default=None,
                help="functional.CSR_FLAGS for the whole run (e.g. 8 = GNNREC_CSR_TWO_LAUNCHES)")
ap.add_argument("--slice", type=int, default=None,
                help="functional.SPMM_SLICE_LEN for the whole run")
a = ap.parse_args()
if a.flags is not None:
    F.CSR_FLAGS = a.flags
if a.slice is not None:
    F.SPMM_SLICE_LEN = a.slice
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
    if a.one:
        x0 = m._initial_table().contiguous()
        for spec in a.one.split(","):
            fl, sl, ht = (int(v) for v in spec.split(":"))
            F.CSR_FLAGS, F.SPMM_SLICE_LEN = fl, sl
            for _ in range(200):
                out, _ = F.lightgcn_forward(g, x0, 3, heavy_threshold=ht)
            torch.cuda.synchronize()
            emit(case="config2_one", flags=fl, slice_len=sl, heavy_threshold=ht, sha=sha(out))
        sys.exit(0)
    t, (u, i) = ms_of(lambda: m(g), 100)
    emit(case="config2_model_forward", ms=t, sha=sha(torch.cat([u, i])))
    x0 = m._initial_table().contiguous()
    for ht in (128, 192, 256, 384, 512, 1024, 4096, 0):
        t, (out, _) = ms_of(lambda: F.lightgcn_forward(g, x0, 3, heavy_threshold=ht), 100)
        emit(case="config2_propagate", heavy_threshold=ht, ms=t, sha=sha(out),
             flags=F.CSR_FLAGS, slice_len=F.SPMM_SLICE_LEN)
    if a.sweep:
        from src.ops import _lib
        flag0, sl0 = F.CSR_FLAGS, F.SPMM_SLICE_LEN
        for light in (_lib.CSR_LIGHT_THROUGHPUT, _lib.CSR_LIGHT_LATENCY):
            for fork in (0, _lib.CSR_FORK):
                for sl in (0, 2048, 1024, 512):
                    for ht in (128, 256, 512, 1024):
                        if sl and sl < ht:
                            continue
                        F.CSR_FLAGS, F.SPMM_SLICE_LEN = light | fork, sl
                        t, (out, _) = ms_of(lambda: F.lightgcn_forward(g, x0, 3, heavy_threshold=ht), 100)
                        emit(case="config2_sweep", heavy_threshold=ht, light=light, fork=fork,
                             slice_len=sl, ms=t, sha=sha(out))
        F.CSR_FLAGS, F.SPMM_SLICE_LEN = flag0, sl0
    if a.g100m:
        g100 = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
        x = torch.randn(2_000_000, 64, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
        F.TILED_HOP = False
        for ht in ((128, 256) if a.sweep else (None,)):
            t, (out, _) = ms_of(lambda: F.lightgcn_forward(g100, x, 3, heavy_threshold=ht), 2)
            emit(case="g100m_csr_propagate", heavy_threshold=ht, ms=t, sha=sha(out))
        F.TILED_HOP = True
    if a.powerlaw:
        sys.path.insert(0, str(ROOT / "tools"))
        from bench_configs import powerlaw_graph
        gp = powerlaw_graph(2_000_000, 2_000_000, 50_000_000, 0.9, 0).to(dev)
        from src.ops import _lib
        knobs = {"r05": (256, 0, _lib.CSR_LIGHT_THROUGHPUT),
                 "r06": (F.SPMM_HEAVY_THRESHOLD, F.SPMM_SLICE_LEN, F.CSR_FLAGS)}
        if a.sweep:
            knobs.update({f"ht{ht}_sl{sl}": (ht, sl, 0) for ht in (128, 256, 512)
                          for sl in (0, 1024, 4096) if not sl or sl >= ht})
        for d in (64, 128):
            x = torch.randn(4_000_000, d, device=dev, generator=torch.Generator(device=dev).manual_seed(d))
            for name, (ht, sl, fl) in knobs.items():
                F.CSR_FLAGS, F.SPMM_SLICE_LEN = fl, sl
                t, (out, _) = ms_of(lambda: F.lightgcn_forward(gp, x, 3, heavy_threshold=ht), 2)
                emit(case=f"powerlaw2m_propagate_d{d}", knobs=name, heavy_threshold=ht,
                     slice_len=sl, flags=fl, ms=t, sha=sha(out))
            F.CSR_FLAGS, F.SPMM_SLICE_LEN = knobs["r06"][2], knobs["r06"][1]
            del x, out
