"""One G100M column-ordered hop at d = 64 gathering from tables of several row strides: the
placed hop table (512-B rows, functional.hop_table), the compact [N, 64] table, and each
64-column block of config 3's placed [N, 256] NGCF concat table (functional.gather_table).
Same plan, same values in every table, so every output must hash the same.

    python tools/exp_hop_stride.py
"""
import hashlib
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
import bench  # noqa: E402
from src.ops import functional as F  # noqa: E402

dev = torch.device("cuda", 0)
g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
n = g.n_rows
x = torch.randn(n, 64, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
tables = {"hop_table_ld128": F.hop_table(n, 64, device=dev), "compact_ld64": torch.empty(n, 64, device=dev)}
cat = F.gather_table(n, 256, 192, device=dev)
for b in range(4):
    tables[f"concat_ld256_block{b}"] = cat[:, 64 * b:64 * (b + 1)]
for t in tables.values():
    t.copy_(x)
plan = F.tiled_plan_for(g, tables["hop_table_ld128"])
y = F.hop_table(n, 64, device=dev)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, t in tables.items():
    F.spmm_tiled_into(g, t, y, plan)
    torch.cuda.synchronize()
    best = []
    for _ in range(3):
        s.record()
        for _ in range(5):
            F.spmm_tiled_into(g, t, y, plan)
        e.record()
        e.synchronize()
        best.append(s.elapsed_time(e) / 5)
    print(json.dumps({"table": name, "ld": t.stride(0), "start_mod_1k": t.data_ptr() % 1024,
                      "ms_per_hop": sorted(best)[1],
                      "sha": hashlib.sha256(y.contiguous().cpu().numpy().tobytes()).hexdigest()[:16]}),
          flush=True)
