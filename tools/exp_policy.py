"""Time the column-ordered hop on G100M d=64 under load cache-policy variants
(GNNREC_TILED_POLICY: an experiment build that instantiated the kernel per policy; the
shipped kernel has no such switch — result in profiles/r02/exp_load_policy.jsonl: the default wins): per variant, median of 15 hops with HIP events,
bits checked against the row-parallel CSR kernel. One JSON line per variant."""
import json
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
import bench  # noqa: E402
from src.ops import functional as F  # noqa: E402

dev = torch.device("cuda", 0)
g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
x = torch.randn(g.shape[0], 64, device=dev, generator=torch.Generator(dev).manual_seed(0)) * 0.1
ref = torch.empty_like(x)
F.TILED_HOP = False
F.spmm_into(g, x, ref)
F.TILED_HOP = True
plan = F.tiled_plan_for(g, x)
y = torch.empty_like(x)
names = {0: "default", 1: "plan nt", 2: "gather sc1", 3: "gather sc1 + plan nt",
         4: "gather sc0 + plan nt", 5: "gather sc0 sc1 + plan nt"}
for rep in range(2):
    for pol in [int(v) for v in (sys.argv[1:] or names)]:
        os.environ["GNNREC_TILED_POLICY"] = str(pol)
        times = []
        for _ in range(15):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            F.spmm_tiled_into(g, x, y, plan)
            b.record()
            torch.cuda.synchronize()
            times.append(a.elapsed_time(b))
        times.sort()
        print(json.dumps({"policy": pol, "what": names.get(pol), "rep": rep,
                          "ms_median": times[7], "ms_min": times[0],
                          "bit_exact": bool(torch.equal(y.view(torch.int32), ref.view(torch.int32)))}),
              flush=True)
