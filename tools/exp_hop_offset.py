"""In config 3 (G100M NGCF + GAS) the second layer's hop runs ~4.0 ms against ~3.35 ms for the
first and third (profiles/r04/config3_trace_*). Each layer's hop gathers its input from a
64-column block of the [N, 256] concat table. This times the same hop (HIP events, median of
10) on every block of
  random   a [N, 256] table of randn * 0.1;
  config3  the config-3 model's own concat output (x0 and the three layer outputs);
and on a compact copy of each config-3 block, to tell a column-offset effect from a data one."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT), str(ROOT / "tools")]
import bench  # noqa: E402
import bench_configs  # noqa: E402
from src.ops import functional as F  # noqa: E402

dev = torch.device("cuda", 0)
g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
n, d = g.shape[0], 64
work = torch.empty(n, d, device=dev)


def hop_ms(x, reps=12):
    plan = F.tiled_plan_for(g, x)
    assert plan is not None
    ev = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        F.spmm_tiled_into(g, x, work, plan)
        e.record()
        ev.append((s, e))
    torch.cuda.synchronize()
    ms = [s.elapsed_time(e) for s, e in ev[2:]]
    return float(np.median(ms)), [round(v, 3) for v in ms]


def stats(x):
    a = x.abs()
    return {"zero_frac": float((x == 0).float().mean()),
            "subnormal_frac": float(((a > 0) & (a < 1.1754944e-38)).float().mean()),
            "abs_median": float(a.median()), "abs_max": float(a.max())}


T = torch.randn(n, 4 * d, device=dev, generator=torch.Generator(dev).manual_seed(0)) * 0.1
for k in range(4):
    med, ms = hop_ms(T[:, k * d:(k + 1) * d])
    print(json.dumps({"table": "random", "block": k, "ms_median": med, "ms": ms}), flush=True)
del T
m = bench_configs.config3_model(dev)
with torch.no_grad():
    out = m._native_concat_forward(g, list(m.gs_layers))
torch.cuda.synchronize()
for k in range(4):
    blk = out[:, k * d:(k + 1) * d]
    med, ms = hop_ms(blk)
    c = blk.contiguous()
    cmed, cms = hop_ms(c)
    print(json.dumps({"table": "config3", "block": k, "ms_median": med, "ms": ms,
                      "compact_ms_median": cmed, **stats(c)}), flush=True)
    del c
