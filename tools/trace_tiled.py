"""Diagnostic: how far apart the workgroups of one XCD group run inside a pass of the
column-ordered hop. Not part of the product.

    python tools/trace_tiled.py --build                 # here: libgnnrec_trace.so (-DGNNREC_TILED_TRACE)
    python tools/trace_tiled.py R:PANEL:SUB[:MEET] ...  # on the GPU box: G100M d=64, one hop each

The trace build stamps wall_clock64 (100 MHz) in wave 0 of every workgroup at each pass start
and each step barrier. Per XCD group (blockIdx % 8), pass and event, the spread is the
latest minus the earliest of the group's 32 stamps; it is compared with the step length.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "gnn-recommendations_amd"
TRACE_LIB = PKG / "lib" / "libgnnrec_trace.so"
EVENTS = 1024   # kTraceEvents


def build():
    sys.path.insert(0, str(PKG))
    import build_native as bn
    out = Path("/tmp/gnnrec_trace_build")
    out.mkdir(exist_ok=True)
    objs = []
    for src in bn.sources():
        obj = out / (src.name + ".o")
        subprocess.run([bn._hipcc(), *bn.CFLAGS, "-DGNNREC_TILED_TRACE", "-c", str(src), "-o",
                        str(obj)], check=True)
        objs.append(str(obj))
    subprocess.run([bn._hipcc(), "-shared", f"--offload-arch={bn.ARCH}", "-o", str(TRACE_LIB),
                    "-fPIC", *objs, "-lpthread"], check=True)
    print(TRACE_LIB)


def main(specs):
    import ctypes as C
    import numpy as np
    os.environ["GNNREC_LIB"] = str(TRACE_LIB)
    sys.path[:0] = [str(PKG), str(ROOT)]
    import torch
    import bench
    from src.ops import _lib, functional as F
    L = _lib.lib()
    L.gnnrec_debug_tiled_trace.argtypes = [C.c_void_p]
    dev = torch.device("cuda", 0)
    g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
    x = torch.randn(g.shape[0], 64, device=dev, generator=torch.Generator(dev).manual_seed(0)) * 0.1
    y = torch.empty_like(x)
    grid = torch.cuda.get_device_properties(dev).multi_processor_count
    buf = torch.zeros(grid * EVENTS, dtype=torch.int64, device=dev)
    for spec in specs:
        R, panel, sub, *rest = (int(v) for v in spec.split(":"))
        meet = rest[0] if rest else F.TILED_MEET_US
        plan = g.tiled_plan(rows_per_block=R, panel=panel, sub_panel=sub)
        assert L.gnnrec_debug_tiled_trace(0) == 0
        F.spmm_tiled_into(g, x, y, plan, meet_us=meet)
        buf.zero_()
        assert L.gnnrec_debug_tiled_trace(buf.data_ptr()) == 0
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        F.spmm_tiled_into(g, x, y, plan, meet_us=meet)
        b.record()
        torch.cuda.synchronize()
        assert L.gnnrec_debug_tiled_trace(0) == 0
        ms = a.elapsed_time(b)
        t = buf.view(grid, EVENTS).cpu().numpy().astype(np.int64)
        ns = int(plan["n_steps"][0].item())
        per_pass = ns + 1
        n_ev = int((t[0] > 0).sum())
        passes = n_ev // per_pass
        t0 = t[t > 0].min()
        spreads, steps, meets, trans, first = [], [], [], [], []
        for blk in range(grid):   # per block: pass transition and first step of a pass
            nsb = int(plan["n_steps"][blk].item())
            for p in range(passes - 1):
                last, nxt = t[blk, p * per_pass + nsb], t[blk, (p + 1) * per_pass]
                if nsb == ns and last > 0 and nxt > 0:
                    trans.append(int(nxt - last))
                    first.append(int(t[blk, (p + 1) * per_pass + 1] - nxt))
        for grp in range(8):
            blocks = list(range(grp, grid, 8))
            for p in range(passes):
                for e in range(per_pass):
                    col = t[blocks, p * per_pass + e]
                    if (col == 0).any():
                        continue
                    (meets if e == 0 else spreads).append(int(col.max() - col.min()))
                    if e > 0:
                        prev = t[blocks, p * per_pass + e - 1]
                        steps.append(float(np.median(col - prev)))
        res = {"R": R, "panel": panel, "sub_panel": sub, "meet_us": meet, "ms": ms,
               "steps_per_pass": ns, "passes_per_block": passes,
               "step_us_median": float(np.median(steps)) / 100,
               "group_spread_at_step_us_median": float(np.median(spreads)) / 100,
               "group_spread_at_step_us_p90": float(np.percentile(spreads, 90)) / 100,
               "group_spread_at_pass_start_us_median": float(np.median(meets)) / 100,
               # last step barrier of a pass -> next pass start (epilogue, meeting, zeroing)
               "pass_transition_us_median": float(np.median(trans)) / 100 if trans else None,
               "first_step_us_median": float(np.median(first)) / 100 if first else None,
               "kernel_span_us": float(t[t > 0].max() - t0) / 100}
        print(json.dumps(res), flush=True)
        np.save(ROOT / "gpurun_out" / f"trace_{R}_{panel}_{sub}_{meet}.npy", t)
        g._plans.clear()


if __name__ == "__main__":
    if sys.argv[1:] == ["--build"]:
        build()
    else:
        main(sys.argv[1:])
