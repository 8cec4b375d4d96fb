"""Experiment (not part of the product): column-ordered hop with LDS accumulators
(tools/exp_tiled.hip) vs the production row-parallel hop on G100M d=64.

Builds the per-(block, wave) edge streams on the GPU with torch, checks the result bit for
bit against the production kernel and times both.

    python tools/exp_tiled.py [--R 600] [--nw 16] [--out gpurun_out/exp_tiled.jsonl]
"""
import argparse
import ctypes as C
import json
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

CH = 16
import os  # noqa: E402
lib = C.CDLL(str(ROOT / "tools" / os.environ.get("EXP_TILED_SO", "exp_tiled.so")))
lib.exp_stepped_hop.argtypes = [C.c_int] + [C.c_void_p] * 6 + [C.c_int64, C.c_void_p, C.c_int64,
                                                              C.c_int, C.c_int, C.c_int,
                                                              C.c_void_p, C.c_int, C.c_void_p]
lib.exp_tiled_hop.argtypes = [C.c_int] + [C.c_void_p] * 6 + [C.c_int64, C.c_int, C.c_int,
                                                              C.c_int, C.c_void_p]


def build_streams(rp, col, val, N, R, NW, mode, order="col"):
    """Per (block, wave) streams. rows of block b = [b*R, (b+1)*R); wave = local % NW."""
    dev = col.device
    nnz = col.numel()
    deg = rp[1:] - rp[:-1]
    row = torch.repeat_interleave(torch.arange(N, device=dev, dtype=torch.int64), deg)
    blk = row // R
    loc = row - blk * R
    w = loc % NW
    s = blk * NW + w
    n_blocks = (N + R - 1) // R
    n_streams = n_blocks * NW
    cbits = int(N).bit_length()
    if order == "col":
        key = (s << (cbits + 11)) | (col.to(torch.int64) << 11) | loc
    else:  # row order inside the stream (= CSR order per wave)
        key = (s << (cbits + 11)) | (loc << cbits) | col.to(torch.int64)
    key, perm = torch.sort(key)
    del key
    s_sorted = s[perm]
    cnt = torch.bincount(s_sorted, minlength=n_streams)
    pcnt = (cnt + CH - 1) // CH * CH
    start = torch.zeros(n_streams + 1, dtype=torch.int64, device=dev)
    start[1:] = torch.cumsum(cnt, 0)
    pstart = torch.zeros(n_streams + 1, dtype=torch.int64, device=dev)
    pstart[1:] = torch.cumsum(pcnt, 0)
    total = int(pstart[-1]) + CH
    rank = torch.arange(nnz, device=dev, dtype=torch.int64) - start[s_sorted]
    pos = pstart[s_sorted] + rank
    scol = torch.zeros(total, dtype=torch.int32, device=dev)
    sval = torch.zeros(total, dtype=torch.float32, device=dev)
    srow = torch.full((total,), R, dtype=torch.int32, device=dev)
    scol[pos] = col[perm]
    sval[pos] = val[perm]
    srow[pos] = loc[perm].to(torch.int32)
    del perm, s_sorted, rank, pos
    # dup chain: prev slot (+1) of the same row within the chunk
    rows = srow.view(-1, CH)
    prev = torch.zeros_like(rows)
    ndup = 0
    for t in range(1, CH):
        eq = rows[:, :t] == rows[:, t:t + 1]
        idx = torch.arange(1, t + 1, device=dev, dtype=torch.int32)
        pv = (eq.to(torch.int32) * idx).max(dim=1).values
        pv = torch.where(rows[:, t] == R, torch.zeros_like(pv), pv)
        prev[:, t] = pv
        ndup += int((pv > 0).sum())
    meta = (srow | (prev.view(-1) << 11)).to(torch.int32)
    meta16 = (meta & 0xFFFF).view(-1, 2)
    meta32 = (meta16[:, 0] | (meta16[:, 1] << 16)).contiguous()
    return dict(scol=scol, sval=sval, smeta=meta32, sptr=pstart, n_blocks=n_blocks,
                padded=total, ndup=ndup)


blib = C.CDLL(str(ROOT / "tools" / "exp_tiled_build.so"))
blib.tiled_build.restype = C.c_void_p
blib.tiled_build.argtypes = [C.c_void_p] * 3 + [C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int,
                                                C.c_int64, C.c_void_p, C.c_void_p]
blib.tiled_emit.argtypes = [C.c_void_p] * 6
blib.tiled_free.argtypes = [C.c_void_p]


def build_stepped(rp, col, val, N, R, Wp, NW=16, ch=CH, row_bytes=256):
    """Host builder (exp_tiled_build.cpp) on numpy CSR arrays -> numpy streams."""
    rp = np.ascontiguousarray(rp, np.int64)
    col = np.ascontiguousarray(col, np.int32)
    val = np.ascontiguousarray(val, np.float32)
    tot, nb = C.c_int64(), C.c_int64()
    h = blib.tiled_build(rp.ctypes.data, col.ctypes.data, val.ctypes.data, N, R, Wp, NW, ch,
                         row_bytes, C.byref(tot), C.byref(nb))
    T = tot.value + ch
    xo = np.zeros(T, np.uint32)
    sv = np.zeros(T, np.float32)
    sm = np.full(T, R, np.uint16)
    wptr = np.zeros(nb.value * NW + 1, np.int64)
    ns = np.zeros(nb.value, np.int32)
    blib.tiled_emit(h, xo.ctypes.data, sv.ctypes.data, sm.ctypes.data, wptr.ctypes.data,
                    ns.ctypes.data)
    blib.tiled_free(h)
    return dict(xoff=xo, sval=sv, smeta=sm, wptr=wptr, nsteps=ns, n_blocks=nb.value,
                padded=T)


def emulate_stepped(S, x, N, R, NW=16, ch=CH):
    """numpy model of stepped_hop (exact fma via float64 is exact for these products? no:
    used only to check the stream structure: order per row and barrier accounting)."""
    y = np.zeros((N, x.shape[1]), np.float64)
    seen = {}
    xo, sv, sm, wptr, ns = S["xoff"], S["sval"], S["smeta"], S["wptr"], S["nsteps"]
    for b in range(S["n_blocks"]):
        acc = np.zeros((R + 1, x.shape[1]))
        events = []  # (step, wave, chunk) order check
        for w in range(NW):
            cur = 0
            for c in range(wptr[b * NW + w], wptr[b * NW + w + 1], ch):
                cur += (int(sm[c]) >> 10) & 31
                for t in range(ch):
                    r = int(sm[c + t]) & 1023
                    events.append((cur, w, r, int(xo[c + t]) // 256, float(sv[c + t])))
            assert cur <= ns[b] - 1 or ns[b] == 0
        events.sort(key=lambda e: e[0])  # steps in order; inside a step rows are disjoint
        last = {}
        for st, w, r, cidx, v in events:
            if r == R:
                continue
            key = r
            assert last.get(key, (-1, -1))[0] < st or last[key][1] == w, "row in two waves in one step"
            last[key] = (st, w)
            acc[r] += v * x[cidx]
        for i in range(R):
            if b * R + i < N:
                y[b * R + i] = acc[i]
    return y


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, nargs="+", default=[600])
    ap.add_argument("--nw", type=int, default=16)
    ap.add_argument("--out", default="gpurun_out/exp_tiled.jsonl")
    ap.add_argument("--pairs", type=int, default=100_000_000)
    ap.add_argument("--fold", type=int, default=0)
    ap.add_argument("--wp", type=int, nargs="*", default=[])
    ap.add_argument("--slack", type=int, nargs="+", default=[0])
    ap.add_argument("--no-ref", action="store_true")
    ap.add_argument("--modes", type=int, nargs="+", default=[0])
    ap.add_argument("--grids", type=int, nargs="+", default=[1])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    t0 = time.perf_counter()
    g = bench.build_graph(1_000_000, 1_000_000, a.pairs, 0, 16)
    print(f"graph {time.perf_counter() - t0:.1f}s nnz={g.nnz}", flush=True)
    gd = g.to(dev)
    N = g.shape[0]
    torch.manual_seed(0)
    x = torch.randn(N, 64, device=dev) * 0.1
    y_ref = torch.empty_like(x)
    st = torch.cuda.current_stream().cuda_stream
    props = torch.cuda.get_device_properties(0)
    ncu = props.multi_processor_count
    res = []

    def ref():
        F.spmm_into(gd, x, y_ref)
    if a.fold:
        gd.col.remainder_(a.fold)
    t_ref = timeit(ref, reps=3 if a.no_ref else 10)
    print(f"production hop {t_ref:.3f} ms", flush=True)
    res.append({"variant": "production spmm_vec_kernel", "ms": t_ref})
    rp, col, val = gd.row_ptr, gd.col, gd.val
    xb = N * 64 * 4
    for R in (a.R if a.wp else []):
        for Wp in a.wp:
            built = {}
            ctr = torch.zeros(8 * 32, dtype=torch.int32, device=dev)
            for mode, gm, slack in [(m, gm, sl) for m in a.modes for gm in a.grids for sl in a.slack]:
                nw = 15 if slack > 0 else a.nw
                if nw not in built:
                    built.clear()
                    t0 = time.perf_counter()
                    H = build_stepped(g.row_ptr.numpy(),
                                      g.col.numpy() % a.fold if a.fold else g.col.numpy(),
                                      g.val.numpy(), N, R, Wp, NW=nw)
                    tb = time.perf_counter() - t0
                    S = {k: (torch.from_numpy(v.view(np.int16) if v.dtype == np.uint16 else
                                              v.view(np.int32) if v.dtype == np.uint32 else v).to(dev)
                             if isinstance(v, np.ndarray) else v) for k, v in H.items()}
                    built[nw] = (S, H, tb)
                S, H, tb = built[nw]
                y = torch.empty_like(x)
                grid = ncu * gm
                def run():
                    rc = lib.exp_stepped_hop(mode, S["xoff"].data_ptr(), S["sval"].data_ptr(),
                                             S["smeta"].data_ptr(), S["wptr"].data_ptr(),
                                             S["nsteps"].data_ptr(), x.data_ptr(), xb,
                                             y.data_ptr(), N, R, S["n_blocks"], grid,
                                             ctr.data_ptr() if slack else None, slack, st)
                    assert rc == 0, rc
                ms = timeit(run)
                same = bool(torch.equal(y.view(torch.int32), y_ref.view(torch.int32)))
                r = {"variant": f"stepped mode={mode}", "R": R, "Wp": Wp, "grid": grid, "slack": slack,
                     "ms": ms, "bitexact": same, "padded": S["padded"], "nnz": g.nnz,
                     "steps": int(H["nsteps"].sum()), "build_s": tb, "fold": a.fold}
                print(json.dumps(r), flush=True)
                res.append(r)
            built.clear()
    for R in ([] if a.wp else a.R):
        for order in ("col",):
            t0 = time.perf_counter()
            S = build_streams(rp, col, val, N, R, a.nw, 0, order)
            torch.cuda.synchronize()
            tb = time.perf_counter() - t0
            y = torch.empty_like(x)
            for mode, gm in [(m, gm) for m in a.modes for gm in a.grids]:
                grid = ncu * gm
                def run():
                    rc = lib.exp_tiled_hop(mode, S["scol"].data_ptr(), S["sval"].data_ptr(),
                                           S["smeta"].data_ptr(), S["sptr"].data_ptr(),
                                           x.data_ptr(), y.data_ptr(), N, R, S["n_blocks"],
                                           grid, st)
                    assert rc == 0, rc
                ms = timeit(run)
                same = bool(torch.equal(y.view(torch.int32), y_ref.view(torch.int32)))
                r = {"variant": f"tiled order={order} mode={mode}", "R": R, "nw": a.nw, "grid": grid,
                     "ms": ms, "bitexact": same, "padded": S["padded"], "nnz": g.nnz,
                     "dup_slots": S["ndup"], "build_s": tb}
                print(json.dumps(r), flush=True)
                res.append(r)
            del S
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    with open(a.out, "a") as f:
        for r in res:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
