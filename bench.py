"""Headline benchmark: LightGCN K=3 propagation throughput on MI355X (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--dim 64] [--layers 3]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N ...

Workload (BASELINE.json configs[2] graph, `metric`): synthetic bipartite graph G100M =
1M users x 1M items, 100M pairs drawn with numpy default_rng(0) and deduplicated
(99,994,938 interactions -> nnz(A) = 199,989,876), symmetric D^-1/2 A D^-1/2 operand,
x0 ~ N(0, 0.1) (lightgcn.yaml init_scale), d = 64, K = 3 hops + layer mean: the body of
LightGCN.forward (lightgcn.py:76-95), eval mode.

One step = one full propagation (K SpMM hops with the layer mean fused into their
epilogues) with the operand and x0 already resident in HBM. value = K * nnz / t_step
(edges/s, every stored nonzero one directed message). N > 1: the SAME graph (strong scaling)
on a grid of F feature groups x N/F destination-row shards (RankGrid, src/ops/distributed.py:
F = gcd(N, d/32) by default, so d = 64 on 2 GPUs runs two 32-feature halves with no exchange
at all); within a feature group, one RCCL exchange per hop of that group's columns —
all-gather, or bipartite point-to-point with 1/4/8 overlap chunks, whichever whole steps time
fastest before the timed region; t_step = max over ranks.

Also reported: roofline of the dominant kernel (the SpMM hop) from HIP events around every
hop launch inside the timed region — `achieved`/`frac` on SURVEY §8(d)'s compulsory bytes
B_hop = 8 nnz + 8 (rows+1) + 4 d |src| + 4 d rows, and beside it the same launch priced with
its fused layer-mean epilogue bytes — the PMC-measured HBM traffic per launch when a profile
summary made from THIS kernel source and plan exists under profiles/ (else null), and the
reference's CPU path (restated op for op in oracle/torch_ref.py) on this host's
cores: the scipy operand build over every pair and the full K-hop torch.sparse.mm propagation
+ stack().mean(0), each compared bit for bit with the GPU's operand, hop 1 and output.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "gnn-recommendations_amd"))
sys.path.insert(0, str(ROOT))

from src.ops import CsrGraph  # noqa: E402
from src.ops import functional as F  # noqa: E402
from src.ops._lib import EPI_ACC_ADD, EPI_ACC_INIT, EPI_ACC_X, EPI_NO_Y  # noqa: E402
from src.ops.distributed import (RankGrid, feature_groups_for,  # noqa: E402
                                 lightgcn_propagate_dist, make_work, _native_hop)

METRIC = "edges/s + achieved HBM GB/s, LightGCN K=3 dim=64, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
G100M_NNZ = 199_989_876


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def host_threads() -> int:
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return max(1, len(os.sched_getaffinity(0)))


def build_graph(n_users: int, n_items: int, n_pairs: int, seed: int, threads: int) -> CsrGraph:
    rng = np.random.default_rng(seed)
    u = rng.integers(0, n_users, n_pairs, dtype=np.int64)
    i = rng.integers(0, n_items, n_pairs, dtype=np.int64)
    return CsrGraph.from_interactions(u, i, n_users, n_items, binary=True, n_threads=threads)


def distinct_cols(g: CsrGraph, n_cols: int) -> int:
    seen = np.zeros(n_cols, dtype=bool)
    seen[g.col.cpu().numpy()] = True
    return int(seen.sum())


class HopTimer:
    """HIP events on the launch stream around every SpMM hop (the dominant kernel)."""

    def __init__(self):
        self.pairs = []
        self.active = False

    def hop(self, adj, x, y, **kw):
        if not self.active:
            return _native_hop(adj, x, y, **kw)
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        _native_hop(adj, x, y, **kw)
        e.record()
        self.pairs.append((s, e))

    hop.native_hop = True   # lightgcn_propagate_dist passes the chunk options through it

    def reset(self, active: bool):
        self.pairs, self.active = [], active

    def durations_ms(self):
        return [s.elapsed_time(e) for s, e in self.pairs]


class ExchangeTimer:
    """HIP events on the compute stream around each per-hop exchange (N > 1): before the
    exchange call and after it returns (torch's RCCL work makes the current stream wait on
    the exchange's completion), i.e. the time the hop chain is held by the exchange — the
    whole transfer when it is not overlapped, its un-overlapped tail when chunks are."""

    def __init__(self, dg):
        self.pairs = []
        self.active = False
        for name in ("exchange", "finish"):
            fn = getattr(dg, name)
            setattr(dg, name, self._wrap(fn))

    def _wrap(self, fn):
        def timed(*a, **kw):
            if not self.active:
                return fn(*a, **kw)
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            r = fn(*a, **kw)
            e.record()
            self.pairs.append((s, e))
            return r
        return timed

    def reset(self, active: bool):
        self.pairs, self.active = [], active

    def durations_ms(self):
        return [s.elapsed_time(e) for s, e in self.pairs]


class Layout:
    """One rank layout of the N-GPU propagation: the RankGrid (F feature groups x R row
    shards), this rank's padded x0 columns, hop buffers, column-ordered plan and timers."""

    def __init__(self, full: CsrGraph, rank: int, world: int, device, d: int, fg, exchange: str):
        self.grid = RankGrid(full, rank, world, device, d, fg,
                             exchange="p2p" if exchange == "auto" else exchange)
        self.dg = self.grid.dg
        log(f"layout F={self.grid.F} x R={self.grid.R}: shard on the device")
        self.src = distinct_cols(self.dg.shard, self.dg.shard.shape[1])
        self.x0_pad = None
        self.work = None
        self.plan_s = 0.0
        self.plan_phases = None
        self.tiled = False
        self.timer = HopTimer()
        self.xtimer = ExchangeTimer(self.dg) if self.dg.world > 1 else None

    def prepare(self, x0: torch.Tensor, device) -> "Layout":
        self.x0_pad = self.grid.x0_table(x0)
        self.work = make_work(self.dg, self.x0_pad.shape[1], device)
        log(f"layout F={self.grid.F} x R={self.grid.R}: tables ready, planning")
        # operand re-layout for the column-ordered hop (built once, outside the timed region);
        # the uploads and table fills queued before it are drained first, so plan_s is the
        # plan's own time. Its pieces are timed in the order tiled_plan_for runs them: the
        # operand's longest row (a device reduction), the kernel's LDS grant for the block size
        # (a driver query), then the plan itself (CsrGraph.tiled_plan: device planner and its
        # sub-phases, degree factors, factor check, quad layout), each synchronised.
        shard = self.dg.shard
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        shard.max_degree()
        torch.cuda.synchronize()
        t_md = time.perf_counter()
        rpb = F._tiled_rows_per_block(shard.n_rows, device)
        F._tiled_supported(device, rpb)
        t_sup = time.perf_counter()
        plan = F.tiled_plan_for(shard, self.x0_pad)
        self.tiled = plan is not None
        torch.cuda.synchronize()
        t_end = time.perf_counter()
        self.plan_s = t_end - t1
        self.plan_phases = None
        if plan is not None:
            self.plan_phases = dict(plan["build_s"], max_degree_s=t_md - t1,
                                    kernel_lds_query_s=t_sup - t_md,
                                    tiled_plan_call_s=t_end - t_sup)
            # the same build again in this (now warm) process: what the first call's one-time
            # costs (first allocations, first use of each kernel) add to plan_s
            for k in [k for k, v in shard._plans.items() if v is plan]:
                del shard._plans[k]
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            plan2 = F.tiled_plan_for(shard, self.x0_pad)
            torch.cuda.synchronize()
            self.plan_phases["warm_rebuild_s"] = time.perf_counter() - t2
            self.plan_phases["warm_rebuild_phases"] = plan2["build_s"]
        return self

    def release(self):
        self.x0_pad = self.work = None
        self.dg.shard._plans.clear()


def hop_bytes_alg(nnz: int, rows: int, src: int, d: int) -> int:
    """SURVEY §8(d) compulsory bytes of one hop: CSR once (int64 row_ptr, int32 col, fp32 val),
    every distinct source row once, every destination row written once. G100M d=64, one
    GPU: 2.640e9 B."""
    return 8 * nnz + 8 * (rows + 1) + 4 * d * src + 4 * d * rows


def hop_bytes(nnz: int, rows: int, src: int, d: int, K: int, world: int,
              deferred: bool = False) -> list:
    """Bytes of each hop launch as the kernel is used here, fused layer-mean epilogue
    included: CSR once, every distinct source row once, then the epilogue's row transfers of
    the hop schedule (F.lightgcn_hop_schedule): the hop output unless NO_Y, the layer-mean
    inputs it reads (x0 on INIT, the acc rows on ADD, its own input rows on ACC_X) and the acc
    write. Eager (N > 1): y, acc written every hop and read from hop 2 on, rank-local x0 rows
    read on hop 1 when sharded (with one GPU they are part of the gathered table already,
    unless the deferred hop 3 reads them again as its self rows)."""
    out = []
    row = 4 * d * rows
    for k, (_, _, epi) in enumerate(F.lightgcn_hop_schedule(K, deferred), start=1):
        b = 8 * nnz + 8 * (rows + 1) + 4 * d * src
        b += row * (not (epi & EPI_NO_Y))
        if epi & (EPI_ACC_INIT | EPI_ACC_ADD):
            b += row                                           # acc write
            b += row * bool(epi & EPI_ACC_ADD)
            b += row * bool(epi & EPI_ACC_X)
            b += row * bool((epi & EPI_ACC_INIT) and (world > 1 or k > 1))
        out.append(b)
    return out


def _code_only(src: str) -> str:
    """C/C++ source without comments and blank lines: a comment edit keeps the kernel key."""
    import re
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    lines = (re.sub(r"//.*$", "", ln).rstrip() for ln in src.splitlines())
    return "\n".join(ln for ln in lines if ln)


def kernel_key(tiled_plan) -> str:
    """Identity of the hop kernel a PMC summary was measured on: SHA-256 of the kernel
    sources that build it (code only, comments stripped) and of the plan parameters the
    launch uses. A summary whose key
    differs from the running build is never reported (traffic: null)."""
    import hashlib
    h = hashlib.sha256()
    csrc = ROOT / "gnn-recommendations_amd" / "csrc"
    files = ["common.h", "tiled.hip"] if tiled_plan is not None else ["common.h", "gather.h",
                                                                      "spmm.hip"]
    for f in files + ["../../include/gnnrec.h"]:
        h.update(_code_only((csrc / f).read_text()).encode())
    if tiled_plan is not None:
        h.update(json.dumps({k: tiled_plan[k] for k in sorted(tiled_plan)
                             if isinstance(tiled_plan[k], (int, float, str))},
                            sort_keys=True).encode())
    return h.hexdigest()[:16]


def load_traffic(workload_key: str, key: str):
    """Per-launch HBM bytes from the committed PMC summary (profiles/pmc_<workload>.json) if
    it was measured on this kernel build and plan (same kernel_key), else (None, reason)."""
    p = ROOT / "profiles" / f"pmc_{workload_key}.json"
    if not p.exists():
        return None, "no PMC summary for this workload"
    try:
        d = json.loads(p.read_text())
    except Exception as e:  # noqa: BLE001
        return None, f"unreadable PMC summary: {e}"
    if d.get("kernel_key") != key:
        return None, f"PMC summary is of kernel_key {d.get('kernel_key')}, running {key}"
    return float(d["hbm_bytes_per_launch"]), p.name


def tiled_plan_info(g: CsrGraph, x: torch.Tensor):
    """The plan parameters of the hop launch (None: the CSR kernel runs)."""
    plan = F.tiled_plan_for(g, x)
    if plan is None:
        return None
    return {k: v for k, v in plan.items() if not isinstance(v, torch.Tensor)}


def cpu_baseline(g: CsrGraph, x0: torch.Tensor, K: int, n_users: int, gpu_hop1: np.ndarray,
                 gpu_out: np.ndarray, reps: int = 2) -> dict:
    """The reference's CPU path as SURVEY §8 d3 specifies it, on this host's cores, for the
    WHOLE workload:
      * graph build (graph_builder.py:16-174: scipy COO -> tocsr -> D^-1/2 A D^-1/2 -> torch
        COO) over every deduplicated pair, compared bit for bit with the GPU's operand;
      * propagation (lightgcn.py:76-95): x = cat(U, I); K x torch.sparse.mm on the
        reference-layout uncoalesced int64 COO; torch.stack(layers).mean(0), no_grad.
    One untimed warm-up hop over a 1 % row slice (thread pool / MKL start-up), then `reps`
    timed full propagations (SURVEY §8 d3 / BASELINE.md §3: >= 2 reps, the median reported,
    every sample listed; ~70 s each at 16 threads for G100M). Every rep's hop 1 and output
    are compared bit for bit with the GPU's (cpu_parity)."""
    import oracle.torch_ref as tr
    threads = host_threads()
    torch.set_num_threads(threads)
    rp = g.row_ptr.cpu().numpy()
    col = g.col.cpu().numpy()
    val = g.val.cpu().numpy()
    N = g.shape[0]
    n_items = N - n_users
    # the deduplicated pairs are the user rows of A: (u, n_users + i)
    nnz_u = int(rp[n_users])
    pu = np.repeat(np.arange(n_users, dtype=np.int64), np.diff(rp[:n_users + 1]))
    pi = col[:nnz_u].astype(np.int64) - n_users
    t0 = time.perf_counter()
    A_ref = tr.scipy_operand(pu, pi, n_users, n_items)
    t_build = time.perf_counter() - t0
    log(f"cpu: reference scipy build {t_build:.1f}s; propagating ...")
    del pu, pi
    ri = A_ref._indices()
    operand_same = bool(A_ref._nnz() == g.nnz
                        and np.array_equal(ri[1].numpy(), col.astype(np.int64))
                        and np.array_equal(np.diff(np.searchsorted(ri[0].numpy(), np.arange(N + 1))),
                                           np.diff(rp))
                        and np.array_equal(A_ref._values().numpy().view(np.uint32),
                                           val.view(np.uint32)))
    del ri
    xc = x0.detach().cpu().contiguous()
    with torch.no_grad():
        warm = tr.coo_operand(rp, col, val, N, slice(0, max(1, N // 100)))
        torch.sparse.mm(warm, xc)
        del warm
        samples, hop1_same, out_same, max_abs = [], True, True, 0.0
        for _ in range(max(1, int(reps))):
            t0 = time.perf_counter()
            layers = [xc]
            x = xc
            for _ in range(K):
                x = torch.sparse.mm(A_ref, x)
                layers.append(x)
            out = torch.stack(layers, dim=0).mean(dim=0)
            samples.append(time.perf_counter() - t0)
            log(f"cpu: rep {len(samples)}: {samples[-1]:.1f}s")
            hop1_same &= bool(np.array_equal(layers[1].numpy().view(np.uint32),
                                             gpu_hop1.view(np.uint32)))
            out_same &= bool(np.array_equal(out.numpy().view(np.uint32), gpu_out.view(np.uint32)))
            max_abs = max(max_abs, float(np.abs(out.numpy() - gpu_out).max()))
            del layers, out, x
    t = float(np.median(samples))
    del A_ref
    cpu_model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": K * g.nnz / t, "unit": "edges/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model, "seconds": t, "seconds_samples": samples,
            "statistic": f"median of {len(samples)} timed reps",
            "sample": f"the whole workload: LightGCN K={K} propagation (x0 [{N}, {xc.shape[1]}], "
                      f"{K} x torch.sparse.mm on the reference-layout uncoalesced int64 COO of "
                      f"all {g.nnz} nnz, graph_builder.py:163-172, then stack().mean(0), "
                      f"lightgcn.py:76-95), no_grad, 1 untimed warm-up hop over a 1% row "
                      f"slice then {len(samples)} timed reps (median); torch {torch.__version__} "
                      f"({torch.get_num_threads()} threads)",
            "graph_build": {"pairs": nnz_u, "seconds": t_build,
                            "what": "scipy COO -> tocsr -> D^-1/2 A D^-1/2 -> torch COO over "
                                    "every deduplicated pair (oracle/torch_ref.scipy_operand)",
                            "bit_exact_vs_gpu_operand": operand_same},
            "cpu_parity": hop1_same and out_same,
            "parity_detail": {"hop1_bit_exact": hop1_same, "output_bit_exact": out_same,
                              "output_max_abs_diff": max_abs}}


def vendor_baseline(g: CsrGraph, x0: torch.Tensor, K: int, hip_out: torch.Tensor, hip_ms: float,
                    device, reps: int = 5) -> dict:
    """The vendor comparator (SURVEY.md §8 d3 / BASELINE.md): the reference's own propagation
    call, `torch.sparse.mm(adj, x)` K times + `torch.stack(layers).mean(0)` (lightgcn.py:76-95),
    on THIS device — ATen's ROCm sparse path (hipSPARSE SpMM) — over the same operand and x0,
    outside the timed region. Two operand forms: the CSR tensor (the vendor library's best
    case) and the reference's own uncoalesced int64 COO moved to the device
    (graph_builder.py:163-172, trainer.py:233-234), which torch coalesces on every call.
    HIP events on torch's stream; 1 untimed rep, then `reps` (median). Compared with the HIP
    path's output (max |diff| and bit-exactness)."""
    N = g.shape[0]
    res = {"what": f"K={K} x torch.sparse.mm(A, x) + stack().mean(0) on {torch.cuda.get_device_name(device)}"
                   f" (torch {torch.__version__}, ATen ROCm sparse / hipSPARSE)",
           "reps": reps, "statistic": "median"}
    xd = x0.to(device)
    for form in ("csr", "coo_reference"):
        A = None
        try:
            rp = g.row_ptr.to(device)
            col = g.col.to(device).to(torch.int64)
            val = g.val.to(device)
            if form == "csr":
                A = torch.sparse_csr_tensor(rp, col, val, (N, N))
            else:
                rows = torch.repeat_interleave(torch.arange(N, device=device), rp[1:] - rp[:-1])
                A = torch.sparse_coo_tensor(torch.stack([rows, col]), val, (N, N))
                del rows
            del rp, col, val

            def prop():
                layers, x = [xd], xd
                for _ in range(K):
                    x = torch.sparse.mm(A, x)
                    layers.append(x)
                return torch.stack(layers, dim=0).mean(dim=0)
            out = prop()
            torch.cuda.synchronize()
            ms = []
            for _ in range(reps):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                o2 = prop()
                e.record()
                torch.cuda.synchronize()
                ms.append(s.elapsed_time(e))
                del o2
            t = float(np.median(ms))
            res[form] = {"ms_per_step": t, "ms_samples": ms, "edges_per_s": K * g.nnz / (t * 1e-3),
                         "max_abs_diff_vs_hip": float((out - hip_out).abs().max()),
                         "bit_exact_vs_hip": bool(torch.equal(out.view(torch.int32),
                                                              hip_out.view(torch.int32))),
                         "hip_speedup": t / hip_ms}
            del out
        except Exception as ex:  # noqa: BLE001 — recorded, not fatal to the bench line
            res[form] = {"error": f"{type(ex).__name__}: {ex}"[:400]}
        del A
        torch.cuda.empty_cache()
        log(f"vendor {form}: {res[form]}")
    return res


ROCSPARSE_ALGS = {"csr": 1, "csr_row_split": 4, "csr_nnz_split": 5, "csr_merge_path": 9}


def rocsparse_baseline(g: CsrGraph, x0: torch.Tensor, K: int, hip_out: torch.Tensor, hip_ms: float,
                       device, reps: int = 5) -> dict:
    """rocSPARSE's generic SpMM called directly (lib/libgnnrec_vendor.so, a ctypes-loaded shim
    of rocsparse_spmm; vendor/rocsparse_spmm.cpp) on the same CSR (int64 row_ptr, int32 col,
    fp32 val) and x0: K x `y = A x` + torch.stack(layers).mean(0) — the library call the
    reference's `torch.sparse.mm(adj, x)` (lightgcn.py:88) stands for, without ATen's sparse
    dispatch. Descriptors, buffer-size and preprocess stages outside the timing; every CSR
    algorithm of rocsparse_spmm timed (HIP events on torch's stream, 1 untimed rep, then
    `reps`, median), the fastest reported as `best`."""
    import ctypes
    libp = ROOT / "gnn-recommendations_amd" / "lib" / "libgnnrec_vendor.so"
    res = {"what": f"K={K} x rocsparse_spmm(CSR i64/i32 f32, row-major B/C, alpha 1, beta 0) + "
                   f"stack().mean(0)", "reps": reps, "statistic": "median"}
    try:
        lib = ctypes.CDLL(str(libp))
    except OSError as ex:
        res["error"] = f"{libp.name} not loadable: {ex}"[:300]
        return res
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    lib.vendor_spmm_create.argtypes = [ctypes.POINTER(vp), vp, vp, vp, i64, i64, i64, vp, i64, vp,
                                       i64, i64, ctypes.c_int, vp]
    lib.vendor_spmm_run.argtypes = [vp, vp, vp, vp]
    lib.vendor_spmm_destroy.argtypes = [vp]
    lib.vendor_spmm_buffer_bytes.argtypes = [vp]
    lib.vendor_spmm_buffer_bytes.restype = i64
    lib.vendor_spmm_last_error.restype = ctypes.c_char_p
    res["rocsparse_version"] = int(lib.vendor_spmm_version())
    N, d = g.shape[0], x0.shape[1]
    rp = g.row_ptr.to(device)
    col = g.col.to(device)
    val = g.val.to(device)
    xd = x0.to(device).contiguous()
    ys = [torch.empty_like(xd) for _ in range(K)]
    stream = torch.cuda.current_stream(device).cuda_stream
    best = None
    for name, alg in ROCSPARSE_ALGS.items():
        ctx = vp()
        try:
            st = lib.vendor_spmm_create(ctypes.byref(ctx), rp.data_ptr(), col.data_ptr(),
                                        val.data_ptr(), N, N, g.nnz, xd.data_ptr(), d,
                                        ys[0].data_ptr(), d, d, alg, stream)
            if st != 0:
                res[name] = {"error": lib.vendor_spmm_last_error().decode()}
                continue

            def prop():
                x = xd
                for k in range(K):
                    s = lib.vendor_spmm_run(ctx, x.data_ptr(), ys[k].data_ptr(), stream)
                    if s != 0:
                        raise RuntimeError(lib.vendor_spmm_last_error().decode())
                    x = ys[k]
                return torch.stack([xd] + ys, dim=0).mean(dim=0)
            out = prop()
            torch.cuda.synchronize()
            ms = []
            for _ in range(reps):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                o2 = prop()
                e.record()
                torch.cuda.synchronize()
                ms.append(s.elapsed_time(e))
                del o2
            t = float(np.median(ms))
            res[name] = {"ms_per_step": t, "ms_samples": ms, "edges_per_s": K * g.nnz / (t * 1e-3),
                         "buffer_bytes": int(lib.vendor_spmm_buffer_bytes(ctx)),
                         "max_abs_diff_vs_hip": float((out - hip_out).abs().max()),
                         "bit_exact_vs_hip": bool(torch.equal(out.view(torch.int32),
                                                              hip_out.view(torch.int32))),
                         "hip_speedup": t / hip_ms}
            if best is None or t < res[best]["ms_per_step"]:
                best = name
            del out
        except Exception as ex:  # noqa: BLE001 — recorded, not fatal to the bench line
            res[name] = {"error": f"{type(ex).__name__}: {ex}"[:300]}
        finally:
            torch.cuda.synchronize()
            if ctx.value:
                lib.vendor_spmm_destroy(ctx)
            torch.cuda.empty_cache()
        log(f"vendor rocsparse {name}: {res[name]}")
    res["best"] = best
    del rp, col, val, xd, ys
    torch.cuda.empty_cache()
    return res


def probe_exchange(dg, mode: str, x0_pad: torch.Tensor) -> None:
    """One exchange of `mode` on an 8-row slice of every piece (the pre-flight of a
    candidate): the same collective calls as a timed hop's exchange, on a small buffer."""
    rows = min(8, dg.rows_pad)
    d = x0_pad.shape[1]
    piece = torch.zeros((rows, d), dtype=torch.float32, device=x0_pad.device)
    out = torch.zeros((dg.world * rows, d), dtype=torch.float32, device=x0_pad.device)
    saved = (dg.exchange_mode, dg.rows_pad)
    try:
        dg.exchange_mode, dg.rows_pad = mode, rows
        dg.exchange(out, piece)
        if x0_pad.is_cuda:
            torch.cuda.synchronize()
    finally:
        dg.exchange_mode, dg.rows_pad = saved


def resolve_verify(flag, world: int) -> bool:
    """--verify / --no-verify as given; unset: on for N > 1 (the driver runs bench.py without
    flags, so its multi-GPU line checks itself), off at N = 1 (the CPU baseline already
    compares the output bit for bit with the reference's CPU path)."""
    return bool(world > 1) if flag is None else bool(flag)


def _single_device_forward(full: CsrGraph, x0: torch.Tensor, K: int, device) -> torch.Tensor:
    g1 = full.to(device)
    ref, _ = F.lightgcn_forward(g1, x0.to(device), K)
    return ref


def verify(dg, full: CsrGraph, x0, K, out, device, cols, world: int,
           reference_fn=_single_device_forward) -> dict:
    """Full-size parity: this rank's rows of the timed (possibly sharded) propagation must equal,
    bit for bit, a single-device propagation of the whole graph (the oracle itself is checked
    against that kernel in tests/, at sizes it finishes in seconds). N > 1: every rank's flag
    is MIN-reduced into `all_ranks_bit_exact` (a collective: every rank calls this).
    reference_fn(full, x0, K, device) -> [N, d]: the single-device propagation (tests inject
    the CPU oracle)."""
    ref = reference_fn(full, x0, K, device)
    mine = out
    same = torch.equal(ref[dg.row_begin:dg.row_end, cols[0]:cols[1]], mine)
    res = {"bit_exact_vs_single_device": bool(same), "rows": int(mine.shape[0])}
    del ref
    if world > 1:
        ok = torch.tensor([1 if same else 0], device=device)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        res["all_ranks_bit_exact"] = bool(ok.item())
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--pairs", type=int, default=100_000_000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-vendor", action="store_true",
                    help="skip the vendor comparator (torch.sparse.mm on the device, N = 1)")
    ap.add_argument("--cpu-reps", type=int, default=2,
                    help="timed reps of the reference CPU path (median reported)")
    ap.add_argument("--verify", action=argparse.BooleanOptionalAction, default=None,
                    help="after timing, compare this rank's rows bit for bit with a single-device "
                         "propagation of the whole graph (default: on when N > 1, so the "
                         "driver's multi-GPU line carries its own check; --no-verify skips it)")
    ap.add_argument("--exchange", default="auto", choices=["auto", "allgather", "p2p"],
                    help="per-hop exchange: allgather, bipartite point-to-point, or auto "
                         "(time both before the timed region, keep the faster)")
    ap.add_argument("--feature-groups", type=int, default=0,
                    help="N > 1: F feature groups x N/F row shards (0 = the largest F dividing "
                         "N and the d/32 feature slices; 1 = row shards only)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: test harness for several ranks sharing one GPU (host-staged "
                         "all-gather); the benchmark itself uses nccl = RCCL")
    a = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    a.verify = resolve_verify(a.verify, world)
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N > 1 needs one process per GPU: launch with "
                             "python -m torch.distributed.run --nproc-per-node N bench.py")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a ROCm GPU")
    device = torch.device("cuda", local_rank % torch.cuda.device_count())
    torch.cuda.set_device(device)
    if world > 1:
        from datetime import timedelta
        # a stuck collective fails the run after 10 minutes instead of holding the node
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device, timeout=timedelta(minutes=10))
        else:
            dist.init_process_group("gloo", timeout=timedelta(minutes=10))

    threads = max(1, host_threads() // max(1, world))
    t0 = time.perf_counter()
    full = build_graph(a.users, a.items, a.pairs, a.seed, threads)
    log(f"graph: N={full.shape[0]} nnz={full.nnz} built in {time.perf_counter() - t0:.1f}s "
        f"({threads} threads)")
    if (a.users, a.items, a.pairs, a.seed) == (1_000_000, 1_000_000, 100_000_000, 0):
        assert full.nnz == G100M_NNZ, f"G100M generator drifted: nnz={full.nnz}"
    N, d, K = full.shape[0], a.dim, a.layers

    torch.manual_seed(0)
    x0 = torch.randn(N, d, dtype=torch.float32) * 0.1  # nn.init.normal_(std=init_scale=0.1)

    # Rank layouts timed at N > 1: the default grid (F = gcd(N, d/32) feature groups x N/F
    # row shards) and, when it differs, the north star's own 1-D destination-row shards with a
    # per-hop exchange over all N ranks (F = 1). --feature-groups F > 0 pins one layout.
    if world > 1 and not a.feature_groups:
        f_default = feature_groups_for(world, d)
        layout_fs = [f_default] + ([1] if f_default != 1 else [])
    else:
        layout_fs = [a.feature_groups or None]
    layouts = []
    for fg in layout_fs:
        t0 = time.perf_counter()
        lay = Layout(full, rank, world, device, d, fg, a.exchange).prepare(x0, device)
        layouts.append(lay)
        log(f"rank {rank}: F={lay.grid.F} x R={lay.grid.R}: rows [{lay.dg.row_begin},"
            f"{lay.dg.row_end}) cols [{lay.grid.cols[0]},{lay.grid.cols[1]}) "
            f"nnz={lay.dg.shard.nnz} src={lay.src} uploaded in {time.perf_counter() - t0:.1f}s "
            f"(tiled plan {lay.plan_s:.1f}s)")
    torch.cuda.synchronize()
    cpu_graph = full if (rank == 0 and world == 1 and not a.no_cpu_baseline) else None
    vendor_graph = full if (rank == 0 and world == 1 and not a.no_vendor) else None
    verify_graph = full if a.verify else None
    del full

    cur = {"lay": layouts[0], "chunks": 1, "reserve": 0}

    def step():
        lay = cur["lay"]
        return lightgcn_propagate_dist(lay.dg, lay.x0_pad, K, hop_fn=lay.timer.hop, work=lay.work,
                                       overlap_chunks=cur["chunks"], reserve_cus=cur["reserve"],
                                       placed_output=True)

    # Exchange form (N > 1): time whole steps of each candidate (layout, exchange, overlap
    # chunks, CUs left to RCCL) before the timed region and keep the fastest (same decision on
    # every rank: max over ranks). Every candidate's ms per step, kernel ms per hop and the
    # ms per exchanged hop that the exchange holds the hop chain are reported.
    exchange_info = {"mode": "none", "overlap_chunks": 1}
    if world > 1:
        cands = []
        for li, lay in enumerate(layouts):
            dg = lay.dg
            if dg.world == 1:              # F = N: one row shard, nothing to exchange
                cands.append((li, "allgather", 1, 0))
                continue
            cc = [] if a.exchange == "p2p" else [(li, "allgather", 1, 0)]
            if not bool(dg.needs.all()) and a.exchange in ("auto", "p2p"):
                cc += [(li, "p2p", 1, 0), (li, "p2p", 4, 0), (li, "p2p", 8, 0),
                       (li, "p2p", 4, 16), (li, "p2p", 8, 16)]
            elif a.exchange == "p2p":
                cc += [(li, "p2p", 1, 0)]
            cands += cc

        def cname(c):
            lay = layouts[c[0]]
            return (f"F{lay.grid.F}xR{lay.grid.R}_" + (f"{c[1]}_x{c[2]}" if lay.dg.world > 1
                                                       else "no_exchange")
                    + (f"_r{c[3]}" if c[3] else ""))
        tried = {}
        def time_candidate(cand):
            lay = layouts[cand[0]]
            cur.update(lay=lay, chunks=cand[2], reserve=cand[3])
            lay.dg.exchange_mode = cand[1]
            step()
            torch.cuda.synchronize()
            dist.barrier()
            lay.timer.reset(True)
            if lay.xtimer is not None:
                lay.xtimer.reset(True)
            t0 = time.perf_counter()
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            dist.barrier()
            out = [(time.perf_counter() - t0) / 3 * 1e3,
                   float(np.sum(lay.timer.durations_ms())) / (3 * K),
                   (float(np.sum(lay.xtimer.durations_ms())) / (3 * max(1, K - 1))
                    if lay.xtimer is not None else 0.0)]
            lay.timer.reset(False)
            if lay.xtimer is not None:
                lay.xtimer.reset(False)
            return out

        # Pre-flight: every rank runs each (layout, exchange form) once on a small piece, in
        # lock-step, catching a form the backend rejects (it raises at the same call on every
        # rank: the calls do not depend on data); the ranks agree on the outcome (MAX) before
        # any timed collective runs.
        preflight = {}
        for key in sorted({c[:2] for c in cands if layouts[c[0]].dg.world > 1}):
            dgk = layouts[key[0]].dg
            try:
                probe_exchange(dgk, key[1], layouts[key[0]].x0_pad)
                bad = 0.0
            except Exception as ex:  # noqa: BLE001
                log(f"pre-flight {key[1]} on layout {key[0]} failed: {type(ex).__name__}: {ex}"[:300])
                bad = 1.0
            flag = torch.tensor([bad], dtype=torch.float64, device=device)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            preflight[key] = float(flag.item()) == 0.0
        for cand in cands:
            log(f"timing candidate {cname(cand)} ...")
            lay = layouts[cand[0]]
            # a candidate whose exchange form failed the pre-flight probe on any rank is
            # dropped on every rank (the flag's MAX reduction keeps the choices identical)
            if not preflight.get(cand[:2] if lay.dg.world > 1 else None, True):
                tried[cname(cand)] = {"failed": True, "why": "exchange pre-flight failed"}
                continue
            try:
                vals = time_candidate(cand)
            except Exception as ex:  # noqa: BLE001
                # past the pre-flight a failure may be on this rank only, with its peers
                # inside a collective: no collective can follow safely, so end the job (the
                # launcher tears the other ranks down) instead of hanging the node
                print(f"[bench rank {rank}] candidate {cname(cand)} failed after the "
                      f"pre-flight: {type(ex).__name__}: {ex}"[:400], file=sys.stderr, flush=True)
                os._exit(3)
            tt = torch.tensor(vals + [0.0], dtype=torch.float64, device=device)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            if float(tt[3]) > 0:
                tried[cname(cand)] = {"failed": True}
                continue
            tried[cname(cand)] = {"ms_per_step": float(tt[0]), "compute_ms_per_hop": float(tt[1]),
                                  "exchange_ms_per_hop": float(tt[2]),
                                  "recv_bytes_per_hop_per_rank":
                                      lay.dg.recv_rows() * lay.x0_pad.shape[1] * 4}
            log(f"candidate {cname(cand)}: {tried[cname(cand)]}")
        cands = [c for c in cands if not tried[cname(c)].get("failed")]
        if not cands:
            raise SystemExit("every exchange candidate failed")
        best = min(cands, key=lambda c: tried[cname(c)]["ms_per_step"])
        lay = layouts[best[0]]
        cur.update(lay=lay, chunks=best[2], reserve=best[3])
        lay.dg.exchange_mode = best[1]
        exchange_info = {"mode": best[1] if lay.dg.world > 1 else "none",
                         "overlap_chunks": best[2], "reserved_cus": best[3],
                         "chosen": cname(best), "candidates": tried}
    lay = cur["lay"]
    grid, dg, x0_pad, work, src, tiled, plan_s = (lay.grid, lay.dg, lay.x0_pad, lay.work, lay.src,
                                                  lay.tiled, lay.plan_s)
    d_loc = x0_pad.shape[1]          # this rank's feature columns (d / F)
    chunks = cur["chunks"]
    timer, xtimer = lay.timer, lay.xtimer
    for other in layouts:
        if other is not lay:
            other.release()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    timer.reset(True)
    if xtimer is not None:
        xtimer.reset(True)
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(a.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    timer.active = False
    if xtimer is not None:
        xtimer.active = False
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = elapsed / a.steps * 1e3

    durs = timer.durations_ms()
    alg_bytes = float(hop_bytes_alg(dg.shard.nnz, dg.n_local, src, d_loc))
    # column-ordered kernel: the deferred layer mean (lightgcn_propagate_dist), on shards too
    # unless the flag hop would be chunked (K > 3 with overlap chunks)
    deferred = tiled and K >= 2 and (K <= 3 or chunks == 1 or world == 1)
    per_hop = hop_bytes(dg.shard.nnz, dg.n_local, src, d_loc, K, dg.world, deferred=deferred)
    launch_bytes = float(np.mean(per_hop))
    # kernel time per hop (= per launch at N=1; the sum of its chunk launches when the hop is
    # split into overlap chunks)
    launch_ms = float(np.sum(durs)) / (a.steps * K)
    achieved = alg_bytes / (launch_ms * 1e-3) / 1e9
    achieved_fused = launch_bytes / (launch_ms * 1e-3) / 1e9

    # cross-rank totals: an edge's d features are split over the F ranks of its row shard,
    # so each rank contributes its nnz times its share of the features
    nnz_total = torch.tensor([float(dg.shard.nnz) * d_loc / d], dtype=torch.float64,
                             device=device)
    if world > 1:
        dist.all_reduce(nnz_total)
    nnz_total = float(round(nnz_total.item()))
    value = K * nnz_total / (ms_per_step * 1e-3)

    check = None
    if a.verify:
        check = verify(dg, verify_graph, x0, K, out, device, grid.cols, world)
        del verify_graph

    workload_key = f"g100m_lightgcn_k{K}_d{d}_n{world}" + ("_tiled" if tiled else "")
    kkey = kernel_key(tiled_plan_info(dg.shard, x0_pad))
    traffic, traffic_src = load_traffic(workload_key, kkey) if world == 1 else (None, "N > 1")

    vendor = None
    if vendor_graph is not None:
        log("timing the vendor comparator (torch.sparse.mm on the device) ...")
        vendor = vendor_baseline(vendor_graph, x0, K, out, ms_per_step, device)
        log("timing rocsparse_spmm called directly ...")
        vendor["rocsparse"] = rocsparse_baseline(vendor_graph, x0, K, out, ms_per_step, device)
        del vendor_graph

    cpu = None
    if cpu_graph is not None:
        # the GPU's hop 1 of the same operand and x0, for the CPU parity check
        hop1 = torch.empty_like(x0_pad)
        F.spmm_into(dg.shard, x0_pad, hop1)
        gpu_hop1 = hop1.cpu().numpy()
        gpu_out = out.cpu().numpy()
        del hop1
        log("timing the reference CPU path (scipy build + K-hop torch.sparse.mm) ...")
        cpu = cpu_baseline(cpu_graph, x0, K, a.users, gpu_hop1, gpu_out, reps=a.cpu_reps)
        del gpu_hop1, gpu_out

    # the backend that actually carried the exchange: "nccl" is RCCL on ROCm; the gloo
    # harness (several ranks sharing one GPU) stages every exchange through the host
    exchange_backend = None
    if world > 1:
        be = dist.get_backend(dg.group)
        exchange_backend = "RCCL" if be == "nccl" else f"{be} (host-staged harness, not RCCL)"
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "edges/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": f"LightGCN K={K} d={d} propagation (eval forward) on "
                            + ("G100M" if nnz_total == G100M_NNZ else f"{a.users}x{a.items} synthetic"),
                "graph": f"{a.users} users x {a.items} items, {a.pairs} pairs default_rng({a.seed}), deduplicated",
                "nnz": int(nnz_total), "n_nodes": N, "n_layers": K, "dim": d,
                "parallelism": (f"{grid.F} feature groups x " if grid.F > 1 else "")
                + f"dst-row shards x{grid.R}" + (
                    f" + per-hop {exchange_backend} exchange ({exchange_info['mode']}, "
                    f"{exchange_info['overlap_chunks']} overlap chunks"
                    + (f", {exchange_info['reserved_cus']} CUs left to RCCL"
                       if exchange_info.get('reserved_cus') else "") + ")"
                    if grid.R > 1 else ""),
                # row stride (floats) of the gathered x0 table: functional.hop_table's
                # placement on one rank, compact across ranks
                "gather_table_ld": int(x0_pad.stride(0)),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "algorithmic_bytes_per_hop": alg_bytes,
                "bytes_model": "SURVEY 8(d) B_hop = 8 nnz + 8 (rows+1) + 4 d |src| + 4 d rows",
                "achieved_with_fused_epilogue": achieved_fused,
                "frac_with_fused_epilogue": achieved_fused / HBM_PEAK_GBPS,
                "kernel_key": kkey,
                "traffic_source": traffic_src,
                "kernel": ("tiled_hop_kernel (column-ordered panels, LDS accumulators; "
                           "one launch per hop)" if tiled else
                           f"spmm_vec_kernel<{d}> (one launch per hop)"),
                "launch_ms": launch_ms,
                # per hop of the step (hop k = every K-th launch; N = 1 without chunks)
                "launch_ms_per_hop": [float(np.mean(durs[k::K])) for k in range(K)]
                if len(durs) == a.steps * K else None,
                "bytes_per_launch_with_fused_epilogue": launch_bytes,
                "layer_mean_schedule": "deferred (hop K forms the mean)"
                if deferred else "eager (every hop's epilogue)",
                # the same launch priced by its MEASURED memory-side traffic (PMC FETCH_SIZE x 2
                # + WRITE_SIZE). FETCH_SIZE counts the L2's requests to the fabric, Infinity-Cache
                # hits included (MI355X_MICROARCH.md § HBM), so this is L2->fabric traffic, an
                # upper bound of the HBM bytes — not HBM bandwidth
                "traffic_what": "L2 -> fabric bytes per launch (FETCH_SIZE incl. Infinity-Cache "
                                "hits, x2 gfx950 correction, + WRITE_SIZE)",
                "fabric_gbps": (traffic / (launch_ms * 1e-3) / 1e9) if traffic else None,
                "fabric_frac_of_hbm_peak": (traffic / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS)
                if traffic else None,
            },
            "cpu_baseline": cpu,
            "vendor": vendor,
            "operand_prep_s": {"tiled_plan_build": plan_s if tiled else None,
                               "phases": lay.plan_phases},
            "edges_per_s_per_interaction": value / 2.0,
            "hbm_gbps_algorithmic_step": K * launch_bytes * world / (ms_per_step * 1e-3) / 1e9,
            "gpu_vs_cpu": (value / cpu["value"]) if cpu else None,
            "exchange": dict(exchange_info, backend=exchange_backend,
                             recv_bytes_per_hop_per_rank=dg.recv_rows() * d_loc * 4,
                             feature_groups=grid.F, row_shards=grid.R,
                             # rank 0's compute-stream view per exchanged hop (K - 1 per step)
                             exchange_ms_per_hop=(float(np.sum(xtimer.durations_ms()))
                                                  / (a.steps * max(1, K - 1))) if xtimer else None,
                             compute_ms_per_hop=launch_ms)
            if world > 1 else None,
        }
        if check:
            line["verify"] = check
        print(json.dumps(line), flush=True)
    del out
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
