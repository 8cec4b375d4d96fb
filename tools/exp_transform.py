"""Streaming MFMA transforms alone (gnnrec_ngcf_transform_f32 / gnnrec_dense_transform_f32)
on G100M-sized tables: ms per launch and streamed GB/s."""
import hashlib
import json
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
from src.ops import _lib  # noqa: E402
from src.ops._lib import check, ptr  # noqa: E402


def t_ms(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


dev = torch.device("cuda", 0)
L = _lib.lib()
st = _lib.stream_of(dev)
n = 2_000_000
res = []
for d in (64, 128):
    g = torch.Generator(device=dev).manual_seed(d)
    work = torch.randn(n, d, device=dev, generator=g)
    x = torch.randn(n, d, device=dev, generator=g)
    y = torch.empty(n, d, device=dev)
    W1, W2 = (torch.randn(d, d, device=dev, generator=g) * 0.1 for _ in range(2))
    b1, b2 = torch.zeros(d, device=dev), torch.zeros(d, device=dev)
    blocks = torch.randn(d // 8, 8, 8, device=dev, generator=g)
    perm = torch.randperm(d, device=dev, generator=g).to(torch.int32)
    for gas in (False, True):
        f = lambda: check(L.gnnrec_ngcf_transform_f32(  # noqa: E731
            n, ptr(work), d, ptr(x), d, ptr(y), d, d, ptr(W1), ptr(b1), ptr(W2), ptr(b2), 0.2,
            ptr(blocks) if gas else None, ptr(perm) if gas else None, 8 if gas else 0, st), "t")
        ms = t_ms(f)
        y1 = y.clone()
        f()
        torch.cuda.synchronize()
        # torch fp32 reference of the same layer (ngcf.py:77-84 + GAS): max |diff|
        nn_ = work @ W1.T + b1 + (x * work) @ W2.T + b2
        o = torch.where(nn_ > 0, nn_, nn_ * 0.2)
        if gas:
            z = torch.einsum("nbc,bce->nbe", o.view(n, d // 8, 8), blocks).reshape(n, d)
            o = z[:, perm.long()]
        res.append({"kind": "ngcf" + ("+gas" if gas else ""), "d": d, "ms": ms,
                    "repeat_bit_identical": bool(torch.equal(y1, y)),
                    "max_abs_diff_vs_torch_fp32": float((y - o).abs().max()),
                    "lib": os.environ.get("GNNREC_LIB", "default"),
                    "y_sha256": hashlib.sha256(y.cpu().numpy().tobytes()).hexdigest()[:16],
                    "GBps": 3 * n * d * 4 / ms / 1e6,
                    "TFLOPs": 2 * n * 2 * d * d / ms / 1e9})
    M = torch.randn(d, d, device=dev, generator=g) * 0.1
    acc = torch.zeros(n, d, device=dev)
    f = lambda: check(L.gnnrec_dense_transform_f32(  # noqa: E731
        n, ptr(work), d, ptr(y), d, d, ptr(M), 0.9, ptr(x), d, 0.1, ptr(acc), d, 2, 0.5, 0.0,
        st), "t")
    ms = t_ms(f)
    res.append({"kind": "ob(resid+acc)", "d": d, "ms": ms, "GBps": 5 * n * d * 4 / ms / 1e6,
                "TFLOPs": 2 * n * d * d / ms / 1e9})
for r in res:
    print(json.dumps(r))
