"""The weight gradient of a 64 x 64 nn.Linear over N rows (NGCF training's W1 / W2:
dW = dY^T X, a 64 x 64 output with an N-long reduction) as torch runs it (one GEMM: two
output tiles walk all N rows) against a split-K form (N cut into C chunks, one batched GEMM,
then a sum over the chunks). Median ms and the max |difference|.

    python tools/exp_linear_dw.py
"""
import json

import torch

dev = torch.device("cuda", 0)


def ms_of(fn, reps=50):
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


def split_k(dy, x, chunk):
    n = dy.shape[0]
    c = n // chunk
    main = torch.bmm(dy[:c * chunk].view(c, chunk, -1).transpose(1, 2),
                     x[:c * chunk].view(c, chunk, -1)).sum(0)
    if c * chunk < n:
        main = main + dy[c * chunk:].t() @ x[c * chunk:]
    return main


for n in (9746, 200_000, 2_000_000):
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(n, 64, device=dev, generator=g)
    dy = torch.randn(n, 64, device=dev, generator=g)
    ref64 = (dy.double().t() @ x.double())
    t0, w0 = ms_of(lambda: dy.t() @ x)
    rec = {"n": n, "torch_mm_ms": t0, "torch_err": (w0.double() - ref64).abs().max().item()}
    for chunk in (256, 1024, 4096):
        t, w = ms_of(lambda: split_k(dy, x, chunk))
        rec[f"splitk{chunk}_ms"] = t
        rec[f"splitk{chunk}_err"] = (w.double() - ref64).abs().max().item()
    print(json.dumps(rec), flush=True)
