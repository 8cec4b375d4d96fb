"""GAT training on the native operand (gnnrec_gat_train_forward_f32 / _backward_f32).

* Every parameter gradient of the reference GAT (gat.py:76-151, 258-297; loss = sum(u_out Ru)
  + sum(i_out Ri), dropout 0) from tests/golden/gat_grad_d64_h4.npz — made by importing the
  reference — against the native differentiable path.
* Attention dropout: the kernels' counter-based keep mask, rebuilt here with the same hash,
  applied to a dense torch restatement of the layer: outputs and gradients agree, and the
  mask is the same in the forward and both backward passes.
* The native path runs no [N, N] buffer and trains above the old dense-fallback bound.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from src.models import GAT
from src.ops import CsrGraph
from src.ops import functional as F

pytestmark = pytest.mark.gpu


def _close(got, ref, what, rel=1e-4):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    err = np.abs(got - ref).max()
    scale = np.abs(ref).max()
    assert err <= rel * scale + 1e-7, f"{what}: max |diff| {err:.3g} vs max |ref| {scale:.3g}"


def test_gat_train_gradients_match_reference(cuda):
    f = load_golden("gat_grad_d64_h4")
    nu, ni = int(f["n_users"]), int(f["n_items"])
    g = CsrGraph.from_interactions(f["users"], f["items"], nu, ni).to(cuda)
    torch.manual_seed(42)
    m = GAT(nu, ni, embedding_dim=64, n_layers=3, n_heads=4, dropout=0.0, alpha=0.2,
            init_scale=0.1).to(cuda).train()
    for name, prm in m.named_parameters():       # the reference's seeded parameters
        np.testing.assert_array_equal(prm.detach().cpu().numpy(), f["param." + name])
    assert all(layer.train_ok(g) for layer in m.layers)
    torch.cuda.reset_peak_memory_stats(cuda)
    ue, ie = m(g)
    loss = (ue * torch.from_numpy(f["Ru"]).to(cuda)).sum() + \
        (ie * torch.from_numpy(f["Ri"]).to(cuda)).sum()
    loss.backward()
    _close(ue.detach().cpu().numpy(), f["user_out"], "user_out")
    _close(ie.detach().cpu().numpy(), f["item_out"], "item_out")
    assert abs(loss.item() - float(f["loss"])) <= 1e-4 * abs(float(f["loss"])) + 1e-6
    for name, prm in m.named_parameters():
        _close(prm.grad.cpu().numpy(), f["grad." + name], name)


def _keep_mask(rows, cols, head, seed, p):
    """numpy restatement of gat_train.hip's drop_keep (test-only mirror of the kernel hash)."""
    M = np.uint64(0xFFFFFFFF)
    r = rows.astype(np.uint64)
    j = cols.astype(np.uint64)
    x = np.uint64(seed) ^ ((r * np.uint64(0x9E3779B1)) & M) ^ (((r >> np.uint64(32)) * np.uint64(0x7FEB352D)) & M)
    x &= M
    x ^= (((j * np.uint64(0x85EBCA77)) & M) + (((j >> np.uint64(32)) * np.uint64(0x846CA68B)) & M)) & M
    x ^= (np.uint64(head) * np.uint64(0xC2B2AE3D)) & M
    x &= M
    x ^= x >> np.uint64(16); x = (x * np.uint64(0x7FEB352D)) & M
    x ^= x >> np.uint64(15); x = (x * np.uint64(0x846CA68B)) & M
    x ^= x >> np.uint64(16)
    u = (x >> np.uint64(8)).astype(np.float64) / 16777216.0
    return np.where(u >= p, 1.0 / (1.0 - p), 0.0).astype(np.float32)


@pytest.mark.parametrize("heads,o", [(4, 16), (2, 32), (1, 64)])
def test_gat_train_dropout_matches_dense_with_the_same_mask(cuda, heads, o):
    rng = np.random.default_rng(8)
    nu, ni = 70, 90
    u = np.concatenate([np.arange(nu), rng.integers(0, nu, ni), rng.integers(0, nu, 900)])
    i = np.concatenate([rng.integers(0, ni, nu), np.arange(ni), rng.integers(0, ni, 900)])
    g = CsrGraph.from_interactions(u, i, nu, ni)
    gd = g.to(cuda)
    n = g.shape[0]
    p, seed = 0.3, 12345
    torch.manual_seed(1)
    h = (torch.randn(n, heads * o) * 0.5).requires_grad_()
    ss = (torch.randn(n, heads) * 0.5).requires_grad_()
    sn = (torch.randn(n, heads) * 0.5).requires_grad_()
    R = torch.randn(n, heads * o)
    # native
    hd, ssd, snd = (t.detach().to(cuda).requires_grad_() for t in (h, ss, sn))
    out = F.gat_aggregate_train(gd, hd, ssd, snd, heads, o, 0.2, p, seed)
    (out * R.to(cuda)).sum().backward()
    # dense restatement with the kernels' mask
    rp, col = g.row_ptr.numpy(), g.col.numpy()
    rows = np.repeat(np.arange(n), np.diff(rp))
    ref_parts = []
    for q in range(heads):
        keep = torch.zeros(n, n)
        keep[rows, col] = torch.from_numpy(_keep_mask(rows, col, q, seed, p))
        mask = torch.zeros(n, n, dtype=torch.bool)
        mask[rows, col] = True
        z = ss[:, q:q + 1] + sn[:, q:q + 1].t()
        e = torch.nn.functional.leaky_relu(z, 0.2).masked_fill(~mask, float("-inf"))
        att = torch.softmax(e, dim=1) * keep
        ref_parts.append(att @ h[:, q * o:(q + 1) * o])
    ref = torch.cat(ref_parts, dim=1)
    (ref * R).sum().backward()
    _close(out.detach().cpu().numpy(), ref.detach().numpy(), "out")
    _close(hd.grad.cpu().numpy(), h.grad.numpy(), "dh")
    _close(ssd.grad.cpu().numpy(), ss.grad.numpy(), "d s_self")
    _close(snd.grad.cpu().numpy(), sn.grad.numpy(), "d s_neigh")
    # the kept fraction is 1 - p
    kept = np.mean([_keep_mask(rows, col, q, seed, p) > 0 for q in range(heads)])
    assert abs(kept - (1 - p)) < 0.05


def test_gat_trains_natively_above_the_dense_bound(cuda):
    """A 200K-node graph (the reference's dense path would need ~2 TB with autograd): one
    BPR-style training step through the native backward, finite gradients, no [N, N] buffer;
    a second step lowers the loss."""
    nu = ni = 100_000
    rng = np.random.default_rng(0)
    u = np.concatenate([np.arange(nu), rng.integers(0, nu, ni), rng.integers(0, nu, 4 * nu)])
    i = np.concatenate([rng.integers(0, ni, nu), np.arange(ni), rng.integers(0, ni, 4 * nu)])
    g = CsrGraph.from_interactions(u, i, nu, ni).to(cuda)
    torch.manual_seed(0)
    m = GAT(nu, ni, embedding_dim=64, n_layers=3, n_heads=4, dropout=0.1).to(cuda).train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    bu = torch.randint(0, nu, (2048,), device=cuda)
    bi = torch.randint(0, ni, (2048,), device=cuda)
    losses = []
    torch.cuda.reset_peak_memory_stats(cuda)
    base = torch.cuda.memory_allocated(cuda)
    for _ in range(3):
        torch.manual_seed(7)                      # the same dropout masks each step
        ue, ie = m(g)
        loss = -(torch.nn.functional.logsigmoid((ue[bu] * ie[bi]).sum(-1))).mean()
        opt.zero_grad()
        loss.backward()
        assert all(torch.isfinite(p.grad).all() for p in m.parameters())
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0]
    assert torch.cuda.max_memory_allocated(cuda) - base < (nu + ni) ** 2    # no [N, N]


@pytest.mark.parametrize("heads,o", [(4, 16), (4, 64), (1, 64)])
def test_gat_train_heavy_split_matches_unsplit(cuda, heads, o):
    """rows above GAT_TRAIN_HEAVY_THRESHOLD run as merged segments in the forward,
    the backward row pass and the column pass (gnnrec_gat_train_*_split_f32). On a power-law
    graph with rows of thousands of neighbours, forced to split at 64 / 32-edge segments, the
    output and all three input gradients equal the unsplit kernels' within fp32 reassociation,
    with attention dropout."""
    rng = np.random.default_rng(21)
    nu, ni, n_pairs = 3000, 2000, 60000
    u = np.concatenate([np.arange(nu), rng.integers(0, nu, ni), rng.zipf(1.5, n_pairs) % nu])
    i = np.concatenate([rng.integers(0, ni, nu), np.arange(ni), rng.zipf(1.4, n_pairs) % ni])
    g = CsrGraph.from_interactions(u, i, nu, ni).to(cuda)
    n = g.n_rows
    assert g.max_degree() > 1000
    torch.manual_seed(3)
    h0 = torch.randn(n, heads * o, device=cuda) * 0.5
    ss0 = torch.randn(n, heads, device=cuda) * 0.5
    sn0 = torch.randn(n, heads, device=cuda) * 0.5
    R = torch.randn(n, heads * o, device=cuda)
    res = {}
    saved = F.GAT_TRAIN_HEAVY_THRESHOLD, F.GAT_TRAIN_SEGMENT
    try:
        for name, (thr, seg) in {"unsplit": (0, 1024), "split": (64, 32)}.items():
            F.GAT_TRAIN_HEAVY_THRESHOLD, F.GAT_TRAIN_SEGMENT = thr, seg
            h, ss, sn = (t.clone().requires_grad_() for t in (h0, ss0, sn0))
            out = F.gat_aggregate_train(g, h, ss, sn, heads, o, 0.2, 0.3, 99)
            (out * R).sum().backward()
            res[name] = [t.detach().cpu().numpy() for t in (out, h.grad, ss.grad, sn.grad)]
    finally:
        F.GAT_TRAIN_HEAVY_THRESHOLD, F.GAT_TRAIN_SEGMENT = saved
    for what, a, b in zip(("out", "dh", "d s_self", "d s_neigh"), res["split"], res["unsplit"]):
        assert np.isfinite(a).all(), what
        _close(a, b, what, rel=1e-5)
