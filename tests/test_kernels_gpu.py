"""HIP kernels vs the oracle and the reference goldens (through the C ABI).

Bit-exact: SpMM (every d, strides, epilogues), fused LightGCN. fp32 tolerance where the
reference's order is MKL's (GAS/NGCF/OB transforms): 1e-5 absolute on O(0.1) values.
"""
import numpy as np
import pytest
import torch

import oracle
from conftest import golden_csr, load_golden

from src.ops import CsrGraph, functional as F
from src.ops import _lib

pytestmark = pytest.mark.gpu


def graph_from_golden(name, device):
    rp, col, val, nu, ni = golden_csr(name)
    g = CsrGraph(torch.from_numpy(rp), torch.from_numpy(col), torch.from_numpy(val),
                 (rp.size - 1, rp.size - 1), nu, ni, symmetric=True)
    return g.to(device), (rp, col, val)


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def random_graph(n_users, n_items, n_pairs, seed, device, heavy_user=None):
    rng = np.random.default_rng(seed)
    u = rng.integers(0, n_users, n_pairs)
    i = rng.integers(0, n_items, n_pairs)
    if heavy_user is not None:  # one very long row (power-law head)
        u = np.concatenate([u, np.full(heavy_user, 0)])
        i = np.concatenate([i, rng.permutation(n_items)[:heavy_user]])
    g = CsrGraph.from_interactions(u, i, n_users, n_items)
    return g.to(device), (g.row_ptr.numpy(), g.col.numpy(), g.val.numpy())


@pytest.mark.parametrize("d", [1, 3, 8, 16, 32, 48, 64, 128, 256])
def test_spmm_bit_exact_all_dims(cuda, d):
    g, (rp, col, val) = graph_from_golden("g_small", cuda)
    x = (torch.randn(g.shape[0], d, generator=torch.Generator().manual_seed(d)) * 0.1)
    y = F.spmm_forward(g, x.to(cuda)).cpu().numpy()
    np.testing.assert_array_equal(bits(y), bits(oracle.spmm(rp, col, val, x.numpy())))


def test_spmm_strided_tables(cuda):
    g, (rp, col, val) = graph_from_golden("g_dup", cuda)
    big = torch.randn(g.shape[0], 80, device=cuda)
    x = big[:, 8:72]                       # ld 80, 16-B aligned view
    y = torch.full((g.shape[0], 96), 7.0, device=cuda)
    F.spmm_into(g, x, y[:, 16:80])
    ref = oracle.spmm(rp, col, val, x.cpu().numpy())
    np.testing.assert_array_equal(bits(y[:, 16:80].cpu().numpy()), bits(ref))
    assert torch.all(y[:, :16] == 7.0) and torch.all(y[:, 80:] == 7.0)


def test_spmm_epilogue_flags(cuda):
    g, (rp, col, val) = graph_from_golden("g_small", cuda)
    n = g.shape[0]
    x = torch.randn(n, 64, device=cuda) * 0.1
    acc = torch.empty_like(x)
    y = torch.empty_like(x)
    F.spmm_into(g, x, y, epi=_lib.EPI_ACC_INIT, self_rows=x, acc=acc)
    yr = oracle.spmm(rp, col, val, x.cpu().numpy())
    np.testing.assert_array_equal(bits(acc.cpu().numpy()), bits(x.cpu().numpy() + yr))
    acc2 = acc.clone()
    F.spmm_into(g, x, None, epi=_lib.EPI_ACC_ADD | _lib.EPI_ACC_DIV | _lib.EPI_NO_Y, acc=acc2,
                acc_div=3.0)
    np.testing.assert_array_equal(bits(acc2.cpu().numpy()),
                                  bits((acc.cpu().numpy() + yr) / np.float32(3.0)))


def test_spmm_empty_rows_and_empty_graph(cuda):
    g, (rp, col, val) = graph_from_golden("g_iso", cuda)  # isolated users/items
    assert np.any(np.diff(rp) == 0)
    x = torch.randn(g.shape[0], 64, device=cuda)
    y = F.spmm_forward(g, x).cpu().numpy()
    np.testing.assert_array_equal(bits(y), bits(oracle.spmm(rp, col, val, x.cpu().numpy())))
    assert np.all(y[np.diff(rp) == 0] == 0) and not np.signbit(y[np.diff(rp) == 0]).any()
    e = CsrGraph.from_interactions(np.zeros(0, np.int64), np.zeros(0, np.int64), 5, 3).to(cuda)
    assert torch.all(F.spmm_forward(e, torch.randn(8, 64, device=cuda)) == 0)


def test_spmm_long_rows_bit_exact(cuda):
    g, (rp, col, val) = random_graph(3000, 20000, 60000, 5, cuda, heavy_user=15000)
    assert np.diff(rp).max() >= 15000
    x = torch.randn(g.shape[0], 64, device=cuda)
    y = F.spmm_forward(g, x).cpu().numpy()
    np.testing.assert_array_equal(bits(y), bits(oracle.spmm(rp, col, val, x.cpu().numpy())))


def test_spmm_deterministic(cuda):
    g, _ = random_graph(5000, 7000, 100000, 9, cuda)
    x = torch.randn(g.shape[0], 64, device=cuda)
    a = F.spmm_forward(g, x)
    b = F.spmm_forward(g, x)
    assert torch.equal(a, b)


@pytest.mark.parametrize("K,d", [(1, 32), (2, 64), (3, 64), (3, 128)])
def test_lightgcn_fused_bit_exact_vs_reference(cuda, K, d):
    f = load_golden(f"lightgcn_K{K}_d{d}")
    g, _ = graph_from_golden("g_small", cuda)
    x0 = torch.from_numpy(np.concatenate([f["user_w"], f["item_w"]])).to(cuda)
    out, layers = F.lightgcn_forward(g, x0, K, return_layers=True)
    nu = f["user_out"].shape[0]
    out = out.cpu().numpy()
    np.testing.assert_array_equal(bits(out[:nu]), bits(f["user_out"]))
    np.testing.assert_array_equal(bits(out[nu:]), bits(f["item_out"]))
    for k in range(K):
        np.testing.assert_array_equal(bits(layers[k].cpu().numpy()), bits(f["layers"][k + 1]))
    out2, none = F.lightgcn_forward(g, x0, K)  # ping-pong buffers, NO_Y last hop
    assert none is None
    np.testing.assert_array_equal(bits(out2.cpu().numpy()), bits(out))


def test_lightgcn_zero_layers(cuda):
    g, _ = graph_from_golden("g_small", cuda)
    x0 = torch.randn(g.shape[0], 64, device=cuda)
    out, _ = F.lightgcn_forward(g, x0, 0)
    assert torch.equal(out, x0)


def test_lightgcn_backward_matches_reference(cuda):
    f = load_golden("lightgcn_grad_K3_d64")
    g, _ = graph_from_golden("g_small", cuda)
    x0 = torch.from_numpy(np.concatenate([f["user_w"], f["item_w"]])).to(cuda).requires_grad_()
    out = F.lightgcn_propagate(g, x0, 3)
    gout = torch.from_numpy(np.concatenate([f["g_u"], f["g_i"]])).to(cuda)
    (out * gout).sum().backward()
    ref = np.concatenate([f["grad_user"], f["grad_item"]])
    np.testing.assert_allclose(x0.grad.cpu().numpy(), ref, rtol=0, atol=1e-6)


def test_gas_vs_reference(cuda):
    f = load_golden("gas_d64_bs8")
    x = torch.from_numpy(f["x"]).to(cuda)
    y = F.gas(x, torch.from_numpy(f["blocks"]), torch.from_numpy(f["perm"]).to(cuda))
    np.testing.assert_allclose(y.cpu().numpy(), f["y"], rtol=0, atol=1e-6)
    np.testing.assert_array_equal(bits(y.cpu().numpy()), bits(oracle.gas(f["x"], f["blocks"], f["perm"])))


def test_spmm_gas_fused(cuda):
    f = load_golden("gas_d64_bs8")
    g, (rp, col, val) = graph_from_golden("g_small", cuda)
    x = torch.randn(g.shape[0], 64, device=cuda) * 0.1
    blocks = torch.from_numpy(f["blocks"]).to(cuda)
    perm = torch.from_numpy(f["perm"]).to(cuda)
    y = F.spmm_gas(g, x, blocks, perm).cpu().numpy()
    ref = oracle.gas(oracle.spmm(rp, col, val, x.cpu().numpy()), f["blocks"], f["perm"])
    np.testing.assert_array_equal(bits(y), bits(ref))


@pytest.mark.parametrize("fused", [False, True])
def test_ngcf_layers_vs_reference(cuda, fused):
    f = load_golden("ngcf_d64")
    g, _ = graph_from_golden("g_small", cuda)
    x = torch.from_numpy(np.concatenate([f["user_w"], f["item_w"]])).to(cuda)
    outs = [x]
    for li in range(3):
        t = lambda k: torch.from_numpy(f[f"{k}_{li}"]).to(cuda)  # noqa: E731
        x = F.ngcf_layer(g, x, t("W1"), t("b1"), t("W2"), t("b2"), 0.2, fused=fused)
        outs.append(x)
    cat = torch.cat(outs, 1).cpu().numpy()
    nu = f["user_out"].shape[0]
    np.testing.assert_allclose(cat[:nu], f["user_out"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(cat[nu:], f["item_out"], rtol=0, atol=1e-5)


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("d", [32, 64, 128])
@pytest.mark.parametrize("n_items", [900, 905])    # 905: a 5-row tail tile (rows past the end
def test_ngcf_gas_vs_oracle(cuda, d, fused, n_items):   # are loaded clamped, never stored)
    g, (rp, col, val) = random_graph(700, n_items, 9000, d, cuda)
    rng = np.random.default_rng(d)
    x = rng.standard_normal((g.shape[0], d)).astype(np.float32) * 0.1
    W1, W2 = (rng.standard_normal((2, d, d)) / np.sqrt(d)).astype(np.float32)
    b1, b2 = (rng.standard_normal((2, d)) * 0.05).astype(np.float32)
    q, _ = np.linalg.qr(rng.standard_normal((d // 8, 8, 8)))
    blocks = q.astype(np.float32)
    perm = rng.permutation(d).astype(np.int32)
    T = lambda a: torch.from_numpy(a).to(cuda)  # noqa: E731
    y = F.ngcf_layer(g, T(x), T(W1), T(b1), T(W2), T(b2), 0.2, gas_blocks=T(blocks),
                     gas_perm=T(perm), fused=fused).cpu().numpy()
    ref = oracle.gas(oracle.ngcf_layer(rp, col, val, x, W1, b1, W2, b2, 0.2), blocks, perm)
    np.testing.assert_allclose(y, ref, rtol=0, atol=1e-5)
    # the epilogue GAS (MFMA for d <= 64, VALU above) == the standalone VALU GAS kernel on
    # the un-transformed layer output, bit for bit
    plain = F.ngcf_layer(g, T(x), T(W1), T(b1), T(W2), T(b2), 0.2, fused=fused)
    np.testing.assert_array_equal(bits(y), bits(F.gas(plain, T(blocks), T(perm)).cpu().numpy()))


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("d", [32, 64, 128])
def test_dense_layer_vs_oracle(cuda, d, fused):
    g, (rp, col, val) = random_graph(500, 800, 7000, 3 * d, cuda)
    rng = np.random.default_rng(d + 1)
    x = rng.standard_normal((g.shape[0], d)).astype(np.float32) * 0.1
    xi = rng.standard_normal((g.shape[0], d)).astype(np.float32) * 0.1
    M = (rng.standard_normal((d, d)) / np.sqrt(d)).astype(np.float32)
    T = lambda a: torch.from_numpy(a).to(cuda)  # noqa: E731
    acc = torch.empty(g.shape[0], d, device=cuda)
    y = F.dense_layer(g, T(x), T(M), 0.9, T(xi), 0.1, acc=acc, acc_mode=1, w_out=0.3, w_res=0.7,
                      fused=fused)
    n = oracle.spmm(rp, col, val, x).astype(np.float64)
    ref = (np.float32(0.9) * (n @ M) + np.float32(0.1) * xi).astype(np.float32)
    np.testing.assert_allclose(y.cpu().numpy(), ref, rtol=0, atol=1e-5)
    np.testing.assert_allclose(acc.cpu().numpy(), np.float32(0.7) * xi + np.float32(0.3) * ref,
                               rtol=0, atol=1e-5)
    acc_before = acc.clone()
    F.dense_layer(g, T(x), T(M), 0.9, T(xi), 0.1, acc=acc, acc_mode=2, w_out=0.5, store_y=False,
                  fused=fused)
    np.testing.assert_allclose(acc.cpu().numpy(), (acc_before + 0.5 * y).cpu().numpy(), rtol=0,
                               atol=1e-6)


# ---- heavy-row split (workgroup-per-row, LDS double-buffered gather) ----------------------
def powerlaw_graph(seed, device, n_users=20000, n_items=6000, n_pairs=60000):
    rng = np.random.default_rng(seed)
    u = rng.integers(0, n_users, n_pairs)
    i = np.minimum(rng.zipf(1.1, n_pairs) - 1, n_items - 1)   # item rows up to ~1e4 long
    u = np.concatenate([u, np.zeros(5000, np.int64), np.full(4097, 1)])   # user rows 0/1 long
    i = np.concatenate([i, rng.permutation(n_items)[:5000], rng.permutation(n_items)[:4097]])
    g = CsrGraph.from_interactions(u, i, n_users, n_items)
    return g.to(device), (g.row_ptr.numpy(), g.col.numpy(), g.val.numpy())


@pytest.mark.parametrize("d", [4, 12, 16, 32, 64, 100, 128, 256])
def test_spmm_heavy_split_bit_exact(cuda, d):
    g, (rp, col, val) = powerlaw_graph(d, cuda)
    deg = np.diff(rp)
    assert (deg > 1024).sum() >= 3 and deg.max() > 4096
    x = torch.randn(g.shape[0], d, generator=torch.Generator().manual_seed(d)) * 0.1
    ref = bits(oracle.spmm(rp, col, val, x.numpy()))
    xd = x.to(cuda)
    for thr in (1024, 256):
        y = torch.full((g.shape[0], d), float("nan"), device=cuda)
        F.spmm_into(g, xd, y, heavy_threshold=thr)
        np.testing.assert_array_equal(bits(y.cpu().numpy()), ref)
    y0 = torch.empty_like(xd)
    F.spmm_into(g, xd, y0, heavy_threshold=0)             # no split: the same bits
    np.testing.assert_array_equal(bits(y0.cpu().numpy()), ref)


def test_spmm_heavy_split_epilogues_and_strides(cuda):
    g, (rp, col, val) = powerlaw_graph(7, cuda)
    n = g.shape[0]
    big = torch.randn(n, 80, device=cuda) * 0.1
    x = big[:, 8:72]
    xs = x.contiguous().cpu().numpy()
    yr = oracle.spmm(rp, col, val, xs)
    acc = torch.empty(n, 64, device=cuda)
    y = torch.full((n, 96), 7.0, device=cuda)
    F.spmm_into(g, x, y[:, 16:80], epi=_lib.EPI_ACC_INIT, self_rows=x, acc=acc, heavy_threshold=512)
    np.testing.assert_array_equal(bits(y[:, 16:80].cpu().numpy()), bits(yr))
    np.testing.assert_array_equal(bits(acc.cpu().numpy()), bits(xs + yr))
    acc2 = acc.clone()
    F.spmm_into(g, x, None, epi=_lib.EPI_ACC_ADD | _lib.EPI_ACC_DIV | _lib.EPI_NO_Y, acc=acc2,
                acc_div=3.0, heavy_threshold=512)
    np.testing.assert_array_equal(bits(acc2.cpu().numpy()),
                                  bits((acc.cpu().numpy() + yr) / np.float32(3.0)))


@pytest.mark.parametrize("K,d", [(3, 64), (2, 128), (3, 32)])
def test_lightgcn_heavy_split_bit_exact(cuda, K, d):
    g, (rp, col, val) = powerlaw_graph(K + d, cuda)
    x = torch.randn(g.shape[0], d, generator=torch.Generator().manual_seed(3)) * 0.1
    out, layers = F.lightgcn_forward(g, x.to(cuda), K, return_layers=True)
    out0, _ = F.lightgcn_forward(g, x.to(cuda), K, heavy_threshold=0)
    ref = oracle.lightgcn(rp, col, val, x.numpy(), K)
    np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(ref))
    np.testing.assert_array_equal(bits(out0.cpu().numpy()), bits(ref))
    assert g.heavy_rows(1024) is not None


def test_lightgcn_hipgraph_capture_replay(cuda):
    """The C ABI promises capture safety (no allocation or sync inside compute calls): the
    fused propagation, heavy-row split included, captured once and replayed gives the same
    bits as eager calls."""
    g, (rp, col, val) = powerlaw_graph(11, cuda)
    x = torch.randn(g.shape[0], 64, device=cuda) * 0.1
    ref, _ = F.lightgcn_forward(g, x, 3)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        F.lightgcn_forward(g, x, 3)              # warm the cached plans outside capture
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out, _ = F.lightgcn_forward(g, x, 3)
    x.mul_(2.0)                                  # replay reads the captured buffers anew
    graph.replay()
    ref2, _ = F.lightgcn_forward(g, x, 3)
    torch.cuda.synchronize()
    assert g.heavy_rows(256) is not None
    np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(ref2.cpu().numpy()))
    assert not torch.equal(ref, ref2)


def test_ngcf_and_dense_split_forms_on_powerlaw_equal_fused(cuda):
    """Split forms (heavy-row aware hop + transform-only kernel) == the fused kernels, bit for
    bit, on an operand with rows far above the heavy threshold."""
    g, _ = powerlaw_graph(21, cuda)
    assert g.heavy_rows(256) is not None
    torch.manual_seed(0)
    n, d = g.shape[0], 64
    x = torch.randn(n, d, device=cuda) * 0.1
    W1, W2 = torch.randn(d, d, device=cuda) * 0.1, torch.randn(d, d, device=cuda) * 0.1
    b1, b2 = torch.randn(d, device=cuda) * 0.01, torch.randn(d, device=cuda) * 0.01
    blocks = torch.linalg.qr(torch.randn(8, 8, 8, device=cuda))[0]
    perm = torch.randperm(d, device=cuda)
    a = F.ngcf_layer(g, x, W1, b1, W2, b2, 0.2, gas_blocks=blocks, gas_perm=perm, fused=False)
    b = F.ngcf_layer(g, x, W1, b1, W2, b2, 0.2, gas_blocks=blocks, gas_perm=perm, fused=True)
    np.testing.assert_array_equal(bits(a.cpu().numpy()), bits(b.cpu().numpy()))
    M = torch.randn(d, d, device=cuda) * 0.1
    acc1, acc2 = torch.zeros_like(x), torch.zeros_like(x)
    y1 = F.dense_layer(g, x, M, 0.9, x, 0.1, acc=acc1, acc_mode=1, w_out=0.3, w_res=0.2)
    y2 = F.dense_layer(g, x, M, 0.9, x, 0.1, acc=acc2, acc_mode=1, w_out=0.3, w_res=0.2, fused=True)
    np.testing.assert_array_equal(bits(y1.cpu().numpy()), bits(y2.cpu().numpy()))
    np.testing.assert_array_equal(bits(acc1.cpu().numpy()), bits(acc2.cpu().numpy()))


@pytest.mark.parametrize("K", [1, 2, 3])
def test_masked_backward_equals_dense(cuda, K):
    """lightgcn_backward (first hops skip the all-zero rows of a sparse gradient) == the dense
    propagation over A^T, bit for bit; and a masked hop == an unmasked one."""
    g, (rp, col, val) = powerlaw_graph(31 + K, cuda)
    n = g.shape[0]
    grad = torch.zeros(n, 64, device=cuda)
    rows = torch.randperm(n, device=cuda)[:50]
    grad[rows] = torch.randn(50, 64, device=cuda)
    grad[rows[0], 3] = -0.0                       # signed zeros inside a non-zero row
    dense_out, _ = F.lightgcn_forward(g.t(), grad, K)
    for mh, ah in ((None, 1), (K, K), (1, 0)):     # default, every hop masked+active, one
        sparse_out = F.lightgcn_backward(g, grad, K, masked_hops=mh, active_hops=ah)
        np.testing.assert_array_equal(bits(sparse_out.cpu().numpy()),
                                      bits(dense_out.cpu().numpy()))
    m = F.row_nonzero(grad)
    assert int(m.sum()) == 50
    y1, y2 = torch.empty_like(grad), torch.empty_like(grad)
    F.spmm_into(g, grad, y1, x_mask=m)
    F.spmm_into(g, grad, y2)
    np.testing.assert_array_equal(bits(y1.cpu().numpy()), bits(y2.cpu().numpy()))


@pytest.mark.parametrize("K,d", [(1, 64), (2, 64), (3, 64), (3, 32), (3, 128), (4, 16)])
def test_lightgcn_forward_rows_equal_full(cuda, K, d):
    """The training forward that computes only the rows a batch reads (and their
    neighbourhoods) gives the full propagation's bits at those rows, heavy rows included."""
    g, _ = powerlaw_graph(41 + K, cuda)
    n = g.shape[0]
    torch.manual_seed(K)
    x0 = torch.randn(n, d, device=cuda)
    full, _ = F.lightgcn_forward(g, x0, K)
    for n_need in (1, 40, 600):
        need = torch.zeros(n, dtype=torch.uint8, device=cuda)
        idx = torch.randperm(n, device=cuda)[:n_need]
        need[idx] = 1
        hr = g.heavy_rows(F.heavy_knobs(n, d)[0])
        if hr is not None and n_need > 1:
            need[hr[:2]] = 1
        out = F.lightgcn_forward_rows(g, x0, K, need)
        sel = need.bool()
        np.testing.assert_array_equal(bits(out[sel].cpu().numpy()), bits(full[sel].cpu().numpy()))
    # a hop restricted by y_active alone: the active rows are exact
    ya = (torch.rand(n, device=cuda) < 0.3).to(torch.uint8)
    y1, y2 = torch.empty_like(x0), torch.empty_like(x0)
    F.spmm_into(g, x0, y1, y_active=ya)
    F.spmm_into(g, x0, y2)
    sel = ya.bool()
    np.testing.assert_array_equal(bits(y1[sel].cpu().numpy()), bits(y2[sel].cpu().numpy()))


# ---- column-ordered ("tiled") hop: gnnrec_spmm_tiled_f32 ------------------------------------
@pytest.mark.parametrize("R,panel,d", [(600, 32768, 64), (37, 64, 64), (1, 1, 64),
                                       (600, 1 << 30, 64), (1117, 4096, 64), (1279, 32768, 32),
                                       (300, 2048, 128), (1277, 131072, 96)])
def test_spmm_tiled_bit_exact(cuda, R, panel, d):
    """Every 32-feature slice of every row equals the oracle's ordered fmaf chain, for plans
    from one row per block to the LDS maximum and d = 32..128 (d/32 sweeps of one plan)."""
    g, (rp, col, val) = random_graph(3000, 2500, 60000, R + panel, cuda, heavy_user=2400)
    x = torch.randn(g.shape[0], d, generator=torch.Generator().manual_seed(R)) * 0.1
    ref = bits(oracle.spmm(rp, col, val, x.numpy()))
    xd = x.to(cuda)
    plan = g.tiled_plan(rows_per_block=R, panel=panel)
    y = torch.full((g.shape[0], d), float("nan"), device=cuda)
    F.spmm_tiled_into(g, xd, y, plan)
    np.testing.assert_array_equal(bits(y.cpu().numpy()), ref)
    y.fill_(float("nan"))
    F.spmm_tiled_into(g, xd, y, plan, meet_us=0)        # no pass-start meeting: same bits
    np.testing.assert_array_equal(bits(y.cpu().numpy()), ref)
    F.spmm_tiled_into(g, xd, y, plan)                   # sync words reset per launch
    np.testing.assert_array_equal(bits(y.cpu().numpy()), ref)


def test_spmm_tiled_epilogues_strides_and_empty_rows(cuda):
    g, (rp, col, val) = random_graph(4000, 3000, 8000, 5, cuda)    # has empty rows
    assert (np.diff(rp) == 0).any()
    n = g.shape[0]
    big = torch.randn(n, 96, device=cuda) * 0.1
    x = big[:, 16:80]                                    # ldx = 96
    xs = x.contiguous().cpu().numpy()
    yr = oracle.spmm(rp, col, val, xs)
    plan = g.tiled_plan(rows_per_block=100, panel=512)
    acc = torch.empty(n, 64, device=cuda)
    y = torch.full((n, 128), 7.0, device=cuda)
    F.spmm_tiled_into(g, x, y[:, 32:96], plan, epi=_lib.EPI_ACC_INIT, self_rows=x, acc=acc)
    np.testing.assert_array_equal(bits(y[:, 32:96].cpu().numpy()), bits(yr))
    assert torch.all(y[:, :32] == 7.0) and torch.all(y[:, 96:] == 7.0)
    np.testing.assert_array_equal(bits(acc.cpu().numpy()), bits(xs + yr))
    acc2 = acc.clone()
    F.spmm_tiled_into(g, x, None, plan, epi=_lib.EPI_ACC_ADD | _lib.EPI_ACC_DIV | _lib.EPI_NO_Y,
                      acc=acc2, acc_div=3.0)
    np.testing.assert_array_equal(bits(acc2.cpu().numpy()),
                                  bits((acc.cpu().numpy() + yr) / np.float32(3.0)))


def test_spmm_tiled_rejects_bad_arguments(cuda):
    g, _ = random_graph(300, 200, 2000, 1, cuda)
    plan = g.tiled_plan()
    x = torch.zeros(g.shape[0], 48, device=cuda)
    with pytest.raises(ValueError, match="multiple of 32"):
        F.spmm_tiled_into(g, x, torch.empty_like(x), plan)
    assert F.tiled_plan_for(g, x) is None                # d = 48 stays on the CSR kernel
    with pytest.raises(ValueError, match="meet_us"):
        F.spmm_tiled_into(g, x[:, :32], torch.empty(g.shape[0], 32, device=cuda), plan,
                          meet_us=-1)
    wide = torch.zeros(g.shape[0], _lib.TILED_MAX_LDX + 32, device=cuda)[:, :32]
    with pytest.raises(ValueError, match="ldx"):
        F.spmm_tiled_into(g, wide, torch.empty(g.shape[0], 32, device=cuda), plan)


def test_spmm_tiled_table_over_4gb(cuda):
    """Gathers beyond the first 4 GB of the x table: each chunk's buffer is based at its
    panel's first source row, so lane offsets stay 32-bit (4.6 GB table, ldx = 1024)."""
    n_users, n_items = 1000, 1_130_000
    rng = np.random.default_rng(11)
    u = rng.integers(0, n_users, 40000)
    i = np.concatenate([rng.integers(0, n_items, 30000),
                        rng.integers(n_items - 100_000, n_items, 10000)])   # rows > 4 GB
    g = CsrGraph.from_interactions(u, i, n_users, n_items).to(cuda)
    n = g.shape[0]
    big = torch.empty(n, _lib.TILED_MAX_LDX, device=cuda)
    assert big.numel() * 4 > 1 << 32
    x = big[:, 64:128]
    x.copy_(torch.randn(n, 64, device=cuda, generator=torch.Generator(cuda).manual_seed(3)))
    rp, col, val = g.row_ptr.cpu().numpy(), g.col.cpu().numpy(), g.val.cpu().numpy()
    ref = bits(oracle.spmm(rp, col, val, x.cpu().numpy()))
    plan = g.tiled_plan(rows_per_block=500, panel=49152)
    y = torch.full((n, 64), float("nan"), device=cuda)
    F.spmm_tiled_into(g, x, y, plan)
    np.testing.assert_array_equal(bits(y.cpu().numpy()), ref)
    del big


def test_lightgcn_through_tiled_hop_is_bit_exact(cuda, monkeypatch):
    """The model path routes d=64 hops through the column-ordered kernel once the operand is
    large enough (here forced): every output bit equals the oracle and the CSR path."""
    g, (rp, col, val) = random_graph(6000, 5000, 150000, 9, cuda)
    x = torch.randn(g.shape[0], 64, generator=torch.Generator().manual_seed(2)) * 0.1
    ref = bits(oracle.lightgcn(rp, col, val, x.numpy(), 3))
    xd = x.to(cuda)
    monkeypatch.setattr(F, "TILED_HOP", False)
    csr, _ = F.lightgcn_forward(g, xd, 3)
    monkeypatch.setattr(F, "TILED_HOP", True)
    monkeypatch.setattr(F, "TILED_MIN_ROWS", 0)
    monkeypatch.setattr(F, "TILED_MIN_TABLE_BYTES", 0)
    assert F.tiled_plan_for(g, xd) is not None
    out, _ = F.lightgcn_forward(g, xd, 3)
    np.testing.assert_array_equal(bits(out.cpu().numpy()), ref)
    np.testing.assert_array_equal(bits(csr.cpu().numpy()), ref)
    m = torch.zeros(g.shape[0], dtype=torch.uint8, device=cuda)
    assert F.tiled_plan_for(g, xd, x_mask=m) is None     # masked hops keep the CSR kernel


@pytest.mark.parametrize("k,p", [(64, 72), (64, 8), (64, 48), (64, 64), (64, 80), (128, 64), (256, 64),
                                 (256, 12)])
def test_rows_gemm_matches_fp32_matmul(cuda, k, p):
    """gnnrec_rows_gemm_f32 (GAT projections) vs a float64 product: fp32-accumulation
    tolerance, ragged tile tails, a strided x view, and no write past p columns."""
    gen = torch.Generator().manual_seed(k + p)
    n = 16 * 37 + 5
    xb = torch.randn(n, k + 8, generator=gen)
    B = torch.randn(k, p, generator=gen) * 0.1
    ref = (xb[:, :k].double() @ B.double()).float()
    x = xb.to(cuda)[:, :k]                       # ld = k + 8
    out = torch.full((n, p + 4), 7.0, device=cuda)
    F.rows_gemm(x, B.to(cuda), out=out[:, :p])
    torch.testing.assert_close(out[:, :p].cpu(), ref, rtol=1e-5, atol=1e-5)
    assert bool((out[:, p:] == 7.0).all())
    assert F.rows_gemm(x[:0], B.to(cuda)).shape == (0, p)


def test_rows_gemm_unsupported_shapes_raise(cuda):
    """No hidden fallback: a shape without a kernel instance, a mismatched B, a tensor on
    another device or a misaligned view raises instead of running torch.matmul."""
    x = torch.randn(100, 64, device=cuda)
    with pytest.raises(NotImplementedError):
        F.rows_gemm(x, torch.randn(64, 84, device=cuda))          # p > 80 at k = 64
    with pytest.raises(NotImplementedError):
        F.rows_gemm(torch.randn(100, 32, device=cuda), torch.randn(32, 8, device=cuda))
    with pytest.raises(ValueError):
        F.rows_gemm(x, torch.randn(128, 8, device=cuda))          # B rows != k
    with pytest.raises(ValueError):
        F.rows_gemm(x, torch.randn(64, 8))                        # B on the host
    with pytest.raises(ValueError):
        F.rows_gemm(torch.randn(100, 65, device=cuda)[:, 1:], torch.randn(64, 8, device=cuda))
    assert not F.rows_gemm_supported(64, 84) and F.rows_gemm_supported(256, 64)


def test_rows_gemm_fused_gat_epilogue(cuda):
    """rows_gemm's ELU + layer-mean epilogue == the same steps in torch (GAT's last layer)."""
    from src.ops._lib import EPI_ACC_ADD, EPI_ACC_DIV, EPI_ACC_INIT, EPI_NO_Y
    gen = torch.Generator().manual_seed(5)
    n = 1000
    z = torch.randn(n, 256, generator=gen).to(cuda)
    W = (torch.randn(256, 64, generator=gen) * 0.05).to(cuda)
    base = torch.randn(n, 64, generator=gen).to(cuda)
    y_ref = torch.nn.functional.elu((z.double() @ W.double()).float())
    for epi, div in [(EPI_ACC_INIT, 1.0), (EPI_ACC_ADD | EPI_ACC_DIV, 4.0)]:
        acc = base.clone() if epi & EPI_ACC_ADD else torch.empty_like(base)
        y = F.rows_gemm(z, W, apply_elu=True, epi=epi, self_rows=base, acc=acc, acc_div=div)
        torch.testing.assert_close(y, y_ref, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(acc, (base + y) / div, rtol=0, atol=0)
    acc = base.clone()
    assert F.rows_gemm(z, W, epi=EPI_ACC_ADD | EPI_NO_Y, acc=acc) is None
    torch.testing.assert_close(acc, base + (z.double() @ W.double()).float(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("flags", ["init_add", "init_x", "add_x", "init_add_x"])
def test_spmm_tiled_multi_input_epilogues(cuda, flags):
    """ABI 6 epilogues of the column-ordered kernel: acc = ((self [+ acc]) [+ x[r]]) + y, in
    that order, then / div; acc updated in place; strided tables."""
    g, (rp, col, val) = random_graph(4000, 3000, 30000, 11, cuda)
    n = g.shape[0]
    big = torch.randn(n, 96, device=cuda) * 0.1
    x = big[:, 16:80]                                    # ldx = 96
    xs = x.contiguous().cpu().numpy()
    yr = oracle.spmm(rp, col, val, xs)
    x0 = torch.randn(n, 64, device=cuda) * 0.1
    acc_in = torch.randn(n, 64, device=cuda) * 0.1
    plan = g.tiled_plan(rows_per_block=333, panel=1024)
    epi = {"init_add": _lib.EPI_ACC_INIT | _lib.EPI_ACC_ADD,
           "init_x": _lib.EPI_ACC_INIT | _lib.EPI_ACC_X,
           "add_x": _lib.EPI_ACC_ADD | _lib.EPI_ACC_X,
           "init_add_x": _lib.EPI_ACC_INIT | _lib.EPI_ACC_ADD | _lib.EPI_ACC_X}[flags]
    terms = []
    if epi & _lib.EPI_ACC_INIT:
        terms.append(x0.cpu().numpy())
    if epi & _lib.EPI_ACC_ADD:
        terms.append(acc_in.cpu().numpy())
    if epi & _lib.EPI_ACC_X:
        terms.append(xs)
    want = terms[0]
    for t in terms[1:]:
        want = want + t
    want = want + yr
    for div in (1.0, 4.0):
        acc = acc_in.clone()
        y = torch.full((n, 64), float("nan"), device=cuda)
        F.spmm_tiled_into(g, x, y, plan, epi=epi | (_lib.EPI_ACC_DIV if div != 1.0 else 0),
                          self_rows=x0, acc=acc, acc_div=div)
        np.testing.assert_array_equal(bits(y.cpu().numpy()), bits(yr))
        w = want / np.float32(div) if div != 1.0 else want
        np.testing.assert_array_equal(bits(acc.cpu().numpy()), bits(w))


def test_csr_rejects_tiled_only_epilogues(cuda):
    g, _ = random_graph(300, 200, 2000, 1, cuda)
    x = torch.zeros(g.shape[0], 64, device=cuda)
    acc = torch.zeros_like(x)
    for epi in (_lib.EPI_ACC_INIT | _lib.EPI_ACC_X, _lib.EPI_ACC_INIT | _lib.EPI_ACC_ADD):
        with pytest.raises(Exception, match="gnnrec_spmm_tiled_f32 only"):
            F.spmm_into(g, x, torch.empty_like(x), epi=epi, self_rows=x, acc=acc)


@pytest.mark.parametrize("K", [1, 2, 3, 4, 5])
def test_lightgcn_deferred_schedule_bit_exact(cuda, monkeypatch, K):
    """lightgcn_forward through the column-ordered kernel (deferred layer mean) and the
    one-device lightgcn_propagate_dist equal the eager CSR launches (gnnrec_lightgcn_split_f32),
    bit for bit, for every K."""
    from src.ops.distributed import DistributedGraph, lightgcn_propagate_dist
    monkeypatch.setattr(F, "TILED_MIN_ROWS", 0)
    monkeypatch.setattr(F, "TILED_MIN_TABLE_BYTES", 0)
    u_i = np.random.default_rng(K)
    nu, ni = 3000, 2000
    from src.ops import CsrGraph
    full = CsrGraph.from_interactions(u_i.integers(0, nu, 40000), u_i.integers(0, ni, 40000), nu, ni)
    g = full.to(cuda)
    x0 = torch.randn(g.shape[0], 64, generator=torch.Generator().manual_seed(K)).to(cuda) * 0.1
    ref, _ = F.lightgcn_forward(g, x0, K, return_layers=True)      # CSR, eager epilogues
    assert F.tiled_plan_for(g, x0) is not None
    out, _ = F.lightgcn_forward(g, x0, K)
    assert torch.equal(bits_t(out), bits_t(ref))
    dg = DistributedGraph(full, 0, 1, cuda)
    xp = dg.pad_table(x0)
    od = lightgcn_propagate_dist(dg, xp, K)
    assert torch.equal(bits_t(od), bits_t(ref))


def bits_t(t):
    return t.contiguous().view(torch.int32)


@pytest.mark.parametrize("K", [2, 3, 4])
def test_masked_backward_deferred_mean_bit_exact(cuda, monkeypatch, K):
    """lightgcn_backward through the column-ordered kernel (forced): a masked first hop on the
    row-parallel kernel, then the deferred layer mean on the tiled hops — equal to the eager
    CSR propagation over A^T, bit for bit."""
    monkeypatch.setattr(F, "TILED_MIN_ROWS", 0)
    monkeypatch.setattr(F, "TILED_MIN_TABLE_BYTES", 0)
    g, _ = random_graph(3000, 2000, 40000, 50 + K, cuda)
    n = g.shape[0]
    grad = torch.zeros(n, 64, device=cuda)
    rows = torch.randperm(n, device=cuda)[:60]
    grad[rows] = torch.randn(60, 64, device=cuda)
    assert F.tiled_plan_for(g.t(), grad) is not None
    ref, _ = F.lightgcn_forward(g.t(), grad, K, return_layers=True)   # CSR, eager epilogues
    for mh, ah in ((None, 1), (1, 0), (2, 1)):
        out = F.lightgcn_backward(g, grad, K, masked_hops=mh, active_hops=ah)
        np.testing.assert_array_equal(bits(out.cpu().numpy()), bits(ref.cpu().numpy()),
                                      err_msg=f"masked_hops={mh} active_hops={ah}")
