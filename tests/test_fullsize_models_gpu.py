"""BASELINE configs 3 and 5 at the size their timings are quoted, against the oracle:

* config 3 — G100M (1M x 1M, 100M pairs, default_rng(0), 199,989,876 nnz), NGCF K=3 d=64 with
  a GAS transform after every layer, the model and seeds of tools/bench_configs.py: every layer
  of the native forward (column-ordered hop + streaming MFMA transform, the path the timed
  config takes) equals oracle.gas(oracle.ngcf_layer(...)) on the same layer input within
  1e-4 relative (ngcf.py:52-86, group_shuffle_layer.py:73-96; the oracle accumulates the two
  Linear layers in float64, so only the kernel's fp32 rounding differs).
* config 5 — the 2M x 2M power-law slice (50M Zipf-0.9 pairs + min-degree fill, 93M nnz,
  max degree ~4e5): the first (concat, head-major) and last (head-averaged, shared-row) GAT
  layer's aggregation, every head against oracle.gat_head (float64 edge softmax, gat.py:76-151),
  with the shipped heavy-row split (segments + merge) — and the fused 3-layer forward against
  the layer-by-layer composition of the same native layers.
"""
import sys

import numpy as np
import pytest
import torch

import oracle
from conftest import ROOT

from src.ops import functional as F

sys.path.insert(0, str(ROOT / "tools"))
import bench_configs  # noqa: E402

pytestmark = pytest.mark.gpu


def _rel_check(got, ref, what, rtol=1e-4, atol=1e-6):
    """allclose(rtol, atol) with the worst element reported."""
    err = np.abs(got - ref)
    bad = err > atol + rtol * np.abs(ref)
    assert not bad.any(), (f"{what}: {int(bad.sum())} elements off; max |diff| {err.max():.3g}, "
                           f"max |ref| {np.abs(ref).max():.3g}")
    return float(err.max())


def test_config3_g100m_ngcf_gas_every_layer_vs_oracle(cuda):
    import bench
    g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16)
    assert g.nnz == bench.G100M_NNZ
    gd = g.to(cuda)
    m = bench_configs.config3_model(cuda)
    x0 = m._initial_table()
    assert F.tiled_plan_for(gd, x0) is not None        # the timed path: column-ordered hop
    with torch.no_grad():
        u, i = m(gd)
    table = torch.cat([u, i]).cpu().numpy()            # cat(x0, x1, x2, x3)  [N, 256]
    del u, i
    rp, col, val = g.row_ptr.numpy(), g.col.numpy(), g.val.numpy()
    np.testing.assert_array_equal(table[:, :64], x0.detach().cpu().numpy())
    for k, (layer, gs) in enumerate(zip(m.layers, m.gs_layers)):
        x = np.ascontiguousarray(table[:, 64 * k:64 * (k + 1)])
        W1, b1, W2, b2 = (t.detach().cpu().numpy() for t in (layer.W1.weight, layer.W1.bias,
                                                             layer.W2.weight, layer.W2.bias))
        with torch.no_grad():
            blocks, perm = gs.blocks().cpu().numpy(), gs.perm.cpu().numpy()
        ref = oracle.gas(oracle.ngcf_layer(rp, col, val, x, W1, b1, W2, b2,
                                           layer.activation.negative_slope), blocks, perm)
        _rel_check(table[:, 64 * (k + 1):64 * (k + 2)], ref, f"layer {k + 1}")


@pytest.fixture(scope="module")
def slice5(cuda):
    g = bench_configs.powerlaw_graph(2_000_000, 2_000_000, 50_000_000, 0.9, 0, 16)
    deg = np.diff(g.row_ptr.numpy())
    assert deg.min() >= 1 and deg.max() > F.gat_knobs(g.n_rows)[0]
    return g, g.to(cuda), bench_configs.config5_model((2_000_000, 2_000_000), cuda)


def test_config5_slice_gat_heads_vs_oracle(cuda, slice5):
    g, gd, m = slice5
    assert gd.heavy_plan(*F.gat_knobs(gd.n_rows)) is not None
    rp, col = g.row_ptr.numpy(), g.col.numpy()
    with torch.no_grad():
        x = m._initial_table()
        xs = [x]
        for layer in m.layers[:-1]:
            xs.append(layer(xs[-1], gd, apply_elu=True))
        for which, layer in (("first", m.layers[0]), ("last", m.layers[-1])):
            xin = xs[0] if which == "first" else xs[-1]
            H = layer.n_heads
            feat, ss, sn = layer.native_inputs(xin)
            shared = layer.shares_input()
            assert shared == (which == "last")
            o = layer.in_dim if shared else layer.out_dim
            z = F.gat_aggregate(gd, feat, ss, sn, H, o, layer.alpha, mean_heads=False,
                                shared_rows=shared)
            fh, ssh, snh = feat.cpu().numpy(), ss.cpu().numpy(), sn.cpu().numpy()
            zh = z.cpu().numpy()
            del z
            for h in range(H):
                hf = fh if shared else fh[:, h * o:(h + 1) * o]
                ref = oracle.gat_head(rp, col, hf, ssh[:, h], snh[:, h], layer.alpha)
                _rel_check(zh[:, h * o:(h + 1) * o], ref, f"{which} layer, head {h}")


def test_config5_slice_fused_forward_equals_layerwise(cuda, slice5):
    """The timed forward (ELU + layer mean fused into the aggregation / head-mean epilogues)
    equals the mean of the layer-by-layer native outputs (gat.py:258-297's composition)."""
    _, gd, m = slice5
    with torch.no_grad():
        u, i = m(gd)
        x = m._initial_table()
        acc = x.clone()
        for layer in m.layers:
            x = layer(x, gd, apply_elu=True)
            acc += x
        ref = acc / float(len(m.layers) + 1)
    got = torch.cat([u, i])
    assert torch.isfinite(got).all()
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-7)


def test_config5_g250m_sampled_rows_vs_oracle(cuda):
    """Config 5 beyond the whole-graph oracle's reach: the 5M x 5M,
    250M-pair power-law graph (437M nnz, max degree ~1.5M), operand built on the device as the
    timed G1B run does. At the 16 heaviest rows plus 1024 random rows per degree decile:
    every head of the first and last layer's native aggregation (heavy split included) vs
    oracle.gat_head, every layer's output vs the reference layer on the native input, and the
    timed forward's layer mean vs the oracle layers' mean — |diff| <= 1e-5 + 1e-4 |ref|
    (oracle/gat_sample.py)."""
    from oracle.gat_sample import check_forward, sample_rows
    from src.ops.distributed import DistributedGraph, gat_forward_dist
    shape = (5_000_000, 5_000_000)
    g = bench_configs.powerlaw_graph(*shape, 250_000_000, 0.9, 0, 16, device=cuda)
    deg = (g.row_ptr[1:] - g.row_ptr[:-1]).cpu().numpy()
    assert deg.min() >= 1 and deg.max() > 1_000_000
    m = bench_configs.config5_model(shape, cuda)
    dg = DistributedGraph(g, 0, 1, cuda)
    with torch.no_grad():
        mine = gat_forward_dist(dg, m, dg.pad_table(m._initial_table()))
    rows = sample_rows(deg, n_heavy=16, per_decile=1024, seed=1)
    res = check_forward(m, g, mine, rows)
    print("\n[config5 G250M sampled]", {k: (v["max_abs_diff"] if isinstance(v, dict) else v)
                                        for k, v in res.items()})
    bad = [k for k, v in res.items() if isinstance(v, dict) and not v["within_tolerance"]]
    assert res["all_within_tolerance"], bad
    assert res["max_row_degree"] == int(deg.max())


@pytest.mark.timeout(400)
def test_config5_g1b_sampled_rows_vs_oracle(cuda):
    """Config 5 at the size its timing is quoted: the 10M x 10M power-law
    graph with 1B Zipf-0.9 pairs + min-degree fill (1,670,276,726 nnz, max degree 4,297,502),
    operand built on the device exactly as tools/bench_configs.py --g1b does; the timed
    single-device forward (gat_forward_dist on a world-1 DistributedGraph, heavy-row segments
    + merge on every layer) at the 16 heaviest rows plus 1024 random rows per degree decile:
    every head of the first and last layer's aggregation vs oracle.gat_head, every layer's
    output vs the reference layer on the native input, and the forward's layer mean vs the
    oracle layers' mean — |diff| <= 1e-5 + 1e-4 |ref| (oracle/gat_sample.py, gat.py:258-297).
    About 20 s to build and 80 s to check."""
    from oracle.gat_sample import check_forward, sample_rows
    from src.ops.distributed import DistributedGraph, gat_forward_dist
    shape = (10_000_000, 10_000_000)
    g = bench_configs.powerlaw_graph(*shape, 1_000_000_000, 0.9, 0, 16, device=cuda)
    assert g.nnz == 1_670_276_726
    deg = (g.row_ptr[1:] - g.row_ptr[:-1]).cpu().numpy()
    assert deg.min() >= 1 and int(deg.max()) == 4_297_502
    m = bench_configs.config5_model(shape, cuda)
    dg = DistributedGraph(g, 0, 1, cuda)
    with torch.no_grad():
        mine = gat_forward_dist(dg, m, dg.pad_table(m._initial_table()))
    torch.cuda.synchronize()
    rows = sample_rows(deg, n_heavy=16, per_decile=1024, seed=1)
    res = check_forward(m, g, mine, rows)
    print("\n[config5 G1B sampled]", {k: (v["max_abs_diff"] if isinstance(v, dict) else v)
                                     for k, v in res.items()})
    bad = [k for k, v in res.items() if isinstance(v, dict) and not v["within_tolerance"]]
    assert res["all_within_tolerance"], bad
    assert res["max_row_degree"] == 4_297_502
