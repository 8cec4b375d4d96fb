"""Pin the CPU oracle to the reference: golden vectors made by importing the reference.

Bit-exact where the reference's arithmetic order is defined (operand values, SpMM, layer
mean, LightGCN); within the stated fp32 tolerance where the reference goes through
MKL sgemm / matrix_exp / softmax.
"""
import numpy as np
import pytest

import oracle
from conftest import golden_csr, load_golden

GRAPHS = ["g_small", "g_dup", "g_selfloop", "g_iso"]


@pytest.mark.parametrize("name", GRAPHS)
def test_operand_values_bit_exact(name):
    g = load_golden(f"graph_{name}")
    rp, col, val = oracle.normalized_graph(g["users"], g["items"], int(g["n_users"]),
                                           int(g["n_items"]), bool(g["self_loop"]))
    rows = np.repeat(np.arange(rp.size - 1), np.diff(rp))
    np.testing.assert_array_equal(rows, g["row"])
    np.testing.assert_array_equal(col, g["col"])
    assert val.dtype == np.float32
    np.testing.assert_array_equal(val.view(np.uint32), g["val"].view(np.uint32))


@pytest.mark.parametrize("K,d", [(1, 32), (2, 64), (3, 64), (3, 128)])
def test_lightgcn_bit_exact(K, d):
    f = load_golden(f"lightgcn_K{K}_d{d}")
    rp, col, val, nu, ni = golden_csr("g_small")
    x0 = np.concatenate([f["user_w"], f["item_w"]])
    out, layers = oracle.lightgcn(rp, col, val, x0, K, return_layers=True)
    for k in range(K):  # every hop: torch.sparse.mm == sequential fmaf chain
        np.testing.assert_array_equal(layers[k], f["layers"][k + 1])
    np.testing.assert_array_equal(out[:nu], f["user_out"])
    np.testing.assert_array_equal(out[nu:], f["item_out"])


def test_gas_matches_reference():
    f = load_golden("gas_d64_bs8")
    y = oracle.gas(f["x"], f["blocks"], f["perm"])
    np.testing.assert_allclose(y, f["y"], rtol=0, atol=1e-6)


def test_ngcf_matches_reference():
    f = load_golden("ngcf_d64")
    rp, col, val, nu, ni = golden_csr("g_small")
    x = np.concatenate([f["user_w"], f["item_w"]])
    outs = [x]
    for li in range(3):
        x = oracle.ngcf_layer(rp, col, val, x, f[f"W1_{li}"], f[f"b1_{li}"], f[f"W2_{li}"],
                              f[f"b2_{li}"], 0.2)
        outs.append(x)
    cat = np.concatenate(outs, axis=1)
    np.testing.assert_allclose(cat[:nu], f["user_out"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(cat[nu:], f["item_out"], rtol=0, atol=1e-5)


def test_topk_matches_reference():
    f = load_golden("topk_d64")
    idx, sc = oracle.score_topk(f["U"], f["I"], 20, f["seen_ptr"], f["seen_col"])
    ref_scores = f["scores"]
    # Scores agree to fp32 rounding (reference: MKL sgemm; oracle: sequential fmaf).
    np.testing.assert_allclose(sc, f["topk_val"], rtol=0, atol=1e-6)
    for b in range(idx.shape[0]):
        if set(idx[b]) != set(f["topk_idx"][b]):
            # only allowed at a near-tie on the boundary
            kth = np.sort(ref_scores[b])[::-1][19]
            diff = set(idx[b]) ^ set(f["topk_idx"][b])
            assert all(abs(ref_scores[b, j] - kth) < 1e-6 for j in diff)
    # the oracle's order is the fixed tie-break: score desc, index asc
    for b in range(idx.shape[0]):
        s = sc[b]
        for t in range(19):
            assert s[t] > s[t + 1] or (s[t] == s[t + 1] and idx[b, t] < idx[b, t + 1])


def _elu(x):
    return np.where(x > 0, x, np.expm1(np.minimum(x, 0))).astype(np.float32)


def gat_forward_oracle(f, rp, col):
    """GAT.forward (gat.py:258-288) composed from the oracle's per-head aggregation."""
    x = np.concatenate([f["user_w"], f["item_w"]]).astype(np.float32)
    outs = [x]
    for li in range(3):
        W, a_s, a_n = f[f"W_{li}"], f[f"a_self_{li}"], f[f"a_neigh_{li}"]
        heads = []
        for h in range(W.shape[0]):
            hh = (x.astype(np.float64) @ W[h].T.astype(np.float64)).astype(np.float32)
            ss = (hh.astype(np.float64) @ a_s[h]).astype(np.float32)
            sn = (hh.astype(np.float64) @ a_n[h]).astype(np.float32)
            heads.append(oracle.gat_head(rp, col, hh, ss, sn, 0.2))
        x = np.concatenate(heads, 1) if int(f[f"concat_{li}"]) else np.mean(np.stack(heads), 0)
        x = _elu(x.astype(np.float32))
        outs.append(x)
    return np.mean(np.stack(outs), 0)


def test_gat_matches_reference():
    f = load_golden("gat_d64_h4")
    nu, ni = int(f["n_users"]), int(f["n_items"])
    rp, col, _ = oracle.normalized_graph(f["users"], f["items"], nu, ni)
    out = gat_forward_oracle(f, rp, col)
    np.testing.assert_allclose(out[:nu], f["user_out"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(out[nu:], f["item_out"], rtol=0, atol=2e-5)


def test_scipy_operand_restatement_matches_golden():
    """oracle/torch_ref.scipy_operand (the CPU graph-build baseline) reproduces the reference's
    normalised operand values on the golden graph."""
    import oracle.torch_ref as tr
    g = load_golden("graph_g_small")
    t = tr.scipy_operand(g["users"], g["items"], int(g["n_users"]), int(g["n_items"]))
    idx, val = t._indices().numpy(), t._values().numpy()
    order = np.lexsort((idx[1], idx[0]))
    ref = np.lexsort((g["col"], g["row"]))
    np.testing.assert_array_equal(idx[0][order], g["row"][ref])
    np.testing.assert_array_equal(idx[1][order], g["col"][ref])
    np.testing.assert_array_equal(val[order].view(np.uint32), g["val"][ref].view(np.uint32))


def test_long_rows_oracle_bit_exact_vs_reference():
    """The oracle's chain order (ascending-column fmaf from +0) equals torch.sparse.mm on rows
    of up to 5 857 neighbours (config 2's graph), every layer, by SHA-256 of the fp32 bytes."""
    from conftest import long_rows_case, sha256
    f, u, i, nu, ni, x0 = long_rows_case()
    rp, col, val = oracle.normalized_graph(u, i, nu, ni)
    assert [sha256(rp), sha256(col.astype(np.int32)), sha256(val)] == list(f["operand_sha256"])
    assert int(np.diff(rp).max()) == int(f["max_degree"]) == 5857
    out, layers = oracle.lightgcn(rp, col, val, x0.numpy(), 3, return_layers=True)
    for k in range(3):
        assert sha256(layers[k]) == f["layers_sha256"][k + 1], f"hop {k + 1}"
        np.testing.assert_array_equal(layers[k][f["heavy_rows"]], f["layers_heavy"][k])
    assert sha256(out) == f["out_sha256"]
    np.testing.assert_array_equal(out, np.concatenate([f["user_out"], f["item_out"]]))
