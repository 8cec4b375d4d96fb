"""Degree factors of factored column-ordered plans (CsrGraph.degree_factors, host side): for a
binary interaction graph every stored value is fl(row_factor[r] * class_table[col_class[c]])
bit for bit — the builder's fl(dis_r * dis_c) (graph_builder.py:119-126) — on the full graph,
on every row shard (columns in the padded gather layout) and on row-slice views; operands
that are not such products (multiplicities) are caught by that check."""
import numpy as np
import pytest

from src.ops import CsrGraph


def _graph(binary=True, seed=0):
    rng = np.random.default_rng(seed)
    nu, ni, n = 700, 500, 12000
    return CsrGraph.from_interactions(rng.integers(0, nu, n), rng.integers(0, ni, n), nu, ni,
                                      binary=binary)


def _products_match(g, f):
    rowf, cc, table = (t.numpy() for t in f)
    rp, col, val = g.row_ptr.numpy(), g.col.numpy(), g.val.numpy()
    rows = np.repeat(np.arange(rp.size - 1), np.diff(rp))   # row_ptr: absolute offsets
    v = rowf[rows] * table[cc[col[rp[0]:rp[-1]]]]
    return np.array_equal(v.astype(np.float32).view(np.uint32),
                          val[rp[0]:rp[-1]].view(np.uint32))


def test_full_graph_factors_reproduce_values():
    g = _graph()
    f = g.degree_factors()
    assert f is not None and f[2].numel() <= 256
    assert _products_match(g, f)


@pytest.mark.parametrize("world", [2, 3])
def test_shard_factors_in_padded_layout(world):
    g = _graph()
    for rank in range(world):
        s = g.shard(rank, world)
        f = s.degree_factors()
        assert f is not None
        assert f[0].numel() == s.n_rows and f[1].numel() == s.shape[1]
        assert _products_match(s, f)
        v = s.row_slice(3, max(4, s.n_rows - 5))
        assert _products_match(v, v.degree_factors())


def test_world1_shard_guesses_its_own_factors():
    g = _graph()
    s = g.shard(0, 1)
    assert _products_match(s, s.degree_factors())


def test_multiplicities_are_not_products():
    g = _graph(binary=False)
    f = g.degree_factors()
    # the guess (row counts) exists but does not reproduce the summed-duplicate values
    assert f is not None and not _products_match(g, f)
