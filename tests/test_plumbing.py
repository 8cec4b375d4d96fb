"""Host plumbing around the path (CPU): the graph_builder API, dataset split, run_all.py."""
import json

import numpy as np
import pandas as pd
import pytest
import torch

from conftest import PKG, load_golden

from src.data import (build_bipartite_graph, build_csr_graph, convert_to_torch_sparse,
                      load_adjacency_matrix, normalize_adjacency_matrix, save_adjacency_matrix)
from src.data.dataset import RecommendationDataset
from src.evaluation import compute_metrics_from_topk


@pytest.mark.parametrize("name", ["g_small", "g_dup", "g_selfloop"])
def test_graph_builder_api_matches_reference(name, tmp_path):
    g = load_golden(f"graph_{name}")
    df = pd.DataFrame({"userId": g["users"], "itemId": g["items"]})
    adj = build_bipartite_graph(df, int(g["n_users"]), int(g["n_items"]),
                                self_loop=bool(g["self_loop"]))
    norm = normalize_adjacency_matrix(adj)
    np.testing.assert_array_equal(norm.row, g["row"])
    np.testing.assert_array_equal(norm.col, g["col"])
    np.testing.assert_array_equal(norm.data.view(np.uint32), g["val"].view(np.uint32))
    t = convert_to_torch_sparse(norm)
    assert t.dtype == torch.float32 and t._indices().dtype == torch.int64 and not t.is_coalesced()
    for fmt in ("npz", "pt"):
        p = str(tmp_path / f"a.{fmt}")
        save_adjacency_matrix(norm, p, fmt)
        back = load_adjacency_matrix(p, fmt).tocsr()
        assert (abs(back - norm.tocsr()) > 0).nnz == 0
    G = build_csr_graph(df, int(g["n_users"]), int(g["n_items"]), self_loop=bool(g["self_loop"]))
    np.testing.assert_array_equal(G.val.numpy().view(np.uint32), g["val"].view(np.uint32))


def test_temporal_split_rules():
    r = pd.DataFrame({"userId": [1, 1, 1, 1, 2, 2, 3] * 1, "itemId": [10, 11, 12, 13, 10, 11, 12],
                      "rating": [5] * 7, "timestamp": [4, 1, 3, 2, 9, 8, 1]})
    ds = RecommendationDataset.from_ratings(r, min_user=1, min_item=1)
    # user 1 (4 items): last (t=4, item 10) test, t=3 (item 12) valid, rest train
    assert len(ds.test_data) == 2 and len(ds.valid_data) == 1
    assert len(ds.train_data) == 4
    assert ds.n_users == 3 and ds.n_items == 4


def test_metrics_from_topk():
    topk = np.array([[0, 1, 2], [3, 4, 5]])
    m = compute_metrics_from_topk(topk, [0, 1], {0: [1], 1: [9]}, n_items=10, k_values=[2])
    assert m["recall@2"] == 0.5 and m["precision@2"] == 0.25
    assert abs(m["ndcg@2"] - 0.5 * (1 / np.log2(3))) < 1e-12


def test_run_all_config1_cpu(tmp_path):
    """BASELINE config 1: LightGCN K=1 d=32 on the ML-100K shape through run_all.py (CPU)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("run_all", PKG / "run_all.py")
    ra = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ra)
    out = tmp_path / "r.json"
    rc = ra.main(["--quick", "--skip-check", "--models", "lightgcn", "--n_layers", "1",
                  "--embedding_dim", "32", "--device", "cpu", "--epochs", "1",
                  "--output", str(out)])
    res = json.loads(out.read_text())
    assert rc == 0 and res[0]["status"] == "success"
    assert 0.0 <= res[0]["test_metrics"]["recall@10"] <= 1.0


def test_embedding_statistics_match_reference():
    """mcs / mad / variance that Evaluator.evaluate adds (evaluator.py:116-121), against the
    reference's own metric functions (tests/golden/emb_stats.npz); mad also through the
    sampled path's chunking (exact_limit above N)."""
    import torch
    from conftest import load_golden
    from src.evaluation import embedding_statistics
    f = load_golden("emb_stats")
    st = embedding_statistics(torch.from_numpy(f["emb"]), chunk=128)
    assert abs(st["mcs"] - float(f["mcs"])) < 1e-6
    assert abs(st["mad"] - float(f["mad"])) < 1e-5 * float(f["mad"])
    assert abs(st["variance"] - float(f["variance"])) < 1e-6 * float(f["variance"])
    assert "mad_sampled" not in st
    st2 = embedding_statistics(torch.from_numpy(f["emb"]), exact_limit=300)
    assert st2["mad_sampled"] == 300.0 and abs(st2["mcs"] - st["mcs"]) < 1e-12
    # the user / item halves as two parts, statistics over small row chunks: no concatenated
    # copy, same values (float64 sums reassociated)
    e = torch.from_numpy(f["emb"])
    h = e.shape[0] // 3
    st3 = embedding_statistics((e[:h], e[h:]), chunk=128, stat_rows=37)
    for key in ("mcs", "mad", "variance"):
        assert abs(st3[key] - st[key]) <= 1e-9 * max(1.0, abs(st[key])), key
    st4 = embedding_statistics((e[:h], e[h:]), exact_limit=300, stat_rows=37)
    assert st4["mad"] == st2["mad"]


def test_bench_cpu_baseline_leg_checks_parity():
    """bench.py's cpu_baseline leg on a small graph: the scipy build equals the
    native operand bit for bit, and hop 1 / the output compare bit-exact against the oracle
    standing in for the GPU's arrays; a perturbed GPU output is reported as a mismatch."""
    import numpy as np
    import torch
    import bench
    import oracle
    from src.ops import CsrGraph
    g = bench.build_graph(300, 500, 6000, 3, 2)
    torch.manual_seed(0)
    x0 = torch.randn(800, 64) * 0.1
    rp, col, val = g.row_ptr.numpy(), g.col.numpy(), g.val.numpy()
    out, layers = oracle.lightgcn(rp, col, val, x0.numpy(), 3, return_layers=True)
    res = bench.cpu_baseline(g, x0, 3, 300, layers[0], out)
    assert res["graph_build"]["bit_exact_vs_gpu_operand"] is True
    assert res["cpu_parity"] is True and res["value"] > 0
    bad = out.copy()
    bad[7, 3] = np.nextafter(bad[7, 3], np.float32(1))
    res = bench.cpu_baseline(g, x0, 3, 300, layers[0], bad)
    assert res["cpu_parity"] is False and res["parity_detail"]["hop1_bit_exact"] is True


def test_heavy_plan_equal_segments():
    """CsrGraph.heavy_plan: every row above the threshold is covered by contiguous segments
    of equal length (one edge apart at most), none longer than seg_len."""
    import numpy as np
    import torch
    from src.ops import CsrGraph
    rng = np.random.default_rng(1)
    u = np.concatenate([rng.integers(0, 500, 20000), np.zeros(2500, np.int64)])
    i = np.concatenate([np.minimum(rng.zipf(1.3, 20000) - 1, 2999), np.arange(2500)])
    g = CsrGraph.from_interactions(u, i, 500, 3000, binary=True)
    rp = g.row_ptr
    deg = rp[1:] - rp[:-1]
    for thr, seg in ((200, 100), (64, 64), (1000, 333)):
        p = g.heavy_plan(thr, seg)
        assert torch.equal(p["heavy_rows"], torch.nonzero(deg > thr).flatten())
        sp = p["heavy_seg_ptr"].tolist()
        for h, r in enumerate(p["heavy_rows"].tolist()):
            a, b = sp[h], sp[h + 1]
            assert b - a == -(-int(deg[r]) // seg)
            assert (p["seg_row"][a:b] == r).all()
            assert int(p["seg_beg"][a]) == int(rp[r]) and int(p["seg_end"][b - 1]) == int(rp[r + 1])
            assert torch.equal(p["seg_beg"][a + 1:b], p["seg_end"][a:b - 1])
            L = p["seg_end"][a:b] - p["seg_beg"][a:b]
            assert int(L.max()) - int(L.min()) <= 1 and int(L.max()) <= seg
