"""Scoring + mask + top-K kernel vs the oracle (bit-exact indices AND scores under the fixed
tie-break: score desc, item index asc) and vs the reference's torch.topk (sets, up to near
ties at the k-th place)."""
import numpy as np
import pytest
import torch

import oracle
from conftest import load_golden

from src.ops import score_topk

pytestmark = pytest.mark.gpu


def test_topk_golden(cuda):
    f = load_golden("topk_d64")
    U, I = torch.from_numpy(f["U"]).to(cuda), torch.from_numpy(f["I"]).to(cuda)
    idx, sc = score_topk(U, I, 20, torch.from_numpy(f["seen_ptr"]),
                         torch.from_numpy(f["seen_col"].astype(np.int32)))
    oi, osc = oracle.score_topk(f["U"], f["I"], 20, f["seen_ptr"], f["seen_col"])
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(sc.cpu().numpy().view(np.uint32), osc.view(np.uint32))
    ref = f["scores"]
    for b in range(idx.shape[0]):
        mine, theirs = set(idx[b].tolist()), set(f["topk_idx"][b].tolist())
        if mine != theirs:
            kth = np.sort(ref[b])[::-1][19]
            assert all(abs(ref[b, j] - kth) < 1e-6 for j in mine ^ theirs)


@pytest.mark.parametrize("k,d", [(1, 64), (20, 64), (50, 32), (128, 128), (7, 16)])
def test_topk_random_with_ties_and_masks(cuda, k, d):
    rng = np.random.default_rng(k * 1000 + d)
    nb, n_items = 150, 3000
    U = (rng.standard_normal((nb, d)) * 0.1).astype(np.float32)
    I = (rng.standard_normal((n_items, d)) * 0.1).astype(np.float32)
    I[100:140] = I[7]                      # 41 identical items: exact score ties
    U[3] = 0.0                             # a user whose scores are all 0 -> pure index order
    lists = [np.unique(rng.integers(0, n_items, rng.integers(0, 60))) for _ in range(nb)]
    lists[5] = np.arange(n_items - 3)      # almost everything seen: -inf entries reach top-k
    seen_ptr = np.cumsum([0] + [len(l) for l in lists]).astype(np.int64)
    seen_col = np.concatenate(lists).astype(np.int32)
    idx, sc = score_topk(torch.from_numpy(U).to(cuda), torch.from_numpy(I).to(cuda), k,
                         torch.from_numpy(seen_ptr), torch.from_numpy(seen_col))
    oi, osc = oracle.score_topk(U, I, k, seen_ptr, seen_col)
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(sc.cpu().numpy().view(np.uint32), osc.view(np.uint32))


def test_topk_fewer_items_than_k(cuda):
    U = torch.randn(5, 32, device=cuda)
    I = torch.randn(10, 32, device=cuda)
    idx, sc = score_topk(U, I, 16)
    oi, osc = oracle.score_topk(U.cpu().numpy(), I.cpu().numpy(), 16)
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    assert (idx[:, 10:] == -1).all() and torch.isinf(sc[:, 10:]).all()


def test_evaluator_native_matches_cpu_path(cuda):
    from src.data.dataset import RecommendationDataset
    from src.evaluation import Evaluator
    from src.models import LightGCN
    ds = RecommendationDataset.synthetic_movielens(n_users=300, n_items=500, n_ratings=8000)
    torch.manual_seed(0)
    m = LightGCN(ds.n_users, ds.n_items, embedding_dim=64, n_layers=2, init_scale=0.1)
    cpu = Evaluator(device=torch.device("cpu")).evaluate(m, ds)
    gpu = Evaluator(device=cuda).evaluate(m.to(cuda), ds)
    assert cpu.keys() == gpu.keys()
    for k in cpu:  # same embeddings; only near-tie order between MKL and fmaf scores may move
        assert abs(cpu[k] - gpu[k]) < 5e-3, (k, cpu[k], gpu[k])


@pytest.mark.parametrize("model", ["lightgcn", "ngcf", "ngcf_gs", "orthogonal_bundle", "gat"])
def test_run_all_on_gpu(cuda, model, tmp_path):
    import importlib.util
    import json
    from conftest import PKG
    spec = importlib.util.spec_from_file_location("run_all", PKG / "run_all.py")
    ra = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ra)
    out = tmp_path / "r.json"
    rc = ra.main(["--quick", "--skip-check", "--models", model, "--epochs", "1",
                  "--device", "cuda", "--output", str(out)])
    res = json.loads(out.read_text())
    assert rc == 0, res
    assert res[0]["status"] == "success"


@pytest.mark.parametrize("n_split", [1, 2, 3, 7, 40])
@pytest.mark.parametrize("k,d", [(20, 64), (128, 32), (5, 256)])
def test_topk_item_split_is_exact(cuda, n_split, k, d):
    """The item-range split + merge (gnnrec_score_topk_split_f32) returns the same bits as the
    oracle, with exact ties across range boundaries, masks and fewer items than k in a range."""
    rng = np.random.default_rng(n_split * 7 + k)
    nb, n_items = 130, 2600
    U = (rng.standard_normal((nb, d)) * 0.1).astype(np.float32)
    I = (rng.standard_normal((n_items, d)) * 0.1).astype(np.float32)
    I[1000:1300] = I[5]                    # ties spanning several ranges
    lists = [np.unique(rng.integers(0, n_items, rng.integers(0, 80))) for _ in range(nb)]
    lists[3] = np.arange(n_items - 2)
    seen_ptr = np.cumsum([0] + [len(l) for l in lists]).astype(np.int64)
    seen_col = np.concatenate(lists).astype(np.int32)
    idx, sc = score_topk(torch.from_numpy(U).to(cuda), torch.from_numpy(I).to(cuda), k,
                         torch.from_numpy(seen_ptr), torch.from_numpy(seen_col), n_split=n_split)
    oi, osc = oracle.score_topk(U, I, k, seen_ptr, seen_col)
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(sc.cpu().numpy().view(np.uint32), osc.view(np.uint32))
