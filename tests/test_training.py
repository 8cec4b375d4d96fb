"""§8f1 training path: the reference's sampler RNG order, the [B, B] BPR broadcast, and three
Adam steps of LightGCN against goldens made by running the reference trainer's own code
(tests/golden/make_golden.py). CPU here; the native (GPU) variant is in test_training_gpu."""
import numpy as np
import pytest
import torch

from conftest import golden_csr, load_golden

from src.models import LightGCN
from src.ops import CsrGraph
from src.training import (BPRLoss, DeviceSampler, ReferenceSampler, Trainer, bpr_scores, make_adam,
                          train_step)


def _golden_graph():
    rp, col, val, nu, ni = golden_csr("g_small")
    g = CsrGraph(torch.from_numpy(rp), torch.from_numpy(col), torch.from_numpy(val),
                 (rp.size - 1, rp.size - 1), nu, ni, True)
    return g, nu, ni


def test_reference_sampler_matches_reference_rng_stream():
    f = load_golden("bpr_train_K3_d64")
    gg = load_golden("graph_g_small")
    pairs = list(zip(gg["users"].tolist(), gg["items"].tolist()))
    s = ReferenceSampler(pairs, int(gg["n_items"]), 64, 1)
    torch.manual_seed(55)
    for b in range(3):
        u, p, n = s()
        np.testing.assert_array_equal(u.numpy(), f["users"][b])
        np.testing.assert_array_equal(p.numpy(), f["pos"][b])
        np.testing.assert_array_equal(n.numpy(), f["neg"][b])
        assert n.shape == (64, 1)


def test_bpr_loss_keeps_the_broadcast():
    pos, neg = torch.randn(5), torch.randn(5, 1)
    ref = -torch.nn.functional.logsigmoid(pos.view(1, 5) - neg.view(5, 1)).mean()
    assert torch.equal(BPRLoss()(pos, neg), ref)


def _run_steps(adj, device, row_subset=True, native_adam=False):
    f = load_golden("bpr_train_K3_d64")
    _, nu, ni = _golden_graph()
    torch.manual_seed(56)
    m = LightGCN(nu, ni, embedding_dim=64, n_layers=3, init_scale=0.1).to(device)
    np.testing.assert_array_equal(m.user_embedding.weight.detach().cpu().numpy(), f["user_w0"])
    opt = (make_adam(m.parameters(), 1e-2, 1e-4, device) if native_adam
           else torch.optim.Adam(m.parameters(), lr=1e-2, weight_decay=1e-4))
    m.train()
    losses = []
    for b in range(3):
        args = [torch.from_numpy(f[k][b]).to(device) for k in ("users", "pos", "neg")]
        losses.append(float(train_step(m, adj, *args, opt, BPRLoss(), 1.0, row_subset)))
    return f, m, np.array(losses)


def test_three_adam_steps_match_reference_cpu():
    g, _, _ = _golden_graph()
    f, m, losses = _run_steps(g.to_torch_sparse_coo(), "cpu")
    np.testing.assert_allclose(losses, f["losses"], rtol=1e-6)
    np.testing.assert_allclose(m.user_embedding.weight.detach().numpy(), f["user_w"], atol=1e-6)
    np.testing.assert_allclose(m.item_embedding.weight.detach().numpy(), f["item_w"], atol=1e-6)


def test_device_sampler_law():
    rng = np.random.default_rng(0)
    nu, ni = 50, 40
    u = rng.integers(0, nu, 1500)
    i = rng.integers(0, ni, 1500)
    s = DeviceSampler(u, i, ni, 256, negative_samples=2, device="cpu", seed=3)
    pos_set = set(zip(u.tolist(), i.tolist()))
    bu, bp, bn = s()
    assert bu.shape == (256,) and bn.shape == (256, 2)
    assert all((a, b) in pos_set for a, b in zip(bu.tolist(), bp.tolist()))
    # a negative may only be a positive when all ten checked draws were positives
    dense = np.array([len({b for a, b in pos_set if a == x}) for x in range(nu)]) / ni
    bad = [(a, n) in pos_set for a, row in zip(bu.tolist(), bn.tolist()) for n in row]
    assert np.mean(bad) <= max(0.05, 3 * float(np.mean(dense ** 10)))
    assert s.is_positive(bu, bp).all()


def test_trainer_runs_and_learns_on_cpu():
    from src.data.dataset import RecommendationDataset
    ds = RecommendationDataset.synthetic_movielens(n_users=120, n_items=200, n_ratings=4000, seed=2)
    torch.manual_seed(0)
    m = LightGCN(ds.n_users, ds.n_items, 32, 2, 0.1)
    cfg = dict(batch_size=256, epochs=3, eval_every=1, learning_rate=5e-3, use_scheduler=True,
               warmup_epochs=1, validation_metrics=["recall@10", "ndcg@10"])
    t = Trainer(m, ds, cfg, device="cpu", sampler="reference")
    res = t.train()
    assert len(res["train_losses"]) == 3 and res["train_losses"][-1] < res["train_losses"][0]
    assert set(res["valid_metrics"][0]) >= {"recall@10", "ndcg@10"}


def test_bpr_scores_shapes():
    ue, ie = torch.randn(4, 8), torch.randn(6, 8)
    p, n = bpr_scores(ue, ie, torch.tensor([0, 1]), torch.tensor([2, 3]), torch.tensor([[4], [5]]))
    assert p.shape == (2,) and n.shape == (2, 1)


def test_row_subset_only_on_large_operands():
    """train_step's row-subset forward is used above functional.SMALL_OPERAND_ROWS rows only
    (on small operands the full propagation is cheaper; the bits are the same either way)."""
    from types import SimpleNamespace

    from src.ops import functional as F
    from src.training import trainer
    assert not trainer._row_subset_pays(SimpleNamespace(n_rows=9746))
    assert trainer._row_subset_pays(SimpleNamespace(n_rows=F.SMALL_OPERAND_ROWS + 1))
    assert trainer._row_subset_pays(object())   # an operand without a row count (torch sparse)


@pytest.mark.parametrize("n,bias", [(5000, True), (70_000, False), (300, True)])
def test_linear_rows_gradients_match_nn_linear(n, bias):
    """functional._LinearRows (the row-chunked weight gradient behind linear_rows): the same
    forward bits as nn.Linear and gradients within fp32 reassociation, with a row count that
    is not a multiple of the chunk."""
    from src.ops import functional as F
    torch.manual_seed(0)
    lin = torch.nn.Linear(64, 48, bias=bias)
    x = torch.randn(n, 64, requires_grad=True)
    g = torch.randn(n, 48)
    y_ref = lin(x)
    (y_ref * g).sum().backward()
    ref = [x.grad.clone(), lin.weight.grad.clone()] + ([lin.bias.grad.clone()] if bias else [])
    x.grad = None
    lin.zero_grad()
    y = F._LinearRows.apply(x, lin.weight, lin.bias)
    assert torch.equal(y, y_ref)
    (y * g).sum().backward()
    got = [x.grad, lin.weight.grad] + ([lin.bias.grad] if bias else [])
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4 * float(b.abs().max()))
