"""§8f1 on the GPU: the reference's three Adam steps (golden) with the native fused
propagation forward and backward (CsrGraph operand), the device sampler and the trainer."""
import numpy as np
import pytest
import torch

from test_training import _golden_graph, _run_steps

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("opt", ["torch", "native"])
def test_three_adam_steps_native_match_reference(cuda, opt):
    """Golden pinned by the reference trainer; "native" is make_adam's GPU optimizer."""
    g, _, _ = _golden_graph()
    f, m, losses = _run_steps(g.to(cuda), cuda, native_adam=opt == "native")
    # forward is bit-exact; the backward sums in a different order than torch's sparse
    # transpose-mm, and Adam normalises the gradient, so hold it to fp32 tolerance
    np.testing.assert_allclose(losses, f["losses"], rtol=1e-5)
    np.testing.assert_allclose(m.user_embedding.weight.detach().cpu().numpy(), f["user_w"], atol=2e-5)
    np.testing.assert_allclose(m.item_embedding.weight.detach().cpu().numpy(), f["item_w"], atol=2e-5)


def test_row_subset_step_same_bits_as_full_propagation(cuda, monkeypatch):
    """The training forward computes only the batch's rows (and their neighbourhoods): the
    loss and the updated weights are bit-identical to the full propagation's. (train_step
    skips the subset on operands this small, trainer._row_subset_pays; forced on here.)"""
    from src.training import trainer
    monkeypatch.setattr(trainer, "_row_subset_pays", lambda adj: True)
    g, _, _ = _golden_graph()
    gd = g.to(cuda)
    _, m1, l1 = _run_steps(gd, cuda, row_subset=True)
    _, m2, l2 = _run_steps(gd, cuda, row_subset=False)
    np.testing.assert_array_equal(l1, l2)
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(p1.detach(), p2.detach())


def test_device_sampler_on_gpu(cuda):
    from src.training import DeviceSampler
    rng = np.random.default_rng(1)
    u, i = rng.integers(0, 500, 20000), rng.integers(0, 300, 20000)
    s = DeviceSampler(u, i, 300, 2048, device=cuda, seed=0)
    bu, bp, bn = s()
    assert bu.is_cuda and bn.shape == (2048, 1)
    assert s.is_positive(bu, bp).all()
    assert s.is_positive(bu.view(-1, 1), bn).float().mean() < 0.01


def test_trainer_native(cuda):
    from src.data.dataset import RecommendationDataset
    from src.models import LightGCN
    from src.training import Trainer
    ds = RecommendationDataset.synthetic_movielens(n_users=300, n_items=400, n_ratings=9000, seed=4)
    torch.manual_seed(0)
    m = LightGCN(ds.n_users, ds.n_items, 64, 3, 0.1)
    t = Trainer(m, ds, dict(batch_size=512, epochs=3, eval_every=1, learning_rate=5e-3,
                            use_scheduler=False, warmup_epochs=0), device=cuda)
    from src.ops import CsrGraph
    assert isinstance(t.adj, CsrGraph) and t.adj.device.type == "cuda"
    res = t.train()
    assert res["train_losses"][-1] < res["train_losses"][0]
    assert res["valid_metrics"][0]["recall@10"] >= 0.0


def test_sharded_step_world1_native_matches_reference(cuda):
    """lightgcn_train_step_dist on one device (native hops) vs the reference trainer golden."""
    from conftest import load_golden
    from src.models import LightGCN
    from src.ops.distributed import DistributedGraph
    from src.training import lightgcn_train_step_dist
    f = load_golden("bpr_train_K3_d64")
    g, nu, ni = _golden_graph()
    torch.manual_seed(56)
    m = LightGCN(nu, ni, embedding_dim=64, n_layers=3, init_scale=0.1)
    x0 = torch.cat([m.user_embedding.weight, m.item_embedding.weight]).detach()
    dg = DistributedGraph(g, 0, 1, cuda)
    emb = torch.nn.Parameter(x0.to(cuda).clone())
    from src.training import make_adam
    opt = make_adam([emb], 1e-2, 1e-4, cuda)      # NativeAdam, clip folded into its update
    losses = [float(lightgcn_train_step_dist(dg, emb, 3, nu,
                                             *[torch.from_numpy(f[k][b]).to(cuda)
                                               for k in ("users", "pos", "neg")], opt))
              for b in range(3)]
    np.testing.assert_allclose(losses, f["losses"], rtol=1e-5)
    np.testing.assert_allclose(emb.detach()[:nu].cpu().numpy(), f["user_w"], atol=2e-5)
    np.testing.assert_allclose(emb.detach()[nu:].cpu().numpy(), f["item_w"], atol=2e-5)


def test_sharded_step_world1_tiled_native_adam(cuda, monkeypatch):
    """The same step with the column-ordered kernel forced onto the golden graph: the
    deferred schedule on one rank (placed hop tables, a strided gradient view) feeds
    NativeAdam, and the result still matches the reference trainer golden."""
    from conftest import load_golden
    from src.models import LightGCN
    from src.ops import functional as F
    from src.ops.distributed import DistributedGraph
    from src.training import lightgcn_train_step_dist, make_adam
    monkeypatch.setattr(F, "TILED_MIN_ROWS", 1)
    monkeypatch.setattr(F, "TILED_MIN_TABLE_BYTES", 0)
    f = load_golden("bpr_train_K3_d64")
    g, nu, ni = _golden_graph()
    torch.manual_seed(56)
    m = LightGCN(nu, ni, embedding_dim=64, n_layers=3, init_scale=0.1)
    x0 = torch.cat([m.user_embedding.weight, m.item_embedding.weight]).detach()
    dg = DistributedGraph(g, 0, 1, cuda)
    assert F.tiled_plan_for(dg.shard, dg.pad_table(x0, hop_layout=True)) is not None
    emb = torch.nn.Parameter(x0.to(cuda).clone())
    opt = make_adam([emb], 1e-2, 1e-4, cuda)
    losses = [float(lightgcn_train_step_dist(dg, emb, 3, nu,
                                             *[torch.from_numpy(f[k][b]).to(cuda)
                                               for k in ("users", "pos", "neg")], opt))
              for b in range(3)]
    np.testing.assert_allclose(losses, f["losses"], rtol=1e-5)
    np.testing.assert_allclose(emb.detach()[:nu].cpu().numpy(), f["user_w"], atol=2e-5)


def test_sharded_step_row_subset_same_bits(cuda):
    """The sharded step's row-subset forward and masked backward (native hops) give the
    same bits as its full propagation."""
    from conftest import load_golden
    from src.models import LightGCN
    from src.ops.distributed import DistributedGraph
    from src.training import lightgcn_train_step_dist
    f = load_golden("bpr_train_K3_d64")
    g, nu, ni = _golden_graph()
    torch.manual_seed(56)
    m = LightGCN(nu, ni, embedding_dim=64, n_layers=3, init_scale=0.1)
    x0 = torch.cat([m.user_embedding.weight, m.item_embedding.weight]).detach()
    dg = DistributedGraph(g, 0, 1, cuda)
    res = []
    for subset in (True, False):
        emb = torch.nn.Parameter(x0.to(cuda).clone())
        opt = torch.optim.Adam([emb], lr=1e-2, weight_decay=1e-4)
        losses = [float(lightgcn_train_step_dist(dg, emb, 3, nu,
                                                 *[torch.from_numpy(f[k][b]).to(cuda)
                                                   for k in ("users", "pos", "neg")], opt,
                                                 row_subset=subset))
                  for b in range(3)]
        res.append((losses, emb.detach().clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])


def test_native_adam_matches_torch_adam(cuda):
    """NativeAdam (one kernel per parameter, optional clip coefficient) follows
    torch.optim.Adam's update within fp32 rounding over several steps, odd sizes included."""
    from src.training import NativeAdam
    torch.manual_seed(0)
    shapes = [(1000, 64), (7,), (33, 3)]
    p1 = [torch.nn.Parameter(torch.randn(s, device=cuda)) for s in shapes]
    p2 = [torch.nn.Parameter(p.detach().clone()) for p in p1]
    o1 = NativeAdam(p1, lr=1e-2, weight_decay=1e-4)
    o2 = torch.optim.Adam(p2, lr=1e-2, weight_decay=1e-4)
    for it in range(5):
        grads = [torch.randn(s, device=cuda) for s in shapes]
        scale = torch.tensor(0.5 if it % 2 else 1.0, device=cuda)
        for a, b, g in zip(p1, p2, grads):
            a.grad = g.clone()
            b.grad = g * scale
        o1.step(grad_scale=scale)
        o2.step()
        assert torch.equal(p1[0].grad, grads[0])          # the gradient is left unscaled
    for a, b in zip(p1, p2):   # a few ulps of the O(1) weights (updates are O(lr) = 1e-2)
        np.testing.assert_allclose(a.detach().cpu().numpy(), b.detach().cpu().numpy(),
                                   rtol=1e-6, atol=1e-6)
    st1, st2 = o1.state[p1[0]], o2.state[p2[0]]
    np.testing.assert_allclose(st1["exp_avg_sq"].cpu().numpy(), st2["exp_avg_sq"].cpu().numpy(),
                               rtol=1e-6, atol=1e-12)
    assert float(st1["step"]) == float(st2["step"]) == 5


def test_sharded_step_deferred_mean_same_bits(cuda, monkeypatch):
    """With the column-ordered kernel forced, the one-device sharded step's backward (a masked
    hop 1, then the deferred layer mean) and its full propagations give the bits of the
    row-parallel kernel's eager schedule, over three Adam steps."""
    from conftest import load_golden
    from src.models import LightGCN
    from src.ops import functional as F
    from src.ops.distributed import DistributedGraph
    from src.training import lightgcn_train_step_dist
    f = load_golden("bpr_train_K3_d64")
    g, nu, ni = _golden_graph()
    torch.manual_seed(56)
    m = LightGCN(nu, ni, embedding_dim=64, n_layers=3, init_scale=0.1)
    x0 = torch.cat([m.user_embedding.weight, m.item_embedding.weight]).detach()
    res = []
    for forced, subset in ((False, True), (True, True), (True, False)):
        if forced:
            monkeypatch.setattr(F, "TILED_MIN_ROWS", 0)
            monkeypatch.setattr(F, "TILED_MIN_TABLE_BYTES", 0)
        dg = DistributedGraph(g, 0, 1, cuda)
        assert (F.tiled_plan_for(dg.shard, x0.to(cuda)) is not None) == forced
        emb = torch.nn.Parameter(x0.to(cuda).clone())
        opt = torch.optim.Adam([emb], lr=1e-2, weight_decay=1e-4)
        losses = [float(lightgcn_train_step_dist(dg, emb, 3, nu,
                                                 *[torch.from_numpy(f[k][b]).to(cuda)
                                                   for k in ("users", "pos", "neg")], opt,
                                                 row_subset=subset))
                  for b in range(3)]
        res.append((losses, emb.detach().clone()))
    for losses, emb in res[1:]:
        assert losses == res[0][0]
        assert torch.equal(emb, res[0][1])


def test_linear_rows_on_device_matches_nn_linear(cuda):
    """functional.linear_rows on a ROCm device above LINEAR_SPLIT_K_MIN_ROWS rows (the
    row-chunked weight gradient, NGCF / GAT training): nn.Linear's forward bits and its
    gradients within fp32 reassociation."""
    from src.ops import functional as F
    torch.manual_seed(0)
    n = F.LINEAR_SPLIT_K_MIN_ROWS + 12_345
    lin = torch.nn.Linear(64, 64).to(cuda)
    x = torch.randn(n, 64, device=cuda, requires_grad=True)
    g = torch.randn(n, 64, device=cuda)
    y_ref = lin(x)
    (y_ref * g).sum().backward()
    ref = [x.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone()]
    x.grad = None
    lin.zero_grad()
    y = F.linear_rows(x, lin)
    assert y.grad_fn is not None and "LinearRows" in type(y.grad_fn).__name__
    assert torch.equal(y, y_ref)
    (y * g).sum().backward()
    for a, b in zip([x.grad, lin.weight.grad, lin.bias.grad], ref):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4 * float(b.abs().max()))
