"""Generate the golden vectors that pin the oracle and the HIP path to the reference.

Run ONLY in the build container, where the reference is importable:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports timur1arkhipov/gnn-recommendations from /root/reference/gnn-recommendations
(read-only; no bytecode is written) and runs the reference's own functions and modules on
small seeded inputs, saving inputs and outputs as plain arrays (np.savez, no pickles) under
tests/golden/. The reference itself never travels to the GPU box; these fixtures do.
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import numpy as np

sys.dont_write_bytecode = True
REF = Path(os.environ.get("GNNREC_REFERENCE", "/root/reference/gnn-recommendations"))
OUT = Path(__file__).resolve().parent


def _import_reference():
    sys.path.insert(0, str(REF))
    import torch  # noqa: F401
    import pandas as pd  # noqa: F401
    from src.data import graph_builder as gb
    from src.models.baselines.lightgcn import LightGCN
    from src.models.baselines.ngcf import NGCF
    from src.models.baselines.gat import GAT
    from src.models.orthogonal_bundle.group_shuffle_layer import GroupShuffleLayer
    from src.models.orthogonal_bundle.bundle_layer import BundleConnectionLayer
    from src.models.orthogonal_bundle.model import OrthogonalBundleGNN
    return gb, LightGCN, NGCF, GAT, GroupShuffleLayer, BundleConnectionLayer, OrthogonalBundleGNN


def interactions(seed, n_users, n_items, n_pairs, dup_frac=0.0, min_deg=False):
    rng = np.random.default_rng(seed)
    u = rng.integers(0, n_users, n_pairs, dtype=np.int64)
    i = rng.integers(0, n_items, n_pairs, dtype=np.int64)
    if min_deg:  # every user and item gets at least one interaction
        u = np.concatenate([u, np.arange(n_users), rng.integers(0, n_users, n_items)])
        i = np.concatenate([i, rng.integers(0, n_items, n_users), np.arange(n_items)])
    key = u * n_items + i
    _, first = np.unique(key, return_index=True)
    keep = np.sort(first)
    u, i = u[keep], i[keep]
    if dup_frac > 0:  # re-append some pairs: the reference sums them to weight 2
        k = int(dup_frac * u.size)
        u = np.concatenate([u, u[:k]])
        i = np.concatenate([i, i[:k]])
    return u, i


def ref_graph(gb, u, i, nu, ni, self_loop=False):
    import pandas as pd
    df = pd.DataFrame({"userId": u, "itemId": i})
    adj = gb.build_bipartite_graph(df, nu, ni, self_loop=self_loop)
    norm = gb.normalize_adjacency_matrix(adj, "symmetric")
    deg = np.maximum(np.array(adj.tocsr().sum(axis=1)).flatten(), 1.0)
    t = gb.convert_to_torch_sparse(norm)
    return norm, deg, t


def main():
    import torch
    gb, LightGCN, NGCF, GAT, GSL, BCL, OBG = _import_reference()
    torch.set_num_threads(1)
    meta = dict(torch=torch.__version__, numpy=np.__version__)
    import scipy
    meta["scipy"] = scipy.__version__

    # ---- a1-a3: operand values (plain, duplicates, self loops) ---------------------------------
    graphs = {}
    for name, (seed, nu, ni, npairs, dup, sl) in {
        "g_small": (0, 300, 500, 5000, 0.0, False),
        "g_dup": (1, 120, 90, 1500, 0.1, False),
        "g_selfloop": (2, 80, 60, 700, 0.0, True),
        "g_iso": (3, 200, 300, 400, 0.0, False),   # sparse: isolated users/items exist
    }.items():
        u, i = interactions(seed, nu, ni, npairs, dup)
        norm, deg, _ = ref_graph(gb, u, i, nu, ni, self_loop=sl)
        graphs[name] = (u, i, nu, ni, norm)
        np.savez(OUT / f"graph_{name}.npz", users=u, items=i, n_users=nu, n_items=ni,
                 self_loop=int(sl), row=norm.row.astype(np.int64), col=norm.col.astype(np.int64),
                 val=norm.data.astype(np.float32), deg=deg.astype(np.float32))

    # ---- a4/a5: LightGCN per layer, K in {1,2,3}, d in {32,64,128} ----------------------------
    u, i, nu, ni, norm = graphs["g_small"]
    t_adj = gb.convert_to_torch_sparse(norm)
    for K, d in [(1, 32), (2, 64), (3, 64), (3, 128)]:
        torch.manual_seed(100 + K * 7 + d)
        m = LightGCN(nu, ni, embedding_dim=d, n_layers=K, init_scale=0.1)
        m.eval()
        with torch.no_grad():
            ue, ie = m(t_adj)
            layers = m.get_layer_embeddings(t_adj)
        np.savez(OUT / f"lightgcn_K{K}_d{d}.npz", graph="g_small",
                 user_w=m.user_embedding.weight.detach().numpy(),
                 item_w=m.item_embedding.weight.detach().numpy(),
                 layers=np.stack([x.numpy() for x in layers]), user_out=ue.numpy(),
                 item_out=ie.numpy())
    # LightGCN gradient of a scalar loss (backward = A^T propagation), d=64 K=3
    torch.manual_seed(7)
    m = LightGCN(nu, ni, embedding_dim=64, n_layers=3, init_scale=0.1)
    ue, ie = m(t_adj)
    g_u = torch.randn_like(ue)
    g_i = torch.randn_like(ie)
    ((ue * g_u).sum() + (ie * g_i).sum()).backward()
    np.savez(OUT / "lightgcn_grad_K3_d64.npz", graph="g_small",
             user_w=m.user_embedding.weight.detach().numpy(),
             item_w=m.item_embedding.weight.detach().numpy(), g_u=g_u.numpy(), g_i=g_i.numpy(),
             grad_user=m.user_embedding.weight.grad.numpy(),
             grad_item=m.item_embedding.weight.grad.numpy())

    # ---- a6: NGCF eval forward, layer_sizes [64,64,64] -----------------------------------------
    torch.manual_seed(11)
    m = NGCF(nu, ni, embedding_dim=64, layer_sizes=[64, 64, 64], dropout=0.1, init_scale=0.01)
    with torch.no_grad():  # non-zero biases so the bias path is exercised
        for L in m.layers:
            L.W1.bias.normal_(0, 0.05)
            L.W2.bias.normal_(0, 0.05)
    m.eval()
    with torch.no_grad():
        ue, ie = m(t_adj)
    arrs = dict(graph="g_small", user_w=m.user_embedding.weight.detach().numpy(),
                item_w=m.item_embedding.weight.detach().numpy(), user_out=ue.numpy(),
                item_out=ie.numpy())
    for li, L in enumerate(m.layers):
        arrs[f"W1_{li}"] = L.W1.weight.detach().numpy()
        arrs[f"b1_{li}"] = L.W1.bias.detach().numpy()
        arrs[f"W2_{li}"] = L.W2.weight.detach().numpy()
        arrs[f"b2_{li}"] = L.W2.bias.detach().numpy()
    np.savez(OUT / "ngcf_d64.npz", **arrs)

    # ---- a7: GroupShuffleLayer, a8: BundleConnectionLayer --------------------------------------
    torch.manual_seed(21)
    gs = GSL(64, 8, init_scale=0.01)
    with torch.no_grad():
        for p in gs.skew_params:
            p.mul_(30.0)  # rotate visibly (still exactly orthogonal through matrix_exp)
    x = torch.randn(257, 64) * 0.1
    with torch.no_grad():
        y = gs(x)
        W = gs._build_orthogonal_matrix()
    blocks = np.stack([W[b * 8:(b + 1) * 8, b * 8:(b + 1) * 8].numpy() for b in range(8)])
    np.savez(OUT / "gas_d64_bs8.npz", skew=np.stack([p.detach().numpy() for p in gs.skew_params]),
             perm=gs.perm.numpy(), blocks=blocks, x=x.numpy(), y=y.numpy(), W=W.numpy())
    torch.manual_seed(22)
    bc = BCL(64, 8)
    with torch.no_grad():
        Wc = bc()
    np.savez(OUT / "bundle_d64_bs8.npz", skew=np.stack([p.detach().numpy() for p in bc.skew_params]),
             shuffle_perm=bc.shuffle_perm.numpy(), W=Wc.numpy())

    # ---- a9: OrthogonalBundleGNN eval forward + layer embeddings ------------------------------
    torch.manual_seed(31)
    m = OBG(nu, ni, embedding_dim=64, n_layers=3, block_size=8, residual_alpha=0.1, dropout=0.0,
            init_scale=0.01, use_parallel_transport=True)
    with torch.no_grad():
        m.layer_weights.copy_(torch.tensor([0.3, -0.2, 0.5, 0.1]))
        for L in list(m.local_transform_layers) + list(m.connection_layers):
            for p in L.skew_params:
                p.mul_(20.0)
    m.eval()
    with torch.no_grad():
        ue, ie = m(adj_matrix=t_adj)
        layers = m.get_layer_embeddings(adj_matrix=t_adj)
    arrs = dict(graph="g_small", user_w=m.user_embedding.weight.detach().numpy(),
                item_w=m.item_embedding.weight.detach().numpy(), user_out=ue.numpy(),
                item_out=ie.numpy(), layer_weights=m.layer_weights.detach().numpy(),
                layers=np.stack([x.numpy() for x in layers]))
    for li in range(3):
        gsl, bcl = m.local_transform_layers[li], m.connection_layers[li]
        arrs[f"gs_skew_{li}"] = np.stack([p.detach().numpy() for p in gsl.skew_params])
        arrs[f"gs_perm_{li}"] = gsl.perm.numpy()
        arrs[f"bc_skew_{li}"] = np.stack([p.detach().numpy() for p in bcl.skew_params])
        arrs[f"bc_perm_{li}"] = bcl.shuffle_perm.numpy()
    np.savez(OUT / "ob_d64.npz", **arrs)

    # ---- §8f1: BPR training (reference sampler RNG order, [B,B] loss quirk, Adam steps) -----
    from types import SimpleNamespace
    from src.training.trainer import Trainer as RefTrainer
    from src.training.losses import BPRLoss as RefBPR
    pairs = list(zip(u.tolist(), i.tolist()))
    fake = SimpleNamespace(batch_size=64, negative_samples=1, device=torch.device("cpu"))
    torch.manual_seed(55)
    batches = [RefTrainer._sample_batch(fake, pairs, ni) for _ in range(3)]
    torch.manual_seed(56)
    m = LightGCN(nu, ni, embedding_dim=64, n_layers=3, init_scale=0.1)
    w0 = (m.user_embedding.weight.detach().clone(), m.item_embedding.weight.detach().clone())
    opt = torch.optim.Adam(m.parameters(), lr=1e-2, weight_decay=1e-4)
    loss_fn = RefBPR()
    losses = []
    m.train()
    for bu, bp, bn in batches:   # the body of trainer.py:248-279
        ue, ie = m.get_all_embeddings(t_adj)
        ps = (ue[bu] * ie[bp]).sum(dim=1)
        ns = (ue[bu].unsqueeze(1) * ie[bn]).sum(dim=2)
        loss = loss_fn(ps, ns)
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
        opt.step()
        losses.append(loss.item())
    np.savez(OUT / "bpr_train_K3_d64.npz", graph="g_small",
             users=np.stack([b[0].numpy() for b in batches]),
             pos=np.stack([b[1].numpy() for b in batches]),
             neg=np.stack([b[2].numpy() for b in batches]),
             user_w0=w0[0].numpy(), item_w0=w0[1].numpy(), losses=np.array(losses),
             user_w=m.user_embedding.weight.detach().numpy(),
             item_w=m.item_embedding.weight.detach().numpy())

    # ---- a11: GAT eval forward (dense reference; min-degree >= 1 so no NaN rows) -------------
    gu, gi = interactions(41, 60, 80, 500, min_deg=True)
    gnorm, _, gt = ref_graph(gb, gu, gi, 60, 80)
    torch.manual_seed(42)
    m = GAT(60, 80, embedding_dim=64, n_layers=3, n_heads=4, dropout=0.1, alpha=0.2,
            init_scale=0.1)
    m.eval()
    with torch.no_grad():
        ue, ie = m(gt)
    arrs = dict(users=gu, items=gi, n_users=60, n_items=80, user_w=m.user_embedding.weight.detach().numpy(),
                item_w=m.item_embedding.weight.detach().numpy(), user_out=ue.numpy(), item_out=ie.numpy())
    for li, L in enumerate(m.layers):
        arrs[f"W_{li}"] = np.stack([w.weight.detach().numpy() for w in L.W])
        arrs[f"a_self_{li}"] = np.stack([a.detach().numpy()[:, 0] for a in L.a_self])
        arrs[f"a_neigh_{li}"] = np.stack([a.detach().numpy()[:, 0] for a in L.a_neigh])
        arrs[f"concat_{li}"] = int(L.concat_heads)
    np.savez(OUT / "gat_d64_h4.npz", **arrs)

    # ---- a13: scores + mask + top-K exactly as evaluator.py:96-105 -----------------------------
    rng = np.random.default_rng(51)
    U = torch.from_numpy(rng.standard_normal((70, 64)).astype(np.float32) * 0.1)
    I = torch.from_numpy(rng.standard_normal((400, 64)).astype(np.float32) * 0.1)
    seen = [sorted(set(rng.integers(0, 400, rng.integers(0, 30)).tolist())) for _ in range(70)]
    scores = U @ I.T
    for r, items in enumerate(seen):
        if items:
            scores[r, items] = float("-inf")
    topk = torch.topk(scores, k=20, dim=1)
    seen_ptr = np.cumsum([0] + [len(s) for s in seen]).astype(np.int64)
    seen_col = np.array([c for s in seen for c in s], dtype=np.int64)
    np.savez(OUT / "topk_d64.npz", U=U.numpy(), I=I.numpy(), seen_ptr=seen_ptr, seen_col=seen_col,
             scores=scores.numpy(), topk_idx=topk.indices.numpy(), topk_val=topk.values.numpy())

    with open(OUT / "VERSIONS.txt", "w") as f:
        for k, v in meta.items():
            f.write(f"{k}={v}\n")
    print("golden vectors written to", OUT)


if __name__ == "__main__":
    main()
