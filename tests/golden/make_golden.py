"""Generate the golden vectors that pin the oracle and the HIP path to the reference.

Run ONLY in the build container, where the reference is importable:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--only long_rows,edge_paths]

It imports timur1arkhipov/gnn-recommendations from /root/reference/gnn-recommendations
(read-only; no bytecode is written) and runs the reference's own functions and modules on
small seeded inputs, saving inputs and outputs as plain arrays (np.savez, no pickles) under
tests/golden/. The reference itself never travels to the GPU box; these fixtures do.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import subprocess
import sys
import tempfile
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


def sha256(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def ml1m_pairs():
    """Config 2's graph (BASELINE configs[1]): the train pairs of the repo's ML-1M-shaped
    synthetic dataset (RecommendationDataset.synthetic_movielens(6040, 3706, 1_000_209,
    seed=1): Zipf item popularity -> rating >= 3, 5-core, temporal split). Made in a child
    process because the repo's package is also named `src`."""
    pkg = Path(__file__).resolve().parents[2] / "gnn-recommendations_amd"
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / "pairs.npz"
        code = ("import sys, numpy as np; sys.path.insert(0, sys.argv[1]); "
                "from src.data.dataset import RecommendationDataset as R; "
                "ds = R.synthetic_movielens(6040, 3706, 1_000_209, seed=1, name='ml-1m'); "
                "np.savez(sys.argv[2], u=ds.train_data.userId.to_numpy(), "
                "i=ds.train_data.itemId.to_numpy(), nu=ds.n_users, ni=ds.n_items)")
        subprocess.run([sys.executable, "-c", code, str(pkg), str(out)], check=True,
                       env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"))
        with np.load(out) as z:
            return z["u"], z["i"], int(z["nu"]), int(z["ni"])


def make_long_rows(gb, LightGCN):
    """LightGCN K=3 d=64 on the ML-1M-shaped graph: rows up to 5 857 neighbours (343 rows
    above the heavy-row threshold), so the reference's torch.sparse.mm chain order is pinned
    on long rows, not only on the <= 28-nnz rows of g_small. Every layer is pinned by the
    SHA-256 of its fp32 bytes (bit-exact or nothing); the final output and the heavy rows of
    every hop are stored as values too."""
    import torch
    u, i, nu, ni = ml1m_pairs()
    norm, deg, t_adj = ref_graph(gb, u, i, nu, ni)
    N = nu + ni
    rp = np.zeros(N + 1, np.int64)
    np.add.at(rp, norm.row.astype(np.int64) + 1, 1)
    rp = np.cumsum(rp)
    col = norm.col.astype(np.int32)
    val = norm.data.astype(np.float32)
    torch.manual_seed(2024)
    m = LightGCN(nu, ni, embedding_dim=64, n_layers=3, init_scale=0.1)
    m.eval()
    with torch.no_grad():
        ue, ie = m(t_adj)
        layers = [x.numpy() for x in m.get_layer_embeddings(t_adj)]
    out = np.concatenate([ue.numpy(), ie.numpy()])
    heavy = np.nonzero(np.diff(rp) > 256)[0].astype(np.int64)
    np.savez_compressed(
        OUT / "lightgcn_ml1m_K3_d64.npz", users=u.astype(np.int16), items=i.astype(np.int16),
        n_users=nu, n_items=ni, seed=2024, nnz=int(rp[-1]), max_degree=int(np.diff(rp).max()),
        operand_sha256=np.array([sha256(rp), sha256(col), sha256(val)]),
        layers_sha256=np.array([sha256(x) for x in layers]), out_sha256=sha256(out),
        user_out=ue.numpy(), item_out=ie.numpy(), heavy_rows=heavy,
        layers_heavy=np.stack([x[heavy] for x in layers[1:]]))
    print(f"long_rows: N={N} nnz={rp[-1]} max degree {np.diff(rp).max()}, {heavy.size} heavy rows")


def make_edge_paths(gb, OBG, ESBC, PT):
    """use_edge_index=True paths of OrthogonalBundleGNN (model.py:160-181, 215-220,
    parallel_transport.py:5-52) with and without parallel transport, and the per-edge-type
    connection EdgeSpecificBundleConnection (bundle_layer.py:106-149) through the 3-D
    bmm branch of parallel_transport_along_edges (:37-43). The edge list is the g_small
    interactions in both directions, shuffled, with 150 repeated edges (multiplicity 2)."""
    import torch
    nu, ni = 300, 500
    u, i = interactions(0, nu, ni, 5000)
    rng = np.random.default_rng(61)
    src = np.concatenate([u, nu + i])
    dst = np.concatenate([nu + i, u])
    rep = rng.choice(src.size, 150, replace=False)
    src = np.concatenate([src, src[rep]])
    dst = np.concatenate([dst, dst[rep]])
    order = rng.permutation(src.size)
    src, dst = src[order], dst[order]
    ei = torch.from_numpy(np.vstack([src, dst]).astype(np.int64))
    for pt in (True, False):
        torch.manual_seed(62 + int(pt))
        m = OBG(nu, ni, embedding_dim=64, n_layers=3, block_size=8, residual_alpha=0.1,
                dropout=0.0, init_scale=0.01, use_parallel_transport=pt, use_edge_index=True)
        with torch.no_grad():
            m.layer_weights.copy_(torch.tensor([0.3, -0.2, 0.5, 0.1]))
            conn = list(m.connection_layers) if pt else []
            for L in list(m.local_transform_layers) + conn:
                for p in L.skew_params:
                    p.mul_(20.0)
        m.eval()
        with torch.no_grad():
            ue, ie = m(edge_index=ei)
            layers = m.get_layer_embeddings(edge_index=ei)
        arrs = dict(edge_index=ei.numpy(), n_users=nu, n_items=ni, seed=62 + int(pt),
                    use_parallel_transport=int(pt),
                    user_w=m.user_embedding.weight.detach().numpy(),
                    item_w=m.item_embedding.weight.detach().numpy(), user_out=ue.numpy(),
                    item_out=ie.numpy(), layers=np.stack([x.numpy() for x in layers]))
        for li in range(3):
            gsl = m.local_transform_layers[li]
            arrs[f"gs_skew_{li}"] = np.stack([p.detach().numpy() for p in gsl.skew_params])
            arrs[f"gs_perm_{li}"] = gsl.perm.numpy()
            if pt:
                bcl = m.connection_layers[li]
                arrs[f"bc_skew_{li}"] = np.stack([p.detach().numpy() for p in bcl.skew_params])
                arrs[f"bc_perm_{li}"] = bcl.shuffle_perm.numpy()
        np.savez_compressed(OUT / f"ob_edge_index_pt{int(pt)}_d64.npz", **arrs)
    torch.manual_seed(71)
    esbc = ESBC(64, 8, n_edge_types=2)
    with torch.no_grad():
        for L in esbc.connection_layers:
            for p in L.skew_params:
                p.mul_(20.0)
    et = torch.from_numpy((src >= nu).astype(np.int64))   # 0: user -> item, 1: item -> user
    x = torch.randn(nu + ni, 64) * 0.1
    with torch.no_grad():
        W = esbc(ei, et)
        y = PT(x, ei, W)
        Wt = np.stack([L().numpy() for L in esbc.connection_layers])
    np.savez_compressed(
        OUT / "edge_specific_d64.npz", edge_index=ei.numpy(), edge_type=et.numpy(), x=x.numpy(),
        y=y.numpy(), W_types=Wt, skew=np.stack([np.stack([p.detach().numpy() for p in L.skew_params])
                                                for L in esbc.connection_layers]),
        perm=np.stack([L.shuffle_perm.numpy() for L in esbc.connection_layers]))
    print(f"edge_paths: E={src.size}")


def ml1m_golden_graph():
    """The ML-1M-shaped pairs stored in lightgcn_ml1m_K3_d64.npz (config 2's graph)."""
    with np.load(OUT / "lightgcn_ml1m_K3_d64.npz", allow_pickle=False) as z:
        return (z["users"].astype(np.int64), z["items"].astype(np.int64), int(z["n_users"]),
                int(z["n_items"]))


def ml1m_rows(norm):
    """The output rows a real-shape fixture keeps: every heavy row (> 256 neighbours, up to
    5 857) plus every 13th row (the whole [N, (K+1) d] tables would be 10 MB per model)."""
    deg = np.bincount(norm.row, minlength=norm.shape[0])
    return np.union1d(np.nonzero(deg > 256)[0], np.arange(0, norm.shape[0], 13)).astype(np.int64)


def make_ml1m_models(gb, NGCF, GSL, OBG):
    """Config 3's models on config 2's real-shape graph (rows of up to 5 857 neighbours)
    instead of the 800-node g_small: the reference's NGCF K=3 d=64 (ngcf.py:52-86, 170-190),
    NGCF + GAS composed from the reference's own NGCFLayer and GroupShuffleLayer
    (x_{l+1} = GS_l(NGCFLayer_l(x_l)), group_shuffle_layer.py:73-96 — the reference has no
    such model class), and OrthogonalBundleGNN on the adjacency path (model.py:120-213)."""
    import torch
    u, i, nu, ni = ml1m_golden_graph()
    norm, _, t_adj = ref_graph(gb, u, i, nu, ni)
    rows = ml1m_rows(norm)

    def ngcf(seed):
        torch.manual_seed(seed)
        m = NGCF(nu, ni, embedding_dim=64, layer_sizes=[64, 64, 64], dropout=0.1,
                 init_scale=0.1)
        with torch.no_grad():
            for L in m.layers:
                L.W1.bias.normal_(0, 0.05)
                L.W2.bias.normal_(0, 0.05)
        return m.eval()

    def ngcf_arrays(m):
        # the embedding tables are re-drawn from the seed by the drop-in class (same RNG
        # order, tests/test_models.py); their hash pins that
        arrs = dict(emb_sha256=np.array([sha256(m.user_embedding.weight.detach().numpy()),
                                         sha256(m.item_embedding.weight.detach().numpy())]))
        for li, L in enumerate(m.layers):
            arrs[f"W1_{li}"] = L.W1.weight.detach().numpy()
            arrs[f"b1_{li}"] = L.W1.bias.detach().numpy()
            arrs[f"W2_{li}"] = L.W2.weight.detach().numpy()
            arrs[f"b2_{li}"] = L.W2.bias.detach().numpy()
        return arrs

    m = ngcf(311)
    with torch.no_grad():
        ue, ie = m(t_adj)
    out = torch.cat([ue, ie]).numpy()
    np.savez_compressed(OUT / "ngcf_ml1m_d64.npz", rows=rows, out_rows=out[rows], seed=311,
                        n_users=nu, n_items=ni, **ngcf_arrays(m))

    m = ngcf(312)
    torch.manual_seed(313)
    gsl = [GSL(64, 8, init_scale=0.01) for _ in range(3)]
    with torch.no_grad():
        for gs in gsl:
            for p in gs.skew_params:
                p.mul_(30.0)
        x = torch.cat([m.user_embedding.weight, m.item_embedding.weight])
        outs = [x]
        for L, gs in zip(m.layers, gsl):
            x = gs(L(x, t_adj))
            outs.append(x)
        out = torch.cat(outs, dim=1).numpy()
    arrs = ngcf_arrays(m)
    for li, gs in enumerate(gsl):
        arrs[f"gs_skew_{li}"] = np.stack([p.detach().numpy() for p in gs.skew_params])
        arrs[f"gs_perm_{li}"] = gs.perm.numpy()
    np.savez_compressed(OUT / "ngcf_gas_ml1m_d64.npz", rows=rows, out_rows=out[rows], seed=312,
                        n_users=nu, n_items=ni, **arrs)

    torch.manual_seed(331)
    m = OBG(nu, ni, embedding_dim=64, n_layers=3, block_size=8, residual_alpha=0.1, dropout=0.0,
            init_scale=0.1, use_parallel_transport=True)
    with torch.no_grad():
        m.layer_weights.copy_(torch.tensor([0.3, -0.2, 0.5, 0.1]))
        for L in list(m.local_transform_layers) + list(m.connection_layers):
            for p in L.skew_params:
                p.mul_(20.0)
    m.eval()
    with torch.no_grad():
        ue, ie = m(adj_matrix=t_adj)
        layers = m.get_layer_embeddings(adj_matrix=t_adj)
    out = torch.cat([ue, ie]).numpy()
    arrs = dict(emb_sha256=np.array([sha256(m.user_embedding.weight.detach().numpy()),
                                     sha256(m.item_embedding.weight.detach().numpy())]),
                seed=331, n_users=nu, n_items=ni,
                layer_weights=m.layer_weights.detach().numpy(), rows=rows, out_rows=out[rows],
                layers_rows=np.stack([x.numpy()[rows] for x in layers]))
    for li in range(3):
        gsl_, bcl = m.local_transform_layers[li], m.connection_layers[li]
        arrs[f"gs_skew_{li}"] = np.stack([p.detach().numpy() for p in gsl_.skew_params])
        arrs[f"gs_perm_{li}"] = gsl_.perm.numpy()
        arrs[f"bc_skew_{li}"] = np.stack([p.detach().numpy() for p in bcl.skew_params])
        arrs[f"bc_perm_{li}"] = bcl.shuffle_perm.numpy()
    np.savez_compressed(OUT / "ob_ml1m_d64.npz", **arrs)
    print(f"ml1m_models: N={nu + ni}, {rows.size} rows kept")


def gat_heavy_pairs():
    """A min-degree-1 power-law bipartite graph with rows above GAT_HEAVY_THRESHOLD (2048):
    3 000 users x 4 000 items, Zipf(1.6) item popularity (the two most popular items reach
    ~2 900 and ~2 600 users), one hub user with 2 500 items, every node at least one edge."""
    rng = np.random.default_rng(91)
    nu, ni = 3000, 4000
    u = rng.integers(0, nu, 40000)
    i = np.minimum(rng.zipf(1.6, 40000) - 1, ni - 1)
    u = np.concatenate([u, np.zeros(2500, np.int64), np.arange(nu), rng.integers(0, nu, ni)])
    i = np.concatenate([i, rng.choice(ni, 2500, replace=False), rng.integers(0, ni, nu),
                        np.arange(ni)])
    key = u * ni + i
    _, first = np.unique(key, return_index=True)
    keep = np.sort(first)
    return u[keep], i[keep], nu, ni


def make_gat_heavy(gb, GAT):
    """Config 5's degree-bucketed path pinned to the reference itself: the reference's dense
    GAT (gat.py:76-151, 258-297; [N, N] masked softmax per head, N = 7 000) K=3 d=64 with 4
    heads on gat_heavy_pairs(), whose longest rows (2 500+ neighbours) exceed the native
    kernel's GAT_HEAVY_THRESHOLD and run through the segment + merge kernels."""
    import torch
    u, i, nu, ni = gat_heavy_pairs()
    _, _, t = ref_graph(gb, u, i, nu, ni)
    torch.manual_seed(92)
    m = GAT(nu, ni, embedding_dim=64, n_layers=3, n_heads=4, dropout=0.1, alpha=0.2,
            init_scale=0.1)
    m.eval()
    with torch.no_grad():
        ue, ie = m(t)
    deg = np.bincount(np.concatenate([u, nu + i]), minlength=nu + ni)
    arrs = dict(users=u.astype(np.int16), items=i.astype(np.int16), n_users=nu, n_items=ni,
                seed=92, max_degree=int(deg.max()), user_out=ue.numpy(), item_out=ie.numpy())
    for li, L in enumerate(m.layers):
        arrs[f"W_{li}"] = np.stack([w.weight.detach().numpy() for w in L.W])
        arrs[f"a_self_{li}"] = np.stack([a.detach().numpy()[:, 0] for a in L.a_self])
        arrs[f"a_neigh_{li}"] = np.stack([a.detach().numpy()[:, 0] for a in L.a_neigh])
    np.savez_compressed(OUT / "gat_heavy_d64_h4.npz", **arrs)
    print(f"gat_heavy: N={nu + ni} nnz={2 * u.size} max degree {deg.max()}, "
          f"{int((deg > 2048).sum())} rows > 2048")


def make_gat_grad(gb, GAT):
    """GAT training gradients (gat.py:76-151 dense masked softmax, 258-297) for the native
    backward (csrc/gat_train.hip): the gat_d64_h4 graph and model seed, dropout 0 (the
    reference's F.dropout draws cannot be reproduced natively), train() mode, loss =
    sum(user_out * Ru) + sum(item_out * Ri) with seeded Ru, Ri; every parameter's gradient."""
    import torch
    gu, gi = interactions(41, 60, 80, 500, min_deg=True)
    _, _, gt = ref_graph(gb, gu, gi, 60, 80)
    torch.manual_seed(42)
    m = GAT(60, 80, embedding_dim=64, n_layers=3, n_heads=4, dropout=0.0, alpha=0.2,
            init_scale=0.1)
    m.train()
    ue, ie = m(gt)
    rng = np.random.default_rng(43)
    Ru = torch.from_numpy(rng.standard_normal(ue.shape).astype(np.float32))
    Ri = torch.from_numpy(rng.standard_normal(ie.shape).astype(np.float32))
    loss = (ue * Ru).sum() + (ie * Ri).sum()
    loss.backward()
    arrs = dict(users=gu, items=gi, n_users=60, n_items=80, Ru=Ru.numpy(), Ri=Ri.numpy(),
                loss=np.float64(loss.item()), user_out=ue.detach().numpy(),
                item_out=ie.detach().numpy())
    for name, prm in m.named_parameters():
        arrs["grad." + name] = prm.grad.detach().numpy()
        arrs["param." + name] = prm.detach().numpy()
    np.savez(OUT / "gat_grad_d64_h4.npz", **arrs)
    print(f"gat_grad: loss {loss.item():.6f}, {len(list(m.parameters()))} parameter gradients")


def make_emb_stats():
    """The over-smoothing statistics Evaluator.evaluate adds (evaluator.py:116-121 ->
    training/metrics.py:229-315) on a table with a zero row and two identical rows."""
    import torch
    from src.training.metrics import (embedding_variance, mean_average_distance,
                                      mean_cosine_similarity)
    torch.manual_seed(81)
    e = torch.randn(700, 64) * 0.1 + 0.02
    e[5] = 0.0
    e[9] = e[3]
    np.savez(OUT / "emb_stats.npz", emb=e.numpy(), mcs=mean_cosine_similarity(e),
             mad=mean_average_distance(e), variance=embedding_variance(e))


def main():
    import torch
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="", help="comma list: long_rows, edge_paths, emb_stats, "
                                               "ml1m_models, gat_heavy, gat_grad")
    only = set(filter(None, ap.parse_args().only.split(",")))
    gb, LightGCN, NGCF, GAT, GSL, BCL, OBG = _import_reference()
    torch.set_num_threads(1)
    if only:
        from src.models.orthogonal_bundle.bundle_layer import EdgeSpecificBundleConnection
        from src.models.orthogonal_bundle.parallel_transport import parallel_transport_along_edges
        if "long_rows" in only:
            make_long_rows(gb, LightGCN)
        if "edge_paths" in only:
            make_edge_paths(gb, OBG, EdgeSpecificBundleConnection, parallel_transport_along_edges)
        if "emb_stats" in only:
            make_emb_stats()
        if "ml1m_models" in only:
            make_ml1m_models(gb, NGCF, GSL, OBG)
        if "gat_heavy" in only:
            make_gat_heavy(gb, GAT)
        if "gat_grad" in only:
            make_gat_grad(gb, GAT)
        return
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

    from src.models.orthogonal_bundle.bundle_layer import EdgeSpecificBundleConnection
    from src.models.orthogonal_bundle.parallel_transport import parallel_transport_along_edges
    make_long_rows(gb, LightGCN)
    make_edge_paths(gb, OBG, EdgeSpecificBundleConnection, parallel_transport_along_edges)
    make_emb_stats()
    make_ml1m_models(gb, NGCF, GSL, OBG)
    make_gat_heavy(gb, GAT)
    make_gat_grad(gb, GAT)

    with open(OUT / "VERSIONS.txt", "w") as f:
        for k, v in meta.items():
            f.write(f"{k}={v}\n")
    print("golden vectors written to", OUT)


if __name__ == "__main__":
    main()
