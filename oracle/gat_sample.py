"""Sampled-row GAT checker for graphs too large for the whole-graph oracle — TEST INFRASTRUCTURE.

Used by tests/ and tools/bench_configs.py (config 5 at G1B / 5M x 5M) as the checker, never
by the product. A row sample (the `n_heavy` heaviest rows plus `per_decile` random rows of
every degree decile) is cut out of the device CSR as a sub-CSR with global column ids; for
those rows:

* `heads_vs_oracle`: the native per-head aggregation (gnnrec_gat_aggregate_f32 + the heavy
  split) against oracle.gat_head (float64 edge softmax, gat.py:99-141 of the reference) on the
  SAME native projections — pins the aggregation kernels;
* `layer_rows`: the reference layer semantics (gat.py:76-151: per head h = W_h x, e =
  LeakyReLU(h_i a_self + h_j a_neigh), softmax over the row's neighbours, sum of alpha h_j;
  concat or head mean; then F.elu, gat.py:283) computed from a native layer input in
  numpy fp32 projections + the float64 oracle aggregation — pins the whole layer, and
  chained over the layers the final layer mean (gat.py:287-288).
"""
from __future__ import annotations

import numpy as np
import torch

from . import gat_head


def sample_rows(deg: np.ndarray, n_heavy: int = 64, per_decile: int = 4096,
                seed: int = 0) -> np.ndarray:
    """Sorted unique row ids: the n_heavy heaviest rows plus per_decile random rows from each
    degree decile (rows of degree 0 excluded: their NaN row is checked elsewhere)."""
    deg = np.asarray(deg)
    n = deg.size
    rng = np.random.default_rng(seed)
    heavy = np.argpartition(-deg, min(n_heavy, n) - 1)[:n_heavy] if n else np.zeros(0, np.int64)
    order = np.argsort(deg, kind="stable")
    picks = [heavy]
    for q in range(10):
        band = order[q * n // 10:(q + 1) * n // 10]
        if band.size:
            picks.append(rng.choice(band, size=min(per_decile, band.size), replace=False))
    rows = np.unique(np.concatenate(picks).astype(np.int64))
    return rows[deg[rows] > 0]


def sub_csr(row_ptr: torch.Tensor, col: torch.Tensor, rows: np.ndarray):
    """(rp_sub int64 [n+1], col_sub int32 global ids) of `rows` of a (device) CSR."""
    dev = row_ptr.device
    r = torch.from_numpy(rows).to(dev)
    beg, end = row_ptr[r], row_ptr[r + 1]
    lens = end - beg
    rp_sub = torch.zeros(rows.size + 1, dtype=torch.int64, device=dev)
    rp_sub[1:] = torch.cumsum(lens, 0)
    total = int(rp_sub[-1])
    idx = torch.repeat_interleave(beg - rp_sub[:-1], lens, output_size=total) + \
        torch.arange(total, device=dev)
    return rp_sub.cpu().numpy(), col[idx].cpu().numpy().astype(np.int32)


def _compact(col_sub: np.ndarray):
    """(needed global ids, col_sub remapped into them)."""
    needed, inv = np.unique(col_sub, return_inverse=True)
    return needed, inv.astype(np.int32)


def _rows(t: torch.Tensor, ids: np.ndarray) -> np.ndarray:
    return t[torch.from_numpy(ids).to(t.device)].float().cpu().numpy()


def heads_vs_oracle(rp_sub, col_sub, rows, feat, ss, sn, z, heads: int, o: int, slope: float,
                    shared: bool, att=None) -> list:
    """Per head: (native aggregation rows of z, oracle.gat_head on the native feat / ss / sn).
    att ([2, heads, o], the scores-from-rows kernels): ss / sn are None and the oracle's
    scores are the float64 dots att[0][h] . feat[r, h], att[1][h] . feat[j, h]."""
    needed, cc = _compact(col_sub)
    fn = _rows(feat, needed)
    zr = _rows(z, rows)
    if att is None:
        snn = _rows(sn, needed)
        ssr = _rows(ss, rows)
    else:
        a = att.detach().double().cpu().numpy()
        fr = _rows(feat, rows).astype(np.float64)
        fn64 = fn.astype(np.float64)
        ssr = np.empty((rows.size, heads), np.float32)
        snn = np.empty((needed.size, heads), np.float32)
        for h in range(heads):
            sl = slice(0, o) if shared else slice(h * o, (h + 1) * o)
            ssr[:, h] = fr[:, sl] @ a[0, h]
            snn[:, h] = fn64[:, sl] @ a[1, h]
    out = []
    for h in range(heads):
        hf = fn[:, :o] if shared else fn[:, h * o:(h + 1) * o]
        ref = gat_head(rp_sub, cc, np.ascontiguousarray(hf), ssr[:, h], snn[:, h], slope)
        out.append((zr[:, h * o:(h + 1) * o], ref))
    return out


def layer_rows(layer, x: torch.Tensor, rp_sub, col_sub, rows) -> np.ndarray:
    """The reference layer (gat.py:76-151) + F.elu at `rows`, from the native input table x
    ([N, in] on any device): fp32 projections as nn.Linear / torch.mm, float64 softmax
    aggregation (oracle.gat_head)."""
    needed, cc = _compact(col_sub)
    xn, xr = _rows(x, needed), _rows(x, rows)
    heads = []
    for h in range(layer.n_heads):
        W = layer.W[h].weight.detach().float().cpu().numpy()           # [o, in]
        a_s = layer.a_self[h].detach().float().cpu().numpy()[:, 0]
        a_n = layer.a_neigh[h].detach().float().cpu().numpy()[:, 0]
        hn = (xn @ W.T).astype(np.float32)
        hr = (xr @ W.T).astype(np.float32)
        ss = (hr @ a_s).astype(np.float32)
        sn = (hn @ a_n).astype(np.float32)
        heads.append(gat_head(rp_sub, cc, hn, ss, sn, layer.alpha))
    out = (np.concatenate(heads, axis=1) if layer.concat_heads
           else np.mean(np.stack(heads), axis=0, dtype=np.float32))
    return np.where(out > 0, out, np.expm1(out)).astype(np.float32)


def close(got: np.ndarray, ref: np.ndarray, rtol: float = 1e-4, atol: float = 1e-5) -> dict:
    """|got - ref| <= atol + rtol |ref| elementwise (the governing tolerance), and the north
    star's bar (embeddings within 1e-4 absolute) reported beside it."""
    err = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    ok = bool(np.all(err <= atol + rtol * np.abs(ref)) and np.all(np.isfinite(got)))
    mx = float(err.max()) if err.size else 0.0
    return {"rtol": rtol, "atol": atol, "within_tolerance": ok, "max_abs_diff": mx,
            "max_abs_ref": float(np.abs(ref).max()) if ref.size else 0.0,
            "within_north_star_1e-4_abs": bool(mx <= 1e-4)}


def check_forward(model, g_dev, mine: torch.Tensor, rows: np.ndarray) -> dict:
    """Config-5 check at the rows sample: per head, the native aggregation of the first and last
    layer against oracle.gat_head; every layer's output against the reference layer on the
    native layer input; the timed forward's layer mean against the oracle layers' mean."""
    from src.ops import functional as F
    rp_sub, col_sub = sub_csr(g_dev.row_ptr, g_dev.col, rows)
    res = {"rows": int(rows.size), "edges": int(col_sub.size),
           "max_row_degree": int(np.diff(rp_sub).max())}
    L = len(model.layers)
    with torch.no_grad():
        x = model._initial_table()
        mean = _rows(x, rows).astype(np.float32)
        for k, layer in enumerate(model.layers, start=1):
            if k in (1, L):
                shared = layer.shares_input()
                o = layer.in_dim if shared else layer.out_dim
                att = None
                if layer.att_ok():        # the forward's kernels: scores from the rows
                    feat, ss, sn = layer.native_rows(x), None, None
                    att = layer.att_vectors()
                    z = F.gat_aggregate_att(g_dev, feat, feat, att, layer.n_heads, o,
                                            layer.alpha, shared_rows=shared)
                else:
                    feat, ss, sn = layer.native_inputs(x)
                    z = F.gat_aggregate(g_dev, feat, ss, sn, layer.n_heads, o, layer.alpha,
                                        mean_heads=False, shared_rows=shared)
                res[f"layer{k}_kernels"] = "scores from rows" if att is not None else "score tables"
                for h, (got, ref) in enumerate(heads_vs_oracle(rp_sub, col_sub, rows, feat, ss,
                                                               sn, z, layer.n_heads, o,
                                                               layer.alpha, shared, att)):
                    res[f"layer{k}_head{h}_aggregation"] = close(got, ref)
                del feat, ss, sn, z
            ref_k = layer_rows(layer, x, rp_sub, col_sub, rows)
            x = layer(x, g_dev, apply_elu=True)          # the native layer output (next input)
            res[f"layer{k}_output"] = close(_rows(x, rows), ref_k)
            mean = mean + ref_k
        mean = (mean / np.float32(L + 1)).astype(np.float32)
    res["forward_layer_mean"] = close(_rows(mine, rows), mean)
    res["all_within_tolerance"] = all(v["within_tolerance"] for v in res.values()
                                      if isinstance(v, dict))
    return res
