"""Test-time evaluation over the native scoring/top-K kernel (reference: evaluator.py:52-124).

Propagate once, then for batches of users one kernel scores every item (MFMA, sequential-k
fmaf order), masks the train+valid items and keeps the top-K under the fixed order
(score desc, item asc) — instead of U[b] @ I^T + a Python masking loop + torch.topk + copy.
On CPU operands the same semantics run in torch (stable sort for the tie order).
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops import CsrGraph, score_topk, uses_native


def compute_metrics_from_topk(topk_items, user_ids: List[int], ground_truth: Dict[int, List[int]],
                              n_items: int, k_values=(10, 20)) -> Dict[str, float]:
    """recall / ndcg / precision / coverage / gini @k (metrics.py:355-432)."""
    topk = np.asarray(topk_items.cpu() if torch.is_tensor(topk_items) else topk_items)
    if topk.size == 0:
        return {}
    out = {}
    for k in k_values:
        k = min(k, topk.shape[1])
        rec, nd, pre = [], [], []
        disc = 1.0 / np.log2(np.arange(k) + 2)
        for row, u in enumerate(user_ids):
            rel = set(ground_truth.get(u, ()))
            if not rel:
                continue
            pred = topk[row, :k]
            hit = np.array([p in rel for p in pred])
            rec.append(hit.sum() / len(rel))
            pre.append(hit.sum() / k)
            idcg = disc[:min(len(rel), k)].sum()
            nd.append((disc * hit).sum() / idcg if idcg > 0 else 0.0)
        out[f"recall@{k}"] = float(np.mean(rec)) if rec else 0.0
        out[f"ndcg@{k}"] = float(np.mean(nd)) if nd else 0.0
        out[f"precision@{k}"] = float(np.mean(pre)) if pre else 0.0
        flat = topk[:, :k].ravel()
        flat = flat[flat >= 0]
        out[f"coverage@{k}"] = len(set(flat.tolist())) / max(1, n_items)
        counts = np.sort(np.bincount(flat, minlength=n_items))
        n = counts.size
        out[f"gini@{k}"] = float(2 * np.sum((np.arange(n) + 1) * counts) / (n * counts.sum())
                                 - (n + 1) / n) if counts.sum() > 0 else 0.0
    return out


def _row_chunks(parts, rows: int):
    """(global first row, fp32 chunk) over the row-concatenation of `parts`, `rows` at a time
    (a chunk never spans two parts; nothing is copied beyond one chunk)."""
    r0 = 0
    for p in parts:
        for s in range(0, p.shape[0], rows):
            yield r0 + s, p[s:s + rows].detach().float()
        r0 += p.shape[0]


def _take_rows(parts, idx: torch.Tensor) -> torch.Tensor:
    """Rows `idx` (global, in that order) of the row-concatenation of `parts`."""
    out = torch.empty((idx.numel(), parts[0].shape[1]), dtype=torch.float32,
                      device=parts[0].device)
    r0 = 0
    for p in parts:
        sel = ((idx >= r0) & (idx < r0 + p.shape[0])).nonzero().flatten()
        if sel.numel():
            out[sel] = p.detach()[idx[sel] - r0].float()
        r0 += p.shape[0]
    return out


def embedding_statistics(emb, exact_limit: int = 65536, chunk: int = 4096,
                         stat_rows: int = 1 << 20) -> Dict[str, float]:
    """The over-smoothing statistics evaluate() adds (evaluator.py:116-121 ->
    training/metrics.py:229-315), on the propagated table where it lives:
    mcs = mean off-diagonal cosine similarity, mad = mean off-diagonal pairwise Euclidean
    distance (||a||^2 + ||b||^2 - 2ab, clamped at 0), variance = mean per-dimension unbiased
    variance. The reference materialises the [N, N] matrices (infeasible past ~5e4 nodes);
    here mcs is the exact identity (||sum e_n||^2 - sum ||e_n||^2) / (N (N-1)) over
    L2-normalised rows and mad runs over row chunks, so nothing N x N is held. Above
    `exact_limit` nodes mad is taken over a fixed-seed sample of that many rows (flagged
    'mad_sampled'). Values agree with the reference to fp32 reassociation.

    `emb` is one [N, d] table or a sequence of tables read as their row-concatenation (the
    user and item halves: no torch.cat copy). mcs and variance run over `stat_rows`-row
    chunks with float64 sums, so the transient memory is a chunk, not the table (G100M:
    ~0.5 GB instead of ~150 GB of float64 copies)."""
    parts = [emb] if torch.is_tensor(emb) else [p for p in emb if p.shape[0] > 0]
    n = sum(p.shape[0] for p in parts)
    out: Dict[str, float] = {}
    if n < 2:
        return {"mcs": float("nan"), "mad": float("nan"), "variance": float("nan")}
    dev = parts[0].device
    d = parts[0].shape[1]
    s = torch.zeros(d, dtype=torch.float64, device=dev)
    ss = torch.zeros((), dtype=torch.float64, device=dev)
    colsum = torch.zeros(d, dtype=torch.float64, device=dev)
    for _, c in _row_chunks(parts, stat_rows):
        en = torch.nn.functional.normalize(c, p=2, dim=1).double()
        s += en.sum(0)
        ss += (en * en).sum()
        colsum += c.double().sum(0)
    out["mcs"] = float(((s @ s) - ss) / (n * (n - 1)))
    mean = colsum / n
    dev2 = torch.zeros(d, dtype=torch.float64, device=dev)
    for _, c in _row_chunks(parts, stat_rows):
        dev2 += ((c.double() - mean) ** 2).sum(0)
    variance = float((dev2 / (n - 1)).mean())
    if n > exact_limit:
        g = torch.Generator(device="cpu").manual_seed(0)
        sub = _take_rows(parts, torch.randperm(n, generator=g)[:exact_limit].to(dev))
        out["mad_sampled"] = float(exact_limit)
    else:
        sub = _take_rows(parts, torch.arange(n, device=dev)) if len(parts) > 1 else \
            parts[0].detach().float()
    m = sub.shape[0]
    nsq = (sub ** 2).sum(1)
    tot = torch.zeros((), dtype=torch.float64, device=dev)
    for r0 in range(0, m, chunk):
        blk = sub[r0:r0 + chunk]
        d2 = nsq[r0:r0 + chunk, None] + nsq[None, :] - 2 * (blk @ sub.T)
        dist = torch.sqrt(torch.clamp(d2, min=0))
        idx = torch.arange(blk.shape[0], device=dev)
        dist[idx, r0 + idx] = 0.0                    # the diagonal is excluded from the mean
        tot += dist.double().sum()
    out["mad"] = float(tot / (m * (m - 1)))
    out["variance"] = variance
    return out


class Evaluator:
    def __init__(self, k_values=(10, 20), device: Optional[torch.device] = None):
        self.k_values = list(k_values)
        self.device = device or torch.device("cuda" if torch.cuda.is_available() else "cpu")

    def topk(self, user_emb, item_emb, users, k, seen_ptr, seen_col, batch_size=None):
        """[len(users), k] int64 top-k item ids (fixed tie order). On the GPU nothing of size
        batch x n_items is materialised, so the batch is large (16384 users) and the kernel's
        item split fills the chip; the CPU path keeps the reference's 2048."""
        if batch_size is None:
            batch_size = 16384 if user_emb.is_cuda else 2048
        rows = []
        for s in range(0, len(users), batch_size):
            b = torch.as_tensor(users[s:s + batch_size], dtype=torch.long, device=user_emb.device)
            bp = seen_ptr[b.cpu().numpy()]
            counts = seen_ptr[b.cpu().numpy() + 1] - bp
            sub_ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
            # gather the batch's seen lists without a per-user loop
            src = np.repeat(bp - sub_ptr[:-1], counts) + np.arange(int(sub_ptr[-1]))
            sub_col = seen_col[src] if src.size else np.zeros(0, np.int32)
            if user_emb.is_cuda:
                idx, _ = score_topk(user_emb[b], item_emb, k, torch.from_numpy(sub_ptr),
                                    torch.from_numpy(sub_col.astype(np.int32)))
            else:
                sc = user_emb[b] @ item_emb.T
                for r in range(len(b)):
                    sc[r, torch.from_numpy(sub_col[sub_ptr[r]:sub_ptr[r + 1]].astype(np.int64))] = float("-inf")
                order = torch.sort(sc, dim=1, descending=True, stable=True).indices
                idx = order[:, :k]
            rows.append(idx.cpu())
        return torch.cat(rows)

    def evaluate(self, model, dataset, test_data=None, adj_matrix=None,
                 mask_valid: bool = True) -> Dict[str, float]:
        """Metrics over test_data (default: the test split) with train (+ valid when
        mask_valid; the trainer's validation masks train items only, trainer.py:321-333)
        items excluded from the ranking."""
        model.eval()
        test_data = dataset.test_data if test_data is None else test_data
        with torch.no_grad():
            adj = adj_matrix if adj_matrix is not None else (
                dataset.get_graph(self.device) if self.device.type == "cuda"
                else dataset.get_torch_adjacency())
            user_emb, item_emb = model.get_all_embeddings(adj)
            gt = defaultdict(list)
            for u, i in zip(test_data["userId"].to_numpy(), test_data["itemId"].to_numpy()):
                gt[int(u)].append(int(i))
            users = sorted(gt)
            if not users:
                return {}
            seen_ptr, seen_col = dataset.seen_items(include_valid=mask_valid)
            topk = self.topk(user_emb, item_emb, users, max(self.k_values), seen_ptr, seen_col)
            metrics = compute_metrics_from_topk(topk, users, gt, dataset.n_items, self.k_values)
            metrics.update(embedding_statistics((user_emb, item_emb)))
            return metrics
