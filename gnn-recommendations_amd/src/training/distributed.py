"""Row-sharded LightGCN BPR training step (SURVEY §8e "Training (next)" + §8f1).

The embedding table x0 = cat(user_embedding, item_embedding) is split by destination rows
exactly like the operand (DistributedGraph): rank p owns rows [b_p, b_{p+1}) of x0 as its
own parameter shard and its Adam state. One step (the body of trainer.py:248-279):

  forward   x0 rows exchanged once (each rank receives the rows its shard references), then
            the K-hop propagation with its per-hop exchanges (lightgcn_propagate_dist);
  loss      the batch (identical on every rank: same sampler seed) needs the output rows of
            its users / positives / negatives; every rank writes the rows it owns into a
            [3B, d] buffer of zeros and one all_reduce(SUM) completes it (x + 0 = x: exact);
            every rank then evaluates the same BPR loss ([B, B] broadcast kept) and its
            gradient with respect to those rows;
  backward  each rank scatters the gradient rows it owns into dY, and the gradient of x0 is
            the SAME propagation applied to dY (A^T = A): mean_k A^k dY, sharded the same way;
  update    clip_grad_norm_ over the global norm (one all_reduce of the squared norm), then
            Adam on the local shard (element-wise, so identical to the single-device update
            of those rows).

No all-reduce of the embedding gradient is needed: the table is row-sharded, not replicated.

With the native hops (`hop_fn` None) and `row_subset`, the forward's last two hops compute
only the rows the batch reads and their neighbourhoods, and the backward's first hops skip
the all-zero rows of the sparse gradient (as ops.lightgcn_forward_rows / lightgcn_backward
on one device: the same bits). The row sets are marked on each rank from its own shard's
rows and OR-ed across ranks (one all_reduce(MAX) of a byte per row per restricted hop).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist

from ..ops.distributed import DistributedGraph, _exchanged, lightgcn_propagate_dist
from .losses import BPRLoss
from .optim import NativeAdam


def _all_reduce(t: torch.Tensor, dg: DistributedGraph, op=dist.ReduceOp.SUM) -> torch.Tensor:
    if dg.world == 1:
        return t
    if t.is_cuda and dist.get_backend(dg.group) == "gloo":   # 1-GPU test harness
        h = t.cpu()
        dist.all_reduce(h, op=op, group=dg.group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=dg.group)
    return t


def _padded_ids(dg: DistributedGraph, ids: torch.Tensor) -> torch.Tensor:
    """Global row ids -> positions in the padded layout (on ids' device)."""
    b = torch.as_tensor(dg.bounds, dtype=torch.int64, device=ids.device)
    owner = torch.searchsorted(b, ids, right=True) - 1
    return owner * dg.rows_pad + (ids - b[owner])


def _reach(dg: DistributedGraph, local_marked: torch.Tensor) -> torch.Tensor:
    """Padded uint8 mask of the columns listed by the marked rows of every rank's shard (for
    a symmetric operand: the rows those rows reach, and the rows they read)."""
    from ..ops.functional import mark_rows
    m = mark_rows(dg.shard.row_ptr, dg.shard.col, local_marked, dg.world * dg.rows_pad)
    return _all_reduce(m, dg, dist.ReduceOp.MAX)


def lightgcn_train_step_dist(dg: DistributedGraph, emb_local: torch.nn.Parameter, n_layers: int,
                             n_users: int, users: torch.Tensor, pos_items: torch.Tensor,
                             neg_items: torch.Tensor, optimizer: torch.optim.Optimizer,
                             loss_fn: Optional[torch.nn.Module] = None,
                             max_grad_norm: float = 1.0,
                             hop_fn: Optional[Callable] = None,
                             row_subset: bool = True) -> torch.Tensor:
    """One BPR step on this rank's shard; returns the (replicated) loss as a 0-d tensor.
    emb_local: this rank's rows [row_begin, row_end) of x0 (a leaf Parameter the optimizer
    owns). users / pos_items / neg_items: the same batch on every rank (global ids; items
    counted from 0 as in the reference). hop_fn: the local hop (default: the native SpMM)."""
    loss_fn = loss_fn or BPRLoss()
    dev = emb_local.device
    b0, b1 = dg.row_begin, dg.row_end
    K = int(n_layers)
    native = hop_fn is None and row_subset
    with torch.no_grad():
        B = users.numel()
        neg2 = neg_items.view(B, -1)
        ids = torch.cat([users.view(-1), n_users + pos_items.view(-1),
                         n_users + neg2.reshape(-1)]).to(dev)
        fwd_masks = None
        if native:   # R_K = the batch rows, R_k = R_K | rows read by R_{k+1} (last two hops)
            need = torch.zeros(dg.world * dg.rows_pad, dtype=torch.uint8, device=dev)
            need[_padded_ids(dg, ids)] = 1
            R = {K: need}
            for k in range(K - 1, max(K - 2, 0), -1):
                R[k] = _reach(dg, dg.local_slice(R[k + 1])).bitwise_or_(need)
            fwd_masks = lambda k, _x: (None, dg.local_slice(R[k])) if k in R else None  # noqa: E731
        x0_pad = _exchanged(dg, emb_local.detach())
        out_local = lightgcn_propagate_dist(dg, x0_pad, K, hop_fn=hop_fn, masks=fwd_masks)
        mine = (ids >= b0) & (ids < b1)
        rows = torch.zeros((ids.numel(), emb_local.shape[1]), dtype=emb_local.dtype, device=dev)
        rows[mine] = out_local[ids[mine] - b0]
        _all_reduce(rows, dg)
    rb = rows.requires_grad_(True)
    u, p, n = rb[:B], rb[B:2 * B], rb[2 * B:].view(B, neg2.shape[1], -1)
    pos_s = (u * p).sum(dim=1)
    neg_s = (u.unsqueeze(1) * n).sum(dim=2)
    if neg_items.dim() == 1:
        neg_s = neg_s.view(B)
    loss = loss_fn(pos_s, neg_s)
    loss.backward()
    with torch.no_grad():
        dy = torch.zeros_like(emb_local)
        # sort-based accumulate (deterministic, as autograd's indexing backward), not
        # index_add_'s atomics: repeated batch rows sum in a fixed order
        dy.index_put_((ids[mine] - b0,), rb.grad[mine], accumulate=True)
        bwd_masks = None
        if native:   # hop 1 skips the zero rows and the rows none reaches; hops 2..K-1 skip
            # the zero rows unless the column-ordered kernel takes the shard (its dense hop is
            # faster there: ops.functional.lightgcn_backward)
            from ..ops.functional import row_nonzero, tiled_plan_for

            def bwd_masks(k, x_in):
                if k >= K or (k > 1 and tiled_plan_for(dg.shard, x_in) is not None):
                    return None
                xm = row_nonzero(x_in)
                ya = dg.local_slice(_reach(dg, dg.local_slice(xm))) if k == 1 else None
                return xm, ya
        # (one rank: the deferred schedule returns a row-major view of its placed output
        # table, functional.hop_table; the optimizers take dense gradients)
        grad = lightgcn_propagate_dist(dg, _exchanged(dg, dy), K, hop_fn=hop_fn,
                                       masks=bwd_masks).contiguous()
        coef = None
        if max_grad_norm > 0:
            sq = (torch.linalg.vector_norm(grad, 2, dtype=torch.float64) ** 2).view(1)
            _all_reduce(sq, dg)
            coef = torch.clamp(max_grad_norm / (sq.sqrt() + 1e-6), max=1.0).to(grad.dtype)
            if not isinstance(optimizer, NativeAdam):
                grad.mul_(coef)
    optimizer.zero_grad()
    emb_local.grad = grad
    if isinstance(optimizer, NativeAdam):
        optimizer.step(grad_scale=coef)
    else:
        optimizer.step()
    return loss.detach()
