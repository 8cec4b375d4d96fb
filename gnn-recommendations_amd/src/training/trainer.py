"""BPR training around the native propagation (reference: src/training/trainer.py), SURVEY §8f1.

What is kept from the reference (trainer.py:40-126, 199-281, 283-347, 469-579): the config
keys and defaults, Adam with weight decay, optional linear warm-up + cosine annealing,
full-graph propagation for EVERY batch, scores and BPRLoss with the reference's [B, 1]
negative scores (so the loss is the [B, B] broadcast mean), clip_grad_norm_, validation
masking train items, early stopping on `early_stopping_metric`.

What changes, and why:
* the operand is built once and stays resident (the reference rebuilds the torch COO tensor
  and copies it host->device every epoch and every validation, trainer.py:233-234,293-294);
  on a ROCm device it is a CsrGraph and the forward AND backward propagation run in the
  native kernels (LightGCN: one fused K-hop launch sequence each way, the backward being the
  same propagation over A^T = A);
* batches come from DeviceSampler (same law as the reference's Python loop, drawn on the
  GPU) unless `sampler="reference"` asks for the reference's exact RNG stream;
* the per-batch `loss.item()` host sync is replaced by an on-device running sum read once
  per epoch.
Checkpoint files, embedding export/warm-start and orthogonality logging are out of scope.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from ..evaluation.evaluator import Evaluator
from .losses import BPRLoss
from .optim import NativeAdam
from .sampler import DeviceSampler, ReferenceSampler


def bpr_scores(user_emb: torch.Tensor, item_emb: torch.Tensor, users: torch.Tensor,
               pos_items: torch.Tensor, neg_items: torch.Tensor):
    """pos [B] and neg [B] or [B, n_neg] scores exactly as trainer.py:256-261."""
    u = user_emb[users]
    pos = (u * item_emb[pos_items]).sum(dim=1)
    if neg_items.dim() == 1:
        neg = (u * item_emb[neg_items]).sum(dim=1)
    else:
        neg = (u.unsqueeze(1) * item_emb[neg_items]).sum(dim=2)
    return pos, neg


def make_adam(params, lr: float, weight_decay: float, device) -> torch.optim.Optimizer:
    """The reference's optimizer (trainer.py:59-63: Adam with L2 weight decay); on a GPU the
    native one-kernel-per-parameter form (NativeAdam)."""
    if torch.device(device).type == "cuda":
        return NativeAdam(params, lr=lr, weight_decay=weight_decay)
    return torch.optim.Adam(params, lr=lr, weight_decay=weight_decay)


def clip_and_step(params, optimizer, max_grad_norm: float) -> None:
    """clip_grad_norm_(params, max_grad_norm) + optimizer.step(); NativeAdam takes the clip
    coefficient into its update instead of scaling the gradients in place (same product)."""
    if max_grad_norm > 0 and isinstance(optimizer, NativeAdam):
        grads = [p.grad for p in params if p.grad is not None]
        total = torch.nn.utils.get_total_norm(grads, 2.0)
        coef = torch.clamp(max_grad_norm / (total + 1e-6), max=1.0)
        optimizer.step(grad_scale=coef)
        return
    if max_grad_norm > 0:
        torch.nn.utils.clip_grad_norm_(params, max_grad_norm)
    optimizer.step()


def batch_rows(n_users: int, n_items: int, users, pos_items, neg_items) -> torch.Tensor:
    """uint8 [n_users + n_items]: 1 at the propagated-table rows a BPR batch reads."""
    need = torch.zeros(n_users + n_items, dtype=torch.uint8, device=users.device)
    need[users] = 1
    need[n_users + pos_items] = 1
    need[n_users + neg_items.reshape(-1)] = 1
    return need


def _row_subset_pays(adj) -> bool:
    """The row-subset forward skips most rows of the last hops on a large operand; on a small
    one (at most functional.SMALL_OPERAND_ROWS rows, e.g. ML-1M) a full hop is one ~40 us
    launch and marking the rows costs more: the ML-1M-shaped LightGCN step 1.31-1.32 ms with
    the subset, 1.13-1.15 ms without, alternating runs (tools/exp_train_ml1m.py,
    profiles/r06/train_ml1m.jsonl). Same loss and gradient bits either way."""
    from ..ops import functional as F
    n = getattr(adj, "n_rows", None)
    return n is None or n > F.SMALL_OPERAND_ROWS


def train_step(model: nn.Module, adj, users, pos_items, neg_items, optimizer,
               loss_fn: Optional[nn.Module] = None, max_grad_norm: float = 1.0,
               row_subset: bool = True) -> torch.Tensor:
    """One batch of trainer.py:248-279: propagation, BPR loss, backward, clip, Adam.
    Returns the loss as a 0-d device tensor (no host sync). The loss reads only the batch's
    rows of the propagated table, so with `row_subset` a model with `forward_rows` computes
    just those (and what they depend on): the same loss and gradient bits as the full
    propagation the reference runs (trainer.py:251-254); on small operands the full
    propagation is cheaper and is used (_row_subset_pays)."""
    loss_fn = loss_fn or BPRLoss()
    if row_subset and hasattr(model, "forward_rows") and _row_subset_pays(adj):
        need = batch_rows(model.n_users, model.n_items, users, pos_items, neg_items)
        user_emb, item_emb = model.forward_rows(adj, need)
    elif hasattr(model, "get_all_embeddings"):
        user_emb, item_emb = model.get_all_embeddings(adj)
    else:
        user_emb, item_emb = model(adj)
    pos, neg = bpr_scores(user_emb, item_emb, users, pos_items, neg_items)
    loss = loss_fn(pos, neg)
    if hasattr(model, "get_regularization_loss"):
        loss = loss + model.get_regularization_loss()
    optimizer.zero_grad()
    loss.backward()
    clip_and_step(list(model.parameters()), optimizer, max_grad_norm)
    return loss.detach()


class Trainer:
    def __init__(self, model: nn.Module, dataset, config: dict, device=None,
                 sampler: str = "device", seed: int = 0):
        self.model, self.dataset, self.config = model, dataset, config
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda" if torch.cuda.is_available() else "cpu")
        self.model.to(self.device)
        lr = float(config.get("learning_rate", 1e-3))
        wd = float(config.get("weight_decay", 1e-4))
        self.batch_size = int(config.get("batch_size", 2048))
        self.epochs = int(config.get("epochs", 300))
        self.eval_every = int(config.get("eval_every", 10))
        self.negative_samples = int(config.get("negative_samples", 1))
        self.optimizer = make_adam(self.model.parameters(), lr, wd, self.device)
        self.use_scheduler = bool(config.get("use_scheduler", True))
        self.warmup_epochs = int(config.get("warmup_epochs", 5))
        self.base_lr = lr
        self.scheduler = (torch.optim.lr_scheduler.CosineAnnealingLR(
            self.optimizer, T_max=max(1, self.epochs - self.warmup_epochs), eta_min=lr * 0.01)
            if self.use_scheduler else None)
        self.loss_fn = BPRLoss()
        self.max_grad_norm = float(config.get("max_grad_norm", 1.0))
        es = config.get("early_stopping", {}) or {}
        self.patience = int(es.get("patience", 20))
        self.min_delta = float(es.get("min_delta", 1e-4))
        self.validation_metrics = list(config.get("validation_metrics", ["recall@10", "ndcg@10"]))
        self.early_stopping_metric = config.get("early_stopping_metric", "recall@10")
        self.current_epoch, self.best_metric, self.best_epoch, self.patience_counter = 0, 0.0, 0, 0
        self.train_losses: List[float] = []
        self.valid_metrics: List[Dict[str, float]] = []

        tr = dataset.train_data
        self.adj = (dataset.get_graph(self.device) if self.device.type == "cuda"
                    else dataset.get_torch_adjacency(normalized=True))
        self.n_train = len(tr)
        if sampler == "reference":
            pairs = list(zip(tr["userId"].astype(int), tr["itemId"].astype(int)))
            self.sampler = ReferenceSampler(pairs, dataset.n_items, self.batch_size,
                                            self.negative_samples, self.device)
        elif sampler == "device":
            self.sampler = DeviceSampler(tr["userId"].to_numpy(), tr["itemId"].to_numpy(),
                                         dataset.n_items, self.batch_size,
                                         self.negative_samples, self.device, seed)
        else:
            raise ValueError(f"unknown sampler: {sampler}")

    def train_epoch(self) -> float:
        self.model.train()
        total = torch.zeros((), dtype=torch.float64, device=self.device)
        n_batches = self.n_train // self.batch_size + 1      # trainer.py:242
        for _ in range(n_batches):
            users, pos, neg = self.sampler()
            total += train_step(self.model, self.adj, users, pos, neg, self.optimizer,
                                self.loss_fn, self.max_grad_norm)
        return float(total.item()) / n_batches

    def _k_values(self) -> List[int]:
        ks = []
        for m in self.validation_metrics:
            if "@" in m:
                try:
                    ks.append(int(m.split("@")[1]))
                except ValueError:
                    pass
        return sorted(set(ks)) or [10]

    def validate(self) -> Dict[str, float]:
        if self.dataset.valid_data is None or len(self.dataset.valid_data) == 0:
            return {}
        ev = Evaluator(k_values=self._k_values(), device=self.device)
        return ev.evaluate(self.model, self.dataset, test_data=self.dataset.valid_data,
                           adj_matrix=self.adj, mask_valid=False)

    def train(self) -> Dict:
        t0 = time.time()
        for epoch in range(1, self.epochs + 1):
            self.current_epoch = epoch
            if epoch <= self.warmup_epochs:
                for g in self.optimizer.param_groups:
                    g["lr"] = self.base_lr * (epoch / self.warmup_epochs)
            elif self.scheduler is not None:
                self.scheduler.step()
            self.train_losses.append(self.train_epoch())
            if epoch % self.eval_every == 0 or epoch == 1:
                vm = self.validate()
                self.valid_metrics.append(vm)
                cur = vm.get(self.early_stopping_metric, 0.0)
                if cur > self.best_metric + self.min_delta:
                    self.best_metric, self.best_epoch, self.patience_counter = cur, epoch, 0
                else:
                    self.patience_counter += 1
                if self.patience_counter >= self.patience:
                    break
        return {"best_metric": self.best_metric, "best_epoch": self.best_epoch,
                "training_time": time.time() - t0, "train_losses": self.train_losses,
                "valid_metrics": self.valid_metrics}
