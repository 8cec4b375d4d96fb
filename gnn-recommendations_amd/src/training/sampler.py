"""BPR batch samplers (reference: training/trainer.py:146-197).

ReferenceSampler reproduces the reference's sampling exactly — the same calls on torch's
global CPU generator in the same order (batch indices, then per row and per negative a
uniform item, redrawn while it is a positive of the user, at most 10 redraws, the last one
unchecked) — so a seeded run draws the reference's batches. It is a Python loop, as there.

DeviceSampler draws the same distribution on the GPU in a handful of kernels: the batch
rows, then 11 candidate items per negative at once; the negative is the first of the first
ten candidates that is not a positive (membership by binary search in the sorted
user*n_items+item keys of the training pairs), else the eleventh. It uses its own
generator, so batches differ from the reference's stream while their law is the same.
"""
from __future__ import annotations

from collections import defaultdict
from typing import List, Tuple

import numpy as np
import torch


class ReferenceSampler:
    def __init__(self, pairs: List[Tuple[int, int]], n_items: int, batch_size: int,
                 negative_samples: int = 1, device="cpu"):
        self.pairs, self.n_items = pairs, int(n_items)
        self.batch_size, self.negative_samples = int(batch_size), int(negative_samples)
        self.device = torch.device(device)
        self.user_pos = defaultdict(set)
        for u, i in pairs:
            self.user_pos[u].add(i)

    def __call__(self):
        b = min(self.batch_size, len(self.pairs))
        idx = torch.randint(0, len(self.pairs), (b,))
        users, pos, neg = [], [], []
        for k in idx:
            u, p = self.pairs[k.item()]
            seen = self.user_pos[u]
            row = []
            for _ in range(self.negative_samples):
                n = torch.randint(0, self.n_items, (1,)).item()
                for _ in range(10):
                    if n not in seen:
                        break
                    n = torch.randint(0, self.n_items, (1,)).item()
                row.append(n)
            users.append(u)
            pos.append(p)
            neg.append(row)
        return (torch.tensor(users, device=self.device), torch.tensor(pos, device=self.device),
                torch.tensor(neg, device=self.device))


class DeviceSampler:
    RETRIES = 10

    def __init__(self, users: np.ndarray, items: np.ndarray, n_items: int, batch_size: int,
                 negative_samples: int = 1, device="cuda", seed: int = 0):
        self.device = torch.device(device)
        self.users = torch.as_tensor(np.asarray(users, np.int64), device=self.device)
        self.items = torch.as_tensor(np.asarray(items, np.int64), device=self.device)
        self.n_items = int(n_items)
        self.batch_size, self.negative_samples = int(batch_size), int(negative_samples)
        self.keys = torch.unique(self.users * self.n_items + self.items)  # sorted
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)

    def is_positive(self, users: torch.Tensor, items: torch.Tensor) -> torch.Tensor:
        q = users * self.n_items + items
        pos = torch.searchsorted(self.keys, q).clamp_(max=self.keys.numel() - 1)
        return self.keys[pos] == q

    def __call__(self):
        n = self.users.numel()
        b = min(self.batch_size, n)
        idx = torch.randint(0, n, (b,), device=self.device, generator=self.gen)
        u, p = self.users[idx], self.items[idx]
        cand = torch.randint(0, self.n_items, (b, self.negative_samples, self.RETRIES + 1),
                             device=self.device, generator=self.gen)
        bad = self.is_positive(u.view(b, 1, 1).expand_as(cand[..., :self.RETRIES]),
                               cand[..., :self.RETRIES])
        ok = ~bad
        first = ok.to(torch.int8).argmax(dim=-1, keepdim=True)
        neg = torch.where(ok.any(dim=-1), cand.gather(-1, first).squeeze(-1), cand[..., -1])
        return u, p, neg
