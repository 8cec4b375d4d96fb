"""Ranking losses (reference: src/training/losses.py:12-160)."""
import torch
import torch.nn as nn
import torch.nn.functional as F


class BPRLoss(nn.Module):
    """mean(-log sigmoid(pos - neg)) (losses.py:12-53). The subtraction broadcasts: with the
    trainer's [B, 1] negative scores against [B] positives it is a [B, B] mean — the
    reference's behaviour, kept."""

    def forward(self, pos_scores: torch.Tensor, neg_scores: torch.Tensor) -> torch.Tensor:
        return -F.logsigmoid(pos_scores - neg_scores).mean()


class BCELoss(nn.Module):
    """Binary cross-entropy with logits over [pos; neg] (losses.py:56-92)."""

    def __init__(self):
        super().__init__()
        self.bce_loss = nn.BCEWithLogitsLoss()

    def forward(self, pos_scores: torch.Tensor, neg_scores: torch.Tensor) -> torch.Tensor:
        scores = torch.cat([pos_scores, neg_scores], dim=0)
        labels = torch.cat([torch.ones_like(pos_scores), torch.zeros_like(neg_scores)], dim=0)
        return self.bce_loss(scores, labels)


class RegularizedLoss(nn.Module):
    """base loss + weight_decay * sum ||p||_2^2 over the trainable parameters
    (losses.py:95-146)."""

    def __init__(self, base_loss: nn.Module, weight_decay: float = 1e-4):
        super().__init__()
        self.base_loss, self.weight_decay = base_loss, weight_decay

    def forward(self, pos_scores, neg_scores, model: nn.Module) -> torch.Tensor:
        loss = self.base_loss(pos_scores, neg_scores)
        if self.weight_decay > 0:
            l2 = 0.0
            for p in model.parameters():
                if p.requires_grad:
                    l2 = l2 + torch.norm(p, p=2) ** 2
            loss = loss + self.weight_decay * l2
        return loss
