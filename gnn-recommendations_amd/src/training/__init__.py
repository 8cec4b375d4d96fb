from .losses import BCELoss, BPRLoss, RegularizedLoss
from .sampler import DeviceSampler, ReferenceSampler
from .trainer import Trainer, bpr_scores, train_step

__all__ = ["BPRLoss", "BCELoss", "RegularizedLoss", "DeviceSampler", "ReferenceSampler",
           "Trainer", "bpr_scores", "train_step"]
