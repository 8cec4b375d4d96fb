from .losses import BCELoss, BPRLoss, RegularizedLoss
from .sampler import DeviceSampler, ReferenceSampler
from .optim import NativeAdam
from .trainer import Trainer, batch_rows, bpr_scores, make_adam, train_step
from .distributed import lightgcn_train_step_dist

__all__ = ["BPRLoss", "BCELoss", "RegularizedLoss", "DeviceSampler", "ReferenceSampler",
           "Trainer", "batch_rows", "bpr_scores", "make_adam", "NativeAdam", "train_step", "lightgcn_train_step_dist"]
