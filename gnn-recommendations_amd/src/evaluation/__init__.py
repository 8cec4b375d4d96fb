from .evaluator import Evaluator, compute_metrics_from_topk

__all__ = ["Evaluator", "compute_metrics_from_topk"]
