from .evaluator import Evaluator, compute_metrics_from_topk, embedding_statistics

__all__ = ["Evaluator", "compute_metrics_from_topk", "embedding_statistics"]
