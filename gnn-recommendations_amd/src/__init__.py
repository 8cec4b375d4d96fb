"""gnnrec-mi355x: MI355X-native drop-in for the propagation path of gnn-recommendations.

Same import surface as the reference's ``src`` package for the hot path
(``src.models``, ``src.data.graph_builder``); the kernels live in ``src.ops``.
"""
