"""Group-and-Shuffle (GAS) layer over the MI355X GAS kernel.

Reference: src/models/orthogonal_bundle/group_shuffle_layer.py:12-189. Parameters and
buffers keep the reference's names and creation order (skew_params: d/bs [bs,bs] tensors
drawn N(0,1)*init_scale, then perm = randperm(d)), so a seeded construction yields the same
layer. Forward: y = (x @ blockdiag(expm(P_b - P_b^T)))[:, perm]. The 8x8 exponentials are a
host-side/tiny torch op; the per-row transform (8 MACs per output, 2 flop/B: HBM-bound) is a
VALU kernel, or an epilogue of the producing SpMM (ops.spmm_gas / ops.ngcf_layer).
"""
from typing import Tuple

import torch
import torch.nn as nn

from ... import ops


def param_key(params) -> tuple:
    """Identity + in-place version of a parameter list (cache key for derived matrices)."""
    return tuple((p.data_ptr(), p._version, p.device) for p in params)


class GroupShuffleLayer(nn.Module):
    def __init__(self, dim: int, block_size: int, init_scale: float = 0.01):
        super().__init__()
        if dim % block_size != 0:
            raise ValueError(f"dim ({dim}) must be divisible by block_size ({block_size})")
        self.dim = dim
        self.block_size = block_size
        self.n_blocks = dim // block_size
        self.skew_params = nn.ParameterList(
            nn.Parameter(torch.randn(block_size, block_size) * init_scale)
            for _ in range(self.n_blocks))
        self.register_buffer("perm", self._create_shuffle_permutation())

    def _create_shuffle_permutation(self) -> torch.Tensor:
        return torch.randperm(self.dim)

    # ---- the orthogonal group element ------------------------------------------------------
    def blocks(self) -> torch.Tensor:
        """[n_blocks, bs, bs] = expm(P_b - P_b^T) (group_shuffle_layer.py:110-124).
        Without autograd the result is cached until a parameter changes (matrix_exp on the
        device synchronises with the host, so recomputing it every forward costs more than
        the propagation kernels)."""
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.skew_params):
            return self._compute_blocks()
        key = param_key(self.skew_params)
        if getattr(self, "_blocks_key", None) != key:
            self._blocks_cache = self._compute_blocks().detach()
            self._blocks_key = key
        return self._blocks_cache

    def _compute_blocks(self) -> torch.Tensor:
        out = []
        for p in self.skew_params:
            a = p - p.T
            try:
                out.append(torch.matrix_exp(a))
            except RuntimeError:
                out.append(self._matrix_exp_alternative(a))
        return torch.stack(out)

    def _build_orthogonal_matrix(self) -> torch.Tensor:
        return torch.block_diag(*self.blocks().unbind(0))

    def _matrix_exp_alternative(self, A: torch.Tensor, n_terms: int = 10) -> torch.Tensor:
        """Truncated Taylor series I + A + A^2/2! + ... (group_shuffle_layer.py:131-154)."""
        result = torch.eye(A.size(0), device=A.device, dtype=A.dtype)
        term = torch.eye(A.size(0), device=A.device, dtype=A.dtype)
        fact = 1.0
        for i in range(1, n_terms + 1):
            term = term @ A
            fact *= i
            result = result + term / fact
        return result

    def fusable(self) -> bool:
        return not (torch.is_grad_enabled() and any(p.requires_grad for p in self.skew_params))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda and x.dim() == 2 and self.fusable() and self.dim in (16, 32, 64, 128) \
                and self.block_size <= 32 and not x.requires_grad:
            return ops.gas(x, self.blocks(), self.perm)
        W = self._build_orthogonal_matrix()
        return (x @ W)[:, self.perm]

    # ---- monitors (group_shuffle_layer.py:156-184) ----------------------------------------
    def get_orthogonality_error(self) -> torch.Tensor:
        W = self._build_orthogonal_matrix()
        eye = torch.eye(self.dim, device=W.device, dtype=W.dtype)
        return torch.norm(W.T @ W - eye, p="fro")

    def get_orthogonality_metrics(self) -> Tuple[torch.Tensor, torch.Tensor]:
        W = self._build_orthogonal_matrix()
        diff = W.T @ W - torch.eye(self.dim, device=W.device, dtype=W.dtype)
        return torch.norm(diff, p="fro"), diff.abs().max()

    def reset_parameters(self):
        for p in self.skew_params:
            nn.init.normal_(p, mean=0.0, std=0.01)
