"""Parameter helpers with the reference's module/buffer names (reference ops/):
``LowerBound`` (ops/bound_ops.py:63-84), ``NonNegativeParametrizer``
(ops/parametrizers.py:23-51), ``ste_round`` (ops/ops.py:20-34).

They hold the buffers that appear in the reference state_dict
(``...lower_bound.bound``, ``...pedestal``).  On the hot path the GDN
reparametrisation itself runs on device in ``lic_gdn_prepare``; these torch
forwards are kept for parameter initialisation / inspection only (they operate
on C- or C^2-element parameter tensors, never on activations).
"""
import torch
import torch.nn as nn

__all__ = ["LowerBound", "NonNegativeParametrizer", "ste_round"]


class LowerBound(nn.Module):
    """torch.max(x, bound) with the reference buffer name ``bound``."""

    def __init__(self, bound: float):
        super().__init__()
        self.register_buffer("bound", torch.Tensor([float(bound)]))

    def forward(self, x):
        return torch.max(x, self.bound)


class NonNegativeParametrizer(nn.Module):
    def __init__(self, minimum: float = 0, reparam_offset: float = 2 ** -18):
        super().__init__()
        self.minimum = float(minimum)
        self.reparam_offset = float(reparam_offset)
        pedestal = self.reparam_offset ** 2
        self.register_buffer("pedestal", torch.Tensor([pedestal]))
        bound = (self.minimum + self.reparam_offset ** 2) ** 0.5
        self.lower_bound = LowerBound(bound)

    def init(self, x):
        return torch.sqrt(torch.max(x + self.pedestal, self.pedestal))

    def forward(self, x):
        out = self.lower_bound(x)
        return out ** 2 - self.pedestal


def ste_round(x):
    """Forward value of the straight-through round (== torch.round(x) bitwise)."""
    return torch.round(x) - x.detach() + x
