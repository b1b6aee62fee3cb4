"""source_net: the factorized-prior plumbing network of the reference (model/source_net.py),
BASELINE.json config 1.  Its forward (source_net.py:839-851) stops right after the hyper
analysis and returns z, so only a_model and h_a take part; every other sub-module of the
reference Net (s_model, hyper synthesis, entropy models, HAN, samplers, ...) is never
reached and its state_dict entries are accepted and ignored by load_state_dict.

HIP path: four ZeroPad2d((1,2,1,2)) + conv5x5 s2 launches (asymmetric pad as tap
offsets) with model/gdn.py GDN between them, then h_a = |.| (conv prologue) -> conv3x3
s1 + ReLU -> conv5x5 s2 + ReLU -> conv5x5 s2 (ReLUs fused into the conv epilogues).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import functional as Fn
from .._ffi import ACT_RELU, PRO_ABS
from ..functional import Act
from ..layers._conv import Conv2d
from .gdn import GDN
from .net_ga import weight_init

_PAD_5S2 = (1, 1, 2, 2)  # ZeroPad2d((1, 2, 1, 2)) as (top, left, bottom, right)


class analysisTransformModel(nn.Module):
    """source_net.py:252-279: 4 x [ZeroPad2d((1,2,1,2)), Conv2d(5, 2, 0)] with GDN between."""

    def __init__(self, in_dim, num_filters, conv_trainable=True):
        super().__init__()
        self.transform = nn.Sequential(
            nn.ZeroPad2d((1, 2, 1, 2)), Conv2d(in_dim, num_filters[0], 5, 2, 0), GDN(num_filters[0]),
            nn.ZeroPad2d((1, 2, 1, 2)), Conv2d(num_filters[0], num_filters[1], 5, 2, 0), GDN(num_filters[1]),
            nn.ZeroPad2d((1, 2, 1, 2)), Conv2d(num_filters[1], num_filters[2], 5, 2, 0), GDN(num_filters[2]),
            nn.ZeroPad2d((1, 2, 1, 2)), Conv2d(num_filters[2], num_filters[3], 5, 2, 0),
        )

    def run(self, x: Act) -> Act:
        t = self.transform
        for conv, gdn in ((t[1], t[2]), (t[4], t[5]), (t[7], t[8])):
            x = gdn.run(conv.run(x, pad=_PAD_5S2))
        return t[10].run(x, pad=_PAD_5S2)

    def forward(self, inputs):
        return self.run(Act.from_nchw(inputs.float().contiguous(), pad16=True)).nchw()


class h_analysisTransformModel(nn.Module):
    """source_net.py:347-361: |x| -> Conv2d(3, s0, 1), ReLU, Conv2d(5, s1, 2), ReLU, Conv2d(5, s2, 2)."""

    def __init__(self, in_dim, num_filters, strides_list, conv_trainable=True):
        super().__init__()
        self.transform = nn.Sequential(
            Conv2d(in_dim, num_filters[0], 3, strides_list[0], 1), nn.ReLU(),
            Conv2d(num_filters[0], num_filters[1], 5, strides_list[1], 2), nn.ReLU(),
            Conv2d(num_filters[1], num_filters[2], 5, strides_list[2], 2),
        )

    def run(self, x: Act) -> Act:
        t = self.transform
        x = t[0].run(x, prologue=PRO_ABS, act=ACT_RELU)
        x = t[2].run(x, act=ACT_RELU)
        return t[4].run(x)

    def forward(self, inputs):
        return self.run(Act.from_nchw(inputs.float().contiguous())).nchw()


class Net(nn.Module):
    """source_net.Net (source_net.py:632-851) for its reachable forward: returns z."""

    arch = "source_net"

    def __init__(self, train_size, test_size, is_high, post_processing, precision: str = "fp32"):
        super().__init__()
        self.train_size, self.test_size = train_size, test_size
        self.is_high, self.post_processing = is_high, post_processing
        self.precision = precision
        N = 384 if is_high else 192
        self.N, self.M = N, (32 if is_high else 16)
        self.a_model = analysisTransformModel(3, [N, N, N, N])
        self.a_model.apply(weight_init)
        self.h_a = h_analysisTransformModel(N, [N, N, N], [1, 2, 2])

    def _dtype(self):
        return {"fp16": torch.float16, "bf16": torch.bfloat16}.get(self.precision, torch.float32)

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        sd = {k: v for k, v in state_dict.items() if k.startswith(("a_model.", "h_a."))}
        return super().load_state_dict(sd, strict=strict, assign=assign)

    @torch.no_grad()
    def forward(self, inputs, mode='train', num=1):
        x = Act.from_nchw(inputs.float().contiguous(), self._dtype(), pad16=True)
        z3 = self.a_model.run(x)
        return Fn.to_nchw_f32(self.h_a.run(z3))
