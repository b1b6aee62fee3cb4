"""net_unet_ha_hs: net_ga's transforms / slice loop / syntax head with the U-Net
hyper networks (reference model/net_unet_ha_hs.py:658-1032, BASELINE config 3).

Reference behaviour reproduced: ``h_s`` ignores ``z_hat`` and consumes the
encoder-side ``middle_x``, ``down_x1`` and ``y`` (net_unet_ha_hs.py:880-895,
Block_unet.py:868-890); it is called twice with identical arguments, so
latent_scales == latent_means — computed once here (bitwise identical) and the
mean/scale slice supports share one buffer.
"""
import torch.nn as nn

from .. import functional as Fn
from ..functional import Act
from .Block_unet import Unet_ha_new, Unet_hs_new
from .net_ga import Net as _NetGA

__all__ = ["Net"]


class Net(_NetGA):
    arch = "net_unet_ha_hs"
    _eb_channels = 512
    _shared_support = True
    _codable = False   # h_s reads encoder-side features: no decodable bitstream

    def _build_hyper(self):
        self.h_a = Unet_ha_new(192, 8, 3)
        self.h_s = Unet_hs_new(192, 8, 3)

    def _hyper_s_modules(self):
        return [self.h_s]

    def _hyper(self, z3: Act, means_out: Act, scales_out: Act):
        z, middle_x, down_x1, inp = self.h_a.run(z3)                     # :880
        z_hat = Fn.quantize_median(z, self._medians(z.t.device))          # :885-889
        self.h_s.run(z_hat, middle_x, down_x1, inp, out=means_out)       # :892 / :895 (identical)
        return z, z_hat
