from .gdn import GDN
from .layers import conv3x3, conv7x7, conv1x1, subpel_conv3x3, Win_noShift_Attention
from .win_attention import WindowAttention, WinBasedAttention, window_partition, window_reverse
from .compressai import (ResidualBlock, ResidualBlockWithStride, AttentionBlock, EntropyBottleneck,
                         GaussianConditional)
from ._conv import Conv2d, ConvTranspose2d, Linear
