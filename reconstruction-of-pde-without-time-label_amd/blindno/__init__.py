"""blindno -- MI355X-native (gfx950 HIP) implementation of BlinDNO's FNO/NIO training hot
path, drop-in for yl602019618/Reconstruction-of-PDE-without-Time-Label's
FNOModules / NIOModules / DeepONetModules / Baselines surface.

All numerics run in libblindno.so (HIP kernels behind the C ABI of include/blindno.h);
there is no CPU fallback.  Importing the package registers the hot-path operators as
``torch.ops.blindno.*`` (blindno/torch_ops.py).
"""
from . import _lib  # noqa: F401
from ._lib import BlindnoError, load as load_library  # noqa: F401
from .fno import FNO1d, FNO2d, FNO3d, MLP, SpectralConv1d, SpectralConv2d, SpectralConv3d  # noqa: F401
from .nio import (NIOFP, NIOFP2D, NIOFP2D_FNO, NIOFP2D_FNO_attn, NIOFP_FNO,  # noqa: F401
                  NIOFP_schrodinger, draw_bag)
from .deeponet import FFN, DeepOnetNoBiasOrg, FeedForwardNN  # noqa: F401
from .encoders import ConvBlock, Encoder, Encoder2D  # noqa: F401
from .unet import (PermInvUNet_attn, PermInvUNet_attn1D, PermInvUNet_attn1D_bag,  # noqa: F401
                   PermInvUNet_attn1D_bag_GPE, PermInvUNet_attn1D_bag_V, PermInvUNet_attn_NC)
from .ops import mse_loss, pad_amount, set_mix_precision  # noqa: F401
from . import torch_ops  # noqa: F401  (registers torch.ops.blindno.*)

__version__ = "0.1.0"
