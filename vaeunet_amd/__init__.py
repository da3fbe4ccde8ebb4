"""MI355X-native (gfx950 HIP) training path for the tmuird/VAEUNET VAE-U-Net.

Drop-in surface (same names / signatures / state_dict keys as the reference):
  unet.UNet, unet.unet_parts.{DoubleConv, Down, Up, AttentionGate, OutConv},
  unet.unet_resnet.{UNetResNet, DecoderBlock}, utils.loss.*, utils.metrics.dice_score
Dispatcher ops: torch.ops.vaeunet.* (vaeunet_amd.ops)
"""
from .unet_model import UNet  # noqa: F401
from .unet_parts import AttentionGate, DoubleConv, Down, Up, OutConv  # noqa: F401
from .unet_resnet import UNetResNet, DecoderBlock  # noqa: F401,E402
from . import ops  # noqa: F401,E402  (registers torch.ops.vaeunet.*)
