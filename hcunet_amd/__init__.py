"""hcunet_amd: MI355X-native (gfx950) 3D U-Net training hot path.

Drop-in for hcat.unet.Unet_Constructor + hcat.loss.cross_entropy(method='pixel')
+ the Adam step, with all arithmetic in hand-written HIP kernels
(libhcunet.so, C-ABI in include/hcunet.h).  See DESIGN.md.
"""
from . import _lib
from .unet import Unet_Constructor, Down, Up, crop
from .loss import cross_entropy
from .optim import Adam
from . import dist

__all__ = ['Unet_Constructor', 'Down', 'Up', 'crop', 'cross_entropy', 'Adam', 'dist']
