"""hcat.r_unet: re-export of the MI355X-native r_unet.py models (see hcunet_amd/r_unet.py)."""
from hcunet_amd.r_unet import (RecursiveUnet, RDCNet, f, Down, Up, StackedDilation,  # noqa: F401
                               RDCBlock, crop)
