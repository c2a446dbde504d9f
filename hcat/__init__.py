"""Import-light `hcat` namespace exposing the MI355X hot path under the
reference's own names (hcat/__init__.py:2 aliases Unet_Constructor as
hcat.unet).  Only the U-Net training path is provided; the reference's
detection/segmentation pipeline is out of scope."""
from hcat.unet import Unet_Constructor as unet  # noqa: F401
from hcat import loss  # noqa: F401
