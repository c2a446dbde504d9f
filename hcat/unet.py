"""hcat.unet: re-export of the MI355X-native Unet_Constructor (see hcunet_amd/unet.py)."""
from hcunet_amd.unet import Unet_Constructor, Down, Up, crop  # noqa: F401
