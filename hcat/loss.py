"""hcat.loss: re-export of the MI355X-native pixel-weighted cross entropy."""
from hcunet_amd.loss import cross_entropy  # noqa: F401
