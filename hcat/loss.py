"""hcat.loss: re-export of the MI355X-native losses (hcat/loss.py:5-178)."""
from hcunet_amd.loss import L1Loss, MSELoss, cross_entropy, dice  # noqa: F401
