"""hcat.dataloader: Stack on the MI355X input path (hcat/dataloader.py:17-92)."""
from hcunet_amd.dataloader import Stack  # noqa: F401
