"""hcat.utils: re-export of the tiling helpers of the inference driver
(hcunet_amd/segment.py; reference hcat/utils.py:33-124)."""
from hcunet_amd.segment import pad_image_with_reflections, calculate_indexes  # noqa: F401
