"""hcat.transforms: the input-path transforms on the MI355X path (hcat/transforms.py:15-157,257-283)."""
from hcunet_amd.transforms import (PendingVolume, joint_transform, normalize, reshape,  # noqa: F401
                                   to_float, to_tensor)
