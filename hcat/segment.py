"""hcat.segment: re-export of the MI355X-native tiled inference driver
(hcunet_amd/segment.py; reference hcat/segment.py:21-136).  Only
predict_segmentation_mask is on the hot path; the watershed/RCNN
post-processing of the reference module is out of scope."""
from hcunet_amd.segment import predict_segmentation_mask  # noqa: F401
