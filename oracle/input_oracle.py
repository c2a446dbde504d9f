"""TEST INFRASTRUCTURE ONLY: numpy restatement of the reference's input path
for one volume, the parity oracle of hcunet_amd.ingest (tests only).

  to_float   hcat/transforms.py:94-116   uint16 / 2**16, uint8 / 2**8 in float64
  reshape    hcat/transforms.py:139-157  [Z,Y,X,C] -> [X,Y,Z,C] (swapaxes(ndim-2, 0))
  normalize  hcat/transforms.py:257-283  per channel (v + -mean) / std, float64
  to_tensor  hcat/transforms.py:118-137  float64 -> float32 -> fp16, [X,Y,Z,C] -> [1,C,X,Y,Z]

Pinned against the reference's own transforms by tests/golden/input_path.npz
(tests/golden/make_input_golden.py).
"""
import numpy as np


def to_float(a):
    if a.dtype == np.uint16:
        return a.astype(np.float64) / 2 ** 16
    if a.dtype == np.uint8:
        return a.astype(np.float64) / 2 ** 8
    if a.dtype == np.float64:
        return a
    raise TypeError('Expected image datatype of uint8 or uint16 ')


def reshape(a):
    return a.swapaxes(a.ndim - 2, 0)


def normalize(a, mean, std):
    a = a.copy()
    for c in range(a.shape[-1]):
        a[..., c] += -mean[c]
        a[..., c] /= std[c]
    return a


def to_tensor(a):
    """float64 [X,Y,Z,C] -> fp16 [1,C,X,Y,Z].  torch.as_tensor(float64, dtype=half)
    (hcat/transforms.py:133) rounds float64 -> float32 -> fp16, each to nearest
    even: so does this (a direct float64 -> fp16 rounding differs where the
    float32 value lands on an fp16 midpoint)."""
    return np.ascontiguousarray(np.moveaxis(a.astype(np.float32).astype(np.float16), -1, 0))[None]


def network_input(raw, mean=None, std=None):
    """to_float -> reshape -> (normalize) -> to_tensor of a [Z,Y,X,C] or [Z,Y,X] volume."""
    if raw.ndim == 3:
        raw = raw[..., None]
    a = reshape(to_float(raw))
    if mean is not None:
        a = normalize(a, mean, std)
    return to_tensor(a)
