"""TEST INFRASTRUCTURE ONLY: deterministic synthetic inputs.

Counter-based splitmix64 so that any tool (numpy here, a C++ loop elsewhere)
regenerates the same volumes without storing them:
  x    = (u16/65536 - 0.5) / 0.5   mimics uint16 -> to_float -> normalize
                                   (hcat/transforms.py:105-107, 273-275)
  mask = Bernoulli(0.5), float16   (to_tensor emits fp16, hcat/transforms.py:133)
  pwl  = U[0, 11) float16          (w0 = 11, hcat/train/train_utils.py:67)
Seeds: x=1, mask=2, pwl=3.
"""
import numpy as np

_G = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed, n):
    with np.errstate(over='ignore'):
        z = np.uint64(seed) * _G + (np.arange(n, dtype=np.uint64) + np.uint64(1)) * _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def make_x(shape, seed=1):
    n = int(np.prod(shape))
    u = (splitmix64(seed, n) & np.uint64(0xFFFF)).astype(np.float64)
    return ((u / 65536.0 - 0.5) / 0.5).astype(np.float32).reshape(shape)


def make_mask(shape, seed=2):
    n = int(np.prod(shape))
    b = (splitmix64(seed, n) >> np.uint64(32)) & np.uint64(1)
    return b.astype(np.float16).reshape(shape)


def make_pwl(shape, seed=3):
    n = int(np.prod(shape))
    h = (splitmix64(seed, n) >> np.uint64(40)).astype(np.float64)
    return (h / float(1 << 24) * 11.0).astype(np.float16).reshape(shape)
