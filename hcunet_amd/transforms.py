"""Drop-in hcat.transforms for the input path: to_float,
reshape, normalize and to_tensor with the reference's names, call convention
(joint lists through `joint_transform`, which also draws the reference's
per-call numpy seed, hcat/transforms.py:15-91) and errors.

The MI355X path is lazy: to_float / reshape / normalize only record what they
would do to the raw stack, and to_tensor runs the whole chain as ONE device
pass (csrc/ingest.hip, `hcu_ingest_volume`): the raw uint16 / uint8 volume is
copied to HBM as is (half or a quarter of the float64 bytes the reference
moves), scaled, transposed [Z,Y,X,C] -> [C,X,Y,Z] and normalised in float64
and rounded once to fp16 -- bit-identical to the reference's
to_float -> reshape -> normalize -> to_tensor, and returned on the GPU.

Reference: to_float hcat/transforms.py:94-116, to_tensor :118-137,
reshape :139-157, normalize :257-283.  The random augmentations of that file
(spekle, random_affine, elastic_deform, ...) are CPU data-loader work outside
the hot path and are not provided.
"""
import ctypes
import functools

import numpy as np
import torch

from . import _lib

_RAW = {np.dtype(np.uint16): _lib.HCU_U16, np.dtype(np.uint8): _lib.HCU_U8,
        np.dtype(np.float64): _lib.HCU_F64}
_TORCH_RAW = {torch.uint16: _lib.HCU_U16, torch.int16: _lib.HCU_U16, torch.uint8: _lib.HCU_U8,
              torch.float64: _lib.HCU_F64}


class PendingVolume:
    """A raw [Z,Y,X,C] (or [Y,X,C]) stack plus the recorded to_float / reshape /
    normalize steps, materialised by to_tensor on the device."""

    def __init__(self, raw, np_dtype=None):
        self.raw = raw
        self.np_dtype = np_dtype   # dtype of the file's array when raw holds its bits
        self.to_float = False
        self.reshaped = False
        self.mean = None
        self.std = None

    @property
    def ndim(self):  # joint_transform compares ndim across the list (:67-72)
        return self.raw.ndim

    @property
    def shape(self):
        s = tuple(self.raw.shape)
        if self.reshaped:
            s = (s[-2],) + s[1:-2] + (s[0], s[-1])
        return s

    def to_ndarray(self):
        """The ndarray the reference's eager chain would hold at this point
        (host numpy, same arithmetic: to_float :104-115, reshape :139-156,
        normalize :266-281), for transforms that need a real array (the
        reference's random augmentations check isinstance(image, np.ndarray))."""
        raw = self.raw
        if isinstance(raw, torch.Tensor):
            a = raw.detach().cpu().numpy()
            if self.np_dtype is not None and np.dtype(self.np_dtype) != a.dtype:
                a = a.view(self.np_dtype)
            elif raw.dtype == torch.int16:
                a = a.view(np.uint16)
        else:
            a = np.asarray(raw)
        if self.to_float:
            if a.dtype == np.uint16:
                a = a.astype(np.float64) / 2 ** 16
            elif a.dtype == np.uint8:
                a = a.astype(np.float64) / 2 ** 8
        else:
            a = a.copy()
        if self.reshaped:
            a = a.swapaxes(a.ndim - 2, 0)
        if self.mean is not None:
            a = np.ascontiguousarray(a)
            for c in range(a.shape[-1]):
                a[..., c] += -self.mean[c]
                a[..., c] /= self.std[c]
        return a

    def _dtype_code(self):
        if self.np_dtype is not None:
            return _RAW.get(np.dtype(self.np_dtype))
        if isinstance(self.raw, torch.Tensor):
            code = _TORCH_RAW.get(self.raw.dtype)
        else:
            code = _RAW.get(np.dtype(self.raw.dtype))
        return code


def _wrap(image):
    return image if isinstance(image, PendingVolume) else PendingVolume(image)


def joint_transform(func):
    """hcat/transforms.py:15-91: apply `func(self, image, seed)` to one image or
    to each image of a list with one seed drawn from numpy's global RNG."""
    @functools.wraps(func)
    def wrapper(*args):
        image_list = args[-1]
        if not type(image_list) == list:
            image_list = [image_list]
        if len(image_list) > 1:
            for i in range(len(image_list) - 1):
                if not image_list[i].ndim == image_list[i + 1].ndim:
                    raise ValueError('Images in joint transforms do not contain identical dimensions.'
                                     + f'Im {i}.ndim:{image_list[i].ndim} != Im {i + 1}.ndim:'
                                     f'{image_list[i + 1].ndim} ')
        seed = np.random.randint(0, 1e8, 1)   # :78, keeps numpy's RNG stream aligned
        out = [func(args[0], image=im, seed=seed) if len(args) > 1 else func(image=im, seed=seed)
               for im in image_list]
        return out[0] if len(out) == 1 else out
    return wrapper


class to_float:
    """uint16 / 2**16, uint8 / 2**8, float64 unchanged; other dtypes: TypeError."""

    @joint_transform
    def __call__(self, image, seed=None):
        v = _wrap(image)
        if v.to_float or v.mean is not None:
            return v
        code = v._dtype_code()
        if code is None:
            raise TypeError('Expected image datatype of uint8 or uint16 ')
        v.to_float = True
        return v


class reshape:
    """[Z,Y,X,C] -> [X,Y,Z,C] (swapaxes(ndim - 2, 0))."""

    @joint_transform
    def __call__(self, image, seed=None):
        if not isinstance(image, (np.ndarray, PendingVolume, torch.Tensor)):
            raise TypeError(f'Expected input type of np.ndarray but got {type(image)}')
        v = _wrap(image)
        if v.reshaped:   # a second swap undoes the first
            v.reshaped = False
        else:
            v.reshaped = True
        return v


class normalize:
    """Per channel (v + -mean) / std on a float image (defaults 0.5 / 0.5)."""

    def __init__(self, mean=None, std=None):
        self.mean = [0.5, 0.5, 0.5, 0.5] if mean is None else mean
        self.std = [0.5, 0.5, 0.5, 0.5] if std is None else std

    def __call__(self, image):
        if isinstance(image, list):   # :268-269: only the first image of a list
            image = image[0]
        v = _wrap(image)
        if v.ndim not in (3, 4):
            raise ValueError(f'Expected a 3 or 4 dimensional image not: {v.ndim} with shape: {v.shape}')
        if not v.to_float and v._dtype_code() != _lib.HCU_F64:
            raise TypeError('normalize expects a float image (apply to_float first)')
        if v.mean is not None:
            raise NotImplementedError('normalize applied twice to one volume')
        C = v.shape[-1]
        v.mean = [float(self.mean[c]) for c in range(C)]
        v.std = [float(self.std[c]) for c in range(C)]
        return v


class to_tensor:
    """[x,y,z,c] -> fp16 [1,c,x,y,z] on the current ROCm device, via one
    hcu_ingest_volume pass over the raw stack."""

    @joint_transform
    def __call__(self, image, seed=None):
        if not isinstance(image, (np.ndarray, PendingVolume)):
            raise TypeError(f'Expected list but got {type(image)}')
        return materialise(_wrap(image))


def _to_device_raw(raw, device):
    if isinstance(raw, torch.Tensor):
        t = raw
    else:
        a = np.ascontiguousarray(raw)
        if a.dtype == np.uint16:
            t = torch.from_numpy(a.view(np.int16))   # raw bits; the kernel reads uint16
        else:
            t = torch.from_numpy(a)
    if t.device.type != 'cuda':
        t = t.contiguous().pin_memory().to(device, non_blocking=True)
    return t.contiguous()


def materialise(v, device=None):
    """Run the recorded chain on the device: fp16 [1,C,X,Y,Z] (reshape applied)
    or [1,C,Z,Y,X] (not applied), as the reference's to_tensor returns."""
    code = v._dtype_code()
    if code is None:
        raise TypeError('Expected image datatype of uint8 or uint16 ')
    device = torch.device('cuda', torch.cuda.current_device()) if device is None else torch.device(device)
    raw = _to_device_raw(v.raw, device)
    shp = tuple(raw.shape)
    two_d = len(shp) == 3
    if two_d:          # [Y,X,C] image: a Z = 1 volume
        shp = (1,) + shp
    if len(shp) != 4:
        raise ValueError(f'Expected a [Z,Y,X,C] or [Y,X,C] stack, got shape {tuple(raw.shape)}')
    Z, Y, X, C = shp
    if v.reshaped:
        out = torch.empty((1, C, X, Y, Z), dtype=torch.float16, device=device)
    else:
        out = torch.empty((1, C, Z, Y, X), dtype=torch.float16, device=device)
    mean = std = None
    if v.mean is not None:
        mean = (ctypes.c_double * C)(*v.mean)
        std = (ctypes.c_double * C)(*v.std)
    with torch.cuda.device(device):
        _lib.check(_lib.lib().hcu_ingest_volume(
            _lib.ptr(raw), code, 1, Z, Y, X, C, int(v.to_float), int(v.reshaped), mean, std,
            _lib.ptr(out), _lib.stream_handle(device)), 'to_tensor')
    if two_d:          # [1,C,X,Y,1] -> [1,C,X,Y] / [1,C,1,Y,X] -> [1,C,Y,X]
        out = out[..., 0] if v.reshaped else out[:, :, 0]
    return out


def ingest(raw, mean=None, std=None, device=None):
    """Batched input path: raw [B,Z,Y,X,C] (or one [Z,Y,X,C] stack) uint16 /
    uint8 -> fp16 [B,C,X,Y,Z] = to_float -> reshape -> normalize(mean, std)
    -> to_tensor of each volume, in one launch."""
    device = torch.device('cuda', torch.cuda.current_device()) if device is None else torch.device(device)
    t = _to_device_raw(raw, device)
    if t.dim() == 4:
        t = t.unsqueeze(0)
    if t.dim() != 5:
        raise ValueError(f'Expected [B,Z,Y,X,C] or [Z,Y,X,C], got {tuple(t.shape)}')
    code = _TORCH_RAW.get(t.dtype)
    if code is None:
        raise TypeError('Expected image datatype of uint8 or uint16 ')
    B, Z, Y, X, C = t.shape
    out = torch.empty((B, C, X, Y, Z), dtype=torch.float16, device=device)
    m = s = None
    if mean is not None:
        m = (ctypes.c_double * C)(*[float(x) for x in mean[:C]])
        s = (ctypes.c_double * C)(*[float(x) for x in std[:C]])
    with torch.cuda.device(device):
        _lib.check(_lib.lib().hcu_ingest_volume(_lib.ptr(t), code, B, Z, Y, X, C, 1, 1, m, s, _lib.ptr(out),
                                                _lib.stream_handle(device)), 'ingest')
    return out
