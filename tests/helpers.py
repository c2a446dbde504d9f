"""Shared helpers for the parity tests (channels-last plumbing, tolerances)."""
import ctypes

import torch

from hcunet_amd import _lib

REF_KW = dict(image_dimensions=3, in_channels=4, out_channels=1,
              kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)}, upsample_kernel=(2, 2, 2),
              max_pool_kernel=(2, 2, 1), upsample_stride=(2, 2, 1))


def rup4(c):
    return (c + 3) // 4 * 4


def to_cl(t):
    """NCXYZ -> channels-last [B,X,Y,Z,Cs] (zero-padded channels) on cuda."""
    B, C = t.shape[:2]
    cl = t.permute(0, 2, 3, 4, 1).contiguous()
    Cs = rup4(C)
    if Cs != C:
        cl = torch.cat([cl, torch.zeros(*cl.shape[:-1], Cs - C, dtype=cl.dtype)], -1)
    return cl.float().cuda().contiguous()


def from_cl(t, C):
    return t[..., :C].permute(0, 4, 1, 2, 3).contiguous().cpu()


def desc(B, Cin, Cout, X, Y, Z, k, stride=(1, 1, 1), dil=(1, 1, 1), groups=1, transposed=0):
    d = _lib.ConvDesc()
    d.B, d.Cin, d.Cout, d.X, d.Y, d.Z = B, Cin, Cout, X, Y, Z
    d.k = _lib.c_int3(*k)
    d.stride = _lib.c_int3(*stride)
    d.dil = _lib.c_int3(*dil)
    d.groups = groups
    d.transposed = transposed
    return d


def out_dims(d):
    o = (ctypes.c_int * 3)()
    _lib.check(_lib.lib().hcu_conv_out_dims(ctypes.byref(d), o))
    return tuple(o)


def scratch_for(d):
    n = _lib.lib().hcu_conv_scratch_bytes(ctypes.byref(d))
    return torch.empty(max(n, 16), dtype=torch.uint8, device='cuda')


def stream():
    return _lib.stream_handle()


def max_abs(a, b):
    return (a.double() - b.double()).abs().max().item()
