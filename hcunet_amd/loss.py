"""Drop-in hcat.loss.cross_entropy whose method='pixel' path runs in libhcunet.so.

Same signature, method validation and errors as hcat/loss.py:5-101.  The
'pixel' method -- the one on the training hot path -- is one fused HIP kernel:
top-left crop of mask/pwl to pred (:51-53), BCE-with-logits (:65,71),
multiplication by (pwl + 1) evaluated in pwl's dtype (:72), mean (:101), with
d(loss)/d(pred) produced in the same pass.  The reference's '+2 on mask' boost
(:61-63) is dead code there (is_pwl_none is always True, :45-48) and is
therefore not applied here either.
"""
import ctypes

import torch

from . import _lib

_DTYPES = {torch.float32: _lib.HCU_F32, torch.float16: _lib.HCU_F16,
           torch.uint8: _lib.HCU_U8, torch.bool: _lib.HCU_U8}


class _PixelBCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, mask, pwl):
        dev = pred.device
        B, C, PX, PY, PZ = pred.shape
        MX, MY, MZ = mask.shape[2:]
        loss = torch.empty((), dtype=torch.float32, device=dev)
        dpred = torch.empty_like(pred) if pred.requires_grad else None
        n = pred.numel()
        scratch = torch.empty(max(_lib.lib().hcu_loss_pixel_scratch_bytes(n), 16),
                              dtype=torch.uint8, device=dev)
        wdt = _DTYPES[pwl.dtype] if pwl is not None else _lib.HCU_F32
        _lib.check(_lib.lib().hcu_loss_pixel_fwd(
            _lib.ptr(pred), B, C, PX, PY, PZ, _lib.ptr(mask), _DTYPES[mask.dtype], _lib.ptr(pwl),
            wdt, MX, MY, MZ, _lib.ptr(loss), _lib.ptr(dpred), _lib.ptr(scratch),
            scratch.numel(), _lib.stream_handle(dev)), 'cross_entropy')
        ctx.save_for_backward(dpred)
        return loss

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad):
        (dpred,) = ctx.saved_tensors
        if dpred is None:
            return None, None, None
        grad = grad.contiguous().float()
        out = torch.empty_like(dpred)
        _lib.check(_lib.lib().hcu_scale_by_device_scalar(
            _lib.ptr(dpred), _lib.ptr(grad), _lib.ptr(out), dpred.numel(),
            _lib.stream_handle(dpred.device)), 'cross_entropy backward')
        return out, None, None


def cross_entropy(pred: torch.Tensor, mask: torch.Tensor, pwl: torch.Tensor, method='pixel',
                  num_random_pixels=None):
    """Pixel-weighted BCE-with-logits loss (hcat/loss.py:5).

    pred [B,C,X,Y,Z] logits; mask, pwl [B,C,X+dx,Y+dy,Z+dz] cropped top-left to
    pred; returns mean(BCE(pred, mask) * (pwl + 1)); pwl=None weighs 2.
    """
    _methods = ['pixel', 'worst_z', 'random', 'sigmoid']
    if method not in _methods:
        raise ValueError(f'Viable methods for cross entropy loss are {_methods}, not {method}.')
    if method == 'random':
        if num_random_pixels is None:
            raise ValueError('the number of random pixels to draw is not defined. Please set '
                             'num_random_pixels to a value larger than 1.')
        if num_random_pixels <= 1:
            raise ValueError(f'num_random_pixels should be greater than 1 not {num_random_pixels}.')
    if method != 'pixel':
        raise NotImplementedError(
            f"cross_entropy(method='{method}') is not on the accelerated path yet; "
            "only method='pixel' (the training hot path) is implemented")
    n_dim = pred.dim()
    if n_dim == 4:  # 2D: a 3D volume with Z = 1
        pred = pred.unsqueeze(-1)
        mask = mask.unsqueeze(-1)
        pwl = pwl.unsqueeze(-1) if pwl is not None else None
    elif n_dim != 5:
        raise IndexError('Unexpected number of predicted mask dimensions. Expected 4 (2D) or 5 (3D) '
                         f'but got {n_dim} dimensions: {pred.shape}')
    _lib.require_device(pred, 'pred')
    _lib.require_device(mask, 'mask')
    if mask.dim() != 5 or mask.shape[:2] != pred.shape[:2] or \
            any(m < p for m, p in zip(mask.shape[2:], pred.shape[2:])):
        raise ValueError(f'Target size ({list(mask.shape)}) must cover the input size '
                         f'({list(pred.shape)})')
    if pwl is not None:
        _lib.require_device(pwl, 'pwl')
        if pwl.shape != mask.shape:
            raise ValueError(f'pwl shape {list(pwl.shape)} must match mask shape {list(mask.shape)}')
        if pwl.dtype not in (torch.float32, torch.float16):
            pwl = pwl.float()
        pwl = pwl.contiguous()
    if mask.dtype not in _DTYPES:
        mask = mask.float()
    mask = mask.contiguous()
    if pred.dtype != torch.float32:
        pred = pred.float()  # hcat/loss.py:71 pred.float()
    pred = pred.contiguous()
    return _PixelBCE.apply(pred, mask, pwl)
