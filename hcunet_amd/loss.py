"""Drop-in hcat.loss (cross_entropy, dice, L1Loss, MSELoss) running in libhcunet.so.

Same signatures, method validation and errors as hcat/loss.py:5-178.  The
'pixel' method -- the one on the training hot path -- is one fused HIP kernel:
top-left crop of mask/pwl to pred (:51-53), BCE-with-logits (:65,71),
multiplication by (pwl + 1) evaluated in pwl's dtype (:72), mean (:101), with
d(loss)/d(pred) produced in the same pass.  The reference's '+2 on mask' boost
(:61-63) is dead code there (is_pwl_none is always True, :45-48) and is
therefore not applied here either.  The other methods and losses
(loss_ext.hip) are a partial-sum pass, a fixed-order finalize and a gradient
pass each; 'random' draws its pixel indices from torch's default CPU generator
exactly as the reference does (hcat/loss.py:87-88), so a seeded run selects the
same pixels.
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


_MODE = {'sigmoid': 0, 'worst_z': 1, 'dice': 2, 'l1': 3, 'mse': 4, 'bce': 5, 'random': 6}


def _geom(pred, mask):
    B, C, PX, PY, PZ = pred.shape
    MX, MY, MZ = mask.shape[2:]
    return (B, C, PX, PY, PZ), (MX, MY, MZ)


class _LossExt(torch.autograd.Function):
    """One of loss_ext.hip's losses: forward = partial sums + finalize; backward
    = one gradient pass scaled by the upstream gradient on the device."""

    @staticmethod
    def forward(ctx, pred, mask, pwl, mode, num_random_pixels):
        dev = pred.device
        L = _lib.lib()
        pg, mg = _geom(pred, mask)
        n = pred.numel()
        loss = torch.empty((), dtype=torch.float32, device=dev)
        mdt = _DTYPES[mask.dtype]
        wdt = _DTYPES[pwl.dtype] if pwl is not None else _lib.HCU_F32
        counts_px = None
        stream = _lib.stream_handle(dev)
        if mode == _MODE['random']:
            rows = L.hcu_loss_random_rows(n)
            counts = torch.empty(rows, 2, dtype=torch.int32, device=dev)
            _lib.check(L.hcu_loss_random_count(_lib.ptr(pred), *pg, _lib.ptr(mask), mdt, *mg,
                                               _lib.ptr(counts), stream), 'cross_entropy')
            counts_h = counts.cpu().long()          # host sync, as the reference's int(...)
            npos, nneg = int(counts_h[:, 0].sum()), int(counts_h[:, 1].sum())
            if npos == 0:                            # hcat/loss.py:84-85
                mode = _MODE['bce']
            else:
                nr = num_random_pixels
                # hcat/loss.py:87-88: the same two draws from torch's default generator
                pos_ind = torch.randint(low=0, high=npos, size=(1, nr))[0, :]
                neg_ind = torch.randint(low=0, high=nneg, size=(1, nr))[0, :]
                offs = torch.zeros_like(counts_h)
                offs[1:] = torch.cumsum(counts_h, 0)[:-1]
                offs = offs.to(torch.int32).to(dev)
                pos_list = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
                neg_list = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
                pos_ind = pos_ind.to(dev)
                neg_ind = neg_ind.to(dev)
                counts_px = torch.zeros(n, dtype=torch.int32, device=dev)
                aux = torch.empty(1, dtype=torch.float32, device=dev)
                scratch = torch.empty(max(16, (2 * nr + 255) // 256) * 16, dtype=torch.uint8, device=dev)
                _lib.check(L.hcu_loss_random_fwd(
                    _lib.ptr(pred), *pg, _lib.ptr(mask), mdt, *mg, _lib.ptr(offs), _lib.ptr(pos_list),
                    _lib.ptr(neg_list), _lib.ptr(pos_ind), _lib.ptr(neg_ind), nr, _lib.ptr(counts_px),
                    _lib.ptr(loss), _lib.ptr(aux), _lib.ptr(scratch), scratch.numel(), stream),
                    'cross_entropy')
        if mode != _MODE['random']:
            PZ = pg[4]
            aux = torch.empty(max(2, PZ), dtype=torch.float32, device=dev)
            zscale = None
            if mode == _MODE['worst_z']:
                zscale = (torch.linspace(1, 2, PZ) ** 2).to(dev)   # hcat/loss.py:76
            scratch = torch.empty(L.hcu_loss_ext_scratch_bytes(mode, n, PZ), dtype=torch.uint8, device=dev)
            _lib.check(L.hcu_loss_ext_fwd(
                mode, _lib.ptr(pred), *pg, _lib.ptr(mask), mdt, _lib.ptr(pwl), wdt, *mg, _lib.ptr(zscale),
                _lib.ptr(loss), _lib.ptr(aux), _lib.ptr(scratch), scratch.numel(), stream), 'loss')
        ctx.mode = mode
        ctx.dt = (mdt, wdt)
        ctx.save_for_backward(pred, mask, pwl, aux, counts_px)
        return loss

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad):
        pred, mask, pwl, aux, counts_px = ctx.saved_tensors
        if not ctx.needs_input_grad[0]:
            return None, None, None, None, None
        grad = grad.contiguous().float()
        dpred = torch.empty_like(pred)
        pg, mg = _geom(pred, mask)
        mdt, wdt = ctx.dt
        _lib.check(_lib.lib().hcu_loss_ext_bwd(
            ctx.mode, _lib.ptr(pred), *pg, _lib.ptr(mask), mdt, _lib.ptr(pwl), wdt, *mg, _lib.ptr(aux),
            _lib.ptr(counts_px), _lib.ptr(grad), _lib.ptr(dpred), _lib.stream_handle(pred.device)),
            'loss backward')
        return dpred, None, None, None, None


def _prep(pred, mask, pwl, what):
    """Shared argument handling: 4D (2D images) become Z = 1 volumes, the
    reference's IndexError for other ranks (hcat/loss.py:54-56), device and
    dtype checks, contiguous fp32 pred."""
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
    return pred.contiguous(), mask, pwl


def cross_entropy(pred: torch.Tensor, mask: torch.Tensor, pwl: torch.Tensor, method='pixel',
                  num_random_pixels=None):
    """Weighted BCE-with-logits loss (hcat/loss.py:5-101).

    pred [B,C,X,Y,Z] logits; mask, pwl [B,C,X+dx,Y+dy,Z+dz] cropped top-left to
    pred.  'pixel': mean(BCE(pred, mask) * (pwl + 1)), pwl=None weighs 2;
    'sigmoid': the same on sigmoid(pred); 'worst_z': per-plane sums sorted
    ascending, weighted by linspace(1,2,Z)^2 / (X*Y), mean; 'random':
    mean BCE of num_random_pixels drawn foreground and as many background
    pixels.
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
        _lib.require_device(mask, 'mask')
        if not bool((mask == 0).any()):   # hcat/loss.py:35-36, on the uncropped mask
            raise ValueError('There are no background pixels in mask.\n\t(mask==0).sum() == 0 -> True')
    pred, mask, pwl = _prep(pred, mask, pwl, 'cross_entropy')
    if method == 'pixel':
        return _PixelBCE.apply(pred, mask, pwl)
    if method == 'random':
        return _LossExt.apply(pred, mask, None, _MODE['random'], int(num_random_pixels))
    return _LossExt.apply(pred, mask, pwl, _MODE[method], 0)


def dice(pred: torch.Tensor, mask: torch.Tensor):
    """1 - (2 sum(sigmoid(pred) * mask) + 1e-10) / (sum(sigmoid(pred) + mask) + 1e-10)
    (hcat/loss.py:104-126), mask cropped top-left to pred."""
    pred, mask, _ = _prep(pred, mask, None, 'dice')
    return _LossExt.apply(pred, mask, None, _MODE['dice'], 0)


def L1Loss(pred: torch.Tensor, mask: torch.Tensor):
    """mean |pred - mask| (hcat/loss.py:128-152), mask cropped top-left to pred."""
    pred, mask, _ = _prep(pred, mask, None, 'L1Loss')
    return _LossExt.apply(pred, mask, None, _MODE['l1'], 0)


def MSELoss(pred: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """mean (pred - mask)^2 (hcat/loss.py:154-178), mask cropped top-left to pred."""
    pred, mask, _ = _prep(pred, mask, None, 'MSELoss')
    return _LossExt.apply(pred, mask, None, _MODE['mse'], 0)
