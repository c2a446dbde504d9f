#!/usr/bin/env python3
"""Generate tests/golden/loss_methods.npz from the REFERENCE hcat/loss.py.

Runs only in the development container (imports /root/reference through the
namespace shim of make_golden.py).  For each case it stores the inputs (small,
so stored whole), the reference's loss value and d(loss)/d(pred) from
autograd.  'random' cases record the torch.manual_seed used right before the
call: the reference draws its pixel indices from torch's default CPU
generator (hcat/loss.py:87-88), and the build consumes the same stream.

Usage:  python tests/golden/make_loss_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import import_reference  # noqa: E402

# name -> (function, method, pred shape, mask shape, mask dtype, pwl dtype or None, n_random, seed)
CASES = {
    'ce_worst_z_f16': ('cross_entropy', 'worst_z', (2, 1, 9, 8, 7), (2, 1, 12, 11, 9), 'f16', 'f16', None, 11),
    'ce_worst_z_f32_nopwl': ('cross_entropy', 'worst_z', (1, 2, 6, 5, 13), (1, 2, 6, 7, 13), 'f32', None, None, 12),
    'ce_sigmoid_f16': ('cross_entropy', 'sigmoid', (2, 1, 9, 8, 5), (2, 1, 12, 11, 7), 'f16', 'f16', None, 13),
    'ce_sigmoid_f32_nopwl': ('cross_entropy', 'sigmoid', (1, 1, 7, 7, 3), (1, 1, 7, 7, 3), 'f32', None, None, 14),
    'ce_random_f16': ('cross_entropy', 'random', (2, 1, 9, 8, 5), (2, 1, 12, 11, 7), 'f16', 'f16', 50, 15),
    'ce_random_f32_big_n': ('cross_entropy', 'random', (1, 1, 16, 16, 4), (1, 1, 16, 16, 4), 'f32', 'f32', 700, 16),
    'ce_random_nopos': ('cross_entropy', 'random', (1, 1, 5, 6, 3), (1, 1, 5, 6, 3), 'zeros', 'f16', 10, 17),
    'ce_pixel_2d': ('cross_entropy', 'pixel', (2, 1, 9, 8), (2, 1, 12, 11), 'f16', 'f16', None, 18),
    'dice_f32': ('dice', None, (2, 1, 9, 8, 5), (2, 1, 12, 11, 7), 'f32', None, None, 19),
    'dice_f16': ('dice', None, (1, 1, 6, 6, 4), (1, 1, 6, 6, 4), 'f16', None, None, 20),
    'l1_f32': ('L1Loss', None, (2, 1, 9, 8, 5), (2, 1, 12, 11, 7), 'f32', None, None, 21),
    'mse_f32': ('MSELoss', None, (2, 1, 9, 8, 5), (2, 1, 12, 11, 7), 'f32', None, None, 22),
    'l1_2d': ('L1Loss', None, (2, 1, 9, 8), (2, 1, 9, 10), 'f32', None, None, 23),
    'mse_2d': ('MSELoss', None, (1, 2, 5, 8), (1, 2, 5, 8), 'f32', None, None, 24),
}


def make_inputs(pshape, mshape, mdt, wdt, seed):
    g = torch.Generator().manual_seed(1000 + seed)
    pred = torch.randn(pshape, generator=g) * 2.5
    if mdt == 'zeros':
        mask = torch.zeros(mshape)
    else:
        mask = (torch.rand(mshape, generator=g) < 0.4).float()
        if mdt == 'f16':
            mask = mask.half()
    pwl = None
    if wdt is not None:
        pwl = torch.rand(mshape, generator=g) * 11.0
        pwl = pwl.half() if wdt == 'f16' else pwl
    return pred, mask, pwl


def main():
    _, loss = import_reference()
    out = {}
    for name, (fn, method, ps, ms, mdt, wdt, nr, seed) in CASES.items():
        pred, mask, pwl = make_inputs(ps, ms, mdt, wdt, seed)
        pr = pred.clone().requires_grad_(True)
        torch.manual_seed(seed)
        if fn == 'cross_entropy':
            val = loss.cross_entropy(pr, mask.clone(), None if pwl is None else pwl.clone(), method=method,
                                     num_random_pixels=nr)
        else:
            val = getattr(loss, fn)(pr, mask.clone())
        val.backward()
        out[name + '.pred'] = pred.numpy()
        out[name + '.mask'] = mask.numpy()
        if pwl is not None:
            out[name + '.pwl'] = pwl.numpy()
        out[name + '.loss'] = np.array(val.item(), dtype=np.float64)
        out[name + '.grad'] = pr.grad.numpy()
        out[name + '.seed'] = np.array(seed)
        print('%-24s loss %.8g  |grad| %.6g' % (name, val.item(), pr.grad.norm().item()))
    # error behaviour of the reference (exception type names)
    errs = {}
    z = torch.zeros(1, 1, 4, 4, 4)
    for key, call in {
        'bad_method': lambda: loss.cross_entropy(z, z, z, method='bogus'),
        'random_none': lambda: loss.cross_entropy(z, z, z, method='random'),
        'random_one': lambda: loss.cross_entropy(z, z, z, method='random', num_random_pixels=1),
        'random_no_background': lambda: loss.cross_entropy(z, torch.ones_like(z), z, method='random',
                                                           num_random_pixels=5),
        'dice_3dim': lambda: loss.dice(torch.zeros(2, 3, 4), torch.zeros(2, 3, 4)),
        'l1_3dim': lambda: loss.L1Loss(torch.zeros(2, 3, 4), torch.zeros(2, 3, 4)),
        'ce_3dim': lambda: loss.cross_entropy(torch.zeros(2, 3, 4), torch.zeros(2, 3, 4), None),
    }.items():
        try:
            call()
            errs[key] = 'none'
        except Exception as e:  # noqa: BLE001  (recording the reference's exception type)
            errs[key] = type(e).__name__
    for k, v in errs.items():
        out['err.' + k] = np.array(v)
        print('error %-22s %s' % (k, v))
    np.savez_compressed(os.path.join(HERE, 'loss_methods.npz'), **out)


if __name__ == '__main__':
    main()
