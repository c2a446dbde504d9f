"""The loss oracle (oracle/loss_oracle.py) against the reference's own outputs
(tests/golden/loss_methods.npz, made by tests/golden/make_loss_golden.py)."""
import os

import numpy as np
import pytest
import torch

from oracle import loss_oracle as lo

GOLD = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'loss_methods.npz'))
CASES = sorted({k.split('.')[0] for k in GOLD.files if not k.startswith('err.')})


def case_inputs(name):
    pred = torch.from_numpy(GOLD[name + '.pred'])
    mask = torch.from_numpy(GOLD[name + '.mask'])
    pwl = torch.from_numpy(GOLD[name + '.pwl']) if name + '.pwl' in GOLD.files else None
    return pred, mask, pwl


def call(mod, name, pred, mask, pwl):
    fn, method, n = CASE_FN[name]
    if fn == 'cross_entropy':
        return mod.cross_entropy(pred, mask, pwl, method=method, num_random_pixels=n)
    return getattr(mod, fn)(pred, mask)


CASE_FN = {
    'ce_worst_z_f16': ('cross_entropy', 'worst_z', None),
    'ce_worst_z_f32_nopwl': ('cross_entropy', 'worst_z', None),
    'ce_sigmoid_f16': ('cross_entropy', 'sigmoid', None),
    'ce_sigmoid_f32_nopwl': ('cross_entropy', 'sigmoid', None),
    'ce_random_f16': ('cross_entropy', 'random', 50),
    'ce_random_f32_big_n': ('cross_entropy', 'random', 700),
    'ce_random_nopos': ('cross_entropy', 'random', 10),
    'ce_pixel_2d': ('cross_entropy', 'pixel', None),
    'dice_f32': ('dice', None, None),
    'dice_f16': ('dice', None, None),
    'l1_f32': ('L1Loss', None, None),
    'mse_f32': ('MSELoss', None, None),
    'l1_2d': ('L1Loss', None, None),
    'mse_2d': ('MSELoss', None, None),
}


def test_cases_cover_golden():
    assert set(CASES) == set(CASE_FN)


@pytest.mark.parametrize('name', CASES)
def test_oracle_matches_reference(name):
    pred, mask, pwl = case_inputs(name)
    pr = pred.clone().requires_grad_(True)
    torch.manual_seed(int(GOLD[name + '.seed']))
    val = call(lo, name, pr, mask, pwl)
    val.backward()
    # same arithmetic as the reference: bit-for-bit equal
    assert val.item() == float(GOLD[name + '.loss'])
    np.testing.assert_array_equal(pr.grad.numpy(), GOLD[name + '.grad'])


def test_oracle_errors_match_reference():
    z = torch.zeros(1, 1, 4, 4, 4)
    calls = {
        'bad_method': lambda: lo.cross_entropy(z, z, z, method='bogus'),
        'random_none': lambda: lo.cross_entropy(z, z, z, method='random'),
        'random_one': lambda: lo.cross_entropy(z, z, z, method='random', num_random_pixels=1),
        'random_no_background': lambda: lo.cross_entropy(z, torch.ones_like(z), z, method='random',
                                                         num_random_pixels=5),
        'dice_3dim': lambda: lo.dice(torch.zeros(2, 3, 4), torch.zeros(2, 3, 4)),
        'l1_3dim': lambda: lo.L1Loss(torch.zeros(2, 3, 4), torch.zeros(2, 3, 4)),
        'ce_3dim': lambda: lo.cross_entropy(torch.zeros(2, 3, 4), torch.zeros(2, 3, 4), None),
    }
    for key, fn in calls.items():
        want = str(GOLD['err.' + key])
        try:
            fn()
            got = 'none'
        except Exception as e:  # noqa: BLE001
            got = type(e).__name__
        assert got == want, key
