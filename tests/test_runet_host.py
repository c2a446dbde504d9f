"""CPU checks of the drop-in hcat.r_unet modules: torch's default
initialisation in the reference's module order (state_dict keys and values
equal to the reference's own, tests/golden/runet_*.npz), and no CPU compute
path (the forward raises without a ROCm device)."""
import os

import numpy as np
import pytest
import torch

from hcat.r_unet import RDCNet, RecursiveUnet, StackedDilation, RDCBlock, f, crop

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def test_rdcnet_init_and_keys_match_reference():
    g = np.load(os.path.join(GOLD, 'runet_rdc.npz'))
    torch.manual_seed(int(g['seed']))
    net = RDCNet(4, 5)
    keys = [k[5:] for k in g.files if k.startswith('init.')]
    assert list(net.state_dict().keys()) == keys
    for k, v in net.state_dict().items():
        np.testing.assert_array_equal(v.numpy(), g['init.' + k], err_msg=k)


def test_recursive_unet_keys_match_reference():
    g = np.load(os.path.join(GOLD, 'runet_rec.npz'))
    torch.manual_seed(int(g['seed']))
    net = RecursiveUnet(image_dimensions=3)
    keys = [k[5:] for k in g.files if k.startswith('init.')]
    assert list(net.state_dict().keys()) == keys
    assert net.model_specification['kernel'] == {'conv1': (3, 3, 3), 'conv2': (3, 3, 3)}
    assert isinstance(net.fz, f) and net.fz.down1 is net.down2_fz


def test_no_cpu_compute_path():
    net = RDCNet(3, 15)
    with pytest.raises(RuntimeError):
        net(torch.zeros(1, 3, 16, 16, 8))
    sd = StackedDilation(4, 4, 5)
    with pytest.raises(RuntimeError):
        sd(torch.zeros(1, 4, 8, 8, 8))
    assert isinstance(RDCBlock(4).grouped_conv, StackedDilation)
    a, b = torch.zeros(1, 2, 5, 6, 7), torch.zeros(1, 2, 3, 4, 5)
    assert crop(a, b).shape == (1, 2, 3, 4, 5)
