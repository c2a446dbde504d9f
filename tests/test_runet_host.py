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


def test_recursive_unet_save_load_roundtrip(tmp_path, monkeypatch):
    """RecursiveUnet.save / load (/root/reference/hcat/r_unet.py:164-204): the
    checkpoint keys and python_files capture of the reference, load re-running
    the default __init__ (:197) then load_state_dict + eval(), returning the
    hyper-parameters; a non-default geometry therefore fails to load with
    torch's size-mismatch RuntimeError, as in the reference."""
    monkeypatch.chdir(tmp_path)
    (tmp_path / 'loop.py').write_text('# a training script\n')
    torch.manual_seed(3)
    m = RecursiveUnet(image_dimensions=3)
    with torch.no_grad():
        for p in m.parameters():
            p.mul_(1.5)
        for b in m.modules():
            if isinstance(b, torch.nn.BatchNorm3d):
                b.running_mean.add_(0.125)
    m.save('rec.unet', hyperparameters={'epochs': 7})
    ck = torch.load('rec.unet', weights_only=True)
    assert set(ck) == {'state_dict', 'model_specifications', 'hyperparameters', 'python_files',
                       'tree_structure'}
    assert './loop.py' in ck['python_files'] and 'loop.py' in ck['tree_structure']
    m2 = RecursiveUnet(image_dimensions=3, out_channels=5)
    with torch.no_grad():
        for p in m2.parameters():
            p.zero_()
    assert m2.load('rec.unet', to_cuda=False) == {'epochs': 7}
    assert not m2.training
    assert m2.model_specification['image_dimensions'] == 2   # the defaults re-init (:197)
    sd, sd2 = m.state_dict(), m2.state_dict()
    assert list(sd) == list(sd2)
    for k in sd:
        assert torch.equal(sd[k], sd2[k]), k
    assert m2.fz.down1 is m2.down2_fz   # the re-init rebuilt the shared sub-networks
    # a checkpoint of another output width does not fit the default geometry
    RecursiveUnet(image_dimensions=3, out_channels=2).save('two.unet')
    with pytest.raises(RuntimeError):
        RecursiveUnet(image_dimensions=3).load('two.unet', to_cuda=False)
