"""CPU: pin the oracle (oracle/unet_oracle.py) against the reference's own
outputs (tests/golden/*.npz, written by tests/golden/make_golden.py from
/root/reference), and check that the drop-in Unet_Constructor reproduces the
reference's seeded initialisation and state_dict layout."""
import os

import numpy as np
import pytest
import torch

from oracle import inputs, unet_oracle as uo

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
KW = dict(image_dimensions=3, in_channels=4, out_channels=1,
          kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)}, upsample_kernel=(2, 2, 2),
          max_pool_kernel=(2, 2, 1), upsample_stride=(2, 2, 1))
NETS = {
    'unet_l2': dict(KW, feature_sizes=[2, 4]),
    'unet_l3': dict(KW, feature_sizes=[2, 4, 8]),
    'unet_l4': dict(KW, feature_sizes=[4, 8, 16, 32]),
    'unet_g2_up8': dict(KW, feature_sizes=[4, 8, 16], groups=2, upsample_kernel=(8, 8, 2)),
    'unet_dil': dict(KW, feature_sizes=[4, 8, 16], dilation={'conv1': (2, 2, 1), 'conv2': 1}),
    'unet_l5_min': dict(KW, feature_sizes=[8, 16, 32, 64, 128]),
}


def _load(name):
    return np.load(os.path.join(GOLD, name + '.npz'))


def _digest(t):
    t = torch.as_tensor(t).detach().double().reshape(-1)
    idx = (inputs.splitmix64(99, 64) % np.uint64(t.numel())).astype(np.int64)
    return np.concatenate([[t.sum().item(), t.norm().item(), t.abs().max().item()],
                           t[torch.from_numpy(idx)].numpy()])


def _cmp(a, g, full, rtol=1e-5, atol=1e-6):
    a = np.asarray(a if full else _digest(a), dtype=np.float64)
    g = np.asarray(g, dtype=np.float64)
    assert a.shape == g.shape
    np.testing.assert_allclose(a, g, rtol=rtol, atol=atol)


def _state_from_golden(d, full, spec):
    if full:
        return {k[5:]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith('init/')}
    return uo.init_state(spec, 0)  # summaries only: regenerate, then check the digest


@pytest.mark.parametrize('name', list(NETS))
def test_oracle_matches_reference(name):
    d = _load(name)
    kw = NETS[name]
    spec = uo.normalize_spec(**kw)
    full = 'init/out_conv.weight' in d.files and d['init/out_conv.weight'].ndim == 5
    state = _state_from_golden(d, full, spec)
    for k in d['state_keys']:
        _cmp(state[str(k)], d['init/' + str(k)], full, rtol=0, atol=0)
    shape = tuple(int(v) for v in d['input_shape'])
    ms = tuple(int(v) for v in d['mask_shape'])
    x = inputs.make_x(shape)
    mask, pwl = inputs.make_mask(ms), inputs.make_pwl(ms)
    r = uo.train_step(spec, state, x, mask, pwl)
    np.testing.assert_allclose(r['out'].numpy(), d['out'], rtol=0, atol=2e-6)
    assert abs(r['loss'].item() - float(d['loss'])) <= 1e-6 * abs(float(d['loss']))
    for n in d['param_names']:
        n = str(n)
        g = d['grad/' + n]
        scale = np.abs(g).max() if full else abs(g[2])
        _cmp(r['grads'][n], g, full, rtol=1e-4, atol=1e-4 * scale + 1e-9)
    for k in d.files:
        if k.startswith('stats/'):
            _cmp(r['state_after'][k[6:]], d[k], full, rtol=1e-5, atol=1e-6)
    for n in d['param_names']:
        n = str(n)
        # Adam moves ~lr per weight; tiny-gradient sign noise may flip a few weights.
        a = r['state_after'][n] if full else None
        if full:
            bad = np.abs(a.numpy() - d['adam/' + n]) > 1e-5
            assert bad.mean() <= 0.02, (n, bad.mean())
    # eval-mode forward after the step, from the reference's own updated state
    if full:
        st = {k[5:]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith('init/')}
        for n in d['param_names']:
            st[str(n)] = torch.from_numpy(np.array(d['adam/' + str(n)]))
        for k in d.files:
            if k.startswith('stats/'):
                st[k[6:]] = torch.from_numpy(np.array(d[k]))
        net = uo.OracleUnet(spec, st)
        with torch.no_grad():
            oe = net.forward(torch.from_numpy(x), training=False)
        np.testing.assert_allclose(oe.numpy(), d['out_eval'], rtol=0, atol=2e-6)


def test_oracle_fp64_matches_reference_fp64():
    d = _load('unet_l3')
    spec = uo.normalize_spec(**NETS['unet_l3'])
    state = _state_from_golden(d, True, spec)
    x = inputs.make_x(tuple(int(v) for v in d['input_shape']))
    ms = tuple(int(v) for v in d['mask_shape'])
    r = uo.train_step(spec, state, x, inputs.make_mask(ms), inputs.make_pwl(ms), dtype=torch.float64)
    np.testing.assert_allclose(r['out'].numpy(), d['f64/out'], rtol=0, atol=1e-12)
    for n in d['param_names']:
        np.testing.assert_allclose(r['grads'][str(n)].numpy(), d['f64/grad/' + str(n)],
                                   rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize('case', ['f16', 'f32', 'none', '2d'])
def test_oracle_pixel_loss_matches_reference(case):
    d = np.load(os.path.join(GOLD, 'loss_pixel.npz'))
    pred = torch.from_numpy(d[case + '/pred']).requires_grad_(True)
    mask = torch.from_numpy(d[case + '/mask'])
    pwl = torch.from_numpy(d[case + '/pwl']) if (case + '/pwl') in d.files else None
    loss = uo.pixel_loss(pred, mask, pwl)
    loss.backward()
    assert loss.item() == pytest.approx(float(d[case + '/loss']), rel=1e-6)
    np.testing.assert_allclose(pred.grad.numpy(), d[case + '/grad'], rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize('name', list(NETS))
def test_dropin_init_and_state_dict_match_reference(name):
    """hcat.unet.Unet_Constructor (the drop-in) consumes the RNG exactly like
    the reference: same keys, same order, same seeded values."""
    from hcat.unet import Unet_Constructor
    d = _load(name)
    full = d['init/out_conv.weight'].ndim == 5
    torch.manual_seed(0)
    m = Unet_Constructor(**NETS[name])
    sd = m.state_dict()
    assert [str(k) for k in d['state_keys']] == list(sd.keys())
    assert [str(n) for n in d['param_names']] == [n for n, _ in m.named_parameters()]
    for k, v in sd.items():
        _cmp(v, d['init/' + k], full, rtol=0, atol=0)


def test_dropin_errors_match_reference():
    from hcat.unet import Unet_Constructor
    d = np.load(os.path.join(GOLD, 'errors.npz'))

    def kind(fn):
        try:
            fn()
        except Exception as e:
            return type(e).__name__
        return 'none'
    assert kind(lambda: Unet_Constructor(image_dimensions=2, in_channels=4, out_channels=1,
                                         feature_sizes=[8, 16])) == str(d['err/2d'])
    assert kind(lambda: Unet_Constructor()) == str(d['err/default'])
    assert kind(lambda: Unet_Constructor(image_dimensions=4)) == str(d['err/dims4'])
    assert kind(lambda: Unet_Constructor(image_dimensions=3, feature_sizes=[8])) == \
        str(d['err/one_feature'])
    assert kind(lambda: Unet_Constructor(image_dimensions=3, feature_sizes=[8, 24])) == \
        str(d['err/not_doubling'])


def test_dropin_shape_errors_match_reference():
    """Errors the reference raises inside forward are raised by the native
    planner (host code, no GPU needed) with the same exception type."""
    from hcat.unet import Unet_Constructor
    from hcunet_amd.unet import _Plan, spec_struct
    d = np.load(os.path.join(GOLD, 'errors.npz'))

    def kind(fn):
        try:
            fn()
        except Exception as e:
            return type(e).__name__
        return 'none'
    m = Unet_Constructor(**dict(KW, feature_sizes=[8, 16, 32, 64, 128]))
    assert kind(lambda: _Plan(spec_struct(m), 1, 100, 100, 6)) == str(d['err/too_small'])
    m2 = Unet_Constructor(**dict(KW, feature_sizes=[2, 4], kernel={'conv1': (3, 3, 1),
                                                                   'conv2': (3, 3, 1)}))
    assert kind(lambda: _Plan(spec_struct(m2), 1, 20, 20, 3)) == str(d['err/up_exceeds_skip'])
