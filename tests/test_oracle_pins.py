"""CPU check of the decision-pinned oracle (unet_oracle.pin_decisions).

Pins are taken from an fp32 oracle forward exactly as the GPU tests take them
from the GPU's saved workspace (pre-BatchNorm y + the scale/shift it was
normalised with).  The fp64 step pinned to those decisions must then agree
with the fp32 step on the same decisions to fp32 accumulation noise, while
the unpinned fp64 step (free to route near-ties differently) may not: that is
what makes the GPU gradient checks strict."""
import torch

from oracle import inputs, unet_oracle as uo
from tests.helpers import REF_KW


def _fp32_pins(spec, state, x):
    net = uo.OracleUnet(spec, state, dtype=torch.float32)
    ys, coefs = {}, {}
    bn = net._bn

    def rec(t, name, training):
        ys[name] = t.detach().clone()
        m = t.detach().double().mean(dim=(0, 2, 3, 4))
        v = t.detach().double().var(dim=(0, 2, 3, 4), unbiased=False)
        sc = (net.params[name + '.weight'].detach().double() / torch.sqrt(v + net.eps))
        sh = net.params[name + '.bias'].detach().double() - m * sc
        coefs[name] = (sc.float(), sh.float())
        return bn(t, name, training)

    net._bn = rec
    with torch.no_grad():
        net.forward(torch.as_tensor(x), training=True)
    return uo.pin_decisions(spec, ys, coefs)


def _rl2(a, b):
    return (a.double() - b.double()).norm().item() / max(b.double().norm().item(), 1e-30)


def test_pinned_fp64_matches_pinned_fp32():
    kw = dict(REF_KW, feature_sizes=[4, 8, 16, 32])
    spec = uo.normalize_spec(**kw)
    torch.manual_seed(0)
    state = uo.init_state(spec, 0)
    x = inputs.make_x((1, 4, 92, 92, 6))
    with torch.no_grad():
        oshape = tuple(uo.OracleUnet(spec, state).forward(torch.from_numpy(x)).shape)
    mask, pwl = inputs.make_mask(oshape), inputs.make_pwl(oshape)
    pins = _fp32_pins(spec, state, x)
    assert set(pins['pool']) == {0, 1, 2}
    p32 = uo.train_step(spec, state, x, mask, pwl, dtype=torch.float32, pins=pins)
    p64 = uo.train_step(spec, state, x, mask, pwl, dtype=torch.float64, pins=pins)
    worst = 0.0
    for n in uo.param_names(spec):
        if n.endswith(('conv1.bias', 'conv2.bias', 'up_conv.bias')):
            assert (p32['grads'][n] - p64['grads'][n].float()).abs().max() < 1e-4
            continue
        worst = max(worst, _rl2(p32['grads'][n], p64['grads'][n]))
    assert worst < 5e-5, worst   # fp32 accumulation noise; RL2_MAX on the GPU is 1e-4
    # the pinned forward is the forward (pins only change routing at near-ties)
    u64 = uo.train_step(spec, state, x, mask, pwl, dtype=torch.float64)
    assert (p64['out'] - u64['out']).abs().max().item() < 1e-6
