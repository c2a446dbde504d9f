"""Whole-network parity: hcat.unet.Unet_Constructor on the MI355X vs the CPU
oracle (oracle/unet_oracle.py, itself pinned to the reference by
tests/golden/).  Covers train-mode forward, loss, every parameter gradient,
running statistics, the Adam step and eval-mode forward."""
import numpy as np
import pytest
import torch

from hcat.loss import cross_entropy
from hcat.unet import Unet_Constructor
from hcunet_amd.optim import Adam
from oracle import inputs, unet_oracle as uo
from tests.helpers import REF_KW

pytestmark = pytest.mark.gpu

CONFIGS = {
    'l2': (dict(REF_KW, feature_sizes=[2, 4]), (2, 4, 18, 18, 3)),
    'l3': (dict(REF_KW, feature_sizes=[4, 8, 16]), (2, 4, 44, 44, 5)),
    'l4': (dict(REF_KW, feature_sizes=[4, 8, 16, 32]), (1, 4, 92, 92, 6)),
    'l5_min': (dict(REF_KW, feature_sizes=[8, 16, 32, 64, 128]), (2, 4, 188, 188, 6)),
    'g2_up8': (dict(REF_KW, feature_sizes=[4, 8, 16], groups=2, upsample_kernel=(8, 8, 2)),
               (1, 4, 64, 60, 6)),
    'dil': (dict(REF_KW, feature_sizes=[4, 8, 16], dilation={'conv1': (2, 2, 1), 'conv2': 1}),
            (1, 4, 68, 66, 6)),
    'odd': (dict(image_dimensions=3, in_channels=3, out_channels=2, feature_sizes=[6, 12],
                 kernel={'conv1': (3, 3, 3), 'conv2': (3, 3, 1)}, upsample_kernel=(2, 2, 2),
                 max_pool_kernel=(2, 2, 2), upsample_stride=(2, 2, 2)), (2, 3, 22, 20, 13)),
}

# Parameters whose exact gradient is 0 (a bias feeding a train-mode BatchNorm):
# judged with an absolute tolerance.
def _bn_cancelled(name):
    return name.endswith('conv1.bias') or name.endswith('conv2.bias') or name.endswith('up_conv.bias')


def _build(kw, shape):
    torch.manual_seed(0)
    m = Unet_Constructor(**kw)
    spec = uo.normalize_spec(**kw)
    state = {k: v.detach().clone() for k, v in m.state_dict().items()}
    x = inputs.make_x(shape)
    return m, spec, state, x


def _mask_pwl(out_shape, pad=(3, 2, 1)):
    B, C, X, Y, Z = out_shape
    ms = (B, C, X + pad[0], Y + pad[1], Z + pad[2])
    return inputs.make_mask(ms), inputs.make_pwl(ms)


@pytest.mark.parametrize("name", list(CONFIGS))
def test_train_step_parity(name):
    kw, shape = CONFIGS[name]
    m, spec, state, x = _build(kw, shape)
    ref32 = uo.train_step(spec, state, x, *_mask_pwl(_oshape(spec, state, x)), dtype=torch.float32)
    ref64 = uo.train_step(spec, state, x, *_mask_pwl(_oshape(spec, state, x)), dtype=torch.float64)
    mask, pwl = _mask_pwl(tuple(ref32['out'].shape))
    m = m.cuda().train()
    opt = Adam(m.parameters(), lr=1e-3)
    opt.zero_grad()
    out = m(torch.from_numpy(x).cuda())
    loss = cross_entropy(out, torch.from_numpy(mask).cuda(), torch.from_numpy(pwl).cuda(),
                         method='pixel')
    loss.backward()
    torch.cuda.synchronize()
    # forward output: within 1e-4 of the fp32 reference (north-star bar)
    err_out = (out.detach().cpu().double() - ref32['out'].double()).abs().max().item()
    assert out.shape == ref32['out'].shape
    assert err_out <= 1e-4, err_out
    assert abs(loss.item() - ref64['loss'].item()) <= 1e-5 * max(1.0, abs(ref64['loss'].item()))
    # gradients: vs fp64 oracle, tolerance tied to the reference's own fp32 noise
    names = uo.param_names(spec)
    params = dict(m.named_parameters())
    # A ReLU input or max-pool top-2 gap of the fp64 step within fp32 rounding
    # reach makes the gradient routing itself undetermined: the GPU may take
    # the other branch than the fp32 reference even though both are right (l5_min
    # at 188x188x6: down_steps.3.batch1 has a pre-ReLU value of 3.3e-6, and a
    # flip there moves every encoder gradient below it by ~3e-3 relative L2).
    # Such steps are judged on relative L2 with a 1e-2 floor instead of 3e-4.
    rl2_floor = 1e-2 if uo.tie_margin(spec, state, x) < 1e-5 else 3e-4
    worst = []
    for n in names:
        g = params[n].grad.detach().cpu().double()
        g64 = ref64['grads'][n].double()
        g32 = ref32['grads'][n].double()
        err = (g - g64).abs().max().item()
        if _bn_cancelled(n):
            tol = 1e-4
        else:
            ref_noise = (g32 - g64).abs().max().item()
            tol = max(8 * ref_noise, 2e-5 * g64.abs().max().item(), 1e-7)
            # A max-pool window whose two largest fp32 values are nearly equal can
            # pick a different argmax under any change of summation order; the
            # gradient of that voxel is then routed to its neighbour.  The fp32
            # reference itself does this against fp64 (config g2_up8: 1.3e-2
            # relative L2).  Such a tensor passes on its relative L2 error instead.
            nrm = max(g64.norm().item(), 1e-30)
            rl2 = (g - g64).norm().item() / nrm
            rl32 = (g32 - g64).norm().item() / nrm
            if err > tol and rl2 <= max(8 * rl32, rl2_floor):
                err = 0.0
        worst.append((err / tol, n, err, tol))
    worst.sort(reverse=True)
    assert worst[0][0] <= 1.0, worst[:5]
    # running statistics after the train-mode forward
    sd = m.state_dict()
    for bn in uo.bn_names(spec):
        for s in ('running_mean', 'running_var'):
            a = sd[bn + '.' + s].cpu().double()
            b = ref32['state_after'][bn + '.' + s].double()
            assert (a - b).abs().max().item() <= 1e-5 * max(1.0, b.abs().max().item()), (bn, s)
        assert int(sd[bn + '.num_batches_tracked']) == 1
    # Adam step
    opt.step()
    torch.cuda.synchronize()
    for n in names:
        a = params[n].detach().cpu().double()
        b = ref64['state_after'][n].double()
        # one Adam step moves each weight by ~lr; sign flips of tiny grads move it by 2*lr
        frac_bad = ((a - b).abs() > 1e-5).double().mean().item()
        if rl2_floor > 3e-4:
            # routing-undetermined step: the first Adam step is p - lr*g/(|g|+eps),
            # so check it exactly on the GPU's own gradient instead
            g = params[n].grad.detach().cpu().double()
            b = state[n].double() - 1e-3 * g / (g.abs() + 1e-8)
            frac_bad = ((a - b).abs() > 1e-6 + 1e-6 * b.abs()).double().mean().item()
        assert frac_bad <= 0.01 or _bn_cancelled(n), (n, frac_bad)
    # eval-mode forward with the updated weights and running stats
    m.eval()
    with torch.no_grad():
        oe = m(torch.from_numpy(x).cuda()).cpu()
    net = uo.OracleUnet(spec, {k: v.cpu() for k, v in m.state_dict().items()})
    with torch.no_grad():
        re = net.forward(torch.from_numpy(x), training=False)
    assert (oe.double() - re.double()).abs().max().item() <= 1e-4


def _oshape(spec, state, x):
    net = uo.OracleUnet(spec, state)
    with torch.no_grad():
        return tuple(net.forward(torch.from_numpy(x), training=False).shape)


def test_deterministic_bitwise():
    kw, shape = CONFIGS['l3']
    m, spec, state, x = _build(kw, shape)
    m = m.cuda()
    xs = torch.from_numpy(x).cuda()
    res = []
    for _ in range(2):
        m.load_state_dict({k: v.cuda() for k, v in state.items()})
        for p in m.parameters():
            p.grad = None
        out = m(xs)
        out.sum().backward()
        torch.cuda.synchronize()
        res.append((out.detach().clone(), [p.grad.clone() for p in m.parameters()]))
    assert torch.equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        assert torch.equal(a, b)


def test_grad_accumulation_and_input_grad():
    kw, shape = CONFIGS['l2']
    m, spec, state, x = _build(kw, shape)
    m = m.cuda()
    xs = torch.from_numpy(x).cuda().requires_grad_(True)
    out = m(xs)
    out.sum().backward()
    g1 = [p.grad.clone() for p in m.parameters()]
    dx = xs.grad.detach().cpu().double()
    m.load_state_dict({k: v.cuda() for k, v in state.items()})
    out = m(xs)
    out.sum().backward()
    for p, a in zip(m.parameters(), g1):
        assert torch.allclose(p.grad, 2 * a, rtol=1e-5, atol=1e-7)
    net = uo.OracleUnet(spec, state, dtype=torch.float64)
    xr = torch.from_numpy(x).double().requires_grad_(True)
    net.forward(xr).sum().backward()
    assert (dx - xr.grad).abs().max().item() <= 1e-5 * xr.grad.abs().max().item() + 1e-7


def test_full_config2_forward_parity():
    """Config 2 at full size: [2,4,256,256,16] -> [2,1,68,68,11] within 1e-4 of
    the fp32 CPU reference restatement."""
    kw = dict(REF_KW, feature_sizes=[8, 16, 32, 64, 128])
    m, spec, state, x = _build(kw, (2, 4, 256, 256, 16))
    net = uo.OracleUnet(spec, state)
    with torch.no_grad():
        ref = net.forward(torch.from_numpy(x), training=True)
    m = m.cuda().train()
    with torch.no_grad():
        out = m(torch.from_numpy(x).cuda()).cpu()
    assert out.shape == (2, 1, 68, 68, 11)
    assert (out.double() - ref.double()).abs().max().item() <= 1e-4
