"""BASELINE config 3's bf16 path: the U-Net under torch.autocast(bf16).

The reference has no bf16 path of its own ("bf16 (config 3) has no
reference path"), so the question is: is this bf16 implementation as accurate
as the reference's ops under PyTorch's own bf16 autocast?  Each test runs
  fp32 oracle                      (the reference's arithmetic, CPU)
  oracle under torch.autocast(cpu, bfloat16)   (torch's bf16 policy, CPU)
  this build under torch.autocast(cuda, bfloat16)
on the same weights and inputs, and requires this build's distance to the
fp32 oracle to be within 1.5x of the autocast oracle's distance (output
relative L2, median per-tensor gradient relative L2; BN-cancelled conv biases
excluded: their exact value is 0), the loss within 1e-2 relative, plus
absolute sanity bounds.  bf16 keeps 8 significant bits; with BatchNorm over few voxels
the bf16 gradients of these small nets differ from fp32 by tens of percent for
torch's own autocast as well (measured: 5-level [32..512] at 188x188x6, B=4:
output 18 %, median gradient 75 %), so a fixed 1e-2 bar is not attainable by
any bf16 implementation at these sizes."""
import numpy as np
import pytest
import torch

from hcat.loss import cross_entropy
from hcat.unet import Unet_Constructor
from oracle import inputs, unet_oracle as uo
from tests.helpers import REF_KW

pytestmark = pytest.mark.gpu

CFG3 = dict(REF_KW, feature_sizes=[32, 64, 128, 256, 512])
SLACK = 1.5


def _rl2(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / max(b.norm().item(), 1e-30)).item()


def _cancelled(n):
    return n.endswith(('conv1.bias', 'conv2.bias', 'up_conv.bias'))


def _metrics(out, loss, grads, ref):
    g = {n: _rl2(grads[n], ref['grads'][n]) for n in grads if not _cancelled(n)}
    return dict(out=_rl2(out, ref['out']),
                loss=abs(float(loss) - ref['loss'].item()) / abs(ref['loss'].item()),
                grad_median=float(np.median(list(g.values()))), grads=g)


def _run(kw, shape, x_dtype=torch.float32):
    torch.manual_seed(0)
    m = Unet_Constructor(**kw)
    spec = uo.normalize_spec(**kw)
    state = {k: v.detach().clone() for k, v in m.state_dict().items()}
    x = torch.from_numpy(inputs.make_x(shape)).to(x_dtype)
    xf = x.float()
    with torch.no_grad():
        oshape = tuple(uo.OracleUnet(spec, state).forward(xf).shape)
    mask, pwl = inputs.make_mask(oshape), inputs.make_pwl(oshape)
    ref = uo.train_step(spec, state, xf.numpy(), mask, pwl, dtype=torch.float32)
    # the reference ops under torch's bf16 autocast (CPU)
    net = uo.OracleUnet(spec, state)
    with torch.autocast('cpu', dtype=torch.bfloat16):
        out_a = net.forward(xf)
        loss_a = uo.pixel_loss(out_a.float(), torch.from_numpy(mask), torch.from_numpy(pwl))
    loss_a.backward()
    auto = _metrics(out_a.detach().float(), loss_a.item(), net.grads(), ref)
    # this build
    m = m.cuda().train()
    with torch.autocast('cuda', dtype=torch.bfloat16):
        out = m(x.cuda())
        loss = cross_entropy(out, torch.from_numpy(mask).cuda(), torch.from_numpy(pwl).cuda(),
                             method='pixel')
    loss.backward()
    torch.cuda.synchronize()
    assert out.dtype == torch.float32 and out.shape == ref['out'].shape
    ours = _metrics(out.detach().cpu(), loss.item(),
                    {n: p.grad.detach().cpu() for n, p in m.named_parameters()}, ref)
    sd = m.state_dict()
    ours['running_var'] = max(_rl2(sd[b + '.running_var'].cpu(), ref['state_after'][b + '.running_var'])
                              for b in uo.bn_names(spec))
    return ours, auto


def _check(ours, auto):
    print('bf16 vs fp32 oracle: ours out %.3g loss %.3g grad median %.3g running_var %.3g | '
          'torch autocast out %.3g loss %.3g grad median %.3g'
          % (ours['out'], ours['loss'], ours['grad_median'], ours['running_var'],
             auto['out'], auto['loss'], auto['grad_median']))
    assert np.isfinite(ours['out']) and np.isfinite(ours['grad_median'])
    assert ours['out'] <= SLACK * auto['out'] + 1e-3, (ours['out'], auto['out'])
    assert ours['loss'] <= 1e-2, (ours['loss'], auto['loss'])
    assert ours['grad_median'] <= SLACK * auto['grad_median'] + 1e-2
    assert ours['running_var'] <= 3e-2
    assert ours['out'] <= 0.3 and ours['loss'] <= 1e-2


def test_bf16_small_net():
    _check(*_run(dict(REF_KW, feature_sizes=[16, 32, 64]), (2, 4, 44, 44, 5)))


def test_bf16_config3_l5_min():
    """The config-3 network ([32..512]) at the smallest 5-level input, B=4."""
    _check(*_run(CFG3, (4, 4, 188, 188, 6)))


def test_bf16_config3_larger_tile():
    """Config 3 at 220x220x8: more voxels per BatchNorm channel."""
    _check(*_run(CFG3, (2, 4, 220, 220, 8)))


@pytest.mark.parametrize('x_dtype', [torch.float16, torch.bfloat16])
def test_bf16_16bit_volume_input(x_dtype):
    """16-bit confocal volumes go straight into the first kernel (no host cast)."""
    _check(*_run(dict(REF_KW, feature_sizes=[16, 32, 64]), (2, 4, 44, 44, 5), x_dtype=x_dtype))


def test_bf16_config3_full_size():
    """BASELINE config 3 exactly as benched: [32..512], B=4, 256x256x16 (the
    tilings come from the persistent table, as in bench.py)."""
    _check(*_run(CFG3, (4, 4, 256, 256, 16)))
