#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the REFERENCE implementation itself.

Runs only in the development container, where /root/reference exists.  The
reference's hcat/__init__.py eagerly imports torchvision/skimage/numba (absent
here), so the two hot-path modules are imported through a namespace shim
(SURVEY.md §8c):
  1. a bare `hcat` package whose __path__ points at /root/reference/hcat, so
     hcat/__init__.py never runs;
  2. a stub `hcat.utils` exposing pad_image_with_reflections (only used by
     Unet_Constructor.evaluate, hcat/unet.py:217);
  3. importlib.import_module('hcat.unet'), ('hcat.loss').
Nothing from the reference is copied: the fixtures hold inputs' seeds, the
reference module's own seeded initial weights and its outputs/gradients.

Training step recorded (reference pattern tests/r_unet_test.py:24,48-56):
  zero_grad -> Unet_Constructor.forward (train mode) ->
  hcat.loss.cross_entropy(out, mask, pwl, method='pixel') -> backward ->
  torch.optim.Adam(lr=1e-3).step -> eval-mode forward with the updated model.

Usage:  python tests/golden/make_golden.py
"""
import importlib
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.path.insert(0, ROOT)

from oracle import inputs  # noqa: E402  (the splitmix64 input generator)


def import_reference():
    if not os.path.isdir(os.path.join(REF, 'hcat')):
        raise SystemExit('make_golden.py needs the reference at %s' % REF)
    for k in [k for k in sys.modules if k == 'hcat' or k.startswith('hcat.')]:
        del sys.modules[k]
    pkg = types.ModuleType('hcat')
    pkg.__path__ = [os.path.join(REF, 'hcat')]
    sys.modules['hcat'] = pkg
    utils = types.ModuleType('hcat.utils')
    utils.pad_image_with_reflections = lambda *a, **k: None
    sys.modules['hcat.utils'] = utils
    unet = importlib.import_module('hcat.unet')
    loss = importlib.import_module('hcat.loss')
    return unet, loss


KW = dict(image_dimensions=3, in_channels=4, out_channels=1,
          kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)}, upsample_kernel=(2, 2, 2),
          max_pool_kernel=(2, 2, 1), upsample_stride=(2, 2, 1))

# name -> (constructor kwargs, input shape, mask/pwl padding, store full tensors?)
NETS = {
    'unet_l2': (dict(KW, feature_sizes=[2, 4]), (2, 4, 18, 18, 3), (3, 2, 1), True),
    'unet_l3': (dict(KW, feature_sizes=[2, 4, 8]), (2, 4, 44, 44, 4), (3, 2, 1), True),
    'unet_l4': (dict(KW, feature_sizes=[4, 8, 16, 32]), (1, 4, 92, 92, 5), (0, 1, 2), True),
    'unet_g2_up8': (dict(KW, feature_sizes=[4, 8, 16], groups=2, upsample_kernel=(8, 8, 2)),
                    (1, 4, 64, 60, 6), (1, 1, 1), True),
    'unet_dil': (dict(KW, feature_sizes=[4, 8, 16], dilation={'conv1': (2, 2, 1), 'conv2': 1}),
                 (1, 4, 68, 66, 6), (2, 0, 1), True),
    'unet_l5_min': (dict(KW, feature_sizes=[8, 16, 32, 64, 128]), (2, 4, 188, 188, 6), (0, 0, 0), False),
}


def summary(t):
    """Size-independent digest of a tensor: sum, L2 norm, max|.|, 64 hashed samples."""
    t = t.detach().double().reshape(-1)
    n = t.numel()
    idx = (inputs.splitmix64(99, 64) % np.uint64(n)).astype(np.int64)
    return np.concatenate([[t.sum().item(), t.norm().item(), t.abs().max().item()],
                           t[torch.from_numpy(idx)].numpy()])


def run_net(ref_unet, ref_loss, name, kw, shape, pad, full, dtype):
    torch.manual_seed(0)
    net = ref_unet.Unet_Constructor(**kw)
    init = {k: v.detach().clone() for k, v in net.state_dict().items()}
    net = net.to(dtype).train()
    x = torch.from_numpy(inputs.make_x(shape)).to(dtype)
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    opt.zero_grad()
    out = net(x)
    B, C, X, Y, Z = out.shape
    ms = (B, C, X + pad[0], Y + pad[1], Z + pad[2])
    mask = torch.from_numpy(inputs.make_mask(ms))
    pwl = torch.from_numpy(inputs.make_pwl(ms))
    loss = ref_loss.cross_entropy(out, mask, pwl, method='pixel')
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters()}
    after_fwd = {k: v.detach().clone() for k, v in net.state_dict().items()}
    opt.step()
    stepped = {k: v.detach().clone() for k, v in net.state_dict().items()}
    net.eval()
    with torch.no_grad():
        out_eval = net(x)
    rec = {'input_shape': np.array(shape), 'mask_shape': np.array(ms),
           'out': out.detach().numpy(), 'loss': np.array(loss.item()),
           'out_eval': out_eval.numpy()}
    pnames = [n for n, _ in net.named_parameters()]
    rec['param_names'] = np.array(pnames)
    rec['state_keys'] = np.array(list(init.keys()))
    for k, v in init.items():
        key = 'init/' + k
        rec[key] = v.numpy() if full else summary(v)
    for n, g in grads.items():
        rec['grad/' + n] = g.numpy() if full else summary(g)
    for k, v in after_fwd.items():
        if 'running' in k or 'num_batches' in k:
            rec['stats/' + k] = v.numpy() if full else summary(v)
    for n in pnames:
        rec['adam/' + n] = stepped[n].numpy() if full else summary(stepped[n])
    return rec


def loss_cases(ref_loss):
    """hcat.loss.cross_entropy(method='pixel') on its own: fp16 pwl, fp32 pwl,
    pwl=None, 4D (2D) inputs, top-left crop."""
    rec = {}
    g = torch.Generator().manual_seed(5)
    cases = {
        'f16': ((2, 1, 7, 6, 5), (2, 1, 9, 8, 6), torch.float16, True),
        'f32': ((1, 2, 5, 5, 3), (1, 2, 5, 7, 4), torch.float32, True),
        'none': ((2, 1, 6, 4, 3), (2, 1, 8, 4, 3), torch.float16, False),
        '2d': ((2, 1, 9, 7), (2, 1, 11, 8), torch.float16, True),
    }
    for name, (ps, ms, pdt, has_pwl) in cases.items():
        pred = (torch.randn(ps, generator=g) * 3).requires_grad_(True)
        mask = (torch.rand(ms, generator=g) < 0.5).half()
        pwl = (torch.rand(ms, generator=g) * 11).to(pdt) if has_pwl else None
        loss = ref_loss.cross_entropy(pred, mask, pwl, method='pixel')
        loss.backward()
        rec[name + '/pred'] = pred.detach().numpy()
        rec[name + '/mask'] = mask.numpy()
        if has_pwl:
            rec[name + '/pwl'] = pwl.numpy()
        rec[name + '/loss'] = np.array(loss.item())
        rec[name + '/grad'] = pred.grad.numpy()
    return rec


def error_cases(ref_unet):
    """Exception type raised by the reference for each bad construction/input."""
    rec = {}

    def kind(fn):
        try:
            fn()
        except Exception as e:  # record the type name only
            return type(e).__name__
        return 'none'
    rec['err/2d'] = np.array(kind(lambda: ref_unet.Unet_Constructor(
        image_dimensions=2, in_channels=4, out_channels=1, feature_sizes=[8, 16])))
    rec['err/default'] = np.array(kind(lambda: ref_unet.Unet_Constructor()))
    rec['err/dims4'] = np.array(kind(lambda: ref_unet.Unet_Constructor(image_dimensions=4)))
    rec['err/one_feature'] = np.array(kind(lambda: ref_unet.Unet_Constructor(
        image_dimensions=3, feature_sizes=[8])))
    rec['err/not_doubling'] = np.array(kind(lambda: ref_unet.Unet_Constructor(
        image_dimensions=3, feature_sizes=[8, 24])))

    def too_small():
        torch.manual_seed(0)
        net = ref_unet.Unet_Constructor(**dict(KW, feature_sizes=[8, 16, 32, 64, 128]))
        net(torch.zeros(1, 4, 100, 100, 6))
    rec['err/too_small'] = np.array(kind(too_small))

    def up_exceeds_skip():
        # Z kernel 1 everywhere with upsample z-kernel 2: upsampled Z > skip Z -> torch.cat fails
        torch.manual_seed(0)
        net = ref_unet.Unet_Constructor(**dict(KW, feature_sizes=[2, 4],
                                               kernel={'conv1': (3, 3, 1), 'conv2': (3, 3, 1)}))
        net(torch.zeros(1, 4, 20, 20, 3))
    rec['err/up_exceeds_skip'] = np.array(kind(up_exceeds_skip))
    return rec


def main():
    torch.set_num_threads(8)
    ref_unet, ref_loss = import_reference()
    for name, (kw, shape, pad, full) in NETS.items():
        rec = run_net(ref_unet, ref_loss, name, kw, shape, pad, full, torch.float32)
        rec64 = run_net(ref_unet, ref_loss, name, kw, shape, pad, full, torch.float64)
        for k in ('out', 'loss', 'out_eval'):
            rec['f64/' + k] = rec64[k]
        for k, v in rec64.items():
            if k.startswith('grad/'):
                rec['f64/' + k] = v
        np.savez_compressed(os.path.join(HERE, name + '.npz'), **rec)
        print(name, 'loss', float(rec['loss']), 'out', rec['out'].shape)
    np.savez_compressed(os.path.join(HERE, 'loss_pixel.npz'), **loss_cases(ref_loss))
    np.savez_compressed(os.path.join(HERE, 'errors.npz'), **error_cases(ref_unet))
    print('wrote', sorted(f for f in os.listdir(HERE) if f.endswith('.npz')))


if __name__ == '__main__':
    main()
