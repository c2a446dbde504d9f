"""The backward's launch modes give bitwise-identical results.

HCU_SIDE (weight-gradient branch on its own stream) and HCU_GRAPHS (hipGraph
capture/replay) are read once per process, so each mode runs in a child
process started before any GPU call of its own: one with both off (serial,
kernel-by-kernel on one stream), one with graphs + split streams and one
with the default (split streams, direct launches).  A missing event wait on the gradient-slot ring would make the
split run read a slot the chain has already rewritten, which shows up as a
bitwise difference in the gradients."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, torch
sys.path.insert(0, %(root)r)
from hcat.unet import Unet_Constructor
from hcat.loss import cross_entropy
from oracle import inputs
kw = %(kw)s
torch.manual_seed(0)
m = Unet_Constructor(**kw).cuda().train()
x = torch.from_numpy(inputs.make_x(%(shape)r)).cuda()
x = x.to({'f16': torch.float16, 'bf16': torch.bfloat16}.get(os.environ.get('HCU_TEST_XDT'), torch.float32))
res = []
for it in range(3):          # 3 steps: the graphed mode replays its capture
    for p in m.parameters():
        p.grad = None
    with torch.autocast('cuda', dtype=torch.bfloat16, enabled=os.environ.get('HCU_TEST_BF16') == '1'):
        out = m(x)
    ms = (x.shape[0], 1) + tuple(out.shape[2:])
    loss = cross_entropy(out, torch.from_numpy(inputs.make_mask(ms)).cuda(),
                         torch.from_numpy(inputs.make_pwl(ms)).cuda(), method='pixel')
    loss.backward()
    res.append([out.detach().cpu()] + [p.grad.detach().cpu() for p in m.parameters()])
torch.cuda.synchronize()
torch.save(res, %(out)r)
'''


KW = ("dict(image_dimensions=3, in_channels=4, out_channels=1, feature_sizes=[8, 16, 32, 64, 128], "
      "kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)}, upsample_kernel=(2, 2, 2), "
      "max_pool_kernel=(2, 2, 1), upsample_stride=(2, 2, 1))")
SHAPE = (2, 4, 188, 188, 6)
# the inference network of hcat/main.py:46-54: grouped convolutions (groups=2)
# and an (8, 8, 2) ConvTranspose3d kernel
KW_GROUPS = ("dict(image_dimensions=3, in_channels=4, out_channels=1, feature_sizes=[16, 32, 64], "
             "kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)}, upsample_kernel=(8, 8, 2), "
             "max_pool_kernel=(2, 2, 1), upsample_stride=(2, 2, 1), dilation=1, groups=2)")
SHAPE_GROUPS = (1, 4, 64, 60, 6)   # test_gpu_unet.py's g2_up8 geometry


def _run(tmp_path, tag, env_extra, kw=KW, shape=SHAPE):
    out = str(tmp_path / ('%s.pt' % tag))
    env = dict(os.environ)
    env.update(env_extra)
    env['HCU_BCONV_TUNE'] = '0'   # measured tile choices may differ between processes
    r = subprocess.run([sys.executable, '-c', CHILD % dict(root=ROOT, out=out, kw=kw, shape=shape)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return torch.load(out, weights_only=True)


def test_split_graphed_equals_serial(tmp_path):
    serial = _run(tmp_path, 'serial', {'HCU_SIDE': '0', 'HCU_GRAPHS': '0'})
    split = _run(tmp_path, 'split', {'HCU_SIDE': '1', 'HCU_GRAPHS': '1'})
    direct = _run(tmp_path, 'direct', {'HCU_SIDE': '1', 'HCU_GRAPHS': '0'})   # the default
    for it in range(3):
        for a, b, d in zip(serial[it], split[it], direct[it]):
            assert torch.equal(a, b)
            assert torch.equal(a, d)


@pytest.mark.parametrize('bf16', ['0', '1'])
def test_split_forward_equals_serial(tmp_path, bf16):
    """The split training forward (the deeper levels' weight images laid out
    on the branch stream while level 0 runs, the chain waiting before level 1;
    the default from 4 M parameters) forced onto this small network
    (HCU_SPLIT_FWD_PARAMS=0) against the serial run (HCU_SIDE=0): outputs and
    gradients bitwise equal over 3 steps, fp32 and bf16."""
    kw = KW if bf16 == '0' else KW.replace('[8, 16, 32, 64, 128]', '[16, 32, 64, 128]')
    serial = _run(tmp_path, 'ser' + bf16, {'HCU_SIDE': '0', 'HCU_TEST_BF16': bf16}, kw=kw)
    split = _run(tmp_path, 'spl' + bf16, {'HCU_SPLIT_FWD_PARAMS': '0', 'HCU_TEST_BF16': bf16}, kw=kw)
    for it in range(3):
        for k, (a, b) in enumerate(zip(serial[it], split[it])):
            assert torch.equal(a, b), (it, k)


def test_bf16_steps_are_deterministic(tmp_path):
    """Two processes running the same bf16 autocast training steps (split
    streams, graphed forward: the default) give bitwise-identical outputs and
    gradients on every step."""
    kw = KW.replace('[8, 16, 32, 64, 128]', '[16, 32, 64, 128]')
    a = _run(tmp_path, 'bfa', {'HCU_TEST_BF16': '1'}, kw=kw)
    b = _run(tmp_path, 'bfb', {'HCU_TEST_BF16': '1'}, kw=kw)
    bad = [(it, k) for it in range(3) for k, (x, y) in enumerate(zip(a[it], b[it])) if not torch.equal(x, y)]
    assert not bad, bad[:8]


@pytest.mark.parametrize('bf16', ['0', '1'])
def test_halo_layout_is_bitwise_neutral(tmp_path, bf16):
    """bconv's planner-chosen halo image layout in LDS (axis order and row
    padding, bconv.hip bconv_halo_layout) only moves where each halo element
    sits: outputs and gradients over 3 training steps are bitwise equal to the
    dense z-fastest image (HCU_HALO_LAYOUT=0).  fp32 runs the search with
    HCU_HALO_LAYOUT=2 (off by default there)."""
    kw = KW if bf16 == '0' else KW.replace('[8, 16, 32, 64, 128]', '[16, 32, 64, 128]')
    dense = _run(tmp_path, 'hl0' + bf16, {'HCU_HALO_LAYOUT': '0', 'HCU_TEST_BF16': bf16}, kw=kw)
    laid = _run(tmp_path, 'hl2' + bf16, {'HCU_HALO_LAYOUT': '2', 'HCU_TEST_BF16': bf16}, kw=kw)
    bad = [(it, k) for it in range(3) for k, (x, y) in enumerate(zip(dense[it], laid[it])) if not torch.equal(x, y)]
    assert not bad, bad[:8]


def test_fresh_input_every_step_matches():
    """A new input tensor each step (data-loader pattern: the input layout change
    runs ahead of the captured graph) gives the same outputs and gradients as
    re-using one tensor."""
    from hcat.loss import cross_entropy
    from hcat.unet import Unet_Constructor
    from oracle import inputs
    kw = dict(image_dimensions=3, in_channels=4, out_channels=1, feature_sizes=[4, 8, 16],
              kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)}, upsample_kernel=(2, 2, 2),
              max_pool_kernel=(2, 2, 1), upsample_stride=(2, 2, 1))
    xs = [torch.from_numpy(inputs.make_x((2, 4, 44, 44, 6), seed=s)).cuda() for s in (1, 2, 3)]
    res = []
    for fresh in (False, True):
        torch.manual_seed(0)
        m = Unet_Constructor(**kw).cuda().train()
        outs = []
        for it in range(6):
            for p in m.parameters():
                p.grad = None
            x = xs[it % 3].clone() if fresh else xs[it % 3]
            out = m(x)
            ms = (2, 1) + tuple(out.shape[2:])
            loss = cross_entropy(out, torch.from_numpy(inputs.make_mask(ms)).cuda(),
                                 torch.from_numpy(inputs.make_pwl(ms)).cuda(), method='pixel')
            loss.backward()
            outs.append([out.detach().cpu()] + [p.grad.detach().cpu() for p in m.parameters()])
        res.append(outs)
    for a_it, b_it in zip(*res):
        for a, b in zip(a_it, b_it):
            assert torch.equal(a, b)


def test_tiled_weight_gradient_finalize(tmp_path):
    """HCU_WGF_TILED=2 (every Conv3d / ConvTranspose3d weight-gradient finalize
    through the coalescing LDS-transposed tile) agrees with HCU_WGF_TILED=0
    (element-parallel slab sums, scattered stores) to fp64-summation rounding:
    both sum the same fp32 slabs in fp64, only the order over the slabs may
    differ (S > 1 splits them), so every gradient matches to 2 fp32 ulps of its
    largest element.  Outputs are bitwise equal (step 1) and each mode is
    deterministic."""
    off = _run(tmp_path, 'wgf0', {'HCU_WGF_TILED': '0'})
    on = _run(tmp_path, 'wgf2', {'HCU_WGF_TILED': '2'})
    on2 = _run(tmp_path, 'wgf2b', {'HCU_WGF_TILED': '2'})
    # grouped convolutions and a ConvTranspose3d with 128 taps
    goff = _run(tmp_path, 'gwgf0', {'HCU_WGF_TILED': '0'}, KW_GROUPS, SHAPE_GROUPS)
    gon = _run(tmp_path, 'gwgf2', {'HCU_WGF_TILED': '2'}, KW_GROUPS, SHAPE_GROUPS)
    for r0, r2, r2b in ((off, on, on2), (goff, gon, gon)):
        assert torch.equal(r0[0][0], r2[0][0])
        for a, b, c in zip(r0[0], r2[0], r2b[0]):
            assert torch.equal(b, c)
            tol = 2.5e-7 * max(a.abs().max().item(), 1e-30)
            assert (a - b).abs().max().item() <= tol


def test_output_split_weight_gradient_matches_wgrad2(tmp_path):
    """wgrad3 (the deep fp32 layers' weight gradient with the waves splitting
    the output rows, wgrad3.hip) against wgrad2 (HCU_WGRAD3=0) on the same
    steps: outputs bitwise (the forward does not change), every gradient to
    fp32 reassociation of the voxel sums (1e-5 of each tensor's largest
    element, plus 1e-6 absolute for the BatchNorm-cancelled conv biases)."""
    a = _run(tmp_path, 'w2', {'HCU_WGRAD3': '0'})
    b = _run(tmp_path, 'w3', {})
    for it in range(3):
        assert torch.equal(a[it][0], b[it][0])
        for k, (x, y) in enumerate(zip(a[it], b[it])):
            tol = 1e-5 * x.abs().max().item() + 1e-6
            assert (x - y).abs().max().item() <= tol, (it, k, (x - y).abs().max().item(), tol)




# Kernel-family switches: each selects another kernel family (or grid size,
# or finalize schedule) for the same layers.  They exist for A/B runs and as
# fallbacks; here every one is held to the default's results.
FALLBACKS_F32 = [{'HCU_NO_CONV8': '1'}, {'HCU_NO_CONV2': '1'}, {'HCU_NO_BCONV_F32': '1'},
                 {'HCU_NO_WGRAD8': '1'}, {'HCU_NO_WGRAD2': '1'}, {'HCU_NO_BNFUSE': '1'},
                 {'HCU_WGF_DEFER': '0'}, {'HCU_SIDE_CUS': '128'}]
FALLBACKS_BF16 = [{'HCU_BW_CUS': '128'}, {'HCU_NO_BNFUSE': '1'},
                  {'HCU_WGF_DEFER': '0'}]


@pytest.mark.parametrize('bf16', ['0', '1'])
def test_kernel_family_switches_match_default(tmp_path, bf16):
    """Every kernel-family / grid / schedule switch gives the default's results
    to the reassociation of the same sums: the forward output within the
    north_star's 1e-4 (fp32; bf16 2e-2 of its largest element) and every
    gradient within a relative L2 distance of 2e-3 (fp32; bf16 3e-2; the
    BatchNorm-cancelled conv biases, rounding noise about 0, excepted): the
    switches reorder the convolution K sums themselves (other kernels), which
    five levels of BatchNorm backward amplify well past the opt-in fusions'
    coefficient-only reassociation bar (the message lists the worst relative
    distance per switch)."""
    import re
    from hcat.unet import Unet_Constructor
    kw = KW if bf16 == '0' else KW.replace('[8, 16, 32, 64, 128]', '[16, 32, 64, 128]')
    names = [n for n, _ in Unet_Constructor(**eval(kw)).named_parameters()]
    # biases ahead of a BatchNorm (the ConvTranspose3d one through the valid conv1,
    # a constant per channel): their gradient is 0 up to
    # rounding noise (the BatchNorm subtracts the batch mean), not compared
    cancelled = {k for k, n in enumerate(names) if re.fullmatch(r'(down|up)_steps\.\d+\.(conv[12]|up_conv)\.bias', n)}
    ref = _run(tmp_path, 'fbdef' + bf16, {'HCU_TEST_BF16': bf16}, kw=kw)
    out_tol, rel = (1e-4, 2e-3) if bf16 == '0' else (2e-2, 3e-2)
    bad, worst = [], {}
    for i, sw in enumerate(FALLBACKS_F32 if bf16 == '0' else FALLBACKS_BF16):
        got = _run(tmp_path, 'fb%d_%s' % (i, bf16), dict(sw, HCU_TEST_BF16=bf16), kw=kw)
        key = ','.join('%s=%s' % kv for kv in sw.items())
        for it in range(3):
            a, b = ref[it][0], got[it][0]
            d = (a - b).abs().max().item()
            tol = out_tol * (1.0 if bf16 == '0' else a.abs().max().item())
            if not d <= tol:
                bad.append((key, it, 'out', d, tol))
            for k, (a, b) in enumerate(zip(ref[it][1:], got[it][1:])):
                na = a.double().norm().item()
                r = (a - b).double().norm().item() / max(na, 1e-30)
                if k in cancelled:
                    continue
                if not r <= rel:
                    bad.append((key, it, names[k], r, rel))
                worst[key] = max(worst.get(key, 0.0), r)
    assert not bad, (bad[:8], {k: '%.2e' % v for k, v in worst.items()})


@pytest.mark.parametrize('bf16,xdt', [('0', 'f32'), ('1', 'f32'), ('1', 'f16'), ('1', 'bf16')])
def test_ncxyz_first_layer_matches_layout_pass(tmp_path, bf16, xdt):
    """The first convolution staging the caller's NCXYZ volume itself (fp32,
    fp16 or bf16; conv8 / bconv NCXYZ instances, weights in their PyTorch
    layout, the channels-last copy for the weight gradient written by the
    tiles that own each voxel) against the separate channels-last pass
    (HCU_NCX=0): outputs and every gradient bitwise equal over 3 steps (the
    same converted values reach the same MFMAs), the graphed forward
    included.  (bf16 plans take the layout pass by default: HCU_NCX=1 forces
    the NCXYZ staging there.)"""
    kw = KW if bf16 == '0' else KW.replace('[8, 16, 32, 64, 128]', '[16, 32, 64, 128]')
    env = {'HCU_TEST_BF16': bf16, 'HCU_TEST_XDT': xdt}
    a = _run(tmp_path, 'lay' + bf16 + xdt, dict(env, HCU_NCX='0'), kw=kw)
    b = _run(tmp_path, 'ncx' + bf16 + xdt, dict(env, HCU_NCX='1'), kw=kw)
    bad = [(it, k, (x - y).abs().max().item())
           for it in range(3) for k, (x, y) in enumerate(zip(a[it], b[it])) if not torch.equal(x, y)]
    assert not bad, bad[:8]
