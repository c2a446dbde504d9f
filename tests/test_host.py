"""CPU: the C-ABI library and the host-side mirror of the reference interface.

No kernel is launched here: only symbol exports, the native planner (pure
host code: shapes, parameter layout, workspace sizes, reference errors) and
the Python API surface (constructor, state_dict, save/load, argument checks,
no silent CPU fallback)."""
import ctypes
import os
import re

import pytest
import torch

from hcunet_amd import _lib
from hcunet_amd.unet import _Plan, spec_struct
from oracle import inputs, unet_oracle as uo

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KW = dict(image_dimensions=3, in_channels=4, out_channels=1,
          kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)}, upsample_kernel=(2, 2, 2),
          max_pool_kernel=(2, 2, 1), upsample_stride=(2, 2, 1))


def _header_functions():
    src = open(os.path.join(ROOT, 'include', 'hcunet.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(hcu_[a-z0-9_]+)\s*\(', src)))


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    names = _header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(L, n), n
    declared = {s[0] for s in _lib.SYMBOLS}
    assert set(names) == declared, set(names) ^ declared


def test_library_version_and_error_channel():
    L = _lib.lib()
    assert L.hcu_version() >= 100
    spec = _lib.UnetSpec()
    spec.levels = 1
    h = ctypes.c_void_p()
    rc = L.hcu_unet_plan_create(ctypes.byref(spec), 1, 8, 8, 8, ctypes.byref(h))
    assert rc == _lib.HCU_ERR_INVALID
    assert 'at least 2' in _lib.last_error()


@pytest.mark.parametrize('fs,shape', [([2, 4], (2, 4, 18, 18, 3)),
                                      ([4, 8, 16, 32], (1, 4, 92, 92, 5)),
                                      ([8, 16, 32, 64, 128], (2, 4, 256, 256, 16)),
                                      ([8, 16, 32, 64, 128], (2, 4, 188, 188, 6))])
def test_plan_shapes_match_oracle(fs, shape):
    from hcat.unet import Unet_Constructor
    kw = dict(KW, feature_sizes=fs)
    m = Unet_Constructor(**kw)
    p = _Plan(spec_struct(m), *[shape[i] for i in (0, 2, 3, 4)])
    spec = uo.normalize_spec(**kw)
    net = uo.OracleUnet(spec, uo.init_state(spec, 0))
    with torch.no_grad():
        if shape[2] > 200:  # full size: shape only, via meta tensors
            out_shape = _meta_out_shape(spec, shape)
        else:
            out_shape = tuple(net.forward(torch.from_numpy(inputs.make_x(shape)), False).shape)
    assert p.out_shape == out_shape
    assert p.n_params == sum(t.numel() for t in m.parameters())
    assert p.n_bn == 2 * (2 * len(fs) - 1)


def _meta_out_shape(spec, shape):
    import torch.nn.functional as F
    st = uo.init_state(spec, 0)
    x = torch.empty(shape, device='meta')
    L = len(spec['feature_sizes'])
    skips = []
    for i in range(L):
        p = 'down_steps.%d.' % i
        x = F.conv3d(x, st[p + 'conv1.weight'].to('meta'))
        x = F.conv3d(x, st[p + 'conv2.weight'].to('meta'))
        if i < L - 1:
            skips.append(x)
            x = F.max_pool3d(x, spec['max_pool_kernel'])
    for j in range(L - 1):
        p = 'up_steps.%d.' % j
        x = F.conv_transpose3d(x, st[p + 'up_conv.weight'].to('meta'), stride=spec['upsample_stride'])
        x = torch.cat((x, x), 1)
        x = F.conv3d(x, st[p + 'conv1.weight'].to('meta'))
        x = F.conv3d(x, st[p + 'conv2.weight'].to('meta'))
    return (shape[0], spec['out_channels']) + tuple(x.shape[2:])


def test_config2_output_and_workspace():
    from hcat.unet import Unet_Constructor
    m = Unet_Constructor(**dict(KW, feature_sizes=[8, 16, 32, 64, 128]))
    p = _Plan(spec_struct(m), 2, 256, 256, 16)
    assert p.out_shape == (2, 1, 68, 68, 11)
    assert p.n_params == 727009
    # saved activations of one B=2 step fit comfortably in HBM (< 2 GB)
    assert 0 < p.saved_bytes < 2 << 30
    assert 0 < p.scratch_bytes < 2 << 30


def test_no_cpu_fallback():
    from hcat.unet import Unet_Constructor
    from hcat.loss import cross_entropy
    m = Unet_Constructor(**dict(KW, feature_sizes=[2, 4]))
    with pytest.raises(RuntimeError, match='ROCm'):
        m(torch.zeros(1, 4, 18, 18, 3))
    with pytest.raises(RuntimeError, match='ROCm'):
        cross_entropy(torch.zeros(1, 1, 2, 2, 1), torch.zeros(1, 1, 2, 2, 1), None)


def test_loss_argument_errors_match_reference():
    from hcat.loss import cross_entropy
    p = torch.zeros(1, 1, 2, 2, 1)
    with pytest.raises(ValueError):
        cross_entropy(p, p, None, method='nope')
    with pytest.raises(ValueError):
        cross_entropy(p, p, None, method='random')
    with pytest.raises(ValueError):
        cross_entropy(p, p, None, method='random', num_random_pixels=1)
    with pytest.raises(IndexError):
        cross_entropy(torch.zeros(2, 2, 2), torch.zeros(2, 2, 2), None)


def test_save_load_roundtrip(tmp_path, monkeypatch):
    from hcat.unet import Unet_Constructor
    monkeypatch.chdir(tmp_path)
    (tmp_path / 'train.py').write_text('# a training script\n')
    torch.manual_seed(0)
    kw = dict(KW, feature_sizes=[2, 4, 8])
    m = Unet_Constructor(**kw)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.25)
    m.save('model.unet', hyperparameters={'lr': 1e-3})
    ck = torch.load('model.unet', weights_only=True)
    assert set(ck) == {'state_dict', 'model_specifications', 'hyperparameters', 'python_files',
                       'tree_structure'}
    assert './train.py' in ck['python_files']
    m2 = Unet_Constructor(**kw)
    hp = m2.load('model.unet', to_cuda=False)
    assert hp == {'lr': 1e-3}
    assert not m2.training
    for (k, a), (k2, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert k == k2 and torch.equal(a, b)


def test_evaluate_input_checks():
    from hcat.unet import Unet_Constructor
    m = Unet_Constructor(**dict(KW, feature_sizes=[2, 4]))
    with pytest.raises(ValueError):
        m.evaluate([1, 2, 3])
    with pytest.raises(ImportError):
        m.evaluate(torch.zeros(1, 3, 18, 18, 3))


def test_inputs_generator_is_deterministic_and_in_range():
    x = inputs.make_x((2, 4, 8, 8, 4))
    assert x.dtype.name == 'float32' and x.min() >= -1 and x.max() < 1
    assert (inputs.make_x((2, 4, 8, 8, 4)) == x).all()
    m = inputs.make_mask((1, 1, 64, 64, 4))
    assert set(m.reshape(-1).tolist()) <= {0.0, 1.0} and 0.4 < m.mean() < 0.6
    w = inputs.make_pwl((1, 1, 64, 64, 4))
    assert w.dtype.name == 'float16' and w.min() >= 0 and w.max() <= 11


def test_step_roofline_matches_survey():
    # config 2 50.17 GFLOP, 0.351 ms; config 3 1498.4 GFLOP, 0.891 ms
    import bench
    from hcunet_amd import roofline
    ms, fl, by = roofline.step_roofline(bench.CONFIGS['2']['kw'], 2, (256, 256, 16))
    assert abs(fl - 50.17e9) < 0.01e9 and abs(ms - 0.351) < 1e-3 and abs(by - 1.34e9) < 0.01e9
    ms, fl, by = roofline.step_roofline(bench.CONFIGS['3']['kw'], 4, (256, 256, 16), bf16=True)
    assert abs(fl - 1498.4e9) < 0.1e9 and abs(ms - 0.891) < 1e-3


def test_tiling_table_modes_and_file(tmp_path):
    # the persistent tiling table ships with the library and its modes switch
    from hcunet_amd import _lib
    table = os.path.join(os.path.dirname(_lib.LIB_PATH), 'tuning', 'bconv_gfx950.txt')
    rows = [ln for ln in open(table) if not ln.startswith('#')]
    assert len(rows) > 10 and all('|' in ln for ln in rows)
    old = _lib.tuning_mode()
    try:
        assert _lib.tuning_mode(_lib.TUNE_TABLE) == _lib.TUNE_TABLE
        n, timed = _lib.tuning_entries()
        assert n >= len(rows) and timed == 0
        out = tmp_path / 't.txt'
        assert _lib.tuning_save(str(out)) == n
        assert sorted(ln for ln in open(out) if not ln.startswith('#')) == sorted(rows)
        with pytest.raises(ValueError):
            _lib.tuning_mode(3)
    finally:
        _lib.tuning_mode(old)


def test_bench_rocprof_names_map_to_timed_labels():
    """bench.py reads the committed rocprofv3 summaries by the labels its
    HIP-event timing uses (tagify): element-type templates, the bconv flags
    and the 4-parameter bwgrad pipelines (equal A / G prefetch depths are
    timed as <MSW,NS,NP>, the all-taps form keeps both), and every dominant
    kernel a bench line names is found in this round's summaries."""
    import bench
    t = bench.tagify
    assert t('void hcu::bconv_kernel<float, 4, 1, 1, 4, 0>(hcu::GConvArgs)') == 'bconv_kernel<f32,4,1,1,4>'
    assert t('void hcu::bconv_kernel<unsigned short, 4, 2, 4, 12, 1>(hcu::GConvArgs)') == \
        'bconv_kernel<bf16,4,2,4,12,bnb>'
    assert t('void hcu::bwgrad_pipe_kernel<5, 4, 16, 16>(hcu::WGradArgs)') == 'bwgrad_pipe_kernel<5,4,16>'
    assert t('void hcu::bwgrad_pipe_kernel<32, 1, 12, 8>(hcu::WGradArgs)') == 'bwgrad_pipe_kernel<32,1,12,8>'
    assert t('void hcu::bn_bwd_apply_vec_kernel<float>(float*, float const*, hcu::BNCoef, long, int)') == \
        'bn_bwd_apply_vec_kernel'
    for cfg, kern in (('2', 'bconv_kernel<f32,4,1,1,4>'), ('3', 'bwgrad_pipe_kernel<5,4,16>')):
        assert bench.rocprof_avg_us(kern, cfg) is not None, (cfg, kern)
        assert bench.rocprof_avg_us(kern, cfg, 'serial_') is not None, (cfg, kern)
        assert bench.load_traffic(kern, cfg) is not None, (cfg, kern)
    assert bench.rocprof_avg_us('bconv_kernel<bf16,1,1,4,8>', 'runet') is not None
