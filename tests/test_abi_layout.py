"""CPU: the ctypes mirrors of the C-ABI structs (hcunet_amd/_lib.py,
hcunet_amd/chain.py) have the size and field offsets of include/hcunet.h as a
C compiler lays them out, and the chain planner's argument checks for the
channels-last boundaries (hcu_chain_spec in_cl / out_cl / in_part_channels)
fail the way the header documents.  No kernel is launched."""
import ctypes
import os
import shutil
import subprocess

import pytest

from hcunet_amd import _lib
from hcunet_amd import chain as ch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STRUCTS = {
    'hcu_unet_spec': (_lib.UnetSpec, ['levels', 'features', 'pool_k', 'bn_eps', 'compute_dtype']),
    'hcu_unet_tensors': (_lib.UnetTensors, ['x', 'grads', 'bn_num_batches_tracked', 'scratch', 'x_dtype']),
    'hcu_conv_desc': (_lib.ConvDesc, ['B', 'k', 'groups', 'dtype']),
    'hcu_bn_layer_info': (_lib.BNLayerInfo, ['y_offset', 'coef_offset', 'C', 'pad']),
    'hcu_chain_op': (ch.ChainOp, ['kind', 'k', 'cat_fold', 'w_off', 'beta_off']),
    'hcu_chain_spec': (ch.ChainSpec, ['n_ops', 'ops', 'bn_eps', 'compute_dtype', 'in_cl', 'out_cl',
                                      'in_part_channels']),
}


@pytest.mark.skipif(shutil.which('gcc') is None, reason='needs a C compiler')
def test_ctypes_structs_match_the_header(tmp_path):
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "hcunet.h"', 'int main(void) {']
    for name, (_, fields) in STRUCTS.items():
        lines.append('printf("%s size %%zu\\n", sizeof(%s));' % (name, name))
        for f in fields:
            lines.append('printf("%s %s %%zu\\n", offsetof(%s, %s));' % (name, f, name, f))
    lines += ['return 0;', '}']
    src = tmp_path / 'abi.c'
    src.write_text('\n'.join(lines))
    exe = tmp_path / 'abi'
    subprocess.run(['gcc', '-std=c11', '-I', os.path.join(ROOT, 'include'), str(src), '-o', str(exe)],
                   check=True, capture_output=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split('\n')
    got = {}
    for ln in out:
        parts = ln.split()
        if len(parts) == 3:
            got[(parts[0], parts[1])] = int(parts[2])
    for name, (cls, fields) in STRUCTS.items():
        assert got[(name, 'size')] == ctypes.sizeof(cls), name
        for f in fields:
            assert got[(name, f)] == getattr(cls, f).offset, (name, f)


def _spec(ops, in_channels, bf16=False, **cl):
    s = ch.ChainSpec()
    s.n_ops = len(ops)
    s.in_channels = in_channels
    for i, (kind, cout, k, bn) in enumerate(ops):
        o = s.ops[i]
        o.kind = kind
        o.out_channels = cout
        o.k = _lib.c_int3(*k)
        o.stride = _lib.c_int3(1, 1, 1)
        o.dil = _lib.c_int3(1, 1, 1)
        o.pad = _lib.c_int3(0, 0, 0)
        o.groups = 1
        o.bn_relu = bn
        o.w_off, o.b_off, o.gamma_off, o.beta_off = 0, -1, -1, -1
    s.bn_eps, s.bn_momentum = 1e-5, 0.1
    s.compute_dtype = _lib.HCU_BF16 if bf16 else _lib.HCU_F32
    s.in_cl, s.out_cl, s.in_part_channels = cl.get('in_cl', 0), cl.get('out_cl', 0), cl.get('in_part', 0)
    return s


def _create(spec, shape=(1, 20, 20, 8)):
    L = _lib.lib()
    h = ctypes.c_void_p()
    rc = L.hcu_chain_plan_create(ctypes.byref(spec), *shape, ctypes.byref(h))
    if rc == 0:
        out = (ctypes.c_int64 * 5)()
        nbn = ctypes.c_int()
        sv, sc = ctypes.c_size_t(), ctypes.c_size_t()
        assert L.hcu_chain_plan_query(h, out, ctypes.byref(nbn), ctypes.byref(sv), ctypes.byref(sc)) == 0
        L.hcu_unet_plan_destroy(h)
        return rc, tuple(out)
    return rc, None


def test_chain_channels_last_boundary_checks():
    conv = (ch.CONV, 10, (1, 1, 1), 0)
    # the channel-wise cat of two padded channels-last tensors feeding a 1x1 conv
    rc, out = _create(_spec([conv], 20, in_cl=1, out_cl=1, in_part=10))
    assert rc == 0 and out == (1, 10, 20, 20, 8)
    rc, _ = _create(_spec([conv], 20, bf16=True, in_cl=1, out_cl=1, in_part=10))
    assert rc == 0
    # parts need a channels-last input, a whole number of parts and a first Conv3d
    assert _create(_spec([conv], 20, in_part=10))[0] == _lib.HCU_ERR_INVALID
    assert _create(_spec([conv], 25, in_cl=1, in_part=10))[0] == _lib.HCU_ERR_INVALID
    # a channels-last output needs a last Conv3d without BatchNorm
    assert _create(_spec([(ch.CONV, 10, (1, 1, 1), 1)], 20, out_cl=1))[0] == _lib.HCU_ERR_UNSUPPORTED
