"""Per-phase cycles of the all-taps bf16 weight gradient (wave 0 of every
block, summed over one RDCNet step's launches) from a measurement build:
  OUT=hcunet_amd/libhcunet_ph.so BDIR=build_ph ./build.sh -DHCU_BW_PHASES
  HCU_LIB_PATH=hcunet_amd/libhcunet_ph.so python tools/bw_phases.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import hcat.loss as hl  # noqa: E402
from hcat.r_unet import RDCNet  # noqa: E402
from hcunet_amd import _lib  # noqa: E402

L = _lib.lib()
fn = L._name if False else None
h = ctypes.CDLL(_lib.LIB_PATH)
rd = h.hcu_debug_bw_phases
rd.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
torch.manual_seed(0)
net = RDCNet(4, 5).cuda().train()
tile = (1, 4, 512, 512, 24)
x = torch.randn(tile, device='cuda')
vec = torch.randn((1, 3) + tile[2:], device='cuda')
mask = (torch.rand((1, 1) + tile[2:], device='cuda') < 0.5).half()
pwl = torch.rand((1, 1) + tile[2:], device='cuda').half()
out = (ctypes.c_ulonglong * 4)()
for it in range(3):
    with torch.autocast('cuda', dtype=torch.bfloat16):
        o = net(x)
        loss = hl.cross_entropy(o[:, 0:1], mask, pwl, method='pixel') + hl.MSELoss(o[:, 2:], vec)
    loss.backward()
    torch.cuda.synchronize()
    assert rd(out) == 0
    t = max(out[3], 1)
    print('step %d: tiles %d | per tile: commit %.0f, barriers+load issue %.0f, MFMA loop %.0f cycles'
          % (it, out[3], out[0] / t, out[1] / t, out[2] / t))
