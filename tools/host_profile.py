"""cProfile of the host side of the config-2 training step (bench.py's step
loop): where the enqueue time goes.   python tools/host_profile.py [--config 2]"""
import argparse
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import hcunet_amd  # noqa: E402
from hcat.loss import cross_entropy  # noqa: E402
from hcat.unet import Unet_Constructor  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--config', default='2')
ap.add_argument('--steps', type=int, default=30)
args = ap.parse_args()
cfg = bench.CONFIGS[args.config]
dev = torch.device('cuda', 0)
torch.manual_seed(0)
m = Unet_Constructor(**cfg['kw']).to(dev).train()
hcunet_amd.dist.broadcast_parameters(m)
opt = hcunet_amd.optim.Adam(m.parameters(), lr=1e-3)
x, mask, pwl = bench.synth_inputs(cfg['batch'], 1000, dev)
bf16 = cfg['dtype'] == 'bf16'


def step():
    opt.zero_grad()
    with torch.autocast('cuda', dtype=torch.bfloat16, enabled=bf16):
        out = m(x)
        loss = cross_entropy(out, mask, pwl, method='pixel')
    loss.backward()
    hcunet_amd.dist.allreduce_gradients(m)
    opt.step()


for _ in range(5):
    step()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(args.steps):
    step()
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats('tottime').print_stats(25)
