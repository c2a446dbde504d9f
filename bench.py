#!/usr/bin/env python3
"""Training throughput of the 5-level 3D U-Net hot path (BASELINE.json metric).

One step = optimizer.zero_grad() -> Unet_Constructor.forward ->
hcat.loss.cross_entropy(method='pixel') -> backward -> (all-reduce of the flat
gradient buffer over RCCL when N > 1) -> Adam.step, on synthetic
[B, 4, 256, 256, 16] volumes resident in HBM (config 2: fp32,
feature_sizes [8..128], B = 2 per GPU).

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Prints one JSON line (rank 0) with the whole-job voxels/s, the roofline of
the dominant kernel (HIP-event timing of every launch during a second pass of
K steps) and the CPU baseline (the oracle restatement of the reference timed
on this host's cores).
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from hcat.loss import cross_entropy  # noqa: E402
from hcat.unet import Unet_Constructor  # noqa: E402
import hcunet_amd  # noqa: E402
from hcunet_amd import _lib  # noqa: E402
import hcunet_amd.chain  # noqa: E402
from hcunet_amd import roofline as roofline_mod  # noqa: E402

PROFILE_TAG = 'r06'   # the round whose committed profiles/ summaries bench.py cites

METRIC = "training voxels/sec (fwd+bwd+step), 5-level 3D U-Net, 256×256×16×4 tiles"
PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix, dense
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA, dense (no sparsity)
PEAK_HBM_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E spec
TILE = (256, 256, 16)

CONFIGS = {
    '2': dict(kw=dict(image_dimensions=3, in_channels=4, out_channels=1,
                      feature_sizes=[8, 16, 32, 64, 128],
                      kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)},
                      upsample_kernel=(2, 2, 2), max_pool_kernel=(2, 2, 1),
                      upsample_stride=(2, 2, 1)),
              batch=2, dtype='fp32', roof_ms=0.351,
              desc='config 2: 3D U-Net feature_sizes=[8,16,32,64,128] fp32'),
    # BASELINE config 3: [32..512], B=4, bf16 (torch.autocast bf16 -> the bf16
    # MFMA path: bf16 activations/gradients/operands, fp32 accumulation, BN
    # statistics, master weights and Adam state).
    '3': dict(kw=dict(image_dimensions=3, in_channels=4, out_channels=1,
                      feature_sizes=[32, 64, 128, 256, 512],
                      kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)},
                      upsample_kernel=(2, 2, 2), max_pool_kernel=(2, 2, 1),
                      upsample_stride=(2, 2, 1)),
              batch=4, dtype='bf16', roof_ms=0.891,
              desc='config 3: 3D U-Net feature_sizes=[32,64,128,256,512] bf16 (autocast)'),
    # BASELINE config 3's shapes ([32..512], B=4) computed in fp32: a
    # capacity/shape check of the fp32 path at those sizes, not config 3
    # itself (config 3 is the bf16 line above).
    '3f32': dict(kw=dict(image_dimensions=3, in_channels=4, out_channels=1,
                         feature_sizes=[32, 64, 128, 256, 512],
                         kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)},
                         upsample_kernel=(2, 2, 2), max_pool_kernel=(2, 2, 1),
                         upsample_stride=(2, 2, 1)),
                 batch=4, dtype='fp32', roof_ms=None,
                 desc='3D U-Net feature_sizes=[32,64,128,256,512] fp32 (config-3 shapes)'),
}


def synth_inputs(B, seed, device):
    """Synthetic stand-ins for to_float -> normalize -> to_tensor volumes
    (hcat/transforms.py:105-136): x in [-1, 1), mask Bernoulli(0.5) fp16,
    pwl U[0, 11) fp16 (w0 = 11, hcat/train/train_utils.py:67)."""
    g = torch.Generator().manual_seed(seed)
    x = (torch.randint(0, 65536, (B, 4) + TILE, generator=g).float() / 65536.0 - 0.5) / 0.5
    mask = (torch.rand((B, 1) + TILE, generator=g) < 0.5).half()
    pwl = (torch.rand((B, 1) + TILE, generator=g) * 11.0).half()
    return x.to(device), mask.to(device), pwl.to(device)


def cpu_baseline(cfg, x, mask, pwl, budget_s=15.0):
    """Oracle restatement of the reference step on host cores (bounded sample)."""
    from oracle import unet_oracle as uo
    threads = max(1, min(16, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    spec = uo.normalize_spec(**cfg['kw'])
    state = uo.init_state(spec, 0)
    x, mask, pwl = x.cpu(), mask.cpu(), pwl.cpu()
    times = []
    t_start = time.perf_counter()
    uo.train_step(spec, state, x, mask, pwl)  # warm-up
    while len(times) < 3 or (time.perf_counter() - t_start < budget_s and len(times) < 20):
        t0 = time.perf_counter()
        r = uo.train_step(spec, state, x, mask, pwl)
        times.append(time.perf_counter() - t0)
        state = r['state_after']
    med = statistics.median(times)
    vox = x.shape[0] * TILE[0] * TILE[1] * TILE[2]
    return {"value": vox / med, "unit": "voxels/s", "cores": threads, "kind": "port",
            "sample": "%d full train steps (B=%d, fwd+loss+bwd+Adam) of the oracle "
                      "restatement of the reference (torch CPU fp32 -- the reference's own "
                      "arithmetic; it has no bf16 path -- %d threads), median %.3f s/step"
                      % (len(times), x.shape[0], threads, med)}


def tagify(rocprof_name):
    """rocprofv3 kernel symbol -> the name bench.py's HIP-event timing uses
    ("void hcu::bconv_kernel<float, 4, 1, 1, 4, false>(hcu::GConvArgs)" ->
    "bconv_kernel<f32,4,1,1,4>"; element-type-only templates lose the <...>)."""
    import re
    n = re.sub(r'^void\s+', '', rocprof_name.strip())
    n = re.sub(r'\(.*\)$', '', n).replace('hcu::', '').replace(' ', '')
    if '<' in n:
        args = n.split('<', 1)[1].rstrip('>').split(',')
        if all(x in ('float', '_Float16', 'bf16_t', 'unsignedshort', 'double', 'unsignedchar') for x in args):
            return n.split('<', 1)[0]   # element-type-only templates: timed under the base name
    n = n.replace('<float,', '<f32,').replace('<unsignedshort,', '<bf16,')
    n = n.replace(',false>', '>').replace(',true>', ',bnb>')
    if n.startswith('bconv_kernel<') and n.count(',') == 5:
        # the fused-BatchNorm-backward flag is an int template argument there
        n = re.sub(r',0>$', '>', re.sub(r',1>$', ',bnb>', n))
    m = re.match(r'^bwgrad_pipe_kernel<(\d+),(\d+),(\d+),(\d+)>$', n)
    if m and m.group(1) != '32' and m.group(3) == m.group(4):
        # equal A / G prefetch depths are timed as <MSW,NS,NP> (bwgrad.hip BWP)
        n = 'bwgrad_pipe_kernel<%s,%s,%s>' % m.group(1, 2, 3)
    return n


def load_traffic(kernel, config='2'):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/<PROFILE_TAG>_traffic_config<config>.json, written by
    tools/pmc_traffic.py), or None."""
    tab = None
    for fn in (('%s_traffic_runet.json' % PROFILE_TAG) if config == 'runet'
               else ('%s_traffic_config%s.json' % (PROFILE_TAG, config)),):
        if not fn:
            continue
        try:
            with open(os.path.join(ROOT, 'profiles', fn)) as f:
                tab = json.load(f)
            break
        except (OSError, ValueError):
            continue
    if tab is None:
        return None
    tot, n = 0.0, 0
    for k, v in tab.items():
        if isinstance(v, dict) and tagify(k) == kernel:
            tot += v['hbm_bytes_per_launch'] * v['launches']
            n += v['launches']
    return tot / n if n else None


def layer_of(key):
    """'kernel@d0.c1.fwd' -> ('d0.c1', 'fwd'); pool -> ('d0.pool', 'fwd');
    untagged / bookkeeping launches -> their own groups."""
    kern, _, tag = key.partition('@')
    if kern.startswith('wgrad_finalize'):
        return 'wgrad.finalize', 'bwd'
    if not tag:
        base = kern.split('<')[0].replace('_kernel', '')
        return {'loss_pixel': 'loss', 'loss_finalize': 'loss', 'scale': 'loss',
                'adam': 'adam'}.get(base, base), '-'
    parts = tag.split('.')
    if len(parts) >= 3:
        layer, phase = '.'.join(parts[:2]), '.'.join(parts[2:])
        if phase == 'pool':
            return parts[0] + '.pool', 'fwd'
        return layer, phase
    return parts[0], '.'.join(parts[1:]) or '-'


def layer_table(detail, cfg, B, steps):
    """Per-layer roofline fractions: each layer's algorithmic FLOPs and
    compulsory bytes (hcunet_amd/roofline.py), its roofline time
    max(bytes / HBM peak, FLOPs / MFMA peak) and the kernel time measured for
    it (HIP events around every launch tagged with the layer, serialized
    pass), per step."""
    bf16 = cfg['dtype'] == 'bf16'
    ref = {r['layer']: r for r in roofline_mod.layers(cfg['kw'], B, TILE, bf16)}
    rows = {}
    for k, v in detail.items():
        layer, phase = layer_of(k)
        r = rows.setdefault(layer, dict(layer=layer, us=0.0, launches=0.0, kernels={}))
        us = v['ms'] * 1e3 / steps
        r['us'] += us
        r['launches'] += v['count'] / steps
        kk = '%s:%s' % (phase, k.partition('@')[0])
        r['kernels'][kk] = round(r['kernels'].get(kk, 0.0) + us, 2)
    out = []
    for layer, r in rows.items():
        a = ref.get(layer)
        row = dict(layer=layer, measured_us=round(r['us'], 2), launches=r['launches'],
                   kernels=r['kernels'])
        if a:
            row.update(gflop=a['flops'] / 1e9, compulsory_mb=a['bytes'] / 1e6,
                       roof_us=round(a['roof_us'], 2), frac=a['roof_us'] / r['us'] if r['us'] else None,
                       bound='mfma' if a['flops'] / (roofline_mod.PEAK_BF16 if bf16 else roofline_mod.PEAK_FP32)
                       > a['bytes'] / roofline_mod.PEAK_HBM else 'hbm')
        out.append(row)
    order = [r['layer'] for r in roofline_mod.layers(cfg['kw'], B, TILE, bf16)]
    out.sort(key=lambda r: (order.index(r['layer']) if r['layer'] in order else len(order), r['layer']))
    return out


def rocprof_avg_us(kernel, config, kind=''):
    """Average duration (us) of `kernel` in the committed rocprofv3
    --kernel-trace --stats summary of this config's bench step
    (profiles/<PROFILE_TAG>_kernel_stats_<kind>config<config>.csv), or None.
    kind '' is the production step (weight-gradient branch concurrent with the
    chain); 'serial_' the same bench with HCU_SIDE=0, one kernel at a time --
    the conditions of the HIP-event timing pass."""
    import csv
    name = ('%s_kernel_stats_%s.csv' % (PROFILE_TAG, config) if config == 'runet'
            else '%s_kernel_stats_%sconfig%s.csv' % (PROFILE_TAG, kind, config))
    path = os.path.join(ROOT, 'profiles', name)
    try:
        with open(path, newline='') as f:
            rows = list(csv.DictReader(f))
    except OSError:
        return None
    tot, calls = 0.0, 0
    for r in rows:
        if tagify(r['Name']) == kernel:
            tot += float(r['TotalDurationNs'])
            calls += int(r['Calls'])
    return tot / calls / 1e3 if calls else None


# The network of the reference's inference pipeline (hcat/main.py:46-54) and
# the tiled driver it runs (hcat/segment.py:21-136), SURVEY §8f-1.
INFER_KW = dict(image_dimensions=3, in_channels=4, out_channels=1, feature_sizes=[16, 32, 64, 128],
                kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)}, upsample_kernel=(8, 8, 2),
                max_pool_kernel=(2, 2, 1), upsample_stride=(2, 2, 1), dilation=1, groups=2)
INFER_VOLUME = (1, 4, 1024, 1024, 40)


def infer_main(args):
    """Tiled inference throughput: hcat.segment.predict_segmentation_mask over a
    synthetic fp16 [1, 4, 1024, 1024, 40] volume (to_tensor output dtype) with the
    main.py network in eval mode, random init; tile size from the device memory
    (288 GB -> [350, 350, 15] + PAD (128, 128, 10)).  One step = the whole volume."""
    from hcunet_amd import segment as seg
    device = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = Unet_Constructor(**INFER_KW).to(device).eval()
    g = torch.Generator().manual_seed(7)
    vol = ((torch.rand(INFER_VOLUME, generator=g) - 0.5) * 2).half()
    vol_dev = vol.to(device)
    ev = seg.eval_image_size(torch.cuda.get_device_properties(device).total_memory)
    n_tiles = 1
    for d in range(3):
        n = INFER_VOLUME[2 + d]
        e = min(ev[d], n) if d == 2 else ev[d]
        p = min(seg.PAD_SIZE[d], n)
        n_tiles *= len(seg.calculate_indexes(seg.PAD_SIZE[d], e, n, n + 2 * p))
    for _ in range(args.warmup):
        seg.predict_segmentation_mask(model, vol_dev, device, use_probability_map=True)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        mask = seg.predict_segmentation_mask(model, vol_dev, device, use_probability_map=True)
    torch.cuda.synchronize(device)
    el = (time.perf_counter() - t0) / args.steps
    vox = INFER_VOLUME[2] * INFER_VOLUME[3] * INFER_VOLUME[4]
    cpu = None
    if not args.no_cpu_baseline:
        # one tile of the oracle restatement (CPU, B=1, eval) on the host cores
        from oracle import unet_oracle as uo
        threads = max(1, min(16, os.cpu_count() or 1))
        torch.set_num_threads(threads)
        spec = uo.normalize_spec(**INFER_KW)
        net = uo.OracleUnet(spec, {k: v.detach().cpu() for k, v in model.state_dict().items()})
        tile = vol[:, :, :ev[0] + 2 * seg.PAD_SIZE[0], :ev[1] + 2 * seg.PAD_SIZE[1],
                   :ev[2] + 2 * seg.PAD_SIZE[2] - 1].float()
        with torch.no_grad():
            net.forward(tile, training=False)
            t1 = time.perf_counter()
            net.forward(tile, training=False)
            tt = time.perf_counter() - t1
        cpu = {"value": 1.0 / tt, "unit": "tiles/s", "cores": threads, "kind": "port",
               "sample": "1 eval forward of one %s tile (oracle restatement, torch CPU fp32, "
                         "%d threads): %.2f s/tile" % ('x'.join(map(str, tile.shape[2:])), threads, tt)}
    line = {"metric": "tiled inference voxels/sec (predict_segmentation_mask, hcat/main.py network)",
            "value": vox / el, "unit": "voxels/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": "tiled eval inference of a %s fp16 volume, tiles %s + pad %s, "
                                   "%d tiles per volume, main.py network [16..128] groups=2 up (8,8,2)"
                                   % ('x'.join(map(str, INFER_VOLUME)), ev, list(seg.PAD_SIZE), n_tiles),
                       "tiles_per_s": n_tiles / el, "mask_mean": float(mask.mean())},
            "cpu_baseline": cpu}
    print(json.dumps(line), flush=True)


RUNET_TILE = (512, 512, 24)


def runet_main(args):
    """BASELINE config 5 on one GPU: hcat.r_unet.RDCNet(4, 5) (the model the
    reference trains, tests/r_unet_test.py:19-56) on 512x512x24 tiles, B=1,
    bf16 autocast, loss = cross_entropy(out[:, :1], pixel) + MSELoss(out[:, 2:])
    then Adam; the input tiles come from pinned host memory, copied to the GPU
    on a side stream while the previous step computes (a ring of two device
    buffers).  One step = one tile per GPU.

    Multi-GPU (BASELINE config 5 names 8 GPUs; launched like the U-Net, one
    process per GPU under torch.distributed.run): the tiles shard by rank
    (rank r draws its own tile stream), the parameters are broadcast once
    from rank 0 and the gradients averaged by hcunet_amd.dist.allreduce_gradients
    (one collective over the flat gradient buffer the layer chains fill)
    before the optimizer step (/root/reference/tests/r_unet_test.py:37-56
    trains one model on such tiles); value = tiles of all ranks / max-over-
    ranks time (weak scaling)."""
    import hcat.loss as hl
    from hcat.r_unet import RDCNet
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    device = torch.device('cuda', local)
    torch.manual_seed(0)
    model = RDCNet(4, 5).to(device).train()
    hcunet_amd.dist.broadcast_parameters(model)
    opt = hcunet_amd.optim.Adam(model.parameters(), lr=1e-3)
    g = torch.Generator().manual_seed(11 + 7919 * rank)
    n_host = 4
    host = [((torch.randint(0, 65536, (1, 4) + RUNET_TILE, generator=g).float() / 65536 - 0.5) / 0.5)
            .pin_memory() for _ in range(n_host)]
    mask = (torch.rand((1, 1) + RUNET_TILE, generator=g) < 0.5).half().to(device)
    pwl = (torch.rand((1, 1) + RUNET_TILE, generator=g) * 11.0).half().to(device)
    vec = (torch.rand((1, 3) + RUNET_TILE, generator=g) * 2 - 1).to(device)
    dev_buf = [torch.empty((1, 4) + RUNET_TILE, device=device) for _ in range(2)]
    copy_stream = torch.cuda.Stream(device)
    ready = [torch.cuda.Event() for _ in range(2)]
    freed = [torch.cuda.Event() for _ in range(2)]
    state = {'i': 0}

    def prefetch(i):
        slot = i % 2
        with torch.cuda.stream(copy_stream):
            copy_stream.wait_event(freed[slot])
            dev_buf[slot].copy_(host[i % n_host], non_blocking=True)
            ready[slot].record(copy_stream)

    for s in range(2):
        freed[s].record(torch.cuda.current_stream(device))
    prefetch(0)

    def step():
        i = state['i']
        slot = i % 2
        prefetch(i + 1)                                   # next tile in flight during this step
        torch.cuda.current_stream(device).wait_event(ready[slot])
        opt.zero_grad()
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out = model(dev_buf[slot])
            loss = hl.cross_entropy(out[:, 0:1], mask, pwl, method='pixel') + hl.MSELoss(out[:, 2:], vec)
        freed[slot].record(torch.cuda.current_stream(device))
        loss.backward()
        hcunet_amd.dist.allreduce_gradients(model)
        opt.step()
        state['i'] = i + 1
        return loss

    def sync():
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    sync()
    el = (time.perf_counter() - t0) / args.steps
    if world > 1:
        t = torch.tensor([el], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    vox = world * RUNET_TILE[0] * RUNET_TILE[1] * RUNET_TILE[2]
    roofline = kernels = None
    layers = None
    if not args.no_kernel_timing and world == 1:
        _lib.lib().hcu_timing_enable(args.steps * 2048)
        _lib.lib().hcu_timing_detail(1)
        hcunet_amd.chain.TAG_CHAINS = True
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(device)
        hcunet_amd.chain.TAG_CHAINS = False
        detail = _lib.timing_report()
        _lib.lib().hcu_timing_detail(0)
        _lib.lib().hcu_timing_disable()
        rep = {}
        per_layer = {}
        for k, v in detail.items():   # per kernel symbol, and per chain op tag
            r = rep.setdefault(k.partition('@')[0], dict(count=0, ms=0.0, flops=0.0, bytes=0.0))
            for f in r:
                r[f] += v[f]
            layer, phase = layer_of(k)
            lr = per_layer.setdefault(layer, dict(layer=layer, us=0.0, launches=0.0, gflop=0.0, kernels={}))
            lr['us'] += v['ms'] * 1e3 / args.steps
            lr['launches'] += v['count'] / args.steps
            lr['gflop'] += v['flops'] / args.steps / 1e9
            kk = '%s:%s' % (phase, k.partition('@')[0])
            lr['kernels'][kk] = round(lr['kernels'].get(kk, 0.0) + v['ms'] * 1e3 / args.steps, 2)
        layers = sorted(({"layer": r['layer'], "measured_us": round(r['us'], 2), "launches": r['launches'],
                          "gflop": round(r['gflop'], 4),
                          "tflops": round(r['gflop'] / r['us'] * 1e3, 2) if r['us'] else None,
                          "kernels": r['kernels']} for r in per_layer.values()),
                        key=lambda r: -r['measured_us'])
        total_ms = sum(v['ms'] for v in rep.values())
        name, d = max(rep.items(), key=lambda kv: kv[1]['ms'])
        avg_s = d['ms'] / d['count'] / 1e3
        bf_kernel = 'bf16' in name or name.startswith('bwgrad')
        if d['flops'] > 0:
            ach, bound, unit = d['flops'] / d['count'] / avg_s / 1e12, 'mfma', 'TFLOP/s'
            peak = PEAK_BF16_MFMA_TFLOPS if bf_kernel else PEAK_FP32_MFMA_TFLOPS
        else:
            ach, bound, unit, peak = d['bytes'] / d['count'] / avg_s / 1e9, 'hbm', 'GB/s', PEAK_HBM_GBS
        rp_us = rocprof_avg_us(name, 'runet')
        roofline = {"bound": bound, "achieved": ach, "peak": peak, "unit": unit, "frac": ach / peak,
                    "traffic": load_traffic(name, 'runet'), "kernel": name, "avg_launch_us": avg_s * 1e6,
                    "flops_per_launch": d['flops'] / d['count'] if d['flops'] > 0 else None,
                    "bytes_per_launch": d['bytes'] / d['count'] if d['bytes'] > 0 else None,
                    "rocprof_avg_launch_us": rp_us,
                    "rocprof_summary": 'profiles/%s_kernel_stats_runet.csv' % PROFILE_TAG if rp_us else None,
                    "launches_per_step": d['count'] / args.steps, "share_of_kernel_time": d['ms'] / total_ms}
        # the step's roofline from the algorithmic FLOPs and bytes every kernel
        # declares (bf16 MFMA peak for the bf16 kernels, fp32 for the rest):
        # sum over kernels of max(bytes / HBM peak, FLOPs / MFMA peak)
        roof_s = 0.0
        for k, v in rep.items():
            pk = PEAK_BF16_MFMA_TFLOPS if ('bf16' in k or k.startswith('bwgrad')) else PEAK_FP32_MFMA_TFLOPS
            roof_s += max(v['bytes'] / (PEAK_HBM_GBS * 1e9), v['flops'] / (pk * 1e12)) / args.steps
        step_roof = {"per_kernel_roofline_ms": roof_s * 1e3, "measured_ms": el * 1e3, "frac": roof_s / el,
                     "flops": sum(v['flops'] for v in rep.values()) / args.steps,
                     "declared_bytes": sum(v['bytes'] for v in rep.values()) / args.steps,
                     "note": "sum over the step's kernels of max(declared bytes / 8 TB/s, FLOPs / dense MFMA "
                             "peak); kernels that declare neither (loss, Adam, copies) count 0"}
        kernels = {"kernel_ms_per_step": total_ms / args.steps,
                   "launches_per_step": sum(v['count'] for v in rep.values()) / args.steps,
                   "algorithmic_tflops_per_step": sum(v['flops'] for v in rep.values()) / args.steps / 1e12,
                   "top": sorted(({"kernel": k, "ms_per_step": v['ms'] / args.steps,
                                   "launches_per_step": v['count'] / args.steps} for k, v in rep.items()),
                                 key=lambda r: -r['ms_per_step'])[:10]}
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        # bounded sample: one fp32 train step of the oracle restatement on the
        # benched 512x512x24 tile (same network, same step; ~10 s on 16 threads)
        from oracle import runet_oracle as ro, loss_oracle as lo
        threads = max(1, min(16, os.cpu_count() or 1))
        torch.set_num_threads(threads)
        tile = RUNET_TILE
        st = ro.state_of(RDCNet(4, 5), torch.float32)
        xs = host[0][:, :, :tile[0], :tile[1], :tile[2]].clone()
        t1 = time.perf_counter()
        o = ro.rdcnet_forward(st, xs)
        ls = lo.cross_entropy(o[:, 0:1], mask[:, :, :tile[0], :tile[1], :tile[2]].cpu().float(),
                              pwl[:, :, :tile[0], :tile[1], :tile[2]].cpu(), method='pixel') + \
            lo.MSELoss(o[:, 2:], vec[:, :, :tile[0], :tile[1], :tile[2]].cpu())
        ls.backward()
        tt = time.perf_counter() - t1
        cpu = {"value": tile[0] * tile[1] * tile[2] / tt, "unit": "voxels/s", "cores": threads, "kind": "port",
               "sample": "1 train step (fwd+loss+bwd, no optimizer) of the oracle restatement of RDCNet "
                         "(torch CPU fp32, %d threads) on a %s tile: %.2f s" % (threads, 'x'.join(map(str, tile)), tt)}
    line = {"metric": "training voxels/sec (fwd+bwd+step), r_unet.py RDCNet, 512x512x24 tiles",
            "value": vox / el, "unit": "voxels/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": el * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16", "data": "synthetic",
            "config": {"workload": "config 5: RDCNet(4, 5) train step (10 recurrent RDCBlock steps, "
                                   "stacked dilations 1..5), B=1, 512x512x24x4 tiles from pinned host "
                                   "memory with async prefetch, bf16 autocast",
                       "global_batch": world, "per_gpu_batch": 1, "parallelism": "dp%d" % world,
                       "final_loss": float(loss.item())},
            "roofline": roofline, "cpu_baseline": cpu, "kernels": kernels, "layers": layers}
    if not args.no_kernel_timing and world == 1:
        line["step_roofline"] = step_roof
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', default='2', choices=sorted(CONFIGS))
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-kernel-timing', action='store_true')
    ap.add_argument('--idle-steps', type=int, default=7,
                    help='extra single steps enqueued onto an idle queue after the '
                         'timed region (host_enqueue_idle_ms); 0 in profiling passes')
    ap.add_argument('--fresh-input', action='store_true',
                    help='clone the input every step (data-loader pattern; checks graph re-use)')
    ap.add_argument('--infer', action='store_true',
                    help='tiled inference driver throughput (SURVEY 8f-1) instead of training')
    ap.add_argument('--runet', action='store_true',
                    help='BASELINE config 5: r_unet.py RDCNet training on 512x512x24 tiles (bf16)')
    ap.add_argument('--input-dtype', default='fp32', choices=['fp32', 'fp16', 'bf16'],
                    help='dtype of the [B,4,X,Y,Z] input volume handed to forward (16-bit confocal '
                         'volumes: bf16 configs only, read directly by the first convolution)')
    args = ap.parse_args()
    if args.infer:
        return infer_main(args)
    if args.runet:
        return runet_main(args)

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    device = torch.device('cuda', local)
    cfg = CONFIGS[args.config]
    B = cfg['batch']

    torch.manual_seed(0)
    model = Unet_Constructor(**cfg['kw']).to(device).train()
    hcunet_amd.dist.broadcast_parameters(model)
    opt = hcunet_amd.optim.Adam(model.parameters(), lr=1e-3)
    x, mask, pwl = synth_inputs(B, 1000 + rank, device)

    bf16 = cfg['dtype'] == 'bf16'
    if args.input_dtype != 'fp32':
        if not bf16:
            raise SystemExit('--input-dtype %s: 16-bit input volumes need a bf16 config (the fp32 '
                             'reference path raises on them)' % args.input_dtype)
        x = x.to(torch.float16 if args.input_dtype == 'fp16' else torch.bfloat16)

    def step():
        opt.zero_grad()
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=bf16):
            # --fresh-input: a new input tensor every step, as a data loader hands over
            out = model(x.clone() if args.fresh_input else x)
            loss = cross_entropy(out, mask, pwl, method='pixel')
        loss.backward()
        hcunet_amd.dist.allreduce_gradients(model)
        opt.step()
        return loss

    def sync():
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    t_enq = time.perf_counter() - t0   # host time to enqueue the K steps
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.item())
    ms_per_step = elapsed / args.steps * 1e3
    # host cost of ONE step enqueued onto an idle, synchronised queue (no
    # backpressure from earlier steps): the median of 7 such steps.  If this
    # approaches ms_per_step the step is host-bound on this box.
    idle_enq = []
    for _ in range(args.idle_steps):
        sync()
        t1 = time.perf_counter()
        step()
        idle_enq.append(time.perf_counter() - t1)
    sync()
    vox = world * B * TILE[0] * TILE[1] * TILE[2] * args.steps
    value = vox / elapsed

    roofline = None
    kernels = None
    layer_rows = None
    tiling = dict(zip(('table_entries', 'timed_by_this_process'), _lib.tuning_entries()))
    tiling['mode'] = _lib.tuning_mode()
    if os.environ.get('HCU_TUNE_SAVE'):
        tiling['saved'] = _lib.tuning_save(os.environ['HCU_TUNE_SAVE'])
    if not args.no_kernel_timing:
        _lib.lib().hcu_timing_enable(args.steps * 512)
        _lib.lib().hcu_timing_detail(1)
        for _ in range(args.steps):
            step()
        sync()
        detail = _lib.timing_report()
        _lib.lib().hcu_timing_detail(0)
        _lib.lib().hcu_timing_disable()
        layer_rows = layer_table(detail, cfg, B, args.steps)
        rep = {}
        for k, v in detail.items():   # per kernel symbol
            r = rep.setdefault(k.partition('@')[0], dict(count=0, ms=0.0, flops=0.0, bytes=0.0))
            for f in r:
                r[f] += v[f]
        total_ms = sum(v['ms'] for v in rep.values())
        name, d = max(rep.items(), key=lambda kv: kv[1]['ms'])
        avg_s = d['ms'] / d['count'] / 1e3
        if d['flops'] > 0:
            ach = d['flops'] / d['count'] / avg_s / 1e12
            bf_kernel = 'bf16' in name or name.startswith('bwgrad')   # bconv_kernel<f32,...> is fp32
            bound, unit = 'mfma', 'TFLOP/s'
            peak = PEAK_BF16_MFMA_TFLOPS if bf_kernel else PEAK_FP32_MFMA_TFLOPS
        else:
            ach = d['bytes'] / d['count'] / avg_s / 1e9
            bound, peak, unit = 'hbm', PEAK_HBM_GBS, 'GB/s'
        rp_us = rocprof_avg_us(name, args.config)
        rp_serial_us = rocprof_avg_us(name, args.config, 'serial_')
        per_launch = (d['flops'] if d['flops'] > 0 else d['bytes']) / d['count']
        scale = 1e12 if d['flops'] > 0 else 1e9
        roofline = {"bound": bound, "achieved": ach, "peak": peak, "unit": unit,
                    "frac": ach / peak, "traffic": load_traffic(name, args.config), "kernel": name,
                    # HIP events around each launch, kernels serialized (timing pass)
                    "avg_launch_us": avg_s * 1e6,
                    # rocprofv3 --stats of the serialized step (HCU_SIDE=0): the
                    # same conditions, so it must agree with avg_launch_us
                    "rocprof_serial_avg_launch_us": rp_serial_us,
                    # rocprofv3 --stats of the production step: the weight-gradient
                    # branch shares the CUs with the chain, so its kernels run longer
                    "rocprof_avg_launch_us": rp_us,
                    "frac_rocprof_serial": (per_launch / (rp_serial_us * 1e-6) / scale / peak
                                            if rp_serial_us else None),
                    "frac_rocprof": (per_launch / (rp_us * 1e-6) / scale / peak if rp_us else None),
                    "launches_per_step": d['count'] / args.steps,
                    "flops_per_launch": d['flops'] / d['count'],
                    "share_of_kernel_time": d['ms'] / total_ms}
        step_flops = sum(v['flops'] for v in rep.values()) / args.steps
        kernels = {"kernel_ms_per_step": total_ms / args.steps,
                   "algorithmic_tflops_per_step": step_flops / 1e12,
                   "step_mfma_tflops": step_flops / (ms_per_step / 1e3) / 1e12,
                   "top": sorted(({"kernel": k, "ms_per_step": v['ms'] / args.steps,
                                   "launches_per_step": v['count'] / args.steps}
                                  for k, v in rep.items()),
                                 key=lambda r: -r['ms_per_step'])[:8]}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, x, mask, pwl)

    if rank == 0:
        line = {"metric": METRIC, "value": value, "unit": "voxels/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": cfg['dtype'], "data": "synthetic",
                "config": {"workload": "%s train step (fwd + pixel BCE + bwd + Adam), B=%d per "
                                       "GPU, %dx%dx%dx4 volumes" % ((cfg['desc'], B) + TILE),
                           "global_batch": B * world, "per_gpu_batch": B,
                           "input_dtype": args.input_dtype,
                           "parallelism": "dp%d" % world, "final_loss": final_loss,
                           "host_enqueue_ms_per_step": t_enq / args.steps * 1e3,
                           "host_enqueue_idle_ms": (statistics.median(idle_enq) * 1e3
                                                    if idle_enq else None)},
                "roofline": roofline, "cpu_baseline": cpu, "kernels": kernels,
                "tiling": tiling}
        # SURVEY §8d per-layer roofline of the whole step (sum over layers of
        # max(bytes / 8 TB/s, flops / dense MFMA peak), hcunet_amd/roofline.py)
        # vs the measured step
        roof_ms, roof_fl, roof_by = roofline_mod.step_roofline(cfg['kw'], B, TILE, bf16)
        line["step_roofline"] = {"per_layer_roofline_ms": roof_ms, "measured_ms": ms_per_step,
                                 "frac": roof_ms / ms_per_step, "flops": roof_fl,
                                 "compulsory_bytes": roof_by}
        if layer_rows is not None:
            line["layers"] = layer_rows
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
