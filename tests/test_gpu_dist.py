"""Data-parallel step on the GPU path, world size 2 over gloo with both ranks
on cuda:0 (the 8-GPU RCCL run is the driver's): real native forward/backward
per batch shard, then hcunet_amd.dist.allreduce_gradients -- ONE logical
reduction of the flat gradient buffer + BatchNorm running statistics, the
statistics moved in and out of it by one kernel each (hcu_gather_vectors):
either one collective (HCU_DP_OVERLAP=0) or, by default, three ranges on a
communication stream that wait for the backward's gradient-ready events
(decoder, deep levels, rest) -- a partition of the same buffer.  Checks: the
collectives cover the buffer exactly once, rank-symmetric results, reduced =
mean of the per-rank values, both modes agree bitwise, and the deterministic
tiling mode every rank plans with."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import inputs

pytestmark = pytest.mark.gpu

KW = dict(image_dimensions=3, in_channels=4, out_channels=1, feature_sizes=[4, 8, 16],
          kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)}, upsample_kernel=(2, 2, 2),
          max_pool_kernel=(2, 2, 1), upsample_stride=(2, 2, 1))
SHAPE = (4, 4, 44, 44, 5)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q, overlap):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['HCU_DP_OVERLAP'] = '1' if overlap else '0'
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from hcat.loss import cross_entropy
        from hcat.unet import Unet_Constructor
        import hcunet_amd
        from hcunet_amd import _lib
        from hcunet_amd.unet import bn_modules
        torch.manual_seed(rank)
        m = Unet_Constructor(**KW).cuda().train()
        hcunet_amd.dist.broadcast_parameters(m)
        mode = _lib.tuning_mode()
        x = torch.from_numpy(inputs.make_x(SHAPE))[rank * 2:rank * 2 + 2].cuda()
        out = m(x)
        ms = (4, 1) + tuple(out.shape[2:])
        mask = torch.from_numpy(inputs.make_mask(ms))[rank * 2:rank * 2 + 2].cuda()
        pwl = torch.from_numpy(inputs.make_pwl(ms))[rank * 2:rank * 2 + 2].cuda()
        cross_entropy(out, mask, pwl, method='pixel').backward()
        torch.cuda.synchronize()
        local = {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()}
        lrs = {k: v.detach().cpu().clone() for k, v in m.state_dict().items() if 'running' in k}
        calls = []
        real = dist.all_reduce

        def counting(*a, **k):
            calls.append(a[0].numel())
            return real(*a, **k)
        dist.all_reduce = counting
        try:
            hcunet_amd.dist.allreduce_gradients(m)
        finally:
            dist.all_reduce = real
        torch.cuda.synchronize()
        q.put((rank, {n: v.numpy() for n, v in local.items()},
               {n: p.grad.detach().cpu().numpy() for n, p in m.named_parameters()},
               {k: v.numpy() for k, v in lrs.items()},
               {k: v.detach().cpu().numpy() for k, v in m.state_dict().items() if 'running' in k},
               calls, mode, len(bn_modules(m))))
    finally:
        dist.destroy_process_group()


def _run(overlap):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, overlap)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, *rest = q.get(timeout=240)
        res[r] = rest
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_dp_step_on_gpu_one_collective_rank_symmetric():
    import numpy as np
    res = _run(False)
    _check(res, overlapped=False)
    res_ov = _run(True)
    _check(res_ov, overlapped=True)
    for r in (0, 1):   # the overlapped ranges reduce the same values: bitwise equal
        for a, b in zip(res[r][1:4], res_ov[r][1:4]):
            for k in a:
                np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def _check(res, overlapped):
    (loc0, red0, lrs0, rs0, calls0, mode0, nbn), (loc1, red1, lrs1, rs1, calls1, mode1, _) = res[0], res[1]
    import numpy as np
    n_params = sum(v.size for v in loc0.values())
    n_stats = sum(v.size for v in rs0.values())
    assert calls0 == calls1
    if overlapped:   # decoder + statistics, deep levels, rest: a partition
        assert len(calls0) == 3 and sum(calls0) == n_params + n_stats, calls0
    else:
        assert calls0 == [n_params + n_stats]
    assert mode0 == mode1 == 1          # the deterministic tiling mode
    for n in red0:
        np.testing.assert_array_equal(red0[n], red1[n])
        np.testing.assert_allclose(red0[n], (loc0[n] + loc1[n]) / 2, rtol=1e-6, atol=1e-9, err_msg=n)
    assert len(rs0) == 2 * nbn
    for k in rs0:
        np.testing.assert_array_equal(rs0[k], rs1[k])
        np.testing.assert_allclose(rs0[k], (lrs0[k] + lrs1[k]) / 2, rtol=1e-6, atol=1e-9, err_msg=k)
