"""Data-parallel step on the GPU path, world size 2 over gloo with both ranks
on cuda:0 (the 8-GPU RCCL run is the driver's): real native forward/backward
per batch shard, then hcunet_amd.dist.allreduce_gradients -- ONE logical
reduction of the flat gradient buffer + BatchNorm running statistics, the
statistics moved in and out of it by one kernel each (hcu_gather_vectors):
either one collective (HCU_DP_OVERLAP=0) or, by default, three ranges on a
communication stream that wait for the backward's gradient-ready events
(decoder, deep levels, rest) -- a partition of the same buffer.

Checks: each rank's native gradients equal the oracle's on that rank's shard
(the reference pattern /root/reference/tests/r_unet_test.py:48-56 per shard);
the collectives cover the buffer exactly once; rank-symmetric results; reduced
= mean of the per-rank values; the overlapped mode, called straight after
backward with no host synchronisation (so each range really waits on its
event), equals the single collective bitwise; with the backward replayed from
a graph (HCU_GRAPHS=1) the events are not live and one collective runs; an
in-place gradient edit between backward and the reduction makes the overlapped
mode fall back to one collective behind the caller's stream."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import inputs, unet_oracle as uo

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


def _worker(rank, world, port, q, overlap, graphs, touch):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['HCU_DP_OVERLAP'] = '1' if overlap else '0'
    if graphs:
        os.environ['HCU_GRAPHS'] = '1'
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
        sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        mode = _lib.tuning_mode()
        sh = slice(rank * 2, rank * 2 + 2)
        x = torch.from_numpy(inputs.make_x(SHAPE))[sh].cuda()
        out = m(x)
        ms = (4, 1) + tuple(out.shape[2:])
        mask = torch.from_numpy(inputs.make_mask(ms))[sh].cuda()
        pwl = torch.from_numpy(inputs.make_pwl(ms))[sh].cuda()
        cross_entropy(out, mask, pwl, method='pixel').backward()
        local, lrs = None, None
        if not overlap:   # the per-rank values, read before the reduction
            torch.cuda.synchronize()
            local = {n: p.grad.detach().cpu().numpy().copy() for n, p in m.named_parameters()}
            lrs = {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items() if 'running' in k}
        if touch:   # in-place gradient work queued on the caller's stream
            with torch.no_grad():
                for p in m.parameters():
                    p.grad.mul_(2.0)
        calls = []
        real = dist.all_reduce

        def counting(*a, **k):
            calls.append(a[0].numel())
            return real(*a, **k)
        dist.all_reduce = counting
        try:
            hcunet_amd.dist.allreduce_gradients(m)   # straight after backward: no host sync
        finally:
            dist.all_reduce = real
        torch.cuda.synchronize()
        oracle = None
        if not overlap and not graphs and not touch:
            # the oracle on this rank's shard, from the broadcast parameters
            spec = uo.normalize_spec(**KW)
            net = uo.OracleUnet(spec, sd)
            o = net.forward(torch.from_numpy(inputs.make_x(SHAPE)[sh]))
            loss = uo.pixel_loss(o, torch.from_numpy(inputs.make_mask(ms)[sh]),
                                 torch.from_numpy(inputs.make_pwl(ms)[sh]))
            loss.backward()
            oracle = {n: g.detach().numpy().copy() for n, g in net.grads().items()}
        q.put((rank, local,
               {n: p.grad.detach().cpu().numpy() for n, p in m.named_parameters()},
               lrs,
               {k: v.detach().cpu().numpy() for k, v in m.state_dict().items() if 'running' in k},
               calls, mode, len(bn_modules(m)), oracle))
    finally:
        dist.destroy_process_group()


def _run(overlap, graphs=False, touch=False):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, overlap, graphs, touch)) for r in range(2)]
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


def _rel(a, b):
    import numpy as np
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def test_dp_step_on_gpu_one_collective_rank_symmetric():
    import numpy as np
    res = _run(False)
    n_params = _check(res, n_coll=1, loc=None)
    # each rank's native gradients = the oracle's on that rank's shard
    for r in (0, 1):
        loc, oracle = res[r][0], res[r][7]
        for n, g in oracle.items():
            if n.endswith('conv1.bias') or n.endswith('conv2.bias') or n.endswith('up_conv.bias'):
                assert np.abs(loc[n] - g).max() <= 1e-4, n   # BN-cancelled: ~0 either way
            else:
                assert _rel(loc[n], g) <= 1e-3, (r, n, _rel(loc[n], g))
    base = {r: res[r][0] for r in (0, 1)}
    # overlapped, straight after backward: the same bits
    res_ov = _run(True)
    _check(res_ov, n_coll=3, loc=base, n_params=n_params)
    for r in (0, 1):
        for a, b in zip(res[r][1:4:2], res_ov[r][1:4:2]):
            for k in a:
                np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    # backward replayed from a graph: events not live -> one collective, same bits
    res_g = _run(True, graphs=True)
    _check(res_g, n_coll=1, loc=base, n_params=n_params)
    for r in (0, 1):
        for k in res[r][1]:
            np.testing.assert_array_equal(res[r][1][k], res_g[r][1][k], err_msg=k)
    # gradients edited in place after backward: the overlapped mode falls back
    res_t = _run(True, touch=True)
    _check(res_t, n_coll=1, loc={r: {k: 2.0 * v for k, v in base[r].items()} for r in (0, 1)},
           n_params=n_params)


def _check(res, n_coll, loc, n_params=None):
    (loc0, red0, lrs0, rs0, calls0, mode0, nbn, _), (loc1, red1, lrs1, rs1, calls1, mode1, _, _) = \
        res[0], res[1]
    import numpy as np
    if loc is not None:
        loc0, loc1 = loc[0], loc[1]
    n_params = n_params or sum(v.size for v in loc0.values())
    n_stats = sum(v.size for v in rs0.values())
    assert calls0 == calls1
    assert len(calls0) == n_coll and sum(calls0) == n_params + n_stats, calls0
    assert mode0 == mode1 == 1          # the deterministic tiling mode
    for n in red0:
        np.testing.assert_array_equal(red0[n], red1[n])
        np.testing.assert_allclose(red0[n], (loc0[n] + loc1[n]) / 2, rtol=1e-6, atol=1e-9, err_msg=n)
    assert len(rs0) == 2 * nbn
    for k in rs0:
        np.testing.assert_array_equal(rs0[k], rs1[k])
        if lrs0 is not None:
            np.testing.assert_allclose(rs0[k], (lrs0[k] + lrs1[k]) / 2, rtol=1e-6, atol=1e-9, err_msg=k)
    return n_params


from tests.test_dist_gloo import RDC_SHAPE  # noqa: E402  (one RDCNet tile per rank)


def _rdc_worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from hcat.r_unet import RDCNet
        import hcunet_amd
        from oracle import runet_oracle as ro
        from tests.test_dist_gloo import _rdc_loss
        torch.manual_seed(rank)                  # different init per rank
        m = RDCNet(4, 5).cuda().train()
        xr = torch.from_numpy(inputs.make_x(RDC_SHAPE)[rank:rank + 1])
        # a step BEFORE the broadcast: the chains keep packed weight images of
        # this rank's own initial weights, which the broadcast must invalidate
        (m(xr.cuda()).float() ** 2).mean().backward()
        hcunet_amd.dist.broadcast_parameters(m)
        m.zero_grad(set_to_none=True)
        sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        out = m(xr.cuda())
        import hcat.loss as hl
        oshape = tuple(out.shape)
        ms = (RDC_SHAPE[0], 1) + oshape[2:]
        sl = slice(rank, rank + 1)
        mask = torch.from_numpy(inputs.make_mask(ms)[sl]).cuda()
        pwl = torch.from_numpy(inputs.make_pwl(ms)[sl]).cuda()
        vec = torch.from_numpy(inputs.make_x((RDC_SHAPE[0], 3) + oshape[2:], seed=4)[sl] * 0.5).cuda()
        (hl.cross_entropy(out[:, 0:1], mask, pwl, method='pixel') + hl.MSELoss(out[:, 2:], vec)).backward()
        torch.cuda.synchronize()
        local = {n: p.grad.detach().cpu().numpy().copy() for n, p in m.named_parameters()}
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
        # the oracle on this rank's tile, from the broadcast parameters
        ref = RDCNet(4, 5)
        ref.load_state_dict(sd)
        st = ro.state_of(ref, torch.float32)
        _rdc_loss(ro.rdcnet_forward(st, xr), rank).backward()
        oracle = {n: st[n].grad.numpy().copy() for n, _ in m.named_parameters()}
        q.put((rank, {k: v.numpy() for k, v in sd.items()}, local,
               {n: p.grad.detach().cpu().numpy() for n, p in m.named_parameters()}, calls, oracle))
    finally:
        dist.destroy_process_group()


def test_dp_rdcnet_on_gpu_tiles_sharded_by_rank():
    """Config 5 data-parallel on the native path, two gloo ranks on one GPU:
    each rank trains RDCNet on its own tile after a step taken BEFORE the
    broadcast (so the chains' cached weight images hold that rank's own
    initial weights and must be invalidated by broadcast_parameters); its
    native gradients equal the oracle's on its tile from rank 0's parameters,
    and ONE collective leaves both ranks with their mean."""
    import numpy as np
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rdc_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, *rest = q.get(timeout=240)
        res[r] = rest
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (sd0, loc0, red0, calls0, or0), (sd1, loc1, red1, calls1, or1) = res[0], res[1]
    n_params = sum(v.size for v in loc0.values())
    assert calls0 == calls1 == [n_params]
    for k in sd0:
        np.testing.assert_array_equal(sd0[k], sd1[k], err_msg=k)
    for loc, orc, r in ((loc0, or0, 0), (loc1, or1, 1)):
        for n, g in orc.items():
            assert _rel(loc[n], g) <= 1e-3, (r, n, _rel(loc[n], g))
    for n in red0:
        np.testing.assert_array_equal(red0[n], red1[n], err_msg=n)
        np.testing.assert_allclose(red0[n], (loc0[n] + loc1[n]) / 2, rtol=1e-6, atol=1e-9, err_msg=n)
