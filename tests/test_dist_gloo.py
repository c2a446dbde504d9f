"""CPU, world_size 2 over gloo: the data-parallel step.

Each rank holds a batch shard; after backward the flat gradient is averaged
with ONE all-reduce (hcunet_amd.dist.allreduce_gradients), so every rank's
gradient equals the mean of the per-shard reference gradients, and the
parameters start identical (broadcast_parameters).  BatchNorm statistics stay
per rank (no SyncBN), as the reference would compute them per shard."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import inputs, unet_oracle as uo

KW = dict(image_dimensions=3, in_channels=4, out_channels=1, feature_sizes=[2, 4],
          kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)}, upsample_kernel=(2, 2, 2),
          max_pool_kernel=(2, 2, 1), upsample_stride=(2, 2, 1))
SHAPE = (4, 4, 18, 18, 3)   # global batch 4 -> 2 per rank


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from hcat.unet import Unet_Constructor
        import hcunet_amd
        from hcunet_amd.unet import bn_modules
        torch.manual_seed(rank)          # deliberately different init per rank
        m = Unet_Constructor(**KW)
        hcunet_amd.dist.broadcast_parameters(m)
        sd = {k: v.clone() for k, v in m.state_dict().items()}
        spec = uo.normalize_spec(**KW)
        x = inputs.make_x(SHAPE)
        shard = slice(rank * 2, rank * 2 + 2)
        net = uo.OracleUnet(spec, sd)
        out = net.forward(torch.from_numpy(x[shard]))
        ms = (2, 1) + tuple(out.shape[2:])
        loss = uo.pixel_loss(out, torch.from_numpy(inputs.make_mask((4,) + ms[1:])[shard]),
                             torch.from_numpy(inputs.make_pwl((4,) + ms[1:])[shard]))
        loss.backward()
        local = net.grads()
        # The production layout, exactly as a GPU backward leaves it: parameters
        # are views of the engine's flat buffer and every .grad is a view of
        # grad_flat, the head of the engine's communication buffer.
        eng = m.engine()
        eng.params_ready(require_gpu=False)
        G, accumulate, finish = eng.grad_target()
        assert accumulate == 0
        off = 0
        for n, p in m.named_parameters():
            G[off:off + p.numel()].copy_(local[n].reshape(-1))
            off += p.numel()
        finish()
        assert all(p.grad.data_ptr() == G.data_ptr() + 4 * o
                   for p, o in zip(m.parameters(), _offsets(m)))
        # per-shard running statistics after the train-mode forward (rank-local)
        for bn, name in zip(bn_modules(m), uo.bn_names(spec)):
            bn.running_mean.copy_(net.state[name + '.running_mean'])
            bn.running_var.copy_(net.state[name + '.running_var'])
        local_rs = {k: v.numpy().copy() for k, v in m.state_dict().items() if 'running' in k}
        calls = []
        real = dist.all_reduce

        def counting_all_reduce(*a, **k):
            calls.append(a[0].numel())
            return real(*a, **k)
        dist.all_reduce = counting_all_reduce
        try:
            hcunet_amd.dist.allreduce_gradients(m)
        finally:
            dist.all_reduce = real
        # numpy copies: tensors in a Queue would be shared with the exiting worker
        q.put((rank, {k: v.numpy().copy() for k, v in sd.items()},
               {n: p.grad.numpy().copy() for n, p in m.named_parameters()},
               {n: g.numpy().copy() for n, g in local.items()},
               {k: v.numpy().copy() for k, v in m.state_dict().items() if 'running' in k},
               local_rs, calls, eng.comm_flat.data_ptr() == G.data_ptr()))
    finally:
        dist.destroy_process_group()


def _offsets(m):
    out, off = [], 0
    for p in m.parameters():
        out.append(off)
        off += p.numel()
    return out


def test_dp_allreduce_matches_mean_of_shard_grads():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, sd, red, local, rs, lrs, calls, headed = q.get(timeout=300)
        res[r] = tuple({k: torch.from_numpy(v) for k, v in d.items()} for d in (sd, red, local, rs, lrs))
        res[r] += (calls, headed)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sd0, red0, loc0, rs0, lrs0, calls0, headed0 = res[0]
    sd1, red1, loc1, rs1, lrs1, calls1, headed1 = res[1]
    # ONE collective per step, over grads + running statistics, on the flat path
    n_params = sum(v.numel() for v in loc0.values())
    n_stats = sum(v.numel() for v in rs0.values())
    assert calls0 == [n_params + n_stats] and calls1 == calls0
    assert headed0 and headed1
    for k in sd0:   # broadcast made the replicas identical (rank 0's init)
        assert torch.equal(sd0[k], sd1[k]), k
    torch.manual_seed(0)
    from hcat.unet import Unet_Constructor
    ref_sd = Unet_Constructor(**KW).state_dict()
    for k in sd0:
        assert torch.equal(sd0[k], ref_sd[k]), k
    for n in red0:
        mean = (loc0[n] + loc1[n]) / 2
        assert torch.allclose(red0[n], mean, rtol=1e-6, atol=1e-9), n
        assert torch.equal(red0[n], red1[n]), n
    # running statistics: rank-symmetric after the step, = mean of the shards'
    for k in rs0:
        assert not torch.equal(lrs0[k], lrs1[k]) or 'var' in k, k   # shards differ
        assert torch.equal(rs0[k], rs1[k]), k
        assert torch.allclose(rs0[k], (lrs0[k] + lrs1[k]) / 2, rtol=1e-6, atol=1e-9), k


def test_bucket_ranges_partition_the_communication_buffer():
    """dist.bucket_ranges: decoder + statistics tail, deep encoder levels, rest
    (out_conv and the shallow levels) -- contiguous, disjoint, covering
    [0, n_params + n_stats), each range holding exactly its modules' params."""
    from hcat.unet import Unet_Constructor
    from hcunet_amd import dist as hd
    kw = dict(KW, feature_sizes=[8, 16, 32, 64, 128])
    m = Unet_Constructor(**kw)
    n = sum(p.numel() for p in m.parameters())
    r = hd.bucket_ranges(m, 3, 100)
    (d0, d1), (e0, e1), (s0, s1) = r
    assert (s0, s1, e1, d1) == (0, e0, d0, n + 100)
    off = 0
    for name, p in m.named_parameters():
        lo, hi = off, off + p.numel()
        off = hi
        if name.startswith('up_steps'):
            assert d0 <= lo and hi <= d1, name
        elif name.startswith('down_steps') and int(name.split('.')[1]) >= 3:
            assert e0 <= lo and hi <= e1, name
        else:
            assert s0 <= lo and hi <= s1, name
    assert hd.bucket_ranges(Unet_Constructor(**KW), 3, 0) is None   # 2 levels: no deep range


def _ranges_worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from hcunet_amd import dist as hd
        g = torch.Generator().manual_seed(rank)
        buf = torch.randn(1000, generator=g)
        whole = buf.clone()
        hd._reduce(whole, None, world)
        for lo, hi in [(600, 1000), (250, 600), (0, 250)]:
            hd._reduce(buf[lo:hi], None, world)
        q.put((rank, whole.numpy().copy(), buf.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_reduction_in_ranges_equals_one_reduction():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ranges_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, whole, parts = q.get(timeout=120)
        res[r] = (whole, parts)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import numpy as np
    for r in (0, 1):
        np.testing.assert_array_equal(res[r][0], res[r][1])
    np.testing.assert_array_equal(res[0][1], res[1][1])


def _runet_worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from hcunet_amd.r_unet import RecursiveUnet
        import hcunet_amd
        torch.manual_seed(0)
        m = RecursiveUnet(image_dimensions=3)
        g = torch.Generator().manual_seed(100 + rank)
        bns = [b for b in m.modules() if isinstance(b, torch.nn.BatchNorm3d)]
        with torch.no_grad():
            for b in bns:   # per-rank running statistics, as a per-shard forward leaves them
                b.running_mean.copy_(torch.randn(b.running_mean.shape, generator=g))
                b.running_var.copy_(torch.rand(b.running_var.shape, generator=g) + 0.5)
            for p in m.parameters():
                p.grad = torch.randn(p.shape, generator=g)
        local = {k: v.clone().numpy() for k, v in m.state_dict().items() if 'running' in k}
        lg = {n: p.grad.clone().numpy() for n, p in m.named_parameters()}
        hcunet_amd.dist.allreduce_gradients(m)
        q.put((rank, len(bns), local, lg,
               {k: v.clone().numpy() for k, v in m.state_dict().items() if 'running' in k},
               {n: p.grad.clone().numpy() for n, p in m.named_parameters()}))
    finally:
        dist.destroy_process_group()


def test_dp_reduces_recursive_unet_batchnorm_statistics():
    """Any module's BatchNorm running statistics join the reduction (not only
    Unet_Constructor's): RecursiveUnet's 16 BatchNorm3d layers
    (/root/reference/hcat/r_unet.py:276-277,326-327) stay rank-symmetric."""
    import numpy as np
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_runet_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, *rest = q.get(timeout=300)
        res[r] = rest
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (nbn, l0, g0, s0, r0), (_, l1, g1, s1, r1) = res[0], res[1]
    assert nbn == 16   # fz / fh alias down2_*/down3_*/up1_*: state_dict repeats those keys
    for k in s0:
        np.testing.assert_array_equal(s0[k], s1[k])
        np.testing.assert_allclose(s0[k], (l0[k] + l1[k]) / 2, rtol=1e-6, atol=1e-7, err_msg=k)
    for n in r0:
        np.testing.assert_array_equal(r0[n], r1[n])
        np.testing.assert_allclose(r0[n], (g0[n] + g1[n]) / 2, rtol=1e-6, atol=1e-7, err_msg=n)


RDC_SHAPE = (2, 4, 24, 24, 10)   # two tiles: one per rank (config 5 shards tiles by rank)


def _rdc_loss(out, rank):
    from oracle import loss_oracle as lo
    oshape = tuple(out.shape)
    ms = (RDC_SHAPE[0], 1) + oshape[2:]
    sl = slice(rank, rank + 1)
    mask = torch.from_numpy(inputs.make_mask(ms)[sl]).float()
    pwl = torch.from_numpy(inputs.make_pwl(ms)[sl])
    vec = torch.from_numpy(inputs.make_x((RDC_SHAPE[0], 3) + oshape[2:], seed=4)[sl] * 0.5)
    return lo.cross_entropy(out[:, 0:1], mask, pwl, method='pixel') + lo.MSELoss(out[:, 2:], vec)


def _rdc_worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from hcat.r_unet import RDCNet
        import hcunet_amd
        from oracle import runet_oracle as ro
        torch.manual_seed(rank)              # different init per rank
        m = RDCNet(4, 5)
        hcunet_amd.dist.broadcast_parameters(m)
        sd = {k: v.numpy().copy() for k, v in m.state_dict().items()}
        st = ro.state_of(m, torch.float32)
        x = torch.from_numpy(inputs.make_x(RDC_SHAPE)[rank:rank + 1])
        _rdc_loss(ro.rdcnet_forward(st, x), rank).backward()
        local = {n: st[n].grad.clone() for n, _ in m.named_parameters()}
        # the production layout of the layer chains (hcunet_amd.chain.FlatParams):
        # every .grad a view of one flat buffer in parameter order
        n_all = sum(p.numel() for p in m.parameters())
        G = torch.zeros(n_all)
        off = 0
        for n, p in m.named_parameters():
            p.grad = G[off:off + p.numel()].view_as(p)
            p.grad.copy_(local[n])
            off += p.numel()
        calls = []
        real = dist.all_reduce

        def counting_all_reduce(*a, **k):
            calls.append((a[0].numel(), a[0].data_ptr() == G.data_ptr()))
            return real(*a, **k)
        dist.all_reduce = counting_all_reduce
        try:
            hcunet_amd.dist.allreduce_gradients(m)
        finally:
            dist.all_reduce = real
        q.put((rank, sd, {n: p.grad.numpy().copy() for n, p in m.named_parameters()},
               {n: g.numpy().copy() for n, g in local.items()}, calls))
    finally:
        dist.destroy_process_group()


def test_dp_rdcnet_tiles_sharded_by_rank():
    """BASELINE config 5 data-parallel (bench.py --runet under torchrun): one
    RDCNet tile per rank, parameters broadcast from rank 0, the gradients
    averaged by ONE in-place collective over the flat gradient buffer the
    layer chains fill -- every rank ends with the mean of the per-tile oracle
    gradients (the reference's training pattern, tests/r_unet_test.py:37-56,
    per tile)."""
    import numpy as np
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rdc_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, sd, red, local, calls = q.get(timeout=300)
        res[r] = (sd, red, local, calls)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (sd0, red0, loc0, calls0), (sd1, red1, loc1, calls1) = res[0], res[1]
    n_params = sum(v.size for v in loc0.values())
    assert calls0 == calls1 == [(n_params, True)]   # one collective, in place on the flat buffer
    from hcat.r_unet import RDCNet
    torch.manual_seed(0)
    ref = RDCNet(4, 5).state_dict()
    for k in sd0:
        np.testing.assert_array_equal(sd0[k], sd1[k], err_msg=k)
        np.testing.assert_array_equal(sd0[k], ref[k].numpy(), err_msg=k)
    for n in red0:
        assert not np.array_equal(loc0[n], loc1[n]), n      # the two tiles differ
        np.testing.assert_array_equal(red0[n], red1[n], err_msg=n)
        np.testing.assert_allclose(red0[n], (loc0[n] + loc1[n]) / 2, rtol=1e-6, atol=1e-9, err_msg=n)
