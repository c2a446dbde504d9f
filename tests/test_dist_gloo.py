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
        for n, p in m.named_parameters():   # hand the shard's grads to the module
            p.grad = local[n].clone()
        hcunet_amd.dist.allreduce_gradients(m)
        # numpy copies: tensors in a Queue would be shared with the exiting worker
        q.put((rank, {k: v.numpy().copy() for k, v in sd.items()},
               {n: p.grad.numpy().copy() for n, p in m.named_parameters()},
               {n: g.numpy().copy() for n, g in local.items()}))
    finally:
        dist.destroy_process_group()


def test_dp_allreduce_matches_mean_of_shard_grads():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, sd, red, local = q.get(timeout=300)
        res[r] = tuple({k: torch.from_numpy(v) for k, v in d.items()} for d in (sd, red, local))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sd0, red0, loc0 = res[0]
    sd1, red1, loc1 = res[1]
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
