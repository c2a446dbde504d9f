"""Data-parallel training over RCCL: batch sharded across ranks (one process
per GPU), one all-reduce of the flat gradient buffer per step.

The reference has no distributed code; this is the one collective
the build adds.  BatchNorm statistics stay per-rank (no SyncBN), as a
per-rank reference run would compute them.
"""
import torch
import torch.distributed as dist


def _avg_supported(group=None):
    return dist.get_backend(group) == 'nccl'


def allreduce_gradients(module, group=None):
    """Average parameter gradients of `module` across ranks in place.

    Uses the module's flat gradient buffer (one collective) when every .grad is
    a view of it, else flattens the gradients into one temporary buffer."""
    if not dist.is_available() or not dist.is_initialized():
        return
    world = dist.get_world_size(group)
    if world == 1:
        return
    params = [p for p in module.parameters() if p.grad is not None]
    if not params:
        return
    eng = getattr(module, '_engine', None)
    G = getattr(eng, 'grad_flat', None) if eng is not None else None
    flat_ok = False
    if G is not None and len(params) == len(list(module.parameters())):
        base, off, flat_ok = G.data_ptr(), 0, True
        for p in params:
            if p.grad.data_ptr() != base + 4 * off:
                flat_ok = False
                break
            off += p.numel()
        flat_ok = flat_ok and off == G.numel()
    buf = G if flat_ok else torch.cat([p.grad.reshape(-1) for p in params])
    if _avg_supported(group):
        dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=group)
    else:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
        buf.div_(world)
    if not flat_ok:
        off = 0
        for p in params:
            k = p.numel()
            p.grad.copy_(buf[off:off + k].view_as(p.grad))
            off += k


def broadcast_parameters(module, src=0, group=None):
    """Make every rank start from rank `src`'s parameters and BN buffers."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src=src, group=group)
