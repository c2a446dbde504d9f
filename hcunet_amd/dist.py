"""Data-parallel training over RCCL: batch sharded across ranks (one process
per GPU), ONE all-reduce per step of one flat buffer holding the parameter
gradients followed by the BatchNorm running statistics.

The reference has no distributed code; this is the one collective
the build adds.  BatchNorm batch statistics stay per-rank (no SyncBN), as a
per-rank reference run computes them; the running mean/var buffers are
averaged in the same collective so that every rank holds the same model (and a
checkpoint saved by rank 0 is the job's model).  num_batches_tracked is equal
on every rank by construction and is not reduced.
"""
import os

import torch
import torch.distributed as dist


def _avg_supported(group=None):
    return dist.get_backend(group) == 'nccl'


def _running_stats(module, with_stats):
    if not with_stats:
        return []
    from .unet import bn_modules
    try:
        bns = bn_modules(module)
    except AttributeError:   # not a Unet_Constructor: reduce gradients only
        return []
    return [bn.running_mean for bn in bns if bn.running_mean is not None] + \
           [bn.running_var for bn in bns if bn.running_var is not None]


def allreduce_gradients(module, group=None, bn_stats=True):
    """Average parameter gradients (and, with bn_stats, the BatchNorm running
    mean/var) of `module` across ranks in place, in ONE collective.

    Production path: every .grad is a view of the engine's flat gradient
    buffer, which is the head of engine.comm_flat; the running statistics are
    copied into its tail, the whole buffer is all-reduced once and the tail is
    copied back.  Otherwise the gradients and statistics are concatenated into
    one temporary buffer (same single collective)."""
    if not dist.is_available() or not dist.is_initialized():
        return
    world = dist.get_world_size(group)
    if world == 1:
        return
    params = [p for p in module.parameters() if p.grad is not None]
    stats = _running_stats(module, bn_stats)
    if not params and not stats:
        return
    eng = getattr(module, '_engine', None)
    G = getattr(eng, 'grad_flat', None) if eng is not None else None
    C = getattr(eng, 'comm_flat', None) if eng is not None else None
    nstat = sum(t.numel() for t in stats)
    flat_ok = False
    if G is not None and C is not None and params and len(params) == len(list(module.parameters())):
        base, off, flat_ok = G.data_ptr(), 0, True
        for p in params:
            if p.grad.data_ptr() != base + 4 * off:
                flat_ok = False
                break
            off += p.numel()
        flat_ok = flat_ok and off == G.numel() and C.data_ptr() == base \
            and C.numel() >= G.numel() + nstat
    native = flat_ok and C.is_cuda and 0 < len(stats) <= 128 and all(t.is_contiguous() for t in stats)
    if flat_ok:
        buf = C[:G.numel() + nstat]
        tail = buf[G.numel():]
        if native:
            _stats_move(stats, tail, unpack=False)   # one launch
        elif stats:
            torch.cat([t.reshape(-1) for t in stats], out=tail)
    else:
        buf = torch.cat([p.grad.reshape(-1) for p in params] + [t.reshape(-1) for t in stats])
    if _avg_supported(group):
        dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=group)
    else:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
        buf.div_(world)
    off = G.numel() if flat_ok else 0
    if not flat_ok:
        for p in params:
            k = p.numel()
            p.grad.copy_(buf[off:off + k].view_as(p.grad))
            off += k
    if native:
        _stats_move(stats, buf[off:], unpack=True)   # one launch
        return
    for t in stats:
        k = t.numel()
        t.copy_(buf[off:off + k].view_as(t))
        off += k


def _stats_move(stats, buf, unpack):
    """The running statistics into (unpack=False) / out of the communication
    buffer's tail in ONE launch (hcu_gather_vectors)."""
    import ctypes
    from . import _lib
    n = len(stats)
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in stats])
    lens = (ctypes.c_int * n)(*[t.numel() for t in stats])
    _lib.check(_lib.lib().hcu_gather_vectors(ptrs, lens, n, ctypes.c_void_p(buf.data_ptr()),
                                             1 if unpack else 0, _lib.stream_handle(buf.device)),
               'allreduce_gradients')


def deterministic_tiling():
    """Every rank must run the same convolution tilings (the same summation
    order): plan from the persistent tiling table, the cost model on a miss,
    never from per-process timing (include/hcunet.h, hcu_tuning_set_mode)."""
    from . import _lib
    if os.path.exists(_lib.LIB_PATH) and _lib.tuning_mode() == _lib.TUNE_TIMED:
        _lib.tuning_mode(_lib.TUNE_TABLE)


def broadcast_parameters(module, src=0, group=None):
    """Make every rank start from rank `src`'s parameters and BN buffers (and
    plan deterministic tilings, see deterministic_tiling)."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    deterministic_tiling()
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src=src, group=group)
