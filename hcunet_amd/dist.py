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
import ctypes
import os
import weakref

import torch
import torch.distributed as dist


def _avg_supported(group=None):
    return dist.get_backend(group) == 'nccl'


def _running_stats(module, with_stats):
    """The BatchNorm running mean/var buffers reduced with the gradients: the
    Unet_Constructor's in the layout its engine reserves room for
    (bn_modules order), any other module's (RecursiveUnet, RDCNet, user
    networks: /root/reference/hcat/r_unet.py:276-277,326-327) in
    module.modules() order -- the same order on every rank."""
    if not with_stats:
        return []
    from .unet import bn_modules
    try:
        bns = bn_modules(module)
    except AttributeError:
        bns = [m for m in module.modules() if isinstance(m, torch.nn.modules.batchnorm._BatchNorm)]
    return [bn.running_mean for bn in bns if bn.running_mean is not None] + \
           [bn.running_var for bn in bns if bn.running_var is not None]


def _reduce(t, group, world):
    if _avg_supported(group):
        dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.div_(world)


def bucket_ranges(module, deep_level, n_stats):
    """Ranges of the flat gradient buffer (+ the statistics tail) reduced
    separately when the reduction overlaps the backward, in the order the
    backward finalizes them: the decoder (up_steps) + the running statistics,
    encoder levels >= deep_level, then the rest (out_conv, the shallow
    levels).  They partition [0, n_params + n_stats): one logical reduction.
    None when the parameter order is not the module layout this assumes."""
    off, up0, deep0 = 0, None, None
    seen_up = False
    for name, p in module.named_parameters():
        top = name.split('.')[0]
        if top == 'down_steps':
            if seen_up:
                return None
            if deep0 is None and int(name.split('.')[1]) >= deep_level:
                deep0 = off
        elif top == 'up_steps':
            if up0 is None:
                up0 = off
            seen_up = True
        elif seen_up:
            return None   # something registered after up_steps
        off += p.numel()
    if up0 is None or deep0 is None or not 0 < deep0 < up0:
        return None
    return [(up0, off + n_stats), (deep0, up0), (0, deep0)]


def prepare_overlap(module, deep_level=None):
    """Arm the backward of `module` (a Unet_Constructor) to record, on its
    weight-gradient stream, when the decoder's and the deep encoder levels'
    gradients are final (include/hcunet.h hcu_unet_set_grad_events), so
    allreduce_gradients reduces those ranges on a communication stream while
    the shallow levels' backward still runs.  deep_level defaults to
    levels - 2 (the two deepest levels hold most parameters).  Returns the
    bucket ranges, or None when the module does not have the U-Net layout."""
    from . import _lib
    eng = module.engine()
    levels = len(module.down_steps)
    if levels < 3:
        return None
    dl = levels - 2 if deep_level is None else int(deep_level)
    if not 1 <= dl < levels:
        raise ValueError('deep_level must be in [1, %d)' % levels)
    if bucket_ranges(module, dl, 0) is None:
        return None
    if eng.grad_events is None:
        evs = []
        for _ in range(2):
            h = ctypes.c_void_p()
            _lib.check(_lib.lib().hcu_event_create(ctypes.byref(h)), 'prepare_overlap')
            evs.append(h)
        eng.grad_events = (evs[0], evs[1], dl)
        eng._comm_stream = None
        weakref.finalize(eng, _destroy_events, evs)
    else:
        eng.grad_events = (eng.grad_events[0], eng.grad_events[1], dl)
    return bucket_ranges(module, dl, 0)


def _destroy_events(evs):
    try:
        from . import _lib
        for h in evs:
            _lib.lib().hcu_event_destroy(h)
    except Exception:
        pass


def allreduce_gradients(module, group=None, bn_stats=True):
    """Average parameter gradients (and, with bn_stats, the BatchNorm running
    mean/var) of `module` across ranks in place, as ONE logical reduction.

    Production path: every .grad is a view of the engine's flat gradient
    buffer, which is the head of engine.comm_flat; the running statistics are
    copied into its tail, the whole buffer is all-reduced and the tail is
    copied back.  After prepare_overlap (broadcast_parameters calls it) the
    buffer is reduced in three ranges on a communication stream, each waiting
    only for the backward's event that its gradients are final: the decoder's
    and the deep levels' reductions run while the shallow levels' backward is
    still executing (call this right after loss.backward(), before anything
    synchronises).  Otherwise the gradients and statistics are concatenated
    into one temporary buffer (one collective)."""
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
    ev = getattr(eng, 'grad_events', None) if eng is not None else None
    # the overlapped ranges wait only for the backward's own events: any
    # in-place gradient work queued since (a changed version counter) makes
    # this step take the single collective behind the caller's stream
    untouched = eng is not None and getattr(eng, 'grad_version', None) is not None \
        and G is not None and G._version == eng.grad_version
    if native and ev is not None and eng.events_recorded and untouched:
        ranges = bucket_ranges(module, ev[2], nstat)
        if ranges is not None and ranges[0][1] == G.numel() + nstat:
            _allreduce_overlapped(eng, C[:G.numel() + nstat], G.numel(), stats, ranges, ev, group, world)
            return
    if flat_ok:
        buf = C[:G.numel() + nstat]
        tail = buf[G.numel():]
        if native:
            _stats_move(stats, tail, unpack=False)   # one launch
        elif stats:
            torch.cat([t.reshape(-1) for t in stats], out=tail)
    else:
        F = _flat_grads(params)
        if F is not None and not stats:
            # the layer chains' models (RDCNet, RecursiveUnet without running
            # statistics, hcunet_amd.chain.FlatParams): every .grad is a view
            # of one flat buffer in parameter order -- reduced in place
            _reduce(F, group, world)
            return
        if F is not None:
            buf = torch.cat([F] + [t.reshape(-1) for t in stats])
        else:
            buf = torch.cat([p.grad.reshape(-1) for p in params] + [t.reshape(-1) for t in stats])
    _reduce(buf, group, world)
    off = G.numel() if flat_ok else 0
    if not flat_ok:
        if F is not None:
            F.copy_(buf[:F.numel()])
            off = F.numel()
        else:
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


def _flat_grads(params):
    """The gradients as ONE flat tensor when every .grad is a contiguous
    view of one storage, in parameter order without gaps (what
    hcunet_amd.chain.FlatParams attaches), else None."""
    g0 = params[0].grad
    if g0.dtype != torch.float32:
        return None
    st, base, off = g0.untyped_storage().data_ptr(), g0.data_ptr(), 0
    for p in params:
        g = p.grad
        if g.dtype != torch.float32 or not g.is_contiguous() or g.untyped_storage().data_ptr() != st \
                or g.data_ptr() != base + 4 * off:
            return None
        off += g.numel()
    return torch.empty(0, dtype=torch.float32, device=g0.device).set_(
        g0.untyped_storage(), g0.storage_offset(), (off,), (1,))


def _allreduce_overlapped(eng, buf, n_grads, stats, ranges, ev, group, world):
    """The three ranges on the engine's communication stream: each waits for
    the backward's event of its gradients (the last one for the whole
    backward), the statistics move in before the first and out after the
    last; the caller's stream then waits for the communication stream."""
    from . import _lib
    dev = buf.device
    main = torch.cuda.current_stream(dev)
    comm = getattr(eng, '_comm_stream', None)
    if comm is None or comm.device != dev:
        comm = eng._comm_stream = torch.cuda.Stream(dev)
    L = _lib.lib()
    waits = [lambda: _lib.check(L.hcu_stream_wait_event(ctypes.c_void_p(comm.cuda_stream), ev[0]),
                                'allreduce_gradients'),
             lambda: _lib.check(L.hcu_stream_wait_event(ctypes.c_void_p(comm.cuda_stream), ev[1]),
                                'allreduce_gradients'),
             lambda: comm.wait_stream(main)]
    with torch.cuda.stream(comm):
        for k, (lo, hi) in enumerate(ranges):
            waits[k]()
            if k == 0:
                _stats_move(stats, buf[n_grads:], unpack=False)
            _reduce(buf[lo:hi], group, world)
        _stats_move(stats, buf[n_grads:], unpack=True)
    main.wait_stream(comm)
    eng.events_recorded = False


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
    # the writes above go through .data (no version-counter bump): packed
    # weight images a chain kept from an earlier forward are stale now
    from .chain import invalidate_weight_images
    invalidate_weight_images()
    if os.environ.get('HCU_DP_OVERLAP', '1') != '0' and hasattr(module, 'engine') \
            and next(module.parameters()).is_cuda:
        prepare_overlap(module)
