"""Layer chains on the native executor (include/hcunet.h, hcu_chain_*).

A chain is a short sequence of Conv3d [+ BatchNorm3d + ReLU] / MaxPool3d /
ConvTranspose3d [+ cat(U, U)] ops that runs as ONE autograd node whose
forward and backward are single calls into libhcunet.so, with the network
executor's kernels and fusions (BatchNorm+ReLU applied while the consumer
stages its operand, statistics in the producer's epilogue, the BatchNorm
backward in the consumer dgrad's epilogue).  It is what calling a single
Down / Up block runs (hcat/unet.py:263-266, 309-315) and what the
r_unet.py models are built from (hcat/r_unet.py:207-378).

Parameters of the modules a chain reads are views of one flat fp32 buffer
(FlatParams), gradients are accumulated into a second one whose views are
attached as .grad (torch's accumulation semantics), so a model that calls
many chains per step (the 10-step recurrences of r_unet.py) gathers every
gradient in place.
"""
import ctypes

import torch
import torch.nn as nn

from . import _lib

CONV, POOL, CONVT = 0, 1, 2
MAX_OPS = 16
# bench.py's per-layer timing pass: each chain call tags its launches with the
# chain's name (hcu_timing_prefix) so the report tells the chains apart
TAG_CHAINS = False


class ChainOp(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int), ("out_channels", ctypes.c_int),
        ("k", _lib.c_int3), ("stride", _lib.c_int3), ("dil", _lib.c_int3), ("pad", _lib.c_int3),
        ("groups", ctypes.c_int), ("bn_relu", ctypes.c_int), ("cat_fold", ctypes.c_int),
        ("w_off", ctypes.c_int64), ("b_off", ctypes.c_int64),
        ("gamma_off", ctypes.c_int64), ("beta_off", ctypes.c_int64),
    ]


class ChainSpec(ctypes.Structure):
    _fields_ = [
        ("n_ops", ctypes.c_int), ("in_channels", ctypes.c_int),
        ("ops", ChainOp * MAX_OPS),
        ("bn_eps", ctypes.c_float), ("bn_momentum", ctypes.c_float),
        ("compute_dtype", ctypes.c_int),
        ("in_cl", ctypes.c_int), ("out_cl", ctypes.c_int), ("in_part_channels", ctypes.c_int),
    ]


def _t3(v):
    if isinstance(v, int):
        return (v, v, v)
    v = tuple(v)
    if len(v) != 3:
        raise ValueError('expected an int or a 3-tuple, got %r' % (v,))
    return v


# ---------------------------------------------------------------------------
class FlatParams:
    """The parameters of `root` as views of one flat fp32 device buffer, and a
    flat gradient buffer of the same layout (hcunet_amd.unet._Engine does the
    same for Unet_Constructor).  Parameters that are already views of one
    contiguous fp32 storage (a Unet_Constructor whose engine flattened them)
    are used in place."""

    def __init__(self, root):
        self.root = root
        self.flat = None
        self.grad = None
        self.params = None
        self.offsets = {}

    def ready(self):
        params = [p for p in self.root.parameters()]
        if self.flat is not None and len(params) == len(self.params) and all(
                p is q and p.data_ptr() == self.flat.data_ptr() + 4 * self.offsets[id(p)]
                for p, q in zip(params, self.params)):
            return self
        dev = params[0].device
        _lib.require_device(params[0], 'module parameters')
        for p in params:
            if p.dtype != torch.float32 or p.device != dev:
                raise RuntimeError('hcunet_amd: parameters must be float32 on one device')
        st = {p.untyped_storage().data_ptr() for p in params}
        if len(st) == 1 and all(p.is_contiguous() for p in params):
            # views of one buffer (e.g. the flat parameters of a Unet_Constructor)
            store = params[0].untyped_storage()
            base = torch.empty(0, dtype=torch.float32, device=dev).set_(
                store, 0, (store.nbytes() // 4,), (1,))
            self.flat = base
            self.offsets = {id(p): p.storage_offset() for p in params}
        else:
            n = sum(p.numel() for p in params)
            flat = torch.empty(n, dtype=torch.float32, device=dev)
            off = 0
            self.offsets = {}
            with torch.no_grad():
                for p in params:
                    k = p.numel()
                    flat[off:off + k].copy_(p.data.reshape(-1))
                    p.data = flat[off:off + k].view_as(p)
                    self.offsets[id(p)] = off
                    off += k
            self.flat = flat
        self.params = params
        self.grad = None
        return self

    def offset(self, p):
        return self.offsets[id(p)] if p is not None else -1

    def grad_target(self):
        """(buffer, finish): gradients accumulate into `buffer`; finish()
        attaches / adds them with torch's .grad semantics."""
        params = self.params
        n = self.flat.numel()
        if self.grad is None or self.grad.numel() != n or self.grad.device != self.flat.device:
            self.grad = torch.zeros(n, dtype=torch.float32, device=self.flat.device)
        G = self.grad
        base = G.data_ptr()

        def view(p):
            o = self.offsets[id(p)]
            return G[o:o + p.numel()].view_as(p)
        trainable = [p for p in params if p.requires_grad]
        if all(p.grad is None for p in trainable):
            G.zero_()

            def finish():
                for p in trainable:
                    p.grad = view(p)
            return G, finish
        if all(p.grad is not None and p.grad.data_ptr() == base + 4 * self.offsets[id(p)]
               for p in trainable):
            return G, (lambda: None)
        tmp = torch.zeros_like(self.flat)

        def finish_mixed():
            for p in trainable:
                o = self.offsets[id(p)]
                g = tmp[o:o + p.numel()].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.add_(g)
        return tmp, finish_mixed


# ---------------------------------------------------------------------------
class Chain:
    """One op sequence over modules of `flat.root`.  ops: list of tuples
    ('conv', nn.Conv3d, bn or None, cat_fold) / ('pool', kernel) /
    ('convt', nn.ConvTranspose3d)."""

    def __init__(self, flat, in_channels, ops, name='', in_cl=False, out_cl=False, in_part=0):
        """in_cl / out_cl: the input / output is a channels-last tensor
        [B, X, Y, Z, Cs] of the compute dtype (cl_channels(C)) instead of
        NCXYZ: consecutive chains then hand their activations over without a
        layout pass.  in_part: the input is torch.cat(..., dim=-1) of such
        tensors with in_part channels each (include/hcunet.h)."""
        if not 1 <= len(ops) <= MAX_OPS:
            raise ValueError('a chain has 1..%d ops' % MAX_OPS)
        self.name = name
        self.in_cl, self.out_cl, self.in_part = bool(in_cl), bool(out_cl), int(in_part)
        self.flat = flat
        self.in_channels = in_channels
        self.ops = ops
        self.bns = [op[2] for op in ops if op[0] == 'conv' and op[2] is not None]
        self.plans = {}
        self._bn_arrays = None

    def spec(self, bf16):
        s = ChainSpec()
        s.n_ops = len(self.ops)
        s.in_channels = self.in_channels
        f = self.flat
        eps, mom = 1e-5, 0.1
        for i, op in enumerate(self.ops):
            o = s.ops[i]
            o.stride = _lib.c_int3(1, 1, 1)
            o.dil = _lib.c_int3(1, 1, 1)
            o.pad = _lib.c_int3(0, 0, 0)
            o.groups = 1
            o.b_off = o.gamma_off = o.beta_off = -1
            if op[0] == 'conv':
                _, conv, bn, fold = op
                if isinstance(conv.padding, str) or conv.padding_mode != 'zeros':
                    raise NotImplementedError('Conv3d: only numeric zero padding')
                o.kind = CONV
                o.out_channels = conv.out_channels
                o.k = _lib.c_int3(*conv.kernel_size)
                o.stride = _lib.c_int3(*conv.stride)
                o.dil = _lib.c_int3(*conv.dilation)
                o.pad = _lib.c_int3(*conv.padding)
                o.groups = conv.groups
                o.cat_fold = 1 if fold else 0
                o.w_off = f.offset(conv.weight)
                o.b_off = f.offset(conv.bias)
                if bn is not None:
                    if not bn.affine or not bn.track_running_stats:
                        raise NotImplementedError('BatchNorm3d must be affine with running statistics')
                    o.bn_relu = 1
                    o.gamma_off = f.offset(bn.weight)
                    o.beta_off = f.offset(bn.bias)
                    eps, mom = bn.eps, bn.momentum
            elif op[0] == 'pool':
                o.kind = POOL
                o.k = _lib.c_int3(*_t3(op[1]))
            elif op[0] == 'convt':
                ct = op[1]
                if any(v != 0 for v in ct.output_padding) or ct.groups != 1 or tuple(ct.dilation) != (1, 1, 1):
                    raise NotImplementedError('ConvTranspose3d: output_padding / groups / dilation')
                o.kind = CONVT
                o.out_channels = ct.out_channels
                o.k = _lib.c_int3(*ct.kernel_size)
                o.stride = _lib.c_int3(*ct.stride)
                o.pad = _lib.c_int3(*ct.padding)
                o.w_off = f.offset(ct.weight)
                o.b_off = f.offset(ct.bias)
            else:
                raise ValueError(op[0])
        for bn in self.bns:
            if bn.eps != eps or bn.momentum != mom:
                raise NotImplementedError('BatchNorm3d layers of one chain must share eps / momentum')
        s.bn_eps = eps
        s.bn_momentum = -1.0 if mom is None else mom
        s.compute_dtype = _lib.HCU_BF16 if bf16 else _lib.HCU_F32
        s.in_cl, s.out_cl, s.in_part_channels = int(self.in_cl), int(self.out_cl), self.in_part
        return s

    def in_cs(self, bf16):
        """Channel stride of a channels-last input (the parts padded on their own)."""
        if self.in_part:
            return self.in_channels // self.in_part * cl_channels(self.in_part, bf16)
        return cl_channels(self.in_channels, bf16)

    def _offsets(self):
        mods = [m for op in self.ops for m in op[1:] if isinstance(m, nn.Module)]
        return tuple(self.flat.offset(q) for m in mods for q in m.parameters(recurse=False))

    def plan(self, shape, bf16):
        # the offsets of this chain's parameters are baked into the plan
        key = (tuple(shape), bool(bf16), self._offsets())
        p = self.plans.get(key)
        if p is None:
            if self.in_cl:
                B, X, Y, Z, C = shape
                if C != self.in_cs(bf16):
                    raise RuntimeError('expected a channels-last input with %d channel slots, got %d'
                                       % (self.in_cs(bf16), C))
            else:
                B, C, X, Y, Z = shape
                if C != self.in_channels:
                    raise RuntimeError('expected input with %d channels, got %d' % (self.in_channels, C))
            p = _ChainPlan(self.spec(bf16), B, X, Y, Z)
            self.plans[key] = p
        return p

    def bn_arrays(self):
        ptrs = [bn.running_mean.data_ptr() for bn in self.bns]
        if self._bn_arrays is None or self._bn_arrays[3] != ptrs:
            n = max(1, len(self.bns))
            rm = (ctypes.c_void_p * n)(*[bn.running_mean.data_ptr() for bn in self.bns])
            rv = (ctypes.c_void_p * n)(*[bn.running_var.data_ptr() for bn in self.bns])
            nb = (ctypes.c_void_p * n)(*[bn.num_batches_tracked.data_ptr() for bn in self.bns])
            self._bn_arrays = (rm, rv, nb, ptrs)
        return self._bn_arrays

    def __call__(self, x, training, bf16=False):
        self.flat.ready()
        params = self.flat.params
        if not isinstance(x, torch.Tensor):
            raise TypeError('expected a torch.Tensor, got %s' % type(x))
        _lib.require_device(x, 'input')
        if x.dim() != 5:
            raise RuntimeError('Expected 5D input [B, C, X, Y, Z] for conv3d, got %dD' % x.dim())
        ok = (torch.float32, torch.float16, torch.bfloat16) if bf16 else (torch.float32, torch.float16)
        if self.in_cl:
            ok = (torch.bfloat16,) if bf16 else (torch.float32,)
            if x.dtype not in ok:
                x = x.to(ok[0])
        elif x.dtype not in ok:
            x = x.float()
        return _ChainFunction.apply(x, self, bool(training), bool(bf16), *params)


# Bumped by hcunet_amd.optim.Adam (which writes the parameters through raw
# pointers, bypassing their version counters) and invalidate_weight_images().
_WEIGHT_EPOCH = [0]


def invalidate_weight_images():
    """Forces every chain to re-lay its packed weight images on its next call:
    needed after parameter writes that bypass the tensors' version counters
    (through .data or raw pointers); in-place torch ops, load_state_dict and
    hcunet_amd.optim.Adam are tracked already."""
    _WEIGHT_EPOCH[0] += 1


def _weight_key(chain):
    return (chain.flat.flat.data_ptr(), _WEIGHT_EPOCH[0]) + tuple(p._version for p in chain.flat.params)


class _ChainPlan:
    def __init__(self, spec, B, X, Y, Z):
        L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(L.hcu_chain_plan_create(ctypes.addressof(spec), B, X, Y, Z, ctypes.byref(h)), 'chain')
        self.handle = h
        out = (ctypes.c_int64 * 5)()
        nbn = ctypes.c_int()
        sv, sc = ctypes.c_size_t(), ctypes.c_size_t()
        _lib.check(L.hcu_chain_plan_query(h, out, ctypes.byref(nbn), ctypes.byref(sv), ctypes.byref(sc)))
        self.out_shape = tuple(int(v) for v in out)
        self.n_bn = int(nbn.value)
        self.saved_bytes = int(sv.value)
        self.scratch_bytes = int(sc.value)
        # packed weight images kept across calls (the last image_bytes of
        # `saved` otherwise): re-laid only when the parameters changed
        self.image_bytes = int(L.hcu_chain_weight_image_bytes(h))
        self.images = None
        self.image_key = None
        self.image_level = 0   # 1: forward images of image_key, 2: also the input-gradient ones

    def images_for(self, key, dev):
        """The image buffer and how much of it holds the images of `key`."""
        if self.images is None or self.images.device != dev:
            self.images = torch.empty(max(self.image_bytes, 16), dtype=torch.uint8, device=dev)
            self.image_key, self.image_level = None, 0
        if key != self.image_key:
            self.image_key, self.image_level = key, 0
        return self.images, self.image_level

    def __del__(self):
        try:
            if self.handle:
                _lib.lib().hcu_unet_plan_destroy(self.handle)
        except Exception:
            pass


_X_DTYPES = {torch.float32: _lib.HCU_F32, torch.float16: _lib.HCU_F16, torch.bfloat16: _lib.HCU_BF16}


def _tensors(chain, x, out, saved, scratch, grads=None):
    rm, rv, nb, _ = chain.bn_arrays()
    t = _lib.UnetTensors()
    t.x = x.data_ptr()
    t.out = out.data_ptr() if out is not None else None
    t.params = chain.flat.flat.data_ptr()
    t.grads = grads.data_ptr() if grads is not None else None
    t.bn_running_mean = ctypes.cast(rm, ctypes.POINTER(ctypes.c_void_p))
    t.bn_running_var = ctypes.cast(rv, ctypes.POINTER(ctypes.c_void_p))
    t.bn_num_batches_tracked = ctypes.cast(nb, ctypes.POINTER(ctypes.c_void_p))
    t.saved = saved.data_ptr()
    t.scratch = scratch.data_ptr()
    t.x_dtype = _X_DTYPES[x.dtype]
    return t


class _ChainFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, chain, training, bf16, *params):
        x = x.contiguous()
        plan = chain.plan(x.shape, bf16)
        dev = x.device
        if chain.out_cl:
            B, C, X, Y, Z = plan.out_shape
            out = torch.empty((B, X, Y, Z, cl_channels(C, bf16)), dtype=torch.bfloat16 if bf16 else torch.float32,
                              device=dev)
        else:
            out = torch.empty(plan.out_shape, dtype=torch.float32, device=dev)
        # the weight images live in the plan's persistent buffer (the end of
        # `saved` is not needed)
        saved = torch.empty(max(plan.saved_bytes - plan.image_bytes, 1), dtype=torch.uint8, device=dev)
        scratch = torch.empty(max(plan.scratch_bytes, 1), dtype=torch.uint8, device=dev)
        t = _tensors(chain, x, out, saved, scratch)
        L = _lib.lib()
        if TAG_CHAINS:
            L.hcu_timing_prefix(chain.name.encode())
        wkey = _weight_key(chain)
        images, level = plan.images_for(wkey, dev)
        with torch.cuda.device(dev):
            _lib.check(L.hcu_chain_forward_images(plan.handle, ctypes.byref(t), 1 if training else 0,
                                                  _lib.stream_handle(dev), ctypes.c_void_p(images.data_ptr()),
                                                  level), 'chain forward')
        plan.image_level = 2 if training else max(level, 1)
        if TAG_CHAINS:
            L.hcu_timing_prefix(b'')
        ctx.chain, ctx.plan, ctx.training, ctx.bf16 = chain, plan, training, bf16
        ctx.weight_key = wkey
        ctx.save_for_backward(x, saved)
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dout):
        x, saved = ctx.saved_tensors
        chain, plan = ctx.chain, ctx.plan
        dev = x.device
        # the backward reads the plan's weight images: they must still be the
        # ones its forward used (a later forward of the same plan after a
        # parameter change re-laid them; stock torch raises on the in-place
        # modification of a saved weight here too)
        if plan.image_key != ctx.weight_key:
            raise RuntimeError('hcunet_amd: a parameter of chain %r was modified (or another forward of '
                               'the chain ran with other weights) between its forward and its backward'
                               % chain.name)
        if chain.out_cl:   # the gradient slots' layout and precision
            dout = dout.contiguous().to(torch.bfloat16 if ctx.bf16 else torch.float32)
        else:
            dout = dout.contiguous().float()
        scratch = torch.empty(max(plan.scratch_bytes, 1), dtype=torch.uint8, device=dev)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(x.shape, dtype=x.dtype if chain.in_cl else torch.float32, device=dev)
        G, finish = chain.flat.grad_target()
        t = _tensors(chain, x, None, saved, scratch, grads=G)
        L = _lib.lib()
        if TAG_CHAINS:
            L.hcu_timing_prefix(chain.name.encode())
        with torch.cuda.device(dev):
            _lib.check(L.hcu_chain_backward_images(plan.handle, ctypes.byref(t),
                                                   ctypes.c_void_p(dout.data_ptr()), _lib.ptr(dx),
                                                   1 if ctx.training else 0, 1, _lib.stream_handle(dev),
                                                   ctypes.c_void_p(plan.images.data_ptr()), plan.image_level),
                       'chain backward')
        plan.image_level = 2
        if TAG_CHAINS:
            L.hcu_timing_prefix(b'')
        finish()
        if dx is not None and dx.dtype != x.dtype:
            dx = dx.to(x.dtype)
        return (dx, None, None, None) + (None,) * len(chain.flat.params)


def cl_channels(c, bf16):
    """Channel slots of a channels-last chain tensor: c rounded up to the
    16-byte vector (8 bf16 / 4 fp32 channels), padding zero."""
    v = 8 if bf16 else 4
    return (c + v - 1) // v * v


def flat_of(module, root=None):
    """The FlatParams of `root` (default: module), created on first use and
    kept on the root module."""
    root = root if root is not None else module
    f = root.__dict__.get('_hcu_flat')
    if f is None:
        f = FlatParams(root)
        root.__dict__['_hcu_flat'] = f
    return f


def bf16_active(module=None):
    cd = getattr(module, 'compute_dtype', None) if module is not None else None
    if cd is not None:
        return cd == torch.bfloat16
    return bool(torch.is_autocast_enabled('cuda') and torch.get_autocast_dtype('cuda') == torch.bfloat16)


def upsample_cat_check(u_shape, skip):
    """hcat/unet.py:311-312 / r_unet.py:332-333: crop(U, skip) returns U sliced
    to the skip's extent; cat((U, crop)) needs equal extents, i.e. U no larger
    than the skip in every spatial dim (then the cat is cat(U, U))."""
    if skip.shape[1] != u_shape[1]:
        raise AssertionError('Inputs do not have same number of feature dimmensions: %s | %s'
                             % (list(u_shape), list(skip.shape)))
    if any(u_shape[d] > skip.shape[d] for d in (2, 3, 4)):
        raise RuntimeError('Sizes of tensors must match except in dimension 1. Expected size %d but got '
                           'size %d for tensor number 1 in the list.'
                           % (u_shape[2], min(u_shape[2], skip.shape[2])))


def is_module(m):
    return isinstance(m, nn.Module)
