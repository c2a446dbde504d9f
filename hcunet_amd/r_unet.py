"""Drop-in hcat.r_unet (RecursiveUnet, RDCNet, f, Down, Up, StackedDilation,
RDCBlock, crop) whose arithmetic runs in libhcunet.so.

Interface parity with the reference (hcat/r_unet.py):
  * constructor signatures, module tree and registration order (so
    state_dict keys and torch's seeded default initialisation match
    key-for-key and bit-for-bit), save / load (:164-204);
  * forward semantics, including the 10-step recurrences (:135-162,
    :219-227), the hard-coded 5-channel / batch-1 state of RecursiveUnet
    (:141) and the ReLU'd, cat(U, U) decoder blocks (:330-336).

Compute: every Conv3d [+ BatchNorm3d + ReLU] / MaxPool3d / ConvTranspose3d
sequence between two recurrence points is ONE layer chain
(hcunet_amd.chain, hcu_chain_* in include/hcunet.h); the gated update of
RecursiveUnet is a native kernel (hcu_gate_fwd / hcu_gate_bwd).  What is
left in torch is RecursiveUnet's channel cat of the input and the state;
RDCNet's recurrence glue is native: the channel cats (cl_cat, hcu_cl_cat),
the residual add with its bf16 cast (resid_add, hcu_resid_fwd / _bwd) and
the gradient sums of the tensors read by several chains (fan,
hcu_sum_parts).  StackedDilation's dilated
5^3 convolutions whose halo does not fit a workgroup run on their dilation
sub-lattices (space-to-batch, hcunet_amd/csrc/layout.hip).  Under
torch.autocast('cuda', torch.bfloat16) (or compute_dtype = torch.bfloat16)
the chains run on the bf16 path, RDCNet's last ConvTranspose3d included
(its 5 output channels padded to 8 columns per stride phase).
"""
import ctypes
import glob

import torch
import torch.nn as nn

from . import _lib
from . import chain as _chain_mod
from .chain import Chain, bf16_active, cl_channels, flat_of, upsample_cat_check


def crop(x, y):
    """hcat/r_unet.py:14-35: x sliced to y's spatial extent (views only)."""
    assert x.shape[1] == y.shape[1], \
        f'Inputs do not have same number of feature dimmensions: {x.shape} | {y.shape}'
    if x.dim() == 4:
        return x[:, :, 0:y.shape[2]:1, 0:y.shape[3]:1]
    if x.dim() == 5:
        return x[:, :, 0:y.shape[2]:1, 0:y.shape[3]:1, 0:y.shape[4]:1]
    return torch.empty(0)


def _chain(owner, root, name, in_channels, ops, **cl):
    """The chain `name` of `owner` over the flat parameters of `root` (cl:
    Chain's channels-last boundary options)."""
    cache = owner.__dict__.setdefault('_hcu_chains', {})
    key = (id(root), name)
    ch = cache.get(key)
    if ch is None or ch.flat.root is not root:
        ch = Chain(flat_of(root), in_channels, ops, '%s.%s' % (type(owner).__name__, name), **cl)
        cache[key] = ch
    return ch


def _t3(v):
    return (v, v, v) if isinstance(v, int) else tuple(v)


def _pool_k(mp):
    k = _t3(mp.kernel_size)
    s = _t3(mp.stride if mp.stride is not None else mp.kernel_size)
    if s != k or _t3(mp.padding) != (0, 0, 0) or _t3(mp.dilation) != (1, 1, 1) or mp.ceil_mode:
        raise NotImplementedError('MaxPool3d must be kernel == stride, no padding, floor mode')
    return k


def _convt_out(ct, shape):
    k, s, p = _t3(ct.kernel_size), _t3(ct.stride), _t3(ct.padding)
    return [shape[0], ct.out_channels] + [(shape[2 + d] - 1) * s[d] - 2 * p[d] + k[d] for d in range(3)]


def _conv_out(cv, shape):
    k, s, p, d = _t3(cv.kernel_size), _t3(cv.stride), _t3(cv.padding), _t3(cv.dilation)
    return [shape[0], cv.out_channels] + [(shape[2 + i] + 2 * p[i] - d[i] * (k[i] - 1) - 1) // s[i] + 1
                                          for i in range(3)]


# ---------------------------------------------------------------------------
class _Gate(torch.autograd.Function):
    """h_t = h_prev * sigmoid(zp) + (-1 * sigmoid(zp) * tanh(hp)), h_prev None:
    ones (hcat/r_unet.py:150-155)."""

    @staticmethod
    def forward(ctx, hp, zp, hprev):
        hp, zp = hp.contiguous(), zp.contiguous()
        if hprev is not None:
            hprev = hprev.contiguous()
            if hprev.shape != hp.shape:
                raise RuntimeError('The size of tensor a (%s) must match the size of tensor b (%s)'
                                   % (list(hprev.shape), list(hp.shape)))
        if zp.shape != hp.shape:
            raise RuntimeError('The size of tensor a (%s) must match the size of tensor b (%s)'
                               % (list(zp.shape), list(hp.shape)))
        out = torch.empty_like(hp)
        _lib.check(_lib.lib().hcu_gate_fwd(_lib.ptr(hp), _lib.ptr(zp), _lib.ptr(hprev), _lib.ptr(out),
                                           hp.numel(), _lib.stream_handle(hp.device)), 'gate')
        ctx.has_prev = hprev is not None
        ctx.save_for_backward(hp, zp, hprev if hprev is not None else hp)
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dout):
        hp, zp, hprev = ctx.saved_tensors
        if not ctx.has_prev:
            hprev = None
        dout = dout.contiguous().float()
        dhp, dzp = torch.empty_like(hp), torch.empty_like(zp)
        dprev = torch.empty_like(hp) if (hprev is not None and ctx.needs_input_grad[2]) else None
        _lib.check(_lib.lib().hcu_gate_bwd(_lib.ptr(hp), _lib.ptr(zp), _lib.ptr(hprev), _lib.ptr(dout),
                                           _lib.ptr(dhp), _lib.ptr(dzp), _lib.ptr(dprev), hp.numel(),
                                           _lib.stream_handle(hp.device)), 'gate backward')
        return dhp, dzp, dprev


def _cl_cat_call(parts, full, split):
    n = len(parts)
    ptrs = (ctypes.c_void_p * n)(*[p.data_ptr() for p in parts])
    rb = (ctypes.c_int * n)(*[p.shape[-1] * p.element_size() for p in parts])
    _lib.check(_lib.lib().hcu_cl_cat(ptrs, rb, n, ctypes.c_void_p(full.data_ptr()), full.numel() // full.shape[-1],
                                     split, _lib.stream_handle(full.device)), 'channel cat')


class _ClCat(torch.autograd.Function):
    """torch.cat(parts, dim=-1) of channels-last chain tensors (hcat/r_unet.py
    :223, :362 in the executor's layout) in one launch; the backward hands
    each part its gradient as a contiguous tensor, again in one launch
    (hcu_cl_cat), instead of strided slices that every consumer copies."""

    @staticmethod
    def forward(ctx, *parts):
        parts = [p.contiguous() for p in parts]
        lead = parts[0].shape[:-1]
        widths = [p.shape[-1] for p in parts]
        out = torch.empty(tuple(lead) + (sum(widths),), dtype=parts[0].dtype, device=parts[0].device)
        _cl_cat_call(parts, out, 0)
        ctx.lead, ctx.widths = tuple(lead), widths
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        g = g.contiguous()
        grads = [torch.empty(ctx.lead + (w,), dtype=g.dtype, device=g.device) for w in ctx.widths]
        _cl_cat_call(grads, g, 1)
        return tuple(grads)


def cl_cat(parts):
    """Channel cat of channels-last tensors with 16-byte channel rows (what
    the chains produce); other inputs go to torch.cat."""
    p0 = parts[0]
    ok = 1 <= len(parts) <= 8 and all(
        p.is_cuda and p.device == p0.device and p.dtype == p0.dtype and p.dim() == p0.dim()
        and p.shape[:-1] == p0.shape[:-1]
        and (p.shape[-1] * p.element_size()) % 16 == 0 for p in parts)
    return _ClCat.apply(*parts) if ok else torch.cat(parts, dim=-1)


class _Resid(torch.autograd.Function):
    """y' = m + y with m the block output in bf16 and y the fp32 residual
    state (hcat/r_unet.py:223-225 under autocast: the sum promotes to fp32),
    returned with its bf16 cast (what the next step's cat and the last conv
    take), in one launch each way (hcu_resid_fwd / hcu_resid_bwd)."""

    @staticmethod
    def forward(ctx, m, y):
        m, y = m.contiguous(), y.contiguous()
        out = torch.empty(y.shape, dtype=torch.float32, device=y.device)
        outc = torch.empty(y.shape, dtype=m.dtype, device=y.device)
        _lib.check(_lib.lib().hcu_resid_fwd(_lib.ptr(m), _lib.ptr(y), _lib.ptr(out), _lib.ptr(outc), y.numel(),
                                            _lib.stream_handle(y.device)), 'residual add')
        ctx.set_materialize_grads(False)
        return out, outc

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g32, gc):
        if g32 is None and gc is None:
            return None, None
        ref = g32 if g32 is not None else gc
        g32 = g32.contiguous().float() if g32 is not None else None
        gc = gc.contiguous().to(torch.bfloat16) if gc is not None else None
        dy = torch.empty(ref.shape, dtype=torch.float32, device=ref.device)
        dm = torch.empty(ref.shape, dtype=torch.bfloat16, device=ref.device)
        _lib.check(_lib.lib().hcu_resid_bwd(_lib.ptr(g32), _lib.ptr(gc), _lib.ptr(dy), _lib.ptr(dm), dy.numel(),
                                            _lib.stream_handle(dy.device)), 'residual add backward')
        return dm, dy


class _PwConv(torch.autograd.Function):
    """cat(parts, -1) -> 1x1x1 Conv3d (no BatchNorm) on bf16 channels-last
    channel parts, without the cat (hcat/r_unet.py:223 cat(x, y) ->
    RDCBlock.conv, :362 the dilated branches' cat -> StackedDilation.out_conv):
    hcu_pw_conv_forward / _backward read and write the parts where they are.
    The weight and bias gradients accumulate into the flat gradient buffer the
    layer chains of the same root use (FlatParams.grad_target)."""

    @staticmethod
    def forward(ctx, conv, flat, part_c, weight, *parts):
        parts = [p.contiguous() for p in parts]
        p0 = parts[0]
        nvox = p0.numel() // p0.shape[-1]
        cout = conv.out_channels
        ocs = cl_channels(cout, True)
        out = torch.empty(tuple(p0.shape[:-1]) + (ocs,), dtype=torch.bfloat16, device=p0.device)
        ptrs = (ctypes.c_void_p * len(parts))(*[p.data_ptr() for p in parts])
        _lib.check(_lib.lib().hcu_pw_conv_forward(ptrs, len(parts), part_c, p0.shape[-1], _lib.ptr(conv.weight),
                                                  _lib.ptr(conv.bias), _lib.ptr(out), nvox, cout, ocs,
                                                  _lib.stream_handle(p0.device)), '1x1x1 convolution')
        ctx.conv, ctx.flat, ctx.part_c = conv, flat, part_c
        ctx.key = _pw_key(conv)
        ctx.save_for_backward(*parts)
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dout):
        parts = ctx.saved_tensors
        conv, flat = ctx.conv, ctx.flat
        if _pw_key(conv) != ctx.key:
            raise RuntimeError('hcunet_amd: a parameter of %r was modified between its forward and its '
                               'backward' % conv)
        p0 = parts[0]
        dev = p0.device
        dout = dout.contiguous().to(torch.bfloat16)
        nvox = p0.numel() // p0.shape[-1]
        cout = conv.out_channels
        ocs = dout.shape[-1]
        L = _lib.lib()
        need = any(ctx.needs_input_grad[4:])
        dparts = [torch.empty_like(p) for p in parts] if need else None
        G, finish = flat.grad_target()
        base = G.data_ptr()
        dw = ctypes.c_void_p(base + 4 * flat.offset(conv.weight))
        db = ctypes.c_void_p(base + 4 * flat.offset(conv.bias)) if conv.bias is not None else ctypes.c_void_p()
        nw = int(L.hcu_pw_conv_work_floats(nvox, len(parts), p0.shape[-1], cout))
        work = torch.empty(max(nw, 1), dtype=torch.float32, device=dev)
        ptrs = (ctypes.c_void_p * len(parts))(*[p.data_ptr() for p in parts])
        dptrs = (ctypes.c_void_p * len(parts))(*[d.data_ptr() for d in dparts]) if need else None
        _lib.check(L.hcu_pw_conv_backward(ptrs, len(parts), ctx.part_c, p0.shape[-1], _lib.ptr(conv.weight),
                                          ctypes.c_void_p(dout.data_ptr()), cout, ocs, dptrs, dw, db, nvox,
                                          ctypes.c_void_p(work.data_ptr()), nw, 1, _lib.stream_handle(dev)),
                   '1x1x1 convolution backward')
        finish()
        return (None, None, None, None) + (tuple(dparts) if need else (None,) * len(parts))


def _pw_key(conv):
    return (_chain_mod._WEIGHT_EPOCH[0], conv.weight._version,
            conv.bias._version if conv.bias is not None else -1)


def pw_conv(conv, root, part_c, parts):
    """The cat of channels-last bf16 parts [..., cl_channels(part_c)] followed
    by the bias-carrying 1x1x1 `conv` of module tree `root`, as one native op
    (_PwConv); None when the shapes are not the ones it takes (the caller then
    runs cl_cat + the layer chain)."""
    p0 = parts[0]
    pcs = cl_channels(part_c, True)
    k = conv.kernel_size if isinstance(conv.kernel_size, tuple) else (conv.kernel_size,) * 3
    if (not p0.is_cuda or p0.dtype != torch.bfloat16 or tuple(k) != (1, 1, 1) or conv.groups != 1
            or tuple(conv.stride) != (1, 1, 1) or tuple(conv.padding) != (0, 0, 0)
            or conv.in_channels != part_c * len(parts) or not 1 <= len(parts) <= 8
            or any(p.dtype != torch.bfloat16 or p.shape != p0.shape or p.device != p0.device for p in parts)
            or p0.shape[-1] != pcs or len(parts) * pcs > 96 or cl_channels(conv.out_channels, True) > 32):
        return None
    flat = flat_of(root).ready()
    return _PwConv.apply(conv, flat, part_c, conv.weight, *parts)


def resid_add(m, y):
    """(m + y, (m + y).to(m.dtype)) for the bf16 block output m and the fp32
    state y of RDCNet's recurrence; other dtypes go to torch."""
    if m.dtype == torch.bfloat16 and y.dtype == torch.float32 and m.shape == y.shape and m.is_cuda \
            and y.is_cuda and m.numel() % 8 == 0:
        return _Resid.apply(m, y)
    s = m + y
    return s, s.to(m.dtype)


class _Fan(torch.autograd.Function):
    """One tensor handed to k consumers (k views); the backward sums their
    gradients in one launch (hcu_sum_parts: fp32 accumulation in consumer
    order, one rounding) instead of autograd's k - 1 pairwise adds."""

    @staticmethod
    def forward(ctx, t, k):
        ctx.set_materialize_grads(False)
        return tuple(t.view_as(t) for _ in range(k))

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, *gs):
        live = [g for g in gs if g is not None]
        if len(live) <= 1:
            return (live[0] if live else None), None
        ref = live[0]
        if ref.dtype not in (torch.bfloat16, torch.float32) or any(g.dtype != ref.dtype for g in live):
            return sum(live[1:], live[0]), None
        gs = [g.contiguous() if g is not None else None for g in gs]
        out = torch.empty(ref.shape, dtype=ref.dtype, device=ref.device)
        ptrs = (ctypes.c_void_p * len(gs))(*[g.data_ptr() if g is not None else None for g in gs])
        _lib.check(_lib.lib().hcu_sum_parts(ptrs, len(gs), _lib.ptr(out), out.numel(),
                                            1 if ref.dtype == torch.bfloat16 else 0,
                                            _lib.stream_handle(out.device)), 'gradient sum')
        return out, None


def fan(t, k):
    """k uses of t whose gradients are summed in one launch (_Fan); plain
    repetition where no gradient flows or the shape does not fit."""
    if k < 2 or k > 16 or not (torch.is_grad_enabled() and t.requires_grad and t.is_cuda) \
            or t.dtype not in (torch.bfloat16, torch.float32) or t.numel() % 8:
        return (t,) * k
    return _Fan.apply(t, k)


def _ready(x, what):
    if not isinstance(x, torch.Tensor):
        raise TypeError('%s must be a torch.Tensor, got %s' % (what, type(x)))
    _lib.require_device(x, what)


# ---------------------------------------------------------------------------
class Down(nn.Module):
    """hcat/r_unet.py:249-283: conv1 (padding) -> BN -> ReLU -> conv2
    (padding 1) -> BN -> ReLU."""

    def __init__(self, in_channels: int, out_channels: int, kernel: dict, dilation: dict, groups: dict,
                 padding=None):
        super().__init__()
        if padding is None:
            padding = 0
        self.conv1 = nn.Conv3d(in_channels, out_channels, kernel['conv1'], dilation=dilation['conv1'],
                               groups=groups['conv1'], padding=padding)
        self.conv2 = nn.Conv3d(out_channels, out_channels, kernel['conv2'], dilation=dilation['conv2'],
                               groups=groups['conv2'], padding=1)
        self.batch1 = nn.BatchNorm3d(out_channels)
        self.batch2 = nn.BatchNorm3d(out_channels)
        self.relu = nn.ReLU(inplace=True)

    def _ops(self):
        return [('conv', self.conv1, self.batch1, False), ('conv', self.conv2, self.batch2, False)]

    def out_shape(self, shape):
        return _conv_out(self.conv2, _conv_out(self.conv1, shape))

    def forward(self, x):
        _ready(x, 'Down input')
        return _chain(self, self, 'down', self.conv1.in_channels, self._ops())(
            x, self.training, bf16_active())


class Up(nn.Module):
    """hcat/r_unet.py:286-336: up_conv (ConvTranspose3d, padding_up) ->
    cat(U, crop(U, y)) -> conv1 -> BN -> ReLU -> conv2 -> BN -> ReLU."""

    def __init__(self, in_channels: int, out_channels: int, kernel: tuple, upsample_kernel: tuple,
                 upsample_stride: int, dilation: dict, groups: dict, padding_down=None, padding_up=None):
        super().__init__()
        if padding_down is None:
            padding_down = 0
        if padding_up is None:
            padding_up = 0
        self.conv1 = nn.Conv3d(in_channels, out_channels, kernel['conv1'], dilation=dilation['conv1'],
                               groups=groups['conv1'], padding=padding_down)
        self.conv2 = nn.Conv3d(out_channels, out_channels, kernel['conv2'], dilation=dilation['conv2'],
                               groups=groups['conv2'], padding=padding_down)
        self.up_conv = nn.ConvTranspose3d(in_channels, out_channels, upsample_kernel, stride=upsample_stride,
                                          padding=padding_up)
        self.lin_up = False
        self.batch1 = nn.BatchNorm3d(out_channels)
        self.batch2 = nn.BatchNorm3d(out_channels)
        self.relu = nn.ReLU(inplace=True)

    def _ops(self):
        return [('convt', self.up_conv), ('conv', self.conv1, self.batch1, True),
                ('conv', self.conv2, self.batch2, False)]

    def check_skip(self, shape, skip_shape):
        u = _convt_out(self.up_conv, shape)
        upsample_cat_check(u, torch.empty(skip_shape, device='meta'))
        return u

    def forward(self, x, y):
        _ready(x, 'Up input')
        self.check_skip(list(x.shape), list(y.shape))
        return _chain(self, self, 'up', self.up_conv.in_channels, self._ops())(
            x, self.training, bf16_active())


class f(nn.Module):
    """hcat/r_unet.py:232-246: down1 -> max_pool -> down2 -> up1(x, b)."""

    def __init__(self, down1, down2, up1, max_pool):
        super().__init__()
        self.down1 = down1
        self.down2 = down2
        self.up1 = up1
        self.max_pool = max_pool

    def _ops(self):
        return (self.down1._ops() + [('pool', _pool_k(self.max_pool))] + self.down2._ops()
                + self.up1._ops())

    def _run(self, x, root, training, bf16):
        b = self.down1.out_shape(list(x.shape))
        p = [b[0], b[1]] + [b[2 + d] // _pool_k(self.max_pool)[d] for d in range(3)]
        self.up1.check_skip(self.down2.out_shape(p), b)
        return _chain(self, root, 'f', self.down1.conv1.in_channels, self._ops())(x, training, bf16)

    def forward(self, x):
        _ready(x, 'f input')
        return self._run(x, self, self.training, bf16_active())


class RecursiveUnet(nn.Module):
    """hcat/r_unet.py:38-204."""

    def __init__(self,
                 image_dimensions=2,
                 in_channels=4,
                 out_channels=5,
                 kernel={'conv1': (3, 3, 3), 'conv2': (3, 3, 3)},
                 upsample_kernel=(6, 6, 5),
                 max_pool_kernel=(2, 2, 1),
                 upsample_stride=(2, 2, 1),
                 dilation=1,
                 groups=1,
                 ):
        super().__init__()
        if type(kernel) is tuple:
            kernel = {'conv1': kernel, 'conv2': kernel}
        if type(dilation) is int or type(dilation) is tuple:
            dilation = {'conv1': dilation, 'conv2': dilation}
        if type(groups) is int or type(groups) is tuple:
            groups = {'conv1': groups, 'conv2': groups}
        self.model_specification = {
            'image_dimensions': image_dimensions,
            'in_channels': in_channels,
            'out_channels': out_channels,
            'kernel': kernel,
            'upsample_kernel': upsample_kernel,
            'max_pool_kernel': max_pool_kernel,
            'upsample_stride': upsample_stride,
            'dilation': dilation,
            'groups': groups
        }
        channels = [16, 32, 64]
        # creation order = the reference's RNG stream (:105-127)
        self.down1 = Down(in_channels=9, out_channels=channels[0], kernel=kernel, dilation=dilation,
                          groups=groups, padding=1)
        self.down2_fz = Down(in_channels=channels[0], out_channels=channels[1], kernel=kernel,
                             dilation=dilation, groups=groups, padding=1)
        self.down3_fz = Down(in_channels=channels[1], out_channels=channels[2], kernel=kernel,
                             dilation=dilation, groups=groups, padding=1)
        self.up1_fz = Up(in_channels=channels[2], out_channels=channels[1], kernel=kernel, dilation=dilation,
                         groups=groups, upsample_kernel=upsample_kernel, upsample_stride=upsample_stride,
                         padding_down=1, padding_up=2)
        self.down2_fh = Down(in_channels=channels[0], out_channels=channels[1], kernel=kernel,
                             dilation=dilation, groups=groups, padding=1)
        self.down3_fh = Down(in_channels=channels[1], out_channels=channels[2], kernel=kernel,
                             dilation=dilation, groups=groups, padding=1)
        self.up1_fh = Up(in_channels=channels[2], out_channels=channels[1], kernel=kernel, dilation=dilation,
                         groups=groups, upsample_kernel=upsample_kernel, upsample_stride=upsample_stride,
                         padding_down=1, padding_up=2)
        self.up2 = Up(in_channels=channels[1], out_channels=channels[0], kernel=kernel, dilation=dilation,
                      groups=groups, upsample_kernel=upsample_kernel, upsample_stride=upsample_stride,
                      padding_down=1, padding_up=2)
        self.out_conv = nn.Conv3d(channels[0], out_channels, 1)
        self.tanh = nn.Tanh()
        self.sigmoid = nn.Sigmoid()
        self.max_pool = nn.MaxPool3d(max_pool_kernel)
        self.fz = f(self.down2_fz, self.down3_fz, self.up1_fz, self.max_pool)
        self.fh = f(self.down2_fh, self.down3_fh, self.up1_fh, self.max_pool)
        # None: follow torch.autocast; torch.float32 / torch.bfloat16: force
        self.compute_dtype = None

    def forward(self, image):
        _ready(image, 'RecursiveUnet input')
        bf16 = bf16_active(self)
        tr = self.training
        mp = _pool_k(self.max_pool)
        c_down1 = _chain(self, self, 'down1', 9, self.down1._ops() + [('pool', mp)])
        c_up2 = _chain(self, self, 'up2', self.up2.up_conv.in_channels,
                       self.up2._ops() + [('conv', self.out_conv, None, False)])
        x = None
        for t in range(10):
            if t == 0:
                s_t = torch.zeros([1, 5, image.shape[2], image.shape[3], image.shape[4]],
                                  device=image.device)
            x = torch.cat((image, s_t), dim=1)
            a = self.down1.out_shape(list(x.shape))           # a = down1(x) (its shape only is used)
            x = c_down1(x, tr, bf16)                           # max_pool(down1(x))
            hp = self.fh._run(x, self, tr, bf16)
            zp = self.fz._run(x, self, tr, bf16)
            h_t = _Gate.apply(hp, zp, None if t == 0 else h_t)
            self.up2.check_skip(list(h_t.shape), a)
            x = c_up2(h_t, tr, bf16)                           # out_conv(up2(h_t, a))
            s_t = x
        return x

    def save(self, filename, hyperparameters=None):
        model = {'state_dict': self.state_dict(),
                 'model_specifications': self.model_specification,
                 'hyperparameters': hyperparameters}
        python_files = {}
        files = glob.glob('./**/*.py', recursive=True) + glob.glob('./**/*.ipynb', recursive=True)
        for fn in files:
            with open(fn, 'r') as fh:
                python_files[fn] = fh.read()
        model['python_files'] = python_files
        model['tree_structure'] = glob.glob('**/*', recursive=True)
        torch.save(model, filename)
        return None

    def load(self, filename, to_cuda=True):
        device = 'cuda:0' if (torch.cuda.is_available() and to_cuda) else 'cpu'
        model = torch.load(filename, map_location=device, weights_only=True)
        self.__init__()          # the reference re-initialises with the defaults (:197)
        self.load_state_dict(model['state_dict'])
        self.eval()
        try:
            return model['hyperparameters']
        except KeyError:
            return None


# ---------------------------------------------------------------------------
class StackedDilation(nn.Module):
    """hcat/r_unet.py:339-364: five 'same' Conv3d at dilation 1..5, cat, 1x1."""

    def __init__(self, in_channels: int, out_channels: int, kernel: tuple):
        super().__init__()
        self.conv1 = nn.Conv3d(in_channels, out_channels, kernel_size=kernel, dilation=1, padding=2)
        self.conv2 = nn.Conv3d(in_channels, out_channels, kernel_size=kernel, dilation=2, padding=4)
        self.conv3 = nn.Conv3d(in_channels, out_channels, kernel_size=kernel, dilation=3, padding=6)
        self.conv4 = nn.Conv3d(in_channels, out_channels, kernel_size=kernel, dilation=4, padding=8)
        self.conv5 = nn.Conv3d(in_channels, out_channels, kernel_size=kernel, dilation=5, padding=10)
        self.out_conv = nn.Conv3d(out_channels * 5, out_channels, kernel_size=1, padding=0)

    def _run(self, x, root, bf16, tr):
        # tr: training flag of the call -- no BatchNorm here; a training call
        # also lays out the input-gradient weight images during the forward
        cin = self.conv1.in_channels
        xs = [_chain(self, root, 'd%d' % i, cin, [('conv', c, None, False)])(x, tr, bf16)
              for i, c in enumerate((self.conv1, self.conv2, self.conv3, self.conv4, self.conv5))]
        out = torch.cat(xs, dim=1)
        return _chain(self, root, 'out', self.out_conv.in_channels, [('conv', self.out_conv, None, False)])(
            out, tr, bf16)

    def forward(self, x):
        _ready(x, 'StackedDilation input')
        return self._run(x, self, bf16_active(), self.training)


class RDCBlock(nn.Module):
    """hcat/r_unet.py:367-378: 1x1 Conv3d (2C -> C) then StackedDilation."""

    def __init__(self, in_channels):
        super().__init__()
        self.conv = nn.Conv3d(in_channels * 2, in_channels, kernel_size=1)
        self.grouped_conv = StackedDilation(in_channels, in_channels, 5)

    def _run(self, x, root, bf16, tr):
        x = _chain(self, root, 'conv', self.conv.in_channels, [('conv', self.conv, None, False)])(
            x, tr, bf16)
        return self.grouped_conv._run(x, root, bf16, tr)

    def forward(self, x):
        _ready(x, 'RDCBlock input')
        return self._run(x, self, bf16_active(), self.training)


class RDCNet(nn.Module):
    """hcat/r_unet.py:207-227: strided Conv3d, ten RDCBlock steps on
    cat(x, y) with a residual state, Conv3d, padded ConvTranspose3d."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        complexity = 10
        self.strided_conv = nn.Conv3d(in_channels, complexity, kernel_size=3, stride=2, padding=1)
        self.RDCblock = RDCBlock(complexity)
        self.out_conv = nn.Conv3d(complexity, out_channels=complexity, kernel_size=3, padding=1)
        self.transposed_conv = nn.ConvTranspose3d(in_channels=complexity, out_channels=out_channels,
                                                  stride=(2, 2, 2), kernel_size=(4, 4, 4), padding=(1, 1, 1))
        self.compute_dtype = None

    def forward(self, x):
        # The recurrence keeps its state channels-last between the chains
        # (Chain in_cl / out_cl): the cat(x, y) of r_unet.py:223 and the
        # StackedDilation cat (:362) are channel-wise cats of padded
        # channels-last tensors that the next 1x1 convolution reads as channel
        # parts (in_part), the residual add (:224) is an add of two such
        # tensors -- no layout pass between the 71 convolutions of a step.
        _ready(x, 'RDCNet input')
        bf16 = bf16_active(self)
        tr = self.training
        C = self.strided_conv.out_channels
        blk, sd = self.RDCblock, self.RDCblock.grouped_conv
        cl = dict(in_cl=True, out_cl=True)
        x = _chain(self, self, 'strided_cl', self.strided_conv.in_channels,
                   [('conv', self.strided_conv, None, False)], out_cl=True)(x, tr, bf16)
        step = _chain(blk, self, 'conv_cl', blk.conv.in_channels, [('conv', blk.conv, None, False)],
                      in_part=C, **cl)
        dil = [_chain(sd, self, 'd%d_cl' % i, C, [('conv', c, None, False)], **cl)
               for i, c in enumerate((sd.conv1, sd.conv2, sd.conv3, sd.conv4, sd.conv5))]
        mix = _chain(sd, self, 'out_cl', sd.out_conv.in_channels, [('conv', sd.out_conv, None, False)],
                     in_part=C, **cl)
        # The residual state y stays fp32, as the reference's under autocast
        # (r_unet.py:223-225: fp32 zeros, and bf16 block output + fp32 y
        # promotes to fp32); it is rounded to the compute dtype only where it
        # enters a convolution (the cat of :223, out_conv of :226).
        y = torch.zeros(x.shape, dtype=torch.float32, device=x.device)
        yc = y.to(x.dtype)                             # y in the compute dtype (the cat's / out_conv's input)
        trace = getattr(self, '_y_trace', None)   # (tests: y after every recurrence step)
        xs = fan(x, 10)
        # the bf16 path: the two cats and their 1x1x1 convolutions as one native
        # op each (pw_conv: the parts are read where they are; HCU_PW_CAT=0 --
        # or HCU_PW=0, which also takes the chains off the pointwise kernels --
        # keeps cl_cat + the chains)
        pw = bf16 and _lib.env_flag('HCU_PW', True) and _lib.env_flag('HCU_PW_CAT', True)
        for t in range(10):
            s_in = [xs[t], yc]
            u = pw_conv(blk.conv, self, C, s_in) if pw else None
            h = fan(u if u is not None else step(cl_cat(s_in), tr, bf16), len(dil))
            d_out = [d(hi, tr, bf16) for d, hi in zip(dil, h)]
            m = pw_conv(sd.out_conv, self, C, d_out) if pw else None
            y, yc = resid_add(m if m is not None else mix(cl_cat(d_out), tr, bf16), y)
            if trace is not None:
                trace.append(y.detach().clone())
        if bf16:
            # autocast runs the ConvTranspose3d in bf16 too (r_unet.py:227):
            # out_conv's output stays channels-last bf16 and the phase-folded
            # ConvTranspose3d reads it directly (its 5 output channels padded
            # to 8 columns per stride phase, GConvArgs::cph)
            y = _chain(self, self, 'out_cl2', self.out_conv.in_channels, [('conv', self.out_conv, None, False)],
                       in_cl=True, out_cl=True)(yc, tr, True)
            return _chain(self, self, 'convt_cl', self.transposed_conv.in_channels,
                          [('convt', self.transposed_conv)], in_cl=True)(y, tr, True)
        y = _chain(self, self, 'out_cl', self.out_conv.in_channels, [('conv', self.out_conv, None, False)],
                   in_cl=True)(yc, tr, bf16)
        return _chain(self, self, 'convt', self.transposed_conv.in_channels,
                      [('convt', self.transposed_conv)])(y, tr, False)
