"""Drop-in hcat.unet.Unet_Constructor whose arithmetic runs in libhcunet.so.

Interface parity with the reference (hcat/unet.py):
  * constructor signature, kwarg normalisation and errors (:16-71),
  * module tree and registration order, hence state_dict keys and the exact
    seeded initialisation (:87-123; nn.Conv3d / nn.BatchNorm3d /
    nn.ConvTranspose3d are used as parameter containers so torch's default
    init consumes the RNG in the reference's order),
  * forward(x) (:125-143), save(filename, hyperparameters) (:145-165),
    load(filename, to_cuda) (:167-196), evaluate(image) (:198-233).

Compute: forward/backward of the whole network are ONE autograd node whose
forward and backward are single calls into the native executor
(hcu_unet_forward / hcu_unet_backward), which enqueue the HIP kernels on the
current stream.

Precision: by default the network computes in fp32, exactly the reference's
arithmetic.  Under torch.autocast('cuda', dtype=torch.bfloat16) (or with
`module.compute_dtype = torch.bfloat16`) it runs the bf16 path of BASELINE
config 3: bf16 activations, gradients and MFMA operands, fp32 accumulation,
BatchNorm statistics, parameters and optimizer state; the input may then be a
fp32, fp16 or bf16 volume (16-bit volumes are read directly by the first
kernel), and the logits are returned in fp32.  Parameters live in one flat fp32 buffer (each nn.Parameter is
a view of it) and gradients are written into one flat buffer whose views are
attached as .grad, so the optimizer step and the data-parallel all-reduce are
single launches over contiguous memory.
"""
import ctypes
import glob
import os

import torch
import torch.nn as nn

from . import _lib


# ---------------------------------------------------------------------------
class Unet_Constructor(nn.Module):
    def __init__(self,
                 image_dimensions=2,
                 in_channels=3,
                 out_channels=2,
                 feature_sizes=[32, 64, 128, 256, 512, 1024],
                 kernel=(3, 3),
                 upsample_kernel=(2, 2),
                 max_pool_kernel=(2, 2),
                 upsample_stride=2,
                 dilation=1,
                 groups=1,
                 ):
        """Generic symmetric U-Net builder (same contract as hcat/unet.py:16-123).

        Dict-valued kernel/dilation/groups select per-step values with keys
        'conv1' and 'conv2'; a tuple/int applies to both steps.
        """
        super().__init__()
        if image_dimensions == 2:
            conv_functions = (nn.Conv2d, nn.ConvTranspose2d, nn.MaxPool2d, nn.BatchNorm2d)
        elif image_dimensions == 3:
            conv_functions = (nn.Conv3d, nn.ConvTranspose3d, nn.MaxPool3d, nn.BatchNorm3d)
        else:
            raise ValueError(f'Does not support {image_dimensions} dimensional images')

        if type(kernel) is tuple:
            kernel = {'conv1': kernel, 'conv2': kernel}
        if type(dilation) is int or type(dilation) is tuple:
            dilation = {'conv1': dilation, 'conv2': dilation}
        if type(groups) is int or type(groups) is tuple:
            groups = {'conv1': groups, 'conv2': groups}

        if len(feature_sizes) < 2:
            raise ValueError(f'The Number of Features must be at least 2, not {len(feature_sizes)}')
        for i, f in enumerate(feature_sizes[0:-1:1]):
            assert f * 2 == feature_sizes[i + 1], \
                f'Feature Sizes must be multiples of two from each other: {f} != {feature_sizes[i - 1]}*2'

        self.model_specification = {
            'image_dimensions': image_dimensions,
            'in_channels': in_channels,
            'out_channels': out_channels,
            'feature_sizes': feature_sizes,
            'kernel': kernel,
            'upsample_kernel': upsample_kernel,
            'max_pool_kernel': max_pool_kernel,
            'upsample_stride': upsample_stride,
            'dilation': dilation,
            'groups': groups,
        }

        # Creation order decides the RNG stream of the default init: all Down
        # blocks, then all Up blocks, then out_conv (hcat/unet.py:87-120).
        down = [Down(conv_functions, in_channels=in_channels, out_channels=feature_sizes[0],
                     kernel=kernel, dilation=dilation, groups=groups)]
        for i in range(1, len(feature_sizes)):
            down.append(Down(conv_functions, in_channels=feature_sizes[i - 1],
                             out_channels=feature_sizes[i], kernel=kernel,
                             dilation=dilation, groups=groups))
        up = []
        for i, f in enumerate(feature_sizes[:0:-1]):
            up.append(Up(conv_functions, in_channels=f, out_channels=feature_sizes[-2 - i],
                         kernel=kernel, upsample_kernel=upsample_kernel,
                         upsample_stride=upsample_stride, dilation=dilation, groups=groups))
        # Registration order (state_dict / parameters()): out_conv first.
        self.out_conv = conv_functions[0](feature_sizes[0], out_channels, 1)
        self.down_steps = nn.ModuleList(down)
        self.up_steps = nn.ModuleList(up)
        self.max_pool = conv_functions[2](max_pool_kernel)
        self._engine = None
        # None: follow torch.autocast; torch.float32 / torch.bfloat16: force
        self.compute_dtype = None

    # -- nn.Module plumbing ------------------------------------------------
    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._engine = None  # parameters were re-materialised: re-flatten lazily
        return out

    def engine(self):
        if self._engine is None:
            self._engine = _Engine(self)
        return self._engine

    def _bf16(self):
        cd = getattr(self, 'compute_dtype', None)
        if cd is not None:
            if cd not in (torch.float32, torch.bfloat16):
                raise ValueError('compute_dtype must be torch.float32 or torch.bfloat16')
            return cd == torch.bfloat16
        return bool(torch.is_autocast_enabled('cuda')
                    and torch.get_autocast_dtype('cuda') == torch.bfloat16)

    def forward(self, x):
        if not isinstance(x, torch.Tensor):
            raise TypeError(f'Expected input of type torch.Tensor, not {type(x)}')
        _lib.require_device(x, 'Unet_Constructor input')
        eng = self.engine()
        bf16 = self._bf16()
        eng.check_input(x, bf16)
        params = eng.params_ready()
        # No gradient can flow (torch.no_grad(), or nothing requires grad): the
        # forward-only plan, which keeps no activations for a backward.
        p_grad = any(p.requires_grad for p in params)
        fwd_only = not (torch.is_grad_enabled() and (x.requires_grad or p_grad))
        # The parameters are not autograd inputs one by one (82 of them cost
        # the host ~0.1 ms per step in Function.apply and the engine): their
        # gradients are written into the flat buffer and attached by the
        # backward itself (_Engine.grad_target), and ONE empty leaf that
        # requires grad when any parameter does stands for them in the graph.
        return _UnetFunction.apply(x, eng, bf16, fwd_only, eng.token(x.device) if p_grad else None)

    # -- checkpointing (hcat/unet.py:145-196) --------------------------------
    def save(self, filename, hyperparameters=None):
        model = {'state_dict': self.state_dict(),
                 'model_specifications': self.model_specification,
                 'hyperparameters': hyperparameters}
        python_files = {}
        files = glob.glob('./**/*.py', recursive=True) + glob.glob('./**/*.ipynb', recursive=True)
        for f in files:
            with open(f, 'r') as fh:
                python_files[f] = fh.read()
        model['python_files'] = python_files
        model['tree_structure'] = glob.glob('**/*', recursive=True)
        torch.save(model, filename)
        return None

    def load(self, filename, to_cuda=True):
        device = 'cuda:0' if (torch.cuda.is_available() and to_cuda) else 'cpu'
        # A .unet checkpoint is a dict of tensors, builtins and strings: the
        # weights-only unpickler loads it without executing code from the file.
        model = torch.load(filename, map_location=device, weights_only=True)
        spec = model['model_specifications']
        self.__init__(
            image_dimensions=spec['image_dimensions'],
            in_channels=spec['in_channels'],
            out_channels=spec['out_channels'],
            feature_sizes=spec['feature_sizes'],
            kernel=spec['kernel'],
            upsample_kernel=spec['upsample_kernel'],
            max_pool_kernel=spec['max_pool_kernel'],
            upsample_stride=spec['upsample_stride'],
            dilation=spec['dilation'],
            groups=spec['groups'],
        )
        self.load_state_dict(model['state_dict'])
        self.eval()
        try:
            return model['hyperparameters']
        except KeyError:
            return None

    def evaluate(self, image: torch.Tensor):
        """Input checks of hcat/unet.py:198-203.  The reference body never fills
        or returns its mask (tiled inference is hcat.segment's job), so this
        returns None like the reference."""
        if not isinstance(image, torch.Tensor):
            raise ValueError(f'Expected image type of torch.Tensor, not {type(image)}')
        if image.shape[1] != self.model_specification['in_channels']:
            raise ImportError(
                f'Image expected to have {self.model_specification["in_channels"]} not {image.shape[1]}')
        self.eval()
        return None


class Down(nn.Module):
    """Parameter container of one encoder block (hcat/unet.py:236-266)."""

    def __init__(self, conv_functions: tuple, in_channels: int, out_channels: int,
                 kernel: dict, dilation: dict, groups: dict):
        super().__init__()
        self.conv1 = conv_functions[0](in_channels, out_channels, kernel['conv1'],
                                       dilation=dilation['conv1'], groups=groups['conv1'],
                                       padding=0)
        self.conv2 = conv_functions[0](out_channels, out_channels, kernel['conv2'],
                                       dilation=dilation['conv2'], groups=groups['conv2'],
                                       padding=0)
        self.batch1 = conv_functions[3](out_channels)
        self.batch2 = conv_functions[3](out_channels)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        """hcat/unet.py:263-266 as one layer chain (hcunet_amd.chain):
        conv1 -> BN -> ReLU -> conv2 -> BN -> ReLU."""
        _lib.require_device(x, 'Down input')
        from .chain import Chain, bf16_active, flat_of
        ch = self.__dict__.get('_hcu_chain')
        if ch is None:
            ch = Chain(flat_of(self), self.conv1.in_channels,
                       [('conv', self.conv1, self.batch1, False), ('conv', self.conv2, self.batch2, False)])
            self.__dict__['_hcu_chain'] = ch
        return ch(x, self.training, bf16_active())


class Up(nn.Module):
    """Parameter container of one decoder block (hcat/unet.py:269-315)."""

    def __init__(self, conv_functions: tuple, in_channels: int, out_channels: int,
                 kernel: dict, upsample_kernel: tuple, upsample_stride: int,
                 dilation: dict, groups: dict):
        super().__init__()
        self.conv1 = conv_functions[0](in_channels, out_channels, kernel['conv1'],
                                       dilation=dilation['conv1'], groups=groups['conv1'],
                                       padding=0)
        self.conv2 = conv_functions[0](out_channels, out_channels, kernel['conv2'],
                                       dilation=dilation['conv2'], groups=groups['conv2'],
                                       padding=0)
        if conv_functions[1] == torch.nn.modules.conv.ConvTranspose3d:
            self.up_conv = conv_functions[1](in_channels, out_channels, upsample_kernel,
                                             stride=upsample_stride, padding=0)
            self.lin_up = False
        elif conv_functions[1] == torch.nn.Upsample:
            self.lin_up = True
        else:
            # hcat/unet.py:302-303: only ConvTranspose3d is accepted, so every
            # 2D network fails here, as it does in the reference.
            raise RuntimeError('unsupported upsampling function', conv_functions[1])
        self.batch1 = conv_functions[3](out_channels)
        self.batch2 = conv_functions[3](out_channels)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x, y):
        """hcat/unet.py:309-315 as one layer chain (hcunet_amd.chain):
        up_conv -> cat(U, crop(U, y)) = cat(U, U) -> conv1 -> BN -> ReLU ->
        conv2 -> BN -> ReLU."""
        _lib.require_device(x, 'Up input')
        from .chain import Chain, bf16_active, flat_of, upsample_cat_check
        k, st, pd = (_triple(self.up_conv.kernel_size), _triple(self.up_conv.stride),
                     _triple(self.up_conv.padding))
        u = [x.shape[0], self.up_conv.out_channels] + [(x.shape[2 + d] - 1) * st[d] - 2 * pd[d] + k[d]
                                                       for d in range(3)]
        upsample_cat_check(u, y)
        ch = self.__dict__.get('_hcu_chain')
        if ch is None:
            ch = Chain(flat_of(self), self.up_conv.in_channels,
                       [('convt', self.up_conv), ('conv', self.conv1, self.batch1, True),
                        ('conv', self.conv2, self.batch2, False)])
            self.__dict__['_hcu_chain'] = ch
        return ch(x, self.training, bf16_active())


def crop(x, y):
    """hcat/unet.py:318-340: x sliced to y's spatial extent (views only)."""
    assert x.shape[1] == y.shape[1], \
        f'Inputs do not have same number of feature dimmensions: {x.shape} | {y.shape}'
    if x.dim() == 4:
        return x[:, :, 0:y.shape[2]:1, 0:y.shape[3]:1]
    if x.dim() == 5:
        return x[:, :, 0:y.shape[2]:1, 0:y.shape[3]:1, 0:y.shape[4]:1]
    return torch.empty(0)


# ---------------------------------------------------------------------------
def _triple(v):
    if isinstance(v, int):
        return (v, v, v)
    v = tuple(v)
    if len(v) != 3:
        raise ValueError('expected an int or a 3-tuple, got %r' % (v,))
    return v


def spec_struct(module):
    """hcu_unet_spec for a 3D Unet_Constructor (parameters read from its modules)."""
    s = module.model_specification
    if s['image_dimensions'] != 3:
        raise RuntimeError('unsupported upsampling function', nn.ConvTranspose2d)
    fs = list(s['feature_sizes'])
    if len(fs) > _lib.MAX_LEVELS:
        raise NotImplementedError('at most %d levels are supported' % _lib.MAX_LEVELS)
    d0 = module.down_steps[0]
    u0 = module.up_steps[0]
    spec = _lib.UnetSpec()
    spec.levels = len(fs)
    spec.in_channels = d0.conv1.in_channels
    spec.out_channels = module.out_conv.out_channels
    for i, f in enumerate(fs):
        spec.features[i] = f
    spec.k1 = _lib.c_int3(*d0.conv1.kernel_size)
    spec.k2 = _lib.c_int3(*d0.conv2.kernel_size)
    spec.d1 = _lib.c_int3(*d0.conv1.dilation)
    spec.d2 = _lib.c_int3(*d0.conv2.dilation)
    spec.g1 = d0.conv1.groups
    spec.g2 = d0.conv2.groups
    if len(u0.up_conv.kernel_size) != 3:
        raise RuntimeError('ConvTranspose3d kernel_size must have 3 elements, got %r'
                           % (u0.up_conv.kernel_size,))
    spec.up_k = _lib.c_int3(*u0.up_conv.kernel_size)
    spec.up_s = _lib.c_int3(*u0.up_conv.stride)
    spec.pool_k = _lib.c_int3(*_triple(module.max_pool.kernel_size))
    mp = module.max_pool
    if _triple(mp.stride) != _triple(mp.kernel_size) or _triple(mp.padding) != (0, 0, 0) \
            or _triple(mp.dilation) != (1, 1, 1) or mp.ceil_mode:
        raise NotImplementedError('max_pool must be kernel == stride, no padding, floor mode')
    bns = bn_modules(module)
    eps, mom = bns[0].eps, bns[0].momentum
    for bn in bns:
        if bn.eps != eps or bn.momentum != mom or not bn.affine or not bn.track_running_stats:
            raise NotImplementedError('all BatchNorm3d layers must share eps/momentum and be '
                                      'affine with running statistics')
    spec.bn_eps = eps
    spec.bn_momentum = -1.0 if mom is None else mom
    # every Down/Up must use the same hyper-parameters (true by construction)
    for blk in list(module.down_steps) + list(module.up_steps):
        for conv, k, d, g in ((blk.conv1, spec.k1, spec.d1, spec.g1),
                              (blk.conv2, spec.k2, spec.d2, spec.g2)):
            if tuple(conv.kernel_size) != tuple(k) or tuple(conv.dilation) != tuple(d) \
                    or conv.groups != g or tuple(conv.stride) != (1, 1, 1) \
                    or tuple(conv.padding) != (0, 0, 0):
                raise NotImplementedError('non-uniform conv hyper-parameters')
    return spec


def bn_modules(module):
    out = []
    for blk in module.down_steps:
        out += [blk.batch1, blk.batch2]
    for blk in module.up_steps:
        out += [blk.batch1, blk.batch2]
    return out


class _Plan:
    def __init__(self, spec, B, X, Y, Z, flags=0):
        L = _lib.lib()
        handle = ctypes.c_void_p()
        _lib.check(L.hcu_unet_plan_create_ex(ctypes.byref(spec), B, X, Y, Z, flags,
                                             ctypes.byref(handle)),
                   'Unet_Constructor')
        self.handle = handle
        out_shape = (ctypes.c_int64 * 5)()
        n_params = ctypes.c_int64()
        n_bn = ctypes.c_int()
        saved = ctypes.c_size_t()
        scratch = ctypes.c_size_t()
        _lib.check(L.hcu_unet_plan_query(handle, out_shape, ctypes.byref(n_params),
                                         ctypes.byref(n_bn), ctypes.byref(saved),
                                         ctypes.byref(scratch)))
        self.out_shape = tuple(int(v) for v in out_shape)
        self.n_params = int(n_params.value)
        self.n_bn = int(n_bn.value)
        self.saved_bytes = int(saved.value)
        self.scratch_bytes = int(scratch.value)

    def __del__(self):
        try:
            if self.handle:
                _lib.lib().hcu_unet_plan_destroy(self.handle)
        except Exception:
            pass


class _Engine:
    """Per-module native state: plans per input shape, flat params/grads."""

    def __init__(self, module):
        self.module_ref = module
        self.spec = spec_struct(module)
        self.plans = {}
        self.flat = None
        self.grad_flat = None
        # grad_flat is the head of comm_flat; the tail is room for the BatchNorm
        # running statistics, so a data-parallel step reduces both in ONE
        # collective (hcunet_amd.dist.allreduce_gradients).
        self.comm_flat = None
        self.params = None
        self._slots = None   # (module, name) of each parameter, in self.params order
        self._bns = None
        self._bn_arrays = None
        # data-parallel overlap (hcunet_amd.dist.prepare_overlap): native events
        # the backward records when gradient groups are final, and whether the
        # last backward recorded them into grad_flat
        self.grad_events = None      # (ev_decoder, ev_deep, deep_level) or None
        self.events_recorded = False
        self.grad_version = None     # grad_flat._version right after the last backward
        # per-parameter views of grad_flat, made once per grad_flat (attaching
        # a cached view costs the host ~0.4 us, slicing a new one ~5 us: 82
        # parameters per step)
        self._grad_views = None
        self._token = None           # the autograd input that stands for the parameters

    def token(self, dev):
        t = self._token
        if t is None or t.device != dev:
            t = self._token = torch.empty(0, device=dev, requires_grad=True)
        return t

    def check_input(self, x, bf16=False):
        m = self.module_ref
        if x.dim() != 5:
            raise RuntimeError('Expected 5D input [B, C, X, Y, Z] for conv3d, got %dD' % x.dim())
        cin = m.down_steps[0].conv1.in_channels
        if x.shape[1] != cin:
            raise RuntimeError('Given groups=%d, expected input%s to have %d channels, but got %d '
                               'channels instead' % (m.down_steps[0].conv1.groups,
                                                     list(x.shape), cin, x.shape[1]))
        ok = (torch.float32, torch.float16, torch.bfloat16) if bf16 else (torch.float32,)
        if x.dtype not in ok:
            raise RuntimeError('Input type (%s) and weight type (float) should be the same' % x.dtype)

    def plan(self, shape, bf16=False, forward_only=False):
        """Launch plan for an input shape.  forward_only: the no-grad plan whose
        forward keeps no activations for a backward (HCU_PLAN_FORWARD_ONLY)."""
        key = tuple(shape) + (bool(bf16), bool(forward_only))
        p = self.plans.get(key)
        if p is None:
            B, _, X, Y, Z = tuple(shape)
            spec = _lib.UnetSpec.from_buffer_copy(self.spec)
            spec.compute_dtype = _lib.HCU_BF16 if bf16 else _lib.HCU_F32
            p = _Plan(spec, B, X, Y, Z, _lib.HCU_PLAN_FORWARD_ONLY if forward_only else 0)
            self.plans[key] = p
        return p

    def params_ready(self, require_gpu=True):
        """Ensure every parameter is a view of one flat fp32 buffer (a device
        buffer for the native path; require_gpu=False lays out host tensors the
        same way, for the CPU tests of the data-parallel host logic).  The
        per-step check follows the (module, name) slots recorded at layout
        time: a replaced Parameter or moved storage is detected; a whole
        submodule swapped into the network after the first forward is not
        (rebuild the model, as the reference's own load() does)."""
        m = self.module_ref
        flat = self.flat
        ok = flat is not None and self.params is not None and self._slots is not None
        if ok:
            # fast path: the (module, name) slots recorded at layout time still
            # hold the same Parameter objects, each still a view of the flat
            # buffer (no recursive module walk per step: host time)
            base = flat.data_ptr()
            off = 0
            for (mod, name), q in zip(self._slots, self.params):
                if mod._parameters.get(name) is not q or q.data_ptr() != base + 4 * off:
                    ok = False
                    break
                off += q.numel()
        if ok:
            return self.params
        params = list(m.parameters())
        ok = flat is not None and self.params is not None and len(params) == len(self.params)
        if ok:
            base = flat.data_ptr()
            off = 0
            for p, q in zip(params, self.params):
                if p is not q or p.data_ptr() != base + 4 * off:
                    ok = False
                    break
                off += p.numel()
        if ok:
            self._slots = [(mod, name) for _, mod in m.named_modules()
                           for name, prm in mod._parameters.items() if prm is not None]
            if len(self._slots) != len(params) or any(mod._parameters[n] is not q
                                                      for (mod, n), q in zip(self._slots, params)):
                self._slots = None
        if not ok:
            dev = params[0].device
            for p in params:
                if p.dtype != torch.float32:
                    raise RuntimeError('hcunet_amd: parameters must be float32')
                if p.device != dev:
                    raise RuntimeError('hcunet_amd: parameters on several devices')
            if require_gpu:
                _lib.require_device(params[0], 'Unet_Constructor parameters')
            n = sum(p.numel() for p in params)
            flat = torch.empty(n, dtype=torch.float32, device=dev)
            off = 0
            with torch.no_grad():
                for p in params:
                    k = p.numel()
                    flat[off:off + k].copy_(p.data.reshape(-1))
                    p.data = flat[off:off + k].view_as(p)
                    off += k
            self.flat = flat
            self.params = params
            self.grad_flat = None
            self.comm_flat = None
            self._bn_arrays = None
            self._slots = [(mod, name) for _, mod in m.named_modules()
                           for name, prm in mod._parameters.items() if prm is not None]
            if len(self._slots) != len(params) or any(mod._parameters[n] is not q
                                                      for (mod, n), q in zip(self._slots, params)):
                self._slots = None   # unusual registration order: keep the full check
        return self.params

    def bn_arrays(self):
        if self._bn_arrays is None:
            bns = bn_modules(self.module_ref)
            self._bns = bns
            for bn in bns:
                if bn.running_mean.dtype != torch.float32 or not bn.running_mean.is_contiguous():
                    raise RuntimeError('hcunet_amd: BatchNorm running stats must be contiguous fp32')
            n = len(bns)
            rm = (ctypes.c_void_p * n)(*[bn.running_mean.data_ptr() for bn in bns])
            rv = (ctypes.c_void_p * n)(*[bn.running_var.data_ptr() for bn in bns])
            nb = (ctypes.c_void_p * n)(*[bn.num_batches_tracked.data_ptr() for bn in bns])
            self._bn_arrays = (rm, rv, nb, [bn.running_mean.data_ptr() for bn in bns])
        else:
            bns = self._bns
            if [bn.running_mean.data_ptr() for bn in bns] != self._bn_arrays[3]:
                self._bn_arrays = None
                return self.bn_arrays()
        return self._bn_arrays

    def tensors(self, x, out, saved, scratch, grads=None):
        rm, rv, nb, _ = self.bn_arrays()
        t = _lib.UnetTensors()
        t.x = x.data_ptr()
        t.out = out.data_ptr() if out is not None else None
        t.params = self.flat.data_ptr()
        t.grads = grads.data_ptr() if grads is not None else None
        t.bn_running_mean = ctypes.cast(rm, ctypes.POINTER(ctypes.c_void_p))
        t.bn_running_var = ctypes.cast(rv, ctypes.POINTER(ctypes.c_void_p))
        t.bn_num_batches_tracked = ctypes.cast(nb, ctypes.POINTER(ctypes.c_void_p))
        t.saved = saved.data_ptr()
        t.scratch = scratch.data_ptr()
        t.x_dtype = _X_DTYPES[x.dtype]
        return t

    def grad_target(self):
        """Decide where backward writes parameter gradients.

        Returns (buffer, accumulate, finish) where finish() attaches/adds the
        gradients with torch's .grad accumulation semantics."""
        params = self.params
        if self.grad_flat is None or self.grad_flat.numel() != self.flat.numel() \
                or self.grad_flat.device != self.flat.device:
            n_stats = 2 * sum(bn.num_features for bn in bn_modules(self.module_ref))
            self.comm_flat = torch.zeros(self.flat.numel() + n_stats, dtype=torch.float32,
                                         device=self.flat.device)
            self.grad_flat = self.comm_flat[:self.flat.numel()]
        G = self.grad_flat
        views = self._grad_views
        if views is None or views[0] is not G or len(views[1]) != len(params):
            offs, vs, off = [], [], 0
            for p in params:
                offs.append(off)
                vs.append(G[off:off + p.numel()].view_as(p))
                off += p.numel()
            views = self._grad_views = (G, vs, offs)
        _, vs, offs = views
        grads = [p.grad for p in params]
        if all(g is None for g in grads):
            def finish():
                for p, v in zip(params, vs):
                    if p.requires_grad:
                        p.grad = v
            return G, 0, finish
        if all(g is v for g, v in zip(grads, vs)):
            return G, 1, (lambda: None)
        base = G.data_ptr()
        if all(g is not None and g.data_ptr() == base + 4 * o and g.shape == p.shape
               for p, g, o in zip(params, grads, offs)):
            return G, 1, (lambda: None)
        tmp = torch.empty_like(self.flat)

        def finish_mixed():
            for p, o in zip(params, offs):
                if not p.requires_grad:
                    continue
                g = tmp[o:o + p.numel()].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.add_(g)
        return tmp, 0, finish_mixed


_POISON = os.environ.get('HCU_POISON') == '1'
_X_DTYPES = {torch.float32: _lib.HCU_F32, torch.float16: _lib.HCU_F16,
             torch.bfloat16: _lib.HCU_BF16}


class _NoCtx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


_NO_CTX = _NoCtx()


def _on_device(dev):
    """torch.cuda.device(dev), skipped when dev is already current (the
    executor creates its side and capture streams on the current device)."""
    return _NO_CTX if dev.index == torch.cuda.current_device() else torch.cuda.device(dev)


class _UnetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, eng, bf16, fwd_only, token):
        x = x.contiguous()
        plan = eng.plan(x.shape, bf16, forward_only=fwd_only)
        dev = x.device
        out = torch.empty(plan.out_shape, dtype=torch.float32, device=dev)
        saved = torch.empty(max(plan.saved_bytes, 1), dtype=torch.uint8, device=dev)
        scratch = torch.empty(max(plan.scratch_bytes, 1), dtype=torch.uint8, device=dev)
        if _POISON:   # debugging: every byte the step does not write reads as NaN
            saved.fill_(255)
            scratch.fill_(255)
        training = 1 if eng.module_ref.training else 0
        t = eng.tensors(x, out, saved, scratch)
        # The executor's graph-capture and side streams are created on the
        # current device: make it the tensors' device.
        with _on_device(dev):
            _lib.check(_lib.lib().hcu_unet_forward(plan.handle, ctypes.byref(t), training,
                                                   _lib.stream_handle(dev)),
                       'Unet_Constructor.forward')
        ctx.eng = eng
        ctx.plan = plan
        ctx.training = training
        if not fwd_only:
            ctx.save_for_backward(x, saved)
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dout):
        x, saved = ctx.saved_tensors
        eng, plan = ctx.eng, ctx.plan
        dev = x.device
        dout = dout.contiguous()
        if dout.dtype != torch.float32:
            dout = dout.float()
        scratch = torch.empty(max(plan.scratch_bytes, 1), dtype=torch.uint8, device=dev)
        if _POISON:
            scratch.fill_(255)
        dx = torch.empty(x.shape, dtype=torch.float32, device=dev) if ctx.needs_input_grad[0] else None
        G, accumulate, finish = eng.grad_target()
        t = eng.tensors(x, None, saved, scratch, grads=G)
        ev = eng.grad_events if G is eng.grad_flat else None
        L = _lib.lib()
        if ev is not None and not L.hcu_unet_grad_events_live(plan.handle):
            ev = None   # a replayed (graphed) backward does not record them
        _lib.check(L.hcu_unet_set_grad_events(
            plan.handle, ev[0] if ev else None, ev[1] if ev else None, ev[2] if ev else 0),
            'Unet_Constructor.backward')
        eng.events_recorded = ev is not None
        with _on_device(dev):
            _lib.check(L.hcu_unet_backward(plan.handle, ctypes.byref(t),
                                           ctypes.c_void_p(dout.data_ptr()),
                                           _lib.ptr(dx), ctx.training, accumulate,
                                           _lib.stream_handle(dev)),
                       'Unet_Constructor.backward')
        finish()
        # in-place work on the gradients between here and allreduce_gradients
        # (clip_grad_norm_, GradScaler.unscale_, .grad edits) bumps this
        # version: the overlapped reduction then falls back to one collective
        # behind the caller's stream (hcunet_amd/dist.py)
        eng.grad_version = eng.grad_flat._version if G is eng.grad_flat else None
        if dx is not None and dx.dtype != x.dtype:
            dx = dx.to(x.dtype)
        return dx, None, None, None, None
