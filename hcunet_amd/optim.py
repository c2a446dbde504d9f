"""Adam for the U-Net training step (torch.optim.Adam semantics, one launch).

Same constructor and update rule as torch.optim.Adam(params, lr=1e-3) used by
the reference training pattern (tests/r_unet_test.py:24,56); amsgrad and
maximize are not on the path.  When a param group's parameters and gradients
are consecutive views of one flat buffer (what Unet_Constructor sets up), the
whole group is updated by a single hcu_adam_step launch; otherwise each
tensor gets its own launch.  Optimizer state keeps torch's per-parameter
layout ('step', 'exp_avg', 'exp_avg_sq'), so state_dict() is compatible.
"""
import ctypes
from itertools import chain as _chain_it

import torch
from torch.optim import optimizer as _topt

from . import _lib


def _flat_run(tensors):
    """(base tensor of the run, total numel) if `tensors` are consecutive fp32
    views of one storage, else None."""
    if not tensors:
        return None
    t0 = tensors[0]
    base = t0.data_ptr()
    off = 0
    for t in tensors:
        if t.dtype != torch.float32 or not t.is_contiguous() or t.data_ptr() != base + 4 * off:
            return None
        off += t.numel()
    return t0, off


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                 amsgrad=False):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 0: {betas[0]}")
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 1: {betas[1]}")
        if not 0.0 <= weight_decay:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if amsgrad:
            raise NotImplementedError('amsgrad is not on the accelerated path')
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      amsgrad=False))

    def _ensure_state(self, ps, flat):
        states = [self.state[p] for p in ps]
        if all('exp_avg' in s for s in states):
            return
        dev = ps[0].device
        if flat:
            n = sum(p.numel() for p in ps)
            M = torch.zeros(n, dtype=torch.float32, device=dev)
            V = torch.zeros(n, dtype=torch.float32, device=dev)
            step = torch.tensor(0.0)   # one step counter shared by the flat group
            off = 0
            for p, s in zip(ps, states):
                k = p.numel()
                s['step'] = step
                s['exp_avg'] = M[off:off + k].view_as(p)
                s['exp_avg_sq'] = V[off:off + k].view_as(p)
                off += k
        else:
            for p, s in zip(ps, states):
                if 'exp_avg' not in s:
                    s['step'] = torch.tensor(0.0)
                    s['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    s['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)

    # Any change of the optimizer's state or groups invalidates the cached flat
    # layouts of _fast_step (a loaded state_dict replaces exp_avg/exp_avg_sq
    # and 'step' with new tensors that the cached flat M/V would not update).
    def load_state_dict(self, state_dict):
        self._fast = {}
        super().load_state_dict(state_dict)
        self._fast = {}

    def add_param_group(self, param_group):
        self._fast = {}
        super().add_param_group(param_group)

    def _fast_step(self, L, gi, group):
        """One launch for a group whose flat layout was verified on a previous
        step: re-checked with O(1) pointer tests instead of a pass over every
        parameter (the per-step host cost of the optimizer)."""
        fast = getattr(self, '_fast', None)
        if fast is None:
            self._fast = fast = {}
        f = fast.get(gi)
        if f is None:
            return False
        plist, n_list, p0, pl, pbase, gbase, n, M, V, step_t = f
        g0, gl = p0.grad, pl.grad
        if (group['params'] is not plist or len(plist) != n_list or g0 is None or gl is None
                or p0.data_ptr() != pbase or g0.data_ptr() != gbase
                or gl.data_ptr() != gbase + 4 * (n - pl.numel())
                or pl.data_ptr() != pbase + 4 * (n - pl.numel())):
            fast.pop(gi, None)
            return False
        # every parameter in between must also have a gradient in the same flat
        # buffer (a clone attached by a mixed-accumulation backward is not), and
        # the optimizer state must still be the cached flat M/V and step tensor
        s0, sl = self.state.get(p0), self.state.get(pl)
        if (s0 is None or sl is None or s0.get('step') is not step_t
                or sl.get('step') is not step_t
                or s0['exp_avg'].data_ptr() != M.data_ptr()
                or s0['exp_avg_sq'].data_ptr() != V.data_ptr()
                or sl['exp_avg'].data_ptr() != M.data_ptr() + 4 * (n - pl.numel())):
            fast.pop(gi, None)
            return False
        off = 0
        for p in plist:
            g = p.grad
            if g is None or g.data_ptr() != gbase + 4 * off:
                fast.pop(gi, None)
                return False
            off += p.numel()
        step = int(step_t.item()) + 1
        step_t.fill_(step)
        b1, b2 = group['betas']
        _lib.check(L.hcu_adam_step(
            ctypes.c_void_p(pbase), ctypes.c_void_p(gbase), _lib.ptr(M), _lib.ptr(V), n,
            group['lr'], b1, b2, group['eps'], group['weight_decay'], step, 1.0,
            _lib.stream_handle(p0.device)), 'Adam.step')
        return True

    def zero_grad(self, set_to_none: bool = True):
        """torch.optim.Optimizer.zero_grad; the set_to_none form without the
        profiler range when no profiler runs (host time per step)."""
        if not set_to_none or torch.autograd._profiler_enabled():
            return super().zero_grad(set_to_none)
        for group in self.param_groups:
            for p in group['params']:
                p.grad = None

    def step(self, closure=None):
        """One Adam step.  torch wraps Optimizer.step in a profiler range and
        the step hooks; this runs the same hooks, and the range only while a
        profiler is recording (marked 'hooked' so torch does not wrap it
        again: ~20 us of host time per step)."""
        if torch.autograd._profiler_enabled():
            with torch.autograd.profiler.record_function('Optimizer.step#Adam.step'):
                return self._hooked_step(closure)
        return self._hooked_step(closure)
    step.hooked = True

    def _hooked_step(self, closure):
        args, kwargs = (self, closure), {}
        for pre_hook in _chain_it(_topt._global_optimizer_pre_hooks.values(),
                                  self._optimizer_step_pre_hooks.values()):
            result = pre_hook(self, args, kwargs)
            if result is not None:
                if isinstance(result, tuple) and len(result) == 2:
                    args, kwargs = result
                else:
                    raise RuntimeError('step pre-hook must return None or a tuple of (new_args, new_kwargs)')
        out = self._step(*args[1:], **kwargs)
        self._optimizer_step_code()
        for post_hook in _chain_it(self._optimizer_step_post_hooks.values(),
                                   _topt._global_optimizer_post_hooks.values()):
            post_hook(self, args, kwargs)
        return out

    @torch.no_grad()
    def _step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        L = _lib.lib()
        for gi, group in enumerate(self.param_groups):
            if self._fast_step(L, gi, group):
                continue
            ps = [p for p in group['params'] if p.grad is not None]
            if not ps:
                continue
            for p in ps:
                _lib.require_device(p, 'Adam parameter')
                if p.grad.is_sparse:
                    raise RuntimeError('Adam does not support sparse gradients')
            b1, b2 = group['betas']
            prun = _flat_run(ps)
            grun = _flat_run([p.grad for p in ps]) if prun else None
            flat = prun is not None and grun is not None
            self._ensure_state(ps, flat)
            states = [self.state[p] for p in ps]
            if flat:
                mrun = _flat_run([s['exp_avg'] for s in states])
                vrun = _flat_run([s['exp_avg_sq'] for s in states])
                steps = {float(s['step']) for s in states}
                flat = mrun is not None and vrun is not None and len(steps) == 1
            stream = _lib.stream_handle(ps[0].device)
            if flat:
                step = int(float(states[0]['step'])) + 1
                shared = all(s['step'] is states[0]['step'] for s in states)
                for s in (states[:1] if shared else states):
                    s['step'].fill_(step)
                _lib.check(L.hcu_adam_step(
                    _lib.ptr(prun[0]), _lib.ptr(grun[0]), _lib.ptr(mrun[0]), _lib.ptr(vrun[0]),
                    prun[1], group['lr'], b1, b2, group['eps'], group['weight_decay'], step, 1.0,
                    stream), 'Adam.step')
                if shared:
                    self._fast[gi] = (group['params'], len(group['params']), ps[0], ps[-1],
                                      prun[0].data_ptr(), grun[0].data_ptr(), prun[1],
                                      mrun[0], vrun[0], states[0]['step'])
            else:
                for p, s in zip(ps, states):
                    g = p.grad
                    if not (p.is_contiguous() and g.is_contiguous()
                            and p.dtype == torch.float32 and g.dtype == torch.float32):
                        raise RuntimeError('hcunet_amd.optim.Adam: contiguous fp32 tensors required')
                    s['step'] += 1
                    _lib.check(L.hcu_adam_step(
                        _lib.ptr(p), _lib.ptr(g), _lib.ptr(s['exp_avg']), _lib.ptr(s['exp_avg_sq']),
                        p.numel(), group['lr'], b1, b2, group['eps'], group['weight_decay'],
                        int(float(s['step'])), 1.0, stream), 'Adam.step')
        # the parameters changed behind their version counters: layer chains
        # re-lay their packed weight images on their next call
        from . import chain as _chain
        _chain.invalidate_weight_images()
        return loss
