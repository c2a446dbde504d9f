"""ctypes binding of the C-ABI in include/hcunet.h (libhcunet.so, built in-tree).

The library is the only compute path of this package: there is no CPU or
PyTorch fallback.  If libhcunet.so is missing the first call raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# HCU_LIB_PATH: a variant build of the same sources (A/B runs, tools/gpu_abx.sh)
LIB_PATH = os.environ.get("HCU_LIB_PATH") or os.path.join(_HERE, "libhcunet.so")

HCU_OK = 0
HCU_ERR_INVALID = 1
HCU_ERR_SHAPE = 2
HCU_ERR_HIP = 3
HCU_ERR_UNSUPPORTED = 4
HCU_ERR_WORKSPACE = 5

HCU_F32, HCU_F16, HCU_U8, HCU_BF16, HCU_U16, HCU_F64 = 0, 1, 2, 3, 4, 5
HCU_PLAN_FORWARD_ONLY = 1
HCU_TILE_BATCH_MAX = 64
MAX_LEVELS = 12

c_int3 = ctypes.c_int * 3


class UnetSpec(ctypes.Structure):
    _fields_ = [
        ("levels", ctypes.c_int),
        ("in_channels", ctypes.c_int),
        ("out_channels", ctypes.c_int),
        ("features", ctypes.c_int * MAX_LEVELS),
        ("k1", c_int3), ("k2", c_int3),
        ("d1", c_int3), ("d2", c_int3),
        ("g1", ctypes.c_int), ("g2", ctypes.c_int),
        ("up_k", c_int3), ("up_s", c_int3),
        ("pool_k", c_int3),
        ("bn_eps", ctypes.c_float),
        ("bn_momentum", ctypes.c_float),
        ("compute_dtype", ctypes.c_int),
    ]


class UnetTensors(ctypes.Structure):
    _fields_ = [
        ("x", ctypes.c_void_p),
        ("out", ctypes.c_void_p),
        ("params", ctypes.c_void_p),
        ("grads", ctypes.c_void_p),
        ("bn_running_mean", ctypes.POINTER(ctypes.c_void_p)),
        ("bn_running_var", ctypes.POINTER(ctypes.c_void_p)),
        ("bn_num_batches_tracked", ctypes.POINTER(ctypes.c_void_p)),
        ("saved", ctypes.c_void_p),
        ("scratch", ctypes.c_void_p),
        ("x_dtype", ctypes.c_int),
    ]


class ConvDesc(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int), ("Cin", ctypes.c_int), ("Cout", ctypes.c_int),
        ("X", ctypes.c_int), ("Y", ctypes.c_int), ("Z", ctypes.c_int),
        ("k", c_int3), ("stride", c_int3), ("dil", c_int3),
        ("groups", ctypes.c_int),
        ("transposed", ctypes.c_int),
        ("dtype", ctypes.c_int),
    ]


class BNLayerInfo(ctypes.Structure):
    _fields_ = [
        ("y_offset", ctypes.c_int64), ("coef_offset", ctypes.c_int64),
        ("B", ctypes.c_int), ("X", ctypes.c_int), ("Y", ctypes.c_int), ("Z", ctypes.c_int),
        ("C", ctypes.c_int), ("Cs", ctypes.c_int), ("elem_bytes", ctypes.c_int),
        ("pad", ctypes.c_int),
    ]


# Every symbol include/hcunet.h declares: (name, restype, argtypes)
_VP, _I, _I64, _F, _SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_size_t
SYMBOLS = [
    ("hcu_last_error", ctypes.c_char_p, []),
    ("hcu_version", _I, []),
    ("hcu_unet_plan_create", _I, [ctypes.POINTER(UnetSpec), _I, _I, _I, _I, ctypes.POINTER(_VP)]),
    ("hcu_unet_plan_create_ex", _I, [ctypes.POINTER(UnetSpec), _I, _I, _I, _I, _I,
                                     ctypes.POINTER(_VP)]),
    ("hcu_unet_plan_destroy", None, [_VP]),
    ("hcu_unet_plan_query", _I, [_VP, ctypes.POINTER(_I64), ctypes.POINTER(_I64),
                                 ctypes.POINTER(_I), ctypes.POINTER(_SZ), ctypes.POINTER(_SZ)]),
    ("hcu_unet_plan_bn_layers", _I, [_VP, ctypes.POINTER(BNLayerInfo), _I]),
    ("hcu_unet_forward", _I, [_VP, ctypes.POINTER(UnetTensors), _I, _VP]),
    ("hcu_unet_backward", _I, [_VP, ctypes.POINTER(UnetTensors), _VP, _VP, _I, _I, _VP]),
    ("hcu_loss_pixel_scratch_bytes", _SZ, [_I64]),
    ("hcu_loss_pixel_fwd", _I, [_VP, _I, _I, _I, _I, _I, _VP, _I, _VP, _I, _I, _I, _I,
                                _VP, _VP, _VP, _SZ, _VP]),
    ("hcu_scale_by_device_scalar", _I, [_VP, _VP, _VP, _I64, _VP]),
    ("hcu_loss_ext_scratch_bytes", _SZ, [_I, _I64, _I]),
    ("hcu_loss_ext_fwd", _I, [_I, _VP, _I, _I, _I, _I, _I, _VP, _I, _VP, _I, _I, _I, _I, _VP, _VP, _VP,
                              _VP, _SZ, _VP]),
    ("hcu_loss_ext_bwd", _I, [_I, _VP, _I, _I, _I, _I, _I, _VP, _I, _VP, _I, _I, _I, _I, _VP, _VP, _VP,
                              _VP, _VP]),
    ("hcu_loss_random_rows", _I, [_I64]),
    ("hcu_loss_random_count", _I, [_VP, _I, _I, _I, _I, _I, _VP, _I, _I, _I, _I, _VP, _VP]),
    ("hcu_loss_random_fwd", _I, [_VP, _I, _I, _I, _I, _I, _VP, _I, _I, _I, _I, _VP, _VP, _VP, _VP, _VP,
                                 _I, _VP, _VP, _VP, _VP, _SZ, _VP]),
    ("hcu_ingest_volume", _I, [_VP, _I, _I, _I, _I, _I, _I, _I, _I, ctypes.POINTER(ctypes.c_double),
                               ctypes.POINTER(ctypes.c_double), _VP, _VP]),
    ("hcu_adam_step", _I, [_VP, _VP, _VP, _VP, _I64, _F, _F, _F, _F, _F, _I64, _F, _VP]),
    ("hcu_conv_scratch_bytes", _SZ, [ctypes.POINTER(ConvDesc)]),
    ("hcu_conv_out_dims", _I, [ctypes.POINTER(ConvDesc), ctypes.POINTER(_I)]),
    ("hcu_conv_fwd_cl", _I, [ctypes.POINTER(ConvDesc), _VP, _VP, _VP, _VP, _VP, _SZ, _VP]),
    ("hcu_conv_dgrad_cl", _I, [ctypes.POINTER(ConvDesc), _VP, _VP, _VP, _VP, _SZ, _VP]),
    ("hcu_conv_wgrad_cl", _I, [ctypes.POINTER(ConvDesc), _VP, _VP, _VP, _VP, _VP, _SZ, _VP]),
    ("hcu_maxpool_fwd_cl", _I, [_I, _I, _I, _I, _I, ctypes.POINTER(_I), _VP, _VP, _VP]),
    ("hcu_tile_gather", _I, [_VP, _I, _I, _I, _I, _I, ctypes.POINTER(_I), ctypes.POINTER(_I), _I,
                             ctypes.POINTER(_I), _I, _VP, _VP]),
    ("hcu_tile_scatter", _I, [_VP, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_I), _VP,
                              _I, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_I), _I,
                              _F, _VP]),
    ("hcu_timing_enable", _I, [_I]),
    ("hcu_timing_disable", _I, []),
    ("hcu_timing_detail", _I, [_I]),
    ("hcu_timing_prefix", _I, [ctypes.c_char_p]),
    ("hcu_timing_report", _I64, [ctypes.c_char_p, _I64]),
    ("hcu_chain_plan_create", _I, [_VP, _I, _I, _I, _I, ctypes.POINTER(_VP)]),
    ("hcu_chain_plan_query", _I, [_VP, ctypes.POINTER(_I64), ctypes.POINTER(_I), ctypes.POINTER(_SZ),
                                  ctypes.POINTER(_SZ)]),
    ("hcu_chain_forward", _I, [_VP, ctypes.POINTER(UnetTensors), _I, _VP]),
    ("hcu_chain_backward", _I, [_VP, ctypes.POINTER(UnetTensors), _VP, _VP, _I, _I, _VP]),
    ("hcu_chain_weight_image_bytes", _SZ, [_VP]),
    ("hcu_chain_forward_images", _I, [_VP, ctypes.POINTER(UnetTensors), _I, _VP, _VP, _I]),
    ("hcu_chain_backward_images", _I, [_VP, ctypes.POINTER(UnetTensors), _VP, _VP, _I, _I, _VP, _VP, _I]),
    ("hcu_gate_fwd", _I, [_VP, _VP, _VP, _VP, _I64, _VP]),
    ("hcu_gate_bwd", _I, [_VP, _VP, _VP, _VP, _VP, _VP, _VP, _I64, _VP]),
    ("hcu_gather_vectors", _I, [ctypes.POINTER(_VP), ctypes.POINTER(_I), _I, _VP, _I, _VP]),
    ("hcu_cl_cat", _I, [ctypes.POINTER(_VP), ctypes.POINTER(_I), _I, _VP, _I64, _I, _VP]),
    ("hcu_resid_fwd", _I, [_VP, _VP, _VP, _VP, _I64, _VP]),
    ("hcu_resid_bwd", _I, [_VP, _VP, _VP, _VP, _I64, _VP]),
    ("hcu_sum_parts", _I, [ctypes.POINTER(_VP), _I, _VP, _I64, _I, _VP]),
    ("hcu_pw_conv_forward", _I, [ctypes.POINTER(_VP), _I, _I, _I, _VP, _VP, _VP, _I64, _I, _I, _VP]),
    ("hcu_pw_conv_work_floats", _SZ, [_I64, _I, _I, _I]),
    ("hcu_pw_conv_backward", _I, [ctypes.POINTER(_VP), _I, _I, _I, _VP, _VP, _I, _I, ctypes.POINTER(_VP),
                                  _VP, _VP, _I64, _VP, _SZ, _I, _VP]),
    ("hcu_unet_set_grad_events", _I, [_VP, _VP, _VP, _I]),
    ("hcu_unet_grad_events_live", _I, [_VP]),
    ("hcu_event_create", _I, [ctypes.POINTER(_VP)]),
    ("hcu_event_destroy", _I, [_VP]),
    ("hcu_stream_wait_event", _I, [_VP, _VP]),
    ("hcu_tuning_set_mode", _I, [_I]),
    ("hcu_tuning_get_mode", _I, []),
    ("hcu_tuning_entries", _I64, [ctypes.POINTER(_I64)]),
    ("hcu_tuning_save", _I64, [ctypes.c_char_p]),
]

TUNE_MODEL, TUNE_TABLE, TUNE_TIMED = 0, 1, 2


def tuning_mode(mode=None):
    """Get (mode=None) or set the convolution tiling mode (include/hcunet.h):
    0 cost model, 1 persistent table + cost model on a miss (deterministic
    across processes), 2 table + timing on a miss (default)."""
    L = lib()
    if mode is not None:
        check(L.hcu_tuning_set_mode(int(mode)), 'hcu_tuning_set_mode')
    return int(L.hcu_tuning_get_mode())


def tuning_entries():
    """(entries in the tiling table, entries timed by this process)."""
    timed = ctypes.c_int64()
    n = lib().hcu_tuning_entries(ctypes.byref(timed))
    return int(n), int(timed.value)


def tuning_save(path=None):
    n = lib().hcu_tuning_save(path.encode() if path else None)
    if n < 0:
        raise RuntimeError(last_error())
    return int(n)

_lib = None


def lib():
    """Load libhcunet.so (once) and declare every exported signature."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                "hcunet_amd: native library %s is missing; build it with ./build.sh "
                "(or __graft_entry__.build()). There is no CPU fallback." % LIB_PATH)
        handle = ctypes.CDLL(LIB_PATH)
        for name, res, args in SYMBOLS:
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def last_error():
    msg = lib().hcu_last_error()
    return msg.decode() if msg else ""


def check(code, what=""):
    """Map a C-ABI error code to the exception type the reference path raises."""
    if code == HCU_OK:
        return
    msg = last_error()
    if what:
        msg = "%s: %s" % (what, msg)
    if code == HCU_ERR_INVALID:
        raise ValueError(msg)
    if code == HCU_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise RuntimeError(msg)


_raw_stream = getattr(torch._C, '_cuda_getCurrentRawStream', None)


def stream_handle(device=None):
    """hipStream_t of torch's current stream on `device` (the raw pointer,
    without building a torch.cuda.Stream object: host time per call)."""
    if _raw_stream is not None:
        if device is None:
            idx = torch.cuda.current_device()
        elif isinstance(device, torch.device):
            idx = device.index if device.index is not None else torch.cuda.current_device()
        else:
            idx = torch.device(device).index
            idx = idx if idx is not None else torch.cuda.current_device()
        return ctypes.c_void_p(_raw_stream(idx))
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def env_flag(name, default):
    """An on/off switch of the environment (A/B runs): '0' is off, any
    other value on, unset `default`."""
    v = os.environ.get(name)
    return default if v is None or v == '' else v != '0'


def require_device(t, what):
    if not isinstance(t, torch.Tensor):
        raise TypeError("%s must be a torch.Tensor, got %s" % (what, type(t)))
    if t.device.type != "cuda":
        raise RuntimeError(
            "hcunet_amd: %s is on %s; the MI355X path runs on ROCm devices only "
            "(move the module and tensors with .to('cuda'))" % (what, t.device))


def timing_report():
    """Per-kernel-symbol totals recorded since hcu_timing_enable():
    {name: dict(count, ms, flops, bytes)} (synchronises the recorded events)."""
    L = lib()
    n = L.hcu_timing_report(None, 0)
    buf = ctypes.create_string_buffer(int(n) + 1)
    L.hcu_timing_report(buf, n + 1)
    out = {}
    for line in buf.value.decode().splitlines():
        name, cnt, ms, fl, by = line.split('\t')
        out[name] = dict(count=int(cnt), ms=float(ms), flops=float(fl), bytes=float(by))
    return out
