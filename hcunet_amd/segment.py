"""Tiled inference driver: drop-in for
``hcat.segment.predict_segmentation_mask`` (hcat/segment.py:21-136) and for
``hcat.utils.pad_image_with_reflections`` / ``calculate_indexes``
(hcat/utils.py:33-124).

Same arguments, tile geometry, tile order, crop, sigmoid/threshold and error
messages as the reference; what changes is where the work runs:

* the volume is copied to HBM once and stays there (the reference pads the
  whole volume on the host with numpy and copies one fp32 tile per forward);
* reflection padding is index arithmetic inside the tile-gather kernel
  (``hcu_tile_gather``), which also applies the reference's NaN -> 0 / Inf -> 1
  cleaning and writes a *batch* of tiles as the network input;
* tiles of equal shape run as one batched forward when the module is in eval
  mode (the reference runs B=1; in train mode BatchNorm uses batch statistics,
  so a batch would change the result and tiles run one by one as there);
* forwards under ``torch.no_grad`` use the forward-only plan
  (``HCU_PLAN_FORWARD_ONLY``): no activation workspace is kept for a backward;
* crop + sigmoid (the reference's in-place x*-1, exp, +1, pow(-1) chain) +
  threshold + the write into the mask are one kernel per tile
  (``hcu_tile_scatter``), issued in the reference's tile order so overlapping
  tiles resolve the same way;
* the reference keys the tile size on ``str(floor(GPU GB))`` and raises
  ``KeyError`` on anything but 4/6/8/11 GB parts (a 288 GB MI355X included,
  segment.py:52-54); here the largest table entry that fits is used.

Deliberate difference: the reference cleans NaN/Inf *in the caller's tensor*
(segment.py:66-67 assigns into ``image``); this driver leaves the caller's
tensor untouched and cleans on the fly.
"""
import ctypes

import numpy as np
import torch

from . import _lib

__all__ = ['predict_segmentation_mask', 'pad_image_with_reflections', 'calculate_indexes',
           'eval_image_size', 'PAD_SIZE']

# hcat/segment.py:48-57
_EVAL_IM_SIZE = {'4': [128, 128, 6],   # In GB
                 '6': [300, 300, 6],
                 '8': [300, 300, 10],
                 '11': [350, 350, 15]}
PAD_SIZE = (128, 128, 10)


def eval_image_size(total_memory_bytes):
    """Tile (evaluation) size for a GPU of `total_memory_bytes`: the entry of the
    reference's table (segment.py:48-52) keyed by the largest size <= the
    device's floor(GB); the smallest entry below 4 GB.  The reference indexes
    the table with str(floor(GB)) and raises KeyError for any other size."""
    gb = int(np.floor(total_memory_bytes / 1e9))
    keys = sorted(int(k) for k in _EVAL_IM_SIZE)
    fit = [k for k in keys if k <= gb]
    return list(_EVAL_IM_SIZE[str(fit[-1] if fit else keys[0])])


def calculate_indexes(pad_size, eval_image_size, image_shape, padded_image_shape):
    """hcat/utils.py:77-124: [start, stop) index pairs covering a padded axis with
    windows of eval_image_size + 2 * pad_size, stepping by eval_image_size (the
    reference's quirks kept: regular windows end at z - 1 + 2 * pad, the last
    window is appended even when it repeats, and an evaluation size larger than
    the image gives [[0, image_shape]])."""
    if eval_image_size > image_shape:
        return [[0, image_shape]]
    if eval_image_size <= 0:
        raise RuntimeError(f'Calculate_indexes has incorrect values {pad_size} | {image_shape} | '
                           f'{eval_image_size}:\nYou are likely trying to have a chunk smaller than '
                           'the set evaluation image size. Please decrease number of chunks.')
    ind_list = list(range(0, image_shape, eval_image_size))
    ind = []
    for i, z in enumerate(ind_list):
        if i == 0:
            continue
        z1 = int(ind_list[i - 1])
        z2 = int(z - 1) + (2 * pad_size)
        if z2 < padded_image_shape:
            ind.append([z1, z2])
        else:
            break
    if not ind:
        ind.append([0, eval_image_size + pad_size * 2])
        ind.append([padded_image_shape - (eval_image_size + pad_size * 2), padded_image_shape])
    else:
        ind.append([padded_image_shape - (eval_image_size + pad_size * 2), padded_image_shape - 1])
    return ind


def _check_pad_args(image, pad_size):
    # hcat/utils.py:44-48
    if not isinstance(image, torch.Tensor):
        raise TypeError(f'Expected image to be of type torch.tensor not {type(image)}')
    for pad in pad_size:
        if pad % 2 != 0:
            raise ValueError('Padding must be divisible by 2')


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError('hcunet_amd: the tiled inference driver needs a GPU (no CPU fallback)')
    return torch.device('cuda', torch.cuda.current_device())


def _as_device_volume(image, dev):
    """[B, C, X, Y, Z] -> contiguous device tensor of fp32 or fp16 (the gather
    kernel's input types), viewed as one sample with B*C channels."""
    x = image
    if x.dtype not in (torch.float32, torch.float16):
        x = x.float()
    return x.to(dev).contiguous()


def _gather(vol, pads, origins, tile_dims, clean, out, stream):
    C = vol.shape[0] * vol.shape[1]
    X, Y, Z = vol.shape[2:]
    I3 = ctypes.c_int * 3
    org = (ctypes.c_int * (3 * len(origins)))(*[v for o in origins for v in o])
    dtype = _lib.HCU_F16 if vol.dtype == torch.float16 else _lib.HCU_F32
    _lib.check(_lib.lib().hcu_tile_gather(
        ctypes.c_void_p(vol.data_ptr()), dtype, C, X, Y, Z, I3(*pads), org, len(origins),
        I3(*tile_dims), int(clean), ctypes.c_void_p(out.data_ptr()), stream), 'tile gather')


def pad_image_with_reflections(image, pad_size=(30, 30, 6)):
    """hcat/utils.py:33-74: reflection-pad X, Y, Z of a [B, C, X, Y, Z] tensor by
    pad_size on both sides (numpy's image[pad-1::-1] | image | image[-1:-pad-1:-1],
    i.e. the edge voxel repeated).  Computed on the GPU by the tile-gather kernel
    (one tile = the whole padded volume); returns a tensor on the input's
    device with the input's dtype (fp32 for other dtypes)."""
    _check_pad_args(image, pad_size)
    dev = _device()
    vol = _as_device_volume(image, dev)
    B, C, X, Y, Z = vol.shape
    pads = [min(int(p), n) for p, n in zip(pad_size, (X, Y, Z))]
    dims = [n + 2 * p for n, p in zip((X, Y, Z), pads)]
    out = torch.empty((B, C) + tuple(dims), dtype=torch.float32, device=dev)
    _gather(vol, pads, [(0, 0, 0)], dims, False, out, _lib.stream_handle(dev))
    out = out.to(vol.dtype)
    return out if image.device == dev else out.to(image.device)


def _slice_len(start, stop, n):
    a, b, _ = slice(start, stop).indices(n)
    return a, max(0, b - a)


def _tile_bytes(unet, C, tdims):
    """Device bytes one tile of a batched forward needs: its fp32 input, its
    output, and the forward's own workspaces (the plan's saved + scratch
    bytes at batch 1; the workspaces scale with the batch)."""
    vox = tdims[0] * tdims[1] * tdims[2]
    eng_fn = getattr(unet, 'engine', None)
    if eng_fn is None:   # not this package's network: a conservative guess
        return 4 * C * vox * 64
    eng = eng_fn()
    # the driver's forward runs under no_grad: the forward-only plan
    plan = eng.plan((1, C) + tuple(tdims), unet._bf16(), forward_only=True)
    out = 4 * plan.out_shape[1] * plan.out_shape[2] * plan.out_shape[3] * plan.out_shape[4]
    return 4 * C * vox + out + plan.saved_bytes + plan.scratch_bytes


def predict_segmentation_mask(unet, image, device=None, use_probability_map=False,
                              mask_cell_prob_threshold=0.5, tiles_per_batch=None,
                              total_memory=None):
    """hcat/segment.py:21-136 on the GPU.  image: [1, C, X, Y, Z] (transforms
    applied), any device; returns the [1, 1, X, Y, Z] mask on the CPU as the
    reference does: fp32 probabilities with use_probability_map, else uint8
    (probability > mask_cell_prob_threshold).  tiles_per_batch bounds the
    batched forward in eval mode (default: as many tiles as fit in a quarter of
    free device memory, at most HCU_TILE_BATCH_MAX).  total_memory overrides the
    device memory size that selects the tile size (the reference's
    hcat.__CUDA_MEM__)."""
    if not isinstance(image, torch.Tensor):
        image = torch.as_tensor(image)
    dev = _device()
    mem = total_memory if total_memory is not None else torch.cuda.get_device_properties(dev).total_memory
    pad = PAD_SIZE
    ev = eval_image_size(mem)
    im_shape = image.shape
    if im_shape[4] < ev[2]:
        ev[2] = im_shape[4]
    _check_pad_args(image, pad)
    vol = _as_device_volume(image, dev)
    _, C, X, Y, Z = vol.shape
    pads = [min(p, n) for p, n in zip(pad, (X, Y, Z))]
    padded = [n + 2 * p for n, p in zip((X, Y, Z), pads)]
    x_ind = calculate_indexes(pad[0], ev[0], im_shape[2], padded[0])
    y_ind = calculate_indexes(pad[1], ev[1], im_shape[3], padded[1])
    z_ind = calculate_indexes(pad[2], ev[2], im_shape[4], padded[2])

    # tiles in the reference's loop order (z, x, y): torch slice semantics of
    # image[:, :, x0:x1, y0:y1, z0:z1]
    tiles = []
    for z in z_ind:
        for x in x_ind:
            for y in y_ind:
                (ox, tx), (oy, ty), (oz, tz) = (_slice_len(x[0], x[1], padded[0]),
                                                _slice_len(y[0], y[1], padded[1]),
                                                _slice_len(z[0], z[1], padded[2]))
                tiles.append(((ox, oy, oz), (tx, ty, tz), (x[0], y[0], z[0])))

    mask = torch.zeros((1, 1, X, Y, Z), dtype=torch.float32, device=dev)
    mdims = (X, Y, Z)
    stream = _lib.stream_handle(dev)
    batch_cap = 1 if unet.training else _lib.HCU_TILE_BATCH_MAX
    if tiles_per_batch is not None:
        batch_cap = max(1, min(batch_cap, int(tiles_per_batch)))

    I3 = ctypes.c_int * 3
    i = 0
    with torch.no_grad():
        while i < len(tiles):
            tdims = tiles[i][1]
            if min(tdims) < 1:
                raise RuntimeError(f'Amount of padding is not sufficient.\nvalid_out.shape: n/a\n'
                                   f'eval_image_size: {ev} ')
            j = i + 1
            cap = batch_cap
            if tiles_per_batch is None and cap > 1:
                free = torch.cuda.mem_get_info(dev)[0]
                cap = max(1, min(cap, int(free / 4 // _tile_bytes(unet, C, tdims))))
            while j < len(tiles) and j - i < cap and tiles[j][1] == tdims:
                j += 1
            batch = tiles[i:j]
            xb = torch.empty((len(batch), C) + tuple(tdims), dtype=torch.float32, device=dev)
            _gather(vol, pads, [t[0] for t in batch], tdims, True, xb, stream)
            # "Occasionally everything is just -1 in the whole mat. Skip for speed"
            skip = (xb == -1).flatten(1).all(1).tolist()
            try:
                out = unet(xb)
            except torch.OutOfMemoryError:
                if len(batch) == 1 or tiles_per_batch is not None:
                    raise
                # the estimate was optimistic (fragmentation, other tenants):
                # retry this run of tiles with half the batch
                del xb
                batch_cap = max(1, len(batch) // 2)
                continue
            except RuntimeError as e:   # native workspace allocation failures
                if len(batch) == 1 or tiles_per_batch is not None or 'out of memory' not in str(e):
                    raise
                del xb
                batch_cap = max(1, len(batch) // 2)
                continue
            if not out.is_contiguous() or out.dtype != torch.float32:
                out = out.float().contiguous()
            Co, OX, OY, OZ = out.shape[1:]
            tile_shape = torch.Size((1, C) + tuple(tdims))
            for b, (org, _, dst) in enumerate(batch):
                if skip[b]:
                    continue
                crop = [_slice_len(p, e + p, n) for p, e, n in zip(pad, ev, (OX, OY, OZ))]
                vshape = torch.Size((1, Co) + tuple(c[1] for c in crop))
                wr = [_slice_len(d, d + e, n) for d, e, n in zip(dst, ev, mdims)]
                tshape = (1, 1) + tuple(w[1] for w in wr)
                ok = Co == 1 and all(v == t or v == 1 for v, t in zip(vshape[2:], tshape[2:]))
                if not ok:
                    raise RuntimeError(f'Amount of padding is not sufficient.\nvalid_out.shape: '
                                       f'{vshape}\neval_image_size: {ev} '
                                       f'\npadded_image_slice.shape{tile_shape} ')
                if not use_probability_map and mask.dtype != torch.uint8:
                    mask = mask.to(torch.uint8)
                mdt = _lib.HCU_U8 if mask.dtype == torch.uint8 else _lib.HCU_F32
                bc = [1 if v == 1 and t != 1 else 0 for v, t in zip(vshape[2:], tshape[2:])]
                src = out[b, 0]
                _lib.check(_lib.lib().hcu_tile_scatter(
                    ctypes.c_void_p(src.data_ptr()), I3(OX, OY, OZ), I3(*[c[0] for c in crop]),
                    I3(*bc), ctypes.c_void_p(mask.data_ptr()), mdt, I3(*mdims),
                    I3(*[w[0] for w in wr]), I3(*[w[1] for w in wr]),
                    0 if use_probability_map else 1, float(mask_cell_prob_threshold), stream),
                    'tile scatter')
            i = j
    return mask.cpu()
