"""Drop-in hcat.dataloader.Stack (hcat/dataloader.py:17-92) feeding the device
input path.

Same constructor, file discovery (`{path}/*.mask.tif` + `.tif` + `.pwl.tif`),
errors and __getitem__ order of transforms as the reference.  What changes:
* the raw stacks are kept as read (uint16 / uint8) in page-locked host memory,
  so a host->device copy is one asynchronous DMA of the raw bytes;
* the default out_transforms is hcunet_amd.transforms.to_tensor, which runs
  the to_float -> reshape -> normalize -> to_tensor chain as one device pass
  and returns fp16 tensors already on the GPU;
* `prefetch(order)` yields items while the next one is copied and converted
  on a side stream (the reference converts on the host and copies float
  tensors, segment.py:89 / the training loop's .cuda()).
Files are read with skimage.io.imread (as the reference) or tifffile when
importable; `reader=` takes any callable path -> ndarray.
"""
import glob
import os

import numpy as np
import torch

from . import transforms as t


def _default_reader():
    try:
        from skimage import io   # the reference's reader (hcat/dataloader.py:3)
        return io.imread
    except ImportError:
        pass
    try:
        import tifffile
        return tifffile.imread
    except ImportError:
        pass
    return None


def _pinned(a):
    """The raw bits as a page-locked tensor (uint16 held as int16: same bytes);
    without a ROCm device (construction on a CPU host) the tensor stays pageable."""
    a = np.ascontiguousarray(a)
    t_ = torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else a)
    if torch.cuda.is_available():
        t_ = t_.pin_memory()
    return t_, a.dtype, a.ndim


class _Raw:
    """A pinned raw stack that behaves like the ndarray the reference holds
    for expand_dims / ndim / dtype purposes and hands the pinned tensor to the
    device path."""

    def __init__(self, a):
        self.tensor, self.np_dtype, _ = _pinned(a)

    def pending(self, expand=False):
        r = self.tensor.unsqueeze(self.tensor.dim()) if expand else self.tensor
        return t.PendingVolume(r, np_dtype=self.np_dtype)


_LAZY = (t.to_float, t.reshape, t.normalize, t.to_tensor)


def _arrays_for(transform, items):
    """The lazy device chain understands PendingVolume; any other transform
    (the reference's random augmentations, a caller's own) gets the ndarray
    the reference's eager chain would hold at that point."""
    if isinstance(transform, _LAZY):
        return items
    return [x.to_ndarray() if isinstance(x, t.PendingVolume) else x for x in items]


class Stack(torch.utils.data.Dataset):
    """Dataloader for hcat.unet: 3D stacks with mask and pixel-weight maps."""

    def __init__(self, path, image_transforms, joint_transforms, out_transforms=None, reader=None):
        if out_transforms is None:
            out_transforms = [t.to_tensor()]
        self.image_transforms = image_transforms
        self.out_transforms = out_transforms
        self.joint_transforms = joint_transforms
        self.files = glob.glob(f'{path}{os.sep}*.mask.tif')
        if len(self.files) == 0:
            raise FileExistsError('No Valid Mask Files Found')
        reader = reader or _default_reader()
        if reader is None:
            raise ImportError('hcat.dataloader.Stack reads .tif stacks with skimage.io or tifffile; '
                              'neither is installed (pass reader=callable)')
        self.image, self.mask, self.pwl = [], [], []
        for mask_path in self.files:
            file_with_mask = os.path.splitext(mask_path)[0]
            image_data_path = os.path.splitext(file_with_mask)[0] + '.tif'
            pwl_data_path = os.path.splitext(file_with_mask)[0] + '.pwl.tif'
            self.image.append(_Raw(reader(image_data_path)))
            m = reader(mask_path)
            try:   # some masks are [Z,Y,X,C], others [Z,Y,X] (:57-61)
                m = m[:, :, :, 0]
            except IndexError:
                pass
            self.mask.append(_Raw(m))
            self.pwl.append(_Raw(reader(pwl_data_path)))

    def __len__(self):
        return len(self.files)

    def __getitem__(self, item):
        # channel axis last (:80-81), on the pinned raw tensors (no copy)
        image = self.image[item].pending()
        mask = self.mask[item].pending(expand=True)
        pwl = self.pwl[item].pending(expand=True)
        for jt in self.joint_transforms:
            image, mask, pwl = _arrays_for(jt, [image, mask, pwl])
            image, mask, pwl = jt([image, mask, pwl])
        for it in self.image_transforms:
            image = _arrays_for(it, [image])[0]
            image = it(image)
        for ot in self.out_transforms:
            image, mask, pwl = _arrays_for(ot, [image, mask, pwl])
            image, mask, pwl = ot([image, mask, pwl])
        return image, mask, pwl

    def prefetch(self, order=None, device=None):
        """Yield self[i] for i in `order`, converting item k+1 on a side stream
        while item k is consumed on the current stream."""
        order = list(range(len(self))) if order is None else list(order)
        device = torch.device('cuda', torch.cuda.current_device()) if device is None else torch.device(device)
        side = torch.cuda.Stream(device)
        main = torch.cuda.current_stream(device)

        def launch(i):
            with torch.cuda.stream(side):
                items = self[i]
            ev = torch.cuda.Event()
            ev.record(side)
            return items, ev

        nxt = launch(order[0]) if order else None
        for k in range(len(order)):
            items, ev = nxt
            if k + 1 < len(order):
                nxt = launch(order[k + 1])
            main.wait_event(ev)
            for x in items:
                if isinstance(x, torch.Tensor):
                    x.record_stream(main)
            yield items
