"""TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's tiled inference
driver, the parity oracle for hcunet_amd/segment.py.

  pad_image_with_reflections   hcat/utils.py:33-74 (numpy reflection slices)
  calculate_indexes            hcat/utils.py:77-124
  predict_segmentation_mask    hcat/segment.py:21-136 (B=1 tiles, crop, in-place
                               sigmoid chain, threshold, writes in z, x, y order)
The network is any callable tile -> output (the tests pass OracleUnet.forward
in eval mode).  Pinned against the reference's own functions by
tests/golden/segment_small.npz (tests/golden/make_segment_golden.py).
"""
import numpy as np
import torch

EVAL_IM_SIZE = {'4': [128, 128, 6], '6': [300, 300, 6], '8': [300, 300, 10],
                '11': [350, 350, 15]}   # hcat/segment.py:48-52
PAD_SIZE = (128, 128, 10)               # hcat/segment.py:54


def pad_image_with_reflections(image, pad_size=(30, 30, 6)):
    """hcat/utils.py:33-74."""
    if not isinstance(image, torch.Tensor):
        raise TypeError(f'Expected image to be of type torch.tensor not {type(image)}')
    for pad in pad_size:
        if pad % 2 != 0:
            raise ValueError('Padding must be divisible by 2')
    a = image.numpy()
    out = a
    for ax, p in zip((2, 3, 4), pad_size):
        idx_l = [slice(None)] * 5
        idx_r = [slice(None)] * 5
        idx_l[ax] = slice(p - 1, None, -1)       # image[..., pad-1::-1]
        idx_r[ax] = slice(-1, -p - 1, -1)        # image[..., -1:-pad-1:-1]
        out = np.concatenate((out[tuple(idx_l)], out, out[tuple(idx_r)]), axis=ax)
    return torch.as_tensor(out.copy())


def calculate_indexes(pad_size, eval_image_size, image_shape, padded_image_shape):
    """hcat/utils.py:77-124."""
    if eval_image_size > image_shape:
        return [[0, image_shape]]
    ind_list = np.arange(0, image_shape, eval_image_size)
    ind = []
    for i in range(1, len(ind_list)):
        z1 = int(ind_list[i - 1])
        z2 = int(ind_list[i] - 1) + 2 * pad_size
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


def predict_segmentation_mask(net, image, total_memory, use_probability_map=False,
                              mask_cell_prob_threshold=0.5):
    """hcat/segment.py:21-136 with `hcat.__CUDA_MEM__ = total_memory` (the
    reference raises KeyError unless floor(total_memory / 1e9) is 4, 6, 8 or 11)."""
    pad = PAD_SIZE
    ev = list(EVAL_IM_SIZE[str(int(np.floor(total_memory / 1e9)))])
    mask = torch.zeros((1, 1) + tuple(image.shape[2:]), dtype=torch.float)
    im_shape = image.shape
    if im_shape[4] < ev[2]:
        ev[2] = im_shape[4]
    image = torch.as_tensor(np.array(image))   # callers pass numpy volumes (segment.py:66)
    image[torch.isnan(image)] = 0
    image[torch.isinf(image)] = 1
    image = pad_image_with_reflections(image, pad_size=pad)
    x_ind = calculate_indexes(pad[0], ev[0], im_shape[2], image.shape[2])
    y_ind = calculate_indexes(pad[1], ev[1], im_shape[3], image.shape[3])
    z_ind = calculate_indexes(pad[2], ev[2], im_shape[4], image.shape[4])
    with torch.no_grad():
        for z in z_ind:
            for x in x_ind:
                for y in y_ind:
                    tile = image[:, :, x[0]:x[1], y[0]:y[1], z[0]:z[1]].float()
                    if (tile == -1).all():
                        continue
                    v = net(tile)
                    v = v[:, :, pad[0]:ev[0] + pad[0], pad[1]:ev[1] + pad[1], pad[2]:ev[2] + pad[2]]
                    v = v.clone()
                    v.mul_(-1)
                    v.exp_()
                    v.add_(1)
                    v.pow_(-1)
                    if not use_probability_map:
                        v.gt_(mask_cell_prob_threshold)
                        v = v.type(torch.uint8)
                        if mask.dtype != torch.uint8:
                            mask = mask.type(torch.uint8)
                    try:
                        mask[:, :, x[0]:x[0] + ev[0], y[0]:y[0] + ev[1], z[0]:z[0] + ev[2]] = v
                    except RuntimeError:
                        raise RuntimeError(f'Amount of padding is not sufficient.\nvalid_out.shape: '
                                           f'{v.shape}\neval_image_size: {ev} '
                                           f'\npadded_image_slice.shape{tile.shape} ')
    return mask
