"""TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's loss functions
(hcat/loss.py), the parity oracle for hcunet_amd.loss on the GPU.

  cross_entropy(method=...)  hcat/loss.py:5-101   ('pixel', 'worst_z', 'random', 'sigmoid')
  dice                       hcat/loss.py:104-126
  L1Loss                     hcat/loss.py:128-152
  MSELoss                    hcat/loss.py:154-178

Pinned against the reference itself by tests/golden/loss_methods.npz
(tests/golden/make_loss_golden.py imports /root/reference/hcat/loss.py in the
development container).  Only tests/ import this module.
"""
import torch
import torch.nn.functional as F

METHODS = ['pixel', 'worst_z', 'random', 'sigmoid']   # hcat/loss.py:25


def _crop(t, ps):
    """Top-left crop to pred's extent (hcat/loss.py:51-56, 113-118, ...)."""
    if len(ps) == 5:
        return t[:, :, 0:ps[2]:1, 0:ps[3]:1, 0:ps[4]:1]
    if len(ps) == 4:
        return t[:, :, 0:ps[2]:1, 0:ps[3]:1]
    raise IndexError('Unexpected number of predicted mask dimensions. Expected 4 (2D) or 5 (3D) '
                     f'but got {len(ps)} dimensions: {ps}')


def cross_entropy(pred, mask, pwl, method='pixel', num_random_pixels=None):
    """hcat/loss.py:5-101."""
    if method not in METHODS:                                          # :25-27
        raise ValueError(f'Viable methods for cross entropy loss are {METHODS}, not {method}.')
    if method == 'random':                                             # :29-36
        if num_random_pixels is None:
            raise ValueError('num_random_pixels undefined')
        if num_random_pixels <= 1:
            raise ValueError('num_random_pixels should be greater than 1')
        if (mask == 0).sum() == 0:
            raise ValueError('There are no background pixels in mask.')
    if method == 'sigmoid':                                            # :38-40
        pred = torch.sigmoid(pred)
    ps = pred.shape
    if pwl is None:                                                    # :45-47
        pwl = torch.ones(pred.shape)
    mask = _crop(mask, ps)                                             # :50-53
    pwl = _crop(pwl, ps)
    # :61-63 ('+2 on mask') is dead code: is_pwl_none is always True (:48)
    if method in ('pixel', 'sigmoid'):                                 # :69-72, :95-97
        loss = F.binary_cross_entropy_with_logits(pred.float(), mask.float(), reduction='none')
        loss = loss * (pwl + 1)
    elif method == 'worst_z':                                          # :74-80
        loss = F.binary_cross_entropy_with_logits(pred.float(), mask.float(), reduction='none')
        loss = loss * (pwl + 1)
        scaling = torch.linspace(1, 2, pred.shape[4]) ** 2
        loss, _ = torch.sort(loss.sum(dim=[0, 1, 2, 3]))
        loss = loss * scaling
        loss = loss / (pred.shape[2] * pred.shape[3])
    else:                                                              # random, :82-93
        pred = pred.reshape(-1)
        mask = mask.reshape(-1)
        if (mask == 1).sum() == 0:
            loss = F.binary_cross_entropy_with_logits(pred.float(), mask.float(), reduction='none')
        else:
            pos_ind = torch.randint(low=0, high=int((mask == 1).sum()), size=(1, num_random_pixels))[0, :]
            neg_ind = torch.randint(low=0, high=int((mask == 0).sum()), size=(1, num_random_pixels))[0, :]
            p = torch.cat([pred[mask == 1][pos_ind], pred[mask == 0][neg_ind]]).unsqueeze(0)
            m = torch.cat([mask[mask == 1][pos_ind], mask[mask == 0][neg_ind]]).unsqueeze(0)
            loss = F.binary_cross_entropy_with_logits(p.float(), m.float(), reduction='none')
    return loss.mean()                                                 # :101


def dice(pred, mask):
    """hcat/loss.py:104-126."""
    mask = _crop(mask, pred.shape)
    pred = torch.sigmoid(pred)
    loss = (2 * (pred * mask).sum() + 1e-10) / ((pred + mask).sum() + 1e-10)
    return 1 - loss


def L1Loss(pred, mask):
    """hcat/loss.py:128-152."""
    return F.l1_loss(pred, _crop(mask, pred.shape))


def MSELoss(pred, mask):
    """hcat/loss.py:154-178."""
    return F.mse_loss(pred, _crop(mask, pred.shape))
