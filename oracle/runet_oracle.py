"""TEST INFRASTRUCTURE ONLY: torch-CPU restatement of the reference's r_unet.py
models (RDCNet, RecursiveUnet), the parity oracle of hcunet_amd.r_unet.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg -- never by the product path.  Each function follows the reference
(hcat/r_unet.py) statement for statement on torch.nn.functional ops, with
parameters taken from a state dict (the reference modules' keys):

  rdcnet_forward      hcat/r_unet.py:207-227 (RDCNet), :367-378 (RDCBlock),
                      :339-364 (StackedDilation)
  runet_forward       hcat/r_unet.py:135-162 (RecursiveUnet), :232-246 (f),
                      :249-283 (Down), :286-336 (Up), :14-35 (crop)

BatchNorm3d in train mode updates the running statistics in the state
(momentum 0.1, unbiased variance), as nn.BatchNorm3d does on every call.
Pinned against the reference itself by tests/golden/runet_*.npz
(tests/golden/make_runet_golden.py; tests/test_runet_oracle.py).
"""
import torch
import torch.nn.functional as F


def _conv(s, key, x, stride=1, padding=0, dilation=1):
    return F.conv3d(x, s[key + '.weight'], s[key + '.bias'], stride=stride, padding=padding,
                    dilation=dilation)


def _bn(s, key, x, training):
    return F.batch_norm(x, s[key + '.running_mean'], s[key + '.running_var'], s[key + '.weight'],
                        s[key + '.bias'], training=training, momentum=0.1, eps=1e-5)


def _bump(s, key, training):
    if training:
        s[key + '.num_batches_tracked'] += 1


# ---- RDCNet (hcat/r_unet.py:207-227, 339-378) -----------------------------
def stacked_dilation(s, key, x):
    xs = [_conv(s, '%s.conv%d' % (key, d), x, padding=2 * d, dilation=d) for d in range(1, 6)]
    return _conv(s, key + '.out_conv', torch.cat(xs, dim=1))


def rdc_block(s, key, x):
    return stacked_dilation(s, key + '.grouped_conv', _conv(s, key + '.conv', x))


def rdcnet_forward(s, x):
    x = _conv(s, 'strided_conv', x, stride=2, padding=1)
    y = None
    for t in range(10):
        if t == 0:
            y = torch.zeros(x.shape, dtype=x.dtype)
        y = rdc_block(s, 'RDCblock', torch.cat((x, y), dim=1)) + y
    y = _conv(s, 'out_conv', y, padding=1)
    return F.conv_transpose3d(y, s['transposed_conv.weight'], s['transposed_conv.bias'], stride=2,
                              padding=1)


# ---- RecursiveUnet (hcat/r_unet.py:38-204, 232-336) ------------------------
def crop(x, y):
    return x[:, :, 0:y.shape[2], 0:y.shape[3], 0:y.shape[4]]


def down(s, key, x, training, padding=1):
    x = F.relu(_bn(s, key + '.batch1', _conv(s, key + '.conv1', x, padding=padding), training))
    x = F.relu(_bn(s, key + '.batch2', _conv(s, key + '.conv2', x, padding=1), training))
    _bump(s, key + '.batch1', training)
    _bump(s, key + '.batch2', training)
    return x


def up(s, key, x, y, training, stride=(2, 2, 1)):
    x = F.conv_transpose3d(x, s[key + '.up_conv.weight'], s[key + '.up_conv.bias'], stride=stride,
                           padding=2)
    y = crop(x, y)
    x = torch.cat((x, y), dim=1)
    x = F.relu(_bn(s, key + '.batch1', _conv(s, key + '.conv1', x, padding=1), training))
    x = F.relu(_bn(s, key + '.batch2', _conv(s, key + '.conv2', x, padding=1), training))
    _bump(s, key + '.batch1', training)
    _bump(s, key + '.batch2', training)
    return x


def f_forward(s, d1, d2, u1, x, training, pool=(2, 2, 1)):
    x = down(s, d1, x, training)
    b = x.clone()
    x = F.max_pool3d(x, pool)
    x = down(s, d2, x, training)
    return up(s, u1, x, b, training)


def runet_forward(s, image, training=True, pool=(2, 2, 1)):
    x = None
    for t in range(10):
        if t == 0:
            s_t = torch.zeros([1, 5, image.shape[2], image.shape[3], image.shape[4]], dtype=image.dtype)
        x = torch.cat((image, s_t), dim=1)
        x = down(s, 'down1', x, training)
        a = x.clone()
        x = F.max_pool3d(x, pool)
        h = torch.tanh(f_forward(s, 'down2_fh', 'down3_fh', 'up1_fh', x, training))
        if t == 0:
            h_t = torch.ones(h.shape, dtype=h.dtype)
        z = torch.sigmoid(f_forward(s, 'down2_fz', 'down3_fz', 'up1_fz', x, training))
        h_t = (h_t * z) + (-1 * z * h)
        x = up(s, 'up2', h_t, a, training)
        x = _conv(s, 'out_conv', x)
        s_t = x
    return x


def state_of(module, dtype=torch.float64):
    """Detached CPU copy of a module's state dict in `dtype` (integer buffers
    kept), parameters requiring grad."""
    out = {}
    for k, v in module.state_dict().items():
        v = v.detach().cpu().clone()
        if v.is_floating_point():
            v = v.to(dtype)
        out[k] = v
    for k, p in module.named_parameters():
        out[k] = out[k].requires_grad_(True)
    return out
