"""Per-layer algorithmic work of the U-Net training step.

For every layer of a Unet_Constructor training step (forward + input
gradient + weight gradient) this gives the algorithmic FLOPs and the
compulsory HBM bytes, and from them the layer's roofline time
max(bytes / HBM peak, FLOPs / MFMA peak).  The step's per-layer roofline is
the sum over layers.  Rules:
  * FLOPs = 2 x MACs of the forward, x3 for forward + input gradient + weight
    gradient, x2 for the first convolution (no input gradient); the decoder's
    conv1 is counted with the cat(U, U) fold (hcat/unet.py:311-312: its input
    has U's channels, not twice them);
  * bytes = E x (|x| + 5 x sum |T| + 3 x |W|) with T every conv, ConvTranspose
    and pool output (written and read once forward; the saved tensor read,
    its gradient written and read once backward) and E the element size of
    the compute dtype; BatchNorm / ReLU / cat are assumed fused.
Shapes follow hcat/unet.py:125-143 (valid convolutions, floor pooling,
ConvTranspose3d out = (in - 1) * s + k).
"""
PEAK_HBM = 8.0e12          # B/s, MI355X HBM3E (MI355X_MICROARCH.md)
PEAK_FP32 = 157.3e12       # FLOP/s dense fp32 MFMA
PEAK_BF16 = 2.5e15         # FLOP/s dense bf16 MFMA


def _t3(v):
    return (v, v, v) if isinstance(v, int) else tuple(v)


def layers(kw, B, shape, bf16=False):
    """[{'layer', 'kind', 'flops', 'bytes', 'roof_us'}] for a Unet_Constructor
    built with kwargs `kw` on an input [B, C, *shape]."""
    E = 2 if bf16 else 4
    peak = PEAK_BF16 if bf16 else PEAK_FP32
    fs = list(kw['feature_sizes'])
    cin = kw['in_channels']
    k = kw['kernel']
    k1 = _t3(k['conv1'] if isinstance(k, dict) else k)
    k2 = _t3(k['conv2'] if isinstance(k, dict) else k)
    d = kw.get('dilation', 1)
    d1 = _t3(d['conv1'] if isinstance(d, dict) else d)
    d2 = _t3(d['conv2'] if isinstance(d, dict) else d)
    g = kw.get('groups', 1)
    g1 = g['conv1'] if isinstance(g, dict) else g
    g2 = g['conv2'] if isinstance(g, dict) else g
    uk, us = _t3(kw['upsample_kernel']), _t3(kw['upsample_stride'])
    pk = _t3(kw['max_pool_kernel'])
    out = []

    def vol(s):
        return s[0] * s[1] * s[2]

    def add(name, kind, flops, tensor_elems, w_elems, extra_elems=0):
        by = E * (5 * tensor_elems + 3 * w_elems + extra_elems)
        out.append(dict(layer=name, kind=kind, flops=flops, bytes=by,
                        roof_us=max(by / PEAK_HBM, flops / peak) * 1e6))

    def conv(name, s, ci, co, kk, dd, gg, first=False):
        o = tuple(s[i] - dd[i] * (kk[i] - 1) for i in range(3))
        macs = B * vol(o) * co * (ci // gg) * vol(kk)
        w = co * (ci // gg) * vol(kk) + co
        add(name, 'conv', 2 * macs * (2 if first else 3), B * vol(o) * co, w,
            B * vol(s) * ci if first else 0)
        return o

    s = tuple(shape)
    c = cin
    for i, f in enumerate(fs):
        s = conv('d%d.c1' % i, s, c, f, k1, d1, g1, first=(i == 0))
        s = conv('d%d.c2' % i, s, f, f, k2, d2, g2)
        c = f
        if i < len(fs) - 1:
            s = tuple(s[j] // pk[j] for j in range(3))
            add('d%d.pool' % i, 'pool', 0.0, B * vol(s) * f, 0)
    for j in range(len(fs) - 1):
        f, o = fs[-1 - j], fs[-2 - j]
        u = tuple((s[i] - 1) * us[i] + uk[i] for i in range(3))
        macs = B * vol(s) * f * o * vol(uk)     # every input voxel meets every tap
        add('u%d.up' % j, 'convT', 6 * macs, B * vol(u) * o, f * o * vol(uk) + o)
        s = conv('u%d.c1' % j, u, o, o, k1, d1, g1)   # cat(U, U) folded
        s = conv('u%d.c2' % j, s, o, o, k2, d2, g2)
    return out


def step_roofline(kw, B, shape, bf16=False):
    """(per-layer roofline ms, FLOPs, bytes) of one training step."""
    ls = layers(kw, B, shape, bf16)
    return (sum(r['roof_us'] for r in ls) / 1e3, sum(r['flops'] for r in ls),
            sum(r['bytes'] for r in ls))
