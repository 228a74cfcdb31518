"""CPU oracle (TEST INFRASTRUCTURE ONLY) — numpy restatement of the int8 arithmetic
that the reference's quantized ConvNet path executes through torch.ao / FBGEMM.

Who may use this module: ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` — as the *checker*, never as the thing that
is measured or shipped.  The product path (``convnet-quantization_amd/``) never
imports anything under ``oracle/``.

Parity pin: every function here is checked bit-for-bit against torch.ao with the
``fbgemm`` engine (torch 2.10.0+rocm7.0, the wheel in this image) by
``oracle/make_golden.py``; the resulting vectors are committed under
``tests/golden/`` and re-checked by ``tests/test_oracle_golden.py``.  The
reference repo itself holds no tests or golden vectors, so the
pin is torch.ao run here, as SURVEY.md §8(c) prescribes.

Reference call sites (``/root/reference``):
  * models/custom_quantization_model.py:41-45   QuantStub -> conv -> DeQuantStub
  * models/custom_quantization_model.py:180-190 fuse_modules (BN fold)
  * models/static_ptq_model.py:28-32            quantize_dynamic (dynamic Linear)
  * models/dynamic_ptq_model.py:289-306         fold + quantize_dynamic
  * models/baseline_model.py:58-83              SimpleConvNet topology
Third-party algorithm (torch 2.10.0 wheel, paths relative to torch/):
  * ao/quantization/observer.py:349-427, 558-569   MinMaxObserver qparams
  * include/fbgemm/QuantUtils.h:68-101              Quantize<T, LEGACY=false>
  * include/fbgemm/OutputProcessing-inl.h:76-127    ReQuantizeOutput::f
  * include/ATen/native/quantized/cpu/QuantUtils.h:70-185  ChooseQuantizationParams
  * nn/utils/fusion.py:56-101, 156-186              fuse_conv_bn / fuse_linear_bn
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
EPS_F32 = F32(np.finfo(np.float32).eps)  # observer eps = 2**-23


# --------------------------------------------------------------------------- A1
def quantize_per_tensor(x, scale, zero_point, qmin=0, qmax=255, out_dtype=np.uint8):
    """aten::quantize_per_tensor on CPU (fbgemm Quantize<T, LEGACY=false>,
    QuantUtils.h:68-101): q = clamp(zp + nearbyint(x * fp32(1/s)), qmin, qmax).
    Round half to even; zero point added *after* rounding."""
    x = np.asarray(x, dtype=F32)
    inv = F32(1.0) / F32(scale)
    t = x * inv
    q = np.rint(t).astype(np.float64) + float(zero_point)
    return np.clip(q, qmin, qmax).astype(out_dtype)


# --------------------------------------------------------------------------- A7
def dequantize(q, scale, zero_point):
    """aten::dequantize: fp32(s) * fp32(q - zp) — one rounding (exact int32 diff)."""
    d = np.asarray(q, dtype=np.int32) - np.int32(zero_point)
    return d.astype(F32) * F32(scale)


# --------------------------------------------------------------------------- A2
def qparams_affine(min_val, max_val, qmin=0, qmax=255):
    """MinMaxObserver._calculate_qparams, per_tensor_affine (observer.py:394-397)."""
    min_neg = min(F32(min_val), F32(0.0))
    max_pos = max(F32(max_val), F32(0.0))
    scale = F32(max_pos - min_neg) / F32(qmax - qmin)
    scale = max(F32(scale), EPS_F32)
    zp = qmin - int(np.rint(F32(min_neg) / F32(scale)))
    zp = int(min(max(zp, qmin), qmax))
    return F32(scale), zp


def qparams_symmetric(min_val, max_val, qmin=-128, qmax=127):
    """MinMaxObserver._calculate_qparams, per_tensor_symmetric qint8
    (observer.py:377-381): scale = max(|min|,|max|) / 127.5, zp = 0.
    Accepts arrays (per-channel) as well as scalars."""
    min_val = np.asarray(min_val, dtype=F32)
    max_val = np.asarray(max_val, dtype=F32)
    min_neg = np.minimum(min_val, F32(0.0))
    max_pos = np.maximum(max_val, F32(0.0))
    amax = np.maximum(-min_neg, max_pos)
    scale = (amax / F32((qmax - qmin) / 2)).astype(F32)
    scale = np.maximum(scale, EPS_F32).astype(F32)
    return scale, np.zeros_like(scale, dtype=np.int64)


def minmax(x):
    """torch.aminmax over the whole tensor (observer.py:563)."""
    x = np.asarray(x, dtype=F32)
    return F32(x.min()), F32(x.max())


# --------------------------------------------------------------------------- A3
def fold_conv_bn(w, b, rm, rv, gamma, beta, eps=1e-5):
    """torch.nn.utils.fusion.fuse_conv_bn_weights (fusion.py:56-101), fp32,
    same op order: rsqrt = 1/sqrt(var+eps); w' = w * (gamma*rsqrt);
    b' = (b - mean) * rsqrt * gamma + beta."""
    w = np.asarray(w, F32)
    if b is None:
        b = np.zeros(w.shape[0], F32)
    rsq = F32(1.0) / np.sqrt(np.asarray(rv, F32) + F32(eps))
    scale = (np.asarray(gamma, F32) * rsq).astype(F32)
    wf = (w * scale.reshape((-1,) + (1,) * (w.ndim - 1))).astype(F32)
    bf = ((((np.asarray(b, F32) - np.asarray(rm, F32)) * rsq) * np.asarray(gamma, F32))
          + np.asarray(beta, F32)).astype(F32)
    return wf, bf


def fold_linear_bn(w, b, rm, rv, gamma, beta, eps=1e-5):
    """torch.nn.utils.fusion.fuse_linear_bn_weights (fusion.py:156-186): unlike
    the conv fold the bias uses the combined scale:
    s = gamma * rsqrt(var+eps); w' = w * s; b' = (b - mean) * s + beta."""
    w = np.asarray(w, F32)
    if b is None:
        b = np.zeros(w.shape[0], F32)
    rsq = F32(1.0) / np.sqrt(np.asarray(rv, F32) + F32(eps))
    s = (np.asarray(gamma, F32) * rsq).astype(F32)
    wf = (w * s.reshape(-1, 1)).astype(F32)
    bf = (((np.asarray(b, F32) - np.asarray(rm, F32)) * s) + np.asarray(beta, F32)).astype(F32)
    return wf, bf


# --------------------------------------------------------------------------- A4
def quantize_weight(w, scale, zero_point=None):
    """Weight quantize (from_float): clamp(rint(w * (1/s)) + zp, -128, 127).
    ``scale`` is a scalar (per-tensor) or a per-output-channel vector."""
    w = np.asarray(w, F32)
    scale = np.asarray(scale, F32)
    if scale.ndim == 0:
        return quantize_per_tensor(w, scale, 0, -128, 127, np.int8)
    out = np.empty(w.shape, np.int8)
    for k in range(w.shape[0]):
        out[k] = quantize_per_tensor(w[k], scale[k], 0, -128, 127, np.int8)
    return out


# --------------------------------------------------------------------------- A6
def fmaf(a, b, c):
    """Exact single-rounding fp32 fused multiply-add fl32(a*b + c), vectorised.
    a*b is exact in float64; the sum is rounded once to double and then to
    float, and the TwoSum error term repairs the only case where that double
    rounding can differ from a single rounding (the double lands exactly on a
    float midpoint)."""
    a64 = np.asarray(a, F32).astype(np.float64)
    b64 = np.asarray(b, F32).astype(np.float64)
    c64 = np.asarray(c, F32).astype(np.float64)
    p = a64 * b64
    s = p + c64
    bb = s - p
    e = (p - (s - bb)) + (c64 - bb)
    r = s.astype(F32)
    r64 = r.astype(np.float64)
    diff = s - r64
    toward = np.where(diff > 0, np.inf, -np.inf).astype(F32)
    nxt = np.nextafter(r, toward)
    mid = (diff != 0) & (s == (r64 + nxt.astype(np.float64)) * 0.5)
    fix = mid & (e != 0) & (np.sign(e) == np.sign(diff))
    return np.where(fix, nxt, r).astype(F32)


def requant_constants(s_x, s_w, s_y, bias):
    """Per-output-channel fp32 constants (u, v, mult) such that the FBGEMM
    epilogue is  t = fmaf(u_k, v_k, fp32(acc)),  ab = fp32(t * mult_k).

    Read from the compiled ``fbgemm::requantizeOutputProcessingAvx2`` in the
    torch 2.10 wheel (QuantUtilsAvx2.h:113 declares it):
      * per-tensor weights: rcp = fp32(1.0f / aws) (``vdivss``) and the bias
        term is FMA-contracted: t = fmaf(b_k, rcp, fp32(acc)) -> (u,v) = (b_k, rcp);
      * per-channel weights: t = fp32(acc) + fp32(b_k / aws_k) (``vdivps`` +
        ``vaddps``) -> (u,v) = (fp32(b_k/aws_k), 1.0), which fmaf reproduces.
    aws_k = fp32(s_x * s_w,k); mult_k = fp32(aws_k / s_y)."""
    s_w = np.atleast_1d(np.asarray(s_w, F32))
    bias = np.asarray(bias, F32)
    aws = (F32(s_x) * s_w).astype(F32)
    mult = (aws / F32(s_y)).astype(F32)
    if aws.size == 1:
        rcp = F32(1.0) / aws[0]
        u = bias.copy()
        v = np.full(bias.shape, rcp, F32)
        mult = np.full(bias.shape, mult[0], F32)
    else:
        u = (bias / aws).astype(F32)
        v = np.ones(bias.shape, F32)
    return u, v, mult


def requantize(acc, u, v, mult, zp_y, relu):
    """ReQuantizeOutput (OutputProcessing-inl.h:76-127, vector form):
    y = clamp(rne(fp32(fmaf(u_k, v_k, fp32(acc)) * mult_k)) + zp_y, relu ? zp_y : 0, 255).
    ``acc`` has the output channel as its last axis."""
    raw = np.asarray(acc, np.int32).astype(F32)
    t = fmaf(np.broadcast_to(np.asarray(u, F32), raw.shape),
             np.broadcast_to(np.asarray(v, F32), raw.shape), raw)
    ab = (t * np.asarray(mult, F32)).astype(F32)
    r = np.rint(ab).astype(np.int64) + int(zp_y)
    lo = int(zp_y) if relu else 0
    return np.clip(r, lo, 255).astype(np.uint8)


# --------------------------------------------------------------------------- A5
def conv3x3_acc_nhwc(qx, zx, qw, zw=0):
    """Exact int32 accumulator of a 3x3/pad-1/stride-1 conv:
    acc[n,h,w,k] = sum_{r,s,c} (q_x - z_x) * (q_w - z_w), with the padding at
    q = z_x (FBGEMM im2col pads with the activation zero point).
    qx: [N,H,W,C] u8 NHWC; qw: [K,3,3,C] s8 (OHWI)."""
    n, h, w, c = qx.shape
    k = qw.shape[0]
    x = qx.astype(np.int32) - int(zx)
    xp = np.zeros((n, h + 2, w + 2, c), np.int32)
    xp[:, 1:h + 1, 1:w + 1, :] = x
    wt = qw.astype(np.int32) - np.asarray(zw, np.int32).reshape(-1, 1, 1, 1)
    acc = np.zeros((n, h, w, k), np.int64)
    for r in range(3):
        for s in range(3):
            patch = xp[:, r:r + h, s:s + w, :].reshape(-1, c).astype(np.int64)
            acc += (patch @ wt[:, r, s, :].T.astype(np.int64)).reshape(n, h, w, k)
    return acc.astype(np.int32)


def conv3x3_q(qx, zx, qw, u, v, mult, zp_y, relu):
    """Quantized conv2d (+ReLU) with FBGEMM requant: u8 NHWC out."""
    return requantize(conv3x3_acc_nhwc(qx, zx, qw), u, v, mult, zp_y, relu)


# -------------------------------------------------------------------------- A10
def maxpool2x2_nhwc(q):
    """nn.MaxPool2d(2, 2) — exact in either the u8 or the fp32 domain."""
    n, h, w, c = q.shape
    return q.reshape(n, h // 2, 2, w // 2, 2, c).max(axis=(2, 4))


# -------------------------------------------------------------------------- A9
def linear_acc(qx, zx, qw, zw=0):
    """acc[m,n] = sum_k (q_x - z_x) * (q_w - z_w)."""
    x = qx.astype(np.int64) - int(zx)
    wt = qw.astype(np.int64) - np.asarray(zw, np.int64).reshape(-1, 1)
    return (x @ wt.T).astype(np.int32)


def linear_q(qx, zx, qw, u, v, mult, zp_y, relu):
    return requantize(linear_acc(qx, zx, qw), u, v, mult, zp_y, relu)


# -------------------------------------------------------------------------- A8
def choose_qparams_dynamic(xmin, xmax, qmin=0, qmax=255, reduce_range=True):
    """ATen ChooseQuantizationParams (QuantUtils.h:70-185), preserve_sparsity=False,
    force_scale_power_of_two=False — double-precision scale, nudged zero point.
    Returns (scale as fp32, zero_point)."""
    if reduce_range:
        qmin, qmax = qmin // 2, qmax // 2
    mn = min(F32(xmin), F32(0.0))
    mx = max(F32(xmax), F32(0.0))
    scale = (float(mx) - float(mn)) / (qmax - qmin)
    if F32(scale) == 0.0 or np.isinf(F32(1.0) / F32(scale)):
        scale = 0.1
    small = 6.1e-5
    if scale < float(F32(small)):
        org = scale
        scale = float(F32(small))
        if mn == 0.0:
            mx = F32(F32(small) * (qmax - qmin))
        elif mx == 0.0:
            mn = F32(-F32(small) * (qmax - qmin))
        else:
            amp = F32(F32(small) / F32(org))
            mn = F32(mn * amp)
            mx = F32(mx * amp)
    zfm = qmin - float(mn) / scale
    zfx = qmax - float(mx) / scale
    efm = abs(qmin) - abs(float(mn) / scale)
    efx = abs(qmax) - abs(float(mx) / scale)
    z0 = zfm if efm < efx else zfx
    if z0 < qmin:
        zp = qmin
    elif z0 > qmax:
        zp = qmax
    else:
        zp = int(np.rint(z0))
    return F32(scale), zp


def quantize_legacy_fma(x, scale, zero_point, qmax=255):
    """fbgemm::QuantizeAvx2<uint8_t, LEGACY=true> (the input packing of the
    dynamic Linear, PackAWithQuantRowOffset): q = clamp(rne(fmaf(x, fp32(1/s),
    fp32(zp))), 0, qmax) — read from the compiled kernel in the torch wheel
    (vdivss, vfmadd132ps, vminps, vcvtps2dq)."""
    x = np.asarray(x, F32)
    inv = F32(1.0) / F32(scale)
    t = fmaf(x, np.full(x.shape, inv, F32), np.full(x.shape, F32(zero_point), F32))
    t = np.minimum(t, F32(qmax))
    return np.clip(np.rint(t), 0, qmax).astype(np.uint8)


def linear_dynamic(x, qw, s_w, bias, reduce_range=True, xrange=None):
    """quantized::linear_dynamic (FBGEMM; torch/ao/nn/quantized/dynamic/modules/
    linear.py:50-67): per-call qparams from the batch's min/max
    (ChooseQuantizationParams, qrange [0,127] with reduce_range), LEGACY
    quantize, exact int GEMM, then ReQuantizeForFloat, which the compiled
    ``requantizeForFloatAvx2`` FMA-contracts: y = fmaf(fp32(acc), fp32(s_x*s_w), b).
    ``xrange=(min, max)`` overrides the batch range (a shard of a larger batch
    quantized with the whole batch's range)."""
    x = np.asarray(x, F32)
    lo, hi = (x.min(), x.max()) if xrange is None else xrange
    s_x, z_x = choose_qparams_dynamic(lo, hi, reduce_range=reduce_range)
    qx = quantize_legacy_fma(x, s_x, z_x)
    acc = linear_acc(qx, z_x, qw)
    s_w = np.atleast_1d(np.asarray(s_w, F32))
    aws = (F32(s_x) * s_w).astype(F32)
    a = acc.astype(F32)
    b = np.zeros(a.shape[1], F32) if bias is None else np.asarray(bias, F32)
    return fmaf(a, np.broadcast_to(aws, a.shape), np.broadcast_to(b, a.shape))


# ------------------------------------------------------------------------- A11
def argmax_rows(x):
    """torch.argmax / topk(1) tie rule: lowest index of the maximum."""
    return np.argmax(np.asarray(x), axis=1).astype(np.int64)


# ----------------------------------------------------------- whole-net (A0)
def nchw_to_nhwc(x):
    return np.ascontiguousarray(np.transpose(x, (0, 2, 3, 1)))


def flatten_perm_nhwc_to_nchw(c=256, h=4, w=4):
    """Index map p such that flat_nchw = flat_nhwc[p] ... used to permute fc1
    columns: W_nhwc[:, j_nhwc] = W_nchw[:, p[j_nhwc]]  (baseline_model.py:78)."""
    idx = np.arange(c * h * w).reshape(c, h, w)  # NCHW flat index at (c,h,w)
    return np.ascontiguousarray(np.transpose(idx, (1, 2, 0))).reshape(-1)


def static_int8_forward(x_nchw, qm, keep=False):
    """Full static-int8 SimpleConvNet forward.

    ``qm`` is a dict of the quantized model (see ``oracle/make_golden.py`` and
    ``qconvnet.qmodel.QuantizedConvNet.to_oracle_dict``):
      in_scale, in_zp, conv{i}_{w,u,v,mult,zp,scale}, fc1_*, fc2_*.
    Returns (logits_fp32 [N,10], q_logits u8 [N,10], intermediates)."""
    inter = {}
    q = quantize_per_tensor(nchw_to_nhwc(np.asarray(x_nchw, F32)), qm["in_scale"], qm["in_zp"])
    inter["q_in"] = q
    zx = qm["in_zp"]
    for i in range(1, 7):
        p = f"conv{i}_"
        q = conv3x3_q(q, zx, qm[p + "w"], qm[p + "u"], qm[p + "v"], qm[p + "mult"],
                      qm[p + "zp"], True)
        zx = qm[p + "zp"]
        if i in (2, 4, 6):
            q = maxpool2x2_nhwc(q)
        if keep:
            inter[f"conv{i}"] = q
    flat = q.reshape(q.shape[0], -1)  # NHWC flatten; fc1_w columns are pre-permuted
    q = linear_q(flat, zx, qm["fc1_w"], qm["fc1_u"], qm["fc1_v"], qm["fc1_mult"], qm["fc1_zp"], True)
    inter["fc1"] = q
    q = linear_q(q, qm["fc1_zp"], qm["fc2_w"], qm["fc2_u"], qm["fc2_v"], qm["fc2_mult"],
                 qm["fc2_zp"], False)
    logits = dequantize(q, qm["fc2_scale"], qm["fc2_zp"])
    return logits, q, inter


# ------------------------------------------- ResNet-style blocks
# Reference: models/custom_quantization_model.py:60-148 (CustomQuantizedBottleneck,
# CustomQuantizedResNet50) with torchvision's ResNet-50 topology (stem 7x7/2 conv,
# 3x3/2 maxpool, [3,4,6,3] bottlenecks with the stride on the 3x3 conv and a
# 1x1 strided downsample, global average pool, fc).  Static int8 semantics as in
# static_int8_forward: BN folded into each conv, ReLU fused into the requant,
# every activation u8 per-tensor affine; the residual join dequantizes both
# operands and adds in fp32 (custom_quantization_model.py:94-101) before the
# ReLU and the next stage's QuantStub.
def conv_acc_nhwc(qx, zx, qw, stride=(1, 1), pad=(0, 0)):
    """Exact int32 accumulator of a general conv (FBGEMM im2col pads with
    q = z_x): acc[n,oy,ox,k] = sum_{r,s,c} (q_x - z_x) * q_w[k,c,r,s].
    qx: [N,H,W,C] u8; qw: OIHW s8 (symmetric weights, zp 0).  The products are
    summed in float64 — exact, since |sum| < 2^53 for any K below 2^37."""
    n, h, w, c = qx.shape
    k, c2, kh, kw = qw.shape
    assert c2 == c, (c2, c)
    sy, sx = stride
    py, px = pad
    oh, ow = (h + 2 * py - kh) // sy + 1, (w + 2 * px - kw) // sx + 1
    xp = np.zeros((n, h + 2 * py, w + 2 * px, c), np.float64)
    xp[:, py:py + h, px:px + w, :] = qx.astype(np.float64) - float(zx)
    wt = qw.astype(np.float64)
    acc = np.zeros((n * oh * ow, k), np.float64)
    for r in range(kh):
        for s in range(kw):
            patch = xp[:, r:r + sy * (oh - 1) + 1:sy, s:s + sx * (ow - 1) + 1:sx, :]
            acc += patch.reshape(-1, c) @ wt[:, :, r, s].T
    return acc.reshape(n, oh, ow, k).astype(np.int64).astype(np.int32)


def conv_q(qx, zx, qw, u, v, mult, zp_y, relu, stride=(1, 1), pad=(0, 0)):
    """QuantizedConv2d / QuantizedConvReLU2d, any kernel/stride/padding."""
    return requantize(conv_acc_nhwc(qx, zx, qw, stride, pad), u, v, mult, zp_y, relu)


def add_relu_q(qa, sa, za, qb, sb, zb, s_out, z_out, relu=True):
    """Residual join: out.dequantize() + identity.dequantize() in fp32, ReLU,
    then quantize_per_tensor with the next stage's qparams
    (custom_quantization_model.py:94-101)."""
    s = (dequantize(qa, sa, za) + dequantize(qb, sb, zb)).astype(F32)
    if relu:
        s = np.maximum(s, F32(0.0))
    return quantize_per_tensor(s, s_out, z_out)


def maxpool3x3s2_nhwc(q):
    """nn.MaxPool2d(3, 2, padding=1) (the ResNet stem); padding never wins."""
    n, h, w, c = q.shape
    oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    xp = np.zeros((n, h + 2, w + 2, c), q.dtype)
    xp[:, 1:h + 1, 1:w + 1, :] = q
    out = np.zeros((n, oh, ow, c), q.dtype)
    for r in range(3):
        for s in range(3):
            out = np.maximum(out, xp[:, r:r + 2 * (oh - 1) + 1:2, s:s + 2 * (ow - 1) + 1:2, :])
    return out


def avgpool_q(q, z_x):
    """AdaptiveAvgPool2d(1) on a quantized NHWC map, qparams kept: torch's
    quantized adaptive_avg_pool2d (ATen quantized/cpu adaptive avg pool,
    probed bit-exact on torch 2.10 fbgemm, 2x2 and 7x7 maps, ties included):
    acc = sum_q - HW*z, q = clamp(z + rne(fp32(acc) * fp32(1/HW)), 0, 255)."""
    n, h, w, c = q.shape
    hw = h * w
    acc = q.reshape(n, hw, c).astype(np.int64).sum(1) - hw * int(z_x)
    t = (acc.astype(F32) * (F32(1.0) / F32(hw))).astype(F32)
    return np.clip(np.rint(t).astype(np.int64) + int(z_x), 0, 255).astype(np.uint8)


def stem_pack(x_nchw, scale, zp):
    """Definition of qcn_stem_pack_f32_nchw (QuantStub + the row im2col of the
    7x7/2/3 stem): [N,H,OW,32] with byte 3*s+c = q(x[n,c,iy,2*ox-3+s])."""
    q = quantize_per_tensor(nchw_to_nhwc(np.asarray(x_nchw, F32)), scale, zp)
    n, h, w, c = q.shape
    ow = (w - 1) // 2 + 1
    xp = np.full((n, h, w + 6, c), zp, np.uint8)
    xp[:, :, 3:3 + w, :] = q
    out = np.full((n, h, ow, 32), zp, np.uint8)
    for s in range(7):
        out[:, :, :, 3 * s:3 * s + c] = xp[:, :, s:s + 2 * (ow - 1) + 1:2, :]
    return out


def _layer_q(q, zx, e, relu):
    u, v, mult = requant_constants(e["s_x"], e["s_w"], e["s_y"], e["b"])
    return conv_q(q, zx, e["w"], u, v, mult, e["z_y"], relu, tuple(e["stride"]), tuple(e["pad"]))


def bottleneck_int8_forward(q, blk):
    """One bottleneck block on u8 NHWC (zero point blk['c1']['z_x'])."""
    zx = blk["c1"]["z_x"]
    y = _layer_q(q, zx, blk["c1"], True)
    y = _layer_q(y, blk["c2"]["z_x"], blk["c2"], True)
    y = _layer_q(y, blk["c3"]["z_x"], blk["c3"], False)
    if blk.get("ds") is not None:
        idn = _layer_q(q, zx, blk["ds"], False)
        si, zi = blk["ds"]["s_y"], blk["ds"]["z_y"]
    else:
        idn, si, zi = q, blk["c1"]["s_x"], zx
    so, zo = blk["out"]
    return add_relu_q(y, blk["c3"]["s_y"], blk["c3"]["z_y"], idn, si, zi, so, zo, True)


def resnet_int8_forward(x_nchw, spec, keep=False):
    """Static-int8 ResNet forward (stem, maxpool, bottlenecks, avgpool, fc).
    ``spec``: see qconvnet.resnet.build_spec.  Returns (logits fp32, inter)."""
    inter = {}
    s_in, z_in = spec["in"]
    q = quantize_per_tensor(nchw_to_nhwc(np.asarray(x_nchw, F32)), s_in, z_in)
    q = _layer_q(q, z_in, spec["stem"], True)
    q = maxpool3x3s2_nhwc(q)
    if keep:
        inter["stem"] = q
    for i, blk in enumerate(spec["blocks"]):
        q = bottleneck_int8_forward(q, blk)
        if keep:
            inter[f"block{i}"] = q
    last = spec["blocks"][-1]["out"] if spec["blocks"] else (spec["stem"]["s_y"], spec["stem"]["z_y"])
    q = avgpool_q(q, last[1])   # qparams kept: the fc's input qparams are `last`
    inter["pool"] = q
    fc = spec["fc"]
    u, v, mult = requant_constants(fc["s_x"], fc["s_w"], fc["s_y"], fc["b"])
    qy = linear_q(q, fc["z_x"], fc["w"], u, v, mult, fc["z_y"], False)
    return dequantize(qy, fc["s_y"], fc["z_y"]), inter


# ----------------------------------------------- §8(f)2, reference semantics
def bn_eval_constants(mean, var, gamma, beta, eps=1e-5):
    """ATen CPU batch_norm (eval) as the torch 2.10 wheel computes it
    (batch_norm_kernel.cpp batch_norm_cpu_collect_linear_and_constant_terms,
    probed bit-exact here on contiguous and channels-last maps):
    invstd = fp32(1 / sqrt(fp32(var + eps))), alpha = fp32(invstd * gamma),
    beta' = fmaf(-mean, alpha, beta); the map is y = fmaf(x, alpha, beta')."""
    var = np.asarray(var, F32)
    invstd = (F32(1.0) / np.sqrt((var + F32(eps)).astype(F32))).astype(F32)
    alpha = (invstd * np.asarray(gamma, F32)).astype(F32)
    return alpha, fmaf(-np.asarray(mean, F32), alpha, np.asarray(beta, F32))


def bn_eval_nhwc(x, alpha, beta):
    return fmaf(x, alpha[None, None, None, :], beta[None, None, None, :])


def relu_f32(x):
    """torch.relu / F.relu on fp32: x where not x < 0, so -0.0 stays -0.0
    (np.maximum(-0.0, 0.0) would return +0.0)."""
    return np.where(x < 0, F32(0.0), x).astype(F32)


def maxpool3x3s2_f32_nhwc(x):
    """nn.MaxPool2d(3, 2, padding=1) on fp32 (padding = -inf)."""
    n, h, w, c = x.shape
    oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    xp = np.full((n, h + 2, w + 2, c), -np.inf, F32)
    xp[:, 1:h + 1, 1:w + 1, :] = x
    out = np.full((n, oh, ow, c), -np.inf, F32)
    for r in range(3):
        for s in range(3):
            out = np.maximum(out, xp[:, r:r + 2 * (oh - 1) + 1:2, s:s + 2 * (ow - 1) + 1:2, :])
    return out


def avgpool_f32_nhwc(x):
    """AdaptiveAvgPool2d(1) on an fp32 channels-last map (ATen
    cpu_adaptive_avg_pool channels-last kernel): sequential fp32 sum over the
    window in row-major order, then fp32(sum / (H*W))."""
    n, h, w, c = x.shape
    acc = np.zeros((n, c), F32)
    for i in range(h):
        for j in range(w):
            acc = (acc + x[:, i, j, :]).astype(F32)
    return (acc / F32(h * w)).astype(F32)


def _qdq_conv(x_f32, e):
    """QuantStub -> int8 conv (requant to the conv's output qparams, no ReLU)
    -> DeQuantStub -> BN (fp32)."""
    q = quantize_per_tensor(x_f32, e["s_x"], e["z_x"])
    u, v, mult = requant_constants(e["s_x"], e["s_w"], e["s_y"], e["b"])
    y = conv_q(q, e["z_x"], e["w"], u, v, mult, e["z_y"], False, tuple(e["stride"]), tuple(e["pad"]))
    return y, bn_eval_nhwc(dequantize(y, e["s_y"], e["z_y"]), *e["bn"])


def resnet_qdq_forward(x_nchw, spec, keep=False):
    """CustomQuantizedResNet50 with live per-layer stubs
    (custom_quantization_model.py:60-143): fp32 NHWC activations between the
    layers, each conv quantized at its own stub.  ``spec`` layout:
    qconvnet.resnet_qdq.build_spec.  Returns (logits fp32, inter) — inter
    holds every conv's u8 output and every block's fp32 output."""
    inter = {}
    x = nchw_to_nhwc(np.asarray(x_nchw, F32))
    y, f = _qdq_conv(x, spec["stem"])
    inter["stem.q"] = y
    x = maxpool3x3s2_f32_nhwc(relu_f32(f))
    inter["stem"] = x
    for i, blk in enumerate(spec["blocks"]):
        y1, f = _qdq_conv(x, blk["c1"])
        y2, f = _qdq_conv(relu_f32(f), blk["c2"])
        y3, out = _qdq_conv(relu_f32(f), blk["c3"])
        idn = x
        if blk.get("ds") is not None:
            yd, idn = _qdq_conv(x, blk["ds"])
            inter[f"block{i}.ds"] = yd
        x = relu_f32((out + idn).astype(F32))
        inter.update({f"block{i}.c1": y1, f"block{i}.c2": y2, f"block{i}.c3": y3, f"block{i}": x})
    p = avgpool_f32_nhwc(x)
    inter["pool"] = p
    fc = spec["fc"]
    q = quantize_per_tensor(p, fc["s_x"], fc["z_x"])
    u, v, mult = requant_constants(fc["s_x"], fc["s_w"], fc["s_y"], fc["b"])
    qy = linear_q(q, fc["z_x"], fc["w"], u, v, mult, fc["z_y"], False)
    inter["fc.q"] = qy
    return dequantize(qy, fc["s_y"], fc["z_y"]), inter
