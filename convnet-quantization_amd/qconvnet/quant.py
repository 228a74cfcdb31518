"""Host-side quantization arithmetic of the product (one-time, at quantize()):
observer qparams, BN folding, weight quantization, and the fp32 epilogue
constants the HIP kernels consume.

Every function reproduces torch.ao / FBGEMM bit for bit (the committed golden
vectors in tests/golden/ pin it; tests/test_host_quant.py checks it):

* qparams_affine / qparams_symmetric — MinMaxObserver._calculate_qparams
  (torch/ao/quantization/observer.py:349-427);
* fold_bn — torch.nn.utils.fusion.fuse_conv_bn_weights / fuse_linear_bn_weights
  (torch/nn/utils/fusion.py:56-101, 156-186), called by the reference at
  /root/reference/models/custom_quantization_model.py:180-190 and
  /root/reference/models/dynamic_ptq_model.py:289-299;
* quantize_weight — the weight quantization done by from_float;
* epilogue_constants — FBGEMM ReQuantizeOutput's fp32 constants
  (torch/include/fbgemm/OutputProcessing-inl.h:76-127, vector form).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
EPS = F32(np.finfo(np.float32).eps)


def qparams_affine(min_val, max_val, qmin=0, qmax=255):
    """quint8 per_tensor_affine: scale = (max+ - min-)/(qmax-qmin) (fp32, >= eps),
    zp = clamp(qmin - rne(min- / scale))."""
    mn = min(F32(min_val), F32(0.0))
    mx = max(F32(max_val), F32(0.0))
    scale = max(F32(F32(mx - mn) / F32(qmax - qmin)), EPS)
    zp = qmin - int(np.rint(F32(mn / scale)))
    return F32(scale), int(min(max(zp, qmin), qmax))


def qparams_symmetric(min_val, max_val):
    """qint8 per_tensor/per_channel_symmetric: scale = max(|min-|, max+)/127.5, zp = 0."""
    mn = np.minimum(np.asarray(min_val, F32), F32(0.0))
    mx = np.maximum(np.asarray(max_val, F32), F32(0.0))
    amax = np.maximum(-mn, mx)
    return np.maximum((amax / F32(127.5)).astype(F32), EPS).astype(F32)


def fold_bn(w, b, mean, var, gamma, beta, eps=1e-5):
    """w' = w * (gamma * rsqrt(var + eps)); b' = (b - mean) * rsqrt * gamma + beta."""
    w = np.asarray(w, F32)
    b = np.zeros(w.shape[0], F32) if b is None else np.asarray(b, F32)
    rsq = (F32(1.0) / np.sqrt((np.asarray(var, F32) + F32(eps)).astype(F32))).astype(F32)
    s = (np.asarray(gamma, F32) * rsq).astype(F32)
    wf = (w * s.reshape((-1,) + (1,) * (w.ndim - 1))).astype(F32)
    bf = ((((b - np.asarray(mean, F32)).astype(F32) * rsq).astype(F32) * np.asarray(gamma, F32)).astype(F32)
          + np.asarray(beta, F32)).astype(F32)
    return wf, bf


def fold_linear_bn(w, b, mean, var, gamma, beta, eps=1e-5):
    """fuse_linear_bn_weights (fusion.py:156-186) — note the different bias order:
    s = gamma * rsqrt(var + eps); w' = w * s; b' = (b - mean) * s + beta."""
    w = np.asarray(w, F32)
    b = np.zeros(w.shape[0], F32) if b is None else np.asarray(b, F32)
    rsq = (F32(1.0) / np.sqrt((np.asarray(var, F32) + F32(eps)).astype(F32))).astype(F32)
    s = (np.asarray(gamma, F32) * rsq).astype(F32)
    wf = (w * s.reshape(-1, 1)).astype(F32)
    bf = (((b - np.asarray(mean, F32)).astype(F32) * s).astype(F32) + np.asarray(beta, F32)).astype(F32)
    return wf, bf


def bn_eval_affine(mean, var, gamma, beta, eps=1e-5):
    """Per-channel (alpha, beta') of an inference BatchNorm in ATen's CPU op
    order (torch 2.10 batch_norm with training=False, probed bit-exact on the
    host): invstd = fp32(1 / sqrt(fp32(var + eps))), alpha = fp32(invstd *
    gamma), beta' = fma(-mean, alpha, beta); then y = fma(x, alpha, beta')."""
    f32 = np.float32
    mean, var = np.asarray(mean, f32), np.asarray(var, f32)
    gamma, beta = np.asarray(gamma, f32), np.asarray(beta, f32)
    invstd = (f32(1.0) / np.sqrt(var + f32(eps))).astype(f32)
    alpha = (invstd * gamma).astype(f32)
    return alpha, fmaf_host(-mean, alpha, beta)


def fmaf_host(a, b, c):
    """fl32(a*b + c) with one rounding, vectorised on the host: a*b is exact
    in float64, the sum rounds once to float64, and when that double lands
    exactly on an fp32 midpoint the TwoSum error term decides the direction
    (the one case where double rounding would differ)."""
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
    nxt = np.nextafter(r, np.where(diff > 0, np.inf, -np.inf).astype(F32))
    mid = (diff != 0) & (s == (r64 + nxt.astype(np.float64)) * 0.5)
    fix = mid & (e != 0) & (np.sign(e) == np.sign(diff))
    return np.where(fix, nxt, r).astype(F32)


def quantize_weight(w, scale):
    """q = clamp(rne(w * fp32(1/s)), -128, 127), per tensor (scalar scale) or per
    output channel (vector scale)."""
    w = np.asarray(w, F32)
    scale = np.asarray(scale, F32)
    if scale.ndim == 0 or scale.size == 1:
        inv = (F32(1.0) / F32(scale.reshape(-1)[0]))
        return np.clip(np.rint((w * inv).astype(F32)), -128, 127).astype(np.int8)
    inv = (F32(1.0) / scale).astype(F32).reshape((-1,) + (1,) * (w.ndim - 1))
    return np.clip(np.rint((w * inv).astype(F32)), -128, 127).astype(np.int8)


def epilogue_constants(s_x, s_w, s_y, bias):
    """(u, v, mult) per output channel for  t = fmaf(u, v, fp32(acc)); ab = t * mult.

    FBGEMM's compiled vector epilogue (requantizeOutputProcessingAvx2 in the torch
    wheel) FMA-contracts the per-tensor bias term with rcp = fp32(1.0f / aws), and
    divides per channel: per-tensor -> (b, rcp); per-channel -> (fp32(b/aws), 1)."""
    s_w = np.atleast_1d(np.asarray(s_w, F32))
    bias = np.asarray(bias, F32)
    aws = (F32(s_x) * s_w).astype(F32)
    mult = (aws / F32(s_y)).astype(F32)
    if aws.size == 1:
        rcp = F32(F32(1.0) / aws[0])
        return bias.copy(), np.full(bias.shape, rcp, F32), np.full(bias.shape, mult[0], F32)
    return (bias / aws).astype(F32), np.ones(bias.shape, F32), mult


def nhwc_flatten_perm(c=256, h=4, w=4):
    """perm such that W_nhwc = W_nchw[:, perm]: fc1 consumes the NHWC-flattened
    pooled tensor while keeping baseline_model.py:78's NCHW flatten semantics."""
    idx = np.arange(c * h * w).reshape(c, h, w)
    return np.ascontiguousarray(np.transpose(idx, (1, 2, 0))).reshape(-1)
