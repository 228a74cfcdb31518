"""Tensor-level wrappers over the C ABI (torch tensors are plumbing: device
memory + the current HIP stream).  Every op launches on
``torch.cuda.current_stream()`` and never synchronizes, so sequences of them
can be captured in a HIP graph (torch.cuda.CUDAGraph is hipGraph on ROCm).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from ._lib import QDQ, check


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _need(t, dtype, name):
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a device tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous tensor")


def lib():
    return _lib.load()


# ----------------------------------------------------------------- A1 / A7
def quantize(x, scale, zero_point, nhwc=True, out=None):
    """fp32 NCHW -> u8 (NHWC if nhwc) with aten quantize_per_tensor numerics."""
    _need(x, torch.float32, "quantize.x")
    n, c, h, w = x.shape
    if out is None:
        shape = (n, h, w, c) if nhwc else (n, c, h, w)
        out = torch.empty(shape, dtype=torch.uint8, device=x.device)
    check(lib().qcn_quantize_f32_u8(_ptr(x), _ptr(out), n, c, h, w, int(bool(nhwc)),
                                    float(scale), int(zero_point), _stream()), "quantize")
    return out


def dequantize(q, scale, zero_point, out=None):
    _need(q, torch.uint8, "dequantize.q")
    if out is None:
        out = torch.empty(q.shape, dtype=torch.float32, device=q.device)
    check(lib().qcn_dequantize_u8_f32(_ptr(q), _ptr(out), q.numel(), float(scale),
                                      int(zero_point), _stream()), "dequantize")
    return out


# ---------------------------------------------------------------------- A2
class MinMaxObserver:
    """Device-side running min/max (MinMaxObserver.forward semantics)."""

    def __init__(self, device="cuda"):
        self.state = torch.empty(2, dtype=torch.float32, device=device)
        self.reset()

    def reset(self):
        check(lib().qcn_minmax_reset(_ptr(self.state), _stream()), "minmax_reset")

    def __call__(self, x):
        _need(x, torch.float32, "minmax.x")
        check(lib().qcn_minmax_f32(_ptr(x), x.numel(), _ptr(self.state), _stream()), "minmax")
        return x

    def values(self):
        v = self.state.cpu().numpy()
        return np.float32(v[0]), np.float32(v[1])


# --------------------------------------------------------------- A10 / A11
def maxpool2x2(x):
    _need(x, torch.uint8, "maxpool.x")
    n, h, w, c = x.shape
    out = torch.empty((n, h // 2, w // 2, c), dtype=torch.uint8, device=x.device)
    check(lib().qcn_maxpool2x2_u8_nhwc(_ptr(x), n, h, w, c, _ptr(out), _stream()), "maxpool")
    return out


def argmax(x):
    _need(x, torch.float32, "argmax.x")
    rows, cols = x.shape
    out = torch.empty(rows, dtype=torch.int64, device=x.device)
    check(lib().qcn_argmax_f32(_ptr(x), rows, cols, _ptr(out), _stream()), "argmax")
    return out


def channel_affine(x, alpha, beta, relu=False, out=None):
    """Inference BatchNorm1d (+ReLU) on [rows, cols] fp32: fma(x, alpha, beta)
    per column (alpha / beta from quant.bn_eval_affine)."""
    _need(x, torch.float32, "channel_affine.x")
    rows, cols = x.shape
    if out is None:
        out = torch.empty_like(x)
    check(lib().qcn_channel_affine_f32(_ptr(x), rows, cols, _ptr(alpha), _ptr(beta), int(bool(relu)),
                                       _ptr(out), _stream()), "channel_affine")
    return out


# ------------------------------------------------------------------- packing
def pack_conv3x3(w_oihw: np.ndarray):
    """Host packing of s8 OIHW weights -> (packed bytes, wsum int32)."""
    w = np.ascontiguousarray(w_oihw, dtype=np.int8)
    cout, cin = w.shape[:2]
    out = np.empty(lib().qcn_conv3x3_packed_size(cin, cout), np.int8)
    wsum = np.empty(cout, np.int32)
    check(lib().qcn_pack_conv3x3_weight(w.ctypes.data, cout, cin, out.ctypes.data,
                                        wsum.ctypes.data), "pack_conv3x3")
    return out, wsum


def pack_conv1(w_oihw: np.ndarray):
    w = np.ascontiguousarray(w_oihw, dtype=np.int8)
    out = np.empty(64 * 32, np.int8)
    wsum = np.empty(64, np.int32)
    check(lib().qcn_pack_conv1_weight(w.ctypes.data, w.shape[0], out.ctypes.data,
                                      wsum.ctypes.data), "pack_conv1")
    return out, wsum


def qdq_struct(s1, z1, s2, z2):
    return QDQ(np.float32(s1), int(z1), np.float32(np.float32(1.0) / np.float32(s2)), int(z2))


# ------------------------------------------------------------- A5/A6 + A9
def conv3x3(x, x_zp, w_packed, cout, u, v, mult, corr, y_zp, relu, pool, qdq=None, out=None):
    _need(x, torch.uint8, "conv.x")
    n, h, w, cin = x.shape
    oh, ow = (h // 2, w // 2) if pool else (h, w)
    if out is None:
        out = torch.empty((n, oh, ow, cout), dtype=torch.uint8, device=x.device)
    check(lib().qcn_conv3x3_u8s8_nhwc(_ptr(x), n, h, w, cin, int(x_zp), _ptr(w_packed), cout,
                                      _ptr(u), _ptr(v), _ptr(mult), _ptr(corr), int(y_zp),
                                      int(bool(relu)), int(bool(pool)),
                                      C.byref(qdq) if qdq is not None else None, _ptr(out),
                                      _stream()), "conv3x3")
    return out


def conv1_f32(x, in_scale, in_zp, w1_packed, u, v, mult, corr, y_zp, relu, qdq=None, out=None,
              q_in=None):
    _need(x, torch.float32, "conv1.x")
    n, c, h, w = x.shape
    if c != 3 or h != w:
        raise ValueError("conv1_f32 expects [n,3,hw,hw]")
    if out is None:
        out = torch.empty((n, h, w, 64), dtype=torch.uint8, device=x.device)
    check(lib().qcn_conv1_f32_nchw(_ptr(x), n, h, float(in_scale), int(in_zp), _ptr(w1_packed),
                                   _ptr(u), _ptr(v), _ptr(mult), _ptr(corr), int(y_zp),
                                   int(bool(relu)), C.byref(qdq) if qdq is not None else None,
                                   _ptr(out), _ptr(q_in), _stream()), "conv1")
    return out


def conv12_fused(x, in_scale, in_zp, l1, l2, out=None):
    """conv1 (+quantize) and conv2 (+pool) of SimpleConvNet in one launch.
    ``l1``/``l2`` carry w, u, v, mult, corr, z_y, relu, qdq (and l2.z_x)."""
    _need(x, torch.float32, "conv12.x")
    n = x.shape[0]
    if tuple(x.shape[1:]) != (3, 32, 32):
        raise ValueError("conv12_fused expects [n,3,32,32]")
    if out is None:
        out = torch.empty((n, 16, 16, 64), dtype=torch.uint8, device=x.device)
    q1 = C.byref(l1.qdq) if l1.qdq is not None else None
    q2 = C.byref(l2.qdq) if l2.qdq is not None else None
    check(lib().qcn_conv12_fused_f32_nchw(
        _ptr(x), n, float(in_scale), int(in_zp), _ptr(l1.w), _ptr(l1.u), _ptr(l1.v), _ptr(l1.mult),
        _ptr(l1.corr), int(l1.z_y), int(bool(l1.relu)), q1, int(l2.z_x), _ptr(l2.w), _ptr(l2.u),
        _ptr(l2.v), _ptr(l2.mult), _ptr(l2.corr), int(l2.z_y), int(bool(l2.relu)), q2, _ptr(out),
        _stream()), "conv12_fused")
    return out


def conv_layers(layers, in_zp):
    """The six conv layers of SimpleConvNet (objects with w, u, v, mult, corr,
    z_x, z_y, relu, qdq) as the qcn_conv_layer_t array convnet_convs() takes.
    Built once per model: it holds the device pointers and the QDQ structs."""
    arr = (_lib.ConvLayer * 6)()
    for i, d in enumerate(layers):
        arr[i] = _lib.ConvLayer(_ptr(d.w), _ptr(d.u), _ptr(d.v), _ptr(d.mult), _ptr(d.corr),
                                int(in_zp) if i == 0 else int(d.z_x), int(d.z_y), int(bool(d.relu)),
                                C.pointer(d.qdq) if d.qdq is not None else None)
    return arr


def convnet_convs(x, in_scale, in_zp, layers, a2, a4, a6, kmajor=True):
    """QuantStub + conv1 .. conv6 in one persistent launch (conv6's pooled
    output chunk-major into a6 [128, n, 32] when kmajor, else NHWC
    [n, 4, 4, 256]).  ``layers``: conv_layers().
    Returns False when the launch does not apply (fewer than 4 images per
    CU, or mixed epilogue forms); the caller then runs the three launches."""
    _need(x, torch.float32, "convnet_convs.x")
    n = x.shape[0]
    if tuple(x.shape[1:]) != (3, 32, 32):
        raise ValueError("convnet_convs expects [n,3,32,32]")
    rc = lib().qcn_convnet_convs_f32_nchw(_ptr(x), n, float(in_scale), int(in_zp), layers, _ptr(a2),
                                          _ptr(a4), _ptr(a6), int(bool(kmajor)), _stream())
    if rc == _lib.QCN_ERR_UNSUPPORTED:
        return False
    check(rc, "convnet_convs")
    return True


def convs36(a2, layers, a4, a6, kmajor=True):
    """conv3 .. conv6 in one persistent launch of one-wave-per-SIMD
    workgroups (qcn_convs36_u8s8): a2 [n,16,16,64] u8 NHWC in, a4 written,
    conv6's pooled output into a6 (chunk-major [128, n, 32] when kmajor, else
    NHWC [n, 4, 4, 256]).  ``layers``: conv_layers() (its conv3 .. conv6
    entries are used).  Returns False when the launch does not apply (mixed
    epilogue forms)."""
    _need(a2, torch.uint8, "convs36.a2")
    n = a2.shape[0]
    if tuple(a2.shape[1:]) != (16, 16, 64):
        raise ValueError("convs36 expects a2 [n,16,16,64]")
    _need(a4, torch.uint8, "convs36.a4")
    _need(a6, torch.uint8, "convs36.a6")
    if a4.numel() != n * 8 * 8 * 128 or a6.numel() != n * 4096:
        raise ValueError("convs36: a4 / a6 sizes do not match the batch")
    l3 = C.cast(C.byref(layers, 2 * C.sizeof(_lib.ConvLayer)), C.POINTER(_lib.ConvLayer))
    rc = lib().qcn_convs36_u8s8(_ptr(a2), n, l3, _ptr(a4), _ptr(a6), int(bool(kmajor)), _stream())
    if rc == _lib.QCN_ERR_UNSUPPORTED:
        return False
    check(rc, "convs36")
    return True


def convnet_convs_form(n, in_scale, in_zp, layers, kmajor=True):
    """Host query (no launch, current device): 1 when convnet_convs() runs one
    image per workgroup for batch n, 2 the persistent form, 0 when it would
    return False (the three launches run instead)."""
    rc = lib().qcn_convnet_convs_form(int(n), float(in_scale), int(in_zp), layers, int(bool(kmajor)))
    if rc == _lib.QCN_ERR_UNSUPPORTED:
        return 0
    if rc < 0:
        check(rc, "convnet_convs_form")
    return rc


def linear_u8(x, x_zp, w, u, v, mult, corr, y_zp, relu, y_scale=0.0, want_fp32=False, out=None,
              out_f=None):
    _need(x, torch.uint8, "linear.x")
    m, k = x.shape
    n = w.shape[0]
    if out is None:
        out = torch.empty((m, n), dtype=torch.uint8, device=x.device)
    if want_fp32 and out_f is None:
        out_f = torch.empty((m, n), dtype=torch.float32, device=x.device)
    check(lib().qcn_linear_u8s8(_ptr(x), m, k, int(x_zp), _ptr(w), n, _ptr(u), _ptr(v), _ptr(mult),
                                _ptr(corr), int(y_zp), int(bool(relu)), _ptr(out),
                                _ptr(out_f) if want_fp32 else None, float(y_scale), _stream()),
          "linear_u8s8")
    return (out, out_f) if want_fp32 else out


def classifier_workspace(m, n1, device):
    """The head's int32 split-K partials (no initialisation needed)."""
    return torch.empty(lib().qcn_classifier_workspace_size(m, n1), dtype=torch.uint8, device=device)


def pack_fc_kmajor(w: np.ndarray):
    """s8 [n, k] -> chunk-major [k/32, n, 32] (the classifier head's fc1 layout)."""
    w = np.ascontiguousarray(w, dtype=np.int8)
    n, k = w.shape
    out = np.empty((k // 32, n, 32), np.int8)
    check(lib().qcn_pack_fc_kmajor(w.ctypes.data, n, k, out.ctypes.data), "pack_fc_kmajor")
    return out


def to_kmajor(x2d):
    """u8 [m, k] -> chunk-major [k/32, m, 32] (torch; tests and fallbacks)."""
    m, k = x2d.shape
    return x2d.view(m, k // 32, 32).permute(1, 0, 2).contiguous()


def from_kmajor(xk):
    """chunk-major [k/32, m, 32] -> [m, k]."""
    kc, m, _ = xk.shape
    return xk.permute(1, 0, 2).reshape(m, kc * 32)


def conv_pair(x, la, lb, out, kmajor=False):
    """conv A (no pool) + conv B (2x2 pool) of one block in one launch (A's
    output stays in LDS).  ``la``/``lb`` carry w, cout, u, v, mult, corr, z_x,
    z_y, relu, qdq.  Returns False when the block shape is not supported."""
    _need(x, torch.uint8, "conv_pair.x")
    n, h, w, cin = x.shape
    rc = lib().qcn_conv3x3_pair_u8s8(
        _ptr(x), n, h, cin, int(la.z_x), _ptr(la.w), la.cout, _ptr(la.u), _ptr(la.v), _ptr(la.mult),
        _ptr(la.corr), int(la.z_y), int(bool(la.relu)), C.byref(la.qdq) if la.qdq is not None else None,
        _ptr(lb.w), lb.cout, _ptr(lb.u), _ptr(lb.v), _ptr(lb.mult), _ptr(lb.corr), int(lb.z_y),
        int(bool(lb.relu)), C.byref(lb.qdq) if lb.qdq is not None else None, int(bool(kmajor)),
        _ptr(out), _stream())
    if rc == _lib.QCN_ERR_UNSUPPORTED:
        return False
    check(rc, "conv_pair")
    return True


def conv3x3_kmajor(x, x_zp, w_packed, cout, u, v, mult, corr, y_zp, relu, pool, out):
    """conv3x3 whose output is chunk-major [oh*ow*cout/32, n, 32] (conv6 -> fc1).
    Returns False when the shape is not supported (caller uses conv3x3)."""
    _need(x, torch.uint8, "conv_kmajor.x")
    n, h, w, cin = x.shape
    rc = lib().qcn_conv3x3_u8s8_kmajor(_ptr(x), n, h, w, cin, int(x_zp), _ptr(w_packed), cout,
                                       _ptr(u), _ptr(v), _ptr(mult), _ptr(corr), int(y_zp),
                                       int(bool(relu)), int(bool(pool)), _ptr(out), _stream())
    if rc == _lib.QCN_ERR_UNSUPPORTED:
        return False
    check(rc, "conv3x3_kmajor")
    return True


def classifier(xk, l1, l2, workspace, y1, y2, y2f):
    """Static fc1(+ReLU) -> fc2 -> dequantize head (two launches).  ``xk`` is the
    chunk-major fc1 input [k/32, m, 32]; ``l1``/``l2`` carry wk (chunk-major fc1
    weights) / w, u, v, mult, (l1) corr, z_y, relu and (l2) s_y.  Returns False
    when the shape is outside the kernel's envelope (caller falls back)."""
    _need(xk, torch.uint8, "classifier.x")
    kc, m, _ = xk.shape
    k = kc * 32
    rc = lib().qcn_classifier_u8s8(_ptr(xk), m, k, _ptr(l1.wk), l1.wk.shape[1], _ptr(l1.u), _ptr(l1.v),
                                   _ptr(l1.mult), _ptr(l1.corr), int(l1.z_y), int(bool(l1.relu)),
                                   _ptr(l2.w), l2.w.shape[0], _ptr(l2.u), _ptr(l2.v), _ptr(l2.mult),
                                   int(l2.z_y), int(bool(l2.relu)), float(l2.s_y), _ptr(workspace),
                                   _ptr(y1), _ptr(y2), _ptr(y2f), _stream())
    if rc == _lib.QCN_ERR_UNSUPPORTED:
        return False
    check(rc, "classifier")
    return True


def classifier_qdq(xk, l1, l2, workspace, y1, y2f):
    """QDQ head (BASELINE config 2): fc1 int8 -> requant -> dequantize ->
    ReLU -> fp32 fc2, two launches.  ``l1`` as for classifier() (wk, u, v,
    mult, corr, z_y, s_y); ``l2`` carries the fp32 w [n2, n1] and b.  Returns
    False outside the kernel's envelope (caller falls back)."""
    _need(xk, torch.uint8, "classifier_qdq.x")
    kc, m, _ = xk.shape
    rc = lib().qcn_classifier_qdq_u8s8(_ptr(xk), m, kc * 32, _ptr(l1.wk), l1.wk.shape[1], _ptr(l1.u),
                                       _ptr(l1.v), _ptr(l1.mult), _ptr(l1.corr), int(l1.z_y),
                                       float(l1.s_y), _ptr(l2.w), l2.w.shape[0], _ptr(l2.b),
                                       _ptr(workspace), _ptr(y1), _ptr(y2f), _stream())
    if rc == _lib.QCN_ERR_UNSUPPORTED:
        return False
    check(rc, "classifier_qdq")
    return True


def minmax_range(x, out=None):
    """[min, max] of a device fp32 tensor as a device float[2] (A2 kernel)."""
    _need(x, torch.float32, "minmax.x")
    if out is None:
        out = torch.empty(2, dtype=torch.float32, device=x.device)
    check(lib().qcn_minmax_reset(_ptr(out), _stream()), "minmax_reset")
    check(lib().qcn_minmax_f32(_ptr(x), x.numel(), _ptr(out), _stream()), "minmax")
    return out


def linear_dynamic(x, w, w_scale, wsum, bias, reduce_range=True, workspace=None, out=None,
                   minmax=None):
    """quantized::linear_dynamic on the device (fp32 in, fp32 out).  With
    ``minmax`` (device float[2]) the activation qparams come from that range
    instead of this batch's own (the sharded, batch-exact form)."""
    _need(x, torch.float32, "linear_dynamic.x")
    m, k = x.shape
    n = w.shape[0]
    if out is None:
        out = torch.empty((m, n), dtype=torch.float32, device=x.device)
    need = lib().qcn_linear_dynamic_workspace_size(m, k)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=x.device)
    per_channel = int(w_scale.numel() > 1)
    if minmax is None:
        check(lib().qcn_linear_dynamic_f32(_ptr(x), m, k, _ptr(w), n, _ptr(w_scale), per_channel,
                                           _ptr(wsum), _ptr(bias), int(bool(reduce_range)),
                                           _ptr(out), _ptr(workspace), _stream()), "linear_dynamic")
    else:
        _need(minmax, torch.float32, "linear_dynamic.minmax")
        check(lib().qcn_linear_dynamic_range_f32(_ptr(x), m, k, _ptr(w), n, _ptr(w_scale),
                                                 per_channel, _ptr(wsum), _ptr(bias),
                                                 int(bool(reduce_range)), _ptr(minmax), _ptr(out),
                                                 _ptr(workspace), _stream()), "linear_dynamic_range")
    return out


def linear_f32(x, w, b, relu_in=False, out=None):
    _need(x, torch.float32, "linear_f32.x")
    m, k = x.shape
    n = w.shape[0]
    if out is None:
        out = torch.empty((m, n), dtype=torch.float32, device=x.device)
    check(lib().qcn_linear_f32(_ptr(x), m, k, _ptr(w), n, _ptr(b), int(bool(relu_in)), _ptr(out),
                               _stream()), "linear_f32")
    return out


# ------------------------------------------------ ResNet blocks
def pack_conv_kmajor(w_oihw: np.ndarray):
    """s8 OIHW -> (chunk-major [kh*kw*cin/32, cout, 32] bytes, wsum int32)."""
    w = np.ascontiguousarray(w_oihw, dtype=np.int8)
    cout, cin, kh, kw = w.shape
    out = np.empty((kh * kw * cin // 32, cout, 32), np.int8)
    wsum = np.empty(cout, np.int32)
    check(lib().qcn_pack_conv_weight_kmajor(w.ctypes.data, cout, cin, kh, kw, out.ctypes.data,
                                            wsum.ctypes.data), "pack_conv_kmajor")
    return out, wsum


def stem_weight_rows(w_oihw: np.ndarray):
    """7x7 stem weights [k][3][7][7] -> the 7x1 conv over the packed rows
    (qcn_stem_pack_f32_nchw): [k][32][7][1], channel 3*s + c holds w[k][c][r][s]."""
    w = np.asarray(w_oihw)
    k, c, kh, kw = w.shape
    if c * kw > 32:
        raise ValueError("stem rows need c * kw <= 32")
    out = np.zeros((k, 32, kh, 1), w.dtype)
    out[:, :c * kw, :, 0] = np.transpose(w, (0, 3, 1, 2)).reshape(k, kw * c, kh)
    return out


def conv(x, x_zp, layer, out=None, resid=None, impl=None):
    """Generic quantized conv on u8 NHWC.  ``layer`` carries w (packed), cout,
    kh, kw, stride (sy, sx), pad (py, px), u, v, mult, corr, z_y, s_y, relu.
    ``resid=(r, s_r, z_r, s_out, z_out)`` fuses the bottleneck's residual join
    (GEMM kernel only).  impl: "gemm" (LDS-tiled, default) or "gen" (the
    register-direct kernel, a second implementation parity-tested beside it)."""
    _need(x, torch.uint8, "conv.x")
    n, h, w, cin = x.shape
    d = layer
    oh = (h + 2 * d.py - d.kh) // d.sy + 1
    ow = (w + 2 * d.px - d.kw) // d.sx + 1
    if out is None:
        out = torch.empty((n, oh, ow, d.cout), dtype=torch.uint8, device=x.device)
    impl = impl or "gemm"
    if impl == "gen" and resid is None:
        check(lib().qcn_conv_u8s8_nhwc(_ptr(x), n, h, w, cin, int(x_zp), _ptr(d.w), d.cout, d.kh,
                                       d.kw, d.sy, d.sx, d.py, d.px, _ptr(d.u), _ptr(d.v),
                                       _ptr(d.mult), _ptr(d.corr), int(d.z_y), int(bool(d.relu)),
                                       _ptr(out), _stream()), "conv")
        return out
    if resid is not None:
        r, s_r, z_r, s_o, z_o = resid
        _need(r, torch.uint8, "conv.resid")
        if tuple(r.shape) != tuple(out.shape):
            raise ValueError("residual operand shape differs from the conv output")
        rp, sy_ = _ptr(r), float(d.s_y)
    else:
        rp, sy_, s_r, z_r, s_o, z_o = None, 0.0, 0.0, 0, 0.0, 0
    check(lib().qcn_conv_gemm_u8s8_nhwc(_ptr(x), n, h, w, cin, int(x_zp), _ptr(d.w), d.cout, d.kh,
                                        d.kw, d.sy, d.sx, d.py, d.px, _ptr(d.u), _ptr(d.v),
                                        _ptr(d.mult), _ptr(d.corr), int(d.z_y), int(bool(d.relu)),
                                        rp, sy_, float(s_r), int(z_r), float(s_o), int(z_o),
                                        _ptr(out), _stream()), "conv_gemm")
    return out


def conv_join_reduce(x, x_zp, layer, resid, nxt, out=None, out2=None):
    """``conv(x, x_zp, layer, resid=resid)`` (the 64 -> 256 expand + residual
    join) and ``conv(result, resid[4], nxt)`` (the next block's 1x1 reduce,
    256 -> 64 or 128) in one launch (qcn_conv1x1_join_reduce_u8s8_nhwc);
    returns (joined, reduced), bit-identical to the two launches.  None when
    the library declines the shape (QCN_ERR_UNSUPPORTED)."""
    _need(x, torch.uint8, "conv_join_reduce.x")
    n, h, w, cin = x.shape
    d, e = layer, nxt
    if d.relu:   # the unfused path (conv with resid) rejects relu with a join too
        raise ValueError("conv_join_reduce: the joined conv takes no ReLU of its own")
    r, s_r, z_r, s_o, z_o = resid
    _need(r, torch.uint8, "conv_join_reduce.resid")
    if out is None:
        out = torch.empty((n, h, w, d.cout), dtype=torch.uint8, device=x.device)
    _need(out, torch.uint8, "conv_join_reduce.out")
    if tuple(out.shape) != (n, h, w, d.cout):
        raise ValueError("conv_join_reduce: out must be [n, h, w, cout]")
    if tuple(r.shape) != tuple(out.shape):
        raise ValueError("residual operand shape differs from the conv output")
    if out2 is None:
        out2 = torch.empty((n, h, w, e.cout), dtype=torch.uint8, device=x.device)
    _need(out2, torch.uint8, "conv_join_reduce.out2")
    if tuple(out2.shape) != (n, h, w, e.cout):
        raise ValueError("conv_join_reduce: out2 must be [n, h, w, next cout]")
    rc = lib().qcn_conv1x1_join_reduce_u8s8_nhwc(
        _ptr(x), n, h, w, cin, int(x_zp), _ptr(d.w), d.cout, _ptr(d.u), _ptr(d.v), _ptr(d.mult),
        _ptr(d.corr), int(d.z_y), _ptr(r), float(d.s_y), float(s_r), int(z_r), float(s_o), int(z_o),
        _ptr(out), _ptr(e.w), e.cout, _ptr(e.u), _ptr(e.v), _ptr(e.mult), _ptr(e.corr), int(e.z_y),
        int(bool(e.relu)), _ptr(out2), _stream())
    if rc == _lib.QCN_ERR_UNSUPPORTED:
        return None
    check(rc, "conv_join_reduce")
    return out, out2


def add_relu(a, sa, za, b, sb, zb, s_out, z_out, relu=True, out=None):
    _need(a, torch.uint8, "add.a")
    _need(b, torch.uint8, "add.b")
    if a.shape != b.shape:
        raise ValueError("add_relu operands differ in shape")
    if out is None:
        out = torch.empty_like(a)
    check(lib().qcn_add_relu_u8(_ptr(a), float(sa), int(za), _ptr(b), float(sb), int(zb), a.numel(),
                                float(s_out), int(z_out), int(bool(relu)), _ptr(out), _stream()),
          "add_relu")
    return out


def maxpool3x3s2(x, out=None):
    _need(x, torch.uint8, "maxpool3.x")
    n, h, w, c = x.shape
    if out is None:
        out = torch.empty((n, (h - 1) // 2 + 1, (w - 1) // 2 + 1, c), dtype=torch.uint8,
                          device=x.device)
    check(lib().qcn_maxpool3x3s2_u8_nhwc(_ptr(x), n, h, w, c, _ptr(out), _stream()), "maxpool3x3s2")
    return out


def stem_pack(x, scale, zp, out=None):
    _need(x, torch.float32, "stem.x")
    n, c, h, w = x.shape
    if c != 3:
        raise ValueError("stem_pack expects 3 input channels")
    if out is None:
        out = torch.empty((n, h, (w - 1) // 2 + 1, 32), dtype=torch.uint8, device=x.device)
    check(lib().qcn_stem_pack_f32_nchw(_ptr(x), n, h, w, float(scale), int(zp), _ptr(out),
                                       _stream()), "stem_pack")
    return out


def stem_fused(x, scale, zp, layer, out=None):
    """QuantStub -> 7x7/2 stem conv (+ReLU requant) -> 3x3/2 max-pool in one
    launch (qcn_resnet_stem_fused); ``layer`` as for conv() with the weights
    packed from stem_weight_rows.  Input [n,3,s,s] fp32, s in {224, 64}."""
    _need(x, torch.float32, "stem.x")
    n, c, h, w = x.shape
    d = layer
    if c != 3 or h != w or d.cout != 64:
        raise ValueError("stem_fused: 3-channel square input, 64 output channels")
    if out is None:
        out = torch.empty((n, h // 4, w // 4, 64), dtype=torch.uint8, device=x.device)
    check(lib().qcn_resnet_stem_fused(_ptr(x), n, h, w, float(scale), int(zp), _ptr(d.w), d.cout,
                                      _ptr(d.u), _ptr(d.v), _ptr(d.mult), _ptr(d.corr), int(d.z_y),
                                      int(bool(d.relu)), _ptr(out), _stream()), "stem_fused")
    return out


def avgpool(x, x_zp, out=None):
    """Global average pool of u8 NHWC [n,h,w,c] -> [n,c], qparams kept
    (torch's quantized adaptive_avg_pool2d)."""
    _need(x, torch.uint8, "avgpool.x")
    n, h, w, c = x.shape
    if out is None:
        out = torch.empty((n, c), dtype=torch.uint8, device=x.device)
    check(lib().qcn_avgpool_u8_nhwc(_ptr(x), n, h * w, c, int(x_zp), _ptr(out), _stream()), "avgpool")
    return out


# -------------------------- §8(f)2 in the reference's semantics (live stubs)
def dq_bn_q(y, s, z, alpha, beta, relu, s_next, z_next, out=None):
    """conv u8 -> DeQuantStub -> BN -> [ReLU] -> the next conv's QuantStub."""
    _need(y, torch.uint8, "dq_bn_q.y")
    if out is None:
        out = torch.empty_like(y)
    check(lib().qcn_dq_bn_q_u8(_ptr(y), y.numel(), y.shape[-1], float(s), int(z), _ptr(alpha),
                               _ptr(beta), int(bool(relu)), float(s_next), int(z_next), _ptr(out),
                               _stream()), "dq_bn_q")
    return out


def dq_bn_relu_maxpool(y, s, z, alpha, beta, s_next=None, z_next=0):
    """Stem hand-off: fp32 max-pool 3x3/2 of relu(bn(dq(y))) and (s_next given)
    its u8 quantize.  Returns (fp32 map, u8 map or None)."""
    _need(y, torch.uint8, "dq_bn_relu_maxpool.y")
    n, h, w, c = y.shape
    shape = (n, (h - 1) // 2 + 1, (w - 1) // 2 + 1, c)
    out = torch.empty(shape, dtype=torch.float32, device=y.device)
    oq = torch.empty(shape, dtype=torch.uint8, device=y.device) if s_next is not None else None
    check(lib().qcn_dq_bn_relu_maxpool_f32(_ptr(y), n, h, w, c, float(s), int(z), _ptr(alpha),
                                           _ptr(beta), _ptr(out), float(s_next or 0.0), int(z_next),
                                           _ptr(oq), _stream()), "dq_bn_relu_maxpool")
    return out, oq


def qdq_join(y3, s3, z3, a3, b3, ident, s_next=None, z_next=0):
    """Residual join: relu(bn3(dq(y3)) + identity); ``ident`` is either the
    fp32 block input or (yd, sd, zd, ad, bd) of the downsample conv.
    Returns (fp32 block output, u8 quantize for the next stubs or None)."""
    _need(y3, torch.uint8, "qdq_join.y3")
    out = torch.empty(y3.shape, dtype=torch.float32, device=y3.device)
    oq = torch.empty_like(y3) if s_next is not None else None
    if isinstance(ident, tuple):
        yd, sd, zd, ad, bd = ident
        _need(yd, torch.uint8, "qdq_join.yd")
        idf = None
    else:
        _need(ident, torch.float32, "qdq_join.identity")
        yd, sd, zd, ad, bd, idf = None, 0.0, 0, None, None, ident
    ref = yd if yd is not None else idf
    if tuple(ref.shape) != tuple(y3.shape):
        raise ValueError("identity shape differs from conv3's output")
    check(lib().qcn_qdq_join_f32(_ptr(y3), float(s3), int(z3), _ptr(a3), _ptr(b3), _ptr(yd), float(sd),
                                 int(zd), _ptr(ad), _ptr(bd), _ptr(idf), y3.numel(), y3.shape[-1],
                                 _ptr(out), float(s_next or 0.0), int(z_next), _ptr(oq), _stream()),
          "qdq_join")
    return out, oq


def avgpool_f32(x):
    _need(x, torch.float32, "avgpool_f32.x")
    n, h, w, c = x.shape
    out = torch.empty((n, c), dtype=torch.float32, device=x.device)
    check(lib().qcn_avgpool_f32_nhwc(_ptr(x), n, h, w, c, _ptr(out), _stream()), "avgpool_f32")
    return out
