"""GPU parity for SURVEY §8(f)2 (ResNet-style bottleneck blocks, config 5):
the general int8 conv, residual join, maxpool 3x3/2, stem packing and average
pool kernels (through the C ABI) against the torch.ao golden vectors and the
numpy oracle, then whole networks: the 1-block-per-stage ResNet at 64x64
bit-exact against torch.ao eager static int8 (tests/golden/net_resnet_int8.npz),
and (on synthetic weights) the same net and the full ResNet-50 at 224x224
bit-exact against oracle.qref.resnet_int8_forward."""
import os

import numpy as np
import pytest
import torch

from oracle import qref

pytestmark = pytest.mark.gpu

F32 = np.float32


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from qconvnet import _lib
    _lib.load()
    return torch.device("cuda:0")


def _layer(dev, w_oihw, s_x, s_w, s_y, b, z_x, z_y, relu, stride, pad):
    from qconvnet import ops
    from qconvnet import quant as Q
    from qconvnet.qmodel import _DevLayer
    d = _DevLayer()
    packed, wsum = ops.pack_conv_kmajor(w_oihw)
    d.cout, _, d.kh, d.kw = w_oihw.shape
    (d.sy, d.sx), (d.py, d.px) = stride, pad
    u, v, mult = Q.epilogue_constants(s_x, s_w, s_y, b)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d.w, d.u, d.v, d.mult = t(packed), t(u), t(v), t(mult)
    d.corr = t(((128 - int(z_x)) * wsum.astype(np.int64)).astype(np.int32))
    d.z_y, d.relu = int(z_y), relu
    return d


@pytest.mark.parametrize("impl", ["gemm", "gen"])
def test_conv_general_golden(dev, golden_dir, impl):
    from qconvnet import ops
    z = dict(np.load(os.path.join(golden_dir, "ops_resnet.npz")))
    ran = 0
    for i in range(int(z["n"])):
        g = lambda k: z[f"c{i}_{k}"]  # noqa: E731
        if g("qx").shape[-1] % 32:
            continue   # the 3-channel stem case runs through stem_pack (below)
        st, pd = int(g("stride")), int(g("pad"))
        d = _layer(dev, g("w"), g("s_x"), g("s_w"), g("s_y"), g("b"), int(g("zx")), int(g("zy")),
                   bool(g("relu")), (st, st), (pd, pd))
        out = ops.conv(torch.from_numpy(g("qx")).to(dev), int(g("zx")), d, impl=impl)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), g("out")), i
        ran += 1
    assert ran == 5


@pytest.mark.parametrize("shape", [
    # n, hw, c, zx, relu, zy, per_channel
    (3, 56, 64, 5, True, 0, True),
    (2, 56, 64, 200, False, 30, False),
    (3, 28, 128, 17, True, 0, True),      # bands of 16 rows: two cross an image boundary
    (5, 28, 128, 0, False, 99, True),     # 140 rows: the last band is partial
    (1, 28, 128, 255, True, 7, False),
])
def test_conv3x3_patch_tiles_oracle(dev, shape):
    """The ResNet 3x3 stride-1 convs on the patch-staged ring kernel
    (qcn_conv3x3_u8s8_nhwc: 56x56 row bands, 28x28 flattened-row bands with
    per-image halos) against the oracle's conv, per-channel and per-tensor."""
    from qconvnet import ops
    n, hw, c, zx, relu, zy, pc = shape
    rng = np.random.default_rng(hash(shape) & 0xffff)
    qx = rng.integers(0, 256, (n, hw, hw, c)).astype(np.uint8)
    wf = (rng.standard_normal((c, c, 3, 3)) * 0.05).astype(F32)
    s_w = qref.qparams_symmetric(wf.reshape(c, -1).min(1), wf.reshape(c, -1).max(1))[0] if pc \
        else qref.qparams_symmetric(wf.min(), wf.max())[0]
    wq = qref.quantize_weight(wf, s_w)
    b = (rng.standard_normal(c) * 0.3).astype(F32)
    s_x, s_y = F32(0.02), F32(0.2)
    u, v, mult = qref.requant_constants(s_x, s_w, s_y, b)
    packed, wsum = ops.pack_conv3x3(wq)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    corr = ((128 - zx) * wsum.astype(np.int64)).astype(np.int32)
    out = ops.conv3x3(T(qx), zx, T(packed), c, T(np.broadcast_to(u, c).astype(F32)),
                      T(np.broadcast_to(v, c).astype(F32)), T(np.broadcast_to(mult, c).astype(F32)),
                      T(corr), zy, relu, False).cpu().numpy()
    ref = qref.conv_q(qx, zx, wq, u, v, mult, zy, relu, (1, 1), (1, 1))
    assert np.array_equal(out, ref)
    assert len(np.unique(ref)) > 8, "degenerate case"


@pytest.mark.parametrize("shape", [
    # n, h, w, cin, cout, kh, kw, stride, pad, zx, relu, zy, per_channel
    (3, 13, 11, 96, 192, 3, 3, 2, 1, 77, False, 30, True),
    (1, 7, 7, 512, 2048, 1, 1, 1, 0, 0, False, 99, True),
    (2, 14, 14, 256, 512, 1, 1, 2, 0, 4, False, 128, True),
    (5, 9, 6, 32, 64, 3, 3, 1, 1, 255, True, 0, False),
    (1, 1, 1, 64, 128, 3, 3, 1, 1, 13, True, 0, True),
    (2, 56, 56, 64, 64, 3, 3, 1, 1, 0, True, 0, True),
    (1, 28, 28, 128, 512, 1, 1, 1, 0, 9, False, 140, True),
    # 256-channel 8-wave tiles (3x3 and 2048-deep 1x1, cout % 256 == 0), ragged pixel counts
    (3, 9, 11, 128, 256, 3, 3, 1, 1, 31, True, 0, True),
    (2, 13, 13, 64, 512, 3, 3, 2, 1, 200, False, 77, False),
    (2, 5, 7, 2048, 512, 1, 1, 1, 0, 3, True, 0, True),
])
@pytest.mark.parametrize("impl", ["gemm", "gen"])
def test_conv_general_oracle(dev, shape, impl):
    from qconvnet import ops
    n, h, w, cin, cout, kh, kw, st, pd, zx, relu, zy, pc = shape
    rng = np.random.default_rng(hash(shape) & 0xffff)
    qx = rng.integers(0, 256, (n, h, w, cin)).astype(np.uint8)
    wf = (rng.standard_normal((cout, cin, kh, kw)) * 0.05).astype(F32)
    s_w = qref.qparams_symmetric(wf.reshape(cout, -1).min(1), wf.reshape(cout, -1).max(1))[0] if pc \
        else qref.qparams_symmetric(wf.min(), wf.max())[0]
    wq = qref.quantize_weight(wf, s_w)
    b = (rng.standard_normal(cout) * 0.3).astype(F32)
    s_x, s_y = F32(0.02), F32(0.9 if cin >= 256 else 0.2)
    d = _layer(dev, wq, s_x, s_w, s_y, b, zx, zy, relu, (st, st), (pd, pd))
    out = ops.conv(torch.from_numpy(qx).to(dev), zx, d, impl=impl).cpu().numpy()
    u, v, mult = qref.requant_constants(s_x, s_w, s_y, b)
    ref = qref.conv_q(qx, zx, wq, u, v, mult, zy, relu, (st, st), (pd, pd))
    assert out.shape == ref.shape
    assert np.array_equal(out, ref)
    assert len(np.unique(ref)) > 8, "degenerate case"
    if not relu:   # the fused residual join equals conv -> add_relu
        d.s_y = s_y
        r = rng.integers(0, 256, ref.shape).astype(np.uint8)
        fused = ops.conv(torch.from_numpy(qx).to(dev), zx, d,
                         resid=(torch.from_numpy(r).to(dev), F32(0.03), 17, F32(0.05), 0)).cpu().numpy()
        assert np.array_equal(fused, qref.add_relu_q(ref, s_y, zy, r, F32(0.03), 17, F32(0.05), 0))


@pytest.mark.parametrize("shape", [
    # n, h, w, cin, cout, zx, relu, zy, per_channel, join z_o
    (3, 7, 9, 64, 256, 5, False, 30, True, 0),        # 189 pixels: ragged last strip
    (2, 56, 56, 64, 256, 0, False, 0, True, 23),      # zy = 0 (cvt-only requant), z_o != 0
    (1, 28, 29, 128, 512, 9, False, 140, False, 0),
    (4, 14, 14, 256, 1024, 3, False, 60, True, 11),
    (2, 17, 5, 256, 64, 200, True, 0, True, None),   # Cout 64: two waves per workgroup
    (1, 11, 13, 64, 64, 77, True, 20, False, None),  # ReLU with zy > 0 (general clamp)
    (1, 1, 1, 128, 128, 0, False, 5, True, 0),       # one pixel
    (7, 31, 33, 128, 256, 130, False, 2, True, 0),   # many chunks, tail chunk shorter
    (2, 9, 7, 512, 2048, 40, False, 11, True, 0),     # K = 512: activations through the LDS ring
    (3, 28, 28, 512, 128, 0, True, 0, True, None),
    (1, 5, 5, 256, 256, 9, False, 3, False, 9),
    # K = 1024: the tiled kernel (the r06 K-split streaming form, tools/patches/resnet_k1024_stream.patch, passed these too)
    (16, 14, 14, 1024, 256, 7, False, 30, True, None),   # the layer-3 reduce, 98 strips
    (1, 14, 15, 1024, 512, 0, True, 0, False, None),     # ReLU at zy 0 (cvt-only requant), ragged
    (3, 7, 9, 1024, 128, 131, True, 12, True, None),     # ReLU floor 12 (general clamp), one group
    (1, 1, 1, 1024, 256, 9, False, 3, True, None),       # one pixel
])
def test_conv1x1_stream_oracle(dev, shape):
    """The streaming 1x1 stride-1 kernel (conv1x1_stream_kernel: K = Cin in
    {64, 128, 256, 512}, weights and constants in registers, 32-pixel strips;
    the K = 1024 cases run the tiled conv_gemm_kernel) against
    the oracle's conv, and with the fused residual join against conv ->
    add_relu_q."""
    from qconvnet import ops
    n, h, w, cin, cout, zx, relu, zy, pc, zo = shape
    rng = np.random.default_rng(hash(shape) & 0xffff)
    qx = rng.integers(0, 256, (n, h, w, cin)).astype(np.uint8)
    wf = (rng.standard_normal((cout, cin, 1, 1)) * 0.05).astype(F32)
    s_w = qref.qparams_symmetric(wf.reshape(cout, -1).min(1), wf.reshape(cout, -1).max(1))[0] if pc \
        else qref.qparams_symmetric(wf.min(), wf.max())[0]
    wq = qref.quantize_weight(wf, s_w)
    b = (rng.standard_normal(cout) * 0.3).astype(F32)
    s_x, s_y = F32(0.02), F32(0.3 if cin >= 256 else 0.15)
    d = _layer(dev, wq, s_x, s_w, s_y, b, zx, zy, relu, (1, 1), (0, 0))
    out = ops.conv(torch.from_numpy(qx).to(dev), zx, d, impl="gemm").cpu().numpy()
    u, v, mult = qref.requant_constants(s_x, s_w, s_y, b)
    ref = qref.conv_q(qx, zx, wq, u, v, mult, zy, relu, (1, 1), (0, 0))
    assert np.array_equal(out, ref)
    if n * h * w > 1:
        assert len(np.unique(ref)) > 8, "degenerate case"
    if zo is not None:
        d.s_y = s_y
        r = rng.integers(0, 256, ref.shape).astype(np.uint8)
        fused = ops.conv(torch.from_numpy(qx).to(dev), zx, d,
                         resid=(torch.from_numpy(r).to(dev), F32(0.03), 17, F32(0.05), zo)).cpu().numpy()
        assert np.array_equal(fused, qref.add_relu_q(ref, s_y, zy, r, F32(0.03), 17, F32(0.05), zo))


@pytest.mark.parametrize("shape", [
    # n, h, w, expand zx, expand zy, join z_o, reduce cout, reduce zy, reduce relu, per_channel
    (3, 7, 9, 5, 30, 0, 64, 0, True, True),        # 189 pixels: ragged last strip
    (2, 56, 56, 0, 0, 23, 64, 0, True, True),      # the layer-1 shape; z_o != 0
    (1, 13, 11, 77, 9, 0, 128, 12, True, False),   # the layer-2 first reduce (cout 128), ReLU floor 12
    (2, 5, 5, 130, 2, 7, 128, 40, False, True),    # no ReLU: general clamp
    (1, 1, 1, 9, 3, 0, 64, 0, True, True),         # one pixel
])
def test_conv1x1_join_reduce_oracle(dev, shape):
    """The expand + join launch with the next block's reduce conv fused
    (qcn_conv1x1_join_reduce_u8s8_nhwc) against the oracle's conv -> add_relu_q
    -> conv, and against the two separate launches."""
    from qconvnet import ops
    n, h, w, zx, zy, zo, cr, zr, relur, pc = shape
    rng = np.random.default_rng(hash(shape) & 0xffff)
    qx = rng.integers(0, 256, (n, h, w, 64)).astype(np.uint8)

    def wts(cout, cin):
        wf = (rng.standard_normal((cout, cin, 1, 1)) * 0.05).astype(F32)
        s_w = qref.qparams_symmetric(wf.reshape(cout, -1).min(1), wf.reshape(cout, -1).max(1))[0] if pc \
            else qref.qparams_symmetric(wf.min(), wf.max())[0]
        return qref.quantize_weight(wf, s_w), s_w, (rng.standard_normal(cout) * 0.3).astype(F32)

    w3, sw3, b3 = wts(256, 64)
    w1, sw1, b1 = wts(cr, 256)
    s_x, s_y, s_o, s_y2 = F32(0.02), F32(0.15), F32(0.05), F32(0.4)
    d3 = _layer(dev, w3, s_x, sw3, s_y, b3, zx, zy, False, (1, 1), (0, 0))
    d3.s_y = s_y
    d1 = _layer(dev, w1, s_o, sw1, s_y2, b1, zo, zr, relur, (1, 1), (0, 0))
    r = rng.integers(0, 256, (n, h, w, 256)).astype(np.uint8)
    T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    resid = (T(r), F32(0.03), 17, s_o, zo)
    got = ops.conv_join_reduce(T(qx), zx, d3, resid, d1)
    assert got is not None, "the library declined a supported shape"
    q, y2 = (t.cpu().numpy() for t in got)
    u, v, mult = qref.requant_constants(s_x, sw3, s_y, b3)
    y3 = qref.conv_q(qx, zx, w3, u, v, mult, zy, False, (1, 1), (0, 0))
    qj = qref.add_relu_q(y3, s_y, zy, r, F32(0.03), 17, s_o, zo)
    u1, v1, m1 = qref.requant_constants(s_o, sw1, s_y2, b1)
    ref2 = qref.conv_q(qj, zo, w1, u1, v1, m1, zr, relur, (1, 1), (0, 0))
    assert np.array_equal(q, qj)
    assert np.array_equal(y2, ref2)
    if n * h * w > 1:
        assert len(np.unique(ref2)) > 8, "degenerate case"
    # the two launches it replaces
    q_sep = ops.conv(T(qx), zx, d3, resid=resid)
    y2_sep = ops.conv(q_sep, zo, d1)
    assert np.array_equal(q_sep.cpu().numpy(), q) and np.array_equal(y2_sep.cpu().numpy(), y2)


@pytest.mark.parametrize("shape", [
    # n, h, w, cin, cout, zx, zy, per_channel
    (3, 28, 28, 256, 512, 7, 90, True),
    (2, 14, 14, 512, 1024, 0, 0, True),
    (3, 13, 11, 256, 128, 200, 31, False),   # odd input sides, ragged last strip
    (2, 14, 14, 1024, 2048, 7, 90, True),    # the layer-4 downsample (K = 1024)
    (3, 13, 11, 1024, 128, 200, 31, False),
])
def test_conv1x1_stride2_stream_oracle(dev, shape):
    """The stride-2 downsample 1x1 on the streaming kernel (rows of the even
    input pixels gathered through the LDS ring) against the oracle's conv."""
    from qconvnet import ops
    n, h, w, cin, cout, zx, zy, pc = shape
    rng = np.random.default_rng(hash(shape) & 0xffff)
    qx = rng.integers(0, 256, (n, h, w, cin)).astype(np.uint8)
    wf = (rng.standard_normal((cout, cin, 1, 1)) * 0.05).astype(F32)
    s_w = qref.qparams_symmetric(wf.reshape(cout, -1).min(1), wf.reshape(cout, -1).max(1))[0] if pc \
        else qref.qparams_symmetric(wf.min(), wf.max())[0]
    wq = qref.quantize_weight(wf, s_w)
    b = (rng.standard_normal(cout) * 0.3).astype(F32)
    s_x, s_y = F32(0.02), F32(0.3)
    d = _layer(dev, wq, s_x, s_w, s_y, b, zx, zy, False, (2, 2), (0, 0))
    out = ops.conv(torch.from_numpy(qx).to(dev), zx, d, impl="gemm").cpu().numpy()
    u, v, mult = qref.requant_constants(s_x, s_w, s_y, b)
    ref = qref.conv_q(qx, zx, wq, u, v, mult, zy, False, (2, 2), (0, 0))
    assert out.shape == ref.shape
    assert np.array_equal(out, ref)
    assert len(np.unique(ref)) > 8, "degenerate case"


@pytest.mark.parametrize("shape", [
    # n, hw, cin, cout, zx, relu, zy, per_channel
    (2, 14, 256, 256, 7, True, 0, True),
    (1, 14, 256, 512, 200, False, 40, False),   # two 256-channel groups per image
    (3, 7, 512, 512, 0, True, 9, True),         # ReLU floor at zy > 0
    (1, 7, 512, 256, 131, False, 0, False),
])
def test_conv3x3_whole_image_oracle(dev, shape):
    """The whole-image 3x3 kernel (conv3x3_img_kernel: the layer-3 14x14x256
    and layer-4 7x7x512 maps, one image x 256 channels per 8-wave workgroup)
    against the oracle's conv, per-channel and per-tensor."""
    from qconvnet import ops
    n, hw, cin, cout, zx, relu, zy, pc = shape
    rng = np.random.default_rng(hash(shape) & 0xffff)
    qx = rng.integers(0, 256, (n, hw, hw, cin)).astype(np.uint8)
    wf = (rng.standard_normal((cout, cin, 3, 3)) * 0.02).astype(F32)
    s_w = qref.qparams_symmetric(wf.reshape(cout, -1).min(1), wf.reshape(cout, -1).max(1))[0] if pc \
        else qref.qparams_symmetric(wf.min(), wf.max())[0]
    wq = qref.quantize_weight(wf, s_w)
    b = (rng.standard_normal(cout) * 0.3).astype(F32)
    s_x, s_y = F32(0.02), F32(0.6)
    d = _layer(dev, wq, s_x, s_w, s_y, b, zx, zy, relu, (1, 1), (1, 1))
    out = ops.conv(torch.from_numpy(qx).to(dev), zx, d, impl="gemm").cpu().numpy()
    u, v, mult = qref.requant_constants(s_x, s_w, s_y, b)
    ref = qref.conv_q(qx, zx, wq, u, v, mult, zy, relu, (1, 1), (1, 1))
    assert out.shape == ref.shape
    assert np.array_equal(out, ref)
    assert len(np.unique(ref)) > 8, "degenerate case"


def test_add_relu_golden_and_ragged(dev, golden_dir):
    from qconvnet import ops
    z = dict(np.load(os.path.join(golden_dir, "ops_resnet.npz")))
    for i in range(int(z["na"])):
        sa, sb, so = z[f"a{i}_p"]
        za, zb, zo = (int(t) for t in z[f"a{i}_z"])
        out = ops.add_relu(torch.from_numpy(z[f"a{i}_qa"]).to(dev), sa, za,
                           torch.from_numpy(z[f"a{i}_qb"]).to(dev), sb, zb, so, zo)
        assert np.array_equal(out.cpu().numpy(), z[f"a{i}_out"]), i
    rng = np.random.default_rng(3)
    for count in (1, 15, 17, 4099):
        qa = rng.integers(0, 256, count).astype(np.uint8)
        qb = rng.integers(0, 256, count).astype(np.uint8)
        for relu in (True, False):
            out = ops.add_relu(torch.from_numpy(qa).to(dev), 0.03, 100, torch.from_numpy(qb).to(dev),
                               0.02, 3, 0.04, 60, relu)
            ref = qref.add_relu_q(qa, 0.03, 100, qb, 0.02, 3, 0.04, 60, relu)
            assert np.array_equal(out.cpu().numpy(), ref), (count, relu)


def test_maxpool3x3s2(dev, golden_dir):
    from qconvnet import ops
    z = dict(np.load(os.path.join(golden_dir, "ops_resnet.npz")))
    out = ops.maxpool3x3s2(torch.from_numpy(z["mp_in"]).to(dev))
    assert np.array_equal(out.cpu().numpy(), z["mp_out"])
    q = np.random.default_rng(4).integers(0, 256, (2, 112, 112, 64)).astype(np.uint8)
    out = ops.maxpool3x3s2(torch.from_numpy(q).to(dev))
    assert np.array_equal(out.cpu().numpy(), qref.maxpool3x3s2_nhwc(q))


def test_stem_pack_and_stem_conv(dev, golden_dir):
    from qconvnet import ops
    rng = np.random.default_rng(6)
    x = rng.standard_normal((2, 3, 37, 41)).astype(F32)
    s, zp = F32(0.02), 120
    rows = ops.stem_pack(torch.from_numpy(x).to(dev), s, zp).cpu().numpy()
    assert np.array_equal(rows, qref.stem_pack(x, s, zp))
    # the golden 7x7/2 stem conv (torch.ao) through the packed rows
    z = dict(np.load(os.path.join(golden_dir, "ops_resnet.npz")))
    i = [j for j in range(int(z["n"])) if z[f"c{j}_qx"].shape[-1] == 3][0]
    g = lambda k: z[f"c{i}_{k}"]  # noqa: E731
    s_x, zx = g("s_x"), int(g("zx"))
    xf = qref.dequantize(g("qx"), s_x, zx).transpose(0, 3, 1, 2).copy()   # re-quantizes exactly
    rows = ops.stem_pack(torch.from_numpy(xf).to(dev), s_x, zx)
    d = _layer(dev, ops.stem_weight_rows(g("w")), s_x, g("s_w"), g("s_y"), g("b"), zx, int(g("zy")),
               bool(g("relu")), (2, 1), (3, 0))
    out = ops.conv(rows, zx, d).cpu().numpy()
    assert np.array_equal(out, g("out"))


def test_avgpool(dev):
    """Quantized global average pool (qparams kept) == the oracle, which is
    pinned to torch's quantized adaptive_avg_pool2d (test_resnet_cpu fixture
    test); 2x2 maps have exact .5 ties."""
    from qconvnet import ops
    g = np.random.default_rng(7)
    for shape, zp in (((3, 7, 7, 2048), 11), ((5, 2, 2, 2048), 0), ((2, 2, 2, 64), 200)):
        q = g.integers(0, 256, shape).astype(np.uint8)
        out = ops.avgpool(torch.from_numpy(q).to(dev), zp).cpu().numpy()
        assert np.array_equal(out, qref.avgpool_q(q, zp)), shape


def _net(dev, layers, hw, seed):
    from models.resnet import synthetic_images, synthetic_resnet
    from qconvnet.resnet import quantize_resnet
    m = synthetic_resnet(seed, layers, num_classes=1000, hw=hw, calib_images=8, device=dev)
    calib = [torch.from_numpy(synthetic_images(8, seed + 10, hw))]
    return m, quantize_resnet(m, calib, dev)


@pytest.mark.parametrize("layers,hw,n", [((1, 1, 1, 1), 64, 4), ((3, 4, 6, 3), 224, 2)])
def test_resnet_bit_exact(dev, layers, hw, n):
    from models.resnet import synthetic_images
    m, qm = _net(dev, layers, hw, 0)
    x = synthetic_images(n, 99, hw)
    logits, inter = qm.run(torch.from_numpy(x).to(dev), keep=True)
    torch.cuda.synchronize()
    ref, rinter = qref.resnet_int8_forward(x, qm.spec, keep=True)
    for k in ("stem", "pool") + tuple(f"block{i}" for i in range(sum(layers))):
        assert np.array_equal(inter[k].cpu().numpy(), rinter[k]), k
    assert np.array_equal(logits.cpu().numpy(), ref)
    # sanity: the int8 net tracks the fp32 net it was quantized from
    with torch.no_grad():
        f = m(torch.from_numpy(x).to(dev)).cpu().numpy()
    rel = np.abs(ref - f).max() / np.abs(f).max()
    assert rel < 0.35, rel


@pytest.mark.parametrize("hw,n,per_channel", [(224, 3, True), (64, 5, True), (64, 4, False)])
def test_stem_fused_equals_three_launches(dev, hw, n, per_channel):
    """qcn_resnet_stem_fused (quantize + 7x7/2 conv + ReLU + 3x3/2 max-pool in
    one launch) equals stem_pack -> 7x1 conv_gemm -> maxpool3x3s2 byte for
    byte, with inputs past the quantization range on both sides (clamps) and
    images whose last band ends at the border."""
    from models.resnet import synthetic_images, synthetic_resnet
    from qconvnet import ops
    from qconvnet.resnet import quantize_resnet
    m = synthetic_resnet(3, (1, 1, 1, 1), num_classes=10, hw=hw, calib_images=4, device=dev)
    qm = quantize_resnet(m, [torch.from_numpy(synthetic_images(4, 13, hw))], dev,
                         per_channel=per_channel)
    x = torch.from_numpy(synthetic_images(n, 17, hw)).to(dev)
    x[0, :, :3, :5] = 50.0     # past the top of the range
    x[-1, 1, -4:, -3:] = -50.0  # past the bottom
    assert qm._stem_fusable(x)
    ref = ops.maxpool3x3s2(ops.conv(ops.stem_pack(x, qm.in_scale, qm.in_zp), qm.in_zp, qm.stem))
    got = ops.stem_fused(x, qm.in_scale, qm.in_zp, qm.stem)
    torch.cuda.synchronize()
    assert got.shape == ref.shape == (n, hw // 4, hw // 4, 64)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("nsplit", [2, 3])
def test_resnet_run_streams_equals_run(dev, nsplit):
    """run_streams (batch slices on their own HIP streams, launches interleaved
    layer by layer) gives the one-stream logits bit for bit, also for a batch
    that does not split evenly."""
    from models.resnet import synthetic_images
    _, qm = _net(dev, (1, 1, 1, 1), 64, 0)
    x = torch.from_numpy(synthetic_images(7, 5, 64)).to(dev)
    ref = qm.run(x).clone()
    for _ in range(2):   # second pass: side streams reused
        out = qm.run_streams(x, nsplit)
        assert torch.equal(out, ref)
    # the layer-1 join with layer 2's first reduce fused (the default) equals
    # the separate launches
    assert qm.fuse_reduce
    qm.fuse_reduce = False
    try:
        assert torch.equal(qm.run(x), ref)
    finally:
        qm.fuse_reduce = True
    torch.cuda.synchronize()


def test_resnet50_batch512_bench_path(dev):
    """Config 5 at the batch it is benchmarked at: ResNet-50 224x224,
    per-channel, batch 512, built exactly as bench.py --workload resnet50
    builds it and run through the bench's own two-stream path
    (run_streams(x, 2)).  Only at this size does the streaming 1x1 kernel walk
    many 32-pixel strips per chunk with its counted-vmcnt prefetch (~196 per
    chunk in layer 1, against 1 at batch 2).  Checks:
      (a) run_streams(x, 2) == run(x) at 512, logits bit for bit;
      (b) the static path is batch-independent, so every image's stem, block
          and pooled u8 outputs and its logits at batch 512 equal the same
          image run at batch 4 (128 small runs cover all 512 rows);
      (c) a 2-image slice (the first and the last image) equals the numpy
          oracle qref.resnet_int8_forward bit for bit, every block included.
    Reference semantics: /root/reference/models/custom_quantization_model.py:79-143."""
    from models.resnet import synthetic_images, synthetic_resnet
    from qconvnet.resnet import quantize_resnet
    fp = synthetic_resnet(0, device=dev, calib_images=32)
    calib = [torch.from_numpy(synthetic_images(32, 1 + i)) for i in range(2)]
    qm = quantize_resnet(fp, calib, dev, per_channel=True)
    B = 512
    xh = synthetic_images(B, 100)
    x = torch.from_numpy(xh).to(dev)
    out2 = qm.run_streams(x, 2).clone()
    full, inter = qm.run(x, keep=True)
    full = full.clone()
    torch.cuda.synchronize()
    assert torch.equal(out2, full)
    keys = ["stem", "pool"] + [f"block{i}" for i in range(len(qm.blocks))]
    for i in range(0, B, 4):
        o, it = qm.run(x[i:i + 4], keep=True)
        assert torch.equal(o, full[i:i + 4]), i
        for k in keys:
            assert torch.equal(it[k], inter[k][i:i + 4]), (i, k)
    idx = [0, B - 1]
    ref, rinter = qref.resnet_int8_forward(xh[idx], qm.spec, keep=True)
    for k in keys:
        assert np.array_equal(inter[k][idx].cpu().numpy(), rinter[k]), k
    assert np.array_equal(full[idx].cpu().numpy(), ref)


def test_resnet_equals_torchao_fixture(dev):
    """§8(f)2 whole-net pin on the GPU: the 1-1-1-1 bottleneck ResNet at 64x64
    with torch.ao's qparams (tests/golden/net_resnet_int8.npz) — stem, every
    block's u8 output, pooled features and logits bit-exact to torch.ao eager
    static int8 (fbgemm)."""
    import resnetfix
    from qconvnet.resnet import QuantizedResNet
    z = resnetfix.load()
    sp = resnetfix.spec(z)
    assert resnetfix.check_weights(sp, z) == []
    qm = QuantizedResNet(sp, dev)
    logits, inter = qm.run(torch.from_numpy(resnetfix.images(z)).to(dev), keep=True)
    torch.cuda.synchronize()
    assert resnetfix.sha(inter["stem"].cpu().numpy()) == str(z["stem_sha"])
    for i in range(len(sp["blocks"])):
        assert resnetfix.sha(inter[f"block{i}"].cpu().numpy()) == str(z[f"block{i}_sha"]), i
    assert np.array_equal(inter["pool"].cpu().numpy(), z["pool"])
    assert np.array_equal(logits.cpu().numpy(), z["logits"])


def test_custom_quantized_resnet50_wrapper(dev):
    """The models.custom_quantization_model drop-in builds the same executor."""
    from models.custom_quantization_model import CustomQuantizedResNet50
    from models.resnet import synthetic_images, synthetic_resnet
    from qconvnet.resnet import quantize_resnet
    m = synthetic_resnet(1, (1, 1, 1, 1), num_classes=10, hw=64, calib_images=8, device=dev)
    calib = [torch.from_numpy(synthetic_images(8, 5, 64))]
    w = CustomQuantizedResNet50(m, calibration_batches=[(calib[0], None)], device=dev)
    x = synthetic_images(3, 6, 64)
    out = w(torch.from_numpy(x))
    assert out.shape == (3, 10) and out.device.type == "cpu"
    ref, _ = qref.resnet_int8_forward(x, w.quantized_model.spec)
    assert np.array_equal(out.numpy(), ref)
    # calibration runs on the CPU by default: a second quantization is identical
    again = quantize_resnet(m, calib, dev)
    assert np.array_equal(again(torch.from_numpy(x)).numpy(), out.numpy())


def test_resnet_reference_semantics_equals_torchao_fixture(dev):
    """§8(f)2 in the reference's own semantics on the GPU
    (CustomQuantizedResNet50 with live per-layer stubs,
    custom_quantization_model.py:60-143; tests/golden/net_resnet_qdq.npz):
    every int8 conv's u8 output, the stem's and every block's fp32 output
    (BN / ReLU / max-pool / residual add in fp32), the fc's u8 output and the
    fp32 logits bit-exact to torch.ao eager (fbgemm) — the fp32 hand-offs use
    ATen's op order, so no tolerance is needed."""
    import resnetfix
    from qconvnet.resnet_qdq import QuantizedResNetQDQ
    z = resnetfix.load_qdq()
    sp = resnetfix.qdq_spec(z, fixture_qparams=True)
    assert resnetfix.check_qdq_spec(sp, z) == []
    qm = QuantizedResNetQDQ(sp, dev)
    logits, inter = qm.run(torch.from_numpy(resnetfix.images(z)).to(dev), keep=True)
    torch.cuda.synchronize()
    keys = [k[:-4] for k in z if k.endswith("_sha") and not k.endswith(".w_sha")
            and k not in ("x_sha", "calib_sha")]
    assert "block3" in keys and "stem.q" in keys and "fc.q" in keys
    for k in keys:
        assert resnetfix.sha(inter[k].cpu().numpy()) == str(z[k + "_sha"]), k
    assert np.array_equal(logits.cpu().numpy(), z["logits"])


def test_custom_quantized_resnet50_reference_mode(dev):
    """CustomQuantizedResNet50(mode="reference") builds the live-stub executor
    and equals the numpy oracle (qref.resnet_qdq_forward) on its own spec."""
    from models.custom_quantization_model import CustomQuantizedResNet50
    from models.resnet import synthetic_images, synthetic_resnet
    m = synthetic_resnet(2, (1, 1, 1, 1), num_classes=10, hw=64, calib_images=8, device=dev)
    calib = [torch.from_numpy(synthetic_images(8, 7, 64))]
    w = CustomQuantizedResNet50(m, calibration_batches=calib, device=dev, mode="reference")
    x = synthetic_images(5, 8, 64)
    out = w(torch.from_numpy(x))
    assert out.shape == (5, 10) and out.device.type == "cpu"
    ref, _ = qref.resnet_qdq_forward(x, w.quantized_model.spec)
    assert np.array_equal(out.numpy(), ref)
