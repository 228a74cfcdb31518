"""GPU parity: the HIP kernels (through the C ABI) against the committed
torch.ao/fbgemm golden vectors and the numpy oracle.  Integer outputs must be
bit-exact; fp32 outputs that follow the same fp32 op order are compared
exactly too (dequantize, dynamic Linear); only the fp32 fc2 of the QDQ model
(a plain fp32 GEMM, summation order differs from MKL) uses a tolerance."""
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
    _lib.load()  # fail loudly if the HIP library is missing
    return torch.device("cuda:0")


def _g(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name)))


def test_quantize_dequantize_golden(dev, golden_dir):
    from qconvnet import ops
    z = _g(golden_dir, "ops_quantize.npz")
    for i in range(5):
        x = z[f"q{i}_x"]
        n = x.size
        xt = torch.from_numpy(x.reshape(1, 1, 1, n)).to(dev)
        q = ops.quantize(xt, z[f"q{i}_scale"], int(z[f"q{i}_zp"]), nhwc=False)
        assert np.array_equal(q.cpu().numpy().reshape(-1), z[f"q{i}_q"]), i
        dq = ops.dequantize(q, z[f"q{i}_scale"], int(z[f"q{i}_zp"]))
        assert np.array_equal(dq.cpu().numpy().reshape(-1), z[f"q{i}_dq"]), i


def test_quantize_nchw_to_nhwc(dev):
    from qconvnet import ops
    rng = np.random.default_rng(3)
    x = (rng.standard_normal((5, 3, 7, 9)) * 2).astype(F32)
    q = ops.quantize(torch.from_numpy(x).to(dev), F32(0.02), 117, nhwc=True)
    ref = qref.quantize_per_tensor(np.transpose(x, (0, 2, 3, 1)), F32(0.02), 117)
    assert np.array_equal(q.cpu().numpy(), ref)


def test_minmax_observer(dev):
    from qconvnet import ops
    rng = np.random.default_rng(4)
    obs = ops.MinMaxObserver(dev)
    lo, hi = np.inf, -np.inf
    for n in (1, 3, 1000, 12345, 1 << 20):
        x = (rng.standard_normal(n) * rng.uniform(0.1, 10)).astype(F32)
        obs(torch.from_numpy(x).to(dev))
        lo, hi = min(lo, x.min()), max(hi, x.max())
        got = obs.values()
        assert got[0] == F32(lo) and got[1] == F32(hi)
    # misaligned view + all-negative data
    x = -np.abs(rng.standard_normal(1001)).astype(F32) - 1
    obs.reset()
    obs(torch.from_numpy(x).to(dev)[1:])
    assert obs.values() == (F32(x[1:].min()), F32(x[1:].max()))


def test_maxpool_argmax(dev):
    from qconvnet import ops
    rng = np.random.default_rng(5)
    for c in (16, 64, 3):
        q = rng.integers(0, 256, (3, 8, 6, c)).astype(np.uint8)
        got = ops.maxpool2x2(torch.from_numpy(q).to(dev)).cpu().numpy()
        assert np.array_equal(got, qref.maxpool2x2_nhwc(q))
    x = rng.integers(0, 4, (257, 10)).astype(F32)  # many ties
    got = ops.argmax(torch.from_numpy(x).to(dev)).cpu().numpy()
    assert np.array_equal(got, qref.argmax_rows(x))


def _conv_case(z, i):
    g = lambda k: z[f"c{i}_{k}"]  # noqa: E731
    return {k: g(k) for k in ("qx", "zx", "s_x", "w", "s_w", "b", "s_y", "zy", "relu", "out")}


def _run_conv(dev, c, pool=False, qdq=None):
    from qconvnet import ops, quant as Q
    w_oihw = np.ascontiguousarray(c["w"].transpose(0, 3, 1, 2))
    packed, wsum = ops.pack_conv3x3(w_oihw)
    u, v, mult = Q.epilogue_constants(c["s_x"], c["s_w"] if c["s_w"].size > 1 else c["s_w"].reshape(-1)[0],
                                      c["s_y"], c["b"])
    corr = ((128 - int(c["zx"])) * wsum.astype(np.int64)).astype(np.int32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    y = ops.conv3x3(T(c["qx"]), int(c["zx"]), T(packed), w_oihw.shape[0], T(u), T(v), T(mult),
                    T(corr), int(c["zy"]), bool(c["relu"]), pool, qdq)
    return y.cpu().numpy()


def test_conv_golden(dev, golden_dir):
    z = _g(golden_dir, "ops_conv.npz")
    for i in range(int(z["n"])):
        c = _conv_case(z, i)
        got = _run_conv(dev, c)
        assert np.array_equal(got, c["out"]), f"case {i}: {(got != c['out']).sum()} mismatches"


@pytest.mark.parametrize("n,h,cin,cout,pool,zx", [
    (3, 32, 64, 64, True, 0), (2, 32, 64, 64, False, 7), (3, 16, 64, 128, False, 0),
    (2, 16, 128, 128, True, 3), (5, 8, 128, 256, False, 0), (5, 8, 256, 256, True, 250),
    (3, 4, 256, 256, True, 0), (1, 6, 64, 64, False, 9), (2, 8, 192, 64, True, 1)])
def test_conv_tuned_vs_oracle(dev, n, h, cin, cout, pool, zx):
    """Every tuned instantiation (and the generic fallback) against the oracle,
    full-range u8 inputs, partial workgroups (odd image counts)."""
    from qconvnet import ops, quant as Q
    rng = np.random.default_rng(n * 1000 + h * 10 + cin + cout)
    qx = rng.integers(0, 256, (n, h, h, cin)).astype(np.uint8)
    w = rng.integers(-127, 128, (cout, cin, 3, 3)).astype(np.int8)
    b = (rng.standard_normal(cout) * 2).astype(F32)
    s_x, s_w, s_y, zy = F32(0.02), F32(0.003), F32(rng.uniform(0.5, 3)), int(rng.integers(0, 60))
    c = dict(qx=qx, zx=np.int64(zx), s_x=s_x, w=np.ascontiguousarray(w.transpose(0, 2, 3, 1)),
             s_w=np.asarray(s_w), b=b, s_y=s_y, zy=np.int64(zy), relu=np.int64(1))
    got = _run_conv(dev, c, pool=pool)
    u, v, mult = qref.requant_constants(s_x, s_w, s_y, b)
    ref = qref.requantize(qref.conv3x3_acc_nhwc(qx, zx, c["w"]) if not pool else
                          _pool_acc(qref.conv3x3_acc_nhwc(qx, zx, c["w"])), u, v, mult, zy, True)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} mismatches"


def _pool_acc(acc):
    n, h, w, c = acc.shape
    return acc.reshape(n, h // 2, 2, w // 2, 2, c).max(axis=(2, 4))


def test_conv_qdq_handoff(dev):
    """Per-layer QDQ epilogue == requant -> dequant -> relu -> quantize(next)."""
    from qconvnet import ops
    rng = np.random.default_rng(11)
    n, h, cin, cout = 2, 16, 64, 128
    qx = rng.integers(0, 256, (n, h, h, cin)).astype(np.uint8)
    w = rng.integers(-100, 101, (cout, cin, 3, 3)).astype(np.int8)
    b = (rng.standard_normal(cout)).astype(F32)
    c = dict(qx=qx, zx=np.int64(17), s_x=F32(0.02), w=np.ascontiguousarray(w.transpose(0, 2, 3, 1)),
             s_w=np.asarray(F32(0.002)), b=b, s_y=F32(1.5), zy=np.int64(131), relu=np.int64(0))
    s2, z2 = F32(0.9), 5
    got = _run_conv(dev, c, qdq=ops.qdq_struct(c["s_y"], 131, s2, z2))
    u, v, mult = qref.requant_constants(c["s_x"], c["s_w"], c["s_y"], b)
    q1 = qref.requantize(qref.conv3x3_acc_nhwc(qx, 17, c["w"]), u, v, mult, 131, False)
    x1 = np.maximum(qref.dequantize(q1, c["s_y"], 131), F32(0))
    ref = qref.quantize_per_tensor(x1, s2, z2)
    assert np.array_equal(got, ref)


def test_conv1_fused_quantize(dev):
    from qconvnet import ops, quant as Q
    rng = np.random.default_rng(12)
    for n, hw in ((3, 32), (5, 16), (9, 8)):
        x = (rng.standard_normal((n, 3, hw, hw)) * 1.3).astype(F32)
        w = rng.integers(-127, 128, (64, 3, 3, 3)).astype(np.int8)
        b = rng.standard_normal(64).astype(F32)
        s_in, z_in, s_w, s_y = F32(0.021), 121, F32(0.004), F32(0.05)
        packed, wsum = ops.pack_conv1(w)
        u, v, mult = Q.epilogue_constants(s_in, s_w, s_y, b)
        corr = ((128 - z_in) * wsum.astype(np.int64)).astype(np.int32)
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        qin = torch.empty((n, hw, hw, 3), dtype=torch.uint8, device=dev)
        y = ops.conv1_f32(T(x), s_in, z_in, T(packed), T(u), T(v), T(mult), T(corr), 0, True,
                          q_in=qin).cpu().numpy()
        q_ref = qref.quantize_per_tensor(qref.nchw_to_nhwc(x), s_in, z_in)
        assert np.array_equal(qin.cpu().numpy(), q_ref)
        u2, v2, m2 = qref.requant_constants(s_in, s_w, s_y, b)
        ref = qref.conv3x3_q(q_ref, z_in, np.ascontiguousarray(w.transpose(0, 2, 3, 1)), u2, v2, m2,
                             0, True)
        assert np.array_equal(y, ref), f"{(y != ref).sum()} mismatches"


def test_linear_golden(dev, golden_dir):
    from qconvnet import ops, quant as Q
    z = _g(golden_dir, "ops_linear.npz")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    for i in range(int(z["n"])):
        g = lambda k: z[f"l{i}_{k}"]  # noqa: E731
        w = g("w")
        wsum = w.astype(np.int64).sum(1)
        u, v, mult = Q.epilogue_constants(g("s_x"), g("s_w"), g("s_y"), g("b"))
        corr = ((128 - int(g("zx"))) * wsum).astype(np.int32)
        y, yf = ops.linear_u8(T(g("qx")), int(g("zx")), T(w), T(u), T(v), T(mult), T(corr),
                              int(g("zy")), bool(g("relu")), y_scale=g("s_y"), want_fp32=True)
        assert np.array_equal(y.cpu().numpy(), g("out")), i
        assert np.array_equal(yf.cpu().numpy(), qref.dequantize(g("out"), g("s_y"), int(g("zy"))))


def test_linear_dynamic_golden(dev, golden_dir):
    from qconvnet import ops
    z = _g(golden_dir, "ops_dynamic_linear.npz")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    for i in range(int(z["n"])):
        w = z[f"d{i}_w"]
        wsum = w.astype(np.int64).sum(1).astype(np.int32)
        y = ops.linear_dynamic(T(z[f"d{i}_x"]), T(w), T(np.atleast_1d(z[f"d{i}_s_w"])), T(wsum),
                               T(z[f"d{i}_b"]))
        got = y.cpu().numpy()
        assert np.array_equal(got, z[f"d{i}_y"]), f"case {i}: {(got != z[f'd{i}_y']).sum()}"


def test_linear_dynamic_shards_with_global_range(dev, golden_dir):
    """§8(f)1: shards quantized with the whole batch's [min, max] (what the
    all-reduce of qconvnet.dist.global_minmax supplies) concatenate to the
    whole-batch golden output; the device observer gives that range."""
    from qconvnet import ops
    z = _g(golden_dir, "ops_dynamic_linear.npz")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    for i in range(int(z["n"])):
        x, w = z[f"d{i}_x"], z[f"d{i}_w"]
        if x.shape[0] < 2:
            continue
        wsum = w.astype(np.int64).sum(1).astype(np.int32)
        args = (T(w), T(np.atleast_1d(z[f"d{i}_s_w"])), T(wsum), T(z[f"d{i}_b"]))
        mm = ops.minmax_range(T(x))
        assert np.array_equal(mm.cpu().numpy(), np.array([x.min(), x.max()], np.float32))
        h = x.shape[0] // 2
        parts = [ops.linear_dynamic(T(x[a:b]), *args, minmax=mm).cpu().numpy()
                 for a, b in ((0, h), (h, x.shape[0]))]
        assert np.array_equal(np.concatenate(parts), z[f"d{i}_y"]), i


@pytest.mark.parametrize("per_channel", [False, True])
def test_full_net_static_int8_golden(dev, per_channel):
    """Whole static-int8 SimpleConvNet vs torch.ao (fbgemm): logits bit-exact,
    every intermediate u8 activation bit-exact (by hash)."""
    import netfix
    from qconvnet.qmodel import QuantizedConvNet
    z = netfix.load(per_channel)
    spec, _ = netfix.static_spec(z)
    assert netfix.check_weights(spec, z) == []
    x = netfix.images(z)
    for fuse in (False, True):   # unfused exposes conv1's activation; fused is the product
        model = QuantizedConvNet(spec, dev, fuse12=fuse)
        logits, bufs = model.run(torch.from_numpy(x).to(dev), keep=True)
        torch.cuda.synchronize()
        assert np.array_equal(bufs["q"].cpu().numpy(), z["q_logits"]), fuse
        assert np.array_equal(logits.cpu().numpy(), z["logits"]), fuse
        for i, name in enumerate(["a1", "a2", "a3", "a4", "a5", "a6"], start=1):
            if fuse and name == "a1":
                continue
            assert netfix.sha(bufs[name].cpu().numpy()) == str(z[f"conv{i}_sha"]), (name, fuse)
        assert netfix.sha(bufs["f1"].cpu().numpy()) == str(z["fc1_sha"])
        assert np.array_equal(model(torch.from_numpy(x)).argmax(1).numpy(), z["argmax"])


@pytest.mark.parametrize("per_channel", [False, True])
def test_full_net_qdq_golden(dev, per_channel):
    """Per-layer QDQ model (reference CustomQuantizedSimpleConvNet with live
    stubs): integer chain bit-exact, fp32 fc2 within 1e-5 relative."""
    import netfix
    from qconvnet.qmodel import QuantizedConvNet
    z = netfix.load(per_channel)
    spec = netfix.qdq_spec(z)
    x = netfix.images(z)
    model = QuantizedConvNet(spec, dev)
    got = model(torch.from_numpy(x)).numpy()
    ref = z["qdq_logits"]
    tol = 1e-5 * np.abs(ref).max()
    assert np.abs(got - ref).max() <= tol, np.abs(got - ref).max()
    assert np.array_equal(got.argmax(1), ref.argmax(1))


def test_batch_split_invariance_and_graph(dev):
    """Static path is batch-independent: a 1024 batch equals its four 256
    shards; the HIP-graph replay equals the eager launch sequence."""
    import netfix
    from qconvnet.qmodel import QuantizedConvNet
    from oracle import torch_ref
    z = netfix.load(False)
    spec, _ = netfix.static_spec(z)
    model = QuantizedConvNet(spec, dev)
    x = torch.from_numpy(torch_ref.synthetic_images(1024, 7)).to(dev)
    full = model.run(x).clone()
    parts = torch.cat([model.run(x[i * 256:(i + 1) * 256]).clone() for i in range(4)])
    assert torch.equal(full, parts)
    xs = x.clone()
    model.capture_graph(xs)
    out = model.replay(1024)
    torch.cuda.synchronize()
    assert torch.equal(out, full)
    xs.copy_(torch.flip(x, [0]))
    out = model.replay(1024)
    torch.cuda.synchronize()
    assert torch.equal(out, torch.flip(full, [0]))


@pytest.mark.parametrize("mode,n", [("static", 37), ("qdq", 37), ("static", 300), ("static", 1024),
                                    ("qdq", 1024)])
def test_fused_conv12_equals_unfused(dev, mode, n):
    """The fused conv1+conv2 launch produces the unfused pair's u8 output
    exactly.  37 images: fewer than the CUs, one image per workgroup; 300:
    workgroups with two images and with one; 1024: four images per workgroup,
    every bottom half reusing two conv1 rows of its top half."""
    import netfix
    from qconvnet.qmodel import QuantizedConvNet
    from oracle import torch_ref
    z = netfix.load(False)
    spec = netfix.static_spec(z)[0] if mode == "static" else netfix.qdq_spec(z)
    x = torch.from_numpy(torch_ref.synthetic_images(n, 9) * 1.5).to(dev)
    a = QuantizedConvNet(spec, dev, fuse12=False).run(x, keep=True)[1]["a2"].clone()
    b = QuantizedConvNet(spec, dev, fuse12=True).run(x, keep=True)[1]["a2"].clone()
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("per_channel,zx,z1,z2", [(False, 0, 0, 131), (True, 17, 0, 90),
                                                   (False, 200, 40, 7)])
def test_classifier_head_equals_two_linears(dev, per_channel, zx, z1, z2):
    """Split-K fc1 on chunk-major operands + fused fc1-finish/fc2
    (qcn_classifier_u8s8) == the two
    static linear kernels (which match fbgemm: test_linear_golden), bit for
    bit on u8 fc1, u8 logits and fp32 logits.  Also the oracle for fc1."""
    from types import SimpleNamespace as NS
    from qconvnet import ops, quant as Q
    rng = np.random.default_rng(7 + zx)
    # 896 rows: below 1024 the split-K runs 64-row workgroups (fc_splitk_kernel<32>)
    m, k, n1, n2 = 896, 4096, 512, 10
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    qx = rng.integers(0, 256, (m, k), dtype=np.uint8)
    w1 = rng.integers(-128, 128, (n1, k), dtype=np.int8)
    w2 = rng.integers(-128, 128, (n2, n1), dtype=np.int8)
    s_x, s_y1, s_y2 = F32(0.02), F32(0.05), F32(0.11)
    s_w1 = (rng.uniform(1e-4, 3e-4, n1).astype(F32) if per_channel else F32(2e-4))
    s_w2 = (rng.uniform(1e-3, 3e-3, n2).astype(F32) if per_channel else F32(2e-3))
    b1 = rng.normal(0, 0.5, n1).astype(F32)
    b2 = rng.normal(0, 0.5, n2).astype(F32)
    u1, v1, m1 = Q.epilogue_constants(s_x, s_w1, s_y1, b1)
    u2, v2, m2 = Q.epilogue_constants(s_y1, s_w2, s_y2, b2)
    corr1 = ((128 - zx) * w1.astype(np.int64).sum(1)).astype(np.int32)
    corr2 = ((128 - z1) * w2.astype(np.int64).sum(1)).astype(np.int32)
    y1_ref = ops.linear_u8(T(qx), zx, T(w1), T(u1), T(v1), T(m1), T(corr1), z1, True)
    y2_ref, y2f_ref = ops.linear_u8(y1_ref, z1, T(w2), T(u2), T(v2), T(m2), T(corr2), z2, False,
                                    y_scale=s_y2, want_fp32=True)
    l1 = NS(w=T(w1), wk=T(ops.pack_fc_kmajor(w1)), u=T(u1), v=T(v1), mult=T(m1), corr=T(corr1),
            z_y=z1, relu=True)
    l2 = NS(w=T(w2), u=T(u2), v=T(v2), mult=T(m2), z_y=z2, relu=False, s_y=s_y2)
    ws = ops.classifier_workspace(m, n1, dev)
    y1 = torch.empty((m, n1), dtype=torch.uint8, device=dev)
    y2 = torch.empty((m, n2), dtype=torch.uint8, device=dev)
    y2f = torch.empty((m, n2), dtype=torch.float32, device=dev)
    assert ops.classifier(ops.to_kmajor(T(qx)), l1, l2, ws, y1, y2, y2f)
    torch.cuda.synchronize()
    assert torch.equal(y1, y1_ref)
    assert torch.equal(y2, y2_ref)
    assert torch.equal(y2f, y2f_ref)
    # the workspace is reusable across launches and batch sizes
    for mm in (m, 128, 384, 640, m):
        y2.zero_()
        y2f.zero_()
        assert ops.classifier(ops.to_kmajor(T(qx[:mm])), l1, l2, ws, y1[:mm], y2[:mm], y2f[:mm])
        torch.cuda.synchronize()
        assert torch.equal(y2[:mm], y2_ref[:mm]) and torch.equal(y2f[:mm], y2f_ref[:mm])
    # fc1 against the numpy oracle on a slice (A9 numerics)
    want = qref.linear_q(qx[:32], zx, w1, u1, v1, m1, z1, True)
    assert np.array_equal(y1[:32].cpu().numpy(), want)
    # outside the envelope -> QCN_ERR_UNSUPPORTED -> False (caller falls back)
    assert not ops.classifier(ops.to_kmajor(T(qx[:100])), l1, l2, ws, y1, y2, y2f)


def test_classifier_head_repeated_full_batch(dev):
    """The classifier head at batch 1024 (split-K fc1 over 256 workgroups +
    the per-row finisher): 20 back-to-back launches on one workspace, each
    bit-identical to fc1 -> fc2 by the two static linear kernels."""
    from types import SimpleNamespace as NS
    from qconvnet import ops, quant as Q
    rng = np.random.default_rng(21)
    m, k, n1, n2 = 1024, 4096, 512, 10
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    qx = rng.integers(0, 256, (m, k), dtype=np.uint8)
    w1 = rng.integers(-128, 128, (n1, k), dtype=np.int8)
    w2 = rng.integers(-128, 128, (n2, n1), dtype=np.int8)
    s_x, s_y1, s_y2, s_w1, s_w2 = F32(0.02), F32(0.05), F32(0.11), F32(2e-4), F32(2e-3)
    b1 = rng.normal(0, 0.5, n1).astype(F32)
    b2 = rng.normal(0, 0.5, n2).astype(F32)
    zx, z1, z2 = 3, 0, 120
    u1, v1, m1 = Q.epilogue_constants(s_x, s_w1, s_y1, b1)
    u2, v2, m2 = Q.epilogue_constants(s_y1, s_w2, s_y2, b2)
    corr1 = ((128 - zx) * w1.astype(np.int64).sum(1)).astype(np.int32)
    corr2 = ((128 - z1) * w2.astype(np.int64).sum(1)).astype(np.int32)
    y1_ref = ops.linear_u8(T(qx), zx, T(w1), T(u1), T(v1), T(m1), T(corr1), z1, True)
    y2_ref, y2f_ref = ops.linear_u8(y1_ref, z1, T(w2), T(u2), T(v2), T(m2), T(corr2), z2, False,
                                    y_scale=s_y2, want_fp32=True)
    l1 = NS(w=T(w1), wk=T(ops.pack_fc_kmajor(w1)), u=T(u1), v=T(v1), mult=T(m1), corr=T(corr1),
            z_y=z1, relu=True)
    l2 = NS(w=T(w2), u=T(u2), v=T(v2), mult=T(m2), z_y=z2, relu=False, s_y=s_y2)
    ws = ops.classifier_workspace(m, n1, dev)
    xk = ops.to_kmajor(T(qx))
    outs = []
    for _ in range(20):
        y1 = torch.empty((m, n1), dtype=torch.uint8, device=dev)
        y2 = torch.empty((m, n2), dtype=torch.uint8, device=dev)
        y2f = torch.empty((m, n2), dtype=torch.float32, device=dev)
        assert ops.classifier(xk, l1, l2, ws, y1, y2, y2f)
        outs.append((y1, y2, y2f))
    torch.cuda.synchronize()
    for y1, y2, y2f in outs:
        assert torch.equal(y1, y1_ref)
        assert torch.equal(y2, y2_ref)
        assert torch.equal(y2f, y2f_ref)


def test_classifier_head_above_65536_rows(dev):
    """The head has no row limit beyond m % 128 == 0 (the workspace holds only
    the split-K partials): 65664 rows run, and rows at both ends equal the two
    static linear kernels bit for bit."""
    from types import SimpleNamespace as NS
    from qconvnet import ops, quant as Q
    rng = np.random.default_rng(5)
    m, k, n1, n2 = 65664, 4096, 512, 10
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    xk = torch.randint(0, 256, (k // 32, m, 32), dtype=torch.uint8, device=dev)
    w1 = rng.integers(-128, 128, (n1, k), dtype=np.int8)
    w2 = rng.integers(-128, 128, (n2, n1), dtype=np.int8)
    s_x, s_y1, s_y2, s_w1, s_w2 = F32(0.02), F32(0.05), F32(0.11), F32(2e-4), F32(2e-3)
    b1 = rng.normal(0, 0.5, n1).astype(F32)
    b2 = rng.normal(0, 0.5, n2).astype(F32)
    zx, z1, z2 = 7, 0, 100
    u1, v1, m1 = Q.epilogue_constants(s_x, s_w1, s_y1, b1)
    u2, v2, m2 = Q.epilogue_constants(s_y1, s_w2, s_y2, b2)
    corr1 = ((128 - zx) * w1.astype(np.int64).sum(1)).astype(np.int32)
    corr2 = ((128 - z1) * w2.astype(np.int64).sum(1)).astype(np.int32)
    l1 = NS(w=T(w1), wk=T(ops.pack_fc_kmajor(w1)), u=T(u1), v=T(v1), mult=T(m1), corr=T(corr1),
            z_y=z1, relu=True)
    l2 = NS(w=T(w2), u=T(u2), v=T(v2), mult=T(m2), z_y=z2, relu=False, s_y=s_y2)
    ws = ops.classifier_workspace(m, n1, dev)
    y1 = torch.empty((m, n1), dtype=torch.uint8, device=dev)
    y2 = torch.empty((m, n2), dtype=torch.uint8, device=dev)
    y2f = torch.empty((m, n2), dtype=torch.float32, device=dev)
    assert ops.classifier(xk, l1, l2, ws, y1, y2, y2f)
    for sl in (slice(0, 128), slice(m - 128, m)):
        x2 = ops.from_kmajor(xk[:, sl]).contiguous()
        r1 = ops.linear_u8(x2, zx, T(w1), T(u1), T(v1), T(m1), T(corr1), z1, True)
        r2, r2f = ops.linear_u8(r1, z1, T(w2), T(u2), T(v2), T(m2), T(corr2), z2, False,
                                y_scale=s_y2, want_fp32=True)
        torch.cuda.synchronize()
        assert torch.equal(y1[sl], r1) and torch.equal(y2[sl], r2) and torch.equal(y2f[sl], r2f)


@pytest.mark.parametrize("pool", [True, False])
def test_conv_kmajor_output(dev, pool):
    """qcn_conv3x3_u8s8_kmajor writes exactly the NHWC result, chunk-major."""
    from qconvnet import ops
    rng = np.random.default_rng(3)
    n, hw, cin, cout = 12, 8, 256, 256
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    qx = rng.integers(0, 256, (n, hw, hw, cin), dtype=np.uint8)
    w = rng.integers(-128, 128, (cout, cin, 3, 3), dtype=np.int8)
    packed, wsum = ops.pack_conv3x3(w)
    u = rng.normal(0, 1, cout).astype(F32)
    v = np.full(cout, F32(1e-3), F32)
    mult = np.full(cout, F32(3e-3), F32)
    corr = ((128 - 9) * wsum.astype(np.int64)).astype(np.int32)
    args = (9, T(packed), cout, T(u), T(v), T(mult), T(corr), 0, True, pool)
    ref = ops.conv3x3(T(qx), *args)
    oh = hw // 2 if pool else hw
    out = torch.empty((oh * oh * cout // 32, n, 32), dtype=torch.uint8, device=dev)
    assert ops.conv3x3_kmajor(T(qx), *args, out)
    torch.cuda.synchronize()
    assert torch.equal(ops.from_kmajor(out), ref.view(n, -1))


@pytest.mark.parametrize("per_channel", [False, True])
def test_conv_pairs_qdq_equal_layerwise(dev, per_channel):
    """Same for the per-layer QDQ model (every qdq hand-off inside the fused
    launches)."""
    import netfix
    from qconvnet.qmodel import QuantizedConvNet
    z = netfix.load(per_channel)
    spec = netfix.qdq_spec(z)
    x = torch.from_numpy(netfix.images(z)).to(dev)
    model = QuantizedConvNet(spec, dev)
    model.fuse_convs = False
    assert "conv34" in model.kernel_names(x.shape)
    out_p = model.run(x).clone()
    a4_p = model.buffers(x.shape[0])["a4"].clone()
    model.fuse_pairs = False
    out_l = model.run(x).clone()
    torch.cuda.synchronize()
    assert torch.equal(a4_p, model.buffers(x.shape[0])["a4"])
    assert torch.equal(out_p, out_l)


@pytest.mark.parametrize("per_channel", [False, True])
def test_conv_pairs_equal_layerwise(dev, per_channel):
    """conv3+conv4 / conv5+conv6 as two pair launches (middle activations in
    LDS only) give the per-layer kernels' outputs bit for bit — the conv4
    output, the chunk-major conv6 output and the logits — and the per-layer
    path itself matches the golden fixture (test_full_net_*)."""
    import netfix
    from qconvnet import ops
    from qconvnet.qmodel import QuantizedConvNet
    z = netfix.load(per_channel)
    spec, _ = netfix.static_spec(z)
    x = torch.from_numpy(netfix.images(z)).to(dev)
    n = x.shape[0]
    model = QuantizedConvNet(spec, dev)
    model.fuse_convs = False
    assert "conv34" in model.kernel_names(x.shape)
    out_p = model.run(x).clone()
    b = model.buffers(n)
    a4_p = b["a4"].clone()
    a6_p = (ops.from_kmajor(b["a6k"]).clone() if model._head_fused(n) else b["a6"].reshape(n, -1).clone())
    model.fuse_pairs = False
    out_l = model.run(x).clone()
    b = model.buffers(n)
    a6_l = (ops.from_kmajor(b["a6k"]) if model._head_fused(n) else b["a6"].reshape(n, -1))
    torch.cuda.synchronize()
    assert torch.equal(a4_p, b["a4"])
    assert torch.equal(a6_p, a6_l)
    assert torch.equal(out_p, out_l)
    assert np.array_equal(out_p.cpu().numpy(), z["logits"])


@pytest.mark.parametrize("mode,n", [("static", n) for n in (1, 6, 255, 256, 257, 300, 511, 512, 513, 1023,
                                                           1024, 1025, 1028, 1031)] +
                         [("qdq", n) for n in (6, 256, 512, 1024, 1031)])
def test_conv_pair_workgroup_shapes_equal_layerwise(dev, mode, n):
    """conv3+conv4 and conv5+conv6 at batch sizes around their tilings (256
    CUs): at or below one image per CU conv3+4 runs one image on 8 waves and
    conv5+6 splits its output channels over two workgroups per image pair
    (the one-launch convs' 8-wave conv5+6 with lane-pooled conv6:
    test_gpu_headline::test_one_launch_convs_equal_three_launches);
    above, conv3+4 runs one image per 4-wave workgroup and conv5+6 two images
    per 4-wave workgroup; from two images per CU conv3+4, and from four conv5+6,
    run the persistent wave-specialised kernel (the last tile of conv5+6 holds
    one image when n is odd).  Static and QDQ hand-offs.  conv4's and conv6's
    outputs and the logits equal the per-layer kernels' bit for bit."""
    import netfix
    from qconvnet.qmodel import QuantizedConvNet
    from oracle import torch_ref
    spec = netfix.static_spec(netfix.load(False))[0] if mode == "static" else netfix.qdq_spec(netfix.load(False))
    x = torch.from_numpy(torch_ref.synthetic_images(n, 13)).to(dev)
    model = QuantizedConvNet(spec, dev)
    model.fuse_convs = False   # the pair launches themselves (the one-launch convs: test_gpu_headline)
    assert model.kernel_names(x.shape)[1:3] == ("conv34", "conv56")
    out_p = model.run(x).clone()
    a4_p = model.buffers(n)["a4"].clone()
    a6_p = model.buffers(n)["a6"].clone()
    model.fuse_pairs = False
    out_l = model.run(x).clone()
    a4_l = model.buffers(n)["a4"]
    a6_l = model.buffers(n)["a6"]
    torch.cuda.synchronize()
    assert torch.equal(a4_p, a4_l)
    if n % 128:   # (n % 128 == 0 writes conv6 chunk-major for the head: checked via the logits)
        assert torch.equal(a6_p, a6_l)
    if mode == "static":
        assert torch.equal(out_p, out_l)
    else:   # QDQ: the split-K head's fp32 fc2 sums in another order than linear_f32
        assert (out_p - out_l).abs().max().item() <= 1e-5 * out_l.abs().max().item()
        assert torch.equal(out_p.argmax(1), out_l.argmax(1))
