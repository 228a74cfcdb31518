"""CPU: the oracle (oracle/qref.py) against the committed torch.ao/fbgemm
golden vectors — the pin that makes every GPU parity claim meaningful."""
import os

import numpy as np
import pytest

from oracle import qref

F32 = np.float32


def _g(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name)))


def test_quantize_dequantize(golden_dir):
    z = _g(golden_dir, "ops_quantize.npz")
    for i in range(5):
        q = qref.quantize_per_tensor(z[f"q{i}_x"], z[f"q{i}_scale"], int(z[f"q{i}_zp"]))
        assert np.array_equal(q, z[f"q{i}_q"])
        assert np.array_equal(qref.dequantize(q, z[f"q{i}_scale"], int(z[f"q{i}_zp"])), z[f"q{i}_dq"])


def test_observer_qparams(golden_dir):
    z = _g(golden_dir, "ops_qparams.npz")
    for lo, hi, s, zp, ss in zip(z["min"], z["max"], z["aff_scale"], z["aff_zp"], z["sym_scale"]):
        assert qref.qparams_affine(lo, hi) == (F32(s), int(zp))
        assert qref.qparams_symmetric(lo, hi)[0] == F32(ss)


def test_conv_requant(golden_dir):
    z = _g(golden_dir, "ops_conv.npz")
    for i in range(int(z["n"])):
        g = lambda k: z[f"c{i}_{k}"]  # noqa: E731
        s_w = g("s_w")
        u, v, mult = qref.requant_constants(g("s_x"), s_w, g("s_y"), g("b"))
        out = qref.conv3x3_q(g("qx"), int(g("zx")), g("w"), u, v, mult, int(g("zy")), bool(g("relu")))
        assert np.array_equal(out, g("out")), i


def test_linear_requant(golden_dir):
    z = _g(golden_dir, "ops_linear.npz")
    for i in range(int(z["n"])):
        g = lambda k: z[f"l{i}_{k}"]  # noqa: E731
        u, v, mult = qref.requant_constants(g("s_x"), g("s_w"), g("s_y"), g("b"))
        out = qref.linear_q(g("qx"), int(g("zx")), g("w"), u, v, mult, int(g("zy")), bool(g("relu")))
        assert np.array_equal(out, g("out")), i


def test_dynamic_linear(golden_dir):
    z = _g(golden_dir, "ops_dynamic_linear.npz")
    for i in range(int(z["n"])):
        y = qref.linear_dynamic(z[f"d{i}_x"], z[f"d{i}_w"], z[f"d{i}_s_w"], z[f"d{i}_b"])
        assert np.array_equal(y, z[f"d{i}_y"]), i


def test_fmaf_exact():
    """The vectorised fmaf helper equals a single-rounding FMA: checked against
    exact rational arithmetic on adversarial near-tie inputs."""
    from fractions import Fraction
    rng = np.random.default_rng(0)
    a = rng.standard_normal(2000).astype(F32)
    b = (np.ldexp(1.0, rng.integers(-30, 30, 2000)) * rng.uniform(1, 2, 2000)).astype(F32)
    c = np.ldexp(rng.integers(-(1 << 24), 1 << 24, 2000).astype(np.float64), rng.integers(-5, 40, 2000)).astype(F32)
    got = qref.fmaf(a, b, c)
    for x, y, w, r in zip(a[:400], b[:400], c[:400], got[:400]):
        exact = Fraction(float(x)) * Fraction(float(y)) + Fraction(float(w))
        lo = np.float32(float(exact))
        cands = [np.nextafter(lo, np.float32(-np.inf)), lo, np.nextafter(lo, np.float32(np.inf))]
        best = min(cands, key=lambda f: (abs(Fraction(float(f)) - exact),
                                          int(np.float32(f).view(np.int32)) & 1))
        assert r == best


@pytest.mark.parametrize("per_channel", [False, True])
def test_full_net_oracle(per_channel):
    """Oracle whole-net forward with the product's host quantization of the
    seeded weights == torch.ao logits (first 8 images: the static path is
    batch-independent)."""
    import netfix
    z = netfix.load(per_channel)
    spec, _ = netfix.static_spec(z)
    assert netfix.check_weights(spec, z) == []
    x = netfix.images(z)[:8]
    logits, q, inter = qref.static_int8_forward(x, netfix.oracle_dict(spec), keep=True)
    assert np.array_equal(q, z["q_logits"][:8])
    assert np.array_equal(logits, z["logits"][:8])
    assert np.array_equal(inter["conv1"][:2, :2, :2], z["conv1_slice"])


@pytest.mark.parametrize("per_channel", [False, True])
def test_headline_fixture_oracle(golden_dir, per_channel):
    """The batch-1024 fixture (configs[2]) is the same model and calibration
    as the batch-64 one: same input qparams, its first 64 images are the
    batch-64 images with the same logits, and the oracle reproduces a slice
    of it (images 1000..1007)."""
    import netfix
    from oracle import torch_ref
    z = netfix.load(per_channel)
    h = _g(golden_dir, "net_static_int8_b1024_pc.npz" if per_channel else "net_static_int8_b1024.npz")
    assert int(h["batch"]) == 1024
    assert (F32(h["qm_in_scale"]), int(h["qm_in_zp"])) == (F32(z["qm_in_scale"]), int(z["qm_in_zp"]))
    assert np.array_equal(h["q_logits"][:64], z["q_logits"])
    assert np.array_equal(h["logits"][:64], z["logits"])
    assert np.array_equal(h["argmax"], qref.argmax_rows(h["logits"]))
    spec, _ = netfix.static_spec(z)
    x = torch_ref.synthetic_images(1024, 0)
    assert netfix.sha(x) == str(h["x_sha"])
    logits, q, _ = qref.static_int8_forward(x[1000:1008], netfix.oracle_dict(spec), keep=True)
    assert np.array_equal(q, h["q_logits"][1000:1008])
    assert np.array_equal(logits, h["logits"][1000:1008])


def test_qdq_config2_fixture(golden_dir):
    """The batch-256 QDQ fixture (configs[1]) is self-consistent: its argmax
    is the argmax of its logits, and its input is seed-2 synthetic data."""
    import netfix
    from oracle import torch_ref
    h = _g(golden_dir, "net_qdq_b256.npz")
    assert int(h["batch"]) == 256 and h["logits"].shape == (256, 10)
    assert netfix.sha(torch_ref.synthetic_images(256, 2)) == str(h["x_sha"])
    assert np.array_equal(h["argmax"], qref.argmax_rows(h["logits"]))


def test_resnet_ops(golden_dir):
    """§8(f)2 ops: general convs (1x1, strided 3x3 / 1x1, 7x7/2 stem), the
    residual join and maxpool 3x3/2 against torch.ao / aten vectors."""
    z = _g(golden_dir, "ops_resnet.npz")
    for i in range(int(z["n"])):
        g = lambda k: z[f"c{i}_{k}"]  # noqa: E731
        u, v, mult = qref.requant_constants(g("s_x"), g("s_w"), g("s_y"), g("b"))
        st, pd = int(g("stride")), int(g("pad"))
        out = qref.conv_q(g("qx"), int(g("zx")), g("w"), u, v, mult, int(g("zy")), bool(g("relu")),
                          (st, st), (pd, pd))
        assert np.array_equal(out, g("out")), i
    for i in range(int(z["na"])):
        sa, sb, so = z[f"a{i}_p"]
        za, zb, zo = (int(t) for t in z[f"a{i}_z"])
        out = qref.add_relu_q(z[f"a{i}_qa"], sa, za, z[f"a{i}_qb"], sb, zb, so, zo, True)
        assert np.array_equal(out, z[f"a{i}_out"]), i
    assert np.array_equal(qref.maxpool3x3s2_nhwc(z["mp_in"]), z["mp_out"])


def test_stem_rows_equal_stem_conv():
    """The packed-row stem (stem_pack + a 7x1 conv with strides (2,1)) is the
    7x7/2/3 conv exactly — the identity the GPU stem relies on."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "convnet-quantization_amd"))
    from qconvnet.ops import stem_weight_rows
    rng = np.random.default_rng(5)
    x = rng.standard_normal((2, 3, 19, 21)).astype(F32)
    w = rng.integers(-128, 128, (64, 3, 7, 7)).astype(np.int8)
    s, zp = F32(0.021), 117
    acc_ref = qref.conv_acc_nhwc(qref.quantize_per_tensor(qref.nchw_to_nhwc(x), s, zp), zp, w,
                                 (2, 2), (3, 3))
    rows = qref.stem_pack(x, s, zp)
    acc = qref.conv_acc_nhwc(rows, zp, stem_weight_rows(w), (2, 1), (3, 0))
    assert np.array_equal(acc, acc_ref)


def test_config2_fixture_pinned_to_reference_class(golden_dir):
    """net_qdq_b256.npz was written after oracle/make_golden.py checked the
    restated _QDQNet against the reference's own CustomQuantizedSimpleConvNet
    (every per-layer stub, fc1's u8 output and the logits bit for bit;
    make_golden.reference_qdq_simpleconvnet)."""
    z = np.load(os.path.join(golden_dir, "net_qdq_b256.npz"))
    assert int(z["pinned_to_reference_class"]) == 1
