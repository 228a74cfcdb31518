"""CPU: the product's host-side quantization logic (qconvnet.quant / qmodel
calibration + qspec) against torch.ao, the oracle and the golden vectors."""
import os

import numpy as np
import pytest
import torch

from oracle import qref
from qconvnet import quant as Q

F32 = np.float32


def test_qparams_match_golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "ops_qparams.npz"))
    for lo, hi, s, zp, ss in zip(z["min"], z["max"], z["aff_scale"], z["aff_zp"], z["sym_scale"]):
        assert Q.qparams_affine(lo, hi) == (F32(s), int(zp))
        assert Q.qparams_symmetric(lo, hi) == F32(ss)


def test_fold_matches_torch():
    from torch.nn.utils.fusion import fuse_conv_bn_weights, fuse_linear_bn_weights
    g = torch.Generator().manual_seed(0)
    for shape in ((64, 3, 3, 3), (128, 64, 3, 3)):
        w = torch.randn(shape, generator=g)
        b = torch.randn(shape[0], generator=g)
        rm, rv = torch.randn(shape[0], generator=g), torch.rand(shape[0], generator=g) + 0.1
        ga, be = torch.randn(shape[0], generator=g), torch.randn(shape[0], generator=g)
        tw, tb = fuse_conv_bn_weights(w, b, rm, rv, 1e-5, ga, be)
        mw, mb = Q.fold_bn(w.numpy(), b.numpy(), rm.numpy(), rv.numpy(), ga.numpy(), be.numpy())
        assert np.array_equal(mw, tw.detach().numpy()) and np.array_equal(mb, tb.detach().numpy())
    w = torch.randn(512, 4096, generator=g)
    b = torch.randn(512, generator=g)
    rm, rv = torch.randn(512, generator=g), torch.rand(512, generator=g) + 0.1
    ga, be = torch.randn(512, generator=g), torch.randn(512, generator=g)
    tw, tb = fuse_linear_bn_weights(w, b, rm, rv, 1e-5, ga, be)
    mw, mb = Q.fold_linear_bn(w.numpy(), b.numpy(), rm.numpy(), rv.numpy(), ga.numpy(), be.numpy())
    assert np.array_equal(mw, tw.detach().numpy()) and np.array_equal(mb, tb.detach().numpy())


def test_weight_quant_matches_torch():
    rng = np.random.default_rng(2)
    w = (rng.standard_normal((64, 64, 3, 3)) * 0.1).astype(F32)
    s = Q.qparams_symmetric(w.min(), w.max())
    tq = torch.quantize_per_tensor(torch.from_numpy(w), float(s), 0, torch.qint8).int_repr().numpy()
    assert np.array_equal(Q.quantize_weight(w, s), tq)
    flat = w.reshape(64, -1)
    sc = Q.qparams_symmetric(flat.min(1), flat.max(1))
    tq = torch.quantize_per_channel(torch.from_numpy(w), torch.from_numpy(sc.astype(np.float64)),
                                    torch.zeros(64, dtype=torch.long), 0, torch.qint8).int_repr().numpy()
    assert np.array_equal(Q.quantize_weight(w, sc), tq)


def test_epilogue_constants_match_oracle():
    rng = np.random.default_rng(3)
    b = rng.standard_normal(64).astype(F32)
    for s_w in (F32(0.0031), rng.uniform(0.001, 0.01, 64).astype(F32)):
        mine = Q.epilogue_constants(F32(0.02), s_w, F32(0.05), b)
        ref = qref.requant_constants(F32(0.02), s_w, F32(0.05), b)
        for a, r in zip(mine, ref):
            assert np.array_equal(a, r)


def test_flatten_perm():
    assert np.array_equal(Q.nhwc_flatten_perm(), qref.flatten_perm_nhwc_to_nchw())
    x = np.arange(2 * 256 * 4 * 4).reshape(2, 256, 4, 4)
    nhwc = x.transpose(0, 2, 3, 1).reshape(2, -1)
    assert np.array_equal(nhwc[:, np.argsort(Q.nhwc_flatten_perm())], x.reshape(2, -1))


@pytest.mark.parametrize("per_channel", [False, True])
def test_quantize_flow_reproduces_torch_ao_qparams(per_channel):
    """The product's quantize() flow on the CPU (fold -> calibrate -> qspec)
    yields the same qparams and int8 weights torch.ao's prepare/convert did."""
    import netfix
    from qconvnet import data
    from qconvnet.qmodel import build_qspec, calibrate, fold_state_dict
    z = netfix.load(per_channel)
    folded = fold_state_dict(netfix.state_dict(z))
    ranges = calibrate(folded, [torch.from_numpy(data.synthetic_images(512, 1))], "cpu")
    spec = build_qspec(folded, ranges, "static", per_channel)
    assert spec["in"] == (F32(z["qm_in_scale"]), int(z["qm_in_zp"]))
    for name in [f"conv{i}" for i in range(1, 7)] + ["fc1", "fc2"]:
        assert spec[name]["s_y"] == F32(z[f"qm_{name}_scale"]), name
        assert spec[name]["z_y"] == int(z[f"qm_{name}_zp"]), name
        assert np.array_equal(np.atleast_1d(spec[name]["s_w"]), np.atleast_1d(z[f"qm_{name}_s_w"]))
    assert netfix.check_weights(spec, z) == []
    qdq = build_qspec(folded, ranges, "qdq", per_channel)
    for i in range(1, 7):
        assert qdq[f"conv{i}"]["s_x"] == F32(z[f"qdq_conv{i}_in_scale"])
        assert qdq[f"conv{i}"]["z_x"] == int(z[f"qdq_conv{i}_in_zp"])
        assert qdq[f"conv{i}"]["s_y"] == F32(z[f"qdq_conv{i}_out_scale"])
        assert qdq[f"conv{i}"]["z_y"] == int(z[f"qdq_conv{i}_out_zp"])
    assert qdq["fc1"]["s_x"] == F32(z["qdq_fc1_in_scale"])
    assert qdq["fc1"]["s_y"] == F32(z["qdq_fc1_out_scale"])


def test_spec_from_torch_ao_matches_native_flow():
    """Importing a torch.ao-converted model gives the same qspec as our flow."""
    import netfix
    from oracle import torch_ref
    from qconvnet import data
    from qconvnet.qmodel import build_qspec, calibrate, fold_state_dict, qspec_from_torch_ao
    z = netfix.load(False)
    sd = netfix.state_dict(z)
    fp = torch_ref.SimpleConvNetRef()
    fp.load_state_dict(sd)
    calib = torch.from_numpy(data.synthetic_images(512, 1))
    q = torch_ref.build_static_int8_cpu(fp.eval(), [calib])
    a = qspec_from_torch_ao(q)
    folded = fold_state_dict(sd)
    b = build_qspec(folded, calibrate(folded, [calib], "cpu"), "static")
    assert a["in"] == b["in"]
    for name in [f"conv{i}" for i in range(1, 7)] + ["fc1", "fc2"]:
        for k in ("w", "b"):
            assert np.array_equal(a[name][k], b[name][k]), (name, k)
        for k in ("s_x", "z_x", "s_y", "z_y"):
            assert a[name][k] == b[name][k], (name, k)


def test_bn_eval_affine_matches_torch_cpu():
    """bn7 of the reference StaticPTQModel runs in fp32 on the host;
    fma(x, alpha, beta') with quant.bn_eval_affine's constants reproduces
    F.batch_norm(training=False) bit for bit."""
    import torch
    from qconvnet import quant as Q
    g = torch.Generator().manual_seed(5)
    x = torch.randn(128, 512, generator=g) * 3
    mean, var = torch.randn(512, generator=g), torch.rand(512, generator=g) + 0.05
    w, b = torch.randn(512, generator=g), torch.randn(512, generator=g)
    want = torch.nn.functional.batch_norm(x, mean, var, w, b, False, 0.0, 1e-5).numpy()
    a, bp = Q.bn_eval_affine(mean.numpy(), var.numpy(), w.numpy(), b.numpy())
    got = (x.numpy().astype(np.float64) * a.astype(np.float64) + bp.astype(np.float64)).astype(np.float32)
    assert np.array_equal(got, want)
