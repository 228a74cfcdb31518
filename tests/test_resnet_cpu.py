"""CPU checks of the §8(f)2 host logic: the fp32 ResNet restatement keeps
torchvision's state-dict layout, BN folding preserves the fp32 function, and
the calibrated static-int8 spec run through the oracle tracks the fp32 net."""
import numpy as np
import torch
import torch.nn.functional as F

from oracle import qref


def _small():
    from models.resnet import synthetic_resnet
    return synthetic_resnet(0, (1, 1, 1, 1), num_classes=10, hw=64, calib_images=4)


def test_resnet50_state_dict_layout():
    from models.resnet import resnet50
    sd = resnet50().state_dict()
    assert len([k for k in sd if k.endswith("conv1.weight")]) == 17
    assert sd["layer3.0.downsample.0.weight"].shape == (1024, 512, 1, 1)
    assert sd["layer4.2.conv2.weight"].shape == (512, 512, 3, 3)
    assert sd["fc.weight"].shape == (1000, 2048)
    assert sum(v.numel() for k, v in sd.items() if "running" not in k and "num_batches" not in k) \
        == 25557032   # torchvision resnet50 parameter count


def test_fold_preserves_fp32_function():
    from qconvnet.resnet import fold_state_dict
    from models.resnet import synthetic_images
    m = _small()
    f = fold_state_dict(m.state_dict())
    x = torch.from_numpy(synthetic_images(2, 3, 64))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    with torch.no_grad():
        ref = m(x)
        y = F.max_pool2d(F.relu(F.conv2d(x, t(f["stem"][0]), t(f["stem"][1]), stride=2, padding=3)),
                         3, 2, 1)
        for b in f["blocks"]:
            cv = lambda inp, k: F.conv2d(inp, t(b[k][0]), t(b[k][1]), stride=b[k][2],  # noqa: E731
                                         padding=b[k][3])
            o = cv(F.relu(cv(F.relu(cv(y, "c1")), "c2")), "c3")
            y = F.relu(o + (cv(y, "ds") if "ds" in b else y))
        y = F.linear(y.mean((2, 3)), t(f["fc"][0]), t(f["fc"][1]))
    assert torch.allclose(y, ref, rtol=1e-4, atol=1e-4)


def test_static_int8_spec_tracks_fp32():
    from qconvnet.resnet import build_spec, calibrate, fold_state_dict
    from models.resnet import synthetic_images
    m = _small()
    f = fold_state_dict(m.state_dict())
    ranges = calibrate(f, [torch.from_numpy(synthetic_images(8, 11, 64))], "cpu")
    spec = build_spec(f, ranges, per_channel=True)
    assert spec["stem"]["s_w"].shape == (64,) and spec["stem"]["z_y"] == 0
    assert spec["blocks"][0]["ds"] is not None and spec["blocks"][1]["ds"] is not None
    x = synthetic_images(4, 12, 64)
    logits, inter = qref.resnet_int8_forward(x, spec, keep=True)
    with torch.no_grad():
        ref = m(torch.from_numpy(x)).numpy()
    assert np.abs(logits - ref).max() / np.abs(ref).max() < 0.3
    assert inter["block3"].shape == (4, 2, 2, 2048)


def test_oracle_matches_torchao_resnet_fixture():
    """§8(f)2 pin: torch.ao eager static int8 of a 1-1-1-1 bottleneck ResNet
    at 64x64 (tests/golden/net_resnet_int8.npz) == the numpy oracle run on the
    product's own folded / quantized weights: stem, every block, the pooled
    features and the logits, bit for bit."""
    import resnetfix
    z = resnetfix.load()
    sp = resnetfix.spec(z)
    assert resnetfix.check_weights(sp, z) == []
    logits, inter = qref.resnet_int8_forward(resnetfix.images(z), sp, keep=True)
    assert resnetfix.sha(inter["stem"]) == str(z["stem_sha"])
    for i in range(len(sp["blocks"])):
        assert resnetfix.sha(inter[f"block{i}"]) == str(z[f"block{i}_sha"]), i
    assert np.array_equal(inter["pool"], z["pool"])
    assert np.array_equal(logits, z["logits"])


def test_product_cpu_calibration_reproduces_torchao_qparams():
    """The product's CPU calibration (qconvnet.resnet.calibrate, default device)
    over the fixture's calibration images gives torch.ao's observer qparams
    exactly (same fp32 ops on the same folded weights)."""
    import resnetfix
    from qconvnet.resnet import build_spec, calibrate, fold_state_dict
    z = resnetfix.load()
    folded = fold_state_dict(resnetfix.fp32_model(z).state_dict())
    ranges = calibrate(folded, [torch.from_numpy(resnetfix.images(z, "calib"))])
    sp = build_spec(folded, ranges, per_channel=True)
    assert (np.float32(sp["in"][0]), sp["in"][1]) == (np.float32(z["in_scale"]), int(z["in_zp"]))
    assert (sp["stem"]["s_y"], sp["stem"]["z_y"]) == (np.float32(z["stem.s_y"]), int(z["stem.z_y"]))
    for i, e in enumerate(sp["blocks"]):
        for k in ("c1", "c2", "c3", "ds"):
            if e[k] is not None:
                assert (e[k]["s_y"], e[k]["z_y"]) == (np.float32(z[f"b{i}.{k}.s_y"]),
                                                      int(z[f"b{i}.{k}.z_y"])), (i, k)
        assert (np.float32(e["out"][0]), e["out"][1]) == (np.float32(z[f"b{i}.out_scale"]),
                                                          int(z[f"b{i}.out_zp"])), i
    assert (sp["fc"]["s_y"], sp["fc"]["z_y"]) == (np.float32(z["fc.s_y"]), int(z["fc.z_y"]))


def test_reference_semantics_oracle_and_host_spec_pinned():
    """§8(f)2 in the reference's semantics (CustomQuantizedResNet50 with live
    per-layer stubs, fp32 BN / ReLU / add / pools between int8 convs): the
    PRODUCT host code (unfolded weights, CPU calibration, qparams, per-channel
    int8 weights, BN eval constants) reproduces torch.ao's converted model,
    and the numpy oracle run on that spec reproduces every conv's u8 output,
    every block's fp32 output and the logits of the golden bit for bit."""
    import hashlib
    import resnetfix
    z = resnetfix.load_qdq()
    sp = resnetfix.qdq_spec(z)
    assert resnetfix.check_qdq_spec(sp, z) == []
    logits, inter = qref.resnet_qdq_forward(resnetfix.images(z), sp, keep=True)
    for k in [k[:-4] for k in z if k.endswith("_sha") and not k.endswith(".w_sha")
              and k not in ("x_sha", "calib_sha")]:
        assert hashlib.sha256(np.ascontiguousarray(inter[k]).tobytes()).hexdigest() == str(z[k + "_sha"]), k
    assert np.array_equal(logits, z["logits"])


def test_bn_eval_constants_product_equals_oracle():
    from qconvnet import quant as Q
    rng = np.random.default_rng(3)
    m, v, g, b = (rng.standard_normal(256).astype(np.float32) for _ in range(4))
    v = np.abs(v) + np.float32(0.01)
    pa, pb = Q.bn_eval_affine(m, v, g, b)
    oa, ob = qref.bn_eval_constants(m, v, g, b)
    assert np.array_equal(pa, oa) and np.array_equal(pb, ob)
