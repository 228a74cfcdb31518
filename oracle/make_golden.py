"""Generate the committed golden vectors under ``tests/golden/`` (run HERE, in
the container that has /root/reference and torch's fbgemm engine):

    python oracle/make_golden.py

What pins what:
  * per-op vectors come from torch.ao / FBGEMM (torch 2.10.0+rocm7.0 wheel,
    engine ``fbgemm``) on seeded random data, and are re-checked against the
    numpy restatement ``oracle/qref.py`` here (assertions below) and in
    ``tests/test_oracle_golden.py``;
  * the whole-net vectors come from the torch.ao eager static-int8 build of the
    restated SimpleConvNet (``oracle/torch_ref.py``); the restatement itself is
    checked against the reference's own ``models.baseline_model.SimpleConvNet``
    and ``models.static_ptq_model.StaticPTQModel`` imported from /root/reference
    (same state_dict -> identical outputs), so the fixtures are pinned to the
    reference's code, not only to our reading of it.

The reference source never leaves /root/reference: only numbers are written.
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np
import torch
import torch.ao.nn.quantized as nnq
import torch.ao.nn.intrinsic.quantized as nniq
import torch.ao.nn.quantized.dynamic as nnqd

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from oracle import qref, torch_ref as tr  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
F32 = np.float32


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def qt(arr, scale, zp, dtype=torch.quint8):
    return torch._make_per_tensor_quantized_tensor(torch.from_numpy(arr), float(scale), int(zp)) \
        if dtype == torch.quint8 else torch._make_per_tensor_quantized_tensor(
            torch.from_numpy(arr), float(scale), int(zp))


# ----------------------------------------------------------------- per-op
def gen_quantize(rng):
    cases = {}
    for i, (scale, zp) in enumerate([(0.0203, 120), (0.5, 11), (1.0, 127), (0.013, 0), (2.0 ** -7, 3)]):
        x = (rng.standard_normal(4096) * 2).astype(F32)
        # exact ties and clamping extremes
        ties = (np.arange(-40, 40) + 0.5).astype(F32) * F32(scale)
        x = np.concatenate([x, ties, np.array([1e9, -1e9, 0.0, -0.0], F32)]).astype(F32)
        q = torch.quantize_per_tensor(torch.from_numpy(x), float(scale), zp, torch.quint8).int_repr().numpy()
        assert (q == qref.quantize_per_tensor(x, scale, zp)).all(), f"quantize case {i}"
        dq = torch.quantize_per_tensor(torch.from_numpy(x), float(scale), zp, torch.quint8).dequantize().numpy()
        assert (dq == qref.dequantize(q, scale, zp)).all()
        cases[f"q{i}_x"] = x
        cases[f"q{i}_scale"] = F32(scale)
        cases[f"q{i}_zp"] = np.int64(zp)
        cases[f"q{i}_q"] = q
        cases[f"q{i}_dq"] = dq
    np.savez_compressed(os.path.join(OUT, "ops_quantize.npz"), **cases)


def gen_qparams(rng):
    import torch.ao.quantization as tq
    mins, maxs, aff_s, aff_z, sym_s = [], [], [], [], []
    for _ in range(400):
        lo = F32(-abs(rng.standard_normal()) * rng.choice([0, 0.01, 1, 10]))
        hi = F32(abs(rng.standard_normal()) * rng.choice([0, 0.01, 1, 10]))
        ob = tq.MinMaxObserver(dtype=torch.quint8, qscheme=torch.per_tensor_affine)
        ob(torch.tensor([lo, hi]))
        s, z = ob.calculate_qparams()
        sym = tq.MinMaxObserver(dtype=torch.qint8, qscheme=torch.per_tensor_symmetric)
        sym(torch.tensor([lo, hi]))
        ss, _ = sym.calculate_qparams()
        ms, mz = qref.qparams_affine(lo, hi)
        assert ms == F32(s.item()) and mz == int(z.item()), (lo, hi)
        assert qref.qparams_symmetric(lo, hi)[0] == F32(ss.item())
        mins.append(lo), maxs.append(hi), aff_s.append(s.item()), aff_z.append(z.item()), sym_s.append(ss.item())
    np.savez_compressed(os.path.join(OUT, "ops_qparams.npz"), min=np.array(mins, F32), max=np.array(maxs, F32),
                        aff_scale=np.array(aff_s, F32), aff_zp=np.array(aff_z, np.int64),
                        sym_scale=np.array(sym_s, F32))


def _conv_case(rng, n, h, cin, cout, zx, relu, per_channel, zy):
    s_x = F32(rng.uniform(0.01, 0.03))
    qx = rng.integers(0, 256, (n, h, h, cin)).astype(np.uint8)
    w = (rng.standard_normal((cout, cin, 3, 3)) * 0.05).astype(F32)
    b = (rng.standard_normal(cout) * 0.5).astype(F32)
    if per_channel:
        s_w, _ = qref.qparams_symmetric(w.reshape(cout, -1).min(1), w.reshape(cout, -1).max(1))
        wq = torch.quantize_per_channel(torch.from_numpy(w), torch.from_numpy(s_w.astype(np.float64)),
                                        torch.zeros(cout, dtype=torch.long), 0, torch.qint8)
    else:
        s_w, _ = qref.qparams_symmetric(w.min(), w.max())
        wq = torch.quantize_per_tensor(torch.from_numpy(w), float(s_w), 0, torch.qint8)
    wi = wq.int_repr().numpy()
    assert (qref.quantize_weight(w, s_w) == wi).all()
    s_y = F32(rng.uniform(0.01, 0.05))
    mod = (nniq.ConvReLU2d if relu else nnq.Conv2d)(cin, cout, 3, padding=1)
    mod.set_weight_bias(wq, torch.from_numpy(b))
    mod.scale, mod.zero_point = float(s_y), int(zy)
    xin = torch._make_per_tensor_quantized_tensor(torch.from_numpy(np.ascontiguousarray(qx.transpose(0, 3, 1, 2))),
                                                  float(s_x), int(zx))
    out = mod(xin).int_repr().permute(0, 2, 3, 1).contiguous().numpy()
    w_ohwi = np.ascontiguousarray(wi.transpose(0, 2, 3, 1))
    u, v, mult = qref.requant_constants(s_x, s_w, s_y, b)
    mine = qref.conv3x3_q(qx, zx, w_ohwi, u, v, mult, zy, relu)
    assert (mine == out).all(), f"conv case mismatch {(mine != out).sum()}"
    return dict(qx=qx, zx=np.int64(zx), s_x=s_x, w=w_ohwi, s_w=np.asarray(s_w, F32), b=b, s_y=s_y,
                zy=np.int64(zy), relu=np.int64(relu), out=out)


def gen_conv(rng):
    cases = {}
    specs = [  # n, h, cin, cout, zx, relu, per_channel, zy
        (2, 8, 3, 64, 120, True, False, 0),
        (2, 8, 64, 64, 0, True, False, 0),
        (2, 8, 64, 128, 0, False, False, 77),
        (1, 8, 128, 256, 5, True, True, 0),
        (2, 4, 256, 256, 0, True, False, 0),
        (2, 16, 64, 64, 9, False, True, 130),
    ]
    for i, sp in enumerate(specs):
        for k, v in _conv_case(rng, *sp).items():
            cases[f"c{i}_{k}"] = v
    cases["n"] = np.int64(len(specs))
    np.savez_compressed(os.path.join(OUT, "ops_conv.npz"), **cases)


def gen_linear(rng):
    cases = {}
    specs = [(16, 1024, 256, 0, True), (16, 512, 10, 0, False), (8, 64, 32, 37, False)]
    for i, (m, k, n, zx, relu) in enumerate(specs):
        s_x = F32(rng.uniform(0.01, 0.03))
        qx = rng.integers(0, 256, (m, k)).astype(np.uint8)
        w = (rng.standard_normal((n, k)) * 0.03).astype(F32)
        b = (rng.standard_normal(n) * 0.5).astype(F32)
        s_w, _ = qref.qparams_symmetric(w.min(), w.max())
        wq = torch.quantize_per_tensor(torch.from_numpy(w), float(s_w), 0, torch.qint8)
        s_y, zy = F32(rng.uniform(0.05, 0.5)), int(rng.integers(0, 200))
        if relu:
            zy = 0
        mod = (nniq.LinearReLU if relu else nnq.Linear)(k, n)
        mod.set_weight_bias(wq, torch.from_numpy(b))
        mod.scale, mod.zero_point = float(s_y), zy
        out = mod(torch._make_per_tensor_quantized_tensor(torch.from_numpy(qx), float(s_x), zx)).int_repr().numpy()
        u, v, mult = qref.requant_constants(s_x, s_w, s_y, b)
        mine = qref.linear_q(qx, zx, wq.int_repr().numpy(), u, v, mult, zy, relu)
        assert (mine == out).all(), f"linear case {i}: {(mine != out).sum()}"
        cases.update({f"l{i}_qx": qx, f"l{i}_zx": np.int64(zx), f"l{i}_s_x": s_x, f"l{i}_w": wq.int_repr().numpy(),
                      f"l{i}_s_w": F32(s_w), f"l{i}_b": b, f"l{i}_s_y": s_y, f"l{i}_zy": np.int64(zy),
                      f"l{i}_relu": np.int64(relu), f"l{i}_out": out})
    cases["n"] = np.int64(len(specs))
    np.savez_compressed(os.path.join(OUT, "ops_linear.npz"), **cases)


def gen_dynamic_linear(rng):
    torch.backends.quantized.engine = "fbgemm"
    cases = {}
    specs = [(32, 1024, 256), (32, 512, 10), (7, 256, 33)]
    for i, (m, k, n) in enumerate(specs):
        lin = torch.nn.Linear(k, n)
        with torch.no_grad():
            lin.weight.copy_(torch.from_numpy((rng.standard_normal((n, k)) * 0.03).astype(F32)))
            lin.bias.copy_(torch.from_numpy((rng.standard_normal(n) * 0.3).astype(F32)))
        dq = torch.ao.quantization.quantize_dynamic(
            torch.nn.Sequential(lin), {torch.nn.Linear}, dtype=torch.qint8)[0]
        x = (rng.standard_normal((m, k)) * rng.uniform(0.5, 3)).astype(F32)
        y = dq(torch.from_numpy(x)).detach().numpy()
        wq = dq.weight()
        mine = qref.linear_dynamic(x, wq.int_repr().numpy(), F32(wq.q_scale()), dq.bias().detach().numpy())
        assert (mine == y).all(), f"dynamic linear case {i}: {(mine != y).sum()} / {y.size}"
        cases.update({f"d{i}_x": x, f"d{i}_w": wq.int_repr().numpy(), f"d{i}_s_w": F32(wq.q_scale()),
                      f"d{i}_b": dq.bias().detach().numpy().astype(F32), f"d{i}_y": y})
    cases["n"] = np.int64(len(specs))
    np.savez_compressed(os.path.join(OUT, "ops_dynamic_linear.npz"), **cases)


# ----------------------------------------------------------------- whole net
def extract_qmodel(q, per_channel=False):
    """Pull the quantized parameters out of the torch.ao static-int8 model into
    the oracle's dict form (qref.static_int8_forward)."""
    qm = {"in_scale": F32(q.quant.scale.item()), "in_zp": int(q.quant.zero_point.item())}
    s_x = qm["in_scale"]
    for name in [f"conv{i}" for i in range(1, 7)] + ["fc1", "fc2"]:
        m = getattr(q, name)
        w = m.weight()
        wi = w.int_repr().numpy()
        if name.startswith("conv"):
            wi = np.ascontiguousarray(wi.transpose(0, 2, 3, 1))
        if w.qscheme() == torch.per_tensor_symmetric or w.qscheme() == torch.per_tensor_affine:
            s_w = F32(w.q_scale())
        else:
            s_w = w.q_per_channel_scales().numpy().astype(F32)
        b = m.bias().detach().numpy().astype(F32)
        s_y, z_y = F32(m.scale), int(m.zero_point)
        u, v, mult = qref.requant_constants(s_x, s_w, s_y, b)
        if name == "fc1":
            wi = np.ascontiguousarray(wi[:, qref.flatten_perm_nhwc_to_nchw()])
        qm.update({name + "_w": wi, name + "_u": u, name + "_v": v, name + "_mult": mult,
                   name + "_zp": z_y, name + "_scale": s_y, name + "_s_w": np.asarray(s_w, F32),
                   name + "_b": b})
        s_x = s_y
    return qm


REF_ROOT = "/root/reference"


def import_reference(module, names):
    """Import ``names`` from the reference's ``module`` (read-only, from
    REF_ROOT) or return None when that tree is absent: the cross-checks that
    run the reference's own classes are opt-in, and the generator still writes
    the fixtures without them (saying so).  The reference imports torchvision
    at the top of models/custom_quantization_model.py (:4) and never uses it;
    the wheel is not installed here, so an empty module stands in for it
    during the import.  The reference's ``models`` package is imported under
    its own name and removed from sys.modules afterwards (ours shares it)."""
    import importlib
    import types
    if not os.path.isdir(os.path.join(REF_ROOT, "models")):
        print(f"note: {REF_ROOT} absent: skipping the cross-check against the reference's {module}")
        return None
    saved = {k: v for k, v in sys.modules.items() if k == "models" or k.startswith("models.")}
    for k in saved:
        del sys.modules[k]
    stub = "torchvision" not in sys.modules
    if stub:
        sys.modules["torchvision"] = types.ModuleType("torchvision")
    sys.path.insert(0, REF_ROOT)
    try:
        mod = importlib.import_module(module)
        return [getattr(mod, n) for n in names]
    finally:
        sys.path.pop(0)
        for k in [k for k in sys.modules if k == "models" or k.startswith("models.")]:
            del sys.modules[k]
        sys.modules.update(saved)
        if stub:
            del sys.modules["torchvision"]


def check_restatement_against_reference(sd):
    """Import the reference models (read-only, here only) and check that our
    restated topology and our StaticPTQModel counterpart agree bit-for-bit."""
    got = import_reference("models.baseline_model", ["SimpleConvNet"])
    got2 = import_reference("models.static_ptq_model", ["StaticPTQModel"])
    if got is None or got2 is None:
        return False
    (SimpleConvNet,), (StaticPTQModel,) = got, got2
    x = torch.from_numpy(tr.synthetic_images(16, 5))
    ref = SimpleConvNet()
    ref.load_state_dict(sd)
    ref.eval()
    mine = tr.SimpleConvNetRef()
    mine.load_state_dict(sd)
    mine.eval()
    with torch.no_grad():
        assert torch.equal(ref(x), mine(x)), "SimpleConvNet restatement differs"
        sp = StaticPTQModel()
        sp.fp32_model.load_state_dict(sd)
        ref_q = sp.quantize()
        my_q = tr.build_static_ptq_cpu(mine)
        assert torch.equal(ref_q(x), my_q(x)), "StaticPTQModel counterpart differs"
    return True


def gen_net(per_channel=False, batch=64):
    torch.manual_seed(0)
    torch.set_num_threads(8)
    calib = tr.synthetic_images(512, 1)
    fp = tr.reference_fp32_model(0, calib)
    sd = fp.state_dict()
    check_restatement_against_reference(sd)
    q = tr.build_static_int8_cpu(fp, [torch.from_numpy(calib)], per_channel=per_channel)
    qm = extract_qmodel(q, per_channel)
    x = tr.synthetic_images(batch, 0)
    with torch.no_grad():
        ref = q(torch.from_numpy(x)).numpy()
    logits, ql, inter = qref.static_int8_forward(x, qm, keep=True)
    assert (logits == ref).all(), "oracle != torch.ao static int8"
    # torch.ao intermediates (NHWC u8) for the per-layer hashes
    outs = {}
    hooks = [getattr(q, f"conv{i}").register_forward_hook(
        lambda m, a, o, k=i: outs.__setitem__(k, o)) for i in range(1, 7)]
    with torch.no_grad():
        q(torch.from_numpy(x))
    for h in hooks:
        h.remove()
    rec = {"batch": np.int64(batch), "x_sha": sha(x), "logits": ref, "q_logits": ql,
           "argmax": qref.argmax_rows(ref), "per_channel": np.int64(per_channel)}
    for i in range(1, 7):
        o = outs[i].int_repr().permute(0, 2, 3, 1).contiguous().numpy()
        if i % 2 == 0:
            o = qref.maxpool2x2_nhwc(o)
        assert (o == inter[f"conv{i}"]).all()
        rec[f"conv{i}_sha"] = sha(o)
        rec[f"conv{i}_slice"] = o[:2, :2, :2, :].copy()
    rec["fc1_sha"] = sha(inter["fc1"])
    # BN statistics after recalibration (the only non-regenerable fp32 state)
    for i in range(1, 8):
        rec[f"bn{i}_mean"] = sd[f"bn{i}.running_mean"].numpy()
        rec[f"bn{i}_var"] = sd[f"bn{i}.running_var"].numpy()
    # quantized parameters: scales/zps in full, int8 weights by hash
    for k, v in qm.items():
        if k.endswith("_w") and not k.endswith("_s_w"):
            rec[k + "_sha"] = sha(v)
        else:
            rec["qm_" + k] = np.asarray(v)
    # CPU reference paths on the same batch (top-1 parity anchors)
    with torch.no_grad():
        xt = torch.from_numpy(x)
        rec["fp32_logits"] = fp(xt).numpy()
        rec["static_ptq_logits"] = tr.build_static_ptq_cpu(fp)(xt).numpy()
        rec["dynamic_ptq_logits"] = tr.build_dynamic_ptq_cpu(fp)(xt).numpy()
        qdq = tr.build_qdq_cpu(fp, [torch.from_numpy(calib)], per_channel=per_channel)
        rec["qdq_logits"] = qdq(xt).numpy()
        for i in range(1, 7):
            c = getattr(qdq, f"conv{i}")
            rec[f"qdq_conv{i}_in_scale"] = F32(c.quant.scale.item())
            rec[f"qdq_conv{i}_in_zp"] = np.int64(c.quant.zero_point.item())
            rec[f"qdq_conv{i}_out_scale"] = F32(c.op.scale)
            rec[f"qdq_conv{i}_out_zp"] = np.int64(c.op.zero_point)
        rec["qdq_fc1_in_scale"] = F32(qdq.fc1.quant.scale.item())
        rec["qdq_fc1_in_zp"] = np.int64(qdq.fc1.quant.zero_point.item())
        rec["qdq_fc1_out_scale"] = F32(qdq.fc1.op.scale)
        rec["qdq_fc1_out_zp"] = np.int64(qdq.fc1.op.zero_point)
    name = "net_static_int8_pc.npz" if per_channel else "net_static_int8.npz"
    np.savez_compressed(os.path.join(OUT, name), **rec)
    return rec


def _nchw_flat_to_nhwc(qflat, c=256, h=4):
    """[n, c*h*h] in NCHW flatten order -> [n, h, h, c] (our conv6 layout)."""
    return np.ascontiguousarray(qflat.reshape(-1, c, h, h).transpose(0, 2, 3, 1))


def gen_net_headline(per_channel=False, batch=1024):
    """BASELINE configs[2] (full static int8, batch 1024): the same model and
    calibration as gen_net, run by torch.ao eager/fbgemm over 1024 images.
    Records what the product's default launch sequence (conv12 -> conv34 ->
    conv56 (chunk-major) -> fused classifier head) leaves in HBM: a2, a4, a6,
    fc1 by hash, the u8 and fp32 logits in full."""
    torch.manual_seed(0)
    torch.set_num_threads(8)
    calib = tr.synthetic_images(512, 1)
    fp = tr.reference_fp32_model(0, calib)
    q = tr.build_static_int8_cpu(fp, [torch.from_numpy(calib)], per_channel=per_channel)
    qm = extract_qmodel(q, per_channel)
    x = tr.synthetic_images(batch, 0)
    outs = {}
    hooks = [getattr(q, f"conv{i}").register_forward_hook(
        lambda m, a, o, k=i: outs.__setitem__(k, o)) for i in (2, 4, 6)]
    hooks.append(q.fc1.register_forward_hook(lambda m, a, o: outs.__setitem__("fc1", o)))
    hooks.append(q.fc2.register_forward_hook(lambda m, a, o: outs.__setitem__("fc2", o)))
    with torch.no_grad():
        ref = q(torch.from_numpy(x)).numpy()
    for h in hooks:
        h.remove()
    logits, ql, inter = qref.static_int8_forward(x, qm, keep=True)
    assert (logits == ref).all(), "oracle != torch.ao static int8 at the headline batch"
    rec = {"batch": np.int64(batch), "x_sha": sha(x), "logits": ref,
           "q_logits": outs["fc2"].int_repr().numpy(), "argmax": qref.argmax_rows(ref),
           "per_channel": np.int64(per_channel), "qm_in_scale": qm["in_scale"],
           "qm_in_zp": np.int64(qm["in_zp"])}
    assert (rec["q_logits"] == ql).all()
    for i, a in ((2, "a2"), (4, "a4"), (6, "a6")):
        o = qref.maxpool2x2_nhwc(outs[i].int_repr().permute(0, 2, 3, 1).contiguous().numpy())
        assert (o == inter[f"conv{i}"]).all()
        rec[f"{a}_sha"] = sha(o)
    f1 = outs["fc1"].int_repr().numpy()
    assert (f1 == inter["fc1"]).all()
    rec["fc1_sha"] = sha(f1)
    name = "net_static_int8_b1024_pc.npz" if per_channel else "net_static_int8_b1024.npz"
    np.savez_compressed(os.path.join(OUT, name), **rec)
    return rec


def gen_qdq_config2(batch=256):
    """BASELINE configs[1] (per-layer QDQ CustomQuantizedSimpleConvNet, batch
    256): torch.ao's integer chain at every stub (each layer's input as the
    next QuantStub quantizes it, NHWC, by hash) and fc1's u8 output, plus the
    fp32 logits."""
    torch.manual_seed(0)
    torch.set_num_threads(8)
    calib = tr.synthetic_images(512, 1)
    fp = tr.reference_fp32_model(0, calib)
    qdq = tr.build_qdq_cpu(fp, [torch.from_numpy(calib)])
    x = tr.synthetic_images(batch, 2)
    outs = {}
    hooks = [getattr(qdq, f"conv{i}").quant.register_forward_hook(
        lambda m, a, o, k=i: outs.__setitem__(f"in{k}", o)) for i in range(1, 7)]
    hooks.append(qdq.fc1.quant.register_forward_hook(lambda m, a, o: outs.__setitem__("in_fc1", o)))
    hooks.append(qdq.fc1.op.register_forward_hook(lambda m, a, o: outs.__setitem__("fc1", o)))
    with torch.no_grad():
        ref = qdq(torch.from_numpy(x)).numpy()
    for h in hooks:
        h.remove()
    pinned = reference_qdq_simpleconvnet(fp.state_dict(), [torch.from_numpy(calib)], x, outs, ref)
    rec = {"batch": np.int64(batch), "x_sha": sha(x), "logits": ref, "argmax": qref.argmax_rows(ref),
           "pinned_to_reference_class": np.int64(bool(pinned))}
    for i in range(2, 7):   # our a_{i-1} = conv_{i-1}'s QDQ hand-off = conv_i's quantized input
        o = outs[f"in{i}"].int_repr().permute(0, 2, 3, 1).contiguous().numpy()
        rec[f"a{i - 1}_sha"] = sha(o)
    rec["a6_sha"] = sha(_nchw_flat_to_nhwc(outs["in_fc1"].int_repr().numpy()))
    rec["fc1_sha"] = sha(outs["fc1"].int_repr().numpy())
    np.savez_compressed(os.path.join(OUT, "net_qdq_b256.npz"), **rec)
    return rec


def reference_qdq_simpleconvnet(state_dict, calib_batches, x, outs, logits):
    """Pin the config-2 restatement (torch_ref._QDQNet) to the reference's own
    CustomQuantizationModel / CustomQuantizedSimpleConvNet
    (/root/reference/models/custom_quantization_model.py:145-261), imported
    read-only: the same state_dict, CustomQuantizationModel.quantize() (its
    conv+bn / fc1+bn7 fusion, :169-195), a qconfig on every
    CustomQuantizedConv2d / CustomQuantizedLinear (their QuantStub -> op ->
    DeQuantStub run live; the outer stubs :205-206 carry none and stay
    identities), MinMax calibration on the same batches, then
    convert.  Every per-layer stub's quantized tensor, fc1's u8 output and the
    logits must equal _QDQNet's (``outs``, ``logits``) bit for bit.

    The reference's forward flattens with ``x.view(-1, 256 * 4 * 4)`` (:255),
    which fails on the channels-last tensor its quantized convs hand back; the
    harness therefore wraps ``pool3`` so its output is made contiguous (a copy,
    values unchanged) — nothing else in the reference's code path is touched.
    Returns False (and writes the fixture unpinned) when /root/reference is
    absent."""
    import torch.nn as nn
    import torch.ao.quantization as tq
    got = import_reference("models.custom_quantization_model",
                           ["CustomQuantizationModel", "CustomQuantizedConv2d", "CustomQuantizedLinear"])
    if got is None:
        return False
    CustomQuantizationModel, CustomQuantizedConv2d, CustomQuantizedLinear = got
    torch.backends.quantized.engine = "fbgemm"
    cm = CustomQuantizationModel()
    cm.load_state_dict(state_dict)
    net = cm.quantize().eval()
    for m in net.modules():
        if isinstance(m, (CustomQuantizedConv2d, CustomQuantizedLinear)):
            m.qconfig = tr.static_qconfig(False)

    class _Contig(nn.Module):
        def __init__(self, pool):
            super().__init__()
            self.pool = pool

        def forward(self, t):
            return self.pool(t).contiguous()

    net.pool3 = _Contig(net.pool3)
    tq.prepare(net, inplace=True)
    with torch.no_grad():
        for xb in calib_batches:
            net(xb)
    tq.convert(net, inplace=True)
    got_outs = {}
    hooks = [getattr(net, f"conv{i}").quant.register_forward_hook(
        lambda m, a, o, k=i: got_outs.__setitem__(f"in{k}", o)) for i in range(1, 7)]
    hooks.append(net.fc1.quant.register_forward_hook(lambda m, a, o: got_outs.__setitem__("in_fc1", o)))
    hooks.append(net.fc1.linear.register_forward_hook(lambda m, a, o: got_outs.__setitem__("fc1", o)))
    with torch.no_grad():
        ref_logits = net(torch.from_numpy(x)).numpy()
    for h in hooks:
        h.remove()
    for k in [f"in{i}" for i in range(1, 7)] + ["in_fc1", "fc1"]:
        a, b = got_outs[k], outs[k]
        assert a.q_scale() == b.q_scale() and a.q_zero_point() == b.q_zero_point(), f"{k}: qparams"
        assert torch.equal(a.int_repr(), b.int_repr()), f"{k}: _QDQNet differs from CustomQuantizedSimpleConvNet"
    assert ref_logits.dtype == logits.dtype and (ref_logits == logits).all(), "config-2 logits"
    print("config 2: _QDQNet equals the reference's CustomQuantizedSimpleConvNet at every stub and in the logits")
    return True


# ------------------------------------------- SURVEY §8(f)2 (ResNet blocks)
def _convgen_case(rng, n, h, cin, cout, k, stride, pad, zx, relu, per_channel, zy):
    s_x = F32(rng.uniform(0.01, 0.03))
    qx = rng.integers(0, 256, (n, h, h, cin)).astype(np.uint8)
    w = (rng.standard_normal((cout, cin, k, k)) * 0.05).astype(F32)
    b = (rng.standard_normal(cout) * 0.5).astype(F32)
    if per_channel:
        s_w, _ = qref.qparams_symmetric(w.reshape(cout, -1).min(1), w.reshape(cout, -1).max(1))
        wq = torch.quantize_per_channel(torch.from_numpy(w), torch.from_numpy(s_w.astype(np.float64)),
                                        torch.zeros(cout, dtype=torch.long), 0, torch.qint8)
    else:
        s_w, _ = qref.qparams_symmetric(w.min(), w.max())
        wq = torch.quantize_per_tensor(torch.from_numpy(w), float(s_w), 0, torch.qint8)
    wi = wq.int_repr().numpy()
    assert (qref.quantize_weight(w, s_w) == wi).all()
    s_y = F32(rng.uniform(0.01, 0.05))
    mod = (nniq.ConvReLU2d if relu else nnq.Conv2d)(cin, cout, k, stride=stride, padding=pad)
    mod.set_weight_bias(wq, torch.from_numpy(b))
    mod.scale, mod.zero_point = float(s_y), int(zy)
    xin = torch._make_per_tensor_quantized_tensor(
        torch.from_numpy(np.ascontiguousarray(qx.transpose(0, 3, 1, 2))), float(s_x), int(zx))
    out = mod(xin).int_repr().permute(0, 2, 3, 1).contiguous().numpy()
    u, v, mult = qref.requant_constants(s_x, s_w, s_y, b)
    mine = qref.conv_q(qx, zx, wi, u, v, mult, zy, relu, (stride, stride), (pad, pad))
    assert (mine == out).all(), f"general conv case mismatch {(mine != out).sum()}"
    return dict(qx=qx, zx=np.int64(zx), s_x=s_x, w=wi, s_w=np.asarray(s_w, F32), b=b, s_y=s_y,
                zy=np.int64(zy), relu=np.int64(relu), stride=np.int64(stride), pad=np.int64(pad),
                out=out)


def gen_resnet_ops(rng):
    """General convs (1x1, strided 3x3, strided 1x1 downsample, the 7x7/2 stem)
    against torch.ao's QuantizedConv(ReLU)2d; the residual join against aten
    dequantize + add + relu + quantize_per_tensor; maxpool 3x3/2 against
    torch's quantized max_pool2d."""
    cases = {}
    specs = [  # n, h, cin, cout, k, stride, pad, zx, relu, per_channel, zy
        (2, 8, 64, 64, 1, 1, 0, 0, True, True, 0),
        (2, 8, 64, 256, 1, 1, 0, 0, False, True, 121),
        (2, 9, 64, 64, 3, 2, 1, 3, True, True, 0),
        (2, 8, 128, 256, 1, 2, 0, 0, False, True, 64),
        (2, 8, 32, 128, 3, 1, 1, 200, True, False, 0),
        (1, 17, 3, 64, 7, 2, 3, 114, True, True, 0),
    ]
    for i, sp in enumerate(specs):
        for k, v in _convgen_case(rng, *sp).items():
            cases[f"c{i}_{k}"] = v
    cases["n"] = np.int64(len(specs))
    # residual join: out.dequantize() + identity.dequantize(), relu, quantize
    adds = [(0.021, 130, 0.017, 0, 0.03, 0), (0.05, 0, 0.05, 0, 0.061, 0), (0.013, 255, 0.02, 7, 0.01, 0)]
    for i, (sa, za, sb, zb, so, zo) in enumerate(adds):
        qa = rng.integers(0, 256, (2, 7, 7, 64)).astype(np.uint8)
        qb = rng.integers(0, 256, (2, 7, 7, 64)).astype(np.uint8)
        ta = torch._make_per_tensor_quantized_tensor(torch.from_numpy(qa), sa, za)
        tb = torch._make_per_tensor_quantized_tensor(torch.from_numpy(qb), sb, zb)
        s = torch.relu(ta.dequantize() + tb.dequantize())
        out = torch.quantize_per_tensor(s, so, zo, torch.quint8).int_repr().numpy()
        mine = qref.add_relu_q(qa, sa, za, qb, sb, zb, so, zo, True)
        assert (mine == out).all(), "add case mismatch"
        cases.update({f"a{i}_qa": qa, f"a{i}_qb": qb, f"a{i}_p": np.array([sa, sb, so], F32),
                      f"a{i}_z": np.array([za, zb, zo], np.int64), f"a{i}_out": out})
    cases["na"] = np.int64(len(adds))
    qm = rng.integers(0, 256, (2, 15, 15, 64)).astype(np.uint8)
    tq = torch._make_per_tensor_quantized_tensor(torch.from_numpy(qm.transpose(0, 3, 1, 2).copy()), 0.1, 3)
    mp = torch.nn.functional.max_pool2d(tq, 3, 2, 1).int_repr().permute(0, 2, 3, 1).contiguous().numpy()
    assert (qref.maxpool3x3s2_nhwc(qm) == mp).all()
    cases["mp_in"], cases["mp_out"] = qm, mp
    np.savez_compressed(os.path.join(OUT, "ops_resnet.npz"), **cases)


def _resnet_spec_from_torchao(q):
    """The oracle's ResNet spec (qref.resnet_int8_forward's format, the same
    as qconvnet.resnet.build_spec's) read out of a converted ResNetRef."""
    def layer(m, s_x, z_x, relu, stride, pad):
        wq = m.weight()
        s_w = (F32(wq.q_scale()) if wq.qscheme() in (torch.per_tensor_affine, torch.per_tensor_symmetric)
               else wq.q_per_channel_scales().numpy().astype(F32))
        return dict(w=wq.int_repr().numpy(), b=m.bias().detach().numpy().astype(F32), s_w=s_w,
                    s_x=F32(s_x), z_x=int(z_x), s_y=F32(m.scale), z_y=int(m.zero_point), relu=relu,
                    stride=(stride, stride), pad=(pad, pad))
    spec = {"per_channel": True, "blocks": [],
            "in": (F32(q.quant.scale.item()), int(q.quant.zero_point.item()))}
    spec["stem"] = layer(q.conv1, *spec["in"], True, 2, 3)
    s_x, z_x = spec["stem"]["s_y"], spec["stem"]["z_y"]
    for li in range(1, 5):
        for blk in getattr(q, f"layer{li}"):
            st = blk.conv2.stride[0]
            e = {"c1": layer(blk.conv1, s_x, z_x, True, 1, 0)}
            e["c2"] = layer(blk.conv2, e["c1"]["s_y"], e["c1"]["z_y"], True, st, 1)
            e["c3"] = layer(blk.conv3, e["c2"]["s_y"], e["c2"]["z_y"], False, 1, 0)
            e["ds"] = (layer(blk.downsample[0], s_x, z_x, False, blk.downsample[0].stride[0], 0)
                       if blk.downsample is not None else None)
            e["out"] = (F32(blk.q_out.scale.item()), int(blk.q_out.zero_point.item()))
            spec["blocks"].append(e)
            s_x, z_x = e["out"]
    fc = q.fc
    wq = fc.weight()
    spec["fc"] = dict(w=wq.int_repr().numpy(), b=fc.bias().detach().numpy().astype(F32),
                      s_w=wq.q_per_channel_scales().numpy().astype(F32), s_x=s_x, z_x=z_x,
                      s_y=F32(fc.scale), z_y=int(fc.zero_point), relu=False)
    return spec


def gen_resnet_net(layers=(1, 1, 1, 1), hw=64, n=8, num_classes=10):
    """SURVEY §8(f)2 whole-network pin: a 1-1-1-1 bottleneck ResNet at 64x64
    as torch.ao eager static int8 (fbgemm; per-channel MinMax weights, MinMax
    u8 activations, float-domain residual join, quantized max-pool /
    avg-pool / fc), calibrated on the CPU.  Stores what regenerates the model
    (BN running statistics; weights come from torch_ref.resnet_state_dict),
    every qparam, int8-weight hashes, every block's u8 output by hash, the
    pooled u8 features and the logits; asserts the numpy oracle
    (qref.resnet_int8_forward) reproduces it bit for bit."""
    torch.manual_seed(0)
    torch.set_num_threads(8)
    imnet = dict(mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225), hw=hw)
    fp = tr.ResNetRef(layers, num_classes)
    fp.load_state_dict(tr.resnet_state_dict(fp, 0))
    tr.recalibrate_bn(fp, torch.from_numpy(tr.synthetic_images(16, 3, **imnet)))
    calib = tr.synthetic_images(8, 4, **imnet)
    q = tr.build_resnet_static_int8_cpu(fp, [torch.from_numpy(calib)])
    x = tr.synthetic_images(n, 5, **imnet)
    outs, order = {}, []
    hooks = [q.maxpool.register_forward_hook(lambda m, a, o: outs.__setitem__("stem", o)),
             q.avgpool.register_forward_hook(lambda m, a, o: outs.__setitem__("pool", o)),
             q.fc.register_forward_hook(lambda m, a, o: outs.__setitem__("fc", o))]
    for li in range(1, 5):
        for bi, blk in enumerate(getattr(q, f"layer{li}")):
            k = f"block{len(order)}"
            order.append(k)
            hooks.append(blk.register_forward_hook(lambda m, a, o, k=k: outs.__setitem__(k, o)))
    with torch.no_grad():
        logits = q(torch.from_numpy(x)).numpy()
    for h in hooks:
        h.remove()
    spec = _resnet_spec_from_torchao(q)
    mine, inter = qref.resnet_int8_forward(x, spec, keep=True)
    nhwc = lambda t: t.int_repr().permute(0, 2, 3, 1).contiguous().numpy()  # noqa: E731
    assert (inter["stem"] == nhwc(outs["stem"])).all(), "stem"
    for k in order:
        assert (inter[k] == nhwc(outs[k])).all(), k
    pool = outs["pool"].int_repr().reshape(n, -1).numpy()
    assert (inter["pool"] == pool).all(), "avgpool"
    assert (mine == logits).all(), "logits"
    rec = {"layers": np.asarray(layers, np.int64), "hw": np.int64(hw), "batch": np.int64(n),
           "num_classes": np.int64(num_classes), "x_sha": sha(x), "calib_sha": sha(calib),
           "logits": logits, "q_logits": outs["fc"].int_repr().numpy(), "pool": pool,
           "stem_sha": sha(inter["stem"])}
    for k in order:
        rec[f"{k}_sha"] = sha(inter[k])
    for k, v in fp.state_dict().items():   # BN running statistics (the recalibrated state)
        if k.endswith("running_mean") or k.endswith("running_var"):
            rec["sd." + k] = v.numpy()
    rec["in_q"] = np.asarray(spec["in"][0], F32), np.int64(spec["in"][1])
    rec["in_scale"], rec["in_zp"] = F32(spec["in"][0]), np.int64(spec["in"][1])
    def put(name, e):
        rec[name + ".s_y"], rec[name + ".z_y"] = F32(e["s_y"]), np.int64(e["z_y"])
        rec[name + ".w_sha"] = sha(e["w"])
    put("stem", spec["stem"])
    for i, e in enumerate(spec["blocks"]):
        for k in ("c1", "c2", "c3", "ds"):
            if e[k] is not None:
                put(f"b{i}.{k}", e[k])
        rec[f"b{i}.out_scale"], rec[f"b{i}.out_zp"] = F32(e["out"][0]), np.int64(e["out"][1])
    put("fc", spec["fc"])
    del rec["in_q"]
    np.savez_compressed(os.path.join(OUT, "net_resnet_int8.npz"), **rec)
    return rec


def _resnet_qdq_spec_from_torchao(q):
    """The oracle's reference-semantics ResNet spec (qref.resnet_qdq_forward's
    format = qconvnet.resnet_qdq.build_spec's) read out of a converted
    RefQDQResNet: per stub (s_x, z_x), per int8 conv its weights, scales,
    output qparams and geometry, per BN its eval constants."""
    def conv(m, bn):
        op = m.op
        wq = op.weight()
        b = op.bias()
        e = dict(w=wq.int_repr().numpy(), s_w=wq.q_per_channel_scales().numpy().astype(F32),
                 b=(np.zeros(wq.shape[0], F32) if b is None else b.detach().numpy().astype(F32)),
                 s_x=F32(m.quant.scale.item()), z_x=int(m.quant.zero_point.item()),
                 s_y=F32(op.scale), z_y=int(op.zero_point))
        if bn is not None:
            e["stride"], e["pad"] = tuple(op.stride), tuple(op.padding)
            e["bn"] = qref.bn_eval_constants(bn.running_mean.numpy(), bn.running_var.numpy(),
                                             bn.weight.detach().numpy(), bn.bias.detach().numpy(), bn.eps)
        return e

    spec = {"per_channel": True, "stem": conv(q.conv1, q.bn1), "blocks": []}
    for li in range(1, 5):
        for blk in getattr(q, f"layer{li}"):
            e = {k: conv(getattr(blk, k), getattr(blk, "bn" + k[-1])) for k in ("conv1", "conv2", "conv3")}
            e = {"c1": e["conv1"], "c2": e["conv2"], "c3": e["conv3"], "ds": None}
            if blk.downsample is not None:
                e["ds"] = conv(blk.downsample[0], blk.downsample[1])
            spec["blocks"].append(e)
    spec["fc"] = conv(q.fc, None)
    return spec


def reference_resnet_qdq(fp, calib_batches, per_channel=True):
    """The reference's OWN CustomQuantizedResNet50 / CustomQuantizedBottleneck
    (/root/reference/models/custom_quantization_model.py:60-143), imported
    read-only from /root/reference, wrapped around a copy of the same ResNetRef
    and converted the way torch.ao eager converts RefQDQResNet: a qconfig on
    every CustomQuantizedConv2d / CustomQuantizedLinear (their QuantStub ->
    op -> DeQuantStub run live), MinMax calibration on the same batches, then
    convert.  The outer QuantStub / DeQuantStub (:107-108) carry no qconfig
    and stay identities, as in RefQDQResNet.

    Imported through import_reference (None when /root/reference is absent:
    the caller then skips this pin)."""
    import copy
    import torch.nn as nn
    import torch.ao.quantization as tq
    got = import_reference("models.custom_quantization_model",
                           ["CustomQuantizedConv2d", "CustomQuantizedLinear", "CustomQuantizedResNet50"])
    if got is None:
        return None
    CustomQuantizedConv2d, CustomQuantizedLinear, CustomQuantizedResNet50 = got
    net = copy.deepcopy(fp).eval()
    for li in range(1, 5):   # torchvision Bottleneck attributes the wrapper reads (:63-71)
        for b in getattr(net, f"layer{li}"):
            b.relu = nn.ReLU()
            b.stride = b.conv2.stride[0]
    torch.backends.quantized.engine = "fbgemm"
    ref = CustomQuantizedResNet50(net).eval()
    for m in ref.modules():
        if isinstance(m, (CustomQuantizedConv2d, CustomQuantizedLinear)):
            m.qconfig = tr.static_qconfig(per_channel)
    tq.prepare(ref, inplace=True)
    with torch.no_grad():
        for xb in calib_batches:
            ref(xb)
    tq.convert(ref, inplace=True)
    return ref.eval()


def gen_resnet_qdq_net(layers=(1, 1, 1, 1), hw=64, n=8, num_classes=10):
    """§8(f)2 in the reference's own semantics: the same 1-1-1-1 ResNet at
    64x64 as CustomQuantizedResNet50 with live per-layer stubs
    (torch_ref.RefQDQResNet, torch.ao eager, fbgemm, CPU calibration; asserted
    equal, block by block and in the logits, to the reference's own
    CustomQuantizedResNet50 built the same way — reference_resnet_qdq):
    fp32 BN / ReLU / max-pool / residual add / avg-pool between int8 convs.
    Stores every stub's and conv's qparams, int8-weight hashes, every conv's
    u8 output and every block's fp32 output by hash, the fc's u8 output and
    the logits; asserts the numpy oracle (qref.resnet_qdq_forward)
    reproduces every one bit for bit."""
    torch.manual_seed(0)
    torch.set_num_threads(8)
    imnet = dict(mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225), hw=hw)
    fp = tr.ResNetRef(layers, num_classes)
    fp.load_state_dict(tr.resnet_state_dict(fp, 0))
    tr.recalibrate_bn(fp, torch.from_numpy(tr.synthetic_images(16, 3, **imnet)))
    calib = tr.synthetic_images(8, 4, **imnet)
    q = tr.build_resnet_qdq_cpu(fp, [torch.from_numpy(calib)])
    x = tr.synthetic_images(n, 5, **imnet)
    outs, hooks = {}, []

    def grab(mod, key):
        hooks.append(mod.register_forward_hook(lambda m, a, o: outs.__setitem__(key, o)))

    grab(q.conv1.op, "stem.q")
    grab(q.maxpool, "stem")
    grab(q.avgpool, "pool")
    grab(q.fc.op, "fc.q")
    bi = 0
    for li in range(1, 5):
        for blk in getattr(q, f"layer{li}"):
            for k in ("conv1", "conv2", "conv3"):
                grab(getattr(blk, k).op, f"block{bi}.c{k[-1]}")
            if blk.downsample is not None:
                grab(blk.downsample[0].op, f"block{bi}.ds")
            grab(blk, f"block{bi}")
            bi += 1
    with torch.no_grad():
        logits = q(torch.from_numpy(x)).numpy()
    for h in hooks:
        h.remove()
    # pin the restatement to the reference's own classes: same fp32 net, same
    # calibration -> every block's fp32 output and the logits bit for bit
    ref = reference_resnet_qdq(fp, [torch.from_numpy(calib)])
    if ref is not None:
        ref_outs, hooks = {}, []
        bi = 0
        for li in range(1, 5):
            for blk in getattr(ref, f"layer{li}"):
                hooks.append(blk.register_forward_hook(
                    lambda m, a, o, key=f"block{bi}": ref_outs.__setitem__(key, o)))
                bi += 1
        with torch.no_grad():
            ref_logits = ref(torch.from_numpy(x)).numpy()
        for h in hooks:
            h.remove()
        assert ref_logits.dtype == logits.dtype and (ref_logits == logits).all(), \
            "RefQDQResNet differs from the reference's CustomQuantizedResNet50"
        for k, t in ref_outs.items():
            assert torch.equal(t, outs[k]), f"{k}: RefQDQBottleneck differs from CustomQuantizedBottleneck"
    spec = _resnet_qdq_spec_from_torchao(q)
    mine, inter = qref.resnet_qdq_forward(x, spec, keep=True)
    nhwc = lambda t: t.permute(0, 2, 3, 1).contiguous().numpy()  # noqa: E731
    rec = {"layers": np.asarray(layers, np.int64), "hw": np.int64(hw), "batch": np.int64(n),
           "num_classes": np.int64(num_classes), "x_sha": sha(x), "calib_sha": sha(calib),
           "logits": logits}
    for k, t in outs.items():
        if k == "pool":
            ref = t.reshape(n, -1).numpy()
        elif t.is_quantized:
            ref = t.int_repr().numpy() if t.dim() == 2 else nhwc(t.int_repr())
        else:
            ref = nhwc(t)
        assert ref.dtype == inter[k].dtype and (ref == inter[k]).all(), k
        rec[k + "_sha"] = sha(inter[k])
    assert (mine == logits).all(), "logits"
    rec["q_logits"] = inter["fc.q"]
    for k, v in fp.state_dict().items():   # BN running statistics (the recalibrated state)
        if k.endswith("running_mean") or k.endswith("running_var"):
            rec["sd." + k] = v.numpy()

    def put(name, e):
        rec[name + ".s_x"], rec[name + ".z_x"] = F32(e["s_x"]), np.int64(e["z_x"])
        rec[name + ".s_y"], rec[name + ".z_y"] = F32(e["s_y"]), np.int64(e["z_y"])
        rec[name + ".w_sha"] = sha(e["w"])
    put("stem", spec["stem"])
    for i, e in enumerate(spec["blocks"]):
        for k in ("c1", "c2", "c3", "ds"):
            if e[k] is not None:
                put(f"b{i}.{k}", e[k])
    put("fc", spec["fc"])
    np.savez_compressed(os.path.join(OUT, "net_resnet_qdq.npz"), **rec)
    return rec


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.backends.quantized.engine = "fbgemm"
    if sys.argv[1:] == ["resnet"]:   # only the §8(f)2 vectors
        gen_resnet_ops(np.random.Generator(np.random.PCG64(4321)))
        return
    if sys.argv[1:] == ["resnet_net"]:   # only the §8(f)2 whole-net vectors
        gen_resnet_net()
        return
    if sys.argv[1:] == ["resnet_qdq"]:   # only the §8(f)2 reference-semantics vectors
        gen_resnet_qdq_net()
        return
    if sys.argv[1:] == ["headline"]:   # only the batch-1024 / batch-256 whole-net vectors
        gen_net_headline(per_channel=False)
        gen_net_headline(per_channel=True)
        gen_qdq_config2()
        return
    rng = np.random.Generator(np.random.PCG64(1234))
    gen_quantize(rng)
    gen_qparams(rng)
    gen_conv(rng)
    gen_linear(rng)
    gen_dynamic_linear(rng)
    gen_net(per_channel=False)
    gen_net(per_channel=True)
    gen_net_headline(per_channel=False)
    gen_net_headline(per_channel=True)
    gen_qdq_config2()
    gen_resnet_ops(np.random.Generator(np.random.PCG64(4321)))
    gen_resnet_net()
    gen_resnet_qdq_net()
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
