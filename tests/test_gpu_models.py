"""GPU: the reference-shaped model surface (models.*, utils.*) end to end."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def z():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import netfix
    return netfix.load(False)


@pytest.fixture(scope="module")
def sd(z):
    import netfix
    return netfix.state_dict(z)


def _torch_ao_on_this_host(sd, calib, qdq=False):
    """The oracle built HERE: fp32 calibration results depend on the host CPU's
    oneDNN kernels, so the torch.ao reference is rebuilt on the same machine."""
    from oracle import torch_ref
    fp = torch_ref.SimpleConvNetRef()
    fp.load_state_dict(sd)
    fp.eval()
    if qdq:
        return torch_ref.build_qdq_cpu(fp, [calib])
    return torch_ref.build_static_int8_cpu(fp, [calib])


def test_static_ptq_model_dropin_bitexact(z, sd):
    """StaticPTQModel().load_state_dict(sd).quantize(loader) -> int8 GPU model
    whose logits equal torch.ao static int8 (fbgemm, same host) bit for bit."""
    import netfix
    from models.static_ptq_model import StaticPTQModel
    from qconvnet import data
    m = StaticPTQModel()
    m.load_state_dict({"model_state_dict": sd, "best_accuracy": 0.0})  # main.py:22-26 format
    loader = data.SyntheticLoader(512, 512, seed=1)                    # 512 calib images, seed 1
    q = m.quantize(loader)
    q.eval()
    q.to("cuda")
    x = torch.from_numpy(netfix.images(z))
    out = q(x.cuda()).cpu().numpy()
    with torch.no_grad():
        ref = _torch_ao_on_this_host(sd, loader.x)(x).numpy()
    assert np.array_equal(out, ref)
    assert q.quantized and m.get_model_size(q) > 0


def test_custom_quantization_model_qdq(z, sd):
    import netfix
    from models.custom_quantization_model import CustomQuantizationModel
    from qconvnet import data
    m = CustomQuantizationModel()
    m.load_state_dict(sd)
    loader = data.SyntheticLoader(512, 512, seed=1)
    m.quantize(loader)
    x = torch.from_numpy(netfix.images(z))
    out = m(x).numpy()
    with torch.no_grad():
        ref = _torch_ao_on_this_host(sd, loader.x, qdq=True)(x).numpy()
    assert np.abs(out - ref).max() <= 1e-5 * np.abs(ref).max()


def test_dynamic_models_close_to_reference(z, sd):
    """fp32 convs on the GPU differ from oneDNN in the last bits, so the dynamic
    activation scales can move by an ulp: compare with a tolerance + argmax."""
    import netfix
    from models.dynamic_ptq_model import DynamicPTQModel
    from models.static_ptq_model import StaticPTQModel
    x = torch.from_numpy(netfix.images(z))
    m = DynamicPTQModel()
    m.load_state_dict(sd)
    m.quantize()
    out = m(x).numpy()
    ref = z["dynamic_ptq_logits"]
    assert np.abs(out - ref).max() < 0.05 * np.abs(ref).max()
    assert (out.argmax(1) == ref.argmax(1)).mean() >= 0.95
    r = StaticPTQModel(mode="reference")
    r.load_state_dict(sd)
    q = r.quantize()
    out = q(x).numpy()
    ref = z["static_ptq_logits"]
    assert np.abs(out - ref).max() < 0.05 * np.abs(ref).max()
    assert (out.argmax(1) == ref.argmax(1)).mean() >= 0.95


def test_dynamic_linear_exact_on_same_input(sd):
    """Given identical fp32 input, the GPU dynamic Linear == FBGEMM exactly."""
    import torch.nn as nn
    from qconvnet import ops
    from qconvnet import quant as Q
    torch.backends.quantized.engine = "fbgemm"
    w = sd["fc1.weight"].numpy()
    lin = nn.Linear(4096, 512)
    with torch.no_grad():
        lin.weight.copy_(sd["fc1.weight"])
        lin.bias.copy_(torch.randn(512))
    dq = torch.ao.quantization.quantize_dynamic(nn.Sequential(lin), {nn.Linear}, dtype=torch.qint8)[0]
    x = torch.randn(1024, 4096) * 1.7
    ref = dq(x).detach().numpy()
    wq = dq.weight().int_repr().numpy()
    assert np.array_equal(wq, Q.quantize_weight(w, Q.qparams_symmetric(w.min(), w.max())))
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    y = ops.linear_dynamic(x.cuda(), T(wq), T(np.atleast_1d(np.float32(dq.weight().q_scale()))),
                           T(wq.astype(np.int64).sum(1).astype(np.int32)),
                           dq.bias().detach().cuda())
    assert np.array_equal(y.cpu().numpy(), ref)


def test_gpu_calibration_observer(sd):
    """calibration_device='cuda' uses the HIP observer; scales agree with the
    CPU calibration to fp32-conv rounding."""
    from qconvnet import data
    from qconvnet.qmodel import calibrate, fold_state_dict
    folded = fold_state_dict(sd)
    batches = data.calibration_batches(None)
    a = calibrate(folded, batches, "cpu")
    b = calibrate(folded, batches, "cuda")
    for k in a:
        np.testing.assert_allclose(np.array(b[k]), np.array(a[k]), rtol=1e-4, atol=1e-5)


def test_inference_benchmark_and_evaluator(sd):
    from models.static_ptq_model import StaticPTQModel
    from qconvnet import data
    from utils.inference_benchmark import InferenceBenchmark
    from utils.model_evaluator import ModelEvaluator
    m = StaticPTQModel()
    m.load_state_dict(sd)
    q = m.quantize()
    loader = data.SyntheticLoader(1024, 1024, seed=3)
    bench = InferenceBenchmark(loader, device="cuda")
    bench.warm_up(q, 3)
    thr = bench.measure_throughput(q, batch_size=1024, num_iterations=5, verbose=False)
    assert thr > 1e4
    t = bench.measure_inference_time(q, batch_size=32, num_iterations=3, verbose=False)
    assert t["batch"][0] > 0
    res = bench.compare_models({"int8": q}, batch_size=32, num_iterations=3, verbose=False)
    assert res["int8"] > 0
    with torch.no_grad():
        from models.baseline_model import SimpleConvNet
        fp = SimpleConvNet()
        fp.load_state_dict(sd)
        fp.eval()
        labels = fp(loader.x).argmax(1)
    ev = ModelEvaluator(data.SyntheticLoader(1024, 256, seed=3, labels=labels))
    top1, top5 = ev.evaluate_accuracy(q, verbose=False)
    assert top1 > 80 and top5 >= top1
