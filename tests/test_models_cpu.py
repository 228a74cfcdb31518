"""CPU checks of the drop-in model surface (no GPU): checkpoint ingestion
(main.py:22-26 / model_trainer.py:93-99 format), SimpleConvNet state-dict keys
and fp32 forward against the oracle's restatement of baseline_model.py:13-83,
and the loud failure of the int8 path on a non-GPU device."""
import pytest
import torch

from models.baseline_model import SimpleConvNet, load_checkpoint_state, synthetic_model
from oracle import torch_ref


def test_checkpoint_formats_load(tmp_path):
    m = SimpleConvNet()
    sd = m.state_dict()
    ckpt = {"epoch": 3, "model_state_dict": sd, "optimizer_state_dict": {}, "best_accuracy": 0.5}
    torch.save(ckpt, tmp_path / "best.pth")
    torch.save(sd, tmp_path / "bare.pth")
    for f in ("best.pth", "bare.pth"):
        obj = torch.load(tmp_path / f, weights_only=True)
        m2 = SimpleConvNet()
        m2.load_state_dict(load_checkpoint_state(obj))
        for k, v in sd.items():
            assert torch.equal(m2.state_dict()[k], v), k


def test_state_dict_keys_match_reference_topology():
    ours = SimpleConvNet().state_dict()
    ref = torch_ref.SimpleConvNetRef().state_dict()
    assert list(ours.keys()) == list(ref.keys())
    for k in ours:
        assert ours[k].shape == ref[k].shape, k


def test_fp32_forward_matches_restatement():
    from qconvnet import data
    calib = torch.from_numpy(data.synthetic_images(64, 1))
    m = synthetic_model(0, calib)
    r = torch_ref.SimpleConvNetRef()
    r.load_state_dict(m.state_dict())
    r.eval()
    x = torch.from_numpy(data.synthetic_images(16, 5))
    with torch.no_grad():
        assert torch.allclose(m(x), r(x), rtol=1e-5, atol=1e-5)


def test_static_ptq_wrapper_rejects_cpu_device():
    from models.static_ptq_model import StaticPTQModel
    from qconvnet.qmodel import QuantizedConvNet
    with pytest.raises(ValueError):
        QuantizedConvNet({"mode": "static"}, "cpu")
    from qconvnet import data
    sp = StaticPTQModel(device="cpu")
    sp.load_state_dict(SimpleConvNet().state_dict())
    assert hasattr(sp, "fp32_model")
    # calibration runs on the host, but the int8 model itself refuses the CPU
    with pytest.raises(ValueError):
        sp.quantize(torch.from_numpy(data.synthetic_images(8, 1)))


class _FixedLogits:
    """A model stand-in that returns a fixed logits table, one batch per call."""

    def __init__(self, logits, batch):
        self.logits, self.batch, self.i = logits, batch, 0

    def eval(self):
        return self

    def cpu(self):
        return self

    def to(self, device):
        return self

    def __call__(self, x):
        out = self.logits[self.i:self.i + x.shape[0]]
        self.i += x.shape[0]
        return out


def test_model_evaluator_matches_numpy_topk():
    """ModelEvaluator's top-1/top-5 (reference model_evaluator.py:36-41) and
    per-class accuracy (:94-112) against a numpy restatement on the same
    logits: top-k = the k largest, per-class = argmax (first max) == label."""
    import numpy as np
    from utils.model_evaluator import ModelEvaluator
    rng = np.random.default_rng(11)
    n, c, bs = 1000, 10, 128
    logits = rng.standard_normal((n, c)).astype(np.float32)
    labels = rng.integers(0, c, n)
    x = torch.zeros(n, 1)
    loader = [(x[i:i + bs], torch.from_numpy(labels[i:i + bs])) for i in range(0, n, bs)]
    ev = ModelEvaluator(loader)
    top1, top5 = ev.evaluate_accuracy(_FixedLogits(torch.from_numpy(logits), bs), verbose=False)
    order = np.argsort(-logits, axis=1, kind="stable")
    assert top1 == 100.0 * (order[:, 0] == labels).sum() / n
    assert top5 == 100.0 * (order[:, :5] == labels[:, None]).any(1).sum() / n
    classes = [f"class{i}" for i in range(c)]
    got = ev.evaluate_class_accuracy(_FixedLogits(torch.from_numpy(logits), bs), classes, verbose=False)
    pred = logits.argmax(1)
    want = {classes[k]: 100.0 * ((pred == k) & (labels == k)).sum() / (labels == k).sum() for k in range(c)}
    assert list(got) == sorted(want, key=lambda k: want[k], reverse=True)
    for k, v in want.items():
        assert abs(got[k] - v) < 1e-9
    res = ev.compare_models({"m": _FixedLogits(torch.from_numpy(logits), bs)}, classes)
    assert abs(res["m"]["accuracy"] - 100.0 * (pred == labels).sum() / n) < 1e-9


def test_custom_quantization_model_is_an_nn_module():
    """CustomQuantizationModel is an nn.Module with the fp32 SimpleConvNet as
    its `model` submodule, like the reference's (custom_quantization_model.py:
    145-151): state_dict keys carry the `model.` prefix, load_state_dict takes
    a bare SimpleConvNet state dict (:163-167), and before quantize() the
    forward is the fp32 net (:196-199)."""
    import torch
    from models.baseline_model import SimpleConvNet
    from models.custom_quantization_model import CustomQuantizationModel
    m = CustomQuantizationModel()
    assert isinstance(m, torch.nn.Module)
    keys = set(m.state_dict())
    assert {"model.conv1.weight", "model.bn7.running_var", "model.fc2.bias"} <= keys
    ref = SimpleConvNet().eval()
    m.load_state_dict(ref.state_dict())
    m.eval()
    assert not m.model.training
    x = torch.randn(2, 3, 32, 32)
    with torch.no_grad():
        assert torch.equal(m(x), ref(x))
