"""GPU parity of the one-wave-per-SIMD conv3 .. conv6 launch (qcn_convs36_u8s8,
csrc/convs36.hip, r06) — SURVEY §8(a) rows A5/A6/A10 on conv3 .. conv6
(/root/reference/models/baseline_model.py:20-33, forward :64-75):

* conv12 + conv3_6 equals the one-launch conv1 .. conv6 (and so the
  three-launch path, test_gpu_headline) bit for bit: a2, a4, conv6's output
  (chunk-major for the split-K head or NHWC), fc1 and the logits, static
  (FBGEMM fast epilogue) and per-layer QDQ (one-fma hand-off) nets, at exactly
  4 images per CU, ragged batches (phantom segments in the last conv3+4 and
  conv5+6 tiles) and several tiles per workgroup;
* the batch-1024 torch.ao fixture (tests/golden/net_static_int8_b1024.npz)
  through the two launches;
* the C entry point's argument checks."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from qconvnet import _lib
    _lib.load()
    return torch.device("cuda:0")


def _models(mode, dev):
    import netfix
    from qconvnet.qmodel import QuantizedConvNet
    z = netfix.load()
    spec = netfix.static_spec(z)[0] if mode == "static" else netfix.qdq_spec(netfix.load())
    w4, one = QuantizedConvNet(spec, dev), QuantizedConvNet(spec, dev)
    w4.convs_w4, one.convs_w4 = True, False
    return w4, one


@pytest.mark.parametrize("mode", ["static", "qdq"])
@pytest.mark.parametrize("per_cu", [4.0, 4.02, 5.5, 8.0, 16.0, 17.3])
def test_convs36_equals_one_launch(dev, mode, per_cu):
    from oracle import torch_ref
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    n = int(round(per_cu * ncu))
    w4, one = _models(mode, dev)
    x = torch.from_numpy(torch_ref.synthetic_images(n, 5)).to(dev)
    head = n % 128 == 0
    tail = ("fc12",) if head else ("fc1", "fc2")
    assert w4.kernel_names(x.shape) == ("conv12", "conv3_6") + tail
    lw = w4.run(x).clone()
    lo = one.run(x).clone()
    torch.cuda.synchronize()
    assert w4.kernel_names(x.shape) == ("conv12", "conv3_6") + tail
    assert one.kernel_names(x.shape)[0] == "conv1_6"
    bw, bo = w4.buffers(n), one.buffers(n)
    for k in ("a2", "a4", "a6k" if head else "a6", "f1"):
        assert torch.equal(bw[k], bo[k]), k
    assert torch.equal(lw, lo)


def test_convs36_equals_torchao_fixture(dev, golden_dir):
    """configs[2]: the torch.ao eager static int8 batch-1024 fixture through
    conv12 + conv3_6 + the split-K head (a2, a4, a6, fc1 by hash; logits)."""
    import netfix
    from oracle import torch_ref
    from qconvnet import ops
    from qconvnet.qmodel import QuantizedConvNet
    z = dict(np.load(os.path.join(golden_dir, "net_static_int8_b1024.npz")))
    zz = netfix.load(False)
    spec, _ = netfix.static_spec(zz)
    model = QuantizedConvNet(spec, dev)
    model.convs_w4 = True
    x = torch.from_numpy(torch_ref.synthetic_images(1024, 0)).to(dev)
    model.run(x)
    torch.cuda.synchronize()
    assert model.kernel_names(x.shape) == ("conv12", "conv3_6", "fc12")
    b = model.buffers(1024)
    assert netfix.sha(b["a2"].cpu().numpy()) == str(z["a2_sha"])
    assert netfix.sha(b["a4"].cpu().numpy()) == str(z["a4_sha"])
    a6 = ops.from_kmajor(b["a6k"]).reshape(-1, 4, 4, 256)
    assert netfix.sha(a6.cpu().numpy()) == str(z["a6_sha"])
    assert netfix.sha(b["f1"].cpu().numpy()) == str(z["fc1_sha"])
    assert np.array_equal(b["q"].cpu().numpy(), z["q_logits"])
    assert np.array_equal(b["logits"].cpu().numpy(), z["logits"])


def test_convs36_arguments(dev):
    import ctypes as C
    from qconvnet import _lib, ops
    lib = _lib.load()
    w4, _ = _models("static", dev)
    layers = ops.conv_layers(w4.L, w4.in_zp)
    l3 = C.cast(C.byref(layers, 2 * C.sizeof(_lib.ConvLayer)), C.POINTER(_lib.ConvLayer))
    a2 = torch.zeros((1024, 16, 16, 64), dtype=torch.uint8, device=dev)
    a4 = torch.empty((1024, 8, 8, 128), dtype=torch.uint8, device=dev)
    a6 = torch.empty((128, 1024, 32), dtype=torch.uint8, device=dev)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t: C.c_void_p(t.data_ptr())   # noqa: E731
    assert lib.qcn_convs36_u8s8(None, 1024, l3, p(a4), p(a6), 1, s) == _lib.QCN_ERR_ARG
    assert lib.qcn_convs36_u8s8(p(a2), 0, l3, p(a4), p(a6), 1, s) == _lib.QCN_ERR_ARG
    assert lib.qcn_convs36_u8s8(p(a2), 1024, None, p(a4), p(a6), 1, s) == _lib.QCN_ERR_ARG
    # conv4's input zero point must be conv3's output zero point
    bad = (_lib.ConvLayer * 6)(*layers)
    bad[3].x_zp = (bad[2].y_zp + 1) % 256
    lb = C.cast(C.byref(bad, 2 * C.sizeof(_lib.ConvLayer)), C.POINTER(_lib.ConvLayer))
    assert lib.qcn_convs36_u8s8(p(a2), 1024, lb, p(a4), p(a6), 1, s) == _lib.QCN_ERR_ARG
    with pytest.raises(ValueError):
        ops.convs36(a2[:, :8], layers, a4, a6)
    assert ops.convs36(a2, layers, a4, a6, kmajor=True)
    torch.cuda.synchronize()
