"""GPU parity at the BASELINE configs themselves (not at a reduced batch):

* configs[2] — full static int8 at batch 1024: the DEFAULT launch sequence
  bench.py times (since r04 conv1 .. conv6 in one persistent launch with
  chunk-major output -> the classifier head; before, conv12 -> conv34 ->
  conv56 -> head, still the path below 4 images per CU) bit-exact to torch.ao eager static int8 (fbgemm) over the
  same 1024 images (tests/golden/net_static_int8_b1024*.npz, written by
  oracle/make_golden.py's gen_net_headline): a2, a4, conv6's chunk-major
  output, fc1 by hash; u8 and fp32 logits in full;
* configs[3]'s total batch (8192 = 8 x 1024) on one GPU: every 1024 shard
  equals the 1024 run and the first shard equals the fixture;
* configs[1] — the per-layer QDQ CustomQuantizedSimpleConvNet at batch 256
  (tests/golden/net_qdq_b256.npz, gen_qdq_config2): every QuantStub's u8
  hand-off and fc1's u8 output bit-exact, fp32 logits within 1e-5 relative
  (fc2 is an fp32 GEMM whose summation order differs from MKL's)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HEADLINE = ("conv1_6", "fc12")
THREE = ("conv12", "conv34", "conv56", "fc12")   # fuse_convs=False / < 4 images per CU


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from qconvnet import _lib
    _lib.load()
    return torch.device("cuda:0")


def _fixture(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name)))


def _headline_model(per_channel, dev):
    import netfix
    from qconvnet.qmodel import QuantizedConvNet
    z = netfix.load(per_channel)   # same model + calibration as the batch-1024 fixture
    spec, _ = netfix.static_spec(z)
    assert netfix.check_weights(spec, z) == []
    return QuantizedConvNet(spec, dev)


def _check_headline_bufs(model, n, z, rows=slice(None)):
    import netfix
    from qconvnet import ops
    b = model.buffers(n)
    assert netfix.sha(b["a2"][rows].cpu().numpy()) == str(z["a2_sha"])
    assert netfix.sha(b["a4"][rows].cpu().numpy()) == str(z["a4_sha"])
    a6 = ops.from_kmajor(b["a6k"])[rows].reshape(-1, 4, 4, 256)
    assert netfix.sha(a6.cpu().numpy()) == str(z["a6_sha"])
    assert netfix.sha(b["f1"][rows].cpu().numpy()) == str(z["fc1_sha"])
    assert np.array_equal(b["q"][rows].cpu().numpy(), z["q_logits"])
    assert np.array_equal(b["logits"][rows].cpu().numpy(), z["logits"])


@pytest.mark.parametrize("per_channel", [False, True])
def test_headline_launch_sequence_equals_torchao(dev, golden_dir, per_channel):
    import netfix
    from oracle import torch_ref
    z = _fixture(golden_dir, "net_static_int8_b1024_pc.npz" if per_channel else "net_static_int8_b1024.npz")
    model = _headline_model(per_channel, dev)
    assert (model.in_scale, model.in_zp) == (np.float32(z["qm_in_scale"]), int(z["qm_in_zp"]))
    n = int(z["batch"])
    x = torch_ref.synthetic_images(n, 0)
    assert netfix.sha(x) == str(z["x_sha"])
    xd = torch.from_numpy(x).to(dev)
    model.run(xd)
    torch.cuda.synchronize()
    assert model.kernel_names(xd.shape) == HEADLINE
    _check_headline_bufs(model, n, z)
    # the HIP-graph replay of the same sequence
    model.capture_graph(xd.clone())
    out = model.replay(n)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), z["logits"])
    assert np.array_equal(model(torch.from_numpy(x)).argmax(1).numpy(), z["argmax"])


@pytest.mark.parametrize("mode", ["static", "qdq"])
@pytest.mark.parametrize("n", [6, 256, 1024, 1031, 1539, 2048])
def test_one_launch_convs_equal_three_launches(dev, golden_dir, mode, n):
    """conv1 .. conv6 in one persistent launch (qcn_convnet_convs_f32_nchw):
    a2, a4, conv6's output and the logits equal the three-launch path
    (conv12 -> conv3+4 -> conv5+6) bit for bit: one image per workgroup at
    <= 1 image per CU (6, 256: the 8-wave small-batch phases), exactly 4
    images per CU, ragged batches (some workgroups one image more, a last
    conv5+6 tile with one image) and 8 per CU; static and per-layer QDQ (the
    one-fma hand-off form) nets."""
    import netfix
    from oracle import torch_ref
    from qconvnet.qmodel import QuantizedConvNet
    z = netfix.load()
    spec = netfix.static_spec(z)[0] if mode == "static" else netfix.qdq_spec(netfix.load())
    one, three = QuantizedConvNet(spec, dev), QuantizedConvNet(spec, dev)
    three.fuse_convs = False
    x = torch.from_numpy(torch_ref.synthetic_images(n, 3)).to(dev)
    head = n % 128 == 0   # the split-K head's row tile; else fc1 / fc2 launches on NHWC a6
    # the library's rule (include/qconvnet.h): one image per workgroup up to
    # one image per CU, the persistent form from four; three launches between
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    fused = n <= ncu or n >= 4 * ncu
    tail = ("fc12",) if head else ("fc1", "fc2")
    want_one = (("conv1_6",) if fused else THREE[:3]) + tail
    # kernel_names is right before the first forward (the library's host
    # query) and after it (what the run recorded)
    assert one.kernel_names(x.shape) == want_one
    l1 = one.run(x).clone()
    l3 = three.run(x).clone()
    torch.cuda.synchronize()
    assert one.kernel_names(x.shape) == want_one
    assert three.kernel_names(x.shape) == THREE[:3] + tail
    b1, b3 = one.buffers(n), three.buffers(n)
    for k in ("a2", "a4", "a6k" if head else "a6", "f1"):
        assert torch.equal(b1[k], b3[k]), k
    assert torch.equal(l1, l3)


def test_batch_8192_shards_equal_1024(dev, golden_dir):
    """configs[3]'s total batch on one GPU: the 8192 run equals its eight 1024
    shards bit for bit (what each rank computes), and its first 1024 rows (the
    same PCG64 stream) equal the torch.ao fixture."""
    from oracle import torch_ref
    z = _fixture(golden_dir, "net_static_int8_b1024.npz")
    model = _headline_model(False, dev)
    x = torch.from_numpy(torch_ref.synthetic_images(8192, 0)).to(dev)
    full = model.run(x).clone()
    torch.cuda.synchronize()
    assert model.kernel_names(x.shape) == HEADLINE
    _check_headline_bufs(model, 8192, z, rows=slice(0, 1024))
    for r in range(8):
        part = model.run(x[r * 1024:(r + 1) * 1024].contiguous())
        torch.cuda.synchronize()
        assert torch.equal(part, full[r * 1024:(r + 1) * 1024]), r


def test_config2_qdq_batch256_equals_torchao(dev, golden_dir):
    import netfix
    from oracle import torch_ref
    from qconvnet import ops
    from qconvnet.qmodel import QuantizedConvNet
    z = _fixture(golden_dir, "net_qdq_b256.npz")
    spec = netfix.qdq_spec(netfix.load(False))
    n = int(z["batch"])
    x = torch_ref.synthetic_images(n, 2)
    assert netfix.sha(x) == str(z["x_sha"])
    xd = torch.from_numpy(x).to(dev)
    model = QuantizedConvNet(spec, dev)
    # default launches at 256 images (<= one per CU): conv1 .. conv6 in one
    # launch (one image per workgroup) with a2, a4, a6 (chunk-major for the
    # split-K head) as its HBM hand-offs, then the split-K QDQ head
    assert model.kernel_names(xd.shape) == HEADLINE
    tol = 1e-5 * np.abs(z["logits"]).max()
    logits = model.run(xd).cpu().numpy()
    assert model.kernel_names(xd.shape) == HEADLINE   # the launches this forward ran
    b = model.buffers(n)
    for a in ("a2", "a4"):
        assert netfix.sha(b[a].cpu().numpy()) == str(z[f"{a}_sha"]), a
    a6 = ops.from_kmajor(b["a6k"]).view(n, 4, 4, 256)
    assert netfix.sha(a6.cpu().numpy()) == str(z["a6_sha"])
    assert netfix.sha(b["f1"].cpu().numpy()) == str(z["fc1_sha"])
    assert np.abs(logits - z["logits"]).max() <= tol
    assert np.array_equal(logits.argmax(1), z["argmax"])
    # the HIP-graph replay bench.py times for config 2: the same bytes
    model.capture_graph(xd.clone())
    out = model.replay(n)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), logits)
    # per-layer launches (keep=True, conv1 unfused): every stub's hand-off
    m2 = QuantizedConvNet(spec, dev, fuse12=False)
    logits2, b = m2.run(xd, keep=True)
    for i in range(1, 7):
        assert netfix.sha(b[f"a{i}"].cpu().numpy()) == str(z[f"a{i}_sha"]), i
    assert netfix.sha(b["f1"].cpu().numpy()) == str(z["fc1_sha"])
    # per-layer fc2 (linear_f32) sums in another fp32 order than the head
    assert np.abs(logits2.cpu().numpy() - z["logits"]).max() <= tol
    assert np.array_equal(logits2.cpu().numpy().argmax(1), z["argmax"])


def test_qdq_head_equals_two_linears(dev, golden_dir):
    """QDQ split-K head (fc1 int8 -> dequantize -> ReLU -> fp32 fc2 in the
    finisher) against the per-layer fc1 (linear_u8s8) + fp32 fc2
    (linear_f32) launches on the same conv6 output: fc1's u8 output
    identical, fp32 logits within the stated fp32 tolerance (different
    summation orders), same argmax; at 384 images (3 row blocks)."""
    import netfix
    from oracle import torch_ref
    from qconvnet.qmodel import QuantizedConvNet
    spec = netfix.qdq_spec(netfix.load(False))
    x = torch.from_numpy(torch_ref.synthetic_images(384, 5)).to(dev)
    model = QuantizedConvNet(spec, dev)
    assert model.kernel_names(x.shape)[-1] == "fc12"
    head = model.run(x).clone()
    f1_head = model.buffers(384)["f1"].clone()
    model.fc_head = False
    assert model.kernel_names(x.shape)[-2:] == ("fc1", "fc2")
    lin = model.run(x).clone()
    torch.cuda.synchronize()
    assert torch.equal(f1_head, model.buffers(384)["f1"])
    tol = 1e-5 * lin.abs().max().item()
    assert (head - lin).abs().max().item() <= tol
    assert torch.equal(head.argmax(1), lin.argmax(1))


def test_model_on_second_device(golden_dir):
    """A model built for cuda:1 runs there while cuda:0 is current (every
    forward enters the model's device; kernel attributes are set per device)."""
    if not torch.cuda.is_available() or torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    from oracle import torch_ref
    z = _fixture(golden_dir, "net_static_int8_b1024.npz")
    torch.cuda.set_device(0)
    model = _headline_model(False, torch.device("cuda:1"))
    x = torch.from_numpy(torch_ref.synthetic_images(1024, 0)).to("cuda:1")
    out = model.run(x)
    torch.cuda.synchronize("cuda:1")
    assert np.array_equal(out.cpu().numpy(), z["logits"])


def test_run_pipelined_equals_sequential(dev, golden_dir):
    """Two batches in flight on two streams (run_pipelined, one activation
    buffer set per stream): every batch's logits equal its own single-stream
    run, and the first equals the torch.ao fixture."""
    from oracle import torch_ref
    z = _fixture(golden_dir, "net_static_int8_b1024.npz")
    model = _headline_model(False, dev)
    xs = [torch.from_numpy(torch_ref.synthetic_images(1024, s)).to(dev) for s in (0, 11, 12, 13)]
    want = [model.run(x).clone() for x in xs]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    got = []
    for k in range(0, 4, 2):   # the slot buffers are reused every len(streams) batches
        got += [o.clone() for o in model.run_pipelined(xs[k:k + 2], streams)]
    torch.cuda.synchronize()
    for g, w in zip(got, want):
        assert torch.equal(g, w)
    assert np.array_equal(got[0].cpu().numpy(), z["logits"])
