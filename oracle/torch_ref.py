"""CPU reference models built on torch.ao (TEST INFRASTRUCTURE ONLY).

Used by ``oracle/make_golden.py`` (fixture generation, in this container) and
by ``bench.py``'s ``cpu_baseline`` leg (timed on the GPU box's host cores).
Never imported by the product package.

* ``SimpleConvNetRef`` — restatement of the reference topology
  (/root/reference/models/baseline_model.py:5-83) with the same parameter
  names, so a reference ``state_dict`` loads unchanged.
* ``make_state_dict`` — version-stable synthetic weights (numpy PCG64) with the
  reference's Kaiming fan_out init statistics (baseline_model.py:45-56).
* ``build_static_ptq_cpu`` — the reference's "static PTQ" model exactly as
  /root/reference/models/static_ptq_model.py:19-34 builds it
  (``quantize_dynamic({Linear, Conv2d}, qint8)``; convs stay fp32).
* ``build_static_int8_cpu`` — full static int8 (torch.ao eager, fbgemm engine):
  the reference's per-layer stubs (custom_quantization_model.py:34-58) activated
  over the whole net, BN folded as at custom_quantization_model.py:180-190,
  Conv+ReLU and fc1+ReLU fused, per-tensor MinMax observers.
* ``build_qdq_cpu`` — the reference's ``CustomQuantizedSimpleConvNet``
  (custom_quantization_model.py:202-261) with its stubs activated: every conv
  (and fc1) is quantize -> int8 op -> dequantize; ReLU/maxpool in fp32; fc2 fp32.
"""
from __future__ import annotations

import copy

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.ao.quantization as tq

CIFAR_MEAN = (0.4914, 0.4822, 0.4465)  # /root/reference/utils/dataset_manager.py:41-44
CIFAR_STD = (0.2023, 0.1994, 0.2010)

CONV_SPECS = [(3, 64), (64, 64), (64, 128), (128, 128), (128, 256), (256, 256)]


class SimpleConvNetRef(nn.Module):
    """Topology of baseline_model.py:13-40 / forward :58-83 (dropout = identity in eval)."""

    def __init__(self):
        super().__init__()
        for i, (ci, co) in enumerate(CONV_SPECS, 1):
            setattr(self, f"conv{i}", nn.Conv2d(ci, co, 3, padding=1))
            setattr(self, f"bn{i}", nn.BatchNorm2d(co))
        self.fc1 = nn.Linear(4096, 512)
        self.bn7 = nn.BatchNorm1d(512)
        self.fc2 = nn.Linear(512, 10)

    def forward(self, x):
        for i in range(1, 7):
            x = F.relu(getattr(self, f"bn{i}")(getattr(self, f"conv{i}")(x)))
            if i % 2 == 0:
                x = F.max_pool2d(x, 2, 2)
        x = x.reshape(-1, 4096)
        x = F.relu(self.bn7(self.fc1(x)))
        return self.fc2(x)


def synthetic_images(n, seed, mean=CIFAR_MEAN, std=CIFAR_STD, hw=32):
    """x = (U[0,1) - mean_c) / std_c, fp32 NCHW, numpy PCG64."""
    rng = np.random.Generator(np.random.PCG64(seed))
    u = rng.random((n, 3, hw, hw), dtype=np.float32)
    m = np.asarray(mean, np.float32).reshape(1, 3, 1, 1)
    s = np.asarray(std, np.float32).reshape(1, 3, 1, 1)
    return ((u - m) / s).astype(np.float32)


def make_state_dict(seed=0):
    """Kaiming-normal(fan_out, relu) weights, zero biases, BN gamma=1/beta=0,
    drawn from numpy PCG64 (bit-stable across numpy versions and machines)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = {}
    for i, (ci, co) in enumerate(CONV_SPECS, 1):
        std = np.sqrt(2.0 / (co * 9))
        sd[f"conv{i}.weight"] = (rng.standard_normal((co, ci, 3, 3)) * std).astype(np.float32)
        sd[f"conv{i}.bias"] = np.zeros(co, np.float32)
        sd[f"bn{i}.weight"] = np.ones(co, np.float32)
        sd[f"bn{i}.bias"] = np.zeros(co, np.float32)
        sd[f"bn{i}.running_mean"] = np.zeros(co, np.float32)
        sd[f"bn{i}.running_var"] = np.ones(co, np.float32)
    for name, (fi, fo) in (("fc1", (4096, 512)), ("fc2", (512, 10))):
        std = np.sqrt(2.0 / fo)
        sd[f"{name}.weight"] = (rng.standard_normal((fo, fi)) * std).astype(np.float32)
        sd[f"{name}.bias"] = np.zeros(fo, np.float32)
    sd["bn7.weight"] = np.ones(512, np.float32)
    sd["bn7.bias"] = np.zeros(512, np.float32)
    sd["bn7.running_mean"] = np.zeros(512, np.float32)
    sd["bn7.running_var"] = np.ones(512, np.float32)
    out = {k: torch.from_numpy(v) for k, v in sd.items()}
    for i in range(1, 8):
        out[f"bn{i}.num_batches_tracked"] = torch.tensor(0, dtype=torch.long)
    return out


def recalibrate_bn(model, x):
    """Fact 8 of SURVEY §0: random-init BN stats make argmax degenerate; set the
    running stats to the statistics of a synthetic calibration batch
    (train-mode forward, cumulative average, no parameter update)."""
    model.train()
    for m in model.modules():
        if isinstance(m, (nn.BatchNorm1d, nn.BatchNorm2d)):
            m.reset_running_stats()
            m.momentum = None
    with torch.no_grad():
        model(x)
    for m in model.modules():
        if isinstance(m, (nn.BatchNorm1d, nn.BatchNorm2d)):
            m.momentum = 0.1
    model.eval()
    return model


def reference_fp32_model(seed=0, calib=None):
    m = SimpleConvNetRef()
    m.load_state_dict(make_state_dict(seed))
    if calib is not None:
        recalibrate_bn(m, torch.from_numpy(calib))
    return m.eval()


# --------------------------------------------------------------------------
class _FusedInt8Net(nn.Module):
    """Eager-mode wrapper: QuantStub -> [conv_i+bn_i+relu] ... -> DeQuantStub."""

    def __init__(self, fp32):
        super().__init__()
        fp32 = copy.deepcopy(fp32).eval()
        self.quant = tq.QuantStub()
        for i in range(1, 7):
            setattr(self, f"conv{i}", getattr(fp32, f"conv{i}"))
            setattr(self, f"bn{i}", getattr(fp32, f"bn{i}"))
            setattr(self, f"relu{i}", nn.ReLU())
        self.pool = nn.MaxPool2d(2, 2)
        # Linear+BN1d+ReLU has no eager fuser: fold bn7 into fc1 first (the same
        # fusion.py:156-186 arithmetic fuse_modules uses), then fuse fc1+ReLU.
        from torch.nn.utils.fusion import fuse_linear_bn_eval
        self.fc1, self.relu7 = fuse_linear_bn_eval(fp32.fc1, fp32.bn7), nn.ReLU()
        self.fc2 = fp32.fc2
        self.dequant = tq.DeQuantStub()

    def forward(self, x):
        x = self.quant(x)
        for i in range(1, 7):
            x = getattr(self, f"relu{i}")(getattr(self, f"bn{i}")(getattr(self, f"conv{i}")(x)))
            if i % 2 == 0:
                x = self.pool(x)
        # FBGEMM conv outputs are channels_last; flatten in NCHW order
        # (baseline_model.py:78 semantics) needs a contiguous copy first.
        x = x.contiguous().reshape(-1, 4096)
        x = self.relu7(self.fc1(x))
        x = self.fc2(x)
        return self.dequant(x)


def static_qconfig(per_channel=False, reduce_range=False):
    act = tq.MinMaxObserver.with_args(dtype=torch.quint8, qscheme=torch.per_tensor_affine,
                                      reduce_range=reduce_range)
    if per_channel:
        wt = tq.PerChannelMinMaxObserver.with_args(dtype=torch.qint8,
                                                   qscheme=torch.per_channel_symmetric)
    else:
        wt = tq.MinMaxObserver.with_args(dtype=torch.qint8, qscheme=torch.per_tensor_symmetric)
    return tq.QConfig(activation=act, weight=wt)


def build_static_int8_cpu(fp32, calib_batches, per_channel=False):
    torch.backends.quantized.engine = "fbgemm"
    net = _FusedInt8Net(fp32).eval()
    fuse = [[f"conv{i}", f"bn{i}", f"relu{i}"] for i in range(1, 7)] + [["fc1", "relu7"]]
    net = tq.fuse_modules(net, fuse, inplace=False)
    net.qconfig = static_qconfig(per_channel)
    tq.prepare(net, inplace=True)
    with torch.no_grad():
        for xb in calib_batches:
            net(xb)
    tq.convert(net, inplace=True)
    return net.eval()


def build_static_ptq_cpu(fp32):
    """static_ptq_model.py:19-34 verbatim semantics (engine left at its default)."""
    m = copy.deepcopy(fp32).eval()
    return torch.ao.quantization.quantize_dynamic(m, {nn.Linear, nn.Conv2d}, dtype=torch.qint8)


def build_dynamic_ptq_cpu(fp32):
    """dynamic_ptq_model.py:281-308: fold conv+bn, fc1+bn7 then quantize_dynamic."""
    torch.backends.quantized.engine = "fbgemm"
    m = copy.deepcopy(fp32).eval()
    fuse = [[f"conv{i}", f"bn{i}"] for i in range(1, 7)] + [["fc1", "bn7"]]
    m = tq.fuse_modules(m, fuse, inplace=False)
    return torch.ao.quantization.quantize_dynamic(m, {nn.Linear, nn.Conv2d}, dtype=torch.qint8)


# --------------------------------------------------------------------------
class _QDQConv(nn.Module):
    def __init__(self, op):
        super().__init__()
        self.quant, self.op, self.dequant = tq.QuantStub(), op, tq.DeQuantStub()

    def forward(self, x):
        return self.dequant(self.op(self.quant(x)))


class _QDQNet(nn.Module):
    """custom_quantization_model.py:202-261 with the per-layer stubs live
    (the outer stub at :234 disabled — fact 6 of SURVEY §0)."""

    def __init__(self, folded):
        super().__init__()
        for i in range(1, 7):
            setattr(self, f"conv{i}", _QDQConv(getattr(folded, f"conv{i}")))
        self.fc1 = _QDQConv(folded.fc1)
        self.fc2 = folded.fc2

    def forward(self, x):
        for i in range(1, 7):
            x = F.relu(getattr(self, f"conv{i}")(x))
            if i % 2 == 0:
                x = F.max_pool2d(x, 2, 2)
        x = x.contiguous().reshape(-1, 4096)
        x = F.relu(self.fc1(x))
        return self.fc2(x)


def build_qdq_cpu(fp32, calib_batches, per_channel=False):
    torch.backends.quantized.engine = "fbgemm"
    m = copy.deepcopy(fp32).eval()
    fuse = [[f"conv{i}", f"bn{i}"] for i in range(1, 7)] + [["fc1", "bn7"]]
    folded = tq.fuse_modules(m, fuse, inplace=False)
    net = _QDQNet(folded).eval()
    for i in range(1, 7):
        getattr(net, f"conv{i}").qconfig = static_qconfig(per_channel)
    net.fc1.qconfig = static_qconfig(per_channel)
    tq.prepare(net, inplace=True)
    with torch.no_grad():
        for xb in calib_batches:
            net(xb)
    tq.convert(net, inplace=True)
    return net.eval()


# -------------------------------------------------------------------------- ResNet
class BottleneckRef(nn.Module):
    """torchvision Bottleneck (v1.5: stride on the 3x3), the block the
    reference wraps as CustomQuantizedBottleneck
    (/root/reference/models/custom_quantization_model.py:60-102); one ReLU
    module per use so torch.ao eager fusion can pair each conv with its own."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu1 = nn.ReLU()
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.relu2 = nn.ReLU()
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.downsample = downsample
        # static-int8 hand-off of the float-domain residual join (:94-101):
        # dequantize both operands, add in fp32, ReLU, quantize
        self.dq_out, self.dq_id, self.q_out = tq.DeQuantStub(), tq.DeQuantStub(), tq.QuantStub()

    def forward(self, x):
        out = self.relu1(self.bn1(self.conv1(x)))
        out = self.relu2(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        idn = self.downsample(x) if self.downsample is not None else x
        return self.q_out(F.relu(self.dq_out(out) + self.dq_id(idn)))


class ResNetRef(nn.Module):
    """torchvision ResNet layout (same state-dict keys as models.resnet /
    torchvision.models.resnet50), quantization stubs at the net's ends."""

    def __init__(self, layers=(1, 1, 1, 1), num_classes=10, base=64):
        super().__init__()
        self.quant, self.dequant = tq.QuantStub(), tq.DeQuantStub()
        self.inplanes = base
        self.conv1 = nn.Conv2d(3, base, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(base)
        self.relu = nn.ReLU()
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        for i, n in enumerate(layers, start=1):
            planes, stride = base * 2 ** (i - 1), 1 if i == 1 else 2
            ds = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False),
                               nn.BatchNorm2d(planes * 4))
            blocks = [BottleneckRef(self.inplanes, planes, stride, ds)]
            self.inplanes = planes * 4
            blocks += [BottleneckRef(self.inplanes, planes) for _ in range(1, n)]
            setattr(self, f"layer{i}", nn.Sequential(*blocks))
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(base * 8 * 4, num_classes)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(self.quant(x)))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.dequant(self.fc(torch.flatten(self.avgpool(x), 1)))


def resnet_state_dict(model, seed=0):
    """Version-stable synthetic weights for a ResNetRef / models.resnet net:
    Kaiming-normal(fan_out) convs, uniform(0.5, 1.5) BN gamma, 0.1 N(0,1) BN
    beta (as models.resnet.synthetic_resnet spreads them), N(0, 0.01) fc,
    zero fc bias, from numpy PCG64 in state-dict order."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = {}
    for k, v in model.state_dict().items():
        shape = tuple(v.shape)
        if k.endswith("num_batches_tracked"):
            sd[k] = torch.tensor(0, dtype=torch.long)
            continue
        if k.endswith("running_mean"):
            a = np.zeros(shape, np.float32)
        elif k.endswith("running_var"):
            a = np.ones(shape, np.float32)
        elif k.startswith("fc."):
            a = (rng.standard_normal(shape) * 0.01).astype(np.float32) if k.endswith("weight") \
                else np.zeros(shape, np.float32)
        elif v.dim() == 4:   # conv
            a = (rng.standard_normal(shape) * np.sqrt(2.0 / (shape[0] * shape[2] * shape[3]))).astype(np.float32)
        elif k.endswith("weight"):   # BN gamma
            a = (0.5 + rng.random(shape)).astype(np.float32)
        else:   # BN beta
            a = (0.1 * rng.standard_normal(shape)).astype(np.float32)
        sd[k] = torch.from_numpy(a)
    return sd


def resnet_fuse_list(model):
    fuse = [["conv1", "bn1", "relu"]]
    for name, mod in model.named_modules():
        if isinstance(mod, BottleneckRef):
            fuse += [[f"{name}.conv1", f"{name}.bn1", f"{name}.relu1"],
                     [f"{name}.conv2", f"{name}.bn2", f"{name}.relu2"],
                     [f"{name}.conv3", f"{name}.bn3"]]
            if mod.downsample is not None:
                fuse.append([f"{name}.downsample.0", f"{name}.downsample.1"])
    return fuse


def build_resnet_static_int8_cpu(fp32, calib_batches, per_channel=True):
    """torch.ao eager static int8 (fbgemm) of a ResNetRef: Conv-BN(-ReLU)
    fused as /root/reference/models/custom_quantization_model.py:264-298 fuses
    them, MinMax observers (per-channel symmetric s8 weights, per-tensor
    affine u8 activations), float-domain residual join, quantized
    max-pool / adaptive avg-pool / Linear."""
    torch.backends.quantized.engine = "fbgemm"
    net = copy.deepcopy(fp32).eval()
    net = tq.fuse_modules(net, resnet_fuse_list(net), inplace=False)
    net.qconfig = static_qconfig(per_channel)
    tq.prepare(net, inplace=True)
    with torch.no_grad():
        for xb in calib_batches:
            net(xb)
    tq.convert(net, inplace=True)
    return net.eval()


class RefQDQBottleneck(nn.Module):
    """CustomQuantizedBottleneck (/root/reference/models/custom_quantization_model.py
    :60-102) with its stubs live: every conv (and the downsample conv) is
    QuantStub -> int8 conv -> DeQuantStub (:34-45), BN and ReLU stay fp32
    modules, the residual add is a float add (:95-101)."""

    def __init__(self, b):
        super().__init__()
        self.conv1, self.bn1 = _QDQConv(b.conv1), b.bn1
        self.conv2, self.bn2 = _QDQConv(b.conv2), b.bn2
        self.conv3, self.bn3 = _QDQConv(b.conv3), b.bn3
        self.downsample = (None if b.downsample is None else
                           nn.Sequential(_QDQConv(b.downsample[0]), b.downsample[1]))

    def forward(self, x):
        identity = x
        out = F.relu(self.bn1(self.conv1(x)))
        out = F.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return F.relu(out + identity)


class RefQDQResNet(nn.Module):
    """CustomQuantizedResNet50 (:104-143) around a ResNetRef with the per-layer
    stubs live.  The outer QuantStub / DeQuantStub (:107-108, :127, :142) stay
    identities: converted, the outer QuantStub would hand conv1's own
    QuantStub an already-quantized tensor, which torch rejects."""

    def __init__(self, fp):
        super().__init__()
        self.conv1, self.bn1, self.maxpool = _QDQConv(fp.conv1), fp.bn1, fp.maxpool
        for i in range(1, 5):
            setattr(self, f"layer{i}", nn.Sequential(*[RefQDQBottleneck(b) for b in getattr(fp, f"layer{i}")]))
        self.avgpool, self.fc = fp.avgpool, _QDQConv(fp.fc)

    def forward(self, x):
        x = self.maxpool(F.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def build_resnet_qdq_cpu(fp32, calib_batches, per_channel=True):
    """torch.ao eager conversion of RefQDQResNet (fbgemm): each stub's MinMax
    observer sees the fp32 network's activations during calibration, as
    prepare() runs the unquantized forward; per-channel symmetric s8 weights."""
    torch.backends.quantized.engine = "fbgemm"
    net = RefQDQResNet(copy.deepcopy(fp32).eval()).eval()
    for m in net.modules():
        if isinstance(m, _QDQConv):
            m.qconfig = static_qconfig(per_channel)
    tq.prepare(net, inplace=True)
    with torch.no_grad():
        for xb in calib_batches:
            net(xb)
    tq.convert(net, inplace=True)
    return net.eval()


def build_optimized_dynamic_cpu(fp32):
    """/root/reference/models/optimized_custom_quantization.py:26-76 on a
    torchvision-layout ResNet (shared ``relu`` per Bottleneck, e.g.
    models.resnet.ResNet): fuse stem conv1+bn1+relu and, per bottleneck,
    conv2+bn2+relu, conv3+bn3, downsample conv+BN (conv1 left unfused), then
    quantize_dynamic with default_dynamic_qconfig everywhere (:108-127)."""
    torch.backends.quantized.engine = "fbgemm"
    m = copy.deepcopy(fp32).cpu().eval()
    fuse = [["conv1", "bn1", "relu"]]
    for name, mod in m.named_modules():
        if hasattr(mod, "conv3") and hasattr(mod, "bn3"):   # a Bottleneck
            fuse.append([f"{name}.conv2", f"{name}.bn2", f"{name}.relu"])
            fuse.append([f"{name}.conv3", f"{name}.bn3"])
            if mod.downsample is not None:
                fuse.append([f"{name}.downsample.0", f"{name}.downsample.1"])
    fused = tq.fuse_modules(m, fuse, inplace=False)
    return torch.ao.quantization.quantize_dynamic(fused, {"": tq.default_dynamic_qconfig},
                                                  dtype=torch.qint8)
