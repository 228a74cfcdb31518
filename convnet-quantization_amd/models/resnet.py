"""fp32 ResNet-50 restated without torchvision.

The reference builds its config-5 model with
``torchvision.models.resnet50(weights=IMAGENET1K_V1)``
(models/dynamic_ptq_model.py:194-195, models/optimized_custom_quantization.py:13)
and wraps the Bottleneck blocks (models/custom_quantization_model.py:60-148).
torchvision is not part of this build, so the topology is written out here with
the same module names, so a torchvision ``resnet50`` state_dict (e.g. a local
IMAGENET1K_V1 ``.pth``) loads unchanged:

  conv1 7x7/2 (3->64) bn1 relu maxpool 3x3/2
  layer1..4: [3, 4, 6, 3] Bottleneck(inplanes, planes, stride), expansion 4,
             stride on conv2 (the 3x3, "ResNet v1.5"), downsample = 1x1/stride
             conv + BN on the first block of each layer
  avgpool (global) fc 2048 -> num_classes

There is no network here, so weights are random (torchvision's init) and the
BatchNorm statistics are re-estimated on synthetic ImageNet-normalised images
(``synthetic_resnet``) so activations have realistic ranges.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        width = planes
        self.conv1 = nn.Conv2d(inplanes, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, planes * self.expansion, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, base=64):
        super().__init__()
        self.inplanes = base
        self.conv1 = nn.Conv2d(3, base, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(base)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(base, layers[0])
        self.layer2 = self._make_layer(base * 2, layers[1], 2)
        self.layer3 = self._make_layer(base * 4, layers[2], 2)
        self.layer4 = self._make_layer(base * 8, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(base * 8 * Bottleneck.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * Bottleneck.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * Bottleneck.expansion, 1, stride=stride, bias=False),
                nn.BatchNorm2d(planes * Bottleneck.expansion))
        mods = [Bottleneck(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * Bottleneck.expansion
        mods += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


def resnet50(num_classes=1000):
    return ResNet((3, 4, 6, 3), num_classes)


def synthetic_images(n, seed, hw=224):
    """ImageNet-normalised synthetic images [n,3,hw,hw] fp32 (smooth random
    fields, so spatial statistics are image-like rather than white noise)."""
    g = np.random.default_rng(seed)
    low = g.standard_normal((n, 3, hw // 16 + 1, hw // 16 + 1)).astype(np.float32)
    up = np.repeat(np.repeat(low, 16, axis=2), 16, axis=3)[:, :, :hw, :hw]
    x = 0.5 + 0.2 * up + 0.05 * g.standard_normal((n, 3, hw, hw)).astype(np.float32)
    x = np.clip(x, 0.0, 1.0)
    mean = np.asarray(IMAGENET_MEAN, np.float32).reshape(1, 3, 1, 1)
    std = np.asarray(IMAGENET_STD, np.float32).reshape(1, 3, 1, 1)
    return ((x - mean) / std).astype(np.float32)


@torch.no_grad()
def synthetic_resnet(seed=0, layers=(3, 4, 6, 3), num_classes=1000, hw=224, calib_images=16,
                     device="cpu"):
    """Random-init ResNet (torchvision init) whose BN running statistics are
    re-estimated on synthetic images (cumulative average, train-mode BN), then
    set to eval.  The BN affine parameters get a small random spread so the
    folded weights differ per channel, as in a trained net."""
    torch.manual_seed(seed)
    m = ResNet(layers, num_classes).to(device)
    g = torch.Generator().manual_seed(seed + 1)
    for mod in m.modules():
        if isinstance(mod, nn.BatchNorm2d):
            c = mod.num_features
            mod.weight.copy_((0.5 + torch.rand(c, generator=g)).to(device))
            mod.bias.copy_((0.1 * torch.randn(c, generator=g)).to(device))
            mod.momentum = None
            mod.reset_running_stats()
    m.train()
    x = torch.from_numpy(synthetic_images(calib_images, seed + 2, hw)).to(device)
    m(x)
    m.eval()
    return m
