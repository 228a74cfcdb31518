"""Launch times of the int8 ResNet-50 forward's stem and layer 1 (batch 512),
with the layer-1 reduce convs fused into the joins (fuse_reduce) and as
separate launches: python tools/resnet_l1_times.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "convnet-quantization_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from models.resnet import synthetic_images, synthetic_resnet  # noqa: E402
from qconvnet.resnet import quantize_resnet  # noqa: E402

B = int(os.environ.get("B", 512))
dev = torch.device("cuda")
fp = synthetic_resnet(0, device=dev, calib_images=16)
m = quantize_resnet(fp, [torch.from_numpy(synthetic_images(16, 1))], dev)
x = torch.from_numpy(synthetic_images(B, 2)).to(dev)
for fuse in (True, False, True, False):
    m.fuse_reduce = fuse
    for _ in range(3):
        m.run(x)
    torch.cuda.synchronize()
    acc = None
    for _ in range(5):
        marks = []
        m.run(x, marks=marks)
        torch.cuda.synchronize()
        t = np.array([e0.elapsed_time(e1) for (_, e0), (_, e1) in zip(marks[:-1], marks[1:])])
        acc = t if acc is None else acc + t
    acc /= 5
    print(f"fuse_reduce={fuse}: {len(acc)} launches, total {acc.sum():.3f} ms; first 14 (ms): "
          + " ".join(f"{v:.3f}" for v in acc[:14]), flush=True)
