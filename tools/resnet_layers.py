"""Per-conv timing of the int8 ResNet-50 forward (batch 512): for each conv
launch print shape, ms, int8 TOPS, algorithmic GB/s and the roofline floor
max(ops/peak, bytes/HBM) — which convs are far from their bound."""
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
m.fuse_reduce = False   # one "conv" mark per conv layer: the rows below match marks to layers by position
x = torch.from_numpy(synthetic_images(B, 2)).to(dev)
for _ in range(3):
    m.run(x)
torch.cuda.synchronize()
reps = 5
acc = None
for _ in range(reps):
    marks = []
    m.run(x, marks=marks)
    torch.cuda.synchronize()
    t = [e0.elapsed_time(e1) for (_, e0), (_, e1) in zip(marks[:-1], marks[1:])]
    names = [n for n, _ in marks[1:]]
    acc = np.array(t) if acc is None else acc + np.array(t)
acc /= reps
convs = m.conv_layers()
hh = (224 + 2 * convs[0].py - convs[0].kh) // convs[0].sy + 1
geo = [(224, 112, 32)]   # (in hw, out hw, cin)
hin = 56
cin = 64
for b in m.blocks:
    ho = (hin + 2 * b["c2"].py - b["c2"].kh) // b["c2"].sy + 1
    if b["ds"] is not None:
        geo.append((hin, ho, cin))
    geo += [(hin, hin, cin), (hin, ho, b["c1"].cout), (ho, ho, b["c2"].cout)]
    hin, cin = ho, b["c3"].cout
ci = 0
tot = {"ms": 0.0, "floor": 0.0}
print(f"{'launch':>9} {'k':>5} {'s':>2} {'hw':>4} {'cin':>5} {'cout':>5} {'ms':>7} {'TOPS':>7} {'GB/s':>7} {'floor':>7} {'eff':>5}")
for n, ms in zip(names, acc):
    if n != "conv":
        print(f"{n:>9} {'':>5} {'':>2} {'':>4} {'':>5} {'':>5} {ms:7.3f}")
        continue
    d = convs[ci]
    hi, ho, c = geo[ci]
    ci += 1
    mac = B * ho * ho * d.cout * d.w.shape[0] * 32
    byts = B * (hi * (hi if d.kw > 1 or d.kh == 1 else hi // 2) * c + ho * ho * d.cout)
    if d.kh == 7:
        byts = B * (224 * 112 * 32 + ho * ho * d.cout)
    floor = max(2 * mac / 5033e12, byts / 8e12) * 1e3
    tot["ms"] += ms
    tot["floor"] += floor
    print(f"{'conv':>9} {d.kh}x{d.kw:<3} {d.sy:>2} {ho:>4} {c:>5} {d.cout:>5} {ms:7.3f} "
          f"{2 * mac / ms / 1e9:7.0f} {byts / ms / 1e6:7.0f} {floor:7.3f} {floor / ms:5.2f}")
print(f"conv total {tot['ms']:.3f} ms, roofline floor {tot['floor']:.3f} ms "
      f"({tot['floor'] / tot['ms']:.2f}); all launches {acc.sum():.3f} ms")
