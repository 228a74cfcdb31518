"""Timing of the conv3+conv4 and conv5+conv6 pair launches at batch B
(diagnostic; run it once per library variant via QCN_LIB for A/B): HIP
events around N back-to-back launches of each, alternating, after a warm-up.

    python tools/conv34_ab.py [B] [N] [ROUNDS]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "convnet-quantization_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

from oracle import torch_ref  # noqa: E402  (weights only)
from qconvnet import ops  # noqa: E402
from qconvnet.qmodel import QuantizedConvNet, build_qspec, calibrate, fold_state_dict  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    R = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    dev = torch.device("cuda:0")
    fp = torch_ref.reference_fp32_model(0, torch_ref.synthetic_images(64, 1))
    folded = fold_state_dict(fp.state_dict())
    ranges = calibrate(folded, [torch.from_numpy(torch_ref.synthetic_images(64, 1))], "cpu")
    model = QuantizedConvNet(build_qspec(folded, ranges, "static"), dev)
    x = torch.from_numpy(torch_ref.synthetic_images(B, 0)).to(dev)
    model.run(x)
    a2 = model.buffers(B)["a2"].clone()
    L = model.L
    out_n = torch.empty((B, 8, 8, 128), dtype=torch.uint8, device=dev)
    a4 = model.buffers(B)["a4"].clone()
    out6 = torch.empty((128, B, 32), dtype=torch.uint8, device=dev)
    forms = {"conv34": lambda: ops.conv_pair(a2, L[2], L[3], out_n, kmajor=False),
             "conv56": lambda: ops.conv_pair(a4, L[4], L[5], out6, kmajor=True)}
    for f in forms.values():
        for _ in range(20):
            f()
    torch.cuda.synchronize()
    res = {k: [] for k in forms}
    for _ in range(R):
        for k, f in forms.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(N):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / N * 1e3)
    for k, v in res.items():
        print(f"{k:10s} B={B}: " + " ".join(f"{t:.2f}" for t in v) + f"  us/launch (min {min(v):.2f})",
              flush=True)


if __name__ == "__main__":
    main()
