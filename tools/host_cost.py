"""Host-side cost of one forward's launch sequence: time model.run() at a
batch so small that the GPU finishes first (the loop then runs at the host's
launch rate), and time the HIP-graph replay of the same forward."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "convnet-quantization_amd"), ROOT]
import torch  # noqa: E402

from oracle import torch_ref  # noqa: E402  (weights only)
from qconvnet.qmodel import QuantizedConvNet, build_qspec, calibrate, fold_state_dict  # noqa: E402

dev = torch.device("cuda:0")
fp = torch_ref.reference_fp32_model(0, torch_ref.synthetic_images(64, 1))
folded = fold_state_dict(fp.state_dict())
ranges = calibrate(folded, [torch.from_numpy(torch_ref.synthetic_images(64, 1))], "cpu")
for mode, B in (("static", 128), ("static", 256), ("qdq", 256), ("static", 1024)):
    model = QuantizedConvNet(build_qspec(folded, ranges, mode), dev)
    model.fuse_convs = "--three" not in sys.argv   # --three: conv12 / conv3+4 / conv5+6 launches
    x = torch.from_numpy(torch_ref.synthetic_images(B, 0)).to(dev)
    for _ in range(20):
        model.run(x)
    torch.cuda.synchronize()
    n = 500
    t0 = time.perf_counter()
    for _ in range(n):
        model.run(x)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    model.capture_graph(x.clone())
    for _ in range(20):
        model.replay(B)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        model.replay(B)
    torch.cuda.synchronize()
    t_g = time.perf_counter() - t0
    print(f"{mode} batch {B}: eager {t_all / n * 1e6:.1f} us/step (host issue {t_host / n * 1e6:.1f} us/step), "
          f"graph replay {t_g / n * 1e6:.1f} us/step", flush=True)
