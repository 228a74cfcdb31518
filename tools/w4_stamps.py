"""Per-step cycles of the one-wave-per-SIMD conv3 .. conv6 launch (diagnostic):
loads the stamped library (tools/build_w4_stamp.sh ->
libqconvnet_w4stamp.so), runs conv12 + conv3_6 back to back for >= 2 s, then
reads the last launch's s_memtime stamps of wave 0 of every workgroup and
prints the median over workgroups of each step of each tile:

    stage   tile input (halos + interior) into patch A, barrier
    loopA   conv A's K-steps (the last one with A's requant fused behind it)
    putA    barrier, patch B halos, the held blocks, barrier
    loopB   conv B's K-steps (the last one with B's pooled requant fused)
    putB    the 16-B stores of B's output, barrier

plus the phase's in-kernel clock (s_memtime / s_memrealtime x 100 MHz) and
its MFMA cycles per SIMD.

    python tools/w4_stamps.py [B]
"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("QCN_LIB", os.path.join(ROOT, "convnet-quantization_amd", "qconvnet",
                                              "libqconvnet_w4stamp.so"))
for _p in (os.path.join(ROOT, "convnet-quantization_amd"), ROOT, os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import netfix  # noqa: E402
from oracle import torch_ref  # noqa: E402  (input images only)
from qconvnet import _lib  # noqa: E402
from qconvnet.qmodel import QuantizedConvNet  # noqa: E402

MAC = {"conv3": 18_874_368, "conv4": 37_748_736, "conv5": 18_874_368, "conv6": 37_748_736}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    lib = _lib.load()
    fn = lib.qcn_w4_stamps
    fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_void_p, C.c_int]
    dev = torch.device("cuda:0")
    spec, _ = netfix.static_spec(netfix.load(False))
    model = QuantizedConvNet(spec, dev)
    model.convs_w4 = True
    x = torch.from_numpy(torch_ref.synthetic_images(B, 0)).to(dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    G = min(B, ncu)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.5:
        for _ in range(50):
            model.run(x)
        torch.cuda.synchronize()
    model.run(x)
    torch.cuda.synchronize()
    mt = np.zeros((G, 2, 32), np.uint64)
    rt = np.zeros((G, 2, 2), np.uint64)
    _lib.check(fn(mt.ctypes.data, rt.ctypes.data, G), "w4_stamps")
    mt = mt.astype(np.int64)
    rt = rt.astype(np.int64)
    per_wg = B / G
    out = {"batch": B, "workgroups": G}
    for ph, (a, b_) in enumerate((("conv3", "conv4"), ("conv5", "conv6"))):
        segs = 2 if ph == 0 else 4
        T = int(np.ceil(per_wg / segs))
        cyc = mt[:, ph, 5 * T] - mt[:, ph, 0]
        ns = (rt[:, ph, 1] - rt[:, ph, 0]) * 10.0
        clock = np.median(cyc / ns)   # GHz
        steps = {}
        prev = mt[:, ph, 0]
        for k in range(T):
            for j, name in enumerate(("stage", "loopA", "putA", "loopB", "putB")):
                cur = mt[:, ph, 1 + 5 * k + j]
                steps[f"t{k}.{name}"] = float(np.median(cur - prev))
                prev = cur
        mfma_a = MAC[a] * per_wg / (4 * 1024)
        mfma_b = MAC[b_] * per_wg / (4 * 1024)
        a_cyc = sum(v for kk, v in steps.items() if kk.split(".")[1] in ("stage", "loopA", "putA"))
        b_cyc = sum(v for kk, v in steps.items() if kk.split(".")[1] in ("loopB", "putB"))
        out[f"{a}+{b_}"] = {
            "cycles_median": float(np.median(cyc)), "us_median": float(np.median(ns) / 1e3), "clock_ghz": float(clock),
            "steps": steps,
            a: {"cycles": a_cyc, "mfma_cycles_per_simd": mfma_a, "issue": mfma_a / a_cyc,
                "frac_at_2p4": mfma_a / a_cyc * clock / 2.4},
            b_: {"cycles": b_cyc, "mfma_cycles_per_simd": mfma_b, "issue": mfma_b / b_cyc,
                 "frac_at_2p4": mfma_b / b_cyc * clock / 2.4}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
