"""Phase stamps of the pipelined conv3+conv4 kernel (diagnostic variant built
with -DQCN_PIPE34_STAMP, loaded via QCN_LIB): ~1 s of back-to-back launches,
then the last launch's per-workgroup s_memtime stamps around every pipeline
barrier; prints the median cycles of every interval over the workgroups and
the in-kernel clock (MI355X_MICROARCH 'DVFS give-back' item 6).

    QCN_LIB=.../libqconvnet_stamp.so python tools/p34_stamps.py [B] [KIND]

KIND 0 / 1: the conv3+conv4 / conv5+conv6 pair launch; 2: the model's default
forward (the one-launch conv1..conv6 under tools/clock's library), printing the
stamps of both pair phases inside it.
"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "convnet-quantization_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import torch_ref  # noqa: E402  (weights only)
from qconvnet import _lib, ops  # noqa: E402
from qconvnet.qmodel import QuantizedConvNet, build_qspec, calibrate, fold_state_dict  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    kind = int(sys.argv[2]) if len(sys.argv) > 2 else 0   # 0: conv3+conv4, 1: conv5+conv6
    dev = torch.device("cuda:0")
    fp = torch_ref.reference_fp32_model(0, torch_ref.synthetic_images(64, 1))
    folded = fold_state_dict(fp.state_dict())
    ranges = calibrate(folded, [torch.from_numpy(torch_ref.synthetic_images(64, 1))], "cpu")
    model = QuantizedConvNet(build_qspec(folded, ranges, "static"), dev)
    x = torch.from_numpy(torch_ref.synthetic_images(B, 0)).to(dev)
    model.run(x)
    a2 = model.buffers(B)["a2"].clone()
    L = model.L
    out = torch.empty((B, 8, 8, 128), dtype=torch.uint8, device=dev)
    a4 = model.buffers(B)["a4"].clone()
    out6 = torch.empty((128, B, 32), dtype=torch.uint8, device=dev)
    t0 = time.time()
    n = 0
    while time.time() - t0 < 1.5:
        for _ in range(100):
            if kind == 0:
                ops.conv_pair(a2, L[2], L[3], out)
            elif kind == 1:
                ops.conv_pair(a4, L[4], L[5], out6, kmajor=True)
            else:
                model.run(x)
        torch.cuda.synchronize()
        n += 100
    lib = _lib.load()
    nwg = min(B, 256)
    for k in ((kind,) if kind < 2 else (0, 1)):
        if kind == 2:
            print(f"## phase {'conv3+4' if k == 0 else 'conv5+6'} of the one-launch convs "
                  f"({model.kernel_names(x.shape)})")
        report(lib, k, nwg, n)


def report(lib, kind, nwg, n):
    buf = np.zeros((1024, 64), np.uint64)
    rc = lib.qcn_diag_p34_stamps(C.c_int(kind), buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), C.c_int(1024))
    assert rc == 0, rc
    s = buf[:nwg].astype(np.int64)
    cnt = int((s[0] != 0).sum())
    # [0] realtime start, [1..cnt-2] memtime stamps, [cnt-1] realtime end
    mt = s[:, 1:cnt - 1]
    rt = s[:, cnt - 1] - s[:, 0]
    clk = (mt[:, -1] - mt[:, 0]) / rt / 10.0   # GHz (realtime ticks at 100 MHz)
    print(f"launches {n}; workgroups {nwg}; stamps per wg {cnt}; clock median {np.median(clk):.3f} GHz "
          f"(min {clk.min():.3f} max {clk.max():.3f})")
    d = np.diff(mt, axis=1)
    tot = mt[:, -1] - mt[:, 0]
    print(f"total cycles per wg: median {np.median(tot):.0f} min {tot.min():.0f} max {tot.max():.0f}")
    for i in range(d.shape[1]):
        print(f"  interval {i:2d}: median {np.median(d[:, i]):8.0f}  p10 {np.percentile(d[:, i], 10):8.0f}  "
              f"p90 {np.percentile(d[:, i], 90):8.0f}")
    # start skew (first stamp relative to the earliest, in realtime ticks -> us)
    st = (s[:, 0] - s[:, 0].min()) / 100.0
    en = (s[:, cnt - 1] - s[:, 0].min()) / 100.0
    print(f"start skew: p50 {np.median(st):.2f} us max {st.max():.2f} us; end: min {en.min():.2f} "
          f"p50 {np.median(en):.2f} max {en.max():.2f} us")


if __name__ == "__main__":
    main()
