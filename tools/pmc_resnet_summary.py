"""Per-conv-launch counters of one ResNet-50 forward (the last forward of
tools/resnet_layers.py in each pass), in launch order."""
import csv
import glob
import os
import sys

O = sys.argv[1]


def rows(tag):
    f = glob.glob(os.path.join(O, tag, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return []
    per = {}
    for r in csv.DictReader(open(f[0])):
        if "conv_gemm_kernel" not in r["Kernel_Name"] and "stem_fused_kernel" not in r["Kernel_Name"]:
            continue
        d = per.setdefault(int(r["Dispatch_Id"]), {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(per)
    return [per[i] for i in ids]


sq, fe, wr = rows("sq"), rows("fetch"), rows("write")
n = 53   # conv launches per forward (the fused stem counts as the first)
sq, fe, wr = sq[-n:], fe[-n:], wr[-n:]
print("idx  valuM  mfmaM  ldsM  waitany  waitinst  mfma_busy  fetchMB  writeMB")
for i in range(min(len(sq), len(fe), len(wr))):
    s, f, w = sq[i], fe[i], wr[i]
    wc = s.get("SQ_WAVE_CYCLES", 1) or 1
    busy = s.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024.0 * w.get("GRBM_GUI_ACTIVE", 1) / 8.0)
    print("%3d %6.1f %6.2f %5.2f  %6.2f  %7.2f  %8.2f  %7.1f  %7.1f" % (
        i, s.get("SQ_INSTS_VALU", 0) / 1e6, s.get("SQ_INSTS_MFMA", 0) / 1e6, s.get("SQ_INSTS_LDS", 0) / 1e6,
        s.get("SQ_WAIT_ANY", 0) / wc, s.get("SQ_WAIT_INST_ANY", 0) / wc, busy,
        2 * f.get("FETCH_SIZE", 0) / 1024, w.get("WRITE_SIZE", 0) / 1024))
