"""Per-kernel effective clock from a rocprofv3 --kernel-trace --pmc pass
(tools/clock_pass.sh): clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time
(MI355X_MICROARCH.md 'DVFS give-back'); MFMA busy fraction =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 CUs)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
cc = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
dur = {}
for f in kt:
    for r in csv.DictReader(open(f)):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for f in cc:
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void qcn::", "").replace("qcn::", "")[:40]
        did = r["Dispatch_Id"]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        if did not in cnt[name]:
            cnt[name].add(did)
            agg[name]["_t"] += dur.get(did, 0.0)
print(f"{'kernel':40s} {'n':>4s} {'us':>8s} {'GHz':>6s} {'mfma%':>6s} {'valu/wave-cyc':>13s}")
for k, a in agg.items():
    n = len(cnt[k])
    t = a["_t"]
    if t <= 0 or n == 0:
        continue
    cyc = a.get("GRBM_GUI_ACTIVE", 0) / 8
    ghz = cyc / t / 1e9
    mf = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(cyc * 256, 1)
    vw = a.get("SQ_INSTS_VALU", 0) / max(a.get("SQ_WAVE_CYCLES", 1), 1)
    print(f"{k:40s} {n:4d} {t / n * 1e6:8.1f} {ghz:6.2f} {100 * mf:6.1f} {vw:13.4f}")
