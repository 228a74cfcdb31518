"""Per-launch duration and the gap before each launch, from a rocprofv3
kernel-trace csv of tools/kbench.py (steady state: the last 100 forwards) or
of bench.py (argv: csv [first_forward count], e.g. 10 50 = timed region A of
the default bench: 10 warm-up forwards, then 50 timed)."""
import collections
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "qcn::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = {"conv12p": "conv12", "ConvCfg<64, 128": "conv34", "ConvCfg<128, 256": "conv56",
         "fc_splitk": "fc_splitk", "fc_finish": "fc_finish", "fc_head_kernel": "fc_head"}


def short(n):
    for k, v in names.items():
        if k in n:
            return v
    return n[:30]


seq = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
per = len([s for s in seq if s[0] == "conv12"])
if len(sys.argv) > 3:
    first, count = int(sys.argv[2]), int(sys.argv[3])
    c12 = [i for i, s in enumerate(seq) if s[0] == "conv12"]
    start = c12[first]
    seq = seq[:c12[first + count]] if first + count < len(c12) else seq
else:
    start = len(seq) - 100 * 5
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
for i in range(max(start, 1), len(seq)):
    n, s, e = seq[i]
    dur[n].append((e - s) / 1e3)
    gap[n].append((s - seq[i - 1][2]) / 1e3)
tot_d = tot_g = 0.0
for n in ("conv12", "conv34", "conv56", "fc_splitk", "fc_finish", "fc_head"):
    if not dur[n]:
        continue
    d = sum(dur[n]) / len(dur[n])
    g = sum(gap[n]) / len(gap[n])
    tot_d += d
    tot_g += g
    print(f"{n:10s} duration {d:7.2f} us   gap before {g:6.2f} us")
print(f"sum of durations {tot_d:.2f} us, sum of gaps {tot_g:.2f} us, step {tot_d + tot_g:.2f} us")
