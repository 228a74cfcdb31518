"""Summarise rocprofv3 PMC csv passes written by tools/gpu_perf.sh."""
import collections
import csv
import sys

d = sys.argv[1]
def load(sub):
    try:
        rows = list(csv.DictReader(open(f"{d}/{sub}/run_counter_collection.csv")))
    except FileNotFoundError:
        return {}
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void qcn::", "")[:48]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in dd.items()} for k, dd in agg.items()}
sq, fe, wr = load("pmc_sq"), load("pmc_fetch"), load("pmc_write")
for k in sq:
    s = sq[k]
    wave = s.get("SQ_WAVE_CYCLES", 1)
    print(f"{k:48s} waitany {s.get('SQ_WAIT_ANY',0)/wave:5.2f} waitinst {s.get('SQ_WAIT_INST_ANY',0)/wave:5.2f} "
          f"ldsconf {s.get('SQ_LDS_BANK_CONFLICT',0)/1e6:6.2f}M mfma {s.get('SQ_VALU_MFMA_BUSY_CYCLES',0)/1e6:6.1f}M "
          f"valu {s.get('SQ_INSTS_VALU',0)/1e6:6.2f}M fetchMB {2*fe.get(k,{}).get('FETCH_SIZE',0)/1024:7.1f} "
          f"writeMB {wr.get(k,{}).get('WRITE_SIZE',0)/1024:7.1f}")
