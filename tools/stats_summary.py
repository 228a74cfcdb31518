"""Print the rocprofv3 --stats kernel summary under DIR: short kernel name,
calls, average and total time (diagnostic; reads *kernel_stats.csv)."""
import csv
import glob
import os
import re
import sys


def short(name):
    n = re.sub(r"\(.*$", "", name)
    n = n.replace("qcn::", "").replace("ConvCfg", "C")
    return n[:110]


def main(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    for f in files:
        print("#", f)
        rows = list(csv.DictReader(open(f)))
        rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
        for r in rows[:25]:
            print(f"{int(r['Calls']):7d} {float(r['AverageNs']) / 1e3:9.2f} us  "
                  f"{float(r['TotalDurationNs']) / 1e6:9.3f} ms  {short(r['Name'])}")


if __name__ == "__main__":
    main(sys.argv[1])
