"""Per-kernel mean of SQ counters from tools/pmc_sq.sh output: python tools/sq_summary.py gpurun_out/sq gpurun_out/sq2"""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        acc = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][:32]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
        for k in acc:
            if "kernel" not in k or "at::" in k:
                continue
            n = len(disp[k])
            print(k, f"({n} dispatches)", "  ".join(f"{c}={v / n:.4g}" for c, v in sorted(acc[k].items())))
