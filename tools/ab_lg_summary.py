"""Summary of tools/gpu_ab_lg.sh: per variant, the sensor kernel's mean dispatch (rocprofv3 stats) and HBM bytes per car
(2 x FETCH_SIZE + WRITE_SIZE, KiB -> B, over the dispatches' cars: grid threads / 16), and model_logic_kernel's."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]


def kname(n):
    n = n.replace("void ", "")
    return n.split("<")[0].split("(")[0]


for kt in sorted(glob.glob(os.path.join(d, "kt*"))):
    if not os.path.isdir(kt):
        continue
    v = os.path.basename(kt)[2:]
    st = glob.glob(kt + "/**/*kernel_stats.csv", recursive=True)
    dur = {}
    for r in csv.DictReader(open(st[0])) if st else []:
        dur[kname(r["Name"])] = float(r["AverageNs"]) / 1000
    per = defaultdict(float)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(os.path.join(d, f"p{v}_{c}") + "/**/*counter_collection.csv", recursive=True)
        acc = defaultdict(lambda: [0.0, 0.0])
        for r in csv.DictReader(open(f[0])) if f else []:
            k = kname(r["Kernel_Name"])
            if k not in ("ray_sensor_kernel", "model_logic_kernel"):
                continue
            g = float(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
            cars = g / 16 if k == "ray_sensor_kernel" else g * 120 / 128
            acc[k][0] += float(r["Counter_Value"]) * 1024 * (2 if c == "FETCH_SIZE" else 1)
            acc[k][1] += cars
        for k, (b, n) in acc.items():
            per[k] += b / max(n, 1)
    print(f"{v}: sensor {dur.get('ray_sensor_kernel', 0):.2f} us/dispatch, {per['ray_sensor_kernel']:.0f} B/car; "
          f"model_logic {dur.get('model_logic_kernel', 0):.2f} us, {per['model_logic_kernel']:.0f} B/car")
