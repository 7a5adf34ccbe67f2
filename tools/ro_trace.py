"""Timeline of one sharded rollout call from a rocprofv3 kernel trace (diagnostic tooling).

    python tools/ro_trace.py <trace dir> [--skip 60] [--count 240]

Takes the shard dispatches (model / logic / ray_sensor kernels on a partial grid) in dispatch order, skips the
warm-up call's, and for the next call prints per stream: first start, last end (us from the call's first start),
steps completed, and the GPU's concurrency profile: how much of the call's span had 0 / 1 / 2 / 3 / 4 shards busy.
"""
import argparse
import collections
import csv
import glob

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--skip", type=int, default=60, help="shard dispatches to skip (the warm-up call)")
ap.add_argument("--count", type=int, default=240)
a = ap.parse_args()
f = glob.glob(a.dir + "/**/*kernel_trace.csv", recursive=True)[0]
rows = []
for r in csv.DictReader(open(f)):
    name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
    if name in ("model_kernel", "logic_kernel", "model_logic_kernel", "ray_sensor_kernel"):
        rows.append((int(r["Dispatch_Id"]), name, int(r["Stream_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     int(r["Grid_Size_X"])))
rows.sort()
full = {k: max(r[5] for r in rows if r[1] == k) for k in set(r[1] for r in rows)}
shard = [r for r in rows if r[5] < full[r[1]]]
call = shard[a.skip:a.skip + a.count]
t0 = min(r[3] for r in call)
t1 = max(r[4] for r in call)
print(f"call span {(t1 - t0) / 1000:.1f} us, dispatches {len(call)}")
by = collections.defaultdict(list)
for r in call:
    by[r[2]].append(r)
for s, rs in sorted(by.items()):
    busy = sum(r[4] - r[3] for r in rs)
    print(f"  stream {s}: first start {(min(r[3] for r in rs) - t0) / 1000:7.1f}  last end {(max(r[4] for r in rs) - t0) / 1000:7.1f}"
          f"  kernels {len(rs)}  busy {busy / 1000:.1f} us")
# concurrency profile: number of streams with a kernel running
ev = []
for s, rs in by.items():
    for r in rs:
        ev.append((r[3], 1, s)); ev.append((r[4], -1, s))
ev.sort()
active = collections.Counter()
prof = collections.Counter()
last = t0
for t, d, s in ev:
    n = sum(1 for v in active.values() if v > 0)
    prof[n] += t - last
    last = t
    active[s] += d
print("  streams busy: " + ", ".join(f"{k}: {v / 1000:.1f} us" for k, v in sorted(prof.items())))
# per stream: kernel durations and the idle gap before each kernel (previous end on the same stream -> start)
for s, rs in sorted(by.items()):
    rs = sorted(rs, key=lambda r: r[3])
    gaps = [(b[3] - a[4]) / 1000 for a, b in zip(rs, rs[1:])]
    dur = collections.defaultdict(list)
    for r in rs:
        dur[r[1]].append((r[4] - r[3]) / 1000)
    g = sorted(gaps)
    print(f"  stream {s}: " + ", ".join(f"{k} mean {sum(v) / len(v):.1f} max {max(v):.1f} us" for k, v in sorted(dur.items()))
          + (f"; gaps mean {sum(g) / len(g):.1f} p50 {g[len(g) // 2]:.1f} max {g[-1]:.1f} us" if g else ""))
# per-step end times per stream (sensor kernel ends)
for s, rs in sorted(by.items()):
    ends = [(r[4] - t0) / 1000 for r in rs if r[1] == "ray_sensor_kernel"]
    print(f"  stream {s} step ends: " + " ".join(f"{e:.0f}" for e in ends))
