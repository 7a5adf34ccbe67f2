"""Summarise a tools/profile_session.sh run.

    python tools/pmc_summary.py <out_dir> <tag>

Reads the rocprofv3 CSVs under <out_dir>/{kt,fetch,write}, and writes
  profiles/<tag>_kernel_stats.csv  (rocprofv3 --stats summary, copied verbatim)
  profiles/<tag>_pmc_step.json     (per-dispatch FETCH_SIZE / WRITE_SIZE of the two kernels of a step)
  profiles/pmc_traffic.json        (read by bench.py for roofline.traffic)
One env step = model_logic_kernel (the default; model_kernel + logic_kernel with the fused kernel off) +
ray_sensor_kernel over every workgroup: one launch each (per-step path) or one launch each per env shard (sharded rollout, a grid of 1/S of the workgroups).  A run holds both, so
every dispatch's counter is scaled to the full grid (value / its grid size x the full grid size) before averaging.
HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE/WRITE_SIZE are in KiB and gfx950 FETCH_SIZE tallies
half the bytes of a wide coalesced read (MI355X_MICROARCH.md "HBM").
The sharded step time is read from the kernel trace: the span of each unbroken run of shard dispatches divided by
the env steps it holds (its model_kernel workgroups / the full grid's), to check the bench's HIP-event time.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("model_logic_kernel", "model_kernel", "logic_kernel", "ray_sensor_kernel")


def _find(d, suffix):
    hits = sorted(glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True))
    return hits[-1] if hits else None


def _bench_line(log):
    for line in open(log):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return None


def _base(name):
    """'void ray_sensor_kernel<4>(Params, ...)' -> 'ray_sensor_kernel'"""
    return name.split("(")[0].replace("void ", "").split("<")[0].strip()


def _per_dispatch(path, counter, kernel):
    """per-dispatch counter totals scaled to the kernel's full grid"""
    vals, grid = defaultdict(float), {}
    for row in csv.DictReader(open(path)):
        if _base(row.get("Kernel_Name", "")) != kernel or row.get("Counter_Name") != counter:
            continue
        vals[row["Dispatch_Id"]] += float(row["Counter_Value"])
        grid[row["Dispatch_Id"]] = int(row["Grid_Size"])
    if not vals:
        return []
    full = max(grid.values())
    return [v / grid[d] * full for d, v in vals.items()]


def _trace_steps(path):
    """full-grid average duration per kernel, and the sharded rollout's per-step time (ns) from a kernel trace"""
    rows = []
    for row in csv.DictReader(open(path)):
        kn = _base(row.get("Kernel_Name", ""))
        if kn in KERNELS:
            g = int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"])
            rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), kn, g))
    if not rows:
        return {}
    rows.sort()
    full = {kn: max(g for _, _, k, g in rows if k == kn) for kn in KERNELS if any(k == kn for _, _, k, _ in rows)}
    res = {}
    for kn in full:
        d = [e - s for s, e, k, g in rows if k == kn and g == full[kn]]
        if d:
            res[f"{kn}_full_grid_avg_ns"] = sum(d) / len(d)
            res[f"{kn}_full_grid_calls"] = len(d)
    spans, steps, run = 0.0, 0.0, []

    mk = "model_logic_kernel" if "model_logic_kernel" in full else "model_kernel"   # one per env step

    def close(run):
        nonlocal spans, steps
        if run:
            mg = sum(g for _, _, k, g in run if k == mk)
            if mg:
                spans += max(e for _, e, _, _ in run) - min(s for s, _, _, _ in run)
                steps += mg / full[mk]
    for r in rows:
        if r[3] < full[r[2]]:
            run.append(r)
        else:
            close(run)
            run = []
    close(run)
    if steps:
        res["sharded_step_ns"] = spans / steps
        res["sharded_steps_traced"] = steps
    return res


def main():
    out, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    res = {"tag": tag}
    stats = _find(os.path.join(out, "kt"), "kernel_stats.csv")
    if stats:
        shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
        for row in csv.DictReader(open(stats)):
            for kn in KERNELS:
                if _base(row["Name"]) == kn:
                    res[f"{kn}_rocprof_avg_ns"] = float(row["AverageNs"])
                    res[f"{kn}_rocprof_calls"] = int(row["Calls"])
        res["step_rocprof_avg_ns"] = sum(res.get(f"{kn}_rocprof_avg_ns", 0.0) for kn in KERNELS)
    kt = _find(os.path.join(out, "kt"), "kernel_trace.csv")
    if kt:
        res.update(_trace_steps(kt))
    b = _bench_line(os.path.join(out, "kt.log"))
    if b:
        res["bench_under_rocprof"] = b
        cfg = b["config"]
        res.update(envs=cfg["envs_per_gpu"], cars=cfg["cars_per_env"], track=cfg["track"],
                   policy=cfg.get("policy", "uniform"), workload=cfg["workload"])
    sha = os.path.join(os.path.dirname(os.path.abspath(out)), "prof_source_sha.txt")
    if os.path.exists(sha):
        res["source_sha"] = open(sha).read().strip()
        res["bench_model_kernel_ms_events"] = b["roofline"]["kernel_ms"]
    f = _find(os.path.join(out, "fetch"), "counter_collection.csv")
    w = _find(os.path.join(out, "write"), "counter_collection.csv")
    if f and w:
        tot_f = tot_w = 0.0
        seen = []
        for kn in KERNELS:
            fv, wv = _per_dispatch(f, "FETCH_SIZE", kn), _per_dispatch(w, "WRITE_SIZE", kn)
            if not (fv and wv):
                continue
            seen.append(kn)
            fk, wk = sum(fv) / len(fv), sum(wv) / len(wv)
            res[f"{kn}_fetch_size_kb"], res[f"{kn}_write_size_kb"] = fk, wk
            res[f"{kn}_bytes"] = (2 * fk + wk) * 1024.0
            tot_f += fk
            tot_w += wk
        ok = "ray_sensor_kernel" in seen and ("model_logic_kernel" in seen or {"model_kernel", "logic_kernel"} <= set(seen))
        if ok:
            res["step_kernels"] = seen
            res.update(fetch_size_kb=tot_f, write_size_kb=tot_w, bytes_per_step=(2 * tot_f + tot_w) * 1024.0,
                       bytes_per_step_uncorrected=(tot_f + tot_w) * 1024.0)
            if "envs" in res:
                res["bytes_per_car_step"] = res["bytes_per_step"] / (res["envs"] * res["cars"])
    json.dump(res, open(os.path.join(prof, f"{tag}_pmc_step.json"), "w"), indent=1)
    if "bytes_per_step" in res and "envs" in res and "source_sha" in res:
        json.dump({k: res[k] for k in ("envs", "cars", "track", "policy", "workload", "source_sha", "bytes_per_step", "bytes_per_step_uncorrected",
                                       "bytes_per_car_step", "fetch_size_kb", "write_size_kb", "tag",
                                       "step_kernels", "model_logic_kernel_bytes", "model_kernel_bytes", "logic_kernel_bytes",
                                       "ray_sensor_kernel_bytes") if k in res},
                  open(os.path.join(prof, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
