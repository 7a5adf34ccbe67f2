"""tools/pmc_summary.py on synthetic rocprofv3 CSVs: counters of quarter-grid shard dispatches scaled to the full
grid, and the sharded rollout's per-step time read from the kernel trace (the roofline cross-check)."""
import csv
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(ROOT, "tools", "pmc_summary.py"))
pmc = importlib.util.module_from_spec(spec)
spec.loader.exec_module(pmc)

KN = {"model_kernel": "model_kernel(Params, void const*, int)", "logic_kernel": "logic_kernel(Params, float*)",
      "ray_sensor_kernel": "ray_sensor_kernel(Params, float*, float*, int)"}
FULL = {"model_kernel": 683 * 128, "logic_kernel": 683 * 128, "ray_sensor_kernel": 683 * 4 * 128}


def _trace(path, rows):
    cols = ["Kind", "Agent_Id", "Queue_Id", "Stream_Id", "Thread_Id", "Dispatch_Id", "Kernel_Id", "Kernel_Name",
            "Correlation_Id", "Start_Timestamp", "End_Timestamp", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
            "Accum_VGPR_Count", "SGPR_Count", "Workgroup_Size_X", "Workgroup_Size_Y", "Workgroup_Size_Z",
            "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"]
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        for i, (kn, t0, t1, grid) in enumerate(rows):
            w.writerow({c: 0 for c in cols} | {"Dispatch_Id": i, "Kernel_Name": KN[kn], "Start_Timestamp": t0,
                                                "End_Timestamp": t1, "Grid_Size_X": grid, "Grid_Size_Y": 1,
                                                "Grid_Size_Z": 1})


def test_trace_steps_full_grid_and_sharded(tmp_path):
    rows, t = [], 0
    for _ in range(3):                          # 3 per-step (full-grid) steps: 100 + 20 + 70 ns
        for kn, d in (("model_kernel", 100), ("logic_kernel", 20), ("ray_sensor_kernel", 70)):
            rows.append((kn, t, t + d, FULL[kn]))
            t += d + 5
    t += 1000
    start = t
    for k in range(4):                          # a 4-step rollout over 4 shards, shards overlapping
        for s in range(4):
            b = start + k * 150 + s * 10
            rows.append(("model_kernel", b, b + 80, FULL["model_kernel"] // 4))
            rows.append(("logic_kernel", b + 80, b + 95, FULL["logic_kernel"] // 4))
            rows.append(("ray_sensor_kernel", b + 95, b + 140, FULL["ray_sensor_kernel"] // 4))
    end = start + 3 * 150 + 3 * 10 + 140
    t = end + 1000
    rows.append(("model_kernel", t, t + 100, FULL["model_kernel"]))   # a full-grid launch closes the run
    p = tmp_path / "run_kernel_trace.csv"
    _trace(p, rows)
    r = pmc._trace_steps(str(p))
    assert r["model_kernel_full_grid_calls"] == 4 and r["model_kernel_full_grid_avg_ns"] == 100
    assert r["logic_kernel_full_grid_avg_ns"] == 20 and r["ray_sensor_kernel_full_grid_avg_ns"] == 70
    assert r["sharded_steps_traced"] == 4
    assert r["sharded_step_ns"] == (end - start) / 4


def test_counters_scaled_to_full_grid(tmp_path):
    cols = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id", "Grid_Size",
            "Kernel_Id", "Kernel_Name", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
            "Accum_VGPR_Count", "SGPR_Count", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]
    p = tmp_path / "run_counter_collection.csv"
    with open(p, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        # one full-grid dispatch (400 KiB over two rows: per-XCD instances sum) and four quarter-grid ones (100 KiB)
        for d, (grid, vals) in enumerate([(4000, (150.0, 250.0)), (1000, (100.0,)), (1000, (60.0, 40.0)),
                                          (1000, (100.0,)), (1000, (100.0,))]):
            for v in vals:
                w.writerow({c: 0 for c in cols} | {"Dispatch_Id": d, "Grid_Size": grid, "Kernel_Name": KN["model_kernel"],
                                                    "Counter_Name": "FETCH_SIZE", "Counter_Value": v})
    vals = pmc._per_dispatch(str(p), "FETCH_SIZE", "model_kernel")
    assert sorted(vals) == [400.0] * 5
    assert pmc._per_dispatch(str(p), "WRITE_SIZE", "model_kernel") == []
