"""cfg5's per-rank cost of the distance sensors' beam lists: device memory and host build time of all 8 tracks.

    python tools/cfg5_memory.py [--cell 1.0] [--envs 4096] [--cars 10]

One process per cell size (the beam lists are cached process-wide per track): creates a BatchedCarEnv with env e on
track e mod 8 (cfg5's rank shape), and prints one JSON line with the device memory the handle took (hipMemGetInfo
before / after, so the state arena is included and reported apart), the wall-clock creation time, and the per-track
list sizes and build times from the engine's NASCAR_VERBOSE log.
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    sys.path.insert(0, ROOT)
    import torch
    from nascargymnasium_amd.batched import BatchedCarEnv
    from nascargymnasium_amd.track import available_tracks
    tracks = available_tracks()
    files = [tracks[e % len(tracks)] for e in range(a.envs)]
    torch.cuda.init()
    free0 = torch.cuda.mem_get_info()[0]
    t0 = time.time()
    env = BatchedCarEnv(a.envs, a.cars, files, device="cuda:0", beam_cell=a.cell)
    torch.cuda.synchronize()
    t1 = time.time()
    free1 = torch.cuda.mem_get_info()[0]
    arena = env.state_bytes() if hasattr(env, "state_bytes") else None
    env.close()
    print(json.dumps({"cell_m": a.cell, "envs": a.envs, "cars": a.cars, "tracks": len(tracks),
                      "device_bytes": free0 - free1, "state_arena_bytes": arena, "create_s": round(t1 - t0, 2)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cell", type=float, default=1.0)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--cars", type=int, default=10)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a)
    with tempfile.TemporaryFile("w+") as err:
        env = dict(os.environ, NASCAR_VERBOSE="1")
        out = subprocess.run([sys.executable, __file__, "--child", "--cell", str(a.cell), "--envs", str(a.envs),
                              "--cars", str(a.cars)], env=env, stdout=subprocess.PIPE, stderr=err, text=True)
        err.seek(0)
        log = err.read()
    if out.returncode != 0:
        sys.stderr.write(log)
        sys.exit(out.returncode)
    line = json.loads(out.stdout.strip().splitlines()[-1])
    per = []
    for m in re.finditer(r"heads ([\d.]+) MB \+ continuations ([\d.]+) MB \+ cell map ([\d.]+) MB, built in ([\d.]+) s", log):
        per.append({"heads_mb": float(m.group(1)), "cont_mb": float(m.group(2)), "cellmap_mb": float(m.group(3)),
                    "build_s": float(m.group(4))})
    line["per_track"] = per
    line["lists_mb"] = round(sum(p["heads_mb"] + p["cont_mb"] + p["cellmap_mb"] for p in per), 1)
    line["build_s_total"] = round(sum(p["build_s"] for p in per), 2)
    print(json.dumps(line))


if __name__ == "__main__":
    main()
