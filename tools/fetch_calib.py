"""FETCH_SIZE / WRITE_SIZE calibration on known byte counts (MI355X_MICROARCH.md: "calibrate on a known byte count in your
own access pattern before trusting an absolute").  Runs each pattern of tools/fetch_calib.hip once over a 1 GiB buffer;
under `rocprofv3 --pmc FETCH_SIZE` (or WRITE_SIZE) the per-dispatch counter divided by the bytes printed here is the
counter's ratio for that pattern.  Diagnostic tooling.

    hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o tools/build/libfetch_calib.so tools/fetch_calib.hip
    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT -o run -- python3 tools/fetch_calib.py
    python3 tools/fetch_calib.py --summary OUT_FETCH OUT_WRITE
"""
import ctypes
import glob
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GiB = 1 << 30
REC = 1 << 20          # gathered records / loaded lines
PATTERNS = [           # (id, kernel name, description, known bytes)
    (0, "stream4", "coalesced stream, 4 B per lane (SoA f32 / i32 fields)", GiB),
    (1, "stream8", "coalesced stream, 8 B per lane (SoA f64 fields)", GiB),
    (2, "stream16", "coalesced stream, 16 B per lane (the guide's reference pattern)", GiB),
    (3, "gather16", "16 lanes x 16 B of one random 256-B record (a car's 16-byte list heads)", REC * 256),
    (4, "gather8", "16 lanes x 8 B of one random 128-B record (a car's 8-byte list heads)", REC * 128),
    (5, "line4", "one 4-B load per random 128-B line (cell map lookups)", REC * 4),
    (6, "line8", "one 8-B load per random 128-B line", REC * 8),
    (7, "wstream4", "coalesced store stream, 4 B per lane", GiB),
    (8, "wstream8", "coalesced store stream, 8 B per lane", GiB),
]


def run():
    import torch
    lib = ctypes.CDLL(os.path.join(ROOT, "tools/build/libfetch_calib.so"))
    lib.calib_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    buf = torch.ones(GiB // 4, dtype=torch.float32, device="cuda")
    out = torch.zeros(1024, dtype=torch.float32, device="cuda")
    flush = torch.ones(GiB // 4, dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for pid, name, desc, known in PATTERNS:
        flush.mul_(1.0001)             # 1 GiB of other traffic between patterns: nothing of buf left in the caches
        torch.cuda.synchronize()
        rc = lib.calib_run(pid, buf.data_ptr(), GiB, REC, out.data_ptr(), s)
        torch.cuda.synchronize()
        assert rc == 0, (name, rc)
        print(f"{name}: {known} bytes ({desc})", flush=True)


def summary(dirs):
    rows = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**/*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].replace("void ", "").split("(")[0].split("<")[0]
                rows.setdefault((k, r["Counter_Name"]), []).append(float(r["Counter_Value"]) * 1024)
    for pid, name, desc, known in PATTERNS:
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            v = [x for (k, cn), xs in rows.items() if cn == c and k == name for x in xs]
            if v:
                per = f", {sum(v) / REC:.1f} B per record / load" if pid in (3, 4, 5, 6) else ""
                print(f"{name:9s} {c}: {sum(v):.4g} B counted / {known:.4g} B known = {sum(v) / known:.3f}{per}  ({desc})")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--summary":
        summary(sys.argv[2:])
    else:
        run()
