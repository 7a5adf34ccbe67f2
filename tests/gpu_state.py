"""Decode libnascar's device state arena (nascar_get_state) into per-car field dicts,
for state-level parity diffs against the CPU oracle.  TEST INFRASTRUCTURE."""
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fields(kind):
    lines = open(os.path.join(ROOT, "nascargymnasium_amd", "csrc", "nascar_layout.h")).read().splitlines()
    i = next(k for k, l in enumerate(lines) if l.startswith("#define NASCAR_%s_FIELDS(X)" % kind))
    body = []
    while True:
        body.append(lines[i])
        if not lines[i].rstrip().endswith("\\"):
            break
        i += 1
    return re.findall(r"X\((\w+)\)", " ".join(body[1:]) if body[0].rstrip().endswith("\\") else body[0])


F32, F64, I32 = _fields("F32"), _fields("F64"), _fields("I32")


def _a256(x):
    return (x + 255) & ~255


def decode(blob: np.ndarray, N: int):
    b = blob.view(np.uint8)
    o = 0
    f32 = b[o:o + 4 * len(F32) * N].view(np.float32).reshape(len(F32), N); o = _a256(o + 4 * len(F32) * N)
    f64 = b[o:o + 8 * len(F64) * N].view(np.float64).reshape(len(F64), N); o = _a256(o + 8 * len(F64) * N)
    i32 = b[o:o + 4 * len(I32) * N].view(np.int32).reshape(len(I32), N)
    out = {}
    for i, f in enumerate(F32):
        out[f] = f32[i]
    for i, f in enumerate(F64):
        out[f] = f64[i]
    for i, f in enumerate(I32):
        out[f] = i32[i]
    return out
