import ctypes, torch
import sys
L = ctypes.CDLL(sys.argv[1] if len(sys.argv) > 1 else "tools/lat_bench.so")
print(sys.argv[1:])
out = torch.zeros(16, dtype=torch.int64, device="cuda"); sink = torch.zeros(256, device="cuda")
L.lat_bench(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(sink.data_ptr()))
o = out.cpu().tolist()
names = ["dep v_add_f32", "4-way indep v_add_f32", "IEEE div (dep)", "IEEE sqrt (dep)", "glibc sincosf", "dep v_fma_f64", "LDS store+load", "dep v_mul_f32", "select chain",
         "flat LDS store+load", "flat LDS + global store", "LDS + global store", "f64 div (dep)", "f64 sqrt (dep)", "global load (dep)"]
per = [256, 256, 64, 64, 64, 256, 64, 256, 64, 64, 64, 64, 64, 64, 64]
for n, v, p in zip(names, o, per): print(f"{n:24s} {v:7d} cycles total, {v/p:7.1f} per op")
