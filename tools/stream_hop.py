"""Latency of a cross-stream event hop vs same-stream ordering (tiny kernels), for the split-step design."""
import torch

dev = torch.device("cuda:0")
x = torch.zeros(1024, device=dev)
s0 = torch.cuda.current_stream()
s1 = torch.cuda.Stream()
for mode in ("same", "hop"):
    for it in range(2):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s0)
        for _ in range(200):
            x.add_(1.0)
            if mode == "hop":
                ev = torch.cuda.Event()
                ev.record(s0)
                s1.wait_event(ev)
                with torch.cuda.stream(s1):
                    x.add_(1.0)
                ev2 = torch.cuda.Event()
                ev2.record(s1)
                s0.wait_event(ev2)
            else:
                x.add_(1.0)
        b.record(s0)
        torch.cuda.synchronize()
        if it:
            print(f"{mode}: {a.elapsed_time(b) * 1e3 / 200:.1f} us per pair of kernels")
