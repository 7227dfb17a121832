#!/usr/bin/env python3
"""Experiment: timing events recorded inside a captured HIP graph (torch.cuda.Event(external=
True)) give per-replay elapsed times on ROCm.  Experiment tooling."""
import torch

s = torch.cuda.Stream()
a = torch.randn(2048, 2048, device="cuda", dtype=torch.float64)
with torch.cuda.stream(s):
    for _ in range(2):
        b = a @ a
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        e0 = torch.cuda.Event(enable_timing=True, external=True)
        e1 = torch.cuda.Event(enable_timing=True, external=True)
        e2 = torch.cuda.Event(enable_timing=True, external=True)
        e0.record()
        b = a @ a
        e1.record()
        c = b @ a
        c = c @ a
        e2.record()
    for i in range(3):
        g.replay()
        torch.cuda.synchronize()
        print("replay", i, "first gemm ms", e0.elapsed_time(e1), "two gemms ms", e1.elapsed_time(e2))
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    b = a @ a
    t1.record()
    torch.cuda.synchronize()
    print("eager gemm ms", t0.elapsed_time(t1))
