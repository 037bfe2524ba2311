"""Ceiling probe (not product code): hipBLASLt (torch.matmul) bf16 throughput on the encoder GEMM shapes of the
bench workload (large-v3, 150 windows = 225,000 rows), to compare with gemm_8p_kernel's rocprof times.

Usage (GPU box): python tools/blas_probe.py [rows]
"""
import sys
import time

import torch


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 225000
    dev = torch.device("cuda:0")
    shapes = [("qkv", 3840, 1280), ("out", 1280, 1280), ("fc1", 5120, 1280), ("fc2", 1280, 5120)]
    g = torch.Generator(device=dev).manual_seed(0)
    for name, N, K in shapes:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g) * 0.02
        for _ in range(3):
            c = a @ w.t()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 10
        e0.record()
        for _ in range(it):
            c = a @ w.t()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        print(f"{name:4s} M={M} N={N} K={K}: {ms:8.3f} ms  {2.0 * M * N * K / ms / 1e9:7.1f} TF/s", flush=True)
        del a, w, c
        time.sleep(0.2)


if __name__ == "__main__":
    main()
