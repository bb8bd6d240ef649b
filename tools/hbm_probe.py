#!/usr/bin/env python3
"""Achievable HBM bandwidth on this GPU with PyTorch's own kernels (write-only fill, read+write copy, read-only
sum) at the decode batch's sizes -- a practical ceiling next to the 8 TB/s datasheet peak."""
import torch


def bench(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    n = 4_500_000_000 // 4
    a = torch.empty(n, dtype=torch.int32, device="cuda")
    b = torch.empty(n, dtype=torch.int32, device="cuda")
    t = bench(lambda: a.fill_(7))
    print("fill (write) %.1f MB: %.3f ms  %.0f GB/s" % (4 * n / 1e6, t, 4 * n / t / 1e6))
    t = bench(lambda: b.copy_(a))
    print("copy (read+write) %.1f MB each: %.3f ms  %.0f GB/s (r+w)" % (4 * n / 1e6, t, 8 * n / t / 1e6))
    t = bench(lambda: a.sum())
    print("sum (read) %.1f MB: %.3f ms  %.0f GB/s" % (4 * n / 1e6, t, 4 * n / t / 1e6))
    m = 450_000_000 // 4
    t = bench(lambda: b[:4 * m * 5 // 4].copy_(a[:m].repeat(5)[: 4 * m * 5 // 4]) if False else b[: 5 * m].view(5, m).copy_(a[:m].expand(5, m)))
    print("expand copy: read %.0f MB, write %.0f MB: %.3f ms  %.0f GB/s (r+w)" % (4 * m / 1e6, 20 * m / 1e6, t, 24 * m / t / 1e6))


if __name__ == "__main__":
    main()
