#!/usr/bin/env python3
"""HBM calibration for PMC readings: a 4 GiB read (sum), a 2 GiB copy and a
2 GiB fill with known byte counts; prints achieved GB/s.  Run under
rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE to calibrate those counters."""
import time

import torch


def timeit(f, n=5):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def main():
    x = torch.ones(1 << 30, device="cuda")  # 4 GiB
    y = torch.empty(1 << 29, device="cuda")
    xs = x[: 1 << 29]
    t = timeit(lambda: x.sum())
    print("read  4 GiB: %.3f ms  %.0f GB/s" % (t * 1e3, 4 * 2**30 / t / 1e9))
    t = timeit(lambda: y.copy_(xs))
    print("copy  2+2 GiB: %.3f ms  %.0f GB/s" % (t * 1e3, 4 * 2**30 / t / 1e9))
    t = timeit(lambda: y.fill_(1.0))
    print("fill  2 GiB: %.3f ms  %.0f GB/s" % (t * 1e3, 2 * 2**30 / t / 1e9))


if __name__ == "__main__":
    main()
