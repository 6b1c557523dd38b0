"""Host-pointer latency of the drop-in path on a small I420 frame (C1: Y 640x480 -> 320x240,
U/V 320x240 -> 160x120, Lanczos-2): plan construction, per-plane resize(), the 3-plane
Yuv420Resizer cycle with the constructor inside the loop (the reference benchmark's timed
region, benchmark/benchmark.cpp:206-229).  Min / median microseconds over N repetitions."""
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import libiqo_amd  # noqa: E402


def timed(fn, n=200):
    for _ in range(10):
        fn()
    t = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return "min %7.1f us  median %7.1f us" % (min(t) * 1e6, statistics.median(t) * 1e6)


W, H, w, h = 640, 480, 320, 240
rng = np.random.default_rng(0)
Y = rng.integers(0, 256, (H, W), dtype=np.uint8)
U = rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8)
V = rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8)
y = np.zeros((h, w), np.uint8)
u = np.zeros((h // 2, w // 2), np.uint8)
v = np.zeros((h // 2, w // 2), np.uint8)
print("plan Lanczos-2 Y            ", timed(lambda: libiqo_amd.LanczosResizer(2, W, H, w, h)))
print("plan Yuv420Resizer          ", timed(lambda: libiqo_amd.Yuv420Resizer("lanczos", 2, W, H, w, h)))
rY = libiqo_amd.LanczosResizer(2, W, H, w, h)
print("resize Y (host pointers)    ", timed(lambda: rY.resize(W, Y, w, y)))
yr = libiqo_amd.Yuv420Resizer("lanczos", 2, W, H, w, h)
print("resize I420 (plan reused)   ", timed(lambda: yr.resize(W, Y, W // 2, U, V, w, y, w // 2, u, v)))


def cycle():
    r = libiqo_amd.Yuv420Resizer("lanczos", 2, W, H, w, h)
    r.resize(W, Y, W // 2, U, V, w, y, w // 2, u, v)


print("I420 cycle, ctor in loop    ", timed(cycle))
