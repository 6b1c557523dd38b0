"""Host-pointer latency of the drop-in path on a small I420 frame (C1: Y 640x480 -> 320x240,
U/V 320x240 -> 160x120, Lanczos-2): plan construction, per-plane resize(), the 3-plane
Yuv420Resizer cycle with the constructor inside the loop (the reference benchmark's timed
region, benchmark/benchmark.cpp:206-229).  Min / median microseconds over N repetitions."""
import statistics
import torch  # noqa: F401  (before libiqo_amd: torch initialises the HIP runtime first)
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

# Large I420 frames (C2: Y 3840x2160 -> 1920x1080, U/V 1920x1080 -> 960x540, Lanczos-3): the
# three-plane host pipeline from pageable and from pinned user buffers (pinned: no staging copy),
# and the Y plane alone, to separate staging, PCIe and the pipeline's own overhead.
import torch  # noqa: E402

assert torch.cuda.is_available()  # initialises the HIP runtime in torch before pin_memory()
W, H, w, h = 3840, 2160, 1920, 1080
for kind in ("pageable", "pinned"):
    def mk(shape, fill=None):
        t = torch.zeros(shape, dtype=torch.uint8)
        if kind == "pinned":
            t = t.pin_memory()
        a = t.numpy()
        if fill is not None:
            a[...] = fill
        return t, a
    (_, Yb), (_, Ub), (_, Vb) = mk((H, W), rng.integers(0, 256, (H, W), dtype=np.uint8)), \
        mk((H // 2, W // 2), 7), mk((H // 2, W // 2), 9)
    (_, yb), (_, ub), (_, vb) = mk((h, w)), mk((h // 2, w // 2)), mk((h // 2, w // 2))
    yr = libiqo_amd.Yuv420Resizer("lanczos", 3, W, H, w, h)
    print("C2 I420 %-8s (plan reused) " % kind,
          timed(lambda: yr.resize(W, Yb, W // 2, Ub, Vb, w, yb, w // 2, ub, vb), n=40))
    rY = libiqo_amd.LanczosResizer(3, W, H, w, h)
    print("C2 Y     %-8s              " % kind, timed(lambda: rY.resize(W, Yb, w, yb), n=40))
