"""Experiment: why C2 per-frame throughput drops past ~130 frames per call.  Times the same
launch on different halves of one 256-frame allocation and on separate allocations."""
import sys
import time

import torch

sys.path.insert(0, ".")
import libiqo_amd  # noqa: E402

dev = torch.device("cuda", 0)
r = libiqo_amd.LanczosResizer(3, 3840, 2160, 1920, 1080)
sw, sh, dw, dh = 3840, 2160, 1920, 1080


def timeit(src, dst, n, reps=30):
    s = torch.cuda.current_stream()
    for _ in range(3):
        r.resize_device(n, sw, sw * sh, src, dw, dw * dh, dst, s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        r.resize_device(n, sw, sw * sh, src, dw, dw * dh, dst, s)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


big = torch.randint(0, 256, (256, sh, sw), dtype=torch.uint8, device=dev)
out = torch.empty((256, dh, dw), dtype=torch.uint8, device=dev)
fb, ob = sw * sh, dw * dh
p, q = big.data_ptr(), out.data_ptr()
print("256 frames one call      %.4f ms" % timeit(p, q, 256))
print("frames 0..127            %.4f ms" % timeit(p, q, 128))
print("frames 128..255          %.4f ms" % timeit(p + 128 * fb, q + 128 * ob, 128))
print("frames 64..191           %.4f ms" % timeit(p + 64 * fb, q + 64 * ob, 128))
print("src 0..127 -> dst 128..  %.4f ms" % timeit(p, q + 128 * ob, 128))
print("src 128.. -> dst 0..127  %.4f ms" % timeit(p + 128 * fb, q, 128))
a = torch.randint(0, 256, (128, sh, sw), dtype=torch.uint8, device=dev)
ao = torch.empty((128, dh, dw), dtype=torch.uint8, device=dev)
print("separate 128 alloc       %.4f ms" % timeit(a.data_ptr(), ao.data_ptr(), 128))
for n in (64, 96, 128, 160, 192):
    print("first %3d frames         %.4f ms  (%.4f per 128)" % (n, timeit(p, q, n), timeit(p, q, n) * 128 / n))
