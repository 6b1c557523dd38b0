#!/usr/bin/env python3
"""Host <-> device transfer rates that bound the host-pointer drop-in path (GPU box tooling).

The C2 I420 cycle moves 12.4 MB up (Y 3840x2160 + U, V 1920x1080) and 3.1 MB down.  Measured here:
pinned H2D / D2H over 1..4 streams at once (each stream a separate SDMA queue), pageable -> pinned
memcpy with 1..16 threads, and pageable H2D through the runtime's own staging.  Min over reps."""
import concurrent.futures as cf
import ctypes
import json
import time

import numpy as np
import torch

dev = torch.device("cuda", 0)
MB = 1 << 20
up, down = 12441600, 3110400
res = {}


def tmin(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


hs = torch.empty(up, dtype=torch.uint8).pin_memory()
hd = torch.empty(down, dtype=torch.uint8).pin_memory()
ds = torch.empty(up, dtype=torch.uint8, device=dev)
dd = torch.empty(down, dtype=torch.uint8, device=dev)
streams = [torch.cuda.Stream(dev) for _ in range(4)]
for n in (1, 2, 3, 4):
    def h2d():
        for i in range(n):
            a, b = up * i // n, up * (i + 1) // n
            with torch.cuda.stream(streams[i]):
                ds[a:b].copy_(hs[a:b], non_blocking=True)
    t = tmin(h2d)
    res["h2d_pinned_%dstreams_GBps" % n] = round(up / t / 1e9, 2)

    def d2h():
        for i in range(n):
            a, b = down * i // n, down * (i + 1) // n
            with torch.cuda.stream(streams[i]):
                hd[a:b].copy_(dd[a:b], non_blocking=True)
    t = tmin(d2h)
    res["d2h_pinned_%dstreams_GBps" % n] = round(down / t / 1e9, 2)


def both():
    with torch.cuda.stream(streams[0]):
        ds[: up // 2].copy_(hs[: up // 2], non_blocking=True)
    with torch.cuda.stream(streams[1]):
        ds[up // 2:].copy_(hs[up // 2:], non_blocking=True)
    with torch.cuda.stream(streams[2]):
        hd.copy_(dd, non_blocking=True)


res["h2d2_plus_d2h_concurrent_ms"] = round(tmin(both) * 1e3, 4)
pg = np.random.default_rng(0).integers(0, 256, up, dtype=np.uint8)
pgt = torch.from_numpy(pg)
res["h2d_pageable_1stream_GBps"] = round(up / tmin(lambda: ds.copy_(pgt)) / 1e9, 2)
hsn = hs.numpy()
for nt in (1, 4, 8, 16):
    pool = cf.ThreadPoolExecutor(nt)

    def cp():
        parts = [(up * i // nt, up * (i + 1) // nt) for i in range(nt)]
        list(pool.map(lambda ab: ctypes.memmove(hsn.ctypes.data + ab[0], pg.ctypes.data + ab[0], ab[1] - ab[0]), parts))
    res["memcpy_pageable_to_pinned_%dthr_GBps" % nt] = round(up / tmin(cp) / 1e9, 2)
    pool.shutdown()
print(json.dumps(res), flush=True)
