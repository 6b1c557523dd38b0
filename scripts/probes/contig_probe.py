#!/usr/bin/env python3
"""C2 x1024: per-batch launch time with the batches in physically contiguous device memory
(hipExtMallocWithFlags(hipDeviceMallocContiguous)) vs torch's allocator (GPU box tooling)."""
import ctypes
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import libiqo_amd

dev = torch.device("cuda", 0)
torch.zeros(1, device=dev)
hip = ctypes.CDLL("libamdhip64.so")
sw, sh, dw, dh, frames, rot = 3840, 2160, 1920, 1080, 1024, 3
S, D = frames * sw * sh, frames * dw * dh
r = libiqo_amd.make_resizer("lanczos", 3, sw, sh, dw, dh, 1, device=0)
stream = torch.cuda.current_stream(dev)
g = torch.Generator(device=dev)
g.manual_seed(1234)


def timeit(srcs, dsts, label):
    k = [0]

    def launch():
        b = k[0] % rot
        k[0] += 1
        r.resize_device(frames, sw, sw * sh, srcs[b], dw, dw * dh, dsts[b], stream.cuda_stream)
    for _ in range(110):
        launch()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(31)]
    e[0].record(stream)
    for i in range(30):
        launch()
        e[i + 1].record(stream)
    torch.cuda.synchronize()
    ts = [e[i].elapsed_time(e[i + 1]) for i in range(30)]
    per = {}
    for i, t in enumerate(ts):
        per.setdefault((110 + i) % rot, []).append(t)
    mean = sum(ts) / len(ts)
    print(json.dumps({"layout": label, "mean_ms": round(mean, 4), "frac": round(frames * (sw * sh + dw * dh) / mean / 1e6 / 8000, 4),
                      "per_batch": {b: round(sorted(v)[len(v) // 2], 4) for b, v in sorted(per.items())}}), flush=True)


def contig(n, flags):
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(n), ctypes.c_uint(flags))
    if rc != 0:
        raise RuntimeError("hipExtMallocWithFlags rc %d" % rc)
    return p.value


for rep in range(2):
    src = torch.randint(0, 256, (rot, frames, sh, sw), dtype=torch.uint8, device=dev, generator=g)
    dst = torch.empty((rot, frames, dh, dw), dtype=torch.uint8, device=dev)
    timeit([src[b].data_ptr() for b in range(rot)], [dst[b].data_ptr() for b in range(rot)], "torch")
    cs = [contig(S, 0x4) for _ in range(rot)]
    cd = [contig(D, 0x4) for _ in range(rot)]
    for b in range(rot):
        hip.hipMemcpy(ctypes.c_void_p(cs[b]), ctypes.c_void_p(src[b].data_ptr()), ctypes.c_size_t(S), 3)
    torch.cuda.synchronize()
    del src, dst
    torch.cuda.empty_cache()
    timeit(cs, cd, "hipDeviceMallocContiguous")
    for p in cs + cd:
        hip.hipFree(ctypes.c_void_p(p))
