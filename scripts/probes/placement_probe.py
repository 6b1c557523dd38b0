#!/usr/bin/env python3
"""C2 x1024 per-batch kernel time by buffer layout (GPU box tooling): the two rotated batches of
bench.py alternate ~1.82 / ~1.90 ms under rocprof.  Layouts: one (rot, frames, h, w) allocation
(bench.py), one allocation per batch, and the destination allocated first; 2 and 3 batches.  After a
~200 ms settle, per-launch HIP-event times are recorded for 40 launches and summarised per batch."""
import os
import sys
import json
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import libiqo_amd

dev = torch.device("cuda", 0)
sw, sh, dw, dh, frames = 3840, 2160, 1920, 1080, 1024
r = libiqo_amd.make_resizer("lanczos", 3, sw, sh, dw, dh, 1, device=0)
stream = torch.cuda.current_stream(dev)
g = torch.Generator(device=dev)
g.manual_seed(1234)


def run(srcs, dsts, label):
    n = len(srcs)
    k = [0]

    def launch():
        b = k[0] % n
        k[0] += 1
        r.resize_device(frames, sw, sw * sh, srcs[b].data_ptr(), dw, dw * dh, dsts[b].data_ptr(), stream.cuda_stream)
    for _ in range(110):
        launch()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(41)]
    evs[0].record(stream)
    for i in range(40):
        launch()
        evs[i + 1].record(stream)
    torch.cuda.synchronize()
    ts = [evs[i].elapsed_time(evs[i + 1]) for i in range(40)]
    start = 110 % n
    per = {}
    for i, t in enumerate(ts):
        per.setdefault((start + i) % n, []).append(t)
    out = {"layout": label, "batches": n,
           "per_batch_ms": {b: round(sorted(v)[len(v) // 2], 4) for b, v in sorted(per.items())},
           "mean_ms": round(sum(ts) / len(ts), 4)}
    out["frac_mean"] = round(frames * (sw * sh + dw * dh) / out["mean_ms"] / 1e6 / 8000, 4)
    print(json.dumps(out), flush=True)


ROTS = [int(x) for x in os.environ.get("PLACE_ROTS", "2 3").split()]
LAYOUTS = os.environ.get("PLACE_LAYOUTS", "one per dfirst").split()
for rot in ROTS:
    for lay in LAYOUTS:
        if lay == "one":
            src = torch.randint(0, 256, (rot, frames, sh, sw), dtype=torch.uint8, device=dev, generator=g)
            dst = torch.empty((rot, frames, dh, dw), dtype=torch.uint8, device=dev)
            run([src[b] for b in range(rot)], [dst[b] for b in range(rot)], "one allocation (bench.py)")
            del src, dst
        elif lay == "per":
            srcs = [torch.randint(0, 256, (frames, sh, sw), dtype=torch.uint8, device=dev, generator=g) for _ in range(rot)]
            dsts = [torch.empty((frames, dh, dw), dtype=torch.uint8, device=dev) for _ in range(rot)]
            run(srcs, dsts, "one allocation per batch")
            del srcs, dsts
        else:
            dsts = [torch.empty((frames, dh, dw), dtype=torch.uint8, device=dev) for _ in range(rot)]
            srcs = [torch.randint(0, 256, (frames, sh, sw), dtype=torch.uint8, device=dev, generator=g) for _ in range(rot)]
            run(srcs, dsts, "destinations first, one per batch")
            del srcs, dsts
        torch.cuda.empty_cache()
