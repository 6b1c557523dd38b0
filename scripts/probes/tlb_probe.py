#!/usr/bin/env python3
"""C2 x1024 on 3 rotated batches (bench.py's layout), 12 launches after a short settle, for a
rocprofv3 --pmc pass: per-dispatch UTCL1 translation counters by batch (GPU box tooling)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import libiqo_amd

dev = torch.device("cuda", 0)
sw, sh, dw, dh, frames, rot = 3840, 2160, 1920, 1080, 1024, 3
r = libiqo_amd.make_resizer("lanczos", 3, sw, sh, dw, dh, 1, device=0)
g = torch.Generator(device=dev)
g.manual_seed(1234)
src = torch.randint(0, 256, (rot, frames, sh, sw), dtype=torch.uint8, device=dev, generator=g)
dst = torch.empty((rot, frames, dh, dw), dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream(dev).cuda_stream
for i in int(os.environ.get("TLB_LAUNCHES", "24")) * [0] and range(int(os.environ.get("TLB_LAUNCHES", "24"))):
    b = i % rot
    r.resize_device(frames, sw, sw * sh, src[b].data_ptr(), dw, dw * dh, dst[b].data_ptr(), s)
torch.cuda.synchronize()
print("done")
