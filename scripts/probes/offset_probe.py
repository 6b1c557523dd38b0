#!/usr/bin/env python3
"""C2 x1024: launch time vs the byte offset between the source and destination buffers (GPU box
tooling).  One pool; three batches; each batch's destination starts OFF bytes after a 2 MiB-aligned
position past the sources.  After a settle, 30 launches per layout; mean ms and frac."""
import os
import sys
import json
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import libiqo_amd

dev = torch.device("cuda", 0)
cfg = os.environ.get("OFF_CFG", "c2")
import bench
m, d, sw, sh, dw, dh, px, frames, label = bench.CONFIGS[cfg]
r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px, device=0)
stream = torch.cuda.current_stream(dev)
S, D = frames * sw * sh, frames * dw * dh
rot = 3
MB2 = 2 << 20
offs = [int(x) for x in os.environ.get("OFFS", "0 4096 65536 1048576 2097280 3145728").split()]
span_src = rot * ((S + MB2 - 1) // MB2 * MB2)
span_dst = rot * ((D + MB2 - 1) // MB2 * MB2 + max(offs) + MB2)
pool = torch.empty(span_src + span_dst + MB2, dtype=torch.uint8, device=dev)
base = (pool.data_ptr() + MB2 - 1) // MB2 * MB2 - pool.data_ptr()
g = torch.Generator(device=dev)
g.manual_seed(5)
srcs = []
for b in range(rot):
    o = base + b * ((S + MB2 - 1) // MB2 * MB2)
    t = pool[o:o + S]
    t.copy_(torch.randint(0, 256, (S,), dtype=torch.uint8, device=dev, generator=g))
    srcs.append(t)
for off in offs:
    dsts = []
    for b in range(rot):
        o = base + span_src + b * ((D + MB2 - 1) // MB2 * MB2 + max(offs) + MB2) + off
        dsts.append(pool[o:o + D])
    k = [0]

    def launch():
        bb = k[0] % rot
        k[0] += 1
        r.resize_device(frames, sw, sw * sh, srcs[bb].data_ptr(), dw, dw * dh, dsts[bb].data_ptr(), stream.cuda_stream)
    n_settle = max(30, int(150 / 2.0))
    for _ in range(n_settle):
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
        per.setdefault((n_settle + i) % rot, []).append(t)
    mean = sum(ts) / len(ts)
    print(json.dumps({"cfg": cfg, "dst_offset": off, "mean_ms": round(mean, 4),
                      "per_batch": {b: round(sorted(v)[len(v) // 2], 4) for b, v in sorted(per.items())},
                      "frac": round(frames * (sw * sh + dw * dh) / mean / 1e6 / 8000, 4)}), flush=True)
