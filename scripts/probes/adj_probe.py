#!/usr/bin/env python3
"""Find where a 2:1 ryx column mode differs from the oracle (GPU box tooling)."""
import sys
import os
os.environ.setdefault("IQO_HIP_TUNING", "1")  # A/B option keys (include/iqo_hip.h)
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch
import libiqo_amd
import oracle_lib as ol

d, sw, sh = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
frames = int(sys.argv[4])
dw, dh = sw // 2, sh // 2
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(1234)
src = torch.randint(0, 256, (frames, sh, sw), dtype=torch.uint8, device=dev, generator=g)
exp0 = ol.run_oracle("lanczos", d, sw, sh, dw, dh, 1, src[0].cpu().numpy())
expL = ol.run_oracle("lanczos", d, sw, sh, dw, dh, 1, src[-1].cpu().numpy())
for opts in ({}, {"ryx_adj": 0}, {"bands": 1}, {"bands": 200}, {"ryx_split": 0}):
    r = libiqo_amd.make_resizer("lanczos", d, sw, sh, dw, dh, 1)
    for k, v in opts.items():
        r.set_option(k, v)
    out = r.resize_tensor(src)
    torch.cuda.synchronize()
    o0, oL = out[0].cpu().numpy(), out[-1].cpu().numpy()
    for name, o, e in (("first", o0, exp0), ("last", oL, expL)):
        bad = np.argwhere(o != e)
        print(opts, r.describe()["kernel"], name, bad.shape[0], bad[:5].tolist(),
              [(int(o[tuple(b)]), int(e[tuple(b)])) for b in bad[:5]], flush=True)
