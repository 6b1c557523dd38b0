#!/usr/bin/env python3
"""Compare 2:1 ryx column modes against each other on whole batches, repeatedly (GPU box tooling)."""
import sys
import os
os.environ.setdefault("IQO_HIP_TUNING", "1")  # A/B option keys (include/iqo_hip.h)
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import libiqo_amd

frames = int(sys.argv[1])
reps = int(sys.argv[2])
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(99)
for d in [int(x) for x in os.environ.get('ADJ_DEGREES', '5 6 7 8 9').split()]:
    sw, sh = 3840, 2160
    dw, dh = sw // 2, sh // 2
    src = torch.randint(0, 256, (frames, sh, sw), dtype=torch.uint8, device=dev, generator=g)
    ref = libiqo_amd.make_resizer("lanczos", d, sw, sh, dw, dh, 1)
    ref.set_option("ryx_adj", 0)
    ref.set_option("ryx_uc", 0)
    want = ref.resize_tensor(src)
    for name, opts in (("adj", {}), ("uc", {"ryx_adj": 0}))[: int(os.environ.get("ADJ_ARMS", "2"))]:
        r = libiqo_amd.make_resizer("lanczos", d, sw, sh, dw, dh, 1)
        for k, v in opts.items():
            r.set_option(k, v)
        bad = 0
        where = []
        per = []
        for _ in range(reps):
            out = r.resize_tensor(src)
            diff = (out != want)
            n = int(diff.sum())
            per.append(n)
            bad += n
            if n and len(where) < 4:
                idx = diff.nonzero()[:2].tolist()
                where += [(i, int(out[tuple(i)]), int(want[tuple(i)])) for i in idx]
        print("L%d %-4s bad pixels over %d reps: %d per rep %s %s" % (d, name, reps, bad, per, where), flush=True)
