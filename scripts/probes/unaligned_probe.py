#!/usr/bin/env python3
"""Do unaligned dword buffer loads work on this GPU?  ryx / ryg on a source whose base and row stride
are not 4-byte aligned (option unaligned_src), compared with the oracle (GPU box tooling)."""
import os
os.environ.setdefault("IQO_HIP_TUNING", "1")  # A/B option keys (include/iqo_hip.h)
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch
import libiqo_amd
import oracle_lib as ol

dev = torch.device("cuda", 0)
for m, d, sw, sh, dw, dh in (("lanczos", 3, 1920, 1080, 1366, 768), ("lanczos", 3, 1920, 1080, 854, 480),
                             ("area", 0, 1920, 1080, 1366, 768)):
    rng = np.random.default_rng(3)
    frame = rng.integers(0, 256, (sh, sw), dtype=np.uint8)
    exp = ol.run_oracle(m, d, sw, sh, dw, dh, 1, frame)
    for off, pad in ((1, 3), (2, 2), (3, 5)):
        st = sw + pad
        buf = torch.zeros(sh * st + 64, dtype=torch.uint8, device=dev)
        view = buf[off:off + sh * st].view(sh, st)
        view[:, :sw] = torch.from_numpy(frame).to(dev)
        out = torch.zeros((dh, dw), dtype=torch.uint8, device=dev)
        r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, 1)
        r.set_option("unaligned_src", 1)
        r.resize_device(1, st, sh * st, view.data_ptr(), dw, dh * dw, out.data_ptr())
        torch.cuda.synchronize()
        bad = int((out.cpu().numpy() != exp).sum())
        print(m, d, sw, sh, dw, dh, "offset", off, "stride", st, "kernel", r.describe()["kernel"], "bad pixels", bad, flush=True)
