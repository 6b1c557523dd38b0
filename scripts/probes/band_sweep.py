#!/usr/bin/env python3
"""Band-count sweep around each config's auto choice (GPU-box tooling): prints the steady_ab.py
command line for arms {auto, auto/2, 2 auto, 3 auto} plus any extra arms, for one config.

  python scripts/probes/band_sweep.py CONFIG [extra arms...]   -> runs steady_ab.py in-process"""
import os
import subprocess
import sys

os.environ.setdefault("IQO_HIP_TUNING", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (before the library: torch's HIP init fails after libiqo_hip.so initialised HIP)

import bench  # noqa: E402
import libiqo_amd  # noqa: E402


def main():
    cfg = sys.argv[1]
    m, d, sw, sh, dw, dh, px, frames, label = bench.CONFIGS[cfg]
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px, device=0)
    src = torch.zeros((frames, sh, sw), dtype=torch.uint8, device="cuda:0")
    r.resize_tensor(src)  # (the auto band count is decided at the first launch)
    b = r.describe()["bands"]
    arms = ["auto:"]
    for v in sorted({max(1, b // 2), 2 * b, 3 * b} - {b}):
        arms.append("b%d:bands=%d" % (v, v))
    arms += sys.argv[2:]
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "probes", "steady_ab.py"), "--config", cfg, "--settle-ms", "120",
           "--reps", "6", "--block", "8", "--tag", "auto_bands=%d" % b]
    for a in arms:
        cmd += ["--arm", a]
    sys.exit(subprocess.call(cmd))


if __name__ == "__main__":
    main()
