#!/usr/bin/env python3
"""Relaunch every bench config's kernel on one batch and compare the outputs bit for bit
(GPU box tooling): a kernel with a synchronisation race gives different bytes from launch to
launch, which one frame checked against the oracle can miss.

  python scripts/probes/determinism.py [--reps 8] [--frames-cap 128] [cfg ...]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--frames-cap", type=int, default=128)
    ap.add_argument("cfgs", nargs="*")
    args = ap.parse_args()
    import torch
    import libiqo_amd
    dev = torch.device("cuda", 0)
    bad_total = 0
    for c in args.cfgs or list(bench.CONFIGS):
        m, d, sw, sh, dw, dh, px, frames, label = bench.CONFIGS[c]
        frames = min(frames, args.frames_cap, max(1, int(2.0e9 // (sw * sh + dw * dh))))
        g = torch.Generator(device=dev)
        g.manual_seed(7)
        src = torch.randint(0, 256, (frames, sh, sw), dtype=torch.uint8, device=dev, generator=g)
        r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px, device=0)
        first = r.resize_tensor(src)
        per = []
        for _ in range(args.reps):
            per.append(int((r.resize_tensor(src) != first).sum()))
        bad_total += sum(per)
        print("%-3s %-14s frames %5d differing bytes per relaunch %s" % (c, r.describe()["kernel"], frames, per), flush=True)
    print("TOTAL differing bytes", bad_total)
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()
