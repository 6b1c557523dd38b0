#!/usr/bin/env python3
"""Host-pointer drop-in throughput (reference resize() semantics: host buffers, synchronous),
against the PCIe bytes it has to move.  Not the headline metric (that is device-resident, see
bench.py); this is SURVEY 8(f)1.

  python benchmark/host_path.py [--config c2] [--reps 50]

Prints one JSON line per buffer kind (pageable numpy / pinned torch): ms per frame, output
Mpix/s, and the PCIe rate it implies ((src + dst bytes) / time).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import bench
    import libiqo_amd

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(bench.CONFIGS))
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    m, d, sw, sh, dw, dh, px, _, label = bench.CONFIGS[args.config]
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    rng = np.random.default_rng(5)
    frame = rng.integers(0, 256, (sh, sw), dtype=np.uint8)
    kinds = {
        "pageable": (frame, np.zeros((dh, dw), np.uint8)),
        "pinned": (torch.from_numpy(frame).pin_memory(), torch.zeros((dh, dw), dtype=torch.uint8).pin_memory()),
    }
    ref = None
    for kind, (src, dst) in kinds.items():
        for _ in range(3):
            r.resize(sw, src, dw, dst)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            r.resize(sw, src, dw, dst)
        dt = (time.perf_counter() - t0) / args.reps
        out = dst if isinstance(dst, np.ndarray) else dst.numpy()
        if ref is None:
            ref = out.copy()
        print(json.dumps({"path": "host-pointer iqo_hip_resize", "buffers": kind, "workload": label,
                          "ms_per_frame": round(dt * 1e3, 4), "out_mpix_s": round(dw * dh / dt / 1e6, 1),
                          "pcie_gb_s": round((sw * sh + dw * dh) / dt / 1e9, 2),
                          "same_output": bool((out == ref).all())}), flush=True)


if __name__ == "__main__":
    main()
