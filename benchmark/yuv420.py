#!/usr/bin/env python3
"""YUV 4:2:0 (I420) batch throughput -- the reference benchmark's three-plane workload
(benchmark/benchmark.cpp:131-229; Lanczos chroma with pxScale 2) on device-resident frames.
Not the headline metric (bench.py); SURVEY 8(d) C1 "also report the YUV420 3-plane figure" and
8(f)2.

  python benchmark/yuv420.py [--config c2|c1|c3|c4] [--frames N] [--steps K]

Prints one JSON line: frames/s, output Mpix/s over all three planes, whether one launch did all
planes, ms per step, and the HBM rate on algorithmic bytes.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import libiqo_amd

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(bench.CONFIGS))
    ap.add_argument("--frames", type=int, default=0)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    m, d, sw, sh, dw, dh, _, default_frames, label = bench.CONFIGS[args.config]
    frames = args.frames or max(1, (default_frames * 2) // 3)  # same bytes as the 1-plane batch
    dev = torch.device("cuda", 0)
    r = libiqo_amd.Yuv420Resizer(m, d, sw, sh, dw, dh)
    ins = sw * sh + 2 * (sw // 2) * (sh // 2)
    outs = dw * dh + 2 * (dw // 2) * (dh // 2)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    src = torch.randint(0, 256, (frames, ins), dtype=torch.uint8, device=dev, generator=g)
    out = torch.empty((frames, outs), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    fused = False
    for _ in range(args.warmup):
        _, fused = r.resize_frames(src, out, stream)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        r.resize_frames(src, out, stream)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    ms = e0.elapsed_time(e1) / args.steps
    print(json.dumps({"workload": "YUV420 " + label.split(" ", 1)[1].replace("1ch", "I420"), "frames": frames,
                      "one_launch": fused, "ms_per_step": round(ms, 4),
                      "frames_per_s": round(frames * args.steps / wall, 1),
                      "out_mpix_s": round(frames * outs * args.steps / wall / 1e6, 1),
                      "hbm_gb_s": round(frames * (ins + outs) / (ms / 1e3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
