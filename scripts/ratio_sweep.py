#!/usr/bin/env python3
"""Kernel time and HBM roofline fraction over common video scaling ratios, on fresh device batches
(distinct batches cycled, >= 2.5 GB per cycle, as bench.py) after an ~80 ms settle of back-to-back
launches per shape (steady GPU clock, round 5), each output checked against the oracle on one frame.
Output: one line per shape (profiles/r05/ratio_sweep.txt).

  python scripts/ratio_sweep.py [--steps 20] [--match linear:1280x720] [--opt ratio_prefetch=1 ...]
"""
import argparse
import os
os.environ.setdefault("IQO_HIP_TUNING", "1")  # A/B option keys (include/iqo_hip.h)
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

SHAPES = [
    # method, degree, srcW, srcH, dstW, dstH
    ("lanczos", 3, 3840, 2160, 2560, 1440),
    ("lanczos", 3, 3840, 2160, 1920, 1080),
    ("lanczos", 3, 3840, 2160, 1280, 720),
    ("lanczos", 3, 1920, 1080, 1280, 720),
    ("lanczos", 3, 1920, 1080, 960, 540),
    ("lanczos", 3, 1920, 1080, 854, 480),
    ("lanczos", 3, 1280, 720, 1920, 1080),
    ("lanczos", 3, 1920, 1080, 3840, 2160),
    ("lanczos", 2, 1920, 1080, 1280, 720),
    ("lanczos", 2, 1920, 1080, 960, 540),
    ("area", 0, 3840, 2160, 1920, 1080),
    ("area", 0, 1920, 1080, 1280, 720),
    ("area", 0, 1920, 1080, 854, 480),
    ("linear", 0, 1920, 1080, 3840, 2160),
    ("linear", 0, 1280, 720, 1920, 1080),
    # round 3: exact 3:1 (lanczos_d31, area_int with 12-column threads)
    ("lanczos", 2, 3840, 2160, 1280, 720),
    ("area", 0, 3840, 2160, 1280, 720),
    ("lanczos", 3, 1920, 1080, 640, 360),
    # round 3: exact vertical ratio, tabled columns (ryx)
    ("lanczos", 2, 1920, 1080, 854, 480),
    ("lanczos", 3, 1920, 1080, 640, 480),
    # round 4: the common shapes VERDICT r03 listed on the tile / walk kernels
    ("linear", 0, 3840, 2160, 1920, 1080),
    ("lanczos", 3, 3840, 2160, 960, 540),
    ("lanczos", 4, 3840, 2160, 1920, 1080),
    ("lanczos", 5, 3840, 2160, 1920, 1080),
    ("lanczos", 6, 3840, 2160, 1920, 1080),
    ("lanczos", 7, 3840, 2160, 1920, 1080),
    ("lanczos", 8, 3840, 2160, 1920, 1080),
    ("lanczos", 9, 3840, 2160, 1920, 1080),
    ("lanczos", 4, 1920, 1080, 960, 540),
    ("lanczos", 2, 3840, 2160, 960, 540),
    ("lanczos", 1, 3840, 2160, 1920, 1080),
    ("lanczos", 3, 1280, 720, 3840, 2160),
    ("linear", 0, 1280, 720, 3840, 2160),
    ("lanczos", 3, 640, 480, 1920, 1080),
    ("lanczos", 2, 640, 480, 1920, 1080),     # 4:9 upscale rows (ryx)
    ("lanczos", 3, 720, 480, 1620, 1080),
    ("lanczos", 3, 1920, 1080, 1366, 768),
    ("area", 0, 1920, 1080, 1366, 768),
    ("lanczos", 2, 1920, 1080, 1024, 576),
    ("linear", 0, 1920, 1080, 1280, 720),
    # round 5, late: ryg past 2:1, Linear on ryg, upscale rows
    ("lanczos", 3, 3840, 2160, 1366, 768),
    ("area", 0, 3840, 2160, 1366, 768),
    ("lanczos", 3, 3840, 2160, 1024, 576),
    ("linear", 0, 1920, 1080, 1366, 768),
    ("lanczos", 3, 1366, 768, 1920, 1080),
    ("lanczos", 3, 1024, 576, 1920, 1080),
    ("linear", 0, 1920, 1080, 1024, 576),
    ("linear", 0, 1920, 1080, 1600, 900),
    ("linear", 0, 2560, 1440, 1920, 1080),
    ("linear", 0, 3840, 2160, 2560, 1440),
    ("lanczos", 3, 2560, 1440, 1920, 1080),
    ("lanczos", 3, 1920, 1080, 1600, 900),
    ("lanczos", 2, 1920, 1080, 1600, 900),
    ("area", 0, 2560, 1440, 1920, 1080),
    ("area", 0, 1920, 1080, 1600, 900),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=80.0, help="untimed back-to-back launches before the timing")
    ap.add_argument("--match", default="", help="only shapes whose 'method:srcWxsrcH->dstWxdstH' contains this")
    ap.add_argument("--opt", action="append", default=[], help="plan option key=value (tuning runs)")
    args = ap.parse_args()
    import torch
    import libiqo_amd
    import oracle_lib as ol
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    print("%-8s %-3s %-11s %-11s %-14s %9s %8s %7s %s" % ("method", "deg", "src", "dst", "kernel", "frames", "ms", "%peak", "parity"))
    for m, d, sw, sh, dw, dh in SHAPES:
        if args.match not in "%s:%dx%d->%dx%d" % (m, sw, sh, dw, dh):
            continue
        per = sw * sh + dw * dh
        frames = max(8, min(256, int(1.3e9 // per)))
        rot = max(2, int(-(-2.5e9 // (per * frames))))
        r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh)
        for kv in args.opt:
            k, v = kv.split("=")
            r.set_option(k, int(v))
        kern = r.describe()["kernel"]
        src = torch.randint(0, 256, (rot, frames, sh, sw), dtype=torch.uint8, device=dev)
        dst = torch.empty((rot, frames, dh, dw), dtype=torch.uint8, device=dev)

        def launch(b):
            r.resize_device(frames, sw, sw * sh, src[b].data_ptr(), dw, dw * dh, dst[b].data_ptr(), s.cuda_stream)

        for i in range(2 * rot):
            launch(i % rot)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if args.settle_ms > 0:
            # the GPU lowers its clock for ~10-20 ms after a streaming kernel starts (round 5,
            # profiles/r05/clock_transient.txt): time the steady state after a continuous settle
            e0.record(s)
            launch(0)
            e1.record(s)
            torch.cuda.synchronize(dev)
            for i in range(int(args.settle_ms / max(e0.elapsed_time(e1), 0.005))):
                launch(i % rot)
        e0.record(s)
        for i in range(args.steps):
            launch(i % rot)
        e1.record(s)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / args.steps
        exp = ol.run_oracle(m, d, sw, sh, dw, dh, 1, src[0, 0].cpu().numpy())
        ok = bool((dst[0, 0].cpu().numpy() == exp).all())
        frac = per * frames / (ms * 1e-3) / 8e12
        print("%-8s %-3d %-11s %-11s %-14s %9d %8.4f %6.1f%% %s" % (m, d, "%dx%d" % (sw, sh), "%dx%d" % (dw, dh), kern,
                                                                  frames, ms, 100 * frac, "bit-exact" if ok else "MISMATCH"),
              flush=True)
        del src, dst
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
