#!/usr/bin/env python3
"""Steady-state A/B of plan options in ONE process (GPU box tooling, not product code).

Why: the MI355X lowers its GFX clock for ~10-20 ms after a streaming kernel starts (a power-
management transient: GRBM_GUI_ACTIVE per C2 dispatch fell from ~2.3 to ~1.5 GHz and recovered
over ~40 launches, profiles/r05/clock_transient.txt).  Short bench runs (warmup 2-5 launches) time
the kernels inside that dip, where they are partly compute-bound, so A/B results from them mix
clock and memory effects.  Here every arm runs after a continuous settle phase, the arms are
interleaved in short blocks of back-to-back launches with no host synchronisation in between, and
the per-block times of each arm are reported (median / min), so slow clock drift hits all arms
alike.

  python scripts/probes/steady_ab.py --config c2 [--frames 256] [--settle-ms 80] [--block 8]
         [--reps 8] --arm base: --arm nb:bands=135,rounds=0 ...

An arm is NAME:key=value,key=value (plan options, iqo_hip_plan_set_option).  The library is the one
libiqo_amd loads (LIBIQO_AMD_LIB selects a variant build).  Each arm's frame 0 is checked bit for
bit against the oracle after the timing.
"""
import argparse
import json
import os
os.environ.setdefault("IQO_HIP_TUNING", "1")  # A/B option keys (include/iqo_hip.h)
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402  (CONFIGS)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--frames", type=int, default=0)
    ap.add_argument("--settle-ms", type=float, default=80.0)
    ap.add_argument("--block", type=int, default=8)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--arm", action="append", default=[])
    ap.add_argument("--trace", action="store_true", help="print the settle phase's per-launch ms")
    ap.add_argument("--tag", default="")
    ap.add_argument("--shape", default="", help="method,degree,srcW,srcH,dstW,dstH,frames instead of --config")
    args = ap.parse_args()
    import torch

    import libiqo_amd

    if args.shape:
        f = args.shape.split(",")
        m, (d, sw, sh, dw, dh, default_frames), px = f[0], map(int, f[1:7]), 1
        args.config = "%s%d:%dx%d->%dx%d" % (m, d, sw, sh, dw, dh)
    else:
        m, d, sw, sh, dw, dh, px, default_frames, label = bench.CONFIGS[args.config]
    frames = args.frames or default_frames
    dev = torch.device("cuda", 0)
    arms = []
    for spec in (args.arm or ["base:"]):
        name, _, opts = spec.partition(":")
        r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px, device=0)
        for kv in filter(None, opts.split(",")):
            k, v = kv.split("=", 1)
            r.set_option(k, int(v))
        arms.append((name, r))
    bytes_launch = float(frames) * (sw * sh + dw * dh)
    rot = max(2, int(-(-2.5e9 // bytes_launch)))
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    src = torch.randint(0, 256, (rot, frames, sh, sw), dtype=torch.uint8, device=dev, generator=g)
    dst = torch.empty((rot, frames, dh, dw), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    k = [0]

    def launch(r):
        b = k[0] % rot
        k[0] += 1
        r.resize_device(frames, sw, sw * sh, src[b].data_ptr(), dw, dw * dh, dst[b].data_ptr(), sp)

    # settle: the first arm back to back for ~settle-ms (per-launch events, to show the transient)
    torch.cuda.synchronize(dev)
    launch(arms[0][1])
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    launch(arms[0][1])
    e1.record(stream)
    torch.cuda.synchronize(dev)
    est = max(e0.elapsed_time(e1), 0.01)
    n_settle = max(1, int(args.settle_ms / est))
    sev = [torch.cuda.Event(enable_timing=True) for _ in range(n_settle + 1)]
    sev[0].record(stream)
    for i in range(n_settle):
        launch(arms[0][1])
        sev[i + 1].record(stream)
    # interleaved blocks, no host sync until the end
    evs = []
    for rep in range(args.reps):
        order = arms if rep % 2 == 0 else arms[::-1]
        for name, r in order:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(args.block):
                launch(r)
            b.record(stream)
            evs.append((name, a, b))
    torch.cuda.synchronize(dev)
    settle = [sev[i].elapsed_time(sev[i + 1]) for i in range(n_settle)]
    res = {}
    for name, a, b in evs:
        res.setdefault(name, []).append(a.elapsed_time(b) / args.block)
    out = {"config": args.config, "frames": frames, "tag": args.tag, "lib": libiqo_amd.LIB_PATH,
           "settle_launches": n_settle, "settle_first_ms": round(settle[0], 4),
           "settle_max_ms": round(max(settle), 4), "settle_last8_ms": round(sum(settle[-8:]) / 8, 4), "arms": {}}
    if args.trace:
        out["settle_trace"] = [round(x, 4) for x in settle]
    import numpy as np

    import oracle_lib as ol
    for name, r in arms:
        v = sorted(res[name])
        med = v[len(v) // 2]
        # parity of this arm: one more launch on batch 0, frame 0 vs the oracle
        r.resize_device(frames, sw, sw * sh, src[0].data_ptr(), dw, dw * dh, dst[0].data_ptr(), sp)
        torch.cuda.synchronize(dev)
        exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, src[0, 0].cpu().numpy())
        ok = bool(np.array_equal(dst[0, 0].cpu().numpy(), exp))
        out["arms"][name] = {"kernel": r.describe()["kernel"], "median_ms": round(med, 4), "min_ms": round(v[0], 4),
                             "max_ms": round(v[-1], 4), "frac_median": round(bytes_launch / med / 1e6 / 8000, 4),
                             "frac_min": round(bytes_launch / v[0] / 1e6 / 8000, 4), "bit_exact_frame0": ok,
                             "blocks": [round(x, 4) for x in res[name]]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
