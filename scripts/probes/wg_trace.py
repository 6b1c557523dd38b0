#!/usr/bin/env python3
"""Workgroup timeline of the block-shared Lanczos streamer (GPU-box tooling, variant builds only).

A library built with -DIQO_VARIANT_DEBUG (scripts/build_variant.sh trace "-DIQO_VARIANT_DEBUG")
records, per workgroup, {start, end} on the 100 MHz clock and where it ran (HW_ID, XCC_ID) when
plan option trace_addr points at a device buffer.  After a settle phase at a steady clock, one
launch is traced and summarised: the span, the ramp (how long until the resident workgroups run
in steady state), the tail (the time from the first slot running out of work to the last
workgroup's end), workgroup durations by launch phase, and per-XCD end times.

  LIBIQO_AMD_LIB=libiqo_amd/variants/trace.so python scripts/probes/wg_trace.py --frames 256
"""
import argparse
import json
import os
import sys

os.environ.setdefault("IQO_HIP_TUNING", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import libiqo_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--settle-ms", type=float, default=150.0)
    ap.add_argument("--option", action="append", default=[])
    ap.add_argument("--dump", default="")
    a = ap.parse_args()
    m, d, sw, sh, dw, dh, px, _, label = bench.CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px, device=0)
    for kv in a.option:
        k, v = kv.split("=", 1)
        r.set_option(k, int(v))
    F = a.frames
    rot = 3
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    src = torch.randint(0, 256, (rot, F, sh, sw), dtype=torch.uint8, device=dev, generator=g)
    dst = torch.empty((rot, F, dh, dw), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)
    k = [0]

    def launch():
        b = k[0] % rot
        k[0] += 1
        r.resize_device(F, sw, sw * sh, src[b].data_ptr(), dw, dw * dh, dst[b].data_ptr(), st.cuda_stream)

    launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    launch()
    e1.record(st)
    torch.cuda.synchronize()
    n = max(1, int(a.settle_ms / max(e0.elapsed_time(e1), 0.01)))
    maxBlocks = F * 1100 * 4
    trace = torch.zeros(maxBlocks * 4, dtype=torch.int64, device=dev)  # (bytes: 16 per workgroup)
    for _ in range(n):
        launch()
    r.set_option("trace_addr", trace.data_ptr())
    launch()  # traced, back to back with the settle launches
    r.set_option("trace_addr", 0)
    for _ in range(4):
        launch()
    torch.cuda.synchronize()
    rec = trace.cpu().numpy().view(np.uint32).reshape(-1, 4)
    rec = rec[(rec[:, 0] != 0) | (rec[:, 1] != 0)]
    t0, t1 = rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64)
    base = t0.min()
    t0 -= base
    t1 -= base
    dur = (t1 - t0) / 100.0  # us
    span = t1.max() / 100.0
    hw, xcc = rec[:, 2], rec[:, 3]
    cu = (hw >> 8) & 0xF
    sh_ = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    slot = (xcc & 0xF) * 1000 + se * 100 + sh_ * 16 + cu
    # active workgroups over time (1 us bins)
    nb = int(span) + 2
    act = np.zeros(nb)
    for s_, e_ in zip(t0, t1):
        act[int(s_ // 100):int(e_ // 100) + 1] += 1
    steady = np.median(act[nb // 4: 3 * nb // 4])
    ramp = int(np.argmax(act >= 0.95 * steady))
    lastFull = nb - 1 - int(np.argmax(act[::-1] >= 0.95 * steady))
    # per-XCD end
    xe = {int(x): float(t1[(xcc & 0xF) == x].max() / 100.0) for x in np.unique(xcc & 0xF)}
    ord_ = np.argsort(t0)
    n_ = len(ord_)
    first = dur[ord_[: n_ // 20]]
    mid = dur[ord_[n_ // 2 - n_ // 40: n_ // 2 + n_ // 40]]
    last = dur[ord_[-n_ // 20:]]
    out = {"config": a.config, "frames": F, "options": a.option, "workgroups": int(n_), "span_us": round(span, 2),
           "steady_active": float(steady), "ramp_us_to_95pct": ramp, "tail_us_below_95pct": round(span - lastFull, 2),
           "idle_slot_us_in_tail": round(float(np.sum(np.clip(steady - act[lastFull:], 0, None))) / max(steady, 1), 2),
           "dur_us_first5pct": [round(float(np.median(first)), 2), round(float(first.max()), 2)],
           "dur_us_mid5pct": [round(float(np.median(mid)), 2), round(float(mid.max()), 2)],
           "dur_us_last5pct": [round(float(np.median(last)), 2), round(float(last.max()), 2)],
           "xcd_end_us": xe, "slots": int(len(np.unique(slot))),
           "active_profile_us": [int(x) for x in act[::max(1, nb // 60)]]}
    print(json.dumps(out), flush=True)
    if a.dump:
        np.save(a.dump, np.stack([t0, t1, hw.astype(np.int64), xcc.astype(np.int64)], 1))


if __name__ == "__main__":
    main()
