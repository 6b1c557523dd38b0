#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X resize hot path.

Metric (BASELINE.json): output Mpix/s of Lanczos-3 U8 3840x2160 -> 1920x1080 (config C2), one
process per GPU, frames sharded by image across ranks (weak scaling: each rank resizes its own
device-resident batch; no data-path collective), plus the HBM roofline fraction of the kernel.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c1] [--frames B]
  torchrun --nproc-per-node N bench.py --gpus N ...

A "step" = one pass of the hot path over the rank's batch (one libiqo_hip launch).  Inputs are
synthetic uniform-random U8 frames generated on the device before timing.  Rank 0 prints ONE
JSON line.  The CPU baseline (rank 0, N=1 only) times the reference's own Generic implementation
(oracle/_ref, compiled from its sources) -- or the oracle restatement when _ref is absent -- on
the host cores over a bounded sample of the same workload.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (method, degree, srcW, srcH, dstW, dstH, pxScale, default frames per GPU, label)
    "c2": ("lanczos", 3, 3840, 2160, 1920, 1080, 1, 128, "C2 Lanczos-3 U8 1ch 3840x2160->1920x1080"),
    "c3": ("area", 0, 7680, 4320, 1920, 1080, 1, 48, "C3 Area U8 1ch 7680x4320->1920x1080"),
    "c4": ("linear", 0, 1920, 1080, 3840, 2160, 1, 128, "C4 Linear U8 1ch 1920x1080->3840x2160"),
    "c1": ("lanczos", 2, 640, 480, 320, 240, 1, 4096, "C1 Lanczos-2 U8 1ch 640x480->320x240"),
    # general-kernel shapes (not BASELINE configs): multi-phase downscale, Lanczos upscale
    "g1": ("lanczos", 3, 1920, 1080, 1280, 720, 1, 128, "G1 Lanczos-3 U8 1ch 1920x1080->1280x720"),
    "g2": ("lanczos", 3, 1920, 1080, 3840, 2160, 1, 32, "G2 Lanczos-3 U8 1ch 1920x1080->3840x2160"),
    "g3": ("area", 0, 1920, 1080, 1280, 720, 1, 128, "G3 Area U8 1ch 1920x1080->1280x720"),
}


def log(msg):
    print("[bench] " + msg, file=sys.stderr, flush=True)


def baseline_metric():
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            return json.load(f)["metric"]
    except Exception:
        return "Mpix/s Lanczos-3 U8 4K->1080p at 1/2/4/8 GPUs; achieved HBM GB/s %peak"


def cpu_baseline(cfg, frame_np, seconds, threads):
    """Bounded CPU sample of the same workload on this node's host cores."""
    import ctypes

    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as ol

    m, d, sw, sh, dw, dh, px = cfg[:7]
    kind, runner = "port", None
    if ol.ref_available():
        try:
            runner = ol.ref().iqo_ref_run_batch
            kind = "reference"
        except OSError:
            runner = None
    if runner is None:
        runner = ol.oracle().iqo_oracle_run_batch
    u8p = ctypes.POINTER(ctypes.c_uint8)
    src = np.ascontiguousarray(frame_np)
    dst = np.zeros((threads, dh, dw), np.uint8)

    def run(nthr, reps):
        t = 0.0
        for _ in range(reps):
            # nthr frames (one per worker), src frame stride 0: each worker resizes the same input
            t += runner(ol.METHODS[m], d, sw, sh, dw, dh, px, nthr, sw, 0, src.ctypes.data_as(u8p), dw, dh * dw,
                        dst.ctypes.data_as(u8p), nthr)
        return t

    t1 = run(1, 1)  # calibrate
    reps1 = max(1, int(0.25 * seconds / max(t1, 1e-6)))
    t1 = run(1, reps1)
    one = reps1 * dw * dh / t1 / 1e6
    tn = run(threads, 1)
    repsn = max(1, int(0.75 * seconds / max(tn, 1e-6)))
    tn = run(threads, repsn)
    alln = repsn * threads * dw * dh / tn / 1e6
    # parity of the baseline itself (worker 0's output) against the oracle
    exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, src)
    ok = bool((dst[0] == exp).all())
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(alln, 2), "unit": "Mpix/s", "cores": threads, "kind": kind,
            "sample": "%d reps x %d frames (one per thread) + 1-thread %d frames of %s, %s impl, src %s" %
                      (repsn, threads, reps1, cfg[8], "Generic" if kind == "reference" else "oracle port",
                       "noise"),
            "value_1thread": round(one, 2), "cpu_model": model, "matches_oracle": ok,
            "seconds": round(t1 + tn, 2)}


def kernel_is_lanczos(method, r):
    return method == "lanczos" and r.describe()["kernel"] == "lanczos_stream"


def read_pmc(config):
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % config)
    try:
        with open(path) as f:
            return json.load(f)
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--frames", type=int, default=0, help="frames per GPU (0 = config default)")
    ap.add_argument("--bands", type=int, default=0, help="row bands per frame (0 = auto)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--force-general", action="store_true")
    ap.add_argument("--debug-flags", type=int, default=0, help="timing experiments (wrong output)")
    ap.add_argument("--prefetch", type=int, default=0, help="Lanczos streamer prefetch depth (0 = default)")
    ap.add_argument("--variant", type=int, default=-1, help="Lanczos streamer: 0 symmetric, 1 ring (A/B)")
    ap.add_argument("--lanes", type=int, default=0, help="symmetric streamer producing lanes per wave (0 = auto)")
    ap.add_argument("--option", action="append", default=[], metavar="KEY=VALUE",
                    help="extra plan option (iqo_hip_plan_set_option), repeatable")
    args = ap.parse_args()

    import torch

    import libiqo_amd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("warning: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    cfg = CONFIGS[args.config]
    m, d, sw, sh, dw, dh, px, default_frames, label = cfg
    frames = args.frames or default_frames
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px, device=local)
    if args.bands:
        r.set_option("bands", args.bands)
    if args.force_general:
        r.set_option("force_general", 1)
    if args.debug_flags:
        r.set_option("debug_flags", args.debug_flags)
    if args.prefetch and kernel_is_lanczos(m, r):
        r.set_option("prefetch", args.prefetch)
    if args.variant >= 0 and kernel_is_lanczos(m, r):
        r.set_option("stream_variant", args.variant)
    if args.lanes and kernel_is_lanczos(m, r):
        r.set_option("lanes", args.lanes)
    for kv in args.option:
        k, v = kv.split("=", 1)
        r.set_option(k, int(v))
    kernel = r.describe()["kernel"]

    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    src = torch.randint(0, 256, (frames, sh, sw), dtype=torch.uint8, device=dev, generator=gen)
    dst = torch.empty((frames, dh, dw), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    def step():
        r.resize_device(frames, sw, sw * sh, src.data_ptr(), dw, dw * dh, dst.data_ptr(), sp)

    log("rank %d/%d %s frames=%d kernel=%s warmup=%d steps=%d" % (rank, world, label, frames, kernel,
                                                                  args.warmup, args.steps))
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps

    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # timing bookkeeping only, not the data path
    wall_max = float(t.item())

    parity = "unchecked"
    if rank == 0 and not args.no_verify:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as ol
        ok = True
        for f in sorted({0, frames - 1}):
            exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, src[f].cpu().numpy())
            ok = ok and bool((dst[f].cpu().numpy() == exp).all())
        parity = "bit-exact vs Generic oracle (frames 0 and last)" if ok else "MISMATCH"
        log("parity: " + parity)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
        threads = max(1, min(threads, 16))
        log("cpu baseline: %d threads, ~%.0f s" % (threads, args.cpu_seconds))
        cpu = cpu_baseline(cfg, src[0].cpu().numpy(), args.cpu_seconds, threads)

    if rank == 0:
        out_px = float(frames) * dw * dh * world * args.steps
        value = out_px / wall_max / 1e6
        bytes_launch = float(frames) * (sw * sh + dw * dh)
        achieved = bytes_launch / (kern_ms / 1e3) / 1e9
        pmc = read_pmc(args.config)
        traffic = None
        if pmc and pmc.get("frames") == frames and pmc.get("kernel") == kernel:
            traffic = pmc.get("hbm_bytes_per_launch")
        res = {
            "metric": baseline_metric() if args.config == "c2" else "Mpix/s " + label,
            "value": round(value, 1),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: uniform random U8 frames generated on device (torch.randint, seed 1234+rank)",
            "config": {"workload": label, "frames_per_gpu": frames, "global_frames": frames * world,
                       "parallelism": "image-sharded x%d (independent shards, no collective)" % world,
                       "kernel": kernel, "bands_per_frame": args.bands or "auto",
                       "step": "one libiqo_hip launch over the rank's device-resident batch"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "kernel_ms_per_launch": round(kern_ms, 4),
                         "algorithmic_bytes_per_launch": int(bytes_launch)},
            "cpu_baseline": cpu,
            "parity": parity,
        }
        if cpu and cpu.get("value"):
            res["gpu_over_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(res), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
