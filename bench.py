#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X resize hot path.

Metric (BASELINE.json): output Mpix/s of Lanczos-3 U8 3840x2160 -> 1920x1080 (config C2), one
process per GPU, plus the HBM roofline fraction of the kernel.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c1|g1|g2|g3]
                  [--frames B] [--shard image|band]
  torchrun --nproc-per-node N bench.py --gpus N ...

--shard image (default): each rank resizes its own device-resident batch of B frames (weak
  scaling, no data-path collective).  A "step" = one libiqo_hip launch over the rank's batch.
--shard band: every frame of one global batch of B frames is split by output-row band over the
  ranks (libiqo_amd/shard.py): each rank holds only its source window (the halo rows its band
  reads) of every frame, generated on its device from per-frame seeds (frame f is reproducible
  from f alone; --band-src host stages the window in pinned host memory instead and uploads it,
  timed as `scatter_ms`), a step = one iqo_hip_resize_band launch over its band of all B frames,
  and the bands are gathered to rank 0 by IPC handle + device copy, timed once, separately from
  the compute steps.  No rank allocates the global source batch.

Inputs are synthetic uniform-random U8 frames generated before timing.  Image mode cycles through
several distinct device batches, one per step (--rotate; auto: >= 3 batches and >= 2.5 GB per cycle): relaunching
the SAME batch lets the 256 MiB Infinity Cache serve part of the reads (C2: ~15 % faster), which no
real pipeline sees; that figure is reported separately as reuse_probe.  Rank 0 prints ONE JSON
line.  With the default config (C2) at N = 1 the line also carries `secondary`: C3 (64 frames) and
C4 (256 frames) timed the same way on their own rotated batches, with parity on frames 0, mid and
last, and a plain streaming kernel of each config's read:write byte mix (libiqo_probe.so) on the
same buffers -- the on-box ceiling each kernel's fraction can be read against.
The CPU baseline (rank 0, N=1 only) times the reference's own CPU path -- its public
classes with their CPUID dispatch (AVX512 on the node) and OpenMP, compiled from its sources into
oracle/_ref -- plus its Generic impl, on the host CPUs this process may use, over a bounded
sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (method, degree, srcW, srcH, dstW, dstH, pxScale, default frames per GPU, label)
    # C2: 1024 frames per launch (round 5) -- C5's whole batch (BASELINE.json configs[4]) on each GPU,
    # and >= BASELINE.md section 4's minimum of 256 for C2.  Why not 256 any more: the MI355X drops
    # its GFX clock to ~1.5 GHz for ~10-20 ms after a streaming kernel starts (power management;
    # GRBM_GUI_ACTIVE per dispatch, profiles/r05/clock_transient.txt), and at 256 frames (0.5 ms per
    # launch) a run of 5 warmup + 20 timed steps sits inside that dip; at 1024 frames (1.9 ms) the
    # warmup steps cover it.  Steady state per launch with round 5's 12-row bands: 1024 frames 1.857 ms
    # (frac 0.715), 256 frames 0.48 ms (0.69) (profiles/r05/steady_c2_final_opts.txt,
    # bench_lines_steady.jsonl).  The line also carries 256 frames (the round-3/4 headline batch) as
    # batch_alt.
    "c2": ("lanczos", 3, 3840, 2160, 1920, 1080, 1, 1024, "C2 Lanczos-3 U8 1ch 3840x2160->1920x1080"),
    "c3": ("area", 0, 7680, 4320, 1920, 1080, 1, 64, "C3 Area U8 1ch 7680x4320->1920x1080"),
    "c4": ("linear", 0, 1920, 1080, 3840, 2160, 1, 256, "C4 Linear U8 1ch 1920x1080->3840x2160"),
    "c1": ("lanczos", 2, 640, 480, 320, 240, 1, 4096, "C1 Lanczos-2 U8 1ch 640x480->320x240"),
    # general-ratio shapes (not BASELINE configs): multi-phase downscale, Lanczos upscale, Area
    "g1": ("lanczos", 3, 1920, 1080, 1280, 720, 1, 128, "G1 Lanczos-3 U8 1ch 1920x1080->1280x720"),
    "g2": ("lanczos", 3, 1920, 1080, 3840, 2160, 1, 32, "G2 Lanczos-3 U8 1ch 1920x1080->3840x2160"),
    "g3": ("area", 0, 1920, 1080, 1280, 720, 1, 128, "G3 Area U8 1ch 1920x1080->1280x720"),
    # video-ladder downscales past 2:1 (round 3 kernels): exact 3:1, exact 9:4 rows, Area 3:1
    "g4": ("lanczos", 3, 3840, 2160, 1280, 720, 1, 128, "G4 Lanczos-3 U8 1ch 3840x2160->1280x720"),
    "g5": ("lanczos", 3, 1920, 1080, 854, 480, 1, 256, "G5 Lanczos-3 U8 1ch 1920x1080->854x480"),
    "g6": ("area", 0, 3840, 2160, 1280, 720, 1, 128, "G6 Area U8 1ch 3840x2160->1280x720"),
    # narrow frames (frame-stacked streamer): the C1 I420 chroma plane size, single channel
    "n1": ("lanczos", 2, 320, 240, 160, 120, 1, 16384, "N1 Lanczos-2 U8 1ch 320x240->160x120"),
    "n2": ("lanczos", 3, 640, 360, 320, 180, 1, 4096, "N2 Lanczos-3 U8 1ch 640x360->320x180"),
    # round 4 kernels: Linear 2:1 (linear_d2), 4:1 and Lanczos-4..9 2:1 (ryx), exact 3x upscales
    "h1": ("linear", 0, 3840, 2160, 1920, 1080, 1, 128, "H1 Linear U8 1ch 3840x2160->1920x1080"),
    "h2": ("lanczos", 3, 3840, 2160, 960, 540, 1, 128, "H2 Lanczos-3 U8 1ch 3840x2160->960x540"),
    "h3": ("lanczos", 4, 3840, 2160, 1920, 1080, 1, 128, "H3 Lanczos-4 U8 1ch 3840x2160->1920x1080"),
    "h4": ("lanczos", 3, 1280, 720, 3840, 2160, 1, 64, "H4 Lanczos-3 U8 1ch 1280x720->3840x2160"),
    "h5": ("linear", 0, 1280, 720, 3840, 2160, 1, 64, "H5 Linear U8 1ch 1280x720->3840x2160"),
    "h6": ("lanczos", 6, 3840, 2160, 1920, 1080, 1, 128, "H6 Lanczos-6 U8 1ch 3840x2160->1920x1080"),
    "h7": ("lanczos", 7, 3840, 2160, 1920, 1080, 1, 128, "H7 Lanczos-7 U8 1ch 3840x2160->1920x1080"),
    "h8": ("lanczos", 8, 3840, 2160, 1920, 1080, 1, 128, "H8 Lanczos-8 U8 1ch 3840x2160->1920x1080"),
    "h9": ("lanczos", 9, 3840, 2160, 1920, 1080, 1, 128, "H9 Lanczos-9 U8 1ch 3840x2160->1920x1080"),
    # round 5: the walker shapes VERDICT r04 listed (1080p -> WXGA rows 45:32, -> 1024x576 rows 15:8)
    "w1": ("lanczos", 3, 1920, 1080, 1366, 768, 1, 256, "W1 Lanczos-3 U8 1ch 1920x1080->1366x768"),
    "w2": ("area", 0, 1920, 1080, 1366, 768, 1, 256, "W2 Area U8 1ch 1920x1080->1366x768"),
    "w3": ("lanczos", 2, 1920, 1080, 1024, 576, 1, 256, "W3 Lanczos-2 U8 1ch 1920x1080->1024x576"),
    "u1": ("lanczos", 3, 640, 480, 1920, 1080, 1, 256, "U1 Lanczos-3 U8 1ch 640x480->1920x1080"),
    "u2": ("lanczos", 3, 1024, 576, 1920, 1080, 1, 256, "U2 Lanczos-3 U8 1ch 1024x576->1920x1080"),
    "u3": ("lanczos", 3, 1366, 768, 1920, 1080, 1, 256, "U3 Lanczos-3 U8 1ch 1366x768->1920x1080"),
    "w4": ("lanczos", 3, 3840, 2160, 1366, 768, 1, 128, "W4 Lanczos-3 U8 1ch 3840x2160->1366x768"),
    "w5": ("area", 0, 3840, 2160, 1366, 768, 1, 128, "W5 Area U8 1ch 3840x2160->1366x768"),
    "w6": ("lanczos", 3, 3840, 2160, 1024, 576, 1, 128, "W6 Lanczos-3 U8 1ch 3840x2160->1024x576"),
    "w7": ("linear", 0, 1920, 1080, 1366, 768, 1, 256, "W7 Linear U8 1ch 1920x1080->1366x768"),
}


def log(msg):
    print("[bench] " + msg, file=sys.stderr, flush=True)


def baseline_metric():
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            return json.load(f)["metric"]
    except Exception:
        return "Mpix/s Lanczos-3 U8 4K->1080p at 1/2/4/8 GPUs; achieved HBM GB/s %peak"


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def cpu_baseline(cfg, seconds):
    """Bounded CPU sample of the same workload on this node's host CPUs (rank 0, N = 1)."""
    import ctypes

    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as ol

    m, d, sw, sh, dw, dh, px = cfg[:7]
    mi = ol.METHODS[m]
    aff, quota, usable = ol.host_cpus()
    u8p = ctypes.POINTER(ctypes.c_uint8)
    rng = np.random.default_rng(4321)
    # one distinct source frame per worker (not one frame re-read from cache by every worker)
    srcs = rng.integers(0, 256, (usable, sh, sw), dtype=np.uint8)
    dsts = np.zeros((usable, dh, dw), np.uint8)
    sp, dp = srcs.ctypes.data_as(u8p), dsts.ctypes.data_as(u8p)
    res = {"unit": "Mpix/s", "cores": usable, "affinity_cpus": aff, "cpu_quota": quota, "cpu_model": _cpu_model()}
    t_all = time.perf_counter()

    def timed(fn, per_call_frames, budget):
        """Calls fn(reps) with reps scaled to ~budget seconds; returns Mpix/s."""
        t = fn(1)
        reps = max(1, int(budget / max(t, 1e-6)))
        t = fn(reps)
        return reps * per_call_frames * dw * dh / t / 1e6

    if ol.ref_cpu_available():
        L = ol.ref_cpu()
        arch = L.iqo_refcpu_arch().decode()

        def rows(reps):  # the reference's own threading: OpenMP rows of one frame at a time
            return sum(L.iqo_refcpu_run_rows(mi, d, sw, sh, dw, dh, px, usable, sw, sw * sh, sp, dw, dw * dh, dp,
                                             usable) for _ in range(reps))

        def frames(reps):  # frame parallelism: one object per thread
            return sum(L.iqo_refcpu_run_frames(mi, d, sw, sh, dw, dh, px, usable, sw, sw * sh, sp, dw, dw * dh, dp,
                                               usable) for _ in range(reps))

        budget = seconds / 4.0
        simd_rows = timed(rows, usable, budget)
        simd_frames = timed(frames, usable, budget)
        simd_1 = timed(lambda reps: sum(L.iqo_refcpu_run_rows(mi, d, sw, sh, dw, dh, px, 1, sw, sw * sh, sp, dw,
                                                              dw * dh, dp, 1) for _ in range(reps)), 1, budget / 4)
        out0 = dsts[0].copy()
        exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, srcs[0])
        diff = np.abs(out0.astype(np.int16) - exp.astype(np.int16))
        best = max(simd_rows, simd_frames)
        res.update({"value": round(best, 2), "kind": "reference", "impl": "%s (reference CPUID dispatch)" % arch,
                    "threading": "OpenMP rows (reference)" if simd_rows >= simd_frames else "one object per thread",
                    arch.lower(): {"rows_openmp": round(simd_rows, 2), "frames_per_thread": round(simd_frames, 2),
                                   "value_1thread": round(simd_1, 2), "threads": usable,
                                   "vs_generic_max_abs_diff": int(diff.max()),
                                   "vs_generic_frac_px_differ": round(float((diff > 0).mean()), 4)}})
        budget_generic = seconds / 4.0
    else:
        res.update({"kind": "port", "impl": "Generic"})
        budget_generic = seconds / 2.0
    # Generic: the reference's own TUs (oracle/_ref) or, without them, the oracle restatement
    if ol.ref_available():
        runner, gkind = ol.ref().iqo_ref_run_batch, "reference"
    else:
        runner, gkind = ol.oracle().iqo_oracle_run_batch, "port"

    def gen_frames(nthr):
        return lambda reps: sum(runner(mi, d, sw, sh, dw, dh, px, nthr, sw, sw * sh, sp, dw, dw * dh, dp, nthr)
                                for _ in range(reps))

    g_all = timed(gen_frames(usable), usable, budget_generic * 0.75)
    g_1 = timed(gen_frames(1), 1, budget_generic * 0.25)
    exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, srcs[0])
    res["generic"] = {"value": round(g_all, 2), "value_1thread": round(g_1, 2), "threads": usable, "kind": gkind,
                      "matches_oracle": bool((dsts[0] == exp).all())}
    if "value" not in res:
        res["value"], res["value_1thread"] = res["generic"]["value"], res["generic"]["value_1thread"]
    res["sample"] = ("%s, %d distinct random frames (one per worker), CPUs: %d in the affinity mask, cgroup quota %s "
                     "-> %d threads; OMP_WAIT_POLICY=%s" % (cfg[8], usable, aff, quota, usable,
                                                           os.environ.get("OMP_WAIT_POLICY", "default")))
    res["seconds"] = round(time.perf_counter() - t_all, 2)
    return res


def reference_benchmark(cfg, cycles=0):
    """The workload as the reference benchmark reports it (benchmark/benchmark.cpp:206-229,
    :1017-1033): one I420 frame (Y at the config's size, U and V at half size; Lanczos chroma
    with pxScale 2), resizer objects constructed inside the timed region, min ms over the cycles
    (256 as the reference for frames up to 1 Mpx, 16 above) -- the reference's CPU path (its own
    TUs + CPUID dispatch, oracle/_ref) on 1 and on all usable host threads, beside the drop-in
    HIP path through host pointers, same cycle."""
    import ctypes

    import numpy as np

    import libiqo_amd

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as ol

    m, d, W, H, w, h = cfg[:6]
    cycles = cycles or (256 if W * H <= 1_000_000 else 16)
    rng = np.random.default_rng(0)
    Y, U, V = (rng.integers(0, 256, sz, dtype=np.uint8) for sz in ((H, W), (H // 2, W // 2), (H // 2, W // 2)))
    y, u, v = (np.zeros(sz, np.uint8) for sz in ((h, w), (h // 2, w // 2), (h // 2, w // 2)))
    u8p = ctypes.POINTER(ctypes.c_uint8)
    p = [a.ctypes.data_as(u8p) for a in (Y, U, V, y, u, v)]
    out = {"cycles": cycles, "workload": "benchmark -m %s -iw %d -ih %d -ow %d -oh %d (I420, ctor in loop)" %
           ("%s%d" % (m, d) if m == "lanczos" else m, W, H, w, h)}
    _, _, usable = ol.host_cpus()
    if ol.ref_cpu_available():
        L = ol.ref_cpu()
        for nthr in sorted({1, usable}):
            t = L.iqo_refcpu_bench_yuv420(ol.METHODS[m], d, W, H, w, h, cycles, nthr, p[0], p[1], p[2], W, W // 2,
                                          p[3], p[4], p[5], w, w // 2)
            out["cpu_ms_per_cycle_%dthr" % nthr] = round(t * 1e3, 4)
        out["cpu_impl"] = L.iqo_refcpu_arch().decode()
    best = 1e9
    for _ in range(cycles):
        t0 = time.perf_counter()
        r = libiqo_amd.Yuv420Resizer(m, d, W, H, w, h)
        r.resize(W, Y, W // 2, U, V, w, y, w // 2, u, v)
        best = min(best, time.perf_counter() - t0)
        del r
    out["gpu_host_ptr_ms_per_cycle"] = round(best * 1e3, 4)
    out["gpu_bit_exact_Y"] = bool((y == ol.run_oracle(m, d, W, H, w, h, 1, Y)).all())
    return out


def reuse_probe(step_batch, rot, dev, reps=10):
    """Kernel ms per launch when the SAME batch is launched again and again (the pre-round-2
    methodology) next to the rotated-batch figure: the Infinity Cache (256 MiB) serves part of a
    repeated launch's reads (C2: ~15 % faster), so `value` is measured on rotating batches and
    this number is context only."""
    import torch

    def timed(fn):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / reps

    same = timed(lambda: step_batch(0))
    cyc = iter(range(1 << 30))
    fresh = timed(lambda: step_batch(next(cyc) % rot))
    return {"same_batch_kernel_ms": round(same, 4), "rotated_kernel_ms": round(fresh, 4)}


def alt_batch(make_step, frames_alt, bytes_per_frame, dev, steps=20, settle_ms=60.0):
    """Kernel ms per launch at a second batch size (context, not the headline), on rotated fresh
    batches like the headline: same kernel, same plan, only the frame count differs.  It runs after
    the CPU-side parity checks, during which the GPU idles, so its untimed warmup is time-based
    (~settle_ms of back-to-back launches): the clock transient a streaming kernel start causes is
    then over (profiles/r05/clock_transient.txt) and the figure is the steady-state one."""
    import time as _t

    import torch

    step, cleanup = make_step(frames_alt)
    t0 = _t.perf_counter()
    n = 0
    while n < 3 or (_t.perf_counter() - t0) * 1e3 < settle_ms:
        step()
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        step()
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / steps
    cleanup()
    gbps = frames_alt * bytes_per_frame / (ms / 1e3) / 1e9
    return {"frames": frames_alt, "kernel_ms_per_launch": round(ms, 4), "ms_per_frame": round(ms / frames_alt, 6),
            "achieved": round(gbps, 1), "frac": round(gbps / HBM_PEAK_GBPS, 4), "untimed_launches": n}


BAND_SEED = 1234


def band_frame(f, sh, sw, device):
    """Source frame f of the band-mode batch: uniform random U8 from seed BAND_SEED + f, so any frame
    can be regenerated from its index alone (rank 0 regenerates the checked frames for parity)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(BAND_SEED + f)
    return torch.randint(0, 256, (sh, sw), dtype=torch.uint8, device=device, generator=g)


def band_window(frames, s0, s1, sh, sw, device):
    """Rows [s0, s1) of every band-mode frame, [frames, s1 - s0, sw] on `device`: one frame is
    generated at a time and only its window rows are kept."""
    import torch
    win = torch.empty((frames, s1 - s0, sw), dtype=torch.uint8, device=device)
    for f in range(frames):
        win[f].copy_(band_frame(f, sh, sw, device)[s0:s1])
    return win


def band_buffers(resizer, frames, sw, dw, dh, rank, world, device, band_src="device", rot=0):
    """This rank's band-mode buffers, bounded by its own shard (shard.band_plan), never by the global
    batch: `rot` device copies of its source window [frames, s1 - s0, sw] and of its output band
    [frames, r1 - r0, dw], plus -- band_src == "host" -- the window staged in (pinned) host memory
    for the timed upload.  Returns (shard, host_window or None, [device windows], [device bands])."""
    import torch

    from libiqo_amd import shard as shard_mod
    mine = shard_mod.make_shards(resizer, dh, list(range(world)))[rank]
    srows, rows = mine.s1 - mine.s0, mine.r1 - mine.r0
    bytes_launch = float(frames) * (srows * sw + rows * dw)
    rot = rot or max(2, int(-(-2.5e9 // max(bytes_launch, 1.0))))
    host = None
    if band_src == "host":
        host = band_window(frames, mine.s0, mine.s1, resizer.srcH, sw, device).cpu()
        if torch.cuda.is_available():
            host = host.pin_memory()
        wins = []
    else:
        wins = [band_window(frames, mine.s0, mine.s1, resizer.srcH, sw, device)]
    bands = [torch.empty((frames, rows, dw), dtype=torch.uint8, device=device) for _ in range(rot)]
    return mine, host, wins, bands, rot


def probe_lib():
    """libiqo_amd/libiqo_probe.so: a streaming read:write kernel (measurement only)."""
    import ctypes
    L = ctypes.CDLL(os.path.join(ROOT, "libiqo_amd", "libiqo_probe.so"))
    L.iqo_probe_stream.restype = ctypes.c_int
    L.iqo_probe_stream.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    return L


def settle_and_time(step, dev, stream, steps, settle_ms=150.0):
    """~settle_ms of back-to-back untimed launches (the GPU's post-start clock dip is over, as
    bench's auto warmup), then `steps` launches between two HIP events on the launch stream."""
    import torch
    t0 = time.perf_counter()
    n = 0
    while n < 3 or (time.perf_counter() - t0) * 1e3 < settle_ms:
        step()
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / steps, n


# read:write byte mix of each config (source : output bytes per frame), as the probe's (R, W) units
PROBE_MIX = {"c2": (4, 1), "c3": (16, 1), "c4": (1, 4)}


def stream_probe(L, mix, src, src_bytes, dst, dst_bytes, dev, stream, steps):
    """The streaming probe with the byte mix `mix` over the rotated buffers src[b] / dst[b] (the
    kernel's own), plain and nontemporal stores; the faster is the ceiling."""
    R, W = mix
    units = min(src_bytes // (1024 * R), dst_bytes // (1024 * W))
    moved = float(units) * 1024 * (R + W)
    out = {"mix_read_write": "%d:%d" % (R, W), "bytes_per_launch": int(moved)}
    sp = stream.cuda_stream
    for nt in (0, 1):
        k = [0]

        def st():
            b = k[0] % src.shape[0]
            k[0] += 1
            rc = L.iqo_probe_stream(R, W, nt, src[b].data_ptr(), src_bytes, dst[b].data_ptr(), dst_bytes, sp)
            if rc:
                raise RuntimeError("iqo_probe_stream failed (%d)" % rc)
        ms, _ = settle_and_time(st, dev, stream, steps, settle_ms=60.0)
        out["nt" if nt else "plain"] = {"ms_per_launch": round(ms, 4), "achieved": round(moved / (ms / 1e3) / 1e9, 1)}
    best = max(out["plain"]["achieved"], out["nt"]["achieved"])
    out["ceiling"] = best
    out["ceiling_frac_of_peak"] = round(best / HBM_PEAK_GBPS, 4)
    return out


def secondary_config(name, frames, dev, stream, steps, verify, probe=None, make=None):
    """One more BASELINE config timed like the headline (rotated fresh device batches, >= 3 and
    >= 2.5 GB per cycle; time-based warmup; HIP events on the launch stream), its frames 0, mid and
    last checked against the oracle, plus the streaming probe of its byte mix on the same buffers."""
    import torch

    import libiqo_amd
    m, d, sw, sh, dw, dh, px, _, label = CONFIGS[name]
    r = make(m, d, sw, sh, dw, dh, px) if make else libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px, device=dev.index)
    kernel = r.describe()["kernel"]
    bytes_launch = float(frames) * (sw * sh + dw * dh)
    rot = max(3, int(-(-2.5e9 // bytes_launch)))
    gen = torch.Generator(device=dev)
    gen.manual_seed(5678)
    src = torch.randint(0, 256, (rot, frames, sh, sw), dtype=torch.uint8, device=dev, generator=gen)
    dst = torch.empty((rot, frames, dh, dw), dtype=torch.uint8, device=dev)
    sp = stream.cuda_stream
    k = [0]

    def st():
        b = k[0] % rot
        k[0] += 1
        r.resize_device(frames, sw, sw * sh, src[b].data_ptr(), dw, dw * dh, dst[b].data_ptr(), sp)
    ms, n = settle_and_time(st, dev, stream, steps)
    gbps = bytes_launch / (ms / 1e3) / 1e9
    res = {"workload": label, "kernel": kernel, "frames": frames, "batches_cycled": rot, "steps": steps,
           "untimed_launches": n, "kernel_ms_per_launch": round(ms, 4), "algorithmic_bytes_per_launch": int(bytes_launch),
           "achieved": round(gbps, 1), "peak": HBM_PEAK_GBPS, "frac": round(gbps / HBM_PEAK_GBPS, 4),
           "value_mpix_s": round(frames * dw * dh / (ms / 1e3) / 1e6, 1)}
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_%s.json" % name)) as f:
            pmc = json.load(f)
        if pmc.get("frames") == frames and pmc.get("kernel") == kernel:
            res["traffic"] = pmc.get("hbm_bytes_per_launch")
            res["traffic_source"] = "profiles/pmc_%s.json (round %s), not measured in this run" % (name, pmc.get("round"))
    except Exception:
        pass
    if verify:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as ol
        ok = True
        for f in sorted({0, frames // 2, frames - 1}):
            exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, src[0, f].cpu().numpy())
            ok = ok and bool((dst[0, f].cpu().numpy() == exp).all())
        res["parity"] = "bit-exact vs Generic oracle (frames 0, mid, last)" if ok else "MISMATCH"
    else:
        res["parity"] = "unchecked"
    if probe is not None:
        res["stream_probe"] = stream_probe(probe, PROBE_MIX[name], src, frames * sw * sh, dst, frames * dw * dh, dev,
                                           stream, steps)
        res["frac_of_probe_ceiling"] = round(gbps / res["stream_probe"]["ceiling"], 4)
    del src, dst
    torch.cuda.empty_cache()
    return res


def spawn_ranks(n):
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE in the environment): start N
    rank processes of this same command line, one per GPU, as torch.distributed.run would (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free MASTER_PORT), wait for them and return
    the worst exit status.  This process never touches the GPU (no torch import): the ranks are
    fresh children, not an exec of an initialised process.  Rank 0 prints the JSON line."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def spawn_probe():
    """--spawn-probe: the rank plumbing of spawn_ranks without a GPU (CPU test): every rank joins a
    gloo group, all-reduces its rank, and rank 0 prints one JSON line."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([float(dist.get_rank())])
    dist.all_reduce(t)
    got = [None] * dist.get_world_size()
    dist.all_gather_object(got, {"rank": dist.get_rank(), "local_rank": int(os.environ["LOCAL_RANK"])})
    if dist.get_rank() == 0:
        print(json.dumps({"world_size": dist.get_world_size(), "rank_sum": t.item(), "ranks": got}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=-1,
                    help="untimed warmup steps (default -1: enough steps for >= 150 ms of launches, at least 10, so "
                         "the timed steps run after the GPU's post-start clock dip, profiles/r05/clock_transient.txt)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--frames", type=int, default=0, help="frames per GPU (band mode: global frames; 0 = default)")
    ap.add_argument("--shard", default="image", choices=["image", "band"])
    ap.add_argument("--band-src", default="device", choices=["device", "host"],
                    help="band mode: each rank's source window generated on its device, or staged in pinned host "
                         "memory and uploaded (timed as scatter_ms)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the C3 / C4 lines and the streaming probes the default C2 run carries at N = 1")
    ap.add_argument("--bands", type=int, default=0, help="row bands per frame inside a launch (0 = auto)")
    ap.add_argument("--cpu-seconds", type=float, default=16.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-probe", action="store_true", help="skip the same-batch reuse probe (N=1)")
    ap.add_argument("--rotate", type=int, default=0,
                    help="distinct device batches cycled through, one per step (0 = auto: >= 3 batches and >= 2.5 GB "
                         "per cycle, 10x the Infinity Cache, so no step re-reads the previous steps' data from it)")
    ap.add_argument("--alt-frames", type=int, default=-1,
                    help="also time this many frames per launch (rotated batches; -1 = 256 for c2, 0 = off)")
    ap.add_argument("--force-general", action="store_true")
    ap.add_argument("--option", action="append", default=[], metavar="KEY=VALUE",
                    help="plan option (iqo_hip_plan_set_option), repeatable; speed-only A/B knobs")
    ap.add_argument("--spawn-probe", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.option:
        os.environ["IQO_HIP_TUNING"] = "1"  # the A/B option keys (include/iqo_hip.h iqo_hip_plan_set_option)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    if args.spawn_probe:
        spawn_probe()
        return

    import torch

    import libiqo_amd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("warning: --gpus %d but WORLD_SIZE %d (launched by torch.distributed.run); using WORLD_SIZE" %
            (args.gpus, world))
    dist = None
    # IQO_BENCH_DIST=gloo rehearses the N>1 image-shard path with several ranks per GPU (rank r uses
    # device r % device_count, control collectives over gloo); the real multi-GPU run uses RCCL
    backend = os.environ.get("IQO_BENCH_DIST", "nccl")
    gpu = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        # control only: barriers and the MAX of the timings (band mode: the IPC handles); never pixels
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)

    cfg = CONFIGS[args.config]
    m, d, sw, sh, dw, dh, px, default_frames, label = cfg
    frames = args.frames or default_frames

    def make(device):
        r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px, device=device)
        if args.bands:
            r.set_option("bands", args.bands)
        if args.force_general:
            r.set_option("force_general", 1)
        for kv in args.option:
            k, v = kv.split("=", 1)
            r.set_option(k, int(v))
        return r

    r = make(gpu)
    kernel = r.describe()["kernel"]
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    band_info = None
    if args.shard == "image":
        gen = torch.Generator(device=dev)
        gen.manual_seed(1234 + rank)
        bytes_launch = float(frames) * (sw * sh + dw * dh)
        out_px_step = float(frames) * dw * dh * world
        # every step resizes a batch the previous steps did not touch: the batches cycle with at
        # least 2.5 GB between two uses of one batch (a repeated launch over the same batch gets
        # part of its reads from the 256 MiB Infinity Cache; real pipelines bring new frames).  At
        # least 3 batches: a launch's time depends on where in HBM its batch landed (C2 x1024: 1.81
        # to 1.91 ms from one batch to the next), and 2 large batches sampled fewer placements
        # (the driver's command: 0.701-0.703 with 2, 0.712-0.714 with 3, alternated on one box,
        # profiles/r05/rotate_placement.txt)
        rot = args.rotate or max(3, int(-(-2.5e9 // bytes_launch)))
        src = torch.randint(0, 256, (rot, frames, sh, sw), dtype=torch.uint8, device=dev, generator=gen)
        dst = torch.empty((rot, frames, dh, dw), dtype=torch.uint8, device=dev)
        nstep = [0]

        def step_batch(b):
            r.resize_device(frames, sw, sw * sh, src[b].data_ptr(), dw, dw * dh, dst[b].data_ptr(), sp)

        def step():
            step_batch(nstep[0] % rot)
            nstep[0] += 1
    else:
        from libiqo_amd import shard
        # this rank's source window only (never the global batch): generated on its device from the
        # per-frame seeds, or (--band-src host) staged in pinned host memory and uploaded, timed
        out = torch.zeros((frames, dh, dw), dtype=torch.uint8, device=dev) if rank == 0 else None
        mine, host_win, wins, bands_out, rot = band_buffers(r, frames, sw, dw, dh, rank, world, dev, args.band_src,
                                                            args.rotate)
        mine = mine._replace(device=gpu)
        # every rank's shard (rows and windows; only their indices and rank 0's own device matter to
        # the gather, which moves the other bands by IPC handle)
        shards = [mine if s.index == rank else s for s in shard.make_shards(r, dh, list(range(world)))]
        t_sc = 0.0
        be = shard.HipBandBackend(lambda device: r if device == mine.device else make(device),
                                  host_win if host_win is not None else wins[0], -1 if host_win is not None else gpu,
                                  out, gpu, src_row0=mine.s0)
        if host_win is not None:
            torch.cuda.synchronize(dev)
            t_sc = time.perf_counter()
            wins.append(be.scatter(mine))
            torch.cuda.synchronize(dev)
            t_sc = time.perf_counter() - t_sc
        else:
            be.paths["scatter"] = {"window generated on the rank's device (per-frame seeds): no upload"}
        rows, srows = mine.r1 - mine.r0, mine.s1 - mine.s0
        bytes_launch = float(frames) * (srows * sw + rows * dw)
        out_px_step = float(frames) * dw * dh  # the whole frame, all ranks together
        # like image mode, steps cycle through distinct copies of the window (>= 2.5 GB per cycle)
        # so no step re-reads its input from the Infinity Cache; copy 0 is the generated / uploaded one
        wins += [wins[0].clone() for _ in range(rot - 1)]
        nstep = [0]

        def step():
            b = nstep[0] % rot
            nstep[0] += 1
            r.resize_band(frames, mine.r0, rows, mine.s0, sw, wins[b].stride(0), wins[b].data_ptr(), dw,
                          bands_out[b].stride(0), bands_out[b].data_ptr(), sp)

    if args.warmup < 0:
        # auto warmup: a cold step, then 3 timed ones size it (>= 150 ms of back-to-back launches,
        # >= 10 steps; the 4 sizing steps are not counted)
        step()
        torch.cuda.synchronize(dev)
        ew0, ew1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ew0.record(stream)
        for _ in range(3):
            step()
        ew1.record(stream)
        torch.cuda.synchronize(dev)
        args.warmup = int(min(5000, max(10, -(-150.0 // max(ew0.elapsed_time(ew1) / 3, 1e-3)))))
    log("rank %d/%d %s shard=%s frames=%d kernel=%s warmup=%d steps=%d" % (rank, world, label, args.shard, frames,
                                                                        kernel, args.warmup, args.steps))
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # events on the stream the kernels run on

    t = torch.tensor([wall, t_sc if args.shard == "band" else 0.0, kern_ms], dtype=torch.float64,
                     device="cpu" if backend == "gloo" else dev)
    rank_kern = [kern_ms]
    pg_world = 1
    if dist:
        # timing bookkeeping only, not the data path: every rank's kernel ms, then the MAX
        allk = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allk, t)
        rank_kern = [float(x[2].item()) for x in allk]
        pg_world = dist.get_world_size()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    # the slowest rank's wall time and the slowest rank's kernel time
    wall_max, scatter_max, kern_ms = float(t[0].item()), float(t[1].item()), float(t[2].item())

    if args.shard == "band":
        # gather the bands to rank 0 (IPC handle + device copy), timed on its own
        be.sync()
        if dist:
            dist.barrier()
        t_g = time.perf_counter()
        last = bands_out[(nstep[0] - 1) % rot]  # the band of the last timed step
        if dist:
            be.gather_distributed(shards, last, rank, world, dist)
        else:
            be.gather(mine, last)
        be.sync()
        if dist:
            dist.barrier()
        t_g = time.perf_counter() - t_g
        band_info = {"ranks": world, "rows_per_rank": rows, "src_window_rows": srows, "band_src": args.band_src,
                     "rank_device_bytes": int(rot * frames * (srows * sw + rows * dw)),
                     "rank_host_bytes": int(host_win.numel()) if host_win is not None else 0,
                     "scatter_ms": round(scatter_max * 1e3, 3), "gather_ms": round(t_g * 1e3, 3),
                     "scatter_path": sorted(be.paths.get("scatter", [])), "gather_path": sorted(be.paths.get("gather", []))}

    parity = "unchecked"
    if rank == 0 and not args.no_verify:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as ol
        ok = True
        for f in sorted({0, frames // 2, frames - 1}):
            if args.shard == "image":
                s_np, o_np = src[0, f].cpu().numpy(), dst[0, f].cpu().numpy()
            else:  # rank 0 regenerates the whole source frame from its seed
                s_np, o_np = band_frame(f, sh, sw, dev).cpu().numpy(), out[f].cpu().numpy()
            exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, s_np)
            ok = ok and bool((o_np == exp).all())
        parity = ("bit-exact vs Generic oracle (frames 0, mid, last%s)" %
                  (", gathered from %d band shards" % world if args.shard == "band" else "")) if ok else "MISMATCH"
        log("parity: " + parity)

    probe = None
    if rank == 0 and world == 1 and args.shard == "image" and not args.no_probe:
        probe = reuse_probe(step_batch, rot, dev)
        log("reuse probe: %s" % json.dumps(probe))

    alt = None
    alt_frames = args.alt_frames if args.alt_frames >= 0 else (256 if args.config == "c2" else 0)
    if args.shard == "image" and alt_frames and alt_frames != frames:
        del src, dst
        torch.cuda.empty_cache()

        def make_alt(n):
            rot_a = max(2, int(-(-2.5e9 // (n * (sw * sh + dw * dh)))))
            g2 = torch.Generator(device=dev)
            g2.manual_seed(4321 + rank)
            sa = torch.randint(0, 256, (rot_a, n, sh, sw), dtype=torch.uint8, device=dev, generator=g2)
            da = torch.empty((rot_a, n, dh, dw), dtype=torch.uint8, device=dev)
            k = [0]

            def st():
                b = k[0] % rot_a
                k[0] += 1
                r.resize_device(n, sw, sw * sh, sa[b].data_ptr(), dw, dw * dh, da[b].data_ptr(), sp)

            def cleanup():
                # bit-exact spot check of the alt batch too (frames 0, mid, last of batch 0)
                if rank == 0 and not args.no_verify:
                    sys.path.insert(0, os.path.join(ROOT, "tests"))
                    import oracle_lib as ol
                    for f in sorted({0, n // 2, n - 1}):
                        exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, sa[0, f].cpu().numpy())
                        if not bool((da[0, f].cpu().numpy() == exp).all()):
                            raise SystemExit("alt batch MISMATCH at frame %d" % f)
            return st, cleanup

        alt = alt_batch(make_alt, alt_frames, sw * sh + dw * dh, dev)
        log("alt batch: %s" % json.dumps(alt))

    secondary = None
    if rank == 0 and world == 1 and args.shard == "image" and args.config == "c2" and not args.no_secondary:
        # C3 / C4 in the same run (the driver's record), after the headline and before the CPU leg
        if "src" in locals():
            del src, dst
        torch.cuda.empty_cache()
        secondary = {}
        try:
            pl = probe_lib()
        except OSError as e:
            pl = None
            secondary["probe_error"] = str(e)
        n_sec = max(20, min(args.steps, 50))
        for name, nf in (("c3", 64), ("c4", 256)):
            secondary[name] = secondary_config(name, nf, dev, stream, n_sec, not args.no_verify, pl, make=None)
            log("secondary %s: %s" % (name, json.dumps(secondary[name])))
            if secondary[name]["parity"] == "MISMATCH":
                raise SystemExit("secondary %s MISMATCH" % name)
        if pl is not None:
            # the headline's own byte mix on fresh buffers of its size (C2 x frames)
            g3 = torch.Generator(device=dev)
            g3.manual_seed(91)
            ps = torch.randint(0, 256, (3, frames * sh * sw), dtype=torch.uint8, device=dev, generator=g3)
            pd = torch.empty((3, frames * dh * dw), dtype=torch.uint8, device=dev)
            secondary["c2_stream_probe"] = stream_probe(pl, PROBE_MIX["c2"], ps, frames * sw * sh, pd, frames * dw * dh,
                                                        dev, stream, n_sec)
            del ps, pd
            torch.cuda.empty_cache()

    cpu = None
    ref_bench = None
    if rank == 0 and world == 1 and not args.no_cpu:
        log("cpu baseline: ~%.0f s" % args.cpu_seconds)
        cpu = cpu_baseline(cfg, args.cpu_seconds)
        if args.config in ("c1", "c2", "c3", "c4"):
            ref_bench = reference_benchmark(cfg)

    if rank == 0:
        value = out_px_step * args.steps / wall_max / 1e6
        achieved = bytes_launch / (kern_ms / 1e3) / 1e9
        traffic, traffic_src = None, None
        try:
            with open(os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)) as f:
                pmc = json.load(f)
            if pmc.get("frames") == frames and pmc.get("kernel") == kernel and args.shard == "image":
                traffic = pmc.get("hbm_bytes_per_launch")
                traffic_src = ("profiles/pmc_%s.json: rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench command "
                               "(scripts/gpu_ci.sh pmc, round %s), not measured in this run" % (args.config, pmc.get("round")))
        except Exception:
            pass
        par = ("image-sharded x%d (independent shards, no collective)" % world if args.shard == "image" else
               "row-band-sharded x%d (halo windows in, bands gathered by IPC + device copy; no collective)" % world)
        res = {
            "metric": baseline_metric() if args.config == "c2" else "Mpix/s " + label,
            "value": round(value, 1),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak" if args.shard == "image" else "strong",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: uniform random U8 frames (torch.randint, seed %s)" %
                    ("1234+rank, on device; %d distinct batches cycled, one per step" % rot if args.shard == "image"
                     else "%d + frame index; each rank generates only its source window (%s)" %
                     (BAND_SEED, "on device" if args.band_src == "device" else "staged in pinned host memory, uploaded")),
            "config": {"workload": label, "frames_per_gpu": frames if args.shard == "image" else None,
                       "global_frames": frames * world if args.shard == "image" else frames,
                       "parallelism": par, "kernel": kernel, "bands_per_frame": args.bands or "auto",
                       "step": "one libiqo_hip launch over the rank's %s" %
                               ("device-resident batch" if args.shard == "image" else "row band of every frame")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "traffic_source": traffic_src, "kernel_ms_per_launch": round(kern_ms, 4),
                         "algorithmic_bytes_per_launch": int(bytes_launch)},
            "cpu_baseline": cpu,
            "parity": parity,
        }
        if dist:
            res["ranks"] = {"process_group_world_size": pg_world, "backend": backend,
                            "kernel_ms_per_launch_min": round(min(rank_kern), 4),
                            "kernel_ms_per_launch_max": round(max(rank_kern), 4),
                            "devices": "one GPU per rank" if backend != "gloo" else
                                       "rank r on device r %% %d (gloo rehearsal)" % torch.cuda.device_count()}
        if band_info:
            res["band"] = band_info
        if alt:
            res["config"]["frames_per_gpu_alt"] = alt["frames"]
            res["batch_alt"] = alt
        if probe:
            res["reuse_probe"] = probe
        if secondary:
            res["secondary"] = secondary
            cp = secondary.get("c2_stream_probe")
            if cp:
                res["roofline"]["stream_probe_ceiling"] = cp["ceiling"]
                res["roofline"]["frac_of_probe_ceiling"] = round(achieved / cp["ceiling"], 4)
        if ref_bench:
            res["reference_benchmark"] = ref_bench
        if cpu and cpu.get("value"):
            res["gpu_over_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(res), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
