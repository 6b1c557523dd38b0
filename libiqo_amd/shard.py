"""Multi-GPU sharding of the resize hot path: no data-path collective.

Two decompositions:

* by image -- a batch of F frames is split into contiguous frame ranges, one per rank (bench.py's
  default, weak scaling);
* by output-row band -- every frame's output rows are split into contiguous bands; a band needs
  only the source rows it reads (its halo window, `iqo_hip_band_src_rows`).  Rows keep their
  global indices, so the stitched bands equal the unsharded result byte for byte.  This is the
  GPU form of the reference's OpenMP row split (src/IQOLanczosResizerImpl_AVX512.cpp:269-308).

The band orchestration is written once, against a small backend interface, and driven two ways:

* `run_bands_local(backend, shards)` -- one process, one shard per device of a list (repeats
  allowed: two bands on device 0 run the whole path on a one-GPU box);
* `run_bands_distributed(backend, shards, rank, world, dist)` -- one process per GPU
  (torch.distributed ranks): rank r runs shard r, the bands are gathered to rank 0.

Each drive has three timed phases -- scatter (source windows to the shard devices), compute,
gather (bands to the root's output) -- so compute scaling is reported apart from data movement.

Backend interface (duck-typed; `HipBandBackend` below is the GPU one, the CPU tests pass a numpy
stub with the same methods):

    scatter(shard)                -> window   (the shard's source rows [s0, s1) of every frame)
    compute(shard, window)        -> band     (output rows [r0, r1) of every frame)
    gather(shard, band)                       (local drive: into the root's output)
    gather_distributed(shards, band, rank, world, dist)   (distributed drive)
    sync(shard=None)                          (wait for the shard's / every device's work)
"""
import time
from collections import namedtuple

Shard = namedtuple("Shard", "index device r0 r1 s0 s1")


def frame_range(n_frames, rank, world):
    """Contiguous frame range [f0, f1) of `rank` (balanced, remainder spread over low ranks)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, rem = divmod(n_frames, world)
    f0 = rank * base + min(rank, rem)
    return f0, f0 + base + (1 if rank < rem else 0)


def row_band(dst_h, rank, world):
    """Contiguous output-row band [r0, r1) of `rank`."""
    return frame_range(dst_h, rank, world)


def band_plan(resizer_or_fn, dst_h, world):
    """For each rank: (r0, r1, s0, s1) = output band and the source-row window it reads.

    `resizer_or_fn` is a libiqo_amd resizer (uses its band_src_rows) or a callable
    (r0, nrows) -> (s0, nsrc)."""
    fn = getattr(resizer_or_fn, "band_src_rows", resizer_or_fn)
    plan = []
    for rank in range(world):
        r0, r1 = row_band(dst_h, rank, world)
        if r1 > r0:
            s0, ns = fn(r0, r1 - r0)
        else:
            s0, ns = 0, 0
        plan.append((r0, r1, s0, s0 + ns))
    return plan


def make_shards(resizer_or_fn, dst_h, devices):
    """One Shard per entry of `devices` (device ids may repeat)."""
    return [Shard(i, d, *b) for i, (d, b) in enumerate(zip(devices, band_plan(resizer_or_fn, dst_h, len(devices))))]


def halo_overhead(plan, src_h):
    """Extra source rows read because of band halos, as a fraction of the frame."""
    return (sum(p[-1] - p[-2] for p in plan) - src_h) / float(src_h)


def run_bands_local(backend, shards, clock=time.perf_counter):
    """One process: scatter every window, compute every band, gather every band (each phase
    timed after a full sync).  Returns {"scatter_s", "compute_s", "gather_s"}."""
    backend.sync()
    t0 = clock()
    windows = [backend.scatter(sh) for sh in shards]
    backend.sync()
    t1 = clock()
    bands = [backend.compute(sh, w) for sh, w in zip(shards, windows)]
    backend.sync()
    t2 = clock()
    for sh, b in zip(shards, bands):
        backend.gather(sh, b)
    backend.sync()
    t3 = clock()
    return {"scatter_s": t1 - t0, "compute_s": t2 - t1, "gather_s": t3 - t2}


def run_bands_distributed(backend, shards, rank, world, dist, clock=time.perf_counter):
    """One process per GPU: rank r runs shards[r]; phases are fenced by barriers, so each time
    is the slowest rank's.  Returns the phase times (same on every rank) and this rank's band."""
    if len(shards) != world:
        raise ValueError("one shard per rank")
    sh = shards[rank]
    backend.sync()
    dist.barrier()
    t0 = clock()
    window = backend.scatter(sh)
    backend.sync(sh)
    dist.barrier()
    t1 = clock()
    band = backend.compute(sh, window)
    backend.sync(sh)
    dist.barrier()
    t2 = clock()
    backend.gather_distributed(shards, band, rank, world, dist)
    backend.sync()
    dist.barrier()
    t3 = clock()
    return {"scatter_s": t1 - t0, "compute_s": t2 - t1, "gather_s": t3 - t2}, band


CopyOp = namedtuple("CopyOp", "dst dst_st src src_st nbytes count")


def gather_ops(sh, src, src_fst, src_pitch, frames, dst, dst_fst, dst_pitch, width):
    """Copy operations that move shard `sh`'s band into the root output.

    The band holds output rows [r0, r1) of every frame at its OWN frame stride `src_fst` and row
    pitch `src_pitch`; the output holds whole frames at `dst_fst` / `dst_pitch`.  Each CopyOp is
    `count` blocks of `nbytes` (block k at dst + k*dst_st and src + k*src_st), the shape of
    iqo_hip_copy_frames.  Equal pitches: one op, a band-sized block per frame.  Different
    pitches: one op per frame, a `width`-byte block per row."""
    rows = sh.r1 - sh.r0
    if rows <= 0 or frames <= 0:
        return []
    if src_pitch == dst_pitch:
        return [CopyOp(dst + sh.r0 * dst_pitch, dst_fst, src, src_fst, (rows - 1) * dst_pitch + width, frames)]
    return [CopyOp(dst + f * dst_fst + sh.r0 * dst_pitch, dst_pitch, src + f * src_fst, src_pitch, width, rows)
            for f in range(frames)]


class HipBandBackend:
    """Row-band shards on gfx950 devices through the C ABI.

    `src` holds the source batch (uint8 torch tensor [F, rows, srcSt]: source rows [src_row0,
    src_row0 + rows) of every frame -- the whole frame, or only the windows this process scatters)
    on device `src_device`, or in (pinned) host memory when src_device < 0; `out` [F, dstH, dstSt] is the
    output batch on `out_device` (the root; in the distributed drive only rank 0 needs it).
    Each shard gets its window by iqo_hip_copy_frames (peer DMA over xGMI, or H2D), runs
    iqo_hip_resize_band on its device's current stream, and its band goes back by
    iqo_hip_copy_frames (local drive) or by IPC handle + peer copy (distributed drive)."""

    def __init__(self, make_resizer, src, src_device, out, out_device, src_row0=0):
        import torch

        self.torch = torch
        self.src, self.src_device, self.src_row0 = src, src_device, src_row0
        self.out, self.root = out, out_device
        self.frames = src.shape[0]
        self.src_st, self.src_fst = src.stride(1), src.stride(0)
        self.dst_st = out.stride(1) if out is not None else None
        self.dst_fst = out.stride(0) if out is not None else None
        self._make = make_resizer
        self._resizers = {}
        self.paths = {}  # phase -> set of copy routes taken

    def _dev(self, d):
        return self.torch.device("cuda", d)

    def resizer(self, device):
        if device not in self._resizers:
            self._resizers[device] = self._make(device)
        return self._resizers[device]

    def _route(self, phase, p):
        from . import COPY_PATHS

        self.paths.setdefault(phase, set()).add(COPY_PATHS.get(p, p))

    def scatter(self, sh):
        from . import copy_frames

        rows = sh.s1 - sh.s0
        if sh.s0 < self.src_row0 or sh.s1 > self.src_row0 + self.src.shape[1]:
            raise ValueError("shard window rows [%d, %d) outside the source rows held [%d, %d)" %
                             (sh.s0, sh.s1, self.src_row0, self.src_row0 + self.src.shape[1]))
        win = self.torch.empty((self.frames, rows, self.src_st), dtype=self.torch.uint8, device=self._dev(sh.device))
        stream = self.torch.cuda.current_stream(self._dev(sh.device))
        base = self.src.data_ptr() + (sh.s0 - self.src_row0) * self.src_st
        p = copy_frames(win.data_ptr(), sh.device, win.stride(0), base, self.src_device, self.src_fst,
                        rows * self.src_st, self.frames, stream)
        self._route("scatter", p)
        return win

    def compute(self, sh, win):
        r = self.resizer(sh.device)
        rows = sh.r1 - sh.r0
        st = self.dst_st or r.dstW
        band = self.torch.empty((self.frames, rows, st), dtype=self.torch.uint8, device=self._dev(sh.device))
        stream = self.torch.cuda.current_stream(self._dev(sh.device))
        r.resize_band(self.frames, sh.r0, rows, sh.s0, self.src_st, win.stride(0), win.data_ptr(), st, band.stride(0),
                      band.data_ptr(), stream)
        return band

    def gather(self, sh, band):
        from . import copy_frames

        stream = self.torch.cuda.current_stream(self._dev(self.root))
        for op in gather_ops(sh, band.data_ptr(), band.stride(0), band.stride(1), self.frames, self.out.data_ptr(),
                             self.dst_fst, self.dst_st, self.out.shape[2]):
            p = copy_frames(op.dst, self.root, op.dst_st, op.src, sh.device, op.src_st, op.nbytes, op.count, stream)
            self._route("gather", p)

    def gather_distributed(self, shards, band, rank, world, dist):
        """Every rank exports its band's IPC handle together with the band's frame stride and row
        pitch (the handles travel over the control group, the pixels never do); rank 0 opens each
        and pulls it by peer copy into `out`, with THAT band's strides: bands are uneven when
        world does not divide dstH, and a rank without `out` allocates its band at pitch dstW."""
        from . import copy_frames, ipc_close, ipc_export, ipc_open

        mine = (ipc_export(band.data_ptr()), band.stride(0), band.stride(1))
        metas = [None] * world
        dist.all_gather_object(metas, mine)
        if rank == 0:
            stream = self.torch.cuda.current_stream(self._dev(self.root))
            for sh in shards:
                handle, fst, pitch = metas[sh.index]
                if sh.index == 0:
                    src, h = band.data_ptr(), None
                else:
                    src, h = ipc_open(handle, self.root)
                for op in gather_ops(sh, src, fst, pitch, self.frames, self.out.data_ptr(), self.dst_fst, self.dst_st,
                                     self.out.shape[2]):
                    p = copy_frames(op.dst, self.root, op.dst_st, op.src, self.root if h is not None else sh.device,
                                    op.src_st, op.nbytes, op.count, stream)
                    self._route("gather", p if h is None else "IPC-mapped peer buffer, copied by the root's DMA")
                if h is not None:
                    self.torch.cuda.synchronize(self._dev(self.root))
                    ipc_close(src, h)
        dist.barrier()  # every band buffer stays alive until rank 0 has copied it

    def sync(self, sh=None):
        devs = (({self.root} if self.root is not None and self.root >= 0 else set()) | set(self._resizers)
                if sh is None else {sh.device})
        for d in devs:
            self.torch.cuda.synchronize(self._dev(d))
