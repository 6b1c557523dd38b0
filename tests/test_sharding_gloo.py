"""Multi-GPU decomposition on CPU: libiqo_amd/shard.py's orchestration driven by 2 gloo ranks (and
by one process with several shards) with a numpy stub backend -- no GPU.

The stub computes a band from its window ONLY (rows outside the window are replaced by noise
before the CPU oracle runs), so a wrong halo plan, a wrong scatter or a wrong gather fails
here.  tests/test_gpu_parity.py drives the same orchestration with HipBandBackend on the GPU."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import libiqo_amd
import oracle_lib as ol
from libiqo_amd import shard

CASES = [("lanczos", 3, 96, 64, 48, 32, 1), ("area", 0, 64, 48, 16, 12, 1), ("linear", 0, 40, 30, 80, 60, 1),
         ("lanczos", 2, 77, 51, 140, 90, 1)]


class StubBackend:
    """numpy backend with HipBandBackend's interface; compute = the oracle on the window alone."""

    def __init__(self, case, src):
        self.case, self.src = case, src
        m, d, sw, sh, dw, dh, px = case
        self.out = np.zeros((src.shape[0], dh, dw), np.uint8)
        self.calls = []

    def scatter(self, sh):
        self.calls.append(("scatter", sh.index))
        return self.src[:, sh.s0:sh.s1].copy()

    def compute(self, sh, win):
        m, d, sw, srch, dw, dh, px = self.case
        self.calls.append(("compute", sh.index))
        band = np.zeros((win.shape[0], sh.r1 - sh.r0, dw), np.uint8)
        for f in range(win.shape[0]):
            full = ol.gen("noise", sw, srch, 7777 + 31 * sh.index + f)  # garbage outside the window
            full[sh.s0:sh.s1] = win[f]
            band[f] = ol.run_oracle(m, d, sw, srch, dw, dh, px, full)[sh.r0:sh.r1]
        return band

    def gather(self, sh, band):
        self.calls.append(("gather", sh.index))
        self.out[:, sh.r0:sh.r1] = band

    def gather_distributed(self, shards, band, rank, world, d):
        got = [None] * world
        d.all_gather_object(got, (rank, band))
        if rank == 0:
            for r, b in got:
                sh = shards[r]
                self.out[:, sh.r0:sh.r1] = b

    def sync(self, sh=None):
        pass


def _frames(ci, sw, sh, n=3):
    return np.stack([ol.gen("noise", sw, sh, 100 * ci + f) for f in range(n)])


def _band_fn(case):
    m, d, sw, sh, dw, dh, px = case
    return lambda r0, n: libiqo_amd.host_band_src_rows(m, d, sw, sh, dw, dh, px, r0, n)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ok = True
        for ci, case in enumerate(CASES):
            m, d, sw, sh, dw, dh, px = case
            frames = _frames(ci, sw, sh, 5)
            ref = np.stack([ol.run_oracle(m, d, sw, sh, dw, dh, px, fr) for fr in frames])
            # --- image sharding: each rank resizes its own frame range, rank 0 collects
            f0, f1 = shard.frame_range(frames.shape[0], rank, world)
            mine = [ol.run_oracle(m, d, sw, sh, dw, dh, px, frames[f]) for f in range(f0, f1)]
            got = [None] * world
            dist.all_gather_object(got, (f0, mine))
            full = np.stack([fr for _, part in sorted(got, key=lambda t: t[0]) for fr in part])
            ok = ok and bool((full == ref).all())
            # --- row-band sharding through the orchestrator (rank r runs band r, gather to rank 0)
            shards = shard.make_shards(_band_fn(case), dh, list(range(world)))
            be = StubBackend(case, frames)
            times, band = shard.run_bands_distributed(be, shards, rank, world, dist)
            ok = ok and set(times) == {"scatter_s", "compute_s", "gather_s"}
            ok = ok and bool((band == ref[:, shards[rank].r0:shards[rank].r1]).all())
            if rank == 0:
                ok = ok and bool((be.out == ref).all())
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_two_rank_image_and_band_sharding(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert results == {r: True for r in range(world)}


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 1, 0], [0, 1, 2, 3]])
def test_local_band_orchestration_matches_unsharded(devices):
    """One process, shards on a device list (repeats allowed: the 1-GPU box runs [0, 0])."""
    for ci, case in enumerate(CASES):
        m, d, sw, sh, dw, dh, px = case
        frames = _frames(ci, sw, sh)
        shards = shard.make_shards(_band_fn(case), dh, devices)
        assert [s.device for s in shards] == devices
        be = StubBackend(case, frames)
        times = shard.run_bands_local(be, shards)
        assert set(times) == {"scatter_s", "compute_s", "gather_s"}
        ref = np.stack([ol.run_oracle(m, d, sw, sh, dw, dh, px, fr) for fr in frames])
        assert (be.out == ref).all(), (case, devices)
        # phases in order: every window out before any compute, every compute before any gather
        kinds = [c[0] for c in be.calls]
        n = len(devices)
        assert kinds == ["scatter"] * n + ["compute"] * n + ["gather"] * n


def test_band_plan_covers_frame_and_halo_is_small():
    plan = shard.band_plan(lambda r0, n: libiqo_amd.host_band_src_rows("lanczos", 3, 3840, 2160, 1920, 1080, 1, r0, n),
                           1080, 8)
    assert plan[0][0] == 0 and plan[-1][1] == 1080
    assert all(a[1] == b[0] for a, b in zip(plan, plan[1:]))
    # Lanczos-3 2:1: 5 rows above + 6 below per cut -> ~10 rows per internal cut
    assert 0 < shard.halo_overhead(plan, 2160) < 0.04
    assert shard.frame_range(1024, 7, 8) == (896, 1024)
    assert [shard.frame_range(10, r, 4) for r in range(4)] == [(0, 3), (3, 6), (6, 8), (8, 10)]
    shards = shard.make_shards(lambda r0, n: (r0, n), 10, [3, 5])
    assert shards == [shard.Shard(0, 3, 0, 5, 0, 5), shard.Shard(1, 5, 5, 10, 5, 10)]


def _apply(ops, dst_buf, src_buf, src_base):
    """Byte-level emulation of iqo_hip_copy_frames for gather_ops (addresses are offsets)."""
    for op in ops:
        for k in range(op.count):
            d, s = op.dst + k * op.dst_st, op.src - src_base + k * op.src_st
            dst_buf[d:d + op.nbytes] = src_buf[s:s + op.nbytes]


@pytest.mark.parametrize("world,dh,root_pad", [(3, 31, 5), (3, 1081, 0), (7, 64, 3), (2, 60, 0)])
def test_gather_ops_uneven_bands_and_padded_root(world, dh, root_pad):
    """bands are uneven when world does not divide dstH and non-root ranks
    allocate their bands at pitch dstW, so the root must copy each band with that band's own frame
    stride and row pitch (HipBandBackend.gather / gather_distributed use gather_ops)."""
    frames, dw = 3, 24
    dst_pitch = dw + root_pad
    ref = np.random.default_rng(dh).integers(0, 256, (frames, dh, dw), dtype=np.uint8)
    out = np.zeros((frames, dh, dst_pitch), np.uint8)
    shards = shard.make_shards(lambda r0, n: (r0, n), dh, list(range(world)))
    assert len({s.r1 - s.r0 for s in shards}) == (1 if dh % world == 0 else 2)
    flat = out.reshape(-1)
    for sh in shards:
        rows = sh.r1 - sh.r0
        pitch = dst_pitch if sh.index == 0 else dw  # compute(): the root uses out's pitch, others dstW
        band = np.zeros((frames, rows, pitch), np.uint8)
        band[:, :, :dw] = ref[:, sh.r0:sh.r1]
        base = 1 << 20  # the band's "address"
        ops = shard.gather_ops(sh, base, rows * pitch, pitch, frames, 0, dh * dst_pitch, dst_pitch, dw)
        _apply(ops, flat, band.reshape(-1), base)
        for op in ops:  # every op stays inside the band and inside the output
            assert op.src - base + (op.count - 1) * op.src_st + op.nbytes <= band.size
            assert op.dst + (op.count - 1) * op.dst_st + op.nbytes <= out.size
    assert (out[:, :, :dw] == ref).all()
    assert (out[:, :, dw:] == 0).all()  # padding never written


@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_one_rank_per_gpu(n):
    """`python bench.py --gpus N` without a launcher starts N rank processes itself (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 per rank, bench.spawn_ranks) -- the path the
    driver's multi-GPU command takes when it does not go through torch.distributed.run.  The hidden
    --spawn-probe mode runs the same spawn and rendezvous with a gloo group and no GPU."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(n), "--spawn-probe"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["world_size"] == n and d["rank_sum"] == n * (n - 1) / 2
    assert sorted(x["local_rank"] for x in d["ranks"]) == list(range(n))


class _HostBandResizer:
    """Stand-in for a libiqo_amd resizer in bench.band_buffers: srcH and the host band window
    (iqo_hip_band_src_rows' host twin), no device."""

    def __init__(self, case):
        self.m, self.d, self.srcW, self.srcH, self.dstW, self.dstH, self.px = case

    def band_src_rows(self, r0, n):
        return libiqo_amd.host_band_src_rows(self.m, self.d, self.srcW, self.srcH, self.dstW, self.dstH, self.px, r0, n)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bench_band_buffers_are_bounded_by_the_rank_window(world):
    """in --shard band every rank held the whole global batch (pageable and
    pinned).  bench.band_buffers allocates only the rank's own source window (shard.band_plan) and
    its band, and the window's rows equal the same rows of the per-frame-seeded global frames."""
    import torch

    import bench
    case = ("lanczos", 3, 384, 216, 192, 108, 1)
    rz = _HostBandResizer(case)
    frames, rot = 5, 2
    plan = shard.band_plan(rz, rz.dstH, world)
    for rank in range(world):
        r0, r1, s0, s1 = plan[rank]
        for src_kind in ("device", "host"):
            mine, host, wins, bands, got_rot = bench.band_buffers(rz, frames, rz.srcW, rz.dstW, rz.dstH, rank, world,
                                                                  "cpu", src_kind, rot)
            assert (mine.r0, mine.r1, mine.s0, mine.s1) == (r0, r1, s0, s1) and got_rot == rot
            win = host if src_kind == "host" else wins[0]
            assert tuple(win.shape) == (frames, s1 - s0, rz.srcW)  # the window, not [frames, srcH, srcW]
            assert (len(wins), host is None) == ((0, False) if src_kind == "host" else (1, True))
            assert len(bands) == rot and all(tuple(b.shape) == (frames, r1 - r0, rz.dstW) for b in bands)
            window_bytes = frames * ((s1 - s0) * rz.srcW + (r1 - r0) * rz.dstW)
            held = sum(t.numel() for t in wins + bands) + (host.numel() if host is not None else 0)
            assert held <= rot * window_bytes < frames * rz.srcH * rz.srcW * rot or world == 1
            for f in (0, frames - 1):  # frame f's window rows = rows [s0, s1) of frame f
                assert torch.equal(win[f], bench.band_frame(f, rz.srcH, rz.srcW, "cpu")[s0:s1])
