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


@pytest.mark.parametrize("world", [2])
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
