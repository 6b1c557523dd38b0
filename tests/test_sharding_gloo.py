"""Multi-GPU decomposition, exercised on CPU with 2 gloo ranks (no GPU): image shards and
output-row bands.  The per-shard compute here is the CPU oracle; what is under test is the
decomposition itself (libiqo_amd/shard.py + the plan's band halo), which the GPU path uses
unchanged (tests/test_gpu_parity.py checks the banded GPU kernels byte for byte)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import libiqo_amd
from libiqo_amd import shard
import oracle_lib as ol

CASES = [("lanczos", 3, 96, 64, 48, 32, 1), ("area", 0, 64, 48, 16, 12, 1), ("linear", 0, 40, 30, 80, 60, 1),
         ("lanczos", 2, 77, 51, 140, 90, 1)]


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
        for ci, (m, d, sw, sh, dw, dh, px) in enumerate(CASES):
            frames = np.stack([ol.gen("noise", sw, sh, 100 * ci + f) for f in range(5)])
            # --- image sharding: each rank resizes its own frame range, then all_gather
            f0, f1 = shard.frame_range(frames.shape[0], rank, world)
            mine = np.stack([ol.run_oracle(m, d, sw, sh, dw, dh, px, frames[f]) for f in range(f0, f1)]) \
                if f1 > f0 else np.zeros((0, dh, dw), np.uint8)
            counts = [shard.frame_range(frames.shape[0], r, world) for r in range(world)]
            maxn = max(b - a for a, b in counts)
            buf = torch.zeros((maxn, dh, dw), dtype=torch.uint8)
            buf[: f1 - f0] = torch.from_numpy(mine)
            gathered = [torch.zeros_like(buf) for _ in range(world)]
            dist.all_gather(gathered, buf)
            full = np.concatenate([gathered[r][: b - a].numpy() for r, (a, b) in enumerate(counts)])
            ref = np.stack([ol.run_oracle(m, d, sw, sh, dw, dh, px, fr) for fr in frames])
            ok = ok and bool((full == ref).all())
            # --- row-band sharding: my band's output depends only on my halo window
            plan = shard.band_plan(lambda r0, n: libiqo_amd.host_band_src_rows(m, d, sw, sh, dw, dh, px, r0, n),
                                   dh, world)
            r0, r1, s0, s1 = plan[rank]
            src = frames[0].copy()
            noisy = ol.gen("noise", sw, sh, 999 + rank)
            src[:s0] = noisy[:s0]      # rows outside the window: garbage
            src[s1:] = noisy[s1:]
            band = ol.run_oracle(m, d, sw, sh, dw, dh, px, src)[r0:r1]
            ok = ok and bool((band == ref[0][r0:r1]).all())
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


def test_band_plan_covers_frame_and_halo_is_small():
    plan = shard.band_plan(lambda r0, n: libiqo_amd.host_band_src_rows("lanczos", 3, 3840, 2160, 1920, 1080, 1, r0, n),
                           1080, 8)
    assert plan[0][0] == 0 and plan[-1][1] == 1080
    assert all(a[1] == b[0] for a, b in zip(plan, plan[1:]))
    # Lanczos-3 2:1: 5 rows above + 6 below per cut -> ~10 rows per internal cut
    assert 0 < shard.halo_overhead(plan, 2160) < 0.04
    assert shard.frame_range(1024, 7, 8) == (896, 1024)
    assert [shard.frame_range(10, r, 4) for r in range(4)] == [(0, 3), (3, 6), (6, 8), (8, 10)]
