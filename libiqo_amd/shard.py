"""Multi-GPU sharding of the resize hot path (one process per GPU, no data-path collective).

Two decompositions:

* by image -- a batch of F frames is split into contiguous frame ranges, one per rank;
* by output-row band -- one frame's output rows are split into contiguous bands; each rank needs
  only the source rows its band reads (the halo), which the plan reports
  (`iqo_hip_band_src_rows`, host-only).  Rows keep their global indices, so stitching the bands
  gives the unsharded result byte for byte.

Everything here is host arithmetic (no torch, no GPU), so it is tested on CPU with gloo ranks.
"""


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


def halo_overhead(plan, src_h):
    """Extra source rows read because of band halos, as a fraction of the frame."""
    return (sum(s1 - s0 for _, _, s0, s1 in plan) - src_h) / float(src_h)
