"""GPU parity: the HIP path (through the C ABI) reproduces the reference's Generic output
bit-exactly.  Checkers: the golden vectors from the reference (tests/golden) and the CPU oracle
(oracle/, a restatement pinned by those vectors) on the same seeded inputs.  At full BASELINE
sizes, size-independent properties are checked too (fast kernel == general kernel on the same
batch, band-sharded == unsharded, flat stays flat).  All tests run in one process."""
import base64
import os

import numpy as np
import pytest

import oracle_lib as ol

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip("needs a GPU", allow_module_level=True)

import libiqo_amd  # noqa: E402

DEV = torch.device("cuda:0")
# Every drop-in C++ object in this process and in the tools these tests start (they inherit the
# environment) must run on the HIP backend: any CPU fallback aborts (libiqo_amd/csrc/resizers.cpp).
os.environ["IQO_REQUIRE_HIP"] = "1"


def _backend(stdout):
    """The "backend: hip H cpu C" line the drop-in tools print (iqo_dropin_backend_counts)."""
    for line in stdout.splitlines():
        t = line.split()
        if t[:1] == ["backend:"] and t[1] == "hip" and t[3] == "cpu":
            return int(t[2]), int(t[4])
    raise AssertionError("no backend line in:\n" + stdout)


def _expected(c):
    if "out_b64" in c and c["ofast_strict_agree"]:
        return np.frombuffer(base64.b64decode(c["out_b64"]), dtype=np.uint8).reshape(c["dstH"], c["dstW"])
    return None


def _run_host(r, src, dw, dh):
    out = np.zeros((dh, dw), np.uint8)
    r.resize(src.shape[1], src, dw, out)
    return out


def test_native_library_is_the_gpu_path():
    assert libiqo_amd.available() >= 1
    r = libiqo_amd.LanczosResizer(3, 3840, 2160, 1920, 1080)
    assert r.describe()["kernel"] == "lanczos_stream"


@pytest.mark.parametrize("variant", ["default", "tile", "force_general"])
def test_golden_vectors_gpu(golden, variant):
    """Every golden case, via the host-pointer entry point (reference resize() semantics): default
    kernels (the wave walker for shapes without a specialised kernel, where its tables fit), the
    separable tile kernel (plan option walk = 0) and the one-row-per-workgroup general_kernel."""
    n = 0
    for c in golden["cases"]:
        sw, sh, dw, dh = c["srcW"], c["srcH"], c["dstW"], c["dstH"]
        if sw * sh > 4_000_000:
            continue
        r = libiqo_amd.make_resizer(c["method"], c["degree"], sw, sh, dw, dh, c["pxScale"])
        if variant == "tile":
            for k in ("walk", "a32", "d32", "d31", "ryx", "up2", "u23", "l23"):
                r.set_option(k, 0)
        elif variant != "default":
            r.set_option(variant, 1)
        src = ol.gen(c["gen"], sw, sh, c["seed"])
        out = _run_host(r, src, dw, dh)
        exp = _expected(c)
        if exp is not None:
            bad = np.argwhere(out != exp)
            assert bad.size == 0, (c["id"], bad[:4].tolist(), out[tuple(bad[0])], exp[tuple(bad[0])])
        want = c["fnv"] if c["ofast_strict_agree"] else c["fnv_strict"]
        assert "%016x" % ol.fnv1a64(out) == want, c["id"]
        n += 1
    assert n > 500


CONFIGS = [
    ("lanczos", 3, 3840, 2160, 1920, 1080, 1),   # C2 (headline)
    ("area", 0, 7680, 4320, 1920, 1080, 1),      # C3
    ("linear", 0, 1920, 1080, 3840, 2160, 1),    # C4
    ("lanczos", 2, 640, 480, 320, 240, 1),       # C1 shape on the GPU
    ("lanczos", 2, 3840, 2160, 1920, 1080, 1),
    ("lanczos", 3, 1920, 1080, 3840, 2160, 1),   # general path (upsampling)
]


def _noise_batch(n, w, h, seed0):
    frames = np.stack([ol.gen("noise", w, h, seed0 + f) for f in range(n)])
    return frames


@pytest.mark.parametrize("cfg", CONFIGS, ids=lambda c: "%s%d_%dx%d_%dx%d" % (c[0], c[1], c[2], c[3], c[4], c[5]))
def test_device_batch_matches_oracle(cfg):
    m, d, sw, sh, dw, dh, px = cfg
    frames = _noise_batch(3, sw, sh, 100)
    frames[2, : sh // 3] = 255  # flat band + noise in one frame
    src = torch.from_numpy(frames).to(DEV)
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    out = r.resize_tensor(src).cpu().numpy()
    torch.cuda.synchronize()
    for f in range(frames.shape[0]):
        exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, frames[f])
        bad = np.argwhere(out[f] != exp)
        assert bad.size == 0, (cfg, f, bad[:4].tolist())


@pytest.mark.parametrize("cfg", CONFIGS[:3], ids=["c2", "c3", "c4"])
def test_padded_and_misaligned_layouts(cfg):
    """Stride = width + 64 (fast path) and a 1-byte misaligned base (general fallback)."""
    m, d, sw, sh, dw, dh, px = cfg
    frame = ol.gen("noise", sw, sh, 9)
    exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, frame)
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    for pad, off in ((64, 0), (0, 1), (16, 3)):
        sst, dstst = sw + pad, dw + pad
        sbuf = torch.zeros(sh * sst + 64, dtype=torch.uint8, device=DEV)
        sview = sbuf[off:off + sh * sst].view(sh, sst)
        sview[:, :sw] = torch.from_numpy(frame).to(DEV)
        dbuf = torch.zeros(dh * dstst + 64, dtype=torch.uint8, device=DEV)
        r.resize_device(1, sst, sh * sst, sview.data_ptr(), dstst, dh * dstst, dbuf.data_ptr() + off)
        torch.cuda.synchronize()
        got = dbuf[off:off + dh * dstst].view(dh, dstst)[:, :dw].cpu().numpy()
        assert (got == exp).all(), (cfg, pad, off)


@pytest.mark.parametrize("cfg", CONFIGS[:3], ids=["c2", "c3", "c4"])
def test_fast_equals_general_full_batch(cfg):
    """Size-independent property at bench scale: the specialised kernel and the general kernel
    (independent code paths) agree on a 16-frame random batch; frame 0 also matches the oracle."""
    m, d, sw, sh, dw, dh, px = cfg
    g = torch.Generator(device=DEV)
    g.manual_seed(1234)
    src = torch.randint(0, 256, (16, sh, sw), dtype=torch.uint8, device=DEV, generator=g)
    fast = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    gen = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    gen.set_option("force_general", 1)
    assert fast.describe()["kernel"] != "general"
    a = fast.resize_tensor(src)
    b = gen.resize_tensor(src)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, src[0].cpu().numpy())
    assert (a[0].cpu().numpy() == exp).all()


@pytest.mark.parametrize("cfg", CONFIGS[:3] + [CONFIGS[5]], ids=["c2", "c3", "c4", "lz3up"])
def test_row_band_sharding_is_byte_identical(cfg):
    """Multi-GPU sharding by output-row band: each band reads only its halo window of source rows
    (copied into a separate buffer, as a remote GPU would hold it) and the concatenation equals
    the unsharded result -- band-boundary rows included."""
    m, d, sw, sh, dw, dh, px = cfg
    g = torch.Generator(device=DEV)
    g.manual_seed(77)
    src = torch.randint(0, 256, (2, sh, sw), dtype=torch.uint8, device=DEV, generator=g)
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    full = r.resize_tensor(src)
    cuts = [0, 1, dh // 3, dh // 3 + 7, (2 * dh) // 3, dh - 2, dh]
    parts = []
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        s0, sn = r.band_src_rows(r0, r1 - r0)
        window = src[:, s0:s0 + sn].contiguous()
        band = torch.empty((2, r1 - r0, dw), dtype=torch.uint8, device=DEV)
        r.resize_band(2, r0, r1 - r0, s0, sw, sn * sw, window, dw, (r1 - r0) * dw, band,
                      torch.cuda.current_stream())
        parts.append(band)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(parts, dim=1), full)


def test_band_window_must_cover_the_halo():
    """A window that starts one row too late is rejected (it would silently read zeros)."""
    r = libiqo_amd.LanczosResizer(3, 3840, 2160, 1920, 1080)
    s0, sn = r.band_src_rows(500, 100)
    src = torch.zeros((1, sn, 3840), dtype=torch.uint8, device=DEV)
    band = torch.empty((1, 100, 1920), dtype=torch.uint8, device=DEV)
    with pytest.raises(libiqo_amd.IqoError):
        r.resize_band(1, 500, 100, s0 + 1, 3840, sn * 3840, src, 1920, 100 * 1920, band)
    with pytest.raises(libiqo_amd.IqoError):  # r0 + rows past the frame (no size_t wrap)
        r.resize_band(1, 1000, 2 ** 64 - 10, s0, 3840, sn * 3840, src, 1920, 100 * 1920, band)
    r.resize_band(1, 500, 100, s0, 3840, sn * 3840, src, 1920, 100 * 1920, band)
    torch.cuda.synchronize()


def _orchestrated(cfg, devices, host_src, frames=3, seed=5):
    from libiqo_amd import shard

    m, d, sw, sh, dw, dh, px = cfg
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    src = torch.randint(0, 256, (frames, sh, sw), dtype=torch.uint8, device=DEV, generator=g)
    full = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px).resize_tensor(src)
    out = torch.zeros((frames, dh, dw), dtype=torch.uint8, device=DEV)
    s = src.cpu().pin_memory() if host_src else src
    be = shard.HipBandBackend(lambda dev: libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px, device=dev),
                              s, -1 if host_src else 0, out, 0)
    shards = shard.make_shards(be.resizer(0), dh, devices)
    times = shard.run_bands_local(be, shards)
    torch.cuda.synchronize()
    return full, out, times, be


@pytest.mark.parametrize("cfg", CONFIGS[:3] + [CONFIGS[5]], ids=["c2", "c3", "c4", "lz3up"])
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0, 0, 0]], ids=["1band", "2bands", "5bands"])
def test_band_orchestrator_local_matches_unsharded(cfg, devices):
    """libiqo_amd.shard with the HIP backend: windows out (device 0 -> shard device by
    iqo_hip_copy_frames), iqo_hip_resize_band per shard, bands gathered back -- byte-identical to
    the unsharded launch.  On a one-GPU box the shards share device 0."""
    full, out, times, be = _orchestrated(cfg, devices, host_src=False)
    assert torch.equal(out, full)
    assert all(v >= 0 for v in times.values())
    assert be.paths["scatter"] == {"same device"} and be.paths["gather"] == {"same device"}


def test_band_orchestrator_host_source():
    """Windows uploaded from pinned host memory (the H2D route of iqo_hip_copy_frames)."""
    full, out, times, be = _orchestrated(CONFIGS[0], [0, 0, 0], host_src=True)
    assert torch.equal(out, full)
    assert be.paths["scatter"] == {"host<->device"}


def _ipc_worker(rank, world, port, q):
    import os

    import torch.distributed as dist
    from libiqo_amd import shard

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)  # control channel only
    try:
        m, d, sw, sh, dw, dh, px = CONFIGS[0]
        torch.cuda.set_device(0)
        g = torch.Generator(device="cuda:0")
        g.manual_seed(11)
        src = torch.randint(0, 256, (2, sh, sw), dtype=torch.uint8, device="cuda:0", generator=g)
        out = torch.zeros((2, dh, dw), dtype=torch.uint8, device="cuda:0") if rank == 0 else None
        be = shard.HipBandBackend(lambda dev: libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px, device=dev),
                                  src, 0, out, 0)
        shards = shard.make_shards(be.resizer(0), dh, [0] * world)
        times, band = shard.run_bands_distributed(be, shards, rank, world, dist)
        ok = True
        if rank == 0:
            full = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px).resize_tensor(src)
            torch.cuda.synchronize()
            ok = bool(torch.equal(out, full))
        q.put((rank, ok, sorted(be.paths.get("gather", []))))
    except Exception as e:  # report, do not hang the parent
        q.put((rank, repr(e), []))
    finally:
        dist.destroy_process_group()


def test_band_orchestrator_distributed_ipc():
    """One process per shard (2 ranks, both on cuda:0 of the one-GPU box; gloo carries only the
    IPC handles): rank 1's band reaches rank 0's output through iqo_hip_ipc_export / _open and a
    device copy -- no collective on the pixels."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ipc_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, ok, paths = q.get(timeout=100)
        res[r] = (ok, paths)
    for p in procs:
        p.join(timeout=30)
    assert res[0][0] is True and res[1][0] is True, res


def test_256_frame_batch_bit_exact():
    """BASELINE.md §4 batch size for C2: one launch over 256 frames; frames 0, 128, 255 against
    the oracle."""
    sw, sh, dw, dh = 3840, 2160, 1920, 1080
    g = torch.Generator(device=DEV)
    g.manual_seed(256)
    src = torch.randint(0, 256, (256, sh, sw), dtype=torch.uint8, device=DEV, generator=g)
    out = libiqo_amd.LanczosResizer(3, sw, sh, dw, dh).resize_tensor(src)
    torch.cuda.synchronize()
    for f in (0, 128, 255):
        exp = ol.run_oracle("lanczos", 3, sw, sh, dw, dh, 1, src[f].cpu().numpy())
        assert (out[f].cpu().numpy() == exp).all(), f
    del src, out
    torch.cuda.empty_cache()


def test_1024_frame_batch_bit_exact():
    """C5's whole batch (BASELINE.json configs[4]) in ONE launch on one GPU: 1024 C2 frames
    (8.5 GB in, 2.1 GB out); frames 0, 511 and 1023 against the oracle, and the rest of the batch
    against a second launch of the general kernel on a sample of frames."""
    sw, sh, dw, dh = 3840, 2160, 1920, 1080
    g = torch.Generator(device=DEV)
    g.manual_seed(1024)
    src = torch.randint(0, 256, (1024, sh, sw), dtype=torch.uint8, device=DEV, generator=g)
    r = libiqo_amd.LanczosResizer(3, sw, sh, dw, dh)
    assert r.describe()["kernel"] == "lanczos_stream"
    out = r.resize_tensor(src)
    torch.cuda.synchronize()
    for f in (0, 511, 1023):
        exp = ol.run_oracle("lanczos", 3, sw, sh, dw, dh, 1, src[f].cpu().numpy())
        assert (out[f].cpu().numpy() == exp).all(), f
    gen = libiqo_amd.LanczosResizer(3, sw, sh, dw, dh)
    gen.set_option("force_general", 1)
    pick = torch.tensor([1, 255, 256, 700, 1022], device=DEV)
    assert torch.equal(gen.resize_tensor(src[pick].contiguous()), out[pick])
    del src, out
    torch.cuda.empty_cache()


STREAM_SHAPES = [
    (3, 3840, 2160, 1920, 1080),  # C2: 4 waves x 60 lanes per row
    (2, 3840, 2160, 1920, 1080),
    (2, 640, 480, 320, 240),      # C1 shape: one wave of 40 lanes per row
    (3, 1936, 1090, 968, 545),    # odd output height, right-edge wave overlaps its neighbour
    (3, 4000, 64, 2000, 32),      # short bands, 5 waves per row
    (2, 2064, 40, 1032, 20),
    (4, 3840, 2160, 1920, 1080),  # Lanczos-4 2:1: block-shared symmetric streamer (12-row window)
    (4, 1936, 1090, 968, 545),
    (4, 640, 480, 320, 240),
    (4, 2064, 40, 1032, 20),
    (5, 3840, 2160, 1920, 1080),  # Lanczos-5 2:1: 16-row window, 5 border columns per side (8 edge sums)
    (5, 640, 480, 320, 240),
    (5, 2064, 40, 1032, 20),
]


@pytest.mark.parametrize("shape", STREAM_SHAPES, ids=lambda s: "L%d_%dx%d" % s[:3])
def test_stream_variants_agree_with_oracle(shape):
    """Every Lanczos streamer (block-shared symmetric in XCD-aware and dispatch order, accumulator
    ring, per-wave symmetric), every prefetch depth, forced lane counts and band splits produce
    the oracle's output."""
    d, sw, sh, dw, dh = shape
    frames = _noise_batch(2, sw, sh, 300)
    frames[1, :, : sw // 5] = 255
    src = torch.from_numpy(frames).to(DEV)
    exp = [ol.run_oracle("lanczos", d, sw, sh, dw, dh, 1, frames[f]) for f in range(2)]
    for variant, pd, lanes, bands in [(0, 1, 0, 0), (0, 2, 0, 7), (0, 3, 0, 0), (0, 2, 62, 3), (0, 3, 33, 0),
                                      (0, 3, 0, 1), (0, 4, 0, 0), (0, 4, 0, 7), (1, 3, 0, 0), (1, 1, 0, 5),
                                      (2, 3, 0, 0), (2, 1, 0, 5), (2, 2, 40, 0), (3, 3, 0, 0), (3, 2, 0, 7),
                                      (3, 3, 41, 0), (3, 3, 0, 1), (4, 4, 0, 0), (4, 4, 0, 7), (4, 3, 0, 3),
                                      (4, 2, 0, 1), (4, 4, 33, 1)]:
        r = libiqo_amd.make_resizer("lanczos", d, sw, sh, dw, dh, 1)
        assert r.describe()["kernel"] == "lanczos_stream"
        if variant == 3:  # block-shared streamer in plain dispatch order
            variant = 0
            r.set_option("xcd_order", 0)
        elif variant == 4:  # packed ring rows (prefetch 4: ring depth 5 = the Lanczos-3 window period)
            variant = 0
            r.set_option("ring_pack", 1)
        r.set_option("stream_variant", variant)
        r.set_option("prefetch", pd)
        r.set_option("lanes", lanes)
        r.set_option("bands", bands)
        out = r.resize_tensor(src).cpu().numpy()
        for f in range(2):
            bad = np.argwhere(out[f] != exp[f])
            assert bad.size == 0, (shape, variant, pd, lanes, bands, f, bad[:4].tolist())


CHROMA_SHAPES = [
    (3, 1920, 1080, 960, 540),  # the 4:2:0 chroma planes of C2 (pxScale 2: 3-tap tables, negative
    (2, 320, 240, 160, 120),    # border denominators) and of C1
    (3, 1936, 1090, 968, 545),
    (3, 640, 480, 320, 240),
    (2, 2064, 40, 1032, 20),
]


@pytest.mark.parametrize("shape", CHROMA_SHAPES, ids=lambda s: "L%d_%dx%d_px2" % s[:3])
def test_chroma_pxscale2_stream_agrees_with_oracle(shape):
    """pxScale-2 (chroma) Lanczos tables run the accumulator-ring streamer, including border rows
    and columns whose valid taps sum to a negative denominator."""
    d, sw, sh, dw, dh = shape
    frames = _noise_batch(2, sw, sh, 700)
    frames[1, sh // 2:, :] = 255
    src = torch.from_numpy(frames).to(DEV)
    exp = [ol.run_oracle("lanczos", d, sw, sh, dw, dh, 2, frames[f]) for f in range(2)]
    for pd, bands in [(1, 0), (2, 3), (3, 0), (3, dh)]:
        r = libiqo_amd.make_resizer("lanczos", d, sw, sh, dw, dh, 2)
        assert r.describe()["kernel"] == "lanczos_stream"
        r.set_option("prefetch", pd)
        r.set_option("bands", bands)
        out = r.resize_tensor(src).cpu().numpy()
        for f in range(2):
            bad = np.argwhere(out[f] != exp[f])
            assert bad.size == 0, (shape, pd, bands, f, bad[:4].tolist())


TILE_SHAPES = [
    ("lanczos", 3, 1920, 1080, 1280, 720, 1),   # 3:2, 2 phases
    ("lanczos", 3, 640, 480, 1280, 960, 1),     # upscale
    ("lanczos", 2, 1000, 700, 333, 250, 1),     # odd ratios, borders everywhere
    ("lanczos", 4, 801, 601, 400, 300, 2),      # pxScale 2, 2:1 odd sizes
    ("area", 0, 1920, 1080, 1280, 720, 1),      # non-integer area (weight-0 tap past the end)
    ("linear", 0, 640, 480, 1000, 700, 1),      # linear, non-2x
    ("lanczos", 3, 64, 48, 640, 480, 1),        # 10x upscale
    ("lanczos", 3, 3840, 2160, 3840, 1080, 1),  # Y only (X identity)
    ("lanczos", 3, 1366, 768, 1000, 562, 1),    # width not a multiple of 4 (byte-aligned rows)
    ("area", 0, 1001, 777, 640, 480, 1),
    ("linear", 0, 1917, 1079, 1280, 720, 1),    # linear downscale
    ("lanczos", 9, 500, 400, 1200, 900, 1),     # degree 9 upscale
    ("lanczos", 1, 1920, 1080, 1000, 600, 1),
    ("lanczos", 3, 1920, 1080, 400, 220, 1),    # 4.8:1, 30 X taps (16 pairs)
    ("lanczos", 3, 13, 9, 5, 40, 1),            # narrow: every group is an edge group
]


@pytest.mark.parametrize("cfg", TILE_SHAPES, ids=lambda c: "%s%d_%dx%d_%dx%d" % c[:6])
def test_tile_streamer_matches_oracle(cfg):
    """General ratios (shapes without a specialised kernel): the wave walker (the default on
    4-byte aligned sources where its tables fit; several band splits and a padded stride), the
    separable tile kernel (plan option walk = 0, and every misaligned layout: 8-byte,
    12-byte-shifted and single-byte loads; dword and byte stores) equal the oracle, and
    general_kernel (tile = 0) on the same batch."""
    m, d, sw, sh, dw, dh, px = cfg
    frames = _noise_batch(2, sw, sh, 1100)
    frames[1, :, : sw // 3] = 255
    exp = [ol.run_oracle(m, d, sw, sh, dw, dh, px, frames[f]) for f in range(2)]
    t = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    for k in ("walk", "a32", "d32", "d31", "ryx", "up2", "u23", "l23"):
        t.set_option(k, 0)
    assert t.describe()["kernel"] == "tile"
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    for k in ("up2", "d32", "d31", "ryx", "a32", "u23", "l23"):  # exact-ratio kernels off: the walker alone (their own tests below)
        r.set_option(k, 0)
    kern = r.describe()["kernel"]
    assert kern in ("walk", "tile")
    src = torch.from_numpy(frames).to(DEV)
    for rr in (r, t):
        out = rr.resize_tensor(src).cpu().numpy()
        for f in range(2):
            bad = np.argwhere(out[f] != exp[f])
            assert bad.size == 0, (cfg, rr.describe()["kernel"], f, bad[:4].tolist())
    if kern == "walk":
        for bands in (1, 3, 7, dh):
            w = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
            for k in ("up2", "d32", "d31", "ryx", "a32", "u23", "l23"):
                w.set_option(k, 0)
            w.set_option("bands", bands)
            out = w.resize_tensor(src).cpu().numpy()
            for f in range(2):
                bad = np.argwhere(out[f] != exp[f])
                assert bad.size == 0, (cfg, "walk bands", bands, f, bad[:4].tolist())
        sst = (sw + 7) & ~3  # 4-byte aligned padded stride: the walker again
        pbuf = torch.zeros((2, sh, sst), dtype=torch.uint8, device=DEV)
        pbuf[:, :, :sw] = src
        dbuf = torch.zeros((2, dh, dw + 3), dtype=torch.uint8, device=DEV)
        r.resize_device(2, sst, sh * sst, pbuf.data_ptr(), dw + 3, dh * (dw + 3), dbuf.data_ptr())
        got = dbuf[:, :, :dw].cpu().numpy()
        for f in range(2):
            assert (got[f] == exp[f]).all(), (cfg, "walk padded", f)
    # misaligned base (byte loads), padded strides
    sst = sw + 3
    sbuf = torch.zeros(sh * sst + 64, dtype=torch.uint8, device=DEV)
    sview = sbuf[1:1 + sh * sst].view(sh, sst)
    sview[:, :sw] = src[0]
    dbuf = torch.zeros(dh * (dw + 5), dtype=torch.uint8, device=DEV)
    r.resize_device(1, sst, sh * sst, sview.data_ptr(), dw + 5, dh * (dw + 5), dbuf.data_ptr())
    got = dbuf.view(dh, dw + 5)[:, :dw].cpu().numpy()
    assert (got == exp[0]).all(), cfg
    g = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    g.set_option("tile", 0)
    assert g.describe()["kernel"] == "general"
    assert torch.equal(g.resize_tensor(src), r.resize_tensor(src))


LINEAR_UP2_SHAPES = [
    (1920, 1080, 2),  # C4: 4 waves x 60 lanes per row
    (640, 480, 2),    # 80 lanes: 2 waves x 40
    (8, 1, 2),        # one producing lane; both output rows are replicated borders
    (24, 2, 2),       # three lanes, one interior row pair
    (504, 7, 2),      # 63 lanes: 2 waves, the right-edge wave overlaps its neighbour
    (1000, 33, 2),
    (1280, 720, 3),   # 3x: 24 output columns per lane, 3 output rows per source row
    (8, 1, 3),
    (24, 3, 3),
    (504, 7, 3),
]


@pytest.mark.parametrize("shape", LINEAR_UP2_SHAPES, ids=lambda s: "%dx%dx%d" % s)
def test_linear_up2_streamer_variants(shape):
    """The exact-2x / 3x Linear streamer at every prefetch depth and band split (bands starting on
    any row phase, one-row bands, bands holding only a border row) produces the oracle's output."""
    sw, sh, f = shape
    dw, dh = f * sw, f * sh
    frames = _noise_batch(2, sw, sh, 500)
    frames[1, :, : max(1, sw // 5)] = 255
    src = torch.from_numpy(frames).to(DEV)
    exp = [ol.run_oracle("linear", 0, sw, sh, dw, dh, 1, frames[f]) for f in range(2)]
    for pd, bands in [(0, 0), (2, 1), (4, 3), (8, 0), (2, dh), (4, max(1, dh // 2 + 1))]:
        r = libiqo_amd.make_resizer("linear", 0, sw, sh, dw, dh, 1)
        assert r.describe()["kernel"] == "linear_up2"
        r.set_option("lin_prefetch", pd)
        r.set_option("bands", bands)
        out = r.resize_tensor(src).cpu().numpy()
        for f in range(2):
            bad = np.argwhere(out[f] != exp[f])
            assert bad.size == 0, (shape, pd, bands, f, bad[:4].tolist())


@pytest.mark.parametrize("cfg", CONFIGS[:4], ids=["c2", "c3", "c4", "c1"])
def test_host_pointer_pipeline_pinned_and_pageable(cfg):
    """The host-pointer drop-in (band-pipelined H2D / kernel / D2H) gives the oracle's output from
    pageable numpy buffers and from pinned host tensors, with padded strides, and repeatedly with
    one plan (the staging set is pooled and reused)."""
    m, d, sw, sh, dw, dh, px = cfg
    frame = ol.gen("noise", sw, sh, 21)
    exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, frame)
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    # pageable, tight strides (twice: the pooled staging set is reused)
    for _ in range(2):
        out = np.zeros((dh, dw), np.uint8)
        r.resize(sw, frame, dw, out)
        assert (out == exp).all(), cfg
    # pinned, padded strides
    sst, dst_st = sw + 32, dw + 48
    src = torch.zeros((sh, sst), dtype=torch.uint8).pin_memory()
    src[:, :sw] = torch.from_numpy(frame)
    out = torch.full((dh, dst_st), 7, dtype=torch.uint8).pin_memory()
    r.resize(sst, src, dst_st, out)
    got = out.numpy()
    assert (got[:, :dw] == exp).all(), cfg
    assert (got[:, dw:] == 7).all(), "bytes past the row written"


YUV_CASES = [
    ("lanczos", 3, 3840, 2160, 1920, 1080, True),   # block-shared symmetric Y + ring chroma, one launch
    ("lanczos", 2, 640, 480, 320, 240, True),       # per-wave symmetric Y (1 wave per row) + ring chroma
    ("area", 0, 7680, 4320, 1920, 1080, True),
    ("linear", 0, 1920, 1080, 3840, 2160, True),
    ("lanczos", 3, 1920, 1080, 1280, 720, False),   # plane by plane: exact 3:2 kernel on Y
    ("lanczos", 3, 960, 540, 1920, 1080, False),     # plane by plane: exact 2x kernel on Y
    ("area", 0, 1920, 1080, 1280, 720, False),       # plane by plane: exact 3:2 Area kernel
]


@pytest.mark.parametrize("case", YUV_CASES, ids=lambda c: "%s%d_%dx%d" % c[:4])
def test_yuv420_planes_match_oracle(case):
    """I420 batch through iqo_hip_resize_yuv420_device: each plane equals the oracle on that plane
    (Lanczos chroma with pxScale 2, as the reference benchmark builds it, benchmark.cpp:222)."""
    m, d, sw, sh, dw, dh, want_fused = case
    n = 2
    cw, ch, cdw, cdh = sw // 2, sh // 2, dw // 2, dh // 2
    y = _noise_batch(n, sw, sh, 900)
    u = _noise_batch(n, cw, ch, 910)
    v = _noise_batch(n, cw, ch, 920)
    v[1, : ch // 2] = 255
    src = torch.from_numpy(np.concatenate([y.reshape(n, -1), u.reshape(n, -1), v.reshape(n, -1)], axis=1)).to(DEV)
    r = libiqo_amd.Yuv420Resizer(m, d, sw, sh, dw, dh)
    out, fused = r.resize_frames(src)
    out = out.cpu().numpy()
    assert fused == want_fused
    pxc = 2 if m == "lanczos" else 1
    for f in range(n):
        oy = out[f, : dw * dh].reshape(dh, dw)
        ou = out[f, dw * dh: dw * dh + cdw * cdh].reshape(cdh, cdw)
        ov = out[f, dw * dh + cdw * cdh:].reshape(cdh, cdw)
        assert (oy == ol.run_oracle(m, d, sw, sh, dw, dh, 1, y[f])).all(), (case, f, "Y")
        assert (ou == ol.run_oracle(m, d, cw, ch, cdw, cdh, pxc, u[f])).all(), (case, f, "U")
        assert (ov == ol.run_oracle(m, d, cw, ch, cdw, cdh, pxc, v[f])).all(), (case, f, "V")


def test_yuv420_host_pointers():
    m, d, sw, sh, dw, dh = "lanczos", 2, 640, 480, 320, 240
    y = ol.gen("noise", sw, sh, 31)
    u = ol.gen("noise", sw // 2, sh // 2, 32)
    v = ol.gen("noise", sw // 2, sh // 2, 33)
    oy = np.zeros((dh, dw), np.uint8)
    ou = np.zeros((dh // 2, dw // 2), np.uint8)
    ov = np.zeros((dh // 2, dw // 2), np.uint8)
    libiqo_amd.Yuv420Resizer(m, d, sw, sh, dw, dh).resize(sw, y, sw // 2, u, v, dw, oy, dw // 2, ou, ov)
    assert (oy == ol.run_oracle(m, d, sw, sh, dw, dh, 1, y)).all()
    assert (ou == ol.run_oracle(m, d, sw // 2, sh // 2, dw // 2, dh // 2, 2, u)).all()
    assert (ov == ol.run_oracle(m, d, sw // 2, sh // 2, dw // 2, dh // 2, 2, v)).all()


@pytest.mark.parametrize("value", [0, 255])
def test_flat_frames_stay_flat_full_size(value):
    for m, d, sw, sh, dw, dh, px in CONFIGS[:3]:
        src = torch.full((4, sh, sw), value, dtype=torch.uint8, device=DEV)
        out = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px).resize_tensor(src)
        torch.cuda.synchronize()
        assert bool((out == value).all()), (m, value)


def test_checkerboard_and_g1_c2():
    m, d, sw, sh, dw, dh, px = CONFIGS[0]
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    for kind in ("checker", "g1", "mt19937"):
        frame = ol.gen(kind, sw, sh)
        out = r.resize_tensor(torch.from_numpy(frame).to(DEV)).cpu().numpy()
        assert (out == ol.run_oracle(m, d, sw, sh, dw, dh, px, frame)).all(), kind


def test_many_frames_grid_chunking():
    """More frames than one grid dimension per launch would allow is chunked internally; here a
    small shape with 70000 frames exercises the >65535 split."""
    m, d, sw, sh, dw, dh, px = ("lanczos", 3, 32, 8, 16, 4, 1)
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    src = torch.randint(0, 256, (70000, sh, sw), dtype=torch.uint8, device=DEV, generator=g)
    out = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px).resize_tensor(src)
    torch.cuda.synchronize()
    for f in (0, 65534, 65535, 69999):
        exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, src[f].cpu().numpy())
        assert (out[f].cpu().numpy() == exp).all(), f


@pytest.mark.parametrize("m,iw,ih,ow,oh", [("lanczos2", 640, 480, 320, 240), ("lanczos3", 3840, 2160, 1920, 1080),
                                           ("area", 7680, 4320, 1920, 1080), ("linear", 1920, 1080, 3840, 2160)])
def test_cpp_dropin_benchmark_cli(tmp_path, m, iw, ih, ow, oh):
    """The reference-compatible benchmark CLI (benchmark/iqo_benchmark.cpp), built against the
    drop-in iqo::*Resizer classes, produces the Generic output on the benchmark's own input
    (std::mt19937(0) Y plane, benchmark.cpp:51-59)."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(libiqo_amd.LIB_PATH), "build", "iqo_benchmark")
    out = tmp_path / "y.raw"
    r = subprocess.run([exe, "-m", m, "-iw", str(iw), "-ih", str(ih), "-ow", str(ow), "-oh", str(oh),
                        "-cycles", "2", "-check", str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ms/cycle" in r.stdout
    hip, cpu = _backend(r.stdout)
    assert hip >= 4 and cpu == 0, r.stdout  # a Y and a UV object per cycle (benchmark.cpp:206-229), 2 cycles, all on HIP
    got = np.fromfile(str(out), dtype=np.uint8).reshape(oh, ow)
    method = "lanczos" if m.startswith("lanczos") else m
    degree = int(m[7]) if method == "lanczos" else 0
    exp = ol.run_oracle(method, degree, iw, ih, ow, oh, 1, ol.gen("mt19937", iw, ih))
    assert (got == exp).all()


@pytest.mark.gpu
@pytest.mark.parametrize("m,iw,ih,ow,oh", [("lanczos3", 400, 300, 200, 150), ("lanczos", 301, 203, 150, 101),
                                           ("area", 640, 480, 320, 240), ("linear", 161, 121, 320, 240)])
def test_sample_yuv420p_file_tool(tmp_path, m, iw, ih, ow, oh):
    """The raw-I420 file tool (sample/iqo_resize_yuv420p.cpp, the reference's
    sample/resize_yuv420p.cpp interface): two frames of a file, every plane equal to the Generic
    oracle on the reference's plane geometry (luma W x H at stride W+W%2, chroma (W+W%2)/2 x
    (H+H%2)/2, Lanczos chroma at pxScale 2).  Even shapes take the one-plan YUV420 path, odd ones
    the three drop-in resizer objects."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(libiqo_amd.LIB_PATH), "build", "iqo_resize_yuv420p")
    sx, sy, dx, dy = iw + iw % 2, ih + ih % 2, ow + ow % 2, oh + oh % 2
    nsrc, ndst = sx * sy * 3 // 2, dx * dy * 3 // 2
    raw = np.concatenate([ol.splitmix_bytes(nsrc, 11), ol.splitmix_bytes(nsrc, 12)]).astype(np.uint8)
    fin, fout = tmp_path / "in.yuv", tmp_path / "out.yuv"
    raw.tofile(str(fin))
    r = subprocess.run([exe, "-m", m, "-i", str(fin), "-iw", str(iw), "-ih", str(ih), "-o", str(fout),
                        "-ow", str(ow), "-oh", str(oh), "-frames", "2"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    hip, cpu = _backend(r.stdout)
    assert cpu == 0 and (hip == 2 or "YUV420 plan: yes" in r.stdout), r.stdout  # a Y and a chroma object
    got = np.fromfile(str(fout), dtype=np.uint8)
    assert got.size == 2 * ndst
    method = "lanczos" if m.startswith("lanczos") else m
    degree = (int(m[7]) if len(m) == 8 else 2) if method == "lanczos" else 0
    pxc = 2 if method == "lanczos" else 1
    for f in range(2):
        s, d = raw[f * nsrc:(f + 1) * nsrc], got[f * ndst:(f + 1) * ndst]
        sY, dY = s[:sx * sy].reshape(sy, sx), d[:dx * dy].reshape(dy, dx)
        exp = ol.run_oracle(method, degree, iw, ih, ow, oh, 1, sY[:ih, :iw])
        assert (dY[:oh, :ow] == exp).all(), (m, f, "Y")
        cs, cd = sx * sy // 4, dx * dy // 4
        for p, name in ((0, "U"), (1, "V")):
            sc = s[sx * sy + p * cs: sx * sy + (p + 1) * cs].reshape(sy // 2, sx // 2)
            dc = d[dx * dy + p * cd: dx * dy + (p + 1) * cd].reshape(dy // 2, dx // 2)
            exp = ol.run_oracle(method, degree, sx // 2, sy // 2, dx // 2, dy // 2, pxc, sc)
            assert (dc == exp).all(), (m, f, name)


_DROPIN = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))), "tests", "native", "_build", "dropin")


@pytest.mark.parametrize("m,iw,ih,ow,oh", [("lanczos3", 640, 480, 320, 240), ("lanczos2", 1920, 1080, 1280, 720),
                                           ("area", 640, 480, 160, 120), ("linear", 320, 240, 640, 480),
                                           ("lanczos3", 401, 301, 200, 151)])
def test_reference_sample_binary_on_gpu(tmp_path, m, iw, ih, ow, oh):
    """The reference's own sample/resize_yuv420p.cpp, compiled UNCHANGED against include/libiqo +
    libiqo_hip.so (tests/native/dropin.mk, built in the build container), run on the GPU: every
    plane of its output file equals the Generic oracle (luma W x H at stride W+W%2, chroma
    (W+W%2)/2 x (H+H%2)/2 with pxScale 2 for Lanczos, resize_yuv420p.cpp:66-163)."""
    import os
    import subprocess
    exe = os.path.join(_DROPIN, "resize_yuv420p")
    if not os.path.exists(exe):
        pytest.skip("reference tools not built (build() builds them where /root/reference exists)")
    sx, sy, dx, dy = iw + iw % 2, ih + ih % 2, ow + ow % 2, oh + oh % 2
    nsrc, ndst = sx * sy * 3 // 2, dx * dy * 3 // 2
    raw = ol.splitmix_bytes(nsrc, 21).astype(np.uint8)
    fin, fout = tmp_path / "in.yuv", tmp_path / "out.yuv"
    raw.tofile(str(fin))
    r = subprocess.run([exe, "-m", m, "-i", str(fin), "-iw", str(iw), "-ih", str(ih), "-o", str(fout),
                        "-ow", str(ow), "-oh", str(oh)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, IQO_DROPIN_REPORT="1"))
    assert r.returncode == 0, r.stdout + r.stderr
    # a Y and a chroma object, three resize() calls (resize_yuv420p.cpp:121-163)
    assert "libiqo_amd drop-in: objects hip=2 cpu=0, resize calls hip=3 cpu=0" in r.stderr, r.stderr
    got = np.fromfile(str(fout), dtype=np.uint8)
    assert got.size == ndst
    method = "lanczos" if m.startswith("lanczos") else m
    degree = int(m[7]) if method == "lanczos" else 0
    sY, dY = raw[:sx * sy].reshape(sy, sx), got[:dx * dy].reshape(dy, dx)
    assert (dY[:oh, :ow] == ol.run_oracle(method, degree, iw, ih, ow, oh, 1, sY[:ih, :iw])).all()
    cs, cd = sx * sy // 4, dx * dy // 4
    for p in (0, 1):
        sc = raw[sx * sy + p * cs: sx * sy + (p + 1) * cs].reshape(sy // 2, sx // 2)
        dc = got[dx * dy + p * cd: dx * dy + (p + 1) * cd].reshape(dy // 2, dx // 2)
        exp = ol.run_oracle(method, degree, sx // 2, sy // 2, dx // 2, dy // 2, 2 if method == "lanczos" else 1, sc)
        assert (dc == exp).all(), (m, p)


@pytest.mark.parametrize("m,iw,ih,ow,oh", [("lanczos3", 3840, 2160, 1920, 1080), ("lanczos2", 640, 480, 320, 240)])
def test_reference_benchmark_binary_on_gpu(tmp_path, m, iw, ih, ow, oh):
    """The reference's own benchmark/benchmark.cpp, compiled unchanged against the drop-in, runs
    its 256-cycle timed loop (resizers constructed inside the loop) on the GPU backend: every
    object and every resize() call on HIP (IQO_DROPIN_REPORT), and the pixels of its first cycle
    (IQO_DROPIN_DUMP: Y, U, V) equal to the Generic oracle on the benchmark's own input
    (std::mt19937(0) per plane, benchmark.cpp:51-59,1013-1015; chroma at pxScale 2, :206-229)."""
    import subprocess
    exe = os.path.join(_DROPIN, "benchmark")
    if not os.path.exists(exe):
        pytest.skip("reference tools not built")
    r = subprocess.run([exe, "-m", m, "-iw", str(iw), "-ih", str(ih), "-ow", str(ow), "-oh", str(oh)],
                       capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, IQO_DROPIN_REPORT="1", IQO_DROPIN_DUMP=str(tmp_path)))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "elapsed time" in r.stdout and "ms/cycle" in r.stdout
    assert "size: %dx%d" % (iw, ih) in r.stdout and "size: %dx%d" % (ow, oh) in r.stdout
    assert "objects hip=512 cpu=0, resize calls hip=768 cpu=0" in r.stderr, r.stderr  # 256 cycles x (1 + 1) objects, 3 calls
    degree = int(m[7])
    planes = [(0, iw, ih, ow, oh, 1), (1, iw // 2, ih // 2, ow // 2, oh // 2, 2), (2, iw // 2, ih // 2, ow // 2, oh // 2, 2)]
    for k, sw, sh, dw, dh, px in planes:
        got = np.fromfile(str(tmp_path / ("resize%d_%dx%d.raw" % (k, dw, dh))), np.uint8).reshape(dh, dw)
        exp = ol.run_oracle("lanczos", degree, sw, sh, dw, dh, px, ol.gen("mt19937", sw, sh, 0))
        assert (got == exp).all(), (m, k)


def test_concurrent_plans_from_host_threads(tmp_path):
    """Distinct drop-in objects (Lanczos / Area / Linear, host pointers) used at the same time from
    12 host threads, 3 rounds, a fresh object per thread and round: every concurrent output equals
    the same job run alone (tests/native/threads_test.cpp), and every solo output equals the
    Generic oracle."""
    import glob
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(libiqo_amd.LIB_PATH), "build", "threads_test")
    r = subprocess.run([exe, str(tmp_path), "12", "3"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    hip, cpu = _backend(r.stdout)
    assert hip == 48 and cpu == 0, r.stdout  # 12 solo + 3 x 12 concurrent objects
    jobs = sorted(glob.glob(str(tmp_path / "*.src")))
    assert len(jobs) == 12
    for sp in jobs:
        name = os.path.basename(sp)[:-4].split("_")
        mi, d = int(name[1]), int(name[2])
        sw, sh = map(int, name[3].split("x"))
        dw, dh = map(int, name[4].split("x"))
        src = np.fromfile(sp, np.uint8).reshape(sh, sw)
        dst = np.fromfile(sp[:-4] + ".dst", np.uint8).reshape(dh, dw)
        m = ("lanczos", "area", "linear")[mi]
        assert (dst == ol.run_oracle(m, d, sw, sh, dw, dh, 1, src)).all(), sp

UP2_SHAPES = [
    ("lanczos", 3, 1920, 1080, 3840, 2160, 1),   # G2
    ("lanczos", 2, 960, 540, 1920, 1080, 1),
    ("lanczos", 3, 640, 360, 1280, 720, 1),
    ("lanczos", 3, 392, 100, 784, 200, 1),       # one wave holding both edges
    ("lanczos", 2, 200, 60, 400, 120, 1),
    ("lanczos", 3, 1280, 720, 3840, 2160, 1),    # 3x: 24 output columns per lane, 3 rows per source row
    ("lanczos", 2, 640, 360, 1920, 1080, 1),
    ("lanczos", 3, 136, 40, 408, 120, 1),        # 3x, one wave holding both edges
]


@pytest.mark.parametrize("cfg", UP2_SHAPES, ids=lambda c: "%s%d_%dx%d" % c[:4])
def test_lanczos_up2_matches_oracle(cfg):
    """Exact 2x Lanczos upscale: lanczos_up2_kernel on every row and column (masked border rows
    and columns divided in the kernel), equal to the oracle on noise and flat frames; with option
    up2 = 0 (walker alone), in band splits and lane counts, in row bands (iqo_hip_resize_band
    windows), and with an unaligned destination stride (walker alone)."""
    m, d, sw, sh, dw, dh, px = cfg
    n = 2 if sw * sh > 1_000_000 else 3
    frames = _noise_batch(n, sw, sh, 1300)
    frames[-1] = 77
    exp = [ol.run_oracle(m, d, sw, sh, dw, dh, px, frames[f]) for f in range(n)]
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    assert r.describe()["kernel"] == "lanczos_up2"
    src = torch.from_numpy(frames).to(DEV)
    out = r.resize_tensor(src).cpu().numpy()
    for f in range(n):
        bad = np.argwhere(out[f] != exp[f])
        assert bad.size == 0, (cfg, f, bad[:4].tolist())
    w = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    w.set_option("up2", 0)
    assert w.describe()["kernel"] in ("walk", "tile")
    assert (w.resize_tensor(src).cpu().numpy() == out).all()
    for opt, val in (("bands", 1), ("bands", 3), ("bands", 7), ("lanes", 5), ("lanes", 62)):
        for alt in (1, 0):  # odd bands walking bottom-up (default) / every band top-down
            b = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
            b.set_option(opt, val)
            b.set_option("ratio_alt", alt)
            assert (b.resize_tensor(src).cpu().numpy() == out).all(), (cfg, opt, val, alt)
    # row bands through their source windows (odd band edges)
    got = torch.zeros((n, dh, dw), dtype=torch.uint8, device=DEV)
    cuts = [0, 3, dh // 3 + 1, dh // 2, dh]
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        s0, sn = r.band_src_rows(r0, r1 - r0)
        win = src[:, s0:s0 + sn].contiguous()
        r.resize_band(n, r0, r1 - r0, s0, sw, sn * sw, win.data_ptr(), dw, dh * dw, got[:, r0].data_ptr())
    torch.cuda.synchronize()
    assert (got.cpu().numpy() == out).all(), cfg
    # destination stride not 16-byte aligned: the walker alone
    dst = torch.zeros((n, dh, dw + 4), dtype=torch.uint8, device=DEV)
    r.resize_device(n, sw, sh * sw, src.data_ptr(), dw + 4, dh * (dw + 4), dst.data_ptr())
    torch.cuda.synchronize()
    assert (dst[:, :, :dw].cpu().numpy() == out).all(), cfg


D32_SHAPES = [
    ("lanczos", 3, 1920, 1080, 1280, 720, 1),    # G1: three waves per row (x0 of the last clamped)
    ("lanczos", 3, 1440, 1080, 960, 720, 1),     # two waves per row
    ("lanczos", 3, 504, 300, 336, 200, 1),       # one wave holding both edges
    ("lanczos", 2, 1920, 1080, 1280, 720, 1),    # Lanczos-2 tap structure
    ("lanczos", 2, 240, 150, 160, 100, 1),
]


@pytest.mark.parametrize("cfg", D32_SHAPES, ids=lambda c: "%s%d_%dx%d" % c[:4])
def test_lanczos_d32_matches_oracle(cfg):
    """Exact 3:2 Lanczos-3 downscale: lanczos_d32_kernel on every row and column (masked border
    rows and columns divided in the kernel); equal to the oracle on noise, flat and
    half-flat frames; with option d32 = 0 (walker alone), in several band splits (odd bands walk
    bottom-up; ratio_alt = 0: every band top-down) and lane counts, in row bands through their
    source windows (odd band edges), with padded strides (d32 again) and a destination stride that
    is not 8-byte aligned (walker alone)."""
    m, d, sw, sh, dw, dh, px = cfg
    n = 3
    frames = _noise_batch(n, sw, sh, 1700)
    frames[1] = 77
    frames[2, :, : sw // 2] = 255
    exp = [ol.run_oracle(m, d, sw, sh, dw, dh, px, frames[f]) for f in range(n)]
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    assert r.describe()["kernel"] == "lanczos_d32"
    src = torch.from_numpy(frames).to(DEV)
    out = r.resize_tensor(src).cpu().numpy()
    for f in range(n):
        bad = np.argwhere(out[f] != exp[f])
        assert bad.size == 0, (cfg, f, bad[:4].tolist())
    w = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    w.set_option("d32", 0)
    assert w.describe()["kernel"] in ("walk", "tile")
    assert (w.resize_tensor(src).cpu().numpy() == out).all()
    for opt, val in (("bands", 1), ("bands", 3), ("bands", 7), ("bands", dh), ("lanes", 8), ("lanes", 62),
                     ("ratio_alt", 0)):
        b = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
        b.set_option(opt, val)
        assert (b.resize_tensor(src).cpu().numpy() == out).all(), (cfg, opt, val)
    # row bands through their source windows (odd band edges)
    got = torch.zeros((n, dh, dw), dtype=torch.uint8, device=DEV)
    cuts = [0, 3, dh // 3 + 1, dh // 2, dh - 5, dh]
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        s0, sn = r.band_src_rows(r0, r1 - r0)
        win = src[:, s0:s0 + sn].contiguous()
        r.resize_band(n, r0, r1 - r0, s0, sw, sn * sw, win.data_ptr(), dw, dh * dw, got[:, r0].data_ptr())
    torch.cuda.synchronize()
    assert (got.cpu().numpy() == out).all(), cfg
    # padded strides (4-byte aligned source rows, 8-byte aligned destination rows): d32 again
    sst, dst_st = sw + 4, dw + 8
    pbuf = torch.zeros((n, sh, sst), dtype=torch.uint8, device=DEV)
    pbuf[:, :, :sw] = src
    dbuf = torch.full((n, dh, dst_st), 9, dtype=torch.uint8, device=DEV)
    r.resize_device(n, sst, sh * sst, pbuf.data_ptr(), dst_st, dh * dst_st, dbuf.data_ptr())
    torch.cuda.synchronize()
    assert (dbuf[:, :, :dw].cpu().numpy() == out).all(), cfg
    assert (dbuf[:, :, dw:].cpu().numpy() == 9).all(), (cfg, "wrote past the row")
    # destination stride not 8-byte aligned: the walker alone
    dst = torch.zeros((n, dh, dw + 4), dtype=torch.uint8, device=DEV)
    r.resize_device(n, sw, sh * sw, src.data_ptr(), dw + 4, dh * (dw + 4), dst.data_ptr())
    torch.cuda.synchronize()
    assert (dst[:, :, :dw].cpu().numpy() == out).all(), cfg


A32_SHAPES = [
    ("area", 0, 1920, 1080, 1280, 720, 1),       # G3: three waves per row (x0 of the last clamped)
    ("area", 0, 504, 300, 336, 200, 1),          # one wave per row
    ("area", 0, 48, 30, 32, 20, 1),
    ("area", 0, 12, 6, 8, 4, 1),                 # one lane per row
]


@pytest.mark.parametrize("cfg", A32_SHAPES, ids=lambda c: "%s_%dx%d" % (c[0], c[2], c[3]))
def test_area_d32_matches_oracle(cfg):
    """Exact 3:2 Area downscale: area_d32_kernel equal to the oracle on noise, flat and half-flat
    frames; with option a32 = 0 (walker or tile kernel), in band splits and lane counts, in row
    bands through their source windows, with padded strides (a32 again) and a destination stride
    that is not 8-byte aligned (walker / tile)."""
    m, d, sw, sh, dw, dh, px = cfg
    n = 3
    frames = _noise_batch(n, sw, sh, 1900)
    frames[1] = 255
    frames[2, :, : sw // 2] = 0
    exp = [ol.run_oracle(m, d, sw, sh, dw, dh, px, frames[f]) for f in range(n)]
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    assert r.describe()["kernel"] == "area_d32"
    src = torch.from_numpy(frames).to(DEV)
    out = r.resize_tensor(src).cpu().numpy()
    for f in range(n):
        bad = np.argwhere(out[f] != exp[f])
        assert bad.size == 0, (cfg, f, bad[:4].tolist())
    w = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    w.set_option("a32", 0)
    assert w.describe()["kernel"] in ("walk", "tile")
    assert (w.resize_tensor(src).cpu().numpy() == out).all()
    for opt, val in (("bands", 1), ("bands", 3), ("bands", dh), ("lanes", 1), ("lanes", 7)):
        b = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
        b.set_option(opt, val)
        assert (b.resize_tensor(src).cpu().numpy() == out).all(), (cfg, opt, val)
    got = torch.zeros((n, dh, dw), dtype=torch.uint8, device=DEV)
    cuts = sorted({0, 1, dh // 3 + 1, dh // 2, dh})
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        s0, sn = r.band_src_rows(r0, r1 - r0)
        win = src[:, s0:s0 + sn].contiguous()
        r.resize_band(n, r0, r1 - r0, s0, sw, sn * sw, win.data_ptr(), dw, dh * dw, got[:, r0].data_ptr())
    torch.cuda.synchronize()
    assert (got.cpu().numpy() == out).all(), cfg
    sst, dst_st = sw + 4, dw + 8
    pbuf = torch.zeros((n, sh, sst), dtype=torch.uint8, device=DEV)
    pbuf[:, :, :sw] = src
    dbuf = torch.full((n, dh, dst_st), 9, dtype=torch.uint8, device=DEV)
    r.resize_device(n, sst, sh * sst, pbuf.data_ptr(), dst_st, dh * dst_st, dbuf.data_ptr())
    torch.cuda.synchronize()
    assert (dbuf[:, :, :dw].cpu().numpy() == out).all(), cfg
    assert (dbuf[:, :, dw:].cpu().numpy() == 9).all(), (cfg, "wrote past the row")
    dst = torch.zeros((n, dh, dw + 4), dtype=torch.uint8, device=DEV)
    r.resize_device(n, sw, sh * sw, src.data_ptr(), dw + 4, dh * (dw + 4), dst.data_ptr())
    torch.cuda.synchronize()
    assert (dst[:, :, :dw].cpu().numpy() == out).all(), cfg


U23_SHAPES = [
    ("lanczos", 3, 1280, 720, 1920, 1080, 1),    # 720p -> 1080p: three waves per row (x0 of the last clamped)
    ("lanczos", 3, 640, 360, 960, 540, 1),       # two waves per row
    ("lanczos", 3, 160, 100, 240, 150, 1),       # one wave holding both edges
]


@pytest.mark.parametrize("cfg", U23_SHAPES, ids=lambda c: "%s%d_%dx%d" % c[:4])
def test_lanczos_u23_matches_oracle(cfg):
    """Exact 2:3 Lanczos-3 upscale: lanczos_u23_kernel on every row and column (masked border rows
    and columns divided in the kernel); equal to the oracle on noise, flat and half-flat frames;
    with option u23 = 0 (walker alone), in band splits and lane counts, in row bands through their
    source windows (odd band edges), with padded strides (u23 again) and a destination stride that
    is not 4-byte aligned (walker / tile)."""
    m, d, sw, sh, dw, dh, px = cfg
    n = 3
    frames = _noise_batch(n, sw, sh, 2100)
    frames[1] = 77
    frames[2, :, : sw // 2] = 255
    exp = [ol.run_oracle(m, d, sw, sh, dw, dh, px, frames[f]) for f in range(n)]
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    assert r.describe()["kernel"] == "lanczos_u23"
    src = torch.from_numpy(frames).to(DEV)
    out = r.resize_tensor(src).cpu().numpy()
    for f in range(n):
        bad = np.argwhere(out[f] != exp[f])
        assert bad.size == 0, (cfg, f, bad[:4].tolist())
    w = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    w.set_option("u23", 0)
    assert w.describe()["kernel"] in ("walk", "tile")
    assert (w.resize_tensor(src).cpu().numpy() == out).all()
    for opt, val in (("bands", 1), ("bands", 3), ("bands", 7), ("bands", dh), ("lanes", 5), ("lanes", 62)):
        b = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
        b.set_option(opt, val)
        assert (b.resize_tensor(src).cpu().numpy() == out).all(), (cfg, opt, val)
    got = torch.zeros((n, dh, dw), dtype=torch.uint8, device=DEV)
    cuts = [0, 4, dh // 3 + 1, dh // 2, dh - 5, dh]
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        s0, sn = r.band_src_rows(r0, r1 - r0)
        win = src[:, s0:s0 + sn].contiguous()
        r.resize_band(n, r0, r1 - r0, s0, sw, sn * sw, win.data_ptr(), dw, dh * dw, got[:, r0].data_ptr())
    torch.cuda.synchronize()
    assert (got.cpu().numpy() == out).all(), cfg
    sst, dst_st = sw + 8, dw + 4
    pbuf = torch.zeros((n, sh, sst), dtype=torch.uint8, device=DEV)
    pbuf[:, :, :sw] = src
    dbuf = torch.full((n, dh, dst_st), 9, dtype=torch.uint8, device=DEV)
    r.resize_device(n, sst, sh * sst, pbuf.data_ptr(), dst_st, dh * dst_st, dbuf.data_ptr())
    torch.cuda.synchronize()
    assert (dbuf[:, :, :dw].cpu().numpy() == out).all(), cfg
    assert (dbuf[:, :, dw:].cpu().numpy() == 9).all(), (cfg, "wrote past the row")
    dst = torch.zeros((n, dh, dw + 2), dtype=torch.uint8, device=DEV)
    r.resize_device(n, sw, sh * sw, src.data_ptr(), dw + 2, dh * (dw + 2), dst.data_ptr())
    torch.cuda.synchronize()
    assert (dst[:, :, :dw].cpu().numpy() == out).all(), cfg


L23_SHAPES = [
    ("linear", 0, 1280, 720, 1920, 1080, 1),     # 720p -> 1080p: three waves per row (x0 of the last clamped)
    ("linear", 0, 640, 360, 960, 540, 1),        # two waves per row
    ("linear", 0, 160, 100, 240, 150, 1),        # one wave holding both edges
]


@pytest.mark.parametrize("cfg", L23_SHAPES, ids=lambda c: "%s%d_%dx%d" % c[:4])
def test_linear_u23_matches_oracle(cfg):
    """Exact 2:3 Linear upscale: linear_u23_kernel on every row and column (the replicated borders
    from the clamped source); equal to the oracle on noise, flat and half-flat frames;
    with option l23 = 0 (walker alone), in band splits and lane counts, in row bands through their
    source windows (odd band edges), with padded strides (l23 again) and a destination stride that
    is not 4-byte aligned (walker / tile)."""
    m, d, sw, sh, dw, dh, px = cfg
    n = 3
    frames = _noise_batch(n, sw, sh, 2100)
    frames[1] = 77
    frames[2, :, : sw // 2] = 255
    exp = [ol.run_oracle(m, d, sw, sh, dw, dh, px, frames[f]) for f in range(n)]
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    r.set_option("l23", 1)
    assert r.describe()["kernel"] == "linear_u23"
    src = torch.from_numpy(frames).to(DEV)
    out = r.resize_tensor(src).cpu().numpy()
    for f in range(n):
        bad = np.argwhere(out[f] != exp[f])
        assert bad.size == 0, (cfg, f, bad[:4].tolist())
    w = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    w.set_option("l23", 0)
    assert w.describe()["kernel"] in ("walk", "tile")
    assert (w.resize_tensor(src).cpu().numpy() == out).all()
    for opt, val in (("bands", 1), ("bands", 3), ("bands", 7), ("bands", dh), ("lanes", 5), ("lanes", 62)):
        b = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
        b.set_option("l23", 1)
        b.set_option(opt, val)
        assert (b.resize_tensor(src).cpu().numpy() == out).all(), (cfg, opt, val)
    got = torch.zeros((n, dh, dw), dtype=torch.uint8, device=DEV)
    cuts = [0, 4, dh // 3 + 1, dh // 2, dh - 5, dh]
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        s0, sn = r.band_src_rows(r0, r1 - r0)
        win = src[:, s0:s0 + sn].contiguous()
        r.resize_band(n, r0, r1 - r0, s0, sw, sn * sw, win.data_ptr(), dw, dh * dw, got[:, r0].data_ptr())
    torch.cuda.synchronize()
    assert (got.cpu().numpy() == out).all(), cfg
    sst, dst_st = sw + 8, dw + 4
    pbuf = torch.zeros((n, sh, sst), dtype=torch.uint8, device=DEV)
    pbuf[:, :, :sw] = src
    dbuf = torch.full((n, dh, dst_st), 9, dtype=torch.uint8, device=DEV)
    r.resize_device(n, sst, sh * sst, pbuf.data_ptr(), dst_st, dh * dst_st, dbuf.data_ptr())
    torch.cuda.synchronize()
    assert (dbuf[:, :, :dw].cpu().numpy() == out).all(), cfg
    assert (dbuf[:, :, dw:].cpu().numpy() == 9).all(), (cfg, "wrote past the row")
    dst = torch.zeros((n, dh, dw + 2), dtype=torch.uint8, device=DEV)
    r.resize_device(n, sw, sh * sw, src.data_ptr(), dw + 2, dh * (dw + 2), dst.data_ptr())
    torch.cuda.synchronize()
    assert (dst[:, :, :dw].cpu().numpy() == out).all(), cfg


AREA_INT_SHAPES = [
    (3840, 2160, 1280, 720),   # 4K -> 720p, exactly 3:1 (12 source columns per thread)
    (1920, 1080, 640, 360),
    (1932, 1083, 644, 361),    # odd output height
    (3840, 2160, 640, 720),    # 6:1 x 3:1
    (3840, 2160, 1280, 1080),  # 3:1 x 2:1
    (3840, 2160, 960, 540),    # 4:1 (16 columns per thread)
]


@pytest.mark.parametrize("shape", AREA_INT_SHAPES, ids=lambda s: "%dx%d_%dx%d" % s)
def test_area_int_matches_oracle(shape):
    """Area at integer ratios (area_int_kernel; 3:1 and 6:1 take 12-byte rows per thread) on noise,
    flat and half-flat frames, dense and padded layouts, and the fused YUV420 launch at 3:1."""
    sw, sh, dw, dh = shape
    r = libiqo_amd.AreaResizer(sw, sh, dw, dh)
    assert r.describe()["kernel"] == "area_int"
    frames = _noise_batch(3, sw, sh, 900)
    frames[1] = 255
    frames[2, :, : sw // 2] = 0
    exp = [ol.run_oracle("area", 0, sw, sh, dw, dh, 1, frames[f]) for f in range(3)]
    out = r.resize_tensor(torch.from_numpy(frames).to(DEV)).cpu().numpy()
    for f in range(3):
        assert (out[f] == exp[f]).all(), (shape, f, np.argwhere(out[f] != exp[f])[:4].tolist())
    # padded strides (still 4-byte aligned rows)
    sst, dst_st = sw + 12, dw + 4
    sbuf = torch.zeros((sh, sst), dtype=torch.uint8, device=DEV)
    sbuf[:, :sw] = torch.from_numpy(frames[0]).to(DEV)
    dbuf = torch.zeros((dh, dst_st), dtype=torch.uint8, device=DEV)
    r.resize_device(1, sst, sh * sst, sbuf.data_ptr(), dst_st, dh * dst_st, dbuf.data_ptr())
    torch.cuda.synchronize()
    assert (dbuf[:, :dw].cpu().numpy() == exp[0]).all()
    if sw % 24 == 0 and sh % 2 == 0 and dw % 2 == 0 and dh % 2 == 0 and sw // dw == 3 and sh // dh == 3:
        y = libiqo_amd.Yuv420Resizer("area", 0, sw, sh, dw, dh)
        cw, ch = sw // 2, sh // 2
        planes = [frames[0], ol.gen("noise", cw, ch, 5), ol.gen("noise", cw, ch, 6)]
        src = torch.from_numpy(np.concatenate([p.ravel() for p in planes])[None]).to(DEV)
        o, fused = y.resize_frames(src)
        o = o.cpu().numpy()[0]
        assert fused
        assert (o[: dw * dh].reshape(dh, dw) == exp[0]).all()
        ce = [ol.run_oracle("area", 0, cw, ch, dw // 2, dh // 2, 1, p) for p in planes[1:]]
        cd = (dw // 2) * (dh // 2)
        assert (o[dw * dh: dw * dh + cd].reshape(dh // 2, dw // 2) == ce[0]).all()
        assert (o[dw * dh + cd:].reshape(dh // 2, dw // 2) == ce[1]).all()


D31_SHAPES = [
    ("lanczos", 3, 3840, 2160, 1280, 720, 1),    # 4K -> 720p: six waves per row (x0 of the last clamped)
    ("lanczos", 3, 1920, 1080, 640, 360, 1),
    ("lanczos", 2, 3840, 2160, 1280, 720, 1),    # Lanczos-2 tap structure
    ("lanczos", 3, 1932, 1083, 644, 361, 1),     # odd output height
    ("lanczos", 3, 336, 204, 112, 68, 1),        # one wave holding both edges
    ("lanczos", 2, 192, 96, 64, 32, 1),
]


@pytest.mark.parametrize("cfg", D31_SHAPES, ids=lambda c: "%s%d_%dx%d" % c[:4])
def test_lanczos_d31_matches_oracle(cfg):
    """Exact 3:1 Lanczos-2/3 downscale: lanczos_d31_kernel on every row and column (masked border
    rows and columns divided in the kernel); equal to the oracle on noise, flat and half-flat
    frames; equal to the general kernels (option d31 = 0); in several band splits, lane counts and
    prefetch depths; in row bands through their source windows; with padded strides; and a
    destination stride that is not 4-byte aligned (general kernels)."""
    m, d, sw, sh, dw, dh, px = cfg
    n = 3
    frames = _noise_batch(n, sw, sh, 3100)
    frames[1] = 201
    frames[2, :, : sw // 2] = 255
    exp = [ol.run_oracle(m, d, sw, sh, dw, dh, px, frames[f]) for f in range(n)]
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    assert r.describe()["kernel"] == "lanczos_d31"
    src = torch.from_numpy(frames).to(DEV)
    out = r.resize_tensor(src).cpu().numpy()
    for f in range(n):
        bad = np.argwhere(out[f] != exp[f])
        assert bad.size == 0, (cfg, f, bad[:4].tolist())
    w = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    w.set_option("d31", 0)
    assert w.describe()["kernel"] in ("walk", "tile")
    assert (w.resize_tensor(src).cpu().numpy() == out).all()
    pds = (1, 5) if d == 3 else (1, 2, 4)
    for opt, val in [("bands", 1), ("bands", 3), ("bands", 7), ("bands", dh), ("lanes", 8), ("lanes", 62),
                     ("ratio_alt", 0)] + \
            [("ratio_prefetch", p) for p in pds]:
        b = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
        b.set_option(opt, val)
        assert (b.resize_tensor(src).cpu().numpy() == out).all(), (cfg, opt, val)
    b = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    b.set_option("ratio_prefetch", 3)  # not instantiated for this kernel: rejected, not ignored
    with pytest.raises(libiqo_amd.IqoError):
        b.resize_tensor(src)
    # row bands through their source windows (odd band edges)
    got = torch.zeros((n, dh, dw), dtype=torch.uint8, device=DEV)
    cuts = [0, 3, dh // 3 + 1, dh // 2, dh - 5, dh]
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        s0, sn = r.band_src_rows(r0, r1 - r0)
        win = src[:, s0:s0 + sn].contiguous()
        r.resize_band(n, r0, r1 - r0, s0, sw, sn * sw, win.data_ptr(), dw, dh * dw, got[:, r0].data_ptr())
    torch.cuda.synchronize()
    assert (got.cpu().numpy() == out).all(), cfg
    # padded strides (4-byte aligned rows): d31 again, nothing written past the row
    sst, dst_st = sw + 4, dw + 4
    pbuf = torch.zeros((n, sh, sst), dtype=torch.uint8, device=DEV)
    pbuf[:, :, :sw] = src
    dbuf = torch.full((n, dh, dst_st), 9, dtype=torch.uint8, device=DEV)
    r.resize_device(n, sst, sh * sst, pbuf.data_ptr(), dst_st, dh * dst_st, dbuf.data_ptr())
    torch.cuda.synchronize()
    assert (dbuf[:, :, :dw].cpu().numpy() == out).all(), cfg
    assert (dbuf[:, :, dw:].cpu().numpy() == 9).all(), (cfg, "wrote past the row")
    # destination stride not 4-byte aligned: the general kernels
    dst = torch.zeros((n, dh, dw + 2), dtype=torch.uint8, device=DEV)
    r.resize_device(n, sw, sh * sw, src.data_ptr(), dw + 2, dh * (dw + 2), dst.data_ptr())
    torch.cuda.synchronize()
    assert (dst[:, :, :dw].cpu().numpy() == out).all(), cfg


RYX_SHAPES = [
    ("lanczos", 3, 1920, 1080, 854, 480, 1),     # 1080p -> 480p: rows 9:4, columns 960:427
    ("lanczos", 2, 1920, 1080, 854, 480, 1),
    ("area", 0, 1920, 1080, 854, 480, 1),
    ("lanczos", 3, 1920, 1080, 640, 480, 1),     # columns 3:1 (10 coefficient pairs)
    ("lanczos", 3, 1280, 720, 570, 320, 1),
    ("lanczos", 2, 720, 576, 1000, 256, 1),      # columns upscaled
    ("area", 0, 720, 576, 360, 256, 1),
    ("lanczos", 3, 1920, 1080, 853, 480, 1),     # odd output width: the last column's 1-byte store
    ("area", 0, 1920, 1080, 853, 480, 1),
    ("lanczos", 2, 1280, 720, 569, 320, 1),
    ("lanczos", 3, 3840, 2160, 960, 540, 1),     # 4:1 (14 of 24 row taps, 13 pairs), two 512-thread parts
    ("lanczos", 2, 1920, 1080, 480, 270, 1),     # 4:1 (14 of 16 row taps)
    ("lanczos", 1, 1280, 720, 640, 360, 1),      # 2:1 Lanczos-1
    ("lanczos", 4, 4096, 1080, 2048, 540, 1),    # 2:1 Lanczos-4 .. -9: 12 .. 24 row taps (Lanczos-4 wider
                                                 # than the symmetric streamer's 4 waves per row)
    ("lanczos", 5, 4096, 720, 2048, 360, 1),     # (wider than the symmetric streamer's 4 waves)
    ("lanczos", 6, 1280, 720, 639, 360, 1),
    ("lanczos", 7, 720, 480, 360, 240, 1),
    ("lanczos", 8, 1280, 720, 640, 360, 1),
    ("lanczos", 9, 3840, 2160, 1920, 1080, 1),
    ("lanczos", 3, 640, 480, 1920, 1080, 1),     # 4:9 upscale rows (480 -> 1080), columns 3x
    ("lanczos", 2, 640, 480, 1920, 1080, 1),
    ("lanczos", 3, 720, 480, 1620, 1080, 1),     # columns 2.25x
    ("lanczos", 3, 320, 240, 721, 540, 1),       # odd output width
]


@pytest.mark.parametrize("cfg", RYX_SHAPES, ids=lambda c: "%s%d_%dx%d_%dx%d" % c[:6])
def test_ryx_matches_oracle(cfg):
    """Exact vertical ratio with tabled columns (ryx_kernel): equal to the oracle on noise, flat and
    half-flat frames, to the general kernels (option ryx = 0), over band splits, in row bands through
    their source windows, with padded strides, and with an odd destination stride (general kernels)."""
    m, d, sw, sh, dw, dh, px = cfg
    n = 3
    frames = _noise_batch(n, sw, sh, 4100)
    frames[1] = 99
    frames[2, :, sw // 3:] = 255
    exp = [ol.run_oracle(m, d, sw, sh, dw, dh, px, frames[f]) for f in range(n)]
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    assert r.describe()["kernel"] == "ryx"
    src = torch.from_numpy(frames).to(DEV)
    out = r.resize_tensor(src).cpu().numpy()
    for f in range(n):
        bad = np.argwhere(out[f] != exp[f])
        assert bad.size == 0, (cfg, f, bad[:4].tolist())
    w = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    w.set_option("ryx", 0)
    assert w.describe()["kernel"] in ("walk", "tile", "general")
    assert (w.resize_tensor(src).cpu().numpy() == out).all()
    for val in (1, 3, 7, dh):
        b = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
        b.set_option("bands", val)
        assert (b.resize_tensor(src).cpu().numpy() == out).all(), (cfg, val)
    for split in (0, 2, 3):  # one 8-wave workgroup per row; 2-wave / 1-wave workgroups
        one = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
        one.set_option("ryx_split", split)
        assert (one.resize_tensor(src).cpu().numpy() == out).all(), (cfg, split)
    # one column per thread pair slot (the default takes adjacent column pairs at 9:4 where they fit)
    sep = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)
    sep.set_option("ryx_adj", 0)
    assert (sep.resize_tensor(src).cpu().numpy() == out).all(), (cfg, "ryx_adj 0")
    two = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, px)  # Lanczos-3 upscales: 2 instead of 4 columns per thread
    two.set_option("ryx_cpt", 0)
    assert (two.resize_tensor(src).cpu().numpy() == out).all(), (cfg, "ryx_cpt 0")
    got = torch.zeros((n, dh, dw), dtype=torch.uint8, device=DEV)
    cuts = [0, 3, dh // 3 + 1, dh // 2, dh - 5, dh]
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        s0, sn = r.band_src_rows(r0, r1 - r0)
        win = src[:, s0:s0 + sn].contiguous()
        r.resize_band(n, r0, r1 - r0, s0, sw, sn * sw, win.data_ptr(), dw, dh * dw, got[:, r0].data_ptr())
    torch.cuda.synchronize()
    assert (got.cpu().numpy() == out).all(), cfg
    sst, dst_st = sw + 8, dw + 6
    pbuf = torch.zeros((n, sh, sst), dtype=torch.uint8, device=DEV)
    pbuf[:, :, :sw] = src
    dbuf = torch.full((n, dh, dst_st), 9, dtype=torch.uint8, device=DEV)
    r.resize_device(n, sst, sh * sst, pbuf.data_ptr(), dst_st, dh * dst_st, dbuf.data_ptr())
    torch.cuda.synchronize()
    assert (dbuf[:, :, :dw].cpu().numpy() == out).all(), cfg
    assert (dbuf[:, :, dw:].cpu().numpy() == 9).all(), (cfg, "wrote past the row")
    dst = torch.zeros((n, dh, dw + 1), dtype=torch.uint8, device=DEV)
    r.resize_device(n, sw, sh * sw, src.data_ptr(), dw + 1, dh * (dw + 1), dst.data_ptr())
    torch.cuda.synchronize()
    assert (dst[:, :, :dw].cpu().numpy() == out).all(), cfg
    # the host-pointer entry point (the reference's resize()): the kernel the host picks for the
    # shape and its result, one frame, tight destination rows (odd widths: odd stride)
    assert libiqo_amd.host_kernel_for(m, d, sw, sh, dw, dh, px) == "ryx"
    hout = np.full((dh, dw), 7, np.uint8)
    r.resize(sw, np.ascontiguousarray(frames[0]), dw, hout)
    assert (hout == exp[0]).all(), (cfg, "host path")
    # destination base not 2-byte aligned (1-byte stores)
    obuf = torch.full((n * dh * dw + 1,), 5, dtype=torch.uint8, device=DEV)
    r.resize_device(n, sw, sh * sw, src.data_ptr(), dw, dh * dw, obuf.data_ptr() + 1)
    torch.cuda.synchronize()
    ob = obuf.cpu().numpy()
    assert ob[0] == 5 and (ob[1:].reshape(n, dh, dw) == out).all(), (cfg, "odd base")


LIN2_SHAPES = [
    (3840, 2160, 1920, 1080),   # Linear 4K -> 1080p
    (1920, 1080, 960, 540),
    (640, 480, 320, 240),
    (48, 6, 24, 3),             # two thread groups per row, three rows (both edge rows)
    (32, 4, 16, 2),
]


@pytest.mark.parametrize("cfg", LIN2_SHAPES, ids=lambda c: "%dx%d_%dx%d" % c)
def test_linear_d2_matches_oracle(cfg):
    """Linear at exactly 2:1 (linear_d2_body through IQO_KERNEL_AREA_INT: taps 2i+1, 2i+2, edge
    rows and columns replicated): equal to the oracle on noise, flat and half-flat frames, in row
    bands through their source windows, with padded strides, and through the host-pointer path;
    the I420 plan runs it for all three planes in one launch."""
    sw, sh, dw, dh = cfg
    n = 3
    frames = _noise_batch(n, sw, sh, 2200)
    frames[1] = 201
    frames[2, :, sw // 3:] = 255
    exp = [ol.run_oracle("linear", 0, sw, sh, dw, dh, 1, frames[f]) for f in range(n)]
    r = libiqo_amd.make_resizer("linear", 0, sw, sh, dw, dh, 1)
    assert r.describe()["kernel"] == "area_int"
    assert libiqo_amd.host_kernel_for("linear", 0, sw, sh, dw, dh, 1) == "area_int"
    src = torch.from_numpy(frames).to(DEV)
    out = r.resize_tensor(src).cpu().numpy()
    for f in range(n):
        bad = np.argwhere(out[f] != exp[f])
        assert bad.size == 0, (cfg, f, bad[:4].tolist())
    got = torch.zeros((n, dh, dw), dtype=torch.uint8, device=DEV)
    cuts = sorted(set([0, 1, dh // 3, dh // 2, max(dh - 1, 1), dh]))
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        s0, sn = r.band_src_rows(r0, r1 - r0)
        win = src[:, s0:s0 + sn].contiguous()
        r.resize_band(n, r0, r1 - r0, s0, sw, sn * sw, win.data_ptr(), dw, dh * dw, got[:, r0].data_ptr())
    torch.cuda.synchronize()
    assert (got.cpu().numpy() == out).all(), cfg
    sst, dst_st = sw + 32, dw + 8
    pbuf = torch.zeros((n, sh, sst), dtype=torch.uint8, device=DEV)
    pbuf[:, :, :sw] = src
    dbuf = torch.full((n, dh, dst_st), 9, dtype=torch.uint8, device=DEV)
    r.resize_device(n, sst, sh * sst, pbuf.data_ptr(), dst_st, dh * dst_st, dbuf.data_ptr())
    torch.cuda.synchronize()
    assert (dbuf[:, :, :dw].cpu().numpy() == out).all(), cfg
    assert (dbuf[:, :, dw:].cpu().numpy() == 9).all(), (cfg, "wrote past the row")
    hout = np.zeros((dh, dw), np.uint8)
    r.resize(sw, np.ascontiguousarray(frames[0]), dw, hout)
    assert (hout == exp[0]).all(), (cfg, "host path")
    if sw % 64 == 0 and sw >= 128 and sh % 4 == 0:  # I420: Y and both chroma planes 2:1, one fused launch
        yuv = libiqo_amd.Yuv420Resizer("linear", 0, sw, sh, dw, dh)
        cw, ch = sw // 2, sh // 2
        chroma = [np.ascontiguousarray(frames[f, :ch, :cw]) for f in range(2)]
        packed = np.stack([np.concatenate([frames[f].ravel(), chroma[f].ravel(), chroma[f][::-1].ravel()])
                           for f in range(2)])
        res, fused = yuv.resize_frames(torch.from_numpy(packed).to(DEV))
        torch.cuda.synchronize()
        assert fused == 1
        res = res.cpu().numpy()
        cdw, cdh = dw // 2, dh // 2
        for f in range(2):
            assert (res[f, :dw * dh].reshape(dh, dw) == exp[f]).all()
            for p, plane in ((0, chroma[f]), (1, np.ascontiguousarray(chroma[f][::-1]))):
                ce = ol.run_oracle("linear", 0, cw, ch, cdw, cdh, 1, plane)
                o0 = dw * dh + p * cdw * cdh
                assert (res[f, o0:o0 + cdw * cdh].reshape(cdh, cdw) == ce).all(), (cfg, f, p)


STACK_SHAPES = [
    (2, 640, 480, 320, 240, 7),   # C1: 3 frames per 2-wave workgroup, a partial last group
    (3, 640, 360, 320, 180, 5),   # Lanczos-3 (window period 5)
    (2, 320, 240, 160, 120, 11),  # 5 frames per workgroup
    (3, 1024, 64, 512, 32, 4),    # 64 source lanes: 1 frame would fill a wave; 2 per workgroup
    (2, 208, 30, 104, 15, 13),    # odd output height, 13 lanes per frame (6 frames, border rows)
]


@pytest.mark.parametrize("shape", STACK_SHAPES, ids=lambda s: "L%d_%dx%d_x%d" % (s[0], s[1], s[2], s[5]))
def test_frame_stacked_streamer_matches_oracle(shape):
    """Narrow frames side by side in one workgroup (lanczos_stack_kernel): every frame of a batch
    whose size is not a multiple of the frames per workgroup, noise / flat / half-flat frames, band
    splits; and the same batch through the one-frame-per-workgroup streamer (option stack = 0)."""
    d, sw, sh, dw, dh, n = shape
    frames = _noise_batch(n, sw, sh, 900)
    frames[1] = 255
    frames[2, :, : sw // 2] = 0
    src = torch.from_numpy(frames).to(DEV)
    exp = [ol.run_oracle("lanczos", d, sw, sh, dw, dh, 1, frames[f]) for f in range(n)]
    ref = None
    for stack, bands in ((2, 0), (2, 1), (2, 3), (1, 0), (0, 0)):
        r = libiqo_amd.make_resizer("lanczos", d, sw, sh, dw, dh, 1)
        r.set_option("stack", stack)
        r.set_option("bands", bands)
        out = r.resize_tensor(src).cpu().numpy()
        for f in range(n):
            bad = np.argwhere(out[f] != exp[f])
            assert bad.size == 0, (shape, stack, bands, f, bad[:4].tolist())
        if ref is None:
            ref = out
        assert (out == ref).all()
    # row bands through their source windows, and padded strides, on the stacked streamer
    r = libiqo_amd.make_resizer("lanczos", d, sw, sh, dw, dh, 1)
    r.set_option("stack", 2)
    got = torch.zeros((n, dh, dw), dtype=torch.uint8, device=DEV)
    cuts = sorted({0, 1, dh // 3, dh // 2 + 1, dh - 2, dh})
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        s0, sn = r.band_src_rows(r0, r1 - r0)
        win = src[:, s0:s0 + sn].contiguous()
        r.resize_band(n, r0, r1 - r0, s0, sw, sn * sw, win.data_ptr(), dw, dh * dw, got[:, r0].data_ptr())
    torch.cuda.synchronize()
    assert (got.cpu().numpy() == ref).all(), (shape, "bands")
    sst, dst_st = sw + 32, dw + 16
    pbuf = torch.zeros((n, sh, sst), dtype=torch.uint8, device=DEV)
    pbuf[:, :, :sw] = src
    dbuf = torch.full((n, dh, dst_st), 7, dtype=torch.uint8, device=DEV)
    r.resize_device(n, sst, sh * sst, pbuf.data_ptr(), dst_st, dh * dst_st, dbuf.data_ptr())
    torch.cuda.synchronize()
    assert (dbuf[:, :, :dw].cpu().numpy() == ref).all(), (shape, "padded")
    assert (dbuf[:, :, dw:].cpu().numpy() == 7).all(), (shape, "wrote past the row")


def test_frame_stacked_c1_full_batch():
    """C1's bench batch size through the stacked streamer equals the one-frame-per-workgroup
    streamer on all 4096 frames, and frames 0, 2047, 4095 equal the oracle."""
    sw, sh, dw, dh = 640, 480, 320, 240
    g = torch.Generator(device=DEV)
    g.manual_seed(4096)
    src = torch.randint(0, 256, (4096, sh, sw), dtype=torch.uint8, device=DEV, generator=g)
    r2 = libiqo_amd.LanczosResizer(2, sw, sh, dw, dh)
    r2.set_option("stack", 2)
    a = r2.resize_tensor(src)
    r0 = libiqo_amd.LanczosResizer(2, sw, sh, dw, dh)
    r0.set_option("stack", 0)
    b = r0.resize_tensor(src)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    for f in (0, 2047, 4095):
        exp = ol.run_oracle("lanczos", 2, sw, sh, dw, dh, 1, src[f].cpu().numpy())
        assert (a[f].cpu().numpy() == exp).all(), f


def test_plan_cache_resets_options():
    """A destroyed plan is handed out again for an identical request (iqo_hip_plan_destroy keeps
    it): the second plan must see default options, whatever the first one set."""
    sw, sh, dw, dh = 960, 540, 640, 360  # the walker / d32 family: options change the kernel
    frame = ol.gen("noise", sw, sh, 5)
    exp = ol.run_oracle("lanczos", 3, sw, sh, dw, dh, 1, frame)
    r = libiqo_amd.LanczosResizer(3, sw, sh, dw, dh)
    default_kernel = r.describe()["kernel"]
    default_rows = r.describe()["tile_rows"]
    assert default_rows > 0
    r.set_option("force_general", 1)
    r.set_option("bands", 3)
    r.set_option("tile_rows", 1 if default_rows != 1 else 2)
    assert r.describe()["tile_rows"] != default_rows
    assert r.describe()["kernel"] == "general"
    del r
    import gc
    gc.collect()
    for _ in range(3):
        r2 = libiqo_amd.LanczosResizer(3, sw, sh, dw, dh)
        assert r2.describe()["kernel"] == default_kernel
        assert r2.describe()["tile_rows"] == default_rows
        r2.prepare()  # eager table upload (iqo_hip_plan_prepare): idempotent, then the resize
        assert (_run_host(r2, frame, dw, dh) == exp).all()
        del r2
        gc.collect()


def _fuzz_shapes():
    """Seeded random shapes over the round-4 kernel families and the general kernels."""
    import random
    rng = random.Random(404)
    out = []
    for _ in range(12):
        a, b = rng.randint(4, 60), rng.randint(4, 40)
        out.append(("lanczos", rng.choice((1, 4, 4, 5, 6, 7, 8, 9)), 16 * a, 2 * b + 24, 8 * a, b + 12))  # 2:1
        out.append(("lanczos", rng.choice((2, 3)), 32 * a, 4 * b + 32, 8 * a, b + 8))                   # 4:1
        out.append(("lanczos", rng.choice((2, 3)), 8 * a, b + 8, 24 * a, 3 * b + 24))                   # 3x
        out.append(("linear", 0, 8 * a, b + 2, 24 * a, 3 * b + 6))                                       # 3x
        out.append(("linear", 0, 16 * a, 2 * b + 2, 8 * a, b + 1))                                       # 2:1
        sw = 4 * rng.randint(20, 300)
        out.append(("lanczos", rng.choice((2, 3)), sw, 9 * b + 36, rng.randint(sw // 4, sw), 4 * b + 16))  # 9:4 rows
        out.append((rng.choice(("lanczos", "area", "linear")), rng.randint(2, 4), rng.randint(40, 900),
                    rng.randint(20, 300), rng.randint(30, 1200), rng.randint(16, 400)))                 # general
    return out


@pytest.mark.parametrize("cfg", _fuzz_shapes(), ids=lambda c: "%s%d_%dx%d_%dx%d" % c)
def test_random_shapes_match_oracle(cfg):
    """Seeded random shapes over every kernel family (whichever kernel the plan picks): two frames
    of noise and one half-flat frame, device batch vs the oracle, bit for bit."""
    m, d, sw, sh, dw, dh = cfg
    if m == "linear" and (dw > 2 * sw or dh > 2 * sh) and (dw != 3 * sw or dh != 3 * sh):
        pytest.skip("Linear upsampling beyond 2x reads outside the reference's row (SURVEY 8a quirks)")
    frames = _noise_batch(3, sw, sh, 9000 + sw + sh)
    frames[2, :, sw // 2:] = 255
    exp = [ol.run_oracle(m, d, sw, sh, dw, dh, 1, frames[f]) for f in range(3)]
    r = libiqo_amd.make_resizer(m, d, sw, sh, dw, dh, 1)
    out = r.resize_tensor(torch.from_numpy(frames).to(DEV)).cpu().numpy()
    for f in range(3):
        bad = np.argwhere(out[f] != exp[f])
        assert bad.size == 0, (cfg, r.describe()["kernel"], f, bad[:4].tolist())
