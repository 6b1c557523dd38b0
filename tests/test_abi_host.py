"""Boundary + host logic, no GPU: the C-ABI library loads, exports every symbol include/*.h
declares, and the product's host plan (table builder, libiqo_amd/csrc/plan.cpp) reproduces the
reference's quantised tables from tests/golden bit for bit."""
import ctypes
import os
import re
import subprocess

import pytest

import libiqo_amd
import oracle_lib as ol

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions(header):
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(iqo_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = libiqo_amd.lib()
    names = _declared_functions(os.path.join(ROOT, "include", "iqo_hip.h"))
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", libiqo_amd.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(r"\bT %s\b" % n, out), n


def test_library_exports_dropin_cpp_classes():
    out = subprocess.run(["nm", "-DC", "--defined-only", libiqo_amd.LIB_PATH], capture_output=True, text=True).stdout
    for sym in ["iqo::LanczosResizer::LanczosResizer(unsigned int, unsigned long, unsigned long, unsigned long, unsigned long, unsigned long)",
                "iqo::LanczosResizer::resize(unsigned long, unsigned char const*, unsigned long, unsigned char*)",
                "iqo::AreaResizer::AreaResizer(unsigned long, unsigned long, unsigned long, unsigned long)",
                "iqo::AreaResizer::resize(unsigned long, unsigned char const*, unsigned long, unsigned char*)",
                "iqo::LinearResizer::LinearResizer(unsigned long, unsigned long, unsigned long, unsigned long)",
                "iqo::LinearResizer::resize(unsigned long, unsigned char const*, unsigned long, unsigned char*)",
                "iqo::LanczosResizer::~LanczosResizer()"]:
        assert sym in out, sym


def test_version_and_errors():
    lib = libiqo_amd.lib()
    assert b"gfx950" in lib.iqo_hip_version()
    assert lib.iqo_hip_strerror(-1) == b"invalid argument"
    p = ctypes.c_void_p()
    assert lib.iqo_hip_plan_lanczos(3, 0, 10, 5, 5, 1, 0, ctypes.byref(p)) != 0
    assert not p.value


def test_no_gpu_means_no_plan():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    assert libiqo_amd.available() == 0
    with pytest.raises(libiqo_amd.IqoError):
        libiqo_amd.LanczosResizer(3, 64, 48, 32, 24)


def test_host_tables_match_reference_golden(golden):
    n = 0
    for c in golden["cases"]:
        for axis, name in ((0, "tableX"), (1, "tableY")):
            # the product builds tables strict-IEEE, like the reference without -Ofast
            key = name if c[name + "_ofast_strict_agree"] else name + "_strict"
            if key not in c:
                continue
            rows = libiqo_amd.host_tables(c["method"], c["degree"], c["srcW"], c["srcH"], c["dstW"], c["dstH"],
                                          c["pxScale"], axis)
            assert [len(rows), len(rows[0])] == c[name + "_shape"], c["id"]
            assert sum(rows, []) == c[key], (c["id"], name)
            n += 1
    assert n > 800


def test_host_tables_match_oracle_random():
    import random
    rng = random.Random(7)
    for _ in range(300):
        m = rng.choice(["lanczos", "area", "linear"])
        d = rng.randint(1, 9)
        px = rng.choice([1, 2, 3])
        sw, sh = rng.randint(1, 3000), rng.randint(1, 3000)
        dw, dh = rng.randint(1, 3000), rng.randint(1, 3000)
        for axis in (0, 1):
            a = libiqo_amd.host_tables(m, d, sw, sh, dw, dh, px, axis)
            b = ol.oracle_tables(m, d, sw, sh, dw, dh, px, axis).tolist()
            assert a == b, (m, d, sw, sh, dw, dh, px, axis)


@pytest.mark.parametrize("cfg,kernel", [
    (("lanczos", 3, 3840, 2160, 1920, 1080, 1), "lanczos_stream"),
    (("lanczos", 2, 640, 480, 320, 240, 1), "lanczos_stream"),
    (("area", 0, 7680, 4320, 1920, 1080, 1), "area_int"),
    (("linear", 0, 1920, 1080, 3840, 2160, 1), "linear_up2"),
    (("lanczos", 3, 1920, 1080, 3840, 2160, 1), "lanczos_up2"),   # exact 2x Lanczos: register-window streamer
    (("lanczos", 3, 1921, 1080, 3842, 2160, 1), "ryg"),           # 2x rows on an odd width (round 5: ryg reads
                                                                  # rows that are not dword-aligned)
    (("lanczos", 4, 1921, 1080, 3000, 2500, 1), "ryg"),           # Lanczos-4 upscale rows (round 5)
    (("lanczos", 5, 1000, 700, 1500, 1000, 1), "walk"),           # Lanczos-5 upscale (no ryg shape): wave walker
    (("lanczos", 2, 1920, 1080, 1280, 720, 1), "lanczos_d32"),    # exact 3:2 Lanczos-2
    (("lanczos", 4, 1920, 1080, 1280, 720, 1), "ryg"),             # 3:2 Lanczos-4: general rows (1 or 2 apart)
    (("lanczos", 3, 1920, 1080, 1366, 768, 1), "ryg"),             # rows 45:32
    (("area", 0, 1920, 1080, 1366, 768, 1), "ryg"),               # Area general rows (round 5: ryg 0.20 vs walker 0.27 ms)
    (("lanczos", 2, 1920, 1080, 1024, 576, 1), "ryg"),             # rows 15:8
    (("lanczos", 3, 1920, 1080, 900, 500, 1), "ryg"),              # 2.16:1 rows (round 5: ryg, 3 rows per output row)
    (("lanczos", 3, 1920, 1080, 600, 340, 1), "ryg"),              # 3.18:1 rows (4 rows per output row)
    (("lanczos", 3, 1920, 1080, 400, 220, 1), "tile"),             # rows shrink by more than 4: tiles
    (("lanczos", 3, 1280, 720, 1920, 1080, 1), "lanczos_u23"),    # exact 2:3 Lanczos-3 upscale
    (("linear", 0, 1280, 720, 1920, 1080, 1), "linear_u23"),      # exact 2:3 Linear upscale
    (("area", 0, 1920, 1080, 1280, 720, 1), "area_d32"),          # exact 3:2 Area: no window, no halo
    (("lanczos", 3, 1920, 1080, 1280, 720, 1), "lanczos_d32"),    # exact 3:2 Lanczos-3: register window
    (("area", 0, 1921, 1080, 1280, 720, 1), "walk"),             # (odd width: the walker when the rows are
                                                                  # 4-byte aligned, else ryg)
    (("area", 0, 1920, 1080, 1600, 900, 1), "walk"),             # Area / Linear rows shrinking by < 1.4: walker
    (("linear", 0, 1920, 1080, 1280, 720, 1), "walk"),           # Linear 3:2 (two row phases): walker
    (("linear", 0, 1366, 768, 1000, 1000, 1), "walk"),             # Linear upscale rows: walker
    (("linear", 0, 1920, 1080, 1366, 768, 1), "ryg"),              # Linear downscale to 2:1 (round 5)
    (("linear", 0, 1920, 1080, 900, 500, 1), "tile"),              # beyond 2:1 (the reference reads past the row)
    (("lanczos", 3, 13, 9, 5, 40, 1), "tile"),                    # 13 columns: no 256-column strip fits the walker's tables
    (("lanczos", 9, 64, 48, 1000, 900, 1), "tile"),               # 64 work columns per row window: tiles
    (("lanczos", 3, 1920, 1080, 960, 540, 2), "lanczos_stream"),   # pxScale-2 chroma (ring streamer)
    (("lanczos", 9, 4000, 3000, 97, 61, 1), "general"),           # 2 x 9 x 41 taps: beyond NP = 16
    (("lanczos", 3, 7, 100, 3, 50, 1), "general"),                 # narrower than one 8-byte group
    (("lanczos", 3, 1280, 720, 3840, 2160, 1), "lanczos_up2"),     # exact 3x: the same streamer, F = 3
    (("lanczos", 3, 3840, 2160, 960, 540, 1), "ryx"),              # 4:1: 14 of 24 row taps
    (("lanczos", 4, 3840, 2160, 1920, 1080, 1), "lanczos_stream"), # Lanczos-4 2:1: symmetric streamer
    (("lanczos", 4, 4096, 2160, 2048, 1080, 1), "ryx"),            # (> 4 waves per row) and -5 .. -9 2:1
    (("lanczos", 5, 3840, 2160, 1920, 1080, 1), "lanczos_stream"), # Lanczos-5 2:1: 8 edge sums per side
    (("lanczos", 6, 3840, 2160, 1920, 1080, 1), "ryx"),
    (("lanczos", 9, 3840, 2160, 1920, 1080, 1), "ryx"),
    (("lanczos", 3, 640, 480, 1920, 1080, 1), "ryx"),              # 4:9 upscale rows            # (taps beyond the tile tables)
    (("linear", 0, 3840, 2160, 1920, 1080, 1), "area_int"),        # Linear 2:1: linear_d2 (area kind 8)
])
def test_fast_path_selection(cfg, kernel):
    assert libiqo_amd.host_kernel_for(*cfg) == kernel


@pytest.mark.parametrize("tool", ["iqo_resize_yuv420p", "iqo_benchmark"])
def test_cli_tools_usage_without_gpu(tool, tmp_path):
    """The two command-line tools are built against the library and reject bad arguments with
    EINVAL and a usage line before touching the device (reference: sample/resize_yuv420p.cpp:48-55,
    benchmark/benchmark.cpp)."""
    exe = os.path.join(os.path.dirname(libiqo_amd.LIB_PATH), "build", tool)
    assert os.access(exe, os.X_OK), exe
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 22 and "usage:" in r.stdout
    if tool == "iqo_resize_yuv420p":
        r = subprocess.run([exe, "-m", "lanczos0", "-i", str(tmp_path / "a"), "-o", str(tmp_path / "b"),
                            "-iw", "4", "-ih", "4", "-ow", "2", "-oh", "2"], capture_output=True, text=True, timeout=60)
        assert r.returncode == 22 and "invalid method" in r.stdout
