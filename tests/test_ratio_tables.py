"""The exact-ratio kernels' host tables (plan.cpp build_d32 / build_up2 / build_a32), run through a
scalar emulation of the kernels' arithmetic (tests/native/ratio_emul.cpp, test-only): zero rows and
columns outside the image, magic-number border divisions, the edge-lane rewrite.  Checked against
the golden vectors they cover and against the oracle on random exact 3:2 and 2x shapes -- the
CPU-side check before the GPU parity tests (tests/test_gpu_parity.py) run the kernels themselves.
"""
import ctypes
import os
import random
import subprocess

import numpy as np
import pytest

import oracle_lib as ol

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
METHODS = {"lanczos": 0, "area": 1, "linear": 2}
KINDS = {"lanczos_d32": 0, "lanczos_up2": 1, "area_d32": 2, "lanczos_u23": 3, "linear_u23": 4, "lanczos_d31": 5, "ryx": 6, "linear_up": 8,
         "linear_d2": 7, "ryg": 9, "ryu": 10, "ryu_run": 11, "ryp": 10}


@pytest.fixture(scope="module")
def emul():
    out = os.path.join(HERE, "native", "_build")
    os.makedirs(out, exist_ok=True)
    so = os.path.join(out, "libratio_emul.so")
    srcs = [os.path.join(HERE, "native", "ratio_emul.cpp"), os.path.join(ROOT, "libiqo_amd", "csrc", "plan.cpp")]
    if not os.path.exists(so) or any(os.path.getmtime(s) > os.path.getmtime(so) for s in srcs):
        # build under a private name and rename: pytest-xdist workers may rebuild at the same time
        tmp = "%s.%d.tmp" % (so, os.getpid())
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-ffp-contract=off",
                               "-I" + os.path.join(ROOT, "libiqo_amd", "csrc"), "-o", tmp] + srcs)
        os.replace(tmp, so)
    lib = ctypes.CDLL(so)
    lib.ratio_emul.restype = ctypes.c_int
    lib.ratio_emul.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint] + [ctypes.c_int] * 5 + [ctypes.c_void_p] * 2
    return lib


def run_emul(lib, kind, method, degree, sw, sh, dw, dh, px, src):
    dst = np.zeros((dh, dw), np.uint8)
    src = np.ascontiguousarray(src)
    rc = lib.ratio_emul(KINDS[kind], METHODS[method], degree, sw, sh, dw, dh, px, src.ctypes.data, dst.ctypes.data)
    return rc, dst


def test_ratio_tables_match_golden(emul, golden):
    covered = 0
    for c in golden["cases"]:
        if c["srcW"] * c["srcH"] > 4_000_000 or c["dstW"] * c["dstH"] > 4_000_000:
            continue
        src = ol.gen(c["gen"], c["srcW"], c["srcH"], c["seed"])
        for kind in KINDS:
            rc, out = run_emul(emul, kind, c["method"], c["degree"], c["srcW"], c["srcH"], c["dstW"], c["dstH"],
                               c["pxScale"], src)
            assert rc in (0, 1), (c["id"], kind)
            if rc:
                continue
            want = c["fnv"] if c["ofast_strict_agree"] else c["fnv_strict"]
            assert "%016x" % ol.fnv1a64(out) == want, (c["id"], kind)
            covered += 1
    assert covered >= 3


def _shapes():
    rng = random.Random(32)
    out = [("lanczos_d32", "lanczos", 3, 1920, 1080, 1280, 720), ("lanczos_d32", "lanczos", 2, 1920, 1080, 1280, 720),
           ("lanczos_u23", "lanczos", 3, 1280, 720, 1920, 1080),
           ("linear_u23", "linear", 0, 1280, 720, 1920, 1080),
           ("lanczos_up2", "lanczos", 3, 1920, 1080, 3840, 2160),
           ("area_d32", "area", 0, 1920, 1080, 1280, 720), ("lanczos_up2", "lanczos", 2, 200, 60, 400, 120),
           ("lanczos_d31", "lanczos", 3, 3840, 2160, 1280, 720), ("lanczos_d31", "lanczos", 2, 1920, 1080, 640, 360),
           ("lanczos_d31", "lanczos", 3, 1932, 1083, 644, 361),
           ("ryx", "lanczos", 3, 1920, 1080, 854, 480), ("ryx", "lanczos", 2, 1920, 1080, 854, 480),
           ("ryx", "area", 0, 1920, 1080, 854, 480), ("ryx", "lanczos", 3, 1920, 1080, 640, 480),
           ("ryx", "lanczos", 3, 1280, 720, 570, 320), ("ryx", "area", 0, 720, 576, 360, 256),
           ("ryx", "lanczos", 3, 1920, 1080, 853, 480), ("ryx", "area", 0, 1920, 1080, 853, 480),  # odd widths
           ("linear_d2", "linear", 0, 3840, 2160, 1920, 1080), ("linear_d2", "linear", 0, 640, 480, 320, 240),
           ("linear_d2", "linear", 0, 32, 4, 16, 2), ("linear_d2", "linear", 0, 48, 6, 24, 3),
           ("lanczos_up2", "lanczos", 3, 1280, 720, 3840, 2160), ("lanczos_up2", "lanczos", 2, 640, 360, 1920, 1080),  # 3x
           ("lanczos_up2", "lanczos", 3, 16, 4, 48, 12), ("lanczos_up2", "lanczos", 2, 16, 5, 48, 15),
           ("linear_up", "linear", 0, 1280, 720, 3840, 2160), ("linear_up", "linear", 0, 1920, 1080, 3840, 2160),
           ("linear_up", "linear", 0, 8, 2, 24, 6), ("linear_up", "linear", 0, 16, 3, 32, 6),
           ("ryx", "lanczos", 3, 3840, 2160, 960, 540), ("ryx", "lanczos", 2, 1920, 1080, 480, 270),  # 4:1
           ("ryx", "lanczos", 4, 2560, 1440, 640, 360), ("ryx", "lanczos", 4, 1000, 600, 250, 150),  # 4:1 Lanczos-4
           ("ryx", "lanczos", 1, 640, 480, 320, 240), ("ryx", "lanczos", 4, 1920, 1080, 960, 540),   # 2:1
           ("ryx", "lanczos", 5, 640, 360, 320, 180), ("ryx", "lanczos", 6, 640, 360, 320, 180),
           ("ryx", "lanczos", 7, 720, 480, 360, 240), ("ryx", "lanczos", 8, 640, 360, 320, 180),
           ("ryx", "lanczos", 9, 3840, 2160, 1920, 1080), ("ryx", "lanczos", 9, 5120, 64, 2560, 32),
           ("ryx", "lanczos", 3, 640, 480, 1920, 1080), ("ryx", "lanczos", 2, 640, 480, 1920, 1080),  # 4:9 up
           ("ryx", "lanczos", 3, 720, 480, 1620, 1080), ("ryx", "lanczos", 3, 320, 240, 720, 540),
           ("ryx", "lanczos", 2, 64, 16, 100, 36),
           # general rows (ryg): 1..2:1, 2..3:1 (NL 3), 3..4:1 (NL 4), upscale rows (NL 1), Area / Linear
           ("ryg", "lanczos", 3, 1920, 1080, 1366, 768), ("ryg", "area", 0, 1920, 1080, 1366, 768),
           ("ryg", "linear", 0, 1920, 1080, 1366, 768), ("ryg", "lanczos", 2, 1920, 1080, 1024, 576),
           ("ryg", "lanczos", 3, 1024, 576, 1920, 1080), ("ryg", "lanczos", 3, 1366, 768, 1920, 1080),
           ("ryg", "lanczos", 3, 3840, 2160, 1366, 768), ("ryg", "lanczos", 3, 3840, 2160, 1024, 576),
           ("ryg", "lanczos", 4, 3840, 2160, 1366, 768), ("ryg", "lanczos", 5, 1920, 1080, 1366, 768),  # round 6
           ("ryg", "lanczos", 4, 3840, 2160, 1024, 576), ("ryg", "lanczos", 4, 1920, 1080, 512, 288),
           ("ryg", "lanczos", 6, 1920, 1080, 1366, 768), ("ryg", "lanczos", 5, 1920, 1080, 854, 600),
           ("ryg", "lanczos", 5, 3840, 2160, 1366, 768),
           ("ryg", "area", 0, 3840, 2160, 1366, 768), ("ryg", "lanczos", 4, 1024, 576, 1920, 1080),
           ("ryg", "lanczos", 3, 1367, 769, 1920, 1080), ("ryg", "lanczos", 2, 1918, 1078, 1366, 768),
           # general upscale rows by window position (ryu, round 6): 15:8, 45:32, Lanczos-2/4, odd sizes
           ("ryu", "lanczos", 3, 1024, 576, 1920, 1080), ("ryu", "lanczos", 3, 1366, 768, 1920, 1080),
           ("ryu", "lanczos", 2, 1024, 576, 1920, 1080), ("ryu", "lanczos", 4, 1024, 576, 1920, 1080),
           ("ryu", "lanczos", 3, 1367, 769, 1920, 1080), ("ryu", "lanczos", 3, 100, 37, 130, 71),
           ("ryu", "lanczos", 2, 64, 9, 96, 17),
           ("ryu_run", "lanczos", 3, 1024, 576, 1920, 1080), ("ryu_run", "lanczos", 3, 1366, 768, 1920, 1080),
           ("ryu_run", "lanczos", 4, 1024, 576, 1920, 1080), ("ryu_run", "lanczos", 2, 100, 37, 130, 71),
           ("ryu_run", "lanczos", 3, 1367, 769, 1921, 1081),
           # rows that grow by 2 .. 3 (round 6: up to 3 rows per window position)
           ("ryu", "lanczos", 3, 640, 480, 1920, 1080), ("ryu_run", "lanczos", 3, 640, 480, 1920, 1080),
           ("ryu_run", "lanczos", 2, 854, 400, 1920, 1080), ("ryu", "lanczos", 3, 100, 30, 250, 88),
           # downscale rows walked by window position (ryp, round 6): 1..2:1, 2..3:1, 3..4:1, Area, Linear
           ("ryp", "lanczos", 3, 1920, 1080, 1366, 768), ("ryp", "lanczos", 2, 1920, 1080, 1024, 576),
           ("ryp", "lanczos", 3, 3840, 2160, 1366, 768), ("ryp", "lanczos", 3, 3840, 2160, 1024, 576),
           ("ryp", "area", 0, 1920, 1080, 1366, 768), ("ryp", "area", 0, 3840, 2160, 1024, 576),
           ("ryp", "linear", 0, 1920, 1080, 1366, 768), ("ryp", "lanczos", 4, 1918, 1078, 1366, 768),
           ("ryp", "lanczos", 3, 301, 170, 100, 45)]
    for _ in range(6):
        a, b = rng.randint(2, 40), rng.randint(4, 60)
        out.append(("lanczos_d32", "lanczos", 3, 12 * a, 3 * b, 8 * a, 2 * b))
        out.append(("lanczos_d32", "lanczos", 2, 12 * a, 3 * b, 8 * a, 2 * b))
        out.append(("lanczos_u23", "lanczos", 3, 8 * a, 2 * b + 8, 12 * a, 3 * b + 12))
        out.append(("linear_u23", "linear", 0, 8 * a, 2 * b, 12 * a, 3 * b))
        out.append(("area_d32", "area", 0, 12 * a, 3 * b, 8 * a, 2 * b))
        out.append(("lanczos_up2", "lanczos", rng.choice((2, 3)), 8 * a, b + 4, 16 * a, 2 * b + 8))
        out.append(("lanczos_up2", "lanczos", rng.choice((2, 3)), 8 * a, b + 4, 24 * a, 3 * b + 12))
        out.append(("lanczos_d31", "lanczos", rng.choice((2, 3)), 12 * a + 48, 3 * b + 24, 4 * a + 16, b + 8))
        sw = 4 * rng.randint(20, 500)
        out.append(("linear_d2", "linear", 0, 16 * a, 2 * b, 8 * a, b))
        f = rng.choice((2, 3))
        out.append(("linear_up", "linear", 0, 8 * a, b, f * 8 * a, f * b))
        out.append(("ryx", rng.choice(("lanczos", "area")), 3, sw, 9 * b + 36,
                    2 * rng.randint(sw // 4 + 1, min(1024, sw - 2) // 2) - rng.randint(0, 1), 4 * b + 16))
        out.append(("ryx", "lanczos", rng.choice((1, 4, 5, 6, 7, 8, 9)), sw, 2 * b + 40, sw // 2, b + 20))
        out.append(("ryx", "lanczos", rng.choice((2, 3)), 4 * sw, 4 * b + 40, sw, b + 10))
        # general rows: a random row ratio in (1, 2), (2, 3) or upscaled, columns by about the same
        hr = rng.choice((1.2, 1.45, 1.8, 2.5, 0.7, 0.55))
        gh = 8 * rng.randint(8, 40)
        out.append(("ryg", rng.choice(("lanczos", "area")) if hr > 1 else "lanczos", rng.choice((2, 3)), sw, gh,
                    max(16, int(sw / hr) & ~1), max(8, int(gh / hr))))
        dh_ = rng.randint(40, 300)  # downscale rows by 1 .. 4 (ryp)
        out.append(("ryp", rng.choice(("lanczos", "area")), rng.choice((2, 3)), sw, int(dh_ * rng.uniform(1.05, 3.4)),
                    max(16, int(sw / rng.uniform(1.05, 2.0)) & ~1), dh_))
        uh = rng.randint(8, 200)  # upscale rows by 1 .. 2 (ryu)
        out.append(("ryu", "lanczos", rng.choice((2, 3, 4)), sw, uh, rng.randint(sw, min(4096, 2 * sw)),
                    rng.randint(uh + 1, 2 * uh)))
        out.append(("ryu_run", "lanczos", rng.choice((2, 3, 4)), sw, uh, rng.randint(sw + 1, min(4096, 2 * sw)),
                    rng.randint(uh + 1, 3 * uh)))
        uw = sw // 2 & ~3  # 4:9 rows, columns upscaled (<= 4 coefficient pairs)
        out.append(("ryx", "lanczos", rng.choice((2, 3)), uw, 4 * b + 16, rng.randint(uw, min(4096, 3 * uw)), 9 * b + 36))
    return out


@pytest.mark.parametrize("cfg", _shapes(), ids=lambda c: "%s_%dx%d" % (c[0], c[3], c[4]))
def test_ratio_tables_match_oracle(emul, cfg):
    kind, m, d, sw, sh, dw, dh = cfg
    for gen, seed in (("noise", 5), ("flat255", 0), ("checker", 0)):
        src = ol.gen(gen, sw, sh, seed)
        rc, out = run_emul(emul, kind, m, d, sw, sh, dw, dh, 1, src)
        if rc == 1 and min(dw, dh) < 16:
            pytest.skip("not eligible for %s" % kind)
        assert rc == 0, (cfg, "not eligible")
        exp = ol.run_oracle(m, d, sw, sh, dw, dh, 1, src)
        bad = np.argwhere(out != exp)
        assert bad.size == 0, (cfg, gen, bad[:4].tolist())
