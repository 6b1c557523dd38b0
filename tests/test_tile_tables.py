"""The separable tile kernel's host tables (plan.cpp build_tile_tables), run through a scalar
emulation of tile_kernel's arithmetic (tests/native/tile_emul.cpp, test-only), reproduce the
golden vectors of every shape they cover -- the CPU-side check of the table folding before the
GPU parity tests (tests/test_gpu_parity.py) run the kernel itself.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as ol

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
METHODS = {"lanczos": 0, "area": 1, "linear": 2}


@pytest.fixture(scope="module")
def emul():
    out = os.path.join(HERE, "native", "_build")
    os.makedirs(out, exist_ok=True)
    so = os.path.join(out, "libtile_emul.so")
    srcs = [os.path.join(HERE, "native", "tile_emul.cpp"), os.path.join(ROOT, "libiqo_amd", "csrc", "plan.cpp")]
    if not os.path.exists(so) or any(os.path.getmtime(s) > os.path.getmtime(so) for s in srcs):
        tmp = "%s.%d.tmp" % (so, os.getpid())  # private name + rename: xdist workers may rebuild together
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-ffp-contract=off",
                               "-I" + os.path.join(ROOT, "libiqo_amd", "csrc"), "-o", tmp] + srcs)
        os.replace(tmp, so)
    lib = ctypes.CDLL(so)
    lib.tile_emul.restype = ctypes.c_int
    lib.tile_emul.argtypes = [ctypes.c_int, ctypes.c_uint] + [ctypes.c_int] * 5 + [ctypes.c_void_p, ctypes.c_void_p,
                                                                                  ctypes.POINTER(ctypes.c_int)]
    return lib


def run_emul(lib, method, degree, sw, sh, dw, dh, px, src):
    dst = np.zeros((dh, dw), np.uint8)
    src = np.ascontiguousarray(src)
    np_ = ctypes.c_int(0)
    rc = lib.tile_emul(METHODS[method], degree, sw, sh, dw, dh, px, src.ctypes.data, dst.ctypes.data, ctypes.byref(np_))
    return rc, dst, np_.value


def test_tile_tables_match_golden(emul, golden):
    covered = 0
    for c in golden["cases"]:
        if c["srcW"] * c["srcH"] > 4_000_000 or c["dstW"] * c["dstH"] > 4_000_000:
            continue
        src = ol.gen(c["gen"], c["srcW"], c["srcH"], c["seed"])
        rc, out, _ = run_emul(emul, c["method"], c["degree"], c["srcW"], c["srcH"], c["dstW"], c["dstH"],
                              c["pxScale"], src)
        assert rc in (0, 1), c["id"]
        if rc:
            continue
        want = c["fnv"] if c["ofast_strict_agree"] else c["fnv_strict"]
        assert "%016x" % ol.fnv1a64(out) == want, c["id"]
        covered += 1
    assert covered > 300


@pytest.mark.parametrize("shape", [
    ("lanczos", 3, 1920, 1080, 1280, 720, 1),
    ("lanczos", 3, 960, 540, 1920, 1080, 1),
    ("lanczos", 9, 404, 300, 1000, 100, 1),
    ("lanczos", 2, 1000, 700, 999, 701, 2),
    ("area", 0, 1920, 1080, 1280, 720, 1),
    ("area", 0, 1004, 300, 333, 301, 1),
    ("linear", 0, 640, 360, 1920, 1080, 1),
    ("linear", 0, 1920, 1080, 1277, 719, 1),
    ("lanczos", 1, 64, 64, 64, 31, 1),      # identity columns
    ("lanczos", 3, 8, 9, 3, 200, 1),        # tiny source
])
def test_tile_tables_match_oracle(emul, shape):
    m, d, sw, sh, dw, dh, px = shape
    src = ol.gen("noise", sw, sh, 7)
    rc, out, _ = run_emul(emul, m, d, sw, sh, dw, dh, px, src)
    assert rc == 0
    exp = ol.run_oracle(m, d, sw, sh, dw, dh, px, src)
    bad = np.argwhere(out != exp)
    assert bad.size == 0, bad[:5].tolist()
