"""The drop-in classes' CPU backend (no GPU visible): iqo::LanczosResizer / AreaResizer /
LinearResizer, called through the reference's public headers by tests/native/dropin_cpu.cpp,
reproduce every golden vector bit for bit.

This is the reference's own fallback (src/IQOLanczosResizer.cpp:33: Generic when no SIMD
implementation is available) restated on the product side: libiqo_amd/csrc/cpu_generic.cpp runs
the host plan that plan.cpp builds for the GPU.  It never loads anything under oracle/."""
import os
import subprocess

import numpy as np
import pytest

import libiqo_amd
import oracle_lib as ol

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "native", "_build")
METHOD = {"lanczos": 0, "area": 1, "linear": 2}


def _gpu_visible():
    try:
        import torch
        return torch.cuda.is_available()
    except ImportError:
        return False


@pytest.fixture(scope="module")
def driver():
    os.makedirs(BUILD, exist_ok=True)
    exe = os.path.join(BUILD, "dropin_cpu")
    src = os.path.join(ROOT, "tests", "native", "dropin_cpu.cpp")
    if not os.path.exists(exe) or os.path.getmtime(exe) < max(os.path.getmtime(src), os.path.getmtime(libiqo_amd.LIB_PATH)):
        tmp = "%s.%d.tmp" % (exe, os.getpid())  # private name + rename: xdist workers may rebuild together
        subprocess.check_call(["g++", "-O2", "-std=c++11", "-I" + os.path.join(ROOT, "include"), "-o", tmp, src,
                               "-L" + os.path.dirname(libiqo_amd.LIB_PATH), "-liqo_hip",
                               "-Wl,-rpath," + os.path.dirname(libiqo_amd.LIB_PATH), "-Wl,-rpath,/opt/rocm/lib",
                               "-Wl,-rpath-link,/opt/rocm/lib"])
        os.replace(tmp, exe)
    return exe


def test_cpu_backend_matches_every_golden_case(golden, driver, tmp_path):
    if _gpu_visible():
        pytest.skip("a GPU is visible: the drop-in classes take the HIP path (tests/test_gpu_parity.py)")
    cases = golden["cases"]
    lines = []
    for i, c in enumerate(cases):
        src = ol.gen(c["gen"], c["srcW"], c["srcH"], c["seed"])
        inp, out = tmp_path / ("in%d.raw" % i), tmp_path / ("out%d.raw" % i)
        src.tofile(inp)
        lines.append("%d %d %d %d %d %d %d %s %s" % (METHOD[c["method"]], c["degree"], c["srcW"], c["srcH"], c["dstW"],
                                                   c["dstH"], c["pxScale"], inp, out))
    env = dict(os.environ)
    env.pop("IQO_REQUIRE_HIP", None)
    r = subprocess.run([driver], input="\n".join(lines) + "\n", capture_output=True, text=True, env=env, timeout=900)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["cases", str(len(cases)), "hip", "0", "cpu", str(len(cases))], r.stdout
    bad = []
    for i, c in enumerate(cases):
        got = np.fromfile(tmp_path / ("out%d.raw" % i), dtype=np.uint8).reshape(c["dstH"], c["dstW"])
        want = c["fnv"] if c["ofast_strict_agree"] else c["fnv_strict"]
        if "%016x" % ol.fnv1a64(got) != want:
            bad.append(c["id"])
    assert not bad, bad[:10]


def test_require_hip_forbids_the_cpu_backend(driver, tmp_path):
    if _gpu_visible():
        pytest.skip("a GPU is visible")
    src = np.zeros((8, 8), np.uint8)
    src.tofile(tmp_path / "in.raw")
    env = dict(os.environ, IQO_REQUIRE_HIP="1")
    r = subprocess.run([driver], input="0 3 8 8 4 4 1 %s %s\n" % (tmp_path / "in.raw", tmp_path / "out.raw"),
                       capture_output=True, text=True, env=env, timeout=60)
    assert r.returncode != 0 and "LanczosResizer construction failed" in r.stderr


def test_product_never_loads_the_oracle():
    """The CPU backend is product code: nothing in libiqo_amd/ names oracle/ or the reference build."""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "libiqo_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hpp", ".hip", ".h")) or f == "Makefile":
                text = open(os.path.join(dirpath, f), errors="replace").read()
                assert "liboracle" not in text and "oracle/_ref" not in text and "oracle_lib" not in text, f
