"""AddressSanitizer + UBSan over the product's host code (the reference's
Debug build runs ASan, CMakeLists.txt:47-48).  VERDICT r05 missing 2: plan.cpp builds every table,
row / column record, band window and ryg / ryx record the kernels index with, and cpu_generic.cpp
is the drop-in fallback; neither had run under a sanitizer.

tests/native/asan.mk builds, with -fsanitize=address,undefined -fno-sanitize-recover=all:
  * dropin_cpu_asan: the drop-in classes (resizers.cpp) on their CPU backend (cpu_generic.cpp,
    plan.cpp) with the device side of the C ABI stubbed as "no device" (asan_nodevice.cpp);
  * host_tables_asan: every plan.cpp builder, band_src_rows over random cuts, and the scalar
    emulations of the kernels' table reads (ratio_emul.cpp incl. ryg, tile_emul.cpp).
Both must exit 0 (any report aborts), and the drop-in outputs must equal the golden vectors."""
import os
import random
import subprocess

import numpy as np
import pytest

import oracle_lib as ol

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(HERE, "native", "_build", "asan")
METHOD = {"lanczos": 0, "area": 1, "linear": 2}
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
ENV.pop("IQO_REQUIRE_HIP", None)
ENV.pop("LD_PRELOAD", None)  # (the sanitizer runtime must come first in the link order)


@pytest.fixture(scope="module")
def asan_bins():
    subprocess.check_call(["make", "-s", "-f", os.path.join(HERE, "native", "asan.mk"), "-j8"], cwd=ROOT)
    return os.path.join(OUT, "dropin_cpu_asan"), os.path.join(OUT, "host_tables_asan")


def _run(exe, text, timeout):
    r = subprocess.run([exe], input=text, capture_output=True, text=True, env=ENV, timeout=timeout)
    assert r.returncode == 0, (exe, r.returncode, r.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, r.stderr[-4000:]
    return r.stdout


def test_dropin_cpu_backend_under_asan(asan_bins, golden, tmp_path):
    """Every golden case (the >4 MP ones once per shape) through the drop-in classes' CPU backend,
    sanitized, bit-exact against the reference's hashes."""
    cases, seen_big = [], set()
    for c in golden["cases"]:
        big = c["srcW"] * c["srcH"] > 4_000_000 or c["dstW"] * c["dstH"] > 4_000_000
        key = (c["method"], c["degree"], c["srcW"], c["srcH"], c["dstW"], c["dstH"], c["pxScale"])
        if big and key in seen_big:
            continue
        seen_big.add(key) if big else None
        cases.append(c)
    lines = []
    for i, c in enumerate(cases):
        inp, out = tmp_path / ("in%d.raw" % i), tmp_path / ("out%d.raw" % i)
        ol.gen(c["gen"], c["srcW"], c["srcH"], c["seed"]).tofile(inp)
        lines.append("%d %d %d %d %d %d %d %s %s" % (METHOD[c["method"]], c["degree"], c["srcW"], c["srcH"], c["dstW"],
                                                   c["dstH"], c["pxScale"], inp, out))
    got = _run(asan_bins[0], "\n".join(lines) + "\n", 1500)
    assert got.split() == ["cases", str(len(cases)), "hip", "0", "cpu", str(len(cases))], got
    bad = []
    for i, c in enumerate(cases):
        o = np.fromfile(tmp_path / ("out%d.raw" % i), dtype=np.uint8).reshape(c["dstH"], c["dstW"])
        if "%016x" % ol.fnv1a64(o) != (c["fnv"] if c["ofast_strict_agree"] else c["fnv_strict"]):
            bad.append(c["id"])
    assert not bad, bad[:10]


def _table_shapes(golden):
    shapes = {(METHOD[c["method"]], c["degree"], c["srcW"], c["srcH"], c["dstW"], c["dstH"], c["pxScale"])
              for c in golden["cases"]}
    import test_ratio_tables as rt
    shapes |= {(METHOD[m], d, sw, sh, dw, dh, 1) for _, m, d, sw, sh, dw, dh in rt._shapes()}
    import bench
    shapes |= {(METHOD[c[0]], c[1], c[2], c[3], c[4], c[5], c[6]) for c in bench.CONFIGS.values()}
    rng = random.Random(606)
    for _ in range(120):  # random ratios, every method, both pxScales, odd sizes
        m = rng.choice((0, 1, 2))
        sw, sh = rng.randint(8, 1500), rng.randint(4, 900)
        f = rng.choice((0.26, 0.34, 0.5, 0.7, 0.9, 1.3, 2.0, 2.25, 3.0))
        shapes.add((m, rng.randint(1, 9) if m == 0 else 0, sw, sh, max(1, int(sw * f)), max(1, int(sh * f)),
                    rng.choice((1, 2)) if m == 0 else 1))
    return sorted(shapes)


def test_host_tables_under_asan(asan_bins, golden):
    shapes = _table_shapes(golden)
    got = _run(asan_bins[1], "\n".join(" ".join(map(str, s)) for s in shapes) + "\n", 1500)
    counts = dict((ln.split()[0], int(ln.split()[1])) for ln in got.strip().splitlines())
    assert counts["shapes"] == len(shapes)
    # every builder and every emulated kernel family accepted some shapes (the run exercised them)
    for k in ("build_plan", "build_tile_tables", "build_walk_tables", "build_up2", "build_d32", "build_d31",
              "build_ryx", "build_ryg", "build_u23", "build_l23", "build_a32", "band_src_rows", "emul_lanczos_d32",
              "emul_lanczos_up2", "emul_area_d32", "emul_lanczos_u23", "emul_linear_u23", "emul_lanczos_d31",
              "emul_ryx", "emul_linear_d2", "emul_linear_up2", "emul_ryg", "emul_tile"):
        assert counts.get(k, 0) > 0, (k, counts)
    print("host_tables_asan:", counts)
