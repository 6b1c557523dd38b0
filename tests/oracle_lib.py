"""ctypes access to the oracle (test infrastructure only).

`liboracle.so` is the C restatement of libiqo's Generic resizers (oracle/iqo_oracle.c);
`oracle/_ref/libiqo_ref*.so` are the reference's own Generic TUs compiled in place by
oracle/Makefile (present only where /root/reference was available at build time).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
REF_DIR = os.path.join(ORACLE_DIR, "_ref")

METHODS = {"lanczos": 0, "area": 1, "linear": 2}

_c_sz = ctypes.c_size_t
_u8p = ctypes.POINTER(ctypes.c_uint8)


def _ptr(a):
    return a.ctypes.data_as(_u8p)


def _load(path):
    return ctypes.CDLL(path)


_oracle = None


def oracle():
    global _oracle
    if _oracle is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"])
        lib = _load(path)
        lib.iqo_oracle_run.restype = ctypes.c_int
        lib.iqo_oracle_run.argtypes = [ctypes.c_int, ctypes.c_uint, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz,
                                       _c_sz, _u8p, _c_sz, _u8p]
        lib.iqo_oracle_new.restype = ctypes.c_void_p
        lib.iqo_oracle_new.argtypes = [ctypes.c_int, ctypes.c_uint, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz]
        lib.iqo_oracle_free.argtypes = [ctypes.c_void_p]
        lib.iqo_oracle_table.restype = ctypes.c_int
        lib.iqo_oracle_table.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                         ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int32), _c_sz]
        lib.iqo_oracle_run_batch.restype = ctypes.c_double
        lib.iqo_oracle_run_batch.argtypes = [ctypes.c_int, ctypes.c_uint, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz,
                                             _c_sz, _c_sz, _c_sz, _u8p, _c_sz, _c_sz, _u8p, ctypes.c_int]
        lib.iqo_gen_g1.argtypes = [_u8p, _c_sz, _c_sz, _c_sz]
        lib.iqo_gen_mt19937.argtypes = [_u8p, _c_sz, ctypes.c_uint32]
        lib.iqo_gen_splitmix.argtypes = [_u8p, _c_sz, ctypes.c_uint64]
        lib.iqo_fnv1a64.restype = ctypes.c_uint64
        lib.iqo_fnv1a64.argtypes = [_u8p, _c_sz, _c_sz, _c_sz]
        _oracle = lib
    return _oracle


_ref = {}


def ref_available():
    return os.path.exists(os.path.join(REF_DIR, "libiqo_ref.so"))


def ref(strict=False):
    key = "strict" if strict else "rel"
    if key not in _ref:
        lib = _load(os.path.join(REF_DIR, "libiqo_ref_strict.so" if strict else "libiqo_ref.so"))
        lib.iqo_ref_run.restype = ctypes.c_int
        lib.iqo_ref_run.argtypes = [ctypes.c_int, ctypes.c_uint, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz,
                                    _c_sz, _u8p, _c_sz, _u8p]
        lib.iqo_ref_run_batch.restype = ctypes.c_double
        lib.iqo_ref_run_batch.argtypes = [ctypes.c_int, ctypes.c_uint, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz,
                                          _c_sz, _c_sz, _c_sz, _u8p, _c_sz, _c_sz, _u8p, ctypes.c_int]
        _ref[key] = lib
    return _ref[key]


def ref_cpu_available():
    return os.path.exists(os.path.join(REF_DIR, "libiqo_ref_cpu.so"))


def ref_cpu():
    """The reference's whole CPU library (CPUID dispatch + OpenMP; oracle/ref_cpu_harness.cpp):
    a SPEED baseline only -- its SIMD paths are f32 and not bit-exact with Generic.

    libgomp reads OMP_WAIT_POLICY when it loads: passive waiting is set first, since spinning
    OpenMP threads on a CPU-quota'd host (the GPU box: 16 CPUs of quota in a 256-CPU affinity
    mask) or on shared vCPUs stall each other (measured: 8 active-spin threads 13x slower than
    one thread in the build container; passive 4.7x faster)."""
    if "cpu" not in _ref:
        os.environ.setdefault("OMP_WAIT_POLICY", "passive")
        lib = _load(os.path.join(REF_DIR, "libiqo_ref_cpu.so"))
        lib.iqo_refcpu_arch.restype = ctypes.c_char_p
        for f in ("iqo_refcpu_run_rows", "iqo_refcpu_run_frames"):
            fn = getattr(lib, f)
            fn.restype = ctypes.c_double
            fn.argtypes = [ctypes.c_int, ctypes.c_uint, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz,
                           _u8p, _c_sz, _c_sz, _u8p, ctypes.c_int]
        lib.iqo_refcpu_bench_yuv420.restype = ctypes.c_double
        lib.iqo_refcpu_bench_yuv420.argtypes = [ctypes.c_int, ctypes.c_uint, _c_sz, _c_sz, _c_sz, _c_sz, ctypes.c_int,
                                                ctypes.c_int, _u8p, _u8p, _u8p, _c_sz, _c_sz, _u8p, _u8p, _u8p,
                                                _c_sz, _c_sz]
        _ref["cpu"] = lib
    return _ref["cpu"]


def host_cpus():
    """(affinity CPUs, cgroup CPU quota or None, usable CPUs = min of the two)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(p)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    return aff, quota, usable


def ref_tables_lib(strict=False):
    key = "tstrict" if strict else "trel"
    if key not in _ref:
        lib = _load(os.path.join(REF_DIR, "libiqo_ref_tables_strict.so" if strict else "libiqo_ref_tables.so"))
        lib.iqo_ref_tables.restype = ctypes.c_int
        lib.iqo_ref_tables.argtypes = [ctypes.c_int, ctypes.c_uint, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                       ctypes.POINTER(ctypes.c_int32), _c_sz]
        _ref[key] = lib
    return _ref[key]


# ----------------------------------------------------------------------------- generators

def gen(kind, w, h, seed=0, st=None):
    """Input generators (definitions shared with the C oracle and the GPU smoke/bench)."""
    st = st or w
    buf = np.zeros((h, st), dtype=np.uint8)
    if kind == "g1":
        i = (np.arange(h, dtype=np.uint64)[:, None] * w + np.arange(w, dtype=np.uint64)[None, :])
        buf[:, :w] = ((i.astype(np.uint32) * np.uint32(2654435761)) >> np.uint32(24)).astype(np.uint8)
    elif kind == "noise":
        buf[:, :w] = splitmix_bytes(w * h, seed).reshape(h, w)
    elif kind == "mt19937":
        tmp = np.zeros(w * h, dtype=np.uint8)
        oracle().iqo_gen_mt19937(_ptr(tmp), w * h, seed)
        buf[:, :w] = tmp.reshape(h, w)
    elif kind == "flat0":
        pass
    elif kind == "flat255":
        buf[:, :w] = 255
    elif kind == "checker":
        yy, xx = np.mgrid[0:h, 0:w]
        buf[:, :w] = (((xx + yy) & 1) * 255).astype(np.uint8)
    else:
        raise ValueError(kind)
    return buf


def splitmix_bytes(n, seed):
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return (z >> np.uint64(56)).astype(np.uint8)


def fnv1a64(arr2d):
    a = np.ascontiguousarray(arr2d)
    return int(oracle().iqo_fnv1a64(_ptr(a), a.shape[1], a.shape[0], a.shape[1]))


# ----------------------------------------------------------------------------- runners

def run_oracle(method, degree, sw, sh, dw, dh, px, src, dst_st=None):
    src = np.ascontiguousarray(src)
    dst_st = dst_st or dw
    dst = np.zeros((dh, dst_st), dtype=np.uint8)
    rc = oracle().iqo_oracle_run(METHODS[method], degree, sw, sh, dw, dh, px, src.shape[1], _ptr(src), dst_st, _ptr(dst))
    assert rc == 0
    return dst[:, :dw]


def run_ref(method, degree, sw, sh, dw, dh, px, src, strict=False):
    src = np.ascontiguousarray(src)
    dst = np.zeros((dh, dw), dtype=np.uint8)
    rc = ref(strict).iqo_ref_run(METHODS[method], degree, sw, sh, dw, dh, px, src.shape[1], _ptr(src), dw, _ptr(dst))
    assert rc == 0
    return dst


def oracle_tables(method, degree, sw, sh, dw, dh, px, axis):
    lib = oracle()
    h = lib.iqo_oracle_new(METHODS[method], degree, sw, sh, dw, dh, px)
    assert h
    try:
        nt, npz = ctypes.c_int(), ctypes.c_int()
        total = lib.iqo_oracle_table(h, axis, ctypes.byref(nt), ctypes.byref(npz), None, 0)
        buf = (ctypes.c_int32 * total)()
        lib.iqo_oracle_table(h, axis, ctypes.byref(nt), ctypes.byref(npz), buf, total)
        return np.array(buf[:], dtype=np.int32).reshape(npz.value, nt.value)
    finally:
        lib.iqo_oracle_free(h)


def ref_tables(method, degree, sw, sh, dw, dh, px, axis, strict=False):
    lib = ref_tables_lib(strict)
    nt, npz = ctypes.c_int(), ctypes.c_int()
    total = lib.iqo_ref_tables(METHODS[method], degree, sw, sh, dw, dh, px, axis, ctypes.byref(nt), ctypes.byref(npz), None, 0)
    buf = (ctypes.c_int32 * total)()
    lib.iqo_ref_tables(METHODS[method], degree, sw, sh, dw, dh, px, axis, ctypes.byref(nt), ctypes.byref(npz), buf, total)
    return np.array(buf[:], dtype=np.int32).reshape(npz.value, nt.value)
