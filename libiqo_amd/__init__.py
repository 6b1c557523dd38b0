"""libiqo_amd -- MI355X-native (gfx950) hot path of libiqo's Lanczos / Area / Linear U8 resize.

Python host mirror of the reference's public interface (include/libiqo/*Resizer.hpp), bound
through ctypes to the C ABI in include/iqo_hip.h (libiqo_amd/libiqo_hip.so).  The classes keep
the reference's names, constructor arguments and `resize(srcSt, src, dstSt, dst)` entry point;
`resize_device` adds the batched, device-resident form used for throughput (pointers may come
from torch tensors -- torch is plumbing here, never part of the computation).

There is no CPU fallback: if the HIP library is missing or no gfx950 device is usable, every
call raises `IqoError`.
"""
import ctypes
import os

__all__ = ["IqoError", "LanczosResizer", "AreaResizer", "LinearResizer", "Yuv420Resizer", "available", "lib",
           "host_tables", "host_kernel_for", "host_band_src_rows", "copy_frames", "ipc_export", "ipc_open",
           "ipc_close", "KERNELS", "COPY_PATHS", "LIB_PATH"]

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# LIBIQO_AMD_LIB selects an alternative build of the same library (A/B experiments only)
LIB_PATH = os.environ.get("LIBIQO_AMD_LIB") or os.path.join(PKG_DIR, "libiqo_hip.so")

KERNELS = {0: "general", 1: "lanczos_stream", 2: "area_int", 3: "linear_up2", 4: "tile", 5: "walk", 6: "lanczos_up2", 7: "lanczos_d32", 8: "area_d32", 9: "lanczos_u23", 10: "linear_u23", 11: "lanczos_d31", 12: "ryx", 13: "ryg"}
_METHODS = {"lanczos": 0, "area": 1, "linear": 2}

_c_sz = ctypes.c_size_t
_vp = ctypes.c_void_p


class IqoError(RuntimeError):
    pass


class PlanDesc(ctypes.Structure):
    _fields_ = [("method", ctypes.c_int), ("device", ctypes.c_int), ("srcW", _c_sz), ("srcH", _c_sz),
                ("dstW", _c_sz), ("dstH", _c_sz), ("tapsX", ctypes.c_int), ("tapsY", ctypes.c_int),
                ("phasesX", ctypes.c_int), ("phasesY", ctypes.c_int), ("kernel", ctypes.c_int),
                ("bandsPerFrame", ctypes.c_int), ("tileRows", ctypes.c_int)]


class IpcHandle(ctypes.Structure):
    """iqo_hip_ipc_handle: hipIpcMemHandle_t bytes + the pointer's offset in its allocation."""
    _fields_ = [("bytes", ctypes.c_ubyte * 64), ("offset", ctypes.c_uint64)]


COPY_PATHS = {0: "same device", 1: "peer DMA (xGMI)", 2: "host staging", 3: "host<->device"}

_lib = None


def lib():
    """Load libiqo_hip.so (raises IqoError if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise IqoError("libiqo_hip.so not built: run `make -C libiqo_amd` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    pp = ctypes.POINTER(_vp)
    L.iqo_hip_available.restype = ctypes.c_int
    L.iqo_hip_plan_lanczos.argtypes = [ctypes.c_uint, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz, ctypes.c_int, pp]
    L.iqo_hip_plan_area.argtypes = [_c_sz, _c_sz, _c_sz, _c_sz, ctypes.c_int, pp]
    L.iqo_hip_plan_linear.argtypes = [_c_sz, _c_sz, _c_sz, _c_sz, ctypes.c_int, pp]
    L.iqo_hip_plan_destroy.argtypes = [_vp]
    L.iqo_hip_plan_destroy.restype = None
    L.iqo_hip_plan_query.argtypes = [_vp, ctypes.POINTER(PlanDesc)]
    L.iqo_hip_plan_prepare.argtypes = [_vp]
    L.iqo_hip_plan_set_option.argtypes = [_vp, ctypes.c_char_p, ctypes.c_long]
    L.iqo_hip_resize.argtypes = [_vp, _c_sz, _vp, _c_sz, _vp]
    L.iqo_hip_resize_device.argtypes = [_vp, _c_sz, _c_sz, _c_sz, _vp, _c_sz, _c_sz, _vp, _vp]
    L.iqo_hip_band_src_rows.argtypes = [_vp, _c_sz, _c_sz, ctypes.POINTER(_c_sz), ctypes.POINTER(_c_sz)]
    L.iqo_hip_resize_band.argtypes = [_vp, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz, _vp, _c_sz, _c_sz, _vp, _vp]
    L.iqo_hip_strerror.restype = ctypes.c_char_p
    L.iqo_hip_strerror.argtypes = [ctypes.c_int]
    L.iqo_hip_version.restype = ctypes.c_char_p
    L.iqo_host_tables.argtypes = [ctypes.c_int, ctypes.c_uint, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                  ctypes.POINTER(ctypes.c_int32), _c_sz]
    L.iqo_host_kernel_for.argtypes = [ctypes.c_int, ctypes.c_uint, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz]
    L.iqo_host_band_src_rows.argtypes = [ctypes.c_int, ctypes.c_uint, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz,
                                         ctypes.POINTER(_c_sz), ctypes.POINTER(_c_sz)]
    L.iqo_hip_plan_yuv420.argtypes = [ctypes.c_int, ctypes.c_uint, _c_sz, _c_sz, _c_sz, _c_sz, ctypes.c_int, pp]
    L.iqo_hip_yuv_plan_destroy.argtypes = [_vp]
    L.iqo_hip_yuv_plan_destroy.restype = None
    L.iqo_hip_yuv_plane.argtypes = [_vp, ctypes.c_int]
    L.iqo_hip_yuv_plane.restype = _vp
    L.iqo_hip_resize_yuv420_device.argtypes = [_vp, _c_sz, _c_sz, _c_sz, _c_sz, _vp, _vp, _vp, _c_sz, _c_sz, _c_sz,
                                               _vp, _vp, _vp, _vp, ctypes.POINTER(ctypes.c_int)]
    L.iqo_hip_resize_yuv420.argtypes = [_vp, _c_sz, _vp, _c_sz, _vp, _vp, _c_sz, _vp, _c_sz, _vp, _vp]
    L.iqo_hip_copy_frames.argtypes = [_vp, ctypes.c_int, _c_sz, _vp, ctypes.c_int, _c_sz, _c_sz, _c_sz, _vp,
                                      ctypes.POINTER(ctypes.c_int)]
    L.iqo_hip_ipc_export.argtypes = [_vp, ctypes.POINTER(IpcHandle)]
    L.iqo_hip_ipc_open.argtypes = [ctypes.POINTER(IpcHandle), ctypes.c_int, ctypes.POINTER(_vp)]
    L.iqo_hip_ipc_close.argtypes = [_vp, ctypes.POINTER(IpcHandle)]
    _lib = L
    return L


def _check(rc, what):
    if rc != 0:
        raise IqoError("%s: %s (%d)" % (what, lib().iqo_hip_strerror(rc).decode(), rc))


def available():
    """Number of usable gfx950 devices."""
    return int(lib().iqo_hip_available())


def copy_frames(dst, dst_device, dst_frame_st, src, src_device, src_frame_st, bytes_per_frame, n_frames,
                stream=None):
    """iqo_hip_copy_frames: n_frames blocks between devices (device < 0 = host).  Returns the
    route taken (COPY_PATHS)."""
    path = ctypes.c_int(-1)
    _check(lib().iqo_hip_copy_frames(_ptr(dst), dst_device, dst_frame_st, _ptr(src), src_device, src_frame_st,
                                     bytes_per_frame, n_frames, _stream_ptr(stream), ctypes.byref(path)),
           "copy_frames")
    return path.value


def ipc_export(ptr):
    """Exportable handle (bytes) of a device buffer for another process (one process per GPU)."""
    h = IpcHandle()
    _check(lib().iqo_hip_ipc_export(_ptr(ptr), ctypes.byref(h)), "ipc_export")
    return bytes(ctypes.string_at(ctypes.addressof(h), ctypes.sizeof(h)))


def ipc_open(handle_bytes, device):
    """Open another process's exported buffer on `device`; returns (address, handle)."""
    h = IpcHandle.from_buffer_copy(handle_bytes)
    p = _vp()
    _check(lib().iqo_hip_ipc_open(ctypes.byref(h), device, ctypes.byref(p)), "ipc_open")
    return p.value, h


def ipc_close(addr, h):
    _check(lib().iqo_hip_ipc_close(addr, ctypes.byref(h)), "ipc_close")


def host_tables(method, degree, srcW, srcH, dstW, dstH, pxScale, axis):
    """Quantised coefficient table (phases x taps) the plan uploads -- host only, no GPU."""
    L = lib()
    nt, npz = ctypes.c_int(), ctypes.c_int()
    total = L.iqo_host_tables(_METHODS[method], degree, srcW, srcH, dstW, dstH, pxScale, axis,
                              ctypes.byref(nt), ctypes.byref(npz), None, 0)
    if total < 0:
        raise IqoError("invalid table request")
    buf = (ctypes.c_int32 * max(1, total))()
    L.iqo_host_tables(_METHODS[method], degree, srcW, srcH, dstW, dstH, pxScale, axis,
                      ctypes.byref(nt), ctypes.byref(npz), buf, total)
    rows = [list(buf[q * nt.value:(q + 1) * nt.value]) for q in range(npz.value)]
    return rows


def host_band_src_rows(method, degree, srcW, srcH, dstW, dstH, pxScale, dstRow0, dstRows):
    """Source-row window (srcRow0, srcRows) read by output rows [dstRow0, dstRow0+dstRows) -- host only."""
    a, b = _c_sz(), _c_sz()
    _check(lib().iqo_host_band_src_rows(_METHODS[method], degree, srcW, srcH, dstW, dstH, pxScale, dstRow0, dstRows,
                                        ctypes.byref(a), ctypes.byref(b)), "host_band_src_rows")
    return a.value, b.value


def host_kernel_for(method, degree, srcW, srcH, dstW, dstH, pxScale=1):
    return KERNELS[lib().iqo_host_kernel_for(_METHODS[method], degree, srcW, srcH, dstW, dstH, pxScale)]


def _ptr(obj):
    """Raw address of a numpy array, a torch tensor or an int."""
    if isinstance(obj, int):
        return obj
    if hasattr(obj, "data_ptr"):
        return obj.data_ptr()
    if hasattr(obj, "ctypes"):
        return obj.ctypes.data
    raise TypeError("expected numpy array, torch tensor or address")


def _stream_ptr(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream  # torch.cuda.Stream on ROCm wraps a hipStream_t


class _Resizer:
    _method = None

    def __init__(self, srcW, srcH, dstW, dstH, device=None):
        self.srcW, self.srcH, self.dstW, self.dstH = int(srcW), int(srcH), int(dstW), int(dstH)
        self.device = 0 if device is None else int(device)
        self._plan = _vp()
        self._make()

    def _make(self):
        raise NotImplementedError

    def __del__(self):
        p = getattr(self, "_plan", None)
        if p and _lib is not None:
            _lib.iqo_hip_plan_destroy(p)
            self._plan = _vp()

    # -- reference entry point (host pointers, byte strides): resize(srcSt, src, dstSt, dst)
    def resize(self, srcSt, src, dstSt, dst):
        _check(lib().iqo_hip_resize(self._plan, srcSt, _ptr(src), dstSt, _ptr(dst)), "resize")

    # -- batched device-resident form (async on `stream`)
    def resize_device(self, nFrames, srcSt, srcFrameSt, src, dstSt, dstFrameSt, dst, stream=None):
        _check(lib().iqo_hip_resize_device(self._plan, nFrames, srcSt, srcFrameSt, _ptr(src), dstSt, dstFrameSt,
                                           _ptr(dst), _stream_ptr(stream)), "resize_device")

    def band_src_rows(self, dstRow0, dstRows):
        a, b = _c_sz(), _c_sz()
        _check(lib().iqo_hip_band_src_rows(self._plan, dstRow0, dstRows, ctypes.byref(a), ctypes.byref(b)),
               "band_src_rows")
        return a.value, b.value

    def resize_band(self, nFrames, dstRow0, dstRows, srcRow0, srcSt, srcFrameSt, src, dstSt, dstFrameSt, dst,
                    stream=None):
        _check(lib().iqo_hip_resize_band(self._plan, nFrames, dstRow0, dstRows, srcRow0, srcSt, srcFrameSt,
                                         _ptr(src), dstSt, dstFrameSt, _ptr(dst), _stream_ptr(stream)),
               "resize_band")

    def set_option(self, key, value):
        _check(lib().iqo_hip_plan_set_option(self._plan, key.encode(), int(value)), "set_option")

    def prepare(self):
        """Upload the device tables now (before graph capture / async-only use)."""
        _check(lib().iqo_hip_plan_prepare(self._plan), "prepare")

    def describe(self):
        d = PlanDesc()
        _check(lib().iqo_hip_plan_query(self._plan, ctypes.byref(d)), "query")
        return {"method": d.method, "device": d.device, "tapsX": d.tapsX, "tapsY": d.tapsY,
                "phasesX": d.phasesX, "phasesY": d.phasesY, "kernel": KERNELS.get(d.kernel, d.kernel),
                "bands": d.bandsPerFrame, "tile_rows": d.tileRows}

    # -- torch convenience: src [F, srcH, srcW] (or [srcH, srcW]) uint8 on the plan's device
    def resize_tensor(self, src, out=None, stream=None):
        import torch
        squeeze = src.dim() == 2
        s = src.unsqueeze(0) if squeeze else src
        if s.dtype != torch.uint8 or not s.is_cuda or s.shape[-2:] != (self.srcH, self.srcW):
            raise IqoError("expected uint8 device tensor [F, %d, %d]" % (self.srcH, self.srcW))
        s = s.contiguous()
        if out is None:
            out = torch.empty((s.shape[0], self.dstH, self.dstW), dtype=torch.uint8, device=s.device)
        o = out.unsqueeze(0) if out.dim() == 2 else out
        if (o.dtype != torch.uint8 or o.device != s.device or tuple(o.shape) != (s.shape[0], self.dstH, self.dstW)
                or o.stride(2) != 1 or o.stride(1) < self.dstW or (o.shape[0] > 1 and o.stride(0) < self.dstH * o.stride(1))):
            raise IqoError("out must be a uint8 tensor [%d, %d, %d] on %s with unit column stride and "
                           "non-overlapping rows and frames" % (s.shape[0], self.dstH, self.dstW, s.device))
        if stream is None:
            stream = torch.cuda.current_stream(s.device)
        self.resize_device(s.shape[0], s.stride(1), s.stride(0), s, o.stride(1), o.stride(0), o, stream)
        return out[0] if squeeze else out


class LanczosResizer(_Resizer):
    """iqo::LanczosResizer(degree, srcW, srcH, dstW, dstH, pxScale=1) -- LanczosResizer.hpp:26-33."""

    def __init__(self, degree, srcW, srcH, dstW, dstH, pxScale=1, device=None):
        self.degree, self.pxScale = int(degree), int(pxScale)
        super().__init__(srcW, srcH, dstW, dstH, device)

    def _make(self):
        _check(lib().iqo_hip_plan_lanczos(self.degree, self.srcW, self.srcH, self.dstW, self.dstH, self.pxScale,
                                          self.device, ctypes.byref(self._plan)), "LanczosResizer")


class AreaResizer(_Resizer):
    """iqo::AreaResizer(srcW, srcH, dstW, dstH) -- AreaResizer.hpp:24-29."""

    def _make(self):
        _check(lib().iqo_hip_plan_area(self.srcW, self.srcH, self.dstW, self.dstH, self.device,
                                       ctypes.byref(self._plan)), "AreaResizer")


class LinearResizer(_Resizer):
    """iqo::LinearResizer(srcW, srcH, dstW, dstH) -- LinearResizer.hpp:24-29."""

    def _make(self):
        _check(lib().iqo_hip_plan_linear(self.srcW, self.srcH, self.dstW, self.dstH, self.device,
                                         ctypes.byref(self._plan)), "LinearResizer")


def make_resizer(method, degree, srcW, srcH, dstW, dstH, pxScale=1, device=None):
    if method == "lanczos":
        return LanczosResizer(degree, srcW, srcH, dstW, dstH, pxScale, device)
    if method == "area":
        return AreaResizer(srcW, srcH, dstW, dstH, device)
    if method == "linear":
        return LinearResizer(srcW, srcH, dstW, dstH, device)
    raise ValueError(method)


class Yuv420Resizer:
    """I420 three-plane resizer: the reference benchmark's workload (benchmark.cpp:131-229), Y at
    full size and U, V at half size with the same method (Lanczos chroma: pxScale 2)."""

    def __init__(self, method, degree, srcW, srcH, dstW, dstH, device=None):
        self.method, self.degree = method, int(degree)
        self.srcW, self.srcH, self.dstW, self.dstH = int(srcW), int(srcH), int(dstW), int(dstH)
        self.device = 0 if device is None else int(device)
        self._plan = _vp()
        _check(lib().iqo_hip_plan_yuv420(_METHODS[method], self.degree, self.srcW, self.srcH, self.dstW, self.dstH,
                                         self.device, ctypes.byref(self._plan)), "Yuv420Resizer")

    def __del__(self):
        p = getattr(self, "_plan", None)
        if p and _lib is not None:
            _lib.iqo_hip_yuv_plan_destroy(p)
            self._plan = _vp()

    def set_option(self, key, value, plane=None):
        for pl in ((0, 1) if plane is None else (plane,)):
            _check(lib().iqo_hip_plan_set_option(lib().iqo_hip_yuv_plane(self._plan, pl), key.encode(), int(value)),
                   "set_option")

    def resize(self, srcStY, srcY, srcStUV, srcU, srcV, dstStY, dstY, dstStUV, dstU, dstV):
        """Host pointers, synchronous."""
        _check(lib().iqo_hip_resize_yuv420(self._plan, srcStY, _ptr(srcY), srcStUV, _ptr(srcU), _ptr(srcV), dstStY,
                                           _ptr(dstY), dstStUV, _ptr(dstU), _ptr(dstV)), "resize_yuv420")

    def resize_device(self, nFrames, srcStY, srcStUV, srcFrameSt, srcY, srcU, srcV, dstStY, dstStUV, dstFrameSt,
                      dstY, dstU, dstV, stream=None):
        """Device-resident batch (async on `stream`); returns True when one launch did all planes."""
        fused = ctypes.c_int(0)
        _check(lib().iqo_hip_resize_yuv420_device(self._plan, nFrames, srcStY, srcStUV, srcFrameSt, _ptr(srcY),
                                                  _ptr(srcU), _ptr(srcV), dstStY, dstStUV, dstFrameSt, _ptr(dstY),
                                                  _ptr(dstU), _ptr(dstV), _stream_ptr(stream), ctypes.byref(fused)),
               "resize_yuv420_device")
        return bool(fused.value)

    def resize_frames(self, src, out=None, stream=None):
        """src: uint8 CUDA tensor [frames, srcH*3/2 * srcW] per frame laid out I420 (Y, then U, then V,
        tightly packed); returns / fills out [frames, dstH*3/2 * dstW].  Returns (out, fused)."""
        import torch
        sw, sh, dw, dh = self.srcW, self.srcH, self.dstW, self.dstH
        cs, cd = (sw // 2) * (sh // 2), (dw // 2) * (dh // 2)
        if (src.dtype != torch.uint8 or not src.is_cuda or src.dim() != 2 or src.shape[1] != sw * sh + 2 * cs
                or not src.is_contiguous()):
            raise IqoError("src must be a contiguous uint8 device tensor [frames, %d]" % (sw * sh + 2 * cs))
        n = src.shape[0]
        if out is None:
            out = torch.empty((n, dw * dh + 2 * cd), dtype=torch.uint8, device=src.device)
        if (out.dtype != torch.uint8 or out.device != src.device or tuple(out.shape) != (n, dw * dh + 2 * cd)
                or not out.is_contiguous()):
            raise IqoError("out must be a contiguous uint8 tensor [%d, %d] on %s" % (n, dw * dh + 2 * cd, src.device))
        b, o = src.data_ptr(), out.data_ptr()
        fused = self.resize_device(n, sw, sw // 2, src.stride(0), b, b + sw * sh, b + sw * sh + cs,
                                   dw, dw // 2, out.stride(0), o, o + dw * dh, o + dw * dh + cd, stream)
        return out, fused
