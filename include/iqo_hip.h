/*
 * iqo_hip.h -- C ABI of the MI355X (gfx950) resize backend for libiqo's hot path.
 *
 * This is the drop-in boundary.  It replaces the per-arch implementation SPI of the reference
 * (the `I*ResizerImpl` interface + `*ResizerImpl_new<Arch>()` factories) with plain C entry
 * points: no C++ or torch types, only pointers, sizes, an opaque plan and an int status.
 *
 *   reference (read-only, /root/reference)                  replaced by
 *   -------------------------------------------------------  ---------------------------------
 *   LanczosResizerImpl_new<Arch>() + init()                  iqo_hip_plan_lanczos()
 *       src/IQOLanczosResizerImpl.hpp:10-29,65-75;
 *       src/IQOLanczosResizerImpl_Generic.cpp:291-339
 *   AreaResizerImpl_new<Arch>() + init()                     iqo_hip_plan_area()
 *       src/IQOAreaResizerImpl.hpp:10-27; src/IQOAreaResizerImpl_Generic.cpp:174-220
 *   LinearResizerImpl_new<Arch>() + init()                   iqo_hip_plan_linear()
 *       src/IQOLinearResizerImpl.hpp:10-27; src/IQOLinearResizerImpl_Generic.cpp:157-191
 *   I*ResizerImpl::resize(srcSt, src, dstSt, dst)            iqo_hip_resize()  (host pointers)
 *       src/IQOLanczosResizerImpl_Generic.cpp:369-454 etc.   iqo_hip_resize_device() (batched,
 *                                                            device pointers, async on a stream)
 *   delete m_Impl  (src/IQOLanczosResizer.cpp:39-42)         iqo_hip_plan_destroy()
 *   HWCap CPUID dispatch (src/IQOHWCap.cpp:32-53)            iqo_hip_available()
 *
 * Semantics: output bytes are identical to the reference's Generic implementation
 * (IQO*ResizerImpl_Generic) for the same inputs.  All functions return IQO_HIP_OK (0) or a
 * negative status; the library never falls back to a CPU path.
 *
 * Threading: a plan may be used from one host thread at a time (like the reference impl, whose
 * work row makes it non-re-entrant, IQOLanczosResizerImpl_Generic.cpp:279); distinct plans are
 * independent.  Device-pointer calls are asynchronous on `stream` (a hipStream_t, or NULL for
 * the default stream).
 */
#ifndef IQO_HIP_H
#define IQO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IQO_HIP_OK 0
#define IQO_HIP_EINVAL (-1)     /* bad argument (zero size, bad degree, null pointer, ...) */
#define IQO_HIP_ENODEV (-2)     /* no gfx950 device / HIP runtime unusable */
#define IQO_HIP_ENOMEM (-3)     /* host or device allocation failed */
#define IQO_HIP_EHIP (-4)       /* a HIP runtime call or kernel launch failed */
#define IQO_HIP_EUNSUP (-5)     /* shape or layout not supported (e.g. > 65535 frames) */

enum { IQO_METHOD_LANCZOS = 0, IQO_METHOD_AREA = 1, IQO_METHOD_LINEAR = 2 };

/* Kernel families a plan can dispatch to (iqo_hip_plan_desc.kernel). */
enum {
    IQO_KERNEL_GENERAL = 0,     /* any shape, any layout: one workgroup per output row (fallback) */
    IQO_KERNEL_LANCZOS_STREAM = 1, /* integer ratio, 1 phase: row-band walker, register window */
    IQO_KERNEL_AREA_INT = 2,    /* integer ratio area */
    IQO_KERNEL_LINEAR_UP2 = 3,  /* exact 2x bilinear upsampling */
    IQO_KERNEL_TILE = 4,        /* general ratios, any layout: separable tiles (TH rows x CT columns) */
    IQO_KERNEL_WALK = 5,        /* general ratios, 4-byte aligned sources: wave walker, per-wave LDS ring */
    IQO_KERNEL_LANCZOS_UP2 = 6, /* exact 2x Lanczos-2/3 upscale: register-window streamer, every row and column in-kernel */
    IQO_KERNEL_LANCZOS_D32 = 7, /* exact 3:2 Lanczos-3 downscale: register-window streamer, borders in-kernel */
    IQO_KERNEL_AREA_D32 = 8,    /* exact 3:2 Area downscale: one wave per strip, no window */
    IQO_KERNEL_LANCZOS_U23 = 9, /* exact 2:3 Lanczos-3 upscale: register-window streamer, borders in-kernel */
    IQO_KERNEL_LINEAR_U23 = 10, /* exact 2:3 Linear upscale: clamped halo, no border code */
    IQO_KERNEL_LANCZOS_D31 = 11, /* exact 3:1 Lanczos-2/3 downscale: register window, symmetric taps, borders in-kernel */
    IQO_KERNEL_RYX = 12,         /* exact vertical ratio (9:4), tabled columns: register window + LDS work row */
    IQO_KERNEL_RYG = 13          /* downscales by 1..2 (e.g. 1080 -> 768 rows), tabled rows and columns: shifting
                                    register window + LDS work row */
};

typedef struct iqo_hip_plan iqo_hip_plan;

typedef struct {
    int method;
    int device;
    size_t srcW, srcH, dstW, dstH;
    int tapsX, tapsY;       /* reference coefficient counts (m_NumCoefsX/Y) */
    int phasesX, phasesY;   /* reference table counts (m_NumTablesX/Y) */
    int kernel;             /* IQO_KERNEL_* used for full frames with aligned layouts */
    int bandsPerFrame;      /* fast-path row bands per frame (tuning) */
    int tileRows;           /* output rows per tile of IQO_KERNEL_TILE (option "tile_rows"; 0 = no tile tables) */
} iqo_hip_plan_desc;

/* Number of usable gfx950 devices (0 when none or the runtime is unusable). */
int iqo_hip_available(void);

/* Plan = coefficient tables + index maps built on the host; the tables a kernel reads from device
 * memory are uploaded to `device` once, on the first launch that needs them.  Destroyed plans are
 * kept in a small process-wide cache (options reset to their defaults) and returned again for an
 * identical request, so constructing a resizer per call, as the reference benchmark does, does not
 * rebuild tables. */
int iqo_hip_plan_lanczos(unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                         size_t pxScale, int device, iqo_hip_plan **out);
int iqo_hip_plan_area(size_t srcW, size_t srcH, size_t dstW, size_t dstH, int device, iqo_hip_plan **out);
int iqo_hip_plan_linear(size_t srcW, size_t srcH, size_t dstW, size_t dstH, int device, iqo_hip_plan **out);
void iqo_hip_plan_destroy(iqo_hip_plan *plan);

int iqo_hip_plan_query(const iqo_hip_plan *plan, iqo_hip_plan_desc *desc);

/* Upload the plan's device tables now (one allocation + one blocking copy on the plan's device)
 * instead of inside the first resize call that needs them.  Call it before capturing resize calls
 * into a hipGraph or issuing them on a stream that must not synchronise with the host: the lazy
 * upload would otherwise do a hipMalloc and a blocking null-stream copy inside that first call
 * (and report IQO_HIP_ENOMEM there).  Plans whose kernels take their coefficients as kernel
 * arguments (the specialised fast kernels) have nothing to upload; the call is then a no-op. */
int iqo_hip_plan_prepare(iqo_hip_plan *plan);

/* Options: "force_general" (0/1: every shape through IQO_KERNEL_GENERAL), "bands" (row bands per
 * frame, 0 = auto) and "host_stage" (host-pointer path of frames >= 4 MiB: 0 the HIP runtime's own
 * pageable copies (default), 1 the pinned-staging band pipeline).  Every option changes speed
 * only, never the output bytes.  IQO_HIP_EINVAL for an unknown key or value.
 * With IQO_HIP_TUNING=1 in the environment the call also takes the A/B keys of
 * libiqo_amd/csrc/abi.hip (kernel family switches "tile", "walk", "up2", "d32", "a32", "u23",
 * "l23", "d31", "ryx", "ryg", "ryu"; schedules "tile_rows", "stack", "rounds", "tail", "prefetch",
 * "ratio_prefetch", "ryx_split", "ryx_adj", "ryx_cpt", "ryx_uc", "ryg_cpt", "ryu_run",
 * "stream_variant", "lanes", "chunk_frames"), which the tests and tuning scripts use; they are not
 * part of the supported interface. */
int iqo_hip_plan_set_option(iqo_hip_plan *plan, const char *key, long value);

/* Drop-in resize with HOST pointers (byte strides), synchronous: H2D, kernels, D2H. */
int iqo_hip_resize(iqo_hip_plan *plan, size_t srcSt, const uint8_t *src, size_t dstSt, uint8_t *dst);

/* Batched resize of nFrames frames resident in device memory, asynchronous on `stream`.
 * Frame f reads dSrc + f*srcFrameSt and writes dDst + f*dstFrameSt. */
int iqo_hip_resize_device(iqo_hip_plan *plan, size_t nFrames, size_t srcSt, size_t srcFrameSt,
                          const uint8_t *dSrc, size_t dstSt, size_t dstFrameSt, uint8_t *dDst,
                          void *stream);

/* Source rows [*srcRow0, *srcRow0 + *srcRows) that output rows [dstRow0, dstRow0 + dstRows)
 * read (the halo of a row band).  Host-only, no device work. */
int iqo_hip_band_src_rows(const iqo_hip_plan *plan, size_t dstRow0, size_t dstRows, size_t *srcRow0,
                          size_t *srcRows);

/* Row-band resize (multi-GPU sharding by output rows): computes global output rows
 * [dstRow0, dstRow0 + dstRows) of each frame.  dSrcWindow points at global source row srcRow0
 * (as returned by iqo_hip_band_src_rows, or any window containing it); dDstBand points at the
 * band's first row.  Rows are computed with their GLOBAL indices, so a banded result is
 * byte-identical to the unsharded one.  IQO_HIP_EINVAL if the window starts below the band's
 * first source row; the kernels read no row past the end of the band's window. */
int iqo_hip_resize_band(iqo_hip_plan *plan, size_t nFrames, size_t dstRow0, size_t dstRows,
                        size_t srcRow0, size_t srcSt, size_t srcFrameSt, const uint8_t *dSrcWindow,
                        size_t dstSt, size_t dstFrameSt, uint8_t *dDstBand, void *stream);

/* ---- YUV 4:2:0 (I420) three-plane resize: the reference benchmark's workload
 * (benchmark/benchmark.cpp:131-229, sample/resize_yuv420p.cpp:121-163): Y srcW x srcH -> dstW x dstH,
 * U and V srcW/2 x srcH/2 -> dstW/2 x dstH/2 with the same method; Lanczos chroma uses pxScale 2.
 * The reference composes three resizer objects; here one plan holds the luma and chroma plans. */
typedef struct iqo_hip_yuv_plan iqo_hip_yuv_plan;
int iqo_hip_plan_yuv420(int method, unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                        int device, iqo_hip_yuv_plan **out);
void iqo_hip_yuv_plan_destroy(iqo_hip_yuv_plan *plan);
/* Plane 0 = the luma plan, 1 = the chroma plan (for iqo_hip_plan_set_option / _query). */
iqo_hip_plan *iqo_hip_yuv_plane(iqo_hip_yuv_plan *plan, int plane);
/* Device-resident batch, asynchronous on `stream`: frame f's planes start at srcY/srcU/srcV +
 * f*srcFrameSt (likewise dst).  All three planes go in ONE launch when the plane kernels have a
 * fused instantiation (*fused = 1; the fast kernels of every BASELINE shape do), else one launch
 * per plane (*fused = 0).  `fused` may be NULL. */
int iqo_hip_resize_yuv420_device(iqo_hip_yuv_plan *plan, size_t nFrames, size_t srcStY, size_t srcStUV,
                                 size_t srcFrameSt, const uint8_t *srcY, const uint8_t *srcU, const uint8_t *srcV,
                                 size_t dstStY, size_t dstStUV, size_t dstFrameSt, uint8_t *dstY, uint8_t *dstU,
                                 uint8_t *dstV, void *stream, int *fused);
/* Host pointers, synchronous: the three planes through the pipelined host path of iqo_hip_resize. */
int iqo_hip_resize_yuv420(iqo_hip_yuv_plan *plan, size_t srcStY, const uint8_t *srcY, size_t srcStUV,
                          const uint8_t *srcU, const uint8_t *srcV, size_t dstStY, uint8_t *dstY, size_t dstStUV,
                          uint8_t *dstU, uint8_t *dstV);

/* ---- Multi-GPU data movement for row-band / image sharding.  The reference
 * splits a frame's output rows over OpenMP threads (src/IQOLanczosResizerImpl_AVX512.cpp:269-308);
 * across GPUs the same split needs each band's source window (halo rows) on its device and the
 * bands gathered back -- byte copies, no reduction, no RCCL collective.
 *
 * Copies nFrames blocks of bytesPerFrame bytes: block f from src + f*srcFrameSt to
 * dst + f*dstFrameSt.  A device < 0 means host memory.  Device to device on different GPUs:
 * hipMemcpyPeerAsync over xGMI when peer access is available, else staged through pinned host
 * memory.  Ordering: every route is ordered after the work already queued on `stream` (of the
 * destination device, or of the source device for device -> host).  The stream-ordered routes
 * (0, 1, 3) are asynchronous on `stream`; the host-staging route (2) first waits for `stream` and
 * the source device, then copies synchronously and has landed when the call returns.  *path (may be NULL) reports the route: 0 same device,
 * 1 peer DMA, 2 host staging, 3 host <-> device. */
int iqo_hip_copy_frames(void *dst, int dstDevice, size_t dstFrameSt, const void *src, int srcDevice,
                        size_t srcFrameSt, size_t bytesPerFrame, size_t nFrames, void *stream, int *path);

/* Cross-process access to another process's device buffer (one process per GPU): an exported
 * handle (64-byte hipIpcMemHandle_t + the pointer's offset in its allocation) is sent through any
 * control channel; the receiver opens it and gets a device pointer for iqo_hip_copy_frames. */
typedef struct {
    unsigned char bytes[64];
    uint64_t offset;
} iqo_hip_ipc_handle;
int iqo_hip_ipc_export(const void *devPtr, iqo_hip_ipc_handle *handle);
int iqo_hip_ipc_open(const iqo_hip_ipc_handle *handle, int device, void **devPtr);
int iqo_hip_ipc_close(void *devPtr, const iqo_hip_ipc_handle *handle);

const char *iqo_hip_strerror(int status);
const char *iqo_hip_version(void);

/* Host-only table query (no GPU needed): the quantised coefficient table the plan would upload
 * for `axis` (0 = X, 1 = Y), widened to int32, phases x taps.  Returns phases*taps or < 0. */
int iqo_host_tables(int method, unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                    size_t pxScale, int axis, int *nTaps, int *nPhases, int32_t *buf, size_t cap);

/* Host-only twin of iqo_hip_band_src_rows (no device needed): the source-row halo of output rows
 * [dstRow0, dstRow0 + dstRows) for the given resizer shape. */
int iqo_host_band_src_rows(int method, unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                           size_t pxScale, size_t dstRow0, size_t dstRows, size_t *srcRow0, size_t *srcRows);

/* Host-only: which kernel family a full-frame, 16-byte-aligned device call would use. */
int iqo_host_kernel_for(int method, unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                        size_t pxScale);

/* Drop-in classes (iqo::LanczosResizer, AreaResizer, LinearResizer): how many objects this process constructed on the
 * HIP backend, and on the CPU backend (no gfx950 device) plus the resize() calls of HIP objects that fell back to the
 * CPU (a device failure, or a call the HIP path rejected).  IQO_REQUIRE_HIP=1 makes any CPU use abort;
 * IQO_DROPIN_REPORT=1 prints the counts at exit (libiqo_amd/csrc/resizers.cpp). */
void iqo_dropin_backend_counts(int *hip, int *cpu);

#ifdef __cplusplus
}
#endif
#endif
