// ref_cpu_harness.cpp -- TEST INFRASTRUCTURE ONLY (the CPU baseline of bench.py).
//
// extern "C" timing shim over the reference's REAL CPU path: the public classes
// iqo::{Lanczos,Area,Linear}Resizer with their CPUID dispatch (src/IQOLanczosResizer.cpp:15-36:
// AVX512 -> AVX2FMA -> SSE4_1 -> Generic) and OpenMP row loops (e.g.
// src/IQOLanczosResizerImpl_AVX512.cpp:242-309), compiled by oracle/Makefile from the reference
// sources where they lie under /root/reference/src with the reference's own per-TU ISA flags
// (src/CMakeLists.txt:34-105), its Release flags (CMakeLists.txt:32-35) and WITH_OPENMP
// (CMakeLists.txt:17,56-62).  Nothing of the reference is copied: this file includes the
// reference's public and SPI headers and calls its classes.  Output only into oracle/_ref/.
//
// The SIMD paths compute in f32 and are NOT bit-exact with Generic; this
// shim is a speed baseline, never a parity oracle.
#include <stddef.h>
#include <stdint.h>
#include <time.h>

#include <pthread.h>
#include <omp.h>

#include <libiqo/iqo.hpp>

#include "IQOHWCap.hpp"

namespace {

double now()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return double(t.tv_sec) + 1e-9 * double(t.tv_nsec);
}

// One public resizer object of the given method (the reference's dispatch picks the impl).
struct Any {
    iqo::LanczosResizer *lz;
    iqo::AreaResizer *ar;
    iqo::LinearResizer *ln;
    Any(int method, unsigned degree, size_t sw, size_t sh, size_t dw, size_t dh, size_t px) : lz(0), ar(0), ln(0)
    {
        if (method == 0)
            lz = new iqo::LanczosResizer(degree, sw, sh, dw, dh, px);
        else if (method == 1)
            ar = new iqo::AreaResizer(sw, sh, dw, dh);
        else
            ln = new iqo::LinearResizer(sw, sh, dw, dh);
    }
    ~Any()
    {
        delete lz;
        delete ar;
        delete ln;
    }
    void resize(size_t srcSt, const uint8_t *src, size_t dstSt, uint8_t *dst)
    {
        if (lz)
            lz->resize(srcSt, src, dstSt, dst);
        else if (ar)
            ar->resize(srcSt, src, dstSt, dst);
        else
            ln->resize(srcSt, src, dstSt, dst);
    }
};

struct Job {
    int method;
    unsigned degree;
    size_t sw, sh, dw, dh, px, f0, f1, srcSt, srcFrameSt, dstSt, dstFrameSt;
    const uint8_t *src;
    uint8_t *dst;
};

void *frame_worker(void *p)
{
    Job *j = static_cast<Job *>(p);
    omp_set_num_threads(1);  // this thread's OpenMP regions stay on this thread
    Any r(j->method, j->degree, j->sw, j->sh, j->dw, j->dh, j->px);
    for (size_t f = j->f0; f < j->f1; ++f)
        r.resize(j->srcSt, j->src + f * j->srcFrameSt, j->dstSt, j->dst + f * j->dstFrameSt);
    return 0;
}

} // namespace

extern "C" {

// The impl the reference's CPUID dispatch selects on this host.
const char *iqo_refcpu_arch(void)
{
    iqo::HWCap cap;
#if defined(IQO_CPU_X86)
    if (cap.hasAVX512())
        return "AVX512";
    if (cap.hasAVX2FMA())
        return "AVX2FMA";
    if (cap.hasSSE4_1())
        return "SSE4_1";
#endif
    return "Generic";
}

// The reference's own threading: ONE public object, its OpenMP row loops on nThreads threads,
// frames one after another.  Returns wall seconds.
double iqo_refcpu_run_rows(int method, unsigned degree, size_t sw, size_t sh, size_t dw, size_t dh, size_t px,
                           size_t nFrames, size_t srcSt, size_t srcFrameSt, const uint8_t *src, size_t dstSt,
                           size_t dstFrameSt, uint8_t *dst, int nThreads)
{
    omp_set_num_threads(nThreads < 1 ? 1 : nThreads);
    Any r(method, degree, sw, sh, dw, dh, px);
    const double t0 = now();
    for (size_t f = 0; f < nFrames; ++f)
        r.resize(srcSt, src + f * srcFrameSt, dstSt, dst + f * dstFrameSt);
    return now() - t0;
}

// Frame parallelism: one public object per pthread (single-threaded OpenMP inside), nFrames
// split into contiguous ranges.  Returns wall seconds (object construction included, as the
// reference benchmark does, benchmark.cpp:215-226).
double iqo_refcpu_run_frames(int method, unsigned degree, size_t sw, size_t sh, size_t dw, size_t dh, size_t px,
                             size_t nFrames, size_t srcSt, size_t srcFrameSt, const uint8_t *src, size_t dstSt,
                             size_t dstFrameSt, uint8_t *dst, int nThreads)
{
    if (nThreads < 1)
        nThreads = 1;
    if (nThreads > 256)
        nThreads = 256;
    pthread_t th[256];
    Job jobs[256];
    const double t0 = now();
    for (int i = 0; i < nThreads; ++i) {
        Job &j = jobs[i];
        j.method = method;
        j.degree = degree;
        j.sw = sw;
        j.sh = sh;
        j.dw = dw;
        j.dh = dh;
        j.px = px;
        j.f0 = nFrames * size_t(i) / size_t(nThreads);
        j.f1 = nFrames * size_t(i + 1) / size_t(nThreads);
        j.srcSt = srcSt;
        j.srcFrameSt = srcFrameSt;
        j.dstSt = dstSt;
        j.dstFrameSt = dstFrameSt;
        j.src = src;
        j.dst = dst;
        pthread_create(&th[i], 0, frame_worker, &j);
    }
    for (int i = 0; i < nThreads; ++i)
        pthread_join(th[i], 0);
    return now() - t0;
}

// The reference benchmark's timed cycle (benchmark/benchmark.cpp:206-229 and :1017-1033): an I420
// frame, Y at W x H and U, V at W/2 x H/2, the resizer objects constructed INSIDE the timed
// region (Lanczos chroma with pxScale 2), OpenMP rows on nThreads threads; the minimum over
// `cycles` cycles (the benchmark runs 256).  Returns seconds per cycle (min).
double iqo_refcpu_bench_yuv420(int method, unsigned degree, size_t W, size_t H, size_t w, size_t h, int cycles,
                               int nThreads, const uint8_t *srcY, const uint8_t *srcU, const uint8_t *srcV,
                               size_t srcStY, size_t srcStC, uint8_t *dstY, uint8_t *dstU, uint8_t *dstV,
                               size_t dstStY, size_t dstStC)
{
    omp_set_num_threads(nThreads < 1 ? 1 : nThreads);
    double best = 1e30;
    for (int c = 0; c < cycles; ++c) {
        const double t0 = now();
        {
            Any y(method, degree, W, H, w, h, 1);
            y.resize(srcStY, srcY, dstStY, dstY);
        }
        {
            Any u(method, degree, W / 2, H / 2, w / 2, h / 2, method == 0 ? 2 : 1);
            u.resize(srcStC, srcU, dstStC, dstU);
            u.resize(srcStC, srcV, dstStC, dstV);
        }
        const double t = now() - t0;
        if (t < best)
            best = t;
    }
    return best;
}

} // extern "C"
