// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.
//
// extern "C" shim over the reference's own Generic implementations, compiled (with
// oracle/Makefile) from the reference sources where they lie under /root/reference/src.
// Nothing of the reference is copied: this file only includes the reference's SPI headers
// (src/IQO*ResizerImpl.hpp) and calls the exported factories
//   iqo::LanczosResizerImpl_new<iqo::ArchGeneric>()  (src/IQOLanczosResizerImpl_Generic.cpp:284-288)
//   iqo::AreaResizerImpl_new<iqo::ArchGeneric>()     (src/IQOAreaResizerImpl_Generic.cpp:167-171)
//   iqo::LinearResizerImpl_new<iqo::ArchGeneric>()   (src/IQOLinearResizerImpl_Generic.cpp:150-154)
// Output goes only to oracle/_ref/ (git-ignored).  Used to generate tests/golden and, when
// present, as the "reference" CPU baseline in bench.py.
#include <stddef.h>
#include <stdint.h>
#include <time.h>

#include <pthread.h>

#include "IQOAreaResizerImpl.hpp"
#include "IQOLanczosResizerImpl.hpp"
#include "IQOLinearResizerImpl.hpp"

namespace {

struct RefImpl {
    int method;
    iqo::ILanczosResizerImpl *lz;
    iqo::IAreaResizerImpl *ar;
    iqo::ILinearResizerImpl *ln;
};

RefImpl *make(int method, unsigned degree, size_t sw, size_t sh, size_t dw, size_t dh, size_t px)
{
    RefImpl *r = new RefImpl();
    r->method = method;
    r->lz = 0;
    r->ar = 0;
    r->ln = 0;
    if (method == 0) {
        r->lz = iqo::LanczosResizerImpl_new<iqo::ArchGeneric>();
        r->lz->init(degree, sw, sh, dw, dh, px);
    } else if (method == 1) {
        r->ar = iqo::AreaResizerImpl_new<iqo::ArchGeneric>();
        r->ar->init(sw, sh, dw, dh);
    } else {
        r->ln = iqo::LinearResizerImpl_new<iqo::ArchGeneric>();
        r->ln->init(sw, sh, dw, dh);
    }
    return r;
}

void run(RefImpl *r, size_t srcSt, const uint8_t *src, size_t dstSt, uint8_t *dst)
{
    if (r->lz)
        r->lz->resize(srcSt, src, dstSt, dst);
    else if (r->ar)
        r->ar->resize(srcSt, src, dstSt, dst);
    else
        r->ln->resize(srcSt, src, dstSt, dst);
}

void destroy(RefImpl *r)
{
    delete r->lz;
    delete r->ar;
    delete r->ln;
    delete r;
}

struct Job {
    int method;
    unsigned degree;
    size_t sw, sh, dw, dh, px, f0, f1, srcSt, srcFrameSt, dstSt, dstFrameSt;
    const uint8_t *src;
    uint8_t *dst;
};

void *worker(void *p)
{
    Job *j = static_cast<Job *>(p);
    RefImpl *r = make(j->method, j->degree, j->sw, j->sh, j->dw, j->dh, j->px);
    for (size_t f = j->f0; f < j->f1; ++f)
        run(r, j->srcSt, j->src + f * j->srcFrameSt, j->dstSt, j->dst + f * j->dstFrameSt);
    destroy(r);
    return 0;
}

} // namespace

extern "C" {

// One-shot: construct the Generic impl, resize once, destroy.  method 0/1/2 = lanczos/area/linear.
int iqo_ref_run(int method, unsigned degree, size_t sw, size_t sh, size_t dw, size_t dh, size_t px,
                size_t srcSt, const uint8_t *src, size_t dstSt, uint8_t *dst)
{
    if (!sw || !sh || !dw || !dh)
        return -1;
    RefImpl *r = make(method, degree, sw, sh, dw, dh, px);
    run(r, srcSt, src, dstSt, dst);
    destroy(r);
    return 0;
}

// Batch timing: one Generic instance per pthread (instances are not re-entrant,
// IQOLanczosResizerImpl_Generic.cpp:279).  Returns wall seconds.
double iqo_ref_run_batch(int method, unsigned degree, size_t sw, size_t sh, size_t dw, size_t dh,
                         size_t px, size_t nFrames, size_t srcSt, size_t srcFrameSt,
                         const uint8_t *src, size_t dstSt, size_t dstFrameSt, uint8_t *dst,
                         int nThreads)
{
    if (nThreads < 1)
        nThreads = 1;
    if (static_cast<size_t>(nThreads) > nFrames)
        nThreads = nFrames ? static_cast<int>(nFrames) : 1;
    pthread_t th[256];
    Job jobs[256];
    if (nThreads > 256)
        nThreads = 256;
    timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < nThreads; ++i) {
        Job &j = jobs[i];
        j.method = method;
        j.degree = degree;
        j.sw = sw;
        j.sh = sh;
        j.dw = dw;
        j.dh = dh;
        j.px = px;
        j.f0 = nFrames * i / nThreads;
        j.f1 = nFrames * (i + 1) / nThreads;
        j.srcSt = srcSt;
        j.srcFrameSt = srcFrameSt;
        j.dstSt = dstSt;
        j.dstFrameSt = dstFrameSt;
        j.src = src;
        j.dst = dst;
        pthread_create(&th[i], 0, worker, &j);
    }
    for (int i = 0; i < nThreads; ++i)
        pthread_join(th[i], 0);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return double(t1.tv_sec - t0.tv_sec) + 1e-9 * double(t1.tv_nsec - t0.tv_nsec);
}

} // extern "C"
