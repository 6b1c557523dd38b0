// abi.hip -- implementation of include/iqo_hip.h (the extern "C" boundary).
//
// A plan owns: the host Plan (tables + index maps, plan.cpp), their device copies, the chunk
// table of the general kernel, and (lazily) a stream
// plus device staging buffers for the host-pointer entry point.  There is no CPU fallback:
// any HIP failure is returned as a negative status.
#include "iqo_hip.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <new>
#include <thread>
#include <string>
#include <vector>

#include "kernels.hpp"
#include "plan.hpp"

using iqo_amd::AxisPlan;
using iqo_amd::CoordInfo;
using iqo_amd::Plan;

struct iqo_hip_plan {
    Plan p;
    int device = 0;
    // plan-cache key (make_plan): identical requests reuse a destroyed plan's tables
    int keyMethod = 0;
    unsigned keyDegree = 0;
    size_t keyDims[5] = {0, 0, 0, 0, 0};
    // Device tables (general / tile / walker / ratio-Y kernels) are staged into one host blob at
    // plan creation and uploaded by ONE allocation and copy the first time a launch needs them:
    // the specialised kernels take their coefficients as kernel arguments, so a plan that only
    // ever runs them costs no device allocation (the reference benchmark constructs its resizers
    // inside the timed loop, benchmark/benchmark.cpp:206-229).
    std::vector<uint8_t> blob;
    std::vector<std::pair<void **, size_t>> blobPtrs;  // member pointer, byte offset in the blob
    uint8_t *dBlob = nullptr;
    bool tablesUp = false;
    std::mutex tablesMu;
    int4 *dX = nullptr, *dY = nullptr, *dChunks = nullptr;
    int *dTabX = nullptr, *dTabY = nullptr;
    int nChunks = 0, ldsInts = 0;
    bool forceGeneral = false;
    int bands = 0;
    int debugFlags = 0;
#ifdef IQO_VARIANT_DEBUG
    uint64_t traceAddr = 0;  // variant builds: workgroup timeline buffer of the block-shared streamer
#endif
    int prefetch = 3;  // streamer prefetch: ring streamer depth 1..3 / symmetric LDS ring K = 3..5
    int streamVariant = 0;  // 0: block-shared symmetric streamer where eligible, 1: accumulator-ring
                            // streamer, 2: per-wave symmetric streamer (all bit-identical)
    int rounds = 0;         // block-shared streamer: target rounds for the auto band count (0 = 6, -1 = makespan model)
    int tail = 0;           // block-shared streamer: short bands for each XCD's last frame (0 auto, -1 off, n bands)
    int stack = 1;          // block-shared streamer: narrow frames side by side in one workgroup (speed only)
    int ryxAdj = 1;         // ratio-Y kernel: adjacent column pairs per thread where they fit (speed only)
    int ryxCpt = 1;         // ratio-Y kernel: 4 output columns per thread at the Lanczos 4:9 upscales (speed only)
    int ryxSplit = 1;       // ratio-Y kernel column parts (speed only; option ryx_split)
    int rygCpt = 0;         // general-row kernel on rows of > 1024 outputs: output columns per thread (0 = auto)
    int ryxUc = 1;          // ratio-Y kernel: uniform column coefficients as scalars where every column has the same
    int lanes = 0;          // symmetric streamer producing lanes per wave (0 = auto)
    int ratioPrefetch = 0;  // exact-ratio kernels: row groups loaded ahead (0 = kernel default)
    int chunkFrames = 0;    // frames per launch (0 = up to 65535)
    // separable tile kernel (shapes without a specialised kernel; plan option "tile" = 0 turns
    // it off, leaving general_kernel)
    iqo_amd::TileTables tt;
    int tileTH0 = 0, tileSrcRows0 = 0;  // the auto tile height (option "tile_rows" changes it; reset_options restores it)
    bool useTile = true;
    int4 *dTRows = nullptr, *dTSpans = nullptr;
    int2 *dTCols = nullptr;
    uint2 *dTRowTap = nullptr;
    uint32_t *dTColCoef = nullptr;
    int32_t *dTColA = nullptr;
    int tileNQp = 0;
    // general-ratio wave walker (plan.hpp WalkTables; option "walk" = 0 keeps tile_kernel)
    iqo_amd::WalkTables wt;
    bool useWalk = true;
    // exact 2x Lanczos upscale kernel, every row and column in-kernel (option "up2" = 0: walker only)
    iqo_amd::Up2Tables ut;
    bool useUp2 = true;
    // exact 3:2 Lanczos-3 downscale kernel on the main rows (option "d32" = 0: walker only)
    iqo_amd::D32Tables dt;
    iqo_amd::D31Tables t31;
    iqo_amd::RyxTables ryx;
    uint32_t *dRyxRowCoef = nullptr, *dRyxColCoef = nullptr;
    int4 *dRyxCols = nullptr;
    int4 *dRyxRowRec = nullptr;  // general-row tables (ryx.general: the ryg kernel, kernels.hpp RygDev)
    bool useRyg = true;
    // general upscale rows by window position (kernels.hip ryu_kernel): records, first window start
    int4 *dRyuPos = nullptr;
    int ryuBase = 0;
    bool hasRyu = false;  // the table exists (every window position holds 1 or 2 rows)
    bool useRyu = true;   // option "ryu" = 0: ryg_kernel's NL = 1 mode instead (A/B)
    uint32_t *dRyuRun = nullptr;  // run-mode column table (plan.hpp colRun), when it exists
    bool useRyuRun = true;        // option "ryu_run" = 0: per-column mode (A/B)
    int hostStage = 0;  // host-pointer path, frames >= 4 MiB: 0 the runtime's own pageable copies, 1 our pinned
                        // staging pipeline (host_pipeline), for A/B
    bool useD32 = true;
    bool useD31 = true;
    bool useRyx = true;
    // exact 2:3 Linear upscale kernel (option "l23" = 0: walker only)
    iqo_amd::L23Tables lt;
    bool useL23 = true;
    // exact 2:3 Lanczos-3 upscale kernel (option "u23" = 0: walker only)
    iqo_amd::U23Tables vt;
    bool useU23 = true;
    // exact 3:2 Area downscale kernel (option "a32" = 0: walker only)
    iqo_amd::A32Tables at;
    bool useA32 = true;
    int4 *dWSpans = nullptr;
    int4 *dWSegs = nullptr;
    uint32_t *dWRowTap = nullptr;
    int4 *dWRows = nullptr;
};

namespace {

constexpr int kChunkOut = 256;     // outputs per general-kernel chunk (= workgroup size)
constexpr int kChunkLds = 8192;    // max work-row ints per chunk (32 KiB LDS)

class DeviceGuard {  // restore the caller's current device
public:
    explicit DeviceGuard(int dev)
    {
        ok_ = hipGetDevice(&prev_) == hipSuccess && hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard()
    {
        if (ok_)
            (void)hipSetDevice(prev_);
    }
    bool ok() const { return ok_; }

private:
    int prev_ = 0;
    bool ok_ = false;
};

// ---- host-pointer path (iqo_hip_resize): staging pool
//
// Device staging frames, pinned host staging, three streams (H2D, kernels, D2H) and per-band
// events, pooled per device for the whole process: constructing a resizer stays cheap (the
// reference benchmark constructs one per call, benchmark.cpp:215-226), and one staging set is
// borrowed per call, so distinct plans can run concurrently from different threads.  The pool
// is never torn down (the HIP runtime may already be gone at static destruction).
constexpr int kHostBands = 8;      // output-row bands of one plane in the host-pointer pipeline
constexpr int kHostBandRows = 64;  // ... each at least this tall
constexpr int kHostChunks = 16;    // (plane, band) chunks of one call: events per staging set
constexpr size_t kHostPipeMinBytes = size_t(4) << 20;  // smaller frames: one band (API latency dominates)

struct HostStage {
    int device = 0;
    hipStream_t sIn = nullptr, sK = nullptr, sOut = nullptr, sIn2 = nullptr;
    hipEvent_t evIn[kHostChunks] = {}, evK[kHostChunks] = {}, evOut[kHostChunks] = {};
    uint8_t *dSrc = nullptr, *dDst = nullptr, *hSrc = nullptr, *hDst = nullptr;
    size_t dSrcCap = 0, dDstCap = 0, hSrcCap = 0, hDstCap = 0;
};

std::mutex g_stageMu;
std::vector<HostStage *> g_stagePool;

void destroy_stage(HostStage *st)
{
    for (int b = 0; b < kHostChunks; ++b) {
        if (st->evIn[b])
            (void)hipEventDestroy(st->evIn[b]);
        if (st->evK[b])
            (void)hipEventDestroy(st->evK[b]);
        if (st->evOut[b])
            (void)hipEventDestroy(st->evOut[b]);
    }
    if (st->sIn)
        (void)hipStreamDestroy(st->sIn);
    if (st->sK)
        (void)hipStreamDestroy(st->sK);
    if (st->sOut)
        (void)hipStreamDestroy(st->sOut);
    if (st->sIn2)
        (void)hipStreamDestroy(st->sIn2);
    (void)hipFree(st->dSrc);
    (void)hipFree(st->dDst);
    (void)hipHostFree(st->hSrc);
    (void)hipHostFree(st->hDst);
    delete st;
}

HostStage *acquire_stage(int device)
{
    {
        std::lock_guard<std::mutex> g(g_stageMu);
        for (size_t i = 0; i < g_stagePool.size(); ++i)
            if (g_stagePool[i]->device == device) {
                HostStage *st = g_stagePool[i];
                g_stagePool.erase(g_stagePool.begin() + static_cast<std::ptrdiff_t>(i));
                return st;
            }
    }
    HostStage *st = new (std::nothrow) HostStage();
    if (!st)
        return nullptr;
    st->device = device;
    bool ok = hipStreamCreateWithFlags(&st->sIn, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&st->sK, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&st->sOut, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&st->sIn2, hipStreamNonBlocking) == hipSuccess;
    for (int b = 0; ok && b < kHostChunks; ++b)
        ok = hipEventCreateWithFlags(&st->evIn[b], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&st->evK[b], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&st->evOut[b], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        // a partly built set is destroyed, never pooled: the next call builds a fresh one
        destroy_stage(st);
        return nullptr;
    }
    return st;
}

void release_stage(HostStage *st)
{
    std::lock_guard<std::mutex> g(g_stageMu);
    g_stagePool.push_back(st);
}

int grow_device(uint8_t **p, size_t *cap, size_t bytes)
{
    if (bytes <= *cap)
        return IQO_HIP_OK;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(reinterpret_cast<void **>(p), bytes) != hipSuccess)
        return IQO_HIP_ENOMEM;
    *cap = bytes;
    return IQO_HIP_OK;
}

int grow_pinned(uint8_t **p, size_t *cap, size_t bytes)
{
    if (bytes <= *cap)
        return IQO_HIP_OK;
    (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipHostMalloc(reinterpret_cast<void **>(p), bytes, hipHostMallocDefault) != hipSuccess)
        return IQO_HIP_ENOMEM;
    *cap = bytes;
    return IQO_HIP_OK;
}

// Host memory the DMA engines reach directly: hipHostMalloc'd or hipHostRegister'ed.
bool is_pinned_host(const void *p)
{
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory reports an error here; clear it
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

void copy_rows(uint8_t *dst, size_t dstSt, const uint8_t *src, size_t srcSt, size_t w, size_t rows)
{
    if (dstSt == w && srcSt == w) {
        std::memcpy(dst, src, w * rows);
        return;
    }
    for (size_t r = 0; r < rows; ++r)
        std::memcpy(dst + r * dstSt, src + r * srcSt, w);
}

// Row copies between pageable user memory and the pinned staging of the host-pointer path, split
// over a small process-wide thread pool: one thread's memcpy (~10 GB/s) is slower than the PCIe
// link the staged rows then cross.  Created on first use and never torn down (as the staging
// pool); one parallel copy at a time -- a caller that finds the pool busy copies alone.
struct RowCopy {
    uint8_t *dst;
    size_t dstSt;
    const uint8_t *src;
    size_t srcSt, w, rows;
};

class CopyPool {
public:
    static CopyPool &instance()
    {
        static CopyPool *p = new CopyPool();
        return *p;
    }
    // up to kMaxJobs row copies (e.g. the three I420 planes) as ONE parallel job: the rows of all
    // of them are split evenly over the workers, so a call pays one wake-up, not one per plane
    static constexpr int kMaxJobs = 3;
    void copy(const RowCopy *jobs, int n)
    {
        size_t bytes = 0, rows = 0;
        for (int j = 0; j < n; ++j) {
            bytes += jobs[j].w * jobs[j].rows;
            rows += jobs[j].rows;
        }
        std::unique_lock<std::mutex> use(useMu_, std::try_to_lock);
        // below ~256 KiB one thread's memcpy beats the wake-up of the pool
        if (!use.owns_lock() || workers_.empty() || n > kMaxJobs || bytes < (size_t(256) << 10) || rows < 32) {
            for (int j = 0; j < n; ++j)
                copy_rows(jobs[j].dst, jobs[j].dstSt, jobs[j].src, jobs[j].srcSt, jobs[j].w, jobs[j].rows);
            return;
        }
        std::unique_lock<std::mutex> g(mu_);
        nJobs_ = n;
        totalRows_ = rows;
        for (int j = 0; j < n; ++j)
            jobs_[j] = jobs[j];
        parts_ = static_cast<int>(workers_.size()) + 1;
        next_ = 0;
        remaining_ = parts_;
        ++gen_;
        cv_.notify_all();
        while (next_ < parts_) {  // the caller takes parts too
            const int part = next_++;
            g.unlock();
            run_part(part);
            g.lock();
            --remaining_;
        }
        done_.wait(g, [&] { return remaining_ == 0; });
    }

private:
    CopyPool()
    {
        const unsigned hw = std::thread::hardware_concurrency();
        const unsigned n = hw >= 4 ? std::min(7u, hw / 2) : 0u;
        for (unsigned i = 0; i < n; ++i)
            workers_.emplace_back([this] { work(); });
        for (auto &t : workers_)
            t.detach();
    }
    // part k copies global rows [R k / parts, R (k+1) / parts) of the jobs' rows laid end to end
    void run_part(int part) const
    {
        size_t r0 = totalRows_ * static_cast<size_t>(part) / static_cast<size_t>(parts_);
        const size_t r1 = totalRows_ * static_cast<size_t>(part + 1) / static_cast<size_t>(parts_);
        size_t base = 0;
        for (int j = 0; j < nJobs_ && r0 < r1; ++j) {
            const RowCopy &c = jobs_[j];
            const size_t a = std::max(r0, base), b = std::min(r1, base + c.rows);
            if (a < b) {
                copy_rows(c.dst + (a - base) * c.dstSt, c.dstSt, c.src + (a - base) * c.srcSt, c.srcSt, c.w, b - a);
                r0 = b;
            }
            base += c.rows;
        }
    }
    void work()
    {
        unsigned long seen = 0;
        std::unique_lock<std::mutex> g(mu_);
        for (;;) {
            cv_.wait(g, [&] { return gen_ != seen; });
            seen = gen_;
            while (next_ < parts_) {
                const int part = next_++;
                g.unlock();
                run_part(part);
                g.lock();
                if (--remaining_ == 0)
                    done_.notify_all();
            }
        }
    }
    std::mutex useMu_, mu_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> workers_;
    RowCopy jobs_[kMaxJobs]{};
    int nJobs_ = 0;
    size_t totalRows_ = 0;
    int parts_ = 0, next_ = 0, remaining_ = 0;
    unsigned long gen_ = 0;
};

void copy_rows_par(uint8_t *dst, size_t dstSt, const uint8_t *src, size_t srcSt, size_t w, size_t rows)
{
    const RowCopy c{dst, dstSt, src, srcSt, w, rows};
    CopyPool::instance().copy(&c, 1);
}

void copy_planes_par(const RowCopy *jobs, int n) { CopyPool::instance().copy(jobs, n); }

bool is_gfx950(int dev)
{
    // the device's architecture cannot change in a process: queried once per device (the
    // property query costs more than building a small plan's tables)
    static std::mutex mu;
    static std::vector<signed char> known;  // -1 unknown, 0 / 1
    std::lock_guard<std::mutex> g(mu);
    if (dev < 0)
        return false;
    if (static_cast<size_t>(dev) >= known.size())
        known.resize(static_cast<size_t>(dev) + 1, -1);
    if (known[static_cast<size_t>(dev)] < 0) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess)
            return false;
        known[static_cast<size_t>(dev)] = std::strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
    }
    return known[static_cast<size_t>(dev)] == 1;
}

template <typename T>
int upload(iqo_hip_plan *h, T **dptr, const T *src, size_t n)
{
    // stage into the plan's blob (256-B aligned sections); ensure_tables uploads it on first use
    const size_t off = (h->blob.size() + 255) & ~static_cast<size_t>(255);
    const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
    h->blob.resize(off + bytes, 0);
    if (src && n)
        std::memcpy(h->blob.data() + off, src, n * sizeof(T));
    h->blobPtrs.emplace_back(reinterpret_cast<void **>(dptr), off);
    *dptr = nullptr;
    return IQO_HIP_OK;
}

// One allocation + one copy of every staged table, then the table pointers point into it.
int ensure_tables(iqo_hip_plan *h)
{
    std::lock_guard<std::mutex> lock(h->tablesMu);
    if (h->tablesUp)
        return IQO_HIP_OK;
    if (!h->blob.empty()) {
        if (hipMalloc(reinterpret_cast<void **>(&h->dBlob), h->blob.size()) != hipSuccess)
            return IQO_HIP_ENOMEM;
        if (hipMemcpy(h->dBlob, h->blob.data(), h->blob.size(), hipMemcpyHostToDevice) != hipSuccess)
            return IQO_HIP_EHIP;
    }
    for (const auto &pr : h->blobPtrs)
        *pr.first = h->dBlob + pr.second;
    h->tablesUp = true;
    return IQO_HIP_OK;
}

// Source-column interval [a, b) that output column x reads (general kernel).
void column_span(const Plan &p, int x, int *a, int *b)
{
    const CoordInfo &c = p.x.coord[static_cast<size_t>(x)];
    const int W = p.srcW;
    if (c.kind == iqo_amd::kIdentity) {
        *a = c.srcO;
        *b = c.srcO + 1;
    } else if (p.method == iqo_amd::kLinear && c.kind != iqo_amd::kMain) {
        *a = c.kind == iqo_amd::kBorderLo ? 0 : W - 1;
        *b = *a + 1;
    } else if (p.method == iqo_amd::kLinear) {
        *a = std::max(0, std::min(c.srcO, W - 1));
        *b = std::max(0, std::min(c.srcO + 1, W - 1)) + 1;
    } else {
        *a = std::max(0, std::min(c.srcO, W - 1));
        *b = std::max(*a + 1, std::min(c.srcO + p.x.taps, W));
    }
}

int build_chunks(const Plan &p, std::vector<int4> *chunks, int *ldsInts)
{
    chunks->clear();
    *ldsInts = 1;
    int x = 0;
    while (x < p.dstW) {
        int lo, hi;
        column_span(p, x, &lo, &hi);
        if (hi - lo > kChunkLds)
            return IQO_HIP_EUNSUP;
        int xe = x + 1;
        while (xe < p.dstW && xe - x < kChunkOut) {
            int a, b;
            column_span(p, xe, &a, &b);
            int nlo = std::min(lo, a), nhi = std::max(hi, b);
            if (nhi - nlo > kChunkLds)
                break;
            lo = nlo;
            hi = nhi;
            ++xe;
        }
        chunks->push_back(make_int4(x, xe, lo, hi));
        *ldsInts = std::max(*ldsInts, hi - lo);
        x = xe;
    }
    return IQO_HIP_OK;
}

void free_plan(iqo_hip_plan *h)
{
    (void)hipFree(h->dBlob);
    delete h;
}

std::vector<int4> coord_records(const AxisPlan &a)
{
    std::vector<int4> v(a.coord.size());
    for (size_t i = 0; i < v.size(); ++i)
        v[i] = make_int4(a.coord[i].srcO, a.coord[i].tabOff, a.coord[i].kind, a.coord[i].aux);
    return v;
}

// Upload the separable tile kernel's tables (TileRec / TileCol have the int4 / int2 layout).
iqo_amd::RyxDev ryx_dev(const iqo_hip_plan *h);

// Window-position records of a general upscale (plan.cpp build_ryu_positions, kernels.hip
// ryu_kernel); none when a position holds more than 2 rows: ryg_kernel's NL = 1 mode runs the plan.
int ryu_positions(iqo_hip_plan *h)
{
    h->hasRyu = iqo_amd::build_ryu_positions(h->p.dstH, &h->ryx);
    if (!h->hasRyu)
        return IQO_HIP_OK;
    static_assert(iqo_amd::kRyuPosPad >= 3, "ryu_kernel reads the records up to a band's last position + 2");
    static_assert(iqo_amd::kRyuRec == 8, "ryu_kernel reads 8-int position records");
    h->ryuBase = h->ryx.posBase;
    int rc = upload(h, &h->dRyuPos, reinterpret_cast<const int4 *>(h->ryx.posRec.data()), h->ryx.posRec.size() / 4);
    if (!rc && iqo_amd::build_ryu_runs(h->p.dstW, &h->ryx))
        rc = upload(h, &h->dRyuRun, h->ryx.colRun.data(), h->ryx.colRun.size());
    return rc;
}

// Tables of the exact-ratio kernels (most take their coefficients as kernel arguments; ryx has
// device tables).  Built whether or not the tile tables exist: ryx also serves shapes whose taps
// exceed the tile kernel's (Lanczos-8/9 2:1).
int upload_exact(iqo_hip_plan *h)
{
    // exact-ratio kernels (no device tables: their coefficients are kernel arguments)
    iqo_amd::build_up2(h->p, h->wt, &h->ut);
    iqo_amd::build_d32(h->p, h->wt, &h->dt);
    iqo_amd::build_d31(h->p, &h->t31);
    iqo_amd::build_ryx(h->p, &h->ryx);
#ifdef IQO_RYU_EXACT  // variant builds (A/B): exact-ratio upscale rows on the general-row kernels instead
    if (h->ryx.ok && h->ryx.Q > h->ryx.P)
        h->ryx = iqo_amd::RyxTables();
#endif
    if (!h->ryx.ok)
        iqo_amd::build_ryg(h->p, &h->ryx);  // general rows (no exact P:Q)
    if (h->ryx.ok && ryx_dev(h).parts == 0)
        h->ryx = iqo_amd::RyxTables();  // no column split fits the workgroup limits
    if (h->ryx.ok && h->ryx.general) {
        // ryg_kernel reads the records of rows up to y1 - 1 + kRygPD + 1 unclamped (its FIFO look-ahead
        // and the next row's record): build_ryg's padding must cover them
        static_assert(iqo_amd::kRygRecPad >= iqo_amd::kRygPD + 2, "ryg row records: padding below the look-ahead");
        std::vector<int4> rr(h->ryx.rowRec.size() / 2);
        for (size_t i = 0; i < rr.size(); ++i) {
            const size_t ia = std::min(rr.size() - 1, i + iqo_amd::kRygPD - 1);  // (rows past the end repeat)
            rr[i] = make_int4(h->ryx.rowRec[2 * i], h->ryx.rowRec[2 * i + 1], h->ryx.rowRec[2 * ia], 0);
        }
        const int rc2 = upload(h, &h->dRyxRowRec, rr.data(), rr.size());
        if (rc2)
            return rc2;
        if (h->ryx.rowLoads == 1) {
            const int rc3 = ryu_positions(h);
            if (rc3)
                return rc3;
        }
    }
    if (h->ryx.ok) {
        std::vector<int4> rc(h->ryx.cols.size() / 4);
        for (size_t i = 0; i < rc.size(); ++i)
            rc[i] = make_int4(h->ryx.cols[4 * i], h->ryx.cols[4 * i + 1], h->ryx.cols[4 * i + 2], 0);
        int rc2 = upload(h, &h->dRyxRowCoef, h->ryx.rowCoef.data(), h->ryx.rowCoef.size());
        if (!rc2)
            rc2 = upload(h, &h->dRyxColCoef, h->ryx.colCoef.data(), h->ryx.colCoef.size());
        if (!rc2)
            rc2 = upload(h, &h->dRyxCols, rc.data(), rc.size());
        if (rc2)
            return rc2;
    }
    iqo_amd::build_a32(h->p, &h->at);
    iqo_amd::build_u23(h->p, &h->vt);
    iqo_amd::build_l23(h->p, &h->lt);
    return IQO_HIP_OK;
}

int upload_tile(iqo_hip_plan *h)
{
    const iqo_amd::TileTables &t = h->tt;
    if (!t.ok)
        return upload_exact(h);
    std::vector<int4> rows(t.rows.size()), spans(t.spans.size());
    std::vector<int2> cols(t.cols.size());
    for (size_t i = 0; i < rows.size(); ++i)
        rows[i] = make_int4(t.rows[i].start, t.rows[i].lo, t.rows[i].hi, t.rows[i].deno);
    for (size_t i = 0; i < cols.size(); ++i)
        cols[i] = make_int2(t.cols[i].a, t.cols[i].D);
    for (size_t i = 0; i < spans.size(); ++i) {
        int border = 0;  // any column of the tile with a Lanczos border division
        for (size_t x = i * t.CT; x < std::min(t.cols.size(), (i + 1) * t.CT); ++x)
            border |= t.cols[x].D != 0;
        spans[i] = make_int4(t.spans[i].lo8, t.spans[i].groups, border, 0);
    }
    // column coefficients transposed to [pair p][column-in-quad k][quad Q] (and window starts to
    // [k][Q]) over the padded tile width, so that a wave's load of one (p, k) is 64 consecutive
    // dwords; padding quads get zero coefficients and their tile's start (woff 0)
    const int nQp = static_cast<int>(spans.size()) * t.CT / 4;
    std::vector<uint32_t> coefT(static_cast<size_t>(t.NP) * 4 * nQp, 0u);
    std::vector<int32_t> colA(static_cast<size_t>(4) * nQp, 0);
    for (int Q = 0; Q < nQp; ++Q)
        for (int k = 0; k < 4; ++k) {
            const int x = 4 * Q + k;
            const bool in = x < static_cast<int>(t.cols.size());
            colA[static_cast<size_t>(k) * nQp + Q] = in ? t.cols[static_cast<size_t>(x)].a : t.spans[static_cast<size_t>(4 * Q / t.CT)].lo8;
            for (int p = 0; p < t.NP; ++p)
                coefT[(static_cast<size_t>(p) * 4 + k) * nQp + Q] = in ? t.colCoef[static_cast<size_t>(x) * t.NP + p] : 0u;
        }
    h->tileNQp = nQp;
    iqo_amd::build_walk_tables(h->p, t, &h->wt);
    if (h->wt.ok) {
        std::vector<int4> ws(h->wt.spans.size());
        for (size_t i = 0; i < ws.size(); ++i)
            ws[i] = make_int4(h->wt.spans[i].lo8, h->wt.spans[i].units, h->wt.spans[i].interior, 0);
        std::vector<int4> sg(2 * h->wt.segs.size());
        for (size_t i = 0; i < h->wt.segs.size(); ++i) {
            const iqo_amd::WalkSeg &g = h->wt.segs[i];
            sg[2 * i] = make_int4(g.first, g.slotOff, g.border, g.firstD);
            sg[2 * i + 1] = make_int4(static_cast<int>(g.yM), g.yS, g.yNeg, 0);
        }
        std::vector<int4> wr(h->wt.rows.size());
        for (size_t i = 0; i < wr.size(); ++i)
            wr[i] = make_int4(h->wt.rows[i].lo, h->wt.rows[i].hi, h->wt.rows[i].hiSlot, h->wt.rows[i].deno);
        const std::vector<uint32_t> &wt = h->wt.rowTap;
        int rc = upload(h, &h->dWSpans, ws.data(), ws.size());
        if (!rc)
            rc = upload(h, &h->dWRows, wr.data(), wr.size());
        if (!rc)
            rc = upload(h, &h->dWRowTap, wt.data(), wt.size());
        if (!rc)
            rc = upload(h, &h->dWSegs, sg.data(), sg.size());
        if (rc)
            return rc;
    }
    if (int rc = upload_exact(h))
        return rc;
    // per (row, tap): coefficient splat and the clamped source row it reads
    std::vector<uint2> rowTap(t.rowCoef.size());
    for (size_t y = 0; y < t.rows.size(); ++y)
        for (int i = 0; i < t.nYp; ++i) {
            const iqo_amd::TileRec &r = t.rows[y];
            const int row = std::min(std::max(r.start + i, r.lo), r.hi);
            rowTap[y * t.nYp + i] = make_uint2(t.rowCoef[y * t.nYp + i], static_cast<uint32_t>(row));
        }
    int rc;
    if ((rc = upload(h, &h->dTRows, rows.data(), rows.size())) || (rc = upload(h, &h->dTCols, cols.data(), cols.size())) ||
        (rc = upload(h, &h->dTSpans, spans.data(), spans.size())) ||
        (rc = upload(h, &h->dTRowTap, rowTap.data(), rowTap.size())) ||
        (rc = upload(h, &h->dTColCoef, coefT.data(), coefT.size())) || (rc = upload(h, &h->dTColA, colA.data(), colA.size())))
        return rc;
    return IQO_HIP_OK;
}

// Every option iqo_hip_plan_set_option can change, back to its default.
void reset_options(iqo_hip_plan *h)
{
    h->forceGeneral = false;
    h->bands = 0;
    h->debugFlags = 0;
    h->prefetch = 3;
    h->streamVariant = 0;
    h->rounds = 0;
    h->tail = 0;
    h->stack = 1;
    h->ryxSplit = 1;
    h->rygCpt = 0;
    h->ryxUc = 1;
    h->ryxAdj = 1;
    h->ryxCpt = 1;
    h->lanes = 0;
    h->ratioPrefetch = 0;
    h->chunkFrames = 0;
    h->useTile = h->useWalk = h->useUp2 = h->useD32 = h->useD31 = h->useRyx = h->useL23 = h->useU23 = h->useA32 = true;
    h->useRyg = true;
    h->useRyu = true;
    h->useRyuRun = true;
    h->hostStage = 0;
    if (h->tt.ok) {  // option "tile_rows"
        h->tt.TH = h->tileTH0;
        h->tt.srcRows = h->tileSrcRows0;
    }
}

// Destroyed plans are kept (options reset) and handed out again for an identical request: the
// reference benchmark constructs and destroys its three resizers in every timed cycle
// (benchmark/benchmark.cpp:206-229), and a plan's host tables cost more to build than a small
// frame takes to resize.  Bounded; the oldest entry is freed first.
constexpr size_t kPlanCache = 16;
std::mutex g_planCacheMu;
std::vector<iqo_hip_plan *> g_planCache;

iqo_hip_plan *plan_cache_take(int m, unsigned degree, const size_t (&dims)[5], int device)
{
    std::lock_guard<std::mutex> g(g_planCacheMu);
    for (size_t i = g_planCache.size(); i-- > 0;) {
        iqo_hip_plan *h = g_planCache[i];
        if (h->keyMethod == m && h->keyDegree == degree && h->device == device &&
            std::equal(dims, dims + 5, h->keyDims)) {
            g_planCache.erase(g_planCache.begin() + static_cast<std::ptrdiff_t>(i));
            return h;
        }
    }
    return nullptr;
}

void plan_cache_put(iqo_hip_plan *h)
{
    reset_options(h);
    iqo_hip_plan *evict = nullptr;
    {
        std::lock_guard<std::mutex> g(g_planCacheMu);
        g_planCache.push_back(h);
        if (g_planCache.size() > kPlanCache) {
            evict = g_planCache.front();
            g_planCache.erase(g_planCache.begin());
        }
    }
    if (evict) {
        DeviceGuard guard(evict->device);
        free_plan(evict);
    }
}

int make_plan(iqo_amd::Method m, unsigned degree, size_t sw, size_t sh, size_t dw, size_t dh, size_t px,
              int device, iqo_hip_plan **out)
{
    if (!out)
        return IQO_HIP_EINVAL;
    *out = nullptr;
    const size_t dims[5] = {sw, sh, dw, dh, px};
    if (iqo_hip_plan *c = plan_cache_take(static_cast<int>(m), degree, dims, device)) {
        *out = c;
        return IQO_HIP_OK;
    }
    iqo_hip_plan *h = new (std::nothrow) iqo_hip_plan();
    if (!h)
        return IQO_HIP_ENOMEM;
    std::string err;
    if (!iqo_amd::build_plan(m, degree, sw, sh, dw, dh, px, &h->p, &err)) {
        delete h;
        return IQO_HIP_EINVAL;
    }
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count || !is_gfx950(device)) {
        delete h;
        return IQO_HIP_ENODEV;
    }
    h->device = device;
    h->keyMethod = static_cast<int>(m);
    h->keyDegree = degree;
    std::copy(dims, dims + 5, h->keyDims);
    DeviceGuard guard(device);
    if (!guard.ok()) {
        delete h;
        return IQO_HIP_ENODEV;
    }
    std::vector<int4> chunks;
    int rc = build_chunks(h->p, &chunks, &h->ldsInts);
    if (rc) {
        delete h;
        return rc;
    }
    h->nChunks = static_cast<int>(chunks.size());
    iqo_amd::build_tile_tables(h->p, &h->tt);
    h->tileTH0 = h->tt.TH;
    h->tileSrcRows0 = h->tt.srcRows;
    std::vector<int4> xr = coord_records(h->p.x), yr = coord_records(h->p.y);
    if ((rc = upload(h, &h->dX, xr.data(), xr.size())) || (rc = upload(h, &h->dY, yr.data(), yr.size())) ||
        (rc = upload(h, &h->dTabX, h->p.x.table.data(), h->p.x.table.size())) ||
        (rc = upload(h, &h->dTabY, h->p.y.table.data(), h->p.y.table.size())) ||
        (rc = upload(h, &h->dChunks, chunks.data(), chunks.size())) || (rc = upload_tile(h))) {
        free_plan(h);
        return rc;
    }
    *out = h;
    return IQO_HIP_OK;
}

uint32_t pair16(int lo, int hi) { return (static_cast<uint32_t>(lo) & 0xffffu) | (static_cast<uint32_t>(hi) << 16); }

bool aligned(const void *p, size_t a, size_t st, size_t fst)
{
    return (reinterpret_cast<uintptr_t>(p) % a) == 0 && (st % a) == 0 && (fst % a) == 0;
}

// Device-side views of a plan for each kernel family (kernel arguments, no device memory).
iqo_amd::LanczosDev lanczos_dev(const iqo_hip_plan *h)
{
    const Plan &p = h->p;
    iqo_amd::LanczosDev l{};
    const iqo_amd::FastLanczos &f = p.flz;
    l.KY = f.KY;
    l.KX = f.KX;
    l.NY = f.NY;
    l.NXP = f.NXP;
    l.offX = f.offX;
    l.srcW = p.srcW;
    l.srcH = p.srcH;
    l.dstW = p.dstW;
    l.dstH = p.dstH;
    l.offY = f.offY;
    for (int i = 0; i < f.NY; ++i)
        l.cy[i] = pair16(f.cy[i], f.cy[i]);
    for (int i = 0; i < f.NXP / 2; ++i)
        l.cx[i] = pair16(f.cx[2 * i], f.cx[2 * i + 1]);
    l.mainBeginY = f.mainBeginY;
    l.mainEndY = f.mainEndY;
    l.mainBeginX = f.mainBeginX;
    l.mainEndX = f.mainEndX;
    for (int i = 0; i < 16; ++i) {
        l.yTopM[i] = f.yTopM[i];
        l.yTopS[i] = f.yTopS[i];
        l.yBotM[i] = f.yBotM[i];
        l.yBotS[i] = f.yBotS[i];
    }
    for (int k = 0; k < 8; ++k) {
        l.xM[k] = f.xM[k];
        l.xT[k] = f.xT[k];
    }
    if (f.NX == 20 && f.NY == 16) {  // Lanczos-5 2:1: kernels.hpp LanczosDev (reused fields)
        for (int k = 0; k < 16; ++k) {
            l.cx[k] = f.xM8[k];
            (k < 8 ? l.xM[k] : reinterpret_cast<uint32_t &>(l.xT[k - 8])) = static_cast<uint32_t>(f.xT8[k]);
        }
    }
    l.yTopNeg = f.yTopNeg;
    l.yBotNeg = f.yBotNeg;
    l.xNeg = f.xNeg;
    l.dbg = h->debugFlags;
#ifdef IQO_VARIANT_DEBUG
    l.trace = h->traceAddr;
#endif
    l.prefetch = h->prefetch;
    l.rounds = h->rounds;
    l.tail = h->tail;
    l.stack = h->stack;
    l.sym = !f.sym || h->streamVariant == 1 ? 0 : (h->streamVariant >= 2 ? h->streamVariant : 1);
    if (f.NY == 12 || f.NY == 16)
        l.sym = 1;  // Lanczos-4 / -5 2:1: the block-shared symmetric streamer is their only instantiation
    l.NX = f.NX;
    l.offXO = f.offXO;
    for (int i = 0; i < f.NX / 2 && i < 10; ++i)
        (i < 8 ? l.cxo[i] : l.cy[i]) = pair16(f.cxo[2 * i], f.cxo[2 * i + 1]);  // (pairs 8, 9: Lanczos-5)
    l.np = h->lanes;
    return l;
}

iqo_amd::AreaDev area_dev(const iqo_hip_plan *h)
{
    const Plan &p = h->p;
    iqo_amd::AreaDev a{};
    a.KY = p.far.KY;
    a.KX = p.far.KX;
    a.srcW = p.srcW;
    a.dstW = p.dstW;
    for (int i = 0; i < a.KY; ++i)
        a.cy[i] = pair16(p.far.cy[i], p.far.cy[i]);
    for (int i = 0; i < (a.KX + 1) / 2; ++i)  // odd KX: the last pair is (c_{KX-1}, 0)
        a.cx[i] = pair16(p.far.cx[2 * i], 2 * i + 1 < a.KX ? p.far.cx[2 * i + 1] : 0);
    a.dstH = p.dstH;
    a.lin = p.far.lin ? 1 : 0;
    a.srcH = p.srcH;
    return a;
}

iqo_amd::LinearDev linear_dev(const iqo_hip_plan *h)
{
    const Plan &p = h->p;
    iqo_amd::LinearDev l{};
    l.srcW = p.srcW;
    l.srcH = p.srcH;
    l.dstW = p.dstW;
    l.dstH = p.dstH;
    l.F = p.fln.F;
    for (int q = 0; q < 3; ++q) {
        l.cx[q] = pair16(p.fln.cx[q][0], p.fln.cx[q][1]);
        l.cy[q] = pair16(p.fln.cy[q][0], p.fln.cy[q][1]);
    }
    l.dbg = h->debugFlags;
    l.np = h->lanes;
    return l;
}

iqo_amd::TileDev tile_dev(const iqo_hip_plan *h)
{
    const iqo_amd::TileTables &t = h->tt;
    iqo_amd::TileDev d;
    d.lanczos = h->p.method == iqo_amd::kLanczos;
    d.srcW = h->p.srcW;
    d.srcH = h->p.srcH;
    d.dstW = h->p.dstW;
    d.NP = t.NP;
    d.nYp = t.nYp;
    d.CT = t.CT;
    d.TH = t.TH;
    d.pitchDw = t.pitchDw;
    d.log2nQ = t.log2nQ;
    d.srcRows = t.srcRows;
    d.spitch = t.spitch;
    d.rows = h->dTRows;
    d.rowTap = h->dTRowTap;
    d.cols = h->dTCols;
    d.colCoef = h->dTColCoef;
    d.colA = h->dTColA;
    d.nQp = h->tileNQp;
    d.spans = h->dTSpans;
    return d;
}

iqo_amd::WalkDev walk_dev(const iqo_hip_plan *h)
{
    const iqo_amd::WalkTables &w = h->wt;
    iqo_amd::WalkDev d;
    d.t = tile_dev(h);
    d.nS = w.nS;
    d.spans = h->dWSpans;
    d.NV = w.NV;
    d.R = w.R;
    d.pitch = w.pitch;
    d.waveBytes = static_cast<int>(w.waveBytes);
    d.rowTap = h->dWRowTap;
    d.rows = h->dWRows;
    d.segs = h->dWSegs;
    return d;
}

iqo_amd::Up2Dev up2_dev(const iqo_hip_plan *h)
{
    const iqo_amd::Up2Tables &u = h->ut;
    iqo_amd::Up2Dev d;
    d.srcW = h->p.srcW;
    d.srcH = h->p.srcH;
    d.dstW = h->p.dstW;
    d.dstH = h->p.dstH;
    d.F = u.F;
    d.NT = u.NT;
    d.np = h->lanes;
    d.cy0 = u.cy0;
    d.cx0 = u.cx0;
    std::memcpy(d.cy1, u.cy1, sizeof d.cy1);
    std::memcpy(d.cx1, u.cx1, sizeof d.cx1);
    std::memcpy(d.xM, u.xM, sizeof d.xM);
    std::memcpy(d.xT, u.xT, sizeof d.xT);
    d.m0 = u.m0;
    d.m1 = u.m1;
    std::memcpy(d.yM, u.yM, sizeof d.yM);
    std::memcpy(d.yS, u.yS, sizeof d.yS);
    return d;
}

iqo_amd::D32Dev d32_dev(const iqo_hip_plan *h)
{
    const iqo_amd::D32Tables &t = h->dt;
    iqo_amd::D32Dev d;
    d.srcW = h->p.srcW;
    d.srcH = h->p.srcH;
    d.dstW = h->p.dstW;
    d.dstH = h->p.dstH;
    d.np = h->lanes;
    d.pd = h->ratioPrefetch;
    d.variant = t.variant;
    std::memcpy(d.cy, t.cy, sizeof d.cy);
    std::memcpy(d.cx, t.cx, sizeof d.cx);
    std::memcpy(d.xM, t.xM, sizeof d.xM);
    std::memcpy(d.xT, t.xT, sizeof d.xT);
    d.m0 = t.m0;
    d.m1 = t.m1;
    std::memcpy(d.yM, t.yM, sizeof d.yM);
    std::memcpy(d.yS, t.yS, sizeof d.yS);
    return d;
}

iqo_amd::D31Dev d31_dev(const iqo_hip_plan *h)
{
    const iqo_amd::D31Tables &t = h->t31;
    iqo_amd::D31Dev d;
    d.srcW = h->p.srcW;
    d.srcH = h->p.srcH;
    d.dstW = h->p.dstW;
    d.dstH = h->p.dstH;
    d.np = h->lanes;
    d.pd = h->ratioPrefetch;
    d.variant = t.variant;
    d.cc = t.cc;
    std::memcpy(d.cp, t.cp, sizeof d.cp);
    std::memcpy(d.cxe, t.cxe, sizeof d.cxe);
    std::memcpy(d.cxo, t.cxo, sizeof d.cxo);
    std::memcpy(d.xM, t.xM, sizeof d.xM);
    std::memcpy(d.xT, t.xT, sizeof d.xT);
    d.m0 = t.m0;
    d.m1 = t.m1;
    std::memcpy(d.yM, t.yM, sizeof d.yM);
    std::memcpy(d.yS, t.yS, sizeof d.yS);
    return d;
}

iqo_amd::RyxDev ryx_dev(const iqo_hip_plan *h)
{
    const iqo_amd::RyxTables &t = h->ryx;
    iqo_amd::RyxDev d;
    d.lanczos = h->p.method == iqo_amd::kLanczos;
    d.srcW = h->p.srcW;
    d.srcH = h->p.srcH;
    d.dstW = h->p.dstW;
    d.dstH = h->p.dstH;
    d.P = t.P;
    d.Q = t.Q;
    d.taps = t.taps;
    d.NP = t.NP;
    d.off = t.off;
    d.m0 = t.m0;
    d.m1 = t.m1;
    std::memcpy(d.yM, t.yM, sizeof d.yM);
    std::memcpy(d.yS, t.yS, sizeof d.yS);
    d.rowCoef = h->dRyxRowCoef;
    d.cols = h->dRyxCols;
    d.colCoef = h->dRyxColCoef;
    // column split into `n` workgroups of `threads` threads: output columns [xs[k], xs[k+1]) (even,
    // 2 per thread) from source columns [cs[k], ce[k]) (multiples of 4, 4 per thread)
    auto split = [&](int n, int threads) -> bool {
        int xs[17], cs[16], ce[16];
        for (int k = 0; k <= n; ++k)
            xs[k] = k == 0 ? 0 : k == n ? d.dstW : (k * d.dstW / n + 1) & ~1;
        for (int k = 0; k < n; ++k) {
            int lo = 1 << 30, hi = -(1 << 30);
            for (int x = xs[k]; x < xs[k + 1]; ++x) {
                const int a = t.cols[static_cast<size_t>(x) * 4] / 2 - iqo_amd::kRyxPad;  // even window start
                lo = std::min(lo, a);
                hi = std::max(hi, a + 2 * t.NP);
            }
            cs[k] = k == 0 ? 0 : std::max(0, lo) & ~3;
            ce[k] = k == n - 1 ? d.srcW : std::min(d.srcW, (hi + 3) & ~3);
            if (ce[k] - cs[k] > 4 * threads || xs[k + 1] - xs[k] > d.cpt * threads || (k > 0 && lo < 0) ||
                (k < n - 1 && hi > d.srcW) || xs[k + 1] <= xs[k])
                return false;
        }
        d.parts = n;
        d.threads = threads;
        for (int k = 0; k < 17; ++k)
            d.xs[k] = k <= n ? xs[k] : d.dstW;
        for (int k = 0; k < 16; ++k) {
            d.cs[k] = k < n ? cs[k] : 0;
            d.ce[k] = k < n ? ce[k] : d.srcW;
        }
        return true;
    };
    // the fewest parts of `threads` threads that hold the row (up to 16)
    auto split_min = [&](int threads) {
        for (int n = 1; n <= 16; ++n)
            if (split(n, threads))
                return true;
        return false;
    };
    // Lanczos: workgroups of 4 waves (half or a quarter of the row each) when their source spans
    // fit 256 threads x 4 columns: barriers over 4 waves instead of 8 (1080p -> 480p: Lanczos-2
    // 0.171 vs 0.182 ms, Lanczos-3 0.232 vs 0.239, profiles/r03/ryx_split.txt; 4K -> 960x540
    // Lanczos-3 0.441 vs 0.404 ms with four parts instead of two of 8 waves; Area 5 % slower,
    // so not for Area).  Option "ryx_split": 0 one 8-wave workgroup per row where it fits, 2 / 3
    // parts of 2 waves / 1 wave.  parts = 0: no split fits (build_plan then drops the kernel).
    d.parts = 0;
    d.threads = 512;
    // Lanczos-3 upscales (4:9 rows, 4 pairs): 4 output columns per thread in one workgroup per row
    // (640 -> 1920 in 480 threads instead of four 256-thread parts of 2 columns per thread: 0.333
    // vs 0.359 ms; Lanczos-2 with 6 columns per thread was slower, 0.379 vs 0.308 ms,
    // profiles/r04/ryx_up49.txt)
    d.cpt = 2;
    if (d.Q > d.P && d.NP >= 4 && h->ryxCpt) {
        d.cpt = 4;
        const int need = std::max((d.srcW + 3) / 4, (d.dstW + d.cpt - 1) / d.cpt);
        if (need <= 512 && split(1, (need + 63) / 64 * 64))
            return d;
        if (split_min(512))
            return d;
        d.cpt = 2;
        d.parts = 0;
    }
    // general rows (ryg): output columns per thread ~ 4 x dstW / srcW, so that the threads of the
    // horizontal pass (CPT columns each) match those of the vertical pass (4 source columns each):
    // 1080p -> 1366x768 with 3 columns per thread (two parts of 256 threads) 0.256 ms vs 4 columns
    // 0.308 (a third of the threads idle in the horizontal pass), 2 columns needed four parts
    // (profiles/r05/steady_ryg_cpt.txt); option "ryg_cpt" forces 2, 3 or 4
    if (t.general) {
        // (12-row windows or 6 column pairs with 4 columns per thread spill: 3 at most there; 16-row
        // windows spill at 3: 2 there, Lanczos-6 1080p -> 1366x768 0.490 -> 0.381 ms,
        // profiles/r06/ryg_l45.txt)
        const int cap = t.taps >= 16 ? 2 : t.taps >= 12 || t.NP >= 6 ? 3 : 4;
        d.cpt = h->rygCpt ? h->rygCpt : std::min(cap, std::max(2, (4 * d.dstW + d.srcW / 2) / d.srcW));
        if (t.rowLoads >= 3)
            d.cpt = 2;  // (downscales past 2:1: 2 columns per thread is the only instantiation)
        // (round 6, late) parts of ONE wave where the row fits 16 of them: a barrier over one wave
        // instead of 4 or 8, and no 512-thread part half idle (2560 columns took two parts of 512
        // threads for 640 columns' work).  Lanczos downscale rows: 2560x1440 -> 1024x576 0.554 ->
        // 0.339 ms, -> 1920x1080 0.393 -> 0.255, 4K -> 1600x900 0.429 -> 0.363, 1080p -> 1366x768
        // -2.6 %; rows that need more than 16 parts of one wave take parts of two waves below 4 rows
        // per output row (4K -> 1366x768 0.399 -> 0.332; at 4 rows the 22-tap kernel, which spills,
        // was 11 % slower in them).  Upscale rows keep one or two workgroups where those hold the
        // row (1024x576 -> 1080p was 6 % slower in one-wave parts) and take one-wave parts where
        // not (1366x768 -> 2560x1440 0.263 -> 0.225).  Area rows keep the 8-wave parts (4K ->
        // 1366x768 12 % slower in one-wave parts).  profiles/r06/ryg_split.txt; option ryx_split = 4
        // restores the previous rule.
        if (h->ryxSplit == 1 && d.lanczos) {
            if (t.rowLoads >= 2 && (split_min(64) || (t.rowLoads < 4 && split_min(128))))
                return d;
            if (t.rowLoads == 1 && !split(2, 256) && !split(1, 512) && split_min(64))
                return d;
        }
        const int split_opt = h->ryxSplit == 4 ? 1 : h->ryxSplit;
        const int tw = split_opt == 2 ? 128 : 64;
        if ((split_opt >= 2 && split_min(tw)) || (split_opt == 1 && split(2, 256)) || split(1, 512))
            return d;  // (ryx_split 0: one 8-wave part where it fits)
        // (round 5, late) one more column per thread when that keeps the row in one workgroup, else
        // the fewest parts, each of the fewest 64-thread multiples that hold it: 1080p -> 1600x900
        // had two 512-thread parts with half their threads idle
        if (!h->rygCpt && t.rowLoads < 3 && d.cpt < cap) {
            ++d.cpt;
            if (split(1, 512))
                return d;
            --d.cpt;
        }
        for (int n = 2; n <= 16; ++n)
            for (int th = 128; th <= 512; th += 64)
                if (split(n, th))
                    return d;
        d.cpt = 2;
        d.parts = 0;
    }
    const int sopt = h->ryxSplit == 4 ? 1 : h->ryxSplit;  // (4: the previous rules, above and here)
    const int tw = sopt == 2 ? 128 : sopt == 3 ? 64 : 256;
    if (!(sopt >= 2 && split_min(tw)) && !(sopt == 1 && d.lanczos && d.dstW >= 64 && split(2, 256)) && !split(1, 512) &&
        !(sopt == 1 && split(4, 256)))
        split_min(512);
    // (round 6, late) Lanczos rows whose parts are less than 3/4 busy take the fewest parts of one
    // wave instead: 2560 columns in four 256-thread parts left 96 threads of each idle (2560x1440 ->
    // 640x360 0.299 -> 0.240 ms, Lanczos-2 -> 1138x640 0.319 -> 0.263, Lanczos-6 -> 720p 0.235 ->
    // 0.191); the 1080p / 4K rows of the bench list fill their parts to 94-97 % and keep them (there
    // one-wave parts were 5-10 % slower), profiles/r06/ryg_split.txt
    if (h->ryxSplit == 1 && d.lanczos && d.parts > 0) {
        int busy = 0;
        for (int k = 0; k < d.parts; ++k)
            busy += std::max((d.ce[k] - d.cs[k] + 3) / 4, (d.xs[k + 1] - d.xs[k] + d.cpt - 1) / d.cpt);
        if (4 * busy < 3 * d.parts * d.threads)
            split_min(64);  // (leaves the split as it is when no one-wave split holds the row)
    }
    // adjacent column pairs per thread (9:4 only, where every pair's windows start 1 or 2 pairs
    // apart, i.e. columns at 2:1 or more): one LDS run of NP + 2 dwords for both columns
    d.adj = 0;
    if (d.parts > 0 && h->ryxAdj && d.P == 2 && d.Q == 1 && d.lanczos && d.cpt == 2) {
        // 2:1 rows with 2:1 columns (uniform coefficients, below): every pair's windows one pair apart
        bool ok = true;
        for (int k = 0; k < d.parts && ok; ++k)
            for (int x = d.xs[k]; x + 1 < d.xs[k + 1] && ok; x += 2)
                ok = t.cols[static_cast<size_t>(x + 1) * 4] - t.cols[static_cast<size_t>(x) * 4] == 4;
        d.adj = ok ? 1 : 0;
    }
    if (d.parts > 0 && h->ryxAdj && d.P == 9 && d.Q == 4) {
        bool ok = true;
        for (int k = 0; k < d.parts && ok; ++k)
            for (int x = d.xs[k]; x + 1 < d.xs[k + 1] && ok; x += 2) {
                const int dl = t.cols[static_cast<size_t>(x + 1) * 4] - t.cols[static_cast<size_t>(x) * 4];
                ok = dl == 4 || dl == 8;
            }
        d.adj = ok ? 1 : 0;
    }
    // uniform column coefficients (Lanczos 2:1 columns): the kernel keeps them in scalar registers,
    // not NP x CPT per-lane registers (Lanczos-9: 38 VGPRs, the difference between 2 and 4 waves
    // per SIMD); option "ryx_uc" = 0 keeps the per-lane tables
    d.uc = 0;
    if (d.parts > 0 && h->ryxUc && d.lanczos && d.P == 2 && d.Q == 1 && d.cpt == 2) {
        bool same = true;
        const size_t np = static_cast<size_t>(t.NP);
        for (size_t x = 1; x < static_cast<size_t>(d.dstW) && same; ++x)
            same = std::equal(t.colCoef.begin() + static_cast<ptrdiff_t>(x * np), t.colCoef.begin() + static_cast<ptrdiff_t>((x + 1) * np),
                              t.colCoef.begin());
        d.uc = same ? 1 : 0;
    }
    if (d.adj && d.P == 2 && !d.uc)
        d.adj = 0;  // (2:1 adjacent pairs: uniform-column instantiations only)
    return d;
}

// The general-row kernel's view: ryx_dev's column split and tables plus the row records.
iqo_amd::RygDev ryg_dev(const iqo_hip_plan *h)
{
    const iqo_amd::RyxDev x = ryx_dev(h);
    iqo_amd::RygDev d;
    d.lanczos = x.lanczos;
    d.srcW = x.srcW;
    d.srcH = x.srcH;
    d.dstW = x.dstW;
    d.dstH = x.dstH;
    d.taps = x.taps;
    d.NP = x.NP;
    d.m0 = x.m0;
    d.m1 = x.m1;
    std::memcpy(d.yM, x.yM, sizeof d.yM);
    std::memcpy(d.yS, x.yS, sizeof d.yS);
    d.rowRec = h->dRyxRowRec;
    d.rowCoef = x.rowCoef;
    d.cols = x.cols;
    d.colCoef = x.colCoef;
    d.parts = x.parts;
    d.threads = x.threads;
    std::memcpy(d.xs, x.xs, sizeof d.xs);
    std::memcpy(d.cs, x.cs, sizeof d.cs);
    std::memcpy(d.ce, x.ce, sizeof d.ce);
    d.cpt = x.cpt;
    d.nl = h->ryx.rowLoads;
    if (d.nl == 1 && h->hasRyu && h->useRyu) {
        d.posRec = h->dRyuPos;
        d.posBase = h->ryuBase;
        d.posRows = h->ryx.posRows;
        // run mode: 4 adjacent columns per thread, every part starting on a multiple of 4 columns
        bool aligned = d.cpt == 4 && h->ryx.runPairs > 0 && h->useRyuRun;
        for (int k = 0; k < d.parts && aligned; ++k)
            aligned = d.xs[k] % 4 == 0;
        if (aligned) {
            d.colRun = h->dRyuRun;
            d.run = h->ryx.runPairs;
        }
    }
    return d;
}

iqo_amd::L23Dev l23_dev(const iqo_hip_plan *h)
{
    iqo_amd::L23Dev d;
    d.srcW = h->p.srcW;
    d.srcH = h->p.srcH;
    d.dstW = h->p.dstW;
    d.dstH = h->p.dstH;
    d.np = h->lanes;
    d.pd = h->ratioPrefetch;
    std::memcpy(d.cy, h->lt.cy, sizeof d.cy);
    std::memcpy(d.cx, h->lt.cx, sizeof d.cx);
    return d;
}

iqo_amd::U23Dev u23_dev(const iqo_hip_plan *h)
{
    const iqo_amd::U23Tables &t = h->vt;
    iqo_amd::U23Dev d;
    d.srcW = h->p.srcW;
    d.srcH = h->p.srcH;
    d.dstW = h->p.dstW;
    d.dstH = h->p.dstH;
    d.np = h->lanes;
    d.pd = h->ratioPrefetch;
    d.cy0 = t.cy0;
    d.cx0 = t.cx0;
    std::memcpy(d.cy, t.cy, sizeof d.cy);
    std::memcpy(d.cx, t.cx, sizeof d.cx);
    std::memcpy(d.xM, t.xM, sizeof d.xM);
    std::memcpy(d.xT, t.xT, sizeof d.xT);
    d.m0 = t.m0;
    d.m1 = t.m1;
    std::memcpy(d.yM, t.yM, sizeof d.yM);
    std::memcpy(d.yS, t.yS, sizeof d.yS);
    return d;
}

iqo_amd::A32Dev a32_dev(const iqo_hip_plan *h)
{
    iqo_amd::A32Dev d;
    d.srcW = h->p.srcW;
    d.srcH = h->p.srcH;
    d.dstW = h->p.dstW;
    d.dstH = h->p.dstH;
    d.np = h->lanes;
    d.pd = h->ratioPrefetch;
    std::memcpy(d.cy, h->at.cy, sizeof d.cy);
    std::memcpy(d.cx, h->at.cx, sizeof d.cx);
    return d;
}

iqo_amd::GeneralDev general_dev(const iqo_hip_plan *h)
{
    const Plan &p = h->p;
    iqo_amd::GeneralDev g{};
    g.method = p.method;
    g.srcW = p.srcW;
    g.srcH = p.srcH;
    g.dstW = p.dstW;
    g.nX = p.x.taps;
    g.nY = p.y.taps;
    g.xInfo = h->dX;
    g.yInfo = h->dY;
    g.tabX = h->dTabX;
    g.tabY = h->dTabY;
    g.chunks = h->dChunks;
    g.nChunks = h->nChunks;
    g.ldsInts = h->ldsInts;
    return g;
}

// The ratio-Y kernel is usable when its tables exist and a column split fits for the plan's
// CURRENT options (ryx_split / ryx_cpt are speed options; upload_exact checked the defaults only).
// The defaults end in split_min(512), the widest split, so when they fit every option does.
bool ryx_usable(const iqo_hip_plan *h)
{
    return h->ryx.ok && !h->ryx.general && h->useRyx && ryx_dev(h).parts > 0;
}

// ... and its general-row variant (build_ryg)
bool ryg_usable(const iqo_hip_plan *h)
{
    return h->ryx.ok && h->ryx.general && h->useRyg && ryx_dev(h).parts > 0;
}

// Area and Linear rows shrinking by less than 1.4, or with two row phases (exact 3:2), keep the wave
// walker when it can run: ryg loads NL = 2 rows per output row and is slower there (steady clock,
// x256: Area 1080p -> 1600x900 0.368 vs 0.267 ms, 1440p -> 1080p 0.415 vs 0.356, Linear 3:2 0.181
// vs 0.163; at 45:32 ryg is ahead, Area 0.198 vs 0.271; profiles/r05/ratio_sweep_ryg_ab.txt)
bool walk_beats_ryg(const iqo_hip_plan *h)
{
    const Plan &p = h->p;
    return p.method != iqo_amd::kLanczos && (5 * p.srcH < 7 * p.dstH || p.y.phases <= 2);
}

// The kernel family a full-frame call with aligned pointers and strides runs.
int plan_kernel(const iqo_hip_plan *h)
{
    int k = h->forceGeneral ? IQO_KERNEL_GENERAL : h->p.kernel;
    if (k == IQO_KERNEL_GENERAL && !h->forceGeneral && h->tt.ok && h->useTile)
        k = IQO_KERNEL_TILE;
    if (k == IQO_KERNEL_TILE && h->wt.ok && h->useWalk)
        k = IQO_KERNEL_WALK;
    if ((k == IQO_KERNEL_WALK || k == IQO_KERNEL_TILE) && h->ut.ok && h->useUp2)
        k = IQO_KERNEL_LANCZOS_UP2;
    if ((k == IQO_KERNEL_WALK || k == IQO_KERNEL_TILE) && h->dt.ok && h->useD32)
        k = IQO_KERNEL_LANCZOS_D32;
    if ((k == IQO_KERNEL_WALK || k == IQO_KERNEL_TILE) && h->t31.ok && h->useD31)
        k = IQO_KERNEL_LANCZOS_D31;
    // (ryx also takes shapes whose taps exceed the tile kernel's tables: Lanczos-8/9 2:1)
    if ((k == IQO_KERNEL_WALK || k == IQO_KERNEL_TILE || (k == IQO_KERNEL_GENERAL && !h->forceGeneral)) &&
        ryx_usable(h))
        k = IQO_KERNEL_RYX;
    if ((k == IQO_KERNEL_WALK || k == IQO_KERNEL_TILE) && h->at.ok && h->useA32)
        k = IQO_KERNEL_AREA_D32;
    if ((k == IQO_KERNEL_WALK || k == IQO_KERNEL_TILE) && h->vt.ok && h->useU23)
        k = IQO_KERNEL_LANCZOS_U23;
    if ((k == IQO_KERNEL_WALK || k == IQO_KERNEL_TILE) && h->lt.ok && h->useL23)
        k = IQO_KERNEL_LINEAR_U23;
    // general rows last: only what no exact-ratio kernel takes
    if ((k == IQO_KERNEL_TILE || (k == IQO_KERNEL_WALK && !walk_beats_ryg(h))) && ryg_usable(h))
        k = IQO_KERNEL_RYG;
    return k;
}

// The kernel family a call with these pointers and strides runs: the plan's fast kernel when the
// layout has the alignment that kernel's vector accesses need, else the general kernel.
int kernel_for_layout(const iqo_hip_plan *h, const void *src, size_t srcSt, size_t srcFrameSt, const void *dst,
                      size_t dstSt, size_t dstFrameSt)
{
    const Plan &p = h->p;
    int kernel = h->forceGeneral ? IQO_KERNEL_GENERAL : p.kernel;
    if (kernel == IQO_KERNEL_LANCZOS_STREAM && !(aligned(src, 16, srcSt, srcFrameSt) && aligned(dst, 16 / p.flz.KX, dstSt, dstFrameSt)))
        kernel = IQO_KERNEL_GENERAL;
    if (kernel == IQO_KERNEL_AREA_INT) {
        // 16-B loads / 16 / KX output bytes per thread; 12-B loads / 12 / KX bytes when KX is 3 or 6
        const int cols = 16 % p.far.KX == 0 ? 16 : 12;
        if (!(aligned(src, cols == 16 ? 16 : 4, srcSt, srcFrameSt) && aligned(dst, cols / p.far.KX, dstSt, dstFrameSt)))
            kernel = IQO_KERNEL_GENERAL;
    }
    if (kernel == IQO_KERNEL_LINEAR_UP2 && !(aligned(src, 8, srcSt, srcFrameSt) && aligned(dst, 16, dstSt, dstFrameSt)))
        kernel = IQO_KERNEL_GENERAL;
    if (kernel == IQO_KERNEL_GENERAL && !h->forceGeneral && h->tt.ok && h->useTile)
        kernel = IQO_KERNEL_TILE;  // any alignment (the kernel adapts per frame)
    // the wave walker loads aligned dwords: 4-byte aligned source frames and rows
    if (kernel == IQO_KERNEL_TILE && h->wt.ok && h->useWalk && aligned(src, 4, srcSt, srcFrameSt))
        kernel = IQO_KERNEL_WALK;
    // the 2x Lanczos kernel loads 8 B per lane and stores 16 B per lane
    if ((kernel == IQO_KERNEL_WALK || kernel == IQO_KERNEL_TILE) && h->ut.ok && h->useUp2 &&
        aligned(src, 8, srcSt, srcFrameSt) &&
        aligned(dst, 16, dstSt, dstFrameSt))
        kernel = IQO_KERNEL_LANCZOS_UP2;
    // the 3:2 Lanczos kernel loads 12 B per lane (4-byte aligned) and stores 8 B per lane
    if ((kernel == IQO_KERNEL_WALK || kernel == IQO_KERNEL_TILE) && h->dt.ok && h->useD32 &&
        aligned(src, 4, srcSt, srcFrameSt) && aligned(dst, 8, dstSt, dstFrameSt))
        kernel = IQO_KERNEL_LANCZOS_D32;
    // the 3:1 Lanczos kernel loads 12 B per lane (4-byte aligned) and stores 4 B per lane
    if ((kernel == IQO_KERNEL_WALK || kernel == IQO_KERNEL_TILE) && h->t31.ok && h->useD31 &&
        aligned(src, 4, srcSt, srcFrameSt) && aligned(dst, 4, dstSt, dstFrameSt))
        kernel = IQO_KERNEL_LANCZOS_D31;
    // exact vertical ratio, tabled columns: dword loads; 2-byte stores (1-byte stores when the
    // destination is not 2-byte aligned, launch_ryx)
    if ((kernel == IQO_KERNEL_WALK || kernel == IQO_KERNEL_TILE || (kernel == IQO_KERNEL_GENERAL && !h->forceGeneral)) &&
        ryx_usable(h))  // (round 5: unaligned dword loads verified on gfx950, profiles/r05/unaligned_src.txt)
        kernel = IQO_KERNEL_RYX;
    if ((kernel == IQO_KERNEL_WALK || kernel == IQO_KERNEL_TILE) && h->at.ok && h->useA32 &&
        aligned(src, 4, srcSt, srcFrameSt) && aligned(dst, 8, dstSt, dstFrameSt))
        kernel = IQO_KERNEL_AREA_D32;
    // the 2:3 Lanczos kernel loads 8 B per lane and stores 12 B per lane
    if ((kernel == IQO_KERNEL_WALK || kernel == IQO_KERNEL_TILE) && h->vt.ok && h->useU23 &&
        aligned(src, 8, srcSt, srcFrameSt) && aligned(dst, 4, dstSt, dstFrameSt))
        kernel = IQO_KERNEL_LANCZOS_U23;
    if ((kernel == IQO_KERNEL_WALK || kernel == IQO_KERNEL_TILE) && h->lt.ok && h->useL23 &&
        aligned(src, 8, srcSt, srcFrameSt) && aligned(dst, 4, dstSt, dstFrameSt))
        kernel = IQO_KERNEL_LINEAR_U23;
    // general rows last (dword loads, byte stores)
    if ((kernel == IQO_KERNEL_TILE || (kernel == IQO_KERNEL_WALK && !walk_beats_ryg(h))) && ryg_usable(h))
        kernel = IQO_KERNEL_RYG;
    return kernel;
}

iqo_amd::Io make_io(size_t frames, const uint8_t *src, size_t srcSt, size_t srcFrameSt, size_t srcRow0, int srcRowEnd,
                    uint8_t *dst, size_t dstSt, size_t dstFrameSt, int dstRow0)
{
    iqo_amd::Io io;
    io.frames = static_cast<int>(frames);
    io.src = src;
    io.srcSt = static_cast<int64_t>(srcSt);
    io.srcFrameSt = static_cast<int64_t>(srcFrameSt);
    io.srcRow0 = static_cast<int>(srcRow0);
    io.srcRowEnd = srcRowEnd;
    io.dst = dst;
    io.dstSt = static_cast<int64_t>(dstSt);
    io.dstFrameSt = static_cast<int64_t>(dstFrameSt);
    io.dstRow0 = dstRow0;
    return io;
}

int run_band(iqo_hip_plan *h, size_t nFrames, size_t r0, size_t rows, size_t srcRow0, size_t srcSt,
             size_t srcFrameSt, const uint8_t *src, size_t dstSt, size_t dstFrameSt, uint8_t *dst, hipStream_t s)
{
    const Plan &p = h->p;
    if (!src || !dst || srcSt < static_cast<size_t>(p.srcW) || dstSt < static_cast<size_t>(p.dstW))
        return IQO_HIP_EINVAL;
    const size_t dstH = static_cast<size_t>(p.dstH);
    if (r0 > dstH || rows > dstH - r0 || srcRow0 >= static_cast<size_t>(p.srcH))
        return IQO_HIP_EINVAL;
    if (rows == 0 || nFrames == 0)
        return IQO_HIP_OK;
    // the window must start at or above the first source row the band reads (iqo_hip_band_src_rows);
    // the kernels read at most up to the window's end s1, never past it
    int s0, s1;
    iqo_amd::band_src_rows(p, static_cast<int>(r0), static_cast<int>(r0 + rows), &s0, &s1);
    if (srcRow0 > static_cast<size_t>(s0))
        return IQO_HIP_EINVAL;
    DeviceGuard guard(h->device);
    if (!guard.ok())
        return IQO_HIP_ENODEV;

    const int kernel = kernel_for_layout(h, src, srcSt, srcFrameSt, dst, dstSt, dstFrameSt);
    if (kernel == IQO_KERNEL_TILE || kernel == IQO_KERNEL_WALK || kernel == IQO_KERNEL_RYX ||
        kernel == IQO_KERNEL_RYG || kernel == IQO_KERNEL_GENERAL) {
        const int rc = ensure_tables(h);
        if (rc)
            return rc;
    }

    const int rb = static_cast<int>(r0), re = static_cast<int>(r0 + rows);
    // Frames per launch: at most 65535 (grid y).  The option "chunk_frames" splits further into
    // equal launches (measured: no gain on MI355X for C2 at 256 frames, a loss for C3 at 48 --
    // the per-frame slowdown of C2 past ~130 frames per call is not a per-launch effect).
    size_t chunk = 65535;
    if (h->chunkFrames > 0) {
        chunk = std::min(chunk, static_cast<size_t>(h->chunkFrames));
        const size_t n = (nFrames + chunk - 1) / chunk;  // equal launches, not one straggler
        chunk = (nFrames + n - 1) / n;
    }
    // the exact-ratio kernels instantiate a few prefetch depths each; any other forced depth is an
    // error, not a silent fall-back to the default kernel
    if (h->ratioPrefetch > 0) {
        const int pd = h->ratioPrefetch;
        bool ok = true;
        if (kernel == IQO_KERNEL_LANCZOS_D32)
            ok = h->dt.variant == 0 ? (pd == 1 || pd == 2 || pd == 4) : (pd == 1 || pd == 3);
        else if (kernel == IQO_KERNEL_LANCZOS_D31)
            ok = h->t31.variant == 0 ? (pd == 1 || pd == 5) : (pd == 1 || pd == 2 || pd == 4);
        else if (kernel == IQO_KERNEL_LANCZOS_U23 || kernel == IQO_KERNEL_LINEAR_U23)
            ok = pd == 1 || pd == 2;
        else if (kernel == IQO_KERNEL_AREA_D32)
            ok = pd == 2 || pd == 4 || pd == 8;
        if (!ok)
            return IQO_HIP_EINVAL;
    }
    for (size_t f0 = 0; f0 < nFrames; f0 += chunk) {
        const iqo_amd::Io io = make_io(std::min(chunk, nFrames - f0), src + f0 * srcFrameSt, srcSt, srcFrameSt, srcRow0,
                                       s1, dst + f0 * dstFrameSt, dstSt, dstFrameSt, rb);
        hipError_t e = hipSuccess;
        if (kernel == IQO_KERNEL_LANCZOS_STREAM)
            e = iqo_amd::launch_lanczos_stream(lanczos_dev(h), io, rb, re, h->bands, s);
        else if (kernel == IQO_KERNEL_AREA_INT)
            e = iqo_amd::launch_area_int(area_dev(h), io, rb, re, s);
        else if (kernel == IQO_KERNEL_LINEAR_UP2)
            e = iqo_amd::launch_linear_up2(linear_dev(h), io, rb, re, h->bands, s);
        else if (kernel == IQO_KERNEL_TILE)
            e = iqo_amd::launch_tile(tile_dev(h), io, rb, re, s);
        else if (kernel == IQO_KERNEL_WALK)
            e = iqo_amd::launch_walk(walk_dev(h), io, rb, re, h->bands, s);
        else if (kernel == IQO_KERNEL_LANCZOS_UP2)
            e = iqo_amd::launch_up2(up2_dev(h), io, rb, re, h->bands, s);
        else if (kernel == IQO_KERNEL_LANCZOS_D32)
            e = iqo_amd::launch_d32(d32_dev(h), io, rb, re, h->bands, s);
        else if (kernel == IQO_KERNEL_LANCZOS_D31)
            e = iqo_amd::launch_d31(d31_dev(h), io, rb, re, h->bands, s);
        else if (kernel == IQO_KERNEL_RYX)
            e = iqo_amd::launch_ryx(ryx_dev(h), io, rb, re, h->bands, s);
        else if (kernel == IQO_KERNEL_RYG)
            e = iqo_amd::launch_ryg(ryg_dev(h), io, rb, re, h->bands, s);
        else if (kernel == IQO_KERNEL_AREA_D32)
            e = iqo_amd::launch_a32(a32_dev(h), io, rb, re, h->bands, s);
        else if (kernel == IQO_KERNEL_LANCZOS_U23)
            e = iqo_amd::launch_u23(u23_dev(h), io, rb, re, h->bands, s);
        else if (kernel == IQO_KERNEL_LINEAR_U23)
            e = iqo_amd::launch_l23(l23_dev(h), io, rb, re, h->bands, s);
        else
            e = iqo_amd::launch_general(general_dev(h), io, rb, re, s);
        // the launchers reject a parameter set they have no instantiation for before launching
        // (hipErrorInvalidValue / hipErrorNotSupported): a plan / kernel mismatch, reported as such
        // (the drop-in classes report those on every call instead of falling back for good)
        if (e == hipErrorInvalidValue)
            return IQO_HIP_EINVAL;
        if (e == hipErrorNotSupported)
            return IQO_HIP_EUNSUP;
        if (e != hipSuccess)
            return IQO_HIP_EHIP;
    }
    return IQO_HIP_OK;
}

} // namespace

extern "C" {

int iqo_hip_available(void)
{
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess)
        return 0;
    int n = 0;
    for (int d = 0; d < count; ++d)
        n += is_gfx950(d) ? 1 : 0;
    return n;
}

int iqo_hip_plan_lanczos(unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH, size_t pxScale,
                         int device, iqo_hip_plan **out)
{
    return make_plan(iqo_amd::kLanczos, degree, srcW, srcH, dstW, dstH, pxScale, device, out);
}

int iqo_hip_plan_area(size_t srcW, size_t srcH, size_t dstW, size_t dstH, int device, iqo_hip_plan **out)
{
    return make_plan(iqo_amd::kArea, 0, srcW, srcH, dstW, dstH, 1, device, out);
}

int iqo_hip_plan_linear(size_t srcW, size_t srcH, size_t dstW, size_t dstH, int device, iqo_hip_plan **out)
{
    return make_plan(iqo_amd::kLinear, 0, srcW, srcH, dstW, dstH, 1, device, out);
}

void iqo_hip_plan_destroy(iqo_hip_plan *plan)
{
    if (!plan)
        return;
    plan_cache_put(plan);  // kept for an identical request (make_plan), or freed when evicted
}

int iqo_hip_plan_query(const iqo_hip_plan *h, iqo_hip_plan_desc *d)
{
    if (!h || !d)
        return IQO_HIP_EINVAL;
    d->method = h->p.method;
    d->device = h->device;
    d->srcW = static_cast<size_t>(h->p.srcW);
    d->srcH = static_cast<size_t>(h->p.srcH);
    d->dstW = static_cast<size_t>(h->p.dstW);
    d->dstH = static_cast<size_t>(h->p.dstH);
    d->tapsX = h->p.x.taps;
    d->tapsY = h->p.y.taps;
    d->phasesX = h->p.x.phases;
    d->phasesY = h->p.y.phases;
    d->kernel = plan_kernel(h);
    d->bandsPerFrame = h->bands;
    d->tileRows = h->tt.ok ? h->tt.TH : 0;
    return IQO_HIP_OK;
}

int iqo_hip_plan_prepare(iqo_hip_plan *h)
{
    if (!h)
        return IQO_HIP_EINVAL;
    DeviceGuard guard(h->device);
    if (!guard.ok())
        return IQO_HIP_ENODEV;
    return ensure_tables(h);
}

// The A/B keys (kernel family switches, band / lane / prefetch / column-split schedules; every one
// speed-only) are accepted only with IQO_HIP_TUNING=1 in the environment -- tests, bench.py
// --option and the tuning scripts set it; a caller of the public ABI sees force_general, bands and
// host_stage only (include/iqo_hip.h).
bool tuning_enabled()
{
    const char *e = std::getenv("IQO_HIP_TUNING");
    return e && *e && std::strcmp(e, "0") != 0;
}

int iqo_hip_plan_set_option(iqo_hip_plan *h, const char *key, long value)
{
    if (!h || !key)
        return IQO_HIP_EINVAL;
    if (!std::strcmp(key, "force_general")) {
        h->forceGeneral = value != 0;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "bands")) {
        if (value < 0)
            return IQO_HIP_EINVAL;
        h->bands = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "host_stage")) {  // host-pointer path of large frames (speed only): 0 the runtime's
        if (value < 0 || value > 1)              // pageable copies, 1 the pinned staging pipeline
            return IQO_HIP_EINVAL;
        h->hostStage = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    if (!tuning_enabled())
        return IQO_HIP_EINVAL;
#ifdef IQO_VARIANT_DEBUG
    if (!std::strcmp(key, "debug_flags")) {  // variant builds only: timing experiments, wrong results
        h->debugFlags = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "trace_addr")) {  // variant builds only: device buffer of 16 B per workgroup
        h->traceAddr = static_cast<uint64_t>(value);
        return IQO_HIP_OK;
    }
#endif
    if (!std::strcmp(key, "tail")) {  // block-shared Lanczos streamer: short tail bands (speed only)
        if (value < -1 || value > 4096)
            return IQO_HIP_EINVAL;
        h->tail = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "rounds")) {  // block-shared Lanczos streamer: auto band count (speed only)
        if (value < -1 || value > 64)
            return IQO_HIP_EINVAL;
        h->rounds = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "ryx_split")) {  // ratio-Y kernel column parts (speed only): 0 one 8-wave
        if (value < 0 || value > 4)          // workgroup per row where it fits, 1 default, 2 / 3 parts of 2 / 1 waves,
                                             // 4 the general rows' round-6 rule before one-wave parts
            return IQO_HIP_EINVAL;
        h->ryxSplit = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "ryx_adj")) {  // ratio-Y kernel adjacent column pairs (speed only): 0 off, 1 where they fit
        if (value < 0 || value > 1)
            return IQO_HIP_EINVAL;
        h->ryxAdj = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "ryx_cpt")) {  // ratio-Y upscales: 0 two output columns per thread, 1 four
                                          // at the Lanczos 4:9 upscales
        if (value < 0 || value > 1)
            return IQO_HIP_EINVAL;
        h->ryxCpt = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "ryx_uc")) {  // ratio-Y kernel: 0 per-lane column coefficients everywhere (speed only)
        h->ryxUc = value != 0;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "ryg_cpt")) {  // general-row kernel, rows of > 1024 outputs: columns per thread
        if (value != 0 && (value < 2 || value > 4))  // (0 auto, 2, 3, 4; speed only)
            return IQO_HIP_EINVAL;
        h->rygCpt = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "stack")) {  // narrow frames side by side in one workgroup (speed only):
        if (value < 0 || value > 2)        // 0 off, 1 where a frame fills <= 1/2 wave, 2 from 2 frames
            return IQO_HIP_EINVAL;
        h->stack = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "prefetch")) {  // Lanczos streamer prefetch depth (rows)
        if (value < 1 || value > 4)
            return IQO_HIP_EINVAL;
        h->prefetch = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "stream_variant")) {  // A/B: 0 symmetric block-shared (default), 1 ring,
        if (value < 0 || value > 2)              // 2 symmetric per-wave
            return IQO_HIP_EINVAL;
        h->streamVariant = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "lanes")) {  // Lanczos / Linear streamers: producing lanes per wave (0 = auto)
        if (value < 0 || value > 62)
            return IQO_HIP_EINVAL;
        h->lanes = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "tile_rows")) {  // output rows per tile of the tile kernel (0 = auto)
        iqo_amd::TileTables t = h->tt;
        if (!t.ok)
            return IQO_HIP_EUNSUP;
        if (value == 0) {
            iqo_amd::build_tile_tables(h->p, &t);
        } else if (!iqo_amd::tile_set_rows(h->p, &t, static_cast<int>(value))) {
            return IQO_HIP_EINVAL;
        }
        h->tt.TH = t.TH;
        h->tt.srcRows = t.srcRows;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "tile")) {  // 0: shapes without a specialised kernel use general_kernel
        h->useTile = value != 0;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "up2")) {  // 0: exact 2x Lanczos upscales use the wave walker alone
        h->useUp2 = value != 0;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "l23")) {  // 0: exact 2:3 Linear upscales use the wave walker alone
        h->useL23 = value != 0;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "u23")) {  // 0: exact 2:3 Lanczos-3 upscales use the wave walker alone
        h->useU23 = value != 0;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "a32")) {  // 0: exact 3:2 Area downscales use the wave walker alone
        h->useA32 = value != 0;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "ratio_prefetch")) {  // exact-ratio kernels: row groups loaded ahead (speed only);
                                                 // a depth the plan's kernel does not instantiate fails the
                                                 // resize call with IQO_HIP_EINVAL
        if (value < 0 || value > 8)
            return IQO_HIP_EINVAL;
        h->ratioPrefetch = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "ryg")) {  // 0: general-row downscales (1 .. 2 : 1) use the wave walker / tile kernel
        h->useRyg = value != 0;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "ryu_run")) {  // 0: general upscale rows read each column's window separately
        h->useRyuRun = value != 0;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "ryu")) {  // 0: general upscale rows walk output rows (ryg_kernel NL = 1), not window positions
        h->useRyu = value != 0;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "ryx")) {  // 0: exact-vertical-ratio downscales use the general kernels
        h->useRyx = value != 0;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "d31")) {  // 0: exact 3:1 Lanczos downscales use the general kernels
        h->useD31 = value != 0;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "d32")) {  // 0: exact 3:2 Lanczos-3 downscales use the wave walker alone
        h->useD32 = value != 0;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "walk")) {  // 0: general ratios use tile_kernel instead of the wave walker
        h->useWalk = value != 0;
        return IQO_HIP_OK;
    }
    if (!std::strcmp(key, "chunk_frames")) {  // frames per launch (0 = auto)
        if (value < 0)
            return IQO_HIP_EINVAL;
        h->chunkFrames = static_cast<int>(value);
        return IQO_HIP_OK;
    }
    return IQO_HIP_EINVAL;
}

int iqo_hip_resize_device(iqo_hip_plan *h, size_t nFrames, size_t srcSt, size_t srcFrameSt, const uint8_t *dSrc,
                          size_t dstSt, size_t dstFrameSt, uint8_t *dDst, void *stream)
{
    if (!h)
        return IQO_HIP_EINVAL;
    return run_band(h, nFrames, 0, static_cast<size_t>(h->p.dstH), 0, srcSt, srcFrameSt, dSrc, dstSt, dstFrameSt,
                    dDst, static_cast<hipStream_t>(stream));
}

int iqo_hip_band_src_rows(const iqo_hip_plan *h, size_t dstRow0, size_t dstRows, size_t *srcRow0, size_t *srcRows)
{
    if (!h || !srcRow0 || !srcRows || dstRow0 + dstRows > static_cast<size_t>(h->p.dstH))
        return IQO_HIP_EINVAL;
    int s0, s1;
    iqo_amd::band_src_rows(h->p, static_cast<int>(dstRow0), static_cast<int>(dstRow0 + dstRows), &s0, &s1);
    *srcRow0 = static_cast<size_t>(s0);
    *srcRows = static_cast<size_t>(s1 - s0);
    return IQO_HIP_OK;
}

int iqo_hip_resize_band(iqo_hip_plan *h, size_t nFrames, size_t dstRow0, size_t dstRows, size_t srcRow0, size_t srcSt,
                        size_t srcFrameSt, const uint8_t *dSrcWindow, size_t dstSt, size_t dstFrameSt, uint8_t *dDstBand,
                        void *stream)
{
    if (!h)
        return IQO_HIP_EINVAL;
    return run_band(h, nFrames, dstRow0, dstRows, srcRow0, srcSt, srcFrameSt, dSrcWindow, dstSt, dstFrameSt,
                    dDstBand, static_cast<hipStream_t>(stream));
}

// The host-pointer drop-in (reference resize(), LanczosResizer.hpp:47-52 semantics: synchronous,
// host buffers).  Output-row bands are pipelined over three streams: band b's new source rows go
// up on sIn, its kernel runs on sK once they have landed, its output rows come down on sOut, so
// the H2D of band b+1, the kernel of band b and the D2H of band b-1 overlap (PCIe is full
// duplex).  Pinned host buffers are DMA'd in place; pageable ones are staged through pinned
// memory by the calling thread one band ahead of the copy engines.
// One plane of a host-pointer call: the user's buffers and the plane's place in the staging set
// (device and pinned staging at byte offsets sOff / dOff, row pitches sPitch / dPitch; pinSrc /
// pinDst: the user buffer is pinned and DMA'd in place).
struct HostPlane {
    iqo_hip_plan *h;
    size_t srcSt;
    const uint8_t *src;
    size_t dstSt;
    uint8_t *dst;
    size_t sOff, dOff, sPitch, dPitch;
    bool pinSrc, pinDst;
};

// The host-pointer pipeline over one or more planes (the I420 planes of one call share it): each
// plane is cut into output-row bands, and chunk c = (plane, band) goes through
//   stage its new source rows into pinned memory (the copy pool) -> H2D (two upload streams,
//   alternating chunks: two SDMA queues) -> the plane's kernel on its band (sK, after the chunk's
//   uploads) -> D2H of the band (sOut) -> unstage into the user's rows,
// so the host staging of chunk c + 1 overlaps the upload of chunk c, and every plane's transfers
// overlap the other planes' instead of each plane paying a synchronous round trip.
int host_pipeline(HostStage *st, HostPlane *planes, int nPlanes)
{
    struct Chunk {
        int plane, r0, r1;
    };
    Chunk ch[kHostChunks];
    int nc = 0;
    for (int q = 0; q < nPlanes; ++q) {
        const int dstH = planes[q].h->p.dstH;
        const int maxBands = nPlanes == 1 ? kHostBands : q == 0 ? kHostBands / 2 : kHostBands / 4;
        const int bands = std::max(1, std::min(maxBands, dstH / kHostBandRows));
        for (int b = 0; b < bands && nc < kHostChunks; ++b)
            ch[nc++] = Chunk{q, static_cast<int>(static_cast<int64_t>(dstH) * b / bands),
                             static_cast<int>(static_cast<int64_t>(dstH) * (b + 1) / bands)};
    }
    int rowsUp[4] = {0, 0, 0, 0};  // per plane: source rows [0, rowsUp) are queued for upload
    int lastUp[4] = {-1, -1, -1, -1};  // per plane: the chunk that queued the latest upload
    for (int c = 0; c < nc; ++c) {
        HostPlane &P = planes[ch[c].plane];
        const Plan &p = P.h->p;
        const size_t W = static_cast<size_t>(p.srcW), w = static_cast<size_t>(p.dstW);
        int s0, s1;
        iqo_amd::band_src_rows(p, ch[c].r0, ch[c].r1, &s0, &s1);
        const bool lastOfPlane = c == nc - 1 || ch[c + 1].plane != ch[c].plane;
        if (lastOfPlane)
            s1 = p.srcH;
        int &up = rowsUp[ch[c].plane];
        const int prevUp = lastUp[ch[c].plane];
        hipStream_t sUp = (c & 1) ? st->sIn2 : st->sIn;
        if (s1 > up) {
            const size_t n = static_cast<size_t>(s1 - up);
            const uint8_t *from = P.src + static_cast<size_t>(up) * P.srcSt;
            size_t fromSt = P.srcSt;
            if (!P.pinSrc) {
                uint8_t *pin = st->hSrc + P.sOff + static_cast<size_t>(up) * P.sPitch;
                copy_rows_par(pin, P.sPitch, from, P.srcSt, W, n);
                from = pin;
                fromSt = P.sPitch;
            }
            if (hipMemcpy2DAsync(st->dSrc + P.sOff + static_cast<size_t>(up) * P.sPitch, P.sPitch, from, fromSt, W, n,
                                 hipMemcpyHostToDevice, sUp) != hipSuccess)
                return IQO_HIP_EHIP;
            up = s1;
            lastUp[ch[c].plane] = c;
        }
        // the band's rows: this chunk's upload, and the halo rows the plane's previous upload brought
        if (hipEventRecord(st->evIn[c], sUp) != hipSuccess || hipStreamWaitEvent(st->sK, st->evIn[c], 0) != hipSuccess ||
            (prevUp >= 0 && prevUp != c && hipStreamWaitEvent(st->sK, st->evIn[prevUp], 0) != hipSuccess))
            return IQO_HIP_EHIP;
        const size_t rows = static_cast<size_t>(ch[c].r1 - ch[c].r0);
        const size_t sBytes = P.sPitch * static_cast<size_t>(p.srcH), dBytes = P.dPitch * static_cast<size_t>(p.dstH);
        int rc = run_band(P.h, 1, static_cast<size_t>(ch[c].r0), rows, 0, P.sPitch, sBytes, st->dSrc + P.sOff, P.dPitch,
                          dBytes, st->dDst + P.dOff + static_cast<size_t>(ch[c].r0) * P.dPitch, st->sK);
        if (rc)
            return rc;
        if (hipEventRecord(st->evK[c], st->sK) != hipSuccess || hipStreamWaitEvent(st->sOut, st->evK[c], 0) != hipSuccess)
            return IQO_HIP_EHIP;
        uint8_t *to = P.pinDst ? P.dst + static_cast<size_t>(ch[c].r0) * P.dstSt
                               : st->hDst + P.dOff + static_cast<size_t>(ch[c].r0) * P.dPitch;
        if (hipMemcpy2DAsync(to, P.pinDst ? P.dstSt : P.dPitch, st->dDst + P.dOff + static_cast<size_t>(ch[c].r0) * P.dPitch,
                             P.dPitch, w, rows, hipMemcpyDeviceToHost, st->sOut) != hipSuccess ||
            hipEventRecord(st->evOut[c], st->sOut) != hipSuccess)
            return IQO_HIP_EHIP;
    }
    // output bands leave the pinned staging as they land
    for (int c = 0; c < nc; ++c) {
        if (hipEventSynchronize(st->evOut[c]) != hipSuccess)
            return IQO_HIP_EHIP;
        const HostPlane &P = planes[ch[c].plane];
        if (!P.pinDst)
            copy_rows_par(P.dst + static_cast<size_t>(ch[c].r0) * P.dstSt, P.dstSt,
                          st->hDst + P.dOff + static_cast<size_t>(ch[c].r0) * P.dPitch, P.dPitch,
                          static_cast<size_t>(P.h->p.dstW), static_cast<size_t>(ch[c].r1 - ch[c].r0));
    }
    return IQO_HIP_OK;
}

// Large frames, the default: whole-plane copies straight from the user's buffers (pageable ones
// through the HIP runtime's own staging, which runs at close to the PCIe rate: 44 GB/s H2D for a
// 12 MB plane set against 53 GB/s from pinned memory, profiles/r05/pcie_probe.json), every plane's
// upload first, then the kernels, then the downloads, one stream, one synchronisation.  Our own
// banded staging pipeline (host_pipeline: pool memcpy into pinned memory + DMA per band, option
// host_stage = 1) spent more host time on its per-band copies, events and launches than the
// transfers take: C2 Y 0.43 -> 0.24 ms from pageable memory, I420 0.58 -> 0.42 ms; from pinned
// buffers the pipeline took 0.33 / 0.38 ms (profiles/r05/host_latency.txt).
int host_direct(HostStage *st, HostPlane *planes, int nPlanes)
{
    for (int q = 0; q < nPlanes; ++q) {
        const HostPlane &P = planes[q];
        const Plan &p = P.h->p;
        const size_t W = static_cast<size_t>(p.srcW), H = static_cast<size_t>(p.srcH);
        const hipError_t e = (P.srcSt == W && P.sPitch == W)
                                 ? hipMemcpyAsync(st->dSrc + P.sOff, P.src, W * H, hipMemcpyHostToDevice, st->sK)
                                 : hipMemcpy2DAsync(st->dSrc + P.sOff, P.sPitch, P.src, P.srcSt, W, H,
                                                    hipMemcpyHostToDevice, st->sK);
        if (e != hipSuccess)
            return IQO_HIP_EHIP;
    }
    for (int q = 0; q < nPlanes; ++q) {
        const HostPlane &P = planes[q];
        const Plan &p = P.h->p;
        const size_t sBytes = P.sPitch * static_cast<size_t>(p.srcH), dBytes = P.dPitch * static_cast<size_t>(p.dstH);
        const int rc = run_band(P.h, 1, 0, static_cast<size_t>(p.dstH), 0, P.sPitch, sBytes, st->dSrc + P.sOff, P.dPitch,
                                dBytes, st->dDst + P.dOff, st->sK);
        if (rc)
            return rc;
    }
    for (int q = 0; q < nPlanes; ++q) {
        const HostPlane &P = planes[q];
        const Plan &p = P.h->p;
        const size_t w = static_cast<size_t>(p.dstW), hh = static_cast<size_t>(p.dstH);
        const hipError_t e = (P.dstSt == w && P.dPitch == w)
                                 ? hipMemcpyAsync(P.dst, st->dDst + P.dOff, w * hh, hipMemcpyDeviceToHost, st->sK)
                                 : hipMemcpy2DAsync(P.dst, P.dstSt, st->dDst + P.dOff, P.dPitch, w, hh,
                                                    hipMemcpyDeviceToHost, st->sK);
        if (e != hipSuccess)
            return IQO_HIP_EHIP;
    }
    return hipStreamSynchronize(st->sK) == hipSuccess ? IQO_HIP_OK : IQO_HIP_EHIP;
}

static int host_resize(iqo_hip_plan *h, HostStage *st, size_t srcSt, const uint8_t *src, size_t dstSt, uint8_t *dst)
{
    const Plan &p = h->p;
    const size_t W = static_cast<size_t>(p.srcW), w = static_cast<size_t>(p.dstW);
    const size_t sPitch = (W + 15) & ~size_t(15);
    const size_t dPitch = (w + 15) & ~size_t(15);
    const size_t sBytes = sPitch * p.srcH, dBytes = dPitch * p.dstH;
    if (grow_device(&st->dSrc, &st->dSrcCap, sBytes) || grow_device(&st->dDst, &st->dDstCap, dBytes))
        return IQO_HIP_ENOMEM;
    // small frames are always staged: the pinned-memory queries cost more than the copy
    const bool small = sBytes < kHostPipeMinBytes;
    const bool pinSrc = !small && is_pinned_host(src), pinDst = !small && is_pinned_host(dst);
    // pinned staging: the small-frame path and the banded pipeline (host_stage = 1) use it; the
    // default large-frame path (host_direct) copies straight from the caller's buffers
    const bool staged = small || h->hostStage;
    if (staged && !pinSrc && grow_pinned(&st->hSrc, &st->hSrcCap, sBytes))
        return IQO_HIP_ENOMEM;
    if (staged && !pinDst && grow_pinned(&st->hDst, &st->hDstCap, dBytes))
        return IQO_HIP_ENOMEM;

    const int dstH = p.dstH;
    if (small) {
        // small frame: upload, kernel and download in order on one stream, one synchronisation
        // (the pipeline's events and cross-stream waits cost more than they overlap here)
        const uint8_t *from = src;
        size_t fromSt = srcSt;
        if (!pinSrc) {
            copy_rows_par(st->hSrc, sPitch, src, srcSt, W, static_cast<size_t>(p.srcH));
            from = st->hSrc;
            fromSt = sPitch;
        }
        if (hipMemcpy2DAsync(st->dSrc, sPitch, from, fromSt, W, static_cast<size_t>(p.srcH), hipMemcpyHostToDevice,
                             st->sK) != hipSuccess)
            return IQO_HIP_EHIP;
        int rc = run_band(h, 1, 0, static_cast<size_t>(dstH), 0, sPitch, sBytes, st->dSrc, dPitch, dBytes, st->dDst,
                          st->sK);
        if (rc)
            return rc;
        uint8_t *to = pinDst ? dst : st->hDst;
        if (hipMemcpy2DAsync(to, pinDst ? dstSt : dPitch, st->dDst, dPitch, w, static_cast<size_t>(dstH),
                             hipMemcpyDeviceToHost, st->sK) != hipSuccess ||
            hipStreamSynchronize(st->sK) != hipSuccess)
            return IQO_HIP_EHIP;
        if (!pinDst)
            copy_rows_par(dst, dstSt, st->hDst, dPitch, w, static_cast<size_t>(dstH));
        return IQO_HIP_OK;
    }
    HostPlane pl{h, srcSt, src, dstSt, dst, 0, 0, sPitch, dPitch, pinSrc, pinDst};
    return h->hostStage ? host_pipeline(st, &pl, 1) : host_direct(st, &pl, 1);
}

int iqo_hip_resize(iqo_hip_plan *h, size_t srcSt, const uint8_t *src, size_t dstSt, uint8_t *dst)
{
    if (!h || !src || !dst)
        return IQO_HIP_EINVAL;
    const Plan &p = h->p;
    if (srcSt < static_cast<size_t>(p.srcW) || dstSt < static_cast<size_t>(p.dstW))
        return IQO_HIP_EINVAL;
    DeviceGuard guard(h->device);
    if (!guard.ok())
        return IQO_HIP_ENODEV;
    HostStage *st = acquire_stage(h->device);
    if (!st)
        return IQO_HIP_EHIP;
    int rc = host_resize(h, st, srcSt, src, dstSt, dst);
    if (rc) {
        // leave nothing in flight on the staging set before it goes back to the pool
        (void)hipStreamSynchronize(st->sIn);
        (void)hipStreamSynchronize(st->sIn2);
        (void)hipStreamSynchronize(st->sK);
        (void)hipStreamSynchronize(st->sOut);
    }
    release_stage(st);
    return rc;
}

// ---- YUV 4:2:0 (I420): the reference benchmark's three-plane workload (benchmark.cpp:131-229)

struct iqo_hip_yuv_plan {
    iqo_hip_plan *y = nullptr, *c = nullptr;  // luma plan, chroma plan (shared by U and V)
};

int iqo_hip_plan_yuv420(int method, unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH, int device,
                        iqo_hip_yuv_plan **out)
{
    if (!out)
        return IQO_HIP_EINVAL;
    *out = nullptr;
    if (srcW < 2 || srcH < 2 || dstW < 2 || dstH < 2)
        return IQO_HIP_EINVAL;
    iqo_hip_yuv_plan *yp = new (std::nothrow) iqo_hip_yuv_plan();
    if (!yp)
        return IQO_HIP_ENOMEM;
    int rc = IQO_HIP_EINVAL;
    if (method == IQO_METHOD_LANCZOS) {
        // chroma: pxScale 2 (benchmark.cpp:222, sample/resize_yuv420p.cpp:159)
        rc = iqo_hip_plan_lanczos(degree, srcW, srcH, dstW, dstH, 1, device, &yp->y);
        if (!rc)
            rc = iqo_hip_plan_lanczos(degree, srcW / 2, srcH / 2, dstW / 2, dstH / 2, 2, device, &yp->c);
    } else if (method == IQO_METHOD_AREA) {
        rc = iqo_hip_plan_area(srcW, srcH, dstW, dstH, device, &yp->y);
        if (!rc)
            rc = iqo_hip_plan_area(srcW / 2, srcH / 2, dstW / 2, dstH / 2, device, &yp->c);
    } else if (method == IQO_METHOD_LINEAR) {
        rc = iqo_hip_plan_linear(srcW, srcH, dstW, dstH, device, &yp->y);
        if (!rc)
            rc = iqo_hip_plan_linear(srcW / 2, srcH / 2, dstW / 2, dstH / 2, device, &yp->c);
    }
    if (rc) {
        iqo_hip_yuv_plan_destroy(yp);
        return rc;
    }
    *out = yp;
    return IQO_HIP_OK;
}

void iqo_hip_yuv_plan_destroy(iqo_hip_yuv_plan *yp)
{
    if (!yp)
        return;
    iqo_hip_plan_destroy(yp->y);
    iqo_hip_plan_destroy(yp->c);
    delete yp;
}

iqo_hip_plan *iqo_hip_yuv_plane(iqo_hip_yuv_plan *yp, int plane)
{
    if (!yp)
        return nullptr;
    return plane == 0 ? yp->y : plane == 1 ? yp->c : nullptr;
}

int iqo_hip_resize_yuv420_device(iqo_hip_yuv_plan *yp, size_t nFrames, size_t srcStY, size_t srcStUV,
                                 size_t srcFrameSt, const uint8_t *srcY, const uint8_t *srcU, const uint8_t *srcV,
                                 size_t dstStY, size_t dstStUV, size_t dstFrameSt, uint8_t *dstY, uint8_t *dstU,
                                 uint8_t *dstV, void *stream, int *fused)
{
    if (fused)
        *fused = 0;
    if (!yp || !yp->y || !yp->c || !srcY || !srcU || !srcV || !dstY || !dstU || !dstV)
        return IQO_HIP_EINVAL;
    iqo_hip_plan *hy = yp->y, *hc = yp->c;
    const Plan &py = hy->p, &pc = hc->p;
    if (srcStY < static_cast<size_t>(py.srcW) || dstStY < static_cast<size_t>(py.dstW) ||
        srcStUV < static_cast<size_t>(pc.srcW) || dstStUV < static_cast<size_t>(pc.dstW))
        return IQO_HIP_EINVAL;
    if (nFrames == 0)
        return IQO_HIP_OK;
    DeviceGuard guard(hy->device);
    if (!guard.ok())
        return IQO_HIP_ENODEV;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int ky = kernel_for_layout(hy, srcY, srcStY, srcFrameSt, dstY, dstStY, dstFrameSt);
    const int ku = kernel_for_layout(hc, srcU, srcStUV, srcFrameSt, dstU, dstStUV, dstFrameSt);
    const int kv = kernel_for_layout(hc, srcV, srcStUV, srcFrameSt, dstV, dstStUV, dstFrameSt);
    if (ky == ku && ku == kv &&
        (ky == IQO_KERNEL_LANCZOS_STREAM || ky == IQO_KERNEL_AREA_INT || ky == IQO_KERNEL_LINEAR_UP2)) {
        // frames per launch: as run_band
        size_t chunk = std::min<size_t>(65535, hy->chunkFrames > 0 ? static_cast<size_t>(hy->chunkFrames) : 65535);
        const size_t n = (nFrames + chunk - 1) / chunk;
        chunk = (nFrames + n - 1) / n;
        hipError_t e = hipSuccess;
        for (size_t f0 = 0; f0 < nFrames && e == hipSuccess; f0 += chunk) {
            const size_t nf = std::min(chunk, nFrames - f0), so = f0 * srcFrameSt, dof = f0 * dstFrameSt;
            const iqo_amd::Io iy = make_io(nf, srcY + so, srcStY, srcFrameSt, 0, py.srcH, dstY + dof, dstStY, dstFrameSt, 0);
            const iqo_amd::Io iu = make_io(nf, srcU + so, srcStUV, srcFrameSt, 0, pc.srcH, dstU + dof, dstStUV, dstFrameSt, 0);
            const iqo_amd::Io iv = make_io(nf, srcV + so, srcStUV, srcFrameSt, 0, pc.srcH, dstV + dof, dstStUV, dstFrameSt, 0);
            if (ky == IQO_KERNEL_LANCZOS_STREAM)
                e = iqo_amd::launch_yuv420_lanczos(lanczos_dev(hy), iy, lanczos_dev(hc), iu, iv, s);
            else if (ky == IQO_KERNEL_AREA_INT)
                e = iqo_amd::launch_yuv420_area(area_dev(hy), iy, area_dev(hc), iu, iv, s);
            else
                e = iqo_amd::launch_yuv420_linear(linear_dev(hy), iy, linear_dev(hc), iu, iv, s);
        }
        if (e == hipSuccess) {
            if (fused)
                *fused = 1;
            return IQO_HIP_OK;
        }
        if (e != hipErrorNotSupported)
            return IQO_HIP_EHIP;
        (void)hipGetLastError();
    }
    // plane by plane
    int rc = run_band(hy, nFrames, 0, static_cast<size_t>(py.dstH), 0, srcStY, srcFrameSt, srcY, dstStY, dstFrameSt,
                      dstY, s);
    if (!rc)
        rc = run_band(hc, nFrames, 0, static_cast<size_t>(pc.dstH), 0, srcStUV, srcFrameSt, srcU, dstStUV, dstFrameSt,
                      dstU, s);
    if (!rc)
        rc = run_band(hc, nFrames, 0, static_cast<size_t>(pc.dstH), 0, srcStUV, srcFrameSt, srcV, dstStUV, dstFrameSt,
                      dstV, s);
    return rc;
}

int iqo_hip_resize_yuv420(iqo_hip_yuv_plan *yp, size_t srcStY, const uint8_t *srcY, size_t srcStUV,
                          const uint8_t *srcU, const uint8_t *srcV, size_t dstStY, uint8_t *dstY, size_t dstStUV,
                          uint8_t *dstU, uint8_t *dstV)
{
    if (!yp || !yp->y || !yp->c || !srcY || !srcU || !srcV || !dstY || !dstU || !dstV)
        return IQO_HIP_EINVAL;
    {
        // small frames: the three planes staged into one buffer, one upload, the fused device
        // launch (iqo_hip_resize_yuv420_device), one download, one synchronisation
        const Plan &py = yp->y->p, &pc = yp->c->p;
        const size_t W = static_cast<size_t>(py.srcW), H = static_cast<size_t>(py.srcH);
        const size_t Wc = static_cast<size_t>(pc.srcW), Hc = static_cast<size_t>(pc.srcH);
        const size_t w = static_cast<size_t>(py.dstW), hh = static_cast<size_t>(py.dstH);
        const size_t wc = static_cast<size_t>(pc.dstW), hc = static_cast<size_t>(pc.dstH);
        if (srcStY < W || srcStUV < Wc || dstStY < w || dstStUV < wc)
            return IQO_HIP_EINVAL;
        const size_t sY = (W + 15) & ~size_t(15), sC = (Wc + 15) & ~size_t(15);
        const size_t dY = (w + 15) & ~size_t(15), dC = (wc + 15) & ~size_t(15);
        const size_t oU = sY * H, oV = oU + sC * Hc, sBytes = oV + sC * Hc;
        const size_t ou = dY * hh, ov = ou + dC * hc, dBytes = ov + dC * hc;
        if (sBytes < kHostPipeMinBytes) {
            DeviceGuard guard(yp->y->device);
            if (!guard.ok())
                return IQO_HIP_ENODEV;
            HostStage *st = acquire_stage(yp->y->device);
            if (!st)
                return IQO_HIP_EHIP;
            int rc = IQO_HIP_OK;
            if (grow_device(&st->dSrc, &st->dSrcCap, sBytes) || grow_device(&st->dDst, &st->dDstCap, dBytes) ||
                grow_pinned(&st->hSrc, &st->hSrcCap, sBytes) || grow_pinned(&st->hDst, &st->hDstCap, dBytes))
                rc = IQO_HIP_ENOMEM;
            if (!rc) {
                const RowCopy in[3] = {{st->hSrc, sY, srcY, srcStY, W, H}, {st->hSrc + oU, sC, srcU, srcStUV, Wc, Hc},
                                       {st->hSrc + oV, sC, srcV, srcStUV, Wc, Hc}};
                copy_planes_par(in, 3);
                if (hipMemcpyAsync(st->dSrc, st->hSrc, sBytes, hipMemcpyHostToDevice, st->sK) != hipSuccess)
                    rc = IQO_HIP_EHIP;
            }
            if (!rc)
                rc = iqo_hip_resize_yuv420_device(yp, 1, sY, sC, sBytes, st->dSrc, st->dSrc + oU, st->dSrc + oV, dY, dC,
                                                  dBytes, st->dDst, st->dDst + ou, st->dDst + ov, st->sK, nullptr);
            if (!rc && (hipMemcpyAsync(st->hDst, st->dDst, dBytes, hipMemcpyDeviceToHost, st->sK) != hipSuccess ||
                        hipStreamSynchronize(st->sK) != hipSuccess))
                rc = IQO_HIP_EHIP;
            if (!rc) {
                const RowCopy out[3] = {{dstY, dstStY, st->hDst, dY, w, hh}, {dstU, dstStUV, st->hDst + ou, dC, wc, hc},
                                        {dstV, dstStUV, st->hDst + ov, dC, wc, hc}};
                copy_planes_par(out, 3);
            } else {
                (void)hipStreamSynchronize(st->sK);
            }
            release_stage(st);
            return rc;
        }
    }
    // large frames: the three planes through ONE host pipeline (their uploads, kernels and
    // downloads overlap each other; one synchronisation per output chunk at the end)
    const Plan &py = yp->y->p, &pc = yp->c->p;
    const size_t sY = (static_cast<size_t>(py.srcW) + 15) & ~size_t(15), sC = (static_cast<size_t>(pc.srcW) + 15) & ~size_t(15);
    const size_t dY = (static_cast<size_t>(py.dstW) + 15) & ~size_t(15), dC = (static_cast<size_t>(pc.dstW) + 15) & ~size_t(15);
    const size_t oU = sY * static_cast<size_t>(py.srcH), oV = oU + sC * static_cast<size_t>(pc.srcH);
    const size_t sBytes = oV + sC * static_cast<size_t>(pc.srcH);
    const size_t ou = dY * static_cast<size_t>(py.dstH), ov = ou + dC * static_cast<size_t>(pc.dstH);
    const size_t dBytes = ov + dC * static_cast<size_t>(pc.dstH);
    DeviceGuard guard(yp->y->device);
    if (!guard.ok())
        return IQO_HIP_ENODEV;
    HostStage *st = acquire_stage(yp->y->device);
    if (!st)
        return IQO_HIP_EHIP;
    int rc = IQO_HIP_OK;
    if (grow_device(&st->dSrc, &st->dSrcCap, sBytes) || grow_device(&st->dDst, &st->dDstCap, dBytes))
        rc = IQO_HIP_ENOMEM;
    const bool pinY = is_pinned_host(srcY), pinU = is_pinned_host(srcU), pinV = is_pinned_host(srcV);
    const bool pinYd = is_pinned_host(dstY), pinUd = is_pinned_host(dstU), pinVd = is_pinned_host(dstV);
    // (pinned staging only for the banded pipeline, host_stage = 1: host_direct copies straight
    // from the caller's buffers)
    const bool staged = yp->y->hostStage != 0;
    if (!rc && staged && !(pinY && pinU && pinV) && grow_pinned(&st->hSrc, &st->hSrcCap, sBytes))
        rc = IQO_HIP_ENOMEM;
    if (!rc && staged && !(pinYd && pinUd && pinVd) && grow_pinned(&st->hDst, &st->hDstCap, dBytes))
        rc = IQO_HIP_ENOMEM;
    if (!rc) {
        HostPlane pl[3] = {{yp->y, srcStY, srcY, dstStY, dstY, 0, 0, sY, dY, pinY, pinYd},
                           {yp->c, srcStUV, srcU, dstStUV, dstU, oU, ou, sC, dC, pinU, pinUd},
                           {yp->c, srcStUV, srcV, dstStUV, dstV, oV, ov, sC, dC, pinV, pinVd}};
        rc = yp->y->hostStage ? host_pipeline(st, pl, 3) : host_direct(st, pl, 3);
    }
    if (rc) {
        (void)hipStreamSynchronize(st->sIn);
        (void)hipStreamSynchronize(st->sIn2);
        (void)hipStreamSynchronize(st->sK);
        (void)hipStreamSynchronize(st->sOut);
    }
    release_stage(st);
    return rc;
}

// ---- multi-GPU data movement (row-band windows out, bands back; no collective)

namespace {

// Peer access dst -> src enabled once per process and pair (hipDeviceEnablePeerAccess is
// per-context state; a second call reports hipErrorPeerAccessAlreadyEnabled).
bool enable_peer(int dst, int src)
{
    static std::mutex mu;
    static std::vector<std::pair<int, int>> done;
    std::lock_guard<std::mutex> g(mu);
    for (const auto &d : done)
        if (d.first == dst && d.second == src)
            return true;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, dst, src) != hipSuccess || !can)
        return false;
    DeviceGuard guard(dst);
    const hipError_t e = hipDeviceEnablePeerAccess(src, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
        (void)hipGetLastError();
        return false;
    }
    (void)hipGetLastError();
    done.emplace_back(dst, src);
    return true;
}

// nFrames blocks of `bytes` at frame strides, one 2-D copy (the frame stride is the pitch).
hipError_t copy_blocks(void *dst, size_t dfs, const void *src, size_t sfs, size_t bytes, size_t n, hipMemcpyKind k,
                       hipStream_t s)
{
    if (n == 1 || (dfs == bytes && sfs == bytes))
        return hipMemcpyAsync(dst, src, bytes * n, k, s);
    return hipMemcpy2DAsync(dst, dfs, src, sfs, bytes, n, k, s);
}

} // namespace

int iqo_hip_copy_frames(void *dst, int dstDevice, size_t dstFrameSt, const void *src, int srcDevice, size_t srcFrameSt,
                        size_t bytesPerFrame, size_t nFrames, void *stream, int *path)
{
    if (path)
        *path = -1;
    if (!dst || !src || (dstDevice < 0 && srcDevice < 0))
        return IQO_HIP_EINVAL;
    if (bytesPerFrame == 0 || nFrames == 0)
        return IQO_HIP_OK;
    if (nFrames > 1 && (dstFrameSt < bytesPerFrame || srcFrameSt < bytesPerFrame))
        return IQO_HIP_EINVAL;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || dstDevice >= count || srcDevice >= count)
        return IQO_HIP_ENODEV;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const auto u8 = [](const void *p) { return static_cast<const uint8_t *>(p); };
    if (dstDevice < 0 || srcDevice < 0) {  // host <-> device
        DeviceGuard guard(dstDevice >= 0 ? dstDevice : srcDevice);
        if (!guard.ok())
            return IQO_HIP_ENODEV;
        const hipMemcpyKind k = srcDevice < 0 ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
        if (copy_blocks(dst, dstFrameSt, src, srcFrameSt, bytesPerFrame, nFrames, k, s) != hipSuccess)
            return IQO_HIP_EHIP;
        if (path)
            *path = 3;
        return IQO_HIP_OK;
    }
    DeviceGuard guard(dstDevice);
    if (!guard.ok())
        return IQO_HIP_ENODEV;
    if (dstDevice == srcDevice) {
        if (copy_blocks(dst, dstFrameSt, src, srcFrameSt, bytesPerFrame, nFrames, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return IQO_HIP_EHIP;
        if (path)
            *path = 0;
        return IQO_HIP_OK;
    }
    if (enable_peer(dstDevice, srcDevice)) {
        // peer DMA over xGMI, one copy per frame block (contiguous blocks: one copy in all)
        const bool contig = nFrames == 1 || (dstFrameSt == bytesPerFrame && srcFrameSt == bytesPerFrame);
        const size_t n = contig ? 1 : nFrames, b = contig ? bytesPerFrame * nFrames : bytesPerFrame;
        for (size_t f = 0; f < n; ++f)
            if (hipMemcpyPeerAsync(static_cast<uint8_t *>(dst) + f * dstFrameSt, dstDevice, u8(src) + f * srcFrameSt,
                                   srcDevice, b, s) != hipSuccess)
                return IQO_HIP_EHIP;
        if (path)
            *path = 1;
        return IQO_HIP_OK;
    }
    // no peer path: stage through pinned host memory, block by block, synchronously.  The blocking
    // hipMemcpy calls run on the devices' null streams, which a caller's non-blocking stream does
    // not order against: first drain `stream` (work still writing src or reading dst) and the
    // source device, so this route is ordered like the stream-ordered ones; when it returns the
    // copy has landed (iqo_hip.h).
    if (s && hipStreamSynchronize(s) != hipSuccess)
        return IQO_HIP_EHIP;
    {
        DeviceGuard sg(srcDevice);
        if (!sg.ok() || hipDeviceSynchronize() != hipSuccess)
            return IQO_HIP_EHIP;
    }
    uint8_t *h = nullptr;
    if (hipHostMalloc(reinterpret_cast<void **>(&h), bytesPerFrame, hipHostMallocDefault) != hipSuccess)
        return IQO_HIP_ENOMEM;
    int rc = IQO_HIP_OK;
    for (size_t f = 0; f < nFrames && rc == IQO_HIP_OK; ++f) {
        {
            DeviceGuard sg(srcDevice);
            if (!sg.ok() || hipMemcpy(h, u8(src) + f * srcFrameSt, bytesPerFrame, hipMemcpyDeviceToHost) != hipSuccess)
                rc = IQO_HIP_EHIP;
        }
        if (rc == IQO_HIP_OK &&
            hipMemcpy(static_cast<uint8_t *>(dst) + f * dstFrameSt, h, bytesPerFrame, hipMemcpyHostToDevice) != hipSuccess)
            rc = IQO_HIP_EHIP;
    }
    (void)hipHostFree(h);
    if (path && rc == IQO_HIP_OK)
        *path = 2;
    return rc;
}

int iqo_hip_ipc_export(const void *devPtr, iqo_hip_ipc_handle *handle)
{
    static_assert(sizeof(hipIpcMemHandle_t) <= sizeof(handle->bytes), "IPC handle size");
    if (!devPtr || !handle)
        return IQO_HIP_EINVAL;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, const_cast<void *>(devPtr)) != hipSuccess || !base)
        return IQO_HIP_EHIP;
    hipIpcMemHandle_t h;
    if (hipIpcGetMemHandle(&h, base) != hipSuccess)
        return IQO_HIP_EHIP;
    std::memset(handle, 0, sizeof(*handle));
    std::memcpy(handle->bytes, &h, sizeof(h));
    handle->offset = static_cast<uint64_t>(static_cast<const uint8_t *>(devPtr) - static_cast<const uint8_t *>(base));
    return IQO_HIP_OK;
}

int iqo_hip_ipc_open(const iqo_hip_ipc_handle *handle, int device, void **devPtr)
{
    if (!handle || !devPtr)
        return IQO_HIP_EINVAL;
    *devPtr = nullptr;
    DeviceGuard guard(device);
    if (!guard.ok())
        return IQO_HIP_ENODEV;
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle->bytes, sizeof(h));
    void *base = nullptr;
    if (hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess || !base)
        return IQO_HIP_EHIP;
    *devPtr = static_cast<uint8_t *>(base) + handle->offset;
    return IQO_HIP_OK;
}

int iqo_hip_ipc_close(void *devPtr, const iqo_hip_ipc_handle *handle)
{
    if (!devPtr || !handle)
        return IQO_HIP_EINVAL;
    return hipIpcCloseMemHandle(static_cast<uint8_t *>(devPtr) - handle->offset) == hipSuccess ? IQO_HIP_OK
                                                                                                : IQO_HIP_EHIP;
}

const char *iqo_hip_strerror(int status)
{
    switch (status) {
    case IQO_HIP_OK:
        return "ok";
    case IQO_HIP_EINVAL:
        return "invalid argument";
    case IQO_HIP_ENODEV:
        return "no usable gfx950 device";
    case IQO_HIP_ENOMEM:
        return "out of memory";
    case IQO_HIP_EHIP:
        return "HIP runtime or kernel launch failure";
    case IQO_HIP_EUNSUP:
        return "unsupported shape or layout";
    default:
        return "unknown status";
    }
}

const char *iqo_hip_version(void) { return "libiqo_amd 0.1 (gfx950)"; }

int iqo_host_tables(int method, unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH, size_t pxScale,
                    int axis, int *nTaps, int *nPhases, int32_t *buf, size_t cap)
{
    if (method < 0 || method > 2)
        return IQO_HIP_EINVAL;
    AxisPlan x, y;
    std::string err;
    if (!iqo_amd::build_tables(static_cast<iqo_amd::Method>(method), degree, srcW, srcH, dstW, dstH, pxScale, &x, &y, &err))
        return IQO_HIP_EINVAL;
    const AxisPlan &a = axis ? y : x;
    if (nTaps)
        *nTaps = a.taps;
    if (nPhases)
        *nPhases = a.phases;
    if (buf && cap >= a.table.size())
        std::memcpy(buf, a.table.data(), a.table.size() * sizeof(int32_t));
    return static_cast<int>(a.table.size());
}

int iqo_host_band_src_rows(int method, unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                           size_t pxScale, size_t dstRow0, size_t dstRows, size_t *srcRow0, size_t *srcRows)
{
    if (method < 0 || method > 2 || !srcRow0 || !srcRows)
        return IQO_HIP_EINVAL;
    Plan p;
    std::string err;
    if (!iqo_amd::build_plan(static_cast<iqo_amd::Method>(method), degree, srcW, srcH, dstW, dstH, pxScale, &p, &err))
        return IQO_HIP_EINVAL;
    if (dstRow0 + dstRows > dstH)
        return IQO_HIP_EINVAL;
    int s0, s1;
    iqo_amd::band_src_rows(p, static_cast<int>(dstRow0), static_cast<int>(dstRow0 + dstRows), &s0, &s1);
    *srcRow0 = static_cast<size_t>(s0);
    *srcRows = static_cast<size_t>(s1 - s0);
    return IQO_HIP_OK;
}

int iqo_host_kernel_for(int method, unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH, size_t pxScale)
{
    if (method < 0 || method > 2)
        return IQO_HIP_EINVAL;
    iqo_hip_plan h;  // host half of a plan only: no device memory
    std::string err;
    if (!iqo_amd::build_plan(static_cast<iqo_amd::Method>(method), degree, srcW, srcH, dstW, dstH, pxScale, &h.p, &err))
        return IQO_HIP_EINVAL;
    if (h.p.kernel != IQO_KERNEL_GENERAL)
        return h.p.kernel;
    iqo_amd::build_tile_tables(h.p, &h.tt);
    if (h.tt.ok)
        iqo_amd::build_walk_tables(h.p, h.tt, &h.wt);
    iqo_amd::build_up2(h.p, h.wt, &h.ut);
    iqo_amd::build_d32(h.p, h.wt, &h.dt);
    iqo_amd::build_d31(h.p, &h.t31);
    iqo_amd::build_ryx(h.p, &h.ryx);
    if (!h.ryx.ok)
        iqo_amd::build_ryg(h.p, &h.ryx);
    if (h.ryx.ok && ryx_dev(&h).parts == 0)
        h.ryx = iqo_amd::RyxTables();
    iqo_amd::build_a32(h.p, &h.at);
    iqo_amd::build_u23(h.p, &h.vt);
    iqo_amd::build_l23(h.p, &h.lt);
    return plan_kernel(&h);
}

} // extern "C"
