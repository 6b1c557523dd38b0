// resizers.cpp -- the reference's public classes (iqo::LanczosResizer / AreaResizer /
// LinearResizer, include/libiqo/*.hpp) on the HIP backend, with the reference's fallback.
//
// Reference dispatch being replaced: src/IQOLanczosResizer.cpp:7-49 (and the Area / Linear
// twins): CPUID probing, *ResizerImpl_new<Arch>() for the best compiled-in SIMD implementation,
// Generic when none is available (:33), m_Impl->init(); resize() forwards.  Here:
//   * a usable gfx950 device (iqo_hip_available() > 0) -> the impl owns an iqo_hip_plan on the
//     caller's current HIP device (the GPU path every parity test and benchmark measures);
//   * no device -> the impl owns the host plan and runs cpu_generic.cpp, the product's own CPU
//     restatement (never the oracle), as the reference runs Generic;
//   * a device-side failure during resize() (IQO_HIP_ENODEV / _EHIP / _ENOMEM: device lost, HIP
//     runtime error, allocation failure) -> a one-time message on stderr, then the CPU path for
//     that call (the public API has no error channel);
//   * any other status (IQO_HIP_EINVAL / _EUNSUP: a plan / kernel / layout mismatch, i.e. a bug
//     or an unsupported argument, not a missing device) -> a message on EVERY such call, then the
//     CPU path.
// IQO_REQUIRE_HIP=1 in the environment turns every fallback into an abort: tests/test_gpu_parity.py
// sets it for the whole GPU test process and its children, so no GPU test can pass on the CPU
// path.  IQO_DROPIN_REPORT=1 prints the backend counts at exit (for binaries that cannot call
// iqo_dropin_backend_counts, e.g. the reference's own tools compiled unchanged), and
// IQO_DROPIN_DUMP=<dir> writes the output of the first kDumpCalls resize() calls of the process
// to <dir>/resize<k>_<W>x<H>.raw (tight rows) so such a binary's pixels can be checked.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include <hip/hip_runtime_api.h>

#include "cpu_generic.hpp"
#include "iqo_hip.h"
#include "libiqo/AreaResizer.hpp"
#include "libiqo/DeviceResizer.hpp"
#include "libiqo/LanczosResizer.hpp"
#include "libiqo/LinearResizer.hpp"
#include "plan.hpp"

namespace iqo {

namespace {

[[noreturn]] void fatal(const char *what, int status)
{
    std::fprintf(stderr, "libiqo_amd: %s failed: %s (%d)\n", what, iqo_hip_strerror(status), status);
    std::abort();
}

bool require_hip()
{
    const char *e = std::getenv("IQO_REQUIRE_HIP");
    return e && *e && std::strcmp(e, "0") != 0;
}

int current_device()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
        dev = 0;
    return dev;
}

std::atomic<int> g_cpuResizers{0}, g_hipResizers{0};
std::atomic<int> g_cpuCalls{0}, g_hipCalls{0};  // resize() calls on each backend
std::atomic<int> g_cpuFallbacks{0};              // ... of which HIP objects' calls that fell back
std::atomic<bool> g_warned{false};

void report_at_exit()
{
    std::fprintf(stderr, "libiqo_amd drop-in: objects hip=%d cpu=%d, resize calls hip=%d cpu=%d\n", g_hipResizers.load(),
                 g_cpuResizers.load(), g_hipCalls.load(), g_cpuCalls.load());
}

// IQO_DROPIN_REPORT / IQO_DROPIN_DUMP (see the header comment); read once
constexpr int kDumpCalls = 8;
struct DebugEnv {
    const char *dumpDir = nullptr;
    std::atomic<int> dumped{0};
    DebugEnv()
    {
        const char *r = std::getenv("IQO_DROPIN_REPORT");
        if (r && *r && std::strcmp(r, "0") != 0)
            std::atexit(report_at_exit);
        const char *d = std::getenv("IQO_DROPIN_DUMP");
        dumpDir = d && *d ? d : nullptr;
    }
};
DebugEnv &debug_env()
{
    static DebugEnv e;
    return e;
}

void dump_output(size_t dstW, size_t dstH, size_t dstSt, const unsigned char *dst)
{
    DebugEnv &e = debug_env();
    if (!e.dumpDir)
        return;
    const int k = e.dumped.fetch_add(1);
    if (k >= kDumpCalls)
        return;
    const std::string path = std::string(e.dumpDir) + "/resize" + std::to_string(k) + "_" + std::to_string(dstW) +
                             "x" + std::to_string(dstH) + ".raw";
    if (FILE *f = std::fopen(path.c_str(), "wb")) {
        for (size_t y = 0; y < dstH; ++y)
            std::fwrite(dst + y * dstSt, 1, dstW, f);
        std::fclose(f);
    }
}

struct PlanHolder {
    iqo_hip_plan *plan = nullptr;  // GPU backend, or
    iqo_amd::Plan host;            // the CPU backend's plan (built when plan == nullptr)

    ~PlanHolder() { iqo_hip_plan_destroy(plan); }

    // hipPlan: the iqo_hip_plan_* call for this method on device `dev`; hostPlan: build_plan
    template <typename HipPlan, typename HostPlan>
    void init(const char *what, HipPlan hipPlan, HostPlan hostPlan)
    {
        debug_env();
        int rc = IQO_HIP_ENODEV;
        if (iqo_hip_available() > 0)
            rc = hipPlan(current_device(), &plan);
        if (rc == 0) {
            ++g_hipResizers;
            return;
        }
        if (require_hip())
            fatal(what, rc);
        plan = nullptr;
        std::string err;
        if (!hostPlan(&host, &err)) {
            std::fprintf(stderr, "libiqo_amd: %s: %s\n", what, err.c_str());
            std::abort();
        }
        ++g_cpuResizers;
    }

    void resize(size_t srcSt, const unsigned char *src, size_t dstSt, unsigned char *dst)
    {
        if (plan) {
            const int rc = iqo_hip_resize(plan, srcSt, src, dstSt, dst);
            if (rc == 0) {
                ++g_hipCalls;
                if (debug_env().dumpDir) {
                    iqo_hip_plan_desc d;
                    if (iqo_hip_plan_query(plan, &d) == 0)
                        dump_output(d.dstW, d.dstH, dstSt, dst);
                }
                return;
            }
            if (require_hip())
                fatal("resize", rc);
            const bool deviceSide = rc == IQO_HIP_ENODEV || rc == IQO_HIP_EHIP || rc == IQO_HIP_ENOMEM;
            if (!deviceSide)  // a plan / kernel / layout mismatch: say so on every call
                std::fprintf(stderr, "libiqo_amd: HIP resize rejected the call (%s, %d); using the CPU path\n",
                             iqo_hip_strerror(rc), rc);
            else if (!g_warned.exchange(true))
                std::fprintf(stderr, "libiqo_amd: HIP resize failed (%s, %d); using the CPU path\n",
                             iqo_hip_strerror(rc), rc);
            if (host.dstW == 0) {
                iqo_hip_plan_desc d;
                std::string err;
                if (iqo_hip_plan_query(plan, &d) != 0 ||
                    !iqo_amd::build_plan(static_cast<iqo_amd::Method>(d.method), m_degree, d.srcW, d.srcH, d.dstW,
                                         d.dstH, m_pxScale, &host, &err))
                    fatal("resize (CPU fallback plan)", rc);
            }
        }
        if (plan)
            ++g_cpuFallbacks;
        ++g_cpuCalls;
        iqo_amd::cpu_resize(host, srcSt, src, dstSt, dst);
        dump_output(static_cast<size_t>(host.dstW), static_cast<size_t>(host.dstH), dstSt, dst);
    }

    unsigned m_degree = 0;
    size_t m_pxScale = 1;
};

} // namespace

class ILanczosResizerImpl : public PlanHolder {};
class IAreaResizerImpl : public PlanHolder {};
class ILinearResizerImpl : public PlanHolder {};

LanczosResizer::LanczosResizer(unsigned int degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                               size_t pxScale)
    : m_Impl(new ILanczosResizerImpl())
{
    m_Impl->m_degree = degree;
    m_Impl->m_pxScale = pxScale;
    m_Impl->init(
        "LanczosResizer construction",
        [&](int dev, iqo_hip_plan **p) { return iqo_hip_plan_lanczos(degree, srcW, srcH, dstW, dstH, pxScale, dev, p); },
        [&](iqo_amd::Plan *p, std::string *e) {
            return iqo_amd::build_plan(iqo_amd::kLanczos, degree, srcW, srcH, dstW, dstH, pxScale, p, e);
        });
}

LanczosResizer::~LanczosResizer() { delete m_Impl; }

void LanczosResizer::resize(size_t srcSt, const unsigned char *src, size_t dstSt, unsigned char *dst)
{
    m_Impl->resize(srcSt, src, dstSt, dst);
}

AreaResizer::AreaResizer(size_t srcW, size_t srcH, size_t dstW, size_t dstH) : m_Impl(new IAreaResizerImpl())
{
    m_Impl->init(
        "AreaResizer construction",
        [&](int dev, iqo_hip_plan **p) { return iqo_hip_plan_area(srcW, srcH, dstW, dstH, dev, p); },
        [&](iqo_amd::Plan *p, std::string *e) {
            return iqo_amd::build_plan(iqo_amd::kArea, 0, srcW, srcH, dstW, dstH, 1, p, e);
        });
}

AreaResizer::~AreaResizer() { delete m_Impl; }

void AreaResizer::resize(size_t srcSt, const unsigned char *src, size_t dstSt, unsigned char *dst)
{
    m_Impl->resize(srcSt, src, dstSt, dst);
}

LinearResizer::LinearResizer(size_t srcW, size_t srcH, size_t dstW, size_t dstH) : m_Impl(new ILinearResizerImpl())
{
    m_Impl->init(
        "LinearResizer construction",
        [&](int dev, iqo_hip_plan **p) { return iqo_hip_plan_linear(srcW, srcH, dstW, dstH, dev, p); },
        [&](iqo_amd::Plan *p, std::string *e) {
            return iqo_amd::build_plan(iqo_amd::kLinear, 0, srcW, srcH, dstW, dstH, 1, p, e);
        });
}

LinearResizer::~LinearResizer() { delete m_Impl; }

void LinearResizer::resize(size_t srcSt, const unsigned char *src, size_t dstSt, unsigned char *dst)
{
    m_Impl->resize(srcSt, src, dstSt, dst);
}

DeviceResizer::DeviceResizer(Method method, size_t srcW, size_t srcH, size_t dstW, size_t dstH, unsigned int degree,
                             size_t pxScale, int device)
    : m_Plan(0), m_Status(0)
{
    if (method == kLanczos)
        m_Status = iqo_hip_plan_lanczos(degree, srcW, srcH, dstW, dstH, pxScale, device, &m_Plan);
    else if (method == kArea)
        m_Status = iqo_hip_plan_area(srcW, srcH, dstW, dstH, device, &m_Plan);
    else
        m_Status = iqo_hip_plan_linear(srcW, srcH, dstW, dstH, device, &m_Plan);
}

DeviceResizer::~DeviceResizer() { iqo_hip_plan_destroy(m_Plan); }

int DeviceResizer::resize(size_t nFrames, size_t srcSt, size_t srcFrameSt, const uint8_t *dSrc, size_t dstSt,
                          size_t dstFrameSt, uint8_t *dDst, void *stream)
{
    if (m_Status)
        return m_Status;
    return iqo_hip_resize_device(m_Plan, nFrames, srcSt, srcFrameSt, dSrc, dstSt, dstFrameSt, dDst, stream);
}

} // namespace iqo

// How many drop-in objects this process built on each backend, the CPU count including resize()
// calls of HIP objects that fell back to the CPU (tests and the tools report it, so a run on the
// CPU path is visible).
extern "C" void iqo_dropin_backend_counts(int *hip, int *cpu)
{
    if (hip)
        *hip = iqo::g_hipResizers.load();
    if (cpu)
        *cpu = iqo::g_cpuResizers.load() + iqo::g_cpuFallbacks.load();
}
