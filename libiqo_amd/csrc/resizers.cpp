// resizers.cpp -- the reference's public classes (iqo::LanczosResizer / AreaResizer /
// LinearResizer, include/libiqo/*.hpp) implemented on the HIP backend through the C ABI.
//
// Reference dispatch being replaced: src/IQOLanczosResizer.cpp:7-49 (and the Area / Linear
// twins): CPUID probing + *ResizerImpl_new<Arch>() + m_Impl->init(); resize() forwards.  Here the
// private impl object simply owns an iqo_hip_plan on the caller's current HIP device.
#include <cstdio>
#include <cstdlib>

#include <hip/hip_runtime_api.h>

#include "iqo_hip.h"
#include "libiqo/AreaResizer.hpp"
#include "libiqo/DeviceResizer.hpp"
#include "libiqo/LanczosResizer.hpp"
#include "libiqo/LinearResizer.hpp"

namespace iqo {

namespace {

[[noreturn]] void fatal(const char *what, int status)
{
    std::fprintf(stderr, "libiqo_amd: %s failed: %s (%d)\n", what, iqo_hip_strerror(status), status);
    std::abort();
}

int current_device()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
        dev = 0;
    return dev;
}

struct PlanHolder {
    iqo_hip_plan *plan = nullptr;
    ~PlanHolder() { iqo_hip_plan_destroy(plan); }
    void resize(size_t srcSt, const unsigned char *src, size_t dstSt, unsigned char *dst)
    {
        int rc = iqo_hip_resize(plan, srcSt, src, dstSt, dst);
        if (rc)
            fatal("resize", rc);
    }
};

} // namespace

class ILanczosResizerImpl : public PlanHolder {};
class IAreaResizerImpl : public PlanHolder {};
class ILinearResizerImpl : public PlanHolder {};

LanczosResizer::LanczosResizer(unsigned int degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                               size_t pxScale)
    : m_Impl(new ILanczosResizerImpl())
{
    int rc = iqo_hip_plan_lanczos(degree, srcW, srcH, dstW, dstH, pxScale, current_device(), &m_Impl->plan);
    if (rc)
        fatal("LanczosResizer construction", rc);
}

LanczosResizer::~LanczosResizer() { delete m_Impl; }

void LanczosResizer::resize(size_t srcSt, const unsigned char *src, size_t dstSt, unsigned char *dst)
{
    m_Impl->resize(srcSt, src, dstSt, dst);
}

AreaResizer::AreaResizer(size_t srcW, size_t srcH, size_t dstW, size_t dstH) : m_Impl(new IAreaResizerImpl())
{
    int rc = iqo_hip_plan_area(srcW, srcH, dstW, dstH, current_device(), &m_Impl->plan);
    if (rc)
        fatal("AreaResizer construction", rc);
}

AreaResizer::~AreaResizer() { delete m_Impl; }

void AreaResizer::resize(size_t srcSt, const unsigned char *src, size_t dstSt, unsigned char *dst)
{
    m_Impl->resize(srcSt, src, dstSt, dst);
}

LinearResizer::LinearResizer(size_t srcW, size_t srcH, size_t dstW, size_t dstH) : m_Impl(new ILinearResizerImpl())
{
    int rc = iqo_hip_plan_linear(srcW, srcH, dstW, dstH, current_device(), &m_Impl->plan);
    if (rc)
        fatal("LinearResizer construction", rc);
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
