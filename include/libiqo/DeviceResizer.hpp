#pragma once

// Additive extension (not in the reference API): batched, device-resident, stream-ordered
// resizing for callers that keep frames in HBM.  Thin RAII wrapper over include/iqo_hip.h.

#include <stddef.h>
#include <stdint.h>

struct iqo_hip_plan;

namespace iqo {

    class DeviceResizer
    {
    public:
        enum Method { kLanczos = 0, kArea = 1, kLinear = 2 };

        //! degree / pxScale are used by kLanczos only; device = HIP ordinal.
        DeviceResizer(Method method, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                      unsigned int degree = 3, size_t pxScale = 1, int device = 0);
        ~DeviceResizer();

        //! Returns 0 or a negative IQO_HIP_* status.  Asynchronous on `stream` (hipStream_t).
        int resize(size_t nFrames, size_t srcSt, size_t srcFrameSt, const uint8_t * dSrc,
                   size_t dstSt, size_t dstFrameSt, uint8_t * dDst, void * stream = 0);

        //! Construction status (0 = ready).
        int status() const { return m_Status; }

    private:
        DeviceResizer(const DeviceResizer &);
        DeviceResizer & operator=(const DeviceResizer &);

        iqo_hip_plan * m_Plan;
        int m_Status;
    };

}
