#pragma once

// Drop-in replacement of libiqo's iqo::LanczosResizer (include/libiqo/LanczosResizer.hpp:14-60):
// same constructor and resize() signatures, output bytes identical to the reference's Generic
// implementation.  Backend, chosen at construction like the reference's CPUID dispatch
// (src/IQOLanczosResizer.cpp:15-36): the current HIP device when a gfx950 device is present,
// otherwise the library's CPU restatement of Generic (libiqo_amd/csrc/cpu_generic.cpp).  A HIP
// failure inside resize() prints one message and runs that call on the CPU path (the API has no
// error channel).  IQO_REQUIRE_HIP=1 in the environment makes both fallbacks abort instead.

#include <stddef.h>

namespace iqo {

    class ILanczosResizerImpl;

    class LanczosResizer
    {
    public:
        //! Build tables for Lanczos-`degree` resampling srcW x srcH -> dstW x dstH.
        //! pxScale is the source pixel pitch in luma pixels (2 for YUV420 chroma planes).
        LanczosResizer(unsigned int degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                       size_t pxScale = 1);
        ~LanczosResizer();

        //! Resize one single-channel U8 image; strides are in bytes; host pointers.
        void resize(size_t srcSt, const unsigned char * src, size_t dstSt, unsigned char * dst);

    private:
        LanczosResizer(const LanczosResizer &);             // non-copyable
        LanczosResizer & operator=(const LanczosResizer &);

        ILanczosResizerImpl * m_Impl;
    };

}
