#pragma once

// Drop-in replacement of libiqo's iqo::LanczosResizer (include/libiqo/LanczosResizer.hpp:14-60):
// same constructor and resize() signatures, output bytes identical to the reference's Generic
// implementation.  Work runs on the current HIP device (gfx950); a HIP failure prints a message
// and aborts (the reference API has no error channel and this library has no CPU fallback).

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
