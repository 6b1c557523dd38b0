#pragma once

// Drop-in replacement of libiqo's iqo::LinearResizer (include/libiqo/LinearResizer.hpp:14-56).
// See LanczosResizer.hpp for backend and error behaviour.

#include <stddef.h>

namespace iqo {

    class ILinearResizerImpl;

    class LinearResizer
    {
    public:
        //! Centre-aligned bilinear resampling srcW x srcH -> dstW x dstH.
        LinearResizer(size_t srcW, size_t srcH, size_t dstW, size_t dstH);
        ~LinearResizer();

        //! Resize one single-channel U8 image; strides are in bytes; host pointers.
        void resize(size_t srcSt, const unsigned char * src, size_t dstSt, unsigned char * dst);

    private:
        LinearResizer(const LinearResizer &);
        LinearResizer & operator=(const LinearResizer &);

        ILinearResizerImpl * m_Impl;
    };

}
