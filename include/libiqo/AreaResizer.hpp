#pragma once

// Drop-in replacement of libiqo's iqo::AreaResizer (include/libiqo/AreaResizer.hpp:14-56).
// See LanczosResizer.hpp for backend and error behaviour.

#include <stddef.h>

namespace iqo {

    class IAreaResizerImpl;

    class AreaResizer
    {
    public:
        //! Box-average (area) resampling srcW x srcH -> dstW x dstH.
        AreaResizer(size_t srcW, size_t srcH, size_t dstW, size_t dstH);
        ~AreaResizer();

        //! Resize one single-channel U8 image; strides are in bytes; host pointers.
        void resize(size_t srcSt, const unsigned char * src, size_t dstSt, unsigned char * dst);

    private:
        AreaResizer(const AreaResizer &);
        AreaResizer & operator=(const AreaResizer &);

        IAreaResizerImpl * m_Impl;
    };

}
