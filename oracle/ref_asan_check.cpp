// ref_asan_check.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Runs ONE shape through the reference's Generic implementation built with
// -fsanitize=address,undefined (oracle/Makefile target `_ref/ref_asan_check`), with exactly
// sized src/dst buffers, so that shapes on which the reference itself reads out of bounds
// (Area non-integer ratios, Linear >2x / downsampling) or divides by
// zero are excluded from the golden sweep.  Exit status 0 = clean.
//
// usage: ref_asan_check method degree srcW srcH dstW dstH pxScale
#include <stdint.h>
#include <stdlib.h>

#include "IQOAreaResizerImpl.hpp"
#include "IQOLanczosResizerImpl.hpp"
#include "IQOLinearResizerImpl.hpp"

int main(int argc, char **argv)
{
    if (argc != 8)
        return 2;
    int method = atoi(argv[1]);
    unsigned degree = static_cast<unsigned>(atoi(argv[2]));
    size_t sw = strtoul(argv[3], 0, 10), sh = strtoul(argv[4], 0, 10);
    size_t dw = strtoul(argv[5], 0, 10), dh = strtoul(argv[6], 0, 10);
    size_t px = strtoul(argv[7], 0, 10);
    uint8_t *src = static_cast<uint8_t *>(malloc(sw * sh));
    uint8_t *dst = static_cast<uint8_t *>(malloc(dw * dh));
    for (size_t i = 0; i < sw * sh; ++i)
        src[i] = static_cast<uint8_t>((i * 2654435761u) >> 24);
    if (method == 0) {
        iqo::ILanczosResizerImpl *p = iqo::LanczosResizerImpl_new<iqo::ArchGeneric>();
        p->init(degree, sw, sh, dw, dh, px);
        p->resize(sw, src, dw, dst);
        delete p;
    } else if (method == 1) {
        iqo::IAreaResizerImpl *p = iqo::AreaResizerImpl_new<iqo::ArchGeneric>();
        p->init(sw, sh, dw, dh);
        p->resize(sw, src, dw, dst);
        delete p;
    } else {
        iqo::ILinearResizerImpl *p = iqo::LinearResizerImpl_new<iqo::ArchGeneric>();
        p->init(sw, sh, dw, dh);
        p->resize(sw, src, dw, dst);
        delete p;
    }
    free(src);
    free(dst);
    return 0;
}
