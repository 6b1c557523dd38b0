// ref_tables.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Table introspection of the reference's Generic implementations (SURVEY.md §8c "Table
// introspection"): this TU opens the private members of the reference classes and #includes
// the reference's Generic translation units from /root/reference/src (compiled in place by
// oracle/Makefile, never copied), so the golden generator can dump the quantised int16/u16
// coefficient tables built by init():
//   LanczosResizerImpl<ArchGeneric>::init  src/IQOLanczosResizerImpl_Generic.cpp:291-339
//   AreaResizerImpl<ArchGeneric>::init     src/IQOAreaResizerImpl_Generic.cpp:174-220
//   LinearResizerImpl<ArchGeneric>::init   src/IQOLinearResizerImpl_Generic.cpp:157-191
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <stddef.h>
#include <stdint.h>
#include <vector>

#define private public
#include "IQOAreaResizerImpl_Generic.cpp"
#include "IQOLanczosResizerImpl_Generic.cpp"
#include "IQOLinearResizerImpl_Generic.cpp"
#undef private

namespace {
template <class V>
int dump(const V &tab, ptrdiff_t nTaps, ptrdiff_t nPhases, int *oTaps, int *oPhases, int32_t *buf, size_t cap)
{
    *oTaps = static_cast<int>(nTaps);
    *oPhases = static_cast<int>(nPhases);
    size_t total = static_cast<size_t>(nTaps * nPhases);
    if (buf && cap >= total)
        for (size_t i = 0; i < total; ++i)
            buf[i] = static_cast<int32_t>(tab[i]);
    return static_cast<int>(total);
}
} // namespace

extern "C" int iqo_ref_tables(int method, unsigned degree, size_t sw, size_t sh, size_t dw, size_t dh,
                              size_t px, int axis, int *nTaps, int *nPhases, int32_t *buf, size_t cap)
{
    if (!sw || !sh || !dw || !dh)
        return -1;
    if (method == 0) {
        iqo::LanczosResizerImpl<iqo::ArchGeneric> impl;
        impl.init(degree, sw, sh, dw, dh, px);
        return axis ? dump(impl.m_TablesY, impl.m_NumCoefsY, impl.m_NumTablesY, nTaps, nPhases, buf, cap)
                    : dump(impl.m_TablesX, impl.m_NumCoefsX, impl.m_NumTablesX, nTaps, nPhases, buf, cap);
    }
    if (method == 1) {
        iqo::AreaResizerImpl<iqo::ArchGeneric> impl;
        impl.init(sw, sh, dw, dh);
        return axis ? dump(impl.m_TablesY, impl.m_NumCoefsY, impl.m_NumTablesY, nTaps, nPhases, buf, cap)
                    : dump(impl.m_TablesX, impl.m_NumCoefsX, impl.m_NumTablesX, nTaps, nPhases, buf, cap);
    }
    iqo::LinearResizerImpl<iqo::ArchGeneric> impl;
    impl.init(sw, sh, dw, dh);
    return axis ? dump(impl.m_TablesY, 2, impl.m_NumTablesY, nTaps, nPhases, buf, cap)
                : dump(impl.m_TablesX, 2, impl.m_NumTablesX, nTaps, nPhases, buf, cap);
}
