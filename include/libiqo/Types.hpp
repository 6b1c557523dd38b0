#pragma once

// libiqo_amd public types.  Same architecture tags as libiqo's include/libiqo/Types.hpp:49-74
// (so code that names iqo::ArchGeneric etc. keeps compiling), plus the HIP backend tag.  The
// CPU SIMD feature macros of the reference are not needed: this build has a single backend.

namespace iqo {

    template<int ARCH> struct Arch {};

    enum EnumArch {
        kArchGeneric,
        kArchSSE4_1,
        kArchAVX2FMA,
        kArchAVX512,
        kArchNEON,
        kArchHIP        //!< MI355X (gfx950) backend of this library
    };

    typedef Arch<kArchGeneric> ArchGeneric;
    typedef Arch<kArchSSE4_1>  ArchSSE4_1;
    typedef Arch<kArchAVX2FMA> ArchAVX2FMA;
    typedef Arch<kArchAVX512>  ArchAVX512;
    typedef Arch<kArchNEON>    ArchNEON;
    typedef Arch<kArchHIP>     ArchHIP;

}
