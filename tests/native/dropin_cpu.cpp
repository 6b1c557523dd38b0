// Drives the drop-in classes (include/libiqo/*Resizer.hpp, the reference's public API) over a
// manifest of cases read from stdin, one per line:
//   method degree srcW srcH dstW dstH pxScale input.raw output.raw
// (method 0 Lanczos, 1 Area, 2 Linear; tight strides).  Prints the backend counts at the end.
// tests/test_dropin_cpu.py runs it where no GPU is visible (the CPU backend) against the golden
// vectors; it uses nothing but the public headers and iqo_dropin_backend_counts.
#include <cstdio>
#include <vector>

#include "iqo_hip.h"
#include "libiqo/iqo.hpp"

int main()
{
    int m, deg;
    size_t sw, sh, dw, dh, px;
    char in[4096], out[4096];
    int n = 0;
    while (std::scanf("%d %d %zu %zu %zu %zu %zu %4095s %4095s", &m, &deg, &sw, &sh, &dw, &dh, &px, in, out) == 9) {
        std::vector<unsigned char> src(sw * sh), dst(dw * dh);
        FILE *f = std::fopen(in, "rb");
        if (!f || std::fread(src.data(), 1, src.size(), f) != src.size())
            return 2;
        std::fclose(f);
        if (m == 0) {
            iqo::LanczosResizer r(static_cast<unsigned>(deg), sw, sh, dw, dh, px);
            r.resize(sw, src.data(), dw, dst.data());
        } else if (m == 1) {
            iqo::AreaResizer r(sw, sh, dw, dh);
            r.resize(sw, src.data(), dw, dst.data());
        } else {
            iqo::LinearResizer r(sw, sh, dw, dh);
            r.resize(sw, src.data(), dw, dst.data());
        }
        f = std::fopen(out, "wb");
        if (!f || std::fwrite(dst.data(), 1, dst.size(), f) != dst.size())
            return 3;
        std::fclose(f);
        ++n;
    }
    int hip = -1, cpu = -1;
    iqo_dropin_backend_counts(&hip, &cpu);
    std::printf("cases %d hip %d cpu %d\n", n, hip, cpu);
    return 0;
}
