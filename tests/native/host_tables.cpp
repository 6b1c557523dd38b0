// TEST INFRASTRUCTURE ONLY (tests/native/asan.mk, tests/test_host_sanitizers.py): drives every
// host-side table builder of the product (libiqo_amd/csrc/plan.cpp) under AddressSanitizer and
// UBSan, over shapes read from stdin, one per line:
//   method degree srcW srcH dstW dstH pxScale
// For each shape: build_plan, the tile / walker tables, every exact-ratio builder (up2, d32, d31,
// a32, u23, l23), ryx and ryg, band_src_rows over random band cuts (full frame, single rows, the
// last row, random [r0, r1)), and the scalar emulations of the kernels that index those tables
// (tests/native/ratio_emul.cpp, tile_emul.cpp) on a random frame -- an emulated kernel reads
// the tables the way the kernel does (row records past the last row included), so a short table
// is an ASan report here instead of a stray device read.  Prints one line per builder: the
// number of shapes it accepted.  Exit status != 0 on any sanitizer report (-fno-sanitize-recover).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "plan.hpp"

extern "C" int ratio_emul(int kind, int method, unsigned degree, int srcW, int srcH, int dstW, int dstH, int pxScale,
                          const uint8_t *src, uint8_t *dst);
extern "C" int tile_emul(int method, unsigned degree, int srcW, int srcH, int dstW, int dstH, int pxScale,
                         const uint8_t *src, uint8_t *dst, int *np_out);

using namespace iqo_amd;

int main()
{
    std::map<std::string, int> ok;
    std::mt19937 rng(12345);
    int m, deg, sw, sh, dw, dh, px, n = 0;
    while (std::scanf("%d %d %d %d %d %d %d", &m, &deg, &sw, &sh, &dw, &dh, &px) == 7) {
        ++n;
        Plan p;
        std::string err;
        if (!build_plan(static_cast<Method>(m), static_cast<unsigned>(deg), sw, sh, dw, dh, px, &p, &err))
            continue;
        ++ok["build_plan"];
        TileTables t;
        build_tile_tables(p, &t);
        WalkTables w;
        if (t.ok) {
            ++ok["build_tile_tables"];
            tile_src_rows(p, t, t.TH);
            tile_lds_bytes(p, t, t.TH);
            build_walk_tables(p, t, &w);
            ok["build_walk_tables"] += w.ok;
        }
        Up2Tables u;
        build_up2(p, w, &u);
        ok["build_up2"] += u.ok;
        D32Tables d32;
        build_d32(p, w, &d32);
        ok["build_d32"] += d32.ok;
        D31Tables d31;
        build_d31(p, &d31);
        ok["build_d31"] += d31.ok;
        RyxTables ryx, ryg;
        build_ryx(p, &ryx);
        ok["build_ryx"] += ryx.ok;
        build_ryg(p, &ryg);
        ok["build_ryg"] += ryg.ok;
        U23Tables u23;
        build_u23(p, &u23);
        ok["build_u23"] += u23.ok;
        L23Tables l23;
        build_l23(p, &l23);
        ok["build_l23"] += l23.ok;
        A32Tables a32;
        build_a32(p, &a32);
        ok["build_a32"] += a32.ok;
        // band windows: whole frame, first / last row, one-row bands and random cuts
        std::vector<std::pair<int, int>> cuts = {{0, dh}, {0, 1}, {dh - 1, dh}, {dh / 2, dh / 2 + 1}};
        for (int k = 0; k < 24; ++k) {
            const int a = static_cast<int>(rng() % static_cast<unsigned>(dh)), b = static_cast<int>(rng() % static_cast<unsigned>(dh));
            cuts.push_back({std::min(a, b), std::max(a, b) + 1});
        }
        for (const auto &c : cuts) {
            int s0 = -1, s1 = -1;
            band_src_rows(p, c.first, c.second, &s0, &s1);
            if (s0 < 0 || s1 > sh || s0 >= s1) {
                std::fprintf(stderr, "band_src_rows(%d, %d) -> [%d, %d) outside [0, %d)\n", c.first, c.second, s0, s1, sh);
                return 4;
            }
        }
        ok["band_src_rows"] += 1;
        // the kernels' table reads, emulated (sizes kept to a few megapixels)
        if (static_cast<int64_t>(sw) * sh <= 9000000 && static_cast<int64_t>(dw) * dh <= 9000000) {
            std::vector<uint8_t> src(static_cast<size_t>(sw) * sh), dst(static_cast<size_t>(dw) * dh);
            for (auto &v : src)
                v = static_cast<uint8_t>(rng());
            static const char *names[] = {"emul_lanczos_d32", "emul_lanczos_up2", "emul_area_d32", "emul_lanczos_u23",
                                          "emul_linear_u23", "emul_lanczos_d31", "emul_ryx", "emul_linear_d2",
                                          "emul_linear_up2", "emul_ryg"};
            for (int kind = 0; kind <= 9; ++kind) {
                const int rc = ratio_emul(kind, m, static_cast<unsigned>(deg), sw, sh, dw, dh, px, src.data(), dst.data());
                if (rc < 0) {
                    std::fprintf(stderr, "ratio_emul kind %d rc %d on %d %d %d %d %d %d %d\n", kind, rc, m, deg, sw, sh, dw,
                                 dh, px);
                    return 5;
                }
                ok[names[kind]] += rc == 0;
            }
            int np = 0;
            ok["emul_tile"] += tile_emul(m, static_cast<unsigned>(deg), sw, sh, dw, dh, px, src.data(), dst.data(), &np) == 0;
        }
    }
    std::printf("shapes %d\n", n);
    for (const auto &kv : ok)
        std::printf("%s %d\n", kv.first.c_str(), kv.second);
    return 0;
}
