// Test-only scalar emulation of kernels.hip tile_kernel over the product's own tile tables
// (libiqo_amd/csrc/plan.cpp build_tile_tables), so the table folding (identity rows/columns,
// Linear replicated borders, masked Lanczos borders, even-aligned column windows, edge-column
// replication) is checked against the oracle / golden vectors on a machine without a GPU.
// Emulates the kernel's arithmetic word for word: 16-bit wrapped vertical sums, v_dot2 pairs,
// the same exact_div.  Never part of the product.
#include "plan.hpp"

#include <cstdint>
#include <cstring>
#include <string>

using namespace iqo_amd;

namespace {

int exact_div(int n, int d)
{
    if (d == 0)
        return 0;
    return static_cast<int>(static_cast<int64_t>(n) / d);  // C truncation, as the kernel's result
}

int clamp255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

}  // namespace

extern "C" {

// Returns 0 on success, 1 if the shape has no tile tables (general_kernel), -1 on bad arguments.
int tile_emul(int method, unsigned degree, int srcW, int srcH, int dstW, int dstH, int pxScale,
              const uint8_t *src, uint8_t *dst, int *np_out)
{
    Plan p;
    std::string err;
    if (!build_plan(static_cast<Method>(method), degree, srcW, srcH, dstW, dstH, pxScale, &p, &err))
        return -1;
    TileTables t;
    build_tile_tables(p, &t);
    if (!t.ok)
        return 1;
    if (np_out)
        *np_out = t.NP;
    const bool lz = method == kLanczos;
    const int nT = (dstW + t.CT - 1) / t.CT;
    std::vector<uint16_t> work(static_cast<size_t>(t.pitchDw) * 2);
    for (int y = 0; y < dstH; ++y) {
        const TileRec &r = t.rows[static_cast<size_t>(y)];
        for (int tx = 0; tx < nT; ++tx) {
            const TileSpan &sp = t.spans[static_cast<size_t>(tx)];
            // vertical: work columns [lo8, lo8 + 8 * groups), source columns clamped
            for (int c = 0; c < 8 * sp.groups; ++c) {
                const int col = std::min(std::max(sp.lo8 + c, 0), srcW - 1);
                uint16_t acc = 0;
                for (int i = 0; i < t.nYp; ++i) {
                    const int row = std::min(std::max(r.start + i, r.lo), r.hi);
                    const uint32_t cc = t.rowCoef[static_cast<size_t>(y) * t.nYp + i] & 0xffffu;
                    acc = static_cast<uint16_t>(acc + src[static_cast<size_t>(row) * srcW + col] * cc);
                }
                if (lz && r.deno != 0)
                    acc = static_cast<uint16_t>(exact_div(static_cast<int16_t>(acc) * 64, r.deno));
                work[static_cast<size_t>(c)] = acc;
            }
            // horizontal
            for (int x = tx * t.CT; x < std::min(dstW, (tx + 1) * t.CT); ++x) {
                const TileCol &cl = t.cols[static_cast<size_t>(x)];
                const int base = cl.a - sp.lo8;
                int s = lz ? (1 << 19) : (1 << 22);
                for (int pp = 0; pp < t.NP; ++pp) {
                    const uint32_t cf = t.colCoef[static_cast<size_t>(x) * t.NP + pp];
                    const uint16_t w0 = work[static_cast<size_t>(base + 2 * pp)], w1 = work[static_cast<size_t>(base + 2 * pp + 1)];
                    if (lz)
                        s += static_cast<int16_t>(w0) * static_cast<int16_t>(cf & 0xffffu) +
                             static_cast<int16_t>(w1) * static_cast<int16_t>(cf >> 16);
                    else
                        s = static_cast<int>(static_cast<uint32_t>(s) + static_cast<uint32_t>(w0) * (cf & 0xffffu) +
                                             static_cast<uint32_t>(w1) * (cf >> 16));
                }
                int v;
                if (lz) {
                    v = cl.D != 0 ? exact_div(s, cl.D) : (s >> 20);
                    v = clamp255(static_cast<int16_t>(v));
                } else {
                    v = static_cast<int>(std::min((static_cast<uint32_t>(s) >> 23) & 0xffffu, 255u));
                }
                dst[static_cast<size_t>(y) * dstW + x] = static_cast<uint8_t>(v);
            }
        }
    }
    return 0;
}

}  // extern "C"
