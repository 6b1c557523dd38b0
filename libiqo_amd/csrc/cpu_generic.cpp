// cpu_generic.cpp -- CPU backend of the drop-in classes (include/libiqo/*Resizer.hpp).
//
// The reference lands on its portable Generic implementation whenever no SIMD implementation is
// available (src/IQOLanczosResizer.cpp:17-33, LanczosResizerImpl_new<ArchGeneric>()); the drop-in
// classes here do the same when no gfx950 device is present (resizers.cpp).  This file is the
// product's own CPU path, not the oracle: it runs the host plan plan.cpp already builds for the
// GPU (quantised tables + one {source origin, table offset, formula, border divisor} record per
// output row and column, which restate the reference's row / column drivers), with the per-pixel
// formulas of the reference's Generic passes:
//   Lanczos  resizeYmain / resizeYborder  src/IQOLanczosResizerImpl_Generic.cpp:464-516
//            resizeXmain / resizeXborder  :539-612, identity shortcuts :378-388, :520-527
//   Area     resizeYmain :303-320, resizeXmain :340-368, shortcuts :259-269, :324-331
//   Linear   resizeYborder / resizeYmain :290-325, resizeXborder / resizeXmain :355-407
// Output rows are split over std::threads (the reference's SIMD variants split rows with OpenMP,
// e.g. src/IQOLanczosResizerImpl_AVX512.cpp:269-308); each thread owns its work row.
#include "cpu_generic.hpp"

#include <algorithm>
#include <thread>
#include <vector>

namespace iqo_amd {
namespace {

inline int clamp255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// uint8(clamp<uint16_t>(0, 255, int16(v))): the Area / Linear output conversion (:364-367, :404-406)
inline int u16clamp(int v)
{
    const uint16_t u = static_cast<uint16_t>(static_cast<int16_t>(v));
    return u > 255 ? 255 : u;
}

// C truncating division; a zero divisor (the reference traps) gives 0
inline int cdiv(int n, int d) { return d == 0 ? 0 : n / d; }

struct Rows {
    const Plan &p;
    size_t srcSt, dstSt;
    const uint8_t *src;
    uint8_t *dst;

    int px(int row, int col) const { return src[static_cast<size_t>(row) * srcSt + static_cast<size_t>(col)]; }

    // the reference's work row for output row y, every source column
    void vertical(int y, std::vector<int> &w) const
    {
        const CoordInfo &c = p.y.coord[static_cast<size_t>(y)];
        const int32_t *tab = p.y.table.data() + c.tabOff;
        const int n = p.y.taps, W = p.srcW, H = p.srcH;
        if (p.method == kLanczos) {
            if (c.kind == kIdentity) {
                for (int x = 0; x < W; ++x)
                    w[x] = static_cast<int16_t>(static_cast<uint16_t>(px(c.srcO, x) * 64));
            } else if (c.kind == kMain) {
                for (int x = 0; x < W; ++x) {
                    int16_t acc = 0;  // int16 wrap (:509-515)
                    for (int i = 0; i < n; ++i)
                        acc = static_cast<int16_t>(acc + px(c.srcO + i, x) * tab[i]);
                    w[x] = acc;
                }
            } else {
                const int i0 = std::max(0, -c.srcO), i1 = std::min(n, H - c.srcO);
                for (int x = 0; x < W; ++x) {
                    int16_t nume = 0;  // masked sum, renormalised by truncating division (:477-489)
                    for (int i = i0; i < i1; ++i)
                        nume = static_cast<int16_t>(nume + px(c.srcO + i, x) * tab[i]);
                    w[x] = static_cast<int16_t>(cdiv(static_cast<int>(nume) * 64, c.aux));
                }
            }
            return;
        }
        if (c.kind == kIdentity) {
            for (int x = 0; x < W; ++x)
                w[x] = static_cast<uint16_t>(px(c.srcO, x) * 256);
            return;
        }
        if (p.method == kArea) {
            for (int x = 0; x < W; ++x) {
                uint16_t acc = 0;  // u16 wrap; the weight-0 tap past the last row is clamped (:58-62)
                for (int i = 0; i < n; ++i)
                    acc = static_cast<uint16_t>(acc + px(std::min(c.srcO + i, H - 1), x) * tab[i]);
                w[x] = acc;
            }
            return;
        }
        if (c.kind == kBorderLo || c.kind == kBorderHi) {  // Linear: replicated first / last row
            const int r = c.kind == kBorderLo ? 0 : H - 1;
            for (int x = 0; x < W; ++x)
                w[x] = static_cast<uint16_t>(px(r, x) * 256);
            return;
        }
        const int r0 = std::max(0, std::min(c.srcO, H - 1)), r1 = std::max(0, std::min(c.srcO + 1, H - 1));
        for (int x = 0; x < W; ++x)
            w[x] = static_cast<uint16_t>(static_cast<uint16_t>(px(r0, x) * tab[0]) + px(r1, x) * tab[1]);
    }

    int horizontal(const std::vector<int> &w, int x) const
    {
        const CoordInfo &c = p.x.coord[static_cast<size_t>(x)];
        const int32_t *tab = p.x.table.data() + c.tabOff;
        const int n = p.x.taps, W = p.srcW;
        auto at = [&](int col) { return w[static_cast<size_t>(std::max(0, std::min(col, W - 1)))]; };
        if (p.method == kLanczos) {
            if (c.kind == kIdentity)
                return clamp255(static_cast<int16_t>((at(c.srcO) + 32) >> 6));
            if (c.kind == kMain) {
                int sum = 0;
                for (int i = 0; i < n; ++i)
                    sum += w[static_cast<size_t>(c.srcO + i)] * tab[i];
                return clamp255(static_cast<int16_t>((sum + (1 << 19)) >> 20));
            }
            int nume = 0;
            for (int i = 0; i < n; ++i) {
                const int col = c.srcO + i;
                if (col >= 0 && col < W)
                    nume += w[static_cast<size_t>(col)] * tab[i];
            }
            return clamp255(static_cast<int16_t>(cdiv(nume + (1 << 19), c.aux * 64)));
        }
        if (c.kind == kIdentity)
            return clamp255(static_cast<int16_t>((at(c.srcO) + 128) >> 8));
        if (p.method == kArea) {
            int sum = 0;
            for (int i = 0; i < n; ++i)
                sum += at(c.srcO + i) * tab[i];
            return u16clamp((sum + (1 << 22)) >> 23);
        }
        if (c.kind == kBorderLo)
            return u16clamp((w[0] + 128) >> 8);
        if (c.kind == kBorderHi)
            return u16clamp((w[static_cast<size_t>(W - 1)] + 128) >> 8);
        const int sum = at(c.srcO) * tab[0] + at(c.srcO + 1) * tab[1];
        return u16clamp((sum + (1 << 22)) >> 23);
    }

    void run(int y0, int y1) const
    {
        std::vector<int> w(static_cast<size_t>(p.srcW));
        for (int y = y0; y < y1; ++y) {
            vertical(y, w);
            uint8_t *d = dst + static_cast<size_t>(y) * dstSt;
            for (int x = 0; x < p.dstW; ++x)
                d[x] = static_cast<uint8_t>(horizontal(w, x));
        }
    }
};

} // namespace

void cpu_resize(const Plan &p, size_t srcSt, const uint8_t *src, size_t dstSt, uint8_t *dst, int threads)
{
    const Rows r{p, srcSt, dstSt, src, dst};
    if (threads <= 0) {
        const unsigned hc = std::thread::hardware_concurrency();
        threads = hc ? static_cast<int>(hc) : 1;
    }
    // at least 16 output rows and ~1 M source pixel-taps per thread, or threading costs more than it saves
    const int64_t work = static_cast<int64_t>(p.srcW) * p.dstH * std::max(1, p.y.taps);
    threads = static_cast<int>(std::min<int64_t>({static_cast<int64_t>(threads), p.dstH / 16 + 1, work / (1 << 20) + 1}));
    if (threads <= 1) {
        r.run(0, p.dstH);
        return;
    }
    std::vector<std::thread> pool;
    pool.reserve(static_cast<size_t>(threads));
    for (int t = 0; t < threads; ++t) {
        const int a = static_cast<int>(static_cast<int64_t>(p.dstH) * t / threads);
        const int b = static_cast<int>(static_cast<int64_t>(p.dstH) * (t + 1) / threads);
        pool.emplace_back([&r, a, b] { r.run(a, b); });
    }
    for (auto &th : pool)
        th.join();
}

} // namespace iqo_amd
