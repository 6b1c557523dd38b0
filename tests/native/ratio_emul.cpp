// Test-only scalar emulation of the exact-ratio kernels of kernels.hip (lanczos_d32_kernel,
// lanczos_up2_kernel, area_d32_kernel, lanczos_u23_kernel, linear_u23_kernel, lanczos_d31_kernel) over the product's own tables (libiqo_amd/csrc/plan.cpp
// build_d32 / build_up2 / build_a32), so the coordinate checks, the zero rows / columns outside
// the image, the magic-number border divisions and the edge-lane rewrite are checked against the
// oracle on a machine without a GPU.  Emulates the kernels' arithmetic word for word: 16-bit
// wrapped vertical sums, v_dot2 pairs with int16 (Lanczos) or u16 (Area) halves, ydiv2, the
// multiply-high edge division, v_ashr_pk_u8_i32 saturation.  Never part of the product.
#include "plan.hpp"

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

using namespace iqo_amd;

namespace {

uint32_t umulhi(uint32_t a, uint32_t b) { return static_cast<uint32_t>((static_cast<uint64_t>(a) * b) >> 32); }

// kernels.hip ydiv2 on one int16 half
uint16_t ydiv1(uint16_t w, uint32_t m, int s)
{
    const int v = static_cast<int16_t>(w);
    const uint32_t q = umulhi(static_cast<uint32_t>(v < 0 ? -v : v) << s, m);
    return static_cast<uint16_t>(v < 0 ? 0u - q : q);
}

int sat_u8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

uint8_t edge_div(int s, uint32_t m, int t)
{
    const uint32_t q = umulhi(static_cast<uint32_t>(s < 0 ? 0 : s), m) >> t;
    return static_cast<uint8_t>(q > 255u ? 255u : q);
}

}  // namespace

extern "C" {

// kind: 0 = lanczos_d32, 1 = lanczos_up2, 2 = area_d32, 3 = lanczos_u23, 4 = linear_u23, 5 = lanczos_d31, 6 = ryx, 7 = linear_d2,
// 8 = linear_up2, 9 = ryg.  Returns 0 on success, 1 if the shape is
// not eligible for that kernel, -1 on bad arguments.
int ratio_emul(int kind, int method, unsigned degree, int srcW, int srcH, int dstW, int dstH, int pxScale,
               const uint8_t *src, uint8_t *dst)
{
    Plan p;
    std::string err;
    if (!build_plan(static_cast<Method>(method), degree, srcW, srcH, dstW, dstH, pxScale, &p, &err))
        return -1;
    TileTables t;
    WalkTables w;
    build_tile_tables(p, &t);
    if (t.ok)
        build_walk_tables(p, t, &w);
    auto px = [&](int r, int c) -> int {
        return (r < 0 || r >= srcH || c < 0 || c >= srcW) ? 0 : src[static_cast<size_t>(r) * srcW + c];
    };
    std::vector<uint16_t> work(static_cast<size_t>(srcW));
    if (kind == 0) {
        D32Tables d;
        build_d32(p, w, &d);
        if (!d.ok)
            return 1;
        // the kernel instantiation's tap structure (kernels.hip launch_d32): GA, NTY, PO1, NPX, BX0
        const int GA = d.variant ? -2 : -4, NTY = d.variant ? 5 : 8, PO1 = 2, NPX = d.variant ? 3 : 5;
        const int BX0 = d.variant ? -2 : -4;
        for (int y = 0; y < dstH; ++y) {
            const int m = y >> 1, ph = y & 1;
            for (int c = 0; c < srcW; ++c) {
                uint16_t acc = 0;
                for (int i = 0; i < NTY; ++i)
                    acc = static_cast<uint16_t>(acc + px(3 * m + GA + (ph ? PO1 : 0) + i, c) * static_cast<uint16_t>(d.cy[ph][i]));
                if (y < d.m0 || y >= d.m1) {
                    const int side = y < d.m0 ? 0 : 1, bi = side ? y - d.m1 : y;
                    acc = ydiv1(acc, d.yM[side][bi], d.yS[side][bi]);
                }
                work[static_cast<size_t>(c)] = acc;
            }
            auto W = [&](int c) -> int { return (c < 0 || c >= srcW) ? 0 : static_cast<int16_t>(work[static_cast<size_t>(c)]); };
            for (int x = 0; x < dstW; ++x) {
                const int q = x & 1, a = 3 * (x >> 1) + BX0 + q;
                int s = 1 << 19;
                for (int k = 0; k < NPX; ++k)
                    s += W(a + 2 * k) * static_cast<int16_t>(d.cx[q][k] & 0xffffu) +
                         W(a + 2 * k + 1) * static_cast<int16_t>(d.cx[q][k] >> 16);
                const int side = x < 8 ? 0 : x >= dstW - 8 ? 1 : -1;
                dst[static_cast<size_t>(y) * dstW + x] = static_cast<uint8_t>(
                    side < 0 ? sat_u8(s >> 20) : edge_div(s, d.xM[side][side ? x - (dstW - 8) : x], d.xT[side][side ? x - (dstW - 8) : x]));
            }
        }
        return 0;
    }
    if (kind == 1) {
        Up2Tables u;
        build_up2(p, w, &u);
        if (!u.ok)
            return 1;
        const int NT = u.NT, OFF = 1 - NT / 2, F = u.F, EC = 8 * F;
        for (int y = 0; y < dstH; ++y) {
            const int k = y / F, j = y % F;
            for (int c = 0; c < srcW; ++c) {
                uint16_t acc;
                if (j == 0) {
                    acc = static_cast<uint16_t>(px(k, c) * static_cast<uint16_t>(u.cy0));
                } else {
                    acc = 0;
                    for (int i = 0; i < NT; ++i)
                        acc = static_cast<uint16_t>(acc + px(k + OFF + i, c) * static_cast<uint16_t>(u.cy1[j - 1][i]));
                }
                if (y < u.m0 || y >= u.m1) {
                    const int side = y < u.m0 ? 0 : 1, bi = side ? y - u.m1 : y;
                    acc = ydiv1(acc, u.yM[side][bi], u.yS[side][bi]);
                }
                work[static_cast<size_t>(c)] = acc;
            }
            auto W = [&](int c) -> int { return (c < 0 || c >= srcW) ? 0 : static_cast<int16_t>(work[static_cast<size_t>(c)]); };
            for (int x = 0; x < dstW; ++x) {
                int s = 1 << 19;
                const int kx = x / F, jx = x % F;
                if (jx == 0) {
                    s += W(kx) * static_cast<int16_t>(u.cx0 & 0xffffu);
                } else {
                    const uint32_t *cx = u.cx1[jx - 1];
                    for (int q = 0; q < NT / 2; ++q)
                        s += W(kx + OFF + 2 * q) * static_cast<int16_t>(cx[q] & 0xffffu) +
                             W(kx + OFF + 2 * q + 1) * static_cast<int16_t>(cx[q] >> 16);
                }
                const int side = x < EC ? 0 : x >= dstW - EC ? 1 : -1;
                dst[static_cast<size_t>(y) * dstW + x] = static_cast<uint8_t>(
                    side < 0 ? sat_u8(s >> 20) : edge_div(s, u.xM[side][side ? x - (dstW - EC) : x], u.xT[side][side ? x - (dstW - EC) : x]));
            }
        }
        return 0;
    }
    if (kind == 3) {
        U23Tables u;
        build_u23(p, &u);
        if (!u.ok)
            return 1;
        for (int y = 0; y < dstH; ++y) {
            const int m = y / 3, ph = y % 3;
            for (int c = 0; c < srcW; ++c) {
                uint16_t acc = 0;
                if (ph == 0)
                    acc = static_cast<uint16_t>(px(2 * m, c) * static_cast<uint16_t>(u.cy0));
                else
                    for (int k = 0; k < 6; ++k)
                        acc = static_cast<uint16_t>(acc + px(2 * m - 2 + (ph - 1) + k, c) * static_cast<uint16_t>(u.cy[ph - 1][k]));
                if (y < u.m0 || y >= u.m1) {
                    const int side = y < u.m0 ? 0 : 1, bi = side ? y - u.m1 : y;
                    acc = ydiv1(acc, u.yM[side][bi], u.yS[side][bi]);
                }
                work[static_cast<size_t>(c)] = acc;
            }
            auto W = [&](int c) -> int { return (c < 0 || c >= srcW) ? 0 : static_cast<int16_t>(work[static_cast<size_t>(c)]); };
            for (int x = 0; x < dstW; ++x) {
                const int g = x / 3, q = x % 3;
                int s = 1 << 19;
                if (q == 0) {
                    s += W(2 * g) * static_cast<int16_t>(u.cx0 & 0xffffu);
                } else {
                    const int a = 2 * g - 2 + (q - 1);
                    for (int k = 0; k < 3; ++k)
                        s += W(a + 2 * k) * static_cast<int16_t>(u.cx[q - 1][k] & 0xffffu) +
                             W(a + 2 * k + 1) * static_cast<int16_t>(u.cx[q - 1][k] >> 16);
                }
                const int side = x < 12 ? 0 : x >= dstW - 12 ? 1 : -1;
                dst[static_cast<size_t>(y) * dstW + x] = static_cast<uint8_t>(
                    side < 0 ? sat_u8(s >> 20) : edge_div(s, u.xM[side][side ? x - (dstW - 12) : x], u.xT[side][side ? x - (dstW - 12) : x]));
            }
        }
        return 0;
    }
    if (kind == 4) {
        L23Tables l;
        build_l23(p, &l);
        if (!l.ok)
            return 1;
        auto cl = [&](int r, int c) {
            r = r < 0 ? 0 : (r >= srcH ? srcH - 1 : r);
            c = c < 0 ? 0 : (c >= srcW ? srcW - 1 : c);
            return static_cast<int>(src[static_cast<size_t>(r) * srcW + c]);
        };
        for (int y = 0; y < dstH; ++y) {
            const int m = y / 3, j = y % 3, r0 = 2 * m + j - 1;
            std::vector<uint16_t> wrow(static_cast<size_t>(srcW) + 2);
            auto Wc = [&](int c) { return static_cast<uint32_t>(static_cast<uint16_t>(
                                       cl(r0, c) * static_cast<uint16_t>(l.cy[j][0]) + cl(r0 + 1, c) * static_cast<uint16_t>(l.cy[j][1]))); };
            for (int x = 0; x < dstW; ++x) {
                const int g = x / 3, q = x % 3, a = 2 * g + q - 1;
                const uint32_t s = (1u << 22) + Wc(a) * (l.cx[q] & 0xffffu) + Wc(a + 1) * (l.cx[q] >> 16);
                dst[static_cast<size_t>(y) * dstW + x] = static_cast<uint8_t>(sat_u8(static_cast<int>(s) >> 23));
            }
        }
        return 0;
    }
    if (kind == 5) {
        D31Tables d;
        build_d31(p, &d);
        if (!d.ok)
            return 1;
        // kernels.hip D31Shape: window rows 3y + YA .., centre CEN, pair distances; columns from 3x + XS
        const int YA = d.variant ? -4 : -6, CEN = d.variant ? 5 : 7, NPY = d.variant ? 4 : 5;
        const int DIST[5] = {1, 2, 4, 5, 7};
        const int XS = d.variant ? -5 : -8, NPX = d.variant ? 6 : 9;
        for (int y = 0; y < dstH; ++y) {
            const int r0 = 3 * y + YA;
            for (int c = 0; c < srcW; ++c) {
                uint16_t acc = static_cast<uint16_t>(px(r0 + CEN, c) * static_cast<uint16_t>(d.cc));
                for (int k = 0; k < NPY; ++k)
                    acc = static_cast<uint16_t>(acc + (px(r0 + CEN - DIST[k], c) + px(r0 + CEN + DIST[k], c)) *
                                                          static_cast<uint16_t>(d.cp[k]));
                if (y < d.m0 || y >= d.m1) {
                    const int side = y < d.m0 ? 0 : 1, bi = side ? y - d.m1 : y;
                    acc = ydiv1(acc, d.yM[side][bi], d.yS[side][bi]);
                }
                work[static_cast<size_t>(c)] = acc;
            }
            auto W = [&](int c) -> int { return (c < 0 || c >= srcW) ? 0 : static_cast<int16_t>(work[static_cast<size_t>(c)]); };
            for (int x = 0; x < dstW; ++x) {
                const int st = 3 * x + XS;
                const bool odd = (st & 1) != 0;
                const int a = odd ? st + 1 : st;
                int s = 1 << 19;
                for (int q = 0; q < NPX; ++q) {
                    const uint32_t cq = odd ? d.cxo[q] : d.cxe[q];
                    s += W(a + 2 * q) * static_cast<int16_t>(cq & 0xffffu) + W(a + 2 * q + 1) * static_cast<int16_t>(cq >> 16);
                }
                const int side = x < 4 ? 0 : x >= dstW - 4 ? 1 : -1;
                dst[static_cast<size_t>(y) * dstW + x] = static_cast<uint8_t>(
                    side < 0 ? sat_u8(s >> 20) : edge_div(s, d.xM[side][side ? x - (dstW - 4) : x], d.xT[side][side ? x - (dstW - 4) : x]));
            }
        }
        return 0;
    }
    if (kind == 6) {
        RyxTables r;
        build_ryx(p, &r);
        if (!r.ok)
            return 1;
        const bool lz = method == 0;
        const int P = r.P, Q = r.Q, T = r.taps, NP = r.NP;
        std::vector<uint16_t> wrow(static_cast<size_t>(srcW + 2 * kRyxPad), 0);
        for (int y = 0; y < dstH; ++y) {
            const int m = y / Q, j = y % Q, r0 = P * m + (P * j) / Q + r.off;
            for (int c = 0; c < srcW; ++c) {
                uint16_t acc = 0;
                for (int k = 0; k < T; ++k)
                    acc = static_cast<uint16_t>(acc + px(r0 + k, c) * static_cast<uint16_t>(r.rowCoef[static_cast<size_t>(j * T + k)]));
                if (lz && (y < r.m0 || y >= r.m1)) {
                    const int side = y < r.m0 ? 0 : 1, bi = side ? y - r.m1 : y;
                    acc = ydiv1(acc, r.yM[side][bi], r.yS[side][bi]);
                }
                wrow[static_cast<size_t>(kRyxPad + c)] = acc;
            }
            for (int x = 0; x < dstW; ++x) {
                const int32_t *cx = &r.cols[static_cast<size_t>(x) * 4];
                const int a = cx[0] / 2;  // u16 index of the even start in the padded row
                int64_t s = lz ? (1 << 19) : (1 << 22);
                for (int q = 0; q < NP; ++q) {
                    const uint32_t c = r.colCoef[static_cast<size_t>(x) * NP + q];
                    const uint16_t w0 = wrow[static_cast<size_t>(a + 2 * q)], w1 = wrow[static_cast<size_t>(a + 2 * q + 1)];
                    if (lz)
                        s += static_cast<int16_t>(w0) * static_cast<int16_t>(c & 0xffffu) + static_cast<int16_t>(w1) * static_cast<int16_t>(c >> 16);
                    else
                        s += static_cast<int64_t>(w0) * (c & 0xffffu) + static_cast<int64_t>(w1) * (c >> 16);
                }
                uint8_t o;
                if (lz) {
                    o = edge_div(static_cast<int>(s), static_cast<uint32_t>(cx[1]), cx[2]);
                } else {
                    const uint16_t u = static_cast<uint16_t>(static_cast<int16_t>(static_cast<int>(static_cast<uint32_t>(s)) >> 23));
                    o = static_cast<uint8_t>(u > 255 ? 255 : u);
                }
                dst[static_cast<size_t>(y) * dstW + x] = o;
            }
        }
        return 0;
    }
    if (kind == 9) {
        // ryg_kernel (general rows, plan.cpp build_ryg): output row y takes the TK taps from rowRec
        // {first window row s(y), coefficient offset c(y)}; rows outside the image read as zero; masked
        // Lanczos border rows divided by ydiv2; columns as ryx.  The kernel reads the records of rows
        // up to y + 2 and, through them, s(y + 2 + kPD - 1) unclamped past the last row (its FIFO
        // look-ahead, kernels.hip ryg_kernel / abi.hip): read them here too, so a sanitizer build
        // catches a record table shorter than that (kRygRecPad)
        RyxTables r;
        build_ryg(p, &r);
        if (!r.ok)
            return 1;
        constexpr int kPD = 4;  // kernels.hpp kRygPD (IQO_RYG_PD)
        const bool lz = method == 0;
        const int TK = r.taps, NP = r.NP;
        const size_t nRec = r.rowRec.size() / 2;
        int64_t touch = 0;
        std::vector<uint16_t> wrow(static_cast<size_t>(srcW + 2 * kRyxPad), 0);
        for (int y = 0; y < dstH; ++y) {
            const int s0 = r.rowRec.at(static_cast<size_t>(2 * y)), co = r.rowRec.at(static_cast<size_t>(2 * y + 1));
            touch += r.rowRec.at(static_cast<size_t>(2 * (y + 2))) + r.rowRec.at(static_cast<size_t>(2 * (y + 2 + kPD - 1)));
            if (static_cast<size_t>(y + 2 + kPD - 1) >= nRec)
                return -2;
            for (int c = 0; c < srcW; ++c) {
                uint16_t acc = 0;
                for (int k = 0; k < TK; ++k)
                    acc = static_cast<uint16_t>(acc + px(s0 + k, c) * static_cast<uint16_t>(r.rowCoef.at(static_cast<size_t>(co + k))));
                if (lz && (y < r.m0 || y >= r.m1)) {
                    const int side = y < r.m0 ? 0 : 1, bi = side ? y - r.m1 : y;
                    acc = ydiv1(acc, r.yM[side][bi < 0 ? 0 : bi > 15 ? 15 : bi], r.yS[side][bi < 0 ? 0 : bi > 15 ? 15 : bi]);
                }
                wrow[static_cast<size_t>(kRyxPad + c)] = acc;
            }
            for (int x = 0; x < dstW; ++x) {
                const int32_t *cx = &r.cols.at(static_cast<size_t>(x) * 4);
                const int a = cx[0] / 2;
                int64_t sum = lz ? (1 << 19) : (1 << 22);
                for (int q = 0; q < NP; ++q) {
                    const uint32_t c = r.colCoef.at(static_cast<size_t>(x) * NP + q);
                    const uint16_t w0 = wrow.at(static_cast<size_t>(a + 2 * q)), w1 = wrow.at(static_cast<size_t>(a + 2 * q + 1));
                    if (lz)
                        sum += static_cast<int16_t>(w0) * static_cast<int16_t>(c & 0xffffu) + static_cast<int16_t>(w1) * static_cast<int16_t>(c >> 16);
                    else
                        sum += static_cast<int64_t>(w0) * (c & 0xffffu) + static_cast<int64_t>(w1) * (c >> 16);
                }
                uint8_t o;
                if (lz) {
                    o = edge_div(static_cast<int>(sum), static_cast<uint32_t>(cx[1]), cx[2]);
                } else {
                    const uint16_t u = static_cast<uint16_t>(static_cast<int16_t>(static_cast<int>(static_cast<uint32_t>(sum)) >> 23));
                    o = static_cast<uint8_t>(u > 255 ? 255 : u);
                }
                dst[static_cast<size_t>(y) * dstW + x] = o;
            }
        }
        return touch == -1 ? -3 : 0;  // (keeps the look-ahead reads)
    }
    if (kind == 10 || kind == 11) {
        // ryu_kernel / ryp_kernel (general rows walked by window position, plan.cpp build_ryu_positions):
        // for each band [y0, y1) the kernel takes positions pA = s(y0) .. s(y1 - 1); position p's
        // record gives the output rows whose window starts at pA + p, clipped to the band, and their
        // tap offsets; it reads the records of positions p + 1 and p + 2 unclamped.  Emulated over
        // several band heights: every band plan must give the same image, every row written once.
        RyxTables r;
        build_ryg(p, &r);
        if (!r.ok || !build_ryu_positions(dstH, &r))
            return 1;
        // kind 11: the run mode (4 adjacent columns from one run of runPairs dwords, build_ryu_runs)
        const bool run = kind == 11;
        if (run && !build_ryu_runs(dstW, &r))
            return 1;
        const bool lz = method == 0;
        const int TK = r.taps, NP = r.NP;
        const size_t nPosRec = r.posRec.size() / kRyuRec;
        std::vector<uint16_t> wrow(static_cast<size_t>(srcW + 2 * kRyxPad), 0);
        std::vector<uint8_t> first;
        for (const int rpb : {dstH, 7, 13, 1, 64}) {
            std::vector<int> written(static_cast<size_t>(dstH), 0);
            for (int y0 = 0; y0 < dstH; y0 += rpb) {
                const int y1 = std::min(dstH, y0 + rpb);
                const int pA = r.rowRec.at(static_cast<size_t>(2 * y0));
                const int nPos = r.rowRec.at(static_cast<size_t>(2 * (y1 - 1))) - pA + 1;
                for (int q = 0; q < nPos; ++q) {
                    const size_t ri = static_cast<size_t>(pA - r.posBase + q);
                    if (ri + 2 >= nPosRec)
                        return -2;  // the kernel's look-ahead would read past the table
                    const int32_t *rc = &r.posRec.at(kRyuRec * ri);
                    const int ya = std::max(rc[0], y0), cnt = std::min(rc[0] + rc[1], y1) - ya;
                    if (cnt <= 0 && (rc[1] == 0 || rc[0] + rc[1] <= y0))
                        continue;  // a position without rows (downscales) or whose rows precede the band
                    if (cnt < 1 || cnt > r.posRows || (q > 0 && ya != rc[0]))
                        return -4;
                    for (int k = 0; k < cnt; ++k) {
                        const int y = ya + k, co = rc[2 + (ya - rc[0]) + k];
                        ++written.at(static_cast<size_t>(y));
                        for (int c = 0; c < srcW; ++c) {
                            uint16_t acc = 0;
                            for (int t2 = 0; t2 < TK; ++t2)
                                acc = static_cast<uint16_t>(acc + px(pA + q + t2, c) *
                                                                      static_cast<uint16_t>(r.rowCoef.at(static_cast<size_t>(co + t2))));
                            if (lz && (y < r.m0 || y >= r.m1)) {
                                const int side = y < r.m0 ? 0 : 1, bi = side ? y - r.m1 : y;
                                acc = ydiv1(acc, r.yM[side][bi < 0 ? 0 : bi > 15 ? 15 : bi], r.yS[side][bi < 0 ? 0 : bi > 15 ? 15 : bi]);
                            }
                            wrow[static_cast<size_t>(kRyxPad + c)] = acc;
                        }
                        for (int x = 0; x < dstW; ++x) {
                            const int32_t *cx = &r.cols.at(static_cast<size_t>(x) * 4);
                            int a = cx[0] / 2;
                            if (run)  // the group's lowest even start
                                for (int k = x & ~3; k < std::min(dstW, (x & ~3) + 4); ++k)
                                    a = std::min(a, r.cols.at(static_cast<size_t>(k) * 4) / 2);
                            const int nq = run ? r.runPairs : NP;
                            int64_t sum = lz ? (1 << 19) : (1 << 22);
                            for (int q2 = 0; q2 < nq; ++q2) {
                                const uint32_t c = run ? r.colRun.at(static_cast<size_t>(x) * nq + q2)
                                                       : r.colCoef.at(static_cast<size_t>(x) * NP + q2);
                                const uint16_t w0 = wrow.at(static_cast<size_t>(a + 2 * q2)), w1 = wrow.at(static_cast<size_t>(a + 2 * q2 + 1));
                                if (lz)
                                    sum += static_cast<int16_t>(w0) * static_cast<int16_t>(c & 0xffffu) +
                                           static_cast<int16_t>(w1) * static_cast<int16_t>(c >> 16);
                                else
                                    sum += static_cast<int64_t>(w0) * (c & 0xffffu) + static_cast<int64_t>(w1) * (c >> 16);
                            }
                            uint8_t o;
                            if (lz) {
                                o = edge_div(static_cast<int>(sum), static_cast<uint32_t>(cx[1]), cx[2]);
                            } else {  // (Area / Linear: ryg_kernel's u16 sums, (s + 2^22) >> 23)
                                const uint16_t u = static_cast<uint16_t>(static_cast<int16_t>(static_cast<int>(static_cast<uint32_t>(sum)) >> 23));
                                o = static_cast<uint8_t>(u > 255 ? 255 : u);
                            }
                            dst[static_cast<size_t>(y) * dstW + x] = o;
                        }
                    }
                }
            }
            for (int y = 0; y < dstH; ++y)
                if (written[static_cast<size_t>(y)] != 1)
                    return -5;
            if (first.empty())
                first.assign(dst, dst + static_cast<size_t>(dstW) * dstH);
            else if (!std::equal(first.begin(), first.end(), dst))
                return -6;
        }
        return 0;
    }
    if (kind == 7) {
        // linear_d2_body (Linear 2:1 through IQO_KERNEL_AREA_INT): main rows / columns blend
        // samples 2i + 1, 2i + 2; edge rows take one source row at 256, edge columns (w + 128) >> 8
        if (p.kernel != 2 || !p.far.lin)
            return 1;
        for (int y = 0; y < dstH; ++y) {
            int r0 = 2 * y + 1, r1 = 2 * y + 2;
            uint16_t c0 = p.far.cy[0], c1 = p.far.cy[1];
            if (y == 0 || y == dstH - 1) {
                r0 = r1 = y == 0 ? 0 : srcH - 1;
                c0 = 256;
                c1 = 0;
            }
            for (int c = 0; c < srcW; ++c)
                work[static_cast<size_t>(c)] = static_cast<uint16_t>(px(r0, c) * c0 + px(r1, c) * c1);
            for (int x = 0; x < dstW; ++x) {
                int v;
                if (x == 0 || x == dstW - 1) {
                    const uint16_t wv = work[static_cast<size_t>(x == 0 ? 0 : srcW - 1)];
                    v = static_cast<int16_t>((wv + 128) >> 8);
                } else {
                    const uint32_t sum = (1u << 22) + work[static_cast<size_t>(2 * x + 1)] * static_cast<uint32_t>(p.far.cx[0]) +
                                         work[static_cast<size_t>(2 * x + 2)] * static_cast<uint32_t>(p.far.cx[1]);
                    v = static_cast<int16_t>(static_cast<int>(sum) >> 23);
                }
                const uint16_t u = static_cast<uint16_t>(v);
                dst[static_cast<size_t>(y) * dstW + x] = static_cast<uint8_t>(u > 255 ? 255 : u);
            }
        }
        return 0;
    }
    if (kind == 8) {
        // linear_up2_kernel_body (Linear exactly 2x / 3x): main row F k + i (i = 1 .. F) blends
        // source rows k, k + 1 with phase i % F; main column x blends work columns m, m + 1,
        // m = (x - 1) / F; edge rows take one source row at 256, edge columns (w * 2^15 + 2^22) >> 23
        if (p.kernel != 3)
            return 1;
        const int F = p.fln.F;
        for (int y = 0; y < dstH; ++y) {
            int r0, c0, c1;
            if (y == 0 || y == dstH - 1) {
                r0 = y == 0 ? 0 : srcH - 1;
                c0 = 256;
                c1 = 0;
            } else {
                r0 = (y - 1) / F;
                c0 = p.fln.cy[y % F][0];
                c1 = p.fln.cy[y % F][1];
            }
            for (int c = 0; c < srcW; ++c)
                work[static_cast<size_t>(c)] = static_cast<uint16_t>(px(r0, c) * c0 + (c1 ? px(r0 + 1, c) * c1 : 0));
            for (int x = 0; x < dstW; ++x) {
                uint32_t s;
                if (x == 0 || x == dstW - 1)
                    s = work[static_cast<size_t>(x == 0 ? 0 : srcW - 1)] * 32768u + (1u << 22);
                else
                    s = work[static_cast<size_t>((x - 1) / F)] * static_cast<uint32_t>(p.fln.cx[x % F][0]) +
                        (p.fln.cx[x % F][1] ? work[static_cast<size_t>((x - 1) / F + 1)] * static_cast<uint32_t>(p.fln.cx[x % F][1]) : 0u) +
                        (1u << 22);
                const int v = static_cast<int>(s) >> 23;
                dst[static_cast<size_t>(y) * dstW + x] = static_cast<uint8_t>(v > 255 ? 255 : v);
            }
        }
        return 0;
    }
    if (kind == 2) {
        A32Tables a;
        build_a32(p, &a);
        if (!a.ok)
            return 1;
        for (int y = 0; y < dstH; ++y) {
            const int m = y >> 1, ph = y & 1;
            for (int c = 0; c < srcW; ++c)
                work[static_cast<size_t>(c)] = static_cast<uint16_t>(px(3 * m + ph, c) * static_cast<uint16_t>(a.cy[ph][0]) +
                                                                     px(3 * m + ph + 1, c) * static_cast<uint16_t>(a.cy[ph][1]));
            for (int x = 0; x < dstW; ++x) {
                const int q = x & 1, s0 = 3 * (x >> 1) + q;
                const uint32_t s = (1u << 22) + work[static_cast<size_t>(s0)] * (a.cx[q] & 0xffffu) +
                                   work[static_cast<size_t>(s0 + 1)] * (a.cx[q] >> 16);
                dst[static_cast<size_t>(y) * dstW + x] = static_cast<uint8_t>(sat_u8(static_cast<int>(s) >> 23));
            }
        }
        return 0;
    }
    return -1;
}

}  // extern "C"
