// kernels.hpp -- launch interface of the gfx950 resize kernels (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace iqo_amd {

// A device-side view of one batched call: frame f reads src + f*srcFrameSt, whose row 0 is
// GLOBAL source row srcRow0, and writes dst + f*dstFrameSt, whose row 0 is global row dstRow0.
struct Io {
    const uint8_t *src;
    int64_t srcSt, srcFrameSt;
    int srcRow0;
    int srcRowEnd;  // one past the last global source row the call may read (end of the window)
    uint8_t *dst;
    int64_t dstSt, dstFrameSt;
    int dstRow0;
    int frames;
};

// --- general kernel: one workgroup per output row; LDS work row built chunk by chunk.
struct GeneralDev {
    int method, srcW, srcH, dstW, nX, nY;
    const int4 *xInfo, *yInfo;   // {srcO, tabOff, kind, aux} per dst column / row
    const int *tabX, *tabY;      // quantised tables (int16 / u16 values widened)
    const int4 *chunks;          // {xs, xe, lo, hi}
    int nChunks;
    int ldsInts;                 // work-row capacity (ints) of the largest chunk
};
hipError_t launch_general(const GeneralDev &g, const Io &io, int rowBegin, int rowEnd, hipStream_t s);
// --- separable tile kernel (general ratios): tables from plan.cpp build_tile_tables.
struct TileDev {
    bool lanczos;                // int16 work + signed dots (else u16 work, Area / Linear)
    int srcW, srcH, dstW;
    int NP, nYp, CT, TH, pitchDw, log2nQ;
    int srcRows, spitch;         // staged source tile: rows (max over any TH output rows), pitch
    const int4 *rows;            // TileRec {start, lo, hi, deno} per output row
    const uint2 *rowTap;         // dstH x nYp {(c, c) splat, clamped source row}
    const int2 *cols;            // TileCol {a, D} per output column
    const uint32_t *colCoef;     // [NP][4][nQp] pairs (pair, column in quad, quad)
    const int *colA;             // [4][nQp] even window starts
    int nQp;                     // quads of the padded tile width
    const int4 *spans;           // {lo8, groups, any border column, 0} per column tile
};
hipError_t launch_tile(const TileDev &t, const Io &io, int rowBegin, int rowEnd, hipStream_t s);

// --- general-ratio wave walker: every wave walks a 256-column strip of one band of rows through
// a private LDS ring of source rows widened to u16 (plan.hpp WalkTables; 4-byte aligned sources).
struct WalkDev {
    TileDev t;                   // column tables (cols, colCoef, colA, nQp), lanczos, srcW / dstW, NP
    int nS;                      // 256-output strips per row
    const int4 *spans;           // {lo8, units, interior, 0} per strip; a unit = 4 work columns
    int NV;                      // units per lane (1, 2)
    int R, pitch;                // ring rows, ring row pitch (bytes)
    int waveBytes;               // LDS per wave: ring + work row + sink
    const uint32_t *rowTap;      // (dstH + 1) x VY x {(c, c) splat, ring byte offset of the clamped row}
    const int4 *rows;            // {lo, hi, hi % R, deno} per output row
    const int4 *segs;            // 2 per row: {first, ring offset of first, border, first of row
                                 // + kWalkD}, {yM, yS, yNeg, 0} (plan.hpp WalkSeg; padded past the end)
};
// strips stripLo + i * stripStride (i < strips; strips < 0: all of them)
hipError_t launch_walk(const WalkDev &w, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s,
                       int stripLo = 0, int strips = -1, int stripStride = 1);

// --- exact 2x Lanczos-2/3 upscale, main rows x middle columns (plan.hpp Up2Tables).
struct Up2Dev {
    int srcW, srcH, dstW, dstH;
    int F;                       // factor: 2 or 3 (output y = F k + j takes phase j)
    int NT;                      // taps per axis (4 or 6)
    int np;                      // producing lanes per wave (0 = auto)
    uint32_t cy0;                // phase 0 rows: (c, c) splat of the single tap (the source row itself)
    uint32_t cy1[2][6];          // phase 1 .. F-1 rows: (c, c) splats of the NT taps
    uint32_t cx0;                // phase 0 columns: (c, 0) of the single tap
    uint32_t cx1[2][3];          // phase 1 .. F-1 columns: int16 coefficient pairs of the NT taps
    uint32_t xM[2][24];          // edge-lane exact divisions (left / right 8 F columns)
    int xT[2][24];
    int m0, m1;                  // main rows; the others are masked border rows divided by
    uint32_t yM[2][16];          //   magic_y (top: row y, bottom: row y - m1)
    int yS[2][16];
};
hipError_t launch_up2(const Up2Dev &u, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s);

// Exact 3:2 Lanczos-3 downscale (plan.hpp D32Tables): main rows x all columns.
struct D32Dev {
    int srcW, srcH, dstW, dstH;
    int np;                      // producing lanes per wave (0 = auto)
    int pd;                      // row groups loaded ahead (1, 2, 4; 0 = default 1)
    int variant;                 // tap structure: 0 Lanczos-3 (10 taps), 1 Lanczos-2 (6 taps)
    uint32_t cy[2][8];           // (c, c) u16 splats: phase p's taps at group rows 2p .. 2p + 7
    uint32_t cx[2][5];           // phase p's (c_2q, c_2q+1) int16 pairs
    uint32_t xM[2][8];           // edge-lane exact divisions (left / right 8 columns)
    int xT[2][8];
    int m0, m1;                  // main rows; the others are masked border rows divided by
    uint32_t yM[2][8];           //   magic_y (top: row y, bottom: row y - m1)
    int yS[2][8];
};
hipError_t launch_d32(const D32Dev &d, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s);

// Exact 3:1 Lanczos-2/3 downscale (plan.hpp D31Tables): every row and column.
struct D31Dev {
    int srcW, srcH, dstW, dstH;
    int np;                      // producing lanes per wave (0 = auto)
    int pd;                      // output rows loaded ahead (Lanczos-3: 1, 5; Lanczos-2: 1, 2, 4; 0 = 1)
    int variant;                 // tap structure: 0 Lanczos-3 (18 taps), 1 Lanczos-2 (12 taps)
    uint32_t cc, cp[5];          // (c, c) u16 splats: the centre tap, the symmetric pairs' taps
    uint32_t cxe[9], cxo[9];     // (c_2q, c_2q+1) / (c_2q+1, c_2q+2) int16 pairs: even / odd window starts
    uint32_t xM[2][4];           // edge-lane exact divisions (left / right 4 columns)
    int xT[2][4];
    int m0, m1;                  // main rows; the others are masked border rows divided by
    uint32_t yM[2][8];           //   magic_y (top: row y, bottom: row y - m1)
    int yS[2][8];
};
hipError_t launch_d31(const D31Dev &d, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s);

// Exact vertical ratio, tabled columns (plan.hpp RyxTables): every row and column.
constexpr int kRyxPadK = 24;     // work-row padding (u16 entries) left of column 0: plan.hpp kRyxPad
struct RyxDev {
    bool lanczos;
    int srcW, srcH, dstW, dstH;
    int P, Q, taps, NP;
    int off;                     // group m's window starts at source row P m + off
    int m0, m1;                  // Lanczos main rows; the others are masked border rows (magic_y)
    uint32_t yM[2][16];
    int yS[2][16];
    const uint32_t *rowCoef;     // Q x taps (c, c) splats
    const int4 *cols;            // per column {work byte offset of the even start, magic, shift, 0}
    const uint32_t *colCoef;     // dstW x NP pairs
    // column split: `parts` workgroups per (band, frame), part k writes output columns
    // [xs[k], xs[k+1]) from source columns [cs[k], ce[k]) (multiples of 4); parts = 1: the whole row
    int parts;                   // 1 .. 16
    int threads;                 // threads per workgroup (4 source columns each, a multiple of 64)
    int xs[17], cs[16], ce[16];
    // 1: every thread's two columns are adjacent (xs[k] + 2i, + 1) with windows 1 or 2 pairs apart
    // (kernels.hip ryx_kernel ADJ); 0: columns i and half + i of the part
    int adj = 0;
    int cpt = 2;                 // output columns per thread (2; 4 at the Lanczos-3 4:9 upscale)
    // 1: every column has the same coefficient pairs (Lanczos 2:1 columns: one phase, windows all
    // starting on the same parity), so the kernel reads them once as scalars (kernels.hip UC)
    int uc = 0;
};
hipError_t launch_ryx(const RyxDev &d, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s);

// General-row variant (plan.hpp build_ryg; kernels.hip ryg_kernel): ryx's tabled columns and column
// parts, rows from a per-row record table instead of an exact P:Q.
#ifndef IQO_RYG_PD
#define IQO_RYG_PD 4  // (variant builds: 6; plan.hpp kRygRecPad must stay >= PD + 2)
#endif
constexpr int kRygPD = IQO_RYG_PD;  // ryg_kernel: output rows loaded ahead (the instantiations' PD)
struct RygDev {
    bool lanczos;
    int srcW, srcH, dstW, dstH;
    int taps, NP;
    int m0, m1;                  // Lanczos main rows; the others are masked border rows (magic_y)
    uint32_t yM[2][16];
    int yS[2][16];
    // per output row y (dstH + padding): {first window row s(y), offset of the row's taps in rowCoef,
    // s(y + kRygPD - 1), 0} -- the kernel fetches row y + 2's record with one scalar load per row
    const int4 *rowRec;
    const uint32_t *rowCoef;     // phases x taps (c, c) splats
    const int4 *cols;            // as RyxDev
    const uint32_t *colCoef;
    int parts, threads;
    int xs[17], cs[16], ce[16];
    int cpt;                     // output columns per thread: 2 .. 4 (abi.hip ryx_dev)
    int nl = 2;                  // rows loaded per output row: 2 (downscales, windows 1 or 2 rows apart),
                                 // 1 (upscales, windows 0 or 1 rows apart)
    // upscales whose window positions hold 1 .. posRows output rows each (kernels.hip ryu_kernel):
    // per window start s, record s - posBase = {first output row, rows, tap offsets of those rows},
    // 8 ints, padded by plan.hpp kRyuPosPad records; null: ryg_kernel's NL = 1 mode
    const int4 *posRec = nullptr;  // (8 ints per record: two int4)
    int posBase = 0;
    int posRows = 2;               // the most output rows a window position holds (2 or 3)
    // ryu_kernel run mode (cpt 4, parts on multiples of 4 columns): dstW x run pairs (plan.hpp colRun)
    const uint32_t *colRun = nullptr;
    int run = 0;
};
hipError_t launch_ryg(const RygDev &d, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s);

// Exact 2:3 Lanczos-3 upscale (plan.hpp U23Tables).
struct U23Dev {
    int srcW, srcH, dstW, dstH;
    int np;                      // producing lanes per wave (0 = auto)
    int pd;                      // row groups loaded ahead (1, 2; 0 = default 1)
    uint32_t cy0, cy[2][6];      // (c, c) u16 splats: phase 0's tap, phases 1 and 2
    uint32_t cx0, cx[2][3];      // (c, 0) / (c_2q, c_2q+1) int16 pairs
    uint32_t xM[2][12];          // edge-lane exact divisions (left / right 12 columns)
    int xT[2][12];
    int m0, m1;                  // main rows; the others are masked border rows
    uint32_t yM[2][8];
    int yS[2][8];
};
hipError_t launch_u23(const U23Dev &d, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s);

// Exact 2:3 Linear upscale (plan.hpp L23Tables).
struct L23Dev {
    int srcW, srcH, dstW, dstH;
    int np;                      // producing lanes per wave (0 = auto)
    int pd;                      // row groups loaded ahead (1, 2; 0 = default 2)
    uint32_t cy[3][2];           // (c, c) u16 splats of phase j's two taps
    uint32_t cx[3];              // phase j's (c_0, c_1) u16 pair
};
hipError_t launch_l23(const L23Dev &d, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s);

// Exact 3:2 Area downscale (plan.hpp A32Tables).
struct A32Dev {
    int srcW, srcH, dstW, dstH;
    int np;                      // producing lanes per wave (0 = auto)
    int pd;                      // row pairs loaded ahead (2, 4, 8; 0 = default 4)
    uint32_t cy[2][2];           // (c, c) u16 splats of phase p's two taps
    uint32_t cx[2];              // phase p's (c_0, c_1) u16 pair
};
hipError_t launch_a32(const A32Dev &d, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s);

// --- Lanczos row-band streamer (integer ratio, single phase).
struct LanczosDev {
    int KY, KX, NY, NXP, offX;
    int srcW, srcH, dstW, dstH;
    int offY;
    uint32_t cy[16];             // (c, c) u16 pairs
    uint32_t cx[16];             // (c_2p, c_2p+1) int16 pairs
    int mainBeginY, mainEndY, mainBeginX, mainEndX;
    // exact border divisions by multiply-high (plan.hpp FastLanczos): kernel arguments, so they
    // arrive in SGPRs and cost no device table
    uint32_t yTopM[16], yBotM[16], xM[8];
    int yTopS[16], yBotS[16], xT[8];
    int yTopNeg, yBotNeg, xNeg;  // bit i: border row / column i has a negative denominator
    int dbg;                     // variant builds only (kernels.hip IQO_DBG); ignored otherwise
    int prefetch;                // prefetch depth in output rows (1..3)
    // symmetric streamer (plan.hpp FastLanczos::sym)
    int sym;                     // 1: block-shared symmetric, 2: per-wave symmetric, 0: accumulator ring
    int NX, offXO;               // unpadded X taps, odd first tap column
    uint32_t cxo[8];             // (c_2p, c_2p+1) int16 pairs of the unpadded X table (Lanczos-5: below)
    int np;                      // producing lanes per wave (0 = auto)
    int rounds;                  // block-shared streamer: target rounds of resident workgroups for the
                                 // auto band count (0 = default 6, -1 = one-round makespan model)
    int stack;                   // narrow frames: several frames per workgroup (lanczos_stack_kernel)
    int tail;                    // block-shared streamer: short bands for each XCD's last frame
                                 // (0 = auto, -1 = off, n = n bands of that frame)
    // Lanczos-5 2:1 (NX = 20, block-shared symmetric streamer only) reuses fields that streamer does
    // not read, so the argument layout of every instantiation stays as it is (growing it cost C2
    // 1.5 %): X pairs 8, 9 in cy[8], cy[9] (the symmetric streamer reads cy[0 .. NY/2)); the edge
    // lanes' 8 exact divisions per side (5 border columns: left lane k < 8, right lane k >= 8,
    // identity in the interior) as multipliers in cx[0 .. 16) (the ring streamer's padded table)
    // and shifts in xM[0 .. 8), xT[0 .. 8) (the 4-column scheme's constants)
#ifdef IQO_VARIANT_DEBUG
    // variant builds only: per-workgroup {start, end (100 MHz clock), HW_ID, XCC_ID} records of the
    // block-shared streamer (scripts/probes/wg_trace.py); 0 = off.  Not in the shipped layout.
    uint64_t trace;
#endif
};
bool lanczos_stream_supported(int KY, int KX, int NY, int NXP, int offX);
hipError_t launch_lanczos_stream(const LanczosDev &l, const Io &io, int rowBegin, int rowEnd, int bands,
                                 hipStream_t s);
int lanczos_stream_block(int srcW);

// --- Area integer-ratio kernel.
struct AreaDev {
    int KY, KX, srcW, dstW, dstH;
    uint32_t cy[16];             // (c, c) u16 pairs
    uint32_t cx[8];              // (c_2p, c_2p+1) u16 pairs
    int lin;                     // 1: Linear at exactly 2:1 (linear_d2_body: taps 2i+1, 2i+2, edge
    int srcH;                    //    rows / columns replicated); cy[0..1] / cx[0] its two taps
};
hipError_t launch_area_int(const AreaDev &a, const Io &io, int rowBegin, int rowEnd, hipStream_t s);

// --- exact 2x bilinear upsampler.
struct LinearDev {
    int srcW, srcH, dstW, dstH;
    int F;                       // exact factor, 2 or 3
    uint32_t cy[3];              // per phase (c0, c1) u16 pairs
    uint32_t cx[3];
    int dbg;                     // variant builds only: 16 = plain (not nontemporal) stores
    int np;                      // producing lanes per wave (0 = auto)
};
hipError_t launch_linear_up2(const LinearDev &l, const Io &io, int rowBegin, int rowEnd, int bands,
                             hipStream_t s);

// --- YUV 4:2:0: the Y, U and V planes of a batch in ONE launch (grid.z = plane) when both plane
// kinds have a fused instantiation; hipErrorNotSupported otherwise (launch plane by plane).
// Frame f of each plane: Io as above; all three Io must hold the same frame count.
hipError_t launch_yuv420_lanczos(const LanczosDev &y, const Io &ioY, const LanczosDev &c, const Io &ioU,
                                 const Io &ioV, hipStream_t s);
hipError_t launch_yuv420_area(const AreaDev &y, const Io &ioY, const AreaDev &c, const Io &ioU, const Io &ioV,
                              hipStream_t s);
hipError_t launch_yuv420_linear(const LinearDev &y, const Io &ioY, const LinearDev &c, const Io &ioU,
                                const Io &ioV, hipStream_t s);

} // namespace iqo_amd
