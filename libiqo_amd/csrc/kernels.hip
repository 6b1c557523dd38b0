// kernels.hip -- gfx950 (CDNA4) kernels for the separable U8 resize hot path: the streamers (C1-C4),
// the general / tile / walker kernels and the fused YUV launches.  The exact- and general-ratio kernels
// live in kernels_ratio.hip; both include kernels_dev.hpp.
//
// All arithmetic restates the reference's Generic fixed point exactly:
//   Lanczos: int16 vertical accumulator with wrap (IQOLanczosResizerImpl_Generic.cpp:499-516),
//            masked + renormalised borders (:464-490, :539-574), int32 horizontal dot product
//            with (sum + 2^19) >> 20 rounding (:582-612).
//   Area:    u16 vertical accumulator (IQOAreaResizerImpl_Generic.cpp:303-320), (sum+2^22)>>23.
//   Linear:  u16 vertical blend, 1-px replicated borders (IQOLinearResizerImpl_Generic.cpp:290-407).
// No MFMA: this is a memory-bound 1-D stencil.  The interior math uses packed 16-bit VALU
// (v_pk_mad_u16 -- its low 16 bits ARE the reference's int16 wrap) for the vertical taps and
// v_dot2 (int16 / u16 pairs, int32 accumulate) for the horizontal taps.
#include "kernels_dev.hpp"

namespace iqo_amd {
namespace {

// ================================================================ general kernel

enum { KMAIN = 0, KLO = 1, KHI = 2, KID = 3 };

struct GeneralArgs {
    GeneralDev g;
    Io io;
    int rowBegin;
};

__device__ __forceinline__ int src_px(const GeneralArgs &a, const uint8_t *srcF, int row, int col)
{
    return srcF[static_cast<int64_t>(row - a.io.srcRow0) * a.io.srcSt + col];
}

// Vertical value at (row record yi, source column col): the reference's work[col].
__device__ int y_value(const GeneralArgs &a, const uint8_t *srcF, int4 yi, int col)
{
    const GeneralDev &g = a.g;
    if (g.method == 0) {  // Lanczos, int16 work row
        if (yi.z == KID)
            return static_cast<int16_t>(static_cast<uint16_t>(src_px(a, srcF, yi.x, col) * 64));
        if (yi.z == KMAIN) {
            int16_t acc = 0;  // resizeYmain :509-515
            for (int i = 0; i < g.nY; ++i)
                acc = static_cast<int16_t>(acc + src_px(a, srcF, yi.x + i, col) * g.tabY[yi.y + i]);
            return acc;
        }
        int16_t nume = 0;  // resizeYborder :477-489
        for (int i = 0; i < g.nY; ++i) {
            int r = yi.x + i;
            if (r >= 0 && r < g.srcH)
                nume = static_cast<int16_t>(nume + src_px(a, srcF, r, col) * g.tabY[yi.y + i]);
        }
        return static_cast<int16_t>(exact_div(static_cast<int>(nume) * 64, yi.w));
    }
    if (yi.z == KID)
        return static_cast<uint16_t>(src_px(a, srcF, yi.x, col) * 256);
    if (g.method == 1) {  // Area, u16 work row (resizeYmain :313-319); weight-0 tap past the end clamped
        uint16_t acc = 0;
        for (int i = 0; i < g.nY; ++i) {
            int r = min(yi.x + i, g.srcH - 1);
            acc = static_cast<uint16_t>(acc + src_px(a, srcF, r, col) * g.tabY[yi.y + i]);
        }
        return acc;
    }
    // Linear (resize :241-281)
    if (yi.z == KLO)
        return static_cast<uint16_t>(src_px(a, srcF, 0, col) * 256);
    if (yi.z == KHI)
        return static_cast<uint16_t>(src_px(a, srcF, g.srcH - 1, col) * 256);
    int r0 = max(0, min(yi.x, g.srcH - 1)), r1 = max(0, min(yi.x + 1, g.srcH - 1));
    uint16_t acc = static_cast<uint16_t>(src_px(a, srcF, r0, col) * g.tabY[yi.y]);
    acc = static_cast<uint16_t>(acc + src_px(a, srcF, r1, col) * g.tabY[yi.y + 1]);
    return acc;
}

// Horizontal value at output column x (record xi) from the LDS work row covering [lo, hi).
__device__ int x_value_rec(const GeneralDev &g, const int *w, int lo, int hi, int x, int4 xi);

__device__ int x_value(const GeneralArgs &a, const int *w, int lo, int hi, int x)
{
    return x_value_rec(a.g, w, lo, hi, x, a.g.xInfo[x]);
}

__device__ int x_value_rec(const GeneralDev &g, const int *w, int lo, int hi, int /*x*/, int4 xi)
{
    auto W = [&](int col) { return w[max(0, min(col, hi - 1) - lo)]; };
    if (g.method == 0) {
        if (xi.z == KID)  // resizeX Y-only branch :520-527
            return clamp255(static_cast<int16_t>((W(xi.x) + 32) >> 6));
        if (xi.z == KMAIN) {  // resizeXmain :605-610
            int sum = 0;
            for (int i = 0; i < g.nX; ++i)
                sum += W(xi.x + i) * g.tabX[xi.y + i];
            return clamp255(static_cast<int16_t>((sum + (1 << 19)) >> 20));
        }
        int nume = 0;  // resizeXborder :563-572
        for (int i = 0; i < g.nX; ++i) {
            int col = xi.x + i;
            if (col >= 0 && col < g.srcW)
                nume += W(col) * g.tabX[xi.y + i];
        }
        return clamp255(static_cast<int16_t>(exact_div(nume + (1 << 19), xi.w * 64)));
    }
    if (xi.z == KID)
        return clamp255(static_cast<int16_t>((W(xi.x) + 128) >> 8));
    auto u16clamp = [](int v) {  // uint8(clamp<uint16_t>(0, 255, int16(v)))
        uint16_t u = static_cast<uint16_t>(static_cast<int16_t>(v));
        return static_cast<int>(u > 255 ? 255 : u);
    };
    if (g.method == 1) {  // Area resizeXmain :349-367
        int sum = 0;
        for (int i = 0; i < g.nX; ++i)
            sum += W(min(xi.x + i, g.srcW - 1)) * g.tabX[xi.y + i];
        return u16clamp((sum + (1 << 22)) >> 23);
    }
    if (xi.z == KLO)  // Linear resizeXborder :355-366
        return u16clamp((W(0) + 128) >> 8);
    if (xi.z == KHI)
        return u16clamp((W(g.srcW - 1) + 128) >> 8);
    int c0 = max(0, min(xi.x, g.srcW - 1)), c1 = max(0, min(xi.x + 1, g.srcW - 1));
    int sum = W(c0) * g.tabX[xi.y] + W(c1) * g.tabX[xi.y + 1];  // :400-405
    return u16clamp((sum + (1 << 22)) >> 23);
}

__global__ __launch_bounds__(256) void general_kernel(GeneralArgs a)
{
    extern __shared__ __attribute__((aligned(16))) int wrow[];
    const int y = a.rowBegin + static_cast<int>(blockIdx.x);
    const uint8_t *srcF = a.io.src + static_cast<int64_t>(blockIdx.y) * a.io.srcFrameSt;
    uint8_t *dstRow = a.io.dst + static_cast<int64_t>(blockIdx.y) * a.io.dstFrameSt +
                      static_cast<int64_t>(y - a.io.dstRow0) * a.io.dstSt;
    const int4 yi = a.g.yInfo[y];
    for (int c = 0; c < a.g.nChunks; ++c) {
        const int4 ch = a.g.chunks[c];
        for (int col = ch.z + static_cast<int>(threadIdx.x); col < ch.w; col += static_cast<int>(blockDim.x))
            wrow[col - ch.z] = y_value(a, srcF, yi, col);
        lds_barrier();
        const int x = ch.x + static_cast<int>(threadIdx.x);
        if (x < ch.y)
            dstRow[x] = static_cast<uint8_t>(x_value(a, wrow, ch.z, ch.w, x));
        lds_barrier();
    }
}

// ================================================================ separable tile kernel
//
// Every shape the specialised kernels do not take: multi-phase ratios (1920 -> 1280), Lanczos
// upscaling and degrees 1-9, non-integer Area, Linear at ratios other than 2x.  A workgroup
// computes a tile of TH output rows x CT output columns of one frame, in two passes through LDS:
//   1. vertical: the work rows of the tile's source-column span [lo8, lo8 + 8*groups), one task
//      = (output row, 8 source columns): nYp taps, each an 8-byte buffer load of a clamped row,
//      a v_perm unpack into u16 pairs (per-lane selectors replicate edge columns) and
//      v_pk_mad_u16 -- whose low 16 bits are the reference's int16 / u16 wrap;
//   2. horizontal: a thread owns 4 adjacent output columns (their coefficient pairs live in
//      VGPRs for the whole tile) and walks the tile's rows: NP v_dot2 over aligned u16 pairs of
//      the work row, the rounding shift (or the exact border division), one dword store.
// The per-row / per-column windows come from build_tile_tables (plan.cpp), which folds the
// reference's identity, replicated-border and masked-border cases into plain tap windows; the
// results are bit-exact with general_kernel / the reference for every shape.

struct TileArgs {
    TileDev t;
    Io io;
    int rowBegin, rowEnd;
    int srcBytes, dstBytes;
    int nTx, nTy;       // column tiles, row tiles per frame
    unsigned nTiles;    // nTx * nTy * frames (flat grid)
};

template <int NP, bool LZ>
__global__ __launch_bounds__(256) void tile_kernel(TileArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t tile_lds[];
    const TileDev &t = a.t;
    const int tid = static_cast<int>(threadIdx.x);
    // Workgroups are dispatched round-robin over the 8 XCDs (flat id L goes to XCD L mod 8), and
    // each XCD has its own L2.  Give XCD x a contiguous range of tiles, row tiles fastest: the
    // tiles resident on one XCD at a time are vertical (and horizontal) neighbours, so the halo
    // rows / columns they share are fetched from HBM once and hit that XCD's L2 afterwards
    // (round 2: column tiles fastest and plain dispatch order both slower, profiles/r02/tile_xcd_ab.txt).
    int tileX, tileY, frame;
    {
        const unsigned lg = xcd_chunks(blockIdx.x, a.nTx * a.nTy, a.nTiles);
        const unsigned rest = lg / static_cast<unsigned>(a.nTy);
        tileY = static_cast<int>(lg - rest * static_cast<unsigned>(a.nTy));
        frame = static_cast<int>(rest / static_cast<unsigned>(a.nTx));
        tileX = static_cast<int>(rest - static_cast<unsigned>(frame) * static_cast<unsigned>(a.nTx));
    }
    const int y0 = a.rowBegin + tileY * t.TH;
    const int nRows = min(t.TH, a.rowEnd - y0);
    // LDS: work rows [TH][pitchDw] | row records [TH] | tap records [TH][nYp] (coefficient, LDS
    // offset of the clamped source row) | border divisors [CT] | source tile [srcRows][spitch]
    uint32_t *const work = tile_lds;
    int4 *const recs = reinterpret_cast<int4 *>(tile_lds + t.TH * t.pitchDw);
    uint2 *const taps = reinterpret_cast<uint2 *>(recs + t.TH);
    int *const DL = reinterpret_cast<int *>(taps + t.TH * t.nYp);
    uint8_t *const srcL = reinterpret_cast<uint8_t *>(DL + t.CT);

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(frame) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(frame) * a.io.dstFrameSt;
    // alignment of this frame (frame strides may be odd): the source buffer starts at the dword
    // below the frame; rows are fetched as 8 bytes when base and stride are dword-aligned, else
    // as 12 dword-aligned bytes and a byte shift.  Stores are dwords only when aligned.
    const int srcMis = static_cast<int>(reinterpret_cast<uintptr_t>(srcFrame) & 3);
    const bool srcA4 = srcMis == 0 && !(a.io.srcSt & 3);
    const bool dstA4 = !(reinterpret_cast<uintptr_t>(dstFrame) & 3) && !(a.io.dstSt & 3);
    const __amdgpu_buffer_rsrc_t srcR = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(srcFrame - srcMis), 0, a.srcBytes + srcMis, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcW = t.srcW, srcSt = static_cast<int>(a.io.srcSt), srcRow0 = a.io.srcRow0;
    const int4 sp = t.spans[tileX];  // {lo8, groups, any border column}
    const int spitch = t.spitch;
    const int rmin = t.rows[y0].y;
    const int nR = t.rows[y0 + nRows - 1].z - rmin + 1;  // row windows are monotone
    const int colStart = max(sp.x, 0);

    // 0. stage the tile's source rows [rmin, rmin + nR) x columns [colStart, lo8 + 8 groups):
    //    one burst of independent 8-byte loads; the last groups of a row (a whole-word load there
    //    could pass the end of the frame) as clamped single bytes, replicating the last column
    {
        const int sG = sp.y - ((colStart - sp.x) >> 3);
        const int gNum = srcW - 12 - colStart;  // groups with c + 12 <= srcW (floor division)
        const int gE = gNum < 0 ? 0 : min(gNum / 8 + 1, sG);
        const int total = nR * gE;
        // n / gE = umulhi(n, mG) (exact for n * gE < 2^32); gE = 1 has no 32-bit magic
        const uint32_t mG = gE > 1 ? 0xffffffffu / static_cast<uint32_t>(gE) + 1u : 0u;
        for (int t0 = tid; t0 < total; t0 += 256 * 8) {
            u32x2 v[8];
            int dstOff[8];
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const int tt = t0 + 256 * b;
                const bool valid = tt < total;
                const int rr = valid ? (gE > 1 ? static_cast<int>(__umulhi(static_cast<uint32_t>(tt), mG)) : tt) : 0;
                const int gg = valid ? tt - rr * gE : 0;
                const int o = static_cast<int>(__umul24(rmin + rr - srcRow0, srcSt)) + srcMis + colStart + 8 * gg;
                if (srcA4) {
                    v[b] = __builtin_amdgcn_raw_buffer_load_b64(srcR, valid ? o : 0x7ff00000, 0, 0);
                } else {
                    const int d = o & 3;
                    const u32x3 w = __builtin_amdgcn_raw_buffer_load_b96(srcR, valid ? o - d : 0x7ff00000, 0, 0);
                    v[b] = u32x2{__builtin_amdgcn_alignbyte(w.y, w.x, d), __builtin_amdgcn_alignbyte(w.z, w.y, d)};
                }
                dstOff[b] = valid ? rr * spitch + 8 * gg : -1;
            }
#pragma unroll
            for (int b = 0; b < 8; ++b)
                if (dstOff[b] >= 0)
                    *reinterpret_cast<u32x2 *>(srcL + dstOff[b]) = v[b];
        }
        const int nEdge = sG - gE;
        for (int tt = tid; tt < nR * nEdge; tt += 256) {
            const int rr = tt / nEdge, gg = gE + (tt - (tt / nEdge) * nEdge);
            const int o = static_cast<int>(__umul24(rmin + rr - srcRow0, srcSt)) + srcMis;
            const int c = colStart + 8 * gg;
            uint32_t w0 = 0, w1 = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t bt = __builtin_amdgcn_raw_buffer_load_b8(srcR, o + min(c + k, srcW - 1), 0, 0);
                if (k < 4)
                    w0 |= bt << (8 * k);
                else
                    w1 |= bt << (8 * (k - 4));
            }
            *reinterpret_cast<u32x2 *>(srcL + rr * spitch + 8 * gg) = u32x2{w0, w1};
        }
    }
    // row records, tap records, border divisors
    for (int i = tid; i < nRows; i += 256)
        recs[i] = t.rows[y0 + i];
    for (int i = tid; i < nRows * t.nYp; i += 256) {
        const uint2 rt = t.rowTap[static_cast<int64_t>(y0) * t.nYp + i];  // (coefficient, clamped row)
        taps[i] = make_uint2(rt.x, static_cast<uint32_t>((static_cast<int>(rt.y) - rmin) * spitch));
    }
    const bool borderTile = LZ && sp.z;
    if (borderTile)
        for (int i = tid; i < t.CT; i += 256)
            DL[i] = tileX * t.CT + i < t.dstW ? t.cols[tileX * t.CT + i].y : 0;

    // horizontal ownership: 4 adjacent output columns per thread, rows jStart, jStart + jStep, ...
    const int nQ = t.CT >> 2;
    const int q = tid & (nQ - 1), jStart = tid >> t.log2nQ, jStep = 256 >> t.log2nQ;
    const int x0 = tileX * t.CT + 4 * q;
    uint32_t cf[4][NP];
    int woff[4];
    const int Q = x0 >> 2;  // coalesced: lane-consecutive quads
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        woff[k] = (t.colA[k * t.nQp + Q] - sp.x) >> 1;
#pragma unroll
        for (int p = 0; p < NP; ++p)
            cf[k][p] = t.colCoef[(p * 4 + k) * t.nQp + Q];
    }
    lds_barrier();

    // 1. vertical pass: tasks (row j, group g), g fastest; taps from the staged tile
    {
        const int nG = sp.y;
        const int dj = 256 / nG, dg = 256 - dj * nG;
        int j = tid / nG, g = tid - (tid / nG) * nG;
        while (j < nRows) {
            const int cb = sp.x + 8 * g;
            uint32_t s0 = 0x0c010c00u, s1 = 0x0c030c02u, s2 = 0x0c050c04u, s3 = 0x0c070c06u;
            if (cb < 0) {  // left edge group: replicate source column 0
                auto b = [&](int k) { return static_cast<uint32_t>(max(cb + k, 0)); };
                s0 = b(0) | (b(1) << 16) | 0x0c000c00u;
                s1 = b(2) | (b(3) << 16) | 0x0c000c00u;
                s2 = b(4) | (b(5) << 16) | 0x0c000c00u;
                s3 = b(6) | (b(7) << 16) | 0x0c000c00u;
            }
            const uint8_t *colL = srcL + (max(cb, 0) - colStart);
            const uint2 *tj = taps + j * t.nYp;
            uint32_t acc0 = 0, acc1 = 0, acc2 = 0, acc3 = 0;
            for (int i = 0; i < t.nYp; i += 2) {
                const uint4 c2 = *reinterpret_cast<const uint4 *>(tj + i);  // (coef, offset) x 2
                const u32x2 v0 = *reinterpret_cast<const u32x2 *>(colL + c2.y);
                const u32x2 v1 = *reinterpret_cast<const u32x2 *>(colL + c2.w);
                acc0 = pk_mad(__builtin_amdgcn_perm(v0.y, v0.x, s0), c2.x, acc0);
                acc1 = pk_mad(__builtin_amdgcn_perm(v0.y, v0.x, s1), c2.x, acc1);
                acc2 = pk_mad(__builtin_amdgcn_perm(v0.y, v0.x, s2), c2.x, acc2);
                acc3 = pk_mad(__builtin_amdgcn_perm(v0.y, v0.x, s3), c2.x, acc3);
                acc0 = pk_mad(__builtin_amdgcn_perm(v1.y, v1.x, s0), c2.z, acc0);
                acc1 = pk_mad(__builtin_amdgcn_perm(v1.y, v1.x, s1), c2.z, acc1);
                acc2 = pk_mad(__builtin_amdgcn_perm(v1.y, v1.x, s2), c2.z, acc2);
                acc3 = pk_mad(__builtin_amdgcn_perm(v1.y, v1.x, s3), c2.z, acc3);
            }
            const int4 r = recs[j];
            if (LZ && r.w != 0) {  // masked + renormalised border row: int16(nume * 64 / deno)
                auto dv = [&](uint32_t pr) {
                    const int lo = exact_div(static_cast<int>(static_cast<int16_t>(pr & 0xffffu)) * 64, r.w);
                    const int hi = exact_div(static_cast<int>(static_cast<int16_t>(pr >> 16)) * 64, r.w);
                    return (static_cast<uint32_t>(lo) & 0xffffu) | (static_cast<uint32_t>(hi) << 16);
                };
                acc0 = dv(acc0);
                acc1 = dv(acc1);
                acc2 = dv(acc2);
                acc3 = dv(acc3);
            }
            *reinterpret_cast<uint4 *>(work + j * t.pitchDw + 4 * g) = make_uint4(acc0, acc1, acc2, acc3);
            j += dj;
            g += dg;
            if (g >= nG) {
                g -= nG;
                ++j;
            }
        }
    }
    lds_barrier();

    // 2. horizontal pass
    const int dstSt = static_cast<int>(a.io.dstSt);
    for (int j = jStart; j < nRows; j += jStep) {
        const uint32_t *w = work + j * t.pitchDw;
        uint32_t bytes[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            int s = LZ ? (1 << 19) : (1 << 22);
#pragma unroll
            for (int p = 0; p < NP; ++p)
                s = LZ ? sdot2(w[woff[k] + p], cf[k][p], s)
                       : static_cast<int>(udot2(w[woff[k] + p], cf[k][p], static_cast<uint32_t>(s)));
            if (LZ) {
                int v = s >> 20;  // within int16: the reference's int16 cast is the identity here
                if (borderTile) {
                    const int Dk = DL[4 * q + k];
                    if (Dk != 0)
                        v = static_cast<int16_t>(exact_div(s, Dk));
                }
                bytes[k] = static_cast<uint32_t>(min(max(v, 0), 255));
            } else {
                bytes[k] = min((static_cast<uint32_t>(s) >> 23) & 0xffffu, 255u);
            }
        }
        const int off = (y0 + j - a.io.dstRow0) * dstSt + x0;
        if (dstA4 && x0 + 4 <= t.dstW) {
            const uint32_t o = opaque(bytes[0] | (bytes[1] << 8)) | (bytes[2] << 16) | (bytes[3] << 24);
            __builtin_amdgcn_raw_buffer_store_b32(o, dstR, off, 0, 0);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (x0 + k < t.dstW)
                    __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(bytes[k]), dstR, off + k, 0, 0);
        }
    }
}

// ================================================================ Lanczos row-band streamer
//
// One WAVE = one row band of one frame x one strip of output columns; waves are independent (no
// LDS, no barriers).  Lane l of a wave owns the 16 source columns [cb, cb + 16), cb = KX*x0 - 16
// + 16*l, and (lanes 1..62) produces the 16/KX output columns that start at x0 + (l-1)*16/KX.
// The wave walks its band's output rows top to bottom; each source row is fetched from HBM once
// per band with coalesced 16-B buffer loads (off-image rows/columns lie outside the buffer
// range and read as zero -- exactly the masked border sums of the reference), unpacked to u16
// pairs, and multiplied into the P = NY/KY output rows that still need it (accumulator ring).
// The vertical sum is the reference's int16 work row; the horizontal taps read it from the
// lane itself and its neighbours (DPP row shifts), then two packed saturating shifts produce the
// output bytes.
//
// Control flow is straight-line: the row loop is unrolled by LV = lcm(P, PD) so every ring slot
// and prefetch slot is a static register (no phase dispatch, no loop-carried register shuffles),
// and only uniform branches remain (priming rows, band end, border rows, edge waves).
//
// Border rows / columns differ from the interior only by a divisor (renormalisation, the
// reference's resizeYborder :487-489 and resizeXborder :572); both are exact multiply-high
// divisions with host-computed constants (plan.cpp magic_y / magic_x).  The last wave of a row
// is aligned to the right image edge (it may overlap its neighbour; overlapping bytes are equal)
// so the at most 4 border columns per side sit at static positions of one lane.

struct LanczosArgs {
    LanczosDev l;
    Io io;
    int rowBegin, rowEnd, rowsPerBand;
    int srcBytes, dstBytes;  // extent of one frame's source window / destination band (buffer range)
    int bands, wavesPerRow;  // wave grid per frame: band-major, column-minor
    int dbg;                 // variant builds only (IQO_DBG): 1 = no stores,
                             // 2 = no source loads, 4 = no edge columns, 8 = no border rows
                             // (wrong output), 32 = all bands walk top-down.  0 in production.
    int np;                  // producing lanes per wave (symmetric streamer)
    int rowPitch, chunks;    // block-shared streamer: LDS ring row pitch, 1-KiB DMA chunks per row
    int lastLanes;           // block-shared streamer: lanes of the last DMA chunk (0 = all 64)
    int fpw, frames;         // frame-stacked streamer: frames per workgroup, frames in the launch
    // block-shared streamer, XCD tail split (tailBands > 0): XCD x takes frames [x F8, (x+1) F8),
    // all but the last in `bands` bands of rowsPerBand rows, the last in tailBands bands of
    // tailRows rows, in that order; grid.x = 8 ((F8 - 1) bands + tailBands)
    int tailBands, tailRows, framesPerXcd;
};

template <int KY, int KX, int NY, int NXP, int OFFXD, int PD>
__device__ __forceinline__ void lanczos_stream_kernel_body(const LanczosArgs &a, const unsigned bx, const unsigned by)
{
    constexpr int OUTS = 16 / KX;            // outputs per producing lane
    constexpr int OPW = 62 * OUTS;           // outputs per wave (lanes 1..62)
    constexpr int P = NY / KY;               // output rows pending at once (accumulator ring)
    static_assert(NY % KY == 0, "NY must be a multiple of KY");
    constexpr int LV = P * PD / cgcd(P, PD);  // unroll: accumulator slot x prefetch slot
    constexpr int DLO = OFFXD;               // first work dword a lane reads, relative to its own
    constexpr int DHI = (OUTS - 1) * KX / 2 + OFFXD + NXP / 2;  // one past the last
    static_assert(DLO >= -8 && DHI <= 16, "horizontal taps must stay within the neighbouring lanes");
    static_assert(OUTS == 8, "edge handling assumes 8 outputs per lane (KX == 2)");

    const LanczosDev &L = a.l;
    const int lane = static_cast<int>(threadIdx.x) & 63;
    // wave in block, made provably wave-uniform: otherwise everything derived from it (band,
    // rows, the row counter) is treated as divergent -- row offsets land in VGPRs, every buffer
    // load becomes a readfirstlane loop and row branches become exec-mask branches
    const int wib = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    const int g = static_cast<int>(bx) * 4 + wib;  // wave index in the (band, column) grid
    if (g >= a.bands * a.wavesPerRow)
        return;  // whole wave: nothing below synchronises across waves
    const int band = g / a.wavesPerRow, wcol = g - band * a.wavesPerRow;
    const int y0 = a.rowBegin + band * a.rowsPerBand;
    const int y1 = min(y0 + a.rowsPerBand, a.rowEnd);
    if (y0 >= y1)
        return;

    // first output column of lane 1; the last wave is aligned to the right edge (dstW % 8 == 0)
    const int x0 = max(0, min(wcol * OPW, L.dstW - OPW));
    const int cb = KX * x0 - 16 + 16 * lane;      // first source column of this lane's block
    const int outX = x0 + (lane - 1) * OUTS;      // first output column of this lane
    const bool produce = lane >= 1 && lane <= 62 && outX < L.dstW;
    const int voff = (cb >= 0 && cb < L.srcW) ? cb : 0x7ff00000;  // off-image blocks read zero
    const bool edgeL = x0 == 0, edgeR = x0 + OPW >= L.dstW;       // wave holds border columns
    const bool laneL = outX == 0, laneR = outX == L.dstW - OUTS;  // ... in this lane

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(by) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(by) * a.io.dstFrameSt;
    const __amdgpu_buffer_rsrc_t srcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcFrame), 0, a.srcBytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0;
    const int dbg = IQO_DBG(a);
    const int svoff = (dbg & 2) ? 0x7ff00000 : voff;
    const int stoff = (produce && !(dbg & 1)) ? outX : 0x7ff00000;  // dropped for non-producers

    // Branch-free row load (r < 0 wraps to a huge unsigned soffset, r >= srcH lies past the
    // range): no branches keep the waitcnt counting exact across the unrolled rows.
    auto load_row = [&](int r) -> uint4 {
        u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(srcR, svoff, (r - srcRow0) * srcSt, 2 /* nt */);
        return make_uint4(q.x, q.y, q.z, q.w);
    };

    // Accumulator ring: a source row is multiplied into the partial sums of the P output rows
    // that still need it (tap NY-KY*(q+1)+j for the q-th pending row); row yy completes in slot
    // (yy - yStart) mod P.  Iterations start P-1 rows early to prime the ring.
    uint32_t accR[P][8];
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
        for (int c = 0; c < 8; ++c)
            accR[q][c] = 0;
    const int yStart = y0 - (P - 1);
    // prefetch ring: the KY new source rows of iteration i live in slot i % PD, issued PD
    // iterations ahead
    uint4 pre[PD][KY];
#pragma unroll
    for (int i = 0; i < PD; ++i)
#pragma unroll
        for (int j = 0; j < KY; ++j)
            pre[i][j] = load_row(KY * (yStart + i) + L.offY + NY - KY + j);

    for (int base = yStart; base < y1; base += LV) {
        static_for<LV>([&](auto uc) {
            constexpr int v = decltype(uc)::value;
            constexpr int u = v % P;   // accumulator slot completing at this row
            constexpr int ps = v % PD; // prefetch slot holding this row's new source rows
            const int yy = base + v;
            uint32_t nw[KY][8];
#pragma unroll
            for (int j = 0; j < KY; ++j)
                unpack16(pre[ps][j], nw[j]);
#pragma unroll
            for (int j = 0; j < KY; ++j)  // (rows past the band end are loaded and unused)
                pre[ps][j] = load_row(KY * (yy + PD) + L.offY + NY - KY + j);
            // vertical taps: int16 wrap == low half of the packed u16 MAD; tap-outer so the 8
            // independent column chains interleave (dependent v_pk_mad_u16 need ~9 wait states)
#pragma unroll
            for (int q = 0; q < P; ++q)
#pragma unroll
                for (int j = 0; j < KY; ++j) {
                    const uint32_t cq = L.cy[NY - KY * (q + 1) + j];
                    uint32_t *ar = accR[(u + q) % P];
#pragma unroll
                    for (int c = 0; c < 8; ++c)
                        ar[c] = (q == P - 1 && j == 0) ? pk_mul(nw[j][c], cq) : pk_mad(nw[j][c], cq, ar[c]);
                }
            if (yy < y0 || yy >= y1)
                return;  // priming row / past the band end (uniform)

            uint32_t acc[8];
#pragma unroll
            for (int c = 0; c < 8; ++c)
                acc[c] = accR[u][c];
            if (yy < L.mainBeginY || yy >= L.mainEndY) {
                // border row (uniform, rare): work = int16(int(nume) * 64 / deno); invalid rows
                // were read as zero, so nume is already the masked sum
                const bool top = yy < L.mainBeginY;
                const int bi = top ? yy : yy - L.mainEndY;
                const uint32_t m = top ? L.yTopM[bi] : L.yBotM[bi];
                const int sh = top ? L.yTopS[bi] : L.yBotS[bi];
                const bool neg = ((top ? L.yTopNeg : L.yBotNeg) >> bi) & 1;  // deno < 0 (uniform)
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    acc[c] = ydiv2(acc[c], m, sh);
                    if (neg)  // trunc(n / -d) == -trunc(n / d), per int16 half
                        acc[c] = __builtin_bit_cast(uint32_t, u16x2{0, 0} - __builtin_bit_cast(u16x2, acc[c]));
                }
            }

            // neighbour work columns by DPP (lane l-1 / l+1), then the horizontal taps
            uint32_t d[DHI - DLO];
#pragma unroll
            for (int j = DLO; j < DHI; ++j) {
                if (j < 0)
                    d[j - DLO] = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(
                        0, static_cast<int>(acc[8 + j]), 0x138 /* wave_shr:1 */, 0xf, 0xf, false));
                else if (j >= 8)
                    d[j - DLO] = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(
                        0, static_cast<int>(acc[j - 8]), 0x130 /* wave_shl:1 */, 0xf, 0xf, false));
                else
                    d[j - DLO] = acc[j];
            }
            int sum[OUTS];
#pragma unroll
            for (int k = 0; k < OUTS; ++k) {
                int sacc = 1 << 19;
#pragma unroll
                for (int p = 0; p < NXP / 2; ++p)
                    sacc = sdot2(d[(KX * k) / 2 + OFFXD - DLO + p], L.cx[p], sacc);
                sum[k] = sacc;
            }
            if (edgeL || edgeR) {
                // edge wave (uniform): values k < 4 of the left edge lane / k >= 4 of the right
                // edge lane become min(255, floor(max(+-sum, 0) / |D|)) -- quotients of the wrong
                // sign clamp to 0 like the reference's int16 -> u8 clamp (the plan guarantees
                // they fit int16) -- re-scaled by 2^20 for the pack
#pragma unroll
                for (int k = 0; k < OUTS; ++k) {
                    const bool side = k < 4 ? edgeL : edgeR;
                    if (side) {
                        const int sv = ((L.xNeg >> k) & 1) ? -sum[k] : sum[k];
                        const uint32_t n = static_cast<uint32_t>(max(sv, 0));
                        const uint32_t q = min(__umulhi(n, L.xM[k]) >> L.xT[k], 255u);
                        sum[k] = (k < 4 ? laneL : laneR) ? static_cast<int>(q << 20) : sum[k];
                    }
                }
            }
            u32x2 o;
            o.x = pack_hi(pack_lo(sum[0], sum[1]), sum[2], sum[3]);
            o.y = pack_hi(pack_lo(sum[4], sum[5]), sum[6], sum[7]);
            __builtin_amdgcn_raw_buffer_store_b64(o, dstR, stoff, (yy - a.io.dstRow0) * dstSt, 0);
        });
    }
}
template <int KY, int KX, int NY, int NXP, int OFFXD, int PD>
__global__ __launch_bounds__(256, 3) void lanczos_stream_kernel(LanczosArgs a)
{
    lanczos_stream_kernel_body<KY, KX, NY, NXP, OFFXD, PD>(a, blockIdx.x, blockIdx.y);
}


// ================================================================ symmetric Lanczos streamer
//
// Same wave geometry and border semantics as the ring streamer above, but the arithmetic and the
// memory pipeline are laid out for gfx950's issue rates (scripts/ubench/isa_rate*.hip on MI355X):
// VOP2 adds and logic ops issue in 2 cycles per wave, while v_pk_mad_u16, v_dot2*, v_perm and DPP
// moves take 4, so the kernel is VALU-bound unless the packed MACs are halved.
//
//  * Vertical: the 2:1 Lanczos Y table is symmetric (c_i == c_{NY-1-i}), so the work value is
//    sum_{p < NY/2} c_p * (s[top+p] + s[top+NY-1-p]).  The pair sums of unpacked u16 bytes are
//    <= 510 per half, so one full-rate v_add_u32 adds both halves; then one v_pk_mad_u16 per pair
//    (its low 16 bits per half ARE the reference's int16 wrap: the sum is taken mod 2^16 in any
//    order).  NY/2 adds + NY/2 packed MACs per column pair instead of NY packed MACs.  This needs
//    all NY source rows of an output row at once: a register WINDOW of NY unpacked rows (8 u16
//    pairs per lane each), refilled with two rows per output row.
//  * Horizontal: bytes are unpacked into ODD-aligned pairs Q_j = (cb+2j-1, cb+2j) (the lane's
//    own pairs j = 1..8; byte cb+16 comes from the right neighbour by DPP).  The taps of output
//    x start at the odd column 2x + offXO, so each output is exactly NX/2 v_dot2_i32_i16 on
//    Q_{k+p+JLO} with no zero padding.  The first dot takes the rounding bias from a VGPR (VOP3P
//    form) and DPP moves use bound_ctrl, so neither needs an initialising move.
//  * Memory: each wave streams its rows through a private LDS ring of K slots (2 rows of 1 KiB
//    each) filled by LDS-DMA (buffer_load_dwordx4 ... lds), K-1 output rows ahead of use.  The
//    prefetch costs no VGPRs, so it can be deeper than a register ring, and the slot index is a
//    runtime value, so the unroll is only NY/2 (the window period).  The DMA is issued from
//    inline asm with explicit vmcnt accounting (the compiler would drain vmcnt(0) before every
//    LDS read of a DMA target): in program order every iteration issues 2 DMAs and 1 store, the
//    prologue issues K-1 dropped stores so that the pattern holds from the first iteration, and
//    iteration i waits with vmcnt(3K-5), which retires exactly DMA(i).
//  * Edge waves (holding the <= 4 border columns per side) run their own copy of the loop, so
//    the border-column divisions cost nothing in the other waves.
//  * A wave has np producing lanes (1..np) and halo lanes 0 and np+1; the host sizes np so the
//    waves of a row tile the output width exactly when it can (1920 = 4 x 60 x 8).  Idle lanes
//    (> np+1) load nothing (out-of-range offsets) and store nothing.  Rows past the band's last
//    needed source row are loaded out of range too (no HBM traffic).

// 16-byte-per-lane LDS-DMA of one source row into LDS bytes [lds, lds + 1024) of this wave, with
// the default cache policy (fresh data, C2: 2.7 % faster than nontemporal -- the halo rows that
// neighbouring bands share stay in L2).  M0 is saved and restored inside the statement (it is
// compiler-reserved).
__device__ __forceinline__ void dma_row(uint32_t lds, int voff, __amdgpu_buffer_rsrc_t rsrc, int soff)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "s"(lds), "v"(voff), "s"(rsrc), "s"(soff)
                 : "memory");
}

// dma_row for the lanes of `mask` only (masked-off lanes write nothing to LDS): the last chunk of a
// ring row DMAs just the bytes the row needs, so the ring rows can be packed tighter than 1 KiB
__device__ __forceinline__ void dma_row_masked(uint32_t lds, int voff, __amdgpu_buffer_rsrc_t rsrc, int soff,
                                               uint64_t mask)
{
    uint32_t keep;
    uint64_t save;
    asm volatile("s_mov_b64 %1, exec\n\ts_mov_b64 exec, %6\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %3, %4, %5 offen lds\n\ts_mov_b32 m0, %0\n\ts_mov_b64 exec, %1"
                 : "=&s"(keep), "=&s"(save)
                 : "s"(lds), "v"(voff), "s"(rsrc), "s"(soff), "s"(mask)
                 : "memory");
}

#ifndef IQO_SYMB_EDGE_BATCH
#define IQO_SYMB_EDGE_BATCH 16  // rows of border-column sums parked before a flush (narrow-row scheme; C2 before the line scheme: 64 -> 16 cut write traffic +4.5% -> +2%)
#endif
#ifndef IQO_SYMB_NT
#define IQO_SYMB_NT 2  // block-shared streamer cache policy: nontemporal DMA loads (1) / stores (2); stores
                       // by default (C2 x256: 0.549 -> 0.544 ms at 24 bands, 0.531 -> 0.520 at 96; nontemporal
                       // loads lose the halo rows neighbouring bands share in L2: 0.560)
#endif
// The block-shared streamer's border-column scheme: whole 128-byte pieces parked and stored once per
// trip (rows of >= 256 outputs with >= 16 producing lanes per wave), else the divided bytes stored
// over the row (narrow rows)
inline __host__ __device__ bool symb_line(int dstW, int np) { return dstW >= 256 && np >= 16; }
// LDS bytes of the block-shared streamer's edge area (after the ring): the line scheme's parked
// pieces and sums of one trip of NY/2 rows, or the narrow-row scheme's sums
// (NX > 16, Lanczos-5: 8 border sums per row and side)
constexpr int symb_edge_bytes(int NY, int NX)
{
    return 2 * (NY / 2) * (128 + (NX > 16 ? 32 : 16)) > 2 * IQO_SYMB_EDGE_BATCH * 16
               ? 2 * (NY / 2) * (128 + (NX > 16 ? 32 : 16))
               : 2 * IQO_SYMB_EDGE_BATCH * 16;
}
// cache policy of dma_row_nt (variant builds, IQO_SYMB_LDPOL): 0 nt, 1 sc0, 2 sc1, 3 sc0 sc1, 4 sc1 nt
#ifndef IQO_SYMB_LDPOL
#define IQO_SYMB_LDPOL 0
#endif
#if IQO_SYMB_LDPOL == 1
#define IQO_SYMB_LDPOL_S "sc0"
#elif IQO_SYMB_LDPOL == 2
#define IQO_SYMB_LDPOL_S "sc1"
#elif IQO_SYMB_LDPOL == 3
#define IQO_SYMB_LDPOL_S "sc0 sc1"
#elif IQO_SYMB_LDPOL == 4
#define IQO_SYMB_LDPOL_S "sc1 nt"
#else
#define IQO_SYMB_LDPOL_S "nt"
#endif
__device__ __forceinline__ void dma_row_nt(uint32_t lds, int voff, __amdgpu_buffer_rsrc_t rsrc, int soff)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %3, %4 offen " IQO_SYMB_LDPOL_S " lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "s"(lds), "v"(voff), "s"(rsrc), "s"(soff)
                 : "memory");
}

// X coefficient pair p of the symmetric streamers (pairs 8, 9 of Lanczos-5 live in cy[8], cy[9]:
// kernels.hpp LanczosDev)
__device__ __forceinline__ uint32_t cxo_at(const LanczosDev &L, int p) { return p < 8 ? L.cxo[p] : L.cy[p]; }


template <int NY, int NX, int OFFX, int K, bool C0ONE>
__device__ __forceinline__ void lanczos_sym_kernel_body(const LanczosArgs &a, const unsigned bx, const unsigned by)
{
    constexpr int H = NY / 2;                   // symmetric pairs = iterations per window cycle
    static_assert(NY % 2 == 0 && NX % 2 == 0 && (OFFX & 1), "even taps, odd first X column");
    static_assert(K >= 2 && 3 * K - 5 >= 0, "ring depth");
    constexpr int JLO = (OFFX + 1) / 2;         // output k, pair p reads Q_{k + p + JLO}
    constexpr int JHI = 7 + NX / 2 + JLO;       // one past the last pair index read
    static_assert(JLO >= -7 && JHI <= 17, "horizontal taps must stay within the neighbouring lanes");
    constexpr int SLOT = 2048;                  // bytes per ring slot (2 rows x 64 lanes x 16 B)
    __shared__ __attribute__((aligned(16))) uint8_t ring[4 * K * SLOT];
    __shared__ int4 edgeSum[4][2][64];          // per wave: parked border-column sums, 64 rows

    const LanczosDev &L = a.l;
    const int lane = static_cast<int>(threadIdx.x) & 63;
    const int wib = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    const int g = static_cast<int>(bx) * 4 + wib;
    if (g >= a.bands * a.wavesPerRow)
        return;
    const int band = g / a.wavesPerRow, wcol = g - band * a.wavesPerRow;
    const int y0 = a.rowBegin + band * a.rowsPerBand;
    const int y1 = min(y0 + a.rowsPerBand, a.rowEnd);
    if (y0 >= y1)
        return;

    const int np = a.np, opw = 8 * np;
    const int x0 = max(0, min(wcol * opw, L.dstW - opw));
    const int cb = 2 * x0 - 16 + 16 * lane;
    const int outX = x0 + (lane - 1) * 8;
    const bool produce = lane >= 1 && lane <= np && outX < L.dstW;
    const int voff = (lane <= np + 1 && cb >= 0 && cb < L.srcW) ? cb : 0x7ff00000;
    const bool edgeL = x0 == 0 && !(IQO_DBG(a) & 4), edgeR = x0 + opw >= L.dstW && !(IQO_DBG(a) & 4);
    const bool laneL = outX == 0, laneR = outX == L.dstW - 8;

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(by) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(by) * a.io.dstFrameSt;
    const __amdgpu_buffer_rsrc_t srcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcFrame), 0, a.srcBytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0;
    const int dbg = IQO_DBG(a);
    const int svoff = (dbg & 2) ? 0x7ff00000 : voff;
    const int stoff = (produce && !(dbg & 1)) ? outX : 0x7ff00000;
    // Odd bands walk bottom-up: a band boundary's halo rows are then read by both bands at the
    // same time (both at their start or both at their end) and the second read hits the
    // Infinity Cache instead of HBM.  The window arithmetic is symmetric, so only the row order
    // changes: walk index t of iteration i is source row rowAt(i, t).
    const int dir = ((band & 1) && !(dbg & 32)) ? -1 : 1;
    const int rFirst = 2 * y0 + L.offY;                 // first source row the band reads
    const int rLast = 2 * (y1 - 1) + L.offY + NY - 1;  // last source row the band reads
    const int nRows = y1 - y0;
    const uint32_t bias = opaque(1u << 19);            // rounding bias (VOP3P src2 of the first dot)

    // LDS ring of this wave: iteration i's two rows live in slot i mod K
    const uint32_t ldsWave = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
                                 (__attribute__((address_space(3))) uint8_t *)ring)) +
                             static_cast<uint32_t>(wib * K * SLOT);
    const uint8_t *ringLane = ring + wib * K * SLOT + lane * 16;
    auto row_soff = [&](int r) { return (r >= rFirst && r <= rLast) ? (r - srcRow0) * srcSt : 0x7ff00000; };
    // iteration i (output row y0 + i, or y1 - 1 - i walking up) brings walk rows NY-2 and NY-1
    auto rowAt = [&](int i, int t) { return dir > 0 ? rFirst + 2 * i + t : rLast - 2 * i - t; };
    auto dma_iter = [&](int i) {
        const uint32_t s = ldsWave + static_cast<uint32_t>((i % K) * SLOT);
        const int r = rowAt(i, NY - 2);
        dma_row(s, svoff, srcR, row_soff(r));
        dma_row(s + 1024, svoff, srcR, row_soff(r + dir));
    };
    auto read_iter = [&](int i, uint4 &r0, uint4 &r1) {
        const uint8_t *p = ringLane + (i % K) * SLOT;
        r0 = *reinterpret_cast<const uint4 *>(p);
        r1 = *reinterpret_cast<const uint4 *>(p + 1024);
    };

    // odd-aligned u16 pairs Q_1..Q_8 of one row: (b1,b2) (b3,b4) ... (b15,b16), b16 = right
    // neighbour's byte 0
    auto unpack_odd = [&](uint4 v, uint32_t (&q)[8]) {
        const uint32_t r = static_cast<uint32_t>(
            __builtin_amdgcn_mov_dpp(static_cast<int>(v.x), 0x130 /* wave_shl:1 */, 0xf, 0xf, true));
        q[0] = __builtin_amdgcn_perm(0u, v.x, 0x0c020c01u);
        q[1] = __builtin_amdgcn_perm(v.y, v.x, 0x0c040c03u);
        q[2] = __builtin_amdgcn_perm(0u, v.y, 0x0c020c01u);
        q[3] = __builtin_amdgcn_perm(v.z, v.y, 0x0c040c03u);
        q[4] = __builtin_amdgcn_perm(0u, v.z, 0x0c020c01u);
        q[5] = __builtin_amdgcn_perm(v.w, v.z, 0x0c040c03u);
        q[6] = __builtin_amdgcn_perm(0u, v.w, 0x0c020c01u);
        q[7] = __builtin_amdgcn_perm(r, v.w, 0x0c040c03u);
    };

    // Border columns of rows [yb, yb + n) from the parked sums: floor(max(S, 0) / D) with the
    // exact multiply-high constants of plan.cpp magic_x (identity for the interior columns of the
    // edge lane), clamped to a byte, one dword per row and side -- stored after the row's main
    // store, so it overwrites those 4 bytes.
    auto flush_edges = [&](int yb, int n) {
        auto fix = [&](int sv, int k) {
            const uint32_t qq = __umulhi(static_cast<uint32_t>(max(sv, 0)), L.xM[k]) >> L.xT[k];
            return min(qq, 255u);
        };
        const int rowOff = (yb + dir * lane - a.io.dstRow0) * dstSt;
        if (edgeL) {
            const int4 e = edgeSum[wib][0][lane & 63];
            const uint32_t w = fix(e.x, 0) | (fix(e.y, 1) << 8) | (fix(e.z, 2) << 16) | (fix(e.w, 3) << 24);
            __builtin_amdgcn_raw_buffer_store_b32(w, dstR, lane < n && !(dbg & 1) ? rowOff : 0x7ff00000, 0, 0);
        }
        if (edgeR) {
            const int4 e = edgeSum[wib][1][lane & 63];
            const uint32_t w = fix(e.x, 4) | (fix(e.y, 5) << 8) | (fix(e.z, 6) << 16) | (fix(e.w, 7) << 24);
            __builtin_amdgcn_raw_buffer_store_b32(w, dstR, lane < n && !(dbg & 1) ? rowOff + L.dstW - 4 : 0x7ff00000,
                                                  0, 0);
        }
    };

    // window: at iteration i the NY walk rows rowAt(i, t) (t < NY) live in slots (2i + t) mod NY;
    // iteration i brings the last two (t = NY-2, NY-1)
    uint32_t win[NY][8];
    {
        // walk rows 0 .. NY-3 of iteration 0 go straight to VGPRs (window slots 0 .. NY-3)
        uint4 w0[NY - 2];
#pragma unroll
        for (int t = 0; t < NY - 2; ++t) {
            u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(srcR, svoff, row_soff(rowAt(0, t)), 0);
            w0[t] = make_uint4(q.x, q.y, q.z, q.w);
        }
#pragma unroll
        for (int t = 0; t < NY - 2; ++t)
            unpack_odd(w0[t], win[t]);
    }
    // ring prologue: DMA(0) .. DMA(K-2), each followed by a dropped store, so that from the first
    // iteration on the vm counter sees the steady-state order DMA(j), S(j-K+1)
#pragma unroll
    for (int j = 0; j < K - 1; ++j) {
        dma_iter(j);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, dstR, 0x7ff00000, 0, 0);
    }

    auto row = [&](auto uc, int base) {
        constexpr int v = decltype(uc)::value;
        const int i = base + v;  // iteration = output row y0 + i
        if (i >= nRows)
            return;  // past the band end (uniform)
        const int yy = dir > 0 ? y0 + i : y1 - 1 - i;
        // DMA(i) retired: after it come 2 DMAs per later iteration (K-2 of them) and the
        // K-1 stores of iterations i-K+1 .. i-1
        wait_vmcnt<3 * K - 5>();
        uint4 n0, n1;
        read_iter(i, n0, n1);
        dma_iter(i + K - 1);  // into slot (i-1) mod K, read in iteration i-1
        unpack_odd(n0, win[(2 * v + NY - 2) % NY]);
        unpack_odd(n1, win[(2 * v + NY - 1) % NY]);

        // vertical: pair p = slots (2v + p, 2v + NY - 1 - p) mod NY
        uint32_t acc[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const uint32_t p0 = win[(2 * v) % NY][c] + win[(2 * v + NY - 1) % NY][c];
            acc[c] = C0ONE ? p0 : pk_mul(p0, L.cy[0]);
        }
#pragma unroll
        for (int p = 1; p < H; ++p)
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const uint32_t pp = win[(2 * v + p) % NY][c] + win[(2 * v + NY - 1 - p) % NY][c];
                acc[c] = pk_mad(pp, L.cy[p], acc[c]);
            }
        if ((yy < L.mainBeginY || yy >= L.mainEndY) && !(dbg & 8)) {
            // border row (uniform, rare): rows outside the image were read as zero
            const bool top = yy < L.mainBeginY;
            const int bi = top ? yy : yy - L.mainEndY;
            const uint32_t m = top ? L.yTopM[bi] : L.yBotM[bi];
            const int sh = top ? L.yTopS[bi] : L.yBotS[bi];
#pragma unroll
            for (int c = 0; c < 8; ++c)
                acc[c] = ydiv2(acc[c], m, sh);
        }

        // Q_j for j in [JLO, JHI): own pairs 1..8, neighbours' by DPP
        uint32_t q[JHI - JLO];
#pragma unroll
        for (int j = JLO; j < JHI; ++j) {
            if (j <= 0)
                q[j - JLO] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(
                    static_cast<int>(acc[j + 7]), 0x138 /* wave_shr:1 */, 0xf, 0xf, true));
            else if (j >= 9)
                q[j - JLO] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(
                    static_cast<int>(acc[j - 9]), 0x130 /* wave_shl:1 */, 0xf, 0xf, true));
            else
                q[j - JLO] = acc[j - 1];
        }
        int sum[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            int sacc;  // VOP3P form: the bias VGPR is src2, no copy into the accumulator
            asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(sacc) : "s"(L.cxo[0]), "v"(q[k]), "v"(bias));
#pragma unroll
            for (int p = 1; p < NX / 2; ++p)
                sacc = sdot2(q[k + p], L.cxo[p], sacc);
            sum[k] = sacc;
        }
        u32x2 o;
        o.x = pack_hi(pack_lo(sum[0], sum[1]), sum[2], sum[3]);
        o.y = pack_hi(pack_lo(sum[4], sum[5]), sum[6], sum[7]);
        __builtin_amdgcn_raw_buffer_store_b64(o, dstR, stoff, (yy - a.io.dstRow0) * dstSt, 0);
        if (edgeL || edgeR) {
            // border columns: the edge lane parks its 4 raw sums (k < 4 left, k >= 4 right) in
            // LDS; every 64 rows and at the band end one pass divides them, one row per lane
            const int slot = i & 63;
            if (edgeL && laneL)
                edgeSum[wib][0][slot] = make_int4(sum[0], sum[1], sum[2], sum[3]);
            if (edgeR && laneR)
                edgeSum[wib][1][slot] = make_int4(sum[4], sum[5], sum[6], sum[7]);
            if (slot == 63 || i == nRows - 1) {
                __builtin_amdgcn_wave_barrier();
                flush_edges(yy - dir * slot, slot + 1);  // after this row's main store (same addresses)
            }
        }
    };
    for (int base = 0; base < nRows; base += H)
        static_for<H>([&](auto uc) { row(uc, base); });

    wait_vmcnt<0>();  // no LDS-DMA may still be writing when the wave (and its LDS) retires
}
template <int NY, int NX, int OFFX, int K, bool C0ONE>
__global__ __launch_bounds__(256, 4) void lanczos_sym_kernel(LanczosArgs a)
{
    lanczos_sym_kernel_body<NY, NX, OFFX, K, C0ONE>(a, blockIdx.x, blockIdx.y);
}


// ================================================================ block-shared symmetric streamer
//
// lanczos_sym_kernel with the source rows shared by the waves of a row band: one WORKGROUP = one
// row band of one frame, wave w = column strip w.  The per-wave rings above fetch every strip's
// 16-B halo lanes from HBM a second time -- 992-B strips that start off a 128-B line touch 8-9
// lines each, +13 % read traffic on C2 (FETCH_SIZE).  Here each row lands ONCE in a shared LDS
// ring slot, in non-overlapping 1-KiB LDS-DMA chunks (chunk c by wave c mod wpr), and every lane
// reads its 16 bytes, halo included, from LDS.  Columns right of the image are zero in LDS (the
// out-of-range lanes of a chunk DMA zeros), and a 16-B zero pad sits left of every ring row.  One
// s_barrier per output row publishes the row's slot and retires the slot read in the previous
// row before it is refilled.  Waves with fewer chunks than CPW DMA into a sink so the vm-counter
// pattern is the same in every wave.

#ifndef IQO_SYMB_EXP
#define IQO_SYMB_EXP 0  // timing experiments in variant builds (wrong output): 1 no vertical MACs,
                        // 2 half the horizontal dots, 3 / 4 dot2 / dot4 in place of the MACs
#endif
template <int NY, int NX, int OFFX, int K, int CPW, bool C0ONE, bool LINE>
__device__ __forceinline__ void lanczos_symb_kernel_body(const LanczosArgs &a, const unsigned bx, const unsigned by,
                                                         const int rpb)
{
    constexpr int H = NY / 2;                   // symmetric pairs = iterations per window cycle
    static_assert(NY % 2 == 0 && NX % 2 == 0 && (OFFX & 1), "even taps, odd first X column");
    static_assert(K >= 3 && CPW >= 1, "ring depth (the LDS look-ahead needs K >= 3)");
    // LDS look-ahead: iteration i reads the ring slot of iteration i+1 (its latency hides behind
    // iteration i's arithmetic), so it waits for DMA(i+1): after this wave's DMA(i+1) come the
    // store of iteration i-K+2 and the 2*CPW DMAs + 1 store of each of iterations i+2 .. i+K-2
    constexpr int WAIT = 1 + (K - 2) * (2 * CPW + 1);   // prologue: DMA(0) retired
    constexpr int WAITLA = 1 + (K - 3) * (2 * CPW + 1); // iteration i: DMA(i+1) retired
    // K == H: the ring period equals the window period, so every slot index in the unrolled body
    // is a compile-time constant (immediate LDS offsets, no per-row slot arithmetic)
    constexpr bool CSLOT = K == H;
    constexpr int JLO = (OFFX + 1) / 2;         // output k, pair p reads Q_{k + p + JLO}
    constexpr int JHI = 7 + NX / 2 + JLO;       // one past the last pair index read
    static_assert(JLO >= -7 && JHI <= 17, "horizontal taps must stay within the neighbouring lanes");
    // LDS: ring [K slots][2 rows][rowPitch] | edge area (symb_edge_bytes) | 1 KiB DMA sink (only
    // when some wave has fewer chunks than CPW).  Edge area: line scheme [2][H][128] parked bytes +
    // int4 [2][H] border sums; narrow rows int4 edgeSum [2][EDGE_BATCH]
    constexpr int EB = IQO_SYMB_EDGE_BATCH;
    static_assert((EB & (EB - 1)) == 0 && EB <= 64, "edge batch: power of two <= 64");
    static_assert(H <= 8, "line-scheme flush: 4 rows per 8-B store, two stores");
    // Lanczos-5 (20 X taps): 5 border columns per side, so the edge lane parks all 8 of its sums
    // and the flush divides 8 bytes per side (L.xM8: identity for the interior ones)
    constexpr bool E8 = NX > 16;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int rowPitch = a.rowPitch, slotBytes = 2 * rowPitch;
    uint8_t *const ring = lds;
    int4 (*const edgeSum)[EB] = reinterpret_cast<int4 (*)[EB]>(lds + K * slotBytes);
    uint8_t *const lineBuf = lds + K * slotBytes;                                      // [2][H][128]
    int4 *const lineSum = reinterpret_cast<int4 *>(lds + K * slotBytes + 2 * H * 128); // [2][H] (E8: [2][H][2])
    const uint32_t sinkLds = static_cast<uint32_t>(K * slotBytes + symb_edge_bytes(NY, NX));
    // the last chunk of a row DMAs only its first lastLanes lanes (the row's pitch ends there)
    const int lastLanes = a.lastLanes > 0 && a.lastLanes < 64 ? a.lastLanes : 64;
    const uint64_t lastMask = lastLanes == 64 ? ~0ull : (1ull << lastLanes) - 1ull;

    const LanczosDev &L = a.l;
    const int lane = static_cast<int>(threadIdx.x) & 63;
    const int wib = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    const int wpr = a.wavesPerRow;                 // = waves of this workgroup
    const int band = static_cast<int>(bx), wcol = wib;
    const int y0 = a.rowBegin + band * rpb;  // rpb: rows per band of this workgroup's band size
    const int y1 = min(y0 + rpb, a.rowEnd);
    if (y0 >= y1)
        return;  // whole workgroup

    const int np = a.np, opw = 8 * np;
    const int x0 = max(0, min(wcol * opw, L.dstW - opw));
    const int cb = 2 * x0 - 16 + 16 * lane;
    const int outX = x0 + (lane - 1) * 8;
    const bool produce = lane >= 1 && lane <= np && outX < L.dstW;
    const int voff = (lane <= np + 1 && cb >= 0 && cb < L.srcW) ? cb : 0x7ff00000;  // prologue loads
    const int ldsCol = lane <= np + 1 ? 16 + cb : 0;  // this lane's 16 bytes in an LDS ring row
    const bool edgeL = x0 == 0 && !(IQO_DBG(a) & 4), edgeR = x0 + opw >= L.dstW && !(IQO_DBG(a) & 4);
    const bool laneL = outX == 0, laneR = outX == L.dstW - 8;
    // Border columns, line scheme (rows of >= 256 outputs, >= 16 producing lanes): the lanes holding
    // the row's first and last 128 output bytes (the edge lanes among them) do not store; they park
    // their 8 bytes per row in LDS, the edge lane also its 4 raw border sums, and once per trip of H
    // rows one pass divides the sums into the parked bytes and stores the two 128-byte pieces of
    // every row whole.  Every output byte is then written once, and a row starting on a 128-B line
    // (the C2 layout) is written in whole lines: storing the 4 divided bytes over an already written
    // line (the narrow-row scheme below) cost C2 2.4 % in partial-line writes, and its per-row
    // parking and flush 7 % of the compute-only time.
    // (LINE: chosen by the host, symb_line(): dstW >= 256 and >= 16 producing lanes)
    const bool regL = LINE && edgeL && produce && outX < 128;
    const bool regR = LINE && edgeR && produce && outX >= L.dstW - 128;
    // the lane's parking byte offset in lineBuf (slot 0; slot v adds 128 v), -1: does not park
    const int parkOff = regL ? outX : regR ? H * 128 + outX - (L.dstW - 128) : -1;

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(by) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(by) * a.io.dstFrameSt;
    const __amdgpu_buffer_rsrc_t srcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcFrame), 0, a.srcBytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0;
    const int dbg = IQO_DBG(a);
    const int svoff = (dbg & 2) ? 0x7ff00000 : voff;
    const int stoff = (produce && !(dbg & 1) && !regL && !regR) ? outX : 0x7ff00000;
#ifdef IQO_SYMB_STAUX
    constexpr int STNT = IQO_SYMB_STAUX;  // variant builds: store cache policy bits (1 sc0, 2 nt, 16 sc1)
#else
    constexpr int STNT = (IQO_SYMB_NT & 2) ? 2 : 0;  // store cache policy (aux: nt)
#endif
    // Odd bands walk bottom-up: a band boundary's halo rows are then read by both bands at the
    // same time (both at their start or both at their end) and the second read hits the
    // Infinity Cache instead of HBM.  The window arithmetic is symmetric, so only the row order
    // changes: walk index t of iteration i is source row rowAt(i, t).
    const int dir = ((band & 1) && !(dbg & 32)) ? -1 : 1;
    const int rFirst = 2 * y0 + L.offY;                 // first source row the band reads
    const int rLast = 2 * (y1 - 1) + L.offY + NY - 1;  // last source row the band reads
    const int nRows = y1 - y0;
    const uint32_t bias = opaque(1u << 19);            // rounding bias (VOP3P src2 of the first dot)
    uint32_t cvx[NX / 2];  // X coefficient pairs in VGPRs (the VOP2 DPP dot needs a VGPR src1)
#pragma unroll
    for (int p = 0; p < NX / 2; ++p)
        cvx[p] = opaque(cxo_at(L, p));

    // shared LDS ring: iteration i's two walk rows live in slot i mod K; chunk c (1 KiB of
    // source columns [1024c, 1024c + 1024) at LDS column 16 + 1024c) is DMA'd by wave c mod wpr
    const uint32_t ldsBase = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
        (__attribute__((address_space(3))) uint8_t *)lds));
    const uint8_t *ringLane = ring + ldsCol;
    auto row_soff = [&](int r) { return (r >= rFirst && r <= rLast) ? (r - srcRow0) * srcSt : 0x7ff00000; };
    // iteration i (output row y0 + i, or y1 - 1 - i walking up) brings walk rows NY-2 and NY-1
    auto rowAt = [&](int i, int t) { return dir > 0 ? rFirst + 2 * i + t : rLast - 2 * i - t; };
    // the DMA rows of iteration j are linear in j and inside [rFirst, rLast] exactly when j < nRows
    // (the last iteration brings the band's last two rows), so their offsets are one running
    // value instead of two range checks per row
    const int dmaSoff0 = (rowAt(0, NY - 2) - srcRow0) * srcSt, dmaStep = 2 * dir * srcSt, dmaNext = dir * srcSt;
    auto dma_iter = [&](int j, int slot) {
        const uint32_t s = ldsBase + static_cast<uint32_t>(slot * slotBytes);
        const bool in = j < nRows;
        const int so0 = in ? dmaSoff0 + j * dmaStep : 0x7ff00000;
        const int so1 = in ? dmaSoff0 + j * dmaStep + dmaNext : 0x7ff00000;
#pragma unroll
        for (int jj = 0; jj < CPW; ++jj) {
            const int c = wcol + jj * wpr;
            const bool real = c < a.chunks;  // uniform; otherwise a same-count DMA into the sink
            const int col = 1024 * c + 16 * lane;
            const int v = (real && col < L.srcW && !(dbg & 2)) ? col : 0x7ff00000;
            const uint32_t d0 = real ? s + 16 + 1024 * c : ldsBase + sinkLds;
            const uint32_t d1 = real ? d0 + rowPitch : d0;
            if (real && c == a.chunks - 1 && lastLanes < 64) {  // uniform
                dma_row_masked(d0, v, srcR, so0, lastMask);
                dma_row_masked(d1, v, srcR, so1, lastMask);
            } else if (IQO_SYMB_NT & 1) {
                dma_row_nt(d0, v, srcR, so0);
                dma_row_nt(d1, v, srcR, so1);
            } else {
                dma_row(d0, v, srcR, so0);
                dma_row(d1, v, srcR, so1);
            }
        }
    };
    auto read_iter = [&](int slot, uint4 &r0, uint4 &r1) {
        const uint8_t *p = ringLane + slot * slotBytes;
        r0 = *reinterpret_cast<const uint4 *>(p);
        r1 = *reinterpret_cast<const uint4 *>(p + rowPitch);
    };

    // odd-aligned u16 pairs Q_1..Q_8 of one row: (b1,b2) (b3,b4) ... (b15,b16), b16 = right
    // neighbour's byte 0
    auto unpack_odd = [&](uint4 v, uint32_t (&q)[8]) {
        const uint32_t r = static_cast<uint32_t>(
            __builtin_amdgcn_mov_dpp(static_cast<int>(v.x), 0x130 /* wave_shl:1 */, 0xf, 0xf, true));
        q[0] = __builtin_amdgcn_perm(0u, v.x, 0x0c020c01u);
        q[1] = __builtin_amdgcn_perm(v.y, v.x, 0x0c040c03u);
        q[2] = __builtin_amdgcn_perm(0u, v.y, 0x0c020c01u);
        q[3] = __builtin_amdgcn_perm(v.z, v.y, 0x0c040c03u);
        q[4] = __builtin_amdgcn_perm(0u, v.z, 0x0c020c01u);
        q[5] = __builtin_amdgcn_perm(v.w, v.z, 0x0c040c03u);
        q[6] = __builtin_amdgcn_perm(0u, v.w, 0x0c020c01u);
        q[7] = __builtin_amdgcn_perm(r, v.w, 0x0c040c03u);
    };

    // Border columns of rows [yb, yb + n) from the parked sums: floor(max(S, 0) / D) with the
    // exact multiply-high constants of plan.cpp magic_x (identity for the interior columns of the
    // edge lane), clamped to a byte, one dword per row and side -- stored after the row's main
    // store, so it overwrites those 4 bytes.
    auto flush_edges = [&](int yb, int n) {
        auto fix = [&](int sv, int k) {
            const uint32_t qq = __umulhi(static_cast<uint32_t>(max(sv, 0)), L.xM[k]) >> L.xT[k];
            return min(qq, 255u);
        };
        const int rowOff = (yb + dir * lane - a.io.dstRow0) * dstSt;
        if (edgeL) {
            const int4 e = edgeSum[0][lane & (EB - 1)];
            const uint32_t w = fix(e.x, 0) | (fix(e.y, 1) << 8) | (fix(e.z, 2) << 16) | (fix(e.w, 3) << 24);
            __builtin_amdgcn_raw_buffer_store_b32(w, dstR, lane < n && !(dbg & 65) ? rowOff : 0x7ff00000, 0, 0);
        }
        if (edgeR) {
            const int4 e = edgeSum[1][lane & (EB - 1)];
            const uint32_t w = fix(e.x, 4) | (fix(e.y, 5) << 8) | (fix(e.z, 6) << 16) | (fix(e.w, 7) << 24);
            __builtin_amdgcn_raw_buffer_store_b32(w, dstR, lane < n && !(dbg & 65) ? rowOff + L.dstW - 4 : 0x7ff00000,
                                                  0, 0);
        }
    };

    // Line scheme flush of the trip's first n rows (rows yb + dir r): lanes r < n divide row r's
    // parked border sums into the first (left) / last (right) 4 parked bytes, then 16 lanes per row
    // store the 128-byte pieces, 4 rows per instruction.  LDS accesses of one wave complete in order.
    auto flush_lines = [&](int yb, int n) {
        auto fix = [&](int sv, int k) {
            const uint32_t qq = __umulhi(static_cast<uint32_t>(max(sv, 0)), L.xM[k]) >> L.xT[k];
            return min(qq, 255u);
        };
        // the lane index through an opaque register: the per-lane addresses below are recomputed
        // here instead of being hoisted out of the row loop, where they would stay live beside the
        // row window (spills)
        const int lane = static_cast<int>(opaque(static_cast<uint32_t>(threadIdx.x) & 63u));
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            if (!(side ? edgeR : edgeL))
                continue;  // uniform
            if (lane < n) {
                if constexpr (E8) {
                    auto fix8 = [&](int sv, int k) {
                        // (Lanczos-5's 16 edge constants: kernels.hpp LanczosDev)
                        const uint32_t sh8 = k < 8 ? L.xM[k] : static_cast<uint32_t>(L.xT[k - 8]);
                        const uint32_t qq = __umulhi(static_cast<uint32_t>(max(sv, 0)), L.cx[k]) >> sh8;
                        return min(qq, 255u);
                    };
                    const int4 e0 = lineSum[2 * (side * H + lane)], e1 = lineSum[2 * (side * H + lane) + 1];
                    const int k0 = 8 * side;
                    const uint32_t w0 = fix8(e0.x, k0) | (fix8(e0.y, k0 + 1) << 8) | (fix8(e0.z, k0 + 2) << 16) |
                                        (fix8(e0.w, k0 + 3) << 24);
                    const uint32_t w1 = fix8(e1.x, k0 + 4) | (fix8(e1.y, k0 + 5) << 8) | (fix8(e1.z, k0 + 6) << 16) |
                                        (fix8(e1.w, k0 + 7) << 24);
                    *reinterpret_cast<u32x2 *>(lineBuf + (side * H + lane) * 128 + (side ? 120 : 0)) = u32x2{w0, w1};
                } else {
                    const int4 e = lineSum[side * H + lane];
                    const uint32_t w = fix(e.x, 4 * side) | (fix(e.y, 4 * side + 1) << 8) |
                                       (fix(e.z, 4 * side + 2) << 16) | (fix(e.w, 4 * side + 3) << 24);
                    *reinterpret_cast<uint32_t *>(lineBuf + (side * H + lane) * 128 + (side ? 124 : 0)) = w;
                }
            }
            const int colBase = side ? L.dstW - 128 : 0;
#pragma unroll
            for (int r0 = 0; r0 < H; r0 += 4) {
                const int r = r0 + (lane >> 4), piece = (lane & 15) * 8;
                const u32x2 val = *reinterpret_cast<const u32x2 *>(lineBuf + (side * H + min(r, H - 1)) * 128 + piece);
                const int off = r < n && !(dbg & 65) ? (yb + dir * r - a.io.dstRow0) * dstSt + colBase + piece : 0x7ff00000;
                __builtin_amdgcn_raw_buffer_store_b64(val, dstR, off, 0, STNT);
            }
        }
    };

    // window: at iteration i the NY walk rows rowAt(i, t) (t < NY) live in slots (2i + t) mod NY;
    // iteration i brings the last two (t = NY-2, NY-1)
    uint32_t win[NY][8];
    {
        // walk rows 0 .. NY-3 of iteration 0 go straight to VGPRs (window slots 0 .. NY-3); the
        // default cache policy: the neighbouring band reads the same halo rows
        uint4 w0[NY - 2];
#pragma unroll
        for (int t = 0; t < NY - 2; ++t) {
            u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(srcR, svoff, row_soff(rowAt(0, t)), 0);
            w0[t] = make_uint4(q.x, q.y, q.z, q.w);
        }
#pragma unroll
        for (int t = 0; t < NY - 2; ++t)
            unpack_odd(w0[t], win[t]);
    }
    // zero pad left of every ring row (the left halo lane of the first strip reads it)
    for (int r = static_cast<int>(threadIdx.x); r < 2 * K; r += static_cast<int>(blockDim.x))
        *reinterpret_cast<uint4 *>(ring + r * rowPitch) = make_uint4(0u, 0u, 0u, 0u);
    // ring prologue: DMA(0) .. DMA(K-2), each followed by a dropped store, so that from the first
    // iteration on the vm counter sees the steady-state order DMA(j), S(j-K+1)
#pragma unroll
    for (int j = 0; j < K - 1; ++j) {
        dma_iter(j, j);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, dstR, 0x7ff00000, 0, 0);
    }

    uint4 n0, n1;  // this iteration's two new rows (read from LDS one iteration ahead)
    wait_vmcnt<WAIT>();
    // the zero pads above are ds_writes that other waves' left halo lanes read: publish them
    // explicitly (as every LDS-publishing barrier since round 5's race fix)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read_iter(0, n0, n1);
    auto row = [&](auto uc, int base) {
        constexpr int v = decltype(uc)::value;
        const int i = base + v;  // iteration = output row y0 + i
        if (i >= nRows)
            return;  // past the band end (uniform)
        const int yy = dir > 0 ? y0 + i : y1 - 1 - i;
        // this wave's DMA(i+1) retired (WAITLA younger vm ops); the barrier publishes slot i+1
        // and retires every wave's reads of slot i-1, which DMA(i+K-1) refills
        wait_vmcnt<WAITLA>();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        uint4 m0, m1;
        read_iter(CSLOT ? (v + 1) % K : (i + 1) % K, m0, m1);
        dma_iter(i + K - 1, CSLOT ? (v + K - 1) % K : (i + K - 1) % K);
        unpack_odd(n0, win[(2 * v + NY - 2) % NY]);
        unpack_odd(n1, win[(2 * v + NY - 1) % NY]);
        n0 = m0;
        n1 = m1;

        // vertical: pair p = slots (2v + p, 2v + NY - 1 - p) mod NY
        uint32_t acc[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const uint32_t p0 = win[(2 * v) % NY][c] + win[(2 * v + NY - 1) % NY][c];
            acc[c] = C0ONE ? p0 : pk_mul(p0, L.cy[0]);
        }
#if IQO_SYMB_EXP == 1  // timing experiment (variant build, wrong output): pair sums only, no MACs
#pragma unroll
        for (int p = 1; p < H; ++p)
#pragma unroll
            for (int c = 0; c < 8; ++c)
                acc[c] += win[(2 * v + p) % NY][c];
#elif IQO_SYMB_EXP == 3  // timing experiment: v_dot2c in place of v_pk_mad_u16
#pragma unroll
        for (int p = 1; p < H; ++p)
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const uint32_t pp = win[(2 * v + p) % NY][c] + win[(2 * v + NY - 1 - p) % NY][c];
                acc[c] = static_cast<uint32_t>(sdot2(pp, L.cy[p], static_cast<int>(acc[c])));
            }
#elif IQO_SYMB_EXP == 4  // timing experiment: v_dot4 in place of v_pk_mad_u16
#pragma unroll
        for (int p = 1; p < H; ++p)
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const uint32_t pp = win[(2 * v + p) % NY][c] + win[(2 * v + NY - 1 - p) % NY][c];
                asm("v_dot4_i32_i8 %0, %1, %2, %0" : "+v"(acc[c]) : "s"(L.cy[p]), "v"(pp));
            }
#else
#pragma unroll
        for (int p = 1; p < H; ++p)
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const uint32_t pp = win[(2 * v + p) % NY][c] + win[(2 * v + NY - 1 - p) % NY][c];
                acc[c] = pk_mad(pp, L.cy[p], acc[c]);
            }
#endif
        if ((yy < L.mainBeginY || yy >= L.mainEndY) && !(dbg & 8)) {
            // border row (uniform, rare): rows outside the image were read as zero
            const bool top = yy < L.mainBeginY;
            const int bi = top ? yy : yy - L.mainEndY;
            const uint32_t m = top ? L.yTopM[bi] : L.yBotM[bi];
            const int sh = top ? L.yTopS[bi] : L.yBotS[bi];
#pragma unroll
            for (int c = 0; c < 8; ++c)
                acc[c] = ydiv2(acc[c], m, sh);
        }

        // horizontal: the neighbour pairs enter the dot products through the DPP source modifier
        // of v_dot2c_i32_i16 (no separate v_mov_dpp); each output starts with an own pair (VOP3P
        // form, the bias VGPR as src2).  s_nop 1: DPP reads of VGPRs the vertical pass just wrote.
        int sum[8];
        asm volatile("s_nop 1" ::: "memory");
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            int pFirst = -1;  // first tap whose pair is this lane's own
#pragma unroll
            for (int p = 0; p < NX / 2; ++p) {
                const int j = k + p + JLO;
                if (pFirst < 0 && j >= 1 && j <= 8)
                    pFirst = p;
            }
            int sacc;
            asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(sacc) : "s"(cxo_at(L, pFirst)), "v"(acc[k + pFirst + JLO - 1]),
                "v"(bias));
#pragma unroll
            for (int p = 0; p < NX / 2; ++p) {
                const int j = k + p + JLO;
                if (p == pFirst || (IQO_SYMB_EXP == 2 && (p & 1)))  // experiment 2: half the taps (timing only)
                    continue;
                if (j <= 0)
                    asm("v_dot2c_i32_i16_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf"
                        : "+v"(sacc) : "v"(acc[j + 7]), "v"(cvx[p]));
                else if (j >= 9)
                    asm("v_dot2c_i32_i16_dpp %0, %1, %2 wave_shl:1 row_mask:0xf bank_mask:0xf"
                        : "+v"(sacc) : "v"(acc[j - 9]), "v"(cvx[p]));
                else
                    sacc = sdot2(acc[j - 1], cxo_at(L, p), sacc);
            }
            sum[k] = sacc;
        }
        u32x2 o;
        o.x = pack_hi(pack_lo(sum[0], sum[1]), sum[2], sum[3]);
        o.y = pack_hi(pack_lo(sum[4], sum[5]), sum[6], sum[7]);
        __builtin_amdgcn_raw_buffer_store_b64(o, dstR, stoff, (yy - a.io.dstRow0) * dstSt, STNT);
        if (LINE && (edgeL || edgeR)) {
            // line scheme: slot v of the trip (its first row is iteration base, slot 0)
            if (parkOff >= 0)
                *reinterpret_cast<u32x2 *>(lineBuf + parkOff + v * 128) = o;
            if constexpr (E8) {
                if (edgeL && laneL) {
                    lineSum[2 * v] = make_int4(sum[0], sum[1], sum[2], sum[3]);
                    lineSum[2 * v + 1] = make_int4(sum[4], sum[5], sum[6], sum[7]);
                }
                if (edgeR && laneR) {
                    lineSum[2 * (H + v)] = make_int4(sum[0], sum[1], sum[2], sum[3]);
                    lineSum[2 * (H + v) + 1] = make_int4(sum[4], sum[5], sum[6], sum[7]);
                }
            } else {
                if (edgeL && laneL)  // (a wave whose x0 is not 0 can still have a lane at outX == dstW - 8)
                    lineSum[v] = make_int4(sum[0], sum[1], sum[2], sum[3]);
                if (edgeR && laneR)
                    lineSum[H + v] = make_int4(sum[4], sum[5], sum[6], sum[7]);
            }
            if (v == H - 1) {  // a band's last, partial trip is flushed after the loop
                __builtin_amdgcn_wave_barrier();
                flush_lines(yy - dir * v, H);
            }
        } else if (!LINE && (edgeL || edgeR)) {
            // border columns: the edge lane parks its 4 raw sums (k < 4 left, k >= 4 right) in
            // LDS; every EB rows and at the band end one pass divides them, one row per lane
            const int slot = i & (EB - 1);
            if (edgeL && laneL)
                edgeSum[0][slot] = make_int4(sum[0], sum[1], sum[2], sum[3]);
            if (edgeR && laneR)
                edgeSum[1][slot] = make_int4(sum[4], sum[5], sum[6], sum[7]);
            if (slot == EB - 1 || i == nRows - 1) {
                __builtin_amdgcn_wave_barrier();
                flush_edges(yy - dir * slot, slot + 1);  // after this row's main store (same addresses)
            }
        }
    };
    for (int base = 0; base < nRows; base += H)
        static_for<H>([&](auto uc) { row(uc, base); });
    if (LINE && (edgeL || edgeR) && nRows % H) {
        // the band's last trip was partial: its nRows % H rows are still parked
        const int baseLast = nRows - nRows % H;
        __builtin_amdgcn_wave_barrier();
        flush_lines(dir > 0 ? y0 + baseLast : y1 - 1 - baseLast, nRows % H);
    }

    wait_vmcnt<0>();  // no LDS-DMA may still be writing when the wave (and its LDS) retires
}
template <int NY, int NX, int OFFX, int K, int CPW, bool C0ONE, bool LINE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NY > 12 ? 2 : NY > 10 ? 3 : 4))) void lanczos_symb_kernel(LanczosArgs a)
{
    unsigned bx = blockIdx.x, by = blockIdx.y;
    int rpb = a.rowsPerBand;
    if (a.tailBands > 0) {
        // XCD tail split (speed only; blocks are dealt to the XCDs round-robin, so block L runs on
        // XCD L mod 8 and each XCD takes its blocks in order): XCD x resizes frames [x F8, (x+1) F8)
        // in order, the last one in short bands, so the workgroups that run last are short and the
        // XCD's CUs finish together; neighbouring bands of a frame share that XCD's L2 (halo rows)
        const int x = static_cast<int>(blockIdx.x & 7u), idx = static_cast<int>(blockIdx.x >> 3);
        const int F8 = a.framesPerXcd, nLong = (F8 - 1) * a.bands;
        // XCD x takes frames x, x + 8, ... (round 6): the 8 XCDs work on 8 neighbouring frames at a
        // time instead of 8 regions F8 frames apart (C2 x256 0.479 -> 0.467 ms; variant builds,
        // debug flag 128: the old contiguous ranges)
        const bool inter = !(IQO_DBG(a) & 128);  // (round 6 default: interleaved, profiles/r06/xcd_chunks.txt)
        if (idx < nLong) {
            const int q = idx / a.bands;
            by = static_cast<unsigned>(inter ? 8 * q + x : x * F8 + q);
            bx = static_cast<unsigned>(idx - q * a.bands);
        } else {
            by = static_cast<unsigned>(inter ? 8 * (F8 - 1) + x : x * F8 + F8 - 1);
            bx = static_cast<unsigned>(idx - nLong);
            rpb = a.tailRows;
            if (static_cast<int>(bx) >= a.tailBands)
                return;
        }
    } else {
        // XCD-aware order (speed only; plain dispatch order was 1 % slower, profiles/r05/steady_c2_final_opts.txt): the band workgroups of one frame go to one XCD, so the
        // halo rows two neighbouring bands share hit that XCD's L2, and each XCD streams from
        // 1/8 of the batch's address range
        const unsigned bands = gridDim.x;
        // (chunks of one frame's bands: 9 .. 45 bands or 2 frames per chunk measured the same or
        // slower, profiles/r06/xcd_chunks.txt)
        const unsigned lg = xcd_chunks(by * bands + bx, bands, bands * gridDim.y);
        by = lg / bands;
        bx = lg - by * bands;
    }
#ifdef IQO_VARIANT_DEBUG
    // workgroup timeline (variant builds): wave 0 records its start and end on the 100 MHz clock and
    // where it ran (HW_ID: wave slot / SIMD / CU / SH / SE fields; XCC_ID), one 16-byte vector store
    // (profiles/r06/wgtrace.txt)
    uint32_t t0 = 0;
    if (a.l.trace && threadIdx.x < 64)
        t0 = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
#endif
    lanczos_symb_kernel_body<NY, NX, OFFX, K, CPW, C0ONE, LINE>(a, bx, by, rpb);
#ifdef IQO_VARIANT_DEBUG
    if (a.l.trace && threadIdx.x == 0) {
        const uint32_t t1 = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
        const uint32_t hw = static_cast<uint32_t>(__builtin_amdgcn_s_getreg(4 | (31 << 11)));   // HW_REG_HW_ID
        const uint32_t xcc = static_cast<uint32_t>(__builtin_amdgcn_s_getreg(20 | (31 << 11))); // HW_REG_XCC_ID
        uint4 *rec = reinterpret_cast<uint4 *>(a.l.trace) + (blockIdx.x + gridDim.x * blockIdx.y);
        *rec = make_uint4(t0, t1, hw, xcc);
    }
#endif
}


// ================================================================ frame-stacked streamer (narrow frames)
//
// The block-shared streamer gives a row of srcW source columns srcW / 16 producing lanes; a
// 640-column frame (C1: 640x480 -> 320x240) fills 40 of a wave's 64 lanes.  Here FPW frames sit
// side by side in the lanes of one 2-wave workgroup: virtual lane v (wave w, lane l: v = 62 w + l;
// each wave's lanes 0 and 63 are its halo) holds, for v = 1 + (np + 1) F + k, frame F's source
// columns [16 k, 16 k + 16) (k < np), and the virtual lanes between frames (k = np) and at both
// ends are zero -- exactly the zero columns outside the image that give the reference's masked
// border sums, so every frame's arithmetic is the block-shared streamer's unchanged (3 frames of
// 40 lanes = 120 of the 128 lanes produce).  Each ring row holds the FPW frames' rows at LDS bytes
// 16 v, DMA'd one frame row per instruction (lanes past the row masked).  Requirements (host):
// srcW = 2 dstW, srcW % 16 == 0, np = srcW / 16, FPW (np + 1) + 1 <= 126.
template <int NY, int NX, int OFFX, int K, int CPW, bool C0ONE>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(4))) void lanczos_stack_kernel(LanczosArgs a)
{
    constexpr int H = NY / 2;
    static_assert(NY % 2 == 0 && NX % 2 == 0 && (OFFX & 1), "even taps, odd first X column");
    static_assert(K == H && CPW >= 1, "ring depth = window period");
    constexpr int WAIT = 1 + (K - 2) * (2 * CPW + 1);
    constexpr int WAITLA = 1 + (K - 3) * (2 * CPW + 1);
    constexpr int JLO = (OFFX + 1) / 2;
    constexpr int EB = 16;                      // rows of parked border-column sums per flush
    constexpr int PITCH = 2048;                 // ring row: 128 virtual lanes x 16 B
    constexpr int SLOT = 2 * PITCH;
    constexpr int OOB = 0x7ff00000;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t *const ring = lds;
    int4 *const edgeSum = reinterpret_cast<int4 *>(lds + K * SLOT);  // [F][side][EB]
    const uint32_t sinkLds = static_cast<uint32_t>(K * SLOT + 2 * CPW * 2 * EB * 16);

    const LanczosDev &L = a.l;
    const int lane = static_cast<int>(threadIdx.x) & 63;
    const int wib = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    const int band = static_cast<int>(blockIdx.x);
    const int y0 = a.rowBegin + band * a.rowsPerBand;
    const int y1 = min(y0 + a.rowsPerBand, a.rowEnd);
    if (y0 >= y1)
        return;  // whole workgroup
    const int np = a.np, fpw = a.fpw;
    const int f0 = static_cast<int>(blockIdx.y) * fpw;
    const int nF = min(fpw, a.frames - f0);     // frames of this workgroup
    const int v = 62 * wib + lane;               // virtual lane
    const int F = v >= 1 ? (v - 1) / (np + 1) : -1, k = v >= 1 ? (v - 1) - F * (np + 1) : -1;
    const bool mine = F >= 0 && F < nF && k < np;  // holds frame F's columns [16k, 16k + 16)
    const bool produce = mine && lane >= 1 && lane <= 62;
    const int Fc = mine ? F : 0;
    const int outX = 8 * k;
    const bool laneL = produce && k == 0, laneR = produce && k == np - 1;

    const int64_t sFrameSt = static_cast<int64_t>(a.io.srcFrameSt), dFrameSt = static_cast<int64_t>(a.io.dstFrameSt);
    const uint8_t *srcBase = a.io.src + static_cast<int64_t>(f0) * sFrameSt;
    uint8_t *dstBase = a.io.dst + static_cast<int64_t>(f0) * dFrameSt;
    // this lane's frame (prologue loads, stores); the DMAs address each frame separately
    const __amdgpu_buffer_rsrc_t srcL =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcBase + Fc * sFrameSt), 0, a.srcBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0;
    const int dbg = IQO_DBG(a);  // variant builds: 1 no stores, 2 no source loads (timing only)
    const int voff = mine && !(dbg & 2) ? 16 * k : OOB;
    const uint32_t ldsLane = static_cast<uint32_t>(16 * v);
    const int dir = (band & 1) ? -1 : 1;
    const int rFirst = 2 * y0 + L.offY;
    const int rLast = 2 * (y1 - 1) + L.offY + NY - 1;
    const int nRows = y1 - y0;
    const uint32_t bias = opaque(1u << 19);
    uint32_t cvx[NX / 2];
#pragma unroll
    for (int p = 0; p < NX / 2; ++p)
        cvx[p] = opaque(L.cxo[p]);

    const uint32_t ldsBase = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
        (__attribute__((address_space(3))) uint8_t *)lds));
    const uint8_t *ringLane = ring + ldsLane;
    auto row_soff = [&](int r) { return (r >= rFirst && r <= rLast) ? (r - srcRow0) * srcSt : OOB; };
    auto rowAt = [&](int i, int t) { return dir > 0 ? rFirst + 2 * i + t : rLast - 2 * i - t; };
    const int dmaSoff0 = (rowAt(0, NY - 2) - srcRow0) * srcSt, dmaStep = 2 * dir * srcSt, dmaNext = dir * srcSt;
    const uint64_t rowMask = np >= 64 ? ~0ull : (1ull << np) - 1ull;  // the lanes of one frame row
    // DMA of iteration j: frame slot c = wib + 2 jj (its rows at virtual lanes 1 + (np + 1) c ...);
    // slots past the workgroup's frames DMA into the sink so every wave's vm count is the same
    auto dma_iter = [&](int j, int slot) {
        const uint32_t s = ldsBase + static_cast<uint32_t>(slot * SLOT);
        const bool in = j < nRows;
        const int so0 = in ? dmaSoff0 + j * dmaStep : OOB;
        const int so1 = in ? dmaSoff0 + j * dmaStep + dmaNext : OOB;
#pragma unroll
        for (int jj = 0; jj < CPW; ++jj) {
            const int c = wib + 2 * jj;
            const bool real = c < nF;  // uniform
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint8_t *>(srcBase + (real ? c : 0) * sFrameSt), 0, a.srcBytes, 0x00020000);
            const int vv = real && !(dbg & 2) ? 16 * lane : OOB;
            const uint32_t d0 = real ? s + static_cast<uint32_t>(16 * (1 + (np + 1) * c)) : ldsBase + sinkLds;
            const uint32_t d1 = real ? d0 + PITCH : d0;
            dma_row_masked(d0, vv, rs, so0, rowMask);
            dma_row_masked(d1, vv, rs, so1, rowMask);
        }
    };
    auto read_iter = [&](int slot, uint4 &r0, uint4 &r1) {
        const uint8_t *p = ringLane + slot * SLOT;
        r0 = *reinterpret_cast<const uint4 *>(p);
        r1 = *reinterpret_cast<const uint4 *>(p + PITCH);
    };
    auto unpack_odd = [&](uint4 w, uint32_t (&q)[8]) {
        const uint32_t r = static_cast<uint32_t>(
            __builtin_amdgcn_mov_dpp(static_cast<int>(w.x), 0x130 /* wave_shl:1 */, 0xf, 0xf, true));
        q[0] = __builtin_amdgcn_perm(0u, w.x, 0x0c020c01u);
        q[1] = __builtin_amdgcn_perm(w.y, w.x, 0x0c040c03u);
        q[2] = __builtin_amdgcn_perm(0u, w.y, 0x0c020c01u);
        q[3] = __builtin_amdgcn_perm(w.z, w.y, 0x0c040c03u);
        q[4] = __builtin_amdgcn_perm(0u, w.z, 0x0c020c01u);
        q[5] = __builtin_amdgcn_perm(w.w, w.z, 0x0c040c03u);
        q[6] = __builtin_amdgcn_perm(0u, w.w, 0x0c020c01u);
        q[7] = __builtin_amdgcn_perm(r, w.w, 0x0c040c03u);
    };
    // border columns of rows [yb, yb + n) of the frames whose edge lanes this wave holds: lane i
    // rewrites row yb + dir i of one (frame, side) per pass
    const int vLo = 62 * wib + 1, vHi = 62 * wib + 62;  // this wave's producing virtual lanes
    auto flush_edges = [&](int yb, int n) {
        auto fix = [&](int sv, int kk) {
            const uint32_t qq = __umulhi(static_cast<uint32_t>(max(sv, 0)), L.xM[kk]) >> L.xT[kk];
            return min(qq, 255u);
        };
        const int rowOff = (yb + dir * lane - a.io.dstRow0) * dstSt;
        for (int G = 0; G < nF; ++G) {
            const int vL = 1 + (np + 1) * G, vR = vL + np - 1;
            uint8_t *dstF = dstBase + G * dFrameSt;
            const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(dstF, 0, a.dstBytes, 0x00020000);
            if (vL >= vLo && vL <= vHi) {
                const int4 e = edgeSum[(G * 2 + 0) * EB + (lane & (EB - 1))];
                const uint32_t w = fix(e.x, 0) | (fix(e.y, 1) << 8) | (fix(e.z, 2) << 16) | (fix(e.w, 3) << 24);
                __builtin_amdgcn_raw_buffer_store_b32(w, dr, lane < n && !(dbg & 1) ? rowOff : OOB, 0, 0);
            }
            if (vR >= vLo && vR <= vHi) {
                const int4 e = edgeSum[(G * 2 + 1) * EB + (lane & (EB - 1))];
                const uint32_t w = fix(e.x, 4) | (fix(e.y, 5) << 8) | (fix(e.z, 6) << 16) | (fix(e.w, 7) << 24);
                __builtin_amdgcn_raw_buffer_store_b32(w, dr, lane < n && !(dbg & 1) ? rowOff + L.dstW - 4 : OOB, 0, 0);
            }
        }
    };

    uint32_t win[NY][8];
    {
        uint4 w0[NY - 2];
#pragma unroll
        for (int t = 0; t < NY - 2; ++t) {
            u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(srcL, voff, row_soff(rowAt(0, t)), 0);
            w0[t] = make_uint4(q.x, q.y, q.z, q.w);
        }
#pragma unroll
        for (int t = 0; t < NY - 2; ++t)
            unpack_odd(w0[t], win[t]);
    }
    // zero every ring byte the DMAs never write (frame gaps, both ends) once
    for (int i = static_cast<int>(threadIdx.x); i < K * 2 * 128; i += static_cast<int>(blockDim.x)) {
        const int vv = i & 127;
        const int FF = vv >= 1 ? (vv - 1) / (np + 1) : -1, kk = vv >= 1 ? (vv - 1) - FF * (np + 1) : -1;
        if (!(FF >= 0 && FF < nF && kk < np))
            *reinterpret_cast<uint4 *>(ring + (i >> 7) * PITCH + 16 * vv) = make_uint4(0u, 0u, 0u, 0u);
    }
    const __amdgpu_buffer_rsrc_t dstL =
        __builtin_amdgcn_make_buffer_rsrc(dstBase + Fc * dFrameSt, 0, a.dstBytes, 0x00020000);
    const int stoff = produce && !(dbg & 1) ? outX : OOB;
#pragma unroll
    for (int j = 0; j < K - 1; ++j) {
        dma_iter(j, j);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, dstL, OOB, 0, 0);  // dropped: steady-state vm order
    }
    uint4 n0, n1;
    wait_vmcnt<WAIT>();
    // the zeroed gaps (LDS writes) and every wave's DMA(0) are visible after the barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read_iter(0, n0, n1);
    auto row = [&](auto uc, int base) {
        constexpr int vv = decltype(uc)::value;
        const int i = base + vv;
        if (i >= nRows)
            return;
        const int yy = dir > 0 ? y0 + i : y1 - 1 - i;
        wait_vmcnt<WAITLA>();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        uint4 m0, m1;
        read_iter((vv + 1) % K, m0, m1);
        dma_iter(i + K - 1, (vv + K - 1) % K);
        unpack_odd(n0, win[(2 * vv + NY - 2) % NY]);
        unpack_odd(n1, win[(2 * vv + NY - 1) % NY]);
        n0 = m0;
        n1 = m1;
        uint32_t acc[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const uint32_t p0 = win[(2 * vv) % NY][c] + win[(2 * vv + NY - 1) % NY][c];
            acc[c] = C0ONE ? p0 : pk_mul(p0, L.cy[0]);
        }
#pragma unroll
        for (int p = 1; p < H; ++p)
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const uint32_t pp = win[(2 * vv + p) % NY][c] + win[(2 * vv + NY - 1 - p) % NY][c];
                acc[c] = pk_mad(pp, L.cy[p], acc[c]);
            }
        if (yy < L.mainBeginY || yy >= L.mainEndY) {
            const bool top = yy < L.mainBeginY;
            const int bi = top ? yy : yy - L.mainEndY;
            const uint32_t m = top ? L.yTopM[bi] : L.yBotM[bi];
            const int sh = top ? L.yTopS[bi] : L.yBotS[bi];
#pragma unroll
            for (int c = 0; c < 8; ++c)
                acc[c] = ydiv2(acc[c], m, sh);
        }
        int sum[8];
        asm volatile("s_nop 1" ::: "memory");
#pragma unroll
        for (int kx = 0; kx < 8; ++kx) {
            int pFirst = -1;
#pragma unroll
            for (int p = 0; p < NX / 2; ++p) {
                const int j = kx + p + JLO;
                if (pFirst < 0 && j >= 1 && j <= 8)
                    pFirst = p;
            }
            int sacc;
            asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(sacc) : "s"(L.cxo[pFirst]), "v"(acc[kx + pFirst + JLO - 1]),
                "v"(bias));
#pragma unroll
            for (int p = 0; p < NX / 2; ++p) {
                const int j = kx + p + JLO;
                if (p == pFirst)
                    continue;
                if (j <= 0)
                    asm("v_dot2c_i32_i16_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf"
                        : "+v"(sacc) : "v"(acc[j + 7]), "v"(cvx[p]));
                else if (j >= 9)
                    asm("v_dot2c_i32_i16_dpp %0, %1, %2 wave_shl:1 row_mask:0xf bank_mask:0xf"
                        : "+v"(sacc) : "v"(acc[j - 9]), "v"(cvx[p]));
                else
                    sacc = sdot2(acc[j - 1], L.cxo[p], sacc);
            }
            sum[kx] = sacc;
        }
        u32x2 o;
        o.x = pack_hi(pack_lo(sum[0], sum[1]), sum[2], sum[3]);
        o.y = pack_hi(pack_lo(sum[4], sum[5]), sum[6], sum[7]);
        __builtin_amdgcn_raw_buffer_store_b64(o, dstL, stoff, (yy - a.io.dstRow0) * dstSt, 0);
        // border columns: park the edge lanes' raw sums, flush every EB rows (every wave holds an
        // edge lane of some frame, so the branch is per frame inside flush_edges)
        const int slot = i & (EB - 1);
        if (laneL)
            edgeSum[(F * 2 + 0) * EB + slot] = make_int4(sum[0], sum[1], sum[2], sum[3]);
        if (laneR)
            edgeSum[(F * 2 + 1) * EB + slot] = make_int4(sum[4], sum[5], sum[6], sum[7]);
        if (slot == EB - 1 || i == nRows - 1) {
            __builtin_amdgcn_wave_barrier();
            flush_edges(yy - dir * slot, slot + 1);
        }
    };
    for (int base = 0; base < nRows; base += H)
        static_for<H>([&](auto uc) { row(uc, base); });

    wait_vmcnt<0>();
}

// ================================================================ general-ratio wave walker
//
// The shapes of tile_kernel (multi-phase ratios, Lanczos upscaling and degrees 1-9, non-integer
// Area, Linear other than 2x) with tile_kernel's arithmetic, laid out like the streamers: every
// WAVE owns a strip of 256 output columns (4 per lane, one dword store) of one band of output
// rows of one frame and walks it top to bottom.  No barrier anywhere: a wave only ever reads the
// LDS it wrote itself, so the waves of a workgroup (and of a CU) never wait for each other.
//
// Per output row s of the band ("segment"):
//   1. widen the source rows first needed by row s, (hi(s-1), hi(s)] -- loaded two segments
//      earlier into VGPRs, one aligned dword per 4-column unit -- to u16 with two v_perm per unit
//      (per-lane selectors also replicate the edge columns) and write them to the wave's LDS
//      ring (slot = source row % R, R = the widest row window);
//   2. issue the dword loads of the rows of row s+2 into the registers just freed;
//   3. vertical pass: per tap one aligned 8-byte LDS read and two v_pk_mad_u16 per unit, tap
//      records (coefficient splat, ring byte offset) read through the scalar cache;
//   4. horizontal pass from the wave's work row: NP dword reads and NP v_dot2 per output, one
//      dword store per lane.
// The source is read once per band (plus the first row's window), the output written once.

struct WalkArgs {
    WalkDev w;
    Io io;
    int rowBegin, rowEnd, rowsPerBand, bands;
    int srcBytes, dstBytes;
    unsigned nWaves;  // strips * bands * frames
    int stripLo, strips, stripStride;  // the strips walked: stripLo + i * stripStride, i < strips
};

constexpr int kWalkD = 4;  // load look-ahead in output rows (plan.hpp kWalkPrefetch)


template <int NP, int VY, int NV, bool LZ>
__global__ __launch_bounds__(256) void walk_kernel(WalkArgs a)
{
    // VY: vertical taps, 2 * NP or 2 * NP - 2 (plan.cpp build_walk_tables)
    constexpr int OOB = 0x7ff00000;      // buffer offset past every range: no traffic, reads 0
    extern __shared__ __attribute__((aligned(16))) uint8_t wl[];
    const WalkDev &W = a.w;
    const TileDev &t = W.t;
    const int lane = static_cast<int>(threadIdx.x) & 63;
    const int wib = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    // flat wave id -> (strip, band, frame); XCD-spread by workgroup, so neighbouring strips and
    // bands (which share halo rows and columns) run on one XCD's L2
    const unsigned gw = xcd_chunks(blockIdx.x, (a.strips * a.bands + 3) / 4, gridDim.x) * 4u + static_cast<unsigned>(wib);
    if (gw >= a.nWaves)
        return;  // whole wave; the kernel has no barrier
    const int strip = a.stripLo + static_cast<int>(gw % static_cast<unsigned>(a.strips)) * a.stripStride;
    const unsigned rest = gw / static_cast<unsigned>(a.strips);
    const int band = static_cast<int>(rest % static_cast<unsigned>(a.bands));
    const int frame = static_cast<int>(rest / static_cast<unsigned>(a.bands));
    const int y0 = a.rowBegin + band * a.rowsPerBand;
    const int y1 = min(y0 + a.rowsPerBand, a.rowEnd);
    if (y0 >= y1)
        return;
    const int4 sp = sload(W.spans + strip);  // {lo8, units, interior, 0}
    const int lo8 = sp.x, units = sp.y;
    const int R = W.R, pitch = W.pitch, srcW = t.srcW;
    const int ringBytes = R * pitch;
    // LDS per wave: ring [R][pitch] | work row [512 NV] | sink [512] (NV = 2: idle lanes' writes)
    uint8_t *const ring = wl + wib * W.waveBytes;
    uint8_t *const work = ring + ringBytes;
    const int sinkOff = ringBytes + 512 * NV;

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(frame) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(frame) * a.io.dstFrameSt;
    const __amdgpu_buffer_rsrc_t srcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcFrame), 0, a.srcBytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0, srcLast = a.io.srcRowEnd - 1;
    const bool dstA4 = !(reinterpret_cast<uintptr_t>(dstFrame) & 3) && !(a.io.dstSt & 3);
    // interior strip: 256 columns, no masked border column, aligned rows: one plain dword store
    const bool interior = sp.z != 0 && dstA4;

    // horizontal ownership: output columns x0 .. x0+3, coefficient pairs in VGPRs
    const int x0 = strip * 256 + 4 * lane;
    const bool hq = x0 < t.dstW;
    const int Q = min(x0, t.dstW - 1) >> 2;
    uint32_t cf[4][NP];
    int woff[4], DL[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        woff[k] = hq ? 4 * ((t.colA[k * t.nQp + Q] - lo8) >> 1) : 0;  // byte offset in the work row
        DL[k] = (LZ && hq && x0 + k < t.dstW) ? t.cols[x0 + k].y : 0;
#pragma unroll
        for (int p = 0; p < NP; ++p)
            cf[k][p] = hq ? t.colCoef[(p * 4 + k) * t.nQp + Q] : 0u;
    }
    bool anyD = false;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        anyD |= DL[k] != 0;

    // widening ownership: units u = lane + 64 m, source columns lo8 + 4u .. +3 clamped to
    // [0, srcW): all four lie in ONE aligned dword (lo8 is a multiple of 8), byte selectors pick
    // them.  Idle lanes (u >= units) load nothing and widen into the sink.
    int gcol[NV], wOff[NV];
    uint32_t sLo[NV], sHi[NV];
#pragma unroll
    for (int m = 0; m < NV; ++m) {
        const int u = lane + 64 * m;
        const bool uv = u < units;
        const int cb = lo8 + 4 * u;
        const int g = min(max(cb, 0), srcW - 1) & ~3;
        gcol[m] = uv ? g : OOB;
        wOff[m] = uv ? 8 * u : 1 << 20;  // idle: past any slot, clamped into the sink below
        int idx[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            idx[k] = min(max(cb + k, 0), srcW - 1) - g;
        sLo[m] = static_cast<uint32_t>(idx[0] | (idx[1] << 16)) | 0x0c000c00u;
        sHi[m] = static_cast<uint32_t>(idx[2] | (idx[3] << 16)) | 0x0c000c00u;
    }
    const int laneOff = 8 * lane;
    // NV = 1: the pitch is 512 and idle lanes widen their zeros into their own slot bytes;
    // NV = 2: every m = 0 lane is busy, idle m = 1 lanes widen into the sink
    auto widen = [&](int slotOff, uint32_t v, int m) {
        const int o = m == 0 ? slotOff + laneOff : min(slotOff + wOff[m], sinkOff + laneOff);
        *reinterpret_cast<uint2 *>(ring + o) =
            make_uint2(__builtin_amdgcn_perm(0u, v, sLo[m]), __builtin_amdgcn_perm(0u, v, sHi[m]));
    };
    auto row_off = [&](int r) { return (min(r, srcLast) - srcRow0) * srcSt; };

    // the window of row y0, 8 rows per batch
    {
        const int4 w0 = sload(W.rows + y0);  // {lo, hi, hi % R, deno}
        for (int r = w0.x; r <= w0.y; r += 8) {
            uint32_t v[8][NV];
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int m = 0; m < NV; ++m)
                    v[j][m] = __builtin_amdgcn_raw_buffer_load_b32(srcR, r + j <= w0.y ? gcol[m] : OOB, row_off(r + j), 0);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (r + j <= w0.y) {
                    const int slotOff = ((r + j) % R) * pitch;
#pragma unroll
                    for (int m = 0; m < NV; ++m)
                        widen(slotOff, v[j][m], m);
                }
        }
    }

    // Segment s (plan.cpp WalkSeg) widens rows first(s) .. first(s)+NV-1 -- loaded during segment
    // s-D -- and loads rows first(s+D) .. +NV-1 into the registers it freed: NV x NV dword loads
    // per segment, no predicate.  Rows past hi(s) are written early; the ring holds the widest
    // window + NV rows, so they never overwrite a live row.
    constexpr int D = kWalkD;
    auto issue = [&](int first, uint32_t (&b)[NV][NV]) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const int soff = row_off(first + j);
#pragma unroll
            for (int m = 0; m < NV; ++m)
                b[j][m] = __builtin_amdgcn_raw_buffer_load_b32(srcR, gcol[m], soff, 0);
        }
    };
    // tap records of row y: {(c, c) splat, ring byte offset} per tap
    auto load_rec = [&](int y, uint32_t (&rc)[VY], uint32_t (&ro)[VY]) {
#pragma unroll
        for (int i = 0; i < VY; ++i) {
            rc[i] = static_cast<uint32_t>(sld(W.rowTap, 2 * (y * VY + i)));
            ro[i] = static_cast<uint32_t>(sld(W.rowTap, 2 * (y * VY + i) + 1));
        }
    };
    // s_waitcnt lgkmcnt(0) the compiler's waitcnt pass sees (so it adds no per-use waits after it)
    auto lgkm0 = [] { __builtin_amdgcn_s_waitcnt(0xc07f); };

    // Segment s: g = {first(s), ring offset of first(s), border row, first(s+D)} (loaded by the
    // previous segment)
    auto segment = [&](auto edge, int s, int4 &g, uint32_t (&b)[NV][NV]) {
        constexpr bool EDGE = decltype(edge)::value;
        const int4 gs = g;
        g = sload(W.segs + 2 * (s + 1));  // the next segment's record (the table is padded)
        uint32_t rc[VY], ro[VY];
        load_rec(s, rc, ro);
        // 1. rows first(s) .. first(s)+NV-1 into the ring
        {
            int off = gs.y;
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                if (j > 0) {
                    off += pitch;
                    off = off >= ringBytes ? off - ringBytes : off;
                }
#pragma unroll
                for (int m = 0; m < NV; ++m)
                    widen(off, b[j][m], m);
            }
        }
        // 2. the rows of segment s+D into the registers just freed
        issue(gs.w, b);
        // 3. vertical pass of row s into the work row (idle lanes compute on whatever they read)
#pragma unroll
        for (int m = 0; m < NV; ++m) {
            const uint8_t *col = ring + laneOff + 512 * m;
            // every tap's LDS read in flight, then one wait: left to itself the scheduler trades
            // this ILP for registers and serialises VY LDS round trips
            uint2 v[VY];
#pragma unroll
            for (int i = 0; i < VY; ++i)
                v[i] = *reinterpret_cast<const uint2 *>(col + ro[i]);
            lgkm0();
            __builtin_amdgcn_sched_barrier(0);
            uint32_t acc0 = 0, acc1 = 0;
#pragma unroll
            for (int i = 0; i < VY; ++i) {
                acc0 = pk_mad(v[i].x, rc[i], acc0);
                acc1 = pk_mad(v[i].y, rc[i], acc1);
            }
            if (LZ && gs.z != 0) {  // masked + renormalised border row: int16(nume * 64 / deno)
                const int4 mg = sload(W.segs + 2 * s + 1);  // {yM, yS, yNeg, 0}
                if (mg.z) {  // n / -d = -n / d
                    acc0 = pk_neg16(acc0);
                    acc1 = pk_neg16(acc1);
                }
                acc0 = ydiv2(acc0, static_cast<uint32_t>(mg.x), mg.y);
                acc1 = ydiv2(acc1, static_cast<uint32_t>(mg.x), mg.y);
            }
            *reinterpret_cast<uint2 *>(work + laneOff + 512 * m) = make_uint2(acc0, acc1);
        }
        // 4. horizontal pass of row s: every LDS read, one wait, then the dot products
        uint32_t wv[4][NP];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int p = 0; p < NP; ++p)
                wv[k][p] = *reinterpret_cast<const uint32_t *>(work + woff[k] + 4 * p);
        lgkm0();
        __builtin_amdgcn_sched_barrier(0);
        int sum[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            sum[k] = LZ ? (1 << 19) : (1 << 22);
#pragma unroll
            for (int p = 0; p < NP; ++p)
                sum[k] = LZ ? sdot2(wv[k][p], cf[k][p], sum[k])
                            : static_cast<int>(udot2(wv[k][p], cf[k][p], static_cast<uint32_t>(sum[k])));
        }
        const int off = (s - a.io.dstRow0) * dstSt + x0;
        if (LZ && !EDGE) {
            // main columns: sat_u8(sum >> 20) packed by v_ashr_pk_u8_i32
            __builtin_amdgcn_raw_buffer_store_b32(pack_hi(pack_lo(sum[0], sum[1]), sum[2], sum[3]), dstR, off, 0, 0);
            return;
        }
        uint32_t bytes[4];
        if (LZ) {
            int v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                v[k] = sum[k] >> 20;
            if (anyD) {  // masked + renormalised edge columns (rare lanes)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (DL[k] != 0)
                        v[k] = static_cast<int16_t>(exact_div(sum[k], DL[k]));
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                bytes[k] = static_cast<uint32_t>(min(max(v[k], 0), 255));
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                bytes[k] = min((static_cast<uint32_t>(sum[k]) >> 23) & 0xffffu, 255u);
        }
        const uint32_t o = opaque(bytes[0] | (bytes[1] << 8)) | (bytes[2] << 16) | (bytes[3] << 24);
        if (!EDGE) {
            __builtin_amdgcn_raw_buffer_store_b32(o, dstR, off, 0, 0);
            return;
        }
        const bool whole = hq && dstA4 && x0 + 4 <= t.dstW;
        __builtin_amdgcn_raw_buffer_store_b32(o, dstR, whole ? off : OOB, 0, 0);
        if (hq && !whole) {  // frame edge / unaligned destination: bytes
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (x0 + k < t.dstW)
                    __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(bytes[k]), dstR, off + k, 0, 0);
        }
    };

    // D register sets, one per row mod D: the loop body is straight-line, so the compiler's vmcnt
    // waits count the loads in flight exactly (the tables are padded past the end)
    auto walk = [&](auto edge) {
        uint32_t b[D][NV][NV];
#pragma unroll
        for (int d = 0; d < D; ++d)
            issue(sload(W.segs + 2 * (y0 + d)).x, b[d]);
        int4 g = sload(W.segs + 2 * y0);
        int s = y0;
        for (; s + D <= y1; s += D) {
#pragma unroll
            for (int d = 0; d < D; ++d)
                segment(edge, s + d, g, b[d]);
        }
#pragma unroll
        for (int d = 0; d < D - 1; ++d)
            if (s + d < y1)
                segment(edge, s + d, g, b[d]);
    };
    if (interior)
        walk(std::integral_constant<bool, false>());
    else
        walk(std::integral_constant<bool, true>());
}

// ================================================================ Area integer ratio
//
// Thread = 16 source columns of one output row: KY coalesced 16-B row loads, packed u16 vertical
// MACs, u16-pair dot products for the KX horizontal taps (all inside the thread's columns).

struct AreaArgs {
    AreaDev g;
    Io io;
    int rowBegin, rowEnd, groups;
};

template <int KX, int KYT>
__device__ __forceinline__ void area_int_kernel_body(const AreaArgs &a, const unsigned bx, const unsigned by)
{
    // a thread owns COLS source columns: 16 (one 16-B load per row) when KX divides 16, else 12
    // (one 12-B load; KX = 3, 6)
    constexpr int COLS = 16 % KX == 0 ? 16 : 12;
    constexpr int OUTS = COLS / KX;
    static_assert(COLS % KX == 0, "whole outputs per thread");
    const int KY = KYT ? KYT : a.g.KY;
    const int64_t gid = static_cast<int64_t>(bx) * blockDim.x + threadIdx.x;
    const int64_t total = static_cast<int64_t>(a.rowEnd - a.rowBegin) * a.groups;
    if (gid >= total)
        return;
    const int y = a.rowBegin + static_cast<int>(gid / a.groups);
    const int gcol = static_cast<int>(gid % a.groups);
    const uint8_t *s = a.io.src + static_cast<int64_t>(by) * a.io.srcFrameSt +
                       static_cast<int64_t>(KY * y - a.io.srcRow0) * a.io.srcSt + COLS * gcol;
    uint32_t acc[COLS / 2] = {};
#pragma unroll 4
    for (int i = 0; i < KY; ++i) {
        uint32_t w[COLS / 2];
        if constexpr (COLS == 16) {
            unpack16(load16_nt(s + static_cast<int64_t>(i) * a.io.srcSt), w);
        } else {
            const u32x3 v = __builtin_nontemporal_load(reinterpret_cast<const u32x3 *>(s + static_cast<int64_t>(i) * a.io.srcSt));
            unpack4(v.x, w[0], w[1]);
            unpack4(v.y, w[2], w[3]);
            unpack4(v.z, w[4], w[5]);
        }
#pragma unroll
        for (int c = 0; c < COLS / 2; ++c)
            acc[c] = pk_mad(w[c], a.g.cy[i], acc[c]);
    }
    uint32_t out[OUTS];
#pragma unroll
    for (int k = 0; k < OUTS; ++k) {
        uint32_t sum = 1u << 22;
        if constexpr (KX % 2 == 0) {
#pragma unroll
            for (int p = 0; p < KX / 2; ++p)
                sum = udot2(acc[(KX * k) / 2 + p], a.g.cx[p], sum);
        } else {
            // odd KX (3): output k's window starts on column 3k; even starts take the aligned pairs
            // (c0, c1), (c2, 0); odd starts the odd-aligned pair (c0, c1) by alignbit, then the
            // pair holding column 3k + 2 in its high half with (0, c2)
            static_assert(KX == 3, "odd ratios: 3");
            const int c0 = 3 * k;
            if (c0 % 2 == 0) {
                sum = udot2(acc[c0 / 2], a.g.cx[0], sum);
                sum = udot2(acc[c0 / 2 + 1], a.g.cx[1], sum);
            } else {
                sum = udot2(__builtin_amdgcn_alignbit(acc[(c0 + 1) / 2], acc[(c0 - 1) / 2], 16), a.g.cx[0], sum);
                sum = udot2(acc[(c0 + 1) / 2], a.g.cx[1] << 16, sum);
            }
        }
        int v = static_cast<int16_t>(static_cast<int>(sum) >> 23);
        uint16_t u = static_cast<uint16_t>(v);
        out[k] = opaque(u > 255 ? 255u : u);
    }
    uint8_t *d = a.io.dst + static_cast<int64_t>(by) * a.io.dstFrameSt +
                 static_cast<int64_t>(y - a.io.dstRow0) * a.io.dstSt + OUTS * gcol;
    if constexpr (OUTS == 8) {
        *reinterpret_cast<uint2 *>(d) = make_uint2(out[0] | (out[1] << 8) | (out[2] << 16) | (out[3] << 24),
                                                   out[4] | (out[5] << 8) | (out[6] << 16) | (out[7] << 24));
    } else if constexpr (OUTS == 4) {
        *reinterpret_cast<uint32_t *>(d) = out[0] | (out[1] << 8) | (out[2] << 16) | (out[3] << 24);
    } else if constexpr (OUTS == 2) {
        *reinterpret_cast<uint16_t *>(d) = static_cast<uint16_t>(out[0] | (out[1] << 8));
    } else {
        d[0] = static_cast<uint8_t>(out[0]);
    }
}
template <int KX, int KYT>
__global__ __launch_bounds__(256) void area_int_kernel(AreaArgs a)
{
    area_int_kernel_body<KX, KYT>(a, blockIdx.x, blockIdx.y);
}

// ================================================================ Linear at exactly 2:1
//
// The reference's Linear resizer at 2:1 (e.g. 3840x2160 -> 1920x1080; plan.cpp
// pick_fast_linear_down): main output i blends source samples 2i + 1 and 2i + 2 on both axes
// (IQOLinearResizerImpl_Generic.cpp:210-282 row loop, :366-407 main columns); the first and last
// rows take the edge source row alone (work = 256 s) and the first and last columns the edge work
// value alone ((w + 128) >> 8; :227-237, :329-364), in the Area arithmetic (u16 work row,
// (s + 2^22) >> 23, int16 cast, clamp).  Thread = the 16 source columns [16g, 16g + 16) plus the
// next aligned dword of an output row's two source rows -> output columns 8g .. 8g + 7 from the
// odd-aligned work pairs (16g + 2k + 1, 16g + 2k + 2): 8 v_perm and 8 packed MACs per source
// row, one v_dot2 per output.  The layout of area_int_kernel (area_kind 8).
__device__ __forceinline__ void linear_d2_body(const AreaArgs &a, const unsigned bx, const unsigned by)
{
    const AreaDev &g = a.g;
    const int64_t gid = static_cast<int64_t>(bx) * blockDim.x + threadIdx.x;
    const int64_t total = static_cast<int64_t>(a.rowEnd - a.rowBegin) * a.groups;
    if (gid >= total)
        return;
    const int y = a.rowBegin + static_cast<int>(gid / a.groups);
    const int gcol = static_cast<int>(gid % a.groups);
    // source rows and their (c, c) splats: edge rows take one row at 256
    int r0 = 2 * y + 1, r1 = 2 * y + 2;
    uint32_t c0 = g.cy[0], c1 = g.cy[1];
    if (y == 0 || y == g.dstH - 1) {
        r0 = r1 = y == 0 ? 0 : g.srcH - 1;
        c0 = 0x01000100u;
        c1 = 0u;
    }
    const uint8_t *sf = a.io.src + static_cast<int64_t>(by) * a.io.srcFrameSt + 16 * gcol;
    const uint8_t *s0 = sf + static_cast<int64_t>(r0 - a.io.srcRow0) * a.io.srcSt;
    const uint8_t *s1 = sf + static_cast<int64_t>(r1 - a.io.srcRow0) * a.io.srcSt;
    // the dword after the 16 columns (the last group: clamped inside the row; its byte then only
    // feeds the high half of the last pair, which the replicated right column does not use)
    const int nxt = 16 * gcol + 16 <= g.srcW - 4 ? 16 : g.srcW - 4 - 16 * gcol;
    const uint4 v0 = *reinterpret_cast<const uint4 *>(s0), v1 = *reinterpret_cast<const uint4 *>(s1);
    const uint32_t e0 = *reinterpret_cast<const uint32_t *>(s0 + nxt), e1 = *reinterpret_cast<const uint32_t *>(s1 + nxt);
    // odd-aligned pairs (b1, b2) (b3, b4) ... (b15, e0) of one row
    auto odd = [](uint4 v, uint32_t e, uint32_t (&q)[8]) {
        q[0] = __builtin_amdgcn_perm(0u, v.x, 0x0c020c01u);
        q[1] = __builtin_amdgcn_perm(v.y, v.x, 0x0c040c03u);
        q[2] = __builtin_amdgcn_perm(0u, v.y, 0x0c020c01u);
        q[3] = __builtin_amdgcn_perm(v.z, v.y, 0x0c040c03u);
        q[4] = __builtin_amdgcn_perm(0u, v.z, 0x0c020c01u);
        q[5] = __builtin_amdgcn_perm(v.w, v.z, 0x0c040c03u);
        q[6] = __builtin_amdgcn_perm(0u, v.w, 0x0c020c01u);
        q[7] = __builtin_amdgcn_perm(e, v.w, 0x0c040c03u);
    };
    uint32_t q0[8], q1[8], w[8];
    odd(v0, e0, q0);
    odd(v1, e1, q1);
#pragma unroll
    for (int k = 0; k < 8; ++k)
        w[k] = pk_mad(q1[k], c1, pk_mul(q0[k], c0));  // u16 work pairs (16-bit wrap)
    uint32_t out[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t sum = udot2(w[k], g.cx[0], 1u << 22);
        const uint16_t u = static_cast<uint16_t>(static_cast<int16_t>(static_cast<int>(sum) >> 23));
        out[k] = opaque(u > 255 ? 255u : u);
    }
    // replicated edge columns: (w + 128) >> 8 of work column 0 / srcW - 1
    auto edge = [](uint32_t wv) {
        const uint16_t u = static_cast<uint16_t>(static_cast<int16_t>(static_cast<int>((wv & 0xffffu) + 128u) >> 8));
        return u > 255 ? 255u : static_cast<uint32_t>(u);
    };
    if (gcol == 0) {
        const uint32_t w0 = pk_mad(__builtin_amdgcn_perm(0u, v1.x, 0x0c010c00u), c1,
                                   pk_mul(__builtin_amdgcn_perm(0u, v0.x, 0x0c010c00u), c0));  // (w0, w1)
        out[0] = opaque(edge(w0));
    }
    if (gcol == a.groups - 1)
        out[7] = opaque(edge(w[7]));  // low half = work column 16g + 15 = srcW - 1
    uint8_t *d = a.io.dst + static_cast<int64_t>(by) * a.io.dstFrameSt +
                 static_cast<int64_t>(y - a.io.dstRow0) * a.io.dstSt + 8 * gcol;
    *reinterpret_cast<uint2 *>(d) = make_uint2(out[0] | (out[1] << 8) | (out[2] << 16) | (out[3] << 24),
                                               out[4] | (out[5] << 8) | (out[6] << 16) | (out[7] << 24));
}
__global__ __launch_bounds__(256) void linear_d2_kernel(AreaArgs a)
{
    linear_d2_body(a, blockIdx.x, blockIdx.y);
}


// ================================================================ exact 2x / 3x bilinear streamer
//
// (3x, F = 3: the same walk; lane l's 24 output columns [3cb, 3cb + 24) read the same work columns
// [cb - 1, cb + 8], output 3cb + j blends columns cb + floor((j - 1) / 3) and the next with phase
// j % 3; a source step yields output rows 3k + 1 .. 3k + 3; 16 + 8-byte stores.)
//
// One WAVE = one row band of one frame x one strip of source columns, walking the band top to
// bottom so every source row is fetched from HBM once per band (2x upsampling reads each source
// row for four output rows; a per-row kernel re-fetched it from L2/MALL each time).
//
// Lane l owns the 8 source columns [cb, cb + 8), cb = x0 - 8 + 8l, and (lanes 1..np) the 16
// output columns [2cb, 2cb + 16), which read work columns [cb - 1, cb + 8]: the two outer ones
// come from the neighbouring lanes by DPP before unpacking, so each source row is one 8-B
// coalesced load + 2 DPP + 5 v_perm into odd-aligned u16 pairs P_q = (cb-1+2q, cb+2q).
//
// Output rows 2k+1 (phase 1) and 2k+2 (phase 0) both blend source rows k and k+1
// (IQOLinearResizerImpl_Generic.cpp:308-325 with o = (y-1)/2 at exact 2x); rows 0 and dstH-1 are
// the replicated first / last source row x 256 (:290-299).  Horizontally output 2cb+j blends
// work columns m, m+1 with m = cb + floor((j-1)/2) and phase j&1 (:374-407): one v_dot2_u32_u16
// per output; (S + 2^22) >> 23 <= 255 always (S <= 65280 * 2^15), so the reference's
// int16 -> u16 clamp is a no-op and the bytes pack with v_ashr_pk_u8_i32.  Columns 0 and dstW-1
// are replicated borders (:343-366): their lanes use a per-lane weight pair (no branch).
//
// The row loop is straight-line (unrolled by the prefetch depth PD, statically named registers)
// and its memory stream branch-free: rows past the band's last source row and stores of rows
// outside the band use out-of-range buffer offsets (no traffic, exact waitcnt accounting).

struct LinearArgs {
    LinearDev g;
    Io io;
    int rowBegin, rowEnd, rowsPerBand;
    int srcBytes, dstBytes;
    int bands, wavesPerRow, np;
};

template <int PD, bool NTST, int F>
__device__ __forceinline__ void linear_up2_kernel_body(const LinearArgs &a, const unsigned bx, const unsigned by)
{
    static_assert(PD % 2 == 0, "the unroll must also cover the 2-slot row ring");
    constexpr int OPL = 8 * F;  // output columns per lane
    __shared__ __attribute__((aligned(16))) uint8_t stage[F == 3 ? 4 * 2048 : 16];  // 3x: store_row24
    const LinearDev &g = a.g;
    const int lane = static_cast<int>(threadIdx.x) & 63;
    const int wib = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    const int gw = static_cast<int>(bx) * 4 + wib;
    if (gw >= a.bands * a.wavesPerRow)
        return;
    const int band = gw / a.wavesPerRow, wcol = gw - band * a.wavesPerRow;
    const int y0 = a.rowBegin + band * a.rowsPerBand;
    const int y1 = min(y0 + a.rowsPerBand, a.rowEnd);
    if (y0 >= y1)
        return;
    const int np = a.np;
    const int x0 = max(0, min(wcol * 8 * np, g.srcW - 8 * np));  // first source column of lane 1
    const int cb = x0 - 8 + 8 * lane;
    const bool produce = lane >= 1 && lane <= np;
    const int voff = (lane <= np + 1 && cb >= 0 && cb < g.srcW) ? cb : 0x7ff00000;
    const int stoff = produce ? F * cb : 0x7ff00000;
    // replicated border columns (work + 128) >> 8 == (work * 2^15 + 2^22) >> 23: the border lanes
    // take the weight pair (0, 2^15) / (2^15, 0) for their outer output, so no branch is needed
    const uint32_t cxFirst = cb == 0 ? 0x80000000u : g.cx[0];
    const uint32_t cxLast = cb + 8 == g.srcW ? 0x00008000u : g.cx[(OPL - 1) % F];

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(by) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(by) * a.io.dstFrameSt;
    const __amdgpu_buffer_rsrc_t srcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcFrame), 0, a.srcBytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0, dstRow0 = a.io.dstRow0;

    // interior output rows of the band: [max(y0, 1), yl); step k covers rows F k + 1 .. F k + F
    const int yl = min(y1, g.dstH - 1);
    const int kLo = y0 <= 1 ? 0 : (y0 - 1) / F;
    const int kHi = (yl + F - 2) / F;          // exclusive
    const int rLast = min(kHi, g.srcH - 1);    // last source row the loop reads (3x: the last main
                                               // row's second sample has weight 0)

    auto load_row = [&](int r) -> u32x2 {
        return __builtin_amdgcn_raw_buffer_load_b64(srcR, voff, r <= rLast ? (r - srcRow0) * srcSt : 0x7ff00000,
                                                    0);  // default policy: 1 % faster than nt on C4
    };
    auto unpack = [&](u32x2 v, uint32_t (&P)[5]) {
        const uint32_t left = static_cast<uint32_t>(
            __builtin_amdgcn_mov_dpp(static_cast<int>(v.y), 0x138 /* wave_shr:1 */, 0xf, 0xf, true));
        const uint32_t right = static_cast<uint32_t>(
            __builtin_amdgcn_mov_dpp(static_cast<int>(v.x), 0x130 /* wave_shl:1 */, 0xf, 0xf, true));
        P[0] = __builtin_amdgcn_perm(v.x, left, 0x0c040c03u);   // (cb-1, cb)
        P[1] = __builtin_amdgcn_perm(0u, v.x, 0x0c020c01u);     // (cb+1, cb+2)
        P[2] = __builtin_amdgcn_perm(v.y, v.x, 0x0c040c03u);    // (cb+3, cb+4)
        P[3] = __builtin_amdgcn_perm(0u, v.y, 0x0c020c01u);     // (cb+5, cb+6)
        P[4] = __builtin_amdgcn_perm(right, v.y, 0x0c040c03u);  // (cb+7, cb+8)
    };
    // horizontal pass + store of one output row from its odd-aligned work pairs
    auto emit = [&](const uint32_t (&W)[5], int y, bool valid) {
        uint32_t E[4];  // even-aligned pairs (cb+2q, cb+2q+1)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            E[q] = __builtin_amdgcn_alignbit(W[q + 1], W[q], 16);
        // output F cb + j blends work columns m, m + 1, m = cb + floor((j - 1) / F), phase j % F
        uint32_t s[OPL];
#pragma unroll
        for (int j = 0; j < OPL; ++j) {
            const int r = j == 0 ? -1 : (j - 1) / F;
            const uint32_t pr = r < 0 ? W[0] : ((r & 1) ? W[(r + 1) >> 1] : E[r >> 1]);
            s[j] = udot2(pr, j == 0 ? cxFirst : (j == OPL - 1 ? cxLast : g.cx[j % F]), 1u << 22);
        }
        uint32_t o[OPL / 4];
#pragma unroll
        for (int q = 0; q < OPL / 4; ++q)
            o[q] = pack23_hi(pack23_lo(s[4 * q], s[4 * q + 1]), s[4 * q + 2], s[4 * q + 3]);
        const int rowOff = valid ? (y - dstRow0) * dstSt : 0x7ff00000;
        if constexpr (F == 3)
            store_row24<NTST ? 2 : 0>(stage + 2048 * wib, o, produce, lane, 24 * np, dstR,
                                      valid ? 3 * x0 + rowOff : 0x7ff00000);
        else
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{o[0], o[1], o[2], o[3]}, dstR, stoff, rowOff, NTST ? 2 : 0);
    };
    auto border_row = [&](int y, int r) {
        uint32_t P[5];
        unpack(__builtin_amdgcn_raw_buffer_load_b64(srcR, voff, (r - srcRow0) * srcSt, 2), P);
#pragma unroll
        for (int q = 0; q < 5; ++q)
            P[q] = pk_mul(P[q], 0x01000100u);
        emit(P, y, true);
    };

    if (y0 == 0)
        border_row(0, 0);

    // row F k + i (i = 1 .. F): phase i % F's (c0, c1) splats
    uint32_t c0[F], c1[F];
#pragma unroll
    for (int i = 1; i <= F; ++i) {
        c0[i - 1] = (g.cy[i % F] & 0xffffu) * 0x10001u;
        c1[i - 1] = (g.cy[i % F] >> 16) * 0x10001u;
    }
    uint32_t U[2][5];
    u32x2 pre[PD];
    unpack(load_row(kLo), U[0]);
    // prologue in the loop's own vm-counter pattern (load, store, store per iteration; the
    // stores are dropped) and issue order, so the waits at the loop header, which must hold for
    // the preheader path too, are the steady-state ones and keep PD rows in flight
#pragma unroll
    for (int i = 0; i < PD; ++i) {
        __builtin_amdgcn_sched_barrier(0);
        pre[i] = load_row(kLo + 1 + i);
#pragma unroll
        for (int j = 0; j < 2 * F - 2; ++j)  // (2x: one store per row, 3x: two)
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, dstR, 0x7ff00000, 0x7ff00000 + 64 * (F * i + j), 0);
    }
    for (int base = kLo; base < kHi; base += PD) {
        static_for<PD>([&](auto uc) {
            constexpr int v = decltype(uc)::value;
            const int k = base + v;
            // iterations past the band end (k >= kHi, fewer than PD) run on zero rows and drop
            // their stores: no branch inside the loop keeps the vm-counter accounting exact
            // keep iterations apart: otherwise the scheduler hoists all PD unpacks to the top
            // of the trip and the wait for them drains the whole prefetch
            __builtin_amdgcn_sched_barrier(0);
            unpack(pre[v], U[(v + 1) % 2]);  // source row k + 1
            pre[v] = load_row(k + 1 + PD);
            const uint32_t(&A)[5] = U[v % 2];
            const uint32_t(&B)[5] = U[(v + 1) % 2];
#pragma unroll
            for (int i = 1; i <= F; ++i) {
                uint32_t W[5];
#pragma unroll
                for (int q = 0; q < 5; ++q)
                    W[q] = pk_mad(B[q], c1[i - 1], pk_mul(A[q], c0[i - 1]));
                const int y = F * k + i;
                emit(W, y, y >= y0 && y < yl);
            }
        });
    }

    if (y1 == g.dstH && g.dstH > 1)
        border_row(g.dstH - 1, g.srcH - 1);
}
template <int PD, bool NTST, int F>
__global__ __launch_bounds__(256) void linear_up2_kernel(LinearArgs a)
{
    // (plain block order, neighbouring bands on different XCDs.  Round 6: an XCD-aware order
    // (xcd_spread, each XCD a contiguous run of (frame, band) blocks) removes the re-read of the
    // source row two bands share -- HBM traffic 1.117x -> 1.0002x algorithmic -- but is 9 % slower
    // (C4 x256 0.508 vs 0.464 ms, profiles/r06/c4_xcd_order.txt): every XCD streaming its own
    // address range spreads the requests over fewer channels at a time)
    linear_up2_kernel_body<PD, NTST, F>(a, blockIdx.x, blockIdx.y);
}


// ================================================================ YUV 4:2:0 in one launch
//
// The three planes of a batch of I420 frames (the reference benchmark's workload,
// benchmark.cpp:206-229: Y at full size, U and V at half size, Lanczos chroma with pxScale 2) in
// ONE launch: grid.z = plane, grid.x covers the larger plane grid, blocks past a plane's own grid
// exit.  The plane bodies are the single-plane kernels' bodies; Y and chroma may use different
// kernels (e.g. block-shared symmetric Y + accumulator-ring chroma).  All bodies use 256-thread
// blocks here (the block-shared Y body only when its row takes exactly 4 waves).

template <typename AY, typename AC>
struct Yuv3Args {
    AY y;
    AC u, v;
    unsigned gxY, gxC;  // grid.x of the Y plane / of each chroma plane
};

template <int NY, int NX, int OFFX, bool ONE, bool LINE>
struct SymbY {
    static __device__ __forceinline__ void run(const LanczosArgs &a, unsigned bx, unsigned by)
    {
        lanczos_symb_kernel_body<NY, NX, OFFX, NY / 2, 1, ONE, LINE>(a, bx, by, a.rowsPerBand);  // ring depth = window period (prep_lanczos)
    }
};
template <int NY, int NX, int OFFX, bool ONE>
struct SymY {
    static __device__ __forceinline__ void run(const LanczosArgs &a, unsigned bx, unsigned by)
    {
        lanczos_sym_kernel_body<NY, NX, OFFX, 4, ONE>(a, bx, by);
    }
};
struct RingChroma {  // pxScale-2 chroma tables of Lanczos-2/3 2:1 (3 taps padded to 4)
    static __device__ __forceinline__ void run(const LanczosArgs &a, unsigned bx, unsigned by)
    {
        lanczos_stream_kernel_body<2, 2, 4, 4, 0, 3>(a, bx, by);
    }
};
template <int KX, int KYT>
struct AreaPlane {
    static __device__ __forceinline__ void run(const AreaArgs &a, unsigned bx, unsigned by)
    {
        area_int_kernel_body<KX, KYT>(a, bx, by);
    }
};
struct LinearD2Plane {
    static __device__ __forceinline__ void run(const AreaArgs &a, unsigned bx, unsigned by)
    {
        linear_d2_body(a, bx, by);
    }
};
struct LinearPlane {
    static __device__ __forceinline__ void run(const LinearArgs &a, unsigned bx, unsigned by)
    {
        linear_up2_kernel_body<2, true, 2>(a, bx, by);
    }
};

template <typename BY, typename BC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void
yuv420_lanczos_kernel(Yuv3Args<LanczosArgs, LanczosArgs> a)
{
    if (blockIdx.z == 0) {
        if (blockIdx.x < a.gxY)
            BY::run(a.y, blockIdx.x, blockIdx.y);
    } else if (blockIdx.x < a.gxC) {
        BC::run(blockIdx.z == 1 ? a.u : a.v, blockIdx.x, blockIdx.y);
    }
}

template <typename B, typename A>
__global__ __launch_bounds__(256) void yuv420_plane_kernel(Yuv3Args<A, A> a)
{
    if (blockIdx.z == 0) {
        if (blockIdx.x < a.gxY)
            B::run(a.y, blockIdx.x, blockIdx.y);
    } else if (blockIdx.x < a.gxC) {
        B::run(blockIdx.z == 1 ? a.u : a.v, blockIdx.x, blockIdx.y);
    }
}

} // namespace

// ================================================================ launchers


hipError_t launch_general(const GeneralDev &g, const Io &io, int rowBegin, int rowEnd, hipStream_t s)
{
    if (rowEnd <= rowBegin || io.frames <= 0)
        return hipSuccess;
    GeneralArgs a{g, io, rowBegin};
    dim3 grid(static_cast<unsigned>(rowEnd - rowBegin), static_cast<unsigned>(io.frames));
    size_t lds = static_cast<size_t>(g.ldsInts) * sizeof(int);
    hipLaunchKernelGGL(general_kernel, grid, dim3(256), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_tile(const TileDev &t, const Io &io, int rowBegin, int rowEnd, hipStream_t s)
{
    if (rowEnd <= rowBegin || io.frames <= 0)
        return hipSuccess;
    const int rows = rowEnd - rowBegin;
    const int64_t sb = static_cast<int64_t>(io.srcRowEnd - io.srcRow0 - 1) * io.srcSt + t.srcW;
    const int64_t db = static_cast<int64_t>(rowEnd - 1 - io.dstRow0) * io.dstSt + t.dstW;  // stores are relative to dstRow0
    if (sb >= (int64_t(1) << 31) || db >= (int64_t(1) << 31) || io.srcSt >= (int64_t(1) << 24) ||
        io.dstSt >= (int64_t(1) << 31) || t.srcH >= (1 << 24))
        return hipErrorInvalidValue;
    const int nTx = (t.dstW + t.CT - 1) / t.CT, nTy = (rows + t.TH - 1) / t.TH;
    const uint64_t nTiles = static_cast<uint64_t>(nTx) * static_cast<uint64_t>(nTy) * static_cast<uint64_t>(io.frames);
    if (nTiles >= (uint64_t(1) << 31))
        return hipErrorInvalidValue;
    TileArgs a{t, io, rowBegin, rowEnd, static_cast<int>(sb), static_cast<int>(db), nTx, nTy,
               static_cast<unsigned>(nTiles)};
    const size_t lds = static_cast<size_t>(t.TH) * (static_cast<size_t>(t.pitchDw) * 4 + 16 + static_cast<size_t>(t.nYp) * 8) +
                       4u * static_cast<size_t>(t.CT) + static_cast<size_t>(t.srcRows) * t.spitch;
    dim3 grid(static_cast<unsigned>(nTiles));
#define IQO_TILE(NP_)                                                                                \
    case NP_:                                                                                        \
        kern = t.lanczos ? reinterpret_cast<const void *>(tile_kernel<NP_, true>)                    \
                         : reinterpret_cast<const void *>(tile_kernel<NP_, false>);                  \
        break;
    const void *kern = nullptr;
    switch (t.NP) {
        IQO_TILE(1)
        IQO_TILE(2)
        IQO_TILE(3)
        IQO_TILE(4)
        IQO_TILE(5)
        IQO_TILE(6)
        IQO_TILE(7)
        IQO_TILE(8)
        IQO_TILE(10)
        IQO_TILE(12)
        IQO_TILE(16)
    default:
        return hipErrorInvalidValue;
    }
#undef IQO_TILE
    void *args[] = {&a};
    return hipLaunchKernel(kern, grid, dim3(256), args, lds, s);
}

hipError_t launch_walk(const WalkDev &w, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s,
                       int stripLo, int strips, int stripStride)
{
    if (strips < 0)
        strips = w.nS;
    if (rowEnd <= rowBegin || io.frames <= 0 || strips == 0)
        return hipSuccess;
    if (stripLo < 0 || stripLo + (strips - 1) * stripStride >= w.nS || stripStride < 1)
        return hipErrorInvalidValue;
    const int rows = rowEnd - rowBegin;
    const TileDev &t = w.t;
    // the buffer range ends at the dword holding the window's last pixel: a dword load that
    // crosses the range end reads as 0, and an aligned dword never crosses a page
    const int64_t sb = static_cast<int64_t>(io.srcRowEnd - io.srcRow0 - 1) * io.srcSt + ((t.srcW + 3) & ~3);
    const int64_t db = static_cast<int64_t>(rowEnd - 1 - io.dstRow0) * io.dstSt + t.dstW;  // stores are relative to dstRow0
    if (sb >= (int64_t(1) << 31) || db >= (int64_t(1) << 31) || io.srcSt >= (int64_t(1) << 24))
        return hipErrorInvalidValue;
    const void *kern = nullptr;
    // (NP, VY = 2NP or 2NP - 2, NV) instantiations
    const int e = 2 * t.NP - t.nYp;
    if ((e != 0 && e != 2) || t.nYp < 2 || (w.NV != 1 && w.NV != 2))
        return hipErrorInvalidValue;
#define IQO_WALK_NV(NP_, VY_, NV_)                                                                   \
    kern = t.lanczos ? reinterpret_cast<const void *>(walk_kernel<NP_, VY_, NV_, true>)              \
                     : reinterpret_cast<const void *>(walk_kernel<NP_, VY_, NV_, false>);
#define IQO_WALK_VY(NP_, VY_)                                                                        \
    if (w.NV == 1) {                                                                                 \
        IQO_WALK_NV(NP_, VY_, 1)                                                                     \
    } else {                                                                                         \
        IQO_WALK_NV(NP_, VY_, 2)                                                                     \
    }
#define IQO_WALK(NP_)                                                                                \
    case NP_:                                                                                        \
        if (e == 0) {                                                                                \
            IQO_WALK_VY(NP_, 2 * NP_)                                                                \
        } else {                                                                                     \
            IQO_WALK_VY(NP_, 2 * NP_ - 2)                                                            \
        }                                                                                            \
        break;
    switch (t.NP) {
    case 1:
        IQO_WALK_VY(1, 2)
        break;
        IQO_WALK(2)
        IQO_WALK(3)
        IQO_WALK(4)
        IQO_WALK(5)
        IQO_WALK(6)
        IQO_WALK(7)
        IQO_WALK(8)
    default:
        return hipErrorInvalidValue;
    }
#undef IQO_WALK
#undef IQO_WALK_VY
#undef IQO_WALK_NV
    const int lds = 4 * w.waveBytes;
    // bands per frame: about 2.5 rounds of resident waves (more waves than slots hide the tail and
    // the latency of each wave's serial walk; MI355X G1/G2/G3 sweeps), bands of >= 16 rows
    if (bands <= 0) {
        const int64_t resident = std::max(1, resident_waves(kern, 256, lds));
        const int64_t perBand = static_cast<int64_t>(strips) * io.frames;
        bands = static_cast<int>(std::min<int64_t>((5 * resident / 2 + perBand - 1) / perBand, std::max(1, rows / 16)));
    }
    bands = std::max(1, std::min(bands, rows));
    const int rpb = (rows + bands - 1) / bands;
    bands = (rows + rpb - 1) / rpb;
    const uint64_t nWaves = static_cast<uint64_t>(strips) * static_cast<uint64_t>(bands) * static_cast<uint64_t>(io.frames);
    if (nWaves >= (uint64_t(1) << 31))
        return hipErrorInvalidValue;
    WalkArgs a{w, io, rowBegin, rowEnd, rpb, bands, static_cast<int>(sb), static_cast<int>(db),
               static_cast<unsigned>(nWaves), stripLo, strips, stripStride};
    void *args[] = {&a};
    return hipLaunchKernel(kern, dim3(static_cast<unsigned>((nWaves + 3) / 4)), dim3(256), args, lds, s);
}



bool lanczos_stream_supported(int KY, int KX, int NY, int NXP, int offX)
{
    return KY == 2 && KX == 2 &&
           ((NY == 10 && NXP == 14 && offX == -6) || (NY == 8 && NXP == 10 && offX == -4) ||
            (NY == 4 && NXP == 4 && offX == 0));
}

int lanczos_stream_block(int) { return 256; }

// One prepared launch of a band-walking kernel: arguments, geometry and the instantiation.
template <typename A>
struct Prep {
    A a;
    dim3 grid;
    int block = 256, lds = 0;
    const void *kern = nullptr;
    int kind = 0;  // Lanczos: 0 accumulator ring, 1 block-shared symmetric, 2 per-wave symmetric
    int pd = 0;    // prefetch / ring depth the instantiation was chosen for
};

hipError_t prep_lanczos(const LanczosDev &l, const Io &io, int rowBegin, int rowEnd, int bands, Prep<LanczosArgs> *P)
{
    const int rows = rowEnd - rowBegin;
    int opw = 62 * (16 / l.KX);
    int wpr = (l.dstW + opw - 1) / opw;
    int np = 62;
    if (l.sym) {
        // producing lanes per wave: the fewest waves per row, then the fewest lanes that still
        // tile the output width (1920 -> 4 waves x 60 lanes x 8 outputs, no overlap)
        const int lanes = (l.dstW + 7) / 8;
        np = l.np > 0 ? min(l.np, 62) : (lanes + wpr - 1) / wpr;
        if (np * 8 > l.dstW)
            np = l.dstW / 8;
        if (l.NY >= 12 && ((l.dstW + 8 * np - 1) / (8 * np) > 4 || (l.NY == 16 && !symb_line(l.dstW, np))))
            np = (lanes + wpr - 1) / wpr;  // (a lane count that needs more than 4 waves or, Lanczos-5,
                                           // leaves the line edge scheme: the default)
        opw = 8 * np;
        wpr = (l.dstW + opw - 1) / opw;
    }
    // the instantiation this call runs
    const int pd = l.prefetch;
    const void *kern = nullptr;
    int block = 256, ldsBytes = 0;
    // block-shared ring rows: a 16-B zero pad, then LDS column 16 + c holds source column c.  A
    // row must hold every source column and the right halo lane's 16 bytes past the last output
    // pair (LDS bytes up to 32 + 2 dstW); it is DMA'd in 1-KiB chunks, the last one masked to
    // the lanes the row needs, so the pitch is that extent and not a whole number of KiB
    const int rowNeed = (std::max(32 + 2 * l.dstW, 16 + l.srcW) + 15) & ~15;
    const int chunks = (rowNeed - 16 + 1023) / 1024;
    const int lastLanes = (rowNeed - 16 - 1024 * (chunks - 1)) / 16;
    const int cpw = (chunks + wpr - 1) / wpr;
    const bool shared = l.sym == 1 && wpr <= 4 && cpw <= 2;
    if ((l.NY == 12 || l.NY == 16) && !shared)
        return hipErrorInvalidValue;  // Lanczos-4 / -5 2:1: block-shared instantiation only (plan.cpp)
    // narrow frames: several frames side by side in one 2-wave workgroup (lanczos_stack_kernel)
    const int npf = l.srcW / 16;
    const int fpwMax = npf >= 1 ? std::min(6, 125 / (npf + 1)) : 0;
    // (only where a frame leaves most of a wave idle: 320 -> 160 columns, 5 frames per workgroup,
    // 0.427 vs 0.529 ms per 16384 frames; at 3 frames of 640 columns (C1) it is no faster, and 3.5 %
    // slower for Lanczos-3 640x360 -> 320x180, profiles/r03/stack_narrow.txt; option "stack" = 2
    // forces it from 2 frames per workgroup)
    const bool stack = shared && l.NY <= 10 && l.stack && wpr == 1 && l.srcW == 2 * l.dstW && l.srcW % 16 == 0 && np == npf &&
                       fpwMax >= (l.stack >= 2 ? 2 : 4) && io.frames >= 2;
    // block-shared ring depth: prefetch 1-2 -> 3, 3 (default) -> the window period NY/2 (4 for
    // Lanczos-2, 5 for Lanczos-3: every ring slot index is then a compile-time constant; C2 x256
    // 0.5226 vs 0.532 ms at depth 4), 4 -> 5.  Depth 5 packs the ring rows to the bytes they need
    // so that four 4-wave workgroups still fit a CU's LDS.
    const int K = pd <= 2 ? 3 : pd == 3 ? (l.NY >= 10 ? 5 : 4) : 5;
    const bool pack = shared && K == 5;
    const int rowPitch = pack ? rowNeed : 16 + 1024 * chunks;
    int fpw = 1;
    if (stack) {
        const bool one = (l.cy[0] & 0xffffu) == 1u;
        fpw = std::min(fpwMax, io.frames);
        const int scpw = (fpw + 1) / 2;
        ldsBytes = l.NY / 2 * 4096 + scpw * 2 * 2 * IQO_SYMB_EDGE_BATCH * 16 + 1024;
        block = 128;
#define IQO_STACK_C(NY_, NX_, OX_, ONE_)                                                                \
    (scpw == 1 ? reinterpret_cast<const void *>(lanczos_stack_kernel<NY_, NX_, OX_, NY_ / 2, 1, ONE_>)         \
     : scpw == 2 ? reinterpret_cast<const void *>(lanczos_stack_kernel<NY_, NX_, OX_, NY_ / 2, 2, ONE_>)       \
                 : reinterpret_cast<const void *>(lanczos_stack_kernel<NY_, NX_, OX_, NY_ / 2, 3, ONE_>))
        if (l.NY == 10 && one)
            kern = IQO_STACK_C(10, 12, -5, true);
        else if (l.NY == 10)
            kern = IQO_STACK_C(10, 12, -5, false);
        else
            kern = IQO_STACK_C(8, 8, -3, false);
#undef IQO_STACK_C
    } else if (shared) {
        // block-shared ring (default): one workgroup of wpr waves per row band
        const bool one = (l.cy[0] & 0xffffu) == 1u;
        const bool line = symb_line(l.dstW, np);  // border columns: whole-line scheme
        if (l.NY == 16 && !line)
            return hipErrorInvalidValue;  // Lanczos-5: 5 border columns need the line scheme's 8 edge sums
        ldsBytes = K * 2 * rowPitch + symb_edge_bytes(l.NY, l.NX) + (cpw * wpr > chunks ? 1024 : 0);
#ifdef IQO_EXP_WGCU  // experiment builds: fewer workgroups per CU by inflating the LDS allocation
        if (const char *ev = getenv("IQO_EXP_WGCU"))
            if (atoi(ev) > 0)
                ldsBytes = std::max(ldsBytes, 163840 / atoi(ev) - 256);
#endif
        block = 64 * wpr;
#define IQO_SYMB_L(NY_, NX_, OX_, K_, CPW_, ONE_)                                                       \
    (line ? reinterpret_cast<const void *>(lanczos_symb_kernel<NY_, NX_, OX_, K_, CPW_, ONE_, true>)             \
          : reinterpret_cast<const void *>(lanczos_symb_kernel<NY_, NX_, OX_, K_, CPW_, ONE_, false>))
#define IQO_SYMB_K(NY_, NX_, OX_, K_, ONE_)                                                             \
    (cpw == 1 ? IQO_SYMB_L(NY_, NX_, OX_, K_, 1, ONE_) : IQO_SYMB_L(NY_, NX_, OX_, K_, 2, ONE_))
#define IQO_SYMB(NY_, NX_, OX_, ONE_)                                                                   \
    (K == 3 ? IQO_SYMB_K(NY_, NX_, OX_, 3, ONE_) : K == 4 ? IQO_SYMB_K(NY_, NX_, OX_, 4, ONE_)          \
            : IQO_SYMB_K(NY_, NX_, OX_, 5, ONE_))
        if (l.NY == 10 && one)
            kern = IQO_SYMB(10, 12, -5, true);
        else if (l.NY == 10)
            kern = IQO_SYMB(10, 12, -5, false);
        else if (l.NY == 12)
            kern = IQO_SYMB(12, 16, -7, false);  // Lanczos-4 2:1 (3 waves per SIMD: the 12-row window)
        else if (l.NY == 16)
            kern = IQO_SYMB(16, 20, -9, false);  // Lanczos-5 2:1 (2 waves per SIMD: the 16-row window)
        else
            kern = IQO_SYMB(8, 8, -3, false);
#undef IQO_SYMB
#undef IQO_SYMB_K
#undef IQO_SYMB_L
    } else if (l.sym) {
        const bool one = (l.cy[0] & 0xffffu) == 1u;
        if (l.NY == 10 && one)
            kern = pd <= 2 ? reinterpret_cast<const void *>(lanczos_sym_kernel<10, 12, -5, 3, true>)
                           : reinterpret_cast<const void *>(lanczos_sym_kernel<10, 12, -5, 4, true>);
        else if (l.NY == 10)
            kern = reinterpret_cast<const void *>(lanczos_sym_kernel<10, 12, -5, 4, false>);
        else
            kern = pd <= 2 ? reinterpret_cast<const void *>(lanczos_sym_kernel<8, 8, -3, 3, false>)
                           : reinterpret_cast<const void *>(lanczos_sym_kernel<8, 8, -3, 4, false>);
    } else if (l.NY == 4) {
        kern = pd <= 1   ? reinterpret_cast<const void *>(lanczos_stream_kernel<2, 2, 4, 4, 0, 1>)
               : pd == 2 ? reinterpret_cast<const void *>(lanczos_stream_kernel<2, 2, 4, 4, 0, 2>)
                         : reinterpret_cast<const void *>(lanczos_stream_kernel<2, 2, 4, 4, 0, 3>);
    } else if (l.NY == 10) {
        kern = pd <= 1   ? reinterpret_cast<const void *>(lanczos_stream_kernel<2, 2, 10, 14, -3, 1>)
               : pd == 2 ? reinterpret_cast<const void *>(lanczos_stream_kernel<2, 2, 10, 14, -3, 2>)
                         : reinterpret_cast<const void *>(lanczos_stream_kernel<2, 2, 10, 14, -3, 3>);
    } else {
        kern = pd <= 1   ? reinterpret_cast<const void *>(lanczos_stream_kernel<2, 2, 8, 10, -2, 1>)
               : pd == 2 ? reinterpret_cast<const void *>(lanczos_stream_kernel<2, 2, 8, 10, -2, 2>)
                         : reinterpret_cast<const void *>(lanczos_stream_kernel<2, 2, 8, 10, -2, 3>);
    }
    const int groups = stack ? (io.frames + fpw - 1) / fpw : io.frames;  // workgroup columns of the grid
    if (bands <= 0) {
        const int resident = resident_waves(kern, block, ldsBytes);
        if (stack) {
            const int64_t want = static_cast<int64_t>(l.rounds > 0 ? l.rounds : 6) * (resident / 2);
            bands = static_cast<int>(std::min<int64_t>((want + groups - 1) / groups, std::max(1, rows / 16)));
        } else if (shared && l.rounds >= 0) {
            // block-shared ring: about `rounds` rounds of resident workgroups (default 6), bands of
            // >= 16 rows.  On fresh data more, shorter bands beat the one-round makespan optimum
            // (C2 x128: 8 bands 0.305 ms, 24 0.296, 48 0.294): workgroups that start and finish at
            // different times spread their requests over the memory channels, and the halo rows of
            // neighbouring bands (same XCD) come from L2
            // Round 4: and bands of at most ~22 rows for 1920-wide outputs, up to 48 for narrower ones
            // (C2 x256: 24 bands 0.525 ms, 48 0.510, 96 0.515, 135 0.530; C1 x4096 (320 columns):
            // 2 bands 0.385, 5 0.366, 10 0.378).  Shorter bands keep the concurrently read source
            // window compact; longer ones pay less per-band prologue, which weighs more on narrow rows.
            // Round 5, at a steady GPU clock (after the power-management transient a streaming
            // launch starts with, profiles/r05/clock_transient.txt): the Lanczos-2/3 windows (NY <= 10)
            // want bands of ~12 rows on rows of >= 640 outputs -- C2 x1024 1.936 ms at 50 bands of 22
            // rows, 1.879 at 90 of 12 (frac 0.686 -> 0.706), x256 0.495 -> 0.480; 1080p -> 540p
            // Lanczos-2 -2.6 % -- and ~24 on narrower rows (C1 x4096: 5 bands 0.331 ms, 10 bands
            // 0.318, 20 bands 0.324); the 12- and 16-row windows keep ~22-row bands (Lanczos-4 4K:
            // 50 bands 0.267 ms, 90 bands 0.270), their per-band halo being larger
            // (profiles/r05/steady_streamer_bands.txt)
            const int64_t want = static_cast<int64_t>(l.rounds > 0 ? l.rounds : 6) * (resident / wpr);
            const int64_t byRounds = (want + io.frames - 1) / io.frames;
            const int rowsMax = l.NY <= 10 ? (l.dstW >= 640 ? 12 : 24)
                                           : std::min(48, std::max(22, 22 * 1920 / std::max(1, l.dstW)));
            const int rowsMin = l.NY <= 10 ? 12 : 16;
            bands = static_cast<int>(std::min<int64_t>(std::max<int64_t>(byRounds, (rows + rowsMax - 1) / rowsMax),
                                                       std::max(1, rows / rowsMin)));
        } else {
            bands = choose_bands(rows, io.frames, wpr, resident, l.NY - 2);
        }
    }
    bands = max(1, min(bands, rows));
    const int rpb = (rows + bands - 1) / bands;
    bands = (rows + rpb - 1) / rpb;
    LanczosArgs &a = P->a;
    a = LanczosArgs{l, io, rowBegin, rowEnd, rpb, 0, 0, bands, wpr, l.dbg, np, rowPitch, chunks,
                    pack ? lastLanes : 64, fpw, io.frames, 0, 0, 0};
    // XCD tail split: each XCD's last frame in short bands (about 8 rows; option "tail"), when
    // the batch splits evenly over the 8 XCDs into at least 2 frames each
    if (shared && !stack && l.tail >= 0 && io.frames % 8 == 0 && io.frames >= 16) {
        const int tb = l.tail > 0 ? min(l.tail, rows) : (rows + 7) / 8;
        const int tr = (rows + tb - 1) / tb;
        a.tailBands = (rows + tr - 1) / tr;
        a.tailRows = tr;
        a.framesPerXcd = io.frames / 8;
        if (a.tailBands <= bands)
            a.tailBands = 0;  // the bands are already short
    }
    // buffer ranges: the source window spans rows [srcRow0, srcRowEnd) of the frame, the destination
    // band rows [rowBegin, rowEnd); both must be addressable with 31-bit offsets
    const int64_t sb = static_cast<int64_t>(io.srcRowEnd - io.srcRow0 - 1) * io.srcSt + l.srcW;
    const int64_t db = static_cast<int64_t>(rowEnd - 1 - io.dstRow0) * io.dstSt + l.dstW;  // stores are relative to dstRow0
    if (sb >= (int64_t(1) << 31) || db >= (int64_t(1) << 31) || io.srcSt >= (int64_t(1) << 31) ||
        io.dstSt >= (int64_t(1) << 31))
        return hipErrorInvalidValue;
    a.srcBytes = static_cast<int>(sb);
    a.dstBytes = static_cast<int>(db);
    const int waves = bands * wpr;
    P->grid = shared ? dim3(static_cast<unsigned>(bands), static_cast<unsigned>(groups))
                       : dim3(static_cast<unsigned>((waves + 3) / 4), static_cast<unsigned>(io.frames));
    if (a.tailBands > 0)
        P->grid = dim3(static_cast<unsigned>(8 * ((a.framesPerXcd - 1) * bands + a.tailBands)), 1u);
    P->block = block;
    P->lds = ldsBytes;
    P->kern = kern;
    P->kind = stack ? 3 : shared ? 1 : (l.sym ? 2 : 0);
    P->pd = pd;
    return hipSuccess;
}

hipError_t launch_lanczos_stream(const LanczosDev &l, const Io &io, int rowBegin, int rowEnd, int bands,
                                 hipStream_t s)
{
    if (rowEnd <= rowBegin || io.frames <= 0)
        return hipSuccess;
    Prep<LanczosArgs> P;
    hipError_t e = prep_lanczos(l, io, rowBegin, rowEnd, bands, &P);
    if (e != hipSuccess)
        return e;
    void *args[] = {&P.a};
    return hipLaunchKernel(P.kern, P.grid, dim3(static_cast<unsigned>(P.block)), args, static_cast<size_t>(P.lds), s);
}

// instantiations of area_int_kernel: <4,4> <2,2> <2,*> <4,*> <8,*> <3,3> <3,*> <6,*>
constexpr int kAreaKinds = 9;  // kind 8: Linear 2:1 (linear_d2_body)
int area_kind(const AreaDev &g)
{
    if (g.lin)
        return 8;
    if (g.KX == 3)
        return g.KY == 3 ? 5 : 6;
    if (g.KX == 6)
        return 7;
    return g.KX == 4 && g.KY == 4 ? 0 : g.KX == 2 && g.KY == 2 ? 1 : g.KX == 2 ? 2 : g.KX == 4 ? 3 : 4;
}

hipError_t prep_area(const AreaDev &g, const Io &io, int rowBegin, int rowEnd, Prep<AreaArgs> *P)
{
    const int cols = 16 % g.KX == 0 ? 16 : 12;  // source columns per thread (area_int_kernel_body)
    P->a = AreaArgs{g, io, rowBegin, rowEnd, g.srcW / cols};
    const int64_t total = static_cast<int64_t>(rowEnd - rowBegin) * P->a.groups;
    P->grid = dim3(static_cast<unsigned>((total + 255) / 256), static_cast<unsigned>(io.frames));
    P->kind = area_kind(g);
    static const void *const kerns[kAreaKinds] = {
        reinterpret_cast<const void *>(area_int_kernel<4, 4>), reinterpret_cast<const void *>(area_int_kernel<2, 2>),
        reinterpret_cast<const void *>(area_int_kernel<2, 0>), reinterpret_cast<const void *>(area_int_kernel<4, 0>),
        reinterpret_cast<const void *>(area_int_kernel<8, 0>), reinterpret_cast<const void *>(area_int_kernel<3, 3>),
        reinterpret_cast<const void *>(area_int_kernel<3, 0>), reinterpret_cast<const void *>(area_int_kernel<6, 0>),
        reinterpret_cast<const void *>(linear_d2_kernel)};
    P->kern = kerns[P->kind];
    return hipSuccess;
}

hipError_t launch_area_int(const AreaDev &g, const Io &io, int rowBegin, int rowEnd, hipStream_t s)
{
    if (rowEnd <= rowBegin || io.frames <= 0)
        return hipSuccess;
    Prep<AreaArgs> P;
    (void)prep_area(g, io, rowBegin, rowEnd, &P);
    void *args[] = {&P.a};
    return hipLaunchKernel(P.kern, P.grid, dim3(256), args, 0, s);
}

hipError_t prep_linear(const LinearDev &g, const Io &io, int rowBegin, int rowEnd, int bands, Prep<LinearArgs> *P)
{
    if (g.srcW % 8 || (g.F != 2 && g.F != 3) || g.dstW != g.F * g.srcW || g.srcW < 8)
        return hipErrorInvalidValue;
    const int rows = rowEnd - rowBegin;
    // producing lanes per wave: the fewest waves per row, then the fewest lanes that tile the width
    const int lanes = g.srcW / 8;
    int wpr = (lanes + 61) / 62;
    int np = g.np > 0 ? min(g.np, min(62, lanes)) : (lanes + wpr - 1) / wpr;
    // round 6, 2x: strips of whole 128-byte output lines (16 np bytes per row, np a multiple of 8)
    // that tile the width exactly, if that costs at most one more wave per row: 1920 columns take 5
    // waves of 48 lanes instead of 4 of 60, whose 960-byte strips split a line at every other
    // boundary between two waves (C4 x256 at 216 bands: 0.471 vs 0.486 ms,
    // profiles/r06/c4_bands_lanes.txt)
    if (g.np <= 0 && g.F == 2)
        for (int c = 56; c >= 8; c -= 8)
            if (lanes % c == 0 && lanes / c <= wpr + 1) {
                np = c;
                break;
            }
    wpr = (lanes + np - 1) / np;
    // nontemporal stores by default (variant builds: dbg 16 = plain stores, for A/B); 2 rows in
    // flight per wave measured best on C4 (the kernel is write-bound: 4 output bytes per source byte)
    const bool nt = g.F == 3 || !(IQO_DBG(g) & 16);
    // (round 2 also instantiated 4 and 8 rows in flight: no faster, removed in round 5)
    const int pd = 2;
    const void *kern = g.F == 3 ? reinterpret_cast<const void *>(linear_up2_kernel<2, true, 3>)
                       : nt     ? reinterpret_cast<const void *>(linear_up2_kernel<2, true, 2>)
                                : reinterpret_cast<const void *>(linear_up2_kernel<2, false, 2>);
    if (bands <= 0 && g.F == 2) {
        // round 6, at a steady clock: bands of ~10 output rows (5 source rows) whatever the batch (C4
        // x256, 48-lane strips: 216 bands 0.471 ms, 180 0.488, 144 0.481, 96 0.501, round 5's 48
        // 0.526; x64: 216 bands 0.120 vs 0.131 ms, profiles/r06/c4_bands_lanes.txt)
        bands = std::max(1, rows / 10);
    } else if (bands <= 0) {
        // ~6 rounds of resident waves, >= 16 rows per band (fresh data, C4 x256: 48 bands 0.537 ms
        // vs 0.555 for the one-round makespan choice)
        const int64_t want = 6 * static_cast<int64_t>(resident_waves(kern)) / wpr;
        bands = static_cast<int>(std::min<int64_t>((want + io.frames - 1) / io.frames, std::max(1, rows / 16)));
    }
    bands = max(1, min(bands, rows));
    const int rpb = (rows + bands - 1) / bands;
    bands = (rows + rpb - 1) / rpb;
    LinearArgs &a = P->a;
    a = LinearArgs{g, io, rowBegin, rowEnd, rpb, 0, 0, bands, wpr, np};
    const int64_t sb = static_cast<int64_t>(io.srcRowEnd - io.srcRow0 - 1) * io.srcSt + g.srcW;
    const int64_t db = static_cast<int64_t>(rowEnd - 1 - io.dstRow0) * io.dstSt + g.dstW;  // stores are relative to dstRow0
    if (sb >= (int64_t(1) << 31) || db >= (int64_t(1) << 31))
        return hipErrorInvalidValue;
    a.srcBytes = static_cast<int>(sb);
    a.dstBytes = static_cast<int>(db);
    const int waves = bands * wpr;
    P->grid = dim3(static_cast<unsigned>((waves + 3) / 4), static_cast<unsigned>(io.frames));
    P->kern = kern;
    P->kind = nt ? 1 : 0;
    P->pd = pd;
    return hipSuccess;
}

hipError_t launch_linear_up2(const LinearDev &g, const Io &io, int rowBegin, int rowEnd, int bands,
                             hipStream_t s)
{
    if (rowEnd <= rowBegin || io.frames <= 0)
        return hipSuccess;
    Prep<LinearArgs> P;
    hipError_t e = prep_linear(g, io, rowBegin, rowEnd, bands, &P);
    if (e != hipSuccess)
        return e;
    void *args[] = {&P.a};
    return hipLaunchKernel(P.kern, P.grid, dim3(256), args, 0, s);
}


// ---- YUV 4:2:0 launchers: one launch for the three planes when the planes' kernels have a fused
// instantiation, else hipErrorNotSupported (the caller then launches plane by plane).

template <typename A>
hipError_t launch_fused3(const void *kern, const Prep<A> &y, const Prep<A> &u, const Prep<A> &v, int block, int lds,
                         hipStream_t s)
{
    Yuv3Args<A, A> a{y.a, u.a, v.a, y.grid.x, u.grid.x};
    const dim3 grid(std::max(y.grid.x, u.grid.x), y.grid.y, 3);
    void *args[] = {&a};
    return hipLaunchKernel(kern, grid, dim3(static_cast<unsigned>(block)), args, static_cast<size_t>(lds), s);
}

hipError_t launch_yuv420_lanczos(const LanczosDev &ly, const Io &ioY, const LanczosDev &lc, const Io &ioU,
                                 const Io &ioV, hipStream_t s)
{
    if (ioY.frames <= 0)
        return hipSuccess;
    if (ioY.frames != ioU.frames || ioU.frames != ioV.frames)
        return hipErrorInvalidValue;
    Prep<LanczosArgs> py, pu, pv;
    hipError_t e;
    LanczosDev lyGrid = ly;
    lyGrid.stack = 0;  // the fused launch has one (band, frame) grid for all three planes
    lyGrid.tail = -1;
    if ((e = prep_lanczos(lyGrid, ioY, 0, ly.dstH, 0, &py)) != hipSuccess ||
        (e = prep_lanczos(lc, ioU, 0, lc.dstH, 0, &pu)) != hipSuccess ||
        (e = prep_lanczos(lc, ioV, 0, lc.dstH, 0, &pv)) != hipSuccess)
        return e;
    // chroma: the ring instantiation at the default depth; Y: a symmetric streamer at K = 4 whose
    // blocks are 256 threads (block-shared only with exactly 4 waves per row)
    if (pu.kind != 0 || lc.NY != 4 || pu.pd != 3 || py.kind == 0 || py.pd < 3)
        return hipErrorNotSupported;
    const bool one = (ly.cy[0] & 0xffffu) == 1u;
    // (4 waves per row: >= 1488 outputs, so the Y body always takes the line edge scheme)
    const bool shared = py.kind == 1 && py.block == 256 && py.a.chunks <= 4 && symb_line(py.a.l.dstW, py.a.np);
    const void *kern = nullptr;
    if (ly.NY == 10 && one)
        kern = shared ? reinterpret_cast<const void *>(yuv420_lanczos_kernel<SymbY<10, 12, -5, true, true>, RingChroma>)
                      : reinterpret_cast<const void *>(yuv420_lanczos_kernel<SymY<10, 12, -5, true>, RingChroma>);
    else if (ly.NY == 8)
        kern = shared ? reinterpret_cast<const void *>(yuv420_lanczos_kernel<SymbY<8, 8, -3, false, true>, RingChroma>)
                      : reinterpret_cast<const void *>(yuv420_lanczos_kernel<SymY<8, 8, -3, false>, RingChroma>);
    else
        return hipErrorNotSupported;
    if (!shared && py.kind == 1) {
        // re-prepare Y as the per-wave symmetric streamer (256-thread blocks of 4 waves)
        LanczosDev l2 = lyGrid;
        l2.sym = 2;
        if ((e = prep_lanczos(l2, ioY, 0, ly.dstH, 0, &py)) != hipSuccess)
            return e;
    }
    // the symmetric Y bodies need their LDS: dynamic for the block-shared body, static otherwise
    return launch_fused3(kern, py, pu, pv, 256, shared ? py.lds : 0, s);
}

hipError_t launch_yuv420_area(const AreaDev &gy, const Io &ioY, const AreaDev &gc, const Io &ioU, const Io &ioV,
                              hipStream_t s)
{
    if (ioY.frames <= 0)
        return hipSuccess;
    if (ioY.frames != ioU.frames || ioU.frames != ioV.frames)
        return hipErrorInvalidValue;
    Prep<AreaArgs> py, pu, pv;
    (void)prep_area(gy, ioY, 0, gy.dstH, &py);
    (void)prep_area(gc, ioU, 0, gc.dstH, &pu);
    (void)prep_area(gc, ioV, 0, gc.dstH, &pv);
    if (py.kind != pu.kind || (py.kind >= 2 && py.kind != 5 && py.kind != 8 && gy.KY != gc.KY))
        return hipErrorNotSupported;
    static const void *const kerns[kAreaKinds] = {
        reinterpret_cast<const void *>(yuv420_plane_kernel<AreaPlane<4, 4>, AreaArgs>),
        reinterpret_cast<const void *>(yuv420_plane_kernel<AreaPlane<2, 2>, AreaArgs>),
        reinterpret_cast<const void *>(yuv420_plane_kernel<AreaPlane<2, 0>, AreaArgs>),
        reinterpret_cast<const void *>(yuv420_plane_kernel<AreaPlane<4, 0>, AreaArgs>),
        reinterpret_cast<const void *>(yuv420_plane_kernel<AreaPlane<8, 0>, AreaArgs>),
        reinterpret_cast<const void *>(yuv420_plane_kernel<AreaPlane<3, 3>, AreaArgs>),
        reinterpret_cast<const void *>(yuv420_plane_kernel<AreaPlane<3, 0>, AreaArgs>),
        reinterpret_cast<const void *>(yuv420_plane_kernel<AreaPlane<6, 0>, AreaArgs>),
        reinterpret_cast<const void *>(yuv420_plane_kernel<LinearD2Plane, AreaArgs>)};
    return launch_fused3(kerns[py.kind], py, pu, pv, 256, 0, s);
}

hipError_t launch_yuv420_linear(const LinearDev &gy, const Io &ioY, const LinearDev &gc, const Io &ioU,
                                const Io &ioV, hipStream_t s)
{
    if (ioY.frames <= 0)
        return hipSuccess;
    if (ioY.frames != ioU.frames || ioU.frames != ioV.frames)
        return hipErrorInvalidValue;
    Prep<LinearArgs> py, pu, pv;
    hipError_t e;
    if ((e = prep_linear(gy, ioY, 0, gy.dstH, 0, &py)) != hipSuccess ||
        (e = prep_linear(gc, ioU, 0, gc.dstH, 0, &pu)) != hipSuccess ||
        (e = prep_linear(gc, ioV, 0, gc.dstH, 0, &pv)) != hipSuccess)
        return e;
    if (py.kind != 1 || pu.kind != 1 || py.pd != 2 || pu.pd != 2 || gy.F != 2 || gc.F != 2)
        return hipErrorNotSupported;
    return launch_fused3(reinterpret_cast<const void *>(yuv420_plane_kernel<LinearPlane, LinearArgs>), py, pu, pv,
                         256, 0, s);
}

} // namespace iqo_amd
