// kernels_ratio.hip -- gfx950 kernels for the exact- and general-ratio shapes (2x / 3x / 2:3 / 3:2 / 3:1,
// exact vertical ratios, general rows): kernels.hip's arithmetic (the reference's Generic fixed
// point) on register windows with the phases compiled in or tabled.
#include "kernels_dev.hpp"

namespace iqo_amd {
namespace {

// ================================================================ exact 2x / 3x Lanczos upscale
//
// (3x, F = 3: output F k + j takes phase j; phase 0 is the single tap, phases 1 and 2 both take NT
// taps from k + 1 - NT/2.  A lane owns the same 8 source columns and 24 output columns, a source
// step yields F output rows, and the edge lanes park 24 sums per row.  1280x720 -> 3840x2160.)
//
// Lanczos-2/3 at exactly 2x (plan.cpp build_up2).  In the reference's tables for this ratio an
// even output row / column sits exactly on a source sample (a single tap: 64 vertically, 2^14
// horizontally) and an odd one takes NT = 2 * degree taps starting NT/2 - 1 samples to its left
// (IQOLanczosResizerImpl_Generic.cpp:144-190, 404-454), at the borders too (masked + renormalised,
// :464-490, :539-574).  The linear_up2 streamer's layout: one WAVE per (row band, output strip,
// frame) walks the band's SOURCE rows top to bottom; lane l (1..np) owns source columns
// [cb, cb + 8) and output columns [2cb, 2cb + 16), lanes 0 and np+1 are the halo.
//
// Every source row is loaded once per band (8 B per lane, NT rows ahead) and widened to four u16
// pairs in a register window of NT rows (static names: the loop is unrolled NT times).  Source
// step k yields output rows 2k (one packed multiply per pair) and 2k+1 (NT packed MACs), the
// coefficient splats in SGPRs.  The horizontal pass needs work columns [cb - 3, cb + 11): the two
// pairs either side come from the neighbouring lanes by DPP, odd-aligned pairs by v_alignbit;
// output 2cb + j is one (j even) or NT/2 (j odd) v_dot2_i32_i16 on pairs chosen at compile time.
// Sixteen outputs pack into one 16-B store per lane.  Arithmetic as everywhere: int16-wrapping
// vertical pass, (s + 2^19) >> 20 saturated to u8.
//
// Borders: source rows and columns outside the image load as zero, so the same sums are the
// reference's masked numerators.  A border row's work pairs are divided by its denominator
// (int16(n * 64 / deno), magic_y) before the horizontal pass; border columns lie in the first /
// last lane of a row, which parks its 16 sums in LDS, and once per trip (2 NT rows) lanes
// 0 .. 2NT-1 rewrite those 16 bytes of one row each with the exact division (magic_x constants,
// identity 2^20 for the lane's interior columns).

struct Up2Args {
    Up2Dev u;
    Io io;
    int rowBegin, rowEnd, rowsPerBand, bands, wavesPerRow, np;
    int srcBytes, dstBytes;
    unsigned nWaves;
};

template <int NT, int F>
__global__ __launch_bounds__(256) void lanczos_up2_kernel(Up2Args a)
{
    constexpr int NW = NT;           // register window rows
    constexpr int H = NT / 2;        // coefficient pairs of a phase 1 .. F-1 output
    constexpr int OFF = 1 - NT / 2;  // window start relative to x / F (y / F)
    constexpr int OPL = 8 * F;       // output columns per lane
    constexpr int OOB = 0x7ff00000;
    const Up2Dev &u = a.u;
    // the rounding bias in a VGPR, the first dot's third operand (sdot2_sv)
    const int bias = static_cast<int>(opaque(1u << 19));
    __shared__ int4 park[4][2][F * NW][OPL / 4];  // per wave, side, row slot: the edge lane's raw sums
    __shared__ __attribute__((aligned(16))) uint8_t stage[F == 3 ? 4 * 2048 : 16];  // 3x: store_row24
    const int lane = static_cast<int>(threadIdx.x) & 63;
    const int wib = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    const unsigned gw = xcd_chunks(blockIdx.x, (a.bands * a.wavesPerRow + 3) / 4, gridDim.x) * 4u + static_cast<unsigned>(wib);
    if (gw >= a.nWaves)
        return;  // whole wave; no barrier in this kernel
    const int wcol = static_cast<int>(gw % static_cast<unsigned>(a.wavesPerRow));
    const unsigned rest = gw / static_cast<unsigned>(a.wavesPerRow);
    const int band = static_cast<int>(rest % static_cast<unsigned>(a.bands));
    const int frame = static_cast<int>(rest / static_cast<unsigned>(a.bands));
    const int y0 = a.rowBegin + band * a.rowsPerBand;
    const int y1 = min(y0 + a.rowsPerBand, a.rowEnd);
    if (y0 >= y1)
        return;

    const int opw = OPL * a.np;
    const int x0 = max(0, min(wcol * opw, u.dstW - opw));  // first output column of lane 1
    const int cb = x0 / F - 8 + 8 * lane;
    const bool produce = lane >= 1 && lane <= a.np;
    const int voff = (lane <= a.np + 1 && cb >= 0 && cb + 8 <= u.srcW) ? cb : OOB;
    const int stoff = produce ? F * cb : OOB;
    const bool edgeL = x0 == 0, edgeR = x0 + opw >= u.dstW;  // wave holds border columns (uniform)
    const bool laneL = edgeL && lane == 1, laneR = edgeR && lane == a.np;

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(frame) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(frame) * a.io.dstFrameSt;
    const __amdgpu_buffer_rsrc_t srcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcFrame), 0, a.srcBytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0, dstRow0 = a.io.dstRow0;

    // source steps k: output rows F k .. F k + F - 1 (those outside [y0, y1) are computed and dropped);
    // step k reads source rows k + OFF .. k + OFF + NT - 1.  Rows outside the image read as zero
    // (the masked border sums); rows of dropped outputs may lie outside the call's window: clamped
    // (never used).  Out-of-range marks go in the (range-checked) VGPR offset.
    const int kLo = y0 / F, kHi = (y1 + F - 1) / F;
    const int rFirst = kLo + OFF;
    const int rLast = kHi - 1 + OFF + NT - 1;
    const int srcLast = a.io.srcRowEnd - 1;
    auto load_row = [&](int r) -> u32x2 {
        const int rc = min(max(r, srcRow0), srcLast);
        const bool in = r >= 0 && r < u.srcH && r >= rFirst && r <= rLast;
        return __builtin_amdgcn_raw_buffer_load_b64(srcR, voff + (in ? (rc - srcRow0) * srcSt : OOB), 0, 0);
    };
    // Odd bands walk bottom-up (round 4, as lanczos_d32_kernel): the halo rows two
    // neighbouring bands share are then read by both at the same time, and the second read hits
    // L2.  Walk row t is source row rFirst + t top-down, rLast - t bottom-up; step j holds walk rows
    // j .. j + NT - 1 in both walks, so walking up, step j (k = kHi - 1 - j) finds tap i of the odd
    // output at walk row j + NT - 1 - i (the taps reversed: c1 below) and the even output's source
    // row k at walk row j + NT - 1 + OFF instead of j - OFF.
    const bool up = band & 1;
    const int wBase = up ? rLast : rFirst, wStep = up ? -1 : 1;
    auto walk_row = [&](int t) { return wBase + wStep * t; };
    uint32_t c1[F - 1][NT];  // phase 1 .. F-1 taps in walk order (SGPR selects, once per band)
#pragma unroll
    for (int j = 0; j < F - 1; ++j)
#pragma unroll
        for (int i = 0; i < NT; ++i)
            c1[j][i] = up ? u.cy1[j][NT - 1 - i] : u.cy1[j][i];
    auto widen = [&](u32x2 v, uint32_t (&P)[4]) {
        P[0] = __builtin_amdgcn_perm(0u, v.x, 0x0c010c00u);  // (cb, cb+1)
        P[1] = __builtin_amdgcn_perm(0u, v.x, 0x0c030c02u);
        P[2] = __builtin_amdgcn_perm(0u, v.y, 0x0c010c00u);
        P[3] = __builtin_amdgcn_perm(0u, v.y, 0x0c030c02u);  // (cb+6, cb+7)
    };
    // one lane's OPL bytes of row y: one 16-B store (F = 2), 16 + 8 B (F = 3)
    auto store_row = [&](const uint32_t (&o)[OPL / 4], int voffs, int y, bool ok) {
        const int off = voffs + (ok ? (y - dstRow0) * dstSt : OOB);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{o[0], o[1], o[2], o[3]}, dstR, off, 0,
                                               2 /* nt: fresh data G2 0.088 vs 0.1015 ms */);
        if constexpr (F == 3)
            __builtin_amdgcn_raw_buffer_store_b64(u32x2{o[4], o[5]}, dstR, off + 16, 0, 2);
    };
    // masked border row (uniform, rare): work = int16(n * 64 / deno)
    auto border_row = [&](uint32_t (&W)[4], int y) {
        if (y < u.m0 || y >= u.m1) {
            const int side = y < u.m0 ? 0 : 1, i = min(max(side ? y - u.m1 : y, 0), 15);
            const uint32_t m = u.yM[side][i];
            const int sh = u.yS[side][i];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                W[q] = ydiv2(W[q], m, sh);
        }
    };
    // horizontal pass + store of output row y from the lane's four work pairs
    auto emit = [&](const uint32_t (&Wk)[4], int y, int slot) {
        uint32_t E[8];  // E[e] = work columns (cb - 4 + 2e, cb - 3 + 2e)
        E[0] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(Wk[2]), 0x138 /* wave_shr:1 */, 0xf, 0xf, true));
        E[1] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(Wk[3]), 0x138, 0xf, 0xf, true));
        E[2] = Wk[0];
        E[3] = Wk[1];
        E[4] = Wk[2];
        E[5] = Wk[3];
        E[6] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(Wk[0]), 0x130 /* wave_shl:1 */, 0xf, 0xf, true));
        E[7] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(Wk[1]), 0x130, 0xf, 0xf, true));
        uint32_t O[7];  // O[e] = work columns (cb - 3 + 2e, cb - 2 + 2e)
#pragma unroll
        for (int e = 0; e < 7; ++e)
            O[e] = __builtin_amdgcn_alignbit(E[e + 1], E[e], 16);
        auto pair = [&](int rel) { return (rel & 1) ? O[(rel - 1) / 2] : E[rel / 2]; };  // low half = column rel
        int sum[OPL];
#pragma unroll
        for (int j = 0; j < OPL; ++j) {
            const int m = j / F, ph = j % F;  // output F (cb + m) + ph
            if (ph == 0) {
                // on a source column: c * w[cb + m] (the pair's high half meets a zero coefficient)
                sum[j] = sdot2_sv(pair(m + 4), u.cx0, bias);
            } else {
                const int rel = m + OFF + 4;
                int acc = sdot2_sv(pair(rel), u.cx1[ph - 1][0], bias);
#pragma unroll
                for (int q = 1; q < H; ++q)
                    acc = sdot2(pair(rel + 2 * q), u.cx1[ph - 1][q], acc);
                sum[j] = acc;
            }
        }
        uint32_t o[OPL / 4];
#pragma unroll
        for (int q = 0; q < OPL / 4; ++q)
            o[q] = pack_hi(pack_lo(sum[4 * q], sum[4 * q + 1]), sum[4 * q + 2], sum[4 * q + 3]);
        if constexpr (F == 3)
            store_row24<2>(stage + 2048 * wib, o, produce, lane, 24 * a.np, dstR,
                           y >= y0 && y < y1 ? x0 + (y - dstRow0) * dstSt : OOB);
        else
            store_row(o, stoff, y, y >= y0 && y < y1);
        if (edgeL || edgeR) {  // uniform
            if (laneL || laneR) {
                int4 *pk = park[wib][laneL ? 0 : 1][slot];
#pragma unroll
                for (int q = 0; q < OPL / 4; ++q)
                    pk[q] = make_int4(sum[4 * q], sum[4 * q + 1], sum[4 * q + 2], sum[4 * q + 3]);
            }
        }
    };
    // once per trip: lane r < F NW rewrites the edge bytes of row yt + r from the parked sums
    auto flush = [&](int yt) {
        uint32_t oL[OPL / 4] = {}, oR[OPL / 4] = {};
        const int r = min(lane, F * NW - 1);
        if (edgeL || edgeR) {  // uniform
            __builtin_amdgcn_wave_barrier();
            auto fix = [&](int side, uint32_t (&w)[OPL / 4]) {
#pragma unroll
                for (int q = 0; q < OPL / 4; ++q) {
                    const int4 p = park[wib][side][r][q];
                    const int sv[4] = {p.x, p.y, p.z, p.w};
                    uint32_t b[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        b[e] = min(__umulhi(static_cast<uint32_t>(max(sv[e], 0)), u.xM[side][4 * q + e]) >>
                                       u.xT[side][4 * q + e],
                                   255u);
                    w[q] = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
                }
            };
            if (edgeL)
                fix(0, oL);
            if (edgeR)
                fix(1, oR);
        }
        const int y = yt + lane;
        const bool ok = lane < F * NW && y >= y0 && y < y1;
        store_row(oL, edgeL ? 0 : OOB, y, ok);
        store_row(oR, edgeR ? u.dstW - OPL : OOB, y, ok);
    };
    const uint32_t zeros[OPL / 4] = {};

    uint32_t R[NW][4];
    // the window of step 0 without its newest row: walk rows 0 .. NT - 2 -> slots 0 .. NT - 2
#pragma unroll
    for (int i = 0; i < NT - 1; ++i)
        widen(load_row(walk_row(i)), R[i]);
    // prefetch: step v adds walk row NT - 1 + v (slot (v + NT - 1) % NW)
    u32x2 pre[NW];
#pragma unroll
    for (int v = 0; v < NW; ++v) {
        __builtin_amdgcn_sched_barrier(0);
        pre[v] = load_row(walk_row(NT - 1 + v));
        // the loop's store pattern (F rows per step), dropped, so the header waits are steady-state
#pragma unroll
        for (int j = 0; j < F; ++j)
            store_row(zeros, OOB, 0, false);
    }
    // and the trip's two flush rows
    store_row(zeros, OOB, 0, false);
    store_row(zeros, OOB, 0, false);
    const int nSteps = kHi - kLo;
    for (int base = 0; base < nSteps; base += NW) {
        static_for<NW>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            const int j = base + v;                      // walk step
            if (j >= nSteps)
                return;  // past the band's last step (uniform; the trip's flush still runs)
            const int k = up ? kHi - 1 - j : kLo + j;    // source step: output rows F k .. F k + F - 1
            const int slot = up ? F * (NW - 1 - v) : F * v;  // park slots: row F k - (the trip's lowest row)
            __builtin_amdgcn_sched_barrier(0);
            widen(pre[v], R[(v + NT - 1) % NW]);  // walk row j + NT - 1
            pre[v] = load_row(walk_row(j + NW + NT - 1));
            uint32_t Wk[4];
            // output row F k: the source row k itself (both candidate rows through opaque(): a plain
            // select of the two let the compiler index the window dynamically, i.e. put it in
            // scratch -- 2 to 3x slower, round 5)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t ru = opaque(R[(v + NT - 1 + OFF) % NW][q]), rd = opaque(R[(v - OFF) % NW][q]);
                Wk[q] = pk_mul(up ? ru : rd, u.cy0);
            }
            border_row(Wk, F * k);
            emit(Wk, F * k, slot);
#pragma unroll
            for (int ph = 1; ph < F; ++ph) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {  // output row F k + ph: walk rows j .. j + NT - 1
                    uint32_t acc = pk_mul(R[v % NW][q], c1[ph - 1][0]);
#pragma unroll
                    for (int i = 1; i < NT; ++i)
                        acc = pk_mad(R[(v + i) % NW][q], c1[ph - 1][i], acc);
                    Wk[q] = acc;
                }
                border_row(Wk, F * k + ph);
                emit(Wk, F * k + ph, slot + ph);
            }
        });
        flush(up ? F * (kHi - NW - base) : F * (kLo + base));
    }
}

// ================================================================ exact 3:2 Lanczos-3 downscale
//
// Lanczos-3 at exactly 2/3 (e.g. 1920x1080 -> 1280x720; plan.cpp build_d32).  In the reference's
// tables for this ratio output y takes the 10 taps of phase y & 1 starting at source row
// 3 (y >> 1) - 4 + (y & 1) (IQOLanczosResizerImpl_Generic.cpp:144-190 tables, :404-454 row loop),
// and the same for columns.  Rows come in groups m = (2m, 2m + 1) over the 10 source rows
// 3m - 4 .. 3m + 5; the even row's non-zero taps are group rows 0..7, the odd row's 2..9, and each
// group adds the 3 source rows 3m + 3 .. 3m + 5.  One WAVE per (row band, output strip, frame)
// walks the band's groups top to bottom, no barrier:
//
// * lane l (1..np) owns output columns [x0 + 8(l-1), +8) and source columns [cb, cb + 12),
//   cb = 3/2 x0 - 12 + 12 l; lanes 0 and np+1 are the halo.  Each source row is loaded once per
//   band (12 B per lane, PD groups ahead, branch-free so the compiler's vm waits are exact) and
//   widened to six u16 pairs in a register window of 12 rows (static names: 4 groups per trip).
// * Vertical: 8 v_pk_mad_u16 per pair and output row (int16 wrap as the reference's work row).
// * Horizontal: work columns cb - 4 .. cb + 15 (two pairs from each neighbour by DPP, odd-aligned
//   pairs by v_alignbit); output j is 5 v_dot2_i32_i16 on pairs fixed at compile time.
// * Border columns (masked, renormalised: :539-574) lie in the first / last lane of a row.  Source
//   columns outside the image load as zero, so the dot products give the reference's masked
//   numerators; the edge lane parks its 8 sums in LDS and once per trip (8 rows) lanes 0..7
//   rewrite those 8 bytes of one row each with the exact division (host multiply-high constants,
//   identity 2^20 for the lane's interior columns).
// * Border rows (masked, renormalised: :464-490): source rows outside the image load as zero, so
//   the window sum is the masked numerator; the row's work pairs are divided by its denominator
//   (int16(n * 64 / deno), magic_y multiply-high) before the horizontal pass.
struct D32Args {
    D32Dev d;
    Io io;
    int rowBegin, rowEnd;   // output rows of this launch (main rows)
    int evenBegin;          // rowBegin & ~1: band b starts at evenBegin + b * rowsPerBand (even)
    int rowsPerBand, bands, wavesPerRow, np;
    int srcBytes, dstBytes;
    unsigned nWaves;
};

// Tap structure (plan.cpp build_d32): group m's window is source rows 3m + GA .. 3m + GA + GW - 1;
// the even row's NTY taps start at group row 0, the odd row's at group row PO1; output column x
// takes NPX coefficient pairs from column 3 (x >> 1) + BX0 + (x & 1).  Lanczos-3: <-4, 10, 8, 2,
// 5, -4>; Lanczos-2: <-2, 7, 5, 2, 3, -2>.
template <int PD, int GA, int GW, int NTY, int PO1, int NPX, int BX0>
__global__ __launch_bounds__(256) void lanczos_d32_kernel(D32Args a)
{
    constexpr int NW = (GW + 2) / 3 * 3;  // register window rows (a multiple of the 3 rows a group adds)
    constexpr int U = NW / 3;             // groups per unrolled trip (window slots repeat)
    static_assert(GW >= 3 && NTY <= 8 && NPX <= 5 && PO1 + NTY == GW, "tap structure (mirror-symmetric)");
    static_assert(BX0 >= -4 && 9 + BX0 + 1 + 2 * NPX - 1 <= 15, "column windows within the lane's work pairs");
    constexpr int OOB = 0x7ff00000;
    static_assert(U % PD == 0, "prefetch slots repeat within a trip");
    const D32Dev &d = a.d;
    __shared__ int4 park[4][2][8][2];  // per wave, side, row slot: the edge lane's 8 raw sums
    const int lane = static_cast<int>(threadIdx.x) & 63;
    const int wib = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    const unsigned gw = xcd_chunks(blockIdx.x, (a.bands * a.wavesPerRow + 3) / 4, gridDim.x) * 4u + static_cast<unsigned>(wib);
    if (gw >= a.nWaves)
        return;  // whole wave; no barrier in this kernel
    const int wcol = static_cast<int>(gw % static_cast<unsigned>(a.wavesPerRow));
    const unsigned rest = gw / static_cast<unsigned>(a.wavesPerRow);
    const int band = static_cast<int>(rest % static_cast<unsigned>(a.bands));
    const int frame = static_cast<int>(rest / static_cast<unsigned>(a.bands));
    const int yb = a.evenBegin + band * a.rowsPerBand;  // even: first row of group kLo
    const int y0 = max(yb, a.rowBegin), y1 = min(yb + a.rowsPerBand, a.rowEnd);
    if (y0 >= y1)
        return;
    const int kLo = yb >> 1;
    const int nG = (y1 - yb + 1) >> 1;  // groups of this band (dropped rows at either end)
    // Odd bands walk bottom-up: the halo rows two neighbouring bands share are then read
    // by both at the same time (both at their ends, or both at their starts) and the second read
    // hits L2 instead of HBM.  Walking up, relative row q is source row rLast - q and group g is
    // group kLo + nG - 1 - g; group row x of the forward walk is window row GW - 1 - x, so with
    // PO1 + NTY = GW the first output of a group (window rows 0 .. NTY-1) is the odd row with the
    // odd phase's taps reversed and the second (rows PO1 ..) the even row with the even taps reversed.
    const bool up = band & 1;
    const int mTop = kLo + nG - 1;

    const int opw = 8 * a.np;
    const int x0 = max(0, min(wcol * opw, d.dstW - opw));
    const int cb = (3 * x0) / 2 - 12 + 12 * lane;
    const bool produce = lane >= 1 && lane <= a.np;
    const int voff = (lane <= a.np + 1 && cb >= 0 && cb + 12 <= d.srcW) ? cb : OOB;
    const int stoff = produce ? x0 + 8 * (lane - 1) : OOB;
    const bool edgeL = x0 == 0, edgeR = x0 + opw >= d.dstW;  // wave holds border columns (uniform)
    const bool laneL = edgeL && lane == 1, laneR = edgeR && lane == a.np;

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(frame) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(frame) * a.io.dstFrameSt;
    const __amdgpu_buffer_rsrc_t srcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcFrame), 0, a.srcBytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0, dstRow0 = a.io.dstRow0;

    // relative source row q = row rBase + q; rows outside the image read as zero (the masked
    // border sums); rows of dropped outputs may lie outside the call's window: clamped (their
    // values are never used); rows past the band's last group are not loaded.  Out-of-range marks
    // go in the (range-checked) VGPR offset.
    const int rBase = 3 * kLo + GA;
    const int rLast = 3 * (kLo + nG - 1) + GA + GW - 1;
    const int srcLast = a.io.srcRowEnd - 1;
    auto load_row = [&](int q) -> u32x3 {
        const int r = up ? rLast - q : rBase + q;
        const int rc = min(max(r, srcRow0), srcLast);
        const bool in = r >= 0 && r < d.srcH && (up ? r >= rBase : r <= rLast);
        return __builtin_amdgcn_raw_buffer_load_b96(srcR, voff + (in ? (rc - srcRow0) * srcSt : OOB), 0, 0);
    };
    auto widen = [&](u32x3 v, uint32_t (&P)[6]) {
        P[0] = __builtin_amdgcn_perm(0u, v.x, 0x0c010c00u);  // (cb, cb+1)
        P[1] = __builtin_amdgcn_perm(0u, v.x, 0x0c030c02u);
        P[2] = __builtin_amdgcn_perm(0u, v.y, 0x0c010c00u);
        P[3] = __builtin_amdgcn_perm(0u, v.y, 0x0c030c02u);
        P[4] = __builtin_amdgcn_perm(0u, v.z, 0x0c010c00u);
        P[5] = __builtin_amdgcn_perm(0u, v.z, 0x0c030c02u);  // (cb+10, cb+11)
    };
    auto store_row = [&](u32x2 o, int voffs, int y, bool ok) {
        __builtin_amdgcn_raw_buffer_store_b64(o, dstR, voffs + (ok ? (y - dstRow0) * dstSt : OOB), 0, 0);
    };
    // horizontal pass of one output row from the lane's six work pairs; the edge lane parks its sums
    auto emit = [&](const uint32_t (&W)[6], int y, int slot) {
        uint32_t E[10];  // E[e] = work columns (cb - 4 + 2e, cb - 3 + 2e)
        E[0] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(W[4]), 0x138 /* wave_shr:1 */, 0xf, 0xf, true));
        E[1] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(W[5]), 0x138, 0xf, 0xf, true));
#pragma unroll
        for (int e = 0; e < 6; ++e)
            E[e + 2] = W[e];
        E[8] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(W[0]), 0x130 /* wave_shl:1 */, 0xf, 0xf, true));
        E[9] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(W[1]), 0x130, 0xf, 0xf, true));
        uint32_t O[9];  // O[e] = work columns (cb - 3 + 2e, cb - 2 + 2e)
#pragma unroll
        for (int e = 0; e < 9; ++e)
            O[e] = __builtin_amdgcn_alignbit(E[e + 1], E[e], 16);
        auto pair = [&](int rel) { return (rel & 1) ? O[(rel + 3) / 2] : E[(rel + 4) / 2]; };  // low half = column cb + rel
        int sum[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int ph = j & 1;
            const int rel = 3 * (j >> 1) + BX0 + ph;  // window start of output x0 + 8(l-1) + j
            int acc = sdot2_sv(pair(rel), d.cx[ph][0], 1 << 19);
#pragma unroll
            for (int q = 1; q < NPX; ++q)
                acc = sdot2(pair(rel + 2 * q), d.cx[ph][q], acc);
            sum[j] = acc;
        }
        u32x2 o;
        o.x = pack_hi(pack_lo(sum[0], sum[1]), sum[2], sum[3]);
        o.y = pack_hi(pack_lo(sum[4], sum[5]), sum[6], sum[7]);
        store_row(o, stoff, y, y >= y0 && y < y1);
        if (edgeL || edgeR) {  // uniform
            if (laneL || laneR) {
                int4 *pk = park[wib][laneL ? 0 : 1][slot];
                pk[0] = make_int4(sum[0], sum[1], sum[2], sum[3]);
                pk[1] = make_int4(sum[4], sum[5], sum[6], sum[7]);
            }
        }
    };
    // once per trip: lane r < 2U rewrites the edge bytes of row yt + r (walking up: yt - r) from
    // the parked sums
    auto flush = [&](int yt) {
        u32x2 oL = {0u, 0u}, oR = {0u, 0u};
        if (edgeL || edgeR) {  // uniform
            __builtin_amdgcn_wave_barrier();
            auto fix = [&](int side) {
                const int4 p0 = park[wib][side][lane & 7][0], p1 = park[wib][side][lane & 7][1];
                const int sv[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
                uint32_t b[8];
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    b[j] = min(__umulhi(static_cast<uint32_t>(max(sv[j], 0)), d.xM[side][j]) >> d.xT[side][j], 255u);
                return u32x2{b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24), b[4] | (b[5] << 8) | (b[6] << 16) | (b[7] << 24)};
            };
            if (edgeL)
                oL = fix(0);
            if (edgeR)
                oR = fix(1);
        }
        const int y = up ? yt - lane : yt + lane;
        const bool ok = lane < 2 * U && y >= y0 && y < y1;
        store_row(oL, edgeL ? 0 : OOB, y, ok);
        store_row(oR, edgeR ? d.dstW - 8 : OOB, y, ok);
    };

    // masked border row (uniform, rare): work = int16(n * 64 / deno)
    auto border_row = [&](uint32_t (&W)[6], int y) {
        if (y < d.m0 || y >= d.m1) {
            const int side = y < d.m0 ? 0 : 1, i = min(max(side ? y - d.m1 : y, 0), 7);
            const uint32_t m = d.yM[side][i];
            const int sh = d.yS[side][i];
#pragma unroll
            for (int c = 0; c < 6; ++c)
                W[c] = ydiv2(W[c], m, sh);
        }
    };

    // the two outputs' taps in walk order (uniform: SGPRs)
    uint32_t cA[NTY], cB[NTY];
#pragma unroll
    for (int t = 0; t < NTY; ++t) {
        cA[t] = up ? d.cy[1][NTY - 1 - t] : d.cy[0][t];
        cB[t] = up ? d.cy[0][NTY - 1 - t] : d.cy[1][t];
    }
    uint32_t R[NW][6];
    // the window of group 0 without the rows group 0 itself adds: relative rows 0 .. GW-4 -> slots
#pragma unroll
    for (int q = 0; q < GW - 3; ++q)
        widen(load_row(q), R[q]);
    // prefetch: group g adds relative rows 3g + GW - 3 .. 3g + GW - 1 (slots mod NW)
    u32x3 pre[PD][3];
#pragma unroll
    for (int v = 0; v < PD; ++v) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 3; ++i)
            pre[v][i] = load_row(3 * v + GW - 3 + i);
        // the loop's store pattern (two rows per group), dropped, so the header waits are steady-state
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, dstR, OOB, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, dstR, OOB, 0, 0);
    }
    // and the trip's two flush stores
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, dstR, OOB, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, dstR, OOB, 0, 0);
    for (int base = 0; base < nG; base += U) {
        static_for<U>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            const int g = base + v;
            if (g >= nG)
                return;  // past the band's last group (uniform; the trip's flush still runs)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 3; ++i)
                widen(pre[v % PD][i], R[(3 * v + GW - 3 + i) % NW]);
#pragma unroll
            for (int i = 0; i < 3; ++i)
                pre[v % PD][i] = load_row(3 * (g + PD) + GW - 3 + i);
            const int yA = up ? 2 * (mTop - g) + 1 : 2 * (kLo + g), yB = up ? yA - 1 : yA + 1;
            uint32_t W[6];
#pragma unroll
            for (int c = 0; c < 6; ++c)
                W[c] = pk_mul(R[(3 * v) % NW][c], cA[0]);
#pragma unroll
            for (int t = 1; t < NTY; ++t)
#pragma unroll
                for (int c = 0; c < 6; ++c)
                    W[c] = pk_mad(R[(3 * v + t) % NW][c], cA[t], W[c]);
            border_row(W, yA);
            emit(W, yA, 2 * v);
#pragma unroll
            for (int c = 0; c < 6; ++c)
                W[c] = pk_mul(R[(3 * v + PO1) % NW][c], cB[0]);
#pragma unroll
            for (int t = 1; t < NTY; ++t)
#pragma unroll
                for (int c = 0; c < 6; ++c)
                    W[c] = pk_mad(R[(3 * v + PO1 + t) % NW][c], cB[t], W[c]);
            border_row(W, yB);
            emit(W, yB, 2 * v + 1);
        });
        flush(up ? 2 * (mTop - base) + 1 : 2 * (kLo + base));
    }
}

// ================================================================ exact 3:1 Lanczos-2/3 downscale
//
// Lanczos-3 (Lanczos-2) at exactly 1/3 (e.g. 3840x2160 -> 1280x720, 1920x1080 -> 640x360;
// plan.cpp build_d31).  The reference's tables for this ratio have one phase: 18 (12) taps,
// window start 3y - 8 (3y - 5), tap 0 zero and taps 1.. symmetric about the centre
// (IQOLanczosResizerImpl_Generic.cpp:144-190 tables, :404-454 row loop, :582-612 columns).  One WAVE
// per (row band, output strip, frame) walks the band's rows top to bottom, no barrier:
//
// * lane l (1..np) owns output columns [x0 + 4(l-1), +4) and source columns [cb, cb + 12),
//   cb = 3 x0 - 12 + 12 l; lanes 0 and np+1 are the halo.  Each source row is loaded once per band
//   (12 B per lane, PD output rows ahead, branch-free so the compiler's vm waits are exact) and
//   widened to six u16 pairs in a register window of NW rows (static names: U = NW / 3 output rows
//   per trip, each adding 3 source rows).
// * Vertical: the symmetric taps pair up -- the window's centre row times its coefficient plus
//   NPY pair sums (s[CEN - d] + s[CEN + d], <= 510 per u16 half, one full-rate v_add_u32 for both
//   halves) times theirs, packed MACs whose low 16 bits are the reference's int16 wrap.
// * Horizontal: work columns cb + EB .. cb + EB + 2 NE - 1 as u16 pairs E[e] (the outer ones from
//   the neighbouring lanes by DPP); output j's window starts at cb + XS + 3j: an even start takes
//   the pairs from its start with coefficient pairs (c0, c1), (c2, c3), ..; an odd start skips
//   tap 0 (zero in these tables) and takes the pairs from start + 1 with (c1, c2), (c3, c4), .. --
//   every pair aligned, no v_alignbit.
// * Borders as lanczos_d32_kernel: source rows / columns outside the image load as zero, so the
//   sums are the reference's masked numerators (:464-490, :539-574); masked border rows divide their
//   work pairs (int16(n * 64 / deno), magic_y); the <= 4 border columns per side lie in the edge
//   lane, which parks its 4 raw sums in LDS, and once per trip lanes 0..U-1 rewrite one row's 4
//   edge bytes each with the exact division.
struct D31Args {
    D31Dev d;
    Io io;
    int rowBegin, rowEnd, rowsPerBand, bands, wavesPerRow, np;
    int srcBytes, dstBytes;
    unsigned nWaves;
};

// tap structure per variant: window rows NR (start 3y + YA), centre row CEN, pair distances, work
// pairs E (first column EB, count NE, NL from each neighbour), column window start XS (tap 0), and
// coefficient pairs per output NPX
template <int VAR>
struct D31Shape;
template <>
struct D31Shape<0> {  // Lanczos-3: 18 taps, non-zero taps 2..16, centre 9
    static constexpr int NR = 15, YA = -6, CEN = 7, NPY = 5;
    static constexpr int DIST[5] = {1, 2, 4, 5, 7};
    static constexpr int EB = -8, NE = 14, NL = 4, XS = -8, NPX = 9;
};
template <>
struct D31Shape<1> {  // Lanczos-2: 12 taps, non-zero taps 1..11, centre 6
    static constexpr int NR = 11, YA = -4, CEN = 5, NPY = 4;
    static constexpr int DIST[5] = {1, 2, 4, 5, 0};
    static constexpr int EB = -4, NE = 10, NL = 2, XS = -5, NPX = 6;
};

template <int PD, int VAR>
__global__ __launch_bounds__(256) void lanczos_d31_kernel(D31Args a)
{
    using S = D31Shape<VAR>;
    constexpr int NW = (S::NR + 2) / 3 * 3;  // register window rows (whole groups of 3)
    constexpr int U = NW / 3;                // output rows per unrolled trip (window slots repeat)
    constexpr int OOB = 0x7ff00000;
    constexpr int OWN = -S::EB / 2;          // E index of the lane's own pair 0
    static_assert(U % PD == 0, "prefetch slots repeat within a trip");
    static_assert(OWN - S::NL >= 0 && OWN + 6 + S::NL == S::NE, "work pairs: NL from each neighbour");
    static_assert(2 * S::CEN == S::NR - 1, "window symmetric about its centre row (bottom-up bands)");
    const D31Dev &d = a.d;
    __shared__ int4 park[4][2][8];  // per wave, side, row slot: the edge lane's 4 raw sums
    const int lane = static_cast<int>(threadIdx.x) & 63;
    const int wib = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    const unsigned gw = xcd_chunks(blockIdx.x, (a.bands * a.wavesPerRow + 3) / 4, gridDim.x) * 4u + static_cast<unsigned>(wib);
    if (gw >= a.nWaves)
        return;  // whole wave; no barrier in this kernel
    const int wcol = static_cast<int>(gw % static_cast<unsigned>(a.wavesPerRow));
    const unsigned rest = gw / static_cast<unsigned>(a.wavesPerRow);
    const int band = static_cast<int>(rest % static_cast<unsigned>(a.bands));
    const int frame = static_cast<int>(rest / static_cast<unsigned>(a.bands));
    const int y0 = a.rowBegin + band * a.rowsPerBand;
    const int y1 = min(y0 + a.rowsPerBand, a.rowEnd);
    if (y0 >= y1)
        return;
    const int nR = y1 - y0;
    // odd bands walk bottom-up (as lanczos_d32_kernel): the window is symmetric about its
    // centre row (2 CEN = NR - 1), so walking up is the same arithmetic on the rows in reverse
    const bool up = band & 1;

    const int opw = 4 * a.np;
    const int x0 = max(0, min(wcol * opw, d.dstW - opw));
    const int cb = 3 * x0 - 12 + 12 * lane;
    const bool produce = lane >= 1 && lane <= a.np;
    const int voff = (lane <= a.np + 1 && cb >= 0 && cb + 12 <= d.srcW) ? cb : OOB;
    const int stoff = produce ? x0 + 4 * (lane - 1) : OOB;
    const bool edgeL = x0 == 0, edgeR = x0 + opw >= d.dstW;  // wave holds border columns (uniform)
    const bool laneL = edgeL && lane == 1, laneR = edgeR && lane == a.np;

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(frame) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(frame) * a.io.dstFrameSt;
    const __amdgpu_buffer_rsrc_t srcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcFrame), 0, a.srcBytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0, dstRow0 = a.io.dstRow0;

    // relative row q = source row rBase + q (output y0 + v reads relative rows 3v .. 3v + NR - 1);
    // rows outside the image read as zero (the masked border sums), rows past the band's last
    // output are not loaded, rows outside the call's window are clamped (never used)
    const int rBase = 3 * y0 + S::YA;
    const int rLast = 3 * (y1 - 1) + S::YA + S::NR - 1;
    const int srcLast = a.io.srcRowEnd - 1;
    auto load_row = [&](int q) -> u32x3 {
        const int r = up ? rLast - q : rBase + q;
        const int rc = min(max(r, srcRow0), srcLast);
        const bool in = r >= 0 && r < d.srcH && (up ? r >= rBase : r <= rLast);
        return __builtin_amdgcn_raw_buffer_load_b96(srcR, voff + (in ? (rc - srcRow0) * srcSt : OOB), 0, 0);
    };
    auto widen = [&](u32x3 v, uint32_t (&P)[6]) {
        P[0] = __builtin_amdgcn_perm(0u, v.x, 0x0c010c00u);  // (cb, cb+1)
        P[1] = __builtin_amdgcn_perm(0u, v.x, 0x0c030c02u);
        P[2] = __builtin_amdgcn_perm(0u, v.y, 0x0c010c00u);
        P[3] = __builtin_amdgcn_perm(0u, v.y, 0x0c030c02u);
        P[4] = __builtin_amdgcn_perm(0u, v.z, 0x0c010c00u);
        P[5] = __builtin_amdgcn_perm(0u, v.z, 0x0c030c02u);  // (cb+10, cb+11)
    };
    auto store_row = [&](uint32_t o, int voffs, int y, bool ok) {
        __builtin_amdgcn_raw_buffer_store_b32(o, dstR, voffs + (ok ? (y - dstRow0) * dstSt : OOB), 0, 0);
    };
    // horizontal pass of one output row from the lane's six work pairs; the edge lane parks its sums
    auto emit = [&](const uint32_t (&W)[6], int y, int slot) {
        uint32_t E[S::NE];
#pragma unroll
        for (int e = 0; e < S::NL; ++e)
            E[e] = static_cast<uint32_t>(
                __builtin_amdgcn_mov_dpp(static_cast<int>(W[6 - S::NL + e]), 0x138 /* wave_shr:1 */, 0xf, 0xf, true));
#pragma unroll
        for (int e = 0; e < 6; ++e)
            E[OWN + e] = W[e];
#pragma unroll
        for (int e = 0; e < S::NL; ++e)
            E[OWN + 6 + e] = static_cast<uint32_t>(
                __builtin_amdgcn_mov_dpp(static_cast<int>(W[e]), 0x130 /* wave_shl:1 */, 0xf, 0xf, true));
        int sum[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            constexpr int dummy = 0;
            (void)dummy;
            const int st = S::XS + 3 * j;           // window start (tap 0) relative to cb
            const bool odd = (st & 1) != 0;
            const int e0 = ((odd ? st + 1 : st) - S::EB) / 2;
            int acc = sdot2_sv(E[e0], odd ? d.cxo[0] : d.cxe[0], 1 << 19);
#pragma unroll
            for (int q = 1; q < S::NPX; ++q)
                acc = sdot2(E[e0 + q], odd ? d.cxo[q] : d.cxe[q], acc);
            sum[j] = acc;
        }
        store_row(pack_hi(pack_lo(sum[0], sum[1]), sum[2], sum[3]), stoff, y, y >= y0 && y < y1);
        if (edgeL || edgeR) {  // uniform
            if (laneL || laneR)
                park[wib][laneL ? 0 : 1][slot] = make_int4(sum[0], sum[1], sum[2], sum[3]);
        }
    };
    // once per trip: lane r < U rewrites the 4 edge bytes of row yt + r (walking up: yt - r) from
    // the parked sums
    auto flush = [&](int yt) {
        uint32_t oL = 0u, oR = 0u;
        if (edgeL || edgeR) {  // uniform
            __builtin_amdgcn_wave_barrier();
            auto fix = [&](int side) {
                const int4 p = park[wib][side][lane & 7];
                const int sv[4] = {p.x, p.y, p.z, p.w};
                uint32_t b[4];
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    b[j] = min(__umulhi(static_cast<uint32_t>(max(sv[j], 0)), d.xM[side][j]) >> d.xT[side][j], 255u);
                return b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
            };
            if (edgeL)
                oL = fix(0);
            if (edgeR)
                oR = fix(1);
        }
        const int y = up ? yt - lane : yt + lane;
        const bool ok = lane < U && y >= y0 && y < y1;
        store_row(oL, edgeL ? 0 : OOB, y, ok);
        store_row(oR, edgeR ? d.dstW - 4 : OOB, y, ok);
    };
    // masked border row (uniform, rare): work = int16(n * 64 / deno)
    auto border_row = [&](uint32_t (&W)[6], int y) {
        if (y < d.m0 || y >= d.m1) {
            const int side = y < d.m0 ? 0 : 1, i = min(max(side ? y - d.m1 : y, 0), 7);
            const uint32_t m = d.yM[side][i];
            const int sh = d.yS[side][i];
#pragma unroll
            for (int c = 0; c < 6; ++c)
                W[c] = ydiv2(W[c], m, sh);
        }
    };

    uint32_t R[NW][6];
    // the window of output y0 without its newest 3 rows: relative rows 0 .. NW-4 -> slots 0 .. NW-4
#pragma unroll
    for (int q = 0; q < NW - 3; ++q)
        widen(load_row(q), R[q]);
    // prefetch: output y0 + v adds relative rows 3v + NW-3 .. 3v + NW-1 (slots mod NW)
    u32x3 pre[PD][3];
#pragma unroll
    for (int v = 0; v < PD; ++v) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 3; ++i)
            pre[v][i] = load_row(3 * v + NW - 3 + i);
        // the loop's store pattern (one row per step), dropped, so the header waits are steady-state
        __builtin_amdgcn_raw_buffer_store_b32(0u, dstR, OOB, 0, 0);
    }
    // and the trip's two flush stores
    __builtin_amdgcn_raw_buffer_store_b32(0u, dstR, OOB, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(0u, dstR, OOB, 0, 0);
    for (int base = 0; base < nR; base += U) {
        static_for<U>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            const int g = base + v;
            if (g >= nR)
                return;  // past the band's last group (uniform; the trip's flush still runs)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 3; ++i)
                widen(pre[v % PD][i], R[(3 * v + NW - 3 + i) % NW]);
#pragma unroll
            for (int i = 0; i < 3; ++i)
                pre[v % PD][i] = load_row(3 * (g + PD) + NW - 3 + i);
            // window row w of this output is slot (3v + w) mod NW
            uint32_t W[6];
#pragma unroll
            for (int c = 0; c < 6; ++c)
                W[c] = pk_mul(R[(3 * v + S::CEN) % NW][c], d.cc);
#pragma unroll
            for (int k = 0; k < S::NPY; ++k)
#pragma unroll
                for (int c = 0; c < 6; ++c)
                    W[c] = pk_mad(R[(3 * v + S::CEN - S::DIST[k]) % NW][c] + R[(3 * v + S::CEN + S::DIST[k]) % NW][c],
                                  d.cp[k], W[c]);
            const int y = up ? y1 - 1 - g : y0 + g;
            border_row(W, y);
            emit(W, y, v);
        });
        flush(up ? y1 - 1 - base : y0 + base);
    }
}

// ================================================================ exact vertical ratio, any horizontal ratio
//
// Downscales whose rows follow an exact ratio P:Q but whose columns do not (1920x1080 -> 854x480:
// rows 9:4, columns 960:427, 427 column phases).  plan.cpp build_ryx.  One WORKGROUP (8 waves) per
// (row band, frame), the whole width:
//
// * Vertical: thread t owns source columns [4t, 4t + 4) (one dword per row) and walks the band's
//   rows with a register window of NW source rows widened to u16 pairs (static names: U groups of Q
//   output rows per trip, each group adding P rows, loaded one group ahead).  Output y = Q m + j
//   takes phase j's taps from window row floor(P j / Q) (IQOLanczosResizerImpl_Generic.cpp:404-454
//   / IQOAreaResizerImpl_Generic.cpp:271-293 row loops): packed MACs, 16-bit wrap; masked Lanczos
//   border rows (rows outside the image load as zero) are divided in place (:464-490).
// * The work row goes to LDS (u16, zero padding either side, double-buffered: one barrier per row).
// * Horizontal: thread t computes output columns t and half + t of its part from the table (one
//   column apart in neighbouring lanes: the work-row reads spread over the LDS banks; 4:1 also
//   rotates the reads of lanes 16-31 of each half by one pair): NP coefficient pairs in VGPRs for
//   the whole band, NP dword reads from the work row at the column's even window start, v_dot2
//   (:582-612 / :340-368); Lanczos columns end in an exact multiply-high division (the identity
//   2^20 in the interior, the border divisor of :539-574 at the edges); one byte store per column.
struct RyxArgs {
    RyxDev d;
    Io io;
    int rowBegin, rowEnd, groupBegin, rowsPerBand, bands;
    int srcBytes, dstBytes;
    unsigned nBlocks;
};

#ifndef IQO_RYX_WPE
#define IQO_RYX_WPE 4  // waves per SIMD the register budget is sized for (variant builds: 5)
#endif
#ifndef IQO_RYX_UC_PD
#define IQO_RYX_UC_PD 2  // Lanczos-8 / -9 2:1 with uniform columns: row groups loaded ahead
#endif
#ifndef IQO_RYX_WPE_WIDE
#define IQO_RYX_WPE_WIDE 2  // ... for windows of more than 20 rows: Lanczos-8 / -9 2:1 spill at 4 (steady clock, 4K 2:1
                            // x128: Lanczos-8 1.154 -> 0.533 ms, Lanczos-9 1.822 -> 0.567, profiles/r05/steady_check2.txt)
#endif
template <bool LZ, int P, int Q, int T, int NP, int PD, bool ADJ, int CPT, bool UC = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(T > 20 && !UC ? IQO_RYX_WPE_WIDE : IQO_RYX_WPE))) void ryx_kernel(RyxArgs a)
{
    static_assert(CPT % 2 == 0 && (!ADJ || CPT == 2), "output columns per thread: pairs");
    static_assert(!UC || !(P == 4 && Q == 1), "uniform columns: no rotated reads");
    // adjacent pairs at 2:1 columns (round 5): the second column's window always starts one pair
    // after the first's, so one run of NP + 1 pairs serves both (NP + 1 LDS dwords instead of 2 NP)
    constexpr bool ADJ2 = ADJ && P == 2 && Q == 1;
    constexpr int SPAN = (P * (Q - 1)) / Q + T;   // window rows of one group of Q outputs
    constexpr int NW0 = (SPAN + P - 1) / P * P;   // register window rows (whole groups of P) ...
    constexpr int NW = ((NW0 / P) * Q) % 2 ? NW0 + P : NW0;  // ... and an even number of rows per trip
    constexpr int U = NW / P;                     // groups per unrolled trip (window slots repeat)
    constexpr int UQ = U * Q;                     // output rows per trip
    constexpr int OOB = 0x7ff00000;
    constexpr int PADB = 2 * kRyxPadK;            // work-row byte padding left of column 0
    static_assert(U % PD == 0, "prefetch slots repeat within a trip");
    static_assert(UQ % 2 == 0, "work-row buffer parity is static within a trip");
    // the next row's vertical pass overlaps this row's LDS reads when the read registers fit
    // beside the window (NP 10 would spill at 4 waves per SIMD)
    constexpr bool PIPE = NP <= 8 || NW <= 18;
    const RyxDev &d = a.d;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int t = static_cast<int>(threadIdx.x);
    const unsigned blk0 = xcd_chunks(blockIdx.x, a.bands * d.parts, gridDim.x);
    if (blk0 >= a.nBlocks)
        return;  // whole workgroup
    // column part (d.parts workgroups per row), then band, then frame
    const int part = static_cast<int>(blk0 % static_cast<unsigned>(d.parts));
    const unsigned blk = blk0 / static_cast<unsigned>(d.parts);
    const int cLo = d.parts > 1 ? d.cs[part] : 0, cHi = d.parts > 1 ? d.ce[part] : d.srcW;
    const int xLo = d.parts > 1 ? d.xs[part] : 0, xHi = d.parts > 1 ? d.xs[part + 1] : d.dstW;
    const int band = static_cast<int>(blk % static_cast<unsigned>(a.bands));
    const int frame = static_cast<int>(blk / static_cast<unsigned>(a.bands));
    const int yb = a.groupBegin + band * a.rowsPerBand;  // a multiple of Q: first row of group mLo
    const int y0 = max(yb, a.rowBegin), y1 = min(yb + a.rowsPerBand, a.rowEnd);
    if (y0 >= y1)
        return;  // whole workgroup
    const int mLo = yb / Q;
    const int nG = (y1 - yb + Q - 1) / Q;

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(frame) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(frame) * a.io.dstFrameSt;
    const __amdgpu_buffer_rsrc_t srcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcFrame), 0, a.srcBytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0, dstRow0 = a.io.dstRow0;
#ifndef IQO_RYX_EXP
#define IQO_RYX_EXP 0  // timing experiments (variant builds, wrong output): 1 no source loads, 2 no stores,
                       // 3 no barriers
#endif
    const int span = cHi - cLo;  // this workgroup's source columns [cLo, cHi), 4 per thread
    // a source width that is not a multiple of 4 (round 5): the thread straddling the row end loads
    // the dword ending at the last column and the byte selectors shift it down, so it never reads past the row and its
    // columns past the end are zero (the masked border taps)
    const int vsh = 4 * t < span ? max(0, cLo + 4 * t + 4 - d.srcW) : 0;
    const int voff = 4 * t < span && IQO_RYX_EXP != 1 ? cLo + 4 * t - vsh : OOB;
    // upscales: waves with no source columns (480 threads over 160 source dwords) skip the
    // vertical pass and its loads (uniform per wave; not at the downscales, where every wave has
    // source columns and the branch costs Lanczos-3 4:1 its prefetch: 0.36 -> 0.82 ms)
    const bool srcWave = Q <= P || 256 * __builtin_amdgcn_readfirstlane(t >> 6) < span;

    // work rows: two buffers of (pad + span + pad) u16, zero padding written once
    const int spanA = (span + 3) & ~3;  // (the last thread's dword, zero past the row end)
    const int pitch = PADB + 2 * spanA + PADB;
    for (int i = t; i < 2 * (PADB / 4); i += static_cast<int>(blockDim.x)) {
        const int buf = i / (PADB / 4), k = i % (PADB / 4);
        *reinterpret_cast<uint32_t *>(lds + buf * pitch + 4 * k) = 0u;
        *reinterpret_cast<uint32_t *>(lds + buf * pitch + PADB + 2 * spanA + 4 * k) = 0u;
    }
    // this thread's two output columns: table entries for the whole band
    // Thread t owns output columns xLo + t and xLo + half + t: neighbouring lanes read windows
    // one output column apart, so the work-row reads spread over the LDS banks (columns 2t, 2t + 1
    // put 4:1 lanes 16 B apart: 8-way bank conflicts, 56 % of the LDS cycles; 9:4 44 %)
    // ADJ (column ratio >= 2, ryx_dev checks every pair): thread t owns the adjacent columns
    // xLo + 2t, xLo + 2t + 1, whose windows start 1 or 2 pairs apart: one run of NP + 2 dwords
    // serves both (10 reads instead of 16 at NP 8), the second column's pairs padded to NP + 1
    // CPT > 2 (upscales, ryx_dev d.cpt): columns xLo + t + k half, k < CPT
    const int half = ADJ ? 1 : (xHi - xLo + CPT - 1) / CPT;
    int xc[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k)
        xc[k] = ADJ ? xLo + 2 * t + k : xLo + k * half + t;
    constexpr int NC1 = ADJ && !ADJ2 ? NP + 1 : NP;  // coefficient pairs of the second column
    uint32_t cf[CPT][NC1];
    int aoff[CPT];
    uint32_t mm[CPT];
    int sh[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        const int x = min(xc[k], xHi - 1);
        const int4 c = d.cols[x];
        aoff[k] = c.x - 2 * cLo;  // work-row byte offset relative to this part's first column
        mm[k] = static_cast<uint32_t>(c.y);
        sh[k] = c.z;
#pragma unroll
        for (int q = 0; q < NP; ++q)
            cf[k][q] = UC ? static_cast<uint32_t>(sld(reinterpret_cast<const int *>(d.colCoef), q)) : d.colCoef[x * NP + q];
    }
    // 4:1: neighbouring lanes' windows are 2 dwords apart, so lanes t and t + 16 of a 32-lane half
    // meet on one bank (ds_read_b32 / ds_read2: bank = dword mod 32).  Lanes 16-31 of each half read
    // their window rotated by one pair (pair q + 1 first, pair 0 last): every read of a half then
    // touches 32 distinct banks.  The coefficient pairs are rotated the same way, once.
    constexpr bool ROT = P == 4 && Q == 1;
    const int rot = ROT ? (t >> 4) & 1 : 0;
    int aoffB[CPT];  // byte offset of the last pair read (aoff[k] + 4 rot + 4 q for the others)
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        if constexpr (ROT) {
            const uint32_t c0 = cf[k][0];
#pragma unroll
            for (int q = 0; q < NP; ++q)
                cf[k][q] = rot ? (q + 1 < NP ? cf[k][q + 1] : c0) : cf[k][q];
        }
        aoffB[k] = rot ? aoff[k] : aoff[k] + 4 * (NP - 1);
        aoff[k] += 4 * rot;
    }
    // ADJ2: reads start at the 8-byte boundary at or before the first column's window (base8);
    // adjS = 1 when the window starts one dword after it (uniform: every 2:1 window has the same
    // parity; lanes past xHi, clamped to the last column, may differ and store nothing)
    const int base8 = ADJ2 ? aoff[0] & ~7 : 0;
    const int adjS = ADJ2 ? (__builtin_amdgcn_readfirstlane(aoff[0]) >> 2) & 1 : 0;
    uint32_t cfA[ADJ2 ? NP + 1 : 1];  // (uniform: scalar registers)
    if constexpr (ADJ2) {
#pragma unroll
        for (int q = 0; q <= NP; ++q)
            cfA[q] = adjS ? (q ? cf[0][q - 1] : 0u) : (q < NP ? cf[0][q] : 0u);
    }
    if constexpr (ADJ && !ADJ2) {  // (ADJ2: the second column's pairs are the first's, one pair later)
        const bool two = aoff[1] - aoff[0] == 8;  // else 4 (the pair's last thread past xHi: unused)
#pragma unroll
        for (int q = NP; q >= 1; --q)
            cf[1][q] = two ? cf[1][q - 1] : q < NP ? cf[1][q] : 0u;
        cf[1][0] = two ? 0u : cf[1][0];
    }
    // interior Lanczos columns divide by 2^20 (magic_x: m = 2^31, shift 19), which is one
    // saturating pack of both columns; only the few border columns take the exact division
    bool edgeAny = false;
#pragma unroll
    for (int k = 0; k < CPT; ++k)
        edgeAny = edgeAny || mm[k] != 0x80000000u || sh[k] != 19;
    // (wave-uniform: the exact division of a border column equals the saturating pack on an interior
    // one, so a wave holding any border column takes it for all its lanes -- no divergent branch)
    const bool edgeT = LZ && __builtin_amdgcn_ballot_w64(edgeAny) != 0;
    // one byte store per column (a wave stores 64 consecutive bytes per instruction)
    int stoff[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k)
        stoff[k] = (ADJ || t < half) && xc[k] < xHi && IQO_RYX_EXP != 2 ? xc[k] : OOB;

    // relative row q = source row rBase + q; group g's window = relative rows P g .. P g + SPAN - 1.
    // Rows outside the image load as zero (the reference's masked border sums); rows past the
    // band's last window are not loaded.  Rows outside the call's source window (band windows) can
    // only be rows no stored output reads, and read as zero (out-of-range offsets).
    const int rBase = P * mLo + d.off;
    const int rLast = P * (mLo + nG - 1) + d.off + SPAN - 1;
    const int qLo = max(0, -rBase), qHi = min(d.srcH - 1, rLast) - rBase;
    const int rowOff0 = (rBase - srcRow0) * srcSt;
    auto load_row = [&](int q) -> uint32_t {
        const bool in = static_cast<unsigned>(q - qLo) <= static_cast<unsigned>(qHi - qLo);
        return __builtin_amdgcn_raw_buffer_load_b32(srcR, voff + (in ? rowOff0 + q * srcSt : OOB), 0, 0);
    };
    // (the straddling thread's shift is folded into the byte selectors: a selector byte 4 .. 6 picks
    // a byte of the zero operand, so columns past the row end widen to zero with no extra VALU)
    const uint32_t selLo = 0x0c010c00u + 0x00010001u * static_cast<uint32_t>(vsh);
    const uint32_t selHi = 0x0c030c02u + 0x00010001u * static_cast<uint32_t>(vsh);
    auto widen = [&](uint32_t v, uint32_t (&W)[2]) {
        W[0] = __builtin_amdgcn_perm(0u, v, selLo);
        W[1] = __builtin_amdgcn_perm(0u, v, selHi);
    };

    uint32_t R[NW][2];
#pragma unroll
    for (int q = 0; q < SPAN - P; ++q)
        widen(load_row(q), R[q]);
    uint32_t pre[PD][P];
#pragma unroll
    for (int v = 0; v < PD; ++v)
#pragma unroll
        for (int i = 0; i < P; ++i)
            pre[v][i] = load_row(SPAN - P + P * v + i);

    // group g (window slot base v = g mod U) brings its P new rows into the window and issues the
    // loads of group g + PD
    auto enter_group = [&](auto vc, int g) {
        constexpr int v = decltype(vc)::value;
#pragma unroll
        for (int i = 0; i < P; ++i)
            widen(pre[v % PD][i], R[(P * v + SPAN - P + i) % NW]);
#pragma unroll
        for (int i = 0; i < P; ++i)
            pre[v % PD][i] = load_row(SPAN - P + P * (g + PD) + i);
    };
    // vertical pass of output row Q (mLo + g) + j into work buffer B: phase j's taps from window
    // row floor(P j / Q) (scalar loads of the splats), packed MACs, 16-bit wrap; masked Lanczos
    // border rows are divided in place
    // (the splats arrive in cy, loaded before the barrier that precedes the pass: scalar loads
    // share the lgkm counter with the LDS reads, and waiting for them after the barrier would
    // also wait for the row's LDS reads)
    // Lanczos 2:1 (one phase, symmetric window: plan.cpp build_ryx checks it): mirrored rows are
    // summed first (widened bytes: <= 510 per half, one v_add_u32 for both halves), then one packed
    // MAC per pair -- T / 2 MACs and T / 2 adds instead of T MACs; the low 16 bits of
    // c (a + b) are those of c a + c b, the reference's int16 wrap
    constexpr bool SYMV = LZ && (P == 2 || P == 4) && Q == 1;  // (round 5: 4:1 too)
    constexpr int TC = SYMV ? T / 2 : T;  // row coefficients the pass reads
    static_assert(!SYMV || T % 2 == 0, "symmetric 2:1 windows have an even tap count");
    auto coefs = [&](auto jc, uint32_t (&cy)[TC]) {
        constexpr int j = decltype(jc)::value;
#pragma unroll
        for (int k = 0; k < TC; ++k)
            cy[k] = static_cast<uint32_t>(sld(d.rowCoef, j * T + k));
    };
    auto vertical = [&](auto vc, auto jc, auto bc, int g, const uint32_t (&cy)[TC]) {
        constexpr int v = decltype(vc)::value, j = decltype(jc)::value, B = decltype(bc)::value;
        constexpr int S0 = (P * j) / Q;
        const int y = Q * (mLo + g) + j;
        uint32_t W[2] = {0u, 0u};
        if constexpr (SYMV) {
#pragma unroll
            for (int k = 0; k < TC; ++k) {
                const int ra = (P * v + S0 + k) % NW, rb = (P * v + S0 + T - 1 - k) % NW;
                W[0] = pk_mad(R[ra][0] + R[rb][0], cy[k], W[0]);
                W[1] = pk_mad(R[ra][1] + R[rb][1], cy[k], W[1]);
            }
        } else {
#pragma unroll
            for (int k = 0; k < T; ++k) {
                W[0] = pk_mad(R[(P * v + S0 + k) % NW][0], cy[k], W[0]);
                W[1] = pk_mad(R[(P * v + S0 + k) % NW][1], cy[k], W[1]);
            }
        }
        if (LZ && static_cast<unsigned>(y - d.m0) >= static_cast<unsigned>(d.m1 - d.m0)) {
            // masked border row (uniform, rare): rows outside the image read as zero
            const int side = y < d.m0 ? 0 : 1, i = min(max(side ? y - d.m1 : y, 0), 15);
            W[0] = ydiv2(W[0], d.yM[side][i], d.yS[side][i]);
            W[1] = ydiv2(W[1], d.yM[side][i], d.yS[side][i]);
        }
        if (4 * t < span)
            *reinterpret_cast<uint2 *>(lds + B * pitch + PADB + 8 * t) = make_uint2(W[0], W[1]);
    };

    // prologue: group 0's rows, output row 0 into buffer 0
    enter_group(std::integral_constant<int, 0>{}, 0);
    {
        uint32_t cy0[TC];
        coefs(std::integral_constant<int, 0>{}, cy0);
        vertical(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, 0,
                 cy0);
    }

    // Row r of a trip (group base + r / Q, phase r % Q): the barrier publishes its work row
    // (written one iteration earlier); its NP-pair windows are read from LDS, and while those
    // reads are in flight the thread computes the vertical pass of row r + 1 into the other buffer
    // (every read of that buffer, row r - 1, completed before the barrier); then the dots
    // (without PIPE the next row's vertical pass comes after the dots).
    for (int base = 0; base < nG; base += U) {
        static_for<UQ>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            constexpr int v = r / Q, j = r % Q, B = r & 1;
            const int g = base + v;
            if (g >= nG)
                return;  // whole workgroup
            constexpr int rn = (r + 1) % UQ, vn = rn / Q, jn = rn % Q;
            uint32_t cyn[TC];  // the next row's splats, complete at the barrier
            coefs(std::integral_constant<int, jn>{}, cyn);
            if (IQO_RYX_EXP != 3)  // experiment 3: no barrier (timing only)
                lds_barrier();
            const uint8_t *wr = lds + B * pitch;
            // window pair q of column k: w[k][q] (ADJ: one run, the second column from pair 1)
            constexpr int NR = ADJ2 ? 2 * ((NP + 3) / 2) : ADJ ? NP + 2 : NP;
            static_assert(!ADJ2 || NR >= NP + 2, "the run holds both columns' windows at either start");
            uint32_t w[ADJ ? 1 : CPT][NR];
            if constexpr (ADJ2) {
                // 8-byte aligned ds_read_b64 from the pair boundary at or before the window: lanes
                // 8 bytes apart, no bank conflicts (4-byte reads 2 dwords apart conflicted 2-way,
                // and some lanes at wave edges then read stale outer taps, profiles/r05/adj_race.txt)
                const uint2 *run = reinterpret_cast<const uint2 *>(__builtin_assume_aligned(wr + base8, 8));
#pragma unroll
                for (int q = 0; q < NR / 2; ++q) {
                    const uint2 v = run[q];
                    w[0][2 * q] = v.x;
                    w[0][2 * q + 1] = v.y;
                }
            } else if constexpr (ADJ) {
#pragma unroll
                for (int q = 0; q < NR; ++q)
                    w[0][q] = reinterpret_cast<const uint32_t *>(wr + aoff[0])[q];
            } else {
#pragma unroll
                for (int k = 0; k < CPT; ++k)
#pragma unroll
                    for (int q = 0; q < NP; ++q)
                        w[k][q] = q + 1 < NP ? reinterpret_cast<const uint32_t *>(wr + aoff[k])[q]
                                             : *reinterpret_cast<const uint32_t *>(wr + aoffB[k]);
            }
            auto wq = [&](int k, int q) -> uint32_t { return ADJ ? w[0][k + q] : w[k][q]; };
            // ADJ2: the two columns' sums over NP + 1 run pairs with the shifted coefficients cfA
            // (column k's window starts at run pair k + adjS)
            int acc2[2] = {0, 0};
            if constexpr (ADJ2) {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    acc2[k] = sdot2_vv(w[0][k], cfA[0], 1 << 19);
#pragma unroll
                    for (int q = 1; q <= NP; ++q)
                        acc2[k] = sdot2(w[0][k + q], cfA[q], acc2[k]);
                }
            }
            // the next row's vertical pass (the next trip's first row after the trip's last)
            auto next_vertical = [&]() {
                const int gn = base + (r + 1) / Q;
                if (gn < nG && srcWave) {
                    if constexpr (jn == 0)
                        enter_group(std::integral_constant<int, vn>{}, gn);
                    vertical(std::integral_constant<int, vn>{}, std::integral_constant<int, jn>{},
                             std::integral_constant<int, B ^ 1>{}, gn, cyn);
                }
            };
            if constexpr (PIPE)
                next_vertical();
            // horizontal: the thread's two columns
            const int y = Q * (mLo + g) + j;
            uint32_t packed[CPT / 2];  // bytes of columns 2i, 2i + 1 in the low half
            if constexpr (LZ) {
                int acc[CPT];
#pragma unroll
                for (int k = 0; k < CPT; ++k) {
                    if constexpr (ADJ2) {
                        acc[k] = acc2[k];
                        continue;
                    }
                    acc[k] = sdot2_vv(wq(k, 0), cf[k][0], 1 << 19);
#pragma unroll
                    for (int q = 1; q < (k ? NC1 : NP); ++q)
                        acc[k] = sdot2(wq(k, q), cf[k][q], acc[k]);
                }
#pragma unroll
                for (int i = 0; i < CPT / 2; ++i) {
                    if (edgeT) {
                        const uint32_t o0 =
                            min(__umulhi(static_cast<uint32_t>(max(acc[2 * i], 0)), mm[2 * i]) >> sh[2 * i], 255u);
                        const uint32_t o1 =
                            min(__umulhi(static_cast<uint32_t>(max(acc[2 * i + 1], 0)), mm[2 * i + 1]) >> sh[2 * i + 1], 255u);
                        packed[i] = opaque(o0) | (opaque(o1) << 8);
                    } else {
                        packed[i] = pack_lo(acc[2 * i], acc[2 * i + 1]);  // sat_u8(acc >> 20) of both columns
                    }
                }
            } else {
                int o[CPT];
#pragma unroll
                for (int k = 0; k < CPT; ++k) {
                    uint32_t acc = 1u << 22;
#pragma unroll
                    for (int q = 0; q < (k ? NC1 : NP); ++q)
                        acc = udot2(wq(k, q), cf[k][q], acc);
                    const uint16_t u = static_cast<uint16_t>(static_cast<int16_t>(static_cast<int>(acc) >> 23));
                    o[k] = u > 255 ? 255 : u;
                }
#pragma unroll
                for (int i = 0; i < CPT / 2; ++i)
                    packed[i] = opaque(static_cast<uint32_t>(o[2 * i])) | (opaque(static_cast<uint32_t>(o[2 * i + 1])) << 8);
            }
            const bool ok = y >= y0 && y < y1;
            const int rowOff = ok ? (y - dstRow0) * dstSt : OOB;
#pragma unroll
            for (int k = 0; k < CPT; ++k)
                __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(packed[k / 2] >> (8 * (k & 1))), dstR,
                                                     stoff[k] + rowOff, 0, 0);
            if constexpr (!PIPE)
                next_vertical();
        });
    }
}

// ================================================================ general-row ratio kernel
//
// ryx_kernel's layout for downscales whose rows shrink by more than 1 and at most 2 with no small
// exact ratio (plan.cpp build_ryg), e.g. 1080 -> 768 rows (45:32) or 1080 -> 576 (15:8), which
// otherwise run the wave walker.  One workgroup per (row band, frame, column part); thread = 4 source
// columns.  Output row y has a record {first window row s(y), offset of its phase's taps}
// (IQO*ResizerImpl_Generic.cpp's row driver: LinearIterator source row and y mod rDst phase,
// Lanczos :369-454, Area :250-294; masked Lanczos border rows :464-490 divided in place as in
// ryx_kernel).  The thread's register window R holds rows s(y) .. s(y) + T - 1 widened to u16
// pairs at FIXED names: moving to row y + 1 shifts it by s(y+1) - s(y), 1 or 2 rows (a uniform
// branch with register moves), and the incoming rows come from a FIFO of raw dwords loaded PD
// output rows ahead -- always the last two rows of that row's window, so every output row issues
// exactly two loads (branch-free memory stream, exact vmcnt waits; when the window moves by one row
// the first of the two is the row the previous pair brought, an L2 hit).  The window is a RING of T
// slots (round 5: fixed names shifted by register moves cost ~40 v_mov per row): window row k of
// output y sits in slot (o(y) + k) mod T, o advancing with the window; one uniform switch on o picks
// a copy of the row step with static slot names, which widens the two incoming rows into their
// slots (when the window moves by one row the first lands on the equal row already there) and runs
// the vertical pass.  Vertical: T packed MACs per u16 pair; horizontal, LDS work rows, the next
// row's vertical pass under this row's LDS reads, column tables and stores: as ryx_kernel with CPT
// output columns per thread.
struct RygArgs {
    RygDev d;
    Io io;
    int rowBegin, rowEnd, rowsPerBand, bands;
    int srcBytes, dstBytes;
    unsigned nBlocks;
};

// (occupancy: two 512-thread workgroups per CU up to 22 row taps -- at 22 the compiler spills a few
// registers and the kernel is still 5.5 % faster than at one workgroup per CU, 4K -> 1024x576
// profiles/r05/steady_ryg_wpe.txt; 24 taps and Lanczos-4's 16 column pairs stay at one)
template <bool LZ, int T, int NP, int PD, int CPT, int NL>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(T > 22 || NP > 13 ? 2 : 4))) void ryg_kernel(RygArgs a)
{
    static_assert(CPT >= 2 && CPT <= 4, "output columns per thread");
    static_assert(NL >= 1 && NL <= 4, "rows loaded per output row: 1 (upscales), 2 .. 4 (down to 2:1 .. 4:1)");
    constexpr int NPK = (CPT + 1) / 2;  // packed column pairs (an odd CPT: the last pair repeats its column)
    constexpr int OOB = 0x7ff00000;
    constexpr int PADB = 2 * kRyxPadK;  // work-row byte padding left of column 0
    static_assert(PD % 2 == 0 && T >= 2, "the unrolled trip covers both work-row buffers");
    const RygDev &d = a.d;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int t = static_cast<int>(threadIdx.x);
    // (xcd_spread here: the chunk map of the other kernels was 3.8 % slower on 1080p -> 1366x768,
    // profiles/r06/xcd_chunks.txt)
    const unsigned blk0 = xcd_spread(blockIdx.x, gridDim.x);
    if (blk0 >= a.nBlocks)
        return;  // whole workgroup
    const int part = static_cast<int>(blk0 % static_cast<unsigned>(d.parts));
    const unsigned blk = blk0 / static_cast<unsigned>(d.parts);
    const int cLo = d.parts > 1 ? d.cs[part] : 0, cHi = d.parts > 1 ? d.ce[part] : d.srcW;
    const int xLo = d.parts > 1 ? d.xs[part] : 0, xHi = d.parts > 1 ? d.xs[part + 1] : d.dstW;
    const int band = static_cast<int>(blk % static_cast<unsigned>(a.bands));
    const int frame = static_cast<int>(blk / static_cast<unsigned>(a.bands));
    const int y0 = a.rowBegin + band * a.rowsPerBand, y1 = min(y0 + a.rowsPerBand, a.rowEnd);
    if (y0 >= y1)
        return;  // whole workgroup
    const int nRows = y1 - y0;

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(frame) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(frame) * a.io.dstFrameSt;
    const __amdgpu_buffer_rsrc_t srcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcFrame), 0, a.srcBytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0, dstRow0 = a.io.dstRow0;
    const int span = cHi - cLo;
    // (a source width that is not a multiple of 4: as ryx_kernel, the straddling thread's dword ends
    // at the last column and is shifted down)
    const int vsh = 4 * t < span ? max(0, cLo + 4 * t + 4 - d.srcW) : 0;
    const int voff = 4 * t < span ? cLo + 4 * t - vsh : OOB;

    // work rows: two buffers of (pad + span + pad) u16, zero padding written once
    const int spanA = (span + 3) & ~3;  // (the last thread's dword, zero past the row end)
    const int pitch = PADB + 2 * spanA + PADB;
    for (int i = t; i < 2 * (PADB / 4); i += static_cast<int>(blockDim.x)) {
        const int buf = i / (PADB / 4), k = i % (PADB / 4);
        *reinterpret_cast<uint32_t *>(lds + buf * pitch + 4 * k) = 0u;
        *reinterpret_cast<uint32_t *>(lds + buf * pitch + PADB + 2 * spanA + 4 * k) = 0u;
    }
    // the thread's output columns xLo + t + k half, k < CPT (neighbouring lanes one column apart)
    const int half = (xHi - xLo + CPT - 1) / CPT;
    int xc[CPT], aoff[CPT], sh[CPT], stoff[CPT];
    uint32_t cf[CPT][NP], mm[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        xc[k] = xLo + k * half + t;
        const int x = min(xc[k], xHi - 1);
        const int4 c = d.cols[x];
        aoff[k] = c.x - 2 * cLo;
        mm[k] = static_cast<uint32_t>(c.y);
        sh[k] = c.z;
#pragma unroll
        for (int q = 0; q < NP; ++q)
            cf[k][q] = d.colCoef[x * NP + q];
        stoff[k] = t < half && xc[k] < xHi ? xc[k] : OOB;
    }
    bool edgeAny = false;
#pragma unroll
    for (int k = 0; k < CPT; ++k)
        edgeAny = edgeAny || mm[k] != 0x80000000u || sh[k] != 19;
    // (wave-uniform: the exact division of a border column equals the saturating pack on an interior
    // one, so a wave holding any border column takes it for all its lanes -- no divergent branch)
    const bool edgeT = LZ && __builtin_amdgcn_ballot_w64(edgeAny) != 0;

    // rows outside the window [srcRow0, srcRowEnd) load as zero: a row above it has a negative
    // offset, one below it an offset past srcBytes, both outside the buffer range (no compares;
    // prep_ryg checks that the offsets stay within 31 bits)
    auto load_row = [&](int r) -> uint32_t {
        return __builtin_amdgcn_raw_buffer_load_b32(srcR, voff + (r - srcRow0) * srcSt, 0, 0);
    };
    // (the straddling thread's shift is in the byte selectors, as ryx_kernel)
    const uint32_t selLo = 0x0c010c00u + 0x00010001u * static_cast<uint32_t>(vsh);
    const uint32_t selHi = 0x0c030c02u + 0x00010001u * static_cast<uint32_t>(vsh);
    auto widen = [&](uint32_t v, uint32_t (&W)[2]) {
        W[0] = __builtin_amdgcn_perm(0u, v, selLo);
        W[1] = __builtin_amdgcn_perm(0u, v, selHi);
    };
    // (plan.cpp build_ryg repeats the last record kRygRecPad >= PD + 2 times: no clamp)
    auto rec_s = [&](int y) { return sld(d.rowRec, 4 * y); };
    auto rec_c = [&](int y) { return sld(d.rowRec, 4 * y + 1); };
    static_assert(PD == kRygPD, "row records carry s(y + PD - 1) for the FIFO (abi.hip)");

    // window of row y0, the FIFO (slot i: the last two window rows of row y0 + 1 + i)
    int curS = rec_s(y0);
    uint32_t R[T][2];
#pragma unroll
    for (int k = 0; k < T; ++k)
        widen(load_row(curS + k), R[k]);
    uint32_t F[PD][NL];  // slot i: window rows T - NL .. T - 1 of row y0 + 1 + i
#pragma unroll
    for (int i = 0; i < PD; ++i) {
        const bool use = i + 1 < nRows;
        const int sF = rec_s(y0 + 1 + i);
#pragma unroll
        for (int l = 0; l < NL; ++l)
            F[i][l] = load_row(use ? sF + T - NL + l : -1);
    }
    // the row step with the window starting at ring slot O: incoming rows (raw dwords f: window
    // rows T - NL .. T - 1) widened into their slots when `fill`, then the packed MACs
    auto ring_mac = [&](auto oc, bool fill, const uint32_t (&f)[NL], const uint32_t (&cy)[T], uint32_t (&W)[2]) {
        constexpr int O = decltype(oc)::value;
        if (fill) {
#pragma unroll
            for (int l = 0; l < NL; ++l)
                widen(f[l], R[(O + T - NL + l) % T]);
        }
        W[0] = 0u;
        W[1] = 0u;
#pragma unroll
        for (int k = 0; k < T; ++k) {
            W[0] = pk_mad(R[(O + k) % T][0], cy[k], W[0]);
            W[1] = pk_mad(R[(O + k) % T][1], cy[k], W[1]);
        }
    };
    auto vertical = [&](auto bc, int y, uint32_t (&W)[2]) {
        constexpr int B = decltype(bc)::value;
        if (LZ && static_cast<unsigned>(y - d.m0) >= static_cast<unsigned>(d.m1 - d.m0)) {
            // masked border row (uniform, rare): rows outside the image read as zero
            const int side = y < d.m0 ? 0 : 1, i = min(max(side ? y - d.m1 : y, 0), 15);
            W[0] = ydiv2(W[0], d.yM[side][i], d.yS[side][i]);
            W[1] = ydiv2(W[1], d.yM[side][i], d.yS[side][i]);
        }
        if (4 * t < span)
            *reinterpret_cast<uint2 *>(lds + B * pitch + PADB + 8 * t) = make_uint2(W[0], W[1]);
    };
    {
        uint32_t cy0[T], W[2];
        const int co = rec_c(y0);
#pragma unroll
        for (int k = 0; k < T; ++k)
            cy0[k] = static_cast<uint32_t>(sld(d.rowCoef, co + k));
        const uint32_t none[NL] = {};
        ring_mac(std::integral_constant<int, 0>{}, false, none, cy0, W);
        vertical(std::integral_constant<int, 0>{}, y0, W);
    }
    int ro = 0;  // ring slot of the current window's first row
    int nextS = rec_s(y0 + 1), nextC = rec_c(y0 + 1);  // record of the next row, one row ahead

    for (int base = 0; base < nRows; base += PD) {
        static_for<PD>([&](auto rc) {
            constexpr int r = decltype(rc)::value, B = r & 1;
            const int i = base + r;
            if (i >= nRows)
                return;  // whole workgroup
            const int y = y0 + i;
            const bool more = i + 1 < nRows;
            // scalar loads before the barrier (they share lgkmcnt with the LDS reads after it)
            uint32_t cyn[T];
#pragma unroll
            for (int k = 0; k < T; ++k)
                cyn[k] = static_cast<uint32_t>(sld(d.rowCoef, nextC + k));
            const int4 r2 = sload(d.rowRec + (y + 2));  // {s, c, s(y + 1 + PD), 0} of row y + 2: one s_load_dwordx4
            const int s2 = r2.x, c2 = r2.y, sF = r2.z;
            lds_barrier();
            const uint8_t *wr = lds + B * pitch;
            uint32_t w[CPT][NP];
#pragma unroll
            for (int k = 0; k < CPT; ++k)
#pragma unroll
                for (int q = 0; q < NP; ++q)
                    w[k][q] = reinterpret_cast<const uint32_t *>(wr + aoff[k])[q];
            // the FIFO slot's rows for the next row's window, the slot's reload, then the next row's
            // ring step and vertical pass
            uint32_t f[NL];
#pragma unroll
            for (int l = 0; l < NL; ++l)
                f[l] = F[r][l];
            const bool useF = i + 1 + PD < nRows;
#pragma unroll
            for (int l = 0; l < NL; ++l)
                F[r][l] = load_row(useF ? sF + T - NL + l : -1);
            if (more) {
                ro += nextS - curS;
                ro = ro >= T ? ro - T : ro;
                curS = nextS;
                uint32_t W[2];
                // (a chain of uniform compares: a binary tree of them let the compiler turn the ring
                // into a dynamically indexed scratch array)
                static_for<T>([&](auto oc) {
                    if (ro == decltype(oc)::value)
                        ring_mac(oc, true, f, cyn, W);
                });
                vertical(std::integral_constant<int, B ^ 1>{}, y + 1, W);
            }
            nextS = s2;
            nextC = c2;
            // horizontal: the thread's CPT columns of row y
            uint32_t packed[NPK];  // bytes of columns 2i, 2i + 1 in the low half
            if constexpr (LZ) {
                int acc[CPT];
#pragma unroll
                for (int k = 0; k < CPT; ++k) {
                    acc[k] = sdot2_vv(w[k][0], cf[k][0], 1 << 19);
#pragma unroll
                    for (int q = 1; q < NP; ++q)
                        acc[k] = sdot2(w[k][q], cf[k][q], acc[k]);
                }
#pragma unroll
                for (int i2 = 0; i2 < NPK; ++i2) {
                    const int j0 = 2 * i2, j1 = min(2 * i2 + 1, CPT - 1);
                    if (edgeT) {
                        const uint32_t o0 = min(__umulhi(static_cast<uint32_t>(max(acc[j0], 0)), mm[j0]) >> sh[j0], 255u);
                        const uint32_t o1 = min(__umulhi(static_cast<uint32_t>(max(acc[j1], 0)), mm[j1]) >> sh[j1], 255u);
                        packed[i2] = opaque(o0) | (opaque(o1) << 8);
                    } else {
                        packed[i2] = pack_lo(acc[j0], acc[j1]);  // sat_u8(acc >> 20) of both columns
                    }
                }
            } else {
                int o[CPT];
#pragma unroll
                for (int k = 0; k < CPT; ++k) {
                    uint32_t acc = 1u << 22;
#pragma unroll
                    for (int q = 0; q < NP; ++q)
                        acc = udot2(w[k][q], cf[k][q], acc);
                    const uint16_t u = static_cast<uint16_t>(static_cast<int16_t>(static_cast<int>(acc) >> 23));
                    o[k] = u > 255 ? 255 : u;
                }
#pragma unroll
                for (int i2 = 0; i2 < NPK; ++i2)
                    packed[i2] = opaque(static_cast<uint32_t>(o[2 * i2])) |
                                 (opaque(static_cast<uint32_t>(o[min(2 * i2 + 1, CPT - 1)])) << 8);
            }
            const int rowOff = (y - dstRow0) * dstSt;
#pragma unroll
            for (int k = 0; k < CPT; ++k)
                __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(packed[k / 2] >> (8 * (k & 1))), dstR,
                                                     stoff[k] + rowOff, 0, 0);
        });
    }
}

// ================================================================ general upscale rows
//
// Lanczos rows that grow by at most 2 with no exact-ratio kernel (e.g. 576 -> 1080 rows, 15:8, or
// 768 -> 1080, 45:32; plan.cpp build_ryg, abi.hip ryu_positions).  ryg_kernel's NL = 1 mode walks
// output rows: its ring start moves by 0 or 1 per row, so each row picks its copy of the row step
// through a chain of uniform compares and reads its record before the next one (U2 issued 0.85
// SALU per VALU, profiles/r05/sq_u2.txt).  Here the walk is over window POSITIONS p (source rows
// p .. p + T - 1, the reference's srcOY of IQOLanczosResizerImpl_Generic.cpp:404-454, which at an
// upscale advances by 0 or 1 per output row): every position holds the 1 or 2 consecutive output
// rows whose window starts at p, and brings exactly one new source row.  The ring slot of window
// row k at the band's i-th position is (i + k) mod T, a compile-time constant in a trip unrolled
// over lcm(T, PD, 2) positions; the FIFO of raw dwords is PD positions deep and its rows are
// consecutive (no records); one s_load_dwordx4 per position gives {first row, rows, tap offsets}.
// One barrier per position publishes both rows' work rows (two buffers per set, two sets): the
// next position's vertical passes run under this position's LDS reads.  Vertical, border rows,
// columns and stores: as ryg_kernel; waves with no source columns skip the vertical pass (ryx).
template <int A, int B>
struct ct_lcm {
    static constexpr int gcd(int x, int y) { return y ? gcd(y, x % y) : x; }
    static constexpr int value = A / gcd(A, B) * B;
};

// RUN > 0 (round 6): thread t owns the 4 ADJACENT output columns xLo + 4t .. + 3, whose windows lie
// in one run of RUN work-row dwords from the first column's even start (upscaled columns: 4 columns
// span about 2 source columns), so a row takes RUN LDS dwords per thread instead of 4 NP, each
// column's coefficient pairs sit at their offset in a zero-padded run of RUN pairs (abi.hip
// ryu_runs: 4 RUN dots per row instead of 4 NP), and the 4 output bytes go out as one dword.
template <int T, int NP, int PD, int CPT, int RUN, int KM>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void ryu_kernel(RygArgs a)
{
    static_assert(CPT >= 2 && CPT <= 4 && T >= 2, "output columns per thread");
    static_assert(RUN == 0 || (CPT == 4 && RUN >= NP), "run mode: 4 adjacent columns per thread");
    static_assert(KM >= 2 && KM <= 6, "output rows per window position (rows grow by at most KM)");
    constexpr int NQ = RUN ? RUN : NP;  // pairs read (and dots) per column
    constexpr int NPK = (CPT + 1) / 2;
    constexpr int OOB = 0x7ff00000;
    constexpr int PADB = 2 * kRyxPadK;
    constexpr int U = ct_lcm<ct_lcm<T, PD>::value, 2>::value;  // positions per unrolled trip
    const RygDev &d = a.d;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int t = static_cast<int>(threadIdx.x);
    const unsigned blk0 = xcd_chunks(blockIdx.x, a.bands * d.parts, gridDim.x);
    if (blk0 >= a.nBlocks)
        return;  // whole workgroup
    const int part = static_cast<int>(blk0 % static_cast<unsigned>(d.parts));
    const unsigned blk = blk0 / static_cast<unsigned>(d.parts);
    const int cLo = d.parts > 1 ? d.cs[part] : 0, cHi = d.parts > 1 ? d.ce[part] : d.srcW;
    const int xLo = d.parts > 1 ? d.xs[part] : 0, xHi = d.parts > 1 ? d.xs[part + 1] : d.dstW;
    const int band = static_cast<int>(blk % static_cast<unsigned>(a.bands));
    const int frame = static_cast<int>(blk / static_cast<unsigned>(a.bands));
    const int y0 = a.rowBegin + band * a.rowsPerBand, y1 = min(y0 + a.rowsPerBand, a.rowEnd);
    if (y0 >= y1)
        return;  // whole workgroup

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(frame) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(frame) * a.io.dstFrameSt;
    const __amdgpu_buffer_rsrc_t srcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcFrame), 0, a.srcBytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0, dstRow0 = a.io.dstRow0;
    const int span = cHi - cLo;
    const int vsh = 4 * t < span ? max(0, cLo + 4 * t + 4 - d.srcW) : 0;
    const int voff = 4 * t < span ? cLo + 4 * t - vsh : OOB;
    // (upscaled columns: 480 threads over 256 source dwords at 1024 -> 1920; the waves with none
    // skip the vertical pass and its loads, uniformly)
    const bool srcWave = 256 * __builtin_amdgcn_readfirstlane(t >> 6) < span;

    // work rows: 2 sets x KM rows of (pad + span + pad) u16, zero padding written once
    const int spanA = (span + 3) & ~3;
    const int pitch = PADB + 2 * spanA + PADB;
    for (int i = t; i < 2 * KM * (PADB / 4); i += static_cast<int>(blockDim.x)) {
        const int buf = i / (PADB / 4), k = i % (PADB / 4);
        *reinterpret_cast<uint32_t *>(lds + buf * pitch + 4 * k) = 0u;
        *reinterpret_cast<uint32_t *>(lds + buf * pitch + PADB + 2 * spanA + 4 * k) = 0u;
    }
    const int half = RUN ? 1 : (xHi - xLo + CPT - 1) / CPT;
    int xc[CPT], aoff[CPT], sh[CPT], stoff[CPT];
    uint32_t cf[CPT][NQ], mm[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
        xc[k] = RUN ? xLo + 4 * t + k : xLo + k * half + t;
        const int x = min(xc[k], xHi - 1);
        const int4 c = d.cols[x];
        aoff[k] = c.x - 2 * cLo;
        mm[k] = static_cast<uint32_t>(c.y);
        sh[k] = c.z;
#pragma unroll
        for (int q = 0; q < NQ; ++q)
            cf[k][q] = RUN ? d.colRun[x * RUN + q] : d.colCoef[x * NP + q];
        stoff[k] = (RUN || t < half) && xc[k] < xHi ? xc[k] : OOB;
    }
    // run mode: the run starts at the group's lowest even start (phase-0 columns' windows are
    // trimmed to their one tap); a thread whose 4 columns are not all inside the part (its last,
    // partial group) stores bytes (wave-uniform branch, rare)
    int runOff = 0;
    if constexpr (RUN > 0)
        runOff = min(min(aoff[0], aoff[1]), min(aoff[2], aoff[3]));
    const bool fullGrp = xc[0] + 3 < xHi;
    const bool anyPartial = RUN && __builtin_amdgcn_ballot_w64(!fullGrp && xc[0] < xHi) != 0;
    bool edgeAny = false;
#pragma unroll
    for (int k = 0; k < CPT; ++k)
        edgeAny = edgeAny || mm[k] != 0x80000000u || sh[k] != 19;
    const bool edgeT = __builtin_amdgcn_ballot_w64(edgeAny) != 0;

    auto load_row = [&](int r) -> uint32_t {
        return __builtin_amdgcn_raw_buffer_load_b32(srcR, voff + (r - srcRow0) * srcSt, 0, 0);
    };
    const uint32_t selLo = 0x0c010c00u + 0x00010001u * static_cast<uint32_t>(vsh);
    const uint32_t selHi = 0x0c030c02u + 0x00010001u * static_cast<uint32_t>(vsh);
    auto widen = [&](uint32_t v, uint32_t (&W)[2]) {
        W[0] = __builtin_amdgcn_perm(0u, v, selLo);
        W[1] = __builtin_amdgcn_perm(0u, v, selHi);
    };

    // the band's window positions [pA, pA + nPos): the first and last rows' window starts
    const int pA = sld(d.rowRec, 4 * y0), nPos = sld(d.rowRec, 4 * (y1 - 1)) - pA + 1;
    // position record (8 ints, plan.cpp build_ryu_positions): {first output row yF, rows n, tap
    // offsets of rows yF .. yF + 5}, padded by kRyuPosPad records past the last position.  Only a
    // band's first position can start before the band (the band then starts inside it) and only its
    // last one end after it (its rows are clipped)
    const int *posRec = reinterpret_cast<const int *>(d.posRec) + 8 * (pA - d.posBase);
    struct PosRec {
        int yF, n, c[KM];
    };
    auto load_rec = [&](int q) {
        PosRec r;
        r.yF = sld(posRec, 8 * q);
        r.n = sld(posRec, 8 * q + 1);
#pragma unroll
        for (int j = 0; j < KM; ++j)
            r.c[j] = sld(posRec, 8 * q + 2 + j);
        return r;
    };
    auto pin = [&](const PosRec &r) {
        asm volatile("" ::"s"(r.yF), "s"(r.n));
#pragma unroll
        for (int j = 0; j < KM; ++j)
            asm volatile("" ::"s"(r.c[j]));
    };

    uint32_t R[T][2];
#pragma unroll
    for (int k = 0; k < T; ++k)
        widen(load_row(pA + k), R[k]);
    uint32_t F[PD];  // slot j: the row entering at position j + 1 (+ a multiple of PD)
#pragma unroll
    for (int j = 0; j < PD; ++j)
        F[j] = load_row(j + 1 < nPos ? pA + T + j : -1);

    // vertical pass of one output row from the window at ring offset O into work buffer b
    auto vertical = [&](auto oc, int b, int y, const uint32_t (&cy)[T]) {
        constexpr int O = decltype(oc)::value;
        uint32_t W[2] = {0u, 0u};
#pragma unroll
        for (int k = 0; k < T; ++k) {
            W[0] = pk_mad(R[(O + k) % T][0], cy[k], W[0]);
            W[1] = pk_mad(R[(O + k) % T][1], cy[k], W[1]);
        }
        if (static_cast<unsigned>(y - d.m0) >= static_cast<unsigned>(d.m1 - d.m0)) {
            // masked border row (uniform, rare): rows outside the image read as zero
            const int side = y < d.m0 ? 0 : 1, i = min(max(side ? y - d.m1 : y, 0), 15);
            W[0] = ydiv2(W[0], d.yM[side][i], d.yS[side][i]);
            W[1] = ydiv2(W[1], d.yM[side][i], d.yS[side][i]);
        }
        if (4 * t < span)
            *reinterpret_cast<uint2 *>(lds + b * pitch + PADB + 8 * t) = make_uint2(W[0], W[1]);
    };
    auto coefs = [&](int c, uint32_t (&cy)[T]) {
#pragma unroll
        for (int k = 0; k < T; ++k)
            cy[k] = static_cast<uint32_t>(sld(d.rowCoef, c + k));
    };
    // horizontal pass + stores of output row y from work buffer b
    constexpr int WK = RUN ? 1 : CPT;  // runs read per row (run mode: one for the 4 columns)
    auto read_row = [&](int b, uint32_t (&w)[WK][NQ]) {
        const uint8_t *wr = lds + b * pitch;
#pragma unroll
        for (int k = 0; k < WK; ++k)
#pragma unroll
            for (int q = 0; q < NQ; ++q)
                w[k][q] = reinterpret_cast<const uint32_t *>(wr + (RUN ? runOff : aoff[k]))[q];
    };
    auto emit_row = [&](const uint32_t (&w)[WK][NQ], int y) {
        int acc[CPT];
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
            acc[k] = sdot2_vv(w[RUN ? 0 : k][0], cf[k][0], 1 << 19);
#pragma unroll
            for (int q = 1; q < NQ; ++q)
                acc[k] = sdot2(w[RUN ? 0 : k][q], cf[k][q], acc[k]);
        }
        uint32_t packed[NPK];
#pragma unroll
        for (int i2 = 0; i2 < NPK; ++i2) {
            const int j0 = 2 * i2, j1 = min(2 * i2 + 1, CPT - 1);
            if (edgeT) {
                const uint32_t o0 = min(__umulhi(static_cast<uint32_t>(max(acc[j0], 0)), mm[j0]) >> sh[j0], 255u);
                const uint32_t o1 = min(__umulhi(static_cast<uint32_t>(max(acc[j1], 0)), mm[j1]) >> sh[j1], 255u);
                packed[i2] = opaque(o0) | (opaque(o1) << 8);
            } else {
                packed[i2] = pack_lo(acc[j0], acc[j1]);
            }
        }
        const int rowOff = (y - dstRow0) * dstSt;
        if constexpr (RUN) {
            const uint32_t word = (packed[0] & 0xffffu) | (packed[1] << 16);
            __builtin_amdgcn_raw_buffer_store_b32(word, dstR, fullGrp ? xc[0] + rowOff : OOB, 0, 0);
            if (anyPartial) {
#pragma unroll
                for (int k = 0; k < CPT; ++k)
                    __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(word >> (8 * k)), dstR,
                                                         fullGrp ? OOB : stoff[k] + rowOff, 0, 0);
            }
        } else {
#pragma unroll
            for (int k = 0; k < CPT; ++k)
                __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(packed[k / 2] >> (8 * (k & 1))), dstR,
                                                     stoff[k] + rowOff, 0, 0);
        }
    };

    // prologue: the rows of position 0 inside the band into set 0 (the band may start inside it)
    PosRec rn = load_rec(1);  // the next position's record
    {
        const PosRec r0 = load_rec(0);
        const int first = y0 - r0.yF, cnt = min(r0.yF + r0.n, y1) - y0;
        if (srcWave) {
#pragma unroll
            for (int j = 0; j < KM; ++j) {
                if (j < cnt) {
                    int c = r0.c[0];
#pragma unroll
                    for (int q = 1; q < KM; ++q)
                        c = first + j == q ? r0.c[q] : c;
                    uint32_t cy[T];
                    coefs(c, cy);
                    vertical(std::integral_constant<int, 0>{}, j, y0 + j, cy);
                }
            }
        }
    }
    int ya = y0, cnt = min(sld(posRec, 0) + sld(posRec, 1), y1) - y0;  // this position's rows

    for (int base = 0; base < nPos; base += U) {
        static_for<U>([&](auto ic) {
            constexpr int i = decltype(ic)::value, S = i & 1;
            const int p = base + i;
            if (p >= nPos)
                return;  // whole workgroup
            // scalar loads before the barrier (they share lgkmcnt with the LDS reads after it): the
            // next position's taps and the record after it (pinned here: otherwise the compiler sinks
            // them past the barrier to their use in the next position's vertical pass, whose lgkmcnt
            // wait then also waits for this position's LDS reads)
            const int yn = rn.yF, cntn = min(rn.yF + rn.n, y1) - yn;  // (inside the band from position 1 on)
            const bool more = p + 1 < nPos;
            uint32_t cyn[KM][T];
#pragma unroll
            for (int j = 0; j < KM; ++j) {
                coefs(rn.c[j], cyn[j]);
#pragma unroll
                for (int q = 0; q < T; ++q)
                    asm volatile("" ::"s"(cyn[j][q]));
            }
            const PosRec r2 = load_rec(p + 2);
            pin(r2);
            lds_barrier();
            uint32_t w[KM][WK][NQ];
            read_row(KM * S, w[0]);
#pragma unroll
            for (int j = 1; j < KM; ++j)
                if (j < cnt)
                    read_row(KM * S + j, w[j]);
            // the row entering at position p + 1 (FIFO slot i mod PD) and that slot's reload
            const uint32_t f = F[i % PD];
            F[i % PD] = load_row(p + 1 + PD < nPos ? pA + p + PD + T : -1);
            if (more && srcWave) {
                // position p + 1: its new source row replaces window row 0 of position p (slot i mod T)
                widen(f, R[i % T]);
#pragma unroll
                for (int j = 0; j < KM; ++j)
                    if (j < cntn)
                        vertical(std::integral_constant<int, (i + 1) % T>{}, KM * (S ^ 1) + j, yn + j, cyn[j]);
            }
            emit_row(w[0], ya);
#pragma unroll
            for (int j = 1; j < KM; ++j)
                if (j < cnt)
                    emit_row(w[j], ya + j);
            ya = yn;
            cnt = cntn;
            rn = r2;
        });
    }
}

// ================================================================ exact 2:3 Lanczos-3 upscale
//
// Lanczos-3 at exactly 3/2 (e.g. 1280x720 -> 1920x1080; plan.cpp build_u23).  Output y = 3m + j
// takes phase j of the reference's table: j = 0 a single tap on source row 2m, j = 1 six taps from
// 2m - 2, j = 2 six taps from 2m - 1 (IQOLanczosResizerImpl_Generic.cpp:144-190, 404-454; the
// masked borders :464-490, :539-574 the same way as lanczos_d32_kernel: zero rows / columns outside
// the image, border rows divided before the horizontal pass, the edge lanes' 12 sums parked and
// rewritten once per trip).  One WAVE per (row band, output strip, frame); lane l (1..np) owns
// source columns [cb, cb + 8) and output columns [3cb/2, 3cb/2 + 12); a group of 3 output rows adds
// 2 source rows to a register window of 8 (4 groups per trip); 12-byte stores.
struct U23Args {
    U23Dev d;
    Io io;
    int rowBegin, rowEnd, row3Begin, rowsPerBand, bands, wavesPerRow, np;
    int srcBytes, dstBytes;
    unsigned nWaves;
};

template <int PD>
__global__ __launch_bounds__(256) void lanczos_u23_kernel(U23Args a)
{
    constexpr int NW = 8, U = 4, OOB = 0x7ff00000;
    static_assert(U % PD == 0, "prefetch slots repeat within a trip");
    const U23Dev &d = a.d;
    __shared__ int4 park[4][2][3 * U][3];  // per wave, side, row slot: the edge lane's 12 raw sums
    const int lane = static_cast<int>(threadIdx.x) & 63;
    const int wib = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    const unsigned gw = xcd_chunks(blockIdx.x, (a.bands * a.wavesPerRow + 3) / 4, gridDim.x) * 4u + static_cast<unsigned>(wib);
    if (gw >= a.nWaves)
        return;
    const int wcol = static_cast<int>(gw % static_cast<unsigned>(a.wavesPerRow));
    const unsigned rest = gw / static_cast<unsigned>(a.wavesPerRow);
    const int band = static_cast<int>(rest % static_cast<unsigned>(a.bands));
    const int frame = static_cast<int>(rest / static_cast<unsigned>(a.bands));
    const int yb = a.row3Begin + band * a.rowsPerBand;  // a multiple of 3
    const int y0 = max(yb, a.rowBegin), y1 = min(yb + a.rowsPerBand, a.rowEnd);
    if (y0 >= y1)
        return;
    const int kLo = yb / 3;
    const int nG = (y1 - yb + 2) / 3;

    const int opw = 12 * a.np;
    const int x0 = max(0, min(wcol * opw, d.dstW - opw));
    const int cb = (2 * x0) / 3 - 8 + 8 * lane;
    const bool produce = lane >= 1 && lane <= a.np;
    const int voff = (lane <= a.np + 1 && cb >= 0 && cb + 8 <= d.srcW) ? cb : OOB;
    const int stoff = produce ? x0 + 12 * (lane - 1) : OOB;
    const bool edgeL = x0 == 0, edgeR = x0 + opw >= d.dstW;
    const bool laneL = edgeL && lane == 1, laneR = edgeR && lane == a.np;

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(frame) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(frame) * a.io.dstFrameSt;
    const __amdgpu_buffer_rsrc_t srcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcFrame), 0, a.srcBytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0, dstRow0 = a.io.dstRow0;

    // relative source row q = row 2 kLo - 2 + q: zero outside the image, clamped outside the call's
    // window (dropped outputs only), not loaded past the band's last group
    const int rBase = 2 * kLo - 2;
    const int rLast = 2 * (kLo + nG - 1) + 4;
    const int srcLast = a.io.srcRowEnd - 1;
    auto load_row = [&](int q) -> u32x2 {
        const int r = rBase + q;
        const int rc = min(max(r, srcRow0), srcLast);
        const bool in = r >= 0 && r < d.srcH && r <= rLast;
        return __builtin_amdgcn_raw_buffer_load_b64(srcR, voff + (in ? (rc - srcRow0) * srcSt : OOB), 0, 0);
    };
    auto widen = [&](u32x2 v, uint32_t (&P)[4]) {
        P[0] = __builtin_amdgcn_perm(0u, v.x, 0x0c010c00u);
        P[1] = __builtin_amdgcn_perm(0u, v.x, 0x0c030c02u);
        P[2] = __builtin_amdgcn_perm(0u, v.y, 0x0c010c00u);
        P[3] = __builtin_amdgcn_perm(0u, v.y, 0x0c030c02u);
    };
    auto store_row = [&](u32x3 o, int voffs, int y, bool ok) {
        __builtin_amdgcn_raw_buffer_store_b96(o, dstR, voffs + (ok ? (y - dstRow0) * dstSt : OOB), 0, 0);
    };
    auto border_row = [&](uint32_t (&W)[4], int y) {
        if (y < d.m0 || y >= d.m1) {
            const int side = y < d.m0 ? 0 : 1, i = min(max(side ? y - d.m1 : y, 0), 7);
            const uint32_t m = d.yM[side][i];
            const int sh = d.yS[side][i];
#pragma unroll
            for (int c = 0; c < 4; ++c)
                W[c] = ydiv2(W[c], m, sh);
        }
    };
    auto emit = [&](const uint32_t (&W)[4], int y, int slot) {
        uint32_t E[7];  // E[e] = work columns (cb - 2 + 2e, cb - 1 + 2e)
        E[0] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(W[3]), 0x138 /* wave_shr:1 */, 0xf, 0xf, true));
#pragma unroll
        for (int e = 0; e < 4; ++e)
            E[e + 1] = W[e];
        E[5] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(W[0]), 0x130 /* wave_shl:1 */, 0xf, 0xf, true));
        E[6] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(W[1]), 0x130, 0xf, 0xf, true));
        uint32_t O[6];  // O[e] = work columns (cb - 1 + 2e, cb + 2e)
#pragma unroll
        for (int e = 0; e < 6; ++e)
            O[e] = __builtin_amdgcn_alignbit(E[e + 1], E[e], 16);
        auto pair = [&](int rel) { return (rel & 1) ? O[(rel + 1) / 2] : E[(rel + 2) / 2]; };  // low half = column cb + rel
        int sum[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const int g = j / 3, ph = j % 3;
            if (ph == 0) {
                sum[j] = sdot2_sv(pair(2 * g), d.cx0, 1 << 19);
            } else {
                const int rel = 2 * g - 2 + (ph - 1);
                int acc = sdot2_sv(pair(rel), d.cx[ph - 1][0], 1 << 19);
#pragma unroll
                for (int q = 1; q < 3; ++q)
                    acc = sdot2(pair(rel + 2 * q), d.cx[ph - 1][q], acc);
                sum[j] = acc;
            }
        }
        u32x3 o;
        o.x = pack_hi(pack_lo(sum[0], sum[1]), sum[2], sum[3]);
        o.y = pack_hi(pack_lo(sum[4], sum[5]), sum[6], sum[7]);
        o.z = pack_hi(pack_lo(sum[8], sum[9]), sum[10], sum[11]);
        store_row(o, stoff, y, y >= y0 && y < y1);
        if (edgeL || edgeR) {  // uniform
            if (laneL || laneR) {
                int4 *pk = park[wib][laneL ? 0 : 1][slot];
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    pk[q] = make_int4(sum[4 * q], sum[4 * q + 1], sum[4 * q + 2], sum[4 * q + 3]);
            }
        }
    };
    // once per trip: lane r < 3U rewrites the edge bytes of row yt + r from the parked sums
    auto flush = [&](int yt) {
        u32x3 oL = {0u, 0u, 0u}, oR = {0u, 0u, 0u};
        const int r = min(lane, 3 * U - 1);
        if (edgeL || edgeR) {  // uniform
            __builtin_amdgcn_wave_barrier();
            auto fix = [&](int side) {
                uint32_t w[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const int4 p = park[wib][side][r][q];
                    const int sv[4] = {p.x, p.y, p.z, p.w};
                    uint32_t b[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        b[e] = min(__umulhi(static_cast<uint32_t>(max(sv[e], 0)), d.xM[side][4 * q + e]) >> d.xT[side][4 * q + e],
                                   255u);
                    w[q] = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
                }
                return u32x3{w[0], w[1], w[2]};
            };
            if (edgeL)
                oL = fix(0);
            if (edgeR)
                oR = fix(1);
        }
        const int y = yt + lane;
        const bool ok = lane < 3 * U && y >= y0 && y < y1;
        store_row(oL, edgeL ? 0 : OOB, y, ok);
        store_row(oR, edgeR ? d.dstW - 12 : OOB, y, ok);
    };

    uint32_t R[NW][4];
    // group 0's window without its own new rows: relative rows 0..4
#pragma unroll
    for (int q = 0; q < 5; ++q)
        widen(load_row(q), R[q]);
    // prefetch: group g adds relative rows 2g + 5, 2g + 6
    u32x2 pre[PD][2];
#pragma unroll
    for (int v = 0; v < PD; ++v) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
            pre[v][i] = load_row(2 * v + 5 + i);
#pragma unroll
        for (int i = 0; i < 3; ++i)  // the loop's three row stores per group, dropped
            __builtin_amdgcn_raw_buffer_store_b96(u32x3{0u, 0u, 0u}, dstR, OOB, 0, 0);
    }
    __builtin_amdgcn_raw_buffer_store_b96(u32x3{0u, 0u, 0u}, dstR, OOB, 0, 0);  // and the trip's two flush stores
    __builtin_amdgcn_raw_buffer_store_b96(u32x3{0u, 0u, 0u}, dstR, OOB, 0, 0);
    for (int base = 0; base < nG; base += U) {
        static_for<U>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            const int g = base + v;
            if (g >= nG)
                return;  // past the band's last group (uniform; the trip's flush still runs)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 2; ++i)
                widen(pre[v % PD][i], R[(2 * v + 5 + i) % NW]);
#pragma unroll
            for (int i = 0; i < 2; ++i)
                pre[v % PD][i] = load_row(2 * (g + PD) + 5 + i);
            const int y = 3 * (kLo + g);
            uint32_t W[4];
#pragma unroll
            for (int c = 0; c < 4; ++c)  // phase 0: source row 2m (relative 2g + 2)
                W[c] = pk_mul(R[(2 * v + 2) % NW][c], d.cy0);
            border_row(W, y);
            emit(W, y, 3 * v);
#pragma unroll
            for (int ph = 0; ph < 2; ++ph) {  // phases 1, 2: six rows from relative 2g + ph
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    W[c] = pk_mul(R[(2 * v + ph) % NW][c], d.cy[ph][0]);
#pragma unroll
                for (int k = 1; k < 6; ++k)
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        W[c] = pk_mad(R[(2 * v + ph + k) % NW][c], d.cy[ph][k], W[c]);
                border_row(W, y + 1 + ph);
                emit(W, y + 1 + ph, 3 * v + 1 + ph);
            }
        });
        flush(3 * (kLo + base));
    }
}

// ================================================================ exact 2:3 Linear upscale
//
// Linear at exactly 3/2 (e.g. 1280x720 -> 1920x1080; plan.cpp build_l23): output y = 3m + j takes
// phase j's two taps from source row 2m + j - 1 (IQOLinearResizerImpl_Generic.cpp:157-208 tables,
// :210-282 rows; u16 vertical blend, (s + 2^22) >> 23 horizontal, :327-346).  With the source
// clamped to the image (rows by address, the halo columns of the frame's first / last lane by
// per-lane byte-broadcast selectors) the same two taps give the reference's replicated border
// pixels, so there is no border code.  Lane layout of lanczos_u23_kernel: 8 source columns ->
// 12 outputs; a group of 3 output rows adds 2 source rows to a window of 4.
struct L23Args {
    L23Dev d;
    Io io;
    int rowBegin, rowEnd, row3Begin, rowsPerBand, bands, wavesPerRow, np;
    int srcBytes, dstBytes;
    unsigned nWaves;
};

template <int PD>
__global__ __launch_bounds__(256) void linear_u23_kernel(L23Args a)
{
    constexpr int NW = 4, U = 2, OOB = 0x7ff00000;
    static_assert(U % PD == 0, "prefetch slots repeat within a trip");
    const L23Dev &d = a.d;
    const int lane = static_cast<int>(threadIdx.x) & 63;
    const int wib = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    const unsigned gw = xcd_chunks(blockIdx.x, (a.bands * a.wavesPerRow + 3) / 4, gridDim.x) * 4u + static_cast<unsigned>(wib);
    if (gw >= a.nWaves)
        return;
    const int wcol = static_cast<int>(gw % static_cast<unsigned>(a.wavesPerRow));
    const unsigned rest = gw / static_cast<unsigned>(a.wavesPerRow);
    const int band = static_cast<int>(rest % static_cast<unsigned>(a.bands));
    const int frame = static_cast<int>(rest / static_cast<unsigned>(a.bands));
    const int yb = a.row3Begin + band * a.rowsPerBand;
    const int y0 = max(yb, a.rowBegin), y1 = min(yb + a.rowsPerBand, a.rowEnd);
    if (y0 >= y1)
        return;
    const int kLo = yb / 3;
    const int nG = (y1 - yb + 2) / 3;

    const int opw = 12 * a.np;
    const int x0 = max(0, min(wcol * opw, d.dstW - opw));
    const int cb = (2 * x0) / 3 - 8 + 8 * lane;
    const bool produce = lane >= 1 && lane <= a.np;
    // the halo lane left of column 0 / right of the last column replicates the edge pixel
    const bool clampL = lane <= a.np + 1 && cb < 0, clampR = lane <= a.np + 1 && cb + 8 > d.srcW;
    const int voff = lane > a.np + 1 ? OOB : clampL ? 0 : clampR ? d.srcW - 8 : cb;
    const uint32_t selA = clampL ? 0x0c000c00u : clampR ? 0x0c070c07u : 0x0c010c00u;
    const uint32_t selB = clampL ? 0x0c000c00u : clampR ? 0x0c070c07u : 0x0c030c02u;
    const uint32_t selC = clampL ? 0x0c000c00u : clampR ? 0x0c070c07u : 0x0c050c04u;
    const uint32_t selD = clampL ? 0x0c000c00u : clampR ? 0x0c070c07u : 0x0c070c06u;
    const int stoff = produce ? x0 + 12 * (lane - 1) : OOB;

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(frame) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(frame) * a.io.dstFrameSt;
    const __amdgpu_buffer_rsrc_t srcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcFrame), 0, a.srcBytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0, dstRow0 = a.io.dstRow0;

    // relative source row q = row 2 kLo - 1 + q, clamped to the image (replicated border rows) and
    // to the call's window (rows of dropped outputs only); not loaded past the band's last group
    const int rBase = 2 * kLo - 1;
    const int rLast = 2 * (kLo + nG - 1) + 2;
    const int rMin = max(0, srcRow0), rMax = min(d.srcH - 1, a.io.srcRowEnd - 1);
    auto load_row = [&](int q) -> u32x2 {
        const int r = rBase + q;
        const int rc = min(max(r, rMin), rMax);
        return __builtin_amdgcn_raw_buffer_load_b64(srcR, voff + (r <= rLast ? (rc - srcRow0) * srcSt : OOB), 0, 0);
    };
    auto widen = [&](u32x2 v, uint32_t (&P)[4]) {
        P[0] = __builtin_amdgcn_perm(v.y, v.x, selA);
        P[1] = __builtin_amdgcn_perm(v.y, v.x, selB);
        P[2] = __builtin_amdgcn_perm(v.y, v.x, selC);
        P[3] = __builtin_amdgcn_perm(v.y, v.x, selD);
    };
    auto emit = [&](const uint32_t (&W)[4], int y) {
        uint32_t E[6];  // E[e] = work columns (cb - 2 + 2e, cb - 1 + 2e)
        E[0] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(W[3]), 0x138 /* wave_shr:1 */, 0xf, 0xf, true));
#pragma unroll
        for (int e = 0; e < 4; ++e)
            E[e + 1] = W[e];
        E[5] = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(W[0]), 0x130 /* wave_shl:1 */, 0xf, 0xf, true));
        uint32_t O[5];  // O[e] = work columns (cb - 1 + 2e, cb + 2e)
#pragma unroll
        for (int e = 0; e < 5; ++e)
            O[e] = __builtin_amdgcn_alignbit(E[e + 1], E[e], 16);
        const uint32_t b = 1u << 22;
        uint32_t sum[12];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            sum[3 * g] = udot2(O[g], d.cx[0], b);          // columns 2g - 1, 2g
            sum[3 * g + 1] = udot2(E[g + 1], d.cx[1], b);  // 2g, 2g + 1
            sum[3 * g + 2] = udot2(O[g + 1], d.cx[2], b);  // 2g + 1, 2g + 2
        }
        u32x3 o;
        o.x = pack23_hi(pack23_lo(sum[0], sum[1]), sum[2], sum[3]);
        o.y = pack23_hi(pack23_lo(sum[4], sum[5]), sum[6], sum[7]);
        o.z = pack23_hi(pack23_lo(sum[8], sum[9]), sum[10], sum[11]);
        __builtin_amdgcn_raw_buffer_store_b96(o, dstR, stoff + (y >= y0 && y < y1 ? (y - dstRow0) * dstSt : OOB), 0, 0);
    };

    uint32_t R[NW][4];
    widen(load_row(0), R[0]);
    widen(load_row(1), R[1]);
    u32x2 pre[PD][2];
#pragma unroll
    for (int v = 0; v < PD; ++v) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
            pre[v][i] = load_row(2 * v + 2 + i);
#pragma unroll
        for (int i = 0; i < 3; ++i)  // the loop's three row stores per group, dropped
            __builtin_amdgcn_raw_buffer_store_b96(u32x3{0u, 0u, 0u}, dstR, OOB, 0, 0);
    }
    for (int base = 0; base < nG; base += U) {
        static_for<U>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            const int g = base + v;
            if (g >= nG)
                return;  // past the band's last group (uniform; the trip's flush still runs)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 2; ++i)
                widen(pre[v % PD][i], R[(2 * v + 2 + i) % NW]);
#pragma unroll
            for (int i = 0; i < 2; ++i)
                pre[v % PD][i] = load_row(2 * (g + PD) + 2 + i);
            const int y = 3 * (kLo + g);
#pragma unroll
            for (int j = 0; j < 3; ++j) {  // phase j: relative rows 2g + j, 2g + j + 1
                uint32_t W[4];
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    W[c] = pk_mad(R[(2 * v + j + 1) % NW][c], d.cy[j][1], pk_mul(R[(2 * v + j) % NW][c], d.cy[j][0]));
                emit(W, y + j);
            }
        });
    }
}

// ================================================================ exact 3:2 Area downscale
//
// Area at exactly 2/3 (plan.cpp build_a32; the reference's Area tables for this ratio,
// IQOAreaResizerImpl_Generic.cpp:11-97, have two non-zero taps per phase): output rows 2m, 2m+1
// read exactly source rows 3m .. 3m + 2 (171/85 and 85/171 of 256) and output columns
// 8g .. 8g + 7 exactly source columns 12g .. 12g + 11, so a lane needs no neighbour and a row
// pair no window.  One WAVE per (row band, 8 * np-column strip, frame); per row pair each lane
// loads its 12 bytes of the 3 rows (PD pairs ahead), widens them to u16 pairs, forms the two u16
// work rows (resizeYmain :313-319, 16-bit wrap) with packed MACs and the 8 outputs with one
// v_dot2_u32_u16 each ((s + 2^22) >> 23, :349-367), one 8-byte store per row.
struct A32Args {
    A32Dev d;
    Io io;
    int rowBegin, rowEnd, evenBegin, rowsPerBand, bands, wavesPerRow, np;
    int srcBytes, dstBytes;
    unsigned nWaves;
};

template <int PD>
__global__ __launch_bounds__(256) void area_d32_kernel(A32Args a)
{
    constexpr int OOB = 0x7ff00000;
    const A32Dev &d = a.d;
    const int lane = static_cast<int>(threadIdx.x) & 63;
    const int wib = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    const unsigned gw = xcd_chunks(blockIdx.x, (a.bands * a.wavesPerRow + 3) / 4, gridDim.x) * 4u + static_cast<unsigned>(wib);
    if (gw >= a.nWaves)
        return;
    const int wcol = static_cast<int>(gw % static_cast<unsigned>(a.wavesPerRow));
    const unsigned rest = gw / static_cast<unsigned>(a.wavesPerRow);
    const int band = static_cast<int>(rest % static_cast<unsigned>(a.bands));
    const int frame = static_cast<int>(rest / static_cast<unsigned>(a.bands));
    const int yb = a.evenBegin + band * a.rowsPerBand;  // even
    const int y0 = max(yb, a.rowBegin), y1 = min(yb + a.rowsPerBand, a.rowEnd);
    if (y0 >= y1)
        return;
    const int kLo = yb >> 1;
    const int nG = (y1 - yb + 1) >> 1;

    const int opw = 8 * a.np;
    const int x0 = max(0, min(wcol * opw, d.dstW - opw));
    const bool produce = lane < a.np;
    const int voff = produce ? (3 * x0) / 2 + 12 * lane : OOB;
    const int stoff = produce ? x0 + 8 * lane : OOB;

    const uint8_t *srcFrame = a.io.src + static_cast<int64_t>(frame) * a.io.srcFrameSt;
    uint8_t *dstFrame = a.io.dst + static_cast<int64_t>(frame) * a.io.dstFrameSt;
    const __amdgpu_buffer_rsrc_t srcR =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(srcFrame), 0, a.srcBytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t dstR = __builtin_amdgcn_make_buffer_rsrc(dstFrame, 0, a.dstBytes, 0x00020000);
    const int srcSt = static_cast<int>(a.io.srcSt), dstSt = static_cast<int>(a.io.dstSt);
    const int srcRow0 = a.io.srcRow0, dstRow0 = a.io.dstRow0;
    const int rLast = 3 * (kLo + nG) - 1;
    const int srcLast = a.io.srcRowEnd - 1;
    // source row r (group rows of dropped outputs may lie outside the call's window: clamped, never
    // used; rows past the band's last group are not loaded)
    auto load_row = [&](int r) -> u32x3 {
        const int rc = min(max(r, srcRow0), srcLast);
        return __builtin_amdgcn_raw_buffer_load_b96(srcR, voff + (r <= rLast ? (rc - srcRow0) * srcSt : OOB), 0,
                                                    0);
    };
    auto widen = [&](u32x3 v, uint32_t (&P)[6]) {
        P[0] = __builtin_amdgcn_perm(0u, v.x, 0x0c010c00u);
        P[1] = __builtin_amdgcn_perm(0u, v.x, 0x0c030c02u);
        P[2] = __builtin_amdgcn_perm(0u, v.y, 0x0c010c00u);
        P[3] = __builtin_amdgcn_perm(0u, v.y, 0x0c030c02u);
        P[4] = __builtin_amdgcn_perm(0u, v.z, 0x0c010c00u);
        P[5] = __builtin_amdgcn_perm(0u, v.z, 0x0c030c02u);
    };
    auto emit = [&](const uint32_t (&E)[6], int y) {
        // output j: pair at column 3 (j >> 1) + (j & 1): E[k] = (2k, 2k+1), odd starts by alignbit
        const uint32_t O1 = __builtin_amdgcn_alignbit(E[1], E[0], 16), O3 = __builtin_amdgcn_alignbit(E[2], E[1], 16);
        const uint32_t O7 = __builtin_amdgcn_alignbit(E[4], E[3], 16), O9 = __builtin_amdgcn_alignbit(E[5], E[4], 16);
        const uint32_t b = 1u << 22;
        u32x2 o;
        o.x = pack23_hi(pack23_lo(udot2(E[0], d.cx[0], b), udot2(O1, d.cx[1], b)), udot2(O3, d.cx[0], b),
                        udot2(E[2], d.cx[1], b));
        o.y = pack23_hi(pack23_lo(udot2(E[3], d.cx[0], b), udot2(O7, d.cx[1], b)), udot2(O9, d.cx[0], b),
                        udot2(E[5], d.cx[1], b));
        __builtin_amdgcn_raw_buffer_store_b64(o, dstR, stoff + (y >= y0 && y < y1 ? (y - dstRow0) * dstSt : OOB), 0, 0);
    };

    u32x3 pre[PD][3];
#pragma unroll
    for (int v = 0; v < PD; ++v) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 3; ++i)
            pre[v][i] = load_row(3 * (kLo + v) + i);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, dstR, OOB, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, dstR, OOB, 0, 0);
    }
    for (int base = 0; base < nG; base += PD) {
        static_for<PD>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            const int g = base + v;
            if (g >= nG)
                return;  // past the band's last group (uniform; the trip's flush still runs)
            __builtin_amdgcn_sched_barrier(0);
            uint32_t A[6], B[6], C[6];
            widen(pre[v][0], A);
            widen(pre[v][1], B);
            widen(pre[v][2], C);
#pragma unroll
            for (int i = 0; i < 3; ++i)
                pre[v][i] = load_row(3 * (kLo + g + PD) + i);
            uint32_t W[6];
#pragma unroll
            for (int c = 0; c < 6; ++c)
                W[c] = pk_mad(B[c], d.cy[0][1], pk_mul(A[c], d.cy[0][0]));
            emit(W, 2 * (kLo + g));
#pragma unroll
            for (int c = 0; c < 6; ++c)
                W[c] = pk_mad(C[c], d.cy[1][1], pk_mul(B[c], d.cy[1][0]));
            emit(W, 2 * (kLo + g) + 1);
        });
    }
}

} // namespace

// ================================================================ launchers

hipError_t launch_up2(const Up2Dev &u, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s)
{
    if (rowEnd <= rowBegin || io.frames <= 0)
        return hipSuccess;
    const int64_t sb = static_cast<int64_t>(io.srcRowEnd - io.srcRow0 - 1) * io.srcSt + u.srcW;
    const int64_t db = static_cast<int64_t>(rowEnd - 1 - io.dstRow0) * io.dstSt + u.dstW;  // stores are relative to dstRow0
    if (sb >= 0x7ff00000 || db >= 0x7ff00000 || io.srcSt >= (int64_t(1) << 24) || io.dstSt >= (int64_t(1) << 24) ||
        (u.NT != 4 && u.NT != 6) || (u.F != 2 && u.F != 3) || u.dstW % (8 * u.F) || u.dstW != u.F * u.srcW ||
        u.dstW < 16 * u.F || u.dstH != u.F * u.srcH)
        return hipErrorInvalidValue;
    const void *kern = u.F == 3 ? (u.NT == 6 ? reinterpret_cast<const void *>(lanczos_up2_kernel<6, 3>)
                                             : reinterpret_cast<const void *>(lanczos_up2_kernel<4, 3>))
                                : (u.NT == 6 ? reinterpret_cast<const void *>(lanczos_up2_kernel<6, 2>)
                                             : reinterpret_cast<const void *>(lanczos_up2_kernel<4, 2>));
    // producing lanes per wave: the fewest waves per row, then the fewest lanes that tile the width
    const int lanes = u.dstW / (8 * u.F);
    int wpr = (lanes + 61) / 62;
    int np = u.np > 0 ? min(u.np, min(62, lanes)) : (lanes + wpr - 1) / wpr;
    wpr = (lanes + np - 1) / np;
    const int rows = rowEnd - rowBegin;
    // bands: one trip (NT source steps, F NT output rows) each -- the most waves with no partial
    // trip (fresh batches, 2x 1080p 125 frames: 12-row bands 54.9 % of 8 TB/s vs 53.2 % at ~2.5
    // rounds of resident waves; 3x 720p 141 frames: 18-row bands 47.4 % vs 39.3 %)
    // (round 6, steady clock: bands of at most 12 rows -- 3x Lanczos-3 720p -> 4K x64: 180 bands of
    // 12 rows 0.149 ms vs 120 of 18 rows 0.164, profiles/r06/band_sweeps.txt)
    if (bands <= 0)
        bands = std::max(1, rows / std::min(u.F * u.NT, 12));
    bands = std::max(1, std::min(bands, rows));
    int rpb = (rows + bands - 1) / bands;
    rpb = (rpb + u.F - 1) / u.F * u.F;  // a band's steps produce whole groups of F rows
    // whole trips (NT steps, F NT rows) when the band is longer than one: the last trip of a band
    // is otherwise partial (2x, 1080 rows: 120 bands of 9 rows 47.6 % vs 90 of 12 rows 55.1 %)
    const int tripRows = u.F * u.NT;
    if (rpb > tripRows)
        rpb = (rpb + tripRows - 1) / tripRows * tripRows;
    bands = (rows + rpb - 1) / rpb;
    const uint64_t nWaves = static_cast<uint64_t>(wpr) * bands * static_cast<uint64_t>(io.frames);
    if (nWaves >= (uint64_t(1) << 31))
        return hipErrorInvalidValue;
    Up2Args a{u, io, rowBegin, rowEnd, rpb, bands, wpr, np, static_cast<int>(sb), static_cast<int>(db),
              static_cast<unsigned>(nWaves)};
    void *args[] = {&a};
    return hipLaunchKernel(kern, dim3(static_cast<unsigned>((nWaves + 3) / 4)), dim3(256), args, 0, s);
}

hipError_t launch_d32(const D32Dev &d, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s)
{
    if (rowEnd <= rowBegin || io.frames <= 0)
        return hipSuccess;
    if (d.dstW % 8 || d.dstW < 16 || 2 * d.srcW != 3 * d.dstW)
        return hipErrorInvalidValue;
    const int64_t sb = static_cast<int64_t>(io.srcRowEnd - io.srcRow0 - 1) * io.srcSt + d.srcW;
    const int64_t db = static_cast<int64_t>(rowEnd - 1 - io.dstRow0) * io.dstSt + d.dstW;  // stores are relative to dstRow0
    if (sb >= 0x7ff00000 || db >= 0x7ff00000 || io.srcSt >= (int64_t(1) << 24) || io.dstSt >= (int64_t(1) << 24))
        return hipErrorInvalidValue;
    // producing lanes per wave: the fewest waves per row, then the fewest lanes that tile the width
    const int lanes = d.dstW / 8;
    int wpr = (lanes + 61) / 62;
    int np = d.np > 0 ? min(d.np, min(62, lanes)) : (lanes + wpr - 1) / wpr;
    wpr = (lanes + np - 1) / np;
    // one group of rows loaded ahead by default (G1, fresh data: 2.5 % faster than 2, 8 % than 4)
    const void *kern = nullptr;
    if (d.variant == 0)
        kern = d.pd == 2   ? reinterpret_cast<const void *>(lanczos_d32_kernel<2, -4, 10, 8, 2, 5, -4>)
               : d.pd == 4 ? reinterpret_cast<const void *>(lanczos_d32_kernel<4, -4, 10, 8, 2, 5, -4>)
                           : reinterpret_cast<const void *>(lanczos_d32_kernel<1, -4, 10, 8, 2, 5, -4>);
    else if (d.variant == 1)
        kern = d.pd == 3 ? reinterpret_cast<const void *>(lanczos_d32_kernel<3, -2, 7, 5, 2, 3, -2>)
                         : reinterpret_cast<const void *>(lanczos_d32_kernel<1, -2, 7, 5, 2, 3, -2>);
    else
        return hipErrorInvalidValue;
    const int evenBegin = rowBegin & ~1;
    const int rows = rowEnd - evenBegin;
    // bands: ~2.5 rounds of resident waves, whole trips (8 rows) per band, >= 16 rows
    // (round 6, steady clock: bands of ~16 rows whatever the batch -- 1080p -> 720p x128: 45 bands
    // 0.0827 ms vs the ~2.5-rounds choice 0.0877, profiles/r06/band_sweeps.txt)
    if (bands <= 0)
        bands = std::max(1, rows / 16);
    const int trip = d.variant == 0 ? 8 : 6;  // output rows per unrolled trip (2 U)
    bands = std::max(1, std::min(bands, (rows + trip - 1) / trip));
    int rpb = (rows + bands - 1) / bands;
    rpb = (rpb + trip - 1) / trip * trip;
    bands = (rows + rpb - 1) / rpb;
    const uint64_t nWaves = static_cast<uint64_t>(wpr) * bands * static_cast<uint64_t>(io.frames);
    if (nWaves >= (uint64_t(1) << 31))
        return hipErrorInvalidValue;
    D32Args a{d, io, rowBegin, rowEnd, evenBegin, rpb, bands, wpr, np, static_cast<int>(sb), static_cast<int>(db),
              static_cast<unsigned>(nWaves)};
    void *args[] = {&a};
    return hipLaunchKernel(kern, dim3(static_cast<unsigned>((nWaves + 3) / 4)), dim3(256), args, 0, s);
}

hipError_t launch_d31(const D31Dev &d, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s)
{
    if (rowEnd <= rowBegin || io.frames <= 0)
        return hipSuccess;
    if (d.dstW % 4 || d.dstW < 16 || d.srcW != 3 * d.dstW)
        return hipErrorInvalidValue;
    const int64_t sb = static_cast<int64_t>(io.srcRowEnd - io.srcRow0 - 1) * io.srcSt + d.srcW;
    const int64_t db = static_cast<int64_t>(rowEnd - 1 - io.dstRow0) * io.dstSt + d.dstW;  // stores are relative to dstRow0
    if (sb >= 0x7ff00000 || db >= 0x7ff00000 || io.srcSt >= (int64_t(1) << 24) || io.dstSt >= (int64_t(1) << 24))
        return hipErrorInvalidValue;
    // producing lanes per wave (4 outputs each): the fewest waves per row, then the fewest lanes
    // that tile the width
    const int lanes = d.dstW / 4;
    int wpr = (lanes + 61) / 62;
    int np = d.np > 0 ? min(d.np, min(62, lanes)) : (lanes + wpr - 1) / wpr;
    wpr = (lanes + np - 1) / np;
    const void *kern = nullptr;
    if (d.variant == 0)
        kern = d.pd == 5 ? reinterpret_cast<const void *>(lanczos_d31_kernel<5, 0>)
                         : reinterpret_cast<const void *>(lanczos_d31_kernel<1, 0>);
    else if (d.variant == 1)
        kern = d.pd == 2   ? reinterpret_cast<const void *>(lanczos_d31_kernel<2, 1>)
               : d.pd == 4 ? reinterpret_cast<const void *>(lanczos_d31_kernel<4, 1>)
                           : reinterpret_cast<const void *>(lanczos_d31_kernel<1, 1>);
    else
        return hipErrorInvalidValue;
    const int rows = rowEnd - rowBegin;
    const int trip = d.variant == 0 ? 5 : 4;  // output rows per unrolled trip (U)
    // bands of two trips (round 6, steady clock: 4K -> 720p x128: 72 bands of 10 rows 0.235 ms vs
    // the ~2.5-rounds choice 0.261, profiles/r06/band_sweeps.txt)
    if (bands <= 0)
        bands = std::max(1, rows / (2 * trip));
    bands = std::max(1, std::min(bands, (rows + trip - 1) / trip));
    int rpb = (rows + bands - 1) / bands;
    rpb = (rpb + trip - 1) / trip * trip;
    bands = (rows + rpb - 1) / rpb;
    const uint64_t nWaves = static_cast<uint64_t>(wpr) * bands * static_cast<uint64_t>(io.frames);
    if (nWaves >= (uint64_t(1) << 31))
        return hipErrorInvalidValue;
    D31Args a{d, io, rowBegin, rowEnd, rpb, bands, wpr, np, static_cast<int>(sb), static_cast<int>(db),
              static_cast<unsigned>(nWaves)};
    void *args[] = {&a};
    return hipLaunchKernel(kern, dim3(static_cast<unsigned>((nWaves + 3) / 4)), dim3(256), args, 0, s);
}

hipError_t launch_ryx(const RyxDev &d, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s)
{
    if (rowEnd <= rowBegin || io.frames <= 0)
        return hipSuccess;
    if (d.srcW < 16 || d.srcW > 8192 || d.dstW > 4096)
        return hipErrorInvalidValue;
    const int64_t sb = static_cast<int64_t>(io.srcRowEnd - io.srcRow0 - 1) * io.srcSt + d.srcW;
    const int64_t db = static_cast<int64_t>(rowEnd - 1 - io.dstRow0) * io.dstSt + d.dstW;  // stores are relative to dstRow0
    if (sb >= 0x7ff00000 || db >= 0x7ff00000 || io.srcSt >= (int64_t(1) << 24) || io.dstSt >= (int64_t(1) << 24))
        return hipErrorInvalidValue;
    // instantiations (plan.cpp build_ryx kShapes): method, P, Q, taps (the reference's taps less the
    // zero outer taps of every phase), column pairs
    // PD: groups of P source rows loaded ahead (ubench: with one group in flight the source loads
    // cost G5 19 % and Lanczos-4 2:1 27 % of the kernel time -- latency, not bandwidth)
    // ADJ: adjacent column pairs per thread (9:4 rows with columns >= 2:1, ryx_dev d.adj)
    // CPT: output columns per thread (upscales, ryx_dev d.cpt)
    struct Inst {
        bool lz;
        int P, Q, T, NP;
        bool adj;
        int cpt;
        bool uc;  // uniform column coefficients (scalars)
        const void *kern;
    };
#define IQO_RYX_C(LZ_, P_, Q_, T_, NP_, PD_, ADJ_, CPT_)                                                        \
    {LZ_, P_, Q_, T_, NP_, ADJ_, CPT_, false, reinterpret_cast<const void *>(ryx_kernel<LZ_, P_, Q_, T_, NP_, PD_, ADJ_, CPT_>)}
#define IQO_RYX_UA(P_, Q_, T_, NP_, PD_, ADJ_)                                                                \
    {true, P_, Q_, T_, NP_, ADJ_, 2, true, reinterpret_cast<const void *>(ryx_kernel<true, P_, Q_, T_, NP_, PD_, ADJ_, 2, true>)}
#define IQO_RYX_U(P_, Q_, T_, NP_, PD_) IQO_RYX_UA(P_, Q_, T_, NP_, PD_, false), IQO_RYX_UA(P_, Q_, T_, NP_, PD_, true)
#define IQO_RYX_A(LZ_, P_, Q_, T_, NP_, PD_, ADJ_) IQO_RYX_C(LZ_, P_, Q_, T_, NP_, PD_, ADJ_, 2)
#define IQO_RYX(LZ_, P_, Q_, T_, NP_, PD_) IQO_RYX_A(LZ_, P_, Q_, T_, NP_, PD_, false)
#define IQO_RYX2(LZ_, P_, Q_, T_, NP_, PD_) IQO_RYX(LZ_, P_, Q_, T_, NP_, PD_), IQO_RYX_A(LZ_, P_, Q_, T_, NP_, PD_, true)
    static const Inst kInst[] = {
        IQO_RYX2(true, 9, 4, 12, 8, 2), IQO_RYX2(true, 9, 4, 12, 10, 2),  // Lanczos-3 9:4 (1080p -> 480p, -> 640x480)
        IQO_RYX2(true, 9, 4, 8, 6, 2), IQO_RYX2(true, 9, 4, 8, 7, 2),     // Lanczos-2 9:4
        IQO_RYX2(false, 9, 4, 4, 3, 2),                                   // Area 9:4
        IQO_RYX(true, 4, 1, 14, 13, 4), IQO_RYX(true, 4, 1, 14, 9, 4),  // Lanczos-3 / -2 4:1 (4K -> 960x540)
        IQO_RYX(true, 4, 1, 22, 17, 3),  // Lanczos-4 4:1 (round 6: 22 of 32 row taps; had run the general kernel)
        IQO_RYX(true, 2, 1, 4, 3, 2),                                   // Lanczos-1 2:1
        IQO_RYX(true, 2, 1, 12, 9, 3), IQO_RYX(true, 2, 1, 16, 11, 4),  // Lanczos-4 / -5 2:1
        IQO_RYX(true, 2, 1, 18, 13, 5), IQO_RYX(true, 2, 1, 20, 15, 5), // Lanczos-6 / -7 2:1
        IQO_RYX(true, 2, 1, 22, 17, 2), IQO_RYX(true, 2, 1, 24, 19, 2), // Lanczos-8 / -9 2:1
        IQO_RYX(true, 4, 9, 6, 4, 2), IQO_RYX(true, 4, 9, 4, 3, 2),     // Lanczos-3 / -2 4:9 up (480 -> 1080 rows)
        IQO_RYX_C(true, 4, 9, 6, 4, 2, false, 4),
        // Lanczos 2:1 columns (uniform coefficients): no per-lane coefficient registers; adjacent
        // column pairs (ryx_dev d.uc, d.adj)
        IQO_RYX_U(2, 1, 4, 3, 2), IQO_RYX_U(2, 1, 12, 9, 3), IQO_RYX_U(2, 1, 16, 11, 4), IQO_RYX_U(2, 1, 18, 13, 5), IQO_RYX_U(2, 1, 20, 15, 5),
        IQO_RYX_U(2, 1, 22, 17, IQO_RYX_UC_PD), IQO_RYX_U(2, 1, 24, 19, IQO_RYX_UC_PD),
    };
#undef IQO_RYX_U
#undef IQO_RYX_UA
#undef IQO_RYX2
#undef IQO_RYX
#undef IQO_RYX_A
#undef IQO_RYX_C
    const void *kern = nullptr;
    int trip = 0;
    bool kernUc = false;
    for (const Inst &k : kInst)
        if (k.lz == d.lanczos && k.P == d.P && k.Q == d.Q && k.T == d.taps && k.NP == d.NP && k.adj == (d.adj != 0) &&
            k.cpt == d.cpt && (!k.uc || d.uc) && (!kern || (k.uc && !kernUc))) {  // (the uniform-column one first)
            kernUc = k.uc;
            kern = k.kern;
            const int span = (k.P * (k.Q - 1)) / k.Q + k.T, nw0 = (span + k.P - 1) / k.P * k.P;
            const int nw = ((nw0 / k.P) * k.Q) % 2 ? nw0 + k.P : nw0;
            trip = nw / k.P * k.Q * 2;  // (as the kernel: output rows per trip) x 2
        }
    if (!kern)
        return hipErrorInvalidValue;
    if (d.parts < 1 || d.parts > 16)
        return hipErrorInvalidValue;
    const int threads = d.threads > 0 ? d.threads : 512;
    if (threads % 64 || threads > 512)
        return hipErrorInvalidValue;
    int maxSpan = d.srcW;
    if (d.parts > 1) {
        // part k: output columns [xs[k], xs[k+1]) (even bounds, <= 2 per thread), source columns
        // [cs[k], ce[k]) (multiples of 4, <= 4 per thread)
        if (d.xs[0] != 0 || d.xs[d.parts] != d.dstW)
            return hipErrorInvalidValue;
        maxSpan = 0;
        for (int k = 0; k < d.parts; ++k) {
            if (d.xs[k] % 2 || d.xs[k + 1] < d.xs[k] || d.xs[k + 1] - d.xs[k] > d.cpt * threads || d.cs[k] % 4 ||
                d.cs[k] < 0 || d.ce[k] > d.srcW || d.ce[k] - d.cs[k] > 4 * threads || d.ce[k] <= d.cs[k])
                return hipErrorInvalidValue;
            maxSpan = std::max(maxSpan, d.ce[k] - d.cs[k]);
        }
    } else if (d.srcW > 4 * threads || d.dstW > d.cpt * threads) {
        return hipErrorInvalidValue;
    }
    const int ldsBytes = 2 * (4 * kRyxPadK + 2 * ((maxSpan + 3) & ~3));
    const int groupBegin = rowBegin - rowBegin % d.Q;
    const int rows = rowEnd - groupBegin;
    // bands: ~2.5 rounds of resident workgroups, whole trips per band
    if (bands <= 0) {
        const int64_t resident = std::max(1, resident_waves(kern, threads, ldsBytes) / (threads / 64));
        const int64_t perBand = static_cast<int64_t>(io.frames) * d.parts;
        bands = static_cast<int>(std::min<int64_t>((5 * resident / 2 + perBand - 1) / perBand, std::max(1, rows / trip)));
    }
    bands = std::max(1, std::min(bands, (rows + d.Q - 1) / d.Q));
    int rpb = (rows + bands - 1) / bands;
    rpb = (rpb + d.Q - 1) / d.Q * d.Q;
    bands = (rows + rpb - 1) / rpb;
    const uint64_t nBlocks = static_cast<uint64_t>(bands) * static_cast<uint64_t>(io.frames) * static_cast<uint64_t>(d.parts);
    if (nBlocks >= (uint64_t(1) << 31))
        return hipErrorInvalidValue;
    RyxArgs a{d, io, rowBegin, rowEnd, groupBegin, rpb, bands, static_cast<int>(sb), static_cast<int>(db),
              static_cast<unsigned>(nBlocks)};
    void *args[] = {&a};
    return hipLaunchKernel(kern, dim3(static_cast<unsigned>(nBlocks)), dim3(static_cast<unsigned>(threads)), args,
                           static_cast<size_t>(ldsBytes), s);
}

static hipError_t iqo_ryg_einval(int where)
{
    if (getenv("IQO_DEBUG_LAUNCH"))
        fprintf(stderr, "launch_ryg: invalid argument at check %d\n", where);
    return hipErrorInvalidValue;
}

hipError_t launch_ryg(const RygDev &d, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s)
{
    if (rowEnd <= rowBegin || io.frames <= 0)
        return hipSuccess;
    if (d.srcW < 16 || d.srcW > 8192 || d.dstW > 4096 || !d.rowRec)
        return iqo_ryg_einval(1);
    const int64_t sb = static_cast<int64_t>(io.srcRowEnd - io.srcRow0 - 1) * io.srcSt + d.srcW;
    const int64_t db = static_cast<int64_t>(rowEnd - 1 - io.dstRow0) * io.dstSt + d.dstW;
    if (sb >= 0x7ff00000 || db >= 0x7ff00000 || io.srcSt >= (int64_t(1) << 24) || io.dstSt >= (int64_t(1) << 24))
        return iqo_ryg_einval(2);
    // instantiations (plan.cpp build_ryg kShapes): taps, column pairs; PD = 4 output rows ahead
    struct Inst {
        bool lz;
        int T, NP, cpt, nl;
        const void *kern;
        int run;  // ryu_kernel run mode: work-row dwords per 4 adjacent columns (0: off)
        int km;   // ryu_kernel: output rows per window position (at most)
    };
#define IQO_RYG_N(LZ_, T_, NP_, NL_)                                                                   \
    {LZ_, T_, NP_, 2, NL_, reinterpret_cast<const void *>(ryg_kernel<LZ_, T_, NP_, kRygPD, 2, NL_>), 0, 0},    \
    {LZ_, T_, NP_, 3, NL_, reinterpret_cast<const void *>(ryg_kernel<LZ_, T_, NP_, kRygPD, 3, NL_>), 0, 0},    \
    {LZ_, T_, NP_, 4, NL_, reinterpret_cast<const void *>(ryg_kernel<LZ_, T_, NP_, kRygPD, 4, NL_>), 0, 0}
#define IQO_RYG(LZ_, T_, NP_) IQO_RYG_N(LZ_, T_, NP_, 2)
    static const Inst kInst[] = {IQO_RYG(true, 4, 3),  IQO_RYG(true, 6, 4),  IQO_RYG(true, 8, 5),  IQO_RYG(true, 10, 5),
                                 IQO_RYG(true, 10, 6), IQO_RYG(true, 12, 7),
                                 IQO_RYG(true, 12, 8),  // (round 6: Lanczos-5 rows of 1 .. 2 : 1, 8 column pairs)
                                 IQO_RYG(true, 16, 10), IQO_RYG(true, 16, 12),  // (round 6: Lanczos-5 / -6 rows of 1 .. 2 : 1)
                                 // upscales (windows 0 or 1 rows apart: one new row per output row)
                                 IQO_RYG_N(true, 4, 3, 1), IQO_RYG_N(true, 6, 4, 1), IQO_RYG_N(true, 8, 5, 1),
                                 // Area downscales of 1 .. 2 : 1 (round 5: after the ring and the columns-per-thread rule)
                                 IQO_RYG(false, 3, 2), IQO_RYG(false, 3, 3),
                                 // Lanczos downscales of 2 .. 3 : 1 (windows 2 or 3 rows apart; 2 columns per thread)
                                 {true, 10, 6, 2, 3, reinterpret_cast<const void *>(ryg_kernel<true, 10, 6, kRygPD, 2, 3>), 0, 0},
                                 {true, 12, 7, 2, 3, reinterpret_cast<const void *>(ryg_kernel<true, 12, 7, kRygPD, 2, 3>), 0, 0},
                                 {true, 14, 8, 2, 3, reinterpret_cast<const void *>(ryg_kernel<true, 14, 8, kRygPD, 2, 3>), 0, 0},
                                 {true, 16, 9, 2, 3, reinterpret_cast<const void *>(ryg_kernel<true, 16, 9, kRygPD, 2, 3>), 0, 0},
                                 {true, 18, 10, 2, 3, reinterpret_cast<const void *>(ryg_kernel<true, 18, 10, kRygPD, 2, 3>), 0, 0},
                                 // (round 6: Lanczos-4 rows of 2 .. 3 : 1, 12 column pairs: 4K -> 1366x768 had run the tile kernel)
                                 {true, 18, 12, 2, 3, reinterpret_cast<const void *>(ryg_kernel<true, 18, 12, kRygPD, 2, 3>), 0, 0},
                                 // (round 6: Lanczos-5 rows of 2 .. 3 : 1, 22 taps, 16 column pairs, one workgroup per CU)
                                 {true, 22, 16, 2, 3, reinterpret_cast<const void *>(ryg_kernel<true, 22, 16, kRygPD, 2, 3>), 0, 0},
                                 // Area downscales of 2 .. 3 : 1
                                 {false, 4, 3, 2, 3, reinterpret_cast<const void *>(ryg_kernel<false, 4, 3, kRygPD, 2, 3>), 0, 0},
                                 {false, 4, 4, 2, 3, reinterpret_cast<const void *>(ryg_kernel<false, 4, 4, kRygPD, 2, 3>), 0, 0},
                                 // downscales of 3 .. 4 : 1 (windows 3 or 4 rows apart)
                                 {true, 14, 8, 2, 4, reinterpret_cast<const void *>(ryg_kernel<true, 14, 8, kRygPD, 2, 4>), 0, 0},
                                 {true, 16, 9, 2, 4, reinterpret_cast<const void *>(ryg_kernel<true, 16, 9, kRygPD, 2, 4>), 0, 0},
                                 {true, 18, 10, 2, 4, reinterpret_cast<const void *>(ryg_kernel<true, 18, 10, kRygPD, 2, 4>), 0, 0},
                                 {true, 20, 11, 2, 4, reinterpret_cast<const void *>(ryg_kernel<true, 20, 11, kRygPD, 2, 4>), 0, 0},
                                 {true, 22, 12, 2, 4, reinterpret_cast<const void *>(ryg_kernel<true, 22, 12, kRygPD, 2, 4>), 0, 0},
                                 {true, 24, 13, 2, 4, reinterpret_cast<const void *>(ryg_kernel<true, 24, 13, kRygPD, 2, 4>), 0, 0},
                                 // (round 6: Lanczos-4 rows of 3 .. 4 : 1, 16 column pairs, one workgroup per CU)
                                 {true, 22, 16, 2, 4, reinterpret_cast<const void *>(ryg_kernel<true, 22, 16, kRygPD, 2, 4>), 0, 0},
                                 {false, 5, 3, 2, 4, reinterpret_cast<const void *>(ryg_kernel<false, 5, 3, kRygPD, 2, 4>), 0, 0},
                                 {false, 5, 4, 2, 4, reinterpret_cast<const void *>(ryg_kernel<false, 5, 4, kRygPD, 2, 4>), 0, 0}};
#undef IQO_RYG_N
#undef IQO_RYG
    // upscale rows by window position (ryu_kernel): PD positions ahead (a trip of lcm(T, PD, 2))
#define IQO_RYU_K(T_, NP_, PD_, KM_)                                                                   \
    {true, T_, NP_, 2, 1, reinterpret_cast<const void *>(ryu_kernel<T_, NP_, PD_, 2, 0, KM_>), 0, KM_},  \
    {true, T_, NP_, 3, 1, reinterpret_cast<const void *>(ryu_kernel<T_, NP_, PD_, 3, 0, KM_>), 0, KM_},  \
    {true, T_, NP_, 4, 1, reinterpret_cast<const void *>(ryu_kernel<T_, NP_, PD_, 4, 0, KM_>), 0, KM_},  \
    {true, T_, NP_, 4, 1, reinterpret_cast<const void *>(ryu_kernel<T_, NP_, PD_, 4, NP_ + 1, KM_>), NP_ + 1, KM_}, \
    {true, T_, NP_, 4, 1, reinterpret_cast<const void *>(ryu_kernel<T_, NP_, PD_, 4, NP_ + 2, KM_>), NP_ + 2, KM_}
#define IQO_RYU(T_, NP_, PD_) IQO_RYU_K(T_, NP_, PD_, 2), IQO_RYU_K(T_, NP_, PD_, 3)
    static const Inst kUp[] = {IQO_RYU(4, 3, 4), IQO_RYU(6, 4, 3), IQO_RYU(8, 5, 4)};
#undef IQO_RYU
#undef IQO_RYU_K
    const void *kern = nullptr;
    const bool byPos = d.nl == 1 && d.posRec;
    for (const Inst &k : kInst)
        if (!byPos && k.lz == d.lanczos && k.T == d.taps && k.NP == d.NP && k.cpt == d.cpt && k.nl == d.nl)
            kern = k.kern;
    for (const Inst &k : kUp)
        if (byPos && d.lanczos && k.T == d.taps && k.NP == d.NP && k.cpt == d.cpt && k.run == (d.colRun ? d.run : 0) &&
            k.km == std::max(2, d.posRows))
            kern = k.kern;
    if (!kern || d.parts < 1 || d.parts > 16)
        return iqo_ryg_einval(3);
    const int threads = d.threads > 0 ? d.threads : 512;
    if (threads % 64 || threads > 512)
        return iqo_ryg_einval(4);
    int maxSpan = d.srcW;
    if (d.parts > 1) {
        if (d.xs[0] != 0 || d.xs[d.parts] != d.dstW)
            return iqo_ryg_einval(5);
        maxSpan = 0;
        for (int k = 0; k < d.parts; ++k) {
            if (d.xs[k] % 2 || d.xs[k + 1] < d.xs[k] || d.xs[k + 1] - d.xs[k] > d.cpt * threads || d.cs[k] % 4 ||
                d.cs[k] < 0 || d.ce[k] > d.srcW || d.ce[k] - d.cs[k] > 4 * threads || d.ce[k] <= d.cs[k])
                return iqo_ryg_einval(6);
            maxSpan = std::max(maxSpan, d.ce[k] - d.cs[k]);
        }
    } else if (d.srcW > 4 * threads || d.dstW > d.cpt * threads) {
        return iqo_ryg_einval(7);
    }
    const int ldsBytes = (byPos ? 2 * std::max(2, d.posRows) : 2) * (4 * kRyxPadK + 2 * ((maxSpan + 3) & ~3));
    const int rows = rowEnd - rowBegin;
    // bands: ~6 rounds of resident workgroups, >= 32 rows each (steady clock, x256: 1080p -> 1366x768
    // 12 bands 0.306 ms vs 5 bands 0.315, 1080p -> 1024x576 equal; profiles/r05/steady_ryg_bands.txt)
    if (bands <= 0) {
        const int64_t resident = std::max(1, resident_waves(kern, threads, ldsBytes) / (threads / 64));
        const int64_t perBand = static_cast<int64_t>(io.frames) * d.parts;
        // (round 6: ~3 rounds at 4 rows per output row, whose 22-24-row windows make a band's halo
        // costly -- 4K -> 1024x576 x128: 6 bands 0.485 ms, 12 bands 0.494, 18 0.506,
        // profiles/r06/c4_xcd_order.txt)
        // ryu_kernel (upscale rows by window position) likewise ~3 rounds: 1024x576 -> 1080p x256
        // 18 bands 0.259 ms, 9 bands 0.248, 6 bands 0.248; 1366x768 -> 1080p 0.285 / 0.269 / 0.269
        // (profiles/r06/band_sweeps.txt)
        const int rounds = d.nl >= 4 || byPos ? 3 : 6;
        bands = static_cast<int>(std::min<int64_t>((rounds * resident + perBand - 1) / perBand, std::max(1, rows / 32)));
    }
    bands = std::max(1, std::min(bands, rows));
    const int rpb = (rows + bands - 1) / bands;
    bands = (rows + rpb - 1) / rpb;
    const uint64_t nBlocks = static_cast<uint64_t>(bands) * static_cast<uint64_t>(io.frames) * static_cast<uint64_t>(d.parts);
    if (nBlocks >= (uint64_t(1) << 31))
        return iqo_ryg_einval(8);
    RygArgs a{d, io, rowBegin, rowEnd, rpb, bands, static_cast<int>(sb), static_cast<int>(db),
              static_cast<unsigned>(nBlocks)};
    void *args[] = {&a};
    return hipLaunchKernel(kern, dim3(static_cast<unsigned>(nBlocks)), dim3(static_cast<unsigned>(threads)), args,
                           static_cast<size_t>(ldsBytes), s);
}

hipError_t launch_u23(const U23Dev &d, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s)
{
    if (rowEnd <= rowBegin || io.frames <= 0)
        return hipSuccess;
    if (d.dstW % 12 || d.dstW < 24 || 3 * d.srcW != 2 * d.dstW)
        return hipErrorInvalidValue;
    const int64_t sb = static_cast<int64_t>(io.srcRowEnd - io.srcRow0 - 1) * io.srcSt + d.srcW;
    const int64_t db = static_cast<int64_t>(rowEnd - 1 - io.dstRow0) * io.dstSt + d.dstW;  // stores are relative to dstRow0
    if (sb >= 0x7ff00000 || db >= 0x7ff00000 || io.srcSt >= (int64_t(1) << 24) || io.dstSt >= (int64_t(1) << 24))
        return hipErrorInvalidValue;
    const int lanes = d.dstW / 12;
    int wpr = (lanes + 61) / 62;
    int np = d.np > 0 ? min(d.np, min(62, lanes)) : (lanes + wpr - 1) / wpr;
    wpr = (lanes + np - 1) / np;
    const void *kern = d.pd == 2 ? reinterpret_cast<const void *>(lanczos_u23_kernel<2>)
                                 : reinterpret_cast<const void *>(lanczos_u23_kernel<1>);
    const int row3Begin = rowBegin - rowBegin % 3;
    const int rows = rowEnd - row3Begin;
    constexpr int trip = 12;  // output rows per unrolled trip
    // bands: ~2.5 rounds of resident waves, whole trips per band, >= 24 rows
    if (bands <= 0) {
        const int64_t resident = std::max(1, resident_waves(kern, 256, 0));
        const int64_t perBand = static_cast<int64_t>(wpr) * io.frames;
        bands = static_cast<int>(std::min<int64_t>((5 * resident / 2 + perBand - 1) / perBand, std::max(1, rows / 24)));
    }
    bands = std::max(1, std::min(bands, (rows + trip - 1) / trip));
    int rpb = (rows + bands - 1) / bands;
    rpb = (rpb + trip - 1) / trip * trip;
    bands = (rows + rpb - 1) / rpb;
    const uint64_t nWaves = static_cast<uint64_t>(wpr) * bands * static_cast<uint64_t>(io.frames);
    if (nWaves >= (uint64_t(1) << 31))
        return hipErrorInvalidValue;
    U23Args a{d, io, rowBegin, rowEnd, row3Begin, rpb, bands, wpr, np, static_cast<int>(sb), static_cast<int>(db),
              static_cast<unsigned>(nWaves)};
    void *args[] = {&a};
    return hipLaunchKernel(kern, dim3(static_cast<unsigned>((nWaves + 3) / 4)), dim3(256), args, 0, s);
}

hipError_t launch_l23(const L23Dev &d, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s)
{
    if (rowEnd <= rowBegin || io.frames <= 0)
        return hipSuccess;
    if (d.dstW % 12 || d.dstW < 24 || 3 * d.srcW != 2 * d.dstW || d.srcW < 8)
        return hipErrorInvalidValue;
    const int64_t sb = static_cast<int64_t>(io.srcRowEnd - io.srcRow0 - 1) * io.srcSt + d.srcW;
    const int64_t db = static_cast<int64_t>(rowEnd - 1 - io.dstRow0) * io.dstSt + d.dstW;  // stores are relative to dstRow0
    if (sb >= 0x7ff00000 || db >= 0x7ff00000 || io.srcSt >= (int64_t(1) << 24) || io.dstSt >= (int64_t(1) << 24))
        return hipErrorInvalidValue;
    const int lanes = d.dstW / 12;
    int wpr = (lanes + 61) / 62;
    int np = d.np > 0 ? min(d.np, min(62, lanes)) : (lanes + wpr - 1) / wpr;
    wpr = (lanes + np - 1) / np;
    const void *kern = d.pd == 1 ? reinterpret_cast<const void *>(linear_u23_kernel<1>)
                                 : reinterpret_cast<const void *>(linear_u23_kernel<2>);
    const int row3Begin = rowBegin - rowBegin % 3;
    const int rows = rowEnd - row3Begin;
    constexpr int trip = 6;  // output rows per unrolled trip
    // bands: ~6 rounds of resident waves (no border code, a 4-row window), whole trips per band
    if (bands <= 0) {
        const int64_t resident = std::max(1, resident_waves(kern, 256, 0));
        const int64_t perBand = static_cast<int64_t>(wpr) * io.frames;
        bands = static_cast<int>(std::min<int64_t>((6 * resident + perBand - 1) / perBand, std::max(1, rows / 12)));
    }
    bands = std::max(1, std::min(bands, (rows + trip - 1) / trip));
    int rpb = (rows + bands - 1) / bands;
    rpb = (rpb + trip - 1) / trip * trip;
    bands = (rows + rpb - 1) / rpb;
    const uint64_t nWaves = static_cast<uint64_t>(wpr) * bands * static_cast<uint64_t>(io.frames);
    if (nWaves >= (uint64_t(1) << 31))
        return hipErrorInvalidValue;
    L23Args a{d, io, rowBegin, rowEnd, row3Begin, rpb, bands, wpr, np, static_cast<int>(sb), static_cast<int>(db),
              static_cast<unsigned>(nWaves)};
    void *args[] = {&a};
    return hipLaunchKernel(kern, dim3(static_cast<unsigned>((nWaves + 3) / 4)), dim3(256), args, 0, s);
}

hipError_t launch_a32(const A32Dev &d, const Io &io, int rowBegin, int rowEnd, int bands, hipStream_t s)
{
    if (rowEnd <= rowBegin || io.frames <= 0)
        return hipSuccess;
    if (d.dstW % 8 || d.dstW < 8 || 2 * d.srcW != 3 * d.dstW)
        return hipErrorInvalidValue;
    const int64_t sb = static_cast<int64_t>(io.srcRowEnd - io.srcRow0 - 1) * io.srcSt + d.srcW;
    const int64_t db = static_cast<int64_t>(rowEnd - 1 - io.dstRow0) * io.dstSt + d.dstW;  // stores are relative to dstRow0
    if (sb >= 0x7ff00000 || db >= 0x7ff00000 || io.srcSt >= (int64_t(1) << 24) || io.dstSt >= (int64_t(1) << 24))
        return hipErrorInvalidValue;
    const int lanes = d.dstW / 8;
    int wpr = (lanes + 63) / 64;
    int np = d.np > 0 ? min(d.np, min(64, lanes)) : (lanes + wpr - 1) / wpr;
    wpr = (lanes + np - 1) / np;
    const void *kern = d.pd == 2   ? reinterpret_cast<const void *>(area_d32_kernel<2>)
                       : d.pd == 8 ? reinterpret_cast<const void *>(area_d32_kernel<8>)
                                   : reinterpret_cast<const void *>(area_d32_kernel<4>);
    const int evenBegin = rowBegin & ~1;
    const int rows = rowEnd - evenBegin;
    // bands: ~6 rounds of resident waves, whole trips (8 rows) per band (fresh data, G3: 90 bands
    // of 8 rows 0.0712 ms vs 0.0742 at ~2.5 rounds; the kernel has no window, so short bands
    // cost nothing)
    if (bands <= 0) {
        const int64_t resident = std::max(1, resident_waves(kern, 256, 0));
        const int64_t perBand = static_cast<int64_t>(wpr) * io.frames;
        bands = static_cast<int>(std::min<int64_t>((6 * resident + perBand - 1) / perBand, std::max(1, rows / 8)));
    }
    bands = std::max(1, std::min(bands, (rows + 7) / 8));
    int rpb = (rows + bands - 1) / bands;
    rpb = (rpb + 7) & ~7;
    bands = (rows + rpb - 1) / rpb;
    const uint64_t nWaves = static_cast<uint64_t>(wpr) * bands * static_cast<uint64_t>(io.frames);
    if (nWaves >= (uint64_t(1) << 31))
        return hipErrorInvalidValue;
    A32Args a{d, io, rowBegin, rowEnd, evenBegin, rpb, bands, wpr, np, static_cast<int>(sb), static_cast<int>(db),
              static_cast<unsigned>(nWaves)};
    void *args[] = {&a};
    return hipLaunchKernel(kern, dim3(static_cast<unsigned>((nWaves + 3) / 4)), dim3(256), args, 0, s);
}

} // namespace iqo_amd
