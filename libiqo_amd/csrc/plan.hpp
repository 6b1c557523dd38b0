// plan.hpp -- host-side resize plan: quantised coefficient tables, per-row / per-column index
// maps and the fast-path decision.  Pure C++ (no HIP), built once per resizer and uploaded.
//
// The tables restate the reference's init() (table construction is host work there too):
//   Lanczos  src/IQOLanczosResizerImpl_Generic.cpp:32-191, 291-367
//   Area     src/IQOAreaResizerImpl_Generic.cpp:11-97, 174-248
//   Linear   src/IQOLinearResizerImpl_Generic.cpp:13-69, 157-208
// and the index maps restate the row/column drivers (resize / resizeX) so that every output
// coordinate carries (first source index, table phase, formula kind) exactly as the reference
// computes it -- including the shared-iterator behaviour of the Lanczos row loops
// (IQOLanczosResizerImpl_Generic.cpp:390-453) on images too small for a main region.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace iqo_amd {

enum Method { kLanczos = 0, kArea = 1, kLinear = 2 };

// Formula applied at one output coordinate of one axis.
enum Kind : int32_t {
    kMain = 0,      // interior formula (no masking)
    kBorderLo = 1,  // Lanczos: masked + renormalised; Linear: replicate first source px/row
    kBorderHi = 2,  // Lanczos: masked + renormalised; Linear: replicate last source px/row
    kIdentity = 3   // srcLen == dstLen shortcut of the reference (resize():378, resizeX():520)
};

// Per output coordinate record, uploaded as int4 {srcO, tabOff, kind, aux}.
struct CoordInfo {
    int32_t srcO;    // source index of tap 0 (may be < 0 or >= srcLen at Lanczos borders)
    int32_t tabOff;  // phase * taps (offset into the axis table)
    int32_t kind;    // Kind
    int32_t aux;     // Lanczos border denominator: Y = wrapped int16 sum of valid taps,
                     // X = int32 sum of valid taps; unused otherwise
};

struct AxisPlan {
    int srcLen = 0, dstLen = 0;
    int taps = 0, phases = 0;     // table geometry (reference m_NumCoefs*, m_NumTables*)
    std::vector<int32_t> table;   // phases * taps; int16 (Lanczos) or u16 (Area/Linear) values
    bool identity = false;
    int mainBegin = 0, mainEnd = 0;
    std::vector<CoordInfo> coord; // dstLen records
};

// Parameters of the fast kernels (IQO_KERNEL_* != GENERAL), filled when eligible.
struct FastLanczos {
    int KY = 0, KX = 0;           // integer decimation factors
    int NY = 0;                   // Y taps after trimming zero coefficients
    int offY = 0;                 // first tap row = KY*y + offY
    int NXP = 0;                  // X taps after trimming + padding to even start and even count
    int offX = 0;                 // first (padded) tap column = KX*x + offX (even)
    std::vector<int16_t> cy;      // NY
    std::vector<int16_t> cx;      // NXP (zero padded)
    // Symmetric streamer (kernels.hip lanczos_sym_kernel): symmetric Y table of even length,
    // X taps unpadded with an odd first column, so the taps of every output fall on odd-aligned
    // column pairs.
    bool sym = false;
    int NX = 0;                   // X taps after trimming zero coefficients (even)
    int offXO = 0;                // first tap column = KX*x + offXO (odd)
    std::vector<int16_t> cxo;     // NX
    int mainBeginY = 0, mainEndY = 0, mainBeginX = 0, mainEndX = 0;
    std::vector<int32_t> denoYTop, denoYBot; // wrapped int16 valid-tap sums per border row
    std::vector<int32_t> dXLeft, dXRight;    // 64 * valid-tap sum per border column
    // Exact division by multiply-high (Granlund-Montgomery), see magic_y / magic_x in plan.cpp.
    // Y border row r: int16(n * 64 / deno) = sign(n) * umulhi(|n| << yS, yM)      (|n| <= 2^15)
    // X edge value k (k < 4: columns k of the left edge lane; k >= 4: columns dstW - 8 + k of the
    // right edge lane): floor(s / D) = umulhi(s, xM) >> xT for 0 <= s < 2^31 (identity magic,
    // D = 2^20, for columns of those lanes that are not border columns).
    uint32_t yTopM[16] = {}, yBotM[16] = {}, xM[8] = {};
    int32_t yTopS[16] = {}, yBotS[16] = {}, xT[8] = {};
    uint32_t xM8[16] = {};  // the same for the edge lanes' 8 outputs each (Lanczos-5 2:1: 5 border
    int32_t xT8[16] = {};   //   columns per side; left lane k < 8, right lane k >= 8)
    // bit i: border row / column i divides by a negative denominator (the pxScale-2 chroma tables;
    // accumulator-ring streamer only)
    int yTopNeg = 0, yBotNeg = 0, xNeg = 0;
};

// Exact-division constants (exposed for tests): false if the divisor is outside the range the
// streamer's formulas are proven for.
bool magic_y(int32_t deno, uint32_t *m, int32_t *s);
bool magic_x(int64_t d, uint32_t *m, int32_t *t);

struct FastArea {
    int KY = 0, KX = 0;
    std::vector<uint16_t> cy, cx;
    bool lin = false;  // Linear at exactly 2:1 (taps 2i + 1, 2i + 2, replicated edges): linear_d2_body
};

struct FastLinear {
    int F = 2;  // exact factor (2 or 3): output F k + i (i = 1 .. F) blends samples k, k + 1, phase i % F
    uint16_t cy[3][2] = {}, cx[3][2] = {};
};

struct Plan {
    Method method = kLanczos;
    unsigned degree = 0;
    size_t pxScale = 1;
    int srcW = 0, srcH = 0, dstW = 0, dstH = 0;
    AxisPlan x, y;
    int kernel = 0;               // IQO_KERNEL_* for aligned full-frame calls
    FastLanczos flz;
    FastArea far;
    FastLinear fln;
};

// Tables of the separable tile kernel (kernels.hip tile_kernel): every shape the specialised
// kernels do not take.  Each output row and column is restated as ONE contiguous tap window
// (start, coefficients) with the reference's special cases folded in -- identity rows/columns
// become a single tap (64 / 2^14 for Lanczos Y / X, 256 / 2^15 for Area and Linear, which give
// the same rounding), Linear's replicated borders a single tap on the first / last source pixel,
// masked Lanczos border taps a zero coefficient -- so the kernel runs one formula per axis:
//   vertical:   work = sum_i px(clamp(start + i, lo, hi)) * c_i    (16-bit wrap, v_pk_mad_u16)
//   horizontal: sum = bias + sum_i work(clamp(a + i)) * pair_i   (v_dot2 over u16 pairs)
// Horizontal windows start on an even column a (one leading zero coefficient when the true start
// is odd), so every pair is one aligned dword of the work row.
struct TileRec {
    int32_t start, lo, hi, deno;  // row: first tap, clamp bounds, Lanczos border divisor (0 = main)
};
struct TileCol {
    int32_t a, D;                 // column: even window start, Lanczos border divisor * 64 (0 = main)
};
struct TileSpan {
    int32_t lo8, groups;          // column tile: first work column (multiple of 8), 8-column groups
};
struct TileTables {
    bool ok = false;
    int NP = 0;                   // coefficient pairs per column (instantiated count)
    int nYp = 0;                  // taps per row, padded to a multiple of 2 (zero coefficients)
    int CT = 256;                 // output columns per tile (256, 512 or 1024)
    int TH = 16;                  // output rows per tile
    int pitchDw = 0;              // LDS work-row pitch (dwords) = 4 * max groups
    int log2nQ = 6;               // log2(CT / 4): threads per row in the horizontal pass
    int srcRows = 0;              // source rows staged per tile: max over any TH consecutive rows
    int spitch = 0;               // staged source row pitch (bytes) = 8 * max groups
    std::vector<TileRec> rows;    // dstH
    std::vector<uint32_t> rowCoef;// dstH x nYp, (c, c) u16 splats
    std::vector<TileCol> cols;    // dstW
    std::vector<uint32_t> colCoef;// dstW x NP, (c_2p, c_2p+1) u16 pairs from the even start
    std::vector<TileSpan> spans;  // ceil(dstW / CT)
};
// Instantiated pair counts of the tile kernel; build_tile_tables rounds NP up to one of these.
constexpr int kTileNP[] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 16};
void build_tile_tables(const Plan &p, TileTables *t);
// Rows per tile: LDS bytes of a workgroup, staged source rows, and setting TH (false if the
// workgroup would need more than 64 KiB of LDS).
size_t tile_lds_bytes(const Plan &p, const TileTables &t, int TH);
int tile_src_rows(const Plan &p, const TileTables &t, int TH);
bool tile_set_rows(const Plan &p, TileTables *t, int TH);

// Geometry of the general-ratio band walker (kernels.hip walk_kernel) over the tile tables:
// column tiles of CTW output columns (at most 1024: one quad of 4 columns per thread), each with
// its work-column span in 4-column units, and an LDS ring of R source rows.
struct WalkSpan {
    int32_t lo8, units;           // first work column (multiple of 8), 4-column units
    int32_t interior;             // 256 columns, none of them a masked border column
};
struct WalkRow {
    int32_t lo, hi;               // clamped source row window of the output row
    int32_t hiSlot;               // hi % R
    int32_t deno;                 // masked border row divisor (0: none)
};
struct WalkSeg {
    int32_t first;                // first source row the output row needs that its predecessor did not
    int32_t slotOff;              // ring byte offset of that row ((first % R) * pitch)
    int32_t border;               // masked border row: int16(n * 64 / deno) by magic_y (yM, yS)
    int32_t firstD;               // first of the output row kWalkPrefetch below (the load look-ahead)
    uint32_t yM;                  // 0 for a divisor of 0 (quotient 0, as in general_kernel)
    int32_t yS, yNeg, pad;        // yNeg: the divisor is negative
};
// The wave walker (kernels.hip walk_kernel): every wave owns a strip of kWalkStrip output columns
// of one band of rows and walks it top to bottom through a private LDS ring of R source rows,
// widened to u16 (8 bytes per 4-column unit, NV units per lane).
constexpr int kWalkStrip = 256;   // output columns per wave (4 per lane, one dword store)
constexpr int kWalkPrefetch = 4;  // output rows of load look-ahead (kernels.hip kWalkD)
struct WalkTables {
    bool ok = false;
    int NV = 0;                   // units per lane (1, 2): a strip reads at most 256 * NV source columns
    int nS = 0;                   // strips per row
    std::vector<WalkSpan> spans;  // nS
    int maxUnits = 0;             // <= 64 * NV
    int R = 0, pitch = 0;         // ring rows (widest row window + NV), ring row pitch (bytes)
    int maxNew = 0;               // most source rows first needed by one output row (<= NV)
    std::vector<WalkRow> rows;    // dstH
    std::vector<WalkSeg> segs;    // dstH + kWalkPrefetch + 1 (the look-ahead reads past the last row)
    std::vector<uint32_t> rowTap; // (dstH + 1) x nYp x {coef splat, ring byte offset of the clamped row}
    size_t waveBytes = 0;         // LDS per wave: ring + work row + sink
};
void build_walk_tables(const Plan &p, const TileTables &t, WalkTables *w);

// Exact 2x and 3x Lanczos upscales (kernels.hip lanczos_up2_kernel).  Output y (x) = F k + j: phase
// 0 is the source sample k times one coefficient, phases 1 .. F-1 take NT = 2 * degree taps starting
// at k + 1 - NT/2, one coefficient set per phase, at the masked borders too.  The kernel takes every
// row and column: source rows / columns outside the image read as zero, and the border rows
// (<= 16 per side) and columns (<= 8F per side) are divided in the kernel.
struct Up2Tables {
    bool ok = false;
    int F = 0;                      // factor (2 or 3): output y = F k + j takes phase j
    int NT = 0;
    int m0 = 0, m1 = 0;             // main rows; the others are masked border rows
    uint32_t xM[2][24] = {};        // edge lanes (left: columns 0 .. 8F-1, right: dstW - 8F ..):
    int32_t xT[2][24] = {};         //   floor(s / D) = umulhi(s, xM) >> xT (D = 2^20 off the border)
    uint32_t yM[2][16] = {};        // border row y (top: y, bottom: y - m1): int16(n * 64 / deno)
    int32_t yS[2][16] = {};
    uint32_t cy0 = 0, cy1[2][6] = {};  // (c, c) u16 splats: phase 0's single tap, phases 1 .. F-1
    uint32_t cx0 = 0, cx1[2][3] = {};  // (c, 0) / (c_2q, c_2q+1) int16 pairs, same phases
};
void build_up2(const Plan &p, const WalkTables &w, Up2Tables *u);

// Exact 3:2 Lanczos-2/3 downscale (kernels.hip lanczos_d32_kernel), e.g. 1920x1080 -> 1280x720.  In
// the reference's tables for this ratio output y (x) takes the taps of phase y & 1 starting at
// 3 * (y >> 1) + B + (y & 1) (Lanczos-3: 10 taps, B = -4; Lanczos-2: 6 taps, B = -2).  Output rows
// come in groups m (rows 2m, 2m+1) over the source rows 3m + B .. (Lanczos-3: 10 rows, the even
// row's non-zero taps group rows 0..7, the odd row's 2..9; Lanczos-2: 7 rows, 0..4 and 2..6).  The kernel
// takes every row and column: source rows / columns outside the image read as zero, so the masked
// border numerators come out of the same sums, and the <= 8 border rows / columns per side are
// divided in the kernel.
struct D32Tables {
    bool ok = false;
    int variant = 0;                // tap structure: 0 Lanczos-3 (10 taps), 1 Lanczos-2 (6 taps)
    int m0 = 0, m1 = 0;             // main rows; rows y < m0 and y >= m1 are masked border rows
    uint32_t yM[2][8] = {};         // border row y (top: y, bottom: y - m1): int16(n * 64 / deno)
    int32_t yS[2][8] = {};          //   by magic_y
    uint32_t cy[2][8] = {};         // (c, c) u16 splats: phase p's taps at group rows 2p .. 2p + 7
    uint32_t cx[2][5] = {};         // phase p's (c_2q, c_2q+1) int16 pairs from its window start
    uint32_t xM[2][8] = {};         // edge lanes (left: columns 0..7, right: dstW - 8 .. dstW - 1):
    int32_t xT[2][8] = {};          //   floor(s / D) = umulhi(s, xM) >> xT (D = 2^20 off the border)
};
void build_d32(const Plan &p, const WalkTables &w, D32Tables *d);

// Exact 3:1 Lanczos-2/3 downscale (kernels.hip lanczos_d31_kernel), e.g. 3840x2160 -> 1280x720.  In
// the reference's tables for this ratio output y (x) takes the single phase's T taps (18 / 12) from
// source row 3y + B (B = -8 / -5); tap 0 is zero and taps 1 .. T-1 are symmetric about the centre
// tap T/2, so a row is the centre row times its coefficient plus pair sums times theirs.  Border
// rows / columns (<= 8 rows, <= 4 columns per side) are masked in the kernel.
struct D31Tables {
    bool ok = false;
    int variant = 0;                // 0 Lanczos-3 (18 taps), 1 Lanczos-2 (12 taps)
    int m0 = 0, m1 = 0;             // main rows; the others are masked border rows
    uint32_t cc = 0, cp[5] = {};    // (c, c) u16 splats: centre tap, symmetric pair taps (kernel order)
    uint32_t cxe[9] = {}, cxo[9] = {};  // (c_2q, c_2q+1) / (c_2q+1, c_2q+2) int16 pairs
    uint32_t xM[2][4] = {};         // edge lanes (left: columns 0..3, right: dstW - 4 ..)
    int32_t xT[2][4] = {};
    uint32_t yM[2][8] = {};         // border row y (top: y, bottom: y - m1)
    int32_t yS[2][8] = {};
};
void build_d31(const Plan &p, D31Tables *t);

// Exact vertical ratio P:Q, any horizontal ratio (kernels.hip ryx_kernel), e.g. 1920x1080 ->
// 854x480 (Y 9:4, X 960:427).  Rows: output y = Q m + j reads the taps of phase j from source row
// P m + floor(P j / Q) + OFF (OFF = 1 - taps/2 for Lanczos, 0 for Area); the vertical pass keeps a
// register window of source rows.  Columns: every output column's window (even start, a leading
// zero coefficient when the reference's start is odd) and coefficient pairs come from a table, with
// an exact division constant per column (Lanczos border columns; the identity 2^20 elsewhere).
struct RyxTables {
    bool ok = false;
    int P = 0, Q = 0, taps = 0, off = 0;   // the instantiation this plan needs (kernels.hip launch_ryx)
    int NP = 0;                            // coefficient pairs per column
    int m0 = 0, m1 = 0;                    // Lanczos main rows; the others are masked border rows
    uint32_t yM[2][16] = {};               // border row y (top: y, bottom: y - m1): magic_y
    int32_t yS[2][16] = {};
    std::vector<uint32_t> rowCoef;         // Q x taps (c, c) u16 splats: phase j's taps
    std::vector<int32_t> cols;             // dstW x 4: {work byte offset of the even start, magic, shift, 0}
    std::vector<uint32_t> colCoef;         // dstW x NP coefficient pairs from the even start
    // general rows (build_ryg, kernels.hip ryg_kernel): no exact P:Q; every output row y has its own
    // record {first window row, offset of its phase's taps in rowCoef} and consecutive windows
    // start 1 or 2 rows apart (downscales of 1 .. 2 : 1)
    bool general = false;
    int rowLoads = 2;                      // general rows: 2 (downscale), 1 (upscale) new rows per output row
    std::vector<int32_t> rowRec;           // dstH x 2
    // general upscale rows walked by window position (build_ryu_positions, kernels.hip ryu_kernel):
    // record s - posBase = {first output row whose window starts at s, rows (1 .. kRyuMaxRows), tap
    // offsets of those rows (then repeats)}, kRyuRec ints each, kRyuPosPad padding records; empty:
    // no such walk
    std::vector<int32_t> posRec;
    int posBase = 0;
    int posRows = 0;  // the most rows any position holds (downscales: 1, positions between rows hold 0)
    // run mode of the upscale walk (build_ryu_runs): groups of 4 adjacent output columns (x = 4g ..
    // 4g + 3) read one run of runPairs work-row dwords from the group's lowest even start; column x's
    // coefficient pairs at their offset in a zero-padded run: dstW x runPairs; empty: per-column mode
    std::vector<uint32_t> colRun;
    int runPairs = 0;
};
// Work-row padding (u16 entries) left of source column 0 in the kernel's LDS work row.
constexpr int kRyxPad = 24;
constexpr int kRygRecPad = 8;  // build_ryg: row records repeated past the last row (kernels.hip ryg_kernel)
void build_ryx(const Plan &p, RyxTables *t);
// The general-row variant of build_ryx (IQO_KERNEL_RYG): Lanczos and Area downscales whose rows
// shrink by more than 1 and at most 2 (e.g. 1080 -> 768, 1080 -> 576) and that no exact-ratio
// kernel takes.  Tabled rows and columns; the kernel's register window advances 1 or 2 rows.
void build_ryg(const Plan &p, RyxTables *t);
// Window-position records of a general upscale (build_ryg with rowLoads 1), in t->posRec / posBase.
// At an upscale the reference's srcOY advances by 0 or 1 per output row, so every window position
// between the first and the last holds at least one row; the kernel takes positions of up to
// kRyuMaxRows rows (rows that grow by at most 3).  Returns false (and leaves posRec empty) otherwise.
constexpr int kRyuPosPad = 8;  // records past the last position (ryu_kernel reads a band's last + 2)
constexpr int kRyuRec = 8;     // ints per position record: {first row, rows, tap offsets of 6 rows}
constexpr int kRyuMaxRows = 3; // rows per position the kernel instantiates (rows that grow by <= 3)
bool build_ryu_positions(int dstH, RyxTables *t);
// The run-mode column table (colRun / runPairs) for groups of 4 adjacent columns whose windows fit in
// NP + 1 or NP + 2 dwords from the group's first even start (upscaled columns); false otherwise.
bool build_ryu_runs(int dstW, RyxTables *t);

// Exact 2:3 Lanczos-3 upscale (kernels.hip lanczos_u23_kernel), e.g. 1280x720 -> 1920x1080.  In the
// reference's tables for this ratio output y (x) = 3m + j takes phase j: j = 0 a single tap on
// source row 2m, j = 1 six taps from 2m - 2, j = 2 six taps from 2m - 1 (at the masked borders
// too).  A group of 3 output rows reads source rows 2m - 2 .. 2m + 4 and adds 2 of them.
struct U23Tables {
    bool ok = false;
    int m0 = 0, m1 = 0;             // main rows; the others are masked border rows
    uint32_t cy0 = 0;               // (c, c) splat of phase 0's single tap
    uint32_t cy[2][6] = {};         // (c, c) splats of phases 1 and 2
    uint32_t cx0 = 0;               // (c, 0) pair of phase 0's tap
    uint32_t cx[2][3] = {};         // phases 1, 2: (c_2q, c_2q+1) int16 pairs
    uint32_t xM[2][12] = {};        // edge lanes (left: columns 0..11, right: dstW - 12 ..)
    int32_t xT[2][12] = {};
    uint32_t yM[2][8] = {};         // border row y (top: y, bottom: y - m1)
    int32_t yS[2][8] = {};
};
void build_u23(const Plan &p, U23Tables *t);

// Exact 2:3 Linear upscale (kernels.hip linear_u23_kernel), e.g. 1280x720 -> 1920x1080: output
// y (x) = 3m + j takes phase j's two taps from source 2m + j - 1.  With the source clamped to the
// image the same formula gives the reference's replicated border pixels (the coordinates it marks
// as borders have both taps on the edge pixel), so the kernel has no border code.
struct L23Tables {
    bool ok = false;
    uint32_t cy[3][2] = {};         // (c, c) u16 splats of phase j's two taps
    uint32_t cx[3] = {};            // phase j's (c_0, c_1) u16 pair
};
void build_l23(const Plan &p, L23Tables *t);

// Exact 3:2 Area downscale (kernels.hip area_d32_kernel), e.g. 1920x1080 -> 1280x720: output y (x)
// takes the 2 non-zero taps of phase y & 1 starting at 3 (y >> 1) + (y & 1) (the third tap of the
// reference's table is 0), so a row pair reads exactly the 3 source rows 3m .. 3m + 2 and a lane's
// 8 outputs exactly its own 12 source columns.
struct A32Tables {
    bool ok = false;
    uint32_t cy[2][2] = {};         // (c, c) u16 splats of phase p's two taps
    uint32_t cx[2] = {};            // phase p's (c_0, c_1) u16 pair
};
void build_a32(const Plan &p, A32Tables *t);

// Build the full plan.  Returns false (with *err) for invalid arguments.
bool build_plan(Method m, unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                size_t pxScale, Plan *out, std::string *err);

// Tables only (cheap; used by the host-only ABI query).
bool build_tables(Method m, unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                  size_t pxScale, AxisPlan *x, AxisPlan *y, std::string *err);

// Source rows read by output rows [r0, r1) (global indices; clamped to [0, srcH)).
void band_src_rows(const Plan &p, int r0, int r1, int *s0, int *s1);

} // namespace iqo_amd
