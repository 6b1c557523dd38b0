// plan.cpp -- host plan construction (see plan.hpp).  Floating-point evaluation follows the
// reference's types and operation order exactly (double windowed sinc, float sums and float
// quantisation), compiled without fast-math so the quantised tables are reproducible.
#include "plan.hpp"

#include <algorithm>
#include <numeric>
#include <cmath>
#include <cstdlib>

namespace iqo_amd {
namespace {

// ---------------------------------------------------------------- integer helpers (src/math.hpp)

int64_t gcd_ref(int64_t a, int64_t b)  // math.hpp:37-49 (result sign as the reference's)
{
    for (int64_t r = a % b; r != 0; r = a % b) {
        a = b;
        b = r;
    }
    return b;
}

int64_t floor_div(int64_t a, int64_t b)  // math.hpp:58-65
{
    return ((a ^ b) < 0) ? (a - b + 1) / b : a / b;
}

// Exact rational stepping of floor(x * dy / dx) -- math.hpp:70-155 (LinearIterator).
class RationalStep {
public:
    RationalStep(int64_t dx, int64_t dy) : dx_(dx), dy_(dy), x_(0), y_(0) {}
    void seek(int64_t x)  // setX(x), math.hpp:87-91
    {
        x_ = (x * dy_) % dx_;
        y_ = (x * dy_) / dx_;
    }
    void seek_rational(int64_t nume, int64_t deno)  // setX(nume, deno), math.hpp:96-112
    {
        y_ = floor_div(nume * dy_, deno * dx_);
        int64_t n = nume * dx_, ndy = dy_ * deno, ndx = dx_ * deno;
        int64_t g = std::llabs(gcd_ref(n, gcd_ref(ndy, ndx)));
        n /= g;
        ndy /= g;
        ndx /= g;
        x_ = n % ndx;
        if (x_ < 0)
            x_ += ndx;
        dx_ = ndx;
        dy_ = ndy;
    }
    void step(int64_t a)  // advance(a), math.hpp:142-149
    {
        x_ += a * dy_;
        while (x_ >= dx_) {
            ++y_;
            x_ -= dx_;
        }
    }
    int64_t next()  // *it++
    {
        int64_t v = y_;
        step(1);
        return v;
    }

private:
    int64_t dx_, dy_, x_, y_;
};

size_t first_max(const std::vector<float> &v)  // std::max_element: first of equal maxima
{
    size_t k = 0;
    for (size_t i = 1; i < v.size(); ++i)
        if (v[k] < v[i])
            k = i;
    return k;
}

// Quantise so the taps sum exactly to `bias`, +-1 fix-ups at the current float maximum,
// zeroing it each time.  Lanczos :341-367 (int16) and Area :222-248 (u16) share this scheme.
template <typename Q>
void quantise(std::vector<float> f, float sum, int bias, int32_t *out)
{
    const size_t n = f.size();
    int total = 0;
    for (size_t i = 0; i < n; ++i) {
        float scaled = f[i] * static_cast<float>(bias) / sum;
        // iqo::round<float> (math.hpp:12-16), then the narrowing the reference's x86-64 build
        // performs: truncate to int32, keep the low 16 bits (explicit, so it is not UB here).
        Q q = static_cast<Q>(static_cast<int32_t>(std::floor(scaled + 0.5f)));
        out[i] = q;
        total += q;
    }
    for (; total < bias; ++total) {
        size_t k = first_max(f);
        out[k] = static_cast<Q>(out[k] + 1);
        f[k] = 0;
    }
    for (; total > bias; --total) {
        size_t k = first_max(f);
        out[k] = static_cast<Q>(out[k] - 1);
        f[k] = 0;
    }
}

// ---------------------------------------------------------------- Lanczos window

double lanczos_weight(int degree, double x)  // IQOLanczosResizerImpl_Generic.cpp:10-29
{
    const double pi = 3.14159265358979;
    double ax = std::fabs(x);
    if (std::fmod(ax, 1.0) < 1e-5)
        return ax < 1e-5 ? 1.0 : 0.0;
    if (static_cast<double>(degree) <= ax)
        return 0.0;
    double px = pi * x, pxa = pi * (x / degree);
    return (std::sin(px) / px) * (std::sin(pxa) / pxa);
}

// calcNumCoefsForLanczos, :32-96
int lanczos_taps(int degree, size_t rs, size_t rd, size_t pxScale)
{
    if (rs <= rd)
        return 2 * degree;
    size_t d2 = std::max<size_t>(1, static_cast<size_t>(degree) / pxScale);
    return static_cast<int>(2 * static_cast<ptrdiff_t>(std::ceil(static_cast<double>(d2 * rs) / static_cast<double>(rd))));
}

// setLanczosTable, :111-191 -- returns float sum; fills f[taps]
float lanczos_phase(int degree, size_t rs, size_t rd, ptrdiff_t phase, size_t px, std::vector<float> &f)
{
    double begin;
    if (rs > rd) {
        int degFactor = std::max(1, static_cast<int>(px) / degree);
        size_t r = static_cast<size_t>(phase) * rs % rd;
        begin = static_cast<double>(-degree * degFactor) - 0.5 * static_cast<double>(px) +
                0.5 * static_cast<double>(rd) * static_cast<double>(px) / static_cast<double>(rs) +
                static_cast<double>((rd - r) * px % rs) / static_cast<double>(rs);
    } else {
        double off = std::fmod(static_cast<double>(static_cast<size_t>(phase) * rs) / static_cast<double>(rd), 1.0);
        begin = -degree + 1.0 - off;
        rs = rd;
        px = 1;
    }
    float sum = 0;
    for (size_t i = 0; i < f.size(); ++i) {
        double x = begin + static_cast<double>(i * rd * px) / static_cast<double>(rs);
        f[i] = static_cast<float>(lanczos_weight(degree, x));
        sum += f[i];
    }
    return sum;
}

// ---------------------------------------------------------------- Area boxes

int area_taps(size_t rs, size_t rd)  // calcNumCoefsForArea, IQOAreaResizerImpl_Generic.cpp:11-65
{
    if (rs < rd)
        return 1;
    size_t whole = (rs / rd) * rd;
    size_t n = (rs + rd - 1) / rd;
    int64_t g = gcd_ref(static_cast<int64_t>(rs), static_cast<int64_t>(whole));
    int64_t l = static_cast<int64_t>(rs) / g * static_cast<int64_t>(whole);
    if (l > static_cast<int64_t>(rs))
        ++n;
    return static_cast<int>(n);
}

float area_phase(size_t rs, size_t rd, ptrdiff_t phase, std::vector<float> &f)  // setAreaTable :74-97
{
    double b = static_cast<double>(static_cast<size_t>(phase) * rs) / static_cast<double>(rd);
    double e = static_cast<double>(static_cast<size_t>(phase + 1) * rs) / static_cast<double>(rd);
    float sum = 0;
    for (size_t i = 0; i < f.size(); ++i) {
        double nx = std::min(e, std::floor(b) + 1.0);
        f[i] = static_cast<float>(nx - b);
        sum += f[i];
        b = nx;
    }
    return sum;
}

// ---------------------------------------------------------------- axis builders

struct Reduced {
    size_t rs, rd;
};

Reduced reduce(size_t s, size_t d)
{
    size_t g = static_cast<size_t>(gcd_ref(static_cast<int64_t>(s), static_cast<int64_t>(d)));
    return Reduced{s / g, d / g};
}

void tables_lanczos(unsigned degree, size_t s, size_t d, size_t px, int bias, AxisPlan *a)
{
    Reduced r = reduce(s, d);
    a->taps = lanczos_taps(static_cast<int>(degree), r.rs, r.rd, px);
    a->phases = static_cast<int>(r.rd);
    a->table.assign(static_cast<size_t>(a->taps) * a->phases, 0);
    std::vector<float> f(static_cast<size_t>(a->taps));
    for (int q = 0; q < a->phases; ++q) {
        float sum = lanczos_phase(static_cast<int>(degree), r.rs, r.rd, q, px, f);
        quantise<int16_t>(f, sum, bias, &a->table[static_cast<size_t>(q) * a->taps]);
    }
}

void tables_area(size_t s, size_t d, int bias, AxisPlan *a)
{
    Reduced r = reduce(s, d);
    a->taps = area_taps(r.rs, r.rd);
    a->phases = static_cast<int>(r.rd);
    a->table.assign(static_cast<size_t>(a->taps) * a->phases, 0);
    std::vector<float> f(static_cast<size_t>(a->taps));
    for (int q = 0; q < a->phases; ++q) {
        float sum = area_phase(r.rs, r.rd, q, f);
        quantise<uint16_t>(f, sum, bias, &a->table[static_cast<size_t>(q) * a->taps]);
    }
}

// setLinearTable + adjustCoefs, IQOLinearResizerImpl_Generic.cpp:29-69, 193-208
void tables_linear(size_t s, size_t d, int bias, AxisPlan *a)
{
    Reduced r = reduce(s, d);
    a->taps = 2;
    a->phases = static_cast<int>(r.rd);
    a->table.assign(2 * static_cast<size_t>(a->phases), 0);
    for (size_t i = 0; i < r.rd; ++i) {
        double ip;
        double x = static_cast<double>(i);
        float c1 = static_cast<float>(std::modf((x + 0.5) * static_cast<double>(r.rs) / static_cast<double>(r.rd) + 0.5, &ip));
        float c0 = 1.0f - c1;
        uint16_t q0 = static_cast<uint16_t>(static_cast<int32_t>(std::floor(c0 * static_cast<float>(bias) + 0.5f)));
        a->table[2 * i] = q0;
        a->table[2 * i + 1] = static_cast<uint16_t>(bias - q0);
    }
}

int clampi(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

// Lanczos Y map: simulate the three row loops with their SHARED iterator and table cursor
// (:390-453); a later loop overwrites rows an earlier one wrote when mainEnd < mainBegin.
void coords_lanczos_y(AxisPlan *a)
{
    const int64_t s = a->srcLen, d = a->dstLen, m = a->taps / 2;
    a->coord.assign(static_cast<size_t>(d), CoordInfo{0, 0, kMain, 0});
    if (s == d) {
        a->identity = true;
        for (int64_t y = 0; y < d; ++y)
            a->coord[y] = CoordInfo{static_cast<int32_t>(y), 0, kIdentity, 0};
        return;
    }
    int64_t mb = ((m - 1) * d + s - 1) / s;
    int64_t me = std::max<int64_t>(0, (s - m) * d / s);
    a->mainBegin = static_cast<int>(mb);
    a->mainEnd = static_cast<int>(me);
    RationalStep it(d, s);
    int64_t cursor = 0;
    auto emit = [&](int64_t y, int32_t kind) {
        int64_t o = it.next() + 1;
        CoordInfo c{static_cast<int32_t>(o - m), static_cast<int32_t>(cursor), kind, 0};
        cursor += a->taps;
        if (cursor == static_cast<int64_t>(a->taps) * a->phases)
            cursor = 0;
        if (kind != kMain) {
            int16_t den = 0;  // wrapped int16 sum over valid rows (resizeYborder :477-485)
            for (int i = 0; i < a->taps; ++i) {
                int64_t r = c.srcO + i;
                if (r >= 0 && r < s)
                    den = static_cast<int16_t>(den + a->table[c.tabOff + i]);
            }
            c.aux = den;
        }
        a->coord[static_cast<size_t>(y)] = c;
    };
    for (int64_t y = 0; y < mb; ++y)
        emit(y, kBorderLo);
    for (int64_t y = mb; y < me; ++y)
        emit(y, kMain);
    for (int64_t y = me; y < d; ++y)
        emit(y, kBorderHi);
}

// Lanczos X map (resizeX / resizeXborder / resizeXmain, :518-612): each column is independent.
void coords_lanczos_x(AxisPlan *a)
{
    const int64_t s = a->srcLen, d = a->dstLen, m = a->taps / 2;
    a->coord.assign(static_cast<size_t>(d), CoordInfo{0, 0, kMain, 0});
    if (s == d) {
        a->identity = true;
        for (int64_t x = 0; x < d; ++x)
            a->coord[x] = CoordInfo{static_cast<int32_t>(x), 0, kIdentity, 0};
        return;
    }
    int64_t mb = ((m - 1) * d + s - 1) / s;
    int64_t me = std::max<int64_t>(0, (s - m) * d / s);
    a->mainBegin = static_cast<int>(mb);
    a->mainEnd = static_cast<int>(me);
    for (int64_t x = 0; x < d; ++x) {
        CoordInfo c;
        c.srcO = static_cast<int32_t>(x * s / d + 1 - m);
        c.tabOff = static_cast<int32_t>((x % a->phases) * a->taps);
        c.kind = (x >= me) ? kBorderHi : (x < mb ? kBorderLo : kMain);
        c.aux = 0;
        if (c.kind != kMain) {
            int32_t den = 0;  // int32 sum over valid columns (resizeXborder :563-570)
            for (int i = 0; i < a->taps; ++i) {
                int64_t col = c.srcO + i;
                if (col >= 0 && col < s)
                    den += a->table[c.tabOff + i];
            }
            c.aux = den;
        }
        a->coord[static_cast<size_t>(x)] = c;
    }
}

// Area map: o = floor(i*s/d), phase i mod rd (IQOAreaResizerImpl_Generic.cpp:271-293, 340-368)
void coords_area(AxisPlan *a)
{
    const int64_t s = a->srcLen, d = a->dstLen;
    a->coord.resize(static_cast<size_t>(d));
    a->identity = (s == d);
    a->mainBegin = 0;
    a->mainEnd = static_cast<int>(d);
    for (int64_t i = 0; i < d; ++i) {
        if (a->identity)
            a->coord[i] = CoordInfo{static_cast<int32_t>(i), 0, kIdentity, 0};
        else
            a->coord[i] = CoordInfo{static_cast<int32_t>(i * s / d), static_cast<int32_t>((i % a->phases) * a->taps), kMain, 0};
    }
}

// Linear map (IQOLinearResizerImpl_Generic.cpp:210-282, 327-407): border width from
// convertCoordinate(srcLen, dstLen, 0) (always 1, :13-22); interior origin from
// LinearIterator(d, s).setX(s - d, 2d) advanced to mainBegin.
void coords_linear(AxisPlan *a)
{
    const int64_t s = a->srcLen, d = a->dstLen;
    a->coord.resize(static_cast<size_t>(d));
    if (s == d) {
        a->identity = true;
        for (int64_t i = 0; i < d; ++i)
            a->coord[i] = CoordInfo{static_cast<int32_t>(i), 0, kIdentity, 0};
        return;
    }
    double toX = (0.5 + static_cast<double>(s)) * 0.0 / static_cast<double>(d) - 0.5;
    int mb0 = static_cast<int>(std::ceil(std::fabs(toX)));
    int mb = clampi(0, static_cast<int>(d), mb0);
    int me = clampi(0, static_cast<int>(d), static_cast<int>(d) - mb);
    a->mainBegin = mb;
    a->mainEnd = me;
    RationalStep it(d, s);
    it.seek_rational(s - d, 2 * d);
    it.step(mb);
    for (int64_t i = 0; i < d; ++i) {
        if (i >= me)
            a->coord[i] = CoordInfo{static_cast<int32_t>(s - 1), 0, kBorderHi, 0};
        else if (i < mb)
            a->coord[i] = CoordInfo{0, 0, kBorderLo, 0};
        else
            a->coord[i] = CoordInfo{static_cast<int32_t>(it.next()), static_cast<int32_t>((i % a->phases) * 2), kMain, 0};
    }
}

// ---------------------------------------------------------------- fast-path eligibility

int ceil_log2(uint64_t d)
{
    int l = 0;
    while ((uint64_t(1) << l) < d)
        ++l;
    return l;
}

} // namespace

// Granlund & Montgomery (PLDI'94) Thm 4.2: with 2^(N+l) <= m*d <= 2^(N+l) + 2^l,
// floor(n / d) == floor(m * n / 2^(N+l)) for all 0 <= n < 2^N.  m = ceil(2^(N+l) / d) with
// l = ceil(log2 d) satisfies it.
//
// Y border rows: n = |nume| * 64 < 2^22 (nume is int16), N = 22, d = deno in [1, 1024] (l <= 10):
// floor(m * n / 2^(22+l)) == umulhi(n << (10 - l), m) == umulhi(|nume| << (16 - l), m).
bool magic_y(int32_t deno, uint32_t *m, int32_t *s)
{
    if (deno < 1 || deno > 1024)
        return false;
    const int l = ceil_log2(static_cast<uint64_t>(deno));
    const uint64_t k = 22 + static_cast<uint64_t>(l);
    const uint64_t mm = ((uint64_t(1) << k) + static_cast<uint64_t>(deno) - 1) / static_cast<uint64_t>(deno);
    if (mm >= (uint64_t(1) << 32))
        return false;
    *m = static_cast<uint32_t>(mm);
    *s = 16 - l;
    return true;
}

// X edge values: n = X sum clamped at 0, n < 2^31, N = 31, d = 64 * deno (>= 2):
// floor(m * n / 2^(31+l)) == umulhi(n, m) >> (l - 1), m < 2^32 because d > 2^(l-1).
bool magic_x(int64_t d, uint32_t *m, int32_t *t)
{
    if (d < 2 || d > (int64_t(1) << 31))
        return false;
    const int l = ceil_log2(static_cast<uint64_t>(d));
    const uint64_t k = 31 + static_cast<uint64_t>(l);
    if (k >= 64)
        return false;
    const uint64_t mm = ((uint64_t(1) << k) + static_cast<uint64_t>(d) - 1) / static_cast<uint64_t>(d);
    if (mm >= (uint64_t(1) << 32))
        return false;
    *m = static_cast<uint32_t>(mm);
    *t = l - 1;
    return true;
}

namespace {

void pick_fast_lanczos(Plan *p)
{
    AxisPlan &x = p->x, &y = p->y;
    if (x.identity || y.identity || x.phases != 1 || y.phases != 1)
        return;
    if (p->srcW % p->dstW || p->srcH % p->dstH)
        return;
    int KX = p->srcW / p->dstW, KY = p->srcH / p->dstH;
    if (x.mainBegin > x.mainEnd || y.mainBegin > y.mainEnd)
        return;
    if (y.mainBegin > 16 || p->dstH - y.mainEnd > 16 || x.mainBegin > 16 || p->dstW - x.mainEnd > 16)
        return;
    FastLanczos &f = p->flz;
    f.KY = KY;
    f.KX = KX;
    // Y: drop zero taps at both ends (exact for main and masked formulas alike).
    int m = y.taps / 2, lo = 0, hi = y.taps;
    while (lo < hi && y.table[lo] == 0)
        ++lo;
    while (hi > lo && y.table[hi - 1] == 0)
        --hi;
    f.NY = hi - lo;
    f.offY = 1 - m + lo;  // first tap row = KY*y + 1 - m + lo  (srcOY = floor(y*KY) + 1)
    f.cy.assign(y.table.begin() + lo, y.table.begin() + hi);
    // the accumulator ring needs NY % KY == 0: pad with zero taps below (a zero tap adds nothing
    // to the interior sum nor to the masked border sum; the border divisors come from the
    // reference coordinates, not from these taps)
    if (KY > 0 && !y.table.empty())
        while (f.NY % KY) {
            f.cy.push_back(0);
            ++f.NY;
        }
    // X: drop zero taps, then pad to an even first column and an even tap count (int16 pairs).
    int mx = x.taps / 2, xl = 0, xh = x.taps;
    while (xl < xh && x.table[xl] == 0)
        ++xl;
    while (xh > xl && x.table[xh - 1] == 0)
        --xh;
    int off = 1 - mx + xl;  // first tap column = KX*x + off
    int pre = (((KX % 2) == 0) && (off & 1)) ? 1 : 0;
    if (KX % 2)
        return;  // odd KX alternates pair parity per output: not instantiated
    f.offX = off - pre;
    int n = (xh - xl) + pre;
    f.NXP = n + (n & 1);
    f.cx.assign(static_cast<size_t>(f.NXP), 0);
    for (int i = xl; i < xh; ++i)
        f.cx[static_cast<size_t>(i - xl + pre)] = static_cast<int16_t>(x.table[i]);
    f.mainBeginY = y.mainBegin;
    f.mainEndY = y.mainEnd;
    f.mainBeginX = x.mainBegin;
    f.mainEndX = x.mainEnd;
    f.denoYTop.clear();
    f.denoYBot.clear();
    for (int r = 0; r < y.mainBegin; ++r)
        f.denoYTop.push_back(y.coord[r].aux);
    for (int r = y.mainEnd; r < p->dstH; ++r)
        f.denoYBot.push_back(y.coord[r].aux);
    f.dXLeft.clear();
    f.dXRight.clear();
    for (int c = 0; c < x.mainBegin; ++c)
        f.dXLeft.push_back(64 * x.coord[c].aux);
    for (int c = x.mainEnd; c < p->dstW; ++c)
        f.dXRight.push_back(64 * x.coord[c].aux);
    // Streamer arithmetic preconditions (kernels.hip, lanczos_stream_kernel):
    //  * the int32 X sum never overflows and (sum >> 20) fits int16 for ANY int16 work values, so
    //    the packed saturating shift (v_ashr_pk_u8_i32) equals clamp255(int16(sum >> 20));
    //  * border divisions use the exact multiply-high forms of magic_y / magic_x;
    //  * output width multiple of 8 and <= 4 border columns per side: the last wave is aligned
    //    to the right edge, so border columns sit at static positions of the edge lanes.
    int64_t sabs = 0;
    for (int16_t c : f.cx)
        sabs += c < 0 ? -c : c;
    const int64_t maxSum = 32768 * sabs + (1 << 19);
    if (maxSum >= (int64_t(1) << 31) || (maxSum >> 20) >= 32768)
        return;
    // Lanczos-5 2:1 (12 + 4 zero Y taps, 20 X taps from 2x - 9): 5 border columns per side, held
    // by the block-shared streamer's line scheme with 8 edge outputs per side (xM8), >= 256 outputs
    const bool l5 = KX == 2 && KY == 2 && f.NY == 16 && (xh - xl) == 20 && off == -9 && p->dstW >= 256 &&
                    p->dstW <= 4 * 62 * 8 && x.mainBegin <= 8 && p->dstW - x.mainEnd <= 8;
    if (p->dstW % 8 || (!l5 && (x.mainBegin > 4 || p->dstW - x.mainEnd > 4)) || y.mainBegin > 16 ||
        p->dstH - y.mainEnd > 16)
        return;
    // negative denominators (a border row / column whose valid taps sum below zero) divide by
    // the magnitude and flip the sign: C truncation is symmetric
    f.yTopNeg = f.yBotNeg = f.xNeg = 0;
    for (size_t i = 0; i < f.denoYTop.size(); ++i) {
        const int32_t dn = f.denoYTop[i];
        if (!magic_y(dn < 0 ? -dn : dn, &f.yTopM[i], &f.yTopS[i]))
            return;
        f.yTopNeg |= dn < 0 ? 1 << i : 0;
    }
    for (size_t i = 0; i < f.denoYBot.size(); ++i) {
        const int32_t dn = f.denoYBot[i];
        if (!magic_y(dn < 0 ? -dn : dn, &f.yBotM[i], &f.yBotS[i]))
            return;
        f.yBotNeg |= dn < 0 ? 1 << i : 0;
    }
    bool neg8 = false;  // a negative denominator among the 8-output edge lanes (not instantiated)
    for (int k = 0; k < 16; ++k) {
        const int c = k < 8 ? k : p->dstW - 16 + k;  // column of edge-lane value k
        int64_t D = int64_t(1) << 20;
        if (k < 8 && c < x.mainBegin)
            D = f.dXLeft[static_cast<size_t>(c)];
        else if (k >= 8 && c >= x.mainEnd && c >= 0)
            D = f.dXRight[static_cast<size_t>(c - x.mainEnd)];
        neg8 |= D < 0;
        if (D < 0)
            D = -D;
        if ((D != (int64_t(1) << 20) && (maxSum / D >= 32768)) || !magic_x(D, &f.xM8[k], &f.xT8[k])) {
            if (l5)
                return;
            break;
        }
    }
    for (int k = 0; k < 8; ++k) {
        const int c = k < 4 ? k : p->dstW - 8 + k;  // column of edge-lane value k
        int64_t D = int64_t(1) << 20;               // identity: floor(s / 2^20) == s >> 20
        if (k < 4 && c < x.mainBegin)
            D = f.dXLeft[static_cast<size_t>(c)];
        else if (k >= 4 && c >= x.mainEnd && c >= 0)
            D = f.dXRight[static_cast<size_t>(c - x.mainEnd)];
        if (D < 0) {
            D = -D;
            f.xNeg |= 1 << k;
        }
        if (D != (int64_t(1) << 20) && (maxSum / D >= 32768))
            return;  // border quotient must fit int16 (it is int16-cast before the clamp)
        if (!magic_x(D, &f.xM[k], &f.xT[k]))
            return;
    }
    // instantiated shapes (kernels.hip): (KY,KX,NY,NXP,offX/2) = (2,2,10,14,-3) Lanczos-3 2:1,
    // (2,2,8,10,-2) Lanczos-2 2:1, (2,2,4,4,0) the pxScale-2 chroma tables of Lanczos-2/3 2:1
    // (3 non-zero taps, IQOLanczosResizerImpl_Generic.cpp:144-190 with degFactor).  Everything
    // else runs the general kernel.
    bool inst = KY == 2 && KX == 2 && ((f.NY == 10 && f.NXP == 14 && f.offX == -6) ||
                                       (f.NY == 8 && f.NXP == 10 && f.offX == -4) ||
                                       (f.NY == 4 && f.NXP == 4 && f.offX == 0));
    // Lanczos-4 2:1 (12 non-zero Y taps, 16 X taps from 2x - 7): the block-shared symmetric
    // streamer only (no ring-streamer instantiation), so only where that one runs: <= 4 waves of
    // 62 producing lanes per row, symmetric Y taps, no negative denominators
    const bool l4 = KY == 2 && KX == 2 && f.NY == 12 && (xh - xl) == 16 && off == -7 && p->dstW <= 4 * 62 * 8;
    if (l5 && neg8)
        return;
    // symmetric variant: (NY, NX, offXO) = (10, 12, -5) Lanczos-3 2:1, (8, 8, -3) Lanczos-2 2:1
    f.NX = xh - xl;
    f.offXO = off;
    f.cxo.assign(x.table.begin() + xl, x.table.begin() + xh);
    bool symY = (f.NY % 2) == 0;
    for (int i = 0; symY && i < f.NY / 2; ++i)
        symY = f.cy[static_cast<size_t>(i)] == f.cy[static_cast<size_t>(f.NY - 1 - i)];
    f.sym = (inst || l4 || l5) && symY && (off & 1) && !f.yTopNeg && !f.yBotNeg && (!f.xNeg || l5) &&
            ((f.NY == 10 && f.NX == 12 && off == -5) || (f.NY == 8 && f.NX == 8 && off == -3) ||
             (f.NY == 12 && f.NX == 16 && off == -7) || (f.NY == 16 && f.NX == 20 && off == -9));
    if ((l4 || l5) && f.sym)
        inst = true;
    if (!inst || (p->srcW % 16) || p->srcW > 8192)
        return;
    p->kernel = 1;  // IQO_KERNEL_LANCZOS_STREAM
}

void pick_fast_area(Plan *p)
{
    AxisPlan &x = p->x, &y = p->y;
    if (x.identity || y.identity || x.phases != 1 || y.phases != 1)
        return;
    if (p->srcW % p->dstW || p->srcH % p->dstH)
        return;
    int KX = p->srcW / p->dstW, KY = p->srcH / p->dstH;
    if (!(KX == 2 || KX == 3 || KX == 4 || KX == 6 || KX == 8) || KY < 2 || KY > 16 || x.taps != KX || y.taps != KY)
        return;
    // kernels.hip area_int_kernel: a thread takes 16 source columns (12 when KX is 3 or 6)
    if (p->srcW % ((16 % KX == 0) ? 32 : 12))
        return;
    p->far.KX = KX;
    p->far.KY = KY;
    p->far.cx.assign(x.table.begin(), x.table.end());
    p->far.cy.assign(y.table.begin(), y.table.end());
    p->kernel = 2;  // IQO_KERNEL_AREA_INT
}

// Linear at exactly 2x or 3x (kernels.hip linear_up2_kernel_body): main output F k + i (i = 1 .. F)
// blends source samples k and k + 1 with phase (i % F)'s two taps (IQOLinearResizerImpl_Generic.cpp
// :252-271 / :384-406, srcO = floor((y + 0.5) / F - 0.5)); the first and last output replicate the
// edge sample (:240-248, :273-281, :343-345).
void pick_fast_linear(Plan *p)
{
    AxisPlan &x = p->x, &y = p->y;
    const int F = p->dstW == 3 * p->srcW ? 3 : 2;
    if (x.identity || y.identity || p->dstW != F * p->srcW || p->dstH != F * p->srcH)
        return;
    if (x.phases != F || y.phases != F || p->dstW % (8 * F))
        return;
    for (const AxisPlan *a : {&x, &y}) {
        if (a->mainBegin != 1 || a->mainEnd != a->dstLen - 1)
            return;
        for (int i = a->mainBegin; i < a->mainEnd; ++i)
            if (a->coord[i].srcO != (i - 1) / F || a->coord[i].tabOff != (i % F) * 2)
                return;
    }
    p->fln.F = F;
    for (int q = 0; q < F; ++q)
        for (int k = 0; k < 2; ++k) {
            p->fln.cx[q][k] = static_cast<uint16_t>(x.table[2 * q + k]);
            p->fln.cy[q][k] = static_cast<uint16_t>(y.table[2 * q + k]);
        }
    p->kernel = 3;  // IQO_KERNEL_LINEAR_UP2
}

// Linear at exactly 2:1 (e.g. 3840x2160 -> 1920x1080): main output i blends source samples 2i + 1
// and 2i + 2 with the table's two taps (IQOLinearResizerImpl_Generic.cpp:210-282, 366-407) and the
// first / last output replicates the edge sample (:227-237, :329-364), on both axes -- the Area
// arithmetic (u16 work row, (s + 2^22) >> 23) on odd-aligned pairs: kernels.hip linear_d2_body,
// dispatched as IQO_KERNEL_AREA_INT (area_kind 8).
void pick_fast_linear_down(Plan *p)
{
    AxisPlan &x = p->x, &y = p->y;
    if (x.identity || y.identity || x.phases != 1 || y.phases != 1 || x.taps != 2 || y.taps != 2)
        return;
    if (p->srcW != 2 * p->dstW || p->srcH != 2 * p->dstH || p->srcW % 16 || p->dstW < 16 || p->dstH < 2)
        return;
    for (const AxisPlan *a : {&x, &y}) {
        const int n = a->dstLen;
        if (a->coord[0].kind != kBorderLo || a->coord[static_cast<size_t>(n - 1)].kind != kBorderHi)
            return;
        for (int i = 1; i < n - 1; ++i) {
            const CoordInfo &c = a->coord[static_cast<size_t>(i)];
            if (c.kind != kMain || c.srcO != 2 * i + 1 || c.tabOff != 0)
                return;
        }
    }
    p->far.KX = 2;
    p->far.KY = 2;
    p->far.lin = true;
    p->far.cx.assign(x.table.begin(), x.table.end());
    p->far.cy.assign(y.table.begin(), y.table.end());
    p->kernel = 2;  // IQO_KERNEL_AREA_INT
}

} // namespace

bool build_tables(Method m, unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                  size_t pxScale, AxisPlan *x, AxisPlan *y, std::string *err)
{
    if (!srcW || !srcH || !dstW || !dstH) {
        if (err)
            *err = "zero-sized image";
        return false;
    }
    if (srcW > (1u << 30) || srcH > (1u << 30) || dstW > (1u << 30) || dstH > (1u << 30)) {
        if (err)
            *err = "image dimension too large";
        return false;
    }
    x->srcLen = static_cast<int>(srcW);
    x->dstLen = static_cast<int>(dstW);
    y->srcLen = static_cast<int>(srcH);
    y->dstLen = static_cast<int>(dstH);
    switch (m) {
    case kLanczos:
        if (degree < 1 || pxScale < 1) {
            if (err)
                *err = "lanczos degree and pxScale must be >= 1";
            return false;
        }
        tables_lanczos(degree, srcW, dstW, pxScale, 1 << 14, x);  // kBias14 (:265-266)
        tables_lanczos(degree, srcH, dstH, pxScale, 1 << 6, y);   // kBias   (:262-263)
        return true;
    case kArea:
        tables_area(srcW, dstW, 1 << 15, x);  // kBias15 (IQOAreaResizerImpl_Generic.cpp:148-149)
        tables_area(srcH, dstH, 1 << 8, y);   // kBias   (:145-146)
        return true;
    case kLinear:
        tables_linear(srcW, dstW, 1 << 15, x);  // IQOLinearResizerImpl_Generic.cpp:135-136
        tables_linear(srcH, dstH, 1 << 8, y);
        return true;
    }
    if (err)
        *err = "unknown method";
    return false;
}

bool build_plan(Method m, unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                size_t pxScale, Plan *p, std::string *err)
{
    *p = Plan();
    if (!build_tables(m, degree, srcW, srcH, dstW, dstH, pxScale, &p->x, &p->y, err))
        return false;
    p->method = m;
    p->degree = degree;
    p->pxScale = pxScale;
    p->srcW = static_cast<int>(srcW);
    p->srcH = static_cast<int>(srcH);
    p->dstW = static_cast<int>(dstW);
    p->dstH = static_cast<int>(dstH);
    switch (m) {
    case kLanczos:
        coords_lanczos_x(&p->x);
        coords_lanczos_y(&p->y);
        pick_fast_lanczos(p);
        break;
    case kArea:
        coords_area(&p->x);
        coords_area(&p->y);
        pick_fast_area(p);
        break;
    case kLinear:
        coords_linear(&p->x);
        coords_linear(&p->y);
        pick_fast_linear(p);
        if (p->kernel == 0)
            pick_fast_linear_down(p);
        break;
    }
    return true;
}

namespace {

// One axis coordinate as a contiguous tap window: source index of tap 0, coefficients (16-bit
// patterns) and the Lanczos border divisor (0 for every other formula).  Follows y_value /
// x_value_rec of kernels.hip (and through them the reference lines cited there).
struct Window {
    int start = 0;
    std::vector<int32_t> c;
    int32_t div = 0;
    bool border = false;
};

Window axis_window(const Plan &p, const AxisPlan &ax, int i, bool isX)
{
    const CoordInfo &ci = ax.coord[static_cast<size_t>(i)];
    const int len = ax.srcLen;
    Window w;
    w.start = ci.srcO;
    if (ci.kind == kIdentity) {
        w.c.assign(1, p.method == kLanczos ? (isX ? 1 << 14 : 64) : (isX ? 1 << 15 : 256));
        return w;
    }
    if (p.method == kLinear && ci.kind != kMain) {  // replicate the first / last source pixel
        w.start = ci.kind == kBorderLo ? 0 : len - 1;
        w.c.assign(1, isX ? 1 << 15 : 256);
        return w;
    }
    w.c.assign(ax.table.begin() + ci.tabOff, ax.table.begin() + ci.tabOff + ax.taps);
    if (p.method == kLanczos && ci.kind != kMain) {
        for (int k = 0; k < ax.taps; ++k)
            if (w.start + k < 0 || w.start + k >= len)
                w.c[static_cast<size_t>(k)] = 0;
        w.border = true;
        w.div = isX ? ci.aux * 64 : ci.aux;
    }
    return w;
}

} // namespace

void build_tile_tables(const Plan &p, TileTables *t)
{
    *t = TileTables();
    if (p.srcW < 8)
        return;
    // rows
    int nY = 1;
    std::vector<Window> wy(static_cast<size_t>(p.dstH));
    for (int y = 0; y < p.dstH; ++y) {
        wy[static_cast<size_t>(y)] = axis_window(p, p.y, y, false);
        nY = std::max(nY, static_cast<int>(wy[static_cast<size_t>(y)].c.size()));
    }
    t->nYp = (nY + 1) & ~1;
    t->rows.resize(static_cast<size_t>(p.dstH));
    t->rowCoef.assign(static_cast<size_t>(p.dstH) * t->nYp, 0u);
    for (int y = 0; y < p.dstH; ++y) {
        const Window &w = wy[static_cast<size_t>(y)];
        const int n = static_cast<int>(w.c.size());
        const int lo = std::max(0, std::min(w.start, p.srcH - 1));
        const int hi = std::max(lo, std::min(w.start + n - 1, p.srcH - 1));
        // a masked border divisor of 0 traps in the reference; exact_div(n, INT_MAX) = 0 here, as
        // in general_kernel
        const int32_t deno = w.border ? (w.div ? w.div : 0x7fffffff) : 0;
        t->rows[static_cast<size_t>(y)] = TileRec{w.start, lo, hi, deno};
        for (int k = 0; k < n; ++k) {
            const uint32_t c = static_cast<uint32_t>(w.c[static_cast<size_t>(k)]) & 0xffffu;
            t->rowCoef[static_cast<size_t>(y) * t->nYp + k] = c | (c << 16);
        }
    }
    // columns
    std::vector<Window> wx(static_cast<size_t>(p.dstW));
    int np = 1;
    for (int x = 0; x < p.dstW; ++x) {
        Window &w = wx[static_cast<size_t>(x)];
        w = axis_window(p, p.x, x, true);
        const int shift = w.start & 1;
        np = std::max(np, (static_cast<int>(w.c.size()) + shift + 1) / 2);
    }
    int NP = 0;
    for (int v : kTileNP)
        if (v >= np) {
            NP = v;
            break;
        }
    if (!NP)
        return;  // wider than the largest instantiation: general_kernel
    t->NP = NP;
    t->cols.resize(static_cast<size_t>(p.dstW));
    t->colCoef.assign(static_cast<size_t>(p.dstW) * NP, 0u);
    for (int x = 0; x < p.dstW; ++x) {
        const Window &w = wx[static_cast<size_t>(x)];
        const int a = w.start & ~1, shift = w.start - a;
        const int32_t D = w.border ? (w.div ? w.div : 0x7fffffff) : 0;
        t->cols[static_cast<size_t>(x)] = TileCol{a, D};
        for (int k = 0; k < static_cast<int>(w.c.size()); ++k) {
            const int slot = k + shift;
            const uint32_t c = static_cast<uint32_t>(w.c[static_cast<size_t>(k)]) & 0xffffu;
            t->colCoef[static_cast<size_t>(x) * NP + slot / 2] |= (slot & 1) ? c << 16 : c;
        }
    }
    // column tiles: wider tiles for upscales, so the vertical pass has enough columns per tile
    const double ratio = static_cast<double>(p.srcW) / p.dstW;
    int CT = ratio >= 1.0 ? 256 : (ratio >= 0.5 ? 512 : 1024);
    while (CT > 256 && CT / 2 >= p.dstW)
        CT /= 2;
    t->CT = CT;
    const int nT = (p.dstW + CT - 1) / CT;
    t->spans.resize(static_cast<size_t>(nT));
    int maxG = 1;
    for (int k = 0; k < nT; ++k) {
        int lo = 1 << 30, hi = -(1 << 30);
        for (int x = k * CT; x < std::min(p.dstW, (k + 1) * CT); ++x) {
            lo = std::min(lo, t->cols[static_cast<size_t>(x)].a);
            hi = std::max(hi, t->cols[static_cast<size_t>(x)].a + 2 * NP);
        }
        const int lo8 = lo & ~7;
        const int g = (hi - lo8 + 7) / 8;
        t->spans[static_cast<size_t>(k)] = TileSpan{lo8, g};
        maxG = std::max(maxG, g);
    }
    t->pitchDw = 4 * maxG;
    t->spitch = 8 * maxG;
    // row windows must be monotone (the kernel stages rows [lo(first), hi(last)] of a tile)
    for (int y = 1; y < p.dstH; ++y)
        if (t->rows[static_cast<size_t>(y)].lo < t->rows[static_cast<size_t>(y - 1)].lo ||
            t->rows[static_cast<size_t>(y)].hi < t->rows[static_cast<size_t>(y - 1)].hi)
            return;
    int l2 = 0;
    while ((4 << l2) < CT)
        ++l2;
    t->log2nQ = l2;
    // rows per tile: 16, fewer when the staged source, the work tile and the tap records outgrow
    // 48 KiB (MI355X, G1 1080p -> 720p x128: 16 rows 0.294 ms, 32 rows 0.315 ms; G3 0.154 vs
    // 0.183 ms)
    int TH = 16;
    while (TH > 2 && tile_lds_bytes(p, *t, TH) > 48 * 1024)
        TH /= 2;
    t->ok = tile_set_rows(p, t, TH);
}

size_t tile_lds_bytes(const Plan &p, const TileTables &t, int TH)
{
    return static_cast<size_t>(TH) * (t.pitchDw * 4 + 16 + t.nYp * 8) + 4u * t.CT +
           static_cast<size_t>(tile_src_rows(p, t, TH)) * t.spitch;
}

int tile_src_rows(const Plan &p, const TileTables &t, int TH)
{
    int m = 1;
    for (int y = 0; y < p.dstH; ++y) {
        const int ye = std::min(p.dstH, y + TH) - 1;
        m = std::max(m, t.rows[static_cast<size_t>(ye)].hi - t.rows[static_cast<size_t>(y)].lo + 1);
    }
    return m;
}

bool tile_set_rows(const Plan &p, TileTables *t, int TH)
{
    if (TH < 1 || TH > 64 || tile_lds_bytes(p, *t, TH) > 64 * 1024)
        return false;
    t->TH = TH;
    t->srcRows = tile_src_rows(p, *t, TH);
    return true;
}

void band_src_rows(const Plan &p, int r0, int r1, int *s0, int *s1)
{
    int lo = p.srcH, hi = 0;
    for (int yy = r0; yy < r1; ++yy) {
        const CoordInfo &c = p.y.coord[static_cast<size_t>(yy)];
        int a, b;  // [a, b) rows touched
        if (c.kind == kIdentity) {
            a = c.srcO;
            b = c.srcO + 1;
        } else if (p.method == kLinear && c.kind != kMain) {
            a = c.kind == kBorderLo ? 0 : p.srcH - 1;
            b = a + 1;
        } else {
            a = c.srcO;
            b = c.srcO + p.y.taps;
        }
        a = std::max(0, std::min(a, p.srcH - 1));
        b = std::max(a + 1, std::min(b, p.srcH));
        lo = std::min(lo, a);
        hi = std::max(hi, b);
    }
    if (lo >= hi) {
        lo = 0;
        hi = 0;
    }
    *s0 = lo;
    *s1 = hi;
}

// The wave walker's tables: the tile tables' rows and column coefficients, 256-column strips, the
// ring geometry and per-row tap records that carry ring byte offsets (the ring slot of source row
// r is r % R for every band, so the offsets are constants of the plan).
void build_walk_tables(const Plan &p, const TileTables &t, WalkTables *w)
{
    *w = WalkTables();
    // the vertical taps are unrolled as 2 * NP or 2 * NP - 2 (the same ratio on both axes: the
    // horizontal pairs also absorb an odd window start), NP <= 8
    if (!t.ok || p.srcW < 4 || t.NP > 8 || t.nYp < 2 || (t.nYp != 2 * t.NP && t.nYp != 2 * t.NP - 2))
        return;
    const int nS = (p.dstW + kWalkStrip - 1) / kWalkStrip;
    int maxU = 1;
    w->spans.resize(static_cast<size_t>(nS));
    for (int k = 0; k < nS; ++k) {
        const int x0 = k * kWalkStrip, x1 = std::min(p.dstW, x0 + kWalkStrip);
        int lo = 1 << 30, hi = -(1 << 30);
        for (int x = x0; x < x1; ++x) {
            lo = std::min(lo, t.cols[static_cast<size_t>(x)].a);
            hi = std::max(hi, t.cols[static_cast<size_t>(x)].a + 2 * t.NP);
        }
        const int lo8 = lo & ~7;
        const int units = (hi - lo8 + 3) / 4;
        bool interior = x1 - x0 == kWalkStrip;
        for (int x = x0; x < x1; ++x)
            interior = interior && t.cols[static_cast<size_t>(x)].D == 0;
        w->spans[static_cast<size_t>(k)] = WalkSpan{lo8, units, interior ? 1 : 0};
        maxU = std::max(maxU, units);
    }
    const int NV = maxU <= 64 ? 1 : (maxU <= 128 ? 2 : 0);
    if (!NV)
        return;  // a strip reads more than 512 source columns (downscales beyond ~1.9x)
    int win = 1, maxNew = 0;
    for (int y = 0; y < p.dstH; ++y) {
        const TileRec &r = t.rows[static_cast<size_t>(y)];
        win = std::max(win, r.hi - r.lo + 1);
        if (y > 0)
            maxNew = std::max(maxNew, r.hi - t.rows[static_cast<size_t>(y - 1)].hi);
    }
    if (maxNew > NV)
        return;  // the load pipeline carries NV rows per output row
    // rows first(y) .. first(y)+NV-1 are widened at row y, up to NV-1 of them early: R = the widest
    // window + NV keeps every slot they overwrite dead
    const int R = win + NV;
    w->NV = NV;
    w->nS = nS;
    w->maxUnits = maxU;
    w->R = R;
    w->pitch = NV == 1 ? 512 : 8 * maxU;
    w->maxNew = maxNew;
    w->waveBytes = static_cast<size_t>(R) * w->pitch + 512u * NV + (NV == 2 ? 512u : 0u);
    if (4 * w->waveBytes > 64 * 1024)
        return;
    const int H = p.dstH;
    w->rows.resize(static_cast<size_t>(H));
    std::vector<int> first(static_cast<size_t>(H));
    for (int y = 0; y < H; ++y)
        first[static_cast<size_t>(y)] = y ? t.rows[static_cast<size_t>(y - 1)].hi + 1 : t.rows[0].lo;
    w->segs.resize(static_cast<size_t>(H) + kWalkPrefetch + 1);
    for (int y = 0; y < H + kWalkPrefetch + 1; ++y) {
        const int yy = std::min(y, H - 1);
        const TileRec &r = t.rows[static_cast<size_t>(yy)];
        const int f = first[static_cast<size_t>(yy)];
        const int fD = first[static_cast<size_t>(std::min(y + kWalkPrefetch, H - 1))];
        WalkSeg g{f, (f % R) * w->pitch, r.deno != 0, fD, 0u, 0, 0, 0};
        if (r.deno != 0 && r.deno != 0x7fffffff) {  // 0x7fffffff: masked divisor 0, quotient 0
            const int32_t ad = r.deno < 0 ? -r.deno : r.deno;
            if (!magic_y(ad, &g.yM, &g.yS))
                return;  // outside the proven range of the multiply-high division: tile_kernel
            g.yNeg = r.deno < 0;
        }
        w->segs[static_cast<size_t>(y)] = g;
    }
    if (static_cast<size_t>(R) * w->pitch > 65535)
        return;  // ring offsets are 16-bit
    w->rowTap.resize(static_cast<size_t>(H + 1) * t.nYp * 2);
    for (int y = 0; y < H + 1; ++y) {
        const int yy = std::min(y, H - 1);
        const TileRec &r = t.rows[static_cast<size_t>(yy)];
        if (y < H)
            w->rows[static_cast<size_t>(y)] = WalkRow{r.lo, r.hi, r.hi % R, r.deno};
        for (int i = 0; i < t.nYp; ++i) {
            const int row = std::min(std::max(r.start + i, r.lo), r.hi);
            const size_t k = (static_cast<size_t>(y) * t.nYp + i) * 2;
            w->rowTap[k] = t.rowCoef[static_cast<size_t>(yy) * t.nYp + i];
            w->rowTap[k + 1] = static_cast<uint32_t>((row % R) * w->pitch);
        }
    }
    w->ok = true;
}


void build_up2(const Plan &p, const WalkTables &w, Up2Tables *u)
{
    *u = Up2Tables();
    (void)w;
    const int F = p.dstW == 2 * p.srcW ? 2 : 3;  // lane: 8 source columns, 8F output columns
    if (p.method != kLanczos || p.x.identity || p.y.identity || p.dstW != F * p.srcW ||
        p.dstH != F * p.srcH || p.dstW % (8 * F) || p.dstW < 16 * F || p.dstH < 4 * F)
        return;
    const int NT = static_cast<int>(p.x.taps);
    if ((NT != 4 && NT != 6) || static_cast<int>(p.y.taps) != NT)
        return;
    // every window (main or masked border) starts where the kernel's fixed offset says and takes
    // its phase's table, so the kernel's unmasked sums over zero-padded rows / columns are the
    // reference's masked numerators
    auto fixed = [&](const AxisPlan &ax, int i, std::vector<int32_t> (&set)[3]) {
        const CoordInfo &ci = ax.coord[static_cast<size_t>(i)];
        if (ci.kind == kIdentity || ci.srcO != i / F + 1 - NT / 2 || ci.tabOff % NT != 0)
            return false;
        const std::vector<int32_t> c(ax.table.begin() + ci.tabOff, ax.table.begin() + ci.tabOff + NT);
        std::vector<int32_t> &ref = set[i % F];
        if (ref.empty())
            ref = c;
        return ref == c;
    };
    std::vector<int32_t> ys[3], xs[3];
    const int EC = 8 * F;  // edge-lane columns
    for (int x = 0; x < p.dstW; ++x) {
        if (!fixed(p.x, x, xs))
            return;
        const Window win = axis_window(p, p.x, x, true);
        const int side = x < EC ? 0 : x >= p.dstW - EC ? 1 : -1;
        if (win.border && side < 0)
            return;
        if (side >= 0) {
            const int j = side ? x - (p.dstW - EC) : x;
            if (!magic_x(win.border ? win.div : (1 << 20), &u->xM[side][j], &u->xT[side][j]))
                return;
        }
    }
    int m0 = -1, m1 = -1;
    for (int y = 0; y < p.dstH; ++y) {
        if (!fixed(p.y, y, ys))
            return;
        const Window win = axis_window(p, p.y, y, false);
        if (!win.border) {
            if (m0 < 0)
                m0 = y;
            else if (m1 >= 0)
                return;  // main rows must be one contiguous run
        } else if (m0 >= 0 && m1 < 0) {
            m1 = y;
        }
    }
    if (m0 < 0)
        return;
    if (m1 < 0)
        m1 = p.dstH;
    for (int j = 0; j < F; ++j)
        if (ys[j].empty() || xs[j].empty())
            return;
    if (m0 > 16 || p.dstH - m1 > 16)
        return;
    for (int y = 0; y < p.dstH; ++y) {
        if (y >= m0 && y < m1)
            continue;
        const Window win = axis_window(p, p.y, y, false);
        const int side = y < m0 ? 0 : 1, i = side ? y - m1 : y;
        if (!magic_y(win.div, &u->yM[side][i], &u->yS[side][i]))
            return;
    }
    auto single = [&](const std::vector<int32_t> &c) {
        for (int i = 0; i < NT; ++i)
            if ((i == NT / 2 - 1) != (c[static_cast<size_t>(i)] != 0))
                return false;
        return true;
    };
    if (!single(ys[0]) || !single(xs[0]))
        return;
    u->F = F;
    u->NT = NT;
    u->m0 = m0;
    u->m1 = m1;
    auto splat = [](int32_t c) { return (static_cast<uint32_t>(c) & 0xffffu) * 0x10001u; };
    u->cy0 = splat(ys[0][static_cast<size_t>(NT / 2 - 1)]);
    u->cx0 = static_cast<uint32_t>(xs[0][static_cast<size_t>(NT / 2 - 1)]) & 0xffffu;
    for (int j = 1; j < F; ++j) {
        for (int i = 0; i < NT; ++i)
            u->cy1[j - 1][i] = splat(ys[j][static_cast<size_t>(i)]);
        for (int q = 0; q < NT / 2; ++q)
            u->cx1[j - 1][q] = (static_cast<uint32_t>(xs[j][static_cast<size_t>(2 * q)]) & 0xffffu) |
                               (static_cast<uint32_t>(xs[j][static_cast<size_t>(2 * q + 1)]) << 16);
    }
    u->ok = true;
}

void build_u23(const Plan &p, U23Tables *u)
{
    *u = U23Tables();
    if (p.method != kLanczos || p.x.identity || p.y.identity || 3 * p.srcW != 2 * p.dstW || 3 * p.srcH != 2 * p.dstH ||
        p.dstW % 12 || p.dstW < 24 || p.dstH < 12 || p.x.taps != 6 || p.y.taps != 6)
        return;
    // every window: start 2 (i / 3) - 2 + (i % 3 == 2), phase i % 3, phase 0 a single centre tap
    auto fixed = [&](const AxisPlan &ax, int i, std::vector<int32_t> (&set)[3]) {
        const CoordInfo &ci = ax.coord[static_cast<size_t>(i)];
        if (ci.kind == kIdentity || ci.srcO != 2 * (i / 3) - 2 + (i % 3 == 2 ? 1 : 0) || ci.tabOff % 6 != 0)
            return false;
        const std::vector<int32_t> c(ax.table.begin() + ci.tabOff, ax.table.begin() + ci.tabOff + 6);
        std::vector<int32_t> &ref = set[i % 3];
        if (ref.empty())
            ref = c;
        return ref == c;
    };
    std::vector<int32_t> xs[3], ys[3];
    for (int x = 0; x < p.dstW; ++x) {
        if (!fixed(p.x, x, xs))
            return;
        const Window win = axis_window(p, p.x, x, true);
        const int side = x < 12 ? 0 : x >= p.dstW - 12 ? 1 : -1;
        if (win.border && side < 0)
            return;
        if (side >= 0) {
            const int j = side ? x - (p.dstW - 12) : x;
            if (!magic_x(win.border ? win.div : (1 << 20), &u->xM[side][j], &u->xT[side][j]))
                return;
        }
    }
    int m0 = -1, m1 = -1;
    for (int y = 0; y < p.dstH; ++y) {
        if (!fixed(p.y, y, ys))
            return;
        const Window win = axis_window(p, p.y, y, false);
        if (!win.border) {
            if (m0 < 0)
                m0 = y;
            else if (m1 >= 0)
                return;
        } else if (m0 >= 0 && m1 < 0) {
            m1 = y;
        }
    }
    if (m0 < 0)
        return;
    if (m1 < 0)
        m1 = p.dstH;
    if (m0 > 8 || p.dstH - m1 > 8)
        return;
    for (int y = 0; y < p.dstH; ++y) {
        if (y >= m0 && y < m1)
            continue;
        const Window win = axis_window(p, p.y, y, false);
        const int side = y < m0 ? 0 : 1, i = side ? y - m1 : y;
        if (!magic_y(win.div, &u->yM[side][i], &u->yS[side][i]))
            return;
    }
    for (int k = 0; k < 6; ++k)
        if ((k == 2) != (ys[0][static_cast<size_t>(k)] != 0) || (k == 2) != (xs[0][static_cast<size_t>(k)] != 0))
            return;
    auto splat = [](int32_t c) { return (static_cast<uint32_t>(c) & 0xffffu) * 0x10001u; };
    u->cy0 = splat(ys[0][2]);
    u->cx0 = static_cast<uint32_t>(xs[0][2]) & 0xffffu;
    for (int ph = 0; ph < 2; ++ph) {
        for (int k = 0; k < 6; ++k)
            u->cy[ph][k] = splat(ys[ph + 1][static_cast<size_t>(k)]);
        for (int q = 0; q < 3; ++q)
            u->cx[ph][q] = (static_cast<uint32_t>(xs[ph + 1][static_cast<size_t>(2 * q)]) & 0xffffu) |
                           (static_cast<uint32_t>(xs[ph + 1][static_cast<size_t>(2 * q + 1)]) << 16);
    }
    u->m0 = m0;
    u->m1 = m1;
    u->ok = true;
}

void build_l23(const Plan &p, L23Tables *t)
{
    *t = L23Tables();
    if (p.method != kLinear || p.x.identity || p.y.identity || 3 * p.srcW != 2 * p.dstW || 3 * p.srcH != 2 * p.dstH ||
        p.dstW % 12 || p.dstW < 24 || p.dstH < 3 || p.x.taps != 2 || p.y.taps != 2 || p.x.phases != 3 || p.y.phases != 3)
        return;
    auto axis = [&](const AxisPlan &ax, std::vector<int32_t> (&set)[3]) {
        for (int i = 0; i < ax.dstLen; ++i) {
            const CoordInfo &ci = ax.coord[static_cast<size_t>(i)];
            const int j = i % 3, start = 2 * (i / 3) + j - 1;
            if (ci.kind == kIdentity)
                return false;
            if (ci.kind == kBorderLo) {  // replicate pixel 0: both clamped taps must land on it
                if (start + 1 > 0)
                    return false;
                continue;
            }
            if (ci.kind == kBorderHi) {  // replicate the last pixel
                if (start < ax.srcLen - 1)
                    return false;
                continue;
            }
            if (ci.srcO != start || ci.tabOff != 2 * j || start < 0 || start + 1 >= ax.srcLen)
                return false;
            const std::vector<int32_t> c(ax.table.begin() + ci.tabOff, ax.table.begin() + ci.tabOff + 2);
            std::vector<int32_t> &ref = set[j];
            if (ref.empty())
                ref = c;
            if (ref != c)
                return false;
        }
        return !set[0].empty() && !set[1].empty() && !set[2].empty();
    };
    std::vector<int32_t> xs[3], ys[3];
    if (!axis(p.x, xs) || !axis(p.y, ys))
        return;
    for (int j = 0; j < 3; ++j) {
        // the clamped border taps must weigh the edge pixel as the reference's replicate does
        if (xs[j][0] + xs[j][1] != (1 << 15) || ys[j][0] + ys[j][1] != 256)
            return;
        for (int k = 0; k < 2; ++k)
            t->cy[j][k] = (static_cast<uint32_t>(ys[j][static_cast<size_t>(k)]) & 0xffffu) * 0x10001u;
        t->cx[j] = (static_cast<uint32_t>(xs[j][0]) & 0xffffu) | (static_cast<uint32_t>(xs[j][1]) << 16);
    }
    t->ok = true;
}

void build_a32(const Plan &p, A32Tables *t)
{
    *t = A32Tables();
    if (p.method != kArea || p.x.identity || p.y.identity || 2 * p.srcW != 3 * p.dstW || 2 * p.srcH != 3 * p.dstH ||
        p.dstW % 8 || p.dstW < 8 || p.dstH < 2 || p.x.taps < 2 || p.y.taps < 2)
        return;
    // every coordinate: the fixed start, its parity's phase, no non-zero tap past the second
    auto axis = [&](const AxisPlan &ax, std::vector<int32_t> (&set)[2]) {
        for (int i = 0; i < ax.dstLen; ++i) {
            const CoordInfo &ci = ax.coord[static_cast<size_t>(i)];
            if (ci.kind != kMain || ci.srcO != 3 * (i >> 1) + (i & 1) || ci.tabOff % ax.taps != 0)
                return false;
            const std::vector<int32_t> c(ax.table.begin() + ci.tabOff, ax.table.begin() + ci.tabOff + ax.taps);
            for (size_t k = 2; k < c.size(); ++k)
                if (c[k] != 0)
                    return false;
            std::vector<int32_t> &ref = set[i & 1];
            if (ref.empty())
                ref = c;
            if (ref != c)
                return false;
        }
        return !set[0].empty() && !set[1].empty();
    };
    std::vector<int32_t> xs[2], ys[2];
    if (!axis(p.x, xs) || !axis(p.y, ys))
        return;
    for (int ph = 0; ph < 2; ++ph) {
        for (int k = 0; k < 2; ++k)
            t->cy[ph][k] = (static_cast<uint32_t>(ys[ph][static_cast<size_t>(k)]) & 0xffffu) * 0x10001u;
        t->cx[ph] = (static_cast<uint32_t>(xs[ph][0]) & 0xffffu) | (static_cast<uint32_t>(xs[ph][1]) << 16);
    }
    t->ok = true;
}

void build_d32(const Plan &p, const WalkTables &w, D32Tables *d)
{
    *d = D32Tables();
    (void)w;
    if (p.method != kLanczos || p.x.identity || p.y.identity || 2 * p.srcW != 3 * p.dstW ||
        2 * p.srcH != 3 * p.dstH || p.dstW % 8 || p.dstW < 16 || p.dstH < 8)
        return;
    // the instantiated tap structures (kernels.hip lanczos_d32_kernel): taps T, group window start
    // GA (= the even rows' window start relative to 3m) and length GW, taps per row NTY, the odd
    // rows' first group row PO1, coefficient pairs per column NPX, column window start BX0
    struct Shape {
        int T, GA, GW, NTY, PO1, NPX, BX0;
    };
    static const Shape kShapes[2] = {{10, -4, 10, 8, 2, 5, -4}, {6, -2, 7, 5, 2, 3, -2}};
    const int T = static_cast<int>(p.x.taps);
    if (static_cast<int>(p.y.taps) != T)
        return;
    int vi = -1;
    for (int k = 0; k < 2; ++k)
        if (kShapes[k].T == T)
            vi = k;
    if (vi < 0)
        return;
    const Shape &S = kShapes[vi];
    auto start_ok = [](const Window &win, int i, int b0) { return win.start == 3 * (i >> 1) + b0 + (i & 1); };
    auto phase_row = [](const AxisPlan &ax, int ph) {
        return std::vector<int32_t>(ax.table.begin() + ph * ax.taps, ax.table.begin() + (ph + 1) * ax.taps);
    };
    // columns: every window (main or masked border) starts where the kernel's fixed offsets say and
    // takes its parity's phase, so the kernel's unmasked sum over zero-padded work columns is the
    // reference's masked numerator; border columns only among the 8 outermost on each side
    std::vector<int32_t> xs[2];
    for (int x = 0; x < p.dstW; ++x) {
        const CoordInfo &ci = p.x.coord[static_cast<size_t>(x)];
        const Window win = axis_window(p, p.x, x, true);
        if (!start_ok(win, x, S.BX0) || ci.tabOff % p.x.taps != 0)
            return;
        const std::vector<int32_t> c = phase_row(p.x, ci.tabOff / p.x.taps);
        std::vector<int32_t> &ref = xs[x & 1];
        if (ref.empty())
            ref = c;
        if (ref != c)
            return;
        const int side = x < 8 ? 0 : x >= p.dstW - 8 ? 1 : -1;
        if (win.border && side < 0)
            return;
        if (side >= 0) {
            const int j = side ? x - (p.dstW - 8) : x;
            if (!magic_x(win.border ? win.div : (1 << 20), &d->xM[side][j], &d->xT[side][j]))
                return;
        }
    }
    // rows: the same fixed window starts and the two phases for every row; one contiguous run of
    // main rows with at most 8 masked border rows above and below
    std::vector<int32_t> ys[2];
    int m0 = -1, m1 = -1;
    for (int y = 0; y < p.dstH; ++y) {
        const CoordInfo &ci = p.y.coord[static_cast<size_t>(y)];
        const Window win = axis_window(p, p.y, y, false);
        if (!start_ok(win, y, S.GA) || ci.tabOff % p.y.taps != 0)
            return;
        std::vector<int32_t> &ref = ys[y & 1];
        const std::vector<int32_t> c = phase_row(p.y, ci.tabOff / p.y.taps);
        if (ref.empty())
            ref = c;
        if (ref != c)
            return;
        if (!win.border) {
            if (win.start < 0 || win.start + T > p.srcH)
                return;
            if (m0 < 0)
                m0 = y;
            else if (m1 >= 0)
                return;
        } else if (m0 >= 0 && m1 < 0) {
            m1 = y;
        }
    }
    if (m0 < 0)
        return;
    if (m1 < 0)
        m1 = p.dstH;
    if (m0 > 8 || p.dstH - m1 > 8 || ys[0].empty() || ys[1].empty() || xs[0].empty() || xs[1].empty())
        return;
    for (int y = 0; y < p.dstH; ++y) {
        if (y >= m0 && y < m1)
            continue;
        const Window win = axis_window(p, p.y, y, false);
        const int side = y < m0 ? 0 : 1, i = side ? y - m1 : y;
        if (!win.border || !magic_y(win.div, &d->yM[side][i], &d->yS[side][i]))
            return;
    }
    // group rows: the even row's tap t is group row t, the odd row's tap t group row t + 1; the
    // kernel multiplies group rows 0 .. NTY-1 (even) and PO1 .. PO1+NTY-1 (odd)
    for (int t = 0; t < T; ++t) {
        if ((t >= S.NTY && ys[0][static_cast<size_t>(t)] != 0) ||
            ((t + 1 < S.PO1 || t + 1 >= S.PO1 + S.NTY) && ys[1][static_cast<size_t>(t)] != 0))
            return;
    }
    auto splat = [](int32_t c) { return (static_cast<uint32_t>(c) & 0xffffu) * 0x10001u; };
    for (int t = 0; t < S.NTY; ++t) {
        d->cy[0][t] = splat(t < T ? ys[0][static_cast<size_t>(t)] : 0);
        const int u = S.PO1 - 1 + t;
        d->cy[1][t] = splat(u >= 0 && u < T ? ys[1][static_cast<size_t>(u)] : 0);
    }
    auto tap = [&](int ph, int k) { return k < T ? xs[ph][static_cast<size_t>(k)] : 0; };
    for (int ph = 0; ph < 2; ++ph)
        for (int q = 0; q < S.NPX; ++q)
            d->cx[ph][q] = (static_cast<uint32_t>(tap(ph, 2 * q)) & 0xffffu) |
                           (static_cast<uint32_t>(tap(ph, 2 * q + 1)) << 16);
    d->variant = vi;
    d->m0 = m0;
    d->m1 = m1;
    d->ok = true;
}

bool ryx_columns(const Plan &p, int NP, RyxTables *t);
int ryx_column_pairs(const Plan &p);

void build_ryx(const Plan &p, RyxTables *t)
{
    *t = RyxTables();
    // widths: launch_ryx's limits (up to 4 column parts of 512 threads; abi.cpp ryx_dev drops the
    // kernel when no split fits)
    if (p.method == kLinear || p.x.identity || p.y.identity || p.srcW > 8192 || p.dstW > 4096 || p.srcW < 16 ||
        p.dstH < 4)
        return;
    // the kernel's register window holds the rows of one group of Q outputs: downscales, and the
    // Lanczos 4:9 upscale (480 -> 1080 rows)
    const int64_t g = std::gcd(static_cast<int64_t>(p.srcH), static_cast<int64_t>(p.dstH));
    const int P = static_cast<int>(p.srcH / g), Q = static_cast<int>(p.dstH / g);
    const int T = p.y.taps;
    if (p.y.phases != Q || Q > 16 || (P <= Q && !(p.method == kLanczos && P == 4 && Q == 9)))
        return;
    // phase j's reference window starts at P m + floor(P j / Q) + offj[j] for every group m (the
    // kernel window covers every phase's nonzero taps, so the offsets may differ between phases)
    std::vector<int> offj(static_cast<size_t>(Q), 0);
    std::vector<bool> seen(static_cast<size_t>(Q), false);
    for (int y = 0; y < p.dstH; ++y) {
        const CoordInfo &ci = p.y.coord[static_cast<size_t>(y)];
        const int m = y / Q, j = y % Q;
        if (ci.kind == kIdentity || ci.tabOff != j * T)
            return;
        const int o = ci.srcO - P * m - (P * j) / Q;
        if (seen[static_cast<size_t>(j)] && offj[static_cast<size_t>(j)] != o)
            return;
        seen[static_cast<size_t>(j)] = true;
        offj[static_cast<size_t>(j)] = o;
    }
    // Lanczos: outer taps that quantise to zero in every phase are dropped (a zero tap adds
    // nothing to the sum; a masked border row's divisor is the reference's own, magic_y below):
    // Lanczos-3 9:4 takes 12 of 14 rows, 4:1 14 of 24, Lanczos-4 2:1 12 of 16.  [lowest,
    // highest]: the rows (relative to P m + floor(P j / Q)) any phase's nonzero taps touch
    int lowest = 1 << 30, highest = -(1 << 30), maxEnd = -(1 << 30);
    for (int j = 0; j < Q; ++j) {
        const int32_t *c = &p.y.table[static_cast<size_t>(j * T)];
        int lo = 0, hi = T - 1;
        if (p.method == kLanczos) {
            while (lo < T && c[lo] == 0)
                ++lo;
            while (hi > lo && c[hi] == 0)
                --hi;
            if (lo == T)
                continue;  // an all-zero phase (none in practice)
        }
        lowest = std::min(lowest, offj[static_cast<size_t>(j)] + lo);
        highest = std::max(highest, offj[static_cast<size_t>(j)] + hi);
        maxEnd = std::max(maxEnd, offj[static_cast<size_t>(j)] + T);
    }
    if (highest < lowest)
        return;
    const int TE = highest - lowest + 1;
    const int minOff = *std::min_element(offj.begin(), offj.end());  // the kernel window stays inside
                                                                     // the reference's windows
    // instantiated (method, P, Q, taps, column pairs) shapes: kernels.hip launch_ryx.  The fewest
    // taps >= TE (the window may keep some zero taps), then the fewest pairs that hold every column
    // window (an odd start takes one more entry)
    struct Shape {
        int method, P, Q, T, NP;
    };
    static const Shape kShapes[] = {{kLanczos, 9, 4, 12, 8},  {kLanczos, 9, 4, 12, 10}, {kLanczos, 9, 4, 8, 6},
                                    {kLanczos, 9, 4, 8, 7},   {kArea, 9, 4, 4, 3},      {kLanczos, 4, 1, 14, 9},
                                    {kLanczos, 4, 1, 14, 13}, {kLanczos, 4, 1, 22, 17}, {kLanczos, 2, 1, 4, 3},   {kLanczos, 2, 1, 12, 9},
                                    {kLanczos, 2, 1, 16, 11}, {kLanczos, 2, 1, 18, 13}, {kLanczos, 2, 1, 20, 15},
                                    {kLanczos, 2, 1, 22, 17}, {kLanczos, 2, 1, 24, 19}, {kLanczos, 4, 9, 6, 4},
                                    {kLanczos, 4, 9, 4, 3}};
    const int needNP = ryx_column_pairs(p);
    const Shape *best = nullptr;
    for (const Shape &S : kShapes)
        if (S.method == p.method && S.P == P && S.Q == Q && S.T >= TE && S.T <= maxEnd - minOff && needNP <= S.NP &&
            (!best || S.T < best->T || (S.T == best->T && S.NP < best->NP)))
            best = &S;
    if (!best)
        return;
    const int TK = best->T, NP = best->NP;
    // the kernel window of output (m, j): TK rows from P m + floor(P j / Q) + off, ending no later
    // than the reference's windows (a downscale: taps [lo, lo + TK) of every phase, lo = the
    // leading zero taps or fewer)
    int off = std::min(lowest, maxEnd - TK);
    // Lanczos 2:1 (symmetric window, below): a window wider than the nonzero taps is padded evenly
    // on both sides (an instantiation with more taps, picked for its column pairs)
    if (p.method == kLanczos && (P == 2 || P == 4) && Q == 1 && (TK - TE) % 2 == 0 && lowest - (TK - TE) / 2 >= minOff &&
        lowest - (TK - TE) / 2 + TK <= maxEnd)
        off = lowest - (TK - TE) / 2;
    t->rowCoef.assign(static_cast<size_t>(Q * TK), 0u);
    for (int j = 0; j < Q; ++j)
        for (int k = 0; k < T; ++k) {
            const int32_t c = p.y.table[static_cast<size_t>(j * T + k)];
            const int w = offj[static_cast<size_t>(j)] + k - off;  // kernel window row of tap k
            if (w < 0 || w >= TK) {
                if (c != 0)
                    return;
                continue;
            }
            t->rowCoef[static_cast<size_t>(j * TK + w)] = (static_cast<uint32_t>(c) & 0xffffu) * 0x10001u;
        }
    // Lanczos 2:1 (one phase): the kernel pair-sums mirrored window rows before the packed MAC
    // (kernels.hip ryx_kernel SYMV), so its window must be symmetric -- the reference's 2:1 tables
    // are, and the zero-tap trim is symmetric too; anything else takes the other kernels
    if (p.method == kLanczos && (P == 2 || P == 4) && Q == 1)
        for (int w = 0; w < TK; ++w)
            if (t->rowCoef[static_cast<size_t>(w)] != t->rowCoef[static_cast<size_t>(TK - 1 - w)])
                return;
    int m0 = 0, m1 = p.dstH;
    if (p.method == kLanczos) {
        m0 = -1;
        m1 = -1;
        for (int y = 0; y < p.dstH; ++y) {
            const Window win = axis_window(p, p.y, y, false);
            if (!win.border) {
                if (win.start < 0 || win.start + T > p.srcH)
                    return;
                if (m0 < 0)
                    m0 = y;
                else if (m1 >= 0)
                    return;
            } else if (m0 >= 0 && m1 < 0) {
                m1 = y;
            }
        }
        if (m0 < 0)
            return;
        if (m1 < 0)
            m1 = p.dstH;
        if (m0 > 16 || p.dstH - m1 > 16)
            return;
        for (int y = 0; y < p.dstH; ++y) {
            if (y >= m0 && y < m1)
                continue;
            const Window win = axis_window(p, p.y, y, false);
            const int side = y < m0 ? 0 : 1, i = side ? y - m1 : y;
            if (!win.border || !magic_y(win.div, &t->yM[side][i], &t->yS[side][i]))
                return;
        }
    }
    if (!ryx_columns(p, NP, t))
        return;
    t->P = P;
    t->Q = Q;
    t->taps = TK;
    t->off = off;
    t->NP = NP;
    t->m0 = m0;
    t->m1 = m1;
    t->ok = true;
}

void build_ryg(const Plan &p, RyxTables *t)
{
    *t = RyxTables();
    // rows shrink by more than 1 and at most 2 (consecutive windows start 1 or 2 rows apart), or
    // grow (round 5: windows 0 or 1 rows apart, one new row per output row); widths as ryx_kernel
    if (p.x.identity || p.y.identity || p.srcW > 8192 || p.dstW > 4096 || p.srcW < 16 || p.dstH < 4 ||
        p.srcH == p.dstH || p.srcH > 4 * p.dstH)
        return;
    const bool up = p.dstH > p.srcH;
    // Linear (round 5): downscales by at most 2 on both axes (no clamped reads,
    // IQOLinearResizerImpl_Generic.cpp:210-282, 327-407).  Its sums are Area's (16-bit vertical
    // sums, the same x rounding), so it runs the Area instantiations with a zero third row tap; the
    // replicated border row / column (one per side) is a one-tap window of weight 256 / 2^15, whose
    // sum rounds as the reference's (v * 256 + 128) >> 8 does
    const bool linear = p.method == kLinear;
    if (linear && (up || p.srcH > 2 * p.dstH || p.srcW <= p.dstW || p.srcW > 2 * p.dstW))
        return;
    const int sm = linear ? static_cast<int>(kArea) : static_cast<int>(p.method);  // the kernel's arithmetic
    // window advance per output row (= rows loaded per output row)
    const int maxAdv = up ? 1 : p.srcH > 3 * p.dstH ? 4 : p.srcH > 2 * p.dstH ? 3 : 2;
    if (up && p.method != kLanczos)
        return;
    const int T = p.y.taps;
    // Lanczos: outer taps that are zero in every phase are dropped (as build_ryx)
    int lo = 0, hi = T - 1;
    if (p.method == kLanczos) {
        lo = T;
        hi = -1;
        for (int j = 0; j < p.y.phases; ++j) {
            const int32_t *c = &p.y.table[static_cast<size_t>(j * T)];
            int a = 0, b = T - 1;
            while (a < T && c[a] == 0)
                ++a;
            while (b > a && c[b] == 0)
                --b;
            if (a == T)
                continue;
            lo = std::min(lo, a);
            hi = std::max(hi, b);
        }
        if (hi < lo)
            return;
    }
    const int TE = hi - lo + 1;
    // instantiated (method, taps, column pairs): kernels.hip launch_ryg
    struct Shape {
        int method, T, NP;
    };
    // (Area, 3 taps: slower than the wave walker with the first ryg (1080p -> 1366x768 x256 0.348 vs
    // 0.275 ms, profiles/r05/steady_ryg.txt), faster since the ring and the columns-per-thread rule:
    // 0.199 vs 0.271 ms, profiles/r05/steady_ryg_area.txt)
    static const Shape kShapes[] = {{kLanczos, 4, 3},  {kLanczos, 6, 4},  {kLanczos, 8, 5},  {kLanczos, 10, 5},
                                    {kLanczos, 10, 6}, {kLanczos, 12, 7}, {kArea, 3, 2},     {kArea, 3, 3},
                                    {kLanczos, 14, 8}, {kLanczos, 16, 9}, {kLanczos, 18, 10}, {kArea, 4, 3},
                                    {kArea, 4, 4},     {kLanczos, 20, 11}, {kLanczos, 22, 12}, {kLanczos, 24, 13},
                                    {kArea, 5, 3},     {kArea, 5, 4},     {kLanczos, 12, 8}, {kLanczos, 18, 12},
                                    {kLanczos, 22, 16}, {kLanczos, 16, 10}, {kLanczos, 16, 12}};
    const int needNP = ryx_column_pairs(p);
    const Shape *best = nullptr;
    for (const Shape &S : kShapes)
        if (S.method == sm && S.T >= TE && S.T <= T + (linear ? 1 : 0) && needNP <= S.NP && (!up || S.T <= 8) &&
            // (kernels.hip instantiations: NL = 3 Lanczos (T, T/2 + 1) for T 10 .. 18 and Area (4, 3 / 4);
            // and (18, 12), (22, 16) (round 6, Lanczos-4 / -5); NL = 4 (T, T/2 + 1) for T 14 .. 24 and (22, 16); NL = 2 up to 12 taps, (12, 8) for Lanczos-5, (16, 10 / 12) for Lanczos-5 / -6; NL = 1 Lanczos 4, 6, 8 taps)
            (maxAdv == 4   ? (sm == kArea ? S.T == 5 : S.T >= 14 && (S.NP == S.T / 2 + 1 || (S.T == 22 && S.NP == 16)))
             : maxAdv == 3 ? (sm == kArea ? S.T == 4
                                           : (S.T >= 10 && S.T <= 18 && (S.NP == S.T / 2 + 1 || (S.T == 18 && S.NP == 12))) ||
                                                 (S.T == 22 && S.NP == 16))
                           : (S.T <= 12 || (S.T == 16 && S.NP >= 10)) && !(sm == kArea && S.T >= 4)) &&
            (!best || S.T < best->T || (S.T == best->T && S.NP < best->NP)))  // (upscales: kernels.hip NL = 1 shapes)
            best = &S;
    if (!best)
        return;
    const int TK = best->T, NP = best->NP;
    const int off = TK > T ? 0 : std::min(lo, T - TK);  // kernel window: taps [off, off + TK) of the reference's
    // per-phase taps as (c, c) splats
    // (Linear: two more phases, the replicated first row (window from row 0) and last row (window
    // from row srcH - 2, its second tap))
    t->rowCoef.assign(static_cast<size_t>(p.y.phases + (linear ? 2 : 0)) * TK, 0u);
    if (linear) {
        t->rowCoef[static_cast<size_t>(p.y.phases) * TK] = 256u * 0x10001u;
        t->rowCoef[static_cast<size_t>(p.y.phases + 1) * TK + 1] = 256u * 0x10001u;
    }
    for (int j = 0; j < p.y.phases; ++j)
        for (int k = 0; k < T; ++k) {
            const int32_t c = p.y.table[static_cast<size_t>(j * T + k)];
            if (k < off || k >= off + TK) {
                if (c != 0)
                    return;
                continue;
            }
            t->rowCoef[static_cast<size_t>(j * TK + k - off)] = (static_cast<uint32_t>(c) & 0xffffu) * 0x10001u;
        }
    // rows: {first window row, tap offset}; windows 1 or 2 rows apart; Lanczos main rows in one
    // range [m0, m1) with their whole window in the image, at most 16 masked border rows per side
    t->rowRec.assign(static_cast<size_t>(p.dstH) * 2, 0);
    int m0 = 0, m1 = p.dstH;
    if (p.method == kLanczos) {
        m0 = -1;
        m1 = -1;
    }
    for (int y = 0; y < p.dstH; ++y) {
        const CoordInfo &ci = p.y.coord[static_cast<size_t>(y)];
        if (ci.kind == kIdentity || ci.tabOff % T)
            return;
        const bool lb = linear && ci.kind != kMain;  // Linear replicated border row
        if (lb && (ci.kind != kBorderLo && ci.kind != kBorderHi))
            return;
        const int s0 = lb ? (ci.kind == kBorderLo ? 0 : p.srcH - 2) : ci.srcO + off;
        if (y > 0) {
            const int adv = s0 - t->rowRec[static_cast<size_t>(2 * y - 2)];
            if (adv < (up ? 0 : maxAdv - 1) || adv > maxAdv)
                return;
        }
        t->rowRec[static_cast<size_t>(2 * y)] = s0;
        t->rowRec[static_cast<size_t>(2 * y + 1)] = lb ? (p.y.phases + (ci.kind == kBorderLo ? 0 : 1)) * TK : ci.tabOff / T * TK;
        if (p.method == kLanczos) {
            const Window win = axis_window(p, p.y, y, false);
            if (!win.border) {
                if (win.start < 0 || win.start + T > p.srcH)
                    return;
                if (m0 < 0)
                    m0 = y;
                else if (m1 >= 0)
                    return;
            } else if (m0 >= 0 && m1 < 0) {
                m1 = y;
            }
        } else if (s0 + TK > p.srcH + 1) {
            return;  // (Area reads at most one row past the end, with weight 0: it loads as zero)
        }
    }
    if (p.method == kLanczos) {
        if (m0 < 0)
            return;
        if (m1 < 0)
            m1 = p.dstH;
        if (m0 > 16 || p.dstH - m1 > 16)
            return;
        for (int y = 0; y < p.dstH; ++y) {
            if (y >= m0 && y < m1)
                continue;
            const Window win = axis_window(p, p.y, y, false);
            const int side = y < m0 ? 0 : 1, i = side ? y - m1 : y;
            if (!win.border || !magic_y(win.div, &t->yM[side][i], &t->yS[side][i]))
                return;
        }
    }
    if (!ryx_columns(p, NP, t))
        return;
    // kRygRecPad copies of the last record: the kernel reads the records of rows up to its prefetch
    // depth + 2 past the band's end without clamping (their loads are masked)
    const int32_t lastS = t->rowRec[static_cast<size_t>(2 * p.dstH - 2)], lastC = t->rowRec[static_cast<size_t>(2 * p.dstH - 1)];
    for (int k = 0; k < kRygRecPad; ++k) {
        t->rowRec.push_back(lastS);
        t->rowRec.push_back(lastC);
    }
    t->general = true;
    t->rowLoads = maxAdv;
    t->P = 0;
    t->Q = 0;
    t->taps = TK;
    t->off = off;
    t->NP = NP;
    t->m0 = m0;
    t->m1 = m1;
    t->ok = true;
}

bool build_ryu_positions(int dstH, RyxTables *t)
{
    t->posRec.clear();
    t->posBase = 0;
    t->posRows = 0;
    if (!t->ok || !t->general || dstH < 1 || t->rowRec.size() < static_cast<size_t>(2 * dstH))
        return false;
    std::vector<int32_t> pos;
    const int32_t s0 = t->rowRec[0];
    int most = 0;
    for (int y = 0; y < dstH; ++y) {
        const int32_t s = t->rowRec[static_cast<size_t>(2 * y)], c = t->rowRec[static_cast<size_t>(2 * y + 1)];
        const int64_t k = static_cast<int64_t>(s) - s0;
        // (downscales: the positions a window skips hold no rows)
        while (static_cast<int64_t>(pos.size() / kRyuRec) < k) {
            pos.insert(pos.end(), kRyuRec, c);
            pos[pos.size() - kRyuRec] = y;
            pos[pos.size() - kRyuRec + 1] = 0;
        }
        const int64_t n = static_cast<int64_t>(pos.size() / kRyuRec);
        if (k == n) {
            pos.insert(pos.end(), kRyuRec, c);  // (tap offsets past the position's rows: its last row's)
            pos[pos.size() - kRyuRec] = y;
            pos[pos.size() - kRyuRec + 1] = 1;
        } else if (k == n - 1 && pos[pos.size() - kRyuRec + 1] >= 1 && pos[pos.size() - kRyuRec + 1] < kRyuRec - 2) {
            const int j = ++pos[pos.size() - kRyuRec + 1];
            for (int q = j + 1; q < kRyuRec; ++q)
                pos[pos.size() - kRyuRec + q] = c;
        } else {
            return false;  // a window that moved back or skipped a row, or too many rows
        }
        most = std::max(most, pos[pos.size() - kRyuRec + 1]);
    }
    if (most > kRyuMaxRows)
        return false;
    std::vector<int32_t> last(pos.end() - kRyuRec, pos.end());
    last[0] = dstH;
    last[1] = 1;
    for (int k = 0; k < kRyuPosPad; ++k)
        pos.insert(pos.end(), last.begin(), last.end());
    t->posRec = std::move(pos);
    t->posBase = s0;
    t->posRows = most;
    return true;
}

bool build_ryu_runs(int dstW, RyxTables *t)
{
    t->colRun.clear();
    t->runPairs = 0;
    const int NP = t->NP;
    if (!t->ok || NP < 1 || dstW < 1 || t->cols.size() < static_cast<size_t>(4 * dstW) ||
        t->colCoef.size() < static_cast<size_t>(NP) * dstW)
        return false;
    // dword offset of each column's window in its group's run (from the lowest even start of the
    // group: a phase-0 column's window is trimmed to its one nonzero tap, so the starts are not
    // monotonic), and the pairs the run must hold
    std::vector<int> off(static_cast<size_t>(dstW));
    int need = 0;
    for (int x = 0; x < dstW; ++x) {
        int lo = t->cols[static_cast<size_t>(4 * x)];
        for (int k = x & ~3; k < std::min(dstW, (x & ~3) + 4); ++k)
            lo = std::min(lo, t->cols[static_cast<size_t>(4 * k)]);
        const int d = t->cols[static_cast<size_t>(4 * x)] - lo;
        if (d % 4)
            return false;
        off[static_cast<size_t>(x)] = d / 4;
        int last = -1;  // the column's last nonzero pair
        for (int q = 0; q < NP; ++q)
            if (t->colCoef[static_cast<size_t>(x) * NP + q])
                last = q;
        need = std::max(need, d / 4 + last + 1);
    }
    const int R = std::max(need, NP + 1);
    if (R > NP + 2)
        return false;  // (kernels.hip instantiates runs of NP + 1 and NP + 2 pairs)
    t->colRun.assign(static_cast<size_t>(dstW) * R, 0u);
    for (int x = 0; x < dstW; ++x)
        for (int q = 0; q < NP; ++q) {
            const int r = off[static_cast<size_t>(x)] + q;
            const uint32_t c = t->colCoef[static_cast<size_t>(x) * NP + q];
            if (r < R)
                t->colRun[static_cast<size_t>(x) * R + r] = c;
            else if (c)
                return false;
        }
    t->runPairs = R;
    return true;
}

// The nonzero taps [first, last] of output column x (round 5: the column tables drop the zero taps
// at either end of a window, e.g. Lanczos-3 1920 -> 1366 has 10-tap windows holding at most 9
// nonzero taps: 5 pairs instead of 6)
static void column_nonzero(const Plan &p, int x, int *first, int *last)
{
    const CoordInfo &ci = p.x.coord[static_cast<size_t>(x)];
    const int32_t *c = &p.x.table[static_cast<size_t>(ci.tabOff)];
    int a = 0, b = p.x.taps - 1;
    while (a < b && c[a] == 0)
        ++a;
    while (b > a && c[b] == 0)
        --b;
    *first = a;
    *last = b;
}

// Linear's replicated border column: a one-tap window on the first / last source column
static bool linear_border_column(const Plan &p, int x, int *start)
{
    const CoordInfo &ci = p.x.coord[static_cast<size_t>(x)];
    if (p.method != kLinear || ci.kind == kMain || ci.kind == kIdentity)
        return false;
    *start = ci.kind == kBorderLo ? 0 : p.srcW - 1;
    return true;
}

int ryx_column_pairs(const Plan &p)
{
    int need = 0;
    for (int x = 0; x < p.dstW; ++x) {
        int a, b, lbs;
        column_nonzero(p, x, &a, &b);
        if (linear_border_column(p, x, &lbs)) {
            a = 0;
            b = 0;
        }
        const int start = linear_border_column(p, x, &lbs) ? lbs : p.x.coord[static_cast<size_t>(x)].srcO + a;
        need = std::max(need, (start + (b - a) - (start & ~1)) / 2 + 1);
    }
    return need;
}

// The tabled columns of ryx_kernel / ryg_kernel: the reference's window less its zero end taps,
// made to start on an even column (a leading zero coefficient), NP pairs; masked Lanczos border
// taps outside the image meet the zero padding of the work row
bool ryx_columns(const Plan &p, int NP, RyxTables *t)
{
    t->cols.assign(static_cast<size_t>(p.dstW) * 4, 0);
    t->colCoef.assign(static_cast<size_t>(p.dstW) * NP, 0u);
    for (int x = 0; x < p.dstW; ++x) {
        const CoordInfo &ci = p.x.coord[static_cast<size_t>(x)];
        if (ci.kind == kIdentity)
            return false;
        int k0, k1, lbs;
        column_nonzero(p, x, &k0, &k1);
        const bool lb = linear_border_column(p, x, &lbs);
        if (lb)
            k1 = k0;
        const int start = lb ? lbs : ci.srcO + k0;
        const int a = start & ~1;  // even start (floor)
        if (a < -kRyxPad || a + 2 * NP > p.srcW + kRyxPad || start - a + (k1 - k0) >= 2 * NP)
            return false;
        std::vector<int32_t> c(static_cast<size_t>(2 * NP), 0);
        for (int k = k0; k <= k1; ++k)
            c[static_cast<size_t>(start - a + k - k0)] = lb ? 1 << 15 : p.x.table[static_cast<size_t>(ci.tabOff + k)];
        for (int q = 0; q < NP; ++q)
            t->colCoef[static_cast<size_t>(x) * NP + q] = (static_cast<uint32_t>(c[static_cast<size_t>(2 * q)]) & 0xffffu) |
                                                       (static_cast<uint32_t>(c[static_cast<size_t>(2 * q + 1)]) << 16);
        uint32_t m = 0;
        int32_t sh = 0;
        if (p.method == kLanczos) {
            const Window win = axis_window(p, p.x, x, true);
            if (!magic_x(win.border ? win.div : (1 << 20), &m, &sh))
                return false;
        }
        int32_t *cx = &t->cols[static_cast<size_t>(x) * 4];
        cx[0] = 2 * (a + kRyxPad);  // byte offset in the work row
        cx[1] = static_cast<int32_t>(m);
        cx[2] = sh;
    }
    return true;
}

void build_d31(const Plan &p, D31Tables *d)
{
    *d = D31Tables();
    if (p.method != kLanczos || p.x.identity || p.y.identity || p.srcW != 3 * p.dstW || p.srcH != 3 * p.dstH ||
        p.dstW % 4 || p.dstW < 16 || p.dstH < 8)
        return;
    // the instantiated tap structures (kernels.hip D31Shape): taps T, window start B relative to 3y,
    // the symmetric pair distances about the centre tap T/2 (non-zero taps only), the zero taps
    struct Shape {
        int T, B, npy;
        int dist[5];
    };
    static const Shape kShapes[2] = {{18, -8, 5, {1, 2, 4, 5, 7}}, {12, -5, 4, {1, 2, 4, 5, 0}}};
    const int T = static_cast<int>(p.x.taps);
    if (static_cast<int>(p.y.taps) != T || p.x.phases != 1 || p.y.phases != 1)
        return;
    int vi = -1;
    for (int k = 0; k < 2; ++k)
        if (kShapes[k].T == T)
            vi = k;
    if (vi < 0)
        return;
    const Shape &S = kShapes[vi];
    const int C = T / 2;
    // every window (main or masked border) starts at 3i + B and takes the one phase
    for (const AxisPlan *ax : {&p.x, &p.y}) {
        const bool isX = ax == &p.x;
        for (int i = 0; i < ax->dstLen; ++i) {
            const CoordInfo &ci = ax->coord[static_cast<size_t>(i)];
            if (ci.kind == kIdentity || ci.tabOff != 0 || axis_window(p, *ax, i, isX).start != 3 * i + S.B)
                return;
        }
    }
    // the Y table: tap 0 zero, taps symmetric about C, non-zero only at C and C +- dist
    const std::vector<int32_t> &ty = p.y.table, &tx = p.x.table;
    if (ty[0] != 0 || tx[0] != 0)
        return;
    for (int k = 1; k < T; ++k) {
        if (ty[static_cast<size_t>(k)] != ty[static_cast<size_t>(2 * C - k)])
            return;
        const int dist = k > C ? k - C : C - k;
        bool used = dist == 0;
        for (int q = 0; q < S.npy; ++q)
            used = used || S.dist[q] == dist;
        if (!used && ty[static_cast<size_t>(k)] != 0)
            return;
    }
    // columns: border columns only among the 4 outermost on each side
    for (int x = 0; x < p.dstW; ++x) {
        const Window win = axis_window(p, p.x, x, true);
        const int side = x < 4 ? 0 : x >= p.dstW - 4 ? 1 : -1;
        if (win.border && side < 0)
            return;
        if (side >= 0) {
            const int j = side ? x - (p.dstW - 4) : x;
            if (!magic_x(win.border ? win.div : (1 << 20), &d->xM[side][j], &d->xT[side][j]))
                return;
        }
    }
    // rows: one contiguous run of main rows with at most 8 masked border rows above and below
    int m0 = -1, m1 = -1;
    for (int y = 0; y < p.dstH; ++y) {
        const Window win = axis_window(p, p.y, y, false);
        if (!win.border) {
            if (win.start < 0 || win.start + T > p.srcH)
                return;
            if (m0 < 0)
                m0 = y;
            else if (m1 >= 0)
                return;
        } else if (m0 >= 0 && m1 < 0) {
            m1 = y;
        }
    }
    if (m0 < 0)
        return;
    if (m1 < 0)
        m1 = p.dstH;
    if (m0 > 8 || p.dstH - m1 > 8)
        return;
    for (int y = 0; y < p.dstH; ++y) {
        if (y >= m0 && y < m1)
            continue;
        const Window win = axis_window(p, p.y, y, false);
        const int side = y < m0 ? 0 : 1, i = side ? y - m1 : y;
        if (!win.border || !magic_y(win.div, &d->yM[side][i], &d->yS[side][i]))
            return;
    }
    auto splat = [](int32_t c) { return (static_cast<uint32_t>(c) & 0xffffu) * 0x10001u; };
    d->cc = splat(ty[static_cast<size_t>(C)]);
    for (int q = 0; q < S.npy; ++q)
        d->cp[q] = splat(ty[static_cast<size_t>(C + S.dist[q])]);
    auto tap = [&](int k) { return k < T ? tx[static_cast<size_t>(k)] : 0; };
    auto pr = [](int32_t lo, int32_t hi) { return (static_cast<uint32_t>(lo) & 0xffffu) | (static_cast<uint32_t>(hi) << 16); };
    for (int q = 0; q < 9; ++q) {
        d->cxe[q] = pr(tap(2 * q), tap(2 * q + 1));
        d->cxo[q] = pr(tap(2 * q + 1), tap(2 * q + 2));
    }
    d->variant = vi;
    d->m0 = m0;
    d->m1 = m1;
    d->ok = true;
}

} // namespace iqo_amd
