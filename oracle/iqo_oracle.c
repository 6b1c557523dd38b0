/*
 * iqo_oracle.c -- TEST INFRASTRUCTURE ONLY (see iqo_oracle.h).
 *
 * A clean-room C99 restatement of libiqo's Generic (scalar fixed-point) resizers.  Every
 * function cites the reference file:line whose behaviour it restates.  It is compiled strict
 * IEEE (-O2 -ffp-contract=off, no fast-math), so its coefficient tables match the reference
 * built without -Ofast; for every shape in tests/golden the Release (-Ofast) build agrees
 * (the generator records shapes where the two reference builds disagree, see gen_golden.py).
 *
 * Type discipline follows the reference exactly: size_t/ptrdiff_t arithmetic, float sums,
 * double evaluation of the windowed sinc, int16/u16 wrapping intermediates, C truncating
 * division, arithmetic right shifts.
 */
#define _POSIX_C_SOURCE 200809L
#include "iqo_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ math.hpp restatement */

/* round(x) = floor(x + 0.5) in float -- src/math.hpp:12-16 (instantiated with T=float) */
static float round_f(float x) { return floorf(x + 0.5f); }

/* gcd(a,b) -- src/math.hpp:37-49 (sign follows C '%'; caller takes |.| where the ref does) */
static int64_t gcd64(int64_t a, int64_t b)
{
    int64_t r = a % b;
    while (r) {
        a = b;
        b = r;
        r = a % b;
    }
    return b;
}

/* lcm -- src/math.hpp:52-55 */
static int64_t lcm64(int64_t a, int64_t b) { return a / gcd64(a, b) * b; }

/* div_floor -- src/math.hpp:58-65 */
static int64_t div_floor64(int64_t a, int64_t b)
{
    if ((a ^ b) < 0)
        return (a - b + 1) / b;
    return a / b;
}

/* LinearIterator -- src/math.hpp:70-155 */
typedef struct {
    int64_t dx, dy, x, y;
} lin_iter;

static void li_init(lin_iter *it, int64_t dx, int64_t dy)
{
    it->dx = dx;
    it->dy = dy;
    it->x = 0;
    it->y = 0;
}

/* setX(x) -- math.hpp:87-91 */
static void li_setx(lin_iter *it, int64_t x)
{
    it->x = (x * it->dy) % it->dx;
    it->y = (x * it->dy) / it->dx;
}

/* setX(nume, deno) -- math.hpp:96-112 */
static void li_setx_rational(lin_iter *it, int64_t nume, int64_t deno)
{
    it->y = div_floor64(nume * it->dy, deno * it->dx);
    int64_t newNume = nume * it->dx;
    int64_t newDY = it->dy * deno;
    int64_t newDX = it->dx * deno;
    int64_t g = gcd64(newNume, gcd64(newDY, newDX));
    if (g < 0)
        g = -g;
    newNume /= g;
    newDY /= g;
    newDX /= g;
    it->x = newNume % newDX;
    if (it->x < 0)
        it->x += newDX;
    it->dx = newDX;
    it->dy = newDY;
}

/* advance(a) -- math.hpp:142-149 */
static void li_advance(lin_iter *it, int64_t a)
{
    it->x += a * it->dy;
    while (it->x >= it->dx) {
        ++it->y;
        it->x -= it->dx;
    }
}

/* *it++ */
static int64_t li_post_inc(lin_iter *it)
{
    int64_t v = it->y;
    li_advance(it, 1);
    return v;
}

static int16_t clamp_i16(int16_t lo, int16_t hi, int16_t v) { return v < lo ? lo : (v > hi ? hi : v); }
static uint16_t clamp_u16(uint16_t lo, uint16_t hi, uint16_t v) { return v < lo ? lo : (v > hi ? hi : v); }

/* first max, as std::max_element */
static size_t argmax_first(const float *p, size_t n)
{
    size_t best = 0;
    for (size_t i = 1; i < n; ++i)
        if (p[best] < p[i])
            best = i;
    return best;
}

/* ------------------------------------------------------------------ Lanczos tables */

/* sinc / lanczos -- src/IQOLanczosResizerImpl_Generic.cpp:10-29 (T = double) */
static double lz_sinc(double x)
{
    double fPi = 3.14159265358979;
    double fPiX = fPi * x;
    return sin(fPiX) / fPiX;
}

static double lz_lanczos(int degree, double x)
{
    double absX = fabs(x);
    if (fmod(absX, 1.0) < 1e-5)
        return absX < 1e-5 ? 1 : 0;
    if ((double)degree <= absX)
        return 0;
    return lz_sinc(x) * lz_sinc(x / degree);
}

/* calcNumCoefsForLanczos -- IQOLanczosResizerImpl_Generic.cpp:32-96 */
static size_t lz_num_coefs(int degree, size_t srcLen, size_t dstLen, size_t pxScale)
{
    if (srcLen <= dstLen)
        return (size_t)(2 * degree);
    size_t degree2 = (size_t)degree / pxScale;
    if (degree2 < 1)
        degree2 = 1;
    return (size_t)(2 * (ptrdiff_t)ceil((double)(degree2 * srcLen) / (double)dstLen));
}

/* setLanczosTable -- IQOLanczosResizerImpl_Generic.cpp:111-191 */
static float lz_set_table(int degree, size_t srcLen, size_t dstLen, ptrdiff_t dstOffset,
                          size_t pxScale, ptrdiff_t numCoefs, float *fTable)
{
    double beginX = 0;
    if (srcLen > dstLen) {
        int degFactor = (int)pxScale / degree;
        if (degFactor < 1)
            degFactor = 1;
        size_t off = (size_t)dstOffset * srcLen % dstLen;
        beginX = (double)(-degree * degFactor) - 0.5 * (double)pxScale +
                 0.5 * (double)dstLen * (double)pxScale / (double)srcLen +
                 (double)((dstLen - off) * pxScale % srcLen) / (double)srcLen;
    } else {
        double srcOffset = fmod((double)((size_t)dstOffset * srcLen) / (double)dstLen, 1.0);
        beginX = -degree + 1.0 - srcOffset;
        srcLen = dstLen;
        pxScale = 1;
    }
    float fSum = 0;
    for (ptrdiff_t i = 0; i < numCoefs; ++i) {
        double x = beginX + (double)((size_t)i * dstLen * pxScale) / (double)srcLen;
        float v = (float)lz_lanczos(degree, x);
        fTable[i] = v;
        fSum += v;
    }
    return fSum;
}

/* adjustCoefs (int16) -- IQOLanczosResizerImpl_Generic.cpp:341-367 */
static void lz_adjust(float *src, size_t n, float srcSum, int bias, int16_t *dst)
{
    int dstSum = 0;
    for (size_t i = 0; i < n; ++i) {
        dst[i] = (int16_t)round_f(src[i] * (float)bias / srcSum);
        dstSum += dst[i];
    }
    while (dstSum < bias) {
        size_t i = argmax_first(src, n);
        dst[i]++;
        src[i] = 0;
        dstSum++;
    }
    while (dstSum > bias) {
        size_t i = argmax_first(src, n);
        dst[i]--;
        src[i] = 0;
        dstSum--;
    }
}

/* ------------------------------------------------------------------ Area tables */

/* calcNumCoefsForArea -- IQOAreaResizerImpl_Generic.cpp:11-65 */
static size_t ar_num_coefs(size_t srcLen, size_t dstLen)
{
    if (srcLen < dstLen)
        return 1;
    size_t iScale = (srcLen / dstLen) * dstLen;
    size_t numCoefs = ((srcLen + (dstLen - 1)) / dstLen * dstLen) / dstLen;
    if (lcm64((int64_t)srcLen, (int64_t)iScale) > (int64_t)srcLen)
        numCoefs++;
    return numCoefs;
}

/* setAreaTable -- IQOAreaResizerImpl_Generic.cpp:74-97 */
static float ar_set_table(size_t srcLen, size_t dstLen, ptrdiff_t dstOffset, ptrdiff_t numCoefs,
                          float *fTable)
{
    double srcBeginX = (double)((size_t)dstOffset * srcLen) / (double)dstLen;
    double srcEndX = (double)((size_t)(dstOffset + 1) * srcLen) / (double)dstLen;
    double srcX = srcBeginX;
    float fSum = 0;
    for (ptrdiff_t i = 0; i < numCoefs; ++i) {
        double fl = floor(srcX) + 1.0;
        double nextSrcX = (fl < srcEndX) ? fl : srcEndX; /* std::min(srcEndX, fl) */
        float v = (float)(nextSrcX - srcX);
        fTable[i] = v;
        fSum += v;
        srcX = nextSrcX;
    }
    return fSum;
}

/* adjustCoefs (u16) -- IQOAreaResizerImpl_Generic.cpp:222-248 */
static void ar_adjust(float *src, size_t n, float srcSum, uint16_t bias, uint16_t *dst)
{
    int k1_0 = bias;
    int dstSum = 0;
    for (size_t i = 0; i < n; ++i) {
        dst[i] = (uint16_t)round_f(src[i] * (float)bias / srcSum);
        dstSum += dst[i];
    }
    while (dstSum < k1_0) {
        size_t i = argmax_first(src, n);
        dst[i]++;
        src[i] = 0;
        dstSum++;
    }
    while (dstSum > k1_0) {
        size_t i = argmax_first(src, n);
        dst[i]--;
        src[i] = 0;
        dstSum--;
    }
}

/* ------------------------------------------------------------------ Linear tables */

/* convertCoordinate -- IQOLinearResizerImpl_Generic.cpp:13-22 */
static ptrdiff_t li_convert_coordinate(ptrdiff_t fromX, ptrdiff_t fromLen, ptrdiff_t toLen)
{
    double toX = (0.5 + (double)fromX) * (double)toLen / (double)fromLen - 0.5;
    return (ptrdiff_t)ceil(fabs(toX));
}

/* setLinearTable -- IQOLinearResizerImpl_Generic.cpp:29-69 */
static void ln_set_table(size_t srcLen, size_t dstLen, float *fTable)
{
    for (size_t i = 0; i < dstLen; i++) {
        double x = (double)i;
        float coef1 = (float)modf((x + 0.5) * (double)srcLen / (double)dstLen + 0.5, &x);
        float coef0 = 1.0f - coef1;
        fTable[i * 2 + 0] = coef0;
        fTable[i * 2 + 1] = coef1;
    }
}

/* adjustCoefs (linear) -- IQOLinearResizerImpl_Generic.cpp:193-208 */
static void ln_adjust(const float *src, size_t numTables, uint16_t bias, uint16_t *dst)
{
    for (size_t i = 0; i < numTables; ++i) {
        uint16_t coef0 = (uint16_t)round_f(src[2 * i] * (float)bias);
        uint16_t coef1 = (uint16_t)(bias - coef0);
        dst[2 * i + 0] = coef0;
        dst[2 * i + 1] = coef1;
    }
}

/* ------------------------------------------------------------------ state */

struct iqo_oracle {
    int method;
    ptrdiff_t srcW, srcH, dstW, dstH;
    ptrdiff_t nX, nY, tX, tY; /* taps and phases ("tables") per axis */
    int16_t *tabX16, *tabY16; /* Lanczos */
    uint16_t *tabXu, *tabYu;  /* Area / Linear */
    int16_t *work16, *deno16;
    uint16_t *worku;
};

void iqo_oracle_free(iqo_oracle *o)
{
    if (!o)
        return;
    free(o->tabX16);
    free(o->tabY16);
    free(o->tabXu);
    free(o->tabYu);
    free(o->work16);
    free(o->deno16);
    free(o->worku);
    free(o);
}

/* init for each method: IQOLanczosResizerImpl_Generic.cpp:291-339,
 * IQOAreaResizerImpl_Generic.cpp:174-220, IQOLinearResizerImpl_Generic.cpp:157-191 */
iqo_oracle *iqo_oracle_new(int method, unsigned degree, size_t srcW, size_t srcH, size_t dstW,
                           size_t dstH, size_t pxScale)
{
    if (!srcW || !srcH || !dstW || !dstH)
        return NULL;
    if (method == IQO_ORACLE_LANCZOS && (degree < 1 || pxScale < 1))
        return NULL;
    iqo_oracle *o = (iqo_oracle *)calloc(1, sizeof(*o));
    if (!o)
        return NULL;
    o->method = method;
    o->srcW = (ptrdiff_t)srcW;
    o->srcH = (ptrdiff_t)srcH;
    o->dstW = (ptrdiff_t)dstW;
    o->dstH = (ptrdiff_t)dstH;
    size_t gW = (size_t)gcd64((int64_t)srcW, (int64_t)dstW);
    size_t gH = (size_t)gcd64((int64_t)srcH, (int64_t)dstH);
    size_t rsW = srcW / gW, rdW = dstW / gW, rsH = srcH / gH, rdH = dstH / gH;
    o->tX = (ptrdiff_t)rdW;
    o->tY = (ptrdiff_t)rdH;
    size_t maxW = srcW > dstW ? srcW : dstW;

    if (method == IQO_ORACLE_LANCZOS) {
        o->nX = (ptrdiff_t)lz_num_coefs((int)degree, rsW, rdW, pxScale);
        o->nY = (ptrdiff_t)lz_num_coefs((int)degree, rsH, rdH, pxScale);
        o->tabX16 = (int16_t *)calloc((size_t)(o->nX * o->tX), sizeof(int16_t));
        o->tabY16 = (int16_t *)calloc((size_t)(o->nY * o->tY), sizeof(int16_t));
        float *f = (float *)calloc((size_t)(o->nX > o->nY ? o->nX : o->nY), sizeof(float));
        o->work16 = (int16_t *)calloc(srcW, sizeof(int16_t));
        o->deno16 = (int16_t *)calloc(maxW, sizeof(int16_t));
        if (!o->tabX16 || !o->tabY16 || !f || !o->work16 || !o->deno16) {
            free(f);
            iqo_oracle_free(o);
            return NULL;
        }
        for (ptrdiff_t d = 0; d < o->tX; ++d) {
            float s = lz_set_table((int)degree, rsW, rdW, d, pxScale, o->nX, f);
            lz_adjust(f, (size_t)o->nX, s, 1 << 14, &o->tabX16[d * o->nX]);
        }
        for (ptrdiff_t d = 0; d < o->tY; ++d) {
            float s = lz_set_table((int)degree, rsH, rdH, d, pxScale, o->nY, f);
            lz_adjust(f, (size_t)o->nY, s, 1 << 6, &o->tabY16[d * o->nY]);
        }
        free(f);
    } else if (method == IQO_ORACLE_AREA) {
        o->nX = (ptrdiff_t)ar_num_coefs(rsW, rdW);
        o->nY = (ptrdiff_t)ar_num_coefs(rsH, rdH);
        o->tabXu = (uint16_t *)calloc((size_t)(o->nX * o->tX), sizeof(uint16_t));
        o->tabYu = (uint16_t *)calloc((size_t)(o->nY * o->tY), sizeof(uint16_t));
        float *f = (float *)calloc((size_t)(o->nX > o->nY ? o->nX : o->nY), sizeof(float));
        o->worku = (uint16_t *)calloc(srcW, sizeof(uint16_t));
        if (!o->tabXu || !o->tabYu || !f || !o->worku) {
            free(f);
            iqo_oracle_free(o);
            return NULL;
        }
        for (ptrdiff_t d = 0; d < o->tX; ++d) {
            float s = ar_set_table(rsW, rdW, d, o->nX, f);
            ar_adjust(f, (size_t)o->nX, s, (uint16_t)(1 << 15), &o->tabXu[d * o->nX]);
        }
        for (ptrdiff_t d = 0; d < o->tY; ++d) {
            float s = ar_set_table(rsH, rdH, d, o->nY, f);
            ar_adjust(f, (size_t)o->nY, s, (uint16_t)(1 << 8), &o->tabYu[d * o->nY]);
        }
        free(f);
    } else if (method == IQO_ORACLE_LINEAR) {
        o->nX = 2;
        o->nY = 2;
        o->tabXu = (uint16_t *)calloc((size_t)(2 * o->tX), sizeof(uint16_t));
        o->tabYu = (uint16_t *)calloc((size_t)(2 * o->tY), sizeof(uint16_t));
        size_t fl = (size_t)(o->tX > o->tY ? o->tX : o->tY) * 2;
        float *f = (float *)calloc(fl, sizeof(float));
        o->worku = (uint16_t *)calloc(srcW, sizeof(uint16_t));
        if (!o->tabXu || !o->tabYu || !f || !o->worku) {
            free(f);
            iqo_oracle_free(o);
            return NULL;
        }
        ln_set_table(rsW, rdW, f);
        ln_adjust(f, rdW, (uint16_t)(1 << 15), o->tabXu);
        ln_set_table(rsH, rdH, f);
        ln_adjust(f, rdH, (uint16_t)(1 << 8), o->tabYu);
        free(f);
    } else {
        free(o);
        return NULL;
    }
    return o;
}

int iqo_oracle_table(const iqo_oracle *o, int axis, int *nTaps, int *nPhases, int32_t *buf, size_t cap)
{
    if (!o)
        return -1;
    ptrdiff_t n = axis ? o->nY : o->nX, t = axis ? o->tY : o->tX;
    if (nTaps)
        *nTaps = (int)n;
    if (nPhases)
        *nPhases = (int)t;
    size_t total = (size_t)(n * t);
    if (buf && cap >= total) {
        for (size_t i = 0; i < total; ++i) {
            if (o->method == IQO_ORACLE_LANCZOS)
                buf[i] = axis ? o->tabY16[i] : o->tabX16[i];
            else
                buf[i] = axis ? o->tabYu[i] : o->tabXu[i];
        }
    }
    return (int)total;
}

/* ------------------------------------------------------------------ Lanczos resize */

/* resizeXborder -- IQOLanczosResizerImpl_Generic.cpp:539-574 */
static void lz_resize_x_border(const iqo_oracle *o, const int16_t *src, uint8_t *dst, ptrdiff_t begin, ptrdiff_t end)
{
    ptrdiff_t m = o->nX / 2;
    ptrdiff_t tableSize = o->tX * o->nX;
    ptrdiff_t iTable = (o->nX * begin) % tableSize;
    lin_iter it;
    li_init(&it, o->dstW, o->srcW);
    li_setx(&it, begin);
    for (ptrdiff_t dstX = begin; dstX < end; ++dstX) {
        ptrdiff_t srcOX = (ptrdiff_t)li_post_inc(&it) + 1;
        const int16_t *coefs = &o->tabX16[iTable];
        int32_t nume = 0, deno = 0;
        iTable += o->nX;
        if (iTable == tableSize)
            iTable = 0;
        for (ptrdiff_t i = 0; i < o->nX; ++i) {
            ptrdiff_t srcX = srcOX - m + i;
            if (0 <= srcX && srcX < o->srcW) {
                int32_t coef = coefs[i];
                nume += src[srcX] * coef;
                deno += coef;
            }
        }
        /* roundedDiv(nume, deno*kBias, 20): int16((a + 2^19) / b) -- :216-220.  deno == 0 traps
         * (SIGFPE) in the reference; such shapes are outside parity, the oracle writes 0. */
        int16_t q = deno ? (int16_t)((nume + (1 << 19)) / (deno * 64)) : 0;
        dst[dstX] = (uint8_t)clamp_i16(0, 255, q);
    }
}

/* resizeXmain -- IQOLanczosResizerImpl_Generic.cpp:582-612 */
static void lz_resize_x_main(const iqo_oracle *o, const int16_t *src, uint8_t *dst, ptrdiff_t begin, ptrdiff_t end)
{
    ptrdiff_t m = o->nX / 2;
    ptrdiff_t tableSize = o->tX * o->nX;
    ptrdiff_t iTable = (o->nX * begin) % tableSize;
    lin_iter it;
    li_init(&it, o->dstW, o->srcW);
    li_setx(&it, begin);
    for (ptrdiff_t dstX = begin; dstX < end; ++dstX) {
        ptrdiff_t srcOX = (ptrdiff_t)li_post_inc(&it) + 1;
        const int16_t *coefs = &o->tabX16[iTable];
        int32_t sum = 0;
        iTable += o->nX;
        if (iTable == tableSize)
            iTable = 0;
        for (ptrdiff_t i = 0; i < o->nX; ++i)
            sum += src[srcOX - m + i] * (int32_t)coefs[i];
        /* convertToInt(sum, 20) -- :223-227 */
        int16_t v = (int16_t)((sum + (1 << 19)) >> 20);
        dst[dstX] = (uint8_t)clamp_i16(0, 255, v);
    }
}

/* resizeX -- IQOLanczosResizerImpl_Generic.cpp:518-537 */
static void lz_resize_x(const iqo_oracle *o, const int16_t *src, uint8_t *dst)
{
    if (o->srcW == o->dstW) {
        for (ptrdiff_t x = 0; x < o->dstW; x++)
            dst[x] = (uint8_t)clamp_i16(0, 255, (int16_t)((src[x] + 32) >> 6));
        return;
    }
    ptrdiff_t m = o->nX / 2;
    ptrdiff_t mainBegin = ((m - 1) * o->dstW + o->srcW - 1) / o->srcW;
    ptrdiff_t mainEnd = (o->srcW - m) * o->dstW / o->srcW;
    if (mainEnd < 0)
        mainEnd = 0;
    lz_resize_x_border(o, src, dst, 0, mainBegin);
    lz_resize_x_main(o, src, dst, mainBegin, mainEnd);
    lz_resize_x_border(o, src, dst, mainEnd, o->dstW);
}

/* resizeYborder -- IQOLanczosResizerImpl_Generic.cpp:464-490 */
static void lz_resize_y_border(iqo_oracle *o, ptrdiff_t srcSt, const uint8_t *src, int16_t *dst,
                               ptrdiff_t srcOY, const int16_t *coefs)
{
    ptrdiff_t m = o->nY / 2;
    ptrdiff_t dstW = o->srcW;
    int16_t *nume = dst, *deno = o->deno16;
    memset(nume, 0, (size_t)dstW * sizeof(*nume));
    memset(deno, 0, (size_t)dstW * sizeof(*deno));
    for (ptrdiff_t i = 0; i < o->nY; ++i) {
        int16_t coef = coefs[i];
        ptrdiff_t srcY = srcOY - m + i;
        if (0 <= srcY && srcY < o->srcH) {
            for (ptrdiff_t x = 0; x < dstW; ++x) {
                nume[x] = (int16_t)(nume[x] + src[x + srcSt * srcY] * coef);
                deno[x] = (int16_t)(deno[x] + coef);
            }
        }
    }
    for (ptrdiff_t x = 0; x < dstW; ++x) /* deno == 0 traps in the reference: outside parity */
        dst[x] = deno[x] ? (int16_t)((int)nume[x] * 64 / deno[x]) : 0;
}

/* resizeYmain -- IQOLanczosResizerImpl_Generic.cpp:499-516 */
static void lz_resize_y_main(iqo_oracle *o, ptrdiff_t srcSt, const uint8_t *src, int16_t *dst,
                             ptrdiff_t srcOY, const int16_t *coefs)
{
    ptrdiff_t m = o->nY / 2;
    ptrdiff_t dstW = o->srcW;
    memset(dst, 0, (size_t)dstW * sizeof(*dst));
    for (ptrdiff_t i = 0; i < o->nY; ++i) {
        int16_t coef = coefs[i];
        ptrdiff_t srcY = srcOY - m + i;
        for (ptrdiff_t x = 0; x < dstW; ++x)
            dst[x] = (int16_t)(dst[x] + src[x + srcSt * srcY] * coef);
    }
}

/* resize -- IQOLanczosResizerImpl_Generic.cpp:369-454 (note: the row iterator and table cursor
 * are shared by the three loops, which matters when mainEnd < mainBegin on tiny images) */
static void lz_resize(iqo_oracle *o, size_t srcSt_, const uint8_t *src, size_t dstSt_, uint8_t *dst)
{
    ptrdiff_t srcSt = (ptrdiff_t)srcSt_, dstSt = (ptrdiff_t)dstSt_;
    int16_t *work = o->work16;
    if (o->srcH == o->dstH) {
        for (ptrdiff_t y = 0; y < o->srcH; ++y) {
            for (ptrdiff_t x = 0; x < o->srcW; ++x)
                work[x] = (int16_t)(uint16_t)(src[srcSt * y + x] * 64);
            lz_resize_x(o, work, &dst[dstSt * y]);
        }
        return;
    }
    ptrdiff_t m = o->nY / 2;
    ptrdiff_t mainBegin = ((m - 1) * o->dstH + o->srcH - 1) / o->srcH;
    ptrdiff_t mainEnd = (o->srcH - m) * o->dstH / o->srcH;
    if (mainEnd < 0)
        mainEnd = 0;
    ptrdiff_t tableSize = o->tY * o->nY;
    ptrdiff_t iTable = 0;
    lin_iter it;
    li_init(&it, o->dstH, o->srcH);

    for (ptrdiff_t dstY = 0; dstY < mainBegin; ++dstY) {
        ptrdiff_t srcOY = (ptrdiff_t)li_post_inc(&it) + 1;
        const int16_t *coefs = &o->tabY16[iTable];
        iTable += o->nY;
        if (iTable == tableSize)
            iTable = 0;
        lz_resize_y_border(o, srcSt, src, work, srcOY, coefs);
        lz_resize_x(o, work, &dst[dstSt * dstY]);
    }
    for (ptrdiff_t dstY = mainBegin; dstY < mainEnd; ++dstY) {
        ptrdiff_t srcOY = (ptrdiff_t)li_post_inc(&it) + 1;
        const int16_t *coefs = &o->tabY16[iTable];
        iTable += o->nY;
        if (iTable == tableSize)
            iTable = 0;
        lz_resize_y_main(o, srcSt, src, work, srcOY, coefs);
        lz_resize_x(o, work, &dst[dstSt * dstY]);
    }
    for (ptrdiff_t dstY = mainEnd; dstY < o->dstH; ++dstY) {
        ptrdiff_t srcOY = (ptrdiff_t)li_post_inc(&it) + 1;
        const int16_t *coefs = &o->tabY16[iTable];
        iTable += o->nY;
        if (iTable == tableSize)
            iTable = 0;
        lz_resize_y_border(o, srcSt, src, work, srcOY, coefs);
        lz_resize_x(o, work, &dst[dstSt * dstY]);
    }
}

/* ------------------------------------------------------------------ Area resize */

/* resizeXmain / resizeX -- IQOAreaResizerImpl_Generic.cpp:322-368 */
static void ar_resize_x(const iqo_oracle *o, const uint16_t *src, uint8_t *dst)
{
    if (o->srcW == o->dstW) {
        for (ptrdiff_t x = 0; x < o->dstW; x++)
            dst[x] = (uint8_t)clamp_i16(0, 255, (int16_t)((src[x] + 128) >> 8));
        return;
    }
    ptrdiff_t tableSize = o->tX * o->nX;
    ptrdiff_t iTable = 0;
    lin_iter it;
    li_init(&it, o->dstW, o->srcW);
    for (ptrdiff_t dstX = 0; dstX < o->dstW; ++dstX) {
        ptrdiff_t srcOX = (ptrdiff_t)li_post_inc(&it);
        const uint16_t *coefs = &o->tabXu[iTable];
        int sum = 0;
        iTable += o->nX;
        if (iTable == tableSize)
            iTable = 0;
        for (ptrdiff_t i = 0; i < o->nX; ++i) {
            ptrdiff_t srcX = srcOX + i;
            /* the reference reads one element past the row with weight 0 for non-integer
             * ratios (:363, ASan heap-overflow); clamp the address. */
            if (srcX >= o->srcW)
                srcX = o->srcW - 1;
            sum += src[srcX] * coefs[i];
        }
        int16_t v = (int16_t)((sum + (1 << 22)) >> 23);
        dst[dstX] = (uint8_t)clamp_u16(0, 255, (uint16_t)v);
    }
}

/* resize / resizeYmain -- IQOAreaResizerImpl_Generic.cpp:250-320 */
static void ar_resize(iqo_oracle *o, size_t srcSt_, const uint8_t *src, size_t dstSt_, uint8_t *dst)
{
    ptrdiff_t srcSt = (ptrdiff_t)srcSt_, dstSt = (ptrdiff_t)dstSt_;
    uint16_t *work = o->worku;
    if (o->srcH == o->dstH) {
        for (ptrdiff_t y = 0; y < o->srcH; ++y) {
            for (ptrdiff_t x = 0; x < o->srcW; ++x)
                work[x] = (uint16_t)(src[srcSt * y + x] * 256);
            ar_resize_x(o, work, &dst[dstSt * y]);
        }
        return;
    }
    ptrdiff_t tableSize = o->tY * o->nY;
    ptrdiff_t iTable = 0;
    lin_iter it;
    li_init(&it, o->dstH, o->srcH);
    for (ptrdiff_t dstY = 0; dstY < o->dstH; ++dstY) {
        ptrdiff_t srcOY = (ptrdiff_t)li_post_inc(&it);
        const uint16_t *coefs = &o->tabYu[iTable];
        iTable += o->nY;
        if (iTable == tableSize)
            iTable = 0;
        memset(work, 0, (size_t)o->srcW * sizeof(*work));
        for (ptrdiff_t i = 0; i < o->nY; ++i) {
            uint16_t coef = coefs[i];
            ptrdiff_t srcY = srcOY + i;
            if (srcY >= o->srcH) /* weight-0 tap past the last row: clamp (see above) */
                srcY = o->srcH - 1;
            for (ptrdiff_t x = 0; x < o->srcW; ++x)
                work[x] = (uint16_t)(work[x] + src[x + srcSt * srcY] * coef);
        }
        ar_resize_x(o, work, &dst[dstSt * dstY]);
    }
}

/* ------------------------------------------------------------------ Linear resize */

static ptrdiff_t clamp_pd(ptrdiff_t lo, ptrdiff_t hi, ptrdiff_t v) { return v < lo ? lo : (v > hi ? hi : v); }

/* resizeX / resizeXborder / resizeXmain -- IQOLinearResizerImpl_Generic.cpp:327-407 */
static void ln_resize_x(const iqo_oracle *o, const uint16_t *src, uint8_t *dst)
{
    if (o->srcW == o->dstW) {
        for (ptrdiff_t x = 0; x < o->dstW; x++)
            dst[x] = (uint8_t)clamp_i16(0, 255, (int16_t)((src[x] + 128) >> 8));
        return;
    }
    ptrdiff_t dstW = o->dstW;
    ptrdiff_t mainBegin0 = li_convert_coordinate(o->srcW, dstW, 0);
    ptrdiff_t mainBegin = clamp_pd(0, dstW, mainBegin0);
    ptrdiff_t mainEnd = clamp_pd(0, dstW, dstW - mainBegin);

    /* left border */
    {
        uint8_t v = (uint8_t)clamp_u16(0, 255, (uint16_t)(int16_t)((src[0] + 128) >> 8));
        for (ptrdiff_t x = 0; x < mainBegin; ++x)
            dst[x] = v;
    }
    /* main */
    {
        ptrdiff_t tableSize = o->tX * 2;
        ptrdiff_t iTable = (2 * mainBegin) % tableSize;
        lin_iter it;
        li_init(&it, o->dstW, o->srcW);
        li_setx_rational(&it, o->srcW - o->dstW, 2 * o->dstW);
        li_advance(&it, mainBegin);
        for (ptrdiff_t dstX = mainBegin; dstX < mainEnd; ++dstX) {
            ptrdiff_t srcOX = (ptrdiff_t)li_post_inc(&it);
            const uint16_t *coefs = &o->tabXu[iTable];
            int32_t sum = 0;
            iTable += 2;
            if (iTable == tableSize)
                iTable = 0;
            for (ptrdiff_t i = 0; i < 2; ++i) {
                /* >2x upsampling / downsampling read outside the row in the reference
                 * (:402, undefined); clamp -- such shapes are excluded from parity. */
                ptrdiff_t srcX = clamp_pd(0, o->srcW - 1, srcOX + i);
                sum += src[srcX] * (int32_t)coefs[i];
            }
            int16_t v = (int16_t)((sum + (1 << 22)) >> 23);
            dst[dstX] = (uint8_t)clamp_u16(0, 255, (uint16_t)v);
        }
    }
    /* right border */
    {
        uint8_t v = (uint8_t)clamp_u16(0, 255, (uint16_t)(int16_t)((src[o->srcW - 1] + 128) >> 8));
        for (ptrdiff_t x = mainEnd; x < dstW; ++x)
            dst[x] = v;
    }
}

/* resize -- IQOLinearResizerImpl_Generic.cpp:210-282 */
static void ln_resize(iqo_oracle *o, size_t srcSt_, const uint8_t *src, size_t dstSt_, uint8_t *dst)
{
    ptrdiff_t srcSt = (ptrdiff_t)srcSt_, dstSt = (ptrdiff_t)dstSt_;
    uint16_t *work = o->worku;
    ptrdiff_t srcW = o->srcW, srcH = o->srcH, dstH = o->dstH;
    if (srcH == dstH) {
        for (ptrdiff_t y = 0; y < srcH; ++y) {
            for (ptrdiff_t x = 0; x < srcW; ++x)
                work[x] = (uint16_t)(src[srcSt * y + x] * 256);
            ln_resize_x(o, work, &dst[dstSt * y]);
        }
        return;
    }
    ptrdiff_t mainBegin0 = li_convert_coordinate(srcH, dstH, 0);
    ptrdiff_t mainBegin = clamp_pd(0, dstH, mainBegin0);
    ptrdiff_t mainEnd = clamp_pd(0, dstH, dstH - mainBegin);

    for (ptrdiff_t dstY = 0; dstY < mainBegin; ++dstY) {
        for (ptrdiff_t x = 0; x < srcW; ++x)
            work[x] = (uint16_t)(src[x] * 256);
        ln_resize_x(o, work, &dst[dstSt * dstY]);
    }
    lin_iter it;
    li_init(&it, dstH, srcH);
    li_setx_rational(&it, srcH - dstH, 2 * dstH);
    li_advance(&it, mainBegin);
    ptrdiff_t tableSize = o->tY * 2;
    ptrdiff_t iTable = mainBegin % o->tY * 2;
    for (ptrdiff_t dstY = mainBegin; dstY < mainEnd; ++dstY) {
        ptrdiff_t srcOY = (ptrdiff_t)li_post_inc(&it);
        const uint16_t *coefs = &o->tabYu[iTable];
        iTable += 2;
        if (iTable == tableSize)
            iTable = 0;
        memset(work, 0, (size_t)srcW * sizeof(*work));
        for (ptrdiff_t i = 0; i < 2; ++i) {
            uint16_t coef = coefs[i];
            ptrdiff_t srcY = clamp_pd(0, srcH - 1, srcOY + i); /* see ln_resize_x note */
            for (ptrdiff_t x = 0; x < srcW; ++x)
                work[x] = (uint16_t)(work[x] + src[x + srcSt * srcY] * coef);
        }
        ln_resize_x(o, work, &dst[dstSt * dstY]);
    }
    for (ptrdiff_t dstY = mainEnd; dstY < dstH; ++dstY) {
        for (ptrdiff_t x = 0; x < srcW; ++x)
            work[x] = (uint16_t)(src[x + srcSt * (srcH - 1)] * 256);
        ln_resize_x(o, work, &dst[dstSt * dstY]);
    }
}

/* ------------------------------------------------------------------ public */

void iqo_oracle_resize(iqo_oracle *o, size_t srcSt, const uint8_t *src, size_t dstSt, uint8_t *dst)
{
    if (!o)
        return;
    if (o->method == IQO_ORACLE_LANCZOS)
        lz_resize(o, srcSt, src, dstSt, dst);
    else if (o->method == IQO_ORACLE_AREA)
        ar_resize(o, srcSt, src, dstSt, dst);
    else
        ln_resize(o, srcSt, src, dstSt, dst);
}

int iqo_oracle_run(int method, unsigned degree, size_t srcW, size_t srcH, size_t dstW, size_t dstH,
                   size_t pxScale, size_t srcSt, const uint8_t *src, size_t dstSt, uint8_t *dst)
{
    iqo_oracle *o = iqo_oracle_new(method, degree, srcW, srcH, dstW, dstH, pxScale);
    if (!o)
        return -1;
    iqo_oracle_resize(o, srcSt, src, dstSt, dst);
    iqo_oracle_free(o);
    return 0;
}

typedef struct {
    int method;
    unsigned degree;
    size_t srcW, srcH, dstW, dstH, pxScale;
    size_t f0, f1, srcSt, srcFrameSt, dstSt, dstFrameSt;
    const uint8_t *src;
    uint8_t *dst;
} batch_job;

static void *batch_worker(void *arg)
{
    batch_job *j = (batch_job *)arg;
    iqo_oracle *o = iqo_oracle_new(j->method, j->degree, j->srcW, j->srcH, j->dstW, j->dstH, j->pxScale);
    if (!o)
        return NULL;
    for (size_t f = j->f0; f < j->f1; ++f)
        iqo_oracle_resize(o, j->srcSt, j->src + f * j->srcFrameSt, j->dstSt, j->dst + f * j->dstFrameSt);
    iqo_oracle_free(o);
    return NULL;
}

double iqo_oracle_run_batch(int method, unsigned degree, size_t srcW, size_t srcH, size_t dstW,
                            size_t dstH, size_t pxScale, size_t nFrames, size_t srcSt,
                            size_t srcFrameSt, const uint8_t *src, size_t dstSt, size_t dstFrameSt,
                            uint8_t *dst, int nThreads)
{
    if (nThreads < 1)
        nThreads = 1;
    if ((size_t)nThreads > nFrames)
        nThreads = (int)(nFrames ? nFrames : 1);
    pthread_t *th = (pthread_t *)calloc((size_t)nThreads, sizeof(pthread_t));
    batch_job *jobs = (batch_job *)calloc((size_t)nThreads, sizeof(batch_job));
    if (!th || !jobs) {
        free(th);
        free(jobs);
        return -1.0;
    }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < nThreads; ++i) {
        batch_job *j = &jobs[i];
        j->method = method;
        j->degree = degree;
        j->srcW = srcW;
        j->srcH = srcH;
        j->dstW = dstW;
        j->dstH = dstH;
        j->pxScale = pxScale;
        j->f0 = nFrames * (size_t)i / (size_t)nThreads;
        j->f1 = nFrames * (size_t)(i + 1) / (size_t)nThreads;
        j->srcSt = srcSt;
        j->srcFrameSt = srcFrameSt;
        j->dstSt = dstSt;
        j->dstFrameSt = dstFrameSt;
        j->src = src;
        j->dst = dst;
        pthread_create(&th[i], NULL, batch_worker, j);
    }
    for (int i = 0; i < nThreads; ++i)
        pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th);
    free(jobs);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ------------------------------------------------------------------ generators / hashing */

void iqo_gen_g1(uint8_t *p, size_t w, size_t h, size_t st)
{
    for (size_t y = 0; y < h; ++y)
        for (size_t x = 0; x < w; ++x)
            p[y * st + x] = (uint8_t)(((uint32_t)(y * w + x) * 2654435761u) >> 24);
}

/* std::mt19937(seed) + std::uniform_int_distribution<int>(0,255) as the benchmark draws its planes
 * (benchmark/benchmark.cpp:51-59), with the mapping of this image's libstdc++ (GCC >= 11): for a
 * full-range 32-bit engine, uniform_int_distribution uses Lemire's nearly-divisionless method,
 * product = r * 256 (64-bit), reject while low32(product) < (2^32 - 256) % 256 (= 0: never),
 * result = product >> 32 = r >> 24.  (The older divide-and-reject mapping, r / (0xffffffff/256),
 * differs from the 75489th draw on.) */
void iqo_gen_mt19937(uint8_t *p, size_t n, uint32_t seed)
{
    uint32_t mt[624];
    int idx = 624;
    mt[0] = seed;
    for (int i = 1; i < 624; ++i)
        mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    const uint64_t range = 256u;
    const uint32_t threshold = (uint32_t)(0u - (uint32_t)range) % (uint32_t)range;
    for (size_t k = 0; k < n; ++k) {
        uint64_t prod;
        do {
            if (idx >= 624) {
                for (int i = 0; i < 624; ++i) {
                    uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
                    mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
                }
                idx = 0;
            }
            uint32_t y = mt[idx++];
            y ^= y >> 11;
            y ^= (y << 7) & 0x9d2c5680u;
            y ^= (y << 15) & 0xefc60000u;
            y ^= y >> 18;
            prod = (uint64_t)y * range;
        } while ((uint32_t)prod < threshold);
        p[k] = (uint8_t)(prod >> 32);
    }
}

void iqo_gen_splitmix(uint8_t *p, size_t n, uint64_t seed)
{
    for (size_t i = 0; i < n; ++i) {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        p[i] = (uint8_t)(z >> 56);
    }
}

uint64_t iqo_fnv1a64(const uint8_t *p, size_t w, size_t h, size_t st)
{
    uint64_t hsh = 0xcbf29ce484222325ull;
    for (size_t y = 0; y < h; ++y)
        for (size_t x = 0; x < w; ++x) {
            hsh ^= p[y * st + x];
            hsh *= 0x100000001b3ull;
        }
    return hsh;
}
