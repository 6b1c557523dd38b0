// C2's memory stream alone (Lanczos-3 3840x2160 -> 1920x1080, 128 frames): per output row two
// 3840-B source rows are read and one 1920-B output row is written; a workgroup walks a band of
// output rows after an 8-row window prologue.  No arithmetic.  What is varied is the ORDER in
// which the resident workgroups take (frame, band) items, the band length, the load form
// (registers or LDS-DMA), the prefetch depth, workgroups per CU, and persistence.  Fresh buffers:
// two batches alternate per launch.  GB/s is ALGORITHMIC bytes (1.327 GB per launch) / time.
//   hipcc -O3 --offload-arch=gfx950 c2mem.hip -o c2mem && ./c2mem    (profiles/r03/ubench_c2mem.txt)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <utility>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int SW = 3840, SH = 2160, DW = 1920, DH = 1080;
constexpr int64_t SF = int64_t(SW) * SH, DF = int64_t(DW) * DH;
constexpr int OOR = 0x7ff00000;

struct P {
    int F, B, R;      // frames, bands per frame, output rows per band
    int ntl, nts;     // nontemporal source loads / output stores
    int order;        // 0 frame-major, 1 frame-major + XCD ranges, 2 band-major, 3 row-interleaved bands per XCD
    int persistent;   // 0: one item per workgroup; else grid size, items strided
    int alt;          // odd bands walk bottom-up
    int nost;         // drop stores
};

__device__ __forceinline__ unsigned xcd_spread(unsigned L, unsigned n)
{
    const unsigned xcd = L & 7u, idx = L >> 3, q = n >> 3, r = n & 7u;
    return xcd < r ? xcd * (q + 1u) + idx : r * (q + 1u) + (xcd - r) * q + idx;
}

template <int N, typename F, int... I>
__device__ __forceinline__ void sfor(F &&f, std::integer_sequence<int, I...>) { (f(std::integral_constant<int, I>{}), ...); }
template <int N, typename F>
__device__ __forceinline__ void sfor(F &&f) { sfor<N>(f, std::make_integer_sequence<int, N>{}); }

__device__ __forceinline__ void dma(uint32_t lds, int voff, __amdgpu_buffer_rsrc_t rsrc, int soff, bool nt = false)
{
    uint32_t keep;
    if (nt)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, %4 offen nt lds\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "s"(lds), "v"(voff), "s"(rsrc), "s"(soff) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "s"(lds), "v"(voff), "s"(rsrc), "s"(soff) : "memory");
}
template <int N>
__device__ __forceinline__ void waitvm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int D, bool DMA, int SM = 0, int NTS = 0>
__global__ __launch_bounds__(256) void c2mem(const uint8_t *src, uint8_t *dst, P p, unsigned *o)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nItems = p.F * p.B;
    unsigned acc = 0;
    const int G = p.persistent ? p.persistent : nItems;
    const int start = p.persistent ? (int)xcd_spread(blockIdx.x, G) : (int)blockIdx.x;
    // order 4 (persistent only): XCD x sweeps the frames x, x + 8, ... in order; its items are
    // (frame, band) pairs frame-major, i -> (x + 8 (i / B), i % B), and its g4 workgroups take
    // i = j, j + g4, ... (a compact window per XCD: g4 / B frames in flight)
    const int g4 = G >> 3, j4 = (int)(blockIdx.x >> 3), x4 = (int)(blockIdx.x & 7);
    int i4 = j4;
    for (int it = start; p.order == 4 ? (x4 + 8 * (i4 / p.B)) < p.F : it < nItems; it += G) {
        int f, b;
        if (p.order == 4) {
            f = x4 + 8 * (i4 / p.B);
            b = i4 % p.B;
            i4 += g4;
        } else if (p.order == 0) { f = it / p.B; b = it % p.B; }
        else if (p.order == 1 || p.order == 3) { const int l = p.persistent ? it : (int)xcd_spread(it, nItems); f = l / p.B; b = l % p.B; }
        else { f = it % p.F; b = it / p.F; }
        int y0, y1;
        if (p.order == 3) { // band b of frame f = output rows b, b + B, ... in R-row chunks: rows [b*R, b*R+R)
            y0 = b * p.R; y1 = min(y0 + p.R, DH);
        } else { y0 = b * p.R; y1 = min(y0 + p.R, DH); }
        if (y0 >= y1) continue;
        const int dir = (p.alt && (b & 1)) ? -1 : 1;
        const int rFirst = 2 * y0 - 4, rLast = 2 * (y1 - 1) + 5, n = y1 - y0;
        const __amdgpu_buffer_rsrc_t sR = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src + f * SF), 0, (int)SF, 0x00020000);
        const __amdgpu_buffer_rsrc_t dR = __builtin_amdgcn_make_buffer_rsrc(dst + f * DF, 0, (int)DF, 0x00020000);
        auto soff = [&](int r) { return (r >= 0 && r < SH) ? r * SW : OOR; };
        auto rowAt = [&](int i, int t) { return dir > 0 ? rFirst + 2 * i + t : rLast - 2 * i - t; };
        const int voffR = tid < 240 ? tid * 16 : OOR;                  // register form: 256 threads x 16 B
        const int voffD = (wave * 1024 + lane * 16) < SW ? wave * 1024 + lane * 16 : OOR;  // DMA: wave w = chunk w
        const int stoff = (tid < 240 && !p.nost) ? tid * 8 : OOR;
        // prologue: 8 window rows
        {
            u32x4 w[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) w[t] = __builtin_amdgcn_raw_buffer_load_b128(sR, DMA ? voffD : voffR, soff(rowAt(0, t)), 0);
#pragma unroll
            for (int t = 0; t < 8; ++t) acc ^= w[t].x ^ w[t].w;
        }
        if constexpr (!DMA) {
            u32x4 ring[D][2];
#pragma unroll
            for (int j = 0; j < D; ++j) {
                ring[j][0] = __builtin_amdgcn_raw_buffer_load_b128(sR, voffR, soff(rowAt(j, 8)), 0);
                ring[j][1] = __builtin_amdgcn_raw_buffer_load_b128(sR, voffR, soff(rowAt(j, 9)), 0);
            }
            for (int base = 0; base < n; base += D) {
                sfor<D>([&](auto uc) {
                    constexpr int v = decltype(uc)::value;
                    const int i = base + v;
                    if (i >= n) return;
                    const int yy = dir > 0 ? y0 + i : y1 - 1 - i;
                    acc += ring[v][0].x ^ ring[v][1].y ^ ring[v][0].z ^ ring[v][1].w;
                    ring[v][0] = __builtin_amdgcn_raw_buffer_load_b128(sR, voffR, soff(i + D < n ? rowAt(i + D, 8) : -1), 0);
                    ring[v][1] = __builtin_amdgcn_raw_buffer_load_b128(sR, voffR, soff(i + D < n ? rowAt(i + D, 9) : -1), 0);
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{acc, (unsigned)i}, dR, stoff, yy * DW, 0);
                });
            }
        } else {
            const uint32_t ldsBase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t *)lds + wave * (D * 2048);
            const uint8_t *mine = lds + wave * (D * 2048) + lane * 16;
            // store modes (S store instructions per iteration, dropped ones out of range):
            //   0: one 8-B store per lane per row (the C2 kernel today)
            //   1: rows in pairs, one 16-B store per lane every second row (lanes 0-119 row a, 120-239 row b)
            //   2: rows in fours, two 16-B stores per lane every fourth row (7680 B)
            constexpr int S = SM == 2 ? 2 : 1;
            constexpr int aux = NTS ? 2 : 0;
            auto issue = [&](int i) {
                const uint32_t s = ldsBase + (i % D) * 2048;
                dma(s, voffD, sR, soff(i < n ? rowAt(i, 8) : -1), p.ntl);
                dma(s + 1024, voffD, sR, soff(i < n ? rowAt(i, 9) : -1), p.ntl);
            };
#pragma unroll
            for (int j = 0; j < D; ++j) {
                issue(j);
#pragma unroll
                for (int k = 0; k < S; ++k)
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, dR, OOR, 0, 0);
            }
            for (int i = 0; i < n; ++i) {
                const int yy = dir > 0 ? y0 + i : y1 - 1 - i;
                waitvm<S + (D - 1) * (2 + S)>();
                const uint8_t *q = mine + (i % D) * 2048;
                const uint4 a0 = *(const uint4 *)q, a1 = *(const uint4 *)(q + 1024);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                acc += a0.x ^ a1.y ^ a0.z ^ a1.w;
                issue(i + D);
                if constexpr (SM == 0) {
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{acc, (unsigned)i}, dR, stoff, yy * DW, aux);
                } else if constexpr (SM == 1) {
                    const int r0 = dir > 0 ? yy - 1 : yy;  // first row of the pair
                    const int off = ((i & 1) && tid < 240 && !p.nost) ? tid * 16 : OOR;
                    __builtin_amdgcn_raw_buffer_store_b128(u32x4{acc, (unsigned)i, 1u, 2u}, dR, off, r0 * DW, aux);
                } else {
                    const int r0 = dir > 0 ? yy - 3 : yy;  // first row of the four
                    const bool go = (i & 3) == 3 && !p.nost;
                    const int o0 = go ? tid * 16 : OOR, o1 = (go && tid < 224) ? 4096 + tid * 16 : OOR;
                    __builtin_amdgcn_raw_buffer_store_b128(u32x4{acc, (unsigned)i, 1u, 2u}, dR, o0, r0 * DW, aux);
                    __builtin_amdgcn_raw_buffer_store_b128(u32x4{acc, (unsigned)i, 3u, 4u}, dR, o1, r0 * DW, aux);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    if (acc == 0x12345u) o[0] = acc;
}

int main(int argc, char **argv)
{
    const int F = 128;
    uint8_t *s[2], *d[2];
    unsigned *o;
    for (int i = 0; i < 2; ++i)
        if (hipMalloc(&s[i], SF * F) || hipMalloc(&d[i], DF * F)) return 1;
    if (hipMalloc(&o, 4)) return 1;
    for (int i = 0; i < 2; ++i) { (void)hipMemset(s[i], 1, SF * F); (void)hipMemset(d[i], 2, DF * F); }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double bytes = double(SF + DF) * F;
    auto t = [&](auto kern, int D, bool dmaf, P p, int perCU, const char *tag) {
        int ldsB = 163840 / perCU - 512;
        if (dmaf && ldsB < 4 * D * 2048) { printf("skip\n"); return; }
        (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, ldsB);
        const int grid = p.persistent ? p.persistent : p.F * p.B;
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), ldsB, 0, s[w & 1], d[w & 1], p, o);
        (void)hipEventRecord(e0);
        for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), ldsB, 0, s[r & 1], d[r & 1], p, o);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-5s D%d B%4d R%3d order%d pers%5d alt%d nost%d %d/CU  %.4f ms  %7.1f GB/s  %s\n", dmaf ? "dma" : "reg", D, p.B, p.R,
               p.order, p.persistent, p.alt, p.nost, perCU, ms / 10, bytes * 10 / (ms * 1e-3) / 1e9, tag);
        fflush(stdout);
    };
    auto mk = [&](int B, int order, int pers, int alt, int nost = 0, int ntl = 0, int nts = 0) {
        return P{F, B, (DH + B - 1) / B, ntl, nts, order, pers, alt, nost};
    };
    const char *only = argc > 1 ? argv[1] : "";
    if (!strcmp(only, "v1")) {
        for (int B : {24, 48, 96})
            for (int order : {0, 1, 2}) {
                t(c2mem<4, true>, 4, true, mk(B, order, 0, 1), 4, "dma");
                t(c2mem<4, false>, 4, false, mk(B, order, 0, 1), 4, "reg");
            }
        return 0;
    }
    if (!strcmp(only, "v3")) {
        // nontemporal loads + stores (the best r2 policy) over grids, band counts, persistence, orders
        for (int rep = 0; rep < 2; ++rep) {
            if (!strcmp(argc > 2 ? argv[2] : "", "sweep")) goto sweep;
            for (int G : {256, 512, 768, 1024})
                for (int B : {24, 48, 72, 135}) {
                    char tag[64];
                    snprintf(tag, sizeof tag, "ntl nts persistent rep%d", rep);
                    t(c2mem<4, true, 0, 1>, 4, true, mk(B, 1, G, 1, 0, 1, 1), G / 256, tag);
                }
            for (int perCU : {1, 2, 4})
                for (int B : {48, 135}) {
                    char tag[64];
                    snprintf(tag, sizeof tag, "ntl nts one item per WG rep%d", rep);
                    t(c2mem<4, true, 0, 1>, 4, true, mk(B, 1, 0, 1, 0, 1, 1), perCU, tag);
                }
        sweep:
            for (int G : {256, 512, 1024})
                for (int B : {8, 16, 24, 32, 48, 64}) {
                    const int R = (DH + B - 1) / B;
                    t(c2mem<4, true, 0, 1>, 4, true, P{F, B, R, 1, 1, 4, G, 0, 0}, G / 256, "ntl nts xcd-sweep");
                    if (B == 32) {
                        t(c2mem<4, true, 0, 0>, 4, true, P{F, B, R, 0, 0, 4, G, 0, 0}, G / 256, "xcd-sweep");
                        t(c2mem<4, true, 0, 1>, 4, true, P{F, B, R, 0, 1, 4, G, 0, 0}, G / 256, "nts xcd-sweep");
                        t(c2mem<4, true, 0, 0>, 4, true, P{F, B, R, 1, 0, 4, G, 0, 0}, G / 256, "ntl xcd-sweep");
                        t(c2mem<4, true, 0, 1>, 4, true, P{F, B, R, 1, 1, 4, G, 1, 0}, G / 256, "ntl nts xcd-sweep alt");
                    }
                }
            t(c2mem<4, true, 0, 1>, 4, true, mk(48, 1, 256, 0, 0, 1, 1), 1, "ntl nts persistent no-alt");
            t(c2mem<2, true, 0, 1>, 2, true, mk(48, 1, 256, 1, 0, 1, 1), 1, "ntl nts persistent D2");
            t(c2mem<3, true, 0, 1>, 3, true, mk(48, 1, 256, 1, 0, 1, 1), 1, "ntl nts persistent D3");
            t(c2mem<6, true, 0, 1>, 6, true, mk(48, 1, 256, 1, 0, 1, 1), 1, "ntl nts persistent D6");
            t(c2mem<4, true, 0, 1>, 4, true, mk(48, 1, 256, 1, 0, 0, 1), 1, "nts persistent");
        }
        return 0;
    }
    // store forms and cache policies on the two best r1 schedules (persistent 256 B48; 4/CU B135)
    for (int sched = 0; sched < 2; ++sched) {
        const int B = sched ? 135 : 48, pers = sched ? 0 : 256, perCU = sched ? 4 : 1;
        for (int ntl : {0, 1}) {
            char tag[64];
            snprintf(tag, sizeof tag, "st8 ntl%d", ntl);
            t(c2mem<4, true, 0, 0>, 4, true, mk(B, 1, pers, 1, 0, ntl, 0), perCU, tag);
            snprintf(tag, sizeof tag, "st8 ntl%d nts", ntl);
            t(c2mem<4, true, 0, 1>, 4, true, mk(B, 1, pers, 1, 0, ntl, 1), perCU, tag);
            snprintf(tag, sizeof tag, "st16pair ntl%d", ntl);
            t(c2mem<4, true, 1, 0>, 4, true, mk(B, 1, pers, 1, 0, ntl, 0), perCU, tag);
            snprintf(tag, sizeof tag, "st16pair ntl%d nts", ntl);
            t(c2mem<4, true, 1, 1>, 4, true, mk(B, 1, pers, 1, 0, ntl, 1), perCU, tag);
            snprintf(tag, sizeof tag, "st16x4rows ntl%d", ntl);
            t(c2mem<4, true, 2, 0>, 4, true, mk(B, 1, pers, 1, 0, ntl, 0), perCU, tag);
            snprintf(tag, sizeof tag, "st16x4rows ntl%d nts", ntl);
            t(c2mem<4, true, 2, 1>, 4, true, mk(B, 1, pers, 1, 0, ntl, 1), perCU, tag);
        }
        t(c2mem<4, true, 0>, 4, true, mk(B, 1, pers, 1, 1, 0, 0), perCU, "no stores");
        t(c2mem<4, true, 0>, 4, true, mk(B, 1, pers, 1, 1, 1, 0), perCU, "no stores ntl");
    }
    // persistent grid sizes and band counts with 16-B paired stores
    // per-XCD frame sweeps with R-row items taken round-robin (compact window per XCD)
    for (int G : {256, 512, 1024})
        for (int R : {2, 4, 8, 16}) {
            const int B = (DH + R - 1) / R;
            t(c2mem<4, true, 1>, 4, true, P{F, B, R, 0, 0, 4, G, 0, 0}, G / 256, "st16pair xcd-sweep");
        }
    for (int G : {256, 512})
        for (int B : {24, 36, 48, 72}) {
            const int perCU = G / 256;
            t(c2mem<4, true, 1>, 4, true, mk(B, 1, G, 1), perCU, "st16pair persistent");
        }
    for (int B : {72, 96, 135, 180})
        for (int perCU : {2, 4})
            t(c2mem<4, true, 1>, 4, true, mk(B, 1, 0, 1), perCU, "st16pair");
    return 0;
}
