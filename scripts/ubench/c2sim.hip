// C2's schedule with synthetic arithmetic (Lanczos-3 3840x2160 -> 1920x1080, 128 frames): the
// block-shared streamer's structure (lanczos_symb_kernel: 4 waves = 4 strips of a row band, one
// shared LDS ring of K slots of 2 source rows filled by 1-KiB LDS-DMA chunks, one s_barrier per
// output row, look-ahead LDS read of the next slot, one 8-B store per lane and row) with the
// real kernel's ~150 VALU instructions per row replaced by NV packed MACs on the loaded data.
// What is varied: NV, the ring depth K, the ring form (shared + barrier, or private per wave),
// cache policies, band count and order, bursts of DMA issue, and per-wave skew.  GB/s is
// ALGORITHMIC bytes (1.327 GB per launch) / time; fresh buffers (two batches alternate).
//   hipcc -O3 --offload-arch=gfx950 c2sim.hip -o c2sim && ./c2sim [set]
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
constexpr int PITCH = 3872;  // LDS ring row pitch of the real kernel (16-B pad + 3840 + pad)

struct P {
    int F, B, R;      // frames, bands per frame, output rows per band
    int ntl, nts;     // nontemporal source loads / output stores
    int persistent;   // 0: one (frame, band) item per workgroup (XCD-spread order); else grid size
    int alt;          // odd bands walk bottom-up
    int noload, nost; // drop loads / stores (out-of-range offsets: the instructions still issue)
    int order;        // persistent only: 0 items strided by the grid, 4 per-XCD frame sweep (c2mem order 4),
                      // 5 dynamic queue (atomic counter o[1]): frames 0..F-F2-1 in B bands of R rows, the
                      // last F2 frames in B2 bands (short bands last: no tail)
    int F2, B2;
};

__device__ __forceinline__ unsigned xcd_spread(unsigned L, unsigned n)
{
    const unsigned xcd = L & 7u, idx = L >> 3, q = n >> 3, r = n & 7u;
    return xcd < r ? xcd * (q + 1u) + idx : r * (q + 1u) + (xcd - r) * q + idx;
}

template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F &&f, std::integer_sequence<int, I...>) { (f(std::integral_constant<int, I>{}), ...); }
template <int N, typename F>
__device__ __forceinline__ void sfor(F &&f) { sfor_impl(f, std::make_integer_sequence<int, N>{}); }

__device__ __forceinline__ void dma(uint32_t lds, int voff, __amdgpu_buffer_rsrc_t rsrc, int soff, int nt)
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
__device__ __forceinline__ uint32_t pk_mad(uint32_t a, uint32_t c, uint32_t acc)
{
    uint32_t d;
    asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(c), "v"(acc));
    return d;
}

// K: ring slots (2 rows each); NV: packed MACs per row (8 independent chains); SHARED: one ring
// per workgroup + barrier (else a private ring per wave, no barrier: each wave reads only the
// chunk it DMA'd); LA: look-ahead LDS read (wait for slot i+1, as the real kernel)
template <int K, int NV, bool SHARED, bool LA>
__global__ __launch_bounds__(256) void c2sim(const uint8_t *src, uint8_t *dst, P p, unsigned *o, unsigned coef)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nItems = p.F * p.B;
    const int G = p.persistent ? p.persistent : nItems;
    const unsigned blk = p.persistent ? blockIdx.x : xcd_spread(blockIdx.x, nItems);
    const uint32_t ldsBase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t *)lds;
    uint32_t acc[8] = {0u, 1u, 2u, 3u, 4u, 5u, 6u, 7u};
    // the real kernel's per-wave store offset: lanes 1..60 of wave w write 8 B at 480 w + 8 (l - 1)
    const int stoff = (lane >= 1 && lane <= 60 && !p.nost) ? 480 * wave + 8 * (lane - 1) : OOR;
    // order 4: XCD x sweeps frames x, x + 8, ...; its G/8 workgroups take (frame, band) items
    // frame-major, j, j + G/8, ... (a compact window of frames per XCD)
    const int g4 = G >> 3, x4 = (int)(blockIdx.x & 7);
    int i4 = (int)(blockIdx.x >> 3);
    __shared__ int qsh;
    const int nLong = (p.F - p.F2) * p.B, R2 = (DH + p.B2 - 1) / max(p.B2, 1);
    for (int it = (int)blk; p.order == 4 ? (x4 + 8 * (i4 / p.B)) < p.F : it < nItems; it += G) {
        int f = it / p.B, b = it % p.B;
        int R = p.R;
        if (p.order == 4) {
            f = x4 + 8 * (i4 / p.B);
            b = i4 % p.B;
            i4 += g4;
        } else if (p.order == 5) {
            if (tid == 0)
                qsh = (int)__hip_atomic_fetch_add(o + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            const int q = qsh;
            __syncthreads();
            if (q < nLong) {
                f = q / p.B;
                b = q - f * p.B;
            } else if (q - nLong < p.F2 * p.B2) {
                const int q2 = q - nLong;
                f = p.F - p.F2 + q2 / p.B2;
                b = q2 % p.B2;
                R = R2;
            } else {
                break;
            }
            it = -G;  // the loop continues until the queue runs dry
        }
        const int y0 = b * R, y1 = min(y0 + R, DH);
        if (y0 >= y1) continue;
        const int dir = (p.alt && (b & 1)) ? -1 : 1;
        const int rFirst = 2 * y0 - 4, rLast = 2 * (y1 - 1) + 5, n = y1 - y0;
        const __amdgpu_buffer_rsrc_t sR = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src + f * SF), 0, (int)SF, 0x00020000);
        const __amdgpu_buffer_rsrc_t dR = __builtin_amdgcn_make_buffer_rsrc(dst + f * DF, 0, (int)DF, 0x00020000);
        auto soff = [&](int r) { return (r >= 0 && r < SH && !p.noload) ? r * SW : OOR; };
        auto rowAt = [&](int i, int t) { return dir > 0 ? rFirst + 2 * i + t : rLast - 2 * i - t; };
        // chunk w of a row = source bytes [1024 w, 1024 w + 1024), the last one 768 B
        const int chunkCol = 1024 * wave + 16 * lane;
        const int voffD = chunkCol < SW ? chunkCol : OOR;
        // prologue window loads: lane l of wave w reads the 16 B of its strip (as the real kernel)
        const int pcol = 960 * wave - 16 + 16 * lane;
        const int voffP = (lane <= 61 && pcol >= 0 && pcol < SW) ? pcol : OOR;
        {
            u32x4 w[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) w[t] = __builtin_amdgcn_raw_buffer_load_b128(sR, voffP, soff(rowAt(0, t)), 0);
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] ^= w[t].x ^ w[t].w;
        }
        // ring: SHARED: slot s rows at s*2*PITCH (+PITCH); private: wave w's 2-KiB slots
        auto slotAddr = [&](int s) -> uint32_t {
            return SHARED ? ldsBase + (uint32_t)(s * 2 * PITCH) : ldsBase + (uint32_t)(wave * K * 2048 + s * 2048);
        };
        auto issue = [&](int i, int s) {
            const uint32_t a = SHARED ? slotAddr(s) + 16 + 1024 * wave : slotAddr(s);
            const bool in = i < n;
            dma(a, voffD, sR, soff(in ? rowAt(i, 8) : -1), p.ntl);
            dma(a + (SHARED ? PITCH : 1024), voffD, sR, soff(in ? rowAt(i, 9) : -1), p.ntl);
        };
        // the lane's 16-B read position: shared ring: the strip's columns (halo lanes included);
        // private ring: its own chunk bytes
        const int rcol = SHARED ? (lane <= 61 ? pcol + 16 : 0) : lane * 16;
        auto rd = [&](int s, uint4 &a0, uint4 &a1) {
            const uint8_t *q = lds + (slotAddr(s) - ldsBase) + rcol;
            a0 = *(const uint4 *)q;
            a1 = *(const uint4 *)(q + (SHARED ? PITCH : 1024));
        };
        constexpr int WAIT = 1 + (K - 2) * 3, WAITLA = LA ? 1 + (K - 3) * 3 : 1 + (K - 2) * 3;
#pragma unroll
        for (int j = 0; j < K - 1; ++j) {
            issue(j, j);
            __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, dR, OOR, 0, 0);
        }
        uint4 n0 = make_uint4(0, 0, 0, 0), n1 = n0;
        if (LA) {
            waitvm<WAIT>();
            if (SHARED) __builtin_amdgcn_s_barrier();
            rd(0, n0, n1);
        }
        for (int base = 0; base < n; base += K) {
            sfor<K>([&](auto uc) {
                constexpr int v = decltype(uc)::value;
                const int i = base + v;
                if (i >= n) return;
                const int yy = dir > 0 ? y0 + i : y1 - 1 - i;
                waitvm<WAITLA>();
                asm volatile("" ::: "memory");
                if (SHARED) __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                uint4 m0, m1;
                if (LA) rd((v + 1) % K, m0, m1);
                else rd(v, m0, m1);
                issue(i + K - 1, (v + K - 1) % K);
                uint4 c0 = LA ? n0 : m0, c1 = LA ? n1 : m1;
                if (LA) { n0 = m0; n1 = m1; }
                const uint32_t x[4] = {c0.x ^ c1.x, c0.y ^ c1.y, c0.z ^ c1.z, c0.w ^ c1.w};
#pragma unroll
                for (int r = 0; r < NV / 8; ++r)
#pragma unroll
                    for (int c = 0; c < 8; ++c) acc[c] = pk_mad(x[(c + r) & 3], coef, acc[c]);
                const u32x2 ov{acc[0] ^ acc[1] ^ acc[2] ^ acc[3], acc[4] ^ acc[5] ^ acc[6] ^ acc[7]};
                if (p.nts)
                    __builtin_amdgcn_raw_buffer_store_b64(ov, dR, stoff, yy * DW, 2);
                else
                    __builtin_amdgcn_raw_buffer_store_b64(ov, dR, stoff, yy * DW, 0);
            });
        }
        waitvm<0>();
        if (SHARED) __builtin_amdgcn_s_barrier();
    }
    if ((acc[0] ^ acc[3] ^ acc[7]) == 0x12345u) o[0] = acc[1];
}

// Persistent workgroups with ONE continuous DMA stream across their bands: item k of workgroup w
// (band of R output rows) is R + 4 ring steps, the first 4 only filling the window (walk rows
// 0..7), so the next band's first rows are in flight while the current band finishes (no
// per-band prologue stall).  Items frame-major; at round k the grid takes items [kG, (k+1)G),
// XCD x the G/8 consecutive items from kG + xG/8 (neighbouring bands on one XCD).
template <int K, int NV, int NVF>
__global__ __launch_bounds__(256) void c2cont(const uint8_t *src, uint8_t *dst, P p, unsigned *o, unsigned coef)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int G = p.persistent, R = p.R, S = R + 4;
    const int nItems = p.F * p.B;
    const int w = (int)blockIdx.x;
    const int first = (w & 7) * (G >> 3) + (w >> 3);
    const int nMine = first < nItems ? (nItems - 1 - first) / G + 1 : 0;
    const int nSteps = nMine * S;
    const uint32_t ldsBase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t *)lds;
    uint32_t acc[8] = {0u, 1u, 2u, 3u, 4u, 5u, 6u, 7u};
    const int stoffL = (lane >= 1 && lane <= 60 && !p.nost) ? 480 * wave + 8 * (lane - 1) : OOR;
    const int chunkCol = 1024 * wave + 16 * lane;
    const int voffD = chunkCol < SW ? chunkCol : OOR;
    const int pcol = 960 * wave - 16 + 16 * lane;
    const int rcol = lane <= 61 ? pcol + 16 : 0;
    // per-item state, advanced incrementally (one division per item): DMA side and compute side
    struct Item {
        int64_t srcBase, dstBase;
        int r, dir, y, n;  // next walk row (DMA) / first output row and its step (compute)
    };
    auto item = [&](int k) {
        Item it;
        const int idx = first + k * G, f = idx / p.B, b = idx - f * p.B;
        const int y0 = b * R, y1 = min(y0 + R, DH);
        it.dir = (p.alt && (b & 1)) ? -1 : 1;
        it.r = it.dir > 0 ? 2 * y0 - 4 : 2 * (y1 - 1) + 5;
        it.y = it.dir > 0 ? y0 : y1 - 1;
        it.n = y1 - y0;
        it.srcBase = int64_t(f) * SF;
        it.dstBase = int64_t(f) * DF;
        return it;
    };
    int dk = 0, dp = 0;  // DMA side: item, pair within the item
    Item di = item(0);
    auto issue = [&](int sl) {
        const uint32_t a = ldsBase + (uint32_t)(sl * 2 * PITCH) + 16 + 1024 * wave;
        const bool live = dk < nMine && dp < di.n + 4 && !p.noload;
        const int r0 = di.r, r1 = di.r + di.dir;
        const int so0 = live && r0 >= 0 && r0 < SH ? r0 * SW : OOR, so1 = live && r1 >= 0 && r1 < SH ? r1 * SW : OOR;
        const __amdgpu_buffer_rsrc_t sR = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src + di.srcBase), 0, (int)SF, 0x00020000);
        dma(a, voffD, sR, so0, p.ntl);
        dma(a + PITCH, voffD, sR, so1, p.ntl);
        di.r += 2 * di.dir;
        if (++dp == S) {
            dp = 0;
            ++dk;
            if (dk < nMine) di = item(dk);
        }
    };
    auto rd = [&](int sl, uint4 &a0, uint4 &a1) {
        const uint8_t *q = lds + sl * 2 * PITCH + rcol;
        a0 = *(const uint4 *)q;
        a1 = *(const uint4 *)(q + PITCH);
    };
    constexpr int WAIT = 1 + (K - 2) * 3, WAITLA = 1 + (K - 3) * 3;
    const __amdgpu_buffer_rsrc_t dummy = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 16, 0x00020000);
#pragma unroll
    for (int j = 0; j < K - 1; ++j) {
        issue(j);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, 0u}, dummy, OOR, 0, 0);
    }
    uint4 n0, n1;
    waitvm<WAIT>();
    __builtin_amdgcn_s_barrier();
    rd(0, n0, n1);
    int ck = 0, cp = 0;  // compute side
    Item ci = item(0);
    for (int base = 0; base < nSteps; base += K) {
        sfor<K>([&](auto uc) {
            constexpr int v = decltype(uc)::value;
            const int q = base + v;
            if (q >= nSteps) return;
            waitvm<WAITLA>();
            asm volatile("" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            uint4 m0, m1;
            rd((v + 1) % K, m0, m1);
            issue((v + K - 1) % K);
            const uint32_t x[4] = {n0.x ^ n1.x, n0.y ^ n1.y, n0.z ^ n1.z, n0.w ^ n1.w};
            n0 = m0;
            n1 = m1;
            int stoff = OOR, rowOff = 0;
            if (cp >= 4) {
#pragma unroll
                for (int r = 0; r < NV / 8; ++r)
#pragma unroll
                    for (int c = 0; c < 8; ++c) acc[c] = pk_mad(x[(c + r) & 3], coef, acc[c]);
                if (cp - 4 < ci.n) {
                    stoff = stoffL;
                    rowOff = ci.y * DW;
                    ci.y += ci.dir;
                }
            } else {
#pragma unroll
                for (int r = 0; r < NVF / 8; ++r)
#pragma unroll
                    for (int c = 0; c < 8; ++c) acc[c] = pk_mad(x[(c + r) & 3], coef, acc[c]);
            }
            const __amdgpu_buffer_rsrc_t dR = __builtin_amdgcn_make_buffer_rsrc(dst + ci.dstBase, 0, (int)DF, 0x00020000);
            const u32x2 ov{acc[0] ^ acc[1] ^ acc[2] ^ acc[3], acc[4] ^ acc[5] ^ acc[6] ^ acc[7]};
            if (p.nts)
                __builtin_amdgcn_raw_buffer_store_b64(ov, dR, stoff, rowOff, 2);
            else
                __builtin_amdgcn_raw_buffer_store_b64(ov, dR, stoff, rowOff, 0);
            if (++cp == S) {
                cp = 0;
                ++ck;
                if (ck < nMine) ci = item(ck);
            }
        });
    }
    waitvm<0>();
    __builtin_amdgcn_s_barrier();
    if ((acc[0] ^ acc[3] ^ acc[7]) == 0x12345u) o[0] = acc[1];
}

int main(int argc, char **argv)
{
    const int F = 128;
    uint8_t *s[2], *d[2];
    unsigned *o;
    for (int i = 0; i < 2; ++i)
        if (hipMalloc(&s[i], SF * F) || hipMalloc(&d[i], DF * F)) return 1;
    if (hipMalloc(&o, 8)) return 1;
    for (int i = 0; i < 2; ++i) { (void)hipMemset(s[i], 1, SF * F); (void)hipMemset(d[i], 2, DF * F); }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double bytes = double(SF + DF) * F;
    auto t = [&](auto kern, int K, bool shared, P p, int perCU, const char *tag) {
        const int need = shared ? K * 2 * PITCH + 512 : 4 * K * 2048;
        const int ldsB = perCU ? 163840 / perCU - 64 : need;
        if (ldsB < need) { printf("skip %s K%d %d/CU\n", tag, K, perCU); return; }
        (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, ldsB);
        const int grid = p.persistent ? p.persistent : p.F * p.B;
        for (int w = 0; w < 3; ++w) {
            (void)hipMemsetAsync(o, 0, 8, 0);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), ldsB, 0, s[w & 1], d[w & 1], p, o, 0x00050003u);
        }
        (void)hipEventRecord(e0);
        for (int r = 0; r < 10; ++r) {
            (void)hipMemsetAsync(o, 0, 8, 0);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), ldsB, 0, s[r & 1], d[r & 1], p, o, 0x00050003u);
        }
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("K%d %-6s B%4d R%3d pers%5d ntl%d nts%d noload%d nost%d lds%6d  %.4f ms  %7.1f GB/s  %s\n", K, shared ? "shared" : "priv",
               p.B, p.R, p.persistent, p.ntl, p.nts, p.noload, p.nost, ldsB, ms / 10, bytes * 10 / (ms * 1e-3) / 1e9, tag);
        fflush(stdout);
    };
    auto mk = [&](int B, int pers = 0, int ntl = 0, int nts = 0, int noload = 0, int nost = 0, int order = 0) {
        return P{F, B, (DH + B - 1) / B, ntl, nts, pers, 1, noload, nost, order, 0, 0};
    };
    const char *set = argc > 1 ? argv[1] : "base";
    if (!strcmp(set, "base")) {
        // the real kernel's structure at its real VALU count, memory-only, compute-only, and the
        // in-between: does the synthetic model reproduce 0.28 / 0.253 / 0.16 ms (real: shipped /
        // memory-only pattern / compute-only)?
        for (int rep = 0; rep < 2; ++rep) {
            t(c2sim<5, 120, true, true>, 5, true, mk(48), 4, "real-like NV120");
            t(c2sim<5, 120, true, true>, 5, true, mk(48, 0, 0, 0, 0, 1), 4, "NV120 no stores");
            t(c2sim<5, 120, true, true>, 5, true, mk(48, 0, 0, 0, 1, 1), 4, "NV120 compute-only");
            t(c2sim<5, 0, true, true>, 5, true, mk(48), 4, "NV0 memory-only");
            t(c2sim<5, 0, true, true>, 5, true, mk(48, 0, 0, 0, 0, 1), 4, "NV0 no stores");
            t(c2sim<5, 64, true, true>, 5, true, mk(48), 4, "NV64");
            t(c2sim<5, 64, true, true>, 5, true, mk(48, 0, 0, 0, 1, 1), 4, "NV64 compute-only");
            t(c2sim<5, 120, true, true>, 5, true, mk(48, 0, 1, 1), 4, "NV120 ntl nts");
            t(c2sim<5, 0, true, true>, 5, true, mk(48, 0, 1, 1), 4, "NV0 ntl nts");
            t(c2sim<5, 120, false, true>, 5, false, mk(48), 4, "NV120 private ring (no barrier)");
            t(c2sim<5, 0, false, true>, 5, false, mk(48), 4, "NV0 private ring");
            t(c2sim<5, 120, true, false>, 5, true, mk(48), 4, "NV120 no look-ahead");
            t(c2sim<3, 120, true, true>, 3, true, mk(48), 4, "NV120 K3");
            t(c2sim<8, 120, true, true>, 8, true, mk(48), 2, "NV120 K8 2/CU");
            t(c2sim<10, 120, true, true>, 10, true, mk(48), 2, "NV120 K10 2/CU");
            t(c2sim<5, 120, true, true>, 5, true, mk(24), 4, "NV120 B24");
            t(c2sim<5, 120, true, true>, 5, true, mk(96), 4, "NV120 B96");
            t(c2sim<5, 120, true, true>, 5, true, mk(32, 1024), 4, "NV120 persistent 1024 B32");
        }
        return 0;
    }
    if (!strcmp(set, "dyn")) {
        // dynamic queue (persistent 1024 workgroups, atomic counter): long bands, the last F2 frames
        // in short bands, vs the grid at several band counts
        auto dq = [&](int B, int F2, int B2, int nts) { P q = mk(B, 1024, 0, nts, 0, 0, 5); q.F2 = F2; q.B2 = B2; return q; };
        for (int rep = 0; rep < 2; ++rep) {
            t(c2sim<5, 120, true, true>, 5, true, mk(48, 0, 0, 1), 4, "grid B48 NV120 nts");
            t(c2sim<5, 120, true, true>, 5, true, mk(135, 0, 0, 1), 4, "grid B135 NV120 nts");
            t(c2sim<5, 120, true, true>, 5, true, dq(24, 0, 0, 1), 4, "dyn B24 NV120 nts");
            t(c2sim<5, 120, true, true>, 5, true, dq(24, 8, 135, 1), 4, "dyn B24 + last 8 frames B135 NV120 nts");
            t(c2sim<5, 120, true, true>, 5, true, dq(48, 8, 135, 1), 4, "dyn B48 + last 8 frames B135 NV120 nts");
            t(c2sim<5, 120, true, true>, 5, true, dq(12, 8, 135, 1), 4, "dyn B12 + last 8 frames B135 NV120 nts");
            t(c2sim<5, 120, true, true>, 5, true, dq(24, 16, 135, 1), 4, "dyn B24 + last 16 frames B135 NV120 nts");
            t(c2sim<5, 120, true, true>, 5, true, dq(135, 0, 0, 1), 4, "dyn B135 NV120 nts");
            t(c2sim<5, 0, true, true>, 5, true, dq(24, 8, 135, 1), 4, "dyn B24 + last 8 B135 NV0 nts");
            t(c2sim<5, 120, true, true>, 5, true, dq(24, 8, 135, 0), 4, "dyn B24 + last 8 B135 NV120");
        }
        return 0;
    }
    if (!strcmp(set, "deep")) {
        // one or two workgroups per CU with a deep ring (the whole LDS): fewer, faster address
        // streams, latency hidden by the ring instead of by co-resident workgroups
        for (int rep = 0; rep < 2; ++rep) {
            for (int B : {36, 72, 135}) {
                t(c2cont<20, 120, 16>, 20, true, mk(B, 256, 0, 1), 1, "cont K20 1/CU NV120 nts");
                t(c2cont<20, 120, 16>, 20, true, mk(B, 256, 1, 1), 1, "cont K20 1/CU NV120 ntl nts");
                t(c2cont<20, 0, 0>, 20, true, mk(B, 256, 1, 1), 1, "cont K20 1/CU NV0 ntl nts");
                t(c2cont<20, 120, 16>, 20, true, mk(B, 256, 0, 1, 1, 1), 1, "cont K20 1/CU NV120 compute-only");
                t(c2cont<10, 120, 16>, 10, true, mk(B, 512, 0, 1), 2, "cont K10 2/CU NV120 nts");
                t(c2cont<10, 120, 16>, 10, true, mk(B, 512, 1, 1), 2, "cont K10 2/CU NV120 ntl nts");
            }
            t(c2cont<12, 120, 16>, 12, true, mk(72, 256, 1, 1), 1, "cont K12 1/CU NV120 ntl nts");
            t(c2sim<20, 120, true, true>, 20, true, mk(72, 0, 0, 1), 1, "grid K20 1/CU NV120 nts");
            t(c2sim<20, 120, true, true>, 20, true, mk(72, 256, 1, 1, 0, 0, 4), 1, "xcd-sweep K20 1/CU NV120 ntl nts");
            t(c2sim<5, 120, true, true>, 5, true, mk(135, 0, 0, 1), 4, "grid NV120 nts (reference)");
            t(c2sim<5, 0, true, true>, 5, true, mk(135, 0, 0, 1), 4, "grid NV0 nts");
        }
        return 0;
    }
    if (!strcmp(set, "cont")) {
        // continuous-stream persistent bands vs the grid with per-band prologues
        for (int rep = 0; rep < 2; ++rep) {
            for (int B : {72, 108, 135}) {
                t(c2sim<5, 120, true, true>, 5, true, mk(B, 0, 0, 1), 4, "grid NV120 nts");
                t(c2cont<5, 120, 16>, 5, true, mk(B, 1024, 0, 1), 4, "cont NV120 nts");
                t(c2cont<5, 120, 16>, 5, true, mk(B, 1024, 0, 0), 4, "cont NV120");
                t(c2cont<5, 0, 0>, 5, true, mk(B, 1024, 0, 1), 4, "cont NV0 nts");
                t(c2cont<5, 120, 16>, 5, true, mk(B, 1024, 0, 1, 1, 1), 4, "cont NV120 compute-only");
            }
            t(c2cont<5, 120, 16>, 5, true, mk(135, 1024, 1, 1), 4, "cont NV120 ntl nts");
            t(c2cont<8, 120, 16>, 8, true, mk(135, 512, 0, 1), 2, "cont K8 2/CU NV120 nts");
            t(c2cont<5, 120, 16>, 5, true, mk(135, 768, 0, 1), 3, "cont 3/CU NV120 nts");
        }
        return 0;
    }
    if (!strcmp(set, "nt")) {
        // cache policies x band counts x schedules, with and without the arithmetic
        for (int rep = 0; rep < 2; ++rep) {
            for (int B : {48, 96, 135}) {
                t(c2sim<5, 120, true, true>, 5, true, mk(B, 0, 0, 0), 4, "NV120");
                t(c2sim<5, 120, true, true>, 5, true, mk(B, 0, 1, 0), 4, "NV120 ntl");
                t(c2sim<5, 120, true, true>, 5, true, mk(B, 0, 0, 1), 4, "NV120 nts");
                t(c2sim<5, 120, true, true>, 5, true, mk(B, 0, 1, 1), 4, "NV120 ntl nts");
                t(c2sim<5, 0, true, true>, 5, true, mk(B, 0, 1, 1), 4, "NV0 ntl nts");
            }
            for (int G : {256, 512, 1024})
                for (int B : {24, 32, 48}) {
                    t(c2sim<5, 120, true, true>, 5, true, mk(B, G, 1, 1, 0, 0, 4), G / 256, "NV120 ntl nts xcd-sweep");
                    t(c2sim<5, 0, true, true>, 5, true, mk(B, G, 1, 1, 0, 0, 4), G / 256, "NV0 ntl nts xcd-sweep");
                }
            t(c2sim<10, 120, true, true>, 10, true, mk(32, 512, 1, 1, 0, 0, 4), 2, "NV120 K10 ntl nts xcd-sweep");
            t(c2sim<5, 120, true, true>, 5, true, mk(32, 1024, 0, 0, 0, 0, 4), 4, "NV120 xcd-sweep default policy");
        }
        return 0;
    }
    return 0;
}
