// kernels_dev.hpp -- device helpers shared by the kernel translation units (kernels.hip,
// kernels_ratio.hip): intrinsic wrappers, compile-time loops, barriers, launch helpers.
#pragma once
#include "kernels.hpp"

#include <algorithm>
#include <climits>
#include <cstdint>
#include <mutex>
#include <type_traits>
#include <unordered_map>
#include <utility>

namespace iqo_amd {
namespace {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));

// Timing-experiment flags (drop stores / loads / border work: WRONG output).  They exist only
// in the variant builds of scripts/build_variant.sh (-DIQO_VARIANT_DEBUG); the shipping library
// compiles every flag test away, so no public option can change its results.
#ifdef IQO_VARIANT_DEBUG
#define IQO_DBG(a) ((a).dbg)
#else
#define IQO_DBG(a) 0
#endif

// Workgroups are dealt round-robin over the 8 XCDs (flat id L runs on XCD L mod 8; placement is
// a speed property only, never relied on for correctness).  xcd_spread maps the flat id to a
// logical id so that XCD x receives the contiguous logical range [s_x, s_x + c_x), a bijection
// of [0, n) for any n.
__device__ __forceinline__ unsigned xcd_spread(unsigned L, unsigned n)
{
    const unsigned xcd = L & 7u, idx = L >> 3, q = n >> 3, r = n & 7u;
    return xcd < r ? xcd * (q + 1u) + idx : r * (q + 1u) + (xcd - r) * q + idx;
}

// Round 6: the XCD map of a frame-major grid.  Chunks of C consecutive logical blocks (about one
// frame's) are dealt round-robin over the XCDs -- XCD x resizes chunks x, x + 8, ... in order -- so
// a frame's neighbouring bands still share one XCD's L2 while the 8 XCDs work on 8 neighbouring
// chunks at a time, not on 8 ranges 1/8 of the batch apart as with xcd_spread (C2 x256: 0.479 ->
// 0.467 ms, x1024 1.871 -> 1.845, profiles/r06/xcd_chunks.txt).  A bijection of [0, n): the blocks
// past the last whole round of 8 chunks fall back to xcd_spread.  (Variant builds with
// -DIQO_XCD_SPREAD keep xcd_spread, for A/B.)
__device__ __forceinline__ unsigned xcd_chunks(unsigned L, unsigned C, unsigned n)
{
#ifdef IQO_XCD_SPREAD
    (void)C;
    return xcd_spread(L, n);
#else
    C = C ? C : 1u;
    const unsigned x = L & 7u, idx = L >> 3, full = n / (8u * C);
    if (idx < full * C) {
        const unsigned q = idx / C;
        return (8u * q + x) * C + (idx - q * C);
    }
    const unsigned base = 8u * full * C;
    return base + xcd_spread(L - base, n - base);
#endif
}

// 16-byte streaming load with the nontemporal hint (source pixels are read once per band; Area
// streamer: 9 % faster on C3 than the default policy.  The Linear 2x streamer keeps the default
// policy: 1 % faster on C4)
__device__ __forceinline__ uint4 load16_nt(const uint8_t *p)
{
    u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint32_t pk_mad(uint32_t a, uint32_t c, uint32_t acc)
{
    u16x2 r = __builtin_bit_cast(u16x2, a) * __builtin_bit_cast(u16x2, c) + __builtin_bit_cast(u16x2, acc);
    return __builtin_bit_cast(uint32_t, r);
}

__device__ __forceinline__ uint32_t pk_mul(uint32_t a, uint32_t c)
{
    u16x2 r = __builtin_bit_cast(u16x2, a) * __builtin_bit_cast(u16x2, c);
    return __builtin_bit_cast(uint32_t, r);
}

__device__ __forceinline__ int sdot2(uint32_t a, uint32_t c, int acc)
{
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(i16x2, a), __builtin_bit_cast(i16x2, c), acc, false);
}

// v_dot2_i32_i16 (VOP3P) with a uniform coefficient pair and the accumulator in a VGPR that stays
// live: the first dot of an output that starts from the rounding bias.  (The builtin is always
// selected as v_dot2c, which needs the accumulator in its destination: a v_mov of the bias per
// output, 72 per source row in the 3x kernel.)
__device__ __forceinline__ int sdot2_sv(uint32_t a, uint32_t c, int acc)
{
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(c), "v"(acc));
    return r;
}

// (and with per-lane coefficients)
__device__ __forceinline__ int sdot2_vv(uint32_t a, uint32_t c, int acc)
{
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(c), "v"(acc));
    return r;
}

__device__ __forceinline__ uint32_t udot2(uint32_t a, uint32_t c, uint32_t acc)
{
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, c), acc, false);
}

// bytes b0..b3 of v -> (b0,b1) and (b2,b3) as zero-extended u16 pairs
__device__ __forceinline__ void unpack4(uint32_t v, uint32_t &lo, uint32_t &hi)
{
    lo = __builtin_amdgcn_perm(0u, v, 0x0c010c00u);
    hi = __builtin_amdgcn_perm(0u, v, 0x0c030c02u);
}

__device__ __forceinline__ void unpack16(uint4 v, uint32_t (&w)[8])
{
    unpack4(v.x, w[0], w[1]);
    unpack4(v.y, w[2], w[3]);
    unpack4(v.z, w[4], w[5]);
    unpack4(v.w, w[6], w[7]);
}

// Exact C (truncating) int32 division n / d for |n| < 2^31, d != 0, |quotient| < 2^22:
// float reciprocal estimate of the magnitudes, then one-step integer correction.
__device__ __forceinline__ int exact_div(int n, int d)
{
    if (d == 0)
        return 0;  // the reference traps (SIGFPE); such shapes are outside parity
    uint32_t an = n < 0 ? 0u - static_cast<uint32_t>(n) : static_cast<uint32_t>(n);
    uint32_t ad = d < 0 ? 0u - static_cast<uint32_t>(d) : static_cast<uint32_t>(d);
    float r = __builtin_amdgcn_rcpf(static_cast<float>(ad));
    uint32_t q = static_cast<uint32_t>(static_cast<float>(an) * r);
    int64_t rem = static_cast<int64_t>(an) - static_cast<int64_t>(q) * ad;
    while (rem < 0) {
        --q;
        rem += ad;
    }
    while (rem >= static_cast<int64_t>(ad)) {
        ++q;
        rem -= ad;
    }
    return ((n ^ d) < 0) ? -static_cast<int>(q) : static_cast<int>(q);
}

__device__ __forceinline__ int clamp255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// A value the instruction combiner cannot see through.  Used on clamped bytes before packing:
// ROCm 7.2 otherwise folds (sat_u8(a >> n), sat_u8(b >> n)) into gfx950's v_ashr_pk_u8_i32 and
// then ORs further bytes into bits 16..31 of its result as if they were zero, which corrupted
// bytes 2-3 of every packed word on the GPU (caught by tests/test_gpu_parity.py).
__device__ __forceinline__ uint32_t opaque(uint32_t v)
{
    asm volatile("" : "+v"(v));
    return v;
}

// One wave's output row of 24-byte lane pieces (the 3x streamers: lanes 1 .. np own output bytes
// [24 (l - 1), 24 l) of the wave's span, nb = 24 np bytes from byte offset `base`) stored as
// contiguous 16-byte pieces: staged through the wave's 2 KB of LDS, then lane l stores pieces l and
// 64 + l.  Two dwordx4 stores at 24-byte strides split most pieces over two 64-byte segments and
// left both 3x streamers at a third of the 2x ones' bandwidth.  Wave-local LDS operations run in
// order, so no barrier separates one row's reads from the next row's writes.
template <int AUX>
__device__ __forceinline__ void store_row24(uint8_t *sb, const uint32_t (&o)[6], bool produce, int lane, int nb,
                                            __amdgpu_buffer_rsrc_t dstR, int base)
{
    constexpr int OOB = 0x7ff00000;
    if (produce) {
        u32x2 *p = reinterpret_cast<u32x2 *>(sb + 24 * (lane - 1));
        p[0] = u32x2{o[0], o[1]};
        p[1] = u32x2{o[2], o[3]};
        p[2] = u32x2{o[4], o[5]};
    }
    __builtin_amdgcn_wave_barrier();
    const u32x4 c0 = *reinterpret_cast<const u32x4 *>(sb + 16 * lane);
    const u32x4 c1 = *reinterpret_cast<const u32x4 *>(sb + 1024 + 16 * lane);
    const bool row = base < OOB;
    __builtin_amdgcn_raw_buffer_store_b128(c0, dstR, row && 16 * lane + 16 <= nb ? base + 16 * lane : OOB, 0, AUX);
    __builtin_amdgcn_raw_buffer_store_b128(c1, dstR, row && 1040 + 16 * lane <= nb ? base + 1024 + 16 * lane : OOB, 0,
                                           AUX);
    if (nb & 8) {  // odd np (uniform): the span's last 8 bytes are half a piece
        const int c = (nb - 8) >> 4;
        const u32x4 h = c < 64 ? c0 : c1;
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{h.x, h.y}, dstR, row && lane == (c & 63) ? base + nb - 8 : OOB, 0,
                                              AUX);
    }
}

// Compile-time loop: f(std::integral_constant<int, 0>) ... f(integral_constant<int, N-1>), so
// register-array indices derived from the induction variable are constants (no scratch).
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, I...>)
{
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f)
{
    static_for_impl(static_cast<F &&>(f), std::make_integer_sequence<int, N>{});
}

// Workgroup barrier that publishes this wave's LDS writes: an explicit lgkmcnt(0) before the
// s_barrier.  (round 5: the compiler drops the wait of __syncthreads' release fence for LDS, and on
// a loop back-edge no other wait preceded the barrier; the 2:1 ratio-Y kernel at 4K x128 then read
// a neighbouring wave's outer taps stale now and then -- 1 to 100 pixels off by one per launch,
// always at wave edges, profiles/r05/adj_race.txt)
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_s_waitcnt(0xc07f);  // vmcnt(63) expcnt(7) lgkmcnt(0)
    __syncthreads();
}

constexpr int cgcd(int a, int b) { return b == 0 ? a : cgcd(b, a % b); }

// (sat_u8(a >> 20), sat_u8(b >> 20)) into bits 0..15 of the result (bits 16..31 undefined) /
// into bits 16..31 of w (bits 0..15 kept).  gfx950 v_ashr_pk_u8_i32: src0 -> byte 0, src1 ->
// byte 1, the other half of the destination is preserved (probed on MI355X,
// scripts/ubench/pk_test.hip).
__device__ __forceinline__ uint32_t pack_lo(int a, int b)
{
    uint32_t w;
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 20" : "=v"(w) : "v"(a), "v"(b));
    return w;
}
__device__ __forceinline__ uint32_t pack_hi(uint32_t w, int a, int b)
{
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 20 op_sel:[0,0,0,1]" : "+v"(w) : "v"(a), "v"(b));
    return w;
}

// int16(n * 64 / deno) for both int16 halves of w (C truncation), deno via (m, s) of magic_y.
__device__ __forceinline__ uint32_t ydiv2(uint32_t w, uint32_t m, int s)
{
    const int lo = static_cast<int16_t>(w & 0xffffu), hi = static_cast<int16_t>(w >> 16);
    const uint32_t qlo = __umulhi(static_cast<uint32_t>(lo < 0 ? -lo : lo) << s, m);
    const uint32_t qhi = __umulhi(static_cast<uint32_t>(hi < 0 ? -hi : hi) << s, m);
    const uint32_t rlo = lo < 0 ? 0u - qlo : qlo, rhi = hi < 0 ? 0u - qhi : qhi;
    return __builtin_amdgcn_perm(rhi, rlo, 0x05040100u);  // (rlo.lo16, rhi.lo16)
}


template <int N>
__device__ __forceinline__ void wait_vmcnt()
{
    static_assert(N >= 0 && N < 64, "vmcnt field");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// (-lo, -hi) of two int16 halves
__device__ __forceinline__ uint32_t pk_neg16(uint32_t w)
{
    return ((0u - (w & 0xffffu)) & 0xffffu) | ((0u - (w >> 16)) << 16);
}

// Wave-uniform reads of read-only tables through the scalar cache (s_load).
__device__ __forceinline__ int sld(const void *p, int i)
{
    return ((const __attribute__((address_space(4))) int *)(p))[i];
}
__device__ __forceinline__ int4 sload(const int4 *p) { return make_int4(sld(p, 0), sld(p, 1), sld(p, 2), sld(p, 3)); }

// v_ashr_pk_u8_i32 with shift 23: (sat_u8(a >> 23), sat_u8(b >> 23)) into the low / high half
__device__ __forceinline__ uint32_t pack23_lo(uint32_t a, uint32_t b)
{
    uint32_t w;
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 23" : "=v"(w) : "v"(a), "v"(b));
    return w;
}
__device__ __forceinline__ uint32_t pack23_hi(uint32_t w, uint32_t a, uint32_t b)
{
    asm("v_ashr_pk_u8_i32 %0, %1, %2, 23 op_sel:[0,0,0,1]" : "+v"(w) : "v"(a), "v"(b));
    return w;
}


// ---- host-side launch helpers

// Waves of `kernel` (256-thread blocks) resident on the whole current device: occupancy x CUs.
// Host-side query, cached per kernel.
int resident_waves(const void *kernel, int block = 256, int ldsBytes = 0)
{
    static std::mutex mu;
    static std::unordered_map<const void *, int> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    // per device and geometry too
    const void *key = static_cast<const char *>(kernel) + dev + 16 * block + 65536 * ldsBytes;
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache.find(key);
        if (it != cache.end())
            return it->second;
    }
    int perCu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCu, kernel, block, static_cast<size_t>(ldsBytes)) !=
            hipSuccess ||
        perCu <= 0)
        perCu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    const int waves = perCu * (block / 64) * cus;
    std::lock_guard<std::mutex> g(mu);
    cache[key] = waves;
    return waves;
}

// Row bands per frame for a band-walking kernel: minimise the makespan in rows walked,
// (waves in flight rounds) x (rows per band + halo rows re-read at every band start), so that
// the grid fills whole rounds of the resident waves instead of leaving a straggler round.
[[maybe_unused]] int choose_bands(int rows, int frames, int wavesPerRow, int resident, int halo)
{
    int best = 1;
    int64_t bestCost = INT64_MAX;
    for (int b = 1; b <= std::min(rows, 512); ++b) {
        const int rpb = (rows + b - 1) / b;
        const int bb = (rows + rpb - 1) / rpb;
        if (bb != b)
            continue;
        const int64_t waves = static_cast<int64_t>(frames) * wavesPerRow * bb;
        const int64_t rounds = (waves + resident - 1) / resident;
        const int64_t cost = rounds * (rpb + halo);
        if (cost < bestCost) {
            bestCost = cost;
            best = bb;
        }
    }
    return best;
}


} // namespace
} // namespace iqo_amd
