// probe.hip -- streaming read:write probe (measurement infrastructure, not the resize path).
//
// bench.py times it on the box beside a resize kernel with the same read:write byte mix (C4: Linear
// 2x, 1 byte read per 4 written; C2 / C3: 4 : 1 and 16 : 1) on the same rotated device buffers,
// so the kernel's roofline fraction can be read against what a plain streaming kernel of that mix
// sustains on the same box in the same run, not only against the 8 TB/s peak.
//
// Layout: wave w moves unit w: R KiB read at src + w R KiB (1 KiB per load instruction, 16 B per
// lane, lane-contiguous), W KiB written at dst + w W KiB.  The written values depend on the loaded
// ones, so no load can be dropped.  Stores are plain or nontemporal (the resize kernels use both).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int R, int W, bool NT>
__global__ __launch_bounds__(256) void stream_mix_kernel(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst,
                                                         unsigned units)
{
    const unsigned wave = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (wave >= units)
        return;
    const u32x4 *s = src + static_cast<size_t>(wave) * R * 64 + lane;
    u32x4 *d = dst + static_cast<size_t>(wave) * W * 64 + lane;
    u32x4 v[R];
#pragma unroll
    for (int k = 0; k < R; ++k)
        v[k] = s[k * 64];
    u32x4 acc = v[0];
#pragma unroll
    for (int k = 1; k < R; ++k)
        acc ^= v[k];
#pragma unroll
    for (int k = 0; k < W; ++k) {
        u32x4 o = acc;
        o.x += static_cast<unsigned>(k);
        if (NT)
            __builtin_nontemporal_store(o, d + k * 64);
        else
            d[k * 64] = o;
    }
}

template <int R, int W>
hipError_t launch(bool nt, const void *src, void *dst, size_t units, hipStream_t s)
{
    const dim3 grid(static_cast<unsigned>((units + 3) / 4)), block(256);
    const auto *sp = static_cast<const u32x4 *>(src);
    auto *dp = static_cast<u32x4 *>(dst);
    if (nt)
        hipLaunchKernelGGL((stream_mix_kernel<R, W, true>), grid, block, 0, s, sp, dp, static_cast<unsigned>(units));
    else
        hipLaunchKernelGGL((stream_mix_kernel<R, W, false>), grid, block, 0, s, sp, dp, static_cast<unsigned>(units));
    return hipGetLastError();
}

} // namespace

// Reads R KiB and writes W KiB per unit, `units` units: srcBytes >= units R KiB, dstBytes >= units
// W KiB (the caller sizes the buffers).  (R, W) in {(1, 4), (1, 1), (4, 1), (16, 1)}.  Returns 0, or
// -1 for an unsupported mix / bad arguments, -2 for a launch error.
extern "C" int iqo_probe_stream(int R, int W, int nt, const void *src, size_t srcBytes, void *dst, size_t dstBytes,
                                void *stream)
{
    if (!src || !dst || R <= 0 || W <= 0)
        return -1;
    const size_t units = std::min(srcBytes / (1024u * static_cast<size_t>(R)), dstBytes / (1024u * static_cast<size_t>(W)));
    if (units == 0 || units > 0xffffffffu)
        return -1;
    auto s = static_cast<hipStream_t>(stream);
    hipError_t e;
    if (R == 1 && W == 4)
        e = launch<1, 4>(nt != 0, src, dst, units, s);
    else if (R == 1 && W == 1)
        e = launch<1, 1>(nt != 0, src, dst, units, s);
    else if (R == 4 && W == 1)
        e = launch<4, 1>(nt != 0, src, dst, units, s);
    else if (R == 16 && W == 1)
        e = launch<16, 1>(nt != 0, src, dst, units, s);
    else
        return -1;
    return e == hipSuccess ? 0 : -2;
}
