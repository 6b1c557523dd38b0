// Does the HBM read:write ceiling depend on how many independent address streams are active?
// C2's block-shared streamer runs ~1024 workgroups at once, each walking its own row band (1024
// streams spread over the whole 1.3 GB batch); mix.hip's workgroups sweep one compact region
// together.  Same 4:1 byte mix, same bytes per launch, fresh buffers alternating per launch:
//   regions: block b streams its own contiguous slice (like C2's bands)
//   sweep:   all blocks advance through one compact window together (like mix.hip)
//   hipcc -O3 --offload-arch=gfx950 streams.hip -o streams && ./streams   (profiles/r02/ubench_streams.txt)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int R, int W, bool REGIONS>
__global__ __launch_bounds__(256) void mix(const unsigned char *src, unsigned char *dst, size_t iters, unsigned *o)
{
    unsigned acc = 0;
    const size_t rs = (size_t)gridDim.x * R * 4096, ws = (size_t)gridDim.x * W * 4096;
    for (size_t it = 0; it < iters; ++it) {
        const size_t ro = REGIONS ? (size_t)blockIdx.x * iters * R * 4096 + it * R * 4096 : it * rs + (size_t)blockIdx.x * R * 4096;
        const size_t wo = REGIONS ? (size_t)blockIdx.x * iters * W * 4096 + it * W * 4096 : it * ws + (size_t)blockIdx.x * W * 4096;
        const unsigned char *s = src + ro + threadIdx.x * 16;
        unsigned char *d = dst + wo + threadIdx.x * 16;
        u32x4 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = __builtin_nontemporal_load((const u32x4 *)(s + r * 4096));
#pragma unroll
        for (int r = 0; r < R; ++r) acc ^= v[r].x ^ v[r].w;
#pragma unroll
        for (int w = 0; w < W; ++w) *(u32x4 *)(d + w * 4096) = u32x4{acc, (unsigned)it, 2u, (unsigned)w};
    }
    if (acc == 0x12345u) o[0] = acc;
}

int main()
{
    const size_t bytes = size_t(3) << 30;
    unsigned char *a[2], *b[2];
    unsigned *o;
    for (int i = 0; i < 2; ++i)
        if (hipMalloc(&a[i], bytes) || hipMalloc(&b[i], bytes)) return 1;
    if (hipMalloc(&o, 4)) return 1;
    for (int i = 0; i < 2; ++i) { (void)hipMemset(a[i], 1, bytes); (void)hipMemset(b[i], 2, bytes); }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto t = [&](auto kern, int R, int W, int grid, const char *name) {
        const size_t per = (size_t)grid * (R + W) * 4096;
        const size_t iters = (size_t(1327104000) + per - 1) / per;
        for (int w = 0; w < 4; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a[w & 1], b[w & 1], iters, o);
        (void)hipEventRecord(e0);
        for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a[r & 1], b[r & 1], iters, o);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s grid %5d  %7.1f GB/s\n", name, grid, double(per) * iters * 10 / (ms * 1e-3) / 1e9);
    };
    for (int grid : {256, 512, 1024, 2048}) {
        t(mix<4, 1, false>, 4, 1, grid, "4:1 sweep (compact)");
        t(mix<4, 1, true>, 4, 1, grid, "4:1 regions (one per block)");
        t(mix<1, 4, false>, 1, 4, grid, "1:4 sweep (compact)");
        t(mix<1, 4, true>, 1, 4, grid, "1:4 regions (one per block)");
    }
    return 0;
}
