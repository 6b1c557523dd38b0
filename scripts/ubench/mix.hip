// Practical HBM ceiling for a read:write byte mix on one MI355X (C2 moves 4:1, C4 1:4, C3 17:1).
//   hipcc -O3 --offload-arch=gfx950 mix.hip -o mix && ./mix   (results: profiles/r02/ubench_mix.txt)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// each block streams R read units and W write units of 4 KiB (256 lanes x 16 B) per iteration
template <int R, int W>
__global__ __launch_bounds__(256) void mix(const unsigned char *src, unsigned char *dst, size_t iters, unsigned *o)
{
    unsigned acc = 0;
    const size_t rs = (size_t)gridDim.x * R * 4096, ws = (size_t)gridDim.x * W * 4096;
    for (size_t it = 0; it < iters; ++it) {
        const unsigned char *s = src + it * rs + (size_t)blockIdx.x * R * 4096 + threadIdx.x * 16;
        unsigned char *d = dst + it * ws + (size_t)blockIdx.x * W * 4096 + threadIdx.x * 16;
        u32x4 v[R > 0 ? R : 1];
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
    unsigned char *a, *b;
    unsigned *o;
    if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&o, 4)) return 1;
    (void)hipMemset(a, 1, bytes);
    (void)hipMemset(b, 2, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto t = [&](auto kern, int R, int W, int grid, const char *name) {
        // about 1.3 GB moved per launch (as one C2 launch of 128 frames)
        const size_t per = (size_t)grid * (R + W) * 4096;
        const size_t iters = (size_t(1327104000) + per - 1) / per;
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a, b, iters, o);
        (void)hipEventRecord(e0);
        for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a, b, iters, o);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-10s grid %5d  %7.1f GB/s\n", name, grid, double(per) * iters * 10 / (ms * 1e-3) / 1e9);
    };
    for (int grid : {1024, 2048, 4096}) {
        t(mix<4, 0>, 4, 0, grid, "read");
        t(mix<4, 1>, 4, 1, grid, "r4:w1");
        t(mix<1, 1>, 1, 1, grid, "r1:w1");
        t(mix<1, 4>, 1, 4, grid, "r1:w4");
        t(mix<0, 4>, 0, 4, grid, "write");
    }
    return 0;
}
