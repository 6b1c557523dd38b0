// Store-bandwidth probe: which store form (plain / nt / buffer, 16 / 8 / 4 B per lane) and how many
// stores in flight reach the highest write rate on MI355X (results: profiles/r02/ubench_store.txt)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <int KIND, int UNR>
__global__ __launch_bounds__(256) void wr(unsigned char *p, size_t bytes)
{
    const size_t per = 256 * 16 * UNR;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7fffffff, 0x00020000);
    for (size_t base = blockIdx.x * per; base < bytes; base += (size_t)gridDim.x * per) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            size_t off = base + u * 256 * 16 + threadIdx.x * 16;
            u32x4 v = {(unsigned)off, 1u, 2u, 3u};
            if (KIND == 0) *(u32x4 *)(p + off) = v;
            if (KIND == 1) __builtin_nontemporal_store(v, (u32x4 *)(p + off));
            if (KIND == 2) __builtin_amdgcn_raw_buffer_store_b128(v, __builtin_amdgcn_make_buffer_rsrc(p + base, 0, 0x7fffffff, 0x00020000), u * 4096 + threadIdx.x * 16, 0, 2);
            if (KIND == 3) __builtin_amdgcn_raw_buffer_store_b128(v, __builtin_amdgcn_make_buffer_rsrc(p + base, 0, 0x7fffffff, 0x00020000), u * 4096 + threadIdx.x * 16, 0, 0);
            if (KIND == 4) {  // dwordx2 x2
                u32x2 a = {v.x, v.y}, b = {v.z, v.w};
                *(u32x2 *)(p + base + u * 4096 + threadIdx.x * 8) = a;
                *(u32x2 *)(p + base + u * 4096 + 2048 + threadIdx.x * 8) = b;
            }
            if (KIND == 5) {  // dword x4
                for (int k = 0; k < 4; ++k) *(unsigned *)(p + base + u * 4096 + k * 1024 + threadIdx.x * 4) = v.x + k;
            }
        }
    }
    (void)r;
}

int main()
{
    const size_t bytes = size_t(2) << 30;
    unsigned char *a;
    if (hipMalloc(&a, bytes)) return 1;
    (void)hipMemset(a, 1, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto t = [&](auto kern, int grid, const char *name) {
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a, bytes);
        (void)hipEventRecord(e0);
        for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a, bytes);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s grid %5d  %7.1f GB/s\n", name, grid, double(bytes) * 10 / (ms * 1e-3) / 1e9);
    };
    for (int grid : {1024, 2048, 4096}) {
        t(wr<0, 1>, grid, "plain x4 unr1");
        t(wr<0, 4>, grid, "plain x4 unr4");
        t(wr<1, 1>, grid, "nt x4 unr1");
        t(wr<1, 4>, grid, "nt x4 unr4");
        t(wr<2, 4>, grid, "buffer nt x4 unr4");
        t(wr<3, 4>, grid, "buffer plain x4 unr4");
        t(wr<4, 4>, grid, "plain x2 unr4");
        t(wr<5, 4>, grid, "plain x1 unr4");
    }
    return 0;
}
