// Microbenchmark: achievable HBM bandwidth on one MI355X for the access patterns of the resize
// kernels -- streaming 16-B-per-lane reads, writes (plain / nontemporal) and a copy -- so the
// roofline fractions in bench.py can be read against what the chip actually sustains.
//   hipcc -O3 --offload-arch=gfx950 bw.hip -o bw && ./bw
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void rd(const u32x4 *p, size_t n, unsigned *out)
{
    unsigned acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256) {
        u32x4 v = NT ? __builtin_nontemporal_load(p + i) : p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u)
        out[0] = acc;  // practically never: keeps the loads alive
}

template <bool NT>
__global__ __launch_bounds__(256) void wr(u32x4 *p, size_t n)
{
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256) {
        u32x4 v = {static_cast<unsigned>(i), 1u, 2u, 3u};
        if (NT)
            __builtin_nontemporal_store(v, p + i);
        else
            p[i] = v;
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void cp(const u32x4 *s, u32x4 *d, size_t n)
{
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256) {
        u32x4 v = __builtin_nontemporal_load(s + i);
        if (NT)
            __builtin_nontemporal_store(v, d + i);
        else
            d[i] = v;
    }
}

int main()
{
    const size_t bytes = size_t(2) << 30, n = bytes / 16;
    u32x4 *a, *b;
    unsigned *o;
    if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&o, 4))
        return 1;
    (void)hipMemset(a, 1, bytes);
    (void)hipMemset(b, 2, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char *names[] = {"read", "read_nt", "write", "write_nt", "copy", "copy_nt_store"};
    for (int grid : {2048, 4096, 8192, 16384}) {
        for (int k = 0; k < 6; ++k) {
            auto launch = [&]() {
                switch (k) {
                case 0: hipLaunchKernelGGL(rd<false>, dim3(grid), dim3(256), 0, 0, a, n, o); break;
                case 1: hipLaunchKernelGGL(rd<true>, dim3(grid), dim3(256), 0, 0, a, n, o); break;
                case 2: hipLaunchKernelGGL(wr<false>, dim3(grid), dim3(256), 0, 0, b, n); break;
                case 3: hipLaunchKernelGGL(wr<true>, dim3(grid), dim3(256), 0, 0, b, n); break;
                case 4: hipLaunchKernelGGL(cp<false>, dim3(grid), dim3(256), 0, 0, a, b, n / 2); break;
                default: hipLaunchKernelGGL(cp<true>, dim3(grid), dim3(256), 0, 0, a, b, n / 2); break;
                }
            };
            for (int w = 0; w < 3; ++w)
                launch();
            (void)hipEventRecord(e0);
            const int reps = 10;
            for (int r = 0; r < reps; ++r)
                launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            // bytes moved per launch: read/write = 2 GiB; copy = 1 GiB read + 1 GiB written
            const double gbps = double(bytes) * reps / (ms * 1e-3) / 1e9;
            printf("grid %5d %-14s %8.1f GB/s  (%.3f ms per 2 GiB)\n", grid, names[k], gbps, ms / reps);
        }
    }
    return 0;
}
