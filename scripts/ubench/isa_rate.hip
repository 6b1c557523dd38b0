// Microbenchmark: issue rate of the integer VALU forms used by the resize kernels on gfx950.
// Each kernel runs 8 independent chains of one instruction kind for ITER iterations; we report
// wall time per (wave-instruction) at full occupancy and at 1 wave per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

#define ITER 4096

template <int KIND>
__global__ void k(unsigned *out, unsigned seed, unsigned c)
{
    unsigned a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (KIND == 0) {  // v_pk_mad_u16
                u16x2 r = __builtin_bit_cast(u16x2, a[i]) * __builtin_bit_cast(u16x2, c) + __builtin_bit_cast(u16x2, a[(i + 1) & 7]);
                a[i] = __builtin_bit_cast(unsigned, r);
            } else if constexpr (KIND == 1) {  // v_dot2c_i32_i16
                a[i] = (unsigned)__builtin_amdgcn_sdot2(__builtin_bit_cast(i16x2, a[(i + 3) & 7]), __builtin_bit_cast(i16x2, c), (int)a[i], false);
            } else if constexpr (KIND == 2) {  // v_perm_b32
                a[i] = __builtin_amdgcn_perm(a[(i + 1) & 7], a[i], c);
            } else if constexpr (KIND == 3) {  // v_add_u32 (reference full-rate op)
                a[i] = a[i] + a[(i + 1) & 7];
            } else if constexpr (KIND == 4) {  // DPP wave_shr
                a[i] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)a[i], 0x138, 0xf, 0xf, false) + c;
            } else if constexpr (KIND == 5) {  // v_dot2_u32_u16
                a[i] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a[(i + 3) & 7]), __builtin_bit_cast(u16x2, c), a[i], false);
            } else if constexpr (KIND == 6) {  // v_dot4_u32_u8
                a[i] = __builtin_amdgcn_udot4(a[(i + 3) & 7], c, a[i], false);
            } else if constexpr (KIND == 7) {  // v_mad_u32_u24
                a[i] = (a[(i + 3) & 7] & 0xffffffu) * (c & 0xffffu) + a[i];
            } else if constexpr (KIND == 8) {  // v_pk_add_u16
                u16x2 r = __builtin_bit_cast(u16x2, a[i]) + __builtin_bit_cast(u16x2, a[(i + 3) & 7]);
                a[i] = __builtin_bit_cast(unsigned, r);
            } else if constexpr (KIND == 9) {  // v_mov_b32_dpp bound_ctrl (no old-value init)
                a[i] = (unsigned)__builtin_amdgcn_mov_dpp((int)a[(i + 3) & 7], 0x138, 0xf, 0xf, true);
            } else if constexpr (KIND == 10) {  // v_fma_f32 (reference)
                a[i] = __builtin_bit_cast(unsigned, __builtin_fmaf(__builtin_bit_cast(float, a[(i + 3) & 7]), 1.0001f, __builtin_bit_cast(float, a[i])));
            } else if constexpr (KIND == 11) {  // v_pk_mul_lo_u16
                u16x2 r = __builtin_bit_cast(u16x2, a[(i + 3) & 7]) * __builtin_bit_cast(u16x2, c);
                a[i] = __builtin_bit_cast(unsigned, r) ^ a[i];
            } else if constexpr (KIND == 12) {  // v_mul_lo_u32 (quarter-rate reference)
                a[i] = a[(i + 3) & 7] * c + a[i];
            }
        }
    }
    unsigned s = 0;
    for (int i = 0; i < 8; ++i) s ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void clk(unsigned long long *o, unsigned *out, unsigned c)
{
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    unsigned a[8];
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 8 + i;
    for (int it = 0; it < 4 * ITER; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i)
            a[i] = __builtin_bit_cast(unsigned, __builtin_fmaf(__builtin_bit_cast(float, a[(i + 3) & 7]), 1.0001f, __builtin_bit_cast(float, a[i])));
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    unsigned s = 0;
    for (int i = 0; i < 8; ++i) s ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) { o[2 * blockIdx.x] = t1 - t0; o[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int KIND>
double run(int blocks, int threads, unsigned *d)
{
    hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(threads), 0, 0, d, 1u, 0x00030005u);
    hipDeviceSynchronize();
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int r = 0; r < 5; ++r)
        hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(threads), 0, 0, d, 1u, 0x00030005u);
    hipDeviceSynchronize();
    double s = std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t0).count() / 5;
    double waveInstr = double(blocks) * (threads / 64) * ITER * 8;
    // per CU per cycle at 2.4 GHz
    return waveInstr / (s * 256 * 2.4e9);
}

int main()
{
    unsigned *d;
    hipMalloc(&d, 1 << 26);
    {
        unsigned long long *o, h[2];
        hipMalloc(&o, 1 << 20);
        hipLaunchKernelGGL(clk, dim3(2048), dim3(256), 0, 0, o, d, 3u);
        hipLaunchKernelGGL(clk, dim3(2048), dim3(256), 0, 0, o, d, 3u);
        hipMemcpy(h, o, 16, hipMemcpyDeviceToHost);
        printf("shader clock under full FMA load: %.0f MHz (memtime %llu ticks / memrealtime %llu @100MHz)\n",
               100.0 * h[0] / h[1], h[0], h[1]);
    }
    const char *names[] = {"v_pk_mad_u16", "v_dot2c_i32_i16", "v_perm_b32", "v_add_u32", "dpp wave_shr mov+add",
                           "v_dot2_u32_u16", "v_dot4_u32_u8", "v_mad_u32_u24", "v_pk_add_u16", "dpp mov bound_ctrl",
                           "v_fma_f32", "v_pk_mul_lo_u16+xor", "v_mul_lo_u32+add"};
    for (int cfg = 0; cfg < 3; ++cfg) {
        // 8 blocks/CU (8 waves/SIMD), 2 blocks/CU (2 waves/SIMD), 1 block/CU (1 wave/SIMD)
        int blocks = cfg == 0 ? 256 * 8 : (cfg == 1 ? 512 : 256), threads = 256;
        double r[13] = {run<0>(blocks, threads, d), run<1>(blocks, threads, d), run<2>(blocks, threads, d),
                        run<3>(blocks, threads, d), run<4>(blocks, threads, d), run<5>(blocks, threads, d),
                        run<6>(blocks, threads, d), run<7>(blocks, threads, d), run<8>(blocks, threads, d),
                        run<9>(blocks, threads, d), run<10>(blocks, threads, d), run<11>(blocks, threads, d),
                        run<12>(blocks, threads, d)};
        for (int i = 0; i < 13; ++i)
            printf("%-22s %s: %.3f wave-instr / CU / cycle\n", names[i], cfg == 0 ? "8 waves/SIMD" : (cfg == 1 ? "2 waves/SIMD" : "1 wave/SIMD "), r[i]);
    }
    return 0;
}
