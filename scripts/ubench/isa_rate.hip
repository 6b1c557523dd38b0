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
            }
        }
    }
    unsigned s = 0;
    for (int i = 0; i < 8; ++i) s ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
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
    const char *names[] = {"v_pk_mad_u16", "v_dot2c_i32_i16", "v_perm_b32", "v_add_u32", "dpp wave_shr mov+add", "v_dot2_u32_u16"};
    for (int cfg = 0; cfg < 2; ++cfg) {
        int blocks = cfg == 0 ? 256 * 8 : 256, threads = 256;  // 8 blocks/CU (8 waves/SIMD) vs 1 block/CU (1 wave/SIMD)
        double r[6] = {run<0>(blocks, threads, d), run<1>(blocks, threads, d), run<2>(blocks, threads, d),
                       run<3>(blocks, threads, d), run<4>(blocks, threads, d), run<5>(blocks, threads, d)};
        for (int i = 0; i < 6; ++i)
            printf("%-22s %s: %.3f wave-instr / CU / cycle\n", names[i], cfg == 0 ? "8 waves/SIMD" : "1 wave/SIMD ", r[i]);
    }
    return 0;
}
