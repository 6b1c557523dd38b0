// Microbenchmark (2): issue rate of simple 32-bit VALU forms on gfx950, to sort full-rate (2 cycles
// per wave64 instruction per SIMD) from half-rate (4 cycles) operations.  8 independent chains.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>
#define ITER 4096
typedef short i16x2 __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ void k(unsigned *out, unsigned seed, unsigned c)
{
    unsigned a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 8 + i;
    unsigned vb = c ^ threadIdx.x;  // a VGPR operand
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            unsigned x = a[(i + 3) & 7], y = a[i], r;
            if constexpr (KIND == 0) asm volatile("v_lshl_add_u32 %0, %1, 3, %2" : "=v"(r) : "v"(x), "v"(y));
            if constexpr (KIND == 1) asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(vb));
            if constexpr (KIND == 2) asm volatile("v_sub_u32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
            if constexpr (KIND == 3) asm volatile("v_and_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
            if constexpr (KIND == 4) asm volatile("v_lshrrev_b32 %0, 8, %1" : "=v"(r) : "v"(x));
            if constexpr (KIND == 5) asm volatile("v_alignbit_b32 %0, %1, %2, 16" : "=v"(r) : "v"(x), "v"(y));
            if constexpr (KIND == 6) asm volatile("v_bfe_u32 %0, %1, 8, 8" : "=v"(r) : "v"(x));
            if constexpr (KIND == 7) asm volatile("v_lshl_or_b32 %0, %1, 8, %2" : "=v"(r) : "v"(x), "v"(y));
            if constexpr (KIND == 8) asm volatile("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(vb));
            if constexpr (KIND == 9) asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
            if constexpr (KIND == 10) asm volatile("v_max_i32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
            if constexpr (KIND == 11) asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
            if constexpr (KIND == 12) asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(r) : "v"(x));
            if constexpr (KIND == 13) asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(*(unsigned long long*)&a[0]) : "v"(*(unsigned long long*)&a[2]), "v"(*(unsigned long long*)&a[4]), "v"(*(unsigned long long*)&a[6]));
            if constexpr (KIND == 14) asm volatile("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(vb));
            if constexpr (KIND == 15) asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(r) : "v"(x), "v"(y));
            if constexpr (KIND == 16) asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
            if constexpr (KIND == 17) asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
            if constexpr (KIND == 18) asm volatile("v_lshlrev_b32 %0, 5, %1" : "=v"(r) : "v"(x));
            if constexpr (KIND == 19) asm volatile("v_pk_sub_u16 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
            if constexpr (KIND == 20) asm volatile("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
            if constexpr (KIND == 21) asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(vb));
            if constexpr (KIND == 22) asm volatile("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(vb));
            if constexpr (KIND == 23) asm volatile("v_add_u16 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
            if constexpr (KIND == 24) asm volatile("v_mad_u16 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(vb));
            if constexpr (KIND == 25) asm volatile("v_mul_lo_u16 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
            if constexpr (KIND == 26) asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(vb));
            if constexpr (KIND == 27) asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0" : "=v"(r) : "v"(x));
            if constexpr (KIND != 13) a[i] = r;
        }
    }
    unsigned s = 0;
    for (int i = 0; i < 8; ++i) s ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND>
double run(int blocks, unsigned *d)
{
    hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, d, 1u, 0x00030005u);
    (void)hipDeviceSynchronize();
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int r = 0; r < 5; ++r)
        hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, d, 1u, 0x00030005u);
    (void)hipDeviceSynchronize();
    double s = std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t0).count() / 5;
    double waveInstr = double(blocks) * 4 * ITER * (KIND == 13 ? 1 : 8);
    return s * 1024 * 2.1e9 / waveInstr;  // cycles per wave-instruction per SIMD at ~2.1 GHz
}

template <int... K>
void all(int blocks, unsigned *d, std::integer_sequence<int, K...>)
{
    const char *names[] = {"v_lshl_add_u32", "v_add3_u32", "v_sub_u32", "v_and_b32", "v_lshrrev_b32", "v_alignbit_b32",
                           "v_bfe_u32", "v_lshl_or_b32", "v_and_or_b32", "v_mov_b32", "v_max_i32", "v_mul_f32",
                           "v_cvt_f32_ubyte1", "v_pk_fma_f32(1 chain)", "v_dot2_i32_i16 vop3", "v_cndmask_b32",
                           "v_add_u32", "v_xor_b32", "v_lshlrev_b32", "v_pk_sub_u16", "v_mul_u32_u24", "v_perm_b32",
                           "v_pk_mad_u16", "v_add_u16", "v_mad_u16", "v_mul_lo_u16", "v_fma_f32", "v_mov_b32_dpp"};
    ((printf("%-24s %d blk/CU: %.2f cyc/wave-instr/SIMD\n", names[K], blocks / 256, run<K>(blocks, d))), ...);
}

int main()
{
    unsigned *d;
    (void)hipMalloc(&d, 1 << 26);
    all(256 * 8, d, std::make_integer_sequence<int, 28>{});
    return 0;
}
