// Probe for a dot4 vertical pass (gfx950):
//  1. ds_read_b64_tr_b8 lane mapping: LDS holds a 16-row x 64-column byte image, byte(r, c) =
//     16 r + (c & 15) + 0x80 (c >> 4 ... per group); lane 2q+p of each 16-lane group supplies the
//     address of row q, columns 16g + 8p .. +7; printed: what lanes 0..17 receive.
//  2. issue cost per wave-instruction (8 independent chains, 4 and 8 waves per SIMD) of
//     v_dot4c_i32_i8 (VOP2), v_dot4_i32_i8 (VOP3P, SGPR operand), v_dot2c_i32_i16 (VOP2),
//     v_dot2_i32_i16 (VOP3P), v_pk_mad_u16, v_add_u32, v_perm_b32, v_xor_b32, ds_write_b16.
//   hipcc -O3 --offload-arch=gfx950 dot4.hip -o dot4 && ./dot4      (profiles/r03/ubench_dot4.txt)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void tr_probe(uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t img[16 * 64];
    const int t = threadIdx.x;
    for (int i = t; i < 16 * 64; i += 64)
        img[i] = static_cast<uint8_t>(((i / 64) << 4) | (i & 15)) ^ static_cast<uint8_t>(((i & 63) >> 4) << 7);
    __syncthreads();
    const int g = t >> 4, q = (t & 15) >> 1, p = t & 1;
    const uint32_t addr = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t *)img)) +
                          static_cast<uint32_t>(q * 64 + 16 * g + 8 * p);
    unsigned long long v;
    asm volatile("ds_read_b64_tr_b8 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    out[2 * t] = static_cast<uint32_t>(v);
    out[2 * t + 1] = static_cast<uint32_t>(v >> 32);
}

#define ITER 2048
template <int KIND>
__global__ __launch_bounds__(256) void rate(uint32_t *out, uint32_t seed, uint32_t c)
{
    __shared__ uint16_t sink[256 * 8];
    uint32_t a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        a[i] = seed * (threadIdx.x + 1) + 77u * i;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (KIND == 0)
                asm volatile("v_dot4c_i32_i8_e32 %0, %1, %2" : "+v"(a[i]) : "s"(c), "v"(a[(i + 3) & 7]));
            else if constexpr (KIND == 1)
                asm volatile("v_dot4_i32_i8 %0, %1, %2, %0" : "+v"(a[i]) : "s"(c), "v"(a[(i + 3) & 7]));
            else if constexpr (KIND == 2)
                asm volatile("v_dot2c_i32_i16_e32 %0, %1, %2" : "+v"(a[i]) : "s"(c), "v"(a[(i + 3) & 7]));
            else if constexpr (KIND == 3)
                asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(a[i]) : "s"(c), "v"(a[(i + 3) & 7]));
            else if constexpr (KIND == 4)
                asm volatile("v_pk_mad_u16 %0, %1, %2, %0" : "+v"(a[i]) : "s"(c), "v"(a[(i + 3) & 7]));
            else if constexpr (KIND == 5)
                asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(a[i]) : "v"(a[(i + 3) & 7]));
            else if constexpr (KIND == 6)
                asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(a[i]) : "v"(a[(i + 3) & 7]), "s"(c));
            else if constexpr (KIND == 7)
                asm volatile("v_xor_b32_e32 %0, %1, %0" : "+v"(a[i]) : "s"(c));
            else if constexpr (KIND == 8) {
                const uint32_t ad = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
                                        (__attribute__((address_space(3))) uint16_t *)sink)) + 2u * (threadIdx.x + 256u * i);
                asm volatile("ds_write_b16 %0, %1" ::"v"(ad), "v"(a[i]) : "memory");
            } else if constexpr (KIND == 9)
                asm volatile("v_dot2c_i32_i16_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(a[(i + 3) & 7]), "v"(c));
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        s ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + sink[threadIdx.x];
}

template <int KIND>
void run(const char *name, uint32_t *d, int cus)
{
    for (int wps : {4, 8}) {  // waves per SIMD: blocks of 4 waves, wps blocks per CU
        const int blocks = cus * wps;
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        rate<KIND><<<blocks, 256>>>(d, 3, 0x01020304u);
        hipEventRecord(e0);
        rate<KIND><<<blocks, 256>>>(d, 5, 0x01020304u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        // cycles per wave-instruction per SIMD, assuming a 2.4 GHz clock (ratios are what matter)
        const double instrPerSimd = double(ITER) * 8 * wps;
        printf("%-28s %d waves/SIMD: %.2f ns per 1000 wave-instr/SIMD  (%.2f cyc @2.4GHz)\n", name, wps,
               ms * 1e6 / instrPerSimd * 1000 / 1000, ms * 1e-3 * 2.4e9 / instrPerSimd);
    }
}

int main()
{
    uint32_t *d;
    hipMalloc(&d, 1 << 24);
    tr_probe<<<1, 64>>>(d);
    uint32_t h[128];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("ds_read_b64_tr_b8: lane: bytes (image byte = 16*row + col%%16, bit 7 = col/16 odd)\n");
    for (int l = 0; l < 20; ++l) {
        printf("lane %2d:", l);
        for (int b = 0; b < 8; ++b)
            printf(" %02x", (b < 4 ? h[2 * l] >> (8 * b) : h[2 * l + 1] >> (8 * (b - 4))) & 0xff);
        printf("\n");
    }
    int dev = 0;
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, dev);
    const int cus = prop.multiProcessorCount;
    run<0>("v_dot4c_i32_i8_e32", d, cus);
    run<1>("v_dot4_i32_i8 (vop3p, sgpr)", d, cus);
    run<2>("v_dot2c_i32_i16_e32", d, cus);
    run<3>("v_dot2_i32_i16 (vop3p)", d, cus);
    run<9>("v_dot2c_i32_i16_dpp", d, cus);
    run<4>("v_pk_mad_u16", d, cus);
    run<5>("v_add_u32_e32", d, cus);
    run<6>("v_perm_b32", d, cus);
    run<7>("v_xor_b32_e32", d, cus);
    run<8>("ds_write_b16", d, cus);
    hipFree(d);
    return 0;
}
