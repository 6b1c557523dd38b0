// Semantics probe for gfx950 v_ashr_pk_u8_i32 (byte order, saturation, bits 16..31).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const int *a, const int *b, unsigned *out, int n)
{
    int i = threadIdx.x;
    if (i >= n) return;
    unsigned d = 0xdeadbeefu;
    asm volatile("v_ashr_pk_u8_i32 %0, %1, %2, 20" : "+v"(d) : "v"(a[i]), "v"(b[i]));
    out[i] = d;
    unsigned e = 0x12345678u;
    asm volatile("v_ashr_pk_u8_i32 %0, %1, %2, 20 op_sel:[0,0,0,1]" : "+v"(e) : "v"(a[i]), "v"(b[i]));
    out[n + i] = e;
}
int main()
{
    const int n = 8;
    int ha[n] = {5 << 20, -1, 300 << 20, 255 << 20, (7 << 20) + 0xfffff, -(3 << 20), 0x7fffffff, 0};
    int hb[n] = {9 << 20, 128 << 20, 2 << 20, 256 << 20, 1 << 20, 77 << 20, (int)0x80000000, 1234567};
    int *da, *db; unsigned *dout, hout[2 * n];
    hipMalloc(&da, sizeof ha); hipMalloc(&db, sizeof hb); hipMalloc(&dout, sizeof hout);
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice); hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    k<<<1, 64>>>(da, db, dout, n);
    hipMemcpy(hout, dout, sizeof hout, hipMemcpyDeviceToHost);
    for (int i = 0; i < n; ++i)
        printf("a=%d b=%d  sh20: %08x   opsel_hi: %08x\n", ha[i] >> 20, hb[i] >> 20, hout[i], hout[n + i]);
    return 0;
}
