// tools/isa_probe.hip -- checks, on the MI355X, the gfx950 instruction semantics the round-3
// IDCT / CSC rewrite relies on (development tool; prints one line per check, exit 1 on any
// mismatch):
//   1. v_dot2_i32_i16 ... clamp        : a.lo*b.lo + a.hi*b.hi + c saturated to int32
//   2. v_ashr_pk_u8_i32 op_sel:[0,0,0,1]: writes its two bytes to bits 16..31, keeps 0..15
//   3. v_sat_pk_u8_i16                 : {sat_u8(lo16), sat_u8(hi16)} in bits 0..15 (and what
//                                        lands in 16..31)
//   4. v_sat_pk_u8_i16 sdwa dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE
//   5. v_pk_add_u16 op_sel_hi:[0,0]    : both lanes from the low halves
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/isa_probe tools/isa_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void probe(const uint32_t* a, const uint32_t* b, const uint32_t* c, uint32_t* o, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t x = a[i], y = b[i], z = c[i];
    uint32_t r1, r2 = z, r3, r4 = z, r5;
    asm volatile("v_dot2_i32_i16 %0, %1, %2, %3 clamp" : "=v"(r1) : "v"(x), "v"(y), "v"(z));
    asm volatile("v_ashr_pk_u8_i32 %0, %1, %2, 3 op_sel:[0,0,0,1]" : "+v"(r2) : "v"(x), "v"(y));
    asm volatile("v_sat_pk_u8_i16 %0, %1" : "=v"(r3) : "v"(x));
    asm volatile("v_sat_pk_u8_i16_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD" : "+v"(r4) : "v"(x));
    asm volatile("v_pk_add_u16 %0, %1, %2 op_sel_hi:[0,0]" : "=v"(r5) : "v"(x), "v"(y));
    o[5 * i + 0] = r1;
    o[5 * i + 1] = r2;
    o[5 * i + 2] = r3;
    o[5 * i + 3] = r4;
    o[5 * i + 4] = r5;
}

static uint64_t st = 88172645463325252ull;
static uint32_t rnd() {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return (uint32_t)st;
}
static uint8_t satu8(int64_t v) { return v < 0 ? 0 : v > 255 ? 255 : (uint8_t)v; }

int main() {
    const int n = 1 << 20;
    uint32_t *a = (uint32_t*)malloc(4 * n), *b = (uint32_t*)malloc(4 * n), *c = (uint32_t*)malloc(4 * n),
             *o = (uint32_t*)malloc(20 * n);
    const uint32_t edge[] = {0x80008000u, 0x7fff7fffu, 0x80007fffu, 0u, 0xffffffffu, 0x00ff0100u, 0xff00ff01u};
    for (int i = 0; i < n; i++) {
        a[i] = i < 7 * 7 ? edge[i % 7] : rnd();
        b[i] = i < 7 * 7 ? edge[i / 7] : rnd();
        c[i] = (i & 3) == 0 ? 0x7fffff00u : (i & 3) == 1 ? 0x80000100u : rnd();
        if ((i & 7) == 5) a[i] &= 0x01ff01ffu;  // small values for the saturation checks
        if ((i & 7) == 6) a[i] |= 0xfe00fe00u;
    }
    uint32_t *da, *db, *dc, *dout;
    hipMalloc(&da, 4 * n);
    hipMalloc(&db, 4 * n);
    hipMalloc(&dc, 4 * n);
    hipMalloc(&dout, 20 * n);
    hipMemcpy(da, a, 4 * n, hipMemcpyHostToDevice);
    hipMemcpy(db, b, 4 * n, hipMemcpyHostToDevice);
    hipMemcpy(dc, c, 4 * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(n / 256), dim3(256), 0, 0, da, db, dc, dout, n);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel failed\n");
        return 2;
    }
    hipMemcpy(o, dout, 20 * n, hipMemcpyDeviceToHost);
    long bad[5] = {0, 0, 0, 0, 0};
    uint32_t hi3_or = 0;
    for (int i = 0; i < n; i++) {
        const int16_t al = (int16_t)a[i], ah = (int16_t)(a[i] >> 16), bl = (int16_t)b[i], bh = (int16_t)(b[i] >> 16);
        int64_t s = (int64_t)al * bl + (int64_t)ah * bh + (int64_t)(int32_t)c[i];
        if (s > INT32_MAX) s = INT32_MAX;
        if (s < INT32_MIN) s = INT32_MIN;
        if (o[5 * i] != (uint32_t)(int32_t)s) bad[0]++;
        const uint32_t pk = satu8((int32_t)a[i] >> 3) | ((uint32_t)satu8((int32_t)b[i] >> 3) << 8);
        if (o[5 * i + 1] != ((c[i] & 0xffffu) | (pk << 16))) bad[1]++;
        const uint32_t sp = satu8(al) | ((uint32_t)satu8(ah) << 8);
        if ((o[5 * i + 2] & 0xffffu) != sp) bad[2]++;
        hi3_or |= o[5 * i + 2] >> 16;
        if (o[5 * i + 3] != ((c[i] & 0xffffu) | (sp << 16))) bad[3]++;
        const uint32_t pa = (uint32_t)(uint16_t)(al + bl) | ((uint32_t)(uint16_t)(al + bl) << 16);
        if (o[5 * i + 4] != pa) bad[4]++;
    }
    const char* names[5] = {"dot2_i32_i16 clamp saturates", "ashr_pk_u8_i32 op_sel dst -> bits 16..31, 0..15 kept",
                            "sat_pk_u8_i16 -> bits 0..15", "sat_pk_u8_i16 sdwa WORD_1 preserve",
                            "pk_add_u16 op_sel_hi:[0,0] broadcasts the low halves"};
    int fails = 0;
    for (int k = 0; k < 5; k++) {
        printf("%-60s %s (%ld of %d mismatched)\n", names[k], bad[k] ? "NO" : "yes", bad[k], n);
        fails += bad[k] != 0;
    }
    printf("sat_pk_u8_i16 bits 16..31 (OR over all lanes): 0x%04x\n", hi3_or);
    return fails ? 1 : 0;
}
