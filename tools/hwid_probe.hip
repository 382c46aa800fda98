// tools/hwid_probe.hip -- which SIMD each wave of a 4-wave workgroup lands on (HW_REG_HW_ID).
// The 4:2:0 / 4:4:4 tiles give IDCT blocks to waves 0-2 only (192 blocks, 256 lanes); if wave 3
// of every workgroup sat on the same SIMD, a quarter of the CU's VALUs would idle through the
// IDCT.  Build: hipcc --offload-arch=gfx950 -O3 tools/hwid_probe.hip -o tools/hwid_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <map>
#include <vector>

template <int LDS>
__global__ void __launch_bounds__(256) hwid_kernel(uint32_t* out, uint32_t spin) {
    __shared__ uint32_t pad[LDS / 4];
    uint32_t id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const uint32_t w = threadIdx.x / 64;
    // keep the workgroup resident a while so that several share a CU
    uint32_t x = threadIdx.x;
    for (uint32_t i = 0; i < spin; i++) x = x * 1664525u + 1013904223u;
    pad[threadIdx.x] = x;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        out[(blockIdx.x * 4 + w) * 2 + 0] = id;
        out[(blockIdx.x * 4 + w) * 2 + 1] = (xcc & 0xf) | (pad[(threadIdx.x + 64) & 255] == 12345u ? 0x100u : 0u);
    }
}

template <int LDS>
static void run(const char* tag, uint32_t nwg) {
    uint32_t* d;
    hipMalloc(&d, (size_t)nwg * 8 * 4);
    hipLaunchKernelGGL(hwid_kernel<LDS>, dim3(nwg), dim3(256), 0, 0, d, 20000u);
    hipDeviceSynchronize();
    std::vector<uint32_t> h((size_t)nwg * 8);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    hipFree(d);
    int cnt[4][4] = {};
    std::map<uint64_t, int> simd3;  // per CU: how many wave-3s on each SIMD
    std::map<uint64_t, std::vector<int>> percu;
    for (uint32_t b = 0; b < nwg; b++)
        for (int w = 0; w < 4; w++) {
            const uint32_t id = h[(b * 4 + w) * 2], xcc = h[(b * 4 + w) * 2 + 1] & 0xf;
            const int simd = (id >> 4) & 3;
            cnt[w][simd]++;
            const uint64_t cu = ((uint64_t)xcc << 16) | ((id >> 8) & 0xff) | (((id >> 13) & 7) << 8) | (((id >> 12) & 1) << 12);
            if (w == 3) {
                auto& v = percu[cu];
                if (v.empty()) v.assign(4, 0);
                v[simd]++;
            }
        }
    printf("%s (%u workgroups of 4 waves, %d B LDS):\n", tag, nwg, LDS);
    for (int w = 0; w < 4; w++) printf("  wave %d on SIMD 0..3: %6d %6d %6d %6d\n", w, cnt[w][0], cnt[w][1], cnt[w][2], cnt[w][3]);
    int shown = 0;
    for (auto& kv : percu) {
        if (shown++ >= 6) break;
        printf("  CU %06llx: wave 3 on SIMD 0..3: %d %d %d %d\n", (unsigned long long)kv.first, kv.second[0], kv.second[1],
               kv.second[2], kv.second[3]);
    }
    printf("  distinct CUs seen: %zu\n", percu.size());
}

int main() {
    run<36 * 1024>("4 per CU (stream kernel LDS)", 8192);
    run<24 * 1024>("6 per CU (batch kernel LDS)", 8192);
    run<4 * 1024>("LDS-light", 8192);
    return 0;
}
