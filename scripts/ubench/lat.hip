// Single-wave latency calibration on gfx950 (diagnostic, not part of the library):
// cycles per instruction for dependent VALU, SALU, v_readlane, LDS read round trips,
// L2-hit global loads and DPP wave reductions, as seen by one wavefront alone on a CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

extern "C" __device__ int __ockl_wfred_add_i32(int);

__global__ void k_lat(unsigned long long* out, const uint64_t* g, int iters) {
    __shared__ uint64_t lds[4096];
    const int lane = threadIdx.x;
    for (int i = lane; i < 4096; i += 64) lds[i] = (uint64_t)((i * 7 + 1) & 4095);
    __syncthreads();
    unsigned long long t0, t1;
    // 1. dependent VALU chain
    uint32_t v = lane;
    t0 = clock64();
    for (int i = 0; i < iters; i++) {
        v = v * 3u + 1u; v ^= v >> 3; v += 7u; v = (v << 1) | 1u;
    }
    t1 = clock64();
    if (lane == 0) out[0] = (t1 - t0);
    out[16 + lane % 4] = v;
    // 2. dependent SALU chain (uniform values)
    uint32_t s = __builtin_amdgcn_readfirstlane(iters);
    t0 = clock64();
    for (int i = 0; i < iters; i++) {
        s = __builtin_amdgcn_readfirstlane(s * 3u + 1u); s ^= s >> 3; s += 7u; s = (s << 1) | 1u;
    }
    t1 = clock64();
    if (lane == 0) { out[1] = (t1 - t0); out[20] = s; }
    // 3. LDS pointer chase (uniform address)
    uint64_t p = 1;
    t0 = clock64();
    for (int i = 0; i < iters; i++) p = lds[p];
    t1 = clock64();
    if (lane == 0) { out[2] = (t1 - t0); out[21] = p; }
    // 4. global pointer chase (L2/L1 hit, 64 distinct lines)
    uint64_t q = 0;
    t0 = clock64();
    for (int i = 0; i < iters; i++) q = g[q];
    t1 = clock64();
    if (lane == 0) { out[3] = (t1 - t0); out[22] = q; }
    // 5. readlane chain: value moves through lanes
    int r = lane;
    t0 = clock64();
    for (int i = 0; i < iters; i++) {
        int x = __builtin_amdgcn_readlane(r, (i & 63));
        r = r + x;
    }
    t1 = clock64();
    if (lane == 0) { out[4] = (t1 - t0); out[23] = r; }
    // 6. DPP wave reduction chain
    int w = lane;
    t0 = clock64();
    for (int i = 0; i < iters; i++) w = __ockl_wfred_add_i32(w) & 1023;
    t1 = clock64();
    if (lane == 0) { out[5] = (t1 - t0); out[24] = w; }
    // 7. ballot + ctz chain
    uint32_t b = lane;
    t0 = clock64();
    for (int i = 0; i < iters; i++) {
        uint64_t m = __ballot(((b + i) & 7) == 0);
        b += (uint32_t)__builtin_ctzll(m | (1ull << 63));
    }
    t1 = clock64();
    if (lane == 0) { out[6] = (t1 - t0); out[25] = b; }
    // 8. global load coherent (sc1) chase
    uint64_t q2 = 0;
    t0 = clock64();
    for (int i = 0; i < iters; i++) q2 = __builtin_nontemporal_load(&g[q2]);
    t1 = clock64();
    if (lane == 0) { out[7] = (t1 - t0); out[26] = q2; }
    // 9. empty loop
    t0 = clock64();
    for (int i = 0; i < iters; i++) __asm__ volatile("" ::: "memory");
    t1 = clock64();
    if (lane == 0) out[8] = (t1 - t0);
    // 10. s_memrealtime vs clock64: clock rate
    unsigned long long r0 = wall_clock64();
    t0 = clock64();
    for (int i = 0; i < iters * 16; i++) { v = v * 3u + 1u; }
    t1 = clock64();
    unsigned long long r1 = wall_clock64();
    if (lane == 0) { out[9] = (t1 - t0); out[10] = r1 - r0; out[27] = v; }
}

int main() {
    const int iters = 4096;
    uint64_t h[64];
    for (int i = 0; i < 64; i++) h[i] = (uint64_t)((i * 17 + 5) % 64) * 8;   // chase across 64 lines
    uint64_t* g; unsigned long long* o;
    hipMalloc(&g, 64 * 8 * 8);
    uint64_t hb[512] = {0};
    for (int i = 0; i < 64; i++) hb[i * 8] = h[i];
    hipMemcpy(g, hb, sizeof hb, hipMemcpyHostToDevice);
    hipMalloc(&o, 64 * 8);
    int rate = 0; hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, o, g, iters);
        hipDeviceSynchronize();
    }
    unsigned long long r[32];
    hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    const char* names[] = {"valu 4-op chain", "salu 4-op chain (+readfirstlane)", "lds chase", "global chase (L1/L2)",
                           "readlane chain", "dpp wfred", "ballot+ctz", "nontemporal chase", "empty loop"};
    for (int i = 0; i < 9; i++) printf("%-36s %8.1f cycles/iter\n", names[i], (double)r[i] / iters);
    printf("clock: %.0f cycles over %llu wall ticks (wall rate %d kHz) -> %.2f GHz\n", (double)r[9], r[10], rate,
           (double)r[9] / ((double)r[10] / (rate * 1e3)) / 1e9);
    return 0;
}
