// Single-wave calibration of the planner's block scan step on gfx950 (diagnostic, not part
// of the library): cycles per iteration of "load a 64-node block's free columns from LDS,
// three ballots, find the first fit", SoA vs AoS rows, with and without a dependent update.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int N = 2048, NB = N / 64;

struct Aos { int64_t c, m; int32_t p, pad; };

__global__ void k_scan(unsigned long long* out, int iters, int64_t seed) {
    extern __shared__ unsigned char raw[];
    int64_t* rc = reinterpret_cast<int64_t*>(raw);
    int64_t* rm = rc + N;
    int32_t* rp = reinterpret_cast<int32_t*>(rm + N);
    uint64_t* vis = reinterpret_cast<uint64_t*>(rp + N);
    Aos* ra = reinterpret_cast<Aos*>(vis + NB);
    const int lane = threadIdx.x;
    for (int i = lane; i < N; i += 64) {
        const int64_t v = (int64_t)((i * 2654435761u) % 1000);
        rc[i] = v; rm[i] = 1000 - v; rp[i] = (i % 7) ? 1 : 0;
        ra[i].c = v; ra[i].m = 1000 - v; ra[i].p = rp[i];
    }
    for (int j = lane; j < NB; j += 64) vis[j] = ~0ull ^ (1ull << (j & 63));
    __syncthreads();
    unsigned long long t0, t1;
    // 1. SoA: block j, three ballots, ctz; the pod request changes per iteration (uniform)
    {
        int32_t j = 0;
        int64_t pc = seed, pm = 1000 - seed;
        uint64_t acc = 0;
        t0 = clock64();
        for (int it = 0; it < iters; it++) {
            const int x = j * 64 + lane;
            const int64_t c = rc[x], m = rm[x];
            const int32_t p = rp[x];
            const uint64_t vw = __builtin_amdgcn_readfirstlane((int)vis[j]) | ((uint64_t)__builtin_amdgcn_readfirstlane((int)(vis[j] >> 32)) << 32);
            const uint64_t fit = vw & __ballot(p >= 1) & __ballot(pc <= c) & __ballot(pm <= m);
            const int f = fit ? __builtin_ctzll(fit) : 64;
            acc += (uint64_t)f;
            j = (j + 1 + (f & 1)) & (NB - 1);
            pc = (pc * 5 + 3) % 1000; pm = 1000 - pc;
        }
        t1 = clock64();
        if (lane == 0) { out[0] = t1 - t0; out[8] = acc; }
    }
    // 2. AoS rows (24-byte records)
    {
        int32_t j = 0;
        int64_t pc = seed, pm = 1000 - seed;
        uint64_t acc = 0;
        t0 = clock64();
        for (int it = 0; it < iters; it++) {
            const int x = j * 64 + lane;
            const int64_t c = ra[x].c, m = ra[x].m;
            const int32_t p = ra[x].p;
            const uint64_t vw = __builtin_amdgcn_readfirstlane((int)vis[j]) | ((uint64_t)__builtin_amdgcn_readfirstlane((int)(vis[j] >> 32)) << 32);
            const uint64_t fit = vw & __ballot(p >= 1) & __ballot(pc <= c) & __ballot(pm <= m);
            const int f = fit ? __builtin_ctzll(fit) : 64;
            acc += (uint64_t)f;
            j = (j + 1 + (f & 1)) & (NB - 1);
            pc = (pc * 5 + 3) % 1000; pm = 1000 - pc;
        }
        t1 = clock64();
        if (lane == 0) { out[1] = t1 - t0; out[9] = acc; }
    }
    // 3. SoA + the AddPod of the found row (lane f writes its row back: a store the next load may hit)
    {
        int32_t j = 0;
        int64_t pc = seed, pm = 1000 - seed;
        uint64_t acc = 0;
        t0 = clock64();
        for (int it = 0; it < iters; it++) {
            const int x = j * 64 + lane;
            const int64_t c = rc[x], m = rm[x];
            const int32_t p = rp[x];
            const uint64_t vw = __builtin_amdgcn_readfirstlane((int)vis[j]) | ((uint64_t)__builtin_amdgcn_readfirstlane((int)(vis[j] >> 32)) << 32);
            const uint64_t fit = vw & __ballot(p >= 1) & __ballot(pc <= c) & __ballot(pm <= m);
            const int f = fit ? __builtin_ctzll(fit) : 64;
            if (lane == f) { rc[x] = c - pc; rm[x] = m - pm; rp[x] = p; }
            acc += (uint64_t)f;
            j = (j + 1 + (f & 1)) & (NB - 1);
            pc = (pc * 5 + 3) % 1000; pm = 1000 - pc;
        }
        t1 = clock64();
        if (lane == 0) { out[2] = t1 - t0; out[10] = acc; }
    }
}

int main() {
    unsigned long long* d = nullptr;
    hipMalloc(&d, 16 * sizeof(unsigned long long));
    const size_t lds = N * (8 + 8 + 4) + NB * 8 + N * sizeof(Aos);
    hipFuncSetAttribute((const void*)k_scan, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const int iters = 100000;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_scan, dim3(1), dim3(64), lds, 0, d, iters, (int64_t)417);
        const hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess) { printf("error %s\n", hipGetErrorString(e)); return 1; }
    }
    unsigned long long h[16];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("cycles/iter: soa %.1f  aos %.1f  soa+addpod %.1f\n", (double)h[0] / iters, (double)h[1] / iters,
           (double)h[2] / iters);
    return 0;
}
