// Hit/miss-mix microbenchmark for MI355X (gfx950): do L2 hits and HBM
// misses of one kernel add up in time, or overlap?
//
// Every thread issues ILP independent random 16-byte loads per iteration; a
// fraction p of them (a hash test per load, so hits and misses interleave in
// every wave) read a 2 MiB table (L2-resident), the rest a 4 GiB table
// (HBM).  For each p the chip-wide rate is compared with the two models the
// classify roofline could use, from the pure rates h (p = 1) and m (p = 0):
//   additive  t = N (p / h + (1 - p) / m)     (bench.py's "frac")
//   overlap   t = N max(p / h, (1 - p) / m)
// One JSON line per p: {"p", "gloads_per_s", "additive_pred", "overlap_pred"}.
//
//   hipcc --offload-arch=gfx950 -O3 -o ubench_mix scripts/ubench_mix.hip
//   ./ubench_mix
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__,                 \
                    hipGetErrorString(e_));                                   \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

constexpr int ILP = 8;

// thr: loads whose hash's low 10 bits fall below it go to the small table
__global__ __launch_bounds__(1024) void k_mix(const uint4 *small, uint32_t smask,
                                              const uint4 *large, uint32_t lmask,
                                              uint32_t thr, int iters, uint32_t *sink)
{
    uint32_t acc = 0;
    const uint32_t seed = blockIdx.x * 1024 + threadIdx.x;
    for (int it = 0; it < iters; it++) {
        uint4 v[ILP];
#pragma unroll
        for (int j = 0; j < ILP; j++) {
            const uint32_t h = mix(seed * 0x9E3779B9u + (uint32_t)(it * ILP + j));
            const bool hit = (h & 1023u) < thr;
            const uint4 *t = hit ? small : large;
            const uint32_t idx = mix(h ^ 0x5bd1e995u) & (hit ? smask : lmask);
            v[j] = t[idx];
        }
#pragma unroll
        for (int j = 0; j < ILP; j++)
            acc += v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
    if (acc == 0x12345678u)
        sink[0] = acc;
}

int main()
{
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const size_t sbytes = 2ull << 20, lbytes = 4ull << 30;
    uint4 *small, *large;
    uint32_t *sink;
    CHECK(hipMalloc(&small, sbytes));
    CHECK(hipMalloc(&large, lbytes));
    CHECK(hipMalloc(&sink, 4));
    CHECK(hipMemset(small, 1, sbytes));
    CHECK(hipMemset(large, 1, lbytes));
    const uint32_t smask = (uint32_t)(sbytes / 16 - 1), lmask = (uint32_t)(lbytes / 16 - 1);
    const int grid = cus * 2, iters = 256;
    const double loads = (double)grid * 1024 * iters * ILP;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const uint32_t thrs[] = {0, 256, 512, 768, 896, 960, 1000, 1024};
    std::vector<double> rate(sizeof(thrs) / sizeof(thrs[0]));
    for (size_t i = 0; i < rate.size(); i++) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {   // (the first warms the small table)
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(k_mix, dim3(grid), dim3(1024), 0, 0, small, smask, large, lmask,
                               thrs[i], iters, sink);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, b));
            if (rep)
                best = ms < best ? ms : best;
        }
        rate[i] = loads / (best * 1e-3) / 1e9;
    }
    const double m = rate[0], h = rate.back();
    for (size_t i = 0; i < rate.size(); i++) {
        const double pf = thrs[i] / 1024.0;
        const double add = 1.0 / (pf / h + (1 - pf) / m);
        const double ovl = 1.0 / std::max(pf / h, (1 - pf) / m);
        printf("{\"p\": %.4f, \"gloads_per_s\": %.2f, \"additive_pred\": %.2f, "
               "\"overlap_pred\": %.2f}\n", pf, rate[i], add, ovl);
    }
    return 0;
}
