// Random-access roofline microbenchmark for MI355X (gfx950).
//
// Measures independent random loads per second (and the 64-B lines they
// touch) from a table of a given size, so the classify kernel's lookup rate
// can be set against what the memory hierarchy delivers for its access
// shape: L2-resident (<= 4 MiB/XCD), Infinity-Cache-resident (<= 256 MiB)
// and HBM-resident tables, 4-byte and 16-byte loads.
//
//   hipcc --offload-arch=gfx950 -O3 -o ubench_random scripts/ubench_random.hip
//   ./ubench_random [MiB ...]  -> one JSON line per (table size, load width,
//                                 loads in flight per lane)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
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

// Each thread issues ILP independent random loads per iteration (addresses
// from a hash, so there is no dependent chain), ITERS iterations.
template <int ILP, bool WIDE>
__global__ __launch_bounds__(1024) void k_random(const uint4 *tab, uint32_t mask,
                                                 int iters, uint32_t *sink)
{
    uint32_t acc = 0;
    uint32_t seed = blockIdx.x * 1024 + threadIdx.x;
    for (int it = 0; it < iters; it++) {
        uint32_t idx[ILP];
#pragma unroll
        for (int j = 0; j < ILP; j++)
            idx[j] = mix(seed * 0x9E3779B9u + (uint32_t)(it * ILP + j)) & mask;
        if (WIDE) {
            uint4 v[ILP];
#pragma unroll
            for (int j = 0; j < ILP; j++)
                v[j] = tab[idx[j]];
#pragma unroll
            for (int j = 0; j < ILP; j++)
                acc += v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
        } else {
            const uint32_t *t = reinterpret_cast<const uint32_t *>(tab);
            uint32_t v[ILP];
#pragma unroll
            for (int j = 0; j < ILP; j++)
                v[j] = t[(size_t)idx[j] * 4];
#pragma unroll
            for (int j = 0; j < ILP; j++)
                acc += v[j];
        }
    }
    if (acc == 0x12345678u)
        sink[0] = acc;
}

template <int ILP>
static float run(bool wide, int grid, const uint4 *tab, uint32_t mask, int iters,
                 uint32_t *sink)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int rep = 0; rep < 2; rep++) {   // first pass warms caches
        CHECK(hipEventRecord(a));
        if (wide)
            hipLaunchKernelGGL((k_random<ILP, true>), dim3(grid), dim3(1024), 0, 0,
                               tab, mask, iters, sink);
        else
            hipLaunchKernelGGL((k_random<ILP, false>), dim3(grid), dim3(1024), 0, 0,
                               tab, mask, iters, sink);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
    }
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return ms;
}

int main(int argc, char **argv)
{
    int cus = 256;
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    cus = p.multiProcessorCount;
    std::vector<size_t> sizes_mb = {1, 2, 8, 32, 64, 128, 192, 512, 4096};
    if (argc > 1) {
        sizes_mb.clear();
        for (int i = 1; i < argc; i++)
            sizes_mb.push_back((size_t)atoi(argv[i]));
    }
    uint32_t *sink;
    CHECK(hipMalloc(&sink, 4));
    for (size_t mb : sizes_mb) {
        size_t bytes = mb << 20;
        size_t n16 = bytes / 16;   // power of two
        uint4 *tab;
        CHECK(hipMalloc(&tab, bytes));
        CHECK(hipMemset(tab, 1, bytes));
        for (int wide = 0; wide < 2; wide++) {
            for (int ilp : {4, 8, 16}) {
                const int grid = cus * 2, iters = 64;
                const uint32_t mask = (uint32_t)(n16 - 1);
                const float ms = ilp == 4 ? run<4>(wide, grid, tab, mask, iters, sink)
                                 : ilp == 8 ? run<8>(wide, grid, tab, mask, iters, sink)
                                            : run<16>(wide, grid, tab, mask, iters, sink);
                const double loads = (double)grid * 1024 * iters * ilp;
                printf("{\"table_mib\": %zu, \"load_bytes\": %d, \"ilp\": %d, "
                       "\"gloads_per_s\": %.2f, \"ms\": %.3f}\n",
                       mb, wide ? 16 : 4, ilp, loads / (ms * 1e-3) / 1e9, ms);
                fflush(stdout);
            }
        }
        CHECK(hipFree(tab));
    }
    return 0;
}
