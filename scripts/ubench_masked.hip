// Cost of partially-active random loads on gfx950: each lane issues ILP
// independent random 16-B loads from an L2-resident table, but only 1 of
// every `every` lanes is active (EXEC-masked wave instructions).  If the
// time stays flat as `every` grows the address path costs per instruction,
// if it falls with the active lanes it costs per lane.
//
//   hipcc --offload-arch=gfx950 -O3 -o ubench_masked scripts/ubench_masked.hip
//   ./ubench_masked            -> one JSON line per active-lane fraction
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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

template <int ILP>
__global__ __launch_bounds__(1024) void k_masked(const uint4 *tab, uint32_t mask,
                                                 int iters, uint32_t every,
                                                 uint32_t *sink)
{
    uint32_t acc = 0;
    const uint32_t seed = blockIdx.x * 1024 + threadIdx.x;
    const bool on = (threadIdx.x % every) == 0;
    for (int it = 0; it < iters; it++) {
        uint4 v[ILP];
#pragma unroll
        for (int j = 0; j < ILP; j++) {
            v[j] = make_uint4(0, 0, 0, 0);
            if (on)
                v[j] = tab[mix(seed * 0x9E3779B9u + (uint32_t)(it * ILP + j)) & mask];
        }
#pragma unroll
        for (int j = 0; j < ILP; j++)
            acc += v[j].x ^ v[j].w;
    }
    if (acc == 0x12345678u)
        sink[0] = acc;
}

int main()
{
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int grid = p.multiProcessorCount * 2, iters = 64;
    const size_t bytes = 2u << 20;
    uint4 *tab;
    uint32_t *sink;
    CHECK(hipMalloc(&tab, bytes));
    CHECK(hipMalloc(&sink, 4));
    CHECK(hipMemset(tab, 1, bytes));
    for (uint32_t every : {1u, 2u, 4u, 8u, 16u, 32u, 64u}) {
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        for (int rep = 0; rep < 2; rep++) {
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL((k_masked<8>), dim3(grid), dim3(1024), 0, 0, tab,
                               (uint32_t)(bytes / 16 - 1), iters, every, sink);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
        }
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        const double instrs = (double)grid * 16 * iters * 8;   // wave-instructions
        const double lanes = (double)grid * 1024 / every * iters * 8;
        printf("{\"active_every\": %u, \"ms\": %.3f, \"g_wave_instr_per_s\": %.3f, "
               "\"g_lane_loads_per_s\": %.2f}\n",
               every, ms, instrs / (ms * 1e-3) / 1e9, lanes / (ms * 1e-3) / 1e9);
        fflush(stdout);
        CHECK(hipEventDestroy(a));
        CHECK(hipEventDestroy(b));
    }
    return 0;
}
