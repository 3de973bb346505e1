// Same-address atomics on MI355X (gfx950): how long does a kernel take when
// every workgroup adds one value to one (or a few) global counters, and how
// does that compare with a plain streaming read of the same grid?
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/ubench_atomics scripts/ubench_atomics.hip
//   ./scripts/ubench_atomics
// One JSON line per (blocks, counters, mode).
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

// each block: stream `per` bytes-worth of uint32 (coalesced), reduce in LDS,
// then thread 0 adds the sum to counters[blockIdx % nc] (mode 1), or writes
// it to part[blockIdx] (mode 0: no atomic)
__global__ __launch_bounds__(256) void k_stream(const uint32_t *in, uint64_t n, uint32_t *ctr,
                                                uint32_t nc, uint32_t *part, int mode)
{
    __shared__ uint32_t red[256];
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        acc += in[i];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < (unsigned)s)
            red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (mode == 1)
            atomicAdd(&ctr[(blockIdx.x % nc) * 16], red[0]);
        else
            part[blockIdx.x] = red[0];
    }
}

int main()
{
    const uint64_t n = 64ull << 20;   // 256 MiB of uint32
    uint32_t *in, *ctr, *part;
    CHECK(hipMalloc(&in, 4 * n));
    CHECK(hipMalloc(&ctr, 4 * 16 * 64));
    CHECK(hipMalloc(&part, 4 * 65536));
    CHECK(hipMemset(in, 1, 4 * n));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const unsigned blocks[] = {1024, 2048, 8192, 32768, 65536};
    const unsigned ncs[] = {1, 8};
    for (unsigned g : blocks)
        for (int mode = 0; mode < 2; mode++)
            for (unsigned nc : ncs) {
                if (mode == 0 && nc != 1)
                    continue;
                float best = 1e30f;
                for (int r = 0; r < 5; r++) {
                    CHECK(hipEventRecord(a));
                    hipLaunchKernelGGL(k_stream, dim3(g), dim3(256), 0, 0, in, n, ctr, nc, part,
                                       mode);
                    CHECK(hipEventRecord(b));
                    CHECK(hipEventSynchronize(b));
                    float ms;
                    CHECK(hipEventElapsedTime(&ms, a, b));
                    if (r)
                        best = ms < best ? ms : best;
                }
                printf("{\"blocks\": %u, \"atomic\": %d, \"counters\": %u, \"ms\": %.4f, "
                       "\"gbs\": %.1f}\n", g, mode, nc, best, 4.0 * n / (best * 1e-3) / 1e9);
            }
    return 0;
}
