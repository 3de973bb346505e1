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
// Stream mode (./ubench_mix stream): the misses of the classify kernels are
// not random table lines but their header stream — coalesced 16-byte-per-lane
// loads of consecutive items, issued one iteration ahead — and the output
// stores.  Each lane-iteration ("item") makes P random 16-byte probes of the
// 2 MiB table (L2 hits), reads the next 16 bytes of a 4 GiB input stream and
// writes 16 bytes of an output stream.  One JSON line per P:
// {"mode": "stream", "probes_per_item", "gitems_per_s", "gprobes_per_s",
//  "stream_gbs"} — bench.py prices a kernel with h L2 hits and b stream
// bytes per header at rate(P = h / (b / 32)) items of 32 stream bytes.
//
//   hipcc --offload-arch=gfx950 -O3 -o ubench_mix scripts/ubench_mix.hip
//   ./ubench_mix; ./ubench_mix stream
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <string>
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

// stream mode: P probes per item, the item's stream word prefetched one
// iteration ahead (as the classify kernels' next-step header loads)
template <int P>
__global__ __launch_bounds__(1024) void k_stream(const uint4 *small, uint32_t smask,
                                                 const uint4 *in, uint4 *out, uint64_t items,
                                                 uint32_t *sink)
{
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 1024;
    uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    uint4 nx = i < items ? in[i] : make_uint4(0, 0, 0, 0);
    for (; i < items; i += stride) {
        const uint4 cur = nx;
        if (i + stride < items)
            nx = in[i + stride];
        uint4 v[P > 0 ? P : 1];
#pragma unroll
        for (int j = 0; j < P; j++)
            v[j] = small[mix(cur.x ^ (uint32_t)(j * 0x9E3779B9u) ^ (uint32_t)i) & smask];
        uint32_t x = cur.y;
#pragma unroll
        for (int j = 0; j < P; j++)
            x += v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
        out[i] = make_uint4(x, cur.z, cur.w, x ^ cur.x);
        acc += x;
    }
    if (acc == 0x12345678u)
        sink[0] = acc;
}

template <int P>
double stream_rate(const uint4 *small, uint32_t smask, const uint4 *in, uint4 *out,
                   uint64_t items, uint32_t *sink, int grid)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    float best = 1e30f;
    for (int rep = 0; rep < 4; rep++) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_stream<P>, dim3(grid), dim3(1024), 0, 0, small, smask, in, out,
                           items, sink);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (rep)
            best = ms < best ? ms : best;
    }
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return (double)items / (best * 1e-3) / 1e9;
}

int stream_main(int cus)
{
    const size_t sbytes = 2ull << 20, ibytes = 4ull << 30;
    const uint64_t items = ibytes / 16;
    uint4 *small, *in, *out;
    uint32_t *sink;
    CHECK(hipMalloc(&small, sbytes));
    CHECK(hipMalloc(&in, ibytes));
    CHECK(hipMalloc(&out, ibytes));
    CHECK(hipMalloc(&sink, 4));
    CHECK(hipMemset(small, 1, sbytes));
    CHECK(hipMemset(in, 3, ibytes));
    const uint32_t smask = (uint32_t)(sbytes / 16 - 1);
    const int grid = cus * 8;
    auto line = [&](int p, double r) {
        printf("{\"mode\": \"stream\", \"probes_per_item\": %d, \"gitems_per_s\": %.3f, "
               "\"gprobes_per_s\": %.2f, \"stream_gbs\": %.1f}\n",
               p, r, r * p, r * 32.0);
    };
    line(0, stream_rate<0>(small, smask, in, out, items, sink, grid));
    line(1, stream_rate<1>(small, smask, in, out, items, sink, grid));
    line(2, stream_rate<2>(small, smask, in, out, items, sink, grid));
    line(3, stream_rate<3>(small, smask, in, out, items, sink, grid));
    line(4, stream_rate<4>(small, smask, in, out, items, sink, grid));
    line(6, stream_rate<6>(small, smask, in, out, items, sink, grid));
    line(8, stream_rate<8>(small, smask, in, out, items, sink, grid));
    line(12, stream_rate<12>(small, smask, in, out, items, sink, grid));
    line(16, stream_rate<16>(small, smask, in, out, items, sink, grid));
    return 0;
}

int main(int argc, char **argv)
{
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    if (argc > 1 && std::string(argv[1]) == "stream")
        return stream_main(cus);
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
