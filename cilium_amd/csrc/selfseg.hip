// Traffic to itself in an egress batch (gfx950): the headers whose
// destination is the sending endpoint's own address, or a service that may
// loop back into it.
//
// An egress batch is one endpoint's packets.  Its two CT stages write keys
// of one direction each (the sender's ct_create writes TUPLE_F_OUT, the
// local destination's TUPLE_F_IN; conntrack.h:487-494, 691-772), and a
// stage's k1 carries the other flag — so a write of the batch is a later
// header's k1 only on a key whose two addresses are the sender's own: an
// endpoint talking to itself (the answer's egress lookup finds the entry
// the opening packet's ingress stage created: CT_REPLY), and a looped-back
// service flow's TUPLE_F_IN entry (:725-748, found by the endpoint's
// answers to IPV4_LOOPBACK).  Such a header's result, verdict and counters
// depend on the headers before it, which one parallel launch cannot see.
// k_self_mark lists those headers (one row each: index, L4 word, meta, the
// address it matched); cfc_classify cuts the batch before each one whose
// keys an earlier listed header of its segment may have written, and runs
// the segments in order, each folded into CT before the next is classified
// (cfc_api.cpp self_cuts).  A batch without such a pair is one launch.
#include <hip/hip_runtime.h>

#include "classify.hpp"

namespace cfc {

namespace {

template <bool V6>
__global__ __launch_bounds__(256) void k_self_mark(SelfArgs A)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < A.n;
         i += (uint64_t)gridDim.x * 256) {
        uint32_t k = ~0u;
        if constexpr (V6) {
            const uint4 d = reinterpret_cast<const uint4 *>(A.daddr)[i];
            for (uint32_t j = 0; j < A.na; j++) {
                const uint4 a = reinterpret_cast<const uint4 *>(A.addrs)[j];
                if (d.x == a.x && d.y == a.y && d.z == a.z && d.w == a.w) {
                    k = j;
                    break;
                }
            }
        } else {
            const uint32_t d = reinterpret_cast<const uint32_t *>(A.daddr)[i];
            for (uint32_t j = 0; j < A.na; j++)
                if (d == A.addrs[j]) {
                    k = j;
                    break;
                }
        }
        // one atomic per wave for the list places
        const bool want = k != ~0u;
        const uint64_t b = __ballot(want);
        if (!b)
            continue;
        const uint32_t lane = __lane_id();
        const uint32_t leader = (uint32_t)__ffsll((unsigned long long)b) - 1;
        uint32_t base = 0;
        if (lane == leader)
            base = atomicAdd(A.cnt, (uint32_t)__popcll(b));
        base = __shfl(base, (int)leader);
        if (want) {
            const uint32_t r = base + (uint32_t)__popcll(b & ((1ull << lane) - 1));
            if (r < A.cap)
                A.rows[r] = make_uint4((uint32_t)i, A.pt[i], A.mt[i], k);
        }
    }
}

}  // namespace

int self_mark(const SelfArgs &A, bool v6, hipStream_t s)
{
    if (!A.n || !A.na)
        return 0;
    const uint64_t blocks = std::min<uint64_t>((A.n + 255) / 256, 8192);
    const dim3 g((unsigned)blocks);
    if (v6)
        hipLaunchKernelGGL(k_self_mark<true>, g, dim3(256), 0, s, A);
    else
        hipLaunchKernelGGL(k_self_mark<false>, g, dim3(256), 0, s, A);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

}  // namespace cfc
