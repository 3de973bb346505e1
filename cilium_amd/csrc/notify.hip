// Monitor events of a classified batch: struct drop_notify records
// (bpf/lib/drop.h:40-78) and struct trace_notify records (trace.h:71-81,
// send_trace_notify :97-155) in header order.
//
// The reference emits one perf-ring sample per dropped packet from
// __send_drop_notify, a tail call armed by send_drop_notify (drop.h:94-109)
// with cb[1] = src << 16 | dst & 0xFFFF, cb[2] = reason, cb[3] = dst_id,
// cb[4] = ifindex.  The classify kernels record which call site ran
// (cfc_out.notify, kern_common.hpp notify_word); here the site words are
// stream-compacted: per-block counts, one scan block, then each block writes
// its records at its offset.  HBM-bound: 4 B notify + 8 B verdict/identity
// per header read, plus 32 B per record and the hash inputs of dropped
// headers only.
#include <cerrno>

#include "kern_common.hpp"

namespace cfc {

namespace {

constexpr int NT_THREADS = 256;
constexpr int NT_ITERS = 16;   // rounds of NT_THREADS headers per block
constexpr uint64_t NT_PER_BLOCK = (uint64_t)NT_THREADS * NT_ITERS;

__device__ __forceinline__ uint32_t fold6(const uint32_t *w)
{
    uint32_t h = fmix32(w[3]);
    h = fmix32(w[2] ^ h);
    h = fmix32(w[1] ^ h);
    return fmix32(w[0] ^ h);
}

// symmetric 5-tuple hash (oracle/oracle.py flow_hash)
// skb->len of the event's packet: after a NAT hop (CFC_NT_NATLEN) the
// translated one — IPv4's header 20 bytes shorter (nat46.h:236-420)
__device__ __forceinline__ uint32_t rec_len(const NotifyArgs &a, uint64_t i, uint32_t w)
{
    const uint32_t len = a.meta[i] >> 16;
    return (w & CFC_NT_NATLEN) ? (a.family == 4 ? len + 20u : len - 20u) : len;
}
__device__ __forceinline__ uint32_t flow_hash(const NotifyArgs &a, uint64_t i)
{
    if (a.hash)   // the batch's skb->hash
        return a.hash[i];
    uint32_t x, y;
    if (a.family == 4) {
        x = a.saddr[i];
        y = a.daddr[i];
    } else {
        x = fold6(a.saddr + 4 * i);
        y = fold6(a.daddr + 4 * i);
    }
    const uint32_t lo = min(x, y), hi = max(x, y);
    const uint32_t pt = a.ports[i];
    const uint32_t sp = pt & 0xFFFF, dp = pt >> 16;
    const uint32_t pw = min(sp, dp) | (max(sp, dp) << 16);
    const uint32_t proto = a.meta[i] & 0xFF;
    return fmix32(lo * 0x9E3779B1u + hi * 0x85EBCA77u + pw * 0xC2B2AE3Du + proto);
}

// the events a call records: drops (kinds 1-3), and traces when asked
__device__ __forceinline__ bool nt_selected(uint32_t w, int traces)
{
    // (a trace whose monitor length is 0 is not sent: trace.h:119-132)
    const uint32_t kind = (w >> 16) & 0xF;
    return w != 0 && (kind < CFC_NT_TRACE || (traces && ((w >> 22) & 3) != 0));
}

__global__ __launch_bounds__(NT_THREADS) void k_nt_count(const uint32_t *notify,
                                                         uint64_t n, int traces,
                                                         uint64_t *blk)
{
    const uint64_t base = (uint64_t)blockIdx.x * NT_PER_BLOCK;
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < NT_ITERS; r++) {
        const uint64_t i = base + (uint64_t)r * NT_THREADS + threadIdx.x;
        c += (i < n && nt_selected(ld_nt(notify + i), traces)) ? 1u : 0u;
    }
    // wave sums, then the block's
    for (int o = 32; o > 0; o >>= 1)
        c += __shfl_xor(c, o);
    __shared__ uint32_t s[NT_THREADS / 64];
    if ((threadIdx.x & 63) == 0)
        s[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < NT_THREADS / 64; w++)
            t += s[w];
        blk[blockIdx.x] = t;
    }
}

// exclusive scan of nb block counts in place (one 1024-thread block), total
// into *count
__global__ __launch_bounds__(1024) void k_nt_scan(uint64_t *blk, uint64_t nb,
                                                  uint64_t *count)
{
    __shared__ uint64_t s[1024];
    const uint64_t per = (nb + 1023) / 1024;
    const uint64_t b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
    uint64_t sum = 0;
    for (uint64_t b = b0; b < b1; b++)
        sum += blk[b];
    s[threadIdx.x] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint64_t v = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0;
        __syncthreads();
        s[threadIdx.x] += v;
        __syncthreads();
    }
    uint64_t run = s[threadIdx.x] - sum;   // exclusive prefix of this chunk
    for (uint64_t b = b0; b < b1; b++) {
        const uint64_t v = blk[b];
        blk[b] = run;
        run += v;
    }
    if (threadIdx.x == 1023)
        *count = s[1023];
}

__global__ __launch_bounds__(NT_THREADS) void k_nt_write(NotifyArgs a,
                                                         const uint64_t *blk)
{
    __shared__ uint32_t s[NT_THREADS / 64];
    const uint64_t base = (uint64_t)blockIdx.x * NT_PER_BLOCK;
    uint64_t off = blk[blockIdx.x];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int r = 0; r < NT_ITERS; r++) {
        const uint64_t i = base + (uint64_t)r * NT_THREADS + threadIdx.x;
        uint32_t w = i < a.n ? ld_nt(a.notify + i) : 0u;
        w = nt_selected(w, a.traces) ? w : 0u;
        const uint64_t m = __ballot(w != 0);
        const uint32_t below = __popcll(m & ((1ull << lane) - 1));
        if (lane == 0)
            s[wave] = __popcll(m);
        __syncthreads();
        uint32_t before = 0, total = 0;
        for (int v = 0; v < NT_THREADS / 64; v++) {
            before += v < wave ? s[v] : 0u;
            total += s[v];
        }
        const uint64_t pos = off + before + below;
        if (w && pos < a.cap && ((w >> 16) & 0xF) >= CFC_NT_TRACE) {
            // trace_notify: src/dst labels in full (trace.h:137-151)
            const uint32_t obs = ((w >> 16) & 0xF) - CFC_NT_TRACE, lxc = w & 0xFFFF;
            const uint32_t reason = (w >> 20) & 3;
            const uint32_t mc = (w >> 22) & 3;   // TRACE_PAYLOAD_LEN / MTU / 1
            const uint32_t mon = mc == 2 ? MTU_LEN : mc == 3 ? 1u : TRACE_PAYLOAD_LEN;
            const uint32_t ident = a.identity[i];
            const uint32_t len = rec_len(a, i, w);
            const uint2 e = a.ep_info[lxc];
            uint32_t src = e.x, dst = 0, dst_id = 0, ifx = 0;
            if (obs == OBS_TO_LXC) {   // the destination's ipv{4,6}_policy
                src = a.mode == CFC_MODE_EGRESS ? a.own_seclabel : ident;
                dst = e.x;
                dst_id = lxc;
                ifx = e.y;
            } else if (obs == OBS_TO_PROXY) {
                ifx = a.host_ifindex;
            } else if (obs == OBS_TO_HOST) {
                dst = 1;   // HOST_ID
                ifx = a.host_ifindex;
            } else {   // TO_STACK: the destination identity
                dst = ident;
            }
            const uint32_t w0 = CFC_NOTIFY_TRACE | obs << 8 | lxc << 16;
            uint4 *p = reinterpret_cast<uint4 *>(a.rec) + 2 * pos;
            p[0] = make_uint4(w0, flow_hash(a, i), len, min(len, mon));
            p[1] = make_uint4(src, dst, dst_id | reason << 16, ifx);
            if (a.hdr_index)
                a.hdr_index[pos] = i;
        } else if (w && pos < a.cap) {
            const uint32_t site = (w >> 16) & 0xF, lxc = w & 0xFFFF;
            const int ver = a.verdict[i];
            const uint32_t ident = a.identity[i];
            const uint32_t len = rec_len(a, i, w);
            uint32_t src = 0, dst = 0, dst_id = 0, ifx = 0, source = 0;
            if (site == CFC_NT_EGRESS) {
                source = lxc;
                src = a.own_seclabel;
                dst = ident;
            } else if (site == CFC_NT_POLICY) {
                const uint2 e = a.ep_info[lxc];
                source = lxc;
                src = a.mode == CFC_MODE_EGRESS ? a.own_seclabel : ident;
                dst = e.x;
                dst_id = lxc;
                ifx = e.y;
            }
            const uint32_t w0 = CFC_NOTIFY_DROP | (((uint32_t)(-ver) & 0xFF) << 8) |
                                (source << 16);
            uint4 *p = reinterpret_cast<uint4 *>(a.rec) + 2 * pos;
            p[0] = make_uint4(w0, flow_hash(a, i), len,
                              min(len, (uint32_t)CFC_TRACE_PAYLOAD_LEN));

            p[1] = make_uint4(src & 0xFFFF, dst & 0xFFFF, dst_id, ifx);
            if (a.hdr_index)
                a.hdr_index[pos] = i;
        }
        off += total;
        __syncthreads();
    }
}

}  // namespace

size_t drop_notify_workspace_bytes(uint64_t n)
{
    return 8 * ((n + NT_PER_BLOCK - 1) / NT_PER_BLOCK + 1);
}

int launch_drop_notify(const NotifyArgs &a, uint64_t *ws, hipStream_t s)
{
    if (a.n == 0) {
        return hipMemsetAsync(a.count, 0, 8, s) == hipSuccess ? 0 : -EINVAL;
    }
    const uint64_t nb = (a.n + NT_PER_BLOCK - 1) / NT_PER_BLOCK;
    if (nb > 0x7FFFFFFFull)
        return -E2BIG;
    k_nt_count<<<(uint32_t)nb, NT_THREADS, 0, s>>>(a.notify, a.n, a.traces, ws);
    k_nt_scan<<<1, 1024, 0, s>>>(ws, nb, a.count);
    k_nt_write<<<(uint32_t)nb, NT_THREADS, 0, s>>>(a, ws);
    return hipGetLastError() == hipSuccess ? 0 : -EINVAL;
}

}  // namespace cfc
