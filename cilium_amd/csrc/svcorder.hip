// The service step of an egress batch in packet order (gfx950), ahead of the
// classify launch.
//
// The reference runs lb4_local / lb6_local one packet at a time
// (bpf_lxc.c:476-492, 149-167).  The first packet of a flow to a service
// finds no CT_SERVICE entry: it selects a backend from its skb->hash
// (lb4_select_slave, lb.h:711-716) and creates the entry with that slave;
// every later packet of the flow takes the stored slave (:723-726), whatever
// its own hash.  A packet whose slave's backend is gone re-selects from its
// own hash through the fall-back service and stores that
// (ct_update4_slave, :737-744).  The service lookups themselves depend only
// on the table and the entry's key, so per CT_SERVICE key the only state
// that passes from packet to packet is the entry: (exists, slave).
//
// Which headers can see an entry other than the batch start's: those of a
// key whose entry is missing at the start (the first one creates it) or
// whose stored slave's backend is gone (the first one re-selects).  A key
// whose entry exists with a live backend stays as it is for the whole batch.
// k_svo_mark lists the others, keyed (entry fingerprint, header order); one
// sort; k_svo_replay walks each entry's headers in order, handing each the
// entry as the ones before it left it (svo).  The classify launch's service
// step (lb.hip, classify6.hip lb6_egress) reads that instead of the table.
// cfc_ct_apply later replays the same per key for the CT writes
// (ctapply.hip k_cta_svc).
#include <hipcub/hipcub.hpp>

#include "ctops.hpp"

namespace cfc {

namespace {

// the header reaches lb4_local / lb6_local with a service (the egress path's
// gates before it: a valid source, bpf_lxc.c:464-469 / lxc.h:46; TCP, UDP
// or ICMP(v6), lb4/6_extract_key; IPv6: not an ICMPv6 the router answers,
// icmp6_handle); e: the CT_SERVICE entry as the batch found it; stable:
// it exists and its slave's backend is there (no header changes it)
template <bool V6>
__device__ __forceinline__ bool svo_reach(const DevTables &T, const SvoArgs &A, uint64_t i,
                                          Addr<V6> &sa, Addr<V6> &da, uint32_t &z, uint32_t &w,
                                          SvcEntry &e, bool &stable)
{
    sa = ld_addr<V6>(A.sa, i);
    da = ld_addr<V6>(A.da, i);
    const uint32_t pt = A.pt[i], mt = A.mt[i], proto = mt & 0xFF;
    const bool l4 = proto == 6 || proto == 17;
    if (!l4 && proto != icmp_proto<V6>())
        return false;
    uint32_t kd = l4 ? pt >> 16 : 0u;
    uint32_t slot;
    const CtProbe k = ct_probe<V6>(proto, pt, CT_SERVICE, A.ct_owner);
    z = k.z1;
    w = k.w1;
    if constexpr (V6) {
        if (icmp6_punt(T, proto, mt, pt, bswap4(da)))
            return false;
        uint4 b, tg;
        if (!lb6_src_ok(T, sa, A.lxc_id) || !lb6_service(T, da, kd, 0, b, tg))
            return false;
        slot = ct6_find(T, da, sa, z, w);
        e.exists = slot != NONE;
        e.slave = (e.exists && T.ct6_lb) ? ld16(T.ct6_lb + slot).y : 0u;
        e.loop = 0;
        stable = e.exists && lb6_get(T, da, kd, e.slave, b, tg);
    } else {
        uint4 a, b;
        if (!lb4_src_ok(T, sa, A.lxc_id) || !lb4_service(T, da, kd, 0, a, b))
            return false;
        slot = ct4_find(T, da, sa, z, w);
        e.exists = slot != NONE;
        const uint4 lw = (e.exists && T.ct4_lb) ? ld16(T.ct4_lb + slot) : make_uint4(0, 0, 0, 0);
        e.slave = lw.y;
        e.loop = (lw.x >> 16) & 1;
        stable = e.exists && lb4_get(T, da, kd, e.slave, a, b);
    }
    return true;
}

__device__ __forceinline__ uint32_t fhash(uint32_t sa, uint32_t da, uint32_t pt, uint32_t proto)
{
    return flow_hash4(sa, da, pt, proto);
}
__device__ __forceinline__ uint32_t fhash(uint4 sa, uint4 da, uint32_t pt, uint32_t proto)
{
    return flow_hash6(sa, da, pt, proto);
}

// one thread per header: the headers of keys a batch header may change
template <bool V6>
__global__ __launch_bounds__(256) void k_svo_mark(DevTables T, SvoArgs A)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    bool want = false;
    uint64_t key = 0;
    if (i < A.n) {
        Addr<V6> sa, da;
        uint32_t z, w;
        SvcEntry e;
        bool stable = true;
        want = svo_reach<V6>(T, A, i, sa, da, z, w, e, stable) && !stable;
        key = (uint64_t)khash(da, sa, z, w) << 32 | (uint32_t)i;
    }
    const uint32_t r = block_count(A.cnt, want);
    if (want)
        A.keys[r] = key;
}

// one thread per run of equal fingerprints in the sorted list: per key in
// it, its headers in order, each handed the entry as the ones before it
// left it (the first finds the batch start's).  done[r]: list entry r was
// handled with an earlier entry's key.
template <bool V6>
__global__ __launch_bounds__(256) void k_svo_replay(DevTables T, SvoArgs A, const uint64_t *keys,
                                                    uint64_t *done, uint32_t m)
{
    const uint32_t r0 = blockIdx.x * 256 + threadIdx.x;
    if (r0 >= m)
        return;
    const uint32_t fp = (uint32_t)(keys[r0] >> 32);
    if (r0 > 0 && (uint32_t)(keys[r0 - 1] >> 32) == fp)
        return;
    uint32_t wrote = 0;   // entry words handed to later headers (cfc_stats.svc_ordered)
    for (uint32_t r = r0; r < m && (uint32_t)(keys[r] >> 32) == fp; r++) {
        if (done[r])
            continue;
        const uint64_t i = (uint32_t)keys[r];
        Addr<V6> sa, da;
        uint32_t z, w;
        SvcEntry e;
        bool stable;
        (void)svo_reach<V6>(T, A, i, sa, da, z, w, e, stable);
        const uint32_t pt = A.pt[i], proto = A.mt[i] & 0xFF;
        const uint32_t h0 = A.hash ? A.hash[i] : fhash(sa, da, pt, proto);
        if constexpr (V6)
            svc_next6(T, da, pt, proto, h0, e);
        else
            svc_next4(T, da, pt, proto, h0, e);
        for (uint32_t q = r + 1; q < m && (uint32_t)(keys[q] >> 32) == fp; q++) {
            if (done[q])
                continue;
            const uint64_t j = (uint32_t)keys[q];
            const Addr<V6> sj = ld_addr<V6>(A.sa, j), dj = ld_addr<V6>(A.da, j);
            const uint32_t ptj = A.pt[j], protoj = A.mt[j] & 0xFF;
            const CtProbe k = ct_probe<V6>(protoj, ptj, CT_SERVICE, A.ct_owner);
            if (k.z1 != z || k.w1 != w || !aeq(sj, sa) || !aeq(dj, da))
                continue;   // (a fingerprint collision: another key)
            done[q] = 1;
            A.svo[j] = svo_word(e);
            wrote++;
            const uint32_t hj = A.hash ? A.hash[j] : fhash(sj, dj, ptj, protoj);
            if constexpr (V6)
                svc_next6(T, dj, ptj, protoj, hj, e);
            else
                svc_next4(T, dj, ptj, protoj, hj, e);
        }
    }
    if (wrote)   // (cnt words 2-3: a running total the host reads for its stats)
        atomicAdd(reinterpret_cast<unsigned long long *>(A.cnt + 2), (unsigned long long)wrote);
}

}  // namespace

size_t svc_order_tmp_bytes(uint64_t n)
{
    size_t t = 0;
    hipcub::DoubleBuffer<uint64_t> k(nullptr, nullptr);
    (void)hipcub::DeviceRadixSort::SortKeys(nullptr, t, k, (int)std::max<uint64_t>(n, 1), 0, 64);
    return t;
}

int svc_order(const DevTables &T, const SvoArgs &A, bool v6, uint32_t *count, hipStream_t s)
{
    *count = 0;
    if (!A.n)
        return 0;
    if (A.n >= (1ull << 31))
        return -E2BIG;
    if (hipMemsetAsync(A.cnt, 0, 4, s) != hipSuccess)
        return -EIO;
    const dim3 g((unsigned)((A.n + 255) / 256));
    if (v6)
        hipLaunchKernelGGL(k_svo_mark<true>, g, dim3(256), 0, s, T, A);
    else
        hipLaunchKernelGGL(k_svo_mark<false>, g, dim3(256), 0, s, T, A);
    // (the list's length sizes the sort: the one host wait of the pass, on
    // egress batches with services only)
    uint32_t m = 0;
    if (hipMemcpyAsync(&m, A.cnt, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    if (m > A.n)
        return -EIO;
    *count = m;
    if (!m)
        return 0;
    size_t tb = A.tmp_bytes;
    hipcub::DoubleBuffer<uint64_t> kb(A.keys, A.keys2);
    if (hipcub::DeviceRadixSort::SortKeys(A.tmp, tb, kb, (int)m, 0, 64, s) != hipSuccess)
        return -EIO;
    // the other buffer holds the done marks (one u64 per entry)
    uint64_t *done = kb.Current() == A.keys ? A.keys2 : A.keys;
    if (hipMemsetAsync(done, 0, 8ull * m, s) != hipSuccess)
        return -EIO;
    const dim3 gr((m + 255) / 256);
    if (v6)
        hipLaunchKernelGGL(k_svo_replay<true>, gr, dim3(256), 0, s, T, A, kb.Current(), done, m);
    else
        hipLaunchKernelGGL(k_svo_replay<false>, gr, dim3(256), 0, s, T, A, kb.Current(), done, m);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

}  // namespace cfc
