// Batched verdict kernels for gfx950 (MI355X).
//
// Shape.  A 1024-thread workgroup owns a contiguous slice of <= 65536 headers
// of the SoA batch; each loop iteration reads 4 KiB of every input array
// coalesced (non-temporal: the 1-GiB stream must not evict the lookup tables
// from the 256-MiB Infinity Cache) and writes the outputs the same way.
//
// Latency.  The lookups are dependent random accesses — DIR-24-8 tbl24/tbl8
// (Infinity Cache), the endpoint / prefilter / policy buckets (L2).  The
// kernel is bound by how many of them are in flight, so each header's chain
// is cut to four memory round trips by issuing every lookup as soon as its
// inputs exist:
//   1. inputs
//   2. tbl24[src|dst], endpoint bucket[dst], prefilter bucket[src]  (together)
//   3. tbl8 (if the /24 is split), endpoint record
//   4. the three policy buckets of __policy_can_access (L4, L3, wildcard-port)
//      loaded speculatively together, resolved in the reference's order.
// Overflowing buckets (never at the load factors flatten.cpp builds) fall
// back to a probing loop.  There is no contraction here, hence no MFMA.
//
// Counters.  The reference bumps policy_entry packets/bytes
// (policy.h:68-69,80-81,92-93) and cilium_metrics (metrics.h:43-61) per
// packet.  Here they are exact u32 sums in LDS (a workgroup sees at most
// 65536 headers, so neither packets nor bytes can wrap), written once per
// workgroup as a partial slab and summed per entry by k_reduce_partials.
// Metrics keys are few and hot (most packets of a batch share one drop
// reason), so they are aggregated across the wave before the LDS atomic.
//
// Reference semantics restated here (file:line in /root/reference):
//   ingress   bpf_netdev.c:128-153 (FROM_HOST identity from skb->mark),
//             :357-453 handle_ipv4, l3.h:103-131 ipv4_local_delivery,
//             bpf_lxc.c:898-1028 ipv4_policy + tail_ipv4_policy
//   egress    bpf_lxc.c:440-704 handle_ipv4_from_lxc
//   policy    bpf/lib/policy.h:46-146
//   ct ports  bpf/lib/conntrack.h:467-590 (tuple->dport of a CT_NEW lookup)
//   xdp       bpf_xdp.c:88-121
#include "classify.hpp"

namespace cfc {

namespace {

constexpr uint32_t HOST_ID = 1, WORLD_ID = 2, CLUSTER_ID = 3, HEALTH_ID = 4;
constexpr uint32_t IPV4_CLUSTER_MASK = 0xff0000u, IPV4_CLUSTER_RANGE = 0x100000u;
constexpr int DROP_INVALID_SIP = -132, DROP_POLICY = -133,
              DROP_CT_UNKNOWN_PROTO = -137, DROP_MISSED_TAIL_CALL = -140;
constexpr int TC_ACT_OK = 0, TC_ACT_SHOT = 2, TC_ACT_REDIRECT = 7;
constexpr int XDP_DROP = 1, XDP_PASS = 2;
constexpr int METRIC_INGRESS = 1, METRIC_EGRESS = 2;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint64_t MAX_PER_BLOCK = 65536;   // keeps u32 LDS sums exact
#ifndef CFC_UNROLL
#define CFC_UNROLL 2   // headers in flight per thread
#endif

template <class T>
__device__ __forceinline__ T ld_nt(const T *p)
{
    return __builtin_nontemporal_load(p);
}
template <class T>
__device__ __forceinline__ void st_nt(T v, T *p)
{
    __builtin_nontemporal_store(v, p);
}

__device__ __forceinline__ uint4 ld16(const void *p)
{
    return *reinterpret_cast<const uint4 *>(p);
}

// ---- endpoint lookup: 16-byte slots, linear probing (layout.h)
// resolve from the first loaded slot; returns the slot (info VALID) or a
// zero slot for a miss
__device__ __forceinline__ uint4 lxc_resolve(const DevTables &T, uint32_t addr,
                                             uint32_t s, uint4 v)
{
    for (;;) {
        if (!(v.w & LXC_VALID))
            return make_uint4(0, 0, 0, 0);
        if (v.x == addr)
            return v;
        s = (s + 1) & T.lxc4_mask;
        v = ld16(T.lxc4 + s);
    }
}

// ---- prefilter /32 set: 16-byte buckets of 4 addresses, 0 = free
__device__ __forceinline__ bool pf_resolve(const DevTables &T, uint32_t addr,
                                           uint32_t b, uint4 v)
{
    if (addr == 0)
        return T.pf_fix_zero != 0;
    for (;;) {
        if (v.x == addr || v.y == addr || v.z == addr || v.w == addr)
            return true;
        if (!v.x || !v.y || !v.z || !v.w)
            return false;
        b = (b + 1) & T.pf_fix_mask;
        v = ld16(T.pf_fix + (size_t)b * PF_SLOTS);
    }
}

__device__ __forceinline__ uint64_t pkey(uint32_t id, uint32_t dport,
                                         uint32_t proto, uint32_t egress)
{
    return (uint64_t)id | ((uint64_t)dport << 32) | ((uint64_t)proto << 48) |
           ((uint64_t)egress << 56);
}

// tuple->dport of a CT_NEW lookup (conntrack.h:496-584): TCP/UDP ports are
// loaded swapped and swapped back by ipv4_ct_tuple_reverse(); ICMP echo puts
// its type (8) in tuple->sport, which becomes the dport; other ICMP -> 0;
// any other protocol -> DROP_CT_UNKNOWN_PROTO.
__device__ __forceinline__ bool ct_new_dport(uint32_t proto, uint32_t ports,
                                             uint32_t *dport)
{
    if (proto == 6 || proto == 17) {
        *dport = ports >> 16;
        return true;
    }
    *dport = (ports & 0xFF) == 8 ? 8u : 0u;
    return proto == 1;
}

// __policy_can_access (policy.h:46-110), cb[CB_POLICY] == 0: the first
// slot of each of the three keys (L4, L3, wildcard port) is loaded at once,
// then the keys are resolved in the reference's order.  Returns the verdict
// (<0 drop) and the matched counter (or NONE).
struct PolicyProbe {
    uint64_t k[3];
    uint32_t s[3];
    uint4 v[3];
};

__device__ __forceinline__ void policy_issue(const DevTables &T, uint32_t base,
                                             uint32_t mask, uint32_t id,
                                             uint32_t dport, uint32_t proto,
                                             uint32_t egress, PolicyProbe &P)
{
    P.k[0] = pkey(id, dport, proto, egress);   // L4
    P.k[1] = pkey(id, 0, 0, egress);           // L3
    P.k[2] = pkey(0, dport, proto, egress);    // wildcard port
#pragma unroll
    for (int j = 0; j < 3; j++) {
        P.s[j] = hash64(P.k[j], mask);
        P.v[j] = ld16(T.pol + base + P.s[j]);
    }
}

__device__ __forceinline__ int policy_resolve(const DevTables &T, uint32_t base,
                                              uint32_t mask, bool frag,
                                              const PolicyProbe &P,
                                              uint32_t *ctr)
{
#pragma unroll
    for (int j = 0; j < 3; j++) {
        if (frag && j != 1)   // fragments: L3 key only (policy.h:61,85)
            continue;
        uint4 v = P.v[j];
        uint32_t s = P.s[j];
        for (;;) {
            const uint64_t key = ((uint64_t)v.y << 32) | v.x;
            if (key == P.k[j]) {
                *ctr = v.w;
                return j == 1 ? TC_ACT_OK : (int)(v.z & 0xFFFF);
            }
            if (key == POL_EMPTY)
                break;
            s = (s + 1) & mask;
            v = ld16(T.pol + base + s);
        }
    }
    *ctr = NONE;
    return DROP_POLICY;   // (DROP_FRAG_NOSUPPORT also becomes DROP_POLICY)
}

__device__ __forceinline__ int policy_access(const DevTables &T, uint32_t base,
                                             uint32_t mask, uint32_t id,
                                             uint32_t dport, uint32_t proto,
                                             uint32_t egress, bool frag,
                                             uint32_t *ctr)
{
    PolicyProbe P;
    policy_issue(T, base, mask, id, dport, proto, egress, P);
    return policy_resolve(T, base, mask, frag, P, ctr);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o);
    return v;
}

// update_metrics for every lane of the wave at once: key = index into the
// metrics block ([reason][dir][count,bytes]) or NONE.  Must be reached by
// the whole wave (uniform control flow).
__device__ __forceinline__ void metrics_wave(uint32_t *s_met, uint64_t *g_met,
                                             uint32_t key, uint32_t len)
{
    uint64_t pending = __ballot(key != NONE);
    const int lane = threadIdx.x & 63;
    while (pending) {
        const int leader = __ffsll((long long)pending) - 1;
        const uint32_t lk = __shfl(key, leader);
        const bool mine = key == lk;
        const uint64_t m = __ballot(mine);
        const uint32_t sum = wave_sum(mine ? len : 0u);
        if (lane == leader) {
            if (s_met) {
                atomicAdd(&s_met[lk], (uint32_t)__popcll(m));
                atomicAdd(&s_met[lk + 1], sum);
            } else {
                atomicAdd((unsigned long long *)&g_met[lk],
                          (unsigned long long)__popcll(m));
                atomicAdd((unsigned long long *)&g_met[lk + 1],
                          (unsigned long long)sum);
            }
        }
        pending &= ~m;
    }
}

__device__ __forceinline__ uint32_t mkey(int reason, int dir)
{
    return ((uint32_t)(uint8_t)(-reason) * METRIC_DIRS + (uint32_t)dir) * 2;
}

template <bool LDS>
__device__ __forceinline__ void count_hit(uint32_t *s_ctr, uint64_t *g_ctr,
                                          uint32_t c, uint32_t len)
{
    if (c == NONE)
        return;
    if (LDS) {
        atomicAdd(&s_ctr[2 * c], 1u);
        atomicAdd(&s_ctr[2 * c + 1], len);
    } else {
        atomicAdd((unsigned long long *)&g_ctr[2 * c], 1ull);
        atomicAdd((unsigned long long *)&g_ctr[2 * c + 1], (unsigned long long)len);
    }
}

// Per-header state carried through the lookup rounds.
struct Hdr {
    uint32_t sa, da, pt, mt, mk;
    bool valid;
    uint32_t e24, pfd, lh, hsh, lxs, lss, pfb;
    uint4 lx, ls, pf, rec;
    uint32_t src_lxc;
    int act, ver;
    uint32_t ident, met0, met1, ctr0, ctr1;
    bool xdp_drop, need_pol, skip_proxy;
    uint32_t pbase, pmask, egress_bit, dport;
    PolicyProbe P;
};

// round 1: the header (non-temporal streaming loads)
template <int MODE>
__device__ __forceinline__ void r1_load(const cfc_hdr_v4 &in, uint64_t i,
                                        uint64_t end, Hdr &h)
{
    h.valid = i < end;
    h.sa = h.da = h.pt = h.mt = h.mk = 0;
    if (h.valid) {
        h.sa = ld_nt(in.saddr + i);
        h.da = ld_nt(in.daddr + i);
        h.pt = ld_nt(in.ports + i);
        h.mt = ld_nt(in.meta + i);
        if (in.mark)
            h.mk = ld_nt(in.mark + i);
    }
}

// round 2: every lookup that only needs the header
template <int MODE>
__device__ __forceinline__ void r2_issue(const DevTables &T, Hdr &h)
{
    constexpr bool XDP = MODE == CFC_MODE_XDP || MODE == CFC_MODE_FULL;
    constexpr bool EGR = MODE == CFC_MODE_EGRESS;
    constexpr bool LPM = MODE != CFC_MODE_XDP;
    h.e24 = h.pfd = 0;
    h.lx = h.ls = h.pf = make_uint4(0, 0, 0, 0);
    h.lh = __builtin_bswap32(EGR ? h.da : h.sa);
    h.hsh = __builtin_bswap32(h.sa);
    h.lxs = h.lss = h.pfb = 0;
    if (!h.valid)
        return;
    if (LPM && T.tbl24)
        h.e24 = T.tbl24[h.lh >> 8];
    if (XDP && T.pf_tbl24)
        h.pfd = T.pf_tbl24[h.hsh >> 8];
    if (T.lxc4) {
        h.lxs = hash32(h.da, T.lxc4_mask);
        h.lx = ld16(T.lxc4 + h.lxs);
        if (EGR) {
            h.lss = hash32(h.sa, T.lxc4_mask);
            h.ls = ld16(T.lxc4 + h.lss);
        }
    }
    if (XDP && T.pf_fix) {
        h.pfb = hash32(h.sa, T.pf_fix_mask);
        h.pf = ld16(T.pf_fix + (size_t)h.pfb * PF_SLOTS);
    }
}

// round 3: second-level LPM, endpoint resolution, prefilter verdict,
// identity, and the first slot of the three policy keys
template <int MODE>
__device__ __forceinline__ void r3_identity(const DevTables &T,
                                            const EgressArgs &E, Hdr &h)
{
    constexpr bool XDP = MODE == CFC_MODE_XDP || MODE == CFC_MODE_FULL;
    constexpr bool EGR = MODE == CFC_MODE_EGRESS;
    if (h.e24 & LPM_GROUP)
        h.e24 = T.tbl8[((h.e24 & ~LPM_GROUP) << 8) | (h.lh & 0xFF)];
    if (h.e24 & LPM_INDIRECT)
        h.e24 = T.lbl_ovf[h.e24 & LPM_PAYLOAD];
    if (h.pfd & LPM_GROUP)
        h.pfd = T.pf_tbl8[((h.pfd & ~LPM_GROUP) << 8) | (h.hsh & 0xFF)];
    // rec: {addr, pol_base, pol_mask, info}; info == 0 -> not local
    h.rec = make_uint4(0, 0, 0, 0);
    uint4 srec = h.rec;
    if (h.valid && T.lxc4) {
        h.rec = lxc_resolve(T, h.da, h.lxs, h.lx);
        if (EGR)
            srec = lxc_resolve(T, h.sa, h.lss, h.ls);
    }
    const bool local = (h.rec.w & LXC_VALID) != 0;
    h.src_lxc = (srec.w & LXC_VALID) ? (srec.w & 0xFFFF) : NONE;

    h.act = TC_ACT_OK;
    h.ver = 0;
    h.ident = 0;
    h.met0 = h.met1 = h.ctr0 = h.ctr1 = NONE;
    h.xdp_drop = false;
    if (XDP && h.valid) {
        bool deny = h.pfd != 0;
        if (!deny && (T.pf_fix || T.pf_fix_zero))
            deny = pf_resolve(T, h.sa, h.pfb, h.pf);
        h.xdp_drop = deny || !local;
        if (MODE == CFC_MODE_XDP || h.xdp_drop) {
            h.act = h.xdp_drop ? XDP_DROP : XDP_PASS;
            h.ver = h.xdp_drop ? CFC_DROP_PREFILTER : 0;
        }
    }

    h.need_pol = h.skip_proxy = false;
    h.pbase = h.pmask = h.egress_bit = h.dport = 0;
    if (!h.valid || MODE == CFC_MODE_XDP || h.xdp_drop)
        return;
    const uint32_t proto = h.mt & 0xFF;
    const bool known = ct_new_dport(proto, h.pt, &h.dport);
    if (!EGR) {
        // handle_identity_from_host (bpf_netdev.c:128-153)
        const uint32_t magic = h.mk & 0xF00u;
        if (magic == 0xA00u || magic == 0xB00u) {
            h.ident = ((h.mk & 0xFF) << 16) | (h.mk >> 16);
            h.skip_proxy = magic == 0xA00u;
        } else {
            h.ident = magic == 0xC00u ? HOST_ID : WORLD_ID;
        }
        // handle_ipv4 (:375-398): reserved identities take the ipcache's
        if (h.ident < HEALTH_ID && h.e24 && h.e24 != CLUSTER_ID && h.e24 != HOST_ID)
            h.ident = h.e24;
        if (local && !(h.rec.w & LXC_HOST)) {
            if (!(h.rec.w & LXC_HAS_POLICY)) {
                h.act = TC_ACT_SHOT;
                h.ver = DROP_MISSED_TAIL_CALL;
                h.met0 = mkey(DROP_MISSED_TAIL_CALL, METRIC_INGRESS);
            } else if (!known) {
                h.act = TC_ACT_SHOT;
                h.ver = DROP_CT_UNKNOWN_PROTO;
                h.met0 = mkey(DROP_CT_UNKNOWN_PROTO, METRIC_INGRESS);
            } else {
                h.need_pol = true;
                h.pbase = h.rec.y;
                h.pmask = h.rec.z;
            }
        }
    } else {
        h.act = TC_ACT_SHOT;
        if (h.src_lxc != E.lxc_id) {   // is_valid_lxc_src_ipv4 (lxc.h:55)
            h.ver = DROP_INVALID_SIP;
            h.met0 = mkey(DROP_INVALID_SIP, METRIC_EGRESS);
        } else if (!known) {
            h.ver = DROP_CT_UNKNOWN_PROTO;
            h.met0 = mkey(DROP_CT_UNKNOWN_PROTO, METRIC_EGRESS);
        } else {
            // destination identity (bpf_lxc.c:516-532)
            h.ident = h.e24 ? h.e24
                            : ((h.da & IPV4_CLUSTER_MASK) == IPV4_CLUSTER_RANGE
                                   ? CLUSTER_ID
                                   : WORLD_ID);
            h.need_pol = true;
            h.pbase = E.pol_base;
            h.pmask = E.pol_mask;
            h.egress_bit = 1;
        }
    }
    if (h.need_pol)
        policy_issue(T, h.pbase, h.pmask, h.ident, h.dport, proto,
                     h.egress_bit, h.P);
}

// round 4: resolve the policy verdict, compose the program result
template <int MODE>
__device__ __forceinline__ void r4_verdict(const DevTables &T,
                                           const EgressArgs &E, Hdr &h)
{
    constexpr bool EGR = MODE == CFC_MODE_EGRESS;
    if (!h.need_pol)
        return;
    const bool frag = (h.mt & CFC_HF_FRAG) != 0;
    const uint32_t proto = h.mt & 0xFF;
    int v = policy_resolve(T, h.pbase, h.pmask, frag && !EGR, h.P, &h.ctr0);
    const int mdir = EGR ? METRIC_EGRESS : METRIC_INGRESS;
    if (v < 0) {
        h.act = TC_ACT_SHOT;
        h.ver = DROP_POLICY;
        h.met0 = mkey(DROP_POLICY, mdir);
    } else if (!EGR) {
        if (h.skip_proxy)
            v = 0;
        if (v > 0) {           // redirect_to_proxy
            h.act = TC_ACT_REDIRECT;
            h.ver = v;
        } else {               // TRACE_TO_LXC
            h.met0 = mkey(0, METRIC_INGRESS);
            h.act = (h.rec.w & LXC_IFINDEX) ? TC_ACT_REDIRECT : TC_ACT_OK;
            h.ver = 0;
        }
    } else if (v > 0) {        // egress proxy (bpf_lxc.c:582-604)
        h.act = TC_ACT_REDIRECT;
        h.ver = v;
    } else {
        h.met0 = mkey(0, METRIC_EGRESS);   // to_host/local/to_stack
        h.ver = 0;
        if (!(h.rec.w & LXC_VALID)) {
            h.act = TC_ACT_OK;
        } else if (h.rec.w & LXC_HOST) {
            h.act = TC_ACT_REDIRECT;
        } else if (!(h.rec.w & LXC_HAS_POLICY)) {
            h.act = TC_ACT_SHOT;
            h.ver = DROP_MISSED_TAIL_CALL;
            h.met1 = mkey(DROP_MISSED_TAIL_CALL, METRIC_EGRESS);
        } else {
            // local delivery: the destination's ipv4_policy with
            // src = SECLABEL of the sending endpoint
            int w = policy_access(T, h.rec.y, h.rec.z, E.seclabel, h.dport,
                                  proto, 0, frag, &h.ctr1);
            if (w < 0) {
                h.act = TC_ACT_SHOT;
                h.ver = DROP_POLICY;
                h.met1 = mkey(DROP_POLICY, METRIC_INGRESS);
            } else if (w > 0) {
                h.act = TC_ACT_REDIRECT;
                h.ver = w;
            } else {
                h.met1 = mkey(0, METRIC_INGRESS);
                h.act = (h.rec.w & LXC_IFINDEX) ? TC_ACT_REDIRECT : TC_ACT_OK;
            }
        }
    }
}

// U headers per thread go through the rounds side by side, so each thread
// keeps U independent lookup chains in flight (occupancy is capped at one
// workgroup per CU by the LDS counter slab).
template <int MODE, bool LDS, int U>
__global__ __launch_bounds__(BLOCK) void k_classify_v4(
    DevTables T, cfc_hdr_v4 in, cfc_out out, EgressArgs E, uint64_t *g_ctr,
    uint64_t *g_met, uint32_t *partial, uint64_t per_block)
{
    extern __shared__ uint32_t smem[];
    const uint32_t n_ctr2 = LDS ? 2 * T.n_ctr : 0;
    for (uint32_t j = threadIdx.x; j < (uint32_t)METRIC_U64 + n_ctr2; j += BLOCK)
        smem[j] = 0;
    __syncthreads();
    uint32_t *s_met = smem;
    uint32_t *s_ctr = smem + METRIC_U64;

    const uint64_t start = (uint64_t)blockIdx.x * per_block;
    const uint64_t end = min(in.n, start + per_block);
    // the trip count is uniform across the workgroup (metrics_wave needs
    // whole waves)
    for (uint64_t base = start; base < end; base += (uint64_t)BLOCK * U) {
        Hdr h[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            r1_load<MODE>(in, base + (uint64_t)u * BLOCK + threadIdx.x, end, h[u]);
#pragma unroll
        for (int u = 0; u < U; u++)
            r2_issue<MODE>(T, h[u]);
#pragma unroll
        for (int u = 0; u < U; u++)
            r3_identity<MODE>(T, E, h[u]);
#pragma unroll
        for (int u = 0; u < U; u++)
            r4_verdict<MODE>(T, E, h[u]);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t i = base + (uint64_t)u * BLOCK + threadIdx.x;
            const uint32_t len = h[u].mt >> 16;
            if (h[u].valid) {
                st_nt(h[u].ver, out.verdict + i);
                st_nt(h[u].ident, out.identity + i);
                if (out.action)
                    out.action[i] = (uint8_t)h[u].act;
                count_hit<LDS>(s_ctr, g_ctr, h[u].ctr0, len);
                count_hit<LDS>(s_ctr, g_ctr, h[u].ctr1, len);
            }
            metrics_wave(s_met, nullptr, h[u].met0, len);
            if (MODE == CFC_MODE_EGRESS)
                metrics_wave(s_met, nullptr, h[u].met1, len);
        }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < (uint32_t)METRIC_U64; j += BLOCK) {
        uint32_t v = smem[j];
        if (v)
            atomicAdd((unsigned long long *)&g_met[j], (unsigned long long)v);
    }
    if (LDS) {
        uint32_t *dst = partial + (size_t)blockIdx.x * n_ctr2;
        for (uint32_t j = threadIdx.x; j < n_ctr2; j += BLOCK)
            st_nt(smem[METRIC_U64 + j], dst + j);
    }
}

// Sum the per-workgroup partial slabs per counter (column sums, coalesced).
// blockIdx.x: 256 columns, blockIdx.y: REDUCE_ROWS partial rows.
constexpr uint32_t REDUCE_ROWS = 32;
__global__ __launch_bounds__(256) void k_reduce_partials(const uint32_t *partial,
                                                         uint32_t nblk,
                                                         uint32_t n2,
                                                         uint64_t *g_ctr)
{
    uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= n2)
        return;
    uint32_t b0 = blockIdx.y * REDUCE_ROWS;
    uint32_t b1 = min(nblk, b0 + REDUCE_ROWS);
    uint64_t s = 0;
    for (uint32_t b = b0; b < b1; b++)
        s += ld_nt(partial + (size_t)b * n2 + j);
    if (s)
        atomicAdd((unsigned long long *)&g_ctr[j], (unsigned long long)s);
}

__global__ __launch_bounds__(256) void k_add_u64(uint64_t *dst,
                                                 const uint64_t *src,
                                                 uint64_t n)
{
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n)
        dst[i] += src[i];
}

template <int MODE, bool LDS>
void launch_mode(const DevTables &T, const cfc_hdr_v4 &in, const cfc_out &out,
                 const EgressArgs &E, uint64_t *g_ctr, uint64_t *g_met,
                 uint32_t *ws, uint32_t grid, uint64_t per_block,
                 hipStream_t s)
{
    size_t lds = 4ull * (METRIC_U64 + (LDS ? 2ull * T.n_ctr : 0));
    auto kern = k_classify_v4<MODE, LDS, CFC_UNROLL>;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void *)kern,
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(4ull * (METRIC_U64 + 2ull * LDS_CTR_MAX)));
        attr_set = true;
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), lds, s, T, in, out, E,
                       g_ctr, g_met, ws, per_block);
    if (LDS && T.n_ctr) {
        uint32_t n2 = 2 * T.n_ctr;
        hipLaunchKernelGGL(k_reduce_partials,
                           dim3((n2 + 255) / 256, (grid + REDUCE_ROWS - 1) / REDUCE_ROWS),
                           dim3(256), 0, s, ws, grid, n2, g_ctr);
    }
}

// Workgroups of <= MAX_PER_BLOCK headers; at least one per CU when the
// batch allows it.
void geometry(uint64_t n, int num_cus, uint32_t *grid, uint64_t *per_block)
{
    uint64_t pb = (n + (uint64_t)num_cus - 1) / (uint64_t)num_cus;
    pb = (pb + BLOCK - 1) / BLOCK * BLOCK;
    if (pb < BLOCK)
        pb = BLOCK;
    if (pb > MAX_PER_BLOCK)
        pb = MAX_PER_BLOCK;
    *per_block = pb;
    *grid = (uint32_t)((n + pb - 1) / pb);
}

}  // namespace

int launch_add_u64(uint64_t *dst, const uint64_t *src, uint64_t n,
                   hipStream_t s)
{
    if (!n)
        return 0;
    hipLaunchKernelGGL(k_add_u64, dim3((unsigned)((n + 255) / 256)), dim3(256),
                       0, s, dst, src, n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

size_t classify_workspace_bytes(uint64_t n, uint32_t n_ctr, int num_cus)
{
    if (n_ctr > LDS_CTR_MAX || n == 0)
        return 0;
    uint32_t grid;
    uint64_t pb;
    geometry(n, num_cus, &grid, &pb);
    return 4ull * 2 * n_ctr * grid;
}

int launch_classify_v4(const DevTables &T, const cfc_hdr_v4 &in,
                       const cfc_out &out, int mode, const EgressArgs &E,
                       uint64_t *g_ctr, uint64_t *g_met, uint32_t *ws,
                       int num_cus, hipStream_t s)
{
    if (in.n == 0)
        return 0;
    bool lds = T.n_ctr <= LDS_CTR_MAX;
    uint32_t grid;
    uint64_t per_block;
    geometry(in.n, num_cus, &grid, &per_block);
#define CFC_LAUNCH(M)                                                         \
    (lds ? launch_mode<M, true>(T, in, out, E, g_ctr, g_met, ws, grid,        \
                                per_block, s)                                 \
         : launch_mode<M, false>(T, in, out, E, g_ctr, g_met, ws, grid,       \
                                 per_block, s))
    switch (mode) {
    case CFC_MODE_INGRESS: CFC_LAUNCH(CFC_MODE_INGRESS); break;
    case CFC_MODE_EGRESS: CFC_LAUNCH(CFC_MODE_EGRESS); break;
    case CFC_MODE_XDP: CFC_LAUNCH(CFC_MODE_XDP); break;
    case CFC_MODE_FULL: CFC_LAUNCH(CFC_MODE_FULL); break;
    default: return -22;
    }
#undef CFC_LAUNCH
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -5;
}

}  // namespace cfc
