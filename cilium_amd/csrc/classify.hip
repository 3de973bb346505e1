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
constexpr uint32_t ENDPOINT_F_HOST = 1;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint64_t MAX_PER_BLOCK = 65536;   // keeps u32 LDS sums exact

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

struct B64 {   // one 64-byte bucket
    uint4 q[4];
};
__device__ __forceinline__ B64 ldb(const void *p)
{
    const uint4 *b = reinterpret_cast<const uint4 *>(p);
    B64 r;
#pragma unroll
    for (int i = 0; i < 4; i++)
        r.q[i] = b[i];
    return r;
}

// ---- lookups on a loaded bucket: 1 hit, 0 definite miss, -1 keep probing
__device__ __forceinline__ int lxc_scan(const B64 &B, uint32_t addr, int *ep)
{
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint4 v = B.q[i];
        if (v.y == EMPTY)
            return 0;
        if (v.x == addr) {
            *ep = (int)v.y;
            return 1;
        }
        if (v.w == EMPTY)
            return 0;
        if (v.z == addr) {
            *ep = (int)v.w;
            return 1;
        }
    }
    return -1;
}

__device__ __forceinline__ int pf_scan(const B64 &B, uint32_t addr)
{
    const uint32_t a[16] = {B.q[0].x, B.q[0].y, B.q[0].z, B.q[0].w,
                            B.q[1].x, B.q[1].y, B.q[1].z, B.q[1].w,
                            B.q[2].x, B.q[2].y, B.q[2].z, B.q[2].w,
                            B.q[3].x, B.q[3].y, B.q[3].z, B.q[3].w};
    const uint32_t cnt = a[15];
    bool hit = false;
#pragma unroll
    for (int i = 0; i < PF_SLOTS; i++)
        hit |= ((uint32_t)i < cnt) & (a[i] == addr);
    return hit ? 1 : (cnt < (uint32_t)PF_SLOTS ? 0 : -1);
}

__device__ __forceinline__ int pol_scan(const B64 &B, uint64_t key,
                                        uint32_t *ctr, uint32_t *proxy)
{
#pragma unroll
    for (int s = 0; s < POL_SLOTS; s++) {
        const uint4 v = B.q[s];
        if (v.w == EMPTY)
            return 0;
        if ((((uint64_t)v.y << 32) | v.x) == key) {
            *ctr = v.w;
            *proxy = v.z & 0xFFFF;
            return 1;
        }
    }
    return -1;
}

// ---- probing continuations (cold paths)
__device__ inline int lxc_probe_from(const DevTables &T, uint32_t addr,
                                           uint32_t b)
{
    for (;;) {
        b = (b + 1) & T.lxc4_mask;
        int ep = -1;
        int r = lxc_scan(ldb(T.lxc4 + (size_t)b * LXC_SLOTS), addr, &ep);
        if (r >= 0)
            return r ? ep : -1;
    }
}

__device__ inline bool pf_probe_from(const DevTables &T, uint32_t addr,
                                           uint32_t b)
{
    for (;;) {
        b = (b + 1) & T.pf_fix_mask;
        int r = pf_scan(ldb(T.pf_fix + (size_t)b * 16), addr);
        if (r >= 0)
            return r == 1;
    }
}

__device__ inline uint32_t pol_probe_from(const PolSlot *pol,
                                                uint32_t base, uint32_t mask,
                                                uint64_t key, uint32_t b,
                                                uint32_t *proxy)
{
    for (;;) {
        b = (b + 1) & mask;
        uint32_t c = NONE;
        int r = pol_scan(ldb(pol + (size_t)(base + b) * POL_SLOTS), key, &c, proxy);
        if (r >= 0)
            return r ? c : NONE;
    }
}

__device__ __forceinline__ int lxc_find(const DevTables &T, uint32_t addr)
{
    if (!T.lxc4)
        return -1;
    uint32_t b = hash32(addr, T.lxc4_mask);
    int ep = -1;
    int r = lxc_scan(ldb(T.lxc4 + (size_t)b * LXC_SLOTS), addr, &ep);
    return r > 0 ? ep : (r == 0 ? -1 : lxc_probe_from(T, addr, b));
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

// __policy_can_access (policy.h:46-110), cb[CB_POLICY] == 0: the three keys'
// buckets are loaded together, the first match in the reference's order
// wins.  Returns the verdict (<0 drop) and the matched counter (or NONE).
struct PolicyProbe {
    uint64_t k[3];
    uint32_t b[3];
    B64 bk[3];
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
        P.b[j] = hash64(P.k[j], mask);
        P.bk[j] = ldb(T.pol + (size_t)(base + P.b[j]) * POL_SLOTS);
    }
}

__device__ __forceinline__ int policy_resolve(const DevTables &T, uint32_t base,
                                              uint32_t mask, bool frag,
                                              const PolicyProbe &P,
                                              uint32_t *ctr)
{
    uint32_t proxy = 0, c = NONE;
#pragma unroll
    for (int j = 0; j < 3; j++) {
        if (frag && j != 1)   // fragments: L3 key only (policy.h:61,85)
            continue;
        int r = pol_scan(P.bk[j], P.k[j], &c, &proxy);
        if (r < 0)
            c = pol_probe_from(T.pol, base, mask, P.k[j], P.b[j], &proxy);
        if (r > 0 || (r < 0 && c != NONE)) {
            *ctr = c;
            return j == 1 ? TC_ACT_OK : (int)proxy;
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

template <int MODE, bool LDS>
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

    constexpr bool XDP = MODE == CFC_MODE_XDP || MODE == CFC_MODE_FULL;
    constexpr bool EGR = MODE == CFC_MODE_EGRESS;
    constexpr bool LPM = MODE != CFC_MODE_XDP;

    const uint64_t start = (uint64_t)blockIdx.x * per_block;
    const uint64_t end = min(in.n, start + per_block);
    // trip count is uniform across the workgroup (metrics_wave needs whole waves)
    for (uint64_t base = start; base < end; base += BLOCK) {
        const uint64_t i = base + threadIdx.x;
        const bool valid = i < end;
        uint32_t sa = 0, da = 0, pt = 0, mt = 0, mk = 0;
        if (valid) {
            sa = ld_nt(in.saddr + i);
            da = ld_nt(in.daddr + i);
            pt = ld_nt(in.ports + i);
            mt = ld_nt(in.meta + i);
            if (in.mark)
                mk = ld_nt(in.mark + i);
        }
        const uint32_t proto = mt & 0xFF, len = mt >> 16;
        const bool frag = (mt & CFC_HF_FRAG) != 0;

        // ---- round 2: every lookup that only needs the header
        uint32_t e24 = 0, pfd = 0;
        B64 lx{}, pf{}, ls{};
        const uint32_t la = EGR ? da : sa;
        const uint32_t lh = __builtin_bswap32(la);
        const uint32_t hsh = __builtin_bswap32(sa);
        uint32_t lxb = 0, pfb = 0, lsb = 0;
        if (valid) {
            if (LPM && T.tbl24)
                e24 = T.tbl24[lh >> 8];
            if (XDP && T.pf_tbl24)
                pfd = T.pf_tbl24[hsh >> 8];
            if (T.lxc4) {
                lxb = hash32(da, T.lxc4_mask);
                lx = ldb(T.lxc4 + (size_t)lxb * LXC_SLOTS);
                if (EGR) {
                    lsb = hash32(sa, T.lxc4_mask);
                    ls = ldb(T.lxc4 + (size_t)lsb * LXC_SLOTS);
                }
            }
            if (XDP && T.pf_fix) {
                pfb = hash32(sa, T.pf_fix_mask);
                pf = ldb(T.pf_fix + (size_t)pfb * 16);
            }
        }

        // ---- round 3: second-level LPM, endpoint records
        if (e24 & LPM_GROUP)
            e24 = T.tbl8[((e24 & ~LPM_GROUP) << 8) | (lh & 0xFF)];
        if (e24 & LPM_INDIRECT)
            e24 = T.lbl_ovf[e24 & LPM_PAYLOAD];
        if (pfd & LPM_GROUP)
            pfd = T.pf_tbl8[((pfd & ~LPM_GROUP) << 8) | (hsh & 0xFF)];
        int ep = -1, es = -1;
        if (valid && T.lxc4) {
            int r = lxc_scan(lx, da, &ep);
            if (r < 0)
                ep = lxc_probe_from(T, da, lxb);
            if (EGR) {
                r = lxc_scan(ls, sa, &es);
                if (r < 0)
                    es = lxc_probe_from(T, sa, lsb);
            }
        }
        EpRec rec{};
        if (ep >= 0)
            rec = T.eps[ep];
        uint32_t src_lxc = NONE;
        if (EGR && es >= 0)
            src_lxc = T.eps[es].lxc_id;

        int act = TC_ACT_OK, ver = 0;
        uint32_t ident = 0, met0 = NONE, met1 = NONE, ctr0 = NONE, ctr1 = NONE;
        bool xdp_drop = false;
        if (XDP && valid) {
            bool deny = pfd != 0;
            if (!deny && T.pf_fix) {
                int r = pf_scan(pf, sa);
                deny = r > 0 || (r < 0 && pf_probe_from(T, sa, pfb));
            }
            xdp_drop = deny || ep < 0;
            if (MODE == CFC_MODE_XDP || xdp_drop) {
                act = xdp_drop ? XDP_DROP : XDP_PASS;
                ver = xdp_drop ? CFC_DROP_PREFILTER : 0;
            }
        }

        // ---- round 4: identity, then the three policy buckets together
        bool need_pol = false, skip_proxy = false;
        uint32_t pbase = 0, pmask = 0, egress_bit = 0, dport = 0, src = 0;
        if (valid && MODE != CFC_MODE_XDP && !xdp_drop) {
            const bool known = ct_new_dport(proto, pt, &dport);
            if (!EGR) {
                // handle_identity_from_host (bpf_netdev.c:128-153)
                const uint32_t magic = mk & 0xF00u;
                if (magic == 0xA00u || magic == 0xB00u) {
                    ident = ((mk & 0xFF) << 16) | (mk >> 16);
                    skip_proxy = magic == 0xA00u;
                } else {
                    ident = magic == 0xC00u ? HOST_ID : WORLD_ID;
                }
                // handle_ipv4 (:375-398): reserved identities take the ipcache's
                if (ident < HEALTH_ID && e24 && e24 != CLUSTER_ID && e24 != HOST_ID)
                    ident = e24;
                if (ep >= 0 && !(rec.flags & ENDPOINT_F_HOST)) {
                    if (!rec.has_policy) {
                        act = TC_ACT_SHOT;
                        ver = DROP_MISSED_TAIL_CALL;
                        met0 = mkey(DROP_MISSED_TAIL_CALL, METRIC_INGRESS);
                    } else if (!known) {
                        act = TC_ACT_SHOT;
                        ver = DROP_CT_UNKNOWN_PROTO;
                        met0 = mkey(DROP_CT_UNKNOWN_PROTO, METRIC_INGRESS);
                    } else {
                        need_pol = true;
                        pbase = rec.pol_base;
                        pmask = rec.pol_mask;
                        src = ident;
                    }
                }
            } else {
                act = TC_ACT_SHOT;
                if (src_lxc != E.lxc_id) {   // is_valid_lxc_src_ipv4 (lxc.h:55)
                    ver = DROP_INVALID_SIP;
                    met0 = mkey(DROP_INVALID_SIP, METRIC_EGRESS);
                } else if (!known) {
                    ver = DROP_CT_UNKNOWN_PROTO;
                    met0 = mkey(DROP_CT_UNKNOWN_PROTO, METRIC_EGRESS);
                } else {
                    // destination identity (bpf_lxc.c:516-532)
                    ident = e24 ? e24
                                : ((da & IPV4_CLUSTER_MASK) == IPV4_CLUSTER_RANGE
                                       ? CLUSTER_ID
                                       : WORLD_ID);
                    need_pol = true;
                    pbase = E.pol_base;
                    pmask = E.pol_mask;
                    egress_bit = 1;
                    src = ident;
                }
            }
        }
        PolicyProbe P;
        if (need_pol)
            policy_issue(T, pbase, pmask, src, dport, proto, egress_bit, P);

        if (need_pol) {
            int v = policy_resolve(T, pbase, pmask, frag && !EGR, P, &ctr0);
            const int mdir = EGR ? METRIC_EGRESS : METRIC_INGRESS;
            if (v < 0) {
                act = TC_ACT_SHOT;
                ver = DROP_POLICY;
                met0 = mkey(DROP_POLICY, mdir);
            } else if (!EGR) {
                if (skip_proxy)
                    v = 0;
                if (v > 0) {           // redirect_to_proxy
                    act = TC_ACT_REDIRECT;
                    ver = v;
                } else {               // TRACE_TO_LXC
                    met0 = mkey(0, METRIC_INGRESS);
                    act = rec.ifindex ? TC_ACT_REDIRECT : TC_ACT_OK;
                    ver = 0;
                }
            } else if (v > 0) {        // egress proxy (bpf_lxc.c:582-604)
                act = TC_ACT_REDIRECT;
                ver = v;
            } else {
                met0 = mkey(0, METRIC_EGRESS);   // to_host/local/to_stack
                ver = 0;
                if (ep < 0) {
                    act = TC_ACT_OK;
                } else if (rec.flags & ENDPOINT_F_HOST) {
                    act = TC_ACT_REDIRECT;
                } else if (!rec.has_policy) {
                    act = TC_ACT_SHOT;
                    ver = DROP_MISSED_TAIL_CALL;
                    met1 = mkey(DROP_MISSED_TAIL_CALL, METRIC_EGRESS);
                } else {
                    // local delivery: the destination's ipv4_policy with
                    // src = SECLABEL of the sending endpoint
                    int w = policy_access(T, rec.pol_base, rec.pol_mask,
                                          E.seclabel, dport, proto, 0, frag,
                                          &ctr1);
                    if (w < 0) {
                        act = TC_ACT_SHOT;
                        ver = DROP_POLICY;
                        met1 = mkey(DROP_POLICY, METRIC_INGRESS);
                    } else if (w > 0) {
                        act = TC_ACT_REDIRECT;
                        ver = w;
                    } else {
                        met1 = mkey(0, METRIC_INGRESS);
                        act = rec.ifindex ? TC_ACT_REDIRECT : TC_ACT_OK;
                    }
                }
            }
        }

        if (valid) {
            st_nt(ver, out.verdict + i);
            st_nt(ident, out.identity + i);
            if (out.action)
                out.action[i] = (uint8_t)act;
            count_hit<LDS>(s_ctr, g_ctr, ctr0, len);
            count_hit<LDS>(s_ctr, g_ctr, ctr1, len);
        }
        metrics_wave(s_met, nullptr, met0, len);
        if (EGR)
            metrics_wave(s_met, nullptr, met1, len);
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
__global__ __launch_bounds__(256) void k_reduce_partials(const uint32_t *partial,
                                                         uint32_t nblk,
                                                         uint32_t n2,
                                                         uint64_t *g_ctr)
{
    uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= n2)
        return;
    uint64_t s = 0;
    for (uint32_t b = 0; b < nblk; b++)
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
    auto kern = k_classify_v4<MODE, LDS>;
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
        hipLaunchKernelGGL(k_reduce_partials, dim3((n2 + 255) / 256), dim3(256),
                           0, s, ws, grid, n2, g_ctr);
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
