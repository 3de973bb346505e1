// Batched verdict kernels for gfx950 (MI355X).
//
// One thread classifies one header at a time; a 1024-thread workgroup owns a
// contiguous slice of the batch, so each loop iteration reads 4 KiB of every
// SoA input array coalesced and writes the outputs coalesced.  The lookups
// are dependent random accesses (DIR-24-8 tbl24/tbl8 in the Infinity Cache,
// the endpoint and policy buckets in L2): this is HBM/latency-bound integer
// work with no contraction, so there is no MFMA here.
//
// Counters follow the reference's exact integer sums.  Per-entry packets and
// bytes (policy.h:68-69,80-81,92-93) and cilium_metrics (metrics.h:43-61)
// are accumulated in LDS as u32 (a wrap carries 2^32 straight to the global
// u64), written once per workgroup as a partial slab, and summed per entry by
// a second kernel — no per-header global atomics.
//
// Reference semantics restated here (file:line in /root/reference):
//   netdev_ingress  bpf_netdev.c:128-153 (FROM_HOST identity from mark),
//                   :357-453 handle_ipv4 (ipcache src identity, lxc lookup)
//   lxc_ingress     bpf_lxc.c:898-1028 ipv4_policy + tail_ipv4_policy
//   lxc_egress      bpf_lxc.c:440-704 handle_ipv4_from_lxc
//   policy_access   bpf/lib/policy.h:46-146
//   ct_new_dport    bpf/lib/conntrack.h:467-590 (ports of a CT_NEW tuple)
//   xdp_v4          bpf_xdp.c:88-121
#include "classify.hpp"

namespace cfc {

namespace {

constexpr uint32_t HOST_ID = 1, WORLD_ID = 2, CLUSTER_ID = 3, HEALTH_ID = 4;
constexpr uint32_t IPV4_CLUSTER_MASK = 0xff0000u, IPV4_CLUSTER_RANGE = 0x100000u;
constexpr int DROP_INVALID_SIP = -132, DROP_POLICY = -133,
              DROP_CT_UNKNOWN_PROTO = -137, DROP_MISSED_TAIL_CALL = -140,
              DROP_FRAG_NOSUPPORT = -157;
constexpr int TC_ACT_OK = 0, TC_ACT_SHOT = 2, TC_ACT_REDIRECT = 7;
constexpr int XDP_DROP = 1, XDP_PASS = 2;
constexpr int METRIC_INGRESS = 1, METRIC_EGRESS = 2;
constexpr uint32_t ENDPOINT_F_HOST = 1;

struct Counters {
    uint32_t *s_met;   // LDS metrics [256][4][2] u32
    uint32_t *s_ctr;   // LDS policy counters [n_ctr][2] u32, or null
    uint64_t *g_ctr;
    uint64_t *g_met;

    __device__ static void add_carry(uint32_t *s, uint64_t *g, uint32_t v)
    {
        uint32_t old = atomicAdd(s, v);
        if (old + v < old)
            atomicAdd((unsigned long long *)g, 1ull << 32);
    }
    __device__ void hit(uint32_t idx, uint32_t len) const
    {
        if (s_ctr) {
            add_carry(&s_ctr[2 * idx], &g_ctr[2 * idx], 1u);
            add_carry(&s_ctr[2 * idx + 1], &g_ctr[2 * idx + 1], len);
        } else {
            atomicAdd((unsigned long long *)&g_ctr[2 * idx], 1ull);
            atomicAdd((unsigned long long *)&g_ctr[2 * idx + 1],
                      (unsigned long long)len);
        }
    }
    // update_metrics(len, dir, -reason); reason is DROP_* (<0) or 0
    __device__ void metric(int reason, int dir, uint32_t len) const
    {
        uint32_t j = (((uint32_t)(uint8_t)(-reason)) * METRIC_DIRS + dir) * 2;
        add_carry(&s_met[j], &g_met[j], 1u);
        add_carry(&s_met[j + 1], &g_met[j + 1], len);
    }
};

__device__ __forceinline__ uint32_t lpm4(const uint32_t *tbl24,
                                         const uint32_t *tbl8,
                                         const uint32_t *ovf, uint32_t addr_be)
{
    if (!tbl24)
        return 0;
    uint32_t h = __builtin_bswap32(addr_be);
    uint32_t e = tbl24[h >> 8];
    if (e & LPM_GROUP)
        e = tbl8[((e & ~LPM_GROUP) << 8) | (h & 0xFF)];
    if (e & LPM_INDIRECT)
        e = ovf[e & LPM_PAYLOAD];
    return e;
}

__device__ __forceinline__ int lxc4_find(const DevTables &T, uint32_t addr)
{
    if (!T.lxc4)
        return -1;
    uint32_t b = hash32(addr, T.lxc4_mask);
    for (;;) {
        const uint4 *bk = reinterpret_cast<const uint4 *>(T.lxc4 + (size_t)b * LXC_SLOTS);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint4 v = bk[q];
            if (v.y == EMPTY)
                return -1;
            if (v.x == addr)
                return (int)v.y;
            if (v.w == EMPTY)
                return -1;
            if (v.z == addr)
                return (int)v.w;
        }
        b = (b + 1) & T.lxc4_mask;
    }
}

__device__ __forceinline__ bool pf_fix_hit(const DevTables &T, uint32_t addr)
{
    if (!T.pf_fix)
        return false;
    uint32_t b = hash32(addr, T.pf_fix_mask);
    for (;;) {
        const uint4 *bk = reinterpret_cast<const uint4 *>(T.pf_fix + (size_t)b * 16);
        uint4 q[4];
#pragma unroll
        for (int i = 0; i < 4; i++)
            q[i] = bk[i];
        uint32_t cnt = q[3].w;
        const uint32_t a[15] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y,
                                q[1].z, q[1].w, q[2].x, q[2].y, q[2].z, q[2].w,
                                q[3].x, q[3].y, q[3].z};
        bool hit = false;
#pragma unroll
        for (int i = 0; i < 15; i++)
            hit |= (i < (int)cnt) & (a[i] == addr);
        if (hit)
            return true;
        if (cnt < (uint32_t)PF_SLOTS)
            return false;
        b = (b + 1) & T.pf_fix_mask;
    }
}

// policy hash probe: returns counter index or EMPTY; *proxy = proxy_port
__device__ __forceinline__ uint32_t pol_find(const PolSlot *pol, uint32_t base,
                                             uint32_t mask, uint64_t key,
                                             uint32_t *proxy)
{
    uint32_t b = hash64(key, mask);
    for (;;) {
        const uint4 *bk = reinterpret_cast<const uint4 *>(pol + (size_t)(base + b) * POL_SLOTS);
#pragma unroll
        for (int s = 0; s < POL_SLOTS; s++) {
            uint4 v = bk[s];
            if (v.w == EMPTY)
                return EMPTY;
            if ((((uint64_t)v.y << 32) | v.x) == key) {
                *proxy = v.z & 0xFFFF;
                return v.w;
            }
        }
        b = (b + 1) & mask;
    }
}

__device__ __forceinline__ uint64_t pkey(uint32_t id, uint32_t dport,
                                         uint32_t proto, uint32_t egress)
{
    return (uint64_t)id | ((uint64_t)dport << 32) | ((uint64_t)proto << 48) |
           ((uint64_t)egress << 56);
}

// __policy_can_access (policy.h:46-110) with cb[CB_POLICY] == 0
__device__ __forceinline__ int policy_access(const DevTables &T, uint32_t base,
                                             uint32_t mask, uint32_t id,
                                             uint32_t dport, uint32_t proto,
                                             uint32_t egress, bool frag,
                                             uint32_t len, const Counters &C)
{
    uint32_t proxy = 0, c;
    if (!frag) {
        c = pol_find(T.pol, base, mask, pkey(id, dport, proto, egress), &proxy);
        if (c != EMPTY) {
            C.hit(c, len);
            return (int)proxy;
        }
    }
    c = pol_find(T.pol, base, mask, pkey(id, 0, 0, egress), &proxy);
    if (c != EMPTY) {
        C.hit(c, len);
        return TC_ACT_OK;
    }
    if (!frag) {
        c = pol_find(T.pol, base, mask, pkey(0, dport, proto, egress), &proxy);
        if (c != EMPTY) {
            C.hit(c, len);
            return (int)proxy;
        }
    }
    return frag ? DROP_FRAG_NOSUPPORT : DROP_POLICY;
}

// tuple->dport of a CT_NEW lookup (conntrack.h:496-584): TCP/UDP ports are
// loaded swapped and swapped back by ipv4_ct_tuple_reverse(); ICMP echo puts
// its type (8) in tuple->sport, which becomes the dport; other ICMP -> 0.
__device__ __forceinline__ bool ct_new_dport(uint32_t proto, uint32_t ports,
                                             uint32_t *dport)
{
    if (proto == 6 || proto == 17) {
        *dport = ports >> 16;
        return true;
    }
    if (proto == 1) {
        *dport = (ports & 0xFF) == 8 ? 8u : 0u;
        return true;
    }
    return false;
}

struct Res {
    int act, ver;
    uint32_t id;
};

// ipv4_policy (bpf_lxc.c:898-1015) of endpoint r, src label `src`
__device__ __forceinline__ void lxc_ingress(const DevTables &T, const EpRec &r,
                                            uint32_t src, uint32_t proto,
                                            uint32_t ports, bool frag,
                                            uint32_t len, bool skip_proxy,
                                            int dir_missed, const Counters &C,
                                            Res &o)
{
    if (!r.has_policy) {  // cilium_policy[lxc_id] tail call missed (l3.h:130)
        o.act = TC_ACT_SHOT;
        o.ver = DROP_MISSED_TAIL_CALL;
        C.metric(DROP_MISSED_TAIL_CALL, dir_missed, len);
        return;
    }
    uint32_t dport;
    if (!ct_new_dport(proto, ports, &dport)) {
        o.act = TC_ACT_SHOT;
        o.ver = DROP_CT_UNKNOWN_PROTO;
        C.metric(DROP_CT_UNKNOWN_PROTO, METRIC_INGRESS, len);
        return;
    }
    int v = policy_access(T, r.pol_base, r.pol_mask, src, dport, proto, 0,
                          frag, len, C);
    if (v < 0) {
        o.act = TC_ACT_SHOT;
        o.ver = DROP_POLICY;
        C.metric(DROP_POLICY, METRIC_INGRESS, len);
        return;
    }
    if (skip_proxy)
        v = 0;
    if (v > 0) {  // redirect_to_proxy -> redirect(HOST_IFINDEX)
        o.act = TC_ACT_REDIRECT;
        o.ver = v;
        return;
    }
    C.metric(0, METRIC_INGRESS, len);  // send_trace_notify(TRACE_TO_LXC)
    o.act = r.ifindex ? TC_ACT_REDIRECT : TC_ACT_OK;
    o.ver = 0;
}

__device__ __forceinline__ void netdev_ingress(const DevTables &T,
                                               uint32_t saddr, uint32_t daddr,
                                               uint32_t ports, uint32_t meta,
                                               uint32_t mark, const Counters &C,
                                               Res &o)
{
    uint32_t magic = mark & 0xF00u, identity;
    bool skip_proxy = false;
    if (magic == 0xA00u || magic == 0xB00u) {  // proxy: identity in mark
        identity = ((mark & 0xFF) << 16) | (mark >> 16);
        skip_proxy = magic == 0xA00u;
    } else {
        identity = magic == 0xC00u ? HOST_ID : WORLD_ID;
    }
    if (identity < HEALTH_ID) {  // identity_is_reserved
        uint32_t l = lpm4(T.tbl24, T.tbl8, T.lbl_ovf, saddr);
        if (l && l != CLUSTER_ID && l != HOST_ID)
            identity = l;
    }
    o.id = identity;
    o.act = TC_ACT_OK;
    o.ver = 0;
    int e = lxc4_find(T, daddr);
    if (e < 0)
        return;
    EpRec r = T.eps[e];
    if (r.flags & ENDPOINT_F_HOST)
        return;
    lxc_ingress(T, r, identity, meta & 0xFF, ports, (meta & CFC_HF_FRAG) != 0,
                meta >> 16, skip_proxy, METRIC_INGRESS, C, o);
}

__device__ __forceinline__ void lxc_egress(const DevTables &T,
                                           const EgressArgs &E, uint32_t saddr,
                                           uint32_t daddr, uint32_t ports,
                                           uint32_t meta, const Counters &C,
                                           Res &o)
{
    uint32_t len = meta >> 16, proto = meta & 0xFF;
    o.id = 0;
    o.act = TC_ACT_SHOT;
    int se = lxc4_find(T, saddr);
    if (se < 0 || T.eps[se].lxc_id != E.lxc_id) {  // is_valid_lxc_src_ipv4
        o.ver = DROP_INVALID_SIP;
        C.metric(DROP_INVALID_SIP, METRIC_EGRESS, len);
        return;
    }
    uint32_t dport;
    if (!ct_new_dport(proto, ports, &dport)) {
        o.ver = DROP_CT_UNKNOWN_PROTO;
        C.metric(DROP_CT_UNKNOWN_PROTO, METRIC_EGRESS, len);
        return;
    }
    uint32_t l = lpm4(T.tbl24, T.tbl8, T.lbl_ovf, daddr);
    uint32_t dst = l ? l
                     : ((daddr & IPV4_CLUSTER_MASK) == IPV4_CLUSTER_RANGE ? CLUSTER_ID
                                                                          : WORLD_ID);
    o.id = dst;
    int v = policy_access(T, E.pol_base, E.pol_mask, dst, dport, proto, 1,
                          false, len, C);
    if (v < 0) {
        o.ver = DROP_POLICY;
        C.metric(DROP_POLICY, METRIC_EGRESS, len);
        return;
    }
    o.ver = v;
    if (v > 0) {  // proxy redirect (bpf_lxc.c:582-604)
        o.act = TC_ACT_REDIRECT;
        return;
    }
    int e = lxc4_find(T, daddr);
    C.metric(0, METRIC_EGRESS, len);  // to_host / local delivery / to_stack
    if (e < 0) {
        o.act = TC_ACT_OK;
        return;
    }
    EpRec r = T.eps[e];
    if (r.flags & ENDPOINT_F_HOST) {
        o.act = TC_ACT_REDIRECT;
        return;
    }
    Res d;
    lxc_ingress(T, r, E.seclabel, proto, ports, (meta & CFC_HF_FRAG) != 0,
                len, false, METRIC_EGRESS, C, d);
    o.act = d.act;
    o.ver = d.ver;
}

// check_v4 (bpf_xdp.c:97-121): dyn LPM, then fixed /32 set, then endpoint
__device__ __forceinline__ bool xdp_pass(const DevTables &T, uint32_t saddr,
                                         uint32_t daddr)
{
    if (lpm4(T.pf_tbl24, T.pf_tbl8, nullptr, saddr))
        return false;
    if (pf_fix_hit(T, saddr))
        return false;
    return lxc4_find(T, daddr) >= 0;
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
    Counters C{smem, LDS ? smem + METRIC_U64 : nullptr, g_ctr, g_met};

    const uint64_t start = (uint64_t)blockIdx.x * per_block;
    const uint64_t end = min(in.n, start + per_block);
    for (uint64_t i = start + threadIdx.x; i < end; i += BLOCK) {
        const uint32_t saddr = in.saddr[i], daddr = in.daddr[i];
        const uint32_t ports = in.ports[i], meta = in.meta[i];
        const uint32_t mark = in.mark ? in.mark[i] : 0u;
        Res o{TC_ACT_OK, 0, 0};
        if (MODE == CFC_MODE_XDP || MODE == CFC_MODE_FULL) {
            bool pass = xdp_pass(T, saddr, daddr);
            if (MODE == CFC_MODE_XDP || !pass) {
                o.act = pass ? XDP_PASS : XDP_DROP;
                o.ver = pass ? 0 : CFC_DROP_PREFILTER;
                o.id = 0;
            } else {
                netdev_ingress(T, saddr, daddr, ports, meta, mark, C, o);
            }
        } else if (MODE == CFC_MODE_EGRESS) {
            lxc_egress(T, E, saddr, daddr, ports, meta, C, o);
        } else {
            netdev_ingress(T, saddr, daddr, ports, meta, mark, C, o);
        }
        out.verdict[i] = o.ver;
        out.identity[i] = o.id;
        if (out.action)
            out.action[i] = (uint8_t)o.act;
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
            dst[j] = smem[METRIC_U64 + j];
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
        s += partial[(size_t)b * n2 + j];
    if (s)
        atomicAdd((unsigned long long *)&g_ctr[j], (unsigned long long)s);
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

uint32_t grid_for(uint64_t n, int num_cus, bool lds)
{
    uint64_t want = (n + BLOCK - 1) / BLOCK;
    uint64_t cap = lds ? (uint64_t)num_cus : (uint64_t)num_cus * 2;
    if (want < 1)
        want = 1;
    return (uint32_t)(want < cap ? want : cap);
}

}  // namespace

namespace {
__global__ __launch_bounds__(256) void k_add_u64(uint64_t *dst,
                                                 const uint64_t *src,
                                                 uint64_t n)
{
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n)
        dst[i] += src[i];
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
    bool lds = n_ctr <= LDS_CTR_MAX;
    if (!lds)
        return 0;
    return 4ull * 2 * n_ctr * grid_for(n, num_cus, true);
}

int launch_classify_v4(const DevTables &T, const cfc_hdr_v4 &in,
                       const cfc_out &out, int mode, const EgressArgs &E,
                       uint64_t *g_ctr, uint64_t *g_met, uint32_t *ws,
                       int num_cus, hipStream_t s)
{
    if (in.n == 0)
        return 0;
    bool lds = T.n_ctr <= LDS_CTR_MAX;
    uint32_t grid = grid_for(in.n, num_cus, lds);
    uint64_t per_block = (in.n + grid - 1) / grid;
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
