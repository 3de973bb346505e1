// Device helpers shared by the IPv4 and IPv6 classify kernels
// (classify.hip, classify6.hip): streaming loads, the LDS image, the Bloom
// filters, __policy_can_access and the per-thread metrics accumulators.
#pragma once
#include "classify.hpp"

namespace cfc {

namespace {

constexpr uint32_t HOST_ID = 1, WORLD_ID = 2, CLUSTER_ID = 3, HEALTH_ID = 4;
constexpr int DROP_INVALID_SIP = -132, DROP_POLICY = -133,
              DROP_CT_UNKNOWN_PROTO = -137, DROP_MISSED_TAIL_CALL = -140,
              DROP_NO_SERVICE = -158, DROP_INVALID = -134;
constexpr int TC_ACT_OK = 0, TC_ACT_SHOT = 2, TC_ACT_REDIRECT = 7;
constexpr int XDP_DROP = 1, XDP_PASS = 2;
constexpr int METRIC_INGRESS = 1, METRIC_EGRESS = 2;
constexpr uint32_t NONE = 0xFFFFFFFFu;
// k_count: the packed u32 byte sums stay exact (64512 headers x 65535
// bytes < 2^32, so they never carry into the packet count)
constexpr uint64_t COUNT_PER_BLOCK = 63 * BLOCK;

// cfc_out.notify word of a header (cfc.h CFC_NT_*): which send_drop_notify
// the reference ran.  dest_stage: an egress batch's drop came from the
// destination endpoint's policy program after local delivery.
__device__ __forceinline__ uint32_t notify_word(int mode, int ver,
                                                bool dest_stage,
                                                uint32_t dest_lxc,
                                                uint32_t ep_lxc)
{
    if (ver >= 0 || ver == CFC_DROP_PREFILTER || ver == CFC_VERDICT_PUNT)
        return 0;
    if (mode == CFC_MODE_EGRESS)
        return dest_stage ? (CFC_NT_POLICY << 16 | dest_lxc)
                          : (CFC_NT_EGRESS << 16 | ep_lxc);
    // bpf_netdev's own errors: the failed tail call of local delivery
    // (l3.h:130) and ipv6_hdrlen's DROP_INVALID_EXTHDR / DROP_FRAG_NOSUPPORT
    const bool netdev = ver == DROP_MISSED_TAIL_CALL || ver == -156 || ver == -157;
    return netdev ? CFC_NT_NETDEV << 16 : (CFC_NT_POLICY << 16 | dest_lxc);
}
// ---- monitor events (cfc.h CFC_NT_*): the trace_notify of a forwarded
// packet.  obs: TRACE_TO_LXC 0, TO_PROXY 1, TO_HOST 2, TO_STACK 3; reason:
// the CT result; mon: the monitor length (0 = not sent, MONITOR_AGGREGATION
// 5 drops traces of flows inside their report interval, trace.h:131-132)
constexpr uint32_t OBS_TO_LXC = 0, OBS_TO_PROXY = 1, OBS_TO_HOST = 2, OBS_TO_STACK = 3;
constexpr uint32_t TRACE_PAYLOAD_LEN = 128, MTU_LEN = 1500;
// mon 0 (not sent) keeps the site with length class 0: cfc_ct_apply
// re-decides the length in packet order (ctapply.hip k_cta_mon)
// one wave appends header i to a list where want (every lane active):
// one atomic per wave
__device__ __forceinline__ void list_append(uint32_t *list, uint32_t *cnt, bool want, uint32_t i)
{
    const uint64_t m = __ballot(want);
    if (!m)
        return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lead = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == lead)
        base = atomicAdd(cnt, (uint32_t)__popcll(m));
    base = __shfl(base, (int)lead, 64);
    if (want)
        list[base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = i;
}
__device__ __forceinline__ uint32_t mon_class(uint32_t mon)
{
    return mon == 0 ? 0u : mon == MTU_LEN ? 2u : mon == 1u ? 3u : 1u;
}
__device__ __forceinline__ uint32_t trace_word(uint32_t obs, uint32_t source,
                                               uint32_t reason, uint32_t mon)
{
    return (CFC_NT_TRACE + obs) << 16 | source | reason << 20 | mon_class(mon) << 22;
}

// workspace: entry indices [n] (egress: a second array at ctr_stride(n)),
// then the partial slabs; both arrays 16-byte aligned for k_count
__host__ __device__ constexpr uint64_t ctr_stride(uint64_t n) { return (n + 3) & ~3ull; }
#ifndef CFC_UNROLL
#define CFC_UNROLL 1   // headers in flight per thread
#endif
#ifndef CFC_WG_PER_CU
#define CFC_WG_PER_CU 2   // 1024-thread workgroups resident per CU
#endif
constexpr int WAVES_PER_SIMD = 4 * CFC_WG_PER_CU;
constexpr size_t LDS_PER_WG = LDS_BYTES_MAX / CFC_WG_PER_CU;

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
// the same at a 32-bit byte offset from a wave-uniform base: the address is
// then the SGPR base plus a VGPR offset (no 64-bit address arithmetic)
template <class T>
__device__ __forceinline__ T ldo_nt(const T *base, uint32_t off)
{
    return __builtin_nontemporal_load(
        reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + off));
}
template <class T>
__device__ __forceinline__ void sto_nt(T v, T *base, uint32_t off)
{
    __builtin_nontemporal_store(v, reinterpret_cast<T *>(reinterpret_cast<char *>(base) + off));
}
template <class T>
__device__ __forceinline__ void sto(T v, T *base, uint32_t off)
{
    *reinterpret_cast<T *>(reinterpret_cast<char *>(base) + off) = v;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// 16-byte non-temporal load (p 16-byte aligned)
__device__ __forceinline__ uint4 ld_nt4(const uint32_t *p)
{
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint4 ld16(const void *p)
{
    return *reinterpret_cast<const uint4 *>(p);
}

// 16-byte table load that stays ONE load: a plain uint4 load whose upper
// half is only used on some paths gets split by the compiler into two
// dependent 8-byte loads (a second L2 round trip); a buffer load is never
// split.  base: the table (wave-uniform, < 4 GiB), off: byte offset.
__device__ __forceinline__ uint4 ldt16(const void *base, uint32_t off)
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void *>(base), (short)0, 0x7FFFFFFF, 0x00020000);
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Workgroup-shared state: LDS copies of the small tables.  Accessed through
// the extern __shared__ symbol with dword offsets (not through pointers kept
// in a struct, which would lose the LDS address space and turn every read
// into a flat load).
extern __shared__ uint4 cfc_smem[];

struct Lds {
    bool lxc, pfb, polb;          // which tables are in LDS
    uint32_t lxc_off;             // uint4 index of the endpoint slots
    uint32_t pfb_off, polb_off;   // dword index of the Bloom filters
    uint32_t pfb_mask, polb_mask;
};

__device__ __forceinline__ unsigned long long *lds_met()
{
    return reinterpret_cast<unsigned long long *>(cfc_smem);
}
__device__ __forceinline__ uint32_t lds_word(uint32_t off)
{
    return reinterpret_cast<const uint32_t *>(cfc_smem)[off];
}

// ---- compact IPv4 LPM (layout.h): walk from the /16 directory word `e`
// through chunks to a leaf or a prefix list; the first list entry that
// matches is the longest prefix.  Returns the label (0 = no match).
__device__ __forceinline__ uint32_t l4_leaf(const DevTables &T, uint32_t e)
{
    return (e & LPM_INDIRECT) ? T.lbl_ovf[e & LPM_PAYLOAD] : e;
}
__device__ __forceinline__ uint32_t l4_list_leaf(const DevTables &T, uint32_t hi)
{
    const uint32_t l = hi & (LL_INDIRECT | LL_PAYLOAD);
    return (l & LL_INDIRECT) ? T.lbl_ovf[l & LL_PAYLOAD] : l;
}
__device__ __forceinline__ uint32_t l4_lookup(const DevTables &T, uint32_t a,
                                              uint4 d)
{
    // the directory's inline prefixes first (longest first, layout.h)
    const uint32_t e1 = (d.z >> 16) | (d.w << 16);
    if (l4_inline_match(a, d.y))
        return l4_list_leaf(T, (d.y >> 21) | (d.z << 11));
    if (l4_inline_match(a, e1))
        return l4_list_leaf(T, d.w >> 5);
    uint32_t e = d.x;
    uint32_t shift = 16;   // address bits below the current node
    while (e & L4_PTR) {
        const uint32_t cnt = (e >> 24) & 127, off = e & L4_OFF;
        if (cnt == 0) {
            shift -= 8;
            e = T.l4c[off + ((a >> shift) & 255)];
            continue;
        }
        for (uint32_t i = 0; i < cnt; i += 2) {
            const uint4 v = ldt16(T.l4l, (off + i) * 8u);
            const bool m0 = l4_match(a, v.x, v.y);
            if (m0 || l4_match(a, v.z, v.w))
                return l4_list_leaf(T, m0 ? v.y : v.w);
        }
        return 0;   // not reached: a list ends with its node's own prefix
    }
    return l4_leaf(T, e);
}

// ---- endpoint lookup: 16-byte slots, linear probing (layout.h).
// Returns the slot (info VALID) or a zero slot for a miss.
__device__ __forceinline__ uint4 lxc_slot(const DevTables &T, const Lds &S,
                                          uint32_t s)
{
    return S.lxc ? cfc_smem[S.lxc_off + s] : ld16(T.lxc4 + s);
}
__device__ __forceinline__ uint4 lxc_resolve(const DevTables &T, const Lds &S,
                                             uint32_t addr, uint32_t s, uint4 v)
{
    for (;;) {
        if (!(v.w & LXC_VALID))
            return make_uint4(0, 0, 0, 0);
        if (v.x == addr)
            return v;
        s = (s + 1) & T.lxc4_mask;
        v = lxc_slot(T, S, s);
    }
}

// ---- prefilter /32 set: 16-byte buckets of 4 addresses, 0 = free
__device__ __forceinline__ bool pf_resolve(const DevTables &T, uint32_t addr,
                                           uint32_t b, uint4 v)
{
    for (;;) {
        if (v.x == addr || v.y == addr || v.z == addr || v.w == addr)
            return true;
        if (!v.x || !v.y || !v.z || !v.w)
            return false;
        b = (b + 1) & T.pf_fix_mask;
        v = ldt16(T.pf_fix, b * 16u);
    }
}

__device__ __forceinline__ bool bloom_maybe(uint32_t off, uint32_t mask,
                                            uint32_t h)
{
    const uint32_t b = bloom_bits(h);
    return (lds_word(off + ((uint32_t)h & mask)) & b) == b;
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
// (Branch-free: a divergent if here costs more scalar exec-mask work than
// the arithmetic itself.)
__device__ __forceinline__ bool ct_new_dport(uint32_t proto, uint32_t ports,
                                             uint32_t *dport)
{
    const bool tu = (proto == 6) | (proto == 17);
    *dport = tu ? ports >> 16 : ((ports & 0xFF) == 8 ? 8u : 0u);
    return tu | (proto == 1);
}

// ---- conntrack: ct_lookup4 / ct_lookup6 (conntrack.h:467-590, :310-437)
constexpr int CT_NEW = 0, CT_ESTABLISHED = 1, CT_REPLY = 2, CT_RELATED = 3;
constexpr int CT_EGRESS = 0, CT_INGRESS = 1, CT_SERVICE = 2;
constexpr uint32_t CTO_DONE = 4u, CTO_CREATE = 8u;   // per-stage CT byte bits

// The tuple words of the two probes.  k1 is the tuple as loaded (packet
// addresses, L4 ports loaded into {dport, sport}, TUPLE_F_OUT for ingress /
// TUPLE_F_IN for egress): a hit is CT_REPLY, or CT_RELATED when the ICMP type
// set TUPLE_F_RELATED.  k2 = ipv4_ct_tuple_reverse(k1): a hit is
// CT_ESTABLISHED, a miss CT_NEW.  td/ts: tuple->dport/sport of k1; the
// policy port is td after a k1 hit and ts otherwise.
struct CtProbe {
    uint32_t z1, z2, w1, w2, td, ts;
};
template <bool V6>
__device__ __forceinline__ CtProbe ct_probe(uint32_t proto, uint32_t pt,
                                            int dir, uint32_t owner)
{
    CtProbe k;
    // TUPLE_F_OUT / TUPLE_F_IN / TUPLE_F_SERVICE (conntrack.h:487-494)
    uint32_t fl = dir == CT_INGRESS ? 0u : dir == CT_SERVICE ? 4u : 1u;
    if (proto == 6 || proto == 17) {
        k.td = pt & 0xFFFF;
        k.ts = pt >> 16;
    } else {   // ICMP / ICMPv6 (callers drop other protocols first)
        const uint32_t type = pt & 0xFF;
        const bool related = V6 ? (type >= 1 && type <= 4)
                                : (type == 3 || type == 11 || type == 12);
        const uint32_t echo = V6 ? 128u : 8u, reply = V6 ? 129u : 0u;
        k.td = (!related && type == reply) ? echo : 0u;
        k.ts = (!related && type == echo) ? echo : 0u;
        fl |= related ? 2u : 0u;
    }
    k.z1 = k.td | k.ts << 16;
    k.z2 = k.ts | k.td << 16;
    k.w1 = ct_word(proto, fl, owner);
    k.w2 = ct_word(proto, fl ^ 1u, owner);
    return k;
}

// Probe sequence from slot i whose first slot s is already loaded.
__device__ __forceinline__ uint32_t ct4_walk(const DevTables &T, uint32_t i,
                                             uint4 s, uint32_t x, uint32_t y,
                                             uint32_t z, uint32_t w)
{
    for (uint32_t p = 0; p <= T.ct4_probe; p++) {
        if (s.w == 0)
            break;
        if (s.x == x && s.y == y && s.z == z && s.w == w)
            return i;
        i = (i + 1) & T.ct4_mask;
        s = ld16(T.ct4 + i);
    }
    return NONE;
}

__device__ __forceinline__ uint32_t ct4_find(const DevTables &T, uint32_t x,
                                             uint32_t y, uint32_t z, uint32_t w)
{
    if (!T.ct4)
        return NONE;
    const uint32_t i = ct_home4(x, y, z, w) & T.ct4_mask;
    return ct4_walk(T, i, ld16(T.ct4 + i), x, y, z, w);
}

__device__ __forceinline__ uint32_t ct6_find(const DevTables &T, const uint4 &d,
                                             const uint4 &sa, uint32_t z,
                                             uint32_t w)
{
    if (!T.ct6)
        return NONE;
    const uint32_t dw[4] = {d.x, d.y, d.z, d.w}, sw[4] = {sa.x, sa.y, sa.z, sa.w};
    uint32_t i = ct_home6(dw, sw, z, w) & T.ct6_mask;
    for (uint32_t p = 0; p <= T.ct6_probe; p++) {
        const Ct6Slot *e = T.ct6 + i;
        const uint4 t = ld16(&e->z);
        if (t.y == 0)
            break;
        if (t.x == z && t.y == w) {
            const uint4 a = ld16(e->d), b = ld16(e->s);
            if (a.x == d.x && a.y == d.y && a.z == d.z && a.w == d.w &&
                b.x == sa.x && b.y == sa.y && b.z == sa.z && b.w == sa.w)
                return i;
        }
        i = (i + 1) & T.ct6_mask;
    }
    return NONE;
}

// One CT lookup stage: result, hit slot (or NONE), policy port.
struct CtResult {
    int res;
    uint32_t slot, dport;
};
__device__ __forceinline__ CtResult ct_stage4(const DevTables &T, uint32_t sa,
                                              uint32_t da, uint32_t proto,
                                              uint32_t pt, int dir,
                                              uint32_t owner)
{
    const CtProbe k = ct_probe<false>(proto, pt, dir, owner);
    CtResult r;
    if (!T.ct4) {
        r.slot = NONE;
        r.res = CT_NEW;
        r.dport = k.ts;
        return r;
    }
    // k1 and k2 share their home slot (ct_home4): one walk from it to the
    // first free slot answers both lookups — k1 wins wherever it sits
    // (__ct_lookup tries the reply direction first), else the slot where k2
    // was passed.  An ESTABLISHED or NEW packet then costs one probe chain,
    // not two.
    uint32_t i = ct_home4(da, sa, k.z1, k.w1) & T.ct4_mask;
    uint4 s = ld16(T.ct4 + i);
    uint32_t s2 = NONE;
    for (uint32_t p = 0; p <= T.ct4_probe; p++) {
        if (s.w == 0)
            break;
        if (s.x == da && s.y == sa && s.z == k.z1 && s.w == k.w1) {
            r.slot = i;
            r.res = (k.w1 & 0x200u) ? CT_RELATED : CT_REPLY;
            r.dport = k.td;
            return r;
        }
        if (s2 == NONE && s.x == sa && s.y == da && s.z == k.z2 && s.w == k.w2)
            s2 = i;
        i = (i + 1) & T.ct4_mask;
        s = ld16(T.ct4 + i);
    }
    r.slot = s2;
    r.res = s2 != NONE ? CT_ESTABLISHED : CT_NEW;
    r.dport = k.ts;
    return r;
}
__device__ __forceinline__ CtResult ct_stage6(const DevTables &T, const uint4 &sa,
                                              const uint4 &da, uint32_t proto,
                                              uint32_t pt, int dir,
                                              uint32_t owner)
{
    const CtProbe k = ct_probe<true>(proto, pt, dir, owner);
    CtResult r;
    r.slot = NONE;
    r.res = CT_NEW;
    r.dport = k.ts;
    if (!T.ct6)
        return r;
    // one walk for k1 and k2 from their shared home slot (ct_home6), as
    // ct_stage4; a slot's {z, w} words are compared first
    const uint32_t dw[4] = {da.x, da.y, da.z, da.w}, sw[4] = {sa.x, sa.y, sa.z, sa.w};
    uint32_t i = ct_home6(dw, sw, k.z1, k.w1) & T.ct6_mask;
    uint32_t s2 = NONE;
    for (uint32_t p = 0; p <= T.ct6_probe; p++) {
        const Ct6Slot *e = T.ct6 + i;
        const uint4 t = ld16(&e->z);
        if (t.y == 0)
            break;
        const bool m1 = t.x == k.z1 && t.y == k.w1, m2 = s2 == NONE && t.x == k.z2 && t.y == k.w2;
        if (m1 || m2) {
            const uint4 a = ld16(e->d), b = ld16(e->s);
            if (m1 && a.x == da.x && a.y == da.y && a.z == da.z && a.w == da.w &&
                b.x == sa.x && b.y == sa.y && b.z == sa.z && b.w == sa.w) {
                r.slot = i;
                r.res = (k.w1 & 0x200u) ? CT_RELATED : CT_REPLY;
                r.dport = k.td;
                return r;
            }
            if (m2 && a.x == sa.x && a.y == sa.y && a.z == sa.z && a.w == sa.w &&
                b.x == da.x && b.y == da.y && b.z == da.z && b.w == da.w)
                s2 = i;
        }
        i = (i + 1) & T.ct6_mask;
    }
    r.slot = s2;
    r.res = s2 != NONE ? CT_ESTABLISHED : CT_NEW;
    return r;
}

// *monitor of a ct_lookup (conntrack.h:221-285, 587-589) against the entry
// as committed: a miss reports TRACE_PAYLOAD_LEN; a hit runs
// __ct_update_timeout's report decision (the flow's interval of
// CT_REPORT_INTERVAL 5 s passed, or the packet carries TCP flags the
// direction has not seen; :125-185) on a copy of the slot's report state,
// as __ct_lookup's action would (re-open a closing entry: CREATE; RST/FIN:
// CLOSE, always reported); a DNS port captures MTU bytes.
// action: 1 CREATE, 2 CLOSE, 0 UNSPEC (ICMP replies and errors).
__device__ __forceinline__ uint32_t ct_action(bool v6, uint32_t proto, uint32_t pt,
                                              uint32_t meta)
{
    if (proto == 6)
        return (meta & CFC_HF_TCP_CLOSE) ? 2u : 1u;
    if (proto == 17)
        return 1u;
    const uint32_t type = pt & 0xFF;
    const bool unspec = v6 ? ((type >= 1 && type <= 4) || type == 129)
                           : (type == 3 || type == 11 || type == 12 || type == 0);
    return unspec ? 0u : 1u;
}
// ct_update_timeout is declared bool: a reported hit's monitor length is 1
__device__ __forceinline__ uint32_t ct_report(uint32_t &last, uint32_t &acc,
                                              uint32_t fl, uint32_t now)
{
    const uint32_t seen = fl | acc;
    if (last + 5u < now || acc != seen) {
        last = now;
        acc = seen;
        return 1u;
    }
    return 0u;
}
// the same against a given report state t (CtTimer as uint4)
__device__ __forceinline__ uint32_t ct_monitor_of(const DevTables &T, uint4 t, int dir,
                                                  uint32_t action, uint32_t fl)
{
    const bool in = dir == CT_INGRESS;
    uint32_t last = in ? t.x : t.y;
    uint32_t acc = in ? (t.z & 0xFF) : ((t.z >> 8) & 0xFF);
    uint32_t clo = (t.z >> 16) & 3;
    uint32_t m = 0;
    if (clo != 3)   // ct_entry_alive
        m = ct_report(last, acc, fl, T.now);
    if (action == 1u) {
        if (clo)
            m = ct_report(last, acc, fl, T.now);
    } else if (action == 2u) {
        m = TRACE_PAYLOAD_LEN;
    }
    return m;
}
// (st: the family's CtState lines, T.ct_st or T.ct_st + T.ct6_acct_base;
// null: no CT table)
__device__ __forceinline__ uint32_t ct_monitor(const DevTables &T, const CtState *st,
                                               uint32_t slot, int dir, uint32_t action,
                                               uint32_t fl, uint32_t dport)
{
    uint32_t m = TRACE_PAYLOAD_LEN;
    if (slot != NONE && st) {
        const uint4 t = ld16(&st[slot].tm);
        const bool in = dir == CT_INGRESS;
        uint32_t last = in ? t.x : t.y;
        uint32_t acc = in ? (t.z & 0xFF) : ((t.z >> 8) & 0xFF);
        uint32_t clo = (t.z >> 16) & 3;
        m = 0;
        if (clo != 3)   // ct_entry_alive
            m = ct_report(last, acc, fl, T.now);
        if (action == 1u) {
            if (clo)
                m = ct_report(last, acc, fl, T.now);
        } else if (action == 2u) {
            m = TRACE_PAYLOAD_LEN;
        }
    }
    return dport == 0x3500u ? MTU_LEN : m;   // conn_is_dns: htons(53)
}

// the engine's stand-in for skb->hash (cfc.h CFC_FLOW_HASH)
__device__ __forceinline__ uint32_t flow_hash4(uint32_t sa, uint32_t da, uint32_t pt,
                                               uint32_t proto)
{
    const uint32_t lo = min(sa, da), hi = max(sa, da);
    const uint32_t sp = pt & 0xFFFF, dp = pt >> 16;
    const uint32_t pw = min(sp, dp) | (max(sp, dp) << 16);
    return fmix32(lo * 0x9E3779B1u + hi * 0x85EBCA77u + pw * 0xC2B2AE3Du + proto);
}

// ---- load balancing (lb.h) -------------------------------------------------
// one cilium_lb4_services lookup (layout.h): the slot's two uint4, false on
// a miss
__device__ __forceinline__ bool lb4_get(const DevTables &T, uint32_t addr, uint32_t dport,
                                        uint32_t slave, uint4 &a, uint4 &b)
{
    const uint32_t ps = dport | slave << 16;
    uint32_t i = lb4_hash(addr, ps) & T.lb4_mask;
    for (uint32_t p = 0; p <= T.lb4_mask; p++) {
        a = ld16(T.lb4 + 2 * i);
        b = ld16(T.lb4 + 2 * i + 1);
        if (!b.y)
            return false;
        if (a.x == addr && a.y == ps)
            return true;
        i = (i + 1) & T.lb4_mask;
    }
    return false;
}
// lb4_lookup_service (lb.h:604-635): the L4 key while its dport is set (a
// miss clears the caller's dport), then the L3 key; count must be nonzero
__device__ __forceinline__ bool lb4_service(const DevTables &T, uint32_t addr,
                                            uint32_t &dport, uint32_t slave, uint4 &a,
                                            uint4 &b)
{
    if (dport) {
        if (lb4_get(T, addr, dport, slave, a, b) && (a.w >> 16))
            return true;
        dport = 0;
    }
    return lb4_get(T, addr, 0, slave, a, b) && (a.w >> 16);
}
// lb4_rev_nat (lb.h:485-588) on a packet {sa, da, pt} for a CT entry whose
// LB state is lw (ct4_lb): the source back to the service address and port,
// and for a looped-back flow the old source into the destination
__device__ __forceinline__ void lb4_rev_nat(const DevTables &T, uint4 lw, uint32_t proto,
                                            uint32_t &sa, uint32_t &da, uint32_t &pt)
{
    const uint32_t rev = lw.x & 0xFFFF;
    if (!rev || !T.rnat4)
        return;
    const uint2 rn = T.rnat4[rev];
    if (!(rn.y >> 16))
        return;
    const uint32_t port = rn.y & 0xFFFF;
    if (port && (proto == 6 || proto == 17))
        pt = (pt & 0xFFFF0000u) | port;   // reverse_map_l4_port: the sport
    if ((lw.x >> 16) & 1)
        da = sa;
    sa = rn.x;
}
// the service step's flags per header (lb.hip, cfc_api.cpp)
constexpr uint32_t LBF_DROP = 1, LBF_SVC = 2, LBF_LOOP = 4;

// ---- IPv6 services (lb.h:306-481; layout.h lb6 slots) ------------------------
// one cilium_lb6_services lookup: the slot's {port | count, rev_nat | weight}
// word pair (b.y, b.z) and target, false on a miss
__device__ __forceinline__ bool lb6_get(const DevTables &T, uint4 addr, uint32_t dport,
                                        uint32_t slave, uint4 &b, uint4 &tgt)
{
    const uint32_t ps = dport | slave << 16;
    uint32_t i = lb6_hash(addr.x, addr.y, addr.z, addr.w, ps) & T.lb6_mask;
    for (uint32_t p = 0; p <= T.lb6_mask; p++) {
        const uint4 a = ld16(T.lb6 + 3 * i);
        b = ld16(T.lb6 + 3 * i + 1);
        if (!b.w)
            return false;
        if (b.x == ps && a.x == addr.x && a.y == addr.y && a.z == addr.z && a.w == addr.w) {
            tgt = ld16(T.lb6 + 3 * i + 2);
            return true;
        }
        i = (i + 1) & T.lb6_mask;
    }
    return false;
}
// lb6_lookup_service (lb.h:352-381): the L4 key while its dport is set (a
// miss clears the caller's dport), then the L3 key; count must be nonzero
__device__ __forceinline__ bool lb6_service(const DevTables &T, uint4 addr, uint32_t &dport,
                                            uint32_t slave, uint4 &b, uint4 &tgt)
{
    if (dport) {
        if (lb6_get(T, addr, dport, slave, b, tgt) && (b.y >> 16))
            return true;
        dport = 0;
    }
    return lb6_get(T, addr, 0, slave, b, tgt) && (b.y >> 16);
}
// lb6_rev_nat (lb.h:306-319, flags 0) on the packet: its source address and
// port from cilium_lb6_reverse_nat[index], when that holds the index
__device__ __forceinline__ void lb6_rev_nat(const DevTables &T, uint32_t index, uint32_t proto,
                                            uint4 &psa, uint32_t &ppt)
{
    if (!index || !T.rnat6)
        return;
    const uint4 pw = ld16(T.rnat6 + 2 * index + 1);
    if (!(pw.x >> 16))
        return;
    const uint32_t port = pw.x & 0xFFFF;
    if (port && (proto == 6 || proto == 17))
        ppt = (ppt & 0xFFFF0000u) | port;   // reverse_map_l4_port: the sport
    psa = ld16(T.rnat6 + 2 * index);
}
// ---- the CT_SERVICE entry a header's lb4_local / lb6_local finds, in packet
// order (svcorder.hip).  The classify launch looks the entry up as the batch
// found it; the reference's first packet of a flow creates it with its own
// selection (lb.h:711-716, 436-441) and ct_update4/6_slave re-selects it
// when the backend is gone (:737-744, 462-468), so a later packet of the
// same flow takes that slave whatever its own skb->hash.  An override word
// per header carries the entry as the header finds it: SVO_SET | slave
// (| SVO_LOOP: its lb_loopback); 0 = the table's entry.
constexpr uint32_t SVO_SET = 1u << 31, SVO_LOOP = 1u << 29;
struct SvcEntry {
    bool exists;
    uint32_t slave, loop;
};
__device__ __forceinline__ uint32_t svo_word(const SvcEntry &e)
{
    return SVO_SET | (e.loop ? SVO_LOOP : 0u) | (e.slave & 0xFFFF);
}
// lb4_local's effect on the entry for one header (gated as the egress path
// gates it: a valid source, TCP / UDP / ICMP, a service): e as the header
// finds it -> as it leaves it
__device__ __forceinline__ void svc_next4(const DevTables &T, uint32_t da, uint32_t pt,
                                          uint32_t proto, uint32_t hash, SvcEntry &e)
{
    const bool l4 = proto == 6 || proto == 17;
    uint32_t kd = l4 ? pt >> 16 : 0u;
    uint4 a, b, c, d;
    if (!lb4_service(T, da, kd, 0, a, b))
        return;
    uint32_t slave = e.exists ? e.slave : hash % (a.w >> 16) + 1;   // lb4_select_slave
    if (!lb4_get(T, da, kd, slave, c, d) && lb4_service(T, da, kd, slave, c, d))
        slave = hash % (c.w >> 16) + 1;                                // ct_update4_slave
    if (!e.exists)
        e.loop = 0;   // (ct_create4 from lb4_local: the lookup's ct_state, loopback 0)
    e.exists = true;
    e.slave = slave;
}
__device__ __forceinline__ void svc_next6(const DevTables &T, uint4 da_raw, uint32_t pt,
                                          uint32_t proto, uint32_t hash, SvcEntry &e)
{
    const bool l4 = proto == 6 || proto == 17;
    uint32_t kd = l4 ? pt >> 16 : 0u;
    uint4 b, tg, b2, tg2;
    if (!lb6_service(T, da_raw, kd, 0, b, tg))
        return;
    uint32_t slave = e.exists ? e.slave : hash % (b.y >> 16) + 1;   // lb6_select_slave
    if (!lb6_get(T, da_raw, kd, slave, b2, tg2) && lb6_service(T, da_raw, kd, slave, b2, tg2))
        slave = hash % (b2.y >> 16) + 1;                               // ct_update6_slave
    e.exists = true;
    e.slave = slave;
    e.loop = 0;
}

// the engine's skb->hash stand-in for IPv6 (notify.hip flow_hash, fold6)
__device__ __forceinline__ uint32_t fold6w(uint4 a)
{
    uint32_t h = fmix32(a.w);
    h = fmix32(a.z ^ h);
    h = fmix32(a.y ^ h);
    return fmix32(a.x ^ h);
}
__device__ __forceinline__ uint32_t flow_hash6(uint4 sa, uint4 da, uint32_t pt, uint32_t proto)
{
    return flow_hash4(fold6w(sa), fold6w(da), pt, proto);
}

__device__ __forceinline__ uint4 bswap4(uint4 v)
{
    return make_uint4(__builtin_bswap32(v.x), __builtin_bswap32(v.y),
                      __builtin_bswap32(v.z), __builtin_bswap32(v.w));
}

// icmp6_handle (icmp6.h:390-412): neighbour solicitations and echo requests
// to the router are answered, not classified.  It reads the type right after
// the fixed header, so with extension headers it never triggers.
__device__ __forceinline__ bool icmp6_punt(const DevTables &T, uint32_t proto,
                                           uint32_t meta, uint32_t ports, uint4 da)
{
    if (proto != 58 || (meta & CFC_HF_EXTHDR))
        return false;
    const uint32_t type = ports & 0xFF;
    return type == 135 || (type == 128 && da.x == T.router6[0] && da.y == T.router6[1] &&
                           da.z == T.router6[2] && da.w == T.router6[3]);
}

// key of CtState[slot].acct[dir] (k_ct_count), NONE for a miss
__device__ __forceinline__ uint32_t ct_acct_key(uint32_t slot, int dir)
{
    return slot == NONE ? NONE : slot * 2 + (uint32_t)dir;
}
// the {packets, bytes} pair of accounting key k (slot * 2 + dir, slot
// counted from the first IPv4 slot)
__device__ __forceinline__ unsigned long long *ct_acct_at(CtState *st, uint64_t k)
{
    return reinterpret_cast<unsigned long long *>(st[k >> 1].acct) + 2 * (k & 1);
}
// A CT_NEW stage leaves in the same key array a tag instead: CK_MISS | a
// hash of its k2 (owner word included) | 1 when k2 carries TUPLE_F_RELATED
// (an ICMP error's); never NONE.  The packet-order pass compares the
// creates' keys with the dropped CT_NEW stages' through them (ctorder.hip)
// without reading the headers again.  Counting skips every key >= CK_MISS
// (hit keys are slot * 2 + dir < 2^27).
constexpr uint32_t CK_MISS = 0x80000000u;
__device__ __forceinline__ uint32_t ck_miss_tag(uint32_t h, uint32_t w2)
{
    return CK_MISS | (h & 0x7FFFFFFCu) | ((w2 & 0x200u) ? 1u : 0u);
}
__device__ __forceinline__ uint32_t ck_miss4(uint32_t sa, uint32_t da, uint32_t proto,
                                             uint32_t pt, int dir, uint32_t owner)
{
    const CtProbe k = ct_probe<false>(proto, pt, dir, owner);
    return ck_miss_tag(ct_hash4(sa, da, k.z2, k.w2), k.w2);
}
__device__ __forceinline__ uint32_t ck_miss6(const uint4 &sa, const uint4 &da, uint32_t proto,
                                             uint32_t pt, int dir, uint32_t owner)
{
    const CtProbe k = ct_probe<true>(proto, pt, dir, owner);
    return ck_miss_tag(ct_hash4(ct_hash4(sa.x, sa.y, sa.z, sa.w),
                                ct_hash4(da.x, da.y, da.z, da.w), k.z2, k.w2), k.w2);
}

// The apply's work bits (ctapply.hip k_cta_scan_w, ctorder.hip): per 64
// headers of a classify launch two words, one bit per header.  work: a CT
// stage that is not a plain hit on a slot of the launch's table — an allowed
// CT_NEW stage (a create), an ICMP error's CT_NEW stage, a hit the launch
// left no slot for (its key a miss tag or NONE), a delete (CT_ESTABLISHED,
// dropped at the header's last stage), a TCP close (ACTION_CLOSE).  probe:
// a dropped CT_NEW stage (no create; its result changes only when a create
// of the batch writes its key).  Every other stage is a plain hit, which the
// launch's accounting summarised (DevTables.ct_sum).
template <bool TWO>
__device__ __forceinline__ bool wl_want(uint32_t ctb, int32_t ver, uint32_t mt, uint32_t k1,
                                        uint32_t k2, bool &probe)
{
    const int last = (ctb & (CTO_DONE << 4)) ? 1 : 0;
    const bool close = (mt & 0xFF) == 6 && (mt & CFC_HF_TCP_CLOSE);
    bool w = false;
    probe = false;
#pragma unroll
    for (int st = 0; st < (TWO ? 2 : 1); st++) {
        const uint32_t cs = (ctb >> (4 * st)) & 0xF;
        if (!(cs & CTO_DONE))
            continue;
        const uint32_t res = cs & 3u, key = st ? k2 : k1;
        const bool dropped = st == last && ver == DROP_POLICY;
        const bool pr = res == 0 && dropped && key != NONE && key >= CK_MISS && !(key & 1);
        probe |= pr;
        w |= (res == 0 && !pr) || close || (res != 0 && key >= CK_MISS) ||
             (res == 1 && dropped);
    }
    return w;
}

// CONNTRACK_ACCOUNTING (lxc_config.h:50, conntrack.h:247-257): the hit
// entry's rx (ingress) or tx (egress) packets/bytes
__device__ __forceinline__ void ct_account(const DevTables &T, uint32_t slot,
                                           int dir, uint32_t len)
{
    if (slot == NONE)
        return;
    unsigned long long *a = ct_acct_at(T.ct_st, slot * 2 + (uint32_t)dir);
    atomicAdd(a, 1ull);
    atomicAdd(a + 1, (unsigned long long)len);
}

// __policy_can_access (policy.h:46-110) with cb[CB_POLICY] == 0, split in
// two halves so the first probe overlaps other headers' lookups:
// policy_issue() filters the three keys and loads the first slot of the
// first key that may exist; policy_resolve() walks the keys in the
// reference's order (L4, L3, wildcard port; fragments: L3 only).
struct PolicyProbe {
    uint32_t id, pp;    // identity; dport | proto << 16
    uint32_t eg;        // egress << 24
    uint32_t maybe;     // bit j: key j may exist (and applies)
    uint32_t j, s;      // key and slot of the issued probe (j = 3: none)
    uint4 v;
    // key j by masking, not by selecting among stored keys: the compiler
    // turns a 3-way select on a per-lane index into a scratch-memory table
    __device__ __forceinline__ uint32_t lo(uint32_t i) const
    {
        return id & (0u - (uint32_t)(i != 2));
    }
    __device__ __forceinline__ uint32_t hi(uint32_t i) const
    {
        return (pp & (0u - (uint32_t)(i != 1))) | eg;
    }
    __device__ __forceinline__ uint64_t key(uint32_t i) const
    {
        return ((uint64_t)hi(i) << 32) | lo(i);
    }
    __device__ __forceinline__ uint32_t pre(uint32_t i) const
    {
        return pol_key_pre(lo(i), hi(i));
    }
};

__device__ __forceinline__ void policy_probe_key(const DevTables &T,
                                                 uint32_t base, uint32_t mask,
                                                 PolicyProbe &P)
{
    P.j = P.maybe ? __builtin_ctz(P.maybe) : 3;
    if (P.j < 3) {
        P.s = pol_slot(P.pre(P.j), mask);
        P.v = ldt16(T.pol, (base + P.s) * 16u);
    }
}

__device__ __forceinline__ void policy_issue(const DevTables &T, const Lds &S,
                                             uint32_t base, uint32_t mask,
                                             uint32_t id, uint32_t dport,
                                             uint32_t proto, uint32_t egress,
                                             bool frag, PolicyProbe &P)
{
    // keys 0: L4 {id, dport, proto}, 1: L3 {id, 0, 0}, 2: wildcard port
    // {0, dport, proto}, all with the direction bit
    P.id = id;
    P.pp = dport | (proto << 16);
    P.eg = egress << 24;
    P.maybe = frag ? 2u : 7u;                // policy.h:61,85
    if (S.polb) {
        const uint32_t salt = pol_bloom_salt(base);
        const bool m0 = bloom_maybe(S.polb_off, S.polb_mask, pol_bloom_hash(salt, P.pre(0)));
        const bool m1 = bloom_maybe(S.polb_off, S.polb_mask, pol_bloom_hash(salt, P.pre(1)));
        const bool m2 = bloom_maybe(S.polb_off, S.polb_mask, pol_bloom_hash(salt, P.pre(2)));
        P.maybe &= (uint32_t)m0 | (uint32_t)m1 << 1 | (uint32_t)m2 << 2;
    }
    policy_probe_key(T, base, mask, P);
}

// Returns the verdict (<0 drop) and the matched counter (or NONE).  Works
// on register copies of the probe state (writing through a pointer into the
// per-header state array would keep that array out of registers).
struct PolicyResult {
    int verdict;
    uint32_t ctr;
};
__device__ __forceinline__ PolicyResult policy_resolve_walk(const DevTables &T,
                                                            uint32_t base,
                                                            uint32_t mask,
                                                            const PolicyProbe &P0)
{
    uint32_t maybe = P0.maybe, j = P0.j, s = P0.s;
    uint4 v = P0.v;
    uint32_t ctr = NONE;
    int verdict = DROP_POLICY;   // (DROP_FRAG_NOSUPPORT also -> DROP_POLICY)
    while (j < 3) {
        const uint64_t want = P0.key(j);
        bool hit = false;
        for (;;) {
            const uint64_t key = ((uint64_t)v.y << 32) | v.x;
            if (key == want) {
                hit = true;
                break;
            }
            if (key == POL_EMPTY)
                break;
            s = (s + 1) & mask;
            v = ldt16(T.pol, (base + s) * 16u);
        }
        if (hit) {
            ctr = v.w;
            verdict = j == 1 ? TC_ACT_OK : (int)(v.z & 0xFFFF);
            break;
        }
        maybe &= ~(1u << j);   // a false positive of the filter
        j = maybe ? __builtin_ctz(maybe) : 3;
        if (j < 3) {
            s = pol_slot(P0.pre(j), mask);
            v = ldt16(T.pol, (base + s) * 16u);
        }
    }
    return PolicyResult{verdict, ctr};
}
// The issued probe decides most headers: its slot holds the key, or is
// empty with no other key that may exist.  Only the rest walk (a probe
// sequence, a Bloom false positive, the next key): kept out of the common
// path, whose wait at the walk's loop would otherwise cover every load
// issued after the probe (vmcnt counts in issue order).
__device__ __forceinline__ PolicyResult policy_resolve(const DevTables &T,
                                                       uint32_t base,
                                                       uint32_t mask,
                                                       const PolicyProbe &P0)
{
    const uint32_t j = P0.j;
    const uint64_t key = ((uint64_t)P0.v.y << 32) | P0.v.x;
    const bool hit = j < 3 && key == P0.key(j);
    const bool done = j >= 3 || hit || (key == POL_EMPTY && !(P0.maybe & ~(1u << j)));
    if (done)
        return hit ? PolicyResult{j == 1 ? TC_ACT_OK : (int)(P0.v.z & 0xFFFF), P0.v.w}
                   : PolicyResult{DROP_POLICY, NONE};
    return policy_resolve_walk(T, base, mask, P0);
}

__device__ __forceinline__ PolicyResult policy_access(
    const DevTables &T, const Lds &S, uint32_t base, uint32_t mask, uint32_t id,
    uint32_t dport, uint32_t proto, uint32_t egress, bool frag)
{
    PolicyProbe P;
    policy_issue(T, S, base, mask, id, dport, proto, egress, frag, P);
    return policy_resolve(T, base, mask, P);
}

// Per-thread update_metrics counts (bytes in u32: a thread sees at most
// 65536 headers between flushes, 65536 x 65535 < 2^32).
template <int N>
struct MetAcc {
    uint32_t cnt[N > 0 ? N : 1], byt[N > 0 ? N : 1];
    __device__ __forceinline__ void clear()
    {
#pragma unroll
        for (int k = 0; k < N; k++)
            cnt[k] = byt[k] = 0;
    }
    __device__ __forceinline__ void add(uint32_t key, uint32_t len)
    {
#pragma unroll
        for (int k = 0; k < N; k++) {
            const bool m = key == (uint32_t)k;
            cnt[k] += m;
            byt[k] += m ? len : 0u;
        }
    }
    // whole-wave sums into the LDS histogram (uniform control flow)
    __device__ __forceinline__ void flush(unsigned long long *s_met)
    {
#pragma unroll
        for (int k = 0; k < N; k++) {
            uint32_t c = cnt[k];
            uint64_t b = byt[k];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                c += __shfl_xor(c, o);
                b += __shfl_xor(b, o);
            }
            if ((threadIdx.x & 63) == 0 && c) {
                atomicAdd(&s_met[2 * k], (unsigned long long)c);
                atomicAdd(&s_met[2 * k + 1], (unsigned long long)b);
            }
        }
        clear();
    }
};

// the policy counter key of a header (CountArgs.ctr)
__device__ __forceinline__ uint32_t ctr_key(const CountArgs &C, uint32_t ctr,
                                            uint32_t len)
{
    return ctr == NONE ? KEY_NONE : C.ctr_packed ? (ctr | len << 16) : ctr;
}
// the identity counter key of a policy verdict (CountArgs.id), KEY_NONE
// when the identity has no histogram range (id_count then)
__device__ __forceinline__ uint32_t id_key(const DevTables &T, uint32_t ident,
                                           bool drop, uint32_t len)
{
    const bool packed = ident < ID_PACK_LIMIT && ((T.id_cover >> id_range_of(ident)) & 1);
    return packed ? ((ident << 1 | (uint32_t)drop) | len << 16) : KEY_NONE;
}
// a per-identity counter bumped directly: identities outside every
// histogram range (from skb->mark, not in the ipcache) — rare, so plain
// global atomics
__device__ __forceinline__ void id_count(const CountArgs &C, uint32_t dir,
                                         uint32_t ident, bool drop, uint32_t len)
{
    unsigned long long *p =
        reinterpret_cast<unsigned long long *>(C.g_id) + id_index(dir, ident, drop);
    atomicAdd(p, 1ull);
    atomicAdd(p + 1, (unsigned long long)len);
}

template <class W>
__device__ __forceinline__ void lds_copy(W *dst, const W *src, uint32_t n)
{
    for (uint32_t j = threadIdx.x; j < n; j += BLOCK)
        dst[j] = src[j];
}

}  // namespace

}  // namespace cfc
