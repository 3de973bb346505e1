// IPv6 verdict kernel for gfx950 (MI355X): k_classify_v6.
//
// Same contract as k_classify_v4 (classify.hip): one pass over a SoA batch
// writes verdict, identity, action and the policy-entry index per header;
// the shared counter kernels (launch_counters) turn the indices into
// packets/bytes.  What differs is the address work:
//   * the ipcache is a 1M-prefix IPv6 LPM (layout.h Lpm6): lengths are
//     probed longest first, each group of lengths screened by one 8-byte
//     Bloom word (L2-resident), so a lookup is usually one Bloom load plus
//     one slot (Infinity Cache): 16 bytes, one load, for the /32-/64 mass,
//     32 bytes, two loads, beyond /64;
//   * endpoints are 32-byte slots keyed by the full address, copied to LDS
//     when the table is small;
//   * the prefilter's exact /128 set and its LPM deny list are Lpm6 tables.
// The per-header work is straight-line: the lookup chain of one header is
// short and the 32 resident waves per CU keep enough of them in flight.
//
// Reference semantics restated here (file:line in /root/reference):
//   ingress   bpf_netdev.c:128-153 (identity from skb->mark), :172-275
//             handle_ipv6 (ipv6_hdrlen drops, icmp6_handle, ipcache
//             override unless CLUSTER_ID), l3.h ipv6_local_delivery,
//             bpf_lxc.c:753-895 ipv6_policy + tail_ipv6_policy
//   egress    bpf_lxc.c:112-436 ipv6_l3_from_lxc / handle_ipv6 (icmp6
//             punt, is_valid_lxc_src_ip, dst identity with the router /64
//             as CLUSTER_ID)
//   ct ports  conntrack.h ct_lookup6 (ICMPv6 echo request -> 128)
//   xdp       bpf_xdp.c:132-156 check_v6
#include "kern_common.hpp"

namespace cfc {

namespace {

constexpr int DROP_INVALID_EXTHDR = -156, DROP_FRAG_NOSUPPORT = -157;
constexpr int VERDICT_PUNT = CFC_VERDICT_PUNT;

// update_metrics keys (reason, direction) per mode
// (egress: + 2 keys for the stage-2 per-identity counters, classify.hip)
constexpr int LDS_MET6_U64 = 22;   // 2 x 11 keys
template <int MODE>
constexpr int met6_n()
{
    return MODE == CFC_MODE_EGRESS ? 9 : MODE == CFC_MODE_XDP ? 0 : 6;
}
template <int MODE>
constexpr int acc6_n()
{
    return met6_n<MODE>() + (MODE == CFC_MODE_EGRESS ? 2 : 0);
}
template <int MODE>
__host__ __device__ constexpr uint32_t met6_reason_dir(int k)
{
    constexpr uint32_t eg[9][2] = {{0, 2},   {132, 2}, {133, 2}, {137, 2}, {140, 2},
                                   {156, 2}, {157, 2}, {0, 1},   {133, 1}};
    constexpr uint32_t in[6][2] = {{0, 1},   {133, 1}, {137, 1},
                                   {140, 1}, {156, 1}, {157, 1}};
    return MODE == CFC_MODE_EGRESS ? eg[k][0] * METRIC_DIRS + eg[k][1]
                                   : in[k][0] * METRIC_DIRS + in[k][1];
}
template <int MODE>
__device__ __forceinline__ uint32_t mkey6(int reason, int dir)
{
    if (MODE == CFC_MODE_EGRESS) {
        if (dir == METRIC_INGRESS)
            return reason == 0 ? 7u : 8u;
        switch (reason) {
        case 0: return 0;
        case -132: return 1;
        case -133: return 2;
        case -137: return 3;
        case -140: return 4;
        case -156: return 5;
        default: return 6;   // -157
        }
    }
    switch (reason) {
    case 0: return 0;
    case -133: return 1;
    case -137: return 2;
    case -140: return 3;
    case -156: return 4;
    default: return 5;       // -157
    }
}

// ---- IPv6 LPM (layout.h Lpm6): the label of the longest prefix holding the
// host-order address a (a matched label 0 shadows shorter prefixes, as the
// reference's trie does), def_label when none
// The first group's Bloom word is a separate step (lpm6_bloom0) so that the
// first loads of independent lookups of one header go out together.
// loff: the dword offset of the table's length list in LDS (LdsPlan6)
__device__ __forceinline__ uint64_t lpm6_bloom0(const Lpm6 &P, uint32_t loff, uint4 a)
{
    if (!P.nlen)
        return 0;
    const uint32_t w[4] = {a.x, a.y, a.z, a.w};
    return P.bloom[l6_group_hash(w, (lds_word(loff) >> 8) & 255) & P.bloom_mask];
}
__device__ __forceinline__ uint32_t lpm6_lookup(const Lpm6 &P, uint32_t loff, uint4 a,
                                                uint64_t bw0)
{
    const uint32_t w[4] = {a.x, a.y, a.z, a.w};
    uint64_t bw = bw0;
    for (uint32_t j = 0; j < P.nlen; j++) {
        const uint32_t e = lds_word(loff + j);   // uniform
        const uint32_t len = e & 255;
        if ((e & L6_GROUP_FIRST) && j)
            bw = P.bloom[l6_group_hash(w, (e >> 8) & 255) & P.bloom_mask];
        const uint32_t m0 = a.x & l6_word_mask(len, 0), m1 = a.y & l6_word_mask(len, 1),
                       m2 = a.z & l6_word_mask(len, 2), m3 = a.w & l6_word_mask(len, 3);
        const uint32_t h = l6_hash(m0, m1, m2, m3, len);
        const uint64_t b = l6_bloom_bits(h);
        if ((bw & b) != b)
            continue;
        if (len <= 64) {   // (uniform) one 16-byte load per probe: {w0, w1, label, len}
            for (uint32_t s = h & P.mask64;; s = (s + 1) & P.mask64) {
                const uint4 k = ld16(P.slots64 + s);
                if (k.w == len && k.x == m0 && k.y == m1)
                    return k.z;
                if (!k.w)
                    break;
            }
            continue;
        }
        for (uint32_t s = h & P.mask;; s = (s + 1) & P.mask) {
            const uint4 k = ld16(&P.slots[s].w[0]);
            const uint4 v = ld16(&P.slots[s].label);   // {label, len, 0, 0}
            if (v.y == len && k.x == m0 && k.y == m1 && k.z == m2 && k.w == m3)
                return v.x;
            if (!v.y)
                break;
        }
    }
    return P.def_label;
}
__device__ __forceinline__ uint32_t lpm6_lookup(const Lpm6 &P, uint32_t loff, uint4 a)
{
    return lpm6_lookup(P, loff, a, lpm6_bloom0(P, loff, a));
}

// ---- endpoints: {pol_base, pol_mask, info, 0} of the slot holding the raw
// address, zeros when it is not local
__device__ __forceinline__ uint4 lxc6_find(const DevTables &T, bool lds,
                                           uint32_t lds_off, uint4 raw)
{
    if (!T.lxc6)
        return make_uint4(0, 0, 0, 0);
    uint32_t s = l6_hash(raw.x, raw.y, raw.z, raw.w, L6_LXC_TAG) & T.lxc6_mask;
    for (;;) {
        uint4 k, v;
        if (lds) {
            k = cfc_smem[lds_off + 2 * s];
            v = cfc_smem[lds_off + 2 * s + 1];
        } else {
            k = ld16(&T.lxc6[s].a[0]);
            v = ld16(&T.lxc6[s].pol_base);
        }
        if (!(v.z & LXC_VALID))
            return make_uint4(0, 0, 0, 0);
        if (k.x == raw.x && k.y == raw.y && k.z == raw.z && k.w == raw.w)
            return v;
        s = (s + 1) & T.lxc6_mask;
    }
}

// tuple->dport of a CT_NEW ct_lookup6: TCP/UDP dport, ICMPv6 echo request
// -> 128 (its type), other ICMPv6 -> 0, anything else DROP_CT_UNKNOWN_PROTO
__device__ __forceinline__ bool ct6_new_dport(uint32_t proto, uint32_t ports,
                                              uint32_t *dport)
{
    if (proto == 6 || proto == 17) {
        *dport = ports >> 16;
        return true;
    }
    *dport = (ports & 0xFF) == 128 ? 128u : 0u;
    return proto == 58;
}

// LDS image of a v6 launch: metrics | endpoint slots | policy Bloom | the
// length lists of the three Lpm6 tables (ipcache, prefilter fix, dyn): a
// lookup reads its next length from LDS, not by a dependent global load
struct LdsPlan6 {
    uint32_t lxc_slots, pol_words, pf_words, nlens;
    __host__ __device__ size_t bytes() const
    {
        return 8ull * LDS_MET6_U64 + 32ull * lxc_slots + 4ull * pol_words + 4ull * pf_words +
               4ull * nlens;
    }
};

__host__ LdsPlan6 lds_plan6(const DevTables &T)
{
    LdsPlan6 p;
    p.lxc_slots = (T.lxc6 && T.lxc6_lds) ? T.lxc6_mask + 1 : 0;
    p.pol_words = T.pol_bloom ? T.pol_bloom_words : 0;
    p.pf_words = T.pf6_bloom ? T.pf6_bloom_words : 0;
    p.nlens = T.ipc6.nlen + T.pf6_fix.nlen + T.pf6_dyn.nlen;
    if (p.bytes() > LDS_PER_WG)   // (the prefilter's filter is an optimisation: drop it first)
        p.pf_words = 0;
    return p;
}

// a policy verdict's per-identity counter: its histogram key, or a direct
// atomic for identities outside every histogram range
__device__ __forceinline__ uint32_t id_event(const DevTables &T, const CountArgs &C,
                                             uint32_t dir, uint32_t ident, bool drop,
                                             uint32_t len, bool valid)
{
    const uint32_t k = id_key(T, ident, drop, len);
    if (k == KEY_NONE && valid)
        id_count(C, dir, ident, drop, len);
    return k;
}

// The egress service step of ipv6_l3_from_lxc (bpf_lxc.c:149-167):
// lb6_extract_key, lb6_lookup_service and lb6_local (lb.h:336-481) against
// the tables as committed (the batch's CT_SERVICE creates are folded in by
// cfc_ct_apply_v6).  A matched service moves the packet's daddr (pda) to the
// backend and its dport (ppt) to the backend's port; returns true for
// DROP_NO_SERVICE.
__device__ __forceinline__ bool lb6_egress(const DevTables &T, const EgressArgs &E,
                                           const cfc_hdr_v6 &in, uint64_t i, uint4 sa_raw,
                                           uint4 da_raw, uint32_t proto, uint32_t pt, uint4 &psa,
                                           uint4 &pda, uint32_t &ppt, uint32_t &rev)
{
    (void)psa;
    const bool l4 = proto == 6 || proto == 17;
    if (!T.lb6 || (!l4 && proto != 58))   // other protocols skip the step
        return false;
    uint32_t kd = l4 ? pt >> 16 : 0u;
    uint4 b, tg;
    if (!lb6_service(T, da_raw, kd, 0, b, tg))
        return false;
    // lb6_local: ct_lookup6(CT_SERVICE), the tuple as loaded, one probe; a
    // hit's slave from the entry, else lb6_select_slave: hash % count + 1
    const CtProbe k = ct_probe<true>(proto, pt, CT_SERVICE, E.ct_owner);
    // (an entry an earlier header of the batch created or re-slaved: E.svo)
    const uint32_t ov = E.svo ? E.svo[i] : 0u;
    const uint32_t slot = (ov & SVO_SET) ? NONE : ct6_find(T, da_raw, sa_raw, k.z1, k.w1);
    uint32_t slave;
    if (ov & SVO_SET) {
        slave = ov & 0xFFFF;
    } else if (slot != NONE) {
        slave = T.ct6_lb ? ld16(T.ct6_lb + slot).y : 0u;
    } else {
        const uint32_t h = in.hash ? in.hash[i] : flow_hash6(sa_raw, da_raw, pt, proto);
        slave = h % (b.y >> 16) + 1;
    }
    uint4 b2, tg2;
    bool ok = lb6_get(T, da_raw, kd, slave, b2, tg2);   // lb6_lookup_slave
    if (!ok)   // the fall-back: the key as it stands, slave set
        ok = lb6_service(T, da_raw, kd, slave, b2, tg2);
    if (!ok)
        return true;
    pda = tg2;   // lb6_xlate
    rev = b2.z & 0xFFFF;   // (state->rev_nat_index, ct_create6's)
    const uint32_t port = b2.y & 0xFFFF;
    if (port && kd != port && l4)
        ppt = (ppt & 0xFFFFu) | port << 16;
    return false;
}

// LB: the launch has an IPv6 load balancer or wants the packet outputs —
// the egress service step (lb6_local), reverse NAT of hits (lb6_rev_nat) and
// ipv6_policy's daddr rewrite are followed, and cfc_out.pkt_* written
template <int MODE, bool CT, bool NT, bool LB>
__global__ __launch_bounds__(BLOCK, WAVES_PER_SIMD) void k_classify_v6(
    DevTables T, LdsPlan6 L, cfc_hdr_v6 in, cfc_out out, EgressArgs E,
    CountArgs C, uint64_t per_block)
{
    constexpr bool XDP = MODE == CFC_MODE_XDP || MODE == CFC_MODE_FULL;
    constexpr bool EGR = MODE == CFC_MODE_EGRESS;
    // LDS image (uint4 units): metrics | endpoint slots | pol Bloom |
    // prefilter Bloom | the length lists
    unsigned long long *s_met = lds_met();
    const uint32_t lxc_off = LDS_MET6_U64 / 2;
    const uint32_t pol4 = lxc_off + 2 * L.lxc_slots;
    const bool lxc_lds = L.lxc_slots != 0;
    Lds S;
    const uint32_t pf4 = pol4 + L.pol_words / 4;
    S.lxc = false;
    S.pfb = L.pf_words != 0;
    S.pfb_off = 4 * pf4;
    S.pfb_mask = L.pf_words - 1;
    S.polb = L.pol_words != 0;
    S.polb_off = 4 * pol4;
    S.polb_mask = L.pol_words - 1;
    for (uint32_t j = threadIdx.x; j < (uint32_t)LDS_MET6_U64; j += BLOCK)
        s_met[j] = 0;
    // the apply's work bits (E.wbits / E.wprobe)
    constexpr bool WL = CT && MODE != CFC_MODE_XDP && !LB;
    lds_copy(cfc_smem + lxc_off, reinterpret_cast<const uint4 *>(T.lxc6),
             2 * L.lxc_slots);
    lds_copy(cfc_smem + pol4, reinterpret_cast<const uint4 *>(T.pol_bloom),
             L.pol_words / 4);
    lds_copy(cfc_smem + pf4, reinterpret_cast<const uint4 *>(T.pf6_bloom), L.pf_words / 4);
    // the length lists (dword offsets)
    const uint32_t lo_ipc = 4 * pf4 + L.pf_words;
    const uint32_t lo_fix = lo_ipc + T.ipc6.nlen, lo_dyn = lo_fix + T.pf6_fix.nlen;
    {
        uint32_t *lw = reinterpret_cast<uint32_t *>(cfc_smem);
        for (uint32_t j = threadIdx.x; j < L.nlens; j += BLOCK)
            lw[lo_ipc + j] = j < T.ipc6.nlen ? T.ipc6.lens[j]
                           : j < T.ipc6.nlen + T.pf6_fix.nlen ? T.pf6_fix.lens[j - T.ipc6.nlen]
                           : T.pf6_dyn.lens[j - T.ipc6.nlen - T.pf6_fix.nlen];
    }
    __syncthreads();

    const uint64_t start = (uint64_t)blockIdx.x * per_block;
    const uint64_t end = min(in.n, start + per_block);
    const uint32_t *sa_in = reinterpret_cast<const uint32_t *>(in.saddr);
    const uint32_t *da_in = reinterpret_cast<const uint32_t *>(in.daddr);
    MetAcc<acc6_n<MODE>()> acc;
    acc.clear();
    uint32_t iter = 0;
    for (uint64_t base = start; base < end; base += BLOCK) {
        // lanes past the end redo the slice's last header (see r1_load)
        const bool valid = base + threadIdx.x < end;
        const uint64_t i = valid ? base + threadIdx.x : end - 1;
        const uint4 sa_raw = ld_nt4(sa_in + 4 * i);
        const uint4 da_raw = ld_nt4(da_in + 4 * i);
        const uint32_t pt = ld_nt(in.ports + i);
        const uint32_t mt = ld_nt(in.meta + i);
        const uint32_t mk = in.mark ? ld_nt(in.mark + i) : 0u;
        const uint32_t tfl = (in.tcp_flags && (mt & 0xFF) == 6) ? (uint32_t)in.tcp_flags[i] : 0u;
        const uint4 sa = bswap4(sa_raw), da = bswap4(da_raw);
        const uint32_t proto = mt & 0xFF;
        // the packet as the programs leave it (LB launches)
        uint4 psa = sa_raw, pda = da_raw;
        uint32_t ppt = pt;

        int act = TC_ACT_OK, ver = 0;
        uint32_t ident = 0, met0 = NONE, met1 = NONE, ctr0 = NONE, ctr1 = NONE;
        uint32_t ctb = 0;   // CT byte (cfc.h CFC_CT_*)
        uint32_t ck1 = NONE, ck2 = NONE;   // CT accounting keys per stage
        uint32_t idw = KEY_NONE, ev2 = 0;  // identity counter key; stage-2 event
        uint32_t evw = 0;                  // trace event word (forwarded)
        bool nat = false, natdrop = false; // NAT64: the hop decides; can't translate
        uint32_t svc_rev = 0;              // the service's rev_nat_index (LB)
        const uint32_t len = mt >> 16;
        // the Bloom words of the prefilter's and the ipcache's lookups of
        // this header's address, loaded together (egress with a load
        // balancer looks up the address after its service step instead)
        // (the prefilter's exact set: its LDS filter first, when it has one)
        const bool pf_maybe = XDP && (!S.pfb || bloom_maybe(S.pfb_off, S.pfb_mask,
                                                            pf6_bloom_hash(sa.x, sa.y, sa.z, sa.w)));
        const uint64_t bwf = (XDP && !S.pfb) ? lpm6_bloom0(T.pf6_fix, lo_fix, sa) : 0ull;
        const uint64_t bwi = MODE == CFC_MODE_XDP ? 0ull
                           : !EGR ? lpm6_bloom0(T.ipc6, lo_ipc, sa)
                           : !LB  ? lpm6_bloom0(T.ipc6, lo_ipc, da) : 0ull;
        const uint4 drec = lxc6_find(T, lxc_lds, lxc_off, da_raw);
        const bool local = (drec.z & LXC_VALID) != 0;
        // the endpoint the packet is delivered to (egress: by the packet's
        // daddr after the service step)
        uint4 erec = drec;
        bool done = false;
        if (XDP) {
            bool deny = lpm6_lookup(T.pf6_dyn, lo_dyn, sa) != 0;
            if (!deny && pf_maybe)
                deny = (S.pfb ? lpm6_lookup(T.pf6_fix, lo_fix, sa)
                              : lpm6_lookup(T.pf6_fix, lo_fix, sa, bwf)) != 0;
            const bool drop = deny || !local;
            if (MODE == CFC_MODE_XDP || drop) {
                act = drop ? XDP_DROP : XDP_PASS;
                ver = drop ? CFC_DROP_PREFILTER : 0;
                done = true;
            }
        }
        if (!done) {
            uint32_t dport;
            const bool known = ct6_new_dport(proto, pt, &dport);
            const int xd = proto == 59 ? DROP_INVALID_EXTHDR
                         : proto == 44 ? DROP_FRAG_NOSUPPORT : 0;
            const bool punt = icmp6_punt(T, proto, mt, pt, da);
            const bool ifx = (drec.z & LXC_IFINDEX) != 0;
            if (!EGR) {
                // handle_identity_from_host (bpf_netdev.c:128-153)
                const uint32_t magic = mk & 0xF00u;
                bool skip_proxy = false;
                if (magic == 0xA00u || magic == 0xB00u) {
                    ident = ((mk & 0xFF) << 16) | (mk >> 16);
                    skip_proxy = magic == 0xA00u;
                } else {
                    ident = magic == 0xC00u ? HOST_ID : WORLD_ID;
                }
                // a NAT46 hop (tail_ipv4_to_ipv6 -> tail_ipv6_policy,
                // bpf_lxc.c:1098-1110): the IPv4 path's source identity, and
                // the skip-proxy mark it carried in tc_index
                const bool hop = E.nat_id != nullptr;
                if (hop)
                    ident = E.nat_id[i];
                if (xd) {   // send_drop_notify_error: no identity recorded
                    act = TC_ACT_SHOT;
                    ver = xd;
                    ident = 0;
                    met0 = mkey6<MODE>(xd, METRIC_INGRESS);
                } else if (punt && !hop) {
                    ver = VERDICT_PUNT;
                    ident = 0;
                } else {
                    // handle_ipv6 (:203-213): reserved identities take the
                    // ipcache's unless it says CLUSTER_ID
                    if (ident < HEALTH_ID && !hop) {
                        const uint32_t label = lpm6_lookup(T.ipc6, lo_ipc, sa, bwi);
                        if (label && label != CLUSTER_ID)
                            ident = label;
                    }
                    if (local && !(drec.z & LXC_HOST)) {
                        if (!(drec.z & LXC_HAS_POLICY)) {
                            act = TC_ACT_SHOT;
                            ver = DROP_MISSED_TAIL_CALL;
                            met0 = mkey6<MODE>(DROP_MISSED_TAIL_CALL, METRIC_INGRESS);
                        } else if (!known) {
                            act = TC_ACT_SHOT;
                            ver = DROP_CT_UNKNOWN_PROTO;
                            met0 = mkey6<MODE>(DROP_CT_UNKNOWN_PROTO, METRIC_INGRESS);
                            if (LB)   // (ipv6_policy's rewrite precedes its ct_lookup6)
                                pda.w &= 0xFFFF0000u;
                        } else {
                            // ipv6_policy's ct_lookup6 (bpf_lxc.c:808)
                            CtResult c{CT_NEW, NONE, dport};
                            if (CT) {
                                const uint32_t own = ct_owner_word(drec.z & 0xFFFF,
                                                                   (drec.z & LXC_CT_LOCAL) != 0);
                                c = ct_stage6(T, sa_raw, da_raw, proto, pt, CT_INGRESS, own);
                                ck1 = c.slot != NONE
                                          ? ct_acct_key(c.slot + T.ct6_acct_base, CT_INGRESS)
                                      : c.res == CT_NEW
                                          ? ck_miss6(sa_raw, da_raw, proto, pt, CT_INGRESS, own)
                                          : NONE;
                            }
                            if (LB) {
                                // ipv6_policy (:785-815): the packet's daddr
                                // loses its last word's low 16 bits; a hit whose
                                // entry has a rev_nat_index is reverse-NATed
                                pda.w &= 0xFFFF0000u;
                                if (CT && c.slot != NONE && T.ct6_lb)
                                    lb6_rev_nat(T, ld16(T.ct6_lb + c.slot).x, proto, psa, ppt);
                            }
                            const bool reply = CT && c.res >= CT_REPLY;
                            const PolicyResult pr = policy_access(
                                T, S, drec.x, drec.y, ident, c.dport, proto, 0, false);
                            ctr0 = pr.ctr;
                            if (CT)
                                ctb = (uint32_t)c.res | CTO_DONE |
                                      ((c.res == CT_NEW && pr.verdict >= 0) ? CTO_CREATE : 0u);
                            idw = id_event(T, C, ID_DIR_INGRESS, ident,
                                           pr.verdict < 0 && !reply, len, valid);
                            if (pr.verdict < 0 && !reply) {
                                act = TC_ACT_SHOT;
                                ver = DROP_POLICY;
                                met0 = mkey6<MODE>(DROP_POLICY, METRIC_INGRESS);
                            } else {
                                const int v = skip_proxy ? 0 : pr.verdict;
                                const bool prox = v > 0 && !reply;
                                act = (prox || ifx) ? TC_ACT_REDIRECT : TC_ACT_OK;
                                ver = prox ? v : 0;
                                met0 = prox ? NONE : mkey6<MODE>(0, METRIC_INGRESS);
                                if (NT)   // TRACE_TO_PROXY / TRACE_TO_LXC (:873)
                                    evw = trace_word(
                                        prox ? OBS_TO_PROXY : OBS_TO_LXC, drec.z & 0xFFFF,
                                        (uint32_t)c.res,
                                        ct_monitor(T, CT ? T.ct_st + T.ct6_acct_base : nullptr, c.slot,
                                                   CT_INGRESS, ct_action(true, proto, pt, mt),
                                                   tfl, c.dport));
                            }
                        }
                    }
                }
            } else if (punt) {
                ver = VERDICT_PUNT;
            } else {
                act = TC_ACT_SHOT;
                const uint4 srec = lxc6_find(T, lxc_lds, lxc_off, sa_raw);
                const bool src_ok = (srec.z & LXC_VALID) && (srec.z & 0xFFFF) == E.lxc_id;
                if (!src_ok) {   // is_valid_lxc_src_ip (lxc.h:46)
                    ver = DROP_INVALID_SIP;
                    met0 = mkey6<MODE>(DROP_INVALID_SIP, METRIC_EGRESS);
                } else if (xd) {
                    ver = xd;
                    met0 = mkey6<MODE>(xd, METRIC_EGRESS);
                } else if (!known) {
                    ver = DROP_CT_UNKNOWN_PROTO;
                    met0 = mkey6<MODE>(DROP_CT_UNKNOWN_PROTO, METRIC_EGRESS);
                } else if (LB && lb6_egress(T, E, in, i, sa_raw, da_raw, proto, pt, psa, pda,
                                            ppt, svc_rev)) {
                    ver = DROP_NO_SERVICE;   // lb6_local found no backend
                    if (valid) {
                        unsigned long long *m = reinterpret_cast<unsigned long long *>(
                            C.g_met + (uint64_t)(-DROP_NO_SERVICE * METRIC_DIRS + METRIC_EGRESS) * 2);
                        atomicAdd(m, 1ull);
                        atomicAdd(m + 1, (unsigned long long)len);
                    }
                } else {
                    // (LB: the service step moved the tuple's daddr and the
                    // packet's dport to the backend's; lb6_local has no
                    // loopback case, so tuple and packet agree)
                    const uint4 tda_raw = LB ? pda : da_raw;
                    const uint32_t tpt = LB ? ppt : pt;
                    const uint4 tda = LB ? bswap4(pda) : da;
                    if (LB)
                        erec = lxc6_find(T, lxc_lds, lxc_off, pda);
                    const bool elocal = (erec.z & LXC_VALID) != 0;
                    if (LB)
                        ct6_new_dport(proto, tpt, &dport);
                    // destination identity (bpf_lxc.c:206-221)
                    const uint32_t label = LB ? lpm6_lookup(T.ipc6, lo_ipc, tda)
                                              : lpm6_lookup(T.ipc6, lo_ipc, tda, bwi);
                    ident = label ? label
                          : (tda.x == T.router6[0] && tda.y == T.router6[1]) ? CLUSTER_ID
                                                                              : WORLD_ID;
                    // ipv6_l3_from_lxc's ct_lookup6 (bpf_lxc.c:190)
                    CtResult c{CT_NEW, NONE, dport};
                    if (CT) {
                        c = ct_stage6(T, sa_raw, tda_raw, proto, tpt, CT_EGRESS, E.ct_owner);
                        ck1 = c.slot != NONE ? ct_acct_key(c.slot + T.ct6_acct_base, CT_EGRESS)
                              : c.res == CT_NEW
                                  ? ck_miss6(sa_raw, tda_raw, proto, tpt, CT_EGRESS, E.ct_owner)
                                  : NONE;
                    }
                    const bool reply = CT && c.res >= CT_REPLY;
                    const PolicyResult pr = policy_access(T, S, E.pol_base, E.pol_mask,
                                                          ident, c.dport, proto, 1, false);
                    ctr0 = pr.ctr;
                    if (CT)
                        ctb = (uint32_t)c.res | CTO_DONE |
                              ((c.res == CT_NEW && pr.verdict >= 0) ? CTO_CREATE : 0u);
                    idw = id_event(T, C, ID_DIR_EGRESS, ident, pr.verdict < 0 && !reply,
                                   len, valid);
                    // the sender's trace: after ct_create6 the v6 egress path
                    // sets monitor = TRACE_PAYLOAD_LEN (bpf_lxc.c:248)
                    const uint32_t mon1 =
                        !NT ? 0u
                        : c.res == CT_NEW ? TRACE_PAYLOAD_LEN
                                          : ct_monitor(T, CT ? T.ct_st + T.ct6_acct_base : nullptr, c.slot,
                                                       CT_EGRESS, ct_action(true, proto, tpt, mt),
                                                       tfl, c.dport);
                    // a reply of a load-balanced flow: the packet's source
                    // back to the service (bpf_lxc.c:255-266)
                    if (LB && CT && reply && c.slot != NONE && T.ct6_lb)
                        lb6_rev_nat(T, ld16(T.ct6_lb + c.slot).x, proto, psa, ppt);
                    if (pr.verdict < 0 && !reply) {
                        ver = DROP_POLICY;
                        met0 = mkey6<MODE>(DROP_POLICY, METRIC_EGRESS);
                    } else if (pr.verdict > 0) {   // to the proxy
                        act = TC_ACT_REDIRECT;
                        ver = pr.verdict;
                        evw = trace_word(OBS_TO_PROXY, E.lxc_id, (uint32_t)c.res, mon1);
                    } else {
                        met0 = mkey6<MODE>(0, METRIC_EGRESS);   // host/local/stack
                        ver = 0;
                        if (!elocal && ident != CLUSTER_ID && pda.x == 0 && pda.y == 0 &&
                            pda.z == 0xFFFF0000u) {
                            // LXC_NAT46: a v4-mapped peer outside the cluster
                            // (::ffff:0:0/96, bpf_lxc.c:353-360, ipv6.h:279-282)
                            // leaves through tail_ipv6_to_ipv4 (:1070-1083):
                            // ipv6_to_ipv4 drops extension headers, and a
                            // sender without LXC_IPV4 cannot be translated;
                            // else the IPv4 egress path decides (nat.hip)
                            met0 = NONE;
                            ident = 0;
                            if ((mt & CFC_HF_EXTHDR) || !E.nat_v4) {
                                ver = (mt & CFC_HF_EXTHDR) ? DROP_INVALID_EXTHDR : DROP_INVALID;
                                if (ver == DROP_INVALID_EXTHDR)
                                    met0 = mkey6<MODE>(DROP_INVALID_EXTHDR, METRIC_EGRESS);
                                else
                                    natdrop = true;
                            } else {
                                act = TC_ACT_OK;
                                nat = true;
                            }
                        } else if (!elocal) {
                            act = TC_ACT_OK;   // TRACE_TO_STACK (:390)
                            evw = trace_word(OBS_TO_STACK, E.lxc_id, (uint32_t)c.res, mon1);
                        } else if (erec.z & LXC_HOST) {
                            act = TC_ACT_REDIRECT;   // TRACE_TO_HOST (:373)
                            evw = trace_word(OBS_TO_HOST, E.lxc_id, (uint32_t)c.res, mon1);
                        } else if (!(erec.z & LXC_HAS_POLICY)) {
                            ver = DROP_MISSED_TAIL_CALL;
                            met1 = mkey6<MODE>(DROP_MISSED_TAIL_CALL, METRIC_EGRESS);
                        } else {
                            // ipv6_local_delivery into the destination's
                            // ipv6_policy with src = SECLABEL, on the packet
                            // as it now is
                            uint32_t dport2 = dport;
                            if (LB)
                                ct6_new_dport(proto, ppt, &dport2);
                            CtResult c2{CT_NEW, NONE, dport2};
                            const uint4 s2 = LB ? psa : sa_raw;
                            bool fresh = false;
                            if (CT) {
                                const uint32_t own2 = ct_owner_word(erec.z & 0xFFFF,
                                                                    (erec.z & LXC_CT_LOCAL) != 0);
                                c2 = ct_stage6(T, s2, tda_raw, proto, LB ? ppt : pt, CT_INGRESS,
                                               own2);
                                if (own2 == E.ct_owner && c.res == CT_NEW) {
                                    // the entries this header's ct_create6 wrote (main,
                                    // and in an ANY map its ICMPv6 entry) are in the map
                                    // the destination's lookup runs on: an endpoint's
                                    // traffic to itself finds its own entry
                                    const CtProbe k0 =
                                        ct_probe<true>(proto, tpt, CT_EGRESS, E.ct_owner);
                                    const CtProbe k =
                                        ct_probe<true>(proto, LB ? ppt : pt, CT_INGRESS, own2);
                                    const uint32_t rw =
                                        ct_word(58u, ((k0.w2 >> 8) & 7) | 2u, E.ct_owner);
                                    auto is_fresh = [&](uint4 d, uint4 sx, uint32_t z, uint32_t w) {
                                        return d.x == sa_raw.x && d.y == sa_raw.y &&
                                               d.z == sa_raw.z && d.w == sa_raw.w &&
                                               sx.x == tda_raw.x && sx.y == tda_raw.y &&
                                               sx.z == tda_raw.z && sx.w == tda_raw.w &&
                                               ((z == k0.z2 && w == k0.w2) ||
                                                (proto != 6 && z == 0 && w == rw));
                                    };
                                    if (is_fresh(tda_raw, s2, k.z1, k.w1)) {
                                        fresh = true;
                                        c2.res = (k.w1 & 0x200u) ? CT_RELATED : CT_REPLY;
                                        c2.dport = k.td;
                                    } else if (c2.res < CT_REPLY &&
                                               is_fresh(s2, tda_raw, k.z2, k.w2)) {
                                        fresh = true;
                                        c2.res = CT_ESTABLISHED;
                                        c2.dport = k.ts;
                                    }
                                    if (fresh)
                                        c2.slot = NONE;   // (not in the table: the apply counts it)
                                }
                                ck2 = c2.slot != NONE
                                          ? ct_acct_key(c2.slot + T.ct6_acct_base, CT_INGRESS)
                                      : c2.res == CT_NEW
                                          ? ck_miss6(s2, tda_raw, proto, LB ? ppt : pt,
                                                     CT_INGRESS, own2)
                                          : NONE;
                            }
                            if (LB) {   // ipv6_policy's rewrites (:785-815)
                                pda.w &= 0xFFFF0000u;
                                if (CT && c2.slot != NONE && T.ct6_lb)
                                    lb6_rev_nat(T, ld16(T.ct6_lb + c2.slot).x, proto, psa, ppt);
                                else if (fresh)   // the entry as ct_create6 just wrote it
                                    lb6_rev_nat(T, svc_rev, proto, psa, ppt);
                            }
                            const bool reply2 = CT && c2.res >= CT_REPLY;
                            const PolicyResult pw = policy_access(
                                T, S, erec.x, erec.y, E.seclabel, c2.dport, proto, 0, false);
                            ctr1 = pw.ctr;
                            if (CT)
                                ctb |= ((uint32_t)c2.res | CTO_DONE |
                                        ((c2.res == CT_NEW && pw.verdict >= 0) ? CTO_CREATE : 0u))
                                       << 4;
                            ev2 = (pw.verdict < 0 && !reply2) ? 2 : 1;
                            if (pw.verdict < 0 && !reply2) {
                                ver = DROP_POLICY;
                                met1 = mkey6<MODE>(DROP_POLICY, METRIC_INGRESS);
                            } else {
                                const bool prox = pw.verdict > 0 && !reply2;
                                const bool eifx = (erec.z & LXC_IFINDEX) != 0;
                                act = (prox || eifx) ? TC_ACT_REDIRECT : TC_ACT_OK;
                                ver = prox ? pw.verdict : 0;
                                met1 = prox ? NONE : mkey6<MODE>(0, METRIC_INGRESS);
                                if (NT) {
                                    const uint32_t a2 = ct_action(true, proto, LB ? ppt : pt, mt);
                                    uint32_t mon2 = ct_monitor(T, CT ? T.ct_st + T.ct6_acct_base : nullptr,
                                                               c2.slot, CT_INGRESS, a2, tfl,
                                                               c2.dport);
                                    if (fresh)   // the entry as ct_create6 just wrote it
                                        mon2 = c2.dport == 0x3500u
                                                   ? MTU_LEN
                                                   : ct_monitor_of(T, make_uint4(0, T.now, 0, 0),
                                                                   CT_INGRESS, a2, tfl);
                                    evw = trace_word(prox ? OBS_TO_PROXY : OBS_TO_LXC,
                                                     erec.z & 0xFFFF, (uint32_t)c2.res, mon2);
                                }
                            }
                        }
                    }
                }
            }
        }
        st_nt(ver, out.verdict + i);
        st_nt(ident, out.identity + i);
        if (out.action)
            out.action[i] = (uint8_t)act;
        if (CT && out.ct)
            out.ct[i] = (uint8_t)ctb;
        if (NT)   // the monitor event word (cfc_out.notify)
            st_nt(ver < 0 ? notify_word(MODE, ver,
                                        EGR && met1 == mkey6<MODE>(DROP_POLICY, METRIC_INGRESS),
                                        erec.z & 0xFFFF, E.lxc_id)
                          : evw,
                  out.notify + i);
        if (LB && out.pkt_saddr) {   // the packet as it leaves (cfc_out.pkt_*)
            *reinterpret_cast<uint4 *>(out.pkt_saddr + 4 * i) = psa;
            *reinterpret_cast<uint4 *>(out.pkt_daddr + 4 * i) = pda;
            st_nt(ppt, out.pkt_ports + i);
        }
        if (CT) {
            st_nt(ck1, C.ct + i);
            if (EGR)
                st_nt(ck2, C.ct2 + i);
        }
        if (WL && E.wbits) {   // (uniform) the wave's 64 headers' work bits
            bool pr;
            const bool w = wl_want<EGR>(ctb, ver, mt, ck1, ck2, pr);
            const uint64_t wb = __ballot(w && valid), pb = __ballot(pr && valid);
            const uint64_t w0 = base + (threadIdx.x & ~63u);
            if ((threadIdx.x & 63) == 0 && w0 < end) {
                E.wbits[w0 >> 6] = wb;
                E.wprobe[w0 >> 6] = pb;
            }
        }
        if (EGR && E.nat_idx)   // (uniform)
            list_append(E.nat_idx, E.nat_cnt, nat && valid, (uint32_t)i);
        if (EGR && natdrop && valid) {   // DROP_INVALID (rare: a direct count)
            unsigned long long *m = reinterpret_cast<unsigned long long *>(
                C.g_met + (uint64_t)(-DROP_INVALID * METRIC_DIRS + METRIC_EGRESS) * 2);
            atomicAdd(m, 1ull);
            atomicAdd(m + 1, (unsigned long long)len);
        }
        if (MODE != CFC_MODE_XDP) {
            st_nt(ctr_key(C, ctr0, len), C.ctr + i);
            if (EGR)
                st_nt(ctr_key(C, ctr1, len), C.ctr2 + i);
            st_nt(idw, C.id + i);
        }
        acc.add(valid ? met0 : NONE, len);
        if (EGR) {
            acc.add(valid ? met1 : NONE, len);
            acc.add(valid && ev2 ? met6_n<MODE>() + ev2 - 1 : NONE, len);
        }
        if (++iter == 65536 / 2) {
            acc.flush(s_met);
            iter = 0;
        }
    }
    acc.flush(s_met);
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < 2u * acc6_n<MODE>(); j += BLOCK) {
        const unsigned long long v = s_met[j];
        if (!v)
            continue;
        const uint32_t k = j >> 1;
        uint64_t *dst = k < (uint32_t)met6_n<MODE>()
                            ? C.g_met + met6_reason_dir<MODE>(k) * 2
                            : C.g_id + id_index(ID_DIR_INGRESS, E.seclabel, k - met6_n<MODE>());
        atomicAdd((unsigned long long *)dst + (j & 1), v);
    }
}

template <int MODE, bool CT, bool NT>
void launch_mode6_nt(const DevTables &T, const cfc_hdr_v6 &in, const cfc_out &out,
                     const EgressArgs &E, const CountArgs &C, uint32_t grid,
                     uint64_t per_block, hipStream_t s)
{
    const LdsPlan6 L = lds_plan6(T);
    const bool lb = MODE != CFC_MODE_XDP && (T.lb6 || T.rnat6 || out.pkt_saddr);
    auto kern = lb ? k_classify_v6<MODE, CT, NT, true> : k_classify_v6<MODE, CT, NT, false>;
    set_lds_limit((const void *)kern, (int)LDS_PER_WG);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), L.bytes(), s, T, L, in,
                       out, E, C, per_block);
}

template <int MODE, bool CT>
void launch_mode6(const DevTables &T, const cfc_hdr_v6 &in, const cfc_out &out,
                  const EgressArgs &E, const CountArgs &C, uint32_t grid,
                  uint64_t per_block, hipStream_t s)
{
    if (out.notify)
        launch_mode6_nt<MODE, CT, true>(T, in, out, E, C, grid, per_block, s);
    else
        launch_mode6_nt<MODE, CT, false>(T, in, out, E, C, grid, per_block, s);
}

}  // namespace

int launch_classify_v6(const DevTables &T, const cfc_hdr_v6 &in,
                       const cfc_out &out, int mode, const EgressArgs &E,
                       uint64_t *g_ctr, uint32_t *ws, int num_cus, hipStream_t s,
                       const LaunchTiming *tm)
{
    if (in.n == 0)
        return 0;
    if (lds_plan6(T).bytes() > LDS_PER_WG)
        return -22;
    if ((reinterpret_cast<uintptr_t>(in.saddr) | reinterpret_cast<uintptr_t>(in.daddr)) & 15)
        return -22;   // 16-byte address loads
    if (out.pkt_saddr && ((reinterpret_cast<uintptr_t>(out.pkt_saddr) |
                           reinterpret_cast<uintptr_t>(out.pkt_daddr)) & 15))
        return -22;   // 16-byte address stores
    if (out.pkt_saddr && mode == CFC_MODE_XDP &&   // the prefilter rewrites nothing
        (hipMemcpyAsync(out.pkt_saddr, in.saddr, 16 * in.n, hipMemcpyDeviceToDevice, s) ||
         hipMemcpyAsync(out.pkt_daddr, in.daddr, 16 * in.n, hipMemcpyDeviceToDevice, s) ||
         hipMemcpyAsync(out.pkt_ports, in.ports, 4 * in.n, hipMemcpyDeviceToDevice, s)))
        return -5;
    const uint64_t nwg = (uint64_t)num_cus * CFC_WG_PER_CU;
    uint64_t per_block = (in.n + nwg - 1) / nwg;
    per_block = (per_block + BLOCK - 1) / BLOCK * BLOCK;
    const uint32_t grid = (uint32_t)((in.n + per_block - 1) / per_block);
    if (tm)
        (void)hipEventRecord(tm->ev[0], s);
    const bool ct = T.ct6 || out.ct;
    const WsLayout w = ws_layout(in.n, T, mode, ct);
    const CountArgs C = count_args(ws, w, T, g_ctr + 2ull * T.n_ctr, mode, ct);
#define CFC_LAUNCH6(M)                                                         \
    (ct ? launch_mode6<M, true>(T, in, out, E, C, grid, per_block, s)          \
        : launch_mode6<M, false>(T, in, out, E, C, grid, per_block, s))
    switch (mode) {
    case CFC_MODE_INGRESS: CFC_LAUNCH6(CFC_MODE_INGRESS); break;
    case CFC_MODE_EGRESS: CFC_LAUNCH6(CFC_MODE_EGRESS); break;
    case CFC_MODE_XDP: launch_mode6<CFC_MODE_XDP, false>(T, in, out, E, C, grid, per_block, s); break;
    case CFC_MODE_FULL: CFC_LAUNCH6(CFC_MODE_FULL); break;
    default: return -22;
    }
#undef CFC_LAUNCH6
    if (tm)
        (void)hipEventRecord(tm->ev[1], s);
    const bool sums = launch_counters(T, in.meta, in.tcp_flags, in.n, mode, ws, g_ctr, s, ct);
    if (E.sums)
        *E.sums = sums;
    if (tm)
        (void)hipEventRecord(tm->ev[2], s);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace cfc
