// Batched verdict kernels for gfx950 (MI355X).
//
// Two kernels per batch:
//   k_classify_v4  every lookup of the verdict path; writes verdict,
//                  identity, action and, per header, the index of the
//                  policy entry whose counters the reference would bump
//                  (policy.h:68-69,80-81,92-93).
//   k_count        the policy-entry packets/bytes: an exact histogram of
//                  those indices in LDS per <= 64512 headers (one packed
//                  u64 {packets << 32 | bytes} atomic per header), written
//                  as a partial slab and summed per entry by
//                  k_reduce_partials.
//
// Why two.  The classify kernel is bound by random accesses that miss the
// CU: the ipcache in L2 or the Infinity Cache (~267 / ~57 G lines/s
// chip-wide measured, profiles/ubench), endpoint / prefilter / policy
// buckets in L2.  Moving the counter histogram out frees its LDS for
// structures that turn those accesses into LDS reads:
//   * the endpoint table (cilium_lxc) itself when it is small;
//   * a blocked Bloom filter over the prefilter's /32 deny set: an address
//     is probed in L2 only when the filter says "maybe";
//   * a blocked Bloom filter over every policy key: of __policy_can_access's
//     three keys (L4, L3, wildcard port) only those that may exist are
//     probed, in the reference's order — usually none (DROP_POLICY) or one.
// A filter never answers "absent" for a present key, so verdicts stay
// exact; a false positive costs one probe that misses.
//
// IPv4 LPM.  Two layouts (layout.h), chosen per epoch by the flattener:
//   compact    the /16 directory word, then (usually) one 16-byte load of
//              that node's prefix list, longest first — about 1-2 MiB in
//              all, L2-resident;
//   DIR-24-8   tbl24 (64 MiB, Infinity Cache) then tbl8 for split /24s.
//
// Shape.  One 1024-thread workgroup per CU owns a contiguous slice of the
// SoA batch; every loop iteration streams 4 KiB of each input array
// (non-temporal: the 1-GiB stream must not evict the tables).  U headers per
// thread go through four rounds side by side so U independent lookup chains
// are in flight per lane:
//   1. inputs
//   2. directory word | tbl24; endpoint slot (LDS); prefilter bucket if
//      "maybe"
//   3. the node's prefix list | tbl8; identity; the first policy key that
//      may exist
//   4. resolve the policy probe (further keys only after a false positive)
// There is no contraction here, hence no MFMA.
//
// Reference semantics restated here (file:line in /root/reference):
//   ingress   bpf_netdev.c:128-153 (FROM_HOST identity from skb->mark),
//             :357-453 handle_ipv4, l3.h:103-131 ipv4_local_delivery,
//             bpf_lxc.c:898-1028 ipv4_policy + tail_ipv4_policy
//   egress    bpf_lxc.c:440-704 handle_ipv4_from_lxc
//   policy    bpf/lib/policy.h:46-146
//   ct ports  bpf/lib/conntrack.h:467-590 (tuple->dport of a CT_NEW lookup)
//   xdp       bpf_xdp.c:88-121
//   metrics   bpf/lib/metrics.h:43-61
#include <algorithm>
#include <mutex>
#include <set>
#include <tuple>
#include <vector>

#include "kern_common.hpp"
#ifndef CFC_EXP
#define CFC_EXP 0   // timing experiments only (1: no LPM, 2: no policy, 3: no key stores)
#endif

namespace cfc {

namespace {

// update_metrics keys (reason, direction) a mode can produce.  A header
// carries the index of its key, or NONE; every thread counts its headers per
// key in registers, and the workgroup sums them in LDS at the end.
// Egress batches add two keys for the per-identity counters of the
// destination endpoint's policy verdict after local delivery, whose source
// identity is the sender's SECLABEL for the whole batch (fwd, drop).
constexpr int LDS_MET_U64 = 18;   // 2 x 9 keys
template <int MODE>
constexpr int met_n()
{
    return MODE == CFC_MODE_EGRESS ? 7 : MODE == CFC_MODE_XDP ? 0 : 4;
}
template <int MODE>
constexpr int acc_n()
{
    return met_n<MODE>() + (MODE == CFC_MODE_EGRESS ? 2 : 0);
}
// reason (as the positive DROP_* magnitude) and direction of key k
template <int MODE>
__host__ __device__ constexpr uint32_t met_reason_dir(int k)
{
    constexpr uint32_t eg[7][2] = {{0, 2}, {132, 2}, {133, 2}, {137, 2},
                                   {140, 2}, {0, 1}, {133, 1}};
    constexpr uint32_t in[4][2] = {{0, 1}, {133, 1}, {137, 1}, {140, 1}};
    return MODE == CFC_MODE_EGRESS ? eg[k][0] * METRIC_DIRS + eg[k][1]
                                   : in[k][0] * METRIC_DIRS + in[k][1];
}

// key index of (reason, dir) in this mode's table (met_reason_dir)
template <int MODE>
__device__ __forceinline__ uint32_t mkey(int reason, int dir)
{
    if (MODE == CFC_MODE_EGRESS) {
        if (dir == METRIC_INGRESS)
            return reason == 0 ? 5u : 6u;
        switch (reason) {
        case 0: return 0;
        case -132: return 1;
        case -133: return 2;
        case -137: return 3;
        default: return 4;   // -140
        }
    }
    switch (reason) {
    case 0: return 0;
    case -133: return 1;
    case -137: return 2;
    default: return 3;       // -140
    }
}

// Per-header state carried through the lookup rounds.
struct Hdr {
    uint32_t sa, da, pt, mt, mk;
    bool valid;
    uint4 l4d;                   // the /16 directory entry (compact LPM)
    uint32_t e24, pfd, lh, hsh, lxs, lss, pfb;
    uint4 lx, ls, pf, rec;
    bool pf_maybe;
    uint32_t src_lxc;
    int act, ver;
    uint32_t ident, met0, met1, ctr0, ctr1;
    bool xdp_drop, need_pol, skip_proxy;
    uint32_t pbase, pmask, egress_bit, dport;
    uint32_t ct_byte, ct_slot;   // CT byte (CFC_CT_*), stage-1 hit slot
    uint32_t ct_k1, ct_k2;       // accounting keys (slot * 2 + dir) per stage
    int ct_res;
    uint32_t idw;                // identity counter key (CountArgs.id)
    bool id_ovf, drop1;          // ident has no histogram range; stage-1 drop
    bool nat;                    // takes the NAT46 hop (nat.hip)
    uint32_t ev2;                // stage-2 identity event: 0, 1 fwd, 2 drop
    uint32_t tf;                 // TCP header byte 13 (cfc_hdr_v4.tcp_flags)
    uint32_t evw;                // trace event word of a forwarded header
    // load balancing (LB launches; else tda = da, tpt = pt, psa = sa):
    // the sender's tuple daddr / L4 word after the service step (lb.hip),
    // the packet's saddr and L4 word as it leaves, the service step's flags
    uint32_t tda, tpt, psa, ppt, lbfl;
    PolicyProbe P;
};

// round 1: the header (non-temporal streaming loads), issued one iteration
// ahead: the loads of iteration k + 1 go out right after iteration k's last
// table probe, so their HBM latency overlaps that probe's (loads return in
// issue order, so waiting for the probe does not wait for them).  Lanes past
// the end of the slice take the slice's last header: they compute exactly
// what its own lane computes and store the same values to the same places,
// so no round needs a validity branch; only the metrics count them out.
struct Raw {
    uint32_t sa, da, pt, mt, mk, tf;
    uint32_t tda, tpt, psa, lbfl;
};
// in: the workgroup's slice (arrays advanced to its first header), i: the
// header's index in it, nloc: the slice's length
template <bool OPT, bool LBE>
__device__ __forceinline__ void r1_issue(const cfc_hdr_v4 &in, const LbIn &L, uint32_t i,
                                         uint32_t nloc, Raw &r)
{
    // no branches here: a load issued on only one side of a branch makes the
    // compiler's wait at the join conservative (vmcnt(0)), which would wait
    // for these HBM loads together with the probe before them.  Absent
    // optional arrays read saddr instead and the value is dropped.
    i = i < nloc ? i : nloc - 1;
#if CFC_EXP == 8   // (timing only: the slice's first 8192 headers again and again, from L2)
    i &= 8191;
#endif
    const uint32_t o = i << 2;
    r.sa = ldo_nt(in.saddr, o);
    r.da = ldo_nt(in.daddr, o);
    r.pt = ldo_nt(in.ports, o);
    r.mt = ldo_nt(in.meta, o);
    r.mk = r.tf = 0;
    if (OPT) {   // (the optional arrays: compiled out when the call has none)
        const uint32_t mk = ldo_nt(in.mark ? in.mark : in.saddr, o);
        const uint32_t tf = *((in.tcp_flags ? in.tcp_flags : (const uint8_t *)in.saddr) + i);
        r.mk = in.mark ? mk : 0u;
        r.tf = in.tcp_flags ? tf : 0u;
    }
    if (LBE) {   // an egress batch's service step (lb.hip)
        r.tda = ldo_nt(L.tda, o);
        r.tpt = ldo_nt(L.tpt, o);
        r.psa = ldo_nt(L.psa, o);
        r.lbfl = ldo_nt(L.fl, o);
    } else {
        r.tda = r.da;
        r.tpt = r.pt;
        r.psa = r.sa;
        r.lbfl = 0;
    }
}
__device__ __forceinline__ void r1_take(const Raw &r, uint32_t i, uint32_t end,
                                        Hdr &h)
{
    h.valid = i < end;
    h.sa = r.sa;
    h.da = r.da;
    h.pt = r.pt;
    h.mt = r.mt;
    h.mk = r.mk;
    h.tf = r.tf;
    h.tda = r.tda;
    h.tpt = r.tpt;
    h.psa = r.psa;
    h.ppt = r.pt;
    h.lbfl = r.lbfl;
}

// round 2: every lookup that only needs the header
template <int MODE>
__device__ __forceinline__ void r2_issue(const DevTables &T, const Lds &S,
                                         Hdr &h)
{
    constexpr bool XDP = MODE == CFC_MODE_XDP || MODE == CFC_MODE_FULL;
    constexpr bool EGR = MODE == CFC_MODE_EGRESS;
    constexpr bool LPM = MODE != CFC_MODE_XDP;
    h.l4d = make_uint4(0, 0, 0, 0);
    h.e24 = h.pfd = 0;
    h.lx = h.ls = h.pf = make_uint4(0, 0, 0, 0);
    h.lh = __builtin_bswap32(EGR ? h.tda : h.sa);
    h.hsh = __builtin_bswap32(h.sa);
    h.lxs = h.lss = h.pfb = 0;
    h.pf_maybe = false;
    if (LPM) {
        if (T.l4d)
#if CFC_EXP == 1
            h.l4d = make_uint4(h.lh & 0xFFFF, 0, 0, 0);
#else
            h.l4d = ldt16(T.l4d, (h.lh >> 16) * 16u);
#endif
        else if (T.tbl24)
            h.e24 = T.tbl24[h.lh >> 8];
    }
    if (XDP && T.pf_tbl24)
        h.pfd = T.pf_tbl24[h.hsh >> 8];
    if (T.lxc4) {
        h.lxs = hash32(h.da, T.lxc4_mask);
        h.lx = lxc_slot(T, S, h.lxs);
        if (EGR) {
            h.lss = hash32(h.sa, T.lxc4_mask);
            h.ls = lxc_slot(T, S, h.lss);
        }
    }
    if (XDP && T.pf_fix && h.sa) {
        h.pf_maybe = !S.pfb || bloom_maybe(S.pfb_off, S.pfb_mask, pf_bloom_hash(h.sa));
        if (h.pf_maybe) {
            h.pfb = hash32(h.sa, T.pf_fix_mask);
            h.pf = ldt16(T.pf_fix, h.pfb * 16u);
        }
    }
}

// round 3: second-level LPM, endpoint resolution, prefilter verdict,
// identity, and the first policy key that may exist
template <int MODE, bool CT, bool LB>
__device__ __forceinline__ void r3_identity(const DevTables &T, const Lds &S,
                                            const EgressArgs &E, Hdr &h)
{
    constexpr bool XDP = MODE == CFC_MODE_XDP || MODE == CFC_MODE_FULL;
    constexpr bool EGR = MODE == CFC_MODE_EGRESS;
    constexpr bool LPM = MODE != CFC_MODE_XDP;
    if (LPM && T.l4d) {
#if CFC_EXP == 4
        h.e24 = (h.l4d.x & L4_PTR) ? 300u : h.l4d.x;
#else
        h.e24 = l4_lookup(T, h.lh, h.l4d);
#endif
    } else {
        if (h.e24 & LPM_GROUP)
            h.e24 = T.tbl8[((h.e24 & ~LPM_GROUP) << 8) | (h.lh & 0xFF)];
        if (h.e24 & LPM_INDIRECT)
            h.e24 = T.lbl_ovf[h.e24 & LPM_PAYLOAD];
    }
    if (h.pfd & LPM_GROUP)
        h.pfd = T.pf_tbl8[((h.pfd & ~LPM_GROUP) << 8) | (h.hsh & 0xFF)];
    // rec: {addr, pol_base, pol_mask, info}; info == 0 -> not local
    h.rec = make_uint4(0, 0, 0, 0);
    uint4 srec = h.rec;
    if (T.lxc4) {
#if CFC_EXP == 7
        h.rec = h.lx;
#else
        h.rec = lxc_resolve(T, S, h.da, h.lxs, h.lx);
#endif
        if (EGR)
            srec = lxc_resolve(T, S, h.sa, h.lss, h.ls);
    }
    const bool local = (h.rec.w & LXC_VALID) != 0;
    h.src_lxc = (srec.w & LXC_VALID) ? (srec.w & 0xFFFF) : NONE;

    h.act = TC_ACT_OK;
    h.ver = 0;
    h.ident = 0;
    h.met0 = h.met1 = h.ctr0 = h.ctr1 = NONE;
    h.xdp_drop = false;
    if (XDP) {
        bool deny = h.pfd != 0;
        if (!deny)
            deny = h.sa ? (h.pf_maybe && pf_resolve(T, h.sa, h.pfb, h.pf))
                        : T.pf_fix_zero != 0;
        h.xdp_drop = deny || !local;
        if (MODE == CFC_MODE_XDP || h.xdp_drop) {
            h.act = h.xdp_drop ? XDP_DROP : XDP_PASS;
            h.ver = h.xdp_drop ? CFC_DROP_PREFILTER : 0;
        }
    }

    h.need_pol = h.skip_proxy = false;
    h.pbase = h.pmask = h.egress_bit = h.dport = 0;
    h.ct_byte = 0;
    h.ct_slot = NONE;
    h.ct_res = CT_NEW;
    h.ct_k1 = h.ct_k2 = NONE;
    h.idw = KEY_NONE;
    h.id_ovf = h.drop1 = false;
    h.nat = false;
    h.ev2 = 0;
    h.evw = 0;
    if (MODE == CFC_MODE_XDP || h.xdp_drop)
        return;
    const uint32_t proto = h.mt & 0xFF;
    const bool known = ct_new_dport(proto, h.tpt, &h.dport);
    if (!EGR) {
        // handle_identity_from_host (bpf_netdev.c:128-153), branch-free
        const uint32_t magic = h.mk & 0xF00u;
        const bool viap = (magic == 0xA00u) | (magic == 0xB00u);
        const uint32_t id = viap ? (((h.mk & 0xFF) << 16) | (h.mk >> 16))
                                 : (magic == 0xC00u ? HOST_ID : WORLD_ID);
        h.skip_proxy = magic == 0xA00u;
        // handle_ipv4 (:375-398): reserved identities take the ipcache's
        const bool ovr = (id < HEALTH_ID) & (h.e24 != 0u) & (h.e24 != CLUSTER_ID) &
                         (h.e24 != HOST_ID);
        h.ident = ovr ? h.e24 : id;
        // the destination endpoint's program: missed tail call, unknown
        // protocol, or its policy
        const bool ep = local & !(h.rec.w & LXC_HOST);
        const bool noprog = ep & !(h.rec.w & LXC_HAS_POLICY);
        const bool unk = ep & !noprog & !known;
        h.need_pol = ep & !noprog & known;
        h.act = (noprog | unk) ? TC_ACT_SHOT : TC_ACT_OK;
        h.ver = noprog ? DROP_MISSED_TAIL_CALL : unk ? DROP_CT_UNKNOWN_PROTO : 0;
        h.met0 = noprog ? mkey<MODE>(DROP_MISSED_TAIL_CALL, METRIC_INGRESS)
                 : unk  ? mkey<MODE>(DROP_CT_UNKNOWN_PROTO, METRIC_INGRESS)
                        : NONE;
        h.pbase = h.rec.y;
        h.pmask = h.rec.z;
        if (CT && h.need_pol) {   // ipv4_policy's ct_lookup4 (bpf_lxc.c:932)
            const CtResult c = ct_stage4(
                T, h.sa, h.da, proto, h.pt, CT_INGRESS,
                ct_owner_word(h.rec.w & 0xFFFF, (h.rec.w & LXC_CT_LOCAL) != 0));
            h.dport = c.dport;
            h.ct_res = c.res;
            h.ct_slot = c.slot;
            h.ct_byte = (uint32_t)c.res | CTO_DONE;
            // LXC_NAT46: a hit on an entry with nat46 (__ct_lookup,
            // conntrack.h:241-244) leaves ipv4_policy for NAT46 and
            // ipv6_policy (bpf_lxc.c:939-944, 1098-1110) when the endpoint
            // has an IPv6 address: that hop decides (nat.hip); nothing here
            // counts but the hit
            if (T.nat46 && c.slot != NONE && (h.rec.w & LXC_HAS6) &&
                (T.ct_st[c.slot].tm.flags & CTT_NAT46)) {
                h.nat = true;
                h.need_pol = false;
                h.ct_k1 = ct_acct_key(c.slot, CT_INGRESS);
            }
            // a reply of a load-balanced flow: its source translated back
            // (bpf_lxc.c:946-955; the packet only)
            if (LB && T.ct4_lb && c.res == CT_REPLY && !h.nat) {
                const uint4 lw = ld16(T.ct4_lb + c.slot);
                if (!((lw.x >> 16) & 1)) {
                    uint32_t da = h.da;
                    lb4_rev_nat(T, lw, proto, h.psa, da, h.ppt);
                }
            }
        }
    } else {
        h.act = TC_ACT_SHOT;
        if (h.src_lxc != E.lxc_id) {   // is_valid_lxc_src_ipv4 (lxc.h:55)
            h.ver = DROP_INVALID_SIP;
            h.met0 = mkey<MODE>(DROP_INVALID_SIP, METRIC_EGRESS);
        } else if (LB && (h.lbfl & LBF_DROP)) {   // lb4_local: no backend
            h.ver = DROP_NO_SERVICE;             // (counted in the store loop)
        } else if (!known) {
            h.ver = DROP_CT_UNKNOWN_PROTO;
            h.met0 = mkey<MODE>(DROP_CT_UNKNOWN_PROTO, METRIC_EGRESS);
        } else {
            // destination identity (bpf_lxc.c:516-532)
            h.ident = h.e24 ? h.e24
                            : ((h.tda & T.v4_cluster_mask) == T.v4_cluster_range
                                   ? CLUSTER_ID
                                   : WORLD_ID);
            h.need_pol = true;
            h.pbase = E.pol_base;
            h.pmask = E.pol_mask;
            h.egress_bit = 1;
            if (CT) {   // handle_ipv4_from_lxc's ct_lookup4 (bpf_lxc.c:509)
                const CtResult c = ct_stage4(T, h.sa, h.tda, proto, h.tpt,
                                             CT_EGRESS, E.ct_owner);
                h.dport = c.dport;
                h.ct_res = c.res;
                h.ct_slot = c.slot;
                h.ct_byte = (uint32_t)c.res | CTO_DONE;
            }
        }
    }
    if (h.need_pol) {
        // ingress fragments look up the L3 key only (policy.h:61,85); the
        // egress path passes is_fragment = false (policy.h:153-154)
        const bool frag = !EGR && (h.mt & CFC_HF_FRAG);
#if CFC_EXP == 2
        h.P.maybe = 0; h.P.j = 3;
        if (0)
#endif
        policy_issue(T, S, h.pbase, h.pmask, h.ident, h.dport, proto,
                     h.egress_bit, frag, h.P);
    }
}

// round 4: resolve the policy verdict, compose the program result.
// The outcome is built in locals and written back once: conditional stores
// to different fields of `h` get merged by the compiler into one store
// through a selected field address, which pushes the whole per-header state
// array into scratch memory.
template <int MODE, bool CT, bool NT, bool LB>
__device__ __forceinline__ void r4_verdict(const DevTables &T, const Lds &S,
                                           const EgressArgs &E, Hdr &h)
{
    constexpr bool EGR = MODE == CFC_MODE_EGRESS;
    if (!h.need_pol)
        return;
    // the monitor length of a trace this header may send (NT: the caller
    // wants the event words)
    const uint32_t action = ct_action(false, h.mt & 0xFF, h.tpt, h.mt);
    const uint32_t tfl = (h.mt & 0xFF) == 6 ? h.tf : 0u;
    const uint32_t mon1 = NT ? ct_monitor(T, CT ? T.ct_st : nullptr, h.ct_slot,
                                          EGR ? CT_EGRESS : CT_INGRESS, action, tfl,
                                          h.dport)
                             : 0u;
    const uint32_t res1 = CT ? (uint32_t)h.ct_res : 0u;
    uint32_t evw = 0;
    // replies and related packets pass whatever the policy says
    // (bpf_lxc.c:963-970 ingress, :538-545 egress)
    const bool reply = CT && h.ct_res >= CT_REPLY;
    uint32_t ctb = h.ct_byte;
    const bool frag = (h.mt & CFC_HF_FRAG) != 0;
    const uint32_t proto = h.mt & 0xFF;
    const PolicyResult pr = policy_resolve(T, h.pbase, h.pmask, h.P);
    const int mdir = EGR ? METRIC_EGRESS : METRIC_INGRESS;
    const bool ifx = (h.rec.w & LXC_IFINDEX) != 0;
    int v = pr.verdict;
    int act, ver;
    uint32_t met0 = NONE, met1 = NONE, ctr1 = NONE;
    const uint32_t len = h.mt >> 16;
    if (CT) {
        // the hit's CONNTRACK_ACCOUNTING key, aggregated by k_ct_count; a
        // CT_NEW stage's miss tag
        h.ct_k1 = h.ct_slot != NONE
                      ? ct_acct_key(h.ct_slot, EGR ? CT_EGRESS : CT_INGRESS)
                  : h.ct_res != CT_NEW ? NONE
                  : EGR ? ck_miss4(h.sa, h.tda, proto, h.tpt, CT_EGRESS, E.ct_owner)
                        : ck_miss4(h.sa, h.da, proto, h.pt, CT_INGRESS,
                                   ct_owner_word(h.rec.w & 0xFFFF, (h.rec.w & LXC_CT_LOCAL) != 0));
        // ct_create4 for a new flow that is not dropped here
        if (h.ct_res == CT_NEW && (v >= 0 || reply))
            ctb |= CTO_CREATE;
    }
    // the per-identity forward/drop counter of this policy verdict
    const bool drop1 = v < 0 && !reply;
    h.drop1 = drop1;
    h.idw = id_key(T, h.ident, drop1, len);
    h.id_ovf = h.idw == KEY_NONE;
    uint32_t ev2 = 0;
    if (!EGR) {
        // (branch-free) drop, or redirect_to_proxy for NEW / ESTABLISHED
        // flows (TRACE_TO_PROXY, lxc.h:117), or TRACE_TO_LXC + delivery
        // (bpf_lxc.c:1006)
        const int v2 = h.skip_proxy ? 0 : v;
        const bool prox = !drop1 & (v2 > 0) & !reply;
        act = drop1 ? TC_ACT_SHOT : (prox | ifx) ? TC_ACT_REDIRECT : TC_ACT_OK;
        ver = drop1 ? DROP_POLICY : prox ? v2 : 0;
        met0 = drop1 ? mkey<MODE>(DROP_POLICY, mdir)
               : prox ? NONE : mkey<MODE>(0, METRIC_INGRESS);
        if (NT)
            evw = drop1 ? 0u
                        : trace_word(prox ? OBS_TO_PROXY : OBS_TO_LXC, h.rec.w & 0xFFFF,
                                     res1, mon1);
    } else if (drop1) {
        act = TC_ACT_SHOT;
        ver = DROP_POLICY;
        met0 = mkey<MODE>(DROP_POLICY, mdir);
    } else if (v > 0) {        // egress proxy (bpf_lxc.c:582-604)
        act = TC_ACT_REDIRECT;
        ver = v;
        evw = trace_word(OBS_TO_PROXY, E.lxc_id, res1, mon1);
    } else {
        met0 = mkey<MODE>(0, METRIC_EGRESS);   // to_host/local/to_stack
        ver = 0;
        if (!(h.rec.w & LXC_VALID)) {
            act = TC_ACT_OK;   // pass_to_stack: TRACE_TO_STACK (bpf_lxc.c:687)
            evw = trace_word(OBS_TO_STACK, E.lxc_id, res1, mon1);
        } else if (h.rec.w & LXC_HOST) {
            act = TC_ACT_REDIRECT;   // to_host: TRACE_TO_HOST (:668)
            evw = trace_word(OBS_TO_HOST, E.lxc_id, res1, mon1);
        } else if (!(h.rec.w & LXC_HAS_POLICY)) {
            act = TC_ACT_SHOT;
            ver = DROP_MISSED_TAIL_CALL;
            met1 = mkey<MODE>(DROP_MISSED_TAIL_CALL, METRIC_EGRESS);
        } else {
            // local delivery: the destination's ipv4_policy with
            // src = SECLABEL of the sending endpoint, after its own
            // ct_lookup4 in the destination's CT maps
            uint32_t dp2 = h.dport;
            CtResult c2{CT_NEW, NONE, 0};
            bool fresh = false;
            if (CT) {
                const uint32_t own2 = ct_owner_word(h.rec.w & 0xFFFF,
                                                    (h.rec.w & LXC_CT_LOCAL) != 0);
                c2 = ct_stage4(T, h.psa, h.da, proto, h.pt, CT_INGRESS, own2);
                dp2 = c2.dport;
                if (own2 == E.ct_owner && h.ct_res == CT_NEW && (v >= 0 || reply)) {
                    // the entries this header's egress stage created (ct_create4:
                    // main, ICMP and, with the service's ct_state, reverse-NAT
                    // entry) are in the map the destination's lookup runs on
                    // (an endpoint's traffic to itself, or a looped-back service)
                    const CtProbe k0 = ct_probe<false>(proto, h.tpt, CT_EGRESS, E.ct_owner);
                    const CtProbe k = ct_probe<false>(proto, h.pt, CT_INGRESS, own2);
                    const bool svc = LB && (h.lbfl & LBF_SVC) != 0;
                    const bool loop = LB && (h.lbfl & LBF_LOOP) != 0;
                    // main: k2 of the egress lookup; ICMP entry (ANY maps
                    // only: a TCP map's is one no lookup reaches): ports 0,
                    // k2's flags | TUPLE_F_RELATED; reverse-NAT entry: its
                    // daddr the service step's address, a looped-back flow's
                    // with TUPLE_F_IN and the sender as saddr
                    const uint32_t ex = loop ? IPV4_LOOPBACK : h.da;
                    const uint32_t ey = loop ? h.sa : h.tda;
                    const uint32_t ew = loop ? ct_word(proto, 1u, E.ct_owner) : k0.w2;
                    const uint32_t rw = ct_word(1u, ((k0.w2 >> 8) & 7) | 2u, E.ct_owner);
                    auto is_fresh = [&](uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
                        return (x == h.sa && y == h.tda &&
                                ((z == k0.z2 && w == k0.w2) || (proto != 6 && z == 0 && w == rw))) ||
                               (svc && x == ex && y == ey && z == k0.z2 && w == ew);
                    };
                    if (is_fresh(h.da, h.psa, k.z1, k.w1)) {
                        fresh = true;
                        c2.res = (k.w1 & 0x200u) ? CT_RELATED : CT_REPLY;
                        c2.dport = k.td;
                    } else if (c2.res < CT_REPLY && is_fresh(h.psa, h.da, k.z2, k.w2)) {
                        fresh = true;
                        c2.res = CT_ESTABLISHED;
                        c2.dport = k.ts;
                    }
                    if (fresh) {
                        c2.slot = NONE;   // (not in the table: the apply counts it)
                        dp2 = c2.dport;
                    }
                }
                h.ct_k2 = c2.slot != NONE ? ct_acct_key(c2.slot, CT_INGRESS)
                          : c2.res == CT_NEW ? ck_miss4(h.psa, h.da, proto, h.pt, CT_INGRESS, own2)
                                             : NONE;
                if (LB && c2.res == CT_REPLY) {   // bpf_lxc.c:946-955, packet only
                    const uint4 lw = fresh ? make_uint4((h.lbfl >> 16) | (h.lbfl & LBF_LOOP) << 14,
                                                        0, 0, 0)
                                           : (T.ct4_lb ? ld16(T.ct4_lb + c2.slot)
                                                       : make_uint4(0, 0, 0, 0));
                    if (!((lw.x >> 16) & 1)) {
                        uint32_t da = h.da;
                        lb4_rev_nat(T, lw, proto, h.psa, da, h.ppt);
                    }
                }
            }
            const bool reply2 = CT && c2.res >= CT_REPLY;
            const PolicyResult pw = policy_access(T, S, h.rec.y, h.rec.z,
                                                  E.seclabel, dp2, proto,
                                                  0, frag);
            const int w = pw.verdict;
            ctr1 = pw.ctr;
            if (CT)
                ctb |= ((uint32_t)c2.res | CTO_DONE |
                        ((c2.res == CT_NEW && (w >= 0 || reply2)) ? CTO_CREATE : 0u)) << 4;
            if (w < 0 && !reply2) {
                act = TC_ACT_SHOT;
                ver = DROP_POLICY;
                met1 = mkey<MODE>(DROP_POLICY, METRIC_INGRESS);
                ev2 = 2;
            } else {
                const bool prox = w > 0 && !reply2;
                act = (prox || ifx) ? TC_ACT_REDIRECT : TC_ACT_OK;
                ver = prox ? w : 0;
                met1 = prox ? NONE : mkey<MODE>(0, METRIC_INGRESS);
                ev2 = 1;
                if (NT) {   // the destination program's trace
                    uint32_t mon2 = ct_monitor(T, CT ? T.ct_st : nullptr,
                                               CT ? c2.slot : NONE, CT_INGRESS,
                                               action, tfl, dp2);
                    if (fresh)   // the entry as ct_create4 just wrote it
                        mon2 = dp2 == 0x3500u ? MTU_LEN
                               : ct_monitor_of(T, make_uint4(0, T.now, 0, 0), CT_INGRESS,
                                               action, tfl);
                    evw = trace_word(prox ? OBS_TO_PROXY : OBS_TO_LXC, h.rec.w & 0xFFFF,
                                     CT ? (uint32_t)c2.res : 0u, mon2);
                }
            }
        }
    }
    h.ev2 = ev2;
    h.evw = evw;
    h.act = act;
    h.ver = ver;
    h.met0 = met0;
    h.met1 = met1;
    h.ctr0 = pr.ctr;
    h.ctr1 = ctr1;
    h.ct_byte = ctb;
}

// LDS image of one launch: the metrics block, then the tables copied in.
struct LdsPlan {
    uint32_t lxc_slots, pf_words, pol_words;
    __host__ __device__ size_t bytes() const
    {
        return 8ull * LDS_MET_U64 + 16ull * lxc_slots + 4ull * pf_words +
               4ull * pol_words;
    }
};

__host__ LdsPlan lds_plan(const DevTables &T)
{
    LdsPlan p;
    p.lxc_slots = (T.lxc4 && T.lxc4_lds) ? T.lxc4_mask + 1 : 0;
    p.pf_words = T.pf_bloom ? T.pf_bloom_words : 0;
    p.pol_words = T.pol_bloom ? T.pol_bloom_words : 0;
    return p;
}

// the workgroup's metrics (and, egress, stage-2 identity) sums into the
// counter block
template <int MODE>
__device__ __forceinline__ void acc_publish(const unsigned long long *s_met,
                                            const CountArgs &C, uint32_t seclabel)
{
    for (uint32_t j = threadIdx.x; j < 2u * acc_n<MODE>(); j += BLOCK) {
        const unsigned long long v = s_met[j];
        if (!v)
            continue;
        const uint32_t k = j >> 1;
        uint64_t *dst = k < (uint32_t)met_n<MODE>()
                            ? C.g_met + met_reason_dir<MODE>(k) * 2
                            : C.g_id + id_index(ID_DIR_INGRESS, seclabel, k - met_n<MODE>());
        atomicAdd((unsigned long long *)dst + (j & 1), v);
    }
}

// OPT: the call passes some optional array (mark, tcp_flags, action, ct);
// without, their pointers and branches are compiled out (fewer live SGPRs)
// LB: the launch has a load balancer — an egress batch reads the service
// step's results (lb.hip), every batch may reverse-NAT replies, and the
// packet outputs (cfc_out.pkt_*) are written
// FAST: the epoch has the common shape (fast_shape): the compact IPv4 LPM,
// no prefilter LPM, the endpoint table and both Bloom filters in LDS, and
// (modes with XDP) a prefilter /32 set.  The tests of that shape and the
// pointers of the other layouts are then compile-time facts, which frees the
// SGPRs and exec-mask pairs they would hold for the whole loop.
template <int MODE, int U, bool CT, bool NT, bool OPT, bool LB, bool FAST>
__global__ __launch_bounds__(BLOCK, WAVES_PER_SIMD) void k_classify_v4(
    DevTables T, LdsPlan L, cfc_hdr_v4 in, cfc_out out, EgressArgs E,
    CountArgs C, uint64_t per_block, LbIn LI)
{
    if (FAST) {
        T.tbl24 = T.tbl8 = T.pf_tbl24 = T.pf_tbl8 = nullptr;
        __builtin_assume(T.l4d != nullptr);
        __builtin_assume(T.lxc4 != nullptr);
        if (MODE == CFC_MODE_XDP || MODE == CFC_MODE_FULL)
            __builtin_assume(T.pf_fix != nullptr);
    }
    // LDS image (uint4 units): metrics | endpoint slots | pf Bloom | pol Bloom
    unsigned long long *s_met = lds_met();
    Lds S;
    S.lxc_off = LDS_MET_U64 / 2;
    const uint32_t pf4 = S.lxc_off + L.lxc_slots;      // uint4 index
    const uint32_t pol4 = pf4 + L.pf_words / 4;
    S.pfb_off = 4 * pf4;
    S.polb_off = 4 * pol4;
    S.lxc = FAST || L.lxc_slots != 0;
    S.pfb = FAST || L.pf_words != 0;
    S.polb = FAST || L.pol_words != 0;
    S.pfb_mask = L.pf_words - 1;
    S.polb_mask = L.pol_words - 1;
    for (uint32_t j = threadIdx.x; j < (uint32_t)LDS_MET_U64; j += BLOCK)
        s_met[j] = 0;
    // the apply's work bits (E.wbits / E.wprobe)
    constexpr bool WL = CT && MODE != CFC_MODE_XDP && !LB;
    lds_copy(cfc_smem + S.lxc_off, reinterpret_cast<const uint4 *>(T.lxc4),
             L.lxc_slots);
    lds_copy(cfc_smem + pf4, reinterpret_cast<const uint4 *>(T.pf_bloom),
             L.pf_words / 4);
    lds_copy(cfc_smem + pol4, reinterpret_cast<const uint4 *>(T.pol_bloom),
             L.pol_words / 4);
    __syncthreads();

    constexpr bool EGR = MODE == CFC_MODE_EGRESS;
    const uint32_t id_dir = EGR ? ID_DIR_EGRESS : ID_DIR_INGRESS;
    const uint64_t start = (uint64_t)blockIdx.x * per_block;
    if (start >= in.n)
        return;   // (uniform: no header for this workgroup; nothing to publish)
    // the workgroup's slice: every array advanced to its first header, so
    // per-lane addresses are 32-bit offsets from wave-uniform bases
    // (launch_classify_v4 keeps per_block < 2^30)
    const uint32_t end = (uint32_t)min(in.n - start, per_block);
    in.saddr += start;
    in.daddr += start;
    in.ports += start;
    in.meta += start;
    if (OPT) {
        if (in.mark)
            in.mark += start;
        if (in.tcp_flags)
            in.tcp_flags += start;
        if (out.action)
            out.action += start;
        if (out.ct)
            out.ct += start;
    }
    out.verdict += start;
    out.identity += start;
    if (out.notify)
        out.notify += start;
    constexpr bool LBE = LB && MODE == CFC_MODE_EGRESS;
    if (LBE) {
        LI.tda += start;
        LI.tpt += start;
        LI.psa += start;
        LI.fl += start;
    }
    if (LB && out.pkt_saddr) {
        out.pkt_saddr += start;
        out.pkt_daddr += start;
        out.pkt_ports += start;
    }
    if (C.ct)
        C.ct += start;
    if (C.ct2)
        C.ct2 += start;
    if (C.ctr)
        C.ctr += start;
    if (C.ctr2)
        C.ctr2 += start;
    if (C.id)
        C.id += start;
    // the trip count is uniform across the workgroup (the metrics flush
    // needs whole waves)
    MetAcc<acc_n<MODE>()> acc;
    acc.clear();
    uint32_t iter = 0;
    Raw nx[U];
#pragma unroll
    for (int u = 0; u < U; u++)
        r1_issue<OPT, LBE>(in, LI, u * BLOCK + threadIdx.x, end, nx[u]);
    for (uint32_t base = 0; base < end; base += BLOCK * U) {
        Hdr h[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            r1_take(nx[u], base + u * BLOCK + threadIdx.x, end, h[u]);
#pragma unroll
        for (int u = 0; u < U; u++)
            r2_issue<MODE>(T, S, h[u]);
#pragma unroll
        for (int u = 0; u < U; u++)
            r3_identity<MODE, CT, LB>(T, S, E, h[u]);
        // the next iteration's headers, behind this one's policy probe (the
        // last iteration re-reads the slice's last header)
        const uint32_t nb = base + BLOCK * U;
#pragma unroll
        for (int u = 0; u < U; u++)
            r1_issue<OPT, LBE>(in, LI, nb + u * BLOCK + threadIdx.x, end, nx[u]);
#pragma unroll
        for (int u = 0; u < U; u++)
            r4_verdict<MODE, CT, NT, LB>(T, S, E, h[u]);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = base + u * BLOCK + threadIdx.x;
            const uint32_t len = h[u].mt >> 16;
            {   // (lanes past the end rewrite the last header's values)
                const uint32_t o = h[u].valid ? i : end - 1, o4 = o << 2;
                sto_nt(h[u].ver, out.verdict, o4);
                sto_nt(h[u].ident, out.identity, o4);
                if (OPT && out.action)
                    sto((uint8_t)h[u].act, out.action, o);
                if (CT && OPT && out.ct)
                    sto((uint8_t)h[u].ct_byte, out.ct, o);
                if (NT)   // the monitor event word (cfc_out.notify)
                    sto_nt((uint32_t)(h[u].ver < 0
                              ? notify_word(MODE, h[u].ver,
                                            EGR && h[u].met1 == mkey<MODE>(DROP_POLICY, METRIC_INGRESS),
                                            h[u].rec.w & 0xFFFF, E.lxc_id)
                              : h[u].evw),
                          out.notify, o4);
                if (CT) {
                    sto_nt(h[u].ct_k1, C.ct, o4);
                    if (EGR)
                        sto_nt(h[u].ct_k2, C.ct2, o4);
                }
                if (LB && out.pkt_saddr) {   // the packet as it leaves
                    sto_nt(h[u].psa, out.pkt_saddr, o4);
                    sto_nt(h[u].da, out.pkt_daddr, o4);
                    sto_nt(h[u].ppt, out.pkt_ports, o4);
                }
                if (MODE != CFC_MODE_XDP) {
#if CFC_EXP != 3
                    sto_nt(ctr_key(C, h[u].ctr0, len), C.ctr, o4);
#endif
                    if (EGR)
                        sto_nt(ctr_key(C, h[u].ctr1, len), C.ctr2, o4);
#if CFC_EXP != 3
                    sto_nt(h[u].idw, C.id, o4);
#endif
                }
            }
            if (WL && E.wbits) {   // (uniform) the wave's 64 headers' work bits
                bool pr;
                const bool w = wl_want<EGR>(h[u].ct_byte, h[u].ver, h[u].mt, h[u].ct_k1,
                                            EGR ? h[u].ct_k2 : NONE, pr);
                const uint64_t wb = __ballot(w && h[u].valid), pb = __ballot(pr && h[u].valid);
                const uint32_t w0 = base + u * BLOCK + (threadIdx.x & ~63u);
                if ((threadIdx.x & 63) == 0 && w0 < end) {
                    E.wbits[(start + w0) >> 6] = wb;
                    E.wprobe[(start + w0) >> 6] = pb;
                }
            }
            if (!EGR && MODE != CFC_MODE_XDP && E.nat_idx)   // (uniform)
                list_append(E.nat_idx, E.nat_cnt, h[u].nat && h[u].valid, (uint32_t)start + i);
            if (MODE != CFC_MODE_XDP && h[u].valid && h[u].id_ovf && h[u].need_pol)
                id_count(C, id_dir, h[u].ident, h[u].drop1, len);
            if (LBE && h[u].valid && h[u].ver == DROP_NO_SERVICE) {   // (rare)
                unsigned long long *m = reinterpret_cast<unsigned long long *>(
                    C.g_met + (uint64_t)(-DROP_NO_SERVICE * METRIC_DIRS + METRIC_EGRESS) * 2);
                atomicAdd(m, 1ull);
                atomicAdd(m + 1, (unsigned long long)len);
            }
#if CFC_EXP != 5
            acc.add(h[u].valid ? h[u].met0 : NONE, len);
#endif
            if (EGR) {
                acc.add(h[u].valid ? h[u].met1 : NONE, len);
                acc.add(h[u].valid && h[u].ev2 ? met_n<MODE>() + h[u].ev2 - 1 : NONE, len);
            }
        }
        if (++iter == 65536 / (2 * U)) {
            acc.flush(s_met);
            iter = 0;
        }
    }
    acc.flush(s_met);
    __syncthreads();
    acc_publish<MODE>(s_met, C, E.seclabel);
}

}  // namespace

// ---- counters ---------------------------------------------------------------
// k_hist: the exact sums behind one key range of one key array, per slice of
// the batch: an LDS histogram of up to HIST_RANGE u64 slots, one packed
// {packets << 40 | bytes} atomic per header (a slice is at most 2^24
// headers of <= 65535 bytes, so neither half carries), written as a partial
// slab; k_hist_reduce sums the slabs per key and adds them into the counter
// block.  One launch runs every job (policy ranges of each stage, identity
// ranges) side by side: blockIdx.y is the job, blockIdx.x the slice.
namespace {

struct HistJob {
    const uint32_t *keys;
    uint64_t poff;        // first u64 of the job's partial slabs
    uint32_t lo, cnt;     // key range [lo, lo + cnt)
    uint32_t kind;        // 0 policy entry, 1 identity (dense << 1 | drop)
    uint32_t packed;      // keys carry len in bits 16-31 (else meta does)
};
constexpr int HIST_JOBS_MAX = 12;
struct HistJobs {
    HistJob j[HIST_JOBS_MAX];
};
constexpr uint64_t BYTES_MASK = (1ull << 40) - 1;
constexpr uint64_t SLICE_MAX = 1ull << 24;

__device__ __forceinline__ void hist_add(unsigned long long *s, const HistJob &jb,
                                         uint32_t w, uint32_t m)
{
    uint32_t k, len;
    if (jb.packed) {
        k = w & 0xFFFF;
        len = w >> 16;
    } else {
        k = w;
        len = m >> 16;
    }
    const uint32_t r = k - jb.lo;
    if (r < jb.cnt)
        atomicAdd(&s[r], (1ull << 40) | len);
}

__global__ __launch_bounds__(BLOCK) void k_hist(HistJobs J, const uint32_t *meta,
                                                uint64_t n, uint64_t per_block,
                                                uint64_t *partial)
{
    const HistJob jb = J.j[blockIdx.y];
    unsigned long long *s = reinterpret_cast<unsigned long long *>(cfc_smem);
    for (uint32_t j = threadIdx.x; j < jb.cnt; j += BLOCK)
        s[j] = 0;
    __syncthreads();
    const uint64_t start = (uint64_t)blockIdx.x * per_block;   // multiple of 4
    const uint64_t end = min(n, start + per_block);
    const uint64_t end4 = start + ((end - start) & ~3ull);
    const bool meta16 = (reinterpret_cast<uintptr_t>(meta) & 15) == 0;
    // the loads of the next two steps are in flight during this step's LDS
    // atomics (one workgroup per CU: a step that waits for its own loads
    // waits a full HBM latency)
    auto load = [&](uint64_t i, uint4 &w, uint4 &m) {
        w = make_uint4(KEY_NONE, KEY_NONE, KEY_NONE, KEY_NONE);
        m = make_uint4(0, 0, 0, 0);
        if (i >= end4)
            return;
        w = ld_nt4(jb.keys + i);
        if (!jb.packed) {
            if (meta16) {
                m = ld_nt4(meta + i);
            } else {
                m.x = meta[i];
                m.y = meta[i + 1];
                m.z = meta[i + 2];
                m.w = meta[i + 3];
            }
        }
    };
    const uint64_t i0 = start + 4 * threadIdx.x;
    uint4 w0, m0, w1, m1;
    load(i0, w0, m0);
    load(i0 + 4 * BLOCK, w1, m1);
    for (uint64_t i = i0; i < end4; i += 4 * BLOCK) {
        uint4 w2, m2;
        load(i + 8 * BLOCK, w2, m2);
        hist_add(s, jb, w0.x, m0.x);
        hist_add(s, jb, w0.y, m0.y);
        hist_add(s, jb, w0.z, m0.z);
        hist_add(s, jb, w0.w, m0.w);
        w0 = w1; m0 = m1;
        w1 = w2; m1 = m2;
    }
    for (uint64_t i = end4 + threadIdx.x; i < end; i += BLOCK)
        hist_add(s, jb, jb.keys[i], jb.packed ? 0u : meta[i]);
    __syncthreads();
    uint64_t *dst = partial + jb.poff + (uint64_t)blockIdx.x * jb.cnt;
    for (uint32_t j = threadIdx.x; j < jb.cnt; j += BLOCK)
        st_nt((uint64_t)s[j], dst + j);
}

// blockIdx.y: job, blockIdx.x: 256 keys of it
// blockIdx.z: a group of REDUCE_ROWS slices
constexpr uint32_t REDUCE_ROWS = 32;
__global__ __launch_bounds__(256) void k_hist_reduce(HistJobs J, const uint64_t *partial,
                                                     uint32_t nblk, uint64_t *g_ctr,
                                                     uint64_t *g_id, uint32_t id_dir)
{
    const HistJob jb = J.j[blockIdx.y];
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= jb.cnt)
        return;
    uint64_t pk = 0, by = 0;
    const uint64_t *p = partial + jb.poff + j;
    const uint32_t b0 = blockIdx.z * REDUCE_ROWS, b1 = min(nblk, b0 + REDUCE_ROWS);
    for (uint32_t b = b0; b < b1; b++) {
        const uint64_t v = ld_nt(p + (uint64_t)b * jb.cnt);
        pk += v >> 40;
        by += v & BYTES_MASK;
    }
    if (!pk)
        return;
    const uint32_t key = jb.lo + j;
    uint64_t *dst = jb.kind == 0 ? g_ctr + 2ull * key
                                 : g_id + id_index(id_dir, key >> 1, key & 1);
    atomicAdd((unsigned long long *)dst, (unsigned long long)pk);
    atomicAdd((unsigned long long *)dst + 1, (unsigned long long)by);
}

// CONNTRACK_ACCOUNTING: the per-header keys (slot * 2 + dir) of a
// <= COUNT_PER_BLOCK slice aggregated in an LDS hash table — Zipf traffic
// puts thousands of a slice's packets on a few flows, and one global u64
// atomic per packet on the same entry would serialise — then flushed with
// one global atomic pair per distinct (entry, dir).  A key that finds no
// LDS slot within 8 probes goes straight to the global counters (those are
// the rare flows, so no contention there).
constexpr uint32_t CT_LDS_SLOTS = 8192;
constexpr uint32_t CT_LDS_BYTES = CT_LDS_SLOTS * 12;
__global__ __launch_bounds__(BLOCK) void k_ct_count(const uint32_t *ct_idx,
                                                    const uint32_t *ct_idx2,
                                                    const uint32_t *meta,
                                                    uint64_t n,
                                                    CtState *st)
{
    uint32_t *keys = reinterpret_cast<uint32_t *>(cfc_smem);
    unsigned long long *vals =
        reinterpret_cast<unsigned long long *>(keys + CT_LDS_SLOTS);
    for (uint32_t j = threadIdx.x; j < CT_LDS_SLOTS; j += BLOCK) {
        keys[j] = NONE;
        vals[j] = 0;
    }
    __syncthreads();
    const uint32_t *idx = blockIdx.y ? ct_idx2 : ct_idx;
    const uint64_t start = (uint64_t)blockIdx.x * COUNT_PER_BLOCK;
    const uint64_t end = min(n, start + COUNT_PER_BLOCK);
    for (uint64_t i = start + threadIdx.x; i < end; i += BLOCK) {
        const uint32_t k = ld_nt(idx + i);
        if (k >= CK_MISS)   // (NONE, or a CT_NEW stage's tag)
            continue;
        const uint32_t len = ld_nt(meta + i) >> 16;
        uint32_t h = fmix32(k) & (CT_LDS_SLOTS - 1);
        bool done = false;
        for (int p = 0; p < 8 && !done; p++) {
            uint32_t cur = keys[h];
            if (cur == NONE) {
                cur = atomicCAS(&keys[h], NONE, k);
                if (cur == NONE)
                    cur = k;
            }
            if (cur == k) {
                // <= 64512 packets of <= 65535 bytes: the byte half of
                // {packets << 32 | bytes} never carries
                atomicAdd(&vals[h], (1ull << 32) | len);
                done = true;
            }
            h = (h + 1) & (CT_LDS_SLOTS - 1);
        }
        if (!done) {
            unsigned long long *a = ct_acct_at(st, k);
            atomicAdd(a, 1ull);
            atomicAdd(a + 1, (unsigned long long)len);
        }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < CT_LDS_SLOTS; j += BLOCK) {
        const uint32_t k = keys[j];
        const unsigned long long v = vals[j];
        if (k != NONE && v) {
            unsigned long long *a = ct_acct_at(st, k);
            atomicAdd(a, v >> 32);
            atomicAdd(a + 1, v & 0xFFFFFFFFull);
        }
    }
}

// ---- CT accounting by key range ---------------------------------------------
// The per-slice LDS table above leaves one global atomic pair per distinct
// (flow, slice) — on Zipf traffic over millions of flows most of the
// packets of the tail, ~25M atomics per 64M-header batch.  Partitioned
// instead, every distinct key of the batch costs one plain read-modify-
// write of its counters, and every pass over the staged records reads and
// writes whole runs (an MSD radix partition in two digits, each digit
// sorted inside a 16384-record chunk in LDS):
//   A k_acc_agg    per slice: the LDS table (hot flows collapse); its entries
//                  and the overflow packets staged as 8-byte records, counted
//                  per (coarse bucket, 16384-record chunk)
//   B k_scan_*     exclusive scan of the [coarse][chunk] counts: where each
//                  chunk's run of each coarse bucket goes
//   C k_acc_part1  per chunk: records sorted by coarse bucket in LDS, written
//                  as runs into coarse order
//   D k_acc_plan   the coarse regions cut into 16384-record chunks
//   E k_acc_part2  per chunk of a coarse region: sorted by fine bucket in
//                  LDS, written back in place; the chunk's fine offsets kept
//   F k_acc_reduce one workgroup per fine bucket (CTP_BUCKET keys): gathers
//                  its run of every chunk of its coarse region, LDS sums per
//                  key, then its counters, which no other workgroup touches
// Records: key (27 bits) << 37 | kind << 36 | payload; kind 0: packets (16)
// << 20 | bytes (20) of an LDS entry; kind 1: one << 25 | hit flags (9) << 16
// | low (16): one = 1, a single packet of length low (the overflow), else an
// LDS entry's high part (bytes >> 20, which can pass 0) and its flags.
// Hit flags (acc_flags): the TCP flags, and 1 << 8 for a TCP packet without
// the close bit — per key (slot, direction) the plain-hit summary the device
// CT apply needs (k_acc_reduce writes it into DevTables.ct_sum).
constexpr uint32_t CTP_BUCKET_BITS = 12, CTP_BUCKET = 1u << CTP_BUCKET_BITS;
constexpr uint32_t CTP_MAX_BUCKETS = 32768;    // keys < 2^27 (64M CT slots)
constexpr uint32_t ACC_FINE_BITS = 7, ACC_FINE = 1u << ACC_FINE_BITS;
constexpr uint32_t ACC_MAX_COARSE = CTP_MAX_BUCKETS / ACC_FINE;      // 256
constexpr int ACC_KEY_SHIFT = 37, ACC_KIND_BIT = 36, ACC_BY_BITS = 20;
constexpr uint32_t ACC_BY_MASK = (1u << ACC_BY_BITS) - 1;
constexpr uint32_t ACC_CHUNK_BITS = 14, ACC_CHUNK = 1u << ACC_CHUNK_BITS;
constexpr uint32_t ACC_PER_THREAD = ACC_CHUNK / BLOCK;                // 16
// records per slice: <= COUNT_PER_BLOCK overflow packets, <= CT_LDS_SLOTS
// entries and as many high parts
constexpr uint32_t ACC_SLICE_CHUNKS = 5;
constexpr uint32_t ACC_RCAP = ACC_SLICE_CHUNKS * ACC_CHUNK;
static_assert(COUNT_PER_BLOCK + 2 * CT_LDS_SLOTS <= ACC_RCAP, "slice records");
static_assert(CTP_BUCKET % BLOCK == 0, "reduce flush");
constexpr int ACC_COARSE_SHIFT = ACC_KEY_SHIFT + CTP_BUCKET_BITS + ACC_FINE_BITS;   // 56
constexpr int ACC_BUCKET_SHIFT = ACC_KEY_SHIFT + CTP_BUCKET_BITS;                   // 49
static_assert(ACC_COARSE_SHIFT + 8 == 64, "coarse bucket: the key's top 8 bits");
constexpr uint32_t ACC_AGG_LDS =
    CT_LDS_SLOTS * 16 + ACC_SLICE_CHUNKS * ACC_MAX_COARSE * 4 + 16;
constexpr uint32_t ACC_SORT_LDS = ACC_CHUNK * 8 + 3 * ACC_MAX_COARSE * 4 + 16;
constexpr uint32_t ACC_RED_LDS = CTP_BUCKET * 16;

// slice of one k_acc_agg workgroup: <= COUNT_PER_BLOCK headers (a multiple
// of 4), sized so that a large batch's slices come in whole rounds of 256
// workgroups (one per CU) rather than four rounds and a few stragglers
uint64_t acc_slice(uint64_t n)
{
    const uint64_t full = 256ull * COUNT_PER_BLOCK;
    if (n <= full)
        return COUNT_PER_BLOCK;
    const uint64_t rounds = (n + full - 1) / full;
    const uint64_t per = (n + 256 * rounds - 1) / (256 * rounds);
    return (per + 3) & ~3ull;
}

__device__ __forceinline__ uint64_t acc_rec(uint32_t k, uint32_t pk, uint32_t by)
{
    return (uint64_t)k << ACC_KEY_SHIFT | (uint64_t)pk << ACC_BY_BITS | by;
}
// kind 1: a single packet (one) or an LDS entry's high bytes, with flags
__device__ __forceinline__ uint64_t acc_rec1(uint32_t k, bool one, uint32_t fl, uint32_t low)
{
    return (uint64_t)k << ACC_KEY_SHIFT | 1ull << ACC_KIND_BIT | (one ? 1ull << 25 : 0ull) |
           (uint64_t)fl << 16 | low;
}
// a header's hit flags (sum_bits in ctops.hpp, per direction)
__device__ __forceinline__ uint32_t acc_flags(uint32_t meta, uint32_t tf)
{
    const bool tcp = (meta & 0xFF) == 6;
    return tcp ? ((tf & 0xFF) | ((meta & CFC_HF_TCP_CLOSE) ? 0u : 0x100u)) : 0u;
}

// slot of this lane in an LDS-counted list, one atomic per wave (the lanes
// of a wave appending together would otherwise serialise on the counter);
// every lane of the wave must call it
__device__ __forceinline__ uint32_t wave_append(uint32_t *ctr, bool want)
{
    const uint64_t m = __ballot(want);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lead = m ? (uint32_t)__builtin_ctzll(m) : 0u;
    uint32_t base = 0;
    if (m && lane == lead)
        base = atomicAdd(ctr, (uint32_t)__popcll(m));
    base = __shfl(base, (int)lead, 64);
    return base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
}
// probes before a key becomes a record of its own: the hot flows take their
// slots early; later keys are mostly the Zipf tail, for which a full table's
// long probe sequences cost more than the record
constexpr int CTP_PROBES = 3;

// A: slice vw's records into rec[vw * ACC_RCAP ...]; cnt[c * nch + vw *
// ACC_SLICE_CHUNKS + q] = records of coarse bucket c in the slice's chunk q
template <bool VEC>
__global__ __launch_bounds__(BLOCK) void k_acc_agg(const uint32_t *ct_idx,
                                                   const uint32_t *ct_idx2,
                                                   const uint32_t *meta, const uint8_t *tf,
                                                   bool sums, uint64_t n,
                                                   uint32_t nco, uint64_t *rec,
                                                   uint32_t *rcnt, uint32_t *cnt, uint64_t per)
{
    uint32_t *keys = reinterpret_cast<uint32_t *>(cfc_smem);
    unsigned long long *vals = reinterpret_cast<unsigned long long *>(keys + CT_LDS_SLOTS);
    uint32_t *fls = reinterpret_cast<uint32_t *>(vals + CT_LDS_SLOTS);
    uint32_t *hist = fls + CT_LDS_SLOTS;
    uint32_t *nrec = hist + ACC_SLICE_CHUNKS * ACC_MAX_COARSE;
    for (uint32_t j = threadIdx.x; j < CT_LDS_SLOTS; j += BLOCK) {
        keys[j] = NONE;
        vals[j] = 0;
        fls[j] = 0;
    }
    for (uint32_t j = threadIdx.x; j < ACC_SLICE_CHUNKS * ACC_MAX_COARSE; j += BLOCK)
        hist[j] = 0;
    if (threadIdx.x == 0)
        *nrec = 0;
    __syncthreads();
    const uint32_t nv = gridDim.x * gridDim.y;
    const uint32_t vw = blockIdx.y * gridDim.x + blockIdx.x;
    const uint32_t *idx = blockIdx.y ? ct_idx2 : ct_idx;
    uint64_t *rs = rec + (uint64_t)vw * ACC_RCAP;
    const uint64_t start = (uint64_t)blockIdx.x * per;
    const uint64_t end = min(n, start + per);
    auto put = [&](uint32_t r, uint64_t v) {
        rs[r] = v;
        atomicAdd(&hist[(r >> ACC_CHUNK_BITS) * ACC_MAX_COARSE + (uint32_t)(v >> ACC_COARSE_SHIFT)],
                  1u);
    };
    // one header: its LDS entry, or a record of its own (every lane of the
    // wave calls it)
    auto one = [&](uint32_t k, uint32_t len, uint32_t fl) {
        uint32_t h = fmix32(k) & (CT_LDS_SLOTS - 1);
        bool done = k >= CK_MISS;   // (NONE, or a CT_NEW stage's tag)
        for (int p = 0; p < CTP_PROBES && !done; p++) {
            uint32_t cur = keys[h];
            if (cur == NONE) {
                cur = atomicCAS(&keys[h], NONE, k);
                if (cur == NONE)
                    cur = k;
            }
            if (cur == k) {
                // <= 64512 packets of <= 65535 bytes: {packets << 32 | bytes}
                atomicAdd(&vals[h], (1ull << 32) | len);
                if (fl && (fls[h] & fl) != fl)
                    atomicOr(&fls[h], fl);
                done = true;
            }
            h = (h + 1) & (CT_LDS_SLOTS - 1);
        }
        const uint32_t r = wave_append(nrec, !done);   // a record of its own
        if (!done)
            put(r, acc_rec1(k, true, fl, len));
    };
    // VEC: four consecutive headers per thread and step (16-byte loads),
    // the loads of the next two steps in flight during this step's LDS work
    // (one 1024-thread workgroup per CU: with one step of look-ahead the
    // pass waits on HBM latency every step)
    constexpr uint32_t W = VEC ? 4 : 1, STEP = W * BLOCK;
    // (tf: four headers' TCP flags in one word; none without the array)
    auto load = [&](uint64_t e, uint4 &kk, uint4 &mm, uint32_t &ff) {
        if (VEC && e + 4 <= end) {
            kk = ld_nt4(idx + e);
            mm = ld_nt4(meta + e);
            ff = tf ? ld_nt(reinterpret_cast<const uint32_t *>(tf + e)) : 0u;
        } else {
            kk = make_uint4(NONE, NONE, NONE, NONE);
            mm = make_uint4(0, 0, 0, 0);
            ff = 0;
            if (e < end) { kk.x = ld_nt(idx + e); mm.x = ld_nt(meta + e); ff = tf ? tf[e] : 0u; }
            if (VEC && e + 1 < end) {
                kk.y = ld_nt(idx + e + 1); mm.y = ld_nt(meta + e + 1);
                ff |= tf ? (uint32_t)tf[e + 1] << 8 : 0u;
            }
            if (VEC && e + 2 < end) {
                kk.z = ld_nt(idx + e + 2); mm.z = ld_nt(meta + e + 2);
                ff |= tf ? (uint32_t)tf[e + 2] << 16 : 0u;
            }
        }
    };
    const uint64_t e0 = start + (uint64_t)threadIdx.x * W;
    uint4 k0, m0, k1, m1;
    uint32_t f0, f1;
    load(e0, k0, m0, f0);
    load(e0 + STEP, k1, m1, f1);
    for (uint64_t i0 = start; i0 < end; i0 += STEP) {   // (uniform trip count)
        uint4 k2, m2;
        uint32_t f2;
        load(e0 + (i0 - start) + 2 * STEP, k2, m2, f2);
        // (no summaries kept: no flags, no records for them)
        one(k0.x, m0.x >> 16, sums ? acc_flags(m0.x, f0) : 0u);
        if (VEC) {
            one(k0.y, m0.y >> 16, sums ? acc_flags(m0.y, f0 >> 8) : 0u);
            one(k0.z, m0.z >> 16, sums ? acc_flags(m0.z, f0 >> 16) : 0u);
            one(k0.w, m0.w >> 16, sums ? acc_flags(m0.w, f0 >> 24) : 0u);
        }
        k0 = k1; m0 = m1; f0 = f1;
        k1 = k2; m1 = m2; f1 = f2;
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < CT_LDS_SLOTS; j += BLOCK) {   // (uniform)
        const uint32_t k = keys[j];
        const unsigned long long v = vals[j];
        const uint32_t by = (uint32_t)v, fl = fls[j];
        const uint32_t r = wave_append(nrec, k != NONE);
        if (k != NONE)
            put(r, acc_rec(k, (uint32_t)(v >> 32), by & ACC_BY_MASK));
        const bool hi = k != NONE && (by > ACC_BY_MASK || fl);
        const uint32_t r2 = wave_append(nrec, hi);
        if (hi)
            put(r2, acc_rec1(k, false, fl, by >> ACC_BY_BITS));
    }
    __syncthreads();
    const uint32_t nch = nv * ACC_SLICE_CHUNKS;
    for (uint32_t j = threadIdx.x; j < nco * ACC_SLICE_CHUNKS; j += BLOCK) {
        const uint32_t c = j / ACC_SLICE_CHUNKS, q = j % ACC_SLICE_CHUNKS;
        cnt[(uint64_t)c * nch + vw * ACC_SLICE_CHUNKS + q] = hist[q * ACC_MAX_COARSE + c];
    }
    if (threadIdx.x == 0)
        rcnt[vw] = *nrec;
}

// Sort m <= ACC_CHUNK records (r[], this thread's share: index threadIdx.x +
// i * BLOCK) by digit (v >> shift) & (nd - 1) in LDS: on return buf[0, m)
// holds them in digit order and base[d] is digit d's first index (base[nd]
// = m).  The order inside a digit is arbitrary (sums do not care).
__device__ __forceinline__ void acc_local_sort(const uint64_t (&r)[ACC_PER_THREAD], uint32_t m,
                                               int shift, uint32_t mask, uint32_t nd,
                                               uint64_t *buf, uint32_t *cnt, uint32_t *base)
{
    for (uint32_t j = threadIdx.x; j < nd; j += BLOCK)
        cnt[j] = 0;
    __syncthreads();
    uint32_t rank[ACC_PER_THREAD];
#pragma unroll
    for (uint32_t i = 0; i < ACC_PER_THREAD; i++) {
        const uint32_t x = threadIdx.x + i * BLOCK;
        if (x < m)
            rank[i] = atomicAdd(&cnt[(uint32_t)(r[i] >> shift) & mask], 1u);
    }
    __syncthreads();
    static_assert(ACC_MAX_COARSE <= 256, "one wave scans four counts per lane");
    if (threadIdx.x < 64) {   // exclusive scan of <= 256 counts by one wave
        const uint32_t l = threadIdx.x;
        uint32_t v[4], x = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            v[q] = 4 * l + q < nd ? cnt[4 * l + q] : 0u;
            x += v[q];
        }
        const uint32_t own = x;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (l >= (uint32_t)d)
                x += y;
        }
        uint32_t e = x - own;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (4 * l + q < nd)
                base[4 * l + q] = e;
            e += v[q];
        }
        if (l == 63)
            base[nd] = x;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < ACC_PER_THREAD; i++) {
        const uint32_t x = threadIdx.x + i * BLOCK;
        if (x < m)
            buf[base[(uint32_t)(r[i] >> shift) & mask] + rank[i]] = r[i];
    }
    __syncthreads();
}

// C: chunk ch = vw * ACC_SLICE_CHUNKS + q of the staged records, sorted by
// coarse bucket, each bucket's run written at off[c * nch + ch]
__global__ __launch_bounds__(BLOCK) void k_acc_part1(const uint64_t *rec, const uint32_t *rcnt,
                                                     const uint32_t *off, uint32_t nch,
                                                     uint32_t nco, uint64_t *outA)
{
    uint64_t *buf = reinterpret_cast<uint64_t *>(cfc_smem);
    uint32_t *cnt = reinterpret_cast<uint32_t *>(buf + ACC_CHUNK);
    uint32_t *base = cnt + ACC_MAX_COARSE;
    uint32_t *goff = base + ACC_MAX_COARSE + 1;
    const uint32_t ch = blockIdx.x, vw = ch / ACC_SLICE_CHUNKS, q = ch % ACC_SLICE_CHUNKS;
    const uint32_t all = rcnt[vw], lo = q * ACC_CHUNK;
    if (lo >= all)
        return;
    const uint32_t m = min(ACC_CHUNK, all - lo);
    const uint64_t *src = rec + (uint64_t)vw * ACC_RCAP + lo;
    for (uint32_t c = threadIdx.x; c < nco; c += BLOCK)
        goff[c] = off[(uint64_t)c * nch + ch];
    uint64_t r[ACC_PER_THREAD];
#pragma unroll
    for (uint32_t i = 0; i < ACC_PER_THREAD; i++) {
        const uint32_t x = threadIdx.x + i * BLOCK;
        r[i] = x < m ? ld_nt(src + x) : 0ull;
    }
    acc_local_sort(r, m, ACC_COARSE_SHIFT, ACC_MAX_COARSE - 1, nco, buf, cnt, base);
#pragma unroll
    for (uint32_t i = 0; i < ACC_PER_THREAD; i++) {
        const uint32_t x = threadIdx.x + i * BLOCK;
        if (x < m) {
            const uint64_t v = buf[x];
            const uint32_t c = (uint32_t)(v >> ACC_COARSE_SHIFT);
            outA[goff[c] + (x - base[c])] = v;
        }
    }
}

// D: plan[c] = first record of coarse bucket c (plan[nco] = all records),
// plan[nco + 1 + c] = its first fine-sort chunk (plan[2 nco + 1] = chunks);
// one wave, two coarse buckets per lane (nco <= 128)
__global__ __launch_bounds__(64) void k_acc_plan(const uint32_t *off, uint32_t nch,
                                                 uint32_t nco, uint32_t *plan)
{
    const uint32_t l = threadIdx.x;
    const uint32_t total = off[(uint64_t)nco * nch];
    uint32_t nc[4], a[4], own = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {   // (four coarse buckets per lane: nco <= 256)
        const uint32_t c = 4 * l + j;
        a[j] = c < nco ? off[(uint64_t)c * nch] : total;
        const uint32_t b = c + 1 < nco ? off[(uint64_t)(c + 1) * nch] : total;
        nc[j] = c < nco ? (b - a[j] + ACC_CHUNK - 1) >> ACC_CHUNK_BITS : 0u;
        own += nc[j];
    }
    uint32_t x = own;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (l >= (uint32_t)d)
            x += y;
    }
    uint32_t e = x - own;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t c = 4 * l + j;
        if (c < nco) {
            plan[c] = a[j];
            plan[nco + 1 + c] = e;
        }
        e += nc[j];
    }
    if (l == 63) {   // the ends (nco may be 256: no lane's own bucket)
        plan[nco] = total;
        plan[2 * nco + 1] = x;
    }
}

// E: fine-sort chunk w of the coarse regions: records [lo, lo + m) of
// coarse bucket c sorted by fine bucket into out[lo ...]; fo[w * (ACC_FINE
// + 1) + f] = fine bucket f's first index in the chunk
__global__ __launch_bounds__(BLOCK) void k_acc_part2(const uint64_t *inA, const uint32_t *plan,
                                                     uint32_t nco, uint64_t *out, uint32_t *fo)
{
    uint64_t *buf = reinterpret_cast<uint64_t *>(cfc_smem);
    uint32_t *cnt = reinterpret_cast<uint32_t *>(buf + ACC_CHUNK);
    uint32_t *base = cnt + ACC_MAX_COARSE;
    uint32_t *sc = base + ACC_MAX_COARSE + 1;
    const uint32_t w = blockIdx.x;
    const uint32_t *pc = plan + nco + 1;
    if (w >= pc[nco])
        return;
    if (threadIdx.x == 0) {   // the coarse bucket holding chunk w
        uint32_t a = 0, b = nco;   // pc[a] <= w < pc[b]
        while (b - a > 1) {
            const uint32_t mid = (a + b) / 2;
            if (pc[mid] <= w)
                a = mid;
            else
                b = mid;
        }
        *sc = a;
    }
    __syncthreads();
    const uint32_t c = *sc;
    const uint32_t lo = plan[c] + ((w - pc[c]) << ACC_CHUNK_BITS);
    const uint32_t m = min(ACC_CHUNK, plan[c + 1] - lo);
    uint64_t r[ACC_PER_THREAD];
#pragma unroll
    for (uint32_t i = 0; i < ACC_PER_THREAD; i++) {
        const uint32_t x = threadIdx.x + i * BLOCK;
        r[i] = x < m ? ld_nt(inA + lo + x) : 0ull;
    }
    acc_local_sort(r, m, ACC_BUCKET_SHIFT, ACC_FINE - 1, ACC_FINE, buf, cnt, base);
#pragma unroll
    for (uint32_t i = 0; i < ACC_PER_THREAD; i++) {
        const uint32_t x = threadIdx.x + i * BLOCK;
        if (x < m)
            out[lo + x] = buf[x];
    }
    for (uint32_t f = threadIdx.x; f <= ACC_FINE; f += BLOCK)
        fo[(uint64_t)w * (ACC_FINE + 1) + f] = base[f];
}

// F: fine bucket b = c * ACC_FINE + f: its run in every chunk of coarse
// bucket c (eight groups of 128 threads, a chunk each), summed per key in
// LDS, then added to its counters (acct[2k] packets, acct[2k + 1] bytes)
__global__ __launch_bounds__(BLOCK) void k_acc_reduce(const uint64_t *recs, const uint32_t *plan,
                                                      const uint32_t *fo, uint32_t nco,
                                                      CtState *st, uint32_t *sum)
{
    uint32_t *pk = reinterpret_cast<uint32_t *>(cfc_smem);
    unsigned long long *by = reinterpret_cast<unsigned long long *>(pk + CTP_BUCKET);
    uint32_t *fl = reinterpret_cast<uint32_t *>(by + CTP_BUCKET);
    for (uint32_t j = threadIdx.x; j < CTP_BUCKET; j += BLOCK) {
        pk[j] = 0;
        by[j] = 0;
        fl[j] = 0;
    }
    __syncthreads();
    const uint32_t b = blockIdx.x, c = b >> ACC_FINE_BITS, f = b & (ACC_FINE - 1);
    const uint32_t *pc = plan + nco + 1;
    const uint32_t w0 = pc[c], w1 = pc[c + 1];
    const uint32_t g = threadIdx.x >> 7, t = threadIdx.x & 127;
    for (uint32_t w = w0 + g; w < w1; w += BLOCK / 128) {
        const uint32_t lo = plan[c] + ((w - w0) << ACC_CHUNK_BITS);
        const uint32_t *o = fo + (uint64_t)w * (ACC_FINE + 1) + f;
        const uint32_t r0 = lo + o[0], r1 = lo + o[1];
        uint64_t nv = r0 + t < r1 ? ld_nt(recs + r0 + t) : 0ull;
        for (uint32_t r = r0 + t; r < r1; r += 128) {
            const uint64_t v = nv;
            nv = r + 128 < r1 ? ld_nt(recs + r + 128) : 0ull;
            const uint32_t j = (uint32_t)(v >> ACC_KEY_SHIFT) & (CTP_BUCKET - 1);
            if ((v >> ACC_KIND_BIT) & 1) {
                const uint32_t low = (uint32_t)v & 0xFFFFu, f = (uint32_t)(v >> 16) & 0x1FFu;
                if ((v >> 25) & 1) {   // a single packet
                    atomicAdd(&pk[j], 1u);
                    atomicAdd(&by[j], (unsigned long long)low);
                } else {
                    atomicAdd(&by[j], (unsigned long long)low << ACC_BY_BITS);
                }
                if (f && (fl[j] & f) != f)
                    atomicOr(&fl[j], f);
            } else {
                atomicAdd(&pk[j], (uint32_t)(v >> ACC_BY_BITS) & 0xFFFFu);
                atomicAdd(&by[j], v & ACC_BY_MASK);
            }
        }
    }
    __syncthreads();
    // the bucket's counters: every touched key's {packets, bytes} loaded
    // before any is written back (in a loop of read-modify-writes the loads
    // of the next key wait behind the store of this one)
    constexpr uint32_t FJ = CTP_BUCKET / BLOCK;
    uint32_t p[FJ];
    ulonglong2 cv[FJ];
#pragma unroll
    for (uint32_t q = 0; q < FJ; q++) {
        const uint32_t j = threadIdx.x + q * BLOCK;
        p[q] = pk[j];
        const uint64_t k = (uint64_t)b * CTP_BUCKET + j;
        cv[q] = p[q] ? *reinterpret_cast<const ulonglong2 *>(ct_acct_at(st, k)) : ulonglong2{0, 0};
    }
#pragma unroll
    for (uint32_t q = 0; q < FJ; q++) {
        if (!p[q])
            continue;
        const uint32_t j = threadIdx.x + q * BLOCK;
        const uint64_t k = (uint64_t)b * CTP_BUCKET + j;
        cv[q].x += p[q];
        cv[q].y += by[j];
        *reinterpret_cast<ulonglong2 *>(ct_acct_at(st, k)) = cv[q];
    }
    if (!sum)
        return;
    // the plain-hit summary per slot (keys 2s: tx, 2s + 1: rx), as
    // ctops.hpp sum_bits lays it out: rx flags, tx flags << 8, rx hit << 16,
    // tx hit << 17, a TCP hit without the close bit << 18
    for (uint32_t q = threadIdx.x; q < CTP_BUCKET / 2; q += BLOCK) {
        const uint32_t jt = 2 * q, jr = 2 * q + 1;
        uint32_t w = 0;
        if (pk[jt])
            w |= (fl[jt] & 0xFFu) << 8 | 1u << 17 | ((fl[jt] >> 8) & 1u) << 18;
        if (pk[jr])
            w |= (fl[jr] & 0xFFu) | 1u << 16 | ((fl[jr] >> 8) & 1u) << 18;
        if (w)
            sum[((uint64_t)b * CTP_BUCKET >> 1) + q] = w;
    }
}

// exclusive scan of n u32 (n < 2^32 total): per 4096-element block, block
// sums, then the sums' offsets added back; out[n] = the total
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *tmp)
{
    // inclusive scan of one value per thread over the 1024-thread block
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d)
            x += y;
    }
    if (lane == 63)
        tmp[wv] = x;
    __syncthreads();
    if (threadIdx.x < 16) {
        uint32_t t = tmp[threadIdx.x];
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const uint32_t y = __shfl_up(t, d, 16);
            if (threadIdx.x >= (uint32_t)d)
                t += y;
        }
        tmp[16 + threadIdx.x] = t;
    }
    __syncthreads();
    const uint32_t before = wv ? tmp[16 + wv - 1] : 0u;
    const uint32_t r = before + x - v;
    __syncthreads();
    return r;
}
__global__ __launch_bounds__(BLOCK) void k_scan_local(const uint32_t *in, uint32_t *out,
                                                      uint64_t n, uint32_t *bsum)
{
    __shared__ uint32_t tmp[32];
    const uint64_t b0 = (uint64_t)blockIdx.x * 4 * BLOCK + 4ull * threadIdx.x;
    uint32_t v[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        v[j] = b0 + j < n ? in[b0 + j] : 0u;
        s += v[j];
    }
    uint32_t e = block_excl_scan(s, tmp);
#pragma unroll
    for (int j = 0; j < 4; j++) {
        if (b0 + j < n)
            out[b0 + j] = e;
        e += v[j];
    }
    if (threadIdx.x == BLOCK - 1)
        bsum[blockIdx.x] = e;
}
__global__ __launch_bounds__(BLOCK) void k_scan_top(uint32_t *bsum, uint32_t nb,
                                                    uint32_t *total)
{
    __shared__ uint32_t tmp[32];
    uint32_t carry = 0;
    for (uint32_t c = 0; c < nb; c += BLOCK) {   // (uniform trip count)
        const uint32_t i = c + threadIdx.x;
        const uint32_t v = i < nb ? bsum[i] : 0u;
        const uint32_t e = block_excl_scan(v, tmp);
        if (i < nb)
            bsum[i] = carry + e;
        carry += tmp[31];   // (block_excl_scan left the block total there)
        __syncthreads();
    }
    if (threadIdx.x == 0)
        *total = carry;
}
__global__ __launch_bounds__(BLOCK) void k_scan_add(uint32_t *out, uint64_t n,
                                                    const uint32_t *bsum)
{
    const uint64_t b0 = (uint64_t)blockIdx.x * 4 * BLOCK + 4ull * threadIdx.x;
    const uint32_t add = bsum[blockIdx.x];
#pragma unroll
    for (int j = 0; j < 4; j++)
        if (b0 + j < n)
            out[b0 + j] += add;
}

__global__ __launch_bounds__(256) void k_add_u64(uint64_t *dst,
                                                 const uint64_t *src,
                                                 uint64_t n)
{
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n)
        dst[i] += src[i];
}

__global__ __launch_bounds__(256) void k_patch16(const Patch16 *rec, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        const uint4 v = *(const uint4 *)rec[i].val;
        *(uint4 *)rec[i].dst = v;
    }
}

#ifndef CFC_FAST
#define CFC_FAST 1   // 0: always the generic kernel (A/B builds)
#endif
// the epoch shape k_classify_v4<..., FAST = true> is compiled for
bool fast_shape(const DevTables &T, int mode, const LdsPlan &L)
{
    if (!CFC_FAST)
        return false;
    const bool xdp = mode == CFC_MODE_XDP || mode == CFC_MODE_FULL;
    return T.l4d && !T.tbl24 && !T.pf_tbl24 && T.lxc4 && L.lxc_slots && L.pol_words &&
           (!xdp || (T.pf_fix && L.pf_words));
}

template <int MODE, bool CT, bool NT>
void launch_mode_nt(const DevTables &T, const cfc_hdr_v4 &in, const cfc_out &out,
                    const EgressArgs &E, const CountArgs &C, uint32_t grid,
                    uint64_t per_block, hipStream_t s, const LbIn *lb)
{
    const LdsPlan L = lds_plan(T);
    const bool opt = in.mark || in.tcp_flags || out.action || (CT && out.ct);
    const bool fast = fast_shape(T, MODE, L);
    auto kern = opt ? (fast ? k_classify_v4<MODE, CFC_UNROLL, CT, NT, true, false, true>
                            : k_classify_v4<MODE, CFC_UNROLL, CT, NT, true, false, false>)
                    : (fast ? k_classify_v4<MODE, CFC_UNROLL, CT, NT, false, false, true>
                            : k_classify_v4<MODE, CFC_UNROLL, CT, NT, false, false, false>);
    const LbIn none{};
    if constexpr (CT && MODE != CFC_MODE_XDP) {
        if (lb)
            kern = k_classify_v4<MODE, CFC_UNROLL, CT, NT, true, true, false>;
    }
    set_lds_limit((const void *)kern, (int)LDS_PER_WG);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), L.bytes(), s, T, L, in,
                       out, E, C, per_block, lb ? *lb : none);
}

// the notify store is compiled in only when the caller asked for it
template <int MODE, bool CT>
void launch_mode(const DevTables &T, const cfc_hdr_v4 &in, const cfc_out &out,
                 const EgressArgs &E, const CountArgs &C, uint32_t grid,
                 uint64_t per_block, hipStream_t s, const LbIn *lb)
{
    if (out.notify)
        launch_mode_nt<MODE, CT, true>(T, in, out, E, C, grid, per_block, s, lb);
    else
        launch_mode_nt<MODE, CT, false>(T, in, out, E, C, grid, per_block, s, lb);
}

// histogram slices of an n-header batch with `slots` keys in all: one per
// CU of an MI355X (a slice of at most 2^24 headers, a multiple of 4), fewer
// when the partial slabs would pass 256 MiB
uint32_t hist_slices(uint64_t n, uint64_t slots)
{
    if (!n || !slots)
        return 0;
    uint64_t nb = std::min<uint64_t>(256, (n + 4095) / 4096);
    nb = std::min<uint64_t>(nb, std::max<uint64_t>(1, (256ull << 20) / (8 * slots)));
    nb = std::max<uint64_t>(nb, (n + SLICE_MAX - 1) / SLICE_MAX);
    return (uint32_t)std::max<uint64_t>(nb, 1);
}

uint64_t hist_per_block(uint64_t n, uint32_t nblk)
{
    const uint64_t pb = (n + nblk - 1) / nblk;
    return (pb + 3) & ~3ull;
}

// key slots the histogram covers: policy entries per stage, identities
uint64_t hist_slots(const DevTables &T, int mode)
{
    if (mode == CFC_MODE_XDP)
        return 0;
    uint64_t id_slots = 0;
    for (uint32_t r = 0; r < ID_RANGES; r++)
        if ((T.id_cover >> r) & 1)
            id_slots += std::min<uint64_t>(2 * ID_RANGE, 2ull * ID_PACK_LIMIT - 2ull * r * ID_RANGE);
    return (mode == CFC_MODE_EGRESS ? 2ull : 1ull) * T.n_ctr + id_slots;
}

}  // namespace

void set_lds_limit(const void *kernel, int bytes)
{
    static std::mutex mu;
    static std::set<std::tuple<int, const void *, int>> done;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    if (done.insert(std::make_tuple(dev, kernel, bytes)).second)
        (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  bytes);
}

size_t classify_lds_bytes(const DevTables &T) { return lds_plan(T).bytes(); }

int launch_patch16(const Patch16 *rec, uint64_t n, hipStream_t s)
{
    if (!n)
        return 0;
    hipLaunchKernelGGL(k_patch16, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, rec, n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_add_u64(uint64_t *dst, const uint64_t *src, uint64_t n,
                   hipStream_t s)
{
    if (!n)
        return 0;
    hipLaunchKernelGGL(k_add_u64, dim3((unsigned)((n + 255) / 256)), dim3(256),
                       0, s, dst, src, n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// key buckets of the CT accounting partition (0: too many keys, the
// per-slice kernel k_ct_count counts instead)
uint32_t ctp_buckets(const DevTables &T)
{
    const uint64_t slots = (T.ct4 ? T.ct4_mask + 1ull : 0) + (T.ct6 ? T.ct6_mask + 1ull : 0);
    const uint64_t nb = (2 * slots + CTP_BUCKET - 1) / CTP_BUCKET;
    return nb <= CTP_MAX_BUCKETS ? (uint32_t)nb : 0u;
}

WsLayout ws_layout(uint64_t n, const DevTables &T, int mode, bool ct)
{
    WsLayout w{};
    if (n == 0 || mode == CFC_MODE_XDP)
        return w;
    const bool egr = mode == CFC_MODE_EGRESS;
    const size_t a = 4 * ctr_stride(n);   // one u32 per header, 16-B aligned
    size_t off = 0;
    w.ctr = off;
    off += a;
    if (egr) {
        w.ctr2 = off;
        off += a;
    }
    w.id = off;
    off += a;
    if (ct) {
        w.ct = off;
        off += a;
        if (egr) {
            w.ct2 = off;
            off += a;
        }
    }
    off = (off + 255) & ~(size_t)255;
    w.partial = off;
    const uint64_t slots = hist_slots(T, mode);
    w.nblk = hist_slices(n, slots);
    off += 8ull * slots * w.nblk;
    const uint32_t nbuck = ctp_buckets(T);
    if (ct && T.ct_st && nbuck) {
        const uint64_t per = acc_slice(n);
        const uint32_t nblk = (uint32_t)((n + per - 1) / per);
        w.ctp_nv = nblk * (egr ? 2u : 1u);
        w.ctp_nbuck = nbuck;
        w.ctp_nco = (nbuck + ACC_FINE - 1) / ACC_FINE;
        const uint64_t cap = (uint64_t)w.ctp_nv * ACC_RCAP;
        const uint64_t nc = (uint64_t)w.ctp_nco * w.ctp_nv * ACC_SLICE_CHUNKS;
        w.ctp_g2 = (uint32_t)((cap + ACC_CHUNK - 1) / ACC_CHUNK + w.ctp_nco);
        auto take = [&](size_t bytes) {
            off = (off + 255) & ~(size_t)255;
            const size_t at = off;
            off += bytes;
            return at;
        };
        w.ctp_rec = take(8 * cap);
        w.ctp_recA = take(8 * cap);
        w.ctp_rcnt = take(4ull * w.ctp_nv);
        w.ctp_cnt = take(4 * nc);
        w.ctp_off = take(4 * nc + 4);
        w.ctp_bsum = take(4 * ((nc + 4 * BLOCK - 1) / (4 * BLOCK)) + 4);
        w.ctp_plan = take(4ull * (2 * w.ctp_nco + 2));
        w.ctp_fo = take(4ull * w.ctp_g2 * (ACC_FINE + 1));
    }
    if (egr && (T.lb4 || T.rnat4)) {   // the service step's six arrays (lb.hip)
        off = (off + 255) & ~(size_t)255;
        w.lb = off;
        off += 6 * a;
    }
    w.total = off;
    return w;
}

CountArgs count_args(uint32_t *ws, const WsLayout &w, const DevTables &T,
                     uint64_t *g_met, int mode, bool ct)
{
    CountArgs C{};
    char *b = reinterpret_cast<char *>(ws);
    if (w.total) {
        C.ctr = reinterpret_cast<uint32_t *>(b + w.ctr);
        C.ctr2 = mode == CFC_MODE_EGRESS ? reinterpret_cast<uint32_t *>(b + w.ctr2) : nullptr;
        C.id = reinterpret_cast<uint32_t *>(b + w.id);
        C.ct = ct ? reinterpret_cast<uint32_t *>(b + w.ct) : nullptr;
        C.ct2 = ct && mode == CFC_MODE_EGRESS ? reinterpret_cast<uint32_t *>(b + w.ct2)
                                              : nullptr;
    }
    C.g_met = g_met;
    C.g_id = g_met + METRIC_U64;
    C.ctr_packed = T.n_ctr < PACK_MAX;
    return C;
}

int launch_classify_v4(const DevTables &T, const cfc_hdr_v4 &in,
                       const cfc_out &out, int mode, const EgressArgs &E,
                       uint64_t *g_ctr, uint32_t *ws, int num_cus, hipStream_t s,
                       const LaunchTiming *tm)
{
    if (in.n == 0)
        return 0;
    if (classify_lds_bytes(T) > LDS_PER_WG)
        return -22;
    // CFC_WG_PER_CU workgroups per CU (the LDS image allows no more), a
    // contiguous slice each, rounded to whole loop iterations
    const uint64_t step = (uint64_t)BLOCK * CFC_UNROLL;
    const uint64_t nwg = (uint64_t)num_cus * CFC_WG_PER_CU;
    uint64_t per_block = (in.n + nwg - 1) / nwg;
    per_block = (per_block + step - 1) / step * step;
    // slices stay below 2^30 headers (32-bit byte offsets in the kernel)
    per_block = std::min<uint64_t>(per_block, (1ull << 30) / step * step);
    const uint32_t grid = (uint32_t)((in.n + per_block - 1) / per_block);
    if (tm)
        (void)hipEventRecord(tm->ev[0], s);
    // conntrack lookups when CT maps hold entries or the caller wants the
    // CT byte (to fold creates into the maps); an empty map misses anyway
    // with a load balancer every tc-path batch looks up CT (service entries,
    // reverse NAT) and runs the LB variant
    const bool lb = (T.lb4 || T.rnat4) && mode != CFC_MODE_XDP;
    const bool ct = T.ct4 || out.ct || lb;
    const WsLayout w = ws_layout(in.n, T, mode, ct);
    const CountArgs C = count_args(ws, w, T, g_ctr + 2ull * T.n_ctr, mode, ct);
    cfc_hdr_v4 hin = in;
    LbIn li{};
    if (lb && mode == CFC_MODE_EGRESS) {
        // the service step first (lb.hip): the classify kernel reads the
        // packet's daddr / L4 word from it and the tuple it left
        uint32_t *a = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(ws) + w.lb);
        const uint64_t st = ctr_stride(in.n);
        LbArgs A{in.saddr, in.daddr, in.ports, in.meta, in.hash, in.n, E.ct_owner,
                 a, a + st, a + 2 * st, a + 3 * st, a + 4 * st, a + 5 * st, E.svo};
        if (int rc = launch_lb4_egress(T, A, s))
            return rc;
        li = LbIn{A.tda, A.tpt, A.psa, A.fl};
        hin.daddr = A.pda;
        hin.ports = A.ppt;
    } else if (out.pkt_saddr && !lb) {   // nothing rewrites the packet
        if (hipMemcpyAsync(out.pkt_saddr, in.saddr, 4 * in.n, hipMemcpyDeviceToDevice, s) ||
            hipMemcpyAsync(out.pkt_daddr, in.daddr, 4 * in.n, hipMemcpyDeviceToDevice, s) ||
            hipMemcpyAsync(out.pkt_ports, in.ports, 4 * in.n, hipMemcpyDeviceToDevice, s))
            return -5;
    }
    const LbIn *lbp = lb ? &li : nullptr;
#define CFC_LAUNCH(M)                                                        \
    (ct ? launch_mode<M, true>(T, hin, out, E, C, grid, per_block, s, lbp)   \
        : launch_mode<M, false>(T, hin, out, E, C, grid, per_block, s, lbp))
    switch (mode) {
    case CFC_MODE_INGRESS: CFC_LAUNCH(CFC_MODE_INGRESS); break;
    case CFC_MODE_EGRESS: CFC_LAUNCH(CFC_MODE_EGRESS); break;
    case CFC_MODE_XDP:
        launch_mode<CFC_MODE_XDP, false>(T, hin, out, E, C, grid, per_block, s, nullptr);
        break;
    case CFC_MODE_FULL: CFC_LAUNCH(CFC_MODE_FULL); break;
    default: return -22;
    }
#undef CFC_LAUNCH
    if (tm)
        (void)hipEventRecord(tm->ev[1], s);
    const bool sums = launch_counters(T, in.meta, in.tcp_flags, in.n, mode, ws, g_ctr, s, ct);
    if (E.sums)
        *E.sums = sums;
    if (tm)
        (void)hipEventRecord(tm->ev[2], s);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -5;
}

bool launch_counters(const DevTables &T, const uint32_t *meta, const uint8_t *tf, uint64_t n,
                     int mode, uint32_t *ws, uint64_t *g_ctr, hipStream_t s,
                     bool ct)
{
    bool sums = false;
    if (!n || mode == CFC_MODE_XDP)
        return sums;
    const WsLayout w = ws_layout(n, T, mode, ct);
    const CountArgs C = count_args(ws, w, T, g_ctr + 2ull * T.n_ctr, mode, ct);
    if (ct && T.ct_st && w.ctp_nv) {
        char *b = reinterpret_cast<char *>(ws);
        uint64_t *rec = reinterpret_cast<uint64_t *>(b + w.ctp_rec);
        uint64_t *recA = reinterpret_cast<uint64_t *>(b + w.ctp_recA);
        uint32_t *rcnt = reinterpret_cast<uint32_t *>(b + w.ctp_rcnt);
        uint32_t *cnt = reinterpret_cast<uint32_t *>(b + w.ctp_cnt);
        uint32_t *off = reinterpret_cast<uint32_t *>(b + w.ctp_off);
        uint32_t *bsum = reinterpret_cast<uint32_t *>(b + w.ctp_bsum);
        uint32_t *plan = reinterpret_cast<uint32_t *>(b + w.ctp_plan);
        uint32_t *fo = reinterpret_cast<uint32_t *>(b + w.ctp_fo);
        const uint64_t per = acc_slice(n);
        const uint32_t nblk = (uint32_t)((n + per - 1) / per);
        const uint32_t nch = w.ctp_nv * ACC_SLICE_CHUNKS;
        const uint64_t nc = (uint64_t)w.ctp_nco * nch;
        const uint32_t nsb = (uint32_t)((nc + 4 * BLOCK - 1) / (4 * BLOCK));
        // 16-byte loads when the header meta allows (the key arrays are
        // 16-byte aligned workspace)
        const bool vec = ((uintptr_t)meta & 15) == 0 && (!T.ct_sum || ((uintptr_t)tf & 3) == 0);
        const void *agg = vec ? (const void *)k_acc_agg<true> : (const void *)k_acc_agg<false>;
        set_lds_limit(agg, (int)ACC_AGG_LDS);
        if (vec)
            hipLaunchKernelGGL(k_acc_agg<true>, dim3(nblk, mode == CFC_MODE_EGRESS ? 2 : 1),
                               dim3(BLOCK), ACC_AGG_LDS, s, C.ct, C.ct2, meta,
                               T.ct_sum ? tf : nullptr, T.ct_sum != nullptr, n,
                               w.ctp_nco, rec, rcnt, cnt, per);
        else
            hipLaunchKernelGGL(k_acc_agg<false>, dim3(nblk, mode == CFC_MODE_EGRESS ? 2 : 1),
                               dim3(BLOCK), ACC_AGG_LDS, s, C.ct, C.ct2, meta,
                               T.ct_sum ? tf : nullptr, T.ct_sum != nullptr, n,
                               w.ctp_nco, rec, rcnt, cnt, per);
        hipLaunchKernelGGL(k_scan_local, dim3(nsb), dim3(BLOCK), 0, s, cnt, off, nc, bsum);
        hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(BLOCK), 0, s, bsum, nsb, off + nc);
        hipLaunchKernelGGL(k_scan_add, dim3(nsb), dim3(BLOCK), 0, s, off, nc, bsum);
        set_lds_limit((const void *)k_acc_part1, (int)ACC_SORT_LDS);
        hipLaunchKernelGGL(k_acc_part1, dim3(nch), dim3(BLOCK), ACC_SORT_LDS, s, rec, rcnt,
                           off, nch, w.ctp_nco, recA);
        hipLaunchKernelGGL(k_acc_plan, dim3(1), dim3(64), 0, s, off, nch, w.ctp_nco, plan);
        // the fine sort writes over the staged records (read by part1 only)
        set_lds_limit((const void *)k_acc_part2, (int)ACC_SORT_LDS);
        hipLaunchKernelGGL(k_acc_part2, dim3(w.ctp_g2), dim3(BLOCK), ACC_SORT_LDS, s, recA,
                           plan, w.ctp_nco, rec, fo);
        set_lds_limit((const void *)k_acc_reduce, (int)ACC_RED_LDS);
        hipLaunchKernelGGL(k_acc_reduce, dim3(w.ctp_nbuck), dim3(BLOCK), ACC_RED_LDS, s, rec,
                           plan, fo, w.ctp_nco, T.ct_st, T.ct_sum);
        sums = T.ct_sum != nullptr;
    } else if (ct && T.ct_st) {
        set_lds_limit((const void *)k_ct_count, (int)CT_LDS_BYTES);
        const uint32_t nblk = (uint32_t)((n + COUNT_PER_BLOCK - 1) / COUNT_PER_BLOCK);
        hipLaunchKernelGGL(k_ct_count, dim3(nblk, mode == CFC_MODE_EGRESS ? 2 : 1),
                           dim3(BLOCK), CT_LDS_BYTES, s, C.ct, C.ct2, meta, n, T.ct_st);
    }
    // the histogram jobs: policy ranges of each stage, identity ranges
    std::vector<HistJob> jobs;
    uint64_t poff = 0;
    auto add_jobs = [&](const uint32_t *keys, uint32_t nkeys, uint32_t kind,
                        uint32_t packed) {
        for (uint32_t lo = 0; lo < nkeys; lo += HIST_RANGE) {
            HistJob j{keys, poff, lo, std::min(HIST_RANGE, nkeys - lo), kind, packed};
            poff += (uint64_t)w.nblk * j.cnt;
            jobs.push_back(j);
        }
    };
    add_jobs(C.ctr, T.n_ctr, 0, C.ctr_packed);
    if (mode == CFC_MODE_EGRESS)
        add_jobs(C.ctr2, T.n_ctr, 0, C.ctr_packed);
    for (uint32_t r = 0; r < ID_RANGES; r++) {   // the identity ranges in use
        if (!((T.id_cover >> r) & 1))
            continue;
        const uint32_t lo = 2 * r * ID_RANGE;
        HistJob j{C.id, poff, lo, std::min(2 * ID_RANGE, 2 * ID_PACK_LIMIT - lo), 1, 1};
        poff += (uint64_t)w.nblk * j.cnt;
        jobs.push_back(j);
    }
    if (jobs.empty())
        return sums;
    uint64_t *partial = reinterpret_cast<uint64_t *>(reinterpret_cast<char *>(ws) + w.partial);
    const uint64_t per_block = hist_per_block(n, w.nblk);
    set_lds_limit((const void *)k_hist, (int)(8 * HIST_RANGE));
    const uint32_t id_dir = mode == CFC_MODE_EGRESS ? ID_DIR_EGRESS : ID_DIR_INGRESS;
    for (size_t a = 0; a < jobs.size(); a += HIST_JOBS_MAX) {
        HistJobs J{};
        const uint32_t nj = (uint32_t)std::min<size_t>(HIST_JOBS_MAX, jobs.size() - a);
        uint32_t cmax = 0;
        for (uint32_t k = 0; k < nj; k++) {
            J.j[k] = jobs[a + k];
            cmax = std::max(cmax, J.j[k].cnt);
        }
        hipLaunchKernelGGL(k_hist, dim3(w.nblk, nj), dim3(BLOCK), 8ull * cmax, s, J,
                           meta, n, per_block, partial);
        hipLaunchKernelGGL(k_hist_reduce,
                           dim3((cmax + 255) / 256, nj, (w.nblk + REDUCE_ROWS - 1) / REDUCE_ROWS),
                           dim3(256), 0, s, J, partial, w.nblk, g_ctr, C.g_id, id_dir);
    }
    return sums;
}

}  // namespace cfc
