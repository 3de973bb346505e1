// Shared device code of the conntrack apply (ctapply.hip) and the
// packet-order resolution (ctorder.hip): the per-slot marks, block-wide
// counters, the address-family templates, one CT stage decoded as an op
// (Op, decode_from), and the device table's find / insert.
#pragma once
#include <type_traits>

#include "kern_common.hpp"

namespace cfc {

namespace {

constexpr uint32_t CT_LIFETIME_TCP = 21600, CT_LIFETIME_NONTCP = 60, CT_SYN_TIMEOUT = 60,
                   CT_CLOSE_TIMEOUT = 10, CT_REPORT_INTERVAL = 5;
constexpr uint32_t RX_CLOSING = 1, TX_CLOSING = 2, NAT46 = 4, SEEN_NON_SYN = 16;   // ct_entry bits
constexpr uint32_t OP_NONE = 0, OP_HIT = 1, OP_DELETE = 2, OP_CREATE = 3;
// per-slot marks of one apply: ordered ops; inserted by this apply; a
// delete among its ops; a create or related-entry write among its ops
constexpr uint32_t MARK_ORDERED = 1, MARK_FRESH = 2, MARK_DEL = 4, MARK_PUTC = 8;
__device__ __forceinline__ void mark_or(uint32_t *m, uint32_t bits)
{
    if ((*m & bits) != bits)
        atomicOr(m, bits);
}
// A slot's word x holds its marks (bits 0-3) and the summary of its plain
// hits (bits 8-26, see k_cta_finish): both only ever OR'ed in.  y holds the
// order of a deleted entry's first delete.  The ordered slots are also bits
// of A.obm, which k_cta_route tests per hit (a few MiB: cache-resident,
// where the per-slot words are not).
constexpr int SUM_SH = 8;
__device__ __forceinline__ uint32_t sum_bits(bool in, bool tcp, bool close, uint32_t tfl)
{
    return ((in ? tfl : tfl << 8) | (in ? 1u << 16 : 1u << 17) |
            ((tcp && !close) ? 1u << 18 : 0u)) << SUM_SH;
}
__device__ __forceinline__ void order_mark(const CtaArgs &A, uint32_t sl, uint32_t bits)
{
    if ((A.ms[sl].x & bits) != bits) {
        atomicOr(&A.ms[sl].x, bits);
        const uint32_t b = 1u << (sl & 31);
        if (!(A.obm[sl >> 5] & b))
            atomicOr(&A.obm[sl >> 5], b);
    }
}
constexpr uint32_t HS_NONE = 0xFFFFFFFFu;

// An op's place in the batch, the low bits of every request and list entry:
// ((2 * i + st) << 3) | sec << 1 — i the header (with a load balancer,
// i = n + h is the CT_SERVICE op of header h), st its CT stage, sec the
// write: the op itself, its create's related ICMP entry, its create's
// reverse-NAT entry (ct_create4 with ct_state->addr), or a hit on an entry
// this batch created (the destination's lookup finding what the sender's
// create just wrote).  Bit 0 is free: a request's first-create mark.
constexpr uint32_t SEC_OP = 0, SEC_REL = 1, SEC_KX = 2, SEC_FHIT = 3;
__device__ __forceinline__ uint32_t ord_of(uint64_t i, int st, uint32_t sec)
{
    return (uint32_t)(((2 * i + (uint64_t)st) << 3) | sec << 1);
}
__device__ __forceinline__ uint64_t ord_hdr(uint32_t o) { return o >> 4; }
__device__ __forceinline__ int ord_st(uint32_t o) { return (int)((o >> 3) & 1); }
__device__ __forceinline__ uint32_t ord_sec(uint32_t o) { return (o >> 1) & 3; }

__device__ __forceinline__ uint32_t wave_count(uint32_t *ctr, bool want)
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

// the same for a whole block of 256 threads: one atomic per block, not per
// wave (a counter every wave of a 64M-header pass bumps serialises at its
// L2 channel).  Every thread of the block calls it.
__device__ __forceinline__ uint32_t block_count(uint32_t *ctr, bool want)
{
    __shared__ uint32_t wsum[16], base;   // (up to 1024 threads)
    const uint64_t m = __ballot(want);
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0)
        wsum[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t k = 0; k < (blockDim.x >> 6); k++)
            t += wsum[k];
        base = t ? atomicAdd(ctr, t) : 0u;
    }
    __syncthreads();
    uint32_t r = base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
    for (uint32_t k = 0; k < wv; k++)
        r += wsum[k];
    __syncthreads();   // wsum and base are reused by the next call
    return r;
}
// n items of this thread in a block-wide list: the first one's index, one
// atomic per block (every thread of the block calls it; up to 1024 threads)
__device__ __forceinline__ uint32_t block_count_n(uint32_t *ctr, uint32_t v)
{
    __shared__ uint32_t wsum[16], base;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d)
            x += y;
    }
    if (lane == 63)
        wsum[wv] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t k = 0; k < (blockDim.x >> 6); k++)
            t += wsum[k];
        base = t ? atomicAdd(ctr, t) : 0u;
    }
    __syncthreads();
    uint32_t r = base + x - v;
    for (uint32_t k = 0; k < wv; k++)
        r += wsum[k];
    __syncthreads();
    return r;
}
// n items of this thread in a block's LDS staging list: their first index
// there (the list's length in *sn); every thread of the block calls it
__device__ __forceinline__ uint32_t block_stage_n(uint32_t *sn, uint32_t v)
{
    __shared__ uint32_t wsum[4], base;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d)
            x += y;
    }
    if (lane == 63)
        wsum[wv] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        base = *sn;
        *sn = base + wsum[0] + wsum[1] + wsum[2] + wsum[3];
    }
    __syncthreads();
    uint32_t r = base + x - v;
    for (uint32_t k = 0; k < wv; k++)
        r += wsum[k];
    __syncthreads();
    return r;
}
// the block's staged list into dst at places taken by one atomic on *ctr
// (cap: dst's capacity); every thread of the block calls it
__device__ __forceinline__ void block_flush(uint64_t *stage, uint32_t *sn, uint32_t *ctr,
                                            uint64_t *dst, uint32_t cap)
{
    __shared__ uint32_t gbase;
    const uint32_t n = *sn;
    if (threadIdx.x == 0)
        gbase = n ? atomicAdd(ctr, n) : 0u;
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < n; j += blockDim.x)
        if (gbase + j < cap)
            dst[gbase + j] = stage[j];
    __syncthreads();
    if (threadIdx.x == 0)
        *sn = 0;
    __syncthreads();
}

// a per-thread count added once per block (every thread of the block calls
// it): counters that every wave of a full-table pass bumps serialise at
// their L2 channel
__device__ __forceinline__ void block_add(uint32_t *ctr, uint32_t v)
{
    __shared__ uint32_t wsum[16];   // (up to 1024 threads)
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0)
        wsum[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t k = 0; k < (blockDim.x >> 6); k++)
            t += wsum[k];
        if (t)
            atomicAdd(ctr, t);
    }
    __syncthreads();
}
// a per-thread count added once per wave (every lane of the wave calls it)
__device__ __forceinline__ void wave_add(uint32_t *ctr, uint32_t v)
{
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v)
        atomicAdd(ctr, v);
}

// ---- the address family.  A CT tuple's addresses are raw (network order,
// loaded little-endian): one word for IPv4, four for IPv6.  The kernels are
// templated on V6; the slot layouts are Ct4Slot / Ct6Slot (layout.h).
template <bool V6>
using Addr = typename std::conditional<V6, uint4, uint32_t>::type;
__device__ __forceinline__ bool aeq(uint32_t a, uint32_t b) { return a == b; }
__device__ __forceinline__ bool aeq(uint4 a, uint4 b)
{
    return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w;
}
__device__ __forceinline__ uint32_t khash(uint32_t d, uint32_t s, uint32_t z, uint32_t w)
{
    return ct_hash4(d, s, z, w);
}
__device__ __forceinline__ uint32_t khash(uint4 d, uint4 s, uint32_t z, uint32_t w)
{
    const uint32_t dw[4] = {d.x, d.y, d.z, d.w}, sw[4] = {s.x, s.y, s.z, s.w};
    return ct_hash6(dw, sw, z, w);
}
// the key's home slot (placement, layout.h ct_home4 / ct_home6; khash is
// the mixer the fingerprints use)
__device__ __forceinline__ uint32_t khome(uint32_t d, uint32_t s, uint32_t z, uint32_t w)
{
    return ct_home4(d, s, z, w);
}
__device__ __forceinline__ uint32_t khome(uint4 d, uint4 s, uint32_t z, uint32_t w)
{
    const uint32_t dw[4] = {d.x, d.y, d.z, d.w}, sw[4] = {s.x, s.y, s.z, s.w};
    return ct_home6(dw, sw, z, w);
}
template <bool V6>
__device__ __forceinline__ Addr<V6> ld_addr(const uint32_t *p, uint64_t i)
{
    if constexpr (V6)
        return ld16(reinterpret_cast<const uint4 *>(p) + i);
    else
        return p[i];
}
// the ICMP protocol of the family (ct_create4/6's related entry)
template <bool V6>
constexpr uint32_t icmp_proto()
{
    return V6 ? 58u : 1u;
}
// the w word of slot i
template <bool V6>
__device__ __forceinline__ uint32_t *slot_w(const CtaArgs &A, uint32_t i)
{
    if constexpr (V6)
        return &A.ct6[i].w;
    else
        return &A.ct4[i].w;
}

// one CT stage of one header, decoded as cfc_api.cpp ct_apply does
template <bool V6>
struct Op {
    uint32_t kind, action, dir;
    bool is_tcp, syn, ki_form;
    uint32_t tfl, len, sec, owner, proto, rev;
    Addr<V6> sa, da;           // k1 = (da, sa, z1, w1), k2 = (sa, da, z2, w2)
    uint32_t z1, w1;           // k1: the tuple as loaded (REPLY / RELATED)
    uint32_t z2, w2;           // k2: reversed (ESTABLISHED / create)
    // the ct_state a create writes with the entry (ct4_lb / ct6_lb words:
    // rev_nat_index | lb_loopback << 16, slave; its related entry's slave)
    uint32_t lbw, slave, slave_rel;
    bool reslave;              // a CT_SERVICE op's ct_update4/6_slave
    // ct_create4's reverse-NAT entry (kx: the create writes one): key
    // (kxa, kxs, z2, kxw)
    bool kx;
    Addr<V6> kxa, kxs;
    uint32_t kxw;
};

// owner word of the destination endpoint's CT maps (cilium_lxc lookup)
__device__ __forceinline__ uint32_t dst_owner(const DevTables &T, uint32_t da)
{
    if (!T.lxc4)
        return 0;
    uint32_t s = hash32(da, T.lxc4_mask);
    for (;;) {
        const uint4 v = ld16(T.lxc4 + s);
        if (!(v.w & LXC_VALID))
            return 0;
        if (v.x == da)
            return ct_owner_word(v.w & 0xFFFF, (v.w & LXC_CT_LOCAL) != 0);
        s = (s + 1) & T.lxc4_mask;
    }
}
__device__ __forceinline__ uint32_t dst_owner(const DevTables &T, uint4 da)
{
    if (!T.lxc6)
        return 0;
    uint32_t s = l6_hash(da.x, da.y, da.z, da.w, L6_LXC_TAG) & T.lxc6_mask;
    for (;;) {
        const uint4 k = ld16(&T.lxc6[s].a[0]);
        const uint4 v = ld16(&T.lxc6[s].pol_base);   // {pol_base, pol_mask, info, 0}
        if (!(v.z & LXC_VALID))
            return 0;
        if (aeq(k, da))
            return ct_owner_word(v.z & 0xFFFF, (v.z & LXC_CT_LOCAL) != 0);
        s = (s + 1) & T.lxc6_mask;
    }
}

// is_valid_lxc_src_ip (lxc.h:46-57): the source address is the sending
// endpoint's (cilium_lxc)
__device__ __forceinline__ bool lb4_src_ok(const DevTables &T, uint32_t sa, uint32_t lxc_id)
{
    if (!T.lxc4)
        return false;
    for (uint32_t s = hash32(sa, T.lxc4_mask);; s = (s + 1) & T.lxc4_mask) {
        const uint4 v = ld16(T.lxc4 + s);
        if (!(v.w & LXC_VALID))
            return false;
        if (v.x == sa)
            return (v.w & 0xFFFF) == lxc_id;
    }
}
__device__ __forceinline__ bool lb6_src_ok(const DevTables &T, uint4 sa, uint32_t lxc_id)
{
    if (!T.lxc6)
        return false;
    for (uint32_t s = l6_hash(sa.x, sa.y, sa.z, sa.w, L6_LXC_TAG) & T.lxc6_mask;;
         s = (s + 1) & T.lxc6_mask) {
        const uint4 k = ld16(&T.lxc6[s].a[0]);
        const uint4 v = ld16(&T.lxc6[s].pol_base);
        if (!(v.z & LXC_VALID))
            return false;
        if (aeq(k, sa))
            return (v.z & 0xFFFF) == lxc_id;
    }
}

template <bool V6>
using LbRecT = typename std::conditional<V6, LbRec6, LbRec4>::type;

// one header's inputs of the apply; with a load balancer (LB) its service
// step's record too, and svcop: the header's CT_SERVICE op (virtual header
// n + i) rather than its CT stages
template <bool V6>
struct ScanIn {
    uint32_t cb, pt, mt, ver, ident, tf, k1, k2;
    Addr<V6> sa, da;
    Addr<V6> tda, psa, pda;
    uint32_t tpt, ppt, lfl, lbw, slv, svc, addr, sva;
    bool svcop;
};

// stage st of a header, from its inputs; dsto: the owner word of the
// destination endpoint's CT maps (the stages that are not the sender's)
template <bool V6, bool LB>
__device__ __forceinline__ Op<V6> decode_from(const CtaArgs &A, const ScanIn<V6> &r, int st,
                                              uint32_t dsto)
{
    Op<V6> o;
    o.kind = OP_NONE;
    o.lbw = o.slave = o.slave_rel = 0;
    o.reslave = o.kx = false;
    if (LB && r.svcop) {
        // lb4_local / lb6_local's ct_lookup4/6(CT_SERVICE): the tuple as
        // loaded with TUPLE_F_SERVICE, one lookup (conntrack.h:580); a miss
        // creates the entry (ct_create4/6 with ct_state {slave}, lb.h:699-
        // 712).  The key sits in the k2 fields, which creates insert.
        if (st != 0 || !(r.lfl & LBF_SVC))
            return o;
        o.proto = r.mt & 0xFF;
        if (o.proto != 6 && o.proto != 17 && o.proto != icmp_proto<V6>())
            return o;
        o.dir = CT_SERVICE;   // (the tx side of the entry, as egress)
        o.owner = A.ep_owner;
        o.len = r.mt >> 16;
        o.is_tcp = o.proto == 6;
        o.syn = (r.mt & CFC_HF_TCP_CLOSE) != 0;
        o.tfl = o.is_tcp ? r.tf : 0u;
        o.action = ct_action(V6, o.proto, r.pt, r.mt);
        o.sec = 0;
        o.rev = 0;
        const CtProbe k = ct_probe<V6>(o.proto, r.pt, CT_SERVICE, o.owner);
        o.sa = r.da;
        o.da = r.sa;
        o.z1 = o.z2 = k.z1;
        o.w1 = o.w2 = k.w1;
        o.ki_form = o.proto == icmp_proto<V6>() && (k.w1 & 0x200u) && k.z1 == 0;
        // the entry's slave: the selection, or ct_update4/6_slave's; its
        // ICMP entry keeps the selection (slave0)
        o.reslave = (r.lfl & LBR_RESLAVE) != 0;
        o.slave = r.slv & 0xFFFF;
        o.slave_rel = r.slv >> 16;
        o.kind = r.svc != NONE ? OP_HIT : OP_CREATE;
        return o;
    }
    const uint32_t cs = (r.cb >> (4 * st)) & 0xF;
    if (!(cs & CFC_CT_DONE))
        return o;
    if (LB && (r.lfl & LBF_DROP))   // (no backend after all: no CT stage ran)
        return o;
    const int last = (r.cb & (CFC_CT_DONE << 4)) ? 1 : 0;
    const bool eg = A.mode == CFC_MODE_EGRESS && st == 0;
    o.dir = eg ? CT_EGRESS : CT_INGRESS;
    o.owner = eg ? A.ep_owner : dsto;
    o.proto = r.mt & 0xFF;
    if (o.proto != 6 && o.proto != 17 && o.proto != icmp_proto<V6>())
        return o;
    // the tuple this stage looked up: with a load balancer, the sender's
    // (saddr, the service step's daddr and L4 word), then the packet as
    // translated and reverse-NATed
    Addr<V6> ka = r.sa, kb = r.da;
    uint32_t pt = r.pt;
    if (LB) {
        ka = eg ? r.sa : r.psa;
        kb = eg ? r.tda : r.pda;
        pt = eg ? r.tpt : r.ppt;
    }
    o.len = r.mt >> 16;
    o.is_tcp = o.proto == 6;
    o.syn = (r.mt & CFC_HF_TCP_CLOSE) != 0;
    o.tfl = o.is_tcp ? r.tf : 0u;
    o.action = ct_action(V6, o.proto, pt, r.mt);
    o.sec = A.mode == CFC_MODE_EGRESS ? A.ep_sec : r.ident;
    // ipv6_policy's rev_nat_index: daddr.s6_addr32[3] as a u16
    // (bpf_lxc.c:787-788); IPv4 creates outside a load balancer carry 0
    if constexpr (V6)
        o.rev = o.dir == CT_INGRESS ? (kb.w & 0xFFFF) : 0u;
    else
        o.rev = 0;
    const bool svc = LB && eg && (r.lfl & LBF_SVC);
    if (svc) {   // lb4_local / lb6_local's ct_state for the create
        o.rev = r.lbw & 0xFFFF;
        o.slave = o.slave_rel = r.slv & 0xFFFF;
    }
    o.lbw = V6 ? o.rev : (svc ? r.lbw : 0u);
    const CtProbe k = ct_probe<V6>(o.proto, pt, (int)o.dir, o.owner);
    o.sa = ka;
    o.da = kb;
    o.z1 = k.z1; o.w1 = k.w1;
    o.z2 = k.z2; o.w2 = k.w2;
    // a k2 of ICMP-error form is its own related entry (ct_create4/6 write
    // the same key twice)
    o.ki_form = o.proto == icmp_proto<V6>() && (k.w2 & 0x200u) && k.z2 == 0;
    if constexpr (!V6) {
        // ct_create4 with ct_state->addr: the entry again with daddr
        // ct_state->addr (a looped-back flow's: TUPLE_F_IN, saddr svc_addr;
        // conntrack.h:731-739)
        if (svc && r.addr) {
            const bool loop = (r.lbw >> 16) & 1;
            o.kx = true;
            o.kxa = r.addr;
            o.kxs = loop ? r.sva : kb;
            o.kxw = loop ? ct_word(o.proto, 1u, o.owner) : k.w2;
        }
    }
    const uint32_t b = cs & CFC_CT_RES_MASK;
    const bool dropped = st == last && (int32_t)r.ver == DROP_POLICY;
    if (b >= 2)
        o.kind = OP_HIT;
    else if (b == 1)
        o.kind = dropped ? OP_DELETE : OP_HIT;
    else if (cs & CFC_CT_CREATE)
        o.kind = OP_CREATE;
    return o;
}

// KEY: the op's key words are needed (not by the fold of an IPv4 batch
// without a load balancer: its slot is the key, and rev is 0)
template <bool V6, bool LB, bool KEY = true>
__device__ __forceinline__ void load_in(const CtaArgs &A, uint64_t i, ScanIn<V6> &r)
{
    r.svcop = LB && i >= A.n;
    if (r.svcop)
        i -= A.n;
    r.cb = A.ctb[i];
    if (KEY || V6 || LB) {
        r.sa = ld_addr<V6>(A.sa, i);
        r.da = ld_addr<V6>(A.da, i);
    } else {
        r.sa = r.da = Addr<V6>{};
    }
    r.pt = A.pt[i];
    r.mt = A.mt[i];
    r.ver = (uint32_t)A.ver[i];
    r.ident = A.ident[i];
    r.tf = A.tf ? A.tf[i] : 0u;
    if constexpr (LB) {
        const LbRecT<V6> &l = reinterpret_cast<const LbRecT<V6> *>(A.lbr)[i];
        r.tda = l.tda;
        r.psa = l.psa;
        r.pda = l.pda;
        r.tpt = l.tpt;
        r.ppt = l.ppt;
        r.lfl = l.fl;
        r.lbw = l.lbw;
        r.slv = l.slv;
        r.svc = l.svc;
        r.addr = l.addr;
        r.sva = l.sva;
    }
}

template <bool V6, bool LB>
__device__ __forceinline__ Op<V6> decode_t(const CtaArgs &A, uint64_t i, int st)
{
    ScanIn<V6> r;
    if (!LB || i < A.n) {
        r.cb = A.ctb[i];
        if (!((r.cb >> (4 * st)) & CFC_CT_DONE)) {
            Op<V6> o;
            o.kind = OP_NONE;
            o.kx = false;
            return o;
        }
    }
    load_in<V6, LB>(A, i, r);
    const bool eg = A.mode == CFC_MODE_EGRESS && st == 0;
    return decode_from<V6, LB>(A, r, st,
                               (eg || r.svcop) ? 0u : dst_owner(A.T, LB ? r.pda : r.da));
}
// op (header i, stage st); i >= n: a CT_SERVICE op (A.lbr)
template <bool V6>
__device__ __forceinline__ Op<V6> decode(const CtaArgs &A, uint64_t i, int st)
{
    return A.lbr ? decode_t<V6, true>(A, i, st) : decode_t<V6, false>(A, i, st);
}

__device__ __forceinline__ uint32_t find(const CtaArgs &A, uint32_t x, uint32_t y, uint32_t z,
                                         uint32_t w)
{
    const uint32_t mask = A.mask;
    for (uint32_t i = ct_home4(x, y, z, w) & mask;; i = (i + 1) & mask) {
        const uint4 s = ld16(A.ct4 + i);
        if (s.w == 0)
            return NONE;
        if (s.x == x && s.y == y && s.z == z && s.w == w)
            return i;
    }
}
__device__ __forceinline__ uint32_t find(const CtaArgs &A, uint4 d, uint4 s, uint32_t z,
                                         uint32_t w)
{
    const uint32_t mask = A.mask;
    for (uint32_t i = khome(d, s, z, w) & mask;; i = (i + 1) & mask) {
        const uint4 t = ld16(&A.ct6[i].z);   // {z, w, 0, 0}: compared first
        if (t.y == 0)
            return NONE;
        if (t.x == z && t.y == w && aeq(ld16(A.ct6[i].d), d) && aeq(ld16(A.ct6[i].s), s))
            return i;
    }
}
// a claimed slot's key words (everything but w)
__device__ __forceinline__ void put_key(const CtaArgs &A, uint32_t i, uint32_t d, uint32_t s,
                                        uint32_t z)
{
    A.ct4[i].x = d;
    A.ct4[i].y = s;
    A.ct4[i].z = z;
}
__device__ __forceinline__ void put_key(const CtaArgs &A, uint32_t i, uint4 d, uint4 s,
                                        uint32_t z)
{
    *reinterpret_cast<uint4 *>(A.ct6[i].d) = d;
    *reinterpret_cast<uint4 *>(A.ct6[i].s) = s;
    A.ct6[i].z = z;
}

// The slot of a key no other thread of this launch inserts: found, or a
// free one claimed (CAS on w: atomics are coherent across the XCDs) and
// filled.  No agent-scope fence between the key words and w: that is an L2
// write-back and invalidate per insert (MI355X_MICROARCH.md), and nothing in
// this launch needs it — the only thread that looks this key up is this one
// (one thread per home slot), another thread's probe only needs to see the
// slot taken (w != 0 once the CAS is done), and a reader on another XCD
// that saw w ahead of the key words would see them as the zeros of the free
// slot, which no CT key has (saddr and daddr are never both 0 on the path).
// The launch's end writes the L2s back for the kernels after it.
template <bool V6>
__device__ uint32_t find_or_insert(const CtaArgs &A, Addr<V6> d, Addr<V6> s, uint32_t z,
                                   uint32_t w, bool *fresh)
{
    const uint32_t f = find(A, d, s, z, w);
    *fresh = f == NONE;
    if (f != NONE)
        return f;
    const uint32_t mask = A.mask;
    for (uint32_t i = khome(d, s, z, w) & mask;; i = (i + 1) & mask) {
        uint32_t *pw = slot_w<V6>(A, i);
        const uint32_t cur = __hip_atomic_load(pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur != 0 && cur != CT_TOMBSTONE)
            continue;
        if (atomicCAS(pw, cur, CT_CLAIM) != cur)
            continue;
        put_key(A, i, d, s, z);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // (store order)
        __hip_atomic_store(pw, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return i;
    }
}

__device__ __forceinline__ uint64_t pack(const CtaArgs &A, uint32_t slot, uint32_t order2)
{
    return ((uint64_t)slot << A.ob) | order2;
}

}  // namespace

}  // namespace cfc
