// Device CT apply (cfc_ct_apply_v4): the conntrack writes of one classified
// IPv4 batch, applied in header order to the device CT table in place —
// what __ct_lookup (conntrack.h:221-285), ct_create4 (:691-772) and
// ct_delete4 do to the CT maps while the reference runs the batch one packet
// at a time, restated for a whole batch:
//
//   scan     per header and CT stage: the op (hit, hit + delete, create),
//            the hit's slot; slots whose ops depend on their order (closing
//            bits, RST/FIN, deletes) are marked "ordered"; creates become
//            requests keyed by their home slot
//   insert   requests sorted by (home slot, header order); one thread per
//            home slot dedups the keys, inserts each new one into the table
//            (CAS on the slot's w word), and the first request of a key
//            creates it: its ICMP "related" entry (ct_create4's second
//            write) is a second round of requests
//   route    every op on an ordered slot goes to the ordered list (the
//            scan folded the plain hits into per-slot summaries with
//            atomicOr: on the other slots their result does not depend on
//            order, see k_cta_finish)
//   fold     the ordered list sorted by (slot, header order), one thread per
//            slot replays its ops in order (cfc_api.cpp ct_hit_update /
//            the oracle's ct_apply pass 2)
//   finish   the summaries become the slots' new state
//
// The table stays the truth until the host reads a CT map: every changed
// slot carries CtInfo dirty bits, and cta_collect() compacts them for the
// host mirror (cfc_api.cpp ct_sync).  ICMP entries ct_create4 writes into a
// TCP map are not in the device table (no lookup reaches them, flatten.cpp
// build_ct): they go to a log the host replays in order.
#include <hipcub/hipcub.hpp>

#include "ctops.hpp"

namespace cfc {

namespace {

// ---- scan: ops, hit slots, ordered marks, create requests.  Four headers
// per thread and step, each phase's loads for all four issued before any is
// waited for: the inputs, then the destination endpoints (the pass is a
// chain of dependent loads per header; one header per thread and step left
// it waiting on one chain at a time).  A slot is ordered by a delete or a
// RST/FIN (ACTION_CLOSE) among its ops, never by the entry's own closing
// bits: k_cta_finish resolves those without a load here (see there).
// TWO: the mode has two CT stages per header (egress); else only stage 0
// exists and the odd hit-slot entries are never read (k_cta_route).
#ifndef CFC_SCAN_U
#define CFC_SCAN_U 4   // headers per scan thread and step (A/B builds)
#endif
constexpr int SCAN_U = CFC_SCAN_U;
// staged create requests per block (24 KiB at four headers per thread)
constexpr uint32_t SCAN_STAGE = 256 * SCAN_U * 2 + 1024;   // (a step's worst case fits)
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_cta_scan(CtaArgs A)
{
    constexpr int NST = TWO ? 2 : 1;
    __shared__ uint64_t s_req[SCAN_STAGE];
    __shared__ uint32_t s_nreq;
    if (threadIdx.x == 0)
        s_nreq = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * 256 * SCAN_U;
    uint32_t nhit = 0, nfh = 0, nrb = 0;
    for (uint64_t base = (uint64_t)blockIdx.x * 256 * SCAN_U; base < A.n; base += stride) {
        // SCAN_U consecutive headers per thread: with the batch's arrays
        // 16-byte aligned (A.vec) their words in one 16-byte load per array
        // (four bytes for the byte arrays) — a scalar load moves 4 bytes per
        // lane, and the pass was bound by the load instructions
        const uint64_t i0 = base + (uint64_t)SCAN_U * threadIdx.x;
        ScanIn<V6> r[SCAN_U];
        if (SCAN_U == 4 && A.vec && i0 + SCAN_U <= A.n) {
            const uint4 pt4 = *reinterpret_cast<const uint4 *>(A.pt + i0);
            const uint4 mt4 = *reinterpret_cast<const uint4 *>(A.mt + i0);
            const uint4 ve4 = *reinterpret_cast<const uint4 *>(A.ver + i0);
            const uint4 id4 = *reinterpret_cast<const uint4 *>(A.ident + i0);
            const uint4 k14 = A.ck1 ? *reinterpret_cast<const uint4 *>(A.ck1 + i0)
                                    : make_uint4(NONE, NONE, NONE, NONE);
            const uint4 k24 = A.ck2 ? *reinterpret_cast<const uint4 *>(A.ck2 + i0)
                                    : make_uint4(NONE, NONE, NONE, NONE);
            const uint32_t cb4 = *reinterpret_cast<const uint32_t *>(A.ctb + i0);
            const uint32_t tf4 = A.tf ? *reinterpret_cast<const uint32_t *>(A.tf + i0) : 0u;
            const uint32_t ptv[4] = {pt4.x, pt4.y, pt4.z, pt4.w};
            const uint32_t mtv[4] = {mt4.x, mt4.y, mt4.z, mt4.w};
            const uint32_t vev[4] = {ve4.x, ve4.y, ve4.z, ve4.w};
            const uint32_t idv[4] = {id4.x, id4.y, id4.z, id4.w};
            const uint32_t k1v[4] = {k14.x, k14.y, k14.z, k14.w};
            const uint32_t k2v[4] = {k24.x, k24.y, k24.z, k24.w};
            if constexpr (V6) {
#pragma unroll
                for (int u = 0; u < SCAN_U; u++) {
                    r[u].sa = ld_addr<V6>(A.sa, i0 + u);
                    r[u].da = ld_addr<V6>(A.da, i0 + u);
                }
            } else {
                const uint4 sa4 = *reinterpret_cast<const uint4 *>(A.sa + i0);
                const uint4 da4 = *reinterpret_cast<const uint4 *>(A.da + i0);
                const uint32_t sav[4] = {sa4.x, sa4.y, sa4.z, sa4.w};
                const uint32_t dav[4] = {da4.x, da4.y, da4.z, da4.w};
#pragma unroll
                for (int u = 0; u < SCAN_U; u++) {
                    r[u].sa = sav[u];
                    r[u].da = dav[u];
                }
            }
#pragma unroll
            for (int u = 0; u < SCAN_U; u++) {
                r[u].svcop = false;
                r[u].cb = (cb4 >> (8 * u)) & 0xFFu;
                r[u].pt = ptv[u];
                r[u].mt = mtv[u];
                r[u].ver = vev[u];
                r[u].ident = idv[u];
                r[u].tf = (tf4 >> (8 * u)) & 0xFFu;
                r[u].k1 = k1v[u];
                r[u].k2 = k2v[u];
            }
        } else {
#pragma unroll
            for (int u = 0; u < SCAN_U; u++) {   // inputs (no branches)
                const uint64_t i = i0 + u;
                const uint64_t j = i < A.n ? i : A.n - 1;
                load_in<V6, false>(A, j, r[u]);
                r[u].k1 = A.ck1 ? A.ck1[j] : NONE;
                r[u].k2 = A.ck2 ? A.ck2[j] : NONE;
                if (i >= A.n)
                    r[u].cb = 0;
            }
        }
        // the destination endpoint's CT owner, for the stages whose key the
        // scan builds (a create, a hit the classify launch did not leave):
        // first probes together.  A hit with the launch's slot needs none
        // (most of a conntrack batch: no endpoint lookup per header).
        uint32_t dsto[SCAN_U];
        bool need[SCAN_U];
#pragma unroll
        for (int u = 0; u < SCAN_U; u++) {
            need[u] = false;
#pragma unroll
            for (int st = 0; st < NST; st++) {
                const uint32_t cs = (r[u].cb >> (4 * st)) & 0xF;
                const bool mine = A.mode == CFC_MODE_EGRESS && st == 0;   // (owner: the sender)
                const uint32_t key = st ? r[u].k2 : r[u].k1;
                // (a CT_NEW stage without a create — dropped — has no op)
                const bool cr = (cs & CFC_CT_RES_MASK) == 0;
                need[u] |= (cs & CFC_CT_DONE) && !mine &&
                           (cr ? (cs & CFC_CT_CREATE) != 0 : key >= CK_MISS);
            }
        }
        if constexpr (V6) {
#pragma unroll
            for (int u = 0; u < SCAN_U; u++)
                dsto[u] = need[u] ? dst_owner(A.T, r[u].da) : 0u;
        } else {
            uint32_t ls[SCAN_U];
            uint4 lv[SCAN_U];
#pragma unroll
            for (int u = 0; u < SCAN_U; u++) {
                ls[u] = A.T.lxc4 ? hash32(r[u].da, A.T.lxc4_mask) : 0u;
                lv[u] = (A.T.lxc4 && need[u]) ? ld16(A.T.lxc4 + ls[u]) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < SCAN_U; u++) {
                dsto[u] = 0;
                if (A.T.lxc4 && need[u]) {
                    uint32_t sl = ls[u];
                    uint4 v = lv[u];
                    for (;;) {
                        if (!(v.w & LXC_VALID))
                            break;
                        if (v.x == r[u].da) {
                            dsto[u] = ct_owner_word(v.w & 0xFFFF, (v.w & LXC_CT_LOCAL) != 0);
                            break;
                        }
                        sl = (sl + 1) & A.T.lxc4_mask;
                        v = ld16(A.T.lxc4 + sl);
                    }
                }
            }
        }
        // per stage: the op, its slot, a create's request, a plain hit's
        // summary bits
        uint32_t slot[SCAN_U][2], kind[SCAN_U][2], act[SCAN_U][2], home[SCAN_U][2];
        uint32_t sb[SCAN_U][2];
        bool fh[SCAN_U][2];
        uint32_t ncr = 0;
#pragma unroll
        for (int u = 0; u < SCAN_U; u++) {
#pragma unroll
            for (int st = 0; st < NST; st++) {
                const Op<V6> o = decode_from<V6, false>(A, r[u], st, dsto[u]);
                kind[u][st] = o.kind;
                act[u][st] = o.kind == OP_NONE ? 0u : o.action;
                slot[u][st] = HS_NONE;
                home[u][st] = 0;
                fh[u][st] = false;
                sb[u][st] = (o.kind == OP_HIT && o.action != 2)
                                ? sum_bits(o.dir == CT_INGRESS, o.is_tcp, o.syn, o.tfl) : 0u;
                if (o.kind == OP_HIT || o.kind == OP_DELETE) {
                    const uint32_t key = st ? r[u].k2 : r[u].k1;
                    const bool rev = ((r[u].cb >> (4 * st)) & CFC_CT_RES_MASK) >= 2;
                    uint32_t sl;
                    if (key < CK_MISS) {   // the slot the classify launch hit (else NONE or a miss tag)
                        sl = (key >> 1) - A.acct_base;
                    } else {
                        sl = rev ? find(A, o.da, o.sa, o.z1, o.w1)
                                 : find(A, o.sa, o.da, o.z2, o.w2);
                    }
                    slot[u][st] = sl == NONE ? HS_NONE : sl;
                    if (sl == NONE) {
                        // a hit on an entry an earlier header of this batch
                        // creates (ctorder.hip): a request, resolved after
                        // the inserts and replayed in the fold
                        fh[u][st] = true;
                        home[u][st] = (rev ? khome(o.da, o.sa, o.z1, o.w1)
                                           : khome(o.sa, o.da, o.z2, o.w2)) & A.mask;
                        ncr++;
                    }
                } else if (o.kind == OP_CREATE) {
                    home[u][st] = khome(o.sa, o.da, o.z2, o.w2) & A.mask;
                    ncr++;
                    nrb += !o.is_tcp && !o.ki_form;
                }
            }
        }
        // the plain hits' slot words, loaded together
        uint32_t cur[SCAN_U][2];
#pragma unroll
        for (int u = 0; u < SCAN_U; u++)
#pragma unroll
            for (int st = 0; st < NST; st++)
                cur[u][st] = (sb[u][st] && slot[u][st] != HS_NONE && !A.nt && !A.sum)
                                 ? A.ms[slot[u][st]].x : 0u;
#pragma unroll
        for (int u = 0; u < SCAN_U; u++) {
            const uint64_t i = i0 + u;
#pragma unroll
            for (int st = 0; st < NST; st++) {
                const uint32_t sl = slot[u][st];
                if (sl == HS_NONE)
                    continue;
                nhit++;
                if (A.nt && kind[u][st] == OP_HIT) {
                    // monitor lengths wanted: every hit replayed in order
                    order_mark(A, sl, MARK_ORDERED);
                } else if (sb[u][st]) {   // a plain hit: into the slot's summary
                    // (unless the launch's accounting summarised it: A.sum)
                    if (!A.sum && (cur[u][st] | sb[u][st]) != cur[u][st])
                        atomicOr(&A.ms[sl].x, sb[u][st]);
                } else if (kind[u][st] == OP_DELETE) {
                    // the entry goes: only its first delete matters
                    // (k_cta_route), unless a create revives the key (a
                    // dropped hot flow deletes its entry once per packet:
                    // only a lower order than the one stored needs the
                    // atomic)
                    order_mark(A, sl, MARK_ORDERED | MARK_DEL);
                    const uint32_t v = 0xFFFFFFFFu - ord_of(i, st, SEC_OP);
                    if (__hip_atomic_load(&A.ms[sl].y, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT) < v)
                        atomicMax(&A.ms[sl].y, v);
                } else if (act[u][st] == 2) {   // RST / FIN: ACTION_CLOSE
                    order_mark(A, sl, MARK_ORDERED);
                }
            }
            if (i < A.n) {
                if (TWO)
                    *reinterpret_cast<uint2 *>(A.hs + 2 * i) = make_uint2(slot[u][0], slot[u][1]);
                else
                    A.hs[i] = slot[u][0];   // (one stage: one word per header)
            }
        }
        // the creates' requests: staged in LDS, the block's list taken from
        // reqA by one atomic when the stage fills and at the end (one
        // atomic per block step on the shared counter serialised there)
        uint32_t rq = block_stage_n(&s_nreq, ncr);
#pragma unroll
        for (int u = 0; u < SCAN_U; u++) {
            const uint64_t i = i0 + u;
#pragma unroll
            for (int st = 0; st < NST; st++) {
                if (fh[u][st]) {
                    s_req[rq++] = pack(A, home[u][st], ord_of(i, st, SEC_FHIT));
                    nfh++;
                    continue;
                }
                if (kind[u][st] != OP_CREATE)
                    continue;
                s_req[rq++] = pack(A, home[u][st], ord_of(i, st, SEC_OP));
            }
        }
        __syncthreads();
        if (s_nreq > SCAN_STAGE - 256 * SCAN_U * NST)   // (uniform)
            block_flush(s_req, &s_nreq, &A.cnt[CTA_NREQA], A.reqA, A.req_cap);
    }
    block_flush(s_req, &s_nreq, &A.cnt[CTA_NREQA], A.reqA, A.req_cap);
    block_add(&A.cnt[CTA_NHIT], nhit);
    block_add(&A.cnt[CTA_NFHIT], nfh);
    block_add(&A.cnt[CTA_NRELB], nrb);
}

// ---- the scan over the classify launch's work bits (A.sparse: A.W, the
// headers with a stage that is not a plain hit on a launch slot,
// kern_common.hpp wl_want).  Every other stage is a plain hit whose summary
// the launch's accounting took (A.sum) and whose slot route reads from the
// launch's keys (A.ck1 / A.ck2), so nothing of it is left to do here.  Per
// work header the dense scan's per-stage work; a hit this scan finds a slot
// for (a key the launch left as a tag) has its slot written into the key
// array for route.  One thread per word of 64 headers; the requests staged
// in LDS, the block's list taken from reqA by one atomic.
constexpr uint32_t SCANW_STAGE = 4096;
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_cta_scan_w(CtaArgs A)
{
    constexpr int NST = TWO ? 2 : 1;
    __shared__ uint64_t s_req[SCANW_STAGE];
    __shared__ uint32_t s_n, s_base;
    if (threadIdx.x == 0)
        s_n = 0;
    __syncthreads();
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t nfh = 0, nrb = 0;
    auto put = [&](uint64_t v) {
        const uint32_t q = atomicAdd(&s_n, 1u);
        if (q < SCANW_STAGE) {
            s_req[q] = v;
        } else {   // (a full stage: straight into the list)
            const uint32_t r = atomicAdd(&A.cnt[CTA_NREQA], 1u);
            if (r < A.req_cap)
                A.reqA[r] = v;
        }
    };
    auto one = [&](uint64_t i) {
        ScanIn<V6> r;
        load_in<V6, false>(A, i, r);
        r.k1 = A.ck1[i];
        r.k2 = TWO ? A.ck2[i] : NONE;
        bool need = false;
#pragma unroll
        for (int st = 0; st < NST; st++) {
            const uint32_t cs = (r.cb >> (4 * st)) & 0xF;
            const bool mine = A.mode == CFC_MODE_EGRESS && st == 0;
            const uint32_t key = st ? r.k2 : r.k1;
            const bool cr = (cs & CFC_CT_RES_MASK) == 0;
            need |= (cs & CFC_CT_DONE) && !mine &&
                    (cr ? (cs & CFC_CT_CREATE) != 0 : key >= CK_MISS);
        }
        const uint32_t dsto = need ? dst_owner(A.T, r.da) : 0u;
#pragma unroll
        for (int st = 0; st < NST; st++) {
            const Op<V6> o = decode_from<V6, false>(A, r, st, dsto);
            if (o.kind == OP_HIT || o.kind == OP_DELETE) {
                const uint32_t key = st ? r.k2 : r.k1;
                const bool rev = ((r.cb >> (4 * st)) & CFC_CT_RES_MASK) >= 2;
                uint32_t sl;
                if (key < CK_MISS) {
                    sl = (key >> 1) - A.acct_base;
                } else {
                    sl = rev ? find(A, o.da, o.sa, o.z1, o.w1) : find(A, o.sa, o.da, o.z2, o.w2);
                    if (sl != NONE)   // (route reads the slot from the key array)
                        const_cast<uint32_t *>(st ? A.ck2 : A.ck1)[i] =
                            ct_acct_key(sl + A.acct_base, (int)o.dir);
                }
                if (sl == NONE) {   // a hit on an entry an earlier header creates
                    const uint32_t home = (rev ? khome(o.da, o.sa, o.z1, o.w1)
                                               : khome(o.sa, o.da, o.z2, o.w2)) & A.mask;
                    put(pack(A, home, ord_of(i, st, SEC_FHIT)));
                    if constexpr (!V6)
                        if (A.rk4)
                            A.rk4[TWO ? 2 * i + st : i] =
                                rev ? make_uint4(o.da, o.sa, o.z1, o.w1)
                                    : make_uint4(o.sa, o.da, o.z2, o.w2);
                    nfh++;
                } else if (o.kind == OP_DELETE) {
                    order_mark(A, sl, MARK_ORDERED | MARK_DEL);
                    const uint32_t v = 0xFFFFFFFFu - ord_of(i, st, SEC_OP);
                    if (__hip_atomic_load(&A.ms[sl].y, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT) < v)
                        atomicMax(&A.ms[sl].y, v);
                } else if (o.action == 2) {   // RST / FIN: ACTION_CLOSE
                    order_mark(A, sl, MARK_ORDERED);
                }
            } else if (o.kind == OP_CREATE) {
                put(pack(A, khome(o.sa, o.da, o.z2, o.w2) & A.mask, ord_of(i, st, SEC_OP)));
                nrb += !o.is_tcp && !o.ki_form;
                if constexpr (!V6)
                    if (A.rk4)
                        A.rk4[TWO ? 2 * i + st : i] = make_uint4(o.sa, o.da, o.z2, o.w2);
                if (!o.is_tcp && !o.ki_form) {
                    // its related entry (ct_create4/6's second write) may
                    // overwrite a live one: route runs before the inserts
                    // here, so that slot is marked now, and its hits go to
                    // the fold in order with the overwrite (every other slot
                    // an insert writes is new: the launch saw no hit on it)
                    const uint32_t rw =
                        ct_word(icmp_proto<V6>(), ((o.w2 >> 8) & 7) | 2u, o.owner);
                    const uint32_t rs = find(A, o.sa, o.da, 0u, rw);
                    if (rs != NONE)
                        order_mark(A, rs, MARK_ORDERED | MARK_PUTC);
                }
            }
        }
    };
    if (A.wl) {   // (the list: a lane per work header, grid-stride)
        const uint32_t nl = *A.nwl;
        for (uint64_t x = t; x < nl; x += (uint64_t)gridDim.x * 256)
            one(A.wl[x]);
    } else {
        for (uint64_t m = t < A.W.words ? A.W.bits[t] : 0; m; m &= m - 1)
            one(64 * t + (uint64_t)(__ffsll((long long)m) - 1));
    }
    __syncthreads();
    const uint32_t ns = min(s_n, SCANW_STAGE);
    if (threadIdx.x == 0)
        s_base = ns ? atomicAdd(&A.cnt[CTA_NREQA], ns) : 0u;
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < ns; q += 256)
        if (s_base + q < A.req_cap)
            A.reqA[s_base + q] = s_req[q];
    block_add(&A.cnt[CTA_NFHIT], nfh);
    block_add(&A.cnt[CTA_NRELB], nrb);
}

// the hit slots of a sparse scan's batch for the eviction's protect pass
// (hs, as the dense scan leaves them): from the launch's keys
__global__ __launch_bounds__(256) void k_cta_hs_fill(CtaArgs A)
{
    const bool two = A.mode == CFC_MODE_EGRESS;
    const uint64_t nk = two ? 2 * A.n : A.n;
    const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= nk)
        return;
    const uint64_t i = two ? k >> 1 : k;
    const uint32_t key = (two && (k & 1)) ? A.ck2[i] : A.ck1[i];
    A.hs[k] = key < CK_MISS ? (key >> 1) - A.acct_base : HS_NONE;
}

// ---- the service step of an egress batch with a load balancer.  The
// reference runs lb4_local / lb6_local packet by packet, so a header finds
// the CT_SERVICE entry as the headers before it left it (created, its slave
// re-selected).  k_cta_lb runs the step for every header against the
// batch's starting table; k_cta_svc replays, per CT_SERVICE key, the headers
// after the first one in order with the entry as it then is; the scan takes
// the records (LbRec4 / LbRec6).

// the CT_SERVICE entry as a header finds it
struct SvcState {
    bool exists;
    uint32_t slave, loop;
};

// lb4_local (lb.h:590-776) for header i, given the entry's state (left as
// the header leaves it), then the egress reply's reverse NAT (bpf_lxc.c:
// 565-576, lb4_rev_nat) against the batch's starting table; svc: the
// entry's slot at the batch's start
__device__ void lb_step(const CtaArgs &A, uint64_t i, uint32_t svc, SvcState &st, LbRec4 &o)
{
    const DevTables &T = A.T;
    const uint32_t sa = A.sa[i], da = A.da[i], pt = A.pt[i], proto = A.mt[i] & 0xFF;
    const bool l4 = proto == 6 || proto == 17;
    o = LbRec4{da, sa, da, pt, pt, 0u, 0u, 0u, svc, 0u, 0u};
    uint32_t kd = l4 ? pt >> 16 : 0u;
    uint4 a, b;
    if (T.lb4 && (l4 || proto == 1) && lb4_service(T, da, kd, 0, a, b)) {
        const uint32_t hash = A.hash ? A.hash[i] : flow_hash4(sa, da, pt, proto);
        // a hit's slave and loopback from the entry, else lb4_select_slave
        uint32_t slave = st.exists ? st.slave : hash % (a.w >> 16) + 1;
        uint32_t loop = st.exists ? st.loop : 0u;
        const uint32_t slave0 = slave;
        uint4 c, d;
        bool ok = lb4_get(T, da, kd, slave, c, d), reslave = false;   // lb4_lookup_slave
        if (!ok) {   // the fall-back: the key as it stands, slave set
            ok = lb4_service(T, da, kd, slave, c, d);
            if (ok) {
                slave = hash % (c.w >> 16) + 1;
                reslave = true;
            }
        }
        o.fl = LBF_SVC | (ok ? 0u : LBF_DROP) | (reslave ? LBR_RESLAVE : 0u);
        if (ok) {
            const uint32_t target = c.z, port = c.w & 0xFFFF;
            o.addr = target;
            if (sa == target) {   // loopback (lb.h:753-767)
                loop = 1;
                o.addr = IPV4_LOOPBACK;
                o.sva = sa;
                o.psa = IPV4_LOOPBACK;
            }
            if (loop)
                o.fl |= LBF_LOOP;
            else
                o.tda = target;
            o.pda = target;
            if (port && kd != port && l4)   // lb4_xlate's L4 dport
                o.ppt = (o.ppt & 0xFFFFu) | port << 16;
            o.tpt = o.ppt;
            o.lbw = (d.x & 0xFFFF) | loop << 16;
        }
        o.slv = (slave & 0xFFFF) | slave0 << 16;
        if (!st.exists)
            st.loop = 0;
        st.exists = true;
        st.slave = slave;
    }
    if (!(o.fl & LBF_DROP) && T.ct4_lb && (l4 || proto == 1)) {
        const CtProbe k = ct_probe<false>(proto, o.tpt, CT_EGRESS, A.ep_owner);
        const uint32_t s1 = ct4_find(T, o.tda, sa, k.z1, k.w1);
        if (s1 != NONE)
            lb4_rev_nat(T, ld16(T.ct4_lb + s1), proto, o.psa, o.pda, o.ppt);
    }
}
// lb6_local (lb.h:427-481, no loopback case), then the egress reply's
// lb6_rev_nat
__device__ void lb_step(const CtaArgs &A, uint64_t i, uint32_t svc, SvcState &st, LbRec6 &o)
{
    const DevTables &T = A.T;
    const uint4 sa = ld_addr<true>(A.sa, i), da = ld_addr<true>(A.da, i);
    const uint32_t pt = A.pt[i], proto = A.mt[i] & 0xFF;
    const bool l4 = proto == 6 || proto == 17;
    o.tda = o.pda = da;
    o.psa = sa;
    o.tpt = o.ppt = pt;
    o.fl = o.lbw = o.slv = o.addr = o.sva = 0;
    o.svc = svc;
    uint32_t kd = l4 ? pt >> 16 : 0u;
    uint4 b, tg;
    if (T.lb6 && (l4 || proto == 58) && lb6_service(T, da, kd, 0, b, tg)) {
        const uint32_t hash = A.hash ? A.hash[i] : flow_hash6(sa, da, pt, proto);
        uint32_t slave = st.exists ? st.slave : hash % (b.y >> 16) + 1;   // lb6_select_slave
        const uint32_t slave0 = slave;
        uint4 b2, tg2;
        bool ok = lb6_get(T, da, kd, slave, b2, tg2), reslave = false;
        if (!ok) {
            ok = lb6_service(T, da, kd, slave, b2, tg2);
            if (ok) {
                slave = hash % (b2.y >> 16) + 1;
                reslave = true;
            }
        }
        o.fl = LBF_SVC | (ok ? 0u : LBF_DROP) | (reslave ? LBR_RESLAVE : 0u);
        if (ok) {
            o.tda = o.pda = tg2;   // lb6_xlate
            const uint32_t port = b2.y & 0xFFFF;
            if (port && kd != port && l4)
                o.ppt = (o.ppt & 0xFFFFu) | port << 16;
            o.tpt = o.ppt;
            o.lbw = b2.z & 0xFFFF;
        }
        o.slv = (slave & 0xFFFF) | slave0 << 16;
        st.exists = true;
        st.slave = slave;
        st.loop = 0;
    }
    if (!(o.fl & LBF_DROP) && T.ct6_lb && (l4 || proto == 58)) {
        const CtProbe k = ct_probe<true>(proto, o.tpt, CT_EGRESS, A.ep_owner);
        const uint32_t s1 = ct6_find(T, o.tda, sa, k.z1, k.w1);
        if (s1 != NONE)
            lb6_rev_nat(T, ld16(T.ct6_lb + s1).x, proto, o.psa, o.ppt);
    }
}

// the CT_SERVICE key of header i: the tuple as loaded, TUPLE_F_SERVICE
template <bool V6>
__device__ __forceinline__ void svc_key(const CtaArgs &A, uint64_t i, Addr<V6> &d, Addr<V6> &s,
                                        uint32_t &z, uint32_t &w)
{
    const CtProbe k = ct_probe<V6>(A.mt[i] & 0xFF, A.pt[i], CT_SERVICE, A.ep_owner);
    d = ld_addr<V6>(A.da, i);
    s = ld_addr<V6>(A.sa, i);
    z = k.z1;
    w = k.w1;
}

// one thread per header: its service step against the starting table, and
// a request for its CT_SERVICE op when the reference reaches lb4_local /
// lb6_local with it (the header reached a CT stage, or lb4_local dropped it)
template <bool V6>
__global__ __launch_bounds__(256) void k_cta_lb(CtaArgs A)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    bool want = false;
    uint32_t home = 0;
    if (i < A.n) {
        const uint32_t proto = A.mt[i] & 0xFF;
        uint32_t svc = NONE;
        SvcState st{false, 0u, 0u};
        Addr<V6> d, s;
        uint32_t z, w;
        svc_key<V6>(A, i, d, s, z, w);
        if (proto == 6 || proto == 17 || proto == icmp_proto<V6>()) {
            svc = find(A, d, s, z, w);
            if (svc != NONE && A.lb) {
                const uint4 lw = A.lb[svc];
                st = SvcState{true, lw.y, V6 ? 0u : (lw.x >> 16) & 1};
            } else if (svc != NONE) {
                st = SvcState{true, 0u, 0u};
            }
        }
        LbRecT<V6> o;
        lb_step(A, i, svc, st, o);
        reinterpret_cast<LbRecT<V6> *>(A.lbr)[i] = o;
        want = (o.fl & LBF_SVC) && ((A.ctb[i] & CFC_CT_DONE) || A.ver[i] == DROP_NO_SERVICE);
        home = khome(d, s, z, w) & A.mask;
    }
    const uint32_t r = block_count(&A.cnt[CTA_NSVC], want);
    if (want)
        A.reqS[r] = pack(A, home, ord_of(A.n + i, 0, SEC_OP));
}

// one thread per home slot of the sorted CT_SERVICE requests: per key, the
// headers after its first in header order, each with the entry as the one
// before it left it
template <bool V6>
__global__ __launch_bounds__(256) void k_cta_svc(CtaArgs A, uint64_t *req, uint32_t nreq)
{
    const uint32_t r0 = blockIdx.x * 256 + threadIdx.x;
    if (r0 >= nreq)
        return;
    const uint64_t home = req[r0] >> A.ob;
    if (r0 > 0 && (req[r0 - 1] >> A.ob) == home)
        return;
    const uint64_t omask = (1ull << A.ob) - 1;
    LbRecT<V6> *L = reinterpret_cast<LbRecT<V6> *>(A.lbr);
    for (uint32_t r = r0; r < nreq && (req[r] >> A.ob) == home; r++) {
        if (req[r] & 1)   // (a later header of a key done before)
            continue;
        const uint64_t i = ord_hdr((uint32_t)(req[r] & omask)) - A.n;
        Addr<V6> d, s;
        uint32_t z, w;
        svc_key<V6>(A, i, d, s, z, w);
        // the entry as header i leaves it: created or hit, its slave the
        // selection (or the re-selection)
        const LbRecT<V6> l = L[i];
        SvcState st{true, l.slv & 0xFFFF, 0u};
        if constexpr (!V6)
            st.loop = (l.svc != NONE && A.lb) ? (A.lb[l.svc].x >> 16) & 1 : 0u;
        for (uint32_t q = r + 1; q < nreq && (req[q] >> A.ob) == home; q++) {
            if (req[q] & 1)
                continue;
            const uint64_t iq = ord_hdr((uint32_t)(req[q] & omask)) - A.n;
            Addr<V6> dq, sq;
            uint32_t zq, wq;
            svc_key<V6>(A, iq, dq, sq, zq, wq);
            if (zq != z || wq != w || !aeq(dq, d) || !aeq(sq, s))
                continue;
            req[q] |= 1ull;
            LbRecT<V6> o;
            lb_step(A, iq, l.svc, st, o);
            L[iq] = o;
        }
    }
}

// ---- scan with a load balancer: one header per thread, its CT_SERVICE op
// (hit slot, or a create request of virtual header n + i) and its stages
// with the service step's tuples.  A stage hit on a key the starting table
// lacks is on an entry this batch creates before it (the sender's create,
// found by the destination's lookup): a request, counted in the fold.
template <bool V6>
__global__ __launch_bounds__(256) void k_cta_scan_lb(CtaArgs A)
{
    uint32_t nhit = 0, nfh = 0, nkx = 0, nrb = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t base = (uint64_t)blockIdx.x * 256; base < A.n; base += stride) {
        const uint64_t i = base + threadIdx.x;
        const bool in = i < A.n;
        ScanIn<V6> r;
        load_in<V6, true>(A, in ? i : A.n - 1, r);
        if (!in)
            r.cb = 0;
        const bool any = (r.cb & (CFC_CT_DONE | CFC_CT_DONE << 4)) != 0;
        const uint32_t dsto = any ? dst_owner(A.T, r.pda) : 0u;
        uint32_t hs2[3] = {HS_NONE, HS_NONE, HS_NONE};
        uint64_t rq[3];
        uint32_t ncr = 0;
        for (int st = 0; st < 2; st++) {
            const Op<V6> o = decode_from<V6, true>(A, r, st, dsto);
            if (o.kind == OP_HIT || o.kind == OP_DELETE) {
                const bool rev = ((r.cb >> (4 * st)) & CFC_CT_RES_MASK) >= 2;
                const uint32_t sl = rev ? find(A, o.da, o.sa, o.z1, o.w1)
                                        : find(A, o.sa, o.da, o.z2, o.w2);
                if (sl == NONE) {
                    const uint32_t h = rev ? khome(o.da, o.sa, o.z1, o.w1)
                                           : khome(o.sa, o.da, o.z2, o.w2);
                    rq[ncr++] = pack(A, h & A.mask, ord_of(i, st, SEC_FHIT));
                    nfh++;
                    continue;
                }
                hs2[st] = sl;
                nhit++;
                if (A.nt && o.kind == OP_HIT) {
                    // monitor lengths wanted: every hit replayed in order
                    order_mark(A, sl, MARK_ORDERED);
                } else if (o.kind == OP_HIT && o.action != 2) {   // a plain hit: its summary
                    const uint32_t b = sum_bits(o.dir == CT_INGRESS, o.is_tcp, o.syn, o.tfl);
                    if ((A.ms[sl].x & b) != b)
                        atomicOr(&A.ms[sl].x, b);
                } else if (o.kind == OP_DELETE) {
                    order_mark(A, sl, MARK_ORDERED | MARK_DEL);
                    const uint32_t v = 0xFFFFFFFFu - ord_of(i, st, SEC_OP);
                    if (__hip_atomic_load(&A.ms[sl].y, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT) < v)
                        atomicMax(&A.ms[sl].y, v);
                } else if (o.action == 2) {
                    order_mark(A, sl, MARK_ORDERED);
                }
            } else if (o.kind == OP_CREATE) {
                rq[ncr++] = pack(A, khome(o.sa, o.da, o.z2, o.w2) & A.mask, ord_of(i, st, SEC_OP));
                nkx += o.kx;
                nrb += !o.is_tcp && !o.ki_form;
            }
        }
        if (in && ((r.cb & CFC_CT_DONE) || (int32_t)r.ver == DROP_NO_SERVICE)) {
            ScanIn<V6> rs = r;
            rs.svcop = true;
            const Op<V6> o = decode_from<V6, true>(A, rs, 0, 0u);
            if (o.kind == OP_HIT) {
                hs2[2] = r.svc;   // (its accounting: k_cta_route)
                nhit++;
                if (o.action == 2) {
                    order_mark(A, r.svc, MARK_ORDERED);
                } else {
                    const uint32_t b = sum_bits(false, o.is_tcp, o.syn, o.tfl);
                    if ((A.ms[r.svc].x & b) != b)
                        atomicOr(&A.ms[r.svc].x, b);
                }
                // ct_update4/6_slave: the entry's last re-selection in
                // header order wins (several headers may re-select): the
                // fold replays the slot's ops in order
                if (o.reslave && A.lb)
                    order_mark(A, r.svc, MARK_ORDERED);
            } else if (o.kind == OP_CREATE) {
                rq[ncr++] = pack(A, khome(o.sa, o.da, o.z2, o.w2) & A.mask,
                                 ord_of(A.n + i, 0, SEC_OP));
                nkx += o.kx;   // (k_cta_related's bound: whatever this op writes)
                nrb += !o.is_tcp && !o.ki_form;
            }
        }
        if (in) {
            *reinterpret_cast<uint2 *>(A.hs + 2 * i) = make_uint2(hs2[0], hs2[1]);
            *reinterpret_cast<uint2 *>(A.hs + 2 * (A.n + i)) = make_uint2(hs2[2], HS_NONE);
        }
        const uint32_t q = block_count_n(&A.cnt[CTA_NREQA], ncr);
        for (uint32_t k = 0; k < ncr; k++)
            if (q + k < A.req_cap)
                A.reqA[q + k] = rq[k];
    }
    wave_add(&A.cnt[CTA_NHIT], nhit);
    wave_add(&A.cnt[CTA_NFHIT], nfh);
    wave_add(&A.cnt[CTA_NKX], nkx);
    wave_add(&A.cnt[CTA_NRELB], nrb);
}

// key of a request, by its write: k2 of its op (a create), the ICMP entry
// k2 relates (ports 0, nexthdr ICMP / ICMPv6, flags | TUPLE_F_RELATED), the
// op's reverse-NAT entry, or the key a hit looked up (k1 for REPLY /
// RELATED, else k2)
template <bool V6>
struct ReqKey {
    Addr<V6> d, s;
    uint32_t z, w;
    __device__ __forceinline__ bool operator==(const ReqKey &o) const
    {
        return z == o.z && w == o.w && aeq(d, o.d) && aeq(s, o.s);
    }
};
template <bool V6>
__device__ __forceinline__ ReqKey<V6> req_key(const CtaArgs &A, uint32_t ord, Op<V6> *po)
{
    const uint64_t i = ord_hdr(ord);
    const int st = ord_st(ord);
    *po = decode<V6>(A, i, st);
    const Op<V6> &o = *po;
    ReqKey<V6> k{o.sa, o.da, o.z2, o.w2};
    switch (ord_sec(ord)) {
    case SEC_REL:
        k.z = 0;
        k.w = ct_word(icmp_proto<V6>(), ((o.w2 >> 8) & 7) | 2u, o.owner);
        break;
    case SEC_KX:
        k.d = o.kxa;
        k.s = o.kxs;
        k.w = o.kxw;
        break;
    case SEC_FHIT:
        if (((A.ctb[i] >> (4 * st)) & CFC_CT_RES_MASK) >= 2)
            k = ReqKey<V6>{o.da, o.sa, o.z1, o.w1};
        break;
    default:
        break;
    }
    return k;
}

// a request's key from the scan's record of it (IPv4 sparse scan: creates
// and hits), else decoded
template <bool V6>
__device__ __forceinline__ ReqKey<V6> req_key_of(const CtaArgs &A, uint32_t ord)
{
    if constexpr (!V6) {
        const uint32_t sec = ord_sec(ord);
        if (A.rk4 && (sec == SEC_OP || sec == SEC_FHIT)) {
            const uint64_t i = ord_hdr(ord);
            const uint4 v = ld16(A.rk4 + (A.mode == CFC_MODE_EGRESS ? 2 * i + ord_st(ord) : i));
            return ReqKey<false>{v.x, v.y, v.z, v.w};
        }
    }
    Op<V6> o;
    return req_key<V6>(A, ord, &o);
}

// ---- insert: one thread per home slot; keys deduped in registers (a fifth
// distinct key of one home slot is found by rescanning the run).  A key's
// first create also writes its related ICMP entry and, with a load
// balancer's ct_state, its reverse-NAT entry (round 1): the request is
// marked (bit 0 of its word) and k_cta_related makes those requests — no
// per-request atomic on a shared counter here.
// (1024-thread blocks for the per-request passes: one counter atomic per
// 1024 requests)
constexpr int RQ_B = 1024;
template <bool V6>
__global__ __launch_bounds__(RQ_B) void k_cta_insert(CtaArgs A, uint64_t *req, uint32_t nreq,
                                                    int round, uint32_t cx_off)
{
    const uint32_t r0 = blockIdx.x * RQ_B + threadIdx.x;
    const uint64_t home = r0 < nreq ? req[r0] >> A.ob : 0;
    // (an all-ones request is an unused place of round 1: skipped)
    const bool lead = r0 < nreq && home <= A.mask && (r0 == 0 || (req[r0 - 1] >> A.ob) != home);
    const uint64_t omask = (1ull << A.ob) - 1;
    uint32_t claims = 0;
    if (lead) {
        ReqKey<V6> kk[4];
        uint32_t ks[4];
        int nk = 0;
        for (uint32_t r = r0; r < nreq && (req[r] >> A.ob) == home; r++) {
            const uint32_t ord = (uint32_t)(req[r] & omask) & ~1u;
            const ReqKey<V6> k = req_key_of<V6>(A, ord);
            uint32_t slot = NONE;
            for (int j = 0; j < nk; j++)
                if (kk[j] == k)
                    slot = ks[j];
            bool first = false;
            if (slot == NONE) {
                // not among the first four keys: an earlier request of the
                // run may still have it
                for (uint32_t q = r0; q < r && nk == 4; q++) {
                    if (req_key_of<V6>(A, (uint32_t)(req[q] & omask) & ~1u) == k) {
                        slot = find(A, k.d, k.s, k.z, k.w);
                        break;
                    }
                }
            }
            if (slot == NONE) {
                bool fresh;
                slot = find_or_insert<V6>(A, k.d, k.s, k.z, k.w, &fresh);
                order_mark(A, slot, MARK_ORDERED | MARK_PUTC | (fresh ? MARK_FRESH : 0u));
                first = fresh;
                claims += fresh;
                if (nk < 4) {
                    kk[nk] = k;
                    ks[nk++] = slot;
                }
            }
            // every create and related-entry write is an ordered op: request
            // r of the round has its own place in the list
            const uint32_t c = cx_off + r;
            if (c < A.cx_cap)
                A.cx[c] = pack(A, slot, ord);
            if (round == 0 && first && ord_sec(ord) == SEC_OP)
                req[r] |= 1ull;
        }
    }
    block_add(&A.cnt[CTA_CLAIMS], claims);
}

// first sighting in this batch of a related entry's key: a CAS into the
// fingerprint set (A.cx as 2 * cx_cap words, zeroed by cta_newkeys; mask:
// its largest power of two - 1).  Fingerprints are two independent 32-bit
// key hashes, never 0.
template <class AD>
__device__ __forceinline__ uint32_t rel_first(const CtaArgs &A, AD sa, AD da, uint32_t w)
{
    const uint64_t fp = ((uint64_t)khash(sa, da, 0x5bd1e995u, w) << 32 |
                         khash(da, sa, 0x27d4eb2fu, ~w)) | 1ull;
    const uint32_t mask = A.rel_mask;
    for (uint32_t i = (uint32_t)fp & mask;; i = (i + 1) & mask) {
        const unsigned long long cur =
            atomicCAS((unsigned long long *)A.cx + i, 0ull, (unsigned long long)fp);
        if (cur == 0)
            return 1;
        if (cur == fp)
            return 0;
    }
}

// ---- the keys round 0 and its second writes would add, counted before any
// insert (when the quick bound says the table may fill): per home slot, each
// distinct key the table lacks, and for a create its related and
// reverse-NAT entries
template <bool V6>
__global__ __launch_bounds__(256) void k_cta_newkeys(CtaArgs A, const uint64_t *req, uint32_t nreq)
{
    const uint32_t r0 = blockIdx.x * 256 + threadIdx.x;
    const uint64_t home = r0 < nreq ? req[r0] >> A.ob : 0;
    const bool lead = r0 < nreq && (r0 == 0 || (req[r0 - 1] >> A.ob) != home);
    const uint64_t omask = (1ull << A.ob) - 1;
    uint32_t nk_new = 0, nk_tcp = 0;   // (keys of a TCP create go to a TCP map)
    if (lead) {
        ReqKey<V6> kk[4];
        int nk = 0;
        for (uint32_t r = r0; r < nreq && (req[r] >> A.ob) == home; r++) {
            const uint32_t ord = (uint32_t)(req[r] & omask) & ~1u;
            Op<V6> o;
            const ReqKey<V6> k = req_key<V6>(A, ord, &o);
            bool seen = false;
            for (int j = 0; j < nk; j++)
                seen |= kk[j] == k;
            for (uint32_t q = r0; q < r && nk == 4 && !seen; q++) {
                Op<V6> oq;
                seen = req_key<V6>(A, (uint32_t)(req[q] & omask) & ~1u, &oq) == k;
            }
            if (seen)
                continue;
            if (nk < 4)
                kk[nk++] = k;
            if (find(A, k.d, k.s, k.z, k.w) != NONE)
                continue;
            uint32_t nk = 1u + (ord_sec(ord) == SEC_OP && o.kx ? 1u : 0u);
            if (ord_sec(ord) == SEC_OP && !o.ki_form) {
                // its related ICMP entry: one per address pair and map, which
                // many creates share — counted once per batch (a set of the
                // keys' 64-bit fingerprints in A.cx) and only when the table
                // lacks it (an ANY map's; a TCP map's is host-side only)
                const uint32_t rw = ct_word(icmp_proto<V6>(), ((o.w2 >> 8) & 7) | 2u, o.owner);
                if (o.is_tcp || find(A, o.sa, o.da, 0u, rw) == NONE) {
                    const uint32_t f = rel_first(A, o.sa, o.da, rw);
                    nk += f;
                    if (f && o.is_tcp && A.emrel) {   // (a TCP map's: the host checks it)
                        const uint32_t q = atomicAdd(&A.emcnt[A.n_emaps], 1u);
                        if (q < A.emrel_cap) {
                            if constexpr (V6) {
                                A.emrel[3 * q] = o.sa;
                                A.emrel[3 * q + 1] = o.da;
                            } else {
                                A.emrel[3 * q] = make_uint4(o.sa, 0, 0, 0);
                                A.emrel[3 * q + 1] = make_uint4(o.da, 0, 0, 0);
                            }
                            A.emrel[3 * q + 2] = make_uint4(rw, 0, 0, 0);
                        }
                    }
                }
            }
            nk_new += nk;
            nk_tcp += o.is_tcp ? nk : 0u;
            if (A.emcnt) {   // the map its keys go to: its owner's, by kind
                const uint32_t sel = o.owner | (o.is_tcp ? 0u : 2u);
                for (uint32_t j = 0; j < A.n_emaps; j++)
                    if (A.emaps[j] == sel) {
                        atomicAdd(&A.emcnt[j], nk);
                        break;
                    }
            }
        }
    }
    wave_add(&A.cnt[CTA_NEWK], nk_new);
    wave_add(&A.cnt[CTA_NEWKT], nk_tcp);
}

// ---- related: one thread per (sorted) round-0 request; a marked one is a
// key's first create, whose related ICMP entry goes into the device table
// for an ANY map (UDP, ICMP echo: a round-1 request) or into the host log
// for a TCP map (no lookup reaches it there), and whose reverse-NAT entry
// (ct_create4 with ct_state->addr) is a round-1 request
template <bool V6>
__global__ __launch_bounds__(RQ_B) void k_cta_related(CtaArgs A, const uint64_t *req,
                                                     uint32_t nreq)
{
    const uint32_t r = blockIdx.x * RQ_B + threadIdx.x;
    const uint64_t v = r < nreq ? req[r] : 0ull;
    const uint32_t ord = (uint32_t)(v & ((1ull << A.ob) - 1)) & ~1u;
    Op<V6> o;
    o.is_tcp = false;
    o.ki_form = true;
    o.kx = false;
    if (v & 1)
        o = decode<V6>(A, ord_hdr(ord), ord_st(ord));
    const bool rel = (v & 1) && !o.ki_form;
    const bool lg = rel && o.is_tcp, rb = rel && !o.is_tcp, kx = (v & 1) && o.kx;
    const uint32_t l = block_count(&A.cnt[CTA_NLOG], lg);
    uint32_t b = block_count_n(&A.cnt[CTA_NREQB], (uint32_t)rb + (uint32_t)kx);
    const uint32_t fl = ((o.w2 >> 8) & 7) | 2u;
    const uint32_t dirlen = (o.dir == CT_INGRESS ? 1u << 31 : 0u) |
                            ((A.nat46 && o.dir == CT_EGRESS) ? CTLOG_NAT46 : 0u) |
                            o.len;
    if (lg && l < A.log_cap) {
        if constexpr (V6) {
            CtLog6 &g = A.log6[A.log_base + l];
            g.x = o.sa;
            g.y = o.da;
            g.w = ct_word(icmp_proto<V6>(), fl, o.owner);
            g.now = A.now;
            g.dirlen = dirlen;
            g.sec = o.sec;
            g.seq = A.seq;
            g.order = ord;
            g.rev = o.rev;
            g.slave = o.slave_rel;
        } else {
            CtLog &g = A.log[A.log_base + l];
            g.x = o.sa;
            g.y = o.da;
            g.w = ct_word(icmp_proto<V6>(), fl, o.owner);
            g.now = A.now;
            g.dirlen = dirlen;
            g.sec = o.sec;
            g.seq = A.seq;
            g.order = ord;
            g.lbw = o.lbw;
            g.slave = o.slave_rel;
        }
    }
    if (rb) {
        if (b < A.req_cap) {
            const uint32_t h =
                khome(o.sa, o.da, 0u, ct_word(icmp_proto<V6>(), fl, o.owner)) & A.mask;
            A.reqB[b] = pack(A, h, ord | SEC_REL << 1);
        }
        b++;
    }
    if (kx && b < A.req_cap)
        A.reqB[b] = pack(A, khome(o.kxa, o.kxs, o.z2, o.kxw) & A.mask, ord | SEC_KX << 1);
}

// ---- route: every op on an ordered slot -> the ordered list (the plain
// hits of the other slots are in their summaries: k_cta_scan / the launch's
// accounting).  RU consecutive header stages per thread and step: their
// hit slots in four 16-byte loads, then the ordered-slot bitmap words, the
// slot's words only for the ordered ones.  (Family-free.)
//
// A slot ordered by its closes alone (no create, related write or delete
// among its ops; no monitor lengths wanted) keeps its plain hits out of the
// list too — the TCP / UDP hits of headers without a work bit (wl_want):
// every one of them is ACTION_CREATE on a live entry, so with one clock per
// batch the run of them between two closes acts as its last one, and all of
// them as one hit at the last one's order with the slot's summary (the
// fold's sum_hit; the closes before it only add their flags, which the
// summary's OR already holds).  Route keeps that order per slot (A.lh, a
// max): a hot flow's hits, millions at C5 --stream seq, are one word, not
// millions of sorted ops.  The maxima are taken per workgroup in an LDS
// table first (a hot slot's atomics on one word would serialise).
constexpr int RU = 16;
constexpr uint32_t LH_N = 1024, LH_EMPTY = 0xFFFFFFFFu;
__global__ __launch_bounds__(256) void k_cta_route(CtaArgs A)
{
    __shared__ uint32_t s_lk[LH_N], s_lv[LH_N];
    const bool summ = A.lh && A.W.bits && !A.nt;
    if (summ) {
        for (uint32_t q = threadIdx.x; q < LH_N; q += 256) {
            s_lk[q] = LH_EMPTY;
            s_lv[q] = 0;
        }
        __syncthreads();
    }
    auto lh_put = [&](uint32_t sl, uint32_t v) {
        uint32_t h = (sl * 0x9E3779B1u) >> 22;
        for (int p = 0; p < 8; p++, h = (h + 1) & (LH_N - 1)) {
            uint32_t k = s_lk[h];
            if (k == LH_EMPTY)
                k = atomicCAS(&s_lk[h], LH_EMPTY, sl);
            if (k == LH_EMPTY || k == sl) {
                atomicMax(&s_lv[h], v);
                return;
            }
        }
        atomicMax(&A.lh[sl], v);   // (a full run of the table)
    };
    // item k is header stage j = k (egress: two CT stages per header) or
    // j = 2k (one stage: the odd stages never hold a hit); with a load
    // balancer (egress) j in [2n, 4n) are the CT_SERVICE ops (virtual
    // headers n..2n-1)
    const bool two = A.mode == CFC_MODE_EGRESS;
    const uint64_t n2 = 2 * A.n, nk = A.lbr ? 2 * n2 : two ? n2 : A.n;
    const uint64_t span = 256ull * RU, stride = (uint64_t)gridDim.x * span;
    for (uint64_t base = (uint64_t)blockIdx.x * span; base < nk; base += stride) {
        const uint64_t k0 = base + (uint64_t)RU * threadIdx.x;
        uint32_t slot[RU], bw[RU];
        if (A.sparse) {
            // the hit slots from the launch's keys (a miss tag or NONE: no
            // slot); items k0.. are headers k0 / 2.. with two stages
            uint32_t kv[RU];
            if (k0 + RU <= nk) {   // (16-byte aligned key arrays)
                if (two) {
                    const uint4 *p1 = reinterpret_cast<const uint4 *>(A.ck1 + (k0 >> 1));
                    const uint4 *p2 = reinterpret_cast<const uint4 *>(A.ck2 + (k0 >> 1));
#pragma unroll
                    for (int q = 0; q < RU / 8; q++) {
                        const uint4 a = p1[q], b = p2[q];
                        kv[8 * q] = a.x, kv[8 * q + 1] = b.x;
                        kv[8 * q + 2] = a.y, kv[8 * q + 3] = b.y;
                        kv[8 * q + 4] = a.z, kv[8 * q + 5] = b.z;
                        kv[8 * q + 6] = a.w, kv[8 * q + 7] = b.w;
                    }
                } else {
                    const uint4 *p1 = reinterpret_cast<const uint4 *>(A.ck1 + k0);
#pragma unroll
                    for (int q = 0; q < RU / 4; q++) {
                        const uint4 a = p1[q];
                        kv[4 * q] = a.x, kv[4 * q + 1] = a.y, kv[4 * q + 2] = a.z,
                                 kv[4 * q + 3] = a.w;
                    }
                }
            } else {
#pragma unroll
                for (int u = 0; u < RU; u++) {
                    const uint64_t k = k0 + u;
                    kv[u] = k >= nk ? NONE : two ? ((k & 1) ? A.ck2 : A.ck1)[k >> 1] : A.ck1[k];
                }
            }
#pragma unroll
            for (int u = 0; u < RU; u++)
                slot[u] = kv[u] < CK_MISS ? (kv[u] >> 1) - A.acct_base : HS_NONE;
        } else if (k0 + RU <= nk) {   // (A.hs: 16-byte aligned)
            const uint4 *hp = reinterpret_cast<const uint4 *>(A.hs + k0);
#pragma unroll
            for (int q = 0; q < RU / 4; q++) {
                const uint4 v = hp[q];
                slot[4 * q] = v.x;
                slot[4 * q + 1] = v.y;
                slot[4 * q + 2] = v.z;
                slot[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int u = 0; u < RU; u++)
                slot[u] = k0 + u < nk ? A.hs[k0 + u] : HS_NONE;
        }
#pragma unroll
        for (int u = 0; u < RU; u++)
            bw[u] = slot[u] != HS_NONE ? A.obm[slot[u] >> 5] : 0u;
        if (A.lbr) {
            // a CT_SERVICE hit on the batch's starting table: its
            // CONNTRACK_ACCOUNTING (__ct_lookup counts every hit; the
            // CT_SERVICE lookup's on the tx side), which no classify launch
            // counts — here, after the apply has committed to the device
            // (a scan may run twice when the table grows)
            for (int u = 0; u < RU; u++) {
                const uint64_t k = k0 + u;
                if (k < n2 || slot[u] == HS_NONE)
                    continue;
                unsigned long long *ac =
                    reinterpret_cast<unsigned long long *>(A.st[slot[u]].acct);
                atomicAdd(ac, 1ull);
                atomicAdd(ac + 1, (unsigned long long)(A.mt[(k >> 1) - A.n] >> 16));
            }
        }
        uint32_t om = 0;   // bit u: item k0 + u goes to the ordered list
#pragma unroll
        for (int u = 0; u < RU; u++)
            if (slot[u] != HS_NONE && ((bw[u] >> (slot[u] & 31)) & 1))
                om |= 1u << u;
        for (uint32_t m = om; m; m &= m - 1) {   // (rare: the ordered slots' ops)
            const int u = __ffs(m) - 1;
            const uint64_t j = two ? k0 + u : 2 * (k0 + u);
            const uint2 v = A.ms[slot[u]];
            bool o;
            if ((v.x & (MARK_DEL | MARK_PUTC)) == MARK_DEL && !A.nt) {
                // a deleted entry: its first delete stands for all its ops
                o = ord_of(j >> 1, (int)(j & 1), SEC_OP) == 0xFFFFFFFFu - v.y;
            } else {
                o = (v.x & MARK_ORDERED) != 0;
                const uint64_t i = j >> 1;
                if (o && summ && !(v.x & (MARK_DEL | MARK_PUTC)) && i < A.n &&
                    !((A.W.bits[i >> 6] >> (i & 63)) & 1)) {
                    const uint32_t proto = A.mt[i] & 0xFF;
                    if (proto == 6 || proto == 17) {   // (a plain hit: summarised)
                        lh_put(slot[u], ord_of(i, (int)(j & 1), SEC_OP) + 1);
                        o = false;
                    }
                }
            }
            if (!o)
                om &= ~(1u << u);
        }
        uint32_t c = A.cx_base + block_count_n(&A.cnt[CTA_NCX], (uint32_t)__popc(om));
        for (uint32_t m = om; m; m &= m - 1) {
            const int u = __ffs(m) - 1;
            const uint64_t j = two ? k0 + u : 2 * (k0 + u);
            if (c < A.cx_cap)
                A.cx[c] = pack(A, slot[u], ord_of(j >> 1, (int)(j & 1), SEC_OP));
            c++;
        }
    }
    if (summ) {   // (the workgroup's maxima)
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < LH_N; q += 256)
            if (s_lk[q] != LH_EMPTY && A.lh[s_lk[q]] < s_lv[q])
                atomicMax(&A.lh[s_lk[q]], s_lv[q]);
    }
}

// ---- the entry state machine (cfc_api.cpp ct_upd / ct_upd_timeout /
// ct_hit_update, conntrack.h:125-207, :221-285)
struct St {
    uint32_t last_rx, last_tx, seen_rx, seen_tx, bits, lifetime;
};
__device__ __forceinline__ uint32_t upd(St &e, uint32_t now, uint32_t life, uint32_t dir,
                                        uint32_t flags)
{
    e.lifetime = now + life;
    uint32_t &acc = dir == CT_INGRESS ? e.seen_rx : e.seen_tx;
    uint32_t &last = dir == CT_INGRESS ? e.last_rx : e.last_tx;
    const uint32_t seen = (flags | acc) & 0xFF;
    if (last + CT_REPORT_INTERVAL < now || acc != seen) {
        last = now;
        acc = seen;
        return 1;   // (ct_update_timeout is bool: TRACE_PAYLOAD_LEN becomes 1)
    }
    return 0;
}
__device__ __forceinline__ uint32_t upd_timeout(St &e, uint32_t now, bool is_tcp, uint32_t dir,
                                                bool syn, uint32_t flags)
{
    uint32_t life = CT_LIFETIME_NONTCP;
    if (is_tcp) {
        if (!syn)
            e.bits |= SEEN_NON_SYN;
        life = (e.bits & SEEN_NON_SYN) ? CT_LIFETIME_TCP : CT_SYN_TIMEOUT;
    }
    return upd(e, now, life, dir, flags);
}
// returns *monitor as __ct_lookup leaves it (0; 1: ct_update_timeout's bool;
// TRACE_PAYLOAD_LEN for ACTION_CLOSE)
template <bool V6>
__device__ __forceinline__ uint32_t hit(St &e, uint32_t now, const Op<V6> &o)
{
    auto alive = [&] { return !(e.bits & RX_CLOSING) || !(e.bits & TX_CLOSING); };
    uint32_t m = 0;
    if (alive())
        m = upd_timeout(e, now, o.is_tcp, o.dir, o.syn, o.tfl);
    if (o.action == 1) {
        if (e.bits & (RX_CLOSING | TX_CLOSING)) {
            e.bits &= ~(RX_CLOSING | TX_CLOSING);
            m = upd_timeout(e, now, o.is_tcp, o.dir, o.syn, o.tfl);
        }
    } else if (o.action == 2) {
        e.bits |= o.dir == CT_INGRESS ? RX_CLOSING : TX_CLOSING;
        m = TRACE_PAYLOAD_LEN;
        if (!alive())
            upd(e, now, CT_CLOSE_TIMEOUT, o.dir, o.tfl);
    }
    return m;
}
// a slot summary's plain hits (sum_bits: bit 16 / 17 a hit per direction
// with its flags in bits 0-7 / 8-15, bit 18 a TCP hit without the close bit)
// as one ACTION_CREATE hit on a live entry: the closing bits cleared, the
// timeout re-armed, per direction with hits flags_seen |= theirs and
// last_report = now iff the interval had passed or the flags grew (see
// k_cta_finish)
__device__ __forceinline__ void sum_hit(St &x, uint32_t now, uint32_t mu)
{
    x.bits &= ~(RX_CLOSING | TX_CLOSING);
    const bool is_tcp = (mu & (1u << 18)) != 0;
    if (is_tcp)
        x.bits |= SEEN_NON_SYN;
    x.lifetime = now + (is_tcp ? CT_LIFETIME_TCP : CT_LIFETIME_NONTCP);
    if (mu & (1u << 16)) {
        const uint32_t seen = (x.seen_rx | (mu & 0xFF)) & 0xFF;
        if (x.last_rx + CT_REPORT_INTERVAL < now || seen != x.seen_rx)
            x.last_rx = now;
        x.seen_rx = seen;
    }
    if (mu & (1u << 17)) {
        const uint32_t seen = (x.seen_tx | ((mu >> 8) & 0xFF)) & 0xFF;
        if (x.last_tx + CT_REPORT_INTERVAL < now || seen != x.seen_tx)
            x.last_tx = now;
        x.seen_tx = seen;
    }
}
// ct_create4/6's entry (seen_flags.syn = is_tcp: seen_non_syn stays clear)
__device__ __forceinline__ St fresh(uint32_t now, bool is_tcp, uint32_t dir)
{
    St e{0, 0, 0, 0, 0, 0};
    upd_timeout(e, now, is_tcp, dir, is_tcp, 0);
    return e;
}
__device__ __forceinline__ St load_state(const CtState *st, uint32_t slot)
{
    const uint4 t = ld16(&st[slot].tm);
    St e;
    e.last_rx = t.x;
    e.last_tx = t.y;
    e.seen_rx = t.z & 0xFF;
    e.seen_tx = (t.z >> 8) & 0xFF;
    e.bits = ((t.z >> 16) & 3) | ((t.z & CTT_NON_SYN) ? SEEN_NON_SYN : 0u) |
             ((t.z & CTT_NAT46) ? NAT46 : 0u);
    e.lifetime = t.w;
    return e;
}
__device__ __forceinline__ void store_state(CtState *st, uint32_t slot, const St &e)
{
    uint4 t;
    t.x = e.last_rx;
    t.y = e.last_tx;
    t.z = e.seen_rx | e.seen_tx << 8 | (e.bits & 3) << 16 |
          ((e.bits & SEEN_NON_SYN) ? CTT_NON_SYN : 0u) | ((e.bits & NAT46) ? CTT_NAT46 : 0u);
    t.w = e.lifetime;
    *reinterpret_cast<uint4 *>(&st[slot].tm) = t;
}

// ---- dedup: in the sorted ordered list, a plain hit identical to the op
// before it on the same slot (same direction, action, protocol, close bit
// and TCP flags) changes nothing — with one clock per batch a hit's state
// update is idempotent: hit(hit(e)) = hit(e) — so only the first of each
// such run is replayed.  A hot flow's hits in a Zipf batch become one op.
// (Creates, deletes and related-entry writes are always kept.)
template <bool V6>
__device__ __forceinline__ uint32_t hit_sig(const CtaArgs &A, uint32_t ord)
{
    const uint64_t i = ord_hdr(ord);
    if (ord_sec(ord) != SEC_OP || i >= A.n)
        return 0;   // a create's second write, a counted hit, a CT_SERVICE op
    const int st = ord_st(ord);
    const uint32_t cb = A.ctb[i];
    const uint32_t cs = (cb >> (4 * st)) & 0xF;
    const uint32_t b = cs & CFC_CT_RES_MASK;
    const int last = (cb & (CFC_CT_DONE << 4)) ? 1 : 0;
    const bool dropped = st == last && A.ver[i] == DROP_POLICY;
    if (!(cs & CFC_CT_DONE) || (b == 0) || (b == 1 && dropped))
        return 0;   // not a plain hit
    const uint32_t mt = A.mt[i], proto = mt & 0xFF;
    const uint32_t tfl = (proto == 6 && A.tf) ? A.tf[i] : 0u;
    const uint32_t act = ct_action(V6, proto, A.pt[i], mt);
    return 1u | (uint32_t)st << 1 | act << 2 | (mt & CFC_HF_TCP_CLOSE ? 1u : 0u) << 4 |
           tfl << 8 | proto << 16;
}
// (each op's signature computed once: the block's in LDS, the one before
// the block's first by its first thread)
template <bool V6>
__global__ __launch_bounds__(256) void k_cta_dedup(CtaArgs A, const uint64_t *cx, uint32_t ncx,
                                                   uint8_t *keep)
{
    __shared__ uint32_t ssig[257];
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    const uint64_t omask = (1ull << A.ob) - 1;
    const uint64_t v = r < ncx ? cx[r] : ~0ull, vp = (r > 0 && r <= ncx) ? cx[r - 1] : ~0ull;
    const uint64_t sl = v >> A.ob;
    // a plain hit on a slot this batch does not write: its signature (a
    // written slot keeps every hit: after the write each one counts; and an
    // op with route's summarised hits between it and the one before, order
    // lh - 1, is not a repeat: those hits may have changed the state)
    const uint32_t lh = (sl <= A.mask && A.lh) ? A.lh[(uint32_t)sl] : 0u;
    const bool cand = sl <= A.mask && (vp >> A.ob) == sl && !(A.ms[(uint32_t)sl].x & MARK_PUTC) &&
                      !(lh && (uint32_t)(vp & omask) < lh - 1 && (uint32_t)(v & omask) >= lh);
    const uint32_t mine = sl <= A.mask ? hit_sig<V6>(A, (uint32_t)(v & omask)) : 0u;
    ssig[threadIdx.x + 1] = mine;
    if (threadIdx.x == 0)
        ssig[0] = (cand && (vp >> A.ob) <= A.mask) ? hit_sig<V6>(A, (uint32_t)(vp & omask)) : 0u;
    __syncthreads();
    if (r >= ncx)
        return;
    // (an unused place of round 1 is dropped)
    keep[r] = sl <= A.mask && (!cand || !mine || mine != ssig[threadIdx.x]);
}

// the monitor length of op `ord` (a header's own stage, not a CT_SERVICE op)
__device__ __forceinline__ void put_mon(const CtaArgs &A, uint32_t ord, uint32_t m)
{
    const uint64_t i = ord_hdr(ord);
    if (A.mon && i < A.n)
        A.mon[2 * i + ord_st(ord)] = m == 0 ? 0 : m == 1 ? 1 : 2;
}

// ---- fold: one thread per slot of the sorted ordered list.  A slot with
// more than FOLD_LONG ops (a hot flow of a Zipf batch whose closes or
// deletes ordered it: millions of ops at C5) is left to k_cta_fold_long,
// one workgroup per such slot: its run is listed (long, A.cnt[CTA_NLONG]).
constexpr uint32_t FOLD_LONG = 512;
template <bool V6, bool LB>
__device__ void fold_run(const CtaArgs &A, const uint64_t *cx, uint32_t ncx, uint32_t r0);
template <bool V6, bool LB>
__global__ __launch_bounds__(256) void k_cta_fold(CtaArgs A, const uint64_t *cx,
                                                  const uint32_t *pncx, uint32_t *lng)
{
    const uint32_t ncx = *pncx;   // (the deduplicated list's length)
    const uint32_t r0 = blockIdx.x * 256 + threadIdx.x;
    if (r0 >= ncx)
        return;
    const uint32_t slot = (uint32_t)(cx[r0] >> A.ob);
    if (r0 > 0 && (uint32_t)(cx[r0 - 1] >> A.ob) == slot)
        return;
    if (r0 + FOLD_LONG < ncx && (uint32_t)(cx[r0 + FOLD_LONG] >> A.ob) == slot) {
        lng[atomicAdd(&A.cnt[CTA_NLONG], 1u)] = r0;   // (LongScratch.start)
        return;
    }
    fold_run<V6, LB>(A, cx, ncx, r0);
}

// the slot's ops in order, one thread (the run starts at r0)
template <bool V6, bool LB>
__device__ void fold_run(const CtaArgs &A, const uint64_t *cx, uint32_t ncx, uint32_t r0)
{
    const uint32_t slot = (uint32_t)(cx[r0] >> A.ob);
    const uint64_t omask = (1ull << A.ob) - 1;
    const bool was_fresh = (A.ms[slot].x & MARK_FRESH) != 0;
    bool live = !was_fresh, created = false, deleted = false, reslaved = false;
    St e = was_fresh ? St{0, 0, 0, 0, 0, 0} : load_state(A.st, slot);
    uint64_t acct[4] = {0, 0, 0, 0};   // [tx pk, tx by, rx pk, rx by] added / set
    uint32_t sec = 0, rev = 0, lbx = 0, lby = 0;
    // the next op's header is loaded (branch-free) while this one is
    // replayed; the owner word does not matter here (the slot is the key),
    // so no endpoint lookup
    // (the plain hits route summarised: one hit at the last one's order)
    const uint32_t lh = A.lh ? A.lh[slot] : 0u;
    const uint32_t mu = lh ? (A.sum ? A.sum[slot] : A.ms[slot].x >> SUM_SH) : 0u;
    bool summed = lh == 0;
    ScanIn<V6> cur;
    load_in<V6, LB, false>(A, ord_hdr((uint32_t)(cx[r0] & omask)), cur);
    for (uint32_t r = r0; r < ncx && (uint32_t)(cx[r] >> A.ob) == slot; r++) {
        const uint32_t ord = (uint32_t)(cx[r] & omask);
        if (!summed && ord >= lh) {   // (past the last summarised hit, ord lh - 1)
            if (live)
                sum_hit(e, A.now, mu);
            summed = true;
        }
        ScanIn<V6> nxt;
        load_in<V6, LB, false>(A, ord_hdr((uint32_t)(cx[r + 1 < ncx ? r + 1 : r] & omask)), nxt);
        const Op<V6> o = decode_from<V6, LB>(A, cur, ord_st(ord), 0u);
        cur = nxt;
        const uint32_t d = o.dir == CT_INGRESS ? 2 : 0;
        const uint32_t wr = ord_sec(ord);
        if (wr == SEC_REL || wr == SEC_KX) {
            // ct_create's related-entry (or reverse-NAT entry) write: overwrite
            e = fresh(A.now, o.is_tcp, o.dir);
            if (wr == SEC_REL)
                e.bits |= SEEN_NON_SYN;
            if (A.nat46 && o.dir == CT_EGRESS)   // a NAT64 hop's create (conntrack.h:714-716)
                e.bits |= NAT46;
            live = created = true;
            acct[0] = acct[1] = acct[2] = acct[3] = 0;
            acct[d] = 1;
            acct[d + 1] = o.len;
            sec = o.sec;
            rev = o.rev;
            lbx = o.lbw;
            lby = wr == SEC_REL ? o.slave_rel : o.slave;
        } else if (wr == SEC_FHIT) {   // a hit the classify launch could not count
            if (live) {
                put_mon(A, ord, hit(e, A.now, o));
                acct[d] += 1;
                acct[d + 1] += o.len;
                if (o.kind == OP_DELETE) {   // (an entry this batch created)
                    live = false;
                    deleted = true;
                }
            }
        } else if (o.kind == OP_CREATE) {
            if (live) {   // created earlier in this batch: a counted hit
                put_mon(A, ord, hit(e, A.now, o));
                acct[d] += 1;
                acct[d + 1] += o.len;
                if (o.reslave) {   // ct_update4/6_slave
                    lby = o.slave;
                    reslaved = true;
                }
            } else {
                e = fresh(A.now, o.is_tcp, o.dir);
                if (o.ki_form)
                    e.bits |= SEEN_NON_SYN;
                if (A.nat46 && o.dir == CT_EGRESS)   // (not its local delivery's)
                    e.bits |= NAT46;
                live = created = true;
                acct[0] = acct[1] = acct[2] = acct[3] = 0;
                acct[d] = 1;
                acct[d + 1] = o.len;
                sec = o.sec;
                rev = o.rev;
                lbx = o.lbw;
                lby = o.slave;
            }
        } else if (live) {   // OP_HIT, OP_DELETE
            put_mon(A, ord, hit(e, A.now, o));
            if (o.reslave) {   // ct_update4/6_slave on an entry the batch found
                lby = o.slave;
                reslaved = true;
            }
            if (created) {
                // a hit after this batch wrote the entry anew (a related
                // entry overwritten by a later create): the launch counted it
                // on the entry as it was, which the write replaced
                acct[d] += 1;
                acct[d + 1] += o.len;
            }
            if (o.kind == OP_DELETE) {
                live = false;
                deleted = true;
            }
        }
    }
    if (!summed && live)
        sum_hit(e, A.now, mu);
    // the load balancer's per-slot ct_state of what this batch wrote
    if (A.lb && live && created)
        A.lb[slot] = make_uint4(lbx, lby, 0, 0);
    else if (A.lb && live && reslaved)
        A.lb[slot].y = lby;
    // (the slot's report state, counters and record: one CtState line)
    unsigned long long *ac = reinterpret_cast<unsigned long long *>(A.st[slot].acct);
    CtInfo inf = A.st[slot].info;
    if (!live) {
        // ct_delete4/6: the entry and its counts go; the key stays readable
        // for the host (w | CT_TOMBSTONE) until it has synchronised
        uint32_t *pw = slot_w<V6>(A, slot);
        *pw = *pw | CT_TOMBSTONE;
        ac[0] = ac[1] = ac[2] = ac[3] = 0;
        inf.y |= CTI_DELETED;
    } else if (created) {
        store_state(A.st, slot, e);
        ac[0] = acct[0];
        ac[1] = acct[1];
        ac[2] = acct[2];
        ac[3] = acct[3];
        inf.sec = sec;
        inf.y = (inf.y & ~0xFFFFu) | rev | CTI_CREATED | (deleted ? CTI_DELETED : 0u) |
                (was_fresh ? CTI_FRESH : 0u) | (inf.y & CTI_FRESH);
    } else {
        store_state(A.st, slot, e);
        ac[0] += acct[0];
        ac[1] += acct[1];
        ac[2] += acct[2];
        ac[3] += acct[3];
        inf.y |= CTI_UPDATED;
    }
    A.st[slot].info = inf;
    A.ms[slot] = make_uint2(0, 0);
    if (A.sum)   // (replayed here: the finish leaves the slot alone)
        A.sum[slot] = 0;
    if (lh)
        A.lh[slot] = 0;
}

// ---- the long runs (k_cta_fold's list).  When every op of a run is a
// plain hit of a TCP or UDP entry the batch found (no create, delete,
// related write or counted hit; no monitor lengths wanted) the final state
// does not need the ops one by one: every such hit runs ct_update_timeout
// (ACTION_CREATE directly or after clearing the closing bits; ACTION_CLOSE
// before setting its bit, or as the close timeout once both are set), so
// with one clock per batch
//   flags_seen[dir] = the entry's | the OR of the direction's hits' flags,
//   last_report[dir] = now iff the direction has hits and its interval had
//     passed or its flags grew (the first report sets it, later ones keep it),
//   seen_non_syn |= any TCP hit without the close bit,
//   closing bits = the closes after the last ACTION_CREATE hit (which leaves
//     none), or the entry's | every close when there is no such hit,
//   lifetime = now + CT_CLOSE_TIMEOUT when both closing bits end set (the
//     last hit was a close on a dead entry), else now + the lifetime of the
//     entry's protocol and seen_non_syn (conntrack.h:125-205, 221-285).
// A run is cut into chunks of FOLD_CH ops reduced by whole workgroups
// (a C5 batch's hottest flow holds millions of ops); any other run is
// replayed in order by one thread (fold_run).
//
// Scratch (the pre-dedup list's buffer, u32 words; R = runs' room, C =
// chunks' room): [0, R) run starts (k_cta_fold), then per run RUN_W words,
// then per chunk its run, the OR of its closes, the OR of its closes after
// its last ACTION_CREATE.
constexpr uint32_t FOLD_CH = 4096;
// A slot whose plain hits route summarised (A.lh) has them as one
// ACTION_CREATE hit at the last one's place: RW_LH, the index + 1 of the
// run's first op after it.
enum { RW_R0, RW_END, RW_CBASE, RW_NCH, RW_BAD, RW_F0, RW_F1, RW_ANY, RW_NONSYN, RW_LASTC,
       RW_LAST, RW_LH, RUN_W };
struct LongScratch {
    uint32_t *start, *run, *crun, *call, *cafter;
    __device__ LongScratch(uint32_t *lng, uint32_t ncx)
    {
        const uint32_t R = ncx / FOLD_LONG + 1, C = ncx / FOLD_CH + R;
        start = lng;
        run = lng + R;
        crun = run + RUN_W * R;
        call = crun + C;
        cafter = call + C;
    }
};
// a plain hit, from the header's words alone (no tuple): false for any
// other op; dir 0 rx (ingress), 1 tx
template <bool V6, bool LB>
__device__ __forceinline__ bool plain_hit(const CtaArgs &A, uint32_t ord, uint32_t &dir,
                                          uint32_t &tfl, uint32_t &close, bool &create,
                                          bool &nonsyn)
{
    const uint64_t i = ord_hdr(ord);
    if (ord_sec(ord) != SEC_OP || i >= A.n)
        return false;
    const int st = ord_st(ord);
    if (LB && (reinterpret_cast<const LbRecT<V6> *>(A.lbr)[i].fl & LBF_DROP))
        return false;
    const uint32_t cb = A.ctb[i], cs = (cb >> (4 * st)) & 0xF;
    if (!(cs & CFC_CT_DONE))
        return false;
    const uint32_t b = cs & CFC_CT_RES_MASK;
    const int last = (cb & (CFC_CT_DONE << 4)) ? 1 : 0;
    if (b == 0 || (b == 1 && st == last && A.ver[i] == DROP_POLICY))
        return false;   // (a create or nothing; a delete)
    const uint32_t mt = A.mt[i], proto = mt & 0xFF;
    if (proto != 6 && proto != 17)
        return false;
    const bool eg = A.mode == CFC_MODE_EGRESS && st == 0;
    dir = eg ? 1u : 0u;
    const bool cl = proto == 6 && (mt & CFC_HF_TCP_CLOSE);   // ACTION_CLOSE
    tfl = (proto == 6 && A.tf) ? A.tf[i] : 0u;
    close = cl ? (eg ? TX_CLOSING : RX_CLOSING) : 0u;
    create = !cl;   // (TCP without RST/FIN, UDP: ACTION_CREATE)
    nonsyn = proto == 6 && !cl;
    return true;
}
// the long runs' ends and chunks
template <bool V6, bool LB>
__global__ __launch_bounds__(256) void k_cta_fold_plan(CtaArgs A, const uint64_t *cx,
                                                       const uint32_t *pncx, uint32_t *lng)
{
    const uint32_t ncx = *pncx, nl = A.cnt[CTA_NLONG];
    LongScratch L(lng, ncx);
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < nl; k += gridDim.x * 256) {
        const uint32_t r0 = L.start[k];
        const uint32_t slot = (uint32_t)(cx[r0] >> A.ob);
        uint32_t lo = r0 + FOLD_LONG, hi = ncx;   // the first index past the slot
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if ((uint32_t)(cx[mid] >> A.ob) == slot)
                lo = mid + 1;
            else
                hi = mid;
        }
        const uint32_t nch = (lo - r0 + FOLD_CH - 1) / FOLD_CH;
        const uint32_t cb = atomicAdd(&A.cnt[CTA_NLCH], nch);
        uint32_t *w = L.run + RUN_W * k;
        w[RW_R0] = r0;
        w[RW_END] = lo;
        w[RW_CBASE] = cb;
        w[RW_NCH] = nch;
        for (int j = RW_BAD; j < RUN_W; j++)
            w[j] = 0;
        const uint32_t lh = A.lh ? A.lh[slot] : 0u;
        if (lh) {   // the first op past order lh - 1
            uint32_t a = r0, b = lo;
            while (a < b) {
                const uint32_t mid = a + (b - a) / 2;
                if ((uint32_t)(cx[mid] & ((1ull << A.ob) - 1)) < lh)
                    a = mid + 1;
                else
                    b = mid;
            }
            w[RW_LH] = a + 1;
        }
        for (uint32_t j = 0; j < nch; j++)
            L.crun[cb + j] = k;
    }
}
// one workgroup per chunk: its ops' aggregates into its run's words
template <bool V6, bool LB>
__global__ __launch_bounds__(256) void k_cta_fold_agg(CtaArgs A, const uint64_t *cx,
                                                      const uint32_t *pncx, uint32_t *lng)
{
    const uint32_t ncx = *pncx, nc = A.cnt[CTA_NLCH];
    const uint64_t omask = (1ull << A.ob) - 1;
    LongScratch L(lng, ncx);
    __shared__ uint32_t s_bad, s_f[2], s_any, s_nonsyn, s_lastc, s_last, s_call, s_cafter;
    for (uint32_t c = blockIdx.x; c < nc; c += gridDim.x) {
        const uint32_t k = L.crun[c];
        uint32_t *w = L.run + RUN_W * k;
        const uint32_t a = w[RW_R0] + (c - w[RW_CBASE]) * FOLD_CH;
        const uint32_t b = min(w[RW_END], a + FOLD_CH);
        if (threadIdx.x == 0)
            s_bad = s_f[0] = s_f[1] = s_any = s_nonsyn = s_lastc = s_last = s_call = s_cafter = 0;
        __syncthreads();
        uint32_t bad = 0, f[2] = {0, 0}, any = 0, ns = 0, lastc = 0, last = 0, call = 0;
        for (uint32_t r = a + threadIdx.x; r < b; r += 256) {
            uint32_t d, tfl, cl;
            bool cr, nsy;
            if (!plain_hit<V6, LB>(A, (uint32_t)(cx[r] & omask), d, tfl, cl, cr, nsy)) {
                bad = 1;
                continue;
            }
            f[d] |= tfl;
            any |= 1u << d;
            ns |= nsy ? 1u : 0u;
            call |= cl;
            if (cr)
                lastc = max(lastc, r + 1);   // (+1: 0 = none)
            last = max(last, r + 1);
        }
        if (bad)
            atomicOr(&s_bad, 1u);
        if (f[0])
            atomicOr(&s_f[0], f[0]);
        if (f[1])
            atomicOr(&s_f[1], f[1]);
        if (any)
            atomicOr(&s_any, any);
        if (ns)
            atomicOr(&s_nonsyn, 1u);
        if (call)
            atomicOr(&s_call, call);
        if (lastc)
            atomicMax(&s_lastc, lastc);
        if (last)
            atomicMax(&s_last, last);
        __syncthreads();
        // the chunk's closes after its last ACTION_CREATE hit (the
        // summarised hits' one among them)
        const uint32_t lhI = w[RW_LH];
        const uint32_t from =
            (lhI && lhI - 1 >= a && lhI - 1 < b) ? max(s_lastc, lhI - 1) : s_lastc;
        uint32_t after = 0;
        if (!s_bad)
            for (uint32_t r = max(a, from) + threadIdx.x; r < b; r += 256) {
                uint32_t d, tfl, cl;
                bool cr, nsy;
                if (plain_hit<V6, LB>(A, (uint32_t)(cx[r] & omask), d, tfl, cl, cr, nsy))
                    after |= cl;
            }
        if (after)
            atomicOr(&s_cafter, after);
        __syncthreads();
        if (threadIdx.x == 0) {
            if (s_bad)
                atomicOr(&w[RW_BAD], 1u);
            atomicOr(&w[RW_F0], s_f[0]);
            atomicOr(&w[RW_F1], s_f[1]);
            atomicOr(&w[RW_ANY], s_any);
            atomicOr(&w[RW_NONSYN], s_nonsyn);
            atomicMax(&w[RW_LASTC], s_lastc);
            atomicMax(&w[RW_LAST], s_last);
            L.call[c] = s_call;
            L.cafter[c] = s_cafter;
        }
        __syncthreads();
    }
}
// one thread per long run: its final state (or its replay)
template <bool V6, bool LB>
__global__ __launch_bounds__(256) void k_cta_fold_fin(CtaArgs A, const uint64_t *cx,
                                                      const uint32_t *pncx, uint32_t *lng)
{
    const uint32_t ncx = *pncx, nl = A.cnt[CTA_NLONG];
    const uint64_t omask = (1ull << A.ob) - 1;
    LongScratch L(lng, ncx);
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < nl; k += gridDim.x * 256) {
        const uint32_t *w = L.run + RUN_W * k;
        const uint32_t r0 = w[RW_R0];
        const uint32_t slot = (uint32_t)(cx[r0] >> A.ob);
        if (w[RW_BAD] || A.mon || (A.ms[slot].x & MARK_FRESH)) {
            fold_run<V6, LB>(A, cx, ncx, r0);
            continue;
        }
        St e = load_state(A.st, slot);
        const uint32_t now = A.now;
        const uint32_t lhI = w[RW_LH];
        const uint32_t mu = lhI ? (A.sum ? A.sum[slot] : A.ms[slot].x >> SUM_SH) : 0u;
        for (int d = 0; d < 2; d++) {   // 0: rx (ingress), 1: tx
            if (!(((w[RW_ANY] | mu >> 16) >> d) & 1))
                continue;
            const uint32_t fl = (d == 0 ? w[RW_F0] : w[RW_F1]) | ((mu >> (8 * d)) & 0xFFu);
            uint32_t &acc = d == 0 ? e.seen_rx : e.seen_tx;
            uint32_t &lr = d == 0 ? e.last_rx : e.last_tx;
            if (lr + CT_REPORT_INTERVAL < now || (fl & ~acc & 0xFFu))
                lr = now;
            acc = (acc | fl) & 0xFF;
        }
        if (w[RW_NONSYN] || (mu & (1u << 18)))
            e.bits |= SEEN_NON_SYN;
        const uint32_t cbase = w[RW_CBASE], nch = w[RW_NCH], lastc = w[RW_LASTC];
        uint32_t cb = 0, j0 = 0;
        if (lhI && lhI - 1 >= lastc) {   // the summarised hits are the last ACTION_CREATE
            const uint32_t x = lhI - 1;
            if (x >= w[RW_END]) {
                j0 = nch;
            } else {
                j0 = (x - r0) / FOLD_CH;
                cb = L.cafter[cbase + j0];
                j0++;
            }
        } else if (lastc) {   // the closes after the last ACTION_CREATE hit
            j0 = (lastc - 1 - r0) / FOLD_CH;
            cb = L.cafter[cbase + j0];
            j0++;
        } else {
            cb = e.bits & 3u;
        }
        for (uint32_t j = j0; j < nch; j++)
            cb |= L.call[cbase + j];
        e.bits = (e.bits & ~3u) | cb;
        const uint32_t ord = (uint32_t)(cx[w[RW_LAST] - 1] & omask);
        const bool tcp = (A.mt[ord_hdr(ord)] & 0xFF) == 6;
        const uint32_t life = !tcp ? CT_LIFETIME_NONTCP
                              : (e.bits & SEEN_NON_SYN) ? CT_LIFETIME_TCP : CT_SYN_TIMEOUT;
        e.lifetime = now + ((cb & 3u) == 3u ? CT_CLOSE_TIMEOUT : life);
        store_state(A.st, slot, e);
        A.st[slot].info.y |= CTI_UPDATED;
        A.ms[slot] = make_uint2(0, 0);
        if (A.sum)
            A.sum[slot] = 0;
        if (lhI)
            A.lh[slot] = 0;
    }
}

// ---- finish: the summaries of unordered slots.  Their hits are plain
// ACTION_CREATE or ACTION_UNSPEC (RST/FIN and deletes are ordered), and a
// closing bit is only ever set by a TCP RST/FIN, on a TCP entry, whose
// other packets are ACTION_CREATE: the first such hit clears both closing
// bits and re-arms the timeout (__ct_lookup, conntrack.h:259-266; a dead
// entry skips the first update and takes the second — one update either
// way), so an entry with closing bits ends with them cleared and the
// summary applied.  With no closing bit set every hit re-arms the timeout,
// so the final state is:
// seen_non_syn |= any TCP hit without the close bit; lifetime from the last
// hit = now + (TCP ? (seen_non_syn ? TCP : SYN) : NONTCP); per direction
// with hits, flags_seen |= their flags and last_report = now iff the
// interval had passed or the flags grew (the first report sets it to now,
// later ones keep it).
template <bool V6>
__global__ __launch_bounds__(256) void k_cta_finish(CtaArgs A)
{
    // FU consecutive slots per thread and step: their summary words in
    // 16-byte loads, then the touched slots' state (a few per step)
    constexpr int FU = 16;
    const uint64_t slots = (uint64_t)A.mask + 1;
    const uint64_t span = 256ull * FU, stride = (uint64_t)gridDim.x * span;
    for (uint64_t base = (uint64_t)blockIdx.x * span; base < slots; base += stride) {
        const uint64_t s0 = base + (uint64_t)FU * threadIdx.x;
        uint32_t m[FU];
        if (s0 + FU <= slots) {   // (slots: a power of two >= FU; arrays aligned)
            if (A.sum) {
                const uint4 *p = reinterpret_cast<const uint4 *>(A.sum + s0);
#pragma unroll
                for (int q = 0; q < FU / 4; q++) {
                    const uint4 v = p[q];
                    m[4 * q] = v.x;
                    m[4 * q + 1] = v.y;
                    m[4 * q + 2] = v.z;
                    m[4 * q + 3] = v.w;
                }
            } else {
                const uint4 *p = reinterpret_cast<const uint4 *>(A.ms + s0);
#pragma unroll
                for (int q = 0; q < FU / 2; q++) {
                    const uint4 v = p[q];   // {ms[2q].x, .y, ms[2q + 1].x, .y}
                    m[2 * q] = v.x >> SUM_SH;
                    m[2 * q + 1] = v.z >> SUM_SH;
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < FU; u++)
                m[u] = s0 + u < slots ? (A.sum ? A.sum[s0 + u] : A.ms[s0 + u].x >> SUM_SH) : 0u;
        }
        uint32_t any = 0;
#pragma unroll
        for (int u = 0; u < FU; u++)
            any |= (m[u] != 0u) << u;
        // the touched slots four at a time, their state loads issued together
        // (one dependent chain per slot left the pass waiting on each)
        for (uint32_t mm = any; mm;) {
            uint32_t sl4[4], m4[4];
            bool on[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                on[j] = mm != 0;
                const int u = on[j] ? __ffs(mm) - 1 : 0;
                mm &= on[j] ? mm - 1 : mm;
                sl4[j] = (uint32_t)(s0 + u);
                m4[j] = m[0];
#pragma unroll
                for (int q = 1; q < FU; q++)   // (m[u], without dynamic indexing)
                    m4[j] = u == q ? m[q] : m4[j];
            }
            // the slot's report state and record: one CtState line.  (The
            // entry's protocol is in the summary: every hit a finish sees
            // is a plain hit without the close bit — closes and deletes
            // are ordered — so a TCP entry's summary always carries bit 18,
            // "a TCP hit without the close bit", and no other entry's does.)
            St x4[4];
            uint32_t iy[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                x4[j] = load_state(A.st, sl4[j]);
                iy[j] = A.st[sl4[j]].info.y;
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
            if (!on[j])
                continue;
            const uint32_t sl = sl4[j];
            St x = x4[j];
            const uint32_t mu = m4[j];
            if (A.sum)
                A.sum[sl] = 0;
            else
                A.ms[sl].x = 0;
            sum_hit(x, A.now, mu);
            store_state(A.st, sl, x);
            A.st[sl].info.y = iy[j] | CTI_UPDATED;
            }
        }
    }
}

// ---- the trace words' CT result and monitor length in packet order (a
// batch whose caller wants the event words): the stage the trace reports
// (local delivery's when it ran) with the result the packet order gave it
// (ctorder.hip) and the length __ct_lookup then left (the fold's; a repeat
// of the same hit that the fold skipped reports nothing — its state update
// already happened — except a close: ACTION_CLOSE reports TRACE_PAYLOAD_LEN
// whatever the entry's state, conntrack.h:268-281), conn_is_dns's MTU
// (conntrack.h:585-586)
template <bool V6>
__global__ __launch_bounds__(256) void k_cta_mon(CtaArgs A)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= A.n)
        return;
    const uint32_t w = A.nt[i];
    if (((w >> 16) & 0xF) < CFC_NT_TRACE)
        return;
    const uint32_t cb = A.ctb[i];
    const int st = (cb & (CFC_CT_DONE << 4)) ? 1 : 0;
    const uint32_t cs = (cb >> (4 * st)) & 0xF;
    if (!(cs & CFC_CT_DONE))
        return;
    const uint32_t res = cs & CFC_CT_RES_MASK;
    uint32_t m = TRACE_PAYLOAD_LEN;
    const uint32_t proto = A.mt[i] & 0xFF;
    // the L4 word the stage's lookup read: with a load balancer the service
    // step's tuple (stage 0) or the packet as it left it (stage 1)
    uint32_t pw = A.pt[i];
    if (A.lbr) {
        if constexpr (V6) {
            const LbRec6 &l = reinterpret_cast<const LbRec6 *>(A.lbr)[i];
            pw = st ? l.ppt : l.tpt;
        } else {
            const LbRec4 &l = reinterpret_cast<const LbRec4 *>(A.lbr)[i];
            pw = st ? l.ppt : l.tpt;
        }
    }
    if (res != CT_NEW) {
        const uint8_t c = A.mon[2 * i + st];
        m = c == 1 ? 1u : c == 2 ? TRACE_PAYLOAD_LEN : 0u;
        if (c == 0xFF && ct_action(V6, proto, pw, A.mt[i]) == 2)
            m = TRACE_PAYLOAD_LEN;
    }
    const CtProbe k = ct_probe<V6>(proto, pw, CT_INGRESS, 0);
    // (ipv6_l3_from_lxc sets TRACE_PAYLOAD_LEN after its ct_create6,
    // bpf_lxc.c:248: a new flow's egress trace is not captured at MTU)
    const bool v6_new_egress = V6 && A.mode == CFC_MODE_EGRESS && st == 0 && res == CT_NEW;
    if ((res >= CT_REPLY ? k.td : k.ts) == 0x3500u && !v6_new_egress)   // conn_is_dns
        m = MTU_LEN;
    A.nt[i] = (w & 0x000FFFFFu) | res << 20 | mon_class(m) << 22;
}

// ---- host synchronisation: the changed slots, compacted
template <bool V6>
struct SyncOf;
template <>
struct SyncOf<false> {
    using Rec = CtSyncRec;
    using Slot = Ct4Slot;
};
template <>
struct SyncOf<true> {
    using Rec = CtSyncRec6;
    using Slot = Ct6Slot;
};
template <bool V6>
__global__ __launch_bounds__(256) void k_cta_collect(const typename SyncOf<V6>::Slot *ct,
                                                     CtState *st, const uint4 *lb,
                                                     uint64_t slots,
                                                     typename SyncOf<V6>::Rec *out,
                                                     uint32_t cap, uint32_t *cnt)
{
    // four slots per thread and step, each phase's loads together
    constexpr int CU = 4;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * CU;
    for (uint64_t base = (uint64_t)blockIdx.x * 256 * CU; base < slots; base += stride) {
        CtInfo in[CU];
        uint32_t nd = 0;
#pragma unroll
        for (int u = 0; u < CU; u++) {
            const uint64_t s = base + u * 256 + threadIdx.x;
            in[u] = s < slots ? st[s].info : CtInfo{0, 0};
            nd += (in[u].y >> 16) != 0;
        }
        uint4 k[CU], t[CU], k2[CU], k3[CU], l[CU];
#pragma unroll
        for (int u = 0; u < CU; u++) {
            const uint64_t s = base + u * 256 + threadIdx.x;
            if ((in[u].y >> 16) != 0) {
                if constexpr (V6) {
                    k[u] = ld16(ct[s].d);
                    k2[u] = ld16(ct[s].s);
                    k3[u] = ld16(&ct[s].z);
                } else {
                    k[u] = ld16(ct + s);
                }
                t[u] = ld16(&st[s].tm);
                l[u] = lb ? ld16(lb + s) : make_uint4(0, 0, 0, 0);
            }
        }
        uint32_t r = block_count_n(cnt, nd);
#pragma unroll
        for (int u = 0; u < CU; u++) {
            const uint64_t s = base + u * 256 + threadIdx.x;
            if ((in[u].y >> 16) == 0)
                continue;
            if (r < cap) {
                typename SyncOf<V6>::Rec &o = out[r];
                o.slot = (uint32_t)s;
                o.info = in[u];
                if constexpr (V6) {
                    o.d[0] = k[u].x; o.d[1] = k[u].y; o.d[2] = k[u].z; o.d[3] = k[u].w;
                    o.s[0] = k2[u].x; o.s[1] = k2[u].y; o.s[2] = k2[u].z; o.s[3] = k2[u].w;
                    o.z = k3[u].x;
                    o.w = k3[u].y;
                } else {
                    o.x = k[u].x;
                    o.y = k[u].y;
                    o.z = k[u].z;
                    o.w = k[u].w;
                }
                o.last_rx = t[u].x;
                o.last_tx = t[u].y;
                o.flags = t[u].z;
                o.lifetime = t[u].w;
                o.pad = lb ? (l[u].y & 0xFFFF) | ((l[u].x >> 16) & 1) << 16 | 1u << 31 : 0u;
                st[s].info.y = in[u].y & 0xFFFFu;
            }
            r++;
        }
    }
}
// after the host has taken them: deleted slots become plain tombstones
// (free for inserts again)
__global__ __launch_bounds__(256) void k_cta_tomb(Ct4Slot *ct4, const CtSyncRec *rec, uint32_t n)
{
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= n)
        return;
    const uint32_t s = rec[r].slot;
    if ((rec[r].w & CT_TOMBSTONE) == CT_TOMBSTONE) {
        const uint4 t = make_uint4(0, 0, 0, CT_TOMBSTONE);
        *reinterpret_cast<uint4 *>(ct4 + s) = t;
    }
}
__global__ __launch_bounds__(256) void k_cta_tomb6(Ct6Slot *ct6, const CtSyncRec6 *rec, uint32_t n)
{
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= n)
        return;
    const uint32_t s = rec[r].slot;
    if ((rec[r].w & CT_TOMBSTONE) == CT_TOMBSTONE) {
        const uint4 z = make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4 *>(ct6[s].d) = z;
        *reinterpret_cast<uint4 *>(ct6[s].s) = z;
        *reinterpret_cast<uint4 *>(&ct6[s].z) = make_uint4(0, CT_TOMBSTONE, 0, 0);
    }
}
// slots whose word is not 0, four per thread and step
template <class Slot>
__global__ __launch_bounds__(256) void k_ct_nonfree(const Slot *ct4, uint64_t slots,
                                                    uint32_t *cnt)
{
    uint32_t c = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * 4;
    for (uint64_t base = (uint64_t)blockIdx.x * 256 * 4; base < slots; base += stride) {
        uint32_t w[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t s = base + u * 256 + threadIdx.x;
            w[u] = s < slots ? ct4[s].w : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            c += w[u] != 0;
    }
    block_add(cnt, c);
}

// ---- device-side growth of a CT table (cfc_api.cpp ct_grow) ---------------
// The reference's CT maps are fixed-size LRU hashes that never stop for an
// insert (bpf_lxc.c:53-89); the device table is open-addressed and sized at
// commit, so a batch that would take it past 3/4 load moves it into a table
// with more slots here, on the device: every slot that holds a key — a live
// entry, or one an apply deleted that the host has not taken yet (w |
// CT_TOMBSTONE: its record goes to the host at the next ct_sync) — is
// inserted at its home slot's probe sequence in the new table (a CAS on the
// free word: the new table has no other writer), with its CtState line and
// load-balancer word; plain tombstones and free slots are dropped.  map[old
// slot] = its new slot (NONE: dropped): the host mirror and the pending GC
// log follow it (ct_grow).  Four old slots per thread and step, each phase's
// loads issued together.
template <bool V6>
__global__ __launch_bounds__(256) void k_ct_rehash(const typename SyncOf<V6>::Slot *ok,
                                                   const CtState *ost, const uint4 *olb,
                                                   uint64_t oslots,
                                                   typename SyncOf<V6>::Slot *nk, CtState *nst,
                                                   uint4 *nlb, uint32_t nmask, uint32_t *map,
                                                   uint32_t *cnt)
{
    constexpr int RU = 4;
    uint32_t moved = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * RU;
    for (uint64_t base = (uint64_t)blockIdx.x * 256 * RU; base < oslots; base += stride) {
        uint32_t w[RU];
#pragma unroll
        for (int u = 0; u < RU; u++) {
            const uint64_t sl = base + u * 256 + threadIdx.x;
            w[u] = sl < oslots ? ok[sl].w : 0u;
        }
#pragma unroll
        for (int u = 0; u < RU; u++) {
            const uint64_t sl = base + u * 256 + threadIdx.x;
            if (sl >= oslots)
                continue;
            if (w[u] == 0 || w[u] == CT_TOMBSTONE) {
                map[sl] = NONE;
                continue;
            }
            // (a deleted entry is placed by its key's own word)
            const uint32_t w0 = (w[u] & CT_TOMBSTONE) == CT_TOMBSTONE ? w[u] & ~CT_TOMBSTONE : w[u];
            uint32_t i;
            if constexpr (V6) {
                const uint4 d = ld16(ok[sl].d), sa = ld16(ok[sl].s);
                const uint32_t z = ok[sl].z;
                const uint32_t dw[4] = {d.x, d.y, d.z, d.w}, sw[4] = {sa.x, sa.y, sa.z, sa.w};
                for (i = ct_home6(dw, sw, z, w0) & nmask;; i = (i + 1) & nmask)
                    if (atomicCAS(&nk[i].w, 0u, w[u]) == 0u)
                        break;
                *reinterpret_cast<uint4 *>(nk[i].d) = d;
                *reinterpret_cast<uint4 *>(nk[i].s) = sa;
                nk[i].z = z;
            } else {
                const uint4 k = ld16(ok + sl);
                for (i = ct_home4(k.x, k.y, k.z, w0) & nmask;; i = (i + 1) & nmask)
                    if (atomicCAS(&nk[i].w, 0u, w[u]) == 0u)
                        break;
                nk[i].x = k.x;
                nk[i].y = k.y;
                nk[i].z = k.z;
            }
            const uint4 *src = reinterpret_cast<const uint4 *>(ost + sl);
            uint4 *dst = reinterpret_cast<uint4 *>(nst + i);
            const uint4 l0 = src[0], l1 = src[1], l2 = src[2], l3 = src[3];
            dst[0] = l0;
            dst[1] = l1;
            dst[2] = l2;
            dst[3] = l3;
            if (olb)
                nlb[i] = olb[sl];
            map[sl] = i;
            moved++;
        }
    }
    block_add(cnt, moved);
}
// slots recorded against an older table, through its map (NONE: dropped)
__global__ __launch_bounds__(256) void k_ct_remap(uint32_t *slot, uint64_t n, uint32_t stride,
                                                  const uint32_t *map)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    uint32_t &v = slot[i * stride];
    v = v == NONE ? NONE : map[v];
}

// ---- the CtState lines from and to the host ---------------------------------
// a built table's report state (the flattened CtTimer array) into its lines
// (the rest of each line zero: no counts, no record)
__global__ __launch_bounds__(256) void k_ct_st_init(CtState *st, const CtTimer *tm, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    uint4 *l = reinterpret_cast<uint4 *>(st + i);
    l[0] = ld16(tm + i);
    l[1] = l[2] = l[3] = make_uint4(0, 0, 0, 0);
}
// the CONNTRACK_ACCOUNTING counts of every line into a dense [slot][4]
// array for the host's fold, and the lines' counts cleared
__global__ __launch_bounds__(256) void k_ct_acct_take(CtState *st, ulonglong2 *out, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    ulonglong2 *a = reinterpret_cast<ulonglong2 *>(st[i].acct);
    const ulonglong2 x = a[0], y = a[1];
    out[2 * i] = x;
    out[2 * i + 1] = y;
    if (x.x | x.y | y.x | y.y)
        a[0] = a[1] = make_ulonglong2(0, 0);
}

// ---- garbage collection (cfc_ct_gc, ctmap.go:303-325 doFiltering) ---------
__device__ __forceinline__ bool gc_in_set(const uint32_t *set, uint32_t n, uint32_t a)
{
    uint32_t lo = 0, hi = n;   // sorted ascending
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (set[mid] < a)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo < n && set[lo] == a;
}
// IPv6 addresses: raw words, sorted lexicographically (x, y, z, w) by the
// host (ct_gc_dev)
__device__ __forceinline__ bool a6_lt(uint4 a, uint4 b)
{
    return a.x != b.x ? a.x < b.x : a.y != b.y ? a.y < b.y : a.z != b.z ? a.z < b.z : a.w < b.w;
}
__device__ __forceinline__ bool gc_in_set(const uint4 *set, uint32_t n, uint4 a)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a6_lt(set[mid], a))
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo < n && aeq(set[lo], a);
}
// doFiltering on the entry's two addresses and lifetime
__device__ __forceinline__ bool gc_delete(const CtGcArgs &A, uint32_t x, uint32_t y,
                                          uint32_t lifetime)
{
    if ((A.flags & CTG_REMOVE_EXPIRED) && lifetime < A.time)
        return true;
    if ((A.flags & CTG_VALID) && !gc_in_set(A.valid, A.n_valid, x) &&
        !gc_in_set(A.valid, A.n_valid, y))
        return true;
    return (A.flags & CTG_MATCH) &&
           (gc_in_set(A.match, A.n_match, x) || gc_in_set(A.match, A.n_match, y));
}
__device__ __forceinline__ bool gc_delete(const CtGcArgs &A, uint4 x, uint4 y, uint32_t lifetime)
{
    if ((A.flags & CTG_REMOVE_EXPIRED) && lifetime < A.time)
        return true;
    if ((A.flags & CTG_VALID) && !gc_in_set(A.valid6, A.n_valid, x) &&
        !gc_in_set(A.valid6, A.n_valid, y))
        return true;
    return (A.flags & CTG_MATCH) &&
           (gc_in_set(A.match6, A.n_match, x) || gc_in_set(A.match6, A.n_match, y));
}
// the selected map an entry belongs to (its CT map: owner word, TCP or ANY
// kind), or -1
__device__ __forceinline__ int gc_map(const uint32_t *smaps, uint32_t n, uint32_t mw)
{
    for (uint32_t j = 0; j < n; j++)
        if (smaps[j] == mw)
            return (int)j;
    return -1;
}

// Four slots per thread and step (grid-stride), each phase's loads issued
// together.  A deleted entry the host mirror may hold is logged for it; one
// a device insert brought in since the last sync (CTI_FRESH) is just
// dropped.  Either way the slot becomes a plain tombstone with no dirty bits
// and zero accounting.  The log's places are taken once per block and step
// (block_count_n): a steady-state GC deletes millions of entries, and one
// atomic per wave on the shared counter serialised at its L2 channel.
constexpr int GC_U = 8;
// (1024-thread blocks, one per CU: one list atomic per 8192 slots)
constexpr int GC_B = 1024;
// V6: the IPv6 table (doGC6, ctmap.go:239, next to doGC4 :272): a slot's
// {z, w} words first (its map and state), its addresses only for an entry
// of a selected map
template <bool V6>
__global__ __launch_bounds__(GC_B) void k_ct_gc(CtGcArgs A)
{
    __shared__ uint32_t smaps[CTG_MAX_MAPS], scnt[CTG_MAX_MAPS];
    __shared__ uint32_t sw[GC_B * GC_U];   // (a step's w words after its deletes)
    for (uint32_t j = threadIdx.x; j < A.n_maps; j += GC_B) {
        smaps[j] = A.maps[j];
        scnt[j] = 0;
    }
    __syncthreads();
    uint32_t fresh = 0, live = 0, nonfree = 0, freed = 0;
    const uint64_t stride = (uint64_t)gridDim.x * GC_B * GC_U;
    // (every thread runs the same number of steps: block_count_n needs the
    // whole block)
    for (uint64_t base = (uint64_t)blockIdx.x * GC_B * GC_U; base < A.slots; base += stride) {
        // k: IPv4 the key {daddr, saddr, ports, w}; IPv6 {z, w, 0, 0}, then
        // the addresses (kd, ks) of the selected maps' entries
        uint4 k[GC_U];
        int j[GC_U];
        uint32_t life[GC_U], infy[GC_U];
#pragma unroll
        for (int u = 0; u < GC_U; u++) {   // (no branches: the loads issue together)
            const uint64_t s = base + u * GC_B + threadIdx.x;
            const uint64_t sc = s < A.slots ? s : A.slots - 1;
            if constexpr (V6) {
                const uint4 t = ld16(&A.ct6[sc].z);
                k[u] = make_uint4(0, 0, t.x, t.y);   // (z, w where the v4 key has them)
            } else {
                k[u] = ld16(A.ct4 + sc);
            }
        }
#pragma unroll
        for (int u = 0; u < GC_U; u++)
            if (base + u * GC_B + threadIdx.x >= A.slots)
                k[u] = make_uint4(0, 0, 0, 0);

        // a tombstone, a claim, or an apply's delete the host has not taken
        // is no entry of a map
#pragma unroll
        for (int u = 0; u < GC_U; u++) {
            nonfree += k[u].w != 0;
            j[u] = (k[u].w != 0 && !(k[u].w & 0xF000u))
                       ? gc_map(smaps, A.n_maps,
                                (k[u].w & 0xFFFF0800u) | ((k[u].w & 0xFF) != 6 ? 2u : 0u))
                       : -1;
        }
#pragma unroll
        for (int u = 0; u < GC_U; u++) {   // (an entry's line only: one per live slot)
            const uint64_t s = base + u * GC_B + threadIdx.x;
            life[u] = j[u] >= 0 ? A.st[s].tm.lifetime : 0u;
        }
        bool del[GC_U], logit[GC_U];
        uint4 kd[GC_U], ks[GC_U];
        if constexpr (V6) {
#pragma unroll
            for (int u = 0; u < GC_U; u++) {
                const uint64_t s = base + u * GC_B + threadIdx.x;
                kd[u] = j[u] >= 0 ? ld16(A.ct6[s].d) : make_uint4(0, 0, 0, 0);
                ks[u] = j[u] >= 0 ? ld16(A.ct6[s].s) : make_uint4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int u = 0; u < GC_U; u++) {
            const uint64_t s = base + u * GC_B + threadIdx.x;
            bool d;
            if constexpr (V6)
                d = gc_delete(A, kd[u], ks[u], life[u]);
            else
                d = gc_delete(A, k[u].x, k[u].y, life[u]);
            del[u] = j[u] >= 0 && d && !(A.protect && ((A.protect[s >> 5] >> (s & 31)) & 1u));
            infy[u] = del[u] ? A.st[s].info.y : 0u;
        }
        uint32_t nl = 0;
#pragma unroll
        for (int u = 0; u < GC_U; u++) {
            live += j[u] >= 0 && !del[u];
            // only a key a device insert brought in since the last sync is
            // unknown to the host
            logit[u] = del[u] && !(infy[u] & CTI_FRESH);
            fresh += del[u] && !logit[u];
            nl += logit[u];
        }
        uint32_t r = block_count_n(&A.cnt[CTG_DELETED], nl);
#pragma unroll
        for (int u = 0; u < GC_U; u++) {
            if (!del[u])
                continue;
            const uint64_t s = base + u * GC_B + threadIdx.x;
            if (logit[u]) {
                if (r < A.log_cap) {
                    if constexpr (V6)
                        A.log6[r] = CtGcRec6{(uint32_t)s, kd[u], ks[u], k[u].z, k[u].w};
                    else
                        A.log[r] = CtGcRec{(uint32_t)s, k[u].x, k[u].y, k[u].z, k[u].w};
                }
                r++;
                atomicAdd(&scnt[j[u]], 1u);
            }
            if constexpr (V6) {
                const uint4 z = make_uint4(0, 0, 0, 0);
                *reinterpret_cast<uint4 *>(A.ct6[s].d) = z;
                *reinterpret_cast<uint4 *>(A.ct6[s].s) = z;
                *reinterpret_cast<uint4 *>(&A.ct6[s].z) = make_uint4(0, CT_TOMBSTONE, 0, 0);
            } else {
                *reinterpret_cast<uint4 *>(A.ct4 + s) = make_uint4(0, 0, 0, CT_TOMBSTONE);
            }
            // (the line's counters and record; its report state is dead)
            ulonglong2 *a = reinterpret_cast<ulonglong2 *>(A.st[s].acct);
            a[0] = a[1] = make_ulonglong2(0, 0);
            A.st[s].info = CtInfo{0, 0};
        }
        // the tails of this step's clusters: a plain tombstone whose run of
        // tombstones ends at a free slot is freed (a live entry keeps the
        // tombstones before it: a probe for it runs through them).  The
        // step's words after its deletes go to LDS and each tombstone walks
        // forward there; the slot after the step's range is read once at L2.
        // A slot only goes live -> tombstone -> free here, so a stale read of
        // it can only keep a tail (one next to another block's slots, which
        // the next GC frees), never free a slot a probe still runs through.
        const uint32_t lim = (uint32_t)min<uint64_t>(GC_B * GC_U, A.slots - base);
        const bool whole = lim == A.slots;   // (the whole table in one step: the walk wraps)
#pragma unroll
        for (int u = 0; u < GC_U; u++)
            sw[u * GC_B + threadIdx.x] = del[u] ? CT_TOMBSTONE : k[u].w;
        const uint32_t *pnext = V6 ? &A.ct6[(base + lim) & A.mask].w : &A.ct4[(base + lim) & A.mask].w;
        const uint32_t wnext = whole ? 1u
                                     : __hip_atomic_load(pnext, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < GC_U; u++) {
            const uint32_t c = u * GC_B + threadIdx.x;
            if (c >= lim || sw[c] != CT_TOMBSTONE)
                continue;
            uint32_t e = c, after = 1;
            for (uint32_t m = 1; m < lim; m++) {
                if (++e == lim) {
                    if (!whole) {
                        after = wnext;
                        break;
                    }
                    e = 0;
                }
                if (sw[e] != CT_TOMBSTONE) {
                    after = sw[e];
                    break;
                }
            }
            if (after == 0) {
                if constexpr (V6)
                    A.ct6[base + c].w = 0u;
                else
                    A.ct4[base + c].w = 0u;
                freed++;
            }
        }
        __syncthreads();   // (sw again next step)
    }
    block_add(&A.cnt[CTG_FREED], freed);
    block_add(&A.cnt[CTG_LIVE], live);
    block_add(&A.cnt[CTG_NONFREE], nonfree);
    block_add(&A.cnt[CTG_FRESH], fresh);
    for (uint32_t j = threadIdx.x; j < A.n_maps; j += GC_B)
        if (scnt[j])
            atomicAdd(&A.mcnt[j], scnt[j]);
}

// the pending TCP-map ICMP entries (CtLog): lifetime as ct_create4 wrote it
// (now + CT_LIFETIME_NONTCP, conntrack.h:741-760; no lookup ever updates
// one), the TCP map of its owner
template <class Log>
__global__ __launch_bounds__(256) void k_ct_gc_log(CtGcArgs A, const Log *in, uint32_t n,
                                                   Log *out)
{
    __shared__ uint32_t smaps[CTG_MAX_MAPS];
    for (uint32_t j = threadIdx.x; j < A.n_maps; j += 256)
        smaps[j] = A.maps[j];
    __syncthreads();
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    Log g{};
    bool keep = false;
    if (i < n) {
        g = in[i];
        keep = gc_map(smaps, A.n_maps, g.w & 0xFFFF0800u) < 0 ||
               !gc_delete(A, g.x, g.y, g.now + CT_LIFETIME_NONTCP);
    }
    // (one list atomic per block: per wave, a million entries' worth
    // serialised at the counter's L2 channel)
    const uint32_t r = block_count(&A.cnt[CTG_LOGKEPT], keep);
    if (keep)
        out[r] = g;
}

__global__ __launch_bounds__(256) void k_ct_protect(const uint32_t *hs, uint64_t nk, uint32_t *bm)
{
    const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t sl = k < nk ? hs[k] : HS_NONE;
    if (sl != HS_NONE)
        atomicOr(&bm[sl >> 5], 1u << (sl & 31));
}

unsigned blocks_for(uint64_t n, unsigned cap)
{
    const uint64_t b = (n + 255) / 256;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(b, cap));
}

// ---- the request and op lists' sort: keys `home slot << ob | order`,
// unique, a few hundred thousand to a few million long, some laid out for a
// bound with all-ones keys in the unused places.  A device-wide radix sort
// of 56-bit keys runs seven passes, each two fills and a launch (≈ 35 µs per
// pass at these sizes, launch- and lookback-bound).  Instead the keys go
// into 2048 buckets (a count, a scan, a scatter — per block an LDS
// histogram and one global atomic per bucket it holds) and a segmented
// radix sort orders each bucket (one block per bucket; fewer than rocprim's
// partitioning threshold of 3000 segments, whose size split reads counts
// back to the host).  The requests' buckets are their home slots' top 11
// bits (the slots are hashed: even buckets).  The op list's are bounded by
// splitters — 2048 keys sampled at even strides, sorted in one workgroup —
// found by a binary search in LDS: its ops crowd on hot
// slots (a hot flow's hits, all ordered by one close), and a bucket per top
// bits left one block sorting a million keys (89 ms per step on the
// dependency stream).  All-ones keys are left out and come back all-ones.
constexpr uint32_t BKT_BITS = 11, BKT_N = 1u << BKT_BITS, BKT_CH = 4096, BKT_MIN = 1u << 15;
constexpr uint32_t BKT_SAMPLES = 2048, BKT_PER_SPLIT = BKT_SAMPLES / BKT_N;
struct BktArgs {
    const uint64_t *in;
    uint64_t *out;
    uint32_t n, bits;
    uint32_t *cnt, *begin, *end, *cur;   // [BKT_N + 1] each (the last: padding)
    uint64_t *split;                     // [BKT_N - 1]
};
// the bucket of key k: SPLIT, how many splitters are below it (sp in LDS);
// else its top BKT_BITS of `bits`
template <bool SPLIT>
__device__ __forceinline__ uint32_t bkt_of(const BktArgs &B, const uint64_t *sp, uint64_t k)
{
    if (k == ~0ull)
        return BKT_N;
    if (!SPLIT)
        return (uint32_t)min<uint64_t>(k >> (B.bits - BKT_BITS), BKT_N - 1);
    uint32_t lo = 0, hi = BKT_N - 1;   // (the answer in [lo, hi])
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sp[mid] < k)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}
// one workgroup: the samples sorted (a block radix sort), each after the
// first a splitter
__global__ __launch_bounds__(512) void k_bkt_sample(BktArgs B)
{
    using Sort = hipcub::BlockRadixSort<uint64_t, 512, BKT_SAMPLES / 512>;
    __shared__ typename Sort::TempStorage ts;
    uint64_t v[BKT_SAMPLES / 512];
#pragma unroll
    for (uint32_t q = 0; q < BKT_SAMPLES / 512; q++)
        v[q] = B.in[(uint64_t)(threadIdx.x * (BKT_SAMPLES / 512) + q) * B.n / BKT_SAMPLES];
    Sort(ts).Sort(v, 0, (int)B.bits);   // (all-ones keys: their low bits are all ones, last)
#pragma unroll
    for (uint32_t q = 0; q < BKT_SAMPLES / 512; q++) {
        const uint32_t m = threadIdx.x * (BKT_SAMPLES / 512) + q;   // (blocked: sample m)
        if (m % BKT_PER_SPLIT == 0 && m >= BKT_PER_SPLIT && m / BKT_PER_SPLIT - 1 < BKT_N - 1)
            B.split[m / BKT_PER_SPLIT - 1] = v[q];
    }
}
__device__ __forceinline__ void bkt_load_split(const BktArgs &B, uint64_t *sp)
{
    for (uint32_t j = threadIdx.x; j < BKT_N - 1; j += 256)
        sp[j] = B.split[j];
}
// a block per BKT_CH keys: its LDS histogram, then one atomic per bucket
template <bool SPLIT>
__global__ __launch_bounds__(256) void k_bkt_count(BktArgs B)
{
    __shared__ uint32_t h[BKT_N + 1];
    __shared__ uint64_t sp[SPLIT ? BKT_N - 1 : 1];
    for (uint32_t j = threadIdx.x; j <= BKT_N; j += 256)
        h[j] = 0;
    if (SPLIT)
        bkt_load_split(B, sp);
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * BKT_CH;
    for (uint32_t j = threadIdx.x; j < BKT_CH; j += 256)
        if (base + j < B.n)
            atomicAdd(&h[bkt_of<SPLIT>(B, sp, B.in[base + j])], 1u);
    __syncthreads();
    for (uint32_t j = threadIdx.x; j <= BKT_N; j += 256)
        if (h[j])
            atomicAdd(&B.cnt[j], h[j]);
}
// one block: the buckets' places (the padding's after the last) and the
// scatter's cursors
__global__ __launch_bounds__(1024) void k_bkt_scan(BktArgs B)
{
    __shared__ uint32_t ws[16];
    constexpr uint32_t PER = (BKT_N + 1024) / 1024;   // (BKT_N + 1 bins)
    uint32_t v[PER], t = 0;
#pragma unroll
    for (uint32_t q = 0; q < PER; q++) {
        const uint32_t j = threadIdx.x * PER + q;
        v[q] = j <= BKT_N ? B.cnt[j] : 0u;
        t += v[q];
    }
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t x = t;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d)
            x += y;
    }
    if (lane == 63)
        ws[wv] = x;
    __syncthreads();
    uint32_t off = x - t;
    for (uint32_t k = 0; k < wv; k++)
        off += ws[k];
#pragma unroll
    for (uint32_t q = 0; q < PER; q++) {
        const uint32_t j = threadIdx.x * PER + q;
        if (j <= BKT_N) {
            B.begin[j] = off;
            B.end[j] = off + v[q];
            B.cur[j] = off;
        }
        off += v[q];
    }
}
// a block per BKT_CH keys again: its places taken per bucket by one atomic
template <bool SPLIT>
__global__ __launch_bounds__(256) void k_bkt_scatter(BktArgs B)
{
    __shared__ uint32_t h[BKT_N + 1];
    __shared__ uint64_t sp[SPLIT ? BKT_N - 1 : 1];
    for (uint32_t j = threadIdx.x; j <= BKT_N; j += 256)
        h[j] = 0;
    if (SPLIT)
        bkt_load_split(B, sp);
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * BKT_CH;
    constexpr uint32_t PER = BKT_CH / 256;
    uint64_t k[PER];
    uint32_t b[PER], r[PER];
#pragma unroll
    for (uint32_t q = 0; q < PER; q++) {
        const uint64_t i = base + q * 256 + threadIdx.x;
        k[q] = i < B.n ? B.in[i] : 0ull;
        b[q] = bkt_of<SPLIT>(B, sp, k[q]);
        r[q] = i < B.n ? atomicAdd(&h[b[q]], 1u) : 0u;
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j <= BKT_N; j += 256)
        if (h[j])
            h[j] = atomicAdd(&B.cur[j], h[j]);
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < PER; q++)
        if (base + q * 256 + threadIdx.x < B.n)
            B.out[h[b[q]] + r[q]] = k[q];
}

size_t bkt_scratch_bytes() { return 4ull * 4 * (BKT_N + 1) + 8ull * BKT_N + 512; }

// pad: the list may hold all-ones keys (a list laid out for a bound);
// crowd: its keys may crowd on a few slots (the op list: splitters)
int sort_keys(const CtaArgs &A, uint64_t *keys, uint64_t *alt, uint32_t n, int bits,
              hipStream_t s, uint64_t **sorted, bool pad = true, bool crowd = false)
{
    *sorted = keys;
    if (n < 2)
        return 0;
    if (n >= BKT_MIN && bits > (int)BKT_BITS + 8) {
        // (scratch after the sorts' temporary storage)
        const size_t tb0 = A.sort_tmp_bytes - bkt_scratch_bytes();
        uint32_t *w = reinterpret_cast<uint32_t *>((reinterpret_cast<uintptr_t>(A.sort_tmp) + tb0 + 255) & ~uintptr_t(255));
        uint64_t *sp = reinterpret_cast<uint64_t *>(
            (reinterpret_cast<uintptr_t>(w + 4 * (BKT_N + 1)) + 255) & ~uintptr_t(255));
        BktArgs B{keys, alt, n, (uint32_t)bits, w, w + (BKT_N + 1), w + 2 * (BKT_N + 1),
                  w + 3 * (BKT_N + 1), sp};
        const unsigned g = (unsigned)((n + BKT_CH - 1) / BKT_CH);
        if (hipMemsetAsync(B.cnt, 0, 4 * (BKT_N + 1), s) != hipSuccess)
            return -EIO;
        if (crowd) {
            hipLaunchKernelGGL(k_bkt_sample, dim3(1), dim3(512), 0, s, B);
            hipLaunchKernelGGL(k_bkt_count<true>, dim3(g), dim3(256), 0, s, B);
        } else {
            hipLaunchKernelGGL(k_bkt_count<false>, dim3(g), dim3(256), 0, s, B);
        }
        hipLaunchKernelGGL(k_bkt_scan, dim3(1), dim3(1024), 0, s, B);
        if (crowd)
            hipLaunchKernelGGL(k_bkt_scatter<true>, dim3(g), dim3(256), 0, s, B);
        else
            hipLaunchKernelGGL(k_bkt_scatter<false>, dim3(g), dim3(256), 0, s, B);
        // the padding (all-ones, after the buckets in alt) is no segment:
        // the output holds all-ones where the segments do not write
        size_t tb = tb0;
        if ((pad && hipMemsetAsync(keys, 0xFF, 8ull * n, s) != hipSuccess) ||
            hipcub::DeviceSegmentedRadixSort::SortKeys(A.sort_tmp, tb, (const uint64_t *)alt, keys,
                                                       (int)n, (int)BKT_N, (const uint32_t *)B.begin,
                                                       (const uint32_t *)B.end, 0,
                                                       crowd ? bits : bits - (int)BKT_BITS,
                                                       s) != hipSuccess)
            return -EIO;
        return 0;
    }
    size_t tb = A.sort_tmp_bytes;
    hipcub::DoubleBuffer<uint64_t> db(keys, alt);
    if (hipcub::DeviceRadixSort::SortKeys(A.sort_tmp, tb, db, (int)n, 0, bits, s) !=
        hipSuccess)
        return -EIO;
    *sorted = db.Current();
    return 0;
}

}  // namespace

size_t cta_sort_tmp_bytes(uint32_t n)
{
    size_t tb = 0, ts = 0;
    hipcub::DoubleBuffer<uint64_t> db(nullptr, nullptr);
    (void)hipcub::DeviceRadixSort::SortKeys(nullptr, tb, db, (int)std::max<uint32_t>(n, 2u), 0,
                                            64, (hipStream_t)0);
    (void)hipcub::DeviceSelect::Flagged(nullptr, ts, (const uint64_t *)nullptr,
                                        (const uint8_t *)nullptr, (uint64_t *)nullptr,
                                        (uint32_t *)nullptr, (int)std::max<uint32_t>(n, 2u),
                                        (hipStream_t)0);
    size_t tg = 0;   // (the bucketed sort's segments; its scratch after all three)
    (void)hipcub::DeviceSegmentedRadixSort::SortKeys(
        nullptr, tg, (const uint64_t *)nullptr, (uint64_t *)nullptr, (int)std::max<uint32_t>(n, 2u),
        (int)BKT_N, (const uint32_t *)nullptr, (const uint32_t *)nullptr, 0, 64, (hipStream_t)0);
    return std::max({tb, ts, tg}) + bkt_scratch_bytes();
}

// an egress batch with a load balancer: the service step of every header
// (k_cta_lb) and its replay per CT_SERVICE key in order (k_cta_svc), the
// per-header records (LbRec) the ordering pass and the scan decode
template <bool V6>
int cta_lb_pre_t(const CtaArgs &A, hipStream_t s)
{
    hipLaunchKernelGGL(k_cta_lb<V6>, dim3((unsigned)((A.n + 255) / 256)), dim3(256), 0, s, A);
    uint32_t ns = 0;
    if (hipMemcpyAsync(&ns, A.cnt + CTA_NSVC, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    uint64_t *sorted;
    if (int rc = sort_keys(A, A.reqS, A.reqS2, ns, A.ob + A.slot_bits, s, &sorted, false))
        return rc;
    if (ns)
        hipLaunchKernelGGL(k_cta_svc<V6>, dim3((ns + 255) / 256), dim3(256), 0, s, A, sorted, ns);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

template <bool V6>
int cta_scan_t(const CtaArgs &A, hipStream_t s)
{
    if (A.lbr) {   // (after cta_lb_pre)
        hipLaunchKernelGGL(k_cta_scan_lb<V6>, dim3(blocks_for(A.n, 2048)), dim3(256), 0, s, A);
        return hipGetLastError() == hipSuccess ? 0 : -EIO;
    }
    if (A.sparse) {   // (the launch's work bits; A.ck1 / A.ck2 and A.sum set)
        const unsigned g = A.wl ? 1024u : (unsigned)((A.W.words + 255) / 256);
        if (A.mode == CFC_MODE_EGRESS)
            hipLaunchKernelGGL((k_cta_scan_w<V6, true>), dim3(g), dim3(256), 0, s, A);
        else
            hipLaunchKernelGGL((k_cta_scan_w<V6, false>), dim3(g), dim3(256), 0, s, A);
        return hipGetLastError() == hipSuccess ? 0 : -EIO;
    }
    if (A.mode == CFC_MODE_EGRESS)
        hipLaunchKernelGGL((k_cta_scan<V6, true>), dim3(blocks_for(A.n, 2048)), dim3(256), 0, s, A);
    else
        hipLaunchKernelGGL((k_cta_scan<V6, false>), dim3(blocks_for(A.n, 2048)), dim3(256), 0, s, A);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// The rest of the apply after the host has read the scan's counts (nreqA)
// and allowed the inserts.  Reads two more counts on the way (the sorts
// take host item counts).
template <bool V6>
int cta_newkeys_t(const CtaArgs &A, uint32_t nreqA, uint64_t **sorted, uint32_t *newk,
                  hipStream_t s)
{
    if (int rc = sort_keys(A, A.reqA, A.reqA2, nreqA, A.ob + A.slot_bits, s, sorted, false))
        return rc;
    if (hipMemsetAsync(A.cnt + CTA_NEWK, 0, 8, s) != hipSuccess ||   // (NEWK, NEWKT)
        hipMemsetAsync(A.cx, 0, 8ull * (A.rel_mask + 1), s) != hipSuccess)
        return -EIO;
    if (nreqA)
        hipLaunchKernelGGL(k_cta_newkeys<V6>, dim3((nreqA + 255) / 256), dim3(256), 0, s, A,
                           (const uint64_t *)*sorted, nreqA);
    if (hipMemcpyAsync(newk, A.cnt + CTA_NEWK, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    return 0;
}

template <bool V6>
int cta_rest_t(const CtaArgs &A, uint32_t nreqA, const uint64_t *presorted, uint32_t *host_cnt,
               hipStream_t s, const uint64_t *routed, uint32_t nroute)
{
    const int bits = A.ob + A.slot_bits;
    uint64_t *sorted = const_cast<uint64_t *>(presorted);
    int rc;
    if (!sorted && (rc = sort_keys(A, A.reqA, A.reqA2, nreqA, bits, s, &sorted, false)))
        return rc;
    // the second round's requests (a create's related and reverse-NAT
    // entries) and their ops' places in the list are laid out for the
    // scan's bound — its creates that are not TCP and whose k2 is not a
    // related entry, and those with a reverse-NAT entry — the unused ones
    // all-ones (sorted last, skipped by the insert, dropped by dedup): no
    // wait for their count
    const uint32_t nbB = (uint32_t)std::min<uint64_t>(
        host_cnt ? (uint64_t)host_cnt[CTA_NRELB] + host_cnt[CTA_NKX] : 2ull * nreqA, A.req_cap);
    if (nbB && (hipMemsetAsync(A.reqB, 0xFF, 8ull * nbB, s) != hipSuccess ||
                (uint64_t)nreqA + nbB > A.cx_cap ||
                hipMemsetAsync(A.cx + nreqA, 0xFF, 8ull * nbB, s) != hipSuccess))
        return -EIO;
    if (nreqA) {
        hipLaunchKernelGGL(k_cta_insert<V6>, dim3((nreqA + RQ_B - 1) / RQ_B), dim3(RQ_B), 0, s, A, sorted,
                           nreqA, 0, 0u);
        hipLaunchKernelGGL(k_cta_related<V6>, dim3((nreqA + RQ_B - 1) / RQ_B), dim3(RQ_B), 0, s, A,
                           (const uint64_t *)sorted, nreqA);
    }
    if ((rc = sort_keys(A, A.reqB, A.reqB2, nbB, bits, s, &sorted)))
        return rc;
    if (nbB)
        hipLaunchKernelGGL(k_cta_insert<V6>, dim3((nbB + RQ_B - 1) / RQ_B), dim3(RQ_B), 0, s, A, sorted,
                           nbB, 1, nreqA);
    // the creates' ops take the list's first nreqA + nbB places, route's
    // ordered hits follow
    uint64_t ncx64;
    if (routed) {   // (routed already: its list appended, no wait)
        ncx64 = (uint64_t)nreqA + nbB + nroute;
        if (ncx64 > A.cx_cap)
            return -EOVERFLOW;
        if (nroute && hipMemcpyAsync(A.cx + nreqA + nbB, routed, 8ull * nroute,
                                     hipMemcpyDeviceToDevice, s) != hipSuccess)
            return -EIO;
    } else {
        CtaArgs R = A;
        R.cx_base = nreqA + nbB;
        const uint64_t nk = A.lbr ? 4 * A.n : A.mode == CFC_MODE_EGRESS ? 2 * A.n : A.n;
        hipLaunchKernelGGL(k_cta_route, dim3(blocks_for((nk + RU - 1) / RU, 2048)), dim3(256), 0,
                           s, R);
        if (hipMemcpyAsync(host_cnt, A.cnt, 4 * CTA_NCNT, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -EIO;
        if (host_cnt[CTA_NREQB] > nbB || host_cnt[CTA_NLOG] > A.log_cap)
            return -EOVERFLOW;
        ncx64 = (uint64_t)nreqA + nbB + host_cnt[CTA_NCX];
    }
    if (ncx64 > A.cx_cap)
        return -EOVERFLOW;
    const uint32_t ncx = (uint32_t)ncx64;
    if ((rc = sort_keys(A, A.cx, A.cx2, ncx, bits, s, &sorted, true, true)))
        return rc;
    if (ncx) {
        // drop the repeated plain hits, compact what stays into the other
        // buffer, fold that
        uint64_t *dst = sorted == A.cx ? A.cx2 : A.cx;
        uint8_t *keep = reinterpret_cast<uint8_t *>(A.hs);   // (hit slots: read by route only)
        uint32_t *nsel = A.cnt + CTA_NDEDUP;
        hipLaunchKernelGGL(k_cta_dedup<V6>, dim3((ncx + 255) / 256), dim3(256), 0, s, A,
                           (const uint64_t *)sorted, ncx, keep);
        size_t tb = A.sort_tmp_bytes;
        if (hipcub::DeviceSelect::Flagged(A.sort_tmp, tb, sorted, keep, dst, nsel, (int)ncx, s) !=
            hipSuccess)
            return -EIO;
        // (the pre-dedup list is free now: the long runs' list)
        uint32_t *lng = reinterpret_cast<uint32_t *>(sorted);
        // (the long runs: plan, chunk reductions, final states; fixed
        // grids over device counts)
#define CFC_FOLD(LBV)                                                                          \
        hipLaunchKernelGGL((k_cta_fold<V6, LBV>), dim3((ncx + 255) / 256), dim3(256), 0, s, A, \
                           (const uint64_t *)dst, (const uint32_t *)nsel, lng);                 \
        hipLaunchKernelGGL((k_cta_fold_plan<V6, LBV>), dim3(16), dim3(256), 0, s, A,            \
                           (const uint64_t *)dst, (const uint32_t *)nsel, lng);                 \
        hipLaunchKernelGGL((k_cta_fold_agg<V6, LBV>), dim3(1024), dim3(256), 0, s, A,          \
                           (const uint64_t *)dst, (const uint32_t *)nsel, lng);                 \
        hipLaunchKernelGGL((k_cta_fold_fin<V6, LBV>), dim3(16), dim3(256), 0, s, A,             \
                           (const uint64_t *)dst, (const uint32_t *)nsel, lng)
        if (A.lbr) {
            CFC_FOLD(true);
        } else {
            CFC_FOLD(false);
        }
#undef CFC_FOLD
    }
    // (a sweep of the whole table: a list of the touched slots, A/B'd,
    // took 0.43 ms against the sweep's 0.30 — its random loads cost more
    // than the sequential ones they save)
    hipLaunchKernelGGL(k_cta_finish<V6>, dim3(blocks_for(((uint64_t)A.mask + 1) / 16 + 1, 2048)),
                       dim3(256), 0, s, A);
    if (A.nt && A.mon && A.n)
        hipLaunchKernelGGL(k_cta_mon<V6>, dim3((unsigned)((A.n + 255) / 256)), dim3(256), 0, s, A);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int ct_protect_hits(const uint32_t *hs, uint64_t nk, uint32_t *bm, hipStream_t s)
{
    if (nk)
        hipLaunchKernelGGL(k_ct_protect, dim3((unsigned)((nk + 255) / 256)), dim3(256), 0, s, hs,
                           nk, bm);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int cta_hs_fill(const CtaArgs &A, hipStream_t s)
{
    const uint64_t nk = A.mode == CFC_MODE_EGRESS ? 2 * A.n : A.n;
    if (nk)
        hipLaunchKernelGGL(k_cta_hs_fill, dim3((unsigned)((nk + 255) / 256)), dim3(256), 0, s, A);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int cta_lb_pre(const CtaArgs &A, bool v6, hipStream_t s)
{
    return v6 ? cta_lb_pre_t<true>(A, s) : cta_lb_pre_t<false>(A, s);
}

int cta_scan(const CtaArgs &A, bool v6, hipStream_t s)
{
    return v6 ? cta_scan_t<true>(A, s) : cta_scan_t<false>(A, s);
}

int cta_rest(const CtaArgs &A, bool v6, uint32_t nreqA, const uint64_t *presorted,
             uint32_t *host_cnt, hipStream_t s, const uint64_t *routed, uint32_t nroute)
{
    return v6 ? cta_rest_t<true>(A, nreqA, presorted, host_cnt, s, routed, nroute)
              : cta_rest_t<false>(A, nreqA, presorted, host_cnt, s, routed, nroute);
}

int cta_route(const CtaArgs &A, hipStream_t s)
{
    const uint64_t nk = A.lbr ? 4 * A.n : A.mode == CFC_MODE_EGRESS ? 2 * A.n : A.n;
    hipLaunchKernelGGL(k_cta_route, dim3(blocks_for((nk + RU - 1) / RU, 2048)), dim3(256), 0, s, A);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int cta_newkeys(const CtaArgs &A, bool v6, uint32_t nreqA, uint64_t **sorted, uint32_t *newk,
                hipStream_t s)
{
    return v6 ? cta_newkeys_t<true>(A, nreqA, sorted, newk, s)
              : cta_newkeys_t<false>(A, nreqA, sorted, newk, s);
}

int cta_collect(const Ct4Slot *ct4, CtState *st, const uint4 *lb, uint64_t slots,
                CtSyncRec *out, uint32_t cap, uint32_t *cnt, hipStream_t s)
{
    hipLaunchKernelGGL(k_cta_collect<false>, dim3(blocks_for(slots, 8192)), dim3(256), 0, s, ct4,
                       st, lb, slots, out, cap, cnt);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int cta_collect6(const Ct6Slot *ct6, CtState *st, const uint4 *lb, uint64_t slots,
                 CtSyncRec6 *out, uint32_t cap, uint32_t *cnt, hipStream_t s)
{
    hipLaunchKernelGGL(k_cta_collect<true>, dim3(blocks_for(slots, 8192)), dim3(256), 0, s, ct6,
                       st, lb, slots, out, cap, cnt);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int ct_gc4(const CtGcArgs &A, hipStream_t s)
{
    if (!A.slots || A.n_maps > CTG_MAX_MAPS)
        return -EINVAL;
    const dim3 g((unsigned)std::max<uint64_t>(
        1, std::min<uint64_t>((A.slots + GC_B * GC_U - 1) / (GC_B * GC_U), 256)));
    if (A.ct6)
        hipLaunchKernelGGL(k_ct_gc<true>, g, dim3(GC_B), 0, s, A);
    else
        hipLaunchKernelGGL(k_ct_gc<false>, g, dim3(GC_B), 0, s, A);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int ct_gc_log(const CtGcArgs &A, const CtLog *in, uint32_t n, CtLog *out, hipStream_t s)
{
    if (A.n_maps > CTG_MAX_MAPS)
        return -EINVAL;
    if (n)
        hipLaunchKernelGGL(k_ct_gc_log<CtLog>, dim3((n + 255) / 256), dim3(256), 0, s, A, in, n,
                           out);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int ct_gc_log6(const CtGcArgs &A, const CtLog6 *in, uint32_t n, CtLog6 *out, hipStream_t s)
{
    if (A.n_maps > CTG_MAX_MAPS)
        return -EINVAL;
    if (n)
        hipLaunchKernelGGL(k_ct_gc_log<CtLog6>, dim3((n + 255) / 256), dim3(256), 0, s, A, in, n,
                           out);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int ct_count_nonfree6(const Ct6Slot *ct6, uint64_t slots, uint32_t *cnt, hipStream_t s)
{
    if (slots)
        hipLaunchKernelGGL(k_ct_nonfree<Ct6Slot>, dim3(blocks_for(slots, 2048)), dim3(256), 0, s,
                           ct6, slots, cnt);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int ct_count_nonfree4(const Ct4Slot *ct4, uint64_t slots, uint32_t *cnt, hipStream_t s)
{
    if (slots)
        hipLaunchKernelGGL(k_ct_nonfree<Ct4Slot>, dim3(blocks_for(slots, 2048)), dim3(256), 0, s, ct4,
                           slots, cnt);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int ct_rehash(bool v6, const void *ok, const CtState *ost, const uint4 *olb, uint64_t oslots,
              void *nk, CtState *nst, uint4 *nlb, uint32_t nmask, uint32_t *map, uint32_t *cnt,
              hipStream_t s)
{
    if (v6)
        hipLaunchKernelGGL(k_ct_rehash<true>, dim3(blocks_for(oslots, 8192)), dim3(256), 0, s,
                           (const Ct6Slot *)ok, ost, olb, oslots, (Ct6Slot *)nk, nst, nlb, nmask,
                           map, cnt);
    else
        hipLaunchKernelGGL(k_ct_rehash<false>, dim3(blocks_for(oslots, 8192)), dim3(256), 0, s,
                           (const Ct4Slot *)ok, ost, olb, oslots, (Ct4Slot *)nk, nst, nlb, nmask,
                           map, cnt);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int ct_remap(uint32_t *slot, uint64_t n, uint32_t stride, const uint32_t *map, hipStream_t s)
{
    if (n)
        hipLaunchKernelGGL(k_ct_remap, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, slot, n,
                           stride, map);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int ct_state_init(CtState *st, const CtTimer *tm, uint64_t n, hipStream_t s)
{
    if (n)
        hipLaunchKernelGGL(k_ct_st_init, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, st,
                           tm, n);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int ct_acct_take(CtState *st, uint64_t *out, uint64_t n, hipStream_t s)
{
    if (n)
        hipLaunchKernelGGL(k_ct_acct_take, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, st,
                           reinterpret_cast<ulonglong2 *>(out), n);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int cta_tomb(Ct4Slot *ct4, const CtSyncRec *rec, uint32_t n, hipStream_t s)
{
    if (n)
        hipLaunchKernelGGL(k_cta_tomb, dim3((n + 255) / 256), dim3(256), 0, s, ct4, rec, n);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int cta_tomb6(Ct6Slot *ct6, const CtSyncRec6 *rec, uint32_t n, hipStream_t s)
{
    if (n)
        hipLaunchKernelGGL(k_cta_tomb6, dim3((n + 255) / 256), dim3(256), 0, s, ct6, rec, n);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

}  // namespace cfc
