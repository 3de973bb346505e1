// Packet-order CT results of one classified batch (cfc_ct_apply, before the
// apply proper).
//
// The classify launch looks every header's CT stages up against the CT maps
// as the batch found them.  The reference runs the batch one packet at a
// time: each packet's ct_lookup sees the ct_create / ct_delete of the packets
// before it (conntrack.h:221-285 __ct_lookup, :615-772 ct_create6/4,
// bpf_lxc.c:963-970 / :538-545 the delete of a denied established flow).
// This pass turns the launch's batch-start results into the reference's.
//
// Which results can differ.  A stage looks up k1 (the tuple as loaded:
// TUPLE_F_OUT for ingress, TUPLE_F_IN for egress; a hit is CT_REPLY /
// CT_RELATED) and then k2 (its reverse, the flag flipped; a hit is
// CT_ESTABLISHED, a miss CT_NEW).  Every write a stage makes has k2's flag:
// ct_create writes k2 and its ICMP "related" entry (k2's flags |
// TUPLE_F_RELATED), ct_delete removes k2.  A batch runs one direction (an
// ingress program, or one endpoint's egress and the local delivery behind
// it), so no write of the batch has a k1 flag: k1's existence — and with it
// every CT_REPLY / CT_RELATED result — is the batch start's.  (A load
// balancer's looped-back flow writes a TUPLE_F_IN entry, ct_create4 with
// ct_state->addr, :731-739; that case stays with the launch's view.)  What
// the order decides is k2's existence, hence CT_NEW vs CT_ESTABLISHED; and
// those two give the same policy key (the tuple is reversed either way,
// :581), so the same verdict, counters and drop decision.  What changes is
// the CT byte (result, create), the trace reason and monitor length, and
// the writes: a later packet of a flow the batch created is ESTABLISHED (no
// second create), a packet after a delete is NEW (a create when allowed).
//
// The state machine per k2 key.  Each stage on the key is a lookup and then
// one write decided by its (order-independent) verdict: allowed, the key
// exists afterwards (created if it was NEW); dropped (DROP_POLICY at the
// header's last stage), it does not (deleted if it was ESTABLISHED).  So
// the state a stage sees is the previous stage's outcome on the same key,
// or the batch start's existence for the first.  The participants: every
// CT_NEW stage (its key may have been created earlier), every
// CT_ESTABLISHED stage that deletes, and — when the batch deletes — every
// CT_ESTABLISHED stage on a deleted slot.  (An ESTABLISHED stage on a key
// nobody deletes sees it exist throughout.)  Sorted by (key, header order),
// each participant's result is its predecessor's outcome: one sort, one
// neighbour compare.  Related entries are a second round: a UDP / ICMP
// create (the ANY map; a TCP map's related entry is unreachable) writes
// one, which an ICMP error's k2 lookup may find.
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ctops.hpp"

namespace cfc {

namespace {

// participant info bits
constexpr uint8_t PI_START = 1;    // k2 existed when the batch started (ESTABLISHED)
constexpr uint8_t PI_POST = 2;     // the key exists after this stage (allowed)
constexpr uint8_t PI_REL = 4;      // a related-entry write (round 2), not a lookup
constexpr uint8_t PI_MKREL = 8;    // a create whose related entry is in the device table
constexpr uint8_t PI_RELKEY = 16;  // the stage's k2 has TUPLE_F_RELATED (an ICMP error)

// a 64-bit key fingerprint (two independent 32-bit hashes)
__device__ __forceinline__ uint64_t fp64(uint32_t d, uint32_t s, uint32_t z, uint32_t w)
{
    return (uint64_t)ct_hash4(d, s, z, w) << 32 | ct_hash4(w ^ 0x27d4eb2fu, z, s, d);
}
__device__ __forceinline__ uint64_t fp64(uint4 d, uint4 s, uint32_t z, uint32_t w)
{
    const uint32_t a = ct_hash4(d.x, d.y, d.z, d.w), b = ct_hash4(s.x, s.y, s.z, s.w);
    return (uint64_t)ct_hash4(a, b, z, w) << 32 | ct_hash4(w ^ 0x27d4eb2fu, z, b, a);
}

// a CT_ESTABLISHED stage's k2 slot at the batch's start: the classify
// launch's hit, or (its keys gone) a probe
template <bool V6>
__device__ __forceinline__ uint32_t start_slot(const CtaArgs &A, const OrdArgs &O, uint64_t i,
                                               int st)
{
    const uint32_t *ck = st ? O.ck2 : O.ck1;
    if (ck) {
        const uint32_t k = ck[i];
        return k >= CK_MISS ? NONE : (k >> 1) - A.acct_base;
    }
    const Op<V6> o = decode<V6>(A, i, st);
    return find(A, o.sa, o.da, o.z2, o.w2);
}

// ---- which stages take part.  Per k2 key the state is a chain of its
// stages in packet order, but most keys need no sort:
//   * a key no stage of the batch writes keeps its batch-start existence:
//     a dropped CT_NEW stage (no create) matters only when some allowed
//     CT_NEW stage of the batch creates its key (the creates' pre-keys in
//     a Bloom filter, k_ord_mark: a false positive only adds a
//     participant), or when its key is an ICMP error's (a related entry a
//     create may write: round 2), or with a load balancer (every one);
//   * a key the batch only deletes (every stage on its slot a denied
//     CT_ESTABLISHED: the common case, one verdict per flow) ends with its
//     first delete in packet order; the later stages see it gone: CT_NEW,
//     no create (k_ord_deltail, from each slot's first delete order D);
//   * a deleted slot that also has an allowed CT_ESTABLISHED stage (a
//     "mixed" slot: the verdict differs between packets of one key, e.g.
//     fragments) goes through the sort with all its stages.
// Participants of the sort: every allowed CT_NEW stage, dropped CT_NEW
// stages whose key a create writes (or an ICMP error's), and the stages of
// mixed slots.

// A stage's pre-key: a hash of its k2 without the owner word (the CT map),
// so without the destination-endpoint lookup a full decode needs: the raw
// addresses and ct_probe's L4 word and flags for the stage's direction.
// Equal k2 keys give equal pre-keys (outside a load balancer's service
// step, which this is not used with); equal pre-keys of different keys only
// add participants.
template <bool V6>
struct PreIn {   // the fields a pre-key derives from
    Addr<V6> sa, da;
    uint32_t pt, mt;
};
template <bool V6>
__device__ __forceinline__ PreIn<V6> pre_in(const CtaArgs &A, uint64_t i)
{
    return PreIn<V6>{ld_addr<V6>(A.sa, i), ld_addr<V6>(A.da, i), A.pt[i], A.mt[i]};
}
template <bool V6>
__device__ __forceinline__ uint64_t prekey_of(const CtaArgs &A, const PreIn<V6> &f, int st)
{
    const int dir = (A.mode == CFC_MODE_EGRESS && st == 0) ? CT_EGRESS : CT_INGRESS;
    const CtProbe k = ct_probe<V6>(f.mt & 0xFF, f.pt, dir, 0);
    uint32_t a, b;
    if constexpr (V6) {
        a = ct_hash4(f.sa.x, f.sa.y, f.sa.z, f.sa.w);
        b = ct_hash4(f.da.x, f.da.y, f.da.z, f.da.w);
    } else {
        a = f.sa;
        b = f.da;
    }
    return (uint64_t)ct_hash4(a, b, k.z2, k.w2) << 32 | ct_hash4(k.w2 ^ 0x27d4eb2fu, k.z2, b, a);
}
template <bool V6>
__device__ __forceinline__ uint64_t prekey(const CtaArgs &A, uint64_t i, int st)
{
    return prekey_of<V6>(A, pre_in<V6>(A, i), st);
}
// an ICMP error's lookup (its k2 carries TUPLE_F_RELATED): types 3, 11, 12
// (IPv4) / 1-4 (IPv6), ct_lookup4/6
template <bool V6>
__device__ __forceinline__ bool icmp_error(uint32_t mt, uint32_t pt)
{
    const uint32_t proto = mt & 0xFF, type = pt & 0xFF;
    if (V6)
        return proto == 58 && type >= 1 && type <= 4;
    return proto == 1 && (type == 3 || type == 11 || type == 12);
}
// the creates' pre-keys: a blocked Bloom filter (one word, three bits)
__device__ __forceinline__ void cb_put(const OrdArgs &O, uint64_t h)
{
    uint32_t *wp = O.cbloom + ((uint32_t)(h >> 32) & O.cb_mask);
    const uint32_t b = bloom_bits((uint32_t)h);
    if ((*wp & b) != b)
        atomicOr(wp, b);
}
__device__ __forceinline__ bool cb_maybe(const OrdArgs &O, uint64_t h)
{
    const uint32_t b = bloom_bits((uint32_t)h);
    return (O.cbloom[(uint32_t)(h >> 32) & O.cb_mask] & b) == b;
}
// a miss tag (kern_common.hpp ck_miss_tag) as a filter key
__device__ __forceinline__ uint64_t tag_key(uint32_t t)
{
    return (uint64_t)fmix32(t) << 32 | (t * 0x9E3779B1u);
}
__device__ __forceinline__ bool tag_ok(uint32_t t) { return t >= CK_MISS && t != NONE; }
constexpr int ORD_IT = 16;   // headers per thread and step (mark, collect)
// The two passes over the whole batch (mark, collect) take ORD_IT
// consecutive headers per thread and step: their CT bytes (one 16-byte
// load) and verdicts (four) loaded together without branches (one wait;
// byte loads were the pass's limit: one instruction per 64 bytes), a cheap
// unrolled pass that
// sorts the stages into bit masks (bit NST * k + st), then the rare stages
// that need more (a key, a probe) in a loop that is not unrolled — with the
// key derivation inlined once the kernel stays small enough for the
// instruction cache.
template <bool TWO>
struct OrdStep {
    static constexpr int NST = TWO ? 2 : 1;
    uint32_t cb[ORD_IT];
    int32_t ver[ORD_IT];
    // header k of this thread's run at base (base: a multiple of 256 * ORD_IT)
    __device__ __forceinline__ static uint64_t at(uint64_t base, int k)
    {
        return base + (uint64_t)ORD_IT * threadIdx.x + (uint64_t)k;
    }
    // vec: ctb and ver 16-byte aligned (OrdArgs.vec)
    __device__ __forceinline__ void load(const CtaArgs &A, uint64_t base, bool vec)
    {
        const uint64_t i0 = at(base, 0);
        if (vec && i0 + ORD_IT <= A.n) {
            const uint4 c = *reinterpret_cast<const uint4 *>(A.ctb + i0);
            const uint4 *vp = reinterpret_cast<const uint4 *>(A.ver + i0);
            const uint4 v0 = vp[0], v1 = vp[1], v2 = vp[2], v3 = vp[3];
            const uint32_t cw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
            for (int k = 0; k < ORD_IT; k++)
                cb[k] = (cw[k / 4] >> (8 * (k % 4))) & 0xFFu;
            const uint4 vv[4] = {v0, v1, v2, v3};
#pragma unroll
            for (int q = 0; q < 4; q++) {
                ver[4 * q] = (int32_t)vv[q].x;
                ver[4 * q + 1] = (int32_t)vv[q].y;
                ver[4 * q + 2] = (int32_t)vv[q].z;
                ver[4 * q + 3] = (int32_t)vv[q].w;
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < ORD_IT; k++) {
            const uint64_t i = i0 + k;
            const uint64_t j = i < A.n ? i : A.n - 1;
            cb[k] = A.ctb[j];
            ver[k] = A.ver[j];
        }
#pragma unroll
        for (int k = 0; k < ORD_IT; k++)
            if (i0 + k >= A.n)
                cb[k] = 0;
    }
    // res: the stage's CT result, or -1 (no CT stage)
    __device__ __forceinline__ int res(int k, int st, bool &dropped) const
    {
        const uint32_t cs = (cb[k] >> (4 * st)) & 0xF;
        const int last = (cb[k] & (CFC_CT_DONE << 4)) ? 1 : 0;
        dropped = st == last && ver[k] == DROP_POLICY;
        return (cs & CFC_CT_DONE) ? (int)(cs & CFC_CT_RES_MASK) : -1;
    }
    __device__ __forceinline__ static uint64_t hdr(uint64_t base, int b)
    {
        return at(base, b / NST);
    }
};

// mark: creates and deletes counted; the creates' pre-keys into the Bloom
// filter; per deleted slot its bit and its first delete's order (read
// first: a hot flow's packets find them set)
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_ord_mark(CtaArgs A, OrdArgs O)
{
    using S = OrdStep<TWO>;
    constexpr int NST = S::NST;
    const uint64_t span = 256ull * ORD_IT, stride = (uint64_t)gridDim.x * span;
    uint32_t ncr = 0, ndel = 0, nnd = 0, nest = 0, ndt = 0, nun = 0, nrk = 0;
    for (uint64_t base = (uint64_t)blockIdx.x * span; base < A.n; base += stride) {
        S x;
        x.load(A, base, O.vec);
        uint32_t crm = 0, delm = 0;
#pragma unroll
        for (int k = 0; k < ORD_IT; k++)
#pragma unroll
            for (int st = 0; st < NST; st++) {
                bool dropped;
                const int r = x.res(k, st, dropped);
                const uint32_t bit = 1u << (NST * k + st);
                if (r == CT_NEW) {
                    nnd += dropped;
                    crm |= dropped ? 0u : bit;
                } else if (r == CT_ESTABLISHED) {
                    nest++;
                    delm |= dropped ? bit : 0u;
                }
            }
        ncr += __popc(crm);
        ndt += __popc(delm);
        if (O.cbloom && O.tagged) {
            // the creates' miss tags, loaded together (predicated: creates
            // are sparse), then into the filter
            uint32_t tg[ORD_IT * NST];
#pragma unroll
            for (int q = 0; q < ORD_IT * NST; q++) {
                tg[q] = NONE;
                if ((crm >> q) & 1)
                    tg[q] = ((q % NST) ? O.ck2 : O.ck1)[S::hdr(base, q)];
            }
            // (the inserts need no answer: no wait on them)
#pragma unroll
            for (int q = 0; q < ORD_IT * NST; q++)
                if ((crm >> q) & 1) {
                    if (tag_ok(tg[q])) {
                        const uint64_t hk = tag_key(tg[q]);
                        atomicOr(O.cbloom + ((uint32_t)(hk >> 32) & O.cb_mask),
                                 bloom_bits((uint32_t)hk));
                        nrk += tg[q] & 1u;
                    } else {
                        nun++;
                    }
                }
        }
        // else the creates' pre-keys, per chunk of PK headers with their
        // fields loaded together (as k_ord_collect's probes)
        constexpr int PK = V6 ? 8 : 16;
#pragma unroll
        for (int c = 0; c < ORD_IT && !O.tagged; c += PK) {
            const uint32_t cm = (uint32_t)(((1ull << (NST * PK)) - 1u) << (NST * c));
            if (!O.cbloom || !__any(crm & cm))   // (wave-uniform)
                continue;
            PreIn<V6> f[PK];
#pragma unroll
            for (int k = 0; k < PK; k++) {
                const uint64_t i = S::at(base, c + k);
                f[k] = pre_in<V6>(A, i < A.n ? i : A.n - 1);
            }
#pragma unroll
            for (int q = 0; q < PK * NST; q++)
                if ((crm >> (NST * c + q)) & 1)
                    cb_put(O, prekey_of<V6>(A, f[q / NST], q % NST));
        }
        for (uint32_t m = delm; m; m &= m - 1) {
            const int b = __ffs(m) - 1, st = b % NST;
            const uint64_t i = S::hdr(base, b);
            const uint32_t sl = start_slot<V6>(A, O, i, st);
            if (sl == NONE)
                continue;
            const uint32_t bb = 1u << (sl & 31), ord = (uint32_t)(i << 1) | (uint32_t)st;
            if (!(O.delbm[sl >> 5] & bb))
                atomicOr(&O.delbm[sl >> 5], bb);
            if (ord < O.dfirst[sl])
                atomicMin(&O.dfirst[sl], ord);
            ndel++;
        }
    }
    block_add(&O.cnt[ORD_NCREATE], ncr);
    block_add(&O.cnt[ORD_NDEL], ndel);
    block_add(&O.cnt[ORD_NNEWDROP], nnd);
    block_add(&O.cnt[ORD_NEST], nest);
    block_add(&O.cnt[ORD_NESTDROP], ndt);
    block_add(&O.cnt[ORD_UNTAGGED], nun);
    block_add(&O.cnt[ORD_RELBOUND], nrk);
}

// mixed: a deleted slot with an allowed CT_ESTABLISHED stage
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_ord_mixed(CtaArgs A, OrdArgs O)
{
    constexpr int NST = TWO ? 2 : 1;
    if (!O.cnt[ORD_NDEL])   // (the sparse passes launch it before their count)
        return;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < A.n;
         i += (uint64_t)gridDim.x * 256) {
        const uint32_t cb = A.ctb[i];
        const int last = (cb & (CFC_CT_DONE << 4)) ? 1 : 0;
#pragma unroll
        for (int st = 0; st < NST; st++) {
            const uint32_t cs = (cb >> (4 * st)) & 0xF;
            if (!(cs & CFC_CT_DONE) || (cs & CFC_CT_RES_MASK) != CT_ESTABLISHED ||
                (st == last && A.ver[i] == DROP_POLICY))
                continue;
            const uint32_t sl = start_slot<V6>(A, O, i, st);
            const uint32_t b = 1u << (sl & 31);
            if (sl != NONE && (O.delbm[sl >> 5] & b) && !(O.mixbm[sl >> 5] & b) &&
                !(atomicOr(&O.mixbm[sl >> 5], b) & b))
                atomicAdd(&O.cnt[ORD_NMIX], 1u);   // (rare: a slot's first)
        }
    }
}

// collect the participants (header << 1 | stage) into O.part: a block's one
// atomic on the list's length covers 256 * ORD_IT headers (a counter every
// block of a 64M-header pass bumps serialises at its L2 channel)
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_ord_collect(CtaArgs A, OrdArgs O)
{
    using S = OrdStep<TWO>;
    constexpr int NST = S::NST;
    const uint64_t span = 256ull * ORD_IT, stride = (uint64_t)gridDim.x * span;
    uint32_t nrk = 0;   // ICMP errors' stages taking part (round 2's bound)
    // (every thread runs the same number of steps: block_count_n)
    for (uint64_t base = (uint64_t)blockIdx.x * span; base < A.n; base += stride) {
        S x;
        x.load(A, base, O.vec);
        uint32_t bits = 0, probe = 0, estm = 0;
#pragma unroll
        for (int k = 0; k < ORD_IT; k++)
#pragma unroll
            for (int st = 0; st < NST; st++) {
                bool dropped;
                const int r = x.res(k, st, dropped);
                const uint32_t bit = 1u << (NST * k + st);
                if (r == CT_NEW) {
                    // (with a service step every dropped CT_NEW stage takes part)
                    if (!dropped || A.lbr)
                        bits |= bit;
                    else
                        probe |= bit;
                } else if (r == CT_ESTABLISHED) {
                    estm |= bit;
                }
            }
        // the probes (a quarter to a half of a policy-heavy batch's headers
        // are dropped CT_NEW stages): with miss tags, the tags and then their
        // filter words loaded together — two waits per step
        if (O.tagged) {
            uint32_t tg[ORD_IT * NST], fw[ORD_IT * NST];
            const uint64_t i0 = S::at(base, 0);
            if (O.vec && i0 + ORD_IT <= A.n) {
                // (dense: every tag of the run, 16-byte loads)
#pragma unroll
                for (int st = 0; st < NST; st++) {
                    const uint4 *kp = reinterpret_cast<const uint4 *>((st ? O.ck2 : O.ck1) + i0);
#pragma unroll
                    for (int q = 0; q < ORD_IT / 4; q++) {
                        const uint4 t4 = probe ? kp[q] : make_uint4(NONE, NONE, NONE, NONE);
                        tg[NST * (4 * q) + st] = t4.x;
                        tg[NST * (4 * q + 1) + st] = t4.y;
                        tg[NST * (4 * q + 2) + st] = t4.z;
                        tg[NST * (4 * q + 3) + st] = t4.w;
                    }
                }
            } else {
#pragma unroll
                for (int q = 0; q < ORD_IT * NST; q++) {
                    tg[q] = NONE;
                    if ((probe >> q) & 1)
                        tg[q] = ((q % NST) ? O.ck2 : O.ck1)[S::hdr(base, q)];
                }
            }
#pragma unroll
            for (int q = 0; q < ORD_IT * NST; q++) {
                fw[q] = 0;
                if (((probe >> q) & 1) && O.cbloom && tag_ok(tg[q]))
                    fw[q] = O.cbloom[(uint32_t)(tag_key(tg[q]) >> 32) & O.cb_mask];
            }
#pragma unroll
            for (int q = 0; q < ORD_IT * NST; q++) {
                // (an untagged stage, an ICMP error's, or a possible create's key)
                const uint32_t fb = bloom_bits((uint32_t)tag_key(tg[q]));
                if (((probe >> q) & 1) &&
                    (!tag_ok(tg[q]) || (tg[q] & 1) || (O.cbloom && (fw[q] & fb) == fb)))
                    bits |= 1u << q;
                nrk += ((probe >> q) & 1) && tag_ok(tg[q]) && (tg[q] & 1);
            }
        }
        // else per chunk of PK headers their fields loaded together (clamped,
        // no branches), then their filter words together — two waits per
        // chunk rather than two per probe
        constexpr int PK = V6 ? 8 : 16;
#pragma unroll
        for (int c = 0; c < ORD_IT && !O.tagged; c += PK) {
            const uint32_t cm = (uint32_t)(((1ull << (NST * PK)) - 1u) << (NST * c));
            if (!__any(probe & cm))   // (wave-uniform)
                continue;
            PreIn<V6> f[PK];
#pragma unroll
            for (int k = 0; k < PK; k++) {
                const uint64_t i = S::at(base, c + k);
                f[k] = pre_in<V6>(A, i < A.n ? i : A.n - 1);
            }
            uint64_t hk[PK * NST];
            bool ie[PK];
#pragma unroll
            for (int k = 0; k < PK; k++) {
                ie[k] = icmp_error<V6>(f[k].mt, f[k].pt);
#pragma unroll
                for (int st = 0; st < NST; st++)
                    hk[NST * k + st] = prekey_of<V6>(A, f[k], st);
            }
            uint32_t fw[PK * NST];
#pragma unroll
            for (int q = 0; q < PK * NST; q++)
                fw[q] = O.cbloom ? O.cbloom[(uint32_t)(hk[q] >> 32) & O.cb_mask] : 0u;
#pragma unroll
            for (int q = 0; q < PK * NST; q++) {
                const int b = NST * c + q;
                const uint32_t fb = bloom_bits((uint32_t)hk[q]);
                if (((probe >> b) & 1) && (ie[q / NST] || (O.cbloom && (fw[q] & fb) == fb)))
                    bits |= 1u << b;
            }
        }
        if (O.ndel)
            for (uint32_t m = estm; m; m &= m - 1) {
                const int b = __ffs(m) - 1;
                const uint32_t sl = start_slot<V6>(A, O, S::hdr(base, b), b % NST);
                if (sl != NONE && ((O.mixbm[sl >> 5] >> (sl & 31)) & 1))
                    bits |= 1u << b;
            }
        uint32_t r = block_count_n(&O.cnt[ORD_NPART], (uint32_t)__popc(bits));
        for (uint32_t m = bits; m; m &= m - 1) {
            const int b = __ffs(m) - 1;
            if (r < O.part_cap)
                O.part[r] = (uint32_t)(S::hdr(base, b) << 1) | (uint32_t)(b % NST);
            r++;
        }
    }
    block_add(&O.cnt[ORD_RELBOUND], nrk);
}

// ---- the same two passes over the classify launch's work bits (O.W,
// kern_common.hpp wl_want) instead of the whole batch: one thread per word
// of 64 headers.  Every create, every deleting stage and every ICMP error's
// stage is a work bit; a dropped CT_NEW stage of another kind is a probe
// bit.  An ESTABLISHED stage outside them is a plain hit, which takes part
// only on a mixed slot: a batch with deletes finds those by two passes over
// the batch (k_ord_mixed, k_ord_collect_mix), and k_ord_write adds a plain
// hit it changes to the work bits and list (the apply's sparse scan then
// sees its create).  ORD_NEST counts the work bits' stages alone.

// a dropped CT_NEW stage that is a probe (its header's probe bit): a key
// tag that is not an ICMP error's
__device__ __forceinline__ bool probe_tag(uint32_t tg) { return tag_ok(tg) && !(tg & 1); }

// The sparse pass takes part only the stages whose key another stage of the
// batch may share — the chains; a key with one stage keeps its batch-start
// existence, so its result stands.  Key tags (CK_MISS | a 29-bit hash, bit
// 0 TUPLE_F_RELATED, bit 1 clear) go into two open-addressing sets of
// cb_mask + 1 words each (O.cbloom).  The main set holds the creates' k2
// tags: a second put of a tag marks it shared (bit 1), and a dropped CT_NEW
// stage (a probe) that finds its tag there shares it and takes part.  The
// related set holds the related-form keys: every ICMP error's k2 (bit 0 of
// the entry: an error's) and every UDP / ICMP create's related entry (the
// key an ICMP error's k2 lookup finds, ct_create4/6's second write); an
// entry an error and another stage put is shared.  Collect then takes the
// creates and ICMP errors whose entries are shared.  Equal tags of
// different keys only add participants (the sort compares the keys).
constexpr uint32_t SET_SHARED = 2u, SET_ERR = 1u, SET_PROBES = 64;
// main set: returns false on a full run (ORD_SETFULL)
__device__ __forceinline__ bool set_put(uint32_t *set, uint32_t mask, uint32_t tg)
{
    uint32_t sl = fmix32(tg) & mask;
    for (uint32_t p = 0; p < SET_PROBES; p++, sl = (sl + 1) & mask) {
        // (the CAS straight away: a first load would add a round trip to
        // the usual empty slot)
        const uint32_t cur = atomicCAS(&set[sl], 0u, tg);
        if (cur == 0)
            return true;
        if ((cur & ~SET_SHARED) == tg) {
            if (!(cur & SET_SHARED))
                atomicOr(&set[sl], SET_SHARED);
            return true;
        }
    }
    return false;
}
// related set: err — an ICMP error's k2 (else a create's related entry)
__device__ __forceinline__ bool rel_put(uint32_t *set, uint32_t mask, uint32_t tg, bool err)
{
    const uint32_t k = tg & ~3u, mine = err ? SET_ERR : 0u;
    uint32_t sl = fmix32(k) & mask;
    for (uint32_t p = 0; p < SET_PROBES; p++, sl = (sl + 1) & mask) {
        const uint32_t cur = atomicCAS(&set[sl], 0u, k | mine);
        if (cur == 0)
            return true;
        if ((cur & ~3u) == k) {
            // another stage put it first: shared when an error is one of them
            if (err || (cur & SET_ERR)) {
                if ((cur & (SET_SHARED | mine)) != (SET_SHARED | mine))
                    atomicOr(&set[sl], SET_SHARED | mine);
            } else if (!(cur & SET_ERR)) {
                // (a second create: shared should an error come later —
                // the error sees the entry there and shares it)
            }
            return true;
        }
    }
    return false;
}
// the entry of a tag (its slot), or NONE; cmp: the bits compared
__device__ __forceinline__ uint32_t set_find(const uint32_t *set, uint32_t mask, uint32_t k,
                                             uint32_t cmp, uint32_t &cur)
{
    uint32_t sl = fmix32(k) & mask;
    for (uint32_t p = 0; p < SET_PROBES; p++, sl = (sl + 1) & mask) {
        cur = set[sl];
        if (cur == 0)
            return NONE;
        if ((cur & cmp) == k)
            return sl;
    }
    return NONE;
}
__device__ __forceinline__ bool main_shared(const OrdArgs &O, uint32_t tg)
{
    uint32_t cur;
    return set_find(O.cbloom, O.cb_mask, tg, ~SET_SHARED, cur) != NONE && (cur & SET_SHARED);
}
__device__ __forceinline__ bool rel_shared(const OrdArgs &O, uint32_t tg)
{
    uint32_t cur;
    return set_find(O.cbloom + O.cb_mask + 1, O.cb_mask, tg & ~3u, ~3u, cur) != NONE &&
           (cur & SET_SHARED);
}
// a UDP / ICMP create's related-entry tag (its k2's addresses, ports 0, the
// ICMP protocol, k2's flags | TUPLE_F_RELATED: ck_miss4 / ck_miss6 of that
// key), or 0 when it writes none (TCP: the TCP map's, which no lookup
// reaches; a k2 of ICMP-error form is its own)
template <bool V6>
__device__ __forceinline__ uint32_t rel_tag(const CtaArgs &A, uint64_t i, int st)
{
    const Op<V6> o = decode<V6>(A, i, st);
    if (o.kind != OP_CREATE || o.is_tcp || o.ki_form)
        return 0;
    const uint32_t rw = ct_word(icmp_proto<V6>(), ((o.w2 >> 8) & 7) | 2u, o.owner);
    if constexpr (V6)
        return ck_miss_tag(ct_hash4(ct_hash4(o.sa.x, o.sa.y, o.sa.z, o.sa.w),
                                    ct_hash4(o.da.x, o.da.y, o.da.z, o.da.w), 0u, rw), rw);
    else
        return ck_miss_tag(ct_hash4(o.sa, o.da, 0u, rw), rw);
}

// the work bits as a list of header indices (in any order — the sets, the
// delete marks and the participants' list are order-free), and the probe
// bits' count.  A block per 1024 words (one atomic per block and counter:
// same-address atomics serialise): a thread per four words counts, then
// each wave writes 256 words' indices, a lane per bit, at consecutive
// positions.
constexpr uint32_t LISTW = 1024;
__global__ __launch_bounds__(256) void k_ord_list_w(OrdArgs O)
{
    __shared__ uint64_t s_b[LISTW];
    __shared__ uint32_t s_r[LISTW];
    const uint64_t w0 = (uint64_t)blockIdx.x * LISTW;
    uint32_t c = 0, np = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint64_t w = w0 + 4 * threadIdx.x + j;
        const uint64_t wb = w < O.W.words ? O.W.bits[w] : 0ull;
        np += w < O.W.words ? (uint32_t)__popcll(O.W.probe[w]) : 0u;
        s_b[4 * threadIdx.x + j] = wb;
        s_r[4 * threadIdx.x + j] = c;
        c += (uint32_t)__popcll(wb);
    }
    const uint32_t base = block_count_n(&O.cnt[ORD_NWL], c);
#pragma unroll
    for (int j = 0; j < 4; j++)
        s_r[4 * threadIdx.x + j] += base;
    block_add(&O.cnt[ORD_NNEWDROP], np);   // (syncs: s_b / s_r written)
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t below = (1ull << lane) - 1;
    for (uint32_t k = (LISTW / 4) * wv; k < (LISTW / 4) * (wv + 1); k++) {
        const uint64_t b = s_b[k];
        if ((b >> lane) & 1)
            O.wl[s_r[k] + (uint32_t)__popcll(b & below)] = (uint32_t)(64 * (w0 + k)) + lane;
    }
}

// the probe filter (OrdArgs.pfilt): a main-set tag's Bloom bits
__device__ __forceinline__ uint32_t *pf_word(const OrdArgs &O, uint32_t tg)
{
    return O.pfilt + ((tg * 0x9E3779B1u) >> 6 & O.pf_mask);
}

// a lane per work-list entry, grid-stride over its device count: the
// creates' tags into the sets (and the probe filter), the ICMP errors' into
// the related set, the deletes' marks (the UDP / ICMP creates' related-entry
// tags, which need the header decoded, are k_ord_rel_w's)
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_ord_mark_w(CtaArgs A, OrdArgs O)
{
    constexpr int NST = TWO ? 2 : 1;
    uint32_t ncr = 0, ndel = 0, nnd = 0, nest = 0, ndt = 0, nun = 0, nrk = 0, full = 0;
    const uint32_t nl = O.cnt[ORD_NWL];
    uint32_t *const rset = O.cbloom + O.cb_mask + 1;
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < nl; x += gridDim.x * blockDim.x) {
        const uint64_t i = O.wl[x];
        const uint32_t cb = A.ctb[i];
        const bool drop = A.ver[i] == DROP_POLICY;
        const bool tcp = (A.mt[i] & 0xFF) == 6;
        const int last = (cb & (CFC_CT_DONE << 4)) ? 1 : 0;
#pragma unroll
        for (int st = 0; st < NST; st++) {
            const uint32_t cs = (cb >> (4 * st)) & 0xF;
            if (!(cs & CFC_CT_DONE))
                continue;
            const uint32_t r = cs & CFC_CT_RES_MASK;
            const bool dropped = st == last && drop;
            if (r == CT_NEW) {
                const uint32_t tg = (st ? O.ck2 : O.ck1)[i];
                if (dropped) {   // (a probe bit's stage is the probe pass's)
                    nnd += !probe_tag(tg);
                    if (tag_ok(tg) && (tg & 1)) {   // an ICMP error's key
                        full += !rel_put(rset, O.cb_mask, tg, true);
                        nrk++;
                    }
                    continue;
                }
                ncr++;
                if (!tag_ok(tg)) {
                    nun++;
                    continue;
                }
                if (tg & 1) {   // an ICMP error's k2, created (its own related entry)
                    full += !rel_put(rset, O.cb_mask, tg, true);
                    nrk++;
                    continue;
                }
                full += !set_put(O.cbloom, O.cb_mask, tg);
                // (no return value waited for: no load first either)
                atomicOr(pf_word(O, tg), bloom_bits(fmix32(tg)));
                if (tcp)   // (a TCP create writes no related entry)
                    O.rtag[TWO ? 2 * i + st : i] = 0u;
            } else if (r == CT_ESTABLISHED) {
                nest++;
                if (!dropped)
                    continue;
                ndt++;
                const uint32_t sl = start_slot<V6>(A, O, i, st);
                if (sl == NONE)
                    continue;
                const uint32_t bb = 1u << (sl & 31), ord = (uint32_t)(i << 1) | (uint32_t)st;
                if (!(O.delbm[sl >> 5] & bb))
                    atomicOr(&O.delbm[sl >> 5], bb);
                if (ord < O.dfirst[sl])
                    atomicMin(&O.dfirst[sl], ord);
                ndel++;
            }
        }
    }
    block_add(&O.cnt[ORD_NCREATE], ncr);
    block_add(&O.cnt[ORD_NDEL], ndel);
    block_add(&O.cnt[ORD_NNEWDROP], nnd);
    block_add(&O.cnt[ORD_NEST], nest);
    block_add(&O.cnt[ORD_NESTDROP], ndt);
    block_add(&O.cnt[ORD_UNTAGGED], nun);
    block_add(&O.cnt[ORD_RELBOUND], nrk);
    block_add(&O.cnt[ORD_SETFULL], full);
}

// the UDP / ICMP creates' related-entry tags into the related set: a lane
// per work-list entry again (its bytes warm from mark), the decode only for
// those creates (mark's own registers stay few)
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_ord_rel_w(CtaArgs A, OrdArgs O)
{
    constexpr int NST = TWO ? 2 : 1;
    uint32_t full = 0, nu = 0;
    const uint32_t nl = O.cnt[ORD_NWL];
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < nl; x += gridDim.x * blockDim.x) {
        const uint64_t i = O.wl[x];
        if ((A.mt[i] & 0xFF) == 6)
            continue;
        const uint32_t cb = A.ctb[i];
        const bool drop = A.ver[i] == DROP_POLICY;
        const int last = (cb & (CFC_CT_DONE << 4)) ? 1 : 0;
#pragma unroll
        for (int st = 0; st < NST; st++) {
            const uint32_t cs = (cb >> (4 * st)) & 0xF;
            if (!(cs & CFC_CT_DONE) || (cs & CFC_CT_RES_MASK) != CT_NEW || (st == last && drop))
                continue;
            const uint32_t tg = (st ? O.ck2 : O.ck1)[i];
            if (!tag_ok(tg) || (tg & 1))   // (mark's: untagged, an ICMP error's k2)
                continue;
            const uint32_t rt = rel_tag<V6>(A, i, st);
            O.rtag[TWO ? 2 * i + st : i] = rt;
            nu++;
            if (rt)
                full += !rel_put(O.cbloom + O.cb_mask + 1, O.cb_mask, rt, false);
        }
    }
    block_add(&O.cnt[ORD_SETFULL], full);
    block_add(&O.cnt[ORD_NUL], nu);
}

// the participants a block finds, staged in LDS and taken from the list by
// one atomic per block (a list atomic per wave or step serialises on the
// counter); a full stage goes straight to the list
constexpr uint32_t PSTAGE = 2048;
struct PartStage {
    uint32_t n, base;
    uint32_t v[PSTAGE];
};
__device__ __forceinline__ void part_put(PartStage &S, const OrdArgs &O, uint32_t v)
{
    const uint32_t q = atomicAdd(&S.n, 1u);
    if (q < PSTAGE) {
        S.v[q] = v;
    } else {
        const uint32_t r = atomicAdd(&O.cnt[ORD_NPART], 1u);
        if (r < O.part_cap)
            O.part[r] = v;
    }
}
// (every thread of the block, after its last part_put)
__device__ __forceinline__ void part_flush(PartStage &S, const OrdArgs &O)
{
    __syncthreads();
    const uint32_t ns = min(S.n, PSTAGE);
    if (threadIdx.x == 0)
        S.base = ns ? atomicAdd(&O.cnt[ORD_NPART], ns) : 0u;
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < ns; q += blockDim.x)
        if (S.base + q < O.part_cap)
            O.part[S.base + q] = S.v[q];
}

// the probes: a dropped CT_NEW stage whose tag the set holds shares the
// entry and takes part (a create of the batch may write its key).  A thread
// per four headers of the probe bits at a step (16-byte loads of their
// keys), grid-stride: the filter first, the set on a maybe.
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_ord_probe_v(CtaArgs A, OrdArgs O)
{
    constexpr int NST = TWO ? 2 : 1;
    __shared__ PartStage S;
    if (threadIdx.x == 0)
        S.n = 0;
    __syncthreads();
    const uint64_t ng = 16 * O.W.words;   // (groups of four headers)
    for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < ng;
         t += (uint64_t)gridDim.x * 256) {
        const uint64_t i0 = 4 * t;
        const bool vec = O.vec && i0 + 4 <= A.n;
        // (the group's keys loaded with its probe bits, not after them: most
        // groups hold a probe, and a dependent load costs a full round trip;
        // streamed once, non-temporal: the filter stays in L2)
        uint32_t c4 = 0;
        uint4 a = make_uint4(NONE, NONE, NONE, NONE), b = a;
        if (vec) {
            c4 = ld_nt(reinterpret_cast<const uint32_t *>(A.ctb + i0));
            a = ld_nt4(O.ck1 + i0);
            if (TWO)
                b = ld_nt4(O.ck2 + i0);
        }
        const uint32_t nib = (uint32_t)(O.W.probe[t >> 4] >> (4 * (t & 15))) & 0xFu;
        if (!nib)
            continue;
        uint32_t cb[4], k1[4], k2[4];
        if (vec) {
            cb[0] = c4 & 0xFF, cb[1] = c4 >> 8 & 0xFF, cb[2] = c4 >> 16 & 0xFF, cb[3] = c4 >> 24;
            k1[0] = a.x, k1[1] = a.y, k1[2] = a.z, k1[3] = a.w;
            k2[0] = b.x, k2[1] = b.y, k2[2] = b.z, k2[3] = b.w;
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const bool in = ((nib >> k) & 1) && i0 + k < A.n;
                cb[k] = in ? A.ctb[i0 + k] : 0u;
                k1[k] = in ? O.ck1[i0 + k] : NONE;
                k2[k] = in && TWO ? O.ck2[i0 + k] : NONE;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (!((nib >> k) & 1))
                continue;
#pragma unroll
            for (int st = 0; st < NST; st++) {
                const uint32_t tg = st ? k2[k] : k1[k];
                // (a probe bit's stage: dropped CT_NEW, the header's last —
                // an egress header's first stage may be an allowed create,
                // collect_w's participant, not a probe)
                const uint32_t cs = (cb[k] >> (4 * st)) & 0xF;
                const int last = (cb[k] & (CFC_CT_DONE << 4)) ? 1 : 0;
                if (st != last || !probe_tag(tg) || !(cs & CFC_CT_DONE) ||
                    (cs & CFC_CT_RES_MASK) != CT_NEW)
                    continue;
                const uint32_t fb = bloom_bits(fmix32(tg));
                if ((*pf_word(O, tg) & fb) != fb)
                    continue;
                uint32_t cur;
                const uint32_t sl = set_find(O.cbloom, O.cb_mask, tg, ~SET_SHARED, cur);
                if (sl == NONE)
                    continue;
                if (!(cur & SET_SHARED))
                    atomicOr(&O.cbloom[sl], SET_SHARED);
                part_put(S, O, (uint32_t)((i0 + k) << 1) | (uint32_t)st);
            }
        }
    }
    part_flush(S, O);
}

// the work bits' participants: a create or an ICMP error whose entry is
// shared (its k2's, or a create's related entry's), and every untagged
// CT_NEW stage.  A lane per work-list entry, grid-stride.
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_ord_collect_w(CtaArgs A, OrdArgs O)
{
    constexpr int NST = TWO ? 2 : 1;
    __shared__ PartStage S;
    if (threadIdx.x == 0)
        S.n = 0;
    __syncthreads();
    const uint32_t nl = O.cnt[ORD_NWL];
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < nl; x += gridDim.x * blockDim.x) {
        const uint64_t i = O.wl[x];
        const uint32_t cb = A.ctb[i];
        const bool drop = A.ver[i] == DROP_POLICY;
        const int last = (cb & (CFC_CT_DONE << 4)) ? 1 : 0;
#pragma unroll
        for (int st = 0; st < NST; st++) {
            const uint32_t cs = (cb >> (4 * st)) & 0xF;
            if (!(cs & CFC_CT_DONE) || (cs & CFC_CT_RES_MASK) != CT_NEW)
                continue;
            const uint32_t tg = (st ? O.ck2 : O.ck1)[i];
            const bool dropped = st == last && drop;
            if (dropped && probe_tag(tg))
                continue;   // (the probe pass's)
            bool take = !tag_ok(tg) || ((tg & 1) ? rel_shared(O, tg) : main_shared(O, tg));
            if (!take && !dropped && !(tg & 1)) {
                const uint32_t rt = O.rtag[TWO ? 2 * i + st : i];
                take = rt && rel_shared(O, rt);
            }
            if (take)
                part_put(S, O, (uint32_t)(i << 1) | (uint32_t)st);
        }
    }
    part_flush(S, O);
}

// the sparse passes' mixed slots (a deleted slot with an allowed
// CT_ESTABLISHED stage, k_ord_mixed): every CT_ESTABLISHED stage on one takes
// part — plain hits outside the work bits among them, so a pass over the
// batch (the launch's keys give the slots).  Nothing to do, and no load past
// the counters, in a batch without deletes or without a mixed slot.
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_ord_collect_mix(CtaArgs A, OrdArgs O)
{
    constexpr int NST = TWO ? 2 : 1;
    __shared__ PartStage S;
    if (threadIdx.x == 0)
        S.n = 0;
    __syncthreads();
    if (O.cnt[ORD_NDEL] && O.cnt[ORD_NMIX]) {
        for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < A.n;
             i += (uint64_t)gridDim.x * 256) {
            const uint32_t cb = A.ctb[i];
#pragma unroll
            for (int st = 0; st < NST; st++) {
                const uint32_t cs = (cb >> (4 * st)) & 0xF;
                if (!(cs & CFC_CT_DONE) || (cs & CFC_CT_RES_MASK) != CT_ESTABLISHED)
                    continue;
                const uint32_t sl = start_slot<V6>(A, O, i, st);
                if (sl != NONE && ((O.mixbm[sl >> 5] >> (sl & 31)) & 1)) {
                    part_put(S, O, (uint32_t)(i << 1) | (uint32_t)st);
                    // (round 2's bounds: an entry with TUPLE_F_RELATED is an
                    // ICMP error's lookup; any other may be re-created after
                    // its delete, with a related entry)
                    atomicAdd(&O.cnt[(*slot_w<V6>(A, sl) & 0x200u) ? ORD_RELBOUND : ORD_NUL], 1u);
                }
            }
        }
    }
    part_flush(S, O);
}

// a deleting stage on a slot only deletes: all but its first delete see
// the entry gone (CT_NEW, no create: they are dropped).  Runs before
// k_ord_write (its stages' bytes are the launch's).
template <bool V6, bool TWO>
__device__ __forceinline__ bool deltail_one(const CtaArgs &A, const OrdArgs &O, uint64_t i)
{
    constexpr int NST = TWO ? 2 : 1;
    bool chg = false;
    const uint32_t cb = A.ctb[i];
    const int last = (cb & (CFC_CT_DONE << 4)) ? 1 : 0;
#pragma unroll
    for (int st = 0; st < NST; st++) {
        const uint32_t cs = (cb >> (4 * st)) & 0xF;
        if (!(cs & CFC_CT_DONE) || (cs & CFC_CT_RES_MASK) != CT_ESTABLISHED ||
            !(st == last && A.ver[i] == DROP_POLICY))
            continue;
        const uint32_t sl = start_slot<V6>(A, O, i, st);
        if (sl == NONE || ((O.mixbm[sl >> 5] >> (sl & 31)) & 1) ||
            O.dfirst[sl] == ((uint32_t)(i << 1) | (uint32_t)st))
            continue;
        const uintptr_t ba = reinterpret_cast<uintptr_t>(O.ctb + i);
        uint32_t *wp = reinterpret_cast<uint32_t *>(ba & ~(uintptr_t)3);
        const uint32_t bs = 8 * (uint32_t)(ba & 3) + 4 * st;
        atomicAnd(wp, ~(0xFu << bs));
        atomicOr(wp, ((uint32_t)CT_NEW | CFC_CT_DONE) << bs);
        uint32_t *ck = st ? O.ck2 : O.ck1;
        if (ck)
            ck[i] = NONE;
        chg = true;
    }
    return chg;
}
// (every deleting stage is a work bit: the sparse passes' list holds them)
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_ord_deltail(CtaArgs A, OrdArgs O)
{
    uint32_t nchg = 0;
    if (O.sparse && O.wl) {
        const uint32_t nl = O.cnt[ORD_NWL];
        for (uint32_t x = blockIdx.x * 256 + threadIdx.x; x < nl; x += gridDim.x * 256)
            nchg += deltail_one<V6, TWO>(A, O, O.wl[x]) ? 1u : 0u;
    } else {
        for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < A.n;
             i += (uint64_t)gridDim.x * 256)
            nchg += deltail_one<V6, TWO>(A, O, i) ? 1u : 0u;
    }
    block_add(&O.cnt[ORD_CHANGED], nchg);
}

// ---- keys: one thread per record r.  r < np: participant r; else the
// related-entry write of the creating participant rel_src[r - np].
template <bool V6>
__device__ __forceinline__ void put_rk(const OrdArgs &O, uint32_t r, Addr<V6> d, Addr<V6> s,
                                       uint32_t z, uint32_t w)
{
    if constexpr (V6) {
        uint4 *k = reinterpret_cast<uint4 *>(O.rk) + 3ull * r;
        k[0] = d;
        k[1] = s;
        k[2] = make_uint4(z, w, 0, 0);
    } else {
        reinterpret_cast<uint4 *>(O.rk)[r] = make_uint4(d, s, z, w);
    }
}
template <bool V6>
__device__ __forceinline__ bool rk_eq(const OrdArgs &O, uint32_t a, uint32_t b)
{
    const uint4 *k = reinterpret_cast<const uint4 *>(O.rk);
    constexpr uint32_t W = V6 ? 3 : 1;
    for (uint32_t j = 0; j < W; j++) {
        const uint4 x = k[W * a + j], y = k[W * b + j];
        if (x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w)
            return false;
    }
    return true;
}

// record r: participant p's lookup, or (rel) the related-entry write of
// the creating participant p
template <bool V6>
__device__ __forceinline__ void ord_record(const CtaArgs &A, const OrdArgs &O, uint32_t r,
                                           uint32_t p, bool rel)
{
    const uint32_t pw = O.part[p];
    const uint64_t i = pw >> 1;
    const int st = (int)(pw & 1);
    const Op<V6> o = decode<V6>(A, i, st);
    uint32_t z = o.z2, w = o.w2;
    if (rel) {   // ct_create's related ICMP entry: ports 0, k2's flags | RELATED
        z = 0;
        w = ct_word(icmp_proto<V6>(), ((o.w2 >> 8) & 7) | 2u, o.owner);
    }
    put_rk<V6>(O, r, o.sa, o.da, z, w);
    // the sort key: a 32-bit key fingerprint, then the header order (a
    // create's related write right after its own lookup).  The fingerprint
    // is fp64's second hash, independent of ct_hash4(sa, da, z, w): the
    // participants were picked by tags (ck_miss4 / ck_miss6) that are that
    // first hash, so two keys whose tags collided would share 29 of its 32
    // bits — a collision in resolve's walk one time in eight, and a key
    // behind a hot flow's thousands of records walks them all, one
    // dependent load at a time (3-15 ms launches in round 6's first traces)
    const uint32_t ord = (uint32_t)(((2 * i + (uint64_t)st) << 1) | (rel ? 1u : 0u));
    O.rh[r] = (fp64(o.sa, o.da, z, w) << 32) | ord;
    O.ridx[r] = r;
    if (rel) {
        O.pinfo[r] = PI_REL | PI_POST;
        return;
    }
    const uint32_t cb = A.ctb[i];
    const uint32_t cs = (cb >> (4 * st)) & 0xF;
    const int last = (cb & (CFC_CT_DONE << 4)) ? 1 : 0;
    const bool dropped = st == last && A.ver[i] == DROP_POLICY;
    uint8_t f = 0;
    if ((cs & CFC_CT_RES_MASK) == CT_ESTABLISHED)
        f |= PI_START;
    if (!dropped)
        f |= PI_POST;
    // a create's related entry lands in the device table for an ANY map
    // (a TCP map's is one no lookup reaches), unless k2 is one itself
    if (!dropped && !o.is_tcp && !o.ki_form)
        f |= PI_MKREL;
    if (w & 0x200u)
        f |= PI_RELKEY;
    O.pinfo[r] = f;
    if (f & PI_RELKEY && r == p)   // (round 1)
        atomicAdd(&O.cnt[ORD_NRELKEY], 1u);
}
// round 1: one thread per participant
template <bool V6>
__global__ __launch_bounds__(256) void k_ord_keys(CtaArgs A, OrdArgs O, uint32_t np)
{
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r < np)
        ord_record<V6>(A, O, r, r, false);
}
// round 2: only the keys with TUPLE_F_RELATED take part — the ICMP errors'
// lookups (ORD_NRK2 of them, copies of their participants: records np..)
// and the related entries the creates write (ORD_NREL) — no other key has
// that flag, so every other participant keeps round 1's result.  Laid out
// for a bound known on the host (n2), the counts read here: the places past
// them are records that sort last and resolve skips — no wait for the counts
template <bool V6>
__global__ __launch_bounds__(256) void k_ord_keys2(CtaArgs A, OrdArgs O, uint32_t np, uint32_t n2)
{
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= n2)
        return;
    const uint32_t nrk = O.cnt[ORD_NRK2], nrel = O.cnt[ORD_NREL];
    if (j < nrk) {
        ord_record<V6>(A, O, np + j, O.rel_src[np + j], false);
    } else if (j < nrk + nrel) {
        ord_record<V6>(A, O, np + j, O.rel_src[j - nrk], true);
    } else {
        O.rh[np + j] = ~0ull;
        O.ridx[np + j] = np + j;
        O.pinfo[np + j] = PI_REL;
    }
}
// round 2's results of the ICMP errors' copies back to their participants
__global__ __launch_bounds__(256) void k_ord_rk2_back(OrdArgs O, uint32_t np, uint32_t n2)
{
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j < n2 && j < O.cnt[ORD_NRK2])
        O.nres[O.rel_src[np + j]] = O.nres[np + j];
}

// ---- resolve: per record in (key, order) order, a lookup's result is the
// outcome of the nearest record before it on the same key (the sorted
// fingerprints group keys; equal fingerprints of different keys — a
// collision — are told apart by the keys themselves), else the batch
// start's.  nres[r]: 1 the key exists (CT_ESTABLISHED), 0 not (CT_NEW).
template <bool V6>
__global__ __launch_bounds__(256) void k_ord_resolve(OrdArgs O, const uint64_t *h,
                                                     const uint32_t *idx, uint32_t n)
{
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n)
        return;
    const uint32_t r = idx[k];
    const uint8_t f = O.pinfo[r];
    if (f & PI_REL)
        return;
    uint8_t state = (f & PI_START) ? 1 : 0;
    const uint32_t fk = (uint32_t)(h[k] >> 32);
    uint32_t coll = 0;
    for (uint32_t j = k; j > 0 && (uint32_t)(h[j - 1] >> 32) == fk; j--) {
        const uint32_t q = idx[j - 1];
        if (rk_eq<V6>(O, q, r)) {
            state = (O.pinfo[q] & PI_POST) ? 1 : 0;
            break;
        }
        coll++;   // (a fingerprint collision: walk on)
    }
    O.nres[r] = state;
    if (coll)
        atomicAdd(&O.cnt[ORD_COLL], coll);
}

// the related-entry writes of the creates round 1 resolved (CT_NEW and
// allowed, ANY map)
__global__ __launch_bounds__(256) void k_ord_relsrc(OrdArgs O, uint32_t np)
{
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    const bool want = p < np && (O.pinfo[p] & PI_MKREL) && O.nres[p] == 0;
    const uint32_t r = block_count(&O.cnt[ORD_NREL], want);
    if (want)
        O.rel_src[r] = p;
    // (and the ICMP errors' participants, listed after np)
    const bool rk = p < np && (O.pinfo[p] & PI_RELKEY);
    const uint32_t q = block_count(&O.cnt[ORD_NRK2], rk);
    if (rk)
        O.rel_src[np + q] = p;
}

// ---- write: the changed stages' CT bytes (result and create bit) and hit
// keys.  A stage now CT_ESTABLISHED on a key the batch created has no slot
// in the starting table: the apply's scan turns it into a request resolved
// after the inserts (SEC_FHIT); one now CT_NEW is a create when allowed.
__global__ __launch_bounds__(256) void k_ord_write(CtaArgs A, OrdArgs O, uint32_t np)
{
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    bool chg = false;
    if (p < np) {
        const uint8_t f = O.pinfo[p];
        const uint32_t now = O.nres[p], was = (f & PI_START) ? 1u : 0u;
        chg = now != was;
        if (chg) {
            const uint32_t pw = O.part[p];
            const uint64_t i = pw >> 1;
            const int st = (int)(pw & 1);
            const uint32_t sh = 4 * st;
            const uint32_t nib = (now ? (uint32_t)CT_ESTABLISHED : (uint32_t)CT_NEW) | CFC_CT_DONE |
                                 ((!now && (f & PI_POST)) ? CFC_CT_CREATE : 0u);
            // (the two stages of a header are different participants: the
            // byte is updated with an atomic on its aligned word)
            const uintptr_t ba = reinterpret_cast<uintptr_t>(O.ctb + i);
            uint32_t *wp = reinterpret_cast<uint32_t *>(ba & ~(uintptr_t)3);
            const uint32_t bs = 8 * (uint32_t)(ba & 3) + sh;
            atomicAnd(wp, ~(0xFu << bs));
            atomicOr(wp, nib << bs);
            uint32_t *ck = st ? O.ck2 : O.ck1;
            if (ck)
                ck[i] = NONE;
            // (sparse passes: a mixed slot's plain hit, outside the work
            // bits, that changed joins them — and the work list the apply's
            // scan runs over — once)
            if (O.sparse && O.wl) {
                unsigned long long *wb = reinterpret_cast<unsigned long long *>(
                    const_cast<uint64_t *>(O.W.bits) + (i >> 6));
                const unsigned long long bit = 1ull << (i & 63);
                if (!(*wb & bit) && !(atomicOr(wb, bit) & bit))
                    O.wl[atomicAdd(&O.cnt[ORD_NWL], 1u)] = (uint32_t)i;
            }
        }
    }
    block_add(&O.cnt[ORD_CHANGED], chg ? 1u : 0u);
}

unsigned grid_for(uint64_t n, unsigned cap)
{
    const uint64_t b = (n + 255) / 256;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(b, cap));
}

template <bool V6>
int sort_records(const OrdArgs &O, uint32_t n, hipStream_t s, const uint64_t **h,
                 const uint32_t **idx)
{
    size_t tb = O.tmp_bytes;
    // one sort by (fingerprint, header order): the records' keys hold both
    // (k_ord_keys writes them again for round 2)
    hipcub::DoubleBuffer<uint64_t> kh(O.rh, O.rh2);
    hipcub::DoubleBuffer<uint32_t> vv(O.ridx, O.ridx2);
    if (hipcub::DeviceRadixSort::SortPairs(O.tmp, tb, kh, vv, (int)n, 0, 64, s) != hipSuccess)
        return -EIO;
    *h = kh.Current();
    *idx = vv.Current();
    return 0;
}

template <bool V6>
int ord_resolve_t(const CtaArgs &A, OrdArgs &O, OrdBufs &B, uint32_t *changed, hipStream_t s)
{
    const bool two = A.mode == CFC_MODE_EGRESS;
    const unsigned g = grid_for(A.n, 2048);
    const unsigned gn = grid_for(A.n, 1u << 30);
    uint32_t hc[ORD_NCNT];
    auto rd = [&]() {
        return hipMemcpyAsync(hc, O.cnt, sizeof(hc), hipMemcpyDeviceToHost, s) == hipSuccess &&
               hipStreamSynchronize(s) == hipSuccess;
    };
#define ORD_LAUNCH(K, grid, ...)                                                         \
    do {                                                                                 \
        if (two)                                                                         \
            hipLaunchKernelGGL((K<V6, true>), dim3(grid), dim3(256), 0, s, __VA_ARGS__);  \
        else                                                                             \
            hipLaunchKernelGGL((K<V6, false>), dim3(grid), dim3(256), 0, s, __VA_ARGS__); \
    } while (0)
    // the mark / collect pass: over the launch's work bits, or the batch
    // (the list passes: grid-stride over a device count; a grid of 1024
    // blocks: their counters' atomics, one per block, serialise)
    const unsigned gw = 1024;
    const unsigned gp = 2048;   // (probe_v, grid-stride)
    auto mark = [&]() {
        if (O.sparse)
            ORD_LAUNCH(k_ord_mark_w, gw, A, O);
        else
            ORD_LAUNCH(k_ord_mark, g, A, O);
    };
    *changed = 0;   // (ORD_CHANGED accumulates on the device: no wait for it)
    if (hipMemsetAsync(O.cnt, 0, 4 * ORD_CHANGED, s) != hipSuccess)
        return -EIO;
    O.part = nullptr;
    O.cbloom = nullptr;
    O.ndel = 0;
    // the creates' pre-keys: a filter of about one word per create, sized by
    // the last batch's count (mark inserts them as it counts); a batch with
    // many more creates than that runs mark again on a filter of its size
    auto filter = [&](uint32_t nc) {
        uint32_t words = 1024;
        while (words < nc && words < (1u << 26))
            words *= 2;
        if (B.fpset.ensure(4ull * words) || hipMemsetAsync(B.fpset.p, 0, 4ull * words, s) != hipSuccess)
            return false;
        O.cbloom = (uint32_t *)B.fpset.p;
        O.cb_mask = words - 1;
        return true;
    };
    // keys from the classify launch's miss tags when this apply follows it
    // (outside a service step); mark counts the creates without one, and a
    // batch with any runs mark again on pre-keys
    O.tagged = A.ck1 && (!two || A.ck2) && !A.lbr;
    O.vec = ((uintptr_t)A.ctb & 15) == 0 && ((uintptr_t)A.ver & 15) == 0 &&
            ((uintptr_t)A.ck1 & 15) == 0 && ((uintptr_t)A.ck2 & 15) == 0;
    O.sparse = O.sparse && O.W.bits && O.W.words && O.tagged && O.rtag &&
               64 * O.W.words <= 0xFFFFFFFFull;   // (u32 header indices)
    if (!O.sparse && !filter(B.creates_hint))
        return -ENOMEM;
    // from the first mark on, the per-slot state (delete bits, mixed bits,
    // first-delete orders) must be zero again when this returns, on every
    // path: the next apply reads it
    struct Clear {
        const OrdArgs &O;
        hipStream_t s;
        bool ok = true, need = true;
        ~Clear()
        {
            if (need)
                ok = hipMemsetAsync(O.delbm, 0, O.bm_bytes, s) == hipSuccess &&
                     hipMemsetAsync(O.mixbm, 0, O.bm_bytes, s) == hipSuccess &&
                     hipMemsetD32Async((hipDeviceptr_t)O.dfirst, 0xFFFFFFFFu, O.slots, s) ==
                         hipSuccess;
        }
    } clear{O, s};
    bool done = false;   // (the sparse passes ran to the participants)
    if (O.sparse) {
        // the key sets instead of the filter: two tables of at least 4 words
        // per create of the last batch (a quarter full: short runs) for the
        // tags they take (a create's, its related entry's, an ICMP error's),
        // and the participants' list sized by the last batch; mark, probe and
        // collect back to back, one wait for all their counts
        // the work list first: room for every header
        if (B.wl.ensure(4 * 64 * O.W.words))
            return -ENOMEM;
        O.wl = (uint32_t *)B.wl.p;
        hipLaunchKernelGGL(k_ord_list_w, dim3((unsigned)((O.W.words + LISTW - 1) / LISTW)),
                           dim3(256), 0, s, O);
        // a context's first apply has no last batch to size its sets by: its
        // own work count (at least its creates) sizes them — one host wait,
        // on that apply only (sized from nothing, its sets overflowed and
        // the mark ran twice: 4.3 ms where a steady one takes 0.14)
        uint32_t hint = B.creates_hint;
        if (!hint) {
            uint32_t nwl = 0;
            if (hipMemcpyAsync(&nwl, O.cnt + ORD_NWL, 4, hipMemcpyDeviceToHost, s) !=
                    hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                return -EIO;
            hint = nwl;
        }
        uint32_t words = 1u << 16, fwords = 1u << 12;
        while (words < 4ull * hint + 4096 && words < (1u << 28))
            words *= 2;
        while (fwords < hint / 2 && fwords < (1u << 26))
            fwords *= 2;
        const uint64_t cap0 = std::max<uint64_t>(B.part.bytes / 4, 2ull * B.part_hint + 65536);
        if (B.fpset.ensure(8ull * words + 4ull * fwords) ||
            hipMemsetAsync(B.fpset.p, 0, 8ull * words + 4ull * fwords, s) != hipSuccess ||
            B.part.ensure(4 * std::min<uint64_t>(cap0, 0x3FFFFFFFull)))
            return -ENOMEM;
        O.cbloom = (uint32_t *)B.fpset.p;
        O.cb_mask = words - 1;
        O.pfilt = O.cbloom + 2ull * words;
        O.pf_mask = fwords - 1;
        O.part = (uint32_t *)B.part.p;
        O.part_cap = (uint32_t)std::min<uint64_t>(B.part.bytes / 4, 0x3FFFFFFFull);
        mark();
        ORD_LAUNCH(k_ord_rel_w, 1024, A, O);
        ORD_LAUNCH(k_ord_probe_v, gp, A, O);
        ORD_LAUNCH(k_ord_collect_w, gw, A, O);
        // a batch that deletes: its mixed slots and their stages (two passes
        // over the batch, each gone at its first load without a delete)
        ORD_LAUNCH(k_ord_mixed, gp, A, O);
        ORD_LAUNCH(k_ord_collect_mix, gw, A, O);
        if (!rd())
            return -EIO;
        if (hc[ORD_UNTAGGED] || hc[ORD_SETFULL]) {
            // a batch with an untagged create, or whose keys the sets cannot
            // hold: the dense passes on the filter (the delete and mixed
            // marks made are idempotent)
            O.sparse = false;
            if (!filter(std::max(B.creates_hint, hc[ORD_NCREATE])) ||
                hipMemsetAsync(O.cnt, 0, 4 * ORD_CHANGED, s) != hipSuccess)
                return -EIO;
            mark();
            if (!rd())
                return -EIO;
        } else {
            if (hc[ORD_NPART] > O.part_cap) {   // (a longer list than the room: again)
                if (B.part.ensure(4ull * hc[ORD_NPART]) ||
                    hipMemsetAsync(O.cnt + ORD_NPART, 0, 4, s) != hipSuccess)
                    return -ENOMEM;
                O.part = (uint32_t *)B.part.p;
                O.part_cap = hc[ORD_NPART];
                ORD_LAUNCH(k_ord_probe_v, gp, A, O);
                ORD_LAUNCH(k_ord_collect_w, gw, A, O);
                ORD_LAUNCH(k_ord_collect_mix, gw, A, O);
                if (!rd())
                    return -EIO;
            }
            done = true;
        }
    } else {
        mark();
        if (!rd())
            return -EIO;
    }
    const bool untagged = O.tagged && hc[ORD_UNTAGGED];
    if (!done &&
        (untagged || (hc[ORD_NCREATE] > 4ull * (O.cb_mask + 1) && O.cb_mask + 1 < (1u << 26)))) {
        // (the delete marks are idempotent; the counts start again)
        O.tagged = O.tagged && !untagged;
        if (!filter(hc[ORD_NCREATE]) || hipMemsetAsync(O.cnt, 0, 4 * ORD_CHANGED, s) != hipSuccess)
            return -ENOMEM;
        mark();
        if (!rd())
            return -EIO;
    }
    const uint32_t ncr = hc[ORD_NCREATE];
    B.creates_hint = ncr;
    O.ndel = hc[ORD_NDEL];
    clear.need = O.ndel != 0;   // (mark sets per-slot state only for deletes)
    if (!done) {
        if (!ncr)
            O.cbloom = nullptr;
        if (O.ndel)
            ORD_LAUNCH(k_ord_mixed, gn, A, O);
        // one collect, into room for every stage that may take part
        const uint64_t cap = (uint64_t)ncr + hc[ORD_NNEWDROP] + (O.ndel ? hc[ORD_NEST] : 0u);
        if (cap > 0x3FFFFFFFull)
            return -E2BIG;
        if (!cap)
            return 0;
        if (B.part.ensure(4 * cap))
            return -ENOMEM;
        O.part = (uint32_t *)B.part.p;
        O.part_cap = (uint32_t)cap;
        ORD_LAUNCH(k_ord_collect, g, A, O);
        if (!rd())
            return -EIO;
    }
    const uint64_t np = hc[ORD_NPART];
    if (np > O.part_cap)
        return -EIO;
    B.part_hint = (uint32_t)np;
    static const bool dbg = getenv("CFC_DEBUG_ORDER") != nullptr;
    if (dbg)
        fprintf(stderr,
                "ord: n %llu creates %u dropped-new %u est %u dropped-est %u deletes %u "
                "participants %llu tagged %d sparse %d work %u udp-creates %u set-words %u\n",
                (unsigned long long)A.n, ncr, hc[ORD_NNEWDROP], hc[ORD_NEST], hc[ORD_NESTDROP],
                O.ndel, (unsigned long long)np, (int)O.tagged, (int)done, hc[ORD_NWL],
                hc[ORD_NUL], O.cbloom ? O.cb_mask + 1 : 0u);
    if (np) {
        // records: up to twice as many as participants
        const uint64_t nr = 2 * np;
        const size_t kw = V6 ? 48 : 16;
        if (B.rel_src.ensure(8 * np) || B.rk.ensure(kw * nr) ||
            B.rh.ensure(8 * nr) || B.rh2.ensure(8 * nr) || B.ridx.ensure(4 * nr) ||
            B.ridx2.ensure(4 * nr) || B.pinfo.ensure(nr) || B.nres.ensure(nr))
            return -ENOMEM;
        {
            size_t t1 = 0, t2 = 0;
            hipcub::DoubleBuffer<uint32_t> a(nullptr, nullptr), b(nullptr, nullptr);
            hipcub::DoubleBuffer<uint64_t> c(nullptr, nullptr);
            (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t1, a, b, (int)nr, 0, 32, s);
            (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t2, c, b, (int)nr, 0, 64, s);
            if (B.tmp.ensure(std::max(t1, t2)))
                return -ENOMEM;
        }
        O.part_cap = (uint32_t)np;
        O.rel_src = (uint32_t *)B.rel_src.p;
        O.rk = B.rk.p;
        O.rh = (uint64_t *)B.rh.p;
        O.rh2 = (uint64_t *)B.rh2.p;
        O.ridx = (uint32_t *)B.ridx.p;
        O.ridx2 = (uint32_t *)B.ridx2.p;
        O.pinfo = (uint8_t *)B.pinfo.p;
        O.nres = (uint8_t *)B.nres.p;
        O.tmp = B.tmp.p;
        O.tmp_bytes = B.tmp.bytes;
        const uint32_t npi = (uint32_t)np;
        const unsigned gp = (unsigned)((npi + 255) / 256);
        hipLaunchKernelGGL(k_ord_keys<V6>, dim3(gp), dim3(256), 0, s, A, O, npi);
        const uint64_t *h;
        const uint32_t *idx;
        if (int rc = sort_records<V6>(O, npi, s, &h, &idx))
            return rc;
        hipLaunchKernelGGL(k_ord_resolve<V6>, dim3(gp), dim3(256), 0, s, O, h, idx, npi);
        if (dbg) {
            if (!rd())
                return -EIO;
            fprintf(stderr, "ord: resolve %u records, %u fingerprint-collision steps\n", npi,
                    hc[ORD_COLL]);
        }
        // round 2 only with an ICMP error among the participants (the
        // sparse passes counted a bound of them, and of the creates that may
        // write a related entry; the dense passes' bound is every participant:
        // an untagged or a mixed stage is not counted there)
        const bool relkeys = !done ? (!O.tagged || O.ndel || hc[ORD_RELBOUND])
                                   : hc[ORD_RELBOUND] != 0;
        if (relkeys) {
            const uint32_t n2 = done ? (uint32_t)std::min<uint64_t>(
                                           np, (uint64_t)hc[ORD_RELBOUND] + hc[ORD_NUL])
                                     : npi;
            // (records np.. : np + n2 <= 2 np, the buffers' room)
            hipLaunchKernelGGL(k_ord_relsrc, dim3(gp), dim3(256), 0, s, O, npi);
            hipLaunchKernelGGL(k_ord_keys2<V6>, dim3((n2 + 255) / 256), dim3(256), 0, s, A, O,
                               npi, n2);
            OrdArgs O2 = O;
            O2.rh += npi;
            O2.rh2 += npi;
            O2.ridx += npi;
            O2.ridx2 += npi;
            if (int rc = sort_records<V6>(O2, n2, s, &h, &idx))
                return rc;
            hipLaunchKernelGGL(k_ord_resolve<V6>, dim3((n2 + 255) / 256), dim3(256), 0, s, O, h,
                               idx, n2);
            hipLaunchKernelGGL(k_ord_rk2_back, dim3((n2 + 255) / 256), dim3(256), 0, s, O, npi,
                               n2);
        }
    }
    // (before k_ord_write: the launch's bytes of the deleting stages)
    if (O.ndel)
        ORD_LAUNCH(k_ord_deltail, done ? gw : gn, A, O);
    if (np)
        hipLaunchKernelGGL(k_ord_write, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, A, O,
                           (uint32_t)np);
    // (debugging: CFC_DEBUG_HDR=i,j,... prints those headers' participant
    // records — result at the batch start, after, and the pass's)
    static const char *dbg_hdr = getenv("CFC_DEBUG_HDR");
    if (dbg_hdr && np && np < (1u << 24)) {
        std::vector<uint32_t> part(np);
        std::vector<uint8_t> pi(np), nr(np);
        if (hipStreamSynchronize(s) == hipSuccess &&
            hipMemcpy(part.data(), O.part, 4 * np, hipMemcpyDeviceToHost) == hipSuccess &&
            hipMemcpy(pi.data(), O.pinfo, np, hipMemcpyDeviceToHost) == hipSuccess &&
            hipMemcpy(nr.data(), O.nres, np, hipMemcpyDeviceToHost) == hipSuccess) {
            std::vector<uint64_t> want;
            for (const char *q = dbg_hdr; *q;) {
                want.push_back(strtoull(q, (char **)&q, 10));
                while (*q == ',')
                    q++;
            }
            for (uint64_t p = 0; p < np; p++)
                for (uint64_t w : want)
                    if ((part[p] >> 1) == w)
                        fprintf(stderr, "ord: part %llu hdr %llu st %u pinfo %02x nres %u\n",
                                (unsigned long long)p, (unsigned long long)w, part[p] & 1,
                                pi[p], nr[p]);
        }
    }
#undef ORD_LAUNCH
    // (the per-slot state is cleared for the next batch as `clear` goes)
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// ---- IPv6: ipv6_policy reverse-NATs the packet of every CT hit whose
// entry's rev_nat_index cilium_lb6_reverse_nat holds (bpf_lxc.c:808-815),
// and a create there stores daddr.s6_addr32[3] & 0xFFFF as that index
// (:787-788).  A stage the ordering pass turned CT_ESTABLISHED hits the entry
// an earlier header's create of the same key (so the same daddr) wrote: its
// packet is reverse-NATed by that index.  One it turned CT_NEW (its entry
// deleted earlier in the batch) is not: its packet is the one before the
// stage.  ct0: the CT bytes before the pass.  One thread per header.
__global__ __launch_bounds__(256) void k_ord_pkt6(CtaArgs A, const uint8_t *ct0, cfc_out out)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= A.n)
        return;
    const uint32_t c0 = ct0[i], c1 = A.ctb[i];
    if (c0 == c1)
        return;
    const int st = A.mode == CFC_MODE_EGRESS ? 1 : 0;   // the ipv6_policy stage
    const uint32_t n0 = (c0 >> (4 * st)) & 0xF, n1 = (c1 >> (4 * st)) & 0xF;
    if (!(n0 & CFC_CT_DONE) || !(n1 & CFC_CT_DONE))
        return;
    const uint32_t r0 = n0 & CFC_CT_RES_MASK, r1 = n1 & CFC_CT_RES_MASK;
    const bool est = r0 == CT_NEW && r1 == CT_ESTABLISHED;
    const bool gone = r0 == CT_ESTABLISHED && r1 == CT_NEW;
    if (!est && !gone)
        return;
    const uint32_t proto = A.mt[i] & 0xFF;
    uint4 *ps = reinterpret_cast<uint4 *>(out.pkt_saddr) + i;
    const LbRec6 *l = A.lbr ? reinterpret_cast<const LbRec6 *>(A.lbr) + i : nullptr;
    if (est) {
        // the stage's lookup daddr: the packet's (ingress), the service
        // step's (egress: local delivery of the translated packet)
        const uint4 da = l ? l->tda : ld16(reinterpret_cast<const uint4 *>(A.da) + i);
        uint4 psa = *ps;
        uint32_t ppt = out.pkt_ports[i];
        lb6_rev_nat(A.T, da.w & 0xFFFF, proto, psa, ppt);
        *ps = psa;
        out.pkt_ports[i] = ppt;
    } else {
        *ps = l ? l->psa : ld16(reinterpret_cast<const uint4 *>(A.sa) + i);
        out.pkt_ports[i] = l ? l->ppt : A.pt[i];
    }
}

}  // namespace

int ord_pkt6(const CtaArgs &A, const uint8_t *ct0, const cfc_out &out, hipStream_t s)
{
    if (!A.n || !out.pkt_saddr || !out.pkt_ports || !A.T.rnat6)
        return 0;
    hipLaunchKernelGGL(k_ord_pkt6, dim3((unsigned)((A.n + 255) / 256)), dim3(256), 0, s, A, ct0,
                       out);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int ord_resolve(const CtaArgs &A, OrdArgs &O, OrdBufs &B, bool v6, uint32_t *changed,
                hipStream_t s)
{
    return v6 ? ord_resolve_t<true>(A, O, B, changed, s) : ord_resolve_t<false>(A, O, B, changed, s);
}

}  // namespace cfc
