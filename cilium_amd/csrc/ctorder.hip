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
        return k == NONE ? NONE : (k >> 1) - A.acct_base;
    }
    const Op<V6> o = decode<V6>(A, i, st);
    return find(A, o.sa, o.da, o.z2, o.w2);
}

// ---- which stages take part.  Per k2 key the state is a chain of its
// stages in packet order, but most keys need no sort:
//   * a key no stage of the batch writes keeps its batch-start existence:
//     a dropped CT_NEW stage (no create) matters only when some allowed
//     CT_NEW stage of the batch creates its key (the creates' fingerprints,
//     k_ord_fpins), or when its key is an ICMP error's (a related entry a
//     create may write: round 2);
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

// mark: creates and deletes counted; per deleted slot its bit and its
// first delete's order (read first: a hot flow's packets find them set)
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_ord_mark(CtaArgs A, OrdArgs O)
{
    constexpr int NST = TWO ? 2 : 1;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint32_t ncr = 0, ndel = 0;
    for (uint64_t base = (uint64_t)blockIdx.x * 256; base < A.n; base += stride) {
        const uint64_t i = base + threadIdx.x;
        const uint32_t cb = i < A.n ? A.ctb[i] : 0u;
        const int32_t ver = i < A.n ? A.ver[i] : 0;
        const int last = (cb & (CFC_CT_DONE << 4)) ? 1 : 0;
#pragma unroll
        for (int st = 0; st < NST; st++) {
            const uint32_t cs = (cb >> (4 * st)) & 0xF;
            if (!(cs & CFC_CT_DONE))
                continue;
            const uint32_t res = cs & CFC_CT_RES_MASK;
            const bool dropped = st == last && ver == DROP_POLICY;
            ncr += res == CT_NEW && !dropped;
            if (res == CT_ESTABLISHED && dropped) {
                const uint32_t sl = start_slot<V6>(A, O, i, st);
                if (sl != NONE) {
                    const uint32_t b = 1u << (sl & 31), ord = (uint32_t)(i << 1) | (uint32_t)st;
                    if (!(O.delbm[sl >> 5] & b))
                        atomicOr(&O.delbm[sl >> 5], b);
                    if (ord < O.dfirst[sl])
                        atomicMin(&O.dfirst[sl], ord);
                    ndel++;
                }
            }
        }
    }
    block_add(&O.cnt[ORD_NCREATE], ncr);
    block_add(&O.cnt[ORD_NDEL], ndel);
}

// the creates' k2 fingerprints into an open-addressed set (fp | 1, 0 free)
__device__ __forceinline__ void fp_put(const OrdArgs &O, uint64_t fp)
{
    fp |= 1ull;
    for (uint32_t j = (uint32_t)(fp >> 32) & O.fp_mask;; j = (j + 1) & O.fp_mask) {
        const unsigned long long cur =
            atomicCAS((unsigned long long *)O.fpset + j, 0ull, (unsigned long long)fp);
        if (cur == 0 || cur == fp)
            return;
    }
}
__device__ __forceinline__ bool fp_has(const OrdArgs &O, uint64_t fp)
{
    fp |= 1ull;
    for (uint32_t j = (uint32_t)(fp >> 32) & O.fp_mask;; j = (j + 1) & O.fp_mask) {
        const uint64_t cur = O.fpset[j];
        if (cur == fp)
            return true;
        if (cur == 0)
            return false;
    }
}
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_ord_fpins(CtaArgs A, OrdArgs O)
{
    constexpr int NST = TWO ? 2 : 1;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= A.n)
        return;
    const uint32_t cb = A.ctb[i];
    const int last = (cb & (CFC_CT_DONE << 4)) ? 1 : 0;
#pragma unroll
    for (int st = 0; st < NST; st++) {
        const uint32_t cs = (cb >> (4 * st)) & 0xF;
        if (!(cs & CFC_CT_DONE) || (cs & CFC_CT_RES_MASK) != CT_NEW ||
            (st == last && A.ver[i] == DROP_POLICY))
            continue;
        const Op<V6> o = decode<V6>(A, i, st);
        fp_put(O, fp64(o.sa, o.da, o.z2, o.w2));
    }
}

// mixed: a deleted slot with an allowed CT_ESTABLISHED stage
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_ord_mixed(CtaArgs A, OrdArgs O)
{
    constexpr int NST = TWO ? 2 : 1;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= A.n)
        return;
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
        if (sl != NONE && (O.delbm[sl >> 5] & b) && !(O.mixbm[sl >> 5] & b))
            atomicOr(&O.mixbm[sl >> 5], b);
    }
}

// collect the participants (header << 1 | stage); count only when O.part
// is null
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_ord_collect(CtaArgs A, OrdArgs O)
{
    constexpr int NST = TWO ? 2 : 1;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    // (every thread runs the same number of steps: block_count_n)
    for (uint64_t base = (uint64_t)blockIdx.x * 256; base < A.n; base += stride) {
        const uint64_t i = base + threadIdx.x;
        const uint32_t cb = i < A.n ? A.ctb[i] : 0u;
        const int32_t ver = i < A.n ? A.ver[i] : 0;
        const int last = (cb & (CFC_CT_DONE << 4)) ? 1 : 0;
        uint32_t want[2] = {0, 0}, nw = 0;
#pragma unroll
        for (int st = 0; st < NST; st++) {
            const uint32_t cs = (cb >> (4 * st)) & 0xF;
            if (!(cs & CFC_CT_DONE))
                continue;
            const uint32_t res = cs & CFC_CT_RES_MASK;
            const bool dropped = st == last && ver == DROP_POLICY;
            bool w = false;
            if (res == CT_NEW) {
                w = !dropped;
                if (dropped) {
                    const Op<V6> o = decode<V6>(A, i, st);
                    w = (o.w2 & 0x200u) || (O.fpset && fp_has(O, fp64(o.sa, o.da, o.z2, o.w2)));
                }
            } else if (res == CT_ESTABLISHED && O.ndel) {
                const uint32_t sl = start_slot<V6>(A, O, i, st);
                w = sl != NONE && ((O.mixbm[sl >> 5] >> (sl & 31)) & 1);
            }
            want[st] = w;
            nw += w;
        }
        uint32_t r = block_count_n(&O.cnt[ORD_NPART], nw);
        if (O.part) {
#pragma unroll
            for (int st = 0; st < NST; st++)
                if (want[st]) {
                    if (r < O.part_cap)
                        O.part[r] = (uint32_t)(i << 1) | (uint32_t)st;
                    r++;
                }
        }
    }
}

// a deleting stage on a slot only deletes: all but its first delete see
// the entry gone (CT_NEW, no create: they are dropped).  Runs before
// k_ord_write (its stages' bytes are the launch's).
template <bool V6, bool TWO>
__global__ __launch_bounds__(256) void k_ord_deltail(CtaArgs A, OrdArgs O)
{
    constexpr int NST = TWO ? 2 : 1;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    bool chg = false;
    if (i < A.n) {
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
    }
    block_add(&O.cnt[ORD_CHANGED], chg ? 1u : 0u);
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

template <bool V6>
__global__ __launch_bounds__(256) void k_ord_keys(CtaArgs A, OrdArgs O, uint32_t np, uint32_t nrel)
{
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= np + nrel)
        return;
    const bool rel = r >= np;
    const uint32_t p = rel ? O.rel_src[r - np] : r;
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
    O.rh[r] = fp64(o.sa, o.da, z, w);
    // header order; a create's related write right after its own lookup
    O.rord[r] = (uint32_t)(((2 * i + (uint64_t)st) << 1) | (rel ? 1u : 0u));
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
    if (f & PI_RELKEY)
        atomicAdd(&O.cnt[ORD_NRELKEY], 1u);
}

// the sorted fingerprints, gathered
__global__ __launch_bounds__(256) void k_ord_gather(const uint64_t *rh, const uint32_t *idx,
                                                    uint64_t *out, uint32_t n)
{
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k < n)
        out[k] = rh[idx[k]];
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
    for (uint32_t j = k; j > 0 && h[j - 1] == h[k]; j--) {
        const uint32_t q = idx[j - 1];
        if (rk_eq<V6>(O, q, r)) {
            state = (O.pinfo[q] & PI_POST) ? 1 : 0;
            break;
        }
        atomicAdd(&O.cnt[ORD_COLL], 1u);   // (a fingerprint collision: walk on)
    }
    O.nres[r] = state;
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
    // by header order, then (stable) by fingerprint: (key, order)
    hipcub::DoubleBuffer<uint32_t> ko(O.rord, O.rord2), vi(O.ridx, O.ridx2);
    if (hipcub::DeviceRadixSort::SortPairs(O.tmp, tb, ko, vi, (int)n, 0, 32, s) != hipSuccess)
        return -EIO;
    hipLaunchKernelGGL(k_ord_gather, dim3((n + 255) / 256), dim3(256), 0, s, (const uint64_t *)O.rh,
                       (const uint32_t *)vi.Current(), O.rh2, n);
    uint32_t *vin = vi.Current(), *vout = vin == O.ridx ? O.ridx2 : O.ridx;
    hipcub::DoubleBuffer<uint64_t> kh(O.rh2, O.rh3);
    hipcub::DoubleBuffer<uint32_t> vv(vin, vout);
    tb = O.tmp_bytes;
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
    const unsigned g = grid_for(A.n, 8192);
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
    *changed = 0;   // (ORD_CHANGED accumulates on the device: no wait for it)
    if (hipMemsetAsync(O.cnt, 0, 4 * ORD_CHANGED, s) != hipSuccess)
        return -EIO;
    O.part = nullptr;
    O.fpset = nullptr;
    O.ndel = 0;
    ORD_LAUNCH(k_ord_mark, g, A, O);
    if (!rd())
        return -EIO;
    const uint32_t ncr = hc[ORD_NCREATE];
    O.ndel = hc[ORD_NDEL];
    if (ncr) {   // the creates' key set, for the dropped CT_NEW stages
        uint32_t cap = 1024;
        while (cap < 4ull * ncr && cap < (1u << 30))
            cap *= 2;
        if (B.fpset.ensure(8ull * cap) || hipMemsetAsync(B.fpset.p, 0, 8ull * cap, s) != hipSuccess)
            return -ENOMEM;
        O.fpset = (uint64_t *)B.fpset.p;
        O.fp_mask = cap - 1;
        ORD_LAUNCH(k_ord_fpins, gn, A, O);
    }
    if (O.ndel)
        ORD_LAUNCH(k_ord_mixed, gn, A, O);
    ORD_LAUNCH(k_ord_collect, g, A, O);
    if (!rd())
        return -EIO;
    const uint64_t np = hc[ORD_NPART];
    if (np > 0x3FFFFFFFull)
        return -E2BIG;
    if (np) {
        // buffers: participants, and up to twice as many records
        const uint64_t nr = 2 * np;
        const size_t kw = V6 ? 48 : 16;
        if (B.part.ensure(4 * np) || B.rel_src.ensure(4 * np) || B.rk.ensure(kw * nr) ||
            B.rh.ensure(8 * nr) || B.rh2.ensure(8 * nr) || B.rh3.ensure(8 * nr) ||
            B.rord.ensure(4 * nr) || B.rord2.ensure(4 * nr) || B.ridx.ensure(4 * nr) ||
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
        O.part = (uint32_t *)B.part.p;
        O.part_cap = (uint32_t)np;
        O.rel_src = (uint32_t *)B.rel_src.p;
        O.rk = B.rk.p;
        O.rh = (uint64_t *)B.rh.p;
        O.rh2 = (uint64_t *)B.rh2.p;
        O.rh3 = (uint64_t *)B.rh3.p;
        O.rord = (uint32_t *)B.rord.p;
        O.rord2 = (uint32_t *)B.rord2.p;
        O.ridx = (uint32_t *)B.ridx.p;
        O.ridx2 = (uint32_t *)B.ridx2.p;
        O.pinfo = (uint8_t *)B.pinfo.p;
        O.nres = (uint8_t *)B.nres.p;
        O.tmp = B.tmp.p;
        O.tmp_bytes = B.tmp.bytes;
        if (hipMemsetAsync(O.cnt + ORD_NPART, 0, 4, s) != hipSuccess)
            return -EIO;
        ORD_LAUNCH(k_ord_collect, g, A, O);
        const uint32_t npi = (uint32_t)np;
        const unsigned gp = (unsigned)((npi + 255) / 256);
        hipLaunchKernelGGL(k_ord_keys<V6>, dim3(gp), dim3(256), 0, s, A, O, npi, 0u);
        const uint64_t *h;
        const uint32_t *idx;
        if (int rc = sort_records<V6>(O, npi, s, &h, &idx))
            return rc;
        hipLaunchKernelGGL(k_ord_resolve<V6>, dim3(gp), dim3(256), 0, s, O, h, idx, npi);
        if (!rd())
            return -EIO;
        if (hc[ORD_NRELKEY]) {
            // round 2: the related entries of the creates round 1 resolved
            hipLaunchKernelGGL(k_ord_relsrc, dim3(gp), dim3(256), 0, s, O, npi);
            if (!rd())
                return -EIO;
            const uint32_t nrel = hc[ORD_NREL];
            if (nrel) {
                hipLaunchKernelGGL(k_ord_keys<V6>, dim3((npi + nrel + 255) / 256), dim3(256), 0, s,
                                   A, O, npi, nrel);
                if (int rc = sort_records<V6>(O, npi + nrel, s, &h, &idx))
                    return rc;
                hipLaunchKernelGGL(k_ord_resolve<V6>, dim3((npi + nrel + 255) / 256), dim3(256), 0,
                                   s, O, h, idx, npi + nrel);
            }
        }
    }
    // (before k_ord_write: the launch's bytes of the deleting stages)
    if (O.ndel)
        ORD_LAUNCH(k_ord_deltail, gn, A, O);
    if (np)
        hipLaunchKernelGGL(k_ord_write, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, A, O,
                           (uint32_t)np);
    if (O.ndel &&   // the per-slot state cleared for the next batch
        (hipMemsetAsync(O.delbm, 0, O.bm_bytes, s) != hipSuccess ||
         hipMemsetAsync(O.mixbm, 0, O.bm_bytes, s) != hipSuccess ||
         hipMemsetD32Async((hipDeviceptr_t)O.dfirst, 0xFFFFFFFFu, O.slots, s) != hipSuccess))
        return -EIO;
#undef ORD_LAUNCH
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

}  // namespace

int ord_resolve(const CtaArgs &A, OrdArgs &O, OrdBufs &B, bool v6, uint32_t *changed,
                hipStream_t s)
{
    return v6 ? ord_resolve_t<true>(A, O, B, changed, s) : ord_resolve_t<false>(A, O, B, changed, s);
}

}  // namespace cfc
