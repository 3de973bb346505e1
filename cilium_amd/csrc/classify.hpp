// Launch interface of the classify kernels (classify.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cerrno>

#include "../../include/cfc.h"
#include "layout.h"

namespace cfc {

// The egress source endpoint: the constants bpf_lxc.c is compiled with
// (LXC_ID, SECLABEL, POLICY_MAP) for the endpoint whose traffic this is.
struct EgressArgs {
    uint32_t lxc_id;
    uint32_t seclabel;
    uint32_t pol_base;
    uint32_t pol_mask;
    uint32_t ct_owner;   // ct_owner_word of the sending endpoint's CT maps
    // LXC_NAT46 (nat.hip).  IPv6 egress: LXC_IPV4 of the sending endpoint
    // (raw; 0 = none: a NAT64 header drops with DROP_INVALID).  nat_idx /
    // nat_cnt (or null): the headers that take a NAT hop, appended in any
    // order (IPv6 egress: NAT64; IPv4 ingress: NAT46).  nat_id (an IPv6
    // ingress batch of NAT46 hops, or null): each header's source identity,
    // cb[CB_SRC_LABEL] of the IPv4 path (bpf_lxc.c:1098-1110)
    uint32_t nat_v4;
    uint32_t *nat_idx, *nat_cnt;
    const uint32_t *nat_id;
    bool *sums;   // (host) set when the launch wrote DevTables.ct_sum
    // an egress batch with services: per header the CT_SERVICE entry as the
    // headers before it left it (kern_common.hpp SVO_*; svcorder.hip), or null
    const uint32_t *svo;
    // (or null) the apply's work bits (kern_common.hpp wl_want): per 64
    // headers of the batch one word each, written by the launch
    uint64_t *wbits, *wprobe;
};

// an apply's view of a launch's work bits (EgressArgs.wbits / wprobe)
struct WList {
    const uint64_t *bits, *probe;
    uint64_t words;
};

constexpr int BLOCK = 1024;
constexpr int LDS_BYTES_MAX = 160 * 1024;

// ---- per-header counter keys (workspace) and the histogram pass
// The classify kernels leave, per header, the key of every counter the
// reference would bump; k_hist (classify.hip) turns them into sums with an
// LDS histogram per slice of the batch and range of keys.
//   policy   the matched policy entry (its counter index); packed with the
//            header's skb->len as ctr | len << 16 when the epoch has fewer
//            than 0xFFFF entries (k_hist then reads 4 bytes per header),
//            else the bare index (and k_hist reads meta for len)
//   identity the per-identity forward/drop counter of the header's policy
//            verdict: identity << 1 | dropped, packed with len << 16, for
//            identities below ID_PACK_LIMIT whose range of ID_RANGE
//            identities has a histogram job (DevTables.id_cover: the ranges
//            holding ipcache identities, and the reserved ones).  Cilium
//            allocates identities upwards from 256 (pkg/identity), so a
//            node's identities fill the first ranges; any other identity
//            is counted by a direct atomic in the classify kernel.
// NONE (0xFFFFFFFF) = nothing to count.
constexpr uint32_t KEY_NONE = 0xFFFFFFFFu;
constexpr uint32_t HIST_RANGE = 18432;   // LDS slots per histogram range (144 KiB)
constexpr uint32_t PACK_MAX = 0xFFFF;    // packed keys: key < PACK_MAX

// Per-identity forward/drop counters (cfc.h cfc_identity_counters): a block
// of u64 [dir 2][ID_SLOTS identities][outcome 2][packets, bytes] after the
// metrics in the counter block.  Identities >= 65536 (outside the
// pkg/identity allocation range) share the last slot.
constexpr uint32_t ID_SLOTS = 65537;
constexpr uint64_t ID_U64 = 2ull * ID_SLOTS * 2 * 2;
__host__ __device__ inline uint64_t id_index(uint32_t dir, uint32_t ident,
                                             uint32_t drop)
{
    const uint32_t s = ident < ID_SLOTS - 1 ? ident : ID_SLOTS - 1;
    return (((uint64_t)dir * ID_SLOTS + s) * 2 + drop) * 2;
}
// dir index of the identity block: 0 ingress, 1 egress (METRIC_* - 1)
constexpr uint32_t ID_DIR_INGRESS = 0, ID_DIR_EGRESS = 1;
constexpr uint32_t ID_RANGE = HIST_RANGE / 2;   // identities per histogram range
constexpr uint32_t ID_PACK_LIMIT = 32768;        // identity << 1 | drop < 2^16
constexpr uint32_t ID_RANGES = (ID_PACK_LIMIT + ID_RANGE - 1) / ID_RANGE;
__host__ __device__ inline uint32_t id_range_of(uint32_t ident) { return ident / ID_RANGE; }

// Per-launch pointers of the counter keys and the counter block.
struct CountArgs {
    uint32_t *ctr;       // policy key per header (stage 1)
    uint32_t *ctr2;      // egress: the destination's policy (stage 2)
    uint32_t *id;        // identity key per header
    uint32_t *ct;        // CT accounting key per header (stage 1)
    uint32_t *ct2;       // egress stage 2
    uint64_t *g_met;     // metrics block
    uint64_t *g_id;      // identity block
    uint32_t ctr_packed; // policy keys packed with len
};

// Optional per-call timing (CFC_OPT_TIMING): events recorded on the launch
// stream before the classify kernel, after it, and after the counter
// kernels.
struct LaunchTiming {
    hipEvent_t ev[3];
    bool v6;            // an IPv6 launch (cfc_timing's *_v6 sums)
};

// Workspace of one launch over n headers: the key arrays of CountArgs, then
// the histogram's partial slabs.
struct WsLayout {
    size_t ctr, ctr2, id, ct, ct2, partial, total;   // byte offsets / size
    uint32_t nblk;                                    // histogram slices
    // CT accounting by key range (launch_counters): staged records (and,
    // after the fine sort, the same space again), the coarse-sorted records,
    // per-(coarse bucket, chunk) counts and their scan, the fine-sort plan
    size_t ctp_rec, ctp_recA, ctp_rcnt, ctp_cnt, ctp_off, ctp_bsum, ctp_plan, ctp_fo;
    uint32_t ctp_nv, ctp_nbuck, ctp_nco, ctp_g2;      // slices x stages, buckets,
                                                      // coarse buckets, fine chunks
    size_t lb;   // EGRESS with a load balancer: tda, tpt, psa, pda, ppt, fl
};
WsLayout ws_layout(uint64_t n, const DevTables &T, int mode, bool ct);
CountArgs count_args(uint32_t *ws, const WsLayout &w, const DevTables &T,
                     uint64_t *g_met, int mode, bool ct);
// LDS image of the classify kernel for these tables (must be <= 160 KiB).
size_t classify_lds_bytes(const DevTables &T);

// In-place table patches (cfc_commit): each record's 16 bytes stored at its
// device address, one record per address
struct alignas(16) Patch16 {
    uint32_t val[4];
    uint64_t dst;
    uint64_t pad;
};
int launch_patch16(const Patch16 *rec, uint64_t n, hipStream_t stream);

// ---- device CT apply (ctapply.hip)
// ct_create4's ICMP entry for a TCP map: not in the device table, replayed
// into the host map in (seq, order) order at the next synchronisation
struct CtLog {
    uint32_t x, y, w;     // key: saddr, daddr (k2 order), ct_word
    uint32_t now;         // the batch clock of the create
    uint32_t dirlen;      // dir << 31 | nat46 << 30 | len
    uint32_t sec;         // src_sec_id
    uint32_t seq, order;  // apply sequence, header order
    uint32_t lbw, slave;  // rev_nat_index | lb_loopback << 16, slave (a load balancer's creates)
};
// the same for an IPv6 create (ct_create6, conntrack.h:615-662): 16-byte
// addresses, and the rev_nat_index ipv6_policy sets (bpf_lxc.c:787-788)
constexpr uint32_t CTLOG_NAT46 = 1u << 30;   // (dirlen) the create carries nat46
struct CtLog6 {
    uint4 x, y;           // saddr, daddr (k2 order), raw
    uint32_t w, now, dirlen, sec, seq, order, rev, slave;
};
// What the service step of an egress batch with a load balancer left for one
// header (k_cta_lb: lb4_local / lb6_local and the egress reply's reverse NAT,
// replayed in header order per CT_SERVICE entry): the tuple of the sender's
// CT lookup (saddr, tda, tpt), the packet every later stage sees (psa, pda,
// ppt), LBF_* | LBR_RESLAVE, the ct_state of the sender's create (lbw:
// rev_nat_index | loopback << 16), slv: slave | slave0 << 16 (slave0: the
// selection a new CT_SERVICE entry's ICMP entry keeps), svc: the CT_SERVICE
// entry's slot when the batch started (NONE), addr / sva: ct_state->addr
// and svc_addr (ct_create4's reverse-NAT entry)
struct LbRec4 {
    uint32_t tda, psa, pda, tpt, ppt, fl, lbw, slv, svc, addr, sva;
};
struct LbRec6 {
    uint4 tda, psa, pda;
    uint32_t tpt, ppt, fl, lbw, slv, svc, addr, sva;
};
constexpr uint32_t LBR_RESLAVE = 8;   // ct_update4/6_slave ran
// one changed slot for the host mirror
struct CtSyncRec {
    uint32_t slot;
    CtInfo info;
    uint32_t x, y, z, w;
    uint32_t last_rx, last_tx, flags, lifetime;
    uint32_t pad;
};
struct CtSyncRec6 {
    uint32_t slot;
    CtInfo info;
    uint32_t d[4], s[4], z, w;
    uint32_t last_rx, last_tx, flags, lifetime;
    uint32_t pad;
};
// (NFHIT: requests that are counted hits; NKX: creates with a reverse-NAT
// entry; NRELB: creates that may write a related entry — not TCP, k2 not one)
enum { CTA_NREQA, CTA_NHIT, CTA_NREQB, CTA_NCX, CTA_CLAIMS, CTA_NLOG, CTA_NDEDUP, CTA_NSVC,
       CTA_NFHIT, CTA_NKX, CTA_NEWK, CTA_NEWKT, CTA_NLONG, CTA_NLCH, CTA_NRELB, CTA_NCNT };
struct CtaArgs {
    DevTables T;
    // addresses: one word per header (IPv4), four (IPv6, raw network order)
    const uint32_t *sa, *da, *pt, *mt;
    const uint8_t *tf;           // may be null
    const uint8_t *ctb;
    const int32_t *ver;
    const uint32_t *ident;
    // the classify launch's CT accounting keys (slot * 2 + dir) of stage 0
    // and 1, when they are still in its workspace: the scan's hit slots
    // without a second probe (null: probe)
    const uint32_t *ck1, *ck2;
    uint64_t n;
    int mode;
    uint32_t ep_owner, ep_sec, now, seq;
    // the family's table (the other is null), its mask, and its first slot
    // in DevTables.ct_st (0 for IPv4, ct6_acct_base for IPv6); st: the
    // family's CtState lines (DevTables.ct_st + acct_base)
    Ct4Slot *ct4;
    Ct6Slot *ct6;
    uint32_t mask, acct_base;
    CtState *st;
    // per slot {mark, summary} of this apply (one 8-byte word: route reads
    // both with one random load)
    uint2 *ms;
    // per slot the order + 1 of the last plain hit route kept out of the
    // ordered list (0: none; k_cta_route), cleared by the fold; null: every
    // hit of an ordered slot is listed
    uint32_t *lh;
    // the classify launch's plain-hit summaries of this family's slots
    // (DevTables.ct_sum + acct_base) when the apply follows that launch:
    // the scan then leaves the summaries alone, the fold clears an ordered
    // slot's, and the finish takes (and clears) them; null: the scan's
    uint32_t *sum;
    bool vec;                    // the batch's arrays 16-byte aligned (the scan's loads)
    uint32_t *hs;                // [2n] hit slot per header and stage ([4n] with lbr)
    // (IPv4, sparse scan) per header stage ([2n] egress, [n] else) the key of
    // the request the scan made for it — a create's k2, a hit's looked-up
    // key — so the insert needs no decode; null: decoded there
    uint4 *rk4;
    // (sparse) the launch's work list: the scan reads it rather than the
    // batch, and route takes the hit slots from ck1 / ck2 (hs is not written)
    WList W;
    bool sparse;
    // (sparse, after the ordering's sparse passes) the work bits as a list of
    // header indices, *nwl long (OrdArgs.wl): the scan runs a lane per entry
    const uint32_t *wl, *nwl;
    // an egress batch with a load balancer: per header LbRec4 / LbRec6 (its
    // CT_SERVICE ops are virtual headers n..2n-1), null otherwise
    void *lbr;
    const uint32_t *hash;        // skb->hash per header, or null (CFC_FLOW_HASH)
    uint64_t *reqS, *reqS2;      // the CT_SERVICE ops' requests, by home slot
    // per slot ct_state of the load balancer (ct4_lb / ct6_lb), or null:
    // written for every entry the apply creates
    uint4 *lb;
    uint64_t *reqA, *reqA2, *reqB, *reqB2, *cx, *cx2;
    uint32_t req_cap, cx_cap;
    uint32_t rel_mask;           // cta_newkeys: A.cx as a set of 2^k words, mask
    // cta_newkeys per CT map (or null): the family's maps' selector words
    // (owner word | 2 for an ANY map), the new keys each would take
    const uint32_t *emaps;
    uint32_t n_emaps;
    uint32_t *emcnt;   // per map; emcnt[n_emaps]: the records in emrel
    // (eviction) the TCP maps' related-entry keys the batch may add, three
    // words each (saddr, daddr, {ct word}): those maps' related entries are
    // host-side only, so the host checks which its map already holds
    uint4 *emrel;
    uint32_t emrel_cap;
    uint32_t cx_base;            // route: its ordered ops start here
    CtLog *log;                  // IPv4 applies
    CtLog6 *log6;                // IPv6 applies
    uint32_t log_base, log_cap;  // entries before this apply, capacity left
    uint32_t *cnt;               // CTA_* counters
    uint32_t *obm;               // ordered slots, one bit each (cleared per apply)
    void *sort_tmp;
    size_t sort_tmp_bytes;
    int ob, slot_bits;           // sort keys: slot << ob | order
    // the batch's monitor event words (cfc_out.notify), or null: then every
    // hit is replayed in order and the trace words get the packet-order
    // monitor length (k_cta_mon); mon: per header stage the length the
    // fold found (MON_* codes), 0xFF not replayed
    uint32_t *nt;
    uint8_t *mon;
    // a NAT64 hop's batch (the IPv4 egress path after tail_ipv6_to_ipv4): its
    // creates carry nat46 (conntrack.h:714-716)
    uint32_t nat46;
};
// a device buffer owned by the host library (grown on demand)
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    ~DevBuf() { reset(); }
    void reset()
    {
        if (p)
            (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    int zeros(size_t n, hipStream_t s)
    {
        reset();
        if (!n)
            return 0;
        if (hipMalloc(&p, n) != hipSuccess) {
            p = nullptr;
            return -ENOMEM;
        }
        bytes = n;
        return hipMemsetAsync(p, 0, n, s) == hipSuccess ? 0 : -EIO;
    }
    // at least n bytes (contents not kept)
    int ensure(size_t n)
    {
        if (bytes >= n && p)
            return 0;
        reset();
        if (hipMalloc(&p, std::max<size_t>(n, 256)) != hipSuccess) {
            p = nullptr;
            return -ENOMEM;
        }
        bytes = std::max<size_t>(n, 256);
        return 0;
    }
    int upload(const void *src, size_t n, hipStream_t s)
    {
        reset();
        if (!n)
            return 0;
        if (hipMalloc(&p, n) != hipSuccess) {
            p = nullptr;
            return -ENOMEM;
        }
        bytes = n;
        if (hipMemcpyAsync(p, src, n, hipMemcpyHostToDevice, s) != hipSuccess)
            return -EIO;
        return 0;
    }
};

// ---- packet-order CT results (ctorder.hip), run by cfc_ct_apply before
// the apply proper
enum { ORD_NPART, ORD_NCREATE, ORD_NDEL, ORD_NNEWDROP, ORD_NEST, ORD_NESTDROP, ORD_UNTAGGED,
       ORD_RELBOUND, ORD_NRELKEY, ORD_NREL, ORD_NRK2, ORD_NMIX,
       ORD_COLL, ORD_SETFULL, ORD_NWL, ORD_NUL, ORD_CHANGED, ORD_NCNT };
struct OrdArgs {
    uint8_t *ctb;                 // the batch's CT bytes (rewritten in place)
    uint32_t *ck1, *ck2;          // the classify launch's hit keys (or null)
    // per CT slot, zero / all-ones between applies: deleted slots, mixed
    // slots (one bit each), each deleted slot's first delete order
    uint32_t *delbm, *mixbm, *dfirst;
    size_t bm_bytes;
    uint64_t slots;
    uint32_t ndel;                // deleting stages (0: no delete pass)
    uint32_t *cbloom;             // the creates' keys (Bloom words, or null)
    uint32_t cb_mask;
    bool vec;                     // ctb, ver (and ck1 / ck2) 16-byte aligned
    bool tagged;                  // the keys from ck1 / ck2's miss tags (CK_MISS), else
                                  // pre-keys from the headers
    uint32_t *cnt;                // ORD_* counters
    uint32_t *part;               // participants: header << 1 | stage
    uint32_t part_cap;
    uint32_t *rel_src;
    void *rk;                     // per record its key (16 B; IPv6 48 B)
    uint64_t *rh, *rh2;           // fingerprint << 32 | header order (sort keys)
    uint32_t *ridx, *ridx2;
    uint8_t *pinfo, *nres;
    void *tmp;
    size_t tmp_bytes;
    // the launch's work list (EgressArgs.wl): with `sparse` the mark and
    // collect passes read it rather than the whole batch (a deleting batch's
    // mixed slots by two passes over it, k_ord_mixed / k_ord_collect_mix);
    // ord_resolve clears `sparse` for an untagged create or full key sets
    // (the dense passes then run)
    WList W;
    bool sparse;
    // (sparse) the batch's key set (cbloom as an open-addressing table of
    // key tags, cb_mask + 1 words; bit 1 of an entry: shared) and per header
    // stage a create's related-entry tag (the apply's hs, unused then)
    uint32_t *rtag;
    // (sparse) the work bits as a list of header indices (ORD_NWL long,
    // k_ord_list_w): the passes run a lane per listed header, not a wave per
    // word of a few percent set bits (ORD_NUL: the UDP / ICMP creates)
    uint32_t *wl;
    // (sparse) a Bloom filter of the main set's tags (pf_mask + 1 words,
    // about 16 bits per create: cache-resident) the probes test first
    uint32_t *pfilt;
    uint32_t pf_mask;
};
struct OrdBufs {
    DevBuf part, rel_src, rk, rh, rh2, ridx, ridx2, pinfo, nres, tmp, fpset, wl;
    uint32_t creates_hint = 0;   // the last batch's creates: the filter's size
    uint32_t part_hint = 0;      // the last batch's participants: the list's room
};
// rewrites the CT bytes (and hit keys) of the stages whose packet-order
// result differs from the launch's; *changed: how many
int ord_resolve(const CtaArgs &A, OrdArgs &O, OrdBufs &B, bool v6, uint32_t *changed,
                hipStream_t s);
// IPv6: the packet outputs of the ipv6_policy stages ord_resolve turned
// CT_ESTABLISHED (reverse-NATed by the index their create stored) or CT_NEW
// (not); ct0: the CT bytes before ord_resolve
int ord_pkt6(const CtaArgs &A, const uint8_t *ct0, const cfc_out &out, hipStream_t s);
size_t cta_sort_tmp_bytes(uint32_t n);
// v6: the batch is IPv6 (A.ct6, A.log6).  A batch with a load balancer's
// service step (A.lbr) runs cta_lb_pre first (with A.cnt zeroed), then the
// ordering pass (its ops decode the service step's records), then cta_scan.
int cta_lb_pre(const CtaArgs &A, bool v6, hipStream_t s);
int cta_scan(const CtaArgs &A, bool v6, hipStream_t s);
// a sparse scan's batch (A.sparse): hs from the launch's keys, for the
// eviction's protect pass
int cta_hs_fill(const CtaArgs &A, hipStream_t s);
// the keys the creates would add, exactly (requests sorted and deduplicated,
// the table probed): newk[0] all of them, newk[1] those of TCP creates (they
// go to TCP maps, the others to ANY maps); *sorted: the sorted requests for
// cta_rest
int cta_newkeys(const CtaArgs &A, bool v6, uint32_t nreqA, uint64_t **sorted, uint32_t *newk,
                hipStream_t s);
// presorted: cta_newkeys' sorted requests, or null
// routed: with route run early (a sparse scan's batch: cta_route into
// `routed`, nroute ops) the rest takes no host wait; host_cnt is then not
// filled (the caller copies the counters behind it)
int cta_rest(const CtaArgs &A, bool v6, uint32_t nreqA, const uint64_t *presorted,
             uint32_t *host_cnt, hipStream_t s, const uint64_t *routed = nullptr,
             uint32_t nroute = 0);
// route alone, into A.cx from A.cx_base (a sparse scan's batch: right
// after the scan, its creates' slots hold no hit of the launch)
int cta_route(const CtaArgs &A, hipStream_t s);
// lb (ct4_lb / ct6_lb, or null): the records carry slave | loopback << 16 |
// 1 << 31 in pad
int cta_collect(const Ct4Slot *ct4, CtState *st, const uint4 *lb, uint64_t slots,
                CtSyncRec *out, uint32_t cap, uint32_t *cnt, hipStream_t s);
int cta_collect6(const Ct6Slot *ct6, CtState *st, const uint4 *lb, uint64_t slots,
                 CtSyncRec6 *out, uint32_t cap, uint32_t *cnt, hipStream_t s);
int cta_tomb(Ct4Slot *ct4, const CtSyncRec *rec, uint32_t n, hipStream_t s);
// the IPv4 table's slots that are not free (live, tombstone or claimed),
// added into *cnt (the exact load: the GC's trim frees tombstones the host
// mirror still counts)
int ct_count_nonfree4(const Ct4Slot *ct4, uint64_t slots, uint32_t *cnt, hipStream_t s);
int ct_count_nonfree6(const Ct6Slot *ct6, uint64_t slots, uint32_t *cnt, hipStream_t s);
int cta_tomb6(Ct6Slot *ct6, const CtSyncRec6 *rec, uint32_t n, hipStream_t s);
// device-side growth (ct_grow): every key-holding slot of the old table
// (ok: Ct4Slot / Ct6Slot, oslots) into the new one (nk, nmask + 1 slots,
// zeroed), with its CtState line (ost -> nst) and LB word (olb -> nlb, when
// olb); map[old slot] = new slot or NONE; *cnt += the slots moved
int ct_rehash(bool v6, const void *ok, const CtState *ost, const uint4 *olb, uint64_t oslots,
              void *nk, CtState *nst, uint4 *nlb, uint32_t nmask, uint32_t *map, uint32_t *cnt,
              hipStream_t s);
// slot[i * stride] = map[slot[i * stride]] for i < n (NONE stays NONE)
int ct_remap(uint32_t *slot, uint64_t n, uint32_t stride, const uint32_t *map, hipStream_t s);
// a built table's CtTimer array (device) into its n CtState lines
int ct_state_init(CtState *st, const CtTimer *tm, uint64_t n, hipStream_t s);
// the n lines' accounting into out ([slot][4] u64, device), cleared in the lines
int ct_acct_take(CtState *st, uint64_t *out, uint64_t n, hipStream_t s);

// ---- CT garbage collection (cfc_ct_gc): ctmap.GC's doFiltering
// (pkg/maps/ctmap/ctmap.go:303-325) over the device CT4 table.  A deleted
// entry's slot becomes a plain tombstone at once (free for inserts); its key
// goes to a log the host mirror replays at its next ct_sync.  Then every
// cluster's trailing run of tombstones is freed (w = 0): no probe sequence
// runs through it to a live entry.
// counters: deletes logged for the host, entries of the selected maps left,
// non-free slots before
// the trim, slots the trim freed, log entries kept, deletes of entries the
// host never saw
enum { CTG_DELETED, CTG_LIVE, CTG_NONFREE, CTG_FREED, CTG_LOGKEPT, CTG_FRESH, CTG_NCNT = 8 };
constexpr uint32_t CTG_MAX_MAPS = 64;
constexpr uint32_t CTG_REMOVE_EXPIRED = 1, CTG_VALID = 2, CTG_MATCH = 4;
struct CtGcRec {
    uint32_t slot, x, y, z, w;
};
struct CtGcRec6 {
    uint32_t slot;
    uint4 d, s;
    uint32_t z, w;
};
struct CtGcArgs {
    Ct4Slot *ct4;                 // the IPv4 table, or
    Ct6Slot *ct6;                 // the IPv6 one (doGC6)
    CtState *st;                  // the family's slots' lines
    uint64_t slots;
    uint32_t mask;
    // the CT maps selected (owner word | kind << 1: 0 TCP map, 1 ANY map);
    // an entry of map j counts into mcnt[j]
    const uint32_t *maps;
    uint32_t n_maps;
    uint32_t *mcnt;
    uint32_t flags, time;
    const uint32_t *valid, *match; // sorted raw be32 addresses
    const uint4 *valid6, *match6;  // (IPv6) sorted raw addresses
    uint32_t n_valid, n_match;
    CtGcRec *log;
    CtGcRec6 *log6;               // (IPv6)
    uint32_t log_cap;
    uint32_t *cnt;                // CTG_* counters
    const uint32_t *protect;      // slots never deleted (one bit each), or null
};
int ct_gc4(const CtGcArgs &A, hipStream_t s);
// Eviction at a CT map's capacity (cfc_ct_apply, cfc_api.cpp ct_evict_maps):
// the slots a batch's lookups hit (hs: nk hit-slot words, HS_NONE none) as
// bits in bm (never evicted)
int ct_protect_hits(const uint32_t *hs, uint64_t nk, uint32_t *bm, hipStream_t s);
// the pending TCP-map ICMP entries of the device applies (CtLog) filtered the
// same way, kept in order of appearance: in[0, n) -> out; the kept count
// into A.cnt[CTG_LOGKEPT]
int ct_gc_log(const CtGcArgs &A, const CtLog *in, uint32_t n, CtLog *out, hipStream_t s);
int ct_gc_log6(const CtGcArgs &A, const CtLog6 *in, uint32_t n, CtLog6 *out, hipStream_t s);

// ---- service load balancing of an egress batch (lb.hip)
struct LbArgs {
    const uint32_t *sa, *da, *pt, *mt, *hash;   // the batch (hash may be null)
    uint64_t n;
    uint32_t ct_owner;                            // the sender's CT maps
    uint32_t *tda, *tpt, *psa, *pda, *ppt, *fl;   // per header (lb.hip)
    const uint32_t *svo;   // per header the CT_SERVICE entry in packet order, or null
};
int launch_lb4_egress(const DevTables &T, const LbArgs &A, hipStream_t stream);
// the service step in packet order (svcorder.hip): the headers whose
// CT_SERVICE entry the batch creates or re-slaves, sorted by entry and
// header order; per such header after the first of its entry the entry as
// the ones before it leave it (svo).  n < 2^31.  *count: such headers (0:
// svo untouched); the caller owns keys (2 x 8n bytes), svo (4n, zero),
// cnt (4), tmp (svc_order_tmp_bytes(n))
struct SvoArgs {
    const uint32_t *sa, *da, *pt, *mt, *hash;   // the batch (IPv6: 4 words per address)
    uint64_t n;
    uint32_t lxc_id, ct_owner;                  // the sending endpoint
    uint64_t *keys, *keys2;
    uint32_t *svo, *cnt;
    void *tmp;
    size_t tmp_bytes;
};
size_t svc_order_tmp_bytes(uint64_t n);
int svc_order(const DevTables &T, const SvoArgs &A, bool v6, uint32_t *count, hipStream_t s);
// traffic to itself (selfseg.hip): the egress headers whose destination is
// one of `addrs` (IPv4: na words; IPv6: na 16-byte rows) — per such header
// a row {index, L4 word, meta, which address}, at most cap rows (cnt counts
// them all; the caller zeroes it)
struct SelfArgs {
    const void *daddr;
    const uint32_t *pt, *mt;
    uint64_t n;
    const uint32_t *addrs;
    uint32_t na;
    uint4 *rows;
    uint32_t *cnt;
    uint32_t cap;
};
int self_mark(const SelfArgs &A, bool v6, hipStream_t s);
// the service step's results a classify launch reads (EGRESS), and the
// packet outputs; all null when the launch has no load balancer
struct LbIn {
    const uint32_t *tda, *tpt, *psa, *fl;
};

// ---- NAT46 / NAT64 hops (nat.hip): the hop batch's rows (row k is header
// idx[k] of the batch that listed it, translated)
struct NatHop4 {          // NAT64: IPv4 egress rows
    uint32_t *sa, *da, *pt, *mt, *hash;   // hash may be null (no load balancer)
    uint8_t *tf;
};
struct NatHop6 {          // NAT46: IPv6 ingress rows
    uint4 *sa, *da;
    uint32_t *pt, *mt, *mk, *id;          // mk: the skip-proxy magic; id: source identity
    uint8_t *tf;
};
size_t nat_sort_tmp_bytes(uint32_t m);
// the listed headers in header order: in[0, m) -> out (n: the batch's size)
int nat_sort(const uint32_t *in, uint32_t *out, uint32_t m, uint64_t n, void *tmp,
             size_t tmp_bytes, hipStream_t s);
int nat64_gather(const cfc_hdr_v6 &in, const uint32_t *idx, uint32_t m, uint32_t sa4,
                 const NatHop4 &h, hipStream_t s);
int nat46_gather(const DevTables &T, const cfc_hdr_v4 &in, const uint32_t *ident,
                 const uint32_t *idx, uint32_t m, const uint4 *ep6, const NatHop6 &h,
                 hipStream_t s);
// the hop batch's outputs (sub) into the header's (out); sub.ct loses the
// hop's second stage
int nat_scatter(const uint32_t *idx, uint32_t m, const cfc_out &sub, const cfc_out &out,
                hipStream_t s);
// before the apply of the headers' own family: verdict 0, CT bits 4-7 and
// the event word cleared (nat_scatter restores them after the hop's apply)
int nat_pre(const uint32_t *idx, uint32_t m, const cfc_out &out, hipStream_t s);

// dst[i] += src[i] for n u64 (counter import)
int launch_add_u64(uint64_t *dst, const uint64_t *src, uint64_t n,
                   hipStream_t stream);

// g_ctr: the counter block (policy entries, then metrics, then identities)
int launch_classify_v4(const DevTables &T, const cfc_hdr_v4 &in,
                       const cfc_out &out, int mode, const EgressArgs &E,
                       uint64_t *g_ctr, uint32_t *workspace, int num_cus,
                       hipStream_t stream, const LaunchTiming *timing = nullptr);

// The counter kernels over the per-header keys the classify kernel left in
// the workspace (both families): policy entries, identities, CT accounting.
// returns true when the accounting reduce wrote T.ct_sum (the launch's
// plain-hit summaries; tf: the batch's TCP flags, or null)
bool launch_counters(const DevTables &T, const uint32_t *meta, const uint8_t *tf, uint64_t n,
                     int mode, uint32_t *workspace, uint64_t *g_ctr,
                     hipStream_t stream, bool ct);

int launch_classify_v6(const DevTables &T, const cfc_hdr_v6 &in,
                       const cfc_out &out, int mode, const EgressArgs &E,
                       uint64_t *g_ctr, uint32_t *workspace, int num_cus,
                       hipStream_t stream, const LaunchTiming *timing = nullptr);

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (device,
// kernel), thread-safe
void set_lds_limit(const void *kernel, int bytes);

// Drop-notify records of one classified batch (notify.hip): the per-header
// cfc_out.notify words compacted in header order into cfc_drop_notify.
struct NotifyArgs {
    const uint32_t *notify;
    const int32_t *verdict;
    const uint32_t *identity;
    const uint32_t *meta;
    const uint32_t *ports;
    const uint32_t *saddr;   // v4: n words; v6: n x 4 words
    const uint32_t *daddr;
    const uint32_t *hash;    // skb->hash per header (v4), or NULL: flow_hash
    uint64_t n;
    int family;              // 4 or 6
    int mode;
    uint32_t own_seclabel;   // SECLABEL of ep_lxc (egress batches)
    const uint2 *ep_info;    // [65536] {SECLABEL, ifindex} by LXC_ID
    uint32_t host_ifindex;   // HOST_IFINDEX (trace records)
    int traces;              // 1: trace records too (cfc_monitor_events)
    cfc_drop_notify *rec;
    uint64_t *hdr_index;     // may be NULL
    uint64_t cap;
    uint64_t *count;
};
// workspace: one u64 per block of headers (counts, then offsets)
size_t drop_notify_workspace_bytes(uint64_t n);
int launch_drop_notify(const NotifyArgs &a, uint64_t *ws, hipStream_t stream);

}  // namespace cfc
