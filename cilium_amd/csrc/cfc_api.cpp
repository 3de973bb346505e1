// C ABI of libcfc.so (include/cfc.h): context, BPF-map emulation, epoch
// publication of the flattened tables, classify dispatch and counters.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_set>
#include <type_traits>
#include <vector>

#include "../../include/cfc.h"
#include "classify.hpp"
#include "selfcut.hpp"
#include "flatten.hpp"
#include "maps.hpp"

using namespace cfc;

namespace {

template <class T>
static int upload_vec(DevBuf &b, const std::vector<T> &v, hipStream_t s)
{
    return b.upload(v.data(), v.size() * sizeof(T), s);
}

// An epoch is four table groups (flatten.hpp GROUP_*), each an immutable
// set of device buffers shared by every epoch built while its maps did not
// change: a commit re-flattens and uploads only the groups whose maps did.
struct GIpc {          // ipcache, IPv4
    DevBuf tbl24, tbl8, ovf, l4d, l4c, l4l;
    int layout = 0;
    uint32_t n_prefix4 = 0, tbl8_groups = 0, lpm4_kib = 0;
    uint64_t bytes = 0;
};
struct GIpc6 {         // ipcache, IPv6 (host copy kept for in-place label patches)
    DevBuf l6[4];   // Lpm6: slots, bloom, lens, slots64
    Lpm6 ipc6{};
    Lpm6Host host;
    uint32_t lpm6_kib = 0, n_prefix6 = 0, lpm6_lengths = 0, lpm6_groups = 0;
    uint64_t bytes = 0;
};
struct GPf {           // prefilter
    DevBuf pf24, pf8, pffix, pfbloom, pf6bloom, l6fix[4], l6dyn[4];
    Lpm6 fix{}, dyn{};
    uint32_t fix_mask = 0, fix_zero = 0, bloom_words = 0, bloom6_words = 0;
    uint32_t n_fix4 = 0, n_dyn4 = 0, n_fix6 = 0, n_dyn6 = 0;
    uint64_t bytes = 0;
};
struct GEp {           // endpoints + policy (+ the counter layout)
    DevBuf lxc4, lxc6, pol, polbloom;
    std::vector<PolSlot> pol_host;    // for in-place proxy-port patches
    uint32_t lxc4_mask = 0, lxc6_mask = 0, pol_bloom_words = 0, n_eps = 0, n_eps6 = 0;
    bool lxc4_lds = false, lxc6_lds = false;
    std::unordered_map<int, PolLoc> pol_loc;
    std::vector<std::pair<Map *, std::string>> ctr_owner;
    std::vector<uint32_t> seclabel;   // SECLABEL by LXC_ID at commit
    // drop notifications: {SECLABEL, ifindex} by LXC_ID, from the same
    // snapshot of the maps as the tables
    DevBuf ep_info;
    // LXC_IPV4 / LXC_IP by LXC_ID (nat.hip): the NAT64 source, and on the
    // device the NAT46 destinations ([65536] raw; null when no endpoint has
    // an IPv6 address)
    std::map<uint16_t, uint32_t> nat4;
    DevBuf nat6;
    uint64_t bytes = 0;
};
struct GLb {           // load balancing: services, reverse NAT
    DevBuf lb4, rnat4, lb6, rnat6;
    uint32_t lb4_mask = 0, n_lb4 = 0, lb6_mask = 0, n_lb6 = 0;
    uint64_t bytes = 0;
};
struct GCt {           // conntrack
    DevBuf ct4, ct6, ct_sum;
    // per slot one CtState line (report state, accounting, the device
    // apply's record): IPv4 slots, then IPv6
    DevBuf ct_st;
    DevBuf ct4_lb, ct6_lb;                // per-slot LB state (with a load balancer)
    DevBuf ct4_ms, ct6_ms;     // device CT apply state (ctapply.hip)
    // the host mirror: slot -> key as the host maps hold it (to fold the
    // accounting, patch host-side changes, take the device's records)
    std::vector<Ct4Slot> ct4_host;
    std::vector<Ct6Slot> ct6_host;
    // the device tables' slots (the mirrors' sizes, once any growth's remap
    // has been applied to them)
    uint64_t slots4 = 0, slots6 = 0;
    // a device growth's remap still to apply to a mirror (mirror_sync): per
    // mirror slot its slot in the current table (NONE: dropped)
    DevBuf pend4, pend6;
    std::map<uint64_t, Map *> ct_maps;   // ct_map_key -> map
    uint32_t ct4_mask = 0, ct4_probe = 0, ct6_mask = 0, ct6_probe = 0;
    uint32_t n_ct4 = 0, n_ct6 = 0;
    uint32_t tomb4 = 0, tomb6 = 0;       // deleted slots (CT_TOMBSTONE)
    uint32_t n_nat46 = 0;                // IPv4 entries with nat46 at the build
    uint64_t bytes = 0;
};
struct Epoch {
    uint64_t id = 0;
    std::shared_ptr<GIpc> ipc;
    std::shared_ptr<GIpc6> ipc6;
    std::shared_ptr<GPf> pf;
    std::shared_ptr<GEp> ep;
    std::shared_ptr<GCt> ct;
    std::shared_ptr<GLb> lb;
    DevTables T{};
    cfc_stats st{};
};
// an epoch replaced while launches on other streams may still read it: kept
// until the events recorded on those streams at the swap have passed
struct Retired {
    std::shared_ptr<Epoch> e;
    std::vector<hipEvent_t> ev;
};

}  // namespace

struct cfc_ctx {
    int device = 0;
    int num_cus = 256;
    std::recursive_mutex mu;
    std::map<std::string, std::unique_ptr<Map>> maps;   // by path
    std::map<int, Map *> fds;
    int next_fd = 3;
    std::vector<uint32_t> seclabel = std::vector<uint32_t>(65536, 0);
    uint64_t seclabel_gen = 0;
    BuildOpts opts;
    // node_config.h defaults (IPV4_CLUSTER_RANGE/MASK, ROUTER_IP)
    cfc_node_config node{0x100000u, 0xff0000u,
                         {0xbe, 0xef, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 1, 0, 0}, 1u};
    uint32_t now = 0;   // bpf_ktime_get_sec() (cfc_set_clock)

    std::shared_ptr<Epoch> epoch;
    uint64_t epoch_seq = 0;
    uint64_t built_sig[6] = {~0ull, ~0ull, ~0ull, ~0ull, ~0ull, ~0ull};   // per group
    uint32_t id_cover = 1;   // identity histogram ranges (reserved + ipcache)
    std::vector<Retired> retired;
    std::vector<hipStream_t> streams;   // streams launched on since the last swap
    // in-place patch records of the last commit (patch_ct)
    std::vector<Patch16> patch_host;
    DevBuf patch_dev;
    // device CT apply (ctapply.hip): the host mirror of the CT maps lags
    // the device table until ct_sync
    int ct_apply_mode = CFC_CT_APPLY_DEVICE;
    bool ct_dirty = false;
    uint64_t cta_claims = 0;     // device creates the host mirror lacks (alive)
    // device-table occupancy for the apply's load check: exact non-free
    // slots at the last GC (ct_used, while ct_used_valid), plus the inserts
    // since (cta_ins); otherwise the host's live + tombstone counts
    uint64_t ct_used = 0, cta_ins = 0;
    bool ct_used_valid = false;
    // least CT table slots (a batch outgrew the table: it was rebuilt larger)
    uint64_t ct_min4 = 0, ct_min6 = 0;
    // deletes of the device GC (cfc_ct_gc) the host mirror has not taken
    DevBuf gc_log, gc_tmp, gc_sets, gc_cnt;
    uint64_t gc_log_used = 0;
    // the same for the IPv6 table (doGC6), and its exact occupancy after a
    // GC or a growth (as ct_used for IPv4)
    DevBuf gc_log6;
    uint64_t gc_log6_used = 0;
    uint64_t ct_used6 = 0;
    bool ct_used6_valid = false;
    uint32_t cta_seq = 0;
    uint32_t n_apply_dev = 0, n_apply_host = 0;
    // the CT table's version: bumped by every commit that changes tables
    // and every CT apply
    uint64_t ct_gen = 0;
    // the last IPv4 classify launch: its CT hit slots (the accounting keys,
    // slot * 2 + dir per stage) stay in the workspace until the next launch,
    // and the device apply of that same batch reads them instead of probing
    // the table again (valid while ct_gen is unchanged)
    struct {
        bool valid = false;
        const void *ct = nullptr, *saddr = nullptr;
        uint64_t n = 0, gen = 0;
        int mode = 0, family = 4;
        uint16_t ep = 0;
        size_t k1 = 0, k2 = 0;   // byte offsets in ws; k2 = 0: no stage 2
        bool sum = false;        // its accounting wrote the plain-hit summaries
        // its work bits for the apply's sparse passes (cta_wbits)
        bool wl = false;
    } last_cls;
    DevBuf cta_wbits;   // per 64 headers: work word, then (second half) probe word
    // DevTables.ct_sum holds summaries no apply has taken (cleared before
    // the next launch that keeps them); sum_pending: the last launch kept
    // summaries and no apply has followed it yet; sum_want: launches keep
    // them — off once a launch's went unused (a lookup-only stream pays
    // nothing), on again when an apply follows its launch
    bool sum_dirty = false, sum_pending = false, sum_want = true;
    uint64_t log_used = 0;       // CtLog entries since the last sync
    DevBuf cta_hs, cta_req, cta_req2, cta_cx, cta_cnt, cta_tmp, cta_log, cta_sync, cta_rk;
    DevBuf cta_lbr, cta_reqs;     // a load balancer's service step per header (LbRec4/6)
    DevBuf cta_obm;               // the apply's ordered-slot bitmap
    // packet-order CT results (ctorder.hip): buffers, the deleted-slot
    // bitmap (zero between applies), counters; the stages it changed
    OrdBufs ordb;
    DevBuf ord_delbm, ord_mixbm, ord_dfirst, ord_cnt;
    DevBuf ord_ct0;               // IPv6: the CT bytes before the pass (ord_pkt6)
    DevBuf cta_mon;               // per header stage: the fold's monitor length
    uint64_t n_ord_changed = 0;
    // LXC_NAT46 (nat.hip): the hop batch of each classified batch that had
    // one, kept for its cfc_ct_apply (by the batch's cfc_out.ct); the
    // classify kernels' list of hop headers; an IPv4 entry may carry nat46
    // (one was built, patched in or created since); the hop apply running
    // is NAT64's (its creates carry nat46)
    struct NatRec {
        int family = 0;            // the listing batch's: 6 NAT64, 4 NAT46
        const void *saddr = nullptr;
        uint64_t n = 0;
        int mode = 0;
        uint16_t ep = 0;
        uint32_t m = 0;            // hop rows
        DevBuf idx, rows, outs, ws;
        cfc_hdr_v4 h4{};
        cfc_hdr_v6 h6{};
        cfc_out o{};
    };
    std::map<const void *, NatRec> nat;
    DevBuf nat_list, nat_cnt, nat_tmp;
    // the service step in packet order (svcorder.hip): sort keys, the
    // per-header CT_SERVICE entry words (zero between launches), count
    DevBuf svo_keys, svo_keys2, svo, svo_cnt, svo_tmp;
    uint64_t n_apply_sparse = 0;   // device applies that took the work list
    bool nat46_seen = false, hop_nat46 = false;
    uint64_t n_nat_hops = 0;
    // eviction at a CT map's capacity (ct_evict; CFC_OPT_CT_EVICT)
    bool ct_evict = true;
    DevBuf evict_bm, evict_maps, evict_rel;
    uint64_t n_evicted = 0;
    uint64_t n_ct_grow = 0;   // device-side CT table growths (ct_grow)
    // traffic to itself (selfseg.hip, self_cuts): the candidate addresses,
    // the listed headers and their count; segments run before the last; the
    // last segment of the last cut batch, which its cfc_ct_apply folds
    DevBuf self_addr, self_rows, self_cnt;
    uint64_t n_self_segs = 0;
    struct {
        bool valid = false;
        const void *ct = nullptr, *saddr = nullptr;
        uint64_t n = 0, off = 0;
        int mode = 0, family = 0;
        uint16_t ep = 0;
    } seg;
    // the IPv6 table's device applies: creates the host lacks, inserts
    // since the last sync, CtLog6 entries
    uint64_t cta_claims6 = 0, cta_ins6 = 0, log6_used = 0;
    // a device apply that took no host wait for its own counts (a sparse
    // scan's, route run early): they follow it into pinned host memory and
    // settle() adds them before the next reader of claims / log_used
    bool pend = false, pend_v6 = false;
    uint32_t *pend_cnt = nullptr;   // CTA_NCNT words, pinned
    hipEvent_t pend_ev = nullptr;
    DevBuf cta_cxr;                 // the early route's list
    DevBuf cta_log6;
    bool ct6_dirty = false;      // an IPv6 device apply since the last sync

    // counters: [n_ctr][2] u64 then metrics
    uint64_t *ctr = nullptr;
    size_t ctr_u64 = 0;
    bool ctr_pending = false;
    hipStream_t last_stream = nullptr;
    hipEvent_t last_done = nullptr;
    uint32_t *ws = nullptr;
    size_t ws_bytes = 0;
    Map *metrics = nullptr;
    // per-identity forward/drop counters folded so far ([dir][slot][fwd,
    // drop][packets, bytes], the device block's layout)
    std::vector<uint64_t> idc = std::vector<uint64_t>(ID_U64, 0);

    DevBuf nt_ws;   // drop-notify block counts / offsets
    hipEvent_t nt_done = nullptr;   // after the last drop-notify launch
    hipStream_t nt_stream = nullptr;
    bool nt_pending = false;

    // CFC_OPT_TIMING: events of the launches since the last collect
    bool timing = false;
    std::vector<LaunchTiming> tpool;
    size_t tused = 0;
};

namespace {

// Order work on stream s after the last classify / counter / notify launch
// when that ran on another stream: folds, CT syncs and applies read the
// counter block, the CT table and the workspace those launches write.
void order_after_launches(cfc_ctx *c, hipStream_t s)
{
    if (c->ctr_pending && c->last_done && c->last_stream != s)
        (void)hipStreamWaitEvent(s, c->last_done, 0);
    if (c->nt_pending && c->nt_done && c->nt_stream != s)
        (void)hipStreamWaitEvent(s, c->nt_done, 0);
}

// Signatures of the maps behind each table group, bit g of GROUP_*
// (0 ipcache v4, 1 prefilter, 2 endpoints + policy, 3 CT, 4 ipcache v6,
// 5 load balancing).
// Structural changes (inserts, deletes) count; a value overwritten in place
// does not where a commit can patch it (ipcache v6 labels, policy entries).
constexpr int NGROUPS = 6;
void group_sigs(cfc_ctx *c, uint64_t sig[NGROUPS])
{
    for (int g = 0; g < NGROUPS; g++)
        sig[g] = 1469598103934665603ull + (uint64_t)g;
    auto mix = [&](int g, uint64_t v) { sig[g] = (sig[g] ^ v) * 1099511628211ull; };
    mix(0, (uint64_t)c->opts.lpm4);
    mix(2, c->seclabel_gen);
    for (auto &kv : c->maps) {
        const Map *m = kv.second.get();
        const uint64_t id = (uint64_t)(uintptr_t)m;
        switch (m->role) {
        case ROLE_IPCACHE:
            mix(0, id); mix(0, m->sgen[0]);
            mix(4, id); mix(4, m->sgen[1]);
            break;
        case ROLE_PF4_FIX: case ROLE_PF4_DYN: case ROLE_PF6_FIX: case ROLE_PF6_DYN:
            mix(1, id); mix(1, m->sgen[0]);
            break;
        case ROLE_LXC:
            mix(2, id); mix(2, m->gen);
            break;
        case ROLE_POLICY:
            mix(2, id); mix(2, m->sgen[0]);
            break;
        case ROLE_CT4: case ROLE_CT6:
            // inserts, deletes and value changes are patched in place
            // (patch_ct); the table is rebuilt when it fills up
            mix(3, id); mix(3, m->sgen[0]);
            mix(2, id);   // endpoints see which CT maps exist
            break;
        case ROLE_LB4_SVC: case ROLE_LB4_RNAT: case ROLE_LB6_SVC: case ROLE_LB6_RNAT:
            mix(5, id); mix(5, m->gen);
            // the CT table carries each entry's LB state while a load
            // balancer is configured
            mix(3, m->kv.empty() ? 0 : 1);
            break;
        default:
            break;
        }
    }
}

// CT map and key bytes of a device slot (the slot holds the whole tuple)
Map *ct_slot_key(const Epoch &E, int family, const uint32_t *d, const uint32_t *sa,
                 uint32_t z, uint32_t w, std::string *key)
{
    const uint32_t al = family == 4 ? 4 : 16;
    char k[38];
    memcpy(k, d, al);
    memcpy(k + al, sa, al);
    memcpy(k + 2 * al, &z, 4);
    k[2 * al + 4] = (char)(w & 0xFF);
    k[2 * al + 5] = (char)((w >> 8) & 7);
    key->assign(k, 2 * al + 6);
    auto it = E.ct->ct_maps.find(ct_map_key(family, w & ~0x7FFu, (w & 0xFF) != 6));
    return it == E.ct->ct_maps.end() ? nullptr : it->second;
}

// struct ct_entry fields the device keeps (CtTimer, CtInfo) into a value:
// lifetime @32, bits @36 (rx/tx_closing, nat46, seen_non_syn, lb_loopback
// with a load balancer; others kept), rev_nat_index @38, slave @40 (with a load
// balancer), tx/rx_flags_seen @42/43, src_sec_id @44, last_tx/rx
// @48/52
void ct_value_from_dev(std::string &v, const CtSyncRec &r, bool created)
{
    uint16_t bits = 0;
    if (!created)
        memcpy(&bits, &v[36], 2);
    bits = (uint16_t)((bits & ~(1u | 2u | 4u | 16u)) | ((r.flags >> 16) & 3) |
                      ((r.flags & CTT_NON_SYN) ? 16u : 0u) | ((r.flags & CTT_NAT46) ? 4u : 0u));
    if (r.pad >> 31) {   // the load balancer's ct_state (ct4_lb / ct6_lb)
        bits = (uint16_t)((bits & ~8u) | (((r.pad >> 16) & 1) ? 8u : 0u));
        const uint16_t slave = (uint16_t)(r.pad & 0xFFFF);
        memcpy(&v[40], &slave, 2);
    }
    memcpy(&v[32], &r.lifetime, 4);
    memcpy(&v[36], &bits, 2);
    v[42] = (char)((r.flags >> 8) & 0xFF);
    v[43] = (char)(r.flags & 0xFF);
    memcpy(&v[48], &r.last_tx, 4);
    memcpy(&v[52], &r.last_rx, 4);
    if (created) {
        const uint16_t rev = (uint16_t)(r.info.y & 0xFFFF);
        memcpy(&v[38], &rev, 2);
        memcpy(&v[44], &r.info.sec, 4);
    }
}

// a pending apply's counts into the host's bookkeeping (its event waited)
void settle(cfc_ctx *c)
{
    if (!c->pend)
        return;
    c->pend = false;
    (void)hipEventSynchronize(c->pend_ev);
    const uint32_t *h = c->pend_cnt;
    uint64_t &claims = c->pend_v6 ? c->cta_claims6 : c->cta_claims;
    uint64_t &ins = c->pend_v6 ? c->cta_ins6 : c->cta_ins;
    uint64_t &log_used = c->pend_v6 ? c->log6_used : c->log_used;
    claims += h[CTA_CLAIMS];
    ins += h[CTA_CLAIMS];
    log_used += h[CTA_NLOG];
}

// A device growth's remap into the host mirror of one family (ct_grow):
// the mirror's entries moved to their slots in the current table, plain
// tombstones dropped with theirs.  *tomb: the mirror's tombstones after.
template <class Slot>
int remap_mirror(std::vector<Slot> &h, DevBuf &pend, uint64_t slots, uint32_t *tomb,
                 hipStream_t s)
{
    if (!pend.p)
        return 0;
    const uint64_t n = h.size();
    std::vector<uint32_t> map(n);
    if (n && (hipMemcpyAsync(map.data(), pend.p, 4 * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
              hipStreamSynchronize(s) != hipSuccess))
        return -EIO;
    std::vector<Slot> nh(slots);
    // (tens of millions of scattered copies: spread over the host's cores)
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<uint64_t> tb(nt, 0);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; t++)
        th.emplace_back([&, t]() {
            for (uint64_t i = n * t / nt, e = n * (t + 1) / nt; i < e; i++)
                if (map[i] != 0xFFFFFFFFu) {   // (NONE: dropped)
                    nh[map[i]] = h[i];
                    tb[t] += h[i].w == CT_TOMBSTONE;
                }
        });
    for (std::thread &x : th)
        x.join();
    uint64_t tt = 0;
    for (uint64_t v : tb)
        tt += v;
    *tomb = (uint32_t)tt;
    h.swap(nh);
    pend.reset();
    return 0;
}
int mirror_sync(GCt &G, hipStream_t s)
{
    if (int rc = remap_mirror(G.ct4_host, G.pend4, G.slots4, &G.tomb4, s))
        return rc;
    return remap_mirror(G.ct6_host, G.pend6, G.slots6, &G.tomb6, s);
}

// The IPv6 table's part of ct_sync: its dirty slots, then its TCP maps'
// ICMPv6 entries (CtLog6).
int ct_sync6(cfc_ctx *c, Epoch &E, hipStream_t s)
{
    GCt &G = *E.ct;
    const uint64_t slots = G.slots6;
    uint32_t *cnt = (uint32_t *)c->cta_cnt.p;
    std::vector<CtSyncRec6> rec;
    if (slots && G.ct_st.p) {
        Ct6Slot *ct6 = (Ct6Slot *)G.ct6.p;
        CtState *st = (CtState *)G.ct_st.p + G.slots4;
        const uint4 *lb6 = (const uint4 *)G.ct6_lb.p;
        uint32_t n = 0;
        if (hipMemsetAsync(cnt, 0, 4, s) != hipSuccess ||
            cta_collect6(ct6, st, lb6, slots, nullptr, 0, cnt, s) ||
            hipMemcpyAsync(&n, cnt, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -EIO;
        rec.resize(n);
        if (n) {
            if (c->cta_sync.ensure(sizeof(CtSyncRec6) * n))
                return -ENOMEM;
            CtSyncRec6 *dr = (CtSyncRec6 *)c->cta_sync.p;
            uint32_t n2 = 0;
            if (hipMemsetAsync(cnt, 0, 4, s) != hipSuccess ||
                cta_collect6(ct6, st, lb6, slots, dr, n, cnt, s) ||
                hipMemcpyAsync(rec.data(), dr, sizeof(CtSyncRec6) * n, hipMemcpyDeviceToHost,
                               s) != hipSuccess ||
                hipMemcpyAsync(&n2, cnt, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
                cta_tomb6(ct6, dr, n, s) || hipStreamSynchronize(s) != hipSuccess || n2 != n)
                return -EIO;
        }
    }
    std::string key;
    // the device GC's deletes first (they precede every dirty record of
    // their slots), as ct_sync does for IPv4
    if (c->gc_log6_used) {
        std::vector<CtGcRec6> gl(c->gc_log6_used);
        if (hipMemcpyAsync(gl.data(), c->gc_log6.p, sizeof(CtGcRec6) * gl.size(),
                           hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -EIO;
        for (const CtGcRec6 &r : gl) {
            uint32_t d[4], sa[4];
            memcpy(d, &r.d, 16);
            memcpy(sa, &r.s, 16);
            if (Map *m = ct_slot_key(E, 6, d, sa, r.z, r.w, &key))
                m->erase_raw(key);
            if (r.slot == 0xFFFFFFFFu) {   // (a growth since dropped its tombstone)
                G.n_ct6--;
                continue;
            }
            Ct6Slot &h = G.ct6_host[r.slot];
            if (h.z == r.z && h.w == r.w && !memcmp(h.d, d, 16) && !memcmp(h.s, sa, 16)) {
                G.n_ct6--;
                G.tomb6++;
            } else if (h.w == 0) {
                G.tomb6++;
            }
            h = Ct6Slot{};
            h.w = CT_TOMBSTONE;
        }
        c->gc_log6_used = 0;
        for (auto &kv : c->maps)
            if (kv.second->role == ROLE_CT6)
                kv.second->gc_pending = 0;
    }
    // deletes first (an entry deleted and created again lives in another
    // slot), then creates and updates
    for (int pass = 0; pass < 2; pass++) {
        for (const CtSyncRec6 &r : rec) {
            const bool del = (r.w & CT_TOMBSTONE) == CT_TOMBSTONE;
            if (del != (pass == 0))
                continue;
            const uint32_t w = r.w & ~CT_TOMBSTONE;
            Ct6Slot &h = G.ct6_host[r.slot];
            const bool prev_live = h.w != 0 && h.w != CT_TOMBSTONE;
            Map *m = ct_slot_key(E, 6, r.d, r.s, r.z, w, &key);
            if (del) {
                if (m)
                    m->erase_raw(key);
                if (prev_live) {
                    G.n_ct6--;
                    G.tomb6++;
                } else if (h.w == 0) {
                    G.tomb6++;
                }
                h = Ct6Slot{};
                h.w = CT_TOMBSTONE;
            } else if (r.info.y & CTI_CREATED) {
                if (m) {
                    CtSyncRec r4{};
                    r4.info = r.info;
                    r4.last_rx = r.last_rx;
                    r4.last_tx = r.last_tx;
                    r4.flags = r.flags;
                    r4.lifetime = r.lifetime;
                    r4.pad = r.pad;
                    std::string v(m->value_bytes(), '\0');
                    ct_value_from_dev(v, r4, true);
                    m->put_raw(key, v);
                }
                if (!prev_live) {
                    G.n_ct6++;
                    if (h.w == CT_TOMBSTONE)
                        G.tomb6--;
                }
                memcpy(h.d, r.d, 16);
                memcpy(h.s, r.s, 16);
                h.z = r.z;
                h.w = w;
            } else if (m) {
                auto it = m->kv.find(key);
                if (it != m->kv.end() && it->second.val.size() >= 56) {
                    CtSyncRec r4{};
                    r4.info = r.info;
                    r4.last_rx = r.last_rx;
                    r4.last_tx = r.last_tx;
                    r4.flags = r.flags;
                    r4.lifetime = r.lifetime;
                    r4.pad = r.pad;
                    ct_value_from_dev(it->second.val, r4, false);
                }
            }
        }
    }
    if (c->log6_used) {
        std::vector<CtLog6> lg(c->log6_used);
        if (hipMemcpyAsync(lg.data(), c->cta_log6.p, sizeof(CtLog6) * lg.size(),
                           hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -EIO;
        std::sort(lg.begin(), lg.end(), [](const CtLog6 &a, const CtLog6 &b) {
            return a.seq != b.seq ? a.seq < b.seq : a.order < b.order;
        });
        for (const CtLog6 &g : lg) {
            // ct_create6's second write into the TCP map (conntrack.h:648-660)
            auto it = G.ct_maps.find(ct_map_key(6, g.w & ~0x7FFu, 0));
            if (it == G.ct_maps.end())
                continue;
            char k[38];
            const uint32_t z = 0;
            memcpy(k, &g.x, 16);
            memcpy(k + 16, &g.y, 16);
            memcpy(k + 32, &z, 4);
            k[36] = (char)(g.w & 0xFF);
            k[37] = (char)((g.w >> 8) & 7);
            std::string v(it->second->value_bytes(), '\0');
            const uint32_t dir = g.dirlen >> 31;
            const uint64_t one = 1, len = g.dirlen & (CTLOG_NAT46 - 1);
            memcpy(&v[dir ? 0 : 16], &one, 8);
            memcpy(&v[dir ? 8 : 24], &len, 8);
            const uint32_t life = g.now + 60, last = 5u < g.now ? g.now : 0u;
            // seen_non_syn ("for ICMP, there is no SYN"), nat46
            const uint16_t bits = (uint16_t)(16u | ((g.dirlen & CTLOG_NAT46) ? 4u : 0u));
            const uint16_t rev = (uint16_t)g.rev, slave = (uint16_t)g.slave;
            memcpy(&v[32], &life, 4);
            memcpy(&v[36], &bits, 2);
            memcpy(&v[38], &rev, 2);
            memcpy(&v[40], &slave, 2);
            memcpy(&v[44], &g.sec, 4);
            memcpy(&v[dir ? 52 : 48], &last, 4);
            it->second->put_raw(std::string(k, 38), v);
        }
    }
    c->log6_used = 0;
    c->cta_claims6 = 0;
    c->cta_ins6 = 0;
    c->ct6_dirty = false;
    c->ct_used6_valid = false;
    if (slots) {   // the device's exact load (a GC's trim freed tombstones the mirror holds)
        uint32_t nonfree = 0;
        if (hipMemsetAsync(cnt, 0, 4, s) != hipSuccess ||
            ct_count_nonfree6((const Ct6Slot *)G.ct6.p, slots, cnt, s) ||
            hipMemcpyAsync(&nonfree, cnt, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -EIO;
        G.tomb6 = nonfree >= G.n_ct6 ? (uint32_t)(nonfree - G.n_ct6) : 0u;
    }
    E.st.ct6_entries = G.n_ct6;
    return 0;
}

// The device CT apply's changes into the host mirror of the CT maps: the
// slots with CtInfo dirty bits (created, updated, deleted) compacted on the
// device, then the TCP maps' ICMP entries of its creates (CtLog) in batch and
// header order.  Runs before anything reads or writes a CT map on the host.
int ct_sync(cfc_ctx *c, hipStream_t s)
{
    settle(c);
    if (c->epoch)
        if (int rc = mirror_sync(*c->epoch->ct, s))
            return rc;
    if (!c->ct_dirty || !c->epoch)
        return 0;
    order_after_launches(c, s);
    // (no ct_gen bump: live entries keep their slots; the deleted ones it
    // turns into tombstones were deleted by an apply, which bumped it)
    Epoch &E = *c->epoch;
    GCt &G = *E.ct;
    const uint64_t slots = G.slots4;
    uint32_t n = 0;
    if (c->cta_cnt.ensure(4 * CTA_NCNT))
        return -ENOMEM;
    uint32_t *cnt = (uint32_t *)c->cta_cnt.p;
    Ct4Slot *ct4 = (Ct4Slot *)G.ct4.p;
    CtState *st = (CtState *)G.ct_st.p;
    const uint4 *lb4 = (const uint4 *)G.ct4_lb.p;
    if (hipMemsetAsync(cnt, 0, 4, s) != hipSuccess ||
        cta_collect(ct4, st, lb4, slots, nullptr, 0, cnt, s) ||
        hipMemcpyAsync(&n, cnt, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    std::vector<CtSyncRec> rec(n);
    if (n) {
        if (c->cta_sync.ensure(sizeof(CtSyncRec) * n))
            return -ENOMEM;
        CtSyncRec *dr = (CtSyncRec *)c->cta_sync.p;
        uint32_t n2 = 0;
        if (hipMemsetAsync(cnt, 0, 4, s) != hipSuccess ||
            cta_collect(ct4, st, lb4, slots, dr, n, cnt, s) ||
            hipMemcpyAsync(rec.data(), dr, sizeof(CtSyncRec) * n, hipMemcpyDeviceToHost, s) !=
                hipSuccess ||
            hipMemcpyAsync(&n2, cnt, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            cta_tomb(ct4, dr, n, s) || hipStreamSynchronize(s) != hipSuccess || n2 != n)
            return -EIO;
    }
    std::string key;
    // the GC's deletes first (they precede every dirty record of their
    // slots: a GC clears the slot's dirty bits), then the applies' deletes
    // (an entry deleted and created again lives in another slot, created
    // after the delete), then creates and updates
    if (c->gc_log_used) {
        std::vector<CtGcRec> gl(c->gc_log_used);
        if (hipMemcpyAsync(gl.data(), c->gc_log.p, sizeof(CtGcRec) * gl.size(),
                           hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -EIO;
        for (const CtGcRec &r : gl) {
            if (Map *m = ct_slot_key(E, 4, &r.x, &r.y, r.z, r.w, &key))
                m->erase_raw(key);
            if (r.slot == 0xFFFFFFFFu) {   // (a growth since dropped its tombstone: ct_grow)
                G.n_ct4--;
                continue;
            }
            Ct4Slot &h = G.ct4_host[r.slot];
            if (h.x == r.x && h.y == r.y && h.z == r.z && h.w == r.w) {
                G.n_ct4--;
                G.tomb4++;
            } else if (h.w == 0) {
                G.tomb4++;
            }
            h = Ct4Slot{0, 0, 0, CT_TOMBSTONE};
        }
        c->gc_log_used = 0;
        for (auto &kv : c->maps)
            if (kv.second->role == ROLE_CT4)
                kv.second->gc_pending = 0;
    }
    for (int pass = 0; pass < 2; pass++) {
        for (const CtSyncRec &r : rec) {
            const bool del = (r.w & CT_TOMBSTONE) == CT_TOMBSTONE;
            if (del != (pass == 0))
                continue;
            const uint32_t w = r.w & ~CT_TOMBSTONE;
            Ct4Slot &h = G.ct4_host[r.slot];
            const bool prev_live = h.w != 0 && h.w != CT_TOMBSTONE;
            Map *m = ct_slot_key(E, 4, &r.x, &r.y, r.z, w, &key);
            if (del) {
                if (m)
                    m->erase_raw(key);
                if (prev_live) {
                    G.n_ct4--;
                    G.tomb4++;
                } else if (h.w == 0) {
                    G.tomb4++;
                }
                h = Ct4Slot{0, 0, 0, CT_TOMBSTONE};
            } else if (r.info.y & CTI_CREATED) {
                if (m) {
                    std::string v(m->value_bytes(), '\0');
                    ct_value_from_dev(v, r, true);
                    m->put_raw(key, v);
                }
                if (!prev_live) {
                    G.n_ct4++;
                    if (h.w == CT_TOMBSTONE)
                        G.tomb4--;
                }
                h = Ct4Slot{r.x, r.y, r.z, w};
            } else if (m) {
                auto it = m->kv.find(key);
                if (it != m->kv.end() && it->second.val.size() >= 56)
                    ct_value_from_dev(it->second.val, r, false);
            }
        }
    }
    if (c->log_used) {
        std::vector<CtLog> lg(c->log_used);
        if (hipMemcpyAsync(lg.data(), c->cta_log.p, sizeof(CtLog) * lg.size(),
                           hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -EIO;
        std::sort(lg.begin(), lg.end(), [](const CtLog &a, const CtLog &b) {
            return a.seq != b.seq ? a.seq < b.seq : a.order < b.order;
        });
        for (const CtLog &g : lg) {
            // ct_create4's second write into the TCP map (conntrack.h:741-760)
            auto it = G.ct_maps.find(ct_map_key(4, g.w & ~0x7FFu, 0));
            if (it == G.ct_maps.end())
                continue;
            char k[14];
            const uint32_t z = 0;
            memcpy(k, &g.x, 4);
            memcpy(k + 4, &g.y, 4);
            memcpy(k + 8, &z, 4);
            k[12] = (char)(g.w & 0xFF);
            k[13] = (char)((g.w >> 8) & 7);
            std::string v(it->second->value_bytes(), '\0');
            const uint32_t dir = g.dirlen >> 31;
            const uint64_t one = 1, len = g.dirlen & (CTLOG_NAT46 - 1);
            memcpy(&v[dir ? 0 : 16], &one, 8);
            memcpy(&v[dir ? 8 : 24], &len, 8);
            const uint32_t life = g.now + 60, last = 5u < g.now ? g.now : 0u;
            // seen_non_syn ("for ICMP, there is no SYN"), and a load
            // balancer's ct_state
            const uint16_t bits = (uint16_t)(16u | (((g.lbw >> 16) & 1) ? 8u : 0u) |
                                             ((g.dirlen & CTLOG_NAT46) ? 4u : 0u));
            const uint16_t rev = (uint16_t)(g.lbw & 0xFFFF), slave = (uint16_t)g.slave;
            memcpy(&v[32], &life, 4);
            memcpy(&v[36], &bits, 2);
            memcpy(&v[38], &rev, 2);
            memcpy(&v[40], &slave, 2);
            memcpy(&v[44], &g.sec, 4);
            memcpy(&v[dir ? 52 : 48], &last, 4);
            it->second->put_raw(std::string(k, 14), v);
        }
    }
    c->log_used = 0;
    c->cta_claims = 0;
    c->cta_ins = 0;
    c->ct_used_valid = false;
    {   // the device's exact load: a GC's trim freed tombstones the mirror
        // still holds as deleted (harmless for probes: a trimmed run ends
        // its cluster), so the count is taken from the table itself
        uint32_t nonfree = 0;
        if (hipMemsetAsync(cnt, 0, 4, s) != hipSuccess ||
            ct_count_nonfree4(ct4, slots, cnt, s) ||
            hipMemcpyAsync(&nonfree, cnt, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -EIO;
        G.tomb4 = nonfree >= G.n_ct4 ? (uint32_t)(nonfree - G.n_ct4) : 0u;
    }
    E.st.ct4_entries = G.n_ct4;
    if (int rc = ct_sync6(c, E, s))
        return rc;
    c->ct_dirty = false;
    return 0;
}

// CONNTRACK_ACCOUNTING counts of the device into the CT entries' rx/tx
// packets and bytes (struct ct_entry offsets 0-31)
int fold_ct(cfc_ctx *c, hipStream_t s)
{
    if (int rc = ct_sync(c, s))
        return rc;
    Epoch &E = *c->epoch;
    const size_t n4 = E.ct->slots4, n = n4 + E.ct->slots6;
    if (!n)
        return 0;
    std::vector<uint64_t> h(4 * n);
    DevBuf tmp;   // (the lines' counts, dense)
    if (tmp.ensure(32 * n) || ct_acct_take((CtState *)E.ct->ct_st.p, (uint64_t *)tmp.p, n, s) ||
        hipMemcpyAsync(h.data(), tmp.p, 32 * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    std::string key;
    for (size_t i = 0; i < n; i++) {
        const uint64_t *a = &h[4 * i];
        if (!(a[0] | a[1] | a[2] | a[3]))
            continue;
        Map *m;
        if (i < n4) {
            const Ct4Slot &e = E.ct->ct4_host[i];
            m = ct_slot_key(E, 4, &e.x, &e.y, e.z, e.w, &key);
        } else {
            const Ct6Slot &e = E.ct->ct6_host[i - n4];
            m = ct_slot_key(E, 6, e.d, e.s, e.z, e.w, &key);
        }
        if (!m)
            continue;
        auto it = m->kv.find(key);
        if (it == m->kv.end())
            continue;   // deleted since (ct_delete): its counts go with it
        uint64_t v[4];   // rx_packets, rx_bytes, tx_packets, tx_bytes
        memcpy(v, it->second.val.data(), 32);
        v[2] += a[0];    // [dir CT_EGRESS 0] -> tx
        v[3] += a[1];
        v[0] += a[2];    // [dir CT_INGRESS 1] -> rx
        v[1] += a[3];
        memcpy(&it->second.val[0], v, 32);
    }
    return 0;
}

int fold_counters(cfc_ctx *c, hipStream_t s)
{
    if (!c->ctr_pending || !c->epoch)
        return 0;
    order_after_launches(c, s);
    if (int rc = fold_ct(c, s))
        return rc;
    std::vector<uint64_t> h(c->ctr_u64);
    if (hipMemcpyAsync(h.data(), c->ctr, c->ctr_u64 * 8, hipMemcpyDeviceToHost,
                       s) != hipSuccess)
        return -EIO;
    if (hipMemsetAsync(c->ctr, 0, c->ctr_u64 * 8, s) != hipSuccess)
        return -EIO;
    if (hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    Epoch &E = *c->epoch;
    size_t nctr = E.ep->ctr_owner.size();
    for (size_t i = 0; i < nctr; i++) {
        uint64_t pk = h[2 * i], by = h[2 * i + 1];
        if (!pk && !by)
            continue;
        Map *m = E.ep->ctr_owner[i].first;
        auto it = m->kv.find(E.ep->ctr_owner[i].second);
        if (it == m->kv.end())
            continue;   // entry deleted since: the kernel's update is lost too
        uint64_t v[2];
        memcpy(v, &it->second.val[8], 16);
        v[0] += pk;
        v[1] += by;
        memcpy(&it->second.val[8], v, 16);
    }
    const uint64_t *idb = h.data() + 2 * nctr + METRIC_U64;
    for (uint64_t i = 0; i < ID_U64; i++)
        c->idc[i] += idb[i];
    const uint64_t *met = h.data() + 2 * nctr;
    for (int r = 0; r < METRIC_REASONS; r++)
        for (int d = 0; d < METRIC_DIRS; d++) {
            uint64_t cnt = met[(r * METRIC_DIRS + d) * 2];
            uint64_t byt = met[(r * METRIC_DIRS + d) * 2 + 1];
            if (!cnt && !byt)
                continue;
            // struct metrics_key {u8 reason; u8 dir:2; u16 reserved[3]}
            uint8_t key[8] = {(uint8_t)r, (uint8_t)d, 0, 0, 0, 0, 0, 0};
            Map *mm = c->metrics;
            std::string nk((const char *)key, 8);
            auto it = mm->kv.find(nk);
            uint64_t v[2] = {0, 0};
            if (it != mm->kv.end())
                memcpy(v, it->second.val.data(), 16);
            v[0] += cnt;
            v[1] += byt;
            if (it == mm->kv.end() && mm->kv.size() >= mm->max_entries)
                continue;   // map_update_elem fails in update_metrics too
            Map::Entry &e = mm->kv[nk];
            e.key = nk;
            e.val.assign((const char *)v, 16);
            mm->gen++;
        }
    c->ctr_pending = false;
    return 0;
}

int upload_lpm6(DevBuf *b, const Lpm6Host &h, Lpm6 *d, hipStream_t s)
{
    int rc;
    if ((rc = upload_vec(b[0], h.slots, s)) || (rc = upload_vec(b[1], h.bloom, s)) ||
        (rc = upload_vec(b[2], h.lens, s)) || (rc = upload_vec(b[3], h.slots64, s)))
        return rc;
    d->slots = (const L6Slot *)b[0].p;
    d->slots64 = (const uint4 *)b[3].p;
    d->mask64 = h.slots64.empty() ? 0 : (uint32_t)h.slots64.size() - 1;
    d->bloom = (const uint64_t *)b[1].p;
    d->lens = (const uint32_t *)b[2].p;
    d->mask = h.slots.empty() ? 0 : (uint32_t)h.slots.size() - 1;
    d->bloom_mask = h.bloom.empty() ? 0 : (uint32_t)h.bloom.size() - 1;
    d->nlen = (uint32_t)h.lens.size();
    d->def_label = h.def_label;
    return 0;
}

// a launch on stream s reads the current epoch
void note_stream(cfc_ctx *c, hipStream_t s)
{
    if (std::find(c->streams.begin(), c->streams.end(), s) == c->streams.end())
        c->streams.push_back(s);
}

// the identity ranges of the labels overwritten in place since the last
// commit (added to the cover; a range is never dropped before a rebuild)
uint32_t identity_cover_touched(cfc_ctx *c)
{
    uint32_t cover = 0;
    for (auto &kv : c->maps) {
        Map *m = kv.second.get();
        if (m->role != ROLE_IPCACHE)
            continue;
        for (auto &t : m->touched) {
            auto it = m->kv.find(t.first);
            if (it == m->kv.end())
                continue;
            uint32_t lab;
            memcpy(&lab, it->second.val.data(), 4);
            if (lab < ID_PACK_LIMIT)
                cover |= 1u << id_range_of(lab);
        }
    }
    return cover;
}

// free the retired epochs whose readers have all passed
void reap_retired(cfc_ctx *c)
{
    auto done = [](const Retired &r) {
        for (hipEvent_t e : r.ev)
            if (hipEventQuery(e) != hipSuccess)
                return false;
        return true;
    };
    for (size_t i = 0; i < c->retired.size();) {
        if (done(c->retired[i])) {
            for (hipEvent_t e : c->retired[i].ev)
                (void)hipEventDestroy(e);
            c->retired.erase(c->retired.begin() + (long)i);
        } else {
            i++;
        }
    }
}

std::shared_ptr<GIpc> build_ipc(const HostImage &img, hipStream_t s, int *rc)
{
    auto g = std::make_shared<GIpc>();
    if ((*rc = upload_vec(g->tbl24, img.tbl24, s)) || (*rc = upload_vec(g->tbl8, img.tbl8, s)) ||
        (*rc = upload_vec(g->ovf, img.lbl_ovf, s)) || (*rc = upload_vec(g->l4d, img.l4d, s)) ||
        (*rc = upload_vec(g->l4c, img.l4c, s)) || (*rc = upload_vec(g->l4l, img.l4l, s)))
        return nullptr;
    g->layout = img.lpm4_layout;
    g->n_prefix4 = img.n_prefix4;
    g->tbl8_groups = (uint32_t)(img.tbl8.size() / 256);
    g->lpm4_kib = (uint32_t)((4ull * (img.l4d.size() + img.l4c.size() + img.tbl24.size() +
                                      img.tbl8.size()) + 8ull * img.l4l.size() + 1023) / 1024);
    g->bytes = 4ull * (img.tbl24.size() + img.tbl8.size() + img.lbl_ovf.size() +
                       img.l4d.size() + img.l4c.size()) + 8ull * img.l4l.size();
    return g;
}

std::shared_ptr<GIpc6> build_ipc6(HostImage &img, hipStream_t s, int *rc)
{
    auto g = std::make_shared<GIpc6>();
    if ((*rc = upload_lpm6(g->l6, img.ipc6, &g->ipc6, s)))
        return nullptr;
    g->n_prefix6 = img.ipc6.n;
    g->lpm6_lengths = (uint32_t)img.ipc6.lens.size();
    g->lpm6_groups = img.ipc6.groups;
    g->lpm6_kib = (uint32_t)((img.ipc6.bytes() + 1023) / 1024);
    g->bytes = img.ipc6.bytes();
    g->host = std::move(img.ipc6);
    return g;
}

// per-identity counters: the histogram ranges holding the reserved
// identities and every ipcache identity; others count directly
uint32_t identity_cover(const std::vector<Map *> &ms)
{
    uint32_t cover = 1u;
    for (Map *m : ms)
        if (m->role == ROLE_IPCACHE)
            for (const auto &kv : m->kv) {
                uint32_t lab;
                memcpy(&lab, kv.second.val.data(), 4);
                if (lab < ID_PACK_LIMIT)
                    cover |= 1u << id_range_of(lab);
            }
    return cover;
}

std::shared_ptr<GPf> build_pf(const HostImage &img, hipStream_t s, int *rc)
{
    auto g = std::make_shared<GPf>();
    if ((*rc = upload_vec(g->pf24, img.pf_tbl24, s)) || (*rc = upload_vec(g->pf8, img.pf_tbl8, s)) ||
        (*rc = upload_vec(g->pffix, img.pf_fix, s)) ||
        (*rc = upload_vec(g->pfbloom, img.pf_bloom, s)) ||
        (*rc = upload_vec(g->pf6bloom, img.pf6_bloom, s)) ||
        (*rc = upload_lpm6(g->l6fix, img.pf6_fix, &g->fix, s)) ||
        (*rc = upload_lpm6(g->l6dyn, img.pf6_dyn, &g->dyn, s)))
        return nullptr;
    g->fix_mask = img.pf_fix_mask;
    g->fix_zero = img.pf_fix_zero;
    g->bloom_words = (uint32_t)img.pf_bloom.size();
    g->bloom6_words = (uint32_t)img.pf6_bloom.size();
    g->n_fix4 = img.n_pf_fix;
    g->n_dyn4 = img.n_pf_dyn;
    g->n_fix6 = img.pf6_fix.n;
    g->n_dyn6 = img.pf6_dyn.n;
    g->bytes = 4ull * (img.pf_tbl24.size() + img.pf_tbl8.size() + img.pf_fix.size() +
                       img.pf_bloom.size() + img.pf6_bloom.size()) + img.pf6_fix.bytes() +
               img.pf6_dyn.bytes();
    return g;
}

std::shared_ptr<GEp> build_ep(cfc_ctx *c, HostImage &img, const std::vector<Map *> &ms,
                              hipStream_t s, int *rc)
{
    auto g = std::make_shared<GEp>();
    if ((*rc = upload_vec(g->lxc4, img.lxc4, s)) || (*rc = upload_vec(g->pol, img.pol, s)) ||
        (*rc = upload_vec(g->polbloom, img.pol_bloom, s)) ||
        (*rc = upload_vec(g->lxc6, img.lxc6, s)))
        return nullptr;
    g->lxc4_mask = img.lxc4_mask;
    g->lxc6_mask = img.lxc6_mask;
    g->lxc4_lds = img.lxc4.size() <= LXC_LDS_MAX_SLOTS;
    g->lxc6_lds = img.lxc6.size() <= LXC6_LDS_MAX_SLOTS;
    g->pol_bloom_words = (uint32_t)img.pol_bloom.size();
    g->pol_host = img.pol;
    g->n_eps = img.n_eps;
    g->n_eps6 = img.n_eps6;
    g->pol_loc = std::move(img.pol_loc);
    g->ctr_owner = std::move(img.ctr_owner);
    g->bytes = sizeof(LxcSlot) * img.lxc4.size() + sizeof(PolSlot) * img.pol.size() +
               4ull * img.pol_bloom.size() + sizeof(Lxc6Slot) * img.lxc6.size();
    // drop notifications: {SECLABEL, ifindex} by LXC_ID (struct
    // endpoint_info), and the SECLABELs the epoch's verdicts use
    g->seclabel = c->seclabel;
    std::vector<uint2> info(65536, make_uint2(0, 0));
    for (uint32_t id = 0; id < 65536; id++)
        info[id].x = c->seclabel[id];
    for (Map *m : ms) {
        if (m->role != ROLE_LXC)
            continue;
        for (auto &e : m->kv) {
            uint32_t ifx;
            uint16_t id;
            memcpy(&ifx, e.second.val.data(), 4);
            memcpy(&id, e.second.val.data() + 6, 2);
            info[id].y = ifx;
        }
    }
    if ((*rc = upload_vec(g->ep_info, info, s)))
        return nullptr;
    g->nat4 = img.nat4;
    if (!img.nat6.empty()) {
        std::vector<uint4> n6(65536, make_uint4(0, 0, 0, 0));
        for (const auto &kv : img.nat6)
            n6[kv.first] = kv.second;
        if ((*rc = upload_vec(g->nat6, n6, s)))
            return nullptr;
    }
    return g;
}

std::shared_ptr<GLb> build_lbg(const HostImage &img, hipStream_t s, int *rc)
{
    auto g = std::make_shared<GLb>();
    if ((*rc = upload_vec(g->lb4, img.lb4, s)) || (*rc = upload_vec(g->rnat4, img.rnat4, s)) ||
        (*rc = upload_vec(g->lb6, img.lb6, s)) || (*rc = upload_vec(g->rnat6, img.rnat6, s)))
        return nullptr;
    g->lb4_mask = img.lb4_mask;
    g->n_lb4 = img.n_lb4;
    g->lb6_mask = img.lb6_mask;
    g->n_lb6 = img.n_lb6;
    g->bytes = 16ull * img.lb4.size() + 8ull * img.rnat4.size() + 16ull * img.lb6.size() +
               16ull * img.rnat6.size();
    return g;
}

std::shared_ptr<GCt> build_ctg(HostImage &img, const std::vector<Map *> &ms, hipStream_t s,
                               int *rc)
{
    auto g = std::make_shared<GCt>();
    if ((*rc = upload_vec(g->ct4, img.ct4, s)) || (*rc = upload_vec(g->ct6, img.ct6, s)) ||
        (*rc = upload_vec(g->ct4_lb, img.ct4_lb, s)) ||
        (*rc = upload_vec(g->ct6_lb, img.ct6_lb, s)))
        return nullptr;
    const size_t nslots = img.ct4.size() + img.ct6.size();
    if (nslots && (*rc = g->ct_sum.zeros(4 * nslots, s)))
        return nullptr;
    const size_t n4 = img.ct4.size(), n6 = img.ct6.size();
    if (nslots) {   // the report states into their lines (through a staging copy)
        DevBuf tm;
        if (g->ct_st.ensure(sizeof(CtState) * nslots) ||
            tm.ensure(sizeof(CtTimer) * std::max(n4, n6))) {
            *rc = -ENOMEM;
            return nullptr;
        }
        g->ct_st.bytes = sizeof(CtState) * nslots;
        CtState *st = (CtState *)g->ct_st.p;
        for (int f = 0; f < 2; f++) {
            const std::vector<CtTimer> &v = f ? img.ct6_tm : img.ct4_tm;
            if (v.empty())
                continue;
            if (hipMemcpyAsync(tm.p, v.data(), sizeof(CtTimer) * v.size(),
                               hipMemcpyHostToDevice, s) != hipSuccess ||
                ct_state_init(st + (f ? n4 : 0), (const CtTimer *)tm.p, v.size(), s) ||
                hipStreamSynchronize(s) != hipSuccess) {   // (tm is freed on return)
                *rc = -EIO;
                return nullptr;
            }
        }
    }
    if (n4 && (*rc = g->ct4_ms.zeros(12 * n4, s)))   // (ms, then lh)
        return nullptr;
    if (n6 && (*rc = g->ct6_ms.zeros(12 * n6, s)))
        return nullptr;
    for (Map *m : ms)
        if (m->role == ROLE_CT4 || m->role == ROLE_CT6)
            g->ct_maps[ct_map_key(m->role == ROLE_CT4 ? 4 : 6,
                                  ct_owner_word((uint32_t)std::max(m->policy_lxc, 0),
                                                m->policy_lxc >= 0),
                                  m->ct_any)] = m;
    g->ct4_mask = img.ct4_mask;
    g->ct4_probe = img.ct4_probe;
    g->ct6_mask = img.ct6_mask;
    g->ct6_probe = img.ct6_probe;
    g->n_ct4 = img.n_ct4;
    g->n_ct6 = img.n_ct6;
    g->n_nat46 = img.n_nat46;
    g->bytes = sizeof(Ct4Slot) * img.ct4.size() + sizeof(Ct6Slot) * img.ct6.size() +
               (sizeof(CtState) + 4) * nslots + 8ull * (n4 + n6) + 16ull * img.ct4_lb.size();
    g->slots4 = img.ct4.size();
    g->slots6 = img.ct6.size();
    g->ct4_host = std::move(img.ct4);
    g->ct6_host = std::move(img.ct6);
    return g;
}

// the kernels' view of an epoch's groups
void assemble(Epoch &E)
{
    DevTables &T = E.T;
    T = DevTables{};
    const GIpc &I = *E.ipc;
    const GIpc6 &I6 = *E.ipc6;
    const GPf &P = *E.pf;
    const GEp &D = *E.ep;
    const GCt &C = *E.ct;
    const GLb &B = *E.lb;
    T.l4d = (const uint4 *)I.l4d.p;
    T.l4c = (const uint32_t *)I.l4c.p;
    T.l4l = (const uint64_t *)I.l4l.p;
    T.tbl24 = (const uint32_t *)I.tbl24.p;
    T.tbl8 = (const uint32_t *)I.tbl8.p;
    T.lbl_ovf = (const uint32_t *)I.ovf.p;
    T.ipc6 = I6.ipc6;
    T.pf_tbl24 = (const uint32_t *)P.pf24.p;
    T.pf_tbl8 = (const uint32_t *)P.pf8.p;
    T.pf_fix = (const uint32_t *)P.pffix.p;
    T.pf_fix_mask = P.fix_mask;
    T.pf_fix_zero = P.fix_zero;
    T.pf_bloom = (const uint32_t *)P.pfbloom.p;
    T.pf_bloom_words = P.bloom_words;
    T.pf6_fix = P.fix;
    T.pf6_bloom = (const uint32_t *)P.pf6bloom.p;
    T.pf6_bloom_words = P.bloom6_words;
    T.pf6_dyn = P.dyn;
    T.lxc4 = (const LxcSlot *)D.lxc4.p;
    T.lxc4_mask = D.lxc4_mask;
    T.lxc4_lds = D.lxc4_lds;
    T.lxc6 = (const Lxc6Slot *)D.lxc6.p;
    T.lxc6_mask = D.lxc6_mask;
    T.lxc6_lds = D.lxc6_lds;
    T.pol = (const PolSlot *)D.pol.p;
    T.pol_bloom = (const uint32_t *)D.polbloom.p;
    T.pol_bloom_words = D.pol_bloom_words;
    T.n_ctr = (uint32_t)D.ctr_owner.size();
    // (a table a device apply may fill counts even while empty)
    T.ct4 = (C.n_ct4 || C.slots4) ? (const Ct4Slot *)C.ct4.p : nullptr;
    T.ct6 = (C.n_ct6 || C.slots6) ? (const Ct6Slot *)C.ct6.p : nullptr;
    T.ct_st = (CtState *)C.ct_st.p;
    T.ct_sum = (uint32_t *)C.ct_sum.p;
    T.ct4_mask = C.ct4_mask;
    // the device CT apply inserts in place: lookups walk to a free slot
    T.ct4_probe = C.ct4_mask;
    T.ct6_mask = C.ct6_mask;
    T.ct6_probe = C.ct6_mask;
    T.ct6_acct_base = (uint32_t)C.slots4;
    T.lb4 = B.n_lb4 ? (const uint4 *)B.lb4.p : nullptr;
    T.lb4_mask = B.lb4_mask;
    T.rnat4 = (const uint2 *)B.rnat4.p;
    T.ct4_lb = T.ct4 ? (const uint4 *)C.ct4_lb.p : nullptr;
    T.lb6 = B.n_lb6 ? (const uint4 *)B.lb6.p : nullptr;
    T.lb6_mask = B.lb6_mask;
    T.rnat6 = (const uint4 *)B.rnat6.p;
    T.ct6_lb = T.ct6 ? (const uint4 *)C.ct6_lb.p : nullptr;
    cfc_stats &st = E.st;
    st = cfc_stats{};
    st.epoch = E.id;
    st.device_bytes = I.bytes + I6.bytes + P.bytes + D.bytes + C.bytes + B.bytes;
    st.ipcache_v4_prefixes = I.n_prefix4;
    st.lpm4_tbl8_groups = I.tbl8_groups;
    st.policy_entries = T.n_ctr;
    st.endpoints = D.n_eps;
    st.prefilter_v4_fix = P.n_fix4;
    st.prefilter_v4_dyn = P.n_dyn4;
    st.lpm4_layout = (uint32_t)I.layout;
    st.lpm4_kib = I.lpm4_kib;
    st.ipcache_v6_prefixes = I6.n_prefix6;
    st.lpm6_lengths = I6.lpm6_lengths;
    st.lpm6_groups = I6.lpm6_groups;
    st.lpm6_kib = I6.lpm6_kib;
    st.endpoints_v6 = D.n_eps6;
    st.prefilter_v6_fix = P.n_fix6;
    st.prefilter_v6_dyn = P.n_dyn6;
    st.ct4_entries = C.n_ct4;
    st.ct6_entries = C.n_ct6;
}

// Build the next epoch: re-flatten and upload the groups whose maps changed,
// share the others with the current epoch, swap without draining the
// device (the old epoch is retired until the streams that used it pass the
// swap point).
// Value-only overwrites since the last commit, patched into the live
// tables in place (a concurrent launch sees the old or the new value, as a
// BPF program racing a map update does): IPv6 ipcache labels, policy
// entries' proxy ports.  IPv4 ipcache labels rebuild that (small) group.
// Returns the groups that still need a rebuild.
bool patch_ct(cfc_ctx *c, hipStream_t s);

unsigned patch_touched(cfc_ctx *c, unsigned groups, hipStream_t s)
{
    Epoch &E = *c->epoch;
    for (auto &kv : c->maps) {
        Map *m = kv.second.get();
        if (m->touched.empty())
            continue;
        if (m->role == ROLE_IPCACHE) {
            for (auto &t : m->touched) {
                auto it = m->kv.find(t.first);
                if (it == m->kv.end())
                    continue;
                const bool v6 = t.first.size() > 7 && (uint8_t)t.first[7] == 2;
                if (!v6) {
                    groups |= GROUP_IPCACHE4;
                    continue;
                }
                if (groups & GROUP_IPCACHE6)
                    continue;
                Pfx6 p;
                const int64_t slot = ipcache_v6_entry(t.first, it->second.val, &p)
                                         ? lpm6_find_slot(E.ipc6->host, p) : -1;
                if (slot < 0) {
                    groups |= GROUP_IPCACHE6;
                    continue;
                }
                uint32_t *lab;
                char *dev;
                if (slot & L6_S64) {   // (a /1-/64 prefix: its 16-byte slot's z)
                    uint4 &d = E.ipc6->host.slots64[slot & ~L6_S64];
                    lab = &d.z;
                    dev = (char *)E.ipc6->l6[3].p + 16 * (slot & ~L6_S64) + 8;
                } else {
                    L6Slot &d = E.ipc6->host.slots[slot];
                    lab = &d.label;
                    dev = (char *)E.ipc6->l6[0].p + sizeof(L6Slot) * slot +
                          offsetof(L6Slot, label);
                }
                *lab = p.label;
                if (hipMemcpyAsync(dev, lab, 4, hipMemcpyHostToDevice, s) != hipSuccess)
                    groups |= GROUP_IPCACHE6;
            }
        } else if (m->role == ROLE_POLICY && !(groups & GROUP_ENDPOINTS)) {
            auto loc = E.ep->pol_loc.find(m->policy_lxc);
            for (auto &t : m->touched) {
                auto it = m->kv.find(t.first);
                if (it == m->kv.end() || loc == E.ep->pol_loc.end())
                    continue;
                uint64_t key;
                memcpy(&key, t.first.data(), 8);
                if (((uint8_t)t.first[7] & 0xFE) != 0)
                    continue;   // not in the device table (flatten.cpp)
                const uint32_t mask = loc->second.mask, base = loc->second.base;
                uint32_t sl = pol_slot(pol_key_pre((uint32_t)key, (uint32_t)(key >> 32)), mask);
                PolSlot *tab = E.ep->pol_host.data() + base;
                uint32_t n = 0;
                while (tab[sl].key != key && tab[sl].key != POL_EMPTY && n++ <= mask)
                    sl = (sl + 1) & mask;
                if (tab[sl].key != key) {
                    groups |= GROUP_ENDPOINTS;
                    break;
                }
                memcpy(&tab[sl].proxy_port, it->second.val.data(), 2);
                char *dev = (char *)E.ep->pol.p + sizeof(PolSlot) * (base + sl) +
                            offsetof(PolSlot, proxy_port);
                if (hipMemcpyAsync(dev, &tab[sl].proxy_port, 2, hipMemcpyHostToDevice,
                                   s) != hipSuccess)
                    groups |= GROUP_ENDPOINTS;
            }
        }
    }
    bool ct = false;
    for (auto &kv : c->maps)
        ct |= kv.second->ct() && !kv.second->touched.empty();
    if (ct && !(groups & GROUP_CT)) {
        if (!patch_ct(c, s)) {
            groups |= GROUP_CT;
        } else {
            const GCt &G = *E.ct;
            E.st.ct4_entries = G.n_ct4;
            E.st.ct6_entries = G.n_ct6;
        }
    }
    return groups;
}

// CT inserts, deletes and value changes since the last commit (the CT maps'
// touched journal) patched into the live CT table: a new entry takes the
// first free or deleted slot of its probe sequence, a deleted one becomes
// CT_TOMBSTONE, a changed value rewrites the slot's report state (CtTimer);
// the accounting of a replaced slot restarts from zero.  The records go up
// in one upload and one scatter launch (k_patch16).  False, with nothing
// changed, when the table would pass 3/4 load (or lacks the family): the
// group is rebuilt instead.
bool patch_ct(cfc_ctx *c, hipStream_t s)
{
    GCt &G = *c->epoch->ct;
    if (mirror_sync(G, s))
        return false;
    uint64_t ins[2] = {0, 0}, any[2] = {0, 0};
    for (auto &kv : c->maps) {
        const Map *m = kv.second.get();
        if (!m->ct())
            continue;
        const int f = m->role == ROLE_CT6;
        for (auto &t : m->touched) {
            any[f]++;
            ins[f] += (t.second & TOUCH_INSERT) ? 1 : 0;
            // an entry with LB state into a table without the LB state
            // array: rebuilt with it
            if (!f && !G.ct4_lb.p) {
                auto it = m->kv.find(t.first);
                if (it != m->kv.end()) {
                    const uint4 l = ct_lb_of(it->second.val);
                    if (l.x | l.y)
                        return false;
                }
            }
        }
    }
    const uint64_t size[2] = {G.slots4, G.slots6};
    const uint64_t used[2] = {(uint64_t)G.n_ct4 + G.tomb4, (uint64_t)G.n_ct6 + G.tomb6};
    for (int f = 0; f < 2; f++)
        if (any[f] && (!size[f] || 4 * (used[f] + ins[f]) > 3 * size[f]))
            return false;
    std::unordered_map<uint64_t, size_t> at_addr;
    std::vector<Patch16> &rec = c->patch_host;
    rec.clear();
    auto put = [&](const void *dst, const void *val) {
        Patch16 p{};
        memcpy(p.val, val, 16);
        p.dst = (uint64_t)(uintptr_t)dst;
        auto r = at_addr.emplace(p.dst, rec.size());
        if (r.second)
            rec.push_back(p);
        else
            rec[r.first->second] = p;
    };
    static const uint32_t zero[4] = {0, 0, 0, 0};
    auto zero_acct = [&](uint64_t slot) {
        char *a = (char *)((CtState *)G.ct_st.p + slot)->acct;
        put(a, zero);
        put(a + 16, zero);
    };
    for (auto &kv : c->maps) {
        Map *m = kv.second.get();
        if (!m->ct() || m->touched.empty())
            continue;
        const bool v6 = m->role == ROLE_CT6;
        for (auto &t : m->touched) {
            Ct4Slot k4;
            Ct6Slot k6;
            if (!ct_slot_of(m, t.first, &k4, &k6))
                continue;   // no lookup reaches it: not in the device table
            auto it = m->kv.find(t.first);
            const bool present = it != m->kv.end();
            // the key's slot, else the first free or deleted one
            const uint32_t mask = (uint32_t)size[v6] - 1;
            int64_t at = -1, slot = -1;
            uint32_t p = 0, pfree = 0;
            uint32_t i = v6 ? ct_home6(k6.d, k6.s, k6.z, k6.w) & mask
                            : ct_home4(k4.x, k4.y, k4.z, k4.w) & mask;
            for (;; i = (i + 1) & mask, p++) {
                const uint32_t w = v6 ? G.ct6_host[i].w : G.ct4_host[i].w;
                if (w == 0 || w == CT_TOMBSTONE) {
                    if (slot < 0) {
                        slot = i;
                        pfree = p;
                    }
                    if (w == 0)
                        break;
                    continue;
                }
                const bool eq = v6 ? (G.ct6_host[i].z == k6.z && w == k6.w &&
                                      !memcmp(G.ct6_host[i].d, k6.d, 16) &&
                                      !memcmp(G.ct6_host[i].s, k6.s, 16))
                                   : (G.ct4_host[i].x == k4.x && G.ct4_host[i].y == k4.y &&
                                      G.ct4_host[i].z == k4.z && w == k4.w);
                if (eq) {
                    at = i;
                    break;
                }
            }
            const uint64_t acct = v6 ? size[0] + (uint64_t)(at >= 0 ? at : slot)
                                     : (uint64_t)(at >= 0 ? at : slot);
            CtState *tm = (CtState *)G.ct_st.p + (v6 ? size[0] : 0);
            if (present) {
                const CtTimer v = ct_timer_of(it->second.val);
                c->nat46_seen |= !v6 && (v.flags & CTT_NAT46);
                if (at < 0) {   // insert
                    at = slot;
                    if (v6) {
                        const bool tomb = G.ct6_host[at].w == CT_TOMBSTONE;
                        G.tomb6 -= tomb;
                        G.n_ct6++;
                        G.ct6_host[at] = k6;
                        G.ct6_probe = std::max(G.ct6_probe, pfree);
                        const uint32_t *w = (const uint32_t *)&k6;
                        char *d = (char *)G.ct6.p + sizeof(Ct6Slot) * at;
                        put(d, w);
                        put(d + 16, w + 4);
                        put(d + 32, w + 8);
                    } else {
                        const bool tomb = G.ct4_host[at].w == CT_TOMBSTONE;
                        G.tomb4 -= tomb;
                        G.n_ct4++;
                        G.ct4_host[at] = k4;
                        G.ct4_probe = std::max(G.ct4_probe, pfree);
                        put((char *)G.ct4.p + sizeof(Ct4Slot) * at, &k4);
                    }
                    zero_acct(acct);
                } else if (t.second & (TOUCH_INSERT | TOUCH_ERASE)) {
                    zero_acct(acct);   // deleted and created again
                }
                put(&tm[at].tm, &v);
                const uint4 l = ct_lb_of(it->second.val);
                if (!v6 && G.ct4_lb.p)
                    put((uint4 *)G.ct4_lb.p + at, &l);
                if (v6 && G.ct6_lb.p) {
                    const uint4 l6 = make_uint4(l.x & 0xFFFF, l.y, 0, 0);
                    put((uint4 *)G.ct6_lb.p + at, &l6);
                }
            } else if (at >= 0) {       // delete
                if (v6) {
                    Ct6Slot d{};
                    d.w = CT_TOMBSTONE;
                    G.ct6_host[at] = d;
                    G.n_ct6--;
                    G.tomb6++;
                    const uint32_t *w = (const uint32_t *)&d;
                    char *dst = (char *)G.ct6.p + sizeof(Ct6Slot) * at;
                    put(dst + 32, w + 8);   // z, w: probes compare these first
                } else {
                    const Ct4Slot d{0, 0, 0, CT_TOMBSTONE};
                    G.ct4_host[at] = d;
                    G.n_ct4--;
                    G.tomb4++;
                    put((char *)G.ct4.p + sizeof(Ct4Slot) * at, &d);
                }
                zero_acct(acct);
            }
        }
    }
    if (rec.empty())
        return true;
    const size_t bytes = rec.size() * sizeof(Patch16);
    if (c->patch_dev.bytes < bytes) {
        if (c->patch_dev.p)
            (void)hipStreamSynchronize(s);
        if (c->patch_dev.zeros(std::max(bytes, (size_t)1 << 20), s))
            return false;
    }
    if (hipMemcpyAsync(c->patch_dev.p, rec.data(), bytes, hipMemcpyHostToDevice, s) !=
            hipSuccess ||
        launch_patch16((const Patch16 *)c->patch_dev.p, rec.size(), s))
        return false;
    return true;
}

int commit_locked(cfc_ctx *c, hipStream_t s)
{
    reap_retired(c);
    uint64_t sig[NGROUPS];
    group_sigs(c, sig);
    unsigned groups = 0;
    bool touched = false;
    for (int g = 0; g < NGROUPS; g++)
        if (!c->epoch || sig[g] != c->built_sig[g])
            groups |= 1u << g;
    for (auto &kv : c->maps)
        touched |= !kv.second->touched.empty() &&
                   (kv.second->role == ROLE_IPCACHE || kv.second->role == ROLE_POLICY ||
                    kv.second->ct());
    if (!groups && !touched)
        return 0;
    c->ct_gen++;
    int rc;
    // host-side CT changes or a CT rebuild: take the device's first
    if ((groups & GROUP_CT) || touched)
        if ((rc = ct_sync(c, s)))
            return rc;
    if (c->epoch && touched) {
        groups = patch_touched(c, groups, s);
        c->id_cover |= identity_cover_touched(c);
        c->epoch->T.id_cover = c->id_cover;
        if (!groups) {   // all patched in place: the epoch stays
            for (auto &kv : c->maps)
                kv.second->touched.clear();
            return hipStreamSynchronize(s) == hipSuccess ? 0 : -EIO;
        }
    }
    // counts made under the old layout go to the maps first: policy-entry
    // counters when the endpoint tables change, CT accounting when CT does
    if (groups & (GROUP_ENDPOINTS | GROUP_CT))
        if ((rc = fold_counters(c, s)))
            return rc;
    std::vector<Map *> ms;
    for (auto &kv : c->maps)
        ms.push_back(kv.second.get());
    HostImage img;
    img.ct_min4 = c->ct_min4;
    img.ct_min6 = c->ct_min6;
    build_image(ms, c->opts, &img, groups);

    auto E = std::make_shared<Epoch>();
    E->id = ++c->epoch_seq;
    rc = 0;
    E->ipc = (groups & GROUP_IPCACHE4) ? build_ipc(img, s, &rc) : c->epoch->ipc;
    if (!rc)
        E->ipc6 = (groups & GROUP_IPCACHE6) ? build_ipc6(img, s, &rc) : c->epoch->ipc6;
    if (!rc)
        E->pf = (groups & GROUP_PREFILTER) ? build_pf(img, s, &rc) : c->epoch->pf;
    if (!rc)
        E->ep = (groups & GROUP_ENDPOINTS) ? build_ep(c, img, ms, s, &rc) : c->epoch->ep;
    if (!rc)
        E->ct = (groups & GROUP_CT) ? build_ctg(img, ms, s, &rc) : c->epoch->ct;
    if (!rc)
        E->lb = (groups & GROUP_LB) ? build_lbg(img, s, &rc) : c->epoch->lb;
    if (rc)
        return rc;
    assemble(*E);
    if (groups & (GROUP_IPCACHE4 | GROUP_IPCACHE6))
        c->id_cover = identity_cover(ms);
    E->T.id_cover = c->id_cover;

    // counters for a new entry layout (the old ones were folded above)
    if (groups & GROUP_ENDPOINTS) {
        const size_t need = 2ull * E->T.n_ctr + METRIC_U64 + ID_U64;
        if (need != c->ctr_u64) {
            if (c->ctr) {
                (void)hipStreamSynchronize(s);
                (void)hipFree(c->ctr);
            }
            c->ctr = nullptr;
            if (hipMalloc((void **)&c->ctr, need * 8) != hipSuccess)
                return -ENOMEM;
            c->ctr_u64 = need;
        }
        if (hipMemsetAsync(c->ctr, 0, need * 8, s) != hipSuccess)
            return -EIO;
    }
    // the uploads read host vectors freed below; launches on other streams
    // keep reading the old epoch, which stays until they pass this point
    if (hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    if (c->epoch) {
        Retired r;
        r.e = c->epoch;
        for (hipStream_t st : c->streams) {
            hipEvent_t ev;
            if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
                hipEventRecord(ev, st) != hipSuccess) {
                (void)hipDeviceSynchronize();   // cannot track it: drain instead
                break;
            }
            r.ev.push_back(ev);
        }
        c->retired.push_back(std::move(r));
    }
    c->streams.clear();
    c->epoch = std::move(E);
    for (int g = 0; g < NGROUPS; g++)
        c->built_sig[g] = sig[g];
    for (auto &kv : c->maps)
        kv.second->touched.clear();
    return 0;
}

Map *get_map(cfc_ctx *c, int fd)
{
    auto it = c->fds.find(fd);
    return it == c->fds.end() ? nullptr : it->second;
}

bool role_geometry_ok(Role r, uint32_t type, uint32_t ks, uint32_t vs)
{
    switch (r) {
    case ROLE_IPCACHE: return type == MT_LPM_TRIE && ks == 24 && vs == 8;
    case ROLE_LXC: return (type == MT_HASH) && ks == 20 && vs == 48;
    case ROLE_POLICY: return type == MT_HASH && ks == 8 && vs == 24;
    case ROLE_METRICS: return type == MT_PERCPU_HASH && ks == 8 && vs == 16;
    case ROLE_PF4_FIX: return type == MT_HASH && ks == 8 && vs == 1;
    case ROLE_PF4_DYN: return type == MT_LPM_TRIE && ks == 8 && vs == 1;
    case ROLE_PF6_FIX: return type == MT_HASH && ks == 20 && vs == 1;
    case ROLE_PF6_DYN: return type == MT_LPM_TRIE && ks == 20 && vs == 1;
    case ROLE_CT4: return (type == MT_LRU_HASH || type == MT_HASH) && ks == 14 && vs == 56;
    case ROLE_CT6: return (type == MT_LRU_HASH || type == MT_HASH) && ks == 38 && vs == 56;
    case ROLE_LB4_SVC: return type == MT_HASH && ks == 8 && vs == 12;     // lbmap/ipv4.go:27
    case ROLE_LB4_RNAT: return type == MT_HASH && ks == 2 && vs == 6;     // :43
    default: return true;
    }
}

// a write to a counter-bearing map must see the counts of every packet
// classified before it (the kernel bumps them in place in the reference)
int before_counter_write(cfc_ctx *c, Map *m)
{
    if (m->ct())
        if (int rc = ct_sync(c, c->last_stream))
            return rc;
    if (m->role == ROLE_POLICY || m->role == ROLE_METRICS || m->role == ROLE_CT4 ||
        m->role == ROLE_CT6)
        return fold_counters(c, c->last_stream);
    return 0;
}

// the next set of timing events (grown on demand, reused after a collect)
const LaunchTiming *next_timing(cfc_ctx *c, bool v6)
{
    if (!c->timing)
        return nullptr;
    if (c->tused == c->tpool.size()) {
        LaunchTiming t;
        for (auto &e : t.ev)
            if (hipEventCreate(&e) != hipSuccess)
                return nullptr;
        c->tpool.push_back(t);
    }
    c->tpool[c->tused].v6 = v6;
    return &c->tpool[c->tused++];
}

void free_timing(cfc_ctx *c)
{
    for (auto &t : c->tpool)
        for (auto &e : t.ev)
            (void)hipEventDestroy(e);
    c->tpool.clear();
    c->tused = 0;
}

}  // namespace

extern "C" {

int cfc_abi_version(void) { return CFC_ABI_VERSION; }
int cfc_num_possible_cpus(void) { return 1; }

int cfc_open(int device, cfc_ctx **out)
{
    if (!out)
        return -EINVAL;
    if (device != CFC_DEVICE_NONE) {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
            return -ENODEV;
        if (device < 0 || device >= ndev)
            return -ENODEV;
        if (hipSetDevice(device) != hipSuccess)
            return -ENODEV;
    }
    auto *c = new cfc_ctx();
    c->device = device;
    if (device != CFC_DEVICE_NONE) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, device) == hipSuccess &&
            p.multiProcessorCount > 0)
            c->num_cus = p.multiProcessorCount;
        (void)hipEventCreateWithFlags(&c->last_done, hipEventDisableTiming);
        (void)hipEventCreateWithFlags(&c->nt_done, hipEventDisableTiming);
    }
    // the datapath owns cilium_metrics (bpf/lib/maps.h:35-41)
    auto m = std::make_unique<Map>();
    m->name = "cilium_metrics";
    m->role = ROLE_METRICS;
    m->type = MT_PERCPU_HASH;
    m->ksz = 8;
    m->vsz = 16;
    m->max_entries = 65536;  // METRICS_MAP_SIZE, node_config.h
    c->metrics = m.get();
    c->maps["cilium_metrics"] = std::move(m);
    *out = c;
    return 0;
}

void cfc_close(cfc_ctx *c)
{
    if (!c)
        return;
    if (c->device != CFC_DEVICE_NONE) {
        (void)hipSetDevice(c->device);
        (void)hipDeviceSynchronize();
    }
    for (Retired &r : c->retired)
        for (hipEvent_t e : r.ev)
            (void)hipEventDestroy(e);
    c->retired.clear();
    c->epoch.reset();
    free_timing(c);
    if (c->ctr)
        (void)hipFree(c->ctr);
    if (c->ws)
        (void)hipFree(c->ws);
    if (c->last_done)
        (void)hipEventDestroy(c->last_done);
    if (c->pend_ev)
        (void)hipEventDestroy(c->pend_ev);
    if (c->pend_cnt)
        (void)hipHostFree(c->pend_cnt);
    if (c->nt_done)
        (void)hipEventDestroy(c->nt_done);
    delete c;
}

int cfc_set_option(cfc_ctx *c, int option, int64_t value)
{
    if (!c)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    switch (option) {
    case CFC_OPT_LPM4:
        if (value < CFC_LPM4_AUTO || value > CFC_LPM4_TRIE)
            return -EINVAL;
        c->opts.lpm4 = (int)value;   // the next commit rebuilds (tables_sig)
        return 0;
    case CFC_OPT_TIMING:
        if (value != 0 && value != 1)
            return -EINVAL;
        if (c->device == CFC_DEVICE_NONE)
            return -ENODEV;
        c->timing = value != 0;
        return 0;
    case CFC_OPT_CT_APPLY:
        if (value != CFC_CT_APPLY_DEVICE && value != CFC_CT_APPLY_HOST)
            return -EINVAL;
        c->ct_apply_mode = (int)value;
        return 0;
    case CFC_OPT_CT_EVICT:
        if (value != 0 && value != 1)
            return -EINVAL;
        c->ct_evict = value != 0;
        return 0;
    default:
        return -EINVAL;
    }
}

int cfc_timing_collect(cfc_ctx *c, cfc_timing *out)
{
    if (!c || !out)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (c->device == CFC_DEVICE_NONE)
        return -ENODEV;
    memset(out, 0, sizeof(*out));
    for (size_t i = 0; i < c->tused; i++) {
        const LaunchTiming &t = c->tpool[i];
        float a = 0, b = 0;
        if (hipEventSynchronize(t.ev[2]) != hipSuccess ||
            hipEventElapsedTime(&a, t.ev[0], t.ev[1]) != hipSuccess ||
            hipEventElapsedTime(&b, t.ev[1], t.ev[2]) != hipSuccess)
            return -EIO;
        out->launches++;
        out->classify_ms += a;
        out->count_ms += b;
        if (t.v6) {
            out->launches_v6++;
            out->classify_v6_ms += a;
            out->count_v6_ms += b;
        }
    }
    c->tused = 0;
    return 0;
}

int cfc_map_open(cfc_ctx *c, const char *path, uint32_t type, uint32_t ks,
                 uint32_t vs, uint32_t max_entries, uint32_t flags, int *fd,
                 int *created)
{
    if (!c || !path || !fd)
        return -EINVAL;
    if (type != MT_HASH && type != MT_PERCPU_HASH && type != MT_LRU_HASH &&
        type != MT_LPM_TRIE)
        return -EINVAL;
    if (!ks || !vs || !max_entries || (type == MT_LPM_TRIE && ks <= 4))
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    std::string p(path);
    std::string base = p.substr(p.find_last_of('/') + 1);
    int lxc = -1, ct_any = 0;
    Role r = role_for(p, &lxc, &ct_any);
    if (!role_geometry_ok(r, type, ks, vs))
        return -EINVAL;
    std::string key = r == ROLE_NONE ? p : base;
    auto it = c->maps.find(key);
    int was_created = 0;
    Map *m;
    if (it != c->maps.end()) {
        m = it->second.get();
        // objCheck (pkg/bpf/bpf.go:306): same geometry or refuse
        if (m->type != type || m->ksz != ks || m->vsz != vs ||
            (m->role != ROLE_METRICS && m->max_entries != max_entries))
            return -EINVAL;
    } else {
        auto nm = std::make_unique<Map>();
        nm->name = key;
        nm->role = r;
        nm->policy_lxc = lxc;
        nm->ct_any = ct_any;
        nm->type = type;
        nm->ksz = ks;
        nm->vsz = vs;
        nm->max_entries = max_entries;
        nm->flags = flags;
        m = nm.get();
        c->maps[key] = std::move(nm);
        was_created = 1;
    }
    *fd = c->next_fd++;
    c->fds[*fd] = m;
    if (created)
        *created = was_created;
    return 0;
}

int cfc_map_close(cfc_ctx *c, int fd)
{
    if (!c)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    return c->fds.erase(fd) ? 0 : -EBADF;
}

int cfc_map_update(cfc_ctx *c, int fd, const void *key, const void *value,
                   uint64_t flags)
{
    if (!c || !key || !value)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    Map *m = get_map(c, fd);
    if (!m)
        return -EBADF;
    int rc = before_counter_write(c, m);
    return rc ? rc : m->update(key, value, flags);
}

int cfc_map_update_batch(cfc_ctx *c, int fd, const void *keys,
                         const void *values, uint64_t count, uint64_t flags)
{
    if (!c || (count && (!keys || !values)))
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    Map *m = get_map(c, fd);
    if (!m)
        return -EBADF;
    int rc = before_counter_write(c, m);
    if (rc)
        return rc;
    const size_t vb = m->value_bytes();
    for (uint64_t i = 0; i < count; i++) {
        rc = m->update((const uint8_t *)keys + i * m->ksz,
                       (const uint8_t *)values + i * vb, flags);
        if (rc)
            return rc;
    }
    return 0;
}

int cfc_map_lookup(cfc_ctx *c, int fd, const void *key, void *value)
{
    if (!c || !key || !value)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    Map *m = get_map(c, fd);
    if (m && m->ct())
        if (int rc = ct_sync(c, c->last_stream))
            return rc;
    return m ? m->lookup(key, value) : -EBADF;
}

int cfc_map_delete(cfc_ctx *c, int fd, const void *key)
{
    if (!c || !key)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    Map *m = get_map(c, fd);
    if (!m)
        return -EBADF;
    int rc = before_counter_write(c, m);
    return rc ? rc : m->erase(key);
}

int cfc_map_get_next_key(cfc_ctx *c, int fd, const void *key, void *next)
{
    if (!c || !next)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    Map *m = get_map(c, fd);
    if (m && m->ct())
        if (int rc = ct_sync(c, c->last_stream))
            return rc;
    return m ? m->next_key(key, next) : -EBADF;
}

int cfc_map_dump(cfc_ctx *c, int fd, void *keys, void *values, uint64_t cap,
                 uint64_t *n)
{
    if (!c || !n || (cap && (!keys || !values)))
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    Map *m = get_map(c, fd);
    if (!m)
        return -EBADF;
    if (m->ct())
        if (int rc = ct_sync(c, c->last_stream))
            return rc;
    const size_t vb = m->value_bytes();
    uint64_t k = 0;
    for (const auto &kv : m->kv) {
        if (k < cap) {
            memcpy((uint8_t *)keys + k * m->ksz, kv.first.data(), m->ksz);
            memcpy((uint8_t *)values + k * vb, kv.second.val.data(), vb);
        }
        k++;
    }
    *n = k;
    return 0;
}

int cfc_endpoint_config(cfc_ctx *c, uint16_t lxc_id, uint32_t seclabel)
{
    if (!c)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (c->seclabel[lxc_id] != seclabel) {
        c->seclabel[lxc_id] = seclabel;
        c->seclabel_gen++;
    }
    return 0;
}

int cfc_set_node_config(cfc_ctx *c, const cfc_node_config *cfg)
{
    if (!c || !cfg)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    c->node = *cfg;
    return 0;
}

int cfc_set_clock(cfc_ctx *c, uint32_t now_sec)
{
    if (!c)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    c->now = now_sec;
    return 0;
}

int cfc_get_node_config(cfc_ctx *c, cfc_node_config *cfg)
{
    if (!c || !cfg)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    *cfg = c->node;
    return 0;
}

int cfc_commit(cfc_ctx *c, void *stream)
{
    if (!c)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (c->device == CFC_DEVICE_NONE)
        return -ENODEV;
    (void)hipSetDevice(c->device);
    return commit_locked(c, (hipStream_t)stream);
}

}  // extern "C"

namespace {

// LXC_NAT46 (nat.hip): the hop batch of a classified batch whose kernel
// listed m > 0 headers for a hop — sorted into header order, gathered
// translated, classified as the other family (NAT64: the sending
// endpoint's IPv4 egress path; NAT46: ipv6_policy of the destination with
// the IPv4 path's source identity), its results scattered back.  Kept for
// the batch's cfc_ct_apply (by its cfc_out.ct).
template <class Hdr>
int nat_hop(cfc_ctx *c, const DevTables &T, const EgressArgs &ea, const Hdr &in,
            const cfc_out &out, int mode, uint16_t ep_lxc, hipStream_t s)
{
    constexpr bool V6 = std::is_same<Hdr, cfc_hdr_v6>::value;
    const void *key = out.ct ? (const void *)out.ct : (const void *)out.verdict;
    uint32_t m = 0;
    if (hipMemcpyAsync(&m, c->nat_cnt.p, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    if (!m) {
        auto it = c->nat.find(key);
        if (it != c->nat.end())
            it->second.family = 0;
        return 0;
    }
    if (m > in.n)
        return -EIO;
    if (c->nat.size() > 16) {   // records applied (or never) of other batches
        (void)hipStreamSynchronize(s);
        for (auto it = c->nat.begin(); it != c->nat.end();)
            it = it->second.family == 0 && it->first != key ? c->nat.erase(it) : std::next(it);
    }
    cfc_ctx::NatRec &r = c->nat[key];
    r.family = V6 ? 6 : 4;
    r.saddr = in.saddr;
    r.n = in.n;
    r.mode = mode;
    r.ep = ep_lxc;
    r.m = m;
    const size_t tb = nat_sort_tmp_bytes(m);
    const size_t m4 = 4ull * ((m + 3) & ~3u);   // (16-byte aligned arrays)
    const size_t rows = V6 ? 5 * m4 + m4 : 8 * m4 + 4 * m4 + m4;
    if (r.idx.ensure(4ull * m) || c->nat_tmp.ensure(tb) || r.rows.ensure(rows) ||
        r.outs.ensure(3 * m4 + 2 * m4))
        return -ENOMEM;
    uint32_t *idx = (uint32_t *)r.idx.p;
    if (int rc = nat_sort((const uint32_t *)c->nat_list.p, idx, m, in.n, c->nat_tmp.p, tb, s))
        return rc;
    char *rp = (char *)r.rows.p, *op = (char *)r.outs.p;
    r.o = cfc_out{};
    r.o.verdict = (int32_t *)op;
    r.o.identity = (uint32_t *)(op + m4);
    r.o.notify = out.notify ? (uint32_t *)(op + 2 * m4) : nullptr;
    r.o.action = (uint8_t *)(op + 3 * m4);
    r.o.ct = (uint8_t *)(op + 4 * m4);
    EgressArgs e2 = ea;
    e2.nat_idx = e2.nat_cnt = nullptr;
    e2.sums = nullptr;
    e2.svo = nullptr;   // (the hop rows are another batch)
    const int smode = V6 ? CFC_MODE_EGRESS : CFC_MODE_INGRESS;
    const WsLayout wl = ws_layout(m, T, smode, true);
    if (r.ws.ensure(wl.total))
        return -ENOMEM;
    DevTables Th = T;   // (a hop launch keeps no plain-hit summaries)
    Th.ct_sum = nullptr;
    int rc;
    if constexpr (V6) {   // NAT64: IPv4 egress rows
        NatHop4 h{};
        h.sa = (uint32_t *)rp;
        h.da = (uint32_t *)(rp + m4);
        h.pt = (uint32_t *)(rp + 2 * m4);
        h.mt = (uint32_t *)(rp + 3 * m4);
        h.hash = T.lb4 ? (uint32_t *)(rp + 4 * m4) : nullptr;
        h.tf = (uint8_t *)(rp + 5 * m4);
        r.h4 = cfc_hdr_v4{h.sa, h.da, h.pt, h.mt, nullptr, h.tf, m, h.hash};
        rc = nat64_gather(in, idx, m, ea.nat_v4, h, s);
        if (!rc)
            rc = launch_classify_v4(Th, r.h4, r.o, smode, e2, c->ctr, (uint32_t *)r.ws.p,
                                    c->num_cus, s, nullptr);
    } else {              // NAT46: IPv6 ingress rows
        NatHop6 h{};
        h.sa = (uint4 *)rp;
        h.da = (uint4 *)(rp + 4 * m4);
        h.pt = (uint32_t *)(rp + 8 * m4);
        h.mt = (uint32_t *)(rp + 9 * m4);
        h.mk = (uint32_t *)(rp + 10 * m4);
        h.id = (uint32_t *)(rp + 11 * m4);
        h.tf = (uint8_t *)(rp + 12 * m4);
        r.h6 = cfc_hdr_v6{(const uint8_t *)h.sa, (const uint8_t *)h.da, h.pt, h.mt, h.mk, h.tf,
                          m, nullptr};
        e2.nat_id = h.id;
        rc = nat46_gather(T, in, out.identity, idx, m, (const uint4 *)c->epoch->ep->nat6.p, h,
                          s);
        if (!rc)
            rc = launch_classify_v6(Th, r.h6, r.o, smode, e2, c->ctr, (uint32_t *)r.ws.p,
                                    c->num_cus, s, nullptr);
    }
    if (!rc)
        rc = nat_scatter(idx, m, r.o, out, s);
    c->n_nat_hops += m;
    if (rc || !out.ct)
        r.family = 0;   // (no apply follows)
    return rc;
}

// cfc_classify_v4 / _v6: validation, auto-commit, workspace, launch
template <class Hdr, class Launch>
int classify_one(cfc_ctx *c, const Hdr *in, const cfc_out *out, int mode,
                 uint16_t ep_lxc, void *stream, Launch launch)
{
    hipStream_t s = (hipStream_t)stream;
    int rc = commit_locked(c, s);
    if (rc)
        return rc;
    Epoch &E = *c->epoch;
    // the launch's copy of the epoch's tables, with the node constants
    DevTables T = E.T;
    T.v4_cluster_range = c->node.ipv4_cluster_range;
    T.v4_cluster_mask = c->node.ipv4_cluster_mask;
    T.host_ifindex = c->node.host_ifindex;
    T.now = c->now;
    for (int w = 0; w < 4; w++) {
        const uint8_t *b = c->node.router_ip6 + 4 * w;
        T.router6[w] = (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
    }
    EgressArgs ea{ep_lxc, E.ep->seclabel[ep_lxc], 0, 0, 0};
    {   // the sending endpoint's CT maps: its own, or the global ones
        for (auto &kv : c->maps)
            if ((kv.second->role == ROLE_CT4 || kv.second->role == ROLE_CT6) &&
                kv.second->policy_lxc == (int)ep_lxc)
                ea.ct_owner = ct_owner_word(ep_lxc, true);
    }
    if (mode == CFC_MODE_EGRESS) {
        auto it = E.ep->pol_loc.find(ep_lxc);
        if (it == E.ep->pol_loc.end())
            return -ENOENT;  // no endpoint program (policy map) for ep_lxc
        ea.pol_base = it->second.base;
        ea.pol_mask = it->second.mask;
    }
    // LXC_NAT46: the kernel lists the headers that take a hop — NAT64 from
    // an IPv6 egress batch of an endpoint with LXC_IPV4, NAT46 from an IPv4
    // ingress batch while an entry may carry nat46 and an endpoint has an
    // IPv6 address
    bool nat_list = false;
    if constexpr (std::is_same<Hdr, cfc_hdr_v6>::value) {
        if (mode == CFC_MODE_EGRESS) {
            auto it = E.ep->nat4.find(ep_lxc);
            ea.nat_v4 = it == E.ep->nat4.end() ? 0u : it->second;
            nat_list = ea.nat_v4 != 0 && in->n;
        }
    } else {
        T.nat46 = (mode == CFC_MODE_INGRESS || mode == CFC_MODE_FULL) && E.T.ct4 &&
                  E.ep->nat6.p && (E.ct->n_nat46 || c->nat46_seen);
        nat_list = T.nat46 && in->n;
    }
    if (nat_list) {
        if (c->nat_list.bytes < 4 * in->n) {
            (void)hipStreamSynchronize(s);
            if (c->nat_list.ensure(4 * in->n))
                return -ENOMEM;
        }
        if (c->nat_cnt.ensure(16) || hipMemsetAsync(c->nat_cnt.p, 0, 4, s) != hipSuccess)
            return -ENOMEM;
        ea.nat_idx = (uint32_t *)c->nat_list.p;
        ea.nat_cnt = (uint32_t *)c->nat_cnt.p;
    }
    const WsLayout wl = ws_layout(in->n, E.T, mode,
                                  E.T.ct4 || E.T.ct6 || out->ct || E.T.lb4 || E.T.rnat4 ||
                                      E.T.lb6 || E.T.rnat6);
    const size_t need = wl.total;
    c->last_cls.valid = false;
    if (need > c->ws_bytes) {
        if (c->ws) {
            (void)hipDeviceSynchronize();
            (void)hipFree(c->ws);
        }
        c->ws = nullptr;
        c->ws_bytes = 0;
        if (hipMalloc((void **)&c->ws, need) != hipSuccess)
            return -ENOMEM;
        c->ws_bytes = need;
    }
    // the workspace is shared: order this launch after the previous one
    if (c->ctr_pending && c->last_stream != s)
        (void)hipStreamWaitEvent(s, c->last_done, 0);
    order_after_launches(c, s);
    // an egress batch with services: the CT_SERVICE entry each header finds
    // in packet order (the creates and re-selections of the headers before
    // it), handed to the launch's service step.  (After the waits above:
    // its per-context words and keys are shared with the previous launch,
    // which may still read them on another stream, and it reads the CT
    // table that launch's apply may still write.)
    uint32_t nsvo = 0;
    if (mode == CFC_MODE_EGRESS && in->n &&
        (std::is_same<Hdr, cfc_hdr_v6>::value ? E.T.lb6 != nullptr : E.T.lb4 != nullptr)) {
        const uint64_t n = in->n;
        const size_t tb = svc_order_tmp_bytes(n);
        if (c->svo_keys.bytes < 8 * n || c->svo.bytes < 4 * n || c->svo_tmp.bytes < tb) {
            (void)hipStreamSynchronize(s);
            if (c->svo_keys.ensure(8 * n) || c->svo_keys2.ensure(8 * n) || c->svo_tmp.ensure(tb) ||
                c->svo.zeros(4 * n, s))
                return -ENOMEM;
        }
        if (!c->svo_cnt.p && c->svo_cnt.zeros(16, s))   // (words 2-3: svc_ordered)
            return -ENOMEM;
        SvoArgs sa{(const uint32_t *)in->saddr, (const uint32_t *)in->daddr, in->ports, in->meta,
                   in->hash, n, ep_lxc, ea.ct_owner,
                   (uint64_t *)c->svo_keys.p, (uint64_t *)c->svo_keys2.p, (uint32_t *)c->svo.p,
                   (uint32_t *)c->svo_cnt.p, c->svo_tmp.p, c->svo_tmp.bytes};
        if ((rc = svc_order(T, sa, std::is_same<Hdr, cfc_hdr_v6>::value, &nsvo, s))) {
            // (words it may have set before failing: zero for the next launch)
            (void)hipMemsetAsync(c->svo.p, 0, 4 * n, s);
            return rc;
        }
        if (nsvo)
            ea.svo = (const uint32_t *)c->svo.p;
    }
    // plain-hit summaries: only of this launch (a batch with NAT hops keeps
    // none: its apply takes the scan's)
    if (c->sum_pending)   // (the last launch's went unused)
        c->sum_want = false;
    c->sum_pending = false;
    if (nat_list || !out->ct || !c->sum_want)   // (no CT bytes: no apply can follow)
        T.ct_sum = nullptr;
    if (T.ct_sum && c->sum_dirty) {
        if (hipMemsetAsync(T.ct_sum, 0, E.ct->ct_sum.bytes, s) != hipSuccess)
            return -EIO;
        c->sum_dirty = false;
    }
    bool sums = false;
    ea.sums = &sums;
    // the apply's work list (kern_common.hpp wl_want): a launch whose apply
    // can take the sparse passes — plain hits summarised (ct_sum), no load
    // balancer or packet outputs (the service-step variants), no NAT hop,
    // no monitor words (those replay every hit)
    {
        const bool v6 = std::is_same<Hdr, cfc_hdr_v6>::value;
        const bool lbk = v6 ? (E.T.lb6 || E.T.rnat6 || out->pkt_saddr) : (E.T.lb4 || E.T.rnat4);
        if (out->ct && in->n && T.ct_sum && !nat_list && !lbk && !out->notify &&
            mode != CFC_MODE_XDP && !getenv("CFC_DENSE_APPLY")) {
            const uint64_t words = (in->n + 63) / 64;
            if (c->cta_wbits.bytes < 16 * words) {
                (void)hipStreamSynchronize(s);
                if (c->cta_wbits.ensure(16 * words))
                    return -ENOMEM;
            }
            ea.wbits = (uint64_t *)c->cta_wbits.p;
            ea.wprobe = ea.wbits + words;
        }
    }
    rc = launch(T, *in, *out, mode, ea, c->ctr, c->ws, c->num_cus, s,
                in->n ? next_timing(c, std::is_same<Hdr, cfc_hdr_v6>::value) : nullptr);
    c->sum_dirty |= sums;
    c->sum_pending = sums;
    if (nsvo &&   // (the entry words zero again for the next launch, on every exit)
        hipMemsetAsync(c->svo.p, 0, 4 * in->n, s) != hipSuccess && !rc)
        rc = -EIO;
    if (rc)
        return rc;
    if (nat_list) {
        if ((rc = nat_hop(c, T, ea, *in, *out, mode, ep_lxc, s)))
            return rc;
    } else if (!c->nat.empty()) {
        auto it = c->nat.find(out->ct ? (const void *)out->ct : (const void *)out->verdict);
        if (it != c->nat.end())
            it->second.family = 0;
    }
    (void)hipEventRecord(c->last_done, s);
    c->last_stream = s;
    note_stream(c, s);
    c->ctr_pending = true;
    if (out->ct && in->n && wl.ct) {
        auto &L = c->last_cls;
        L.valid = true;
        L.family = std::is_same<Hdr, cfc_hdr_v4>::value ? 4 : 6;
        L.ct = out->ct;
        L.saddr = in->saddr;
        L.n = in->n;
        L.gen = c->ct_gen;
        L.mode = mode;
        L.ep = ep_lxc;
        L.k1 = wl.ct;
        L.k2 = mode == CFC_MODE_EGRESS ? wl.ct2 : 0;
        L.sum = sums;
        L.wl = ea.wbits && sums;
    }
    return 0;
}

// a batch's headers [a, a + m) as a batch of their own (same arrays)
cfc_hdr_v4 sub_batch(const cfc_hdr_v4 &h, uint64_t a, uint64_t m)
{
    cfc_hdr_v4 r = h;
    r.saddr += a;
    r.daddr += a;
    r.ports += a;
    r.meta += a;
    if (r.mark)
        r.mark += a;
    if (r.tcp_flags)
        r.tcp_flags += a;
    if (r.hash)
        r.hash += a;
    r.n = m;
    return r;
}

cfc_hdr_v6 sub_batch(const cfc_hdr_v6 &h, uint64_t a, uint64_t m)
{
    cfc_hdr_v6 r = h;
    r.saddr += 16 * a;
    r.daddr += 16 * a;
    r.ports += a;
    r.meta += a;
    if (r.mark)
        r.mark += a;
    if (r.tcp_flags)
        r.tcp_flags += a;
    if (r.hash)
        r.hash += a;
    r.n = m;
    return r;
}

cfc_out sub_out(const cfc_out &o, uint64_t a, bool v6)
{
    cfc_out r = o;
    r.verdict += a;
    r.identity += a;
    if (r.action)
        r.action += a;
    if (r.ct)
        r.ct += a;
    if (r.notify)
        r.notify += a;
    const uint64_t pw = v6 ? 4 * a : a;   // (IPv6: 16-byte address rows)
    if (r.pkt_saddr)
        r.pkt_saddr += pw;
    if (r.pkt_daddr)
        r.pkt_daddr += pw;
    if (r.pkt_ports)
        r.pkt_ports += a;
    return r;
}

template <class Hdr>
int ct_apply(cfc_ctx *c, int family, const Hdr *in, const cfc_out *out, int mode,
             uint16_t ep_lxc, void *stream);

// Traffic to itself (selfseg.hip): where an egress batch of `ep` must be
// cut so that no header's k1 is a key an earlier header of its own segment
// may have written.  Such keys have both addresses the sender's own
// (conntrack.h:487-494) or are a looped-back service flow's TUPLE_F_IN entry
// (:725-748), so only headers to one of these destinations take part: the
// endpoint's own addresses (cilium_lxc), and with services IPV4_LOOPBACK and
// the services that have the endpoint as a backend (lb4_local's loopback;
// an IPv6 service simply delivers back to it).  Header j is cut from an
// earlier listed header i of its segment when i's writes may hold one of
// j's lookup keys: any pair that involves a service or IPV4_LOOPBACK (the
// translated ports are not in the header); an ICMP error (its RELATED keys
// are every create's ICMP entry); an ICMP echo / other ICMP after an ICMP
// one; TCP / UDP after the same protocol on the same two ports, in either
// order (the answer finds the opening packet's entry).  cuts: segment
// starts after 0, ascending (empty: one launch).  One host wait, on egress
// batches with CT outputs only.
template <class Hdr>
int self_cuts(cfc_ctx *c, const Hdr &in, const cfc_out &out, int mode, uint16_t ep,
              hipStream_t s, std::vector<uint64_t> *cuts)
{
    constexpr bool V6 = std::is_same<Hdr, cfc_hdr_v6>::value;
    cuts->clear();
    if (mode != CFC_MODE_EGRESS || !out.ct || in.n < 2 || getenv("CFC_NO_SELF_CUTS"))
        return 0;
    int rc = commit_locked(c, s);
    if (rc)
        return rc;
    const Epoch &E = *c->epoch;
    if (V6 ? !E.T.ct6 : !E.T.ct4)
        return 0;
    const uint32_t al = V6 ? 16 : 4;
    std::vector<uint8_t> own;   // the endpoint's addresses, then the loopback ones
    auto add = [&](const uint8_t *a) {
        for (size_t o = 0; o < own.size(); o += al)
            if (!memcmp(&own[o], a, al))
                return;
        own.insert(own.end(), a, a + al);
    };
    for (auto &kv : c->maps) {
        if (kv.second->role != ROLE_LXC)
            continue;
        for (auto &e : kv.second->kv) {
            const uint8_t *k = (const uint8_t *)e.first.data();
            const uint8_t *v = (const uint8_t *)e.second.val.data();
            if (e.first.size() < 20 || e.second.val.size() < 12 || k[16] != (V6 ? 2 : 1))
                continue;
            uint16_t id;
            uint32_t fl;
            memcpy(&id, v + 6, 2);
            memcpy(&fl, v + 8, 4);
            if (id == ep && !(fl & 1))   // (not the host's own entry)
                add(k);
        }
    }
    const uint32_t n_own = (uint32_t)(own.size() / al);
    if (!n_own)
        return 0;
    // services with the endpoint as a backend (a slave slot whose target is
    // one of its addresses), and IPV4_LOOPBACK
    for (auto &kv : c->maps) {
        if (kv.second->role != (V6 ? ROLE_LB6_SVC : ROLE_LB4_SVC))
            continue;
        for (auto &e : kv.second->kv) {
            const uint8_t *k = (const uint8_t *)e.first.data();
            const uint8_t *v = (const uint8_t *)e.second.val.data();
            if (e.first.size() < al + 4 || e.second.val.size() < al)
                continue;
            uint16_t slave;
            memcpy(&slave, k + al + 2, 2);
            if (!slave)
                continue;
            for (uint32_t j = 0; j < n_own; j++)
                if (!memcmp(v, &own[j * al], al)) {
                    add(k);
                    break;
                }
        }
        if (!V6) {
            const uint32_t lo = IPV4_LOOPBACK;
            add((const uint8_t *)&lo);
        }
    }
    const uint32_t na = (uint32_t)(own.size() / al);
    const uint32_t cap = (uint32_t)std::min<uint64_t>(in.n, 1u << 24);
    if (c->self_addr.bytes < own.size() || c->self_rows.bytes < 16ull * cap) {
        (void)hipStreamSynchronize(s);
        if (c->self_addr.ensure(own.size()) || c->self_rows.ensure(16ull * cap))
            return -ENOMEM;
    }
    if (c->self_cnt.ensure(16))
        return -ENOMEM;
    // (the previous launch may still read these: order after it)
    if (c->ctr_pending && c->last_stream != s)
        (void)hipStreamWaitEvent(s, c->last_done, 0);
    if (hipMemcpyAsync(c->self_addr.p, own.data(), own.size(), hipMemcpyHostToDevice, s) !=
            hipSuccess ||
        hipMemsetAsync(c->self_cnt.p, 0, 4, s) != hipSuccess)
        return -EIO;
    SelfArgs A{(const void *)in.daddr, in.ports, in.meta, in.n, (const uint32_t *)c->self_addr.p,
               na, (uint4 *)c->self_rows.p, (uint32_t *)c->self_cnt.p, cap};
    if ((rc = self_mark(A, V6, s)))
        return rc;
    uint32_t m = 0;
    if (hipMemcpyAsync(&m, c->self_cnt.p, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    if (m < 2)
        return 0;
    if (m > cap)
        return -E2BIG;
    std::vector<uint4> rows(m);
    if (hipMemcpyAsync(rows.data(), c->self_rows.p, 16ull * m, hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    std::sort(rows.begin(), rows.end(), [](const uint4 &a, const uint4 &b) { return a.x < b.x; });
    self_cut_rule(rows, n_own, V6, cuts);   // (selfcut.hpp)
    return 0;
}

template <class Hdr, class Launch>
int classify(cfc_ctx *c, const Hdr *in, const cfc_out *out, int mode,
             uint16_t ep_lxc, void *stream, Launch launch)
{
    if (!c || !in || !out || !out->verdict || !out->identity)
        return -EINVAL;
    if (in->n && (!in->saddr || !in->daddr || !in->ports || !in->meta))
        return -EINVAL;
    if (mode < CFC_MODE_INGRESS || mode > CFC_MODE_FULL)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (c->device == CFC_DEVICE_NONE)
        return -ENODEV;
    (void)hipSetDevice(c->device);
    hipStream_t s = (hipStream_t)stream;
    constexpr bool V6 = std::is_same<Hdr, cfc_hdr_v6>::value;
    c->seg.valid = false;
    std::vector<uint64_t> cuts;
    int rc = self_cuts(c, *in, *out, mode, ep_lxc, s, &cuts);
    if (rc)
        return rc;
    if (cuts.empty())
        return classify_one(c, in, out, mode, ep_lxc, stream, launch);
    // the segments in order: each classified against the maps the ones
    // before it left, and folded into them before the next (the caller's
    // cfc_ct_apply folds the last)
    cuts.push_back(in->n);
    uint64_t a = 0;
    for (size_t k = 0; k < cuts.size(); k++) {
        const uint64_t b = cuts[k];
        const Hdr si = sub_batch(*in, a, b - a);
        const cfc_out so = sub_out(*out, a, V6);
        if ((rc = classify_one(c, &si, &so, mode, ep_lxc, stream, launch)))
            return rc;
        if (k + 1 < cuts.size()) {
            // (cfc_stats counts the caller's applies: these are the segments')
            const uint32_t nd = c->n_apply_dev, nh = c->n_apply_host;
            if ((rc = ct_apply(c, V6 ? 6 : 4, &si, &so, mode, ep_lxc, stream)))
                return rc;
            c->n_apply_dev = nd;
            c->n_apply_host = nh;
            c->n_self_segs++;
        }
        a = b;
    }
    c->seg.valid = true;
    c->seg.ct = out->ct;
    c->seg.saddr = in->saddr;
    c->seg.n = in->n;
    c->seg.off = cuts[cuts.size() - 2];
    c->seg.mode = mode;
    c->seg.family = V6 ? 6 : 4;
    c->seg.ep = ep_lxc;
    return 0;
}

}  // namespace

extern "C" {

int cfc_classify_v4(cfc_ctx *c, const cfc_hdr_v4 *in, const cfc_out *out,
                    int mode, uint16_t ep_lxc, void *stream)
{
    return classify(c, in, out, mode, ep_lxc, stream, launch_classify_v4);
}

int cfc_classify_v6(cfc_ctx *c, const cfc_hdr_v6 *in, const cfc_out *out,
                    int mode, uint16_t ep_lxc, void *stream)
{
    return classify(c, in, out, mode, ep_lxc, stream, launch_classify_v6);
}

}  // extern "C"

namespace {

// cfc_drop_notify_v4 / _v6
template <class Hdr>
int drop_notify(cfc_ctx *c, const Hdr *in, const cfc_out *out, int mode,
                uint16_t ep_lxc, cfc_drop_notify *rec, uint64_t *hdr_index,
                uint64_t cap, uint64_t *count, void *stream, int family,
                int traces)
{
    if (!c || !in || !out || !count || (cap && !rec))
        return -EINVAL;
    if (reinterpret_cast<uintptr_t>(rec) & 15)
        return -EINVAL;   // records are written as 16-byte stores (cfc.h)
    if (in->n && (!out->notify || !out->verdict || !out->identity ||
                  !in->saddr || !in->daddr || !in->ports || !in->meta))
        return -EINVAL;
    if (mode < CFC_MODE_INGRESS || mode > CFC_MODE_FULL)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (c->device == CFC_DEVICE_NONE)
        return -ENODEV;
    (void)hipSetDevice(c->device);
    hipStream_t s = (hipStream_t)stream;
    if (!c->epoch)
        return -ENOENT;   // nothing classified yet
    Epoch &E = *c->epoch;
    // the workspace and the endpoint table are shared: order this call
    // after the previous one when it ran on another stream
    if (c->nt_pending && c->nt_stream != s)
        (void)hipStreamWaitEvent(s, c->nt_done, 0);
    const size_t need = drop_notify_workspace_bytes(in->n);
    if (need > c->nt_ws.bytes) {
        (void)hipDeviceSynchronize();
        int rc = c->nt_ws.zeros(need, s);
        if (rc)
            return rc;
    }
    NotifyArgs a{};
    a.notify = out->notify;
    a.verdict = out->verdict;
    a.identity = out->identity;
    a.meta = in->meta;
    a.ports = in->ports;
    a.saddr = reinterpret_cast<const uint32_t *>(in->saddr);
    a.daddr = reinterpret_cast<const uint32_t *>(in->daddr);
    a.hash = in->hash;
    a.n = in->n;
    a.family = family;
    a.mode = mode;
    a.own_seclabel = E.ep->seclabel[ep_lxc];   // as the batch was classified
    a.ep_info = reinterpret_cast<const uint2 *>(E.ep->ep_info.p);
    a.host_ifindex = c->node.host_ifindex;
    a.traces = traces;
    a.rec = rec;
    a.hdr_index = hdr_index;
    a.cap = cap;
    a.count = count;
    int rc = launch_drop_notify(a, reinterpret_cast<uint64_t *>(c->nt_ws.p), s);
    if (rc)
        return rc;
    (void)hipEventRecord(c->nt_done, s);
    c->nt_stream = s;
    c->nt_pending = true;
    note_stream(c, s);   // it reads the epoch's endpoint table
    return 0;
}

}  // namespace

extern "C" {

int cfc_drop_notify_v4(cfc_ctx *c, const cfc_hdr_v4 *in, const cfc_out *out,
                       int mode, uint16_t ep_lxc, cfc_drop_notify *rec,
                       uint64_t *hdr_index, uint64_t cap, uint64_t *count,
                       void *stream)
{
    return drop_notify(c, in, out, mode, ep_lxc, rec, hdr_index, cap, count,
                       stream, 4, 0);
}

int cfc_drop_notify_v6(cfc_ctx *c, const cfc_hdr_v6 *in, const cfc_out *out,
                       int mode, uint16_t ep_lxc, cfc_drop_notify *rec,
                       uint64_t *hdr_index, uint64_t cap, uint64_t *count,
                       void *stream)
{
    return drop_notify(c, in, out, mode, ep_lxc, rec, hdr_index, cap, count,
                       stream, 6, 0);
}

int cfc_monitor_events_v4(cfc_ctx *c, const cfc_hdr_v4 *in, const cfc_out *out,
                          int mode, uint16_t ep_lxc, void *rec,
                          uint64_t *hdr_index, uint64_t cap, uint64_t *count,
                          void *stream)
{
    return drop_notify(c, in, out, mode, ep_lxc, (cfc_drop_notify *)rec, hdr_index,
                       cap, count, stream, 4, 1);
}

int cfc_monitor_events_v6(cfc_ctx *c, const cfc_hdr_v6 *in, const cfc_out *out,
                          int mode, uint16_t ep_lxc, void *rec,
                          uint64_t *hdr_index, uint64_t cap, uint64_t *count,
                          void *stream)
{
    return drop_notify(c, in, out, mode, ep_lxc, (cfc_drop_notify *)rec, hdr_index,
                       cap, count, stream, 6, 1);
}

int cfc_counters_device(cfc_ctx *c, uint64_t **dev, uint64_t *n)
{
    if (!c || !dev || !n)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (c->device == CFC_DEVICE_NONE)
        return -ENODEV;
    int rc = commit_locked(c, c->last_stream);
    if (rc)
        return rc;
    *dev = c->ctr;
    *n = c->ctr_u64;
    c->ctr_pending = true;  // the caller may write (all-reduce) into it
    return 0;
}

int cfc_counters_sync(cfc_ctx *c, void *stream)
{
    if (!c)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (c->device == CFC_DEVICE_NONE)
        return -ENODEV;
    (void)hipSetDevice(c->device);
    return fold_counters(c, (hipStream_t)stream);
}

int cfc_counters_clear(cfc_ctx *c, void *stream)
{
    if (!c)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (c->device == CFC_DEVICE_NONE)
        return -ENODEV;
    if (c->ctr && hipMemsetAsync(c->ctr, 0, c->ctr_u64 * 8,
                                 (hipStream_t)stream) != hipSuccess)
        return -EIO;
    c->ctr_pending = false;
    return 0;
}

int cfc_counters_export(cfc_ctx *c, uint64_t *dst, uint64_t n, void *stream)
{
    if (!c || !dst)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (c->device == CFC_DEVICE_NONE)
        return -ENODEV;
    int rc = commit_locked(c, (hipStream_t)stream);
    if (rc)
        return rc;
    if (n != c->ctr_u64)
        return -EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (c->ctr_pending && c->last_stream != s)
        (void)hipStreamWaitEvent(s, c->last_done, 0);
    if (hipMemcpyAsync(dst, c->ctr, n * 8, hipMemcpyDeviceToDevice, s) != hipSuccess ||
        hipMemsetAsync(c->ctr, 0, n * 8, s) != hipSuccess)
        return -EIO;
    (void)hipEventRecord(c->last_done, s);
    c->last_stream = s;
    note_stream(c, s);
    return 0;
}

int cfc_counters_import(cfc_ctx *c, const uint64_t *src, uint64_t n,
                        void *stream)
{
    if (!c || !src)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (c->device == CFC_DEVICE_NONE)
        return -ENODEV;
    if (!c->epoch || n != c->ctr_u64)
        return -EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (c->last_stream != s)
        (void)hipStreamWaitEvent(s, c->last_done, 0);
    int rc = launch_add_u64(c->ctr, src, n, s);
    if (rc)
        return rc;
    (void)hipEventRecord(c->last_done, s);
    c->last_stream = s;
    note_stream(c, s);
    c->ctr_pending = true;
    return 0;
}

int cfc_identity_counters(cfc_ctx *c, cfc_identity_count *rows, uint64_t cap,
                          uint64_t *n)
{
    if (!c || !n || (cap && !rows))
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    uint64_t k = 0;
    for (uint32_t id = 0; id < ID_SLOTS; id++)
        for (uint32_t dir = 0; dir < 2; dir++) {
            const uint64_t *v = &c->idc[id_index(dir, id, 0)];   // fwd, then drop
            if (!(v[0] | v[1] | v[2] | v[3]))
                continue;
            if (k < cap) {
                cfc_identity_count &r = rows[k];
                memset(&r, 0, sizeof(r));
                r.identity = id == ID_SLOTS - 1 ? CFC_IDENTITY_OUT_OF_RANGE : id;
                r.dir = (uint8_t)(dir + 1);
                r.fwd_packets = v[0];
                r.fwd_bytes = v[1];
                r.drop_packets = v[2];
                r.drop_bytes = v[3];
            }
            k++;
        }
    *n = k;
    return 0;
}

int cfc_get_stats(cfc_ctx *c, cfc_stats *st)
{
    if (!c || !st)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (!c->epoch)
        return -ENOENT;
    *st = c->epoch->st;
    st->ct_apply_device = c->n_apply_dev;
    st->ct_apply_host = c->n_apply_host;
    // (the device applies' count accumulates on the device: read after the
    // last launch, on this context's device; folded into the 64-bit total
    // and zeroed so the 32-bit device word never wraps)
    if (c->ord_cnt.p && c->device != CFC_DEVICE_NONE) {
        (void)hipSetDevice(c->device);
        uint32_t dev_changed = 0;
        if (c->last_done)
            (void)hipEventSynchronize(c->last_done);
        if (hipMemcpy(&dev_changed, (uint32_t *)c->ord_cnt.p + ORD_CHANGED, 4,
                      hipMemcpyDeviceToHost) == hipSuccess && dev_changed &&
            hipMemset((uint32_t *)c->ord_cnt.p + ORD_CHANGED, 0, 4) == hipSuccess)
            c->n_ord_changed += dev_changed;
    }
    st->ct_order_changed = c->n_ord_changed;
    st->nat_hops = c->n_nat_hops;
    st->ct_evicted = c->n_evicted;
    // (the replay's running total of entry words it handed on)
    uint64_t svo_total = 0;
    if (c->svo_cnt.p && c->device != CFC_DEVICE_NONE &&
        hipMemcpy(&svo_total, (char *)c->svo_cnt.p + 8, 8, hipMemcpyDeviceToHost) != hipSuccess)
        svo_total = 0;
    st->svc_ordered = svo_total;
    st->ct_self_segments = c->n_self_segs;
    st->ct_apply_sparse = c->n_apply_sparse;
    st->ct_grown = (uint32_t)c->n_ct_grow;
    st->ct_slots = (c->epoch && c->epoch->ct) ? (uint32_t)(c->epoch->ct->slots4 + c->epoch->ct->slots6)
                            : 0u;
    return 0;
}

const char *cfc_strerror(int err)
{
    return strerror(err < 0 ? -err : err);
}

}  // extern "C"

namespace {

// ---- cfc_ct_apply: the per-packet CT map writes of one classified batch
struct CtApply {
    cfc_ctx *c;
    int family;
    Map *lxc = nullptr;
    std::vector<uint8_t> local = std::vector<uint8_t>(65536, 0);

    explicit CtApply(cfc_ctx *cc, int fam) : c(cc), family(fam)
    {
        for (auto &kv : c->maps) {
            Map *m = kv.second.get();
            if (m->role == ROLE_LXC)
                lxc = m;
            if ((m->role == ROLE_CT4 || m->role == ROLE_CT6) && m->policy_lxc >= 0)
                local[m->policy_lxc] = 1;
        }
    }
    // lxc_id of the local endpoint owning addr (cilium_lxc), or -1
    int endpoint(const uint8_t *addr) const
    {
        if (!lxc)
            return -1;
        char k[20] = {0};
        memcpy(k, addr, family == 4 ? 4 : 16);
        k[16] = (char)(family == 4 ? 1 : 2);
        auto it = lxc->kv.find(std::string(k, 20));
        if (it == lxc->kv.end() || it->second.val.size() < 8)
            return -1;
        uint16_t id;
        memcpy(&id, it->second.val.data() + 6, 2);
        return id;
    }
    Map *ct_map(int owner_lxc, int any) const
    {
        const Role r = family == 4 ? ROLE_CT4 : ROLE_CT6;
        const int want = (owner_lxc >= 0 && local[owner_lxc]) ? owner_lxc : -1;
        for (auto &kv : c->maps) {
            Map *m = kv.second.get();
            if (m->role == r && m->policy_lxc == want && m->ct_any == any)
                return m;
        }
        return nullptr;
    }
};

// struct ct_entry (bpf/lib/common.h:380-406)
struct CtEntry {
    uint64_t rx_packets, rx_bytes, tx_packets, tx_bytes;
    uint32_t lifetime;
    uint16_t bits;   // rx_closing:1 tx_closing:1 nat46:1 lb_loopback:1 seen_non_syn:1
    uint16_t rev_nat_index, slave;
    uint8_t tx_flags_seen, rx_flags_seen;
    uint32_t src_sec_id, last_tx_report, last_rx_report;
};
static_assert(sizeof(CtEntry) == 56, "struct ct_entry is 56 bytes");
constexpr uint16_t CTB_RX_CLOSING = 1, CTB_TX_CLOSING = 2, CTB_NAT46 = 4, CTB_LB_LOOPBACK = 8,
                   CTB_SEEN_NON_SYN = 16;
// conntrack.h:31-35
constexpr uint32_t CT_LIFETIME_TCP = 21600, CT_LIFETIME_NONTCP = 60, CT_SYN_TIMEOUT = 60,
                   CT_CLOSE_TIMEOUT = 10, CT_REPORT_INTERVAL = 5;

// __ct_update_timeout (conntrack.h:125-185)
void ct_upd(CtEntry &e, uint32_t now, uint32_t lifetime, int dir, uint8_t flags)
{
    e.lifetime = now + lifetime;
    uint8_t &acc = dir == 1 ? e.rx_flags_seen : e.tx_flags_seen;
    uint32_t &last = dir == 1 ? e.last_rx_report : e.last_tx_report;
    const uint8_t seen = (uint8_t)(flags | acc);
    if (last + CT_REPORT_INTERVAL < now || acc != seen) {
        last = now;
        acc = seen;
    }
}
// ct_update_timeout (:191-205); syn is bit 0 of TCP byte 12 (union tcp_flags)
void ct_upd_timeout(CtEntry &e, uint32_t now, bool is_tcp, int dir, bool syn,
                    uint8_t flags)
{
    uint32_t lifetime = CT_LIFETIME_NONTCP;
    if (is_tcp) {
        if (!syn)
            e.bits |= CTB_SEEN_NON_SYN;
        lifetime = (e.bits & CTB_SEEN_NON_SYN) ? CT_LIFETIME_TCP : CT_SYN_TIMEOUT;
    }
    ct_upd(e, now, lifetime, dir, flags);
}

// What __ct_lookup (:221-285) does to a hit entry, applied in header order
// at the batch's clock: timeouts, report times, seen flags, the closing
// bits of ACTION_CREATE / ACTION_CLOSE; with count, CONNTRACK_ACCOUNTING
// for a hit the device did not see (a flow created earlier in the batch)
void ct_hit_update(Map *m, Map::Entry &me, int action, int dir, bool count,
                   uint32_t len, uint32_t now, bool is_tcp, bool syn, uint8_t flags)
{
    CtEntry e;
    memcpy(&e, me.val.data(), sizeof(e));
    if (count) {
        (dir == 1 ? e.rx_packets : e.tx_packets) += 1;
        (dir == 1 ? e.rx_bytes : e.tx_bytes) += len;
    }
    auto alive = [&] { return !(e.bits & CTB_RX_CLOSING) || !(e.bits & CTB_TX_CLOSING); };
    if (alive())
        ct_upd_timeout(e, now, is_tcp, dir, syn, flags);
    if (action == 1) {            // ACTION_CREATE re-opens a closing entry
        if (e.bits & (CTB_RX_CLOSING | CTB_TX_CLOSING)) {
            e.bits &= (uint16_t)~(CTB_RX_CLOSING | CTB_TX_CLOSING);
            ct_upd_timeout(e, now, is_tcp, dir, syn, flags);
        }
    } else if (action == 2) {     // ACTION_CLOSE: rx_closing / tx_closing
        e.bits |= dir == 1 ? CTB_RX_CLOSING : CTB_TX_CLOSING;
        if (!alive())
            ct_upd(e, now, CT_CLOSE_TIMEOUT, dir, flags);
    }
    memcpy(&me.val[0], &e, sizeof(e));
    m->touched[me.key] |= TOUCH_VALUE;
    m->gen++;
}

// ---- load balancing on the host CT maps (cfc_ct_apply_v4 with a load
// balancer): cilium_lb4_services / cilium_lb4_reverse_nat as the kernels see
// them (lb.hip), for the apply's replay of the service step
struct LbHost {
    const Map *svc = nullptr, *rnat = nullptr;
    explicit LbHost(cfc_ctx *c)
    {
        for (auto &kv : c->maps) {
            if (kv.second->role == ROLE_LB4_SVC)
                svc = kv.second.get();
            else if (kv.second->role == ROLE_LB4_RNAT)
                rnat = kv.second.get();
        }
    }
    bool on() const { return (svc && !svc->kv.empty()) || (rnat && !rnat->kv.empty()); }
    // struct lb4_service {target, port, count, rev_nat_index, weight}
    struct Svc {
        uint32_t target;
        uint16_t port, count, rev_nat, weight;
    };
    bool get(uint32_t addr, uint16_t dport, uint16_t slave, Svc *v) const
    {
        if (!svc)
            return false;
        char k[8];
        memcpy(k, &addr, 4);
        memcpy(k + 4, &dport, 2);
        memcpy(k + 6, &slave, 2);
        auto it = svc->kv.find(std::string(k, 8));
        if (it == svc->kv.end() || it->second.val.size() < 12)
            return false;
        memcpy(v, it->second.val.data(), 12);
        return true;
    }
    // lb4_lookup_service (lb.h:604-635)
    bool service(uint32_t addr, uint16_t &dport, uint16_t slave, Svc *v) const
    {
        if (dport) {
            if (get(addr, dport, slave, v) && v->count)
                return true;
            dport = 0;
        }
        return get(addr, 0, slave, v) && v->count;
    }
    // lb4_rev_nat (lb.h:485-588) on a packet for an entry with LB state
    void rev_nat(const CtEntry &e, uint8_t proto, uint32_t &sa, uint32_t &da,
                 uint32_t &pt) const
    {
        if (!e.rev_nat_index || !rnat)
            return;
        auto it = rnat->kv.find(std::string((const char *)&e.rev_nat_index, 2));
        if (it == rnat->kv.end() || it->second.val.size() < 6)
            return;
        uint32_t addr;
        uint16_t port;
        memcpy(&addr, it->second.val.data(), 4);
        memcpy(&port, it->second.val.data() + 4, 2);
        if (port && (proto == 6 || proto == 17))
            pt = (pt & 0xFFFF0000u) | port;
        if (e.bits & CTB_LB_LOOPBACK)
            da = sa;
        sa = addr;
    }
};

// cfc.h CFC_FLOW_HASH (kern_common.hpp flow_hash4)
uint32_t flow_hash4_host(uint32_t sa, uint32_t da, uint32_t pt, uint32_t proto)
{
    const uint32_t lo = std::min(sa, da), hi = std::max(sa, da);
    const uint32_t sp = pt & 0xFFFF, dp = pt >> 16;
    const uint32_t pw = std::min(sp, dp) | (std::max(sp, dp) << 16);
    return fmix32(lo * 0x9E3779B1u + hi * 0x85EBCA77u + pw * 0xC2B2AE3Du + proto);
}

// IPv6 (cilium_lb6_services / cilium_lb6_reverse_nat) for the apply's
// replay of ipv6_l3_from_lxc's service step (bpf_lxc.c:149-167)
struct LbHost6 {
    const Map *svc = nullptr, *rnat = nullptr;
    explicit LbHost6(cfc_ctx *c)
    {
        for (auto &kv : c->maps) {
            if (kv.second->role == ROLE_LB6_SVC)
                svc = kv.second.get();
            else if (kv.second->role == ROLE_LB6_RNAT)
                rnat = kv.second.get();
        }
    }
    bool on() const { return (svc && !svc->kv.empty()) || (rnat && !rnat->kv.empty()); }
    // struct lb6_service {target[16], port, count, rev_nat_index, weight}
    struct Svc {
        uint8_t target[16];
        uint16_t port, count, rev_nat, weight;
    };
    bool get(const uint8_t *addr, uint16_t dport, uint16_t slave, Svc *v) const
    {
        if (!svc)
            return false;
        char k[20];
        memcpy(k, addr, 16);
        memcpy(k + 16, &dport, 2);
        memcpy(k + 18, &slave, 2);
        auto it = svc->kv.find(std::string(k, 20));
        if (it == svc->kv.end() || it->second.val.size() < 24)
            return false;
        memcpy(v, it->second.val.data(), 24);
        return true;
    }
    // lb6_lookup_service (lb.h:352-381)
    bool service(const uint8_t *addr, uint16_t &dport, uint16_t slave, Svc *v) const
    {
        if (dport) {
            if (get(addr, dport, slave, v) && v->count)
                return true;
            dport = 0;
        }
        return get(addr, 0, slave, v) && v->count;
    }
    // lb6_rev_nat (lb.h:306-319, flags 0) on a packet
    void rev_nat(uint16_t index, uint8_t proto, uint8_t *sa, uint32_t &pt) const
    {
        if (!index || !rnat)
            return;
        auto it = rnat->kv.find(std::string((const char *)&index, 2));
        if (it == rnat->kv.end() || it->second.val.size() < 18)
            return;
        uint16_t port;
        memcpy(&port, it->second.val.data() + 16, 2);
        if (port && (proto == 6 || proto == 17))
            pt = (pt & 0xFFFF0000u) | port;
        memcpy(sa, it->second.val.data(), 16);
    }
};

// cfc.h CFC_FLOW_HASH over IPv6 addresses (kern_common.hpp flow_hash6)
uint32_t fold6_host(const uint8_t *a)
{
    uint32_t w[4];
    memcpy(w, a, 16);
    uint32_t h = fmix32(w[3]);
    h = fmix32(w[2] ^ h);
    h = fmix32(w[1] ^ h);
    return fmix32(w[0] ^ h);
}

// what lb6_local leaves (lb.h:427-481): the CT_SERVICE tuple and ct_state
struct LbState6 {
    bool svc = false, drop = false, reslave = false;
    uint8_t tda[16];
    uint16_t slave0 = 0, slave = 0, rev_nat = 0;
    std::string ksvc;
};
LbState6 lb6_step(const LbHost6 &L, Map *m, const uint8_t *sa, const uint8_t *da, uint32_t &pt,
                  uint8_t proto, uint32_t hash)
{
    LbState6 x;
    memcpy(x.tda, da, 16);
    const bool l4 = proto == 6 || proto == 17;
    if (!L.svc || (!l4 && proto != 58))
        return x;
    uint16_t kd = l4 ? (uint16_t)(pt >> 16) : 0;
    LbHost6::Svc v, b;
    if (!L.service(da, kd, 0, &v))
        return x;
    x.svc = true;
    uint16_t td, ts;
    uint8_t fl = 4;   // TUPLE_F_SERVICE
    if (l4) {
        td = (uint16_t)(pt & 0xFFFF);
        ts = (uint16_t)(pt >> 16);
    } else {
        const uint32_t type = pt & 0xFF;
        const bool rel = type >= 1 && type <= 4;
        td = (!rel && type == 129) ? 128 : 0;
        ts = (!rel && type == 128) ? 128 : 0;
        fl |= rel ? 2 : 0;
    }
    char k[38];
    memcpy(k, da, 16);
    memcpy(k + 16, sa, 16);
    memcpy(k + 32, &td, 2);
    memcpy(k + 34, &ts, 2);
    k[36] = (char)proto;
    k[37] = (char)fl;
    x.ksvc.assign(k, 38);
    auto it = m ? m->kv.find(x.ksvc) : decltype(m->kv.end()){};
    if (m && it != m->kv.end()) {   // ct_state from the entry
        CtEntry e;
        memcpy(&e, it->second.val.data(), sizeof(e));
        x.slave = e.slave;
    } else {
        x.slave = (uint16_t)(hash % v.count + 1);   // lb6_select_slave
    }
    x.slave0 = x.slave;
    if (!L.get(da, kd, x.slave, &b)) {
        if (!L.service(da, kd, x.slave, &b)) {
            x.drop = true;
            return x;
        }
        x.slave = (uint16_t)(hash % b.count + 1);
        x.reslave = true;
    }
    x.rev_nat = b.rev_nat;
    memcpy(x.tda, b.target, 16);
    if (b.port && kd != b.port && l4)   // lb6_xlate
        pt = (pt & 0xFFFFu) | (uint32_t)b.port << 16;
    return x;
}

// the ct_state lb4_local leaves for ct_create4 (common.h:452-461)
struct LbState {
    bool svc = false, drop = false, reslave = false;
    uint32_t tda = 0;             // tuple daddr after the service step
    uint16_t slave0 = 0, slave = 0, rev_nat = 0;
    bool loopback = false;
    uint32_t addr = 0, svc_addr = 0;
    std::string ksvc;             // the CT_SERVICE tuple
    Map *svc_map = nullptr;
};

// What handle_ipv4_from_lxc's service step does (bpf_lxc.c:476-492,
// lb.h:590-776) for one header, against the maps as they now are (the
// batch's earlier CT_SERVICE creates included).  pt: the packet's first L4
// word, rewritten; psa: the packet's saddr.
LbState lb4_step(const LbHost &L, Map *m, uint32_t sa, uint32_t da, uint32_t &pt,
                 uint32_t &psa, uint32_t &pda, uint8_t proto, uint32_t hash)
{
    LbState x;
    x.tda = da;
    const bool l4 = proto == 6 || proto == 17;
    if (!L.svc || (!l4 && proto != 1))
        return x;
    uint16_t kd = l4 ? (uint16_t)(pt >> 16) : 0;
    LbHost::Svc v, b;
    if (!L.service(da, kd, 0, &v))
        return x;
    x.svc = true;
    x.svc_map = m;
    // the CT_SERVICE tuple: as loaded, flags TUPLE_F_SERVICE (| RELATED for
    // an ICMP error)
    uint16_t td, ts;
    uint8_t fl = 4;
    if (l4) {
        td = (uint16_t)(pt & 0xFFFF);
        ts = (uint16_t)(pt >> 16);
    } else {
        const uint32_t type = pt & 0xFF;
        const bool rel = type == 3 || type == 11 || type == 12;
        td = (!rel && type == 0) ? 8 : 0;
        ts = (!rel && type == 8) ? 8 : 0;
        fl |= rel ? 2 : 0;
    }
    char k[14];
    memcpy(k, &da, 4);
    memcpy(k + 4, &sa, 4);
    memcpy(k + 8, &td, 2);
    memcpy(k + 10, &ts, 2);
    k[12] = (char)proto;
    k[13] = (char)fl;
    x.ksvc.assign(k, 14);
    auto it = m ? m->kv.find(x.ksvc) : decltype(m->kv.end()){};
    if (m && it != m->kv.end()) {   // CT_REPLY: ct_state from the entry
        CtEntry e;
        memcpy(&e, it->second.val.data(), sizeof(e));
        x.slave = e.slave;
        x.loopback = (e.bits & CTB_LB_LOOPBACK) != 0;
    } else {
        x.slave = (uint16_t)(hash % v.count + 1);   // lb4_select_slave
    }
    x.slave0 = x.slave;
    if (!L.get(da, kd, x.slave, &b)) {
        if (!L.service(da, kd, x.slave, &b)) {
            x.drop = true;
            return x;
        }
        x.slave = (uint16_t)(hash % b.count + 1);
        x.reslave = true;
    }
    x.rev_nat = b.rev_nat;
    x.addr = b.target;
    if (sa == b.target) {
        x.loopback = true;
        x.addr = IPV4_LOOPBACK;
        x.svc_addr = sa;
        psa = IPV4_LOOPBACK;
    }
    if (!x.loopback)
        x.tda = b.target;
    pda = b.target;
    if (b.port && kd != b.port && l4)
        pt = (pt & 0xFFFFu) | (uint32_t)b.port << 16;
    return x;
}

// Device slot of a CT key in the current epoch, or -1.  A write that
// removes or replaces an entry drops the counts the batch's lookups made on
// it (in the reference they land on the entry before it goes), so its
// accounting slot is zeroed before the fold.
int64_t ct_dev_slot(const Epoch &E, const Map *m, const std::string &k)
{
    const bool v6 = m->role == ROLE_CT6;
    const size_t al = v6 ? 16 : 4;
    const uint32_t owner = ct_owner_word((uint32_t)std::max(m->policy_lxc, 0),
                                         m->policy_lxc >= 0);
    uint32_t z;
    memcpy(&z, k.data() + 2 * al, 4);
    const uint8_t nh = (uint8_t)k[2 * al + 4];
    // entries no lookup reaches are not in the device table (build_ct); the
    // same tuple in the other map kind is a different entry
    if (m->ct_any ? (nh != 17 && nh != (v6 ? 58 : 1)) : nh != 6)
        return -1;
    const uint32_t w = ct_word(nh, (uint8_t)k[2 * al + 5], owner);
    if (!v6) {
        if (!E.ct->slots4)
            return -1;
        uint32_t x, y;
        memcpy(&x, k.data(), 4);
        memcpy(&y, k.data() + 4, 4);
        const uint32_t mask = (uint32_t)E.ct->slots4 - 1;
        for (uint32_t i = ct_home4(x, y, z, w) & mask;; i = (i + 1) & mask) {
            const Ct4Slot &e = E.ct->ct4_host[i];
            if (!e.w)
                return -1;
            if (e.x == x && e.y == y && e.z == z && e.w == w)
                return i;
        }
    }
    if (!E.ct->slots6)
        return -1;
    uint32_t d[4], sa[4];
    memcpy(d, k.data(), 16);
    memcpy(sa, k.data() + 16, 16);
    const uint32_t mask = (uint32_t)E.ct->slots6 - 1;
    for (uint32_t i = ct_home6(d, sa, z, w) & mask;; i = (i + 1) & mask) {
        const Ct6Slot &e = E.ct->ct6_host[i];
        if (!e.w)
            return -1;
        if (e.z == z && e.w == w && !memcmp(e.d, d, 16) && !memcmp(e.s, sa, 16))
            return (int64_t)E.ct->slots4 + i;
    }
}

void ct_drop_counts(cfc_ctx *c, const Map *m, const std::string &k, hipStream_t s)
{
    if (!c->epoch || !c->epoch->ct->ct_st.p || mirror_sync(*c->epoch->ct, s))
        return;
    const int64_t slot = ct_dev_slot(*c->epoch, m, k);
    if (slot >= 0)
        (void)hipMemsetAsync(((CtState *)c->epoch->ct->ct_st.p + slot)->acct, 0, 32, s);
}

int ct_gc_dev(cfc_ctx *c, const std::vector<Map *> &sel, const cfc_ct_gc_filter &f,
              cfc_ct_gc_stats &st, hipStream_t s, const uint32_t *protect);

// A batch whose creates would take CT maps past max_entries (want[j]: the
// entries map j would hold): the reference's LRU hash evicts its least
// recently used entries as the inserts come (kernel order, per-CPU lists —
// not reproducible).  Here, before the inserts, each overflowing map loses
// exactly its excess: the entries no lookup of this batch hit (they are the
// most recently used) with the earliest last refresh — lifetime minus the
// timeout its state sets (conntrack.h:125-205: CT_CLOSE_TIMEOUT once both
// closing bits are set, else CT_LIFETIME_TCP for a TCP entry past its SYN,
// CT_SYN_TIMEOUT before, CT_LIFETIME_NONTCP otherwise) — ties broken by key
// bytes.  Chosen on the host mirror (synced before), deleted there and
// patched into the device table (patch_ct).  Every overflowing map is
// checked before any is touched: 0 done, 1 a map has too few candidates
// (nothing deleted: the host path), 2 deleted but the table could not be
// patched (the host path; the next commit rebuilds), < 0 error.
int ct_evict_maps(cfc_ctx *c, bool v6, const std::vector<Map *> &fmaps,
                  const std::vector<uint64_t> &want, const uint32_t *hs, uint64_t nk,
                  hipStream_t s)
{
    Epoch &E = *c->epoch;
    GCt &G = *E.ct;
    if (int rc = mirror_sync(G, s))
        return rc;
    const uint64_t slots = v6 ? G.slots6 : G.slots4;
    const uint64_t base6 = v6 ? G.slots4 : 0;   // (ct_dev_slot's IPv6 offset)
    const size_t words = (slots + 31) / 32;
    std::vector<uint32_t> bm(words);
    if (c->evict_bm.ensure(4 * words) ||
        hipMemsetAsync(c->evict_bm.p, 0, 4 * words, s) != hipSuccess ||
        ct_protect_hits(hs, nk, (uint32_t *)c->evict_bm.p, s) ||
        hipMemcpyAsync(bm.data(), c->evict_bm.p, 4 * words, hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    using It = std::map<std::string, Map::Entry>::iterator;
    struct Cand {
        int64_t refresh;
        It it;
    };
    std::vector<std::vector<It>> del(fmaps.size());
    for (size_t j = 0; j < fmaps.size(); j++) {
        Map *m = fmaps[j];
        if (want[j] <= m->max_entries)
            continue;
        const uint64_t excess = want[j] - m->max_entries;
        const size_t al = v6 ? 16 : 4;
        std::vector<Cand> cand;
        cand.reserve(m->kv.size());
        for (It it = m->kv.begin(); it != m->kv.end(); ++it) {
            const int64_t ds = ct_dev_slot(E, m, it->first);
            if (ds >= 0) {
                const uint64_t sl = (uint64_t)ds - base6;
                if (sl < slots && ((bm[sl >> 5] >> (sl & 31)) & 1u))
                    continue;   // hit by this batch
            }
            const std::string &v = it->second.val;
            if (v.size() < 38)
                continue;
            uint32_t life;
            uint16_t bits;
            memcpy(&life, &v[32], 4);
            memcpy(&bits, &v[36], 2);
            const bool tcp = (uint8_t)it->first[2 * al + 4] == 6;
            const uint32_t to = (bits & 3) == 3 ? 10u      // CT_CLOSE_TIMEOUT
                                : !tcp ? 60u                // CT_LIFETIME_NONTCP
                                : (bits & 16) ? 21600u      // CT_LIFETIME_TCP
                                              : 60u;        // CT_SYN_TIMEOUT
            cand.push_back(Cand{(int64_t)life - to, it});
        }
        if (cand.size() < excess)
            return 1;
        auto lt = [](const Cand &a, const Cand &b) {
            return a.refresh != b.refresh ? a.refresh < b.refresh : a.it->first < b.it->first;
        };
        std::nth_element(cand.begin(), cand.begin() + (excess - 1), cand.end(), lt);
        for (uint64_t k = 0; k < excess; k++)
            del[j].push_back(cand[k].it);
    }
    uint64_t n = 0;
    for (size_t j = 0; j < fmaps.size(); j++)
        for (It it : del[j]) {
            // (an entry the device table does not hold needs no patch)
            const bool dev = ct_dev_slot(E, fmaps[j], it->first) >= 0;
            fmaps[j]->ct_erase_at(it, dev);
            n++;
        }
    c->n_evicted += n;
    if (!n)
        return 0;
    // the deletes into the live CT table only (patch_ct), not a commit: the
    // other groups' pending changes stay pending and the epoch — whose
    // tables the rest of this apply reads — stays
    if (!patch_ct(c, s)) {
        c->built_sig[3] = ~0ull;   // (the next commit rebuilds the CT group)
        return 2;                  // the batch to the host path
    }
    uint64_t sig[NGROUPS];
    group_sigs(c, sig);
    c->built_sig[3] = sig[3];
    for (auto &kv : c->maps)
        if (kv.second->ct())
            kv.second->touched.clear();
    E.st.ct4_entries = G.n_ct4;
    E.st.ct6_entries = G.n_ct6;
    c->ct_gen++;
    return hipStreamSynchronize(s) == hipSuccess ? 0 : -EIO;
}

// Device-side growth of family v6's CT table to `want` slots (a power of
// two): the rehash kernel (ctapply.hip k_ct_rehash) moves every key-holding
// slot, its CtState line and LB word into new buffers; the other family's
// lines are copied as they are (the IPv6 lines start after the IPv4 ones);
// the plain-hit summaries start empty.  The apply never stops for a host
// rebuild: the host mirror follows lazily (mirror_sync, before its next
// reader), and the pending GC log's slots are remapped on the device.  The
// replaced buffers are retired like an epoch (launches on other streams may
// still read them).  0 grown, 1 not possible (the host path), < 0 error.
int ct_grow(cfc_ctx *c, bool v6, uint64_t want, hipStream_t s)
{
    Epoch &E = *c->epoch;
    GCt &G = *E.ct;
    const uint64_t n4 = G.slots4, n6 = G.slots6, o = v6 ? n6 : n4;
    if (!o || want <= o || want > (1ull << 30) || (want & (want - 1)))
        return 1;
    const uint64_t m4 = v6 ? n4 : want, m6 = v6 ? want : n6;
    const size_t ksz = v6 ? sizeof(Ct6Slot) : sizeof(Ct4Slot);
    DevBuf &key = v6 ? G.ct6 : G.ct4, &lb = v6 ? G.ct6_lb : G.ct4_lb, &ms = v6 ? G.ct6_ms : G.ct4_ms;
    auto nk = std::make_unique<DevBuf>(), nst = std::make_unique<DevBuf>(),
         nsum = std::make_unique<DevBuf>(), nms = std::make_unique<DevBuf>(),
         nlb = std::make_unique<DevBuf>();
    DevBuf map;
    // (every new line zero: the rehash writes only the moved slots', and a
    // free slot's record must read as no entry, no dirty bits)
    if (nk->zeros(ksz * want, s) || nst->zeros(sizeof(CtState) * (m4 + m6), s) ||
        nsum->zeros(4 * (m4 + m6), s) || nms->zeros(12 * want, s) ||
        (lb.p && nlb->zeros(16 * want, s)) || map.ensure(4 * o) ||
        c->cta_cnt.ensure(4 * CTA_NCNT))
        return -ENOMEM;
    CtState *ost = (CtState *)G.ct_st.p, *ns = (CtState *)nst->p;
    uint32_t *cnt = (uint32_t *)c->cta_cnt.p, moved = 0;
    const uint64_t other = v6 ? n4 : n6;
    if ((other && hipMemcpyAsync(v6 ? ns : ns + m4, v6 ? ost : ost + n4, sizeof(CtState) * other,
                                 hipMemcpyDeviceToDevice, s) != hipSuccess) ||
        hipMemsetAsync(cnt, 0, 4, s) != hipSuccess ||
        ct_rehash(v6, key.p, ost + (v6 ? n4 : 0), (const uint4 *)lb.p, o, nk->p,
                  ns + (v6 ? m4 : 0), (uint4 *)nlb->p, (uint32_t)(want - 1), (uint32_t *)map.p,
                  cnt, s))
        return -EIO;
    // the GC log's slots (its deletes the host has not taken)
    if (!v6 && c->gc_log_used &&
        ct_remap(&((CtGcRec *)c->gc_log.p)->slot, c->gc_log_used, sizeof(CtGcRec) / 4,
                 (const uint32_t *)map.p, s))
        return -EIO;
    if (v6 && c->gc_log6_used &&
        ct_remap(&((CtGcRec6 *)c->gc_log6.p)->slot, c->gc_log6_used, sizeof(CtGcRec6) / 4,
                 (const uint32_t *)map.p, s))
        return -EIO;
    // the host mirror's remap: this one, or composed with one still pending
    DevBuf &pend = v6 ? G.pend6 : G.pend4;
    if (pend.p) {
        if (ct_remap((uint32_t *)pend.p, v6 ? G.ct6_host.size() : G.ct4_host.size(), 1,
                     (const uint32_t *)map.p, s))
            return -EIO;
    } else {
        std::swap(pend.p, map.p);
        std::swap(pend.bytes, map.bytes);
    }
    if (hipMemcpyAsync(&moved, cnt, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    // the replaced buffers stay until the launches on other streams that
    // may read them have passed this point
    {
        auto old = std::make_shared<Epoch>();
        old->ct = std::make_shared<GCt>();
        GCt &R = *old->ct;
        auto give = [](DevBuf &from, DevBuf &to, std::unique_ptr<DevBuf> &nb) {
            std::swap(to.p, from.p);
            std::swap(to.bytes, from.bytes);
            if (nb) {
                std::swap(from.p, nb->p);
                std::swap(from.bytes, nb->bytes);
            }
        };
        give(key, v6 ? R.ct6 : R.ct4, nk);
        give(G.ct_st, R.ct_st, nst);
        give(G.ct_sum, R.ct_sum, nsum);
        give(ms, v6 ? R.ct6_ms : R.ct4_ms, nms);
        if (lb.p)
            give(lb, v6 ? R.ct6_lb : R.ct4_lb, nlb);
        Retired r;
        r.e = old;
        for (hipStream_t st : c->streams) {
            if (st == s)
                continue;   // (stream-ordered behind this call already)
            hipEvent_t ev;
            if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
                hipEventRecord(ev, st) != hipSuccess) {
                (void)hipDeviceSynchronize();
                break;
            }
            r.ev.push_back(ev);
        }
        c->retired.push_back(std::move(r));
    }
    if (v6) {
        G.slots6 = want;
        G.ct6_mask = (uint32_t)(want - 1);
        G.ct6_probe = G.ct6_mask;
        G.tomb6 = moved > G.n_ct6 ? (uint32_t)(moved - G.n_ct6) : 0u;
        c->ct_used6 = moved;
        c->ct_used6_valid = true;
        c->cta_ins6 = 0;
        c->ct_min6 = std::max<uint64_t>(c->ct_min6, want);
    } else {
        G.slots4 = want;
        G.ct4_mask = (uint32_t)(want - 1);
        G.ct4_probe = G.ct4_mask;
        G.tomb4 = moved > G.n_ct4 ? (uint32_t)(moved - G.n_ct4) : 0u;
        c->ct_used = moved;
        c->ct_used_valid = true;
        c->cta_ins = 0;
        c->ct_min4 = std::max<uint64_t>(c->ct_min4, want);
    }
    assemble(E);
    E.T.id_cover = c->id_cover;
    // the table moved under every hit slot and summary a launch left
    c->ct_gen++;
    c->last_cls.valid = false;
    c->sum_dirty = c->sum_pending = false;
    c->ct_dirty = true;   // (the mirror lags the table until mirror_sync)
    c->n_ct_grow++;
    return 0;
}

// cfc_ct_apply_v4/v6 on the device (ctapply.hip).  1: take the host path
// instead (nothing changed), 0 done, <0 error.
template <class Hdr>
int ct_apply_dev(cfc_ctx *c, const Hdr *in, const cfc_out *out, int mode, uint16_t ep_lxc,
                 hipStream_t s, bool may_grow = true, bool order = true)
{
    constexpr bool V6 = std::is_same<Hdr, cfc_hdr_v6>::value;
    settle(c);
    if (c->ct_apply_mode != CFC_CT_APPLY_DEVICE || !c->epoch)
        return 1;
    // the device table must be the maps as committed: no host-side CT
    // change waiting for a commit
    uint64_t sig[NGROUPS];
    group_sigs(c, sig);
    if (sig[3] != c->built_sig[3])
        return 1;
    bool local_ep = false;
    for (auto &kv : c->maps) {
        const Map *m = kv.second.get();
        if (m->ct() && !m->touched.empty())
            return 1;
        local_ep |= m->ct() && m->policy_lxc == (int)ep_lxc;
    }
    Epoch &E = *c->epoch;
    GCt &G = *E.ct;
    // a load balancer: its per-slot ct_state is on the device (the apply
    // writes it with every create), and an egress batch replays the service
    // step (lb4_local / lb6_local, the egress reply's reverse NAT: k_cta_lb)
    const bool lbt = V6 ? (E.T.lb6 || E.T.rnat6) : (E.T.lb4 || E.T.rnat4);
    DevBuf &lbst = V6 ? G.ct6_lb : G.ct4_lb;
    if (lbt && !lbst.p)
        return 1;
    const bool lbm = lbt && mode == CFC_MODE_EGRESS;
    const uint64_t k3 = lbm ? 3 : 2;   // requests per header, writes per create
    const uint64_t n = in->n, slots = V6 ? G.slots6 : G.slots4;
    if (!slots && may_grow && n < (1ull << 27)) {
        // no table yet (the family's maps were empty at the build): build
        // one sized for this batch and apply on it — unless other map groups
        // wait for a commit (the tables the batch was classified with)
        bool maps = false, others = false;
        for (auto &kv : c->maps)
            maps |= kv.second->role == (V6 ? ROLE_CT6 : ROLE_CT4);
        uint64_t sg[NGROUPS];
        group_sigs(c, sg);
        for (int g = 0; g < NGROUPS; g++)
            others |= g != 3 && sg[g] != c->built_sig[g];
        if (maps && !others) {
            uint64_t &mn = V6 ? c->ct_min6 : c->ct_min4;
            mn = std::max<uint64_t>({mn, 1ull << 16, 8 * n});
            c->built_sig[3] = ~0ull;
            if (int rc = commit_locked(c, s))
                return rc;
            return ct_apply_dev(c, in, out, mode, ep_lxc, s, false, true);
        }
    }
    if (!slots || !G.ct_st.p || n >= (lbm ? 1ull << 27 : 1ull << 28))
        return 1;
    // the batch's classify (its CT bytes, verdicts and the workspace's hit
    // slots) may have run on another stream
    order_after_launches(c, s);
    int ob = 4, sb = 1;   // (op order: ((2 * header + stage) << 3) | write << 1)
    while ((1ull << ob) < (lbm ? 32 : 16) * n)
        ob++;
    while ((1ull << sb) < slots)
        sb++;
    if (ob + sb > 64)
        return 1;
    const uint64_t obm_bytes = 4 * ((slots + 31) / 32);
    if (c->cta_hs.ensure((lbm ? 16 : 8) * n) || c->cta_req.ensure(8 * k3 * n) ||
        c->cta_cnt.ensure(4 * CTA_NCNT) || c->cta_obm.ensure(obm_bytes))
        return -ENOMEM;
    if (lbm && (c->cta_lbr.ensure((V6 ? sizeof(LbRec6) : sizeof(LbRec4)) * n) ||
                c->cta_reqs.ensure(16 * n) ||
                c->cta_tmp.ensure(cta_sort_tmp_bytes((uint32_t)n))))
        return -ENOMEM;
    CtaArgs A{};
    A.T = E.T;
    A.sa = (const uint32_t *)in->saddr;
    A.da = (const uint32_t *)in->daddr;
    A.pt = in->ports;
    A.mt = in->meta;
    A.tf = in->tcp_flags;
    A.ctb = out->ct;
    A.ver = out->verdict;
    A.ident = (const uint32_t *)out->identity;
    A.n = n;
    A.mode = mode;
    A.ep_owner = mode == CFC_MODE_EGRESS ? ct_owner_word(ep_lxc, local_ep) : 0u;
    A.ep_sec = c->seclabel[ep_lxc];
    A.now = c->now;
    A.seq = c->cta_seq;
    A.nat46 = c->hop_nat46 ? 1u : 0u;
    if (V6) {
        A.ct6 = (Ct6Slot *)G.ct6.p;
        A.mask = G.ct6_mask;
        A.acct_base = E.T.ct6_acct_base;
        A.st = (CtState *)G.ct_st.p + A.acct_base;
        A.ms = (uint2 *)G.ct6_ms.p;
        A.lh = (uint32_t *)(A.ms + slots);
    } else {
        A.ct4 = (Ct4Slot *)G.ct4.p;
        A.mask = G.ct4_mask;
        A.acct_base = 0;
        A.st = (CtState *)G.ct_st.p;
        A.ms = (uint2 *)G.ct4_ms.p;
        A.lh = (uint32_t *)(A.ms + slots);
    }
    A.hs = (uint32_t *)c->cta_hs.p;
    A.reqA = (uint64_t *)c->cta_req.p;
    A.req_cap = (uint32_t)std::min<uint64_t>(k3 * n, 0xFFFFFFFFu);
    A.cnt = (uint32_t *)c->cta_cnt.p;
    A.obm = (uint32_t *)c->cta_obm.p;
    A.ob = ob;
    A.slot_bits = sb;
    A.lb = lbst.p ? (uint4 *)lbst.p : nullptr;
    if (lbm) {
        A.lbr = c->cta_lbr.p;
        A.hash = in->hash;
        A.reqS = (uint64_t *)c->cta_reqs.p;
        A.reqS2 = A.reqS + n;
        A.sort_tmp = c->cta_tmp.p;
        A.sort_tmp_bytes = c->cta_tmp.bytes;
    }
    {   // this batch's hit slots from its classify launch, if still there
        // (not with a service step: its tuples may differ from the launch's)
        const auto &L = c->last_cls;
        if (!lbm && L.valid && L.family == (V6 ? 6 : 4) && L.gen == c->ct_gen && L.ct == out->ct &&
            L.saddr == (const void *)in->saddr && L.n == n && L.mode == mode && L.ep == ep_lxc) {
            A.ck1 = (const uint32_t *)((const char *)c->ws + L.k1);
            A.ck2 = L.k2 ? (const uint32_t *)((const char *)c->ws + L.k2) : nullptr;
            // and its plain-hit summaries (taken once: this apply clears them)
            if (L.sum && c->sum_dirty && G.ct_sum.p)
                A.sum = (uint32_t *)G.ct_sum.p + A.acct_base;
            // and its work list: the sparse scan and ordering passes
            if (L.wl && A.sum && !out->notify && (mode != CFC_MODE_EGRESS || A.ck2)) {
                const uint64_t words = (n + 63) / 64;
                A.W = WList{(const uint64_t *)c->cta_wbits.p,
                            (const uint64_t *)c->cta_wbits.p + words, words};
                A.sparse = true;
            }
            c->last_cls.wl = false;
            c->last_cls.sum = false;
            c->sum_want = true;   // (applies follow their launches: keep them)
            c->sum_pending = false;
        }
    }
    {   // 16-byte loads of four headers' words in the scan
        auto al = [](const void *p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; };
        A.vec = al(A.sa, 16) && al(A.da, 16) && al(A.pt, 16) && al(A.mt, 16) && al(A.ver, 16) &&
                al(A.ident, 16) && al(A.ck1, 16) && al(A.ck2, 16) && al(A.ctb, 4) && al(A.tf, 4);
    }
    // a load balancer's service step first: the ordering pass and the scan
    // decode its per-header records
    if (hipMemsetAsync(A.cnt, 0, 4 * CTA_NCNT, s) != hipSuccess ||
        hipMemsetAsync(A.obm, 0, obm_bytes, s) != hipSuccess || (lbm && cta_lb_pre(A, V6, s)))
        return -EIO;
    // the reference's packet-order CT results (ctorder.hip): the stages a
    // CT write earlier in the batch changes get their CT byte rewritten
    // before the apply folds it (once per call: not again after a rebuild)
    if (order) {
        // (per-slot state, clear between applies: grown with the table)
        if (c->ord_delbm.bytes < obm_bytes &&
            (c->ord_delbm.zeros(obm_bytes, s) || c->ord_mixbm.zeros(obm_bytes, s)))
            return -ENOMEM;
        if (c->ord_dfirst.bytes < 4 * slots) {
            if (c->ord_dfirst.ensure(4 * slots) ||
                hipMemsetD32Async((hipDeviceptr_t)c->ord_dfirst.p, 0xFFFFFFFFu,
                                  c->ord_dfirst.bytes / 4, s) != hipSuccess)
                return -ENOMEM;
        }
        if (!c->ord_cnt.p && c->ord_cnt.zeros(4 * ORD_NCNT, s))   // (ORD_CHANGED accumulates)
            return -ENOMEM;
        OrdArgs O{};
        O.ctb = out->ct;
        O.ck1 = const_cast<uint32_t *>(A.ck1);
        O.ck2 = const_cast<uint32_t *>(A.ck2);
        O.delbm = (uint32_t *)c->ord_delbm.p;
        O.mixbm = (uint32_t *)c->ord_mixbm.p;
        O.dfirst = (uint32_t *)c->ord_dfirst.p;
        O.bm_bytes = c->ord_delbm.bytes;
        O.slots = c->ord_dfirst.bytes / 4;
        O.cnt = (uint32_t *)c->ord_cnt.p;
        O.W = A.W;
        O.sparse = A.sparse;
        O.rtag = A.sparse ? A.hs : nullptr;   // (hs: the dense scan's, unused)
        uint32_t changed = 0;
        // (IPv6 with reverse NAT: the packet outputs follow the new results)
        const bool pkt6 = V6 && out->pkt_saddr && out->pkt_ports && E.T.rnat6;
        if (pkt6 && (c->ord_ct0.ensure(n) ||
                     hipMemcpyAsync(c->ord_ct0.p, out->ct, n, hipMemcpyDeviceToDevice, s) !=
                         hipSuccess))
            return -ENOMEM;
        if (int rc = ord_resolve(A, O, c->ordb, V6, &changed, s))
            return rc;
        A.sparse = A.sparse && O.sparse;   // (a batch that deletes: the dense scan)
        if (A.sparse) {   // (the ordering's list of the work bits)
            A.wl = O.wl;
            A.nwl = O.cnt + ORD_NWL;
        }
        if (pkt6)
            if (int rc = ord_pkt6(A, (const uint8_t *)c->ord_ct0.p, *out, s))
                return rc;
        c->n_ord_changed += changed;
    }
    // the caller wants the event words: the trace words' monitor lengths in
    // packet order (every hit replayed by the fold, k_cta_mon)
    if (out->notify) {
        if (c->cta_mon.ensure(2 * n) || hipMemsetAsync(c->cta_mon.p, 0xFF, 2 * n, s) != hipSuccess)
            return -ENOMEM;
        A.nt = out->notify;
        A.mon = (uint8_t *)c->cta_mon.p;
    }
    uint32_t hc[CTA_NCNT];
    // a sparse scan's batch routes its ordered hits right after the scan
    // (the creates' slots hold no hit of the launch), into a list of its
    // own: one wait for both passes' counts, none after the inserts
    const bool early = A.sparse && !lbm && !out->notify;
    const uint64_t nroute_cap = mode == CFC_MODE_EGRESS ? 2 * n : n;
    if (early && (c->cta_cxr.ensure(8 * nroute_cap) ||
                  (!c->pend_cnt && (hipHostMalloc((void **)&c->pend_cnt, 4 * CTA_NCNT,
                                                  hipHostMallocDefault) != hipSuccess ||
                                    hipEventCreateWithFlags(&c->pend_ev, hipEventDisableTiming) !=
                                        hipSuccess))))
        return -ENOMEM;
    // (IPv4 sparse scan: the requests' keys for the insert, per header stage)
    A.rk4 = nullptr;
    if (!V6 && A.sparse && !A.lbr) {
        if (c->cta_rk.ensure(16ull * nroute_cap))
            return -ENOMEM;
        A.rk4 = (uint4 *)c->cta_rk.p;
    }
    if (cta_scan(A, V6, s))
        return -EIO;
    if (early) {
        CtaArgs R = A;
        R.cx = (uint64_t *)c->cta_cxr.p;
        R.cx_base = 0;
        R.cx_cap = (uint32_t)nroute_cap;
        if (cta_route(R, s))
            return -EIO;
    }
    if (hipMemcpyAsync(hc, A.cnt, sizeof(hc), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    // (a sparse scan does not count the plain hits: route's bound is every stage)
    const uint64_t nreqA = hc[CTA_NREQA],
                   nhit = A.sparse ? (mode == CFC_MODE_EGRESS ? 2 * n : n) : hc[CTA_NHIT];
    uint64_t &claims = V6 ? c->cta_claims6 : c->cta_claims;
    uint64_t &ins = V6 ? c->cta_ins6 : c->cta_ins;
    uint64_t &log_used = V6 ? c->log6_used : c->log_used;
    DevBuf &logbuf = V6 ? c->cta_log6 : c->cta_log;
    const size_t log_rec = V6 ? sizeof(CtLog6) : sizeof(CtLog);
    auto used_now = [&]() -> uint64_t {
        return V6 ? (c->ct_used6_valid ? c->ct_used6 : (uint64_t)G.n_ct6 + G.tomb6)
                  : (c->ct_used_valid ? c->ct_used : (uint64_t)G.n_ct4 + G.tomb4);
    };
    uint64_t used = used_now();
    const uint64_t nr = std::max<uint64_t>(nreqA, 1);
    const uint64_t cx_cap = nhit + (k3 + 1) * nreqA + 64;   // (round 1 laid out for 2 per create)
    const uint64_t log_need = log_used + nreqA;
    bool ok = nreqA <= A.req_cap && cx_cap <= 0xFFFFFFFFu;
    if (ok && (c->cta_req2.ensure(40 * nr) || c->cta_cx.ensure(16 * cx_cap) ||
               c->cta_tmp.ensure(cta_sort_tmp_bytes((uint32_t)std::max<uint64_t>(cx_cap, 2 * nr)))))
        return -ENOMEM;
    uint64_t *r2 = (uint64_t *)c->cta_req2.p, *cx = (uint64_t *)c->cta_cx.p;
    A.reqA2 = r2;
    A.sort_tmp = c->cta_tmp.p;
    A.sort_tmp_bytes = c->cta_tmp.bytes;
    // room for every key the batch adds: the table below 3/4 load, each CT
    // map below max_entries; else the host path (which rebuilds).  First the
    // quick bound — each create its key and its related entry, a load
    // balancer's creates their reverse-NAT entry (counted hits add none) —
    // and when that fails the exact count (k_cta_newkeys), per map when the
    // family has no more than CTG_MAX_MAPS of them (else per map kind: TCP
    // or ANY — an over-estimate for a map the batch does not write)
    uint64_t newk = 2 * (nreqA - hc[CTA_NFHIT]) + hc[CTA_NKX];
    uint64_t newk_kind[2] = {newk, newk};   // [TCP map, ANY map]
    std::vector<Map *> fmaps;               // the family's CT maps
    for (auto &kv : c->maps)
        if (kv.second->role == (V6 ? ROLE_CT6 : ROLE_CT4))
            fmaps.push_back(kv.second.get());
    std::vector<uint64_t> newk_map;   // per fmaps[j], once counted exactly
    // the TCP maps' related entries among those keys (saddr, daddr, ct word:
    // three uint4 each), which only the host maps can tell present or not
    std::vector<uint4> tcp_rel;
    auto map_want = [&](size_t j) -> uint64_t {
        const Map *m = fmaps[j];
        return m->kv.size() - m->gc_pending + claims + log_used +
               (newk_map.empty() ? newk_kind[m->ct_any ? 1 : 0] : newk_map[j]);
    };
    auto fits = [&](uint64_t nk) { return 4 * (used + ins + nk) <= 3 * slots; };
    auto maps_fit = [&]() {
        for (size_t j = 0; j < fmaps.size(); j++)
            if (map_want(j) > fmaps[j]->max_entries)
                return false;
        return true;
    };
    auto room = [&](uint64_t nk) { return fits(nk) && maps_fit(); };
    uint64_t *presorted = nullptr;
    if (ok && !room(newk)) {
        uint32_t exact[2] = {0, 0};
        A.cx = cx;   // (its set of related keys; the list reuses it later)
        A.rel_mask = 1;
        while (2ull * A.rel_mask + 1 <= 2 * cx_cap && A.rel_mask < (1u << 30))
            A.rel_mask = 2 * A.rel_mask + 1;
        const size_t nm = fmaps.size();
        if (nm && nm <= CTG_MAX_MAPS) {
            std::vector<uint32_t> sel(2 * nm + 1, 0);
            for (size_t j = 0; j < nm; j++)
                sel[j] = ct_owner_word((uint32_t)std::max(fmaps[j]->policy_lxc, 0),
                                       fmaps[j]->policy_lxc >= 0) | (fmaps[j]->ct_any ? 2u : 0u);
            const uint32_t rcap = (uint32_t)std::min<uint64_t>(nreqA, 1u << 22);
            if (c->evict_maps.ensure(4 * (2 * nm + 1)) || c->evict_rel.ensure(48ull * rcap + 48) ||
                hipMemcpyAsync(c->evict_maps.p, sel.data(), 4 * sel.size(), hipMemcpyHostToDevice,
                               s) != hipSuccess)
                return -EIO;
            A.emaps = (const uint32_t *)c->evict_maps.p;
            A.n_emaps = (uint32_t)nm;
            A.emcnt = (uint32_t *)c->evict_maps.p + nm;
            A.emrel = (uint4 *)c->evict_rel.p;
            A.emrel_cap = rcap;
        }
        if (cta_newkeys(A, V6, (uint32_t)nreqA, &presorted, exact, s))
            return -EIO;
        newk = exact[0];
        newk_kind[0] = exact[1];
        newk_kind[1] = exact[0] - exact[1];
        if (A.emcnt) {
            std::vector<uint32_t> cnt(nm + 1);
            if (hipMemcpyAsync(cnt.data(), A.emcnt, 4 * (nm + 1), hipMemcpyDeviceToHost, s) !=
                    hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                return -EIO;
            newk_map.assign(cnt.begin(), cnt.begin() + nm);
            if (cnt[nm] <= A.emrel_cap) {   // (else the count stays an upper bound)
                tcp_rel.resize(3ull * cnt[nm]);
                if (cnt[nm] &&
                    (hipMemcpyAsync(tcp_rel.data(), A.emrel, 16 * tcp_rel.size(),
                                    hipMemcpyDeviceToHost, s) != hipSuccess ||
                     hipStreamSynchronize(s) != hipSuccess))
                    return -EIO;
            }
            A.emaps = A.emcnt = nullptr;
            A.emrel = nullptr;
            A.n_emaps = 0;
        }
    }
    static const bool grow_host = getenv("CFC_CT_GROW_HOST") != nullptr;
    if (ok && !fits(newk) && may_grow && maps_fit() && grow_host) {
        // (A/B and debugging only: the old growth — the device state synced
        // into the maps, the CT group rebuilt larger through a commit —
        // unless other groups wait for a commit)
        bool others = false;
        uint64_t sg[NGROUPS];
        group_sigs(c, sg);
        for (int g = 0; g < NGROUPS; g++)
            others |= g != 3 && sg[g] != c->built_sig[g];
        if (!others) {
            uint64_t &mn = V6 ? c->ct_min6 : c->ct_min4;
            mn = std::max<uint64_t>(mn, 2 * (used + ins + newk));
            if (hipMemsetAsync(A.ms, 0, 12 * slots, s) != hipSuccess)
                return -EIO;
            c->built_sig[3] = ~0ull;
            if (int rc = commit_locked(c, s))
                return rc;
            return ct_apply_dev(c, in, out, mode, ep_lxc, s, false, false);
        }
    }
    if (ok && !fits(newk) && may_grow && maps_fit() && !grow_host) {
        // the batch outgrows the table but not its maps: the table grows on
        // the device (ct_grow: at least twice the slots, room for this
        // batch at under half load) and the batch is applied again on it —
        // its CT bytes keep the packet order already resolved
        uint64_t want = 2 * slots;
        while (want < 2 * (used + ins + newk))
            want *= 2;
        const int g = ct_grow(c, V6, want, s);
        if (g < 0)
            return g;
        if (g == 0)
            return ct_apply_dev(c, in, out, mode, ep_lxc, s, false, false);
    }
    if (ok && fits(newk) && !maps_fit() && c->ct_evict && !newk_map.empty()) {
        // a map at capacity (its exact new keys known): the device's own
        // pending inserts and log entries into the host mirror first (then
        // every map's size is its own), and if a map still overflows, evict
        // (ct_evict_maps: every overflowing map or none)
        if (claims || log_used || ins) {
            std::vector<uint32_t> keep(CTA_NCNT);   // (ct_sync reuses the counters)
            if (hipMemcpyAsync(keep.data(), A.cnt, 4 * CTA_NCNT, hipMemcpyDeviceToHost, s) !=
                    hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                return -EIO;
            if (int rc = ct_sync(c, s))
                return rc;
            if (hipMemcpyAsync(A.cnt, keep.data(), 4 * CTA_NCNT, hipMemcpyHostToDevice, s) !=
                    hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                return -EIO;
        }
        // a TCP map's related entry the batch's first create of its address
        // pair writes is a new key only when the map lacks it
        for (size_t q = 0; q + 2 < tcp_rel.size(); q += 3) {
            const uint32_t w = tcp_rel[q + 2].x;
            const size_t al = V6 ? 16 : 4;
            char k[38];
            const uint32_t z = 0;
            memcpy(k, &tcp_rel[q], al);
            memcpy(k + al, &tcp_rel[q + 1], al);
            memcpy(k + 2 * al, &z, 4);
            k[2 * al + 4] = (char)(w & 0xFF);
            k[2 * al + 5] = (char)((w >> 8) & 7);
            auto mit = G.ct_maps.find(ct_map_key(V6 ? 6 : 4, w & ~0x7FFu, 0));
            if (mit == G.ct_maps.end())
                continue;
            for (size_t j = 0; j < fmaps.size(); j++)
                if (fmaps[j] == mit->second && newk_map[j] &&
                    fmaps[j]->kv.count(std::string(k, 2 * al + 6)))
                    newk_map[j]--;
        }
        tcp_rel.clear();
        if (!maps_fit()) {
            std::vector<uint64_t> want(fmaps.size());
            for (size_t j = 0; j < fmaps.size(); j++)
                want[j] = map_want(j);
            const uint64_t nk = lbm ? 4 * n : mode == CFC_MODE_EGRESS ? 2 * n : n;
            if (A.sparse && cta_hs_fill(A, s))   // (the protect pass reads hs)
                return -EIO;
            const int rc = ct_evict_maps(c, V6, fmaps, want, A.hs, nk, s);
            if (rc < 0)
                return rc;
            if (rc == 2)   // (evicted on the host, not patched in: the host path)
                ok = false;
        }
        used = used_now();
    }
    ok = ok && room(newk);
    if (!ok && getenv("CFC_DEBUG_APPLY"))
        fprintf(stderr, "cfc: CT apply to the host path: %llu requests, %llu new keys, "
                        "%llu used of %llu slots\n", (unsigned long long)nreqA,
                (unsigned long long)newk, (unsigned long long)(used + ins),
                (unsigned long long)slots);
    if (!ok) {   // the scan's marks (and delete orders) go
        if (hipMemsetAsync(A.ms, 0, 12 * slots, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -EIO;
        return 1;
    }
    if (logbuf.bytes < log_rec * log_need) {   // grow, keeping the entries
        DevBuf nl;
        if (nl.ensure(log_rec * std::max<uint64_t>(2 * log_need, 1 << 16)))
            return -ENOMEM;
        if (log_used && (hipMemcpyAsync(nl.p, logbuf.p, log_rec * log_used,
                                        hipMemcpyDeviceToDevice, s) != hipSuccess ||
                         hipStreamSynchronize(s) != hipSuccess))
            return -EIO;
        std::swap(nl.p, logbuf.p);
        std::swap(nl.bytes, logbuf.bytes);
    }
    A.reqB = r2 + nr;        // (a create's related entry and reverse-NAT entry)
    A.reqB2 = r2 + 3 * nr;
    A.req_cap = (uint32_t)(2 * nr);
    A.cx = cx;
    A.cx2 = cx + cx_cap;
    A.cx_cap = (uint32_t)cx_cap;
    A.log = V6 ? nullptr : (CtLog *)logbuf.p;
    A.log6 = V6 ? (CtLog6 *)logbuf.p : nullptr;
    A.log_base = (uint32_t)log_used;
    A.log_cap = (uint32_t)(logbuf.bytes / log_rec - log_used);
    // from here the device table changes: the host mirror lags until ct_sync
    c->ct_dirty = true;
    c->ct6_dirty |= V6;
    // (no wait for the fold: the host's bookkeeping below was read after
    // route, the rest is stream-ordered before anything that reads the table)
    if (early && hc[CTA_NCX] > nroute_cap)
        return -EOVERFLOW;
    int rc = early ? cta_rest(A, V6, (uint32_t)nreqA, presorted, hc, s,
                              (const uint64_t *)c->cta_cxr.p, hc[CTA_NCX])
                   : cta_rest(A, V6, (uint32_t)nreqA, presorted, hc, s);
    if (rc) {
        // the table may hold some of the batch's inserts: no per-slot mark
        // or summary may leak into the next apply, the claims made count,
        // and the next commit rebuilds the CT group from the synced maps
        (void)hipStreamSynchronize(s);
        (void)hipMemsetAsync(A.ms, 0, 12 * slots, s);
        uint32_t cl = 0;
        (void)hipMemcpyAsync(&cl, A.cnt + CTA_CLAIMS, 4, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        claims += cl;
        ins += cl;
        c->built_sig[3] = ~0ull;
        return rc;
    }
    if (early) {
        // its counts follow it (settle() adds them before their next reader)
        if (hipMemcpyAsync(c->pend_cnt, A.cnt, 4 * CTA_NCNT, hipMemcpyDeviceToHost, s) !=
                hipSuccess ||
            hipEventRecord(c->pend_ev, s) != hipSuccess)
            return -EIO;
        c->pend = true;
        c->pend_v6 = V6;
    } else {
        claims += hc[CTA_CLAIMS];
        ins += hc[CTA_CLAIMS];
        log_used += hc[CTA_NLOG];
    }
    c->cta_seq++;
    c->n_apply_sparse += A.sparse;
    if (A.sum)   // (the finish cleared every summary the launch wrote)
        c->sum_dirty = false;
    return 0;
}

template <class Hdr>
int ct_apply_one(cfc_ctx *c, int family, const Hdr *in, const cfc_out *out, int mode,
                 uint16_t ep_lxc, void *stream)
{
    if (!c || !in || !out || !out->ct || !out->verdict || !out->identity)
        return -EINVAL;
    if (mode < CFC_MODE_INGRESS || mode > CFC_MODE_FULL)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (c->device == CFC_DEVICE_NONE)
        return -ENODEV;
    (void)hipSetDevice(c->device);
    const size_t n = in->n;
    if (!n || mode == CFC_MODE_XDP)
        return 0;
    hipStream_t s = (hipStream_t)stream;
    {
        const int rc = ct_apply_dev(c, in, out, mode, ep_lxc, s);
        c->ct_gen++;   // (the table, or the host maps, change from here)
        c->n_apply_dev += rc == 0;
        if (rc == 0) {
            // the creates' CONNTRACK_ACCOUNTING is in the device counts now:
            // they wait for a fold like a classify launch's (a CT group the
            // apply grew was folded before the rebuild, which cleared the flag)
            (void)hipEventRecord(c->last_done, s);
            c->last_stream = s;
            c->ctr_pending = true;
        }
        if (rc <= 0)
            return rc;
    }
    c->n_apply_host++;
    if (int rc = ct_sync(c, s))
        return rc;
    const size_t al = family == 4 ? 4 : 16;
    std::vector<uint8_t> sa(al * n), da(al * n), ct(n), tf(n, 0);
    std::vector<uint32_t> pt(n), mt(n), ident(n);
    std::vector<int32_t> ver(n);
    if (hipMemcpyAsync(sa.data(), in->saddr, al * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(da.data(), in->daddr, al * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(pt.data(), in->ports, 4 * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(mt.data(), in->meta, 4 * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(ident.data(), out->identity, 4 * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(ver.data(), out->verdict, 4 * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(ct.data(), out->ct, n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        (in->tcp_flags &&
         hipMemcpyAsync(tf.data(), in->tcp_flags, n, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    std::vector<uint32_t> hs;
    if (in->hash) {
        hs.resize(n);
        if (hipMemcpyAsync(hs.data(), in->hash, 4 * n, hipMemcpyDeviceToHost, s) !=
                hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -EIO;
    }
    CtApply A(c, family);
    const LbHost L(c);
    const bool lbon = family == 4 && L.on();
    const LbHost6 L6(c);
    const bool lb6on = family == 6 && L6.on();
    const uint32_t now = c->now;
    const uint8_t icmp = family == 4 ? 1 : 58;
    const uint32_t echo = family == 4 ? 8 : 128, echo_reply = family == 4 ? 0 : 129;
    // whether each key this apply writes was in the maps when the batch was
    // classified: a hit on an entry that was not (one a header's own egress
    // stage created, which its destination stage then finds) was not counted
    // by the device, so the walk counts it
    // (keyed by map and tuple: one tuple can live in several maps, e.g. a
    // TCP and a UDP create's ICMP entry, or a global and a local map)
    // (and a hit after this walk wrote the key anew — a related entry a later
    // create overwrote — counts too: the device's count of it went with the
    // entry the write replaced, ct_drop_counts)
    std::map<std::pair<const Map *, std::string>, bool> initial;
    std::set<std::pair<const Map *, std::string>> written;
    auto note = [&](Map *mp, const std::string &key) {
        initial.emplace(std::make_pair((const Map *)mp, key), mp->kv.count(key) != 0);
    };
    auto put_new = [&](Map *mp, const std::string &key, const CtEntry &e) {
        note(mp, key);
        written.emplace((const Map *)mp, key);
        (void)mp->update(key.data(), &e, 0);
    };
    auto fresh = [&](const Map *mp, const std::string &key) {
        auto it = initial.find(std::make_pair(mp, key));
        return (it != initial.end() && !it->second) || written.count(std::make_pair(mp, key));
    };
    bool ct_changed = false;   // (CT bytes the packet order changed)
    for (size_t i = 0; i < n; i++) {
        const uint8_t cb = ct[i];
        const uint32_t proto = mt[i] & 0xFF, len = mt[i] >> 16;
        const bool is_tcp = proto == 6, syn = (mt[i] & CFC_HF_TCP_CLOSE) != 0;
        const uint8_t tflags = is_tcp ? tf[i] : 0;
        // lb4_local / lb6_local created its CT_SERVICE entry before it found
        // no backend
        const bool no_svc = (lbon || lb6on) && mode == CFC_MODE_EGRESS &&
                            ver[i] == -158;   // DROP_NO_SERVICE
        if (!(cb & (CFC_CT_DONE | CFC_CT_DONE << 4)) && !no_svc)
            continue;
        const uint8_t *s_ = &sa[al * i], *d_ = &da[al * i];
        // the tuple of the sender's lookup (stage 0 of an egress batch) and
        // the packet every later stage sees: a service step and a reply's
        // reverse NAT move them (IPv4 with a load balancer)
        uint32_t tsa = 0, tda = 0, tpt = pt[i], psa = 0, pda = 0, ppt = pt[i];
        if (family == 4) {
            memcpy(&tsa, s_, 4);
            memcpy(&tda, d_, 4);
            psa = tsa;
            pda = tda;
        }
        LbState x;
        if (lbon && mode == CFC_MODE_EGRESS && ((cb & CFC_CT_DONE) || no_svc)) {
            Map *m0 = A.ct_map((int)ep_lxc, proto != 6);
            const uint32_t h = hs.empty() ? flow_hash4_host(tsa, tda, pt[i], proto) : hs[i];
            uint32_t p2 = pt[i];
            x = lb4_step(L, m0, tsa, tda, p2, psa, pda, (uint8_t)proto, h);
            if (x.svc) {
                tda = x.tda;
                tpt = ppt = p2;
            }
            if (x.svc && m0) {   // the CT_SERVICE entry: hit (updated) or created
                const uint32_t type = pt[i] & 0xFF;
                const int act = proto == 6 ? (syn ? 2 : 1) : proto == 17 ? 1
                                : (type == 3 || type == 11 || type == 12 || type == 0) ? 0 : 1;
                auto it = m0->kv.find(x.ksvc);
                if (it != m0->kv.end()) {
                    ct_hit_update(m0, it->second, act, 0, true, len, now, is_tcp, syn, tflags);
                    if (x.reslave && !x.drop)   // ct_update4_slave
                        memcpy(&it->second.val[40], &x.slave, 2);
                } else {
                    CtEntry e{};
                    e.slave = x.slave0;
                    ct_upd_timeout(e, now, is_tcp, 0, is_tcp, 0);
                    e.tx_packets = 1;
                    e.tx_bytes = len;
                    CtEntry es = e;
                    if (x.reslave && !x.drop)   // ct_update4_slave: this entry only
                        es.slave = x.slave;
                    put_new(m0, x.ksvc, es);
                    std::string ki = x.ksvc;
                    memset(&ki[8], 0, 4);
                    ki[12] = (char)icmp;
                    ki[13] = (char)(4 | 2);
                    e.bits |= CTB_SEEN_NON_SYN;
                    if (m0->kv.count(ki))
                        ct_drop_counts(c, m0, ki, s);
                    put_new(m0, ki, e);
                }
            }
        }
        // IPv6: lb6_local's CT_SERVICE entry, and the tuple / packet it
        // leaves (no loopback case: the packet's daddr is the tuple's)
        uint8_t t6da[16], p6sa[16], p6da[16];
        uint32_t p6pt = pt[i];
        memcpy(p6sa, s_, al == 16 ? 16 : 0);
        memcpy(t6da, d_, al == 16 ? 16 : 0);
        LbState6 x6;
        if (lb6on && mode == CFC_MODE_EGRESS && ((cb & CFC_CT_DONE) || no_svc)) {
            Map *m0 = A.ct_map((int)ep_lxc, proto != 6);
            const uint32_t h = hs.empty() ? flow_hash4_host(fold6_host(s_), fold6_host(d_), pt[i],
                                                            proto)
                                          : hs[i];
            x6 = lb6_step(L6, m0, s_, d_, p6pt, (uint8_t)proto, h);
            if (x6.svc) {
                memcpy(t6da, x6.tda, 16);
                x.drop = x6.drop;
            }
            if (x6.svc && m0) {   // the CT_SERVICE entry: hit (updated) or created
                const uint32_t type = pt[i] & 0xFF;
                const int act = proto == 6 ? (syn ? 2 : 1) : proto == 17 ? 1
                                : ((type >= 1 && type <= 4) || type == 129) ? 0 : 1;
                auto it = m0->kv.find(x6.ksvc);
                if (it != m0->kv.end()) {
                    ct_hit_update(m0, it->second, act, 0, true, len, now, is_tcp, syn, tflags);
                    if (x6.reslave && !x6.drop)   // ct_update6_slave
                        memcpy(&it->second.val[40], &x6.slave, 2);
                } else {
                    CtEntry e{};
                    e.slave = x6.slave0;
                    ct_upd_timeout(e, now, is_tcp, 0, is_tcp, 0);
                    e.tx_packets = 1;
                    e.tx_bytes = len;
                    CtEntry es = e;
                    if (x6.reslave && !x6.drop)
                        es.slave = x6.slave;
                    put_new(m0, x6.ksvc, es);
                    std::string ki = x6.ksvc;
                    memset(&ki[32], 0, 4);
                    ki[36] = (char)icmp;
                    ki[37] = (char)(4 | 2);
                    e.bits |= CTB_SEEN_NON_SYN;
                    if (m0->kv.count(ki))
                        ct_drop_counts(c, m0, ki, s);
                    put_new(m0, ki, e);
                }
            }
        }
        memcpy(p6da, t6da, al == 16 ? 16 : 0);
        if (x.drop)
            continue;
        const int last = (cb & (CFC_CT_DONE << 4)) ? 1 : 0;
        for (int st = 0; st < 2; st++) {
            const uint8_t cs = (uint8_t)(cb >> (4 * st));
            if (!(cs & CFC_CT_DONE))
                continue;
            const bool eg = mode == CFC_MODE_EGRESS && st == 0;
            const int dir = eg ? 0 : 1;   // CT_EGRESS / CT_INGRESS
            // the addresses and L4 word this stage's lookup read
            const uint8_t *ks = s_, *kd_ = d_;
            uint32_t kp = pt[i];
            if (family == 4) {
                ks = eg ? (const uint8_t *)&tsa : (const uint8_t *)&psa;
                kd_ = eg ? (const uint8_t *)&tda : (const uint8_t *)&pda;
                kp = eg ? tpt : ppt;
            } else if (lb6on) {
                ks = eg ? s_ : p6sa;
                kd_ = eg ? t6da : p6da;
                kp = p6pt;
            }
            const int dst = A.endpoint(family == 4 ? (const uint8_t *)&pda : lb6on ? p6da : d_);
            Map *m = A.ct_map(eg ? (int)ep_lxc : dst, proto != 6);
            if (!m)
                continue;
            // the tuple exactly as ct_lookup4/6 builds it (conntrack.h)
            uint32_t td, ts, fl = dir == 1 ? 0u : 1u;
            int action;
            if (proto == 6 || proto == 17) {
                td = kp & 0xFFFF;
                ts = kp >> 16;
                action = (proto == 6 && (mt[i] & CFC_HF_TCP_CLOSE)) ? 2 : 1;
            } else if (proto == icmp) {
                const uint32_t type = kp & 0xFF;
                const bool rel = family == 4 ? (type == 3 || type == 11 || type == 12)
                                             : (type >= 1 && type <= 4);
                td = (!rel && type == echo_reply) ? echo : 0;
                ts = (!rel && type == echo) ? echo : 0;
                fl |= rel ? 2u : 0u;
                action = (rel || type == echo_reply) ? 0 : 1;
            } else {
                continue;
            }
            auto tuple = [&](const uint8_t *d, const uint8_t *sr, uint32_t dp,
                             uint32_t sp, uint32_t f) {
                char k[38];
                memcpy(k, d, al);
                memcpy(k + al, sr, al);
                const uint16_t a = (uint16_t)dp, b = (uint16_t)sp;
                memcpy(k + 2 * al, &a, 2);
                memcpy(k + 2 * al + 2, &b, 2);
                k[2 * al + 4] = (char)proto;
                k[2 * al + 5] = (char)f;
                return std::string(k, 2 * al + 6);
            };
            const std::string k1 = tuple(kd_, ks, td, ts, fl);
            const std::string k2 = tuple(ks, kd_, ts, td, fl ^ 1u);
            int b = cs & CFC_CT_RES_MASK;
            const bool dropped = st == last && ver[i] == -133;   // DROP_POLICY
            if (b < 2) {
                // CT_NEW / CT_ESTABLISHED as the headers before left k2 (the
                // reference's packet order, ctorder.hip); the launch's k1
                // result stands (no write of the batch has k1's flag)
                const bool allowed = (cs & CFC_CT_CREATE) || (b == 1 && !dropped);
                b = m->kv.count(k2) ? 1 : 0;
                const uint8_t ncs = (uint8_t)(b | CFC_CT_DONE | ((b == 0 && allowed) ? CFC_CT_CREATE : 0));
                if (ncs != cs) {
                    ct[i] = (uint8_t)((ct[i] & ~(0xF << (4 * st))) | ncs << (4 * st));
                    ct_changed = true;
                    c->n_ord_changed++;
                }
            }
            const uint8_t csn = (uint8_t)(ct[i] >> (4 * st));
            if (b >= 2) {                       // CT_REPLY / CT_RELATED
                auto it = m->kv.find(k1);
                if (it != m->kv.end()) {
                    ct_hit_update(m, it->second, action, dir, fresh(m, k1), len, now,
                                  is_tcp, syn, tflags);
                    if (lbon && eg) {   // the egress reply's reverse NAT
                        CtEntry e;
                        memcpy(&e, it->second.val.data(), sizeof(e));
                        L.rev_nat(e, (uint8_t)proto, psa, pda, ppt);
                    }
                    if (lb6on && eg) {
                        CtEntry e;
                        memcpy(&e, it->second.val.data(), sizeof(e));
                        L6.rev_nat(e.rev_nat_index, (uint8_t)proto, p6sa, p6pt);
                    }
                }
            } else if (b == 1) {                // CT_ESTABLISHED
                auto it = m->kv.find(k2);
                if (it != m->kv.end()) {
                    ct_hit_update(m, it->second, action, dir, fresh(m, k2), len, now,
                                  is_tcp, syn, tflags);
                    if (dropped) {              // ct_delete4/6
                        ct_drop_counts(c, m, k2, s);
                        note(m, k2);
                        (void)m->erase(k2.data());
                    }
                }
            } else if (csn & CFC_CT_CREATE) {
                auto it = m->kv.find(k2);
                if (it != m->kv.end()) {        // created earlier in this batch
                    ct_hit_update(m, it->second, action, dir, true, len, now, is_tcp,
                                  syn, tflags);
                    continue;
                }
                // ct_create4/6 (conntrack.h:615-662, :691-772): timeouts
                // with seen_flags.syn = is_tcp (lower_bits stay 0)
                CtEntry e{};
                ct_upd_timeout(e, now, is_tcp, dir, is_tcp, 0);
                (dir == 1 ? e.rx_packets : e.tx_packets) = 1;
                (dir == 1 ? e.rx_bytes : e.tx_bytes) = len;
                e.src_sec_id = mode == CFC_MODE_EGRESS ? c->seclabel[ep_lxc] : ident[i];
                if (family == 6 && dir == 1)    // ipv6_policy, bpf_lxc.c:787-788
                    e.rev_nat_index = (uint16_t)(kd_[12] | kd_[13] << 8);
                if (family == 6 && eg && x6.svc) {   // lb6_local's ct_state
                    e.rev_nat_index = x6.rev_nat;
                    e.slave = x6.slave;
                }
                if (eg && x.svc) {              // lb4_local's ct_state
                    e.rev_nat_index = x.rev_nat;
                    e.slave = x.slave;
                    if (x.loopback)
                        e.bits |= CTB_LB_LOOPBACK;
                }
                if (c->hop_nat46 && dir != 1)   // a NAT64 hop's egress create (conntrack.h:714-716)
                    e.bits |= CTB_NAT46;
                put_new(m, k2, e);
                if (eg && x.svc && x.addr) {    // the reverse-NAT entry
                    std::string kx = k2;
                    memcpy(&kx[0], &x.addr, 4);
                    if (x.loopback) {
                        kx[13] = 1;             // TUPLE_F_IN
                        memcpy(&kx[4], &x.svc_addr, 4);
                    }
                    if (m->kv.count(kx))
                        ct_drop_counts(c, m, kx, s);
                    put_new(m, kx, e);
                }
                e.bits |= CTB_SEEN_NON_SYN;     // "For ICMP, there is no SYN"
                const std::string ki = [&] {
                    std::string t = k2;
                    memset(&t[2 * al], 0, 4);
                    t[2 * al + 4] = (char)icmp;
                    t[2 * al + 5] = (char)((fl ^ 1u) | 2u);
                    return t;
                }();
                if (m->kv.count(ki))            // overwritten
                    ct_drop_counts(c, m, ki, s);
                put_new(m, ki, e);
            }
        }
    }
    if (ct_changed &&
        hipMemcpyAsync(out->ct, ct.data(), n, hipMemcpyHostToDevice, s) != hipSuccess)
        return -EIO;
    if (hipStreamSynchronize(s) != hipSuccess)
        return -EIO;
    return 0;
}

// cfc_ct_apply_v4 / _v6: the batch's own stages, then — a batch with a NAT
// hop batch (nat_hop) — the hops' stages into the other family's maps
// (apply_hop of the oracle): NAT64 as the endpoint's IPv4 egress batch
// (its creates carry nat46), NAT46 as an IPv6 ingress batch.  While its own
// family folds, a hop header's stage counts as allowed (it led to the hop)
// and alone (bits 4-7, the event word aside); nat_scatter puts the hop's
// results back afterwards, with its packet-order CT result.
template <class Hdr>
int ct_apply(cfc_ctx *c, int family, const Hdr *in, const cfc_out *out, int mode,
             uint16_t ep_lxc, void *stream)
{
    if (!c || !in || !out || !out->ct || !out->verdict || !out->identity)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (c->seg.valid && c->seg.ct == (const void *)out->ct && c->seg.saddr == in->saddr &&
        c->seg.n == in->n && c->seg.mode == mode && c->seg.ep == ep_lxc &&
        c->seg.family == family) {
        // a batch cut for traffic to itself: its segments before the last
        // were folded by cfc_classify; fold the last
        c->seg.valid = false;
        const uint64_t a = c->seg.off;
        const Hdr si = sub_batch(*in, a, in->n - a);
        const cfc_out so = sub_out(*out, a, family == 6);
        return ct_apply(c, family, &si, &so, mode, ep_lxc, stream);
    }
    auto it = c->nat.find((const void *)out->ct);
    if (it == c->nat.end() || it->second.family != family || it->second.saddr != in->saddr ||
        it->second.n != in->n || it->second.mode != mode || it->second.ep != ep_lxc)
        return ct_apply_one(c, family, in, out, mode, ep_lxc, stream);
    cfc_ctx::NatRec &r = it->second;
    r.family = 0;   // (consumed; its buffers stay for the next hop batch)
    hipStream_t s = (hipStream_t)stream;
    (void)hipSetDevice(c->device);
    const uint32_t *idx = (const uint32_t *)r.idx.p;
    if (nat_pre(idx, r.m, *out, s))
        return -EIO;
    int rc = ct_apply_one(c, family, in, out, mode, ep_lxc, stream);
    if (!rc) {
        c->hop_nat46 = family == 6;
        rc = family == 6 ? ct_apply_one(c, 4, &r.h4, &r.o, CFC_MODE_EGRESS, ep_lxc, stream)
                         : ct_apply_one(c, 6, &r.h6, &r.o, CFC_MODE_INGRESS, (uint16_t)0, stream);
        c->hop_nat46 = false;
        c->nat46_seen |= family == 6;
    }
    const int rc2 = nat_scatter(idx, r.m, r.o, *out, s);
    return rc ? rc : rc2;
}

// ---- cfc_ct_gc: ctmap.GC with doFiltering (pkg/maps/ctmap/ctmap.go:303-350)
struct GcFilterHost {
    const cfc_ct_gc_filter &f;
    // doFiltering on a CT key's two addresses (daddr at 0, saddr at al)
    bool in(const cfc_ip *set, uint32_t n, int fam, const uint8_t *a) const
    {
        const size_t al = fam == 4 ? 4 : 16;
        for (uint32_t i = 0; i < n; i++)
            if (set[i].family == fam && !memcmp(set[i].addr, a, al))
                return true;
        return false;
    }
    bool del(int fam, const uint8_t *key, uint32_t lifetime) const
    {
        const size_t al = fam == 4 ? 4 : 16;
        const uint8_t *da = key, *sa = key + al;
        if ((f.flags & CFC_GC_REMOVE_EXPIRED) && lifetime < f.time)
            return true;
        if ((f.flags & CFC_GC_VALID_IPS) && !in(f.valid_ips, f.n_valid, fam, da) &&
            !in(f.valid_ips, f.n_valid, fam, sa))
            return true;
        return (f.flags & CFC_GC_MATCH_IPS) &&
               (in(f.match_ips, f.n_match, fam, da) || in(f.match_ips, f.n_match, fam, sa));
    }
};

// the IPv4 part on the device: the CT table and the pending CtLog
int ct_gc_dev(cfc_ctx *c, const std::vector<Map *> &sel, const cfc_ct_gc_filter &f,
              cfc_ct_gc_stats &st, hipStream_t s, const uint32_t *protect)
{
    settle(c);
    Epoch &E = *c->epoch;
    GCt &G = *E.ct;
    const uint64_t slots = G.slots4;
    // the selected maps' selector words, and the IPv4 addresses of the sets
    std::vector<uint32_t> mw;
    std::vector<Map *> mm;
    for (Map *m : sel)
        if (m->role == ROLE_CT4) {
            mw.push_back(ct_owner_word((uint32_t)std::max(m->policy_lxc, 0), m->policy_lxc >= 0) |
                         (m->ct_any ? 2u : 0u));
            mm.push_back(m);
        }
    if (mw.empty())
        return 0;
    auto v4set = [](const cfc_ip *set, uint32_t n) {
        std::vector<uint32_t> v;
        for (uint32_t i = 0; i < n; i++)
            if (set[i].family == 4) {
                uint32_t a;
                memcpy(&a, set[i].addr, 4);
                v.push_back(a);
            }
        std::sort(v.begin(), v.end());
        return v;
    };
    const std::vector<uint32_t> va = (f.flags & CFC_GC_VALID_IPS) ? v4set(f.valid_ips, f.n_valid)
                                                                   : std::vector<uint32_t>();
    const std::vector<uint32_t> ma = (f.flags & CFC_GC_MATCH_IPS) ? v4set(f.match_ips, f.n_match)
                                                                   : std::vector<uint32_t>();
    // every entry the host mirror holds can be deleted once before its next
    // sync (one the host never saw needs no log record): the log's room
    const uint64_t need = c->gc_log_used + G.n_ct4 + 1;
    if (c->gc_log.bytes < sizeof(CtGcRec) * need) {
        DevBuf nl;
        if (nl.ensure(sizeof(CtGcRec) * need))
            return -ENOMEM;
        if (c->gc_log_used &&
            (hipMemcpyAsync(nl.p, c->gc_log.p, sizeof(CtGcRec) * c->gc_log_used,
                            hipMemcpyDeviceToDevice, s) != hipSuccess ||
             hipStreamSynchronize(s) != hipSuccess))
            return -EIO;
        std::swap(nl.p, c->gc_log.p);
        std::swap(nl.bytes, c->gc_log.bytes);
    }
    const size_t set_words = CTG_MAX_MAPS * 2 + va.size() + ma.size() + 1;
    if (c->gc_sets.ensure(4 * set_words) || c->gc_cnt.ensure(4 * CTG_NCNT) ||
        (c->log_used && c->gc_tmp.ensure(sizeof(CtLog) * c->log_used)))
        return -ENOMEM;
    uint32_t *sets = (uint32_t *)c->gc_sets.p, *cnt = (uint32_t *)c->gc_cnt.p;
    uint64_t deleted = 0, fresh = 0, live = 0, nonfree = 0, freed = 0, last_freed = 0;
    uint32_t logkept = (uint32_t)c->log_used, logn = (uint32_t)c->log_used;
    for (size_t a = 0; a < mw.size(); a += CTG_MAX_MAPS) {
        const uint32_t nm = (uint32_t)std::min<size_t>(CTG_MAX_MAPS, mw.size() - a);
        std::vector<uint32_t> hs(CTG_MAX_MAPS * 2, 0);
        std::copy(mw.begin() + (long)a, mw.begin() + (long)a + nm, hs.begin());
        hs.insert(hs.end(), va.begin(), va.end());
        hs.insert(hs.end(), ma.begin(), ma.end());
        CtGcArgs A{};
        A.ct4 = (Ct4Slot *)G.ct4.p;
        A.st = (CtState *)G.ct_st.p;
        A.slots = slots;
        A.mask = (uint32_t)(slots - 1);
        A.maps = sets;
        A.n_maps = nm;
        A.mcnt = sets + CTG_MAX_MAPS;
        A.flags = ((f.flags & CFC_GC_REMOVE_EXPIRED) ? CTG_REMOVE_EXPIRED : 0u) |
                  ((f.flags & CFC_GC_VALID_IPS) ? CTG_VALID : 0u) |
                  ((f.flags & CFC_GC_MATCH_IPS) ? CTG_MATCH : 0u);
        A.time = f.time;
        A.valid = sets + 2 * CTG_MAX_MAPS;
        A.n_valid = (uint32_t)va.size();
        A.match = A.valid + va.size();
        A.n_match = (uint32_t)ma.size();
        A.log = (CtGcRec *)c->gc_log.p + c->gc_log_used + deleted;
        A.log_cap = (uint32_t)(c->gc_log.bytes / sizeof(CtGcRec) - c->gc_log_used - deleted);
        A.cnt = cnt;
        A.protect = protect;
        uint32_t hc[CTG_NCNT], hm[CTG_MAX_MAPS];
        if (hipMemcpyAsync(sets, hs.data(), 4 * hs.size(), hipMemcpyHostToDevice, s) !=
                hipSuccess ||
            hipMemsetAsync(cnt, 0, 4 * CTG_NCNT, s) != hipSuccess || ct_gc4(A, s))
            return -EIO;
        // the pending TCP-map ICMP entries of the applies, compacted (all
        // logn places copied back: the kept ones lead, the rest is past the
        // new count — no wait for that count first)
        if (logn && (ct_gc_log(A, (const CtLog *)c->cta_log.p, logn, (CtLog *)c->gc_tmp.p, s) ||
                     hipMemcpyAsync(c->cta_log.p, c->gc_tmp.p, sizeof(CtLog) * logn,
                                    hipMemcpyDeviceToDevice, s) != hipSuccess))
            return -EIO;
        if (hipMemcpyAsync(hc, cnt, 4 * CTG_NCNT, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(hm, A.mcnt, 4 * nm, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -EIO;
        if (hc[CTG_DELETED] > A.log_cap)
            return -EIO;   // (not reached: the log has room for every entry)
        for (uint32_t j = 0; j < nm; j++)
            mm[a + j]->gc_pending += hm[j];
        deleted += hc[CTG_DELETED];
        fresh += hc[CTG_FRESH];
        live += hc[CTG_LIVE];
        nonfree = hc[CTG_NONFREE];
        freed += hc[CTG_FREED];
        last_freed = hc[CTG_FREED];
        if (logn) {
            logkept = hc[CTG_LOGKEPT];
            logn = logkept;
        }
    }
    c->gc_log_used += deleted;
    c->cta_claims -= std::min(c->cta_claims, fresh);
    // exact occupancy now: the non-free slots the last pass saw, less what
    // its trim freed (an earlier chunk's deletes are tombstones it counted)
    c->ct_used = nonfree >= last_freed ? nonfree - last_freed : 0;
    c->cta_ins = 0;
    c->ct_used_valid = true;
    if (deleted || fresh)
        c->ct_dirty = true;
    c->ct_gen++;   // the table changed under any classify launch's hit slots
    st.device_deleted += deleted + fresh;
    st.log_deleted += c->log_used - logkept;
    st.alive += live + logkept;
    st.slots_freed += freed;
    c->log_used = logkept;
    return 0;
}

// the IPv6 part on the device (doGC6, ctmap.go:239): the CT6 table and the
// pending CtLog6 — the same passes as ct_gc_dev (k_ct_gc<true>), a slot's
// addresses read only for the selected maps' entries
int ct_gc_dev6(cfc_ctx *c, const std::vector<Map *> &sel, const cfc_ct_gc_filter &f,
               cfc_ct_gc_stats &st, hipStream_t s)
{
    settle(c);
    Epoch &E = *c->epoch;
    GCt &G = *E.ct;
    const uint64_t slots = G.slots6;
    std::vector<uint32_t> mw;
    std::vector<Map *> mm;
    for (Map *m : sel)
        if (m->role == ROLE_CT6) {
            mw.push_back(ct_owner_word((uint32_t)std::max(m->policy_lxc, 0), m->policy_lxc >= 0) |
                         (m->ct_any ? 2u : 0u));
            mm.push_back(m);
        }
    if (mw.empty() || !slots)
        return 0;
    auto v6set = [](const cfc_ip *set, uint32_t n) {
        std::vector<uint4> v;
        for (uint32_t i = 0; i < n; i++)
            if (set[i].family == 6) {
                uint4 a;
                memcpy(&a, set[i].addr, 16);
                v.push_back(a);
            }
        std::sort(v.begin(), v.end(), [](const uint4 &a, const uint4 &b) {
            return a.x != b.x ? a.x < b.x : a.y != b.y ? a.y < b.y : a.z != b.z ? a.z < b.z
                                                                                : a.w < b.w;
        });
        return v;
    };
    const std::vector<uint4> va = (f.flags & CFC_GC_VALID_IPS) ? v6set(f.valid_ips, f.n_valid)
                                                                : std::vector<uint4>();
    const std::vector<uint4> ma = (f.flags & CFC_GC_MATCH_IPS) ? v6set(f.match_ips, f.n_match)
                                                                : std::vector<uint4>();
    const uint64_t need = c->gc_log6_used + G.n_ct6 + 1;
    if (c->gc_log6.bytes < sizeof(CtGcRec6) * need) {
        DevBuf nl;
        if (nl.ensure(sizeof(CtGcRec6) * need))
            return -ENOMEM;
        if (c->gc_log6_used &&
            (hipMemcpyAsync(nl.p, c->gc_log6.p, sizeof(CtGcRec6) * c->gc_log6_used,
                            hipMemcpyDeviceToDevice, s) != hipSuccess ||
             hipStreamSynchronize(s) != hipSuccess))
            return -EIO;
        std::swap(nl.p, c->gc_log6.p);
        std::swap(nl.bytes, c->gc_log6.bytes);
    }
    // sets: the maps' words (2 * CTG_MAX_MAPS u32), then the addresses (uint4)
    const size_t set_bytes = 8 * CTG_MAX_MAPS + 16 * (va.size() + ma.size() + 1);
    if (c->gc_sets.ensure(set_bytes) || c->gc_cnt.ensure(4 * CTG_NCNT) ||
        (c->log6_used && c->gc_tmp.ensure(sizeof(CtLog6) * c->log6_used)))
        return -ENOMEM;
    uint32_t *sets = (uint32_t *)c->gc_sets.p, *cnt = (uint32_t *)c->gc_cnt.p;
    uint64_t deleted = 0, fresh = 0, live = 0, nonfree = 0, freed = 0, last_freed = 0;
    uint32_t logkept = (uint32_t)c->log6_used, logn = (uint32_t)c->log6_used;
    for (size_t a = 0; a < mw.size(); a += CTG_MAX_MAPS) {
        const uint32_t nm = (uint32_t)std::min<size_t>(CTG_MAX_MAPS, mw.size() - a);
        std::vector<uint32_t> hs(CTG_MAX_MAPS * 2, 0);
        std::copy(mw.begin() + (long)a, mw.begin() + (long)a + nm, hs.begin());
        std::vector<uint4> addrs(va);
        addrs.insert(addrs.end(), ma.begin(), ma.end());
        CtGcArgs A{};
        A.ct6 = (Ct6Slot *)G.ct6.p;
        A.st = (CtState *)G.ct_st.p + G.slots4;
        A.slots = slots;
        A.mask = (uint32_t)(slots - 1);
        A.maps = sets;
        A.n_maps = nm;
        A.mcnt = sets + CTG_MAX_MAPS;
        A.flags = ((f.flags & CFC_GC_REMOVE_EXPIRED) ? CTG_REMOVE_EXPIRED : 0u) |
                  ((f.flags & CFC_GC_VALID_IPS) ? CTG_VALID : 0u) |
                  ((f.flags & CFC_GC_MATCH_IPS) ? CTG_MATCH : 0u);
        A.time = f.time;
        A.valid6 = (const uint4 *)(sets + 2 * CTG_MAX_MAPS);
        A.n_valid = (uint32_t)va.size();
        A.match6 = A.valid6 + va.size();
        A.n_match = (uint32_t)ma.size();
        A.log6 = (CtGcRec6 *)c->gc_log6.p + c->gc_log6_used + deleted;
        A.log_cap = (uint32_t)(c->gc_log6.bytes / sizeof(CtGcRec6) - c->gc_log6_used - deleted);
        A.cnt = cnt;
        uint32_t hc[CTG_NCNT], hm[CTG_MAX_MAPS];
        if (hipMemcpyAsync(sets, hs.data(), 4 * hs.size(), hipMemcpyHostToDevice, s) !=
                hipSuccess ||
            (!addrs.empty() &&
             hipMemcpyAsync(sets + 2 * CTG_MAX_MAPS, addrs.data(), 16 * addrs.size(),
                            hipMemcpyHostToDevice, s) != hipSuccess) ||
            hipMemsetAsync(cnt, 0, 4 * CTG_NCNT, s) != hipSuccess || ct_gc4(A, s))
            return -EIO;
        if (logn && (ct_gc_log6(A, (const CtLog6 *)c->cta_log6.p, logn, (CtLog6 *)c->gc_tmp.p, s) ||
                     hipMemcpyAsync(c->cta_log6.p, c->gc_tmp.p, sizeof(CtLog6) * logn,
                                    hipMemcpyDeviceToDevice, s) != hipSuccess))
            return -EIO;
        if (hipMemcpyAsync(hc, cnt, 4 * CTG_NCNT, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(hm, A.mcnt, 4 * nm, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -EIO;
        if (hc[CTG_DELETED] > A.log_cap)
            return -EIO;
        for (uint32_t j = 0; j < nm; j++)
            mm[a + j]->gc_pending += hm[j];
        deleted += hc[CTG_DELETED];
        fresh += hc[CTG_FRESH];
        live += hc[CTG_LIVE];
        nonfree = hc[CTG_NONFREE];
        freed += hc[CTG_FREED];
        last_freed = hc[CTG_FREED];
        if (logn) {
            logkept = hc[CTG_LOGKEPT];
            logn = logkept;
        }
    }
    c->gc_log6_used += deleted;
    c->cta_claims6 -= std::min(c->cta_claims6, fresh);
    c->ct_used6 = nonfree >= last_freed ? nonfree - last_freed : 0;
    c->cta_ins6 = 0;
    c->ct_used6_valid = true;
    if (deleted || fresh) {
        c->ct_dirty = true;
        c->ct6_dirty = true;
    }
    c->ct_gen++;
    st.device_deleted += deleted + fresh;
    st.log_deleted += c->log6_used - logkept;
    st.alive += live + logkept;
    st.slots_freed += freed;
    c->log6_used = logkept;
    return 0;
}

int ct_gc(cfc_ctx *c, int fd, const cfc_ct_gc_filter *f, cfc_ct_gc_stats *out, hipStream_t s)
{
    if (f->flags & ~(CFC_GC_REMOVE_EXPIRED | CFC_GC_VALID_IPS | CFC_GC_MATCH_IPS))
        return -EINVAL;
    if (((f->flags & CFC_GC_VALID_IPS) && f->n_valid && !f->valid_ips) ||
        ((f->flags & CFC_GC_MATCH_IPS) && f->n_match && !f->match_ips))
        return -EINVAL;
    std::vector<Map *> sel;
    if (fd >= 0) {
        Map *m = get_map(c, fd);
        if (!m)
            return -EBADF;
        if (!m->ct())
            return -EINVAL;
        sel.push_back(m);
    } else {
        for (auto &kv : c->maps)
            if (kv.second->ct())
                sel.push_back(kv.second.get());
    }
    // host-side CT changes into the device table first
    if (int rc = commit_locked(c, s))
        return rc;
    order_after_launches(c, s);
    cfc_ct_gc_stats st{};
    Epoch &E = *c->epoch;
    const bool dev4 = E.ct->slots4 && E.ct->ct_st.p, dev6 = E.ct->slots6 && E.ct->ct_st.p;
    // both families on the device (doGC4 / doGC6); an IPv6 map without a
    // device table is collected on the host after its device applies are
    // synchronised (their pending-log entries first)
    bool v6host = false;
    for (Map *m : sel)
        v6host |= m->role == ROLE_CT6 && !m->kv.empty() && !dev6;
    if (v6host && c->ct6_dirty)
        if (int rc = ct_sync(c, s))
            return rc;
    if (dev4)
        if (int rc = ct_gc_dev(c, sel, *f, st, s, nullptr))
            return rc;
    if (dev6)
        if (int rc = ct_gc_dev6(c, sel, *f, st, s))
            return rc;
    // what only the host holds: maps without a device table, the TCP maps'
    // ICMP entries (no lookup reaches them: not in the device table)
    const GcFilterHost H{*f};
    for (Map *m : sel) {
        const bool v6 = m->role == ROLE_CT6, all = v6 ? !dev6 : !dev4;
        if (!all && !m->n_aux)
            continue;
        uint64_t kept = 0, gone = 0;
        for (auto it = m->kv.begin(); it != m->kv.end();) {
            const std::string &k = it->first;
            if (!all && !m->aux_key(k)) {
                ++it;
                continue;
            }
            uint32_t life = 0;
            if (it->second.val.size() >= 36)
                memcpy(&life, &it->second.val[32], 4);
            if (H.del(v6 ? 6 : 4, (const uint8_t *)k.data(), life)) {
                // journaled where the device table holds it: the next commit
                // turns its slot into a tombstone
                it = m->ct_erase_at(it, all);
                gone++;
            } else {
                kept++;
                ++it;
            }
        }
        st.host_deleted += gone;
        st.alive += kept;
    }
    st.deleted = st.device_deleted + st.log_deleted + st.host_deleted;
    if (out)
        *out = st;
    return 0;
}

}  // namespace

extern "C" {

int cfc_ct_apply_v4(cfc_ctx *c, const cfc_hdr_v4 *in, const cfc_out *out,
                    int mode, uint16_t ep_lxc, void *stream)
{
    return ct_apply(c, 4, in, out, mode, ep_lxc, stream);
}

int cfc_ct_apply_v6(cfc_ctx *c, const cfc_hdr_v6 *in, const cfc_out *out,
                    int mode, uint16_t ep_lxc, void *stream)
{
    return ct_apply(c, 6, in, out, mode, ep_lxc, stream);
}

int cfc_ct_gc(cfc_ctx *c, int fd, const cfc_ct_gc_filter *filter, cfc_ct_gc_stats *stats,
              void *stream)
{
    if (!c || !filter)
        return -EINVAL;
    std::lock_guard<std::recursive_mutex> g(c->mu);
    if (c->device == CFC_DEVICE_NONE)
        return -ENODEV;
    (void)hipSetDevice(c->device);
    const int rc = ct_gc(c, fd, filter, stats, (hipStream_t)stream);
    if (!rc)
        (void)hipStreamSynchronize((hipStream_t)stream);
    return rc;
}

}  // extern "C"
