// Flattening of the host maps into the device layouts of layout.h.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "layout.h"
#include "maps.hpp"

namespace cfc {

struct PolLoc {
    uint32_t base = 0, mask = 0, present = 0;
};

// IPv4 ipcache layouts (cfc_set_option CFC_OPT_LPM4)
enum Lpm4Layout { LPM4_AUTO = 0, LPM4_DIR24_8 = 1, LPM4_TRIE = 2 };

struct BuildOpts {
    int lpm4 = LPM4_AUTO;
};

// IPv6 LPM (layout.h Lpm6), host side
struct Pfx6 {
    uint32_t w[4];   // host-order words, masked
    uint8_t plen;
    uint32_t label;
};
struct Lpm6Host {
    std::vector<L6Slot> slots;     // prefixes longer than /64
    std::vector<uint4> slots64;    // /1-/64: {w0, w1, label, len}
    std::vector<uint64_t> bloom;
    std::vector<uint32_t> lens;
    uint32_t def_label = 0;
    uint32_t n = 0;        // prefixes (incl. /0)
    uint32_t groups = 0;   // Bloom groups
    uint64_t bytes() const
    {
        return sizeof(L6Slot) * slots.size() + 16ull * slots64.size() + 8ull * bloom.size() +
               4ull * lens.size();
    }
};
// lpm6_find_slot's answer for a prefix in slots64: L6_S64 | its slot
constexpr int64_t L6_S64 = (int64_t)1 << 40;
void build_lpm6(const std::vector<Pfx6> &pfx, Lpm6Host *out);
// one ipcache entry (normalised key, value) as an IPv6 prefix; false when it
// is not one the IPv6 table holds on its own (prefix within the static part)
bool ipcache_v6_entry(const std::string &nk, const std::string &val, Pfx6 *p);
// the slot of prefix p in a built table, or -1
int64_t lpm6_find_slot(const Lpm6Host &t, const Pfx6 &p);
// host reference of the device lookup (unit tests): the label of the
// longest prefix containing w, def_label when none
uint32_t lpm6_lookup_host(const Lpm6Host &t, const uint32_t w[4]);

struct HostImage {
    // the CT tables' least slot counts (a device apply that outgrew the
    // table asked for more: cfc_api.cpp ct_apply_dev)
    uint64_t ct_min4 = 0, ct_min6 = 0;
    // IPv4 ipcache: compact multibit (l4c/l4l) or DIR-24-8 (tbl24/tbl8)
    std::vector<uint32_t> tbl24, tbl8, lbl_ovf;
    std::vector<uint32_t> l4d, l4c;    // l4d: 4 words per /16
    std::vector<uint64_t> l4l;
    int lpm4_layout = 0;           // LPM4_DIR24_8 / LPM4_TRIE, 0 = empty
    uint32_t n_prefix4 = 0;
    // prefilter
    std::vector<uint32_t> pf_tbl24, pf_tbl8;
    uint32_t n_pf_dyn = 0;
    std::vector<uint32_t> pf_fix;
    uint32_t pf_fix_mask = 0, pf_fix_zero = 0, n_pf_fix = 0;
    std::vector<uint32_t> pf_bloom;                 // words (pow2) or empty
    std::vector<uint32_t> pf6_bloom;                // over pf6_fix (all /128), or empty
    // endpoints
    std::vector<LxcSlot> lxc4;
    uint32_t lxc4_mask = 0, n_eps = 0;
    // policy
    std::vector<PolSlot> pol;
    std::vector<uint32_t> pol_bloom;
    std::unordered_map<int, PolLoc> pol_loc;       // lxc_id -> table
    // IPv6
    Lpm6Host ipc6, pf6_fix, pf6_dyn;
    std::vector<Lxc6Slot> lxc6;
    uint32_t lxc6_mask = 0, n_eps6 = 0;
    // per LXC_ID its IPv4 / IPv6 address (raw), endpoints with one
    std::map<uint16_t, uint32_t> nat4;
    std::map<uint16_t, uint4> nat6;
    std::vector<std::pair<Map *, std::string>> ctr_owner;  // ctr -> entry
    // conntrack (layout.h): every CT map in one table per family
    std::vector<Ct4Slot> ct4;
    std::vector<Ct6Slot> ct6;
    std::vector<CtTimer> ct4_tm, ct6_tm;     // parallel to ct4 / ct6
    uint32_t ct4_mask = 0, ct4_probe = 0, ct6_mask = 0, ct6_probe = 0;
    uint32_t n_ct4 = 0, n_ct6 = 0;           // entries placed
    uint32_t n_nat46 = 0;                    // IPv4 entries with nat46
    std::vector<uint8_t> ct_local;           // lxc_id -> has local CT maps
    // load balancing (layout.h): service slots, reverse NAT, and per CT4
    // slot the entry's LB state (built with GROUP_CT when lb_ct is set)
    std::vector<uint4> lb4;
    uint32_t lb4_mask = 0, n_lb4 = 0;
    std::vector<uint2> rnat4;
    std::vector<uint4> ct4_lb;
    bool lb_ct = false;                      // ct4_lb wanted
    std::vector<uint4> lb6;                  // IPv6: 3 per slot
    uint32_t lb6_mask = 0, n_lb6 = 0;
    std::vector<uint4> rnat6;                // 2 per index
    std::vector<uint4> ct6_lb;
    bool lb6_ct = false;                     // ct6_lb wanted
    uint64_t device_bytes() const;
};

// the CT map a slot's entry lives in: (family 4/6, owner word, any) key
uint64_t ct_map_key(int family, uint32_t owner, int any);
// the device slot of a CT map entry; false when no lookup reaches it
bool ct_slot_of(const Map *m, const std::string &key, Ct4Slot *s4, Ct6Slot *s6);
// the report state the kernels read (CtTimer) of a struct ct_entry value
CtTimer ct_timer_of(const std::string &val);
// the LB state a CT4 slot carries (ct4_lb) of a struct ct_entry value
uint4 ct_lb_of(const std::string &val);

// Table groups an epoch is built from; a commit rebuilds only the groups
// whose maps changed (the others' device buffers carry over).
enum : unsigned {
    GROUP_IPCACHE4 = 1,   // ipcache, IPv4 LPM (+ lbl_ovf)
    GROUP_PREFILTER = 2,  // XDP prefilter, both families
    GROUP_ENDPOINTS = 4,  // cilium_lxc + every policymap (+ counter layout)
    GROUP_CT = 8,         // every CT map
    GROUP_IPCACHE6 = 16,  // ipcache, IPv6 LPM
    GROUP_LB = 32,        // cilium_lb{4,6}_services, cilium_lb{4,6}_reverse_nat
    GROUP_ALL = 63,
};
// maps: every map of the context; groups: which parts of img to build
// (ct_local, which only depends on which CT maps exist, always is).
void build_image(const std::vector<Map *> &maps, const BuildOpts &opt,
                 HostImage *img, unsigned groups = GROUP_ALL);

// exposed for host-side unit tests of the LPM builders
struct Pfx4 {
    uint32_t addr;   // host byte order
    uint8_t plen;
    uint32_t leaf;   // encoded LPM leaf
};
void build_dir24_8(std::vector<Pfx4> pfx, std::vector<uint32_t> *tbl24,
                   std::vector<uint32_t> *tbl8);
// compact multibit layout (layout.h); labels too wide for a list entry get
// lbl_ovf entries.  False when an offset would not fit its 24 bits.
bool build_l4trie(std::vector<Pfx4> pfx, std::vector<uint32_t> *ovf,
                  std::vector<uint32_t> *l4d, std::vector<uint32_t> *l4c,
                  std::vector<uint64_t> *l4l);

}  // namespace cfc
