// Device table layouts shared by the host flattener (flatten.cpp) and the
// HIP kernels (classify.hip).  Everything here is plain data: the kernels get
// one DevTables by value per launch.
//
// Every probe is ONE 16-byte load per lane (global_load_dwordx4): on gfx950
// the per-CU address unit (TA) spends a cycle per distinct cache line a wave
// instruction touches, so a random-access kernel is bound by the number of
// divergent load instructions, not by bytes.  Tables are therefore sized for
// short probe sequences (load factor <= 25%) rather than for compactness —
// they are small next to 288 GB of HBM3E and stay L2/Infinity-Cache resident.
//
// HBM layout of one epoch (read-only while classifying):
//   lpm4      IPv4 ipcache: the compact multibit layout (l4d directory +
//             l4c chunks + l4l prefix lists, L2-resident), or DIR-24-8: tbl24 (2^24 x u32 =
//             64 MiB, Infinity Cache) + 256-entry tbl8 groups for /25-/32
//   pf4_dyn   same structure for the prefilter LPM deny-list (when used)
//   pf4_fix   exact /32 deny set: 16-B buckets of 4 addresses (0 = empty)
//   lxc4      local endpoints by IPv4: 16-B slots with the endpoint record
//   pol       every endpoint's policy table: 16-B slots
//             {key u64, proxy u16, pad, counter index u32}
//   lbl_ovf   identities >= 2^30 (rare) referenced from LPM leaves
//   pf_bloom  blocked Bloom filter over pf4_fix   } copied into LDS by
//   pol_bloom blocked Bloom filter over all pol   } every workgroup
// Counters (read-write): u64 packets/bytes per policy entry + metrics.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace cfc {

// ---- LPM (DIR-24-8) entry encoding -----------------------------------------
// 0                      no match (also label 0: the reference treats a
//                        matched sec_label of 0 exactly like a miss:
//                        bpf_netdev.c:377-379, bpf_lxc.c:521)
// bit31 set              pointer to tbl8 group (bits 0..30 = group index)
// bit30 set (bit31 clr)  indirect label: lbl_ovf[bits 0..29]
// otherwise              the label itself (< 2^30)
constexpr uint32_t LPM_GROUP = 0x80000000u;
constexpr uint32_t LPM_INDIRECT = 0x40000000u;
constexpr uint32_t LPM_PAYLOAD = 0x3FFFFFFFu;

constexpr uint32_t EMPTY = 0xFFFFFFFFu;

// ---- IPv4 LPM, compact multibit layout (default) --------------------------
// DIR-24-8 costs ~1.3 Infinity-Cache accesses per lookup (tbl24 is 64 MiB).
// The compact layout keeps the whole ipcache in about 2-3 MiB, resident in
// every XCD's 4 MiB L2, and resolves most lookups with ONE 16-byte load:
//   l4d (16 B x 65536) the /16 directory.  x = the node word (below); y, z, w
//                    hold up to two of the node's prefixes longer than /16
//                    inline (48-bit entries, below), its longest two, which
//                    a lookup checks before following x: a /16 with at most
//                    two longer prefixes is a single load (x is then the
//                    covering leaf), a longer list continues in l4l
//   l4c (u32 nodes)  256-entry chunks for the next 8 bits.  A node word is
//      bit31 clear              a leaf (LPM leaf encoding above; 0 = none)
//      bit31 set, cnt == 0      a chunk at l4c[off] for the next 8 bits
//      bit31 set, cnt  > 0      a list of cnt prefixes at l4l[off]
//                    (off = bits 0-23, cnt = bits 24-30)
//   l4l (u64)        per-node prefix lists, longest first, ending with the
//                    node's own covering prefix (which always matches), padded
//                    to an even length so that one 16-byte load reads two:
//                    lo = prefix address (host order, masked),
//                    hi = (len & 31) << 27 | leaf27 (LL_INDIRECT -> lbl_ovf)
// A node lists its prefixes while it has fewer than L4_LIST_MAX, and is
// split into a chunk beyond (a split /16 has no inline entries).
// Inline entry (48 bits; e0 = y | (z & 0xFFFF) << 32, e1 = z >> 16 | w << 16):
//   bits 0-15 the prefix's address bits 0-15 (masked), bits 16-20 len - 16
//   (1..16: never 0, so a zero entry is empty), bits 21-47 leaf27.
constexpr uint32_t L4_PTR = 0x80000000u;
constexpr uint32_t L4_OFF = 0xFFFFFFu;
constexpr uint32_t L4_LIST_MAX = 16;
constexpr uint32_t L4_INLINE = 2;
constexpr uint32_t LL_INDIRECT = 1u << 26;
constexpr uint32_t LL_PAYLOAD = (1u << 26) - 1;
__host__ __device__ inline bool l4_match(uint32_t a, uint32_t addr, uint32_t hi)
{
    const uint32_t len = hi >> 27;   // 0 stands for 32
    const uint32_t m = len ? 0xFFFFFFFFu << (32 - len) : 0xFFFFFFFFu;
    return (a & m) == addr;
}
__host__ __device__ inline uint64_t l4_inline_entry(uint32_t addr, uint32_t len,
                                                    uint32_t leaf27)
{
    return (uint64_t)(addr & 0xFFFFu) | (uint64_t)(len - 16) << 16 |
           (uint64_t)leaf27 << 21;
}
// does inline entry e (nonzero) hold a prefix containing address a (whose
// top 16 bits are the directory index)
__host__ __device__ inline bool l4_inline_match(uint32_t a, uint32_t e_lo32)
{
    const uint32_t l = (e_lo32 >> 16) & 31;            // len - 16, 0 = empty
    const uint32_t m = (0xFFFFu << (16 - l)) & 0xFFFFu;
    return l != 0 && ((a ^ e_lo32) & m) == 0;
}

// ---- policy: open addressing, linear probing over 16-byte slots -------------
// The datapath only ever looks up keys whose pad bits (byte 7, bits 1-7) are
// zero (policy.h:53-59), so an all-ones key marks a free slot and stored keys
// with pad bits set — which no lookup can match — are left out of the table.
constexpr uint64_t POL_EMPTY = ~0ull;
struct alignas(16) PolSlot {
    uint64_t key;                  // struct policy_key raw bytes (LE load)
    uint16_t proxy_port;           // policy_entry.proxy_port (be16 raw)
    uint16_t pad;
    uint32_t ctr;                  // counter index
};

// ---- endpoints (cilium_lxc), IPv4 keys: 16-byte slots, linear probing -------
// info: bits 0-15 lxc_id, then flags
constexpr uint32_t LXC_HOST = 1u << 16;       // ENDPOINT_F_HOST
constexpr uint32_t LXC_HAS_POLICY = 1u << 17; // an endpoint program exists
constexpr uint32_t LXC_IFINDEX = 1u << 18;    // ifindex != 0 (redirect)
constexpr uint32_t LXC_CT_LOCAL = 1u << 19;   // has its own CT maps (else global)
constexpr uint32_t LXC_HAS6 = 1u << 20;       // (IPv4 slots) the endpoint has an IPv6
                                              // address: NAT46 can deliver to it
constexpr uint32_t LXC_VALID = 1u << 31;      // 0 = free slot
struct alignas(16) LxcSlot {
    uint32_t addr;                 // be32 raw
    uint32_t pol_base;             // first slot of its policy table
    uint32_t pol_mask;             // slots - 1 (power of two)
    uint32_t info;
};

// ---- prefilter /32 set: 16-byte buckets of 4 addresses, 0 = empty -----------
constexpr int PF_SLOTS = 4;

// Hashes of the raw keys: 32-bit multiply / xor-shift mixes (a 64-bit
// multiply costs several VALU instructions on the GPU).  (A mixer on 24-bit
// multiplies, full-rate on gfx950, loses 8 bits of every intermediate:
// measured 8% key collisions on CT tuples, so the tables keep fmix32.)
__host__ __device__ inline uint32_t fmix32(uint32_t h)
{
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}
__host__ __device__ inline uint32_t hash32(uint32_t k, uint32_t mask)
{
    uint64_t x = (uint64_t)k * 0x9E3779B97F4A7C15ull;
    return (uint32_t)(x >> 32) & mask;
}
// struct policy_key as a u64 (lo = identity, hi = dport | nexthdr << 16 |
// egress << 24), folded to 32 bits and mixed once: the table slot and the
// Bloom filter word both derive from that one mix
__host__ __device__ inline uint32_t pol_key_pre(uint32_t lo, uint32_t hi)
{
    return fmix32(lo * 0x9E3779B1u ^ hi);
}
__host__ __device__ inline uint32_t pol_slot(uint32_t pre, uint32_t mask)
{
    return pre & mask;
}

// ---- blocked Bloom filters (LDS-resident while classifying) ----------------
// One 32-bit word per key, three bits set in it: a query is one ds_read_b32.
// They only ever answer "absent" or "maybe"; a "maybe" is resolved by the
// exact table, so a false positive costs one extra probe and never a wrong
// verdict.  The word is h & (words - 1) (at most 13 bits), the bits come
// from bits 17-31 of h.
__host__ __device__ inline uint32_t bloom_bits(uint32_t h)
{
    return (1u << ((h >> 17) & 31)) | (1u << ((h >> 22) & 31)) | (1u << (h >> 27));
}
// policy keys are filtered per endpoint table (its first slot): the word
// index is rotated by the table, the bits are the key's own
__host__ __device__ inline uint32_t pol_bloom_salt(uint32_t base)
{
    return (base + 1u) * 0x9E3779B1u;
}
__host__ __device__ inline uint32_t pol_bloom_hash(uint32_t salt, uint32_t pre)
{
    return pre ^ (salt >> 16) ^ (pre >> 19);
}
__host__ __device__ inline uint32_t pf_bloom_hash(uint32_t addr)
{
    return fmix32(addr ^ 0x5bd1e995u);
}
// (sized so that two 1024-thread workgroups fit one CU's 160 KiB of LDS)
constexpr uint32_t POL_BLOOM_MAX_WORDS = 8192;    // 32 KiB
constexpr uint32_t PF_BLOOM_MAX_WORDS = 8192;     // 32 KiB
constexpr uint32_t LXC_LDS_MAX_SLOTS = 512;       // 8 KiB of endpoint slots

// ---- IPv6 LPM: one hash table over every (prefix, length), probed longest
// length first, screened by a blocked Bloom filter.
// A 1M-prefix ipcache cannot be cache-resident whatever its layout (>= 16 MB
// of keys), so the layout minimises Infinity-Cache accesses: the slots are
// touched about once per lookup and everything before that is L2-resident.
//   slots   32 bytes: masked address as host-order words (w[0] = bits 0-31),
//           label, length (0 = free slot); linear probing, load <= 50%;
//           prefixes of at most /64 in slots64 (16 bytes: w[0], w[1], label,
//           length), probed with the same hash
//   lens    the lengths present (> 0), longest first:
//           len | sel << 8 | L6_GROUP_FIRST; consecutive lengths form a
//           group sharing one Bloom word, chosen by the address masked to
//           the group's shortest length `sel` (so one 8-byte load screens
//           the whole group), the bits by the key itself
//   bloom   u64 words; key (m, len) sets bits (h >> 20) & 63 and h >> 26,
//           h = l6_hash(m, len); the slot index is h & mask
// A /0 prefix is def_label (no probe).  The builder closes a group when the
// addresses masked to the next length would pile more than L6_GROUP_MAX keys
// into one word.
constexpr uint32_t L6_GROUP_FIRST = 1u << 16;
constexpr uint32_t L6_GROUP_MAX = 4;
struct alignas(16) L6Slot {
    uint32_t w[4];
    uint32_t label;
    uint32_t len;
    uint32_t pad[2];
};
// Prefixes of at most 64 bits (the /32-/64 mass of an ipcache) sit in a
// table of their own with 16-byte slots {w0, w1, label, len} (len 0: free;
// their masked address has w2 = w3 = 0): a probe is one load.  Longer ones
// keep the 32-byte slots (two loads: key, then {label, len}).
struct Lpm6 {
    const L6Slot *slots;           // prefixes longer than /64 (null: none)
    const uint4 *slots64;          // prefixes of /1-/64 (null: none)
    const uint64_t *bloom;
    const uint32_t *lens;
    uint32_t mask;                 // slots - 1
    uint32_t mask64;               // slots64 - 1
    uint32_t bloom_mask;           // words - 1
    uint32_t nlen;                 // entries of lens
    uint32_t def_label;            // label of ::/0 (0: none)
};
__host__ __device__ inline uint32_t l6_word_mask(uint32_t len, int i)
{
    const int b = (int)len - 32 * i;   // bits of word i inside the prefix
    return b >= 32 ? 0xFFFFFFFFu : b <= 0 ? 0u : 0xFFFFFFFFu << (32 - b);
}
__host__ __device__ inline uint32_t l6_hash(uint32_t w0, uint32_t w1, uint32_t w2,
                                            uint32_t w3, uint32_t tag)
{
    return fmix32(w0 * 0x9E3779B1u + w1 * 0x85EBCA77u + w2 * 0xC2B2AE3Du +
                  w3 * 0x27D4EB2Fu + tag * 0x165667B1u);
}
// Bloom word of a group with shortest length sel / key bits of (m, len)
__host__ __device__ inline uint32_t l6_group_hash(const uint32_t w[4], uint32_t sel)
{
    return l6_hash(w[0] & l6_word_mask(sel, 0), w[1] & l6_word_mask(sel, 1),
                   w[2] & l6_word_mask(sel, 2), w[3] & l6_word_mask(sel, 3),
                   sel | 0x100u);
}
__host__ __device__ inline uint64_t l6_bloom_bits(uint32_t h)
{
    return (1ull << ((h >> 20) & 63)) | (1ull << (h >> 26));
}
// the IPv6 prefilter's exact /128 set (v6_fix, bpf_xdp.c:132-156): its
// addresses (host-order words) in an LDS Bloom filter of the same kind, so
// that a header whose source is not in the set costs no global load
__host__ __device__ inline uint32_t pf6_bloom_hash(uint32_t w0, uint32_t w1, uint32_t w2,
                                                   uint32_t w3)
{
    return fmix32(l6_hash(w0, w1, w2, w3, 0x300u) ^ 0x5bd1e995u);
}

// ---- IPv6 endpoints: 32-byte slots {raw address words, pol_base, pol_mask,
// info (as LxcSlot.info), 0}, linear probing on l6_hash(raw, L6_LXC_TAG)
constexpr uint32_t L6_LXC_TAG = 0x200u;
struct alignas(16) Lxc6Slot {
    uint32_t a[4];                 // network-order bytes, loaded LE
    uint32_t pol_base, pol_mask, info, pad;
};
constexpr uint32_t LXC6_LDS_MAX_SLOTS = 256;      // 8 KiB

// ---- conntrack (cilium_ct{4,_any4,6,_any6}_{global,<lxc_id>}) ---------------
// One open-addressed table per family holds every CT map: a slot is the
// struct ipv{4,6}_ct_tuple plus a word naming the map.  TCP maps are only
// ever probed with nexthdr 6 and ANY maps with the others
// (get_ct_map4/6, bpf_lxc.c:91-107), so entries a lookup can never reach
// (an ICMP "related" entry in a TCP map, conntrack.h:648-660) are left out
// and the map kind is implied by nexthdr.  Linear probing, load <= 1/2,
// w == 0 marks a free slot; ct_probe bounds the longest probe sequence.
//   v4 slot (16 B): x daddr, y saddr, z dport | sport << 16 (tuple bytes
//                   8-11), w = ct_word(nexthdr, flags, owner)
//   v6 slot (48 B): daddr[4], saddr[4], {z, w, 0, 0}
// owner: 0 = the global maps, else 1 << 11 | lxc_id << 16 (local maps).
// Per-slot accounting (CONNTRACK_ACCOUNTING, conntrack.h:247-257) lives in
// the slot's CtState line (acct[dir][packets, bytes], dir: CT_EGRESS 0 /
// CT_INGRESS 1).
__host__ __device__ inline uint32_t ct_word(uint32_t nexthdr, uint32_t flags,
                                            uint32_t owner)
{
    return nexthdr | (flags & 7u) << 8 | owner;
}
// a deleted slot (cfc_commit patches deletes in place): nonzero, so probe
// sequences run through it, and bits 12-15 are never set in a real w
constexpr uint32_t CT_TOMBSTONE = 0xF000u;
__host__ __device__ inline uint32_t ct_owner_word(uint32_t lxc, bool local)
{
    return local ? (1u << 11 | lxc << 16) : 0u;
}
__host__ __device__ inline uint32_t ct_hash4(uint32_t x, uint32_t y, uint32_t z,
                                             uint32_t w)
{
    uint32_t h = fmix32(x ^ 0x9e3779b9u);
    h = fmix32(h ^ y);
    h = fmix32(h ^ z);
    return fmix32(h ^ w);
}
__host__ __device__ inline uint32_t ct_hash6(const uint32_t d[4], const uint32_t s[4],
                                             uint32_t z, uint32_t w)
{
    uint32_t h = ct_hash4(d[0], d[1], d[2], d[3]);
    h = fmix32(h ^ s[0]);
    h = fmix32(h ^ s[1]);
    h = fmix32(h ^ s[2]);
    h = fmix32(h ^ s[3]);
    return ct_hash4(h, z, w, 0x7f4a7c15u);
}
// The home slot of a CT key (the placement hash; ct_hash4 / ct_hash6 stay
// the plain mixers the fingerprints use).  It is symmetric in the tuple's
// direction: the two addresses and the two ports are taken as unordered
// pairs and the direction flag (TUPLE_F_IN, bit 8 of w) is left out, so a
// packet's two lookups — k1 = (daddr, saddr, ports as loaded, flags) for
// REPLY / RELATED and k2 = (saddr, daddr, ports swapped, flags ^ IN) for
// ESTABLISHED (__ct_lookup via ct_lookup4/6, conntrack.h:467-590) — start
// their probe at the same slot, and one walk from it answers both.
__host__ __device__ inline uint32_t ct_home4(uint32_t x, uint32_t y, uint32_t z, uint32_t w)
{
    const uint32_t lo = x < y ? x : y, hi = x < y ? y : x;
    const uint32_t pa = z & 0xFFFFu, pb = z >> 16;
    const uint32_t zs = (pa < pb ? pa : pb) | (pa < pb ? pb : pa) << 16;
    return ct_hash4(lo, hi, zs, w & ~0x100u);
}
__host__ __device__ inline uint32_t ct_home6(const uint32_t d[4], const uint32_t s[4],
                                             uint32_t z, uint32_t w)
{
    const uint32_t hd = ct_hash4(d[0], d[1], d[2], d[3]), hs = ct_hash4(s[0], s[1], s[2], s[3]);
    const uint32_t pa = z & 0xFFFFu, pb = z >> 16;
    const uint32_t zs = (pa < pb ? pa : pb) | (pa < pb ? pb : pa) << 16;
    return ct_hash4(hd < hs ? hd : hs, hd < hs ? hs : hd, zs, (w & ~0x100u) ^ 0x7f4a7c15u);
}
struct alignas(16) Ct4Slot {
    uint32_t x, y, z, w;
};
// The mutable state of a CT slot's entry (struct ct_entry, common.h:380-406):
// what decides whether a hit is traced (__ct_update_timeout,
// conntrack.h:125-185) and what the device CT apply (ctapply.hip) updates:
// last_{rx,tx}_report, rx/tx_flags_seen, the rx/tx_closing and seen_non_syn
// bits, lifetime.  The packet/byte counts sit beside it in CtState.
struct alignas(16) CtTimer {
    uint32_t last_rx, last_tx;
    uint32_t flags;      // rx_flags_seen | tx_flags_seen << 8 | closing << 16
                         // | seen_non_syn << 18 | nat46 << 19
    uint32_t lifetime;
};
constexpr uint32_t CTT_NON_SYN = 1u << 18;
constexpr uint32_t CTT_NAT46 = 1u << 19;   // ct_entry.nat46 (conntrack.h:241-244, 714-716)
// per-slot state of the device CT apply (ctapply.hip): src_sec_id and
// rev_nat_index of an entry the device created, and what changed since the
// host last synchronised (CTI_*, bits 16-18 of y)
struct CtInfo {
    uint32_t sec;
    uint32_t y;          // rev_nat_index | dirty << 16
};
constexpr uint32_t CTI_UPDATED = 1u << 16, CTI_CREATED = 2u << 16, CTI_DELETED = 4u << 16;
// the slot was claimed by a device insert since the host's last sync: its
// key is new to the table (CTI_CREATED alone may be an overwrite, e.g. a
// related ICMP entry written again, of a key the host holds)
constexpr uint32_t CTI_FRESH = 8u << 16;
// a slot being filled by a device insert (never matched, never free)
constexpr uint32_t CT_CLAIM = 0xE000u;
struct alignas(16) Ct6Slot {
    uint32_t d[4], s[4], z, w, pad[2];
};
// Everything a CT slot's entry holds besides its key, in ONE 64-byte line
// (struct ct_entry, common.h:380-406, as __ct_lookup / ct_create4/6 touch
// it, conntrack.h:221-285, 615-772): the report state, the
// CONNTRACK_ACCOUNTING counters and the device apply's per-slot record.  A
// hit's fold, the finish, the GC and the accounting reduce each touch one
// line per slot here (three to four separate arrays before).  The keys stay
// a dense array of their own (Ct4Slot / Ct6Slot): the lookups probe only
// keys, and a dense key array keeps a Zipf batch's hot keys in L2.
//   tm     CtTimer
//   acct   [dir][packets, bytes], dir CT_EGRESS 0 (tx) / CT_INGRESS 1 (rx)
//   info   CtInfo
// One array for both families: IPv4 slots, then IPv6 slots from
// DevTables.ct6_acct_base (the accounting key slot * 2 + dir indexes it).
struct alignas(64) CtState {
    CtTimer tm;
    uint64_t acct[4];
    CtInfo info;
    uint32_t pad[2];
};
static_assert(sizeof(CtState) == 64, "one line per CT slot");

// ---- service load balancing (cilium_lb4_services, cilium_lb4_reverse_nat)
// Services: open-addressed 32-byte slots keyed by struct lb4_key {address,
// dport, slave} (load <= 1/2, linear probing, used == 0 marks a free slot):
//   {addr, dport | slave << 16, target, port | count << 16,
//    rev_nat_index | weight << 16, used, 0, 0}
// Reverse NAT: direct-indexed by rev_nat_index, {address, port | 1 << 16}
// (bit 16: present).  Per CT4 slot (ct4_lb, with a load balancer): the
// entry's {rev_nat_index | lb_loopback << 16, slave, 0, 0}.
__host__ __device__ inline uint32_t lb4_hash(uint32_t addr, uint32_t ps)
{
    return fmix32(fmix32(addr ^ 0x85ebca6bu) ^ ps);
}
constexpr uint32_t IPV4_LOOPBACK = 0x1FFFF50Au;   // node_config.h:45 (be32 raw)
// IPv6 (cilium_lb6_services, cilium_lb6_reverse_nat): 48-byte service slots
// keyed by struct lb6_key {address[16], dport, slave}, load <= 1/2:
//   {address words}, {dport | slave << 16, port | count << 16,
//    rev_nat_index | weight << 16, used}, {target words}
// Reverse NAT direct-indexed: {address words}, {port | 1 << 16, 0, 0, 0}.
// Per CT6 slot (ct6_lb, with a load balancer): {rev_nat_index, slave, 0, 0}.
__host__ __device__ inline uint32_t lb6_hash(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3,
                                             uint32_t ps)
{
    return l6_hash(a0, a1, a2, a3, ps ^ 0x6b43a9b5u);
}

struct DevTables {
    const uint4 *l4d;              // compact IPv4 LPM /16 directory, or null
    const uint32_t *l4c;           // its chunks
    const uint64_t *l4l;           // its prefix lists
    const uint32_t *tbl24;         // DIR-24-8 layout (null: none or compact)
    const uint32_t *tbl8;
    const uint32_t *lbl_ovf;
    const uint32_t *pf_tbl24;      // null when the dyn prefilter is empty
    const uint32_t *pf_tbl8;
    const uint32_t *pf_fix;        // buckets of 4 u32, null when empty
    const LxcSlot *lxc4;           // null when no IPv4 endpoints
    const PolSlot *pol;
    const uint32_t *pf_bloom;      // Bloom filter over pf_fix, or null
    const uint32_t *pol_bloom;     // Bloom filter over every policy key
    uint32_t pf_fix_mask;          // buckets - 1
    uint32_t pf_fix_zero;          // 0.0.0.0/32 is in the deny set
    uint32_t lxc4_mask;            // slots - 1
    uint32_t n_ctr;                // policy entries (counter slots)
    uint32_t pf_bloom_words;       // power of two, 0 = no filter
    uint32_t pol_bloom_words;      // power of two, 0 = no filter
    uint32_t lxc4_lds;             // 1: the endpoint table is copied to LDS
    // IPv6
    Lpm6 ipc6;                     // ipcache
    Lpm6 pf6_fix;                  // prefilter exact /128 set (one length)
    Lpm6 pf6_dyn;                  // prefilter LPM deny list
    const uint32_t *pf6_bloom;     // Bloom filter over pf6_fix (all /128), or null
    uint32_t pf6_bloom_words;      // power of two, 0 = no filter
    const Lxc6Slot *lxc6;          // null when no IPv6 endpoints
    uint32_t lxc6_mask;
    uint32_t lxc6_lds;             // 1: copied to LDS
    // conntrack (null: every map empty -> every lookup is CT_NEW)
    const Ct4Slot *ct4;
    const Ct6Slot *ct6;
    CtState *ct_st;                // per slot, v4 then v6 (from ct6_acct_base)
    // per slot (as ct_acct) the plain-hit summary of the launch's hits
    // (ctapply.hip k_cta_finish's bits: flags per direction, hit per
    // direction, a TCP hit without the close bit), written by the
    // accounting reduce (classify.hip k_acc_reduce) for the device CT apply
    // that follows the launch; cleared by that apply.  Null: not kept.
    uint32_t *ct_sum;
    uint32_t ct4_mask, ct4_probe;
    uint32_t ct6_mask, ct6_probe;
    uint32_t ct6_acct_base;        // first v6 slot in ct_st
    // the launch: bpf_ktime_get_sec() (cfc_set_clock), HOST_IFINDEX
    uint32_t now;
    uint32_t host_ifindex;
    // LXC_NAT46 (lxc_config.h:28, nat46.h:30-32): 1 when an IPv4 entry may
    // carry nat46 and an endpoint has an IPv6 address — the IPv4 ingress
    // path then checks its CT hits for it (bpf_lxc.c:939-944)
    uint32_t nat46;
    // per-identity counters: bit r set = identities [r * ID_RANGE,
    // (r + 1) * ID_RANGE) have a histogram range (classify.hpp)
    uint32_t id_cover;
    // node_config.h constants (cfc_set_node_config), filled in per launch
    uint32_t v4_cluster_range;     // IPV4_CLUSTER_RANGE, be32 raw
    uint32_t v4_cluster_mask;      // IPV4_CLUSTER_MASK, be32 raw
    uint32_t router6[4];           // ROUTER_IP as host-order words
    // load balancing (null: no service, no reverse NAT)
    const uint4 *lb4;              // 2 uint4 per service slot
    uint32_t lb4_mask;             // slots - 1
    const uint2 *rnat4;            // [65536] or null
    const uint4 *ct4_lb;           // per CT4 slot, or null
    const uint4 *lb6;              // 3 uint4 per IPv6 service slot, or null
    uint32_t lb6_mask;
    const uint4 *rnat6;            // [65536][2] or null
    const uint4 *ct6_lb;           // per CT6 slot, or null
};

// metrics block: [reason 256][dir 4][count, bytes]
// (policy-entry counters live in their own block: [n_ctr][packets, bytes])
constexpr int METRIC_REASONS = 256;
constexpr int METRIC_DIRS = 4;
constexpr int METRIC_U64 = METRIC_REASONS * METRIC_DIRS * 2;

}  // namespace cfc
