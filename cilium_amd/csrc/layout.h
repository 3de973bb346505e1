// Device table layouts shared by the host flattener (flatten.cpp) and the
// HIP kernels (classify.hip).  Everything here is plain data: the kernels get
// one DevTables by value per launch.
//
// HBM layout of one epoch (all read-only while classifying):
//   lpm4      DIR-24-8 IPv4 ipcache: tbl24 (2^24 x u32 = 64 MiB, sits in the
//             256 MiB Infinity Cache) + 256-entry tbl8 groups for /25-/32.
//   pf4_dyn   same structure for the prefilter LPM deny-list (only if used)
//   pf4_fix   exact /32 deny set: 64-B buckets of 15 addresses + count
//   lxc4      local endpoints by IPv4: 64-B buckets of 8 {addr, ep index}
//   eps       endpoint records (32 B)
//   pol       all endpoints' policy hash tables: 64-B buckets of 4 slots
//             {key u64, proxy u16, pad, counter index u32}
//   lbl_ovf   identities >= 2^30 (rare) referenced indirectly from LPM leaves
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

// ---- 64-byte bucket hash tables --------------------------------------------
constexpr uint32_t EMPTY = 0xFFFFFFFFu;

struct alignas(16) PolSlot {       // 16 B; 4 per 64-B bucket
    uint64_t key;                  // struct policy_key raw bytes (LE load)
    uint16_t proxy_port;           // policy_entry.proxy_port (be16 raw)
    uint16_t pad;
    uint32_t ctr;                  // counter index, EMPTY = free slot
};
constexpr int POL_SLOTS = 4;

struct Lxc4Slot {                  // 8 B; 8 per bucket
    uint32_t addr;                 // be32 raw
    uint32_t ep;                   // index into eps, EMPTY = free slot
};
constexpr int LXC_SLOTS = 8;

constexpr int PF_SLOTS = 15;       // pf4_fix bucket: u32 addr[15] + u32 count

struct alignas(16) EpRec {         // 32 B
    uint32_t lxc_id;
    uint32_t ifindex;
    uint32_t flags;                // ENDPOINT_F_HOST = 1
    uint32_t seclabel;             // SECLABEL of the endpoint program
    uint32_t pol_base;             // first bucket of its policy table
    uint32_t pol_mask;             // buckets - 1 (power of two), 0 = empty table
    uint32_t has_policy;
    uint32_t pad;
};

// Hashes: multiplicative (Fibonacci) hashing of the raw key, top bits.
__host__ __device__ inline uint32_t hash64(uint64_t k, uint32_t mask)
{
    k ^= k >> 29;
    k *= 0xbf58476d1ce4e5b9ull;
    k ^= k >> 32;
    return (uint32_t)k & mask;
}
__host__ __device__ inline uint32_t hash32(uint32_t k, uint32_t mask)
{
    uint64_t x = (uint64_t)k * 0x9E3779B97F4A7C15ull;
    return (uint32_t)(x >> 32) & mask;
}

struct DevTables {
    const uint32_t *tbl24;         // may be null when no v4 ipcache prefixes
    const uint32_t *tbl8;
    const uint32_t *lbl_ovf;
    uint32_t lpm4_default;         // tbl24 == null: value of a /0 prefix (or 0)
    const uint32_t *pf_tbl24;      // null when the dyn prefilter is empty
    const uint32_t *pf_tbl8;
    const uint32_t *pf_fix;        // buckets of 16 u32, null when empty
    uint32_t pf_fix_mask;
    uint32_t pf_dyn_default;       // pf_tbl24 == null: 1 if a /0 deny exists
    const Lxc4Slot *lxc4;          // buckets of LXC_SLOTS slots
    uint32_t lxc4_mask;
    uint32_t n_eps;
    const EpRec *eps;
    const PolSlot *pol;            // buckets of POL_SLOTS slots
    uint32_t n_ctr;                // policy entries (counter slots)
    uint32_t pad;
};

// metrics block: [reason 256][dir 4][count, bytes]
constexpr int METRIC_REASONS = 256;
constexpr int METRIC_DIRS = 4;
constexpr int METRIC_U64 = METRIC_REASONS * METRIC_DIRS * 2;

}  // namespace cfc
