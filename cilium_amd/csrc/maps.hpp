// Host mirror of the BPF maps behind the C ABI.
//
// Semantics follow the kernel map types the reference uses through pkg/bpf
// (pkg/bpf/bpf.go:108-252): HASH (kernel/bpf/hashtab.c: -E2BIG when full,
// BPF_NOEXIST/-EEXIST, BPF_EXIST/-ENOENT), LRU_HASH (evicts instead of
// failing), PERCPU_HASH (one CPU slot here), LPM_TRIE (kernel/bpf/lpm_trie.c:
// key = u32 prefixlen + data, -ENOSPC when full, lookups are longest-prefix
// matches bounded by the key's prefixlen, data bits past prefixlen ignored).
#pragma once
#include <cstdint>
#include <map>
#include <string>

namespace cfc {

enum MapType : uint32_t {
    MT_HASH = 1,
    MT_PERCPU_HASH = 5,
    MT_LRU_HASH = 9,
    MT_LPM_TRIE = 11,
};

enum Role {
    ROLE_NONE = 0,
    ROLE_IPCACHE,   // cilium_ipcache
    ROLE_LXC,       // cilium_lxc
    ROLE_POLICY,    // cilium_policy_<lxc_id>
    ROLE_METRICS,   // cilium_metrics
    ROLE_PF4_FIX,   // cilium_cidr_v4_fix
    ROLE_PF4_DYN,   // cilium_cidr_v4_dyn
    ROLE_PF6_FIX,   // cilium_cidr_v6_fix
    ROLE_PF6_DYN,   // cilium_cidr_v6_dyn
    ROLE_CT4,       // cilium_ct4_* / cilium_ct_any4_* (global or <lxc_id>)
    ROLE_CT6,       // cilium_ct6_* / cilium_ct_any6_*
    ROLE_LB4_SVC,   // cilium_lb4_services
    ROLE_LB4_RNAT,  // cilium_lb4_reverse_nat
    ROLE_LB6_SVC,   // cilium_lb6_services
    ROLE_LB6_RNAT,  // cilium_lb6_reverse_nat
};

enum : int { TOUCH_VALUE = 1, TOUCH_INSERT = 2, TOUCH_ERASE = 4 };

struct Map {
    std::string name;
    Role role = ROLE_NONE;
    int policy_lxc = -1;   // ROLE_POLICY, ROLE_CT*: lxc_id (-1: global CT)
    int ct_any = 0;        // ROLE_CT*: 1 = the ANY map, 0 = the TCP map
    uint32_t type = 0, ksz = 0, vsz = 0, max_entries = 0, flags = 0;
    uint64_t gen = 0;   // bumped on every mutation
    // structural mutations (insert, delete, eviction): ipcache keys by
    // family (sgen[0] IPv4, sgen[1] IPv6), other maps in sgen[0]
    uint64_t sgen[2] = {0, 0};
    // keys whose value was overwritten in place since the last commit (a
    // commit may patch those into the device tables instead of rebuilding);
    // CT maps also journal inserts and deletes here (TOUCH_* bits), which
    // a commit patches into the device CT table in place
    std::map<std::string, int> touched;
    bool ct() const { return role == ROLE_CT4 || role == ROLE_CT6; }
    // entries of a TCP CT map that no lookup reaches (ct_create4/6's ICMP
    // "related" entry, nexthdr != TCP at key byte 12 / 36): they live only
    // here, not in the device CT table (flatten.cpp build_ct), so the CT GC
    // filters them on the host; counted so a GC skips maps without any
    uint64_t n_aux = 0;
    bool aux_key(const std::string &k) const
    {
        return !ct_any && ((role == ROLE_CT4 && k.size() >= 13 && (uint8_t)k[12] != 6) ||
                           (role == ROLE_CT6 && k.size() >= 37 && (uint8_t)k[36] != 6));
    }
    // CT entries the device GC deleted that the host mirror still holds
    // (erased at the next ct_sync)
    uint64_t gc_pending = 0;

    struct Entry {
        std::string key;  // key bytes as last written
        std::string val;
    };
    // ordered by normalised key -> deterministic iteration and flattening
    std::map<std::string, Entry> kv;

    bool lpm() const { return type == MT_LPM_TRIE; }
    // a structural change to a normalised key: the ipcache's IPv6 keys
    // count apart (struct ipcache_key: family at byte 7, after the
    // prefixlen word); a prefix shorter than the family byte counts for both
    void bump_sgen(const std::string &nk)
    {
        uint32_t plen = 32;
        if (nk.size() >= 4)
            plen = (uint8_t)nk[0] | (uint8_t)nk[1] << 8 | (uint8_t)nk[2] << 16 |
                   (uint32_t)(uint8_t)nk[3] << 24;
        if (role != ROLE_IPCACHE || nk.size() <= 7 || plen < 32) {
            sgen[0]++;
            sgen[1]++;
        } else {
            sgen[(uint8_t)nk[7] == 2 ? 1 : 0]++;
        }
    }
    uint32_t value_bytes() const;  // per-CPU rounded for PERCPU maps
    // normalised key: raw for hashes; prefixlen + masked data for LPM.
    // Returns false for an invalid LPM key (prefixlen too large).
    bool norm(const uint8_t *k, std::string *out) const;

    // the device CT apply's changes, taken into the host mirror: no journal,
    // no structural generation (the device table already has them)
    void put_raw(const std::string &k, const std::string &v)
    {
        auto ins = kv.emplace(k, Entry{});
        if (ins.second && aux_key(k))
            n_aux++;
        Entry &e = ins.first->second;
        e.key = k;
        e.val = v;
        gen++;
    }
    void erase_raw(const std::string &k)
    {
        if (kv.erase(k)) {
            gen++;
            if (aux_key(k))
                n_aux--;
        }
    }

    // a CT entry removed while walking the map (the CT GC): journaled for
    // the next commit unless the device table never held it
    std::map<std::string, Entry>::iterator ct_erase_at(std::map<std::string, Entry>::iterator it,
                                                       bool journal)
    {
        if (aux_key(it->first))
            n_aux--;
        if (journal)
            touched[it->first] = TOUCH_ERASE;
        gen++;
        return kv.erase(it);
    }

    int update(const void *key, const void *value, uint64_t flags);
    int lookup(const void *key, void *value) const;
    int erase(const void *key);
    int next_key(const void *key, void *next) const;
};

Role role_for(const std::string &path, int *policy_lxc, int *ct_any = nullptr);

}  // namespace cfc
