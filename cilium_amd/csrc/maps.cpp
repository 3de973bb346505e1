#include "maps.hpp"

#include <cerrno>
#include <cstring>

namespace cfc {

static constexpr uint64_t BPF_NOEXIST = 1, BPF_EXIST = 2;  // BPF_ANY = 0

uint32_t Map::value_bytes() const
{
    if (type == MT_PERCPU_HASH)
        return (vsz + 7) & ~7u;  // one possible CPU
    return vsz;
}

bool Map::norm(const uint8_t *k, std::string *out) const
{
    if (!lpm()) {
        out->assign((const char *)k, ksz);
        return true;
    }
    uint32_t plen;
    memcpy(&plen, k, 4);
    uint32_t dbytes = ksz - 4;
    if (plen > dbytes * 8)
        return false;
    out->assign(ksz, '\0');
    memcpy(&(*out)[0], &plen, 4);
    for (uint32_t i = 0; i < dbytes; i++) {
        int b = (int)plen - 8 * (int)i;
        uint8_t m = b >= 8 ? 0xFF : b <= 0 ? 0 : (uint8_t)(0xFF << (8 - b));
        (*out)[4 + i] = (char)(k[4 + i] & m);
    }
    return true;
}

int Map::update(const void *key, const void *value, uint64_t flags)
{
    if (flags > BPF_EXIST)
        return -EINVAL;
    std::string nk;
    if (!norm((const uint8_t *)key, &nk))
        return -EINVAL;
    auto it = kv.find(nk);
    if (it != kv.end()) {
        if (flags == BPF_NOEXIST)
            return -EEXIST;
        touched[nk] |= TOUCH_VALUE;
    } else {
        if (flags == BPF_EXIST)
            return -ENOENT;
        if (kv.size() >= max_entries) {
            if (type == MT_LRU_HASH && !kv.empty()) {
                // stand-in for least recently used
                if (ct())
                    touched[kv.begin()->first] = TOUCH_ERASE;
                else
                    bump_sgen(kv.begin()->first);
                if (aux_key(kv.begin()->first))
                    n_aux--;
                kv.erase(kv.begin());
            } else {
                return lpm() ? -ENOSPC : -E2BIG;
            }
        }
        if (ct())
            touched[nk] = TOUCH_INSERT;
        else
            bump_sgen(nk);
        if (aux_key(nk))
            n_aux++;
    }
    Entry &e = kv[nk];
    e.key.assign((const char *)key, ksz);
    e.val.assign((const char *)value, value_bytes());
    gen++;
    return 0;
}

int Map::lookup(const void *key, void *value) const
{
    if (!lpm()) {
        auto it = kv.find(std::string((const char *)key, ksz));
        if (it == kv.end())
            return -ENOENT;
        memcpy(value, it->second.val.data(), value_bytes());
        return 0;
    }
    // longest stored prefix <= key prefixlen that matches (trie_lookup_elem)
    uint32_t plen;
    memcpy(&plen, key, 4);
    uint32_t maxbits = (ksz - 4) * 8;
    if (plen > maxbits)
        plen = maxbits;
    std::string probe((const char *)key, ksz);
    for (int p = (int)plen; p >= 0; p--) {
        uint32_t up = (uint32_t)p;
        memcpy(&probe[0], &up, 4);
        std::string nk;
        norm((const uint8_t *)probe.data(), &nk);
        auto it = kv.find(nk);
        if (it != kv.end()) {
            memcpy(value, it->second.val.data(), value_bytes());
            return 0;
        }
    }
    return -ENOENT;
}

int Map::erase(const void *key)
{
    std::string nk;
    if (!norm((const uint8_t *)key, &nk))
        return -EINVAL;
    auto it = kv.find(nk);
    if (it == kv.end())
        return -ENOENT;
    kv.erase(it);
    if (aux_key(nk))
        n_aux--;
    if (ct()) {
        touched[nk] = TOUCH_ERASE;
    } else {
        touched.erase(nk);
        bump_sgen(nk);
    }
    gen++;
    return 0;
}

int Map::next_key(const void *key, void *next) const
{
    if (kv.empty())
        return -ENOENT;
    auto it = kv.begin();
    if (key) {
        std::string nk;
        if (norm((const uint8_t *)key, &nk)) {
            auto cur = kv.find(nk);
            if (cur != kv.end()) {
                it = std::next(cur);
                if (it == kv.end())
                    return -ENOENT;
            }
        }
    }
    memcpy(next, it->second.key.data(), ksz);
    return 0;
}

// "<decimal lxc_id>" -> id, "global" -> -1; false otherwise
static bool parse_owner(const std::string &id, int *lxc)
{
    if (id == "global") {
        *lxc = -1;
        return true;
    }
    if (id.empty() || id.size() > 5 || id.find_first_not_of("0123456789") != std::string::npos)
        return false;
    long v = std::stol(id);
    if (v > 0xFFFF)
        return false;
    *lxc = (int)v;
    return true;
}

Role role_for(const std::string &path, int *policy_lxc, int *ct_any)
{
    std::string b = path.substr(path.find_last_of('/') + 1);
    *policy_lxc = -1;
    // pkg/maps/ctmap/ctmap.go:59-69: cilium_ct4_, cilium_ct_any4_, ...
    static const struct {
        const char *pfx;
        Role r;
        int any;
    } ct[] = {{"cilium_ct4_", ROLE_CT4, 0}, {"cilium_ct_any4_", ROLE_CT4, 1},
              {"cilium_ct6_", ROLE_CT6, 0}, {"cilium_ct_any6_", ROLE_CT6, 1}};
    for (const auto &c : ct) {
        const std::string pfx = c.pfx;
        int lxc;
        if (b.size() > pfx.size() && b.compare(0, pfx.size(), pfx) == 0 &&
            parse_owner(b.substr(pfx.size()), &lxc)) {
            *policy_lxc = lxc;
            if (ct_any)
                *ct_any = c.any;
            return c.r;
        }
    }
    if (b == "cilium_ipcache")
        return ROLE_IPCACHE;
    if (b == "cilium_lb4_services")
        return ROLE_LB4_SVC;
    if (b == "cilium_lb4_reverse_nat")
        return ROLE_LB4_RNAT;
    if (b == "cilium_lb6_services")
        return ROLE_LB6_SVC;
    if (b == "cilium_lb6_reverse_nat")
        return ROLE_LB6_RNAT;
    if (b == "cilium_lxc")
        return ROLE_LXC;
    if (b == "cilium_metrics")
        return ROLE_METRICS;
    if (b == "cilium_cidr_v4_fix" || b == "v4_fix")
        return ROLE_PF4_FIX;
    if (b == "cilium_cidr_v4_dyn" || b == "v4_dyn")
        return ROLE_PF4_DYN;
    if (b == "cilium_cidr_v6_fix" || b == "v6_fix")
        return ROLE_PF6_FIX;
    if (b == "cilium_cidr_v6_dyn" || b == "v6_dyn")
        return ROLE_PF6_DYN;
    const std::string pfx = "cilium_policy_";
    if (b.size() > pfx.size() && b.compare(0, pfx.size(), pfx) == 0) {
        std::string id = b.substr(pfx.size());
        if (id.find_first_not_of("0123456789") == std::string::npos &&
            id.size() <= 5) {
            long v = std::stol(id);
            if (v <= 0xFFFF) {
                *policy_lxc = (int)v;
                return ROLE_POLICY;
            }
        }
    }
    return ROLE_NONE;
}

}  // namespace cfc
