#include "flatten.hpp"

#include <algorithm>
#include <cstring>
#include <map>

namespace cfc {

static constexpr uint64_t POL_SLOTS_PER_KEY = 4;
static uint32_t pow2_at_least(uint64_t x)
{
    uint32_t p = 1;
    while (p < x)
        p <<= 1;
    return p;
}

uint64_t HostImage::device_bytes() const
{
    return 4ull * (tbl24.size() + tbl8.size() + lbl_ovf.size() +
                   pf_tbl24.size() + pf_tbl8.size() + pf_fix.size() +
                   pf_bloom.size() + pol_bloom.size()) +
           4ull * (l4d.size() + l4c.size()) + 8ull * l4l.size() +
           sizeof(LxcSlot) * lxc4.size() + sizeof(PolSlot) * pol.size() +
           ipc6.bytes() + pf6_fix.bytes() + pf6_dyn.bytes() +
           sizeof(Lxc6Slot) * lxc6.size() + sizeof(Ct4Slot) * ct4.size() +
           sizeof(Ct6Slot) * ct6.size() + 48ull * (ct4.size() + ct6.size());
}

// DIR-24-8: every prefix <= /24 fills its tbl24 range in ascending length
// order (longer prefixes overwrite), then every /25../32 expands its /24 into
// a 256-entry tbl8 group seeded with the covering value.
void build_dir24_8(std::vector<Pfx4> pfx, std::vector<uint32_t> *tbl24,
                   std::vector<uint32_t> *tbl8)
{
    std::stable_sort(pfx.begin(), pfx.end(),
                     [](const Pfx4 &a, const Pfx4 &b) { return a.plen < b.plen; });
    tbl24->assign(1u << 24, 0);
    tbl8->clear();
    uint32_t *t24 = tbl24->data();
    for (const Pfx4 &p : pfx) {
        if (p.plen > 24)
            break;
        uint32_t start = p.plen ? (p.addr >> 8) & ~((1u << (24 - p.plen)) - 1) : 0;
        std::fill(t24 + start, t24 + start + (1u << (24 - p.plen)), p.leaf);
    }
    for (const Pfx4 &p : pfx) {
        if (p.plen <= 24)
            continue;
        uint32_t idx = p.addr >> 8;
        if (!(t24[idx] & LPM_GROUP)) {
            uint32_t g = (uint32_t)(tbl8->size() >> 8);
            tbl8->resize(tbl8->size() + 256, t24[idx]);
            t24[idx] = LPM_GROUP | g;
        }
        uint32_t g = t24[idx] & ~LPM_GROUP;
        uint32_t lo = p.addr & 0xFF & ~((1u << (32 - p.plen)) - 1);
        uint32_t *grp = tbl8->data() + ((size_t)g << 8);
        std::fill(grp + lo, grp + lo + (1u << (32 - p.plen)), p.leaf);
    }
}

namespace {

// Builder of the compact multibit layout (layout.h).
struct L4Trie {
    std::vector<uint32_t> *d, *c, *ovf;
    std::vector<uint64_t> *l;
    bool ok = true;

    // list-entry leaf: 26 payload bits, wider labels through lbl_ovf
    uint32_t list_leaf(uint32_t leaf)
    {
        if (leaf & LPM_INDIRECT)
            return LL_INDIRECT | (leaf & LPM_PAYLOAD);
        if (leaf > LL_PAYLOAD) {
            ovf->push_back(leaf);
            return LL_INDIRECT | (uint32_t)(ovf->size() - 1);
        }
        return leaf;
    }
    uint64_t entry(uint32_t addr, int len, uint32_t leaf)
    {
        return ((uint64_t)(((uint32_t)len & 31) << 27 | list_leaf(leaf)) << 32) | addr;
    }

    // The node for the range `base`/`lvl` whose own covering leaf is `def`;
    // `longp` holds the prefixes longer than lvl inside the range.  At the
    // /16 level (dir != null) the longest two go into the directory entry.
    uint32_t node(std::vector<Pfx4> &longp, uint32_t base, int lvl, uint32_t def,
                  uint32_t *dir = nullptr)
    {
        if (longp.empty())
            return def;
        if (longp.size() + 1 < L4_LIST_MAX) {
            std::stable_sort(longp.begin(), longp.end(),
                             [](const Pfx4 &a, const Pfx4 &b) { return a.plen > b.plen; });
            size_t first = 0;
            if (dir) {
                uint64_t e[L4_INLINE] = {0, 0};
                for (; first < longp.size() && first < L4_INLINE; first++)
                    e[first] = l4_inline_entry(longp[first].addr, longp[first].plen,
                                               list_leaf(longp[first].leaf));
                dir[1] = (uint32_t)e[0];
                dir[2] = (uint32_t)(e[0] >> 32) | (uint32_t)(e[1] << 16);
                dir[3] = (uint32_t)(e[1] >> 16);
                if (first == longp.size())
                    return def;
            }
            const size_t off = l->size();   // always even
            for (size_t i = first; i < longp.size(); i++)
                l->push_back(entry(longp[i].addr, longp[i].plen, longp[i].leaf));
            l->push_back(entry(base, lvl, def));
            if (l->size() & 1)
                l->push_back(l->back());
            if (off > L4_OFF)
                ok = false;
            return L4_PTR | (uint32_t)(l->size() - off) << 24 | (uint32_t)(off & L4_OFF);
        }
        // split: a chunk for the next 8 bits
        const int nl = lvl + 8;
        const uint32_t sh = 32 - nl;
        const size_t off = c->size();
        c->resize(off + 256, 0);
        uint32_t defs[256];
        std::fill(defs, defs + 256, def);
        std::vector<std::vector<Pfx4>> sub(256);
        std::stable_sort(longp.begin(), longp.end(),
                         [](const Pfx4 &a, const Pfx4 &b) { return a.plen < b.plen; });
        for (const Pfx4 &p : longp) {
            const uint32_t j = (p.addr >> sh) & 255;
            if (p.plen <= nl) {
                const uint32_t span = 1u << (nl - p.plen);
                std::fill(defs + (j & ~(span - 1)), defs + (j & ~(span - 1)) + span, p.leaf);
            } else {
                sub[j].push_back(p);
            }
        }
        for (uint32_t j = 0; j < 256; j++) {
            const uint32_t e = node(sub[j], base | (j << sh), nl, defs[j]);
            (*c)[off + j] = e;
        }
        if (off > L4_OFF)
            ok = false;
        return L4_PTR | (uint32_t)off;
    }
};

}  // namespace

bool build_l4trie(std::vector<Pfx4> pfx, std::vector<uint32_t> *ovf,
                  std::vector<uint32_t> *l4d, std::vector<uint32_t> *l4c,
                  std::vector<uint64_t> *l4l)
{
    std::stable_sort(pfx.begin(), pfx.end(),
                     [](const Pfx4 &a, const Pfx4 &b) { return a.plen < b.plen; });
    l4d->assign(4u << 16, 0);
    l4c->clear();
    l4l->clear();
    // /0../16: paint the directory's covering leaves, shortest first
    for (const Pfx4 &p : pfx) {
        if (p.plen > 16)
            break;
        const uint32_t start = p.plen ? (p.addr >> 16) & ~((1u << (16 - p.plen)) - 1) : 0;
        for (uint32_t j = start; j < start + (1u << (16 - p.plen)); j++)
            (*l4d)[4 * j] = p.leaf;
    }
    std::map<uint32_t, std::vector<Pfx4>> by16;
    for (const Pfx4 &p : pfx)
        if (p.plen > 16)
            by16[p.addr >> 16].push_back(p);
    L4Trie b{l4d, l4c, ovf, l4l};
    for (auto &g : by16) {
        uint32_t *dir = l4d->data() + 4 * g.first;
        dir[0] = b.node(g.second, g.first << 16, 16, dir[0], dir);
    }
    return b.ok;
}

// ---- IPv6 LPM (layout.h Lpm6)
namespace {

typedef std::pair<uint64_t, uint64_t> U128;

U128 masked128(const uint32_t w[4], uint32_t len)
{
    uint32_t m[4];
    for (int i = 0; i < 4; i++)
        m[i] = w[i] & l6_word_mask(len, i);
    return {(uint64_t)m[0] << 32 | m[1], (uint64_t)m[2] << 32 | m[3]};
}

// most keys of lengths L[i..k] that share one address masked to L[k]
size_t max_pile(const std::vector<std::vector<const Pfx6 *>> &by_len,
                const std::vector<uint32_t> &L, size_t i, size_t k)
{
    std::vector<U128> v;
    for (size_t j = i; j <= k; j++)
        for (const Pfx6 *p : by_len[L[j]])
            v.push_back(masked128(p->w, L[k]));
    std::sort(v.begin(), v.end());
    size_t best = 0;
    for (size_t a = 0; a < v.size();) {
        size_t b = a;
        while (b < v.size() && v[b] == v[a])
            b++;
        best = std::max(best, b - a);
        a = b;
    }
    return best;
}

}  // namespace

void build_lpm6(const std::vector<Pfx6> &pfx, Lpm6Host *out)
{
    *out = Lpm6Host();
    out->n = (uint32_t)pfx.size();
    std::vector<std::vector<const Pfx6 *>> by_len(129);
    size_t nkeys = 0;
    for (const Pfx6 &p : pfx) {
        if (p.plen == 0) {
            out->def_label = p.label;
        } else {
            by_len[p.plen].push_back(&p);
            nkeys++;
        }
    }
    std::vector<uint32_t> L;
    for (uint32_t l = 128; l >= 1; l--)
        if (!by_len[l].empty())
            L.push_back(l);
    if (L.empty())
        return;
    // Bloom groups: extend a group to the next shorter length while the
    // addresses masked to it keep at most L6_GROUP_MAX keys per word
    uint32_t sel_of[129] = {0};
    for (size_t i = 0; i < L.size();) {
        size_t k = i;
        while (k + 1 < L.size() && max_pile(by_len, L, i, k + 1) <= L6_GROUP_MAX)
            k++;
        for (size_t j = i; j <= k; j++) {
            out->lens.push_back(L[j] | L[k] << 8 | (j == i ? L6_GROUP_FIRST : 0));
            sel_of[L[j]] = L[k];
        }
        out->groups++;
        i = k + 1;
    }
    out->bloom.assign(pow2_at_least(std::max<size_t>(64, nkeys / 4)), 0);
    const uint32_t bmask = (uint32_t)out->bloom.size() - 1;
    size_t n64 = 0;
    for (uint32_t len : L)
        n64 += len <= 64 ? by_len[len].size() : 0;
    if (nkeys > n64)
        out->slots.assign(pow2_at_least(std::max<size_t>(16, 2 * (nkeys - n64))), L6Slot{});
    if (n64)
        out->slots64.assign(pow2_at_least(std::max<size_t>(16, 2 * n64)), make_uint4(0, 0, 0, 0));
    const uint32_t ns = (uint32_t)out->slots.size(), ns64 = (uint32_t)out->slots64.size();
    for (uint32_t len : L)
        for (const Pfx6 *p : by_len[len]) {
            const uint32_t h = l6_hash(p->w[0], p->w[1], p->w[2], p->w[3], len);
            out->bloom[l6_group_hash(p->w, sel_of[len]) & bmask] |= l6_bloom_bits(h);
            if (len <= 64) {
                uint32_t s = h & (ns64 - 1);
                while (out->slots64[s].w)
                    s = (s + 1) & (ns64 - 1);
                out->slots64[s] = make_uint4(p->w[0], p->w[1], p->label, len);
                continue;
            }
            uint32_t s = h & (ns - 1);
            while (out->slots[s].len)
                s = (s + 1) & (ns - 1);
            L6Slot &d = out->slots[s];
            memcpy(d.w, p->w, 16);
            d.label = p->label;
            d.len = len;
        }
}

uint32_t lpm6_lookup_host(const Lpm6Host &t, const uint32_t w[4])
{
    const uint32_t mask = (uint32_t)t.slots.size() - 1;
    const uint32_t bmask = (uint32_t)t.bloom.size() - 1;
    uint64_t bw = 0;
    for (uint32_t e : t.lens) {
        const uint32_t len = e & 255;
        if (e & L6_GROUP_FIRST)
            bw = t.bloom[l6_group_hash(w, (e >> 8) & 255) & bmask];
        uint32_t m[4];
        for (int i = 0; i < 4; i++)
            m[i] = w[i] & l6_word_mask(len, i);
        const uint32_t h = l6_hash(m[0], m[1], m[2], m[3], len);
        const uint64_t b = l6_bloom_bits(h);
        if ((bw & b) != b)
            continue;
        if (len <= 64) {
            const uint32_t mask64 = (uint32_t)t.slots64.size() - 1;
            for (uint32_t s = h & mask64;; s = (s + 1) & mask64) {
                const uint4 &d = t.slots64[s];
                if (!d.w)
                    break;
                if (d.w == len && d.x == m[0] && d.y == m[1])
                    return d.z;
            }
            continue;
        }
        for (uint32_t s = h & mask;; s = (s + 1) & mask) {
            const L6Slot &d = t.slots[s];
            if (!d.len)
                break;
            if (d.len == len && !memcmp(d.w, m, 16))
                return d.label;
        }
    }
    return t.def_label;
}

// Blocked Bloom filter with ~`per_word` keys per 32-bit word, capped.
static void bloom_size(std::vector<uint32_t> *b, size_t keys, uint32_t max_words)
{
    uint32_t w = pow2_at_least(std::max<size_t>(64, keys));
    b->assign(std::min(w, max_words), 0u);
}
static inline void bloom_add(std::vector<uint32_t> *b, uint32_t h)
{
    (*b)[h & (b->size() - 1)] |= bloom_bits(h);
}

static uint32_t leaf_for(uint32_t label, std::vector<uint32_t> *ovf)
{
    if (label < LPM_INDIRECT)
        return label;
    ovf->push_back(label);
    return LPM_INDIRECT | (uint32_t)(ovf->size() - 1);
}

static inline uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// Effective IPv4 prefixes of the ipcache LPM map.  A datapath v4 lookup key
// is {prefixlen 64, pad 0,0, family 1, addr, zeros} (eps.h:70-80); a stored
// entry with total prefixlen P matches iff P <= 64 and its first P bits agree,
// so entries with P <= 32 whose static bits agree act as v4 /0.  Among
// entries collapsing onto the same v4 prefix the longest P wins (trie).
static void ipcache_v4(const Map *m, std::vector<Pfx4> *out,
                       std::vector<uint32_t> *ovf)
{
    static const uint8_t stat4[4] = {0, 0, 0, 1};
    std::map<std::pair<uint32_t, int>, std::pair<uint32_t, uint32_t>> best;
    for (const auto &kv : m->kv) {
        const uint8_t *k = (const uint8_t *)kv.first.data();  // normalised
        uint32_t P;
        memcpy(&P, k, 4);
        if (P > 64)
            continue;
        bool ok = true;
        for (uint32_t bit = 0; bit < std::min<uint32_t>(P, 32); bit++) {
            uint32_t byte = bit >> 3, sh = 7 - (bit & 7);
            if (((k[4 + byte] >> sh) & 1) != ((stat4[byte] >> sh) & 1)) {
                ok = false;
                break;
            }
        }
        if (!ok)
            continue;
        int plen = P > 32 ? (int)(P - 32) : 0;
        uint32_t a;
        memcpy(&a, k + 8, 4);  // already masked by norm()
        uint32_t label;
        memcpy(&label, kv.second.val.data(), 4);
        auto key = std::make_pair(bswap(a), plen);
        auto it = best.find(key);
        if (it == best.end() || it->second.first < P)
            best[key] = {P, label};
    }
    for (const auto &b : best)
        out->push_back({b.first.first, (uint8_t)b.first.second,
                        leaf_for(b.second.second, ovf)});
}

// Effective IPv6 prefixes of the ipcache: as ipcache_v4 with the v6 lookup
// key {prefixlen 160, pad 0,0, family 2, addr} (eps.h:56-66).
bool ipcache_v6_entry(const std::string &nk, const std::string &val, Pfx6 *p)
{
    static const uint8_t stat6[4] = {0, 0, 0, 2};
    const uint8_t *k = (const uint8_t *)nk.data();
    uint32_t P;
    memcpy(&P, k, 4);
    if (P <= 32 || P > 160 || nk.size() < 24 || val.size() < 4)
        return false;
    for (uint32_t bit = 0; bit < 32; bit++) {
        uint32_t byte = bit >> 3, sh = 7 - (bit & 7);
        if (((k[4 + byte] >> sh) & 1) != ((stat6[byte] >> sh) & 1))
            return false;
    }
    p->plen = (uint8_t)(P - 32);
    for (int i = 0; i < 4; i++) {
        uint32_t a;
        memcpy(&a, k + 8 + 4 * i, 4);
        p->w[i] = bswap(a) & l6_word_mask(p->plen, i);
    }
    memcpy(&p->label, val.data(), 4);
    return true;
}

int64_t lpm6_find_slot(const Lpm6Host &t, const Pfx6 &p)
{
    if (p.plen && p.plen <= 64) {
        if (t.slots64.empty())
            return -1;
        const uint32_t mask = (uint32_t)t.slots64.size() - 1;
        uint32_t s = l6_hash(p.w[0], p.w[1], p.w[2], p.w[3], p.plen) & mask;
        for (uint32_t n = 0; n <= mask; n++, s = (s + 1) & mask) {
            const uint4 &d = t.slots64[s];
            if (!d.w)
                return -1;
            if (d.w == p.plen && d.x == p.w[0] && d.y == p.w[1])
                return L6_S64 | s;
        }
        return -1;
    }
    if (t.slots.empty() || !p.plen)
        return -1;
    const uint32_t mask = (uint32_t)t.slots.size() - 1;
    uint32_t s = l6_hash(p.w[0], p.w[1], p.w[2], p.w[3], p.plen) & mask;
    for (uint32_t n = 0; n <= mask; n++, s = (s + 1) & mask) {
        const L6Slot &d = t.slots[s];
        if (!d.len)
            return -1;
        if (d.len == p.plen && !memcmp(d.w, p.w, 16))
            return s;
    }
    return -1;
}

static void ipcache_v6(const Map *m, std::vector<Pfx6> *out)
{
    static const uint8_t stat6[4] = {0, 0, 0, 2};
    std::map<std::pair<U128, int>, std::pair<uint32_t, Pfx6>> best;
    for (const auto &kv : m->kv) {
        const uint8_t *k = (const uint8_t *)kv.first.data();  // normalised
        uint32_t P;
        memcpy(&P, k, 4);
        if (P > 160)
            continue;
        bool ok = true;
        for (uint32_t bit = 0; bit < std::min<uint32_t>(P, 32); bit++) {
            uint32_t byte = bit >> 3, sh = 7 - (bit & 7);
            if (((k[4 + byte] >> sh) & 1) != ((stat6[byte] >> sh) & 1)) {
                ok = false;
                break;
            }
        }
        if (!ok)
            continue;
        Pfx6 p;
        p.plen = (uint8_t)(P > 32 ? P - 32 : 0);
        for (int i = 0; i < 4; i++) {
            uint32_t a;
            memcpy(&a, k + 8 + 4 * i, 4);
            p.w[i] = bswap(a) & l6_word_mask(p.plen, i);
        }
        memcpy(&p.label, kv.second.val.data(), 4);
        auto key = std::make_pair(masked128(p.w, p.plen), (int)p.plen);
        auto it = best.find(key);
        if (it == best.end() || it->second.first < P)
            best[key] = {P, p};
    }
    for (const auto &b : best)
        out->push_back(b.second.second);
}

// prefilter v6 maps: key {u32 prefixlen, 16-byte address}
static void prefilter_v6(const Map *m, bool exact, std::vector<Pfx6> *out)
{
    for (const auto &kv : m->kv) {
        const uint8_t *k = (const uint8_t *)kv.first.data();
        uint32_t P;
        memcpy(&P, k, 4);
        if (exact && P != 128)   // check_v6 looks up {128, saddr} exactly
            continue;
        if (P > 128)
            continue;
        Pfx6 p;
        p.plen = (uint8_t)P;
        p.label = 1;
        for (int i = 0; i < 4; i++) {
            uint32_t a;
            memcpy(&a, k + 4 + 4 * i, 4);
            p.w[i] = bswap(a) & l6_word_mask(P, i);
        }
        out->push_back(p);
    }
}

// struct endpoint_info {u32 ifindex; u16 unused; u16 lxc_id; u32 flags; ...}
static uint32_t lxc_info(const HostImage *img, const uint8_t *v, PolLoc *loc)
{
    uint32_t ifindex, flags;
    uint16_t id;
    memcpy(&ifindex, v, 4);
    memcpy(&id, v + 6, 2);
    memcpy(&flags, v + 8, 4);
    uint32_t info = id | LXC_VALID | ((flags & 1) ? LXC_HOST : 0) |
                    (ifindex ? LXC_IFINDEX : 0) |
                    (img->ct_local.size() > id && img->ct_local[id] ? LXC_CT_LOCAL : 0);
    auto it = img->pol_loc.find(id);
    *loc = PolLoc();
    if (it != img->pol_loc.end()) {
        *loc = it->second;
        info |= LXC_HAS_POLICY;
    }
    return info;
}

static Lxc6Slot lxc6_slot(const HostImage *img, const uint8_t *k, const uint8_t *v)
{
    Lxc6Slot r{};
    memcpy(r.a, k, 16);
    PolLoc loc;
    r.info = lxc_info(img, v, &loc);
    r.pol_base = loc.base;
    r.pol_mask = loc.mask;
    return r;
}

uint64_t ct_map_key(int family, uint32_t owner, int any)
{
    return (uint64_t)family << 40 | (uint64_t)owner << 8 | (uint64_t)any;
}

bool ct_slot_of(const Map *m, const std::string &key, Ct4Slot *s4, Ct6Slot *s6)
{
    const bool v6 = m->role == ROLE_CT6;
    const uint32_t al = v6 ? 16 : 4;
    if (key.size() != 2 * al + 6)
        return false;
    const uint8_t *k = (const uint8_t *)key.data();
    const uint8_t nh = k[2 * al + 4], fl = k[2 * al + 5];
    const uint8_t icmp = v6 ? 58 : 1;
    if (!(m->ct_any ? (nh == 17 || nh == icmp) : nh == 6) || (fl & ~7u))
        return false;
    uint32_t z;
    memcpy(&z, k + 2 * al, 4);
    const uint32_t w = ct_word(nh, fl, ct_owner_word((uint32_t)std::max(m->policy_lxc, 0),
                                                      m->policy_lxc >= 0));
    if (!v6) {
        memcpy(&s4->x, k, 4);
        memcpy(&s4->y, k + 4, 4);
        s4->z = z;
        s4->w = w;
    } else {
        *s6 = Ct6Slot{};
        memcpy(s6->d, k, 16);
        memcpy(s6->s, k + 16, 16);
        s6->z = z;
        s6->w = w;
    }
    return true;
}

// struct ct_entry: bits @36, tx/rx_flags_seen @42/43, last_tx/rx_report @48/52
CtTimer ct_timer_of(const std::string &val)
{
    CtTimer tm{};
    if (val.size() >= 56) {
        const uint8_t *v = (const uint8_t *)val.data();
        uint16_t bits;
        memcpy(&bits, v + 36, 2);
        memcpy(&tm.last_tx, v + 48, 4);
        memcpy(&tm.last_rx, v + 52, 4);
        tm.flags = v[43] | (uint32_t)v[42] << 8 | (uint32_t)(bits & 3) << 16 |
                   ((bits & 16) ? CTT_NON_SYN : 0u) | ((bits & 4) ? CTT_NAT46 : 0u);
        memcpy(&tm.lifetime, v + 32, 4);
    }
    return tm;
}

// struct ct_entry: rev_nat_index @38, bits @36 (lb_loopback = bit 3),
// slave @40
uint4 ct_lb_of(const std::string &val)
{
    uint16_t bits = 0, rev = 0, slave = 0;
    if (val.size() >= 42) {
        memcpy(&bits, &val[36], 2);
        memcpy(&rev, &val[38], 2);
        memcpy(&slave, &val[40], 2);
    }
    return make_uint4(rev | ((bits >> 3) & 1u) << 16, slave, 0, 0);
}

// cilium_lb6_services / cilium_lb6_reverse_nat (layout.h)
static void build_lb6(const Map *svc, const Map *rnat, HostImage *img)
{
    if (svc && !svc->kv.empty()) {
        const uint32_t ns = pow2_at_least(std::max<uint64_t>(16, 2ull * svc->kv.size()));
        img->lb6.assign(3ull * ns, make_uint4(0, 0, 0, 0));
        img->lb6_mask = ns - 1;
        for (const auto &kv : svc->kv) {
            if (kv.first.size() != 20 || kv.second.val.size() < 24)
                continue;
            uint32_t k[5], v[6];
            memcpy(k, kv.first.data(), 20);
            memcpy(v, kv.second.val.data(), 24);
            uint32_t i = lb6_hash(k[0], k[1], k[2], k[3], k[4]) & img->lb6_mask;
            while (img->lb6[3 * i + 1].w)
                i = (i + 1) & img->lb6_mask;
            img->lb6[3 * i] = make_uint4(k[0], k[1], k[2], k[3]);
            img->lb6[3 * i + 1] = make_uint4(k[4], v[4], v[5], 1);
            img->lb6[3 * i + 2] = make_uint4(v[0], v[1], v[2], v[3]);
            img->n_lb6++;
        }
    }
    if (rnat && !rnat->kv.empty()) {
        img->rnat6.assign(2ull * 65536, make_uint4(0, 0, 0, 0));
        for (const auto &kv : rnat->kv) {
            if (kv.first.size() != 2 || kv.second.val.size() < 18)
                continue;
            uint16_t idx, port;
            uint32_t a[4];
            memcpy(&idx, kv.first.data(), 2);
            memcpy(a, kv.second.val.data(), 16);
            memcpy(&port, kv.second.val.data() + 16, 2);
            img->rnat6[2ull * idx] = make_uint4(a[0], a[1], a[2], a[3]);
            img->rnat6[2ull * idx + 1] = make_uint4(port | 1u << 16, 0, 0, 0);
        }
    }
}

// cilium_lb4_services / cilium_lb4_reverse_nat (layout.h)
static void build_lb(const Map *svc, const Map *rnat, HostImage *img)
{
    if (svc && !svc->kv.empty()) {
        const uint32_t ns = pow2_at_least(std::max<uint64_t>(16, 2ull * svc->kv.size()));
        img->lb4.assign(2ull * ns, make_uint4(0, 0, 0, 0));
        img->lb4_mask = ns - 1;
        for (const auto &kv : svc->kv) {
            if (kv.first.size() != 8 || kv.second.val.size() < 12)
                continue;
            uint32_t k[2], v[3];
            memcpy(k, kv.first.data(), 8);
            memcpy(v, kv.second.val.data(), 12);
            uint32_t i = lb4_hash(k[0], k[1]) & img->lb4_mask;
            while (img->lb4[2 * i + 1].y)
                i = (i + 1) & img->lb4_mask;
            img->lb4[2 * i] = make_uint4(k[0], k[1], v[0], v[1]);
            img->lb4[2 * i + 1] = make_uint4(v[2], 1, 0, 0);
            img->n_lb4++;
        }
    }
    if (rnat && !rnat->kv.empty()) {
        img->rnat4.assign(65536, make_uint2(0, 0));
        for (const auto &kv : rnat->kv) {
            if (kv.first.size() != 2 || kv.second.val.size() < 6)
                continue;
            uint16_t idx, port;
            uint32_t addr;
            memcpy(&idx, kv.first.data(), 2);
            memcpy(&addr, kv.second.val.data(), 4);
            memcpy(&port, kv.second.val.data() + 4, 2);
            img->rnat4[idx] = make_uint2(addr, port | 1u << 16);
        }
    }
}

// CT maps -> one open-addressed table per family (layout.h).  Entries no
// lookup can reach (nexthdr not served by their map) are left out.  A
// commit patches later inserts and deletes into the same table
// (cfc_api.cpp patch_ct; deleted slots become CT_TOMBSTONE).
static void build_ct(const std::vector<const Map *> &cts, HostImage *img)
{
    size_t n4 = 0, n6 = 0;
    for (const Map *m : cts)
        (m->role == ROLE_CT4 ? n4 : n6) += m->kv.size();
    // (an empty family keeps no table unless a device apply asked for one)
    if (n4 || img->ct_min4) {
        uint32_t ns = pow2_at_least(std::max<uint64_t>({16, 2ull * n4, img->ct_min4}));
        img->ct4.assign(ns, Ct4Slot{});
        img->ct4_tm.assign(ns, CtTimer{});
        img->ct4_mask = ns - 1;
    }
    // with a load balancer the kernels read each CT4 entry's LB state; an
    // entry that carries one asks for it too
    bool lb = img->lb_ct;
    for (const Map *m : cts)
        if (!lb && m->role == ROLE_CT4)
            for (const auto &kv : m->kv) {
                const uint4 l = ct_lb_of(kv.second.val);
                if (l.x | l.y) {
                    lb = true;
                    break;
                }
            }
    img->lb_ct = lb;
    if (!img->ct4.empty() && lb)
        img->ct4_lb.assign(img->ct4.size(), make_uint4(0, 0, 0, 0));
    if (n6 || img->ct_min6) {
        uint32_t ns = pow2_at_least(std::max<uint64_t>({16, 2ull * n6, img->ct_min6}));
        img->ct6.assign(ns, Ct6Slot{});
        img->ct6_tm.assign(ns, CtTimer{});
        img->ct6_mask = ns - 1;
        if (img->lb6_ct)   // (IPv6 entries always carry rev_nat_index)
            img->ct6_lb.assign(ns, make_uint4(0, 0, 0, 0));
    }
    for (const Map *m : cts) {
        const bool v6 = m->role == ROLE_CT6;
        if (m->ksz != (v6 ? 38u : 14u))
            continue;
        for (const auto &kv : m->kv) {
            Ct4Slot e;
            Ct6Slot e6;
            if (!ct_slot_of(m, kv.first, &e, &e6))
                continue;
            const CtTimer tm = ct_timer_of(kv.second.val);
            if (!v6) {
                uint32_t i = ct_home4(e.x, e.y, e.z, e.w) & img->ct4_mask, p = 0;
                while (img->ct4[i].w) {
                    i = (i + 1) & img->ct4_mask;
                    p++;
                }
                img->ct4[i] = e;
                img->ct4_tm[i] = tm;
                if (!img->ct4_lb.empty())
                    img->ct4_lb[i] = ct_lb_of(kv.second.val);
                img->ct4_probe = std::max(img->ct4_probe, p);
                img->n_ct4++;
                img->n_nat46 += (tm.flags & CTT_NAT46) != 0;
            } else {
                const Ct6Slot &e = e6;
                uint32_t i = ct_home6(e.d, e.s, e.z, e.w) & img->ct6_mask, p = 0;
                while (img->ct6[i].w) {
                    i = (i + 1) & img->ct6_mask;
                    p++;
                }
                img->ct6[i] = e;
                img->ct6_tm[i] = tm;
                if (!img->ct6_lb.empty()) {
                    const uint4 l = ct_lb_of(kv.second.val);
                    img->ct6_lb[i] = make_uint4(l.x & 0xFFFF, l.y, 0, 0);
                }
                img->ct6_probe = std::max(img->ct6_probe, p);
                img->n_ct6++;
            }
            if (m->policy_lxc >= 0)
                img->ct_local[m->policy_lxc] = 1;
        }
        if (m->policy_lxc >= 0)
            img->ct_local[m->policy_lxc] = 1;
    }
}

void build_image(const std::vector<Map *> &maps, const BuildOpts &opt,
                 HostImage *img, unsigned groups)
{
    const uint64_t ct_min4 = img->ct_min4, ct_min6 = img->ct_min6;   // (the caller's)
    *img = HostImage();
    img->ct_min4 = ct_min4;
    img->ct_min6 = ct_min6;
    img->ct_local.assign(65536, 0);
    std::vector<const Map *> cts;
    for (Map *m : maps)
        if (m->role == ROLE_CT4 || m->role == ROLE_CT6) {
            cts.push_back(m);
            if (m->policy_lxc >= 0)
                img->ct_local[m->policy_lxc] = 1;
        }
    const Map *lbsvc = nullptr, *lbrnat = nullptr, *lb6svc = nullptr, *lb6rnat = nullptr;
    for (Map *m : maps) {
        if (m->role == ROLE_LB4_SVC)
            lbsvc = m;
        else if (m->role == ROLE_LB4_RNAT)
            lbrnat = m;
        else if (m->role == ROLE_LB6_SVC)
            lb6svc = m;
        else if (m->role == ROLE_LB6_RNAT)
            lb6rnat = m;
    }
    img->lb_ct = (lbsvc && !lbsvc->kv.empty()) || (lbrnat && !lbrnat->kv.empty());
    img->lb6_ct = (lb6svc && !lb6svc->kv.empty()) || (lb6rnat && !lb6rnat->kv.empty());
    if (groups & GROUP_LB) {
        build_lb(lbsvc, lbrnat, img);
        build_lb6(lb6svc, lb6rnat, img);
    }
    if (groups & GROUP_CT)
        build_ct(cts, img);
    const Map *ipc = nullptr, *lxc = nullptr, *pf4fix = nullptr,
              *pf4dyn = nullptr, *pf6fix = nullptr, *pf6dyn = nullptr;
    std::map<int, Map *> pols;
    for (Map *m : maps) {
        switch (m->role) {
        case ROLE_IPCACHE: ipc = m; break;
        case ROLE_LXC: lxc = m; break;
        case ROLE_PF4_FIX: pf4fix = m; break;
        case ROLE_PF4_DYN: pf4dyn = m; break;
        case ROLE_PF6_FIX: pf6fix = m; break;
        case ROLE_PF6_DYN: pf6dyn = m; break;
        case ROLE_POLICY: pols[m->policy_lxc] = m; break;
        default: break;
        }
    }

    const Map *ipc6m = (groups & GROUP_IPCACHE6) ? ipc : nullptr;
    if (!(groups & GROUP_IPCACHE4))
        ipc = nullptr;
    if (!(groups & GROUP_PREFILTER))
        pf4fix = pf4dyn = pf6fix = pf6dyn = nullptr;
    if (!(groups & GROUP_ENDPOINTS)) {
        lxc = nullptr;
        pols.clear();
    }
    // ---- ipcache v4: the compact multibit layout unless forced (or its
    //      offsets overflow), DIR-24-8 otherwise
    if (ipc) {
        std::vector<Pfx4> pfx;
        ipcache_v4(ipc, &pfx, &img->lbl_ovf);
        img->n_prefix4 = (uint32_t)pfx.size();
        if (!pfx.empty()) {
            const size_t n_ovf = img->lbl_ovf.size();
            bool trie = opt.lpm4 != LPM4_DIR24_8;
            if (trie && !build_l4trie(pfx, &img->lbl_ovf, &img->l4d, &img->l4c,
                                      &img->l4l)) {
                img->l4d.clear();
                img->l4c.clear();
                img->l4l.clear();
                img->lbl_ovf.resize(n_ovf);
                trie = false;
            }
            if (trie) {
                img->lpm4_layout = LPM4_TRIE;
            } else {
                build_dir24_8(pfx, &img->tbl24, &img->tbl8);
                img->lpm4_layout = LPM4_DIR24_8;
            }
        }
    }

    // ---- ipcache v6
    if (ipc6m) {
        std::vector<Pfx6> pfx;
        ipcache_v6(ipc6m, &pfx);
        build_lpm6(pfx, &img->ipc6);
    }

    // ---- prefilter
    if (pf6fix && pf6fix->ksz == 20) {
        std::vector<Pfx6> pfx;
        prefilter_v6(pf6fix, true, &pfx);
        build_lpm6(pfx, &img->pf6_fix);
        // (check_v6 looks up {prefixlen 128, saddr} exactly: a filter over
        // the addresses screens it, as pf_bloom does for IPv4)
        bool all128 = !pfx.empty();
        for (const Pfx6 &p : pfx)
            all128 &= p.plen == 128;
        if (all128) {
            bloom_size(&img->pf6_bloom, 2 * pfx.size(), PF_BLOOM_MAX_WORDS);
            for (const Pfx6 &p : pfx)
                bloom_add(&img->pf6_bloom, pf6_bloom_hash(p.w[0], p.w[1], p.w[2], p.w[3]));
        }
    }
    if (pf6dyn && pf6dyn->ksz == 20) {
        std::vector<Pfx6> pfx;
        prefilter_v6(pf6dyn, false, &pfx);
        build_lpm6(pfx, &img->pf6_dyn);
    }
    if (pf4dyn && pf4dyn->ksz == 8) {
        std::vector<Pfx4> pfx;
        for (const auto &kv : pf4dyn->kv) {
            const uint8_t *k = (const uint8_t *)kv.first.data();
            uint32_t P, a;
            memcpy(&P, k, 4);
            memcpy(&a, k + 4, 4);
            pfx.push_back({bswap(a), (uint8_t)P, 1u});
        }
        img->n_pf_dyn = (uint32_t)pfx.size();
        if (!pfx.empty())
            build_dir24_8(pfx, &img->pf_tbl24, &img->pf_tbl8);
    }
    if (pf4fix && pf4fix->ksz == 8) {
        std::vector<uint32_t> addrs;
        for (const auto &kv : pf4fix->kv) {
            const uint8_t *k = (const uint8_t *)kv.first.data();
            uint32_t P, a;
            memcpy(&P, k, 4);
            memcpy(&a, k + 4, 4);
            if (P != 32)   // check_v4 looks up {prefixlen 32, saddr} exactly
                continue;
            if (a == 0)
                img->pf_fix_zero = 1;   // 0 marks free slots
            else
                addrs.push_back(a);
        }
        img->n_pf_fix = (uint32_t)addrs.size() + img->pf_fix_zero;
        if (!addrs.empty()) {
            // ~1 key per 4 bits of filter at most: 25k deny addresses in
            // 32 KiB give ~1.5% false positives
            bloom_size(&img->pf_bloom, 2 * addrs.size(), PF_BLOOM_MAX_WORDS);
            for (uint32_t a : addrs)
                bloom_add(&img->pf_bloom, pf_bloom_hash(a));
            // load factor <= 25%: 4-address buckets, one per expected address
            uint32_t nb = pow2_at_least(addrs.size());
            img->pf_fix.assign((size_t)nb * PF_SLOTS, 0);
            img->pf_fix_mask = nb - 1;
            for (uint32_t a : addrs) {
                uint32_t b = hash32(a, nb - 1);
                for (;;) {
                    uint32_t *bk = &img->pf_fix[(size_t)b * PF_SLOTS];
                    int s = 0;
                    while (s < PF_SLOTS && bk[s])
                        s++;
                    if (s < PF_SLOTS) {
                        bk[s] = a;
                        break;
                    }
                    b = (b + 1) & (nb - 1);
                }
            }
        }
    }

    // ---- policy tables (deterministic: ascending lxc id, key order);
    //      linear probing over 16-byte slots at load factor <= 25%: a hit is
    //      one 16-byte load 5 times in 6 (at 50% it was every other hit that
    //      needed a second, dependent, L2 round trip); the Bloom filter
    //      screens out most lookups of absent keys
    size_t n_pol_keys = 0;
    for (auto &pm : pols)
        n_pol_keys += pm.second->kv.size();
    if (n_pol_keys)
        bloom_size(&img->pol_bloom, n_pol_keys, POL_BLOOM_MAX_WORDS);
    for (auto &pm : pols) {
        Map *m = pm.second;
        PolLoc loc;
        loc.present = 1;
        uint32_t n = 0;
        for (const auto &kv : m->kv)
            n += ((uint8_t)kv.first[7] & 0xFE) == 0;
        uint32_t ns = pow2_at_least(std::max<uint64_t>(8, POL_SLOTS_PER_KEY * n));
        loc.base = (uint32_t)img->pol.size();
        loc.mask = ns - 1;
        PolSlot empty{};
        empty.key = POL_EMPTY;
        empty.ctr = EMPTY;
        img->pol.resize(img->pol.size() + ns, empty);
        PolSlot *tab = img->pol.data() + loc.base;
        for (const auto &kv : m->kv) {
            uint64_t key;
            memcpy(&key, kv.first.data(), 8);
            if (((uint8_t)kv.first[7] & 0xFE) != 0)
                continue;   // pad bits set: no datapath lookup can match it
            uint16_t proxy;
            memcpy(&proxy, kv.second.val.data(), 2);
            const uint32_t pre = pol_key_pre((uint32_t)key, (uint32_t)(key >> 32));
            uint32_t s = pol_slot(pre, loc.mask);
            while (tab[s].key != POL_EMPTY)
                s = (s + 1) & loc.mask;
            tab[s].key = key;
            bloom_add(&img->pol_bloom, pol_bloom_hash(pol_bloom_salt(loc.base), pre));
            tab[s].proxy_port = proxy;
            tab[s].ctr = (uint32_t)img->ctr_owner.size();
            img->ctr_owner.emplace_back(m, kv.first);
        }
        img->pol_loc[pm.first] = loc;
    }

    // ---- endpoints (cilium_lxc): IPv4 keys {ip4, 0 x12, family 1, 0, 0},
    //      the endpoint record inlined in the slot
    if (lxc && lxc->ksz == 20 && lxc->vsz >= 12) {
        std::vector<LxcSlot> v4;
        std::vector<Lxc6Slot> v6;
        for (const auto &kv : lxc->kv) {
            const uint8_t *k = (const uint8_t *)kv.first.data();
            const uint8_t *v = (const uint8_t *)kv.second.val.data();
            bool is_v4 = k[16] == 1 && k[17] == 0 && k[18] == 0 && k[19] == 0;
            for (int i = 4; i < 16 && is_v4; i++)
                is_v4 = k[i] == 0;
            if (!is_v4) {
                if (k[16] == 2 && k[17] == 0 && k[18] == 0 && k[19] == 0)
                    v6.push_back(lxc6_slot(img, k, (const uint8_t *)kv.second.val.data()));
                continue;
            }
            LxcSlot r{};
            memcpy(&r.addr, k, 4);
            PolLoc loc;
            r.info = lxc_info(img, v, &loc);
            r.pol_base = loc.base;
            r.pol_mask = loc.mask;
            v4.push_back(r);
        }
        // LXC_IPV4 / LXC_IP of each endpoint (the NAT46 / NAT64 addresses,
        // nat46.h:236-420): the lowest address of its family in cilium_lxc
        img->nat4.clear();
        img->nat6.clear();
        for (const LxcSlot &e : v4) {
            if (e.info & LXC_HOST)
                continue;
            const uint16_t id = (uint16_t)(e.info & 0xFFFF);
            auto it = img->nat4.find(id);
            if (it == img->nat4.end() || memcmp(&e.addr, &it->second, 4) < 0)
                img->nat4[id] = e.addr;
        }
        for (const Lxc6Slot &e : v6) {
            if (e.info & LXC_HOST)
                continue;
            const uint16_t id = (uint16_t)(e.info & 0xFFFF);
            auto it = img->nat6.find(id);
            if (it == img->nat6.end() || memcmp(e.a, &it->second, 16) < 0)
                img->nat6[id] = make_uint4(e.a[0], e.a[1], e.a[2], e.a[3]);
        }
        for (LxcSlot &e : v4)
            if (img->nat6.count((uint16_t)(e.info & 0xFFFF)))
                e.info |= LXC_HAS6;
        img->n_eps = (uint32_t)v4.size();
        if (!v4.empty()) {
            uint32_t ns = pow2_at_least(std::max<uint64_t>(8, 4ull * v4.size()));
            img->lxc4.assign(ns, LxcSlot{});
            img->lxc4_mask = ns - 1;
            for (const LxcSlot &e : v4) {
                uint32_t s = hash32(e.addr, ns - 1);
                while (img->lxc4[s].info & LXC_VALID)
                    s = (s + 1) & (ns - 1);
                img->lxc4[s] = e;
            }
        }
        img->n_eps6 = (uint32_t)v6.size();
        if (!v6.empty()) {
            uint32_t ns = pow2_at_least(std::max<uint64_t>(8, 4ull * v6.size()));
            img->lxc6.assign(ns, Lxc6Slot{});
            img->lxc6_mask = ns - 1;
            for (const Lxc6Slot &e : v6) {
                uint32_t s = l6_hash(e.a[0], e.a[1], e.a[2], e.a[3], L6_LXC_TAG) & (ns - 1);
                while (img->lxc6[s].info & LXC_VALID)
                    s = (s + 1) & (ns - 1);
                img->lxc6[s] = e;
            }
        }
    }
}

}  // namespace cfc
