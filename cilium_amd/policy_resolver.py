"""Label-selector policy -> per-endpoint policymap (MapState), restated from
the reference's userspace resolver for the rule kinds examples/policies/
{l3,l4} use.  It turns CiliumNetworkPolicy JSON into the cilium_policy_<id>
entries the datapath (and this engine) looks up; the engine itself only ever
sees the resulting map contents.

Restated (file:line in /root/reference):
  * rule selection, ingress/egress enablement   pkg/policy/repository.go:624-643
  * L3 label access (FromRequires first, then   pkg/policy/rule.go:352-440,
    FromEndpoints/FromEntities/FromCIDR...)     repository.go:80-126
  * L4 filters per port/proto, wildcard peers   pkg/policy/rule.go:115-213,
    and FromRequires folded into FromEndpoints  :227-270, :521-560,
                                                repository.go:245-283,
                                                pkg/policy/l4.go:162-200
  * MapState: L4 keys per selected identity,    pkg/endpoint/policy.go:92-129,
    localhost / world keys, L3 keys per         :143-190, :273-395
    identity (allow-all when not enabled)
  * entities -> reserved-label selectors        pkg/policy/api/entity.go:45-70
  * CIDR selectors, CIDRSet except expansion,   pkg/policy/api/cidr.go:70-132,
    CIDR identity labels                        pkg/labels/cidr.go, pkg/labels/cidr/cidr.go:33-70
  * an L7 port's filter also takes the peers    pkg/policy/repository.go:127-234
    of L3-only and L3/L4 rules (wildcardL3L4Rules)

Not restated (they need services the reference's agent talks to): toFQDNs
(DNS proxy), toServices (Kubernetes endpoints), the L7 rules' contents and
the proxy redirect (an L7 port's keys carry proxy port 0 here).  The
reference resolver is Go and this image has no Go toolchain: rule selection,
label access and L4 resolution are pinned to the reference's own
known-answer tests (pkg/policy/repository_test.go, restated as data in
tests/test_policy_repository_ref.py); the MapState step (policy.go), which
no reference test covers, is pinned to hand-derived MapStates of the
example policies; the datapath verdicts over it are pinned by the reference
BPF programs (oracle/gen_golden.py scenario c1_ingress_v4).
"""
from __future__ import annotations

import ipaddress
import json
from dataclasses import dataclass, field

# reserved identities and their labels (pkg/identity/numericidentity.go)
HOST_ID, WORLD_ID, CLUSTER_ID, HEALTH_ID, INIT_ID = 1, 2, 3, 4, 5
RESERVED = {HOST_ID: "host", WORLD_ID: "world", CLUSTER_ID: "cluster",
            HEALTH_ID: "health", INIT_ID: "init"}
LOCAL_IDENTITY_FLAG = 1 << 24      # CIDR identities are node-local
INGRESS, EGRESS = 0, 1
PROTO = {"TCP": 6, "UDP": 17}

WILDCARD = "*"                     # the selector that matches every label set


def reserved_labels(ident: int) -> frozenset:
    return frozenset({f"reserved:{RESERVED[ident]}="})


def cidr_labels(prefix: str, cluster: str = "10.0.0.0/8") -> frozenset:
    """Labels of a CIDR identity: cidr:<prefix masked to /i> for i = 0..len
    and reserved:world (reserved:cluster inside the cluster range)."""
    net = ipaddress.ip_network(prefix, strict=False)
    out = set()
    if net.prefixlen > 0:
        for i in range(net.prefixlen + 1):
            sup = net.supernet(new_prefix=i) if i < net.prefixlen else net
            out.add(f"cidr:{sup}=")
    cl = ipaddress.ip_network(cluster)
    inside = net.version == cl.version and net.subnet_of(cl) and net.prefixlen >= cl.prefixlen
    out.add("reserved:cluster=" if inside else "reserved:world=")
    return frozenset(out)


def pod_labels(d: dict) -> frozenset:
    return frozenset(f"{k}={v}" for k, v in d.items())


# ------------------------------------------------------------- selectors
@dataclass(frozen=True)
class Selector:
    """EndpointSelector: every matchLabels pair present (keys without a
    source match any source), plus extra 'requires' selectors (FromRequires
    folded in as match expressions)."""
    labels: frozenset = frozenset()
    requires: tuple = ()

    @staticmethod
    def parse(obj) -> "Selector":
        ml = (obj or {}).get("matchLabels", {}) or {}
        return Selector(frozenset(f"{k}={v}" for k, v in ml.items()))

    def matches(self, lbls: frozenset) -> bool:
        return self.labels <= lbls and all(r.matches(lbls) for r in self.requires)

    def selects_all(self) -> bool:
        return not self.labels and not self.requires


def entity_selector(e: str):
    """pkg/policy/api/entity.go:45-70 (unknown entities select nothing)."""
    if e == "all":
        return Selector()
    if e in ("world", "cluster", "host", "init"):
        return Selector(frozenset({f"reserved:{e}="}))
    return None


def cidr_rule_set(rules) -> list:
    """ComputeResultantCIDRSet: each CIDRRule's cidr minus its exceptions."""
    out = []
    for r in rules:
        nets = [ipaddress.ip_network(r["cidr"], strict=False)]
        for ex in r.get("except", []):
            e = ipaddress.ip_network(ex, strict=False)
            nxt = []
            for n in nets:   # (pkg/ip/ip.go RemoveCIDRs)
                if n.version != e.version or not n.overlaps(e):
                    nxt.append(n)
                elif e.subnet_of(n):
                    nxt.extend(n.address_exclude(e))
                # else n lies inside the exception: removed
            nets = nxt
        out.extend(str(n) for n in sorted(nets))
    return out


def cidr_selectors(cidrs) -> list:
    """CIDRSlice.GetAsEndpointSelectors (cidr.go:70-86)."""
    out, world = [], False
    for c in cidrs:
        n = ipaddress.ip_network(c, strict=False)
        if n.prefixlen == 0 and not world:
            world = True
            out.append(Selector(frozenset({"reserved:world="})))
        out.append(Selector(frozenset({f"cidr:{n}="})))
    return out


def peer_selectors(r: dict, ingress: bool) -> list:
    """GetSourceEndpointSelectors / GetDestinationEndpointSelectors."""
    p = "from" if ingress else "to"
    sel = [Selector.parse(s) for s in r.get(f"{p}Endpoints", []) or []]
    for e in r.get(f"{p}Entities", []) or []:
        s = entity_selector(e)
        if s is not None:
            sel.append(s)
    sel += cidr_selectors(r.get(f"{p}CIDR", []) or [])
    sel += cidr_selectors(cidr_rule_set(r.get(f"{p}CIDRSet", []) or []))
    return sel


def label_based(r: dict, ingress: bool) -> bool:
    """IngressRule / EgressRule IsLabelBased (api/ingress.go:120-122,
    api/egress.go:148-150): no requirements, CIDRs (or services)."""
    keys = ("fromRequires", "fromCIDR", "fromCIDRSet") if ingress else \
        ("toRequires", "toCIDR", "toCIDRSet", "toServices")
    return not any(r.get(k) for k in keys)


def rule_cidrs(r: dict, ingress: bool) -> list:
    p = "from" if ingress else "to"
    return list(r.get(f"{p}CIDR", []) or []) + cidr_rule_set(r.get(f"{p}CIDRSet", []) or [])


@dataclass
class Rule:
    selector: Selector
    ingress: list = field(default_factory=list)
    egress: list = field(default_factory=list)
    name: str = ""


def parse_rules(objs, origin="") -> list:
    rules = []
    for r in objs:
        name = ",".join(f"{x['key']}={x['value']}" for x in r.get("labels", []))
        rules.append(Rule(Selector.parse(r.get("endpointSelector")),
                          r.get("ingress", []) or [], r.get("egress", []) or [],
                          name or origin))
    return rules


def load_rules(paths) -> list:
    """Rules from policy JSON files (each a list of rules)."""
    out = []
    for p in paths:
        out += parse_rules(json.load(open(p)), p)
    return out


def load_fixture(path) -> list:
    """Rules from tests/golden/c1_policies.json ({file: [rules]}, sorted)."""
    d = json.load(open(path))
    out = []
    for k in sorted(d):
        out += parse_rules(d[k], k)
    return out


# ------------------------------------------------------------- repository
class Repository:
    def __init__(self, rules, always_allow_localhost=True, host_allows_world=True):
        # k8s mode defaults: AllowLocalhost auto -> always, legacy
        # host-allows-world (daemon/daemon.go:1136-1147)
        self.rules = list(rules)
        self.always_allow_localhost = always_allow_localhost
        self.host_allows_world = host_allows_world

    def cidrs(self) -> list:
        """Every CIDR the rules name (the prefixes the agent allocates CIDR
        identities and ipcache entries for)."""
        out = []
        for r in self.rules:
            for x in r.ingress:
                out += rule_cidrs(x, True)
            for x in r.egress:
                out += rule_cidrs(x, False)
        return sorted(set(out), key=lambda c: (ipaddress.ip_network(c).network_address,
                                               ipaddress.ip_network(c).prefixlen))

    def enabled(self, lbls):
        """GetRulesMatching (repository.go:624-643)."""
        ing = any(r.selector.matches(lbls) and len(r.ingress) > 0 for r in self.rules)
        eg = any(r.selector.matches(lbls) and len(r.egress) > 0 for r in self.rules)
        return ing, eg

    def _can_reach(self, subject, peer, ingress) -> bool:
        """AllowsIngress/EgressLabelAccess (repository.go:80-126, rule.go:352-440)."""
        decision = None
        req_key = "fromRequires" if ingress else "toRequires"
        for r in self.rules:
            if not r.selector.matches(subject):
                continue
            sect = r.ingress if ingress else r.egress
            denied = any(not Selector.parse(s).matches(peer)
                         for x in sect for s in x.get(req_key, []) or [])
            if denied:
                return False
            for x in sect:
                if any(s.matches(peer) for s in peer_selectors(x, ingress)) and \
                        not (x.get("toPorts") or []):
                    decision = True
                    break
        return bool(decision)

    def _l4(self, subject, ingress) -> dict:
        """ResolveL4Ingress/EgressPolicy: {(port, proto): [selectors] | WILDCARD}."""
        req_key = "fromRequires" if ingress else "toRequires"
        ep_key = "fromEndpoints" if ingress else "toEndpoints"
        reqs = []
        for r in self.rules:
            if r.selector.matches(subject):
                for x in (r.ingress if ingress else r.egress):
                    reqs += [Selector.parse(s) for s in x.get(req_key, []) or []]
        res, l7 = {}, set()

        def add(k, sel, wild):
            cur = res.get(k, [])
            if wild or cur == WILDCARD:
                res[k] = WILDCARD
            else:
                res[k] = cur + [s for s in sel if s not in cur]

        def keys_of(pr):
            for p in pr.get("ports", []) or []:
                protos = [p.get("protocol", "ANY").upper()]
                if protos[0] == "ANY":
                    protos = ["TCP", "UDP"]
                for proto in protos:
                    yield (int(p["port"]), PROTO[proto])
        for r in self.rules:
            if not r.selector.matches(subject):
                continue
            for x in (r.ingress if ingress else r.egress):
                if not (x.get("toPorts") or []):
                    continue
                sel = peer_selectors(x, ingress)
                if reqs:   # requirements join each From/ToEndpoints selector
                    n_ep = len(x.get(ep_key, []) or [])
                    sel = [Selector(s.labels, s.requires + tuple(reqs)) if i < n_ep else s
                           for i, s in enumerate(sel)]
                wild = not sel or any(s.selects_all() for s in sel)
                for pr in x["toPorts"]:
                    for k in keys_of(pr):
                        add(k, sel, wild)
                        if pr.get("rules"):   # (an L7 parser on the port)
                            l7.add(k)
        # wildcardL3L4Rules (repository.go:166-234, wildcardL3L4Rule :127-164):
        # a port with L7 rules also takes, with allow-all L7 rules, the peers
        # of the label-based L3-only rules (every such port of TCP and UDP)
        # and of the L3/L4 rules without L7 rules on the same port — they
        # become L4 keys (the reference redirects them to its proxy)
        if l7:
            for r in self.rules:
                if not r.selector.matches(subject):
                    continue
                for x in (r.ingress if ingress else r.egress):
                    if not label_based(x, ingress):
                        continue
                    sel = peer_selectors(x, ingress)
                    wild = any(s.selects_all() for s in sel)
                    tps = x.get("toPorts") or []
                    if not tps:
                        targets = [k for k in l7 if k[1] in (6, 17)]
                    else:
                        targets = [k for pr in tps if not pr.get("rules")
                                   for k in keys_of(pr) if k in l7]
                    for k in targets:
                        if sel:
                            add(k, sel, wild)
        return res

    def map_state(self, subject: frozenset, identities: dict) -> dict:
        """computeDesiredPolicyMapState (pkg/endpoint/policy.go:273-395):
        {(identity, dport host-order, proto, direction): proxy_port}."""
        ing, eg = self.enabled(subject)
        keys = {}
        for d, on in ((INGRESS, ing), (EGRESS, eg)):
            if not on:
                continue
            for (port, proto), sel in self._l4(subject, d == INGRESS).items():
                for ident, lbls in identities.items():
                    if sel == WILDCARD or any(s.matches(lbls) for s in sel):
                        keys[(ident, port, proto, d)] = 0
        if self.always_allow_localhost:
            keys[(HOST_ID, 0, 0, INGRESS)] = 0
            if self.host_allows_world:
                keys[(WORLD_ID, 0, 0, INGRESS)] = 0
        for ident, lbls in identities.items():
            if not ing or self._can_reach(subject, lbls, True):
                keys[(ident, 0, 0, INGRESS)] = 0
            if not eg or self._can_reach(subject, lbls, False):
                keys[(ident, 0, 0, EGRESS)] = 0
        return keys


def identity_cache(pods: dict, cidr_ids: dict) -> dict:
    """The resolver's identity -> labels cache: reserved identities, pod
    identities and CIDR identities."""
    out = {i: reserved_labels(i) for i in RESERVED}
    out.update(pods)
    out.update(cidr_ids)
    return out
