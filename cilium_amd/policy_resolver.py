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
  * Rule.Sanitize (the errors a rule is         pkg/policy/api/rule_validation.go
    refused with) and net.ParseCIDR / ParseIP
  * the CIDR policy and its prefix-length       pkg/policy/rule.go:279-345,
    counts (class masks for bare addresses)     l3.go:66-96, repository.go:340-353

  * rule management: Add (sanitized),          pkg/policy/repository.go:
    SearchRLocked, DeleteByLabels,              495-586
    ContainsAllRLocked, the revision
  * endpoint selectors: matchLabels and        pkg/policy/api/selector.go:
    matchExpressions (In, NotIn, Exists,        162-175, 277-300
    DoesNotExist); unconvertible ones match
    nothing
  * L4 filters with their L7 parser and L7     pkg/policy/l4.go:52-223,
    rules per peer selector, merge conflicts    rule.go:36-141

Not restated (they need services the reference's agent talks to): toFQDNs
(DNS proxy), toServices (Kubernetes endpoints), the evaluation of L7 rules
and the proxy redirect (an L7 port's keys carry proxy port 0 here).  The
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
_SEL_OPS = ("In", "NotIn", "Exists", "DoesNotExist")


@dataclass(frozen=True)
class Selector:
    """EndpointSelector (pkg/policy/api/selector.go): every matchLabels pair
    present (keys without a source match any source), every
    matchExpressions requirement (k8s In / NotIn / Exists / DoesNotExist),
    plus extra 'requires' selectors (FromRequires folded in as match
    expressions).  A selector k8s refuses to convert (an unknown operator,
    In / NotIn without values, Exists / DoesNotExist with values) matches
    nothing, as EndpointSelector.Matches does when its requirements are nil
    (selector.go:162-175, 277-288)."""
    labels: frozenset = frozenset()
    requires: tuple = ()
    exprs: tuple = ()          # ((key, operator, frozenset(values)), ...)
    invalid: bool = False

    @staticmethod
    def _key(k: str) -> str:
        """A selector key's source: pod labels here are the k8s source's,
        so `k8s:` and `any:` keys match them plainly (labels.ParseSelectLabel:
        no source is `any`); `reserved:` and other sources stay."""
        for src in ("k8s:", "any:"):
            if k.startswith(src):
                return k[len(src):]
        return k

    @staticmethod
    def parse(obj) -> "Selector":
        ml = (obj or {}).get("matchLabels", {}) or {}
        exprs, invalid = [], False
        for e in (obj or {}).get("matchExpressions", []) or []:
            op, vals = e.get("operator"), tuple(e.get("values") or ())
            if op not in _SEL_OPS or (op in ("In", "NotIn")) != bool(vals):
                invalid = True
            exprs.append((Selector._key(e.get("key", "")), op, frozenset(vals)))
        return Selector(frozenset(f"{Selector._key(k)}={v}" for k, v in ml.items()), (),
                        tuple(sorted(exprs, key=lambda x: (x[0], str(x[1]), sorted(x[2])))),
                        invalid)

    @staticmethod
    def _expr(lbls: frozenset, key: str, op: str, vals: frozenset) -> bool:
        present = {lb.split("=", 1)[1] for lb in lbls if lb.split("=", 1)[0] == key}
        if op == "In":
            return bool(present & vals)
        if op == "NotIn":
            return not (present & vals)
        if op == "Exists":
            return bool(present)
        return not present   # DoesNotExist

    def matches(self, lbls: frozenset) -> bool:
        if self.invalid:
            return False
        if "reserved:all=" in self.labels:   # (selector.go:290-294: matches all,
            return True                       # yet is no wildcard selector)
        return (self.labels <= lbls and
                all(self._expr(lbls, *e) for e in self.exprs) and
                all(r.matches(lbls) for r in self.requires))

    def selects_all(self) -> bool:
        return not self.labels and not self.requires and not self.exprs and not self.invalid


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
    labels: frozenset = frozenset()   # the rule's LabelArray: (source, key, value)


def rule_labels(r: dict) -> frozenset:
    """api.Rule.Labels as a set of (source, key, value)."""
    return frozenset((x.get("source", ""), x.get("key", ""), x.get("value", ""))
                     for x in r.get("labels", []) or [])


def parse_rules(objs, origin="", sanitize=True) -> list:
    """api.Rules -> the repository's rules, each checked by Rule.Sanitize
    first (PolicyError), as the agent's policy import does."""
    rules = []
    for r in objs:
        if sanitize:
            sanitize_rule(r)
        name = ",".join(f"{x['key']}={x['value']}" for x in r.get("labels", []))
        rules.append(Rule(Selector.parse(r.get("endpointSelector")),
                          r.get("ingress", []) or [], r.get("egress", []) or [],
                          name or origin, rule_labels(r)))
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


# ------------------------------------------------------------- validation
class PolicyError(ValueError):
    """An error of Rule.Sanitize (pkg/policy/api/rule_validation.go): the
    rule is refused before it reaches the repository."""


MAX_PORTS = 40                  # rule_validation.go:27
MAX_CIDR_PREFIX_LENGTHS = 40    # :29
L4_PROTOS = ("TCP", "UDP", "ANY")


def go_parse_ip(s: str):
    """net.ParseIP: a dotted IPv4 address or an IPv6 address (no zone, no
    mask) -> ipaddress object, or None."""
    if not isinstance(s, str) or "%" in s or "/" in s:
        return None
    try:
        return ipaddress.ip_address(s)
    except ValueError:
        return None


def go_parse_cidr(s: str):
    """net.ParseCIDR: <address>/<decimal prefix length within the family's
    bits> -> the network (host bits cleared), or None.  (No netmask
    notation: Go reads the part after '/' as a decimal length only.)"""
    if not isinstance(s, str):
        return None
    addr, sep, plen = s.partition("/")
    if not sep or not plen or not all("0" <= ch <= "9" for ch in plen):
        return None
    ip = go_parse_ip(addr)
    if ip is None or int(plen) > (32 if ip.version == 4 else 128):
        return None
    return ipaddress.ip_network(f"{addr}/{int(plen)}", strict=False)


def parse_port(port) -> int:
    """PortProtocol.sanitize's port (rule_validation.go:309-321):
    strconv.ParseUint(port, 0, 16) — decimal, 0x hex or 0 octal — not 0."""
    t = str(port) if port is not None else ""
    if t == "":
        raise PolicyError("Port must be specified")
    base, digits = 10, t
    if t[:2] in ("0x", "0X"):
        base, digits = 16, t[2:]
    elif len(t) > 1 and t[0] == "0":
        base, digits = 8, t[1:]
    ok = "0123456789abcdef"[:base]
    if not digits or any(ch.lower() not in ok for ch in digits) or int(digits, base) > 0xFFFF:
        raise PolicyError(f"Unable to parse port: {t}")
    v = int(digits, base)
    if v == 0:
        raise PolicyError("Port cannot be 0")
    return v


def parse_l4_proto(proto) -> str:
    """ParseL4Proto (api/utils.go:103-110): upper-cased, empty is ANY."""
    p = (proto or "").upper()
    if p == "":
        return "ANY"
    if p not in L4_PROTOS:   # L4Proto.Validate (utils.go:92-100)
        raise PolicyError(f'invalid protocol "{p}", must be {{ tcp | udp | any }}')
    return p


def cidr_sanitize(c) -> int:
    """CIDR.sanitize (rule_validation.go:333-356): a prefix, or a bare
    address (prefix length 0 returned)."""
    if not c:
        raise PolicyError("IP must be specified")
    n = go_parse_cidr(c)
    if n is not None:
        return n.prefixlen
    if go_parse_ip(c) is None:
        raise PolicyError(f"Unable to parse CIDR: {c}")
    return 0


def cidr_rule_sanitize(r: dict) -> int:
    """CIDRRule.sanitize (rule_validation.go:361-395): <address>/<prefix>
    only, every exception's address inside it (same family)."""
    n = go_parse_cidr(r.get("cidr", ""))
    if n is None:
        raise PolicyError(f"Unable to parse CIDRRule {r.get('cidr', '')!r}")
    for ex in r.get("except", []) or []:
        e = go_parse_cidr(ex)
        if e is None:
            raise PolicyError(f"invalid CIDR address: {ex}")
        if e.version != n.version or e.network_address not in n:
            raise PolicyError(f"allow CIDR prefix {r['cidr']} does not contain "
                              f"exclude CIDR prefix {ex}")
    return n.prefixlen


def _l7_sanitize(rules: dict):
    """L7Rules.sanitize (rule_validation.go:248-285): HTTP method / path
    regular expressions compile (Python's re stands in for Go's RE2), key
    / value rules need a parser and no empty key (l7.go:27-33), one L7 type
    per rule.  (Kafka: API key and role exclusive; the key / role tables
    are not restated.)"""
    import re
    n = 0
    if rules.get("http") is not None:
        n += 1
        for h in rules["http"]:
            for f in ("path", "method"):
                if h.get(f):
                    try:
                        re.compile(h[f])
                    except re.error as e:
                        raise PolicyError(str(e)) from None
    if rules.get("kafka") is not None:
        n += 1
        for k in rules["kafka"]:
            if k.get("apiKey") and k.get("role"):
                raise PolicyError(f"Cannot set both Role:{k['role']!r} and "
                                  f"APIKey :{k['apiKey']!r} together")
    if rules.get("l7") is not None and not rules.get("l7proto"):
        raise PolicyError("'l7' may only be specified when a 'l7proto' is also specified")
    if rules.get("l7proto"):
        n += 1
        for kv in rules.get("l7") or []:
            if any(k == "" for k in kv):
                raise PolicyError("Empty key not allowed")
    if n > 1:
        raise PolicyError("multiple L7 protocol rule types specified in single rule")


def _l7_empty(rules) -> bool:
    """L7Rules.IsEmpty (api/l4.go:97-99)."""
    return not rules or all(rules.get(k) is None for k in ("http", "kafka", "l7"))


def _port_rule_sanitize(pr: dict):
    """PortRule.sanitize (rule_validation.go:287-307)."""
    ports = pr.get("ports", []) or []
    if len(ports) > MAX_PORTS:
        raise PolicyError(f"too many ports, the max is {MAX_PORTS}")
    l7 = not _l7_empty(pr.get("rules"))
    for p in ports:
        parse_port(p.get("port"))
        proto = parse_l4_proto(p.get("protocol"))
        if l7 and proto != "TCP":
            raise PolicyError(f"L7 rules can only apply exclusively to TCP, not {proto}")
    if l7:
        _l7_sanitize(pr["rules"])


_L3_MEMBERS = {True: (("fromEndpoints", True), ("fromCIDR", False), ("fromCIDRSet", False),
                      ("fromEntities", True)),
               False: (("toCIDR", True), ("toCIDRSet", True), ("toEndpoints", True),
                       ("toEntities", True), ("toServices", True), ("toFQDNs", True))}


def _direction_sanitize(x: dict, ingress: bool):
    """IngressRule / EgressRule .sanitize (rule_validation.go:67-198)."""
    members = [(k, l4ok) for k, l4ok in _L3_MEMBERS[ingress] if x.get(k)]
    if len(members) > 1:
        raise PolicyError(f"Combining {members[0][0]} and {members[1][0]} is not supported yet")
    tps = x.get("toPorts") or []
    for k, l4ok in members:
        if tps and not l4ok:
            raise PolicyError(f"Combining {k} and ToPorts is not supported yet")
    for pr in tps:
        _port_rule_sanitize(pr)
    p = "from" if ingress else "to"
    lengths = {cidr_sanitize(c) for c in x.get(f"{p}CIDR", []) or []}
    lengths |= {cidr_rule_sanitize(c) for c in x.get(f"{p}CIDRSet", []) or []}
    for e in x.get(f"{p}Entities", []) or []:
        if entity_selector(e) is None:
            raise PolicyError(f"unsupported entity: {e}")
    if len(lengths) > MAX_CIDR_PREFIX_LENGTHS:
        raise PolicyError(f"too many {'ingress' if ingress else 'egress'} CIDR prefix lengths "
                          f"{len(lengths)}/{MAX_CIDR_PREFIX_LENGTHS}")


def sanitize_rule(r: dict):
    """Rule.Sanitize (rule_validation.go:37-65): raises PolicyError."""
    for lb in r.get("labels", []) or []:
        if lb.get("source") == "cilium-generated":
            raise PolicyError("rule labels cannot have cilium-generated source")
    if r.get("endpointSelector") is None:
        raise PolicyError("rule cannot have nil EndpointSelector")
    for x in r.get("ingress", []) or []:
        _direction_sanitize(x, True)
    for x in r.get("egress", []) or []:
        _direction_sanitize(x, False)


def cidr_policy_key(c: str):
    """CIDRPolicyMap.Insert's prefix (pkg/policy/l3.go:66-96): a prefix as
    given, or a bare address with its class mask (/8, /16, /24) when the
    bits after it are zero, else the full mask -> (key, family, length)."""
    n = go_parse_cidr(c)
    if n is None:
        ip = go_parse_ip(c)
        if ip is None:
            raise PolicyError(f"Unable to parse CIDR: {c}")
        if ip.version == 6 and ip.ipv4_mapped is not None:
            ip = ip.ipv4_mapped   # (ip.To4())
        if ip.version == 6:
            n = ipaddress.ip_network(f"{ip}/128")
        else:
            b0 = int(ip) >> 24   # net.IP.DefaultMask
            cls = 8 if b0 < 0x80 else 16 if b0 < 0xC0 else 24
            m = ipaddress.ip_network(f"{ip}/{cls}", strict=False)
            n = m if m.network_address == ip else ipaddress.ip_network(f"{ip}/32")
    return f"{n.network_address}/{n.prefixlen}", n.version, n.prefixlen


# ------------------------------------------------------------- L4 filters
WILDCARD_SELECTOR = Selector()   # api.WildcardEndpointSelector


def _selects_all(sels) -> bool:
    """EndpointSelectorSlice.SelectsAllEndpoints (api/selector.go:356-369)."""
    return not sels or any(s.selects_all() for s in sels)


def _l7_len(rules) -> int:
    """L7Rules.Len."""
    return sum(len(rules.get(k) or []) for k in ("http", "kafka", "l7"))


def _l7_norm(rules) -> dict:
    """An L7Rules value: {http, kafka, l7: list or None (Go nil), l7proto}."""
    r = rules or {}
    return {"http": list(r["http"]) if r.get("http") is not None else None,
            "kafka": list(r["kafka"]) if r.get("kafka") is not None else None,
            "l7proto": r.get("l7proto") or "",
            "l7": list(r["l7"]) if r.get("l7") is not None else None}


@dataclass
class L4Filter:
    """L4Filter (pkg/policy/l4.go:52-73) without its rule labels: the peers
    (endpoints; the wildcard selector when it selects all), the L7 parser
    ("" for ParserTypeNone) and the L7 rules per peer selector (L7DataMap,
    keyed by selector value — the Go map's key is the selector struct, so
    the reference's tests, which reuse one selector variable, key it the
    same way)."""
    port: int
    proto: int
    endpoints: list
    parser: str = ""
    l7: dict = field(default_factory=dict)
    derived: list = field(default_factory=list)   # DerivedFromRules: rule labels

    def allows_all(self) -> bool:
        """AllowsAllAtL3 (l4.go:112-114)."""
        return _selects_all(self.endpoints)

    def merge(self, new: "L4Filter", peers):
        """mergeL4Port (rule.go:36-108)."""
        if self.allows_all() or new.allows_all():
            self.endpoints = [WILDCARD_SELECTOR]
        else:
            self.endpoints = self.endpoints + list(peers)
        if new.parser:
            if not self.parser:
                self.parser = new.parser
            elif new.parser != self.parser:
                raise PolicyError(f"Cannot merge conflicting L7 parsers "
                                  f"({new.parser}/{self.parser})")
        for sel, nr in new.l7.items():
            ep = self.l7.get(sel)
            if ep is None:
                self.l7[sel] = _l7_norm(nr)
                continue
            if nr["http"]:
                if ep["kafka"] or ep["l7proto"]:
                    raise PolicyError("Cannot merge conflicting L7 rule types")
                ep["http"] = (ep["http"] or []) + [x for x in nr["http"]
                                                    if x not in (ep["http"] or [])]
            elif nr["kafka"]:
                if ep["http"] or ep["l7proto"]:
                    raise PolicyError("Cannot merge conflicting L7 rule types")
                ep["kafka"] = (ep["kafka"] or []) + [x for x in nr["kafka"]
                                                      if x not in (ep["kafka"] or [])]
            elif nr["l7proto"]:
                if ep["kafka"] or ep["http"] or (ep["l7proto"] and ep["l7proto"] != nr["l7proto"]):
                    raise PolicyError("Cannot merge conflicting L7 rule types")
                ep["l7proto"] = ep["l7proto"] or nr["l7proto"]
                ep["l7"] = (ep["l7"] or []) + [x for x in (nr["l7"] or [])
                                                if x not in (ep["l7"] or [])]

    def wildcard_l7(self, peers, rlabels=frozenset()):
        """wildcardL3L4Rule's body (repository.go:127-164): the peers allowed
        at every L7 resource of the parser, and added to the filter."""
        for sel in peers:
            if self.parser == "http":
                self.l7[sel] = _l7_norm({"http": [{}]})
            elif self.parser == "kafka":
                self.l7[sel] = _l7_norm({"kafka": [{}]})
            else:
                self.l7[sel] = _l7_norm({"l7proto": self.parser, "l7": []})
        self.endpoints = self.endpoints + list(peers)
        self.derived.append(rlabels)


# ------------------------------------------------------------- repository
class Repository:
    def __init__(self, rules, always_allow_localhost=True, host_allows_world=True):
        # k8s mode defaults: AllowLocalhost auto -> always, legacy
        # host-allows-world (daemon/daemon.go:1136-1147)
        self.rules = list(rules)
        self.always_allow_localhost = always_allow_localhost
        self.host_allows_world = host_allows_world
        self.revision = 1   # NewPolicyRepository (repository.go)

    # ---- the repository's rule management (repository.go:495-586)
    def add(self, r: dict) -> int:
        """Add: Rule.Sanitize, then AddListLocked -> the new revision;
        PolicyError (the revision unchanged) for a refused rule."""
        self.rules += parse_rules([r])
        self.revision += 1
        return self.revision

    def search(self, lbls) -> list:
        """SearchRLocked: the rules whose labels contain all of `lbls`."""
        need = frozenset(lbls)
        return [r for r in self.rules if need <= r.labels]

    def delete_by_labels(self, lbls) -> tuple:
        """DeleteByLabelsLocked -> (revision, deleted): the revision moves
        only when a rule went."""
        need = frozenset(lbls)
        keep = [r for r in self.rules if not need <= r.labels]
        n = len(self.rules) - len(keep)
        if n:
            self.rules = keep
            self.revision += 1
        return self.revision, n

    def contains_all(self, needed) -> bool:
        """ContainsAllRLocked: every label array of `needed` holds all the
        labels of some rule that has labels."""
        return all(any(r.labels and r.labels <= frozenset(n) for r in self.rules)
                   for n in needed)

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

    def cidr_policy(self, subject) -> dict:
        """ResolveCIDRPolicy (repository.go:340-353, rule.go:279-345): the
        CIDR prefixes of the rules selecting `subject` — ingress L3-only
        rules (CIDR + L4 is mergeL4Ingress's), egress every rule — with the
        per-family prefix-length counts that size the datapath's prefix
        list: {"ingress"|"egress": {"map": {key: (family, length)},
        "v4": {length: n}, "v6": {length: n}, "derived": {key: [the labels
        of each rule that named it]}}}."""
        out = {}
        for d, ingress in (("ingress", True), ("egress", False)):
            m, cnt, derived = {}, {4: {}, 6: {}}, {}
            for r in self.rules:
                if not r.selector.matches(subject):
                    continue
                for x in (r.ingress if ingress else r.egress):
                    cs = rule_cidrs(x, ingress)
                    if ingress and cs and (x.get("toPorts") or []):
                        continue
                    for c in cs:
                        key, fam, ln = cidr_policy_key(c)
                        if key not in m:
                            m[key] = (fam, ln)
                            cnt[fam][ln] = cnt[fam].get(ln, 0) + 1
                        derived.setdefault(key, []).append(r.labels)   # (DerivedFromRules)
            out[d] = {"map": m, "v4": cnt[4], "v6": cnt[6], "derived": derived}
        return out

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

    def l4_filters(self, subject, ingress, wildcard_l3l4=True) -> dict:
        """ResolveL4IngressPolicy / ResolveL4EgressPolicy (repository.go:
        245-330): {(port, proto): L4Filter}, every rule selecting `subject`
        merged port by port (rule.go:36-141 mergeL4Port, :227-270; l4.go:
        143-223 CreateL4Filter / CreateL4IngressFilter), FromRequires /
        ToRequires joined into each From/ToEndpoints selector, then the L7
        wildcarding of label-based L3-only and L3/L4 peers
        (wildcardL3L4Rules, repository.go:127-234) unless `wildcard_l3l4`
        is False (a single rule's resolveL4*Policy).  Conflicting L7 parsers
        or rule types on one port raise PolicyError, as the Go call returns
        its error."""
        req_key = "fromRequires" if ingress else "toRequires"
        ep_key = "fromEndpoints" if ingress else "toEndpoints"
        reqs = []
        for r in self.rules:
            if r.selector.matches(subject):
                for x in (r.ingress if ingress else r.egress):
                    reqs += [Selector.parse(s) for s in x.get(req_key, []) or []]
        res = {}
        for r in self.rules:
            if not r.selector.matches(subject):
                continue
            for x in (r.ingress if ingress else r.egress):
                if not (x.get("toPorts") or []):
                    continue
                peers = peer_selectors(x, ingress)
                if reqs:   # requirements join each From/ToEndpoints selector
                    n_ep = len(x.get(ep_key, []) or [])
                    peers = [Selector(s.labels, s.requires + tuple(reqs), s.exprs, s.invalid)
                             if i < n_ep else s
                             for i, s in enumerate(peers)]
                for pr in x["toPorts"]:
                    for p in pr.get("ports", []) or []:
                        port = parse_port(p.get("port"))
                        pn = parse_l4_proto(p.get("protocol"))
                        for proto in (("TCP", "UDP") if pn == "ANY" else (pn,)):
                            f = self._create_filter(peers, pr, port, proto, ingress)
                            f.derived = [r.labels]
                            k = (port, PROTO[proto])
                            if k in res:
                                res[k].merge(f, peers)
                                res[k].derived.append(r.labels)
                            else:
                                res[k] = f
        if wildcard_l3l4 and any(f.parser for f in res.values()):
            for r in self.rules:
                if not r.selector.matches(subject):
                    continue
                for x in (r.ingress if ingress else r.egress):
                    if not label_based(x, ingress):
                        continue
                    peers = peer_selectors(x, ingress)
                    tps = x.get("toPorts") or []
                    if not tps:    # L3-only: every port of TCP and UDP
                        targets = [("TCP", 0), ("UDP", 0)]
                    else:          # L3/L4-only ports (an ANY port matches no filter)
                        targets = [(parse_l4_proto(p.get("protocol")), parse_port(p.get("port")))
                                   for pr in tps if _l7_empty(pr.get("rules"))
                                   for p in pr.get("ports", []) or []]
                    for proto, port in targets:
                        for (fp, fpr), f in res.items():
                            if PROTO.get(proto) == fpr and (port == 0 or port == fp) and f.parser:
                                f.wildcard_l7(peers, r.labels)
        return res

    def _create_filter(self, peers, pr, port, proto, ingress) -> "L4Filter":
        """CreateL4Filter (l4.go:162-200) and, ingress, CreateL4IngressFilter
        (:209-223): the host (and world) selectors wildcarded at L7 when the
        port rule has L7 rules and localhost is always allowed."""
        f = L4Filter(port, PROTO[proto],
                     [WILDCARD_SELECTOR] if _selects_all(peers) else list(peers))
        rules = pr.get("rules")
        if proto == "TCP" and rules is not None:
            f.parser = ("http" if rules.get("http") else "kafka" if rules.get("kafka")
                        else rules.get("l7proto") or "")
            if not _l7_empty(rules) and _l7_len(rules) > 0:   # addRulesForEndpoints
                for s in f.endpoints:
                    f.l7[s] = _l7_norm(rules)
        if ingress and not _l7_empty(rules) and self.always_allow_localhost:
            f.l7[entity_selector("host")] = _l7_norm({})
            if self.host_allows_world:
                f.l7[entity_selector("world")] = _l7_norm({})
        return f

    def _l4(self, subject, ingress) -> dict:
        """The L4 filters' peers: {(port, proto): [selectors] | WILDCARD}."""
        out = {}
        for k, f in self.l4_filters(subject, ingress).items():
            if f.allows_all():
                out[k] = WILDCARD
            else:
                out[k] = []
                for s_ in f.endpoints:
                    if s_ not in out[k]:
                        out[k].append(s_)
        return out

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
