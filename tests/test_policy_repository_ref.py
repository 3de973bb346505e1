"""The C1 resolver (cilium_amd/policy_resolver.py) against the reference
resolver's own known-answer tests, pkg/policy/repository_test.go,
rule_test.go, cidr_test.go and api/{entity,cidr,rule_validation}_test.go:
the same rules, the same label contexts, the answers the Go tests assert
(a Go error is a PolicyError).  The Go
code cannot run here (no Go toolchain); these cases are its expected values,
restated as data.

Mapping: a Go label "foo" / "id=foo" (labels.ParseSelectLabel: source any)
is the resolver's "foo=" / "id=foo"; api.Rule is the CiliumNetworkPolicy
JSON shape the resolver reads.  AllowsIngress/EgressRLocked without ports is
the label verdict (CanReach), `Repository._can_reach`; ResolveL4*Policy is
`Repository._l4` (port/proto -> peer selectors; the Go L4Filter's
Endpoints as a set — the Go list repeats selectors that several rules add,
which its test comments call an artifact — and without the L7 rule
contents, which the resolver does not restate).  One difference is the
API's, not the datapath's: the Go call answers Denied for an endpoint no
rule selects, while that endpoint's policymap allows every identity
(pkg/endpoint/policy.go: policy enforcement off), which is what the resolver
computes; those cases check `enabled`."""
import pytest

from cilium_amd import policy_resolver as R


def lab(s):
    """a Go label string -> the resolver's: the k8s / any sources dropped
    (selectors without a source match any), reserved: kept"""
    for src in ("k8s:", "any:"):
        if s.startswith(src):
            s = s[len(src):]
    k, _, v = s.partition("=")
    return f"{k}={v}"


def lbls(*xs):
    return frozenset(lab(x) for x in xs)


def es(*xs):
    return {"matchLabels": {lab(x).split("=", 1)[0]: lab(x).split("=", 1)[1] for x in xs}}


def sel(*xs):
    return R.Selector(lbls(*xs))


def repo(*rules):
    return R.Repository(R.parse_rules(list(rules)))


def tcp(port, rules=None):
    pr = {"ports": [{"port": str(port), "protocol": "TCP"}]}
    if rules:
        pr["rules"] = rules
    return [pr]


def ingress_allowed(rp, frm, to):
    """AllowsIngressRLocked (label verdict); None: no rule selects `to`"""
    if not rp.enabled(to)[0]:
        return None
    return rp._can_reach(to, frm, True)


def egress_allowed(rp, frm, to):
    if not rp.enabled(frm)[1]:
        return None
    return rp._can_reach(frm, to, False)


def l4_sets(d):
    return {k: (v if v == R.WILDCARD else frozenset(v)) for k, v in d.items()}


def test_can_reach_ingress():
    # repository_test.go:193-285
    assert ingress_allowed(repo(), lbls("foo"), lbls("bar")) is None   # no rules: Denied
    rp = repo({"endpointSelector": es("bar"), "ingress": [{"fromEndpoints": [es("foo")]}]},
              {"endpointSelector": es("groupA"), "ingress": [{"fromRequires": [es("groupA")]}]},
              {"endpointSelector": es("bar2"), "ingress": [{"fromEndpoints": [es("foo")]}]})
    assert ingress_allowed(rp, lbls("foo"), lbls("bar")) is True
    assert ingress_allowed(rp, lbls("foo"), lbls("bar2")) is True
    assert ingress_allowed(rp, lbls("foo", "groupA"), lbls("bar", "groupA")) is True
    assert ingress_allowed(rp, lbls("foo", "groupB"), lbls("bar", "groupA")) is False
    assert ingress_allowed(rp, lbls("foo", "groupB"), lbls("bar", "groupB")) is True
    # foo => bar3, no rule: Denied by the API; bar3's map allows all
    assert ingress_allowed(rp, lbls("foo"), lbls("bar3")) is None


def test_can_reach_egress():
    # repository_test.go:287-383
    assert egress_allowed(repo(), lbls("foo"), lbls("bar")) is None
    rp = repo({"endpointSelector": es("foo"), "egress": [{"toEndpoints": [es("bar")]}]},
              {"endpointSelector": es("groupA"), "egress": [{"toRequires": [es("groupA")]}]},
              {"endpointSelector": es("foo"), "egress": [{"toEndpoints": [es("bar2")]}]})
    assert egress_allowed(rp, lbls("foo"), lbls("bar")) is True
    assert egress_allowed(rp, lbls("foo"), lbls("bar2")) is True
    assert egress_allowed(rp, lbls("foo", "groupA"), lbls("bar", "groupA")) is True
    assert egress_allowed(rp, lbls("bar", "groupA"), lbls("foo", "groupB")) is False
    assert egress_allowed(rp, lbls("foo", "groupB"), lbls("bar", "groupB")) is True
    assert egress_allowed(rp, lbls("foo"), lbls("bar3")) is False


def test_minikube_getting_started():
    # repository_test.go:1313-1453: app1 admits app2 on 80/TCP (three rules,
    # two with HTTP rules); app3 has no L4 access, neither has L3 access
    http = {"http": [{"method": "GET", "path": "/"}]}
    rp = repo(*[{"endpointSelector": es("id=app1"),
                 "ingress": [{"fromEndpoints": [es("id=app2")], "toPorts": tcp(80, r)}]}
                for r in (None, http, http)])
    assert l4_sets(rp._l4(lbls("id=app1"), True)) == {(80, 6): frozenset({sel("id=app2")})}
    assert ingress_allowed(rp, lbls("id=app2"), lbls("id=app1")) is False
    assert ingress_allowed(rp, lbls("id=app3"), lbls("id=app1")) is False
    ms = rp.map_state(lbls("id=app1"), {1000: lbls("id=app2"), 1001: lbls("id=app3")})
    assert (1000, 80, 6, R.INGRESS) in ms and (1001, 80, 6, R.INGRESS) not in ms
    assert (1000, 0, 0, R.INGRESS) not in ms and (1001, 0, 0, R.INGRESS) not in ms


def test_l3_dependent_l4_from_requires():
    # repository_test.go:685-808: FromRequires / ToRequires joins each
    # From/ToEndpoints selector of the endpoint's L4 rules
    for ingress in (True, False):
        d, peers, req = (("ingress", "fromEndpoints", "fromRequires") if ingress else
                         ("egress", "toEndpoints", "toRequires"))
        rp = repo({"endpointSelector": es("id=foo"),
                   d: [{peers: [es("id=bar1")], "toPorts": tcp(80)}, {req: [es("id=bar2")]}]})
        want = R.Selector(lbls("id=bar1"), (sel("id=bar2"),))
        assert rp._l4(lbls("id=foo"), ingress) == {(80, 6): [want]}
        # (no identity has both id=bar1 and id=bar2: the port admits none)
        ms = rp.map_state(lbls("id=foo"), {1000: lbls("id=bar1"), 1001: lbls("id=bar2")})
        dr = R.INGRESS if ingress else R.EGRESS
        assert not any(k[1] == 80 and k[3] == dr for k in ms)


def _wildcard_l3_rules(ingress):
    d, peers = ("ingress", "fromEndpoints") if ingress else ("egress", "toEndpoints")
    kafka = {"kafka": [{"apiKey": "produce"}]}
    http = {"http": [{"method": "GET", "path": "/"}]}
    rules = [{"endpointSelector": es("id=foo"), d: [{peers: [es("id=bar1")]}]},
             {"endpointSelector": es("id=foo"),
              d: [{peers: [es("id=bar2")], "toPorts": tcp(9092, kafka)}]},
             {"endpointSelector": es("id=foo"),
              d: [{peers: [es("id=bar2")], "toPorts": tcp(80, http)}]}]
    if ingress:   # (the ingress test also has a generic L7 parser on 9090)
        rules.append({"endpointSelector": es("id=foo"),
                      d: [{peers: [es("id=bar2")],
                           "toPorts": tcp(9090, {"l7proto": "tester",
                                                 "l7": [{"method": "GET", "path": "/"}]})}]})
    return repo(*rules)


def test_wildcard_l3_rules():
    # repository_test.go:385-542 (ingress), :810-926 (egress): the L3-only
    # rule's peer joins every L7 port's filter (wildcardL3L4Rules)
    for ingress, ports in ((True, (9092, 80, 9090)), (False, (9092, 80))):
        got = l4_sets(_wildcard_l3_rules(ingress)._l4(lbls("id=foo"), ingress))
        assert got == {(p, 6): frozenset({sel("id=bar2"), sel("id=bar1")}) for p in ports}


def test_wildcard_l4_rules():
    # repository_test.go:544-683 (ingress), :928-1067 (egress): L3/L4 rules
    # without L7 join the L7 filter of their own port
    kafka = {"kafka": [{"apiKey": "produce"}]}
    http = {"http": [{"method": "GET", "path": "/"}]}
    for ingress in (True, False):
        d, peers = ("ingress", "fromEndpoints") if ingress else ("egress", "toEndpoints")
        rp = repo({"endpointSelector": es("id=foo"),
                   d: [{peers: [es("id=bar1")], "toPorts": tcp(9092)}]},
                  {"endpointSelector": es("id=foo"),
                   d: [{peers: [es("id=bar2")], "toPorts": tcp(9092, kafka)}]},
                  {"endpointSelector": es("id=foo"),
                   d: [{peers: [es("id=bar1")], "toPorts": tcp(80)}]},
                  {"endpointSelector": es("id=foo"),
                   d: [{peers: [es("id=bar2")], "toPorts": tcp(80, http)}]})
        got = l4_sets(rp._l4(lbls("id=foo"), ingress))
        assert got == {(p, 6): frozenset({sel("id=bar1"), sel("id=bar2")}) for p in (80, 9092)}


def test_wildcard_l3_rules_entities():
    # repository_test.go:1069-1189 (ingress), :1191-1311 (egress): an
    # L3-only entity rule (world) joins the L7 filters as the entity's
    # selector (api.EntitySelectorMapping[world] = reserved:world)
    kafka = {"kafka": [{"apiKey": "produce"}]}
    http = {"http": [{"method": "GET", "path": "/"}]}
    for ingress in (True, False):
        d, peers, ent = (("ingress", "fromEndpoints", "fromEntities") if ingress else
                         ("egress", "toEndpoints", "toEntities"))
        rp = repo({"endpointSelector": es("id=foo"), d: [{ent: ["world"]}]},
                  {"endpointSelector": es("id=foo"),
                   d: [{peers: [es("id=bar2")], "toPorts": tcp(9092, kafka)}]},
                  {"endpointSelector": es("id=foo"),
                   d: [{peers: [es("id=bar2")], "toPorts": tcp(80, http)}]})
        world = R.Selector(frozenset({"reserved:world="}))
        got = l4_sets(rp._l4(lbls("id=foo"), ingress))
        assert got == {(p, 6): frozenset({sel("id=bar2"), world}) for p in (9092, 80)}


# rule_test.go:1438-1460: the shared contexts
A, B, C = lbls("id=a"), lbls("id1=b", "id2=c"), lbls("id=c")
WORLD, FOO = lbls("reserved:world"), lbls("k8s:app=foo")
WILD = {"matchLabels": {}}   # api.WildcardEndpointSelector


def allows(rp, subject, peer, ingress, port=None):
    """AllowsIngress/EgressRLocked on the datapath's terms: the subject's
    policymap (map_state) admits the peer — at L3, or at L4 on `port`/TCP
    when the context carries one; None: no rule selects the subject"""
    if not rp.enabled(subject)[0 if ingress else 1]:
        return None
    d = R.INGRESS if ingress else R.EGRESS
    ms = rp.map_state(subject, {1000: peer})
    return (1000, 0, 0, d) in ms or (port is not None and (1000, port, 6, d) in ms)


def test_rule_can_reach():
    # rule_test.go:31-108 (one rule in the repository: Undecided is Denied)
    rp = repo({"endpointSelector": es("bar"),
               "ingress": [{"fromEndpoints": [es("foo", "foo2")]}]})
    assert allows(rp, lbls("bar"), lbls("foo", "foo2"), True) is True
    assert allows(rp, lbls("bar"), lbls("foo"), True) is False
    rp = repo({"endpointSelector": es("bar"),
               "ingress": [{"fromEndpoints": [es("foo")], "fromRequires": [es("baz")]}]})
    assert allows(rp, lbls("bar"), lbls("foo"), True) is False
    assert allows(rp, lbls("bar"), lbls("baz"), True) is False
    assert allows(rp, lbls("bar"), lbls("foo", "baz"), True) is True


def test_ingress_allow_all():
    # rule_test.go:1495-1520, 1522-1554, 1556-1590
    rp = repo({"endpointSelector": es("id=c"), "ingress": [{"fromEndpoints": [WILD]}]})
    assert allows(rp, B, A, True) is None          # (the API: Denied)
    assert allows(rp, C, A, True) is True
    assert allows(rp, C, A, True, 80) and allows(rp, C, A, True, 90)
    rp = repo({"endpointSelector": es("id=c"),
               "ingress": [{"fromEndpoints": [WILD]}, {"toPorts": tcp(80)}]})
    assert allows(rp, C, A, True, 80) and allows(rp, C, A, True, 90)
    rp = repo({"endpointSelector": es("id=c"), "ingress": [{"toPorts": tcp(80)}]})
    assert allows(rp, C, A, True, 80) is True
    assert allows(rp, C, A, True, 90) is False
    assert rp._l4(C, True) == {(80, 6): R.WILDCARD}


def test_egress_allow_all():
    # rule_test.go:1592-1616, 1618-1658
    rp = repo({"endpointSelector": es("id=a"), "egress": [{"toEndpoints": [WILD]}]})
    assert allows(rp, A, B, False) is True and allows(rp, A, C, False) is True
    assert allows(rp, A, C, False, 80) and allows(rp, A, C, False, 90)
    rp = repo({"endpointSelector": es("id=a"), "egress": [{"toPorts": tcp(80)}]})
    assert allows(rp, A, C, False, 80) is True
    assert allows(rp, A, C, False, 90) is False


def test_egress_world_and_all_entities():
    # rule_test.go:1660-1719 (L4 to world), 1721-1780 (L4 to all),
    # 1782-1824 (L3 to world), 1826-1868 (L3 to all)
    cases = (({"toEntities": ["world"], "toPorts": tcp(80)},
              {(WORLD, 80): True, (WORLD, 90): False, (FOO, 80): False, (FOO, 90): False}),
             ({"toEntities": ["all"], "toPorts": tcp(80)},
              {(WORLD, 80): True, (WORLD, 90): False, (FOO, 80): True, (FOO, 90): False}),
             ({"toEntities": ["world"]},
              {(WORLD, 80): True, (WORLD, 90): True, (FOO, 80): False, (FOO, 90): False}),
             ({"toEntities": ["all"]},
              {(WORLD, 80): True, (WORLD, 90): True, (FOO, 80): True, (FOO, 90): True}))
    for rule, want in cases:
        rp = repo({"endpointSelector": es("id=a"), "egress": [rule]})
        for (peer, port), ok in want.items():
            assert allows(rp, A, peer, False, port) is ok, (rule, sorted(peer), port)
        if "toPorts" in rule:   # one selector on 80/TCP (world, or all)
            f = rp._l4(A, False)[(80, 6)]
            assert f == R.WILDCARD or len(f) == 1


def test_l4_policy():
    # rule_test.go:110-315: L4 rules without peers select every identity;
    # ProtoAny gives TCP and UDP; a rule that does not select the endpoint
    # resolves to nothing
    http = {"http": [{"method": "GET", "path": "/"}]}
    rule1 = {"endpointSelector": es("bar"),
             "ingress": [{"toPorts": [{"ports": [{"port": "80", "protocol": "TCP"},
                                                 {"port": "8080", "protocol": "TCP"}],
                                       "rules": http}]}],
             "egress": [{"toPorts": [{"ports": [{"port": "3000", "protocol": "ANY"}]}]}]}
    rp = repo(rule1)
    assert rp._l4(lbls("bar"), True) == {(80, 6): R.WILDCARD, (8080, 6): R.WILDCARD}
    assert rp._l4(lbls("bar"), False) == {(3000, 6): R.WILDCARD, (3000, 17): R.WILDCARD}
    assert rp._l4(lbls("foo"), True) == {} and rp._l4(lbls("foo"), False) == {}
    rule2 = {"endpointSelector": es("bar"),
             "ingress": [{"toPorts": tcp(80)}, {"toPorts": tcp(80, http)}],
             "egress": [{"toPorts": [{"ports": [{"port": "3000", "protocol": "ANY"}]}]}]}
    rp = repo(rule2)
    assert rp._l4(lbls("bar"), True) == {(80, 6): R.WILDCARD}
    assert rp._l4(lbls("bar"), False) == {(3000, 6): R.WILDCARD, (3000, 17): R.WILDCARD}


def test_merge_l4_policy():
    # rule_test.go:317-362 (ingress), 364-416 (egress): two rules' peers on
    # one port merge, in rule order
    for ingress in (True, False):
        d, peers = ("ingress", "fromEndpoints") if ingress else ("egress", "toEndpoints")
        rp = repo({"endpointSelector": es("bar"),
                   d: [{peers: [es("foo")], "toPorts": tcp(80)},
                       {peers: [es("baz")], "toPorts": tcp(80)}]})
        assert rp._l4(lbls("bar"), ingress) == {(80, 6): [sel("foo"), sel("baz")]}


def test_l4_wildcard_merge():
    # rule_test.go:1870-2068: an L4-only rule (no peers, or the wildcard
    # selector) on the port of an L3-dependent L7 rule, in either order,
    # leaves the port open to every identity
    http = {"http": [{"method": "GET", "path": "/"}]}
    l7 = {"fromEndpoints": [es("id=c")], "toPorts": tcp(80, http)}
    for l4 in ({"toPorts": tcp(80)}, {"fromEndpoints": [WILD], "toPorts": tcp(80)}):
        for pair in ((l7, l4), (l4, l7)):
            rp = repo({"endpointSelector": es("id=a"), "ingress": list(pair)})
            assert rp._l4(A, True) == {(80, 6): R.WILDCARD}
            assert allows(rp, A, FOO, True, 80) is True
            assert allows(rp, A, FOO, True, 90) is False


def test_prefixes_from_cidr():
    # cidr_test.go:27-47 (getPrefixesFromCIDR: ip.ParseCIDRs, a bare address
    # is a host prefix) — what the CIDR selectors' labels carry
    # (labels.IPStringToLabel, pkg/labels/cidr.go:58-73)
    for inp, want in (("0.0.0.0/0", "0.0.0.0/0"), ("192.0.2.3", "192.0.2.3/32"),
                      ("192.0.2.3/32", "192.0.2.3/32"), ("192.0.2.3/24", "192.0.2.0/24"),
                      ("192.0.2.0/24", "192.0.2.0/24"), ("::/0", "::/0"),
                      ("fdff::ff", "fdff::ff/128")):
        got = R.cidr_selectors([inp])
        assert got[-1] == R.Selector(frozenset({f"cidr:{want}="})), inp
        # (a /0 also selects reserved:world, once: api/cidr.go:70-86)
        assert len(got) == (2 if want.endswith("/0") else 1)


def test_get_cidr_prefixes():
    # cidr_test.go:49-132 (GetCIDRPrefixes; the resolver keeps the set, the
    # Go call lists every occurrence)
    rp = repo({"endpointSelector": es("bar"),
               "ingress": [{"fromCIDR": ["192.0.2.0/24"]}],
               "egress": [{"toCIDR": ["192.0.2.0/24", "192.0.3.0/24"]}]})
    assert set(rp.cidrs()) == {"192.0.2.0/24", "192.0.3.0/24"}
    rp = repo({"endpointSelector": es("bar"),
               "ingress": [{"fromCIDRSet": [{"cidr": "192.0.2.0/24",
                                             "except": ["192.0.2.128/25"]}]}],
               "egress": [{"toCIDRSet": [{"cidr": "10.0.0.0/8", "except": ["10.0.0.0/16"]}]}]})
    assert set(rp.cidrs()) == {"192.0.2.0/25", "10.128.0.0/9", "10.64.0.0/10", "10.32.0.0/11",
                               "10.16.0.0/12", "10.8.0.0/13", "10.4.0.0/14", "10.2.0.0/15",
                               "10.1.0.0/16"}


def test_entities():
    # api/entity_test.go:23-62 (EntityCluster does not select the host:
    # an EndpointSelector cannot express OR)
    host, cl, world, foo = (lbls("reserved:host"), lbls("reserved:cluster"),
                            lbls("reserved:world"), lbls("id=foo"))
    want = {"host": (True, False, False, False), "all": (True, True, True, True),
            "cluster": (False, True, False, False), "world": (False, False, True, False)}
    for e, w in want.items():
        s = R.entity_selector(e)
        assert tuple(s.matches(x) for x in (host, cl, world, foo)) == w, e
    assert R.entity_selector("host").matches(lbls("reserved:host", "id=foo"))
    sl = [R.entity_selector("host"), R.entity_selector("world")]
    assert [any(s.matches(x) for s in sl) for x in (host, world, foo)] == [True, True, False]


def test_cidr_endpoint_selectors():
    # api/cidr_test.go:24-88: /0 matches all and brings reserved:world (once)
    world = R.Selector(frozenset({"reserved:world="}))
    v4, v6 = (R.Selector(frozenset({"cidr:0.0.0.0/0="})),
              R.Selector(frozenset({"cidr:::/0="})))
    assert R.cidr_selectors(["0.0.0.0/0"]) == [world, v4]
    assert R.cidr_selectors(["::/0"]) == [world, v6]
    assert R.cidr_selectors(["0.0.0.0/0", "::/0", "192.168.128.10/24"]) == \
        [world, v4, v6, R.Selector(frozenset({"cidr:192.168.128.0/24="}))]
    assert any(s.matches(lbls("reserved:world")) for s in R.cidr_selectors(["0.0.0.0/0"]))
    assert R.cidr_selectors(["192.0.2.0/24"]) == [R.Selector(frozenset({"cidr:192.0.2.0/24="}))]


def test_rule_can_reach_entities():
    # rule_test.go:1067-1111 (ingress from world / cluster), 1113-1157
    # (egress to them): the entities allow, another peer is undecided
    for ingress in (True, False):
        d, ent = ("ingress", "fromEntities") if ingress else ("egress", "toEntities")
        rp = repo({"endpointSelector": es("bar"), d: [{ent: ["world", "cluster"]}]})
        for peer, ok in ((lbls("reserved:world"), True), (lbls("reserved:cluster"), True),
                         (lbls("foo"), False)):
            assert rp._can_reach(lbls("bar"), peer, ingress) is ok


def test_l3_policy():
    # rule_test.go:887-1018: the CIDR policy of the rule selecting bar — a
    # bare IPv4 address takes its class mask when the bits after it are zero
    # (192.168.2.0 -> /24), else /32; a bare IPv6 address /128; a CIDRSet
    # its exceptions removed — and the prefix-length counts
    rule = {"endpointSelector": es("bar"),
            "ingress": [{"fromCIDR": ["10.0.1.0/24", "192.168.2.0", "10.0.3.1",
                                      "2001:db8::1/48", "2001:db9::"]}],
            "egress": [{"toCIDR": ["10.1.0.0/16", "2001:dbf::/64"]},
                       {"toCIDRSet": [{"cidr": "10.0.0.0/8", "except": ["10.96.0.0/12"]}]}]}
    cp = repo(rule).cidr_policy(lbls("bar"))
    assert cp["ingress"]["map"] == {"10.0.1.0/24": (4, 24), "192.168.2.0/24": (4, 24),
                                    "10.0.3.1/32": (4, 32), "2001:db8::/48": (6, 48),
                                    "2001:db9::/128": (6, 128)}
    assert cp["ingress"]["v4"] == {32: 1, 24: 2} and cp["ingress"]["v6"] == {128: 1, 48: 1}
    assert cp["egress"]["map"] == {"10.1.0.0/16": (4, 16), "10.128.0.0/9": (4, 9),
                                   "10.0.0.0/10": (4, 10), "10.64.0.0/11": (4, 11),
                                   "10.112.0.0/12": (4, 12), "2001:dbf::/64": (6, 64)}
    assert cp["egress"]["v4"] == {16: 1, 12: 1, 11: 1, 10: 1, 9: 1}
    assert cp["egress"]["v6"] == {64: 1}
    # a rule that does not select the endpoint contributes nothing
    assert repo(rule).cidr_policy(lbls("foo"))["ingress"]["map"] == {}
    # Sanitize refuses: an unparsable CIDR, a CIDRSet without a cidr or with a
    # bare address, an exception outside the cidr, a netmask, a length
    # beyond the family's bits
    bad = [{"fromCIDR": ["10.0.1..0/24"]}, {"fromCIDRSet": [{"cidr": ""}]},
           {"fromCIDRSet": [{"cidr": "10.0.1.32"}]},
           {"fromCIDRSet": [{"cidr": "10.0.0.0/10", "except": ["10.64.0.0/11"]}]},
           {"fromCIDR": ["10.0.1.0/128.0.0.128"]}, {"fromCIDR": ["10.0.1.0/34"]}]
    for x in bad:
        with pytest.raises(R.PolicyError):
            R.sanitize_rule({"endpointSelector": es("bar"), "ingress": [x]})
    R.sanitize_rule({"endpointSelector": es("bar"),
                     "ingress": [{"fromCIDRSet": [{"cidr": "10.0.1.0/24"}]}]})


def test_l3_policy_restrictions():
    # rule_test.go:1020-1041: 41 prefix lengths are too many, either way;
    # :1043-1065: ToCIDR and ToEndpoints cannot combine
    cidrs = [f"{i}::/{i}" for i in range(1, 42)]
    for d, k in (("ingress", "fromCIDR"), ("egress", "toCIDR")):
        with pytest.raises(R.PolicyError, match="too many"):
            R.sanitize_rule({"endpointSelector": es("bar"), d: [{k: cidrs}]})
        R.sanitize_rule({"endpointSelector": es("bar"), d: [{k: cidrs[:40]}]})
    with pytest.raises(R.PolicyError, match="Combining"):
        R.sanitize_rule({"endpointSelector": es("bar"),
                         "egress": [{"toCIDR": ["10.1.0.0/16", "2001:dbf::/64"],
                                     "toEndpoints": [es("foo")]}]})


def test_entity_validation():
    # rule_test.go:1159-1216: world and host pass, an unknown entity fails
    for d, k in (("ingress", "fromEntities"), ("egress", "toEntities")):
        for ents, ok in ((["world"], True), (["host"], True), (["trololo"], False),
                         (["world", "host"], True)):
            r = {"endpointSelector": es("bar"), d: [{k: ents}]}
            if ok:
                R.sanitize_rule(r)
            else:
                with pytest.raises(R.PolicyError, match="unsupported entity"):
                    R.sanitize_rule(r)


def _l7_rule(ports, rules):
    return {"endpointSelector": WILD,
            "ingress": [{"fromEndpoints": [WILD],
                         "toPorts": [{"ports": [{"port": p, "protocol": q} for p, q in ports],
                                      "rules": rules}]}]}


def test_l7_rules_with_non_tcp_protocols():
    # api/rule_validation_test.go:24-147
    http = {"http": [{"method": "GET", "path": "/"}]}
    R.sanitize_rule(_l7_rule([("80", "TCP"), ("81", "TCP")], http))
    for ports, proto in (([("80", "UDP")], "UDP"), ([("80", "ANY")], "ANY"),
                         ([("80", "TCP"), ("12345", "UDP")], "UDP"),
                         ([("80", "UDP"), ("12345", "TCP")], "UDP")):
        with pytest.raises(R.PolicyError) as e:
            R.sanitize_rule(_l7_rule(ports, http))
        assert str(e.value) == f"L7 rules can only apply exclusively to TCP, not {proto}"


def test_http_rule_regexes_and_l7_rules():
    # api/rule_validation_test.go:151-198 (regexes), 274-347 (key/value rules)
    tcp2 = [("80", "TCP"), ("81", "TCP")]
    for h in ({"method": "GET", "path": "*"}, {"method": "*", "path": "/"}):
        with pytest.raises(R.PolicyError):
            R.sanitize_rule(_l7_rule(tcp2, {"http": [h]}))
    R.sanitize_rule(_l7_rule(tcp2, {"l7proto": "test.lineparser",
                                    "l7": [{"method": "PUT", "path": "/"},
                                           {"method": "GET", "path": "/"}]}))
    R.sanitize_rule(_l7_rule(tcp2, {"l7proto": "test.lineparser"}))
    with pytest.raises(R.PolicyError, match="Empty key"):
        R.sanitize_rule(_l7_rule(tcp2, {"l7proto": "test.lineparser",
                                        "l7": [{"method": "PUT", "": "Foo"}]}))


def test_cidr_rule_sanitize():
    # api/rule_validation_test.go:201-238: the prefix length, or an error
    for c, n in (("0.0.0.0/0", 0), ("10.0.0.0/24", 24), ("192.0.2.3/32", 32), ("::/0", 0),
                 ("ff02::/64", 64), ("2001:0db8:85a3:0000:0000:8a2e:0370:7334/128", 128)):
        assert R.cidr_rule_sanitize({"cidr": c}) == n
    with pytest.raises(R.PolicyError):
        R.cidr_rule_sanitize({"cidr": "10.0.0.0/254.0.0.255"})


def test_to_services_sanitize():
    # api/rule_validation_test.go:240-271: ToServices with ToPorts is allowed
    R.sanitize_rule({"endpointSelector": WILD,
                     "egress": [{"toServices": [{"k8sServiceSelector": {
                         "selector": {"matchLabels": {"app": "tested-service"}}}}],
                                 "toPorts": tcp(80) + tcp(81)}]})


# l4Filter_test.go: the L4 filters themselves (peers, parser, L7 rules per
# peer selector).  The Go tests run with AllowLocalhost unset (no host / world
# L7 override) but case 12; a single rule's resolveL4IngressPolicy has no
# wildcardL3L4Rules step, ResolveL4IngressPolicy (cases 1, 2B) has.
SA, SC, W = R.Selector(lbls("id=a")), R.Selector(lbls("id=c")), R.WILDCARD_SELECTOR
GET = {"http": [{"method": "GET", "path": "/"}]}
KFOO = {"kafka": [{"topic": "foo"}]}


def _fr(*ingress_rules, localhost=False):
    return R.Repository(R.parse_rules([{"endpointSelector": es("id=a"),
                                        "ingress": list(ingress_rules)}]),
                        always_allow_localhost=localhost, host_allows_world=False)


def _ir(peers, rules=None, port="80"):
    pr = {"ports": [{"port": port, "protocol": "TCP"}]}
    if rules is not None:
        pr["rules"] = rules
    return {"fromEndpoints": peers, "toPorts": [pr]}


def _one(rp, wildcard=False, subject=A):
    fs = rp.l4_filters(subject, True, wildcard_l3l4=wildcard)
    if not fs:
        return None
    (k, f), = fs.items()
    return k, f


def _l7(**kw):
    return R._l7_norm(kw)


def test_l4filter_allow_all_l3_and_l7():
    # l4Filter_test.go:74-162 (case 1A explicit wildcard, 1B implicit)
    for peers in ([WILD], []):
        k, f = _one(_fr(_ir(peers), _ir(peers)), wildcard=True)
        assert k == (80, 6) and f.allows_all() and f.parser == "" and f.l7 == {}


def test_l4filter_allow_all_l3_and_shadowed_l7():
    # :164-278 — 2A: the rule alone keeps the HTTP rule on the wildcard
    # selector; 2B: the repository's wildcardL3L4Rules turns it allow-all
    k, f = _one(_fr(_ir([WILD]), _ir([WILD], GET)))
    assert f.allows_all() and f.parser == "http"
    assert f.l7 == {W: _l7(http=[{"method": "GET", "path": "/"}])}
    assert f.derived == [frozenset(), frozenset()]   # (DerivedFromRules {nil, nil})
    k, f = _one(_fr(_ir([WILD], GET), _ir([WILD])), wildcard=True)
    assert f.allows_all() and f.parser == "http" and len(f.l7) == 1


def test_l4filter_identical_restricted_l7():
    # :280-350 (HTTP), :352-425 (Kafka): identical rules merge into one
    for rules, port, parser in ((GET, "80", "http"), (KFOO, "9092", "kafka")):
        k, f = _one(_fr(_ir([WILD], rules, port), _ir([WILD], rules, port)))
        assert k == (int(port), 6) and f.allows_all() and f.parser == parser
        assert f.l7 == {W: R._l7_norm(rules)}
        # a rule that does not select the endpoint resolves to nothing
        assert _one(_fr(_ir([WILD], rules, port)), subject=lbls("foo")) is None


def test_l4filter_mismatching_parsers():
    # :427-613: Kafka / HTTP in either order, HTTP then a generic parser,
    # and (egress) a generic parser without rules then HTTP: an error
    tester = {"l7proto": "testing", "l7": [{"method": "PUT", "path": "/Foo"}]}
    for r1, r2 in ((KFOO, GET), (GET, KFOO), (GET, tester)):
        with pytest.raises(R.PolicyError, match="conflicting L7"):
            _fr(_ir([WILD], r1), _ir([WILD], r2)).l4_filters(A, True, wildcard_l3l4=False)
    rp = R.Repository(R.parse_rules([{"endpointSelector": es("id=a"), "egress": [
        {"toEndpoints": [es("id=c")], "toPorts": [{"ports": [{"port": "80", "protocol": "TCP"}],
                                                   "rules": {"l7proto": "testing"}}]},
        {"toEndpoints": [es("id=c")], "toPorts": [{"ports": [{"port": "80", "protocol": "TCP"}],
                                                   "rules": GET}]}]}]),
        always_allow_localhost=False)
    with pytest.raises(R.PolicyError, match="conflicting L7"):
        rp.l4_filters(A, False, wildcard_l3l4=False)


def test_l4filter_l3_shadowed_by_allow_all():
    # :615-730 (case 6): the wildcard rule shadows the id=a rule, either order
    for pair in ((_ir([es("id=a")]), _ir([WILD])), (_ir([WILD]), _ir([es("id=a")]))):
        k, f = _one(_fr(*pair))
        assert f.endpoints == [W] and f.parser == "" and f.l7 == {}
        assert _one(_fr(*pair), subject=lbls("foo")) is None


def test_l4filter_l7_partially_and_fully_shadowed():
    # :732-871 (case 7): id=a's HTTP rule stays on its selector, L3 is all;
    # :873-1029 (case 8): both selectors keep the HTTP rule
    http = _l7(http=[{"method": "GET", "path": "/"}])
    for pair in ((_ir([es("id=a")], GET), _ir([WILD])), (_ir([WILD]), _ir([es("id=a")], GET))):
        k, f = _one(_fr(*pair))
        assert f.endpoints == [W] and f.parser == "http" and f.l7 == {SA: http}
    for pair in ((_ir([es("id=a")], GET), _ir([WILD], GET)),
                 (_ir([WILD], GET), _ir([es("id=a")], GET))):
        k, f = _one(_fr(*pair))
        assert f.endpoints == [W] and f.parser == "http" and f.l7 == {W: http, SA: http}


def test_l4filter_conflicting_l7_with_endpoint():
    # :1031-1136 (case 9): Kafka on id=a and HTTP on all, either order
    for pair in ((_ir([es("id=a")], KFOO), _ir([WILD], GET)),
                 (_ir([WILD], GET), _ir([es("id=a")], KFOO))):
        with pytest.raises(R.PolicyError):
            _fr(*pair).l4_filters(A, True, wildcard_l3l4=False)


def test_l4filter_different_endpoints():
    # :1138-1217 (case 10: the same L7 rule for id=a and id=c), :1219-1283
    # (case 11: no L7 rules): both peers, in rule order
    http = _l7(http=[{"method": "GET", "path": "/"}])
    k, f = _one(_fr(_ir([es("id=a")], GET), _ir([es("id=c")], GET)))
    assert f.endpoints == [SA, SC] and f.parser == "http" and f.l7 == {SC: http, SA: http}
    k, f = _one(_fr(_ir([es("id=a")]), _ir([es("id=c")])))
    assert f.endpoints == [SA, SC] and f.parser == "" and f.l7 == {}


def test_l4filter_localhost_shadows_l7():
    # :1285-1340 (case 12): AllowLocalhost=always puts the host selector at
    # L7 allow-all (an empty L7Rules) beside the rule's own HTTP rule
    k, f = _one(_fr(_ir([WILD], GET), localhost=True))
    assert f.endpoints == [W] and f.parser == "http"
    assert f.l7 == {W: _l7(http=[{"method": "GET", "path": "/"}]),
                    R.entity_selector("host"): _l7()}


def test_l3_l4_l7_merge():
    # rule_test.go:2070-2168: an HTTP rule for every peer and an L4 rule for
    # id=c on port 80, either order: the filter admits all, [wildcard, id=c],
    # with the HTTP parser and L7 rules for both selectors
    l7 = {"toPorts": [{"ports": [{"port": "80", "protocol": "TCP"}], "rules": GET}]}
    for pair in ((l7, _ir([es("id=c")])), (_ir([es("id=c")]), l7)):
        k, f = _one(_fr(*pair), wildcard=True)
        assert f.endpoints == [W, SC] and f.parser == "http" and len(f.l7) == 2
        assert f.l7[SC] == _l7(http=[{}])   # (id=c: allowed at every L7 resource)


def test_parse_l4_proto_and_selects_all():
    # api/utils_test.go:93-117, api/selector_test.go:32-47
    assert [R.parse_l4_proto(x) for x in ("TCP", "UDP", "ANY", "tcp", "Any", "")] == \
        ["TCP", "UDP", "ANY", "TCP", "ANY", "ANY"]
    for bad in ("TCP2", "t", "foo2"):
        with pytest.raises(R.PolicyError, match="invalid protocol"):
            R.parse_l4_proto(bad)
    bar, foo = R.Selector(lbls("bar")), R.Selector(lbls("foo"))
    assert R._selects_all([]) and R._selects_all([W]) and R._selects_all([W, bar])
    assert not R._selects_all([bar, foo])


def test_label_selector_requirements():
    # api/selector_test.go:49-75: matchLabels become Equals requirements and
    # matchExpressions join them (k8s LabelSelectorAsSelector); a selector
    # that does not convert matches nothing (selector.go:162-175, 277-288)
    s = R.Selector.parse({"matchLabels": {"foo": "bar", "baz": "alice"},
                          "matchExpressions": [{"key": "foo", "operator": "NotIn",
                                                "values": ["default"]}]})
    assert s.matches(lbls("foo=bar", "baz=alice", "x=y"))
    assert not s.matches(lbls("foo=bar")) and not s.matches(lbls("foo=default", "baz=alice"))
    e = {"matchExpressions": [{"key": "env", "operator": "In", "values": ["prod", "qa"]},
                              {"key": "tier", "operator": "Exists"},
                              {"key": "debug", "operator": "DoesNotExist"},
                              {"key": "zone", "operator": "NotIn", "values": ["b"]}]}
    s = R.Selector.parse(e)
    assert s.matches(lbls("env=qa", "tier=web")) and s.matches(lbls("env=prod", "tier=", "zone=a"))
    for bad in (lbls("env=dev", "tier=web"), lbls("env=qa"), lbls("env=qa", "tier=web", "debug=1"),
                lbls("env=qa", "tier=web", "zone=b")):
        assert not s.matches(bad)
    assert not s.selects_all()
    for inval in ({"key": "a", "operator": "Equals", "values": ["x"]},
                  {"key": "a", "operator": "In", "values": []},
                  {"key": "a", "operator": "Exists", "values": ["x"]}):
        s = R.Selector.parse({"matchExpressions": [inval]})
        assert not s.matches(lbls("a=x")) and not s.matches(lbls()) and not s.selects_all()
    # source prefixes: k8s: / any: keys match the (k8s-sourced) pod labels
    assert R.Selector.parse({"matchLabels": {"k8s:app": "x", "any:env": "p"}}) == \
        R.Selector.parse({"matchLabels": {"app": "x", "env": "p"}})
    assert R.Selector.parse({"matchLabels": {"reserved:host": ""}}).matches(lbls("reserved:host"))
    # a reserved:all key matches every label set, yet is no wildcard
    s = R.Selector.parse({"matchLabels": {"reserved:all": ""}})
    assert s.matches(lbls("foo")) and s.matches(lbls()) and not s.selects_all()
    # in a rule: the endpoint selector and a peer selector with expressions
    rp = repo({"endpointSelector": {"matchExpressions": [{"key": "role", "operator": "In",
                                                          "values": ["db", "cache"]}]},
               "ingress": [{"fromEndpoints": [{"matchExpressions": [
                   {"key": "role", "operator": "NotIn", "values": ["public"]}]}]}]})
    assert ingress_allowed(rp, lbls("role=web"), lbls("role=db")) is True
    assert ingress_allowed(rp, lbls("role=public"), lbls("role=cache")) is False
    assert ingress_allowed(rp, lbls("role=web"), lbls("role=web")) is None   # not selected


def _L(*kv, src="unspec"):
    return [{"source": src, "key": k, "value": v} for k, v in kv]


def _T(*kv, src="unspec"):
    return {(src, k, v) for k, v in kv}


def test_add_search_delete():
    # repository_test.go:29-112
    rp = R.Repository([])
    with pytest.raises(R.PolicyError):
        rp.add({})                      # cannot add an empty rule
    assert rp.revision == 1
    l1, l2 = _L(("tag1", ""), ("tag2", "")), _L(("tag3", ""), src="any")
    r1 = {"endpointSelector": es("foo"), "labels": l1}
    r2 = {"endpointSelector": es("bar"), "labels": l1}
    r3 = {"endpointSelector": es("bar"), "labels": l2}
    assert rp.add(r1) == 2 and rp.add(r2) == 3
    assert rp.search(_T(("tag3", ""), src="any")) == []
    assert rp.add(r3) == 4
    got = rp.search(_T(("tag1", ""), ("tag2", "")))
    assert [r.selector for r in got] == [sel("foo"), sel("bar")]
    assert len(rp.search(_T(("tag3", ""), src="any"))) == 1
    assert rp.delete_by_labels(_T(("tag1", ""), ("tag2", ""))) == (5, 2)
    assert rp.delete_by_labels(_T(("tag1", ""), ("tag2", ""))) == (5, 0)
    assert len(rp.search(_T(("tag3", ""), src="any"))) == 1
    assert rp.delete_by_labels(_T(("tag3", ""), src="any")) == (6, 1)
    assert rp.search(_T(("tag3", ""), src="any")) == []


def test_contains_all():
    # repository_test.go:114-191
    a = [_T(("1", "1"), ("2", "2"), ("3", "3"), src="1"),
         _T(("4", "4"), ("5", "5"), ("6", "6"), src="1"),
         _T(("7", "7"), ("8", "8"), ("9", "9"), src="1")]
    b = a[:2]

    def mk(sel_key, lab):
        return {"endpointSelector": es(sel_key),
                "labels": [{"source": s_, "key": k, "value": v} for s_, k, v in sorted(lab)]}
    rpa = R.Repository([])
    for lab, k in zip(a, ("foo", "bar", "bar")):
        rpa.add(mk(k, lab))
    rpb = R.Repository([])
    for lab, k in zip(b, ("foo", "bar")):
        rpb.add(mk(k, lab))
    rpe = R.Repository([])
    rpe.add({"endpointSelector": es("bar")})
    assert rpa.contains_all(b) and not rpb.contains_all(a)
    assert rpa.contains_all([]) and rpe.contains_all([]) and not rpe.contains_all(a)


def test_l4_rule_labels():
    # rule_test.go:1322-1436: each filter's DerivedFromRules lists the labels
    # of the rules it came from; a rule without ports adds none
    def rule(name, ing=None, eg=None):
        r = {"endpointSelector": es("bar"), "labels": _L(("name", name))}
        if ing:
            r["ingress"] = [{"toPorts": tcp(ing)}]
        if eg:
            r["egress"] = [{"toPorts": tcp(eg)}]
        return r
    rules = {"rule0": rule("apiRule0"), "rule1": rule("apiRule1", 1010, 1100),
             "rule2": rule("apiRule2", 1020, 1200)}
    lab = {k: frozenset(_T(("name", "apiRule" + k[-1]))) for k in rules}
    for apply, want_in, want_eg in (
            (["rule0"], {}, {}),
            (["rule1"], {1010: ["rule1"]}, {1100: ["rule1"]}),
            (["rule0", "rule1", "rule2"], {1010: ["rule1"], 1020: ["rule2"]},
             {1100: ["rule1"], 1200: ["rule2"]})):
        rp = R.Repository(R.parse_rules([rules[k] for k in apply]))
        for ingress, want in ((True, want_in), (False, want_eg)):
            fs = rp.l4_filters(lbls("bar"), ingress, wildcard_l3l4=False)
            assert {k[0]: [x for x in f.derived] for k, f in fs.items()} == \
                {p: [lab[n] for n in ns] for p, ns in want.items()}


def test_l3_rule_labels():
    # rule_test.go:1218-1320: each CIDR prefix's DerivedFromRules
    def rule(name, i=None, e=None):
        r = {"endpointSelector": es("bar"), "labels": _L(("name", name))}
        if i:
            r["ingress"] = [{"fromCIDR": [i]}]
        if e:
            r["egress"] = [{"toCIDR": [e]}]
        return r
    rules = {"rule0": rule("apiRule0"), "rule1": rule("apiRule1", "10.0.1.0/32", "10.1.0.0/32"),
             "rule2": rule("apiRule2", "10.0.2.0/32", "10.2.0.0/32")}
    lab = {k: frozenset(_T(("name", "apiRule" + k[-1]))) for k in rules}
    for apply, want_in, want_eg in (
            (["rule0"], {}, {}),
            (["rule1"], {"10.0.1.0/32": ["rule1"]}, {"10.1.0.0/32": ["rule1"]}),
            (["rule0", "rule1", "rule2"], {"10.0.1.0/32": ["rule1"], "10.0.2.0/32": ["rule2"]},
             {"10.1.0.0/32": ["rule1"], "10.2.0.0/32": ["rule2"]})):
        cp = R.Repository(R.parse_rules([rules[k] for k in apply])).cidr_policy(lbls("bar"))
        for d, want in (("ingress", want_in), ("egress", want_eg)):
            assert cp[d]["derived"] == {p: [lab[n] for n in ns] for p, ns in want.items()}
