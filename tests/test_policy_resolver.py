"""The C1 policy resolver (cilium_amd/policy_resolver.py): CIDR-set
expansion against the reference's own test vectors (pkg/ip/ip_test.go:96-163),
and the MapState the example policies give, derived by hand from the rules
in tests/golden/c1_policies.json (examples/policies/{l3,l4}) and the
reference's resolver semantics (pkg/endpoint/policy.go, pkg/policy/rule.go).
The Go resolver cannot run here (no Go toolchain): these pin the restatement
to the reference's tests and rules, not to its output ("parity unpinned")."""
import ipaddress
import os

import numpy as np
import pytest

from cilium_amd import policy_resolver as R
from cilium_amd import synth as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def nets(xs):
    return {ipaddress.ip_network(x, strict=False) for x in xs}


def test_cidr_except_reference_vectors():
    # pkg/ip/ip_test.go:97-109
    got = R.cidr_rule_set([{"cidr": "10.0.0.0/8",
                            "except": ["10.96.0.0/12", "10.112.0.0/13"]}])
    assert nets(got) == nets(["10.128.0.0/9", "10.0.0.0/10", "10.64.0.0/11",
                              "10.120.0.0/13"])
    # :111-147 (overlapping exceptions, an unmasked one)
    got = R.cidr_rule_set([{"cidr": "10.0.0.0/8",
                            "except": ["10.96.0.0/12", "10.112.0.0/13", "10.62.0.33/32",
                                       "10.93.0.4/30", "10.63.0.5/13"]}])
    want = ["10.128.0.0/9", "10.0.0.0/11", "10.32.0.0/12", "10.48.0.0/13",
            "10.120.0.0/13", "10.64.0.0/12", "10.80.0.0/13", "10.88.0.0/14",
            "10.94.0.0/15", "10.92.0.0/16", "10.93.128.0/17", "10.93.64.0/18",
            "10.93.32.0/19", "10.93.16.0/20", "10.93.8.0/21", "10.93.4.0/22",
            "10.93.2.0/23", "10.93.1.0/24", "10.93.0.128/25", "10.93.0.64/26",
            "10.93.0.32/27", "10.93.0.16/28", "10.93.0.8/29", "10.93.0.0/30"]
    assert nets(got) == nets(want)
    # :155-161 (IPv6)
    got = R.cidr_rule_set([{"cidr": "fd44:7089:ff32:712b:ff00::/64",
                            "except": ["fd44:7089:ff32:712b::/66"]}])
    assert nets(got) == nets(["fd44:7089:ff32:712b:8000::/65",
                              "fd44:7089:ff32:712b:4000::/66"])


def test_cidr_identity_labels():
    lb = R.cidr_labels("192.0.2.0/24")
    assert "cidr:192.0.2.0/24=" in lb and "cidr:0.0.0.0/0=" in lb
    assert "cidr:192.0.0.0/16=" in lb and "reserved:world=" in lb
    assert len([x for x in lb if x.startswith("cidr:")]) == 25
    assert "reserved:cluster=" in R.cidr_labels("10.1.0.0/16")


@pytest.fixture(scope="module")
def c1():
    return S.config_c1(1)


def keys_of(t, lxc):
    p = t.policy[lxc]
    return {(int(r["identity"]), int(S.ntohs(r["dport"])), int(r["proto"]),
             int(r["egress"])) for r in p}


def ids_where(ctx, pred):
    return {i for i, lb in ctx["identities"].items() if pred(lb)}


def test_c1_backend(c1):
    """role=backend: l3.json (L3 from role=frontend), multi_rule.json (the
    same, plus 80/TCP from every identity: its toPorts section has no
    fromEndpoints, so the filter's peers are the wildcard selector,
    l4.go:171-173, and policy.go:115-127 makes one key per identity),
    l3_l4_combined.json (80/TCP from role=frontend).  No rule selects it on
    egress: allow-all, one L3 key per identity (policy.go:357-380)."""
    t, ctx = c1
    k = keys_of(t, S.EP_LXC_ID)
    every = set(ctx["identities"])
    front = ids_where(ctx, lambda lb: "role=frontend" in lb)
    assert {(i, 0, 0, 0) for i in front} <= k
    assert {(i, 80, 6, 0) for i in every} <= k
    assert {(i, 0, 0, 1) for i in every} <= k
    assert (R.HOST_ID, 0, 0, 0) in k and (R.WORLD_ID, 0, 0, 0) in k   # k8s-mode localhost
    l3_in = {x[0] for x in k if x[1:] == (0, 0, 0)}
    assert l3_in == front | {R.HOST_ID, R.WORLD_ID}
    assert len(k) == len(front | {1, 2}) + 2 * len(every)


def test_c1_my_service(c1):
    """app=myService: egress l4.json (80/TCP to every identity) and cidr.json
    (L3 to the CIDR identities of 20.1.1.1/32 and of 10.0.0.0/8 minus
    10.96.0.0/12, whose selectors cidr:<prefix> also match any CIDR identity
    inside those prefixes); ingress from_init.json: 53/UDP from
    reserved:init only."""
    t, ctx = c1
    lxc = [x for x in t.policy if t.seclabel[x] == 257][0]
    k = keys_of(t, lxc)
    every = set(ctx["identities"])
    assert {(i, 80, 6, 1) for i in every} <= k
    eg_l3 = {x[0] for x in k if x[1:] == (0, 0, 1)}
    want = ids_where(ctx, lambda lb: "cidr:20.1.1.1/32=" in lb or any(
        f"cidr:{p}=" in lb for p in ("10.0.0.0/10", "10.64.0.0/11", "10.112.0.0/12",
                                     "10.128.0.0/9")))
    assert eg_l3 == want and len(want) >= 5
    ing = {x for x in k if x[3] == 0}
    assert ing == {(R.INIT_ID, 53, 17, 0), (R.HOST_ID, 0, 0, 0), (R.WORLD_ID, 0, 0, 0)}


def test_c1_restricted_and_requires(c1):
    """role=restricted: egress-default-deny.json enables egress with an
    empty rule: no egress key at all.  env=prod + role=backend:
    requires.json denies L3 from every identity without env=prod
    (rule.go:352-373 runs FromRequires before any allow)."""
    t, ctx = c1
    by_sec = {t.seclabel[x]: x for x in t.policy}
    k = keys_of(t, by_sec[256 + S.C1_LOCAL.index({"role": "restricted"})])
    assert not [x for x in k if x[3] == 1]
    k = keys_of(t, by_sec[256 + S.C1_LOCAL.index({"env": "prod", "role": "backend"})])
    l3_in = {x[0] for x in k if x[1:] == (0, 0, 0)}
    want = ids_where(ctx, lambda lb: "role=frontend" in lb and "env=prod" in lb)
    assert l3_in == want | {R.HOST_ID, R.WORLD_ID}


def test_c1_tables_shape(c1):
    t, ctx = c1
    assert len(ctx["identities"]) >= 105            # ~100 pods + reserved + CIDR
    assert len(t.policy) == len(S.C1_LOCAL)
    fam = t.ipcache["family"] == 1
    assert fam.all() and len(t.ipcache) > 150
    # every CIDR a rule names is in the ipcache under its CIDR identity
    cidr = t.ipcache[t.ipcache["label"] >= R.LOCAL_IDENTITY_FLAG]
    assert sorted(int(x) for x in cidr["plen"]) == sorted(
        ipaddress.ip_network(c).prefixlen
        for c in R.Repository(R.load_fixture(os.path.join(ROOT, S.C1_POLICIES))).cidrs())
    h = S.headers_c1(t, 50_000)
    assert len(h) == 50_000 and set(np.unique(h.proto)) <= {1, 6, 17}
