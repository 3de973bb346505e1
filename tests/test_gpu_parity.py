"""GPU parity: the HIP engine (libcfc.so, through its C ABI) against
  (1) the golden vectors produced by the reference's BPF programs, and
  (2) the pinned CPU oracle on larger seeded streams, every output and
      every counter bit-exact, for all modes and table shapes.
Run on an MI355X: pytest -m gpu."""
import numpy as np
import pytest

import golden_io as G
import oracle as O
from cilium_amd import synth as S
from cilium_amd import _lib as L
from cilium_amd import metricsmap
from cilium_amd.datapath import Datapath, pack, pack_v4
from cilium_amd.loader import ct_rows, load_tables, policy_rows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "needs a GPU"
    return torch


LAYOUTS = {"dir24_8": L.LPM4_DIR24_8, "trie": L.LPM4_TRIE}


def run_gpu(torch, t, h, mode, ep_lxc=0, chunks=1, lpm4=L.LPM4_AUTO,
            ct_apply=L.CT_APPLY_DEVICE, interpose=False):
    dp = Datapath(0)
    dp.set_option(L.OPT_LPM4, lpm4)
    dp.set_option(L.OPT_CT_APPLY, ct_apply)
    pms = load_tables(dp, t)
    if lpm4 != L.LPM4_AUTO and (t.ipcache["family"] == 1).any():
        assert dp.stats()["lpm4_layout"] == lpm4
    b = pack(h)
    n = len(h)
    act = np.empty(n, np.int32)
    ver = np.empty(n, np.int32)
    ide = np.empty(n, np.uint32)
    ctb = np.empty(n, np.uint8)
    use_ct = getattr(t, "ct", None) is not None
    step = (n + chunks - 1) // chunks
    for a in range(0, n, step):
        sub = b.slice(a, a + step)
        out = dp.classify(sub, mode, ep_lxc, want_ct=use_ct)
        if use_ct:   # fold this batch's creates/deletes before the next one
            if interpose:   # another (empty) launch in between: the apply probes
                import ctypes
                from cilium_amd.datapath import hdr_struct, out_struct
                hdr = hdr_struct(sub)
                hdr.n = 0
                L.check(dp.L.cfc_classify_v4(dp.h, ctypes.byref(hdr),
                                             ctypes.byref(out_struct(out)), mode,
                                             ep_lxc, dp._stream(None)), "classify")
            dp.ct_apply(sub, out, mode, ep_lxc)
            ctb[a:a + step] = out.ct.cpu().numpy()
        torch.cuda.synchronize()
        act[a:a + step] = out.action.cpu().numpy()
        ver[a:a + step] = out.verdict.cpu().numpy()
        ide[a:a + step] = out.identity.cpu().numpy().view(np.uint32)
    dp.counters_sync()
    counters = {lxc: np.array(policy_rows(pm), np.uint64).reshape(-1, 7)
                for lxc, pm in pms.items()}
    metrics = np.array(metricsmap.dump_rows(dp), np.uint64).reshape(-1, 4)
    run_gpu.ct = (ctb, ct_rows(dp, dp.ct_fds)) if use_ct else None
    run_gpu.identity = dp.identity_counters()
    run_gpu.stats = dp.stats()
    dp.close()
    return act, ver, ide, counters, metrics


@pytest.mark.parametrize("layout", sorted(LAYOUTS))
@pytest.mark.parametrize("name", G.names())
def test_golden(torch, name, layout):
    g = G.Golden(name)
    act, ver, ide, counters, metrics = run_gpu(torch, g.tables, g.headers,
                                               g.mode, g.ep_lxc,
                                               lpm4=LAYOUTS[layout])
    bad = G.mismatches(g, act, ver, ide)
    assert len(bad) == 0, f"{len(bad)} differ; first {bad[:8]}"
    for lxc, exp in g.counters.items():
        np.testing.assert_array_equal(counters[lxc], exp)
    np.testing.assert_array_equal(metrics, g.metrics)
    # and every output, identity bits included, against the pinned oracle
    o = O.Oracle(g.tables)
    use_ct = g.ct_after is not None
    oa, ov, oi, oct_ = o.classify(g.headers, g.mode, g.ep_lxc, nthreads=8,
                                  want_ct=True, apply_ct=use_ct)
    np.testing.assert_array_equal(act, oa)
    np.testing.assert_array_equal(ver, ov)
    np.testing.assert_array_equal(ide, oi)
    np.testing.assert_array_equal(run_gpu.identity, o.identity_counters())
    if use_ct:
        # CT byte per header, and the CT maps afterwards: against the
        # reference (clock-derived fields masked) and, every byte, the oracle
        ctb, rows = run_gpu.ct
        np.testing.assert_array_equal(ctb, oct_)
        a, b = G.ct_masked(rows), G.ct_masked(g.ct_after)
        if a.shape == b.shape:
            for r in np.nonzero((a != b).any(1))[0][:4]:
                cols = np.nonzero(a[r] != b[r])[0]
                print("ct row", r, cols, a[r][cols], b[r][cols], a[r].tobytes().hex())
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(rows, o.ct_dump())


def compare_with_oracle(torch, t, h, mode, ep_lxc=0, chunks=1, lpm4=L.LPM4_AUTO,
                        ct_apply=L.CT_APPLY_DEVICE, interpose=False):
    act, ver, ide, counters, metrics = run_gpu(torch, t, h, mode, ep_lxc, chunks,
                                               lpm4, ct_apply, interpose)
    o = O.Oracle(t)
    use_ct = getattr(t, "ct", None) is not None
    if use_ct:   # the same batches, each folded into CT before the next
        step = (len(h) + chunks - 1) // chunks
        parts = [o.classify(h.slice(a, a + step), mode, ep_lxc, nthreads=16,
                            want_ct=True, apply_ct=True)
                 for a in range(0, len(h), step)]
        oa, ov, oi, oct_ = (np.concatenate([p[k] for p in parts]) for k in range(4))
        ctb, rows = run_gpu.ct
        bad = np.nonzero(ctb != oct_)[0]
        assert len(bad) == 0, f"ct byte: {len(bad)} differ, first {bad[:8]}"
        want = o.ct_dump()
        if rows.shape == want.shape:
            for r in np.nonzero((rows != want).any(1))[0][:6]:
                cols = np.nonzero(rows[r] != want[r])[0]
                print("ct row", r, cols, rows[r][cols], want[r][cols],
                      rows[r].tobytes().hex())
        else:
            print("ct rows", rows.shape, want.shape)
        np.testing.assert_array_equal(rows, want)
    else:
        oa, ov, oi = o.classify(h, mode, ep_lxc, nthreads=16)
    for name, a, b in (("action", act, oa), ("verdict", ver, ov),
                       ("identity", ide, oi)):
        bad = np.nonzero(a != b)[0]
        assert len(bad) == 0, f"{name}: {len(bad)} differ, first {bad[:8]}"
    for lxc in t.policy:
        np.testing.assert_array_equal(counters[lxc], o.policy_counters(lxc))
    np.testing.assert_array_equal(metrics, o.metrics())
    np.testing.assert_array_equal(run_gpu.identity, o.identity_counters())
    return act, ver


@pytest.mark.parametrize("mode", [0, 2, 3])
def test_c2_full_tables_vs_oracle(torch, mode):
    """C2 tables (100k prefixes, 16k policy entries), 4M headers."""
    t = S.config_c2(2)
    t.prefilter = _prefilter(t)
    h = S.headers_c2(t, 4_000_000, seed=21)
    act, ver = compare_with_oracle(torch, t, h, mode, chunks=3)
    assert len(np.unique(act)) >= 2


def test_c2_layouts_and_auto_choice(torch):
    """The layout AUTO picks at C2 scale, and the other one forced, give the
    same bits."""
    t = S.config_c2(2)
    dp = Datapath(0)
    load_tables(dp, t)
    st = dp.stats()
    dp.close()
    assert st["lpm4_layout"] == L.LPM4_TRIE
    assert st["lpm4_kib"] <= 4096
    h = S.headers_c2(t, 1_000_000, seed=23)
    compare_with_oracle(torch, t, h, 0, lpm4=L.LPM4_DIR24_8)


def _prefilter(t):
    rng = np.random.default_rng(99)
    pf = np.zeros(3000, S.PREFILTER_DT)
    pf["family"] = 1
    pf["plen"][:2500] = 32
    pf["plen"][2500:] = rng.choice([8, 16, 20, 24, 30], size=500)
    addr = rng.integers(1 << 24, 224 << 24, size=3000, dtype=np.uint64).astype(np.uint32)
    host = addr & (np.uint64(0xFFFFFFFF) << (32 - pf["plen"].astype(np.uint64))).astype(np.uint32)
    pf["addr"][:, :4] = S.be32_to_bytes(S.byteswap32(host))
    pf["dyn"][2500:] = 1
    _, u = np.unique(np.stack([pf["dyn"], pf["plen"], host], 1), axis=0,
                     return_index=True)
    return pf[np.sort(u)]


def test_c2_egress_vs_oracle(torch):
    t = S.config_c2(3, n_endpoints=3)
    rng = np.random.default_rng(5)
    h = S.gen_headers_v4(rng, 2_000_000, t.ipcache, S.local_v4_addrs(t),
                         local_frac=0.1, src_fixed=S.LXC_IPV4)
    h.saddr[rng.random(len(h)) < 0.01] = S.ip4("64.48.32.17")
    compare_with_oracle(torch, t, h, 1, ep_lxc=S.EP_LXC_ID)


def test_many_endpoints_global_counter_path(torch):
    """> LDS_CTR_MAX policy entries in total: global-atomic counter path."""
    t = S.config_c2(4, n_prefixes=20_000, n_policy=8000, n_endpoints=4)
    h = S.headers_c2(t, 1_000_000, seed=4)
    compare_with_oracle(torch, t, h, 0)


@pytest.mark.parametrize("layout", sorted(LAYOUTS))
def test_wide_labels_and_edge_tables(torch, layout):
    """identities >= 2^30 (indirect LPM leaves), /0 and /32 prefixes,
    labels HOST/CLUSTER/0 that the ingress override ignores."""
    rng = np.random.default_rng(11)
    ipc = S.gen_ipcache_v4(rng, 5000)
    ipc["label"][:100] = 0x40000000 + np.arange(100)
    ipc["label"][100:120] = S.HOST_ID
    ipc["label"][120:140] = S.CLUSTER_ID
    ipc["label"][140:160] = 0
    ipc["label"][160:180] = (1 << 26) + np.arange(20)   # > a list entry's leaf field
    ipc = np.concatenate([ipc, S._v4_entries(np.array([0], np.uint32), [0], [77])])
    t = S.Tables(ipc, S.config_c2(1, n_prefixes=10, n_policy=10).endpoints, {},
                 np.zeros(0, S.PREFILTER_DT), {S.EP_LXC_ID: 2})
    idents = np.unique(ipc["label"])
    t.policy = {S.EP_LXC_ID: S.gen_policy(rng, 3000, idents, proxy_frac=0.1)}
    h = S.gen_headers_v4(rng, 500_000, ipc, S.local_v4_addrs(t),
                         proxy_ident=idents[:50], frag=0.05, other_proto=0.02)
    compare_with_oracle(torch, t, h, 0, lpm4=LAYOUTS[layout])


def test_empty_tables(torch):
    t = S.Tables(np.zeros(0, S.IPCACHE_DT), np.zeros(0, S.ENDPOINT_DT), {},
                 np.zeros(0, S.PREFILTER_DT), {})
    rng = np.random.default_rng(1)
    h = S.gen_headers_v4(rng, 10000, S.gen_ipcache_v4(rng, 10),
                         np.array([S.LXC_IPV4], np.uint32))
    for mode in (0, 2, 3):
        compare_with_oracle(torch, t, h, mode)


def test_counters_accumulate_across_batches_and_updates(torch):
    """Counters fold into policy values across launches; a policymap update
    between launches resets that entry like the kernel's map update does."""
    t = S.config_c2(6, n_prefixes=2000, n_policy=500)
    h = S.headers_c2(t, 200_000, seed=6)
    dp = Datapath(0)
    pms = load_tables(dp, t)
    b = pack_v4(h)
    dp.classify_v4(b, 0)
    dp.classify_v4(b, 0)
    dp.counters_sync()
    o = O.Oracle(t)
    o.classify(h, 0, nthreads=8)
    o.classify(h, 0, nthreads=8)
    np.testing.assert_array_equal(np.array(policy_rows(pms[S.EP_LXC_ID]), np.uint64),
                                  o.policy_counters(S.EP_LXC_ID))
    # reset one hit entry through the mirror API, classify again
    pm = pms[S.EP_LXC_ID]
    top = max(pm.DumpToSlice(), key=lambda d: d.PolicyEntry.Packets)
    assert top.PolicyEntry.Packets > 0
    from cilium_amd import policymap
    dp.update_element(pm.Fd, top.Key.pack(),
                      policymap.PolicyEntry(top.PolicyEntry.ProxyPort).pack())
    dp.classify_v4(b, 0)
    dp.counters_sync()
    after = pm.Lookup(top.Key)
    o2 = O.Oracle(t)
    o2.classify(h, 0, nthreads=8)
    rows = {tuple(r[:4]): r for r in o2.policy_counters(S.EP_LXC_ID)}
    k = top.Key
    exp = rows[(k.Identity, k.DestPort, k.Nexthdr, k.TrafficDirection)]
    assert (after.Packets, after.Bytes) == (exp[5], exp[6])
    dp.close()


# ------------------------------------------------------------------ IPv6
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_c3_vs_oracle(torch, mode):
    """C3-shaped dual-stack tables (200k IPv6 + 20k IPv4 prefixes, 20k-entry
    prefilter), 1M IPv6 headers, every mode."""
    t = S.config_c3(3, n_prefixes=200_000, n_v4_prefixes=20_000,
                    n_endpoints=3, n_prefilter=20_000)
    rng = np.random.default_rng(30 + mode)
    if mode == 1:
        ipc6 = t.ipcache[t.ipcache["family"] == 2]
        h = S.gen_headers_v6(rng, 1_000_000, ipc6, S.local_v6_addrs(t),
                             local_frac=0.1, src_fixed=S.LXC_IPV6, ext=0.05,
                             exthdr_drop=0.01, mark_host=0, mark_proxy=0)
        h.daddr = S._addr_in_prefix_v6(rng, ipc6, rng.integers(0, len(ipc6), size=len(h)))
        r = rng.random(len(h))
        loc = S.local_v6_addrs(t)
        h.daddr[r < 0.1] = loc[rng.integers(0, len(loc), size=int((r < 0.1).sum()))]
        cl = r > 0.97
        h.daddr[cl, :8] = S.ROUTER_IPV6[:8]
        h.saddr[rng.random(len(h)) < 0.01] = S.ip6("2001:db8::dead")
    else:
        h = S.headers_c3(t, 1_000_000, seed=31 + mode, ext=0.05, exthdr_drop=0.01,
                         local_frac=0.9)
        if mode in (2, 3):
            fix = t.prefilter[(t.prefilter["family"] == 2) & (t.prefilter["dyn"] == 0)]
            sel = rng.random(len(h)) < 0.2
            h.saddr[sel] = fix["addr"][rng.integers(0, len(fix), size=int(sel.sum()))]
    # punted ICMPv6 (NS, echo request to the router) in every mode
    k = np.arange(0, len(h), 997)
    h.proto[k] = 58
    h.sport[k] = np.where(k % 2, 135, 128).astype(np.uint16)
    h.daddr[k[k % 4 == 0]] = S.ROUTER_IPV6
    act, ver = compare_with_oracle(torch, t, h, mode, ep_lxc=S.EP_LXC_ID, chunks=2)
    # XDP verdicts are pass/drop only; the tc modes also see proxy ports
    assert len(np.unique(ver)) >= (2 if mode == 2 else 3)


def _v6_entries(rng, specs):
    out = []
    for n, lens, labels in specs:
        a = rng.integers(0, 256, size=(n, 16), dtype=np.uint16).astype(np.uint8)
        a[:, 0] = 0x20 | (a[:, 0] & 0x0F)
        out.append(S._v6_entries(a, rng.choice(lens, size=n), labels))
    e = np.concatenate(out)
    _, u = np.unique(np.concatenate([e["plen"][:, None], e["addr"]], 1), axis=0,
                     return_index=True)
    return e[np.sort(u)]


def test_v6_edge_tables(torch):
    """Every length /1-/128, labels >= 2^30, 0 (shadowing shorter prefixes),
    HOST and CLUSTER, a ::/0 entry; prefixes piled under one /48 and /64
    (the Bloom groups split); a dynamic v6 prefilter."""
    rng = np.random.default_rng(17)
    ipc = _v6_entries(rng, [(20000, np.arange(1, 129), 256 + np.arange(20000) % 5000)])
    ipc["label"][:200] = 0x40000000 + np.arange(200)
    ipc["label"][200:400] = 0
    ipc["label"][400:450] = S.HOST_ID
    ipc["label"][450:500] = S.CLUSTER_ID
    base = S.ip6("2001:db8:5::")
    pods = np.tile(base, (3000, 1))
    pods[:, 6:8] = rng.integers(0, 4, size=(3000, 2))
    pods[:, 8:] = rng.integers(0, 256, size=(3000, 8))
    piled = np.concatenate([
        S._v6_entries(pods, [128] * 3000, 9000 + np.arange(3000)),
        S._v6_entries(pods[:40], [64] * 40, 8000 + np.arange(40)),
        S._v6_entries(base[None, :], [48], [7777]),
        S._v6_entries(np.zeros((1, 16), np.uint8), [0], [77])])
    ipc = np.concatenate([ipc, piled])
    _, u = np.unique(np.concatenate([ipc["plen"][:, None], ipc["addr"]], 1), axis=0,
                     return_index=True)
    ipc = ipc[np.sort(u)]
    t = S.config_c3(5, n_prefixes=10, n_v4_prefixes=10, n_policy=10, n_prefilter=0)
    t.ipcache = ipc
    idents = np.unique(ipc["label"])
    t.policy = {S.EP_LXC_ID: S.gen_policy(rng, 4000, idents, proxy_frac=0.1)}
    pf = np.zeros(600, S.PREFILTER_DT)
    pf["family"] = 2
    pf["dyn"] = 1
    pa = rng.integers(0, 256, size=(600, 16), dtype=np.uint16).astype(np.uint8)
    pa[:, 0] = 0x30 | (pa[:, 0] & 0x0F)
    pl = rng.integers(8, 129, size=600)
    pf["plen"] = pl
    pf["addr"] = S.mask_v6(pa, pl)
    _, u = np.unique(np.concatenate([pf["plen"][:, None], pf["addr"]], 1), axis=0,
                     return_index=True)
    t.prefilter = pf[np.sort(u)]
    h = S.headers_c3(t, 600_000, seed=17, ext=0.05, local_frac=0.9)
    h.saddr[::5] = S._addr_in_prefix_v6(rng, t.ipcache[-3100:],
                                        rng.integers(0, 3100, size=len(h.saddr[::5])))
    h.saddr[1::7] = S._addr_in_prefix_v6(rng, t.prefilter, rng.integers(0, len(t.prefilter), size=len(h.saddr[1::7])))
    dp = Datapath(0)
    load_tables(dp, t)
    st = dp.stats()
    dp.close()
    assert st["lpm6_lengths"] == 128 and st["lpm6_groups"] >= 2, st
    for mode in (0, 3):
        compare_with_oracle(torch, t, h, mode)


def test_v6_only_endpoints_and_empty(torch):
    """No IPv4 state at all; then no tables at all."""
    t = S.config_c3(8, n_prefixes=5000, n_v4_prefixes=10, n_policy=500, n_prefilter=0)
    t.ipcache = t.ipcache[t.ipcache["family"] == 2]
    t.endpoints = t.endpoints[t.endpoints["family"] == 2]
    h = S.headers_c3(t, 100_000, seed=8)
    for mode in (0, 2, 3):
        compare_with_oracle(torch, t, h, mode)
    e = S.Tables(np.zeros(0, S.IPCACHE_DT), np.zeros(0, S.ENDPOINT_DT), {},
                 np.zeros(0, S.PREFILTER_DT), {})
    for mode in (0, 2, 3):
        compare_with_oracle(torch, e, h, mode)


@pytest.mark.parametrize("apply", ["device", "host"])
@pytest.mark.parametrize("mode", [0, 3])
def test_c5_conntrack_vs_oracle(torch, mode, apply):
    """C5 shape at reduced size: 300k live flows (Zipf traffic, ESTABLISHED
    and REPLY packets, 5% new flows), three batches each folded into CT
    (cfc_ct_apply, on the device or the host) before the next: outputs, CT
    bytes, policy counters, metrics and every CT entry (accounting
    included) bit-exact."""
    t, flows = S.config_c5(5, n_flows=300_000, n_prefixes=100_000)
    h = S.headers_c5(t, flows, 1_200_000, seed=31)
    act, ver = compare_with_oracle(
        torch, t, h, mode, chunks=3,
        ct_apply=L.CT_APPLY_DEVICE if apply == "device" else L.CT_APPLY_HOST)
    st = run_gpu.stats
    assert (st["ct_apply_device"], st["ct_apply_host"]) == ((3, 0) if apply == "device"
                                                             else (0, 3))
    assert (ver == 0).sum() > len(h) // 3


def test_c5_conntrack_apply_after_other_launch(torch):
    """The device apply of a batch whose classify launch is no longer the
    last one (an empty launch in between): it cannot take the launch's hit
    slots from the workspace and probes the table itself — same CT entries,
    accounting included, as the oracle."""
    t, flows = S.config_c5(5, n_flows=300_000, n_prefixes=100_000)
    h = S.headers_c5(t, flows, 1_200_000, seed=37)
    compare_with_oracle(torch, t, h, 3, chunks=3, interpose=True)
    assert run_gpu.stats["ct_apply_device"] == 3


def test_c5_egress_and_local_ct(torch):
    """Egress with local delivery: the sender's and the receiver's CT maps
    (per-endpoint local maps), two batches with apply in between."""
    g = G.Golden("ct_egress_v4")
    t = g.tables
    rng = np.random.default_rng(5)
    h = S.concat([g.headers] * 3)
    h = S.take(h, rng.permutation(len(h)))
    compare_with_oracle(torch, t, h, 1, ep_lxc=S.EP_LXC_ID, chunks=2)


def test_node_config_runtime(torch):
    """cfc_set_node_config: IPV4_CLUSTER_RANGE/MASK and ROUTER_IP other than
    the compiled-in node_config.h values (daemon/daemon.go:916-934) change
    the egress CLUSTER_ID fallback and the ICMPv6 router punt exactly as
    the oracle configured the same way."""
    rng = np.random.default_rng(41)
    # IPv4: cluster 10.0.0.0/8 (raw be32 0x0a, mask 0xff)
    t = S.config_c2(41, n_prefixes=20_000, n_policy=4000, n_endpoints=2)
    t.node = (0x0000000A, 0x000000FF, S.ip6("fd00:1:2:3::1"))
    h = S.gen_headers_v4(rng, 300_000, t.ipcache, S.local_v4_addrs(t),
                         local_frac=0.1, src_fixed=S.LXC_IPV4)
    cl = rng.random(len(h)) < 0.3
    h.daddr[cl] = (h.daddr[cl] & np.uint32(0xFFFFFF00)) | np.uint32(0x0A)
    act, ver = compare_with_oracle(torch, t, h, 1, ep_lxc=S.EP_LXC_ID)
    # IPv6: destinations inside the configured router /64, echo requests to it
    t6 = S.config_c3(42, n_prefixes=20_000, n_v4_prefixes=100, n_policy=2000,
                     n_endpoints=2, n_prefilter=0)
    router = S.ip6("fd00:1:2:3::1")
    t6.node = (0x0000000A, 0x000000FF, router)
    ipc6 = t6.ipcache[t6.ipcache["family"] == 2]
    h6 = S.gen_headers_v6(rng, 300_000, ipc6, S.local_v6_addrs(t6), local_frac=0.1,
                          src_fixed=S.LXC_IPV6, mark_host=0, mark_proxy=0)
    sel = rng.random(len(h6)) < 0.3
    h6.daddr[sel, :8] = router[:8]
    k = np.arange(0, len(h6), 101)
    h6.proto[k] = 58
    h6.sport[k] = 128
    h6.daddr[k] = router
    h6.flags[k] = 0
    for mode, ep in ((1, S.EP_LXC_ID), (0, 0)):
        compare_with_oracle(torch, t6, h6, mode, ep_lxc=ep)
    o = O.Oracle(t6)
    _, ov, oi = o.classify(h6, 1, S.EP_LXC_ID)
    assert (ov == L.VERDICT_PUNT).sum() >= len(k) // 2
    assert (oi == S.CLUSTER_ID).sum() > 1000


@pytest.mark.parametrize("apply", ["device", "host"])
@pytest.mark.parametrize("mode", [0, 3])
def test_c5_v6_conntrack_vs_oracle(torch, mode, apply):
    """IPv6 conntrack writes (ct_create6 / ct_delete6 / timers, conntrack.h:
    615-662) on the device CT6 table: 100k live IPv6 flows, Zipf traffic,
    three batches each folded into CT before the next; outputs, CT bytes,
    counters and every CT6 entry (rev_nat_index, accounting) bit-exact
    against the oracle, and no batch on the host walk."""
    t, flows = S.config_c5_v6(6, n_flows=100_000, n_prefixes=50_000)
    h = S.headers_c5_v6(t, flows, 600_000, seed=41)
    compare_with_oracle(
        torch, t, h, mode, chunks=3,
        ct_apply=L.CT_APPLY_DEVICE if apply == "device" else L.CT_APPLY_HOST)
    st = run_gpu.stats
    assert (st["ct_apply_device"], st["ct_apply_host"]) == ((3, 0) if apply == "device"
                                                             else (0, 3))


def test_c5_v6_egress_and_local_ct(torch):
    """IPv6 egress with local delivery (the sender's and the receiver's CT6
    maps), the reference's ct_egress_v6 stream three times over in two
    batches, on the device table."""
    g = G.Golden("ct_egress_v6")
    rng = np.random.default_rng(6)
    h = S.concat([g.headers] * 3)
    h = S.take(h, rng.permutation(len(h)))
    compare_with_oracle(torch, g.tables, h, g.mode, ep_lxc=g.ep_lxc, chunks=2)
    assert run_gpu.stats["ct_apply_host"] == 0
