"""Incremental commits (cfc_api.cpp commit_locked): a commit re-flattens only
the table groups whose maps changed (ipcache / prefilter / endpoints+policy
/ conntrack), shares the rest with the previous epoch, and swaps without
draining the device; an epoch replaced while another stream still reads it
stays alive until that stream passes the swap.  Every result is checked
against the oracle on the updated tables.  Run on an MI355X: pytest -m gpu."""
import numpy as np
import pytest

import oracle as O
from cilium_amd import _lib as LL
from cilium_amd import ipcache, metricsmap, policymap
from cilium_amd import synth as S
from cilium_amd.datapath import Datapath, pack
from cilium_amd.loader import ct_rows, load_tables, policy_rows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "needs a GPU"
    return torch


def check(out, o, h, mode=3):
    oa, ov, oi = o.classify(h, mode, 0, nthreads=16)
    for name, a, b in (("action", out.action.cpu().numpy().astype(np.int32), oa),
                       ("verdict", out.verdict.cpu().numpy(), ov),
                       ("identity", out.identity.cpu().numpy().view(np.uint32), oi)):
        bad = np.flatnonzero(a != b)
        assert len(bad) == 0, f"{name}: {len(bad)} of {len(a)} differ, first {bad[:8]}"


def ipcache_upserts(t, rng, n):
    """n new /24../32 prefixes with fresh labels, as IPCACHE_DT rows."""
    a = rng.integers(1 << 24, 224 << 24, size=n, dtype=np.uint64).astype(np.uint32)
    plen = rng.choice(np.array([24, 28, 32]), size=n)
    a &= (np.uint32(0xFFFFFFFF) << (32 - plen).astype(np.uint32)).astype(np.uint32)
    lab = rng.integers(256, 256 + 16384, size=n).astype(np.uint32)
    return S._v4_entries(S.byteswap32(a), plen, lab)


def apply_ipcache(dp, rows):
    m = ipcache.Map(dp)
    for e in rows:
        k = ipcache.Key(32 + int(e["plen"]), int(e["family"]), bytes(e["addr"]))
        m.Update(k, ipcache.RemoteEndpointInfo(int(e["label"]), b"\0\0\0\0"))


def merge_ipcache(t, rows):
    """The oracle's table after the same upserts (a prefix already present
    takes the new label)."""
    key = lambda r: (int(r["family"]), int(r["plen"]), bytes(r["addr"]))   # noqa: E731
    d = {key(r): r for r in t.ipcache}
    for r in rows:
        d[key(r)] = r
    t.ipcache = np.array(list(d.values()), S.IPCACHE_DT)


def test_incremental_groups_and_counters(torch):
    t, flows = S.config_c5(5, n_flows=50_000, n_prefixes=20_000, n_policy=2000, now=1000)
    dp = Datapath(0)
    pms = load_tables(dp, t)
    e0 = dp.stats()["epoch"]
    h = S.headers_c5(t, flows, 300_000, seed=4)
    b = pack(h)
    o = O.Oracle(t)
    check(dp.classify(b, 3), o, h)
    # ipcache upserts: only the ipcache group is rebuilt; the counters made
    # so far stay on the device (same layout) and keep accumulating
    rng = np.random.default_rng(8)
    rows = ipcache_upserts(t, rng, 500)
    apply_ipcache(dp, rows)
    out = dp.classify(b, 3)
    assert dp.stats()["epoch"] == e0 + 1
    merge_ipcache(t, rows)
    o2 = O.Oracle(t)
    check(out, o2, h)
    # a policymap update: the endpoint group (and the counter layout) is
    # rebuilt, the counters of both batches fold first
    pm = pms[S.EP_LXC_ID]
    key = policymap.PolicyKey(S.WORLD_ID, 0, 0, 0)
    dp.update_element(pm.Fd, key.pack(), policymap.PolicyEntry(0).pack())
    t.policy[S.EP_LXC_ID] = np.concatenate(
        [t.policy[S.EP_LXC_ID][~((t.policy[S.EP_LXC_ID]["identity"] == S.WORLD_ID) &
                                 (t.policy[S.EP_LXC_ID]["dport"] == 0) &
                                 (t.policy[S.EP_LXC_ID]["proto"] == 0) &
                                 (t.policy[S.EP_LXC_ID]["egress"] == 0))],
         np.array([(S.WORLD_ID, 0, 0, 0, 0)], S.POLICY_DT)])
    out = dp.classify(b, 3)
    assert dp.stats()["epoch"] == e0 + 2
    o3 = O.Oracle(t)
    check(out, o3, h)
    dp.counters_sync()
    # counters: batch 1 on the first tables, batch 2 after the ipcache
    # change, batch 3 after the policy change; the rewritten entry restarts
    # from zero like the reference's map update
    want = {}
    for i, oo in enumerate((o, o2, o3)):
        for r in oo.policy_counters(S.EP_LXC_ID):
            k = tuple(int(x) for x in r[:4])
            if k == (S.WORLD_ID, 0, 0, 0) and i < 2:
                continue
            want[k] = want.get(k, np.zeros(2, np.uint64)) + r[5:7].astype(np.uint64)
    got = {tuple(int(x) for x in r[:4]): r[5:7]
           for r in np.array(policy_rows(pm), np.uint64).reshape(-1, 7)}
    assert set(got) == set(want)
    for k in got:
        np.testing.assert_array_equal(got[k], want[k], err_msg=str(k))
    m = np.array(metricsmap.dump_rows(dp), np.uint64).reshape(-1, 4)
    mw = {}
    for oo in (o, o2, o3):
        for r in oo.metrics():
            k = (int(r[0]), int(r[1]))
            mw[k] = mw.get(k, np.zeros(2, np.uint64)) + r[2:4].astype(np.uint64)
    assert {(int(r[0]), int(r[1])): tuple(r[2:4]) for r in m} == \
        {k: tuple(v) for k, v in mw.items()}
    dp.close()


def test_commit_while_another_stream_runs(torch):
    """A long batch on stream 1 against the old tables; meanwhile an
    ipcache change is committed and a batch classified on stream 2.  Each
    batch's results match the oracle on the tables it was launched with."""
    t = S.config_c2(7, n_prefixes=50_000, n_policy=4000)
    dp = Datapath(0)
    load_tables(dp, t)
    h1 = S.headers_c2(t, 8_000_000, seed=71)
    h2 = S.headers_c2(t, 500_000, seed=72)
    b1, b2 = pack(h1), pack(h2)
    o_old = O.Oracle(t)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    out1 = dp.classify(b1, 3, stream=s1)
    rows = ipcache_upserts(t, np.random.default_rng(9), 2000)
    apply_ipcache(dp, rows)
    dp.commit(stream=s2)
    out2 = dp.classify(b2, 3, stream=s2)
    torch.cuda.synchronize()
    check(out1, o_old, h1)
    merge_ipcache(t, rows)
    check(out2, O.Oracle(t), h2)
    dp.close()


def test_endpoint_rebuild_while_another_stream_counts(torch):
    """A long conntrack batch on stream 1; meanwhile a new policy entry
    (a structural change: the endpoint group and its counter layout are
    rebuilt) is committed on stream 2, which must fold stream 1's counts
    under the old layout first, and a second batch runs on stream 2.  Policy
    entry counters and metrics equal the oracle's run of the
    two batches on their own tables (CT accounting is compared after
    applies, in test_gpu_parity / test_gpu_fullsize)."""
    t, flows = S.config_c5(5, n_flows=50_000, n_prefixes=20_000, n_policy=2000, now=1000)
    dp = Datapath(0)
    pms = load_tables(dp, t)
    h1 = S.headers_c5(t, flows, 8_000_000, seed=81)
    h2 = S.headers_c5(t, flows, 300_000, seed=82)
    b1, b2 = pack(h1), pack(h2)
    o = O.Oracle(t)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    dp.classify(b1, 3, stream=s1)
    # an identity no header carries: the verdicts stay, the layout moves
    new = (70_000, 0, 0, 0, 0)
    pm = pms[S.EP_LXC_ID]
    dp.update_element(pm.Fd, policymap.PolicyKey(*new[:4]).pack(),
                      policymap.PolicyEntry(0).pack())
    dp.commit(stream=s2)
    out2 = dp.classify(b2, 3, stream=s2)
    dp.counters_sync(stream=s2)
    torch.cuda.synchronize()
    o.classify(h1, 3, 0, nthreads=16)
    o.L.cfo_policy_add(o.h, S.EP_LXC_ID, *new)
    t.policy[S.EP_LXC_ID] = np.concatenate(
        [t.policy[S.EP_LXC_ID], np.array([new], S.POLICY_DT)])
    check(out2, O.Oracle(t), h2)
    o.classify(h2, 3, 0, nthreads=16)
    want = {tuple(int(x) for x in r[:4]): tuple(r[5:7]) for r in o.policy_counters(S.EP_LXC_ID)}
    got = {tuple(int(x) for x in r[:4]): tuple(r[5:7])
           for r in np.array(policy_rows(pm), np.uint64).reshape(-1, 7)}
    assert got == want
    m = np.array(metricsmap.dump_rows(dp), np.uint64).reshape(-1, 4)
    assert sorted(map(tuple, m.tolist())) == sorted(map(tuple, o.metrics().tolist()))
    dp.close()


def test_in_place_patches(torch):
    """Value-only overwrites: IPv6 ipcache labels and policy proxy ports are
    patched into the live tables (the epoch stays); an IPv4 label overwrite
    rebuilds the IPv4 group only.  Results against the oracle each time."""
    t = S.config_c3(3, n_prefixes=100_000, n_v4_prefixes=10_000, n_endpoints=2,
                    n_prefilter=2000)
    dp = Datapath(0)
    pms = load_tables(dp, t)
    h6 = S.headers_c3(t, 400_000, seed=31)
    h4 = S.headers_c2(t, 200_000, seed=32)
    b6, b4 = pack(h6), pack(h4)
    e0 = dp.stats()["epoch"]
    rng = np.random.default_rng(5)
    # IPv6 labels of existing prefixes
    i6 = np.flatnonzero(t.ipcache["family"] == 2)
    pick = rng.choice(i6, size=2000, replace=False)
    rows = t.ipcache[pick].copy()
    rows["label"] = rng.integers(256, 256 + 16384, size=len(rows))
    apply_ipcache(dp, rows)
    t.ipcache["label"][pick] = rows["label"]
    out = dp.classify(b6, 0)
    assert dp.stats()["epoch"] == e0, "patched in place, no new epoch"
    check(out, O.Oracle(t), h6, mode=0)
    # policy proxy ports of existing entries
    pm = pms[S.EP_LXC_ID]
    pol = t.policy[S.EP_LXC_ID]
    sel = rng.choice(len(pol), size=200, replace=False)
    for j in sel:
        r = pol[j]
        key = policymap.PolicyKey(int(r["identity"]), int(r["dport"]), int(r["proto"]),
                                  int(r["egress"]))
        port = int(S.htons(10001 + int(j) % 4)) if r["dport"] else 0
        dp.update_element(pm.Fd, key.pack(), policymap.PolicyEntry(port).pack())
        pol["proxy_port"][j] = port
    out = dp.classify(b6, 0)
    assert dp.stats()["epoch"] == e0
    check(out, O.Oracle(t), h6, mode=0)
    # IPv4 labels: the IPv4 group is rebuilt
    i4 = np.flatnonzero(t.ipcache["family"] == 1)
    pick = rng.choice(i4, size=500, replace=False)
    rows = t.ipcache[pick].copy()
    rows["label"] = rng.integers(256, 256 + 16384, size=len(rows))
    apply_ipcache(dp, rows)
    t.ipcache["label"][pick] = rows["label"]
    out = dp.classify(b4, 0)
    assert dp.stats()["epoch"] == e0 + 1
    check(out, O.Oracle(t), h4, mode=0)
    dp.close()


def ct_table_from_maps(dp):
    """The CT maps' contents (host truth) as CT_DT records for an oracle."""
    rows = ct_rows(dp, dp.ct_fds)
    ct = np.zeros(len(rows), S.CT_DT)
    ct["family"] = rows[:, 3]
    ct["lxc"] = rows[:, 0].astype(np.int32) + rows[:, 1].astype(np.int32) * 256 - 1
    ct["any"] = rows[:, 2]
    ct["tuple"] = rows[:, 4:42]
    ct["entry"] = rows[:, 44:100]
    return ct


def check_ct(out, t, h, mode=3):
    o = O.Oracle(t)
    oa, ov, oi, oc = o.classify(h, mode, 0, nthreads=16, want_ct=True)
    for name, a, b in (("action", out.action.cpu().numpy().astype(np.int32), oa),
                       ("verdict", out.verdict.cpu().numpy(), ov),
                       ("identity", out.identity.cpu().numpy().view(np.uint32), oi),
                       ("ct", out.ct.cpu().numpy(), oc)):
        bad = np.flatnonzero(a != b)
        assert len(bad) == 0, f"{name}: {len(bad)} of {len(a)} differ, first {bad[:8]}"


@pytest.mark.parametrize("apply", ["device", "host"])
def test_ct_patched_in_place(torch, apply):
    """CT creates (cfc_ct_apply), deletes and re-inserts through the map API
    are patched into the live CT table: the epoch stays, deleted slots
    become tombstones that later inserts reuse.  Past 3/4 load the CT group
    is rebuilt instead.  Each step against an oracle built from the CT
    maps' contents."""
    t, flows = S.config_c5(5, n_flows=50_000, n_prefixes=20_000, n_policy=2000, now=1000)
    dp = Datapath(0)
    dp.set_option(LL.OPT_CT_APPLY, LL.CT_APPLY_DEVICE if apply == "device" else LL.CT_APPLY_HOST)
    load_tables(dp, t)
    h = S.headers_c5(t, flows, 300_000, seed=11)
    b = pack(h)
    out = dp.classify(b, 3, want_ct=True)
    e0, n0 = dp.stats()["epoch"], dp.stats()["ct4_entries"]
    check_ct(out, t, h)
    dp.ct_apply(b, out, 3)
    # the writes of batch 1 are in the live table: same epoch
    h2 = S.headers_c5(t, flows, 300_000, seed=12)
    b2 = pack(h2)
    out = dp.classify(b2, 3, want_ct=True)
    t.ct = ct_table_from_maps(dp)
    st = dp.stats()
    # creates and deletes (established flows the policy now denies)
    assert st["epoch"] == e0 and st["ct4_entries"] != n0
    check_ct(out, t, h2)
    # deletes through the map API (global v4 maps)
    rng = np.random.default_rng(3)
    fds = {k: fd for k, fd in dp.ct_fds.items() if k[0] == 1 and k[1] == -1}
    gone = {}
    for k, fd in fds.items():
        keys, vals = dp.dump(fd)
        sel = rng.choice(len(keys), size=min(5000, len(keys) // 4), replace=False)
        gone[k] = (keys[sel], vals[sel])
        for kk in keys[sel]:
            dp.delete_element(fd, kk.tobytes())
    out = dp.classify(b2, 3, want_ct=True)
    assert dp.stats()["epoch"] == e0
    t.ct = ct_table_from_maps(dp)
    check_ct(out, t, h2)
    # the same entries back: they land in the deleted slots
    for k, (keys, vals) in gone.items():
        dp.update_batch(fds[k], keys, vals)
    out = dp.classify(b2, 3, want_ct=True)
    assert dp.stats()["epoch"] == e0
    t.ct = ct_table_from_maps(dp)
    check_ct(out, t, h2)
    # bulk inserts, 20k per commit, until the table passes 3/4 load and the
    # CT group is rebuilt
    for it in range(40):
        for k, fd in fds.items():
            keys, vals = dp.dump(fd)
            rep = rng.integers(0, len(keys), size=10_000)
            nk = keys[rep].copy()
            nk[:, 8:12] = rng.integers(0, 256, size=(len(rep), 4), dtype=np.uint8)
            dp.update_batch(fd, nk, vals[rep])
        out = dp.classify(b2, 3, want_ct=True)
        if dp.stats()["epoch"] != e0:
            break
    assert dp.stats()["epoch"] == e0 + 1 and it > 0
    t.ct = ct_table_from_maps(dp)
    check_ct(out, t, h2)
    dp.close()
