"""GPU parity of the drop notifications (cfc_drop_notify_v4/v6): the
struct drop_notify records (bpf/lib/drop.h:40-78) of every dropped header, in
header order, against the pinned oracle — which the CPU suite pins to the
send_drop_notify arguments the reference left in skb->cb[]
(test_oracle_golden.py).  Run on an MI355X: pytest -m gpu."""
import numpy as np
import pytest

import golden_io as G
import oracle as O
from cilium_amd import synth as S
from cilium_amd.datapath import Datapath, pack
from cilium_amd.loader import load_tables

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "needs a GPU"
    return torch


def gpu_notify(torch, t, h, mode, ep_lxc=0, cap=None, chunks=1, seq=False):
    """-> per chunk: (notify words, records, header indices, total).  seq:
    each chunk classified and folded into the CT maps (cfc_ct_apply, which
    rewrites the event words into the reference's packet order)."""
    dp = Datapath(0)
    load_tables(dp, t)
    b = pack(h)
    n = len(h)
    step = max(1, (n + chunks - 1) // chunks)
    res = []
    for a in range(0, max(n, 1), step):
        sub = b.slice(a, a + step)
        out = dp.classify(sub, mode, ep_lxc, want_notify=True, want_ct=seq)
        if seq:
            dp.ct_apply(sub, out, mode, ep_lxc)
        rec, idx, total = dp.drop_notify(sub, out, mode, ep_lxc, cap=cap)
        torch.cuda.synchronize()
        words = out.notify.cpu().numpy().view(np.uint32)
        recs = np.ascontiguousarray(rec.cpu().numpy()).view(O.DROP_NOTIFY_DT).reshape(-1)
        res.append((a, words, recs, idx.cpu().numpy().astype(np.uint64), total))
    dp.close()
    return res


def oracle_notify(t, h, mode, ep_lxc=0, seq=False):
    o = O.Oracle(t)
    act, ver, ide, nt = o.classify(h, mode, ep_lxc, nthreads=8,
                                   want_notify=True, apply_ct=seq)
    rec, idx = o.drop_notify(h, mode, ep_lxc, ver, ide, nt)
    return nt, rec, idx


def check(torch, t, h, mode, ep_lxc=0, chunks=1, seq=False):
    nt, rec, idx = oracle_notify(t, h, mode, ep_lxc, seq)
    got = gpu_notify(torch, t, h, mode, ep_lxc, chunks=chunks, seq=seq)
    words = np.concatenate([g[1] for g in got])[:len(h)]
    np.testing.assert_array_equal(words, nt)
    grec = np.concatenate([g[2] for g in got])
    gidx = np.concatenate([g[3] + np.uint64(g[0]) for g in got])
    assert sum(g[4] for g in got) == len(rec)
    np.testing.assert_array_equal(gidx, idx)
    for k in O.DROP_NOTIFY_DT.names:
        np.testing.assert_array_equal(grec[k], rec[k], err_msg=k)
    return rec


NAMES = [n for n in G.names() if G.Golden(n).cb is not None]


@pytest.mark.parametrize("name", NAMES)
def test_golden_notify(torch, name):
    g = G.Golden(name)
    # (a fixture with CT state: classify + cfc_ct_apply, the reference's
    # packet order, against the oracle's sequential run)
    rec = check(torch, g.tables, g.headers, g.mode, g.ep_lxc, seq=g.ct_after is not None)
    want_idx, want = G.expected_drop_notify(g)
    assert len(rec) == len(want_idx)
    np.testing.assert_array_equal(rec["subtype"].astype(np.int64),
                                  want["subtype"])


@pytest.mark.parametrize("mode", [0, 1, 3])
def test_c2_notify_vs_oracle(torch, mode):
    """C2 tables, 2M headers, three endpoints (local delivery drops on the
    egress side too)."""
    t = S.config_c2(2, n_endpoints=3)
    rng = np.random.default_rng(40 + mode)
    if mode == 1:
        h = S.gen_headers_v4(rng, 2_000_000, t.ipcache, S.local_v4_addrs(t),
                             local_frac=0.3, src_fixed=S.LXC_IPV4)
        h.saddr[rng.random(len(h)) < 0.01] = S.ip4("64.48.32.17")
    else:
        h = S.headers_c2(t, 2_000_000, seed=41 + mode)
    rec = check(torch, t, h, mode, S.EP_LXC_ID if mode == 1 else 0, chunks=2)
    assert len(np.unique(rec["subtype"])) >= 2 and len(rec) > 1000


@pytest.mark.parametrize("mode", [0, 1])
def test_c3_v6_notify_vs_oracle(torch, mode):
    t = S.config_c3(3, n_prefixes=50_000, n_v4_prefixes=5_000,
                    n_endpoints=3, n_prefilter=2_000)
    rng = np.random.default_rng(50 + mode)
    if mode == 1:
        ipc6 = t.ipcache[t.ipcache["family"] == 2]
        loc = S.local_v6_addrs(t)
        h = S.gen_headers_v6(rng, 500_000, ipc6, loc, local_frac=0.3,
                             src_fixed=S.LXC_IPV6, ext=0.05, exthdr_drop=0.01,
                             mark_host=0, mark_proxy=0)
    else:
        h = S.headers_c3(t, 500_000, seed=52, ext=0.05, exthdr_drop=0.01,
                         local_frac=0.9)
    rec = check(torch, t, h, mode, S.EP_LXC_ID if mode == 1 else 0)
    assert len(rec) > 100


def test_conntrack_notify_vs_oracle(torch):
    """With CT maps: replies pass, denied established flows still notify."""
    g = G.Golden("ct_ingress_v4")
    check(torch, g.tables, g.headers, g.mode, g.ep_lxc)


def test_cap_and_empty(torch):
    g = G.Golden("c2_ingress_v4")
    nt, rec, idx = oracle_notify(g.tables, g.headers, g.mode)
    (a, words, grec, gidx, total), = gpu_notify(torch, g.tables, g.headers,
                                                g.mode, cap=100)
    assert total == len(rec) > 100
    assert len(grec) == 100
    np.testing.assert_array_equal(gidx, idx[:100])
    np.testing.assert_array_equal(grec.view(np.uint8), rec[:100].view(np.uint8))
    e = G.Golden("empty_ingress_v4")
    h0 = e.headers
    (a, words, grec, gidx, total), = gpu_notify(torch, e.tables, h0, e.mode)
    assert total == int((oracle_notify(e.tables, h0, e.mode)[0] != 0).sum())


def test_two_streams(torch):
    """Back-to-back calls on two streams share the notify workspace: the
    second waits for the first's kernels (hipStreamWaitEvent on the
    library's event), with no host synchronisation between them."""
    g = G.Golden("c2_ingress_v4")
    dp = Datapath(0)
    load_tables(dp, g.tables)
    b = pack(g.headers)
    out = dp.classify(b, g.mode, g.ep_lxc, want_notify=True)
    small_b = b.slice(0, 5000)
    small_out = dp.classify(small_b, g.mode, g.ep_lxc, want_notify=True)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    # a large batch on s1, then a small one on s2, neither waited for
    big = dp.drop_notify(b, out, g.mode, g.ep_lxc, stream=s1, sync=False)
    small = dp.drop_notify(small_b, small_out, g.mode, g.ep_lxc, stream=s2,
                           sync=False)
    torch.cuda.synchronize()
    nt, rec, idx = oracle_notify(g.tables, g.headers, g.mode)
    nb = int(big[2].item())
    assert nb == len(rec)
    np.testing.assert_array_equal(big[1][:nb].cpu().numpy().astype(np.uint64), idx)
    np.testing.assert_array_equal(
        np.ascontiguousarray(big[0][:nb].cpu().numpy()).view(np.uint8).reshape(-1),
        rec.view(np.uint8))
    ns = int(small[2].item())
    k = int((idx < 5000).sum())
    assert ns == k
    np.testing.assert_array_equal(small[1][:ns].cpu().numpy().astype(np.uint64), idx[:k])
    np.testing.assert_array_equal(
        np.ascontiguousarray(small[0][:ns].cpu().numpy()).view(np.uint8).reshape(-1),
        rec[:k].view(np.uint8))
    dp.close()


def test_records_use_the_classified_epoch(torch):
    """An endpoint's SECLABEL changed between classify and drop_notify: the
    records carry the labels the batch was classified with (the epoch's
    snapshot), not the new ones."""
    g = G.Golden("c2_egress_v4")
    dp = Datapath(0)
    load_tables(dp, g.tables)
    b = pack(g.headers)
    out = dp.classify(b, g.mode, g.ep_lxc, want_notify=True)
    dp.endpoint_config(g.ep_lxc, 0xABCDE)
    rec, idx, total = dp.drop_notify(b, out, g.mode, g.ep_lxc)
    nt, orec, oidx = oracle_notify(g.tables, g.headers, g.mode, g.ep_lxc)
    assert total == len(orec) > 0
    np.testing.assert_array_equal(
        np.ascontiguousarray(rec.cpu().numpy()).view(np.uint8).reshape(-1),
        orec.view(np.uint8))
    dp.close()


def gpu_events(torch, t, h, mode, ep_lxc=0, clock=0, chunks=1):
    """-> (event words, records, header indices, total) of the engine,
    chunk by chunk (CT folded between chunks)."""
    dp = Datapath(0)
    load_tables(dp, t)
    dp.set_clock(clock)
    b = pack(h)
    n = len(h)
    step = max(1, (n + chunks - 1) // chunks)
    use_ct = getattr(t, "ct", None) is not None
    words, recs, idxs, tot = [], [], [], 0
    for a in range(0, max(n, 1), step):
        sub = b.slice(a, a + step)
        out = dp.classify(sub, mode, ep_lxc, want_notify=True, want_ct=use_ct)
        if use_ct:   # (the apply settles the trace words in packet order)
            dp.ct_apply(sub, out, mode, ep_lxc)
        rec, idx, total = dp.monitor_events(sub, out, mode, ep_lxc)
        torch.cuda.synchronize()
        words.append(out.notify.cpu().numpy().view(np.uint32))
        recs.append(np.ascontiguousarray(rec.cpu().numpy()).view(O.EVENT_DT).reshape(-1))
        idxs.append(idx.cpu().numpy().astype(np.uint64) + a)
        tot += total
    dp.close()
    return (np.concatenate(words)[:n], np.concatenate(recs), np.concatenate(idxs), tot)


def oracle_events(t, h, mode, ep_lxc=0, clock=0, chunks=1):
    o = O.Oracle(t)
    o.set_clock(clock)
    n = len(h)
    step = max(1, (n + chunks - 1) // chunks)
    use_ct = getattr(t, "ct", None) is not None
    words, recs, idxs = [], [], []
    for a in range(0, max(n, 1), step):
        part = h.slice(a, a + step)
        act, ver, ide, nt = o.classify(part, mode, ep_lxc, nthreads=16,
                                       want_notify=True, apply_ct=use_ct)
        rec, idx = o.events(part, mode, ep_lxc, ver, ide, nt)
        words.append(nt)
        recs.append(rec)
        idxs.append(idx + np.uint64(a))
    return np.concatenate(words)[:n], np.concatenate(recs), np.concatenate(idxs)


def check_events(torch, t, h, mode, ep_lxc=0, clock=0, chunks=1):
    ow, orec, oidx = oracle_events(t, h, mode, ep_lxc, clock, chunks)
    gw, grec, gidx, total = gpu_events(torch, t, h, mode, ep_lxc, clock, chunks)
    bad = np.nonzero(gw != ow)[0]
    assert len(bad) == 0, f"event words: {len(bad)} differ, first {bad[:5]} " \
                          f"{gw[bad[:5]]} vs {ow[bad[:5]]}"
    assert total == len(orec)
    np.testing.assert_array_equal(gidx, oidx)
    np.testing.assert_array_equal(grec.view(np.uint8), orec.view(np.uint8))
    return orec


@pytest.mark.parametrize("name", G.names())
def test_golden_monitor_events(torch, name):
    """Drop and trace records of every fixture, engine vs the oracle (which
    the CPU suite pins record by record to the reference's perf ring) on the
    same batch at the fixture's clock."""
    g = G.Golden(name)
    clock = int(np.median(g.clock[g.clock != 0xFFFFFFFF])) if g.clock is not None else 0
    rec = check_events(torch, g.tables, g.headers, g.mode, g.ep_lxc, clock)
    if g.ev is not None and (g.ev["type"] == 4).any():
        assert (rec["type"] == 4).any(), name


@pytest.mark.parametrize("mode", [0, 1, 3])
def test_c2_monitor_events(torch, mode):
    t = S.config_c2(2, n_endpoints=3)
    if mode == 1:
        rng = np.random.default_rng(9)
        h = S.gen_headers_v4(rng, 2_000_000, t.ipcache, S.local_v4_addrs(t),
                             local_frac=0.2, src_fixed=S.LXC_IPV4)
    else:
        h = S.headers_c2(t, 2_000_000, seed=9)
    rec = check_events(torch, t, h, mode, S.EP_LXC_ID if mode == 1 else 0)
    assert set(np.unique(rec["type"])) == {1, 4}


def test_c5_monitor_events(torch):
    """Conntrack hits: which packets of an active flow are traced (report
    interval, new TCP flags, closes), at a clock inside and past the
    flows' report interval, three batches folded into CT in between."""
    t, flows = S.config_c5(5, n_flows=200_000, n_prefixes=50_000, now=1000)
    h = S.headers_c5(t, flows, 900_000, seed=8)
    rng = np.random.default_rng(3)
    h.tcpflags = rng.choice(np.array([0x10, 0x18, 0x02, 0x12], np.uint8), size=len(h))
    for clock in (1003, 2000):
        rec = check_events(torch, t, h, 3, 0, clock, chunks=3)
        caps = np.unique(rec["len_cap"][rec["type"] == 4])
        assert 1 in caps and 128 in caps, caps


def test_c3_monitor_events(torch):
    t = S.config_c3(3, n_prefixes=100_000, n_v4_prefixes=10_000, n_endpoints=3,
                    n_prefilter=5000)
    h = S.headers_c3(t, 500_000, seed=12, ext=0.05, exthdr_drop=0.01, local_frac=0.9)
    for mode in (0, 3):
        check_events(torch, t, h, mode)
