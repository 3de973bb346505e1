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


def gpu_notify(torch, t, h, mode, ep_lxc=0, cap=None, chunks=1):
    """-> per chunk: (notify words, records, header indices, total)."""
    dp = Datapath(0)
    load_tables(dp, t)
    b = pack(h)
    n = len(h)
    step = max(1, (n + chunks - 1) // chunks)
    res = []
    for a in range(0, max(n, 1), step):
        sl = lambda x: x[a:a + step] if x is not None else None   # noqa: E731
        sub = type(b)(sl(b.saddr), sl(b.daddr), sl(b.ports), sl(b.meta),
                      sl(b.mark))
        out = dp.classify(sub, mode, ep_lxc, want_notify=True)
        rec, idx, total = dp.drop_notify(sub, out, mode, ep_lxc, cap=cap)
        torch.cuda.synchronize()
        words = out.notify.cpu().numpy().view(np.uint32)
        recs = np.ascontiguousarray(rec.cpu().numpy()).view(O.DROP_NOTIFY_DT).reshape(-1)
        res.append((a, words, recs, idx.cpu().numpy().astype(np.uint64), total))
    dp.close()
    return res


def oracle_notify(t, h, mode, ep_lxc=0):
    o = O.Oracle(t)
    act, ver, ide, nt = o.classify(h, mode, ep_lxc, nthreads=8,
                                   want_notify=True)
    rec, idx = o.drop_notify(h, mode, ep_lxc, ver, ide, nt)
    return nt, rec, idx


def check(torch, t, h, mode, ep_lxc=0, chunks=1):
    nt, rec, idx = oracle_notify(t, h, mode, ep_lxc)
    got = gpu_notify(torch, t, h, mode, ep_lxc, chunks=chunks)
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
    rec = check(torch, g.tables, g.headers, g.mode, g.ep_lxc)
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
    small_b = type(b)(b.saddr[:5000], b.daddr[:5000], b.ports[:5000],
                      b.meta[:5000], b.mark[:5000] if b.mark is not None else None)
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
