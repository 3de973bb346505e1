"""Conntrack garbage collection (cfc_ct_gc: ctmap.GC with doFiltering,
pkg/maps/ctmap/ctmap.go:303-350) against the oracle's restatement
(cfo_ct_gc).  IPv4 and IPv6 entries are collected on the device CT tables
(doGC4 / doGC6: tombstones, trimmed cluster tails, a delete log the host
mirror replays lazily); the ICMP entries of TCP maps, which no lookup
reaches and the device table does not hold, on the host.  After every GC the
CT maps — keys, values, accounting — equal the oracle's byte for byte, and
applies after a GC (reusing the freed slots) stay exact.
Run on an MI355X: pytest -m gpu."""
import numpy as np
import pytest

import golden_io as G
import oracle as O
from cilium_amd import ctmap
from cilium_amd import synth as S
from cilium_amd.datapath import Datapath, pack, pack_v4
from cilium_amd.loader import ct_rows, load_tables

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "needs a GPU"
    return torch


def step(torch, dp, o, h, now, mode=3):
    dp.set_clock(now)
    o.set_clock(now)
    b = pack_v4(h)
    out = dp.classify_v4(b, mode, want_ct=True)
    dp.ct_apply(b, out, mode)
    _, ov, _, oct_ = o.classify(h, mode, 0, nthreads=16, want_ct=True, apply_ct=True)
    torch.cuda.synchronize()
    assert np.array_equal(out.verdict.cpu().numpy(), ov)
    assert np.array_equal(out.ct.cpu().numpy(), oct_)


def same_ct(dp, o):
    dp.counters_sync()   # the host mirror takes the device's changes
    got, want = ct_rows(dp, dp.ct_fds), o.ct_dump()
    if got.shape != want.shape:
        gk = {r[:44].tobytes(): r for r in got}
        wk = {r[:44].tobytes(): r for r in want}
        extra = [gk[k].tobytes().hex() for k in gk.keys() - wk.keys()][:6]
        miss = [wk[k].tobytes().hex() for k in wk.keys() - gk.keys()][:6]
        import os
        os.makedirs("gpurun_out", exist_ok=True)
        with open("gpurun_out/ct_diff.txt", "w") as fo:
            fo.write("\n".join(["extra"] + extra + ["missing"] + miss) + "\n")
        assert False, (got.shape, want.shape, len(extra), len(miss))
    bad = np.nonzero((got != want).any(1))[0]
    assert len(bad) == 0, f"{len(bad)} CT rows differ, first {got[bad[0]].tobytes().hex()}"


def same_count(st, n):
    """gcStats.deleted against the oracle's: exact for the table and the
    host's entries; a pending ICMP entry of a TCP map written twice before
    the host took it (two creates relating to one address pair) counts once
    per write"""
    assert st["device_deleted"] + st["host_deleted"] <= n <= st["deleted"], (st, n)


def test_gc_expiry_and_ip_filters_vs_oracle(torch):
    t, flows = S.config_c5(5, n_flows=100_000, n_prefixes=20_000, n_policy=2000, now=1000)
    dp = Datapath(0)
    load_tables(dp, t)
    o = O.Oracle(t)
    h = S.headers_c5(t, flows, 400_000, seed=6)
    step(torch, dp, o, h.slice(0, 200_000), 1000)
    step(torch, dp, o, h.slice(200_000, 400_000), 1030)
    # RemoveExpired at 1065: the loaded flows no packet refreshed (lifetime
    # 1060) and the first batch's new UDP / SYN entries go, the second's stay
    f = ctmap.GCFilter(remove_expired=True)
    ctmap.GC(dp, -1, f, now=1065)
    n = o.ct_gc(time=1065)
    same_ct(dp, o)
    assert n > 0
    same_count(f.stats, n)
    # applies reuse the freed slots; then ValidIPs and MatchIPs
    h2 = S.headers_c5(t, flows, 200_000, seed=7)
    step(torch, dp, o, h2, 1070)
    remote = np.unique(np.asarray(flows.saddr, np.uint32))[:300]
    rb = [int(a).to_bytes(4, "little") for a in remote]
    st = dp.ct_gc(-1, 0, False, match_ips=rb[:150])
    n = o.ct_gc(remove_expired=False, match=[(4, b) for b in rb[:150]])
    same_ct(dp, o)
    assert n > 0
    same_count(st, n)
    valid = rb + [int(S.LXC_IPV4).to_bytes(4, "little")]
    st = dp.ct_gc(-1, 0, False, valid_ips=valid[:200])
    n = o.ct_gc(remove_expired=False, valid=[(4, b) for b in valid[:200]])
    same_ct(dp, o)
    same_count(st, n)
    step(torch, dp, o, h.slice(0, 100_000), 1080)
    same_ct(dp, o)
    dp.close()


def test_gc_steady_state_cycles(torch):
    """apply + GC cycles at the reference's cadence (a GC interval per
    batch, the new flows of every batch different), with a host sync
    (counters, CT maps read) after every GC: the device path holds (no host
    walk), the device table keeps its size (the sync takes the load from
    the table itself, not from a mirror that still counts the tombstones
    the GC's trim freed), and the maps stay the oracle's."""
    t, flows = S.config_c5(5, n_flows=60_000, n_prefixes=20_000, n_policy=2000, now=1000)
    dp = Datapath(0)
    load_tables(dp, t)
    o = O.Oracle(t)
    now, sizes, slots = 1000, [], []
    for k in range(8):
        h = S.headers_c5(t, flows, 150_000, seed=20 + k)
        step(torch, dp, o, h, now)
        now += ctmap.GC_INTERVAL_DEFAULT + 1
        dp.set_clock(now)
        f = ctmap.GCFilter(remove_expired=True)
        ctmap.GC(dp, -1, f)   # (Time: the datapath's clock)
        assert f.time == now
        same_count(f.stats, o.ct_gc(time=now))
        dp.counters_sync()
        sizes.append(len(o.ct_dump()))
        slots.append(dp.stats()["ct_slots"])
    assert dp.stats()["ct_apply_host"] == 0
    assert max(sizes[2:]) < 1.3 * min(sizes[2:]), sizes
    assert len(set(slots[1:])) == 1, slots
    same_ct(dp, o)
    dp.close()


@pytest.mark.parametrize("name", [n for n in G.names() if n.startswith("ct_")])
def test_gc_golden_tables(torch, name):
    """The reference's own CT state (both families on the device, their TCP
    maps' ICMP entries on the host), one map at a time and all
    at once, at a time inside the spread of lifetimes."""
    g = G.Golden(name)
    dp = Datapath(0)
    load_tables(dp, g.tables)
    dp.commit()
    o = O.Oracle(g.tables)
    life = g.tables.ct["entry"][:, 32:36].copy().view("<u4").ravel()
    mid = int(np.median(life))
    fds = sorted(dp.ct_fds.items())
    (fam, lxc, anyk), fd = fds[0]
    n = o.ct_gc(time=mid, family=fam, owner=0 if lxc < 0 else lxc + 1, kind=anyk)
    assert dp.ct_gc(fd, mid)["deleted"] == n
    same_ct(dp, o)
    st = dp.ct_gc(-1, mid + 7)
    assert st["deleted"] == o.ct_gc(time=mid + 7)   # nothing pending: exact
    same_ct(dp, o)
    dp.close()


def step6(torch, dp, o, h, now, mode=0):
    dp.set_clock(now)
    o.set_clock(now)
    b = pack(h)
    out = dp.classify(b, mode, 0, want_ct=True)
    dp.ct_apply(b, out, mode, 0)
    _, ov, _, oct_ = o.classify(h, mode, 0, nthreads=16, want_ct=True, apply_ct=True)
    torch.cuda.synchronize()
    assert np.array_equal(out.verdict.cpu().numpy(), ov)
    assert np.array_equal(out.ct.cpu().numpy(), oct_)


def test_gc6_on_device_vs_oracle(torch):
    """doGC6 (ctmap.go:239) on the device CT6 table (k_ct_gc<true>): expiry,
    then MatchIPs and ValidIPs over 16-byte addresses, each against the
    oracle's maps byte for byte, with device applies before and after (the
    freed slots reused) and the IPv6 TCP maps' ICMPv6 entries filtered on the
    host."""
    t, flows = S.config_c5_v6(6, n_flows=100_000, n_prefixes=20_000, now=1000)
    dp = Datapath(0)
    load_tables(dp, t)
    o = O.Oracle(t)
    h = S.headers_c5_v6(t, flows, 400_000, seed=6)
    step6(torch, dp, o, h.slice(0, 200_000), 1000)
    step6(torch, dp, o, h.slice(200_000, 400_000), 1030)
    f = ctmap.GCFilter(remove_expired=True)
    ctmap.GC(dp, -1, f, now=1065)
    n = o.ct_gc(time=1065)
    same_ct(dp, o)
    assert n > 0 and f.stats["device_deleted"] > 0, f.stats
    same_count(f.stats, n)
    h2 = S.headers_c5_v6(t, flows, 200_000, seed=7)
    step6(torch, dp, o, h2, 1070)
    remote = np.unique(np.asarray(flows.saddr, np.uint8).reshape(-1, 16), axis=0)[:300]
    rb = [bytes(r) for r in remote]
    st = dp.ct_gc(-1, 0, False, match_ips=rb[:150])
    n = o.ct_gc(remove_expired=False, match=[(6, b) for b in rb[:150]])
    same_ct(dp, o)
    assert n > 0 and st["device_deleted"] > 0, st
    same_count(st, n)
    valid = rb + [bytes(np.asarray(S.local_v6_addrs(t)[0], np.uint8))]
    st = dp.ct_gc(-1, 0, False, valid_ips=valid[:200])
    n = o.ct_gc(remove_expired=False, valid=[(6, b) for b in valid[:200]])
    same_ct(dp, o)
    same_count(st, n)
    step6(torch, dp, o, h.slice(0, 100_000), 1080)
    same_ct(dp, o)
    assert dp.stats()["ct_apply_host"] == 0
    dp.close()


def test_gc6_steady_state_cycles(torch):
    """IPv6 apply + GC cycles at the reference's cadence, every GC on the
    device: no host walk, the table keeps its size, the maps the oracle's."""
    t, flows = S.config_c5_v6(6, n_flows=60_000, n_prefixes=20_000, now=1000)
    dp = Datapath(0)
    load_tables(dp, t)
    o = O.Oracle(t)
    now, sizes, slots = 1000, [], []
    for k in range(6):
        h = S.headers_c5_v6(t, flows, 150_000, seed=30 + k)
        step6(torch, dp, o, h, now)
        now += ctmap.GC_INTERVAL_DEFAULT + 1
        dp.set_clock(now)
        f = ctmap.GCFilter(remove_expired=True)
        ctmap.GC(dp, -1, f)
        same_count(f.stats, o.ct_gc(time=now))
        assert f.stats["device_deleted"] > 0, f.stats
        dp.counters_sync()
        sizes.append(len(o.ct_dump()))
        slots.append(dp.stats()["ct_slots"])
    assert dp.stats()["ct_apply_host"] == 0
    assert len(set(slots[1:])) == 1, slots
    same_ct(dp, o)
    dp.close()
