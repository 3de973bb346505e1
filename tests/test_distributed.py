"""Multi-rank path on CPU (gloo, world_size 2): the header stream is sharded
contiguously, every rank classifies its shard against replicated tables, and
the u64 counter blocks — policy entries and the per-identity forward/drop
counters — are SUM-all-reduced (cilium_amd/distributed.py).
No GPU here, so the oracle stands in for each rank's engine; the engine's
side of the exchange (cfc_counters_export -> sum -> cfc_counters_import ->
cfc_counters_sync) is tests/test_gpu_distributed.py, and bench.py --gpus N
runs it over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from cilium_amd import synth as S
from cilium_amd.distributed import allreduce_block, gather_drop_notify, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_partitions_the_stream():
    for n in (0, 1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            got = [shard_range(n, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            for (a, b), (c, d) in zip(got, got[1:]):
                assert b == c and a <= b
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1


def identity_block(rows):
    """cfc_identity_counters rows -> the device block's identity part
    ([dir][65537][fwd, drop][packets, bytes], include/cfc.h)"""
    blk = np.zeros((2, 65537, 4), np.uint64)
    for r in rows:
        ident = 65536 if int(r[0]) == 0xFFFFFFFF else int(r[0])
        blk[int(r[1]) - 1, ident] = r[2:6]
    return blk.reshape(-1)


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = S.config_c2(2, n_prefixes=5000, n_policy=1024, n_endpoints=2)
        h = S.headers_c2(t, 40_000, seed=11)
        a, b = shard_range(len(h), rank, world)
        o = O.Oracle(t)
        part = h.slice(a, b)
        _, ver, ide, nt = o.classify(part, 0, 0, want_notify=True)
        rec, idx = o.drop_notify(part, 0, 0, ver, ide, nt)
        grec, gidx = gather_drop_notify(
            torch.from_numpy(rec.view(np.int32).reshape(-1, 8).copy()),
            torch.from_numpy(idx.astype(np.int64)), a)
        gathered = None if grec is None else (grec.numpy().copy(), gidx.numpy().copy())
        lxc = sorted(t.policy)[0]
        pc = o.policy_counters(lxc)             # rows: ..., packets, bytes
        blk = np.concatenate([pc[:, 5], pc[:, 6],
                              identity_block(o.identity_counters())]).astype(np.uint64)
        # u64 counters travel as int64 (two's complement == mod 2^64)
        tb = torch.from_numpy(blk.view(np.int64).copy())
        allreduce_block(tb)
        # wrap-around stays exact: add 2^64-1 on rank 0, +1 on rank 1
        w = torch.tensor([-1 if rank == 0 else 1], dtype=torch.int64)
        allreduce_block(w)
        q.put((rank, ver, ide, tb.numpy().view(np.uint64), int(w.item()),
               gathered))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_shards_and_counter_allreduce():
    import oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(world)), key=lambda r: r[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    # the concatenated shard verdicts are the whole stream's
    t = S.config_c2(2, n_prefixes=5000, n_policy=1024, n_endpoints=2)
    h = S.headers_c2(t, 40_000, seed=11)
    o = O.Oracle(t)
    _, ver, ide = o.classify(h, 0, 0)
    np.testing.assert_array_equal(np.concatenate([r[1] for r in res]), ver)
    np.testing.assert_array_equal(np.concatenate([r[2] for r in res]), ide)
    # the all-reduced counter block equals the single-rank totals
    pc = o.policy_counters(sorted(t.policy)[0])
    idrows = o.identity_counters()
    assert idrows[:, 2].sum() > 0 and idrows[:, 4].sum() > 0
    want = np.concatenate([pc[:, 5], pc[:, 6],
                           identity_block(idrows)]).astype(np.uint64)
    for r in res:
        np.testing.assert_array_equal(r[3], want)
        assert r[4] == 0
    # rank 0 holds every shard's drop records, in stream order, equal to the
    # single-rank records of the whole stream
    _, ver1, ide1, nt = o.classify(h, 0, 0, want_notify=True)
    rec, idx = o.drop_notify(h, 0, 0, ver1, ide1, nt)
    assert res[1][5] is None
    grec, gidx = res[0][5]
    np.testing.assert_array_equal(gidx, idx.astype(np.int64))
    np.testing.assert_array_equal(grec.view(np.uint8).reshape(-1),
                                  rec.view(np.uint8))


def _sorted_rows(rows):
    rows = np.asarray(rows, np.uint8)
    if not len(rows):
        return rows
    order = np.lexsort(rows.T[::-1])
    return rows[order]


def _ct_worker(rank, world, port, family, q):
    import torch
    import torch.distributed as dist
    import oracle as O
    from cilium_amd.distributed import shard_ct, shard_headers
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t, h, mode = _ct_case(family)
        t.ct = shard_ct(t.ct, rank, world)
        o = O.Oracle(t)
        vers = []
        for a, b in _ct_batches(len(h)):
            part, idx = shard_headers(h.slice(a, b), rank, world)
            _, ver, _, _ = o.classify(part, mode, 0, want_ct=True, apply_ct=True)
            vers.append((idx + a, ver))
        rows = o.ct_dump()
        # every rank's CT rows to rank 0 (uint8 rows travel as int64 words)
        n = torch.tensor([len(rows)], dtype=torch.int64)
        counts = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(counts, n)
        cmax = max(int(c) for c in counts)
        buf = np.zeros((max(cmax, 1), 104), np.uint8)
        buf[:len(rows)] = rows
        tb = torch.from_numpy(buf.view(np.int64).copy())
        got = [torch.zeros_like(tb) for _ in range(world)] if rank == 0 else None
        dist.gather(tb, got, dst=0)
        union = None
        if rank == 0:
            union = np.concatenate([g.numpy().view(np.uint8).reshape(-1, 104)[:int(c)]
                                    for g, c in zip(got, counts)])
        q.put((rank, vers, union))
    finally:
        dist.destroy_process_group()


def _ct_case(family):
    if family == 4:
        t, flows = S.config_c5(5, n_flows=20_000, n_prefixes=20_000, n_policy=2000)
        return t, S.headers_c5(t, flows, 60_000, seed=13), 0
    t, flows = S.config_c5_v6(6, n_flows=10_000, n_prefixes=10_000, n_policy=2000)
    return t, S.headers_c5_v6(t, flows, 40_000, seed=14), 3


def _ct_batches(n):
    return [(0, n // 2), (n // 2, n)]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("family", [4, 6])
def test_two_rank_conntrack_shards(family):
    """CT across GPUs: each rank takes the
    headers and CT entries of the address pairs it owns
    (distributed.shard_headers / shard_ct) and applies its own CT writes,
    batch by batch.  After two applied batches the ranks' CT maps together
    are, byte for byte, the single-rank result of the same two batches, and
    every header's verdict is the single-rank verdict."""
    import oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ct_worker, args=(r, world, port, family, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(world)), key=lambda r: r[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    t, h, mode = _ct_case(family)
    o = O.Oracle(t)
    want_ver = np.empty(len(h), np.int32)
    for a, b in _ct_batches(len(h)):
        _, ver, _, _ = o.classify(h.slice(a, b), mode, 0, want_ct=True, apply_ct=True)
        want_ver[a:b] = ver
    got_ver = np.full(len(h), 12345, np.int32)
    for r in res:
        for idx, ver in r[1]:
            got_ver[idx] = ver
    np.testing.assert_array_equal(got_ver, want_ver)
    want = _sorted_rows(o.ct_dump())
    got = _sorted_rows(res[0][2])
    assert len(want) > 1000
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("world", [2, 4])
def test_c5_rank_setup_partitions_ct_and_stream(world):
    """bench.py --workload c5 --gpus N: each rank loads the CT entries of the
    address pairs it owns and draws its stream from its own live flows and
    new flows it owns (distributed.c5_rank_setup, synth.headers_c5(owner)).
    The ranks' CT shards partition the node's entries; every header of a
    rank's stream is that rank's under shard_headers; the live flows'
    headers find their entries in the rank's own shard."""
    from cilium_amd.distributed import addr_keys, c5_rank_setup, pair_owner, shard_headers
    t, flows = S.config_c5(5, n_flows=20_000, n_prefixes=5_000, n_policy=500)
    full = np.sort(t.ct.view(np.dtype((np.void, t.ct.dtype.itemsize))).ravel())
    shards, nflows = [], 0
    for r in range(world):
        ct_r, fl_r = c5_rank_setup(t, flows, r, world)
        shards.append(ct_r)
        nflows += len(fl_r)
        own = pair_owner(addr_keys(fl_r.saddr, 4), addr_keys(fl_r.daddr, 4), world)
        assert (own == r).all()
        h, new = S.headers_c5(t, fl_r, 5000, seed=100 + r, return_new=True,
                              owner=(r, world))
        assert len(h) == 5000 and new.sum() == 5000 - int(5000 * 0.95)
        mine, idx = shard_headers(h, r, world)
        assert len(idx) == len(h)   # every header is the rank's own
    assert nflows == len(flows)
    got = np.sort(np.concatenate(shards).view(
        np.dtype((np.void, t.ct.dtype.itemsize))).ravel())
    np.testing.assert_array_equal(got, full)   # a partition: nothing lost or doubled
