"""The multi-GPU path of SURVEY.md §8e on hardware, as two ranks sharing the
one GPU of the test box: two processes (torch.distributed, gloo, started
before either touches the GPU), each with its own Datapath(0) context and the
same replicated tables, classify their contiguous shards of one stream and
call the real cilium_amd.distributed.allreduce_counters — export the device
counter block, SUM all-reduce it through torch.distributed, import the total,
fold it into the rank's maps.  Each rank's policy-entry counters,
cilium_metrics and per-identity forward/drop counters then equal the oracle's
over the whole stream; the shards' verdicts concatenate to the stream's.
On an 8-GPU node the same code runs over RCCL (bench.py --gpus N).
Run on an MI355X: pytest -m gpu."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from cilium_amd import synth as S

pytestmark = pytest.mark.gpu

N_HDR = 1_000_000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tables():
    return S.config_c2(7, n_prefixes=50_000, n_policy=8000, n_endpoints=2)


def _worker(rank, world, port, mode, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cilium_amd import metricsmap
        from cilium_amd.datapath import Datapath, pack_v4
        from cilium_amd.distributed import allreduce_counters, shard_range
        from cilium_amd.loader import load_tables, policy_rows
        torch.cuda.set_device(0)
        t = _tables()
        h = S.headers_c2(t, N_HDR, seed=17)
        ep = S.EP_LXC_ID if mode == 1 else 0
        a, b = shard_range(len(h), rank, world)
        dp = Datapath(0)
        pms = load_tables(dp, t)
        out = dp.classify_v4(pack_v4(h.slice(a, b)), mode, ep)
        torch.cuda.synchronize()
        ver = out.verdict.cpu().numpy()
        ide = out.identity.cpu().numpy().view(np.uint32)
        blk = allreduce_counters(dp)
        torch.cuda.synchronize()
        pol = {lxc: np.array(policy_rows(pm), np.uint64) for lxc, pm in pms.items()}
        met = np.array(metricsmap.dump_rows(dp), np.uint64).reshape(-1, 4)
        q.put((rank, ver, ide, pol, met, dp.identity_counters(),
               blk.cpu().numpy().view(np.uint64).copy()))
        dp.close()
    except BaseException as e:   # the parent reports it
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("mode", [0, 3])
def test_two_ranks_allreduce_counters_on_gpu(mode):
    import oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = [q.get(timeout=300) for _ in range(world)]
    finally:
        for p in ps:
            p.join(60)
            if p.exitcode is None:
                p.kill()
    for r in res:
        assert len(r) > 2, f"rank {r[0]} failed: {r[1]}"
    res.sort(key=lambda r: r[0])
    for p in ps:
        assert p.exitcode == 0
    t = _tables()
    h = S.headers_c2(t, N_HDR, seed=17)
    ep = S.EP_LXC_ID if mode == 1 else 0
    o = O.Oracle(t)
    _, ver, ide = o.classify(h, mode, ep, nthreads=16)
    np.testing.assert_array_equal(np.concatenate([r[1] for r in res]), ver)
    np.testing.assert_array_equal(np.concatenate([r[2] for r in res]), ide)
    idrows = o.identity_counters()
    assert idrows[:, 2].sum() > 0 and idrows[:, 4].sum() > 0
    for r in res:
        for lxc, rows in r[3].items():
            np.testing.assert_array_equal(rows, o.policy_counters(lxc))
        np.testing.assert_array_equal(r[4], o.metrics())
        np.testing.assert_array_equal(r[5], idrows)
    # both ranks hold the same all-reduced block
    np.testing.assert_array_equal(res[0][6], res[1][6])


def _ct_case(family):
    if family == 4:
        t, flows = S.config_c5(5, n_flows=200_000, n_prefixes=50_000, n_policy=4000)
        return t, S.headers_c5(t, flows, 800_000, seed=23), 0
    t, flows = S.config_c5_v6(6, n_flows=100_000, n_prefixes=50_000, n_policy=4000)
    return t, S.headers_c5_v6(t, flows, 400_000, seed=24), 3


def _ct_worker(rank, world, port, family, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cilium_amd.datapath import Datapath, pack
        from cilium_amd.distributed import shard_ct, shard_headers
        from cilium_amd.loader import ct_rows, load_tables
        torch.cuda.set_device(0)
        t, h, mode = _ct_case(family)
        t.ct = shard_ct(t.ct, rank, world)
        dp = Datapath(0)
        load_tables(dp, t)
        vers = []
        n = len(h)
        for a, b in ((0, n // 2), (n // 2, n)):
            part, idx = shard_headers(h.slice(a, b), rank, world)
            bt = pack(part)
            out = dp.classify(bt, mode, 0, want_ct=True)
            dp.ct_apply(bt, out, mode, 0)
            torch.cuda.synchronize()
            vers.append((idx + a, out.verdict.cpu().numpy()))
        dp.counters_sync()   # the device's CONNTRACK_ACCOUNTING into the maps
        rows = np.asarray(ct_rows(dp, dp.ct_fds), np.uint8).reshape(-1, 104)
        st = dp.stats()
        dp.close()
        q.put((rank, vers, rows, st["ct_apply_device"], st["ct_apply_host"]))
    except BaseException as e:
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("family", [4, 6])
def test_two_ranks_conntrack_shards_on_gpu(family):
    """CT across GPUs on hardware: two ranks on the one GPU,
    each owning the address pairs distributed.shard_headers / shard_ct give
    it, classify and apply their CT writes on the device for two batches.
    Their CT maps together equal the single-rank oracle's after the same two
    batches byte for byte, and every verdict is the single-rank one."""
    import oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ct_worker, args=(r, world, port, family, q))
          for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = [q.get(timeout=300) for _ in range(world)]
    finally:
        for p in ps:
            p.join(60)
            if p.exitcode is None:
                p.kill()
    for r in res:
        assert len(r) > 2, f"rank {r[0]} failed: {r[1]}"
        assert (r[3], r[4]) == (2, 0)   # both batches on the device path
    t, h, mode = _ct_case(family)
    o = O.Oracle(t)
    n = len(h)
    want = np.empty(n, np.int32)
    for a, b in ((0, n // 2), (n // 2, n)):
        _, ver, _, _ = o.classify(h.slice(a, b), mode, 0, nthreads=16, want_ct=True,
                                  apply_ct=True)
        want[a:b] = ver
    got = np.full(n, 12345, np.int32)
    for r in res:
        for idx, ver in r[1]:
            got[idx] = ver
    np.testing.assert_array_equal(got, want)

    def srt(rows):
        return rows[np.lexsort(rows.T[::-1])]
    union = np.concatenate([r[2] for r in res])
    np.testing.assert_array_equal(srt(union), srt(o.ct_dump()))
