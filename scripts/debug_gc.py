"""Diagnose a CT GC mismatch (GPU box): the scenario of
tests/test_gpu_ctgc.py::test_gc_expiry_and_ip_filters_vs_oracle with the
oracle's rows before the GC for every key the engine keeps and the oracle
does not."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import oracle as O  # noqa: E402
from cilium_amd import synth as S  # noqa: E402
from cilium_amd.datapath import Datapath, pack_v4  # noqa: E402
from cilium_amd.loader import ct_rows, load_tables  # noqa: E402

sync_first = len(sys.argv) > 1 and sys.argv[1] == "sync"
t, flows = S.config_c5(5, n_flows=100_000, n_prefixes=20_000, n_policy=2000, now=1000)
dp = Datapath(0)
load_tables(dp, t)
o = O.Oracle(t)
h = S.headers_c5(t, flows, 400_000, seed=6)
for a, now in ((0, 1000), (200_000, 1030)):
    dp.set_clock(now)
    o.set_clock(now)
    part = h.slice(a, a + 200_000)
    b = pack_v4(part)
    out = dp.classify_v4(b, 3, want_ct=True)
    dp.ct_apply(b, out, 3)
    o.classify(part, 3, 0, nthreads=16, want_ct=True, apply_ct=True)
print("stats", dp.stats())
pre = {r[:44].tobytes(): r for r in o.ct_dump()}
if sync_first:
    dp.counters_sync()
    g0 = {r[:44].tobytes(): r for r in ct_rows(dp, dp.ct_fds)}
    d = [k for k in g0 if k not in pre or not np.array_equal(g0[k], pre[k])]
    print("before GC: engine rows", len(g0), "oracle", len(pre), "differing", len(d))
st = dp.ct_gc(-1, 1065)
print("gc", st, "oracle deleted", o.ct_gc(time=1065))
dp.counters_sync()
got = {r[:44].tobytes(): r for r in ct_rows(dp, dp.ct_fds)}
want = {r[:44].tobytes(): r for r in o.ct_dump()}
extra = [k for k in got if k not in want]
miss = [k for k in want if k not in got]
print("extra", len(extra), "missing", len(miss))
for k in extra[:6]:
    e = got[k][44:100]
    p = pre.get(k)
    print("key", k.hex(), "engine life", int.from_bytes(e[32:36], "little"),
          "oracle before GC:", None if p is None else
          (int.from_bytes(p[44 + 32:44 + 36], "little"), p[44:100].tobytes().hex()))
