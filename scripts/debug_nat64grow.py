"""Debug: the nat64_local_v6 stream as test_gpu_nat runs it (one batch),
the engine's CT rows against the sequential oracle's; the rows only one
side has, in hex, and the engine's stats.  CFC_CT_GROW_HOST=1 selects the
host rebuild for growth (A/B)."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), ROOT]
import torch  # noqa: E402
import golden_io as G  # noqa: E402
from cilium_amd import synth as S  # noqa: E402
from test_gpu_ctorder import run_both  # noqa: E402

g = G.Golden("nat64_local_v6")
rng = np.random.default_rng(7)
h = S.concat([g.headers] * 3)
h = S.take(h, rng.permutation(len(h)))
for chunks in (1, 2):
    gg, want = run_both(torch, g.tables, h, 1, S.EP_LXC_ID, clock=1003, chunks=chunks)
    a = {r[:44].tobytes(): r for r in gg["rows"]}
    b = {r[:44].tobytes(): r for r in want["rows"]}
    print("chunks", chunks, "rows", len(a), len(b), "stats", gg["stats"])
    for k in sorted(a.keys() - b.keys()):
        print("  extra  ", a[k].tobytes().hex())
    for k in sorted(b.keys() - a.keys()):
        print("  missing", b[k].tobytes().hex())
    for k in sorted(a.keys() & b.keys()):
        if not np.array_equal(a[k], b[k]):
            print("  differ ", a[k].tobytes().hex(), b[k].tobytes().hex())
