"""Diagnose the load-balancer CT apply mismatches (GPU box): the lb_egress_v4
golden through the device apply, engine and oracle CT rows saved for a diff
on the build host; the 200k-header egress service stream with the apply's
path reasons (CFC_DEBUG_APPLY)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
os.environ["CFC_DEBUG_APPLY"] = "1"
import torch  # noqa: E402
import golden_io as G  # noqa: E402
import oracle as O  # noqa: E402
import test_gpu_lb as T  # noqa: E402

out = {}
for name in ("lb_egress_v4", "lb_egress_v6"):
    g = G.Golden(name)
    r = T._run(torch, g.tables, g.headers, g.mode, g.ep_lxc)
    o = O.Oracle(g.tables)
    o.classify(g.headers, g.mode, g.ep_lxc, nthreads=8, want_ct=True, want_pkt=True,
               apply_ct=True)
    out[name + "_dev"] = r["ct_rows"]
    out[name + "_orc"] = o.ct_dump()
    out[name + "_ct"] = r["ct"]
    print(name, r["stats"], flush=True)
t, h = T._lb_stream(72, 200_000, 1)
r = T._run(torch, t, h, 1, T.S.EP_LXC_ID)
print("stream", r["stats"], flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "debug_lb.npz"), **out)
