"""Diagnose load-balancer parity on the GPU box: every lb_* golden and the
200k-header service streams through classify + the device apply; the
engine's outputs (action, verdict, identity, CT bytes, packets, event words)
and CT rows saved for a diff against the oracle on the build host
(gpurun_out/debug_lb.npz)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import golden_io as G  # noqa: E402
import test_gpu_lb as T  # noqa: E402

which = sys.argv[1:] or ["lb_egress_v4", "lb_reply_v4", "lb_egress_v6", "lb_reply_v6"]
out = {}
for name in which:
    if name.startswith("stream"):   # stream<fam>_<mode>
        fam, mode = int(name[6]), int(name[8])
        t, h = (T._lb_stream if fam == 4 else T._lb_stream6)(71 + mode + (10 if fam == 6 else 0),
                                                            200_000, mode)
        ep = T.S.EP_LXC_ID if mode == 1 else 0
    else:
        g = G.Golden(name)
        t, h, mode, ep = g.tables, g.headers, g.mode, g.ep_lxc
    r = T._run(torch, t, h, mode, ep)
    for k in ("act", "ver", "ide", "ct", "pkt", "ct_rows"):
        out[f"{name}_{k}"] = r[k]
    print(name, r["stats"], flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "debug_lb.npz"), **out)
