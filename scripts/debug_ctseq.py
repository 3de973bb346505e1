"""Debug helper: one golden CT stream through the GPU path and the oracle,
the headers whose CT byte differs and the other headers of their flows.
usage: python3 scripts/debug_ctseq.py <golden name> [layout 1|2]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import golden_io as G          # noqa: E402
import oracle as O             # noqa: E402
from cilium_amd import _lib as L   # noqa: E402
from test_gpu_parity import run_gpu   # noqa: E402


def main(name, layout=1):
    import torch
    g = G.Golden(name)
    run_gpu(torch, g.tables, g.headers, g.mode, g.ep_lxc, lpm4=layout)
    ctb, _ = run_gpu.ct
    o = O.Oracle(g.tables)
    oa, ov, oi, oct_ = o.classify(g.headers, g.mode, g.ep_lxc, nthreads=8, want_ct=True,
                                  apply_ct=True)
    h = g.headers
    from cilium_amd.datapath import Datapath, pack
    from cilium_amd.loader import load_tables
    dp = Datapath(0)
    dp.set_option(L.OPT_LPM4, layout)
    load_tables(dp, g.tables)
    lo = dp.classify(pack(h), g.mode, g.ep_lxc, want_ct=True)
    l0 = lo.ct.cpu().numpy()
    dp.close()
    bad = np.flatnonzero(ctb != oct_)
    print("differ", len(bad), "of", len(h))
    key = lambda i: (int(np.asarray(h.saddr[i]).sum()), int(np.asarray(h.daddr[i]).sum()),
                     int(h.proto[i]))
    seen = set()
    print("bad", bad.tolist())
    for i in bad[:4]:
        k = key(i)
        if k in seen:
            continue
        seen.add(k)
        print(f"-- flow of {i}: {k}")
        for j in range(len(h)):
            if key(j) == k or (key(j)[0], key(j)[1]) == (k[1], k[0]):
                print(f"  {j:6d} sp {int(h.sport[j]):5d} dp {int(h.dport[j]):5d} fl {int(h.flags[j]):3d} "
                      f"tf {int(h.tcpflags[j]):3d} ver {int(ov[j]):4d} gpu {int(ctb[j]):3d} "
                      f"ora {int(oct_[j]):3d} launch {int(l0[j]):3d}{'  <--' if ctb[j] != oct_[j] else ''}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
