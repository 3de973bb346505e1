"""Load the golden fixtures written by oracle/gen_golden.py."""
import glob
import os

import numpy as np

from cilium_amd import synth as S

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names():
    return sorted(os.path.basename(p)[:-4]
                  for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))


class Golden:
    def __init__(self, name):
        self.name = name
        d = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
        self.mode = int(d["mode"])
        self.ep_lxc = int(d["ep_lxc"])
        policy = {int(k.split("_")[1]): d[k] for k in d.files
                  if k.startswith("policy_")}
        seclabel = {int(a): int(b) for a, b in d["seclabel"]}
        self.tables = S.Tables(d["ipcache"], d["endpoints"], policy,
                               d["prefilter"], seclabel)
        self.headers = S.Headers(int(d["h_family"]), d["h_saddr"], d["h_daddr"],
                                 d["h_sport"], d["h_dport"], d["h_proto"],
                                 d["h_flags"], d["h_length"], d["h_mark"])
        self.action = d["x_action"]
        self.verdict = d["x_verdict"]
        self.identity = d["x_identity"]
        self.idmask = d["x_idmask"]
        self.metrics = d["x_metrics"]
        self.counters = {int(k.split("_")[2]): d[k] for k in d.files
                         if k.startswith("x_counters_")}


def mismatches(g: Golden, action, verdict, identity):
    """Indices where (action, verdict, pinned identity bits) differ."""
    bad = (action != g.action) | (verdict != g.verdict) | \
          ((identity & g.idmask) != (g.identity & g.idmask))
    return np.nonzero(bad)[0]
