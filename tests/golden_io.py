"""Load the golden fixtures written by oracle/gen_golden.py."""
import glob
import os

import numpy as np

import oracle as O
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
                               d["prefilter"], seclabel,
                               d["ct"] if "ct" in d.files else None)
        if "lb4" in d.files:   # service load balancing (LB4_DT, REVNAT4_DT)
            self.tables.lb4 = d["lb4"]
            self.tables.revnat4 = d["revnat4"]
        # CT maps after the stream, oracle row format (None: no CT state)
        self.ct_after = d["x_ct"] if "x_ct" in d.files else None
        self.headers = S.Headers(int(d["h_family"]), d["h_saddr"], d["h_daddr"],
                                 d["h_sport"], d["h_dport"], d["h_proto"],
                                 d["h_flags"], d["h_length"], d["h_mark"],
                                 d["h_tcpflags"] if "h_tcpflags" in d.files else None)
        # skb->hash of each header as the reference's records reported it
        # (lb4_select_slave's input), and the packet the program left:
        # (saddr, daddr, first L4 word); None in fixtures without a service
        self.hash_ok = d["x_hash_ok"] if "x_hash_ok" in d.files else None
        if self.hash_ok is not None:
            self.headers.hash = d["x_hash"]
        self.pkt = d["x_pkt"] if "x_pkt" in d.files else None
        # the cilium_events perf-ring samples (trace_notify / drop_notify,
        # 32 bytes each, EVENT_DT) and the header of each; None in older
        # fixtures
        self.ev = (d["x_ev"].reshape(-1).view(O.EVENT_DT)
                   if "x_ev" in d.files else None)
        self.ev_hdr = d["x_ev_hdr"] if "x_ev_hdr" in d.files else None
        # bpf_ktime_get_sec() while each header ran (0xFFFFFFFF: a second
        # boundary fell inside its run); None in older fixtures
        self.clock = d["x_clock"] if "x_clock" in d.files else None
        self.action = d["x_action"]
        self.verdict = d["x_verdict"]
        self.identity = d["x_identity"]
        self.idmask = d["x_idmask"]
        self.metrics = d["x_metrics"]
        # skb->cb[0..4] after the reference ran (None in older fixtures)
        self.cb = d["x_cb"] if "x_cb" in d.files else None
        self.counters = {int(k.split("_")[2]): d[k] for k in d.files
                         if k.startswith("x_counters_")}


def mismatches(g: Golden, action, verdict, identity):
    """Indices where (action, verdict, pinned identity bits) differ."""
    bad = (action != g.action) | (verdict != g.verdict) | \
          ((identity & g.idmask) != (g.identity & g.idmask))
    return np.nonzero(bad)[0]


# ct_entry bytes the comparison ignores: lifetime (offset 32, clock),
# seen_non_syn (bit 4 of offset 36) and the seen-TCP-flag bytes (42, 43:
# TCP flag bits the header batch does not carry), last_{tx,rx}_report
# (48-55, clock).  Row offsets: entry starts at 44.
def ct_masked(rows):
    r = np.array(rows, np.uint8).reshape(-1, S.CT_ROW).copy()
    e = 44
    r[:, e + 32:e + 36] = 0
    r[:, e + 36] &= 0xEF
    r[:, e + 42:e + 44] = 0
    r[:, e + 48:e + 56] = 0
    return r


def expected_drop_notify(g: Golden):
    """(header indices, fields) of the drop notifications the reference's
    send_drop_notify armed (drop.h:98-102): cb[1] = src << 16 | dst & 0xFFFF,
    cb[2] = reason, cb[3] = dst_id, cb[4] = ifindex.  XDP drops notify
    nothing (bpf_xdp.c has no send_drop_notify)."""
    tc = g.mode != 2
    idx = np.flatnonzero((g.action == 2) & (g.verdict < 0) & (g.verdict != -1)
                         if tc else np.zeros(len(g.action), bool))
    cb = g.cb[idx].astype(np.int64)
    f = dict(subtype=(-cb[:, 2]) & 0xFF,
             src_label=(cb[:, 1] >> 16) & 0xFFFF,
             dst_label=cb[:, 1] & 0xFFFF,
             dst_id=cb[:, 3] & 0xFFFFFFFF,
             ifindex=cb[:, 4] & 0xFFFFFFFF)
    return idx.astype(np.uint64), f
