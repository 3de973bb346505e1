"""Debug: engine vs oracle event words on one golden fixture (GPU)."""
import sys
import numpy as np
sys.path[:0] = ["tests", "oracle", "."]
import golden_io as G
import oracle as O
from cilium_amd.datapath import Datapath, pack
from cilium_amd.loader import load_tables
import torch

name = sys.argv[1] if len(sys.argv) > 1 else "ct_egress_v4"
g = G.Golden(name)
dp = Datapath(0)
load_tables(dp, g.tables)
b = pack(g.headers)
out = dp.classify(b, g.mode, g.ep_lxc, want_notify=True, want_ct=True)
torch.cuda.synchronize()
gw = out.notify.cpu().numpy().view(np.uint32)
gct = out.ct.cpu().numpy()
o = O.Oracle(g.tables)
oa, ov, oi, oct_, ow = o.classify(g.headers, g.mode, g.ep_lxc, want_ct=True, want_notify=True)
bad = np.flatnonzero(gw != ow)
print(name, "bad", len(bad), "of", len(gw))
h = g.headers
tf = h.tcpflags if h.tcpflags is not None else np.zeros(len(h), np.uint8)
for i in bad[:12]:
    print(i, "proto", h.proto[i], "flags", h.flags[i], "tcpfl", hex(tf[i]), "gw", hex(gw[i]),
          "ow", hex(ow[i]), "ct", hex(gct[i]), hex(oct_[i]), "mon", hex(o.mon[i]))
print("tcp_flags on device:", b.tcp_flags[:8].cpu().numpy(), tf[:8])
import ctypes
from cilium_amd import _lib as LL
for nm in ("ct_ingress_v4", "ct_ingress_v6", "ct_egress_v6"):
    g = G.Golden(nm)
    dp = Datapath(0)
    load_tables(dp, g.tables)
    b = pack(g.headers)
    out = dp.classify(b, g.mode, g.ep_lxc, want_notify=True, want_ct=True)
    torch.cuda.synchronize()
    gw = out.notify.cpu().numpy().view(np.uint32)
    o = O.Oracle(g.tables)
    oa, ov, oi, oct_, ow = o.classify(g.headers, g.mode, g.ep_lxc, want_ct=True, want_notify=True)
    bad = np.flatnonzero(gw != ow)
    print(nm, "bad", len(bad), [(hex(gw[i]), hex(ow[i])) for i in bad[:4]])
    dp.close()
