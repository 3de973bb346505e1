"""Populate a Datapath from synth.Tables through the pkg/maps mirrors —
the same calls the agent makes (ipcache BPFListener updates, lxcmap
WriteEndpoint, per-endpoint policymap sync, prefilter inserts)."""
from __future__ import annotations

import struct

from . import cidrmap, ipcache, lxcmap, policymap
from .datapath import Datapath


def load_tables(dp: Datapath, t, commit=True):
    ipc = ipcache.Map(dp, max_entries=max(ipcache.MaxEntries, len(t.ipcache) + 16))
    for e in t.ipcache:
        k = ipcache.Key(32 + int(e["plen"]), int(e["family"]), bytes(e["addr"]))
        ipc.Update(k, ipcache.RemoteEndpointInfo(int(e["label"]),
                                                 struct.pack("<I", int(e["tunnel"]))))
    lxc = lxcmap.LXCMap(dp)
    for e in t.endpoints:
        k = lxcmap.EndpointKey(bytes(e["addr"]), int(e["family"]))
        lxc.WriteEndpoint([k], lxcmap.EndpointInfo(int(e["ifindex"]),
                                                   int(e["lxc_id"]),
                                                   int(e["flags"])))
    for lxc_id, lab in t.seclabel.items():
        dp.endpoint_config(int(lxc_id), int(lab))
    pms = {}
    for lxc_id, pol in t.policy.items():
        pm, _ = policymap.OpenMap(dp, policymap.path_for(int(lxc_id)))
        for r in pol:
            # raw network-order key/entry (syncPolicyMap writes PolicyKey
            # already converted ToNetwork(), endpoint.go:2572-2652)
            key = policymap.PolicyKey(int(r["identity"]), int(r["dport"]),
                                      int(r["proto"]), int(r["egress"]))
            dp.update_element(pm.Fd, key.pack(),
                              policymap.PolicyEntry(int(r["proxy_port"])).pack())
        pms[int(lxc_id)] = pm
    if len(t.prefilter):
        fix4 = cidrmap.OpenMapElems(dp, cidrmap.MapName + "v4_fix", 32, False,
                                    cidrmap.maxHKeys)
        dyn4 = cidrmap.OpenMapElems(dp, cidrmap.MapName + "v4_dyn", 32, True,
                                    cidrmap.maxLKeys)
        fam = set(int(f) for f in t.prefilter["family"])
        if 2 in fam:
            fix6 = cidrmap.OpenMapElems(dp, cidrmap.MapName + "v6_fix", 128, False,
                                        cidrmap.maxHKeys)
            dyn6 = cidrmap.OpenMapElems(dp, cidrmap.MapName + "v6_dyn", 128, True,
                                        cidrmap.maxLKeys)
        for p in t.prefilter:
            if int(p["family"]) == 1:
                key = struct.pack("<I", int(p["plen"])) + bytes(p["addr"][:4])
                dp.update_element((dyn4 if p["dyn"] else fix4).Fd, key, b"\x00")
            else:
                key = struct.pack("<I", int(p["plen"])) + bytes(p["addr"])
                dp.update_element((dyn6 if p["dyn"] else fix6).Fd, key, b"\x00")
    if commit:
        dp.commit()
    return pms


def policy_rows(pm: policymap.PolicyMap):
    """Sorted (identity, dport, proto, egress, proxy, packets, bytes) rows,
    the layout of the golden fixtures' counter dumps."""
    rows = []
    for d in pm.DumpToSlice():
        k, e = d.Key, d.PolicyEntry
        rows.append((k.Identity, k.DestPort, k.Nexthdr, k.TrafficDirection,
                     e.ProxyPort, e.Packets, e.Bytes))
    return sorted(rows)
