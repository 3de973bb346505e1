"""Populate a Datapath from synth.Tables through the pkg/maps mirrors —
the same calls the agent makes (ipcache BPFListener updates, lxcmap
WriteEndpoint, per-endpoint policymap sync, prefilter inserts)."""
from __future__ import annotations

import struct

from . import cidrmap, ipcache, lbmap, lxcmap, policymap
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
    if getattr(t, "ct", None) is not None:
        dp.ct_fds = load_ct(dp, t)
    if getattr(t, "node", None) is not None:
        dp.set_node_config(*t.node)
    if getattr(t, "lb4", None) is not None or getattr(t, "revnat4", None) is not None:
        lbmap.LBMap(dp).load_rows(getattr(t, "lb4", None), getattr(t, "revnat4", None))
    if getattr(t, "lb6", None) is not None or getattr(t, "revnat6", None) is not None:
        lbmap.LBMap6(dp).load_rows(getattr(t, "lb6", None), getattr(t, "revnat6", None))
    if commit:
        dp.commit()
    return pms


# pkg/maps/ctmap (ctmap.go:59-69): TCP and ANY maps per family, global or
# per endpoint; LRU_HASH, key struct ipv{4,6}_ct_tuple, value struct ct_entry
CT_TYPE, CT_VSZ = 9, 56


def ct_map_name(family, lxc, any_map):
    f = "4" if family == 1 else "6"
    owner = "global" if lxc < 0 else str(lxc)
    return f"cilium_ct{'_any' if any_map else ''}{f}_{owner}"


def open_ct_maps(dp: Datapath, lxc_ids, max_entries=1 << 20):
    """Every endpoint's local CT maps (the reference compiles CT_MAP_* per
    endpoint, lxc_config.h:40-45); lxc -1 = the global maps."""
    fds = {}
    for lxc in lxc_ids:
        for fam in (1, 2):
            for any_map in (0, 1):
                name = ct_map_name(fam, lxc, any_map)
                fd, _ = dp.open_or_create_map(name, CT_TYPE,
                                              14 if fam == 1 else 38, CT_VSZ,
                                              max_entries)
                fds[(fam, lxc, any_map)] = fd
    return fds


def load_ct(dp: Datapath, t):
    ct = t.ct
    # local CT maps (the reference's per-endpoint CT_MAP_*) for every
    # endpoint program when the table uses them, else the global maps only
    lxcs = set(int(x) for x in ct["lxc"])
    if any(x >= 0 for x in lxcs):
        lxcs |= set(int(x) for x in t.policy)
    lxcs = sorted(lxcs | {-1})
    # (t.ct_max_entries: the maps' capacity, when a test wants more room than
    # the entries it loads — the device table is sized by the entries)
    n = getattr(t, "ct_max_entries", None) or max(1 << 16, 2 * len(ct))
    fds = open_ct_maps(dp, lxcs, max_entries=n)
    import numpy as np
    for (fam, lxc, any_map), fd in fds.items():
        sel = ct[(ct["family"] == fam) & (ct["lxc"] == lxc) & (ct["any"] == any_map)]
        if len(sel):
            ksz = 14 if fam == 1 else 38
            dp.update_batch(fd, np.ascontiguousarray(sel["tuple"][:, :ksz]),
                            np.ascontiguousarray(sel["entry"]))
    return fds


def ct_rows(dp: Datapath, fds):
    """Live CT entries in the oracle's dump format (oracle/cfc_oracle.h
    CFO_CT_ROW: u16 owner (lxc + 1, 0 global), u8 map (0 TCP / 1 ANY),
    u8 family, tuple[40], ct_entry[56], pad[4]), sorted."""
    import numpy as np
    parts = []
    for (fam, lxc, any_map), fd in fds.items():
        k, v = dp.dump(fd)                 # cfc_map_dump
        r = np.zeros((len(k), 104), np.uint8)
        r[:, 0:2] = np.uint16(lxc + 1).tobytes()[0], np.uint16(lxc + 1).tobytes()[1]
        r[:, 2] = any_map
        r[:, 3] = fam
        r[:, 4:4 + k.shape[1]] = k
        r[:, 44:100] = v[:, :56]
        parts.append(r)
    rows = np.concatenate(parts) if parts else np.zeros((0, 104), np.uint8)
    # sort by the first 44 bytes in memcmp order, as the oracle's dump:
    # lexicographic over big-endian 8-byte words
    w = np.zeros((len(rows), 48), np.uint8)
    w[:, :44] = rows[:, :44]
    keys = w.view(">u8").astype(np.uint64)
    order = np.lexsort(keys.T[::-1])
    return rows[order]


def policy_rows(pm: policymap.PolicyMap):
    """Sorted (identity, dport, proto, egress, proxy, packets, bytes) rows,
    the layout of the golden fixtures' counter dumps."""
    rows = []
    for d in pm.DumpToSlice():
        k, e = d.Key, d.PolicyEntry
        rows.append((k.Identity, k.DestPort, k.Nexthdr, k.TrafficDirection,
                     e.ProxyPort, e.Packets, e.Bytes))
    return sorted(rows)
