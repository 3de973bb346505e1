"""pkg/maps/lbmap mirror (cilium_amd/lbmap.py) on a host-only context: the
reference's Service4Key / Service4Value / RevNat4 layouts and byte order, and
UpdateService's slot layout (lbmap.go:351-420)."""
import struct

import numpy as np

from cilium_amd import lbmap, synth as S
from cilium_amd.datapath import host_only


def test_update_service_slots_and_byte_order():
    dp = host_only()
    m = lbmap.LBMap(dp)
    fe = lbmap.Service4Key("172.20.0.9", 80)
    bes = [lbmap.Service4Value(target="10.1.0.1", port=8080, rev_nat=7),
           lbmap.Service4Value(target="10.1.0.2", port=8080, rev_nat=7, weight=3)]
    m.UpdateService(fe, bes, add_revnat=True, revnat_id=7)
    k, v = dp.dump(m.svc)
    rows = {bytes(a): bytes(b) for a, b in zip(k, v)}
    assert len(rows) == 3
    vip = S.ip4("172.20.0.9")
    master = struct.pack("<IHH", vip, int(S.htons(80)), 0)
    # master slot: count 2 (host order), one non-zero weight (network order)
    assert struct.unpack("<IHHHH", rows[master]) == (0, 0, 2, 0, int(S.htons(1)))
    b1 = struct.pack("<IHH", vip, int(S.htons(80)), 1)
    t, port, cnt, rev, w = struct.unpack("<IHHHH", rows[b1])
    assert (t, port, cnt, rev) == (S.ip4("10.1.0.1"), int(S.htons(8080)), 0, int(S.htons(7)))
    k, v = dp.dump(m.rnat)
    assert bytes(k[0]) == struct.pack("<H", int(S.htons(7)))
    assert bytes(v[0]) == struct.pack("<IH", vip, int(S.htons(80)))
    # shrinking the service removes the stale slot
    m.UpdateService(fe, bes[:1], add_revnat=False)
    k, v = dp.dump(m.svc)
    assert len(k) == 2
    m.DeleteService(fe)
    k, v = dp.dump(m.svc)
    assert len(k) == 0
    dp.close()


def test_synth_rows_load():
    """synth.lb4_services rows go in as raw map bytes (loader.load_tables)."""
    rng = np.random.default_rng(3)
    t = S.config_c2(3, n_prefixes=500, n_policy=50, n_endpoints=2)
    lb, rn, vips, ports, protos = S.lb4_services(rng, t, n_services=12)
    dp = host_only()
    m = lbmap.LBMap(dp)
    m.load_rows(lb, rn)
    k, v = dp.dump(m.svc)
    assert len(k) == len(lb)
    got = sorted(bytes(a) + bytes(b) for a, b in zip(k, v))
    want = sorted(r.tobytes() for r in lb)
    assert got == want
    dp.close()


def test_lb_map_geometry_checked():
    """objCheck: the load balancer's maps only with the reference's geometry"""
    import errno
    import pytest
    dp = host_only()
    with pytest.raises(OSError) as e:
        dp.open_or_create_map("cilium_lb4_services", 1, 8, 16, 65536)
    assert e.value.errno == errno.EINVAL
    with pytest.raises(OSError):
        dp.open_or_create_map("cilium_lb4_reverse_nat", 1, 4, 6, 65536)
    dp.close()
