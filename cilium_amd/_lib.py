"""ctypes binding of libcfc.so (include/cfc.h).

The shared library is the product: there is no Python or CPU fallback for the
datapath.  If it is missing this module raises at import of the binding.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# CFC_LIB selects an alternative in-tree build (kernel A/B experiments)
LIB_PATH = os.path.join(HERE, os.environ.get("CFC_LIB", "libcfc.so"))

CFC_DEVICE_NONE = -1
MODE_INGRESS, MODE_EGRESS, MODE_XDP, MODE_FULL = 0, 1, 2, 3
HF_FRAG, HF_TCP_CLOSE, HF_EXTHDR = 0x100, 0x200, 0x400
DROP_PREFILTER, VERDICT_PUNT = -1, -2
OPT_LPM4, OPT_TIMING, OPT_CT_APPLY, OPT_CT_EVICT = 1, 2, 3, 4
CT_APPLY_DEVICE, CT_APPLY_HOST = 0, 1
LPM4_AUTO, LPM4_DIR24_8, LPM4_TRIE = 0, 1, 2

# every symbol include/cfc.h declares
EXPORTS = (
    "cfc_open", "cfc_close", "cfc_abi_version", "cfc_map_open",
    "cfc_drop_notify_v4", "cfc_drop_notify_v6",
    "cfc_map_close", "cfc_map_update", "cfc_map_lookup", "cfc_map_delete",
    "cfc_map_get_next_key", "cfc_num_possible_cpus", "cfc_endpoint_config",
    "cfc_commit", "cfc_classify_v4", "cfc_counters_device",
    "cfc_counters_sync", "cfc_counters_clear", "cfc_counters_export",
    "cfc_counters_import", "cfc_get_stats", "cfc_strerror",
    "cfc_set_option", "cfc_timing_collect", "cfc_classify_v6",
    "cfc_ct_apply_v4", "cfc_ct_apply_v6", "cfc_map_update_batch",
    "cfc_set_node_config", "cfc_get_node_config", "cfc_identity_counters",
    "cfc_set_clock", "cfc_monitor_events_v4", "cfc_monitor_events_v6",
    "cfc_map_dump", "cfc_ct_gc",
)
# CT byte (cfc_out.ct): per stage (bits 0-3, then 4-7 for the destination's
# ingress lookup after egress local delivery)
CT_NEW, CT_ESTABLISHED, CT_REPLY, CT_RELATED = 0, 1, 2, 3
CT_RES_MASK, CT_DONE, CT_CREATE = 0x3, 0x4, 0x8


class CfcError(OSError):
    pass


# cfc_ct_gc (include/cfc.h): struct GCFilter flags and types
GC_REMOVE_EXPIRED, GC_VALID_IPS, GC_MATCH_IPS = 1, 2, 4


class Ip(ctypes.Structure):
    _fields_ = [("family", ctypes.c_uint8), ("pad", ctypes.c_uint8 * 3),
                ("addr", ctypes.c_uint8 * 16)]


class GcFilter(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_uint32), ("time", ctypes.c_uint32),
                ("valid_ips", ctypes.c_void_p), ("n_valid", ctypes.c_uint32),
                ("pad0", ctypes.c_uint32),
                ("match_ips", ctypes.c_void_p), ("n_match", ctypes.c_uint32),
                ("pad1", ctypes.c_uint32)]


class GcStats(ctypes.Structure):
    _fields_ = [("deleted", ctypes.c_uint64), ("alive", ctypes.c_uint64),
                ("device_deleted", ctypes.c_uint64), ("log_deleted", ctypes.c_uint64),
                ("host_deleted", ctypes.c_uint64), ("slots_freed", ctypes.c_uint64)]


_HDR = [("saddr", ctypes.c_void_p), ("daddr", ctypes.c_void_p),
        ("ports", ctypes.c_void_p), ("meta", ctypes.c_void_p),
        ("mark", ctypes.c_void_p), ("tcp_flags", ctypes.c_void_p),
        ("n", ctypes.c_uint64)]


class HdrV4(ctypes.Structure):
    _fields_ = _HDR + [("hash", ctypes.c_void_p)]


class HdrV6(ctypes.Structure):
    _fields_ = _HDR + [("hash", ctypes.c_void_p)]


class Out(ctypes.Structure):
    _fields_ = [("verdict", ctypes.c_void_p), ("identity", ctypes.c_void_p),
                ("action", ctypes.c_void_p), ("ct", ctypes.c_void_p),
                ("notify", ctypes.c_void_p), ("pkt_saddr", ctypes.c_void_p),
                ("pkt_daddr", ctypes.c_void_p), ("pkt_ports", ctypes.c_void_p)]


class Stats(ctypes.Structure):
    _fields_ = [("epoch", ctypes.c_uint64), ("device_bytes", ctypes.c_uint64),
                ("ipcache_v4_prefixes", ctypes.c_uint32),
                ("lpm4_tbl8_groups", ctypes.c_uint32),
                ("policy_entries", ctypes.c_uint32),
                ("endpoints", ctypes.c_uint32),
                ("prefilter_v4_fix", ctypes.c_uint32),
                ("prefilter_v4_dyn", ctypes.c_uint32),
                ("lpm4_layout", ctypes.c_uint32),
                ("lpm4_kib", ctypes.c_uint32),
                ("ipcache_v6_prefixes", ctypes.c_uint32),
                ("lpm6_lengths", ctypes.c_uint32),
                ("lpm6_groups", ctypes.c_uint32),
                ("lpm6_kib", ctypes.c_uint32),
                ("endpoints_v6", ctypes.c_uint32),
                ("prefilter_v6_fix", ctypes.c_uint32),
                ("prefilter_v6_dyn", ctypes.c_uint32),
                ("ct4_entries", ctypes.c_uint32),
                ("ct6_entries", ctypes.c_uint32),
                ("ct_apply_device", ctypes.c_uint32),
                ("ct_apply_host", ctypes.c_uint32),
                ("ct_slots", ctypes.c_uint32),
                ("ct_grown", ctypes.c_uint32),
                ("ct_order_changed", ctypes.c_uint64),
                ("nat_hops", ctypes.c_uint64),
                ("ct_evicted", ctypes.c_uint64),
                ("svc_ordered", ctypes.c_uint64),
                ("ct_apply_sparse", ctypes.c_uint64),
                ("ct_self_segments", ctypes.c_uint64)]


class NodeConfig(ctypes.Structure):
    _fields_ = [("ipv4_cluster_range", ctypes.c_uint32),
                ("ipv4_cluster_mask", ctypes.c_uint32),
                ("router_ip6", ctypes.c_uint8 * 16),
                ("host_ifindex", ctypes.c_uint32)]


class IdentityCount(ctypes.Structure):
    _fields_ = [("identity", ctypes.c_uint32), ("dir", ctypes.c_uint8),
                ("pad", ctypes.c_uint8 * 3),
                ("fwd_packets", ctypes.c_uint64), ("fwd_bytes", ctypes.c_uint64),
                ("drop_packets", ctypes.c_uint64), ("drop_bytes", ctypes.c_uint64)]


IDENTITY_OUT_OF_RANGE = 0xFFFFFFFF


class Timing(ctypes.Structure):
    _fields_ = [("launches", ctypes.c_uint64), ("classify_ms", ctypes.c_double),
                ("count_ms", ctypes.c_double), ("launches_v6", ctypes.c_uint64),
                ("classify_v6_ms", ctypes.c_double), ("count_v6_ms", ctypes.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CfcError(2, f"{LIB_PATH} is not built (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    pint = ctypes.POINTER(ctypes.c_int)
    L.cfc_open.argtypes = [i32, ctypes.POINTER(vp)]
    L.cfc_close.argtypes = [vp]
    L.cfc_close.restype = None
    L.cfc_map_open.argtypes = [vp, ctypes.c_char_p, u32, u32, u32, u32, u32,
                               pint, pint]
    L.cfc_map_close.argtypes = [vp, i32]
    L.cfc_map_update.argtypes = [vp, i32, vp, vp, u64]
    L.cfc_map_lookup.argtypes = [vp, i32, vp, vp]
    L.cfc_map_update_batch.argtypes = [vp, i32, vp, vp, u64, u64]
    L.cfc_map_delete.argtypes = [vp, i32, vp]
    L.cfc_map_get_next_key.argtypes = [vp, i32, vp, vp]
    L.cfc_map_dump.argtypes = [vp, i32, vp, vp, u64, ctypes.POINTER(u64)]
    L.cfc_endpoint_config.argtypes = [vp, ctypes.c_uint16, u32]
    L.cfc_set_node_config.argtypes = [vp, ctypes.POINTER(NodeConfig)]
    L.cfc_get_node_config.argtypes = [vp, ctypes.POINTER(NodeConfig)]
    L.cfc_commit.argtypes = [vp, vp]
    L.cfc_classify_v4.argtypes = [vp, ctypes.POINTER(HdrV4), ctypes.POINTER(Out),
                                  i32, ctypes.c_uint16, vp]
    L.cfc_classify_v6.argtypes = [vp, ctypes.POINTER(HdrV6), ctypes.POINTER(Out),
                                  i32, ctypes.c_uint16, vp]
    L.cfc_ct_apply_v4.argtypes = [vp, ctypes.POINTER(HdrV4), ctypes.POINTER(Out),
                                  i32, ctypes.c_uint16, vp]
    L.cfc_ct_apply_v6.argtypes = [vp, ctypes.POINTER(HdrV6), ctypes.POINTER(Out),
                                  i32, ctypes.c_uint16, vp]
    L.cfc_set_clock.argtypes = [vp, u32]
    L.cfc_ct_gc.argtypes = [vp, i32, ctypes.POINTER(GcFilter), ctypes.POINTER(GcStats), vp]
    for f in (L.cfc_drop_notify_v4, L.cfc_drop_notify_v6,
              L.cfc_monitor_events_v4, L.cfc_monitor_events_v6):
        f.argtypes = [vp, vp, ctypes.POINTER(Out), i32, ctypes.c_uint16, vp, vp,
                      u64, vp, vp]
    L.cfc_counters_device.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(u64)]
    L.cfc_counters_sync.argtypes = [vp, vp]
    L.cfc_counters_clear.argtypes = [vp, vp]
    L.cfc_counters_export.argtypes = [vp, vp, u64, vp]
    L.cfc_counters_import.argtypes = [vp, vp, u64, vp]
    L.cfc_get_stats.argtypes = [vp, ctypes.POINTER(Stats)]
    L.cfc_identity_counters.argtypes = [vp, vp, u64, ctypes.POINTER(u64)]
    L.cfc_set_option.argtypes = [vp, i32, ctypes.c_int64]
    L.cfc_timing_collect.argtypes = [vp, ctypes.POINTER(Timing)]
    L.cfc_strerror.argtypes = [i32]
    L.cfc_strerror.restype = ctypes.c_char_p
    _lib = L
    return L


def check(rc, what):
    if rc < 0:
        raise CfcError(-rc, f"{what}: {os.strerror(-rc)}")
    return rc
