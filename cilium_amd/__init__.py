"""cilium_amd — MI355X-native batch flow classification for Cilium's
datapath verdict path (prefilter -> ipcache LPM -> policymap).

The engine is libcfc.so (HIP, gfx950) behind the C ABI in include/cfc.h;
this package is the host-side mirror of the reference's map-population
APIs (pkg/bpf, pkg/maps/{policymap,ipcache,lxcmap,cidrmap,metricsmap},
pkg/policy/prefilter.go) plus the batch entry point.
"""
from ._lib import (CfcError, MODE_EGRESS, MODE_FULL, MODE_INGRESS,  # noqa: F401
                   MODE_XDP, HF_FRAG, HF_TCP_CLOSE, DROP_PREFILTER)
from .datapath import Datapath, HeaderBatchV4, Verdicts, host_only, pack_v4  # noqa: F401

__version__ = "0.1.0"
