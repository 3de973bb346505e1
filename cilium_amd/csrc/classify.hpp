// Launch interface of the classify kernels (classify.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cfc.h"
#include "layout.h"

namespace cfc {

// The egress source endpoint: the constants bpf_lxc.c is compiled with
// (LXC_ID, SECLABEL, POLICY_MAP) for the endpoint whose traffic this is.
struct EgressArgs {
    uint32_t lxc_id;
    uint32_t seclabel;
    uint32_t pol_base;
    uint32_t pol_mask;
    uint32_t ct_owner;   // ct_owner_word of the sending endpoint's CT maps
};

// The counter kernel keeps one packed u64 per policy entry in LDS when
// n_ctr of them fit in the 160 KiB LDS (one 1024-thread block per CU);
// beyond, global atomics.
constexpr uint32_t LDS_CTR_MAX = 18432;
constexpr int BLOCK = 1024;
constexpr int LDS_BYTES_MAX = 160 * 1024;

// Optional per-call timing (CFC_OPT_TIMING): events recorded on the launch
// stream before the classify kernel, after it, and after the counter
// kernels.
struct LaunchTiming {
    hipEvent_t ev[3];
};

// Bytes of workspace a launch over n headers needs: the matched policy-entry
// index per header (two per header in EGRESS mode) + the counter kernel's
// partial slabs.
// With ct, followed by the per-header CT accounting keys
// (slot * 2 + dir, NONE: no hit) the CT counter kernel aggregates.
size_t classify_workspace_bytes(uint64_t n, uint32_t n_ctr, int mode,
                                bool ct = false);
uint32_t *ct_idx_ptr(uint32_t *ws, uint64_t n, uint32_t n_ctr, int mode);
// LDS image of the classify kernel for these tables (must be <= 160 KiB).
size_t classify_lds_bytes(const DevTables &T);

// dst[i] += src[i] for n u64 (counter import)
int launch_add_u64(uint64_t *dst, const uint64_t *src, uint64_t n,
                   hipStream_t stream);

int launch_classify_v4(const DevTables &T, const cfc_hdr_v4 &in,
                       const cfc_out &out, int mode, const EgressArgs &E,
                       uint64_t *g_ctr, uint64_t *g_met, uint32_t *workspace,
                       int num_cus, hipStream_t stream,
                       const LaunchTiming *timing = nullptr);

// The policy-entry counter kernels over the per-header entry indices the
// classify kernel left in the workspace (both families).
void launch_counters(const DevTables &T, const uint32_t *meta, uint64_t n,
                     int mode, uint32_t *workspace, uint64_t *g_ctr,
                     hipStream_t stream, bool ct = false);

int launch_classify_v6(const DevTables &T, const cfc_hdr_v6 &in,
                       const cfc_out &out, int mode, const EgressArgs &E,
                       uint64_t *g_ctr, uint64_t *g_met, uint32_t *workspace,
                       int num_cus, hipStream_t stream,
                       const LaunchTiming *timing = nullptr);

// Drop-notify records of one classified batch (notify.hip): the per-header
// cfc_out.notify words compacted in header order into cfc_drop_notify.
struct NotifyArgs {
    const uint32_t *notify;
    const int32_t *verdict;
    const uint32_t *identity;
    const uint32_t *meta;
    const uint32_t *ports;
    const uint32_t *saddr;   // v4: n words; v6: n x 4 words
    const uint32_t *daddr;
    uint64_t n;
    int family;              // 4 or 6
    int mode;
    uint32_t own_seclabel;   // SECLABEL of ep_lxc (egress batches)
    const uint2 *ep_info;    // [65536] {SECLABEL, ifindex} by LXC_ID
    cfc_drop_notify *rec;
    uint64_t *hdr_index;     // may be NULL
    uint64_t cap;
    uint64_t *count;
};
// workspace: one u64 per block of headers (counts, then offsets)
size_t drop_notify_workspace_bytes(uint64_t n);
int launch_drop_notify(const NotifyArgs &a, uint64_t *ws, hipStream_t stream);

}  // namespace cfc
