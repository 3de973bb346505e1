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
};

// LDS-privatised policy counters are used when 2*n_ctr u32 fit next to the
// metrics block in the 160 KiB LDS (one 1024-thread block per CU).
constexpr uint32_t LDS_CTR_MAX = 18432;
constexpr int BLOCK = 1024;

// Bytes of workspace (u32 partial counters) a launch over n headers needs.
size_t classify_workspace_bytes(uint64_t n, uint32_t n_ctr, int num_cus);

// dst[i] += src[i] for n u64 (counter import)
int launch_add_u64(uint64_t *dst, const uint64_t *src, uint64_t n,
                   hipStream_t stream);

int launch_classify_v4(const DevTables &T, const cfc_hdr_v4 &in,
                       const cfc_out &out, int mode, const EgressArgs &E,
                       uint64_t *g_ctr, uint64_t *g_met, uint32_t *workspace,
                       int num_cus, hipStream_t stream);

}  // namespace cfc
