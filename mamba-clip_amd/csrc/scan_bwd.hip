// scan_bwd.hip -- selective-scan backward (placeholder until the kernel lands).
#include "mc_common.h"
#include "../../include/mc_scan.h"

extern "C" size_t mc_scan_bwd_workspace_bytes(int32_t, int32_t, int32_t, int32_t, int32_t) { return 0; }

extern "C" int mc_scan_bwd(const mc_scan_bwd_params* p, void* stream) {
  (void)p; (void)stream;
  MC_CHECK(false, MC_ERR_INVALID, "mc_scan_bwd: not implemented yet");
}
