// k_expand_nodes.hip — KExpandCoop<0, EmitNodes>: one level of tree nodes
// (the precomputed subtree roots of a large expansion, kernels_capi.cc).
#include "expand_device.h"

namespace dpf_amd {

int LaunchExpandNodes(hipStream_t st, const ExpandArgs& a, const VtDev& vt) {
  return LaunchExpandCoop<0, EmitNodes>(st, a, vt);
}

}  // namespace dpf_amd
