// k_expand_generic2.hip — KExpand with the descriptor-driven emitter for any
// value type needing 2 hashed block(s) (tuples, IntModN, mixed widths).
#include "expand_device.h"

namespace dpf_amd {

int LaunchExpandGeneric2(int D, int grid, hipStream_t st, const ExpandArgs& a,
                         const VtDev& vt) {
  return LaunchExpandAnyD<EmitGeneric<2>>(D, grid, st, a, vt);
}

}  // namespace dpf_amd
