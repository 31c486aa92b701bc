// k_expand_c5.hip — KExpand for Tuple<uint32, IntModN<uint64, 2^64 - c>> (the c5
// benchmark type).
#include "expand_device.h"

namespace dpf_amd {

int LaunchExpandU32ModN64(int D, int grid, hipStream_t st, const ExpandArgs& a,
                          const VtDev& vt) {
  return LaunchExpandAnyD<EmitU32ModN64>(D, grid, st, a, vt);
}

}  // namespace dpf_amd
