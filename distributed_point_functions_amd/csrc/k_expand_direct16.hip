// k_expand_direct16.hip — KExpand for a directly convertible 16-byte integer or
// XorWrapper value type (vth:216-228, 586-598).
#include "expand_device.h"

namespace dpf_amd {

int LaunchExpandDirect16(int D, int grid, hipStream_t st, const ExpandArgs& a, const VtDev& vt) {
  return LaunchExpandAnyD<EmitDirect<16>>(D, grid, st, a, vt);
}

}  // namespace dpf_amd
