// scan_group_global.hip -- k_scan instantiations of the HBM dense group table plan (MODE_GROUP_GLOBAL).
#include "scan_kernel.h"

namespace ph {

void launch_scan_group_global(const KParams& p, int ng, int grid, size_t lds, hipStream_t s) {
  launch_mode<MODE_GROUP_GLOBAL>(p, ng, value_variant(p), grid, lds, s);
}

}  // namespace ph
