// scan_group_lds.hip -- k_scan instantiations of the LDS-private dense group table plan (MODE_GROUP_LDS).
#include "scan_kernel.h"

namespace ph {

void launch_scan_group_lds(const KParams& p, int ng, int grid, size_t lds, hipStream_t s) {
  launch_mode<MODE_GROUP_LDS>(p, ng, (p.num_vals <= 1 && !p.val_op[0]) ? 1 : 0, grid, lds, s);
}

}  // namespace ph
