// scan_count.hip -- k_scan instantiations of the aggregation-only plans (MODE_COUNT, MODE_AGG).
#include "scan_kernel.h"

namespace ph {

void launch_scan_agg(const KParams& p, int mode, int grid, size_t lds, hipStream_t s) {
  if (mode == MODE_COUNT) {
    launch_late<MODE_COUNT, 0, 0>(p, grid, lds, s);
  } else if (p.num_vals <= 1 && !p.val_op[0]) {
    launch_late<MODE_AGG, 0, 1>(p, grid, lds, s);  // ValCap 1
  } else {
    launch_late<MODE_AGG, 0, 0>(p, grid, lds, s);
  }
}

}  // namespace ph
