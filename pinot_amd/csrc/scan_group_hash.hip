// scan_group_hash.hip -- k_scan instantiations of the hash-table group-by plan (MODE_GROUP_HASH): key spaces too
// large for dense tables aggregate into a global open-addressing table keyed by the raw mixed-radix key.
#include "scan_kernel.h"

namespace ph {

void launch_scan_group_hash(const KParams& p, int ng, int grid, size_t lds, hipStream_t s) {
  launch_mode<MODE_GROUP_HASH>(p, ng, value_variant(p), grid, lds, s);
}

}  // namespace ph
