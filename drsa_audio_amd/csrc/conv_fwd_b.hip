// Instantiations of the 3x3 conv kernel (lrp_conv_kernel.h), split across files so the
// build compiles them in parallel.
#include "lrp_conv_kernel.h"

namespace drsa_conv {
static const Entry kTableFwdB_e[] = {
    FWD_SET(32, 64, 8),
};
extern const Table kTableFwdB = {kTableFwdB_e, (int)(sizeof(kTableFwdB_e) / sizeof(kTableFwdB_e[0]))};
}  // namespace drsa_conv
