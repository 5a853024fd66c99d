// Instantiations of the 3x3 conv kernel (lrp_conv_kernel.h), split across files so the
// build compiles them in parallel.  VGGish-BN first layer (1 -> 64, create_model.py:100-137).
#include "lrp_conv_kernel.h"

namespace drsa_conv {
static const Entry kTableFwdD_e[] = {
    FWD_SET(1, 64, 1),
};
extern const Table kTableFwdD = {kTableFwdD_e, (int)(sizeof(kTableFwdD_e) / sizeof(kTableFwdD_e[0]))};
}  // namespace drsa_conv
