// Instantiations of the 3x3 conv kernel (lrp_conv_kernel.h), split across files so the
// build compiles them in parallel.  VGGish-BN blocks 3-5 (100/128 -> 128 channels padded).
#include "lrp_conv_kernel.h"

namespace drsa_conv {
static const Entry kTableFwdE_e[] = {
    FWD_SET(128, 128, 8),
};
extern const Table kTableFwdE = {kTableFwdE_e, (int)(sizeof(kTableFwdE_e) / sizeof(kTableFwdE_e[0]))};
}  // namespace drsa_conv
