// Instantiations of the 3x3 conv kernel (lrp_conv_kernel.h), split across files so the
// build compiles them in parallel.
#include "lrp_conv_kernel.h"

#ifndef DRSA_CONV_CIC_FWD32
#define DRSA_CONV_CIC_FWD32 8
#endif

namespace drsa_conv {
static const Entry kTableFwdA_e[] = {
    FWD_SET(1, 32, 1),
    FWD_SET(32, 32, DRSA_CONV_CIC_FWD32),
};
extern const Table kTableFwdA = {kTableFwdA_e, (int)(sizeof(kTableFwdA_e) / sizeof(kTableFwdA_e[0]))};
}  // namespace drsa_conv
