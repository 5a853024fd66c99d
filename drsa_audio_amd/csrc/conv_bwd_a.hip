// Instantiations of the 3x3 conv kernel (lrp_conv_kernel.h), split across files so the
// build compiles them in parallel.
#include "lrp_conv_kernel.h"

#ifndef DRSA_CONV_CIC_BWD64
#define DRSA_CONV_CIC_BWD64 16
#endif

namespace drsa_conv {
static const Entry kTableBwdA_e[] = {
    BWD_SET(128, 64, DRSA_CONV_CIC_BWD64),
    BWD_SET(64, 64, DRSA_CONV_CIC_BWD64),
};
extern const Table kTableBwdA = {kTableBwdA_e, (int)(sizeof(kTableBwdA_e) / sizeof(kTableBwdA_e[0]))};
}  // namespace drsa_conv
