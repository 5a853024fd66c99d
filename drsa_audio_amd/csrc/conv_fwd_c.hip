// Instantiations of the 3x3 conv kernel (lrp_conv_kernel.h), split across files so the
// build compiles them in parallel.
#include "lrp_conv_kernel.h"

#ifndef DRSA_CONV_CIC_FWD64_64
#define DRSA_CONV_CIC_FWD64_64 4   // 8 x 8 tiles: 116 VGPRs, 4 waves/SIMD (conv_fwd:features.9 0.266 -> 0.257 ms)
#endif
#ifndef DRSA_CONV_CIC_FWD64_128
#define DRSA_CONV_CIC_FWD64_128 4   // 8 x 8 tiles at 3 waves/SIMD (166 VGPRs)
#endif

namespace drsa_conv {
static const Entry kTableFwdC_e[] = {
    FWD_SET(64, 64, DRSA_CONV_CIC_FWD64_64),
    FWD_SET(64, 128, DRSA_CONV_CIC_FWD64_128),
};
extern const Table kTableFwdC = {kTableFwdC_e, (int)(sizeof(kTableFwdC_e) / sizeof(kTableFwdC_e[0]))};
}  // namespace drsa_conv
