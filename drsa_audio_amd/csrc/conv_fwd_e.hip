// Instantiations of the 3x3 conv kernel (lrp_conv_kernel.h), split across files so the
// build compiles them in parallel.  VGGish-BN blocks 3-5 (100/128 -> 128 channels padded).
#include "lrp_conv_kernel.h"

#ifndef DRSA_CONV_CIC_FWD128_128
#define DRSA_CONV_CIC_FWD128_128 4   // 8 x 8 tiles at 3 waves/SIMD (168 VGPRs): conv_fwd:features.12 0.106 -> 0.092 ms
#endif

namespace drsa_conv {
static const Entry kTableFwdE_e[] = {
    FWD_SET(128, 128, DRSA_CONV_CIC_FWD128_128),
};
extern const Table kTableFwdE = {kTableFwdE_e, (int)(sizeof(kTableFwdE_e) / sizeof(kTableFwdE_e[0]))};
}  // namespace drsa_conv
