// Instantiations of the 3x3 conv kernel with the 2x4 max-pool fused into the forward epilogue
// (lrp_conv_kernel.h, PW = 4): VGGish-BN block 1 (64 -> 64 at 128x256, pool_kernels[0] = (2,4),
// create_model.py:61), fp32 (CIC 8) and bf16 operands.
#include "lrp_conv_kernel.h"

namespace drsa_conv {
static const Entry kTableFwdP4_e[] = {
    FWD_SET_P4(64, 64, 8, 0),
    FWD_SET_P4(64, 64, 16, 1),
};
extern const Table kTableFwdP4 = {kTableFwdP4_e, (int)(sizeof(kTableFwdP4_e) / sizeof(kTableFwdP4_e[0]))};
}  // namespace drsa_conv
