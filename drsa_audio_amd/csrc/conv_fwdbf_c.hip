// Instantiations of the bf16-operand forward conv (lrp_conv_kernel.h, ET = 1), split across
// files so the build compiles them in parallel.  VGGish-BN blocks 3-5 (100 channels pad to 128).
#include "lrp_conv_kernel.h"

namespace drsa_conv {
static const Entry kTableFwdBfC_e[] = {
    FWD_SET_BF(64, 128),
    FWD_SET_BF(128, 128)
};
extern const Table kTableFwdBfC = {kTableFwdBfC_e, (int)(sizeof(kTableFwdBfC_e) / sizeof(kTableFwdBfC_e[0]))};
}  // namespace drsa_conv
