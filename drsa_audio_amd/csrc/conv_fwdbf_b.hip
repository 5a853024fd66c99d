// Instantiations of the bf16-operand forward conv (lrp_conv_kernel.h, ET = 1), split across
// files so the build compiles them in parallel.  64-channel trunk (GTZAN blocks 3-4, VGGish blocks 1-2).
#include "lrp_conv_kernel.h"

namespace drsa_conv {
static const Entry kTableFwdBfB_e[] = {
    FWD_SET_BF(64, 64)
};
extern const Table kTableFwdBfB = {kTableFwdBfB_e, (int)(sizeof(kTableFwdBfB_e) / sizeof(kTableFwdBfB_e[0]))};
}  // namespace drsa_conv
