// Instantiations of the bf16-operand forward conv (lrp_conv_kernel.h, ET = 1), split across
// files so the build compiles them in parallel.  GTZAN trunk widths (create_model.py:100-137).
#include "lrp_conv_kernel.h"

namespace drsa_conv {
static const Entry kTableFwdBfA_e[] = {
    FWD_SET_BF(32, 32),
    FWD_SET_BF(32, 64)
};
extern const Table kTableFwdBfA = {kTableFwdBfA_e, (int)(sizeof(kTableFwdBfA_e) / sizeof(kTableFwdBfA_e[0]))};
}  // namespace drsa_conv
