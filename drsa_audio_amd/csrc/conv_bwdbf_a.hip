// Instantiations of the bf16-operand per-clone backward conv (lrp_conv_kernel.h, ET = 1, EPI_BWD),
// split across files so the build compiles them in parallel: the GTZAN and VGGish trunk widths
// (backward cin = forward cout, backward cout = forward cin, both padded to 32).
#include "lrp_conv_kernel.h"

namespace drsa_conv {
static const Entry kTableBwdBfA_e[] = {
    BWD_SET_BF(32, 32),
    BWD_SET_BF(64, 32),
    BWD_SET_BF(64, 64),
    BWD_SET_BF_P4(64, 64),
};
extern const Table kTableBwdBfA = {kTableBwdBfA_e, (int)(sizeof(kTableBwdBfA_e) / sizeof(kTableBwdBfA_e[0]))};
}  // namespace drsa_conv
