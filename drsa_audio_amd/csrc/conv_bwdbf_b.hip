// Instantiations of the bf16-operand per-clone backward conv (see conv_bwdbf_a.hip): 128-wide g.
#include "lrp_conv_kernel.h"

namespace drsa_conv {
static const Entry kTableBwdBfB_e[] = {
    BWD_SET_BF(128, 64),
    BWD_SET_BF(128, 128),
};
extern const Table kTableBwdBfB = {kTableBwdBfB_e, (int)(sizeof(kTableBwdBfB_e) / sizeof(kTableBwdBfB_e[0]))};
}  // namespace drsa_conv
