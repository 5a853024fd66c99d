// Instantiations of the 3x3 conv kernel (lrp_conv_kernel.h), split across files so the
// build compiles them in parallel.
#include "lrp_conv_kernel.h"

namespace drsa_conv {
static const Entry kTableBwdB_e[] = {
    BWD_SET(64, 32, 16),
    BWD_SET(32, 32, 16),
};
extern const Table kTableBwdB = {kTableBwdB_e, (int)(sizeof(kTableBwdB_e) / sizeof(kTableBwdB_e[0]))};
}  // namespace drsa_conv
