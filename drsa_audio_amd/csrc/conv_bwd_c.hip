// Instantiations of the 3x3 conv kernel (lrp_conv_kernel.h), split across files so the
// build compiles them in parallel.  VGGish-BN blocks 3-5 backward (128 -> 128 padded).
#include "lrp_conv_kernel.h"

namespace drsa_conv {
static const Entry kTableBwdC_e[] = {
    BWD_SET(128, 128, 8),
};
extern const Table kTableBwdC = {kTableBwdC_e, (int)(sizeof(kTableBwdC_e) / sizeof(kTableBwdC_e[0]))};
}  // namespace drsa_conv
