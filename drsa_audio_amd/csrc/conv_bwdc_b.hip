// Instantiations of the clone-sharing backward conv (lrp_conv_clones.h): 64-channel blocks.
#include "lrp_conv_clones.h"

namespace drsa_conv {
static const Entry kTableBwdcB_e[] = {
    BWDC_SET(64, 64, 16),
    BWDC_SET(128, 64, 16),
};
extern const Table kTableBwdcB = {kTableBwdcB_e, (int)(sizeof(kTableBwdcB_e) / sizeof(kTableBwdcB_e[0]))};
}  // namespace drsa_conv
