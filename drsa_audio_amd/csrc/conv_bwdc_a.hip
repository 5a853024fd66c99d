// Instantiations of the clone-sharing backward conv (lrp_conv_clones.h): GTZAN/toy CNN trunk.
#include "lrp_conv_clones.h"

namespace drsa_conv {
static const Entry kTableBwdcA_e[] = {
    BWDC_SET(32, 32, 8),
    BWDC_SET(64, 32, 8),
};
extern const Table kTableBwdcA = {kTableBwdcA_e, (int)(sizeof(kTableBwdcA_e) / sizeof(kTableBwdcA_e[0]))};
}  // namespace drsa_conv
