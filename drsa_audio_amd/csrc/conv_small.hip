// Instantiations of the 3x3 conv kernel (lrp_conv_kernel.h) on 4 x 8 tiles (one 32-pixel m-tile
// per workgroup) for the small maps where 8 x 8 tiles leave the chip under-filled: lrp_conv.hip's
// launch() takes one of these in place of the 8 x 8 entry of the same layer when the 8 x 8 grid
// would have fewer than kSmallWorkgroups workgroups (GTZAN features.12 at 8 x 8, the VGGish blocks
// 4-5 at 16 x 16 and 8 x 8 with their batch of 32).  Same k order, same bits.
#include "lrp_conv_kernel.h"

#define SMALL_FWD(CIN, COUT, CIC)                                                          \
  CONV_ENTRY(CIN, COUT, 4, 8, 4, CIC, 1, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_POOL),     \
  CONV_ENTRY(CIN, COUT, 4, 8, 4, CIC, 2, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_POOL),     \
  CONV_ENTRY(CIN, COUT, 4, 8, 4, CIC, 3, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_POOL),     \
  CONV_ENTRY(CIN, COUT, 4, 8, 4, CIC, 1, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_RELU),     \
  CONV_ENTRY(CIN, COUT, 4, 8, 4, CIC, 2, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_RELU),     \
  CONV_ENTRY(CIN, COUT, 4, 8, 4, CIC, 3, drsa_conv::A_DENSE, drsa_conv::EPI_FWD_RELU)
#define SMALL_BWD(CIN, COUT, CIC)                                                          \
  CONV_ENTRY(CIN, COUT, 4, 8, 4, CIC, 1, drsa_conv::A_DENSE, drsa_conv::EPI_BWD),          \
  CONV_ENTRY(CIN, COUT, 4, 8, 4, CIC, 2, drsa_conv::A_DENSE, drsa_conv::EPI_BWD),          \
  CONV_ENTRY(CIN, COUT, 4, 8, 4, CIC, 1, drsa_conv::A_POOLSPARSE, drsa_conv::EPI_BWD),     \
  CONV_ENTRY(CIN, COUT, 4, 8, 4, CIC, 2, drsa_conv::A_POOLSPARSE, drsa_conv::EPI_BWD)

namespace drsa_conv {
static const Entry kTableSmall_e[] = {
    SMALL_FWD(64, 128, 4),
    SMALL_FWD(128, 128, 4),
    SMALL_BWD(128, 64, 16),
    SMALL_BWD(128, 128, 8),
};
extern const Table kTableSmall = {kTableSmall_e, (int)(sizeof(kTableSmall_e) / sizeof(kTableSmall_e[0]))};
}  // namespace drsa_conv
