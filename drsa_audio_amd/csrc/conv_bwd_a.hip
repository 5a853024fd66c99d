// Instantiations of the 3x3 conv kernel (lrp_conv_kernel.h), split across files so the
// build compiles them in parallel.
#include "lrp_conv_kernel.h"

// backward into 64 channels: 8 x 16 tiles at W >= 32 (lrp_conv.hip's find(); the 8 x 32 tile with
// either chunk size spills) and 8 x 8 tiles below, 8-channel chunks except the 8 x 8 tiles of the
// backward from 128 channels (16).  At W >= 32 (VGGish blocks 1-2) the 8-channel chunk takes 124
// VGPRs, 4 waves/SIMD instead of 3 (16-channel chunks: 148): conv_bwd:features.3 0.75 -> 0.66 ms,
// .7 0.107 -> 0.092 ms, fp32 standard LRP 7.94k -> 8.11k samples/s.
#ifndef DRSA_CONV_CIC_BWD64
#define DRSA_CONV_CIC_BWD64 8
#endif
#ifndef DRSA_CONV_CIC_BWD64_T8
#define DRSA_CONV_CIC_BWD64_T8 8
#endif

#define CONV_FAMILY_BWD64(CIN, NG, AM, C8)                                              \
  CONV_ENTRY(CIN, 64, 8, 16, 8, DRSA_CONV_CIC_BWD64, NG, AM, drsa_conv::EPI_BWD),       \
  CONV_ENTRY(CIN, 64, 8, 8, 4, C8, NG, AM, drsa_conv::EPI_BWD)
// C8: the chunk of the 8 x 8 tile (64 -> 64: 8, 0.212 -> 0.193 ms; 128 -> 64: 16, 0.053 vs 0.057 ms)
#define BWD_SET64(CIN, C8)                                          \
  CONV_FAMILY_BWD64(CIN, 1, drsa_conv::A_DENSE, C8),                \
  CONV_FAMILY_BWD64(CIN, 2, drsa_conv::A_DENSE, C8),                \
  CONV_FAMILY_BWD64(CIN, 1, drsa_conv::A_POOLSPARSE, C8),           \
  CONV_FAMILY_BWD64(CIN, 2, drsa_conv::A_POOLSPARSE, C8)

namespace drsa_conv {
static const Entry kTableBwdA_e[] = {
    BWD_SET64(128, 16),
    BWD_SET64(64, DRSA_CONV_CIC_BWD64_T8),
    // the (2,4) pool backward folded into the staging (VGGish block 1 at W = 256: 8 x 16 tiles)
    CONV_ENTRY_P4B(64, 64, 8, 16, 8, DRSA_CONV_CIC_BWD64),
};
extern const Table kTableBwdA = {kTableBwdA_e, (int)(sizeof(kTableBwdA_e) / sizeof(kTableBwdA_e[0]))};
}  // namespace drsa_conv
