// Instantiations of the 3x3 conv kernel (lrp_conv_kernel.h), split across files so the
// build compiles them in parallel.
#include "lrp_conv_kernel.h"

#ifndef DRSA_CONV_CIC_BWD32
#define DRSA_CONV_CIC_BWD32 8
#endif
#ifndef DRSA_CONV_CIC_BWD64_32
#define DRSA_CONV_CIC_BWD64_32 8
#endif

namespace drsa_conv {
static const Entry kTableBwdB_e[] = {
    BWD_SET(64, 32, DRSA_CONV_CIC_BWD64_32),
    BWD_SET(32, 32, DRSA_CONV_CIC_BWD32),
};
extern const Table kTableBwdB = {kTableBwdB_e, (int)(sizeof(kTableBwdB_e) / sizeof(kTableBwdB_e[0]))};
}  // namespace drsa_conv

#ifdef DRSA_CONV_STAMP
extern "C" int drsa_amd_debug_conv_stamps(void* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(drsa_conv::g_conv_stamps), &buf, sizeof(buf));
}
#endif
