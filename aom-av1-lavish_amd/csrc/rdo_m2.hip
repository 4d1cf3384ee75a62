// rdo_m2.hip -- instantiations of the C4 RDO kernels for mode 2 (pixel-domain decision);
// one translation unit per mode so the kernels build in parallel.
#define LAVISH_RDO_KERNELS
#include "rdo_kern.h"

namespace lavish {
int rdo_launch_m2(int tx_size, const RdoArgs& a, hipStream_t s) { return launch_size<2>(tx_size, a, s); }
}  // namespace lavish
