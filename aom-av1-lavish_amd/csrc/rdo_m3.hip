// rdo_m3.hip -- instantiations of the C4 RDO kernels for mode 3 (TX-domain decision ranked by the coefficient rate);
// one translation unit per mode so the kernels build in parallel.
#define LAVISH_RDO_KERNELS
#include "rdo_kern.h"

namespace lavish {
int rdo_launch_m3(int tx_size, const RdoArgs& a, hipStream_t s) { return launch_size<3>(tx_size, a, s); }
}  // namespace lavish
