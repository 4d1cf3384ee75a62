// rdo_m0.hip -- instantiations of the C4 RDO kernels for mode 0 (the txq_plane contract of the 64-point sizes);
// one translation unit per mode so the kernels build in parallel.
#define LAVISH_RDO_KERNELS
#include "rdo_kern.h"

namespace lavish {
int rdo_launch_m0(int tx_size, const RdoArgs& a, hipStream_t s) { return launch_size<0>(tx_size, a, s); }
}  // namespace lavish
