// rdo_m1.hip -- instantiations of the C4 RDO kernels for mode 1 (TX-domain decision);
// one translation unit per mode so the kernels build in parallel.
#define LAVISH_RDO_KERNELS
#include "rdo_kern.h"

namespace lavish {
int rdo_launch_m1(int tx_size, const RdoArgs& a, hipStream_t s) { return launch_size<1>(tx_size, a, s); }
int rdo_small_launch_m1(const RdoSmall& m, hipStream_t s) {
  if (m.first[3] <= 0) return 0;
  hipLaunchKernelGGL(rdo_small_kernel<1>, dim3(m.first[3]), dim3(256), 0, s, m);
  LAVISH_CHECK(hipGetLastError());
  return 0;
}
}  // namespace lavish
