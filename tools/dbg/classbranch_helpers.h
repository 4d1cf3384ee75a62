// The class-branching get_nz_mag / get_br_ctx helpers that ROCm 7.2
// miscompiles for the vertical class once inlined into the trellis walk
// (profiles/r03_trellis_miscompile_isa.txt).  Not part of the product: only
// tools/dbg/build_trellis_cb.sh compiles them (force-included into a copy of
// trellis.hip) to reproduce the fault.
#pragma once
#include "../../aom-av1-lavish_amd/csrc/coeffcost_dev.h"
namespace lavish {
namespace cc {
// get_nz_mag (txb_common.h:150-173) + get_nz_map_ctx_from_stats over the map
__device__ __forceinline__ int lower_ctx(int cls, int wlt, int wgt, const uint8_t* lv, int stride,
                                         int pos, int col, int row) {
  const uint8_t* l = lv + col * stride + row;
  int mag = min3(l[stride]) + min3(l[1]);
  if (cls == 0) {
    mag += min3(l[stride + 1]) + min3(l[2 * stride]) + min3(l[2]);
  } else if (cls == 2) {
    mag += min3(l[2]) + min3(l[3]) + min3(l[4]);
  } else {
    mag += min3(l[2 * stride]) + min3(l[3 * stride]) + min3(l[4 * stride]);
  }
  return nz_ctx(cls, wlt, wgt, mag, pos, col, row);
}

// get_br_ctx (txb_common.h:103-135) over the map
__device__ __forceinline__ int br_ctx(int cls, const uint8_t* lv, int stride, int pos, int col,
                                      int row) {
  const uint8_t* l = lv + col * stride + row;
  const int third = cls == 0 ? l[stride + 1] : (cls == 1 ? l[2 * stride] : l[2]);
  return br_ctx_mag(cls, l[1] + l[stride] + third, pos, col, row);
}

}  // namespace cc
}  // namespace lavish
