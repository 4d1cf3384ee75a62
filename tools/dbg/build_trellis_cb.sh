#!/bin/bash
# A/B build for the trellis "miscompile" question:
# liblavish_hip.so with trellis.hip switched back to the class-branching
# lower_ctx / br_ctx helpers (the form before f80efb2), everything else the
# in-tree objects.  Output: tools/dbg/liblavish_cb.so (+ both ISA listings
# under /tmp/tv).  Run the trellis tests against it with
#   LAVISH_HIP_LIB=tools/dbg/liblavish_cb.so python -m pytest tests/test_gpu_trellis.py
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
P=$R/aom-av1-lavish_amd
T=/tmp/tv
mkdir -p $T
sed -e 's/lower_ctx_off(nb, cls,/lower_ctx(cls,/' -e 's/br_ctx_off(nb, cls,/br_ctx(cls,/g' \
    $P/csrc/trellis.hip > $P/csrc/_trellis_cb.hip
grep -c "lower_ctx(cls\|br_ctx(cls" $P/csrc/_trellis_cb.hip
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics"
CB="-include $R/tools/dbg/classbranch_helpers.h"
/opt/rocm/bin/hipcc $F $CB -c $P/csrc/_trellis_cb.hip -o $T/trellis_cb.o
/opt/rocm/bin/hipcc $F $CB --cuda-device-only -S $P/csrc/_trellis_cb.hip -o $T/trellis_cb.s
/opt/rocm/bin/hipcc $F --cuda-device-only -S $P/csrc/trellis.hip -o $T/trellis_off.s
rm -f $P/csrc/_trellis_cb.hip
objs=$(ls $P/build/*.o | grep -v '/trellis.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $R/tools/dbg/liblavish_cb.so $objs $T/trellis_cb.o
echo built $R/tools/dbg/liblavish_cb.so
