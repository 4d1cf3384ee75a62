// lavish_internal.h -- host-side plumbing shared by the HIP translation units
// of liblavish_hip.so (error reporting, tables, launch helpers).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/lavish_dsp.h"

namespace lavish {

// Sticky status (lavish_hip_status): the reference's DSP entry points have no
// error channel (void / value returns), so a device failure is recorded here
// and reported loudly on stderr; by default the process aborts, because a
// silent wrong answer is worse than a crash for an encoder.
void set_error(const char* what, hipError_t e, const char* file, int line);

#define LAVISH_CHECK(x)                                              \
  do {                                                               \
    hipError_t e__ = (x);                                            \
    if (e__ != hipSuccess) ::lavish::set_error(#x, e__, __FILE__, __LINE__); \
  } while (0)

int tx_w(int tx_size);
int tx_h(int tx_size);
int max_eob(int tx_size);
int tx_scale(int tx_size);
bool tx_type_valid(int tx_size, int tx_type);
int scan_kind(int tx_type);  // 0 default, 1 mcol, 2 mrow

// host copies of the scan / inverse-scan orders (av1_scan_orders)
const int16_t* host_scan(int tx_size, int tx_type);
const int16_t* host_iscan(int tx_size, int tx_type);
// device copies (uploaded on first use, per device)
const int16_t* dev_iscan(int tx_size, int tx_type);
const int16_t* dev_iscan_rows(int tx_size);  // [3 kinds][KH][KW], lane-row order
const int16_t* dev_scan(int tx_size, int tx_type);

// lavish_txq_plane for the 64-point TX sizes (rdo.hip)
int txq_plane_64(const int16_t* residual, int stride, int width, int height, int tx_size,
                 uint32_t type_mask, int bd, int quant_kind, const LavishQuantParams* qp,
                 int32_t* qcoeff, int32_t* dqcoeff, uint16_t* eob, int32_t* coeff,
                 hipStream_t s);

// inverse transform batch (inv.hip); slot_cnt (device, nullable): the job
// list is njobs / slot_cap slots of slot_cap jobs, of which the first
// slot_cnt[slot] are live (job lists built on the device)
// the C4 reconstruction's inverse transforms in one launch (inv.hip): per
// candidate size t (jobs[t] != nullptr) the per-SB job slots and counts
// sb_decide_kernel wrote, the dequantized coefficients, the SBs' chosen sizes
struct InvSbArgs {
  const int32_t* dq[19];
  const LavishInvJob* jobs[19];
  const uint16_t* cnt[19];
  const uint8_t* sb_tx_size;
  int nsb;
  uint16_t* dst;
  int stride;
};
int recon_sb_launch(const InvSbArgs& a, int bd, hipStream_t s);
int inv_txfm_add_batch(const int32_t* dq, int tx_size, const LavishInvJob* jobs, int njobs,
                       void* dst, int stride, int bd, int highbd, hipStream_t s,
                       const uint16_t* slot_cnt = nullptr, int slot_cap = 0);
// the coefficient-rate decision (lavish_rdo_plane_rate): device CoeffCosts,
// per-block TXB_CTX (nullable) and get_tx_type_cost per tx type (host, nullable)
struct RateCfg {
  const LavishCoeffCosts* costs;
  const LavishTxbCtx* txb_ctx;
  const int32_t* tx_type_costs;
};
struct RdoArgs;
// args_only (mode 1 only): fill *args_only instead of launching
int rdo_plane(const uint16_t* src, const uint16_t* pred, int stride, int width, int height,
              int tx_size, uint32_t type_mask, int bd, const LavishQuantParams* qp, int rdmult,
              LavishRdoBlock* out, int32_t* qcoeff, int32_t* dqcoeff, hipStream_t s,
              int px = 0, const uint16_t* block_mask = nullptr,
              const uint8_t* block_map = nullptr, const RateCfg* rate = nullptr,
              RdoArgs* args_only = nullptr);

// inter prediction batch (inter.hip); custom = an RTCD shim's own kernels
int inter_pred_batch(const void* ref, int ref_stride, int ref_width, int ref_height, int ss_x,
                     int ss_y, int w, int h, const LavishInterPredJob* jobs, int njobs,
                     const LavishSubpelResult* mvs, void* dst, int dst_stride, int bd, int highbd,
                     const int16_t* custom, int r0, int r1, hipStream_t s);

// fork / join over the library's per-thread internal streams
int fan_width();
int set_fan_width(int w);
hipStream_t* fan_out(hipStream_t caller);
void fan_in(hipStream_t caller);
// a private set of internal streams and fork / join events: while installed
// (fan_use) this thread's fan_out / fan_in use it instead of the shared
// per-thread set (nullptr: back to the shared set).  A captured graph's
// fan-out gets its own set, so its fork / join events and streams are never
// the ones uncaptured calls record and wait on.
struct FanSet;
FanSet* fan_create();
void fan_destroy(FanSet* f);
void fan_use(FanSet* f);

// av1_highbd_iwht4x4_add (av1/common/idct.c:34-40) on a host u16 4x4 block
// (wht.hip): the lossless branch of the inverse-transform shims
void iwht_host(const int32_t* input, uint16_t* dest, int stride, int eob, int bd);

// per-thread scratch device buffer for the per-call (host pointer) shims
void* shim_scratch(size_t bytes);
hipStream_t shim_stream();

// Argument rejection inside a per-call shim (which has no error channel):
// recorded in the sticky status like a HIP failure, then abort unless
// lavish_hip_set_abort_on_error(0).
void shim_reject(const char* what, int rc);

// Device scratch reused by calls that may be queued on different streams.
// acquire() makes `s` wait for the event the previous user's release()
// recorded, so the buffer is never rewritten while an earlier kernel (on any
// stream) may still read it; growing it waits for that event on the host.
struct StreamScratch {
  int device = -1;
  void* ptr = nullptr;
  size_t cap = 0;
  hipEvent_t done = nullptr;
  bool pending = false;
  void* acquire(size_t bytes, hipStream_t s);
  void release(hipStream_t s);
};

// Under-aligned word vectors for byte-addressed loads (pixel rows at any byte
// offset).  aligned(1) makes no alignment promise to the compiler, so it
// cannot split, merge or scalarise on an assumed 8 / 16-byte boundary; the
// queues run in unaligned-access mode, so each still lowers to one
// global_load_dwordx2 / x4 (or ds_read_b64 / b128) at the byte address.
typedef uint32_t u32x2u __attribute__((ext_vector_type(2), aligned(1)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));

// Wave-local memory ordering: lanes of one wave exchange data through LDS
// with no workgroup barrier (each wave owns its tile); these fences only stop
// the compiler from moving LDS accesses across the exchange point (LDS ops of
// one wave are processed in order).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace lavish
