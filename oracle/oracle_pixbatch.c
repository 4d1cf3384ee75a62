/* oracle_pixbatch.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Batch driver over the oracle's restated 8-bit pixel primitives, for the
 * `pixel` bench workload's CPU baseline: per job (the LavishPixJob layout)
 * the 4-candidate SAD of aom_sad{w}x{h}x4d (aom_dsp/sad.c:60-78, here
 * orc_sad per candidate) and aom_variance{w}x{h} against candidate 0
 * (aom_dsp/variance.c:38-55, orc_variance).  Jobs split over pthreads.
 */
#include <pthread.h>
#include <stdint.h>

#include "oracle.h"

typedef struct {
  int64_t src_off, ref_off[4], aux_off;
  int32_t xoff, yoff;
} PixJob;

typedef struct {
  const uint8_t *src, *ref;
  int ss, rs, w, h;
  const PixJob *jobs;
  uint32_t *sad, *var, *sse;
  long lo, hi;
} PbArg;

static void *pb_worker(void *p) {
  const PbArg *a = (const PbArg *)p;
  for (long j = a->lo; j < a->hi; ++j) {
    const PixJob *jb = &a->jobs[j];
    for (int k = 0; k < 4; ++k)
      a->sad[4 * j + k] =
          orc_sad(a->src + jb->src_off, a->ss, a->ref + jb->ref_off[k], a->rs, a->w, a->h);
    unsigned int sse = 0;
    a->var[j] = orc_variance(a->src + jb->src_off, a->ss, a->ref + jb->ref_off[0], a->rs, a->w,
                             a->h, &sse);
    a->sse[j] = sse;
  }
  return NULL;
}

void orc_pixel_batch(const uint8_t *src, int ss, const uint8_t *ref, int rs, int w, int h,
                     const void *jobs, long njobs, uint32_t *sad, uint32_t *var, uint32_t *sse,
                     int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  PbArg args[256];
  for (int t = 0; t < threads; ++t) {
    PbArg *a = &args[t];
    a->src = src;
    a->ref = ref;
    a->ss = ss;
    a->rs = rs;
    a->w = w;
    a->h = h;
    a->jobs = (const PixJob *)jobs;
    a->sad = sad;
    a->var = var;
    a->sse = sse;
    a->lo = njobs * t / threads;
    a->hi = njobs * (t + 1) / threads;
    if (threads > 1) pthread_create(&tid[t], NULL, pb_worker, a);
    else pb_worker(a);
  }
  if (threads > 1)
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
}
