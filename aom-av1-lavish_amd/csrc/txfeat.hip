// txfeat.hip -- TX-type pruning features for gfx950.
//
// prune_tx_2D (av1/encoder/tx_search.c:1487-1537) scores the 16 TX types of
// a block with two small neural nets whose inputs are
//   get_energy_distribution_finer (tx_search.c:1411-1473): the block's
//     energy on a (w/2 for w > 8) x (h/2 for h > 8) grid, projected on the
//     columns / rows and normalised (float), and
//   av1_get_horver_correlation_full (av1/encoder/rdopt.c:514-609, an RTCD
//     function): the horizontal / vertical lag-1 correlation of the residual
//     (float).
// One 256-thread workgroup per block: the integer sums are exact (int64 /
// u32 accumulations, reduced through LDS), the float tails run in the
// reference's operation order with IEEE single precision -- correctly
// rounded division and sqrt (hipcc's default), no contraction -- so the
// results match the C reference bit for bit (the reference's own test allows
// 1e-6, test/horver_correlation_test.cc:70-73).
#include <stddef.h>
#include <string.h>

#include <map>
#include <mutex>
#include <vector>

#include "lavish_internal.h"

#pragma clang fp contract(off)

namespace lavish {
namespace {

constexpr int kTfThreads = 256;

// 12 exact sums of av1_get_horver_correlation_full
struct HvSums {
  int64_t v[12];  // x, x2, xy, xz, firstrow, finalrow, firstcol, finalcol, and their x2
};

__device__ __forceinline__ int64_t wg_sum64(int64_t v, int64_t* red) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) v += __shfl_xor(v, m);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// horver correlation of the w x h block at d (stride): every thread returns
// the same (hcorr, vcorr)
__device__ void horver(const int16_t* d, int stride, int w, int h, float& hcorr, float& vcorr,
                       int64_t* red) {
  int64_t s[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int p = threadIdx.x; p < w * h; p += kTfThreads) {
    const int i = p / w, j = p - i * w;
    const int x = d[(int64_t)i * stride + j];
    const int x2 = x * x;
    s[0] += x;
    s[1] += x2;
    if (j >= 1) s[2] += x * d[(int64_t)i * stride + j - 1];
    if (i >= 1) s[3] += x * d[(int64_t)(i - 1) * stride + j];
    if (i == 0) { s[4] += x; s[8] += x2; }
    if (i == h - 1) { s[5] += x; s[9] += x2; }
    if (j == 0) { s[6] += x; s[10] += x2; }
    if (j == w - 1) { s[7] += x; s[11] += x2; }
  }
#pragma unroll
  for (int k = 0; k < 12; ++k) s[k] = wg_sum64(s[k], red);
  const int64_t x_sum = s[0], x2_sum = s[1], xy_sum = s[2], xz_sum = s[3];
  const int64_t xhor_sum = x_sum - s[7], xver_sum = x_sum - s[5];
  const int64_t y_sum = x_sum - s[6], z_sum = x_sum - s[4];
  const int64_t x2hor_sum = x2_sum - s[11], x2ver_sum = x2_sum - s[9];
  const int64_t y2_sum = x2_sum - s[10], z2_sum = x2_sum - s[8];
  const float num_hor = (float)(h * (w - 1));
  const float num_ver = (float)((h - 1) * w);
  // C: int64 - (int64 / float): both int64 operands convert to float
  const float xhor_var_n = (float)x2hor_sum - (float)(xhor_sum * xhor_sum) / num_hor;
  const float xver_var_n = (float)x2ver_sum - (float)(xver_sum * xver_sum) / num_ver;
  const float y_var_n = (float)y2_sum - (float)(y_sum * y_sum) / num_hor;
  const float z_var_n = (float)z2_sum - (float)(z_sum * z_sum) / num_ver;
  const float xy_var_n = (float)xy_sum - (float)(xhor_sum * y_sum) / num_hor;
  const float xz_var_n = (float)xz_sum - (float)(xver_sum * z_sum) / num_ver;
  if (xhor_var_n > 0 && y_var_n > 0) {
    hcorr = xy_var_n / sqrtf(xhor_var_n * y_var_n);
    hcorr = hcorr < 0 ? 0 : hcorr;
  } else {
    hcorr = 1.0f;
  }
  if (xver_var_n > 0 && z_var_n > 0) {
    vcorr = xz_var_n / sqrtf(xver_var_n * z_var_n);
    vcorr = vcorr < 0 ? 0 : vcorr;
  } else {
    vcorr = 1.0f;
  }
}

// av1_get_horver_correlation_full over jobs of w x h blocks
__global__ __launch_bounds__(kTfThreads) void horver_kernel(const int16_t* __restrict__ res,
                                                            int stride, int bw, int nbx, int w,
                                                            int h, float* hcorr, float* vcorr) {
  __shared__ int64_t red[4];
  const int blk = blockIdx.x;
  const int by = blk / nbx, bx = blk - by * nbx;
  float hc, vc;
  horver(res + (int64_t)by * h * stride + (int64_t)bx * bw, stride, w, h, hc, vc, red);
  if (threadIdx.x == 0) {
    hcorr[blk] = hc;
    vcorr[blk] = vc;
  }
}

// prune_tx_2D's two feature vectors (tx_search.c:1516-1529) of the block at
// d into hf / vf (16 floats each, global or LDS): [0, n - 1) energy
// projection, [n - 1] correlation, the rest zero.  All threads call it.
__device__ void block_features(const int16_t* d, int stride, int bw, int bh, float* hf, float* vf,
                               int64_t* red, uint32_t* esq) {
  const int ws = bw <= 8 ? 0 : 1, hs = bh <= 8 ? 0 : 1;
  const int ew = bw >> ws, eh = bh >> hs, esz = ew * eh;
  // downscaled energies (get_energy_distribution_finer's esq)
  uint64_t tot = 0;
  for (int e = threadIdx.x; e < esz; e += kTfThreads) {
    const int ei = e / ew, ej = e - ei * ew;
    uint32_t acc = 0;
    for (int yy = 0; yy <= hs; ++yy)
      for (int xx = 0; xx <= ws; ++xx) {
        const int v = d[(int64_t)((ei << hs) + yy) * stride + (ej << ws) + xx];
        acc += (uint32_t)(v * v);
      }
    esq[e] = acc;
    tot += acc;
  }
  const uint64_t total = (uint64_t)wg_sum64((int64_t)tot, red);  // also orders esq[]
  const int t = threadIdx.x;
  if (total == 0) {
    if (t < ew - 1) hf[t] = 1.0f / ew;
    if (t >= 16 && t - 16 < eh - 1) vf[t - 16] = 1.0f / eh;
  } else {
    const float e_recip = 1.0f / (float)total;
    if (t < ew - 1) {  // hordist[t]: rows in order
      float a = 0.0f;
      for (int i = 0; i < eh; ++i) a += (float)esq[i * ew + t];
      hf[t] = a * e_recip;
    }
    if (t >= 16 && t - 16 < eh - 1) {  // verdist[i]: columns in order
      const int i = t - 16;
      float a = 0.0f;
      for (int j = 0; j < ew; ++j) a += (float)esq[i * ew + j];
      vf[i] = a * e_recip;
    }
  }
  if (t >= 32 && t < 48 && t - 32 >= ew) hf[t - 32] = 0.0f;
  if (t >= 48 && t < 64 && t - 48 >= eh) vf[t - 48] = 0.0f;
  float hc, vc;
  horver(d, stride, bw, bh, hc, vc, red);
  if (t == 0) {
    hf[ew - 1] = hc;
    vf[eh - 1] = vc;
  }
}

__global__ __launch_bounds__(kTfThreads) void prune_features_kernel(
    const int16_t* __restrict__ res, int stride, int nbx, int bw, int bh, float* hfeat,
    float* vfeat) {
  __shared__ int64_t red[4];
  __shared__ uint32_t esq[256];
  const int blk = blockIdx.x;
  const int by = blk / nbx, bx = blk - by * nbx;
  const int16_t* d = res + (int64_t)by * bh * stride + (int64_t)bx * bw;
  block_features(d, stride, bw, bh, hfeat + (int64_t)blk * 16, vfeat + (int64_t)blk * 16, red,
                 esq);
}

// ---- prune_tx_2D: the two nets, softmax, thresholds, sort, pruning ----
// A model on the device: header + weights / biases (float offsets into data).
struct DevNN {
  int nin, nout, nhl, hidden[10];
  int woff[11], boff[11];
  float data[1];
};

// tx_type_table_2D (tx_search.c:1493-1498) as TX_TYPE values
__constant__ uint8_t kTable2D[16] = {0, 2, 5, 10, 1, 3, 7, 12, 4, 8, 6, 14, 11, 13, 15, 9};
// av1_sort_fi32_16 / _8 comparator sequences (av1/encoder/sorting_network.h)
__constant__ uint8_t kSort16[65][2] = {
    {0, 1},  {2, 3},   {4, 5},   {6, 7},   {8, 9},   {10, 11}, {12, 13}, {14, 15}, {0, 2},
    {1, 3},  {4, 6},   {5, 7},   {8, 10},  {9, 11},  {12, 14}, {13, 15}, {1, 2},   {5, 6},
    {0, 4},  {3, 7},   {9, 10},  {13, 14}, {8, 12},  {11, 15}, {1, 5},   {2, 6},   {9, 13},
    {10, 14}, {0, 8},  {7, 15},  {1, 4},   {3, 6},   {9, 12},  {11, 14}, {2, 4},   {3, 5},
    {10, 12}, {11, 13}, {1, 9},  {6, 14},  {3, 4},   {11, 12}, {1, 8},   {2, 10},  {5, 13},
    {7, 14}, {3, 11},  {2, 8},   {4, 12},  {7, 13},  {3, 10},  {5, 12},  {3, 9},   {6, 12},
    {3, 8},  {7, 12},  {5, 9},   {6, 10},  {4, 8},   {7, 11},  {5, 8},   {7, 10},  {6, 8},
    {7, 9},  {7, 8}};
__constant__ uint8_t kSort8[19][2] = {{0, 1}, {2, 3}, {4, 5}, {6, 7}, {0, 2}, {1, 3}, {4, 6},
                                      {5, 7}, {1, 2}, {5, 6}, {0, 4}, {3, 7}, {1, 5}, {2, 6},
                                      {1, 4}, {3, 6}, {2, 4}, {3, 5}, {3, 4}};

// one layer of av1_nn_predict_c: node j (one thread each) sums its inputs in
// order; relu for hidden layers
__device__ __forceinline__ float nn_node(const DevNN* m, int layer, int node, const float* in,
                                         int nin, bool relu) {
  const float* w = m->data + m->woff[layer] + node * nin;
  float val = m->data[m->boff[layer] + node];
  for (int i = 0; i < nin; ++i) val += w[i] * in[i];
  return relu ? (val > 0.0f ? val : 0.0f) : val;
}

// av1_nn_predict_c(.., reduce_prec = 1) of both nets: threads [0, 128) run
// the horizontal model, [128, 256) the vertical one; out[0..3] / out[4..7]
__device__ void nn_pair(const DevNN* hm, const DevNN* vm, const float* hf, const float* vf,
                        float (*buf)[2][128], float* out) {
  const int side = threadIdx.x >> 7, j = threadIdx.x & 127;
  const DevNN* m = side ? vm : hm;
  const float* in = side ? vf : hf;
  int nin = m->nin;
  for (int layer = 0; layer < m->nhl; ++layer) {  // same depth for both: checked on the host
    const int nout = m->hidden[layer];
    float* o = buf[side][layer & 1];
    if (j < nout) o[j] = nn_node(m, layer, j, in, nin, true);
    __syncthreads();
    in = o;
    nin = nout;
  }
  if (j < m->nout) {
    const float v = nn_node(m, m->nhl, j, in, nin, false);
    // av1_nn_output_prec_reduce: (int)(v * 512 + 0.5) in double, * (float)(1.0 / 512)
    out[side * 4 + j] = (float)(int)((double)(v * 512.0f) + 0.5) * (float)(1.0 / 512);
  }
  __syncthreads();
}

__device__ __forceinline__ float approx_exp(float y) {
  constexpr float kA = (1 << 23) / 0.69314718056f;
  return __int_as_float((int32_t)(y * kA) + ((127 << 23) - 60801));
}

__device__ void sort_net(float* k, int* v, const uint8_t (*pairs)[2], int n) {
  for (int p = 0; p < n; ++p) {
    const int i = pairs[p][0], j = pairs[p][1];
    const bool ge = k[i] >= k[j];
    const float maxf = ge ? k[i] : k[j], minf = ge ? k[j] : k[i];
    const int maxi = ge ? v[i] : v[j], mini = ge ? v[j] : v[i];
    k[i] = maxf;
    k[j] = minf;
    v[i] = maxi;
    v[j] = mini;
  }
}

// the decision of prune_tx_2D (tx_search.c:1535-1640), one thread
__device__ void prune_decide(const float* hs, const float* vs, float thresh, int mode,
                             uint16_t mask_in, uint16_t* mask_out, uint8_t* map) {
  float raw[16];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) raw[i * 4 + j] = vs[i] * hs[j];
  // av1_nn_fast_softmax_16_c
  float mx = raw[0];
  for (int i = 1; i < 16; ++i) mx = mx > raw[i] ? mx : raw[i];
  float sum = 0.0f;
  for (int i = 0; i < 16; ++i) {
    const float t = raw[i] - mx;
    raw[i] = approx_exp(t > -10.0f ? t : -10.0f);
    sum += raw[i];
  }
  for (int i = 0; i < 16; ++i) raw[i] /= sum;
  int max_i = 0, count = 0;
  float max_score = 0.0f, ssum = 0.0f;
  uint16_t allow = 0;
  int allowed[16];
  float sc[16];
  for (int i = 0; i < 16; ++i) {
    allowed[i] = 255;
    sc[i] = -1.0f;
  }
  for (int t = 0; t < 16; ++t) {
    const int ty = kTable2D[t];
    if (!(mask_in & (1 << ty))) continue;
    if (raw[t] > max_score) {
      max_score = raw[t];
      max_i = t;
    }
    if (raw[t] >= thresh) {
      allow |= (uint16_t)(1 << ty);
      ssum += raw[t];
      sc[count] = raw[t];
      allowed[count] = ty;
      count++;
    }
  }
  if (!(allow & (1 << kTable2D[max_i]))) {
    *mask_out = allow | (uint16_t)(1 << kTable2D[max_i]);
    for (int i = 0; i < 16; ++i) map[i] = kTable2D[i];
    return;
  }
  if (count <= 8)
    sort_net(sc, allowed, kSort8, 19);
  else
    sort_net(sc, allowed, kSort16, 65);
  if (mode >= 4) {
    float temp = 0.0f, ratio = 0.0f;
    int t, n = 0;
    const float inv_sum = 100 / ssum;
    for (t = 0; t < count; t++) {
      if ((double)ratio > 30.0 && n >= 2) break;
      temp += sc[t];
      ratio = temp * inv_sum;
      n++;
    }
    for (; t < count; t++) allow &= (uint16_t)~(1 << allowed[t]);
  }
  for (int i = 0; i < 16; ++i) map[i] = (uint8_t)allowed[i];
  *mask_out = allow;
}

__global__ __launch_bounds__(kTfThreads) void prune_tx_2d_kernel(
    const int16_t* __restrict__ res, int stride, int nbx, int bw, int bh, const DevNN* hm,
    const DevNN* vm, float thresh, int mode, const uint16_t* allowed_in, uint16_t allowed_default,
    uint16_t* allowed_out, uint8_t* maps) {
  __shared__ int64_t red[4];
  __shared__ uint32_t esq[256];
  __shared__ float hf[16], vf[16], scores[8];
  __shared__ float buf[2][2][128];
  const int blk = blockIdx.x;
  const int by = blk / nbx, bx = blk - by * nbx;
  const int16_t* d = res + (int64_t)by * bh * stride + (int64_t)bx * bw;
  block_features(d, stride, bw, bh, hf, vf, red, esq);
  __syncthreads();
  nn_pair(hm, vm, hf, vf, buf, scores);
  if (threadIdx.x == 0) {
    const uint16_t m = allowed_in ? allowed_in[blk] : allowed_default;
    prune_decide(scores, scores + 4, thresh, mode, m, allowed_out + blk, maps + (int64_t)blk * 16);
  }
}

// av1_nn_predict_c for a batch of input vectors (one 128-thread workgroup each)
__global__ __launch_bounds__(128) void nn_predict_kernel(const DevNN* m, const float* in, int n,
                                                         int reduce_prec, float* out) {
  __shared__ float buf[2][128];
  __shared__ float x[128];
  const int v = blockIdx.x, j = threadIdx.x;
  if (j < m->nin) x[j] = in[(int64_t)v * m->nin + j];
  __syncthreads();
  const float* cur = x;
  int nin = m->nin;
  for (int layer = 0; layer < m->nhl; ++layer) {
    const int nout = m->hidden[layer];
    float* o = buf[layer & 1];
    if (j < nout) o[j] = nn_node(m, layer, j, cur, nin, true);
    __syncthreads();
    cur = o;
    nin = nout;
  }
  if (j < m->nout) {
    float r = nn_node(m, m->nhl, j, cur, nin, false);
    if (reduce_prec) r = (float)(int)((double)(r * 512.0f) + 0.5) * (float)(1.0 / 512);
    out[(int64_t)v * m->nout + j] = r;
  }
}

__global__ void prune_passthrough_kernel(int nb, const uint16_t* allowed_in,
                                         uint16_t allowed_default, uint16_t* allowed_out,
                                         uint8_t* maps) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb * 16) return;
  maps[i] = (uint8_t)(i & 15);
  if ((i & 15) == 0) allowed_out[i >> 4] = allowed_in ? allowed_in[i >> 4] : allowed_default;
}


// ---- NN models on the device (uploaded once per distinct content) ----
std::mutex g_nn_mu;
std::map<uint64_t, DevNN*> g_nn;

// nullptr when the config is out of this library's range (nodes <= 128,
// layers <= 10)
const DevNN* upload_nn(const LavishNNConfig* c) {
  if (!c || c->num_inputs < 1 || c->num_inputs > 128 || c->num_outputs < 1 ||
      c->num_outputs > 128 || c->num_hidden_layers < 0 || c->num_hidden_layers > 10)
    return nullptr;
  DevNN h{};
  h.nin = c->num_inputs;
  h.nout = c->num_outputs;
  h.nhl = c->num_hidden_layers;
  std::vector<float> data;
  int nin = h.nin;
  for (int l = 0; l <= h.nhl; ++l) {
    const int nout = l == h.nhl ? h.nout : c->num_hidden_nodes[l];
    if (nout < 1 || nout > 128 || !c->weights[l] || !c->bias[l]) return nullptr;
    if (l < h.nhl) h.hidden[l] = nout;
    h.woff[l] = (int)data.size();
    data.insert(data.end(), c->weights[l], c->weights[l] + (size_t)nin * nout);
    h.boff[l] = (int)data.size();
    data.insert(data.end(), c->bias[l], c->bias[l] + nout);
    nin = nout;
  }
  const size_t hdr = offsetof(DevNN, data);
  std::vector<char> blob(hdr + data.size() * sizeof(float));
  memcpy(blob.data(), &h, hdr);
  memcpy(blob.data() + hdr, data.data(), data.size() * sizeof(float));
  uint64_t key = 1469598103934665603ull;  // FNV-1a over the packed model
  for (char ch : blob) key = (key ^ (uint8_t)ch) * 1099511628211ull;
  std::lock_guard<std::mutex> lk(g_nn_mu);
  auto it = g_nn.find(key);
  if (it != g_nn.end()) return it->second;
  void* d = nullptr;
  LAVISH_CHECK(hipMalloc(&d, blob.size()));
  LAVISH_CHECK(hipMemcpy(d, blob.data(), blob.size(), hipMemcpyHostToDevice));
  g_nn[key] = (DevNN*)d;
  return (const DevNN*)d;
}

// prune_2D_adaptive_thresholds (tx_search.c:1336-1392); rows without a
// model have no entries
const float kThresh[19][14] = {
    {0.00549f, 0.01306f, 0.02039f, 0.02747f, 0.03406f, 0.04065f, 0.04724f, 0.05383f, 0.06067f,
     0.06799f, 0.07605f, 0.08533f, 0.09778f, 0.11780f},
    {0.00037f, 0.00183f, 0.00525f, 0.01038f, 0.01697f, 0.02502f, 0.03381f, 0.04333f, 0.05286f,
     0.06287f, 0.07434f, 0.08850f, 0.10803f, 0.14124f},
    {0.01404f, 0.02000f, 0.04211f, 0.05164f, 0.05798f, 0.06335f, 0.06897f, 0.07629f, 0.08875f,
     0.11169f},
    {}, {},
    {0.00183f, 0.00745f, 0.01428f, 0.02185f, 0.02966f, 0.03723f, 0.04456f, 0.05188f, 0.05920f,
     0.06702f, 0.07605f, 0.08704f, 0.10168f, 0.12585f},
    {0.00085f, 0.00476f, 0.01135f, 0.01892f, 0.02698f, 0.03528f, 0.04358f, 0.05164f, 0.05994f,
     0.06848f, 0.07849f, 0.09021f, 0.10583f, 0.13123f},
    {0.00037f, 0.00232f, 0.00671f, 0.01257f, 0.01965f, 0.02722f, 0.03552f, 0.04382f, 0.05237f,
     0.06189f, 0.07336f, 0.08728f, 0.10730f, 0.14221f},
    {0.00061f, 0.00330f, 0.00818f, 0.01453f, 0.02185f, 0.02966f, 0.03772f, 0.04578f, 0.05383f,
     0.06262f, 0.07288f, 0.08582f, 0.10339f, 0.13464f},
    {}, {}, {}, {},
    {0.00232f, 0.00671f, 0.01257f, 0.01941f, 0.02673f, 0.03430f, 0.04211f, 0.04968f, 0.05750f,
     0.06580f, 0.07507f, 0.08655f, 0.10242f, 0.12878f},
    {0.00110f, 0.00525f, 0.01208f, 0.01990f, 0.02795f, 0.03601f, 0.04358f, 0.05115f, 0.05896f,
     0.06702f, 0.07629f, 0.08752f, 0.10217f, 0.12610f},
    {}, {}, {}, {}};
const int kThreshLen[19] = {14, 14, 10, 0, 0, 14, 14, 14, 14, 0, 0, 0, 0, 14, 14, 0, 0, 0, 0};

}  // namespace

int horver_batch(const int16_t* residual, int stride, int width, int height, int bw, int bh,
                 float* hcorr, float* vcorr, hipStream_t s) {
  if (bw < 2 || bh < 2 || bw > 128 || bh > 128) return -1;
  if (width < 0 || height < 0 || stride < width) return -4;
  const int nbx = width / bw, nb = nbx * (height / bh);
  if (nb == 0) return 0;
  hipLaunchKernelGGL(horver_kernel, dim3(nb), dim3(kTfThreads), 0, s, residual, stride, bw, nbx,
                     bw, bh, hcorr, vcorr);
  LAVISH_CHECK(hipGetLastError());
  return 0;
}

}  // namespace lavish

using namespace lavish;

extern "C" int lavish_horver_correlation_batch(const int16_t* residual, int stride, int width,
                                               int height, int bw, int bh, float* hcorr,
                                               float* vcorr, void* stream) {
  return horver_batch(residual, stride, width, height, bw, bh, hcorr, vcorr,
                      (hipStream_t)stream);
}

extern "C" int lavish_tx_prune_features_batch(const int16_t* residual, int stride, int width,
                                              int height, int tx_size, float* hfeatures,
                                              float* vfeatures, void* stream) {
  if (tx_size < 0 || tx_size >= 19) return -1;
  const int bw = tx_w(tx_size), bh = tx_h(tx_size);
  if (bw > 32 || bh > 32) return -2;  // prune_tx_2D: at most 16 features per direction
  if (width < 0 || height < 0 || stride < width) return -4;
  const int nbx = width / bw, nb = nbx * (height / bh);
  if (nb == 0) return 0;
  hipLaunchKernelGGL(prune_features_kernel, dim3(nb), dim3(kTfThreads), 0, (hipStream_t)stream,
                     residual, stride, nbx, bw, bh, hfeatures, vfeatures);
  LAVISH_CHECK(hipGetLastError());
  return 0;
}

extern "C" int lavish_prune_tx_2d_batch(const int16_t* residual, int stride, int width,
                                        int height, int tx_size, int tx_set_type,
                                        int prune_2d_txfm_mode, const LavishNNConfig* nn_hor,
                                        const LavishNNConfig* nn_ver,
                                        const uint16_t* allowed_in, uint16_t allowed_default,
                                        uint16_t* allowed_out, uint8_t* txk_map, void* stream) {
  if (tx_size < 0 || tx_size >= 19) return -1;
  if (width < 0 || height < 0 || stride < width) return -4;
  const int bw = tx_w(tx_size), bh = tx_h(tx_size);
  const int nbx = width / bw, nb = nbx * (height / bh);
  // get_adaptive_thresholds' aggressiveness (tx_search.c:1394-1409)
  static const int aggr[5][2] = {{4, 1}, {6, 3}, {9, 6}, {9, 6}, {12, 9}};
  int ag = -1;
  if (prune_2d_txfm_mode >= 1 && prune_2d_txfm_mode <= 5) {
    if (tx_set_type == 5) ag = aggr[prune_2d_txfm_mode - 1][0];       // EXT_TX_SET_ALL16
    else if (tx_set_type == 4) ag = aggr[prune_2d_txfm_mode - 1][1];  // DTT9_IDTX_1DDCT
  }
  const bool active = ag >= 0 && nn_hor && nn_ver;
  hipStream_t s = (hipStream_t)stream;
  if (nb == 0) return 0;
  if (!active) {  // prune_tx_2D returns without touching mask / map
    hipLaunchKernelGGL(prune_passthrough_kernel, dim3((nb * 16 + 255) / 256), dim3(256), 0, s,
                       nb, allowed_in, allowed_default, allowed_out, txk_map);
    LAVISH_CHECK(hipGetLastError());
    return 0;
  }
  if (bw > 32 || bh > 32) return -2;          // at most 16 features per direction
  if (ag >= kThreshLen[tx_size]) return -2;   // no threshold: the reference has no model here
  const int hn = bw <= 8 ? bw : bw / 2, vn = bh <= 8 ? bh : bh / 2;
  if (nn_hor->num_inputs > 16 || nn_ver->num_inputs > 16 || nn_hor->num_inputs < 1 ||
      nn_ver->num_inputs < 1 || nn_hor->num_outputs != 4 || nn_ver->num_outputs != 4 ||
      nn_hor->num_hidden_layers != nn_ver->num_hidden_layers)
    return -3;
  (void)hn;
  (void)vn;
  const DevNN* hm = upload_nn(nn_hor);
  const DevNN* vm = upload_nn(nn_ver);
  if (!hm || !vm) return -3;
  hipLaunchKernelGGL(prune_tx_2d_kernel, dim3(nb), dim3(kTfThreads), 0, s, residual, stride, nbx,
                     bw, bh, hm, vm, kThresh[tx_size][ag], prune_2d_txfm_mode, allowed_in,
                     allowed_default, allowed_out, txk_map);
  LAVISH_CHECK(hipGetLastError());
  return 0;
}

extern "C" int lavish_nn_predict_batch(const float* inputs, const LavishNNConfig* nn_config,
                                       int reduce_prec, float* outputs, int n, void* stream) {
  if (n < 0) return -4;
  const DevNN* m = upload_nn(nn_config);
  if (!m) return -3;
  if (n == 0) return 0;
  hipLaunchKernelGGL(nn_predict_kernel, dim3(n), dim3(128), 0, (hipStream_t)stream, m, inputs, n,
                     reduce_prec, outputs);
  LAVISH_CHECK(hipGetLastError());
  return 0;
}
