// elementwise.hip -- HBM-bound wave-level kernels of the diffusion hot path:
// timestep embedding, DDPM/DDIM scheduler math and nearest upsampling.
//
// Every tensor kernel moves 8 elements per lane (16 B for bf16, 2x16 B for
// fp32) when the per-sample length allows it, and gathers the per-sample
// schedule scalars from the fp32 tables on device (no host sync on t).
#include "vd_common.h"
#include <math.h>

namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t work) {
  int64_t g = vd_cdiv(work, kBlock);
  const int64_t cap = 256 * 16;  // 16 blocks per CU, then grid-stride
  return (int)(g < cap ? (g > 0 ? g : 1) : cap);
}

// ------------------------------------------------------------ timestep embedding
// freqs: the caller's table (nullptr: computed here)
__global__ void temb_kernel(const int64_t* __restrict__ t, int B, int dim, float log_max_period,
                            const float* __restrict__ freqs, float* __restrict__ out) {
  const int half = dim / 2;
  const int n = B * dim;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int b = i / dim, j = i % dim;
    float v = 0.f;
    if (j < 2 * half) {
      const int f = j < half ? j : j - half;
      // utils.py:150-152: exp(-ln(max_period) * arange(half) / half) in fp32
      const float freq = freqs ? freqs[f] : expf(-log_max_period * (float)f / (float)half);
      const float arg = (float)t[b] * freq;
      v = j < half ? cosf(arg) : sinf(arg);
    }
    out[i] = v;
  }
}

// ------------------------------------------------------------ scheduler math
// A per-element op sees (b, scalars) and 8-wide vectors of its inputs.
struct QSample {
  const float *sa, *s1m;
  __device__ void operator()(int64_t tb, const float* xa, const float* xb, const float*,
                             float* o0, float*, int n) const {
    const float a = sa[tb], c = s1m[tb];
    for (int i = 0; i < n; ++i) o0[i] = a * xa[i] + c * xb[i];
  }
};

struct PSampleV1 {
  const float *betas, *alphas, *acp, *s1m;
  __device__ void operator()(int64_t tb, const float* xt, const float* eps, const float* z,
                             float* xprev, float* x0, int n) const {
    const float s1 = s1m[tb];
    const float sq_acp = sqrtf(acp[tb]);
    const float beta = betas[tb];
    const float sq_alpha = sqrtf(alphas[tb]);
    float sigma = 0.f;
    if (tb > 0) sigma = sqrtf((1.f - acp[tb - 1]) / (1.f - acp[tb]) * beta);
    for (int i = 0; i < n; ++i) {
      float x = (xt[i] - s1 * eps[i]) / sq_acp;
      x0[i] = fminf(fmaxf(x, -1.f), 1.f);
      float mean = (xt[i] - (beta * eps[i]) / s1) / sq_alpha;
      xprev[i] = tb > 0 ? mean + sigma * z[i] : mean;
    }
  }
};

struct PSampleV2 {
  const float *betas, *alphas, *acp, *sa, *s1m;
  __device__ void operator()(int64_t tb, const float* xt, const float* eps, const float* z,
                             float* xprev, float* x0, int n) const {
    const float s1 = s1m[tb];
    const float sq_alpha = sqrtf(alphas[tb]);
    const float sigma = sqrtf((1.f - acp[tb]) * betas[tb]);
    const float a = sa[tb];
    for (int i = 0; i < n; ++i) {
      float mean = xt[i] - (s1 * eps[i]) / sq_alpha;
      xprev[i] = mean + sigma * z[i];
      float x = (xt[i] - s1 * eps[i]) / a;
      x0[i] = fminf(fmaxf(x, -1.f), 1.f);
    }
  }
};

struct PSampleCos {
  const float *acp, *sa, *s1m;
  __device__ void operator()(int64_t tb, const float* xt, const float* eps, const float* z,
                             float* xprev, float* mean_out, int n) const {
    const float s1 = s1m[tb], a = sa[tb];
    float sigma = 0.f;
    if (tb > 0) sigma = sqrtf(acp[tb - 1] * (1.f - acp[tb]) / (1.f - acp[tb - 1]));
    for (int i = 0; i < n; ++i) {
      float mean = (xt[i] - s1 * eps[i]) / a;
      mean_out[i] = mean;
      xprev[i] = tb > 0 ? mean + sigma * z[i] : mean;
    }
  }
};

struct DDIMStep {
  const float* acp;
  const int64_t* tprev;
  float eta;
  int clip;
  int has_z;
  // b index is passed through tb via the high bits? no: operator gets tb and b.
  __device__ void run(int64_t tb, int64_t tp, const float* xt, const float* eps, const float* z,
                      float* xprev, float* x0o, int n) const {
    const float at = acp[tb];
    const float ap = tp >= 0 ? acp[tp] : 1.f;
    const float sq_at = sqrtf(at), sq_1mat = sqrtf(1.f - at);
    const float sigma = eta * sqrtf((1.f - ap) / (1.f - at) * (1.f - at / ap));
    const float dir = sqrtf(fmaxf(1.f - ap - sigma * sigma, 0.f));
    const float sq_ap = sqrtf(ap);
    for (int i = 0; i < n; ++i) {
      float x0 = (xt[i] - sq_1mat * eps[i]) / sq_at;
      if (clip) x0 = fminf(fmaxf(x0, -1.f), 1.f);
      x0o[i] = x0;
      float v = sq_ap * x0 + dir * eps[i];
      if (has_z) v += sigma * z[i];
      xprev[i] = v;
    }
  }
};

template <typename T>
__device__ __forceinline__ void ld_vec(const T* p, float (&v)[8], int n) {
  if (n == 8) {
    load8(p, v);
  } else {
    for (int i = 0; i < n; ++i) v[i] = Elem<T>::ld(p + i);
  }
}
template <typename T>
__device__ __forceinline__ void st_vec(T* p, const float (&v)[8], int n) {
  if (n == 8) {
    store8(p, v);
  } else {
    for (int i = 0; i < n; ++i) Elem<T>::st(p + i, v[i]);
  }
}

// Generic 3-in / 2-out per-sample op.  VEC = 8 when per_sample % 8 == 0.
template <typename T, typename Op, int VEC>
__global__ void sched_kernel(Op op, const T* __restrict__ a, const T* __restrict__ b,
                             const T* __restrict__ c, T* __restrict__ o0, T* __restrict__ o1,
                             const int64_t* __restrict__ t, int64_t B, int64_t per_sample) {
  const int64_t nvec = B * per_sample / VEC;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec;
       v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = v * VEC;
    const int64_t bi = e / per_sample;
    float xa[8], xb[8], xc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, y0[8], y1[8];
    ld_vec(a + e, xa, VEC);
    ld_vec(b + e, xb, VEC);
    if (c) ld_vec(c + e, xc, VEC);
    op(t[bi], xa, xb, xc, y0, y1, VEC);
    st_vec(o0 + e, y0, VEC);
    if (o1) st_vec(o1 + e, y1, VEC);
  }
}

template <typename T, int VEC>
__global__ void ddim_kernel(DDIMStep op, const T* __restrict__ xt, const T* __restrict__ eps,
                            const T* __restrict__ z, T* __restrict__ xprev, T* __restrict__ x0,
                            const int64_t* __restrict__ t, int64_t B, int64_t per_sample) {
  const int64_t nvec = B * per_sample / VEC;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec;
       v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = v * VEC;
    const int64_t bi = e / per_sample;
    float xa[8], xb[8], xc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, y0[8], y1[8];
    ld_vec(xt + e, xa, VEC);
    ld_vec(eps + e, xb, VEC);
    if (z) ld_vec(z + e, xc, VEC);
    op.run(t[bi], op.tprev[bi], xa, xb, xc, y0, y1, VEC);
    st_vec(xprev + e, y0, VEC);
    if (x0) st_vec(x0 + e, y1, VEC);
  }
}

template <typename Op>
int launch_sched(Op op, const void* a, const void* b, const void* c, void* o0, void* o1,
                 const int64_t* t, int64_t B, int64_t per_sample, int dtype, void* stream) {
  VD_REQUIRE(a && b && o0 && t, "null tensor argument");
  VD_REQUIRE(B > 0 && per_sample > 0, "empty tensor (B=%lld, per_sample=%lld)", (long long)B,
             (long long)per_sample);
  const bool v8 = per_sample % 8 == 0;
  const int64_t work = B * per_sample / (v8 ? 8 : 1);
  return VD_DISPATCH_DTYPE(dtype, T, {
    if (v8)
      sched_kernel<T, Op, 8><<<grid_for(work), kBlock, 0, VD_STREAM(stream)>>>(
          op, (const T*)a, (const T*)b, (const T*)c, (T*)o0, (T*)o1, t, B, per_sample);
    else
      sched_kernel<T, Op, 1><<<grid_for(work), kBlock, 0, VD_STREAM(stream)>>>(
          op, (const T*)a, (const T*)b, (const T*)c, (T*)o0, (T*)o1, t, B, per_sample);
  });
}

// ------------------------------------------------------------ upsample
template <typename T, int VEC>
__global__ void upsample_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t BT, int H,
                                int W, int C) {
  const int cv = C / VEC;
  const int64_t n = BT * H * W * cv;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cv) * VEC;
    int64_t p = i / cv;
    const int w = (int)(p % W);
    p /= W;
    const int h = (int)(p % H);
    const int64_t bt = p / H;
    float v[8];
    ld_vec(x + i * VEC, v, VEC);
    const int64_t W2 = 2 * W;
    const int64_t row0 = ((bt * 2 * H + 2 * h) * W2 + 2 * w) * C + c0;
    st_vec(y + row0, v, VEC);
    st_vec(y + row0 + C, v, VEC);
    st_vec(y + row0 + W2 * C, v, VEC);
    st_vec(y + row0 + W2 * C + C, v, VEC);
  }
}

template <typename T, int VEC>
__global__ void upsample_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int64_t BT,
                                    int H, int W, int C) {
  const int cv = C / VEC;
  const int64_t n = BT * H * W * cv;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cv) * VEC;
    int64_t p = i / cv;
    const int w = (int)(p % W);
    p /= W;
    const int h = (int)(p % H);
    const int64_t bt = p / H;
    const int64_t W2 = 2 * W;
    const int64_t row0 = ((bt * 2 * H + 2 * h) * W2 + 2 * w) * C + c0;
    float a[8], b[8], c[8], d[8], s[8];
    ld_vec(dy + row0, a, VEC);
    ld_vec(dy + row0 + C, b, VEC);
    ld_vec(dy + row0 + W2 * C, c, VEC);
    ld_vec(dy + row0 + W2 * C + C, d, VEC);
    for (int k = 0; k < VEC; ++k) s[k] = (a[k] + b[k]) + (c[k] + d[k]);
    st_vec(dx + i * VEC, s, VEC);
  }
}

// ------------------------------------------------------------ MSE loss (train.py:103, 130)
// Fixed-order two-launch reduction: mse_partial_kernel sums a fixed contiguous range per
// block (8 elements per lane, a lane's sum, then an LDS tree) into partial[block];
// mse_finish_kernel (one block) sums the partials in block order and scales by 1/n.  No
// semaphore, no memset, no cross-block communication inside a launch: the same bits every
// run, eager or replayed from a HIP graph (torch's one-launch multi-block
// mean -- a hipMemsetAsync'd semaphore plus a last-block combine -- returned stale values
// when replayed under HIP's graph packet capture).
constexpr int kMseBlocks = 1024;

inline int mse_blocks(int64_t n) {
  const int64_t per = (int64_t)kBlock * 8;
  const int64_t g = vd_cdiv(n, per);
  return (int)(g < kMseBlocks ? (g > 0 ? g : 1) : kMseBlocks);
}

template <typename T>
__global__ void __launch_bounds__(kBlock) mse_partial_kernel(
    const T* __restrict__ pred, const T* __restrict__ tgt, int64_t n, int64_t chunk,
    float* __restrict__ partial) {
  __shared__ float red[kBlock];
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  float s = 0.f;
  // chunk is a multiple of 8: every 8-vector lies in one block's range
  for (int64_t i = lo + (int64_t)threadIdx.x * 8; i < hi; i += (int64_t)kBlock * 8) {
    if (i + 8 <= hi) {
      float a[8], b[8];
      load8(pred + i, a);
      load8(tgt + i, b);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = a[k] - b[k];
        s = fmaf(d, d, s);
      }
    } else {
      for (int64_t j = i; j < hi; ++j) {
        const float d = Elem<T>::ld(pred + j) - Elem<T>::ld(tgt + j);
        s = fmaf(d, d, s);
      }
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
#pragma unroll
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(kBlock) mse_finish_kernel(const float* __restrict__ partial,
                                                            int nblocks, float inv_n,
                                                            float* __restrict__ out) {
  __shared__ float red[kBlock];
  float s = 0.f;
  for (int i = threadIdx.x; i < nblocks; i += kBlock) s += partial[i];
  red[threadIdx.x] = s;
  __syncthreads();
#pragma unroll
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0] * inv_n;
}

// d loss / d pred = 2 (pred - tgt) / n * g, g = the loss gradient (a device scalar)
template <typename T>
__global__ void __launch_bounds__(kBlock) mse_bwd_kernel(
    const T* __restrict__ pred, const T* __restrict__ tgt, const float* __restrict__ gout,
    float scale, int64_t n, T* __restrict__ gpred) {
  const float c = scale * *gout;
  const int64_t nv = n / 8;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv;
       v += (int64_t)gridDim.x * blockDim.x) {
    float a[8], b[8];
    load8(pred + 8 * v, a);
    load8(tgt + 8 * v, b);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = c * (a[k] - b[k]);
    store8(gpred + 8 * v, a);
  }
  for (int64_t j = nv * 8 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x)
    Elem<T>::st(gpred + j, c * (Elem<T>::ld(pred + j) - Elem<T>::ld(tgt + j)));
}

}  // namespace


// ---------------------------------------------------------------- conv glue
// Per-(sample, channel) sums of a channels-last activation: the bias gradient and the
// ResBlock emb-add (chan_add) gradient of a conv in one pass over dY (reference autograd of
// conv_nd's bias, utils.py:59-69, and of `h + emb_out` at unet.py:255-258).  Stage 1: a
// block owns a run of rows of one sample, each thread sums 8 channels over its rows in fp32,
// the block reduces through LDS and stores its partial row part[b][blk][C].  Stage 2 sums
// the partial rows per channel (deterministic; no same-address atomics, which serialise).
constexpr int kSumBlocks = 1024;  // stage-1 blocks per sample (upper bound: finish registers)
// stage-1 blocks per sample actually launched (default 256; VDIFF_CSUM_BLOCKS, <= kSumBlocks,
// for A/B runs) and the rows each stage-1 thread keeps in flight (VDIFF_CSUM_UNROLL 1 or 4;
// default 4 since round 4: the step's sums 1.10 -> 0.73 ms, e.g. 192 x 262144 36.3 -> 19.4 us
// at 5.2 TB/s, bit-identical (same add order); profiles/r04af_ab_channel_sums.txt)
static int csum_env(const char* name, int dflt, int lo, int hi) {
  const char* e = getenv(name);
  const int v = e ? atoi(e) : dflt;
  return v < lo ? lo : (v > hi ? hi : v);
}
const int g_csum_blocks = csum_env("VDIFF_CSUM_BLOCKS", 256, 1, kSumBlocks);
const int g_csum_unroll = csum_env("VDIFF_CSUM_UNROLL", 4, 1, 4);

template <typename T, int U>
__global__ __launch_bounds__(256) void channel_sums_kernel(const T* __restrict__ x, int64_t S,
                                                           int C, int cs, int64_t rows_per_blk,
                                                           float* __restrict__ part) {
  __shared__ float red[256 * 8];
  const int b = blockIdx.y;
  const int tpr = C / 8;                 // threads per row (C <= 2048)
  const int rpi = 256 / tpr;             // rows per iteration
  const int tid = threadIdx.x;
  const int lr = tid / tpr, c8 = (tid % tpr) * 8;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
  int64_t r1 = r0 + rows_per_blk;
  if (r1 > S) r1 = S;
  if (lr < rpi) {
    const T* base = x + (int64_t)b * S * cs + c8;
    int64_t r = r0 + lr;
    if constexpr (U > 1) {  // U rows' loads in flight before their adds (same add order)
      for (; r + (U - 1) * rpi < r1; r += U * rpi) {
        float v[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u) load8(base + (r + u * rpi) * cs, v[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += v[u][e];
      }
    }
    for (; r < r1; r += rpi) {
      float v[8];
      load8(base + r * cs, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[tid * 8 + e] = acc[e];
  __syncthreads();
  // thread t < C sums channel t over the rpi row lanes
  float* dst = part + ((int64_t)b * gridDim.x + blockIdx.x) * C;
  for (int c = tid; c < C; c += 256) {
    const int g = c / 8, e = c % 8;
    float sum = 0.f;
    for (int k = 0; k < rpi; ++k) sum += red[(k * tpr + g) * 8 + e];
    dst[c] = sum;
  }
}

// 32 channels per block, 32 row lanes per channel: at most 8 independent partial loads per
// lane (kSumBlocks = 1024 / 32), all in flight before the adds; fixed-order LDS reduce
__global__ __launch_bounds__(1024) void channel_sums_finish_kernel(const float* __restrict__ part,
                                                                   int nblk, int C,
                                                                   float* __restrict__ out) {
  __shared__ float red[32][33];
  const int cl = threadIdx.x & 31, kl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl, b = blockIdx.y;
  float v[kSumBlocks / 32];
#pragma unroll
  for (int i = 0; i < kSumBlocks / 32; ++i) {
    const int k = kl + 32 * i;
    v[i] = (c < C && k < nblk) ? part[((int64_t)b * nblk + k) * C + c] : 0.f;
  }
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < kSumBlocks / 32; ++i) sum += v[i];
  red[kl][cl] = sum;
  __syncthreads();
  if (kl == 0 && c < C) {
#pragma unroll
    for (int k = 1; k < 32; ++k) sum += red[k][cl];
    out[(int64_t)b * C + c] = sum;
  }
}

// fp32 torch weight [Co][Ci][taps] -> packed operand in the activation dtype, channels
// zero-padded: fwd  [Co][taps][Cip]  (transpose = 0)
//              bwd  [Cip][taps][Cop] (transpose = 1, the transposed-conv operand)
template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ w, int Co, int Ci, int taps, int Cip,
                                   int Cop, int transpose, T* __restrict__ out) {
  const int64_t total = transpose ? (int64_t)Cip * taps * Cop : (int64_t)Co * taps * Cip;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int co, ci, tap;
    if (!transpose) {
      ci = (int)(i % Cip);
      tap = (int)((i / Cip) % taps);
      co = (int)(i / ((int64_t)Cip * taps));
    } else {
      co = (int)(i % Cop);
      tap = (int)((i / Cop) % taps);
      ci = (int)(i / ((int64_t)Cop * taps));
    }
    const float v = (co < Co && ci < Ci) ? w[((int64_t)co * Ci + ci) * taps + tap] : 0.f;
    Elem<T>::st(out + i, v);
  }
}

// vd_conv_pack_weights: the step's conv operands in one launch, as LDS-tiled transposes.
// A tile is 4 output channels x 64 input channels (the [Co][taps][Ci] layout) or 8 input
// channels x 64 output channels (the transposed [Ci][taps][Co] layout), all taps: the source
// rows w[co][ci0 ..][0 .. taps) are read contiguously (fp32), transposed in LDS, and the
// destination rows of 64 channels written as 16-B vectors.  Every block derives the jobs' tile
// counts and their prefix sums itself (the descriptors live on the device) and walks the
// tiles grid-stride.  A job with more than kPackMaxTaps taps (none in the UNet) is packed
// element by element in blocks of 2048 outputs.  Round 4's element-wise form (64-bit index
// math and a job search per element, strided reads) took 0.69 ms per train step.
constexpr int kPackMaxTaps = 27;
constexpr int kPackRow = 65;  // LDS row of 64 channels + 1: consecutive taps on distinct banks
constexpr int kPackSmem = 8 * kPackMaxTaps * kPackRow * 4;  // the transposed tile, the larger

// rows (outer channels) per tile: ~100-200 source floats per row of taps, so that a tile
// carries enough work for its two barriers (1x1 jobs: 64 x 64 tiles)
__host__ __device__ constexpr int pack_rows(int taps, bool transpose) {
  return taps == 1 ? 64 : taps <= 9 ? 16 : (transpose ? 8 : 4);
}

__device__ __forceinline__ int pack_tiles(const vd_pack_desc& d) {
  if (d.taps > kPackMaxTaps) return (int)((d.transpose ? (int64_t)d.Cip * d.taps * d.Cop
                                                       : (int64_t)d.Co * d.taps * d.Cip) +
                                          2047) / 2048;
  // the row counts pack_tile<T, TAPS> uses: specialised 1 / 9 / 27 taps, else the 27-tap rows
  const bool spec = d.taps == 1 || d.taps == 9 || d.taps == 27;
  const int R = pack_rows(spec ? d.taps : kPackMaxTaps, d.transpose);
  return d.transpose ? ((d.Cip + R - 1) / R) * ((d.Cop + 63) / 64)
                     : ((d.Co + R - 1) / R) * ((d.Cip + 63) / 64);
}

// One tile: NO outer rows (co, or ci when transposed) x 64 inner channels x all taps.  The
// source of outer row o is the run w[...][inner0 ..][0 .. taps) (non-transposed: contiguous
// 64 * taps floats of w[co]; transposed: R * taps floats of w[co][ci0 ..] for each of the
// 64 co) -- both read as (row, r) pairs with 32-bit offsets; LDS image [o][tap][65].
template <typename T, int TAPS>
__device__ __forceinline__ void pack_tile(const vd_pack_desc& d, int lt, float* ptile) {
  const int tp = TAPS ? TAPS : d.taps;
  const bool tr = d.transpose;
  constexpr int RN = pack_rows(TAPS ? TAPS : kPackMaxTaps, false);
  constexpr int RT = pack_rows(TAPS ? TAPS : kPackMaxTaps, true);
  // load rows: non-transposed RN co rows of 64 * tp floats; transposed 64 co rows of RT * tp
  const int nrows = tr ? 64 : RN;
  const int per = tr ? RT * tp : 64 * tp;
  const int ninner = tr ? d.Cop : d.Cip;                 // padded inner extent of the output
  const int nib = (ninner + 63) / 64;
  const int outer0 = (lt / nib) * (tr ? RT : RN), inner0 = (lt % nib) * 64;
  const int co0 = tr ? inner0 : outer0, ci0 = tr ? outer0 : inner0;
  const int rowlen = d.Ci * tp;                          // floats per co in w
  const float* src = d.w + co0 * rowlen + ci0 * tp;      // (co0, ci0, tap 0)
  const int ci_lim = d.Ci - ci0, co_lim = d.Co - co0;
  constexpr int NL = 16;
  for (int base = 0; base < nrows * per; base += NL * kBlock) {
    float v[NL];
    int dst[NL];
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int idx = base + u * kBlock + threadIdx.x;
      const int row = idx / per, r = idx - row * per;    // row: co offset (both layouts read
      const int cil = r / tp, tap = r - cil * tp;        // w[co] rows); r: (ci offset, tap)
      const bool ok = idx < nrows * per && row < co_lim && cil < ci_lim;
      v[u] = ok ? src[row * rowlen + r] : 0.f;
      // LDS [outer][tap][inner]: non-transposed outer = co (row), inner = ci (cil);
      // transposed outer = ci (cil), inner = co (row)
      dst[u] = idx < nrows * per ? ((tr ? cil : row) * tp + tap) * kPackRow + (tr ? row : cil)
                                 : -1;
    }
#pragma unroll
    for (int u = 0; u < NL; ++u)
      if (dst[u] >= 0) ptile[dst[u]] = v[u];
  }
  __syncthreads();
  const int orows = tr ? RT : RN;                        // output rows: (outer, tap)
  const int olim = tr ? d.Cip - ci0 : d.Co - co0;
  T* out = (T*)d.out;
  for (int idx = threadIdx.x; idx < orows * tp * 8; idx += kBlock) {
    const int row = idx >> 3, c8 = (idx & 7) * 8;
    const int o = row / tp, tap = row - o * tp;
    if (o < olim && inner0 + c8 < ninner) {
      float f[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = ptile[row * kPackRow + c8 + k];
      store8(out + ((int64_t)(outer0 + o) * tp + tap) * ninner + inner0 + c8, f);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) pack_weights_kernel(
    const vd_pack_desc* __restrict__ descs, int n) {
  extern __shared__ __attribute__((aligned(16))) float ptile[];
  __shared__ int tstart[1025];
  // tstart[j + 1] = the jobs' tile counts, then an inclusive Hillis-Steele scan over them
  // (parallel: a serial walk over the descriptors costs a global-load latency per job)
  if (threadIdx.x == 0) tstart[0] = 0;
  for (int j = threadIdx.x; j < n; j += kBlock) tstart[j + 1] = pack_tiles(descs[j]);
  __syncthreads();
  for (int off = 1; off < n; off <<= 1) {
    int v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int j = threadIdx.x + k * kBlock + 1;
      v[k] = (j <= n && j - off >= 1) ? tstart[j - off] : 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int j = threadIdx.x + k * kBlock + 1;
      if (j <= n) tstart[j] += v[k];
    }
    __syncthreads();
  }
  const int ntiles = tstart[n];
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {  // the last job whose first tile <= t
      const int mid = (lo + hi + 1) >> 1;
      if (tstart[mid] <= t) lo = mid; else hi = mid - 1;
    }
    const vd_pack_desc d = descs[lo];
    const int lt = t - tstart[lo];
    const int taps = d.taps;
    T* out = (T*)d.out;
    if (taps > kPackMaxTaps) {  // element-wise fallback
      const int inner = d.transpose ? d.Cop : d.Cip;
      const int64_t size = d.transpose ? (int64_t)d.Cip * taps * d.Cop
                                       : (int64_t)d.Co * taps * d.Cip;
      for (int64_t e = (int64_t)lt * 2048 + threadIdx.x; e < size && e < (int64_t)(lt + 1) * 2048;
           e += kBlock) {
        const int64_t rest = e / inner;
        const int in = (int)(e % inner), tap = (int)(rest % taps), o = (int)(rest / taps);
        const int co = d.transpose ? in : o, ci = d.transpose ? o : in;
        Elem<T>::st(out + e, (co < d.Co && ci < d.Ci)
                                 ? d.w[((int64_t)co * d.Ci + ci) * taps + tap] : 0.f);
      }
      continue;
    }
    switch (taps) {  // compile-time divisors (a runtime integer division costs ~40 VALU)
      case 27: pack_tile<T, 27>(d, lt, ptile); break;
      case 9: pack_tile<T, 9>(d, lt, ptile); break;
      case 1: pack_tile<T, 1>(d, lt, ptile); break;
      default: pack_tile<T, 0>(d, lt, ptile); break;
    }
    __syncthreads();  // the tile buffer is reused by the next tile
  }
}

extern "C" {

size_t vd_mse_loss_workspace_size(int64_t n) {
  return (size_t)mse_blocks(n) * sizeof(float);
}

int vd_mse_loss(const void* pred, const void* target, int64_t n, int dtype, float* out,
                void* workspace, size_t workspace_bytes, void* stream) {
  VD_REQUIRE(pred && target && out && workspace, "null argument");
  VD_REQUIRE(n > 0, "empty tensor");
  VD_REQUIRE(dtype == VD_F32 || dtype == VD_BF16, "bad dtype %d", dtype);
  VD_REQUIRE((reinterpret_cast<uintptr_t>(pred) | reinterpret_cast<uintptr_t>(target)) % 16 == 0,
             "pred / target must be 16-B aligned");
  const int nb = mse_blocks(n);
  VD_REQUIRE(workspace_bytes >= (size_t)nb * sizeof(float), "workspace too small");
  const int64_t chunk = vd_cdiv(vd_cdiv(n, nb), 8) * 8;
  float* partial = static_cast<float*>(workspace);
  hipStream_t st = VD_STREAM(stream);
  if (dtype == VD_F32)
    mse_partial_kernel<float><<<nb, kBlock, 0, st>>>(static_cast<const float*>(pred),
                                                     static_cast<const float*>(target), n,
                                                     chunk, partial);
  else
    mse_partial_kernel<bf16_t><<<nb, kBlock, 0, st>>>(static_cast<const bf16_t*>(pred),
                                                      static_cast<const bf16_t*>(target), n,
                                                      chunk, partial);
  mse_finish_kernel<<<1, kBlock, 0, st>>>(partial, nb, (float)(1.0 / (double)n), out);
  return vd::check_launch("vd_mse_loss");
}

int vd_mse_loss_bwd(const void* pred, const void* target, const float* grad_loss, int64_t n,
                    int dtype, void* grad_pred, void* stream) {
  VD_REQUIRE(pred && target && grad_loss && grad_pred, "null argument");
  VD_REQUIRE(n > 0, "empty tensor");
  VD_REQUIRE(dtype == VD_F32 || dtype == VD_BF16, "bad dtype %d", dtype);
  VD_REQUIRE((reinterpret_cast<uintptr_t>(pred) | reinterpret_cast<uintptr_t>(target) |
              reinterpret_cast<uintptr_t>(grad_pred)) % 16 == 0, "buffers must be 16-B aligned");
  const float scale = (float)(2.0 / (double)n);
  hipStream_t st = VD_STREAM(stream);
  const int g = grid_for(vd_cdiv(n, 8));
  if (dtype == VD_F32)
    mse_bwd_kernel<float><<<g, kBlock, 0, st>>>(static_cast<const float*>(pred),
                                                static_cast<const float*>(target), grad_loss,
                                                scale, n, static_cast<float*>(grad_pred));
  else
    mse_bwd_kernel<bf16_t><<<g, kBlock, 0, st>>>(static_cast<const bf16_t*>(pred),
                                                 static_cast<const bf16_t*>(target), grad_loss,
                                                 scale, n, static_cast<bf16_t*>(grad_pred));
  return vd::check_launch("vd_mse_loss_bwd");
}

int vd_timestep_embedding(const int64_t* t, int B, int dim, float max_period, float* out,
                          void* stream) {
  VD_REQUIRE(t && out, "null argument");
  VD_REQUIRE(B > 0 && dim > 0, "bad shape B=%d dim=%d", B, dim);
  temb_kernel<<<grid_for((int64_t)B * dim), kBlock, 0, VD_STREAM(stream)>>>(
      t, B, dim, logf(max_period), nullptr, out);
  return vd::check_launch("vd_timestep_embedding");
}

int vd_timestep_embedding_tab(const int64_t* t, int B, int dim, const float* freqs, float* out,
                              void* stream) {
  VD_REQUIRE(t && out && (freqs || dim < 2), "null argument");
  VD_REQUIRE(B > 0 && dim > 0, "bad shape B=%d dim=%d", B, dim);
  temb_kernel<<<grid_for((int64_t)B * dim), kBlock, 0, VD_STREAM(stream)>>>(t, B, dim, 0.f,
                                                                            freqs, out);
  return vd::check_launch("vd_timestep_embedding_tab");
}

int vd_q_sample(const void* x0, const void* eps, void* xt, const int64_t* t, const float* sqrt_acp,
                const float* sqrt_1m_acp, int64_t B, int64_t per_sample, int dtype, void* stream) {
  VD_REQUIRE(sqrt_acp && sqrt_1m_acp, "null table");
  return launch_sched(QSample{sqrt_acp, sqrt_1m_acp}, x0, eps, nullptr, xt, nullptr, t, B,
                      per_sample, dtype, stream);
}

int vd_p_sample_v1(const void* xt, const void* eps, const void* z, void* x_prev, void* x0,
                   const int64_t* t, const float* betas, const float* alphas, const float* acp,
                   const float* sqrt_1m_acp, int64_t B, int64_t per_sample, int dtype,
                   void* stream) {
  VD_REQUIRE(betas && alphas && acp && sqrt_1m_acp, "null table");
  VD_REQUIRE(z && x0, "p_sample_v1 needs z and x0 buffers");
  return launch_sched(PSampleV1{betas, alphas, acp, sqrt_1m_acp}, xt, eps, z, x_prev, x0, t, B,
                      per_sample, dtype, stream);
}

int vd_p_sample_v2(const void* xt, const void* eps, const void* z, void* x_prev, void* x0,
                   const int64_t* t, const float* betas, const float* alphas, const float* acp,
                   const float* sqrt_acp, const float* sqrt_1m_acp, int64_t B,
                   int64_t per_sample, int dtype, void* stream) {
  VD_REQUIRE(betas && alphas && acp && sqrt_acp && sqrt_1m_acp, "null table");
  VD_REQUIRE(z && x0, "p_sample_v2 needs z and x0 buffers");
  return launch_sched(PSampleV2{betas, alphas, acp, sqrt_acp, sqrt_1m_acp}, xt, eps, z, x_prev,
                      x0, t, B, per_sample, dtype, stream);
}

int vd_p_sample_cosine(const void* xt, const void* eps, const void* z, void* x_prev,
                       void* mean_out, const int64_t* t, const float* acp, const float* sqrt_acp,
                       const float* sqrt_1m_acp, int64_t B, int64_t per_sample, int dtype,
                       void* stream) {
  VD_REQUIRE(acp && sqrt_acp && sqrt_1m_acp, "null table");
  VD_REQUIRE(z && mean_out, "p_sample_cosine needs z and mean buffers");
  return launch_sched(PSampleCos{acp, sqrt_acp, sqrt_1m_acp}, xt, eps, z, x_prev, mean_out, t, B,
                      per_sample, dtype, stream);
}

int vd_ddim_step(const void* xt, const void* eps, const void* z, void* x_prev, void* x0,
                 const int64_t* t, const int64_t* t_prev, const float* acp, float eta, int clip,
                 int64_t B, int64_t per_sample, int dtype, void* stream) {
  VD_REQUIRE(xt && eps && x_prev && t && t_prev && acp, "null argument");
  VD_REQUIRE(B > 0 && per_sample > 0, "empty tensor");
  VD_REQUIRE(eta == 0.f || z, "eta > 0 needs z");
  DDIMStep op{acp, t_prev, eta, clip, z != nullptr};
  const bool v8 = per_sample % 8 == 0;
  const int64_t work = B * per_sample / (v8 ? 8 : 1);
  return VD_DISPATCH_DTYPE(dtype, T, {
    if (v8)
      ddim_kernel<T, 8><<<grid_for(work), kBlock, 0, VD_STREAM(stream)>>>(
          op, (const T*)xt, (const T*)eps, (const T*)z, (T*)x_prev, (T*)x0, t, B, per_sample);
    else
      ddim_kernel<T, 1><<<grid_for(work), kBlock, 0, VD_STREAM(stream)>>>(
          op, (const T*)xt, (const T*)eps, (const T*)z, (T*)x_prev, (T*)x0, t, B, per_sample);
  });
}

int vd_upsample_nearest_hw(const void* x, void* y, int B, int T, int H, int W, int C, int dtype,
                           void* stream) {
  VD_REQUIRE(x && y, "null argument");
  VD_REQUIRE(B > 0 && T > 0 && H > 0 && W > 0 && C > 0, "bad shape");
  const int64_t BT = (int64_t)B * T;
  const bool v8 = C % 8 == 0;
  const int64_t work = BT * H * W * (v8 ? C / 8 : C);
  return VD_DISPATCH_DTYPE(dtype, Tp, {
    if (v8)
      upsample_kernel<Tp, 8><<<grid_for(work), kBlock, 0, VD_STREAM(stream)>>>(
          (const Tp*)x, (Tp*)y, BT, H, W, C);
    else
      upsample_kernel<Tp, 1><<<grid_for(work), kBlock, 0, VD_STREAM(stream)>>>(
          (const Tp*)x, (Tp*)y, BT, H, W, C);
  });
}

int vd_upsample_nearest_hw_bwd(const void* dy, void* dx, int B, int T, int H, int W, int C,
                               int dtype, void* stream) {
  VD_REQUIRE(dy && dx, "null argument");
  VD_REQUIRE(B > 0 && T > 0 && H > 0 && W > 0 && C > 0, "bad shape");
  const int64_t BT = (int64_t)B * T;
  const bool v8 = C % 8 == 0;
  const int64_t work = BT * H * W * (v8 ? C / 8 : C);
  return VD_DISPATCH_DTYPE(dtype, Tp, {
    if (v8)
      upsample_bwd_kernel<Tp, 8><<<grid_for(work), kBlock, 0, VD_STREAM(stream)>>>(
          (const Tp*)dy, (Tp*)dx, BT, H, W, C);
    else
      upsample_bwd_kernel<Tp, 1><<<grid_for(work), kBlock, 0, VD_STREAM(stream)>>>(
          (const Tp*)dy, (Tp*)dx, BT, H, W, C);
  });
}

size_t vd_channel_sums_workspace_size(int B, int C) {
  if (B <= 0 || C <= 0) return 0;
  return (size_t)B * kSumBlocks * C * sizeof(float);
}

int vd_channel_sums(const void* x, int B, int64_t S, int C, int cstride, int dtype, float* out,
                    void* workspace, void* stream) {
  VD_REQUIRE(x && out && workspace, "null argument");
  VD_REQUIRE(B > 0 && S > 0 && C > 0 && C % 8 == 0 && C <= 2048, "bad shape B=%d C=%d", B, C);
  const int cs = cstride ? cstride : C;
  VD_REQUIRE(cs >= C && cs % 8 == 0, "bad channel stride %d", cs);
  hipStream_t st = VD_STREAM(stream);
  // about kSumBlocks blocks per sample, at least 4 row iterations each
  const int64_t rpi = 256 / (C / 8);
  int64_t blocks = g_csum_blocks;
  int64_t maxb = vd_cdiv(S, rpi * 4);
  if (blocks > maxb) blocks = maxb;
  if (blocks < 1) blocks = 1;
  const int64_t rows = vd_cdiv(S, blocks);
  blocks = vd_cdiv(S, rows);
  float* part = reinterpret_cast<float*>(workspace);
  return VD_DISPATCH_DTYPE(dtype, Tp, {
    if (g_csum_unroll >= 4)
      channel_sums_kernel<Tp, 4><<<dim3((unsigned)blocks, (unsigned)B), 256, 0, st>>>(
          (const Tp*)x, S, C, cs, rows, part);
    else
      channel_sums_kernel<Tp, 1><<<dim3((unsigned)blocks, (unsigned)B), 256, 0, st>>>(
          (const Tp*)x, S, C, cs, rows, part);
    channel_sums_finish_kernel<<<dim3((unsigned)vd_cdiv(C, 32), (unsigned)B), 1024, 0, st>>>(
        part, (int)blocks, C, out);
  });
}

int vd_conv_pack_weights(const vd_pack_desc* descs, int n, int64_t total, int dtype,
                         void* stream) {
  VD_REQUIRE(descs && n > 0 && n <= 1024 && total > 0, "bad pack job list");
  return VD_DISPATCH_DTYPE(dtype, Tp, {
    (void)total;
    pack_weights_kernel<Tp><<<2048, kBlock, kPackSmem, VD_STREAM(stream)>>>(descs, n);
  });
}

int vd_conv_pack_weight(const float* w, int Co, int Ci, int taps, int Cip, int Cop, int transpose,
                        int dtype, void* out, void* stream) {
  VD_REQUIRE(w && out, "null argument");
  VD_REQUIRE(Co > 0 && Ci > 0 && taps > 0 && Cip >= Ci && Cop >= Co, "bad weight shape");
  const int64_t total = transpose ? (int64_t)Cip * taps * Cop : (int64_t)Co * taps * Cip;
  return VD_DISPATCH_DTYPE(dtype, Tp, {
    pack_weight_kernel<Tp><<<grid_for(total), kBlock, 0, VD_STREAM(stream)>>>(
        w, Co, Ci, taps, Cip, Cop, transpose, (Tp*)out);
  });
}

}  // extern "C"
