// groupnorm.hip -- fused GroupNorm(32) + SiLU, forward and backward, on
// channels-last activations [B][S][C] (S = T*H*W).
//
// Replaces GroupNorm32 (reference utils.py:54-56: fp32 statistics, eps 1e-5,
// affine) + nn.SiLU (unet.py:194-198, 218-225, 624-628) and the bare GN of
// AttentionBlock (unet.py:297, silu = 0).
//
// HBM traffic (the bound): fwd = 2 reads + 1 write of x; bwd = 2 reads of x
// and dy + 1 write of dx.  Statistics are fp32 and combined with Chan's
// parallel formula (per-thread shifted sums -> per-chunk -> per-sample), so
// the variance does not cancel when |mean| >> std.
#include <atomic>

#include "vd_common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kVec = 8;             // channels per lane
// workgroups per launch (B * nchunk) and chunk partials per gn_bwd_sum_kernel workgroup;
// VDIFF_GN_CHUNKS / VDIFF_GN_SUMPER override them for A/B runs (read once per process).
// 1024 (round 4; 2048 before): the forward 7-10 us faster on 8 of the step's 9 shapes (half
// the chunk partials for the finalize pass), the backward 2-6 us on 7 of 9, +4 us on C = 192
// at 16x128x128 (tools/gn_bench.py --capi, profiles/r04ad_ab_gn_chunks.txt)
static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  const int v = e ? atoi(e) : 0;
  return v > 0 ? v : dflt;
}
const int kTargetChunks = env_int("VDIFF_GN_CHUNKS", 1024);
const int kSumPer = env_int("VDIFF_GN_SUMPER", 64);
// The kernels take U, the pixel rows whose loads each thread keeps in flight (same summation
// order for every U).  Round 6 re-measured them interleaved in one process (vd_groupnorm_set_unroll,
// tools/gn_bench.py --capi --unroll, profiles/r06z5_gn_unroll.txt): over the step's 9 shapes
// U = 2 fwd 309 / bwd 470 us, U = 1 311 / 484, U = 4 313 / 505 -- U = 2 is the default
// (VDIFF_GN_UNROLL at load; round 4 had found U = 2 / 4 equal or slower with 2048 chunks).
std::atomic<int> g_gn_unroll{env_int("VDIFF_GN_UNROLL", 2)};

struct GNPlan {
  int rows_per_iter;  // pixel rows a WG covers per iteration
  int64_t chunk_px;   // pixels per WG
  int nchunk;         // chunks per sample
};

inline GNPlan gn_plan(int B, int64_t S, int C) {
  GNPlan p;
  const int nvec = C / kVec;
  p.rows_per_iter = kThreads / nvec;
  if (p.rows_per_iter < 1) p.rows_per_iter = 1;
  int64_t want = vd_cdiv(S * B, kTargetChunks);
  if (want < p.rows_per_iter) want = p.rows_per_iter;
  want = vd_cdiv(want, p.rows_per_iter) * p.rows_per_iter;
  p.chunk_px = want;
  p.nchunk = (int)vd_cdiv(S, want);
  return p;
}

struct Stat {  // count, mean, M2
  float n, m, q;
};
__device__ __forceinline__ Stat chan(Stat a, Stat b) {
  const float n = a.n + b.n;
  if (n == 0.f) return a;
  const float d = b.m - a.m;
  const float fb = b.n / n;
  Stat r;
  r.n = n;
  r.m = a.m + d * fb;
  r.q = a.q + b.q + d * d * a.n * fb;
  return r;
}

// train-mode dropout after the SiLU (ResBlock.out_layers, unet.py:221)
// `ctr` (optional, device memory): a step counter mixed into the seed when the kernel runs,
// so a replayed HIP graph -- whose launch arguments, host seed included, are frozen at capture
// -- draws a fresh mask each step (vd_set_dropout_counter).  Kernels call resolved() once.
struct Drop {
  float p, inv_keep;
  uint64_t seed;
  const uint64_t* ctr;
  __device__ __forceinline__ Drop resolved() const {
    Drop d = *this;
    if (p > 0.f && ctr) d.seed = seed ^ ((*ctr + 1) * 0x9E3779B97F4A7C15ull);
    d.ctr = nullptr;
    return d;
  }
  __device__ __forceinline__ float mul(int64_t idx) const {
    return p > 0.f ? dropout_mul(seed, idx, p, inv_keep) : 1.f;
  }
};

static const uint64_t* g_drop_ctr = nullptr;  // vd_set_dropout_counter

// ---------------------------------------------------------------- forward
// grid (nchunk, B).  Per WG: per-group (n, mean, M2) over its chunk.
template <typename T, int U>
__global__ __launch_bounds__(kThreads) void gn_stats_kernel(const T* __restrict__ x, int64_t S,
                                                            int C, int G, int64_t chunk_px,
                                                            int rows_per_iter,
                                                            float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Stat* sh = reinterpret_cast<Stat*>(smem);  // [rows_per_iter][C]
  const int nvec = C / kVec;
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  const int r = tid / nvec, cv = tid % nvec;
  const int64_t p0 = (int64_t)blockIdx.x * chunk_px;
  int64_t p1 = p0 + chunk_px;
  if (p1 > S) p1 = S;
  const T* xb = x + (int64_t)b * S * C;
  const bool active = r < rows_per_iter;
  float shift[kVec], s1[kVec], s2[kVec];
  float cnt = 0.f;
#pragma unroll
  for (int j = 0; j < kVec; ++j) s1[j] = s2[j] = shift[j] = 0.f;
  if (active && p0 + r < p1) load8(xb + (p0 + r) * C + cv * kVec, shift);
  if (active) {
    int64_t p = p0 + r;
    if constexpr (U > 1) {
      for (; p + (U - 1) * rows_per_iter < p1; p += U * rows_per_iter) {
        float v[U][kVec];
#pragma unroll
        for (int u = 0; u < U; ++u) load8(xb + (p + u * rows_per_iter) * C + cv * kVec, v[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int j = 0; j < kVec; ++j) {
            const float d = v[u][j] - shift[j];
            s1[j] += d;
            s2[j] += d * d;
          }
          cnt += 1.f;
        }
      }
    }
    for (; p < p1; p += rows_per_iter) {
      float v[kVec];
      load8(xb + p * C + cv * kVec, v);
#pragma unroll
      for (int j = 0; j < kVec; ++j) {
        const float d = v[j] - shift[j];
        s1[j] += d;
        s2[j] += d * d;
      }
      cnt += 1.f;
    }
#pragma unroll
    for (int j = 0; j < kVec; ++j) {
      Stat s;
      s.n = cnt;
      s.m = cnt > 0.f ? shift[j] + s1[j] / cnt : 0.f;
      s.q = cnt > 0.f ? fmaxf(s2[j] - s1[j] * s1[j] / cnt, 0.f) : 0.f;
      sh[r * C + cv * kVec + j] = s;
    }
  }
  __syncthreads();
  // one thread per channel: combine rows
  for (int c = tid; c < C; c += kThreads) {
    Stat a = sh[c];
    for (int rr = 1; rr < rows_per_iter; ++rr) a = chan(a, sh[rr * C + c]);
    sh[c] = a;
  }
  __syncthreads();
  const int cpg = C / G;
  for (int g = tid; g < G; g += kThreads) {
    Stat a = sh[g * cpg];
    for (int k = 1; k < cpg; ++k) a = chan(a, sh[g * cpg + k]);
    float* o = part + (((int64_t)b * gridDim.x + blockIdx.x) * G + g) * 3;
    o[0] = a.n;
    o[1] = a.m;
    o[2] = a.q;
  }
}

// grid (G, B), 256 threads: combine the nchunk partials of one (b, g) -> mean, rstd
// (strided per-thread Chan combine, then a shuffle / LDS tree)
__device__ __forceinline__ Stat chan_shfl(Stat a, int off) {
  Stat o{__shfl_xor(a.n, off, 64), __shfl_xor(a.m, off, 64), __shfl_xor(a.q, off, 64)};
  return chan(a, o);
}
__global__ __launch_bounds__(kThreads) void gn_finalize_kernel(const float* __restrict__ part,
                                                               int nchunk, int G, float eps,
                                                               float* __restrict__ mean,
                                                               float* __restrict__ rstd) {
  __shared__ Stat sh[kThreads / 64];
  const int g = blockIdx.x, b = blockIdx.y;
  Stat a{0.f, 0.f, 0.f};
  // the first four strided partials' loads all in flight before the (same-order) combines
  // (round 6: the loop waited a memory latency per partial; nchunk <= 1024 = 4 x 256)
  constexpr int PRE = 4;
  Stat v[PRE];
#pragma unroll
  for (int u = 0; u < PRE; ++u) {
    const int k = threadIdx.x + u * kThreads;
    v[u] = Stat{0.f, 0.f, 0.f};
    if (k < nchunk) {
      const float* p = part + (((int64_t)b * nchunk + k) * G + g) * 3;
      v[u] = Stat{p[0], p[1], p[2]};
    }
  }
#pragma unroll
  for (int u = 0; u < PRE; ++u)
    if (threadIdx.x + u * kThreads < nchunk) a = chan(a, v[u]);
  for (int k = threadIdx.x + PRE * kThreads; k < nchunk; k += kThreads) {
    const float* p = part + (((int64_t)b * nchunk + k) * G + g) * 3;
    a = chan(a, Stat{p[0], p[1], p[2]});
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) a = chan_shfl(a, off);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    Stat t = sh[0];
    for (int k = 1; k < kThreads / 64; ++k) t = chan(t, sh[k]);
    const float var = t.n > 0.f ? t.q / t.n : 0.f;  // biased, as torch GroupNorm
    mean[b * G + g] = t.m;
    rstd[b * G + g] = rsqrtf(var + eps);
  }
}

// grid (nchunk, B): each thread keeps one 8-channel vector for all its pixel rows, so the
// per-channel scale/shift (gamma * rstd, beta - mean * gamma * rstd) is computed once and
// the loop is one FMA (+ SiLU, dropout) per element -- no index division per element.
template <typename T, bool SILU, int U>
__global__ __launch_bounds__(kThreads) void gn_apply_kernel(const T* __restrict__ x,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            T* __restrict__ y, int64_t S, int C,
                                                            int G, int64_t chunk_px,
                                                            int rows_per_iter, Drop drop_in) {
  const Drop drop = drop_in.resolved();
  const int nvec = C / kVec, cpg = C / G;
  const int b = blockIdx.y, tid = threadIdx.x;
  const int r = tid / nvec, cv = tid % nvec;
  if (r >= rows_per_iter) return;
  float sc[kVec], sh[kVec];
#pragma unroll
  for (int j = 0; j < kVec; ++j) {
    const int c = cv * kVec + j, g = b * G + c / cpg;
    sc[j] = gamma[c] * rstd[g];
    sh[j] = beta[c] - mean[g] * sc[j];
  }
  const int64_t p0 = (int64_t)blockIdx.x * chunk_px;
  int64_t p1 = p0 + chunk_px;
  if (p1 > S) p1 = S;
  int64_t p = p0 + r;
  if constexpr (U > 1) {
    for (; p + (U - 1) * rows_per_iter < p1; p += U * rows_per_iter) {
      float v[U][kVec];
#pragma unroll
      for (int u = 0; u < U; ++u)
        load8(x + ((int64_t)b * S + p + u * rows_per_iter) * C + cv * kVec, v[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t e0 = ((int64_t)b * S + p + u * rows_per_iter) * C + cv * kVec;
#pragma unroll
        for (int j = 0; j < kVec; ++j) {
          const float z = v[u][j] * sc[j] + sh[j];
          v[u][j] = (SILU ? silu_f(z) : z) * drop.mul(e0 + j);
        }
        store8(y + e0, v[u]);
      }
    }
  }
  for (; p < p1; p += rows_per_iter) {
    const int64_t e0 = ((int64_t)b * S + p) * C + cv * kVec;
    float v[kVec];
    load8(x + e0, v);
#pragma unroll
    for (int j = 0; j < kVec; ++j) {
      const float z = v[j] * sc[j] + sh[j];
      v[j] = (SILU ? silu_f(z) : z) * drop.mul(e0 + j);
    }
    store8(y + e0, v);
  }
}

// ---------------------------------------------------------------- backward
// grid (nchunk, B): per-channel partial sums A = sum dz, Bs = sum dz * xhat
template <typename T, bool SILU, int U>
__global__ __launch_bounds__(kThreads) void gn_bwd_reduce_kernel(
    const T* __restrict__ x, const T* __restrict__ dy, const float* __restrict__ gamma,
    const float* __restrict__ beta, const float* __restrict__ mean, const float* __restrict__ rstd,
    int64_t S, int C, int G, int64_t chunk_px, int rows_per_iter, float* __restrict__ part,
    Drop drop_in) {
  const Drop drop = drop_in.resolved();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* sh = reinterpret_cast<float2*>(smem);  // [rows_per_iter][C]
  const int nvec = C / kVec;
  const int cpg = C / G;
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  const int r = tid / nvec, cv = tid % nvec;
  const int64_t p0 = (int64_t)blockIdx.x * chunk_px;
  int64_t p1 = p0 + chunk_px;
  if (p1 > S) p1 = S;
  const T* xb = x + (int64_t)b * S * C;
  const T* db = dy + (int64_t)b * S * C;
  float mu[kVec], rs[kVec], ga[kVec], be[kVec], sa[kVec], sb[kVec];
  if (r < rows_per_iter) {
#pragma unroll
    for (int j = 0; j < kVec; ++j) {
      const int c = cv * kVec + j;
      mu[j] = mean[b * G + c / cpg];
      rs[j] = rstd[b * G + c / cpg];
      ga[j] = gamma[c];
      be[j] = beta[c];
      sa[j] = sb[j] = 0.f;
    }
    auto row = [&](int64_t p, const float* v, const float* d) {
#pragma unroll
      for (int j = 0; j < kVec; ++j) {
        const float xh = (v[j] - mu[j]) * rs[j];
        float dz = d[j] * drop.mul(((int64_t)b * S + p) * C + cv * kVec + j);
        if (SILU) {
          const float z = xh * ga[j] + be[j];
          const float sg = 1.f / (1.f + __expf(-z));
          dz *= sg * (1.f + z * (1.f - sg));
        }
        sa[j] += dz;
        sb[j] += dz * xh;
      }
    };
    int64_t p = p0 + r;
    if constexpr (U > 1) {
      for (; p + (U - 1) * rows_per_iter < p1; p += U * rows_per_iter) {
        float v[U][kVec], d[U][kVec];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          load8(xb + (p + u * rows_per_iter) * C + cv * kVec, v[u]);
          load8(db + (p + u * rows_per_iter) * C + cv * kVec, d[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) row(p + u * rows_per_iter, v[u], d[u]);
      }
    }
    for (; p < p1; p += rows_per_iter) {
      float v[kVec], d[kVec];
      load8(xb + p * C + cv * kVec, v);
      load8(db + p * C + cv * kVec, d);
      row(p, v, d);
    }
#pragma unroll
    for (int j = 0; j < kVec; ++j) sh[r * C + cv * kVec + j] = make_float2(sa[j], sb[j]);
  }
  __syncthreads();
  for (int c = tid; c < C; c += kThreads) {
    float2 a = sh[c];
    for (int rr = 1; rr < rows_per_iter; ++rr) {
      a.x += sh[rr * C + c].x;
      a.y += sh[rr * C + c].y;
    }
    float* o = part + (((int64_t)b * gridDim.x + blockIdx.x) * C + c) * 2;
    o[0] = a.x;
    o[1] = a.y;
  }
}

// grid (ceil(C/64), B, ksplit), 1024 threads = 64 channels x 16 chunk lanes: per-(b, c) sums
// of the chunk partials (coalesced 512-B rows, 16-way parallel over chunks).  Workgroup z sums
// chunks [z * kper, (z + 1) * kper) in a fixed order and WRITES sums[z][b][c][2]; the finalize
// kernel adds the ksplit slices in order.  No atomics: the backward is bit-reproducible
// (the same-address float atomics of round 3 summed in arrival order).
__global__ __launch_bounds__(1024) void gn_bwd_sum_kernel(const float* __restrict__ part,
                                                          int nchunk, int C, int kper,
                                                          float* __restrict__ sums) {
  __shared__ float2 sh[16][64];
  const int cl = threadIdx.x & 63, kl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, b = blockIdx.y;
  const int k0 = blockIdx.z * kper;
  int k1 = k0 + kper;
  if (k1 > nchunk) k1 = nchunk;
  float2 a = make_float2(0.f, 0.f);
  if (c < C) {
    int k = k0 + kl;
    // four chunk rows' loads in flight per iteration, added in the same order (round 6)
    for (; k + 48 < k1; k += 64) {
      float2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = *reinterpret_cast<const float2*>(
            part + (((int64_t)b * nchunk + k + 16 * u) * C + c) * 2);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a.x += v[u].x;
        a.y += v[u].y;
      }
    }
    for (; k < k1; k += 16) {
      const float2 v = *reinterpret_cast<const float2*>(part + (((int64_t)b * nchunk + k) * C + c) * 2);
      a.x += v.x;
      a.y += v.y;
    }
  }
  sh[kl][cl] = a;
  __syncthreads();
  if (kl == 0 && c < C) {
    for (int k = 1; k < 16; ++k) {
      a.x += sh[k][cl].x;
      a.y += sh[k][cl].y;
    }
    float* o = sums + (((int64_t)blockIdx.z * gridDim.y + b) * C + c) * 2;
    o[0] = a.x;
    o[1] = a.y;
  }
}

// one WG: the ksplit slices of sums[z][b][c][2] added in order into slice 0, then group
// coefficients per (b, g) and dgamma/dbeta per channel
__global__ void gn_bwd_finalize_kernel(float* __restrict__ sums, int ksplit, int B, int C, int G,
                                       int64_t S, const float* __restrict__ gamma,
                                       float* __restrict__ coef, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta) {
  const int64_t slice = (int64_t)B * C * 2;
  for (int i = threadIdx.x; i < B * C; i += blockDim.x) {
    float a = sums[2 * i], s = sums[2 * i + 1];
#pragma unroll 8
    for (int z = 1; z < ksplit; ++z) {
      a += sums[z * slice + 2 * i];
      s += sums[z * slice + 2 * i + 1];
    }
    sums[2 * i] = a;
    sums[2 * i + 1] = s;
  }
  __syncthreads();
  const int cpg = C / G;
  const float inv_n = 1.f / ((float)cpg * (float)S);
  for (int bg = threadIdx.x; bg < B * G; bg += blockDim.x) {
    const int b = bg / G, g = bg % G;
    float a = 0.f, s = 0.f;
    for (int k = 0; k < cpg; ++k) {
      const int c = g * cpg + k;
      a += gamma[c] * sums[((int64_t)b * C + c) * 2];
      s += gamma[c] * sums[((int64_t)b * C + c) * 2 + 1];
    }
    coef[bg * 2 + 0] = a * inv_n;
    coef[bg * 2 + 1] = s * inv_n;
  }
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f, s = 0.f;
    for (int b = 0; b < B; ++b) {
      a += sums[((int64_t)b * C + c) * 2];
      s += sums[((int64_t)b * C + c) * 2 + 1];
    }
    dbeta[c] = a;
    dgamma[c] = s;
  }
}

// grid (nchunk, B), per-thread channel constants as gn_apply_kernel
template <typename T, bool SILU, int U>
__global__ __launch_bounds__(kThreads) void gn_bwd_apply_kernel(
    const T* __restrict__ x, const T* __restrict__ dy, const float* __restrict__ gamma,
    const float* __restrict__ beta, const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ coef, const T* __restrict__ dadd, T* __restrict__ dx, int64_t S,
    int C, int G, int64_t chunk_px, int rows_per_iter, Drop drop_in) {
  const Drop drop = drop_in.resolved();
  const int nvec = C / kVec, cpg = C / G;
  const int b = blockIdx.y, tid = threadIdx.x;
  const int r = tid / nvec, cv = tid % nvec;
  if (r >= rows_per_iter) return;
  float mu[kVec], rs[kVec], ga[kVec], be[kVec], c0[kVec], c1[kVec];
#pragma unroll
  for (int j = 0; j < kVec; ++j) {
    const int c = cv * kVec + j, g = b * G + c / cpg;
    mu[j] = mean[g];
    rs[j] = rstd[g];
    ga[j] = gamma[c];
    be[j] = beta[c];
    c0[j] = coef[2 * g];
    c1[j] = coef[2 * g + 1];
  }
  const int64_t p0 = (int64_t)blockIdx.x * chunk_px;
  int64_t p1 = p0 + chunk_px;
  if (p1 > S) p1 = S;
  auto row = [&](int64_t e0, float (&v)[kVec], const float (&d)[kVec]) {
#pragma unroll
    for (int j = 0; j < kVec; ++j) {
      const float xh = (v[j] - mu[j]) * rs[j];
      float dz = d[j] * drop.mul(e0 + j);
      if (SILU) {
        const float z = xh * ga[j] + be[j];
        const float sg = 1.f / (1.f + __expf(-z));
        dz *= sg * (1.f + z * (1.f - sg));
      }
      v[j] = rs[j] * (ga[j] * dz - c0[j] - xh * c1[j]);
    }
    if (dadd) {  // the input's other gradient (a residual branch), added before the one rounding
      float a[kVec];
      load8(dadd + e0, a);
#pragma unroll
      for (int j = 0; j < kVec; ++j) v[j] += a[j];
    }
    store8(dx + e0, v);
  };
  int64_t p = p0 + r;
  if constexpr (U > 1) {
    for (; p + (U - 1) * rows_per_iter < p1; p += U * rows_per_iter) {
      float v[U][kVec], d[U][kVec];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t e0 = ((int64_t)b * S + p + u * rows_per_iter) * C + cv * kVec;
        load8(x + e0, v[u]);
        load8(dy + e0, d[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        row(((int64_t)b * S + p + u * rows_per_iter) * C + cv * kVec, v[u], d[u]);
    }
  }
  for (; p < p1; p += rows_per_iter) {
    const int64_t e0 = ((int64_t)b * S + p) * C + cv * kVec;
    float v[kVec], d[kVec];
    load8(x + e0, v);
    load8(dy + e0, d);
    row(e0, v, d);
  }
}


int gn_check(const void* x, int B, int64_t S, int C, int G) {
  VD_REQUIRE(x, "null tensor");
  VD_REQUIRE(B > 0 && S > 0 && C > 0 && G > 0, "bad shape B=%d S=%lld C=%d G=%d", B,
             (long long)S, C, G);
  VD_REQUIRE(C % G == 0, "C=%d not divisible by groups=%d", C, G);
  VD_REQUIRE(C % kVec == 0, "C=%d must be a multiple of %d", C, kVec);
  VD_REQUIRE(C / kVec <= kThreads, "C=%d too large", C);
  VD_REQUIRE(G <= kThreads, "G=%d too large", G);
  VD_REQUIRE(C <= 4 * kThreads, "C=%d too large for bwd finalize", C);
  return VD_OK;
}

}  // namespace

extern "C" {

size_t vd_groupnorm_workspace_size(int B, int64_t S, int C, int G) {
  if (B <= 0 || S <= 0 || C <= 0 || G <= 0 || C % kVec) return 0;
  GNPlan p = gn_plan(B, S, C);
  size_t fwd = (size_t)B * p.nchunk * G * 3 * sizeof(float);
  const size_t ksplit = vd_cdiv(p.nchunk, kSumPer);
  size_t bwd = ((size_t)B * p.nchunk * C * 2 + (size_t)B * G * 2 + ksplit * B * C * 2) *
               sizeof(float);
  return (fwd > bwd ? fwd : bwd) + 256;
}

void vd_set_dropout_counter(const uint64_t* counter) { g_drop_ctr = counter; }

int vd_groupnorm_set_unroll(int u) {
  if (u != 1 && u != 2 && u != 4) {
    (void)vd::fail(VD_EINVAL, "groupnorm unroll %d (1, 2, 4)", u);
    return -2;
  }
  return g_gn_unroll.exchange(u);
}

int vd_groupnorm_silu_fwd(const void* x, const float* gamma, const float* beta, void* y,
                          float* mean, float* rstd, int B, int64_t S, int C, int G, float eps,
                          int silu, float drop_p, uint64_t seed, int dtype, void* workspace,
                          void* stream) {
  int rc = gn_check(x, B, S, C, G);
  if (rc) return rc;
  VD_REQUIRE(gamma && beta && y && mean && rstd && workspace, "null argument");
  VD_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "dropout p=%f out of [0, 1)", drop_p);
  VD_REQUIRE(drop_p == 0.f || silu, "dropout is fused only after SiLU");
  const Drop drop{drop_p, drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f, seed, g_drop_ctr};
  GNPlan p = gn_plan(B, S, C);
  float* part = reinterpret_cast<float*>(workspace);
  hipStream_t st = VD_STREAM(stream);
  const size_t lds = (size_t)p.rows_per_iter * C * sizeof(Stat);
  const dim3 grid(p.nchunk, B);
#define VD_GN_FWD(U)                                                                             \
  gn_stats_kernel<T, U><<<grid, kThreads, lds, st>>>((const T*)x, S, C, G, p.chunk_px,          \
                                                     p.rows_per_iter, part);                    \
  gn_finalize_kernel<<<dim3(G, B), kThreads, 0, st>>>(part, p.nchunk, G, eps, mean, rstd);     \
  if (silu)                                                                                      \
    gn_apply_kernel<T, true, U><<<grid, kThreads, 0, st>>>((const T*)x, gamma, beta, mean,      \
                                                           rstd, (T*)y, S, C, G, p.chunk_px,    \
                                                           p.rows_per_iter, drop);              \
  else                                                                                           \
    gn_apply_kernel<T, false, U><<<grid, kThreads, 0, st>>>((const T*)x, gamma, beta, mean,     \
                                                            rstd, (T*)y, S, C, G, p.chunk_px,   \
                                                            p.rows_per_iter, drop)
  const int u = g_gn_unroll.load(std::memory_order_relaxed);
  return VD_DISPATCH_DTYPE(dtype, T, {
    if (u == 4) {
      VD_GN_FWD(4);
    } else if (u == 2) {
      VD_GN_FWD(2);
    } else {
      VD_GN_FWD(1);
    }
  });
#undef VD_GN_FWD
}

int vd_groupnorm_silu_bwd(const void* x, const void* dy, const float* gamma, const float* beta,
                          const float* mean, const float* rstd, void* dx, float* dgamma,
                          float* dbeta, int B, int64_t S, int C, int G, int silu, float drop_p,
                          uint64_t seed, int dtype, void* workspace, void* stream) {
  return vd_groupnorm_silu_bwd_add(x, dy, nullptr, gamma, beta, mean, rstd, dx, dgamma, dbeta, B,
                                   S, C, G, silu, drop_p, seed, dtype, workspace, stream);
}

int vd_groupnorm_silu_bwd_add(const void* x, const void* dy, const void* dadd, const float* gamma,
                              const float* beta, const float* mean, const float* rstd, void* dx,
                              float* dgamma, float* dbeta, int B, int64_t S, int C, int G,
                              int silu, float drop_p, uint64_t seed, int dtype, void* workspace,
                              void* stream) {
  int rc = gn_check(x, B, S, C, G);
  if (rc) return rc;
  VD_REQUIRE(dy && gamma && beta && mean && rstd && dx && dgamma && dbeta && workspace,
             "null argument");
  VD_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "dropout p=%f out of [0, 1)", drop_p);
  const Drop drop{drop_p, drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f, seed, g_drop_ctr};
  GNPlan p = gn_plan(B, S, C);
  float* part = reinterpret_cast<float*>(workspace);
  float* coef = part + (size_t)B * p.nchunk * C * 2;
  float* sums = coef + (size_t)B * G * 2;
  hipStream_t st = VD_STREAM(stream);
  const size_t lds = (size_t)p.rows_per_iter * C * sizeof(float2);
  const dim3 grid(p.nchunk, B);
  const int ksplit = (int)vd_cdiv(p.nchunk, kSumPer);
#define VD_GN_BWD(U)                                                                             \
  if (silu)                                                                                      \
    gn_bwd_reduce_kernel<T, true, U><<<grid, kThreads, lds, st>>>(                               \
        (const T*)x, (const T*)dy, gamma, beta, mean, rstd, S, C, G, p.chunk_px,                 \
        p.rows_per_iter, part, drop);                                                            \
  else                                                                                           \
    gn_bwd_reduce_kernel<T, false, U><<<grid, kThreads, lds, st>>>(                              \
        (const T*)x, (const T*)dy, gamma, beta, mean, rstd, S, C, G, p.chunk_px,                 \
        p.rows_per_iter, part, drop);                                                            \
  gn_bwd_sum_kernel<<<dim3((unsigned)vd_cdiv(C, 64), B, ksplit), 1024, 0, st>>>(                \
      part, p.nchunk, C, kSumPer, sums);                                                         \
  gn_bwd_finalize_kernel<<<1, kThreads, 0, st>>>(sums, ksplit, B, C, G, S, gamma, coef, dgamma,  \
                                                 dbeta);                                          \
  if (silu)                                                                                      \
    gn_bwd_apply_kernel<T, true, U><<<grid, kThreads, 0, st>>>(                                  \
        (const T*)x, (const T*)dy, gamma, beta, mean, rstd, coef, (const T*)dadd, (T*)dx, S, C,  \
        G, p.chunk_px, p.rows_per_iter, drop);                                                   \
  else                                                                                           \
    gn_bwd_apply_kernel<T, false, U><<<grid, kThreads, 0, st>>>(                                 \
        (const T*)x, (const T*)dy, gamma, beta, mean, rstd, coef, (const T*)dadd, (T*)dx, S, C,  \
        G, p.chunk_px, p.rows_per_iter, drop)
  const int u = g_gn_unroll.load(std::memory_order_relaxed);
  return VD_DISPATCH_DTYPE(dtype, T, {
    if (u == 4) {
      VD_GN_BWD(4);
    } else if (u == 2) {
      VD_GN_BWD(2);
    } else {
      VD_GN_BWD(1);
    }
  });
#undef VD_GN_BWD
}

}  // extern "C"
