// layernorm.hip -- the per-token ops of the ViViT lipreading encoder:
// LayerNorm over the hidden size (VivitLayer.layernorm_before / layernorm_after and the
// final VivitModel.layernorm, eps 1e-6) and the tanh GELU of VivitMLP (hidden_act
// "gelu_fast").  Reference: lipreading/huggingface_vivit_model.py:18-33 wraps
// transformers' VivitModel (main.py:57-58 builds it); the GEMMs run on the conv kernel
// (1x1 implicit GEMM) and the attention on attention.hip.
//
// LayerNorm rows are tokens, [rows][C] contiguous, C % 8 == 0 and C <= 2048: one wave per
// row holds the row in registers (<= 4 chunks of 8 per lane), so the forward reads x once
// and the backward reads x and dy once.  Statistics and affine parameters are fp32.  The
// weight / bias gradients are per-block partial column sums, then a deterministic finish.
#include "vd_common.h"

namespace {

constexpr int kLnMaxChunks = 4;          // 8-element chunks per lane: C <= 64 * 8 * 4
constexpr int kLnWaves = 4;              // waves (rows in flight) per block
constexpr int kLnRowsPerBlockBwd = 64;   // rows per block of the backward partial sums

template <typename T>
__global__ __launch_bounds__(64 * kLnWaves) void ln_fwd_kernel(
    const T* __restrict__ x, const float* __restrict__ w, const float* __restrict__ b,
    T* __restrict__ y, float* __restrict__ mean, float* __restrict__ rstd, int rows, int C,
    float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kLnWaves + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nch = C / 8;
  const T* xr = x + (int64_t)row * C;
  float v[kLnMaxChunks][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kLnMaxChunks; ++k) {
    const int c = lane + 64 * k;
    if (c < nch) {
      load8(xr + 8 * c, v[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[k][j];
    }
  }
  const float mu = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < kLnMaxChunks; ++k)
    if (lane + 64 * k < nch)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[k][j] - mu;
        q += d * d;
      }
  const float rs = rsqrtf(wave_sum(q) / C + eps);
#pragma unroll
  for (int k = 0; k < kLnMaxChunks; ++k) {
    const int c = lane + 64 * k;
    if (c < nch) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mu) * rs * w[8 * c + j] + b[8 * c + j];
      store8(y + (int64_t)row * C + 8 * c, o);
    }
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * w; per-block partial
// sum(dy * xhat) and sum(dy) per column into part[block][2][C].
template <typename T>
__global__ __launch_bounds__(64 * kLnWaves) void ln_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const float* __restrict__ w,
    const float* __restrict__ mean, const float* __restrict__ rstd, T* __restrict__ dx,
    float* __restrict__ part, int rows, int C) {
  __shared__ float red[kLnWaves][2][64 * 8 * kLnMaxChunks / 4];  // reused per 1/4 of C
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = C / 8;
  float pw[kLnMaxChunks][8], pb[kLnMaxChunks][8];
#pragma unroll
  for (int k = 0; k < kLnMaxChunks; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) pw[k][j] = pb[k][j] = 0.f;
  const int r0 = blockIdx.x * kLnRowsPerBlockBwd;
  const int r1 = min(rows, r0 + kLnRowsPerBlockBwd);
  for (int row = r0 + wave; row < r1; row += kLnWaves) {
    const float mu = mean[row], rs = rstd[row];
    float xh[kLnMaxChunks][8], g[kLnMaxChunks][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < kLnMaxChunks; ++k) {
      const int c = lane + 64 * k;
      if (c < nch) {
        float xv[8], gv[8];
        load8(x + (int64_t)row * C + 8 * c, xv);
        load8(dy + (int64_t)row * C + 8 * c, gv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[k][j] = (xv[j] - mu) * rs;
          pw[k][j] += gv[j] * xh[k][j];
          pb[k][j] += gv[j];
          g[k][j] = gv[j] * w[8 * c + j];
          s1 += g[k][j];
          s2 += g[k][j] * xh[k][j];
        }
      }
    }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
#pragma unroll
    for (int k = 0; k < kLnMaxChunks; ++k) {
      const int c = lane + 64 * k;
      if (c < nch) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs * (g[k][j] - s1 - xh[k][j] * s2);
        store8(dx + (int64_t)row * C + 8 * c, o);
      }
    }
  }
  // fixed-order reduction of the kLnWaves waves' column partials, one chunk index k at a time
  float* out = part + (int64_t)blockIdx.x * 2 * C;
#pragma unroll
  for (int k = 0; k < kLnMaxChunks; ++k) {
    if (64 * k >= nch) break;  // block-uniform
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[wave][0][8 * lane + j] = pw[k][j];
      red[wave][1][8 * lane + j] = pb[k][j];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * 512; i += 64 * kLnWaves) {
      const int which = i / 512, e = i % 512;
      const int col = 512 * k + e;
      if (col < C) {
        float s = 0.f;
#pragma unroll
        for (int wv = 0; wv < kLnWaves; ++wv) s += red[wv][which][e];
        out[which * C + col] = s;
      }
    }
    __syncthreads();
  }
}

__global__ void ln_bwd_finish_kernel(const float* __restrict__ part, int nblk, int C,
                                     float* __restrict__ dw, float* __restrict__ db) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * C) return;
  const int which = i / C, col = i % C;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += part[((int64_t)b * 2 + which) * C + col];
  (which ? db : dw)[col] = s;
}

constexpr float kGeluK0 = 0.7978845608f, kGeluK1 = 0.044715f;

template <typename T>
__global__ void gelu_tanh_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v[8];
    load8(x + 8 * i, v);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = 0.5f * v[j] * (1.f + tanhf(kGeluK0 * v[j] * (1.f + kGeluK1 * v[j] * v[j])));
    store8(y + 8 * i, v);
  }
}

template <typename T>
__global__ void gelu_tanh_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                     T* __restrict__ dx, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v[8], g[8];
    load8(x + 8 * i, v);
    load8(dy + 8 * i, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float a = v[j], a2 = a * a;
      const float t = tanhf(kGeluK0 * a * (1.f + kGeluK1 * a2));
      g[j] *= 0.5f * (1.f + t) + 0.5f * a * (1.f - t * t) * kGeluK0 * (1.f + 3.f * kGeluK1 * a2);
    }
    store8(dx + 8 * i, g);
  }
}

int grid8(int64_t n8) { return (int)std::min<int64_t>(vd_cdiv(n8, 256), 256 * 16); }

}  // namespace

extern "C" {

size_t vd_layernorm_workspace_size(int rows, int C) {
  return (size_t)vd_cdiv(rows, kLnRowsPerBlockBwd) * 2 * C * sizeof(float);
}

int vd_layernorm_fwd(const void* x, const float* w, const float* b, void* y, float* mean,
                     float* rstd, int rows, int C, float eps, int dtype, void* stream) {
  VD_REQUIRE(x && w && b && y && mean && rstd, "null layernorm argument");
  VD_REQUIRE(rows > 0 && C > 0 && C % 8 == 0 && C <= 64 * 8 * kLnMaxChunks,
             "layernorm: C %d must be a multiple of 8 and <= %d", C, 64 * 8 * kLnMaxChunks);
  return VD_DISPATCH_DTYPE(dtype, T, {
    ln_fwd_kernel<T><<<(unsigned)vd_cdiv(rows, kLnWaves), 64 * kLnWaves, 0, VD_STREAM(stream)>>>(
        (const T*)x, w, b, (T*)y, mean, rstd, rows, C, eps);
  });
}

int vd_layernorm_bwd(const void* dy, const void* x, const float* w, const float* mean,
                     const float* rstd, void* dx, float* dw, float* db, int rows, int C,
                     int dtype, void* workspace, size_t workspace_bytes, void* stream) {
  VD_REQUIRE(dy && x && w && mean && rstd && dx && dw && db && workspace,
             "null layernorm_bwd argument");
  VD_REQUIRE(rows > 0 && C > 0 && C % 8 == 0 && C <= 64 * 8 * kLnMaxChunks,
             "layernorm_bwd: C %d must be a multiple of 8 and <= %d", C, 64 * 8 * kLnMaxChunks);
  VD_REQUIRE(workspace_bytes >= vd_layernorm_workspace_size(rows, C),
             "layernorm_bwd: workspace %zu < %zu", workspace_bytes,
             vd_layernorm_workspace_size(rows, C));
  const int nblk = (int)vd_cdiv(rows, kLnRowsPerBlockBwd);
  float* part = (float*)workspace;
  return VD_DISPATCH_DTYPE(dtype, T, {
    ln_bwd_kernel<T><<<nblk, 64 * kLnWaves, 0, VD_STREAM(stream)>>>(
        (const T*)dy, (const T*)x, w, mean, rstd, (T*)dx, part, rows, C);
    ln_bwd_finish_kernel<<<(unsigned)vd_cdiv(2 * C, 256), 256, 0, VD_STREAM(stream)>>>(
        part, nblk, C, dw, db);
  });
}

int vd_gelu_tanh(const void* x, void* y, int64_t n, int dtype, void* stream) {
  VD_REQUIRE(x && y && n > 0 && n % 8 == 0, "gelu: n %lld must be a positive multiple of 8",
             (long long)n);
  return VD_DISPATCH_DTYPE(dtype, T, {
    gelu_tanh_kernel<T><<<grid8(n / 8), 256, 0, VD_STREAM(stream)>>>((const T*)x, (T*)y, n / 8);
  });
}

int vd_gelu_tanh_bwd(const void* x, const void* dy, void* dx, int64_t n, int dtype,
                     void* stream) {
  VD_REQUIRE(x && dy && dx && n > 0 && n % 8 == 0,
             "gelu_bwd: n %lld must be a positive multiple of 8", (long long)n);
  return VD_DISPATCH_DTYPE(dtype, T, {
    gelu_tanh_bwd_kernel<T><<<grid8(n / 8), 256, 0, VD_STREAM(stream)>>>(
        (const T*)x, (const T*)dy, (T*)dx, n / 8);
  });
}

}  // extern "C"
