// cond.hip -- UNetAudio conditioning assembly and flat SiLU.
//
// vd_cond_concat replaces the broadcast + nearest-resize + th.cat of
// UNetAudio.forward (reference unet_audio.py:52-61): it writes the
// [image | image-cond | audio | zero pad] channels of every pixel straight
// into the channels-last input buffer of the first conv, so the
// expand()-ed audio/image tensors are never materialised.
// vd_silu / vd_silu_bwd serve the timestep-embedding MLP (unet.py:483-487)
// and ResBlock.emb_layers (unet.py:211-217).
#include "vd_common.h"

namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t work) {
  int64_t g = vd_cdiv(work, kBlock);
  return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

// torch "nearest" source index for an in -> out resize
__device__ __forceinline__ int nearest_src(int dst, int in, int out) {
  const float scale = (float)in / (float)out;
  int s = (int)floorf((float)dst * scale);
  return s < in - 1 ? s : in - 1;
}

template <typename T>
__global__ void silu_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    Elem<T>::st(y + i, silu_f(Elem<T>::ld(x + i)));
}

template <typename T>
__global__ void silu_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                T* __restrict__ dx, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float z = Elem<T>::ld(x + i);
    const float s = 1.f / (1.f + __expf(-z));
    Elem<T>::st(dx + i, Elem<T>::ld(dy + i) * s * (1.f + z * (1.f - s)));
  }
}

// one thread per (pixel, output channel)
template <typename T>
__global__ void cond_concat_kernel(const T* __restrict__ image, const T* __restrict__ imc,
                                   const T* __restrict__ audio, T* __restrict__ out, int B, int T_,
                                   int H, int W, int Cx, int h, int w, int Ci, int Ca, int Cs) {
  const int64_t n = (int64_t)B * T_ * H * W * Cs;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cs);
    int64_t p = i / Cs;
    const int x = (int)(p % W);
    p /= W;
    const int y = (int)(p % H);
    p /= H;
    const int t = (int)(p % T_);
    const int b = (int)(p / T_);
    float v = 0.f;
    if (c < Cx) {
      v = Elem<T>::ld(image + ((((int64_t)b * T_ + t) * H + y) * W + x) * Cx + c);
    } else if (c < Cx + Ci) {
      const int ys = nearest_src(y, h, H), xs = nearest_src(x, w, W);
      v = Elem<T>::ld(imc + (((int64_t)b * h + ys) * w + xs) * Ci + (c - Cx));
    } else if (c < Cx + Ci + Ca) {
      v = Elem<T>::ld(audio + ((int64_t)b * T_ + t) * Ca + (c - Cx - Ci));
    }
    Elem<T>::st(out + i, v);
  }
}

// One thread per (pixel, 16-byte chunk of output channels): the pixel's coordinates are
// decoded once per chunk (32-bit), the chunk's channels gathered from their section, and
// the chunk written with one 16-B store.  Needs out_cstride % (16 / sizeof(T)) == 0.
// (The per-element form above took 233 us for 262144 pixels x 200 channels: four 64-bit
// divisions per element.)
template <typename T>
__global__ void cond_concat_vec_kernel(const T* __restrict__ image, const T* __restrict__ imc,
                                       const T* __restrict__ audio, T* __restrict__ out, int P,
                                       int T_, int H, int W, int Cx, int h, int w, int Ci, int Ca,
                                       int Cs) {
  constexpr int E = 16 / sizeof(T);
  const int nch = Cs / E;
  const int64_t n = (int64_t)P * nch;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(i / nch), c0 = (int)(i - (int64_t)p * nch) * E;
    const int x = p % W, r = p / W, y = r % H, bt = r / H, b = bt / T_;
    const int ys = nearest_src(y, h, H), xs = nearest_src(x, w, W);
    const T* ip = image + (int64_t)p * Cx;
    const T* cp = imc + ((int64_t)(b * h + ys) * w + xs) * Ci - Cx;
    const T* ap = audio + (int64_t)bt * Ca - Cx - Ci;
    T v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int c = c0 + e;
      v[e] = c < Cx ? ip[c] : c < Cx + Ci ? cp[c] : c < Cx + Ci + Ca ? ap[c] : T{};
    }
    *reinterpret_cast<uint4*>(out + (int64_t)p * Cs + c0) = *reinterpret_cast<const uint4*>(v);
  }
}

// d_audio partials: part[chunk][bt][c] = sum over the chunk's (y, x) rows; grid (B*T, chunks)
template <typename T>
__global__ void cond_audio_bwd_kernel(const T* __restrict__ dout, float* __restrict__ part, int BT,
                                      int H, int W, int off, int Ca, int Cs, int rows_per_block) {
  const int bt = blockIdx.x;
  const int64_t HW = (int64_t)H * W;
  const int64_t p0 = (int64_t)blockIdx.y * rows_per_block;
  int64_t p1 = p0 + rows_per_block;
  if (p1 > HW) p1 = HW;
  for (int c = threadIdx.x; c < Ca; c += blockDim.x) {
    float s = 0.f;
    for (int64_t p = p0; p < p1; ++p)
      s += Elem<T>::ld(dout + ((int64_t)bt * HW + p) * Cs + off + c);
    part[((int64_t)blockIdx.y * BT + bt) * Ca + c] = s;
  }
}

// d_audio[bt][c] = the chunk partials added in ascending chunk order (bit-reproducible; the
// round-3 kernel added them with float atomics in arrival order)
__global__ void cond_audio_finish_kernel(const float* __restrict__ part, int chunks, int64_t n,
                                         float* __restrict__ da) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int k = 0; k < chunks; ++k) s += part[k * n + i];
  da[i] = s;
}

// first destination index whose nearest source is >= src (nearest_src is non-decreasing)
__device__ __forceinline__ int nearest_first(int src, int in, int out) {
  int d = (int)(((int64_t)src * out) / in) - 2;
  if (d < 0) d = 0;
  while (d < out && nearest_src(d, in, out) < src) ++d;
  return d;
}

// d_imc[b][ys][xs][c] = sum over t and the (y, x) whose nearest source is (ys, xs): each
// thread owns one source element and walks its preimage rectangle in a fixed order
// (no atomics: bit-reproducible for any resize ratio)
template <typename T>
__global__ void cond_imc_bwd_kernel(const T* __restrict__ dout, float* __restrict__ di, int B,
                                    int T_, int H, int W, int off, int h, int w, int Ci, int Cs) {
  const int64_t n = (int64_t)B * h * w * Ci;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % Ci);
    int64_t q = i / Ci;
    const int xs = (int)(q % w);
    q /= w;
    const int ys = (int)(q % h);
    const int b = (int)(q / h);
    const int y0 = nearest_first(ys, h, H), x0 = nearest_first(xs, w, W);
    float s = 0.f;
    for (int t = 0; t < T_; ++t)
      for (int y = y0; y < H && nearest_src(y, h, H) == ys; ++y)
        for (int x = x0; x < W && nearest_src(x, w, W) == xs; ++x)
          s += Elem<T>::ld(dout + ((((int64_t)b * T_ + t) * H + y) * W + x) * Cs + off + c);
    di[i] = s;
  }
}

constexpr int kAudioRows = 256;  // (y, x) rows per d_audio partial

}  // namespace

extern "C" {

int vd_silu(const void* x, void* y, int64_t n, int dtype, void* stream) {
  VD_REQUIRE(x && y && n > 0, "bad silu arguments");
  return VD_DISPATCH_DTYPE(dtype, T, {
    silu_kernel<T><<<grid_for(n), kBlock, 0, VD_STREAM(stream)>>>((const T*)x, (T*)y, n);
  });
}

int vd_silu_bwd(const void* x, const void* dy, void* dx, int64_t n, int dtype, void* stream) {
  VD_REQUIRE(x && dy && dx && n > 0, "bad silu_bwd arguments");
  return VD_DISPATCH_DTYPE(dtype, T, {
    silu_bwd_kernel<T><<<grid_for(n), kBlock, 0, VD_STREAM(stream)>>>((const T*)x, (const T*)dy,
                                                                      (T*)dx, n);
  });
}

int vd_cond_concat(const void* image, const void* imc, const void* audio, void* out, int B, int T,
                   int H, int W, int Cx, int h, int w, int Ci, int Ca, int out_cstride, int dtype,
                   void* stream) {
  VD_REQUIRE(image && out, "null tensor");
  VD_REQUIRE((Ci == 0 || imc) && (Ca == 0 || audio), "null conditioning tensor");
  VD_REQUIRE(B > 0 && T > 0 && H > 0 && W > 0 && Cx > 0 && h > 0 && w > 0, "bad shape");
  VD_REQUIRE(out_cstride >= Cx + Ci + Ca, "out_cstride %d < %d", out_cstride, Cx + Ci + Ca);
  const int64_t n = (int64_t)B * T * H * W * out_cstride;
  const int64_t P = (int64_t)B * T * H * W;
  const int E = dtype == VD_BF16 ? 8 : 4;
  if (out_cstride % E == 0 && P < (1ll << 31) && (reinterpret_cast<uintptr_t>(out) & 15) == 0)
    return VD_DISPATCH_DTYPE(dtype, Tp, {
      const int64_t work = P * (out_cstride / E);
      int64_t g = vd_cdiv(work, kBlock);
      if (g > 65536) g = 65536;
      cond_concat_vec_kernel<Tp><<<(unsigned)g, kBlock, 0, VD_STREAM(stream)>>>(
          (const Tp*)image, (const Tp*)imc, (const Tp*)audio, (Tp*)out, (int)P, T, H, W, Cx, h,
          w, Ci, Ca, out_cstride);
    });
  return VD_DISPATCH_DTYPE(dtype, Tp, {
    cond_concat_kernel<Tp><<<grid_for(n), kBlock, 0, VD_STREAM(stream)>>>(
        (const Tp*)image, (const Tp*)imc, (const Tp*)audio, (Tp*)out, B, T, H, W, Cx, h, w, Ci,
        Ca, out_cstride);
  });
}

size_t vd_cond_concat_bwd_workspace_size(int B, int T, int H, int W, int Ca) {
  if (B <= 0 || T <= 0 || H <= 0 || W <= 0 || Ca <= 0) return 0;
  return (size_t)vd_cdiv((int64_t)H * W, kAudioRows) * B * T * Ca * sizeof(float) + 256;
}

int vd_cond_concat_bwd(const void* dout, float* d_imc, float* d_audio, int B, int T, int H, int W,
                       int Cx, int h, int w, int Ci, int Ca, int out_cstride, int dtype,
                       void* workspace, void* stream) {
  VD_REQUIRE(dout, "null tensor");
  VD_REQUIRE(B > 0 && T > 0 && H > 0 && W > 0 && h > 0 && w > 0, "bad shape");
  VD_REQUIRE(!(d_audio && Ca > 0) || workspace, "d_audio needs the workspace");
  hipStream_t st = VD_STREAM(stream);
  return VD_DISPATCH_DTYPE(dtype, Tp, {
    if (d_audio && Ca > 0) {
      const int chunks = (int)vd_cdiv((int64_t)H * W, kAudioRows);
      float* part = reinterpret_cast<float*>(workspace);
      dim3 grid((unsigned)(B * T), (unsigned)chunks);
      cond_audio_bwd_kernel<Tp><<<grid, 128, 0, st>>>((const Tp*)dout, part, B * T, H, W,
                                                      Cx + Ci, Ca, out_cstride, kAudioRows);
      const int64_t n = (int64_t)B * T * Ca;
      cond_audio_finish_kernel<<<(unsigned)vd_cdiv(n, 256), 256, 0, st>>>(part, chunks, n,
                                                                          d_audio);
    }
    if (d_imc && Ci > 0) {
      const int64_t n = (int64_t)B * h * w * Ci;
      cond_imc_bwd_kernel<Tp><<<grid_for(n), kBlock, 0, st>>>((const Tp*)dout, d_imc, B, T, H, W,
                                                              Cx, h, w, Ci, out_cstride);
    }
  });
}

}  // extern "C"
