// data.hip -- the data path of TalkingFaceFrameDataset (reference video-generation/dataset.py)
// on this build: host-side audio window DSP (dataset.py:51-66, 113-130) and a GPU kernel for
// the frame transform (dataset.py:109-111 with train.py:70-75's transforms).
//
// Frames: ToPILImage -> Resize((128, 128)) -> ToTensor -> Normalize(0.5, 0.5).  torchvision
// hands a PIL image to PIL's bilinear resample, which always antialiases: a separable
// triangle filter whose support widens with the downscale factor, 22-bit fixed-point
// coefficients, a horizontal pass into an 8-bit intermediate image (rounded and clipped),
// then a vertical pass (PIL libImaging/Resample.c).  vd_resize_plan computes those integer
// coefficients on the host exactly as PIL does (double arithmetic, same rounding); the two
// passes run on the GPU (vd_frames_resize_normalize), so the uint8 result is bit-identical
// to PIL and the normalised output is (v / 255 - 0.5) / 0.5 in fp32 or bf16.
//
// Audio (host, per item; a few thousand samples): the reference's window
// [(out - 5) / fps, out / fps) s of the track, torchaudio highpass_biquad(300 Hz)
// (lfilter with clamping to [-1, 1]), (x - mean) / std (unbiased), then process_audio:
// resample, pad / trim to 4000 samples, and the Wav2Vec2 processor's zero-mean unit-variance
// normalisation.  process_audio's resample compares the CHANNEL count with 16000
// (dataset.py:53) and so resamples from orig_freq = channels; bug_compatible = 1 reproduces
// that (torchaudio's sinc_interp_hann kernel, width 6, rolloff 0.99), 0 resamples from the
// track's true rate (identity at 16 kHz).
#include "vd_common.h"

#include <math.h>
#include <string.h>

#include <algorithm>
#include <numeric>
#include <vector>

namespace {

// ------------------------------------------------------------------ frames (GPU)
constexpr int kPrecisionBits = 32 - 8 - 2;  // PIL Resample.c PRECISION_BITS

__device__ __forceinline__ uint8_t clip8(int64_t v) {
  v >>= kPrecisionBits;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// pass 1: [N][H][W][3] -> [N][H][OW][3] along x (one thread per output byte)
__global__ void resize_h_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                int64_t rows, int W, int OW, const int* __restrict__ bounds,
                                const int* __restrict__ coef, int ksize) {
  const int64_t total = rows * OW * 3;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % 3);
    const int ox = (int)((i / 3) % OW);
    const int64_t row = i / (3 * (int64_t)OW);
    const int x0 = bounds[2 * ox], n = bounds[2 * ox + 1];
    const uint8_t* src = in + (row * W + x0) * 3 + c;
    const int* k = coef + (int64_t)ox * ksize;
    int64_t ss = 1 << (kPrecisionBits - 1);
    for (int x = 0; x < n; ++x) ss += (int64_t)src[3 * x] * k[x];
    out[i] = clip8(ss);
  }
}

// pass 2: [N][H][OW][3] -> normalised [N][3][OH][OW] (or channels-last [N][OH][OW][3])
template <typename T>
__global__ void resize_v_kernel(const uint8_t* __restrict__ in, T* __restrict__ out, int64_t n,
                                int H, int OH, int OW, const int* __restrict__ bounds,
                                const int* __restrict__ coef, int ksize, int64_t frame_stride,
                                int channels_last) {
  const int64_t total = n * OH * OW * 3;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % 3);
    const int ox = (int)((i / 3) % OW);
    const int oy = (int)((i / (3 * (int64_t)OW)) % OH);
    const int64_t f = i / (3 * (int64_t)OW * OH);
    const int y0 = bounds[2 * oy], m = bounds[2 * oy + 1];
    const uint8_t* src = in + ((f * H + y0) * OW + ox) * 3 + c;
    const int* k = coef + (int64_t)oy * ksize;
    int64_t ss = 1 << (kPrecisionBits - 1);
    for (int y = 0; y < m; ++y) ss += (int64_t)src[(int64_t)3 * OW * y] * k[y];
    const float v = ((float)clip8(ss) / 255.f - 0.5f) / 0.5f;
    const int64_t o = channels_last ? f * frame_stride + ((int64_t)oy * OW + ox) * 3 + c
                                    : f * frame_stride + ((int64_t)c * OH + oy) * OW + ox;
    Elem<T>::st(out + o, v);
  }
}

// ------------------------------------------------------------------ PIL coefficient plan
double bilinear(double x) {
  if (x < 0.0) x = -x;
  return x < 1.0 ? 1.0 - x : 0.0;
}

// Resample.c precompute_coeffs + normalize_coeffs_8bpc for the bilinear filter
int plan_axis(int in_size, int out_size, int* bounds, int* coef, int ksize_cap) {
  const double scale = (double)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const int ksize = (int)ceil(support) * 2 + 1;
  if (ksize > ksize_cap) return -1;
  std::vector<double> k(ksize);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      const double w = bilinear((x + xmin - center + 0.5) * ss);
      k[x] = w;
      ww += w;
    }
    for (int x = 0; x < ksize; ++x) {
      const double w = x < xmax ? (ww != 0.0 ? k[x] / ww : k[x]) : 0.0;
      coef[(int64_t)xx * ksize + x] =
          w < 0 ? (int)(-0.5 + w * (1 << kPrecisionBits)) : (int)(0.5 + w * (1 << kPrecisionBits));
    }
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  return ksize;
}

// ------------------------------------------------------------------ audio (host)
// torchaudio.functional.highpass_biquad (Q = 1/sqrt 2) -> lfilter(clamp=True): coefficients
// normalised by a0, direct-form difference equation, output clamped to [-1, 1]
void highpass_biquad(const float* x, float* y, int64_t n, int sr, double cutoff) {
  const double Q = 0.707;
  const double w0 = 2.0 * M_PI * cutoff / sr;
  const double alpha = sin(w0) / 2.0 / Q;
  const double b0 = (1 + cos(w0)) / 2, b1 = -1 - cos(w0), b2 = b0;
  const double a0 = 1 + alpha, a1 = -2 * cos(w0), a2 = 1 - alpha;
  // torchaudio normalises in the waveform dtype (fp32)
  const float nb0 = (float)(b0 / a0), nb1 = (float)(b1 / a0), nb2 = (float)(b2 / a0);
  const float na1 = (float)(a1 / a0), na2 = (float)(a2 / a0);
  float x1 = 0.f, x2 = 0.f, y1 = 0.f, y2 = 0.f;
  for (int64_t i = 0; i < n; ++i) {
    const float xi = x[i];
    float yi = nb0 * xi + nb1 * x1 + nb2 * x2 - na1 * y1 - na2 * y2;
    x2 = x1;
    x1 = xi;
    y2 = y1;
    y1 = yi;  // the recursion runs on the unclamped output
    y[i] = yi < -1.f ? -1.f : (yi > 1.f ? 1.f : yi);
  }
}

// torchaudio.functional.resample (sinc_interp_hann, lowpass_filter_width 6, rolloff 0.99),
// first `keep` output samples of one channel
void sinc_resample(const float* x, int64_t n, int orig, int nw, float* out, int64_t keep) {
  const int g = std::gcd(orig, nw);
  if (orig == nw) {
    for (int64_t i = 0; i < keep; ++i) out[i] = i < n ? x[i] : 0.f;
    return;
  }
  const int of = orig / g, nf = nw / g;
  const double base = std::min(of, nf) * 0.99;
  const int width = (int)ceil(6.0 * of / base);
  const int klen = 2 * width + of;
  const int64_t target = (int64_t)ceil((double)nf * n / of);
  for (int64_t j = 0; j < keep; ++j) {
    if (j >= target) {
      out[j] = 0.f;
      continue;
    }
    const int64_t pos = j / nf;  // conv output position (stride of)
    const int phase = (int)(j % nf);
    double acc = 0.0;
    for (int kk = 0; kk < klen; ++kk) {
      const int64_t src = pos * of + kk - width;  // index into the unpadded input
      if (src < 0 || src >= n) continue;
      double t = (-(double)phase / nf + (double)(kk - width) / of) * base;
      if (t < -6.0) t = -6.0;
      if (t > 6.0) t = 6.0;
      const double win = cos(t * M_PI / 6.0 / 2.0);
      const double tp = t * M_PI;
      const double sinc = tp == 0.0 ? 1.0 : sin(tp) / tp;
      acc += (double)(float)(sinc * win * win * base / of) * x[src];
    }
    out[j] = (float)acc;
  }
}

}  // namespace

extern "C" {

int vd_resize_plan(int in_size, int out_size, int* bounds, int* coef, int ksize_cap) {
  VD_REQUIRE(in_size > 0 && out_size > 0 && bounds && coef, "bad resize plan arguments");
  const int k = plan_axis(in_size, out_size, bounds, coef, ksize_cap);
  VD_REQUIRE(k > 0, "resize %d -> %d needs %d taps > cap %d", in_size, out_size,
             (int)ceil((double)in_size / out_size) * 2 + 1, ksize_cap);
  return VD_OK;
}

int vd_frames_resize_normalize(const uint8_t* frames, int64_t n, int H, int W, int OH, int OW,
                               const int* xb, const int* xc, int xk, const int* yb,
                               const int* yc, int yk, uint8_t* tmp, void* out, int dtype,
                               int64_t frame_stride, int channels_last, void* stream) {
  VD_REQUIRE(frames && out && tmp && xb && xc && yb && yc && n > 0, "null tensor");
  VD_REQUIRE(H > 0 && W > 0 && OH > 0 && OW > 0 && xk > 0 && yk > 0, "bad frame shape");
  hipStream_t st = VD_STREAM(stream);
  const int64_t t1 = n * H * OW * 3;
  int g = (int)std::min<int64_t>(vd_cdiv(t1, 256), 16384);
  resize_h_kernel<<<g, 256, 0, st>>>(frames, tmp, n * H, W, OW, xb, xc, xk);
  int rc = vd::check_launch("resize_h");
  if (rc) return rc;
  const int64_t t2 = n * OH * OW * 3;
  g = (int)std::min<int64_t>(vd_cdiv(t2, 256), 16384);
  return VD_DISPATCH_DTYPE(dtype, T, resize_v_kernel<T><<<g, 256, 0, st>>>(
      tmp, (T*)out, n, H, OH, OW, yb, yc, yk, frame_stride, channels_last));
}

int vd_audio_window(const float* wave, int channels, int64_t n, int sr, double fps,
                    int out_frame, int buffer_frames, int target_len, int target_sr,
                    int bug_compatible, float* out) {
  VD_REQUIRE(wave && out && channels > 0 && n > 0 && sr > 0 && fps > 0 && target_len > 0,
             "bad audio window arguments");
  // dataset.py:114-122
  const double fd = 1.0 / fps;
  const double start_sec = std::max(0.0, (out_frame - buffer_frames) * fd);
  const double end_sec = out_frame * fd;
  int64_t s0 = (int64_t)(sr * start_sec), s1 = (int64_t)(sr * end_sec);
  s0 = std::min(std::max<int64_t>(s0, 0), n);
  s1 = std::min(std::max<int64_t>(s1, s0), n);
  const int64_t len = s1 - s0;
  std::vector<float> seg((size_t)channels * std::max<int64_t>(len, 1));
  // dataset.py:123: normalize_waveform(high_pass_filter(seg)) -- statistics over all channels
  for (int c = 0; c < channels; ++c) highpass_biquad(wave + (int64_t)c * n + s0, &seg[c * len], len, sr, 300.0);
  const int64_t cnt = (int64_t)channels * len;
  double mean = 0.0;
  for (int64_t i = 0; i < cnt; ++i) mean += seg[i];
  mean /= (double)std::max<int64_t>(cnt, 1);
  double var = 0.0;
  for (int64_t i = 0; i < cnt; ++i) var += (seg[i] - mean) * (seg[i] - mean);
  const float mf = (float)mean;
  const float sd = (float)sqrt(var / (double)std::max<int64_t>(cnt - 1, 1));  // torch .std()
  for (int64_t i = 0; i < cnt; ++i) seg[i] = (seg[i] - mf) / sd;
  // process_audio (dataset.py:51-66): resample (orig_freq = channels when bug-compatible),
  // then pad with zeros / trim to target_len
  const int orig = bug_compatible ? channels : sr;
  for (int c = 0; c < channels; ++c) {
    float* o = out + (int64_t)c * target_len;
    if (bug_compatible && channels == target_sr)
      for (int64_t i = 0; i < target_len; ++i) o[i] = i < len ? seg[c * len + i] : 0.f;
    else
      sinc_resample(&seg[c * len], len, orig, target_sr, o, target_len);
    // Wav2Vec2FeatureExtractor zero_mean_unit_var_norm: (x - mean) / sqrt(var + 1e-7)
    double m = 0.0, v = 0.0;
    for (int i = 0; i < target_len; ++i) m += o[i];
    m /= target_len;
    for (int i = 0; i < target_len; ++i) v += (o[i] - m) * (o[i] - m);
    v /= target_len;
    const double inv = 1.0 / sqrt(v + 1e-7);
    for (int i = 0; i < target_len; ++i) o[i] = (float)((o[i] - m) * inv);
  }
  return VD_OK;
}

}  // extern "C"
