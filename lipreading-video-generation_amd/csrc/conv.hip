// conv.hip -- channels-last 3-D convolution as implicit GEMM on MFMA (gfx950).
//
// Replaces conv_nd (reference utils.py:59-69) at every call site of the hot
// path: 3x3x3 stride-1 convs (unet.py:110,197,223,231,494,627), the (1,2,2)-
// strided Downsample conv (unet.py:143-145), 1x1x1 skip convs (unet.py:234)
// and AttentionBlock's 1x1 Conv1d qkv / proj_out (unet.py:298,306).
//
//   fwd       : Y[m][n]  = sum_k A[m][k] W[n][k] (+bias[n] +chan_add[b][n] +res[m][n])
//               m = output pixel, n = Co, k = (tap, ci), A gathered from X.
//   bwd_data  : the same kernel in TRANSPOSED gather mode: m = input pixel,
//               n = Ci, k = (tap, co), A gathered from dY where
//               (pos + pad - tap) is divisible by the stride.
//   bwd_weight: dW[co][(tap,ci)] += sum_m dY[m][co] X[src(m,tap)][ci], split-K
//               over m with fp32 atomics; both operands are read transposed
//               from natural [pixel][channel] LDS tiles (ds_read_b64_tr_b16).
//
// bf16: v_mfma_f32_16x16x32_bf16, fp32 accumulate.  fp32 (parity mode):
// v_mfma_f32_16x16x4_f32, exact fp32 products.  Tiles are staged global ->
// registers -> LDS (double buffered, one barrier per K step); LDS rows of
// 64 B use a chunk XOR swizzle that is conflict-free for the fragment reads.
#include "vd_common.h"
#include <stdio.h>
#include <stdlib.h>

#include <atomic>

namespace {

constexpr int kThreads = 256;
constexpr int kBK = 32;  // K elements per step

template <typename T> struct Cfg;
template <> struct Cfg<bf16_t> {
  static constexpr int EPC = 8;                  // elements per 16-B chunk
  static constexpr int CPR = kBK / EPC;          // chunks per LDS row (4)
  static constexpr int LDK = kBK;                // LDS row length (elements)
};
template <> struct Cfg<float> {
  static constexpr int EPC = 4;
  static constexpr int CPR = kBK / EPC;          // 8
  static constexpr int LDK = kBK + 4;            // padded rows: scalar fragment reads
};

// physical 16-B chunk of logical chunk kc in LDS row r (bf16 rows are 64 B)
__device__ __forceinline__ int swz(int r, int kc) {
  const int t = (r >> 2) & 3;
  return kc ^ ((0x1320 >> (4 * t)) & 3);  // table {0,2,3,1}
}

template <typename T>
__device__ __forceinline__ int lds_off(int r, int kc) {  // element offset of chunk (r, kc)
  if constexpr (sizeof(T) == 2) return r * Cfg<T>::LDK + swz(r, kc) * Cfg<T>::EPC;
  else return r * Cfg<T>::LDK + kc * Cfg<T>::EPC;
}

struct GemmGeom {
  int B;
  int sT, sH, sW, sC, sCs;  // gathered source: spatial, channels (K per tap), pixel stride
  int dT, dH, dW, N, dNs;   // GEMM rows decode (output pixels), N, output pixel stride
  int kt, kh, kw, st, sh, sw, pt, ph, pw;
  int64_t M;
  int K;
};

// ----------------------------------------------------------------- fwd / bwd-data
template <typename T, int BN, bool TRANSPOSED>
__global__ __launch_bounds__(kThreads, 2) void conv_gemm_kernel(
    GemmGeom g, const T* __restrict__ src, const T* __restrict__ wt, T* __restrict__ dst,
    const float* __restrict__ bias, const float* __restrict__ chan_add,
    const T* __restrict__ residual) {
  constexpr int BM = 128;
  constexpr int EPC = Cfg<T>::EPC, CPR = Cfg<T>::CPR, LDK = Cfg<T>::LDK;
  constexpr int A_CH = BM * CPR / kThreads;  // A chunks per thread
  constexpr int B_CH = BN * CPR / kThreads;
  constexpr int WN = BN / 2;                 // wave tile: 64 x WN
  constexpr int NI = 4, NJ = WN / 16;
  constexpr int A_ELEMS = BM * LDK, B_ELEMS = BN * LDK;
  constexpr int STAGE = A_ELEMS + B_ELEMS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* lds = reinterpret_cast<T*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int ntap_hw = g.kh * g.kw;

  // ---- per-thread A rows (fixed for the whole K loop)
  const int a_kc = tid % CPR;
  int a_b[A_CH], a_t[A_CH], a_h[A_CH], a_w[A_CH];
  bool a_ok[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int r = tid / CPR + i * (kThreads / CPR);
    int64_t m = m0 + r;
    a_ok[i] = m < g.M;
    if (!a_ok[i]) m = 0;
    a_w[i] = (int)(m % g.dW); m /= g.dW;
    a_h[i] = (int)(m % g.dH); m /= g.dH;
    a_t[i] = (int)(m % g.dT);
    a_b[i] = (int)(m / g.dT);
  }
  const int b_kc = tid % CPR;

  auto load_tile = [&](int k0, uint4 (&ra)[A_CH], uint4 (&rb)[B_CH]) {
    const int k = k0 + a_kc * EPC;
    const bool kin = k < g.K;
    const int tap = kin ? k / g.sC : 0;
    const int c = k - tap * g.sC;
    const int ta = tap / ntap_hw, rem = tap - ta * ntap_hw;
    const int tb = rem / g.kw, tc = rem - tb * g.kw;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      int st_, sh_, sw_;
      bool ok = a_ok[i] && kin;
      if (!TRANSPOSED) {
        st_ = a_t[i] * g.st - g.pt + ta;
        sh_ = a_h[i] * g.sh - g.ph + tb;
        sw_ = a_w[i] * g.sw - g.pw + tc;
      } else {
        const int nt = a_t[i] + g.pt - ta, nh = a_h[i] + g.ph - tb, nw = a_w[i] + g.pw - tc;
        ok = ok && nt >= 0 && nh >= 0 && nw >= 0 && nt % g.st == 0 && nh % g.sh == 0 &&
             nw % g.sw == 0;
        st_ = nt / g.st;
        sh_ = nh / g.sh;
        sw_ = nw / g.sw;
      }
      ok = ok && (unsigned)st_ < (unsigned)g.sT && (unsigned)sh_ < (unsigned)g.sH &&
           (unsigned)sw_ < (unsigned)g.sW;
      if (ok) {
        const int64_t pix = (((int64_t)a_b[i] * g.sT + st_) * g.sH + sh_) * g.sW + sw_;
        ra[i] = *reinterpret_cast<const uint4*>(src + pix * g.sCs + c);
      } else {
        ra[i] = make_uint4(0, 0, 0, 0);
      }
    }
    const int kb = k0 + b_kc * EPC;
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int n = n0 + tid / CPR + i * (kThreads / CPR);
      if (n < g.N && kb < g.K)
        rb[i] = *reinterpret_cast<const uint4*>(wt + (int64_t)n * g.K + kb);
      else
        rb[i] = make_uint4(0, 0, 0, 0);
    }
  };
  auto store_tile = [&](int stage, const uint4 (&ra)[A_CH], const uint4 (&rb)[B_CH]) {
    T* As = lds + stage * STAGE;
    T* Bs = As + A_ELEMS;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int r = tid / CPR + i * (kThreads / CPR);
      *reinterpret_cast<uint4*>(As + lds_off<T>(r, a_kc)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int r = tid / CPR + i * (kThreads / CPR);
      *reinterpret_cast<uint4*>(Bs + lds_off<T>(r, b_kc)) = rb[i];
    }
  };

  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (g.K + kBK - 1) / kBK;
  uint4 ra[A_CH], rb[B_CH];
  load_tile(0, ra, rb);
  store_tile(0, ra, rb);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) load_tile((kt + 1) * kBK, ra, rb);
    const T* As = lds + (kt & 1) * STAGE;
    const T* Bs = As + A_ELEMS;
    if constexpr (sizeof(T) == 2) {
      bf16x8 af[NI], bfr[NJ];
#pragma unroll
      for (int i = 0; i < NI; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(As + lds_off<T>(wm * 64 + 16 * i + fr, fq));
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + lds_off<T>(wn * WN + 16 * j + fr, fq));
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < kBK / 4; ++s) {
        float af[NI], bfv[NJ];
#pragma unroll
        for (int i = 0; i < NI; ++i) af[i] = As[(wm * 64 + 16 * i + fr) * LDK + 4 * s + fq];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfv[j] = Bs[(wn * WN + 16 * j + fr) * LDK + 4 * s + fq];
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfv[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) store_tile((kt + 1) & 1, ra, rb);
    __syncthreads();
  }

  // ---- epilogue: stage the fp32 tile in LDS, then coalesced 8-wide stores
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int LDC = BN + 4;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * 64 + 16 * i + fq * 4 + r) * LDC + wn * WN + 16 * j + fr] = acc[i][j][r];
  __syncthreads();
  const int64_t pix_per_b = (int64_t)g.dT * g.dH * g.dW;
  const bool vec = (g.N % 8 == 0) && (g.dNs % 8 == 0);
  for (int v = tid; v < BM * BN / 8; v += kThreads) {
    const int r = v / (BN / 8), c = (v % (BN / 8)) * 8;
    const int64_t m = m0 + r;
    const int n = n0 + c;
    if (m >= g.M || n >= g.N) continue;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = Cs[r * LDC + c + e];
    const int lim = g.N - n < 8 ? g.N - n : 8;
    if (bias)
      for (int e = 0; e < lim; ++e) o[e] += bias[n + e];
    if (chan_add) {
      const int bidx = (int)(m / pix_per_b);  // 64-bit division only where it is needed
      for (int e = 0; e < lim; ++e) o[e] += chan_add[(int64_t)bidx * g.N + n + e];
    }
    T* out = dst + m * g.dNs + n;
    if (vec) {
      if (residual) {
        float rv[8];
        load8(residual + m * g.dNs + n, rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += rv[e];
      }
      store8(out, o);
    } else {
      for (int e = 0; e < lim; ++e) {
        float val = o[e];
        if (residual) val += Elem<T>::ld(residual + m * g.dNs + n + e);
        Elem<T>::st(out + e, val);
      }
    }
  }
}

// ----------------------------------------------------------------- bwd-weight
// dW[co][tap][ci] += sum_m dY[m][co] * X[src(m, tap)][ci]
// grid.x = co_tiles * taps * ci_tiles, grid.y = K splits over m.
struct WgtGeom {
  int B;
  int Ti, Hi, Wi, Ci, xCs;  // X (gathered)
  int To, Ho, Wo, Co, yCs;  // dY
  int kt, kh, kw, st, sh, sw, pt, ph, pw;
  int64_t M;                // B*To*Ho*Wo
  int64_t m_per_split;
  // 0: atomicAdd into dw (vd_conv3d_bwd_weight).  > 0: split y WRITES its partial dW to
  // dw + y * split_stride (vd_conv3d_bwd_weight_det; summed in a fixed order afterwards)
  int64_t split_stride;
  // XCD-aware 1-D grid (wgrad_dma_kernel): xcd_tiles > 0 = the (tile, split) pairs in
  // split-major order are laid out so that each XCD runs a contiguous range of them, i.e.
  // all tiles of one pixel split on ONE XCD, whose L2 then serves the split's dY rows and X
  // strips to every tile (MI355X: workgroup b runs on XCD b % 8, each XCD has its own L2).
  int xcd_tiles, xcd_total;
};

// (tile, split) of this workgroup
__device__ __forceinline__ bool wg_tile(const WgtGeom& g, int* tile, int* split) {
  if (g.xcd_tiles == 0) {
    *tile = blockIdx.x;
    *split = blockIdx.y;
    return true;
  }
  const int per = gridDim.x / 8;
  const int L = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (L >= g.xcd_total) return false;
  *tile = L % g.xcd_tiles;
  *split = L / g.xcd_tiles;
  return true;
}

// one fp32 partial of dW: accumulated (atomics) or stored into the split's own slice
__device__ __forceinline__ void wg_out(const WgtGeom& g, float* dw, int split, int64_t off,
                                       float v) {
  if (g.split_stride)
    dw[(int64_t)split * g.split_stride + off] = v;
  else
    atomicAdd(dw + off, v);
}

template <typename T>
__global__ __launch_bounds__(kThreads) void conv_wgrad_kernel(WgtGeom g, const T* __restrict__ x,
                                                              const T* __restrict__ dy,
                                                              float* __restrict__ dw) {
  constexpr int TM = 64, TN = 64;       // co x ci tile
  constexpr int PK = 32;                // pixels per step
  constexpr int PAD = sizeof(T) == 2 ? 8 : 4;
  constexpr int LD = TM + PAD;          // LDS row (pixel) length, elements
  constexpr int EPC = 16 / sizeof(T);
  constexpr int CPRW = TM / EPC;        // 16-B chunks per 64-channel row
  constexpr int CH = PK * CPRW / kThreads;  // chunks per thread per operand (1 bf16, 2 f32)
  constexpr int STAGE = 2 * PK * LD;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* lds = reinterpret_cast<T*>(smem);

  const int taps = g.kt * g.kh * g.kw;
  const int co_tiles = (g.Co + TM - 1) / TM;
  const int ci_tiles = (g.Ci + TN - 1) / TN;
  int bid = blockIdx.x;
  const int cot = bid % co_tiles; bid /= co_tiles;
  const int cit = bid % ci_tiles; bid /= ci_tiles;
  const int tap = bid;
  const int ta = tap / (g.kh * g.kw), tb = (tap / g.kw) % g.kh, tc = tap % g.kw;
  const int co0 = cot * TM, ci0 = cit * TN;
  const int64_t mbeg = (int64_t)blockIdx.y * g.m_per_split;
  int64_t mend = mbeg + g.m_per_split;
  if (mend > g.M) mend = g.M;
  if (mbeg >= mend) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;  // wave tile 32 (co) x 32 (ci)

  auto load = [&](int64_t mk, uint4 (&ry)[CH], uint4 (&rx)[CH]) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int q = tid + i * kThreads;
      const int p = q / CPRW, c = (q % CPRW) * EPC;
      const int64_t m = mk + p;
      ry[i] = make_uint4(0, 0, 0, 0);
      rx[i] = make_uint4(0, 0, 0, 0);
      if (m < mend) {
        if (co0 + c < g.Co)
          ry[i] = *reinterpret_cast<const uint4*>(dy + m * g.yCs + co0 + c);
        int64_t mm = m;
        const int w = (int)(mm % g.Wo); mm /= g.Wo;
        const int h = (int)(mm % g.Ho); mm /= g.Ho;
        const int t = (int)(mm % g.To);
        const int b = (int)(mm / g.To);
        const int s_t = t * g.st - g.pt + ta, s_h = h * g.sh - g.ph + tb, s_w = w * g.sw - g.pw + tc;
        if ((unsigned)s_t < (unsigned)g.Ti && (unsigned)s_h < (unsigned)g.Hi &&
            (unsigned)s_w < (unsigned)g.Wi && ci0 + c < g.Ci) {
          const int64_t pix = (((int64_t)b * g.Ti + s_t) * g.Hi + s_h) * g.Wi + s_w;
          rx[i] = *reinterpret_cast<const uint4*>(x + pix * g.xCs + ci0 + c);
        }
      }
    }
  };
  auto store = [&](int stage, const uint4 (&ry)[CH], const uint4 (&rx)[CH]) {
    T* Ys = lds + stage * STAGE;
    T* Xs = Ys + PK * LD;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int q = tid + i * kThreads;
      const int p = q / CPRW, c = (q % CPRW) * EPC;
      *reinterpret_cast<uint4*>(Ys + p * LD + c) = ry[i];
      *reinterpret_cast<uint4*>(Xs + p * LD + c) = rx[i];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = (int)((mend - mbeg + PK - 1) / PK);
  uint4 ry[CH], rx[CH];
  load(mbeg, ry, rx);
  store(0, ry, rx);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int s = 0; s < nsteps; ++s) {
    const bool more = s + 1 < nsteps;
    if (more) load(mbeg + (int64_t)(s + 1) * PK, ry, rx);
    const T* Ys = lds + (s & 1) * STAGE;
    const T* Xs = Ys + PK * LD;
    if constexpr (sizeof(T) == 2) {
      // A[co][k=px] and B[k=px][ci] from [px][ch] tiles via transposed reads:
      // group lane 4q+p reads row (8*fq + q [+4]), cols c0 + 4p .. +3
      const int q4 = fr >> 2, p4 = fr & 3;
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c0 = wm * 32 + 16 * i;
        const T* base = Ys + (8 * fq + q4) * LD + c0 + 4 * p4;
        bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base));
        bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base + 4 * LD));
        af[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c0 = wn * 32 + 16 * j;
        const T* base = Xs + (8 * fq + q4) * LD + c0 + 4 * p4;
        bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base));
        bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base + 4 * LD));
        bfr[j] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int kk = 0; kk < PK / 4; ++kk) {
        const int p = 4 * kk + fq;
        float af[2], bfv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = Ys[p * LD + wm * 32 + 16 * i + fr];
#pragma unroll
        for (int j = 0; j < 2; ++j) bfv[j] = Xs[p * LD + wn * 32 + 16 * j + fr];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfv[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) store((s + 1) & 1, ry, rx);
    __syncthreads();
  }
  const int64_t krow = (int64_t)taps * g.Ci;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ci = ci0 + wn * 32 + 16 * j + fr;
      if (ci >= g.Ci) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * 32 + 16 * i + fq * 4 + r;
        if (co < g.Co) wg_out(g, dw, blockIdx.y, (int64_t)co * krow + (int64_t)tap * g.Ci + ci, acc[i][j][r]);
      }
    }
}

// ----------------------------------------------------------------- bf16 implicit GEMM, tap-outer
// bf16 fwd / bwd-data.  K is walked tap-major: for each of the kt*kh*kw taps the source
// pixel of every tile row is one add and three range checks away from a per-row base
// computed once per workgroup (no per-step integer division), then the tap's channels
// go in 64-wide K steps (two 16x16x32 MFMA k-slices per LDS stage, one barrier per step).
// Tile BM x BN, 4 waves laid out WAVES_M x (4 / WAVES_M), wave tile (BM / WAVES_M) x
// (BN * WAVES_M / 4).  LDS rows are 128 B (64 bf16); chunk c of row r sits at
// c ^ ((r >> 1) & 7): a 16-lane group of a 16x16x32 fragment read (rows r0..r0+15, one
// chunk) then covers all 64 banks once, and the 8-lane groups of the 16-B stores write
// one row each.  Register-staged double buffer: the next step's global loads are in flight
// during this step's MFMAs.
constexpr int kIgBK = 64;
// VDIFF_CONV_LEGACY=1: the previous k-major kernel for bf16 too (A/B measurements)
// VDIFF_CONV_DMA=0: the register-staged tap-outer kernel instead of the LDS-DMA ring
const bool g_conv_dma = [] {
  const char* e = getenv("VDIFF_CONV_DMA");
  return !(e && e[0] == '0');
}();
const bool g_legacy_conv = [] {
  const char* e = getenv("VDIFF_CONV_LEGACY");
  return e && e[0] == '1';
}();

__device__ __forceinline__ int ig_off(int r, int c) {  // element offset of chunk c, row r
  return r * kIgBK + ((c ^ ((r >> 1) & 7)) << 3);
}

template <int BM, int BN, int WAVES_M, bool TR>
__global__ __launch_bounds__(kThreads, 2) void igemm_bf16_kernel(
    GemmGeom g, const bf16_t* __restrict__ src, const bf16_t* __restrict__ wt,
    bf16_t* __restrict__ dst, const float* __restrict__ bias, const float* __restrict__ chan_add,
    const bf16_t* __restrict__ residual) {
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int NI = WTM / 16, NJ = WTN / 16;
  constexpr int RA = BM / 32, RB = BN / 32;  // 16-B chunks per thread per stage
  constexpr int A_ELEMS = BM * kIgBK, B_ELEMS = BN * kIgBK, STAGE = A_ELEMS + B_ELEMS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WAVES_M, wn = wave / WAVES_M;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int ch = tid & 7;   // 16-B chunk of the 64-wide K step this thread stages
  const int rr = tid >> 3;  // first staged row (then + 32 i)
  const int C = g.sC;
  const int taps = g.kt * g.kh * g.kw;
  const bool unit = g.st == 1 && g.sh == 1 && g.sw == 1;

  // per staged A row: base source coordinates and the pixel index at tap (0, 0, 0)
  int a_t[RA], a_h[RA], a_w[RA];
  int64_t a_pix[RA];
#pragma unroll
  for (int i = 0; i < RA; ++i) {
    int64_t m = m0 + rr + 32 * i;
    const bool ok = m < g.M;
    if (!ok) m = 0;
    const int w = (int)(m % g.dW); m /= g.dW;
    const int h = (int)(m % g.dH); m /= g.dH;
    const int t = (int)(m % g.dT);
    const int b = (int)(m / g.dT);
    if (!TR) {
      a_t[i] = t * g.st - g.pt; a_h[i] = h * g.sh - g.ph; a_w[i] = w * g.sw - g.pw;
    } else {  // dY row of input pixel (t, h, w) at tap (a, b, c): (t + pt - a) / st, ...
      a_t[i] = t + g.pt; a_h[i] = h + g.ph; a_w[i] = w + g.pw;
    }
    if (!ok) a_t[i] = -(1 << 28);  // never in range
    a_pix[i] = (int64_t)b * g.sT * g.sH * g.sW;
  }

  auto load = [&](int tap, int c0, uint4 (&ra)[RA], uint4 (&rb)[RB]) {
    const int ta = tap / (g.kh * g.kw), rem = tap - ta * (g.kh * g.kw);
    const int tb = rem / g.kw, tc = rem - tb * g.kw;
    const int c = c0 + ch * 8;
    const bool cin = c < C;
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      int st_, sh_, sw_;
      bool ok = cin;
      if (!TR) {
        st_ = a_t[i] + ta; sh_ = a_h[i] + tb; sw_ = a_w[i] + tc;
      } else if (unit) {
        st_ = a_t[i] - ta; sh_ = a_h[i] - tb; sw_ = a_w[i] - tc;
      } else {
        const int nt = a_t[i] - ta, nh = a_h[i] - tb, nw = a_w[i] - tc;
        ok = ok && nt >= 0 && nh >= 0 && nw >= 0 && nt % g.st == 0 && nh % g.sh == 0 &&
             nw % g.sw == 0;
        st_ = nt / g.st; sh_ = nh / g.sh; sw_ = nw / g.sw;
      }
      ok = ok && (unsigned)st_ < (unsigned)g.sT && (unsigned)sh_ < (unsigned)g.sH &&
           (unsigned)sw_ < (unsigned)g.sW;
      const int64_t pix = a_pix[i] + ((int64_t)st_ * g.sH + sh_) * g.sW + sw_;
      ra[i] = ok ? *reinterpret_cast<const uint4*>(src + pix * g.sCs + c) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int n = n0 + rr + 32 * i;
      rb[i] = (n < g.N && cin)
                  ? *reinterpret_cast<const uint4*>(wt + (int64_t)n * g.K + (int64_t)tap * C + c)
                  : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&](int stage, const uint4 (&ra)[RA], const uint4 (&rb)[RB]) {
    bf16_t* As = lds + stage * STAGE;
    bf16_t* Bs = As + A_ELEMS;
#pragma unroll
    for (int i = 0; i < RA; ++i) *reinterpret_cast<uint4*>(As + ig_off(rr + 32 * i, ch)) = ra[i];
#pragma unroll
    for (int i = 0; i < RB; ++i) *reinterpret_cast<uint4*>(Bs + ig_off(rr + 32 * i, ch)) = rb[i];
  };

  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int csteps = (C + kIgBK - 1) / kIgBK;
  const int nk = taps * csteps;
  uint4 ra[RA], rb[RB];
  load(0, 0, ra, rb);
  store(0, ra, rb);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  int tap = 0, cs = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (++cs == csteps) {
      cs = 0;
      ++tap;
    }
    if (more) load(tap, cs * kIgBK, ra, rb);
    const bf16_t* As = lds + (kt & 1) * STAGE;
    const bf16_t* Bs = As + A_ELEMS;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[NI], bfr[NJ];
#pragma unroll
      for (int i = 0; i < NI; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(As + ig_off(wm * WTM + 16 * i + fr, 4 * s + fq));
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + ig_off(wn * WTN + 16 * j + fr, 4 * s + fq));
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) store((kt + 1) & 1, ra, rb);
    __syncthreads();
  }

  // ---- epilogue: the fp32 tile through LDS, then coalesced 16-B stores
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int LDC = BN + 4;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * WTM + 16 * i + fq * 4 + r) * LDC + wn * WTN + 16 * j + fr] = acc[i][j][r];
  __syncthreads();
  const int64_t pix_per_b = (int64_t)g.dT * g.dH * g.dW;
  const bool vec = (g.N % 8 == 0) && (g.dNs % 8 == 0);
  for (int v = tid; v < BM * BN / 8; v += kThreads) {
    const int r = v / (BN / 8), c = (v % (BN / 8)) * 8;
    const int64_t m = m0 + r;
    const int n = n0 + c;
    if (m >= g.M || n >= g.N) continue;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = Cs[r * LDC + c + e];
    const int lim = g.N - n < 8 ? g.N - n : 8;
    if (bias)
      for (int e = 0; e < lim; ++e) o[e] += bias[n + e];
    if (chan_add) {
      const int bidx = (int)(m / pix_per_b);  // 64-bit division only where it is needed
      for (int e = 0; e < lim; ++e) o[e] += chan_add[(int64_t)bidx * g.N + n + e];
    }
    bf16_t* out = dst + m * g.dNs + n;
    if (vec) {
      if (residual) {
        float rv[8];
        load8(residual + m * g.dNs + n, rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += rv[e];
      }
      store8(out, o);
    } else {
      for (int e = 0; e < lim; ++e) {
        float val = o[e];
        if (residual) val += bf2f(residual[m * g.dNs + n + e]);
        out[e] = f2bf(val);
      }
    }
  }
}

template <int BM, int BN, int WM, bool TR>
void launch_ig(const GemmGeom& g, const void* src, const void* wt, void* dst, const float* bias,
               const float* ca, const void* res, hipStream_t st) {
  const size_t lds_ab = 2 * (size_t)(BM + BN) * kIgBK * 2;
  const size_t lds_c = (size_t)BM * (BN + 4) * 4;
  const size_t lds = lds_ab > lds_c ? lds_ab : lds_c;
  auto kern = igemm_bf16_kernel<BM, BN, WM, TR>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  dim3 grid((unsigned)vd_cdiv(g.M, BM), (unsigned)vd_cdiv(g.N, BN));
  kern<<<grid, kThreads, lds, st>>>(g, (const bf16_t*)src, (const bf16_t*)wt, (bf16_t*)dst, bias,
                                    ca, (const bf16_t*)res);
}

// Tile choice: N <= 64 -> 256 x 64 (4 waves along M); otherwise 128 x 128, or 64 x 128 when
// 128 x 128 tiles would leave the chip with fewer than two workgroups per CU.
template <bool TR>
int launch_igemm(const GemmGeom& g, const void* src, const void* wt, void* dst, const float* bias,
                 const float* ca, const void* res, hipStream_t st) {
  if (g.N <= 64) {
    launch_ig<256, 64, 4, TR>(g, src, wt, dst, bias, ca, res, st);
  } else if (vd_cdiv(g.M, 128) * vd_cdiv(g.N, 128) < 512) {
    launch_ig<64, 128, 2, TR>(g, src, wt, dst, bias, ca, res, st);
  } else {
    launch_ig<128, 128, 2, TR>(g, src, wt, dst, bias, ca, res, st);
  }
  return VD_OK;
}

// ----------------------------------------------------------------- bf16 weight gradient, kw-strip
// dW[co][tap][ci] += sum_m dY[m][co] X[src(m, tap)][ci] for stride-1 "same" 3x3(x3) convs.
// A workgroup owns a 64 (co) x 64 (ci) tile for the three taps of one kernel row
// (ta, tb, tc = 0..2) and a contiguous pixel range, in 64-pixel K steps.  A step's pixels
// are R = 64 / Wc image rows of Wc = min(Wo, 64) pixels; the three taps read the SAME
// dY tile and one X strip of Wc + 2 pixels per row, shifted by tc rows in LDS -- 3x fewer
// operand loads than one tap per workgroup.  Both operands are read transposed from
// [pixel][channel] LDS rows (ds_read_b64_tr_b16; each lane addresses its own row, so the
// shifted windows cost nothing).  Pixel coordinates advance incrementally (no division in
// the loop); the fp32 result is added into dW with atomics (split-K over pixels).
template <int RW>  // R x (Wc + 2) strip rows, padded to a multiple of 32
__global__ __launch_bounds__(kThreads, 2) void wgrad_bf16_kernel(
    WgtGeom g, int wc, const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
    float* __restrict__ dw) {
  constexpr int LD = 72;              // LDS row: 64 channels + 8 pad (144 B)
  constexpr int YROWS = 64, XROWS = RW;
  constexpr int STAGE = (YROWS + XROWS) * LD;
  constexpr int XCH = XROWS * 8 / kThreads;  // X chunks per thread
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);

  const int co_tiles = (g.Co + 63) / 64, ci_tiles = (g.Ci + 63) / 64;
  int bid = blockIdx.x;
  const int cot = bid % co_tiles; bid /= co_tiles;
  const int cit = bid % ci_tiles; bid /= ci_tiles;
  const int tab = bid;                      // ta * kh + tb
  const int ta = tab / g.kh, tb = tab % g.kh;
  const int co0 = cot * 64, ci0 = cit * 64;
  const int64_t mbeg = (int64_t)blockIdx.y * g.m_per_split;
  int64_t mend = mbeg + g.m_per_split;
  if (mend > g.M) mend = g.M;
  if (mbeg >= mend) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ch = tid & 7, r0 = tid >> 3;
  const int R = 64 / wc, SW = wc + 2;       // rows per step, strip width
  // this thread's strip rows: row-in-step rr and strip column j (pixel w0 + j - 1)
  int x_rr[XCH], x_j[XCH];
#pragma unroll
  for (int i = 0; i < XCH; ++i) {
    const int sr = r0 + 32 * i;
    x_rr[i] = sr / SW;
    x_j[i] = sr - x_rr[i] * SW;
    if (x_rr[i] >= R) x_rr[i] = -1;  // padding row: zero
  }
  // coordinates of the first pixel of the current step (incremental)
  int cb, ct, chh, cw;
  {
    int64_t m = mbeg;
    cw = (int)(m % g.Wo); m /= g.Wo;
    chh = (int)(m % g.Ho); m /= g.Ho;
    ct = (int)(m % g.To);
    cb = (int)(m / g.To);
  }
  auto advance = [&]() {  // by 64 pixels
    cw += 64;
    while (cw >= g.Wo) {
      cw -= g.Wo;
      if (++chh == g.Ho) {
        chh = 0;
        if (++ct == g.To) {
          ct = 0;
          ++cb;
        }
      }
    }
  };

  auto load = [&](int64_t ms, uint4 (&ry)[2], uint4 (&rx)[XCH]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t m = ms + r0 + 32 * i;
      ry[i] = (m < mend && co0 + ch * 8 < g.Co)
                  ? *reinterpret_cast<const uint4*>(dy + m * g.yCs + co0 + ch * 8)
                  : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      rx[i] = make_uint4(0, 0, 0, 0);
      if (x_rr[i] < 0 || ci0 + ch * 8 >= g.Ci) continue;
      // image row x_rr of this step: (cb, ct, chh + x_rr) with carry; w from cw
      int b = cb, t = ct, h = chh + x_rr[i];
      while (h >= g.Ho) {
        h -= g.Ho;
        if (++t == g.To) {
          t = 0;
          ++b;
        }
      }
      const int ti = t - g.pt + ta, hi = h - g.ph + tb, wi = cw + x_j[i] - g.pw;
      if (b < g.B && (unsigned)ti < (unsigned)g.Ti && (unsigned)hi < (unsigned)g.Hi &&
          (unsigned)wi < (unsigned)g.Wi) {
        const int64_t pix = (((int64_t)b * g.Ti + ti) * g.Hi + hi) * g.Wi + wi;
        rx[i] = *reinterpret_cast<const uint4*>(x + pix * g.xCs + ci0 + ch * 8);
      }
    }
  };
  auto store = [&](int stage, const uint4 (&ry)[2], const uint4 (&rx)[XCH]) {
    bf16_t* Ys = lds + stage * STAGE;
    bf16_t* Xs = Ys + YROWS * LD;
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<uint4*>(Ys + (r0 + 32 * i) * LD + ch * 8) = ry[i];
#pragma unroll
    for (int i = 0; i < XCH; ++i) *reinterpret_cast<uint4*>(Xs + (r0 + 32 * i) * LD + ch * 8) = rx[i];
  };

  // wave tile: co [32 wm, +32) x ci [32 wn, +32) x 3 taps
  const int wm = wave & 1, wn = wave >> 1;
  f32x4 acc[3][2][2];
#pragma unroll
  for (int tc = 0; tc < 3; ++tc)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[tc][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = (int)((mend - mbeg + 63) / 64);
  uint4 ry[2], rx[XCH];
  load(mbeg, ry, rx);
  store(0, ry, rx);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4, q4 = fr >> 2, p4 = fr & 3;
  for (int s = 0; s < nsteps; ++s) {
    const bool more = s + 1 < nsteps;
    if (more) {
      advance();
      load(mbeg + (int64_t)(s + 1) * 64, ry, rx);
    }
    const bf16_t* Ys = lds + (s & 1) * STAGE;
    const bf16_t* Xs = Ys + YROWS * LD;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // lane group fq covers pixels p = 32 ks + 8 fq + (0..7); block row q4 (+4)
      const int p_lo = 32 * ks + 8 * fq + q4, p_hi = p_lo + 4;
      bf16x8 af[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c0 = wm * 32 + 16 * i + 4 * p4;
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(Ys + p_lo * LD + c0));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(Ys + p_hi * LD + c0));
        af[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      // strip row of pixel p at tap tc: (p / wc) * (wc + 2) + p % wc + tc
      const int s_lo = (p_lo / wc) * SW + p_lo % wc, s_hi = (p_hi / wc) * SW + p_hi % wc;
#pragma unroll
      for (int tc = 0; tc < 3; ++tc) {
        bf16x8 bfr[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c0 = wn * 32 + 16 * j + 4 * p4;
          const bf16x4 lo =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(Xs + (s_lo + tc) * LD + c0));
          const bf16x4 hi =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(Xs + (s_hi + tc) * LD + c0));
          bfr[j] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[tc][i][j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[tc][i][j], 0, 0, 0);
      }
    }
    if (more) store((s + 1) & 1, ry, rx);
    __syncthreads();
  }
  const int taps = g.kt * g.kh * g.kw;
  const int64_t krow = (int64_t)taps * g.Ci;
#pragma unroll
  for (int tc = 0; tc < 3; ++tc) {
    const int tap = tab * g.kw + tc;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ci = ci0 + wn * 32 + 16 * j + fr;
        if (ci >= g.Ci) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = co0 + wm * 32 + 16 * i + fq * 4 + r;
          if (co < g.Co) wg_out(g, dw, blockIdx.y, (int64_t)co * krow + (int64_t)tap * g.Ci + ci, acc[tc][i][j][r]);
        }
      }
  }
}

// ----------------------------------------------------------- bf16 weight gradient, kw-strip, DMA
// wgrad_bf16_kernel's tiling (three kw taps share one dY tile and one X strip) with the
// operands staged global -> LDS by buffer_load ... lds into an NST-stage ring, as
// igemm_dma_kernel: the register-staged version spent more LDS cycles on ds_write_b128 than
// on the transposed reads the MFMAs need.  LDS rows are 128 B (64 channels) unpadded; the
// 16-B chunk c of row r sits at c ^ wg_swz(r), which keeps the ds_read_b64_tr_b16 pattern
// (rows b..b+3 and b+8..b+11 in one 32-lane group, for any b) free of bank conflicts.
// COT output channels per workgroup (64 or 128, split in COT / 64 planes of 64 rows).
__device__ __forceinline__ int wg_swz(int r) {
  const int u = r >> 1;
  return ((u + 2 * (u >> 2)) & 3) << 1;
}
__device__ __forceinline__ int wg_off(int r, int c) {  // element offset of channel c, row r
  return r * 64 + ((((c >> 3) ^ wg_swz(r)) << 3) | (c & 7));
}

// PLANE (round 2): all nine (kh, kw) taps of one kt per workgroup -- the X strip holds the
// three input rows above / at / below the step's 64-pixel output row (W % 64 == 0, so a step
// is one row segment), and one dY tile feeds nine taps instead of three.
//
template <int RW, int COT, int NST, bool ONE, bool PLANE = false>  // ONE: 1x1 stride-1 unpadded conv, X rows = dY rows
__global__ __launch_bounds__(kThreads, PLANE ? 1 : 2) void wgrad_dma_kernel(
    WgtGeom g, int wc, const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
    float* __restrict__ dw) {
  constexpr int PY = COT / 32, PX = RW / 32;  // pieces per wave per step
  constexpr int PIECES = PY + PX;
  constexpr int Y_BYTES = COT * 128, STAGE = (COT + RW) * 128;
  constexpr int WTM = COT / 2, NI = WTM / 16;
  constexpr int NT = ONE ? 1 : (PLANE ? 9 : 3);  // taps per workgroup
  static_assert(!PLANE || RW >= 3 * 66, "plane: three strip rows of 66 pixels");
  static_assert(!ONE || RW == 64, "1x1: the X tile is the step's 64 pixels");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const bf16_t* lds = reinterpret_cast<const bf16_t*>(smem);

  const int co_tiles = (g.Co + COT - 1) / COT, ci_tiles = (g.Ci + 63) / 64;
  int bid, wsplit;
  if (!wg_tile(g, &bid, &wsplit)) return;  // padding of the XCD-aware grid
  const int cot = bid % co_tiles; bid /= co_tiles;
  const int cit = bid % ci_tiles; bid /= ci_tiles;
  const int tab = bid;  // PLANE: kt index; otherwise (kt, kh) index
  const int ta = PLANE ? tab : tab / g.kh, tb = PLANE ? 0 : tab % g.kh;
  const int co0 = cot * COT, ci0 = cit * 64;
  const int64_t mbeg = (int64_t)wsplit * g.m_per_split;
  int64_t mend = mbeg + g.m_per_split;
  if (mend > g.M) mend = g.M;
  if (mbeg >= mend) return;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane >> 3, pc = lane & 7;
  const int R = 64 / wc, SW = wc + 2;
  // dY pieces: plane (wave * PY + i) / 8, pixel row ((wave * PY + i) % 8) * 8 + lr
  int y_p[PY], y_col[PY];
#pragma unroll
  for (int i = 0; i < PY; ++i) {
    const int pi = wave * PY + i;
    const int p = (pi & 7) * 8 + lr;
    const int c = pc ^ wg_swz(p);
    y_p[i] = p;
    y_col[i] = co0 + (pi >> 3) * 64 + c * 8;
  }
  // X pieces: strip row sr -> step row rr and strip column j (pixel w0 + j - 1)
  int x_rr[PX], x_j[PX], x_col[PX];
#pragma unroll
  for (int i = 0; i < PX; ++i) {
    const int sr = (wave * PX + i) * 8 + lr;
    if (ONE) {
      x_rr[i] = 0;
      x_j[i] = sr;
      x_col[i] = ci0 + (pc ^ wg_swz(sr)) * 8;
      continue;
    }
    x_rr[i] = sr / SW;
    x_j[i] = sr - x_rr[i] * SW;
    if (x_rr[i] >= (PLANE ? 3 : R)) x_rr[i] = -1;
    x_col[i] = ci0 + (pc ^ wg_swz(sr)) * 8;
  }
  const rsrc_t rs_y = make_rsrc(dy, (uint32_t)(g.M * g.yCs * 2));
  const rsrc_t rs_x = make_rsrc(x, (uint32_t)((int64_t)g.B * g.Ti * g.Hi * g.Wi * g.xCs * 2));

  // first pixel of the step being issued (incremental)
  int cb, ct, chh, cw;
  {
    int64_t m = mbeg;
    cw = (int)(m % g.Wo); m /= g.Wo;
    chh = (int)(m % g.Ho); m /= g.Ho;
    ct = (int)(m % g.To);
    cb = (int)(m / g.To);
  }
  const int nsteps = (int)((mend - mbeg + 63) / 64);
  auto issue = [&](int s) {
    char* st = smem + (s % NST) * STAGE;
    const bool live = s < nsteps;
    // 32-bit offsets: the launcher takes this kernel only when dY and X span < 2 GiB
    const int ms = (int)mbeg + s * 64, me = (int)mend;
#pragma unroll
    for (int i = 0; i < PY; ++i) {
      const bool ok = live & (ms + y_p[i] < me) & (y_col[i] < g.Co);
      dma_lds<16>(rs_y, lds_addr(st + (wave * PY + i) * 1024),
                  ok ? (uint32_t)(((ms + y_p[i]) * g.yCs + y_col[i]) * 2) : 0x80000000u);
    }
#pragma unroll
    for (int i = 0; i < PX; ++i) {
      uint32_t off = 0x80000000u;
      if (ONE) {
        if (live & (ms + x_j[i] < me) & (x_col[i] < g.Ci))
          off = (uint32_t)(((ms + x_j[i]) * g.xCs + x_col[i]) * 2);
      } else if (PLANE) {  // strip row r: input row chh - 1 + r of the step's own frame
        const int ti = ct - g.pt + ta, hi = chh - 1 + x_rr[i], wi = cw + x_j[i] - g.pw;
        if (live & (x_rr[i] >= 0) & (x_col[i] < g.Ci) & ((unsigned)ti < (unsigned)g.Ti) &
            ((unsigned)hi < (unsigned)g.Hi) & ((unsigned)wi < (unsigned)g.Wi)) {
          const int pix = ((cb * g.Ti + ti) * g.Hi + hi) * g.Wi + wi;
          off = (uint32_t)((pix * g.xCs + x_col[i]) * 2);
        }
      } else if (live & (x_rr[i] >= 0) & (x_col[i] < g.Ci)) {
        int b = cb, t = ct, h = chh + x_rr[i];
        while (h >= g.Ho) {
          h -= g.Ho;
          if (++t == g.To) {
            t = 0;
            ++b;
          }
        }
        const int ti = t - g.pt + ta, hi = h - g.ph + tb, wi = cw + x_j[i] - g.pw;
        if (b < g.B && (unsigned)ti < (unsigned)g.Ti && (unsigned)hi < (unsigned)g.Hi &&
            (unsigned)wi < (unsigned)g.Wi) {
          const int pix = ((b * g.Ti + ti) * g.Hi + hi) * g.Wi + wi;
          off = (uint32_t)((pix * g.xCs + x_col[i]) * 2);
        }
      }
      dma_lds<16>(rs_x, lds_addr(st + Y_BYTES + (wave * PX + i) * 1024), off);
    }
    if (!ONE && live) {  // advance by 64 pixels
      cw += 64;
      while (cw >= g.Wo) {
        cw -= g.Wo;
        if (++chh == g.Ho) {
          chh = 0;
          if (++ct == g.To) {
            ct = 0;
            ++cb;
          }
        }
      }
    }
  };

  // wave tile: co [WTM wm, +WTM) x ci [32 wn, +32) x 3 taps
  const int wm = wave & 1, wn = wave >> 1;
  f32x4 acc[NT][NI][2];
#pragma unroll
  for (int tc = 0; tc < NT; ++tc)
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[tc][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  vm_drain();
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue(s);
  const int fr = lane & 15, fq = lane >> 4, q4 = fr >> 2, p4 = fr & 3;
  for (int s = 0; s < nsteps; ++s) {
    vm_wait_barrier<(NST - 2) * PIECES>();
    issue(s + NST - 1);
    const bf16_t* Ys = lds + (s % NST) * (STAGE / 2);
    const bf16_t* Xs = Ys + Y_BYTES / 2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int p_lo = 32 * ks + 8 * fq + q4, p_hi = p_lo + 4;
      bf16x8 af[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int c = wm * WTM + 16 * i + 4 * p4;
        const bf16_t* plane = Ys + (c >> 6) * 4096;
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_bf16x4*)(plane + wg_off(p_lo, c & 63)));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_bf16x4*)(plane + wg_off(p_hi, c & 63)));
        af[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      const int s_lo = ONE ? p_lo : (p_lo / wc) * SW + p_lo % wc;
      const int s_hi = ONE ? p_hi : (p_hi / wc) * SW + p_hi % wc;
#pragma unroll
      for (int tc = 0; tc < NT; ++tc) {
        bf16x8 bfr[2];
        const int sh_t = PLANE ? (tc / 3) * SW + tc % 3 : tc;  // strip shift of the tap
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c = wn * 32 + 16 * j + 4 * p4;
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_bf16x4*)(Xs + wg_off(s_lo + sh_t, c)));
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_bf16x4*)(Xs + wg_off(s_hi + sh_t, c)));
          bfr[j] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[tc][i][j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[tc][i][j], 0, 0, 0);
      }
    }
  }
  vm_drain();
  const int taps = g.kt * g.kh * g.kw;
  const int64_t krow = (int64_t)taps * g.Ci;
#pragma unroll
  for (int tc = 0; tc < NT; ++tc) {
    const int tap = ONE ? 0 : (PLANE ? ta * 9 + tc : tab * g.kw + tc);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ci = ci0 + wn * 32 + 16 * j + fr;
        if (ci >= g.Ci) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = co0 + wm * WTM + 16 * i + fq * 4 + r;
          if (co < g.Co) wg_out(g, dw, wsplit, (int64_t)co * krow + (int64_t)tap * g.Ci + ci, acc[tc][i][j][r]);
        }
      }
  }
}

// ---- round 6: the kw-strip weight gradient with its step loop unrolled by the ring depth.
// wgrad_dma_kernel spent ~150 VALU and ~60 SALU instructions per 24-MFMA step (SQ_INSTS_VALU
// 7380 per wave, 64->64 at 16x128x128): every transposed fragment read recomputed its
// swizzled address from the runtime ring stage, and the X strip's source pixels were found by
// divergent wrap loops.  Here the ring stage is a compile-time constant (the loop body is
// unrolled NST times), so every ds_read_b64_tr_b16 is a precomputed per-lane base plus an
// immediate, and an X piece's source pixel is the step's first pixel plus a per-lane constant
// (same-size stride-1 conv: pixel = m + (kt - pt) H W + (kh - ph) W + row * wc + j - pw) with a
// branch-free bounds test.  Same tiles, DMA pieces and summation order as wgrad_dma_kernel.
// KIND 0: kw strip, a step is R = 64 / Wo whole image rows; 1: kw strip, a step is one 64-pixel
// row segment (W % 64 == 0); 2: 1x1 stride-1 unpadded conv (X rows = dY rows, one tap).
template <int RW, int COT, int NST, int KIND, bool ER = true>
__global__ __launch_bounds__(kThreads, 2) void wgrad_strip_kernel(WgtGeom g, int wc,
                                                                  const bf16_t* __restrict__ x,
                                                                  const bf16_t* __restrict__ dy,
                                                                  float* __restrict__ dw) {
  constexpr int PY = COT / 32, PX = RW / 32;  // pieces per wave per step
  constexpr int PIECES = PY + PX;
  constexpr int Y_BYTES = COT * 128, STAGE = (COT + RW) * 128;
  constexpr bool ROW1 = KIND == 1, ONE = KIND == 2;
  constexpr int WTM = COT / 2, NI = WTM / 16, NT = ONE ? 1 : 3;
  static_assert(!ONE || RW == 64, "1x1: the X tile is the step's 64 pixels");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int co_tiles = (g.Co + COT - 1) / COT, ci_tiles = (g.Ci + 63) / 64;
  int bid, wsplit;
  if (!wg_tile(g, &bid, &wsplit)) return;  // padding of the XCD-aware grid
  const int cot = bid % co_tiles; bid /= co_tiles;
  const int cit = bid % ci_tiles; bid /= ci_tiles;
  const int tab = bid;  // (kt, kh) index
  const int ta = tab / g.kh, tb = tab % g.kh;
  const int co0 = cot * COT, ci0 = cit * 64;
  const int64_t mbeg = (int64_t)wsplit * g.m_per_split;
  int64_t mend = mbeg + g.m_per_split;
  if (mend > g.M) mend = g.M;
  if (mbeg >= mend) return;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane >> 3, pc = lane & 7;
  const int R = 64 / wc, SW = wc + 2;
  const int HWi = g.Hi * g.Wi;
  const int delta = (ta - g.pt) * HWi + (tb - g.ph) * g.Wi;  // source pixel of output pixel 0
  int y_off[PY];
  bool y_ok[PY];
#pragma unroll
  for (int i = 0; i < PY; ++i) {
    const int pi = wave * PY + i;
    const int p = (pi & 7) * 8 + lr;
    const int c = pc ^ wg_swz(p);
    const int col = co0 + (pi >> 3) * 64 + c * 8;
    y_ok[i] = col < g.Co;
    y_off[i] = (p * g.yCs + col) * 2;  // + step pixel * yCs * 2
  }
  // X pieces: strip row sr -> step row rr and strip column j (pixel w0 + j - pw)
  int x_rr[PX], x_j[PX], x_off[PX];
  bool x_ok[PX];
#pragma unroll
  for (int i = 0; i < PX; ++i) {
    const int sr = (wave * PX + i) * 8 + lr;
    const int col = ci0 + (pc ^ wg_swz(sr)) * 8;
    if constexpr (ONE) {  // X row sr = the step's pixel sr
      x_rr[i] = 0;
      x_j[i] = sr;
      x_ok[i] = col < g.Ci;
      x_off[i] = (sr * g.xCs + col) * 2;
      continue;
    }
    const int rr = sr / SW, j = sr - rr * SW;
    x_rr[i] = rr;
    x_j[i] = j - g.pw;
    x_ok[i] = rr < R && col < g.Ci && (ROW1 || (unsigned)(j - g.pw) < (unsigned)g.Wi);
    x_off[i] = ((delta + rr * wc + j - g.pw) * g.xCs + col) * 2;  // + step pixel * xCs * 2
  }
  const rsrc_t rs_y = make_rsrc(dy, (uint32_t)(g.M * g.yCs * 2));
  const rsrc_t rs_x = make_rsrc(x, (uint32_t)((int64_t)g.B * g.Ti * g.Hi * g.Wi * g.xCs * 2));

  // first pixel of the step being issued (incremental): w, h, t of its first row
  int cw, chh, ct;
  {
    int64_t m = mbeg;
    cw = (int)(m % g.Wo); m /= g.Wo;
    chh = (int)(m % g.Ho); m /= g.Ho;
    ct = (int)(m % g.To);
  }
  const int nsteps = (int)((mend - mbeg + 63) / 64);
  const int ms0 = (int)mbeg, me = (int)mend;
  auto issue = [&](int s, int stage) {
    char* st = smem + stage * STAGE;
    const bool live = s < nsteps;
    const int ms = ms0 + s * 64;
#pragma unroll
    for (int i = 0; i < PY; ++i) {
      // (kw strips: M and every split bound are multiples of 64, so only 1x1 steps run short)
      const bool ok = live & y_ok[i] & (!ONE || ms + ((wave * PY + i) & 7) * 8 + lr < me);
      dma_lds<16>(rs_y, lds_addr(st + (wave * PY + i) * 1024),
                  ok ? (uint32_t)(y_off[i] + ms * g.yCs * 2) : 0x80000000u);
    }
    if constexpr (ONE) {
#pragma unroll
      for (int i = 0; i < PX; ++i) {
        const bool ok = live & x_ok[i] & (ms + x_j[i] < me);
        dma_lds<16>(rs_x, lds_addr(st + Y_BYTES + (wave * PX + i) * 1024),
                    ok ? (uint32_t)(x_off[i] + ms * g.xCs * 2) : 0x80000000u);
      }
      return;
    } else if constexpr (ROW1) {  // every strip row is the step's own output row: (ct, chh) uniform
      const int ti = ct + ta - g.pt, hi = chh + tb - g.ph;
      const bool row_ok = live & (ms < me) & ((unsigned)ti < (unsigned)g.Ti) &
                          ((unsigned)hi < (unsigned)g.Hi);
#pragma unroll
      for (int i = 0; i < PX; ++i) {
        const int wi = cw + x_j[i];
        const bool ok = row_ok & x_ok[i] & ((unsigned)wi < (unsigned)g.Wi);
        dma_lds<16>(rs_x, lds_addr(st + Y_BYTES + (wave * PX + i) * 1024),
                    ok ? (uint32_t)(x_off[i] + ms * g.xCs * 2) : 0x80000000u);
      }
    } else {
      // R = 64 / Wo whole rows per step, all of one frame (the launcher takes this kind only
      // when Ho % R == 0, so a 64-aligned step never crosses a frame): (ct, chh) is the step's
      // first row, and a lane's strip row rr reads input row chh + rr + kh - ph of frame
      // ct + kt - pt (its column range test is loop-invariant, in x_ok)
      const int ti = ct + ta - g.pt, h0 = chh + tb - g.ph;
      const bool t_ok = live & ((unsigned)ti < (unsigned)g.Ti);
#pragma unroll
      for (int i = 0; i < PX; ++i) {
        const bool ok = t_ok & x_ok[i] & ((unsigned)(h0 + x_rr[i]) < (unsigned)g.Hi);
        dma_lds<16>(rs_x, lds_addr(st + Y_BYTES + (wave * PX + i) * 1024),
                    ok ? (uint32_t)(x_off[i] + ms * g.xCs * 2) : 0x80000000u);
      }
      if (live) {  // advance by R rows
        chh += R;
        if (chh >= g.Ho) {
          chh = 0;
          if (++ct == g.To) ct = 0;
        }
      }
      return;
    }
    if (live) {  // advance by 64 pixels (scalar; Wo % 64 == 0: at most one row wrap)
      cw += 64;
      if (cw >= g.Wo) {
        cw -= g.Wo;
        if (++chh == g.Ho) {
          chh = 0;
          if (++ct == g.To) ct = 0;
        }
      }
    }
  };

  // wave tile: co [WTM wm, +WTM) x ci [32 wn, +32) x 3 taps
  const int wm = wave & 1, wn = wave >> 1;
  f32x4 acc[NT][NI][2];
#pragma unroll
  for (int tc = 0; tc < NT; ++tc)
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[tc][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4, q4 = fr >> 2, p4 = fr & 3;
  // LDS byte addresses (stage 0) of every transposed fragment read (loop-invariant); a read of
  // stage u adds u * STAGE as the instruction's immediate offset
  const uint32_t lb = lds_addr(smem);
  uint32_t abase[2][2][NI], xbase[2][2][NT][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int hl = 0; hl < 2; ++hl) {
      const int p = 32 * ks + 8 * fq + q4 + 4 * hl;
      const int sp = ONE ? p : (p / wc) * SW + p % wc;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int c = wm * WTM + 16 * i + 4 * p4;
        abase[ks][hl][i] = lb + ((c >> 6) * 4096 + wg_off(p, c & 63)) * 2;
      }
#pragma unroll
      for (int tc = 0; tc < NT; ++tc)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          xbase[ks][hl][tc][j] = lb + Y_BYTES + wg_off(sp + tc, wn * 32 + 16 * j + 4 * p4) * 2;
    }

  vm_drain();
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue(s, s);
  for (int s0 = 0; s0 < nsteps; s0 += NST) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) {
#pragma unroll
        for (int i = 0; i < NI; ++i) asm volatile("" : "+v"(abase[ks][hl][i]));
#pragma unroll
        for (int tc = 0; tc < NT; ++tc)
#pragma unroll
          for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(xbase[ks][hl][tc][j]));
      }
#pragma unroll
    for (int u = 0; u < NST; ++u) {
      const int s = s0 + u;
      if (s >= nsteps) break;
      vm_lgk_wait_barrier<(NST - 2) * PIECES>();
      issue(s + NST - 1, (u + NST - 1) % NST);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[NI], bfr[NT][2];
        auto rd = [&](uint32_t a0, uint32_t a1) {
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_bf16x4*)(uintptr_t)(a0 + u * STAGE));
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_bf16x4*)(uintptr_t)(a1 + u * STAGE));
          return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        };
#pragma unroll
        for (int i = 0; i < NI; ++i) af[i] = rd(abase[ks][0][i], abase[ks][1][i]);
        if constexpr (ER) {
          // round 6: every fragment of this k-half read before its first MFMA (pinned by the
          // scheduling barrier), so one LDS latency is exposed per k-half instead of one per tap
#pragma unroll
          for (int tc = 0; tc < NT; ++tc)
#pragma unroll
            for (int j = 0; j < 2; ++j) bfr[tc][j] = rd(xbase[ks][0][tc][j], xbase[ks][1][tc][j]);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int tc = 0; tc < NT; ++tc) {
          if constexpr (!ER) {  // the compiler's placement (A/B: vd_conv_set_wgrad(2))
#pragma unroll
            for (int j = 0; j < 2; ++j) bfr[tc][j] = rd(xbase[ks][0][tc][j], xbase[ks][1][tc][j]);
          }
#pragma unroll
          for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[tc][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[tc][j],
                                                                      acc[tc][i][j], 0, 0, 0);
        }
      }
    }
  }
  vm_drain();
  const int taps = g.kt * g.kh * g.kw;
  const int64_t krow = (int64_t)taps * g.Ci;
#pragma unroll
  for (int tc = 0; tc < NT; ++tc) {
    const int tap = ONE ? 0 : tab * g.kw + tc;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ci = ci0 + wn * 32 + 16 * j + fr;
        if (ci >= g.Ci) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = co0 + wm * WTM + 16 * i + fq * 4 + r;
          if (co < g.Co)
            wg_out(g, dw, wsplit, (int64_t)co * krow + (int64_t)tap * g.Ci + ci,
                   acc[tc][i][j][r]);
        }
      }
  }
}

// ----------------------------------------------------------------- bf16 implicit GEMM, LDS-DMA ring
// Same GEMM and tap-major K walk as igemm_bf16_kernel, but the A rows (gathered pixels) and
// B rows (packed weights) go global -> LDS by buffer_load ... lds, in 1-KiB pieces of 8
// rows x 128 B, into an NST-stage ring two K steps ahead.  Staging through registers cost
// a ds_write_b128 per 16 B (13 LDS cycles each, MI355X_MICROARCH.md "LDS") -- more LDS time
// than the MFMAs it fed; the DMA needs no VGPRs and no store instructions.  The ring is
// ordered by a counted vmcnt and one barrier per step; steps past the end issue out-of-range
// (zero-fill, no traffic) pieces so every wait counts the same.  Lane l of a piece writes row
// l / 8, physical chunk l % 8; it fetches logical chunk (l % 8) ^ ((row >> 1) & 7), so the
// LDS image is the XOR-swizzled one ig_off() reads.  A source pixel outside the image (the
// tap bit is clear) gets an offset past the buffer end and reads zeros.
template <int BM, int BN, int WAVES_M, bool TR, int NST>
__global__ __launch_bounds__(kThreads, 2) void igemm_dma_kernel(
    GemmGeom g, const bf16_t* __restrict__ src, const bf16_t* __restrict__ wt,
    bf16_t* __restrict__ dst, const float* __restrict__ bias, const float* __restrict__ chan_add,
    const bf16_t* __restrict__ residual) {
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int NI = WTM / 16, NJ = WTN / 16;
  constexpr int IA = BM / 32, IB = BN / 32;  // pieces per wave per step (A, B)
  constexpr int PIECES = IA + IB;
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const bf16_t* lds = reinterpret_cast<const bf16_t*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WAVES_M, wn = wave / WAVES_M;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int C = g.sC;
  const int taps = g.kt * g.kh * g.kw, khw = g.kh * g.kw;
  const int csteps = (C + kIgBK - 1) / kIgBK;
  const int nk = taps * csteps;
  const int lr = lane >> 3, pc = lane & 7;

  // this lane's A rows (one per piece): source byte offset at tap 0 incl. its chunk, the
  // tap-validity bits, and the chunk's first channel
  int a_off[IA], a_c[IA];
  uint32_t a_ok[IA];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int r = (wave * IA + i) * 8 + lr;
    const int c = pc ^ ((r >> 1) & 7);
    a_c[i] = c * 8;
    int m = (int)m0 + r;
    const bool in = m < (int)g.M;
    if (!in) m = 0;
    const int w = m % g.dW; m /= g.dW;
    const int h = m % g.dH; m /= g.dH;
    const int t = m % g.dT;
    const int b = m / g.dT;
    int bt, bh, bw;
    if (!TR) {
      bt = t * g.st - g.pt; bh = h * g.sh - g.ph; bw = w * g.sw - g.pw;
    } else {
      bt = t + g.pt; bh = h + g.ph; bw = w + g.pw;
    }
    uint32_t vt = 0, vh = 0, vw = 0;
    for (int a = 0; a < g.kt; ++a) vt |= (uint32_t)((unsigned)(TR ? bt - a : bt + a) < (unsigned)g.sT) << a;
    for (int a = 0; a < g.kh; ++a) vh |= (uint32_t)((unsigned)(TR ? bh - a : bh + a) < (unsigned)g.sH) << a;
    for (int a = 0; a < g.kw; ++a) vw |= (uint32_t)((unsigned)(TR ? bw - a : bw + a) < (unsigned)g.sW) << a;
    uint32_t ok = 0;
    for (int a = 0; a < g.kt; ++a)
      for (int c2 = 0; c2 < g.kh; ++c2)
        if (((vt >> a) & (vh >> c2) & 1u) != 0) ok |= vw << (a * khw + c2 * g.kw);
    a_ok[i] = in ? ok : 0u;
    a_off[i] = (((b * g.sT + bt) * g.sH + bh) * g.sW + bw) * g.sCs * 2 + c * 16;
  }
  int b_off[IB], b_c[IB];
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int r = (wave * IB + i) * 8 + lr;
    const int c = pc ^ ((r >> 1) & 7);
    b_c[i] = c * 8;
    const int n = n0 + r;
    b_off[i] = n < g.N ? n * g.K * 2 + c * 16 : (int)0x80000000;
  }
  const rsrc_t rs_a = make_rsrc(src, (uint32_t)((int64_t)g.B * g.sT * g.sH * g.sW * g.sCs * 2));
  const rsrc_t rs_b = make_rsrc(wt, (uint32_t)((int64_t)g.N * g.K * 2));

  // K-step cursor: issue() is called for s = 0, 1, 2, ... in order, so the step's (tap,
  // channel step) and the tap's (a, b, c) advance incrementally -- the divisions by the
  // runtime csteps / kh*kw / kw took ~100 scalar instructions per step (the CU's scalar
  // unit, shared by all its waves, was close to saturated)
  int cur_ci = 0, cur_tap = 0, cur_a = 0, cur_b = 0, cur_c = 0, cur_toff = 0;
  auto issue = [&](int s) {  // K step s into ring stage s % NST
    char* st = smem + (s % NST) * STAGE;
    const bool live = s < nk;  // steps past the end: every piece out of range (zero fill)
    const int tap = live ? cur_tap : 0, c0 = cur_ci * kIgBK, toff = cur_toff;
    if (++cur_ci == csteps) {  // next tap: its (a, b, c) and source offset, once per tap
      cur_ci = 0;
      ++cur_tap;
      if (++cur_c == g.kw) {
        cur_c = 0;
        if (++cur_b == g.kh) {
          cur_b = 0;
          ++cur_a;
        }
      }
      cur_toff = ((cur_a * g.sH + cur_b) * g.sW + cur_c) * g.sCs * 2;
    }
    const int astep = (TR ? -toff : toff) + c0 * 2;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      // bitwise, not short-circuit: && here compiled to exec-mask branches per piece
      const bool ok = live & (c0 + a_c[i] < C) & (((a_ok[i] >> tap) & 1u) != 0);
      dma_lds<16>(rs_a, lds_addr(st + (wave * IA + i) * 1024),
                  ok ? (uint32_t)(a_off[i] + astep) : 0x80000000u);
    }
    const int bstep = (tap * C + c0) * 2;
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const bool ok = live & (c0 + b_c[i] < C);
      dma_lds<16>(rs_b, lds_addr(st + A_BYTES + (wave * IB + i) * 1024),
                  ok ? (uint32_t)(b_off[i] + bstep) : 0x80000000u);
    }
  };

  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  vm_drain();
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue(s);
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    vm_wait_barrier<(NST - 2) * PIECES>();  // step kt landed everywhere; step kt-1 consumed
    issue(kt + NST - 1);
    const bf16_t* As = lds + (kt % NST) * (STAGE / 2);
    const bf16_t* Bs = As + A_BYTES / 2;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[NI], bfr[NJ];
#pragma unroll
      for (int i = 0; i < NI; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(As + ig_off(wm * WTM + 16 * i + fr, 4 * s + fq));
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + ig_off(wn * WTN + 16 * j + fr, 4 * s + fq));
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  vm_drain();  // the zero-fill pieces past the end land before the epilogue reuses LDS
  __syncthreads();

  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int LDC = BN + 4;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * WTM + 16 * i + fq * 4 + r) * LDC + wn * WTN + 16 * j + fr] = acc[i][j][r];
  __syncthreads();
  const int64_t pix_per_b = (int64_t)g.dT * g.dH * g.dW;
  const bool vec = (g.N % 8 == 0) && (g.dNs % 8 == 0);
  for (int v = tid; v < BM * BN / 8; v += kThreads) {
    const int r = v / (BN / 8), c = (v % (BN / 8)) * 8;
    const int64_t m = m0 + r;
    const int n = n0 + c;
    if (m >= g.M || n >= g.N) continue;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = Cs[r * LDC + c + e];
    const int lim = g.N - n < 8 ? g.N - n : 8;
    if (bias)
      for (int e = 0; e < lim; ++e) o[e] += bias[n + e];
    if (chan_add) {
      const int bidx = (int)(m / pix_per_b);  // 64-bit division only where it is needed
      for (int e = 0; e < lim; ++e) o[e] += chan_add[(int64_t)bidx * g.N + n + e];
    }
    bf16_t* out = dst + m * g.dNs + n;
    if (vec) {
      if (residual) {
        float rv[8];
        load8(residual + m * g.dNs + n, rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += rv[e];
      }
      store8(out, o);
    } else {
      for (int e = 0; e < lim; ++e) {
        float val = o[e];
        if (residual) val += bf2f(residual[m * g.dNs + n + e]);
        out[e] = f2bf(val);
      }
    }
  }
}

template <int BM, int BN, int WM, bool TR, int NST>
void launch_igd(const GemmGeom& g, const void* src, const void* wt, void* dst, const float* bias,
                const float* ca, const void* res, hipStream_t st) {
  const size_t lds_ab = (size_t)NST * (BM + BN) * 128;
  const size_t lds_c = (size_t)BM * (BN + 4) * 4;
  const size_t lds = lds_ab > lds_c ? lds_ab : lds_c;
  auto kern = igemm_dma_kernel<BM, BN, WM, TR, NST>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  dim3 grid((unsigned)vd_cdiv(g.M, BM), (unsigned)vd_cdiv(g.N, BN));
  kern<<<grid, kThreads, lds, st>>>(g, (const bf16_t*)src, (const bf16_t*)wt, (bf16_t*)dst, bias,
                                    ca, (const bf16_t*)res);
}

// ----------------------------------------------------------------- 3x3x3 stride 1: halo tile
// The gathered-tile kernel above DMAs every tap's A tile separately: for 64 output channels
// that is 4 of the 5 LDS-DMA pieces a wave issues per 32 MFMAs (and ~60 cycles of issue each,
// MI355X_MICROARCH.md), so the 64-channel convs are DMA-issue bound.  Here a workgroup owns an
// output tile of 2 x 4 x 16 pixels (t, h, w) x 64 channels; per KS-channel step the input halo
// of the tile (4 x 6 x 18 pixels) lands in LDS once, and all 27 taps read their A fragments
// from it at shifted pixel offsets.  Only each tap's 64 x KS weight slice streams, through a
// 3-stage ring (one workgroup barrier per tap).  Transposed (bwd-data, stride 1): the same halo
// with the tap offsets mirrored (source pixel = out + 1 - tap).  Needs W % 16 == 0; partial
// t / h tiles are masked (zero halo rows, skipped stores).
// Output tile 2 x NW x 16 pixels (t, h, w) for NW waves (two 16-pixel rows per wave): NW = 4
// (the default) or 8 (round 6, A/B: one tile shared by 8 waves halves the weight-slice DMA per
// output and the halo pixels per output drop from 3.4 to 2.8).
constexpr int kHoT = 2, kHoW = 16;
constexpr int kHaT = kHoT + 2, kHaW = kHoW + 2;
template <int NW>
constexpr int halo_px() { return kHaT * (NW + 2) * kHaW; }  // 432 (NW 4) / 720 (NW 8) pixels
// KS channels per step: 64 (128-B LDS rows, 80 KiB per 4-wave workgroup, two per CU) or 32
// (64-B rows, 40 KiB, four per CU); weight ring stages NSTB (prefetch distance NSTB - 1).
template <int NSTB, int KS, int NW = 4>
constexpr size_t halo_lds() { return (size_t)(halo_px<NW>() + NSTB * 64) * 2 * KS + 1024; }
static_assert(halo_px<4>() % 16 == 0 && halo_px<8>() % 16 == 0, "whole halo pieces");
// Round 6: every tap unrolled.  The rolled tap loop spent ~35 SALU and ~16 VALU instructions
// per tap deriving (dt, dh, dw) by division, the ring stage and the fragment addresses
// (SQ_INSTS_SALU 2011 per wave for 432 MFMAs, 64->64 at 16x128x128), all on the wave's path
// between two barriers.  Here the 27 taps are unrolled, so the tap offsets and ring stages are
// immediates.  The halo swizzle is keyed on the pixel's column w inside its halo line (c ^ (w &
// 6) for 128-B rows, c ^ ((w >> 1) & 2) for 64-B rows), so a fragment read is a per-lane base
// chosen by dw (3 per fragment row) plus a compile-time offset.  ds_read_b128 serves lanes in
// groups of 16 ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and the same + 32): one LDS cycle
// mixes rows r, r + 12 (even fq) with r + 4, r + 8 (odd fq); these XOR terms give those lanes
// 16 distinct bank quads for any start row (searched exhaustively; the round-5 (r >> 2) & 3 /
// (r >> 1) & 7 terms were 2-way conflicted: SQ_LDS_BANK_CONFLICT was 47 % of the LDS cycles).
// A fragments of tap t + 1 are read during tap t (the halo is stable within a channel step;
// only the weight ring needs the per-tap barrier).
template <int KS>
__device__ __forceinline__ int h2_swz(int w) {
  if constexpr (KS == 64) return w & 6;
  else return (w >> 1) & 2;
}

// (round 6: compiling the 32-channel-step kernel for 3 waves per SIMD instead of 4 -- no spills,
// three workgroups per CU -- measured equal, profiles/r06z4_halo_wpe3_ab.txt)
template <bool TR, int KS, int NW, bool EA = true, bool EH = false>
__global__ __launch_bounds__(64 * NW, KS == 32 ? 4 : 2) void halo_conv_kernel(
    GemmGeom g, const bf16_t* __restrict__ src, const bf16_t* __restrict__ wt,
    bf16_t* __restrict__ dst, const float* __restrict__ bias, const float* __restrict__ chan_add,
    const bf16_t* __restrict__ residual) {
  constexpr int NSTB = 3, PD = NSTB - 1, TH = NW, kHaH = TH + 2, kHaP = halo_px<NW>();
  constexpr int RB = 2 * KS, PPP = 1024 / RB, CPR = KS / 8;  // row bytes, rows per piece, chunks
  constexpr int HP = kHaP / PPP;                                // halo pieces
  constexpr int BN = 64, NI = 2, NJ = 4, TAPS = 27, NS = KS / 32;
  constexpr int WP = BN / PPP, IB = WP >= NW ? WP / NW : 1;     // weight pieces per tap, per wave
  constexpr int HPW = (HP + NW - 1) / NW;                       // halo pieces per wave
  static_assert(WP % NW == 0 || NW % WP == 0, "weight pieces spread evenly");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem + kHaP * RB;
  char* junk = ring + NSTB * BN * RB;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // waves that stream weight pieces (all but NW = 8 at 32-channel steps: waves 0-3)
  const bool wl = WP >= NW || wave * IB < WP;
  const int tilesW = g.dW / kHoW, tilesH = (g.dH + TH - 1) / TH;
  const int tilesT = (g.dT + kHoT - 1) / kHoT;
  int mt = blockIdx.x;
  const int w0 = (mt % tilesW) * kHoW;
  mt /= tilesW;
  const int h0 = (mt % tilesH) * TH;
  mt /= tilesH;
  const int t0 = (mt % tilesT) * kHoT;
  const int b = mt / tilesT;
  const int n0 = blockIdx.y * BN;
  const int C = g.sC, csteps = (C + KS - 1) / KS;
  const int lr = lane / CPR, pc = lane % CPR;
  const rsrc_t rs_a = make_rsrc(src, (uint32_t)((int64_t)g.B * g.sT * g.sH * g.sW * g.sCs * 2));
  const rsrc_t rs_b = make_rsrc(wt, (uint32_t)((int64_t)g.N * g.K * 2));

  // (the chunk's channel test only matters in a ragged last channel step: recomputed there
  // rather than held in HPW more registers through the tap loop)
  int h_off[HPW];
  auto h_chunk = [&](int i) {
    const int hw = (PPP * (wave + NW * i) + lr) % kHaW;
    return (pc ^ h2_swz<KS>(hw)) * 8;
  };
#pragma unroll
  for (int i = 0; i < HPW; ++i) {
    const int q = wave + NW * i, p = PPP * q + lr;
    const int hw = p % kHaW, hh = (p / kHaW) % kHaH, ht = p / (kHaW * kHaH);
    const int c = pc ^ h2_swz<KS>(hw);
    const int st = t0 - 1 + ht, sh = h0 - 1 + hh, sw = w0 - 1 + hw;
    const bool in = q < HP && (unsigned)st < (unsigned)g.sT &&
                    (unsigned)sh < (unsigned)g.sH && (unsigned)sw < (unsigned)g.sW;
    h_off[i] = in ? (((b * g.sT + st) * g.sH + sh) * g.sW + sw) * g.sCs * 2 + c * 16 : -1;
  }
  // EH (round 6, forward only): the next channel step's first halo pieces -- wholly inside halo
  // frames 0-1, which the forward's taps 0-8 read first and no tap from 18 on reads -- are
  // issued at tap 18 of the current step, so a step boundary waits only for the rest.  The
  // split is by piece index i (the same on every wave, so the vmcnt counts are uniform): pieces
  // i < IE hold px < 16 IE NW - 1, inside frames 0-1 for every wave and covering the rows the
  // first three taps (dh = 0) read.
  constexpr int IE = ((2 * kHaH * kHaW) / PPP - NW) / NW + 1, NL = HPW - IE;
  static_assert(!EH || (!TR && EA && NW == 4 && (IE - 1) * NW + NW - 1 < (2 * kHaH * kHaW) / PPP &&
                        IE * NW * PPP >= kHaW * (kHaH + 3 + 1)),
                "early halo pieces: frames 0-1 only, covering the dh = 0 taps");
  auto issue_halo = [&](int cs, int i0, int i1) {
    const bool cfull = (cs + 1) * KS <= C;
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      if (i < i0 || i >= i1) continue;
      const int q = wave + NW * i;
      const bool ok = (h_off[i] >= 0) & (cfull || cs * KS + h_chunk(i) < C);
      dma_lds<16>(rs_a, lds_addr(q < HP ? smem + q * 1024 : junk),
                  ok ? (uint32_t)(h_off[i] + cs * KS * 2) : 0x80000000u);
    }
  };
  int b_off[IB], b_c[IB];
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int r = (wave * IB + i) * PPP + lr;
    const int c = pc ^ h2_swz<KS>(r);
    b_c[i] = c * 8;
    const int n = n0 + r;
    b_off[i] = n < g.N ? n * g.K * 2 + c * 16 : -1;
  }
  auto issue_b = [&](int cs, int tap) {  // tap >= 27: zero fill into the free stage
    char* st = ring + (tap % NSTB) * (BN * RB);
    const int c0 = cs * KS;
    if (!wl) return;
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const bool ok = (tap < TAPS) & (b_off[i] >= 0) & (c0 + b_c[i] < C);
      dma_lds<16>(rs_b, lds_addr(st + (wave * IB + i) * 1024),
                  ok ? (uint32_t)(b_off[i] + (tap * C + c0) * 2) : 0x80000000u);
    }
  };

  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  // byte offsets (from smem) of this lane's A fragment rows at tap (0, 0, dw), sub-step s
  int abase[NI][3][NS];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int rb = NI * wave + i, tl = rb / TH, hl = rb % TH;
    const int line = tl * kHaH + hl;
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int w = fr + d;
        abase[i][d][s] = (line * kHaW + w) * RB + (((4 * s + fq) ^ h2_swz<KS>(w)) << 4);
      }
  }
  int bbase[NJ][NS];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int r = 16 * j + fr;
      bbase[j][s] = kHaP * RB + r * RB + (((4 * s + fq) ^ h2_swz<KS>(r)) << 4);
    }

  vm_drain();
  for (int cs = 0; cs < csteps; ++cs) {
    lgk_wait_barrier();  // every wave's reads of the previous step's halo and ring returned
    // pre: this step's early pieces were issued at the previous step's tap 18
    const bool pre = EH && cs > 0, nxt = EH && cs + 1 < csteps;
    if (!pre) issue_halo(cs, 0, HPW);
#pragma unroll
    for (int i = 0; i < PD; ++i) issue_b(cs, i);
    if (pre) issue_halo(cs, IE, HPW);  // after B0 / B1: tap 0 waits for B0 only
    // opaque per channel step: the compiler would otherwise hoist all 27 x NI per-tap fragment
    // addresses out of the loop into VGPRs instead of folding the tap offsets into ds_read
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int s = 0; s < NS; ++s) asm volatile("" : "+v"(abase[i][d][s]));
    bf16x8 af[2][NI][NS];
    auto read_a = [&](int tp) {  // A fragments of tap tp from the halo
      const int a = tp / 9, bb = (tp / 3) % 3, cc = tp % 3;
      const int dt = TR ? 2 - a : a, dh = TR ? 2 - bb : bb, dw = TR ? 2 - cc : cc;
      const int lofs = (dt * kHaH + dh) * kHaW * RB;
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int s = 0; s < NS; ++s)
          af[tp & 1][i][s] = *reinterpret_cast<const bf16x8*>(smem + abase[i][dw][s] + lofs);
    };
#pragma unroll
    for (int tap = 0; tap < TAPS; ++tap) {
      // this tap's weights (and at tap 0 the halo) landed everywhere; stage tap-1 is free
      if constexpr (EH) {
        // newer than this tap's weight pieces: the late halo pieces (taps 0, 1 of a step whose
        // early pieces came before) or the next step's early pieces (taps 19, 20)
        if ((tap == 0 || tap == 1) && pre) vm_lgk_wait_barrier<(PD - 1) * IB + NL>();
        else if ((tap == 19 || tap == 20) && nxt) vm_lgk_wait_barrier<(PD - 1) * IB + IE>();
        else vm_lgk_wait_barrier<(PD - 1) * IB>();
      } else if (wl) {
        vm_lgk_wait_barrier<(PD - 1) * IB>();
      } else {
        vm_lgk_wait_barrier<0>();
      }
      issue_b(cs, tap + PD);
      if constexpr (EH) {
        if (tap == 18 && nxt) issue_halo(cs + 1, 0, IE);  // frames 0-1 are free from tap 18 on
      }
      const int so = (tap % NSTB) * (BN * RB);
      if constexpr (EA) {
        // round 6: this tap's B fragments, then the next tap's A fragments, all issued before
        // the MFMAs (pinned by the scheduling barrier): the A reads land during this tap's
        // MFMAs instead of being issued after their last use of the registers, where the next
        // barrier's lgkmcnt(0) waited out their whole latency
        if (tap == 0) read_a(0);
        bf16x8 bfr[NS][NJ];
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            bfr[s][j] = *reinterpret_cast<const bf16x8*>(smem + bbase[j][s] + so);
        if (tap + 1 < TAPS) read_a(tap + 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[tap & 1][i][s], bfr[s][j],
                                                                  acc[i][j], 0, 0, 0);
      } else {  // the compiler's placement (A/B: vd_conv_set_halo(4))
        if (tap == 0) read_a(0);
        if (tap + 1 < TAPS) read_a(tap + 1);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          bf16x8 bfr[NJ];
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            bfr[j] = *reinterpret_cast<const bf16x8*>(smem + bbase[j][s] + so);
#pragma unroll
          for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[tap & 1][i][s], bfr[j],
                                                                  acc[i][j], 0, 0, 0);
        }
      }
    }
  }
  vm_drain();  // the zero-fill pieces past the last tap land before the epilogue reuses LDS
  __syncthreads();

  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int LDC = BN + 4;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(16 * (NI * wave + i) + fq * 4 + r) * LDC + 16 * j + fr] = acc[i][j][r];
  __syncthreads();
  // every thread stores the same 8-channel chunk of 4 rows (256 threads, 8 chunks per row):
  // its bias + per-(b, co) add is loaded once, and the residual rows are all requested before
  // the first store (round 6: the per-element scalar adds and the serialised residual loads took
  // 35 us of the 105 us of a 64->64 ResBlock conv at 16x128x128, tools/conv3_bench.py
  // --epilogue)
  constexpr int ROWS = kHoT * TH * kHoW, ITER = ROWS * BN / 8 / (64 * NW);
  const int cq = tid % (BN / 8), n = n0 + cq * 8;
  const int lim = g.N - n < 8 ? g.N - n : 8;
  float cadd[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) cadd[e] = 0.f;
  if (lim == 8) {
    float tv[8];
    if (bias) {
      load8(bias + n, tv);
#pragma unroll
      for (int e = 0; e < 8; ++e) cadd[e] += tv[e];
    }
    if (chan_add) {
      load8(chan_add + (int64_t)b * g.N + n, tv);
#pragma unroll
      for (int e = 0; e < 8; ++e) cadd[e] += tv[e];
    }
  } else {
    for (int e = 0; e < lim; ++e)
      cadd[e] = (bias ? bias[n + e] : 0.f) + (chan_add ? chan_add[(int64_t)b * g.N + n + e] : 0.f);
  }
  const bool vec = lim == 8 && (g.dNs % 8 == 0);
  int64_t mrow[ITER];
  float rv[ITER][8];
#pragma unroll
  for (int k = 0; k < ITER; ++k) {
    const int r = tid / (BN / 8) + k * (64 * NW / (BN / 8));
    const int t = t0 + r / (TH * kHoW), h = h0 + (r / kHoW) % TH, w = w0 + r % kHoW;
    mrow[k] = (t < g.dT && h < g.dH && lim > 0) ? (((int64_t)b * g.dT + t) * g.dH + h) * g.dW + w
                                                : -1;
#pragma unroll
    for (int e = 0; e < 8; ++e) rv[k][e] = 0.f;
    if (residual && vec && mrow[k] >= 0) load8(residual + mrow[k] * g.dNs + n, rv[k]);
  }
#pragma unroll
  for (int k = 0; k < ITER; ++k) {
    if (mrow[k] < 0) continue;
    const int r = tid / (BN / 8) + k * (64 * NW / (BN / 8));
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = Cs[r * LDC + cq * 8 + e] + cadd[e] + rv[k][e];
    bf16_t* out = dst + mrow[k] * g.dNs + n;
    if (vec) {
      store8(out, o);
    } else {
      for (int e = 0; e < lim; ++e) {
        float val = o[e];
        if (residual) val += bf2f(residual[mrow[k] * g.dNs + n + e]);
        out[e] = f2bf(val);
      }
    }
  }
}

// halo-tile eligibility: 3x3x3, stride 1, pad 1, same-size in / out, W a multiple of 16
bool halo_ok(const GemmGeom& g) {
  return g.kt == 3 && g.kh == 3 && g.kw == 3 && g.st == 1 && g.sh == 1 && g.sw == 1 &&
         g.pt == 1 && g.ph == 1 && g.pw == 1 && g.sT == g.dT && g.sH == g.dH && g.sW == g.dW &&
         g.dW % kHoW == 0;
}
// VDIFF_CONV_HALO / vd_conv_set_halo: 0 never (the gathered-tile kernel), 1 and 2 (default)
// every eligible conv.  Round 6: with the conflict-free swizzle and the unrolled taps the halo
// tile beats the gathered 128 x 128 tiles on every 3x3x3 shape of the step, fwd and bwd-data
// (tools/conv3_bench.py, profiles/r06_conv3_ab.txt), so the round-2 per-shape selection (halo
// only for N <= 64 and at the 32x32 level) is gone.
std::atomic<int> g_halo_mode{[] {
  const char* e = getenv("VDIFF_CONV_HALO");
  return e ? atoi(e) : 2;
}()};
int conv_halo_mode() { return g_halo_mode.load(std::memory_order_relaxed); }
// kw-strip weight-gradient kernel: 1 (default) wgrad_strip_kernel, 0 the round-5
// wgrad_dma_kernel (A/B; vd_conv_set_wgrad, VDIFF_WGRAD_STRIP)
std::atomic<int> g_wgrad_mode{[] {
  const char* e = getenv("VDIFF_WGRAD_STRIP");
  return e ? atoi(e) : 1;
}()};

// Channels per halo step for this conv, 0 = the gathered-tile kernel: 64-channel steps (80 KiB,
// two workgroups per CU) at the 32x32 level and from 128 reduction channels on, 32-channel
// steps (40 KiB, four per CU) otherwise; VDIFF_CONV_HALO_KS forces one (A/B).  sC = the GEMM's
// reduction channels (Ci fwd, Co bwd-data).
int halo_ks(const GemmGeom& g, bool /*tr*/) {
  if (conv_halo_mode() == 0 || !halo_ok(g)) return 0;
  static const int force = [] {
    const char* e = getenv("VDIFF_CONV_HALO_KS");
    return e ? atoi(e) : 0;
  }();
  if (force == 32 || force == 64) return force;
  return (g.dW <= 32 || g.sC >= 128) ? 64 : 32;
}
template <bool TR, int KS, int NW, bool EA = true, bool EH = false>
void launch_halo_tile(const GemmGeom& g, const void* src, const void* wt, void* dst,
                  const float* bias, const float* ca, const void* res, hipStream_t st) {
  const size_t lds_c = (size_t)kHoT * NW * kHoW * (64 + 4) * 4;  // the epilogue's fp32 tile
  const size_t lds = halo_lds<3, KS, NW>() > lds_c ? halo_lds<3, KS, NW>() : lds_c;
  auto kern = halo_conv_kernel<TR, KS, NW, EA, EH>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  const int64_t tiles = (int64_t)g.B * vd_cdiv(g.dT, kHoT) * vd_cdiv(g.dH, NW) * (g.dW / kHoW);
  dim3 grid((unsigned)tiles, (unsigned)vd_cdiv(g.N, 64));
  kern<<<grid, 64 * NW, lds, st>>>(g, (const bf16_t*)src, (const bf16_t*)wt, (bf16_t*)dst, bias,
                                   ca, (const bf16_t*)res);
}
// (round 6, measured and removed: two taps per ring stage and barrier at three workgroups per CU
// -- equal; a barrier-free form where each wave streams its own 16 weight rows for all 128
// pixels -- 7 % slower, LDS-read bound at 9 fragment reads per 8 MFMAs.  Round 5: 8 waves per
// workgroup, a 5-stage ring, a 4-frame tile.)
template <bool TR>
void launch_halo(const GemmGeom& g, int ks, const void* src, const void* wt, void* dst,
                 const float* bias, const float* ca, const void* res, hipStream_t st) {
  if (conv_halo_mode() == 3) {  // A/B: 8-wave workgroups on 2 x 8 x 16 tiles
    if (ks == 32) launch_halo_tile<TR, 32, 8>(g, src, wt, dst, bias, ca, res, st);
    else launch_halo_tile<TR, 64, 8>(g, src, wt, dst, bias, ca, res, st);
    return;
  }
  if (conv_halo_mode() == 4) {  // A/B: round-6 tap loop with the compiler's read placement
    if (ks == 32) launch_halo_tile<TR, 32, 4, false>(g, src, wt, dst, bias, ca, res, st);
    else launch_halo_tile<TR, 64, 4, false>(g, src, wt, dst, bias, ca, res, st);
    return;
  }
  if constexpr (!TR) {
    if (conv_halo_mode() != 5) {  // forward: early halo pieces (mode 5: without, A/B)
      if (ks == 32) launch_halo_tile<TR, 32, 4, true, true>(g, src, wt, dst, bias, ca, res, st);
      else launch_halo_tile<TR, 64, 4, true, true>(g, src, wt, dst, bias, ca, res, st);
      return;
    }
  }
  if (ks == 32) launch_halo_tile<TR, 32, 4>(g, src, wt, dst, bias, ca, res, st);
  else launch_halo_tile<TR, 64, 4>(g, src, wt, dst, bias, ca, res, st);
}

// ----------------------------------------------------------------- 1x1 convs: streaming GEMM
// A 1x1, stride-1, unpadded conv (qkv / proj_out / skip, fwd and bwd-data) is an HBM-bound
// GEMM over pixels: Y[p][n] = sum_k X[p][k] W[n][k] with K = 32 KS <= 256 and a weight slice
// of whole 64-channel chunks that fits the LDS.  Persistent workgroups load their weight slice (NS output channels) into LDS
// once and stream 16-pixel tiles: each wave takes whole tiles, loads the tile's X rows
// straight into MFMA B operands (lane = pixel, 16 B of channels each: no LDS for X), keeps
// the next tile's loads in flight while it computes, and emits C^T = W X^T so every lane
// stores 16 consecutive channels (two 16-B stores) of one pixel per 64-channel chunk.  Bias, per-batch channel add and the
// residual are fused into the store.  W rows are padded by 16 B: the 16 rows of an A-operand
// read land in distinct bank quads for every K.
constexpr int kPwMaxLds = 40 * 1024;

template <int KS>
__global__ __launch_bounds__(256) void pw_gemm_kernel(
    const bf16_t* __restrict__ src, int sCs, const bf16_t* __restrict__ wt, int N, int NS,
    bf16_t* __restrict__ dst, int dNs, const float* __restrict__ bias,
    const float* __restrict__ chan_add, int64_t ppb, const bf16_t* __restrict__ residual,
    int64_t M) {
  constexpr int K = 32 * KS, RS = K + 8;  // LDS row stride in bf16 (16-B pad)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* wl = reinterpret_cast<bf16_t*>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nbase = blockIdx.y * NS;
  const int nsl = N - nbase < NS ? N - nbase : NS;  // channels of this slice (multiple of 16)
  const int nrow = (nsl + 63) / 64 * 64;  // rows read by the MFMAs (zero past nsl)
  for (int c = tid; c < nrow * (K / 8); c += 256) {
    const int r = c / (K / 8), k8 = c % (K / 8);
    *reinterpret_cast<uint4*>(wl + r * RS + k8 * 8) =
        r < nsl ? *reinterpret_cast<const uint4*>(wt + (int64_t)(nbase + r) * K + k8 * 8)
                : make_uint4(0, 0, 0, 0);
  }
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  const int64_t ntiles = (M + 15) / 16;
  const int64_t stride = (int64_t)gridDim.x * 4;
  auto load = [&](bf16x8 (&x)[KS], int64_t tile) __attribute__((always_inline)) {
    const int64_t p = tile * 16 + fr;
    const bool ok = tile < ntiles && p < M;
    const bf16_t* row = src + (ok ? p : 0) * (int64_t)sCs + 8 * fq;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const uint4 v = ok ? *reinterpret_cast<const uint4*>(row + 32 * kk) : make_uint4(0, 0, 0, 0);
      x[kk] = __builtin_bit_cast(bf16x8, v);
    }
  };
  bf16x8 xc[KS], xn[KS];
  int64_t tile = (int64_t)blockIdx.x * 4 + wave;
  load(xc, tile);
  for (; tile < ntiles; tile += stride) {
    load(xn, tile + stride);  // next tile in flight while this one computes and stores
    const int64_t p = tile * 16 + fr;
    const bool pok = p < M;
    const int b = chan_add ? (int)((pok ? p : 0) / ppb) : 0;
    bf16_t* out = dst + (pok ? p : 0) * (int64_t)dNs + nbase;
    const bf16_t* res = residual ? residual + (pok ? p : 0) * (int64_t)dNs + nbase : nullptr;
    for (int n0 = 0; n0 < nsl; n0 += 64) {
      // block j's A row r is channel n0 + 16 (r >> 2) + 4 j + (r & 3), so accumulator
      // register i of block j on lane (fq, pixel) is channel n0 + 16 fq + 4 j + i: each lane
      // ends with 16 consecutive channels of its pixel (two 16-B stores)
      f32x4 acc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bf16_t* wr = wl + (n0 + 16 * (fr >> 2) + 4 * j + (fr & 3)) * RS + 8 * fq;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(wr + 32 * kk);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, xc[kk], acc[j], 0, 0, 0);
        }
      }
      const int nl = n0 + 16 * fq;  // this lane's first channel within the slice
      if (nl < nsl && pok) {
        float o[16];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) o[4 * j + i] = acc[j][i];
        if (bias) {
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            const float4 bv = *reinterpret_cast<const float4*>(bias + nbase + nl + 4 * q4);
            o[4 * q4] += bv.x; o[4 * q4 + 1] += bv.y; o[4 * q4 + 2] += bv.z; o[4 * q4 + 3] += bv.w;
          }
        }
        if (chan_add) {
          const float* cr = chan_add + (int64_t)b * N + nbase + nl;
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            const float4 cv = *reinterpret_cast<const float4*>(cr + 4 * q4);
            o[4 * q4] += cv.x; o[4 * q4 + 1] += cv.y; o[4 * q4 + 2] += cv.z; o[4 * q4 + 3] += cv.w;
          }
        }
        if (res) {
          float rv[8];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            load8(res + nl + 8 * h, rv);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[8 * h + e] += rv[e];
          }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float v8[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v8[e] = o[8 * h + e];
          store8(out + nl + 8 * h, v8);
        }
      }
    }
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) xc[kk] = xn[kk];
  }
}

// 1x1 conv on the streaming kernel when the shape allows (else -1): K = 32..256 in steps of
// 32, N a multiple of 16, 16-B aligned rows, 8-B aligned output / residual rows.
int pw_gemm_launch(const GemmGeom& g, const void* src, const void* wt, void* dst,
                   const float* bias, const float* ca, const void* res, hipStream_t st) {
  const int K = g.sC;
  if (g.kt * g.kh * g.kw != 1 || g.st != 1 || g.sh != 1 || g.sw != 1 || g.pt || g.ph || g.pw)
    return -1;
  if (K % 32 || K > 256 || g.N % 16 || g.sCs % 8 || g.dNs % 8 || g.K != K) return -1;
  if ((reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(wt) & 15) ||
      (reinterpret_cast<uintptr_t>(dst) & 15) || (reinterpret_cast<uintptr_t>(res) & 15))
    return -1;
  if (bias && (reinterpret_cast<uintptr_t>(bias) & 15)) return -1;
  if (ca && ((reinterpret_cast<uintptr_t>(ca) & 15) || g.N % 4)) return -1;
  const int row_bytes = (K + 8) * 2;
  int NS = (kPwMaxLds / row_bytes) / 64 * 64;  // slices of whole 64-channel chunks
  if (NS < 64) return -1;
  int slices = (int)vd_cdiv(g.N, NS);
  NS = (int)vd_cdiv(vd_cdiv(g.N, slices), 64) * 64;  // even slices
  slices = (int)vd_cdiv(g.N, NS);
  const size_t lds = (size_t)NS * row_bytes;
  const int64_t tiles = vd_cdiv(g.M, 16);
  int64_t wgs = vd_cdiv(tiles, 4);
  // persistent: <= 4 workgroups per CU in all (8 measured 4-30 % slower on 6 of the 7 UNet
  // shapes: fewer waves contend less for the write path; profiles/r05u_prof_conv1x1.md)
  const int64_t cap = (int64_t)256 * 4 / slices;
  if (wgs > cap) wgs = cap < 256 ? 256 : cap;
  const int64_t ppb = (int64_t)g.dT * g.dH * g.dW;
  dim3 grid((unsigned)wgs, (unsigned)slices);
#define VD_PW_CASE(KS_)                                                                          \
  case KS_: {                                                                                    \
    auto kern = pw_gemm_kernel<KS_>;                                                             \
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,     \
                              (int)lds);                                                         \
    kern<<<grid, 256, lds, st>>>((const bf16_t*)src, g.sCs, (const bf16_t*)wt, g.N, NS,          \
                                 (bf16_t*)dst, g.dNs, bias, ca, ppb, (const bf16_t*)res, g.M);   \
    return VD_OK;                                                                                \
  }
  switch (K / 32) {
    VD_PW_CASE(1) VD_PW_CASE(2) VD_PW_CASE(3) VD_PW_CASE(4)
    VD_PW_CASE(5) VD_PW_CASE(6) VD_PW_CASE(7) VD_PW_CASE(8)
  }
#undef VD_PW_CASE
  return -1;
}

#ifndef VD_PW_DEFAULT
#define VD_PW_DEFAULT 1
#endif
// VDIFF_CONV_PW=0 turns the streaming 1x1 kernel off (A/B)
const bool g_conv_pw = [] {
  const char* e = getenv("VDIFF_CONV_PW");
  return e ? atoi(e) != 0 : VD_PW_DEFAULT != 0;
}();

// Single-K-step GEMMs (1x1 convs with Ci <= 64: qkv, proj_out, skip) are load -> MFMA ->
// store with nothing to overlap inside a workgroup, so the tile is picked for workgroups
// per CU: 64 x 64 (32 KB LDS, five per CU) moves 64->192 x 262144 in 95 us against 114 us
// for the 256 x 64 tile (tools/conv1x1_bench.py).  Env VDIFF_CONV_1X1 (A/B): 0 = the
// general tiles below, 1 = 128 x 64 (97 us), 2 = one 64 x 192 tile for N = 192 (127 us),
// 3 = 64 x 64 (default).
int conv_1x1_variant() {
  static const int v = [] {
    const char* e = getenv("VDIFF_CONV_1X1");
    return e ? atoi(e) : 3;
  }();
  return v;
}

template <bool TR>
int launch_igemm_dma(const GemmGeom& g, const void* src, const void* wt, void* dst,
                     const float* bias, const float* ca, const void* res, hipStream_t st) {
  if (!TR && g.kt * g.kh * g.kw == 1 && g.sC <= kIgBK) {  // forward (the measured case)
    const int v = conv_1x1_variant();
    if (v == 1) {
      launch_igd<128, 64, 4, TR, 2>(g, src, wt, dst, bias, ca, res, st);
      return VD_OK;
    }
    if (v == 3) {
      launch_igd<64, 64, 4, TR, 2>(g, src, wt, dst, bias, ca, res, st);
      return VD_OK;
    }
    if (v == 2 && g.N > 128 && g.N <= 192) {
      launch_igd<64, 192, 1, TR, 2>(g, src, wt, dst, bias, ca, res, st);
      return VD_OK;
    }
  }
  // two or more workgroups per CU (double-buffered ring): measured faster than one workgroup with a
  // three-stage ring on every UNet shape (tools/conv_ab4.sh).  N that is a multiple of 64 but
  // not of 128 (the qkv conv, N = 192) takes 64-wide tiles: no half-empty column tile.
  if (g.N <= 64 || (g.N % 128 != 0 && g.N % 64 == 0)) {
    // 128 x 64 tiles (three workgroups per CU): since the K-step cursor made the DMA issue
    // cheap, they beat 256 x 64 (the 200-channel first conv 455 -> 382 us, 64->64 at
    // 262144 pixels 111 -> 109 us; profiles/r02_ab_conv_scalar.txt).  VDIFF_CONV_N64 (A/B):
    // 0 = 256 x 64, 2 = 64 x 64
    static const int n64 = [] {
      const char* e = getenv("VDIFF_CONV_N64");
      return e ? atoi(e) : 1;
    }();
    if (n64 == 0) launch_igd<256, 64, 4, TR, 2>(g, src, wt, dst, bias, ca, res, st);
    else if (n64 == 2) launch_igd<64, 64, 4, TR, 2>(g, src, wt, dst, bias, ca, res, st);
    else launch_igd<128, 64, 4, TR, 2>(g, src, wt, dst, bias, ca, res, st);
  } else if (vd_cdiv(g.M, 128) * vd_cdiv(g.N, 128) < 512) {
    // fewer than two 128 x 128 tiles per CU: 64 x 128 (256->256 at 16x32x32: 1.00 -> 0.91 ms)
    launch_igd<64, 128, 2, TR, 2>(g, src, wt, dst, bias, ca, res, st);
  } else {
    launch_igd<128, 128, 2, TR, 2>(g, src, wt, dst, bias, ca, res, st);
  }
  return VD_OK;
}

int check_desc(const vd_conv_desc* d) {
  VD_REQUIRE(d, "null descriptor");
  VD_REQUIRE(d->B > 0 && d->Ti > 0 && d->Hi > 0 && d->Wi > 0 && d->Ci > 0 && d->To > 0 &&
                 d->Ho > 0 && d->Wo > 0 && d->Co > 0,
             "bad conv shape");
  VD_REQUIRE(d->kt > 0 && d->kh > 0 && d->kw > 0 && d->st > 0 && d->sh > 0 && d->sw > 0 &&
                 d->pt >= 0 && d->ph >= 0 && d->pw >= 0,
             "bad conv kernel/stride/pad");
  VD_REQUIRE(d->Ci % 8 == 0, "Ci=%d must be a multiple of 8 (pad channels)", d->Ci);
  VD_REQUIRE(d->To == (d->Ti + 2 * d->pt - d->kt) / d->st + 1 &&
                 d->Ho == (d->Hi + 2 * d->ph - d->kh) / d->sh + 1 &&
                 d->Wo == (d->Wi + 2 * d->pw - d->kw) / d->sw + 1,
             "output shape does not match input/kernel/stride/pad");
  VD_REQUIRE(d->x_cstride == 0 || (d->x_cstride >= d->Ci && d->x_cstride % 8 == 0),
             "bad x_cstride");
  VD_REQUIRE(d->y_cstride == 0 || d->y_cstride >= d->Co, "bad y_cstride");
  return VD_OK;
}

template <typename T, bool TR>
int launch_gemm(const GemmGeom& g, const void* src, const void* wt, void* dst, const float* bias,
                const float* ca, const void* res, hipStream_t st) {
  if constexpr (sizeof(T) == 2) {
    if (!g_legacy_conv && g_conv_pw && pw_gemm_launch(g, src, wt, dst, bias, ca, res, st) == VD_OK)
      return VD_OK;
    const bool unit = g.st == 1 && g.sh == 1 && g.sw == 1;
    // LDS-DMA ring: 32-bit buffer offsets, taps <= 32 (validity bits), unit-stride gather
    // when transposed
    if (!g_legacy_conv && g_conv_dma && g.kt * g.kh * g.kw <= 32 && (!TR || unit) &&
        (int64_t)g.B * g.sT * g.sH * g.sW * g.sCs * 2 < ((int64_t)1 << 31) &&
        (int64_t)g.N * g.K * 2 < ((int64_t)1 << 31)) {
      if (const int ks = halo_ks(g, TR)) {
        launch_halo<TR>(g, ks, src, wt, dst, bias, ca, res, st);
        return VD_OK;
      }
      return launch_igemm_dma<TR>(g, src, wt, dst, bias, ca, res, st);
    }
    if (!g_legacy_conv) return launch_igemm<TR>(g, src, wt, dst, bias, ca, res, st);
  }
  const int64_t mt = vd_cdiv(g.M, 128);
  const bool narrow = g.N <= 64;
  if (narrow) {
    constexpr int BN = 64;
    const size_t lds_ab = 2 * (128 + BN) * Cfg<T>::LDK * sizeof(T);
    const size_t lds_c = 128 * (BN + 4) * sizeof(float);
    dim3 grid((unsigned)mt, (unsigned)vd_cdiv(g.N, BN));
    conv_gemm_kernel<T, BN, TR><<<grid, kThreads, lds_ab > lds_c ? lds_ab : lds_c, st>>>(
        g, (const T*)src, (const T*)wt, (T*)dst, bias, ca, (const T*)res);
  } else {
    constexpr int BN = 128;
    const size_t lds_ab = 2 * (128 + BN) * Cfg<T>::LDK * sizeof(T);
    const size_t lds_c = 128 * (BN + 4) * sizeof(float);
    dim3 grid((unsigned)mt, (unsigned)vd_cdiv(g.N, BN));
    conv_gemm_kernel<T, BN, TR><<<grid, kThreads, lds_ab > lds_c ? lds_ab : lds_c, st>>>(
        g, (const T*)src, (const T*)wt, (T*)dst, bias, ca, (const T*)res);
  }
  return VD_OK;
}

}  // namespace

extern "C" {

int vd_conv3d_fwd(const vd_conv_desc* d, const void* x, const void* w_fwd, const float* bias,
                  const float* chan_add, const void* residual, void* y, void* stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  VD_REQUIRE(x && w_fwd && y, "null tensor");
  GemmGeom g;
  g.B = d->B;
  g.sT = d->Ti; g.sH = d->Hi; g.sW = d->Wi; g.sC = d->Ci;
  g.sCs = d->x_cstride ? d->x_cstride : d->Ci;
  g.dT = d->To; g.dH = d->Ho; g.dW = d->Wo; g.N = d->Co;
  g.dNs = d->y_cstride ? d->y_cstride : d->Co;
  g.kt = d->kt; g.kh = d->kh; g.kw = d->kw;
  g.st = d->st; g.sh = d->sh; g.sw = d->sw;
  g.pt = d->pt; g.ph = d->ph; g.pw = d->pw;
  g.M = (int64_t)d->B * d->To * d->Ho * d->Wo;
  g.K = d->kt * d->kh * d->kw * d->Ci;
  return VD_DISPATCH_DTYPE(d->dtype, T, {
    launch_gemm<T, false>(g, x, w_fwd, y, bias, chan_add, residual, VD_STREAM(stream));
  });
}

int vd_conv_set_wgrad(int mode) {
  if (mode < 0 || mode > 2) {
    (void)vd::fail(VD_EINVAL, "conv wgrad mode %d (0, 1, 2)", mode);
    return -2;
  }
  return g_wgrad_mode.exchange(mode);
}

int vd_conv_set_halo(int mode) {
  if (mode < 0 || mode > 5) {
    (void)vd::fail(VD_EINVAL, "conv halo mode %d (0 - 5)", mode);
    return -2;
  }
  return g_halo_mode.exchange(mode);
}

int vd_conv3d_bwd_data(const vd_conv_desc* d, const void* dy, const void* w_bwd, void* dx,
                       void* stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  VD_REQUIRE(dy && w_bwd && dx, "null tensor");
  VD_REQUIRE(d->Co % 8 == 0, "bwd_data needs Co %% 8 == 0 (got %d)", d->Co);
  VD_REQUIRE(d->y_cstride == 0 || d->y_cstride % 8 == 0, "bad y_cstride");
  GemmGeom g;
  g.B = d->B;
  g.sT = d->To; g.sH = d->Ho; g.sW = d->Wo; g.sC = d->Co;
  g.sCs = d->y_cstride ? d->y_cstride : d->Co;
  g.dT = d->Ti; g.dH = d->Hi; g.dW = d->Wi; g.N = d->Ci;
  g.dNs = d->x_cstride ? d->x_cstride : d->Ci;
  g.kt = d->kt; g.kh = d->kh; g.kw = d->kw;
  g.st = d->st; g.sh = d->sh; g.sw = d->sw;
  g.pt = d->pt; g.ph = d->ph; g.pw = d->pw;
  g.M = (int64_t)d->B * d->Ti * d->Hi * d->Wi;
  g.K = d->kt * d->kh * d->kw * d->Co;
  return VD_DISPATCH_DTYPE(d->dtype, T, {
    launch_gemm<T, true>(g, dy, w_bwd, dx, nullptr, nullptr, nullptr, VD_STREAM(stream));
  });
}

}  // extern "C"

// The weight-gradient launch.  `splits_out` receives the number of pixel splits (grid.y);
// with dry = true nothing is launched (workspace sizing); split_stride as in WgtGeom.
static int wgrad_run(const vd_conv_desc* d, const void* x, const void* dy, float* dw,
                     int64_t split_stride, int64_t* splits_out, bool dry, void* stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  VD_REQUIRE(dry || (x && dy && dw), "null tensor");
  VD_REQUIRE(d->Co % 8 == 0, "bwd_weight needs Co %% 8 == 0 (got %d)", d->Co);
  WgtGeom g;
  g.split_stride = split_stride;
  g.xcd_tiles = g.xcd_total = 0;
  g.B = d->B;
  g.Ti = d->Ti; g.Hi = d->Hi; g.Wi = d->Wi; g.Ci = d->Ci;
  g.xCs = d->x_cstride ? d->x_cstride : d->Ci;
  g.To = d->To; g.Ho = d->Ho; g.Wo = d->Wo; g.Co = d->Co;
  g.yCs = d->y_cstride ? d->y_cstride : d->Co;
  g.kt = d->kt; g.kh = d->kh; g.kw = d->kw;
  g.st = d->st; g.sh = d->sh; g.sw = d->sw;
  g.pt = d->pt; g.ph = d->ph; g.pw = d->pw;
  g.M = (int64_t)d->B * d->To * d->Ho * d->Wo;
  const int taps = d->kt * d->kh * d->kw;
  // bf16 stride-1 "same" 3x3(x3) convs with image rows that tile into 64-pixel steps:
  // the kw-strip kernel (three taps per workgroup)
  const bool strip = d->dtype == VD_BF16 && !g_legacy_conv && d->kh == 3 && d->kw == 3 &&
                     (d->kt == 1 || d->kt == 3) && d->st == 1 && d->sh == 1 && d->sw == 1 &&
                     d->pt == d->kt / 2 && d->ph == 1 && d->pw == 1 &&
                     (d->Wo % 64 == 0 || (64 % d->Wo == 0 && 64 / d->Wo <= d->Ho));
  const bool one = d->dtype == VD_BF16 && !g_legacy_conv && taps == 1 && d->st == 1 &&
                   d->sh == 1 && d->sw == 1 && d->pt == 0 && d->ph == 0 && d->pw == 0;
  const int64_t x_bytes = (int64_t)d->B * d->Ti * d->Hi * d->Wi * g.xCs * 2;
  const bool dma = g_conv_dma && (strip || one) && g.xCs % 8 == 0 && g.yCs % 8 == 0 &&
                   x_bytes < (1ll << 31) && g.M * g.yCs * 2 < (1ll << 31);
  hipStream_t st = VD_STREAM(stream);
  if (dma) {
    // LDS-DMA kernels: kw-strip (three taps per workgroup) or 1x1 (a plain GEMM over pixels)
    const int wc = one ? 64 : (d->Wo < 64 ? d->Wo : 64);
    const int rows = one ? 64 : (64 / wc) * (wc + 2);
    // 1x1 (A/B knob VDIFF_WGRAD1=nst,cot): ring depth 2 / 4 / 6 and 64 / 128 / 192 output
    // channels per workgroup (192: X read once per 192 channels of the qkv projections).
    // Default 4,64 since the occupancy-round split rule (round 4: 0.667 -> 0.622 ms per step,
    // the 256->768 / 256->256 / 128->128 shapes 9-19 % faster, the rest equal;
    // profiles/r04x_ab_wgrad_knobs.txt); round 3 had measured 4,128 best under the old split
    // rule (0.864 -> 0.722 ms, profiles/r03_ab_wgrad1x1.txt)
    static const int w1 = [] {
      const char* e = getenv("VDIFF_WGRAD1");
      int n = 4, c = 64;
      if (e) sscanf(e, "%d,%d", &n, &c);
      return n * 1000 + c;
    }();
    const int w1_nst = w1 / 1000, w1_cot = (w1 % 1000 == 192 && d->Co % 192 == 0) ? 192
                                             : (w1 % 1000 == 128 && d->Co % 128 == 0 ? 128 : 64);
    // 3x3(x3) kw-strip (A/B knob VDIFF_WGRAD3=nst,cot): ring depth and 64 / 128 output
    // channels per workgroup
    // cot 0 (the default): 128 output channels per workgroup where Co % 128 == 0 and that
    // grid can still fill 90 % of the chip's resident slots (2 workgroups per CU at 128, the
    // ring being 2 x (128 + RW) rows), else 64 -- under the occupancy-round split rule below
    // 128-wide tiles won on 9 of the step's 11 such shapes, losing only where the grid stays
    // under one round (128->256 on 16x32x32, 64->128 on 16x64x64): the step's 3x3x3 weight
    // gradients 4.75 -> 4.46 ms (profiles/r04v_ab_wgrad3_cot.txt)
    static const int w3 = [] {  // nst,cot[,pixels per split / 64]
      const char* e = getenv("VDIFF_WGRAD3");
      int n = 2, c = 0, m = 32;
      if (e) sscanf(e, "%d,%d,%d", &n, &c, &m);
      return m * 1000000 + n * 1000 + c;
    }();
    const int w3_nst = w3 / 1000 % 1000, w3_msteps = w3 / 1000000;
    const int w3_c = w3 % 1000;
    const int w3_rw = rows <= 96 ? 96 : rows <= 128 ? 128 : 192;
    const bool w3_fill128 =
        (int64_t)vd_cdiv(d->Co, 128) * vd_cdiv(d->Ci, 64) * d->kt * d->kh *
            vd_cdiv(g.M, 64 * (int64_t)w3_msteps) * 10 >=
        9 * 256 * (int64_t)std::max(1, std::min(3, 163840 / ((w3_nst >= 3 ? 3 : 2) * (128 + w3_rw) * 128)));
    const int w3_cot = d->Co % 128 == 0 && (w3_c == 128 || (w3_c == 0 && w3_fill128)) ? 128 : 64;
    const int cot = one ? w1_cot : w3_cot;
    // nine-tap planes (VDIFF_CONV_WPLANE=1, A/B): image rows of whole 64-pixel steps
    static const int wplane = [] {
      const char* e = getenv("VDIFF_CONV_WPLANE");
      return e ? atoi(e) : 0;
    }();
    const bool plane = !one && wplane && d->Wo % 64 == 0;
    // (the K-split-wave and 128 x 128-tile forms of round 4 measured slower on every shape:
    // DESIGN section 4, removed in round 5)
    const int64_t tiles = (int64_t)vd_cdiv(d->Co, cot) * vd_cdiv(d->Ci, 64) *
                          (one ? 1 : (plane ? d->kt : d->kt * d->kh));
    // ~2048 workgroups, but at least 32 K steps each for the strip kernel (shorter pixel
    // ranges lose more to the ring's fill and the atomic epilogue than they gain in
    // occupancy: 64->64 at 128x128 0.13 -> 0.116 ms, tools/conv_ab.sh); planes do three
    // times the MFMA work per step: at least 16 steps
    int64_t splits = vd_cdiv(2048, tiles);
    int64_t maxs = vd_cdiv(g.M, (one || plane) ? 1024 : 64 * w3_msteps);
    if (splits > maxs) splits = maxs;
    // occupancy rounds (default since round 4; VDIFF_WGRAD_QRULE=0 turns it off, =c applies
    // it only where the rule above gives at most c splits): the grid of equal-length
    // workgroups runs in ceil(r) rounds of the resident slots (r = workgroups / slots), so
    // r = 1.5 pays for 2; take the fewest splits (down to a third) whose r >= 0.9 fills its
    // last round to >= 93 %, else the best fill (profiles/r04r_wgrad_split_sweep.txt: e.g.
    // 384->128 on 16x64x64 7 splits 217 us, 8 splits 263, the rule's 19 241).  The step's
    // weight gradients 5.81-5.93 -> 5.47-5.48 ms (profiles/r04u_ab_wgrad_qrule.txt)
    static const int wq = [] {
      const char* e = getenv("VDIFF_WGRAD_QRULE");
      return e ? atoi(e) : (1 << 30);
    }();
    if (wq > 0 && splits <= wq && !plane) {
      // resident workgroups per CU: LDS ring (160 KiB per CU) and registers (3 per CU for
      // the kw strip's 134-136 VGPRs)
      const int nst = one ? (cot >= 128 ? (w1_nst >= 4 ? 4 : 2)
                                        : (w1_nst >= 6 ? 6 : w1_nst >= 4 ? 4 : 2))
                          : (w3_nst >= 3 ? 3 : 2);
      const int ring = nst * (cot + (one ? 64 : (rows <= 96 ? 96 : rows <= 128 ? 128 : 192))) * 128;
      const int64_t slots = 256 * (int64_t)std::max(1, std::min(3, 163840 / ring));
      int64_t pick = 0, fill_pick = 0;
      double best_fill = -1.0;
      for (int64_t s = std::max<int64_t>(1, splits / 3); s <= splits; ++s) {
        const int64_t sr = vd_cdiv(g.M, vd_cdiv(vd_cdiv(g.M, s), 64) * 64);
        const double r = (double)(tiles * sr) / (double)slots;
        if (r < 0.9) continue;
        const double fill = r / std::ceil(r);
        if (fill >= 0.93) { pick = s; break; }
        if (fill > best_fill + 1e-9) { best_fill = fill; fill_pick = s; }
      }
      if (!pick) pick = fill_pick;
      if (pick) splits = pick;
    }
    // diagnostic (tools/wgrad_splits.py): VDIFF_WGRAD_SPLITS=s forces s pixel splits
    static const int wsplits = [] {
      const char* e = getenv("VDIFF_WGRAD_SPLITS");
      return e ? atoi(e) : 0;
    }();
    if (wsplits > 0) splits = std::min<int64_t>(wsplits, vd_cdiv(g.M, 64));
    if (splits < 1) splits = 1;
    g.m_per_split = vd_cdiv(vd_cdiv(g.M, splits), 64) * 64;
    splits = vd_cdiv(g.M, g.m_per_split);
    *splits_out = splits;
    if (dry) return VD_OK;
    dim3 grid((unsigned)tiles, (unsigned)splits);
    // XCD-aware 1-D grid (A/B knob VDIFF_WGRAD_XCD=0 restores the 2-D grid)
    static const int wxcd = [] {
      const char* e = getenv("VDIFF_WGRAD_XCD");
      return e ? atoi(e) : 1;
    }();
    if (wxcd && tiles > 1) {
      g.xcd_tiles = (int)tiles;
      g.xcd_total = (int)(tiles * splits);
      grid = dim3((unsigned)vd_cdiv(tiles * splits, 8) * 8, 1);
    }
#define VD_WGD(RW, COT, NST, ONE, ...)                                                     \
  do {                                                                                     \
    auto kern = wgrad_dma_kernel<RW, COT, NST, ONE, ##__VA_ARGS__>;                        \
    const int lds = NST * (COT + RW) * 128;                                                \
    (void)hipFuncSetAttribute((const void*)kern,                                           \
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);            \
    kern<<<grid, kThreads, lds, st>>>(g, wc, (const bf16_t*)x, (const bf16_t*)dy, dw);     \
  } while (0)
    // 64 x 64 tiles, double-buffered (40 KiB at RW = 96: three workgroups per CU).
    // Measured against COT = 128 and a three-stage ring: both slower (tools/conv_ab.sh).
#define VD_WG1(COT, NST)                                                                   \
  do {                                                                                     \
    /* 1x1: the compiler's read placement (early reads measured equal, 0.78 ms per step) */ \
    auto kern = wgrad_strip_kernel<64, COT, NST, 2, false>;                                \
    const int lds = NST * (COT + 64) * 128;                                                \
    (void)hipFuncSetAttribute((const void*)kern,                                           \
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);            \
    kern<<<grid, kThreads, lds, st>>>(g, wc, (const bf16_t*)x, (const bf16_t*)dy, dw);     \
  } while (0)
    // (KIND 0 needs whole-frame steps: Ho % (64 / Wo) == 0, else the round-5 kernel)
    const int wmode = g_wgrad_mode.load(std::memory_order_relaxed);
    const bool v2 = wmode >= 1 && (one || wc == 64 || d->Ho % (64 / wc) == 0);
    // early fragment reads for the kw strips (round 6: 3x3x3 3.88 -> 3.70 ms per step,
    // profiles/r06z2_wgrad3_ab_early_reads.txt); mode 2: the compiler's placement (A/B)
    const bool wer = wmode != 2;
    if (one && v2) {  // round 6: unrolled stages (the 1x1 form of wgrad_strip_kernel)
      if (cot == 192 && w1_nst >= 4) VD_WG1(192, 4);
      else if (cot == 192) VD_WG1(192, 2);
      else if (cot == 128 && w1_nst >= 4) VD_WG1(128, 4);
      else if (cot == 128) VD_WG1(128, 2);
      else if (w1_nst >= 6) VD_WG1(64, 6);
      else if (w1_nst >= 4) VD_WG1(64, 4);
      else VD_WG1(64, 2);
    }
#undef VD_WG1
    else if (one && cot == 192 && w1_nst >= 4) VD_WGD(64, 192, 4, true);
    else if (one && cot == 192) VD_WGD(64, 192, 2, true);
    else if (one && cot == 128 && w1_nst >= 4) VD_WGD(64, 128, 4, true);
    else if (one && cot == 128) VD_WGD(64, 128, 2, true);
    else if (one && w1_nst >= 6) VD_WGD(64, 64, 6, true);
    else if (one && w1_nst >= 4) VD_WGD(64, 64, 4, true);
    else if (one) VD_WGD(64, 64, 2, true);
    else if (plane) VD_WGD(224, 64, 2, false, true);
    else if (v2) {  // round 6: unrolled stages
#define VD_WGS(RW, COT, NST)                                                               \
  do {                                                                                     \
    auto kern = wc == 64 ? (wer ? wgrad_strip_kernel<RW, COT, NST, 1>                      \
                                : wgrad_strip_kernel<RW, COT, NST, 1, false>)              \
                         : (wer ? wgrad_strip_kernel<RW, COT, NST, 0>                      \
                                : wgrad_strip_kernel<RW, COT, NST, 0, false>);             \
    const int lds = NST * (COT + RW) * 128;                                                \
    (void)hipFuncSetAttribute((const void*)kern,                                           \
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);            \
    kern<<<grid, kThreads, lds, st>>>(g, wc, (const bf16_t*)x, (const bf16_t*)dy, dw);     \
  } while (0)
      if (cot == 128 && w3_nst >= 3 && rows <= 96) VD_WGS(96, 128, 3);
      else if (cot == 128 && w3_nst >= 3 && rows <= 128) VD_WGS(128, 128, 3);
      else if (cot == 128 && w3_nst >= 3) VD_WGS(192, 128, 3);
      else if (cot == 128 && rows <= 96) VD_WGS(96, 128, 2);
      else if (cot == 128 && rows <= 128) VD_WGS(128, 128, 2);
      else if (cot == 128) VD_WGS(192, 128, 2);
      else if (w3_nst >= 3 && rows <= 96) VD_WGS(96, 64, 3);
      else if (w3_nst >= 3 && rows <= 128) VD_WGS(128, 64, 3);
      else if (w3_nst >= 3) VD_WGS(192, 64, 3);
      else if (rows <= 96) VD_WGS(96, 64, 2);
      else if (rows <= 128) VD_WGS(128, 64, 2);
      else VD_WGS(192, 64, 2);
#undef VD_WGS
    }
    else if (cot == 128 && w3_nst >= 3 && rows <= 96) VD_WGD(96, 128, 3, false);
    else if (cot == 128 && w3_nst >= 3 && rows <= 128) VD_WGD(128, 128, 3, false);
    else if (cot == 128 && w3_nst >= 3) VD_WGD(192, 128, 3, false);
    else if (cot == 128 && rows <= 96) VD_WGD(96, 128, 2, false);
    else if (cot == 128 && rows <= 128) VD_WGD(128, 128, 2, false);
    else if (cot == 128) VD_WGD(192, 128, 2, false);
    else if (w3_nst >= 3 && rows <= 96) VD_WGD(96, 64, 3, false);
    else if (w3_nst >= 3 && rows <= 128) VD_WGD(128, 64, 3, false);
    else if (w3_nst >= 3) VD_WGD(192, 64, 3, false);
    else if (rows <= 96) VD_WGD(96, 64, 2, false);
    else if (rows <= 128) VD_WGD(128, 64, 2, false);
    else VD_WGD(192, 64, 2, false);
#undef VD_WGD
    return vd::check_launch("conv_wgrad_dma");
  }
  if (strip) {
    const int wc = d->Wo < 64 ? d->Wo : 64;
    const int rows = (64 / wc) * (wc + 2);
    const int64_t tiles = (int64_t)vd_cdiv(d->Co, 64) * vd_cdiv(d->Ci, 64) * d->kt * d->kh;
    int64_t splits = vd_cdiv(2048, tiles);
    int64_t maxs = vd_cdiv(g.M, 1024);
    if (splits > maxs) splits = maxs;
    if (splits < 1) splits = 1;
    g.m_per_split = vd_cdiv(vd_cdiv(g.M, splits), 64) * 64;
    splits = vd_cdiv(g.M, g.m_per_split);
    *splits_out = splits;
    if (dry) return VD_OK;
    dim3 grid((unsigned)tiles, (unsigned)splits);
#define VD_WG(RW)                                                                        \
  wgrad_bf16_kernel<RW><<<grid, kThreads, 2 * (64 + RW) * 72 * 2, st>>>(                \
      g, wc, (const bf16_t*)x, (const bf16_t*)dy, dw)
    if (rows <= 96) VD_WG(96);
    else if (rows <= 128) VD_WG(128);
    else VD_WG(192);
#undef VD_WG
    return vd::check_launch("conv_wgrad");
  }
  const int64_t tiles = (int64_t)vd_cdiv(d->Co, 64) * vd_cdiv(d->Ci, 64) * taps;
  // split the pixel reduction so the grid has ~2048 workgroups, >= 512 px each
  int64_t splits = vd_cdiv(2048, tiles);
  int64_t maxs = vd_cdiv(g.M, 512);
  if (splits > maxs) splits = maxs;
  if (splits < 1) splits = 1;
  g.m_per_split = vd_cdiv(vd_cdiv(g.M, splits), 32) * 32;
  splits = vd_cdiv(g.M, g.m_per_split);
  *splits_out = splits;
  if (dry) return VD_OK;
  return VD_DISPATCH_DTYPE(d->dtype, T, {
    constexpr int LD = 64 + (sizeof(T) == 2 ? 8 : 4);
    const size_t lds = 2 * 2 * 32 * LD * sizeof(T);
    conv_wgrad_kernel<T><<<dim3((unsigned)tiles, (unsigned)splits), kThreads, lds,
                           VD_STREAM(stream)>>>(g, (const T*)x, (const T*)dy, dw);
  });
}

// grid (ceil(n4 / 16)), 256 threads: 16 float4 outputs (4 consecutive ci of one (co, tap)
// row of the partials part[s][co][tap][ci]) x 16 split groups per workgroup.  Group k sums
// splits k, k + 16, ... in ascending order, then the 16 group sums are added in group order:
// a fixed summation order for a given split count (deterministic), with the splits' serial
// chain cut 16-fold (one thread per output had to walk all 128-256 splits of a 1x1 or
// narrow-N weight gradient: 77 vs 20 us at 64->64 x 262144 px, profiles/r04b_wgrad_*.log).
// Output in the torch weight layout out[co][ci][tap] (co < Co_out, ci < Ci_out).
__global__ __launch_bounds__(256) void wgrad_finish_kernel(const float* __restrict__ part,
                                                           int splits, int64_t sstride, int Ci,
                                                           int taps, int Co_out, int Ci_out,
                                                           float* __restrict__ out) {
  __shared__ float4 sums[16][17];
  const int oi = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int64_t i = (int64_t)blockIdx.x * 16 + oi;
  const int ci4 = Ci / 4;
  const int64_t n4 = (int64_t)Co_out * taps * ci4;
  const int64_t row = i / ci4;  // co * taps + tap
  const int ci = (int)(i % ci4) * 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  auto add = [&](const float4& v) {
    a.x += v.x;
    a.y += v.y;
    a.z += v.z;
    a.w += v.w;
  };
  if (i < n4 && ci < Ci_out) {
    const float* p = part + row * Ci + ci;
    // four of the group's splits in flight per iteration, added in the same ascending order
    // (round 6: the one-load-per-iteration loop waited a full memory latency per split;
    // bit-identical result)
    int sp = grp;
    for (; sp + 48 < splits; sp += 64) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = *reinterpret_cast<const float4*>(p + (int64_t)(sp + 16 * u) * sstride);
#pragma unroll
      for (int u = 0; u < 4; ++u) add(v[u]);
    }
    for (; sp < splits; sp += 16) add(*reinterpret_cast<const float4*>(p + (int64_t)sp * sstride));
  }
  sums[grp][oi] = a;
  __syncthreads();
  if (grp != 0 || i >= n4 || ci >= Ci_out) return;
  a = sums[0][oi];
  for (int k = 1; k < 16; ++k) {
    const float4 v = sums[k][oi];
    a.x += v.x;
    a.y += v.y;
    a.z += v.z;
    a.w += v.w;
  }
  const int tap = (int)(row % taps), co = (int)(row / taps);
  float* o = out + ((int64_t)co * Ci_out + ci) * taps + tap;
  const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (ci + k < Ci_out) o[(int64_t)k * taps] = av[k];
}

extern "C" {

int vd_conv3d_bwd_weight(const vd_conv_desc* d, const void* x, const void* dy, float* dw,
                         void* stream) {
  int64_t splits = 0;
  return wgrad_run(d, x, dy, dw, 0, &splits, false, stream);
}

size_t vd_conv3d_bwd_weight_workspace_size(const vd_conv_desc* d) {
  int64_t splits = 0;
  if (!d || wgrad_run(d, nullptr, nullptr, nullptr, 1, &splits, true, nullptr)) return 0;
  return (size_t)splits * d->Co * d->kt * d->kh * d->kw * d->Ci * sizeof(float) + 256;
}

int vd_conv3d_bwd_weight_det(const vd_conv_desc* d, const void* x, const void* dy, float* dw,
                             int Co_out, int Ci_out, void* workspace, size_t workspace_bytes,
                             void* stream) {
  int64_t splits = 0;
  int rc = wgrad_run(d, x, dy, nullptr, 1, &splits, true, stream);
  if (rc) return rc;
  VD_REQUIRE(x && dy && dw && workspace, "null tensor");
  VD_REQUIRE(Co_out > 0 && Co_out <= d->Co && Ci_out > 0 && Ci_out <= d->Ci,
             "dw extent %dx%d outside the descriptor's %dx%d", Co_out, Ci_out, d->Co, d->Ci);
  VD_REQUIRE(d->Ci % 4 == 0, "bwd_weight_det needs Ci %% 4 == 0 (got %d)", d->Ci);
  VD_REQUIRE((reinterpret_cast<uintptr_t>(workspace) & 15) == 0, "workspace not 16-B aligned");
  const int taps = d->kt * d->kh * d->kw;
  const int64_t sstride = (int64_t)d->Co * taps * d->Ci;
  VD_REQUIRE(workspace_bytes >= (size_t)splits * sstride * sizeof(float),
             "workspace %zu B < %lld B", workspace_bytes,
             (long long)(splits * sstride * (int64_t)sizeof(float)));
  float* part = reinterpret_cast<float*>(workspace);
  // every split writes every element of its slice (all co / ci tiles x taps, split ranges
  // non-empty: splits = ceil(M / m_per_split)), so the slices need no clearing
  rc = wgrad_run(d, x, dy, part, sstride, &splits, false, stream);
  if (rc) return rc;
  const int64_t n4 = (int64_t)Co_out * taps * (d->Ci / 4);
  wgrad_finish_kernel<<<(unsigned)vd_cdiv(n4, 16), 256, 0, VD_STREAM(stream)>>>(
      part, (int)splits, sstride, d->Ci, taps, Co_out, Ci_out, dw);
  return vd::check_launch("conv_wgrad_finish");
}

}  // extern "C"
