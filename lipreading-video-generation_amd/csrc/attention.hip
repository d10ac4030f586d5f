// attention.hip -- flash attention forward / backward on MFMA (gfx950).
//
// Replaces QKVAttentionLegacy.forward (reference unet.py:349-366) and
// QKVAttention.forward (unet.py:388-401): softmax(q k^T / sqrt(ch)) v with an
// fp32 softmax (unet.py:364), and its autograd backward (the reference
// recomputes the whole block under CheckpointFunction, utils.py:179-207).
// The N x N score matrix is never materialised; O(N) state (the row
// log-sum-exp) is saved instead.
//
// Sequence i of the descriptor starts at (i/groups)*batch_stride +
// (i%groups)*group_stride; tokens are token_stride apart.  This covers
// joint (all T*H*W tokens), spatial (per frame) and temporal (per pixel)
// attention over a channels-last [B][T][H][W][3C] qkv buffer without copies.
//
// Layout of the work (32x32 MFMA tiles, 64-wide waves):
//   forward  : WG = 4 waves x 32 queries; loop over 64-key tiles staged in
//              LDS.  S^T = K Q^T puts the query on the lane, so the online
//              softmax is per-lane; P^T is then the B operand of
//              O^T += V^T P^T straight from the accumulator registers; V^T
//              comes from the row-major V tile by ds_read_b64_tr_b16.
//   bwd dQ   : same tiling; recomputes P^T from the saved LSE, dP^T = V dO^T,
//              dS^T = P^T (dP^T - delta), dQ^T += K^T dS^T.
//   bwd dK,dV: WG = 4 waves x 32 keys; loop over 64-query tiles; S = Q K^T
//              and dP = dO V^T put the key on the lane; dV^T += dO^T P,
//              dK^T += Q^T dS.  No atomics: dQ and dK/dV are separate
//              passes, so the backward is deterministic.
// bf16: v_mfma_f32_32x32x16_bf16 (P / dS rounded to bf16 for the second
// product, fp32 softmax and accumulation).  fp32 parity mode:
// v_mfma_f32_32x32x2_f32 with the same structure (exact fp32 products).
#include "vd_common.h"
#include <math.h>

namespace {

constexpr int kThreads = 256;  // 4 waves
constexpr int kRows = 128;     // queries (fwd, dQ) or keys (dKdV) per workgroup
constexpr int kTile = 64;      // keys (fwd, dQ) or queries (dKdV) per LDS tile
constexpr float kLog2e = 1.4426950408889634f;

// ------------------------------------------------------------------ LDS tiles
// bf16 tile [64][D]: 16-B chunks XOR-swizzled per row so the 32-row fragment
// reads (ds_read_b128) hit distinct bank slots.  fp32 tile: rows of D+1 floats.
template <int D>
__device__ __forceinline__ int swz_row(int r) {
  if constexpr (D == 32) return (0x1320 >> (4 * ((r >> 2) & 3))) & 3;
  else if constexpr (D == 64) return (r >> 1) & 7;
  else return r & 15;
}
template <typename T, int D>
__device__ __forceinline__ int toff(int r, int c) {
  if constexpr (sizeof(T) == 2) return r * D + (((c >> 3) ^ swz_row<D>(r)) << 3) + (c & 7);
  else return r * (D + 1) + c;
}
template <typename T, int D>
constexpr int tile_elems() { return sizeof(T) == 2 ? kTile * D : kTile * (D + 1); }

// global rows [tok0, tok0+64) x [0, D) -> LDS tile (zero rows beyond n)
template <typename T, int D>
struct Stager {
  static constexpr int EPC = 16 / sizeof(T);
  static constexpr int CPR = D / EPC;
  static constexpr int NCH = kTile * CPR / kThreads;
  uint4 r[NCH > 0 ? NCH : 1];
  __device__ __forceinline__ void load(const T* base, int64_t ts, int tok0, int n, int tid) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int q = tid + i * kThreads;
      const int row = q / CPR, cc = q % CPR;
      const int tok = tok0 + row;
      r[i] = tok < n ? *reinterpret_cast<const uint4*>(base + (int64_t)tok * ts + cc * EPC)
                     : make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void store(T* tile, int tid) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int q = tid + i * kThreads;
      const int row = q / CPR, cc = q % CPR;
      if constexpr (sizeof(T) == 2) {
        *reinterpret_cast<uint4*>(tile + toff<T, D>(row, cc * EPC)) = r[i];
      } else {
        float* t = reinterpret_cast<float*>(tile) + toff<T, D>(row, cc * EPC);
        t[0] = __uint_as_float(r[i].x);
        t[1] = __uint_as_float(r[i].y);
        t[2] = __uint_as_float(r[i].z);
        t[3] = __uint_as_float(r[i].w);
      }
    }
  }
};

// ------------------------------------------------------------------ fragments
// B-operand fragments of 32 rows (row = lane&31) over the full D, from global.
template <typename T, int D> struct RowFrag;
template <int D> struct RowFrag<bf16_t, D> {
  bf16x8 f[D / 16];
  __device__ __forceinline__ void load(const bf16_t* base, int64_t ts, int tok, int n, int lane) {
    const int hh = lane >> 5;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      uint4 v = tok < n ? *reinterpret_cast<const uint4*>(base + (int64_t)tok * ts + 16 * s + 8 * hh)
                        : make_uint4(0, 0, 0, 0);
      f[s] = __builtin_bit_cast(bf16x8, v);
    }
  }
};
template <int D> struct RowFrag<float, D> {
  float f[D / 2];
  __device__ __forceinline__ void load(const float* base, int64_t ts, int tok, int n, int lane) {
    const int hh = lane >> 5;
#pragma unroll
    for (int s = 0; s < D / 2; ++s) f[s] = tok < n ? base[(int64_t)tok * ts + 2 * s + hh] : 0.f;
  }
};

// acc[32 rows of the LDS tile from row0][32 cols = fragment rows] over D
template <typename T, int D>
__device__ __forceinline__ void mma_rows(f32x16& acc, const T* tile, int row0,
                                         const RowFrag<T, D>& b, int lane) {
  const int r = row0 + (lane & 31), hh = lane >> 5;
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(tile + toff<T, D>(r, 16 * s + 8 * hh));
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b.f[s], acc, 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int s = 0; s < D / 2; ++s) {
      const float a = tile[toff<T, D>(r, 2 * s + hh)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b.f[s], acc, 0, 0, 0);
    }
  }
}

__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

// acc[32 tile cols from col0 (rows of the result)][32 lanes] +=
//   tile[sum0 .. sum0+32][col0 ..]^T  x  X, where X is a 32x32 accumulator whose
// ROW index (registers) is the summed index.
template <typename T, int D>
__device__ __forceinline__ void mma_tr(f32x16& acc, const T* tile, int sum0, int col0,
                                       const f32x16& X, int lane) {
  const int hh = lane >> 5;
  if constexpr (sizeof(T) == 2) {
    const int g = lane >> 4, fr = lane & 15;
    const int q4 = fr >> 2, p4 = fr & 3;
    const int col = col0 + 16 * (g & 1) + 4 * p4;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const uint4 w = make_uint4(pack_bf16(X[8 * s2 + 0], X[8 * s2 + 1]),
                                 pack_bf16(X[8 * s2 + 2], X[8 * s2 + 3]),
                                 pack_bf16(X[8 * s2 + 4], X[8 * s2 + 5]),
                                 pack_bf16(X[8 * s2 + 6], X[8 * s2 + 7]));
      const bf16x8 bop = __builtin_bit_cast(bf16x8, w);
      const int kr = sum0 + 16 * s2 + 4 * (g >> 1) + q4;
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_bf16x4*)(tile + toff<T, D>(kr, col)));
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_bf16x4*)(tile + toff<T, D>(kr + 8, col)));
      const bf16x8 aop = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aop, bop, acc, 0, 0, 0);
    }
  } else {
    const int c = col0 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float a = tile[toff<T, D>(sum0 + (r & 3) + 8 * (r >> 2) + 4 * hh, c)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, X[r], acc, 0, 0, 0);
    }
  }
}

// row index (0..31) of accumulator register r for this lane half
__device__ __forceinline__ int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

// write acc tiles (rows = d in [d0, d0 + 32*NT), lane = token) to out[tok][d] * mul
template <typename T, int NT>
__device__ __forceinline__ void store_transposed(T* base, int64_t ts, int tok, int n, int d0,
                                                 const f32x16 (&acc)[NT], float mul, int lane) {
  if (tok >= n) return;
  const int hh = lane >> 5;
  T* row = base + (int64_t)tok * ts;
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = d0 + 32 * i + 8 * g + 4 * hh;
      const float a = acc[i][4 * g] * mul, b = acc[i][4 * g + 1] * mul;
      const float c = acc[i][4 * g + 2] * mul, e = acc[i][4 * g + 3] * mul;
      if constexpr (sizeof(T) == 2) {
        *reinterpret_cast<uint2*>(row + d) = make_uint2(pack_bf16(a, b), pack_bf16(c, e));
      } else {
        *reinterpret_cast<float4*>(row + d) = make_float4(a, b, c, e);
      }
    }
}

struct SeqAddr {
  int64_t bs, gs;
  int groups;
  __device__ __forceinline__ int64_t operator()(int i) const {
    return (int64_t)(i / groups) * bs + (int64_t)(i % groups) * gs;
  }
};

template <typename T> constexpr int kStages = sizeof(T) == 2 ? 2 : 1;

// ================================================================== forward
template <typename T, int D>
__global__ __launch_bounds__(kThreads, 1) void attn_fwd_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, T* __restrict__ o,
    float* __restrict__ lse, int n, SeqAddr qa, int64_t ts, SeqAddr oa, int64_t ots, float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TE = tile_elems<T, D>();
  constexpr int ST = kStages<T>;
  T* lds = reinterpret_cast<T*>(smem);  // [ST][K, V]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5;
  const int seq = blockIdx.y;
  const int q0 = blockIdx.x * kRows + wave * 32;
  const int64_t base = qa(seq);
  const T* qb = q + base;
  const T* kb = k + base;
  const T* vb = v + base;
  const int myq = q0 + (lane & 31);

  RowFrag<T, D> qf;
  qf.load(qb, ts, myq, n, lane);
  f32x16 oacc[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) oacc[i] = f32x16{};
  float m = -INFINITY, l = 0.f;
  const float c = scale * kLog2e;

  Stager<T, D> sk, sv;
  const int ntiles = (n + kTile - 1) / kTile;
  sk.load(kb, ts, 0, n, tid);
  sv.load(vb, ts, 0, n, tid);
  sk.store(lds, tid);
  sv.store(lds + TE, tid);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int key0 = t * kTile;
    const bool more = t + 1 < ntiles;
    if (more) {
      sk.load(kb, ts, key0 + kTile, n, tid);
      sv.load(vb, ts, key0 + kTile, n, tid);
    }
    const T* Kt = lds + (t % ST) * 2 * TE;
    const T* Vt = Kt + TE;
    f32x16 s[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      s[h] = f32x16{};
      mma_rows<T, D>(s[h], Kt, 32 * h, qf, lane);
    }
    // online softmax in the log2 domain; keys on registers, query on the lane
    float tmax = -INFINITY;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = key0 + 32 * h + acc_row(r, hh);
        const float x = key < n ? s[h][r] * c : -INFINITY;
        s[h][r] = x;
        tmax = fmaxf(tmax, x);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mnew = fmaxf(m, tmax);
    const float alpha = exp2f(m - mnew);
    m = mnew;
    float psum = 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = exp2f(s[h][r] - mnew);
        s[h][r] = p;
        psum += p;
      }
    l = l * alpha + psum;
#pragma unroll
    for (int i = 0; i < D / 32; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[i][r] *= alpha;
#pragma unroll
    for (int i = 0; i < D / 32; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) mma_tr<T, D>(oacc[i], Vt, 32 * h, 32 * i, s[h], lane);
    if (ST == 1) __syncthreads();
    if (more) {
      T* nxt = lds + ((t + 1) % ST) * 2 * TE;
      sk.store(nxt, tid);
      sv.store(nxt + TE, tid);
    }
    __syncthreads();
  }
  l += __shfl_xor(l, 32, 64);
  const float inv = 1.f / l;
  store_transposed<T, D / 32>(o + oa(seq), ots, myq, n, 0, oacc, inv, lane);
  if (hh == 0 && myq < n) lse[(int64_t)seq * n + myq] = (m + log2f(l)) / kLog2e;
}

// ================================================================== delta = rowsum(dO * O)
template <typename T, int D>
__global__ void attn_delta_kernel(const T* __restrict__ o, const T* __restrict__ dout,
                                  float* __restrict__ delta, int nseq, int n, SeqAddr oa,
                                  int64_t ots) {
  const int64_t rows = (int64_t)nseq * n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int seq = (int)(i / n), tok = (int)(i % n);
    const int64_t off = oa(seq) + (int64_t)tok * ots;
    float acc = 0.f;
#pragma unroll 4
    for (int d = 0; d < D; d += 8) {
      float a[8], b[8];
      load8(o + off + d, a);
      load8(dout + off + d, b);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += a[e] * b[e];
    }
    delta[i] = acc;
  }
}

// ================================================================== backward: dQ
template <typename T, int D>
__global__ __launch_bounds__(kThreads, 1) void attn_bwd_dq_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v,
    const T* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ delta,
    T* __restrict__ dq, int n, SeqAddr qa, int64_t ts, SeqAddr oa, int64_t ots, float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TE = tile_elems<T, D>();
  constexpr int ST = kStages<T>;
  T* lds = reinterpret_cast<T*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5;
  const int seq = blockIdx.y;
  const int q0 = blockIdx.x * kRows + wave * 32;
  const int64_t base = qa(seq);
  const int myq = q0 + (lane & 31);
  const float c = scale * kLog2e;

  RowFrag<T, D> qf, of;
  qf.load(q + base, ts, myq, n, lane);
  of.load(dout + oa(seq), ots, myq, n, lane);
  const float lse2 = myq < n ? lse[(int64_t)seq * n + myq] * kLog2e : 0.f;
  const float dlt = myq < n ? delta[(int64_t)seq * n + myq] : 0.f;
  f32x16 acc[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) acc[i] = f32x16{};

  const T* kb = k + base;
  const T* vb = v + base;
  Stager<T, D> sk, sv;
  const int ntiles = (n + kTile - 1) / kTile;
  sk.load(kb, ts, 0, n, tid);
  sv.load(vb, ts, 0, n, tid);
  sk.store(lds, tid);
  sv.store(lds + TE, tid);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int key0 = t * kTile;
    const bool more = t + 1 < ntiles;
    if (more) {
      sk.load(kb, ts, key0 + kTile, n, tid);
      sv.load(vb, ts, key0 + kTile, n, tid);
    }
    const T* Kt = lds + (t % ST) * 2 * TE;
    const T* Vt = Kt + TE;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x16 s = f32x16{}, dp = f32x16{};
      mma_rows<T, D>(s, Kt, 32 * h, qf, lane);
      mma_rows<T, D>(dp, Vt, 32 * h, of, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = key0 + 32 * h + acc_row(r, hh);
        const float p = key < n ? exp2f(s[r] * c - lse2) : 0.f;
        s[r] = p * (dp[r] - dlt);  // dS^T
      }
#pragma unroll
      for (int i = 0; i < D / 32; ++i) mma_tr<T, D>(acc[i], Kt, 32 * h, 32 * i, s, lane);
    }
    if (ST == 1) __syncthreads();
    if (more) {
      T* nxt = lds + ((t + 1) % ST) * 2 * TE;
      sk.store(nxt, tid);
      sv.store(nxt + TE, tid);
    }
    __syncthreads();
  }
  store_transposed<T, D / 32>(dq + base, ts, myq, n, 0, acc, scale, lane);
}

// ================================================================== backward: dK, dV
// grid.z splits the OUTPUT columns of dK/dV in DO-wide slices (register budget
// at D = 256); S and dP always contract over the full D.
template <typename T, int D, int DO>
__global__ __launch_bounds__(kThreads, 1) void attn_bwd_dkdv_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v,
    const T* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ delta,
    T* __restrict__ dk, T* __restrict__ dv, int n, SeqAddr qa, int64_t ts, SeqAddr oa,
    int64_t ots, float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TE = tile_elems<T, D>();
  constexpr int ST = kStages<T>;
  T* lds = reinterpret_cast<T*>(smem);  // [ST][Q, dO]
  float* rowc = reinterpret_cast<float*>(smem + (size_t)ST * 2 * TE * sizeof(T));  // [ST][2][64]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5;
  const int seq = blockIdx.y;
  const int d0 = blockIdx.z * DO;
  const int k0 = blockIdx.x * kRows + wave * 32;
  const int64_t base = qa(seq), obase = oa(seq);
  const int mykey = k0 + (lane & 31);
  const float c = scale * kLog2e;

  RowFrag<T, D> kf, vf;
  kf.load(k + base, ts, mykey, n, lane);
  vf.load(v + base, ts, mykey, n, lane);
  f32x16 adv[DO / 32], adk[DO / 32];
#pragma unroll
  for (int i = 0; i < DO / 32; ++i) adv[i] = adk[i] = f32x16{};

  const T* qb = q + base;
  const T* ob = dout + obase;
  const float* lrow = lse + (int64_t)seq * n;
  const float* drow = delta + (int64_t)seq * n;
  Stager<T, D> sq, so;
  float rl = 0.f, rd = 0.f;
  auto load_rows = [&](int tok0) {
    if (tid < kTile) {
      const int tk = tok0 + tid;
      rl = tk < n ? lrow[tk] * kLog2e : 0.f;
      rd = tk < n ? drow[tk] : 0.f;
    }
  };
  auto store_rows = [&](int stage) {
    if (tid < kTile) {
      rowc[stage * 128 + tid] = rl;
      rowc[stage * 128 + 64 + tid] = rd;
    }
  };
  const int ntiles = (n + kTile - 1) / kTile;
  sq.load(qb, ts, 0, n, tid);
  so.load(ob, ots, 0, n, tid);
  load_rows(0);
  sq.store(lds, tid);
  so.store(lds + TE, tid);
  store_rows(0);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int qt0 = t * kTile;
    const bool more = t + 1 < ntiles;
    if (more) {
      sq.load(qb, ts, qt0 + kTile, n, tid);
      so.load(ob, ots, qt0 + kTile, n, tid);
      load_rows(qt0 + kTile);
    }
    const int stage = t % ST;
    const T* Qt = lds + stage * 2 * TE;
    const T* Ot = Qt + TE;
    const float* L = rowc + stage * 128;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x16 s = f32x16{}, dp = f32x16{};
      mma_rows<T, D>(s, Qt, 32 * h, kf, lane);   // S[q][key]
      mma_rows<T, D>(dp, Ot, 32 * h, vf, lane);  // dP[q][key]
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ql = 32 * h + acc_row(r, hh);
        const bool ok = qt0 + ql < n && mykey < n;
        const float p = ok ? exp2f(s[r] * c - L[ql]) : 0.f;
        s[r] = p;
        dp[r] = p * (dp[r] - L[64 + ql]);  // dS
      }
#pragma unroll
      for (int i = 0; i < DO / 32; ++i) {
        mma_tr<T, D>(adv[i], Ot, 32 * h, d0 + 32 * i, s, lane);   // dV^T += dO^T P
        mma_tr<T, D>(adk[i], Qt, 32 * h, d0 + 32 * i, dp, lane);  // dK^T += Q^T dS
      }
    }
    if (ST == 1) __syncthreads();
    if (more) {
      const int ns = (t + 1) % ST;
      T* nxt = lds + ns * 2 * TE;
      sq.store(nxt, tid);
      so.store(nxt + TE, tid);
      store_rows(ns);
    }
    __syncthreads();
  }
  store_transposed<T, DO / 32>(dk + base, ts, mykey, n, d0, adk, scale, lane);
  store_transposed<T, DO / 32>(dv + base, ts, mykey, n, d0, adv, 1.f, lane);
}

// ------------------------------------------------------------------ launchers
int check_attn(const vd_attn_desc* d) {
  VD_REQUIRE(d, "null descriptor");
  VD_REQUIRE(d->nseq > 0 && d->seq_len > 0 && d->groups > 0, "bad attention shape");
  VD_REQUIRE(d->head_dim == 32 || d->head_dim == 64 || d->head_dim == 128 || d->head_dim == 256,
             "head_dim %d unsupported (32/64/128/256)", d->head_dim);
  return VD_OK;
}

template <typename T, int D>
int fwd_impl(const vd_attn_desc* d, const void* q, const void* k, const void* v, void* o,
             float* lse, hipStream_t st) {
  const size_t lds = (size_t)kStages<T> * 2 * tile_elems<T, D>() * sizeof(T);
  auto kern = attn_fwd_kernel<T, D>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  dim3 grid((unsigned)vd_cdiv(d->seq_len, kRows), (unsigned)d->nseq);
  kern<<<grid, kThreads, lds, st>>>((const T*)q, (const T*)k, (const T*)v, (T*)o, lse,
                                    d->seq_len, SeqAddr{d->batch_stride, d->group_stride, d->groups},
                                    d->token_stride,
                                    SeqAddr{d->o_batch_stride, d->o_group_stride, d->groups},
                                    d->o_token_stride, d->scale);
  return vd::check_launch("attn_fwd");
}

template <typename T, int D>
int bwd_dq_impl(const vd_attn_desc* d, const void* q, const void* k, const void* v, const void* o,
                const void* dout, const float* lse, void* dq, void* ws, hipStream_t st) {
  const SeqAddr qa{d->batch_stride, d->group_stride, d->groups};
  const SeqAddr oa{d->o_batch_stride, d->o_group_stride, d->groups};
  float* delta = reinterpret_cast<float*>(ws);
  const int64_t rows = (int64_t)d->nseq * d->seq_len;
  int g = (int)vd_cdiv(rows, 256);
  if (g > 4096) g = 4096;
  attn_delta_kernel<T, D><<<g, 256, 0, st>>>((const T*)o, (const T*)dout, delta, d->nseq,
                                              d->seq_len, oa, d->o_token_stride);
  int rc = vd::check_launch("attn_delta");
  if (rc) return rc;
  const size_t lds = (size_t)kStages<T> * 2 * tile_elems<T, D>() * sizeof(T);
  auto kern = attn_bwd_dq_kernel<T, D>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  dim3 grid((unsigned)vd_cdiv(d->seq_len, kRows), (unsigned)d->nseq);
  kern<<<grid, kThreads, lds, st>>>((const T*)q, (const T*)k, (const T*)v, (const T*)dout, lse,
                                    delta, (T*)dq, d->seq_len, qa, d->token_stride, oa,
                                    d->o_token_stride, d->scale);
  return vd::check_launch("attn_bwd_dq");
}

template <typename T, int D>
int bwd_dkdv_impl(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                  const void* dout, const float* lse, void* dk, void* dv, void* ws,
                  hipStream_t st) {
  const SeqAddr qa{d->batch_stride, d->group_stride, d->groups};
  const SeqAddr oa{d->o_batch_stride, d->o_group_stride, d->groups};
  const float* delta = reinterpret_cast<const float*>(ws);
  constexpr int DO = D > 128 ? 128 : D;
  const size_t lds = (size_t)kStages<T> * 2 * tile_elems<T, D>() * sizeof(T) +
                     (size_t)kStages<T> * 128 * sizeof(float);
  auto kern = attn_bwd_dkdv_kernel<T, D, DO>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  dim3 grid((unsigned)vd_cdiv(d->seq_len, kRows), (unsigned)d->nseq, D / DO);
  kern<<<grid, kThreads, lds, st>>>((const T*)q, (const T*)k, (const T*)v, (const T*)dout, lse,
                                    delta, (T*)dk, (T*)dv, d->seq_len, qa, d->token_stride, oa,
                                    d->o_token_stride, d->scale);
  return vd::check_launch("attn_bwd_dkdv");
}

#define VD_DISPATCH_HEAD(D_, FN, ...)                        \
  switch (D_) {                                              \
    case 32: return FN<T, 32>(__VA_ARGS__);                  \
    case 64: return FN<T, 64>(__VA_ARGS__);                  \
    case 128: return FN<T, 128>(__VA_ARGS__);                \
    case 256: return FN<T, 256>(__VA_ARGS__);                \
    default: return vd::fail(VD_EUNSUPPORTED, "head_dim");   \
  }

}  // namespace

extern "C" {

int vd_attention_fwd(const vd_attn_desc* d, const void* q, const void* k, const void* v, void* o,
                     float* lse, void* stream) {
  int rc = check_attn(d);
  if (rc) return rc;
  VD_REQUIRE(q && k && v && o && lse, "null tensor");
  hipStream_t st = VD_STREAM(stream);
  if (d->dtype == VD_BF16) {
    using T = bf16_t;
    VD_DISPATCH_HEAD(d->head_dim, fwd_impl, d, q, k, v, o, lse, st);
  } else if (d->dtype == VD_F32) {
    using T = float;
    VD_DISPATCH_HEAD(d->head_dim, fwd_impl, d, q, k, v, o, lse, st);
  }
  return vd::fail(VD_EUNSUPPORTED, "dtype %d", d->dtype);
}

size_t vd_attention_bwd_workspace_size(const vd_attn_desc* d) {
  if (!d || d->nseq <= 0 || d->seq_len <= 0) return 0;
  return (size_t)d->nseq * d->seq_len * sizeof(float) + 256;
}

int vd_attention_bwd_dq(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                        const void* o, const void* dout, const float* lse, void* dq,
                        void* workspace, void* stream) {
  int rc = check_attn(d);
  if (rc) return rc;
  VD_REQUIRE(q && k && v && o && dout && lse && dq && workspace, "null tensor");
  hipStream_t st = VD_STREAM(stream);
  if (d->dtype == VD_BF16) {
    using T = bf16_t;
    VD_DISPATCH_HEAD(d->head_dim, bwd_dq_impl, d, q, k, v, o, dout, lse, dq, workspace, st);
  } else if (d->dtype == VD_F32) {
    using T = float;
    VD_DISPATCH_HEAD(d->head_dim, bwd_dq_impl, d, q, k, v, o, dout, lse, dq, workspace, st);
  }
  return vd::fail(VD_EUNSUPPORTED, "dtype %d", d->dtype);
}

int vd_attention_bwd_dkdv(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                          const void* dout, const float* lse, void* dk, void* dv, void* workspace,
                          void* stream) {
  int rc = check_attn(d);
  if (rc) return rc;
  VD_REQUIRE(q && k && v && dout && lse && dk && dv && workspace, "null tensor");
  hipStream_t st = VD_STREAM(stream);
  if (d->dtype == VD_BF16) {
    using T = bf16_t;
    VD_DISPATCH_HEAD(d->head_dim, bwd_dkdv_impl, d, q, k, v, dout, lse, dk, dv, workspace, st);
  } else if (d->dtype == VD_F32) {
    using T = float;
    VD_DISPATCH_HEAD(d->head_dim, bwd_dkdv_impl, d, q, k, v, dout, lse, dk, dv, workspace, st);
  }
  return vd::fail(VD_EUNSUPPORTED, "dtype %d", d->dtype);
}

int vd_attention_bwd(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                     const void* o, const void* dout, const float* lse, void* dq, void* dk,
                     void* dv, void* workspace, void* stream) {
  int rc = vd_attention_bwd_dq(d, q, k, v, o, dout, lse, dq, workspace, stream);
  if (rc) return rc;
  return vd_attention_bwd_dkdv(d, q, k, v, dout, lse, dk, dv, workspace, stream);
}

}  // extern "C"
