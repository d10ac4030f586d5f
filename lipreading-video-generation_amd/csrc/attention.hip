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
#include "vd_asm.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <type_traits>

namespace {

// A workgroup is NW waves (4 or 8); each wave owns NB x 32 rows (queries for fwd / dQ,
// keys for dK/dV), so a workgroup covers 32 * NB * NW rows and shares every LDS tile
// among its NW waves.
constexpr int kTile = 64;      // keys (fwd, dQ) or queries (dKdV) per LDS tile
constexpr float kLog2e = 1.4426950408889634f;

// Diagnostic build only (-DVD_ATTN_STAMPS, tools/attn_stamps.py): s_memtime stamps of
// lane 0 of every wave of workgroups 0..63 (grid row 0) for the first 64 tiles.
#ifdef VD_ATTN_STAMPS
__device__ unsigned long long g_stamps[64][8][4][64];
#define VD_STAMP(kind, t)                                                                   \
  do {                                                                                      \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 64 && blockIdx.y == 0 && (t) < 64)         \
      g_stamps[blockIdx.x][threadIdx.x >> 6][kind][t] = __builtin_amdgcn_s_memtime();      \
  } while (0)
#else
#define VD_STAMP(kind, t) \
  do {                    \
  } while (0)
#endif

// ------------------------------------------------------------------ LDS tiles
// bf16 tile [64][D]: 16-B chunks XOR-swizzled per row.  Two read shapes must both be
// conflict-free (bank = byte/4 mod 64, MI355X_MICROARCH.md "LDS"):
//  * ds_read_b128 row fragments: a 16-lane group reads one chunk of 16 rows
//    {0-3,12-15,20-27} or {4-11,16-19,28-31} (+32) -> those rows need distinct slots;
//  * ds_read_b64_tr_b16: a 32-lane group reads 4 consecutive chunks of rows 4m..4m+3
//    -> the four 64-B pieces must fall in different quarters of the 256-B bank line.
// D = 64 (two rows per bank line): bit 2 of the XOR alternates between rows 4m and 4m+2;
// D >= 128: bits 2-3 of the XOR are r & 3.  fp32 tile: rows of D+1 floats.
template <int D>
__device__ __forceinline__ int swz_row(int r) {
  if constexpr (D == 32) return (0x1320 >> (4 * ((r >> 2) & 3))) & 3;
  else if constexpr (D == 64) return (((r >> 1) & 1) << 2) | ((r >> 2) & 3);
  else return ((r & 3) << 2) | ((r >> 2) & 3);
}
template <typename T, int D>
__device__ __forceinline__ int toff(int r, int c) {
  if constexpr (sizeof(T) == 2) return r * D + (((c >> 3) ^ swz_row<D>(r)) << 3) + (c & 7);
  else return r * (D + 1) + c;
}
template <typename T, int D>
constexpr int tile_elems() { return sizeof(T) == 2 ? kTile * D : kTile * (D + 1); }

// global rows [tok0, tok0+64) x [0, D) -> LDS tile (zero rows beyond n)
template <typename T, int D, int NW>
struct Stager {
  static constexpr int EPC = 16 / sizeof(T);
  static constexpr int CPR = D / EPC;
  static constexpr int NCH = kTile * CPR / (64 * NW);
  uint4 r[NCH > 0 ? NCH : 1];
  __device__ __forceinline__ void load(const T* base, int64_t ts, int tok0, int n, int tid) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int q = tid + i * 64 * NW;
      const int row = q / CPR, cc = q % CPR;
      const int tok = tok0 + row;
      r[i] = tok < n ? *reinterpret_cast<const uint4*>(base + (int64_t)tok * ts + cc * EPC)
                     : make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void store(T* tile, int tid) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int q = tid + i * 64 * NW;
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
  // pre-multiply by the softmax scale (x log2 e): the MFMA then emits S in log2 units, so
  // no per-element scaling is left in the softmax (one extra bf16 rounding of the operand)
  __device__ __forceinline__ void scale(float c) {
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      const uint4 w = __builtin_bit_cast(uint4, f[s]);
      const uint32_t in[4] = {w.x, w.y, w.z, w.w};
      uint32_t out[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        out[e] = pack2bf(__uint_as_float(in[e] << 16) * c, __uint_as_float(in[e] & 0xffff0000u) * c);
      f[s] = __builtin_bit_cast(bf16x8, make_uint4(out[0], out[1], out[2], out[3]));
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
  __device__ __forceinline__ void scale(float c) {
#pragma unroll
    for (int s = 0; s < D / 2; ++s) f[s] *= c;
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

__device__ __forceinline__ uint32_t pack_bf16(float a, float b) { return pack2bf(a, b); }

// A 32x32 accumulator X used as the B operand of a following product (its ROW
// index, in registers, is the summed index; SS 3 of the HIP guide): bf16 packs it
// once into two 16-deep k-step fragments, fp32 keeps the registers.
template <typename T> struct XOp;
template <> struct XOp<bf16_t> {
  bf16x8 b[2];
  XOp() = default;
  __device__ __forceinline__ explicit XOp(const f32x16& X) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const uint4 w = make_uint4(pack_bf16(X[8 * s2 + 0], X[8 * s2 + 1]),
                                 pack_bf16(X[8 * s2 + 2], X[8 * s2 + 3]),
                                 pack_bf16(X[8 * s2 + 4], X[8 * s2 + 5]),
                                 pack_bf16(X[8 * s2 + 6], X[8 * s2 + 7]));
      b[s2] = __builtin_bit_cast(bf16x8, w);
    }
  }
};
template <> struct XOp<float> {
  f32x16 x;
  XOp() = default;
  __device__ __forceinline__ explicit XOp(const f32x16& X) : x(X) {}
};

// acc[32 tile cols from col0 (rows of the result)][32 lanes] +=
//   tile[sum0 .. sum0+32][col0 ..]^T  x  X
template <typename T, int D>
__device__ __forceinline__ void mma_tr(f32x16& acc, const T* tile, int sum0, int col0,
                                       const XOp<T>& X, int lane) {
  const int hh = lane >> 5;
  if constexpr (sizeof(T) == 2) {
    const int g = lane >> 4, fr = lane & 15;
    const int q4 = fr >> 2, p4 = fr & 3;
    const int col = col0 + 16 * (g & 1) + 4 * p4;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 bop = X.b[s2];
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
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, X.x[r], acc, 0, 0, 0);
    }
  }
}

// NB-block forms: one LDS fragment read feeds NB MFMAs (NB 32-row blocks per wave), which
// halves the LDS bytes per FLOP at NB = 2 -- the fragment reads, not the MFMAs, bound the
// single-block kernels.
template <typename T, int D, int NB>
__device__ __forceinline__ void mma_rows_nb(f32x16 (&acc)[NB], const T* tile, int row0,
                                            const RowFrag<T, D> (&b)[NB], int lane) {
  const int r = row0 + (lane & 31), hh = lane >> 5;
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(tile + toff<T, D>(r, 16 * s + 8 * hh));
#pragma unroll
      for (int j = 0; j < NB; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[j].f[s], acc[j], 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int s = 0; s < D / 2; ++s) {
      const float a = tile[toff<T, D>(r, 2 * s + hh)];
#pragma unroll
      for (int j = 0; j < NB; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b[j].f[s], acc[j], 0, 0, 0);
    }
  }
}

template <typename T, int D, int NB>
__device__ __forceinline__ void mma_tr_nb(f32x16 (&acc)[NB], const T* tile, int sum0, int col0,
                                          const XOp<T> (&X)[NB], int lane) {
  const int hh = lane >> 5;
  if constexpr (sizeof(T) == 2) {
    const int g = lane >> 4, fr = lane & 15;
    const int q4 = fr >> 2, p4 = fr & 3;
    const int col = col0 + 16 * (g & 1) + 4 * p4;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int kr = sum0 + 16 * s2 + 4 * (g >> 1) + q4;
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_bf16x4*)(tile + toff<T, D>(kr, col)));
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_bf16x4*)(tile + toff<T, D>(kr + 8, col)));
      const bf16x8 aop = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
      for (int j = 0; j < NB; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aop, X[j].b[s2], acc[j], 0, 0, 0);
    }
  } else {
    const int c = col0 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float a = tile[toff<T, D>(sum0 + (r & 3) + 8 * (r >> 2) + 4 * hh, c)];
#pragma unroll
      for (int j = 0; j < NB; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, X[j].x[r], acc[j], 0, 0, 0);
    }
  }
}

// The two k16 A-operand steps of tile[sum0 .. sum0+32][col0 .. col0+32]^T (as mma_tr reads
// them), into registers.
template <int D>
__device__ __forceinline__ void load_tr(bf16x8 (&f)[2], const bf16_t* tile, int sum0, int col0,
                                        int lane) {
  const int g = lane >> 4, fr = lane & 15;
  const int q4 = fr >> 2, p4 = fr & 3;
  const int col = col0 + 16 * (g & 1) + 4 * p4;
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int kr = sum0 + 16 * s2 + 4 * (g >> 1) + q4;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_bf16x4*)(tile + toff<bf16_t, D>(kr, col)));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_bf16x4*)(tile + toff<bf16_t, D>(kr + 8, col)));
    f[s2] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}
template <int D>
__device__ __forceinline__ void load_tr(bf16x8 (&f)[2], const float*, int, int, int) {}

#ifdef VD_ATTN_NOPRELOAD
constexpr bool kPreload = false;
#else
constexpr bool kPreload = true;
#endif

// v_exp_f32 directly (inputs here are <= 0 or -inf; no range reduction needed)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

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

// The K/V rows of sequence i: self-attention uses the query's own addressing; cross-
// attention (vd_cross_attention_*) has a K/V buffer of its own, with its own length and
// strides (e.g. the audio tokens of a frame).
struct KvAddr {
  SeqAddr a;
  int64_t ts;  // token stride of the K/V rows
  int n;       // K/V rows per sequence
};


// ------------------------------------------------------------------ tile pipelines
// bf16: LDS ring of NST stages filled by buffer_load ... lds (LDS-DMA, no register
// staging).  The buffer range check zero-fills rows past the sequence end.  Tile t+NST-1
// is issued at the top of iteration t, so NST-1 tiles are in flight while tile t is
// computed; one raw s_barrier per tile, behind a counted vmcnt (never vmcnt(0) in the
// loop: __syncthreads() would drain the ring).
// fp32 (parity mode): one register-staged stage (rows of D+1 floats).

template <typename T> constexpr bool kDMA = sizeof(T) == 2;

template <int D> constexpr int nstage() { return D <= 64 ? 4 : (D == 128 ? 3 : 2); }
// DMA instructions (1 KiB each) per wave per tile
template <int D, int NW, int TR = kTile> constexpr int dma_ipw() { return TR * D * 2 / 1024 / NW; }

// this wave's share of one [TR x D] bf16 tile: logical 16-B chunk c of row r lands at the
// swizzled position toff(r, 8c) (the DMA writes lane-linearly, so the SOURCE chunk is
// permuted by the same involution)
template <int D, int NW, int TR = kTile>
__device__ __forceinline__ void dma_tile(rsrc_t rs, char* lds, int tok0, int n,
                                         uint32_t ts_bytes, int wave, int lane) {
  constexpr int CPL = D / 8, RPI = 64 / CPL, IPW = dma_ipw<D, NW, TR>();
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int gi = wave * IPW + i;
    const int row = gi * RPI + lane / CPL;
    const int c = (lane % CPL) ^ swz_row<D>(row);
    const int tok = tok0 + row;
    const uint32_t voff = tok < n ? (uint32_t)tok * ts_bytes + (uint32_t)c * 16u : 0x80000000u;
    dma_lds<16>(rs, lds_addr(lds + gi * 1024), voff);
  }
}

// 64 fp32 row constants (one dword per lane)
__device__ __forceinline__ void dma_rowc(rsrc_t rs, char* lds, int tok0, int lane) {
  dma_lds<4>(rs, lds_addr(lds), (uint32_t)(tok0 + lane) * 4u);
}

__device__ __forceinline__ uint32_t seq_bytes(int n, int64_t ts, int D, int esz) {
  return (uint32_t)(((int64_t)(n - 1) * ts + D) * esz);
}

// Runs body(t, tileA, tileB) over all 64-row tiles of two row streams (a, b) of one
// sequence; with RC, the fp32 row constants rc0/rc1 of the tile are staged too and
// passed as body's fourth argument (float* [rc0 64 | rc1 64]).
template <typename T, int D, bool RC, int NW, int NSTO = 0, typename Body>
__device__ __forceinline__ void tile_loop(char* smem, const T* a, const T* b, int64_t ts_a,
                                          int64_t ts_b, const float* rc0, const float* rc1, int n,
                                          int tid, Body&& body) {
  constexpr int TE = tile_elems<T, D>();
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntiles = (n + kTile - 1) / kTile;
  if constexpr (kDMA<T>) {
    constexpr int NST = NSTO ? NSTO : nstage<D>();  // NSTO: ring stages override
    constexpr int STAGE_BYTES = 2 * TE * 2 + (RC ? 768 : 0);
    constexpr int PER_TILE = 2 * dma_ipw<D, NW>() + (RC ? 1 : 0);
    const auto ra = make_rsrc(a, seq_bytes(n, ts_a, D, 2));
    const auto rb = make_rsrc(b, seq_bytes(n, ts_b, D, 2));
    rsrc_t r0, r1;
    if constexpr (RC) {
      r0 = make_rsrc(rc0, (uint32_t)n * 4u);
      r1 = make_rsrc(rc1, (uint32_t)n * 4u);
    }
    const uint32_t tsa = (uint32_t)(ts_a * 2), tsb = (uint32_t)(ts_b * 2);
    auto issue = [&](int t) {
      char* st = smem + (t % NST) * STAGE_BYTES;
      const int tok0 = t * kTile;
      dma_tile<D, NW>(ra, st, tok0, n, tsa, wave, lane);
      dma_tile<D, NW>(rb, st + TE * 2, tok0, n, tsb, wave, lane);
      if constexpr (RC) {  // waves 0/1 stage the two constants, the others a throw-away copy
        // (every wave issues the same number of DMAs, so one vmcnt fits all)
        char* rcs = st + 4 * TE + (wave < 2 ? wave * 256 : 512);
        dma_rowc(wave == 1 ? r1 : r0, rcs, tok0, lane);
      }
    };
    vm_drain();  // fragments loaded before the loop are in; the ring's counts start clean
#pragma unroll
    for (int s = 0; s < NST - 1; ++s) issue(s);
    for (int t = 0; t < ntiles; ++t) {
      VD_STAMP(0, t);
      vm_wait_barrier<(NST - 2) * PER_TILE>();
      VD_STAMP(1, t);
      issue(t + NST - 1);  // beyond the end: fully out-of-range rows (zero fill, no traffic)
      const char* st = smem + (t % NST) * STAGE_BYTES;
      body(t, reinterpret_cast<const T*>(st), reinterpret_cast<const T*>(st + TE * 2),
           reinterpret_cast<const float*>(st + 4 * TE));
      VD_STAMP(3, t);
    }
    vm_drain();
  } else {
    T* lds = reinterpret_cast<T*>(smem);
    float* rcl = reinterpret_cast<float*>(smem + 2 * TE * sizeof(T));
    Stager<T, D, NW> sa, sb;
    float v0 = 0.f, v1 = 0.f;
    auto ldrc = [&](int tok0) {
      if constexpr (RC) {
        if (tid < kTile) {
          v0 = tok0 + tid < n ? rc0[tok0 + tid] : 0.f;
          v1 = tok0 + tid < n ? rc1[tok0 + tid] : 0.f;
        }
      }
    };
    auto strc = [&]() {
      if constexpr (RC) {
        if (tid < kTile) {
          rcl[tid] = v0;
          rcl[64 + tid] = v1;
        }
      }
    };
    sa.load(a, ts_a, 0, n, tid);
    sb.load(b, ts_b, 0, n, tid);
    ldrc(0);
    sa.store(lds, tid);
    sb.store(lds + TE, tid);
    strc();
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
      const bool more = t + 1 < ntiles;
      if (more) {
        sa.load(a, ts_a, (t + 1) * kTile, n, tid);
        sb.load(b, ts_b, (t + 1) * kTile, n, tid);
        ldrc((t + 1) * kTile);
      }
      body(t, lds, lds + TE, rcl);
      __syncthreads();
      if (more) {
        sa.store(lds, tid);
        sb.store(lds + TE, tid);
        strc();
      }
      __syncthreads();
    }
  }
}

// Software-pipelined ring (bf16, D <= 128).  Work is cut into 32-row blocks (two per
// 64-row tile); per block a kernel has an MFMA step M (this block's S / dP products plus
// the gradient / PV products of the PREVIOUS block) and a VALU step V (softmax of this
// block).  Program order per wave is M(0) V(0) M(1) V(1) ... G(last): M(b+1)'s MFMAs do
// not depend on V(b), so the MFMA pipe and the VALU stay busy together.  With 8 waves the
// SIMD partners (waves w and w+4) take the tile barrier at different points of that
// sequence -- waves 0-3 run [M V M V] between barriers, waves 4-7 [V M V M] -- so one
// partner's MFMAs run beside the other's softmax instead of in lockstep with it.
// Four stages, prefetch distance 2: tiles t and t-1 are read while t+1, t+2 land.
// S(b): the block's S / dP products; G(b): its gradient / PV products (needs V(b));
// V(b): its softmax.  Order: S(2t) G(2t-1) V(2t) S(2t+1) G(2t) V(2t+1).
template <typename T> struct BlockRef {
  const T* a;       // stream a rows of the block's tile (K for fwd / dQ, Q for dK/dV)
  const T* b;       // stream b rows (V, or dO)
  const float* rc;  // row constants of the tile (dK/dV): rc0 rows ...
  const float* rc1; // ... and rc1 rows
  int row0;         // 0, 32 (, 64, 96): the block's rows within its tile
  int idx;          // block index: rows [32 idx, 32 idx + 32) of the sequence
};

// Optional instruction-group schedule for one block (IGroupLP sched_group_barrier):
// SR LDS reads, SM MFMAs (S), GR LDS reads, then GM x {1 MFMA (G), VP VALU (softmax)}.
// All zero: leave the order to the compiler.
template <int SR, int SM, int GR, int GM, int VP> struct BlockSched {
  static constexpr bool on = SM > 0;
  __device__ __forceinline__ static void emit() {
    if constexpr (SM > 0) {
      __builtin_amdgcn_sched_group_barrier(0x100, SR, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, SM, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, GR, 0);
#pragma unroll
      for (int i = 0; i < GM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, VP, 0);
      }
    }
  }
};
using NoSched = BlockSched<0, 0, 0, 0, 0>;

// TR: rows per LDS tile (64, or 128 = four blocks per tile, half the barriers per row).
// Row constants (RC) of a tile: rc0 [TR floats] | rc1 [TR floats] | a 256-B throw-away slot.
template <int D, bool RC, int TR = kTile>
constexpr int pipe_stage_bytes() { return 2 * TR * D * 2 + (RC ? 2 * TR * 4 + 256 : 0); }

#ifndef VD_PIPE_UNROLL
#define VD_PIPE_UNROLL 1
#endif
template <typename T, int D, bool RC, int NW, typename SCH = NoSched, int TR = kTile,
          typename SF, typename GF, typename VF>
__device__ __forceinline__ void tile_pipe(char* smem, const T* a, const T* b, int64_t ts_a,
                                          int64_t ts_b, const float* rc0, const float* rc1,
                                          int n, int tid, bool late, SF&& S, GF&& G, VF&& V) {
  static_assert(kDMA<T> && D <= 128, "pipelined ring: bf16, D <= 128");
  static_assert(TR == 64 || TR == 128, "64- or 128-row tiles");
  constexpr int TE = TR * D;     // bf16 elements per tile
  constexpr int BPT = TR / 32;   // 32-row blocks per tile
  constexpr int LB = BPT == 2 ? 1 : 2;
  constexpr int NST = 4, PD = 2;
  constexpr int STAGE_BYTES = pipe_stage_bytes<D, RC, TR>();
  constexpr int NRC = 2 * TR / 64;  // 64-dword row-constant pieces per tile
  static_assert(!RC || NW >= NRC, "one row-constant piece per wave");
  constexpr int PER_TILE = 2 * dma_ipw<D, NW, TR>() + (RC ? 1 : 0);
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntiles = (n + TR - 1) / TR;
  const auto ra = make_rsrc(a, seq_bytes(n, ts_a, D, 2));
  const auto rb = make_rsrc(b, seq_bytes(n, ts_b, D, 2));
  rsrc_t r0, r1;
  if constexpr (RC) {
    r0 = make_rsrc(rc0, (uint32_t)n * 4u);
    r1 = make_rsrc(rc1, (uint32_t)n * 4u);
  }
  const uint32_t tsa = (uint32_t)(ts_a * 2), tsb = (uint32_t)(ts_b * 2);
  auto issue = [&](int t) {
    char* st = smem + (t % NST) * STAGE_BYTES;
    const int tok0 = t * TR;
    dma_tile<D, NW, TR>(ra, st, tok0, n, tsa, wave, lane);
    dma_tile<D, NW, TR>(rb, st + TE * 2, tok0, n, tsb, wave, lane);
    if constexpr (RC) {  // waves < NRC stage the constants, the others a throw-away copy
      // (every wave issues the same number of DMAs, so one vmcnt fits all)
      const bool real = wave < NRC;
      const int stream = real ? wave / (TR / 64) : 0, part = real ? wave % (TR / 64) : 0;
      char* rcs = st + 4 * TE + (real ? (stream * TR + part * 64) * 4 : 2 * TR * 4);
      dma_rowc(stream ? r1 : r0, rcs, tok0 + part * 64, lane);
    }
  };
  auto blk_at = [&](const char* st, int bi) {
    const float* rc = reinterpret_cast<const float*>(st + 4 * TE);
    return BlockRef<T>{reinterpret_cast<const T*>(st), reinterpret_cast<const T*>(st + TE * 2),
                       rc, rc + TR, 32 * (bi & (BPT - 1)), bi};
  };
  auto blk = [&](int bi) {  // bi = -1: the last block of tile -1 (the zeroed stage NST-1)
    return blk_at(smem + ((bi >> LB) & (NST - 1)) * STAGE_BYTES, bi);
  };
  // Stage NST-1 stands in for tile -1: zeroed, so G(-1) (the previous block's products at
  // t = 0) reads zero rows and adds nothing -- the loop body needs no t > 0 branch.
  {
    uint4* z = reinterpret_cast<uint4*>(smem + (NST - 1) * STAGE_BYTES);
    for (int i = tid; i < STAGE_BYTES / 16; i += 64 * NW) z[i] = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  vm_drain();
#pragma unroll
  for (int s = 0; s < PD; ++s) issue(s);
  // One loop copy per wave role, so each tile's body is one basic block (MFMA and VALU
  // of neighbouring steps can interleave in the schedule).
  // One tile step.  SG >= 0: the tile's ring stage is the compile-time SG (the loop is
  // unrolled by NST), so every LDS fragment address is a loop-invariant lane offset plus
  // an immediate; SG < 0: the stage is computed from t.
  auto step = [&](int t, auto late_c, auto sg_c) __attribute__((always_inline)) {
    constexpr bool LATE = decltype(late_c)::value;
    constexpr int SG = decltype(sg_c)::value;
    auto bk = [&](int bi, int j) __attribute__((always_inline)) {  // j: block - b0 (-1..BPT-1)
      if constexpr (SG >= 0) {
        constexpr int SP = (SG + NST - 1) % NST;
        return blk_at(smem + (j < 0 ? SP : SG) * STAGE_BYTES, bi);
      } else {
        return blk(bi);
      }
    };
    vm_wait_barrier<(PD - 1) * PER_TILE>();  // tile t landed; tile t-2 no longer read
    issue(t + PD);
    const int b0 = BPT * t;
    if constexpr (LATE) V(bk(b0 - 1, -1));
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      S(bk(b0 + j, j));
      G(bk(b0 + j - 1, j - 1));
      if (!LATE || j < BPT - 1) V(bk(b0 + j, j));
    }
    if constexpr (SCH::on && !LATE) {
#pragma unroll
      for (int j = 0; j < BPT; ++j) SCH::emit();
    }
  };
  auto run = [&](auto late_c) {
    constexpr bool LATE = decltype(late_c)::value;
    int t = 0;
#if VD_PIPE_UNROLL
    if constexpr (D <= 64)  // at D = 128 the unrolled copies spill
    // Long sequences: whole groups of NST tiles with compile-time stages.  Tiles past the
    // end are zero-filled by the DMA range check and add nothing (dQ: zero K rows; dK/dV:
    // zero Q / dO rows and row constants), so the tile count is rounded up to NST.
    if (ntiles >= 4 * NST) {
      const int nt = (ntiles + NST - 1) / NST * NST;
      for (; t < nt; t += NST) {
        step(t, late_c, std::integral_constant<int, 0>{});
        step(t + 1, late_c, std::integral_constant<int, 1>{});
        step(t + 2, late_c, std::integral_constant<int, 2>{});
        step(t + 3, late_c, std::integral_constant<int, 3>{});
      }
    }
#endif
    for (; t < ntiles; ++t) step(t, late_c, std::integral_constant<int, -1>{});
    if constexpr (LATE) V(blk(BPT * t - 1));
    G(blk(BPT * t - 1));
  };
  if (late) run(std::true_type{});
  else run(std::false_type{});
  vm_drain();
}

template <int D, bool RC, int TR = kTile>
constexpr size_t tile_pipe_lds() { return 4 * (size_t)pipe_stage_bytes<D, RC, TR>(); }

// Tile rows of the 8-wave head_dim-64 pipelined backward kernels (A/B: -DVD_PIPE_TR=128).
#ifndef VD_PIPE_TR
#define VD_PIPE_TR 64
#endif
template <int D, int NW> constexpr int pipe_tr() { return D == 64 && NW == 8 ? VD_PIPE_TR : kTile; }


template <typename T, int D, bool RC, int NSTO = 0>
size_t tile_loop_lds() {
  if constexpr (kDMA<T>)
    return (size_t)(NSTO ? NSTO : nstage<D>()) * (2 * tile_elems<T, D>() * 2 + (RC ? 768 : 0));
  else return 2 * tile_elems<T, D>() * sizeof(T) + (RC ? 512 : 0);
}

// ================================================================== forward
// WG = 4 waves x NB x 32 queries.
//
// Softmax VALU is what bounds this kernel at D = 64 (per score: exp 8 cycles + add 4 +
// half a cvt, against 2 x 16 MACs of MFMA), so the per-score work is cut to the minimum:
//  * Q is pre-scaled by scale*log2(e), so S' = S * scale * log2(e) leaves the MFMA;
//  * the S' accumulator starts at -m (a per-lane splat: the query is on the lane), so the
//    MFMA emits S' - m and the probability is a bare v_exp_f32;
//  * no per-tile max: m is a reference point that may lag the true running max.  While
//    every p stays below 2^kLag the sums are exact in fp32 (O / l is invariant to m); a
//    tile whose row sum reaches 2^kLag (or is inf, e.g. the first tile with m = -inf) is
//    recomputed with its true max (rare path), which resets m and rescales O and l.
constexpr float kLagSum = 65536.f;  // 2^16: p <= 2^16, l <= 2^16 * N -- far from overflow

// KV split (flash-decoding style, for shapes whose query grid leaves CUs idle): workgroup
// z of grid.z takes the key tiles [z * tps, (z + 1) * tps) and writes its unnormalised O^T
// (fp32) and (m, l) to `part`; attn_fwd_combine_kernel merges the splits.  part == nullptr:
// one split, normalised output as before.
struct FwdSplit {
  float* part;  // [splits][nseq][n][D] O (or dQ), then [splits][nseq][n][2] (m, l)
  int tps;      // key tiles per split
};

template <typename T, int D, int NB, int NW>
__global__ __launch_bounds__(64 * NW, 1) void attn_fwd_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, T* __restrict__ o,
    float* __restrict__ lse, int n, SeqAddr qa, int64_t ts, SeqAddr oa, int64_t ots, float scale,
    FwdSplit split, KvAddr kv) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), hh = lane >> 5;
  const int seq = blockIdx.y;
  const int q0 = blockIdx.x * (32 * NB * NW) + wave * 32 * NB;
  const int64_t base = qa(seq);
  // this workgroup's keys: [kofs, kofs + nk)
  const int kofs = blockIdx.z * split.tps * kTile;
  const int nk = split.part ? min(kv.n - kofs, split.tps * kTile) : kv.n;
  const int64_t kbase = kv.a(seq) + (int64_t)kofs * kv.ts;

  RowFrag<T, D> qf[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    qf[j].load(q + base, ts, q0 + 32 * j + (lane & 31), n, lane);
    qf[j].scale(scale * kLog2e);
  }
  f32x16 oacc[D / 32][NB];
#pragma unroll
  for (int i = 0; i < D / 32; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) oacc[i][j] = f32x16{};
  float m[NB], l[NB];
  f32x16 negm[NB];  // -m splat: the initial S' accumulator
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    m[j] = -INFINITY;
    l[j] = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) negm[j][r] = INFINITY;
  }

  tile_loop<T, D, false, NW>(smem, k + kbase, v + kbase, kv.ts, kv.ts, nullptr, nullptr, nk, tid,
                         [&](int t, const T* Kt, const T* Vt, const float*) {
    const int key0 = t * kTile;
    const bool tail = key0 + kTile > nk;  // only the last tile masks keys (wave-uniform)
    auto mask = [&](f32x16 (&s)[2][NB]) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (key0 + 32 * h + acc_row(r, hh) >= nk)
#pragma unroll
            for (int j = 0; j < NB; ++j) s[h][j][r] = -INFINITY;
    };
    f32x16 s[2][NB];
    // NB = 1, bf16: every LDS fragment of the tile is read up front (K rows for S', V^T for
    // PV; 64 VGPRs), so no MFMA waits on a just-issued read
    constexpr bool kPre = kDMA<T> && NB == 1 && D <= 64 && kPreload;
    bf16x8 kfr[2][D / 16];
    bf16x8 vfr[D / 32][2][2];
    if constexpr (kPre) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int ss = 0; ss < D / 16; ++ss)
          kfr[h][ss] = *reinterpret_cast<const bf16x8*>(
              Kt + toff<T, D>(32 * h + (lane & 31), 16 * ss + 8 * hh));
#pragma unroll
      for (int i = 0; i < D / 32; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) load_tr<D>(vfr[i][h], Vt, 32 * h, 32 * i, lane);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        s[h][0] = negm[0];
#pragma unroll
        for (int ss = 0; ss < D / 16; ++ss)
          s[h][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kfr[h][ss], qf[0].f[ss], s[h][0],
                                                            0, 0, 0);
      }
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int j = 0; j < NB; ++j) s[h][j] = negm[j];
        mma_rows_nb<T, D, NB>(s[h], Kt, 32 * h, qf, lane);
      }
    }
    if (tail) mask(s);
    float psum[NB];
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      psum[j] = 0.f;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pv = fast_exp2(s[h][j][r]);
          s[h][j][r] = pv;
          psum[j] += pv;
        }
      ok = ok && psum[j] < kLagSum;  // false for inf / NaN too
    }
    VD_STAMP(2, t);
    if (!__all(ok)) {  // rare: recompute S' with the true max of this tile
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int j = 0; j < NB; ++j) s[h][j] = f32x16{};
        mma_rows_nb<T, D, NB>(s[h], Kt, 32 * h, qf, lane);
      }
      if (tail) mask(s);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        float tmax = s[0][j][0];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, s[h][j][r]);
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float mnew = fmaxf(m[j], tmax);
        const float alpha = fast_exp2(m[j] - mnew);  // m = -inf: 0 (O and l are 0 then)
        m[j] = mnew;
        l[j] *= alpha;
#pragma unroll
        for (int i = 0; i < D / 32; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) oacc[i][j][r] *= alpha;
#pragma unroll
        for (int r = 0; r < 16; ++r) negm[j][r] = -mnew;
        psum[j] = 0.f;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float pv = fast_exp2(s[h][j][r] - mnew);
            s[h][j][r] = pv;
            psum[j] += pv;
          }
      }
    }
    XOp<T> p[2][NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      l[j] += psum[j];
#pragma unroll
      for (int h = 0; h < 2; ++h) p[h][j] = XOp<T>(s[h][j]);
    }
    if constexpr (kPre) {
#pragma unroll
      for (int i = 0; i < D / 32; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
            oacc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vfr[i][h][s2], p[h][0].b[s2],
                                                                 oacc[i][0], 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < D / 32; ++i) {
        mma_tr_nb<T, D, NB>(oacc[i], Vt, 0, 32 * i, p[0], lane);
        mma_tr_nb<T, D, NB>(oacc[i], Vt, 32, 32 * i, p[1], lane);
      }
    }
  });
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int myq = q0 + 32 * j + (lane & 31);
    const float lt = l[j] + __shfl_xor(l[j], 32, 64);
    f32x16 out[D / 32];
#pragma unroll
    for (int i = 0; i < D / 32; ++i) out[i] = oacc[i][j];
    if (split.part) {
      const int64_t row0 = ((int64_t)blockIdx.z * gridDim.y + seq) * n;
      store_transposed<float, D / 32>(split.part + row0 * D, D, myq, n, 0, out, 1.f, lane);
      float* ml = split.part + (int64_t)gridDim.z * gridDim.y * n * D;
      if (hh == 0 && myq < n) {
        ml[(row0 + myq) * 2] = m[j];
        ml[(row0 + myq) * 2 + 1] = lt;
      }
    } else {
      store_transposed<T, D / 32>(o + oa(seq), ots, myq, n, 0, out, 1.f / lt, lane);
      if (hh == 0 && myq < n) lse[(int64_t)seq * n + myq] = (m[j] + log2f(lt)) / kLog2e;
    }
  }
}

// Merge the KV splits of attn_fwd_kernel: per query row, M = max m_z,
// O = sum_z 2^(m_z - M) O_z / sum_z 2^(m_z - M) l_z, lse = (M + log2 L) / log2(e).
// One thread per (row, 8 output columns).
template <typename T, int D>
__global__ void attn_fwd_combine_kernel(const float* __restrict__ part, int splits, int nseq,
                                        int n, T* __restrict__ o, SeqAddr oa, int64_t ots,
                                        float* __restrict__ lse) {
  constexpr int CPR = D / 8;
  const int64_t rows = (int64_t)nseq * n;
  const float* ml = part + (int64_t)splits * rows * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows * CPR;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / CPR;
    const int c8 = (int)(i % CPR) * 8;
    float mz[4], M = -INFINITY;
    for (int z = 0; z < splits; ++z) {
      mz[z] = ml[((int64_t)z * rows + row) * 2];
      M = fmaxf(M, mz[z]);
    }
    float L = 0.f, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int z = 0; z < splits; ++z) {
      const float w = fast_exp2(mz[z] - M);
      L += w * ml[((int64_t)z * rows + row) * 2 + 1];
      float v8[8];
      load8(part + ((int64_t)z * rows + row) * D + c8, v8);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += w * v8[e];
    }
    const float inv = 1.f / L;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    const int seq = (int)(row / n), tok = (int)(row % n);
    store8(o + oa(seq) + (int64_t)tok * ots + c8, acc);
    if (c8 == 0) lse[row] = (M + log2f(L)) / kLog2e;
  }
}

// ================================================================== row constants
// Per query row, into the backward workspace: ndelta = -rowsum(dO * O) and
// nlse2 = -lse * log2(e).  Both are the initial MFMA accumulators of the backward
// kernels (dP - delta and S' - lse come out of the MFMA), negated once here.
template <typename T, int D>
__global__ void attn_delta_kernel(const T* __restrict__ o, const T* __restrict__ dout,
                                  const float* __restrict__ lse, float* __restrict__ ndelta,
                                  float* __restrict__ nlse2, int nseq, int n, SeqAddr oa,
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
    ndelta[i] = -acc;
    nlse2[i] = -lse[i] * kLog2e;
  }
}

// ================================================================== backward: dQ
// Q pre-scaled as in the forward; S' accumulator starts at -lse*log2(e) and dP^T at
// -delta (per-lane splats, the query is on the lane), so P^T = exp2(acc) and
// dS^T = P^T * acc_dP leave one exp and one multiply per score.
// KV split as the forward: z takes key tiles [z * tps, (z + 1) * tps) and writes its
// (scaled) fp32 dQ partial to part[z][nseq][n][D]; attn_dq_sum_kernel adds the splits.
template <typename T, int D, int NB, int NW>
__global__ __launch_bounds__(64 * NW, 1) void attn_bwd_dq_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v,
    const T* __restrict__ dout, const float* __restrict__ nlse2, const float* __restrict__ ndelta,
    T* __restrict__ dq, int n, SeqAddr qa, int64_t ts, SeqAddr oa, int64_t ots, float scale,
    FwdSplit split, KvAddr kv) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int seq = blockIdx.y;
  const int q0 = blockIdx.x * (32 * NB * NW) + wave * 32 * NB;
  const int64_t base = qa(seq);
  const int kofs = blockIdx.z * split.tps * kTile;
  const int nk = split.part ? min(kv.n - kofs, split.tps * kTile) : kv.n;
  const int64_t kbase = kv.a(seq) + (int64_t)kofs * kv.ts;

  RowFrag<T, D> qf[NB], of[NB];
  f32x16 il[NB], id[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int myq = q0 + 32 * j + (lane & 31);
    qf[j].load(q + base, ts, myq, n, lane);
    qf[j].scale(scale * kLog2e);
    of[j].load(dout + oa(seq), ots, myq, n, lane);
    const float a = myq < n ? nlse2[(int64_t)seq * n + myq] : 0.f;
    const float b = myq < n ? ndelta[(int64_t)seq * n + myq] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      il[j][r] = a;
      id[j][r] = b;
    }
  }
  f32x16 acc[D / 32][NB];
#pragma unroll
  for (int i = 0; i < D / 32; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x16{};

  tile_loop<T, D, false, NW>(smem, k + kbase, v + kbase, kv.ts, kv.ts, nullptr, nullptr, nk, tid,
                         [&](int, const T* Kt, const T* Vt, const float*) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x16 s[NB], dp[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        s[j] = il[j];
        dp[j] = id[j];
      }
      mma_rows_nb<T, D, NB>(s, Kt, 32 * h, qf, lane);
      mma_rows_nb<T, D, NB>(dp, Vt, 32 * h, of, lane);
      // keys past n have zero K/V rows: their dS^T multiplies a zero K row in the
      // dQ product, so no mask is needed here
      XOp<T> ds[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[j][r] = fast_exp2(s[j][r]) * dp[j][r];  // dS^T
        ds[j] = XOp<T>(s[j]);
      }
#pragma unroll
      for (int i = 0; i < D / 32; ++i) mma_tr_nb<T, D, NB>(acc[i], Kt, 32 * h, 32 * i, ds, lane);
    }
  });
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    f32x16 out[D / 32];
#pragma unroll
    for (int i = 0; i < D / 32; ++i) out[i] = acc[i][j];
    if (split.part)
      store_transposed<float, D / 32>(
          split.part + ((int64_t)blockIdx.z * gridDim.y + seq) * n * D, D,
          q0 + 32 * j + (lane & 31), n, 0, out, scale, lane);
    else
      store_transposed<T, D / 32>(dq + base, ts, q0 + 32 * j + (lane & 31), n, 0, out, scale,
                                  lane);
  }
}

// dq = sum over the KV splits of the fp32 partials (one thread per 8 columns)
template <typename T, int D>
__global__ void attn_dq_sum_kernel(const float* __restrict__ part, int splits, int nseq, int n,
                                   T* __restrict__ dq, SeqAddr qa, int64_t ts) {
  constexpr int CPR = D / 8;
  const int64_t rows = (int64_t)nseq * n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows * CPR;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / CPR;
    const int c8 = (int)(i % CPR) * 8;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int z = 0; z < splits; ++z) {
      float v8[8];
      load8(part + ((int64_t)z * rows + row) * D + c8, v8);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v8[e];
    }
    const int seq = (int)(row / n), tok = (int)(row % n);
    store8(dq + qa(seq) + (int64_t)tok * ts + c8, acc);
  }
}

// ================================================================== backward: dK, dV
// WG = 4 waves x NB x 32 keys.  grid.z splits the OUTPUT columns of dK/dV in DO-wide
// slices (register budget at D = 256); S and dP always contract over the full D.
// K pre-scaled by scale*log2(e); the tile's row constants (-lse*log2 e, -delta; the query
// is the accumulator row here) are read from LDS straight into the initial accumulators.
template <typename T, int D, int DO, int NB, int NW>
__global__ __launch_bounds__(64 * NW, 1) void attn_bwd_dkdv_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v,
    const T* __restrict__ dout, const float* __restrict__ nlse2, const float* __restrict__ ndelta,
    T* __restrict__ dk, T* __restrict__ dv, int n, SeqAddr qa, int64_t ts, SeqAddr oa,
    int64_t ots, float scale, KvAddr kv, FwdSplit qsplit) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), hh = lane >> 5;
  const int seq = blockIdx.y;
  constexpr int NZ = D / DO;
  const int d0 = (blockIdx.z % NZ) * DO;
  // query split (grids too small for the chip, e.g. cross-attention onto a few audio
  // tokens): z takes the query tiles [qz * tps, (qz + 1) * tps) and writes fp32 partial
  // dK / dV; attn_dkdv_sum_kernel adds the splits
  const int qz = blockIdx.z / NZ;
  const int qofs = qz * qsplit.tps * kTile;
  const int nq = qsplit.part ? min(n - qofs, qsplit.tps * kTile) : n;
  const int k0 = blockIdx.x * (32 * NB * NW) + wave * 32 * NB;
  const int64_t base = qa(seq) + (int64_t)qofs * ts, obase = oa(seq) + (int64_t)qofs * ots;
  const int64_t kb = kv.a(seq);

  RowFrag<T, D> kf[NB], vf[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    kf[j].load(k + kb, kv.ts, k0 + 32 * j + (lane & 31), kv.n, lane);
    kf[j].scale(scale * kLog2e);
    vf[j].load(v + kb, kv.ts, k0 + 32 * j + (lane & 31), kv.n, lane);
  }
  f32x16 adv[DO / 32][NB], adk[DO / 32][NB];
#pragma unroll
  for (int i = 0; i < DO / 32; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) adv[i][j] = adk[i][j] = f32x16{};

  // query rows past n have zero Q / dO rows and zero row constants, so they add nothing
  // to dV (dO = 0) or dK (dS = p * (0 - 0)): no mask needed.
  tile_loop<T, D, true, NW>(smem, q + base, dout + obase, ts, ots,
                        nlse2 + (int64_t)seq * n + qofs, ndelta + (int64_t)seq * n + qofs, nq, tid,
                        [&](int, const T* Qt, const T* Ot, const float* L) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // registers 4g..4g+3 are rows 8g + 4hh + 0..3: one b128 read per constant
      f32x16 il, id;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 ls = *reinterpret_cast<const float4*>(L + 32 * h + 8 * g + 4 * hh);
        const float4 dl = *reinterpret_cast<const float4*>(L + 64 + 32 * h + 8 * g + 4 * hh);
        il[4 * g + 0] = ls.x; il[4 * g + 1] = ls.y; il[4 * g + 2] = ls.z; il[4 * g + 3] = ls.w;
        id[4 * g + 0] = dl.x; id[4 * g + 1] = dl.y; id[4 * g + 2] = dl.z; id[4 * g + 3] = dl.w;
      }
      f32x16 s[NB], dp[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        s[j] = il;
        dp[j] = id;
      }
      mma_rows_nb<T, D, NB>(s, Qt, 32 * h, kf, lane);   // S'[q][key] - lse'
      mma_rows_nb<T, D, NB>(dp, Ot, 32 * h, vf, lane);  // dP[q][key] - delta
      XOp<T> pp[NB], ds[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pv = fast_exp2(s[j][r]);
          s[j][r] = pv;
          dp[j][r] *= pv;  // dS
        }
        pp[j] = XOp<T>(s[j]);
        ds[j] = XOp<T>(dp[j]);
      }
#pragma unroll
      for (int i = 0; i < DO / 32; ++i) {
        mma_tr_nb<T, D, NB>(adv[i], Ot, 32 * h, d0 + 32 * i, pp, lane);  // dV^T += dO^T P
        mma_tr_nb<T, D, NB>(adk[i], Qt, 32 * h, d0 + 32 * i, ds, lane);  // dK^T += Q^T dS
      }
    }
  });
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int mykey = k0 + 32 * j + (lane & 31);
    f32x16 ok[DO / 32], ov[DO / 32];
#pragma unroll
    for (int i = 0; i < DO / 32; ++i) {
      ok[i] = adk[i][j];
      ov[i] = adv[i][j];
    }
    if (qsplit.part) {
      float* pb = qsplit.part + ((int64_t)qz * gridDim.y + seq) * kv.n * (2 * D);
      store_transposed<float, DO / 32>(pb, 2 * D, mykey, kv.n, d0, ok, scale, lane);
      store_transposed<float, DO / 32>(pb + D, 2 * D, mykey, kv.n, d0, ov, 1.f, lane);
    } else {
      store_transposed<T, DO / 32>(dk + kb, kv.ts, mykey, kv.n, d0, ok, scale, lane);
      store_transposed<T, DO / 32>(dv + kb, kv.ts, mykey, kv.n, d0, ov, 1.f, lane);
    }
  }
}

// ------------------------------------------------------------------ dK / dV, head_dim 256
// Role-split pairs: waves w and w + 4 (one SIMD) own the same 32 keys.  Wave A (w < 4) keeps
// K in registers and the full-width dV^T accumulators; wave B keeps V and dK^T.  Per 32-query
// block A computes S' and P = exp2(S' - lse') and hands P (fp32) to B through LDS; B computes
// dP - delta, dS = P * (dP - delta) and dK^T += Q^T dS while A runs dV^T += dO^T P.  Each
// product runs once: 8 N^2 D executed against 12 for the output-column split, and each wave
// needs 64 + 128 + ~40 registers (the full-width single-wave form needs > 512).
//   A: [S MFMAs, exp] bar2 [write P] bar1 [dV MFMAs]
//   B: [dP MFMAs]     bar2           bar1 [read P, dS, dK MFMAs]
// bar2 orders A's write of block h after B's read of block h - 1; bar1 B's read after A's
// write.  Both roles run their own copy of the tile loop (their accumulators never share a
// live range) and pass the same barriers in the same order.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt / expcnt untouched
  __builtin_amdgcn_s_barrier();
}

// VD_ROLE_NW: waves per workgroup (8: two per SIMD, 256 registers each; 4: one per SIMD)
#ifndef VD_ROLE_NW
#define VD_ROLE_NW 4
#endif
// VD_ROLE_G: k-steps per scheduling-fenced group in the role kernel's products (16: none)
#ifndef VD_ROLE_G
#define VD_ROLE_G 16
#endif
constexpr int kRoleG = VD_ROLE_G;
// mma_rows / mma_tr in groups of G k-steps / tiles behind scheduling fences: bounds how far
// the compiler hoists LDS operand reads (registers, at 256 per wave)
template <int D, int G>
__device__ __forceinline__ void mma_rows_fenced(f32x16& acc, const bf16_t* tile, int row0,
                                                const RowFrag<bf16_t, D>& b, int lane) {
  const int r = row0 + (lane & 31), hh = lane >> 5;
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    if (G < D / 16 && s % G == 0) __builtin_amdgcn_sched_barrier(0);
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(tile + toff<bf16_t, D>(r, 16 * s + 8 * hh));
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b.f[s], acc, 0, 0, 0);
  }
}

template <int D, int NW>
__global__ __launch_bounds__(64 * NW, 1) void attn_bwd_dkdv_role_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ nlse2,
    const float* __restrict__ ndelta, bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int n,
    SeqAddr qa, int64_t ts, SeqAddr oa, int64_t ots, float scale, KvAddr kv, FwdSplit qsplit) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int NP = NW / 2;  // wave pairs: wave w (A) and w + NP (B)
  const int hh = lane >> 5, pair = wave % NP;
  const int seq = blockIdx.y, qz = blockIdx.z;
  const int qofs = qz * qsplit.tps * kTile;
  const int nq = qsplit.part ? min(n - qofs, qsplit.tps * kTile) : n;
  const int k0 = blockIdx.x * (32 * NP) + pair * 32;
  const int mykey = k0 + (lane & 31);
  const int64_t base = qa(seq) + (int64_t)qofs * ts, obase = oa(seq) + (int64_t)qofs * ots;
  const int64_t kb = kv.a(seq);
  const float* rc0 = nlse2 + (int64_t)seq * n + qofs;
  const float* rc1 = ndelta + (int64_t)seq * n + qofs;
  // P hand-off of this pair: [4 register groups][64 lanes][4 floats] (conflict-free b128)
  constexpr int RING = nstage<D>() * (2 * kTile * D * 2 + 768);  // tile_loop_lds<bf16, D, RC>
  float* xch = reinterpret_cast<float*>(smem + RING) + pair * 1024;
  float* part = qsplit.part ? qsplit.part + ((int64_t)qz * gridDim.y + seq) * kv.n * (2 * D)
                            : nullptr;
  // registers 4g..4g+3 are query rows 8g + 4hh + 0..3 of the block
  auto rows = [&](f32x16& x, const float* L) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 c = *reinterpret_cast<const float4*>(L + 8 * g + 4 * hh);
      x[4 * g + 0] = c.x; x[4 * g + 1] = c.y; x[4 * g + 2] = c.z; x[4 * g + 3] = c.w;
    }
  };
  if (wave < NP) {  // A: S, P, dV
    RowFrag<bf16_t, D> kf;
    kf.load(k + kb, kv.ts, mykey, kv.n, lane);
    kf.scale(scale * kLog2e);
    f32x16 adv[D / 32];
#pragma unroll
    for (int i = 0; i < D / 32; ++i) adv[i] = f32x16{};
    tile_loop<bf16_t, D, true, NW>(smem, q + base, dout + obase, ts, ots, rc0, rc1, nq, tid,
                                   [&](int, const bf16_t* Qt, const bf16_t* Ot, const float* L) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x16 sx;
        rows(sx, L + 32 * h);
        mma_rows_fenced<D, kRoleG>(sx, Qt, 32 * h, kf, lane);  // S'[q][key] - lse'
#pragma unroll
        for (int r = 0; r < 16; ++r) sx[r] = fast_exp2(sx[r]);
        const XOp<bf16_t> pp(sx);
        lds_barrier();  // bar2
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(xch + (g * 64 + lane) * 4) =
              make_float4(sx[4 * g], sx[4 * g + 1], sx[4 * g + 2], sx[4 * g + 3]);
        lds_barrier();  // bar1
#pragma unroll
        for (int i = 0; i < D / 32; ++i) {
          if (kRoleG < 16 && i % 2 == 0) __builtin_amdgcn_sched_barrier(0);
          mma_tr<bf16_t, D>(adv[i], Ot, 32 * h, 32 * i, pp, lane);
        }
      }
    });
    if (part) store_transposed<float, D / 32>(part + D, 2 * D, mykey, kv.n, 0, adv, 1.f, lane);
    else store_transposed<bf16_t, D / 32>(dv + kb, kv.ts, mykey, kv.n, 0, adv, 1.f, lane);
  } else {  // B: dP, dS, dK
    RowFrag<bf16_t, D> vf;
    vf.load(v + kb, kv.ts, mykey, kv.n, lane);
    f32x16 adk[D / 32];
#pragma unroll
    for (int i = 0; i < D / 32; ++i) adk[i] = f32x16{};
    tile_loop<bf16_t, D, true, NW>(smem, q + base, dout + obase, ts, ots, rc0, rc1, nq, tid,
                                   [&](int, const bf16_t* Qt, const bf16_t* Ot, const float* L) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x16 dp;
        rows(dp, L + 64 + 32 * h);
        mma_rows_fenced<D, kRoleG>(dp, Ot, 32 * h, vf, lane);  // dP[q][key] - delta
        lds_barrier();  // bar2
        lds_barrier();  // bar1
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 pv = *reinterpret_cast<const float4*>(xch + (g * 64 + lane) * 4);
          dp[4 * g + 0] *= pv.x; dp[4 * g + 1] *= pv.y; dp[4 * g + 2] *= pv.z; dp[4 * g + 3] *= pv.w;
        }
        const XOp<bf16_t> ds(dp);
#pragma unroll
        for (int i = 0; i < D / 32; ++i) {
          if (kRoleG < 16 && i % 2 == 0) __builtin_amdgcn_sched_barrier(0);
          mma_tr<bf16_t, D>(adk[i], Qt, 32 * h, 32 * i, ds, lane);
        }
      }
    });
    if (part) store_transposed<float, D / 32>(part, 2 * D, mykey, kv.n, 0, adk, scale, lane);
    else store_transposed<bf16_t, D / 32>(dk + kb, kv.ts, mykey, kv.n, 0, adk, scale, lane);
  }
}

// dK | dV = sum over the query splits of the fp32 partials [split][nseq][nkv][dK D | dV D]
// (one thread per 8 columns)
template <typename T, int D>
__global__ void attn_dkdv_sum_kernel(const float* __restrict__ part, int splits, int nseq,
                                     int nkv, T* __restrict__ dk, T* __restrict__ dv, SeqAddr ka,
                                     int64_t kts) {
  constexpr int CPR = 2 * D / 8;
  const int64_t rows = (int64_t)nseq * nkv;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows * CPR;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / CPR;
    const int c8 = (int)(i % CPR) * 8;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int z = 0; z < splits; ++z) {
      float v8[8];
      load8(part + ((int64_t)z * rows + row) * (2 * D) + c8, v8);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v8[e];
    }
    const int seq = (int)(row / nkv), tok = (int)(row % nkv);
    T* dst = (c8 < D ? dk + c8 : dv + (c8 - D)) + ka(seq) + (int64_t)tok * kts;
    store8(dst, acc);
  }
}

// ================================================================== backward: dK, dV, paired
// head_dim 128 with two waves per SIMD.  The 4-wave kernel above holds 32 keys' K and V
// fragments (64 VGPRs) and their full dK^T / dV^T accumulators (128 VGPRs) per wave, so it
// runs one wave per SIMD and nothing hides the S -> exp -> dV/dK dependency chain.  Here a
// workgroup of 8 waves owns 128 keys: K (pre-scaled by scale*log2 e) and V of those keys sit
// in LDS for the whole launch (64 KiB, read as the B operand exactly as the query tiles are
// read as the A operand), and the SIMD partners w and w + 4 share one 32-key group: wave w
// takes query rows 0-31 of every 64-row tile, wave w + 4 rows 32-63.  Each wave keeps its
// own fp32 dK^T / dV^T partials (same products, half the queries each); the partners' sums
// are added through LDS at the end.  Two ring stages (64 KiB + the resident K/V fit in 160).
template <int D>
__global__ __launch_bounds__(512, 1) void attn_bwd_dkdv_pair_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ nlse2,
    const float* __restrict__ ndelta, bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int n,
    SeqAddr qa, int64_t ts, SeqAddr oa, int64_t ots, float scale, KvAddr kv) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KEYS = 128, GTE = 32 * D;  // keys per workgroup; bf16 per 32-key group
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, kg = wave & 3, half = wave >> 2;
  const int seq = blockIdx.y;
  const int kw0 = blockIdx.x * KEYS;  // first key of the workgroup
  const int64_t base = qa(seq), obase = oa(seq), kb = kv.a(seq);
  bf16_t* kl = reinterpret_cast<bf16_t*>(smem);  // [4 groups][32 keys][D], tile swizzle
  bf16_t* vl = kl + 4 * GTE;
  char* ring = smem + 8 * GTE * 2;
  // stage the workgroup's K (scaled) and V rows: 16 B per thread per step
  {
    const float c = scale * kLog2e;
    constexpr int CPR = D / 8;
    for (int i = tid; i < KEYS * CPR; i += 512) {
      const int r = i / CPR, cc = i % CPR, key = kw0 + r;
      uint4 kk = make_uint4(0, 0, 0, 0), vv = kk;
      if (key < kv.n) {
        kk = *reinterpret_cast<const uint4*>(k + kb + (int64_t)key * kv.ts + cc * 8);
        vv = *reinterpret_cast<const uint4*>(v + kb + (int64_t)key * kv.ts + cc * 8);
      }
      const uint32_t in[4] = {kk.x, kk.y, kk.z, kk.w};
      uint32_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = pack2bf(__uint_as_float(in[e] << 16) * c, __uint_as_float(in[e] & 0xffff0000u) * c);
      const int off = (r >> 5) * GTE + toff<bf16_t, D>(r & 31, cc * 8);
      *reinterpret_cast<uint4*>(kl + off) = make_uint4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<uint4*>(vl + off) = vv;
    }
  }
  __syncthreads();
  const bf16_t* kgl = kl + kg * GTE;
  const bf16_t* vgl = vl + kg * GTE;
  f32x16 adv[D / 32], adk[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) adv[i] = adk[i] = f32x16{};
  const int row0 = 32 * half;
#ifdef VD_PAIR_PRIO
  if (half) __builtin_amdgcn_s_setprio(1);  // A/B: static priority for the second half
#endif

  tile_loop<bf16_t, D, true, 8, 2>(ring, q + base, dout + obase, ts, ots,
                                   nlse2 + (int64_t)seq * n, ndelta + (int64_t)seq * n, n, tid,
                                   [&](int, const bf16_t* Qt, const bf16_t* Ot, const float* L) {
    f32x16 s, dp;
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // registers 4g..4g+3 = query rows 8g + 4hh + 0..3
      const float4 ls = *reinterpret_cast<const float4*>(L + row0 + 8 * g + 4 * hh);
      const float4 dl = *reinterpret_cast<const float4*>(L + 64 + row0 + 8 * g + 4 * hh);
      s[4 * g + 0] = ls.x; s[4 * g + 1] = ls.y; s[4 * g + 2] = ls.z; s[4 * g + 3] = ls.w;
      dp[4 * g + 0] = dl.x; dp[4 * g + 1] = dl.y; dp[4 * g + 2] = dl.z; dp[4 * g + 3] = dl.w;
    }
    const int r = row0 + (lane & 31);
#pragma unroll
    for (int ss = 0; ss < D / 16; ++ss) {  // S'[q][key] - lse', dP[q][key] - delta
      const bf16x8 qa8 = *reinterpret_cast<const bf16x8*>(Qt + toff<bf16_t, D>(r, 16 * ss + 8 * hh));
      const bf16x8 kb8 = *reinterpret_cast<const bf16x8*>(kgl + toff<bf16_t, D>(lane & 31, 16 * ss + 8 * hh));
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa8, kb8, s, 0, 0, 0);
      const bf16x8 oa8 = *reinterpret_cast<const bf16x8*>(Ot + toff<bf16_t, D>(r, 16 * ss + 8 * hh));
      const bf16x8 vb8 = *reinterpret_cast<const bf16x8*>(vgl + toff<bf16_t, D>(lane & 31, 16 * ss + 8 * hh));
      dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(oa8, vb8, dp, 0, 0, 0);
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float pv = fast_exp2(s[e]);
      s[e] = pv;
      dp[e] *= pv;  // dS
    }
    const XOp<bf16_t> pp(s), ds(dp);
#pragma unroll
    for (int i = 0; i < D / 32; ++i) {
      mma_tr<bf16_t, D>(adv[i], Ot, row0, 32 * i, pp, lane);  // dV^T += dO^T P
      mma_tr<bf16_t, D>(adk[i], Qt, row0, 32 * i, ds, lane);  // dK^T += Q^T dS
    }
  });
  // partner sums: waves 4-7 hand their partials to waves 0-3 through LDS (lane-interleaved,
  // conflict-free); the ring and the K/V area are free once every wave left the loop
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem) + (int64_t)kg * (2 * D / 32) * 16 * 64;
  if (half) {
#pragma unroll
    for (int i = 0; i < D / 32; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        red[((2 * i) * 16 + e) * 64 + lane] = adk[i][e];
        red[((2 * i + 1) * 16 + e) * 64 + lane] = adv[i][e];
      }
  }
  __syncthreads();
  if (!half) {
#pragma unroll
    for (int i = 0; i < D / 32; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        adk[i][e] += red[((2 * i) * 16 + e) * 64 + lane];
        adv[i][e] += red[((2 * i + 1) * 16 + e) * 64 + lane];
      }
    const int mykey = kw0 + 32 * kg + (lane & 31);
    store_transposed<bf16_t, D / 32>(dk + kb, kv.ts, mykey, kv.n, 0, adk, scale, lane);
    store_transposed<bf16_t, D / 32>(dv + kb, kv.ts, mykey, kv.n, 0, adv, 1.f, lane);
  }
}

// ================================================================== pipelined kernels
// VD_BWD_STAGGER=0 (A/B): the 8-wave dQ / dK/dV pipelines without the staggered half
#ifndef VD_BWD_STAGGER
#define VD_BWD_STAGGER 1
#endif


// Same math as the kernels above (one 32-row block per wave, NB = 1), on tile_pipe.


// Forward with the lagged-max check deferred to the tile boundary, so the loop body is one
// basic block.  PV runs one tile (two 32-key blocks) behind the softmax: the check of tile
// t-1's blocks opens tile t, before their PV; on the rare path it recomputes both blocks
// from the still-resident K tile against their true max and rescales O and l, which then
// hold exactly the blocks before them.  Order per tile (waves 0-3 of 8, or all waves
// without STAGGER): [check(t-1)] S(2t) G(2t-2) V(2t) S(2t+1) G(2t-1) V(2t+1);
// staggered waves 4-7: V(2t-1) [check(t-1)] S(2t) G(2t-2) V(2t) S(2t+1) G(2t-1).
// Same ring as tile_pipe (4 stages, prefetch distance 2): tile t-1 stays resident while
// t+1 and t+2 land.  bf16, D = 64 (the issue-bound shape).
// Measured and retired (profiles/r01_ab_*, r02_ab_defer_*): every LDS fragment of the body
// loaded up front (18.0 vs 17.4 ms), row sums on the matrix pipe (22.1 vs 18.0 ms: the sum
// MFMAs serialise on the exp -> cvt -> MFMA chain), one barrier per two tiles (17.4 vs 16.7
// ms), the softmax spread by sched_group_barrier (15.4-15.6 vs 15.3 ms).
template <int D, int NW> constexpr int defer_nst() { return 4; }

template <typename T, int D, int NW, bool STAGGER>
__global__ __launch_bounds__(64 * NW, 8 / NW) void attn_fwd_defer_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, T* __restrict__ o,
    float* __restrict__ lse, int n, SeqAddr qa, int64_t ts, SeqAddr oa, int64_t ots, float scale) {
  static_assert(kDMA<T> && (D == 64 || D == 128), "deferred-check forward: bf16, D = 64 / 128");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TE = kTile * D, NST = defer_nst<D, NW>(), PD = 2;
  constexpr int STAGE_BYTES = pipe_stage_bytes<D, false, kTile>();
  constexpr int PER_TILE = 2 * dma_ipw<D, NW, kTile>();
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), hh = lane >> 5;
  const int seq = blockIdx.y;
  const int q0 = blockIdx.x * (32 * NW) + wave * 32;
  const int64_t base = qa(seq);
  const bool late = STAGGER && wave >= NW / 2;
  const int ntiles = (n + kTile - 1) / kTile;

  RowFrag<T, D> qf;
  qf.load(q + base, ts, q0 + (lane & 31), n, lane);
  qf.scale(scale * kLog2e);
  f32x16 oacc[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) oacc[i] = f32x16{};
  float m = -INFINITY;
  float l = 0.f, psa = 0.f, psb = 0.f;
  f32x16 negm, sa, sb;
  XOp<T> pa{}, pb{};  // zero: G(-2), G(-1) add nothing
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    negm[r] = INFINITY;  // m = -inf: the first tile's sums are inf -> rare path sets m
    sb[r] = -INFINITY;   // a staggered wave's V(-1) yields p = 0, psum = 0
  }

  const auto ra = make_rsrc(k + base, seq_bytes(n, ts, D, 2));
  const auto rb = make_rsrc(v + base, seq_bytes(n, ts, D, 2));
  const uint32_t tsb = (uint32_t)(ts * 2);
  auto issue = [&](int t) __attribute__((always_inline)) {
    char* st = smem + (t % NST) * STAGE_BYTES;
    dma_tile<D, NW>(ra, st, t * kTile, n, tsb, wave, lane);
    dma_tile<D, NW>(rb, st + TE * 2, t * kTile, n, tsb, wave, lane);
  };
  // block bi: rows [32 (bi & 1), +32) of tile bi >> 1 (bi < 0: the zeroed stage NST-1)
  auto kblk = [&](int bi) __attribute__((always_inline)) {
    return reinterpret_cast<const T*>(smem + ((bi >> 1) & (NST - 1)) * STAGE_BYTES);
  };
  auto vblk = [&](int bi) __attribute__((always_inline)) { return kblk(bi) + TE; };
  auto mask = [&](f32x16& s, int bi) __attribute__((always_inline)) {
    const int key0 = 32 * bi;
    if (key0 + 32 > n)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (key0 + acc_row(r, hh) >= n) s[r] = -INFINITY;
  };
  // st: the block's ring stage (nullptr: from bi)
  auto S = [&](f32x16& s, int bi, const char* st = nullptr) __attribute__((always_inline)) {
    s = negm;
    mma_rows<T, D>(s, st ? reinterpret_cast<const T*>(st) : kblk(bi), 32 * (bi & 1), qf, lane);
  };
  auto G = [&](const XOp<T>& p, int bi, const char* st = nullptr) __attribute__((always_inline)) {
    const T* vb = st ? reinterpret_cast<const T*>(st) + TE : vblk(bi);
#pragma unroll
    for (int i = 0; i < D / 32; ++i) mma_tr<T, D>(oacc[i], vb, 32 * (bi & 1), 32 * i, p, lane);
  };
  // MK: the block may hold keys >= n (only the last tile's blocks can)
  auto V = [&](f32x16& s, XOp<T>& p, float& ps, int bi, auto mk) __attribute__((always_inline)) {
    if constexpr (decltype(mk)::value) mask(s, bi);
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = fast_exp2(s[r]);
    // pairwise: a 4-deep dependency chain instead of 16 (A/B build flag)
    float t8[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) t8[r] = s[2 * r] + s[2 * r + 1];
#pragma unroll
    for (int r = 0; r < 4; ++r) t8[r] = t8[2 * r] + t8[2 * r + 1];
    ps = (t8[0] + t8[1]) + (t8[2] + t8[3]);
    p = XOp<T>(s);
  };
  // blocks 2tp, 2tp+1 hold p against the current m; their PV has not run yet
  auto check = [&](int tp) __attribute__((always_inline)) {
    const bool ok = psa < kLagSum && psb < kLagSum;
    if (!__all(ok)) {  // rare: true max of the tile
      // sa / sb are dead here (their blocks' softmax ran): reuse them, no extra registers
      f32x16& s0 = sa;
      f32x16& s1 = sb;
      s0 = f32x16{};
      s1 = f32x16{};
      mma_rows<T, D>(s0, kblk(2 * tp), 0, qf, lane);
      mma_rows<T, D>(s1, kblk(2 * tp + 1), 32, qf, lane);
      mask(s0, 2 * tp);
      mask(s1, 2 * tp + 1);
      float tmax = fmaxf(s0[0], s1[0]);
#pragma unroll
      for (int r = 1; r < 16; ++r) tmax = fmaxf(tmax, fmaxf(s0[r], s1[r]));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mnew = fmaxf(m, tmax);
      const float alpha = fast_exp2(m - mnew);  // m = -inf: 0 (O and l are 0 then)
      m = mnew;
      l *= alpha;
#pragma unroll
      for (int i = 0; i < D / 32; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[i][r] *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        negm[r] = -mnew;
        s0[r] -= mnew;
        s1[r] -= mnew;
      }
      V(s0, pa, psa, 2 * tp, std::false_type{});  // masked above
      V(s1, pb, psb, 2 * tp + 1, std::false_type{});
    }
    l += psa + psb;
  };

  {  // zero the stage that stands in for tile -1
    uint4* z = reinterpret_cast<uint4*>(smem + (NST - 1) * STAGE_BYTES);
    for (int i = tid; i < STAGE_BYTES / 16; i += 64 * NW) z[i] = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  vm_drain();
#pragma unroll
  for (int s = 0; s < PD; ++s) issue(s);
  // The last tile runs its own copy of the body, the only one that masks keys >= n: the
  // steady-state body carries no branch besides the check at its top.
  // SG >= 0: tile t's ring stage as a compile-time constant (the loop unrolled by NST:
  // LDS fragment addresses become loop-invariant lane offsets plus immediates)
  auto tile = [&](int t, auto late_c, auto mk, auto sg_c) __attribute__((always_inline)) {
    constexpr bool LATE = decltype(late_c)::value;
    constexpr int SG = decltype(sg_c)::value;
    const char* cur = SG >= 0 ? smem + SG * STAGE_BYTES : nullptr;
    const char* prv = SG >= 0 ? smem + ((SG + NST - 1) % NST) * STAGE_BYTES : nullptr;
    vm_wait_barrier<(PD - 1) * PER_TILE>();  // tile t landed; tile t-2 no longer read
    issue(t + PD);
    const int b0 = 2 * t;
    if constexpr (LATE) V(sb, pb, psb, b0 - 1, std::false_type{});
    check(t - 1);
    S(sa, b0, cur);
    G(pa, b0 - 2, prv);
    V(sa, pa, psa, b0, mk);
    S(sb, b0 + 1, cur);
    G(pb, b0 - 1, prv);
    if constexpr (!LATE) V(sb, pb, psb, b0 + 1, mk);
  };
  auto run = [&](auto late_c) __attribute__((always_inline)) {
    constexpr bool LATE = decltype(late_c)::value;
    using Dyn = std::integral_constant<int, -1>;
    int t = 0;
#if VD_PIPE_UNROLL
    if constexpr (D <= 64)  // at D = 128 the unrolled copies spill (256 VGPRs)
    for (; t + NST <= ntiles - 1; t += NST) {
      tile(t, late_c, std::false_type{}, std::integral_constant<int, 0>{});
      tile(t + 1, late_c, std::false_type{}, std::integral_constant<int, 1>{});
      tile(t + 2, late_c, std::false_type{}, std::integral_constant<int, 2>{});
      tile(t + 3, late_c, std::false_type{}, std::integral_constant<int, 3>{});
    }
#endif
    for (; t < ntiles - 1; ++t) tile(t, late_c, std::false_type{}, Dyn{});
    tile(ntiles - 1, late_c, std::true_type{}, Dyn{});
    if constexpr (LATE) V(sb, pb, psb, 2 * ntiles - 1, std::true_type{});
    check(ntiles - 1);
    G(pa, 2 * ntiles - 2);
    G(pb, 2 * ntiles - 1);
  };
  // static priority for the second-dispatched wave half (MI355X_MICROARCH.md): measured
  // 17.7 vs 17.9-18.0 ms at N = 262144
  if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  if (late) run(std::true_type{});
  else run(std::false_type{});
  vm_drain();

  const int myq = q0 + (lane & 31);
  const float lt = l + __shfl_xor(l, 32, 64);
  store_transposed<T, D / 32>(o + oa(seq), ots, myq, n, 0, oacc, 1.f / lt, lane);
  if (hh == 0 && myq < n) lse[(int64_t)seq * n + myq] = (m + log2f(lt)) / kLog2e;
}

// NB: 32-row blocks per wave (NB = 2 with 4 waves: one wave per SIMD with the whole
// register file; each LDS fragment read feeds two MFMAs, half the LDS bytes per FLOP).
template <typename T, int D, int NW, int NB = 1>
__global__ __launch_bounds__(64 * NW, 1) void attn_bwd_dq_pipe_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v,
    const T* __restrict__ dout, const float* __restrict__ nlse2, const float* __restrict__ ndelta,
    T* __restrict__ dq, int n, SeqAddr qa, int64_t ts, SeqAddr oa, int64_t ots, float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int seq = blockIdx.y;
  const int q0 = blockIdx.x * (32 * NB * NW) + wave * 32 * NB;
  const int64_t base = qa(seq);
  const bool late = VD_BWD_STAGGER && NW == 8 && wave >= 4;

  RowFrag<T, D> qf[NB], of[NB];
  f32x16 il[NB], id[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int myq = q0 + 32 * j + (lane & 31);
    qf[j].load(q + base, ts, myq, n, lane);
    qf[j].scale(scale * kLog2e);
    of[j].load(dout + oa(seq), ots, myq, n, lane);
    const float a = myq < n ? nlse2[(int64_t)seq * n + myq] : 0.f;
    const float b = myq < n ? ndelta[(int64_t)seq * n + myq] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      il[j][r] = a;
      id[j][r] = b;
    }
  }
  f32x16 acc[D / 32][NB], s[NB], dp[NB];
#pragma unroll
  for (int i = 0; i < D / 32; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x16{};
#pragma unroll
  for (int j = 0; j < NB; ++j) s[j] = dp[j] = f32x16{};  // a staggered wave's V(-1) reads them
  // zero operands (explicitly: G of block -1 multiplies them by the zeroed ring stage, and
  // uninitialised registers could hold NaN bit patterns)
  XOp<T> ds[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) ds[j] = XOp<T>(f32x16{});
  // static priority for the second-dispatched half (MI355X_MICROARCH.md): 23.3 vs 23.45 ms
  // at N = 262144 (dK/dV measured no gain, so it stays off there)
  if (NW == 8 && wave >= 4) __builtin_amdgcn_s_setprio(1);

  tile_pipe<T, D, false, NW, NoSched,
            pipe_tr<D, NW>()>(
      smem, k + base, v + base, ts, ts, nullptr, nullptr, n, tid, late,
      [&](const BlockRef<T>& bs) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          s[j] = il[j];
          dp[j] = id[j];
        }
        mma_rows_nb<T, D, NB>(s, bs.a, bs.row0, qf, lane);
        mma_rows_nb<T, D, NB>(dp, bs.b, bs.row0, of, lane);
      },
      [&](const BlockRef<T>& bg) {  // dQ^T += K^T dS^T (keys past n: zero K rows)
#pragma unroll
        for (int i = 0; i < D / 32; ++i) mma_tr_nb<T, D, NB>(acc[i], bg.a, bg.row0, 32 * i, ds, lane);
      },
      [&](const BlockRef<T>&) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
#pragma unroll
          for (int r = 0; r < 16; ++r) s[j][r] = fast_exp2(s[j][r]) * dp[j][r];
          ds[j] = XOp<T>(s[j]);
        }
      });
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    f32x16 out[D / 32];
#pragma unroll
    for (int i = 0; i < D / 32; ++i) out[i] = acc[i][j];
    store_transposed<T, D / 32>(dq + base, ts, q0 + 32 * j + (lane & 31), n, 0, out, scale, lane);
  }
}

template <typename T, int D, int NW, int NB = 1>
__global__ __launch_bounds__(64 * NW, 1) void attn_bwd_dkdv_pipe_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v,
    const T* __restrict__ dout, const float* __restrict__ nlse2, const float* __restrict__ ndelta,
    T* __restrict__ dk, T* __restrict__ dv, int n, SeqAddr qa, int64_t ts, SeqAddr oa,
    int64_t ots, float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), hh = lane >> 5;
  const int seq = blockIdx.y;
  const int k0 = blockIdx.x * (32 * NB * NW) + wave * 32 * NB;
  const int64_t base = qa(seq), obase = oa(seq);
  const bool late = VD_BWD_STAGGER && NW == 8 && wave >= 4;

  RowFrag<T, D> kf[NB], vf[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    kf[j].load(k + base, ts, k0 + 32 * j + (lane & 31), n, lane);
    kf[j].scale(scale * kLog2e);
    vf[j].load(v + base, ts, k0 + 32 * j + (lane & 31), n, lane);
  }
  f32x16 adv[D / 32][NB], adk[D / 32][NB], s[NB], dp[NB];
#pragma unroll
  for (int i = 0; i < D / 32; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) adv[i][j] = adk[i][j] = f32x16{};
#pragma unroll
  for (int j = 0; j < NB; ++j) s[j] = dp[j] = f32x16{};  // a staggered wave's V(-1) reads them
  XOp<T> pp[NB], ds[NB];  // zero operands for G of block -1 (see the dQ kernel)
#pragma unroll
  for (int j = 0; j < NB; ++j) pp[j] = ds[j] = XOp<T>(f32x16{});
#ifdef VD_DKDV_PRIO
  if (NW == 8 && wave >= 4) __builtin_amdgcn_s_setprio(1);  // A/B: as the dQ kernel
#endif

  tile_pipe<T, D, true, NW, NoSched,
            pipe_tr<D, NW>()>(
      smem, q + base, dout + obase, ts, ots, nlse2 + (int64_t)seq * n, ndelta + (int64_t)seq * n,
      n, tid, late,
      [&](const BlockRef<T>& bs) {
        // registers 4g..4g+3 are query rows 8g + 4hh + 0..3 of the block (the same rows
        // for every key block j: one load, the MFMA chains start from it)
        f32x16 ls0, dl0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 ls = *reinterpret_cast<const float4*>(bs.rc + bs.row0 + 8 * g + 4 * hh);
          const float4 dl = *reinterpret_cast<const float4*>(bs.rc1 + bs.row0 + 8 * g + 4 * hh);
          ls0[4 * g + 0] = ls.x; ls0[4 * g + 1] = ls.y; ls0[4 * g + 2] = ls.z; ls0[4 * g + 3] = ls.w;
          dl0[4 * g + 0] = dl.x; dl0[4 * g + 1] = dl.y; dl0[4 * g + 2] = dl.z; dl0[4 * g + 3] = dl.w;
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          s[j] = ls0;
          dp[j] = dl0;
        }
        mma_rows_nb<T, D, NB>(s, bs.a, bs.row0, kf, lane);   // S'[q][key] - lse'
        mma_rows_nb<T, D, NB>(dp, bs.b, bs.row0, vf, lane);  // dP[q][key] - delta
      },
      [&](const BlockRef<T>& bg) {
#pragma unroll
        for (int i = 0; i < D / 32; ++i) {
          mma_tr_nb<T, D, NB>(adv[i], bg.b, bg.row0, 32 * i, pp, lane);  // dV^T += dO^T P
          mma_tr_nb<T, D, NB>(adk[i], bg.a, bg.row0, 32 * i, ds, lane);  // dK^T += Q^T dS
        }
      },
      [&](const BlockRef<T>&) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            s[j][r] = fast_exp2(s[j][r]);
            dp[j][r] *= s[j][r];
          }
          pp[j] = XOp<T>(s[j]);
          ds[j] = XOp<T>(dp[j]);
        }
      });
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int mykey = k0 + 32 * j + (lane & 31);
    f32x16 ok[D / 32], ov[D / 32];
#pragma unroll
    for (int i = 0; i < D / 32; ++i) {
      ok[i] = adk[i][j];
      ov[i] = adv[i][j];
    }
    store_transposed<T, D / 32>(dk + base, ts, mykey, n, 0, ok, scale, lane);
    store_transposed<T, D / 32>(dv + base, ts, mykey, n, 0, ov, 1.f, lane);
  }
}

// ------------------------------------------------------------------ launchers
int check_attn(const vd_attn_desc* d) {
  VD_REQUIRE(d, "null descriptor");
  VD_REQUIRE(d->nseq > 0 && d->seq_len > 0 && d->groups > 0, "bad attention shape");
  VD_REQUIRE(d->head_dim == 32 || d->head_dim == 64 || d->head_dim == 128 || d->head_dim == 256,
             "head_dim %d unsupported (32/64/128/256)", d->head_dim);
  if (d->dtype == VD_BF16) {  // 32-bit buffer offsets of the LDS-DMA ring
    VD_REQUIRE(((int64_t)d->seq_len * d->token_stride + d->head_dim) * 2 < 0x7fffffffLL &&
                   ((int64_t)d->seq_len * d->o_token_stride + d->head_dim) * 2 < 0x7fffffffLL,
               "sequence spans >= 2 GiB");
  }
  return VD_OK;
}

// Work shape per kernel: NB x 32 rows per wave, NW waves per workgroup.
//   kNB2 : NB 2, NW 4 -- each LDS fragment feeds two MFMAs (bf16, D <= 128)
//   kW8  : NB 1, NW 8 -- two waves per SIMD from one workgroup, each LDS tile shared by
//          8 waves (bf16, D <= 128; at D = 128 the 256-register budget holds dQ, while the
//          forward spills and dK/dV needs a 64-column output slice per workgroup)
//   kBase: NB 1, NW 4
// VDIFF_ATTN_CFG=base|nb2|w8|p8|p4 overrides the choice for A/B measurements.
//   kP8 / kP4: the software-pipelined kernels (tile_pipe) with 8 / 4 waves (bf16, D <= 128;
//          8 waves only at D = 64)
//   kD8 / kD8N: the deferred-check forward (attn_fwd_defer_kernel, bf16, D = 64), 8 waves
//          with / without the staggered second half; other kernels keep their default
//   kD4: the deferred-check forward with 4 waves, two workgroups per CU (the SIMD partners
//          then come from different workgroups and share no barrier)
//   kRole: head_dim-256 dK/dV with role-split wave pairs (attn_bwd_dkdv_role_kernel)
//   kP4N2: the pipelined backward kernels with 4 waves x 2 blocks (one wave per SIMD,
//          each LDS fragment feeds two MFMAs; bf16, D = 64; fwd keeps its default)
//   kSP: retired (the fragment-pipelined backward measured equal to kP8, which it now
//          selects; profiles/r02_ab_sp.txt)
//   kAsm: the hand-scheduled kernels (asm/): head_dim-64 forward and backward, head_dim-128
//          backward; one wave per SIMD
//   kP8 / kP4 forward: retired (5 % slower than the deferred-check forward, which they select)
enum AttnCfg { kBase = 0, kNB2 = 1, kW8 = 2, kP8 = 3, kP4 = 4, kD8 = 5, kD8N = 6, kD4 = 7,
               kPair = 8, kP4N2 = 9, kRole = 10, kSP = 11, kAsm = 12, kCfgLast = kAsm };

int cfg_from_env() {
  const char* e = getenv("VDIFF_ATTN_CFG");
  if (!e) return -1;
  if (!strcmp(e, "nb2")) return (int)kNB2;
  if (!strcmp(e, "w8")) return (int)kW8;
  if (!strcmp(e, "p8")) return (int)kP8;
  if (!strcmp(e, "p4")) return (int)kP4;
  if (!strcmp(e, "base")) return (int)kBase;
  if (!strcmp(e, "d8")) return (int)kD8;
  if (!strcmp(e, "d8n")) return (int)kD8N;
  if (!strcmp(e, "d4")) return (int)kD4;
  if (!strcmp(e, "pair")) return (int)kPair;
  if (!strcmp(e, "p4n2")) return (int)kP4N2;
  if (!strcmp(e, "role")) return (int)kRole;
  if (!strcmp(e, "sp")) return (int)kSP;
  if (!strcmp(e, "asm")) return (int)kAsm;
  return -1;
}
std::atomic<int> g_cfg{cfg_from_env()};  // -1: per-kernel default (vd_attention_set_config)

// D = 256 hand-scheduled backward as the default (round 4; VDIFF_ASM256=0 restores the
// compiled base dQ / role-split dK/dV): dQ 0.506 -> 0.339 ms, dK/dV 0.804 -> 0.458 ms at
// N = 16384 on one box (tools/gpu_r04f.sh, profiles/r04f_ab_asm256_timing.txt)
const bool g_asm256 = [] {
  const char* e = getenv("VDIFF_ASM256");
  return !(e && atoi(e) == 0);
}();

// D = 256 hand-scheduled forward (asm/gen_fwd256.py) as the default (round 4;
// VDIFF_ASM256_FWD=0 restores the compiled 4-wave forward): 364-406 -> 240-242 us at
// N = 16384 on one box (tools/fwd256_ab.py, profiles/r04p_fwd256_ab.txt)
const bool g_asm256fwd = [] {
  const char* e = getenv("VDIFF_ASM256_FWD");
  return !(e && atoi(e) == 0);
}();

AttnCfg pick_cfg(int D, bool bf16, int kind) {
  const int env = g_cfg.load(std::memory_order_relaxed);
  if (!bf16) return kBase;
  AttnCfg c = kBase;
  // defaults = the fastest measured (tools/attn_bench.py, MI355X):
  //   D = 64 : fwd W8 17.2 ms, dQ P8 21.6 ms, dK/dV P8 29.1 ms (N = 262144); fwd D8N
  //            (deferred check, static priority) 17.7 vs W8 17.9-18.1 on the same box
  //   D = 128: fwd NB2 2.0 ms, dQ W8 2.8 ms (P4 3.7), dK/dV base 4.7 ms (N = 65536); fwd D8N
  //            2.01 vs NB2 2.32-2.35 ms on the same box (tools/attn_ab.sh); dK/dV PAIR
  //            (round 2) 3.84-3.96 vs base 4.84-4.85 ms on the same box (tools/ab_d128.sh)
  //   D = 64 backward (round 3): hand-scheduled dQ 18.8 / dK/dV 24.6 ms vs P8 20.8 / 28.9 ms
  //            on the same box (tools/gpu_asm.sh)
  //   D = 128 backward (round 3): hand-scheduled dQ 2.55-2.60 / dK/dV 3.37-3.40 ms vs W8 2.96 /
  //            PAIR 3.97-3.99 ms on the same box (tools/gpu_asm128.sh); forward 1.67-1.68 vs
  //            D8N 2.04-2.05 ms (tools/gpu_r03c.sh)
  //   D = 256 backward (round 4): hand-scheduled dQ 0.339 / dK/dV 0.458 ms vs base 0.506 /
  //            ROLE 0.804 ms (tools/gpu_r04f.sh); forward 0.240 vs base 0.364-0.406 ms
  //            (tools/fwd256_ab.py)
  if (env >= 0 && !((env == kD8 || env == kD8N || env == kD4) &&
                    ((D != 64 && !(D == 128 && env == kD8N)) || kind != 0)) &&
      !(env == kPair && (D != 128 || kind != 2)) &&  // the paired kernel: D = 128 dK/dV only
      !(env == kP4N2 && (D != 64 || kind == 0)) &&   // 2-block pipelined: D = 64 backward
      !(env == kSP && (D != 64 || kind == 0)) &&     // fragment-pipelined: D = 64 backward
      !(env == kAsm && D != 64 && D != 128 && D != 256) &&  // hand-scheduled
      !(env == kRole && (D != 256 || kind != 2)))    // role-split pairs: D = 256 dK/dV
    c = (AttnCfg)env;
  else if (D == 64) c = kAsm;  // falls back to D8N / P8 off its shapes
  else if (D == 128) c = kAsm;  // asm falls back to D8N / W8 / PAIR off its shapes
  else if (D == 256 && kind != 0) c = g_asm256 ? kAsm : (kind == 2 ? kRole : kBase);
  else if (D == 256 && kind == 0 && g_asm256fwd) c = kAsm;
  if (c == kNB2 && (D == 256 || (kind == 2 && D > 64))) c = kBase;
  if (c == kW8 && D != 64 && D != 128) c = kBase;  // 8 waves need >= 1 DMA piece each
  if (c == kP8 && D != 64) c = kP4;
  if (c == kP4 && D > 128) c = kBase;
  return c;
}

// KV splits for a query grid of `wgs` workgroups: enough to give every CU one (>= 256),
// at most 4, at least 4 key tiles each; 1 = no split.  bf16 only.
int kv_splits(const vd_attn_desc* d, int64_t wgs, int nkv) {
  if (d->dtype != VD_BF16 || wgs >= 256) return 1;
  int s = (int)((256 + wgs - 1) / wgs);
  if (s > 4) s = 4;
  const int64_t tiles = vd_cdiv(nkv, kTile);
  while (s > 1 && tiles / s < 4) --s;
  return s;
}
int split_tps(int len, int s) { return (int)vd_cdiv(vd_cdiv(len, kTile), s); }

KvAddr self_kv(const vd_attn_desc* d) {
  return KvAddr{SeqAddr{d->batch_stride, d->group_stride, d->groups}, d->token_stride,
                d->seq_len};
}

// dK/dV output-column slice of the 4-wave generic kernel (register budget at D = 256)
template <int D, int NW> constexpr int dkdv_do() { return D > 128 ? 128 : (D == 128 && NW == 8 ? 64 : D); }

// Query splits of the 4-wave dK/dV kernel when its key grid leaves CUs idle (bf16):
// at most 16, at least 4 query tiles each; 1 = no split.
template <int D>
int q_splits(const vd_attn_desc* d, int nkv) {
  if (d->dtype != VD_BF16) return 1;
  const int64_t wgs = vd_cdiv(nkv, 128) * d->nseq * (D / dkdv_do<D, 4>());
  if (wgs >= 256) return 1;
  int s = (int)((256 + wgs - 1) / wgs);
  if (s > 16) s = 16;
  const int64_t tiles = vd_cdiv(d->seq_len, kTile);
  while (s > 1 && tiles / s < 4) --s;
  return s;
}

// query splits of the role-split head_dim-256 dK/dV grid (16 NW keys per workgroup)
int role_q_splits(const vd_attn_desc* d, int nkv) {
  const int64_t wgs = vd_cdiv(nkv, 16 * VD_ROLE_NW) * d->nseq;
  if (wgs >= 256) return 1;
  int s = (int)((256 + wgs - 1) / wgs);
  if (s > 16) s = 16;
  const int64_t tiles = vd_cdiv(d->seq_len, kTile);
  while (s > 1 && tiles / s < 4) --s;
  return s;
}

// key splits (log2) of the hand-scheduled head_dim-256 dQ: the query grid (128 queries per
// workgroup) times the splits covers the 256 CUs, at most 4 splits, every split non-empty
// and a whole number of 4-tile (128-key) loop iterations
// VDIFF_ASM256_DQ_L / VDIFF_ASM256_DKDV_L (diagnostics): cap the split count's log2
static int lsplit_cap(const char* env, int dflt) {
  const char* e = getenv(env);
  return e ? std::max(0, std::min(dflt, atoi(e))) : dflt;
}
int dq256_lsplit(const vd_attn_desc* d) {
  const int64_t n = d->seq_len, wgs = vd_cdiv(n, 128) * d->nseq;
  const int cap = lsplit_cap("VDIFF_ASM256_DQ_L", 2);
  int l = 0;
  while (l < cap && (wgs << l) < 256) {
    const int64_t S = 2 << l, kps = vd_cdiv(vd_cdiv(n, S), 128) * 128;
    if ((S - 1) * kps >= n) break;
    ++l;
  }
  return l;
}
int64_t dq256_kps(const vd_attn_desc* d, int l) {
  return vd_cdiv(vd_cdiv(d->seq_len, (int64_t)1 << l), 128) * 128;
}
// key splits (log2) of the hand-scheduled head_dim-256 forward: the dQ rule (128 queries per
// workgroup, 128-key iterations, every split non-empty); attn_fwd_combine_kernel merges <= 4
int fwd256_lsplit(const vd_attn_desc* d) {
  const int64_t n = d->seq_len, wgs = vd_cdiv(n, 128) * d->nseq;
  const int cap = lsplit_cap("VDIFF_ASM256_FWD_L", 2);
  int l = 0;
  while (l < cap && (wgs << l) < 256) {
    const int64_t S = 2 << l, kps = vd_cdiv(vd_cdiv(n, S), 128) * 128;
    if ((S - 1) * kps >= n) break;
    ++l;
  }
  return l;
}

// query splits (log2) of the hand-scheduled head_dim-256 dK/dV (64 keys per workgroup): up to
// 16, every split non-empty and a whole number of 4-tile (128-query) loop iterations
int dkdv256_lsplit(const vd_attn_desc* d) {
  const int64_t n = d->seq_len, wgs = vd_cdiv(n, 64) * d->nseq;
  const int cap = lsplit_cap("VDIFF_ASM256_DKDV_L", 4);
  int l = 0;
  while (l < cap && (wgs << l) < 256) {
    const int64_t S = 2 << l, qps = vd_cdiv(vd_cdiv(n, S), 128) * 128;
    if ((S - 1) * qps >= n) break;
    ++l;
  }
  return l;
}

// Backward workspace: [ndelta rows][nlse2 rows][64 floats][dQ KV-split partials]
// [dK/dV query-split partials]; rows = nseq * seq_len (queries).
struct BwdWs {
  int sdq, sq;       // KV splits of the dQ pass, query splits of the dK/dV pass
  size_t dq_off, kv_off, bytes;  // float offsets of the partials; total bytes
};
template <int D>
BwdWs bwd_ws(const vd_attn_desc* d, int nkv, bool cross) {
  BwdWs w{1, 1, 0, 0, 0};
  const size_t rows = (size_t)d->nseq * d->seq_len;
  if (d->dtype == VD_BF16 && (cross || pick_cfg(D, true, 1) == kBase))
    w.sdq = kv_splits(d, vd_cdiv(d->seq_len, 128) * d->nseq, nkv);
  // hand-scheduled D = 256 dQ: its key splits (the compiled fallback of a misaligned call
  // splits as the base shape does; the partial region fits either)
  if (D == 256 && !cross && d->dtype == VD_BF16 && pick_cfg(D, true, 1) == kAsm)
    w.sdq = std::max(1 << dq256_lsplit(d), kv_splits(d, vd_cdiv(d->seq_len, 128) * d->nseq, nkv));
  if (cross || (d->dtype == VD_BF16 && pick_cfg(D, true, 2) == kBase)) w.sq = q_splits<D>(d, nkv);
  else if (D == 256 && d->dtype == VD_BF16 && pick_cfg(D, true, 2) == kRole)
    w.sq = role_q_splits(d, nkv);
  else if (D == 256 && d->dtype == VD_BF16 && pick_cfg(D, true, 2) == kAsm)
    w.sq = std::max(1 << dkdv256_lsplit(d), q_splits<D>(d, nkv));  // (+ the base fallback)
  w.dq_off = 2 * rows + 64;
  w.kv_off = w.dq_off + (w.sdq > 1 ? (size_t)w.sdq * rows * D : 0);
  const size_t kvp = w.sq > 1 ? (size_t)w.sq * d->nseq * nkv * 2 * D : 0;
  w.bytes = (w.kv_off + kvp) * sizeof(float);
  return w;
}

template <typename T, int D, int NB, int NW>
int fwd_launch(const vd_attn_desc* d, KvAddr kv, const void* q, const void* k, const void* v,
               void* o, float* lse, void* ws, size_t ws_bytes, hipStream_t st) {
  const size_t lds = tile_loop_lds<T, D, false>();
  auto kern = attn_fwd_kernel<T, D, NB, NW>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  const int64_t qwg = vd_cdiv(d->seq_len, 32 * NB * NW);
  int s = kv_splits(d, qwg * d->nseq, kv.n);
  const size_t need = (size_t)s * d->nseq * d->seq_len * (D + 2) * sizeof(float);
  if (s > 1 && (!ws || ws_bytes < need)) s = 1;
  FwdSplit split{s > 1 ? (float*)ws : nullptr, split_tps(kv.n, s)};
  if (s > 1) s = (int)vd_cdiv(vd_cdiv(kv.n, kTile), split.tps);
  dim3 grid((unsigned)qwg, (unsigned)d->nseq, (unsigned)s);
  const SeqAddr oa{d->o_batch_stride, d->o_group_stride, d->groups};
  kern<<<grid, 64 * NW, lds, st>>>((const T*)q, (const T*)k, (const T*)v, (T*)o, lse,
                                   d->seq_len, SeqAddr{d->batch_stride, d->group_stride, d->groups},
                                   d->token_stride, oa, d->o_token_stride, d->scale, split, kv);
  if (s > 1) {
    const int rc = vd::check_launch("attn_fwd");
    if (rc) return rc;
    const int64_t work = (int64_t)d->nseq * d->seq_len * (D / 8);
    int g = (int)vd_cdiv(work, 256);
    if (g > 4096) g = 4096;
    attn_fwd_combine_kernel<T, D><<<g, 256, 0, st>>>(split.part, s, d->nseq, d->seq_len, (T*)o,
                                                     oa, d->o_token_stride, lse);
  }
  return vd::check_launch("attn_fwd");
}

// bytes of the KV-split forward workspace of this shape (0: no split is used)
template <int D>
size_t fwd_ws_bytes(const vd_attn_desc* d, int nkv, bool cross) {
  if (d->dtype != VD_BF16) return 0;
  int s = 1;
  if (D == 256 && !cross && pick_cfg(D, true, 0) == kAsm)  // the asm split or the base fallback
    s = std::max(1 << fwd256_lsplit(d), kv_splits(d, vd_cdiv(d->seq_len, 128) * d->nseq, nkv));
  else if (!cross && pick_cfg(D, true, 0) != kBase) return 0;  // only the 4-wave shape splits
  else s = kv_splits(d, vd_cdiv(d->seq_len, 128) * d->nseq, nkv);
  return s > 1 ? (size_t)s * d->nseq * d->seq_len * (D + 2) * sizeof(float) : 0;
}


template <typename T, int D, int NW, bool STAGGER>
int fwd_defer_launch(const vd_attn_desc* d, const void* q, const void* k, const void* v, void* o,
                     float* lse, hipStream_t st) {
  const size_t lds = (size_t)defer_nst<D, NW>() * pipe_stage_bytes<D, false, kTile>();
  auto kern = attn_fwd_defer_kernel<T, D, NW, STAGGER>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  dim3 grid((unsigned)vd_cdiv(d->seq_len, 32 * NW), (unsigned)d->nseq);
  kern<<<grid, 64 * NW, lds, st>>>((const T*)q, (const T*)k, (const T*)v, (T*)o, lse,
                                   d->seq_len, SeqAddr{d->batch_stride, d->group_stride, d->groups},
                                   d->token_stride,
                                   SeqAddr{d->o_batch_stride, d->o_group_stride, d->groups},
                                   d->o_token_stride, d->scale);
  return vd::check_launch("attn_fwd");
}

// hand-scheduled head_dim-64 dQ (asm/gen_attn_asm.py): one wave per SIMD, 256 queries per
// workgroup, tiles rounded up to the 4-stage ring; 32-bit buffer offsets of every row it
// touches (the last DMA'd tiles run up to 5 tiles past the end), 16-B aligned rows
inline bool asm_dq_ok(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                      const void* dout, const void* dq, int D = 64) {
  const int64_t n = d->seq_len;
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return d->dtype == VD_BF16 && d->head_dim == D && n >= 16 * kTile && d->nseq % d->groups == 0 &&
         d->token_stride % 8 == 0 && d->o_token_stride % 8 == 0 && d->token_stride >= D &&
         d->o_token_stride >= D && d->batch_stride % 8 == 0 && d->group_stride % 8 == 0 &&
         d->o_batch_stride % 8 == 0 && d->o_group_stride % 8 == 0 &&
         (n + 512) * d->token_stride * 2 < 0x7fffffffLL &&
         (n + 512) * d->o_token_stride * 2 < 0x7fffffffLL && al(q) && al(k) && al(v) &&
         al(dout) && al(dq);
}

// hand-scheduled head_dim-64 forward (asm/gen_fwd.py): the dQ kernel's shape conditions
// (the DMA runs up to 12 tiles past the end of the sequence: the 512-key rounding plus the
// 4-tile prefetch) and a 4-byte aligned lse
inline bool asm_fwd_ok(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                       const void* o, const float* lse, int D = 64) {
  const int64_t n = d->seq_len;
  return asm_dq_ok(d, q, k, v, o, o, D) && (n + 1024) * d->token_stride * 2 < 0x7fffffffLL &&
         ((uintptr_t)lse & 3) == 0;
}

// hand-scheduled forward: head_dim 64 (64-key tiles, asm/gen_fwd.py) or 128 (32-key tiles,
// asm/gen_fwd128.py); 8 tiles per iteration, the last iteration masked
int fwd_asm_launch(const vd_attn_desc* d, const void* q, const void* k, const void* v, void* o,
                   float* lse, hipStream_t st) {
  const int64_t n = d->seq_len;
  const int D = d->head_dim, TR = D == 128 ? 32 : 64;
  vd::AsmFwdArgs a{};
  a.q = q; a.k = k; a.v = v; a.o = o; a.lse = lse;
  a.n = (uint32_t)n;
  a.ts_bytes = (uint32_t)(d->token_stride * 2);
  a.ots_bytes = (uint32_t)(d->o_token_stride * 2);
  a.groups = (uint32_t)d->groups;
  a.bs_bytes = (uint64_t)d->batch_stride * 2;
  a.gs_bytes = (uint64_t)d->group_stride * 2;
  a.obs_bytes = (uint64_t)d->o_batch_stride * 2;
  a.ogs_bytes = (uint64_t)d->o_group_stride * 2;
  a.qscale = d->scale * kLog2e;  // the fp32 product RowFrag::scale receives
  a.kv_bytes = (uint32_t)(((n - 1) * d->token_stride + D) * 2);
  a.o_bytes = (uint32_t)(((n - 1) * d->o_token_stride + D) * 2);
  a.tile_bytes = (uint32_t)(TR * d->token_stride * 2);
  a.niter = (uint32_t)vd_cdiv(n, 8 * TR);
  a.klim0 = (uint32_t)(n - 8 * TR * (int64_t)(a.niter - 1));
  const unsigned gx = (unsigned)vd_cdiv(n, 256), gy = (unsigned)d->groups,
                 gz = (unsigned)(d->nseq / d->groups);
  const int rc = D == 128 ? vd::asm_fwd_d128(a, gx, gy, gz, st) : vd::asm_fwd_d64(a, gx, gy, gz, st);
  return rc ? rc : vd::check_launch("attn_fwd");
}

// hand-scheduled head_dim-256 forward (asm/gen_fwd256.py, 128 queries per workgroup) with its
// key split into FwdSplit partials (ws: the forward workspace; too small -> no split)
int fwd256_asm_launch(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                      void* o, float* lse, void* ws, size_t ws_bytes, hipStream_t st) {
  const int64_t n = d->seq_len;
  const size_t rows = (size_t)d->nseq * n;
  int l = fwd256_lsplit(d);
  if (l && (!ws || ws_bytes < ((size_t)1 << l) * rows * (256 + 2) * sizeof(float))) l = 0;
  const int64_t kps = dq256_kps(d, l);
  vd::AsmFwd256Args a{};
  vd::AsmFwdArgs& b = a.b;
  b.q = q; b.k = k; b.v = v; b.o = o; b.lse = lse;
  b.n = (uint32_t)n;
  b.ts_bytes = (uint32_t)(d->token_stride * 2);
  b.ots_bytes = (uint32_t)(d->o_token_stride * 2);
  b.groups = (uint32_t)d->groups;
  b.bs_bytes = (uint64_t)d->batch_stride * 2;
  b.gs_bytes = (uint64_t)d->group_stride * 2;
  b.obs_bytes = (uint64_t)d->o_batch_stride * 2;
  b.ogs_bytes = (uint64_t)d->o_group_stride * 2;
  b.qscale = d->scale * kLog2e;
  b.kv_bytes = (uint32_t)(((n - 1) * d->token_stride + 256) * 2);
  b.o_bytes = (uint32_t)(((n - 1) * d->o_token_stride + 256) * 2);
  b.tile_bytes = (uint32_t)(32 * d->token_stride * 2);
  float* part = l ? (float*)ws : nullptr;
  a.part = part;
  a.kps = (uint32_t)kps;
  a.lsplit = (uint32_t)l;
  a.split_bytes = (uint64_t)rows * 1024;
  a.ml_off = ((uint64_t)1 << l) * rows * 1024;
  a.ml_split_bytes = (uint32_t)(rows * 8);
  const unsigned gy = (unsigned)d->groups, gz = (unsigned)(d->nseq / d->groups) << l;
  int rc = vd::asm_fwd_d256(a, (unsigned)vd_cdiv(n, 128), gy, gz, st);
  if (rc) return rc;
  if (l) {
    rc = vd::check_launch("attn_fwd");
    if (rc) return rc;
    const SeqAddr oa{d->o_batch_stride, d->o_group_stride, d->groups};
    const int64_t work = (int64_t)rows * (256 / 8);
    int g = (int)vd_cdiv(work, 256);
    if (g > 4096) g = 4096;
    attn_fwd_combine_kernel<bf16_t, 256><<<g, 256, 0, st>>>(part, 1 << l, d->nseq, (int)n,
                                                           (bf16_t*)o, oa, d->o_token_stride,
                                                           lse);
  }
  return vd::check_launch("attn_fwd");
}

template <typename T, int D>
int fwd_impl(const vd_attn_desc* d, KvAddr kv, bool cross, const void* q, const void* k,
             const void* v, void* o, float* lse, void* ws, size_t ws_bytes, hipStream_t st) {
  // cross-attention runs on the generic 4-wave kernel (its K/V sequences are short)
  if constexpr (kDMA<T>) if (!cross) {
    const AttnCfg c = pick_cfg(D, true, 0);
    if constexpr (D != 256)
      if (c == kNB2) return fwd_launch<T, D, 2, 4>(d, kv, q, k, v, o, lse, nullptr, 0, st);
    if constexpr (D == 64 || D == 128)
      if (c == kW8) return fwd_launch<T, D, 1, 8>(d, kv, q, k, v, o, lse, nullptr, 0, st);
    if constexpr (D == 64) {
      if (c == kAsm && asm_fwd_ok(d, q, k, v, o, lse))
        return fwd_asm_launch(d, q, k, v, o, lse, st);
      if (c == kP8 || c == kAsm) return fwd_defer_launch<T, D, 8, false>(d, q, k, v, o, lse, st);
      if (c == kD8) return fwd_defer_launch<T, D, 8, true>(d, q, k, v, o, lse, st);
      if (c == kD8N) return fwd_defer_launch<T, D, 8, false>(d, q, k, v, o, lse, st);
      if (c == kD4) return fwd_defer_launch<T, D, 4, false>(d, q, k, v, o, lse, st);
    }
    if constexpr (D == 128)
      if (c == kAsm && asm_fwd_ok(d, q, k, v, o, lse, D))
        return fwd_asm_launch(d, q, k, v, o, lse, st);
    if constexpr (D == 256)
      if (c == kAsm && asm_fwd_ok(d, q, k, v, o, lse, D))
        return fwd256_asm_launch(d, q, k, v, o, lse, ws, ws_bytes, st);
    if constexpr (D == 128)
      if (c == kD8N || c == kAsm) return fwd_defer_launch<T, D, 8, false>(d, q, k, v, o, lse, st);
    if constexpr (D == 64 || D == 128)  // the pipelined forward is retired: its successor
      if (c == kP4) return fwd_defer_launch<T, D, 8, false>(d, q, k, v, o, lse, st);
  }
  return fwd_launch<T, D, 1, 4>(d, kv, q, k, v, o, lse, ws, ws_bytes, st);
}

template <typename T, int D, int NB, int NW>
int dq_launch(const vd_attn_desc* d, KvAddr kv, const void* q, const void* k, const void* v,
              const void* dout, const float* nlse2, const float* ndelta, void* dq,
              hipStream_t st, float* part = nullptr, int sdq = 1) {
  const SeqAddr qa{d->batch_stride, d->group_stride, d->groups};
  const SeqAddr oa{d->o_batch_stride, d->o_group_stride, d->groups};
  const size_t lds = tile_loop_lds<T, D, false>();
  auto kern = attn_bwd_dq_kernel<T, D, NB, NW>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  const int64_t qwg = vd_cdiv(d->seq_len, 32 * NB * NW);
  int s = part ? sdq : 1;
  FwdSplit split{s > 1 ? part : nullptr, split_tps(kv.n, s)};
  if (s > 1) s = (int)vd_cdiv(vd_cdiv(kv.n, kTile), split.tps);
  dim3 grid((unsigned)qwg, (unsigned)d->nseq, (unsigned)s);
  kern<<<grid, 64 * NW, lds, st>>>((const T*)q, (const T*)k, (const T*)v, (const T*)dout, nlse2,
                                   ndelta, (T*)dq, d->seq_len, qa, d->token_stride, oa,
                                   d->o_token_stride, d->scale, split, kv);
  if (s > 1) {
    const int rc = vd::check_launch("attn_bwd_dq");
    if (rc) return rc;
    const int64_t work = (int64_t)d->nseq * d->seq_len * (D / 8);
    int g = (int)vd_cdiv(work, 256);
    if (g > 4096) g = 4096;
    attn_dq_sum_kernel<T, D><<<g, 256, 0, st>>>(split.part, s, d->nseq, d->seq_len, (T*)dq, qa,
                                               d->token_stride);
  }
  return vd::check_launch("attn_bwd_dq");
}

template <typename T, int D, int NW, int NB = 1>
int dq_pipe_launch(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                   const void* dout, const float* nlse2, const float* ndelta, void* dq,
                   hipStream_t st) {
  const SeqAddr qa{d->batch_stride, d->group_stride, d->groups};
  const SeqAddr oa{d->o_batch_stride, d->o_group_stride, d->groups};
  const size_t lds = tile_pipe_lds<D, false, pipe_tr<D, NW>()>();
  auto kern = attn_bwd_dq_pipe_kernel<T, D, NW, NB>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  dim3 grid((unsigned)vd_cdiv(d->seq_len, 32 * NB * NW), (unsigned)d->nseq);
  kern<<<grid, 64 * NW, lds, st>>>((const T*)q, (const T*)k, (const T*)v, (const T*)dout, nlse2,
                                   ndelta, (T*)dq, d->seq_len, qa, d->token_stride, oa,
                                   d->o_token_stride, d->scale);
  return vd::check_launch("attn_bwd_dq");
}

// hand-scheduled dQ: head_dim 64 (256 queries per workgroup) or 128 (asm/gen_d128.py, 128)
int dq_asm_launch(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                  const void* dout, const float* nlse2, const float* ndelta, void* dq,
                  hipStream_t st) {
  const int64_t n = d->seq_len;
  const int D = d->head_dim;
  vd::AsmDqArgs a{};
  a.q = q; a.k = k; a.v = v; a.dout = dout; a.nlse2 = nlse2; a.ndelta = ndelta; a.dq = dq;
  a.n = (uint32_t)n;
  a.ts_bytes = (uint32_t)(d->token_stride * 2);
  a.ots_bytes = (uint32_t)(d->o_token_stride * 2);
  a.groups = (uint32_t)d->groups;
  a.bs_bytes = (uint64_t)d->batch_stride * 2;
  a.gs_bytes = (uint64_t)d->group_stride * 2;
  a.obs_bytes = (uint64_t)d->o_batch_stride * 2;
  a.ogs_bytes = (uint64_t)d->o_group_stride * 2;
  a.scale = d->scale;
  a.qscale = d->scale * kLog2e;  // the fp32 product RowFrag::scale receives
  a.kv_bytes = (uint32_t)(((n - 1) * d->token_stride + D) * 2);
  a.o_bytes = (uint32_t)(((n - 1) * d->o_token_stride + D) * 2);
  a.tile_bytes = (uint32_t)(kTile * d->token_stride * 2);
  a.niter = (uint32_t)vd_cdiv(vd_cdiv(n, kTile), 4);
  const unsigned gy = (unsigned)d->groups, gz = (unsigned)(d->nseq / d->groups);
  const int rc = D == 128 ? vd::asm_bwd_dq_d128(a, (unsigned)vd_cdiv(n, 128), gy, gz, st)
                          : vd::asm_bwd_dq_d64(a, (unsigned)vd_cdiv(n, 256), gy, gz, st);
  return rc ? rc : vd::check_launch("attn_bwd_dq");
}

// hand-scheduled head_dim-256 dQ (asm/gen_d256.py, 128 queries per workgroup) with its key
// split into fp32 partials (part: the dQ partial region of the backward workspace)
int dq256_asm_launch(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                     const void* dout, const float* nlse2, const float* ndelta, void* dq,
                     float* part, hipStream_t st) {
  const int64_t n = d->seq_len;
  const int l = dq256_lsplit(d);
  const int64_t kps = dq256_kps(d, l);
  vd::AsmDq256Args a{};
  vd::AsmDqArgs& b = a.b;
  b.q = q; b.k = k; b.v = v; b.dout = dout; b.nlse2 = nlse2; b.ndelta = ndelta; b.dq = dq;
  b.n = (uint32_t)n;
  b.ts_bytes = (uint32_t)(d->token_stride * 2);
  b.ots_bytes = (uint32_t)(d->o_token_stride * 2);
  b.groups = (uint32_t)d->groups;
  b.bs_bytes = (uint64_t)d->batch_stride * 2;
  b.gs_bytes = (uint64_t)d->group_stride * 2;
  b.obs_bytes = (uint64_t)d->o_batch_stride * 2;
  b.ogs_bytes = (uint64_t)d->o_group_stride * 2;
  b.scale = d->scale;
  b.qscale = d->scale * kLog2e;
  b.kv_bytes = (uint32_t)(((n - 1) * d->token_stride + 256) * 2);
  b.o_bytes = (uint32_t)(((n - 1) * d->o_token_stride + 256) * 2);
  b.tile_bytes = (uint32_t)(32 * d->token_stride * 2);
  b.niter = (uint32_t)vd_cdiv(vd_cdiv(kps, 32), 4);
  a.part = l ? part : nullptr;
  a.kps = (uint32_t)kps;
  a.lsplit = (uint32_t)l;
  a.split_bytes = (uint64_t)d->nseq * n * 1024;
  a.part_bytes = (uint32_t)(n * 1024);
  const unsigned gy = (unsigned)d->groups, gz = (unsigned)(d->nseq / d->groups) << l;
  int rc = vd::asm_bwd_dq_d256(a, (unsigned)vd_cdiv(n, 128), gy, gz, st);
  if (rc) return rc;
  if (l) {
    rc = vd::check_launch("attn_bwd_dq");
    if (rc) return rc;
    const SeqAddr qa{d->batch_stride, d->group_stride, d->groups};
    const int64_t work = (int64_t)d->nseq * n * (256 / 8);
    int g = (int)vd_cdiv(work, 256);
    if (g > 4096) g = 4096;
    attn_dq_sum_kernel<bf16_t, 256><<<g, 256, 0, st>>>(part, 1 << l, d->nseq, (int)n,
                                                       (bf16_t*)dq, qa, d->token_stride);
  }
  return vd::check_launch("attn_bwd_dq");
}

// hand-scheduled head_dim-256 dK/dV (asm/gen_d256dk.py, role-split wave pairs, 64 keys per
// workgroup) with its query split into fp32 partials (part: the dK/dV partial region)
int dkdv256_asm_launch(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                       const void* dout, const float* nlse2, const float* ndelta, void* dk,
                       void* dv, float* part, hipStream_t st) {
  const int64_t n = d->seq_len;
  const int l = dkdv256_lsplit(d);
  const int64_t qps = vd_cdiv(vd_cdiv(n, (int64_t)1 << l), 128) * 128;
  vd::AsmDkdv256Args a{};
  vd::AsmDkdvArgs& b = a.b;
  b.q = q; b.k = k; b.v = v; b.dout = dout; b.nlse2 = nlse2; b.ndelta = ndelta;
  b.dk = dk; b.dv = dv;
  b.n = (uint32_t)n;
  b.ts_bytes = (uint32_t)(d->token_stride * 2);
  b.ots_bytes = (uint32_t)(d->o_token_stride * 2);
  b.groups = (uint32_t)d->groups;
  b.bs_bytes = (uint64_t)d->batch_stride * 2;
  b.gs_bytes = (uint64_t)d->group_stride * 2;
  b.obs_bytes = (uint64_t)d->o_batch_stride * 2;
  b.ogs_bytes = (uint64_t)d->o_group_stride * 2;
  b.scale = d->scale;
  b.kscale = d->scale * kLog2e;
  b.kv_bytes = (uint32_t)(((n - 1) * d->token_stride + 256) * 2);
  b.o_bytes = (uint32_t)(((n - 1) * d->o_token_stride + 256) * 2);
  b.tile_bytes = (uint32_t)(32 * d->token_stride * 2);
  b.otile_bytes = (uint32_t)(32 * d->o_token_stride * 2);
  b.niter = (uint32_t)vd_cdiv(vd_cdiv(qps, 32), 4);
  a.part = l ? part : nullptr;
  a.qps = (uint32_t)qps;
  a.lsplit = (uint32_t)l;
  a.split_bytes = (uint64_t)d->nseq * n * 2048;
  a.part_bytes = (uint32_t)(n * 2048);
  const unsigned gy = (unsigned)d->groups, gz = (unsigned)(d->nseq / d->groups) << l;
  int rc = vd::asm_bwd_dkdv_d256(a, (unsigned)vd_cdiv(n, 64), gy, gz, st);
  if (rc) return rc;
  if (l) {
    rc = vd::check_launch("attn_bwd_dkdv");
    if (rc) return rc;
    const int64_t work = (int64_t)d->nseq * n * (2 * 256 / 8);
    int g = (int)vd_cdiv(work, 256);
    if (g > 4096) g = 4096;
    attn_dkdv_sum_kernel<bf16_t, 256><<<g, 256, 0, st>>>(part, 1 << l, d->nseq, (int)n,
                                                         (bf16_t*)dk, (bf16_t*)dv,
                                                         self_kv(d).a, d->token_stride);
  }
  return vd::check_launch("attn_bwd_dkdv");
}

// hand-scheduled dK/dV: head_dim 64 (256 keys per workgroup) or 128 (asm/gen_d128.py, 128)
int dkdv_asm_launch(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                    const void* dout, const float* nlse2, const float* ndelta, void* dk, void* dv,
                    hipStream_t st) {
  const int D = d->head_dim;
  const int64_t n = d->seq_len;
  vd::AsmDkdvArgs a{};
  a.q = q; a.k = k; a.v = v; a.dout = dout; a.nlse2 = nlse2; a.ndelta = ndelta;
  a.dk = dk; a.dv = dv;
  a.n = (uint32_t)n;
  a.ts_bytes = (uint32_t)(d->token_stride * 2);
  a.ots_bytes = (uint32_t)(d->o_token_stride * 2);
  a.groups = (uint32_t)d->groups;
  a.bs_bytes = (uint64_t)d->batch_stride * 2;
  a.gs_bytes = (uint64_t)d->group_stride * 2;
  a.obs_bytes = (uint64_t)d->o_batch_stride * 2;
  a.ogs_bytes = (uint64_t)d->o_group_stride * 2;
  a.scale = d->scale;
  a.kscale = d->scale * kLog2e;
  a.kv_bytes = (uint32_t)(((n - 1) * d->token_stride + D) * 2);
  a.o_bytes = (uint32_t)(((n - 1) * d->o_token_stride + D) * 2);
  a.tile_bytes = (uint32_t)(kTile * d->token_stride * 2);
  a.otile_bytes = (uint32_t)(kTile * d->o_token_stride * 2);
  a.niter = (uint32_t)vd_cdiv(vd_cdiv(n, kTile), 4);
  const unsigned gy = (unsigned)d->groups, gz = (unsigned)(d->nseq / d->groups);
  const int rc = D == 128 ? vd::asm_bwd_dkdv_d128(a, (unsigned)vd_cdiv(n, 128), gy, gz, st)
                          : vd::asm_bwd_dkdv_d64(a, (unsigned)vd_cdiv(n, 256), gy, gz, st);
  return rc ? rc : vd::check_launch("attn_bwd_dkdv");
}

template <typename T, int D>
int bwd_dq_impl(const vd_attn_desc* d, KvAddr kv, bool cross, const void* q, const void* k,
                const void* v, const void* o, const void* dout, const float* lse, void* dq,
                void* ws, hipStream_t st) {
  const SeqAddr oa{d->o_batch_stride, d->o_group_stride, d->groups};
  const int64_t rows = (int64_t)d->nseq * d->seq_len;
  float* ndelta = reinterpret_cast<float*>(ws);  // workspace: [ndelta rows][nlse2 rows]
  float* nlse2 = ndelta + rows;
  int g = (int)vd_cdiv(rows, 256);
  if (g > 4096) g = 4096;
  attn_delta_kernel<T, D><<<g, 256, 0, st>>>((const T*)o, (const T*)dout, lse, ndelta, nlse2,
                                              d->nseq, d->seq_len, oa, d->o_token_stride);
  int rc = vd::check_launch("attn_delta");
  if (rc) return rc;
  if constexpr (kDMA<T>) if (!cross) {
    const AttnCfg c = pick_cfg(D, true, 1);
    if constexpr (D != 256)
      if (c == kNB2) return dq_launch<T, D, 2, 4>(d, kv, q, k, v, dout, nlse2, ndelta, dq, st);
    if constexpr (D == 128)
      if (c == kAsm && asm_dq_ok(d, q, k, v, dout, dq, D))
        return dq_asm_launch(d, q, k, v, dout, nlse2, ndelta, dq, st);
    if constexpr (D == 64 || D == 128)
      if (c == kW8 || (D == 128 && c == kAsm))
        return dq_launch<T, D, 1, 8>(d, kv, q, k, v, dout, nlse2, ndelta, dq, st);
    if constexpr (D == 64)
      if (c == kAsm && asm_dq_ok(d, q, k, v, dout, dq))
        return dq_asm_launch(d, q, k, v, dout, nlse2, ndelta, dq, st);
    if constexpr (D == 64)
      if (c == kP8 || c == kSP || c == kAsm)
        return dq_pipe_launch<T, D, 8>(d, q, k, v, dout, nlse2, ndelta, dq, st);
    if constexpr (D == 64)
      if (c == kP4N2) return dq_pipe_launch<T, D, 4, 2>(d, q, k, v, dout, nlse2, ndelta, dq, st);
    if constexpr (D <= 128)
      if (c == kP4) return dq_pipe_launch<T, D, 4>(d, q, k, v, dout, nlse2, ndelta, dq, st);
    if constexpr (D == 256)
      if (c == kAsm && asm_dq_ok(d, q, k, v, dout, dq, D)) {
        const BwdWs w = bwd_ws<D>(d, kv.n, cross);
        return dq256_asm_launch(d, q, k, v, dout, nlse2, ndelta, dq,
                                reinterpret_cast<float*>(ws) + w.dq_off, st);
      }
  }
  // the 4-wave, 32-row shape splits the keys when its grid leaves CUs idle (bf16, D = 256):
  // fp32 partials after the row constants in the workspace (vd_attention_bwd_workspace_size)
  const BwdWs w = bwd_ws<D>(d, kv.n, cross);
  return dq_launch<T, D, 1, 4>(d, kv, q, k, v, dout, nlse2, ndelta, dq, st,
                               reinterpret_cast<float*>(ws) + w.dq_off, w.sdq);
}

template <typename T, int D, int NB, int NW>
int dkdv_launch(const vd_attn_desc* d, KvAddr kv, const void* q, const void* k, const void* v,
                const void* dout, const float* nlse2, const float* ndelta, void* dk, void* dv,
                hipStream_t st, float* part = nullptr, int sq = 1) {
  const SeqAddr qa{d->batch_stride, d->group_stride, d->groups};
  const SeqAddr oa{d->o_batch_stride, d->o_group_stride, d->groups};
  // output-column slice per workgroup (grid.z = D / DO): register budget at D = 256, and at
  // D = 128 with 8 waves (two per SIMD: 256 registers each)
  constexpr int DO = dkdv_do<D, NW>();
  const size_t lds = tile_loop_lds<T, D, true>();
  auto kern = attn_bwd_dkdv_kernel<T, D, DO, NB, NW>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  if (!part) sq = 1;
  FwdSplit qsplit{sq > 1 ? part : nullptr, split_tps(d->seq_len, sq)};
  if (sq > 1) sq = (int)vd_cdiv(vd_cdiv(d->seq_len, kTile), qsplit.tps);
  dim3 grid((unsigned)vd_cdiv(kv.n, 32 * NB * NW), (unsigned)d->nseq, (D / DO) * sq);
  kern<<<grid, 64 * NW, lds, st>>>((const T*)q, (const T*)k, (const T*)v, (const T*)dout, nlse2,
                                   ndelta, (T*)dk, (T*)dv, d->seq_len, qa, d->token_stride, oa,
                                   d->o_token_stride, d->scale, kv, qsplit);
  if (sq > 1) {
    const int rc = vd::check_launch("attn_bwd_dkdv");
    if (rc) return rc;
    const int64_t work = (int64_t)d->nseq * kv.n * (2 * D / 8);
    int g = (int)vd_cdiv(work, 256);
    if (g > 4096) g = 4096;
    attn_dkdv_sum_kernel<T, D><<<g, 256, 0, st>>>(qsplit.part, sq, d->nseq, kv.n, (T*)dk,
                                                  (T*)dv, kv.a, kv.ts);
  }
  return vd::check_launch("attn_bwd_dkdv");
}

template <typename T, int D, int NW, int NB = 1>
int dkdv_pipe_launch(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                     const void* dout, const float* nlse2, const float* ndelta, void* dk, void* dv,
                     hipStream_t st) {
  const SeqAddr qa{d->batch_stride, d->group_stride, d->groups};
  const SeqAddr oa{d->o_batch_stride, d->o_group_stride, d->groups};
  const size_t lds = tile_pipe_lds<D, true, pipe_tr<D, NW>()>();
  auto kern = attn_bwd_dkdv_pipe_kernel<T, D, NW, NB>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  dim3 grid((unsigned)vd_cdiv(d->seq_len, 32 * NB * NW), (unsigned)d->nseq);
  kern<<<grid, 64 * NW, lds, st>>>((const T*)q, (const T*)k, (const T*)v, (const T*)dout, nlse2,
                                   ndelta, (T*)dk, (T*)dv, d->seq_len, qa, d->token_stride, oa,
                                   d->o_token_stride, d->scale);
  return vd::check_launch("attn_bwd_dkdv");
}

template <int D>
int dkdv_pair_launch(const vd_attn_desc* d, KvAddr kv, const void* q, const void* k,
                     const void* v, const void* dout, const float* nlse2, const float* ndelta,
                     void* dk, void* dv, hipStream_t st) {
  const SeqAddr qa{d->batch_stride, d->group_stride, d->groups};
  const SeqAddr oa{d->o_batch_stride, d->o_group_stride, d->groups};
  const size_t lds = (size_t)8 * 32 * D * 2 + tile_loop_lds<bf16_t, D, true, 2>();
  auto kern = attn_bwd_dkdv_pair_kernel<D>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  dim3 grid((unsigned)vd_cdiv(kv.n, 128), (unsigned)d->nseq);
  kern<<<grid, 512, lds, st>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                               (const bf16_t*)dout, nlse2, ndelta, (bf16_t*)dk, (bf16_t*)dv,
                               d->seq_len, qa, d->token_stride, oa, d->o_token_stride, d->scale,
                               kv);
  return vd::check_launch("attn_bwd_dkdv");
}

template <int D, int NW = VD_ROLE_NW>
int dkdv_role_launch(const vd_attn_desc* d, KvAddr kv, const void* q, const void* k,
                     const void* v, const void* dout, const float* nlse2, const float* ndelta,
                     void* dk, void* dv, hipStream_t st, float* part, int sq) {
  const SeqAddr qa{d->batch_stride, d->group_stride, d->groups};
  const SeqAddr oa{d->o_batch_stride, d->o_group_stride, d->groups};
  const size_t lds = tile_loop_lds<bf16_t, D, true>() + (NW / 2) * 1024 * sizeof(float);
  auto kern = attn_bwd_dkdv_role_kernel<D, NW>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  if (!part) sq = 1;
  FwdSplit qsplit{sq > 1 ? part : nullptr, split_tps(d->seq_len, sq)};
  if (sq > 1) sq = (int)vd_cdiv(vd_cdiv(d->seq_len, kTile), qsplit.tps);
  dim3 grid((unsigned)vd_cdiv(kv.n, 16 * NW), (unsigned)d->nseq, (unsigned)sq);
  kern<<<grid, 64 * NW, lds, st>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                               (const bf16_t*)dout, nlse2, ndelta, (bf16_t*)dk, (bf16_t*)dv,
                               d->seq_len, qa, d->token_stride, oa, d->o_token_stride, d->scale,
                               kv, qsplit);
  if (sq > 1) {
    const int rc = vd::check_launch("attn_bwd_dkdv");
    if (rc) return rc;
    const int64_t work = (int64_t)d->nseq * kv.n * (2 * D / 8);
    int g = (int)vd_cdiv(work, 256);
    if (g > 4096) g = 4096;
    attn_dkdv_sum_kernel<bf16_t, D><<<g, 256, 0, st>>>(qsplit.part, sq, d->nseq, kv.n,
                                                       (bf16_t*)dk, (bf16_t*)dv, kv.a, kv.ts);
  }
  return vd::check_launch("attn_bwd_dkdv");
}

template <typename T, int D>
int bwd_dkdv_impl(const vd_attn_desc* d, KvAddr kv, bool cross, const void* q, const void* k,
                  const void* v, const void* dout, const float* lse, void* dk, void* dv,
                  void* ws, hipStream_t st) {
  (void)lse;  // read through the workspace copy written by the dQ pass
  const float* ndelta = reinterpret_cast<const float*>(ws);
  const float* nlse2 = ndelta + (int64_t)d->nseq * d->seq_len;
  if constexpr (kDMA<T>) if (!cross) {
    // (NB = 2 above D = 64 needs > 512 registers; hipcc 7.2 also crashes on it)
    const AttnCfg c = pick_cfg(D, true, 2);
    if constexpr (D <= 64)
      if (c == kNB2) return dkdv_launch<T, D, 2, 4>(d, kv, q, k, v, dout, nlse2, ndelta, dk, dv, st);
    if constexpr (D == 64 || D == 128)
      if (c == kW8) return dkdv_launch<T, D, 1, 8>(d, kv, q, k, v, dout, nlse2, ndelta, dk, dv, st);
    if constexpr (D == 64)
      if (c == kAsm && asm_dq_ok(d, q, k, v, dout, dk) && asm_dq_ok(d, q, k, v, dout, dv))
        return dkdv_asm_launch(d, q, k, v, dout, nlse2, ndelta, dk, dv, st);
    if constexpr (D == 64)
      if (c == kP8 || c == kSP || c == kAsm)
        return dkdv_pipe_launch<T, D, 8>(d, q, k, v, dout, nlse2, ndelta, dk, dv, st);
    if constexpr (D == 64)
      if (c == kP4N2)
        return dkdv_pipe_launch<T, D, 4, 2>(d, q, k, v, dout, nlse2, ndelta, dk, dv, st);
    if constexpr (D <= 128)
      if (c == kP4) return dkdv_pipe_launch<T, D, 4>(d, q, k, v, dout, nlse2, ndelta, dk, dv, st);
    if constexpr (D == 128)
      if (c == kAsm && asm_dq_ok(d, q, k, v, dout, dk, D) && asm_dq_ok(d, q, k, v, dout, dv, D))
        return dkdv_asm_launch(d, q, k, v, dout, nlse2, ndelta, dk, dv, st);
    if constexpr (D == 128)
      if (c == kPair || c == kAsm)
        return dkdv_pair_launch<D>(d, kv, q, k, v, dout, nlse2, ndelta, dk, dv, st);
    if constexpr (D == 256)
      if (c == kAsm && asm_dq_ok(d, q, k, v, dout, dk, D) && asm_dq_ok(d, q, k, v, dout, dv, D)) {
        const BwdWs w = bwd_ws<D>(d, kv.n, cross);
        return dkdv256_asm_launch(d, q, k, v, dout, nlse2, ndelta, dk, dv,
                                  reinterpret_cast<float*>(ws) + w.kv_off, st);
      }
    if constexpr (D == 256)
      if (c == kRole) {
        const BwdWs w = bwd_ws<D>(d, kv.n, cross);
        return dkdv_role_launch<D>(d, kv, q, k, v, dout, nlse2, ndelta, dk, dv, st,
                                   reinterpret_cast<float*>(ws) + w.kv_off, w.sq);
      }
  }
  const BwdWs w = bwd_ws<D>(d, kv.n, cross);
  return dkdv_launch<T, D, 1, 4>(d, kv, q, k, v, dout, nlse2, ndelta, dk, dv, st,
                                 reinterpret_cast<float*>(ws) + w.kv_off, w.sq);
}

#define VD_DISPATCH_HEAD(D_, FN, ...)                        \
  switch (D_) {                                              \
    case 32: return FN<T, 32>(__VA_ARGS__);                  \
    case 64: return FN<T, 64>(__VA_ARGS__);                  \
    case 128: return FN<T, 128>(__VA_ARGS__);                \
    case 256: return FN<T, 256>(__VA_ARGS__);                \
    default: return vd::fail(VD_EUNSUPPORTED, "head_dim");   \
  }

int check_xattn(const vd_xattn_desc* x) {
  VD_REQUIRE(x, "null descriptor");
  int rc = check_attn(&x->q);
  if (rc) return rc;
  VD_REQUIRE(x->kv_len > 0 && x->kv_token_stride > 0, "bad cross-attention K/V shape");
  if (x->q.dtype == VD_BF16)
    VD_REQUIRE(((int64_t)x->kv_len * x->kv_token_stride + x->q.head_dim) * 2 < 0x7fffffffLL,
               "K/V sequence spans >= 2 GiB");
  return VD_OK;
}

KvAddr cross_kv(const vd_xattn_desc* x) {
  return KvAddr{SeqAddr{x->kv_batch_stride, x->kv_group_stride, x->q.groups},
                x->kv_token_stride, x->kv_len};
}

#define VD_DISPATCH_DT(d, FN, ...)                                       \
  do {                                                                   \
    if ((d)->dtype == VD_BF16) {                                         \
      using T = bf16_t;                                                  \
      VD_DISPATCH_HEAD((d)->head_dim, FN, __VA_ARGS__);                  \
    } else if ((d)->dtype == VD_F32) {                                   \
      using T = float;                                                   \
      VD_DISPATCH_HEAD((d)->head_dim, FN, __VA_ARGS__);                  \
    }                                                                    \
    return vd::fail(VD_EUNSUPPORTED, "dtype %d", (d)->dtype);            \
  } while (0)

int fwd_any(const vd_attn_desc* d, KvAddr kv, bool cross, const void* q, const void* k,
            const void* v, void* o, float* lse, void* ws, size_t ws_bytes, hipStream_t st) {
  VD_DISPATCH_DT(d, fwd_impl, d, kv, cross, q, k, v, o, lse, ws, ws_bytes, st);
}
int dq_any(const vd_attn_desc* d, KvAddr kv, bool cross, const void* q, const void* k,
           const void* v, const void* o, const void* dout, const float* lse, void* dq, void* ws,
           hipStream_t st) {
  VD_DISPATCH_DT(d, bwd_dq_impl, d, kv, cross, q, k, v, o, dout, lse, dq, ws, st);
}
int dkdv_any(const vd_attn_desc* d, KvAddr kv, bool cross, const void* q, const void* k,
             const void* v, const void* dout, const float* lse, void* dk, void* dv, void* ws,
             hipStream_t st) {
  VD_DISPATCH_DT(d, bwd_dkdv_impl, d, kv, cross, q, k, v, dout, lse, dk, dv, ws, st);
}
size_t fwd_ws_any(const vd_attn_desc* d, int nkv, bool cross) {
  switch (d->head_dim) {
    case 32: return fwd_ws_bytes<32>(d, nkv, cross);
    case 64: return fwd_ws_bytes<64>(d, nkv, cross);
    case 128: return fwd_ws_bytes<128>(d, nkv, cross);
    case 256: return fwd_ws_bytes<256>(d, nkv, cross);
    default: return 0;
  }
}
size_t bwd_ws_any(const vd_attn_desc* d, int nkv, bool cross) {
  switch (d->head_dim) {
    case 32: return bwd_ws<32>(d, nkv, cross).bytes;
    case 64: return bwd_ws<64>(d, nkv, cross).bytes;
    case 128: return bwd_ws<128>(d, nkv, cross).bytes;
    case 256: return bwd_ws<256>(d, nkv, cross).bytes;
    default: return 0;
  }
}

}  // namespace

namespace vd {
bool short_attn_ok(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                   const void* o);
int short_attn_fwd(const vd_attn_desc* d, const void* q, const void* k, const void* v, void* o,
                   float* lse, hipStream_t st);
int short_attn_bwd(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                   const void* o, const void* dout, const float* lse, void* dq, void* dk,
                   void* dv, hipStream_t st);
}  // namespace vd

namespace {
// the short-sequence kernels (attn_short.hip) for seq_len <= 32; VDIFF_ATTN_SHORT=0 or
// vd_attention_set_short(0) routes those shapes to the flash kernels (A/B, tests)
std::atomic<int> g_short{[] {
  const char* e = std::getenv("VDIFF_ATTN_SHORT");
  return (e && e[0] == '0') ? 0 : 1;
}()};
}  // namespace

extern "C" {

#ifdef VD_ATTN_STAMPS
int vd_debug_attn_stamps(void* dst, size_t bytes) {
  if (bytes > sizeof(g_stamps)) bytes = sizeof(g_stamps);
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamps), bytes, 0, hipMemcpyDeviceToHost) ==
                 hipSuccess
             ? 0
             : 1;
}
#endif

int vd_attention_fwd_ws(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                        void* o, float* lse, void* workspace, size_t workspace_bytes,
                        void* stream) {
  int rc = check_attn(d);
  if (rc) return rc;
  VD_REQUIRE(q && k && v && o && lse, "null tensor");
  if (g_short.load() && vd::short_attn_ok(d, q, k, v, o))
    return vd::short_attn_fwd(d, q, k, v, o, lse, VD_STREAM(stream));
  return fwd_any(d, self_kv(d), false, q, k, v, o, lse, workspace, workspace_bytes,
                 VD_STREAM(stream));
}

int vd_attention_short_path(const vd_attn_desc* d) {
  if (!d || check_attn(d)) return 0;
  static const char kAligned[16] __attribute__((aligned(16))) = {};
  return g_short.load() && vd::short_attn_ok(d, kAligned, kAligned, kAligned, kAligned) ? 1 : 0;
}

// the backward's own decision on the real buffers (advisor r05: a descriptor-only check could
// pick the short kernel for misaligned buffers, which then refused the call)
static bool short_bwd_ok(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                         const void* o, const void* dout, const void* dq, const void* dk,
                         const void* dv) {
  if (!g_short.load() || !d || check_attn(d) || !vd::short_attn_ok(d, q, k, v, o)) return false;
  return ((reinterpret_cast<uintptr_t>(dout) | reinterpret_cast<uintptr_t>(dq) |
           reinterpret_cast<uintptr_t>(dk) | reinterpret_cast<uintptr_t>(dv)) % 16) == 0;
}

int vd_attention_bwd_short_path(const vd_attn_desc* d, const void* q, const void* k,
                                const void* v, const void* o, const void* dout, const void* dq,
                                const void* dk, const void* dv) {
  return short_bwd_ok(d, q, k, v, o, dout, dq, dk, dv) ? 1 : 0;
}

int vd_attention_set_short(int on) { return g_short.exchange(on ? 1 : 0); }

int vd_attention_fwd(const vd_attn_desc* d, const void* q, const void* k, const void* v, void* o,
                     float* lse, void* stream) {
  return vd_attention_fwd_ws(d, q, k, v, o, lse, nullptr, 0, stream);
}

size_t vd_attention_fwd_workspace_size(const vd_attn_desc* d) {
  if (!d || d->nseq <= 0 || d->seq_len <= 0) return 0;
  return fwd_ws_any(d, d->seq_len, false);
}

int vd_attention_set_config(int cfg) {
  if (cfg < -1 || cfg > (int)kCfgLast) {
    (void)vd::fail(VD_EINVAL, "attention config %d", cfg);
    return -2;
  }
  return g_cfg.exchange(cfg);
}

size_t vd_attention_bwd_workspace_size(const vd_attn_desc* d) {
  if (!d || d->nseq <= 0 || d->seq_len <= 0) return 0;
  return bwd_ws_any(d, d->seq_len, false);
}

int vd_attention_bwd_dq(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                        const void* o, const void* dout, const float* lse, void* dq,
                        void* workspace, void* stream) {
  int rc = check_attn(d);
  if (rc) return rc;
  VD_REQUIRE(q && k && v && o && dout && lse && dq && workspace, "null tensor");
  return dq_any(d, self_kv(d), false, q, k, v, o, dout, lse, dq, workspace, VD_STREAM(stream));
}

int vd_attention_bwd_dkdv(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                          const void* dout, const float* lse, void* dk, void* dv, void* workspace,
                          void* stream) {
  int rc = check_attn(d);
  if (rc) return rc;
  VD_REQUIRE(q && k && v && dout && lse && dk && dv && workspace, "null tensor");
  return dkdv_any(d, self_kv(d), false, q, k, v, dout, lse, dk, dv, workspace,
                  VD_STREAM(stream));
}

int vd_attention_bwd(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                     const void* o, const void* dout, const float* lse, void* dq, void* dk,
                     void* dv, void* workspace, void* stream) {
  if (short_bwd_ok(d, q, k, v, o, dout, dq, dk, dv)) {
    VD_REQUIRE(q && k && v && o && dout && lse && dq && dk && dv, "null tensor");
    return vd::short_attn_bwd(d, q, k, v, o, dout, lse, dq, dk, dv, VD_STREAM(stream));
  }
  int rc = vd_attention_bwd_dq(d, q, k, v, o, dout, lse, dq, workspace, stream);
  if (rc) return rc;
  return vd_attention_bwd_dkdv(d, q, k, v, dout, lse, dk, dv, workspace, stream);
}

// ---- cross-attention: queries / output as vd_attn_desc, K/V rows of their own
int vd_cross_attention_fwd(const vd_xattn_desc* x, const void* q, const void* k, const void* v,
                           void* o, float* lse, void* workspace, size_t workspace_bytes,
                           void* stream) {
  int rc = check_xattn(x);
  if (rc) return rc;
  VD_REQUIRE(q && k && v && o && lse, "null tensor");
  return fwd_any(&x->q, cross_kv(x), true, q, k, v, o, lse, workspace, workspace_bytes,
                 VD_STREAM(stream));
}

size_t vd_cross_attention_fwd_workspace_size(const vd_xattn_desc* x) {
  if (check_xattn(x)) return 0;
  return fwd_ws_any(&x->q, x->kv_len, true);
}

size_t vd_cross_attention_bwd_workspace_size(const vd_xattn_desc* x) {
  if (check_xattn(x)) return 0;
  return bwd_ws_any(&x->q, x->kv_len, true);
}

int vd_cross_attention_bwd_dq(const vd_xattn_desc* x, const void* q, const void* k,
                              const void* v, const void* o, const void* dout, const float* lse,
                              void* dq, void* workspace, void* stream) {
  int rc = check_xattn(x);
  if (rc) return rc;
  VD_REQUIRE(q && k && v && o && dout && lse && dq && workspace, "null tensor");
  return dq_any(&x->q, cross_kv(x), true, q, k, v, o, dout, lse, dq, workspace,
                VD_STREAM(stream));
}

int vd_cross_attention_bwd_dkdv(const vd_xattn_desc* x, const void* q, const void* k,
                                const void* v, const void* dout, const float* lse, void* dk,
                                void* dv, void* workspace, void* stream) {
  int rc = check_xattn(x);
  if (rc) return rc;
  VD_REQUIRE(q && k && v && dout && lse && dk && dv && workspace, "null tensor");
  return dkdv_any(&x->q, cross_kv(x), true, q, k, v, dout, lse, dk, dv, workspace,
                  VD_STREAM(stream));
}

}  // extern "C"
