// attn_short.hip -- self-attention over SHORT sequences (seq_len <= 32), bf16: the temporal
// half of the spatial_temporal mode (one sequence per pixel over its T = 16 / 25 frames,
// head_dim 64 / 128 / 256) and the ViViT encoder (9 tokens, head_dim 32).
//
// The flash kernels (attention.hip) tile 32-128 query rows per wave and 64 keys per tile:
// at T = 16 a sequence fills a quarter of a query tile and a quarter of a key tile, so
// they execute 16x the products and stream a whole workgroup for 16 tokens.  Here ONE WAVE
// owns one sequence, padded to Lp = 16 or 32 tokens (executed / algorithmic FLOP = 1 at
// T = 16), with 16x16 MFMA tiles:
//   * forward: S^T = K Q^T (v_mfma_f32_16x16x32_bf16, K and Q row fragments straight from
//     HBM, 16 B per lane), softmax in registers (a query per lane column, its keys in the 4
//     accumulator rows x 4 lane groups), O^T = V^T P^T (v_mfma_f32_16x16x16_bf16) with V^T
//     read from the wave's own LDS copy of the V rows by ds_read_b64_tr_b16;
//   * backward, fused (dQ, dK, dV of the sequence in one wave, no atomics, no partials):
//     S^T and dP^T once (query on the lane column), delta = rowsum(P * dP) from them (no O
//     read),
//     dQ^T = K^T dS^T from registers, dK^T = Q^T dS and dV^T = dO^T P with P and dS turned
//     key-on-lane through LDS; Q / K / dO rows in LDS for the transposed operands: 5
//     products for the 4 algorithmic ones.
// The bytes are the sequence's q | k | v rows in and o (+ lse) out (backward: q, k, v, dO,
// lse in, dq, dk, dv out) -- 8 FLOP per byte at
// T = 16, D = 64: HBM-bound.  The waves of a workgroup take consecutive
// sequences, i.e. neighbouring pixels, whose token rows are adjacent in the channels-last
// qkv buffer.  No barrier: each wave has its own LDS region.
#include "vd_common.h"
#include <math.h>
#include <cstdlib>

namespace {

constexpr float kLog2eS = 1.4426950408889634f;

typedef __attribute__((address_space(3))) bf16x4 lds4_t;

struct ShortArgs {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  const bf16_t* o;      // backward: the forward output (unused: delta from P and dP)
  const bf16_t* dout;   // backward
  bf16_t* out;          // forward: o; backward: dq
  bf16_t* dk;
  bf16_t* dv;
  float* lse;           // [nseq][seq_len], natural log
  int64_t bs, gs, ts;   // q/k/v (and dq/dk/dv) sequence addressing
  int64_t obs, ogs, ots;  // o / dout
  int nseq, seq_len, groups;
  float scale;
};

__device__ __forceinline__ int64_t seq_off(int s, int groups, int64_t bs, int64_t gs) {
  return (int64_t)(s / groups) * bs + (int64_t)(s % groups) * gs;
}

__device__ __forceinline__ bf16x8 ld16(const bf16_t* p, bool ok) {
  return ok ? *reinterpret_cast<const bf16x8*>(p) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
}

__device__ __forceinline__ float bmax4(float x) {  // over the 4 lane groups (lane >> 4)
  x = fmaxf(x, __shfl_xor(x, 16));
  return fmaxf(x, __shfl_xor(x, 32));
}
__device__ __forceinline__ float bsum4(float x) {
  x += __shfl_xor(x, 16);
  return x + __shfl_xor(x, 32);
}

__device__ __forceinline__ bf16x4 pack4(const f32x4& a) {
  const uint32_t lo = pack2bf(a[0], a[1]), hi = pack2bf(a[2], a[3]);
  bf16x4 r;
  r[0] = (short)(lo & 0xffff); r[1] = (short)(lo >> 16);
  r[2] = (short)(hi & 0xffff); r[3] = (short)(hi >> 16);
  return r;
}

// LDS image of one wave's [Lp][D] bf16 rows: row stride D + 8 elements (16 B of padding
// breaks the power-of-two row stride for the transposed reads)
template <int D>
constexpr int kRowS = D + 8;

// the 16x16x16 A operand T^T[d0..d0+15][r0..r0+15] from a row-major tile T[row][d]:
// lane 4q+p of each 16-lane group g supplies row r0 + 4g + q, columns d0 + 4p .. +3, and
// receives column d0 + (lane & 15) of those 4 rows (cdna_hip_programming.md T10)
template <int D>
__device__ __forceinline__ bf16x4 tr_read(const bf16_t* tile, int r0, int d0, int lane) {
  const int g = (lane >> 4) & 3, q = (lane >> 2) & 3, p = lane & 3;
  const bf16_t* a = tile + (r0 + 4 * g + q) * kRowS<D> + d0 + 4 * p;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4_t*)a);
}

// a lane's 16-B row fragment (row r of block, chunk ks) into the LDS image
template <int D>
__device__ __forceinline__ void st_frag(bf16_t* tile, int row, int col, const bf16x8& f) {
  *reinterpret_cast<bf16x8*>(tile + row * kRowS<D> + col) = f;
}

__device__ __forceinline__ void lds_fence() {
  // the wave's own ds_write -> ds_read through LDS: LDS executes a wave's instructions in
  // order; the wait keeps the compiler from moving the reads above the writes' issue
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------- forward
// One wave per sequence: q / k / v fragments straight from HBM into registers (16 B per
// lane), S^T on 16x16 MFMA tiles with the query on the lane column, the softmax in registers,
// V^T through the wave's LDS image by transposed reads, O staged through a second image and
// written as whole rows.  (Two or four sequences per wave with the next one's fragments
// prefetched measured the same: the kernel is store / occupancy bound, not load-latency bound.)
template <int D, int NB>
struct FwdFrags {
  static constexpr int KS = D / 32;
  bf16x8 q[KS][NB], k[KS][NB], v[KS][NB];
};

template <int D, int NB>
__device__ __forceinline__ void fwd_load(const ShortArgs& a, int s, FwdFrags<D, NB>& f, int col,
                                         int grp) {
  const int64_t base = seq_off(s, a.groups, a.bs, a.gs);
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int r = 16 * b + col, c = ks * 32 + 8 * grp;
      const bool ok = r < a.seq_len;
      const int64_t off = base + (int64_t)r * a.ts + c;
      f.q[ks][b] = ld16(a.q + off, ok);
      f.k[ks][b] = ld16(a.k + off, ok);
      f.v[ks][b] = ld16(a.v + off, ok);
    }
}

template <int D, int NB>
__device__ __forceinline__ void fwd_one(const ShortArgs& a, int s, bool live,
                                        const FwdFrags<D, NB>& f, bf16_t* vt, int lane) {
  constexpr int KS = D / 32, DB = D / 16;
  const int L = a.seq_len, col = lane & 15, grp = lane >> 4;
  f32x4 st[NB][NB];  // S^T[kb][qb]: column = query, rows = keys
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) st[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
    for (int b = 0; b < NB; ++b) st_frag<D>(vt, 16 * b + col, ks * 32 + 8 * grp, f.v[ks][b]);
#pragma unroll
    for (int kb = 0; kb < NB; ++kb)
#pragma unroll
      for (int qb = 0; qb < NB; ++qb)
        st[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.k[ks][kb], f.q[ks][qb],
                                                             st[kb][qb], 0, 0, 0);
  }
  const float c2 = a.scale * kLog2eS;
  bf16x4 pb[NB][NB];
  float rl[NB];
#pragma unroll
  for (int qb = 0; qb < NB; ++qb) {
    float m = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = 16 * kb + 4 * grp + i;
        const float x = key < L ? st[kb][qb][i] * c2 : -INFINITY;
        st[kb][qb][i] = x;
        m = fmaxf(m, x);
      }
    m = bmax4(m);
    float l = 0.f;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = exp2f(st[kb][qb][i] - m);  // exp2(-inf) = 0 for masked keys
        st[kb][qb][i] = e;
        l += e;
      }
      pb[kb][qb] = pack4(st[kb][qb]);
    }
    l = bsum4(l);
    rl[qb] = 1.f / l;
    const int qr = 16 * qb + col;
    if (live && grp == 0 && qr < L) a.lse[(int64_t)s * L + qr] = (m + log2f(l)) / kLog2eS;
  }
  lds_fence();
  // O^T (column = query, rows = d 16 db + 4 grp + i) into the wave's [Lp][D + 8] O image,
  // then written out as whole rows: 16 B per lane, a row's D * 2 bytes by consecutive lanes
  // (8-B stores of 4 d each had every lane-group write a quarter of a cache line)
  bf16_t* ot = vt + 16 * NB * kRowS<D>;
#pragma unroll
  for (int db = 0; db < DB; ++db) {
    bf16x4 vtr[NB];
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) vtr[kb] = tr_read<D>(vt, 16 * kb, 16 * db, lane);
#pragma unroll
    for (int qb = 0; qb < NB; ++qb) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < NB; ++kb)
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vtr[kb], pb[kb][qb], acc, 0, 0, 0);
      const uint32_t lo = pack2bf(acc[0] * rl[qb], acc[1] * rl[qb]);
      const uint32_t hi = pack2bf(acc[2] * rl[qb], acc[3] * rl[qb]);
      *reinterpret_cast<uint2*>(ot + (16 * qb + col) * kRowS<D> + 16 * db + 4 * grp) =
          make_uint2(lo, hi);
    }
  }
  lds_fence();
  bf16_t* op = a.out + seq_off(s, a.groups, a.obs, a.ogs);
  constexpr int CPR = D / 8;                      // 16-B chunks per row
#pragma unroll
  for (int k = 0; k < (16 * NB * CPR + 63) / 64; ++k) {
    const int idx = k * 64 + lane, r = idx / CPR, c = (idx % CPR) * 8;
    if (live && r < L && idx < 16 * NB * CPR)
      *reinterpret_cast<bf16x8*>(op + (int64_t)r * a.ots + c) =
          *reinterpret_cast<const bf16x8*>(ot + r * kRowS<D> + c);
  }
}

template <int D, int NB, int WPB>
__global__ void __launch_bounds__(64 * WPB) short_attn_fwd_kernel(ShortArgs a) {
  constexpr int Lp = 16 * NB;
  __shared__ __attribute__((aligned(16))) bf16_t lds[WPB * 2 * Lp * kRowS<D>];  // V | O images
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  bf16_t* vt = lds + w * 2 * Lp * kRowS<D>;
  // every lane of the wave stays in (the transposed read needs EXEC all ones): a wave past
  // the last sequence reads sequence nseq - 1 and stores nothing
  const int s = blockIdx.x * WPB + w;
  const int sc = s < a.nseq ? s : a.nseq - 1;
  FwdFrags<D, NB> f;
  fwd_load<D, NB>(a, sc, f, col, grp);
  fwd_one<D, NB>(a, sc, s < a.nseq, f, vt, lane);
}

// ---------------------------------------------------------------- backward (fused)
// S^T and dP^T once, with the query on the lane column (X orientation): P and
// dS = P (dP - delta) feed dQ^T = K^T dS^T there; for dK^T = Q^T dS and dV^T = dO^T P the
// key must be on the lane column, so P and dS go through the wave's LDS as [query][key]
// bf16 images (one ds_write_b64 per 16x16 block) and come back transposed by
// ds_read_b64_tr_b16.  5 products per sequence: executed / algorithmic = 5 / 4.
template <int L>
constexpr int kPS = L + 8;  // row stride of the [query][key] P / dS images (elements)

template <int D, int NB, int WPB>
__global__ void __launch_bounds__(64 * WPB) short_attn_bwd_kernel(ShortArgs a) {
  constexpr int KS = D / 32, DB = D / 16, Lp = 16 * NB, TS = Lp * kRowS<D>;
  constexpr int PS = Lp * kPS<Lp>, WS = 3 * TS + 2 * PS;
  __shared__ __attribute__((aligned(16))) bf16_t lds[WPB * WS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int s_raw = blockIdx.x * WPB + w;
  const bool live = s_raw < a.nseq;
  const int s = live ? s_raw : a.nseq - 1;
  const int L = a.seq_len, col = lane & 15, grp = lane >> 4;
  bf16_t* qt = lds + w * WS;
  bf16_t* kt = qt + TS;
  bf16_t* dt = kt + TS;
  bf16_t* pimg = dt + TS;
  bf16_t* simg = pimg + PS;
  const int64_t base = seq_off(s, a.groups, a.bs, a.gs);
  const int64_t obase = seq_off(s, a.groups, a.obs, a.ogs);
  const bf16_t *qp = a.q + base, *kp = a.k + base, *vp = a.v + base;
  const bf16_t* dop = a.dout + obase;

  f32x4 sx[NB][NB], px[NB][NB];  // [kb][qb]: column = query, rows = keys
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) sx[i][j] = px[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int c = ks * 32 + 8 * grp;
    bf16x8 qf[NB], kf[NB], vf[NB], df[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int r = 16 * b + col;
      const bool ok = r < L;
      qf[b] = ld16(qp + (int64_t)r * a.ts + c, ok);
      kf[b] = ld16(kp + (int64_t)r * a.ts + c, ok);
      vf[b] = ld16(vp + (int64_t)r * a.ts + c, ok);
      df[b] = ld16(dop + (int64_t)r * a.ots + c, ok);
      st_frag<D>(qt, r, c, qf[b]);
      st_frag<D>(kt, r, c, kf[b]);
      st_frag<D>(dt, r, c, df[b]);
    }
#pragma unroll
    for (int kb = 0; kb < NB; ++kb)
#pragma unroll
      for (int qb = 0; qb < NB; ++qb) {
        sx[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kb], qf[qb], sx[kb][qb], 0, 0, 0);
        px[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[kb], df[qb], px[kb][qb], 0, 0, 0);
      }
  }
  const float c2 = a.scale * kLog2eS;
  bf16x4 dsx[NB][NB];
#pragma unroll
  for (int qb = 0; qb < NB; ++qb) {
    const int qr = 16 * qb + col;
    const float lse2 = qr < L ? a.lse[(int64_t)s * L + qr] * kLog2eS : 0.f;
    // P of the query's whole row (all its keys are in this wave), then the softmax backward
    // dS = P (dP - rowsum(P dP)) -- the reference's autograd of softmax -- so the backward
    // never reads O (FA's rowsum(dO O) is the same sum when O = P V)
    f32x4 pr[NB];
    float del = 0.f;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = 16 * kb + 4 * grp + i;
        pr[kb][i] = (key < L && qr < L) ? exp2f(sx[kb][qb][i] * c2 - lse2) : 0.f;
        del = fmaf(pr[kb][i], px[kb][qb][i], del);
      }
    del = bsum4(del);
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      const f32x4 p = pr[kb];
      f32x4 d;
#pragma unroll
      for (int i = 0; i < 4; ++i) d[i] = p[i] * (px[kb][qb][i] - del);
      const bf16x4 pb = pack4(p);
      dsx[kb][qb] = pack4(d);
      // [query][key] images: this lane's 4 keys are 4 consecutive elements of row qr
      *reinterpret_cast<bf16x4*>(pimg + qr * kPS<Lp> + 16 * kb + 4 * grp) = pb;
      *reinterpret_cast<bf16x4*>(simg + qr * kPS<Lp> + 16 * kb + 4 * grp) = dsx[kb][qb];
    }
  }
  lds_fence();
  // the key-on-lane operands P[qb][kb], dS[qb][kb]: B[k = query 4 grp + j][n = key col]
  bf16x4 pyb[NB][NB], dsy[NB][NB];
#pragma unroll
  for (int qb = 0; qb < NB; ++qb)
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
      pyb[qb][kb] = tr_read<Lp>(pimg, 16 * qb, 16 * kb, lane);
      dsy[qb][kb] = tr_read<Lp>(simg, 16 * qb, 16 * kb, lane);
    }
  bf16_t* dqp = a.out + base;
  bf16_t* dkp = a.dk + base;
  bf16_t* dvp = a.dv + base;
  // STAGE: the packed outputs are kept in registers and, once every transposed read is done,
  // written through the Q / K / dO images as whole rows (16 B per lane; 8-B stores of 4 d
  // each write a quarter of a cache line per lane group).  Larger D * NB stores directly.
  constexpr bool STAGE = 3 * DB * NB * 2 <= 96;
  uint2 outq[STAGE ? DB : 1][NB], outk[STAGE ? DB : 1][NB], outv[STAGE ? DB : 1][NB];
#pragma unroll
  for (int db = 0; db < DB; ++db) {
    bf16x4 qtr[NB], ktr[NB], dtr[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      qtr[b] = tr_read<D>(qt, 16 * b, 16 * db, lane);
      ktr[b] = tr_read<D>(kt, 16 * b, 16 * db, lane);
      dtr[b] = tr_read<D>(dt, 16 * b, 16 * db, lane);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      // dQ^T[db][qb = b] = sum_kb K^T[db][kb] dS^T[kb][qb];  column = query
      // dK^T[db][kb = b] = sum_qb Q^T[db][qb] dS[qb][kb];    column = key
      // dV^T[db][kb = b] = sum_qb dO^T[db][qb] P[qb][kb];    column = key
      f32x4 aq = f32x4{0.f, 0.f, 0.f, 0.f}, ak = aq, av = aq;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        aq = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ktr[j], dsx[j][b], aq, 0, 0, 0);
        ak = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(qtr[j], dsy[j][b], ak, 0, 0, 0);
        av = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(dtr[j], pyb[j][b], av, 0, 0, 0);
      }
      const uint2 vq = make_uint2(pack2bf(aq[0] * a.scale, aq[1] * a.scale),
                                  pack2bf(aq[2] * a.scale, aq[3] * a.scale));
      const uint2 vk = make_uint2(pack2bf(ak[0] * a.scale, ak[1] * a.scale),
                                  pack2bf(ak[2] * a.scale, ak[3] * a.scale));
      const uint2 vv = make_uint2(pack2bf(av[0], av[1]), pack2bf(av[2], av[3]));
      if constexpr (STAGE) {
        outq[db][b] = vq;
        outk[db][b] = vk;
        outv[db][b] = vv;
      } else {
        const int r = 16 * b + col;
        if (live && r < L) {
          const int64_t off = (int64_t)r * a.ts + 16 * db + 4 * grp;
          *reinterpret_cast<uint2*>(dqp + off) = vq;
          *reinterpret_cast<uint2*>(dkp + off) = vk;
          *reinterpret_cast<uint2*>(dvp + off) = vv;
        }
      }
    }
  }
  if constexpr (STAGE) {
    lds_fence();  // every transposed read of the images has returned
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int o = (16 * b + col) * kRowS<D> + 16 * db + 4 * grp;
        *reinterpret_cast<uint2*>(qt + o) = outq[db][b];
        *reinterpret_cast<uint2*>(kt + o) = outk[db][b];
        *reinterpret_cast<uint2*>(dt + o) = outv[db][b];
      }
    lds_fence();
    constexpr int CPR = D / 8;  // 16-B chunks per row
#pragma unroll
    for (int k = 0; k < (16 * NB * CPR + 63) / 64; ++k) {
      const int idx = k * 64 + lane, r = idx / CPR, c = (idx % CPR) * 8;
      if (live && r < L && idx < 16 * NB * CPR) {
        const int64_t off = (int64_t)r * a.ts + c;
        *reinterpret_cast<bf16x8*>(dqp + off) =
            *reinterpret_cast<const bf16x8*>(qt + r * kRowS<D> + c);
        *reinterpret_cast<bf16x8*>(dkp + off) =
            *reinterpret_cast<const bf16x8*>(kt + r * kRowS<D> + c);
        *reinterpret_cast<bf16x8*>(dvp + off) =
            *reinterpret_cast<const bf16x8*>(dt + r * kRowS<D> + c);
      }
    }
  }
}

// waves (= sequences) per workgroup: 4, or fewer where the static LDS would pass 64 KiB
template <int D, int NB, int TILES>
constexpr int wpb() {
  // TILES [Lp][D + 8] row images, plus (backward) the two [Lp][Lp + 8] P / dS images
  constexpr int per_wave = TILES * 16 * NB * kRowS<D> * 2 +
                           (TILES == 3 ? 2 * 16 * NB * (16 * NB + 8) * 2 : 0);
  return 4 * per_wave <= 65536 ? 4 : 2 * per_wave <= 65536 ? 2 : 1;
}

template <int D, int NB>
int launch_fwd(const ShortArgs& a, hipStream_t st) {
  constexpr int W = wpb<D, NB, 2>();  // V and O images
  short_attn_fwd_kernel<D, NB, W><<<(a.nseq + W - 1) / W, 64 * W, 0, st>>>(a);
  return vd::check_launch("short_attn_fwd");
}
template <int D, int NB>
int launch_bwd(const ShortArgs& a, hipStream_t st) {
  constexpr int W = wpb<D, NB, 3>();  // Q, K, dO images
  short_attn_bwd_kernel<D, NB, W><<<(a.nseq + W - 1) / W, 64 * W, 0, st>>>(a);
  return vd::check_launch("short_attn_bwd");
}

ShortArgs make_args(const vd_attn_desc* d) {
  ShortArgs a{};
  a.bs = d->batch_stride; a.gs = d->group_stride; a.ts = d->token_stride;
  a.obs = d->o_batch_stride; a.ogs = d->o_group_stride; a.ots = d->o_token_stride;
  a.nseq = d->nseq; a.seq_len = d->seq_len; a.groups = d->groups; a.scale = d->scale;
  return a;
}

#define VD_SHORT_DISPATCH(FN, d, ...)                                               \
  do {                                                                             \
    const int nb = (d)->seq_len <= 16 ? 1 : 2;                                     \
    switch ((d)->head_dim * 4 + nb) {                                              \
      case 32 * 4 + 1: return FN<32, 1>(__VA_ARGS__);                              \
      case 32 * 4 + 2: return FN<32, 2>(__VA_ARGS__);                              \
      case 64 * 4 + 1: return FN<64, 1>(__VA_ARGS__);                              \
      case 64 * 4 + 2: return FN<64, 2>(__VA_ARGS__);                              \
      case 128 * 4 + 1: return FN<128, 1>(__VA_ARGS__);                            \
      case 128 * 4 + 2: return FN<128, 2>(__VA_ARGS__);                            \
      case 256 * 4 + 1: return FN<256, 1>(__VA_ARGS__);                            \
      case 256 * 4 + 2: return FN<256, 2>(__VA_ARGS__);                            \
      default: return vd::fail(VD_EUNSUPPORTED, "short attention head_dim %d",     \
                               (d)->head_dim);                                     \
    }                                                                              \
  } while (0)

bool aligned16(int64_t elems) { return elems % 8 == 0; }

}  // namespace

namespace vd {

// the short-sequence kernels serve bf16 sequences of <= 32 tokens with 16-B aligned rows
bool short_attn_ok(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                   const void* o) {
  if (d->dtype != VD_BF16 || d->seq_len > 32) return false;
  if (!(d->head_dim == 32 || d->head_dim == 64 || d->head_dim == 128 || d->head_dim == 256))
    return false;
  if (!aligned16(d->batch_stride) || !aligned16(d->group_stride) || !aligned16(d->token_stride) ||
      !aligned16(d->o_batch_stride) || !aligned16(d->o_group_stride) ||
      !aligned16(d->o_token_stride))
    return false;
  const uintptr_t m = reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
                      reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(o);
  return m % 16 == 0;
}

int short_attn_fwd(const vd_attn_desc* d, const void* q, const void* k, const void* v, void* o,
                   float* lse, hipStream_t st) {
  ShortArgs a = make_args(d);
  a.q = static_cast<const bf16_t*>(q);
  a.k = static_cast<const bf16_t*>(k);
  a.v = static_cast<const bf16_t*>(v);
  a.out = static_cast<bf16_t*>(o);
  a.lse = lse;
  VD_SHORT_DISPATCH(launch_fwd, d, a, st);
}

int short_attn_bwd(const vd_attn_desc* d, const void* q, const void* k, const void* v,
                   const void* o, const void* dout, const float* lse, void* dq, void* dk,
                   void* dv, hipStream_t st) {
  VD_REQUIRE((reinterpret_cast<uintptr_t>(dout) | reinterpret_cast<uintptr_t>(dq) |
              reinterpret_cast<uintptr_t>(dk) | reinterpret_cast<uintptr_t>(dv)) % 16 == 0,
             "short attention backward: buffers must be 16-B aligned");
  ShortArgs a = make_args(d);
  a.q = static_cast<const bf16_t*>(q);
  a.k = static_cast<const bf16_t*>(k);
  a.v = static_cast<const bf16_t*>(v);
  a.o = static_cast<const bf16_t*>(o);
  a.dout = static_cast<const bf16_t*>(dout);
  a.out = static_cast<bf16_t*>(dq);
  a.dk = static_cast<bf16_t*>(dk);
  a.dv = static_cast<bf16_t*>(dv);
  a.lse = const_cast<float*>(lse);
  VD_SHORT_DISPATCH(launch_bwd, d, a, st);
}

}  // namespace vd
