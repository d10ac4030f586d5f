// Micro-benchmark: cycles per loop iteration of an attention-like instruction mix on one
// SIMD (gfx950).  V=0: 8 MFMA 32x32x16 bf16 only.  V=1: + 16 v_exp + 16 adds + 8 cvt_pk on
// independent registers.  V=2: the exp inputs are the previous iteration's MFMA results
// (the flash-attention dependency: S(b) -> softmax(b) while S(b+1), PV(b-1) run).
// Usage: ./mfma_valu  (prints cycles/iteration for 1 and 2 waves per SIMD)
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int V>
__global__ __launch_bounds__(512, 1) void kern(float* out, long long* cyc, int iters, float seed) {
  const int lane = threadIdx.x & 63;
  bf16x8 a0, a1, b0, b1;
  for (int i = 0; i < 8; ++i) {
    a0[i] = (short)(lane * 3 + i); a1[i] = (short)(lane * 5 + i);
    b0[i] = (short)(lane * 7 + i); b1[i] = (short)(lane * 11 + i);
  }
  f32x16 s0 = {}, s1 = {}, o0 = {}, o1 = {}, x;
  for (int r = 0; r < 16; ++r) x[r] = seed * (r + lane);
  float psum = 0.f;
  uint32_t pk[8] = {};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    f32x16 sn = -x;  // "negm" init
    sn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, sn, 0, 0, 0);
    sn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, sn, 0, 0, 0);
    sn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, sn, 0, 0, 0);
    sn = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, sn, 0, 0, 0);
    o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, o0, 0, 0, 0);
    o0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, o0, 0, 0, 0);
    o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, o1, 0, 0, 0);
    o1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, o1, 0, 0, 0);
    if constexpr (V >= 1) {
      f32x16& src = (V == 2 || V == 4) ? s0 : x;
      f32x16 p;
      for (int r = 0; r < 16; ++r) {
        p[r] = __builtin_amdgcn_exp2f(src[r]);
        psum += p[r];
      }
      for (int r = 0; r < 8; ++r) {
        uint32_t w;
        asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(w) : "v"(p[2 * r]), "v"(p[2 * r + 1]));
        pk[r] ^= w;
      }
      if constexpr (V == 1) x[0] += 1e-7f;
    }
    if constexpr (V >= 3) {
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, V == 3 ? 5 : 6, 0);
      }
    }
    s0 = sn;
    b0[0] ^= (short)pk[it & 7];
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float acc = psum;
  for (int r = 0; r < 16; ++r) acc += s0[r] + o0[r] + o1[r];
  for (int r = 0; r < 8; ++r) acc += (float)pk[r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
void run(int threads) {
  const int blocks = 256, iters = 20000;
  float* out; long long* cyc;
  hipMalloc(&out, blocks * threads * 4);
  hipMalloc(&cyc, blocks * 8);
  kern<V><<<blocks, threads>>>(out, cyc, 100, 0.001f);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  kern<V><<<blocks, threads>>>(out, cyc, iters, 0.001f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  long long h[256];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  long long med = h[128];
  printf("V=%d waves/SIMD=%d: %.1f cycles/iter (s_memtime), %.3f ms, %.1f MFMA-util%% at 2.4GHz\n",
         V, threads / 256, (double)med / iters, ms,
         100.0 * 8 * 32 * (threads / 256) * iters / (ms * 1e-3 * 2.4e9));
  hipFree(out); hipFree(cyc);
}
int main() {
  for (int t : {256, 512}) { run<0>(t); run<1>(t); run<2>(t); run<3>(t); run<4>(t); }
  return 0;
}
