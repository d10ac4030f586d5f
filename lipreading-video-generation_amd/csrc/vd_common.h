// vd_common.h -- shared device/host helpers for libvdiff (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include "../../include/vdiff.h"

// ---------------------------------------------------------------- errors
namespace vd {
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);
int check_launch(const char* what);
}  // namespace vd

#define VD_REQUIRE(cond, ...)                                   \
  do {                                                          \
    if (!(cond)) return vd::fail(VD_EINVAL, __VA_ARGS__);       \
  } while (0)

#define VD_STREAM(s) (reinterpret_cast<hipStream_t>(s))

// ---------------------------------------------------------------- types
typedef uint16_t bf16_t;  // raw bf16 storage
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}
// fp32 -> bf16, round-to-nearest-even, NaN stays NaN: one v_cvt_pk_bf16_f32 on gfx950
// (an integer-arithmetic rounding with a NaN test compiles to a divergent branch per
// element).
typedef __bf16 bf16x2_hw __attribute__((ext_vector_type(2)));
typedef float f32x2_hw __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_hw){a, b}, bf16x2_hw));
}

// Load/store N consecutive elements of T as fp32 (N*sizeof(T) must be 8 or 16 B aligned).
template <typename T> struct Elem;
template <> struct Elem<float> {
  static constexpr int kDtype = VD_F32;
  __device__ __forceinline__ static float ld(const float* p) { return *p; }
  __device__ __forceinline__ static void st(float* p, float v) { *p = v; }
};
template <> struct Elem<bf16_t> {
  static constexpr int kDtype = VD_BF16;
  __device__ __forceinline__ static float ld(const bf16_t* p) { return bf2f(*p); }
  __device__ __forceinline__ static void st(bf16_t* p, float v) { *p = f2bf(v); }
};

// 8 elements <-> 8 floats, vectorised (bf16: one 16-B access, f32: two).
__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void load8(const bf16_t* p, float (&v)[8]) {
  uint4 r = *reinterpret_cast<const uint4*>(p);
  uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void store8(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void store8(bf16_t* p, const float (&v)[8]) {
  *reinterpret_cast<uint4*>(p) = make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]),
                                            pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
}

// counter-based dropout keep mask (splitmix64 of seed + idx); returns 0 or 1/(1-p)
__device__ __forceinline__ float dropout_mul(uint64_t seed, int64_t idx, float p, float inv_keep) {
  uint64_t z = seed + (uint64_t)idx * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const float u = (float)(uint32_t)(z >> 40) * (1.0f / 16777216.0f);
  return u >= p ? inv_keep : 0.f;
}

__device__ __forceinline__ float silu_f(float z) { return z / (1.0f + __expf(-z)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// dispatch on the runtime dtype tag
#define VD_DISPATCH_DTYPE(dtype, T, ...)                               \
  [&]() -> int {                                                       \
    if ((dtype) == VD_F32) { using T = float; __VA_ARGS__; }           \
    else if ((dtype) == VD_BF16) { using T = bf16_t; __VA_ARGS__; }    \
    else return vd::fail(VD_EUNSUPPORTED, "unknown dtype %d", (int)(dtype)); \
    return vd::check_launch(__func__);                                 \
  }()

static inline int64_t vd_cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------- LDS-DMA (buffer_load ... lds)
// shared by the attention ring and the conv GEMM
typedef __attribute__((address_space(3))) void lds_void;
// Buffer resource words: base, stride 0, num_records = bytes (the range check zero-fills
// beyond it), raw dword format.
typedef int __attribute__((ext_vector_type(4))) rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  return rsrc_t{(int)(uint32_t)a, (int)(uint32_t)((a >> 32) & 0xffff), (int)bytes, 0x00020000};
}
__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return (uint32_t)(uintptr_t)(const lds_void*)p;
}

// The LDS-DMA is issued from inline asm on purpose: the compiler's waitcnt pass cannot tell
// which LDS bytes a builtin buffer_load...lds writes, so it put an s_waitcnt vmcnt(0) in
// front of the first LDS read after it -- draining the whole ring every tile.  The ring's
// own counted vmcnt + s_barrier (vm_wait_barrier) is what orders these writes.
// M0 (the LDS destination) is an input operand bound with the "{m0}" constraint: the
// compiler itself writes M0 and knows this statement reads it, so it never keeps a value
// of its own there across the DMA.
template <int BYTES>
__device__ __forceinline__ void dma_lds(rsrc_t rs, uint32_t lds, uint32_t voff) {
  if constexpr (BYTES == 16)
    asm volatile("buffer_load_dwordx4 %1, %2, 0 offen lds"
                 ::"{m0}"(lds), "v"(voff), "s"(rs));
  else
    asm volatile("buffer_load_dword %1, %2, 0 offen lds"
                 ::"{m0}"(lds), "v"(voff), "s"(rs));
}

template <int N>
__device__ __forceinline__ void vm_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}
// the same, after every LDS read of this wave has returned: the compiler may schedule the MFMAs
// that consume earlier ds_reads (and so its own lgkmcnt waits) after an asm barrier, which would
// leave a read of a stage in flight while another wave's DMA refills it
template <int N>
__device__ __forceinline__ void vm_lgk_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lgk_wait_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// compiler-visible (the waitcnt pass then knows every earlier global load has landed and
// puts no waits of its own inside the ring loop); 0x0F70 = vmcnt(0), expcnt/lgkmcnt untouched
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

