// Shared helpers for the V-JEPA 2 gfx950 kernel library (libvjepa_hip.so).
// CDNA4 only: wave64, MFMA bf16, LDS-DMA (buffer_load ... lds), ds_read_b64_tr_b16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef unsigned short bf16_t;  // storage type of a bf16 element in global memory

#define LDS_AS __attribute__((address_space(3)))

// ----- error reporting (C ABI: every entry point returns 0 or a VJ_ERR_* code) -----
enum {
  VJ_OK = 0,
  VJ_ERR_ARG = 1,       // bad argument (shape / null pointer / alignment)
  VJ_ERR_LAUNCH = 2,    // hipGetLastError after a launch
  VJ_ERR_UNSUPPORTED = 3,
};

void vj_set_error(const char* fmt, ...);

#define VJ_CHECK_ARG(cond, ...)          \
  do {                                   \
    if (!(cond)) {                       \
      vj_set_error(__VA_ARGS__);         \
      return VJ_ERR_ARG;                 \
    }                                    \
  } while (0)

#define VJ_LAUNCH_CHECK(what)                                                    \
  do {                                                                           \
    hipError_t e_ = hipGetLastError();                                           \
    if (e_ != hipSuccess) {                                                      \
      vj_set_error("%s: launch failed: %s", what, hipGetErrorString(e_));        \
      return VJ_ERR_LAUNCH;                                                      \
    }                                                                            \
  } while (0)

// ----- bf16 <-> f32 (round-to-nearest-even; NaN-preserving via the hardware cvt) -----
__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32 on gfx950
  return __builtin_bit_cast(bf16_t, b);
}
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// ----- wave reductions (64 lanes) -----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ----- buffer resource (SRD) for LDS-DMA loads with hardware range check -----
// Buffer descriptor for a wave-uniform base/size. The values are forced into SGPRs: if the compiler
// cannot prove uniformity it would wrap every buffer instruction in a readfirstlane waterfall loop.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  const unsigned long long a = (unsigned long long)base;
  const unsigned long long lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)a);
  const unsigned long long hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(lo | (hi << 32)), (short)0, n, 0x00020000);
}
// 16 bytes per lane, global(rsrc + voffset) -> LDS(lds_wave_base + lane*16). Out-of-range -> zeros.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, LDS_AS void* lds_wave_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, lds_wave_base, 16, voff, 0, 0, 0);
}
#define VJ_OOB 0x80000000u

__device__ __forceinline__ s16x4 ds_read_tr16(const LDS_AS void* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)p);
}
// The same read as inline asm. The compiler's wait-count pass treats the builtin as a possible
// reader of in-flight LDS-DMA data and puts an s_waitcnt vmcnt(0) before it, which serialises the
// next tile's DMA with the current tile's reads. The asm form is invisible to that pass: its result
// must be released with lds_wait() + tie() before use.
__device__ __forceinline__ s16x4 ds_read_tr16_async(const LDS_AS void* p) {
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"((uint32_t)(uintptr_t)p) : "memory");
  return r;
}
__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// Orders every later use of x after the preceding lds_wait() (volatile asm keeps program order).
template <typename T, int N>
__device__ __forceinline__ void tie(T (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(x[i]));
}

// 4 f32 -> 4 fp8 e4m3 (OCP, RNE), clamped to the format's +-448 (e4m3fn has no infinity)
__device__ __forceinline__ uint32_t f8pack4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(a, -448.f, 448.f),
                                          __builtin_amdgcn_fmed3f(b, -448.f, 448.f), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(c, -448.f, 448.f),
                                      __builtin_amdgcn_fmed3f(d, -448.f, 448.f), w, true);
  return (uint32_t)w;
}

static inline int vj_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// nn.GELU() (exact erf form, vision_transformer.py:100) and its derivative in one pass (the erf
// and Gaussian terms are shared). erf by Abramowitz-Stegun 7.1.26, |abs err| <= 1.5e-7: far below
// the bf16 rounding of the outputs.
// The argument is pre-scaled by sqrt(log2 e) (zs = z sqrt(log2 e), the A-S constant divided by the
// same) so the Gaussian is one v_exp_f32 (exp2) of -zs^2 with no extra multiply, and the CDF is one
// fma: 14 -> 12 VALU per element besides the two transcendentals.
__device__ __forceinline__ void gelu_fwd_grad(float x, float& y, float& dy) {
  const float zs = x * 0.84932180028801904f;  // x / sqrt(2) * sqrt(log2 e)
  const float a = fabsf(zs);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.27273748087922250f, a, 1.f));  // 0.3275911 / sqrt(log2 e)
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-zs * zs);  // exp(-x^2 / 2)
  const float cdf = fmaf(0.5f, copysignf(fmaf(-p, e, 1.f), zs), 0.5f);
  y = x * cdf;
  dy = fmaf(x * 0.39894228040143268f, e, cdf);
}

// 3-axis RoPE applied to the q and k columns of a fused QKV projection (modules.py:26-50, 343-365),
// as a GEMM epilogue argument
struct VjRope {
  const int* ids;   // token id per row (NULL -> row % mod)
  int mod, tpf, tpr;
  int half, hd, D;  // half = slice/2, head dim, q/k block width (= H * hd)
  const float* cos_t;
  const float* sin_t;
  int npos;         // table rows (positions); every position of every id is < npos
};

__device__ __forceinline__ uint32_t clamp_u31(long b) {
  if (b < 0) return 0;
  return b > 0x7fffffffL ? 0x7fffffffu : (uint32_t)b;
}
