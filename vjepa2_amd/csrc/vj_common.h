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
// Two values -> one packed bf16 pair with ONE v_cvt_pk_bf16_f32 (the same RNE conversion as f2bf; the
// scalar form compiled to two conversions + a shift + an or_sdwa per pair)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2_t));
}

// ----- cross-lane exchanges on the VALU (DPP / gfx950 permlane swaps) -----
// __shfl_xor compiles to ds_bpermute_b32, an LDS-unit round trip (~100+ cycles) per step; these stay
// in the vector ALU. Each pairs lane l with a partner and both lanes compute the same commutative
// op, so every lane ends with the bitwise-identical result.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
constexpr int DPP_XOR1 = 0xB1;        // quad_perm [1, 0, 3, 2]: lane l <-> l ^ 1
constexpr int DPP_XOR2 = 0x4E;        // quad_perm [2, 3, 0, 1]: lane l <-> l ^ 2
constexpr int DPP_HALF_MIRROR = 0x141;  // within 8 lanes: i <-> 7 - i
constexpr int DPP_MIRROR = 0x140;       // within 16 lanes: i <-> 15 - i
// (own, partner) pairs: lane l <-> l ^ 16 / l ^ 32 (v_permlane16_swap / v_permlane32_swap)
__device__ __forceinline__ float sum_xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float sum_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float max_xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float max_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// ----- wave reductions (64 lanes; every lane gets the total) -----
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp<DPP_XOR1>(v);         // pairs
  v += dpp<DPP_XOR2>(v);         // quads
  v += dpp<DPP_HALF_MIRROR>(v);  // 8 lanes: quad sums of both halves
  v += dpp<DPP_MIRROR>(v);       // 16 lanes
  v = sum_xor16(v);              // 32
  return sum_xor32(v);           // 64
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp<DPP_XOR1>(v));
  v = fmaxf(v, dpp<DPP_XOR2>(v));
  v = fmaxf(v, dpp<DPP_HALF_MIRROR>(v));
  v = fmaxf(v, dpp<DPP_MIRROR>(v));
  v = max_xor16(v);
  return max_xor32(v);
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
// Timing-only diagnostic macros (VJ_DIAG_*: loads skipped or misplaced, WRONG results) exist for
// variant libraries only (python -m vjepa2_amd.build --variant NAME -DVJ_DIAG_...), never libvjepa_hip.so.
#if !defined(VJ_VARIANT_BUILD) && (defined(VJ_DIAG_NODMA) || defined(VJ_DIAG_NOWAIT) || defined(VJ_DIAG_SAMEADDR) || \
                                   defined(VJ_DIAG_FULL128))
#error "VJ_DIAG_* macros are for variant builds only"
#endif
#ifndef VJ_DMA_CPOL
#define VJ_DMA_CPOL 0
#endif
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, LDS_AS void* lds_wave_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, lds_wave_base, 16, voff, 0, 0, VJ_DMA_CPOL);
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

// GEMM epilogues: ONE numbering for every GEMM source (vj_gemm.hip, vj_gemm256.hip, vj_gemm_pp.hip,
// vj_f32.hip) and the public header (include/vjepa_hip.h VJ_EPI_*). EPI_PARTIAL is internal (split-K
// f32 partial slabs), and so is EPI_PARTIAL_RS (the same with A's row sums per K slice: the fused
// bias gradient of vj_gemm_bf16_wgrad); EPI_BF16_RESID: bf16 residual in (aux), bf16 out.
enum { EPI_BF16 = 0, EPI_F32 = 1, EPI_F32_RESID = 2, EPI_GELU = 3, EPI_GELU_BWD = 4, EPI_ROPE = 5, EPI_PARTIAL = 6,
       EPI_BF16_RESID = 7, EPI_PARTIAL_RS = 8 };

static inline int vj_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// nn.GELU() (exact erf form, vision_transformer.py:100) and its derivative in one pass (the erf
// and Gaussian terms are shared). erf by Abramowitz-Stegun 7.1.26, |abs err| <= 1.5e-7: far below
// the bf16 rounding of the outputs.
// The argument is pre-scaled by sqrt(log2 e) (zs = z sqrt(log2 e), the A-S constant divided by the
// same) so the Gaussian is one v_exp_f32 (exp2) of -zs^2 with no extra multiply, and the CDF is one
// fma: 14 -> 12 VALU per element besides the two transcendentals.
// gelu_cdf_grad gives the multiplier cdf = Phi(x) (GELU(x) = x * cdf, exactly as below) and GELU'(x);
// the GEMM's table epilogue (vj_gemm_tile.h) stores these two per bf16 input, so its y = x * cdf is the
// same f32 operation on the same operands as here.
__device__ __forceinline__ void gelu_cdf_grad(float x, float& cdf, float& dy) {
  const float zs = x * 0.84932180028801904f;  // x / sqrt(2) * sqrt(log2 e)
  const float a = fabsf(zs);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.27273748087922250f, a, 1.f));  // 0.3275911 / sqrt(log2 e)
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-zs * zs);  // exp(-x^2 / 2)
  cdf = fmaf(0.5f, copysignf(fmaf(-p, e, 1.f), zs), 0.5f);
  dy = fmaf(x * 0.39894228040143268f, e, cdf);
}
__device__ __forceinline__ void gelu_fwd_grad(float x, float& y, float& dy) {
  float cdf;
  gelu_cdf_grad(x, cdf, dy);
  y = x * cdf;
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

// ----- dropout keep masks (nn.Dropout / F.scaled_dot_product_attention dropout_p, modules.py:75-82,
// 246, 257, 370, 381): a counter-based hash of (seed, row, column), so the backward regenerates the
// forward's mask from the seed alone. Element (row r, column c) of a call with seed s is kept iff
// drop_u(drop_row(s, r), c) >= thresh, thresh = round(p * 2^32); kept values are scaled by 1 / (1 - p).
// Rows: the token row of an activation, or token * H + head of an attention score row (query token);
// columns: the feature, or the key's index in its sequence. Restated for the tests in
// tests/test_dropout.py (vj_dropout_mask_ref).
__device__ __forceinline__ uint32_t drop_mix(uint32_t x) {  // "lowbias32" integer hash
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t drop_row(uint32_t seed, uint32_t row) { return drop_mix(seed ^ (row * 0x9e3779b1u)); }
__device__ __forceinline__ uint32_t drop_u(uint32_t rowkey, uint32_t col) { return drop_mix(rowkey + col * 0x85ebca77u); }
uint32_t vj_drop_thresh(float p);  // round(p * 2^32), saturated (vj_variants.hip)
