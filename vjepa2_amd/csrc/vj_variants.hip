// Block variants the shipped V-JEPA 2 configs leave off, on the same token-major layout as the fused
// block (functions.block_forward / block_backward):
//  * the SwiGLU gate of SwiGLUFFN (src/models/utils/modules.py:86-106, act_layer=nn.SiLU): the fc1 / fc2
//    GEMMs write x1 | x2 side by side ([M, 2h] bf16), one pass makes hidden = silu(x1) * x2 and one
//    pass its gradients (dx1 | dx2, again side by side: the two weight-gradient GEMMs read halves);
//  * stochastic depth (timm drop_path via DropPath, modules.py:53-64, applied at :561-562): a
//    per-sample factor (0 or 1 / keep) on the branch output before the residual add, and on the
//    branch's output gradient in the backward;
//  * dropout (nn.Dropout: MLP.drop after the activation and after fc2, modules.py:75-82; proj_drop
//    after the attention projection, :257 / :381): the element mask of vj_common.h's drop_row /
//    drop_u, so the backward (the same mask times the incoming gradient) needs only the seed.
// Rounding follows the reference under bf16 autocast (app/vjepa/train.py:438): every intermediate
// the reference materialises in bf16 is rounded to bf16 here at the same point; the arithmetic
// between roundings is f32, as in PyTorch's elementwise kernels (opmath = float).
// All passes are HBM-bound streams of 16-B (bf16 x 8) or float4 (f32 x 4) chunks.
#include "vj_common.h"

namespace {

__device__ __forceinline__ float bfr(float x) { return bf2f(f2bf(x)); }  // round to bf16 and back

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }  // F.silu (opmath f32)

inline int stream_blocks(long chunks) {
  const long b = (chunks + 255) / 256;
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

// hidden[m, c] = bf16( bf16(silu(x1)) * x2 ), x1 = x12[m, c], x2 = x12[m, h + c] (modules.py:103-105)
__global__ void k_swiglu_fwd(int M, int h8, const bf16_t* __restrict__ x12, long ld, bf16_t* __restrict__ out,
                             long ldo) {
  const long n = (long)M * h8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long m = i / h8;
    const int c = (int)(i - m * h8) * 8;
    const uint4 a = *(const uint4*)(x12 + m * ld + c);
    const uint4 b = *(const uint4*)(x12 + m * ld + (long)h8 * 8 + c);
    const bf16_t* av = (const bf16_t*)&a;
    const bf16_t* bv = (const bf16_t*)&b;
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float s0 = bfr(silu_f(bf2f(av[2 * j]))), s1 = bfr(silu_f(bf2f(av[2 * j + 1])));
      o[j] = pack_bf2(s0 * bf2f(bv[2 * j]), s1 * bf2f(bv[2 * j + 1]));
    }
    *(uint4*)(out + m * ldo + c) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// Autograd of hidden = a * x2, a = silu(x1), in bf16 (mul backward, then silu_backward):
//   dx2 = bf16(dh * a),   ga = bf16(dh * x2),   dx1 = bf16(ga * sig * (1 + x1 * (1 - sig))), sig = sigmoid(x1)
__global__ void k_swiglu_bwd(int M, int h8, const bf16_t* __restrict__ dh, long lddh, const bf16_t* __restrict__ x12,
                             long ld, bf16_t* __restrict__ dx12, long lddx) {
  const long n = (long)M * h8;
  const long hh = (long)h8 * 8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long m = i / h8;
    const int c = (int)(i - m * h8) * 8;
    const uint4 g = *(const uint4*)(dh + m * lddh + c);
    const uint4 a = *(const uint4*)(x12 + m * ld + c);
    const uint4 b = *(const uint4*)(x12 + m * ld + hh + c);
    const bf16_t* gv = (const bf16_t*)&g;
    const bf16_t* av = (const bf16_t*)&a;
    const bf16_t* bv = (const bf16_t*)&b;
    float d1[8], d2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x1 = bf2f(av[j]), x2 = bf2f(bv[j]), gy = bf2f(gv[j]);
      const float e = expf(-x1);
      const float sig = 1.0f / (1.0f + e);
      d2[j] = gy * bfr(x1 / (1.0f + e));  // a = silu(x1) as the forward rounded it
      d1[j] = bfr(gy * x2) * sig * (1.0f + x1 * (1.0f - sig));
    }
    *(uint4*)(dx12 + m * lddx + c) =
        make_uint4(pack_bf2(d1[0], d1[1]), pack_bf2(d1[2], d1[3]), pack_bf2(d1[4], d1[5]), pack_bf2(d1[6], d1[7]));
    *(uint4*)(dx12 + m * lddx + hh + c) =
        make_uint4(pack_bf2(d2[0], d2[1]), pack_bf2(d2[2], d2[3]), pack_bf2(d2[4], d2[5]), pack_bf2(d2[6], d2[7]));
  }
}

// out[m, n] = resid[m, n] + bf16( bf16(y[m, n]) * bf16(scale[m]) ): the branch output (bf16 under
// autocast) times drop_path's random_tensor (x.new_empty(...) in the branch's dtype), added to the
// residual stream (f32; bf16 on the no-grad target encoder's bf16 residual, RB).
template <bool RB>
__global__ void k_rowscale_add(int M, int n4, const float* __restrict__ y, long ldy, const float* __restrict__ scale,
                               const void* __restrict__ resid, long ldr, void* __restrict__ out, long ldo) {
  const long n = (long)M * n4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long m = i / n4;
    const int c = (int)(i - m * n4) * 4;
    const float s = bfr(scale[m]);
    const float4 v = *(const float4*)(y + m * ldy + c);
    const float b0 = bfr(bfr(v.x) * s), b1 = bfr(bfr(v.y) * s), b2 = bfr(bfr(v.z) * s), b3 = bfr(bfr(v.w) * s);
    if constexpr (RB) {
      const uint2 r = *(const uint2*)((const bf16_t*)resid + m * ldr + c);
      const float r0 = __uint_as_float(r.x << 16), r1 = __uint_as_float(r.x & 0xffff0000u);
      const float r2 = __uint_as_float(r.y << 16), r3 = __uint_as_float(r.y & 0xffff0000u);
      *(uint2*)((bf16_t*)out + m * ldo + c) = make_uint2(pack_bf2(r0 + b0, r1 + b1), pack_bf2(r2 + b2, r3 + b3));
    } else {
      const float4 r = *(const float4*)((const float*)resid + m * ldr + c);
      *(float4*)((float*)out + m * ldo + c) = make_float4(r.x + b0, r.y + b1, r.z + b2, r.w + b3);
    }
  }
}

// out[m, n] = bf16( bf16(dx[m, n]) * bf16(scale[m]) ): the residual add's gradient cast to the branch
// dtype, then drop_path's multiply backward (the branch output-projection's dY)
__global__ void k_rowscale_bf16(int M, int n4, const float* __restrict__ dx, long ld, const float* __restrict__ scale,
                                bf16_t* __restrict__ out, long ldo) {
  const long n = (long)M * n4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long m = i / n4;
    const int c = (int)(i - m * n4) * 4;
    const float s = bfr(scale[m]);
    const float4 v = *(const float4*)(dx + m * ld + c);
    *(uint2*)(out + m * ldo + c) = make_uint2(pack_bf2(bfr(v.x) * s, bfr(v.y) * s), pack_bf2(bfr(v.z) * s, bfr(v.w) * s));
  }
}

// Dropout, elementwise (F.dropout in the branch's bf16 under autocast: y = bf16(bf16(x) * z) with
// z = 1 / (1 - p) on kept elements, 0 on dropped ones; the backward is the same op on the gradient).
// MODE 0: out = y (bf16); 1: out = resid + y (f32 residual stream); 2: the same on a bf16 residual;
// 3: out = bf16(y * aux) (aux bf16: GELU'(pre), the activation's backward after the dropout's).
template <bool XF32, int MODE>
__global__ void k_dropout(int M, int n4, const void* __restrict__ x, long ldx, const bf16_t* __restrict__ aux,
                          long lda, const void* __restrict__ resid, long ldr, void* __restrict__ out, long ldo,
                          uint32_t thresh, float scale, uint32_t seed) {
  const long n = (long)M * n4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long m = i / n4;
    const int c = (int)(i - m * n4) * 4;
    float v[4];
    if constexpr (XF32) {
      const float4 t = *(const float4*)((const float*)x + m * ldx + c);
      v[0] = bfr(t.x); v[1] = bfr(t.y); v[2] = bfr(t.z); v[3] = bfr(t.w);
    } else {
      const uint2 t = *(const uint2*)((const bf16_t*)x + m * ldx + c);
      v[0] = __uint_as_float(t.x << 16); v[1] = __uint_as_float(t.x & 0xffff0000u);
      v[2] = __uint_as_float(t.y << 16); v[3] = __uint_as_float(t.y & 0xffff0000u);
    }
    const uint32_t rk = drop_row(seed, (uint32_t)m);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = bfr(v[j] * (drop_u(rk, (uint32_t)(c + j)) >= thresh ? scale : 0.f));
    if constexpr (MODE == 3) {
      const uint2 t = *(const uint2*)(aux + m * lda + c);
      v[0] *= __uint_as_float(t.x << 16); v[1] *= __uint_as_float(t.x & 0xffff0000u);
      v[2] *= __uint_as_float(t.y << 16); v[3] *= __uint_as_float(t.y & 0xffff0000u);
    }
    if constexpr (MODE == 1) {
      const float4 r = *(const float4*)((const float*)resid + m * ldr + c);
      *(float4*)((float*)out + m * ldo + c) = make_float4(r.x + v[0], r.y + v[1], r.z + v[2], r.w + v[3]);
    } else {
      if constexpr (MODE == 2) {
        const uint2 r = *(const uint2*)((const bf16_t*)resid + m * ldr + c);
        v[0] += __uint_as_float(r.x << 16); v[1] += __uint_as_float(r.x & 0xffff0000u);
        v[2] += __uint_as_float(r.y << 16); v[3] += __uint_as_float(r.y & 0xffff0000u);
      }
      *(uint2*)((bf16_t*)out + m * ldo + c) = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
    }
  }
}

}  // namespace

uint32_t vj_drop_thresh(float p) {
  const double t = (double)p * 4294967296.0;
  return t <= 0.0 ? 0u : (t >= 4294967295.0 ? 4294967295u : (uint32_t)(t + 0.5));
}

extern "C" int vj_dropout(int M, int N, const void* x, long ldx, int x_f32, const void* aux, long ldaux,
                          const void* resid, long ldr, int resid_f32, void* out, long ldo, float p, unsigned seed,
                          void* stream) {
  if (M == 0 || N == 0) return VJ_OK;
  VJ_CHECK_ARG(M > 0 && N > 0 && x && out && !(aux && resid), "vj_dropout: bad arguments");
  VJ_CHECK_ARG(p >= 0.f && p < 1.f, "vj_dropout: p must be in [0, 1) (got %g)", (double)p);
  VJ_CHECK_ARG(N % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 && (!aux || ldaux % 4 == 0) && (!resid || ldr % 4 == 0) &&
                   !((uintptr_t)x & (x_f32 ? 15 : 7)) && !((uintptr_t)aux & 7) &&
                   !((uintptr_t)resid & (resid_f32 ? 15 : 7)) && !((uintptr_t)out & (resid && resid_f32 ? 15 : 7)),
               "vj_dropout: N, strides must be multiples of 4 and the rows aligned");
  const int n4 = N / 4;
  const uint32_t th = vj_drop_thresh(p);
  const float sc = 1.f / (1.f - p);
  const dim3 g(stream_blocks((long)M * n4)), b(256);
  hipStream_t st = (hipStream_t)stream;
  const int mode = resid ? (resid_f32 ? 1 : 2) : (aux ? 3 : 0);
#define VJ_DROP_LAUNCH(XF, MD) \
  hipLaunchKernelGGL((k_dropout<XF, MD>), g, b, 0, st, M, n4, x, ldx, (const bf16_t*)aux, ldaux, resid, ldr, out, ldo, th, sc, seed)
  if (x_f32) {
    switch (mode) {
      case 0: VJ_DROP_LAUNCH(true, 0); break;
      case 1: VJ_DROP_LAUNCH(true, 1); break;
      case 2: VJ_DROP_LAUNCH(true, 2); break;
      default: VJ_DROP_LAUNCH(true, 3); break;
    }
  } else {
    switch (mode) {
      case 0: VJ_DROP_LAUNCH(false, 0); break;
      case 1: VJ_DROP_LAUNCH(false, 1); break;
      case 2: VJ_DROP_LAUNCH(false, 2); break;
      default: VJ_DROP_LAUNCH(false, 3); break;
    }
  }
#undef VJ_DROP_LAUNCH
  VJ_LAUNCH_CHECK("vj_dropout");
  return VJ_OK;
}

extern "C" int vj_swiglu_fwd(int M, int h, const void* x12, long ld, void* out, long ldo, void* stream) {
  if (M == 0 || h == 0) return VJ_OK;
  VJ_CHECK_ARG(M > 0 && h > 0 && x12 && out, "vj_swiglu_fwd: bad arguments");
  VJ_CHECK_ARG(h % 8 == 0 && ld % 8 == 0 && ldo % 8 == 0 && ld >= 2L * h && ldo >= h &&
                   !(((uintptr_t)x12 | (uintptr_t)out) & 15),
               "vj_swiglu_fwd: h, strides must be multiples of 8 (ld >= 2h) and the pointers 16-B aligned");
  const int h8 = h / 8;
  hipLaunchKernelGGL(k_swiglu_fwd, dim3(stream_blocks((long)M * h8)), dim3(256), 0, (hipStream_t)stream, M, h8,
                     (const bf16_t*)x12, ld, (bf16_t*)out, ldo);
  VJ_LAUNCH_CHECK("vj_swiglu_fwd");
  return VJ_OK;
}

extern "C" int vj_swiglu_bwd(int M, int h, const void* dh, long lddh, const void* x12, long ld, void* dx12, long lddx,
                             void* stream) {
  if (M == 0 || h == 0) return VJ_OK;
  VJ_CHECK_ARG(M > 0 && h > 0 && dh && x12 && dx12, "vj_swiglu_bwd: bad arguments");
  VJ_CHECK_ARG(h % 8 == 0 && lddh % 8 == 0 && ld % 8 == 0 && lddx % 8 == 0 && lddh >= h && ld >= 2L * h &&
                   lddx >= 2L * h && !(((uintptr_t)dh | (uintptr_t)x12 | (uintptr_t)dx12) & 15),
               "vj_swiglu_bwd: h, strides must be multiples of 8 (ld, lddx >= 2h) and the pointers 16-B aligned");
  const int h8 = h / 8;
  hipLaunchKernelGGL(k_swiglu_bwd, dim3(stream_blocks((long)M * h8)), dim3(256), 0, (hipStream_t)stream, M, h8,
                     (const bf16_t*)dh, lddh, (const bf16_t*)x12, ld, (bf16_t*)dx12, lddx);
  VJ_LAUNCH_CHECK("vj_swiglu_bwd");
  return VJ_OK;
}

extern "C" int vj_rowscale_add(int M, int N, const float* y, long ldy, const float* scale, const void* resid, long ldr,
                               void* out, long ldo, int bf16_resid, void* stream) {
  if (M == 0 || N == 0) return VJ_OK;
  VJ_CHECK_ARG(M > 0 && N > 0 && y && scale && resid && out, "vj_rowscale_add: bad arguments");
  VJ_CHECK_ARG(N % 4 == 0 && ldy % 4 == 0 && ldr % 4 == 0 && ldo % 4 == 0 &&
                   !(((uintptr_t)y | (uintptr_t)resid | (uintptr_t)out) & (bf16_resid ? 7 : 15)) &&
                   !((uintptr_t)y & 15),
               "vj_rowscale_add: N, strides must be multiples of 4 and the rows aligned");
  const int n4 = N / 4;
  if (bf16_resid)
    hipLaunchKernelGGL(k_rowscale_add<true>, dim3(stream_blocks((long)M * n4)), dim3(256), 0, (hipStream_t)stream, M,
                       n4, y, ldy, scale, resid, ldr, out, ldo);
  else
    hipLaunchKernelGGL(k_rowscale_add<false>, dim3(stream_blocks((long)M * n4)), dim3(256), 0, (hipStream_t)stream, M,
                       n4, y, ldy, scale, resid, ldr, out, ldo);
  VJ_LAUNCH_CHECK("vj_rowscale_add");
  return VJ_OK;
}

extern "C" int vj_rowscale_bf16(int M, int N, const float* dx, long ld, const float* scale, void* out, long ldo,
                                void* stream) {
  if (M == 0 || N == 0) return VJ_OK;
  VJ_CHECK_ARG(M > 0 && N > 0 && dx && scale && out, "vj_rowscale_bf16: bad arguments");
  VJ_CHECK_ARG(N % 4 == 0 && ld % 4 == 0 && ldo % 4 == 0 && !((uintptr_t)dx & 15) && !((uintptr_t)out & 7),
               "vj_rowscale_bf16: N, strides must be multiples of 4 and the rows aligned");
  const int n4 = N / 4;
  hipLaunchKernelGGL(k_rowscale_bf16, dim3(stream_blocks((long)M * n4)), dim3(256), 0, (hipStream_t)stream, M, n4, dx,
                     ld, scale, (bf16_t*)out, ldo);
  VJ_LAUNCH_CHECK("vj_rowscale_bf16");
  return VJ_OK;
}
