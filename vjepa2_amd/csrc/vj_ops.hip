// Memory-bound kernels of the V-JEPA 2 train step (gfx950). All are HBM-bound: vectorised 16-B
// accesses, one wave per row for row-wise ops, deterministic two-level reductions (no atomics).
//
//   LayerNorm fwd/bwd           nn.LayerNorm in Block (modules.py:556-563), encoder/predictor norm
//   RoPE fwd/bwd (in place)     rotate_queries_or_keys (modules.py:26-50) on q,k of RoPEAttention (:343-365)
//   tubelet im2col gather       PatchEmbed3D Conv3d (patch_embed.py:42-52) + apply_masks (masks/utils.py:9-21)
//   row gather/scatter/fill/add apply_masks, predictor token assembly & (un)sort (predictor.py:182-242)
//   stable-rank index build     torch.argsort(cat(masks_x, masks_y)) (predictor.py:210-217, 240)
//   fused target-LN + L1 loss   forward_target F.layer_norm + loss_fn (app/vjepa/train.py:414-435)
//   AdamW, finite-check, EMA    torch.optim.AdamW foreach math (app/vjepa/utils.py:239), train.py:456-465
//   column sums (bias grads), f32->bf16 casts
#include "vj_common.h"

static_assert(sizeof(float4) == 16, "");

namespace {

// ------------------------------------------------------------------------------------------------
// LayerNorm forward: wave per row. x f32 or bf16 [M, ldx]; y bf16 or f32 [M, ldy]; optional affine.
constexpr int LN_MAXV = 8;  // float4 per lane -> D <= 64*4*8 = 2048

// e4m3 per-row scale exponent: the least e with amax * 2^-e <= 448 (0 for an all-zero or non-finite row)
__device__ __forceinline__ int f8_row_exp(float amax) {
  if (!(amax > 0.f) || !(amax <= 3.0e38f)) return 0;
  int e = (int)ceilf(__log2f(amax / 448.f));
  if (ldexpf(amax, -e) > 448.f) ++e;
  if (ldexpf(amax, -(e - 1)) <= 448.f) --e;
  return min(max(e, -120), 120);
}

// LN_RPW rows per wave: gamma / beta are loaded once per wave and the next row's x is fetched while
// the current row is reduced and written (one row per wave re-read the 8 KB of gamma / beta for
// every 4-6 KB row of traffic)
constexpr int LN_RPW = 4;

template <bool XBF, int NV>
__device__ __forceinline__ void ln_load_row(const void* __restrict__ x, long ldx, long row, int D, int lane,
                                            float4 (&v)[NV]) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < D) {
      if constexpr (XBF) {
        const uint2 u = *(const uint2*)((const bf16_t*)x + row * ldx + c);
        v[i] = make_float4(bf2f(u.x & 0xffff), bf2f(u.x >> 16), bf2f(u.y & 0xffff), bf2f(u.y >> 16));
      } else {
        v[i] = *(const float4*)((const float*)x + row * ldx + c);
      }
    }
  }
}

template <bool XBF, bool YF32, int NV, bool YF8 = false>
__global__ __launch_bounds__(256) void k_ln_fwd(int M, int D, const void* __restrict__ x, long ldx,
                                                const float* __restrict__ gamma, const float* __restrict__ beta,
                                                float eps, void* __restrict__ y, long ldy, float* __restrict__ mean,
                                                float* __restrict__ rstd, int* __restrict__ yexp = nullptr) {
  const int lane = threadIdx.x & 63;
  const long row0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * LN_RPW;
  if (row0 >= M) return;
  float4 g[NV], bb[NV], v[NV], vn[NV];
  if (gamma) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      if (c < D) {
        g[i] = *(const float4*)(gamma + c);
        bb[i] = *(const float4*)(beta + c);
      }
    }
  }
  ln_load_row<XBF, NV>(x, ldx, row0, D, lane, v);
#pragma unroll 1
  for (int rr = 0; rr < LN_RPW; ++rr) {
    const long row = row0 + rr;
    if (row >= M) break;
    if (rr + 1 < LN_RPW && row + 1 < M) ln_load_row<XBF, NV>(x, ldx, row + 1, D, lane, vn);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if ((i * 64 + lane) * 4 < D) s += v[i].x + v[i].y + v[i].z + v[i].w;
    const float mu = wave_sum(s) / D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if ((i * 64 + lane) * 4 < D) {
        const float a = v[i].x - mu, b = v[i].y - mu, cc = v[i].z - mu, d = v[i].w - mu;
        q += a * a + b * b + cc * cc + d * d;
      }
    }
    const float rs = rsqrtf(wave_sum(q) / D + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      if (c < D) {
        float o[4] = {(v[i].x - mu) * rs, (v[i].y - mu) * rs, (v[i].z - mu) * rs, (v[i].w - mu) * rs};
        if (gamma) {
          o[0] = o[0] * g[i].x + bb[i].x; o[1] = o[1] * g[i].y + bb[i].y;
          o[2] = o[2] * g[i].z + bb[i].z; o[3] = o[3] * g[i].w + bb[i].w;
        }
        if constexpr (YF8) {
          v[i] = make_float4(o[0], o[1], o[2], o[3]);  // kept for the scaled fp8 pass below
        } else if constexpr (YF32) {
          *(float4*)((float*)y + row * ldy + c) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
          *(uint2*)((bf16_t*)y + row * ldy + c) = make_uint2(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]));
        }
      }
    }
    if constexpr (YF8) {  // per-row scaled e4m3: y8 = e4m3(y * 2^-e), e = the least exponent with amax * 2^-e <= 448
      float am = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i)
        if ((i * 64 + lane) * 4 < D)
          am = fmaxf(am, fmaxf(fmaxf(fabsf(v[i].x), fabsf(v[i].y)), fmaxf(fabsf(v[i].z), fabsf(v[i].w))));
      am = wave_max(am);
      const int e = f8_row_exp(am);
      const float sc = ldexpf(1.f, -e);
      const bool bad = !(am <= 3.0e38f);  // inf / NaN row: every byte NaN (e4m3fn has no infinity)
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = (i * 64 + lane) * 4;
        if (c < D)
          *(uint32_t*)((unsigned char*)y + row * ldy + c) =
              bad ? 0x7f7f7f7fu : f8pack4(v[i].x * sc, v[i].y * sc, v[i].z * sc, v[i].w * sc);
      }
      if (lane == 0) yexp[row] = e;
    }
    if (lane == 0) {
      if (mean) mean[row] = mu;
      if (rstd) rstd[row] = rs;
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = vn[i];
  }
}

// LayerNorm forward with every row of a wave in flight at once: a wave owns R consecutive rows and
// issues all their 16-B loads (E = 8 bf16 or 4 f32 elements per lane-vector, kept packed as loaded)
// before the first reduction, so a CU holds R x the bytes in flight of a one-row-lookahead loop at
// a lower register cost (bf16 rows stay packed: 8 VGPRs per 1024-wide row). Element map: vector i of
// lane l holds elements (64 i + l) E ... + E - 1. Outputs: bf16 rows as 16-B (E = 8) / 8-B stores,
// f32 rows as 16-B stores; gamma / beta re-read per row (L1 hits) instead of held in registers.
template <bool XBF, bool YF32, int NV, int R>
__global__ __launch_bounds__(256) void k_ln_fwd3(int M, int D, const void* __restrict__ x, long ldx,
                                                 const float* __restrict__ gamma, const float* __restrict__ beta,
                                                 float eps, void* __restrict__ y, long ldy, float* __restrict__ mean,
                                                 float* __restrict__ rstd) {
  constexpr int E = XBF ? 8 : 4;
  const int lane = threadIdx.x & 63;
  const long row0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= M) return;
  auto ok = [&](int i) { return (i * 64 + lane) * E < D; };
  uint4 raw[R][NV];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      raw[r][i] = make_uint4(0u, 0u, 0u, 0u);
      if (ok(i) && row0 + r < M) {
        const long off = (row0 + r) * ldx + (i * 64 + lane) * E;
        raw[r][i] = XBF ? *(const uint4*)((const bf16_t*)x + off) : *(const uint4*)((const float*)x + off);
      }
    }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const long row = row0 + r;
    if (row >= M) break;
    float v[NV][E];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const uint32_t w[4] = {raw[r][i].x, raw[r][i].y, raw[r][i].z, raw[r][i].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if constexpr (XBF) {
          v[i][2 * k] = __builtin_bit_cast(float, w[k] << 16);
          v[i][2 * k + 1] = __builtin_bit_cast(float, w[k] & 0xffff0000u);
        } else {
          v[i][k] = __builtin_bit_cast(float, w[k]);
        }
      }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (ok(i))
#pragma unroll
        for (int k = 0; k < E; ++k) s += v[i][k];
    const float mu = wave_sum(s) / D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (ok(i))
#pragma unroll
        for (int k = 0; k < E; ++k) {
          const float a = v[i][k] - mu;
          q += a * a;
        }
    const float rs = rsqrtf(wave_sum(q) / D + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (!ok(i)) continue;
      const int c = (i * 64 + lane) * E;
      float o[E];
#pragma unroll
      for (int k = 0; k < E; ++k) o[k] = (v[i][k] - mu) * rs;
      if (gamma) {
#pragma unroll
        for (int k = 0; k < E; k += 4) {
          const float4 gg = *(const float4*)(gamma + c + k), bb = *(const float4*)(beta + c + k);
          o[k] = o[k] * gg.x + bb.x; o[k + 1] = o[k + 1] * gg.y + bb.y;
          o[k + 2] = o[k + 2] * gg.z + bb.z; o[k + 3] = o[k + 3] * gg.w + bb.w;
        }
      }
      const long off = row * ldy + c;
      if constexpr (YF32) {
#pragma unroll
        for (int k = 0; k < E; k += 4) *(float4*)((float*)y + off + k) = make_float4(o[k], o[k + 1], o[k + 2], o[k + 3]);
      } else if constexpr (E == 8) {
        *(uint4*)((bf16_t*)y + off) = make_uint4(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]), pack_bf2(o[4], o[5]),
                                                 pack_bf2(o[6], o[7]));
      } else {
        *(uint2*)((bf16_t*)y + off) = make_uint2(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]));
      }
    }
    if (lane == 0) {
      if (mean) mean[row] = mu;
      if (rstd) rstd[row] = rs;
    }
  }
}

// Per-row fp8 quantisation of a [M, K] f32 / bf16 matrix (the fp8 target encoder's weights, one
// scale per output channel): wave per row, two passes over the row (amax, then scaled e4m3 bytes).
template <bool XBF>
__global__ __launch_bounds__(256) void k_quant_rows_fp8(int M, int K, const void* __restrict__ x, long ldx,
                                                        unsigned char* __restrict__ y, long ldy, int* __restrict__ yexp) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  auto load4 = [&](int c) {
    if constexpr (XBF) {
      const uint2 u = *(const uint2*)((const bf16_t*)x + row * ldx + c);
      return make_float4(bf2f(u.x & 0xffff), bf2f(u.x >> 16), bf2f(u.y & 0xffff), bf2f(u.y >> 16));
    } else {
      return *(const float4*)((const float*)x + row * ldx + c);
    }
  };
  float am = 0.f;
  for (int c = lane * 4; c < K; c += 256) {
    const float4 v = load4(c);
    am = fmaxf(am, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
  am = wave_max(am);
  const int e = f8_row_exp(am);
  const float sc = ldexpf(1.f, -e);
  const bool bad = !(am <= 3.0e38f);
  for (int c = lane * 4; c < K; c += 256) {
    const float4 v = load4(c);
    *(uint32_t*)(y + row * ldy + c) = bad ? 0x7f7f7f7fu : f8pack4(v.x * sc, v.y * sc, v.z * sc, v.w * sc);
  }
  if (lane == 0) yexp[row] = e;
}

// LayerNorm backward. dy bf16 [M, lddy]; x f32 [M, ldx]; dres f32 [M, ldr] = (dres_in or 0) + dx;
// optional bf16 copy of the resulting dres; per-block partials of dgamma/dbeta -> ws[blk][2][D].
template <bool ACC, int NV>
__global__ __launch_bounds__(256) void k_ln_bwd(int M, int D, const bf16_t* __restrict__ dy, long lddy,
                                                const float* __restrict__ x, long ldx, const float* __restrict__ mean,
                                                const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                const float* __restrict__ dres_in, long ldri, float* __restrict__ dres,
                                                long ldr, bf16_t* __restrict__ dres_bf, long ldrb, float* __restrict__ ws,
                                                int nsum) {
  // column partials per block, [nsum][D]: dgamma, dbeta, then (nsum == 4) sum of dres_in and of dres
  // (the bias gradients of the Linear layers whose outputs these are: fc2 and proj, modules.py:77-83)
  __shared__ float red[4][NV * 256];  // D <= 2048
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float4 acc[4][NV];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int i = 0; i < NV; ++i) acc[k][i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (long row = (long)blockIdx.x * 4 + wave; row < M; row += (long)gridDim.x * 4) {
    const float mu = mean[row], rs = rstd[row];
    float4 xh[NV], g[NV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      if (c < D) {
        const float4 xv = *(const float4*)(x + row * ldx + c);
        const uint2 u = *(const uint2*)(dy + row * lddy + c);
        const float4 d = make_float4(bf2f(u.x & 0xffff), bf2f(u.x >> 16), bf2f(u.y & 0xffff), bf2f(u.y >> 16));
        xh[i] = make_float4((xv.x - mu) * rs, (xv.y - mu) * rs, (xv.z - mu) * rs, (xv.w - mu) * rs);
        acc[1][i].x += d.x; acc[1][i].y += d.y; acc[1][i].z += d.z; acc[1][i].w += d.w;
        acc[0][i].x += d.x * xh[i].x; acc[0][i].y += d.y * xh[i].y;
        acc[0][i].z += d.z * xh[i].z; acc[0][i].w += d.w * xh[i].w;
        float4 gm = make_float4(1.f, 1.f, 1.f, 1.f);
        if (gamma) gm = *(const float4*)(gamma + c);
        g[i] = make_float4(d.x * gm.x, d.y * gm.y, d.z * gm.z, d.w * gm.w);
        s1 += g[i].x + g[i].y + g[i].z + g[i].w;
        s2 += g[i].x * xh[i].x + g[i].y * xh[i].y + g[i].z * xh[i].z + g[i].w * xh[i].w;
      }
    }
    const float m1 = wave_sum(s1) / D, m2 = wave_sum(s2) / D;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 4;
      if (c < D) {
        float4 dx = make_float4(rs * (g[i].x - m1 - xh[i].x * m2), rs * (g[i].y - m1 - xh[i].y * m2),
                                rs * (g[i].z - m1 - xh[i].z * m2), rs * (g[i].w - m1 - xh[i].w * m2));
        if constexpr (ACC) {
          const float4 o = *(const float4*)(dres_in + row * ldri + c);
          acc[2][i].x += o.x; acc[2][i].y += o.y; acc[2][i].z += o.z; acc[2][i].w += o.w;
          dx.x += o.x; dx.y += o.y; dx.z += o.z; dx.w += o.w;
        }
        acc[3][i].x += dx.x; acc[3][i].y += dx.y; acc[3][i].z += dx.z; acc[3][i].w += dx.w;
        *(float4*)(dres + row * ldr + c) = dx;
        if (dres_bf)
          *(uint2*)(dres_bf + row * ldrb + c) = make_uint2(pack_bf2(dx.x, dx.y), pack_bf2(dx.z, dx.w));
      }
    }
  }
  if (!ws) return;
  // block reduction of the per-wave partials, waves added in fixed order (deterministic)
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (k >= nsum) break;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const int c = (i * 64 + lane) * 4;
          if (c < D) {
            float4* a = (float4*)&red[k][c];
            if (w == 0) {
              *a = acc[k][i];
            } else {
              const float4 v = *a;
              *a = make_float4(v.x + acc[k][i].x, v.y + acc[k][i].y, v.z + acc[k][i].z, v.w + acc[k][i].w);
            }
          }
        }
      }
    }
    __syncthreads();
  }
  for (int k = 0; k < nsum; ++k)
    for (int c = threadIdx.x; c < D; c += 256) ws[((long)blockIdx.x * nsum + k) * D + c] = red[k][c];
}

// LayerNorm backward, 16-B accesses: lane l's vector i holds the 8 columns (64 i + l) * 8 .. + 7 of
// every operand (dy bf16 16 B, x / dres_in / dres f32 2 x 16 B, dres bf16 16 B); dres_in is loaded
// with x and dy, before the row's reductions. Same outputs and fixed-order partials as k_ln_bwd.
// BFR (the bf16 residual stream of the trained encoder, the reference's autocast precision): x and
// dres_in are bf16 rows and the result is written as bf16 only (dres_bf; dres unused): 8 B / element
// instead of 16 + 2.
template <bool ACC, int NV, bool SUMS, bool BFR = false>
__global__ __launch_bounds__(256) void k_ln_bwd2(int M, int D, const bf16_t* __restrict__ dy, long lddy,
                                                 const void* __restrict__ xv_, long ldx, const float* __restrict__ mean,
                                                 const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                 const void* __restrict__ dres_in_, long ldri, float* __restrict__ dres,
                                                 long ldr, bf16_t* __restrict__ dres_bf, long ldrb, float* __restrict__ ws,
                                                 int nsum) {
  auto unpack8 = [](const uint4& u, float (&o)[8]) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[2 * k] = __builtin_bit_cast(float, w[k] << 16);
      o[2 * k + 1] = __builtin_bit_cast(float, w[k] & 0xffff0000u);
    }
  };
  constexpr int E = 8;
  __shared__ float red[4][NV * 64 * E];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  auto ok = [&](int i) { return (i * 64 + lane) * E < D; };
  constexpr int NS = SUMS ? 4 : 2;  // column partials kept: dgamma, dbeta (+ sums of dres_in, dres)
  float acc[NS][NV][E];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int k = 0; k < E; ++k)
#pragma unroll
      for (int q = 0; q < NS; ++q) acc[q][i][k] = 0.f;
  for (long row = (long)blockIdx.x * 4 + wave; row < M; row += (long)gridDim.x * 4) {
    const float mu = mean[row], rs = rstd[row];
    float xh[NV][E], g[NV][E], ri[NV][E];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (!ok(i)) continue;
      const int c = (i * 64 + lane) * E;
      float xv[E];
      if constexpr (BFR) {
        unpack8(*(const uint4*)((const bf16_t*)xv_ + row * ldx + c), xv);
      } else {
        const float* x = (const float*)xv_;
        const float4 x0 = *(const float4*)(x + row * ldx + c), x1 = *(const float4*)(x + row * ldx + c + 4);
        xv[0] = x0.x; xv[1] = x0.y; xv[2] = x0.z; xv[3] = x0.w; xv[4] = x1.x; xv[5] = x1.y; xv[6] = x1.z; xv[7] = x1.w;
      }
      const uint4 u = *(const uint4*)(dy + row * lddy + c);
      if constexpr (ACC) {
        if constexpr (BFR) {
          unpack8(*(const uint4*)((const bf16_t*)dres_in_ + row * ldri + c), ri[i]);
        } else {
          const float* dres_in = (const float*)dres_in_;
          const float4 r0 = *(const float4*)(dres_in + row * ldri + c), r1 = *(const float4*)(dres_in + row * ldri + c + 4);
          ri[i][0] = r0.x; ri[i][1] = r0.y; ri[i][2] = r0.z; ri[i][3] = r0.w;
          ri[i][4] = r1.x; ri[i][5] = r1.y; ri[i][6] = r1.z; ri[i][7] = r1.w;
        }
      }
      float gm[E];  // gamma re-read per row (cache-resident) rather than held in 16 VGPRs
      if (gamma) {
        const float4 g0 = *(const float4*)(gamma + c), g1 = *(const float4*)(gamma + c + 4);
        gm[0] = g0.x; gm[1] = g0.y; gm[2] = g0.z; gm[3] = g0.w; gm[4] = g1.x; gm[5] = g1.y; gm[6] = g1.z; gm[7] = g1.w;
      } else {
#pragma unroll
        for (int k = 0; k < E; ++k) gm[k] = 1.f;
      }
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int k = 0; k < E; ++k) {
        const float d = __builtin_bit_cast(float, (k & 1) ? (w[k >> 1] & 0xffff0000u) : (w[k >> 1] << 16));
        xh[i][k] = (xv[k] - mu) * rs;
        acc[1][i][k] += d;
        acc[0][i][k] += d * xh[i][k];
        g[i][k] = d * gm[k];
        s1 += g[i][k];
        s2 += g[i][k] * xh[i][k];
      }
    }
    const float m1 = wave_sum(s1) / D, m2 = wave_sum(s2) / D;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (!ok(i)) continue;
      const int c = (i * 64 + lane) * E;
      float dx[E];
#pragma unroll
      for (int k = 0; k < E; ++k) {
        dx[k] = rs * (g[i][k] - m1 - xh[i][k] * m2);
        if constexpr (ACC) {
          if constexpr (SUMS) acc[2][i][k] += ri[i][k];
          dx[k] += ri[i][k];
        }
        if constexpr (SUMS) acc[3][i][k] += dx[k];
      }
      if constexpr (!BFR) {
        *(float4*)(dres + row * ldr + c) = make_float4(dx[0], dx[1], dx[2], dx[3]);
        *(float4*)(dres + row * ldr + c + 4) = make_float4(dx[4], dx[5], dx[6], dx[7]);
      }
      if (BFR || dres_bf)
        *(uint4*)(dres_bf + row * ldrb + c) = make_uint4(pack_bf2(dx[0], dx[1]), pack_bf2(dx[2], dx[3]),
                                                         pack_bf2(dx[4], dx[5]), pack_bf2(dx[6], dx[7]));
    }
  }
  if (!ws) return;
  // block reduction of the per-wave partials, waves added in fixed order (deterministic)
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        if (k >= nsum) break;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          if (!ok(i)) continue;
#pragma unroll
          for (int e = 0; e < E; ++e) {
            float* a = &red[k][(i * 64 + lane) * E + e];
            *a = w == 0 ? acc[k][i][e] : *a + acc[k][i][e];
          }
        }
      }
    }
    __syncthreads();
  }
  for (int k = 0; k < nsum; ++k)
    for (int c = threadIdx.x; c < D; c += 256) ws[((long)blockIdx.x * nsum + k) * D + c] = red[k][c];
}

// ------------------------------------------------------------------------------------------------
// Column sums. Stage 1: ws[s][n] = sum over the rows of slice s; thread = 8 consecutive columns
// (16-B bf16 / 2x16-B f32 loads), 4 row groups per block combined through LDS in fixed order.
template <bool BF>
__global__ __launch_bounds__(256) void k_colsum1(int M, int N, const void* __restrict__ x, long ld, int rows_per_slice,
                                                 float* __restrict__ ws) {
  __shared__ float red[4][512];
  const int cg = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c0 = (blockIdx.x * 64 + cg) * 8;
  const long r0 = (long)blockIdx.y * rows_per_slice;
  const long r1 = min((long)M, r0 + rows_per_slice);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto add = [&](const uint4 (&u)[BF ? 1 : 2]) {
    if constexpr (BF) {
      const uint32_t w[4] = {u[0].x, u[0].y, u[0].z, u[0].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[2 * j] += bf2f(w[j] & 0xffff);
        acc[2 * j + 1] += bf2f(w[j] >> 16);
      }
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        acc[4 * h] += __uint_as_float(u[h].x); acc[4 * h + 1] += __uint_as_float(u[h].y);
        acc[4 * h + 2] += __uint_as_float(u[h].z); acc[4 * h + 3] += __uint_as_float(u[h].w);
      }
    }
  };
  auto load = [&](long r, uint4 (&u)[BF ? 1 : 2]) {
    if constexpr (BF) {
      u[0] = *(const uint4*)((const bf16_t*)x + r * ld + c0);
    } else {
      u[0] = *(const uint4*)((const float*)x + r * ld + c0);
      u[1] = *(const uint4*)((const float*)x + r * ld + c0 + 4);
    }
  };
  if (c0 < N) {
    // 4 rows per step with every load issued before the adds (4 x 16-32 B in flight per thread);
    // the per-column add order stays the row order of this thread's rows
    long r = r0 + rg;
    for (; r + 12 < r1; r += 16) {
      uint4 u[4][BF ? 1 : 2];
#pragma unroll
      for (int k = 0; k < 4; ++k) load(r + 4 * k, u[k]);
#pragma unroll
      for (int k = 0; k < 4; ++k) add(u[k]);
    }
    for (; r < r1; r += 4) {
      uint4 u[BF ? 1 : 2];
      load(r, u);
      add(u);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rg][cg * 8 + j] = acc[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int n = blockIdx.x * 512 + i;
    if (n < N) ws[(long)blockIdx.y * N + n] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  }
}
// Stage 2: out[n] (+)= sum_s ws[s][n] (columns n >= split go to out2[n - split]). Block = 32
// columns x 32 row groups; each thread keeps 4 independent partial sums so 8 loads are in flight,
// then a fixed-order combine (deterministic, no atomics).
__global__ __launch_bounds__(1024) void k_colsum2(int S, int N, const float* __restrict__ ws, long ws_ld,
                                                  float* __restrict__ out, float* __restrict__ out2, int split,
                                                  int acc) {
  __shared__ float red[32][33];
  const int c = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int n = blockIdx.x * 32 + c;
  float s4[4] = {0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    int i = rg;
    for (; i + 7 * 32 < S; i += 8 * 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ws[(long)(i + u * 32) * ws_ld + n];
#pragma unroll
      for (int u = 0; u < 8; ++u) s4[u & 3] += v[u];
    }
    for (int u = 0; i < S; i += 32, ++u) s4[u & 3] += ws[(long)i * ws_ld + n];
  }
  red[rg][c] = (s4[0] + s4[1]) + (s4[2] + s4[3]);
  __syncthreads();
  if (rg == 0 && n < N) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < 32; ++r) t += red[r][c];
    float* o = n < split ? out + n : out2 + (n - split);
    *o = acc ? *o + t : t;
  }
}

// k_colsum2 for up to 4 column-sum vectors of one partial slab in ONE launch (the LayerNorm
// backward's dgamma / dbeta / bias-gradient sums): blockIdx.y = vector k, partial rows of stride
// ws_ld, vector k at column offset k * N; vectors with a null output are skipped.
struct ColsumOuts {
  float* out[4];
};
__global__ __launch_bounds__(1024) void k_colsum2_multi(int S, int N, const float* __restrict__ ws, long ws_ld,
                                                        ColsumOuts outs) {
  __shared__ float red[32][33];
  float* out = outs.out[blockIdx.y];
  if (out == nullptr) return;  // uniform per block
  const float* w = ws + (long)blockIdx.y * N;
  const int c = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int n = blockIdx.x * 32 + c;
  float s4[4] = {0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    int i = rg;
    for (; i + 7 * 32 < S; i += 8 * 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = w[(long)(i + u * 32) * ws_ld + n];
#pragma unroll
      for (int u = 0; u < 8; ++u) s4[u & 3] += v[u];
    }
    for (int u = 0; i < S; i += 32, ++u) s4[u & 3] += w[(long)i * ws_ld + n];
  }
  red[rg][c] = (s4[0] + s4[1]) + (s4[2] + s4[3]);
  __syncthreads();
  if (rg == 0 && n < N) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < 32; ++r) t += red[r][c];
    out[n] += t;
  }
}

// ------------------------------------------------------------------------------------------------
// RoPE on q and k of a [T, ld] bf16 qkv buffer, in place. Per head: three rotated slices of width
// sw = 2*((hd/3)/2) (depth, height, width positions), rest untouched. Element j of a slice uses
// angle theta_{j mod sw/2}; partner y_{2i} = -x_{2i+1}, y_{2i+1} = x_{2i} (modules.py:43-50).
// Angles come from host-built tables cos/sin[pos][i] (computed with the reference's fp32 ops).
// Thread = one 8-element chunk of one head of q or k.
template <bool F32>
__global__ void k_rope(int T, int H, int hd, void* __restrict__ qkv_, long ld, int q_off, int k_off,
                       const int* __restrict__ ids, int ids_mod, int tpf, int tpr, const float* __restrict__ ctab,
                       const float* __restrict__ stab, int half, int inverse) {
  const int cpr = hd / 8;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)T * 2 * H * cpr;
  if (i >= total) return;
  const int chunk = (int)(i % cpr);
  long rest = i / cpr;
  const int h = (int)(rest % H);
  rest /= H;
  const int which = (int)(rest % 2);
  const long t = rest / 2;
  const int sw = 2 * half;
  const int e0 = chunk * 8;
  if (e0 >= 3 * sw) return;  // untouched tail
  const int id = ids ? ids[t] : (int)(t % ids_mod);
  const int fr = id / tpf;
  const int hr = (id - tpf * fr) / tpr;
  const int wc = (id - tpf * fr) - tpr * hr;
  const long off = t * ld + (which ? k_off : q_off) + h * hd + e0;
  float x[8], o[8];
  if constexpr (F32) {  // fp32-operand parity mode
    const float4* p = (const float4*)((float*)qkv_ + off);
    const float4 a = p[0], b = p[1];
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  } else {
    bf16_t v[8];
    *(uint4*)v = *(const uint4*)((bf16_t*)qkv_ + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = bf2f(v[j]);
  }
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const int e = e0 + j;  // even element index within the head
    if (e >= 3 * sw) {
      o[j] = x[j];
      o[j + 1] = x[j + 1];
      continue;
    }
    const int ax = e / sw;
    const int js = e - ax * sw;  // even position within the slice
    const int pos = ax == 0 ? fr : (ax == 1 ? hr : wc);
    const int f0 = js % half, f1 = (js + 1) % half;
    const float c0 = ctab[pos * half + f0], s0 = stab[pos * half + f0];
    const float c1 = ctab[pos * half + f1], s1 = stab[pos * half + f1];
    if (!inverse) {
      o[j] = x[j] * c0 - x[j + 1] * s0;
      o[j + 1] = x[j + 1] * c1 + x[j] * s1;
    } else {  // transpose of the forward map (gradient)
      o[j] = x[j] * c0 + x[j + 1] * s1;
      o[j + 1] = -x[j] * s0 + x[j + 1] * c1;
    }
  }
  if constexpr (F32) {
    float4* p = (float4*)((float*)qkv_ + off);
    p[0] = make_float4(o[0], o[1], o[2], o[3]);
    p[1] = make_float4(o[4], o[5], o[6], o[7]);
  } else {
    bf16_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = f2bf(o[j]);
    *(uint4*)((bf16_t*)qkv_ + off) = *(uint4*)v;
  }
}

// ------------------------------------------------------------------------------------------------
// Tubelet im2col (Conv3d k = s = (tub, p, p) as a GEMM operand), gathering only the listed tokens.
// clip f32 [B, C, Tf, Hf, Wf]; row r -> (b, token) with token = idx ? idx[r] : r % N, b = r / K.
// out bf16 [R, C*tub*p*p], column = c*tub*p*p + kt*p*p + kh*p + kw (= Conv3d weight flattening).
template <bool F32>
__global__ void k_im2col(int R, int K, const long* __restrict__ idx, int C, int Tf, int Hf, int Wf, int tub,
                         int pch, const float* __restrict__ clip, void* __restrict__ out) {
  const int r = blockIdx.x;
  if (r >= R) return;
  const int b = r / K;
  const int Hp = Hf / pch, Wp = Wf / pch;
  const int tok = idx ? (int)idx[r] : (r % K);
  const int tt = tok / (Hp * Wp), hh = (tok % (Hp * Wp)) / Wp, ww = tok % Wp;
  const int kdim = C * tub * pch * pch;
  // each thread handles 4 consecutive kw of one (c, kt, kh) row: pch % 4 == 0
  const int nq = kdim / 4;
  for (int q = threadIdx.x; q < nq; q += blockDim.x) {
    const int col = q * 4;
    const int kw = col % pch;
    const int kh = (col / pch) % pch;
    const int kt = (col / (pch * pch)) % tub;
    const int c = col / (pch * pch * tub);
    const float* src = clip + ((((long)b * C + c) * Tf + (tt * tub + kt)) * Hf + (hh * pch + kh)) * Wf + ww * pch + kw;
    const float4 v = *(const float4*)src;
    if constexpr (F32) *(float4*)((float*)out + (long)r * kdim + col) = v;  // fp32-operand parity mode
    else *(uint2*)((bf16_t*)out + (long)r * kdim + col) = make_uint2(pack_bf2(v.x, v.y), pack_bf2(v.z, v.w));
  }
}

// ------------------------------------------------------------------------------------------------
// Row ops (bit-exact copies). elem = 2 or 4 bytes; ncols*elem % 16 == 0 handled by 4-B lanes.
__global__ void k_gather_rows(int R, int rowbytes, const char* __restrict__ src, long lds, const int* __restrict__ idx,
                              char* __restrict__ dst, long ldd, int scatter) {
  const int r = blockIdx.x;
  if (r >= R) return;
  const long sr = scatter ? r : idx[r];
  const long dr = scatter ? idx[r] : r;
  const uint4* s = (const uint4*)(src + sr * lds);
  uint4* d = (uint4*)(dst + dr * ldd);
  for (int i = threadIdx.x; i < rowbytes / 16; i += blockDim.x) d[i] = s[i];
}

// dst[idx[r]] = vec (f32 row broadcast; mask tokens)
__global__ void k_fill_rows(int R, int D, float* __restrict__ dst, long ldd, const int* __restrict__ idx,
                            const float* __restrict__ vec) {
  const int r = blockIdx.x;
  if (r >= R) return;
  float* d = dst + (long)idx[r] * ldd;
  for (int i = threadIdx.x; i < D; i += blockDim.x) d[i] = vec[i];
}

// dst[r] += table[idx[r]]   (sincos positional embeddings, non-RoPE variant). Ids outside [0, trows)
// are never read (the row is left as is): a bad device index cannot fault; host callers validate
// CPU indices and raise as the reference's gather would.
__global__ void k_add_rows(int R, int D, float* __restrict__ dst, long ldd, const float* __restrict__ table,
                           long ldt, int trows, const int* __restrict__ idx, int idx_mod) {
  const int r = blockIdx.x;
  if (r >= R) return;
  const long t = idx ? idx[r] : (r % idx_mod);
  if (t < 0 || t >= trows) return;
  for (int i = threadIdx.x; i < D; i += blockDim.x) dst[(long)r * ldd + i] += table[t * ldt + i];
}

// ------------------------------------------------------------------------------------------------
// Predictor index build for one (masks_x, masks_y) pair (predictor.py:206-242): per row b, the
// stable rank of every element of cat(mx[b], my[b]) (= torch.argsort for unique ids), written as
//   pos[row0 + b*n + rank]      = id          (RoPE positions of the sorted sequence)
//   ctx_dst[b*K + i]            = row0 + b*n + rank(i)        (where context token i goes)
//   tgt_rows[b*Kp + j]          = row0 + b*n + rank(K + j)    (where target token j sits)
//   loss_rows[b*Kp + j]         = (b % bmod)*N + my[b][j]     (row of the target-encoder output)
// One block per b, ids staged in LDS. The collator's masks are sorted ascending per row
// (multiseq_multiblock3d.py:201-202, argwhere / nonzero), so the rank is a merge-path position:
// rank(mx[i]) = i + #{my < mx[i]}, rank(my[j]) = j + #{mx <= my[j]} (binary searches in LDS, the
// <= keeps argsort's stability: equal ids of masks_x come first). Rows that are not sorted fall back
// to counting ranks over the whole row (O(n^2), same result).
__device__ __forceinline__ int lower_bound_lds(const int* a, int n, int v) {  // #{a < v}
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int upper_bound_lds(const int* a, int n, int v) {  // #{a <= v}
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
__global__ void k_pred_index(int K, int Kp, const long* __restrict__ mx, const long* __restrict__ my, int row0,
                             int bmod, int N, int* __restrict__ pos, int* __restrict__ ctx_dst,
                             int* __restrict__ tgt_rows, int* __restrict__ loss_rows) {
  extern __shared__ int ids[];
  __shared__ int unsorted;
  const int b = blockIdx.x;
  const int n = K + Kp;
  if (threadIdx.x == 0) unsorted = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    ids[i] = (int)(i < K ? mx[(long)b * K + i] : my[(long)b * Kp + (i - K)]);
  __syncthreads();
  bool bad = false;
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    if (i + 1 < n && i + 1 != K && ids[i + 1] < ids[i]) bad = true;
  if (bad) unsorted = 1;
  __syncthreads();
  const bool sorted = unsorted == 0;
  const int* xs = ids;
  const int* ys = ids + K;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int v = ids[i];
    int rank = 0;
    if (sorted) {
      rank = i < K ? i + lower_bound_lds(ys, Kp, v) : (i - K) + upper_bound_lds(xs, K, v);
    } else {
      for (int j = 0; j < n; ++j) {
        const int w = ids[j];
        rank += (w < v) || (w == v && j < i);
      }
    }
    const int dst = row0 + b * n + rank;
    pos[dst] = v;
    if (i < K) ctx_dst[(long)b * K + i] = dst;
    else {
      tgt_rows[(long)b * Kp + (i - K)] = dst;
      if (loss_rows) loss_rows[(long)b * Kp + (i - K)] = (b % bmod) * N + v;
    }
  }
}

// int64 mask [B, K] -> int32 token ids (RoPE positions of a context pass)
__global__ void k_ids64to32(long n, const long* __restrict__ in, int* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int)in[i];
}

// ------------------------------------------------------------------------------------------------
// Fused target normalisation + JEPA L1 loss (+ gradient), wave per predicted row:
//   h   = LN2(LN1(tgt[loss_rows[r]]; gamma, beta, eps1); eps2)     (encoder norm, then F.layer_norm)
//   d   = z[r] - h;  row_loss[r] = w_g * sum |d|^p / p;  dz[r] = w_g * |d|^(p-1) * sign(d)
// with w_g = 1 / (rows_g * D * ngroups) for the mask group g of row r (train.py:425-435).
struct LossGroups {
  int ngroups;
  int rows[4];
  float pair_weight;  // 1 / (number of (fpc, mask) pairs averaged by the loss)
};
template <bool ZBF, bool TBF>
__global__ __launch_bounds__(256) void k_jepa_loss(int R, int D, const void* __restrict__ zp, long ldz,
                                                   const void* __restrict__ tgt, long ldt,
                                                   const int* __restrict__ loss_rows, const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, float eps1, float eps2, float p,
                                                   LossGroups lg, bf16_t* __restrict__ dz, long lddz,
                                                   float* __restrict__ row_loss) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  int g = 0;
  long acc = lg.rows[0];
  while (g < lg.ngroups - 1 && r >= acc) acc += lg.rows[++g];
  const float w = lg.pair_weight / ((float)lg.rows[g] * (float)D);
  const long trow = (long)loss_rows[r] * ldt;
  float4 v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < D) {
      if constexpr (TBF) {  // bf16 target rows (the target encoder's bf16 residual stream)
        const uint2 u = *(const uint2*)((const bf16_t*)tgt + trow + c);
        v[i] = make_float4(bf2f(u.x & 0xffff), bf2f(u.x >> 16), bf2f(u.y & 0xffff), bf2f(u.y >> 16));
      } else {
        v[i] = *(const float4*)((const float*)tgt + trow + c);
      }
      s += v[i].x + v[i].y + v[i].z + v[i].w;
    }
  }
  float mu = wave_sum(s) / D, q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < D) {
      const float a = v[i].x - mu, b = v[i].y - mu, cc = v[i].z - mu, d = v[i].w - mu;
      q += a * a + b * b + cc * cc + d * d;
    }
  }
  float rs = rsqrtf(wave_sum(q) / D + eps1);
  s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < D) {
      const float4 gm = *(const float4*)(gamma + c);
      const float4 bt = *(const float4*)(beta + c);
      v[i] = make_float4((v[i].x - mu) * rs * gm.x + bt.x, (v[i].y - mu) * rs * gm.y + bt.y,
                         (v[i].z - mu) * rs * gm.z + bt.z, (v[i].w - mu) * rs * gm.w + bt.w);
      s += v[i].x + v[i].y + v[i].z + v[i].w;
    }
  }
  mu = wave_sum(s) / D;
  q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < D) {
      const float a = v[i].x - mu, b = v[i].y - mu, cc = v[i].z - mu, d = v[i].w - mu;
      q += a * a + b * b + cc * cc + d * d;
    }
  }
  rs = rsqrtf(wave_sum(q) / D + eps2);
  float lsum = 0.f;
  const bool p1 = (p == 1.f);
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < D) {
      float4 zv;
      if constexpr (ZBF) {
        const uint2 u = *(const uint2*)((const bf16_t*)zp + r * ldz + c);
        zv = make_float4(bf2f(u.x & 0xffff), bf2f(u.x >> 16), bf2f(u.y & 0xffff), bf2f(u.y >> 16));
      } else {
        zv = *(const float4*)((const float*)zp + r * ldz + c);
      }
      const float hv[4] = {(v[i].x - mu) * rs, (v[i].y - mu) * rs, (v[i].z - mu) * rs, (v[i].w - mu) * rs};
      const float zz[4] = {zv.x, zv.y, zv.z, zv.w};
      float gd[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = zz[j] - hv[j];
        const float ad = fabsf(d);
        const float sg = (d > 0.f) ? 1.f : ((d < 0.f) ? -1.f : 0.f);
        if (p1) {
          lsum += ad;
          gd[j] = w * sg;
        } else {
          lsum += powf(ad, p) / p;
          gd[j] = w * powf(ad, p - 1.f) * sg;
        }
      }
      *(uint2*)(dz + r * lddz + c) = make_uint2(pack_bf2(gd[0], gd[1]), pack_bf2(gd[2], gd[3]));
    }
  }
  lsum = wave_sum(lsum);
  if (lane == 0) row_loss[r] = lsum * w;
}

// Deterministic final reduction: out[0] = sum_i in[i] (one block, fixed order).
__global__ void k_sum1(long n, const float* __restrict__ in, float* __restrict__ out) {
  __shared__ float red[256];
  float s = 0.f;
  for (long i = threadIdx.x; i < n; i += 256) s += in[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

// ------------------------------------------------------------------------------------------------
// Optimizer / EMA over flat fp32 arenas (float4 per thread; n % 4 == 0).
__global__ void k_check_finite(long n4, const float4* __restrict__ g, int* __restrict__ found_inf) {
  bool bad = false;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = g[i];
    bad |= !isfinite(v.x) || !isfinite(v.y) || !isfinite(v.z) || !isfinite(v.w);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) *found_inf = 1;
}

struct AdamHP {
  float decay;       // 1 - lr * weight_decay
  float beta1, beta2;
  float one_m_b1, one_m_b2;
  float neg_step;    // -(lr / (1 - beta1^t))
  float bc2_sqrt;    // sqrt(1 - beta2^t)
  float eps;
  float grad_scale;  // gradients are multiplied by this first (1/world for an unaveraged sum)
};
// EMA (optional, t != nullptr): the target encoder's update from the just-updated parameters, fused
// so the online parameters are not read a second time (target <- target * mom + (1 - mom) * p, the
// two roundings of k_ema); on a skipped step (found_inf) the EMA still runs, on the old parameters,
// as train.py:446-465 does after a skipped scaler.step.
__global__ void k_adamw(long n4, float4* __restrict__ p, const float4* __restrict__ g, float4* __restrict__ m,
                        float4* __restrict__ v, uint2* __restrict__ pbf, AdamHP hp, const int* __restrict__ found_inf,
                        float4* __restrict__ t = nullptr, uint2* __restrict__ tbf = nullptr, float mom = 0.f,
                        float one_m = 0.f) {
  const bool skip = found_inf && *found_inf;  // GradScaler.step semantics: skip the update on inf/NaN
  if (skip && !t) return;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float pp[4];
    *(float4*)pp = p[i];
    if (!skip) {
      float gg[4], mm[4], vv[4];
      *(float4*)gg = g[i];
      *(float4*)mm = m[i];
      *(float4*)vv = v[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float gr = gg[j] * hp.grad_scale;
        pp[j] = pp[j] * hp.decay;
        mm[j] = mm[j] + hp.one_m_b1 * (gr - mm[j]);
        vv[j] = vv[j] * hp.beta2;
        vv[j] = vv[j] + hp.one_m_b2 * gr * gr;
        const float den = sqrtf(vv[j]) / hp.bc2_sqrt + hp.eps;
        pp[j] = pp[j] + hp.neg_step * (mm[j] / den);
      }
      p[i] = *(float4*)pp;
      m[i] = *(float4*)mm;
      v[i] = *(float4*)vv;
      if (pbf) pbf[i] = make_uint2(pack_bf2(pp[0], pp[1]), pack_bf2(pp[2], pp[3]));
    }
    if (t) {
      float a[4];
      *(float4*)a = t[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x = a[j] * mom;
        a[j] = x + one_m * pp[j];
      }
      t[i] = *(float4*)a;
      if (tbf) tbf[i] = make_uint2(pack_bf2(a[0], a[1]), pack_bf2(a[2], a[3]));
    }
  }
}

// target <- target * m + (1 - m) * online   (two roundings, as _foreach_mul_ + _foreach_add_)
__global__ void k_ema(long n4, float4* __restrict__ t, const float4* __restrict__ e, float mom, float one_m,
                      uint2* __restrict__ tbf) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float a[4], b[4];
    *(float4*)a = t[i];
    *(float4*)b = e[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x = a[j] * mom;
      a[j] = x + one_m * b[j];
    }
    t[i] = *(float4*)a;
    if (tbf) tbf[i] = make_uint2(pack_bf2(a[0], a[1]), pack_bf2(a[2], a[3]));
  }
}

__global__ void k_cast_bf16(long n4, const float4* __restrict__ in, uint2* __restrict__ out) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = in[i];
    out[i] = make_uint2(pack_bf2(v.x, v.y), pack_bf2(v.z, v.w));
  }
}

// 8 x 8 bf16 block transpose in registers: a[j] = row j (8 bf16 in 4 dwords) -> b[i] = column i.
// b[i] dword k = (a[2k][i], a[2k+1][i]): v_perm_b32 picks the low (i even) or high halves.
__device__ __forceinline__ void transpose8x8(const uint4 (&a)[8], uint4 (&b)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t sel = (i & 1) ? 0x07060302u : 0x05040100u;
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t* lo = (const uint32_t*)&a[2 * k];
      const uint32_t* hi = (const uint32_t*)&a[2 * k + 1];
      w[k] = __builtin_amdgcn_perm(hi[i >> 1], lo[i >> 1], sel);
    }
    b[i] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// One 64 x 64 tile per wave, no LDS: lane (br = lane >> 3, bc = lane & 7) loads the 8 x 8 block at
// rows r0 + 8 br .. + 7, columns c0 + 8 bc .. + 7 (8 x 16 B; the 8 lanes of a block row read one
// 128-B line per row), transposes it in registers and stores rows c0 + 8 bc .. + 7 of dst at columns
// r0 + 8 br .. + 7 (the 8 lanes of a bc read-out again cover 128 contiguous bytes per row).
__device__ __forceinline__ void transpose_tile64(const bf16_t* __restrict__ src, long lds_, bf16_t* __restrict__ dst,
                                                 long ldd, int rows, int cols, int r0, int c0, int lane) {
  const int r = r0 + 8 * (lane >> 3), c = c0 + 8 * (lane & 7);
  if (r >= rows || c >= cols) return;  // rows, cols are multiples of 8: a block is whole or absent
  uint4 a[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = *(const uint4*)(src + (long)(r + j) * lds_ + c);
  transpose8x8(a, b);
#pragma unroll
  for (int i = 0; i < 8; ++i) *(uint4*)(dst + (long)(c + i) * ldd + r) = b[i];
}

// Batched transpose of many weights in one launch (the per-step W^T copies of the data-gradient
// GEMMs): desc[i] = {src, dst, rows, cols, ld_src, ld_dst, first tile, tiles across} (int64 each),
// tiles of 64 x 64 numbered consecutively over the batch; a wave finds its matrix by binary search.
__global__ __launch_bounds__(256) void k_transpose_bf16_batch(const long* __restrict__ desc, int n, long total) {
  const int lane = threadIdx.x & 63;
  for (long t = (long)blockIdx.x * 4 + (threadIdx.x >> 6); t < total; t += (long)gridDim.x * 4) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {  // last i with desc[i].first <= t
      const int mid = (lo + hi + 1) >> 1;
      if (desc[mid * 8 + 6] <= t) lo = mid;
      else hi = mid - 1;
    }
    const long* d = desc + lo * 8;
    const long loc = t - d[6];
    const int tx = (int)d[7];
    const int by = (int)(loc / tx), bx = (int)(loc - (long)by * tx);
    transpose_tile64((const bf16_t*)d[0], d[4], (bf16_t*)d[1], d[5], (int)d[2], (int)d[3], by * 64, bx * 64, lane);
  }
}

// bf16 transpose dst[c][r] = src[r][c]: 4 waves per block, one 64 x 64 tile per wave (tiles along
// the columns: block x covers column tiles 4 x .. 4 x + 3)
__global__ __launch_bounds__(256) void k_transpose_bf16(int rows, int cols, const bf16_t* __restrict__ src, long lds_,
                                                        bf16_t* __restrict__ dst, long ldd) {
  const int tx = blockIdx.x * 4 + (threadIdx.x >> 6);
  transpose_tile64(src, lds_, dst, ldd, rows, cols, blockIdx.y * 64, tx * 64, threadIdx.x & 63);
}

inline int grid_stride_blocks(long n4) {
  long b = (n4 + 255) / 256;
  return (int)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

}  // namespace

static int ln_nv(int D) {  // float4 per lane for a row of D floats (templated register footprint)
  const int v = (D + 255) / 256;
  return v <= 1 ? 1 : v <= 2 ? 2 : v <= 4 ? 4 : v <= 6 ? 6 : 8;
}

extern "C" int vj_layernorm_fwd(int M, int D, const void* x, int x_bf16, long ldx, const float* gamma,
                                const float* beta, float eps, void* y, int y_f32, long ldy, float* mean, float* rstd,
                                void* stream) {
  if (M == 0) return VJ_OK;
  VJ_CHECK_ARG(D % 4 == 0 && D <= 64 * 4 * LN_MAXV, "vj_layernorm_fwd: D=%d must be %%4 and <= 2048", D);
  VJ_CHECK_ARG((gamma == nullptr) == (beta == nullptr), "vj_layernorm_fwd: gamma/beta both or neither");
  VJ_CHECK_ARG(ldx % 4 == 0 && ldy % 4 == 0, "vj_layernorm_fwd: strides must be %%4");
  hipStream_t st = (hipStream_t)stream;
  // k_ln_fwd3 (all rows of a wave in flight, 16-B accesses) for bf16 inputs where the row fits its
  // register budget and the strides allow 16-B vectors; else the one-row-lookahead k_ln_fwd.
  // Measured (profiles/r04_ln_fwd_kernels.txt): bf16 target rows 42.3 -> 37.6 us, but f32 rows (the
  // training path's residual stream) 18.0 -> 20.4 / 27.9 -> 31.2 us, so f32 inputs keep k_ln_fwd.
  // VJ_LN_FWD=1 forces k_ln_fwd, 3 forces k_ln_fwd3 where it applies (A/B). (Round 3's persistent
  // 16-B variant k_ln_fwd2 measured slower than k_ln_fwd and was removed.)
  const int E = x_bf16 ? 8 : 4;
  const int nv3 = (D + 64 * E - 1) / (64 * E);
  const char* e = getenv("VJ_LN_FWD");
  const bool v3 = !(e && e[0] == '1') && (x_bf16 || (e && e[0] == '3')) && D % E == 0 && ldx % E == 0 && ldy % (y_f32 ? 4 : E) == 0 && nv3 <= 4 &&
                  !((uintptr_t)x & 15) && !((uintptr_t)y & 15) && !((uintptr_t)gamma & 15) && !((uintptr_t)beta & 15);
  if (v3) {
    constexpr int R = 4;
    dim3 grid((M + 4 * R - 1) / (4 * R));
#define LNF(XB, YF, NVV) hipLaunchKernelGGL((k_ln_fwd3<XB, YF, NVV, R>), grid, dim3(256), 0, st, M, D, x, ldx, gamma, beta, eps, y, ldy, mean, rstd)
#define LNF_NV(XB, YF) switch (nv3) { case 1: LNF(XB, YF, 1); break; case 2: LNF(XB, YF, 2); break; case 3: LNF(XB, YF, 3); break; default: LNF(XB, YF, 4); }
    if (x_bf16 && y_f32) { LNF_NV(true, true) }
    else if (x_bf16) { LNF_NV(true, false) }
    else if (y_f32) { LNF_NV(false, true) }
    else { LNF_NV(false, false) }
#undef LNF_NV
#undef LNF
    VJ_LAUNCH_CHECK("vj_layernorm_fwd");
    return VJ_OK;
  }
  dim3 grid((M + 4 * LN_RPW - 1) / (4 * LN_RPW));
  const int nv = ln_nv(D);
#define LNF(XB, YF, NVV) hipLaunchKernelGGL((k_ln_fwd<XB, YF, NVV>), grid, dim3(256), 0, st, M, D, x, ldx, gamma, beta, eps, y, ldy, mean, rstd)
#define LNF_NV(XB, YF) switch (nv) { case 1: LNF(XB, YF, 1); break; case 2: LNF(XB, YF, 2); break; case 4: LNF(XB, YF, 4); break; case 6: LNF(XB, YF, 6); break; default: LNF(XB, YF, 8); }
  if (x_bf16 && y_f32) { LNF_NV(true, true) }
  else if (x_bf16) { LNF_NV(true, false) }
  else if (y_f32) { LNF_NV(false, true) }
  else { LNF_NV(false, false) }
#undef LNF_NV
#undef LNF
  VJ_LAUNCH_CHECK("vj_layernorm_fwd");
  return VJ_OK;
}

extern "C" int vj_layernorm_bwd_blocks(int M) {
  const int b = (M + 3) / 4;
  return b < 1024 ? (b > 0 ? b : 1) : 1024;
}

extern "C" int vj_colsum_f32(int M, int N, const void* x, int x_bf16, long ld, float* out, int accumulate,
                             float* ws, long ws_floats, void* stream);

extern "C" int vj_layernorm_bwd(int M, int D, const void* dy, long lddy, const float* x, long ldx, const float* mean,
                                const float* rstd, const float* gamma, const float* dres_in, long ldri, float* dres,
                                long ldr, void* dres_bf16, long ldrb, float* dgamma, float* dbeta, float* sum_in,
                                float* sum_out, float* ws, long ws_floats, void* stream) {
  if (M == 0) return VJ_OK;
  VJ_CHECK_ARG(D % 4 == 0 && D <= 64 * 4 * LN_MAXV, "vj_layernorm_bwd: bad D=%d", D);
  VJ_CHECK_ARG(!sum_in || dres_in, "vj_layernorm_bwd: sum_in needs dres_in");
  const int nb = vj_layernorm_bwd_blocks(M);
  const bool want_sums = sum_in || sum_out;
  const int nsum = want_sums ? 4 : ((dgamma || dbeta) ? 2 : 0);
  if (nsum) {
    VJ_CHECK_ARG(ws && ws_floats >= (long)nb * nsum * D, "vj_layernorm_bwd: workspace needs %ld floats",
                 (long)nb * nsum * D);
  }
  hipStream_t st = (hipStream_t)stream;
  float* part = nsum ? ws : nullptr;
  // k_ln_bwd2 (16-B accesses); k_ln_bwd for strides that do not allow 16-B vectors
  const bool v2 = D % 8 == 0 && lddy % 8 == 0 && ldx % 4 == 0 && ldr % 4 == 0 &&
                  (!dres_in || ldri % 4 == 0) && (!dres_bf16 || ldrb % 8 == 0) && D <= 2048;
  int nbl = nb;  // blocks launched (<= nb: the workspace sizing of vj_layernorm_bwd_blocks)
  if (v2) {  // 16-B accesses (8 columns per lane-vector); a grid every CU holds at once (3 blocks)
    const int nv8 = (D + 511) / 512;
    nbl = nb < 768 ? nb : 768;
    const int nb = nbl;
#define LNB(AC, NVV) do { if (nsum == 4) hipLaunchKernelGGL((k_ln_bwd2<AC, NVV, true>), dim3(nb), dim3(256), 0, st, M, D, (const bf16_t*)dy, lddy, (const void*)x, ldx, mean, rstd, gamma, (const void*)dres_in, ldri, dres, ldr, (bf16_t*)dres_bf16, ldrb, part, nsum); else hipLaunchKernelGGL((k_ln_bwd2<AC, NVV, false>), dim3(nb), dim3(256), 0, st, M, D, (const bf16_t*)dy, lddy, (const void*)x, ldx, mean, rstd, gamma, (const void*)dres_in, ldri, dres, ldr, (bf16_t*)dres_bf16, ldrb, part, nsum); } while (0)
#define LNB_NV(AC) switch (nv8) { case 1: LNB(AC, 1); break; case 2: LNB(AC, 2); break; case 3: LNB(AC, 3); break; default: LNB(AC, 4); }
    if (dres_in) { LNB_NV(true) }
    else { LNB_NV(false) }
#undef LNB_NV
#undef LNB
  } else {
    const int nv = ln_nv(D);
#define LNB(AC, NVV) hipLaunchKernelGGL((k_ln_bwd<AC, NVV>), dim3(nb), dim3(256), 0, st, M, D, (const bf16_t*)dy, lddy, x, ldx, mean, rstd, gamma, dres_in, ldri, dres, ldr, (bf16_t*)dres_bf16, ldrb, part, nsum)
#define LNB_NV(AC) switch (nv) { case 1: LNB(AC, 1); break; case 2: LNB(AC, 2); break; case 4: LNB(AC, 4); break; case 6: LNB(AC, 6); break; default: LNB(AC, 8); }
    if (dres_in) { LNB_NV(true) }
    else { LNB_NV(false) }
#undef LNB_NV
#undef LNB
  }
  VJ_LAUNCH_CHECK("vj_layernorm_bwd");
  // partials laid out [nb][nsum][D]: column k sums over rows of stride nsum*D
  if (nsum) {  // every requested vector in one launch (same fixed-order sums as one launch each)
    ColsumOuts o{{dgamma, dbeta, nsum > 2 ? sum_in : nullptr, nsum > 2 ? sum_out : nullptr}};
    hipLaunchKernelGGL(k_colsum2_multi, dim3((D + 31) / 32, nsum), dim3(1024), 0, st, nbl, D, ws, (long)nsum * D, o);
  }
  VJ_LAUNCH_CHECK("vj_layernorm_bwd(reduce)");
  return VJ_OK;
}

// GELU and GELU' of bf16 inputs by the GEMM epilogues' exact evaluation (gelu_fwd_grad): the reference
// the table epilogue of the fc1 GEMM is checked against, bitwise, over every bf16 input.
namespace {
__global__ __launch_bounds__(256) void k_gelu_eval(int n, const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                   bf16_t* __restrict__ dy) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float a, d;
  gelu_fwd_grad(bf2f(x[i]), a, d);
  y[i] = f2bf(a);
  dy[i] = f2bf(d);
}
}  // namespace

extern "C" int vj_gelu_eval(int n, const void* x, void* y, void* dy, void* stream) {
  if (n == 0) return VJ_OK;
  VJ_CHECK_ARG(n > 0 && x && y && dy, "vj_gelu_eval: bad arguments");
  hipLaunchKernelGGL(k_gelu_eval, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, (const bf16_t*)x,
                     (bf16_t*)y, (bf16_t*)dy);
  VJ_LAUNCH_CHECK("vj_gelu_eval");
  return VJ_OK;
}

// LayerNorm backward on the bf16 residual stream (the trained context encoder under bf16 autocast,
// app/vjepa/train.py:437-439: x = x + attn(norm1(x)) is a bf16 add there, modules.py:561-562): x and
// dres_in bf16 rows, dres = dres_in + dLN/dx (f32 math) written once as bf16. Same fixed-order column
// partials (dgamma, dbeta, sums of dres_in / dres) as vj_layernorm_bwd.
extern "C" int vj_layernorm_bwd_bf16(int M, int D, const void* dy, long lddy, const void* x, long ldx,
                                     const float* mean, const float* rstd, const float* gamma, const void* dres_in,
                                     long ldri, void* dres, long ldr, float* dgamma, float* dbeta, float* sum_in,
                                     float* sum_out, float* ws, long ws_floats, void* stream) {
  if (M == 0) return VJ_OK;
  VJ_CHECK_ARG(D % 8 == 0 && D <= 2048, "vj_layernorm_bwd_bf16: D=%d must be %%8 and <= 2048", D);
  VJ_CHECK_ARG(lddy % 8 == 0 && ldx % 8 == 0 && ldr % 8 == 0 && (!dres_in || ldri % 8 == 0),
               "vj_layernorm_bwd_bf16: strides must be multiples of 8");
  VJ_CHECK_ARG(!(((uintptr_t)dy | (uintptr_t)x | (uintptr_t)dres | (uintptr_t)dres_in) & 15),
               "vj_layernorm_bwd_bf16: rows must be 16-B aligned");
  VJ_CHECK_ARG(dy && x && mean && rstd && dres, "vj_layernorm_bwd_bf16: null operand");
  VJ_CHECK_ARG(!sum_in || dres_in, "vj_layernorm_bwd_bf16: sum_in needs dres_in");
  const int nb = vj_layernorm_bwd_blocks(M);
  const int nsum = (sum_in || sum_out) ? 4 : ((dgamma || dbeta) ? 2 : 0);
  if (nsum) {
    VJ_CHECK_ARG(ws && ws_floats >= (long)nb * nsum * D, "vj_layernorm_bwd_bf16: workspace needs %ld floats",
                 (long)nb * nsum * D);
  }
  hipStream_t st = (hipStream_t)stream;
  float* part = nsum ? ws : nullptr;
  const int nv8 = (D + 511) / 512;
  const int nbl = nb < 768 ? nb : 768;
#define LNB(AC, NVV) do { if (nsum == 4) hipLaunchKernelGGL((k_ln_bwd2<AC, NVV, true, true>), dim3(nbl), dim3(256), 0, st, M, D, (const bf16_t*)dy, lddy, x, ldx, mean, rstd, gamma, dres_in, ldri, nullptr, 0L, (bf16_t*)dres, ldr, part, nsum); else hipLaunchKernelGGL((k_ln_bwd2<AC, NVV, false, true>), dim3(nbl), dim3(256), 0, st, M, D, (const bf16_t*)dy, lddy, x, ldx, mean, rstd, gamma, dres_in, ldri, nullptr, 0L, (bf16_t*)dres, ldr, part, nsum); } while (0)
#define LNB_NV(AC) switch (nv8) { case 1: LNB(AC, 1); break; case 2: LNB(AC, 2); break; case 3: LNB(AC, 3); break; default: LNB(AC, 4); }
  if (dres_in) { LNB_NV(true) }
  else { LNB_NV(false) }
#undef LNB_NV
#undef LNB
  VJ_LAUNCH_CHECK("vj_layernorm_bwd_bf16");
  if (nsum) {
    ColsumOuts o{{dgamma, dbeta, nsum > 2 ? sum_in : nullptr, nsum > 2 ? sum_out : nullptr}};
    hipLaunchKernelGGL(k_colsum2_multi, dim3((D + 31) / 32, nsum), dim3(1024), 0, st, nbl, D, ws, (long)nsum * D, o);
  }
  VJ_LAUNCH_CHECK("vj_layernorm_bwd_bf16(reduce)");
  return VJ_OK;
}

extern "C" int vj_colsum_f32(int M, int N, const void* x, int x_bf16, long ld, float* out, int accumulate, float* ws,
                             long ws_floats, void* stream) {
  if (N == 0) return VJ_OK;
  VJ_CHECK_ARG(N % 8 == 0 && ld % 8 == 0, "vj_colsum_f32: N and ld must be multiples of 8");
  int S = (M + 63) / 64;
  if (S > 256) S = 256;
  if (S < 1) S = 1;
  VJ_CHECK_ARG(ws && ws_floats >= (long)S * N, "vj_colsum_f32: workspace needs %ld floats", (long)S * N);
  const int rps = (M + S - 1) / S;
  hipStream_t st = (hipStream_t)stream;
  dim3 g1((N + 511) / 512, S);
  if (x_bf16) hipLaunchKernelGGL(k_colsum1<true>, g1, dim3(256), 0, st, M, N, x, ld, rps, ws);
  else hipLaunchKernelGGL(k_colsum1<false>, g1, dim3(256), 0, st, M, N, x, ld, rps, ws);
  hipLaunchKernelGGL(k_colsum2, dim3((N + 31) / 32), dim3(1024), 0, st, S, N, ws, (long)N, out, nullptr, N, accumulate);
  VJ_LAUNCH_CHECK("vj_colsum_f32");
  return VJ_OK;
}

extern "C" int vj_rope(int T, int H, int hd, void* qkv, long ld, int q_off, int k_off, const int* ids, int ids_mod,
                       int tokens_per_frame, int tokens_per_row, const float* cos_tab, const float* sin_tab, int half,
                       int inverse, void* stream) {
  if (T == 0) return VJ_OK;
  VJ_CHECK_ARG(hd % 8 == 0 && ld % 8 == 0 && q_off % 8 == 0 && k_off % 8 == 0, "vj_rope: alignment");
  VJ_CHECK_ARG(half == (hd / 3) / 2 && half >= 1, "vj_rope: half=%d inconsistent with hd=%d", half, hd);
  VJ_CHECK_ARG(ids || ids_mod > 0, "vj_rope: ids or ids_mod required");
  const long total = (long)T * 2 * H * (hd / 8);
  hipLaunchKernelGGL(k_rope<false>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, T, H,
                     hd, qkv, ld, q_off, k_off, ids, ids_mod, tokens_per_frame, tokens_per_row, cos_tab, sin_tab, half,
                     inverse);
  VJ_LAUNCH_CHECK("vj_rope");
  return VJ_OK;
}

// vj_rope on an f32 qkv buffer (fp32-operand parity mode); same arguments, ld / offsets in floats.
extern "C" int vj_rope_f32(int T, int H, int hd, float* qkv, long ld, int q_off, int k_off, const int* ids,
                           int ids_mod, int tokens_per_frame, int tokens_per_row, const float* cos_tab,
                           const float* sin_tab, int half, void* stream) {
  if (T == 0) return VJ_OK;
  VJ_CHECK_ARG(hd % 8 == 0 && ld % 4 == 0 && q_off % 4 == 0 && k_off % 4 == 0, "vj_rope_f32: alignment");
  VJ_CHECK_ARG(half == (hd / 3) / 2 && half >= 1, "vj_rope_f32: half=%d inconsistent with hd=%d", half, hd);
  VJ_CHECK_ARG(ids || ids_mod > 0, "vj_rope_f32: ids or ids_mod required");
  const long total = (long)T * 2 * H * (hd / 8);
  hipLaunchKernelGGL(k_rope<true>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, T, H,
                     hd, (void*)qkv, ld, q_off, k_off, ids, ids_mod, tokens_per_frame, tokens_per_row, cos_tab,
                     sin_tab, half, 0);
  VJ_LAUNCH_CHECK("vj_rope_f32");
  return VJ_OK;
}

extern "C" int vj_im2col_tubelet(int R, int K, const long* idx, int B, int C, int Tf, int Hf, int Wf, int tub, int pch,
                                 const float* clip, void* out, void* stream) {
  if (R == 0) return VJ_OK;
  VJ_CHECK_ARG(pch % 4 == 0 && Tf % tub == 0 && Hf % pch == 0 && Wf % pch == 0, "vj_im2col_tubelet: bad geometry");
  VJ_CHECK_ARG(R <= (long)B * K, "vj_im2col_tubelet: R=%d > B*K", R);
  hipLaunchKernelGGL(k_im2col<false>, dim3(R), dim3(256), 0, (hipStream_t)stream, R, K, idx, C, Tf, Hf, Wf, tub, pch,
                     clip, out);
  VJ_LAUNCH_CHECK("vj_im2col_tubelet");
  return VJ_OK;
}

// vj_im2col_tubelet with f32 rows (fp32-operand parity mode)
extern "C" int vj_im2col_tubelet_f32(int R, int K, const long* idx, int B, int C, int Tf, int Hf, int Wf, int tub,
                                     int pch, const float* clip, float* out, void* stream) {
  if (R == 0) return VJ_OK;
  VJ_CHECK_ARG(pch % 4 == 0 && Tf % tub == 0 && Hf % pch == 0 && Wf % pch == 0, "vj_im2col_tubelet_f32: bad geometry");
  VJ_CHECK_ARG(R <= (long)B * K, "vj_im2col_tubelet_f32: R=%d > B*K", R);
  hipLaunchKernelGGL(k_im2col<true>, dim3(R), dim3(256), 0, (hipStream_t)stream, R, K, idx, C, Tf, Hf, Wf, tub, pch,
                     clip, (void*)out);
  VJ_LAUNCH_CHECK("vj_im2col_tubelet_f32");
  return VJ_OK;
}

extern "C" int vj_gather_rows(int R, int rowbytes, const void* src, long src_ld_bytes, const int* idx, void* dst,
                              long dst_ld_bytes, int scatter, void* stream) {
  if (R == 0) return VJ_OK;
  VJ_CHECK_ARG(rowbytes % 16 == 0 && src_ld_bytes % 16 == 0 && dst_ld_bytes % 16 == 0, "vj_gather_rows: 16-B rows");
  hipLaunchKernelGGL(k_gather_rows, dim3(R), dim3(64), 0, (hipStream_t)stream, R, rowbytes, (const char*)src,
                     src_ld_bytes, idx, (char*)dst, dst_ld_bytes, scatter);
  VJ_LAUNCH_CHECK("vj_gather_rows");
  return VJ_OK;
}

extern "C" int vj_fill_rows(int R, int D, float* dst, long ldd, const int* idx, const float* vec, void* stream) {
  if (R == 0) return VJ_OK;
  hipLaunchKernelGGL(k_fill_rows, dim3(R), dim3(128), 0, (hipStream_t)stream, R, D, dst, ldd, idx, vec);
  VJ_LAUNCH_CHECK("vj_fill_rows");
  return VJ_OK;
}

extern "C" int vj_add_rows(int R, int D, float* dst, long ldd, const float* table, long ldt, int trows,
                           const int* idx, int idx_mod, void* stream) {
  if (R == 0) return VJ_OK;
  VJ_CHECK_ARG(idx || idx_mod > 0, "vj_add_rows: idx or idx_mod");
  VJ_CHECK_ARG(trows > 0 && (idx || idx_mod <= trows), "vj_add_rows: idx_mod %d exceeds the table's %d rows", idx_mod,
               trows);
  hipLaunchKernelGGL(k_add_rows, dim3(R), dim3(128), 0, (hipStream_t)stream, R, D, dst, ldd, table, ldt, trows, idx,
                     idx_mod);
  VJ_LAUNCH_CHECK("vj_add_rows");
  return VJ_OK;
}

extern "C" int vj_pred_index(int B, int K, int Kp, const long* mx, const long* my, int row0, int bmod, int N, int* pos,
                             int* ctx_dst, int* tgt_rows, int* loss_rows, void* stream) {
  if (B == 0) return VJ_OK;
  const int n = K + Kp;
  VJ_CHECK_ARG(n >= 1 && n <= 16384, "vj_pred_index: sequence length %d out of range", n);
  hipLaunchKernelGGL(k_pred_index, dim3(B), dim3(256), n * sizeof(int), (hipStream_t)stream, K, Kp, mx, my, row0,
                     bmod > 0 ? bmod : B, N, pos, ctx_dst, tgt_rows, loss_rows);
  VJ_LAUNCH_CHECK("vj_pred_index");
  return VJ_OK;
}

extern "C" int vj_ids64to32(long n, const long* in, int* out, void* stream) {
  if (n == 0) return VJ_OK;
  hipLaunchKernelGGL(k_ids64to32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n, in, out);
  VJ_LAUNCH_CHECK("vj_ids64to32");
  return VJ_OK;
}

extern "C" int vj_jepa_loss(int R, int D, const void* z, int z_bf16, long ldz, const void* tgt, int tgt_bf16, long ldt,
                            const int* loss_rows, const float* gamma, const float* beta, float eps1, float eps2,
                            float loss_exp, int ngroups, const int* group_rows, float pair_weight, void* dz, long lddz,
                            float* row_loss, float* loss_out, void* stream) {
  if (R == 0) return VJ_OK;
  VJ_CHECK_ARG(D % 4 == 0 && D <= 2048, "vj_jepa_loss: bad D=%d", D);
  VJ_CHECK_ARG(ngroups >= 1 && ngroups <= 4, "vj_jepa_loss: 1..4 groups");
  LossGroups lg{};
  lg.ngroups = ngroups;
  lg.pair_weight = pair_weight;
  long tot = 0;
  for (int i = 0; i < ngroups; ++i) {
    lg.rows[i] = group_rows[i];
    tot += group_rows[i];
  }
  VJ_CHECK_ARG(tot == R, "vj_jepa_loss: groups cover %ld rows, R=%d", tot, R);
  hipStream_t st = (hipStream_t)stream;
#define JL(ZB, TB)                                                                                                \
  hipLaunchKernelGGL((k_jepa_loss<ZB, TB>), dim3((R + 3) / 4), dim3(256), 0, st, R, D, z, ldz, tgt, ldt, loss_rows, \
                     gamma, beta, eps1, eps2, loss_exp, lg, (bf16_t*)dz, lddz, row_loss)
  if (z_bf16 && tgt_bf16) JL(true, true);
  else if (z_bf16) JL(true, false);
  else if (tgt_bf16) JL(false, true);
  else JL(false, false);
#undef JL
  hipLaunchKernelGGL(k_sum1, dim3(1), dim3(256), 0, st, (long)R, row_loss, loss_out);
  VJ_LAUNCH_CHECK("vj_jepa_loss");
  return VJ_OK;
}

extern "C" int vj_check_finite(long n, const float* g, int* found_inf, void* stream) {
  if (n == 0) return VJ_OK;
  VJ_CHECK_ARG(n % 4 == 0 && ((uintptr_t)g & 15) == 0, "vj_check_finite: n %% 4 and 16-B alignment");
  const long n4 = n / 4;
  hipLaunchKernelGGL(k_check_finite, dim3(grid_stride_blocks(n4)), dim3(256), 0, (hipStream_t)stream, n4,
                     (const float4*)g, found_inf);
  VJ_LAUNCH_CHECK("vj_check_finite");
  return VJ_OK;
}

static AdamHP adam_hp(float lr, float beta1, float beta2, float eps, float weight_decay, int step, float grad_scale);
extern "C" int vj_adamw_ema(long n, float* p, const float* g, float* m, float* v, void* p_bf16, float lr, float beta1,
                            float beta2, float eps, float weight_decay, int step, float grad_scale, const int* found_inf,
                            float* target, void* target_bf16, float momentum, void* stream);

extern "C" int vj_adamw(long n, float* p, const float* g, float* m, float* v, void* p_bf16, float lr, float beta1,
                        float beta2, float eps, float weight_decay, int step, float grad_scale, const int* found_inf,
                        void* stream) {
  return vj_adamw_ema(n, p, g, m, v, p_bf16, lr, beta1, beta2, eps, weight_decay, step, grad_scale, found_inf, nullptr,
                      nullptr, 0.f, stream);
}

extern "C" int vj_adamw_ema(long n, float* p, const float* g, float* m, float* v, void* p_bf16, float lr, float beta1,
                            float beta2, float eps, float weight_decay, int step, float grad_scale, const int* found_inf,
                            float* target, void* target_bf16, float momentum, void* stream) {
  if (n == 0) return VJ_OK;
  VJ_CHECK_ARG(n % 4 == 0, "vj_adamw: n must be %%4");
  VJ_CHECK_ARG(step >= 1, "vj_adamw: step must be >= 1");
  VJ_CHECK_ARG(target || !target_bf16, "vj_adamw_ema: target_bf16 without target");
  const AdamHP hp = adam_hp(lr, beta1, beta2, eps, weight_decay, step, grad_scale);
  const long n4 = n / 4;
  hipLaunchKernelGGL(k_adamw, dim3(grid_stride_blocks(n4)), dim3(256), 0, (hipStream_t)stream, n4, (float4*)p,
                     (const float4*)g, (float4*)m, (float4*)v, (uint2*)p_bf16, hp, found_inf, (float4*)target,
                     (uint2*)target_bf16, momentum, (float)(1.0 - (double)momentum));
  VJ_LAUNCH_CHECK("vj_adamw");
  return VJ_OK;
}

static AdamHP adam_hp(float lr, float beta1, float beta2, float eps, float weight_decay, int step, float grad_scale) {
  AdamHP hp;
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  hp.decay = (float)(1.0 - (double)lr * (double)weight_decay);
  hp.beta1 = beta1;
  hp.beta2 = beta2;
  hp.one_m_b1 = (float)(1.0 - (double)beta1);
  hp.one_m_b2 = (float)(1.0 - (double)beta2);
  hp.neg_step = (float)(-((double)lr / bc1));
  hp.bc2_sqrt = (float)sqrt(bc2);
  hp.eps = eps;
  hp.grad_scale = grad_scale;
  return hp;
}

extern "C" int vj_ema(long n, float* target, const float* online, float momentum, void* target_bf16, void* stream) {
  if (n == 0) return VJ_OK;
  VJ_CHECK_ARG(n % 4 == 0, "vj_ema: n must be %%4");
  const long n4 = n / 4;
  hipLaunchKernelGGL(k_ema, dim3(grid_stride_blocks(n4)), dim3(256), 0, (hipStream_t)stream, n4, (float4*)target,
                     (const float4*)online, momentum, (float)(1.0 - (double)momentum), (uint2*)target_bf16);
  VJ_LAUNCH_CHECK("vj_ema");
  return VJ_OK;
}

// scalar elements [i0, n) of a cast whose length is not a multiple of 4 (tiny inputs, e.g. 7-wide actions)
__global__ void k_cast_bf16_tail(long i0, long n, const float* __restrict__ in, bf16_t* __restrict__ out) {
  const long i = i0 + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = f2bf(in[i]);
}

extern "C" int vj_cast_bf16(long n, const float* in, void* out, void* stream) {
  if (n == 0) return VJ_OK;
  VJ_CHECK_ARG(in && out, "vj_cast_bf16: null pointer");
  const bool vec = !(((uintptr_t)in & 15) | ((uintptr_t)out & 7));
  const long n4 = vec ? n / 4 : 0;
  if (n4)
    hipLaunchKernelGGL(k_cast_bf16, dim3(grid_stride_blocks(n4)), dim3(256), 0, (hipStream_t)stream, n4,
                       (const float4*)in, (uint2*)out);
  if (n4 * 4 < n)
    hipLaunchKernelGGL(k_cast_bf16_tail, dim3(vj_cdiv(n - n4 * 4, 256)), dim3(256), 0, (hipStream_t)stream, n4 * 4, n,
                       in, (bf16_t*)out);
  VJ_LAUNCH_CHECK("vj_cast_bf16");
  return VJ_OK;
}

extern "C" int vj_transpose_bf16(int rows, int cols, const void* src, long ld_src, void* dst, long ld_dst,
                                 void* stream) {
  if (rows == 0 || cols == 0) return VJ_OK;
  VJ_CHECK_ARG(rows > 0 && cols > 0 && src && dst, "vj_transpose_bf16: bad arguments");
  VJ_CHECK_ARG(rows % 8 == 0 && cols % 8 == 0 && ld_src % 8 == 0 && ld_dst % 8 == 0 && ld_src >= cols &&
                   ld_dst >= rows && !(((uintptr_t)src | (uintptr_t)dst) & 15),
               "vj_transpose_bf16: rows, cols, strides must be multiples of 8 and the pointers 16-B aligned");
  const dim3 grid(vj_cdiv(vj_cdiv(cols, 64), 4), vj_cdiv(rows, 64));
  hipLaunchKernelGGL(k_transpose_bf16, grid, dim3(256), 0, (hipStream_t)stream, rows, cols, (const bf16_t*)src,
                     ld_src, (bf16_t*)dst, ld_dst);
  VJ_LAUNCH_CHECK("vj_transpose_bf16");
  return VJ_OK;
}

// n transposes in one launch. desc: DEVICE array of n x 8 int64 {src, dst, rows, cols, ld_src, ld_dst,
// first_tile, tiles_x} (first_tile = running sum of ceil(rows/64) * ceil(cols/64); tiles_x =
// ceil(cols/64)), built by the caller once per weight set; total_tiles = the sum over all n. Every
// matrix must satisfy vj_transpose_bf16's constraints (checked by the caller when it builds desc).
extern "C" int vj_transpose_bf16_batch(int n, const long* desc, long total_tiles, void* stream) {
  if (n == 0 || total_tiles == 0) return VJ_OK;
  VJ_CHECK_ARG(n > 0 && desc && total_tiles > 0, "vj_transpose_bf16_batch: bad arguments");
  const long blocks = (total_tiles + 3) / 4;
  const dim3 grid((unsigned)(blocks < 16384 ? blocks : 16384));
  hipLaunchKernelGGL(k_transpose_bf16_batch, grid, dim3(256), 0, (hipStream_t)stream, desc, n, total_tiles);
  VJ_LAUNCH_CHECK("vj_transpose_bf16_batch");
  return VJ_OK;
}

extern "C" int vj_layernorm_fwd_fp8(int M, int D, const void* x, int x_bf16, long ldx, const float* gamma,
                                    const float* beta, float eps, void* y8, long ldy, int* yexp, float* mean,
                                    float* rstd, void* stream) {
  if (M == 0) return VJ_OK;
  VJ_CHECK_ARG(D % 4 == 0 && D <= 64 * 4 * LN_MAXV, "vj_layernorm_fwd_fp8: D=%d must be %%4 and <= 2048", D);
  VJ_CHECK_ARG((gamma == nullptr) == (beta == nullptr), "vj_layernorm_fwd_fp8: gamma/beta both or neither");
  VJ_CHECK_ARG(ldx % 4 == 0 && ldy % 16 == 0 && !((uintptr_t)y8 & 15) && yexp,
               "vj_layernorm_fwd_fp8: fp8 rows must be 16-B aligned, exponents required");
  dim3 grid((M + 4 * LN_RPW - 1) / (4 * LN_RPW));
  hipStream_t st = (hipStream_t)stream;
#define LNF8(XB, NVV)                                                                                             \
  hipLaunchKernelGGL((k_ln_fwd<XB, false, NVV, true>), grid, dim3(256), 0, st, M, D, x, ldx, gamma, beta, eps, y8, \
                     ldy, mean, rstd, yexp)
  switch (ln_nv(D)) {
    case 1: if (x_bf16) LNF8(true, 1); else LNF8(false, 1); break;
    case 2: if (x_bf16) LNF8(true, 2); else LNF8(false, 2); break;
    case 4: if (x_bf16) LNF8(true, 4); else LNF8(false, 4); break;
    case 6: if (x_bf16) LNF8(true, 6); else LNF8(false, 6); break;
    default: if (x_bf16) LNF8(true, 8); else LNF8(false, 8);
  }
#undef LNF8
  VJ_LAUNCH_CHECK("vj_layernorm_fwd_fp8");
  return VJ_OK;
}

extern "C" int vj_quant_rows_fp8(int M, int K, const void* x, int x_bf16, long ldx, void* y8, long ldy, int* yexp,
                                 void* stream) {
  if (M == 0) return VJ_OK;
  VJ_CHECK_ARG(K > 0 && K % 4 == 0 && ldx % 4 == 0 && ldy % 16 == 0 && ldy >= K && x && y8 && yexp,
               "vj_quant_rows_fp8: K %% 4, ldy %% 16 and non-null operands required");
  VJ_CHECK_ARG(!((uintptr_t)y8 & 15) && !((uintptr_t)x & 15), "vj_quant_rows_fp8: 16-B aligned rows");
  const dim3 grid((M + 3) / 4);
  if (x_bf16)
    hipLaunchKernelGGL(k_quant_rows_fp8<true>, grid, dim3(256), 0, (hipStream_t)stream, M, K, x, ldx,
                       (unsigned char*)y8, ldy, yexp);
  else
    hipLaunchKernelGGL(k_quant_rows_fp8<false>, grid, dim3(256), 0, (hipStream_t)stream, M, K, x, ldx,
                       (unsigned char*)y8, ldy, yexp);
  VJ_LAUNCH_CHECK("vj_quant_rows_fp8");
  return VJ_OK;
}

// ------------------------------------------------------------------------------------------------
// JEPA multi-block 3-D masks on the device (src/masks/multiseq_multiblock3d.py:155-239). The host
// draws the block size and positions with the reference's RNG calls (they define the stream) and
// rejects empty contexts as it draws; the device builds every sample's context / target id lists:
// token (f, r, c) is KEPT unless it lies in one of the npred blocks [start, start+t) x [top, top+h)
// x [left, left+w) or f >= max_ctx (the context frame limit, :165-169). Lists are ascending (the
// torch.nonzero / argwhere order), truncated to the batch minimum (:210-215) and written as the
// int64 [B, K] tensors the step consumes.
namespace {

constexpr int MASK_THREADS = 256;

__device__ __forceinline__ bool mask_kept(int tok, int HW, int W, int npred, const int* __restrict__ box, int t, int h,
                                          int w, int max_ctx) {
  const int f = tok / HW, rem = tok - f * HW, r = rem / W, c = rem - r * W;
  if (f >= max_ctx) return false;
  for (int j = 0; j < npred; ++j) {
    const int s = box[3 * j], tp = box[3 * j + 1], lf = box[3 * j + 2];
    if (f >= s && f < s + t && r >= tp && r < tp + h && c >= lf && c < lf + w) return false;
  }
  return true;
}

// exclusive block scan of one int per thread (MASK_THREADS threads)
__device__ __forceinline__ int mask_scan(int v, int* sh, int& total) {
  const int tid = threadIdx.x;
  sh[tid] = v;
  __syncthreads();
  for (int o = 1; o < MASK_THREADS; o <<= 1) {
    const int x = tid >= o ? sh[tid - o] : 0;
    __syncthreads();
    sh[tid] += x;
    __syncthreads();
  }
  total = sh[MASK_THREADS - 1];
  const int excl = sh[tid] - v;
  __syncthreads();
  return excl;
}

// per-sample number of kept tokens
__global__ __launch_bounds__(MASK_THREADS) void k_mask_count(int N, int HW, int W, int npred, const int* __restrict__ boxes,
                                                              int t, int h, int w, int max_ctx, int* __restrict__ counts) {
  __shared__ int sh[MASK_THREADS];
  const int b = blockIdx.x;
  const int* box = boxes + (long)b * npred * 3;
  int n = 0;
  for (int tok = threadIdx.x; tok < N; tok += MASK_THREADS) n += mask_kept(tok, HW, W, npred, box, t, h, w, max_ctx);
  int total;
  mask_scan(n, sh, total);
  if (threadIdx.x == 0) counts[b] = total;
}

// mode 0: enc = first k_enc kept ids, pred = first k_pred masked ids; 1 (full_complement): pred =
// complement of enc; 2 (pred_full_complement): enc = complement of pred. Each thread owns a
// contiguous token chunk, so the block scan of chunk counts yields ascending output order.
__global__ __launch_bounds__(MASK_THREADS) void k_mask_emit(int N, int HW, int W, int npred, const int* __restrict__ boxes,
                                                             int t, int h, int w, int max_ctx, int mode, int k_enc,
                                                             int k_pred, long* __restrict__ enc, long* __restrict__ pred) {
  __shared__ int sh[MASK_THREADS];
  const int b = blockIdx.x;
  const int* box = boxes + (long)b * npred * 3;
  const int per = (N + MASK_THREADS - 1) / MASK_THREADS;
  const int t0 = threadIdx.x * per, t1 = min(N, t0 + per);
  int nk = 0;
  for (int tok = t0; tok < t1; ++tok) nk += mask_kept(tok, HW, W, npred, box, t, h, w, max_ctx);
  int tot_k;
  const int rk = mask_scan(nk, sh, tot_k);  // kept ids before this chunk
  const int rm = t0 - rk;                   // masked ids before this chunk
  // ranks among the emitted lists: enc keeps kept ids with rank < k_enc (mode 0 / 1) or everything
  // outside pred[:k_pred] (mode 2); pred symmetric
  int ne = 0, np = 0;
  {
    int ik = rk, im = rm;
    for (int tok = t0; tok < t1; ++tok) {
      const bool kept = mask_kept(tok, HW, W, npred, box, t, h, w, max_ctx);
      const bool in_enc = mode == 2 ? !(!kept && im < k_pred) : (kept && ik < k_enc);
      const bool in_pred = mode == 1 ? !(kept && ik < k_enc) : (!kept && im < k_pred);
      ne += in_enc;
      np += in_pred;
      ik += kept;
      im += !kept;
    }
  }
  int tot_e, tot_p;
  int oe = mask_scan(ne, sh, tot_e);
  int op = mask_scan(np, sh, tot_p);
  long* erow = enc + (long)b * (mode == 2 ? N - k_pred : k_enc);
  long* prow = pred + (long)b * (mode == 1 ? N - k_enc : k_pred);
  int ik = rk, im = rm;
  for (int tok = t0; tok < t1; ++tok) {
    const bool kept = mask_kept(tok, HW, W, npred, box, t, h, w, max_ctx);
    const bool in_enc = mode == 2 ? !(!kept && im < k_pred) : (kept && ik < k_enc);
    const bool in_pred = mode == 1 ? !(kept && ik < k_enc) : (!kept && im < k_pred);
    if (in_enc) erow[oe++] = tok;
    if (in_pred) prow[op++] = tok;
    ik += kept;
    im += !kept;
  }
}

}  // namespace

extern "C" int vj_mask_count(int B, int duration, int height, int width, int npred, const int* boxes, int t, int h,
                             int w, int max_ctx, int* counts, void* stream) {
  if (B == 0) return VJ_OK;
  VJ_CHECK_ARG(B > 0 && duration > 0 && height > 0 && width > 0 && npred >= 1 && boxes && counts,
               "vj_mask_count: bad arguments");
  const int N = duration * height * width;
  hipLaunchKernelGGL(k_mask_count, dim3(B), dim3(MASK_THREADS), 0, (hipStream_t)stream, N, height * width, width, npred,
                     boxes, t, h, w, max_ctx, counts);
  VJ_LAUNCH_CHECK("vj_mask_count");
  return VJ_OK;
}

extern "C" int vj_mask_emit(int B, int duration, int height, int width, int npred, const int* boxes, int t, int h,
                            int w, int max_ctx, int mode, int k_enc, int k_pred, long* enc, long* pred, void* stream) {
  if (B == 0) return VJ_OK;
  const int N = duration * height * width;
  VJ_CHECK_ARG(B > 0 && N > 0 && npred >= 1 && boxes && enc && pred && mode >= 0 && mode <= 2,
               "vj_mask_emit: bad arguments");
  VJ_CHECK_ARG(k_enc >= 0 && k_enc <= N && k_pred >= 0 && k_pred <= N, "vj_mask_emit: bad lengths");
  hipLaunchKernelGGL(k_mask_emit, dim3(B), dim3(MASK_THREADS), 0, (hipStream_t)stream, N, height * width, width, npred,
                     boxes, t, h, w, max_ctx, mode, k_enc, k_pred, enc, pred);
  VJ_LAUNCH_CHECK("vj_mask_emit");
  return VJ_OK;
}

// ------------------------------------------------------------------------------------------------
// Video clip transform (app/vjepa/transforms.py:37-116, VideoTransform without auto-augment /
// motion shift / random erasing): uint8 frames [B][T][H][W][C] -> f32 clips [B][C][T][S][S] =
// normalize(hflip(bilinear_resize(crop))). The crop box and the flip come from the host's draws
// (the reference's RNG calls, video/transforms.py:470-507 and :149-180); the resize is
// F.interpolate(mode="bilinear", align_corners=False) (:537-542) with ATen's source-index rule
// src = max((dst + 0.5) * in / out - 0.5, 0), idx1 = idx0 + (idx0 < in - 1), lambdas in f32; the
// normalisation is (x - 255 mean_c) / (255 std_c) (:139-152). One thread per output element.
namespace {

__global__ void k_video_transform(long total, int T, int H, int W, int C, int S, const unsigned char* __restrict__ frames,
                                  const int* __restrict__ params, const float* __restrict__ mean,
                                  const float* __restrict__ stdv, float* __restrict__ out) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int x = (int)(e % S);
  long r = e / S;
  const int y = (int)(r % S);
  r /= S;
  const int t = (int)(r % T);
  r /= T;
  const int c = (int)(r % C);
  const int b = (int)(r / C);
  const int* p = params + 5 * b;  // top, left, height, width, flip
  const int ci = p[0], cj = p[1], ch = p[2], cw = p[3];
  const int xs = p[4] ? S - 1 - x : x;  // flip after the resize: read the mirrored output column
  const float sh = (float)ch / (float)S, sw = (float)cw / (float)S;
  const float fy = fmaxf(sh * ((float)y + 0.5f) - 0.5f, 0.f);
  const float fx = fmaxf(sw * ((float)xs + 0.5f) - 0.5f, 0.f);
  const int y0 = (int)fy, x0 = (int)fx;
  const int y1 = y0 + (y0 < ch - 1 ? 1 : 0), x1 = x0 + (x0 < cw - 1 ? 1 : 0);
  const float ly1 = fy - (float)y0, lx1 = fx - (float)x0;
  const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
  const unsigned char* f = frames + (((long)b * T + t) * H) * (long)W * C;
  auto px = [&](int yy, int xx) { return (float)f[((long)(ci + yy) * W + (cj + xx)) * C + c]; };
  const float v = ly0 * (lx0 * px(y0, x0) + lx1 * px(y0, x1)) + ly1 * (lx0 * px(y1, x0) + lx1 * px(y1, x1));
  out[e] = (v - mean[c]) / stdv[c];
}

}  // namespace

extern "C" int vj_video_transform(int B, int T, int H, int W, int C, int S, const void* frames, const int* params,
                                  const float* mean, const float* stdv, float* out, void* stream) {
  if (B == 0) return VJ_OK;
  VJ_CHECK_ARG(B > 0 && T > 0 && H > 0 && W > 0 && C > 0 && S > 0 && frames && params && mean && stdv && out,
               "vj_video_transform: bad arguments");
  const long total = (long)B * C * T * S * S;
  hipLaunchKernelGGL(k_video_transform, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     total, T, H, W, C, S, (const unsigned char*)frames, params, mean, stdv, out);
  VJ_LAUNCH_CHECK("vj_video_transform");
  return VJ_OK;
}

// ---- RCCL CU-occupancy proxy (diagnostic, bench.py --rccl-proxy-cus): a copy run by `blocks`
// persistent 256-thread workgroups, one per CU, the way RCCL's channel kernels hold CUs beside the
// backward's persistent GEMM grids while a bucket is all-reduced at world > 1. 16-B accesses,
// grid-stride; bytes % 16 == 0. mode 0: plain loads / stores; 1: non-temporal (nt) loads / stores;
// 2: no memory traffic, every workgroup holds its CU for the time the copy takes at 40 GB/s per
// workgroup (s_memrealtime, 100 MHz) - separates the CUs held from the bytes moved.
namespace {
__global__ __launch_bounds__(256) void k_proxy_copy(long n16, const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                    int mode, long ticks) {
  if (mode == 2) {
    const long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    return;
  }
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long)gridDim.x * 256) {
    if (mode == 1) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = __builtin_nontemporal_load((const u32x4*)(src + i));
      __builtin_nontemporal_store(v, (u32x4*)(dst + i));
    } else {
      dst[i] = src[i];
    }
  }
}
}  // namespace

extern "C" int vj_proxy_copy(void* dst, const void* src, long bytes, int blocks, int mode, void* stream) {
  if (bytes == 0) return VJ_OK;
  VJ_CHECK_ARG(dst && src && bytes > 0 && bytes % 16 == 0 && blocks > 0 && blocks <= 4096 && mode >= 0 && mode <= 2 &&
                   !(((uintptr_t)dst | (uintptr_t)src) & 15),
               "vj_proxy_copy: bad arguments (bytes=%ld blocks=%d mode=%d)", bytes, blocks, mode);
  hipLaunchKernelGGL(k_proxy_copy, dim3(blocks), dim3(256), 0, (hipStream_t)stream, bytes / 16, (const uint4*)src,
                     (uint4*)dst, mode, bytes / ((long)blocks * 400));
  VJ_LAUNCH_CHECK("vj_proxy_copy");
  return VJ_OK;
}
