// Cross-attention of a few learned queries over a long token sequence (the frozen-encoder probe:
// CrossAttention, src/models/utils/modules.py:566-594; AttentivePooler, attentive_pooler.py:91-100).
//
// Shapes: q [B*nq, D] (head h at columns h*hd), kv [B*N, 2D] (k at h*hd, v at D + h*hd), nq <= a few
// (1 or 3 in the reference's probes), N = encoder tokens (2048 per 16x256^2 clip, x clips). The work
// is 4*nq*N*hd flops against 4*N*hd bytes of K/V per (batch, head): nq flop/B, far under the MFMA
// ridge for any nq in use, so the kernels are HBM-bound on the K/V read and run on the VALU.
//
// Split-KV: one 256-thread workgroup per (key chunk of XCH = 128 keys, batch*head). The chunk's K and
// V rows are staged in LDS with coalesced 16-B loads (consecutive threads take consecutive 16-B pieces
// of a row); scores are computed key-per-thread (the 2 thread halves split the queries), the softmax
// statistics per query by one wave, P.V by (key-group, column) threads. Partials (m, l, unnormalised O)
// go to a workspace; a combine kernel merges the chunks in fixed order (deterministic, no atomics).
// Queries are processed XQ = 16 at a time (the host walks larger nq in blocks; the backward then
// accumulates dK / dV over the blocks in an f32 workspace).
//
// Backward (SDPA's, for training the probe): per chunk, p = 2^(s2 - lse2), dp = dO.v, ds = p (dp - Dq)
// with Dq = rowsum(dO * O); dK / dV rows of the chunk are complete (sums over the few queries) and
// stored directly; dQ = scale * sum_keys ds k is a cross-chunk sum: partials + a combine kernel.
#include "vj_common.h"

namespace {

constexpr int XCH = 128;   // keys per workgroup
constexpr int XQ = 16;     // queries per launch
constexpr int XHD = 128;   // max head dim (multiple of 8)
constexpr int XNT = 256;   // threads
constexpr float LOG2E = 1.4426950408889634f;

struct XArgs {
  const bf16_t* q;
  long ldq;
  const bf16_t* kv;
  long ldkv;
  int B, nq_all, q0, nq, N, H, hd, D;
  float scale;
  int nchunk;
  float* ws;  // fwd: [B*H][nchunk][XQ][hd + 2] (m2, l, o[hd]); bwd: [B*H][nchunk][XQ][hd] dq partials
  bf16_t* o;
  long ldo;
  float* lse2;  // [B*H][nq_all]: log2-domain lse of the scaled scores (s2 = scale*log2e*q.k)
  const bf16_t* dout;
  long lddo;
  bf16_t* dq;
  long lddq;
  bf16_t* dkv;
  long lddkv;
  // backward over more than XQ queries: dK / dV sum over every query block, accumulated in f32 rows
  // laid out like dkv (first block writes, middle blocks add, the last block writes bf16 dkv)
  float* dkv_acc;
  int blk_first, blk_last;
};

// K / V rows of a chunk -> LDS [XCH][hd + 8] bf16 (row pad of 16 B: the per-key 16-B reads of the
// score loop spread over the banks); rows past N are not loaded (their scores are masked)
__device__ __forceinline__ void stage_kv(const XArgs& a, int b, int h, int k0, int nk, bf16_t* ks, bf16_t* vs) {
  const int cpr = a.hd >> 3;  // 16-B pieces per row
  const int rs = a.hd + 8;
  for (int p = threadIdx.x; p < nk * cpr; p += XNT) {
    const int j = p / cpr, c = p - j * cpr;
    const bf16_t* row = a.kv + (long)(b * a.N + k0 + j) * a.ldkv + h * a.hd + 8 * c;
    const uint4 kk = *(const uint4*)row;
    const uint4 vv = *(const uint4*)(row + a.D);
    *(uint4*)(ks + j * rs + 8 * c) = kk;
    *(uint4*)(vs + j * rs + 8 * c) = vv;
  }
}

// dot of an f32 LDS row (broadcast reads) with a bf16 LDS row
__device__ __forceinline__ float dot_row(const float* x, const bf16_t* r, int hd) {
  float s = 0.f;
  for (int d = 0; d < hd; d += 8) {
    const uint4 u = *(const uint4*)(r + d);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s = fmaf(x[d + 2 * e], __uint_as_float(w[e] << 16), s);
      s = fmaf(x[d + 2 * e + 1], __uint_as_float(w[e] & 0xffff0000u), s);
    }
  }
  return s;
}

// dynamic LDS: the chunk's K and V images, [XCH][hd + 8] bf16 each
extern __shared__ __attribute__((aligned(16))) bf16_t xkv_lds[];
inline size_t kv_lds_bytes(int hd) { return 2ul * XCH * (hd + 8) * sizeof(bf16_t); }

__global__ __launch_bounds__(XNT) void k_xattn_fwd_part(XArgs a) {
  bf16_t* ks = xkv_lds;
  bf16_t* vs = xkv_lds + XCH * (a.hd + 8);
  __shared__ float qs[XQ][XHD];
  __shared__ float sc[XQ][XCH];
  __shared__ float red[XQ][XHD];  // P.V partial sums of the key groups
  const int c = blockIdx.x, bh = blockIdx.y;
  const int b = bh / a.H, h = bh - b * a.H;
  const int k0 = c * XCH, nk = min(XCH, a.N - k0);
  const int hd = a.hd, nq = a.nq, rs = hd + 8;
  const int t = threadIdx.x;
  const float sl2 = a.scale * LOG2E;
  for (int i = t; i < nq * hd; i += XNT) {
    const int qi = i / hd, d = i - qi * hd;
    qs[qi][d] = bf2f(a.q[(long)(b * a.nq_all + a.q0 + qi) * a.ldq + h * hd + d]) * sl2;
  }
  stage_kv(a, b, h, k0, nk, ks, vs);
  __syncthreads();
  {  // scores (log2 domain), key per thread, query halves
    const int j = t & (XCH - 1);
    for (int qi = t / XCH; qi < nq; qi += XNT / XCH)
      sc[qi][j] = j < nk ? dot_row(qs[qi], ks + j * rs, hd) : -INFINITY;
  }
  __syncthreads();
  const int wave = t >> 6, lane = t & 63;
  __shared__ float mq[XQ], lq[XQ];
  for (int qi = wave; qi < nq; qi += XNT / 64) {  // per-query max, exponentials, sum (one wave each)
    const float s0 = sc[qi][lane], s1 = sc[qi][lane + 64];
    const float m = wave_max(fmaxf(s0, s1));
    const float p0 = exp2f(s0 - m), p1 = exp2f(s1 - m);  // nk >= 1: m is finite
    sc[qi][lane] = p0;
    sc[qi][lane + 64] = p1;
    const float l = wave_sum(p0 + p1);
    if (lane == 0) {
      mq[qi] = m;
      lq[qi] = l;
    }
  }
  __syncthreads();
  // P.V: thread (key group g, column d); key groups interleave the chunk's keys
  const int KG = XNT / hd;
  const int g = t / hd, d = t - g * hd;
  float acc[XQ];
#pragma unroll
  for (int qi = 0; qi < XQ; ++qi) acc[qi] = 0.f;
  if (g < KG) {
    for (int j = g; j < nk; j += KG) {
      const float v = bf2f(vs[j * rs + d]);
#pragma unroll
      for (int qi = 0; qi < XQ; ++qi)
        if (qi < nq) acc[qi] = fmaf(sc[qi][j], v, acc[qi]);
    }
  }
  // fixed-order reduction of the key groups: group gg hands its sums to group 0, in order
  for (int gg = 1; gg < KG; ++gg) {
    __syncthreads();
    if (g == gg)
#pragma unroll
      for (int qi = 0; qi < XQ; ++qi)
        if (qi < nq) red[qi][d] = acc[qi];
    __syncthreads();
    if (g == 0)
#pragma unroll
      for (int qi = 0; qi < XQ; ++qi)
        if (qi < nq) acc[qi] += red[qi][d];
  }
  if (g == 0) {
    float* w = a.ws + ((long)bh * a.nchunk + c) * XQ * (hd + 2);
    for (int qi = 0; qi < nq; ++qi) {
      w[qi * (hd + 2) + 2 + d] = acc[qi];
      if (d == 0) {
        w[qi * (hd + 2)] = mq[qi];
        w[qi * (hd + 2) + 1] = lq[qi];
      }
    }
  }
}

// merge the chunks of one (batch, head): O = sum_c 2^(m_c - M) o_c / L, lse2 = M + log2 L
__global__ __launch_bounds__(XNT) void k_xattn_fwd_combine(XArgs a) {
  const int bh = blockIdx.x;
  const int b = bh / a.H, h = bh - b * a.H;
  const int hd = a.hd;
  const float* w0 = a.ws + (long)bh * a.nchunk * XQ * (hd + 2);
  for (int i = threadIdx.x; i < a.nq * hd; i += XNT) {
    const int qi = i / hd, d = i - qi * hd;
    float M = -INFINITY;
    for (int c = 0; c < a.nchunk; ++c) M = fmaxf(M, w0[(long)c * XQ * (hd + 2) + qi * (hd + 2)]);
    float L = 0.f, O = 0.f;
    for (int c = 0; c < a.nchunk; ++c) {
      const float* w = w0 + (long)c * XQ * (hd + 2) + qi * (hd + 2);
      const float f = exp2f(w[0] - M);
      L = fmaf(w[1], f, L);
      O = fmaf(w[2 + d], f, O);
    }
    a.o[(long)(b * a.nq_all + a.q0 + qi) * a.ldo + h * hd + d] = f2bf(O / L);
    if (d == 0) a.lse2[(long)bh * a.nq_all + a.q0 + qi] = M + log2f(L);
  }
}

__global__ __launch_bounds__(XNT) void k_xattn_bwd_part(XArgs a) {
  bf16_t* ks = xkv_lds;
  bf16_t* vs = xkv_lds + XCH * (a.hd + 8);
  __shared__ __attribute__((aligned(16))) float qs[XQ][XHD];   // q (unscaled)
  __shared__ __attribute__((aligned(16))) float dos[XQ][XHD];  // dO
  __shared__ float pp[XQ][XCH], dss[XQ][XCH];
  __shared__ float red[XQ][XHD];
  __shared__ float l2[XQ], dq_[XQ];
  const int c = blockIdx.x, bh = blockIdx.y;
  const int b = bh / a.H, h = bh - b * a.H;
  const int k0 = c * XCH, nk = min(XCH, a.N - k0);
  const int hd = a.hd, nq = a.nq, rs = hd + 8;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const float sl2 = a.scale * LOG2E;
  for (int i = t; i < nq * hd; i += XNT) {
    const int qi = i / hd, d = i - qi * hd;
    const long row = b * a.nq_all + a.q0 + qi;
    qs[qi][d] = bf2f(a.q[row * a.ldq + h * hd + d]);
    dos[qi][d] = bf2f(a.dout[row * a.lddo + h * hd + d]);
  }
  stage_kv(a, b, h, k0, nk, ks, vs);
  __syncthreads();
  for (int qi = wave; qi < nq; qi += XNT / 64) {  // Dq = rowsum(dO * O) (bf16 O, as stored)
    const long row = b * a.nq_all + a.q0 + qi;
    float s = 0.f;
    for (int d = lane; d < hd; d += 64) s = fmaf(dos[qi][d], bf2f(a.o[row * a.ldo + h * hd + d]), s);
    s = wave_sum(s);
    if (lane == 0) {
      dq_[qi] = s;
      l2[qi] = a.lse2[(long)bh * a.nq_all + a.q0 + qi];
    }
  }
  __syncthreads();
  {
    const int j = t & (XCH - 1);
    for (int qi = t / XCH; qi < nq; qi += XNT / XCH) {
      float p = 0.f, ds = 0.f;
      if (j < nk) {
        p = exp2f(dot_row(qs[qi], ks + j * rs, hd) * sl2 - l2[qi]);
        const float dp = dot_row(dos[qi], vs + j * rs, hd);
        ds = p * (dp - dq_[qi]);
      }
      pp[qi][j] = p;
      dss[qi][j] = ds;
    }
  }
  __syncthreads();
  {  // dK (threads 0..127) / dV (128..255) rows of this chunk, 8 columns at a time, straight to HBM
    const int j = t & (XCH - 1);
    const bool isv = t >= XCH;
    if (j < nk) {
      const float(*X)[XHD] = isv ? dos : qs;
      const float(*P)[XCH] = isv ? pp : dss;
      const float f = isv ? 1.f : a.scale;
      bf16_t* dst = a.dkv + (long)(b * a.N + k0 + j) * a.lddkv + (isv ? a.D : 0) + h * hd;
      float* acc = a.dkv_acc ? a.dkv_acc + (long)(b * a.N + k0 + j) * (2L * a.D) + (isv ? a.D : 0) + h * hd : nullptr;
      for (int d = 0; d < hd; d += 8) {
        float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int qi = 0; qi < nq; ++qi) {
          const float pq = P[qi][j];
#pragma unroll
          for (int e = 0; e < 8; ++e) s[e] = fmaf(pq, X[qi][d + e], s[e]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] *= f;
        if (acc && !a.blk_first) {  // add the earlier query blocks' sums (fixed order: deterministic)
          const float4 u = *(const float4*)(acc + d), w = *(const float4*)(acc + d + 4);
          s[0] += u.x; s[1] += u.y; s[2] += u.z; s[3] += u.w; s[4] += w.x; s[5] += w.y; s[6] += w.z; s[7] += w.w;
        }
        if (acc && !a.blk_last) {
          *(float4*)(acc + d) = make_float4(s[0], s[1], s[2], s[3]);
          *(float4*)(acc + d + 4) = make_float4(s[4], s[5], s[6], s[7]);
        } else {
          *(uint4*)(dst + d) = make_uint4(pack_bf2(s[0], s[1]), pack_bf2(s[2], s[3]), pack_bf2(s[4], s[5]),
                                          pack_bf2(s[6], s[7]));
        }
      }
    }
  }
  // dQ partial: thread (key group g, column d), fixed-order group reduction
  const int KG = XNT / hd;
  const int g = t / hd, d = t - g * hd;
  float acc[XQ];
#pragma unroll
  for (int qi = 0; qi < XQ; ++qi) acc[qi] = 0.f;
  if (g < KG)
    for (int j = g; j < nk; j += KG) {
      const float k = bf2f(ks[j * rs + d]);
#pragma unroll
      for (int qi = 0; qi < XQ; ++qi)
        if (qi < nq) acc[qi] = fmaf(dss[qi][j], k, acc[qi]);
    }
  for (int gg = 1; gg < KG; ++gg) {
    __syncthreads();
    if (g == gg)
#pragma unroll
      for (int qi = 0; qi < XQ; ++qi)
        if (qi < nq) red[qi][d] = acc[qi];
    __syncthreads();
    if (g == 0)
#pragma unroll
      for (int qi = 0; qi < XQ; ++qi)
        if (qi < nq) acc[qi] += red[qi][d];
  }
  if (g == 0) {
    float* w = a.ws + ((long)bh * a.nchunk + c) * XQ * hd;
    for (int qi = 0; qi < nq; ++qi) w[qi * hd + d] = acc[qi];
  }
}

__global__ __launch_bounds__(XNT) void k_xattn_bwd_combine(XArgs a) {
  const int bh = blockIdx.x;
  const int b = bh / a.H, h = bh - b * a.H;
  const int hd = a.hd;
  const float* w0 = a.ws + (long)bh * a.nchunk * XQ * hd;
  for (int i = threadIdx.x; i < a.nq * hd; i += XNT) {
    const int qi = i / hd, d = i - qi * hd;
    float s = 0.f;
    for (int c = 0; c < a.nchunk; ++c) s += w0[(long)c * XQ * hd + qi * hd + d];
    a.dq[(long)(b * a.nq_all + a.q0 + qi) * a.lddq + h * hd + d] = f2bf(a.scale * s);
  }
}

int check(const char* who, int B, int nq, int N, int H, int hd, long ldq, long ldkv, const void* q, const void* kv) {
  VJ_CHECK_ARG(B > 0 && nq > 0 && N > 0 && H > 0, "%s: bad dims B=%d nq=%d N=%d H=%d", who, B, nq, N, H);
  VJ_CHECK_ARG(hd % 8 == 0 && hd >= 8 && hd <= XHD, "%s: head_dim %d must be a multiple of 8 in [8, %d]", who, hd,
               XHD);
  VJ_CHECK_ARG(XNT / hd >= 1, "%s: head_dim too large", who);
  VJ_CHECK_ARG(q && kv, "%s: null operand", who);
  VJ_CHECK_ARG(ldq >= (long)H * hd && ldkv >= 2L * H * hd && ldkv % 8 == 0, "%s: bad strides (ldq=%ld ldkv=%ld)", who,
               ldq, ldkv);
  VJ_CHECK_ARG(((uintptr_t)kv & 15) == 0, "%s: kv must be 16-B aligned", who);
  return VJ_OK;
}

}  // namespace

static long ws_floats_needed(int B, int N, int H, int hd) { return (long)B * H * vj_cdiv(N, XCH) * XQ * (hd + 2); }
// backward with more than XQ queries: + the f32 dK / dV accumulator [B * N][2 * H * hd]
static long bwd_acc_floats(int B, int nq, int N, int H, int hd) { return nq > XQ ? 2L * B * N * H * hd : 0; }

extern "C" int vj_xattn_ws_floats(int B, int nq, int N, int H, int hd, long* out) {
  VJ_CHECK_ARG(out, "vj_xattn_ws_floats: null output");
  *out = ws_floats_needed(B, N, H, hd) + bwd_acc_floats(B, nq, N, H, hd);
  return VJ_OK;
}

extern "C" int vj_xattn_fwd(int B, int nq, int N, int H, int hd, const void* q, long ldq, const void* kv, long ldkv,
                            void* o, long ldo, float* lse2, float scale, float* ws, long ws_floats, void* stream) {
  if (B == 0 || nq == 0) return VJ_OK;
  if (int rc = check("vj_xattn_fwd", B, nq, N, H, hd, ldq, ldkv, q, kv)) return rc;
  VJ_CHECK_ARG(o && lse2 && ws, "vj_xattn_fwd: null output / workspace");
  VJ_CHECK_ARG(ws_floats >= ws_floats_needed(B, N, H, hd), "vj_xattn_fwd: workspace needs %ld floats",
               ws_floats_needed(B, N, H, hd));
  hipStream_t st = (hipStream_t)stream;
  XArgs a{};
  a.q = (const bf16_t*)q; a.ldq = ldq; a.kv = (const bf16_t*)kv; a.ldkv = ldkv;
  a.B = B; a.nq_all = nq; a.N = N; a.H = H; a.hd = hd; a.D = H * hd; a.scale = scale;
  a.nchunk = vj_cdiv(N, XCH); a.ws = ws; a.o = (bf16_t*)o; a.ldo = ldo; a.lse2 = lse2;
  for (int q0 = 0; q0 < nq; q0 += XQ) {  // query blocks of XQ (the workspace is reused in stream order)
    a.q0 = q0;
    a.nq = nq - q0 < XQ ? nq - q0 : XQ;
    hipLaunchKernelGGL(k_xattn_fwd_part, dim3(a.nchunk, B * H), dim3(XNT), kv_lds_bytes(hd), st, a);
    hipLaunchKernelGGL(k_xattn_fwd_combine, dim3(B * H), dim3(XNT), 0, st, a);
  }
  VJ_LAUNCH_CHECK("vj_xattn_fwd");
  return VJ_OK;
}

extern "C" int vj_xattn_bwd(int B, int nq, int N, int H, int hd, const void* q, long ldq, const void* kv, long ldkv,
                            const void* o, long ldo, const void* dout, long lddo, const float* lse2, float scale,
                            void* dq, long lddq, void* dkv, long lddkv, float* ws, long ws_floats, void* stream) {
  if (B == 0 || nq == 0) return VJ_OK;
  if (int rc = check("vj_xattn_bwd", B, nq, N, H, hd, ldq, ldkv, q, kv)) return rc;
  VJ_CHECK_ARG(o && dout && lse2 && dq && dkv && ws, "vj_xattn_bwd: null argument");
  VJ_CHECK_ARG(lddkv >= 2L * H * hd && lddkv % 8 == 0 && ((uintptr_t)dkv & 15) == 0,
               "vj_xattn_bwd: dkv must be 16-B aligned with lddkv %% 8 == 0 (lddkv=%ld)", lddkv);
  const long need = ws_floats_needed(B, N, H, hd) + bwd_acc_floats(B, nq, N, H, hd);
  VJ_CHECK_ARG(ws_floats >= need, "vj_xattn_bwd: workspace needs %ld floats", need);
  hipStream_t st = (hipStream_t)stream;
  XArgs a{};
  a.q = (const bf16_t*)q; a.ldq = ldq; a.kv = (const bf16_t*)kv; a.ldkv = ldkv;
  a.B = B; a.nq_all = nq; a.q0 = 0; a.nq = nq; a.N = N; a.H = H; a.hd = hd; a.D = H * hd; a.scale = scale;
  a.nchunk = vj_cdiv(N, XCH); a.ws = ws; a.o = (bf16_t*)o; a.ldo = ldo; a.lse2 = (float*)lse2;
  a.dout = (const bf16_t*)dout; a.lddo = lddo; a.dq = (bf16_t*)dq; a.lddq = lddq; a.dkv = (bf16_t*)dkv;
  a.lddkv = lddkv;
  a.dkv_acc = nq > XQ ? ws + ws_floats_needed(B, N, H, hd) : nullptr;
  for (int q0 = 0; q0 < nq; q0 += XQ) {  // query blocks of XQ, in order (dq partials reuse the workspace)
    a.q0 = q0;
    a.nq = nq - q0 < XQ ? nq - q0 : XQ;
    a.blk_first = q0 == 0;
    a.blk_last = q0 + XQ >= nq;
    hipLaunchKernelGGL(k_xattn_bwd_part, dim3(a.nchunk, B * H), dim3(XNT), kv_lds_bytes(hd), st, a);
    hipLaunchKernelGGL(k_xattn_bwd_combine, dim3(B * H), dim3(XNT), 0, st, a);
  }
  VJ_LAUNCH_CHECK("vj_xattn_bwd");
  return VJ_OK;
}
