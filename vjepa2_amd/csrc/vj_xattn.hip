// Cross-attention of a few learned queries over a long token sequence (the frozen-encoder probe:
// CrossAttention, src/models/utils/modules.py:566-594; AttentivePooler, attentive_pooler.py:91-100).
//
// Shapes: q [B*nq, D] (head h at columns h*hd), kv [B*N, 2D] (k at h*hd, v at D + h*hd), nq <= a few
// (1 or 3 in the reference's probes), N = encoder tokens (2048 per 16x256^2 clip, x clips). The work
// is 4*nq*N*hd flops against 4*N*hd bytes of K/V per (batch, head): nq flop/B, far under the MFMA
// ridge for any nq in use, so the kernels are HBM-bound on the K/V read and run on the VALU.
//
// Split-KV: one 256-thread workgroup per (key chunk of XCH = 64 keys, batch*head). Every LDS buffer is
// sized for the launch's (nq, hd) so that up to 8 workgroups share a CU (nq = 1, hd = 64: ~20 KB each):
// the kernels are latency-bound per workgroup (load -> compute -> store), so the K/V bytes in flight
// per CU come from many resident workgroups. Each thread issues all of its 16-B K and V loads before
// the first LDS store (one HBM round trip per chunk). Scores are key-per-thread (the 4 waves split the
// queries), the softmax statistics per query by one wave, P.V by (key-group, column) threads with a
// one-barrier fixed-order reduction. Partials (m, l, unnormalised O) go to a workspace; a combine kernel
// merges the chunks in fixed order (deterministic, no atomics). Queries are processed XQ = 16 at a time
// (the host walks larger nq in blocks; the backward then accumulates dK / dV over the blocks in an f32
// workspace).
//
// Backward (SDPA's, for training the probe): per chunk, p = 2^(s2 - lse2), dp = dO.v, ds = p (dp - Dq)
// with Dq = rowsum(dO * O); dK / dV rows of the chunk are complete (sums over the few queries) and
// stored directly (all 256 threads: key x {dK, dV} x interleaved 8-column pieces); dQ = scale * sum_keys
// ds k is a cross-chunk sum: partials + a combine kernel.
#include "vj_common.h"

namespace {

constexpr int XCH = 64;    // keys per workgroup (one wave's lanes)
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
  int nqb;  // query rows per chunk in the workspace / LDS layouts: min(nq_all, XQ)
  float scale;
  int nchunk;
  float* ws;  // fwd: [B*H][nchunk][nqb][hd + 2] (m2, l, o[hd]); bwd: [B*H][nchunk][nqb][hd] dq partials
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
// score loop spread over the banks); rows past N are not loaded (their scores are masked). A thread
// holds at most 4 pieces of each (XCH * hd / 8 <= 4 * XNT for hd <= 128): all loads first, then stores.
__device__ __forceinline__ void stage_kv(const XArgs& a, int b, int h, int k0, int nk, bf16_t* ks, bf16_t* vs) {
  const int cpr = a.hd >> 3;  // 16-B pieces per row
  const int rs = a.hd + 8, np = nk * cpr;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 kk[4], vv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {  // out-of-range pieces re-read piece 0 (always valid), not stored
    const int p = threadIdx.x + u * XNT < np ? threadIdx.x + u * XNT : 0;
    const int j = p / cpr, c = p - j * cpr;
    const bf16_t* row = a.kv + (long)(b * a.N + k0 + j) * a.ldkv + h * a.hd + 8 * c;
    kk[u] = *(const u32x4*)row;
    vv[u] = *(const u32x4*)(row + a.D);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int p = threadIdx.x + u * XNT;
    if (p < np) {
      const int j = p / cpr, c = p - j * cpr;
      *(u32x4*)(ks + j * rs + 8 * c) = kk[u];
      *(u32x4*)(vs + j * rs + 8 * c) = vv[u];
    }
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

// dynamic LDS, carved identically on host (sizes) and device (pointers):
//   ks, vs   [XCH][hd + 8] bf16      the chunk's K and V images
//   x0, x1   [nqb][hd] f32           fwd: scaled q (x1 unused); bwd: q, dO
//   s0, s1   [nqb][XCH] f32          fwd: scores -> p (s1 unused); bwd: p, ds
//   red      [KG - 1][nqb][hd] f32   key-group partial sums (KG = XNT / hd)
//   st0, st1 [nqb] f32               fwd: m, l; bwd: lse2, Dq
extern __shared__ __attribute__((aligned(16))) unsigned char x_lds[];
struct XLds {
  bf16_t *ks, *vs;
  float *x0, *x1, *s0, *s1, *red, *st0, *st1;
};
__host__ __device__ inline size_t x_lds_carve(int hd, int nqb, XLds* p) {
  const int kg = XNT / hd;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 15) & ~size_t(15);
    return o;
  };
  const size_t oks = take(2ul * XCH * (hd + 8)), ovs = take(2ul * XCH * (hd + 8));
  const size_t ox0 = take(4ul * nqb * hd), ox1 = take(4ul * nqb * hd);
  const size_t os0 = take(4ul * nqb * XCH), os1 = take(4ul * nqb * XCH);
  const size_t ored = take(4ul * (kg - 1) * nqb * hd);
  const size_t ost0 = take(4ul * nqb), ost1 = take(4ul * nqb);
  if (p) {
#ifdef __HIP_DEVICE_COMPILE__
    unsigned char* base = x_lds;
#else
    unsigned char* base = nullptr;
#endif
    p->ks = (bf16_t*)(base + oks);
    p->vs = (bf16_t*)(base + ovs);
    p->x0 = (float*)(base + ox0);
    p->x1 = (float*)(base + ox1);
    p->s0 = (float*)(base + os0);
    p->s1 = (float*)(base + os1);
    p->red = (float*)(base + ored);
    p->st0 = (float*)(base + ost0);
    p->st1 = (float*)(base + ost1);
  }
  return off;
}

// sum over the KG key groups of thread (g, d)'s per-query partials, fixed order, one barrier; the
// result is valid in group 0
__device__ __forceinline__ void group_reduce(float* acc, float* red, int g, int KG, int nq, int hd, int d) {
  if (g >= 1 && g < KG)
#pragma unroll
    for (int qi = 0; qi < XQ; ++qi)
      if (qi < nq) red[((g - 1) * nq + qi) * hd + d] = acc[qi];
  __syncthreads();
  if (g == 0)
    for (int gg = 1; gg < KG; ++gg)
#pragma unroll
      for (int qi = 0; qi < XQ; ++qi)
        if (qi < nq) acc[qi] += red[((gg - 1) * nq + qi) * hd + d];
}

__global__ __launch_bounds__(XNT) void k_xattn_fwd_part(XArgs a) {
  XLds L;
  x_lds_carve(a.hd, a.nqb, &L);
  const int c = blockIdx.x, bh = blockIdx.y;
  const int b = bh / a.H, h = bh - b * a.H;
  const int k0 = c * XCH, nk = min(XCH, a.N - k0);
  const int hd = a.hd, nq = a.nq, rs = hd + 8;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const float sl2 = a.scale * LOG2E;
  stage_kv(a, b, h, k0, nk, L.ks, L.vs);
  for (int i = t; i < nq * hd; i += XNT) {
    const int qi = i / hd, d = i - qi * hd;
    L.x0[i] = bf2f(a.q[(long)(b * a.nq_all + a.q0 + qi) * a.ldq + h * hd + d]) * sl2;
  }
  __syncthreads();
  // scores (log2 domain) key per lane, then the query's max, exponentials and sum in the same wave;
  // the waves split the queries
  for (int qi = wave; qi < nq; qi += XNT / 64) {
    const float s = lane < nk ? dot_row(L.x0 + qi * hd, L.ks + lane * rs, hd) : -INFINITY;
    const float m = wave_max(s);  // nk >= 1: m is finite
    const float p = exp2f(s - m);
    L.s0[qi * XCH + lane] = p;
    const float l = wave_sum(p);
    if (lane == 0) {
      L.st0[qi] = m;
      L.st1[qi] = l;
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
      const float v = bf2f(L.vs[j * rs + d]);
#pragma unroll
      for (int qi = 0; qi < XQ; ++qi)
        if (qi < nq) acc[qi] = fmaf(L.s0[qi * XCH + j], v, acc[qi]);
    }
  }
  group_reduce(acc, L.red, g, KG, nq, hd, d);
  if (g == 0) {
    float* w = a.ws + ((long)bh * a.nchunk + c) * a.nqb * (hd + 2);
    for (int qi = 0; qi < nq; ++qi) {
      w[qi * (hd + 2) + 2 + d] = acc[qi];
      if (d == 0) {
        w[qi * (hd + 2)] = L.st0[qi];
        w[qi * (hd + 2) + 1] = L.st1[qi];
      }
    }
  }
}

// merge the chunks of one (batch, head): O = sum_c 2^(m_c - M) o_c / L, lse2 = M + log2 L. One wave per
// query finds M and L; the (query, column) sums are split over G thread groups (chunks c = g mod G)
// and added in group order.
__global__ __launch_bounds__(XNT) void k_xattn_fwd_combine(XArgs a) {
  __shared__ float Ms[XQ], Ls[XQ], cred[XNT];
  const int bh = blockIdx.x;
  const int b = bh / a.H, h = bh - b * a.H;
  const int hd = a.hd, nq = a.nq, t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const long cs = (long)a.nqb * (hd + 2);  // chunk stride
  const float* w0 = a.ws + (long)bh * a.nchunk * cs;
  for (int qi = wave; qi < nq; qi += XNT / 64) {
    float m = -INFINITY;
    for (int c = lane; c < a.nchunk; c += 64) m = fmaxf(m, w0[c * cs + qi * (hd + 2)]);
    m = wave_max(m);
    float l = 0.f;
    for (int c = lane; c < a.nchunk; c += 64) {
      const float* w = w0 + c * cs + qi * (hd + 2);
      l = fmaf(w[1], exp2f(w[0] - m), l);
    }
    l = wave_sum(l);
    if (lane == 0) {
      Ms[qi] = m;
      Ls[qi] = l;
    }
  }
  __syncthreads();
  const int nqd = nq * hd;
  const int G = nqd <= XNT ? XNT / nqd : 1;
  const int g = t / nqd;
  for (int i0 = 0; i0 < nqd; i0 += XNT) {  // one pass unless nq * hd > XNT
    const int i = G > 1 ? t - g * nqd : i0 + t;
    const bool act = G > 1 ? g < G : i < nqd;
    float O = 0.f;
    if (act) {
      const int qi = i / hd, d = i - qi * hd;
      for (int c = G > 1 ? g : 0; c < a.nchunk; c += G) {
        const float* w = w0 + c * cs + qi * (hd + 2);
        O = fmaf(w[2 + d], exp2f(w[0] - Ms[qi]), O);
      }
    }
    if (G > 1) {
      if (act) cred[t] = O;
      __syncthreads();
      if (g == 0)
        for (int gg = 1; gg < G; ++gg) O += cred[gg * nqd + i];
    }
    if (act && (G == 1 || g == 0)) {
      const int qi = i / hd, d = i - qi * hd;
      a.o[(long)(b * a.nq_all + a.q0 + qi) * a.ldo + h * hd + d] = f2bf(O / Ls[qi]);
      if (d == 0) a.lse2[(long)bh * a.nq_all + a.q0 + qi] = Ms[qi] + log2f(Ls[qi]);
    }
    if (G > 1) break;
  }
}

__global__ __launch_bounds__(XNT) void k_xattn_bwd_part(XArgs a) {
  XLds L;
  x_lds_carve(a.hd, a.nqb, &L);
  const int c = blockIdx.x, bh = blockIdx.y;
  const int b = bh / a.H, h = bh - b * a.H;
  const int k0 = c * XCH, nk = min(XCH, a.N - k0);
  const int hd = a.hd, nq = a.nq, rs = hd + 8;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const float sl2 = a.scale * LOG2E;
  float* qs = L.x0;   // q (unscaled)
  float* dos = L.x1;  // dO
  float* pp = L.s0;
  float* dss = L.s1;
  stage_kv(a, b, h, k0, nk, L.ks, L.vs);
  for (int i = t; i < nq * hd; i += XNT) {
    const int qi = i / hd, d = i - qi * hd;
    const long row = b * a.nq_all + a.q0 + qi;
    qs[i] = bf2f(a.q[row * a.ldq + h * hd + d]);
    dos[i] = bf2f(a.dout[row * a.lddo + h * hd + d]);
  }
  for (int qi = wave; qi < nq; qi += XNT / 64) {  // Dq = rowsum(dO * O) (bf16 O, as stored)
    const long row = b * a.nq_all + a.q0 + qi;
    float s = 0.f;
    for (int d = lane; d < hd; d += 64)
      s = fmaf(bf2f(a.dout[row * a.lddo + h * hd + d]), bf2f(a.o[row * a.ldo + h * hd + d]), s);
    s = wave_sum(s);
    if (lane == 0) {
      L.st1[qi] = s;
      L.st0[qi] = a.lse2[(long)bh * a.nq_all + a.q0 + qi];
    }
  }
  __syncthreads();
  for (int qi = wave; qi < nq; qi += XNT / 64) {  // p, ds: key per lane, the waves split the queries
    float p = 0.f, ds = 0.f;
    if (lane < nk) {
      p = exp2f(dot_row(qs + qi * hd, L.ks + lane * rs, hd) * sl2 - L.st0[qi]);
      const float dp = dot_row(dos + qi * hd, L.vs + lane * rs, hd);
      ds = p * (dp - L.st1[qi]);
    }
    pp[qi * XCH + lane] = p;
    dss[qi * XCH + lane] = ds;
  }
  __syncthreads();
  {  // dK / dV rows of this chunk: thread (key j, dK|dV, column parity), 8 columns at a time, to HBM
    const int j = t & (XCH - 1);
    const bool isv = (t >> 6) & 1;
    const int par = t >> 7;
    if (j < nk) {
      const float* X = isv ? dos : qs;
      const float* P = isv ? pp : dss;
      const float f = isv ? 1.f : a.scale;
      bf16_t* dst = a.dkv + (long)(b * a.N + k0 + j) * a.lddkv + (isv ? a.D : 0) + h * hd;
      float* acc = a.dkv_acc ? a.dkv_acc + (long)(b * a.N + k0 + j) * (2L * a.D) + (isv ? a.D : 0) + h * hd : nullptr;
      for (int d = 8 * par; d < hd; d += 16) {
        float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int qi = 0; qi < nq; ++qi) {
          const float pq = P[qi * XCH + j];
#pragma unroll
          for (int e = 0; e < 8; ++e) s[e] = fmaf(pq, X[qi * hd + d + e], s[e]);
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
      const float k = bf2f(L.ks[j * rs + d]);
#pragma unroll
      for (int qi = 0; qi < XQ; ++qi)
        if (qi < nq) acc[qi] = fmaf(dss[qi * XCH + j], k, acc[qi]);
    }
  group_reduce(acc, L.red, g, KG, nq, hd, d);
  if (g == 0) {
    float* w = a.ws + ((long)bh * a.nchunk + c) * a.nqb * hd;
    for (int qi = 0; qi < nq; ++qi) w[qi * hd + d] = acc[qi];
  }
}

__global__ __launch_bounds__(XNT) void k_xattn_bwd_combine(XArgs a) {
  __shared__ float cred[XNT];
  const int bh = blockIdx.x;
  const int b = bh / a.H, h = bh - b * a.H;
  const int hd = a.hd, nq = a.nq, t = threadIdx.x;
  const long cs = (long)a.nqb * hd;
  const float* w0 = a.ws + (long)bh * a.nchunk * cs;
  const int nqd = nq * hd;
  const int G = nqd <= XNT ? XNT / nqd : 1;
  const int g = t / nqd;
  for (int i0 = 0; i0 < nqd; i0 += XNT) {
    const int i = G > 1 ? t - g * nqd : i0 + t;
    const bool act = G > 1 ? g < G : i < nqd;
    float s = 0.f;
    if (act)
      for (int c = G > 1 ? g : 0; c < a.nchunk; c += G) s += w0[c * cs + i];
    if (G > 1) {
      if (act) cred[t] = s;
      __syncthreads();
      if (g == 0)
        for (int gg = 1; gg < G; ++gg) s += cred[gg * nqd + i];
    }
    if (act && (G == 1 || g == 0)) {
      const int qi = i / hd, d = i - qi * hd;
      a.dq[(long)(b * a.nq_all + a.q0 + qi) * a.lddq + h * hd + d] = f2bf(a.scale * s);
    }
    if (G > 1) break;
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

static int nqb_of(int nq) { return nq < XQ ? nq : XQ; }
static long ws_floats_needed(int B, int nq, int N, int H, int hd) {
  return (long)B * H * vj_cdiv(N, XCH) * nqb_of(nq) * (hd + 2);
}
// backward with more than XQ queries: + the f32 dK / dV accumulator [B * N][2 * H * hd]
static long bwd_acc_floats(int B, int nq, int N, int H, int hd) { return nq > XQ ? 2L * B * N * H * hd : 0; }

// dynamic LDS of a (nqb, hd) launch; above 64 KB (nqb = 16 with hd = 128) the kernel's limit is raised
template <typename K>
static int x_lds_bytes(K kern, int hd, int nqb, size_t* bytes) {
  *bytes = x_lds_carve(hd, nqb, nullptr);
  if (*bytes > 65536) {
    VJ_CHECK_ARG(*bytes <= 160 * 1024, "xattn: %zu B of LDS", *bytes);
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)*bytes) != hipSuccess)
      VJ_CHECK_ARG(false, "xattn: cannot raise the LDS limit to %zu B", *bytes);
  }
  return VJ_OK;
}

extern "C" int vj_xattn_ws_floats(int B, int nq, int N, int H, int hd, long* out) {
  VJ_CHECK_ARG(out, "vj_xattn_ws_floats: null output");
  *out = ws_floats_needed(B, nq, N, H, hd) + bwd_acc_floats(B, nq, N, H, hd);
  return VJ_OK;
}

extern "C" int vj_xattn_fwd(int B, int nq, int N, int H, int hd, const void* q, long ldq, const void* kv, long ldkv,
                            void* o, long ldo, float* lse2, float scale, float* ws, long ws_floats, void* stream) {
  if (B == 0 || nq == 0) return VJ_OK;
  if (int rc = check("vj_xattn_fwd", B, nq, N, H, hd, ldq, ldkv, q, kv)) return rc;
  VJ_CHECK_ARG(o && lse2 && ws, "vj_xattn_fwd: null output / workspace");
  VJ_CHECK_ARG(ws_floats >= ws_floats_needed(B, nq, N, H, hd), "vj_xattn_fwd: workspace needs %ld floats",
               ws_floats_needed(B, nq, N, H, hd));
  size_t lds;
  if (int rc = x_lds_bytes(k_xattn_fwd_part, hd, nqb_of(nq), &lds)) return rc;
  hipStream_t st = (hipStream_t)stream;
  XArgs a{};
  a.q = (const bf16_t*)q; a.ldq = ldq; a.kv = (const bf16_t*)kv; a.ldkv = ldkv;
  a.B = B; a.nq_all = nq; a.N = N; a.H = H; a.hd = hd; a.D = H * hd; a.scale = scale; a.nqb = nqb_of(nq);
  a.nchunk = vj_cdiv(N, XCH); a.ws = ws; a.o = (bf16_t*)o; a.ldo = ldo; a.lse2 = lse2;
  for (int q0 = 0; q0 < nq; q0 += XQ) {  // query blocks of XQ (the workspace is reused in stream order)
    a.q0 = q0;
    a.nq = nq - q0 < XQ ? nq - q0 : XQ;
    hipLaunchKernelGGL(k_xattn_fwd_part, dim3(a.nchunk, B * H), dim3(XNT), lds, st, a);
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
  const long need = ws_floats_needed(B, nq, N, H, hd) + bwd_acc_floats(B, nq, N, H, hd);
  VJ_CHECK_ARG(ws_floats >= need, "vj_xattn_bwd: workspace needs %ld floats", need);
  size_t lds;
  if (int rc = x_lds_bytes(k_xattn_bwd_part, hd, nqb_of(nq), &lds)) return rc;
  hipStream_t st = (hipStream_t)stream;
  XArgs a{};
  a.q = (const bf16_t*)q; a.ldq = ldq; a.kv = (const bf16_t*)kv; a.ldkv = ldkv;
  a.B = B; a.nq_all = nq; a.q0 = 0; a.nq = nq; a.N = N; a.H = H; a.hd = hd; a.D = H * hd; a.scale = scale;
  a.nqb = nqb_of(nq);
  a.nchunk = vj_cdiv(N, XCH); a.ws = ws; a.o = (bf16_t*)o; a.ldo = ldo; a.lse2 = (float*)lse2;
  a.dout = (const bf16_t*)dout; a.lddo = lddo; a.dq = (bf16_t*)dq; a.lddq = lddq; a.dkv = (bf16_t*)dkv;
  a.lddkv = lddkv;
  a.dkv_acc = nq > XQ ? ws + ws_floats_needed(B, nq, N, H, hd) : nullptr;
  for (int q0 = 0; q0 < nq; q0 += XQ) {  // query blocks of XQ, in order (dq partials reuse the workspace)
    a.q0 = q0;
    a.nq = nq - q0 < XQ ? nq - q0 : XQ;
    a.blk_first = q0 == 0;
    a.blk_last = q0 + XQ >= nq;
    hipLaunchKernelGGL(k_xattn_bwd_part, dim3(a.nchunk, B * H), dim3(XNT), lds, st, a);
    hipLaunchKernelGGL(k_xattn_bwd_combine, dim3(B * H), dim3(XNT), 0, st, a);
  }
  VJ_LAUNCH_CHECK("vj_xattn_bwd");
  return VJ_OK;
}
