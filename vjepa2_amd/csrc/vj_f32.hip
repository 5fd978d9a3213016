// fp32-operand parity mode: the encoder forward with every operand and intermediate in f32, on the
// matrix cores (v_mfma_f32_32x32x2_f32: f32 products, f32 accumulation) and an exact-softmax
// attention. It exists to show that the bf16 path's distance to the fp32 oracle is operand rounding
// only: with these kernels in place of the bf16 GEMMs / attention (same LayerNorm, RoPE, epilogue
// math), the ViT-L/16 encoder output matches the oracle to ~1e-6 (tests/test_gpu_model.py).
// Throughput is not a goal here (simple 64x64 tiles, one thread per query in the attention).
#include "vj_common.h"

namespace {

// epilogue numbering (EPI_F32, EPI_F32_RESID, EPI_GELU): vj_common.h, as vj_gemm_bf16's

__device__ __forceinline__ int acc_row32(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// C[m, n] = sum_k A[m, k] B[n, k] + bias[n] (+ R[m, n]); EPI_GELU: C = pre-activation, C2 = GELU
// (exact erf form, nn.GELU() of vision_transformer.py:100). Tile 64 x 64, 4 waves (2 x 2) of one
// 32 x 32 accumulator each; K tiles of 16 staged in LDS (row pad 17: conflict-free column reads).
template <int EPI>
__global__ __launch_bounds__(256) void k_gemm_f32(int M, int N, int K, const float* __restrict__ A, long lda,
                                                  const float* __restrict__ B, long ldb, const float* __restrict__ bias,
                                                  const float* __restrict__ R, long ldr, float* __restrict__ C, long ldc,
                                                  float* __restrict__ C2, long ldc2) {
  __shared__ float As[64][17], Bs[64][17];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int k0 = 0; k0 < K; k0 += 16) {
#pragma unroll
    for (int i = tid; i < 64 * 16; i += 256) {
      const int r = i >> 4, c = i & 15;
      As[r][c] = (m0 + r < M && k0 + c < K) ? A[(long)(m0 + r) * lda + k0 + c] : 0.f;
      Bs[r][c] = (n0 + r < N && k0 + c < K) ? B[(long)(n0 + r) * ldb + k0 + c] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; kk += 2) {
      // A 32 x 2: lane l holds A(l & 31, l >> 5); B 2 x 32: lane l holds B(k = l >> 5, n = l & 31)
      const float a = As[wr * 32 + (lane & 31)][kk + (lane >> 5)];
      const float b = Bs[wc * 32 + (lane & 31)][kk + (lane >> 5)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  const int n = n0 + wc * 32 + (lane & 31);
  if (n >= N) return;
  const float bv = bias ? bias[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wr * 32 + acc_row32(r, lane);
    if (m >= M) continue;
    float v = acc[r] + bv;
    if constexpr (EPI == EPI_F32_RESID) v += R[(long)m * ldr + n];
    C[(long)m * ldc + n] = v;
    if constexpr (EPI == EPI_GELU) C2[(long)m * ldc2 + n] = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
  }
}

// Exact-softmax attention over ragged groups of equal-length sequences (the layout of
// vj_attn_fwd): q / k / v f32 rows of one token-major buffer (RoPE already applied), one thread per
// query, keys streamed through LDS in tiles of 32, online softmax with an exact rescale at every new
// maximum. O f32 [T, H*hd]; lse (natural log) [H][T].
constexpr int F32_MAXG = 4;
struct F32Groups {
  int ngroups;
  int nseq[F32_MAXG], len[F32_MAXG], tok0[F32_MAXG], blk0[F32_MAXG + 1];
};

template <int HD>
__global__ __launch_bounds__(128) void k_attn_fwd_f32(int T, int H, const float* __restrict__ qkv, long ld, int q_off,
                                                      int k_off, int v_off, float* __restrict__ o, long ldo,
                                                      float* __restrict__ lse, float scale, F32Groups sg) {
  __shared__ float Ks[32][HD], Vs[32][HD];
  const int h = blockIdx.y;
  int g = 0;
#pragma unroll
  for (int i = 1; i < F32_MAXG; ++i)
    if (i < sg.ngroups && (int)blockIdx.x >= sg.blk0[i]) g = i;
  const int len = sg.len[g];
  const int bps = (len + 127) / 128;
  const int local = blockIdx.x - sg.blk0[g];
  const int s = local / bps, qt = local - s * bps;
  const long seq0 = sg.tok0[g] + (long)s * len;
  const int qi = qt * 128 + threadIdx.x;
  const bool qok = qi < len;
  float q[HD], acc[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    q[d] = qok ? qkv[(seq0 + qi) * ld + q_off + h * HD + d] : 0.f;
    acc[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < len; k0 += 32) {
    for (int i = threadIdx.x; i < 32 * HD; i += 128) {
      const int r = i / HD, d = i - r * HD;
      const bool ok = k0 + r < len;
      Ks[r][d] = ok ? qkv[(seq0 + k0 + r) * ld + k_off + h * HD + d] : 0.f;
      Vs[r][d] = ok ? qkv[(seq0 + k0 + r) * ld + v_off + h * HD + d] : 0.f;
    }
    __syncthreads();
    const int nk = min(32, len - k0);
    for (int j = 0; j < nk; ++j) {
      float sc = 0.f;
#pragma unroll
      for (int d = 0; d < HD; ++d) sc = fmaf(q[d], Ks[j][d], sc);
      sc *= scale;
      if (sc > m) {
        const float corr = expf(m - sc);  // 0 on the first key
        l *= corr;
#pragma unroll
        for (int d = 0; d < HD; ++d) acc[d] *= corr;
        m = sc;
      }
      const float p = expf(sc - m);
      l += p;
#pragma unroll
      for (int d = 0; d < HD; ++d) acc[d] = fmaf(p, Vs[j][d], acc[d]);
    }
    __syncthreads();
  }
  if (!qok) return;
  const float inv = 1.f / l;
#pragma unroll
  for (int d = 0; d < HD; ++d) o[(seq0 + qi) * ldo + h * HD + d] = acc[d] * inv;
  if (lse) lse[(long)h * T + seq0 + qi] = m + logf(l);
}

}  // namespace

extern "C" int vj_gemm_f32(int M, int N, int K, const float* A, long lda, const float* B, long ldb, int epi,
                           const float* bias, const float* resid, long ldr, float* C, long ldc, float* C2, long ldc2,
                           void* stream) {
  if (M == 0 || N == 0) return VJ_OK;
  VJ_CHECK_ARG(M > 0 && N > 0 && K > 0 && lda >= K && ldb >= K && ldc >= N, "vj_gemm_f32: bad shape");
  VJ_CHECK_ARG(A && B && C, "vj_gemm_f32: null operand");
  VJ_CHECK_ARG(epi != EPI_F32_RESID || (resid && ldr >= N), "vj_gemm_f32: EPI_F32_RESID needs the residual");
  VJ_CHECK_ARG(epi != EPI_GELU || (C2 && ldc2 >= N), "vj_gemm_f32: EPI_GELU needs the activation output");
  const dim3 grid(vj_cdiv(N, 64), vj_cdiv(M, 64));
  hipStream_t st = (hipStream_t)stream;
  switch (epi) {
    case EPI_F32:
      hipLaunchKernelGGL(k_gemm_f32<EPI_F32>, grid, dim3(256), 0, st, M, N, K, A, lda, B, ldb, bias, resid, ldr, C, ldc,
                         C2, ldc2);
      break;
    case EPI_F32_RESID:
      hipLaunchKernelGGL(k_gemm_f32<EPI_F32_RESID>, grid, dim3(256), 0, st, M, N, K, A, lda, B, ldb, bias, resid, ldr,
                         C, ldc, C2, ldc2);
      break;
    case EPI_GELU:
      hipLaunchKernelGGL(k_gemm_f32<EPI_GELU>, grid, dim3(256), 0, st, M, N, K, A, lda, B, ldb, bias, resid, ldr, C,
                         ldc, C2, ldc2);
      break;
    default: vj_set_error("vj_gemm_f32: unsupported epilogue %d", epi); return VJ_ERR_ARG;
  }
  VJ_LAUNCH_CHECK("vj_gemm_f32");
  return VJ_OK;
}

extern "C" int vj_attn_fwd_f32(int T, int H, int hd, const float* qkv, long ld, int q_off, int k_off, int v_off,
                               float* o, long ldo, float* lse, float scale, int ngroups, const int* nseq,
                               const int* len, void* stream) {
  if (T == 0) return VJ_OK;
  VJ_CHECK_ARG(hd == 32 || hd == 64 || hd == 80 || hd == 88, "vj_attn_fwd_f32: head_dim 32/64/80/88 (got %d)", hd);
  VJ_CHECK_ARG(ngroups >= 1 && ngroups <= F32_MAXG, "vj_attn_fwd_f32: 1..%d groups", F32_MAXG);
  F32Groups sg{};
  sg.ngroups = ngroups;
  long tok = 0, blk = 0;
  for (int g = 0; g < F32_MAXG; ++g) {
    sg.tok0[g] = (int)tok;
    sg.blk0[g] = (int)blk;
    if (g < ngroups) {
      VJ_CHECK_ARG(nseq[g] >= 0 && len[g] >= 1, "vj_attn_fwd_f32: bad group %d", g);
      sg.nseq[g] = nseq[g];
      sg.len[g] = len[g];
      tok += (long)nseq[g] * len[g];
      blk += (long)nseq[g] * ((len[g] + 127) / 128);
    } else {
      sg.len[g] = 1;
    }
  }
  sg.blk0[F32_MAXG] = (int)blk;
  VJ_CHECK_ARG(tok == T, "vj_attn_fwd_f32: groups cover %ld tokens but T=%d", tok, T);
  const dim3 grid((unsigned)blk, H);
  hipStream_t st = (hipStream_t)stream;
  switch (hd) {
    case 32: hipLaunchKernelGGL(k_attn_fwd_f32<32>, grid, dim3(128), 0, st, T, H, qkv, ld, q_off, k_off, v_off, o, ldo, lse, scale, sg); break;
    case 64: hipLaunchKernelGGL(k_attn_fwd_f32<64>, grid, dim3(128), 0, st, T, H, qkv, ld, q_off, k_off, v_off, o, ldo, lse, scale, sg); break;
    case 80: hipLaunchKernelGGL(k_attn_fwd_f32<80>, grid, dim3(128), 0, st, T, H, qkv, ld, q_off, k_off, v_off, o, ldo, lse, scale, sg); break;
    default: hipLaunchKernelGGL(k_attn_fwd_f32<88>, grid, dim3(128), 0, st, T, H, qkv, ld, q_off, k_off, v_off, o, ldo, lse, scale, sg); break;
  }
  VJ_LAUNCH_CHECK("vj_attn_fwd_f32");
  return VJ_OK;
}
