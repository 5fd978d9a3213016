// bf16 MFMA GEMM for gfx950 with fused epilogues.
//
//   C[m, n] = sum_k A(m, k) * B(n, k)      (fp32 accumulate, v_mfma_f32_32x32x16_bf16)
//
// Operand layouts (both bf16):
//   A K-major : A(m,k) = A[m*lda + k]      (activations X[M,K]; dY[M,N] for dgrad)
//   A MN-major: A(m,k) = A[k*lda + m]      (dY^T for weight-grad: k = token)
//   B K-major : B(n,k) = B[n*ldb + k]      (nn.Linear weight W[N,K] in forward)
//   B MN-major: B(n,k) = B[k*ldb + n]      (W[N,K] read as W^T in dgrad; X in weight-grad)
// This covers forward (Y = X W^T), dgrad (dX = dY W) and wgrad (dW = dY^T X) of every
// nn.Linear / Conv3d-as-GEMM on the V-JEPA hot path without any
// transpose pass: MN-major tiles are staged as [k][m] rows and read with ds_read_b64_tr_b16.
//
// Tile 128x128x64, 256 threads = 4 waves (2x2), each wave 64x64 = 2x2 MFMA 32x32 tiles.
// Global->LDS by LDS-DMA (buffer_load_dwordx4 ... lds) with hardware range check: any chunk
// outside [M)x[K) / [N)x[K) is redirected out of range and lands as zeros, so ragged M / N / K
// need no padding. LDS images are XOR-swizzled on the SOURCE address (the DMA writes lane-linear):
//   K-major  [128 rows][64 k] (128-B rows): phys chunk = chunk ^ ((row>>1)&7)  -> b128 reads conflict-free
//   MN-major [64 k][128 rows] (256-B rows): phys chunk = chunk ^ ((k&3)<<2)   -> tr_b16 reads conflict-free
// Two LDS stages (64 KB) -> 2 workgroups / CU.
#include <stdlib.h>
#include "vj_common.h"

namespace {

// epilogue numbering: vj_common.h (shared with vj_gemm256.hip and the public header)

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  int M, N, K;
  long lda, ldb;
  void* C;
  long ldc;
  void* C2;
  long ldc2;
  const float* bias;
  const void* aux;  // EPI_GELU_BWD: bf16 GELU derivative (saved by EPI_GELU); EPI_F32_RESID: f32 residual
  long ldaux;
  int kslice;  // split-K: K range of blockIdx.z is [z*kslice, min(K, (z+1)*kslice))
  float* ws;   // EPI_PARTIAL: f32 partial tiles [splitk][M][N]
  // split-K reduce only: rs_out[m] (+)= sum_z rs_ws[z][m] (the fused bias gradient of vj_gemm_bf16_wgrad)
  const float* rs_ws = nullptr;
  float* rs_out = nullptr;
  int rs_acc = 0;
};

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = BM * BK * 2;  // 16 KB per operand per stage

__device__ __forceinline__ uint32_t clamp_bytes(long b) {
  if (b < 0) return 0;
  return b > 0x7fffffffL ? 0x7fffffffu : (uint32_t)b;
}

// Stage one 128 x 64 operand tile (rows [r0, r0+128) of M or N, k in [k0, k0+64)).
template <bool KMAJ>
__device__ __forceinline__ void stage_tile(__amdgpu_buffer_rsrc_t rs, long ld, int rows_left, int k0, int K,
                                           LDS_AS char* lds, int wave, int lane) {
  if constexpr (KMAJ) {
    // 16 DMA pieces of 8 rows x 128 B; 4 per wave.
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int blk = wave * 4 + i;
      const int r = blk * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int kk = k0 + c * 8;
      const bool ok = (r < rows_left) && (kk < K);
      const uint32_t voff = ok ? (uint32_t)(((long)r * ld + kk) * 2) : VJ_OOB;
      dma16(rs, lds + blk * 1024, voff);
    }
  } else {
    // 16 DMA pieces of 4 k-rows x 256 B; 4 per wave.
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int blk = wave * 4 + i;
      const int kr = blk * 4 + (lane >> 4);
      const int c = (lane & 15) ^ ((kr & 3) << 2);
      const int rr = c * 8;
      const bool ok = (k0 + kr < K) && (rr < rows_left);
      const uint32_t voff = ok ? (uint32_t)(((long)(k0 + kr) * ld + rr) * 2) : VJ_OOB;
      dma16(rs, lds + blk * 1024, voff);
    }
  }
}

// Fragment (8 bf16) of a 32-row subtile at row base rb, k-step s (16 wide), 32x32x16 operand map:
// lane l holds X(rb + (l&31), 16s + 8(l>>5) + j), j = 0..7.
template <bool KMAJ>
__device__ __forceinline__ bf16x8 load_frag(const LDS_AS char* lds, int rb, int s, int lane) {
  if constexpr (KMAJ) {
    const int r = rb + (lane & 31);
    const int c = (2 * s + (lane >> 5)) ^ ((r >> 1) & 7);
    return *(const LDS_AS bf16x8*)(lds + r * 128 + c * 16);
  } else {
    const int r = rb + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
    const int kr = 16 * s + 8 * (lane >> 5) + ((lane >> 2) & 3);
    const int sw = (kr & 3) << 2;
    const int off = ((r >> 3) ^ sw) * 16 + (r & 7) * 2;
    const s16x4 lo = ds_read_tr16(lds + kr * 256 + off);
    const s16x4 hi = ds_read_tr16(lds + (kr + 4) * 256 + off);
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

template <bool AK, bool BKM, int EPI>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem_raw[4 * TILE_BYTES];
  LDS_AS char* smem = (LDS_AS char*)smem_raw;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;

  // Descriptors based at the tile origin (keeps 32-bit offsets small).
  const bf16_t* abase = AK ? g.A + (long)m0 * g.lda : g.A + m0;
  const bf16_t* bbase = BKM ? g.B + (long)n0 * g.ldb : g.B + n0;
  const uint32_t abytes = AK ? clamp_bytes((long)(g.M - m0) * g.lda * 2) : clamp_bytes(((long)g.K * g.lda - m0) * 2);
  const uint32_t bbytes = BKM ? clamp_bytes((long)(g.N - n0) * g.ldb * 2) : clamp_bytes(((long)g.K * g.ldb - n0) * 2);
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(abase, abytes);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(bbase, bbytes);
  const int mleft = g.M - m0, nleft = g.N - n0;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int kb = blockIdx.z * g.kslice;
  const int ke = min(g.K, kb + g.kslice);
  const int nk = (ke - kb + BK - 1) / BK;
  stage_tile<AK>(ra, g.lda, mleft, kb, ke, smem, wave, lane);
  stage_tile<BKM>(rb, g.ldb, nleft, kb, ke, smem + TILE_BYTES, wave, lane);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      LDS_AS char* nxt = smem + (cur ^ 1) * 2 * TILE_BYTES;
      stage_tile<AK>(ra, g.lda, mleft, kb + (kt + 1) * BK, ke, nxt, wave, lane);
      stage_tile<BKM>(rb, g.ldb, nleft, kb + (kt + 1) * BK, ke, nxt + TILE_BYTES, wave, lane);
    }
    const LDS_AS char* As = smem + cur * 2 * TILE_BYTES;
    const LDS_AS char* Bs = As + TILE_BYTES;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 a0 = load_frag<AK>(As, wm * 64, s, lane);
      bf16x8 a1 = load_frag<AK>(As, wm * 64 + 32, s, lane);
      bf16x8 b0 = load_frag<BKM>(Bs, wn * 64, s, lane);
      bf16x8 b1 = load_frag<BKM>(Bs, wn * 64 + 32, s, lane);
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }

  // Epilogue. Accumulator map (32x32x16): col n = lane&31, row m = (r&3) + 8(r>>2) + 4(lane>>5).
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 64 + j * 32 + (lane & 31);
    if (n >= g.N) continue;
    const float bv = (EPI != EPI_PARTIAL && g.bias) ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= g.M) continue;
        const float v = acc[i][j][r] + bv;
        if constexpr (EPI == EPI_PARTIAL) {
          g.ws[((long)blockIdx.z * g.M + m) * g.N + n] = v;
        } else if constexpr (EPI == EPI_BF16) {
          ((bf16_t*)g.C)[(long)m * g.ldc + n] = f2bf(v);
        } else if constexpr (EPI == EPI_F32) {
          ((float*)g.C)[(long)m * g.ldc + n] = v;
        } else if constexpr (EPI == EPI_F32_RESID) {
          const float res = ((const float*)g.aux)[(long)m * g.ldaux + n];
          ((float*)g.C)[(long)m * g.ldc + n] = res + v;
        } else if constexpr (EPI == EPI_BF16_RESID) {
          const float res = bf2f(((const bf16_t*)g.aux)[(long)m * g.ldaux + n]);
          ((bf16_t*)g.C)[(long)m * g.ldc + n] = f2bf(res + v);
        } else if constexpr (EPI == EPI_GELU) {
          float y, dy;
          gelu_fwd_grad(bf2f(f2bf(v)), y, dy);  // on the bf16 pre-activation
          if (g.C) ((bf16_t*)g.C)[(long)m * g.ldc + n] = f2bf(dy);  // saved for EPI_GELU_BWD
          ((bf16_t*)g.C2)[(long)m * g.ldc2 + n] = f2bf(y);
        } else if constexpr (EPI == EPI_GELU_BWD) {
          const float dg = bf2f(((const bf16_t*)g.aux)[(long)m * g.ldaux + n]);  // saved GELU derivative
          ((bf16_t*)g.C)[(long)m * g.ldc + n] = f2bf(acc[i][j][r] * dg);
        }
      }
    }
  }
}

// the fused row sums (bias gradient) of row m, by the thread of the row's first columns: fixed z order
__device__ __forceinline__ void reduce_rowsum(const GemmArgs& g, int splitk, int m) {
  float s = 0.f;
  for (int z = 0; z < splitk; ++z) s += g.rs_ws[(long)z * g.M + m];
  g.rs_out[m] = g.rs_acc ? g.rs_out[m] + s : s;
}

// Split-K combine, 4 columns per thread (N % 4 == 0): C = epilogue(sum_z ws[z]) in fixed z order.
__global__ void k_splitk_reduce4(GemmArgs g, int splitk, int epi) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const long total = (long)g.M * g.N;
  if (i >= total) return;
  const int m = (int)(i / g.N), n = (int)(i % g.N);
  if (g.rs_out && n == 0) reduce_rowsum(g, splitk, m);
  float4 v = g.bias ? *(const float4*)(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int z = 0; z < splitk; ++z) {
    const float4 w = *(const float4*)(g.ws + (long)z * total + i);
    v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
  }
  if (epi == EPI_F32_RESID) {
    const float4 r = *(const float4*)((const float*)g.aux + (long)m * g.ldaux + n);
    *(float4*)((float*)g.C + (long)m * g.ldc + n) = make_float4(r.x + v.x, r.y + v.y, r.z + v.z, r.w + v.w);
  } else if (epi == EPI_F32) {
    *(float4*)((float*)g.C + (long)m * g.ldc + n) = v;
  } else {
    *(uint2*)((bf16_t*)g.C + (long)m * g.ldc + n) = make_uint2(pack_bf2(v.x, v.y), pack_bf2(v.z, v.w));
  }
}

// Split-K combine: C = epilogue(sum_z ws[z]) in fixed z order (deterministic).
__global__ void k_splitk_reduce(GemmArgs g, int splitk, int epi) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)g.M * g.N;
  if (i >= total) return;
  const int m = (int)(i / g.N), n = (int)(i % g.N);
  if (g.rs_out && n == 0) reduce_rowsum(g, splitk, m);
  float v = g.bias ? g.bias[n] : 0.f;
  for (int z = 0; z < splitk; ++z) v += g.ws[(long)z * total + i];
  if (epi == EPI_F32_RESID) {
    ((float*)g.C)[(long)m * g.ldc + n] = ((const float*)g.aux)[(long)m * g.ldaux + n] + v;
  } else if (epi == EPI_F32) {
    ((float*)g.C)[(long)m * g.ldc + n] = v;
  } else {
    ((bf16_t*)g.C)[(long)m * g.ldc + n] = f2bf(v);
  }
}

template <bool AK, bool BKM>
int launch_epi(int epi, const GemmArgs& g, dim3 grid, hipStream_t st) {
  switch (epi) {
    case EPI_PARTIAL: hipLaunchKernelGGL((k_gemm<AK, BKM, EPI_PARTIAL>), grid, dim3(256), 0, st, g); break;
    case EPI_BF16: hipLaunchKernelGGL((k_gemm<AK, BKM, EPI_BF16>), grid, dim3(256), 0, st, g); break;
    case EPI_F32: hipLaunchKernelGGL((k_gemm<AK, BKM, EPI_F32>), grid, dim3(256), 0, st, g); break;
    case EPI_F32_RESID: hipLaunchKernelGGL((k_gemm<AK, BKM, EPI_F32_RESID>), grid, dim3(256), 0, st, g); break;
    case EPI_GELU: hipLaunchKernelGGL((k_gemm<AK, BKM, EPI_GELU>), grid, dim3(256), 0, st, g); break;
    case EPI_GELU_BWD: hipLaunchKernelGGL((k_gemm<AK, BKM, EPI_GELU_BWD>), grid, dim3(256), 0, st, g); break;
    case EPI_BF16_RESID: hipLaunchKernelGGL((k_gemm<AK, BKM, EPI_BF16_RESID>), grid, dim3(256), 0, st, g); break;
    default: vj_set_error("vj_gemm_bf16: unknown epilogue %d", epi); return VJ_ERR_ARG;
  }
  VJ_LAUNCH_CHECK("vj_gemm_bf16");
  return VJ_OK;
}

}  // namespace

int vj_gemm256_partial(int M, int N, int K, const void* A, long lda, int a_kmajor, const void* B, long ldb,
                       int b_kmajor, int kslice, int splitk, float* ws, hipStream_t st, float* rsum);
int vj_gemm256_dispatch(int M, int N, int K, const void* A, long lda, int a_kmajor, const void* B, long ldb,
                        int b_kmajor, int epi, const float* bias, const void* aux, long ldaux, void* C, long ldc,
                        void* C2, long ldc2, hipStream_t st, const void* rope);

// The split-K GEMM. rs_out (or null): also rs_out[m] (+= if rs_acc) = sum_k A[m, k], fused into the
// 256-row partial kernel when that runs (*rs_done = 1; ws then holds splitk * (M * N + M) floats),
// else left to the caller (*rs_done = 0).
static int gemm_splitk(int M, int N, int K, const void* A, long lda, int a_kmajor, const void* B, long ldb,
                       int b_kmajor, int epi, const float* bias, const void* aux, long ldaux, void* C, long ldc,
                       void* C2, long ldc2, int splitk, float* ws, long ws_floats, void* stream, float* rs_out,
                       int rs_acc, int* rs_done) {
  if (rs_done) *rs_done = 0;
  if (M == 0 || N == 0) return VJ_OK;
  VJ_CHECK_ARG(M > 0 && N > 0 && K > 0, "vj_gemm_bf16: bad dims M=%d N=%d K=%d", M, N, K);
  VJ_CHECK_ARG(epi == EPI_BF16 || epi == EPI_F32 || epi == EPI_F32_RESID || epi == EPI_GELU || epi == EPI_GELU_BWD ||
                   epi == EPI_BF16_RESID,
               "vj_gemm_bf16: epilogue %d is not a public epilogue (0-4, 7; include/vjepa_hip.h)", epi);
  VJ_CHECK_ARG(A && B, "vj_gemm_bf16: null operand");
  VJ_CHECK_ARG(((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0, "vj_gemm_bf16: operands must be 16-B aligned");
  VJ_CHECK_ARG(lda % 8 == 0 && ldb % 8 == 0, "vj_gemm_bf16: lda/ldb must be multiples of 8 (lda=%ld ldb=%ld)", lda, ldb);
  // The contiguous dimension of each operand must be a multiple of 8 (16-B DMA chunks).
  VJ_CHECK_ARG(a_kmajor ? (K % 8 == 0) : (M % 8 == 0), "vj_gemm_bf16: A contiguous dim must be %%8");
  VJ_CHECK_ARG(b_kmajor ? (K % 8 == 0) : (N % 8 == 0), "vj_gemm_bf16: B contiguous dim must be %%8");
  VJ_CHECK_ARG(a_kmajor ? lda >= K : lda >= M, "vj_gemm_bf16: lda too small");
  VJ_CHECK_ARG(b_kmajor ? ldb >= K : ldb >= N, "vj_gemm_bf16: ldb too small");
  VJ_CHECK_ARG(epi == EPI_GELU ? (C2 != nullptr) : (C != nullptr), "vj_gemm_bf16: null output");
  VJ_CHECK_ARG((epi != EPI_F32_RESID && epi != EPI_GELU_BWD && epi != EPI_BF16_RESID) || aux,
               "vj_gemm_bf16: epilogue needs aux");
  // 32-bit DMA offsets: every operand must span < 2 GB from its tile origin.
  VJ_CHECK_ARG((a_kmajor ? (long)M * lda : (long)K * lda) * 2 < 0x7fffffffL, "vj_gemm_bf16: A too large");
  VJ_CHECK_ARG((b_kmajor ? (long)N * ldb : (long)K * ldb) * 2 < 0x7fffffffL, "vj_gemm_bf16: B too large");
  if (splitk < 1) splitk = 1;
  int kslice = K;
  if (splitk > 1) {
    VJ_CHECK_ARG(epi == EPI_BF16 || epi == EPI_F32 || epi == EPI_F32_RESID,
                 "vj_gemm_bf16_splitk: split-K supports the BF16/F32/F32_RESID epilogues");
    kslice = vj_cdiv(vj_cdiv(K, splitk), BK) * BK;
    splitk = vj_cdiv(K, kslice);
    VJ_CHECK_ARG(ws && ws_floats >= (long)splitk * M * N, "vj_gemm_bf16_splitk: workspace needs %ld floats",
                 (long)splitk * M * N);
  }
  GemmArgs g{(const bf16_t*)A, (const bf16_t*)B, M, N, K, lda, ldb, C, ldc, C2, ldc2, bias, aux, ldaux, kslice, ws};
  dim3 grid(vj_cdiv(N, BN), vj_cdiv(M, BM), splitk);
  VJ_CHECK_ARG(grid.y <= 65535, "vj_gemm_bf16: M too large");
  hipStream_t st = (hipStream_t)stream;
  // the 256-row persistent kernel (vj_gemm256.hip) where it takes the shape; this file's 128 x 128
  // kernel for the rest (small M / N, layouts it declines)
  if (splitk == 1 && M >= 1024 && N >= 128) {
    const int rc = vj_gemm256_dispatch(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, epi, bias, aux, ldaux, C, ldc, C2,
                                       ldc2, st, nullptr);
    if (rc != VJ_ERR_UNSUPPORTED) return rc;
  }
  if (splitk > 1) {
    int rc = VJ_ERR_UNSUPPORTED;
    const bool rs = rs_out && ws_floats >= (long)splitk * M * N + (long)splitk * M;
    rc = vj_gemm256_partial(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, kslice, splitk, ws, st,
                            rs ? ws + (long)splitk * M * N : nullptr);
    if (rc == VJ_OK && rs) {
      g.rs_ws = ws + (long)splitk * M * N;
      g.rs_out = rs_out;
      g.rs_acc = rs_acc;
      if (rs_done) *rs_done = 1;
    }
    if (rc == VJ_ERR_UNSUPPORTED) {
      if (a_kmajor && b_kmajor) rc = launch_epi<true, true>(EPI_PARTIAL, g, grid, st);
      else if (a_kmajor && !b_kmajor) rc = launch_epi<true, false>(EPI_PARTIAL, g, grid, st);
      else if (!a_kmajor && b_kmajor) rc = launch_epi<false, true>(EPI_PARTIAL, g, grid, st);
      else rc = launch_epi<false, false>(EPI_PARTIAL, g, grid, st);
    }
    if (rc) return rc;
    const long total = (long)M * N;
    const bool vec = N % 4 == 0 && ldc % 4 == 0 && (epi != EPI_F32_RESID || ldaux % 4 == 0) &&
                     ((uintptr_t)C & 15) == 0 && ((uintptr_t)aux & 15) == 0 && ((uintptr_t)bias & 15) == 0;
    if (vec)
      hipLaunchKernelGGL(k_splitk_reduce4, dim3((unsigned)((total / 4 + 255) / 256)), dim3(256), 0, st, g, splitk, epi);
    else
      hipLaunchKernelGGL(k_splitk_reduce, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, g, splitk, epi);
    VJ_LAUNCH_CHECK("vj_gemm_bf16_splitk(reduce)");
    return VJ_OK;
  }
  if (a_kmajor && b_kmajor) return launch_epi<true, true>(epi, g, grid, st);
  if (a_kmajor && !b_kmajor) return launch_epi<true, false>(epi, g, grid, st);
  if (!a_kmajor && b_kmajor) return launch_epi<false, true>(epi, g, grid, st);
  return launch_epi<false, false>(epi, g, grid, st);
}

extern "C" int vj_gemm_bf16_splitk(int M, int N, int K, const void* A, long lda, int a_kmajor, const void* B,
                                   long ldb, int b_kmajor, int epi, const float* bias, const void* aux, long ldaux,
                                   void* C, long ldc, void* C2, long ldc2, int splitk, float* ws, long ws_floats,
                                   void* stream) {
  return gemm_splitk(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, epi, bias, aux, ldaux, C, ldc, C2, ldc2, splitk, ws,
                     ws_floats, stream, nullptr, 0, nullptr);
}

extern "C" int vj_colsum_f32(int M, int N, const void* x, int x_bf16, long ld, float* out, int accumulate, float* ws,
                             long ws_floats, void* stream);

// nn.Linear's weight and bias gradients from one read of dY: dw[M, N] (+)= dY^T X and db[M] (+)=
// dY.sum(0), with dY [K, M] and X [K, N] row-major (K = tokens). Split-K as vj_gemm_bf16_splitk;
// the bias sums ride in the 256-row partial kernel (v_dot2 of the dY fragments it already holds)
// when it runs, else a column-sum pass follows (same results up to f32 summation order).
extern "C" int vj_gemm_bf16_wgrad(int M, int N, int K, const void* dy, long lddy, const void* x, long ldx,
                                  float* dw, long lddw, int accumulate, float* db, int db_accumulate, int splitk,
                                  float* ws, long ws_floats, void* stream) {
  VJ_CHECK_ARG(dw, "vj_gemm_bf16_wgrad: null dw");
  int done = 0;
  const int rc = gemm_splitk(M, N, K, dy, lddy, 0, x, ldx, 0, accumulate ? EPI_F32_RESID : EPI_F32, nullptr,
                             accumulate ? dw : nullptr, lddw, dw, lddw, nullptr, 0, splitk, ws, ws_floats, stream, db,
                             db_accumulate, &done);
  if (rc || !db || done || M == 0) return rc;
  return vj_colsum_f32(K, M, dy, 1, lddy, db, db_accumulate, ws, ws_floats, stream);
}

extern "C" int vj_gemm_bf16(int M, int N, int K, const void* A, long lda, int a_kmajor, const void* B, long ldb,
                            int b_kmajor, int epi, const float* bias, const void* aux, long ldaux, void* C, long ldc,
                            void* C2, long ldc2, void* stream) {
  return vj_gemm_bf16_splitk(M, N, K, A, lda, a_kmajor, B, ldb, b_kmajor, epi, bias, aux, ldaux, C, ldc, C2, ldc2, 1,
                             nullptr, 0, stream);
}
