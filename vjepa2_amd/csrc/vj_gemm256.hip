// Large-tile bf16 GEMM for gfx950: 256 x BN x 64 tiles (BN = 256 or 128), 512 threads = 8 waves
// (2 in M x 4 in N), one workgroup per CU (LDS 128 / 96 KB), v_mfma_f32_16x16x32_bf16.
// Same operand/epilogue contract as vj_gemm.hip (K-major or MN-major A and B, fused epilogues);
// used for the forward and data-gradient GEMMs of the encoder / predictor blocks (M = tokens).
//
// Schedule (per wave, tile t in LDS slot t&1): 4 phases per K-tile = (k-step, M-half), each
// 4 x NTN MFMAs on a 64x(BN/4) quarter of the wave tile; the next phase's fragments (16 + 16 VGPRs,
// double-buffered) are read from LDS while the current phase's MFMAs run, so LDS latency hides under
// MFMA with 128 accumulator + 64 fragment registers (no spill at 2 waves / SIMD). ONE barrier per
// tile (before the last phase): it retires this wave's DMA of tile t+1 (issued one tile earlier)
// and its reads of tile t; tile t+2 is then DMA'd into slot t&1 and stays in flight across it. Epilogue: accumulators staged through LDS (conflict-free padded image) and written as
// whole 16-B row segments with bias / residual / GELU fused.
#include <stdlib.h>
#include "vj_common.h"

namespace {

enum { EPI_BF16 = 0, EPI_F32 = 1, EPI_F32_RESID = 2, EPI_GELU = 3, EPI_GELU_BWD = 4, EPI_ROPE = 5, EPI_PARTIAL = 6 };

// 3-axis RoPE applied to the q and k columns of a fused QKV projection (modules.py:26-50, 343-365)
struct RopeP {
  const int* ids;   // token id per row (NULL -> row % mod)
  int mod, tpf, tpr;
  int half, hd, D;  // half = slice/2, head dim, q/k block width (= H * hd)
  const float* cos_t;
  const float* sin_t;
  int npos;         // table rows (positions); every position of every id is < npos <= 1024
};

struct G256 {
  const bf16_t* A;
  const bf16_t* B;
  int M, N, K;
  long lda, ldb;
  void* C;
  long ldc;
  void* C2;
  long ldc2;
  const float* bias;
  const void* aux;
  long ldaux;
  int tiles_m, tiles_n;
  RopeP rope;
  int kslice;  // EPI_PARTIAL: blockIdx.y = K slice z covers [z*kslice, min(K, (z+1)*kslice))
  float* ws;   // EPI_PARTIAL: f32 partial products [splitk][M][N]
};

constexpr int BK = 64;

__device__ __forceinline__ uint32_t clampb(long b) {
  if (b < 0) return 0;
  return b > 0x7fffffffL ? 0x7fffffffu : (uint32_t)b;
}

__device__ __forceinline__ int mn_swz(int k) { return 2 * (k & 3) + 8 * ((k >> 3) & 1); }

// K-major image: [ROWS][64] bf16, 128-B rows, chunk ^= (row>>1)&7.
// MN-major image: [64][ROWS] bf16, ROWS*2-B rows, chunk ^= mn_swz(k).
// PERM (K-major B only): LDS row r of each WN-row group holds global row NTN*(r%16) + r/16 of the
// group, so n-tile j of the MFMA accumulators covers the group's columns {NTN*c + j}: each lane
// then owns NTN CONSECUTIVE output columns and the epilogue stores straight from registers.
template <bool KMAJ, int ROWS, bool PERM = false>
__device__ __forceinline__ void stage(__amdgpu_buffer_rsrc_t rs, long ld, int rows_left, int k0, int K,
                                      LDS_AS char* lds, int wave, int lane) {
  constexpr int PIECES = ROWS / 8;  // 1-KB DMA pieces per operand tile
#pragma unroll
  for (int i = 0; i < PIECES / 8; ++i) {
    const int p = wave * (PIECES / 8) + i;
    uint32_t voff;
    if constexpr (KMAJ) {
      const int r = p * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int kk = k0 + c * 8;
      int gr = r;
      if constexpr (PERM) {
        constexpr int WN = ROWS / 4, NTN = WN / 16;
        const int rl = r % WN;
        gr = (r - rl) + NTN * (rl & 15) + (rl >> 4);
      }
      voff = (gr < rows_left && kk < K) ? (uint32_t)(((long)gr * ld + kk) * 2) : VJ_OOB;
    } else {
      constexpr int CPR = ROWS / 8;     // chunks per LDS row
      constexpr int RPP = 64 / CPR;     // k-rows per piece
      const int kr = p * RPP + lane / CPR;
      const int c = (lane % CPR) ^ mn_swz(kr);
      const int col = c * 8;
      voff = (k0 + kr < K && col < rows_left) ? (uint32_t)(((long)(k0 + kr) * ld + col) * 2) : VJ_OOB;
    }
    dma16(rs, lds + p * 1024, voff);
  }
}

// 16x16x32 operand fragment: lane l holds X(rb + (l&15), 32s + 8(l>>4) + j), j = 0..7.
template <bool KMAJ, int ROWS>
__device__ __forceinline__ bf16x8 frag(const LDS_AS char* lds, int rb, int s, int lane) {
  if constexpr (KMAJ) {
    const int r = rb + (lane & 15);
    const int c = (4 * s + (lane >> 4)) ^ ((r >> 1) & 7);
    return *(const LDS_AS bf16x8*)(lds + r * 128 + c * 16);
  } else {
    const int gi = lane & 15;
    const int k0 = 32 * s + 8 * (lane >> 4) + (gi >> 2);
    const int col = rb + 4 * (gi & 3);
    const int within = (col & 7) * 2;
    const int c = col >> 3;
    const s16x4 lo = ds_read_tr16_async(lds + k0 * (ROWS * 2) + ((c ^ mn_swz(k0)) * 16) + within);
    const s16x4 hi = ds_read_tr16_async(lds + (k0 + 4) * (ROWS * 2) + ((c ^ mn_swz(k0 + 4)) * 16) + within);
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// erf with |abs err| <= 1.5e-7 (Abramowitz-Stegun 7.1.26): far below the bf16 rounding of the output.
__device__ __forceinline__ float erf_fast(float z) {
  const float a = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float r = 1.f - p * __expf(-a * a);
  return copysignf(r, z);
}
__device__ __forceinline__ float gelu_fast(float x) { return 0.5f * x * (1.f + erf_fast(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad_fast(float x) {
  return 0.5f * (1.f + erf_fast(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}

template <bool AK, bool BKM, int EPI, int BN>
__global__ __launch_bounds__(512, 2) void k_gemm256(G256 g) {
  constexpr int BM = 256;
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int WN = BN / 4;      // wave tile columns (64 / 32)
  constexpr int NTN = WN / 16;    // 16-wide n tiles per wave (4 / 2)
  constexpr int NH = NTN / 2;     // n tiles per N-half register set
  // K-major B with 4 n-tiles per wave: permuted B staging + stores straight from registers (16-B
  // f32 / 8-B bf16 per row); 128-wide tiles would store 4-8 B per lane, so they keep the LDS path
  constexpr bool DIRECT = BKM && NTN == 4;
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * STAGE];
  LDS_AS char* smem = (LDS_AS char*)smem_raw;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  // XCD-aware bijective remap: each XCD (blocks b % 8) takes a contiguous run of tiles, n fastest.
  const int nb = g.tiles_m * g.tiles_n;
  const int b = blockIdx.x, xcd = b & 7, q = nb >> 3, rmd = nb & 7;
  const int wg = (xcd < rmd ? xcd * (q + 1) : rmd * (q + 1) + (xcd - rmd) * q) + (b >> 3);
  const int tm = wg / g.tiles_n, tn = wg - tm * g.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // split-K (EPI_PARTIAL): this block's K range starts at kb; Keff = its length
  const int kb = EPI == EPI_PARTIAL ? (int)blockIdx.y * g.kslice : 0;
  const int Keff = EPI == EPI_PARTIAL ? min(g.K, kb + g.kslice) - kb : g.K;
  const bf16_t* abase = AK ? g.A + (long)m0 * g.lda + kb : g.A + (long)kb * g.lda + m0;
  const bf16_t* bbase = BKM ? g.B + (long)n0 * g.ldb + kb : g.B + (long)kb * g.ldb + n0;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(
      abase, AK ? clampb((long)(g.M - m0) * g.lda * 2 - kb * 2L) : clampb(((long)(g.K - kb) * g.lda - m0) * 2));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(
      bbase, BKM ? clampb((long)(g.N - n0) * g.ldb * 2 - kb * 2L) : clampb(((long)(g.K - kb) * g.ldb - n0) * 2));
  const int mleft = g.M - m0, nleft = g.N - n0;
  const int nk = (Keff + BK - 1) / BK;

  f32x4 acc[8][NTN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NTN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 Aa[4], Ab[4], Ba[NTN], Bb[NTN];
  // RoPE epilogue operands, fetched now so their latency hides under the main loop: the token id
  // of tile row tid and entry tid of the cos/sin tables.
  int pf_id = 0;
  float pf_c = 0.f, pf_s = 0.f;
  if constexpr (EPI == EPI_ROPE) {
    const int t = threadIdx.x;
    if (t < BM && m0 + t < g.M) pf_id = g.rope.ids ? g.rope.ids[m0 + t] : (m0 + t) % g.rope.mod;
    if (t < g.rope.npos * g.rope.half) {
      pf_c = g.rope.cos_t[t];
      pf_s = g.rope.sin_t[t];
    }
  }

  auto load_tile = [&](int t) {
    LDS_AS char* s = smem + (t & 1) * STAGE;
    stage<AK, BM>(ra, g.lda, mleft, t * BK, Keff, s, wave, lane);
    stage<BKM, BN, DIRECT>(rb, g.ldb, nleft, t * BK, Keff, s + A_BYTES, wave, lane);
  };
  // A fragments of M-half mh (4 m-tiles), k-step ks; B fragments of all NTN n-tiles, k-step ks
  auto rdA = [&](bf16x8 (&X)[4], int t, int mh, int ks) {
    const LDS_AS char* s = smem + (t & 1) * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) X[i] = frag<AK, BM>(s, wr * 128 + (mh * 4 + i) * 16, ks, lane);
  };
  auto rdB = [&](bf16x8 (&Y)[NTN], int t, int ks) {
    const LDS_AS char* s = smem + (t & 1) * STAGE + A_BYTES;
#pragma unroll
    for (int j = 0; j < NTN; ++j) Y[j] = frag<BKM, BN>(s, wc * WN + j * 16, ks, lane);
  };
  auto mm = [&](const bf16x8 (&X)[4], int mh, const bf16x8 (&Y)[NTN]) {
#if VJ_GEMM_PRIO
    __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NTN; ++j)
        acc[mh * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(X[i], Y[j], acc[mh * 4 + i][j], 0, 0, 0);
#if VJ_GEMM_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  };

  // prologue: tiles 0 and 1 in flight, then the first fragments (phase 0 of tile 0)
  load_tile(0);
  if (nk > 1) load_tile(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  rdA(Aa, 0, 0, 0);
  rdB(Ba, 0, 0);

  // Per K-tile t: 4 phases (k-step, M-half) = (0,0) (0,1) (1,0) (1,1), 4*NTN MFMAs each; the
  // fragments of the NEXT phase are read while the current phase's MFMAs run. One barrier per
  // tile, before phase 3 (whose prefetch reads tile t+1): it retires this wave's DMA of tile t+1
  // (issued one tile earlier) and its reads of tile t; then tile t+2 is DMA'd into slot t&1.
  // MN-major operands are read with asm transposed reads (ds_read_tr16_async): each phase first
  // waits for the fragments it consumes (read in the previous phase), then issues the next reads.
  constexpr bool ASYNC = !AK || !BKM;
  auto release = [&](bf16x8 (&X)[4], bf16x8 (&Y)[NTN]) {
    if constexpr (ASYNC) {
      lds_wait();
      tie(X);
      tie(Y);
    }
  };
  for (int t = 0; t < nk; ++t) {
    release(Aa, Ba);
    rdA(Ab, t, 1, 0);
    __builtin_amdgcn_sched_barrier(0);
    mm(Aa, 0, Ba);
    __builtin_amdgcn_sched_barrier(0);
    release(Ab, Ba);
    rdA(Aa, t, 0, 1);
    rdB(Bb, t, 1);
    __builtin_amdgcn_sched_barrier(0);
    mm(Ab, 1, Ba);
    __builtin_amdgcn_sched_barrier(0);
    release(Aa, Bb);
    rdA(Ab, t, 1, 1);
    __builtin_amdgcn_sched_barrier(0);
    mm(Aa, 0, Bb);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if constexpr (ASYNC) {
      tie(Ab);
      tie(Bb);
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 2 < nk) load_tile(t + 2);
    if (t + 1 < nk) {
      rdA(Aa, t + 1, 0, 0);
      rdB(Ba, t + 1, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    mm(Ab, 1, Bb);
    __builtin_amdgcn_sched_barrier(0);
  }

  if constexpr (DIRECT) {
    // ---- direct epilogue (K-major B staged with PERM): lane (c = lane&15, g = lane>>4) owns rows
    // i*16 + 4g + r of m-tile i and the NTN consecutive columns nb .. nb+NTN-1, so every row goes
    // out of registers as one 8/16-B store; no LDS round trip.
    const int nb = n0 + wc * WN + NTN * (lane & 15);
    const bool nok = nb < g.N;
    const int mb = m0 + wr * 128 + 4 * (lane >> 4);
    float bias[NTN];
#pragma unroll
    for (int j = 0; j < NTN; ++j) bias[j] = 0.f;
    if (EPI != EPI_GELU_BWD && EPI != EPI_PARTIAL && g.bias && nok)
#pragma unroll
      for (int j = 0; j < NTN; ++j) bias[j] = g.bias[nb + j];
    // RoPE (modules.py:26-50, 343-365): tile rows' (frame, row, col) positions + interleaved
    // cos/sin table in LDS; this lane's NTN/2 column pairs fix slice/axis/frequency once.
    [[maybe_unused]] LDS_AS int* rpos = (LDS_AS int*)smem;
    [[maybe_unused]] LDS_AS f32x2* rtab = (LDS_AS f32x2*)(smem + BM * 4);
    [[maybe_unused]] bool ract[NTN / 2];
    [[maybe_unused]] int rsh[NTN / 2], rf0[NTN / 2], rf1[NTN / 2];
    if constexpr (EPI == EPI_ROPE) {
      __syncthreads();  // every wave is done with the operand stages
      const RopeP& r = g.rope;
      const int t = threadIdx.x;
      if (t < BM) {
        const int fr = pf_id / r.tpf, rem = pf_id - r.tpf * fr, hr = rem / r.tpr;
        rpos[t] = fr | (hr << 10) | ((rem - r.tpr * hr) << 20);
      }
      const int ntab = r.npos * r.half;
      if (t < ntab) rtab[t] = f32x2{pf_c, pf_s};
      for (int i = t + 512; i < ntab; i += 512) rtab[i] = f32x2{r.cos_t[i], r.sin_t[i]};
      const int sw = 2 * r.half, e0 = (nb % r.D) % r.hd;
#pragma unroll
      for (int p = 0; p < NTN / 2; ++p) {
        const int e = e0 + 2 * p, ax = e / sw, js = e - ax * sw;
        ract[p] = nok && nb < 2 * r.D && e < 3 * sw;
        rsh[p] = 10 * ax;
        rf0[p] = js % r.half;
        rf1[p] = (js + 1) % r.half;
      }
      __syncthreads();
    }
    // residual (f32) / pre-activation (bf16) rows: m-tile i+1's fetched while m-tile i is stored
    constexpr bool AUX = EPI == EPI_F32_RESID || EPI == EPI_GELU_BWD;
    [[maybe_unused]] float aux[2][4][NTN];
    auto fetch = [&](int i, float (&dst)[4][NTN]) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mb + i * 16 + r;
        const bool ok = m < g.M && nok;
        const long off = ok ? (long)m * g.ldaux + nb : 0;
        if constexpr (EPI == EPI_F32_RESID) {
          if constexpr (NTN == 4) {
            const float4 x = *(const float4*)((const float*)g.aux + off);
            dst[r][0] = x.x; dst[r][1] = x.y; dst[r][2] = x.z; dst[r][3] = x.w;
          } else {
            const float2 x = *(const float2*)((const float*)g.aux + off);
            dst[r][0] = x.x; dst[r][1] = x.y;
          }
        } else {
          if constexpr (NTN == 4) {
            const uint2 x = *(const uint2*)((const bf16_t*)g.aux + off);
            dst[r][0] = bf2f(x.x & 0xffff); dst[r][1] = bf2f(x.x >> 16);
            dst[r][2] = bf2f(x.y & 0xffff); dst[r][3] = bf2f(x.y >> 16);
          } else {
            const uint32_t x = *(const uint32_t*)((const bf16_t*)g.aux + off);
            dst[r][0] = bf2f(x & 0xffff); dst[r][1] = bf2f(x >> 16);
          }
        }
      }
    };
    if constexpr (AUX) fetch(0, aux[0]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (AUX) {
        if (i + 1 < 8) fetch(i + 1, aux[(i + 1) & 1]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mb + i * 16 + r;
        if (m >= g.M || !nok) continue;
        float v[NTN];
#pragma unroll
        for (int j = 0; j < NTN; ++j) v[j] = acc[i][j][r] + bias[j];
        if constexpr (EPI == EPI_ROPE) {
          const int rp = rpos[wr * 128 + i * 16 + 4 * (lane >> 4) + r];
#pragma unroll
          for (int p = 0; p < NTN / 2; ++p) {
            if (!ract[p]) continue;
            const int pos = min((rp >> rsh[p]) & 1023, g.rope.npos - 1) * g.rope.half;
            const f32x2 a = rtab[pos + rf0[p]], b = rtab[pos + rf1[p]];
            const float x0 = v[2 * p], x1 = v[2 * p + 1];
            v[2 * p] = x0 * a[0] - x1 * a[1];
            v[2 * p + 1] = x1 * b[0] + x0 * b[1];
          }
        }
        if constexpr (EPI == EPI_F32_RESID) {
#pragma unroll
          for (int j = 0; j < NTN; ++j) v[j] += aux[i & 1][r][j];
        }
        if constexpr (EPI == EPI_F32 || EPI == EPI_F32_RESID || EPI == EPI_PARTIAL) {
          float* dst = EPI == EPI_PARTIAL ? g.ws + ((long)blockIdx.y * g.M + m) * g.N + nb
                                          : (float*)g.C + (long)m * g.ldc + nb;
          if constexpr (NTN == 4) *(float4*)dst = make_float4(v[0], v[1], v[2], v[3]);
          else *(float2*)dst = make_float2(v[0], v[1]);
        } else {
          uint32_t pk[NTN / 2];
#pragma unroll
          for (int q = 0; q < NTN / 2; ++q) {
            if constexpr (EPI == EPI_GELU_BWD)
              pk[q] = pack_bf2(v[2 * q] * gelu_grad_fast(aux[i & 1][r][2 * q]),
                               v[2 * q + 1] * gelu_grad_fast(aux[i & 1][r][2 * q + 1]));
            else
              pk[q] = pack_bf2(v[2 * q], v[2 * q + 1]);
          }
          if (EPI != EPI_GELU || g.C) {
            bf16_t* dst = (bf16_t*)g.C + (long)m * g.ldc + nb;
            if constexpr (NTN == 4) *(uint2*)dst = make_uint2(pk[0], pk[1]);
            else *(uint32_t*)dst = pk[0];
          }
          if constexpr (EPI == EPI_GELU) {
            uint32_t ga[NTN / 2];
#pragma unroll
            for (int q = 0; q < NTN / 2; ++q)
              ga[q] = pack_bf2(gelu_fast(bf2f(pk[q] & 0xffff)), gelu_fast(bf2f(pk[q] >> 16)));
            bf16_t* dst2 = (bf16_t*)g.C2 + (long)m * g.ldc2 + nb;
            if constexpr (NTN == 4) *(uint2*)dst2 = make_uint2(ga[0], ga[1]);
            else *(uint32_t*)dst2 = ga[0];
          }
        }
      }
    }
    return;
  }
  // ---- epilogue: 4 passes of 2 m-tiles (32 rows) per wave through a padded LDS image
  constexpr int STR = WN + 4;  // floats per staged row (conflict-free ds_write_b32)
  constexpr int LPR = WN / 4;  // lanes per staged row (16-B each)
  constexpr int RPI = 64 / LPR;  // rows per wave-instruction
  __syncthreads();
  LDS_AS float* wl = (LDS_AS float*)(smem + wave * 32 * STR * 4);
  // RoPE (modules.py:26-50, 343-365) on q/k columns: the tile rows' (frame, row, col) positions and
  // the interleaved cos/sin table go to LDS behind the staging image; each thread's 4 columns fix
  // its slice/axis/frequency once, so a store costs 1 + 4 LDS reads and 8 FMAs.
  constexpr int ROPE_OFF = 8 * 32 * STR * 4;
  LDS_AS int* rpos = (LDS_AS int*)(smem + ROPE_OFF);
  LDS_AS f32x2* rtab = (LDS_AS f32x2*)(smem + ROPE_OFF + BM * 4);
  bool ract[2] = {false, false};
  int rsh[2] = {0, 0}, rf0[2] = {0, 0}, rf1[2] = {0, 0};
  if constexpr (EPI == EPI_ROPE) {
    const RopeP& r = g.rope;
    const int t = threadIdx.x;
    if (t < BM) {
      const int fr = pf_id / r.tpf, rem = pf_id - r.tpf * fr, hr = rem / r.tpr;
      rpos[t] = fr | (hr << 10) | ((rem - r.tpr * hr) << 20);
    }
    const int ntab = r.npos * r.half;
    if (t < ntab) rtab[t] = f32x2{pf_c, pf_s};
    for (int i = t + 512; i < ntab; i += 512) rtab[i] = f32x2{r.cos_t[i], r.sin_t[i]};
    const int n = n0 + wc * WN + (lane % LPR) * 4, sw = 2 * r.half, e0 = (n % r.D) % r.hd;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int e = e0 + 2 * p, ax = e / sw, js = e - ax * sw;
      ract[p] = n < 2 * r.D && e < 3 * sw;
      rsh[p] = 10 * ax;
      rf0[p] = js % r.half;
      rf1[p] = (js + 1) % r.half;
    }
    __syncthreads();
  }
  const int col = (lane % LPR) * 4;  // this thread's 4 columns, fixed for every row it stores
  const int ncol = n0 + wc * WN + col;
  float4 bias4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (EPI != EPI_GELU_BWD && EPI != EPI_PARTIAL && g.bias && ncol < g.N) bias4 = *(const float4*)(g.bias + ncol);
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < NTN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          wl[(ii * 16 + (lane >> 4) * 4 + r) * STR + j * 16 + (lane & 15)] = acc[pass * 2 + ii][j][r];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own writes visible to own reads (wave-private)
    // residual / GELU pre-activation rows of this pass fetched up front: one memory latency per
    // pass instead of one per row
    constexpr int IT = 32 / RPI;
    [[maybe_unused]] float4 rres[EPI == EPI_F32_RESID ? IT : 1];
    [[maybe_unused]] uint2 rpre[EPI == EPI_GELU_BWD ? IT : 1];
    if constexpr (EPI == EPI_F32_RESID || EPI == EPI_GELU_BWD) {
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int m = m0 + wr * 128 + pass * 32 + it * RPI + lane / LPR;
        const bool ok = m < g.M && ncol < g.N;
        const long mm = ok ? m : 0;
        const int nn = ok ? ncol : 0;
        if constexpr (EPI == EPI_F32_RESID) rres[it] = *(const float4*)((const float*)g.aux + mm * g.ldaux + nn);
        else rpre[it] = *(const uint2*)((const bf16_t*)g.aux + mm * g.ldaux + nn);
      }
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int row = it * RPI + lane / LPR;
      const f32x4 v4 = *(const LDS_AS f32x4*)(wl + row * STR + col);
      const int m = m0 + wr * 128 + pass * 32 + row;
      const int n = ncol;
      if (m >= g.M || n >= g.N) continue;
      float v[4] = {v4[0] + bias4.x, v4[1] + bias4.y, v4[2] + bias4.z, v4[3] + bias4.w};
      if constexpr (EPI == EPI_BF16 || EPI == EPI_ROPE) {
        if constexpr (EPI == EPI_ROPE) {
          const int rp = rpos[wr * 128 + pass * 32 + row];
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            if (!ract[p]) continue;
            const int pos = min((rp >> rsh[p]) & 1023, g.rope.npos - 1) * g.rope.half;
            const f32x2 a = rtab[pos + rf0[p]], b = rtab[pos + rf1[p]];
            const float x0 = v[2 * p], x1 = v[2 * p + 1];
            v[2 * p] = x0 * a[0] - x1 * a[1];
            v[2 * p + 1] = x1 * b[0] + x0 * b[1];
          }
        }
        *(uint2*)((bf16_t*)g.C + (long)m * g.ldc + n) = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
      } else if constexpr (EPI == EPI_F32) {
        *(float4*)((float*)g.C + (long)m * g.ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
      } else if constexpr (EPI == EPI_PARTIAL) {
        *(float4*)(g.ws + ((long)blockIdx.y * g.M + m) * g.N + n) = make_float4(v[0], v[1], v[2], v[3]);
      } else if constexpr (EPI == EPI_F32_RESID) {
        const float4 rr = rres[it];
        *(float4*)((float*)g.C + (long)m * g.ldc + n) = make_float4(rr.x + v[0], rr.y + v[1], rr.z + v[2], rr.w + v[3]);
      } else if constexpr (EPI == EPI_GELU) {
        const uint32_t p0 = pack_bf2(v[0], v[1]), p1 = pack_bf2(v[2], v[3]);
        if (g.C) *(uint2*)((bf16_t*)g.C + (long)m * g.ldc + n) = make_uint2(p0, p1);
        const float x0 = bf2f(p0 & 0xffff), x1 = bf2f(p0 >> 16), x2 = bf2f(p1 & 0xffff), x3 = bf2f(p1 >> 16);
        *(uint2*)((bf16_t*)g.C2 + (long)m * g.ldc2 + n) =
            make_uint2(pack_bf2(gelu_fast(x0), gelu_fast(x1)), pack_bf2(gelu_fast(x2), gelu_fast(x3)));
      } else {  // EPI_GELU_BWD
        const uint2 pu = rpre[it];
        const float x0 = bf2f(pu.x & 0xffff), x1 = bf2f(pu.x >> 16), x2 = bf2f(pu.y & 0xffff), x3 = bf2f(pu.y >> 16);
        *(uint2*)((bf16_t*)g.C + (long)m * g.ldc + n) =
            make_uint2(pack_bf2(v[0] * gelu_grad_fast(x0), v[1] * gelu_grad_fast(x1)),
                       pack_bf2(v[2] * gelu_grad_fast(x2), v[3] * gelu_grad_fast(x3)));
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
  }
}

template <bool AK, bool BKM, int BN>
int launch256(int epi, const G256& g, hipStream_t st, int splitk = 1) {
  dim3 grid(g.tiles_m * g.tiles_n, splitk);
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_BF16, BN>), grid, dim3(512), 0, st, g); break;
    case EPI_F32: hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_F32, BN>), grid, dim3(512), 0, st, g); break;
    case EPI_F32_RESID: hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_F32_RESID, BN>), grid, dim3(512), 0, st, g); break;
    case EPI_GELU: hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_GELU, BN>), grid, dim3(512), 0, st, g); break;
    case EPI_GELU_BWD: hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_GELU_BWD, BN>), grid, dim3(512), 0, st, g); break;
    case EPI_ROPE: hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_ROPE, BN>), grid, dim3(512), 0, st, g); break;
    case EPI_PARTIAL:  // split-K weight gradients only: dY^T X, both operands MN-major
      if constexpr (!AK && !BKM) {
        hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_PARTIAL, BN>), grid, dim3(512), 0, st, g);
        break;
      } else {
        return VJ_ERR_UNSUPPORTED;
      }
    default: vj_set_error("gemm256: bad epilogue %d", epi); return VJ_ERR_ARG;
  }
  VJ_LAUNCH_CHECK("vj_gemm256");
  return VJ_OK;
}

}  // namespace

// Called by vj_gemm_bf16_splitk (splitk == 1) when the problem suits a 256-row tile; arguments
// already validated there. Returns VJ_ERR_UNSUPPORTED when it declines.
int vj_gemm256_dispatch(int M, int N, int K, const void* A, long lda, int a_kmajor, const void* B, long ldb,
                        int b_kmajor, int epi, const float* bias, const void* aux, long ldaux, void* C, long ldc,
                        void* C2, long ldc2, hipStream_t st, const void* rope) {
  if (epi < EPI_BF16 || epi > EPI_ROPE || N % 8 || ldc % 4 || ldc2 % 4 || ldaux % 4) return VJ_ERR_UNSUPPORTED;
  if (((uintptr_t)C & 15) || ((uintptr_t)C2 & 15) || ((uintptr_t)aux & 15) || ((uintptr_t)bias & 15))
    return VJ_ERR_UNSUPPORTED;
  const int bn = (N % 256 == 0) ? 256 : 128;
  G256 g{(const bf16_t*)A, (const bf16_t*)B, M, N, K, lda, ldb, C, ldc, C2, ldc2, bias, aux, ldaux,
         vj_cdiv(M, 256), vj_cdiv(N, bn), RopeP{}, 0, nullptr};
  if (epi == EPI_ROPE) {
    if (!rope) return VJ_ERR_UNSUPPORTED;
    g.rope = *(const RopeP*)rope;
    if (g.rope.hd % 4 || g.rope.D % 4 || g.rope.npos < 1 || g.rope.npos > 1024) return VJ_ERR_UNSUPPORTED;
    const long lds_need = 8L * 32 * (bn / 4 + 4) * 4 + 256 * 4 + (long)g.rope.npos * g.rope.half * 8;
    if (lds_need > 2L * (256 * BK * 2 + bn * BK * 2)) return VJ_ERR_UNSUPPORTED;
  }
  if (bn == 256) {
    if (a_kmajor && b_kmajor) return launch256<true, true, 256>(epi, g, st);
    if (a_kmajor && !b_kmajor) return launch256<true, false, 256>(epi, g, st);
    if (!a_kmajor && b_kmajor) return launch256<false, true, 256>(epi, g, st);
    return launch256<false, false, 256>(epi, g, st);
  }
  if (a_kmajor && b_kmajor) return launch256<true, true, 128>(epi, g, st);
  if (a_kmajor && !b_kmajor) return launch256<true, false, 128>(epi, g, st);
  if (!a_kmajor && b_kmajor) return launch256<false, true, 128>(epi, g, st);
  return launch256<false, false, 128>(epi, g, st);
}

// Split-K partial products ws[z] = A[:, z-th K slice] B[z-th K slice, :]^T (f32, [splitk][M][N]) with
// 256-row tiles; the caller reduces the slabs. Returns VJ_ERR_UNSUPPORTED when it declines.
int vj_gemm256_partial(int M, int N, int K, const void* A, long lda, int a_kmajor, const void* B, long ldb,
                       int b_kmajor, int kslice, int splitk, float* ws, hipStream_t st) {
  if (a_kmajor || b_kmajor || N % 8 || M < 256 || N < 128) return VJ_ERR_UNSUPPORTED;
  const int bn = (N % 256 == 0) ? 256 : 128;
  G256 g{(const bf16_t*)A, (const bf16_t*)B, M, N, K, lda, ldb, nullptr, 0, nullptr, 0, nullptr, nullptr, 0,
         vj_cdiv(M, 256), vj_cdiv(N, bn), RopeP{}, kslice, ws};
  if (splitk > 65535) return VJ_ERR_UNSUPPORTED;
  return bn == 256 ? launch256<false, false, 256>(EPI_PARTIAL, g, st, splitk)
                   : launch256<false, false, 128>(EPI_PARTIAL, g, st, splitk);
}

extern "C" int vj_gemm_bf16(int M, int N, int K, const void* A, long lda, int a_kmajor, const void* B, long ldb,
                            int b_kmajor, int epi, const float* bias, const void* aux, long ldaux, void* C, long ldc,
                            void* C2, long ldc2, void* stream);
extern "C" int vj_rope(int T, int H, int hd, void* qkv, long ld, int q_off, int k_off, const int* ids, int ids_mod,
                       int tokens_per_frame, int tokens_per_row, const float* cos_tab, const float* sin_tab, int half,
                       int inverse, void* stream);

// Fused QKV projection + 3-axis RoPE of q and k (modules.py:330 + 343-365): one launch whose epilogue
// rotates the f32 accumulator rows before the bf16 store; falls back to GEMM + vj_rope for shapes
// the 256-row kernel declines.
extern "C" int vj_qkv_rope_gemm(int M, int K, const void* A, long lda, const void* B, long ldb, const float* bias,
                                void* C, long ldc, int H, int hd, const int* ids, int ids_mod, int tpf, int tpr,
                                const float* cos_t, const float* sin_t, int npos, void* stream) {
  if (M == 0) return VJ_OK;
  const int N = 3 * H * hd;
  VJ_CHECK_ARG(hd % 8 == 0 && cos_t && sin_t && (ids || ids_mod > 0), "vj_qkv_rope_gemm: bad rope arguments");
  VJ_CHECK_ARG(tpf > 0 && tpr > 0 && npos > 0, "vj_qkv_rope_gemm: tokens_per_frame/row and npos must be > 0");
  const int half = (hd / 3) / 2;
  const char* e = getenv("VJ_GEMM256");
  if (M >= 1024 && !(e && e[0] == '0')) {
    RopeP rp{ids, ids_mod, tpf, tpr, half, hd, H * hd, cos_t, sin_t, npos};
    const int rc = vj_gemm256_dispatch(M, N, K, A, lda, 1, B, ldb, 1, EPI_ROPE, bias, nullptr, 0, C, ldc, nullptr, 0,
                                       (hipStream_t)stream, &rp);
    if (rc != VJ_ERR_UNSUPPORTED) return rc;
  }
  int rc = vj_gemm_bf16(M, N, K, A, lda, 1, B, ldb, 1, EPI_BF16, bias, nullptr, 0, C, ldc, nullptr, 0, stream);
  if (rc) return rc;
  return vj_rope(M, H, hd, C, ldc, 0, H * hd, ids, ids_mod, tpf, tpr, cos_t, sin_t, half, 0, stream);
}
