// Ping-pong bf16 GEMM for gfx950: the forward and data-gradient GEMMs of the encoder / predictor
// blocks (K-major A and B: X W^T and dY (W^T)^T), with every fused epilogue of vj_gemm256.hip
// (bias, f32 / bf16 residual, GELU(erf) + GELU', GELU backward, QKV RoPE).
//
// Why: in the one-tile-per-workgroup kernel (vj_gemm256.hip) all 8 waves finish a 256 x 256 tile's
// K-loop together and then run its epilogue together, so the matrix cores idle for the whole
// epilogue (~33k of ~88k cycles per tile at K = 1024: residual reads, GELU's transcendentals, stores).
// Here the 8 waves form two groups of 4, one wave of each group per SIMD, and each group owns its own
// 256 x 128 tiles; the groups alternate: while group g runs the K-loop of its tile i (MFMA), group
// 1-g runs the epilogue of its tile i-1 (VALU + memory) on the same SIMDs. The SIMD's vector-issue
// slots left free by the MFMAs (8 of every 16 cycles of a 16x16x32 MFMA) carry the epilogue.
//
// Pipeline: ONE ring of 3 LDS stages (48 KB each: A 256 x 64, B 128 x 64 bf16) carries the K-tiles
// of the block's tiles in order (tile 0's K-tiles, tile 1's, ...; tile p belongs to group p & 1).
// Barrier b (one per K-tile, workgroup-wide) is reached by the K-loop group after its reads of
// K-tile b and by the epilogue group between two slices of its epilogue: the epilogue of a tile is
// cut into as many slices as the running K-loop has K-tiles. The K-loop group DMAs K-tile b + 3 right
// after barrier b (into the slot K-tile b frees) and retires it (vmcnt) before barrier b + 2; across
// a group hand-over the finishing group retires its last DMA at the start of its epilogue, before
// the next barrier. Per wave the tile is 128 x 64 (8 x 4 MFMA tiles of 16 x 16, 128 accumulator
// VGPRs), the K-loop is the 4-phase schedule of vj_gemm256.hip (fragments of the next phase read
// under the current phase's MFMAs), and B is staged row-permuted so each lane owns 4 consecutive
// output columns and the epilogue stores straight from registers.
//
// M32 = true: the same pipeline on v_mfma_f32_32x32x16_bf16. One 32x32x16 MFMA holds its SIMD's
// vector-issue port for 8 of its 32 cycles (the 16x16x32 form: 8 of 16), so the epilogue group gets
// three times the issue slots per flop. Per wave the tile is 64 x 128 (2 x 4 accumulator blocks of
// 32 x 32, the 4 waves of a group stacked in M), B is staged with a 32-row permutation (LDS row r of
// the 128-row tile holds global row 4 (r % 32) + r / 32, so lane l again owns 4 consecutive output
// columns 4 (l & 31) .. + 3), and each K-tile's 12 DMA pieces are spread over four phases (3 per
// phase: the 8 MFMAs of a phase cannot cover 12 pieces' issue) — pieces 0-2 of K-tile b + 3 after
// barrier b, pieces 3-11 in the three phases before barrier b + 1, so the vmcnt(12) count is unchanged.
//
// Requirements (host-checked, else the caller falls back): A and B K-major, K % 64 == 0 (no K-tail:
// DMA offsets are per-lane constants plus a scalar k offset), K >= 192 (a tile has at least as many
// K-tiles as the ring has stages), N % 8 == 0, 16-B aligned pointers.
#include <stdlib.h>
#include <type_traits>
#include "vj_gemm_tile.h"

#ifndef VJ_PP_PRIO
#define VJ_PP_PRIO 1  // K-loop group at s_setprio 1 (the epilogue group's VALU yields to its issue)
#endif

namespace {

constexpr int NST = 3;          // LDS stages of the K-tile ring
constexpr int DMA_PIECES = 12;  // 1-KB LDS-DMA pieces per wave per K-tile (A 8 + B 4)
constexpr int PP_RPOS_BYTES = 8 * 128 * 4;  // per-wave RoPE row positions (128 rows x 8 waves)
constexpr int PP_ROPE_TAB_MAX = (TAB_BYTES - PP_RPOS_BYTES) / 8;

// 16-B LDS-DMA with a scalar byte offset (the K position of the tile)
__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t r, LDS_AS void* lds_wave_base, uint32_t voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, lds_wave_base, 16, voff, soff, 0, 0);
}

template <int EPI, bool M32>
__global__ __launch_bounds__(512, 2) void k_gemm_pp(G256 g) {
  constexpr int BM = 256, BN = 128, NTN = 4;
  constexpr int WN = M32 ? 128 : 64;  // wave tile columns (M32: one wave column, 4 wave rows of 64)
  constexpr int WM = M32 ? 64 : 128;  // wave tile rows
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr bool AUX = EPI == EPI_F32_RESID || EPI == EPI_GELU_BWD || EPI == EPI_BF16_RESID;
  constexpr bool F32OUT = EPI == EPI_F32 || EPI == EPI_F32_RESID;
  static_assert(EPI != EPI_PARTIAL, "split-K partials stay on k_gemm256");
  // NST stages (3: 144 KB) + the RoPE tables: the whole 160 KB of the CU
  __shared__ __attribute__((aligned(16))) char smem_raw[NST * STAGE + TAB_BYTES];
  LDS_AS char* smem = (LDS_AS char*)smem_raw;
  LDS_AS char* tab = smem + NST * STAGE;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wave >> 2, w4 = wave & 3, wr = M32 ? w4 : w4 >> 1, wc = M32 ? 0 : w4 & 1;

  // Persistent walk (as k_gemm256): the logical tiles are cut into 8 runs, one per XCD; the P
  // blocks of an XCD walk its run with stride P. This block's tiles: first, first + P, ...
  const int ntile = g.tiles_m * g.tiles_n;
  const int P = gridDim.x >> 3;
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int q = ntile >> 3, rmd = ntile & 7;
  const int run0 = xcd < rmd ? xcd * (q + 1) : rmd * (q + 1) + (xcd - rmd) * q;
  const int runend = run0 + q + (xcd < rmd ? 1 : 0);
  const int first = run0 + jb;
  if (first >= runend) return;
  const int ntl = __builtin_amdgcn_readfirstlane((runend - first + P - 1) / P);
  const int nk = __builtin_amdgcn_readfirstlane(g.K / BK);
  const int nkt = ntl * nk;

  auto make_tile = [&](int p) {
    Tile T;
    const int w = first + p * P;
    int tm, tn;
    if (g.group > 0) {
      const int per = g.group * g.tiles_n, gi = w / per, f = gi * g.group;
      const int gm = min(g.tiles_m - f, g.group), loc = w - gi * per;
      tm = f + loc % gm;
      tn = loc / gm;
    } else {
      tm = w / g.tiles_n;
      tn = w - tm * g.tiles_n;
    }
    T.m0 = __builtin_amdgcn_readfirstlane(tm * BM);
    T.n0 = __builtin_amdgcn_readfirstlane(tn * BN);
    T.z = 0;
    T.Keff = g.K;
    T.nk = nk;
    return T;
  };

  // Per-lane DMA offsets, fixed for the whole kernel (K % 64 == 0: no K-tail). A: group wave w4
  // issues pieces 8 w4 + i (8 rows of 128 B each, chunk ^= (row >> 1) & 7); B (row-permuted, see
  // stage() in vj_gemm_tile.h): pieces 4 w4 + i. Piece i's offset = base[i & 1] + i-dependent rows.
  uint32_t aoff[2], boff[2];
  {
    const int r8 = lane >> 3;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int ra = w4 * 64 + e * 8 + r8;
      const int ca = (lane & 7) ^ ((ra >> 1) & 7);
      aoff[e] = (uint32_t)(ra * g.lda * 2 + ca * 16);
      const int rb = w4 * 32 + e * 8 + r8;  // LDS row
      int gr;
      if constexpr (M32) {  // LDS row r -> global row 4 (r % 32) + r / 32 (the whole 128-row tile)
        gr = 4 * (rb & 31) + (rb >> 5);
      } else {
        const int rl = rb % WN;
        gr = (rb - rl) + NTN * (rl & 15) + (rl >> 4);
      }
      const int cb = (lane & 7) ^ ((rb >> 1) & 7);
      boff[e] = (uint32_t)(gr * g.ldb * 2 + cb * 16);
    }
  }
  // Buffer descriptors of tile p's A and B panels (the range check zero-fills rows past M / N)
  auto tile_rsrc = [&](int p, __amdgpu_buffer_rsrc_t& ra, __amdgpu_buffer_rsrc_t& rb) {
    const Tile T = make_tile(min(p, ntl - 1));
    ra = make_rsrc(g.A + (long)T.m0 * g.lda, clampb((long)(g.M - T.m0) * g.lda * 2));
    rb = make_rsrc(g.B + (long)T.n0 * g.ldb, clampb((long)(g.N - T.n0) * g.ldb * 2));
  };
  // One K-tile (k offset kb bytes) -> LDS slot `slot`, issued by the calling group's 4 waves;
  // kill = VJ_OOB makes every piece out of range (zero-fill dummies past the block's last K-tile,
  // so every K-tile issues the same number of pieces and the vmcnt counts stay constant)
  // Piece q (0-7: A, 8-11: B) of one K-tile: A rows (w4 * 8 + q) * 8 .. + 7 = base + 16 (q >> 1)
  // rows; B LDS rows (w4 * 4 + i) * 8 .. + 7 (global rows permuted): piece i & 1 shifted by the
  // permutation's row step (16-wide: 1 global row per 16 LDS rows; M32: 64 global rows per 16)
  constexpr int BSTEP = M32 ? 64 : 1;
  auto dma_piece = [&](__amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int kb, uint32_t kill, LDS_AS char* s,
                       int q) {
    if (q < 8)
      dma16s(ra, s + (w4 * 8 + q) * 1024, (aoff[q & 1] + (uint32_t)((q >> 1) * 16 * g.lda * 2)) | kill, kb);
    else
      dma16s(rb, s + A_BYTES + (w4 * 4 + (q - 8)) * 1024,
             (boff[q & 1] + (uint32_t)(((q - 8) >> 1) * BSTEP * g.ldb * 2)) | kill, kb);
  };
  auto dma_issue = [&](__amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int kb, uint32_t kill, int slot,
                       int q0 = 0, int q1 = DMA_PIECES) {
    LDS_AS char* s = smem + slot * STAGE;
#pragma unroll
    for (int q = 0; q < DMA_PIECES; ++q)
      if (q >= q0 && q < q1) dma_piece(ra, rb, kb, kill, s, q);
  };

  // RoPE tables: interleaved cos/sin (read once per workgroup) behind the per-wave row positions
  constexpr int RTR = EPI == EPI_ROPE ? (PP_ROPE_TAB_MAX + 511) / 512 : 0;
  [[maybe_unused]] LDS_AS int* rposw = (LDS_AS int*)tab + wave * 128;
  [[maybe_unused]] LDS_AS f32x2* rtab = (LDS_AS f32x2*)(tab + PP_RPOS_BYTES);
  [[maybe_unused]] const int ntab = EPI == EPI_ROPE ? g.rope.npos * g.rope.half : 0;
  if constexpr (EPI == EPI_ROPE) {
    f32x2 rpf[RTR];
#pragma unroll
    for (int i = 0; i < RTR; ++i) {
      const int e = threadIdx.x + 512 * i;
      rpf[i] = e < ntab ? f32x2{g.rope.cos_t[e], g.rope.sin_t[e]} : f32x2{0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < RTR; ++i) {
      const int e = threadIdx.x + 512 * i;
      if (e < ntab) rtab[e] = rpf[i];
    }
  }
  if (grp == 0) {  // the first NST K-tiles (all of tile 0: nk >= NST); M32: of K-tile 2 only the
    // pieces 0-2 (its pieces 3-11 are issued in K-tile 0's phases 0-2)
    __amdgpu_buffer_rsrc_t ra, rb;
    tile_rsrc(0, ra, rb);
    for (int v = 0; v < NST; ++v) dma_issue(ra, rb, v * BK * 2, 0u, v, 0, M32 && v == NST - 1 ? 3 : DMA_PIECES);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  [[maybe_unused]] f32x4 acc[8][NTN];
  [[maybe_unused]] f32x16 acc32[2][NTN];  // M32: [m-block][n-block], 32 x 32 each
  bf16x8 Aa[4], Ab[4], Ba[NTN], Bb[NTN];
  // accumulator of row group i (4 rows: 16-wide m-tile i; M32: m-block i >> 2, register quad i & 3),
  // n-tile j, row r of the group
  auto accv = [&](int i, int j, int r) -> float {
    if constexpr (M32) return acc32[i >> 2][j][4 * (i & 3) + r];
    else return acc[i][j][r];
  };
  // Fragment reads (the K-major frag() of vj_gemm_tile.h, written out): every fragment row block
  // starts at a multiple of 16 rows, so the XOR swizzle depends on the lane only and a read is
  // slot base + wave base + lane offset (one VGPR per k-step) + a compile-time immediate. Three
  // 48-KB slots do not fit the 64-KB ds_read offset field, so the per-slot base is added per read
  // group instead of being folded into precomputed addresses (which cost ~30 VGPRs).
  uint32_t loff[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) loff[ks] = (lane & 15) * 128 + (((4 * ks + (lane >> 4)) ^ ((lane >> 1) & 7)) * 16);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  auto rdA = [&](bf16x8 (&X)[4], int slot, int mh, int ks) {
    const uint32_t base = lds0 + slot * STAGE + wr * 128 * 128;
    const LDS_AS char* p = (const LDS_AS char*)(uintptr_t)(base + loff[ks]);
#pragma unroll
    for (int i = 0; i < 4; ++i) X[i] = *(const LDS_AS bf16x8*)(p + (mh * 4 + i) * 16 * 128);
  };
  auto rdB = [&](bf16x8 (&Y)[NTN], int slot, int ks) {
    const uint32_t base = lds0 + slot * STAGE + A_BYTES + wc * WN * 128;
    const LDS_AS char* p = (const LDS_AS char*)(uintptr_t)(base + loff[ks]);
#pragma unroll
    for (int j = 0; j < NTN; ++j) Y[j] = *(const LDS_AS bf16x8*)(p + j * 16 * 128);
  };
  auto mm = [&](const bf16x8 (&X)[4], int mh, const bf16x8 (&Y)[NTN]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NTN; ++j)
        acc[mh * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(X[i], Y[j], acc[mh * 4 + i][j], 0, 0, 0);
  };

  // single-fragment reads and one phase = 16 MFMAs on (M-half mh) x (4 n-tiles), each followed by
  // side(q) (reads / DMA for later phases), the order pinned by scheduling barriers
  auto rdA1 = [&](bf16x8 (&X)[4], int i, int slot, int mh, int ks) {
    const uint32_t base = lds0 + slot * STAGE + wr * 128 * 128;
    X[i] = *(const LDS_AS bf16x8*)((const LDS_AS char*)(uintptr_t)(base + loff[ks]) + (mh * 4 + i) * 16 * 128);
  };
  auto rdB1 = [&](bf16x8 (&Y)[NTN], int j, int slot, int ks) {
    const uint32_t base = lds0 + slot * STAGE + A_BYTES + wc * WN * 128;
    Y[j] = *(const LDS_AS bf16x8*)((const LDS_AS char*)(uintptr_t)(base + loff[ks]) + j * 16 * 128);
  };
  auto phase = [&](const bf16x8 (&X)[4], int mh, const bf16x8 (&Y)[NTN], auto&& side) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      acc[mh * 4 + (q >> 2)][q & 3] =
          __builtin_amdgcn_mfma_f32_16x16x32_bf16(X[q >> 2], Y[q & 3], acc[mh * 4 + (q >> 2)][q & 3], 0, 0, 0);
      side(q);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- the K-loop of one tile (nk barriers); u0 = its first K-tile in the pipeline
  // The K-loop of tile p (first K-tile u0 of the pipeline). After barrier b = u0 + t it DMAs K-tile
  // b + NST: K-tile t + NST of this tile, else K-tile t + NST - nk of tile p + 1 (nk >= NST), whose
  // descriptors are built once here (no per-K-tile division / tile arithmetic on the scalar unit).
  auto kloop = [&](int u0, int p) {
    __amdgpu_buffer_rsrc_t raC, rbC, raN, rbN;
    tile_rsrc(p, raC, rbC);
    tile_rsrc(p + 1, raN, rbN);
    const uint32_t killN = p + 1 < ntl ? 0u : VJ_OOB;
#if VJ_PP_PRIO
    __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NTN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    rdA(Aa, u0 % NST, 0, 0);
    rdB(Ba, u0 % NST, 0);
    int sl = u0 % NST;  // slot of K-tile u0 + t
    for (int t = 0; t < nk; ++t) {
      const int sn = sl + 1 == NST ? 0 : sl + 1;
      // phases 0-2: 16 MFMAs each with the next phase's fragment reads issued one per MFMA gap
      // (a lone wave per SIMD drives the matrix pipe here: nothing may bunch in front of the MFMAs)
      phase(Aa, 0, Ba, [&](int q) { if (q < 4) rdA1(Ab, q, sl, 1, 0); });
      phase(Ab, 1, Ba, [&](int q) {
        if (q < 4) rdA1(Aa, q, sl, 0, 1);
        else if (q < 8) rdB1(Bb, q - 4, sl, 1);
      });
      phase(Aa, 0, Bb, [&](int q) { if (q < 4) rdA1(Ab, q, sl, 1, 1); });
      // Retire K-tile b + 1 = u0 + t + 1 and this wave's reads of K-tile b: every K-tile issues
      // exactly DMA_PIECES pieces per wave (past the last K-tile of the block they are dummies into
      // the freed slot), so "all but the youngest DMA_PIECES" leaves only K-tile b + 2 in flight.
      // For t < 2 the K-tiles b + 1 came from the other group (retired at the start of its
      // epilogue) and this wave's older VMEM ops are its epilogue's stores, drained before the
      // epilogue's last barrier: the same wait is then a no-op.
      static_assert(NST == 3 && DMA_PIECES == 12, "vmcnt count written for 3 stages x 12 pieces");
      asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // phase 3 (the K-tile's last 16 MFMAs) with the next K-tile's phase-0 fragments (past the
      // tile's last K-tile: harmless reads of the next tile's data, overwritten before use) and the
      // 12 LDS-DMA pieces of K-tile b + NST (into slot sl, just freed) issued in its MFMA gaps
      {
        const int td = t + NST;
        const bool own = td < nk;
        const __amdgpu_buffer_rsrc_t ra = own ? raC : raN, rb = own ? rbC : rbN;
        const int kb = (own ? td : td - nk) * BK * 2;
        const uint32_t kill = own ? 0u : killN;
        LDS_AS char* st = smem + sl * STAGE;
        phase(Ab, 1, Bb, [&](int q) {
          if (q < 4) rdA1(Aa, q, sn, 0, 0);
          else if (q < 8) rdB1(Ba, q - 4, sn, 0);
          if (q < DMA_PIECES) dma_piece(ra, rb, kb, kill, st, q);
        });
      }
      sl = sn;
    }
#if VJ_PP_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  };

  // ---- M32: 32x32x16 fragments. Lane l reads row (l & 31) of a 32-row block, 16-B chunk
  // 2 ks + (l >> 5) of k-step ks (16 deep); the K-major swizzle (chunk ^= (row >> 1) & 7) keeps every
  // 16-lane quarter on 16 distinct bank slots. A: the wave's 2 m-blocks (rows wr * 64 + 32 i), B: the
  // tile's 4 n-blocks (LDS rows 32 j, permuted at staging).
  [[maybe_unused]] uint32_t loff32[4];
  if constexpr (M32) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      loff32[ks] = (lane & 31) * 128 + (((2 * ks + (lane >> 5)) ^ (((lane & 31) >> 1) & 7)) * 16);
  }
  // fragment q of a k-step: q < 2 A m-block q (into X), else B n-block q - 2 (into Y)
  auto rd32 = [&](bf16x8 (&X)[4], bf16x8 (&Y)[NTN], int q, int slot, int ks) {
    const uint32_t base = lds0 + slot * STAGE + loff32[ks];
    if (q < 2) X[q] = *(const LDS_AS bf16x8*)((const LDS_AS char*)(uintptr_t)(base + wr * 64 * 128) + q * 32 * 128);
    else Y[q - 2] = *(const LDS_AS bf16x8*)((const LDS_AS char*)(uintptr_t)(base + A_BYTES) + (q - 2) * 32 * 128);
  };
  // one k-step = 8 MFMAs (2 m-blocks x 4 n-blocks), each followed by side(q)
  auto phase32 = [&](const bf16x8 (&X)[4], const bf16x8 (&Y)[NTN], auto&& side) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      acc32[q >> 2][q & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(X[q >> 2], Y[q & 3], acc32[q >> 2][q & 3], 0, 0, 0);
      side(q);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // The M32 K-loop of tile p. In K-tile iteration b = u0 + t: phases 0-2 (k-steps 0-2) issue pieces
  // 3-11 of K-tile b + 2 (into its slot, freed at barrier b - 1), phase 3 (after barrier b) pieces
  // 0-2 of K-tile b + 3 (into slot b, just freed). K-tile b + 2 is then complete before the wait
  // ahead of barrier b + 1, whose vmcnt(12) leaves exactly its 12 pieces in flight. A group's first
  // K-tile continues the K-tile b + 2 the other group started in its last phase 3.
  auto kloop32 = [&](int u0, int p) {
    __amdgpu_buffer_rsrc_t raC, rbC, raN, rbN;
    tile_rsrc(p, raC, rbC);
    tile_rsrc(p + 1, raN, rbN);
    const uint32_t killN = p + 1 < ntl ? 0u : VJ_OOB;
#if VJ_PP_PRIO
    __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NTN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc32[i][j][e] = 0.f;
    int sl = u0 % NST;  // slot of K-tile u0 + t
#pragma unroll
    for (int q = 0; q < 6; ++q) rd32(Aa, Ba, q, sl, 0);
    for (int t = 0; t < nk; ++t) {
      const int sn = sl + 1 == NST ? 0 : sl + 1;
      const int sp = sn + 1 == NST ? 0 : sn + 1;  // slot of K-tile b + 2 (= b - 1)
      {  // pieces 3-11 of K-tile b + 2: three per phase, in the gaps after MFMAs 1, 4, 7
        const int td = t + 2;
        const bool own = td < nk;
        const __amdgpu_buffer_rsrc_t ra = own ? raC : raN, rb = own ? rbC : rbN;
        const int kb = (own ? td : td - nk) * BK * 2;
        const uint32_t kill = own ? 0u : killN;
        LDS_AS char* st = smem + sp * STAGE;
        auto dq = [&](int ph, int q) {
          if (q == 1 || q == 4 || q == 7) dma_piece(ra, rb, kb, kill, st, 3 + 3 * ph + (q == 1 ? 0 : q == 4 ? 1 : 2));
        };
        phase32(Aa, Ba, [&](int q) { if (q < 6) rd32(Ab, Bb, q, sl, 1); dq(0, q); });
        phase32(Ab, Bb, [&](int q) { if (q < 6) rd32(Aa, Ba, q, sl, 2); dq(1, q); });
        phase32(Aa, Ba, [&](int q) { if (q < 6) rd32(Ab, Bb, q, sl, 3); dq(2, q); });
      }
      static_assert(NST == 3 && DMA_PIECES == 12, "vmcnt count written for 3 stages x 12 pieces");
      asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      {  // phase 3: k-step 3, the next K-tile's k-step-0 fragments, pieces 0-2 of K-tile b + 3
        const int td = t + NST;
        const bool own = td < nk;
        const __amdgpu_buffer_rsrc_t ra = own ? raC : raN, rb = own ? rbC : rbN;
        const int kb = (own ? td : td - nk) * BK * 2;
        const uint32_t kill = own ? 0u : killN;
        LDS_AS char* st = smem + sl * STAGE;
        phase32(Ab, Bb, [&](int q) {
          if (q < 6) rd32(Aa, Ba, q, sn, 0);
          if (q == 1 || q == 4 || q == 7) dma_piece(ra, rb, kb, kill, st, q == 1 ? 0 : q == 4 ? 1 : 2);
        });
      }
      sl = sn;
    }
#if VJ_PP_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  };

  // ---- the epilogue of one tile, cut by `nbar` barriers (0: the block's last tile, nothing runs
  // beside it); m-tile i (16 rows of the wave tile) is followed by barriers up to (i + 1) nbar / 8
  auto epilogue = [&](const Tile& cur, int nbar) {
    int lane_e = lane;
    asm volatile("" : "+v"(lane_e));  // epilogue addressing is not hoisted into the K-loop
    const int lane = lane_e;
    // m-tiles spread over the first ~3/4 of the barriers; the stores are then drained (vmcnt(0))
    // before the last barriers, so the next K-loop of this wave starts with no VMEM op pending
    int done = 0;
    const int nfront = nbar - (nbar >> 2);
    auto bars = [&](int i) {
      const int tgt = ((i + 1) * nfront) >> 3;
      while (done < tgt) {
        __builtin_amdgcn_s_barrier();
        ++done;
      }
    };
    // lane's 4 columns nb .. nb + 3; row r of row group i: mb + rofs(i) + r (16-wide: m-tile i, rows
    // 4 (lane >> 4) + r; M32: m-block i >> 2, rows 8 (i & 3) + 4 (lane >> 5) + r of the block)
    const int nb = cur.n0 + wc * WN + NTN * (lane & (M32 ? 31 : 15));
    const bool nok = nb < g.N;
    const int mrow = M32 ? 4 * (lane >> 5) : 4 * (lane >> 4);  // row of the lane within a row group
    const int mb = cur.m0 + wr * WM + mrow;
    auto rofs = [](int i) { return M32 ? (i >> 2) * 32 + (i & 3) * 8 : i * 16; };
    float bias[NTN];
#pragma unroll
    for (int j = 0; j < NTN; ++j) bias[j] = 0.f;
    if (EPI != EPI_GELU_BWD && g.bias && nok)
#pragma unroll
      for (int j = 0; j < NTN; ++j) bias[j] = g.bias[nb + j];
    [[maybe_unused]] bool ract[NTN / 2];
    [[maybe_unused]] int rsh[NTN / 2], rf0[NTN / 2], rf1[NTN / 2];
    if constexpr (EPI == EPI_ROPE) {
      const VjRope& r = g.rope;
      // this wave's WM rows: (frame | row << 10 | col << 20), wave-private LDS
#pragma unroll
      for (int h = 0; h < WM / 64; ++h) {
        const int m = cur.m0 + wr * WM + lane + 64 * h;
        int id = 0;
        if (m < g.M) id = r.ids ? r.ids[m] : m % r.mod;
        const int fr = id / r.tpf, rem = id - r.tpf * fr, hr = rem / r.tpr;
        rposw[lane + 64 * h] = fr | (hr << 10) | ((rem - r.tpr * hr) << 20);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int sw = 2 * r.half, e0 = (nb % r.D) % r.hd;
#pragma unroll
      for (int p = 0; p < NTN / 2; ++p) {
        const int e = e0 + 2 * p, ax = e / sw, js = e - ax * sw;
        ract[p] = nok && nb < 2 * r.D && e < 3 * sw;
        rsh[p] = 10 * ax;
        rf0[p] = js % r.half;
        rf1[p] = (js + 1) % r.half;
      }
    }
    constexpr int AUX_PF = VJ_GEMM_AUX_PF;
    [[maybe_unused]] float aux[AUX_PF + 1][4][NTN];
    auto fetch = [&](int i, float (&dst)[4][NTN]) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mb + rofs(i) + r;
        const bool ok = m < g.M && nok;
        const long off = ok ? (long)m * g.ldaux + nb : 0;
        if constexpr (EPI == EPI_F32_RESID) {
          const float4 x = *(const float4*)((const float*)g.aux + off);
          dst[r][0] = x.x; dst[r][1] = x.y; dst[r][2] = x.z; dst[r][3] = x.w;
        } else {
          auto lo = [](uint32_t u) { return __builtin_bit_cast(float, u << 16); };
          auto hi = [](uint32_t u) { return __builtin_bit_cast(float, u & 0xffff0000u); };
          const uint2 x = *(const uint2*)((const bf16_t*)g.aux + off);
          dst[r][0] = lo(x.x); dst[r][1] = hi(x.x);
          dst[r][2] = lo(x.y); dst[r][3] = hi(x.y);
        }
      }
    };
    const bool odd = lane & 1;
    const int nb8 = nb - (odd ? 4 : 0);
    const bool nok8 = nb8 < g.N;
    auto store_wide = [&](bf16_t* base, long ld, int i, const uint32_t (&pk)[4][2]) {
      uint32_t snd[4], rcv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) snd[k] = odd ? pk[k >> 1][k & 1] : pk[2 + (k >> 1)][k & 1];
#pragma unroll
      for (int k = 0; k < 4; ++k) rcv[k] = dpp_u<DPP_XOR1>(snd[k]);  // lane pair exchange on the VALU
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = odd ? 2 + h : h;
        const int m = mb + rofs(i) + r;
        if (m < g.M && nok8) {
          const uint4 v = odd ? make_uint4(rcv[2 * h], rcv[2 * h + 1], pk[r][0], pk[r][1])
                              : make_uint4(pk[r][0], pk[r][1], rcv[2 * h], rcv[2 * h + 1]);
          *(uint4*)(base + (long)m * ld + nb8) = v;
        }
      }
    };
    if constexpr (AUX)
#pragma unroll
      for (int i = 0; i < AUX_PF; ++i) fetch(i, aux[i]);
    auto rows = [&](auto save_c) {
      constexpr bool SAVE_D = decltype(save_c)::value;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (AUX) {
          if (i + AUX_PF < 8) fetch(i + AUX_PF, aux[(i + AUX_PF) % (AUX_PF + 1)]);
        }
        if constexpr (F32OUT) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = mb + rofs(i) + r;
            float v[NTN];
#pragma unroll
            for (int j = 0; j < NTN; ++j) {
              v[j] = accv(i, j, r) + bias[j];
              if constexpr (EPI == EPI_F32_RESID) v[j] += aux[i % (AUX_PF + 1)][r][j];
            }
            if (m < g.M && nok) *(float4*)((float*)g.C + (long)m * g.ldc + nb) = make_float4(v[0], v[1], v[2], v[3]);
          }
        } else {
          uint32_t pk[4][2], ga[4][2];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v[NTN];
#pragma unroll
            for (int j = 0; j < NTN; ++j) v[j] = accv(i, j, r) + bias[j];
            if constexpr (EPI == EPI_ROPE) {
              const int rp = rposw[rofs(i) + mrow + r];
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
            if constexpr (EPI == EPI_BF16_RESID) {
#pragma unroll
              for (int j = 0; j < NTN; ++j) v[j] += aux[i % (AUX_PF + 1)][r][j];
            }
#pragma unroll
            for (int q2 = 0; q2 < 2; ++q2) {
              if constexpr (EPI == EPI_GELU_BWD)
                pk[r][q2] = pack_bf2(v[2 * q2] * aux[i % (AUX_PF + 1)][r][2 * q2],
                                     v[2 * q2 + 1] * aux[i % (AUX_PF + 1)][r][2 * q2 + 1]);
              else
                pk[r][q2] = pack_bf2(v[2 * q2], v[2 * q2 + 1]);
              if constexpr (EPI == EPI_GELU) ga[r][q2] = gelu_pair(pk[r][q2], SAVE_D ? &pk[r][q2] : nullptr);
            }
          }
          if (EPI != EPI_GELU || SAVE_D) store_wide((bf16_t*)g.C, g.ldc, i, pk);
          if constexpr (EPI == EPI_GELU) store_wide((bf16_t*)g.C2, g.ldc2, i, ga);
        }
        bars(i);
      }
    };
    if (EPI == EPI_GELU && g.C) rows(std::true_type{});
    else rows(std::false_type{});
    if (nbar > 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      while (done < nbar) {
        __builtin_amdgcn_s_barrier();
        ++done;
      }
    }
  };

  // ---- periods: in period p group (p & 1) runs tile p's K-loop, the other group the epilogue of
  // its tile p - 1 (or, in period 0, only the barriers)
  int u0 = 0;
  for (int p = 0; p < ntl; ++p, u0 += nk) {
    if ((p & 1) == grp) {
      if constexpr (M32) kloop32(u0, p);
      else kloop(u0, p);
    } else if (p == 0) {
      for (int b = 0; b < nk; ++b) __builtin_amdgcn_s_barrier();
    } else {
      // the DMAs this group issued after its last NST - 1 barriers (the next tile's first K-tiles)
      // are read after the coming barriers: retire them before the epilogue's first barrier
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      epilogue(make_tile(p - 1), nk);
    }
  }
  // the block's last tile: its group finishes alone (no K-loop left to pace against)
  if (((ntl - 1) & 1) == grp) epilogue(make_tile(ntl - 1), 0);
}

template <int EPI>
void launch_pp(bool m32, dim3 gr, hipStream_t st, const G256& g) {
  if (m32) hipLaunchKernelGGL((k_gemm_pp<EPI, true>), gr, dim3(512), 0, st, g);
  else hipLaunchKernelGGL((k_gemm_pp<EPI, false>), gr, dim3(512), 0, st, g);
}

}  // namespace

// Which K-major GEMMs come here: VJ_GEMM_PP=0 none, =1 all, unset: the epilogues in the bit mask
// VJ_GEMM_PP_EPIS (default none). Measured (tools/bench_kernels.py @VJ_GEMM_PP=0 @VJ_GEMM_PP=1,
// MI355X): faster only on the context / predictor QKV + RoPE shapes (76 vs 84-87 us), slower on the
// target QKV and every other epilogue (the lone-wave K-loop runs at ~0.9 of the two-wave one and
// the epilogues do not fully hide under it); the step measured 192.2 clips/s with the RoPE shapes
// routed here vs 193.4 without (bench.py A/B in one call), so the default stays k_gemm256.
// VJ_GEMM_PP=2 (or the epilogue's bit in VJ_GEMM_PP32_EPIS) selects the M32 (32x32x16) form.
// Returns 0 (k_gemm256), 1 (ping-pong, 16x16x32) or 2 (ping-pong, 32x32x16).
int vj_gemm_pp_mode(int epi) {
  const char* e = getenv("VJ_GEMM_PP");
  if (e && (e[0] == '0' || e[0] == '1' || e[0] == '2')) return e[0] - '0';
  const char* m2 = getenv("VJ_GEMM_PP32_EPIS");
  if (m2 && ((strtol(m2, nullptr, 0) >> epi) & 1)) return 2;
  const char* m = getenv("VJ_GEMM_PP_EPIS");
  return (m && ((strtol(m, nullptr, 0) >> epi) & 1)) ? 1 : 0;
}

// Called by vj_gemm256_dispatch for K-major A and B; VJ_ERR_UNSUPPORTED when the shape is not one
// this kernel takes (the caller then uses k_gemm256).
int vj_gemm_pp_dispatch(int M, int N, int K, const void* A, long lda, const void* B, long ldb, int epi,
                        const float* bias, const void* aux, long ldaux, void* C, long ldc, void* C2, long ldc2,
                        hipStream_t st, const void* rope, int group, int grid, int mode) {
  if (K % BK || K < NST * BK || N % 8) return VJ_ERR_UNSUPPORTED;  // whole K-tiles, nk >= NST
  if (epi == EPI_PARTIAL || epi < EPI_BF16 || (epi > EPI_ROPE && epi != EPI_BF16_RESID)) return VJ_ERR_UNSUPPORTED;
  if ((long)(M + 255) * lda * 2 > 0x7fffffffL || (long)(N + 127) * ldb * 2 > 0x7fffffffL) return VJ_ERR_UNSUPPORTED;
  const int tm = vj_cdiv(M, 256), tn = vj_cdiv(N, 128);
  G256 g{(const bf16_t*)A, (const bf16_t*)B, M, N, K, lda, ldb, C, ldc, C2, ldc2, bias, aux, ldaux,
         tm, tn, VjRope{}, K, 1, nullptr, group};
  if (epi == EPI_ROPE) {
    if (!rope) return VJ_ERR_UNSUPPORTED;
    g.rope = *(const VjRope*)rope;
    if ((long)g.rope.npos * g.rope.half > PP_ROPE_TAB_MAX) return VJ_ERR_UNSUPPORTED;
  }
  const dim3 gr(grid);
  const bool m32 = mode == 2;
  switch (epi) {
    case EPI_BF16: launch_pp<EPI_BF16>(m32, gr, st, g); break;
    case EPI_F32: launch_pp<EPI_F32>(m32, gr, st, g); break;
    case EPI_F32_RESID: launch_pp<EPI_F32_RESID>(m32, gr, st, g); break;
    case EPI_GELU: launch_pp<EPI_GELU>(m32, gr, st, g); break;
    case EPI_GELU_BWD: launch_pp<EPI_GELU_BWD>(m32, gr, st, g); break;
    case EPI_ROPE: launch_pp<EPI_ROPE>(m32, gr, st, g); break;
    case EPI_BF16_RESID: launch_pp<EPI_BF16_RESID>(m32, gr, st, g); break;
    default: return VJ_ERR_UNSUPPORTED;
  }
  VJ_LAUNCH_CHECK("vj_gemm_pp");
  return VJ_OK;
}
