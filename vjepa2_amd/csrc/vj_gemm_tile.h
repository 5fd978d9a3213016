// Device helpers of the 256-row bf16 / fp8 GEMM kernel (vj_gemm256.hip): the kernel argument block, LDS-DMA
// staging of K-major / MN-major operand tiles with the XOR swizzles, MFMA fragment reads and the
// GELU epilogue pair. Everything sits in an anonymous namespace: each translation unit compiles
// its own copy (no cross-TU codegen coupling of the kernels).
#pragma once
#include "vj_common.h"

namespace {

// epilogue numbering: vj_common.h (EPI_BF16_RESID: the no-grad target encoder's residual stream in the
// reference's own autocast precision, x = x + proj(...) in bf16, half the epilogue bytes of F32_RESID)

using RopeP = VjRope;

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
  int kslice;  // K range of one K slice (= K unless EPI_PARTIAL)
  int nsplit;  // K slices: slice z covers [z*kslice, min(K, (z+1)*kslice)) (EPI_PARTIAL only; else 1)
  float* ws;   // EPI_PARTIAL: f32 partial products [nsplit][M][N]
  int group;   // tile rows per group of the grouped tile order (0: row-major, n fastest)
  // F8 kernels: A / B are fp8 e4m3 (OCP) viewed as bf16 pairs (K, lda, ldb above in 2-byte units);
  // ea[m] / eb[n] = power-of-two exponents of the per-row (A: token) / per-row (B: output channel)
  // scales: A(m, k) = a8 * 2^ea[m], B(n, k) = b8 * 2^eb[n] (E8M0 scale operands of the MFMA)
  const int* ea = nullptr;
  const int* eb = nullptr;
  // EPI_PARTIAL: f32 row sums of A over each K slice, [nsplit][M] (the bias gradient fused into a
  // weight-gradient GEMM: A = dY^T, so row m of A summed over the tokens is db[m]); null: none
  float* rsum = nullptr;
};

constexpr int BK = 64;
// LDS behind the two operand stages for the per-kernel tables: the GELU tables (f32 derivative:
// 13 KB) or the RoPE tile positions (1 KB) + interleaved cos/sin table (npos * half * 8 B).
constexpr int TAB_BYTES = 16384;
constexpr int ROPE_TAB_MAX = (TAB_BYTES - 256 * 4) / 8;  // cos/sin pairs that fit behind the positions

__device__ __forceinline__ uint32_t clampb(long b) {
  if (b < 0) return 0;
  return b > 0x7fffffffL ? 0x7fffffffu : (uint32_t)b;
}

__device__ __forceinline__ int mn_swz(int k) { return 2 * (k & 3) + 8 * ((k >> 3) & 1); }

// 64-B K-major rows (32-deep K tiles): the 16-B chunk swizzle. A 16x16x32 fragment read (row rb + (l &
// 15), chunk l >> 4) is serviced in the lane groups {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, {32-35,
// 44-47, 52-59}, {36-43, 48-51, 60-63} (MI355X_MICROARCH.md, LDS), each of which holds rows j, j+4,
// j+8, j+12 at chunks (g, g^1, g^1, g) for some g: conflict-free iff swz over the row quarters
// q = (r >> 2) & 3 makes {swz(0), swz(1)^1, swz(2)^1, swz(3)} distinct. swz = 3 * (q >> 1) does;
// (r >> 2) & 3 (used until round 5) gave {0, 0, 3, 3}: every group 2-way conflicted (PMC: bank-conflict
// cycles = half the LDS cycles of the staggered GEMM).
__device__ __forceinline__ int kswz32(int r) { return 3 * ((r >> 3) & 1); }

// K-major image: [ROWS][64] bf16, 128-B rows, chunk ^= (row>>1)&7 ([ROWS][32]: 64-B rows, kswz32).
// MN-major image: [64][ROWS] bf16, ROWS*2-B rows, chunk ^= mn_swz(k).
// PERM (K-major B only): LDS row r of each WN-row group holds global row NTN*(r%PB) + r/PB of the
// group (PB = the MFMA output block width, 16 or 32; NTN = WN / PB), so n block j of the MFMA
// accumulators covers the group's columns {NTN*c + j}: each lane then owns NTN CONSECUTIVE output
// columns and the epilogue stores straight from registers.
// NW waves issue the tile's 1-KB pieces (waves 0 .. NW-1).
template <bool KMAJ, int ROWS, bool PERM = false, int NW = 8, int BKT = 64, int WNX = 4, int PB = 16>
__device__ __forceinline__ void stage(__amdgpu_buffer_rsrc_t rs, long ld, int rows_left, int k0, int K,
                                      LDS_AS char* lds, int wave, int lane) {
  constexpr int PIECES = ROWS * BKT * 2 / 1024;  // 1-KB DMA pieces per operand tile
  constexpr int PPW = PIECES / NW;
  static_assert(KMAJ || BKT == 64, "MN-major staging is written for 64-deep K tiles");
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int p = wave * PPW + i;
    uint32_t voff;
    if constexpr (KMAJ) {
      // 128-B rows (BK 64): chunk ^= (row>>1)&7; 64-B rows (BK 32): chunk ^= kswz32(row)
      constexpr int CPR = BKT / 8, RPP = 64 / CPR;  // 16-B chunks per row, rows per piece
      const int r = p * RPP + lane / CPR;
      const int c = (lane % CPR) ^ (BKT == 64 ? ((r >> 1) & 7) : kswz32(r));
      const int kk = k0 + c * 8;
      int gr = r;
      if constexpr (PERM) {
        constexpr int WN = ROWS / WNX, NTN = WN / PB;
        const int rl = r % WN;
        gr = (r - rl) + NTN * (rl % PB) + (rl / PB);
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
template <bool KMAJ, int ROWS, int BKT = 64>
__device__ __forceinline__ bf16x8 frag(const LDS_AS char* lds, int rb, int s, int lane) {
  if constexpr (KMAJ) {
    const int r = rb + (lane & 15);
    if constexpr (BKT == 32) {  // 64-B rows, one k-step
      const int c = (lane >> 4) ^ kswz32(r);
      return *(const LDS_AS bf16x8*)(lds + r * 64 + c * 16);
    }
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

// GELU (nn.GELU(), vision_transformer.py:100) in the epilogues: the forward evaluates it on the bf16
// pre-activation (the reference's autocast order) and, when the caller saves for the backward, the
// derivative gelu'(pre) in the same pass (its erf and Gaussian terms are already computed); the
// backward epilogue then multiplies by the saved derivative (one VALU op per element).
__device__ __forceinline__ uint32_t gelu_pair(uint32_t pk, uint32_t* dpk) {
  float y0, d0, y1, d1;
  gelu_fwd_grad(__builtin_bit_cast(float, pk << 16), y0, d0);
  gelu_fwd_grad(__builtin_bit_cast(float, pk & 0xffff0000u), y1, d1);
  if (dpk) *dpk = pack_bf2(d0, d1);
  return pack_bf2(y0, y1);
}

// ---- GELU by table (the staggered fc1 kernel's epilogue). The pre-activation is a bf16 value (the
// reference's autocast rounding point), so GELU(pre) and GELU'(pre) are functions of its 16 bits.
// Entry (i, s) of the LDS table (interleaved: byte 16 i + 8 s) holds {cdf, dy} = gelu_cdf_grad(x) for
// x = (-1)^s * bf16(GT_LO - 1 + i) (i >= 1), x = (-1)^s * 0 (i = 0); the epilogue forms y = x * cdf,
// the same f32 product gelu_fwd_grad takes, and dy as stored. Magnitudes outside [2^-10, 16) share
// one entry per side because their bf16 outputs are the same:
//  * |x| < 2^-10 -> the +-0 entry: cdf(x) = 0.5 +- 0.4|x| stays within 2^-10.3 of 0.5 (relative),
//    inside half a bf16 ulp of x / 2 for y and of 0.5 for dy; below 2^-24 cdf(x) IS cdf(+-0) (rcp(1 +
//    0.27 a) = 1, exp2(-zs^2) = 1), which keeps the f32-denormal products (round-half-even ties of
//    x / 2 in bf16) those of the exact evaluation;
//  * |x| >= 16 -> the largest entry below 16: exp2(-zs^2) underflows to 0, so cdf = 1 (x > 0) or
//    0 (x < 0) and dy = 1 or 0 exactly, as for every larger |x|;
//  * inf / NaN: y = x * cdf gives what the exact evaluation gives; dy = fma(x, 0, dy_tab) is NaN for
//    them (x * 0) and dy_tab otherwise (dy is never -0).
// ~9 VALU + one LDS read per element instead of ~17 VALU + rcp + exp2; bitwise equal to gelu_fwd_grad
// on all 65536 bf16 inputs (tests/test_gpu_kernels.py::test_gelu_epilogues_bitwise_all_bf16).
constexpr uint32_t GT_LO = 0x3A80;       // bf16 bits of 2^-10
constexpr uint32_t GT_HI = 0x417F;       // largest bf16 below 16
constexpr int GT_N = GT_HI - GT_LO + 2;  // entries per sign (index 0: |x| < 2^-10, zero, denormals)
constexpr int GT_BYTES = 2 * GT_N * 8;   // 28.7 KB

__device__ __forceinline__ void gelu_tab_fill(LDS_AS f32x2* tab, int tid, int nthreads) {
  for (int e = tid; e < 2 * GT_N; e += nthreads) {
    const uint32_t i = (uint32_t)e >> 1, sg = (uint32_t)e & 1;
    const uint32_t bits = (i == 0 ? 0u : GT_LO - 1 + i) | (sg << 15);
    float cdf, dy;
    gelu_cdf_grad(__builtin_bit_cast(float, bits << 16), cdf, dy);
    tab[e] = f32x2{cdf, dy};
  }
}

// GELU (and GELU' into *dpk when SAVE_D) of the two bf16 pre-activations packed in pk, by table
template <bool SAVE_D>
__device__ __forceinline__ uint32_t gelu_pair_tab(uint32_t pk, const LDS_AS char* tab, uint32_t* dpk) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  const u16x2 b = __builtin_bit_cast(u16x2, pk);
  u16x2 i = __builtin_elementwise_sub_sat(b & (u16x2)0x7fff, (u16x2)(GT_LO - 1));
  i = __builtin_elementwise_min(i, (u16x2)(GT_N - 1));
  const uint32_t a = __builtin_bit_cast(uint32_t, (u16x2)((i << 4) | ((b >> 12) & (u16x2)8)));
  const float x0 = __builtin_bit_cast(float, pk << 16), x1 = __builtin_bit_cast(float, pk & 0xffff0000u);
  if constexpr (SAVE_D) {
    const f32x2 t0 = *(const LDS_AS f32x2*)(tab + (a & 0xffffu));
    const f32x2 t1 = *(const LDS_AS f32x2*)(tab + (a >> 16));
    *dpk = pack_bf2(fmaf(x0, 0.f, t0[1]), fmaf(x1, 0.f, t1[1]));
    return pack_bf2(x0 * t0[0], x1 * t1[0]);
  } else {
    const float c0 = *(const LDS_AS float*)(tab + (a & 0xffffu));
    const float c1 = *(const LDS_AS float*)(tab + (a >> 16));
    return pack_bf2(x0 * c0, x1 * c1);
  }
}

struct Tile {
  int m0, n0, z, Keff, nk;  // buffer descriptors are rebuilt per DMA: SGPRs are the scarce resource
};

}  // namespace
