// Large-tile bf16 GEMM for gfx950: 256 x BN x 64 tiles (BN = 256 or 128), 512 threads = 8 waves,
// one workgroup per CU (LDS 144 / 112 KB), v_mfma_f32_16x16x32_bf16, waves 2 (M) x 4 (N), wave tile
// 128 x 64. (A 32x32x16 form of the tile, waves 4 x 2, measured no faster per kernel and 3 % slower
// per train step in round 4 - profiles/r04_gemm_mf32_*.txt - and was removed.)
// Same operand/epilogue contract as vj_gemm.hip (K-major or MN-major A and B, fused epilogues);
// used for the forward and data-gradient GEMMs of the encoder / predictor blocks (M = tokens) and the
// split-K weight gradients.
//
// Persistent: one workgroup per CU walks a run of tiles. The next tile's first two K stages are
// DMA'd while this tile finishes (stage 0 during the last K-tile, stage 1 before or during the
// epilogue), so the prologue latency and the block launch hide behind the epilogue; per-kernel LDS
// tables (GELU, RoPE cos/sin) are loaded once per workgroup.
//
// Schedule (per wave, K-tile t in LDS slot (t + par) & 1): 4 phases per K-tile = (k-step, M-half),
// each 4 x NTN MFMAs on a 64x(BN/4) quarter of the wave tile; the next phase's fragments (16 + 16
// VGPRs, double-buffered) are read from LDS while the current phase's MFMAs run, so LDS latency hides
// under MFMA with 128 accumulator + 64 fragment registers (no spill at 2 waves / SIMD). ONE barrier per
// K-tile (before the last phase): it retires this wave's DMA of tile t+1 (issued one tile earlier)
// and its reads of tile t; tile t+2 is then DMA'd into the freed slot and stays in flight across it.
// Epilogue: stores straight from registers (K-major B, 256-wide tiles: B rows staged permuted) or
// through a padded LDS image in the freed slot, with bias / residual / GELU / GELU' / RoPE fused.
#include <stdlib.h>
#include <atomic>
#include <type_traits>
#include "vj_gemm_tile.h"

// Schedule choices fixed by round-3 measurements (the variants were removed from the source; the
// numbers are in DESIGN.md and profiles/r03_gemm_*):
//  * 8-wave main loop: only the A pieces of K-tile t + 2 go out after the barrier; the B pieces are
//    issued after 3 of the last phase's 4 m-tiles (SPLIT_AT): -2..-7 % and a further 0..-5 % on the
//    ViT-L shapes (r03_gemm_spread_kernels.txt,
//    r03_gemm_split_kernels.txt). Also the A pieces after the first m-tile: slower.
//  * on 256-wide bf16 tiles without a VALU-heavy epilogue only waves 0-3 issue the main-loop LDS-DMA
//    (DMA_WAVES; their SIMD partners keep issuing MFMAs); the next tile's stage 1, issued around the
//    epilogue, goes out from all 8 waves (r03_gemm_dmaw4_kernels.txt, r03_gemm_s1all_step_ab.txt).
//    Slower and removed: the RoPE / GELU tiles on 4 DMA waves, A / B pieces split over waves 0-3 /
//    4-7, the DMA from waves 4-7, s_setprio around the MFMA clusters or for waves 4-7.
//  * one m-tile of residual / saved-derivative rows prefetched ahead in the direct epilogue (deeper:
//    no faster, r03 stamps).
constexpr int SPLIT_AT = 3;
constexpr int DMA_WAVES = 4;
constexpr int AUX_PF = 1;

namespace {

#if VJ_GEMM_STAMPS  // diagnostic build: s_memtime per tile (start, main loop done, epilogue done) of wave 0
__device__ long vj_gemm_stamps[2048 * 16 * 4];
// S64: s_memtime after each of the 16 barriers of K steps 1-4 of the block's second tile, waves 0 and 4
__device__ long vj_gemm_istamps[2048 * 2 * 16];
#endif

// counted wait for this wave's vector-memory operations (LDS-DMA pieces included): at most N in flight
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N <= 24 && N % 4 == 0, "vm_wait: add the count");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N == 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
}


// NWV = 8: 8 waves (2 x 4), 64-deep K tiles, one workgroup per CU. NWV = 4 ("2W"): 4 waves (2 x 2),
// TWO workgroups per CU, so one workgroup's epilogue (HBM / VALU) runs under the other's main loop
// (MFMA); K-major operands only; 192 x 128 tiles 64 deep (80 KB, the default) or 256 x 128 tiles 32
// deep (64 KB + the RoPE table area).
// BMT = 192 (8-wave, K-major bf16, 256-wide direct-store tiles only): 96-row wave tiles (3 m-tiles
// per M-half) for problems whose 256-row tile count leaves a round of CUs under-filled (context
// GEMMs, M ~ 11.7k: 184 tiles of 256 x 256 on 256 CUs -> 244 tiles of 192 x 256).
// VJ_STG_CPOL: cache-policy bits of the staggered loop's LDS-DMA pieces (0; sc1 = 16 measured within
// noise, nt = 2 up to 2x slower). VJ_DIAG_NODMA / NOWAIT / SAMEADDR / FULL128: timing-only builds that
// compute WRONG results (no DMA after the prologue; relaxed unit wait; every piece from one 1-KB block;
// pieces of 8 whole 128-B rows) - profiles/r05_gemm_dma_diag.txt, never in the shipped library.
#ifndef VJ_STG_CPOL
#define VJ_STG_CPOL 0
#endif
#ifndef VJ_DIAG_NODMA
#define VJ_DIAG_NODMA 0
#endif
template <bool AK, bool BKM, int EPI, int BN, bool F8 = false, int NWV = 8, int BMT = 256, int STG = 0>
__global__ __launch_bounds__(NWV * 64, 2) void k_gemm256(G256 g) {
  constexpr bool PART = EPI == EPI_PARTIAL || EPI == EPI_PARTIAL_RS;  // split-K partial slabs (RS: + row sums)
  static_assert(!STG || (AK && BKM && !F8 && NWV == 8 && BMT == 256 && BN == 256 && !PART),
                "staggered main loop: 8-wave K-major bf16 256 x 256 tiles");
  static_assert(!F8 || (AK && BKM && !PART && EPI != EPI_GELU_BWD), "fp8: forward GEMMs only");
  static_assert(NWV == 8 || (NWV == 4 && AK && BKM && !F8), "2-workgroup GEMM: K-major bf16 operands only");
  constexpr int BM = BMT;
  constexpr int MH = BM / 64;     // virtual 16-row m-tiles per half of the wave's rows (4 / 3)
  // 2-workgroup kernels: 256 x 128 tiles 32 deep (64-B LDS rows), or 192 x 128 tiles 64 deep (128-B
  // rows: whole cache lines per DMA piece, half the L1 -> L2 requests; 80 KB, no table: RoPE excluded)
  constexpr int BK = (NWV == 8 || BMT == 192) ? 64 : 32;
  constexpr int NT = NWV * 64;
  constexpr int WNX = NWV / 2;  // waves across N (4 / 2)
  constexpr int WMX = NWV / WNX;          // waves across M (2 / 4)
  constexpr int WM = BM / WMX;            // wave tile rows (128 / 96)
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int WN = BN / WNX;    // wave tile columns (64 / 32)
  constexpr int PB = 16;         // MFMA output block width
  constexpr int NTN = WN / PB;    // n blocks per wave (4 / 2)
  // LDS-DMA issuers: DMA_WAVES = 4 -> waves 0-3 only on 256-wide tiles (their SIMD partners 4-7 keep
  // issuing MFMAs meanwhile), except the RoPE / GELU / GELU-backward tiles, whose next-tile stage 1
  // goes out right before (or in) their VALU-heavy epilogue, where waves 0-3 would start it 16
  // pieces late; 128-wide tiles (the predictor's N = 384) measured slower with it.
  constexpr bool VALU_EPI = EPI == EPI_ROPE || EPI == EPI_GELU || EPI == EPI_GELU_BWD;
  constexpr int DMAW = NWV != 8 ? NWV : (VALU_EPI || BN != 256 || F8) ? 8 : DMA_WAVES;
  // K-major B with 4 n blocks per wave: permuted B staging + stores straight from registers (16-B
  // f32 / 8-B bf16 per row); 128-wide tiles would store 4-8 B per lane, so they keep the LDS path
  constexpr bool DIRECT = BKM && NTN == 4;
  static_assert(BMT == 256 || (BMT == 192 && !F8 && AK && DIRECT && (NWV == 8 || EPI != EPI_ROPE)),
                "192-row tiles: direct K-major bf16 (the 4-wave kernel without the RoPE table)");
  constexpr bool AUX = EPI == EPI_F32_RESID || EPI == EPI_GELU_BWD || EPI == EPI_BF16_RESID;
  constexpr bool F32OUT = EPI == EPI_F32 || EPI == EPI_F32_RESID || PART;

  // The next tile's stage 0 is DMA'd during this tile's last K-tile. Its stage 1 goes out right
  // after the last barrier, unless the epilogue still needs that LDS slot (staged epilogue: after
  // it) or issues global loads that would queue behind the DMA in vmcnt order (AUX: once the last
  // aux rows are fetched).
  constexpr bool EARLY1 = DIRECT && !AUX;
  // STG: ring of NSL 32-KB unit slots, DMA distance NSL - 2 units; 5 slots (all 160 KB of the CU's
  // LDS, distance 3) unless the RoPE epilogue needs the table area (4 slots + table, distance 2)
  // (GTAB: the GELU epilogue by table, 4 slots behind the 28.7-KB table at LDS offset 0, whose byte
  // offsets then fit the 16-bit lanes the lookup computes them in)
  constexpr bool GTAB = STG && EPI == EPI_GELU;
#ifndef VJ_STG_NSL4
#define VJ_STG_NSL4 0  // variant builds: every staggered kernel on 4 ring slots (distance 2)
#endif
  constexpr int NSL = STG ? ((EPI == EPI_ROPE || GTAB || VJ_STG_NSL4) ? 4 : 5) : 1;
  constexpr int DIST = NSL - 2;
  // S64 (STG == 2, round 6): the staggered loop on 64-deep K steps, so every 1-KB LDS-DMA piece is 8
  // WHOLE 128-B rows (the 32-deep units above fetch 16 half lines: twice the L1 -> L2 requests, which
  // bound that loop - profiles/r05_gemm_dma_diag.txt). The LDS budget is kept by splitting each K step
  // of the tile into 16-KB granules of 128 rows x 64: A0 / A1 (tile rows 0-127 / 128-255) and Blo / Bhi
  // (columns 0-127 / 128-255). Waves 0-3 stream the A granules, waves 4-7 the B granules, one granule
  // per wave group and load interval (4 pieces per wave). A wave (wr, wc) owns rows {128 h + 64 wr +
  // 0..63 : h = 0, 1} x columns 64 wc + 0..63; per K step it runs L0 (A0 and B fragments: 16
  // ds_read_b128) | M0 (rows of A0: 32 MFMAs) | L1 (A1 fragments, B kept in registers: 8 reads) | M1,
  // waves 4-7 one interval behind as before. Every output sums the same MFMAs in the same k order as
  // the other forms: bitwise the same results. Rings: SA A slots, SB B slots (DMA distance SA - 1 /
  // SB - 1 granules, 4 + 4 x 16 KB = the 4-slot ring's 128 KB, beside the GELU / RoPE tables).
  constexpr bool S64 = STG == 2;
  constexpr int GSZ = 16384;
  // B ring depth (variant builds: VJ_S64_SB = 5 / 6 on the kernels without an LDS table). Deeper B
  // rings removed the DMA stalls of a tile's first K steps (interval stamps) but slowed every later
  // step: qkv tgt 260 -> 274 us, step -0.6 % (profiles/r06_gemm_s64.txt); 4 kept
#ifndef VJ_S64_SB
#define VJ_S64_SB 4
#endif
  constexpr int SA = 4, SB = (EPI == EPI_ROPE || GTAB) ? 4 : VJ_S64_SB;
  constexpr int EA = SA - 1, EB = SB - 1;
  static_assert(EA >= 2 && EB >= 3, "S64 waits assume at least one interval of DMA lead");
  // first row of the wave's rows (S64: the wave's 64-row band in each 128-row half) and the first row
  // of virtual m-tile i relative to it
  constexpr int WRS = S64 ? 64 : WM;
  auto rowoff = [](int i) { return S64 ? (i >> 2) * 128 + (i & 3) * 16 : i * 16; };
  constexpr int RING0 = GTAB ? 32768 : 0;  // LDS offset of the STG ring
  static_assert(!S64 || (SA + SB) * 16384 + RING0 + ((EPI == EPI_ROPE) ? TAB_BYTES : 0) <= 163840, "S64 rings exceed LDS");
  constexpr int TABB = (NWV == 4 && BMT == 192) ? 0 : TAB_BYTES;  // 2 x 80 KB per CU leaves no table room
  __shared__ __attribute__((aligned(16))) char smem_raw[GTAB ? RING0 + 4 * 32768 : STG && NSL == 5 ? 5 * 32768 : 2 * STAGE + TABB];
  LDS_AS char* smem = (LDS_AS char*)smem_raw;
  LDS_AS char* tab = smem + 2 * STAGE;
  [[maybe_unused]] LDS_AS char* ring = smem + RING0;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / WNX, wc = wave % WNX;

  // Persistent walk. The logical tiles (K slice outermost, then the tile order) are cut into 8
  // contiguous runs, one per XCD (blocks b and b + 8 share an XCD); the P blocks of an XCD walk its
  // run with stride P, so the tiles an XCD has in flight are consecutive and share A / B panels in
  // its L2. Every block leaves after its last tile: no inter-block dependency.
  const int ntile = g.tiles_m * g.tiles_n;
  const int nb = ntile * g.nsplit;
  const int P = gridDim.x >> 3;
  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int q = nb >> 3, rmd = nb & 7;
  const int run0 = xcd < rmd ? xcd * (q + 1) : rmd * (q + 1) + (xcd - rmd) * q;
  const int runend = run0 + q + (xcd < rmd ? 1 : 0);
  if (run0 + jb >= runend) return;

  auto make_tile = [&](int wg) {
    Tile T;
    const int z = wg / ntile, w = wg - z * ntile;
    int tm, tn;
    if (g.group > 0) {  // runs of `group` tile rows walked column by column
      const int per = g.group * g.tiles_n, grp = w / per, first = grp * g.group;
      const int gm = min(g.tiles_m - first, g.group), loc = w - grp * per;
      tm = first + loc % gm;
      tn = loc / gm;
    } else {
      tm = w / g.tiles_n;
      tn = w - tm * g.tiles_n;
    }
    // wave-uniform by construction; readfirstlane keeps them in SGPRs (the divisions above run on
    // the VALU, and VGPRs are all taken by the accumulators and fragments)
    T.m0 = __builtin_amdgcn_readfirstlane(tm * BM);
    T.n0 = __builtin_amdgcn_readfirstlane(tn * BN);
    T.z = __builtin_amdgcn_readfirstlane(z);
    const int kb = T.z * g.kslice;
    T.Keff = min(g.K, kb + g.kslice) - kb;
    T.nk = (T.Keff + BK - 1) / BK;
    return T;
  };
  // buffer descriptors of a tile's A and B panels (from its K slice on; the range check zero-fills
  // ragged M / N / K)
  auto rsrc_a = [&](const Tile& T) {
    const int kb = T.z * g.kslice;
    const bf16_t* abase = AK ? g.A + (long)T.m0 * g.lda + kb : g.A + (long)kb * g.lda + T.m0;
    return make_rsrc(abase, AK ? clampb((long)(g.M - T.m0) * g.lda * 2 - kb * 2L)
                               : clampb(((long)(g.K - kb) * g.lda - T.m0) * 2));
  };
  auto rsrc_b = [&](const Tile& T) {
    const int kb = T.z * g.kslice;
    const bf16_t* bbase = BKM ? g.B + (long)T.n0 * g.ldb + kb : g.B + (long)kb * g.ldb + T.n0;
    return make_rsrc(bbase, BKM ? clampb((long)(g.N - T.n0) * g.ldb * 2 - kb * 2L)
                                : clampb(((long)(g.K - kb) * g.ldb - T.n0) * 2));
  };
  const bool iss = DMAW == 8 || wave < DMAW;  // this wave issues main-loop LDS-DMA pieces
  auto load_k = [&](__amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, const Tile& T, int t, int slot,
                    int lane) {
    LDS_AS char* s = smem + slot * STAGE;
#if VJ_DIAG_NODMA
    if (t >= 2) return;
#endif
    if (iss) {
      stage<AK, BM, false, DMAW, BK, WNX, PB>(ra, g.lda, g.M - T.m0, t * BK, T.Keff, s, wave, lane);
      stage<BKM, BN, DIRECT, DMAW, BK, WNX, PB>(rb, g.ldb, g.N - T.n0, t * BK, T.Keff, s + A_BYTES, wave, lane);
    }
  };
  auto load_tile = [&](const Tile& T, int t, int slot, int lane) {
    load_k(rsrc_a(T), rsrc_b(T), T, t, slot, lane);
  };
  // the next tile's stage 1, issued around the epilogue (no MFMAs to keep fed): all 8 waves
  auto load_tile8 = [&](const Tile& T, int t, int slot, int lane) {
    LDS_AS char* s = smem + slot * STAGE;
    stage<AK, BM, false, NWV, BK, WNX, PB>(rsrc_a(T), g.lda, g.M - T.m0, t * BK, T.Keff, s, wave, lane);
    stage<BKM, BN, DIRECT, NWV, BK, WNX, PB>(rsrc_b(T), g.ldb, g.N - T.n0, t * BK, T.Keff, s + A_BYTES, wave, lane);
  };

  // per-kernel tables (RoPE): global loads issued before the first DMA (so their waits do not queue
  // behind it), written to the table area after it; the first barrier of the tile loop publishes them
  constexpr int RTR = EPI == EPI_ROPE ? (ROPE_TAB_MAX + NT - 1) / NT : 0;
  [[maybe_unused]] f32x2 rpf[RTR > 0 ? RTR : 1];
  [[maybe_unused]] const int ntab = EPI == EPI_ROPE ? g.rope.npos * g.rope.half : 0;  // <= ROPE_TAB_MAX (host)
  if constexpr (EPI == EPI_ROPE) {
#pragma unroll
    for (int i = 0; i < RTR; ++i) {
      const int e = threadIdx.x + NT * i;
      rpf[i] = e < ntab ? f32x2{g.rope.cos_t[e], g.rope.sin_t[e]} : f32x2{0.f, 0.f};
    }
  }
  // tile-row positions (frame | row << 10 | col << 20) and the interleaved cos/sin table (RoPE)
  [[maybe_unused]] LDS_AS int* rpos = (LDS_AS int*)tab;
  [[maybe_unused]] LDS_AS f32x2* rtab = (LDS_AS f32x2*)(tab + BM * 4);

  int wg = run0 + jb;
  Tile cur = make_tile(wg);
  int par = 0;  // LDS slot of K-tile t of the current tile: (t + par) & 1

  // ---- STG: staggered main loop (GEMM). 32-deep K units in a ring of 4 LDS slots (A
  // 256 x 32 then B 256 x 32, 16 KB each); the block's tiles form ONE stream of units (position q =
  // unit q % nku of the block's tile q / nku), and position q + 2 is DMA'd while q is computed, so the
  // next tile's first units arrive under this tile's last ones and its epilogue. Each wave issues 4
  // of the 32 1-KB pieces of every unit (waves 0-3: A, 4-7: B; their lane offsets are fixed per
  // tile, the unit's K offset rides in soffset), 2 per load interval; past the stream end the pieces
  // zero-fill an unread slot, so the per-wave vmcnt count stays 4.
  constexpr int USZ = 32768;
  [[maybe_unused]] const int nku = STG ? (g.K + 31) / 32 : 0;
  [[maybe_unused]] int dwg = wg, dku = 0, dpos = 0;
  [[maybe_unused]] __amdgpu_buffer_rsrc_t drs;
  [[maybe_unused]] uint32_t dvo[4];
  const bool isA = wave < 4;
  auto dma_setup = [&]() {  // lane offsets / descriptor of this wave's operand of DMA tile dwg
    if (dwg < runend) {
      const Tile T = make_tile(dwg);
      const int left = isA ? g.M - T.m0 : g.N - T.n0;
      const long ld = isA ? g.lda : g.ldb;
      if (isA) drs = make_rsrc(g.A + (long)T.m0 * g.lda, clampb((long)left * g.lda * 2));
      else drs = make_rsrc(g.B + (long)T.n0 * g.ldb, clampb((long)left * g.ldb * 2));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = (4 * (wave & 3) + j) * 16 + (lane >> 2);  // LDS row of the lane's 16-B chunk
        const int c = (lane & 3) ^ kswz32(r);                   // its logical chunk (64-B row swizzle)
        int gr = r;
        if (!isA) {  // PERM (stage()): LDS row r of a 64-row group holds group row 4 (r % 16) + r / 16
          const int rl = r & 63;
          gr = (r - rl) + 4 * (rl & 15) + (rl >> 4);
        }
        dvo[j] = gr < left ? (uint32_t)(gr * ld * 2 + c * 16) : VJ_OOB;
#if VJ_DIAG_FULL128
        dvo[j] = (uint32_t)(((4 * (wave & 3) + j) * 8 + (lane >> 3)) * ld * 2 + (lane & 7) * 16);
#endif
#if VJ_DIAG_SAMEADDR
        dvo[j] = (uint32_t)(lane * 16);
#endif
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) dvo[j] = VJ_OOB;
    }
  };
  // this wave's pieces 2h, 2h + 1 of stream position dpos (into slot dpos % NSL)
  auto dma_half = [&](auto h_c) {
    constexpr int h = decltype(h_c)::value;
    LDS_AS char* dst = ring + (dpos % NSL) * USZ + (isA ? 0 : 16384) + (4 * (wave & 3) + 2 * h) * 1024;
#if VJ_DIAG_FULL128
    const int soff = __builtin_amdgcn_readfirstlane((dku >> 1) * 128 + (dku & 1) * 128 * (int)(isA ? g.lda : g.ldb) * 2);
#else
    const int soff = __builtin_amdgcn_readfirstlane(dku * 64);
#endif
#if VJ_DIAG_NODMA
    if (dpos < DIST)
#endif
    {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(drs, dst, 16, dvo[2 * h], soff, 0, VJ_STG_CPOL);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(drs, dst + 1024, 16, dvo[2 * h + 1], soff, 0, VJ_STG_CPOL);
    }
    if constexpr (h == 1) {
      ++dpos;
      if (++dku == nku) {
        dku = 0;
        dwg += P;
        dma_setup();
      }
    }
  };
  // ---- S64 stream: this wave group's operand (A: waves 0-3, B: waves 4-7) as granules; position dq of
  // the group's stream = (tile, step dk >> 1, half dk & 1), into slot dq % SA (A) / SA + dq % SB (B).
  // Each wave DMAs rows 32 (wave & 3) .. + 31 of every granule (4 pieces of 8 rows); its lane offsets
  // are fixed for the launch (rows relative to the granule's first row), the descriptor's range check
  // (from that row to the operand's end) zero-fills rows past M / N and, past the stream end (dleft 0),
  // whole granules, so the per-wave vmcnt counts never change.
  [[maybe_unused]] const int nks = S64 ? g.K >> 6 : 0;
  [[maybe_unused]] const long dld = isA ? g.lda : g.ldb;
  [[maybe_unused]] const bf16_t* dbase = isA ? g.A : g.B;
  [[maybe_unused]] int dleft = 0, dq = 0, dk = 0, q64 = 0;
  auto dma_setup64 = [&]() {
    if (dwg < runend) {
      const Tile T = make_tile(dwg);
      dbase = isA ? g.A + (long)T.m0 * g.lda : g.B + (long)T.n0 * g.ldb;
      dleft = isA ? g.M - T.m0 : g.N - T.n0;
    } else {
      dleft = 0;
    }
  };
  auto dma_gran = [&]() {
    const int h = dk & 1;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(dbase + (h ? 128 * dld : 0), clampb((long)(dleft - 128 * h) * dld * 2));
    const int soff = __builtin_amdgcn_readfirstlane((dk >> 1) * 128);
    LDS_AS char* dst = ring + (isA ? dq % SA : SA + dq % SB) * GSZ + (wave & 3) * 4096;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, dst + k * 1024, 16, dvo[k], soff, 0, VJ_STG_CPOL);
    ++dq;
    if (++dk == 2 * nks) {
      dk = 0;
      dwg += P;
      dma_setup64();
    }
  };
  if constexpr (S64) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = 32 * (wave & 3) + 8 * k + (lane >> 3);  // granule row of the lane's 16-B chunk
      const int c = (lane & 7) ^ ((r >> 1) & 7);            // its logical chunk (128-B row swizzle)
      const int rl = r & 63;                                 // B: PERM within 64-row groups (stage())
      const int gr = isA ? r : (r - rl) + 4 * (rl & 15) + (rl >> 4);
      dvo[k] = (uint32_t)(gr * dld * 2 + c * 16);
    }
    dma_setup64();
    for (int i = 0; i < (isA ? EA : EB); ++i) dma_gran();
  } else if constexpr (STG) {
    dma_setup();
#pragma unroll
    for (int i = 0; i < DIST; ++i) {
      dma_half(std::integral_constant<int, 0>{});
      dma_half(std::integral_constant<int, 1>{});
    }
  } else {
    load_tile(cur, 0, 0, lane);
    if (cur.nk > 1) load_tile(cur, 1, 1, lane);
  }
  if constexpr (EPI == EPI_ROPE) {
#pragma unroll
    for (int i = 0; i < RTR; ++i) {
      const int e = threadIdx.x + NT * i;
      if (e < ntab) rtab[e] = rpf[i];
    }
  }
  // GELU table: computed once per (persistent) workgroup under the first units' DMA; read only in the
  // epilogues, after the first tile's barriers
  if constexpr (GTAB) gelu_tab_fill((LDS_AS f32x2*)smem, threadIdx.x, NT);

  // Accumulators: acc[i][j] = m-tile i (16 rows), n block j; the epilogue walks the 2 * MH m-tiles,
  // 4 rows per lane (rows rowoff(i) + 4 (lane >> 4) + r of the wave tile).
  f32x4 acc[2 * MH][NTN];
  auto accv = [&](int i, int j, int r) -> float { return acc[i][j][r]; };
  auto accs = [&](int i, int j, int r, float v) { acc[i][j][r] = v; };
  bf16x8 Aa[MH], Ab[MH], Ba[NTN], Bb[NTN];
  // A fragments of M-half mh (4 m-tiles), k-step ks; B fragments of all NTN n-tiles, k-step ks
  auto rdA = [&](bf16x8 (&X)[MH], int slot, int mh, int ks) {
    const LDS_AS char* s = smem + slot * STAGE;
#pragma unroll
    for (int i = 0; i < MH; ++i) X[i] = frag<AK, BM, BK>(s, wr * WM + (mh * MH + i) * 16, ks, lane);
  };
  auto rdB = [&](bf16x8 (&Y)[NTN], int slot, int ks) {
    const LDS_AS char* s = smem + slot * STAGE + A_BYTES;
#pragma unroll
    for (int j = 0; j < NTN; ++j) Y[j] = frag<BKM, BN, BK>(s, wc * WN + j * 16, ks, lane);
  };
  // ---- fp8 (F8): one K-tile row is 128 B = 128 e4m3 values = ONE v_mfma_scale_f32_16x16x128_f8f6f4
  // per 16x16 output tile. Its 32-B lane operand is the two 16-B fragments the bf16 path reads for
  // k-steps 0 and 1 (chunks g and 4 + g of the row). A and B take the same byte -> k assignment, so
  // the product sums the same 128 terms. Fragments are read straight into 8-VGPR operand tuples (as
  // many VGPRs as the bf16 path's): Xa / Xb = the two m-tiles of an m-quarter q, alternating, and
  // Y8 = the n-tiles. The per-row scales are the same for every k of a row, so they ride in the
  // MFMA's per-lane E8M0 scale operands whatever the lane's k assignment: lane l of m-tile i scales
  // A row (i * 16 + (l & 15)) by 2^ea, of n-tile j B row (j * 16 + (l & 15)) by 2^eb (loaded per tile).
  [[maybe_unused]] int f8sa[8], f8sb[NTN];
  [[maybe_unused]] i32x8 Xa[2], Xb[2], Y8[NTN];
  auto cat = [](bf16x8 lo, bf16x8 hi) {
    const i32x4 l = __builtin_bit_cast(i32x4, lo), h = __builtin_bit_cast(i32x4, hi);
    return __builtin_shufflevector(l, h, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto rdA8 = [&](i32x8 (&X)[2], int slot, int qq) {
    const LDS_AS char* s = smem + slot * STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      X[i] = cat(frag<AK, BM>(s, wr * 128 + (2 * qq + i) * 16, 0, lane),
                 frag<AK, BM>(s, wr * 128 + (2 * qq + i) * 16, 1, lane));
  };
  auto rdB8 = [&](int j0, int j1, int slot) {
    const LDS_AS char* s = smem + slot * STAGE + A_BYTES;
#pragma unroll
    for (int j = j0; j < j1; ++j)
      Y8[j] = cat(frag<BKM, BN>(s, wc * WN + j * 16, 0, lane), frag<BKM, BN>(s, wc * WN + j * 16, 1, lane));
  };
  auto mm8 = [&](const i32x8 (&X)[2], int qq, int j0, int j1) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = j0; j < j1; ++j)
        acc[2 * qq + i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(X[i], Y8[j], acc[2 * qq + i][j], 0, 0,
                                                                              0, f8sa[2 * qq + i], 0, f8sb[j]);
  };
  // Fused bias gradient (EPI_PARTIAL_RS, tiles of column tile 0): row sums of the A
  // fragments the MFMAs already hold. Wave (wr, wc) sums m-tiles 2 wc and 2 wc + 1 of its 128-row
  // band (so the 4 waves of a band cover its 8 m-tiles once), in M-half wc / 2, with v_dot2 against
  // bf16 ones: 4 VALU per m-tile and k-step beside 16 MFMAs, two f32 registers per lane (lane l:
  // row l & 15, k = 8 (l >> 4) .. + 7; the 4 lane groups are summed in the epilogue).
  constexpr bool RS = EPI == EPI_PARTIAL_RS;
  [[maybe_unused]] float rsa = 0.f, rsb = 0.f;
  [[maybe_unused]] bool rs_on = false;
  auto rsum8 = [](const bf16x8& x, float s) {
    typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
    const bf16x2_t one = {(__bf16)1.0f, (__bf16)1.0f};
    s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(x, x, 0, 1), one, s, false);
    s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(x, x, 2, 3), one, s, false);
    s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(x, x, 4, 5), one, s, false);
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(x, x, 6, 7), one, s, false);
  };
  auto rs_phase = [&](const bf16x8 (&X)[MH], int mh) {
    if constexpr (RS && MH == 4) {
      if (rs_on && (wc >> 1) == mh) {  // wave-uniform
        if (wc & 1) {
          rsa = rsum8(X[2], rsa);
          rsb = rsum8(X[3], rsb);
        } else {
          rsa = rsum8(X[0], rsa);
          rsb = rsum8(X[1], rsb);
        }
      }
    }
  };
  auto mm = [&](const bf16x8 (&X)[MH], int mh, const bf16x8 (&Y)[NTN]) {
#pragma unroll
    for (int i = 0; i < MH; ++i)
#pragma unroll
      for (int j = 0; j < NTN; ++j)
        acc[mh * MH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(X[i], Y[j], acc[mh * MH + i][j], 0, 0, 0);
    rs_phase(X, mh);
  };
  // m-tiles i0 .. i1 - 1 of one phase (the last phase is split around the B DMA pieces)
  auto mm_rows = [&](const bf16x8 (&X)[MH], int mh, const bf16x8 (&Y)[NTN], int i0, int i1) {
#pragma unroll
    for (int i = 0; i < MH; ++i)
      if (i >= i0 && i < i1)
#pragma unroll
        for (int j = 0; j < NTN; ++j)
          acc[mh * MH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(X[i], Y[j], acc[mh * MH + i][j], 0, 0, 0);
    if (i1 == MH) rs_phase(X, mh);
  };
  // MN-major operands are read with asm transposed reads (ds_read_tr16_async): each phase first
  // waits for the fragments it consumes (read in the previous phase), then issues the next reads.
  constexpr bool ASYNC = !AK || !BKM;
  auto release = [&](bf16x8 (&X)[MH], bf16x8 (&Y)[NTN]) {
    if constexpr (ASYNC) {
      lds_wait();
      tie(X);
      tie(Y);
    }
  };

#if VJ_GEMM_STAMPS
  int stamp_it = 0;
#endif
  for (;;) {
#if VJ_GEMM_STAMPS
    const long st0 = __builtin_amdgcn_s_memtime();
    long st_k1 = 0;  // staggered loops: after the tile's first 64-deep K step
#endif
    const int wgn = wg + P;
    const bool has_next = wgn < runend;
    // the next tile's descriptors are rebuilt where they are used (SGPR pressure: 106 is the cap)
    const int nk = cur.nk;
    const int parn = (nk + par) & 1;     // the next tile's stage 0 reuses the slot this tile frees first
    const int sle = (nk - 1 + par) & 1;  // slot of the last K-tile: free once the loop ends
    [[maybe_unused]] int pf_id = 0;  // RoPE: token id of tile row threadIdx.x, read under the main loop
    if constexpr (EPI == EPI_ROPE) {
      const int t = threadIdx.x;
      if (t < BM && cur.m0 + t < g.M) pf_id = g.rope.ids ? g.rope.ids[cur.m0 + t] : (cur.m0 + t) % g.rope.mod;
    }
#pragma unroll
    for (int i = 0; i < 2 * MH; ++i)
#pragma unroll
      for (int j = 0; j < NTN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (RS) {
      rs_on = g.rsum && cur.n0 == 0;
      rsa = rsb = 0.f;
    }
    if constexpr (F8) {  // this tile's per-row scale exponents (retired by the wait below)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = cur.m0 + wr * 128 + i * 16 + (lane & 15);
        f8sa[i] = 127 + (m < g.M ? g.ea[m] : 0);
      }
#pragma unroll
      for (int j = 0; j < NTN; ++j) {
        int r = wc * WN + j * 16 + (lane & 15);
        if constexpr (DIRECT) {  // permuted B staging: LDS row r holds global row NTN*(r%16) + r/16 of its group
          const int rl = r % WN;
          r = (r - rl) + NTN * (rl & 15) + (rl >> 4);
        }
        const int n = cur.n0 + r;
        f8sb[j] = 127 + (n < g.N ? g.eb[n] : 0);
      }
    }
    // STG: the bias columns are loaded before the main loop (in the epilogue the load would wait for
    // the next tile's DMA pieces issued after it: vmcnt counts in order)
    // (loads issued between the DMA pieces only ever make the main loop's counted vmcnt waits wait
    // longer, never shorter: its counts assume the DMA pieces alone)
    [[maybe_unused]] float biasp[NTN];
    if constexpr (STG) {
      const int nbp = cur.n0 + wc * WN + NTN * (lane & 15);
#pragma unroll
      for (int j = 0; j < NTN; ++j) biasp[j] = 0.f;
      if (EPI != EPI_GELU_BWD && g.bias && nbp < g.N) {
        const float4 bv = *(const float4*)(g.bias + nbp);
        biasp[0] = bv.x; biasp[1] = bv.y; biasp[2] = bv.z; biasp[3] = bv.w;
      }
    }
    // STG with a residual / saved-derivative epilogue: the first m-tile of aux rows is fetched one
    // unit before the tile ends (after that unit's DMA wait), so the epilogue's first reads do not
    // wait behind the next tile's DMA pieces
    [[maybe_unused]] f32x4 auxr[AUX && STG ? 4 : 1];
    auto stg_aux = [&] {
      if constexpr (AUX && STG) {
        const int m = cur.m0 + wr * WRS + 4 * (lane >> 4);
        const int n = cur.n0 + wc * WN + NTN * (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = m + r < g.M && n < g.N;
          const long off = ok ? (long)(m + r) * g.ldaux + n : 0;
          if constexpr (EPI == EPI_F32_RESID) {
            auxr[r] = *(const f32x4*)((const float*)g.aux + off);
          } else {
            const uint2 x = *(const uint2*)((const bf16_t*)g.aux + off);
            auxr[r] = f32x4{__builtin_bit_cast(float, x.x), __builtin_bit_cast(float, x.y), 0.f, 0.f};
          }
        }
      }
    };
    if constexpr (S64) {
      // S64 main loop (above). Waits, with j = the group's load-interval index (A position j / B
      // position j are DMA'd EA / EB intervals ahead): waves 0-3 end every L with A position j + 1
      // landed (vmcnt(4 (EA - 1))); waves 4-7 end each L1 with the next step's Blo / Bhi (B positions
      // up to j + 2) landed (vmcnt(4 (EB - 2))); the barrier after an L publishes them to every wave.
      // The aux rows of a residual / saved-derivative epilogue (4 loads per lane) are fetched in the last
      // step's L0, after its DMA pieces: the L1 waits after them count 4 more.
      if (wg == run0 + jb) {  // first tile: A position 0 and B positions 0, 1 landed, RoPE table published
        if (isA) vm_wait<4 * (EA - 1)>();
        else vm_wait<4 * (EB - 2)>();
        __builtin_amdgcn_s_barrier();
        if (wr == 1) __builtin_amdgcn_s_barrier();
      }
      auto bar = [] {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      };
      // Aa / Ab: A fragments (m-tiles 0-3 of the wave's band) at k-steps 0 / 1; Ba / Bb: B fragments
      auto mm64 = [&](auto h_c) {
        constexpr int h = decltype(h_c)::value;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[4 * h + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Aa[i], Ba[j], acc[4 * h + i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[4 * h + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ab[i], Bb[j], acc[4 * h + i][j], 0, 0, 0);
      };
      const int qt = q64;  // stream position of this tile's A0 / Blo of step 0
#if VJ_GEMM_STAMPS
      long* ist = (stamp_it == 1 && (wave & 3) == 0 && lane == 0 && blockIdx.x < 2048)
                      ? vj_gemm_istamps + ((long)blockIdx.x * 2 + (wave >> 2)) * 16 : nullptr;
      auto istamp = [&](int s, int k) {
        if (ist && s >= 1 && s <= 4) ist[(s - 1) * 4 + k] = __builtin_amdgcn_s_memtime();
      };
#else
      auto istamp = [](int, int) {};
#endif
      for (int s = 0; s < nks; ++s) {
        const int p = qt + 2 * s;
        const LDS_AS char* sA0 = ring + (p % SA) * GSZ;
        const LDS_AS char* sA1 = ring + ((p + 1) % SA) * GSZ;
        const LDS_AS char* sB = ring + (SA + (p + (wc >> 1)) % SB) * GSZ;
        const bool last = s + 1 == nks;
        // L0
#pragma unroll
        for (int i = 0; i < 4; ++i) Aa[i] = frag<true, 128, 64>(sA0, wr * 64 + i * 16, 0, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) Ba[j] = frag<true, 128, 64>(sB, (wc & 1) * 64 + j * 16, 0, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) Ab[i] = frag<true, 128, 64>(sA0, wr * 64 + i * 16, 1, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) Bb[j] = frag<true, 128, 64>(sB, (wc & 1) * 64 + j * 16, 1, lane);
        dma_gran();
        if (isA) vm_wait<4 * (EA - 1)>();
        if (AUX && last) stg_aux();
        bar();
        istamp(s, 0);
        mm64(std::integral_constant<int, 0>{});
        bar();
        istamp(s, 1);
        // L1
#pragma unroll
        for (int i = 0; i < 4; ++i) Aa[i] = frag<true, 128, 64>(sA1, wr * 64 + i * 16, 0, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) Ab[i] = frag<true, 128, 64>(sA1, wr * 64 + i * 16, 1, lane);
        dma_gran();
        // counts: pieces issued after the awaited granule (+ 4 aux loads in the last step)
        constexpr int WA = 4 * (EA - 1), WB = 4 * (EB - 2);
        if (AUX && last) {
          if (isA) vm_wait<WA + 4>();
          else vm_wait<WB + 4>();
        } else {
          if (isA) vm_wait<WA>();
          else vm_wait<WB>();
        }
        bar();
        istamp(s, 2);
        mm64(std::integral_constant<int, 1>{});
#if VJ_GEMM_STAMPS
        if (s == 0) st_k1 = __builtin_amdgcn_s_memtime();
#endif
        if (!last || wr == 0) bar();
        istamp(s, 3);
      }
      q64 = qt + 2 * nks;
    } else if constexpr (STG) {
      // Staggered main loop. Per unit, each wave runs L | M (intervals between workgroup
      // barriers): L = the unit's fragment reads (A m-tiles 0-7, B n-tiles 0-3: 12 ds_read_b128) + its
      // 4 DMA pieces of unit q + 2, M = the unit's 32 MFMAs. Waves 4-7 run one interval behind waves
      // 0-3 (one extra barrier before their first tile), so while one wave of a SIMD pair issues
      // MFMAs the other reads LDS / issues DMA. Every wave waits for its own pieces of unit q + 1 at
      // the end of L of unit q (vmcnt(4): the 4 pieces of unit q + 2 stay in flight); the barrier
      // after it orders them before any wave's reads of q + 1.
      // Tile boundary: waves 0-3 go from the last M1's barrier into the epilogue and on to the next
      // tile's L0; waves 4-7 skip that barrier (their epilogue starts right after the last MFMAs)
      // and take it after the epilogue, before the next tile's L0 - the pairing (and the
      // half-interval stagger) is unchanged and the two epilogues overlap.
      if (wg == run0 + jb) {  // first tile: unit 0 landed everywhere, RoPE table published
        if constexpr (DIST == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (wr == 1) __builtin_amdgcn_s_barrier();
      }
      const int q0 = dpos - DIST;  // stream position of this tile's unit 0
      auto bar = [] {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      };
      for (int u = 0; u < nku; ++u) {
        const LDS_AS char* sA = ring + ((q0 + u) % NSL) * USZ;
        const LDS_AS char* sB = sA + 16384;
#pragma unroll
        for (int i = 0; i < 4; ++i) Aa[i] = frag<true, 256, 32>(sA, wr * 128 + i * 16, 0, lane);
#pragma unroll
        for (int j = 0; j < NTN; ++j) Ba[j] = frag<true, 256, 32>(sB, wc * WN + j * 16, 0, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) Ab[i] = frag<true, 256, 32>(sA, wr * 128 + 64 + i * 16, 0, lane);
        dma_half(std::integral_constant<int, 0>{});
        dma_half(std::integral_constant<int, 1>{});
        // unit q + 1 landed: the pieces of units q + 2 .. q + DIST (4 each) stay in flight, and the aux
        // rows fetched one unit ago
        // rows fetched one unit ago (exactly 4 loads per lane: one per row). Any other load issued
        // after unit q + 1's pieces (the tile's bias / RoPE ids) only lengthens the wait.
        if (AUX && u == nku - 1 && nku > 1) {
          if constexpr (DIST == 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
#if VJ_DIAG_NOWAIT
          asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
#else
          if constexpr (DIST == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
#endif
        }
        if (AUX && u == nku - 2) stg_aux();
        if (AUX && nku == 1) stg_aux();
        bar();
        mm(Aa, 0, Ba);
        mm(Ab, 1, Ba);
#if VJ_GEMM_STAMPS
        if (u == 1) st_k1 = __builtin_amdgcn_s_memtime();
#endif
        if (u + 1 < nku || wr == 0) bar();
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if constexpr (F8) {
        rdA8(Xa, par, 0);
        rdB8(0, NTN / 2, par);
      } else {
        rdA(Aa, par, 0, 0);
        rdB(Ba, par, 0);
      }

      // Per K-tile t: 4 phases, each with the fragments of the NEXT phase read while the current
      // phase's MFMAs run: (k-step, M-half) = (0,0) (0,1) (1,0) (1,1), 4*NTN MFMAs each. One barrier
      // per tile, before phase 3 (whose prefetch reads
      // tile t+1): it retires this wave's DMA of tile t+1 (issued one tile earlier) and its reads of
      // tile t; then slot (t + par) & 1 is free for the DMA of tile t+2, or of the next tile's stages
      // once this tile has none left.
      const __amdgpu_buffer_rsrc_t ra = rsrc_a(cur), rb = rsrc_b(cur);
      // 8-wave bf16 main loop: only the A pieces of K-tile t + 2 go out after the barrier; the B pieces
      // are issued inside the last phase's MFMAs (SPLIT: m-tiles / MFMAs before them)
      constexpr bool SPREAD = NWV == 8 && !F8 && BK == 64;
      constexpr int SPLIT = MH == 4 ? SPLIT_AT : MH - 1;
      // one K-tile; TAIL (the last two K-tiles) DMAs the next tile's stages instead of this tile's
      auto ktile = [&](const int t, auto tail_c) {
        constexpr bool TAIL = decltype(tail_c)::value;
        const int sl = (t + par) & 1;
        if constexpr (F8) {
          // m-quarters q0..q2 (A: Aa, Ab alternate); B's upper n-tiles of this K-tile arrive under
          // q0's lower-half MFMAs
          rdB8(NTN / 2, NTN, sl);
          rdA8(Xb, sl, 1);
          __builtin_amdgcn_sched_barrier(0);
          mm8(Xa, 0, 0, NTN / 2);
          mm8(Xa, 0, NTN / 2, NTN);
          __builtin_amdgcn_sched_barrier(0);
          rdA8(Xa, sl, 2);
          __builtin_amdgcn_sched_barrier(0);
          mm8(Xb, 1, 0, NTN);
          __builtin_amdgcn_sched_barrier(0);
          rdA8(Xb, sl, 3);
          __builtin_amdgcn_sched_barrier(0);
          mm8(Xa, 2, 0, NTN);
          __builtin_amdgcn_sched_barrier(0);
        } else if constexpr (BK == 32) {
          // one k-step: phase 0 = (M-half 0) under the read of M-half 1's A fragments; phase 1 after
          // the barrier, the next K-tile's fragments read under its MFMAs
          rdA(Ab, sl, 1, 0);
          __builtin_amdgcn_sched_barrier(0);
          mm(Aa, 0, Ba);
          __builtin_amdgcn_sched_barrier(0);
        } else {
          release(Aa, Ba);
          rdA(Ab, sl, 1, 0);
          __builtin_amdgcn_sched_barrier(0);
          mm(Aa, 0, Ba);
          __builtin_amdgcn_sched_barrier(0);
          release(Ab, Ba);
          rdA(Aa, sl, 0, 1);
          rdB(Bb, sl, 1);
          __builtin_amdgcn_sched_barrier(0);
          mm(Ab, 1, Ba);
          __builtin_amdgcn_sched_barrier(0);
          release(Aa, Bb);
          rdA(Ab, sl, 1, 1);
          __builtin_amdgcn_sched_barrier(0);
          mm(Aa, 0, Bb);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the next tile's stage 0 stays in flight
        if constexpr (ASYNC) {
          tie(Ab);
          tie(Bb);
        }
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!TAIL) {
          if constexpr (SPREAD) {
            if (iss && !VJ_DIAG_NODMA)
              stage<AK, BM, false, DMAW, BK, WNX, PB>(ra, g.lda, g.M - cur.m0, (t + 2) * BK, cur.Keff,
                                                       smem + sl * STAGE, wave, lane);
          } else {
            load_k(ra, rb, cur, t + 2, sl, lane);
          }
        } else if (has_next) {
          // slot sl is free: the next tile's stage 0 (t == nk-2) or stage 1 (t == nk-1; stage 0 goes
          // to the other, unused slot when nk == 1); stage 1 waits for the epilogue unless EARLY1
          int lt = lane;
          asm volatile("" : "+v"(lt));  // tail-only addressing: not hoisted across the main loop
          const Tile nx = make_tile(wgn);
          if (t + 2 == nk) {
            load_tile(nx, 0, sl, lt);
          } else {
            if (nk == 1) load_tile(nx, 0, sl ^ 1, lt);
            if (EARLY1 && nx.nk > 1) load_tile8(nx, 1, sl, lt);
          }
        }
        auto b_pieces = [&] {
          if (iss && !VJ_DIAG_NODMA)
            stage<BKM, BN, DIRECT, DMAW, BK, WNX, PB>(rb, g.ldb, g.N - cur.n0, (t + 2) * BK, cur.Keff,
                                                       smem + sl * STAGE + A_BYTES, wave, lane);
        };
        if constexpr (F8) {
          // q3; the next K-tile's q0 A fragments and lower B n-tiles are read under it
          if (t + 1 < nk) rdA8(Xa, sl ^ 1, 0);
          __builtin_amdgcn_sched_barrier(0);
          mm8(Xb, 3, 0, NTN / 2);
          __builtin_amdgcn_sched_barrier(0);
          if (t + 1 < nk) rdB8(0, NTN / 2, sl ^ 1);
          __builtin_amdgcn_sched_barrier(0);
          mm8(Xb, 3, NTN / 2, NTN);
          __builtin_amdgcn_sched_barrier(0);
        } else if constexpr (BK == 32) {
          mm(Ab, 1, Ba);
          __builtin_amdgcn_sched_barrier(0);
          if (t + 1 < nk) {  // overwrite Aa / Ba once phase 1's MFMAs have been issued
            rdA(Aa, sl ^ 1, 0, 0);
            rdB(Ba, sl ^ 1, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
        } else {
          if (t + 1 < nk) {
            rdA(Aa, sl ^ 1, 0, 0);
            rdB(Ba, sl ^ 1, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (SPREAD && !TAIL) {
            mm_rows(Ab, 1, Bb, 0, SPLIT);
            __builtin_amdgcn_sched_barrier(0);
            b_pieces();
            __builtin_amdgcn_sched_barrier(0);
            mm_rows(Ab, 1, Bb, SPLIT, MH);
          } else {
            mm(Ab, 1, Bb);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      int t = 0;
      for (; t + 2 < nk; ++t) ktile(t, std::false_type{});
      for (; t < nk; ++t) ktile(t, std::true_type{});
    }

    // the epilogue's lane-derived addressing is recomputed per tile (an opaque copy of the lane id
    // keeps the compiler from hoisting it out of the tile loop, where it would hold VGPRs across the
    // main loop)
#if VJ_GEMM_STAMPS
    const long st1 = __builtin_amdgcn_s_memtime();
#endif
    int lane_e = lane;
    asm volatile("" : "+v"(lane_e));
    if constexpr (DIRECT) {
      const int lane = lane_e;
      const int lrow = 4 * (lane >> 4);  // the lane's row offset in an m-tile
      // ---- direct epilogue (K-major B staged with PERM): lane (c = lane&15, g = lane>>4) owns rows
      // rowoff(i) + 4g + r of m-tile i and the NTN
      // consecutive columns nb .. nb+NTN-1, so every row goes out of registers as one 8/16-B store;
      // no LDS round trip.
      const int nb = cur.n0 + wc * WN + NTN * (lane & 15);
      const bool nok = nb < g.N;
      const int mb = cur.m0 + wr * WRS + lrow;
      float bias[NTN];
#pragma unroll
      for (int j = 0; j < NTN; ++j) bias[j] = STG ? biasp[j] : 0.f;
      if (!STG && EPI != EPI_GELU_BWD && !PART && g.bias && nok)
#pragma unroll
        for (int j = 0; j < NTN; ++j) bias[j] = g.bias[nb + j];
      // RoPE (modules.py:26-50, 343-365): tile rows' (frame, row, col) positions + interleaved
      // cos/sin table in LDS; this lane's NTN/2 column pairs fix slice/axis/frequency once.
      [[maybe_unused]] bool ract[NTN / 2];
      [[maybe_unused]] int rsh[NTN / 2], rf0[NTN / 2], rf1[NTN / 2];
      if constexpr (EPI == EPI_ROPE) {
        const RopeP& r = g.rope;
        const int t = threadIdx.x;
        if (t < BM) {  // the previous tile's readers are past this tile's main-loop barriers
          const int fr = pf_id / r.tpf, rem = pf_id - r.tpf * fr, hr = rem / r.tpr;
          rpos[t] = fr | (hr << 10) | ((rem - r.tpr * hr) << 20);
        }
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
      // residual (f32) / pre-activation (bf16 bits) rows: m-tile i+1's fetched while m-tile i is stored
      // AUX_PF m-tiles of rows in flight. Stamped (tools/gemm_stamps.py): the residual epilogue takes
      // ~36k cycles per tile vs ~10k without the reads, but deeper prefetch (3, 5, 7) measured no
      // faster: the 64 MB of residual every CU reads at once is the bound, not the latency chain
      [[maybe_unused]] float aux[AUX_PF + 1][4][NTN];
      // per-tile lane offsets (elements): row r of virtual m-tile i is then + (rowoff(i) + r) * ld, a
      // wave-uniform (scalar) product, instead of a 64-bit multiply per row
      [[maybe_unused]] const long off_aux = AUX ? (long)mb * g.ldaux + nb : 0;
      auto fetch = [&](int i, float (&dst)[4][NTN]) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = mb + rowoff(i) + r;
          const bool ok = m < g.M && nok;
          const long off = ok ? off_aux + (long)(rowoff(i) + r) * g.ldaux : 0;
          if constexpr (EPI == EPI_F32_RESID) {
            if constexpr (NTN == 4) {
              const float4 x = *(const float4*)((const float*)g.aux + off);
              dst[r][0] = x.x; dst[r][1] = x.y; dst[r][2] = x.z; dst[r][3] = x.w;
            } else {
              const float2 x = *(const float2*)((const float*)g.aux + off);
              dst[r][0] = x.x; dst[r][1] = x.y;
            }
          } else {
            auto lo = [](uint32_t u) { return __builtin_bit_cast(float, u << 16); };  // bf16 -> f32, exact
            auto hi = [](uint32_t u) { return __builtin_bit_cast(float, u & 0xffff0000u); };
            if constexpr (NTN == 4) {  // saved GELU derivative
              const uint2 x = *(const uint2*)((const bf16_t*)g.aux + off);
              dst[r][0] = lo(x.x); dst[r][1] = hi(x.x);
              dst[r][2] = lo(x.y); dst[r][3] = hi(x.y);
            } else {
              const uint32_t x = *(const uint32_t*)((const bf16_t*)g.aux + off);
              dst[r][0] = lo(x); dst[r][1] = hi(x);
            }
          }
        }
      };
      // bf16 rows widened to 16-B stores: lanes c (even) and c + 1 swap row halves, so the even lane
      // stores rows 0, 1 and the odd lane rows 2, 3 of the 8 columns 4 (c & ~1) .. + 7 (N % 8 == 0)
      const bool odd = lane & 1;
      const int nb8 = nb - (odd ? 4 : 0);
      const bool nok8 = nb8 < g.N;
      const int mrow = mb + (odd ? 2 : 0);  // first row this lane stores of a virtual m-tile
      // every register index below is a compile-time constant (a lane-dependent row index into pk
      // compiled to a compare / select chain over all 8 words per store)
      auto store_wide = [&](bf16_t* base, long ld, long off, int i, const uint32_t (&pk)[4][2]) {
        uint32_t snd[4], keep[4], rcv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          snd[k] = odd ? pk[k >> 1][k & 1] : pk[2 + (k >> 1)][k & 1];
          keep[k] = odd ? pk[2 + (k >> 1)][k & 1] : pk[k >> 1][k & 1];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) rcv[k] = dpp_u<DPP_XOR1>(snd[k]);  // lane pair exchange on the VALU
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (mrow + rowoff(i) + h < g.M && nok8) {
            const uint32_t a = 2 * h, b = 2 * h + 1;
            const uint4 v = make_uint4(odd ? rcv[a] : keep[a], odd ? rcv[b] : keep[b], odd ? keep[a] : rcv[a],
                                       odd ? keep[b] : rcv[b]);
            *(uint4*)(base + off + (long)(rowoff(i) + h) * ld) = v;
          }
        }
      };
      // per-tile lane offsets of the bf16 outputs (C, C2) and the f32 output rows
      [[maybe_unused]] const long off_c = (long)mrow * g.ldc + nb8;
      [[maybe_unused]] const long off_c2 = EPI == EPI_GELU ? (long)mrow * g.ldc2 + nb8 : 0;
      [[maybe_unused]] const long off_f = PART ? ((long)cur.z * g.M + mb) * g.N + nb
                                                             : (long)mb * g.ldc + nb;
      [[maybe_unused]] const long ld_f = PART ? (long)g.N : g.ldc;
      [[maybe_unused]] float* const base_f = PART ? g.ws : (float*)g.C;
      if constexpr (AUX)
#pragma unroll
        for (int i = 0; i < AUX_PF; ++i) {
          if constexpr (STG) {  // m-tile 0, fetched under the last unit
            static_assert(AUX_PF == 1, "STG prefetches one m-tile of aux rows");
            auto lo = [](float u) { return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, u) << 16); };
            auto hi = [](float u) { return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, u) & 0xffff0000u); };
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if constexpr (EPI == EPI_F32_RESID) {
#pragma unroll
                for (int j = 0; j < NTN; ++j) aux[0][r][j] = auxr[r][j];
              } else {
                aux[0][r][0] = lo(auxr[r][0]); aux[0][r][1] = hi(auxr[r][0]);
                aux[0][r][2] = lo(auxr[r][1]); aux[0][r][3] = hi(auxr[r][1]);
              }
            }
          } else {
            fetch(i, aux[i]);
          }
        }
      // GELU: the derivative pass is compiled separately, for callers that save it (g.C)
      auto rows = [&](auto save_c) {
      constexpr bool SAVE_D = decltype(save_c)::value;
#pragma unroll
      for (int i = 0; i < 2 * MH; ++i) {
        if constexpr (AUX) {
          if (i + AUX_PF < 2 * MH) fetch(i + AUX_PF, aux[(i + AUX_PF) % (AUX_PF + 1)]);
          if (!STG && i == 2 * MH - 1 - AUX_PF && has_next) {  // behind the last aux fetch
            const Tile nxt = make_tile(wgn);
            if (nxt.nk > 1) load_tile8(nxt, 1, sle, lane);
          }
        }
        if constexpr (F32OUT && NTN == 4) {
          // f32 rows stored from the accumulators themselves: a 4x4 in-place transpose (tied swaps)
          // turns accv(i, r, 0..3) into row r's 4 columns, bias / residual are added in place (tied
          // adds). Stores read their data registers after issue, so staging copies recycled from row
          // to row cost one memory latency per 16-B store; the accumulators are not reused before the
          // next tile.
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = a + 1; b < 4; ++b) {
              float x = accv(i, a, b), y = accv(i, b, a);
              asm volatile("v_swap_b32 %0, %1" : "+v"(x), "+v"(y));
              accs(i, a, b, x);
              accs(i, b, a, y);
            }
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float x = accv(i, r, e);
              asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(bias[e]));
              if constexpr (EPI == EPI_F32_RESID) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(aux[i % (AUX_PF + 1)][r][e]));
              accs(i, r, e, x);
            }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = mb + rowoff(i) + r;
            if (m < g.M && nok) {
              float* dst = base_f + off_f + (long)(rowoff(i) + r) * ld_f;
              *(f32x4*)dst = acc[i][r];
            }
          }
          continue;
        }
        [[maybe_unused]] uint32_t pk[4][2], ga[4][2];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = mb + rowoff(i) + r;
          float v[NTN];
#pragma unroll
          for (int j = 0; j < NTN; ++j) v[j] = accv(i, j, r) + bias[j];
          if constexpr (EPI == EPI_ROPE) {
            const int rp = rpos[wr * WRS + rowoff(i) + lrow + r];
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
          if constexpr (EPI == EPI_F32_RESID || EPI == EPI_BF16_RESID) {
#pragma unroll
            for (int j = 0; j < NTN; ++j) v[j] += aux[i % (AUX_PF + 1)][r][j];
          }
          if constexpr (F32OUT) {
            if (m < g.M && nok) {
              float* dst = base_f + off_f + (long)(rowoff(i) + r) * ld_f;
              *(float4*)dst = make_float4(v[0], v[1], v[2], v[3]);
            }
          } else {
#pragma unroll
            for (int q2 = 0; q2 < 2; ++q2) {
              if constexpr (EPI == EPI_GELU_BWD)
                pk[r][q2] = pack_bf2(v[2 * q2] * aux[i % (AUX_PF + 1)][r][2 * q2],
                                     v[2 * q2 + 1] * aux[i % (AUX_PF + 1)][r][2 * q2 + 1]);
              else
                pk[r][q2] = pack_bf2(v[2 * q2], v[2 * q2 + 1]);
              if constexpr (EPI == EPI_GELU) {  // pk: the bf16 pre-activation -> GELU, derivative (if saved)
                if constexpr (GTAB) ga[r][q2] = gelu_pair_tab<SAVE_D>(pk[r][q2], smem, &pk[r][q2]);
                else ga[r][q2] = gelu_pair(pk[r][q2], SAVE_D ? &pk[r][q2] : nullptr);
              }
            }
          }
        }
        if constexpr (!F32OUT) {
          if (EPI != EPI_GELU || SAVE_D) store_wide((bf16_t*)g.C, g.ldc, off_c, i, pk);
          if constexpr (EPI == EPI_GELU) store_wide((bf16_t*)g.C2, g.ldc2, off_c2, i, ga);
        }
      }
      };
      if (EPI == EPI_GELU && g.C) rows(std::true_type{});
      else rows(std::false_type{});
    } else {
      const int lane = lane_e;
      // ---- staged epilogue: passes of MTP m-tiles (16*MTP rows) per wave through a padded image in
      // the last K-tile's slot (free now; the next tile's stage 1 is DMA'd there afterwards): 2 m-tiles
      // per pass where the image fits the slot (BN = 128), else 1
      constexpr int STR = WN + 4;    // floats per staged row (conflict-free ds_write_b32)
      constexpr int LPR = WN / 4;    // lanes per staged row (16-B each)
      constexpr int RPI = 64 / LPR;  // rows per wave-instruction
      constexpr int MTP = (8 * 32 * STR * 4 <= STAGE) ? 2 : 1;
      constexpr int PR = 16 * MTP;   // rows per pass
      constexpr int IT = PR / RPI;   // row-instructions per pass
      static_assert(8 * PR * STR * 4 <= STAGE, "staging image must fit one operand slot");
      LDS_AS float* wl = (LDS_AS float*)(smem + sle * STAGE + wave * PR * STR * 4);
      if constexpr (RS && MH == 4) {
        if (rs_on) {  // the row sums: lane groups (k sub-ranges) added, rows 32 wc + 16 (lane >> 4) + (lane & 15)
          float sa = rsa + __shfl_xor(rsa, 16), sb = rsb + __shfl_xor(rsb, 16);
          sa += __shfl_xor(sa, 32);
          sb += __shfl_xor(sb, 32);
          const int m = cur.m0 + wr * 128 + 32 * wc + (lane & 31);
          if (lane < 32 && m < g.M) g.rsum[(long)cur.z * g.M + m] = lane < 16 ? sa : sb;
        }
      }
      bool ract[2] = {false, false};
      int rsh[2] = {0, 0}, rf0[2] = {0, 0}, rf1[2] = {0, 0};
      const int col = (lane % LPR) * 4;  // this thread's 4 columns, fixed for every row it stores
      const int ncol = cur.n0 + wc * WN + col;
      if constexpr (EPI == EPI_ROPE) {
        const RopeP& r = g.rope;
        const int t = threadIdx.x;
        if (t < BM) {
          const int fr = pf_id / r.tpf, rem = pf_id - r.tpf * fr, hr = rem / r.tpr;
          rpos[t] = fr | (hr << 10) | ((rem - r.tpr * hr) << 20);
        }
        const int sw = 2 * r.half, e0 = (ncol % r.D) % r.hd;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int e = e0 + 2 * p, ax = e / sw, js = e - ax * sw;
          ract[p] = ncol < 2 * r.D && e < 3 * sw;
          rsh[p] = 10 * ax;
          rf0[p] = js % r.half;
          rf1[p] = (js + 1) % r.half;
        }
        __syncthreads();
      }
      float4 bias4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (EPI != EPI_GELU_BWD && !PART && g.bias && ncol < g.N) bias4 = *(const float4*)(g.bias + ncol);
#pragma unroll
      for (int pass = 0; pass < 8 / MTP; ++pass) {
#pragma unroll
        for (int ii = 0; ii < MTP; ++ii)
#pragma unroll
          for (int j = 0; j < NTN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              wl[(ii * 16 + (lane >> 4) * 4 + r) * STR + j * 16 + (lane & 15)] = acc[pass * MTP + ii][j][r];
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own writes visible to own reads (wave-private)
        // residual / GELU pre-activation rows of this pass fetched up front: one memory latency per
        // pass instead of one per row
        [[maybe_unused]] float4 rres[EPI == EPI_F32_RESID ? IT : 1];
        [[maybe_unused]] uint2 rpre[EPI == EPI_GELU_BWD || EPI == EPI_BF16_RESID ? IT : 1];
        if constexpr (AUX) {
#pragma unroll
          for (int it = 0; it < IT; ++it) {
            const int m = cur.m0 + wr * 128 + pass * PR + it * RPI + lane / LPR;
            const bool ok = m < g.M && ncol < g.N;
            const long mm2 = ok ? m : 0;
            const int nn = ok ? ncol : 0;
            if constexpr (EPI == EPI_F32_RESID) rres[it] = *(const float4*)((const float*)g.aux + mm2 * g.ldaux + nn);
            else rpre[it] = *(const uint2*)((const bf16_t*)g.aux + mm2 * g.ldaux + nn);
          }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
          const int row = it * RPI + lane / LPR;
          const f32x4 v4 = *(const LDS_AS f32x4*)(wl + row * STR + col);
          const int m = cur.m0 + wr * 128 + pass * PR + row;
          const int n = ncol;
          if (m >= g.M || n >= g.N) continue;
          float v[4] = {v4[0] + bias4.x, v4[1] + bias4.y, v4[2] + bias4.z, v4[3] + bias4.w};
          if constexpr (EPI == EPI_BF16 || EPI == EPI_ROPE) {
            if constexpr (EPI == EPI_ROPE) {
              const int rp = rpos[wr * 128 + pass * PR + row];
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
          } else if constexpr (PART) {
            *(float4*)(g.ws + ((long)cur.z * g.M + m) * g.N + n) = make_float4(v[0], v[1], v[2], v[3]);
          } else if constexpr (EPI == EPI_F32_RESID) {
            const float4 rr = rres[it];
            *(float4*)((float*)g.C + (long)m * g.ldc + n) = make_float4(rr.x + v[0], rr.y + v[1], rr.z + v[2], rr.w + v[3]);
          } else if constexpr (EPI == EPI_GELU) {
            uint32_t d0, d1;
            const uint32_t a0 = gelu_pair(pack_bf2(v[0], v[1]), &d0), a1 = gelu_pair(pack_bf2(v[2], v[3]), &d1);
            if (g.C) *(uint2*)((bf16_t*)g.C + (long)m * g.ldc + n) = make_uint2(d0, d1);
            *(uint2*)((bf16_t*)g.C2 + (long)m * g.ldc2 + n) = make_uint2(a0, a1);
          } else if constexpr (EPI == EPI_BF16_RESID) {
            const uint2 pu = rpre[it];  // bf16 residual
            auto lo = [](uint32_t u) { return __builtin_bit_cast(float, u << 16); };
            auto hi = [](uint32_t u) { return __builtin_bit_cast(float, u & 0xffff0000u); };
            *(uint2*)((bf16_t*)g.C + (long)m * g.ldc + n) =
                make_uint2(pack_bf2(lo(pu.x) + v[0], hi(pu.x) + v[1]), pack_bf2(lo(pu.y) + v[2], hi(pu.y) + v[3]));
          } else {  // EPI_GELU_BWD
            const uint2 pu = rpre[it];  // saved GELU derivative (bf16)
            auto lo = [](uint32_t u) { return __builtin_bit_cast(float, u << 16); };
            auto hi = [](uint32_t u) { return __builtin_bit_cast(float, u & 0xffff0000u); };
            *(uint2*)((bf16_t*)g.C + (long)m * g.ldc + n) =
                make_uint2(pack_bf2(v[0] * lo(pu.x), v[1] * hi(pu.x)), pack_bf2(v[2] * lo(pu.y), v[3] * hi(pu.y)));
          }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
      }
      __syncthreads();  // every wave is done with its image before the slot is DMA'd
      if (has_next) {
        const Tile nxt = make_tile(wgn);
        if (nxt.nk > 1) load_tile8(nxt, 1, sle, lane);
      }
    }

#if VJ_GEMM_STAMPS
    {
      if constexpr (!STG) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // STG: the DMA stream runs on
      const long st2 = __builtin_amdgcn_s_memtime();
      if (threadIdx.x == 0 && blockIdx.x < 2048 && stamp_it < 16) {
        long* d = vj_gemm_stamps + ((long)blockIdx.x * 16 + stamp_it) * 4;
        d[0] = st0; d[1] = st1; d[2] = st2; d[3] = st_k1;
      }
      ++stamp_it;
    }
#endif
    if constexpr (STG) {
      // waves 4-7: the barrier skipped after their last MFMAs (see the main loop); waves 0-3: the
      // matching one after the block's last tile, so both halves end with equal barrier counts
      if (wr == 1 || !has_next) __builtin_amdgcn_s_barrier();
    }
    if (!has_next) break;
    wg = wgn;
    cur = make_tile(wgn);
    par = parn;
  }
}

int num_cus() {
  static int cus[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cus[dev] <= 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cus[dev] = v;
  }
  return cus[dev];
}

// Persistent grid: one block per CU (capped by the tile count), a multiple of 8 so every XCD gets
// the same number of blocks. VJ_GEMM_PXCD caps the blocks per XCD (tests: many tiles per block).
// (A phase offset between the blocks of an XCD, so odd blocks' epilogues fall under the even
// blocks' main loops, measured no gain in round 3 and was removed.)
// CUs the persistent grids leave free (vj_set_reserved_cus): while a data-parallel rank's gradient
// buckets are all-reduced, RCCL's channel kernels hold CUs; a persistent GEMM block that cannot be
// placed on one of them only starts when it frees, and its statically assigned tiles then run after
// every other block's (measured on one GPU with a 16-CU proxy copy: step -11.6 %,
// profiles/r06_rccl_proxy_ab.txt). Set by distributed.GradReducer around its bucket window.
std::atomic<int> g_reserved_cus{0};

int grid256(long nb, int per_cu = 1) {
  int per_xcd = per_cu * (num_cus() - g_reserved_cus.load(std::memory_order_relaxed)) / 8;
  const char* e = getenv("VJ_GEMM_PXCD");
  if (e && atoi(e) > 0) per_xcd = atoi(e);
  if (per_xcd < 1) per_xcd = 1;
  const long need = (nb + 7) / 8;
  return 8 * (int)(need < per_xcd ? need : per_xcd);
}

// Grouped tile order (tile rows per group): a square-ish set of the ~32 tiles an XCD has in flight
// shares fewer A / B panels in its L2. Measured (tools/bench_kernels.py, MI355X): groups of 8 rows
// pay on tall problems (target fc1 M = 49152: -7 %, predictor fc1 / fc2 / dgrad M = 71232: -3..-10 %)
// and cost 2-5 % on the ~46-row-tile context problems (round 3). With the round-4 kernels and the
// concurrent streams, groups of 4 rows on every problem measured best per step: +0.4 % / +0.25 % over
// 8-or-row-major, +0.1 % over 8 on the tall ones with 4 on the rest (profiles/r04_gemm_group_ab.txt;
// in isolation 8 is still ~1 % ahead on the target fc1 / QKV, 4 ahead on context QKV / dgrad).
// VJ_GEMM_GROUP overrides (0 = row-major; tests: grouped order at small sizes).
int tile_group(int tiles_m, int tiles_n) {
  const char* e = getenv("VJ_GEMM_GROUP");
  if (e) return atoi(e) > 0 ? atoi(e) : 0;
  (void)tiles_m;
  (void)tiles_n;
  return 4;
}

template <int BN>
int launch256_f8(int epi, const G256& g, hipStream_t st) {
  const dim3 grid(grid256((long)g.tiles_m * g.tiles_n));
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL((k_gemm256<true, true, EPI_BF16, BN, true>), grid, dim3(512), 0, st, g); break;
    case EPI_F32: hipLaunchKernelGGL((k_gemm256<true, true, EPI_F32, BN, true>), grid, dim3(512), 0, st, g); break;
    case EPI_F32_RESID:
      hipLaunchKernelGGL((k_gemm256<true, true, EPI_F32_RESID, BN, true>), grid, dim3(512), 0, st, g);
      break;
    case EPI_GELU: hipLaunchKernelGGL((k_gemm256<true, true, EPI_GELU, BN, true>), grid, dim3(512), 0, st, g); break;
    case EPI_ROPE: hipLaunchKernelGGL((k_gemm256<true, true, EPI_ROPE, BN, true>), grid, dim3(512), 0, st, g); break;
    default: vj_set_error("vj_gemm_fp8: unsupported epilogue %d", epi); return VJ_ERR_ARG;
  }
  VJ_LAUNCH_CHECK("vj_gemm_fp8");
  return VJ_OK;
}

// Two-workgroups-per-CU kernel (NWV = 4, 256 x 128 tiles, 32-deep K) for K-major GEMMs whose N
// needs 128-wide tiles: its direct-store epilogue overlaps the other workgroup's MFMAs. Measured
// (tools/bench_kernels.py): predictor fc2 N = 384 (f32 residual epilogue) -14 %, N = 384 bf16 even;
// on 256-wide shapes its 32-deep main loop loses 10-20 %, so they stay on the 8-wave kernel.
// VJ_GEMM_2W: 0 = never, 1 = every K-major GEMM, unset = the 128-wide shapes.
int use_2w(bool narrow) {
  const char* e = getenv("VJ_GEMM_2W");
  if (e && e[0] == '0') return 0;
  if (e && e[0] == '1') return 1;
  return narrow ? 1 : 0;
}

int launch2w(int epi, G256 g, hipStream_t st) {
  const dim3 grid(grid256((long)g.tiles_m * g.tiles_n, 2));
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL((k_gemm256<true, true, EPI_BF16, 128, false, 4>), grid, dim3(256), 0, st, g); break;
    case EPI_F32: hipLaunchKernelGGL((k_gemm256<true, true, EPI_F32, 128, false, 4>), grid, dim3(256), 0, st, g); break;
    case EPI_F32_RESID:
      hipLaunchKernelGGL((k_gemm256<true, true, EPI_F32_RESID, 128, false, 4>), grid, dim3(256), 0, st, g);
      break;
    case EPI_GELU: hipLaunchKernelGGL((k_gemm256<true, true, EPI_GELU, 128, false, 4>), grid, dim3(256), 0, st, g); break;
    case EPI_GELU_BWD:
      hipLaunchKernelGGL((k_gemm256<true, true, EPI_GELU_BWD, 128, false, 4>), grid, dim3(256), 0, st, g);
      break;
    case EPI_ROPE: hipLaunchKernelGGL((k_gemm256<true, true, EPI_ROPE, 128, false, 4>), grid, dim3(256), 0, st, g); break;
    case EPI_BF16_RESID:
      hipLaunchKernelGGL((k_gemm256<true, true, EPI_BF16_RESID, 128, false, 4>), grid, dim3(256), 0, st, g);
      break;
    default: vj_set_error("gemm2w: bad epilogue %d", epi); return VJ_ERR_ARG;
  }
  VJ_LAUNCH_CHECK("vj_gemm256(2w)");
  return VJ_OK;
}

// The 4-wave two-workgroup kernel on 192 x 128 tiles, 64 deep: each 1-KB DMA piece is 8 whole 128-B
// rows, where the 256 x 128 tiles' 32-deep pieces fetch 16 half lines (twice the L1 -> L2 requests,
// which bound that kernel: profiles/r05_gemm_dma_diag.txt). Bitwise the same outputs; predictor fc2
// 132 -> 115 us, QKV / proj data gradients -8..-11 %, step +0.4 % (profiles/r05_gemm_2w192_ab.txt).
// VJ_GEMM_2W192=0 restores the 256 x 128 form; RoPE keeps it (no room for its table at 2 x 80 KB).
int launch2w192(int epi, G256 g, hipStream_t st) {
  g.tiles_m = vj_cdiv(g.M, 192);
  g.group = tile_group(g.tiles_m, g.tiles_n);
  const dim3 grid(grid256((long)g.tiles_m * g.tiles_n, 2));
#define L2W(E) hipLaunchKernelGGL((k_gemm256<true, true, E, 128, false, 4, 192>), grid, dim3(256), 0, st, g); break
  switch (epi) {
    case EPI_BF16: L2W(EPI_BF16);
    case EPI_F32: L2W(EPI_F32);
    case EPI_F32_RESID: L2W(EPI_F32_RESID);
    case EPI_GELU: L2W(EPI_GELU);
    case EPI_GELU_BWD: L2W(EPI_GELU_BWD);
    case EPI_BF16_RESID: L2W(EPI_BF16_RESID);
    default: vj_set_error("gemm2w192: bad epilogue %d", epi); return VJ_ERR_ARG;
  }
#undef L2W
  VJ_LAUNCH_CHECK("vj_gemm256(2w192)");
  return VJ_OK;
}
bool use_2w192(int epi) {
  const char* e = getenv("VJ_GEMM_2W192");
  return !(e && e[0] == '0') && epi != EPI_ROPE;
}

// one-tile launch; 192-row tiles (BMT = 192) for the K-major 256-wide shapes use_bm192() picks
int launch192(int epi, const G256& g, hipStream_t st) {
  const dim3 grid(grid256((long)g.tiles_m * g.tiles_n));
#define L192(E) hipLaunchKernelGGL((k_gemm256<true, true, E, 256, false, 8, 192>), grid, dim3(512), 0, st, g); break
  switch (epi) {
    case EPI_BF16: L192(EPI_BF16);
    case EPI_F32: L192(EPI_F32);
    case EPI_F32_RESID: L192(EPI_F32_RESID);
    case EPI_GELU: L192(EPI_GELU);
    case EPI_GELU_BWD: L192(EPI_GELU_BWD);
    case EPI_ROPE: L192(EPI_ROPE);
    case EPI_BF16_RESID: L192(EPI_BF16_RESID);
    default: vj_set_error("gemm192: bad epilogue %d", epi); return VJ_ERR_ARG;
  }
#undef L192
  VJ_LAUNCH_CHECK("vj_gemm256(192)");
  return VJ_OK;
}

// Tile rows for a K-major 256-wide GEMM: 192 when its rounds of tiles over the CUs cost clearly less
// than with 256 rows: rounds x rows, 192-row tiles charged 8 % for their lower MFMA : fragment-read
// ratio (measured 6-9 % on full-round shapes), and at least 15 % predicted gain (a predictor step
// whose M made the 8 % rule pick 192 ran its fc1 / dgrad slower). Context GEMMs (M ~ 11.7k,
// N = 1024 / 3072) take 192; the target / predictor shapes keep 256. VJ_GEMM_BM192: 0 = never,
// 1 = always, unset = the cost model.
bool use_bm192(int M, int tn) {
  const char* e = getenv("VJ_GEMM_BM192");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  const long cus = num_cus();
  const long r256 = ((long)vj_cdiv(M, 256) * tn + cus - 1) / cus;
  const long r192 = ((long)vj_cdiv(M, 192) * tn + cus - 1) / cus;
  return r192 * 192 * 108 < r256 * 256 * 85;
}

// Staggered main loop (STG) for the K-major 256 x 256-tile GEMMs: form 1 = 32-deep units (K % 32 == 0),
// form 2 = S64, 64-deep whole-line granules (K % 64 == 0); 0 = the one-tile kernel. Measured, round 4
// (profiles/r04_gemm_staggered_step.txt): form 1 pays on the GELU / RoPE / bf16 / f32 epilogues (-1.6..-1.8 %
// in the step) and not on the residual / saved-derivative ones. Round 6 (profiles/r06_gemm_s64.txt):
// isolated, S64 runs a K step 3-4 % faster where the operand panels stream from beyond L2 (K = 4096:
// target fc2 -2.4..-4 %) and takes the residual epilogues below the one-tile kernel (target proj / fc2,
// bf16 or f32 residual, -1..-4 %), but is 4-12 % slower per K step on the L2-resident K = 1024 panels of
// the QKV / GELU / RoPE / data-gradient GEMMs; in the train step, where the side streams' GEMMs share the
// chip (and its L2), S64 on every shape beats both the round-5 choice (+0.8 %) and S64 only on K >= 2048
// and the residual epilogues (+0.55 %), two interleaved runs each in one call. Default: S64 wherever
// K % 64 == 0, else form 1 on the epilogues without aux rows. VJ_GEMM_STG: 0 = never, 1 = every epilogue
// (form 1 where S64 cannot run); VJ_GEMM_STG64: 0 / 1 forces form 1 / 2 wherever a staggered loop runs.
int use_stg(int K, int epi) {
  if (K % 32) return 0;
  const char* e = getenv("VJ_GEMM_STG");
  if (e && e[0] == '0') return 0;
  const bool aux = epi == EPI_F32_RESID || epi == EPI_BF16_RESID || epi == EPI_GELU_BWD;
  int form = 2;
  const char* f = getenv("VJ_GEMM_STG64");
  if (f && f[0] == '0') form = 1;
  if (f && f[0] == '1') form = 2;
  if (form == 2 && K % 64) form = 1;
  if (aux && form == 1 && !(e && e[0] == '1')) return 0;
  return form;
}

template <int FORM>
int launch_stg(int epi, const G256& g, hipStream_t st) {
  const dim3 grid(grid256((long)g.tiles_m * g.tiles_n));
#define LSTG(E) hipLaunchKernelGGL((k_gemm256<true, true, E, 256, false, 8, 256, FORM>), grid, dim3(512), 0, st, g); break
  switch (epi) {
    case EPI_BF16: LSTG(EPI_BF16);
    case EPI_F32: LSTG(EPI_F32);
    case EPI_F32_RESID: LSTG(EPI_F32_RESID);
    case EPI_GELU: LSTG(EPI_GELU);
    case EPI_GELU_BWD: LSTG(EPI_GELU_BWD);
    case EPI_ROPE: LSTG(EPI_ROPE);
    case EPI_BF16_RESID: LSTG(EPI_BF16_RESID);
    default: vj_set_error("gemm256(stg): bad epilogue %d", epi); return VJ_ERR_ARG;
  }
#undef LSTG
  VJ_LAUNCH_CHECK("vj_gemm256(stg)");
  return VJ_OK;
}

template <bool AK, bool BKM, int BN>
int launch256(int epi, const G256& g, hipStream_t st) {
  const dim3 grid(grid256((long)g.tiles_m * g.tiles_n * g.nsplit));
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_BF16, BN>), grid, dim3(512), 0, st, g); break;
    case EPI_F32: hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_F32, BN>), grid, dim3(512), 0, st, g); break;
    case EPI_F32_RESID: hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_F32_RESID, BN>), grid, dim3(512), 0, st, g); break;
    case EPI_GELU: hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_GELU, BN>), grid, dim3(512), 0, st, g); break;
    case EPI_GELU_BWD: hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_GELU_BWD, BN>), grid, dim3(512), 0, st, g); break;
    case EPI_ROPE: hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_ROPE, BN>), grid, dim3(512), 0, st, g); break;
    case EPI_BF16_RESID:  // forward GEMMs only (A and B K-major); other layouts take the generic kernel
      if constexpr (AK && BKM) {
        hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_BF16_RESID, BN>), grid, dim3(512), 0, st, g);
        break;
      } else {
        return VJ_ERR_UNSUPPORTED;
      }
    case EPI_PARTIAL:  // split-K weight gradients only: dY^T X, both operands MN-major
      if constexpr (!AK && !BKM) {
        hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_PARTIAL, BN>), grid, dim3(512), 0, st, g);
        break;
      } else {
        return VJ_ERR_UNSUPPORTED;
      }
    case EPI_PARTIAL_RS:  // the same with the fused bias gradient (g.rsum)
      if constexpr (!AK && !BKM) {
        hipLaunchKernelGGL((k_gemm256<AK, BKM, EPI_PARTIAL_RS, BN>), grid, dim3(512), 0, st, g);
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

extern "C" int vj_set_reserved_cus(int n) {
  VJ_CHECK_ARG(n >= 0 && n <= num_cus() - 8, "vj_set_reserved_cus: %d of %d CUs", n, num_cus());
  g_reserved_cus.store(n, std::memory_order_relaxed);
  return VJ_OK;
}

// 256-wide column tiles unless the last one would waste more than 15 % of the work (measured,
// tools/bench_kernels.py: predictor QKV N = 1152 -17 % with 256-wide tiles; N = 384 +14 %)
#ifndef VJ_WIDE_ALL
#define VJ_WIDE_ALL 0  // variant builds: 256-wide column tiles for every N > 256
#endif
bool wide_tile_ok(int N) {
  return N % 256 == 0 || (N > 256 && (VJ_WIDE_ALL || vj_cdiv(N, 256) * 256L * 100 <= 115L * N));
}

// Called by vj_gemm_bf16_splitk (splitk == 1) when the problem suits a 256-row tile; arguments
// already validated there. Returns VJ_ERR_UNSUPPORTED when it declines.
int vj_gemm256_dispatch(int M, int N, int K, const void* A, long lda, int a_kmajor, const void* B, long ldb,
                        int b_kmajor, int epi, const float* bias, const void* aux, long ldaux, void* C, long ldc,
                        void* C2, long ldc2, hipStream_t st, const void* rope) {
  if (epi < EPI_BF16 || (epi > EPI_ROPE && epi != EPI_BF16_RESID) || N % 8 || ldc % 4 || ldc2 % 4 || ldaux % 4)
    return VJ_ERR_UNSUPPORTED;
  if (((uintptr_t)C & 15) || ((uintptr_t)C2 & 15) || ((uintptr_t)aux & 15) || ((uintptr_t)bias & 15))
    return VJ_ERR_UNSUPPORTED;
  const int bn = wide_tile_ok(N) ? 256 : 128;  // direct-store epilogue on the 256-wide tiles
  const int tm = vj_cdiv(M, 256), tn = vj_cdiv(N, bn);
  G256 g{(const bf16_t*)A, (const bf16_t*)B, M, N, K, lda, ldb, C, ldc, C2, ldc2, bias, aux, ldaux,
         tm, tn, RopeP{}, K, 1, nullptr, tile_group(tm, tn)};
  if (epi == EPI_ROPE) {
    if (!rope) return VJ_ERR_UNSUPPORTED;
    g.rope = *(const RopeP*)rope;
    if (g.rope.hd % 4 || g.rope.D % 4 || g.rope.npos < 1 || g.rope.npos > 1024) return VJ_ERR_UNSUPPORTED;
    if ((long)g.rope.npos * g.rope.half > ROPE_TAB_MAX) return VJ_ERR_UNSUPPORTED;
  }
  if (a_kmajor && b_kmajor && use_2w(bn == 128)) {
    g.tiles_n = vj_cdiv(N, 128);
    if (use_2w192(epi)) return launch2w192(epi, g, st);
    return launch2w(epi, g, st);
  }
  if (bn == 256) {
    // 192-row tiles run the one-tile main loop; where S64 can run instead (K % 64 == 0) the 256-row S64
    // tiles measured +0.2 % per step over the cost model's 192-row picks (the context GEMMs;
    // VJ_GEMM_BM192=0 vs default, two same-call runs each, profiles/r06_gemm_s64.txt).
    // VJ_GEMM_BM192=1 still forces them.
    const char* bm = getenv("VJ_GEMM_BM192");
    const bool s64_ok = a_kmajor && b_kmajor && use_stg(K, epi) == 2 && !(bm && bm[0] == '1');
    if (a_kmajor && b_kmajor && !s64_ok && use_bm192(M, tn)) {
      g.tiles_m = vj_cdiv(M, 192);
      g.group = tile_group(g.tiles_m, tn);
      return launch192(epi, g, st);
    }
    if (a_kmajor && b_kmajor) {
      const int form = use_stg(K, epi);
      if (form == 2) return launch_stg<2>(epi, g, st);
      if (form == 1) return launch_stg<1>(epi, g, st);
    }
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
// 256-row tiles; the caller reduces the slabs. rsum (or null): the row sums of A per K slice,
// [splitk][M] (fused bias gradient). Returns VJ_ERR_UNSUPPORTED when it declines.
int vj_gemm256_partial(int M, int N, int K, const void* A, long lda, int a_kmajor, const void* B, long ldb,
                       int b_kmajor, int kslice, int splitk, float* ws, hipStream_t st, float* rsum) {
  if (a_kmajor || b_kmajor || N % 8 || M < 256 || N < 128) return VJ_ERR_UNSUPPORTED;
  // 256-wide tiles unless the last one would waste more than 15 % of the columns (the forward GEMMs'
  // rule): ViT-g's N = 1408 runs 6 tiles of 256 instead of 11 of 128 (twice the work per operand byte)
  const int bn = wide_tile_ok(N) ? 256 : 128;
  const int tm = vj_cdiv(M, 256), tn = vj_cdiv(N, bn);
  if ((long)tm * tn * splitk > 0x7fffffffL) return VJ_ERR_UNSUPPORTED;
  G256 g{(const bf16_t*)A, (const bf16_t*)B, M, N, K, lda, ldb, nullptr, 0, nullptr, 0, nullptr, nullptr, 0,
         tm, tn, RopeP{}, kslice, splitk, ws, tile_group(tm, tn)};
  g.rsum = rsum;
  const int epi = rsum ? EPI_PARTIAL_RS : EPI_PARTIAL;
  return bn == 256 ? launch256<false, false, 256>(epi, g, st) : launch256<false, false, 128>(epi, g, st);
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
  if (M >= 1024) {
    RopeP rp{ids, ids_mod, tpf, tpr, half, hd, H * hd, cos_t, sin_t, npos};
    const int rc = vj_gemm256_dispatch(M, N, K, A, lda, 1, B, ldb, 1, EPI_ROPE, bias, nullptr, 0, C, ldc, nullptr, 0,
                                       (hipStream_t)stream, &rp);
    if (rc != VJ_ERR_UNSUPPORTED) return rc;
  }
  int rc = vj_gemm_bf16(M, N, K, A, lda, 1, B, ldb, 1, EPI_BF16, bias, nullptr, 0, C, ldc, nullptr, 0, stream);
  if (rc) return rc;
  return vj_rope(M, H, hd, C, ldc, 0, H * hd, ids, ids_mod, tpf, tpr, cos_t, sin_t, half, 0, stream);
}

// ---- fp8 forward GEMMs (opt-in fp8 target-encoder path, BASELINE configs[4]) -----------------------
// A [M, K] and B [N, K] are OCP e4m3 bytes, both K-major (X W^T), with per-row power-of-two scales:
// A(m, k) = A8[m, k] * 2^ea[m], B(n, k) = B8[n, k] * 2^eb[n] (ea / eb device int32; vj_quant_rows_fp8
// or vj_layernorm_fwd_fp8 produce them). The 256-row kernel reads the bytes as bf16 pairs: K, lda and
// ldb must be multiples of 16 bytes. Epilogues as vj_gemm_bf16 (BF16, F32, F32_RESID, GELU) / RoPE.
static int gemm256_f8(int M, int N, int K, const void* A, long lda, const int* ea, const void* B, long ldb,
                      const int* eb, int epi, const float* bias, const void* aux, long ldaux, void* C, long ldc,
                      void* C2, long ldc2, hipStream_t st, const RopeP* rope) {
  if (M == 0 || N == 0) return VJ_OK;
  VJ_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 16 == 0 && lda % 16 == 0 && ldb % 16 == 0 && lda >= K && ldb >= K,
               "vj_gemm_fp8: K, lda, ldb must be multiples of 16 (M=%d N=%d K=%d lda=%ld ldb=%ld)", M, N, K, lda, ldb);
  VJ_CHECK_ARG(N % 8 == 0 && ldc % 4 == 0 && ldc2 % 4 == 0 && ldaux % 4 == 0, "vj_gemm_fp8: N %% 8, ld %% 4");
  VJ_CHECK_ARG(!(((uintptr_t)A | (uintptr_t)B | (uintptr_t)C | (uintptr_t)C2 | (uintptr_t)aux | (uintptr_t)bias) & 15),
               "vj_gemm_fp8: operands must be 16-B aligned");
  VJ_CHECK_ARG(A && B && ea && eb, "vj_gemm_fp8: null operand or scale exponents");
  VJ_CHECK_ARG(epi == EPI_BF16 || epi == EPI_F32 || epi == EPI_F32_RESID || epi == EPI_GELU || epi == EPI_ROPE,
               "vj_gemm_fp8: epilogue %d unsupported (forward only)", epi);
  VJ_CHECK_ARG(epi != EPI_F32_RESID || aux, "vj_gemm_fp8: EPI_F32_RESID needs the residual");
  VJ_CHECK_ARG(epi != EPI_GELU || C2, "vj_gemm_fp8: EPI_GELU needs the activation output C2");
  VJ_CHECK_ARG(epi == EPI_GELU || C, "vj_gemm_fp8: output C is required");
  VJ_CHECK_ARG((long)M * lda < 0x7fffffffL && (long)N * ldb < 0x7fffffffL, "vj_gemm_fp8: operand too large");
  // 256 x 128 tiles: the 256-wide fp8 tile needs ~20 VGPRs more than the bf16 one and spills
  const int bn = 128;
  const int tm = vj_cdiv(M, 256), tn = vj_cdiv(N, bn);
  G256 g{(const bf16_t*)A, (const bf16_t*)B, M, N, K / 2, lda / 2, ldb / 2, C, ldc, C2, ldc2, bias, aux, ldaux,
         tm, tn, RopeP{}, K / 2, 1, nullptr, tile_group(tm, tn), ea, eb};
  if (epi == EPI_ROPE) {
    VJ_CHECK_ARG(rope != nullptr, "vj_gemm_fp8: EPI_ROPE needs the rope tables");
    g.rope = *rope;
    VJ_CHECK_ARG(g.rope.hd % 4 == 0 && g.rope.D % 4 == 0 && g.rope.npos >= 1 && g.rope.npos <= 1024 &&
                     (long)g.rope.npos * g.rope.half <= ROPE_TAB_MAX,
                 "vj_gemm_fp8: rope table too large (npos=%d)", g.rope.npos);
  }
  return launch256_f8<128>(epi, g, st);
}

extern "C" int vj_gemm_fp8(int M, int N, int K, const void* A, long lda, const int* ea, const void* B, long ldb,
                           const int* eb, int epi, const float* bias, const void* aux, long ldaux, void* C, long ldc,
                           void* C2, long ldc2, void* stream) {
  VJ_CHECK_ARG(epi != EPI_ROPE, "vj_gemm_fp8: use vj_qkv_rope_gemm_fp8 for the RoPE epilogue");
  return gemm256_f8(M, N, K, A, lda, ea, B, ldb, eb, epi, bias, aux, ldaux, C, ldc, C2, ldc2, (hipStream_t)stream,
                    nullptr);
}

// vj_qkv_rope_gemm on fp8 operands (no unfused fallback: an fp8 request the kernel declines fails)
extern "C" int vj_qkv_rope_gemm_fp8(int M, int K, const void* A, long lda, const int* ea, const void* B, long ldb,
                                    const int* eb, const float* bias, void* C, long ldc, int H, int hd,
                                    const int* ids, int ids_mod, int tpf, int tpr, const float* cos_t,
                                    const float* sin_t, int npos, void* stream) {
  if (M == 0) return VJ_OK;
  VJ_CHECK_ARG(hd % 8 == 0 && cos_t && sin_t && (ids || ids_mod > 0), "vj_qkv_rope_gemm_fp8: bad rope arguments");
  VJ_CHECK_ARG(tpf > 0 && tpr > 0 && npos > 0, "vj_qkv_rope_gemm_fp8: tokens_per_frame/row and npos must be > 0");
  const RopeP rp{ids, ids_mod, tpf, tpr, (hd / 3) / 2, hd, H * hd, cos_t, sin_t, npos};
  return gemm256_f8(M, 3 * H * hd, K, A, lda, ea, B, ldb, eb, EPI_ROPE, bias, nullptr, 0, C, ldc, nullptr, 0,
                    (hipStream_t)stream, &rp);
}

#if VJ_GEMM_STAMPS
extern "C" int vj_debug_gemm_stamps(void* dst, long nbytes) {
  hipMemset(dst, 0, 0);
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(vj_gemm_stamps), nbytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
extern "C" int vj_debug_gemm_istamps(void* dst, long nbytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(vj_gemm_istamps), nbytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
extern "C" int vj_debug_gemm_stamps_clear() {
  static long z[2048 * 16 * 4];
  return hipMemcpyToSymbol(HIP_SYMBOL(vj_gemm_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : 1;
}
#endif
