// Varlen flash attention (non-causal, no dropout) for gfx950, forward + deterministic backward.
// Replaces F.scaled_dot_product_attention in RoPEAttention.forward (src/models/utils/modules.py:367-372)
// and Attention.forward (modules.py:411-418) for head_dim 64 (ViT-L / vit_giant_xformers encoders,
// SURVEY §8a A6), 32 (predictor, A9), 80 (vit_huge) and 88 (vit_giant). The head dim is padded to a
// multiple of 32 (HDP) in LDS and in the MFMA loops: the padding columns are zero-filled by the DMA
// range check / masked loads and never stored, so they add exact zeros.
//
// Layout: tokens of all sequences are concatenated ("ragged batch"): q/k/v rows live in one
// token-major bf16 buffer (the fused QKV GEMM output [T, 3*H*hd]), head h at column off + h*hd.
// Sequences are described by up to 4 groups of equal-length sequences (both JEPA mask passes of a
// step run as ONE launch). O is written token-major [T, H*hd] (= the proj GEMM's A operand).
//
// MFMA formulation (v_mfma_f32_32x32x16_bf16; accumulator: col = lane&31, row = (r&3)+8(r>>2)+4(lane>>5)):
//  forward, wave = 32 queries:  S^T = K Q^T (query on the lane -> softmax stats are per lane),
//                               O^T += V^T P^T, P^T taken straight from the S^T accumulator (k-permuted),
//                               V^T fragments by ds_read_b64_tr_b16.
//  dK/dV kernel, wave = 32 keys: S = Q K^T, dP = dO V^T (key on the lane), dV^T += dO^T P, dK^T += Q^T dS.
//  dQ kernel, wave = 32 queries: S^T = K Q^T, dP^T = V dO^T, dQ^T += K^T dS^T.
// No atomics: dQ and dK/dV come from separate sweeps, so the backward is bitwise reproducible.
// LDS images (one per tile, read both by rows and transposed): 16-B chunk index XOR-swizzled,
//   HD=64 (128-B rows): sw(r) = (((r>>1)&1)<<2) | ((r>>2)&3);  HD=32 (64-B rows): sw(r) = (r>>2)&3.
// Both keep ds_read_b128 row reads and ds_read_b64_tr_b16 transposed reads bank-conflict free.
#include <stdlib.h>
#include <type_traits>

#include "vj_common.h"

// Launch shapes fixed by the round-2/3 measurements (attention; the variants were removed
// from the source): 32-row key (dK/dV sweep) and query (dQ sweep) tiles per wave: 2 at head dim 32,
// 1 otherwise; forward at 3 workgroups per CU (head dims <= 64) with s_setprio 1 around the head-dim-64
// S and PV MFMA clusters; dQ sweep at 3 workgroups per CU for head dim 64. Measured slower and
// removed: a K / V^T fragment ring at 4 forward workgroups per CU (spills), the V-tile DMA under the
// softmax, priority around the backward MFMAs, the fused backward (dQ partials from the dK/dV sweep
// plus a reduce pass; 192.7 vs 196.9 clips/s) and a separate delta kernel.
#ifndef VJ_KW32
#define VJ_KW32 2
#endif
#ifndef VJ_QW32
#define VJ_QW32 2
#endif
constexpr int KW32 = VJ_KW32, QW32 = VJ_QW32, KW64 = 1, QW64 = 1;
// Forward occupancy hint (hd <= 64): the launch bound asks for 2 waves per SIMD, but the kernel compiles
// to 160 VGPRs (hd 64) / 94 (hd 32) and runs 3 / 5 per SIMD; with the bound at 3 the register allocator
// lands on 166 and a different schedule: target forward 425.7 -> 415.7 us, N = 8192 725 -> 717 us
// with this bound (profiles/r05_attn_fwd_occ_kernels.txt). Keep an eye on the VGPR count: above 168
// the hd-64 forward would drop to 2 waves per SIMD.
constexpr int FWD_OCC = 2;
constexpr int DQ64_OCC = 3;   // dQ sweep, head dim 64: 168 VGPRs (one dword reloaded per key tile)

namespace {

constexpr int MAXG = 4;
struct SeqGroups {
  int ngroups;
  int nseq[MAXG];
  int len[MAXG];
  int tok0[MAXG];
  int tiles_prefix[MAXG + 1];  // cumulative tile counts (tile size set by the kernel)
};

struct AttnArgs {
  const bf16_t* qkv;  // q, k, v (RoPE already applied to q, k)
  long ld;            // row stride of qkv (elements)
  int q_off, k_off, v_off;
  bf16_t* o;  // forward output / backward: dO input
  long ldo;
  const bf16_t* dout;  // backward: dO
  long lddo;
  float* stats;  // [2][H][T]: lse2 = log2(sum_k 2^(scale*log2e*s_k)), -delta = -rowsum(dO*O)
  bf16_t* dqkv;  // backward output, same layout as qkv
  long ldd;
  int H, T;
  float scale;  // softmax scale (head_dim^-0.5)
  SeqGroups sg;
  // backward: inverse 3-axis RoPE fused into the dq / dk stores (cos_t == NULL -> none)
  const int* rope_ids;
  int rope_mod, rope_tpf, rope_tpr, rope_half;
  const float* cos_t;
  const float* sin_t;
  // frame-causal (block-causal) mask: token i of a sequence attends to key j iff j / fblk <= i / fblk
  // (build_action_block_causal_attention_mask, modules.py:12-23, with fblk = cond tokens + H*W);
  // 0 = non-causal (every key of the sequence)
  int fblk;
  // dropout on the attention probabilities (F.scaled_dot_product_attention dropout_p, modules.py:246,
  // 370, 417): score (query token t, head h, key j of the sequence) is kept iff
  // drop_u(drop_row(drop_seed, t * H + h), j) >= drop_thresh, kept probabilities scaled by drop_scale
  uint32_t drop_thresh, drop_seed;
  float drop_scale;
};

// key limit of query qloc (keys [0, klim) are visible) and its block-uniform bounds
__device__ __forceinline__ int fc_klim(int fblk, int qloc, int len) {
  return fblk ? min(len, (qloc / fblk + 1) * fblk) : len;
}

// padded head dim of the LDS images and MFMA loops
template <int HD>
struct Hd {
  static constexpr int P = (HD + 31) / 32 * 32;
};

__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// Per-token RoPE positions (frame, row, col) for the inverse rotation (modules.py:293-324).
struct TokPos {
  int fr, hr, wc;
};
__device__ __forceinline__ TokPos tok_pos(const AttnArgs& a, int token) {
  const int id = a.rope_ids ? a.rope_ids[token] : (token % a.rope_mod);
  const int fr = id / a.rope_tpf;
  const int hr = (id - a.rope_tpf * fr) / a.rope_tpr;
  return TokPos{fr, hr, (id - a.rope_tpf * fr) - a.rope_tpr * hr};
}
// Transpose of rotate_queries_or_keys (modules.py:26-50) applied to the dq / dk rows a lane holds
// (pairs (d, d+1), d = d0*32 + acc_row(r), r even). The slice width and frequency count follow
// from HD (half = (HD/3)/2, checked at launch), so the index math is by constants; all table
// values are loaded before any is used so the loads overlap.
template <int HD>
__device__ __forceinline__ void rope_inv_rows(const AttnArgs& a, const TokPos& tp, int lane,
                                              f32x16 (&x)[Hd<HD>::P / 32]) {
  constexpr int half = (HD / 3) / 2, sw = 2 * half;
  constexpr int ND = Hd<HD>::P / 32;
  float c0[ND][8], s0[ND][8], c1[ND][8], s1[ND][8];
  const bool hi = lane >= 32;
  // table index of pair (d, d+1) for a compile-time d (after unrolling): folds to one position
  auto idx = [&](int d, int o) {
    if (d >= 3 * sw) return 0;  // inactive pairs read entry 0 and keep their values
    const int ax = d / sw, js = d - ax * sw;
    return (ax == 0 ? tp.fr : (ax == 1 ? tp.hr : tp.wc)) * half + (js + o) % half;
  };
#pragma unroll
  for (int d0 = 0; d0 < ND; ++d0)
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const int da = d0 * 32 + (r & 3) + 8 * (r >> 2);  // lanes 0-31; lanes 32-63 hold da + 4
      const int i0 = hi ? idx(da + 4, 0) : idx(da, 0), i1 = hi ? idx(da + 4, 1) : idx(da, 1);
      c0[d0][r / 2] = a.cos_t[i0];
      s0[d0][r / 2] = a.sin_t[i0];
      c1[d0][r / 2] = a.cos_t[i1];
      s1[d0][r / 2] = a.sin_t[i1];
    }
#pragma unroll
  for (int d0 = 0; d0 < ND; ++d0)
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      if (d0 * 32 + acc_row(r, lane) >= 3 * sw) continue;
      const float x0 = x[d0][r], x1 = x[d0][r + 1];
      x[d0][r] = x0 * c0[d0][r / 2] + x1 * s1[d0][r / 2];
      x[d0][r + 1] = -x0 * s0[d0][r / 2] + x1 * c1[d0][r / 2];
    }
}

// XCD-aware block order. The dispatcher sends linear block b (x fastest) to XCD b % 8; each XCD is
// handed a contiguous range of the (head, tile) space instead, so the query / key tiles of one
// (sequence, head) run on one XCD and re-read that sequence's K / V (forward, dQ) or Q / dO (dK/dV)
// from its L2. Measured before: every XCD fetched every sequence's K / V, ~3x the qkv bytes per
// launch from HBM (rocprofv3 FETCH_SIZE, profiles/r02_pmc_bench.txt).
__device__ __forceinline__ void xcd_tile(int& tile, int& head) {
  const int nx = gridDim.x;
  const int total = nx * gridDim.y;
  const int b = blockIdx.y * nx + blockIdx.x;
  const int per = total >> 3, rem = total & 7, x = b & 7;
  const int id = x * per + min(x, rem) + (b >> 3);
  head = id / nx;
  tile = id - head * nx;
}

// Locate (sequence start, length, tile index in sequence) of a flat tile id.
__device__ __forceinline__ void locate(const SeqGroups& sg, int tile, int tiles_per_seq_div, int& seq_start,
                                       int& len, int& t_in_seq, int* grp = nullptr, int* seq = nullptr) {
  int g = 0;
#pragma unroll
  for (int i = 1; i < MAXG; ++i)
    if (i < sg.ngroups && tile >= sg.tiles_prefix[i]) g = i;
  const int local = tile - sg.tiles_prefix[g];
  len = sg.len[g];
  const int tps = (len + tiles_per_seq_div - 1) / tiles_per_seq_div;
  const int s = local / tps;
  t_in_seq = local - s * tps;
  seq_start = sg.tok0[g] + s * len;
  if (grp) *grp = g;
  if (seq) *seq = s;
}

template <int HDP>
__device__ __forceinline__ int swz(int r) {
  if constexpr (HDP == 64) return (((r >> 1) & 1) << 2) | ((r >> 2) & 3);
  else return (r >> 2) & 3;  // 32 (64-B rows) and 96 (192-B rows): stays inside groups of 4 chunks
}
template <int HDP>
__device__ __forceinline__ int lds_off(int r, int chunk) {  // byte offset of 16-B chunk
  return r * (HDP * 2) + ((chunk ^ swz<HDP>(r)) * 16);
}

// Stage ROWS rows of HD bf16 starting at token row0 (< nvalid valid rows) into an LDS image of
// HDP-wide rows. Pieces of 1 KB (one wave-instruction, lane-linear in LDS); lane -> (row, physical
// chunk) from its byte offset; logical chunks >= HD/8 (head-dim padding) and invalid rows are
// zero-filled by the buffer range check.
template <int HD, int ROWS>
__device__ __forceinline__ void stage_rows(__amdgpu_buffer_rsrc_t rs, long ld, int row0, int nvalid,
                                           LDS_AS char* lds, int wave, int lane, int nwaves) {
  constexpr int HDP = Hd<HD>::P;
  constexpr int RB = HDP * 2;                  // bytes per LDS row
  constexpr int PIECES = ROWS * RB / 1024;
  static_assert(ROWS * RB % 1024 == 0, "tile must be whole 1-KB pieces");
#if VJ_DIAG_NODMA
  if (row0 >= 2 * ROWS) return;  // timing-only build (wrong results): tiles past the second not loaded
#endif
  // nwaves is 4 at every call site: pieces wave, wave + 4, ... (fully unrolled, wave is uniform)
#pragma unroll
  for (int i = 0; i < (PIECES + 3) / 4; ++i) {
    const int p = wave + 4 * i;
    if (PIECES % 4 != 0 && p >= PIECES) break;
    const int off = p * 1024 + lane * 16;
    const int r = off / RB;
    const int phys = (off - r * RB) >> 4;
    const int c = phys ^ swz<HDP>(r);
    uint32_t voff;
    if constexpr (HD == HDP) {
      // rows past the sequence end are out of the descriptor's range (every caller's descriptor
      // spans exactly nvalid rows) and zero-fill without a per-lane test: one lane-constant register
      // per piece (r * ld + c * 8) stays live across the sweep instead of offsets and masks
      (void)nvalid;
      voff = (uint32_t)(((long)(row0 + r) * ld + c * 8) * 2);
    } else {
      const bool ok = (row0 + r) < nvalid && c < HD / 8;
      voff = ok ? (uint32_t)(((long)(row0 + r) * ld + c * 8) * 2) : VJ_OOB;
    }
    dma16(rs, lds + p * 1024, voff);
  }
  (void)nwaves;
}

// A-operand row fragment (rows rb + lane&31, k-step s): 8 bf16 at chunk 2s + (lane>>5).
template <int HDP>
__device__ __forceinline__ bf16x8 row_frag(const LDS_AS char* lds, int rb, int s, int lane) {
  const int r = rb + (lane & 31);
  return *(const LDS_AS bf16x8*)(lds + lds_off<HDP>(r, 2 * s + (lane >> 5)));
}
// Transposed fragment: lane gets X[rows kb+8(j>>2)+4h+(j&3)][col cb + (lane&31)], j = 0..7
// (the k-permuted order of an accumulator used as an operand). Asm reads (ds_read_tr16_async):
// callers release them with lds_wait() + tie() before use, which lets the next tile's LDS-DMA be
// issued at the top of the iteration without the compiler serialising the reads behind it.
template <int HDP>
__device__ __forceinline__ bf16x8 tr_frag(const LDS_AS char* lds, int kb, int cb, int lane) {
  const int h = lane >> 5;
  const int q = (lane >> 2) & 3;
  const int col = cb + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  const int r0 = kb + 4 * h + q;
  const int r1 = r0 + 8;
  const int within = (col & 7) * 2;
  const s16x4 lo = ds_read_tr16_async(lds + lds_off<HDP>(r0, col >> 3) + within);
  const s16x4 hi = ds_read_tr16_async(lds + lds_off<HDP>(r1, col >> 3) + within);
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// tr_frag with the lane's addressing split off: for rows kb that are multiples of 16 the swizzle of
// row kb + x equals that of row x (it reads row bits 1-3 only), so the byte offset of a fragment is
// a per-lane part (tr_lane_off: column block d, half lo / hi) plus kb * row bytes, folded with the
// image's own LDS position into the instruction's immediate. A sweep then holds 2 * HDP / 32
// address registers instead of one per (k-step, column block, half).
template <int HDP>
__device__ __forceinline__ uint32_t tr_lane_off(int d, int half, int lane) {
  const int h = lane >> 5;
  const int q = (lane >> 2) & 3;
  const int col = d * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  const int r = 4 * h + q + 8 * half;
  return (uint32_t)(lds_off<HDP>(r, col >> 3) + (col & 7) * 2);
}
template <int IMM>
__device__ __forceinline__ s16x4 ds_read_tr16_imm(uint32_t addr) {
  static_assert(IMM >= 0 && IMM < 65536, "ds offset field");
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(IMM) : "memory");
  return r;
}
// fragment (rows KB.., column block d) of the image at LDS byte IMG; lo / hi = tr_lane_off(d, 0 / 1)
// + the LDS base address
template <int HDP, int IMG, int KB>
__device__ __forceinline__ bf16x8 tr_frag_at(uint32_t lo, uint32_t hi) {
  static_assert(KB % 16 == 0, "row block must keep the swizzle phase");
  const s16x4 a = ds_read_tr16_imm<IMG + KB * HDP * 2>(lo);
  const s16x4 b = ds_read_tr16_imm<IMG + KB * HDP * 2>(hi);
  s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Accumulator registers 8s..8s+7 -> bf16 operand fragment.
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& a, int s) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (__bf16)a[8 * s + j];
  return v;
}

__device__ __forceinline__ bf16x8 gload8(const bf16_t* p, bool ok) {
  if (!ok) {
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (__bf16)0.f;
    return z;
  }
  return *(const bf16x8*)p;
}


constexpr float LOG2E = 1.4426950408889634f;

// A wave's 32 x HD output tile (O, dQ, dK or dV) held as accumulators x[d] (token = lane & 31, head
// dim d*32 + acc_row(r, lane)), stored through LDS as whole rows: the lane's 4 consecutive dims
// (accumulator rows 4j..4j+3) go to a wave-private LDS image (16-B chunks XOR-swizzled by row), read
// back as 16-B row chunks and stored 64 / (HD/8) rows per instruction. Replaces 4-B stores at a row
// stride, where every store instruction touched 32-64 cache lines.
template <int HD>
struct OutTile {
  static constexpr int NCH = HD / 8;  // 16-B chunks stored per row
  static constexpr int CH = Hd<HD>::P / 8 <= 4 ? 4 : (Hd<HD>::P / 8 <= 8 ? 8 : 16);  // per LDS row
  static constexpr int SWM = CH < 8 ? CH - 1 : 7;
  static constexpr int BYTES = 32 * CH * 16;  // one wave's image
};
template <int HD>
__device__ __forceinline__ void wave_store_rows(const f32x16 (&x)[Hd<HD>::P / 32], float scale, LDS_AS char* buf,
                                                bf16_t* out, long ld, int nvalid, int lane) {
  using OT = OutTile<HD>;
  const int r = lane & 31, hl = lane >> 5;
#pragma unroll
  for (int d = 0; d < Hd<HD>::P / 32; ++d)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (d * 32 + 8 * j >= HD) continue;  // head-dim padding (HD is a multiple of 8: wave-uniform)
      const int c = d * 4 + j;
      typedef int i32x2 __attribute__((ext_vector_type(2)));
      i32x2 v;
      v[0] = (int)pack_bf2(x[d][4 * j] * scale, x[d][4 * j + 1] * scale);
      v[1] = (int)pack_bf2(x[d][4 * j + 2] * scale, x[d][4 * j + 3] * scale);
      *(LDS_AS i32x2*)(buf + r * (OT::CH * 16) + ((c ^ (r & OT::SWM)) * 16) + hl * 8) = v;
    }
#pragma unroll
  for (int i0 = 0; i0 < 32 * OT::NCH; i0 += 64) {
    const int i = i0 + lane;
    const int row = i / OT::NCH, c = i - row * OT::NCH;
    if ((32 * OT::NCH) % 64 == 0 || i < 32 * OT::NCH) {
      const i32x4 v = *(const LDS_AS i32x4*)(buf + row * (OT::CH * 16) + ((c ^ (row & OT::SWM)) * 16));
      if (row < nvalid) *(i32x4*)(out + (long)row * ld + c * 8) = v;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Forward: block = 4 waves x 32 queries, KV tiles of 64 keys double-buffered in LDS.
template <int HD, bool DROP>
__global__ __launch_bounds__(256, (HD <= 64 ? FWD_OCC : 2)) void k_attn_fwd(AttnArgs a) {
  constexpr int HDP = Hd<HD>::P;
  constexpr int KT = 64;
  constexpr int TB = KT * HDP * 2;  // bytes per K or V tile
  __shared__ __attribute__((aligned(16))) char smem_raw[4 * TB];
  LDS_AS char* smem = (LDS_AS char*)smem_raw;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int tile_id, h;
  xcd_tile(tile_id, h);
  int seq0, len, qt;
  locate(a.sg, tile_id, 128, seq0, len, qt);
  const int qloc = qt * 128 + wave * 32 + (lane & 31);
  const bool qok = qloc < len;
  const int hl = lane >> 5;
  // frame-causal: this lane's key limit; the block's keys end at its last query's limit, and tiles
  // past its first query's limit take the per-lane mask (both = len when non-causal)
  const int klim = fc_klim(a.fblk, qloc, len);
  const int kend = fc_klim(a.fblk, min(qt * 128 + 127, len - 1), len);
  const int kmask0 = fc_klim(a.fblk, qt * 128, len);
  [[maybe_unused]] const uint32_t drow = DROP ? drop_row(a.drop_seed, (uint32_t)((seq0 + qloc) * a.H + h)) : 0u;

  // Q^T fragments (B operand of S^T = K Q^T): lane holds Q[q][16s + 8h + j] (zero past HD).
  bf16x8 qf[HDP / 16];
  const bf16_t* qrow = a.qkv + (long)(seq0 + qloc) * a.ld + a.q_off + h * HD;
#pragma unroll
  for (int s = 0; s < HDP / 16; ++s) qf[s] = gload8(qrow + 16 * s + 8 * hl, qok && 16 * s + 8 * hl < HD);

  const bf16_t* kbase = a.qkv + (long)seq0 * a.ld + a.k_off + h * HD;
  const bf16_t* vbase = a.qkv + (long)seq0 * a.ld + a.v_off + h * HD;
  const uint32_t bytes = (uint32_t)min((long)len * a.ld * 2, 0x7fffffffL);
  const __amdgpu_buffer_rsrc_t rk = make_rsrc(kbase, bytes);
  const __amdgpu_buffer_rsrc_t rv = make_rsrc(vbase, bytes);

  // O^T accumulators; lsum = this lane's share of l = sum_k p (its 16 key rows of each 32-key
  // half; lanes q and q + 32 together hold query q's keys), summed on the VALU in f32
  f32x16 ot[HDP / 32];
  float lsum = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r)
#pragma unroll
    for (int d = 0; d < HDP / 32; ++d) ot[d][r] = 0.f;
  // Lazy rescaling: p = exp2(c*s - c*m_use) with m_use the raw-score max seen when O was last
  // rescaled (the deferred-max rule below); the result is invariant to m_use.
  float m_use = -INFINITY, cm = 0.f;
  const float c = a.scale * LOG2E;

  // per-lane V^T read addresses (tr_frag_at): LDS base + lane part, d = column block
  uint32_t vlo[HDP / 32], vhi[HDP / 32];
#pragma unroll
  for (int d = 0; d < HDP / 32; ++d) {
    vlo[d] = (uint32_t)(uintptr_t)smem + tr_lane_off<HDP>(d, 0, lane);
    vhi[d] = (uint32_t)(uintptr_t)smem + tr_lane_off<HDP>(d, 1, lane);
  }
  const int nkt = (kend + KT - 1) / KT;
  stage_rows<HD, KT>(rk, a.ld, 0, len, smem, wave, lane, 4);
  stage_rows<HD, KT>(rv, a.ld, 0, len, smem + TB, wave, lane, 4);
  __syncthreads();
  // head dim 64: s_setprio 1 around the S and PV MFMA clusters, so a wave's MFMA chain keeps the
  // issue arbitration over the other waves' softmax VALU (-2.3 % target, r03_attn_prio_kernels.txt)
  constexpr bool PRIO_S = HD == 64;
  constexpr bool PRIO_PV = HD == 64;
  // loop body with the LDS buffer index as a compile-time constant (unrolled by 2), so every LDS
  // address is a per-lane base register plus an immediate offset
  // S^T = K Q^T of the tile's two 32-key halves (kf: the K fragments, all read before the MFMAs)
  auto s_tile = [&](const LDS_AS char* Ks, f32x16 (&st)[2]) {
    bf16x8 kf[2][HDP / 16];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int s = 0; s < HDP / 16; ++s) kf[kk][s] = row_frag<HDP>(Ks, kk * 32, s, lane);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int r = 0; r < 16; ++r) st[kk][r] = 0.f;
    if (PRIO_S) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < HDP / 16; ++s)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        st[kk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kk][s], qf[s], st[kk], 0, 0, 0);
    if (PRIO_S) __builtin_amdgcn_s_setprio(0);
  };
  // keys past the limit get -inf (ragged last tile, frame-causal boundary tiles)
  auto mask_tile = [&](const int kb, f32x16 (&st)[2]) {
    if (kb + KT > kmask0) {
      asm volatile("");  // keeps the compiler from if-converting this into every tile
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kb + kk * 32 + acc_row(r, lane) >= klim) st[kk][r] = -INFINITY;
    }
  };
  // m_use := the running row max (exact), O and l rescaled to it
  auto to_row_max = [&](const f32x16 (&st)[2]) {
    float mx = st[0][0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, st[0][r]);
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[1][r]);
    mx = max_xor32(mx);
    const float m_new = fmaxf(m_use, mx);
    const float alpha = __builtin_amdgcn_exp2f((m_use - m_new) * c);
    m_use = m_new;
    cm = m_new * c;
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int d = 0; d < HDP / 32; ++d) ot[d][r] *= alpha;
    lsum *= alpha;
  };
  // p = 2^(c s - c m_use) in place; returns this lane's sum of its 32 p (two partial chains)
  auto exp_tile = [&](f32x16 (&st)[2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int r = 0; r < 16; ++r) st[kk][r] = __builtin_amdgcn_exp2f(fmaf(st[kk][r], c, -cm));
    float ls0 = st[0][0], ls1 = st[1][0];
#pragma unroll
    for (int r = 1; r < 16; ++r) {
      ls0 += st[0][r];
      ls1 += st[1][r];
    }
    return ls0 + ls1;
  };
  // Deferred max (round 5): after the first tile the exponentials are taken against the running m_use
  // without the tile's row max (24 of ~140 VALU per tile); the lane's p sum bounds every p, so while
  // no lane's sum exceeds PLIM every p <= PLIM (range-safe in f32 / bf16, and the result does not
  // depend on m_use). A lane over the bound (a max that grew, an overflow, a NaN) sends the wave down
  // the exact path: S recomputed from the K tile (still in LDS) and Q, row max, rescale, exponentials.
  constexpr float PLIM = 4096.f;
  // loop body with the LDS buffer index as a compile-time constant (unrolled by 2), so every LDS
  // address is a per-lane base register plus an immediate offset
  auto tile_iter = [&](const int kt, auto cur_c, auto first_c) {
    constexpr int cur = decltype(cur_c)::value;
    constexpr bool FIRST = decltype(first_c)::value;
    const LDS_AS char* Ks = smem + cur * 2 * TB;
    if (kt + 1 < nkt) {  // next tile's DMA: lands during this whole iteration
      LDS_AS char* nx = smem + (cur ^ 1) * 2 * TB;
      stage_rows<HD, KT>(rk, a.ld, (kt + 1) * KT, len, nx, wave, lane, 4);
      stage_rows<HD, KT>(rv, a.ld, (kt + 1) * KT, len, nx + TB, wave, lane, 4);
    }
    f32x16 st[2];
    s_tile(Ks, st);
    // V^T fragments: issued before the softmax so their LDS latency hides under it (per-lane base
    // registers + immediates: the buffer and the k-step are compile-time)
    constexpr int VIMG = cur * 2 * TB + TB;
    bf16x8 vf[4][HDP / 32];
#pragma unroll
    for (int d = 0; d < HDP / 32; ++d) {
      vf[0][d] = tr_frag_at<HDP, VIMG, 0>(vlo[d], vhi[d]);
      vf[1][d] = tr_frag_at<HDP, VIMG, 16>(vlo[d], vhi[d]);
      vf[2][d] = tr_frag_at<HDP, VIMG, 32>(vlo[d], vhi[d]);
      vf[3][d] = tr_frag_at<HDP, VIMG, 48>(vlo[d], vhi[d]);
    }
    const int kb = kt * KT;
    mask_tile(kb, st);
    if constexpr (FIRST) to_row_max(st);
    float ls = exp_tile(st);
    if constexpr (!FIRST) {
      if (__builtin_amdgcn_ballot_w64(!(ls <= PLIM))) {
        asm volatile("");  // a real (rare) branch, not if-converted into every tile
        lds_wait();        // the V reads in flight complete first (LDS returns in order)
        s_tile(Ks, st);
        mask_tile(kb, st);
        to_row_max(st);
        ls = exp_tile(st);
      }
    }
    lsum += ls;
    if constexpr (DROP) {  // l sums every p; the PV product takes the kept ones (x drop_scale at the end)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (drop_u(drow, (uint32_t)(kb + kk * 32 + acc_row(r, lane))) < a.drop_thresh) st[kk][r] = 0.f;
    }
    // O^T += V^T P^T over 4 key-steps of 16
    lds_wait();
    {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) tie(vf[ks]);
      if (PRIO_PV) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 pf = acc_frag(st[ks >> 1], ks & 1);
#pragma unroll
        for (int d = 0; d < HDP / 32; ++d) ot[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[ks][d], pf, ot[d], 0, 0, 0);
      }
      if (PRIO_PV) __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  tile_iter(0, I0{}, std::true_type{});
  for (int kt0 = 1; kt0 < nkt; kt0 += 2) {
    tile_iter(kt0, I1{}, std::false_type{});
    if (kt0 + 1 < nkt) tile_iter(kt0 + 1, I0{}, std::false_type{});
  }
  const float l_tot = sum_xor32(lsum);
  const float inv = DROP ? a.drop_scale / l_tot : 1.f / l_tot;
  if constexpr (HD == 32) {
    // head dim 32 (5 workgroups per CU): the direct 4-B stores measured faster than the LDS image
    // (predictor forward 269 vs 278 us, profiles/r05_attn_row_stores_ab.txt)
    if (qok) {
      bf16_t* orow = a.o + (long)(seq0 + qloc) * a.ldo + h * HD;
#pragma unroll
      for (int r = 0; r < 16; r += 2) *(uint32_t*)(orow + acc_row(r, lane)) = pack_bf2(ot[0][r] * inv, ot[0][r + 1] * inv);
    }
  } else {
    // the K / V buffers are free after the last tile's barrier
    static_assert(4 * OutTile<HD>::BYTES <= 4 * TB, "output images fit the K / V buffers");
    const int q0 = qt * 128 + wave * 32;
    wave_store_rows<HD>(ot, inv, smem + wave * OutTile<HD>::BYTES, a.o + (long)(seq0 + q0) * a.ldo + h * HD, a.ldo,
                        len - q0, lane);
  }
  if (qok && hl == 0) a.stats[(long)h * a.T + seq0 + qloc] = m_use * c + __log2f(l_tot);  // log2 units
}

// ------------------------------------------------------------------------------------------------
// dK/dV: block = 4 waves x (32 KW) keys; sweep query tiles of 32 (Q, dO, lse, delta staged in LDS).
// Each wave owns KW 32-key tiles (key tile kw of wave w: keys kw*128 + w*32 + 0..31 of the block),
// so every staged Q / dO fragment feeds KW independent MFMA chains per barrier.
template <int HD, int KW, bool DROP>
__global__ __launch_bounds__(256) void k_attn_bwd_dkdv(AttnArgs a) {
  constexpr int HDP = Hd<HD>::P;
  constexpr int QT = 32;
  constexpr int TB = QT * HDP * 2;
  // per stage: Q tile, dO tile, 32 lse + 32 delta floats
  constexpr int STAGE = 2 * TB + 256;
  constexpr int SMEM = 2 * STAGE > 4 * OutTile<HD>::BYTES ? 2 * STAGE : 4 * OutTile<HD>::BYTES;
  __shared__ __attribute__((aligned(16))) char smem_raw[SMEM];
  LDS_AS char* smem = (LDS_AS char*)smem_raw;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int tile_id, h;
  xcd_tile(tile_id, h);
  int seq0, len, kt;
  locate(a.sg, tile_id, 128 * KW, seq0, len, kt);
  int kloc[KW];
  bool kok[KW];
#pragma unroll
  for (int kw = 0; kw < KW; ++kw) {
    kloc[kw] = kt * 128 * KW + kw * 128 + wave * 32 + (lane & 31);
    kok[kw] = kloc[kw] < len;
  }
  const int hl = lane >> 5;

  // K^T and V^T fragments (B operands): lane holds K[key][16s + 8h + j].
  bf16x8 kf[KW][HDP / 16], vf[KW][HDP / 16];
#pragma unroll
  for (int kw = 0; kw < KW; ++kw) {
    const bf16_t* krow = a.qkv + (long)(seq0 + kloc[kw]) * a.ld + a.k_off + h * HD;
    const bf16_t* vrow = a.qkv + (long)(seq0 + kloc[kw]) * a.ld + a.v_off + h * HD;
#pragma unroll
    for (int s = 0; s < HDP / 16; ++s) {
      kf[kw][s] = gload8(krow + 16 * s + 8 * hl, kok[kw] && 16 * s + 8 * hl < HD);
      vf[kw][s] = gload8(vrow + 16 * s + 8 * hl, kok[kw] && 16 * s + 8 * hl < HD);
    }
  }
  const uint32_t qbytes = (uint32_t)min((long)len * a.ld * 2, 0x7fffffffL);
  const uint32_t dbytes = (uint32_t)min((long)len * a.lddo * 2, 0x7fffffffL);
  const __amdgpu_buffer_rsrc_t rq = make_rsrc(a.qkv + (long)seq0 * a.ld + a.q_off + h * HD, qbytes);
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(a.dout + (long)seq0 * a.lddo + h * HD, dbytes);
  // stats: lse at [h][seq0 + i], delta at [H*T + h*T + seq0 + i]
  const __amdgpu_buffer_rsrc_t rs =
      make_rsrc(a.stats + (long)h * a.T + seq0, (uint32_t)min(((long)a.H * a.T + len) * 4, 0x7fffffffL));
  const long dstat = (long)a.H * a.T;  // element distance lse -> delta
  f32x16 dvt[KW][HDP / 32], dkt[KW][HDP / 32];
#pragma unroll
  for (int kw = 0; kw < KW; ++kw)
#pragma unroll
    for (int d = 0; d < HDP / 32; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) dvt[kw][d][r] = dkt[kw][d][r] = 0.f;
  const float c = a.scale * LOG2E;
  const float rc = -1.f / c;

  auto stage = [&](int qt, LDS_AS char* st) {
    stage_rows<HD, QT>(rq, a.ld, qt * QT, len, st, wave, lane, 4);
    stage_rows<HD, QT>(rd, a.lddo, qt * QT, len, st + TB, wave, lane, 4);
    if (wave == 3) {  // 64 lanes x 4 B: lanes 0-31 lse, 32-63 delta
      const int i = qt * QT + (lane & 31);
      const uint32_t voff = (i < len) ? (uint32_t)((i + (lane >= 32 ? dstat : 0)) * 4) : VJ_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, st + 2 * TB, 4, voff, 0, 0, 0);
    }
  };

  // per-lane transposed-read addresses (tr_frag_at) of the Q / dO images
  uint32_t tlo[HDP / 32], thi[HDP / 32];
#pragma unroll
  for (int d = 0; d < HDP / 32; ++d) {
    tlo[d] = (uint32_t)(uintptr_t)smem + tr_lane_off<HDP>(d, 0, lane);
    thi[d] = (uint32_t)(uintptr_t)smem + tr_lane_off<HDP>(d, 1, lane);
  }
  const int nqt = (len + QT - 1) / QT;
  // frame-causal: key k is seen by queries from its frame block's start on; the sweep starts at the
  // block's first key's frame start, and query tiles before its last key's frame start take the mask
  int qlo[KW];
#pragma unroll
  for (int kw = 0; kw < KW; ++kw) qlo[kw] = a.fblk ? (min(kloc[kw], len - 1) / a.fblk) * a.fblk : 0;
  const int kfirst = kt * 128 * KW, klast = min(kfirst + 128 * KW - 1, len - 1);
  const int qt_first = a.fblk ? ((kfirst / a.fblk) * a.fblk) / QT : 0;
  const int qmask_end = a.fblk ? (klast / a.fblk) * a.fblk : 0;  // tiles starting below this are masked
  stage(qt_first, smem);
  __syncthreads();
  // Rows of queries past the sequence end are zero (DMA range check) with lse2 = delta = 0, so they
  // add exactly 0 to dV and dK; columns of keys past the end are never stored. No masks needed.
  // loop body with the LDS buffer index as a compile-time constant (unrolled by 2), so every LDS
  // address is a per-lane base register plus an immediate offset
  auto tile_iter = [&](const int qt, auto cur_c) {
    constexpr int cur = decltype(cur_c)::value;
    if (qt + 1 < nqt) stage(qt + 1, smem + (cur ^ 1) * STAGE);
    const LDS_AS char* Qs = smem + cur * STAGE;
    const LDS_AS char* Ds = Qs + TB;
    const LDS_AS float* Ls = (const LDS_AS float*)(Qs + 2 * TB);
    bf16x8 qa[HDP / 16], da[HDP / 16];
#pragma unroll
    for (int s = 0; s < HDP / 16; ++s) {
      qa[s] = row_frag<HDP>(Qs, 0, s, lane);
      da[s] = row_frag<HDP>(Ds, 0, s, lane);
    }
    // S - lse2/c = Q K^T - lse2/c (rows: queries, col: key); dP - delta = dO V^T - delta: the
    // per-query terms are the accumulators' initial values, so no per-row registers stay live
    f32x16 sacc[KW], dp[KW];
    [[maybe_unused]] float dlr[DROP ? 16 : 1];  // dropout: -delta per query row (dS = p (z dP - delta))
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qi = acc_row(r, lane);
      const float l2 = Ls[qi] * rc, dl = Ls[32 + qi];
      if constexpr (DROP) dlr[r] = dl;
#pragma unroll
      for (int kw = 0; kw < KW; ++kw) {
        sacc[kw][r] = l2;
        dp[kw][r] = DROP ? 0.f : dl;
      }
    }
#pragma unroll
    for (int s = 0; s < HDP / 16; ++s)
#pragma unroll
      for (int kw = 0; kw < KW; ++kw) {
        sacc[kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa[s], kf[kw][s], sacc[kw], 0, 0, 0);
        dp[kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da[s], vf[kw][s], dp[kw], 0, 0, 0);
      }
    bf16x8 dtf[2][HDP / 32], qtf[2][HDP / 32];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int d = 0; d < HDP / 32; ++d) {
        dtf[s2][d] = s2 ? tr_frag_at<HDP, cur * STAGE + TB, 16>(tlo[d], thi[d])
                        : tr_frag_at<HDP, cur * STAGE + TB, 0>(tlo[d], thi[d]);
        qtf[s2][d] = s2 ? tr_frag_at<HDP, cur * STAGE, 16>(tlo[d], thi[d])
                        : tr_frag_at<HDP, cur * STAGE, 0>(tlo[d], thi[d]);
      }
    if (qt * QT < qmask_end) {  // frame-causal: queries of earlier frames than the key see nothing
      asm volatile("");
#pragma unroll
      for (int kw = 0; kw < KW; ++kw)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (qt * QT + acc_row(r, lane) < qlo[kw]) sacc[kw][r] = -INFINITY;
    }
    // P = 2^(c*S - lse2); dS = P * (dP - delta). Dropout (z = drop_scale or 0): dV takes P z, and
    // dS = P (z dP - delta), dP = dO V^T being the gradient of the dropped probabilities
    if constexpr (DROP) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint32_t rk = drop_row(a.drop_seed, (uint32_t)((seq0 + qt * QT + acc_row(r, lane)) * a.H + h));
#pragma unroll
        for (int kw = 0; kw < KW; ++kw) {
          const float p = __builtin_amdgcn_exp2f(sacc[kw][r] * c);
          const float z = drop_u(rk, (uint32_t)kloc[kw]) >= a.drop_thresh ? a.drop_scale : 0.f;
          dp[kw][r] = p * fmaf(z, dp[kw][r], dlr[r]);
          sacc[kw][r] = p * z;
        }
      }
    } else {
#pragma unroll
      for (int kw = 0; kw < KW; ++kw)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(sacc[kw][r] * c);
          sacc[kw][r] = p;
          dp[kw][r] *= p;
        }
    }
    // dV^T += dO^T P ; dK^T += Q^T dS   (k-permuted accumulators as B operands)
    lds_wait();
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      tie(dtf[s2]);
      tie(qtf[s2]);
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int kw = 0; kw < KW; ++kw) {
        const bf16x8 pf = acc_frag(sacc[kw], s2);
        const bf16x8 sf = acc_frag(dp[kw], s2);
#pragma unroll
        for (int d = 0; d < HDP / 32; ++d) {
          dvt[kw][d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(dtf[s2][d], pf, dvt[kw][d], 0, 0, 0);
          dkt[kw][d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qtf[s2][d], sf, dkt[kw][d], 0, 0, 0);
        }
      }
    __syncthreads();
  };
  for (int qt0 = qt_first; qt0 < nqt; qt0 += 2) {
    tile_iter(qt0, std::integral_constant<int, 0>{});
    if (qt0 + 1 < nqt) tile_iter(qt0 + 1, std::integral_constant<int, 1>{});
  }
  // the Q / dO buffers are free after the last tile's barrier: rows go out through a wave-private image
  LDS_AS char* ob = smem + wave * OutTile<HD>::BYTES;
#pragma unroll
  for (int kw = 0; kw < KW; ++kw) {
    const int k0 = kt * 128 * KW + kw * 128 + wave * 32;
    if (k0 >= len) continue;  // wave-uniform
    const bool rope = a.cos_t != nullptr;
    const TokPos tp = rope ? tok_pos(a, seq0 + min(kloc[kw], len - 1)) : TokPos{0, 0, 0};
    // rotate everything before the first store (the stores could alias the tables, so the
    // table loads would otherwise be serialised behind them)
#pragma unroll
    for (int d = 0; d < HDP / 32; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) dkt[kw][d][r] *= a.scale;
    if (rope) rope_inv_rows<HD>(a, tp, lane, dkt[kw]);
    const long row0 = (long)(seq0 + k0) * a.ldd + h * HD;
    wave_store_rows<HD>(dkt[kw], 1.f, ob, a.dqkv + row0 + a.k_off, a.ldd, len - k0, lane);
    wave_store_rows<HD>(dvt[kw], 1.f, ob, a.dqkv + row0 + a.v_off, a.ldd, len - k0, lane);
  }
}

// ------------------------------------------------------------------------------------------------
// dQ: block = 4 waves x (32 QW) queries; sweep key tiles of 64 (K, V staged in LDS). Each wave owns
// QW 32-query tiles (tile qw of wave w: queries qw*128 + w*32 + 0..31 of the block), so every K / V
// fragment read from LDS feeds QW independent MFMA chains.
// It runs first and computes delta = rowsum(dO * O) itself (from its dO fragments and O), writing
// -delta to stats for the dK/dV sweep.
template <int HD, int QW, bool DROP>
__global__ __launch_bounds__(256, (HD == 64 ? DQ64_OCC : 1)) void k_attn_bwd_dq(AttnArgs a) {
  constexpr int HDP = Hd<HD>::P;
  constexpr int KT = 64;
  constexpr int TB = KT * HDP * 2;
  __shared__ __attribute__((aligned(16))) char smem_raw[4 * TB];
  LDS_AS char* smem = (LDS_AS char*)smem_raw;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int tile_id, h;
  xcd_tile(tile_id, h);
  int seq0, len, qt;
  locate(a.sg, tile_id, 128 * QW, seq0, len, qt);
  const int hl = lane >> 5;
  int qloc[QW];
  bool qok[QW];
  bf16x8 qf[QW][HDP / 16], gf[QW][HDP / 16];
  float lse2[QW], dl[QW];
#pragma unroll
  for (int qw = 0; qw < QW; ++qw) {
    qloc[qw] = qt * 128 * QW + qw * 128 + wave * 32 + (lane & 31);
    qok[qw] = qloc[qw] < len;
    const bf16_t* qrow = a.qkv + (long)(seq0 + qloc[qw]) * a.ld + a.q_off + h * HD;
    const bf16_t* grow = a.dout + (long)(seq0 + qloc[qw]) * a.lddo + h * HD;
#pragma unroll
    for (int s = 0; s < HDP / 16; ++s) {
      qf[qw][s] = gload8(qrow + 16 * s + 8 * hl, qok[qw] && 16 * s + 8 * hl < HD);
      gf[qw][s] = gload8(grow + 16 * s + 8 * hl, qok[qw] && 16 * s + 8 * hl < HD);
    }
    lse2[qw] = qok[qw] ? a.stats[(long)h * a.T + seq0 + qloc[qw]] : 0.f;
    {  // -delta = -sum_d dO * O: lanes q and q + 32 hold the two halves of each 16-dim step
      const bf16_t* orow = a.o + (long)(seq0 + qloc[qw]) * a.ldo + h * HD;
      float sd = 0.f;
#pragma unroll
      for (int s = 0; s < HDP / 16; ++s) {
        const bf16x8 ov = gload8(orow + 16 * s + 8 * hl, qok[qw] && 16 * s + 8 * hl < HD);
#pragma unroll
        for (int j = 0; j < 8; ++j) sd = fmaf((float)gf[qw][s][j], (float)ov[j], sd);
      }
      sd = sum_xor32(sd);
      dl[qw] = qok[qw] ? -sd : 0.f;
      if (qok[qw] && hl == 0) a.stats[(long)a.H * a.T + (long)h * a.T + seq0 + qloc[qw]] = -sd;
    }
  }

  const uint32_t bytes = (uint32_t)min((long)len * a.ld * 2, 0x7fffffffL);
  const __amdgpu_buffer_rsrc_t rk = make_rsrc(a.qkv + (long)seq0 * a.ld + a.k_off + h * HD, bytes);
  const __amdgpu_buffer_rsrc_t rv = make_rsrc(a.qkv + (long)seq0 * a.ld + a.v_off + h * HD, bytes);

  f32x16 dqt[QW][HDP / 32];
#pragma unroll
  for (int qw = 0; qw < QW; ++qw)
#pragma unroll
    for (int d = 0; d < HDP / 32; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) dqt[qw][d][r] = 0.f;
  const float c = a.scale * LOG2E;
  [[maybe_unused]] uint32_t drow[QW];
#pragma unroll
  for (int qw = 0; qw < QW; ++qw) drow[qw] = DROP ? drop_row(a.drop_seed, (uint32_t)((seq0 + qloc[qw]) * a.H + h)) : 0u;
  float nl2[QW];  // -lse2 / c: initial value of the S^T accumulators, so p = 2^(c * acc)
#pragma unroll
  for (int qw = 0; qw < QW; ++qw) nl2[qw] = -lse2[qw] / c;
  // frame-causal key limits (as in the forward)
  int klim[QW];
#pragma unroll
  for (int qw = 0; qw < QW; ++qw) klim[qw] = fc_klim(a.fblk, qloc[qw], len);
  const int q_first = qt * 128 * QW;
  const int kend = fc_klim(a.fblk, min(q_first + 128 * QW - 1, len - 1), len);
  const int kmask0 = fc_klim(a.fblk, q_first, len);

  // per-lane transposed-read addresses (tr_frag_at) of the K images
  uint32_t klo[HDP / 32], khi[HDP / 32];
#pragma unroll
  for (int d = 0; d < HDP / 32; ++d) {
    klo[d] = (uint32_t)(uintptr_t)smem + tr_lane_off<HDP>(d, 0, lane);
    khi[d] = (uint32_t)(uintptr_t)smem + tr_lane_off<HDP>(d, 1, lane);
  }
  const int nkt = (kend + KT - 1) / KT;
  stage_rows<HD, KT>(rk, a.ld, 0, len, smem, wave, lane, 4);
  stage_rows<HD, KT>(rv, a.ld, 0, len, smem + TB, wave, lane, 4);
  __syncthreads();
  // loop body with the LDS buffer index as a compile-time constant (unrolled by 2), so every LDS
  // address is a per-lane base register plus an immediate offset
  auto tile_iter = [&](const int kt, auto cur_c) {
    constexpr int cur = decltype(cur_c)::value;
    const LDS_AS char* Ks = smem + cur * 2 * TB;
    const LDS_AS char* Vs = Ks + TB;
    if (kt + 1 < nkt) {  // next tile's DMA: lands during this whole iteration
      LDS_AS char* nx = smem + (cur ^ 1) * 2 * TB;
      stage_rows<HD, KT>(rk, a.ld, (kt + 1) * KT, len, nx, wave, lane, 4);
      stage_rows<HD, KT>(rv, a.ld, (kt + 1) * KT, len, nx + TB, wave, lane, 4);
    }
    const bool ragged = (kt + 1) * KT > kmask0;
    // Per 32-key half kk: S^T = K Q^T and dP^T - delta = V dO^T - delta for the QW query tiles, then
    // dQ^T += K^T dS^T. Halves run one after the other so only one half's fragments are live.
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 ka[HDP / 16], va[HDP / 16], ktf[2][HDP / 32];
#pragma unroll
      for (int s = 0; s < HDP / 16; ++s) {
        ka[s] = row_frag<HDP>(Ks, kk * 32, s, lane);
        va[s] = row_frag<HDP>(Vs, kk * 32, s, lane);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int d = 0; d < HDP / 32; ++d)
          ktf[s2][d] = (kk * 2 + s2 == 0)   ? tr_frag_at<HDP, cur * 2 * TB, 0>(klo[d], khi[d])
                       : (kk * 2 + s2 == 1) ? tr_frag_at<HDP, cur * 2 * TB, 16>(klo[d], khi[d])
                       : (kk * 2 + s2 == 2) ? tr_frag_at<HDP, cur * 2 * TB, 32>(klo[d], khi[d])
                                            : tr_frag_at<HDP, cur * 2 * TB, 48>(klo[d], khi[d]);
      f32x16 st[QW], dpt[QW];
#pragma unroll
      for (int qw = 0; qw < QW; ++qw)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          st[qw][r] = nl2[qw];
          dpt[qw][r] = DROP ? 0.f : dl[qw];
        }
#pragma unroll
      for (int s = 0; s < HDP / 16; ++s)
#pragma unroll
        for (int qw = 0; qw < QW; ++qw) {
          st[qw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka[s], qf[qw][s], st[qw], 0, 0, 0);
          dpt[qw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va[s], gf[qw][s], dpt[qw], 0, 0, 0);
        }
      // keys past the end are zero rows of K and V; masked on the ragged last tile only so an
      // extreme lse cannot turn 2^(-lse2) * 0 into inf * 0
      if (ragged) {  // uniform branch, last tile only
        asm volatile("");  // keeps the compiler from if-converting this into every tile
#pragma unroll
        for (int qw = 0; qw < QW; ++qw)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kt * KT + kk * 32 + acc_row(r, lane) >= klim[qw]) st[qw][r] = -INFINITY;
      }
#pragma unroll
      for (int qw = 0; qw < QW; ++qw)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(st[qw][r] * c);
          if constexpr (DROP) {  // dS = P (z dP - delta), dP = dO V^T (see k_attn_bwd_dkdv)
            const uint32_t kl = (uint32_t)(kt * KT + kk * 32 + acc_row(r, lane));
            const float z = drop_u(drow[qw], kl) >= a.drop_thresh ? a.drop_scale : 0.f;
            dpt[qw][r] = p * fmaf(z, dpt[qw][r], dl[qw]);
          } else {
            dpt[qw][r] *= p;
          }
        }
      lds_wait();
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) tie(ktf[s2]);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int qw = 0; qw < QW; ++qw) {
          const bf16x8 sf = acc_frag(dpt[qw], s2);
#pragma unroll
          for (int d = 0; d < HDP / 32; ++d)
            dqt[qw][d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ktf[s2][d], sf, dqt[qw][d], 0, 0, 0);
        }
    }
    __syncthreads();
  };
  for (int kt0 = 0; kt0 < nkt; kt0 += 2) {
    tile_iter(kt0, std::integral_constant<int, 0>{});
    if (kt0 + 1 < nkt) tile_iter(kt0 + 1, std::integral_constant<int, 1>{});
  }
  // the K / V buffers are free after the last tile's barrier: rows go out through a wave-private image
  static_assert(4 * OutTile<HD>::BYTES <= 4 * TB, "output images fit the K / V buffers");
  LDS_AS char* ob = smem + wave * OutTile<HD>::BYTES;
#pragma unroll
  for (int qw = 0; qw < QW; ++qw) {
    const int q0 = qt * 128 * QW + qw * 128 + wave * 32;
    if (q0 >= len) continue;  // wave-uniform
    const bool rope = a.cos_t != nullptr;
    const TokPos tp = rope ? tok_pos(a, seq0 + min(qloc[qw], len - 1)) : TokPos{0, 0, 0};
#pragma unroll
    for (int d = 0; d < HDP / 32; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) dqt[qw][d][r] *= a.scale;
    if (rope) rope_inv_rows<HD>(a, tp, lane, dqt[qw]);  // rotate first, then store (see k_attn_bwd_dkdv)
    wave_store_rows<HD>(dqt[qw], 1.f, ob, a.dqkv + (long)(seq0 + q0) * a.ldd + a.q_off + h * HD, a.ldd, len - q0,
                        lane);
  }
}

int fill_groups(SeqGroups& sg, int ngroups, const int* nseq, const int* len, int tile, long T) {
  VJ_CHECK_ARG(ngroups >= 1 && ngroups <= MAXG, "attention: 1..%d sequence groups supported (got %d)", MAXG, ngroups);
  sg.ngroups = ngroups;
  long tok = 0, tiles = 0;
  for (int g = 0; g < MAXG; ++g) {
    if (g < ngroups) {
      VJ_CHECK_ARG(nseq[g] >= 0 && len[g] >= 1, "attention: bad group %d (nseq=%d len=%d)", g, nseq[g], len[g]);
      sg.nseq[g] = nseq[g];
      sg.len[g] = len[g];
      sg.tok0[g] = (int)tok;
      sg.tiles_prefix[g] = (int)tiles;
      tok += (long)nseq[g] * len[g];
      tiles += (long)nseq[g] * ((len[g] + tile - 1) / tile);
    } else {
      sg.nseq[g] = 0;
      sg.len[g] = 1;
      sg.tok0[g] = (int)tok;
      sg.tiles_prefix[g] = (int)tiles;
    }
  }
  sg.tiles_prefix[MAXG] = (int)tiles;
  VJ_CHECK_ARG(tok == T, "attention: groups cover %ld tokens but T=%ld", tok, T);
  return VJ_OK;
}

int check_common(int H, int hd, long ld, long ldo) {
  VJ_CHECK_ARG(hd == 64 || hd == 32 || hd == 80 || hd == 88,
               "attention: head_dim must be 32, 64, 80 or 88 (got %d)", hd);
  VJ_CHECK_ARG(H >= 1 && H <= 65535, "attention: bad H=%d", H);
  VJ_CHECK_ARG(ld % 8 == 0 && ldo % 8 == 0, "attention: row strides must be multiples of 8");
  return VJ_OK;
}

}  // namespace

// Forward / backward with SDPA's attention dropout (dropout_p = p, modules.py:246 / 370 / 417; p = 0 is
// the plain kernels): the mask is regenerated from `seed` by the backward, which must get the same p and
// seed as the forward it differentiates.
extern "C" int vj_attn_fwd_ex(int T, int H, int hd, const void* qkv, long ld, int q_off, int k_off, int v_off,
                              void* o, long ldo, float* lse_stats, float scale, int ngroups, const int* nseq,
                              const int* len, int fblk, float dropout_p, unsigned seed, void* stream) {
  if (T == 0) return VJ_OK;
  int rc = check_common(H, hd, ld, ldo);
  if (rc) return rc;
  VJ_CHECK_ARG(fblk >= 0, "vj_attn_fwd: bad frame block %d", fblk);
  VJ_CHECK_ARG(dropout_p >= 0.f && dropout_p < 1.f, "vj_attn_fwd: dropout_p must be in [0, 1)");
  AttnArgs a{};
  a.fblk = fblk;
  a.qkv = (const bf16_t*)qkv; a.ld = ld; a.q_off = q_off; a.k_off = k_off; a.v_off = v_off;
  a.o = (bf16_t*)o; a.ldo = ldo; a.stats = lse_stats; a.H = H; a.T = T; a.scale = scale;
  a.drop_thresh = vj_drop_thresh(dropout_p); a.drop_seed = seed; a.drop_scale = 1.f / (1.f - dropout_p);
  rc = fill_groups(a.sg, ngroups, nseq, len, 128, T);
  if (rc) return rc;
  dim3 grid(a.sg.tiles_prefix[MAXG], H);
  hipStream_t st = (hipStream_t)stream;
  auto go = [&](auto drop_c) {
    constexpr bool D = decltype(drop_c)::value;
    switch (hd) {
      case 64: hipLaunchKernelGGL((k_attn_fwd<64, D>), grid, dim3(256), 0, st, a); break;
      case 32: hipLaunchKernelGGL((k_attn_fwd<32, D>), grid, dim3(256), 0, st, a); break;
      case 80: hipLaunchKernelGGL((k_attn_fwd<80, D>), grid, dim3(256), 0, st, a); break;
      default: hipLaunchKernelGGL((k_attn_fwd<88, D>), grid, dim3(256), 0, st, a); break;
    }
  };
  if (a.drop_thresh) go(std::true_type{});
  else go(std::false_type{});
  VJ_LAUNCH_CHECK("vj_attn_fwd");
  return VJ_OK;
}

extern "C" int vj_attn_fwd_fc(int T, int H, int hd, const void* qkv, long ld, int q_off, int k_off, int v_off,
                              void* o, long ldo, float* lse_stats, float scale, int ngroups, const int* nseq,
                              const int* len, int fblk, void* stream) {
  return vj_attn_fwd_ex(T, H, hd, qkv, ld, q_off, k_off, v_off, o, ldo, lse_stats, scale, ngroups, nseq, len, fblk,
                        0.f, 0u, stream);
}

extern "C" int vj_attn_fwd(int T, int H, int hd, const void* qkv, long ld, int q_off, int k_off, int v_off, void* o,
                           long ldo, float* lse_stats, float scale, int ngroups, const int* nseq, const int* len,
                           void* stream) {
  return vj_attn_fwd_ex(T, H, hd, qkv, ld, q_off, k_off, v_off, o, ldo, lse_stats, scale, ngroups, nseq, len, 0, 0.f,
                        0u, stream);
}

extern "C" int vj_attn_bwd_ex(int T, int H, int hd, const void* qkv, long ld, int q_off, int k_off, int v_off,
                              const void* o, long ldo, const void* dout, long lddo, float* stats, void* dqkv,
                              long ldd, float scale, int ngroups, const int* nseq, const int* len,
                              const int* rope_ids, int rope_mod, int rope_tpf, int rope_tpr, const float* cos_t,
                              const float* sin_t, int fblk, float dropout_p, unsigned seed, void* stream) {
  if (T == 0) return VJ_OK;
  int rc = check_common(H, hd, ld, ldo);
  if (rc) return rc;
  VJ_CHECK_ARG(fblk >= 0, "vj_attn_bwd: bad frame block %d", fblk);
  VJ_CHECK_ARG(dropout_p >= 0.f && dropout_p < 1.f, "vj_attn_bwd: dropout_p must be in [0, 1)");
  VJ_CHECK_ARG(lddo % 8 == 0 && ldd % 8 == 0, "vj_attn_bwd: strides must be multiples of 8");
  VJ_CHECK_ARG(!cos_t || (sin_t && (rope_ids || rope_mod > 0) && rope_tpf > 0 && rope_tpr > 0),
               "vj_attn_bwd: incomplete RoPE arguments");
  AttnArgs a{};
  a.rope_ids = rope_ids;
  a.rope_mod = rope_mod;
  a.rope_tpf = rope_tpf;
  a.rope_tpr = rope_tpr;
  a.rope_half = (hd / 3) / 2;
  a.cos_t = cos_t;
  a.sin_t = sin_t;
  a.qkv = (const bf16_t*)qkv; a.ld = ld; a.q_off = q_off; a.k_off = k_off; a.v_off = v_off;
  a.o = (bf16_t*)o; a.ldo = ldo; a.dout = (const bf16_t*)dout; a.lddo = lddo; a.stats = stats;
  a.dqkv = (bf16_t*)dqkv; a.ldd = ldd; a.H = H; a.T = T; a.scale = scale; a.fblk = fblk;
  a.drop_thresh = vj_drop_thresh(dropout_p); a.drop_seed = seed; a.drop_scale = 1.f / (1.f - dropout_p);
  // key / query 32-row tiles per wave of the two sweeps (block tile = 128 x that)
  const int kw = hd == 32 ? KW32 : hd == 64 ? KW64 : 1;
  const int qw = hd == 32 ? QW32 : hd == 64 ? QW64 : 1;
  AttnArgs ak = a, aq = a;
  rc = fill_groups(ak.sg, ngroups, nseq, len, 128 * kw, T);
  if (rc) return rc;
  rc = fill_groups(aq.sg, ngroups, nseq, len, 128 * qw, T);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  const dim3 gk(ak.sg.tiles_prefix[MAXG], H), gq(aq.sg.tiles_prefix[MAXG], H);
  // dQ sweep first: it writes -delta for the dK/dV sweep
  auto go = [&](auto drop_c) {
    constexpr bool D = decltype(drop_c)::value;
    switch (hd) {
      case 64:
        hipLaunchKernelGGL((k_attn_bwd_dq<64, QW64, D>), gq, dim3(256), 0, st, aq);
        hipLaunchKernelGGL((k_attn_bwd_dkdv<64, KW64, D>), gk, dim3(256), 0, st, ak);
        break;
      case 32:
        hipLaunchKernelGGL((k_attn_bwd_dq<32, QW32, D>), gq, dim3(256), 0, st, aq);
        hipLaunchKernelGGL((k_attn_bwd_dkdv<32, KW32, D>), gk, dim3(256), 0, st, ak);
        break;
      case 80:
        hipLaunchKernelGGL((k_attn_bwd_dq<80, 1, D>), gq, dim3(256), 0, st, aq);
        hipLaunchKernelGGL((k_attn_bwd_dkdv<80, 1, D>), gk, dim3(256), 0, st, ak);
        break;
      default:
        hipLaunchKernelGGL((k_attn_bwd_dq<88, 1, D>), gq, dim3(256), 0, st, aq);
        hipLaunchKernelGGL((k_attn_bwd_dkdv<88, 1, D>), gk, dim3(256), 0, st, ak);
        break;
    }
  };
  if (a.drop_thresh) go(std::true_type{});
  else go(std::false_type{});
  VJ_LAUNCH_CHECK("vj_attn_bwd");
  return VJ_OK;
}

extern "C" int vj_attn_bwd_fc(int T, int H, int hd, const void* qkv, long ld, int q_off, int k_off, int v_off,
                              const void* o, long ldo, const void* dout, long lddo, float* stats, void* dqkv,
                              long ldd, float scale, int ngroups, const int* nseq, const int* len,
                              const int* rope_ids, int rope_mod, int rope_tpf, int rope_tpr, const float* cos_t,
                              const float* sin_t, int fblk, void* stream) {
  return vj_attn_bwd_ex(T, H, hd, qkv, ld, q_off, k_off, v_off, o, ldo, dout, lddo, stats, dqkv, ldd, scale, ngroups,
                        nseq, len, rope_ids, rope_mod, rope_tpf, rope_tpr, cos_t, sin_t, fblk, 0.f, 0u, stream);
}

extern "C" int vj_attn_bwd(int T, int H, int hd, const void* qkv, long ld, int q_off, int k_off, int v_off,
                           const void* o, long ldo, const void* dout, long lddo, float* stats, void* dqkv, long ldd,
                           float scale, int ngroups, const int* nseq, const int* len, const int* rope_ids,
                           int rope_mod, int rope_tpf, int rope_tpr, const float* cos_t, const float* sin_t,
                           void* stream) {
  return vj_attn_bwd_ex(T, H, hd, qkv, ld, q_off, k_off, v_off, o, ldo, dout, lddo, stats, dqkv, ldd, scale, ngroups,
                        nseq, len, rope_ids, rope_mod, rope_tpf, rope_tpr, cos_t, sin_t, 0, 0.f, 0u, stream);
}
