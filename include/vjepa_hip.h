/*
 * libvjepa_hip.so — C ABI of the MI355X (gfx950) V-JEPA 2 train-step kernels.
 *
 * The reference (weipeilun/vjepa2) is pure PyTorch: its hot path has no FFI. Each entry point below
 * replaces the ATen call(s) named in its comment (reference file:line); the Python host layer
 * (vjepa2_amd/) binds them with ctypes (INTEGRATION.md shows the binding) behind the reference's
 * module API (VisionTransformer / VisionTransformerPredictor forward(), app/vjepa train step).
 *
 * Conventions
 *  - All pointers are device pointers unless stated; dims/strides are in ELEMENTS unless *_bytes.
 *  - bf16 tensors are raw 16-bit storage; f32 is IEEE float.
 *  - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream); every call only enqueues
 *    work on it: no host sync, no allocation, so every call is graph-capturable.
 *  - Return 0 on success, else an error code; vj_get_last_error() gives the message (thread-local).
 *    The library never exits the process and never frees caller memory.
 *  - Deterministic: no floating-point atomics anywhere (reductions are fixed-order two-level).
 */
#ifndef VJEPA_HIP_H
#define VJEPA_HIP_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

int vj_version(void);
/* CRC-32 (zlib) of this header as the library was built from it, as an int bit pattern (the binding
 * refuses a stale build). */
int vj_header_crc(void);
int vj_get_last_error(char* buf, size_t n);
int vj_device_sync(void);

/* GEMM epilogues. vj_gemm_bf16 accepts 0-4 and 7; 5 and 6 are internal (5: vj_qkv_rope_gemm's RoPE
 * epilogue, 6: the split-K partial slabs of vj_gemm_bf16_splitk) and are rejected there. */
enum {
  VJ_EPI_BF16 = 0,       /* C(bf16) = acc + bias                                                      */
  VJ_EPI_F32 = 1,        /* C(f32)  = acc + bias                                                      */
  VJ_EPI_F32_RESID = 2,  /* C(f32)  = aux(f32 residual) + acc + bias   (Block residual add)            */
  VJ_EPI_GELU = 3,       /* C(bf16) = GELU'(pre) if C != NULL, C2(bf16) = GELU_erf(pre), pre = bf16(acc + bias) */
  VJ_EPI_GELU_BWD = 4,   /* C(bf16) = acc * aux (the saved bf16 GELU'(pre))                             */
  VJ_EPI_ROPE = 5,       /* internal: QKV + 3-axis RoPE (vj_qkv_rope_gemm)                               */
  VJ_EPI_PARTIAL = 6,    /* internal: f32 split-K partial slabs (vj_gemm_bf16_splitk)                    */
  VJ_EPI_BF16_RESID = 7  /* C(bf16) = bf16(aux(bf16 residual) + acc + bias) (no-grad target encoder)    */
};

/* C[m,n] = sum_k A(m,k) B(n,k) (+ epilogue), bf16 operands, f32 accumulate. M >= 1024 runs the 256-row
 * tile kernels on v_mfma_f32_16x16x32_bf16 (vj_gemm256.hip: the one-tile main loop, or the staggered
 * one for the K-major 256-wide GELU / RoPE / bf16 / f32 GEMMs), smaller M the 128-row kernel on
 * v_mfma_f32_32x32x16_bf16 (vj_gemm.hip).
 * A(m,k) = a_kmajor ? A[m*lda+k] : A[k*lda+m];  B(n,k) = b_kmajor ? B[n*ldb+k] : B[k*ldb+n].
 * Replaces nn.Linear forward/backward (modules.py:77-83, 330, 379-381; predictor.py:182, 244) and the
 * Conv3d tubelet projection as a GEMM over im2col rows (patch_embed.py:42-52). */
int vj_gemm_bf16(int M, int N, int K, const void* A, long lda, int a_kmajor, const void* B, long ldb, int b_kmajor,
                 int epi, const float* bias, const void* aux, long ldaux, void* C, long ldc, void* C2, long ldc2,
                 void* stream);
/* Same with deterministic split-K over K (weight gradients: K = tokens, small M x N): blockIdx.z
 * computes a K slice into ws [splitk][M][N] (f32), then one pass sums the slices in fixed order and
 * applies the epilogue (BF16 / F32 / F32_RESID only). ws >= splitk*M*N floats. */
int vj_gemm_bf16_splitk(int M, int N, int K, const void* A, long lda, int a_kmajor, const void* B, long ldb,
                        int b_kmajor, int epi, const float* bias, const void* aux, long ldaux, void* C, long ldc,
                        void* C2, long ldc2, int splitk, float* ws, long ws_floats, void* stream);
/* nn.Linear's weight AND bias gradients from one read of dY (the autograd of F.linear, modules.py:77-83,
 * 330, 379-381): dw[M, N] (+)= dY^T X (accumulate), db[M] (+)= sum_k dY[k, m] (db_accumulate; db may be
 * NULL), dY [K, M] and X [K, N] row-major bf16 (K = tokens), split-K as vj_gemm_bf16_splitk. The bias sums
 * are fused into the split-K GEMM's 256-row kernel (f32, fixed order) when it runs, else computed by a
 * column-sum pass. ws >= max(splitk > 1 ? splitk * (M * N + M) : 0, min(256, ceil(K / 64)) * M) floats. */
int vj_gemm_bf16_wgrad(int M, int N, int K, const void* dy, long lddy, const void* x, long ldx, float* dw, long lddw,
                       int accumulate, float* db, int db_accumulate, int splitk, float* ws, long ws_floats,
                       void* stream);

/* Varlen non-causal flash attention, head_dim 32, 64, 80 or 88 (80 / 88 padded to 96 in LDS and in the
 * MFMA loops; F.scaled_dot_product_attention,
 * modules.py:367-372 / 411-418). Tokens of `ngroups` groups of equal-length sequences are
 * concatenated: group g has nseq[g] sequences of len[g] tokens. q/k/v at columns q_off/k_off/v_off
 * + h*hd of the [T, ld] bf16 buffer; O bf16 [T, ldo] at column h*hd.
 * stats: f32 [2][H][T]; forward writes stats[0] = log2-sum-exp2 of the scaled scores in base-2 units
 * (= logsumexp(scale * s) * log2(e)) per (head, token). */
int vj_attn_fwd(int T, int H, int hd, const void* qkv, long ld, int q_off, int k_off, int v_off, void* o, long ldo,
                float* stats, float scale, int ngroups, const int* nseq, const int* len, void* stream);
/* Backward: writes dq/dk/dv (bf16) into dqkv at the same column offsets; uses stats[0] and writes
 * stats[1] = -rowsum(dO * O). Deterministic (separate dK/dV and dQ sweeps, no atomics). With cos_t
 * non-NULL the transpose of the 3-axis RoPE (see vj_rope) is applied to dq and dk before the store,
 * i.e. dqkv is the gradient w.r.t. the UN-rotated q, k (the QKV projection output). */
int vj_attn_bwd(int T, int H, int hd, const void* qkv, long ld, int q_off, int k_off, int v_off, const void* o,
                long ldo, const void* dout, long lddo, float* stats, void* dqkv, long ldd, float scale, int ngroups,
                const int* nseq, const int* len, const int* rope_ids, int rope_mod, int rope_tpf, int rope_tpr,
                const float* cos_t, const float* sin_t, void* stream);
/* Frame-causal (block-causal) variants for the action-conditioned predictor: with fblk > 0, token i
 * of a sequence attends to key j iff j / fblk <= i / fblk, i.e. F.scaled_dot_product_attention with the
 * attn_mask of build_action_block_causal_attention_mask (src/models/utils/modules.py:12-23; fblk = action
 * tokens + H*W per frame, ACRoPEAttention.forward modules.py:243-247). fblk = 0 is vj_attn_fwd / _bwd. */
int vj_attn_fwd_fc(int T, int H, int hd, const void* qkv, long ld, int q_off, int k_off, int v_off, void* o, long ldo,
                   float* stats, float scale, int ngroups, const int* nseq, const int* len, int fblk, void* stream);
int vj_attn_bwd_fc(int T, int H, int hd, const void* qkv, long ld, int q_off, int k_off, int v_off, const void* o,
                   long ldo, const void* dout, long lddo, float* stats, void* dqkv, long ldd, float scale, int ngroups,
                   const int* nseq, const int* len, const int* rope_ids, int rope_mod, int rope_tpf, int rope_tpr,
                   const float* cos_t, const float* sin_t, int fblk, void* stream);
/* With attention dropout (F.scaled_dot_product_attention(..., dropout_p=self.proj_drop_prob),
 * src/models/utils/modules.py:246 / 370 / 417; applied whether or not the module is training, as there):
 * score (query token t, head h, key j of its sequence) is kept iff
 * drop_u(drop_row(seed, t*H + h), j) >= round(p * 2^32) (the hash of vj_dropout below); the kept
 * probabilities are scaled by 1 / (1 - p) and stats[0] stays the log-sum-exp of the undropped scores.
 * The backward regenerates the mask: it must get the forward's p and seed. p = 0: vj_attn_*_fc. */
int vj_attn_fwd_ex(int T, int H, int hd, const void* qkv, long ld, int q_off, int k_off, int v_off, void* o, long ldo,
                   float* stats, float scale, int ngroups, const int* nseq, const int* len, int fblk, float dropout_p,
                   unsigned seed, void* stream);
int vj_attn_bwd_ex(int T, int H, int hd, const void* qkv, long ld, int q_off, int k_off, int v_off, const void* o,
                   long ldo, const void* dout, long lddo, float* stats, void* dqkv, long ldd, float scale, int ngroups,
                   const int* nseq, const int* len, const int* rope_ids, int rope_mod, int rope_tpf, int rope_tpr,
                   const float* cos_t, const float* sin_t, int fblk, float dropout_p, unsigned seed, void* stream);

/* Fused QKV projection + RoPE of q and k: C[M, 3*H*hd] (bf16) = A[M,K] W[3*H*hd, K]^T + bias, then
 * q, k columns rotated (modules.py:330 + 343-365) in the GEMM epilogue. Same RoPE arguments as vj_rope;
 * npos = rows of the cos/sin tables, every frame/row/column position of an id must be < npos (<= 1024). */
int vj_qkv_rope_gemm(int M, int K, const void* A, long lda, const void* B, long ldb, const float* bias, void* C,
                     long ldc, int H, int hd, const int* ids, int ids_mod, int tpf, int tpr, const float* cos_t,
                     const float* sin_t, int npos, void* stream);

/* fp8 (OCP e4m3) forward GEMMs of the opt-in fp8 target encoder (BASELINE configs[4]; the reference has
 * no fp8: judged by its error envelope). A [M, K] and B [N, K] e4m3 bytes, both K-major (X W^T), with
 * per-row power-of-two scales: A(m, k) = A8[m, k] * 2^ea[m], B(n, k) = B8[n, k] * 2^eb[n] (device int32
 * exponents, applied exactly by the MFMA's E8M0 scale operands); f32 accumulation. K, lda, ldb multiples
 * of 16 bytes. Epilogues: VJ_EPI_BF16 / VJ_EPI_F32 / VJ_EPI_F32_RESID / VJ_EPI_GELU (bf16 act) as vj_gemm_bf16;
 * replaces the QKV (+RoPE, modules.py:330 + 343-365) and fc1 (+GELU, :77-83) Linears of the target encoder. */
int vj_gemm_fp8(int M, int N, int K, const void* A, long lda, const int* ea, const void* B, long ldb, const int* eb,
                int epi, const float* bias, const void* aux, long ldaux, void* C, long ldc, void* C2, long ldc2,
                void* stream);
int vj_qkv_rope_gemm_fp8(int M, int K, const void* A, long lda, const int* ea, const void* B, long ldb, const int* eb,
                         const float* bias, void* C, long ldc, int H, int hd, const int* ids, int ids_mod, int tpf,
                         int tpr, const float* cos_t, const float* sin_t, int npos, void* stream);
/* Per-row e4m3 quantisation: y8[m, :] = e4m3(x[m, :] * 2^-e[m]), e[m] the least exponent with
 * max|x[m, :]| * 2^-e <= 448 (0 for a zero row; a non-finite row becomes NaN bytes). x f32 or bf16. */
int vj_quant_rows_fp8(int M, int K, const void* x, int x_bf16, long ldx, void* y8, long ldy, int* yexp, void* stream);
/* LayerNorm whose output row is written as per-row scaled e4m3 (as vj_quant_rows_fp8) for the fp8 GEMMs. */
int vj_layernorm_fwd_fp8(int M, int D, const void* x, int x_bf16, long ldx, const float* gamma, const float* beta,
                         float eps, void* y8, long ldy, int* yexp, float* mean, float* rstd, void* stream);

/* LayerNorm (nn.LayerNorm / F.layer_norm, modules.py:556-563, train.py:417): x f32 or bf16, y bf16 or f32,
 * gamma/beta optional (both or neither); mean/rstd optional outputs. D % 4 == 0, D <= 2048. */
int vj_layernorm_fwd(int M, int D, const void* x, int x_bf16, long ldx, const float* gamma, const float* beta,
                     float eps, void* y, int y_f32, long ldy, float* mean, float* rstd, void* stream);
/* Backward (dy bf16): dres(f32) = (dres_in or 0) + dx; optional bf16 copy of dres; dgamma/dbeta
 * accumulated (+=) through a workspace of vj_layernorm_bwd_blocks(M)*2*D floats. Optional sum_in / sum_out
 * (+=) column sums of dres_in / dres (the fc2 / proj bias gradients, modules.py:77-83, 326-382); with
 * either, the workspace needs vj_layernorm_bwd_blocks(M)*4*D floats. */
int vj_layernorm_bwd_blocks(int M);
int vj_layernorm_bwd(int M, int D, const void* dy, long lddy, const float* x, long ldx, const float* mean,
                     const float* rstd, const float* gamma, const float* dres_in, long ldri, float* dres, long ldr,
                     void* dres_bf16, long ldrb, float* dgamma, float* dbeta, float* sum_in, float* sum_out, float* ws,
                     long ws_floats, void* stream);
/* The same on the bf16 residual stream of the trained encoder under bf16 autocast (modules.py:561-562:
 * x = x + attn(norm1(x)) is a bf16 add there): x, dres_in and dres are bf16 rows (D % 8 == 0, strides
 * % 8, 16-B aligned), dres = bf16(dres_in + dx) with the sum in f32; column partials as above. */
int vj_layernorm_bwd_bf16(int M, int D, const void* dy, long lddy, const void* x, long ldx, const float* mean,
                          const float* rstd, const float* gamma, const void* dres_in, long ldri, void* dres, long ldr,
                          float* dgamma, float* dbeta, float* sum_in, float* sum_out, float* ws, long ws_floats,
                          void* stream);

/* GELU(x) and GELU'(x) (nn.GELU(), vision_transformer.py:100) of n bf16 inputs, bf16 outputs, by the exact
 * evaluation the GEMM epilogues use (the fc1 GEMM's table epilogue equals it bitwise on every bf16 input). */
int vj_gelu_eval(int n, const void* x, void* y, void* dy, void* stream);

/* out[n] (+)= sum_m x[m, n]  (bias gradients), N % 8 == 0. ws >= min(256, ceil(M/64)) * N floats. */
int vj_colsum_f32(int M, int N, const void* x, int x_bf16, long ld, float* out, int accumulate, float* ws,
                  long ws_floats, void* stream);

/* 3-axis RoPE of q and k, in place (rotate_queries_or_keys, modules.py:26-50, applied at :343-365).
 * Token id -> (frame, row, col) with tokens_per_frame / tokens_per_row (modules.py:293-324).
 * ids: int32 [T] or NULL (then id = t % ids_mod). cos/sin tables f32 [pos][half], half = (hd/3)/2.
 * inverse = 1 applies the transpose (gradient). */
int vj_rope(int T, int H, int hd, void* qkv, long ld, int q_off, int k_off, const int* ids, int ids_mod,
            int tokens_per_frame, int tokens_per_row, const float* cos_tab, const float* sin_tab, int half,
            int inverse, void* stream);

/* Tubelet im2col for the Conv3d patch embedding, gathering only the kept tokens (PatchEmbed3D +
 * apply_masks, patch_embed.py:49-52, vision_transformer.py:188-192). Row r = sample r/K, token
 * idx[r] (int64 mask [B,K] flattened) or r%K when idx is NULL. out bf16 [R, C*tub*p*p]. */
int vj_im2col_tubelet(int R, int K, const long* idx, int B, int C, int Tf, int Hf, int Wf, int tub, int pch,
                      const float* clip, void* out, void* stream);

/* Bit-exact row moves (apply_masks gather, predictor sort/unsort, predictor.py:194-241):
 * scatter=0: dst[r] = src[idx[r]];  scatter=1: dst[idx[r]] = src[r]. */
int vj_gather_rows(int R, int rowbytes, const void* src, long src_ld_bytes, const int* idx, void* dst,
                   long dst_ld_bytes, int scatter, void* stream);
/* dst[idx[r]] = vec (mask tokens, predictor.py:194-197). */
int vj_fill_rows(int R, int D, float* dst, long ldd, const int* idx, const float* vec, void* stream);
/* dst[r] += table[idx ? idx[r] : r % idx_mod] (sincos pos-embed add, non-RoPE variant); table has
 * trows rows: an id outside [0, trows) is not read and leaves its row unchanged. */
int vj_add_rows(int R, int D, float* dst, long ldd, const float* table, long ldt, int trows, const int* idx,
                int idx_mod, void* stream);

/* Predictor sort indices for one mask pair: stable rank of cat(mx[b], my[b]) (= torch.argsort for
 * unique ids, predictor.py:210-217; inverse at :240-242). Outputs int32 (see vj_ops.hip). */
int vj_pred_index(int B, int K, int Kp, const long* mx, const long* my, int row0, int bmod, int N, int* pos,
                  int* ctx_dst, int* tgt_rows, int* loss_rows, void* stream);
int vj_ids64to32(long n, const long* in, int* out, void* stream);

/* Fused forward_target normalisation + JEPA loss + dL/dz (train.py:414-435). */
/* z: predictor output rows (bf16 if z_bf16 else f32); tgt: target-encoder rows (bf16 if tgt_bf16
 * else f32); rows split into ngroups mask groups of group_rows[g] rows; per-row weight
 * pair_weight / (group_rows[g] * D). dz is bf16. */
int vj_jepa_loss(int R, int D, const void* z, int z_bf16, long ldz, const void* tgt, int tgt_bf16, long ldt,
                 const int* loss_rows,
                 const float* gamma, const float* beta, float eps1, float eps2, float loss_exp, int ngroups,
                 const int* group_rows, float pair_weight, void* dz, long lddz, float* row_loss, float* loss_out,
                 void* stream);

/* Optimizer and EMA over flat fp32 arenas (torch.optim.AdamW foreach math, app/vjepa/utils.py:239;
 * GradScaler inf-skip train.py:446-451; EMA train.py:456-465). p_bf16 / target_bf16: optional
 * bf16 shadow copies written in the same pass (the next forward's GEMM operands). */
int vj_check_finite(long n, const float* g, int* found_inf, void* stream);
int vj_adamw(long n, float* p, const float* g, float* m, float* v, void* p_bf16, float lr, float beta1, float beta2,
             float eps, float weight_decay, int step, float grad_scale, const int* found_inf, void* stream);
int vj_ema(long n, float* target, const float* online, float momentum, void* target_bf16, void* stream);
/* vj_adamw + vj_ema in one pass (train.py:443-465): the parameters are updated, then
 * target = target * momentum + (1 - momentum) * p from the new values (on a step skipped by found_inf,
 * from the unchanged ones) with its bf16 shadow; target / target_bf16 NULL = plain vj_adamw. */
int vj_adamw_ema(long n, float* p, const float* g, float* m, float* v, void* p_bf16, float lr, float beta1,
                 float beta2, float eps, float weight_decay, int step, float grad_scale, const int* found_inf,
                 float* target, void* target_bf16, float momentum, void* stream);
int vj_cast_bf16(long n, const float* in, void* out, void* stream);
/* Diagnostic (bench.py --rccl-proxy-cus, no reference counterpart): copy `bytes` (multiple of 16,
 * 16-B aligned) with `blocks` persistent 256-thread workgroups, standing in for RCCL's channel kernels
 * holding CUs during the data-parallel gradient all-reduce (app/vjepa/train.py:279-281). mode 0: plain
 * loads / stores, 1: non-temporal, 2: hold the CUs for the copy's time at 40 GB/s per workgroup, no bytes. */
int vj_proxy_copy(void* dst, const void* src, long bytes, int blocks, int mode, void* stream);
/* Persistent GEMM grids launched from now on leave n CUs free (0: every CU): a data-parallel rank sets
 * it while its gradient all-reduce (app/vjepa/train.py:279-281, RCCL channel kernels) runs beside the
 * backward. Host state only (no device call). */
int vj_set_reserved_cus(int n);
/* dst[c][r] = src[r][c] (bf16; rows, cols, strides multiples of 8): the K-major copy W^T that the
 * data-gradient GEMM dX = dY W (nn.Linear backward) reads as its B operand. */
int vj_transpose_bf16(int rows, int cols, const void* src, long ld_src, void* dst, long ld_dst, void* stream);
/* n bf16 transposes in one launch (the per-step W^T copies): desc = DEVICE int64 [n][8] =
 * {src, dst, rows, cols, ld_src, ld_dst, first_tile, tiles_x} with 64 x 64 tiles numbered
 * consecutively (first_tile = running sum of ceil(rows/64)*ceil(cols/64), tiles_x = ceil(cols/64));
 * each matrix meets vj_transpose_bf16's constraints. Replaces one vj_transpose_bf16 launch per weight. */
int vj_transpose_bf16_batch(int n, const long* desc, long total_tiles, void* stream);

/* Block variants off the shipped configs (vj_variants.hip), bf16-autocast rounding points.
 * SwiGLU gate (SwiGLUFFN.forward, src/models/utils/modules.py:102-106): x12 = [M][2h] bf16 holding
 * fc1(x) | fc2(x); out[m][c] = bf16(bf16(silu(x1)) * x2). Backward: dh [M][h] -> dx12 = dx1 | dx2
 * (mul backward, then silu_backward). h, strides multiples of 8, pointers 16-B aligned. */
int vj_swiglu_fwd(int M, int h, const void* x12, long ld, void* out, long ldo, void* stream);
int vj_swiglu_bwd(int M, int h, const void* dh, long lddh, const void* x12, long ld, void* dx12, long lddx,
                  void* stream);
/* Stochastic depth (timm drop_path, applied in Block.forward modules.py:561-562): per-row factor
 * scale[m] (0 or 1 / keep, the sample's draw repeated over its tokens).
 * vj_rowscale_add: out = resid + bf16(bf16(y) * bf16(scale[m])), y f32 [M][N] (the branch's output
 * projection), resid / out f32 or, bf16_resid = 1, bf16. vj_rowscale_bf16: out bf16 = bf16(bf16(dx) *
 * bf16(scale[m])) (the branch's dY in the backward). N, strides multiples of 4. */
int vj_rowscale_add(int M, int N, const float* y, long ldy, const float* scale, const void* resid, long ldr, void* out,
                    long ldo, int bf16_resid, void* stream);
int vj_rowscale_bf16(int M, int N, const float* dx, long ld, const float* scale, void* out, long ldo, void* stream);
/* Dropout (nn.Dropout: MLP.drop after the activation and after fc2, modules.py:75-82; proj_drop after
 * the attention projection, :257 / :381), on [M][N]: element (m, n) is kept iff
 * drop_u(drop_row(seed, m), n) >= round(p * 2^32), with drop_mix = the "lowbias32" integer hash,
 * drop_row(s, r) = drop_mix(s ^ (r * 0x9e3779b1)), drop_u(k, c) = drop_mix(k + c * 0x85ebca77) (uint32
 * arithmetic). y = bf16(bf16(x) * z), z = 1 / (1 - p) if kept else 0; x f32 (x_f32 = 1) or bf16.
 * out = y (bf16); with resid: out = resid + y (f32, or bf16 when resid_f32 = 0); with aux (bf16):
 * out = bf16(y * aux). The backward of a dropout is the same call on the gradient with the same seed.
 * N, strides multiples of 4; p in [0, 1). */
int vj_dropout(int M, int N, const void* x, long ldx, int x_f32, const void* aux, long ldaux, const void* resid,
               long ldr, int resid_f32, void* out, long ldo, float dropout_p, unsigned seed, void* stream);

/* JEPA multi-block 3-D masks on the device (src/masks/multiseq_multiblock3d.py:155-239): the host
 * makes the reference's RNG draws (block size, (start, top, left) per block: boxes int32
 * [B][npred][3]); vj_mask_count writes each sample's kept-token count, vj_mask_emit the ascending
 * context / target id lists truncated to k_enc / k_pred (int64 [B][K]; mode 1 = full_complement,
 * 2 = pred_full_complement: the complement of the other list). Replaces the per-sample
 * torch.ones / slicing / argwhere / nonzero / default_collate of _MaskGenerator.__call__. */
int vj_mask_count(int B, int duration, int height, int width, int npred, const int* boxes, int t, int h, int w,
                  int max_ctx, int* counts, void* stream);
int vj_mask_emit(int B, int duration, int height, int width, int npred, const int* boxes, int t, int h, int w,
                 int max_ctx, int mode, int k_enc, int k_pred, long* enc, long* pred, void* stream);

/* Video clip transform (app/vjepa/transforms.py:37-116 without auto-augment / motion shift /
 * erasing): uint8 frames [B][T][H][W][C] -> f32 [B][C][T][S][S] = normalize(hflip(bilinear resize
 * (crop))). params int32 [B][5] = (top, left, height, width, flip) from the host's draws (the
 * reference's RNG order, video/transforms.py:470-507, :149-180); mean / stdv f32 [C] in uint8
 * units (255 x the config's values). Replaces random_resized_crop + horizontal_flip +
 * _tensor_normalize_inplace. */
int vj_video_transform(int B, int T, int H, int W, int C, int S, const void* frames, const int* params,
                       const float* mean, const float* stdv, float* out, void* stream);

/* Cross-attention of nq learned queries over N tokens (frozen-encoder probe: CrossAttention.forward,
 * src/models/utils/modules.py:577-594 = F.scaled_dot_product_attention(q, k, v) with q [B, H, nq, hd],
 * k / v [B, H, N, hd]; used by CrossAttentionBlock :606-610 and AttentivePooler attentive_pooler.py:91-100).
 * q bf16 [B*nq][ldq] (head h at column h*hd), kv bf16 [B*N][ldkv] (k at h*hd, v at H*hd + h*hd: the
 * reference's kv Linear output reshaped (B, N, 2, H, hd)), o bf16 [B*nq][ldo]; lse2 f32 [B*H][nq] =
 * log2-domain log-sum-exp of scale*log2(e)*q.k, kept for the backward. hd % 8 == 0, hd <= 128.
 * ws: f32 workspace of vj_xattn_ws_floats() floats (split-KV partials, 64 keys per chunk). */
int vj_xattn_ws_floats(int B, int nq, int N, int H, int hd, long* out);
int vj_xattn_fwd(int B, int nq, int N, int H, int hd, const void* q, long ldq, const void* kv, long ldkv, void* o,
                 long ldo, float* lse2, float scale, float* ws, long ws_floats, void* stream);
/* SDPA backward of vj_xattn_fwd: dq bf16 [B*nq][lddq], dkv bf16 [B*N][lddkv] (dk | dv, same layout as
 * kv, every element written). Deterministic: dq's cross-chunk sum and, for nq > 16, the dk / dv sum over
 * query blocks (f32, in the workspace vj_xattn_ws_floats sizes) are fixed-order. */
int vj_xattn_bwd(int B, int nq, int N, int H, int hd, const void* q, long ldq, const void* kv, long ldkv,
                 const void* o, long ldo, const void* dout, long lddo, const float* lse2, float scale, void* dq,
                 long lddq, void* dkv, long lddkv, float* ws, long ws_floats, void* stream);

/* fp32-operand parity mode (vj_f32.hip): the encoder forward with f32 operands throughout, to show
 * the bf16 path's distance from the fp32 reference is operand rounding only. Not on the training
 * path. vj_gemm_f32: C = A B^T + bias (+ resid), epi as vj_gemm_bf16 (F32 = 1, F32_RESID = 2,
 * GELU = 3: C = pre-activation, C2 = GELU) on v_mfma_f32_32x32x2_f32 (replaces the f32 math of
 * nn.Linear, modules.py:77-83 / 330 / 372). vj_attn_fwd_f32: exact-softmax attention on an f32 qkv
 * buffer (F.scaled_dot_product_attention, modules.py:367-372); lse in natural log. vj_rope_f32 /
 * vj_im2col_tubelet_f32: vj_rope / vj_im2col_tubelet on f32 rows. */
int vj_gemm_f32(int M, int N, int K, const float* A, long lda, const float* B, long ldb, int epi, const float* bias,
                const float* resid, long ldr, float* C, long ldc, float* C2, long ldc2, void* stream);
int vj_attn_fwd_f32(int T, int H, int hd, const float* qkv, long ld, int q_off, int k_off, int v_off, float* o,
                    long ldo, float* lse, float scale, int ngroups, const int* nseq, const int* len, void* stream);
int vj_rope_f32(int T, int H, int hd, float* qkv, long ld, int q_off, int k_off, const int* ids, int ids_mod,
                int tokens_per_frame, int tokens_per_row, const float* cos_tab, const float* sin_tab, int half,
                void* stream);
int vj_im2col_tubelet_f32(int R, int K, const long* idx, int B, int C, int Tf, int Hf, int Wf, int tub, int pch,
                          const float* clip, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VJEPA_HIP_H */
