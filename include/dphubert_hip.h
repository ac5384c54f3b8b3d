/*
 * dphubert_hip.h — C ABI of the MI355X (gfx950) DPHuBERT distill-step kernels.
 *
 * The reference (seas2nada/DPHuBERT) has no FFI: its boundary is the Python
 * module API.  Every entry point below replaces the ATen /
 * cuDNN / cuBLAS work behind one reference call site, cited per function.
 * The Python host mirror (dphubert_amd/_lib.py, ctypes) binds these symbols;
 * INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - plain pointers + sizes, no torch types; all buffers (incl. workspace) are
 *     caller-owned device memory; nothing here allocates;
 *   - every call is stream-ordered on the hipStream_t it is given and
 *     re-entrant (no mutable global state);
 *   - bf16 tensors are raw 16-bit storage (uint16_t), row-major;
 *   - return 0 on success or a negative DPH_E* code; dph_last_error() gives a
 *     thread-local message for the last failure on the calling thread.
 */
#ifndef DPHUBERT_HIP_H
#define DPHUBERT_HIP_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPH_OK 0
#define DPH_EINVAL (-1)
#define DPH_ELAUNCH (-2)
#define DPH_EUNSUPPORTED (-3)

const char* dph_last_error(void);
int dph_abi_version(void);

/* Deterministic mode (process-wide, read at launch time; initial value from the environment variable
 * DPH_DETERMINISTIC, default on): every reduction of float partials across blocks -- bias / LayerNorm-affine
 * column sums, mask gradients, conv0 GroupNorm sums, head-mask sums, WavLM relative-position sums -- writes
 * per-block partials to its workspace and sums them in a fixed order, so repeated runs of a step (eager or a
 * HIP-graph replay) produce bitwise identical gradients (the reproducibility contract of the reference's
 * pl.seed_everything, distill.py:30).  Off: same-address float atomics (last-bit run-to-run noise).  A captured
 * graph keeps the kernels it recorded: set the mode before capturing.  The entry points that take a workspace
 * size it with their *_workspace function for either mode. */
int dph_set_deterministic(int on);
int dph_get_deterministic(void);

/* Deferred column reductions (deterministic mode only; ABI 21).  Between dph_defer_reductions(1) and
 * dph_defer_reductions(0), the fixed-order partial-slab column sums that dph_layernorm_bwd*, dph_colsum /
 * dph_colsum3, the rowblock reductions and dph_gemm's column-sum epilogues would launch as their own small grid
 * are queued instead; dph_flush_reductions launches the queue as one grid per 96 problems, each problem summed
 * in the same fixed order as its own launch (bitwise identical results).  The caller keeps every queued
 * workspace alive and the queued outputs unread until the flush, which must be issued on the stream the
 * reductions were queued on.  Queued problems whose outputs overlap are flushed in queue order (an overlapping
 * enqueue flushes the queue first).  dph_deferred_reductions: the queue length.
 * ABI 23: dph_discard_reductions drops the queue without launching it (the error path of a deferred block, whose
 * slabs may already be freed) and returns how many were dropped; dph_reductions_pushed counts every problem ever
 * queued (a caller keeps a call's slab alive only when that call queued something). */
int dph_defer_reductions(int on);
int dph_flush_reductions(hipStream_t stream);
int64_t dph_deferred_reductions(void);
int64_t dph_discard_reductions(void);
int64_t dph_reductions_pushed(void);

/* ------------------------------------------------------------------------ *
 * Generic bf16 MFMA GEMM with fused epilogues.
 *   C[z][m][n] = epi( alpha * sum_k A[z][m][k] * B[z][k][n] )
 * Replaces every nn.Linear / conv1d matmul of the hot path (fwd, dgrad,
 * wgrad): components.py:107 (conv1..6 as implicit GEMM over channels-last
 * activations), :272 (feature projection), :328 (grouped pos-conv as a
 * batched GEMM), :406-408/:430 (QKV, out_proj), :733/:741 (FFN),
 * lightning.py:258 (distill projections).
 * ------------------------------------------------------------------------ */
typedef struct DphMat {
  void* ptr;
  /* address of row r (elements): rpb > 0 ? (r/rpb)*batch_stride + (r%rpb)*row_stride
   *                                       : r*row_stride                          */
  int64_t rows_per_batch;
  int64_t batch_stride;
  int64_t row_stride;
  /* offset of grid batch z: z_div > 0 ? (z/z_div)*z_outer + (z%z_div)*z_inner : z*z_inner */
  int64_t z_div;
  int64_t z_outer;
  int64_t z_inner;
} DphMat;

#define DPH_ACT_NONE 0
#define DPH_ACT_GELU 1      /* v = gelu(v), optional pre-activation store        */
#define DPH_ACT_GELU_BWD 2  /* v = v*drop*colmask*gelu'(aux); colsum_aux += v*drop*gelu(aux) */
/* GELU backward from what the forward stored: aux_in = the forward's pre_out under DPH_GEMM_PRE_DGK
 * (gelu'(pre)*colmask*keep/(1-p)), residual = the forward's output f (gelu(pre)*colmask*keep/(1-p)):
 * v = v*aux; colsum_aux += v*residual/colmask (0 where colmask == 0); colsum_out += stored v.
 * residual may be NULL (then colsum_aux gets zeros): the mask gradient comes from dph_colprod over the FFN2
 * weight gradient instead, and this epilogue reads one input less.
 * No dropout / smask arguments (they are folded into aux).  Ping-pong layouts only (dph_gemm checks). */
#define DPH_ACT_GELU_BWD_DGK 3

#define DPH_OUT_BF16 0
#define DPH_OUT_F32 1
#define DPH_OUT_F32_ACCUM 2

typedef struct DphGemmArgs {
  int64_t M, N, K;
  int32_t batch;      /* grid batches (z)                                    */
  int32_t splits;     /* split-K factor; >1 needs workspace M*N*splits*batch fp32 */
  int32_t a_kcontig;  /* 1: A is [M][K] (k contiguous); 0: A is [K][M]         */
  int32_t b_kcontig;  /* 1: B is [N][K] (k contiguous); 0: B is [K][N]         */
  DphMat A, B, C;     /* C layout is shared by pre_out / aux_in / residual     */
  int32_t c_dtype;    /* DPH_OUT_*                                            */
  int32_t act;        /* DPH_ACT_*                                            */
  float alpha;
  float dropout_p;
  uint64_t seed;
  const float* bias;      /* [N], added after alpha                          */
  const float* colmask;   /* [N], multiplies after the activation             */
  const float* smask;     /* scalar device pointer (layer mask)               */
  int64_t vec_z_inner;    /* per-batch offset of bias/colmask/colsum vectors = (z % C.z_div)*vec_z_inner */
  void* pre_out;          /* bf16, pre-activation (after bias)                */
  const void* aux_in;     /* bf16, GELU_BWD pre-activation input              */
  const void* residual;   /* bf16, added last                                 */
  float* colsum_out;      /* [N] += column sums of the stored value              */
  float* colsum_aux;      /* [N] += GELU_BWD mask gradient                        */
  const int64_t* row_len; /* zero rows with (m % len_rows) >= row_len[m / len_rows] */
  int64_t len_rows;
  int64_t drop_row_offset;/* dropout element index = (drop_row_offset + m)*N + n (per batch z adds z*M*N) */
  void* workspace;        /* split-K partials; with column sums (batch 1): >= 2*ceil(M/64)*N fp32 of
                           * per-tile partial rows, summed after the GEMM (required in deterministic mode) */
  int64_t workspace_bytes;
  int64_t colsum_n;       /* column sums only for n < colsum_n (0: all N); padded-width operands */
  int64_t flags;          /* DPH_GEMM_* bits below                                */
  /* device-side extents {m, n, k} (int32, <= 0: the static M / N / K): blocks past m / n return at once, the
   * K loop stops at k (a multiple of 64, >= 128, with zero operand columns up to it).  The FFN GEMMs over the
   * packed active units (dph_ffn_compact) read the active count this way inside a captured step graph.
   * Ping-pong kernels only (pp_gemm_kernel: m / n / k, ppw_gemm_kernel: m / n); NULL = static.            */
  const int32_t* dyn_ext;
  /* stream-K scratch (ABI 23; sized by dph_gemm_sk_plan): sk_ws = fp32 partial tiles (sk_ws_bytes), sk_flags =
   * sk_nflags int32 hand-off flags that must be ZERO at launch (the library never resets them: give each call
   * fresh zeros).  NULL sk_ws: the stream-K kernel is not used for this call.                              */
  void* sk_ws;
  int64_t sk_ws_bytes;
  int32_t* sk_flags;
  int64_t sk_nflags;
} DphGemmArgs;

/* flags: one tile per block even where the persistent ring grid applies -- for GEMMs that share the
 * GPU with another stream's kernels (the teacher forward runs concurrently with the student forward):
 * a persistent grid sized to the CUs stalls on the CUs the other kernels hold, a tile grid rebalances */
#define DPH_GEMM_NO_PERSIST 1
/* DPH_ACT_GELU with pre_out: store gelu'(pre)*colmask*keep/(1-p) instead of pre (the aux input of the
 * matching DPH_ACT_GELU_BWD_DGK input-gradient GEMM).  Ping-pong layouts only. */
#define DPH_GEMM_PRE_DGK 2
/* residual is fp32 (same element layout as C): the pre-norm residual stream x + f(LN(x)) carried in fp32 across
 * the layers (components.py:846, :850), whose 2 x L bf16 roundings would otherwise accumulate.  Forward epilogues
 * only (not with DPH_ACT_GELU_BWD / _DGK). */
#define DPH_GEMM_RESID_F32 4

int dph_gemm(const DphGemmArgs* args, hipStream_t stream);
/* Stream-K route (ABI 23): 1 when dph_gemm would run these args (sk_* fields ignored) on the persistent stream-K
 * 256 x 256 ping-pong kernel -- the M = B*T projections with N >= 2048 (QKV forward, FFN1 forward, FFN2 input
 * gradient: components.py:406-408, :733-741) -- and then the partial-tile bytes and zeroed flags it needs; 0 otherwise
 * (off unless DPH_GEMM_SK=1 / all: measured slower than the tile kernels on the step's shapes, gemm_sk.hip). */
int dph_gemm_sk_plan(const DphGemmArgs* args, int64_t* ws_bytes, int64_t* nflags);
/* Grouped (mn, mn) weight gradients: n <= DPH_GEMM_GROUP_MAX independent dW_i (+)= dY_i^T X_i of ONE shape in one
 * launch (grid batch z = problem i, operand i at a[i] / b[i] / c[i]).  ``args`` describes every problem: batch == n,
 * splits = dph_gemm_mn_plan(M, N, K, n) with the workspace sized for n problems, A / B / C ptr ignored, their
 * z offsets 0.  The per-layer weight-gradient GEMMs of the encoder layers (components.py:406-408, :430, :733,
 * :741), deferred over a group of layers: the group fills the CUs without (or with fewer) split-K slices.
 * DPH_EUNSUPPORTED when the layout / alignment is outside the ping-pong weight-gradient kernel (the caller then
 * runs the problems one dph_gemm at a time). */
#define DPH_GEMM_GROUP_MAX 16
typedef struct DphGemmGroup {
  int32_t n;
  int32_t reserved;
  const void* a[DPH_GEMM_GROUP_MAX];
  const void* b[DPH_GEMM_GROUP_MAX];
  void* c[DPH_GEMM_GROUP_MAX];
} DphGemmGroup;
int dph_gemm_grouped(const DphGemmArgs* args, const DphGemmGroup* group, hipStream_t stream);
/* name (as it appears in rocprof kernel names) of the kernel dph_gemm launches for these args */
const char* dph_gemm_variant(const DphGemmArgs* args);
/* split-K factor of the ping-pong weight-gradient plan for an (mn, mn) GEMM of this shape (A = [K][M], B = [K][N]:
 * dW = dY^T X, K = frames of the batch); 0 = no plan.  A dph_gemm with exactly these splits (workspace sized for
 * them) and an eligible layout runs ppw_gemm_kernel + splitk_reduce; replaces the split heuristic of the
 * register-staged kernel for the wgrads of components.py:107/:272/:406-408/:430/:733/:741, lightning.py:258 */
int dph_gemm_mn_plan(int64_t M, int64_t N, int64_t K, int64_t batch);

/* ------------------------------------------------------------------------ *
 * FFN units with an exactly-zero HardConcrete mask (hardconcrete.py:99; components.py:733-741): the layer's FFN
 * GEMMs run over the active units packed to the front of Fc-wide images (Fc % 64 == 0, Fc >= max(F, 128)).
 * dph_ffn_compact: idx[Fc] = the active units in order (-1 past them), ext[10] = three {m, n, k} dyn_ext
 * triplets (N, K, M dynamic = keff = max(128, active count rounded up to 64)) and the active count.
 * Gathers pack W1 rows / W2 columns / vectors by idx (zero past the active count); scatters add the packed
 * gradients back to the full-width ones (accumulate = 1) or overwrite their active entries (0).
 * ------------------------------------------------------------------------ */
int dph_ffn_compact(const float* mask, int64_t F, int64_t Fc, int32_t* idx, int32_t* ext, hipStream_t stream);
int dph_gather_rows_bf16(const void* src, int64_t ld_src, const int32_t* idx, void* dst, int64_t rows, int64_t cols,
                         hipStream_t stream);
int dph_gather_cols_bf16(const void* src, int64_t ld_src, const int32_t* idx, void* dst, int64_t rows, int64_t Fc,
                         hipStream_t stream);
int dph_gather_vec_f32(const float* src, const int32_t* idx, float* dst, int64_t Fc, hipStream_t stream);
int dph_scatter_rows_f32(const float* src, const int32_t* idx, float* dst, int64_t ld_dst, int64_t rows, int64_t cols,
                         int accumulate, hipStream_t stream);
int dph_scatter_cols_f32(const float* src, const int32_t* idx, float* dst, int64_t ld_dst, int64_t rows, int64_t Fc,
                         int accumulate, hipStream_t stream);
/* one launch for every packed FFN operand of a layer (forward and backward GEMMs): W1 rows, W2 columns, the rows
 * of W2^T and the columns of W1^T (w2t / w1t may be NULL: then w2gt / w1gt are not written), b1 (may be NULL:
 * zeros) and mask; and one launch adding the packed gradients back: dW2 columns (row stride ld2), dW1 rows, db1,
 * dmask (db1 / dm may be NULL) */
int dph_ffn_pack(const void* w1, const void* w2, const void* w2t, const void* w1t, const float* b1, const float* mask,
                 const int32_t* idx, void* w1g, void* w2g, void* w2gt, void* w1gt, float* b1g, float* mg, int64_t Fp,
                 int64_t Fc, int64_t D, hipStream_t stream);
int dph_ffn_unpack_grads(const float* dw2g, const float* dw1g, const float* db1g, const float* dmg, const int32_t* idx,
                         float* dw2, int64_t ld2, float* dw1, float* db1, float* dm, int64_t Fc, int64_t D,
                         hipStream_t stream);

/* ------------------------------------------------------------------------ *
 * LayerNorm over the last dim (rows x D), fp32 statistics, eps=1e-5.
 * components.py:271, :853, :856, :889 (nn.LayerNorm), :54-61.
 * y = (x*xscale - mean)*rstd*gamma + beta, then optional dropout.
 * ------------------------------------------------------------------------ */
int dph_layernorm_fwd(const void* x, const float* xscale, const float* gamma, const float* beta, void* y,
                      float* mean, float* rstd, int64_t rows, int64_t D, float eps, float dropout_p,
                      uint64_t seed, hipStream_t stream);
/* fused LayerNorm + exact GELU + channel mask (layer_norm-mode conv layers, components.py:54-61,
 * :110-114): y = GELU(LN(x)) * mask[c] computed from the fp32 LN value; h (may be NULL) receives
 * the bf16 LN output for the GELU backward; x is bf16, or fp32 when x_f32.  D % 4 == 0. */
int dph_layernorm_gelu_fwd(const void* x, int x_f32, const float* gamma, const float* beta, void* h, const float* mask,
                           void* y, float* mean, float* rstd, int64_t rows, int64_t D, float eps, hipStream_t stream);
/* LN backward with an fp32 input x (the fp32 pre-LN conv outputs of layer_norm-mode extractors);
 * dy / dx bf16, dgamma / dbeta accumulate */
int dph_layernorm_bwd_x32(const void* dy, const float* x, const float* gamma, const float* mean, const float* rstd,
                          void* dx, float* dgamma, float* dbeta, int64_t rows, int64_t D, float* ws, int64_t ws_bytes,
                          hipStream_t stream);
/* dx = LN backward; dgamma/dbeta accumulate (atomics).  Optional branch output
 * (residual sub-branch gradient): branch = dx * drop(branch_p, branch_seed) * (*branch_smask),
 * branch_colsum += column sums of branch, branch_sdot += sum(dx*drop*branch_pre).
 * dx_add (optional) is added to dx (other gradient contributions of the LN input). */
int dph_layernorm_bwd(const void* dy, const void* x, const float* xscale, const float* gamma, const float* mean,
                      const float* rstd, void* dx, float* dgamma, float* dbeta, int64_t rows, int64_t D,
                      float dropout_p, uint64_t seed, void* branch, float branch_p, uint64_t branch_seed,
                      const float* branch_smask, float* branch_colsum, const void* branch_pre,
                      float* branch_sdot, float* ws, int64_t ws_bytes, hipStream_t stream);
/* workspace (bytes) of dph_layernorm_bwd(_ld): per-block column-partial slab, reduced by a second
 * kernel (same-address atomics from hundreds of blocks serialise at the memory side), + the per-block
 * branch_sdot partials of deterministic mode */
int64_t dph_layernorm_bwd_workspace(int64_t rows, int64_t D);

/* the same over rows of stride ld >= D (ld % 4 == 0): columns [D, ld) are row padding (pruned
 * students' channel counts padded to multiples of 8), read as 0 and written as 0 */
int dph_layernorm_fwd_ld(const void* x, const float* xscale, const float* gamma, const float* beta, void* y,
                         float* mean, float* rstd, int64_t rows, int64_t D, int64_t ld, float eps, float dropout_p,
                         uint64_t seed, hipStream_t stream);
/* dx_add (optional, bf16 with the same stride): added to dx -- the pre-norm residual path
 * (components.py:835-850: x + f(LN(x))); the branch output stays the LN-path gradient */
int dph_layernorm_bwd_ld(const void* dy, const void* x, const float* xscale, const float* gamma, const float* mean,
                         const float* rstd, void* dx, float* dgamma, float* dbeta, int64_t rows, int64_t D, int64_t ld,
                         float dropout_p, uint64_t seed, void* branch, float branch_p, uint64_t branch_seed,
                         const float* branch_smask, float* branch_colsum, const void* branch_pre, float* branch_sdot,
                         const void* dx_add, float* ws, int64_t ws_bytes, hipStream_t stream);
/* pre-norm residual stream in fp32 (components.py:835-850: x + attn(LN(x)), x + FFN(LN(x)) carried across the layers
 * without a bf16 rounding per add): LN forward of an fp32 x (y bf16: the next GEMM's operand), and the LN backward
 * whose input gradient is the fp32 stream's: dx (fp32) = LN backward of dy (bf16) + dx_add (fp32, optional: the
 * residual path's gradient); dgamma / dbeta accumulate (ws: dph_layernorm_bwd_workspace bytes). */
int dph_layernorm_fwd_x32(const float* x, const float* gamma, const float* beta, void* y, float* mean, float* rstd,
                          int64_t rows, int64_t D, float eps, hipStream_t stream);
int dph_layernorm_bwd_res32(const void* dy, const float* x, const float* gamma, const float* mean, const float* rstd,
                            float* dx, float* dgamma, float* dbeta, int64_t rows, int64_t D, const float* dx_add,
                            float* ws, int64_t ws_bytes, hipStream_t stream);
/* per-utterance waveform LayerNorm, model.py:96-103 (normalize_waveform, wav2vec2-Large):
 * y[b][:len_b] = (x - mean) / sqrt(var + eps) over the first len_b samples, y[b][len_b:] = 0
 * (lengths == NULL: full rows) */
int dph_wave_layernorm(const float* x, const int64_t* lengths, int64_t B, int64_t S, float eps, float* y,
                       hipStream_t stream);

/* out[n] += s(n) * sum_r a[r][n] * b[r][n], s(n) = 1/colmask[n] (0 where colmask[n] == 0; colmask NULL: 1), for
 * a bf16 [R][lda] and b fp32 [R][ldb], n < N.  The FFN intermediate-mask gradient from the FFN2 weight gradient
 * (components.py:733-741): d loss/d mask_n = sum_o W2[o][n] dW2[o][n] / mask_n, dW2 = dY^T f of this micro-batch --
 * the contraction the FFN2 input-gradient epilogue otherwise evaluates by re-reading f */
int dph_colprod(const void* a, int64_t lda, const float* b, int64_t ldb, const float* colmask, float* out, int64_t R,
                int64_t N, hipStream_t stream);
/* column sums of a bf16 matrix (bias gradients): out[n] += sum_m x[m][n]; ws: per-row-block partial
 * slab of dph_colsum_workspace(rows, cols) bytes */
int dph_colsum(const void* x, float* out, int64_t rows, int64_t cols, float* ws, int64_t ws_bytes, hipStream_t stream);
int64_t dph_colsum_workspace(int64_t rows, int64_t cols);
/* the same over a [rows][3*seg] matrix into three segment outputs out0/out1/out2 (+=; a NULL output skips its
 * segment; ws: dph_colsum_workspace(rows, 3*seg) bytes).  q/k/v bias gradients (components.py:406-408): the k
 * segment is skipped, its gradient is exactly zero by softmax shift invariance (components.py:411-417) */
int dph_colsum3(const void* x, float* out0, float* out1, float* out2, int64_t rows, int64_t seg, float* ws,
                int64_t ws_bytes, hipStream_t stream);

/* ------------------------------------------------------------------------ *
 * Fused multi-head self-attention (flash style), head dim 64.
 * components.py:405-426: q,k,v read from the fused QKV buffer
 * [B*T][3*H*64] (q | k | v), scores (scale*q)k^T + (-1e4 key padding),
 * softmax, dropout(p), @v, x head_mask.  Writes o_unmasked ([B*T][H*64] fp32:
 * the backward's D = rowsum(dO*O) must cancel sum_j P_j dP_j to fp32 accuracy), o_masked
 * ([B*T][H*64] bf16, the out_proj input) and the per-row log-sum-exp [B][H][T].  o_unmasked and lse may be
 * NULL (a forward without backward: the teacher) -- not written then.
 * ------------------------------------------------------------------------ */
int dph_attention_fwd(const void* qkv, void* o_unmasked, void* o_masked, float* lse, const float* head_mask,
                      const int64_t* key_len, int64_t B, int64_t T, int64_t H, float scale, float dropout_p,
                      uint64_t seed, void* keep_bits, hipStream_t stream);
/* keep_bits (dropout_p > 0, optional, 8-B aligned, dph_attention_keep_bytes(B, T, H) bytes): the forward
 * stores its dropout keep decisions (1 bit per probability, uint16 per (row, 64-key tile, lane group)) and
 * the backward reads them instead of re-hashing (NULL on both sides: regenerated from (seed, element)) */
int64_t dph_attention_keep_bytes(int64_t B, int64_t T, int64_t H);
/* backward prep: D[b][h][t] = rowdot = sum_d do_m*o_u (o_u fp32) ; dhead_mask[h] += sum rowdot.
 * (ABI 22: D is the rowdot of do_m itself -- dph_attention_bwd forms dP and dS from do_m and applies head_mask
 * to dq / dk / dv in fp32 -- where ABI <= 21 took the rowdot of bf16(head_mask * do_m).)  ws (deterministic mode with dhead_mask): the per-row-block head sums,
 * dph_attention_bwd_prep_workspace(B, T, H) bytes (may be NULL otherwise) */
int64_t dph_attention_bwd_prep_workspace(int64_t B, int64_t T, int64_t H);
int dph_attention_bwd_prep(const void* do_masked, const void* o_unmasked, const float* head_mask, float* Dvec,
                           float* dhead_mask, int64_t B, int64_t T, int64_t H, float* ws, int64_t ws_bytes,
                           hipStream_t stream);
/* dq|dk|dv into dqkv [B*T][3*H*64] (bf16) */
int dph_attention_bwd(const void* qkv, const void* do_masked, const float* head_mask, const float* lse,
                      const float* Dvec, void* dqkv, const int64_t* key_len, int64_t B, int64_t T, int64_t H,
                      float scale, float dropout_p, uint64_t seed, const void* keep_bits, hipStream_t stream);
/* ABI 24: dph_attention_bwd plus the q_proj / v_proj bias gradients (replaces the reference's autograd column sums
 * of the q / v projection output gradients: components.py:365-366 v_proj / q_proj, nn.Linear(bias=True)):
 * dbq[H*64], dbv[H*64] (ACCUMULATED) += the column sums of dQ / dV in fp32 (before dqkv's bf16 rounding; padded keys
 * < T included as in dqkv, rows >= T excluded), summed by each backward wave over its 32 rows in a fixed order into
 * ws (16-B aligned, dph_attention_bwd_qv_workspace(B, T, H) bytes = one [q | v] fp32 row per wave) and reduced
 * over the rows in order (inside a dph_defer_reductions block: queued).  The k_proj bias gradient is exactly zero
 * (softmax shift invariance) and is not produced. */
int64_t dph_attention_bwd_qv_workspace(int64_t B, int64_t T, int64_t H);
int dph_attention_bwd_qv(const void* qkv, const void* do_masked, const float* head_mask, const float* lse,
                         const float* Dvec, void* dqkv, const int64_t* key_len, int64_t B, int64_t T, int64_t H,
                         float scale, float dropout_p, uint64_t seed, const void* keep_bits, float* dbq, float* dbv,
                         float* ws, int64_t ws_bytes, hipStream_t stream);

/* ------------------------------------------------------------------------ *
 * WavLM gated relative-position bias (WavLMSelfAttention, components.py:486-659).
 * The reference builds position_bias (B*H,T,T) = Embedding(bucket(k-q)) in
 * layer 0 (compute_bias :546-561, _relative_positions_bucket :563-600), passes
 * it to every layer, multiplies it per layer by the gate of :637-644 and adds
 * it to the scores (:649-651 -> SelfAttention :413).  Here no T x T tensor
 * exists: rel_tab [H][2T-1] fp32 is one value per diagonal r = k-q+T-1 for each
 * remaining head, gate [B][H][T] fp32 one value per query row.
 * ------------------------------------------------------------------------ */
/* attention forward with score += gate[b,h,q] * rel_tab[h][k-q+T-1] (T <= 3584) */
int dph_attention_fwd_relpos(const void* qkv, void* o_unmasked, void* o_masked, float* lse, const float* head_mask,
                             const int64_t* key_len, const float* rel_tab, const float* gate, int64_t B, int64_t T,
                             int64_t H, float scale, float dropout_p, uint64_t seed, void* keep_bits,
                             hipStream_t stream);
/* its backward: dqkv as dph_attention_bwd, plus dgate [B][H][T] (written) = sum_k dS*rel_tab and
 * drel_tab [H][2T-1] (ACCUMULATED, zero it first) = diagonal sums of dS*gate.  ws (deterministic mode): the
 * per-query-block diagonal sums, dph_attention_bwd_relpos_workspace(B, T, H) bytes (may be NULL otherwise) */
int64_t dph_attention_bwd_relpos_workspace(int64_t B, int64_t T, int64_t H);
int dph_attention_bwd_relpos(const void* qkv, const void* do_masked, const float* head_mask, const float* lse,
                             const float* Dvec, void* dqkv, const int64_t* key_len, const float* rel_tab,
                             const float* gate, float* dgate, float* drel_tab, int64_t B, int64_t T, int64_t H,
                             float scale, float dropout_p, uint64_t seed, const void* keep_bits, float* ws,
                             int64_t ws_bytes, hipStream_t stream);
/* ABI 24: dph_attention_bwd_relpos plus dbq / dbv as dph_attention_bwd_qv (bws: its workspace) */
int dph_attention_bwd_relpos_qv(const void* qkv, const void* do_masked, const float* head_mask, const float* lse,
                                const float* Dvec, void* dqkv, const int64_t* key_len, const float* rel_tab,
                                const float* gate, float* dgate, float* drel_tab, int64_t B, int64_t T, int64_t H,
                                float scale, float dropout_p, uint64_t seed, const void* keep_bits, float* ws,
                                int64_t ws_bytes, float* dbq, float* dbv, float* bws, int64_t bws_bytes,
                                hipStream_t stream);
/* rel_tab[h][r] = embed[bucket(r-(T-1))][heads[h]] (embed [num_buckets][Htot] fp32; heads [H] int64 or NULL =
 * identity); buckets [2T-1] int64 (optional) receives the bucket index table; either output may be NULL */
int dph_relpos_table(const float* embed, const int64_t* heads, float* rel_tab, int64_t* buckets, int64_t T,
                     int64_t H, int64_t Htot, int64_t num_buckets, int64_t max_distance, hipStream_t stream);
/* dembed[bucket][heads[h]] += drel_tab[h][r] (the Embedding backward) */
int dph_relpos_table_bwd(const float* drel_tab, const int64_t* heads, float* dembed, int64_t T, int64_t H,
                         int64_t Htot, int64_t num_buckets, int64_t max_distance, hipStream_t stream);
/* gate[b][h][t] = ga*(gb*gconst[hh]-1)+2, (ga, gb) = sigmoid of the 2 group sums of Linear(64, 8)(x[b,t,hh*64:+64])
 * (components.py:637-643; x bf16 [B*T][ldx], hh = heads[h]) */
int dph_wavlm_gate_fwd(const void* x, int64_t ldx, const float* w, const float* bias, const float* gconst,
                       const int64_t* heads, float* gate, int64_t B, int64_t T, int64_t H, int64_t head_dim,
                       hipStream_t stream);
/* its backward: dx (bf16, ld lddx) += the gate's input gradient; dw [8][64], db [8], dconst [Htot] ACCUMULATE;
 * ws: dph_wavlm_gate_bwd_workspace(B, T, H) bytes */
int64_t dph_wavlm_gate_bwd_workspace(int64_t B, int64_t T, int64_t H);
int dph_wavlm_gate_bwd(const void* x, int64_t ldx, const float* w, const float* bias, const float* gconst,
                       const int64_t* heads, const float* dgate, void* dx, int64_t lddx, float* dw, float* db,
                       float* dconst, float* ws, int64_t ws_bytes, int64_t B, int64_t T, int64_t H, int64_t head_dim,
                       hipStream_t stream);

/* ------------------------------------------------------------------------ *
 * Conv frontend (FeatureExtractor, components.py:94-120, 158-185,
 * 1071-1076): conv0 (1 -> C, kernel k0, stride s0, no bias) + GroupNorm(C,C)
 * + GELU + HardConcrete channel mask, output channels-last bf16 [B][L][C].
 * ------------------------------------------------------------------------ */
/* mean / rstd [B][C]: the GroupNorm statistics, computed in closed form from the waveform's per-utterance tap
 * sums and Gram matrix (fp64); ws: >= B * 16 * 65 * 8 bytes (per-chunk Gram partials) */
int dph_conv0_gn_fwd(const float* wave, int64_t B, int64_t S, const float* w, int64_t C, int64_t k0, int64_t s0,
                     const float* gamma, const float* beta, const float* mask, void* y, float* mean, float* rstd,
                     float* ws, int64_t ws_bytes, hipStream_t stream);
/* backward scratch: per-(b,c) partial sums (fp32) + per-utterance waveform Gram matrix (fp64) + (deterministic
 * mode) the per-(utterance, time block) partials, reduced in block order */
int64_t dph_conv0_gn_bwd_workspace(int64_t B, int64_t S, int64_t C);
int dph_conv0_gn_bwd(const float* wave, int64_t B, int64_t S, const float* w, int64_t C, int64_t k0, int64_t s0,
                     const float* gamma, const float* beta, const float* mask, const float* mean, const float* rstd,
                     const void* dy, float* dw, float* dgamma, float* dbeta, float* dmask, float* ws,
                     int64_t ws_bytes, hipStream_t stream);
/* plain conv0 (no norm, used by layer_norm-mode extractors): y[b][t][c] = sum_j w[c][j]*x[b][s0*t+j] (+bias) */
int dph_conv0_fwd(const float* wave, int64_t B, int64_t S, const float* w, const float* bias, int64_t C,
                  int64_t k0, int64_t s0, void* y, hipStream_t stream);

/* its backward (dz = gradient of the conv0 output, LN/GELU/mask backward already applied):
 * dw[c][j] += sum dz[b][t][c] * x[b][s0*t+j], dbias[c] += sum dz (dbias may be NULL); accumulates.
 * ws (deterministic mode): dph_conv0_bwd_workspace(B, S, C) bytes of per-(utterance, time block) partials */
int64_t dph_conv0_bwd_workspace(int64_t B, int64_t S, int64_t C);
int dph_conv0_bwd(const float* wave, int64_t B, int64_t S, int64_t C, int64_t k0, int64_t s0, const void* dz,
                  float* dw, float* dbias, float* ws, int64_t ws_bytes, hipStream_t stream);
/* y = GELU(h) * mask[c] on a dense bf16 [rows][C] tensor (C % 8 == 0; mask may be NULL):
 * layer_norm-mode conv layers after their LayerNorm (components.py:110-114) */
int dph_gelu_mask_fwd(const void* h, const float* mask, void* y, int64_t rows, int64_t C, hipStream_t stream);

/* Fused col2im + GELU/mask backward for a strided conv layer (k, s):
 * dy_in[b][t'][c] = sum_{t,j: s*t+j==t'} dcols[b][t][j*C+c]; then, if z_pre != NULL,
 * out = dy_in*mask[c]*gelu'(z_pre), dmask[c] += dy_in*gelu(z_pre); else out = dy_in.
 * ws (deterministic mode with dmask): dph_rowblock_workspace(B * Lin, C) bytes (may be NULL otherwise) */
int dph_col2im_gelu_bwd(const void* dcols, int64_t B, int64_t Lout, int64_t Lin, int64_t C, int64_t k, int64_t s,
                        const void* z_pre, const float* mask, void* out, float* dmask, float* ws, int64_t ws_bytes,
                        hipStream_t stream);
/* GELU/mask backward on a dense [rows][C] tensor (no col2im); ws as above: dph_rowblock_workspace(rows, C) */
int dph_gelu_mask_bwd(const void* dy, const void* z_pre, const float* mask, void* out, float* dmask, int64_t rows,
                      int64_t C, float* ws, int64_t ws_bytes, hipStream_t stream);
/* workspace (bytes) of the per-row-block column reductions (dph_col2im_gelu_bwd, dph_gelu_mask_bwd,
 * dph_branch_bwd(_f32)) in deterministic mode */
int64_t dph_rowblock_workspace(int64_t rows, int64_t cols);

/* pos-conv layout helpers: x [B][T][G*Cg] bf16 -> xg [B][G][pad_front + T + pad_back][Cg] zero-padded */
int dph_regroup_pad(const void* x, void* xg, int64_t B, int64_t T, int64_t G, int64_t Cg, int64_t pad_front,
                    int64_t pad_back, hipStream_t stream);
/* weight norm (dim=2): w = g*v/||v||_(dims 0,1) (deterministic reduction: workspace of
 * ceil(Cout*Cin_g/64)*K floats), also writes the bf16 GEMM images
 * wk [G][Cg_out][K*Cg_in] (k-major: index j*Cg_in+c) and its flipped transpose
 * wt [G][Cg_in][K*Cg_out] (index jj*Cg_out+o, jj=K-1-j) used by the input-gradient GEMM. */
int dph_weight_norm_fwd(const float* g, const float* v, int64_t Cout, int64_t Cin_g, int64_t K, int64_t G,
                        float* w, float* norm, void* wk, void* wt, float* ws, int64_t ws_bytes, hipStream_t stream);
/* dW_img [G][Cg_out][K*Cg_in] fp32 (GEMM layout) -> dg [K], dv [Cout][Cin_g][K] */
int dph_weight_norm_bwd(const float* dw_img, const float* g, const float* v, const float* norm, int64_t Cout,
                        int64_t Cin_g, int64_t K, int64_t G, float* dg, float* dv, float* ws, int64_t ws_bytes,
                        hipStream_t stream);

/* ------------------------------------------------------------------------ *
 * Casting / layout helpers for the bf16 GEMM images of fp32 master weights.
 * ------------------------------------------------------------------------ */
/* dst[r][c] = bf16(src[r][c] * (colscale ? colscale[c] : 1)) */
int dph_cast_bf16(const float* src, void* dst, int64_t n, hipStream_t stream);
/* bf16 [R][C] -> [C][R] (R, C multiples of 8): k-contiguous weight image W^T for input-gradient GEMMs */
int dph_transpose_bf16(const void* src, int64_t R, int64_t C, void* dst, hipStream_t stream);
/* batched refresh of the bf16 GEMM images after an optimizer step (replaces one dph_cast_bf16 /
 * dph_transpose_bf16 launch per weight): device tables of {src fp32*, dst bf16*, n} resp.
 * {src bf16*, dst bf16*, R, C} int64 entries (R, C multiples of 8) */
int dph_cast_bf16_multi(const int64_t* table, int64_t n_entries, hipStream_t stream);
/* batched fp32 copies / zero fills in one launch: device table of {src fp32* (0 = zeros), dst fp32*, n}
 * int64 entries, max_n >= every n (sizes the grid).  The q/k/v bias concatenations refreshed after an
 * optimizer step and the gradient buckets zeroed before a backward (replaces an ATen cat / fill each). */
int dph_copy_f32_multi(const int64_t* table, int64_t n_entries, int64_t max_n, hipStream_t stream);
/* frame lengths after the conv stack (components.py:179-181, every layer in one launch);
 * kernel_sizes / strides are HOST arrays of n_layers (<= 16) entries, read at call time */
int dph_conv_lengths(const int64_t* len_in, int64_t* len_out, int64_t n, int64_t n_layers,
                     const int32_t* kernel_sizes, const int32_t* strides, hipStream_t stream);
int dph_transpose_bf16_multi(const int64_t* table, int64_t n_entries, hipStream_t stream);
/* conv weight [O][C][k] fp32 -> bf16 [Op][k*Cp] (index j*Cp+c), zero for o >= O or c >= C
 * (channel counts of pruned students padded to multiples of 8) */
int dph_conv_weight_pack(const float* w, void* dst, int64_t O, int64_t C, int64_t k, int64_t Op, int64_t Cp,
                         hipStream_t stream);
/* grad of packed conv weight: fp32 [>=O][k*Cp] -> [O][C][k] (accumulate if accum) */
int dph_conv_weight_unpack_grad(const float* g, float* dst, int64_t O, int64_t C, int64_t k, int64_t Cp, int accum,
                                hipStream_t stream);
/* residual-branch gradient: out = dy*drop(p,seed)*(*smask), padded rows zeroed
 * ((m % len_rows) >= row_len[m/len_rows]); colsum += out; sdot += sum(dy*drop*pre).
 * ws (deterministic mode with colsum / sdot): dph_rowblock_workspace(rows, cols) bytes.
 * Backward of components.py:273,845 (dropout), :432-434,:744-746 (layer masks), :980 (pad zeroing). */
int dph_branch_bwd(const void* dy, void* out, int64_t rows, int64_t cols, float p, uint64_t seed, const float* smask,
                   const int64_t* row_len, int64_t len_rows, float* colsum, const void* pre, float* sdot, float* ws,
                   int64_t ws_bytes, hipStream_t stream);
/* the same with an fp32 dy (the pre-norm residual stream's gradient); out is bf16, or fp32 when out_f32 (the
 * pre-norm pos-conv output's dropout, components.py:891, forward) */
int dph_branch_bwd_f32(const float* dy, void* out, int out_f32, int64_t rows, int64_t cols, float p, uint64_t seed,
                       const float* smask, const int64_t* row_len, int64_t len_rows, float* colsum, const void* pre,
                       float* sdot, float* ws, int64_t ws_bytes, hipStream_t stream);
/* bf16 -> f32 copy / accumulate helpers */
int dph_add_bf16(const void* a, const void* b, void* out, int64_t n, hipStream_t stream);

/* ------------------------------------------------------------------------ *
 * Distillation loss (lightning.py:116-139) over student s (fp32, layer-major
 * [L][B][T][D]: each distill layer's projection is one dense GEMM output) and
 * teacher layers t_l (bf16), given as L pointers to [B][T][D] hidden states.
 * The loss is a mean over all (l,b,t) rows, so the layer-major order is
 * equivalent to the reference's torch.stack(dim=1) (B,L,T,D).
 * out[0..3] = loss, mse, l1, cos.  rowstats [B*L*T][3] saved for backward.
 * partial: DPH_LOSS_PARTIAL_FLOATS fp32 of scratch (one (l1, l2, cos) triple per block, summed in a fixed
 * order by a finalize kernel: deterministic, no atomics, no memset).
 * ------------------------------------------------------------------------ */
#define DPH_MAX_DISTILL_LAYERS 16
#define DPH_LOSS_PARTIAL_FLOATS 3072
int dph_distill_loss_fwd(const float* s, const void* const* t_layers, int64_t B, int64_t L, int64_t T, int64_t D,
                         float l2w, float l1w, float cosw, int cos_logsig, float* rowstats, float* partial,
                         float* out, hipStream_t stream);
/* ds (bf16, (B,L,T,D)) = dloss * d loss/ds; dbias[l][D] (fp32 atomics, per layer) optional */
int dph_distill_loss_bwd(const float* s, const void* const* t_layers, const float* rowstats, const float* dloss,
                         int64_t B, int64_t L, int64_t T, int64_t D, float l2w, float l1w, float cosw,
                         int cos_logsig, void* ds, hipStream_t stream);

/* the same with per-layer teacher dtypes: layer l is fp32 when bit l of t_f32_mask is set, else bf16 (the
 * hiddens of pre-norm encoders are their fp32 residual stream, components.py:846-850: read unrounded) */
int dph_distill_loss_fwd_ex(const float* s, const void* const* t_layers, uint32_t t_f32_mask, int64_t B, int64_t L,
                            int64_t T, int64_t D, float l2w, float l1w, float cosw, int cos_logsig, float* rowstats,
                            float* partial, float* out, hipStream_t stream);
int dph_distill_loss_bwd_ex(const float* s, const void* const* t_layers, uint32_t t_f32_mask, const float* rowstats,
                            const float* dloss, int64_t B, int64_t L, int64_t T, int64_t D, float l2w, float l1w,
                            float cosw, int cos_logsig, void* ds, hipStream_t stream);

/* Lagrangian sparsity regulariser and total loss (lightning.py:221-229, DistillModule._step):
 * es = 1 - num/orig_params, d = es - target, reg = lambda1*d + lambda2*d^2, out[0..2] = distill + reg,
 * reg, es.  target from target_dev when non-NULL (the HIP-graph step block), else `target`.  All
 * pointers are device fp32 scalars. */
int dph_reg_loss_fwd(const float* distill, const float* num, const float* lambda1, const float* lambda2,
                     const float* target_dev, float target, float orig_params, float* out, hipStream_t stream);
/* grads[0..2] = d/d(num, lambda1, lambda2) of g_loss*loss + g_reg*reg + g_es*es (any g may be NULL = 0);
 * d/d(distill) is g_loss.  sink_l1 / sink_l2 (optional): the lambdas' gradient-bucket slots, += their
 * gradients (the data-parallel sinks: no AccumulateGrad launch). */
int dph_reg_loss_bwd(const float* g_loss, const float* g_reg, const float* g_es, const float* num,
                     const float* lambda1, const float* lambda2, const float* target_dev, float target,
                     float orig_params, float* grads, float* sink_l1, float* sink_l2, hipStream_t stream);

/* ------------------------------------------------------------------------ *
 * HardConcrete (hardconcrete.py:85-116) + expected parameter count
 * (model.py:109-113 and the get_num_params chain).
 * ------------------------------------------------------------------------ */
/* mask = clamp(sigmoid((logit(u)+la)/beta)*(r-l)+l, 0, 1); u = uniform(eps, 1-eps) from (seed, i)
 * unless u_in != NULL.  u_out (optional) receives u. */
int dph_hc_sample_fwd(const float* log_alpha, const float* u_in, float* u_out, float* mask, int64_t n, uint64_t seed,
                      float beta, float limit_l, float limit_r, float eps, hipStream_t stream);
/* dlog_alpha += dmask * dmask/dlog_alpha */
int dph_hc_sample_bwd(const float* log_alpha, const float* u, const float* dmask, float* dlog_alpha, int64_t n,
                      float beta, float limit_l, float limit_r, hipStream_t stream);

/* Batched gates: every HardConcrete module of a model in ONE forward launch and ONE backward launch
 * (per DPH_HC_BANK_CHUNK entries) instead of a pair per module (hardconcrete.py:85-99 called by
 * components.py:112-114, :424-434, :735-746 once per module and step).  The host array `entries` is
 * read at call time and travels by value in the kernel arguments (capturable in a HIP graph).
 * fwd: u_flat[off+i] = u_in ? u_in[i] : U(eps, 1-eps) from (seed, off+i); mask_flat[off+i] = gate.
 * bwd: for entries with dmask != NULL: dlog_alpha[i] += dmask[i] * dgate/dlog_alpha (u from u_flat). */
#define DPH_HC_BANK_CHUNK 32
typedef struct DphHcEntry {
  const float* log_alpha;  /* [n] */
  const float* u_in;       /* fwd: injected noise [n] or NULL */
  const float* dmask;      /* bwd: [n] or NULL */
  float* dlog_alpha;       /* bwd: [n], accumulated */
  int64_t n;
  int64_t offset;          /* into u_flat / mask_flat */
} DphHcEntry;
int dph_hc_bank_fwd(const DphHcEntry* entries, int64_t n_entries, float* u_flat, float* mask_flat, uint64_t seed,
                    float beta, float limit_l, float limit_r, float eps, hipStream_t stream);
int dph_hc_bank_bwd(const DphHcEntry* entries, int64_t n_entries, const float* u_flat, float beta, float limit_l,
                    float limit_r, hipStream_t stream);

/* Expected #params as a polynomial in the l0 norms of n_groups HardConcrete
 * modules: value = const + sum_t coef[t] * prod_{i<3, idx[t][i]>=0} l0[idx[t][i]],
 * l0[g] = sum sigmoid(la_g + bias).  la_ptrs/la_sizes: device arrays of
 * per-module pointers / lengths. */
int dph_expected_params_fwd(const float* const* la_ptrs, const int64_t* la_sizes, int64_t n_groups,
                            const double* coef, const int32_t* idx, int64_t n_terms, double constant, float hc_bias,
                            float* l0, float* out, hipStream_t stream);
/* grad_flat[grad_offsets[g] + i] += dout * dE/dl0[g] * sigmoid'(la_g[i] + bias) */
int dph_expected_params_bwd(const float* const* la_ptrs, float* grad_flat, const int64_t* grad_offsets,
                            const int64_t* la_sizes, int64_t n_groups, const double* coef, const int32_t* idx,
                            int64_t n_terms, const float* l0, const float* dout, float hc_bias, hipStream_t stream);

/* ------------------------------------------------------------------------ *
 * Optimiser: multi-tensor AdamW (torch.optim.AdamW semantics,
 * lightning.py:200-228) with global-norm gradient clipping
 * (Trainer(gradient_clip_val=10), distill.py:48).
 * ------------------------------------------------------------------------ */
typedef struct DphTensorSlot {
  float* param;
  float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t n;
  int32_t group;
  int32_t pad_;
} DphTensorSlot;

typedef struct DphAdamGroup {
  float lr;
  float weight_decay;
  float beta1;
  float beta2;
  float eps;
  float pad_[3];
} DphAdamGroup;

/* sumsq[0] = sum over all slots of grad^2.  sumsq holds DPH_SUMSQ_FLOATS fp32: [0] the result, [1..] one
 * partial per block, summed in a fixed order by a finalize kernel (deterministic clip norm) */
#define DPH_SUMSQ_FLOATS 1025
int dph_grad_sumsq(const DphTensorSlot* slots, int64_t n_slots, const int64_t* chunk_slot,
                   const int64_t* chunk_start, int64_t n_chunks, float* sumsq, hipStream_t stream);
/* clip coef = min(1, max_norm/(sqrt(sumsq)+1e-6)) applied to grads, then AdamW step `step` (1-based) */
int dph_adamw_step(const DphTensorSlot* slots, int64_t n_slots, const int64_t* chunk_slot, const int64_t* chunk_start,
                   int64_t n_chunks, const DphAdamGroup* groups, int64_t n_groups, int64_t step,
                   const float* sumsq, float max_norm, hipStream_t stream);
/* the same with the per-group hyper-parameters and the (1-based) step read from DEVICE memory at
 * run time, so a captured HIP graph replays a changing LR schedule (lightning.py:22-44) */
typedef struct DphAdamDyn {
  DphAdamGroup g[4];
  float step;
  float pad_[3];
} DphAdamDyn;
int dph_adamw_step_dev(const DphTensorSlot* slots, int64_t n_slots, const int64_t* chunk_slot,
                       const int64_t* chunk_start, int64_t n_chunks, const DphAdamDyn* dyn, const float* sumsq,
                       float max_norm, hipStream_t stream);
/* either of the above (dyn != NULL: device hyper-parameters, else groups / step) that also writes each updated
 * master, cast to bf16 (round to nearest even, as dph_cast_bf16), to img[slot] (a device table of n_slots bf16
 * addresses, 0 = none): the bf16 GEMM images of the weights refreshed by the optimizer kernel itself instead of
 * a second pass that re-reads every master (replaces the torch param.data -> bf16 copy of the next forward) */
int dph_adamw_step_img(const DphTensorSlot* slots, int64_t n_slots, const int64_t* chunk_slot,
                       const int64_t* chunk_start, int64_t n_chunks, const DphAdamDyn* dyn, const DphAdamGroup* groups,
                       int64_t n_groups, int64_t step, const float* sumsq, float max_norm, const uint64_t* img,
                       hipStream_t stream);

/* ------------------------------------------------------------------------ *
 * Per-step RNG epoch: every dropout / HardConcrete kernel adds (*epoch) * 0x9E3779B97F4A7C15 to
 * its seed at entry (device word, uint64).  The trainer bumps the word with a stream-ordered op
 * once per step, so HIP-graph replays draw fresh noise and a step's backward regenerates its
 * forward's masks.  NULL detaches (seeds as passed).  Not stream-ordered; call outside capture.
 * ------------------------------------------------------------------------ */
int dph_set_rng_epoch(const uint64_t* epoch);

/* ------------------------------------------------------------------------ *
 * Timing events for live per-kernel durations (bench.py roofline): recorded as external
 * event-record nodes when the stream is being captured into a HIP graph.  ev is a hipEvent_t.
 * ------------------------------------------------------------------------ */
int dph_event_create(void** ev);
int dph_event_record(void* ev, hipStream_t stream);
int dph_event_elapsed_ms(void* start, void* stop, float* ms);
int dph_event_destroy(void* ev);

#ifdef __cplusplus
}
#endif
#endif /* DPHUBERT_HIP_H */
