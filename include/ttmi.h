/* ttmi.h — C ABI of libttmi.so, the MI355X (gfx950) two-tower training-step kernels.
 *
 * Drop-in boundary: the reference exposes no operator registry; its hot
 * path is the PyTorch nn.Module API of src/models driven by src/train.py.  Each entry
 * point below replaces the implicit PyTorch/cuBLAS/cuDNN work behind one reference call
 * site, cited as reference-file:line.  The Python host (music-recommendation-multimodal_amd)
 * binds these through ctypes and rebuilds the reference's constructors, forward(batch)
 * contract and state_dict names on top (see INTEGRATION.md for the binding).
 *
 * Conventions
 *  - Plain device pointers and sizes; all tensors row-major and contiguous unless an
 *    explicit leading dimension (ld*) is given.  No allocation, no hidden mutable
 *    state; every call is asynchronous on `stream` and safe to capture in a hipGraph.
 *  - dtype arguments: TTMI_F32 or TTMI_BF16 (bf16 = uint16 bit pattern).  Reductions,
 *    normalisation statistics, softmax/LSE and the loss are always fp32.
 *  - Dropout: (p, seed) where `seed` points to a uint64 in DEVICE memory (read at kernel
 *    entry, so a captured graph replays with whatever seed the step wrote there; may be
 *    NULL when p == 0).  With h = lowbias32(((i >> 1) + lo32(seed)) ^ hi32(seed)),
 *    keep(i) = (i odd ? h >> 16 : h & 0xFFFF) >= floor(p * 65536) over the flat element
 *    index i stated per call (one hash per element pair); kept values are scaled by
 *    1/(1-p).  p = 0 is the identity (reference parity runs).
 *  - Return 0 (TTMI_OK) on success; otherwise an error code, with a message available
 *    from ttmi_last_error() (thread-local).  Invalid shapes are rejected before launch.
 */
#ifndef TTMI_H
#define TTMI_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { TTMI_OK = 0, TTMI_ERR_ARG = 1, TTMI_ERR_LAUNCH = 2 };
enum { TTMI_F32 = 0, TTMI_BF16 = 1 };

/* Error message of the last failing call on this thread ("" if none). */
const char* ttmi_last_error(void);
/* ABI version (bumped on any signature change). */
int ttmi_abi_version(void);

/* Embedding-id range flags (ABI 20; block layout ABI 22).  The reference's nn.Embedding lookups
 * raise IndexError for an id outside the table (user_tower.py:26,30-31 item / gender / country
 * embeddings, two_tower.py:82-87 callers; the DeBERTa word embedding behind item_tower.py:47; the
 * catalogue index assignment evaluate_metrics.py:102, inference.py:204).  The device entry
 * points that index such a table take `int32_t* id_err` (may be NULL): an id outside [0, rows)
 * never reads or writes outside the table (it is clamped, or its row reads as zero / is skipped,
 * as each call states), and flag TTMI_IDERR_<key> is set to 1 by plain stores (racing writers
 * store the same value).  id_err points to a 16-B aligned block in DEVICE memory: int32
 * flags[8], then at byte 32 an `int32_t*` to a host-mapped int32[8] (may be NULL); both arrays
 * get the flag (the device one as 0x3F800000, the bit pattern of 1.0f, so that a data-parallel
 * step can SUM-all-reduce the flags of every rank as floats; the host one as 1).  The library never clears either: the host polls the host-mapped copy (no
 * device sync) and raises IndexError naming the key; the device copy is what ttmi_adamw*'s
 * `skip_if` reads (the train step clears it when it stages a batch). */
enum { TTMI_IDERR_HISTORY = 0, TTMI_IDERR_GENDER = 1, TTMI_IDERR_COUNTRY = 2,
       TTMI_IDERR_TEXT = 3, TTMI_IDERR_CATALOGUE = 4,
       TTMI_IDERR_HEAD_POLL = 7,  /* not an id: ttmi_user_item_head_fwd_ac's stage-C poll timed out
                                     (its item outputs are invalid); set through the user head's id_err */
       TTMI_IDERR_WORDS = 8 };

/* ------------------------------------------------------------------------------------
 * GEMM with fused epilogue — every nn.Linear on the path, forward and backward:
 *   user_tower.py:37-45 (MHA in_proj/out_proj, linear1/linear2 of TransformerEncoderLayer),
 *   user_tower.py:51-57 (user fusion MLP), item_tower.py:122-129 (item fusion head),
 *   two_tower.py:106 (logits = û·îᵀ/τ) and the InfoNCE gradient products.
 *
 *   C[m,n] (=|+=) epi( alpha * Σ_k A(m,k)·B(n,k) )
 *   A(m,k) = a_kmajor ? A[m*lda+k] : A[k*lda+m];  B(n,k) = b_kmajor ? B[n*ldb+k] : B[k*ldb+n]
 *   epi: v += bias[n]; v = act(v) (0 none, 1 relu, 2 GELU (erf), 3 none: see gate);
 *        v = dropout(v, idx = r(m)*ld_drop + n) with r(m) = drop_rows ? drop_rows[m] : m;
 *        v = gate ? (gate[m*ld_gate+n] > 0 ? v*gate_scale : 0) : v;  colsum[n] += v;
 *        act 3 instead multiplies by GELU'(gate[m*ld_gate+n]) (gate = the stored pre-activation:
 *        the input gradient of a GELU-activated Linear, DeBERTa intermediate.dense).
 *        v += residual[m*ld_res+n];  C = v (c_mode 0) or C += v atomically (c_mode 1, f32 C).
 *   rowsum_a (may be NULL): rowsum_a[m] += Σ_k A(m,k) — with A = dYᵀ of a weight-gradient
 *   GEMM this is the bias gradient, taken from the operand fragments already in registers.
 *   Operands A and B share `dtype`; C has `c_dtype`.  split_k > 1 partitions K over
 *   workgroups and requires c_mode 1 and act 0 (bias/residual are added by split 0 only).
 *   Alignment: rows of a k-major operand need K % 8 == 0 (bf16) / K % 4 == 0 (f32);
 *   a non-k-major operand needs M (or N) % 8 == 0 (bf16) / % 4 == 0 (f32).
 * ---------------------------------------------------------------------------------- */
typedef struct {
  int dtype;
  int64_t M, N, K;
  const void* A; int64_t lda; int a_kmajor;
  const void* B; int64_t ldb; int b_kmajor;
  void* C; int64_t ldc; int c_dtype; int c_mode;
  float alpha;
  const float* bias;
  int act;
  float drop_p; const uint64_t* drop_seed; int64_t ld_drop;
  const void* gate; int gate_dtype; int64_t ld_gate; float gate_scale;
  const float* residual; int64_t ld_res;
  float* colsum;
  int split_k;
  const int32_t* drop_rows;
  float* rowsum_a;
  void* pre_out;      /* ABI 8; may be NULL.  With act 2 (GELU), bf16 C, c_mode 0 and no
                         dropout / gate / residual / colsum / split: pre_out[m*ldc+n] = the
                         pre-activation (after bias), bf16 — DebertaV2Intermediate's dense output
                         kept for the GELU' of the backward, written by the same epilogue that
                         writes C = GELU(pre) (item_tower.py:41-83, modeling_deberta_v2). */
} ttmi_gemm_desc;
int ttmi_gemm(const ttmi_gemm_desc* d, hipStream_t stream);

/* ------------------------------------------------------------------------------------
 * Deterministic nn.Linear weight gradient (every Linear's backward on the path:
 * user_tower.py:37-57, item_tower.py:85-129 — autograd's dW = dYᵀ·X, db = Σ_r dY):
 *   dw[m, n] (+)= alpha · Σ_r dy[r, m] · x[r, n];   db[m] (+)= Σ_r dy[r, m]   (db may be NULL)
 * dy bf16 [R][ld_dy], x bf16 [R][ld_x] (row-major over the reduction), dw fp32 [M][ld_dw].
 * The reduction is split over workgroups; split partials go to `workspace`
 * (ttmi_wgrad_workspace bytes; 0 when one split suffices) and are summed in split order, so
 * the result is bit-reproducible (no float atomics).  defer = 1 leaves the partials in the
 * workspace: a later ttmi_wgrad_fold over the same descriptors (several GEMMs per launch)
 * completes dw / db.  M, N % 8 == 0; ld_dw % 4 == 0; operands 16-byte aligned.  ABI 10.
 * ---------------------------------------------------------------------------------- */
typedef struct {
  int64_t R, M, N;
  const void* dy; int64_t ld_dy;
  const void* x; int64_t ld_x;
  float* dw; int64_t ld_dw;
  float* db;
  float alpha;
  int accumulate;
  void* workspace; int64_t workspace_bytes;
  int defer;
} ttmi_wgrad_desc;
int64_t ttmi_wgrad_workspace(int64_t R, int64_t M, int64_t N, int64_t ld_dy, int64_t ld_x);
int ttmi_wgrad(const ttmi_wgrad_desc* d, hipStream_t stream);
/* Generic split fold: C[m*ldc + n] (+)= Σ_{s < S, in order} part[s*s_stride + m*N + n].
 * accumulate: bit 0 = add to C (else overwrite); bit 1 (ABI 15) = zero the partials read
 * (a workspace that must be zero on the next use, e.g. ttmi_seq_embed_bwd's).
 * fx_shift (ABI 16): 0 = fp32 partials; > 0 = int64 fixed-point partials (value = q·2^-fx_shift,
 * the order-independent accumulators of ttmi_seq_embed_bwd / ttmi_user_head_bwd / ...). */
typedef struct {
  const void* part; int64_t S, s_stride, M, N;
  float* C; int64_t ldc;
  int accumulate;
  int fx_shift;
} ttmi_fold_desc;
/* Completes the deferred ttmi_wgrad calls `descs` and the generic folds `folds` (one launch
 * per 16 segments). */
int ttmi_wgrad_fold(int n, const ttmi_wgrad_desc* const* descs, int nf,
                    const ttmi_fold_desc* folds, hipStream_t stream);
/* Computes the n weight gradients `descs` (their `defer` fields ignored) as one grouped
 * launch (per 16 GEMMs), then folds their partials and the generic folds `folds`: a
 * backward's weight gradients in two launches.  The operands must still hold their values
 * when this runs (the caller keeps them alive and unmodified).  ABI 10. */
int ttmi_wgrad_batch(int n, const ttmi_wgrad_desc* const* descs, int nf,
                     const ttmi_fold_desc* folds, hipStream_t stream);
/* ABI 19: the fold of ttmi_wgrad_batch left to the optimizer.  ttmi_wgrad_batch_plan runs the
 * grouped GEMMs and records their partials' segments (and the generic folds') in `plan` instead
 * of folding them (plan->n = 0 when they do not fit: then it folds them itself);
 * ttmi_adamw_folded is ttmi_adamw_fx that sums each planned segment in the fold's order and
 * applies AdamW to it in the same launch (one process: nothing reads the folded gradient in
 * between).  The partials' workspaces must stay alive and unmodified until it has run; a plan
 * whose segments do not tile the flat buffer in float4 units folds first, then updates. */
typedef struct ttmi_fold_plan {
  int32_t n, reserved;
  uint64_t seg[32 * 16];           /* opaque */
} ttmi_fold_plan;
int ttmi_wgrad_batch_plan(int n, const ttmi_wgrad_desc* const* descs, int nf,
                          const ttmi_fold_desc* folds, ttmi_fold_plan* plan, hipStream_t stream);
/* ttmi_adamw_folded leaving [skip_off, skip_off + skip_len) (float4-aligned; fx must be NULL)
 * untouched: a range already updated by its own ttmi_adamw_fx launch (the item-embedding rows,
 * updated beside the weight-gradient GEMMs while they run on a side stream). */
int ttmi_adamw_folded_skip(int64_t n, float* p, float* g, float* m, float* v, uint16_t* p_bf16,
                           const double* hyper, const int32_t* step, int zero_grad, int64_t* fx,
                           int64_t fx_off, int64_t fx_len, int fx_shift, const ttmi_fold_plan* plan,
                           int64_t skip_off, int64_t skip_len, const int32_t* skip_if,
                           hipStream_t stream);
/* Append src's segments to dst (one update for GEMMs planned early on a side stream and folds
 * planned later); when dst has no room left, src's segments are folded on `stream` instead. */
int ttmi_fold_plan_merge(ttmi_fold_plan* dst, const ttmi_fold_plan* src, hipStream_t stream);
/* ABI 22: the plan's folds as ordinary fold launches (ttmi_wgrad_batch's second half): the
 * data-parallel step plans its GEMMs early (side stream) like the one-process step, but must
 * complete the gradient before the all-reduce, so it folds the plan itself. */
int ttmi_fold_plan_run(const ttmi_fold_plan* plan, hipStream_t stream);
int ttmi_adamw_folded(int64_t n, float* p, float* g, float* m, float* v, uint16_t* p_bf16,
                      const double* hyper, const int32_t* step, int zero_grad, int64_t* fx,
                      int64_t fx_off, int64_t fx_len, int fx_shift, const ttmi_fold_plan* plan,
                      const int32_t* skip_if, hipStream_t stream);

/* ------------------------------------------------------------------------------------
 * LayerNorm over rows of width D (64 <= D <= 1024, D % 64 == 0) — TransformerEncoderLayer
 * norm1/norm2 (user_tower.py:37-45), user fusion LN (user_tower.py:54), item head final
 * LN (item_tower.py:128).  Optional ReLU and dropout (idx = row*D + col) after the affine.
 * Writes y (y_dtype, ldy) and per-row mean/rstd (fp32) for the backward.
 * ---------------------------------------------------------------------------------- */
int ttmi_layernorm_fwd(int64_t M, int D, const float* x, int64_t ldx, const float* w,
                       const float* b, float eps, int relu, float drop_p, const uint64_t* drop_seed,
                       void* y, int y_dtype, int64_t ldy, float* mean, float* rstd,
                       hipStream_t stream);
/* Backward of the above.  dy (fp32) is the gradient w.r.t. y; if gate != NULL it is first
 * multiplied by (gate > 0 ? gate_scale : 0) (gate = the stored y when ReLU/dropout followed
 * the affine).  dx = res + LN'(dy) (res may alias dx or be NULL); dw/db are accumulated
 * (fp32).  ws: ttmi_layernorm_bwd_workspace(D) bytes, zero on entry and left zero: int64
 * fixed-point replica rows of the column sums (ABI 16: order-independent, so dw / db are
 * bit-reproducible), folded once (may be NULL when dw and db are both NULL).  defer != 0
 * (ABI 16) leaves the fold to the caller: ttmi_layernorm_bwd_folds writes its
 * ttmi_fold_desc, one per non-NULL dw, db (in that order).  dx16 (optional, bf16, row stride ld16) receives
 * bf16(dropout(dx)) with keep index m*D + n (drop_p may be 0): the next GEMM's operand, with
 * the residual branch's dropout backward fused (saves a launch). */
int64_t ttmi_layernorm_bwd_workspace(int D);
int ttmi_layernorm_bwd_folds(int D, void* ws, float* dw, float* db, ttmi_fold_desc* out);
int ttmi_layernorm_bwd(int64_t M, int D, const float* dy, int64_t lddy, const float* x,
                       int64_t ldx, const float* mean, const float* rstd, const float* w,
                       const void* gate, int gate_dtype, int64_t ldg, float gate_scale,
                       const float* res, float* dx, int64_t lddx, float* dw, float* db,
                       void* ws, void* dx16, int64_t ld16, float drop_p,
                       const uint64_t* drop_seed, int defer, hipStream_t stream);

/* ------------------------------------------------------------------------------------
 * SASRec input block (user_tower.py:83-93):
 *   x[b,l,:] = dropout(LN(E[ids[b,l]] + P[l]))   (dropout idx = (b*L+l)*D + c)
 * E [V,D], P [>=L,D] fp32 master tables; x [B*L,D] fp32 residual stream.
 * Optional (y1 != NULL): the first encoder layer's norm1 on the same rows,
 *   y1 = bf16(LN(x) * w1 + b1), mean1 / rstd1 its row statistics (user_tower.py:111-116,
 *   TransformerEncoderLayer(norm_first=True) layer 0), fused while the row is in registers.
 * An id outside [0, V) reads a zero embedding row and sets id_err[TTMI_IDERR_HISTORY] (ABI 20).
 * ---------------------------------------------------------------------------------- */
int ttmi_seq_embed_fwd(int B, int L, int D, const int64_t* ids, const float* E, int64_t V,
                       const float* P, const float* w, const float* b, float eps,
                       float drop_p, const uint64_t* drop_seed, float* x, float* mean, float* rstd,
                       const float* w1, const float* b1, float eps1, void* y1, float* mean1,
                       float* rstd1, int32_t* id_err, hipStream_t stream);
/* Backward: dE[ids] += g (rows with ids == padding_idx skipped, nn.Embedding(padding_idx=0)
 * user_tower.py:27; ids outside [0, V) contribute nothing), dP[l] += Σ_b g, dw/db += LN affine
 * grads.  All accumulate (fp32).  ABI 16: the cross-row sums go to int64 fixed-point
 * accumulators in ws (ttmi_seq_embed_bwd_workspace(V, L, D) bytes, 16-byte aligned, zero on
 * entry and left zero by the fold; one buffer may serve every call on one stream), so the
 * gradients are bit-reproducible whatever order the token rows land in.  defer = 0 folds
 * them into dE / dP / dw / db before returning; defer != 0 leaves the 4 folds to the caller
 * (ttmi_seq_embed_bwd_folds writes the 4 ttmi_fold_desc, to run with its deferred weight
 * gradients).  D % 4 == 0. */
int64_t ttmi_seq_embed_bwd_workspace(int64_t V, int L, int D);
int ttmi_seq_embed_bwd_folds(int64_t V, int L, int D, void* ws, float* dE, float* dP, float* dw,
                             float* db, ttmi_fold_desc* out);
int ttmi_seq_embed_bwd(int B, int L, int D, int64_t V, const int64_t* ids, const float* E,
                       const float* P, const float* w, const float* mean, const float* rstd,
                       float drop_p, const uint64_t* drop_seed, const float* dx, float* dE, float* dP,
                       float* dw, float* db, int64_t padding_idx, void* ws, int defer,
                       hipStream_t stream);

/* ------------------------------------------------------------------------------------
 * Multi-head self-attention core (SDPA inside nn.MultiheadAttention, user_tower.py:111-116):
 *   per (b,h): S = Q·Kᵀ/√Dh, causal (key j <= query i) + key padding (key_valid[b,j] != 0;
 *   pass history_mask, or history_ids when the mask is None), softmax, dropout on the
 *   probabilities (idx = ((b*H+h)*L+i)*L+j), O = P·V.  Query rows with no valid key give 0.
 * qkv [B*L, 3*H*Dh] (q|k|v, dtype), ctx [B*L, H*Dh] (dtype), lse [B*H*L] fp32 (+inf for
 * fully masked rows).  L <= TTMI_ATTN_LMAX, Dh <= 64, Dh % 8 == 0; L <= 64 runs whole sequences
 * in one LDS image (MFMA), 64 < L <= TTMI_ATTN_LMAX (ABI 17) the tiled long-sequence kernels
 * (online softmax over 64-key blocks).  The one-query ttmi_mha_q1_* calls take the same range.
 * ---------------------------------------------------------------------------------- */
#define TTMI_ATTN_LMAX 2048
int ttmi_mha_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                 const int64_t* key_valid, float drop_p, const uint64_t* drop_seed, void* ctx,
                 float* lse, hipStream_t stream);
int ttmi_mha_bwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                 const int64_t* key_valid, const float* lse, const void* dctx, float drop_p,
                 const uint64_t* drop_seed, void* dqkv, hipStream_t stream);
/* The same attention for the shapes ttmi_mha_fwd / _bwd refuse (ABI 22, ttmi_attn_generic.hip):
 * any L, head widths 0 < Dh <= 512 (not only multiples of 8 up to 64).  Same operands, masks,
 * dropout indices and lse convention (natural log, +inf on a row with no allowed key); a wave
 * per query row / key row, no tiling: the path that keeps a model the reference accepts
 * trainable, not a fast one.  The backward also needs the forward's ctx rows (D_i = dO_i·O_i)
 * and a float workspace of B·H·L (dsum_ws). */
int ttmi_mha_generic_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                         const int64_t* key_valid, float drop_p, const uint64_t* drop_seed, void* ctx,
                         float* lse, hipStream_t stream);
int ttmi_mha_generic_bwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                         const int64_t* key_valid, const float* lse, const void* ctx, const void* dctx,
                         float drop_p, const uint64_t* drop_seed, float* dsum_ws, void* dqkv,
                         hipStream_t stream);
/* The encoder layer's whole attention sub-block forward in one launch (ABI 21; reference
 * user_tower.py:37-45, norm_first): ttmi_qkv_attn_fwd's qkv / ctx / lse, then
 *   x1 = res + drop1(ctx·woᵀ + bo)   (fp32 [B*L, 128]; drop1 index m·128 + n)
 *   a2 = norm2(x1) (bf16), m2 / r2 its row mean / rstd
 * as ttmi_linear_res_ln computes them (the row statistics summed in another order).  bf16,
 * H*Dh = 128 with Dh = 32, 38 <= L <= 64 (two sequences per workgroup). */
typedef struct ttmi_attn_block_desc {
  int B, L, H, Dh;
  const void* a; const void* w_in; const float* b_in; const int64_t* key_valid;
  float drop_p; const uint64_t* drop_seed;         /* the attention probabilities */
  void* qkv; void* ctx; float* lse;
  const void* wo; const float* bo; const float* res; const float* n2w; const float* n2b;
  float eps;
  float drop1_p; const uint64_t* drop1_seed;       /* the out-projection's output */
  float* x1; void* a2; float* m2; float* r2;
} ttmi_attn_block_desc;
int ttmi_attn_block_fwd(const ttmi_attn_block_desc* d, hipStream_t stream);
/* The encoder layer's feed-forward sub-block forward and the next layer's norm1 in one launch
 * (ABI 21; reference user_tower.py:37-45, norm_first, then :111-116 for layer i + 1):
 *   h  = drop_f(relu(a·w1ᵀ + b1))     bf16 [M, F] (drop_f index m·F + n; the FFN1 row panel's bits)
 *   x2 = res + drop2(h·w2ᵀ + b2)       fp32 [M, D] (drop2 index m·D + n)
 *   y  = bf16(LN(x2)·lnw + lnb), mean / rstd its row statistics
 * as ttmi_linear(act = ReLU) + ttmi_linear_res_ln compute them, h never read back (x2 summed in
 * hidden-unit order: equal to fp32 rounding).  bf16, D = 128, F in {256, 512}, M·F·2 < 2 GB;
 * ttmi_ffn_block_supported(dtype, D, F) says whether a shape is served. */
typedef struct ttmi_ffn_block_desc {
  int M, D, F;
  const void* a;                                   /* [M, D] bf16: norm2's output */
  const void* w1; const float* b1;                 /* [F, D] bf16, [F] */
  const void* w2; const float* b2;                 /* [D, F] bf16, [D] */
  const float* res;                                /* [M, D] fp32: the sub-block's input x1 */
  float dropf_p; const uint64_t* dropf_seed;
  float drop2_p; const uint64_t* drop2_seed;
  void* h; float* x2;
  const float* lnw; const float* lnb; float eps;
  void* y; float* mean; float* rstd;
  /* ABI 22 (kv may be NULL): the next layer's K / V input projection of y in the same launch,
   * kv[m·ld_kv + n] = bf16(y[m]·wkv[n]ᵀ + bkv[n]) for n < 2·D (wkv [2D, D] bf16 = in_proj_weight
   * rows D..3D): the pruned last layer's full-length K / V (its Q is projected for the gathered
   * rows only), with the row panel's fragments and MFMA order (ttmi_gemm's bits). */
  const void* wkv; const float* bkv; void* kv; int64_t ld_kv;
} ttmi_ffn_block_desc;
int ttmi_ffn_block_supported(int dtype, int D, int F);
/* ABI 22: the forward also serves D = 256 with F = 1024 (the reference's default width; its
 * A / W1 fragments read k = 128 (c >> 2) + 32 lg + 8 (c & 3), so h agrees with the FFN1 row panel to bf16 rounding
 * there); ttmi_ffn_block_bwd_supported(dtype, D, F) says which shapes the backward serves
 * (the same: D = 128 with F in {256, 512}, D = 256 with F = 1024). */
int ttmi_ffn_block_bwd_supported(int dtype, int D, int F);
int ttmi_ffn_block_fwd(const ttmi_ffn_block_desc* d, hipStream_t stream);
/* Its input-grad half (ABI 21): on the transposed weight mirrors w2t = linear2.weightᵀ [F, D],
 * w1t = linear1.weightᵀ [D, F] (bf16, k-major),
 *   dz1 = (dy2·w2ᵀᵀ) ⊙ [h > 0]·gate_scale   bf16 [M, F] (ttmi_linear with gate = h: its bits)
 *   dY  = dz1·w1 (not stored); norm2's backward as ttmi_linear_ln_bwd: dx1 = LN2ᵀ(dY) + res
 *   (fp32), dy1 = bf16(drop1ᵀ(dx1)) (index m·D + n), and per workgroup Σ_rows dY·x̂ (norm2.weight)
 *   and Σ_rows dY (norm2.bias) -> sum_ws[blk][2][D], blk < ttmi_ffn_block_bwd_sum_blocks(M):
 *   the caller folds them in workgroup order (ttmi_fold_desc: S = blocks, s_stride = 2·D).
 * dY sums in hidden-unit order: dx1 / dy1 / the sums agree with the row panels to fp32 rounding.
 * Shapes as ttmi_ffn_block_fwd. */
typedef struct ttmi_ffn_block_bwd_desc {
  int M, D, F;
  const void* dy2;                                 /* [M, D] bf16: FFN output grad (drop2ᵀ applied) */
  const void* w2t; const void* w1t;
  const void* h; float gate_scale;                 /* [M, F] bf16: the forward's h; 1 / (1 - p_ffn) */
  void* dz1;                                       /* [M, F] bf16 out */
  const float* x1; const float* m2; const float* r2; const float* n2w;   /* norm2's input, stats, weight */
  const float* res;                                /* [M, D] fp32: added to dx1 */
  float* dx1; void* dy1;
  float drop1_p; const uint64_t* drop1_seed;
  float* sum_ws;
} ttmi_ffn_block_bwd_desc;
int ttmi_ffn_block_bwd_sum_blocks(int M);
int ttmi_ffn_block_bwd(const ttmi_ffn_block_bwd_desc* d, hipStream_t stream);
/* ttmi_mha_bwd with dctx computed in the launch from the out-projection's output gradient
 * (ABI 21): dctx = dy·W_o (dy [B*L, 128] bf16; wot = W_oᵀ, the transposed k-major mirror,
 * [128, 128] bf16), rounded to bf16 with ttmi_linear's fragment and MFMA order, so dqkv is
 * bit-identical to ttmi_linear(dy, wot) + ttmi_mha_bwd where the row-panel kernel serves that
 * linear (M >= 2048).  bf16, H*Dh = 128 with Dh = 32, L <= 64. */
int ttmi_mha_bwd_dy(int B, int L, int H, int Dh, const void* qkv, const int64_t* key_valid,
                    const float* lse, const void* dy, const void* wot, float drop_p,
                    const uint64_t* drop_seed, void* dqkv, hipStream_t stream);
/* The encoder layer's input projection and attention in one launch (ABI 21; reference
 * user_tower.py:111-116, nn.MultiheadAttention in_proj then SDPA): qkv = a·w_inᵀ + b_in
 * (a [B*L, 128] bf16 normed rows, w_in [384, 128] bf16, b_in [384] fp32), written to qkv as
 * ttmi_linear's panel kernel would (bit-identical to ttmi_linear from M = 2048 rows, where
 * that kernel serves it), then ctx / lse exactly as ttmi_mha_fwd on that qkv.  Served shapes: ttmi_qkv_attn_supported() (bf16, H*Dh = 128, Dh = 32,
 * L <= 64); anything else is TTMI_ERR_ARG. */
int ttmi_qkv_attn_supported(int dtype, int L, int H, int Dh);
int ttmi_qkv_attn_fwd(int dtype, int B, int L, int H, int Dh, const void* a, const void* w_in,
                      const float* b_in, const int64_t* key_valid, float drop_p,
                      const uint64_t* drop_seed, void* qkv, void* ctx, float* lse,
                      hipStream_t stream);

/* ------------------------------------------------------------------------------------
 * Last-valid gather + demographics concat (user_tower.py:118-139):
 *   len_b = Σ_l (len_src[b,l] != 0) - 1 clamped >= 0; rows[b] = b*L + len_b
 *   (len_src == NULL: x is already gathered, rows[b] = b*L with L == 1);
 *   comb[b] = [x[rows[b]], G[gender[b]], C[country[b]]]   ([B, D+dg+dc], dtype)
 * G has n_genders rows, C n_countries (ABI 20): an id outside its table reads the clamped row
 * and sets id_err[TTMI_IDERR_GENDER / _COUNTRY].
 * ---------------------------------------------------------------------------------- */
int ttmi_user_concat_fwd(int dtype, int B, int L, int D, const float* x,
                         const int64_t* len_src, const int64_t* gender, const float* G, int dg,
                         const int64_t* country, const float* C, int dc, void* comb,
                         int32_t* rows, int n_genders, int n_countries, int32_t* id_err,
                         hipStream_t stream);
/* Backward: dx[rows[b]] += dcomb[b,:D] (accumulate != 0; = when 0; rows distinct);
 * dG[gender[b]] += ...; dC[country[b]] += ... into int64 fixed-point accumulators (ABI 16,
 * scale 2^36 = TTMI_FX_GRAD_SHIFT, zero on entry; the caller folds them with a
 * ttmi_fold_desc of fx_shift 36; may be NULL).  Ids are clamped as in the forward. */
int ttmi_user_concat_bwd(int B, int D, const float* dcomb, const int32_t* rows,
                         const int64_t* gender, int dg, const int64_t* country, int dc,
                         float* dx, int64_t* dG, int64_t* dC, int accumulate, int n_genders,
                         int n_countries, hipStream_t stream);

/* ------------------------------------------------------------------------------------
 * BatchNorm1d + ReLU + dropout (item_tower.py:122-126 fusion head, item_tower.py:89-93
 * tabular MLP).  training != 0: batch statistics (biased var) normalise, the running
 * buffers get momentum updates with the unbiased var, num_batches_tracked += 1, and
 * mean/rstd (may be NULL) receive the batch statistics.  training == 0: running statistics,
 * no update.  z [B,C] fp32 -> y [B,C] (dtype); dropout idx = b*C + c.
 * ---------------------------------------------------------------------------------- */
int ttmi_batchnorm_fwd(int dtype, int B, int C, const float* z, const float* w, const float* b,
                       float eps, float momentum, float* running_mean, float* running_var,
                       int64_t* num_batches_tracked, int training, int relu, float drop_p,
                       const uint64_t* drop_seed, void* y, float* mean, float* rstd,
                       hipStream_t stream);
/* dz = BN'(dy ⊙ (y > 0 ? gate_scale : 1 when relu/dropout)); dw/db accumulate. */
int ttmi_batchnorm_bwd(int dtype, int B, int C, const float* dy, const float* z,
                       const float* w, const float* mean, const float* rstd, const void* y,
                       float gate_scale, int gated, float* dz, float* dw, float* db,
                       void* dz16, hipStream_t stream);

/* ------------------------------------------------------------------------------------
 * Symmetric in-batch InfoNCE (two_tower.py:98-140), fp32 throughout:
 *   û = u/max(|u|,1e-12), î likewise; S = û·îᵀ·inv_tau; S[i,j] = -1e4 where
 *   user_idx[i] == user_idx[j] and i != j (user_idx may be NULL: no collision mask);
 *   loss = ½(CE(S, arange) + CE(Sᵀ, arange)) with mean reduction.
 * Outputs: û, î [B,D]; norms [2B]; logits [B,B] (masked, as the reference returns them);
 * lse [2B] (row LSEs then column LSEs); loss [1].  ws: ttmi_infonce_workspace(B, D) bytes.
 * Any B >= 1 when D % 64 == 0 and D <= 256 (the fused kernels; a ragged last batch of the
 * reference DataLoader, train.py:259-266, has no drop_last); otherwise B % 4 == 0.  ABI 10.
 * ---------------------------------------------------------------------------------- */
int64_t ttmi_infonce_workspace(int B, int D);
int ttmi_infonce_fwd(int B, int D, const float* u, const float* it, const int64_t* user_idx,
                     float inv_tau, float* u_hat, float* i_hat, float* norms, float* logits,
                     float* lse, float* loss, void* ws, hipStream_t stream);
/* ttmi_infonce_fwd on rows the producers already normalised (ABI 15): u_hat, i_hat [B, D] and
 * norms [2B] (u norms, then i norms) as the l2norm launch would write them (the fused user /
 * item heads' u_hat / out_hat outputs); logits, lse, loss, ws as ttmi_infonce_fwd.  counters
 * (optional, ttmi_infonce_counter_bytes(B) bytes, zero on entry and left zero): the lse / loss
 * combine runs inside the logits launch (last-arriving workgroups; deterministic order)
 * instead of a launch of its own; then loss_acc (optional, device float) += loss in the same
 * launch (a training loop's running loss sum, src/train.py:68's total_loss, without a host
 * sync or an add launch per step).  The backward (ttmi_infonce_bwd / _bwd16) is unchanged. */
int ttmi_infonce_fwd_pre(int B, int D, const int64_t* user_idx, float inv_tau, const float* u_hat,
                         const float* i_hat, const float* norms, float* logits, float* lse,
                         float* loss, void* ws, int32_t* counters, float* loss_acc,
                         hipStream_t stream);
/* ABI 19: ttmi_infonce_fwd with the lse / loss combine inside the logits launch (persistent
 * zero `counters` of ttmi_infonce_counter_bytes(B)) and loss_acc (may be NULL) += loss: two
 * launches.  D % 64 == 0, D <= 256. */
int ttmi_infonce_fwd_acc(int B, int D, const float* u, const float* it, const int64_t* user_idx,
                         float inv_tau, float* u_hat, float* i_hat, float* norms, float* logits,
                         float* lse, float* loss, void* ws, int32_t* counters, float* loss_acc,
                         hipStream_t stream);
int64_t ttmi_infonce_counter_bytes(int B);
/* Backward given dloss (device scalar; NULL means 1): writes du, di [B,D]. */
int ttmi_infonce_bwd(int B, int D, const float* u_hat, const float* i_hat, const float* norms,
                     const float* logits, const float* lse, const int64_t* user_idx,
                     float inv_tau, const float* dloss, float* du, float* di, void* ws,
                     hipStream_t stream);
/* As ttmi_infonce_bwd, plus du16 (may be NULL): a bf16 copy of du [B,D] written by the same
 * kernel (the user tower's fusion-MLP backward consumes du as a bf16 GEMM operand).  ABI 9. */
int ttmi_infonce_bwd16(int B, int D, const float* u_hat, const float* i_hat, const float* norms,
                       const float* logits, const float* lse, const int64_t* user_idx,
                       float inv_tau, const float* dloss, float* du, float* di, uint16_t* du16,
                       void* ws, hipStream_t stream);
/* ttmi_infonce_bwd16 in ONE launch (ABI 18): the last of each 16-row block's key-split
 * workgroups (arrival count in `counters`, ttmi_infonce_bwd_counter_bytes(B) bytes, zero on
 * entry and left zero) sums the split partials in split order and runs the normalise backward
 * (bit-identical to the two-launch form).  counters NULL, or shapes the fused kernels do not
 * take: ttmi_infonce_bwd16. */
int ttmi_infonce_bwd_fused(int B, int D, const float* u_hat, const float* i_hat, const float* norms,
                           const float* logits, const float* lse, const int64_t* user_idx,
                           float inv_tau, const float* dloss, float* du, float* di, uint16_t* du16,
                           void* ws, int32_t* counters, hipStream_t stream);
int64_t ttmi_infonce_bwd_counter_bytes(int B);

/* ------------------------------------------------------------------------------------
 * Global in-batch negatives (BASELINE cfg 5; the reference InfoNCE two_tower.py:98-140
 * applied to the concatenation of every rank's batch).  Per rank r with B local pairs and
 * C = world·B gathered, L2-normalised rows:
 *   loss_r = (Σ CE_rows(û_r·Îᵀ/τ) + Σ CE_rows(î_r·Ûᵀ/τ)) / 2B,  positives at column r·B + i,
 *   collisions (same user_idx, different global index) masked to -1e4.
 * The caller all-gathers Û, Î, user_idx and reduce-scatters the key grads; mean over ranks
 * of loss_r is the global loss.  With world = 1 this is ttmi_infonce_fwd/bwd exactly.
 * ---------------------------------------------------------------------------------- */
/* y = x / max(||x||, 1e-12) per row; norms[n] = ||x|| (F.normalize). */
int ttmi_l2norm_fwd(int n, int D, const float* x, float* y, float* norms, hipStream_t stream);
/* dx = normalize backward of (dy + dy2) (dy2 may be NULL: the reduce-scattered key grads). */
int ttmi_l2norm_bwd(int n, int D, const float* y, const float* norms, const float* dy,
                    const float* dy2, float* dx, hipStream_t stream);
/* logits[R,C] = q·kᵀ·inv_tau, masked in place; lse[R]; ce[R] = lse − logits[i, row0+i].
 * uid_q/uid_k may both be NULL (no collision mask).  C % 4 == 0, row0 + R <= C. */
int ttmi_rowce_fwd(int R, int C, int D, const float* q, const float* k, const int64_t* uid_q,
                   const int64_t* uid_k, int64_t row0, float inv_tau, float* logits, float* lse,
                   float* ce, hipStream_t stream);
int64_t ttmi_rowce_workspace(int R, int C);
/* dS = dloss·scale·(softmax − onehot(row0+i)) (0 where masked); dq = dS·k·inv_tau [R,D],
 * dk = dSᵀ·q·inv_tau [C,D] (both written). */
int ttmi_rowce_bwd(int R, int C, int D, const float* q, const float* k, const float* logits,
                   const float* lse, const int64_t* uid_q, const int64_t* uid_k, int64_t row0,
                   float inv_tau, const float* dloss, float scale, float* dq, float* dk, void* ws,
                   hipStream_t stream);
/* out[0] = scale · Σ x[0:n) (fixed order: deterministic). */
int ttmi_sum_scaled(int n, const float* x, float scale, float* out, hipStream_t stream);

/* ------------------------------------------------------------------------------------
 * 2-D convolution (ResNet-18 audio/visual encoders, reference item_tower.py:9-39 on
 * torchvision resnet18): implicit GEMM over NHWC bf16 activations, C and Co multiples of 8
 * (stems zero-padded with ttmi_nchw_to_nhwc), square stride/pad, no bias.
 *   mode 0 FWD:   y[n,ho,wo,co] = Σ x[n, ho·s−p+kh, wo·s−p+kw, ci] W[co,ci,kh,kw]   (out bf16),
 *                 colsum/colsumsq [TTMI_CONV_STAT_REPS][Co] int64 fixed point, scale 2^24
 *                 (TTMI_FX_STAT_SHIFT; ABI 16; zero on entry, may both be NULL):
 *                 Σ_r colsum[r][co]·2^-24 = Σ y, Σ y² (BatchNorm stats, spread over replica
 *                 rows so the workgroups' atomics do not serialise on one address; integer
 *                 adds, so the statistics do not depend on the workgroups' order)
 *   mode 1 DGRAD: dx[n,h,w,ci] = Σ dy[n,(h+p−kh)/s,(w+p−kw)/s,co] W[co,ci,kh,kw] (+ addend)
 *                 over the stride lattice (out bf16; needs Cin == C, Co % 64 == 0, stride <= 2)
 *   mode 2 WGRAD: dW[co,ci,kh,kw] += Σ dy·x (out fp32, torch layout, ci < Cin); split-K
 *                 partials go to `workspace` (ttmi_conv2d_workspace(d) bytes), then are
 *                 summed in a fixed order (deterministic)
 *   mode 3 / 4:   FWD / WGRAD of the 7x7/2/3 stem (resnet18 conv1; ABI 17) over the
 *                 space-to-depth input of ttmi_stem_s2d: the descriptor states the stem on
 *                 the image (H, W even; Cin image channels; C = the s2d channel count >= 4 Cin;
 *                 KH = KW = 7, stride 2, pad 3; Co % 64 == 0), w is ttmi_stem_weight_prep's
 *                 [Co][4][4][C] mirror, and the conv runs as the equivalent 4x4/1 conv with
 *                 K = 16·C (128 / 256 for 1 / 3 channels instead of 49·8 = 392 padded taps).
 *                 WGRAD writes torch's [Co][Cin][7][7] layout like mode 2.
 * w is the bf16 mirror from ttmi_conv_weight_prep: Wf = [Co][KH][KW][C] for FWD,
 * Wd = [Cin][KH][KW][Co] for DGRAD.  Every tensor must have < 2^31 elements.
 * ---------------------------------------------------------------------------------- */
#define TTMI_CONV_STAT_REPS 16
typedef struct ttmi_conv_desc {
  int mode;
  int N, H, W, C, Cin, Co, KH, KW, stride, pad;
  const void* x;          /* bf16 NHWC [N,H,W,C] */
  const void* dy;         /* bf16 NHWC [N,Ho,Wo,Co] */
  const void* w;          /* bf16 mirror (FWD: Wf, DGRAD: Wd) */
  void* out;
  const void* addend;     /* DGRAD: bf16 [N,H,W,C] added before the store, or NULL */
  int64_t* colsum; int64_t* colsumsq;
  void* workspace;        /* WGRAD scratch (device), or NULL for FWD/DGRAD */
  int64_t workspace_bytes;
  /* DGRAD only (ABI 17): the backward reduction of the BatchNorm(+ReLU) that produced this
   * conv's input x, fused into the epilogue (bn_sums NULL: off).  Then out receives
   * g = bf16(dx) ⊙ (bn_gate > 0) instead of dx (bn_gate = that BN's output, bf16 [N,H,W,C];
   * NULL: no ReLU) and bn_sums [TTMI_CONV_STAT_REPS][2C] (int64 fixed point 2^36, zero on
   * entry) += Σ g, Σ g·(bn_x − mean)·rstd per channel (bn_x = that BN's input) — exactly
   * ttmi_bn2d_bwd_reduce's, so ttmi_bn2d_bwd_apply(g, ...) completes the BatchNorm backward. */
  const void* bn_gate; const void* bn_x; const float* bn_mean; const float* bn_rstd;
  int64_t* bn_sums;
} ttmi_conv_desc;
int ttmi_conv2d(const ttmi_conv_desc* d, hipStream_t stream);
/* Bytes of WGRAD scratch ttmi_conv2d needs for this descriptor (0 for FWD/DGRAD; -1 on a bad
 * descriptor). */
int64_t ttmi_conv2d_workspace(const ttmi_conv_desc* d);
/* wf[co][kh][kw][c] = bf16(w[co][ci][kh][kw]) zero for Cin <= c < Cp; wd[ci][kh][kw][co]
 * likewise (wd may be NULL). w is torch's fp32 Conv2d.weight. */
int ttmi_conv_weight_prep(int Co, int Cin, int Cp, int KH, int KW, const float* w, uint16_t* wf,
                          uint16_t* wd, hipStream_t stream);
/* Every conv's mirrors in one launch (ABI 17): items[i] as ttmi_conv_weight_prep's arguments,
 * or (s2d = 1, KH = KW = 7) ttmi_stem_weight_prep's [Co][4][4][Cp] mirror (wd unused).  At
 * most TTMI_WPREP_MAX items per launch (more are split over launches). */
#define TTMI_WPREP_MAX 24
typedef struct ttmi_conv_wprep {
  int Co, Cin, Cp, KH, KW, s2d;
  const float* w;
  uint16_t* wf;
  uint16_t* wd;           /* may be NULL */
} ttmi_conv_wprep;
int ttmi_conv_weight_prep_batch(int n, const ttmi_conv_wprep* items, hipStream_t stream);
/* y = bf16 NHWC [N,H,W,Cp] of x fp32 NCHW [N,Cin,H,W] (channels >= Cin zero). */
int ttmi_nchw_to_nhwc(int N, int Cin, int H, int W, int Cp, const float* x, uint16_t* y,
                      hipStream_t stream);
/* Space-to-depth stem input (ABI 17): y = bf16 [N][H/2][W/2][Cp] of x fp32 NCHW [N,Cin,H,W]
 * (H, W even), channel (ph·2 + pw)·Cin + ci = x[n][ci][2h+ph][2w+pw], channels >= 4·Cin zero
 * (Cp % 8 == 0).  Replaces the stem's ttmi_nchw_to_nhwc for conv modes 3 / 4. */
int ttmi_stem_s2d(int N, int Cin, int H, int W, int Cp, const float* x, uint16_t* y,
                  hipStream_t stream);
/* wf[co][a][b][(ph·2+pw)·Cin + ci] = bf16(w[co][ci][2a+ph−1][2b+pw−1]), zero off the 7x7
 * window and for channels >= 4·Cin: the stem weight (torch fp32 [Co][Cin][7][7]) as the 4x4
 * kernel over ttmi_stem_s2d's input (ABI 17). */
int ttmi_stem_weight_prep(int Co, int Cin, int Cp, const float* w, uint16_t* wf, hipStream_t stream);

/* BatchNorm2d, train mode, over NHWC bf16 [M = N·H·W, C] (C % 8 == 0, C <= 512), batch
 * statistics from the producing conv's colsum/colsumsq ([TTMI_CONV_STAT_REPS][C] int64 fixed
 * point, summed exactly; mean / variance in double):  y = act(w·x̂ + b + residual)
 * (act = ReLU if relu; residual bf16 or NULL); running stats updated with momentum and the
 * unbiased variance, *num_batches_tracked += 1 (all three may be NULL: eval-free path);
 * save_mean/save_rstd [C] for the backward (nn.BatchNorm2d + torchvision BasicBlock tail).
 * Eval mode (nn.BatchNorm2d.eval()): colsum = colsumsq = NULL normalises with
 * running_mean/running_var and updates nothing. */
int ttmi_bn2d_fwd(int64_t M, int C, const uint16_t* x, const int64_t* colsum, const int64_t* colsumsq,
                  const float* w, const float* b, float eps, float momentum, float* running_mean,
                  float* running_var, int64_t* num_batches_tracked, const uint16_t* residual,
                  int relu, uint16_t* y, float* save_mean, float* save_rstd, hipStream_t stream);
/* Backward: g = dy ⊙ (gate > 0) (gate = the ReLU output, or NULL); dx = w·rstd·(g − Σg/M −
 * x̂·Σgx̂/M); dw += Σgx̂, db += Σg.  sums [TTMI_CONV_STAT_REPS][2C] int64 fixed point (scale
 * 2^36, TTMI_FX_GRAD_SHIFT; ABI 16: order-independent) must be zero on entry (scratch);
 * g_out (bf16, may be NULL) receives g for the residual branch. */
int ttmi_bn2d_bwd(int64_t M, int C, const uint16_t* dy, const uint16_t* gate, const uint16_t* x,
                  const float* mean, const float* rstd, const float* w, int64_t* sums,
                  uint16_t* g_out, uint16_t* dx, float* dw, float* db, hipStream_t stream);
/* resnet18 stem tail (ABI 17): bn1 (train statistics from the conv's colsum/colsumsq, or eval
 * with colsum = colsumsq = NULL, as ttmi_bn2d_fwd) → ReLU → max-pool 3/2/1 over the conv output
 * x [N,H,W,C] bf16 without storing the BN output: y [N,Ho,Wo,C] bf16 pooled, idx the window tap
 * (uint8, first on ties) — bit-identical to ttmi_bn2d_fwd(relu) + ttmi_maxpool_fwd. */
int ttmi_stem_pool_fwd(int N, int H, int W, int C, const uint16_t* x, const int64_t* colsum,
                       const int64_t* colsumsq, const float* w, const float* b, float eps, float momentum,
                       float* running_mean, float* running_var, int64_t* num_batches_tracked, uint16_t* y,
                       uint8_t* idx, float* save_mean, float* save_rstd, hipStream_t stream);
/* Its backward: the pooled gradient dy is gathered onto the conv output (as ttmi_maxpool_bwd),
 * gated by the recomputed BN+ReLU output, and run through the BatchNorm backward (as
 * ttmi_bn2d_bwd: sums [TTMI_CONV_STAT_REPS][2C] int64 zero on entry; dw, db accumulate):
 * dx [N,H,W,C] bf16 = the gradient at the conv output.  b is bn1.bias (for the gate). */
int ttmi_stem_pool_bwd(int N, int H, int W, int C, const uint16_t* dy, const uint8_t* idx,
                       const uint16_t* x, const float* mean, const float* rstd, const float* w,
                       const float* b, int64_t* sums, uint16_t* dx, float* dw, float* db,
                       hipStream_t stream);
/* The two passes of ttmi_bn2d_bwd as separate calls (ABI 17), for a reduction fused elsewhere
 * (ttmi_conv_desc.bn_sums): _reduce accumulates sums (and writes g_out = dy ⊙ (gate > 0) when
 * g_out != NULL; g_out may alias dy); _apply computes dx from g (gate NULL: dy is already g)
 * and adds the sums into dw, db. */
int ttmi_bn2d_bwd_reduce(int64_t M, int C, const uint16_t* dy, const uint16_t* gate, const uint16_t* x,
                         const float* mean, const float* rstd, int64_t* sums, uint16_t* g_out,
                         hipStream_t stream);
int ttmi_bn2d_bwd_apply(int64_t M, int C, const uint16_t* dy, const uint16_t* gate, const uint16_t* x,
                        const float* mean, const float* rstd, const float* w, const int64_t* sums,
                        uint16_t* dx, float* dw, float* db, hipStream_t stream);
/* Max-pool k x k / stride, -inf padding (resnet18 maxpool 3/2/1), NHWC bf16; idx (uint8 per
 * output element) = the window tap of the max, first on ties.  Backward gathers. */
int ttmi_maxpool_fwd(int N, int H, int W, int C, int k, int stride, int pad, const uint16_t* x,
                     uint16_t* y, uint8_t* idx, hipStream_t stream);
int ttmi_maxpool_bwd(int N, int H, int W, int C, int k, int stride, int pad, const uint16_t* dy,
                     const uint8_t* idx, uint16_t* dx, hipStream_t stream);
/* Global average pool (AdaptiveAvgPool2d(1) + flatten): y[n,c] = mean_p x[n,p,c] (bf16);
 * backward dx[n,p,c] = dy[n,c]/HW ⊙ (gate > 0 if gate != NULL). */
int ttmi_avgpool_fwd(int N, int HW, int C, const uint16_t* x, uint16_t* y, hipStream_t stream);
int ttmi_avgpool_bwd(int N, int HW, int C, const void* dy, int dy_dtype, const uint16_t* gate,
                     uint16_t* dx, hipStream_t stream);

/* ------------------------------------------------------------------------------------
 * Fused AdamW over flat fp32 buffers (torch.optim.AdamW defaults, train.py:302):
 *   t = ++(*step); p *= 1 - lr*wd; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g²;
 *   p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps).
 * hyper (device, fp64) = {lr, beta1, beta2, eps, weight_decay}; step (device int32) holds
 * t (the caller increments it with ttmi_step_inc before the update), so a captured graph
 * replays with the live step count and learning rate.  zero_grad != 0 also clears g after
 * reading it (optimizer.zero_grad folded into the update).  p_bf16 (optional)
 * receives the bf16 mirror used as GEMM operand by the next step.
 * ---------------------------------------------------------------------------------- */
/* skip_if (ABI 22, may be NULL): the device half of an id_err block.  When any of its 8 flags is
 * set, p, m, v and p_bf16 are left untouched (the step whose lookups met an id outside a table
 * updates nothing, as the reference's nn.Embedding raises before optimizer.step()); g and the
 * fixed-point accumulators are still cleared.  Same parameter in ttmi_adamw_fx /
 * ttmi_adamw_folded / ttmi_adamw_folded_skip. */
int ttmi_adamw(int64_t n, float* p, float* g, float* m, float* v, uint16_t* p_bf16,
               const double* hyper, const int32_t* step, int zero_grad, const int32_t* skip_if,
               hipStream_t stream);
/* ttmi_adamw where the gradient of elements [fx_off, fx_off + fx_len) is read from an int64
 * fixed-point accumulator fx (value = fx[i - fx_off]·2^-fx_shift; ttmi_seq_embed_bwd's
 * item-embedding rows, ABI 16) instead of g, and fx (not g) is cleared there: the train step
 * then skips the fold that would convert it into g.  fx_off, fx_len multiples of 4, fx 16-B
 * aligned; fx = NULL is ttmi_adamw. */
int ttmi_adamw_fx(int64_t n, float* p, float* g, float* m, float* v, uint16_t* p_bf16,
                  const double* hyper, const int32_t* step, int zero_grad, int64_t* fx,
                  int64_t fx_off, int64_t fx_len, int fx_shift, const int32_t* skip_if,
                  hipStream_t stream);
int ttmi_step_inc(int32_t* step, hipStream_t stream);

/* ------------------------------------------------------------------------------------
 * Elementwise helpers.
 * ---------------------------------------------------------------------------------- */
/* seeds[s] = splitmix64(splitmix64(base) ^ (*step * 64 + s)), s < n <= 256: per-site dropout
 * seeds of the current step, derived on device from the live step counter.  inc_step != 0
 * increments *step first (ttmi_step_inc in the same launch). */
int ttmi_dropout_seeds(uint64_t base, int32_t* step, uint64_t* seeds, int n, int inc_step,
                       hipStream_t stream);
/* dst[i][0:nbytes[i]] = src[i][...] for i < n <= 16 device buffers, in one launch (stages a
 * batch's tensors into a captured step's static inputs). */
int ttmi_batch_copy(int n, void* const* dst, const void* const* src, const int64_t* nbytes,
                    hipStream_t stream);
/* Input grad of an nn.Linear fused with the LayerNorm backward (and dropout backward) that
 * consume it — the reversed TransformerEncoderLayer (norm_first) sub-block
 *   dY = dH · Wᵀᵀ  (dH [M,K] bf16, wt = Wᵀ [N,K] bf16 mirror, N = 128),
 *   dx = LN'(dY; x, mean, rstd, ln_w) + res,  ln_dw += Σ dY·x̂,  ln_db += Σ dY,
 *   next = bf16(dropout(dx)) with keep over (drop_rows ? drop_rows[m] : m)*ld_drop + n,
 * replacing linear_dx + ttmi_layernorm_bwd + ttmi_dropout_bwd (reference
 * src/models/user_tower.py:37-45 TransformerEncoderLayer(norm_first=True) backward).
 * res / next / drop_rows / ln_dw / ln_db may be NULL.  N = 128: K % 128 == 0, K <= 512.
 * ABI 19: N = 256 (the reference's default width) with K in {256, 512, 768, 1024} (W streamed
 * through LDS; dh and wt each under 4 GB, ln_w 16-byte aligned). */
typedef struct ttmi_linear_ln_bwd_desc {
  int64_t M, N, K;
  const void* dh; int64_t ld_dh;        /* bf16 [M, K] */
  const void* wt; int64_t ld_wt;        /* bf16 [N, K] */
  const float* x; int64_t ldx;          /* LayerNorm input [M, N] */
  const float* mean; const float* rstd; /* [M] */
  const float* ln_w;                    /* [N] */
  const float* res; int64_t ld_res;     /* [M, N] or NULL */
  float* dx; int64_t lddx;              /* [M, N] */
  void* next; int64_t ld_next;          /* bf16 [M, N] or NULL */
  float drop_p; const uint64_t* drop_seed; int64_t ld_drop; const int32_t* drop_rows;
  float* ln_dw; float* ln_db;           /* [N], accumulated */
  float* sum_ws;   /* ABI 10; NULL: ln_dw / ln_db take float atomics.  Else [G][2][N] fp32 with
                      G = ttmi_linear_ln_bwd_sum_blocks_n(M, N): each workgroup's dw / db rows,
                      plain stores; ln_dw / ln_db are then left to a fold (ttmi_wgrad_fold with
                      {part = sum_ws (+ N for db), S = G, s_stride = 2N, M = 1}): deterministic. */
  const int32_t* res_rows; int64_t res_L;  /* ABI 13; non-NULL: res is [M / res_L, N] and its row
                      b is added only to row res_rows[b] (b = m / res_L), other rows get none —
                      the pruned last layer's gathered residual (replaces ttmi_scatter_add_rows) */
  const float* dy_add; int64_t ld_add;     /* ABI 21 (N = 128, needs res_rows): [M / res_L, N] fp32
                      added to the GEMM output dY of row res_rows[b] BEFORE the LayerNorm backward
                      — the pruned layer's query-row term dq·W_q (its dqkv keeps K / V columns only) */
} ttmi_linear_ln_bwd_desc;
int64_t ttmi_linear_ln_bwd_sum_blocks(int64_t M);           /* N = 128 */
int64_t ttmi_linear_ln_bwd_sum_blocks_n(int64_t M, int64_t N);   /* ABI 19: any supported N */
int ttmi_linear_ln_bwd(const ttmi_linear_ln_bwd_desc* d, hipStream_t stream);
/* Fused residual sub-block end + the next LayerNorm (N = 128 with K % 128 == 0, K <= 512; ABI 19:
 * N = 256 with K in {256, 512, 768, 1024}, x and w each under 4 GB, bias / LN params 16-byte aligned):
 *   out = residual + dropout(x · wᵀ + bias)   (fp32 [M, N]; dropout keep index m*ld_drop + n)
 *   y = bf16(LN(out) * ln_w + ln_b), mean / rstd = the row statistics
 * i.e. TransformerEncoderLayer(norm_first=True)'s `x = x + dropout(out_proj(...))` followed by
 * norm2(x) (or `x = x + dropout(linear2(...))` followed by the next layer's norm1(x)), the
 * ttmi_gemm(residual) + ttmi_layernorm_fwd pair in one kernel (reference
 * src/models/user_tower.py:37-45, torch TransformerEncoderLayer._sa_block/_ff_block). */
typedef struct ttmi_linear_res_ln_desc {
  int64_t M, N, K;
  const void* x; int64_t ldx;           /* bf16 [M, K] */
  const void* w; int64_t ldw;           /* bf16 [N, K] (nn.Linear weight) */
  const float* bias;                    /* [N] or NULL */
  float drop_p; const uint64_t* drop_seed; int64_t ld_drop;
  const float* residual; int64_t ld_res;/* fp32 [M, N] */
  float* out; int64_t ld_out;           /* fp32 [M, N] */
  const float* ln_w; const float* ln_b; float eps;
  void* y; int64_t ldy;                 /* bf16 [M, N] */
  float* mean; float* rstd;             /* [M] */
} ttmi_linear_res_ln_desc;
int ttmi_linear_res_ln(const ttmi_linear_res_ln_desc* d, hipStream_t stream);
/* dst[i] = transpose(src[i]) for i < n <= 16 row-major bf16 matrices of rows[i] x cols[i],
 * in one launch (the transposed weight mirrors that make nn.Linear input-grad GEMMs
 * k-major: dX = dY·W = dY·(Wᵀ)ᵀ; replaces the W-operand layout of user_tower.py's
 * TransformerEncoderLayer backward, reference src/models/user_tower.py:37-45). */
int ttmi_transpose_bf16_batch(int n, void* const* dst, const void* const* src,
                              const int64_t* rows, const int64_t* cols, hipStream_t stream);
/* ttmi_transpose_bf16_batch plus, in one extra workgroup of the same launch, the step's
 * dropout seeds exactly as ttmi_dropout_seeds(seed_base, step, seeds, n_seeds, inc_step)
 * (0 < n_seeds <= 256; n_seeds = 0: transposes only; n = 0: seeds only).  The per-step
 * prologue of the captured train step (mirror refresh after AdamW + dropout seeds of the
 * reference's nn.Dropout draws) in one dispatch.  ABI 7. */
int ttmi_transpose_bf16_batch_seeds(int n, void* const* dst, const void* const* src,
                                    const int64_t* rows, const int64_t* cols, uint64_t seed_base,
                                    int32_t* step, uint64_t* seeds, int n_seeds, int inc_step,
                                    hipStream_t stream);
/* ABI 22: the train step's whole prologue in one dispatch — ttmi_batch_copy of the n_copy
 * tensors (the batch staged into the captured graph's static inputs, the id-range flags
 * cleared, the data-parallel BatchNorm buffers restored), ttmi_transpose_bf16_batch_seeds'
 * transposes, and its seed workgroup (n_seeds seeds; n_seeds = 0 with inc_step: only the step
 * count advances, ttmi_step_inc).  Issued on the stream ahead of the graph replay (the copy
 * sources change every step), it replaces one launch per step; same semantics as the three. */
int ttmi_step_prologue(int n_copy, void* const* cdst, const void* const* csrc,
                       const int64_t* nbytes, int n_tr, void* const* tdst, const void* const* tsrc,
                       const int64_t* rows, const int64_t* cols, uint64_t seed_base, int32_t* step,
                       uint64_t* seeds, int n_seeds, int inc_step, hipStream_t stream);
/* dst = bf16(src) (parameter mirror for bf16 GEMM operands). */
int ttmi_cast_f32_bf16(int64_t n, const float* src, uint16_t* dst, hipStream_t stream);
/* Residual-branch dropout backward (TransformerEncoderLayer dropout1/dropout2):
 * dy[m,n] = dx[m,n]·keep(r(m)*ld_drop+n)/(1-p) cast to dtype, r(m) = drop_rows ? drop_rows[m]
 * : m; colsum[n] += dy[m,n] (bias grad, may be NULL). */
int ttmi_dropout_bwd(int dtype, int64_t M, int N, const float* dx, int64_t ldx, float drop_p,
                     const uint64_t* drop_seed, int64_t ld_drop, const int32_t* drop_rows,
                     void* dy, int64_t ldy, float* colsum, hipStream_t stream);
/* colsum[n] += Σ_m x[m*ldx+n]  (bias grads of GEMMs fed by attention backward). */
int ttmi_colsum(int dtype, int64_t M, int N, const void* x, int64_t ldx, float* colsum,
                hipStream_t stream);

/* ------------------------------------------------------------------------------------
 * Last-layer pruning (SURVEY §8d F_min).  The last encoder layer's output is consumed only
 * at the last valid position of each sequence (user_tower.py:118-132) and nothing after its
 * attention mixes tokens, so it needs K/V for every token but Q, the attention output,
 * out_proj, FFN and both residual adds only for B gathered rows.  Dropout indices stay the
 * full-tensor ones (row-mapped), so results equal the unpruned layer's.
 * ---------------------------------------------------------------------------------- */
/* rows[b] = b*L + max(Σ_l (len_src[b,l] != 0) - 1, 0). */
int ttmi_last_rows(int B, int L, const int64_t* len_src, int32_t* rows, hipStream_t stream);
/* ttmi_last_rows + ttmi_gather_rows in one launch. */
int ttmi_last_rows_gather(int B, int L, int D, const int64_t* len_src, const float* x,
                          int32_t* rows, float* out, hipStream_t stream);
/* out[b,:] = x[rows[b],:] (fp32, row width D). */
int ttmi_gather_rows(int B, int D, const float* x, const int32_t* rows, float* out,
                     hipStream_t stream);
/* dst[rows[b],:] += src[b,:] (rows distinct). */
int ttmi_scatter_add_rows(int B, int D, const float* src, const int32_t* rows, float* dst,
                          hipStream_t stream);
/* Single-query causal attention for query row rows[b] of each sequence (position
 * p = rows[b] - b*L): keys j <= p with key_valid[b,j] != 0; dropout idx as ttmi_mha_fwd
 * with i = p.  qkv [B*L, 3HDh]; ctx [B, HDh]; lse [B*H]. */
int ttmi_mha_q1_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                    const int64_t* key_valid, const int32_t* rows, float drop_p,
                    const uint64_t* drop_seed, void* ctx, float* lse, hipStream_t stream);
/* ttmi_mha_q1_fwd with the last-valid rows found in the same launch (ABI 13): rows[b] =
 * b·L + max(len_b - 1, 0), len_b = the count of non-zero key_valid[b, :] (the reference's
 * right-padding gather, user_tower.py:131-136), x_rows[b, :] = x[rows[b], :] (fp32 [M, H·Dh]),
 * then the one-query attention of ttmi_mha_q1_fwd.  Replaces ttmi_last_rows_gather +
 * ttmi_mha_q1_fwd. */
int ttmi_mha_q1_gather_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                           const int64_t* key_valid, const float* x, int32_t* rows, float* x_rows,
                           float drop_p, const uint64_t* drop_seed, void* ctx, float* lse,
                           hipStream_t stream);
/* ttmi_mha_q1_gather_fwd whose query rows are projected in the launch (ABI 21; the pruned last
 * encoder layer, user_tower.py:111-116 evaluated only where :131-136 reads it): for each
 * gathered row r, q = a_in[r]·wq[h·Dh ..]ᵀ + bq (a_in [B·L, 128] bf16 normed rows, wq the first
 * 128 rows of in_proj_weight, bq its first 128 biases, fp32 sums rounded to bf16), written into
 * qkv[r, 0:128]; qkv's K / V columns come from the caller (a 256-column projection), its other
 * Q entries are never read.  bf16, H·Dh = 128 with Dh = 32, L <= 64; `it` (nullable): the item
 * head's stage A on the same grid, as ttmi_mha_q1_gather_item_fwd. */
struct ttmi_item_head_desc;
int ttmi_mha_q1_proj_gather_fwd(int B, int L, int H, int Dh, void* qkv, const int64_t* key_valid,
                                const void* a_in, const void* wq, const float* bq, const float* x,
                                int32_t* rows, float* x_rows, float drop_p, const uint64_t* drop_seed,
                                void* ctx, float* lse, const struct ttmi_item_head_desc* it,
                                hipStream_t stream);
/* The pruned layer's one-query backward for the K / V-only in_proj input grad (ABI 21; bf16,
 * H = 4, Dh = 32, L <= 64): dqkv's K / V columns as ttmi_mha_q1_bwd writes them, its Q columns
 * left untouched, and
 *   dq_rows[b] = bf16(dQ of row rows[b])   a_rows[b] = a_in[rows[b]]      (bf16 [B, 128])
 *   dyq[b]     = dq_rows[b]·W_q (fp32 [B, 128]; wqt = in_projᵀ [128, 3·128], row-major, ld_wqt)
 * so that the LN1-backward panel takes K = 256 (dy_add = dyq) and in_proj's Q-row weight
 * gradient is a B-row GEMM (dq_rows, a_rows).  bn: ttmi_mha_q1_bnr_bwd's co-launched BatchNorm1d
 * backward (may be NULL). */
typedef struct ttmi_q1_kv_bwd_desc {
  int B, L, H, Dh;
  const void* qkv; const int64_t* key_valid; const int32_t* rows; const float* lse; const void* dctx;
  float drop_p; const uint64_t* drop_seed;
  void* dqkv;
  const void* wqt; int64_t ld_wqt; const void* a_in;
  void* dq_rows; void* a_rows; float* dyq;
  const struct ttmi_bn_bwd_desc* bn;
} ttmi_q1_kv_bwd_desc;
int ttmi_mha_q1_kv_bwd(const ttmi_q1_kv_bwd_desc* d, hipStream_t stream);
/* Backward: writes the full dqkv [B*L, 3HDh] (dQ only on the query rows, zero elsewhere;
 * dK, dV on every row). */
int ttmi_mha_q1_bwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                    const int64_t* key_valid, const int32_t* rows, const float* lse,
                    const void* dctx, float drop_p, const uint64_t* drop_seed, void* dqkv,
                    hipStream_t stream);
/* BatchNorm1d backward arguments of ttmi_batchnorm_bwd as a descriptor (ABI 18). */
typedef struct ttmi_bn_bwd_desc {
  int dtype, B, C;
  const float* dy; const float* z; const float* w; const float* mean; const float* rstd;
  const void* y; float gate_scale; int gated;
  float* dz; float* dw; float* db; void* dz16;
} ttmi_bn_bwd_desc;
/* ttmi_mha_q1_bwd with ttmi_batchnorm_bwd(bn) on the same grid (ABI 18; bn may be NULL): the
 * item head's BatchNorm1d backward (item_tower.py:125) does not depend on the user tower's
 * attention, so its column blocks run on the one-query launch's grid (L <= 64, bn->B <= 1024;
 * otherwise two launches).  Results equal the two separate calls. */
int ttmi_mha_q1_bnr_bwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                        const int64_t* key_valid, const int32_t* rows, const float* lse,
                        const void* dctx, float drop_p, const uint64_t* drop_seed, void* dqkv,
                        const ttmi_bn_bwd_desc* bn, hipStream_t stream);

/* ------------------------------------------------------------------------------------
 * mDeBERTa-v3 text encoder (cfg 4; reference src/models/item_tower.py:41-83 = transformers
 * DebertaV2Model + peft LoRA + masked mean-pool; modeling_deberta_v2.py).  d_head = 64.
 * ---------------------------------------------------------------------------------- */
/* DebertaV2Embeddings.forward: y = dropout(LN(table[ids]) · mask) per token row (H % 64 == 0);
 * y32 (fp32 [M,H], may be NULL) and y16 (bf16, row stride ld16). table is the bf16 copy of
 * word_embeddings.weight ([V, H]); mask may be NULL.  ABI 20: an id outside [0, V) reads the
 * clamped row and sets id_err[TTMI_IDERR_TEXT]. */
int ttmi_deb_embed_fwd(int64_t M, int H, const int64_t* ids, const uint16_t* table,
                       const float* ln_w, const float* ln_b, float eps, const int64_t* mask,
                       float drop_p, const uint64_t* drop_seed, float* y32, uint16_t* y16,
                       int64_t ld16, int64_t V, int32_t* id_err, hipStream_t stream);
/* Post-LayerNorm (DebertaV2SelfOutput / DebertaV2Output LayerNorm(h + residual)): y = LN(z),
 * z fp32 [M,H]; y32 (fp32, may be NULL) and y16 (bf16, stride ld16, may be NULL); mean/rstd.
 * yq / yv (bf16 [M,H], may be NULL; H % 256 == 0): bf16(dropout(y)) with the next layer's
 * peft lora_dropout masks of query_proj / value_proj (seed_q / seed_v, keep index m*H + n). */
int ttmi_deb_ln_fwd(int64_t M, int H, const float* z, const float* ln_w, const float* ln_b,
                    float eps, float* y32, uint16_t* y16, int64_t ld16, float* mean,
                    float* rstd, uint16_t* yq, uint16_t* yv, float drop_p, const uint64_t* seed_q,
                    const uint64_t* seed_v, hipStream_t stream);
/* Disentangled self-attention (DisentangledSelfAttention with share_att_key, c2p|p2c):
 *   score[i,j] = (Q_i·K_j + Q_i·posK[δ(i-j)] + K_j·posQ[δ(i-j)]) · inv_scale, masked by
 *   mask_i·mask_j (finfo.min), softmax, dropout(p), ·V.  δ = delta[i - j + S - 1] =
 *   clamp(log-bucket(i - j) + span, 0, npos - 1) (make_log_bucket_position).  Q/K/V rows are
 *   b·S + s with head h at column h·64 (ldqkv); posq/posk are [npos, ·] (ldpos) projections of
 *   the LayerNorm'd relative table; ctx like Q; lse [B, nh, S] fp32 (saved for backward).
 * Backward: dq/dk/dv (bf16, lddqkv) from dctx, recomputing the scores; posK gets no gradient
 * (frozen).  With lora_u != NULL (the query_proj LoRA down-projection of the relative table,
 * [npos, 8] fp32) it also writes the rank-8 contractions that carry the LoRA gradient through
 * posQ = query_proj(rel): lora_hu [B·S, nh, 8] = Σ_i dS_ij·u[δ_ij] and lora_pb [npos, 8]
 * = Σ_{b,h} Σ_ij dS_ij·(K_j·Bq_h)[δ_ij] (overwritten), with lora_bq = lora_B of query_proj [nh·64, 8] fp32 and dS the
 * gradient of the unscaled score terms.  S <= 256.
 * Padded tail: let end_b = 1 + the last position with mask != 0.  64-row blocks at or past
 * end_b are skipped (as keys they are masked for every valid query; as queries they reach
 * nothing the encoder returns): their ctx rows are written as 0 and lse as 0, and padded
 * query rows inside a live block attend uniformly over the live blocks' keys instead of all S
 * (a don't-care value: the masked mean-pool never reads it).  Backward requires dctx == 0 on
 * padded rows (the mean-pool's gradient is 0 there); outputs on valid rows, and every
 * gradient, are then those of the full computation (padded-block gradients are exactly 0). */
typedef struct ttmi_dis_attn_desc {
  int B, S, nh, d_head, npos;
  const void* q; const void* k; const void* v; int64_t ldqkv;
  const void* posq; const void* posk; int64_t ldpos;
  const int64_t* mask;
  const int16_t* delta;
  float inv_scale;
  float drop_p; const uint64_t* drop_seed;
  void* ctx; int64_t ldctx;
  float* lse;
  const void* dctx; int64_t lddctx;
  void* dq; void* dk; void* dv; int64_t lddqkv;
  const float* lora_u; const float* lora_bq; float* lora_hu; float* lora_pb;
  float* dq_scratch;      /* backward: fp32 workspace of >= B·nh·S floats (D_i = dO_i·O_i) */
  float* lora_pbx;        /* backward with LoRA: fp32 workspace of ttmi_dis_attn_pbx_floats()
                             (per block pair, PB over the pair's expanded window rows) */
  const int32_t* order;   /* ABI 11; NULL or ttmi_dis_attn_order()'s [B] batch order: one
                             workgroup per (batch, head) runs every block pair of the sequence,
                             longest sequences first (the longest-processing-time order keeps
                             the last wave of workgroups short) */
} ttmi_dis_attn_desc;
int ttmi_dis_attn_fwd(const ttmi_dis_attn_desc* d, hipStream_t stream);
int ttmi_dis_attn_bwd(const ttmi_dis_attn_desc* d, hipStream_t stream);
int64_t ttmi_dis_attn_pbx_floats(int B, int S, int nh);
/* order [B] int32: the batch indices sorted by live 64-row block count (1 + the last position
 * with mask != 0, rounded up to 64) in descending order.  One launch per batch mask; every
 * layer's ttmi_dis_attn_fwd/bwd of that batch reuses it. */
int ttmi_dis_attn_order(const int64_t* mask, int B, int S, int32_t* order, hipStream_t stream);

/* The item tower's late-fusion MLP forward in training mode (reference item_tower.py:122-129:
 * Linear(512, 512) -> BatchNorm1d(512) -> ReLU -> Dropout -> Linear(512, D) -> LayerNorm(D),
 * D = 128) in three launches instead of five (ABI 14): modal16 = bf16(modal) and
 * z = modal16·W0ᵀ + b0 in one; the BatchNorm + ReLU + dropout of ttmi_batchnorm_fwd (batch
 * statistics, running stats with momentum, keep index m·512 + n; running_* / num_batches_tracked
 * may be NULL) into y1 (bf16), bn_mean, bn_rstd; y2 = y1·W4ᵀ + b4 (fp32) and out = LN(y2) with
 * m5 / r5 in one.  W0 [512, 512], W4 [128, 512] bf16 row-major; ws unused (may be NULL). */
typedef struct ttmi_item_head_desc {
  int B, K, N1, D;
  const float* modal; const void* w0; const float* b0;
  const float* bn_w; const float* bn_b; float bn_eps; float momentum;
  float* running_mean; float* running_var; int64_t* num_batches_tracked;
  float drop_p; const uint64_t* drop_seed;
  const void* w4; const float* b4; const float* ln_w; const float* ln_b; float ln_eps;
  void* modal16; float* z; float* bn_mean; float* bn_rstd; void* y1; float* y2;
  float* out; float* m5; float* r5;
  float* ws;
  float* out_hat; float* out_norm;   /* ABI 15, optional (NULL): F.normalize(out) and ||out|| */
  /* ABI 15, optional (NULL: a separate BatchNorm launch): with B <= 512 the BatchNorm batch
   * statistics are merged inside stage A (bn_part [ttmi_item_head_bn_part_floats(B)] scratch,
   * bn_cnt [ttmi_item_head_bn_counter_bytes] zero on entry and left zero) and applied in C. */
  float* bn_part; int32_t* bn_cnt;
} ttmi_item_head_desc;
int64_t ttmi_item_head_bn_part_floats(int B);
int64_t ttmi_item_head_bn_counter_bytes(int B);
int ttmi_item_head_fwd(const ttmi_item_head_desc* d, hipStream_t stream);

/* User tower head, one launch (ABI 12; reference user_tower.py:37-57, :131-144) on the B
 * gathered last-valid rows of the pruned last encoder layer (bf16 operands, fp32 math):
 *   x1 = res + drop1(ctx·Woᵀ + bo); a2 = LN2(x1) (m2, r2); h = dropf(relu(a2·W1ᵀ + b1));
 *   x2 = x1 + drop2(h·W2ᵀ + b2); comb = [x2, G[gender], C[country]] (rows[b] = b);
 *   z = comb·Wf0ᵀ + bf0; az = relu(LN(z)) (mz, rz); u = az·Wf3ᵀ + bf3.
 * Weights are k-major bf16 [out, in] (Wo, W1, W2, Wf3 with ld = in; Wf0 [D, D + dg + dc]);
 * dropout indices drop_rows[b]·N + n with N the Linear's output width (the unfused
 * ttmi_gemm's ld_drop).  D == 128, F % 256 == 0 and F <= 512, dg == 16, dc == 32. */
typedef struct ttmi_user_head_desc {
  int B, D, F, dg, dc;
  float eps;
  const void* ctx; const float* res; const int32_t* drop_rows;
  const void* wo; const float* bo; const float* n2w; const float* n2b;
  const void* w1; const float* b1; const void* w2; const float* b2;
  const int64_t* gender; const float* G; const int64_t* country; const float* C;
  const void* wf0; const float* bf0; const float* lnw; const float* lnb;
  const void* wf3; const float* bf3;
  float d1_p; const uint64_t* d1_seed;
  float dff_p; const uint64_t* dff_seed;
  float d2_p; const uint64_t* d2_seed;
  float* x1; void* a2; float* m2; float* r2; void* h; void* comb; int32_t* rows;
  float* z; void* az; float* mz; float* rz; float* u;
  float* u_hat; float* u_norm;       /* ABI 15, optional (NULL): F.normalize(u) and ||u|| */
  int n_genders, n_countries;        /* ABI 20: rows of G / C; an id outside its table reads the */
  int32_t* id_err;                   /* clamped row and sets id_err[TTMI_IDERR_GENDER / _COUNTRY] */
  void* ffn_ws;                      /* ABI 21, optional: ttmi_user_head_ffn_ws_bytes(B, F) bytes, */
                                     /* zero before first use (every launch leaves it reusable): */
                                     /* the FFN runs split over its hidden units, F / 128 */
                                     /* workgroups per 16-row block, whose last arriver sums the */
                                     /* partials in split order and runs the fusion MLP */
} ttmi_user_head_desc;
/* ABI 21: D = 256 with F = 1024 (the reference's default width) is served by the FFN-split
 * kernel only: ffn_ws is required there and no item head stage may ride in the launch. */
int ttmi_user_head_fwd(const ttmi_user_head_desc* d, hipStream_t stream);
/* Bytes of ffn_ws for B rows and FFN width F (sized for D = 256). */
int64_t ttmi_user_head_ffn_ws_bytes(int B, int F);
/* Its backward, one launch (ABI 12), from du (bf16 [B, D]) and the forward's saved values:
 *   daz = du·Wf3; dz = LNᵀ(daz ⊙ [az > 0]); dcomb = dz·Wf0 (dG[gender] / dC[country] +=);
 *   dy2 = drop2ᵀ(dcomb[:, :D]); dz1 = (dy2·W2) ⊙ [h > 0]·ffn_scale;
 *   dx1 = LN2ᵀ(dz1·W1) + dcomb[:, :D]; dy1 = drop1ᵀ(dx1); dctx = dy1·Wo.
 * The *t weights are the transposed k-major mirrors ([in, out]).  Outputs dz16, dy2, dz1, dy1
 * (bf16: the weight-gradient GEMMs' dY operands), dx1 (fp32), dctx (bf16).  ws
 * [ttmi_user_head_bwd_ws_floats(B)] receives per-16-row-block column sums of the four
 * LayerNorm parameter gradients (dlnw, dlnb, dn2w, dn2b, [nblk][4][D], nblk = ceil(B / 16);
 * the size function covers D = 256) to be folded.  ABI 21: D = 256 with F = 1024 runs on
 * the FFN-split kernel (ffn_ws required, no item head co-launch), as the forward.
 * ABI 16: dG / dC are int64 fixed-point accumulators ([n_genders][dg], [n_countries][dc],
 * scale 2^36, TTMI_FX_GRAD_SHIFT; zero on entry): adds in any order give the same bits.  The
 * caller converts them into the fp32 gradients with a ttmi_fold_desc (fx_shift = 36, S = 1,
 * accumulate = 3). */
#define TTMI_FX_GRAD_SHIFT 36
#define TTMI_FX_STAT_SHIFT 24
typedef struct ttmi_user_head_bwd_desc {
  int B, D, F, dg, dc;
  float ffn_scale;
  const void* du; const void* az; const float* z; const float* mz; const float* rz;
  const void* h; const float* x1; const float* m2; const float* r2;
  const int32_t* drop_rows; const int64_t* gender; const int64_t* country;
  const void* wf3t; const void* wf0t; const void* w2t; const void* w1t; const void* wot;
  const float* lnw; const float* n2w;
  float d1_p; const uint64_t* d1_seed;
  float d2_p; const uint64_t* d2_seed;
  int64_t* dG; int64_t* dC;
  void* dz16; void* dy2; void* dz1; float* dx1; void* dy1; void* dctx; float* ws;
  int n_genders, n_countries;        /* ABI 20: ids clamped into the tables as in the forward */
  void* ffn_ws;                      /* ABI 21, optional: as ttmi_user_head_desc::ffn_ws (the */
                                     /* same size; the backward's FFN split over hidden units) */
} ttmi_user_head_bwd_desc;
int ttmi_user_head_bwd(const ttmi_user_head_bwd_desc* d, hipStream_t stream);
int64_t ttmi_user_head_bwd_ws_floats(int B);

/* Co-launched heads (ABI 15).  The user head kernels occupy one workgroup per 16 rows (32 of
 * 256 CUs at B = 512); the item tower's row-local head work is independent of them, so it
 * rides in the same launch on the idle CUs (workgroups past the user head's):
 *  - ttmi_item_head_fwd_stages: ttmi_item_head_fwd split by stage mask 1 = A (cast +
 *    Linear 0), 2 = BatchNorm + ReLU + dropout, 4 = C (Linear 4 + LayerNorm), in that order;
 *    ttmi_item_head_fwd == stages 7.
 *  - ttmi_user_item_head_fwd: ttmi_user_head_fwd plus item stage A of `it` (NULL: user head
 *    only).  Stages 2 | 4 must follow.
 *  - ttmi_item_head_bwd_c: the item head backward's row-local part (replaces the
 *    ttmi_layernorm_bwd + Linear-4 input-grad launches of item_tower.py:122-129 under
 *    autograd): dy2 = LayerNorm(fusion_layer.5) backward of dout (bf16 [B, D] out), dy1 =
 *    dy2·W4 (fp32 [B, N1]; w4t = W4ᵀ [N1, D] bf16); ws [ttmi_item_head_bwd_ws_floats(B)]
 *    receives per-16-row-block column sums of the LN weight / bias gradients ([nblk][2][D]).
 *  - ttmi_user_item_head_bwd: ttmi_user_head_bwd plus ttmi_item_head_bwd_c of `it` (NULL:
 *    user head only).  D == 128, N1 == 512. */
typedef struct ttmi_item_head_bwd_desc {
  int B, D, N1;
  const float* dout; const float* y2; const float* m5; const float* r5; const float* ln_w;
  const void* w4t;
  void* dy2; float* dy1; float* ws;
} ttmi_item_head_bwd_desc;
int ttmi_item_head_fwd_stages(const ttmi_item_head_desc* d, int stages, hipStream_t stream);
int ttmi_user_item_head_fwd(const ttmi_user_head_desc* d, const ttmi_item_head_desc* it,
                            hipStream_t stream);
int ttmi_item_head_bwd_c(const ttmi_item_head_bwd_desc* d, hipStream_t stream);
int64_t ttmi_item_head_bwd_ws_floats(int B);
int ttmi_user_item_head_bwd(const ttmi_user_head_bwd_desc* d, const ttmi_item_head_bwd_desc* it,
                            hipStream_t stream);
/* ABI 18: the item head's stage A on the one-query forward's grid, stage C on the user head's.
 *  - ttmi_mha_q1_gather_item_fwd: ttmi_mha_q1_gather_fwd plus item stage A of `it` (with its
 *    fused BatchNorm statistics), dispatched first on the same grid (NULL: attention only).
 *  - ttmi_user_item_head_fwd_c: ttmi_user_head_fwd plus item stage C of `it` (BatchNorm +
 *    ReLU + dropout + Linear 4 + LayerNorm [+ l2norm]); needs the fused statistics of stage A
 *    (it->bn_part / bn_cnt, B <= 512).  Together: the item head costs no launch of its own. */
int ttmi_mha_q1_gather_item_fwd(int dtype, int B, int L, int H, int Dh, const void* qkv,
                                const int64_t* key_valid, const float* x, int32_t* rows, float* x_rows,
                                float drop_p, const uint64_t* drop_seed, void* ctx, float* lse,
                                const ttmi_item_head_desc* it, hipStream_t stream);
int ttmi_user_item_head_fwd_c(const ttmi_user_head_desc* d, const ttmi_item_head_desc* it,
                              hipStream_t stream);
/* ttmi_user_head_fwd plus BOTH item stages in one launch (ABI 18): stage A's workgroups, then
 * stage C's, which wait inside the launch (a bounded poll of an arrival count in it->bn_cnt)
 * until A's column-quarter mergers have published the BatchNorm statistics (handed over by
 * write-through stores and loads).  Needs the fused statistics (B <= 512).  bn_cnt must hold
 * ttmi_item_head_bn_counter_bytes(B) zero bytes; every call leaves them zero except the last
 * word, which a C workgroup sets to 1 if its poll timed out (then its outputs are invalid; ABI
 * 20: d->id_err[TTMI_IDERR_HEAD_POLL] is set too, so the host can raise). */
int ttmi_user_item_head_fwd_ac(const ttmi_user_head_desc* d, const ttmi_item_head_desc* it,
                               hipStream_t stream);
/* y = GELU(x) (erf form), bf16, n % 8 == 0 (DebertaV2Intermediate). */
int ttmi_deb_gelu(int64_t n, const uint16_t* x, uint16_t* y, hipStream_t stream);
/* TextEncoder mean-pool (item_tower.py:73-80): out[b] = Σ_s m·x[b,s] / max(Σ_s m, 1e-9);
 * backward dx[b,s] = m·dout[b] / max(Σ m, 1e-9).  x, dx fp32 [B·S, H]. */
int ttmi_deb_pool_fwd(int B, int S, int H, const float* x, const int64_t* mask, float* out,
                      hipStream_t stream);
int ttmi_deb_pool_bwd(int B, int S, int H, const float* dout, const int64_t* mask, float* dx,
                      hipStream_t stream);

/* Rank-8 LoRA weight gradient (peft LoRA on query_proj/value_proj, item_tower.py:51-59):
 * C[m·ldc_m + c·ldc_c] += alpha · Σ_r W[r·ldw + m] · S[r·lds + (m / group)·sgs + c] for
 * m < Mw (Mw % 8 == 0), c < 8, r < R.  W bf16; S bf16 (s_f32 = 0) or fp32 (s_f32 = 1).
 * dB = dYᵀ·t (group = Mw), dA = dLᵀ·drop(x) (ldc_m = 1), and the relative-path
 * Σ_j K_jᵀ·HU_j per head (group = 64, sgs = 8).  acc (ABI 16): int64 scratch in C's layout
 * (element (m, c) at m·ldc_m + c·ldc_c), zero on entry and left zero: the per-workgroup
 * partials are summed there in fixed point (order-independent, so C is bit-reproducible),
 * then added into C by a second launch. */
int ttmi_skinny_wgrad(int64_t R, int Mw, const uint16_t* W, int64_t ldw, const void* S, int s_f32,
                      int64_t lds, int group, int sgs, float alpha, float* C, int64_t ldc_m,
                      int64_t ldc_c, int64_t* acc, hipStream_t stream);
/* LoRA input gradient of query_proj + value_proj: dx[m, n] += scale · (drop_q(dL[m, 0:8]·Aq[:, n])
 * + drop_v(dL[m, 8:16]·Av[:, n])), masks regenerated from the forward's LoRA-dropout seeds at
 * index m·ld_drop + n.  dL bf16 [M, ld_dl >= 16]; Aq, Av bf16 [8, H]; dx fp32. */
int ttmi_lora_dx(int64_t M, int H, const uint16_t* dL, int64_t ld_dl, const uint16_t* aq,
                 const uint16_t* av, float scale, float drop_p, const uint64_t* seed_q,
                 const uint64_t* seed_v, int64_t ld_drop, float* dx, int64_t ld_dx,
                 hipStream_t stream);

/* ------------------------------------------------------------------------------------
 * Item-modality preprocessing (the batch contract of the reference's missing
 * src/data/dataset.py; transforms per report/chapters/dataset.tex:23 and :38).
 * ---------------------------------------------------------------------------------- */
/* Mel power spectrogram (librosa 0.11 melspectrogram: center=True, pad_mode='constant',
 * n_fft = 2048, periodic Hann `window` [2048], power 2): x [B, ldx] fp32 waveforms of N
 * samples -> out [B, n_mels, 1 + N/hop].  twiddle [1024][2] = exp(-2πi k/2048); the filterbank
 * is given sparsely: band m has band_len[m] weights band_w[band_off[m]..] on rfft bins
 * band_start[m].. */
int ttmi_mel_power(int B, int64_t N, const float* x, int64_t ldx, int hop, int n_mels,
                   const float* window, const float* twiddle, const int* band_start,
                   const int* band_len, const int* band_off, const float* band_w, float* out,
                   hipStream_t stream);
/* In place, per clip of n values: power_to_db(ref = max, amin, top_db) then min-max to [0,1]
 * (a clip with no dynamic range becomes all zeros). */
int ttmi_mel_db_minmax(int B, int64_t n, float amin, float top_db, float* mel, hipStream_t stream);
/* Album covers: img = B uint8 HWC images (stride ld_img bytes) -> antialiased bilinear resize to
 * OH x OW (align_corners = False) -> (v/255 - mean[c]) / std[c] (mean, std: 3 host floats) ->
 * out_nchw fp32 [B, 3, OH, OW] and/or out_nhwc8 bf16 [B, OH, OW, 8] (channels 3..7 zero). */
int ttmi_cover_prep(int B, int H, int W, const uint8_t* img, int64_t ld_img, int OH, int OW,
                    const float* mean, const float* std, float* out_nchw, uint16_t* out_nhwc8,
                    hipStream_t stream);

/* ------------------------------------------------------------------------------------
 * Global retrieval (reference src/evaluate_metrics.py:107-192 calculate_metrics_global):
 * scores = û·Îᵀ (ttmi_gemm) then per row the top-K item indices.
 * ---------------------------------------------------------------------------------- */
/* Per row r of scores [R, V] (fp32, row stride ld): the K largest values sorted descending
 * (ties: lower index first) -> out_val [R, K], out_idx [R, K] (int64).  skip_first: column 0
 * counts as -inf (the padding item, evaluate_metrics.py:157).  K <= 64, K <= V. */
int ttmi_topk_rows(int R, int V, int K, const float* scores, int64_t ld, int skip_first,
                   float* out_val, int64_t* out_idx, hipStream_t stream);
/* Catalogue index rows (evaluate_metrics.py:58-104 compute_all_item_embeddings,
 * inference.py:175-201 index_catalog): for each of n item-tower outputs x [n][ldx] (fp32),
 * e = x / max(|x|, 1e-12) (get_item_embedding), NaN -> 0, e / max(|e|, 1e-8), written to row
 * ids[r] of the dense [V][D] index (ids outside [0, V) skipped and flagged in
 * id_err[TTMI_IDERR_CATALOGUE], ABI 20; other rows untouched).  ABI 10. */
int ttmi_catalogue_rows(int n, int D, const float* x, int64_t ldx, const int64_t* ids, int64_t V,
                        float* dense, int32_t* id_err, hipStream_t stream);
/* scores[r, ids[r, j]] = -inf for j < Lh and 0 <= id < V (serving: exclude the user's history,
 * reference src/inference.py:294-303). */
int ttmi_mask_items(int R, int V, float* scores, int64_t ld, const int64_t* ids, int Lh,
                    hipStream_t stream);
/* rank[b] = first j with idx[b, j] == target[b], or K when absent (Recall@k: rank < k,
 * NDCG@k: 1/log2(rank + 2) when rank < k). */
int ttmi_rank_of(int B, int K, const int64_t* idx, const int64_t* target, int32_t* rank,
                 hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* TTMI_H */
