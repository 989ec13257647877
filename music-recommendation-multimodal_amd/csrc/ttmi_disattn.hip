// ttmi_disattn.hip — fused disentangled self-attention of the cfg-4 text encoder
// (DebertaV2 DisentangledSelfAttention with share_att_key, c2p|p2c and log position buckets;
// reference src/models/item_tower.py:41-83 -> transformers modeling_deberta_v2.py).
//
//   score[i,j] = (Q_i·K_j + Q_i·posK[δ(i-j)] + K_j·posQ[δ(i-j)]) · inv_scale
//
// Expanded relative windows.  For a 64x64 block pair (query rows i0.., key rows j0..) every
// relative offset i - j is i0 - j0 - 63 + r with r = il - jl + 63 in [0, 127).  The kernels
// stage, per block pair, the 128-row windows PKexp[r] = posK[δ(i0 - j0 - 63 + r)] and
// PQexp[r] = posQ[δ(...)] (rows gathered through δ, so log-bucket rows repeat instead of
// being binned).  Then
//   * c2p / p2c are one MFMA product against the window each, read back at column r;
//   * the positional gradients need no binning: with SkewQ[il][r] = dS[il][il - r + 63] and
//     SkewK[jl][r] = dS[jl + r - 63][jl] (the block's raw-score gradient written along its
//     diagonals), dQ_pos = SkewQ·PKexp and dK_pos = SkewK·PQexp are plain MFMA products, and
//     the query_proj-LoRA contractions are HU = SkewK·Uexp (Uexp[r] = u[δ(...)]) and
//     PBexp = SkewKᵀ·KB (binned to δ rows by a small reduction kernel).
//
// Kernels (4 waves, 16 rows per wave, < 80 KB LDS so two workgroups share a CU):
//   dis_fwd_kernel   per (query block, head, batch): online softmax over key blocks -> ctx, lse
//   dis_dq_kernel    per (query block, head, batch): recomputes P, writes dQ and D = dO·O
//   dis_dkv_kernel   per (key block, head, batch): recomputes Pᵀ, writes dK, dV, HU, PBexp
//   dis_pb_kernel    sums PBexp over (batch, head) and bins its rows to δ -> PB [npos, 8]
// Per block pair each kernel has three barriers: after staging, after the shared window
// product (p2c for the query-side kernels, c2p for dis_dkv), and before the next staging.
// The c2p (query side) / p2c (key side) window is private to each wave and lives in the
// LDS of the window it no longer needs (PQexp / PKexp).
#include "ttmi_common.h"

namespace {

constexpr int DH = 64;                 // head width
constexpr int TP = 144;                // LDS pitch (bytes) of a bf16 [rows][64] tile
constexpr int WIN = 128;               // expanded window rows per block pair
constexpr int WP = 272;                // LDS pitch (bytes) of a bf16 [rows][128] window product
constexpr int UP = 32;                 // LDS pitch (bytes) of the bf16 [rows][16] LoRA images
constexpr float FMIN = -3.4028234663852886e38f;   // torch.finfo(torch.float32).min
constexpr int MAXS = 256;

typedef __attribute__((ext_vector_type(4))) short s16x4_t;

TTMI_DEV uint2 lds8(const char* p) { return *reinterpret_cast<const uint2*>(p); }
TTMI_DEV uint2 lds_tr8(const char* p) {
  const s16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p));
  return __builtin_bit_cast(uint2, v);
}
// MFMA operand fragment (16 rows x 32 k; lane group g holds k = 4g..4g+3, 16+4g..16+4g+3)
// from a [row][k] bf16 image ...
template <int P>
TTMI_DEV uint4 fk(const char* s, int row0, int c, int lane) {
  const char* p = s + (row0 + (lane & 15)) * P + c * 64 + (lane >> 4) * 8;
  const uint2 lo = lds8(p), hi = lds8(p + 32);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}
// ... from a [k][row] bf16 image (transposing LDS read) ...
template <int P>
TTMI_DEV uint4 ft(const char* s, int row0, int c, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const char* p = s + (c * 32 + 4 * g + (i >> 2)) * P + (row0 + 4 * (i & 3)) * 2;
  const uint2 lo = lds_tr8(p), hi = lds_tr8(p + 16 * P);
  return make_uint4(lo.x, lo.y, hi.x, hi.y);
}
TTMI_DEV uint32_t pk2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }
// ... and from score-layout registers (tile t holds columns 16t + 4·lg + e of row lane & 15).
TTMI_DEV uint4 freg(const f32x4_t& lo, const f32x4_t& hi) {
  return make_uint4(pk2(lo[0], lo[1]), pk2(lo[2], lo[3]), pk2(hi[0], hi[1]), pk2(hi[2], hi[3]));
}
// Fragment of 16 rows of a global bf16 [rows][ld] matrix, k chunk c (same permutation as fk).
TTMI_DEV uint4 fglob(const bf16_t* base, int64_t ld, int row, int nrows, int c, int lane) {
  const int rr = min(row, nrows - 1);
  const char* p = reinterpret_cast<const char*>(base + (int64_t)rr * ld) + c * 64 + (lane >> 4) * 8;
  const uint2 lo = *reinterpret_cast<const uint2*>(p), hi = *reinterpret_cast<const uint2*>(p + 32);
  return row < nrows ? make_uint4(lo.x, lo.y, hi.x, hi.y) : make_uint4(0u, 0u, 0u, 0u);
}
TTMI_DEV void st_bf4(char* p, const f32x4_t& v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pk2(v[0], v[1]), pk2(v[2], v[3]));
}
TTMI_DEV float lds_bf(const char* base, int off_elems) {
  return bf2f(reinterpret_cast<const bf16_t*>(base)[off_elems]);
}

struct DisArgs {
  int B, S, nh, npos, nqb;
  const bf16_t* q; const bf16_t* k; const bf16_t* v; int64_t ldqkv;   // head h at column h·64
  const bf16_t* posq; const bf16_t* posk; int64_t ldpos;
  const int64_t* mask;              // [B, S]
  const int16_t* delta;             // [2S-1]: δ(i - j) at index i - j + S - 1
  float inv_scale;
  DropParams drop;                  // probs dropout, index ((b·nh + h)·S + i)·S + j
  bf16_t* ctx; int64_t ldctx;
  float* lse;                       // [B, nh, S]
  const bf16_t* dctx; int64_t lddctx;
  bf16_t* dq; bf16_t* dk; bf16_t* dv; int64_t lddqkv;
  float* dsum;                      // [B, nh, S]: D_i = dO_i·O_i (written by dis_dq)
  const float* u;                   // [npos, 8] LoRA down-projection of the relative table
  const float* bq;                  // [nh·64, 8] LoRA B of query_proj
  float* hu;                        // [B·S, nh, 8]
  float* pbx;                       // [B·nh, nqb, nqb, 128, 8]
  float* pb;                        // [npos, 8] (summed over batch and heads)
};

TTMI_DEV int win_row(const DisArgs& a, int rel) {
  rel = min(max(rel, -(a.S - 1)), a.S - 1);
  return a.delta[rel + a.S - 1];
}

// End of sequence b's attended range: 1 + the last position whose mask is set (0 if none).
// Blocks of 64 rows at or past it hold only padded tokens: as keys they are masked for every
// valid query (probability exactly 0), and as queries their outputs reach nothing the encoder
// returns (the masked mean-pool) and their gradients are exactly 0.  The kernels skip those
// blocks (block-uniform: every thread of the workgroup computes the same value).
TTMI_DEV int seq_end(const DisArgs& a, int64_t rowb, int* red) {
  if (threadIdx.x == 0) *red = 0;
  __syncthreads();
  int e = 0;
  for (int t = threadIdx.x; t < a.S; t += blockDim.x)
    if (a.mask[rowb + t] != 0) e = t + 1;
  if (e) atomicMax(red, e);
  __syncthreads();
  return *red;
}

// rows [r0, r0 + R) x 64 bf16 of src -> LDS image (pitch TP); rows >= nrows are zero.  Loads
// are unconditional from a clamped row (a guarded load compiles to a branch + vmcnt(0)).
template <int R>
TTMI_DEV void stage_rows(char* dst, const bf16_t* src, int64_t ld, int r0, int nrows, int tid) {
  constexpr int C = R * 8 / 256;
  uint4 v[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int idx = tid + 256 * c, r = idx >> 3, ch = idx & 7;
    v[c] = *reinterpret_cast<const uint4*>(src + (int64_t)min(r0 + r, nrows - 1) * ld + ch * 8);
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int idx = tid + 256 * c, r = idx >> 3, ch = idx & 7;
    const bool ok = r0 + r < nrows;
    *reinterpret_cast<uint4*>(dst + r * TP + ch * 16) =
        ok ? v[c] : make_uint4(0u, 0u, 0u, 0u);
  }
}
// Expanded window: row r = table[δ(rel0 + r)] (head slice at column h·64), r < 128.
TTMI_DEV void stage_win(char* dst, const DisArgs& a, const bf16_t* table, int rel0, int tid) {
  uint4 v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int idx = tid + 256 * c, r = idx >> 3, ch = idx & 7;
    v[c] = *reinterpret_cast<const uint4*>(table + (int64_t)win_row(a, rel0 + r) * a.ldpos + ch * 8);
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int idx = tid + 256 * c, r = idx >> 3, ch = idx & 7;
    *reinterpret_cast<uint4*>(dst + r * TP + ch * 16) = v[c];
  }
}

// Window product of 16 rows (operand fragments a0, a1) against a 128-row window image:
// acc[t] lane = C[row 16·? + li][r = 16t + 4lg + e]; written bf16 into `out` (pitch WP) rows.
TTMI_DEV void win_product(const char* win, uint4 a0, uint4 a1, char* out, int lane) {
  f32x4_t acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    Mma<bf16_t>::run(acc[t], fk<TP>(win, 16 * t, 0, lane), a0);
    Mma<bf16_t>::run(acc[t], fk<TP>(win, 16 * t, 1, lane), a1);
  }
  char* row = out + (lane & 15) * WP + (lane >> 4) * 8;
#pragma unroll
  for (int t = 0; t < 8; ++t) st_bf4(row + 32 * t, acc[t]);
}

// Zero 16 rows x 128 bf16 of a WP-pitch image (one wave).
TTMI_DEV void zero_rows16(char* img, int lane) {
  char* p = img + (lane >> 2) * WP + (lane & 3) * 64;
#pragma unroll
  for (int k = 0; k < 4; ++k) *reinterpret_cast<uint4*>(p + 16 * k) = make_uint4(0u, 0u, 0u, 0u);
}

// ------------------------------------------------------------------ query-side staging
struct QSide {
  char sK[64 * TP];
  char sV[64 * TP];
  char sPK[WIN * TP];
  char sPQ[WIN * TP];     // PQexp, then the waves' private c2p / SkewQ images (4 x 16 x WP)
  char sX[64 * WP];       // shared p2c: [key jl][r]
  float sMk[64];
};
static_assert(4 * 16 * WP <= WIN * TP, "private images must fit the PQexp window");
static_assert(sizeof(QSide) <= 80 * 1024, "two workgroups per CU");

// Stage key block j0 and the expanded windows of the pair (i0, j0), then the shared p2c
// product; returns after the barrier that publishes sX.  `priv` = this wave's image.
TTMI_DEV void qside_stage(QSide& L, const DisArgs& a, int b, int h, int i0, int j0, int tid, int w,
                          int lane) {
  const int64_t rowb = (int64_t)b * a.S;
  stage_rows<64>(L.sK, a.k + rowb * a.ldqkv + h * DH, a.ldqkv, j0, a.S, tid);
  stage_rows<64>(L.sV, a.v + rowb * a.ldqkv + h * DH, a.ldqkv, j0, a.S, tid);
  stage_win(L.sPK, a, a.posk + h * DH, i0 - j0 - 63, tid);
  stage_win(L.sPQ, a, a.posq + h * DH, i0 - j0 - 63, tid);
  if (tid < 64) {
    const int j = j0 + tid;
    L.sMk[tid] = j < a.S ? (a.mask[rowb + j] != 0 ? 1.f : 0.f) : -1.f;
  }
  __syncthreads();
  // shared p2c: this wave's 16 keys against PQexp
  win_product(L.sPQ, fk<TP>(L.sK, 16 * w, 0, lane), fk<TP>(L.sK, 16 * w, 1, lane),
              L.sX + 16 * w * WP, lane);
  __syncthreads();
}

// Masked, scaled scores of this wave's 16 query rows (i = i0 + 16w + li) against key block j0:
// sc[t][e] for key jl = 16t + 4lg + e.  Writes the private c2p image first (PQexp is dead).
TTMI_DEV void qside_scores(QSide& L, const DisArgs& a, const uint4 (&qf)[2], bool qvalid, int w,
                           int lane, f32x4_t (&sc)[4]) {
  const int li = lane & 15, lg = lane >> 4;
  char* priv = L.sPQ + 16 * w * WP;
  win_product(L.sPK, qf[0], qf[1], priv, lane);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    sc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    Mma<bf16_t>::run(sc[t], fk<TP>(L.sK, 16 * t, 0, lane), qf[0]);
    Mma<bf16_t>::run(sc[t], fk<TP>(L.sK, 16 * t, 1, lane), qf[1]);
  }
  const int il = 16 * w + li;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int jl = 16 * t + 4 * lg + e, r = il - jl + 63;
      const float raw = sc[t][e] + lds_bf(priv, li * (WP / 2) + r) + lds_bf(L.sX, jl * (WP / 2) + r);
      const float mk = L.sMk[jl];
      sc[t][e] = mk < 0.f ? -INFINITY : ((qvalid && mk > 0.f) ? raw * a.inv_scale : FMIN);
    }
}

__global__ __launch_bounds__(256, 2) void dis_fwd_kernel(DisArgs a) {
  __shared__ __attribute__((aligned(16))) QSide L;
  __shared__ int s_end;
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int S = a.S, i0 = qb * 64, i = i0 + 16 * w + li;
  const int64_t rowb = (int64_t)b * S;
  const DropKeys dk = resolve_drop(a.drop);
  const bool irow = i < S;
  const int send = seq_end(a, rowb, &s_end);
  if (i0 >= send) {                      // padded query block: finite placeholder outputs
    if (!irow) return;
    bf16_t* dst = a.ctx + (rowb + i) * a.ldctx + h * DH;
#pragma unroll
    for (int u = 0; u < 4; ++u) st_bf4(reinterpret_cast<char*>(dst + 16 * u + 4 * lg), f32x4_t{0.f, 0.f, 0.f, 0.f});
    if (lg == 0) a.lse[((int64_t)b * a.nh + h) * S + i] = 0.f;
    return;
  }
  const bool qvalid = irow && a.mask[rowb + i] != 0;
  const uint4 qf[2] = {fglob(a.q + rowb * a.ldqkv + h * DH, a.ldqkv, i, S, 0, lane),
                       fglob(a.q + rowb * a.ldqkv + h * DH, a.ldqkv, i, S, 1, lane)};
  float m_run = -INFINITY, l_run = 0.f;
  f32x4_t o[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) o[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < send; j0 += 64) {
    qside_stage(L, a, b, h, i0, j0, tid, w, lane);
    f32x4_t sc[4];
    qside_scores(L, a, qf, qvalid, w, lane, sc);
    float rmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) rmax = fmaxf(rmax, sc[t][e]);
    rmax = fmaxf(rmax, __shfl_xor(rmax, 16, 64));
    rmax = fmaxf(rmax, __shfl_xor(rmax, 32, 64));
    const float m_new = fmaxf(m_run, rmax);
    const float corr = __expf(m_run - m_new);
    float rsum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float p = __expf(sc[t][e] - m_new);
        rsum += p;
        const uint32_t idx = (uint32_t)((((int64_t)b * a.nh + h) * S + i) * S + j0 + 16 * t + 4 * lg + e);
        sc[t][e] = dk.on ? (drop_keep(dk, idx) ? p * dk.scale : 0.f) : p;
      }
    rsum += __shfl_xor(rsum, 16, 64);
    rsum += __shfl_xor(rsum, 32, 64);
    l_run = l_run * corr + rsum;
    m_run = m_new;
#pragma unroll
    for (int u = 0; u < 4; ++u) o[u] *= corr;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const uint4 af = freg(sc[2 * c], sc[2 * c + 1]);
#pragma unroll
      for (int u = 0; u < 4; ++u) Mma<bf16_t>::run(o[u], ft<TP>(L.sV, 16 * u, c, lane), af);
    }
    __syncthreads();
  }
  if (!irow) return;
  const float inv = 1.f / l_run;
  bf16_t* dst = a.ctx + (rowb + i) * a.ldctx + h * DH;
#pragma unroll
  for (int u = 0; u < 4; ++u) st_bf4(reinterpret_cast<char*>(dst + 16 * u + 4 * lg), o[u] * inv);
  if (lg == 0) a.lse[((int64_t)b * a.nh + h) * S + i] = m_run + __logf(l_run);
}

__global__ __launch_bounds__(256, 2) void dis_dq_kernel(DisArgs a) {
  __shared__ __attribute__((aligned(16))) QSide L;
  __shared__ int s_end;
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int S = a.S, i0 = qb * 64, i = i0 + 16 * w + li;
  const int64_t rowb = (int64_t)b * S;
  const DropKeys dk = resolve_drop(a.drop);
  const bool irow = i < S;
  const int send = seq_end(a, rowb, &s_end);
  if (i0 >= send) {                      // padded query block: dS = 0, so dQ = 0 and D = 0
    if (!irow) return;
    bf16_t* dst = a.dq + (rowb + i) * a.lddqkv + h * DH;
#pragma unroll
    for (int u = 0; u < 4; ++u) st_bf4(reinterpret_cast<char*>(dst + 16 * u + 4 * lg), f32x4_t{0.f, 0.f, 0.f, 0.f});
    if (lg == 0) a.dsum[((int64_t)b * a.nh + h) * S + i] = 0.f;
    return;
  }
  const bool qvalid = irow && a.mask[rowb + i] != 0;
  const uint4 qf[2] = {fglob(a.q + rowb * a.ldqkv + h * DH, a.ldqkv, i, S, 0, lane),
                       fglob(a.q + rowb * a.ldqkv + h * DH, a.ldqkv, i, S, 1, lane)};
  const uint4 of[2] = {fglob(a.dctx + rowb * a.lddctx + h * DH, a.lddctx, i, S, 0, lane),
                       fglob(a.dctx + rowb * a.lddctx + h * DH, a.lddctx, i, S, 1, lane)};
  // D_i = dO_i · O_i (lanes li, li+16, li+32, li+48 split the row)
  float Di = 0.f;
  {
    const int ic = min(i, S - 1);
    const bf16_t* o = a.ctx + (rowb + ic) * a.ldctx + h * DH + 16 * lg;
    const bf16_t* go = a.dctx + (rowb + ic) * a.lddctx + h * DH + 16 * lg;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float x[8], y[8];
      unpack8(*reinterpret_cast<const uint4*>(o + 8 * c), x);
      unpack8(*reinterpret_cast<const uint4*>(go + 8 * c), y);
#pragma unroll
      for (int e = 0; e < 8; ++e) Di += x[e] * y[e];
    }
    Di += __shfl_xor(Di, 16, 64);
    Di += __shfl_xor(Di, 32, 64);
    if (!irow) Di = 0.f;
    if (irow && lg == 0) a.dsum[((int64_t)b * a.nh + h) * S + i] = Di;
  }
  const float lse = irow ? a.lse[((int64_t)b * a.nh + h) * S + i] : 0.f;
  f32x4_t dq[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) dq[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  char* priv = L.sPQ + 16 * w * WP;
  for (int j0 = 0; j0 < send; j0 += 64) {
    qside_stage(L, a, b, h, i0, j0, tid, w, lane);
    f32x4_t sc[4], dp[4];
    qside_scores(L, a, qf, qvalid, w, lane, sc);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      dp[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      Mma<bf16_t>::run(dp[t], fk<TP>(L.sV, 16 * t, 0, lane), of[0]);
      Mma<bf16_t>::run(dp[t], fk<TP>(L.sV, 16 * t, 1, lane), of[1]);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int jl = 16 * t + 4 * lg + e;
        const float mk = L.sMk[jl];
        // a fully padded query row attends uniformly to the S keys (finfo.min everywhere);
        // its masked_fill'ed scores are constants and receive no gradient
        const float p = !irow ? 0.f : (qvalid ? __expf(sc[t][e] - lse) : (mk >= 0.f ? 1.f / (float)S : 0.f));
        const uint32_t idx = (uint32_t)((((int64_t)b * a.nh + h) * S + i) * S + j0 + jl);
        const float keep = dk.on ? (drop_keep(dk, idx) ? dk.scale : 0.f) : 1.f;
        sc[t][e] = qvalid ? p * (dp[t][e] * keep - Di) * a.inv_scale : 0.f;   // d raw score
      }
    // dQ += dS·K
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const uint4 af = freg(sc[2 * c], sc[2 * c + 1]);
#pragma unroll
      for (int u = 0; u < 4; ++u) Mma<bf16_t>::run(dq[u], ft<TP>(L.sK, 16 * u, c, lane), af);
    }
    // SkewQ[il][r] = dS[il][il - r + 63] (private image, after this wave's c2p reads)
    zero_rows16(priv, lane);
    {
      bf16_t* pr = reinterpret_cast<bf16_t*>(priv) + li * (WP / 2);
      const int il = 16 * w + li;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) pr[il - (16 * t + 4 * lg + e) + 63] = f2bf(sc[t][e]);
    }
    // dQ += SkewQ·PKexp
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint4 af = fk<WP>(priv, 0, c, lane);
#pragma unroll
      for (int u = 0; u < 4; ++u) Mma<bf16_t>::run(dq[u], ft<TP>(L.sPK, 16 * u, c, lane), af);
    }
    __syncthreads();
  }
  if (!irow) return;
  bf16_t* dst = a.dq + (rowb + i) * a.lddqkv + h * DH;
#pragma unroll
  for (int u = 0; u < 4; ++u) st_bf4(reinterpret_cast<char*>(dst + 16 * u + 4 * lg), dq[u]);
}

// ------------------------------------------------------------------ key side
struct KSide {
  char sQ[64 * TP];
  char sdO[64 * TP];
  char sPK[WIN * TP];     // PKexp, then the waves' private p2c images
  char sPQ[WIN * TP];
  char sX[64 * WP];       // shared c2p [query il][r], then SkewK [key jl][r]
  char sU[WIN * UP];      // Uexp [r][16] (8 used)
  char sKB[64 * UP];      // KB [key jl][16] (8 used)
  float sLse[64], sD[64], sQm[64];
};
static_assert(4 * 16 * WP <= WIN * TP, "private images must fit the PKexp window");
static_assert(sizeof(KSide) <= 80 * 1024, "two workgroups per CU");

// PBexp of a skipped (query block, key block) pair: zero (dis_pb sums every pair).
TTMI_DEV void zero_pbx(const DisArgs& a, int64_t bh, int qb, int kb) {
  float* dst = a.pbx + ((bh * a.nqb + qb) * a.nqb + kb) * WIN * 8;
  for (int t = threadIdx.x; t < WIN * 8 / 4; t += blockDim.x)
    reinterpret_cast<float4*>(dst)[t] = make_float4(0.f, 0.f, 0.f, 0.f);
}

__global__ __launch_bounds__(256, 2) void dis_dkv_kernel(DisArgs a) {
  __shared__ __attribute__((aligned(16))) KSide L;
  __shared__ int s_end;
  const int kb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int S = a.S, j0 = kb * 64, jl = 16 * w + li, j = j0 + jl;
  const int64_t rowb = (int64_t)b * S;
  const int64_t bh = (int64_t)b * a.nh + h;
  const DropKeys dk = resolve_drop(a.drop);
  const bool lora = a.u != nullptr;
  const bool jrow = j < S;
  const int send = seq_end(a, rowb, &s_end);
  if (j0 >= send) {                      // padded key block: masked for every valid query
    if (lora)
      for (int qb = 0; qb < a.nqb; ++qb) zero_pbx(a, bh, qb, kb);
    if (!jrow) return;
    bf16_t* pk = a.dk + (rowb + j) * a.lddqkv + h * DH;
    bf16_t* pv = a.dv + (rowb + j) * a.lddqkv + h * DH;
    const f32x4_t z = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      st_bf4(reinterpret_cast<char*>(pk + 16 * u + 4 * lg), z);
      st_bf4(reinterpret_cast<char*>(pv + 16 * u + 4 * lg), z);
    }
    if (lora && lg < 2)
      *reinterpret_cast<float4*>(a.hu + ((rowb + j) * a.nh + h) * 8 + 4 * lg) = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const bool kvalid = jrow && a.mask[rowb + j] != 0;
  const uint4 kf[2] = {fglob(a.k + rowb * a.ldqkv + h * DH, a.ldqkv, j, S, 0, lane),
                       fglob(a.k + rowb * a.ldqkv + h * DH, a.ldqkv, j, S, 1, lane)};
  const uint4 vf[2] = {fglob(a.v + rowb * a.ldqkv + h * DH, a.ldqkv, j, S, 0, lane),
                       fglob(a.v + rowb * a.ldqkv + h * DH, a.ldqkv, j, S, 1, lane)};
  if (lora) {                 // KB[jl][c] = K_j · Bq[h·64 + :, c] (bf16 image, columns 8-15 zero)
    const int r = tid >> 2, c0 = (tid & 3) * 2;
    const bf16_t* kr = a.k + (rowb + min(j0 + r, S - 1)) * a.ldqkv + h * DH;
    float s0 = 0.f, s1 = 0.f;
    for (int d = 0; d < DH; d += 8) {
      float kv[8];
      unpack8(*reinterpret_cast<const uint4*>(kr + d), kv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s0 += kv[e] * a.bq[(h * DH + d + e) * 8 + c0];
        s1 += kv[e] * a.bq[(h * DH + d + e) * 8 + c0 + 1];
      }
    }
    if (j0 + r >= S) s0 = s1 = 0.f;
    uint32_t* row = reinterpret_cast<uint32_t*>(L.sKB + r * UP);
    row[c0 / 2] = pk2(s0, s1);
    row[4 + c0 / 2] = 0u;
  }
  f32x4_t dka[4], dva[4], hua;
#pragma unroll
  for (int u = 0; u < 4; ++u) dka[u] = dva[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  hua = f32x4_t{0.f, 0.f, 0.f, 0.f};
  char* priv = L.sPK + 16 * w * WP;
  for (int qb = 0; qb < a.nqb; ++qb) {
    const int i0 = qb * 64, rel0 = i0 - j0 - 63;
    if (i0 >= send) {                    // padded query block: dS = 0 and dO = 0
      if (lora) zero_pbx(a, bh, qb, kb);
      continue;
    }
    stage_rows<64>(L.sQ, a.q + rowb * a.ldqkv + h * DH, a.ldqkv, i0, S, tid);
    stage_rows<64>(L.sdO, a.dctx + rowb * a.lddctx + h * DH, a.lddctx, i0, S, tid);
    stage_win(L.sPK, a, a.posk + h * DH, rel0, tid);
    stage_win(L.sPQ, a, a.posq + h * DH, rel0, tid);
    if (tid < 64) {
      const int i = i0 + tid;
      const bool ok = i < S;
      L.sLse[tid] = ok ? a.lse[bh * S + i] : 0.f;
      L.sD[tid] = ok ? a.dsum[bh * S + i] : 0.f;
      L.sQm[tid] = ok ? (a.mask[rowb + i] != 0 ? 1.f : 0.f) : -1.f;
    }
    if (lora) {
      const int r = tid >> 1, c0 = (tid & 1) * 4;
      const float* ur = a.u + (int64_t)win_row(a, rel0 + r) * 8 + c0;
      uint32_t* row = reinterpret_cast<uint32_t*>(L.sU + r * UP);
      row[c0 / 2] = pk2(ur[0], ur[1]);
      row[c0 / 2 + 1] = pk2(ur[2], ur[3]);
      row[4 + c0 / 2] = 0u;
      row[5 + c0 / 2] = 0u;
    }
    __syncthreads();
    // shared c2p: this wave's 16 queries against PKexp
    win_product(L.sPK, fk<TP>(L.sQ, 16 * w, 0, lane), fk<TP>(L.sQ, 16 * w, 1, lane),
                L.sX + 16 * w * WP, lane);
    __syncthreads();
    // private p2c: own 16 keys against PQexp (into the dead PKexp window)
    win_product(L.sPQ, kf[0], kf[1], priv, lane);
    f32x4_t sc[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sc[t] = dp[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      Mma<bf16_t>::run(sc[t], fk<TP>(L.sQ, 16 * t, 0, lane), kf[0]);
      Mma<bf16_t>::run(sc[t], fk<TP>(L.sQ, 16 * t, 1, lane), kf[1]);
      Mma<bf16_t>::run(dp[t], fk<TP>(L.sdO, 16 * t, 0, lane), vf[0]);
      Mma<bf16_t>::run(dp[t], fk<TP>(L.sdO, 16 * t, 1, lane), vf[1]);
    }
    f32x4_t pd[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float4 lse4 = *reinterpret_cast<const float4*>(L.sLse + 16 * t + 4 * lg);
      const float4 d4 = *reinterpret_cast<const float4*>(L.sD + 16 * t + 4 * lg);
      const float4 qm4 = *reinterpret_cast<const float4*>(L.sQm + 16 * t + 4 * lg);
      const float lse_[4] = {lse4.x, lse4.y, lse4.z, lse4.w}, d_[4] = {d4.x, d4.y, d4.z, d4.w};
      const float qm_[4] = {qm4.x, qm4.y, qm4.z, qm4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int il = 16 * t + 4 * lg + e, r = il - jl + 63;
        const float raw = sc[t][e] + lds_bf(L.sX, il * (WP / 2) + r) + lds_bf(priv, li * (WP / 2) + r);
        const bool qv = qm_[e] > 0.f, irow = qm_[e] >= 0.f;
        const float s = (qv && kvalid) ? raw * a.inv_scale : FMIN;
        const float p = (!irow || !jrow) ? 0.f : (qv ? __expf(s - lse_[e]) : 1.f / (float)S);
        const uint32_t idx = (uint32_t)((bh * S + i0 + il) * S + j);
        const float keep = dk.on ? (drop_keep(dk, idx) ? dk.scale : 0.f) : 1.f;
        pd[t][e] = p * keep;
        sc[t][e] = qv ? p * (dp[t][e] * keep - d_[e]) * a.inv_scale : 0.f;      // d raw score
      }
    }
    // dV += Pdᵀ·dO, dK += dSᵀ·Q
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const uint4 ap = freg(pd[2 * c], pd[2 * c + 1]), as = freg(sc[2 * c], sc[2 * c + 1]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        Mma<bf16_t>::run(dva[u], ft<TP>(L.sdO, 16 * u, c, lane), ap);
        Mma<bf16_t>::run(dka[u], ft<TP>(L.sQ, 16 * u, c, lane), as);
      }
    }
    __syncthreads();                      // every wave is done reading the shared c2p image
    // SkewK[jl][r] = dS[jl + r - 63][jl] (own rows of sX)
    char* skew = L.sX + 16 * w * WP;
    zero_rows16(skew, lane);
    {
      bf16_t* pr = reinterpret_cast<bf16_t*>(skew) + li * (WP / 2);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) pr[16 * t + 4 * lg + e - jl + 63] = f2bf(sc[t][e]);
    }
    // dK += SkewK·PQexp;  HU += SkewK·Uexp
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint4 af = fk<WP>(skew, 0, c, lane);
#pragma unroll
      for (int u = 0; u < 4; ++u) Mma<bf16_t>::run(dka[u], ft<TP>(L.sPQ, 16 * u, c, lane), af);
      if (lora) Mma<bf16_t>::run(hua, ft<UP>(L.sU, 0, c, lane), af);
    }
    if (lora) {
      __syncthreads();                    // all SkewK rows written
      // PBexp[r][c] = Σ_jl SkewK[jl][r]·KB[jl][c]: this wave's r tiles 2w, 2w+1
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int rt = 2 * w + q;
        f32x4_t pbv = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 2; ++c) Mma<bf16_t>::run(pbv, ft<UP>(L.sKB, 0, c, lane), ft<WP>(L.sX, 16 * rt, c, lane));
        if (lg < 2) {
          float* dst = a.pbx + (((bh * a.nqb + qb) * a.nqb + kb) * WIN + 16 * rt + li) * 8 + 4 * lg;
          *reinterpret_cast<float4*>(dst) = make_float4(pbv[0], pbv[1], pbv[2], pbv[3]);
        }
      }
    }
    __syncthreads();
  }
  if (!jrow) return;
  bf16_t* pk = a.dk + (rowb + j) * a.lddqkv + h * DH;
  bf16_t* pv = a.dv + (rowb + j) * a.lddqkv + h * DH;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    st_bf4(reinterpret_cast<char*>(pk + 16 * u + 4 * lg), dka[u]);
    st_bf4(reinterpret_cast<char*>(pv + 16 * u + 4 * lg), dva[u]);
  }
  if (lora && lg < 2)
    *reinterpret_cast<float4*>(a.hu + ((rowb + j) * a.nh + h) * 8 + 4 * lg) = make_float4(hua[0], hua[1], hua[2], hua[3]);
}

// PB[δ][c] = Σ_{b,h} Σ_pairs Σ_{r: δ(i0 - j0 - 63 + r) = δ} PBexp[b,h][pair][r][c]: each thread
// sums one PBexp column over a chunk of (b,h) rows (coalesced 1 KB rows), then adds it to its
// δ row (the r -> δ map depends only on the pair).  PB is zeroed by the launcher.
constexpr int PB_ROWS = 64;
__global__ __launch_bounds__(256) void dis_pb_kernel(DisArgs a) {
  const int np = a.nqb * a.nqb, ncol = np * WIN * 8;
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= ncol) return;
  const int64_t r0 = (int64_t)blockIdx.y * PB_ROWS, r1 = min((int64_t)a.B * a.nh, r0 + PB_ROWS);
  float v = 0.f;
  for (int64_t bh = r0; bh < r1; ++bh) v += a.pbx[bh * ncol + col];
  const int p = col / (WIN * 8), r = (col / 8) % WIN, c = col % 8;
  const int rel = (p / a.nqb) * 64 - (p % a.nqb) * 64 - 63 + r;
  if (rel > -a.S && rel < a.S) atomicAdd(a.pb + win_row(a, rel) * 8 + c, v);
}

}  // namespace

// ---------------------------------------------------------------- C ABI
static int dis_check(const ttmi_dis_attn_desc* d) {
  TTMI_REQUIRE(d != nullptr, "ttmi_dis_attn: null descriptor");
  TTMI_REQUIRE(d->B > 0 && d->S > 0 && d->S <= MAXS && d->nh > 0, "ttmi_dis_attn: need 0 < S <= %d", MAXS);
  TTMI_REQUIRE(d->d_head == DH, "ttmi_dis_attn: d_head must be 64");
  TTMI_REQUIRE(d->npos > 0 && d->npos <= 512, "ttmi_dis_attn: npos must be in (0, 512]");
  TTMI_REQUIRE(d->q && d->k && d->v && d->posq && d->posk && d->mask && d->delta && d->ctx && d->lse,
               "ttmi_dis_attn: null argument");
  TTMI_REQUIRE(d->ldqkv % 8 == 0 && d->ldpos % 8 == 0 && d->ldctx % 8 == 0,
               "ttmi_dis_attn: leading dimensions must be multiples of 8");
  TTMI_REQUIRE(d->drop_p == 0.f || d->drop_seed, "ttmi_dis_attn: dropout needs a seed");
  TTMI_REQUIRE((int64_t)d->B * d->nh * d->S * d->S < (1ll << 32), "ttmi_dis_attn: dropout index overflow");
  return TTMI_OK;
}

static DisArgs dis_args(const ttmi_dis_attn_desc* d) {
  DisArgs a{};
  a.B = d->B; a.S = d->S; a.nh = d->nh; a.npos = d->npos; a.nqb = (d->S + 63) / 64;
  a.q = (const bf16_t*)d->q; a.k = (const bf16_t*)d->k; a.v = (const bf16_t*)d->v; a.ldqkv = d->ldqkv;
  a.posq = (const bf16_t*)d->posq; a.posk = (const bf16_t*)d->posk; a.ldpos = d->ldpos;
  a.mask = d->mask; a.delta = d->delta; a.inv_scale = d->inv_scale;
  a.drop = make_drop(d->drop_p, d->drop_seed);
  a.ctx = (bf16_t*)d->ctx; a.ldctx = d->ldctx; a.lse = d->lse;
  a.dctx = (const bf16_t*)d->dctx; a.lddctx = d->lddctx;
  a.dq = (bf16_t*)d->dq; a.dk = (bf16_t*)d->dk; a.dv = (bf16_t*)d->dv; a.lddqkv = d->lddqkv;
  a.dsum = d->dq_scratch;
  a.u = d->lora_u; a.bq = d->lora_bq; a.hu = d->lora_hu; a.pb = d->lora_pb; a.pbx = d->lora_pbx;
  return a;
}

extern "C" int64_t ttmi_dis_attn_pbx_floats(int B, int S, int nh) {
  const int64_t nb = (S + 63) / 64;
  return (int64_t)B * nh * nb * nb * WIN * 8;
}

extern "C" int ttmi_dis_attn_fwd(const ttmi_dis_attn_desc* d, hipStream_t s) {
  int rc = dis_check(d);
  if (rc) return rc;
  const DisArgs a = dis_args(d);
  hipLaunchKernelGGL(dis_fwd_kernel, dim3((unsigned)a.nqb, (unsigned)d->nh, (unsigned)d->B), dim3(256), 0, s, a);
  return ttmi_check_launch("ttmi_dis_attn_fwd");
}

extern "C" int ttmi_dis_attn_bwd(const ttmi_dis_attn_desc* d, hipStream_t s) {
  int rc = dis_check(d);
  if (rc) return rc;
  TTMI_REQUIRE(d->dctx && d->dq && d->dk && d->dv && d->dq_scratch,
               "ttmi_dis_attn_bwd: null gradient argument (dq_scratch: fp32 [B·nh·S])");
  TTMI_REQUIRE(d->lddctx % 8 == 0 && d->lddqkv % 4 == 0, "ttmi_dis_attn_bwd: bad leading dimension");
  TTMI_REQUIRE(!d->lora_u || (d->lora_bq && d->lora_hu && d->lora_pb && d->lora_pbx),
               "ttmi_dis_attn_bwd: LoRA outputs need u, bq, hu, pb and the pbx workspace together");
  const DisArgs a = dis_args(d);
  const dim3 grid((unsigned)a.nqb, (unsigned)d->nh, (unsigned)d->B);
  hipLaunchKernelGGL(dis_dq_kernel, grid, dim3(256), 0, s, a);
  hipLaunchKernelGGL(dis_dkv_kernel, grid, dim3(256), 0, s, a);
  if (d->lora_u) {
    if (hipMemsetAsync(d->lora_pb, 0, (size_t)d->npos * 8 * sizeof(float), s) != hipSuccess)
      return ttmi_check_launch("ttmi_dis_attn_bwd (pb memset)");
    const int ncol = a.nqb * a.nqb * WIN * 8;
    const int64_t rows = (int64_t)d->B * d->nh;
    hipLaunchKernelGGL(dis_pb_kernel, dim3((unsigned)((ncol + 255) / 256), (unsigned)((rows + PB_ROWS - 1) / PB_ROWS)),
                       dim3(256), 0, s, a);
  }
  return ttmi_check_launch("ttmi_dis_attn_bwd");
}
