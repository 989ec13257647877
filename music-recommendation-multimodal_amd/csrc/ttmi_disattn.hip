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
// Kernels (4 waves, 16 rows per wave, <= 80 KB LDS so two workgroups share a CU):
//   dis_fwd_kernel   per (query block, head, batch): online softmax over key blocks -> ctx, lse
//   dis_dq_kernel    per (query block, head, batch): recomputes P, writes dQ and D = dO·O
//   dis_dkv_kernel   per (key block, head, batch): recomputes Pᵀ, writes dK, dV, HU, PBexp
//   dis_pb_kernel    sums PBexp over (batch, head) and bins its rows to δ -> PB [npos, 8]
// Per block pair each kernel has three barriers: after staging, after the shared window
// product (p2c for the query-side kernels, c2p for dis_dkv), and before the next staging.
// The c2p (query side) / p2c (key side) window is private to each wave and lives in the
// LDS of the window it no longer needs (PQexp / PKexp).
//
// Latency and VALU (round 2, from the SQ counters of round 1: waves parked on s_waitcnt for
// half their lifetime, 4-5 vector instructions per MFMA):
//   * software pipeline: the global loads of the NEXT block pair's rows and windows are
//     issued into registers right after the staging barrier and written to LDS after the
//     pair's last barrier, so their latency hides behind the pair's products;
//   * δ lives in LDS (the window gather was two dependent global loads per row);
//   * scores are kept in log2 units (inv_scale·log2 e folded into one fma with the key mask,
//     exp2 on the VALU), lse is saved in log2 units;
//   * the dropout hash serves an element pair: two hashes per four scores (fwd, dq), and in
//     dis_dkv (pairs straddle two lanes) two hashes per four scores plus a DPP lane swap;
//   * workgroups of one (batch, head) run on one XCD (shared K/V/Q/dO rows in its L2).
#include "ttmi_common.h"

namespace {

constexpr int DH = 64;                 // head width
constexpr int TP = 144;                // LDS pitch (bytes) of a bf16 [rows][64] tile
constexpr int WIN = 128;               // expanded window rows per block pair
constexpr int WP = 272;                // LDS pitch (bytes) of a bf16 [rows][128] window product
constexpr int UP = 32;                 // LDS pitch (bytes) of the bf16 [rows][16] LoRA images
constexpr float FMIN = -3.4028234663852886e38f;   // torch.finfo(torch.float32).min
constexpr float LOG2E = 1.4426950408889634f;
constexpr int MAXS = 256;

typedef __attribute__((ext_vector_type(4))) short s16x4_t;
// Staging registers are clang vectors, not HIP's uint4 struct: copies of the struct lower to
// memcpy through a stack slot when they cross a loop's conditional blocks.
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

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
TTMI_DEV uint32_t pk2(float a, float b) { return pk_bf2(a, b); }
// ... and from score-layout registers (tile t holds columns 16t + 4·lg + e of row lane & 15).
TTMI_DEV uint4 freg(const f32x4_t& lo, const f32x4_t& hi) {
  return make_uint4(pk2(lo[0], lo[1]), pk2(lo[2], lo[3]), pk2(hi[0], hi[1]), pk2(hi[2], hi[3]));
}
// Element offset of row r (< 2^9: a row of one sequence or of the relative table) at leading
// dimension ld (< 2^23, checked by the launcher): one full-rate 24-bit multiply instead of the
// 64-bit multiply-add sequence.
TTMI_DEV uint32_t rowoff(int r, int64_t ld) { return __umul24((uint32_t)r, (uint32_t)ld); }
// Fragment of 16 rows of a global bf16 [rows][ld] matrix, k chunk c (same permutation as fk).
TTMI_DEV uint4 fglob(const bf16_t* base, int64_t ld, int row, int nrows, int c, int lane) {
  const int rr = min(row, nrows - 1);
  const char* p = reinterpret_cast<const char*>(base + rowoff(rr, ld)) + c * 64 + (lane >> 4) * 8;
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
  float* lse;                       // [B, nh, S], log2 units: m + log2 Σ 2^(s - m)
  const bf16_t* dctx; int64_t lddctx;
  bf16_t* dq; bf16_t* dk; bf16_t* dv; int64_t lddqkv;
  float* dsum;                      // [B, nh, S]: D_i = dO_i·O_i (written by dis_dq)
  const float* u;                   // [npos, 8] LoRA down-projection of the relative table
  const float* bq;                  // [nh·64, 8] LoRA B of query_proj
  float* hu;                        // [B·S, nh, 8]
  float* pbx;                       // [B·nh, nqb, nqb, 128, 8]
  float* pb;                        // [npos, 8] (summed over batch and heads)
  int64_t* pbacc;                   // its int64 fixed-point accumulator (in the pbx workspace)
  const int32_t* order;             // [B] batch order (longest first) or null
};

TTMI_DEV int win_row(const DisArgs& a, int rel) {
  rel = min(max(rel, -(a.S - 1)), a.S - 1);
  return a.delta[rel + a.S - 1];
}

// Workgroup -> (batch, head) of the per-sequence kernels: longest sequences first.
struct BH { int b, h; };
TTMI_DEV BH bh_of(const DisArgs& a) {
  const int k = (int)blockIdx.x, bi = k / a.nh;
  BH r;
  r.h = k - bi * a.nh;
  r.b = a.order ? a.order[bi] : bi;
  return r;
}

// End of sequence b's attended range: 1 + the last position whose mask is set (0 if none).
// Blocks of 64 rows at or past it hold only padded tokens: as keys they are masked for every
// valid query (probability exactly 0), and as queries their outputs reach nothing the encoder
// returns (the masked mean-pool) and their gradients are exactly 0.  The kernels skip those
// blocks (block-uniform: every thread of the workgroup computes the same value).  The
// barriers also publish the δ table the caller copied to LDS before the call.
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
TTMI_DEV void load_delta(int16_t* sdel, const DisArgs& a) {
  for (int t = threadIdx.x; t < 2 * a.S - 1; t += blockDim.x) sdel[t] = a.delta[t];
}

// ------------------------------------------------------------------ register-staged loads
// rows [r0, r0 + 64) x 64 bf16 of src: two 16-byte pieces per thread (clamped row: a guarded
// load compiles to a branch + vmcnt(0)) ...
TTMI_DEV void pf_rows(u32x4 (&v)[2], const bf16_t* src, int64_t ld, int r0, int nrows, int tid) {
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int idx = tid + 256 * c, r = idx >> 3, ch = idx & 7;
    v[c] = *reinterpret_cast<const u32x4*>(src + rowoff(min(r0 + r, nrows - 1), ld) + ch * 8);
  }
}
// ... written to an LDS image (pitch TP), rows >= nrows zero.
TTMI_DEV void put_rows(char* dst, const u32x4 (&v)[2], int r0, int nrows, int tid) {
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int idx = tid + 256 * c, r = idx >> 3, ch = idx & 7;
    *reinterpret_cast<u32x4*>(dst + r * TP + ch * 16) = r0 + r < nrows ? v[c] : u32x4{0u, 0u, 0u, 0u};
  }
}
// Expanded window: row r = table[δ(rel0 + r)] (head slice at column h·64), r < 128.
TTMI_DEV void pf_win(u32x4 (&v)[4], const int16_t* sdel, const bf16_t* table, int64_t ld, int rel0,
                     int S, int tid) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int idx = tid + 256 * c, r = idx >> 3, ch = idx & 7;
    const int rel = min(max(rel0 + r, -(S - 1)), S - 1);
    v[c] = *reinterpret_cast<const u32x4*>(table + rowoff(sdel[rel + S - 1], ld) + ch * 8);
  }
}
TTMI_DEV void put_win(char* dst, const u32x4 (&v)[4], int tid) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int idx = tid + 256 * c, r = idx >> 3, ch = idx & 7;
    *reinterpret_cast<u32x4*>(dst + r * TP + ch * 16) = v[c];
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

// ------------------------------------------------------------------ dropout keep factors
TTMI_DEV float keepf(const DropKeys& d, uint32_t u16) { return u16 >= d.thresh ? d.scale : 0.f; }
// Keep factors (0 or 1/(1-p)) of the flat indices idx0 .. idx0 + 3, one hash per aligned
// pair.  EVEN: idx0 is even (every lane, when S is even).
template <bool EVEN>
TTMI_DEV void keep4_row(const DropKeys& d, uint32_t idx0, float (&k)[4]) {
  const uint32_t p0 = idx0 >> 1;
  const uint32_t ha = drop_hash(d, p0), hb = drop_hash(d, p0 + 1);
  if (EVEN) {
    k[0] = keepf(d, ha & 0xFFFFu); k[1] = keepf(d, ha >> 16);
    k[2] = keepf(d, hb & 0xFFFFu); k[3] = keepf(d, hb >> 16);
  } else {
    const uint32_t hc = drop_hash(d, p0 + 2);
    const bool odd = idx0 & 1u;
    k[0] = keepf(d, odd ? ha >> 16 : ha & 0xFFFFu);
    k[1] = keepf(d, odd ? hb & 0xFFFFu : ha >> 16);
    k[2] = keepf(d, odd ? hb >> 16 : hb & 0xFFFFu);
    k[3] = keepf(d, odd ? hc & 0xFFFFu : hb >> 16);
  }
}
// Swap with the neighbouring lane (lane ^ 1): DPP quad_perm [1, 0, 3, 2].
TTMI_DEV uint32_t swap_adj(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}
// Keep factors of 4 scores of one key column j (lane) at query rows i0 .. i0 + 3, flat index
// idx(e) = row(e)·S + j.  EVEN (S even): the pair of idx(e) is (j, j ^ 1) = this lane and its
// neighbour, so each lane hashes two of the four pairs and the neighbour sends the others.
template <bool EVEN>
TTMI_DEV void keep4_col(const DropKeys& d, uint32_t idx0, uint32_t S, bool odd_lane, float (&k)[4]) {
  if (EVEN) {
    const uint32_t e0 = odd_lane ? 2u : 0u;
    const uint32_t h0 = drop_hash(d, (idx0 + e0 * S) >> 1), h1 = drop_hash(d, (idx0 + (e0 + 1) * S) >> 1);
    const uint32_t o0 = swap_adj(h0), o1 = swap_adj(h1);
    const uint32_t g0 = odd_lane ? o0 : h0, g1 = odd_lane ? o1 : h1;   // pairs of e = 0, 1
    const uint32_t g2 = odd_lane ? h0 : o0, g3 = odd_lane ? h1 : o1;   // pairs of e = 2, 3
    k[0] = keepf(d, odd_lane ? g0 >> 16 : g0 & 0xFFFFu);
    k[1] = keepf(d, odd_lane ? g1 >> 16 : g1 & 0xFFFFu);
    k[2] = keepf(d, odd_lane ? g2 >> 16 : g2 & 0xFFFFu);
    k[3] = keepf(d, odd_lane ? g3 >> 16 : g3 & 0xFFFFu);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) k[e] = drop_keep(d, idx0 + e * S) ? d.scale : 0.f;
  }
}

// ------------------------------------------------------------------ query side
struct QSide {
  char sK[64 * TP];
  char sV[64 * TP];
  char sPK[WIN * TP];
  char sPQ[WIN * TP];     // PQexp, then the waves' private c2p / SkewQ images (4 x 16 x WP)
  char sX[64 * WP];       // shared p2c: [key jl][r]
  float sCol[2][64][2];   // per key column {mul, add}: [0] valid query rows, [1] padded rows
  int16_t sDel[2 * MAXS];
};
static_assert(4 * 16 * WP <= WIN * TP, "private images must fit the PQexp window");
static_assert(sizeof(QSide) <= 80 * 1024, "two workgroups per CU");

// The next pair's key rows, values and key mask, held in registers across a block pair (its
// windows are prefetched separately, with pf_win, later in the pair).
struct QRows {
  u32x4 k[2], v[2];
  int64_t mk;             // mask of key j0 + tid (tid < 64)
};
TTMI_DEV void qrows_load(QRows& st, const DisArgs& a, int64_t rowb, int h, int j0, int tid) {
  pf_rows(st.k, a.k + rowb * a.ldqkv + h * DH, a.ldqkv, j0, a.S, tid);
  pf_rows(st.v, a.v + rowb * a.ldqkv + h * DH, a.ldqkv, j0, a.S, tid);
  // unconditional load from a clamped index: a guarded load is a branch + vmcnt(0), which
  // would wait for the prefetch just issued
  st.mk = a.mask[rowb + min(j0 + (tid & 63), a.S - 1)];
}
TTMI_DEV void qrows_store(const QRows& st, QSide& L, int S, int j0, float c, int tid) {
  put_rows(L.sK, st.k, j0, S, tid);
  put_rows(L.sV, st.v, j0, S, tid);
  if (tid < 64) {
    const bool in = j0 + tid < S;
    const float add = in ? FMIN : -INFINITY;
    const bool valid = in && st.mk != 0;
    L.sCol[0][tid][0] = valid ? c : 0.f;
    L.sCol[0][tid][1] = valid ? 0.f : add;
    L.sCol[1][tid][0] = 0.f;
    L.sCol[1][tid][1] = add;
  }
}

TTMI_DEV void qside_prologue(QSide& L, const DisArgs& a, int64_t rowb, int h, int i0, float c, int tid) {
  QRows st;
  qrows_load(st, a, rowb, h, 0, tid);
  u32x4 pk[4], pq[4];
  pf_win(pk, L.sDel, a.posk + h * DH, a.ldpos, i0 - 63, a.S, tid);
  pf_win(pq, L.sDel, a.posq + h * DH, a.ldpos, i0 - 63, a.S, tid);
  qrows_store(st, L, a.S, 0, c, tid);
  put_win(L.sPK, pk, tid);
  put_win(L.sPQ, pq, tid);
}

// Raw scores (c2c + c2p + p2c, unscaled) of this wave's 16 query rows (i = i0 + 16w + li)
// against key block j0: sc[t][e] for key jl = 16t + 4lg + e.  Writes the private c2p image
// first (PQexp is dead after the shared p2c product).
TTMI_DEV void qside_raw(QSide& L, const uint4 (&qf)[2], int w, int lane, f32x4_t (&sc)[4]) {
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
      sc[t][e] += lds_bf(priv, li * (WP / 2) + r) + lds_bf(L.sX, jl * (WP / 2) + r);
    }
}
// s = raw·mul + add for this lane's 16 columns (log2 units).
TTMI_DEV void apply_cols(const float (*col)[2], int lg, f32x4_t (&sc)[4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float4 c01 = *reinterpret_cast<const float4*>(&col[16 * t + 4 * lg][0]);
    const float4 c23 = *reinterpret_cast<const float4*>(&col[16 * t + 4 * lg + 2][0]);
    sc[t][0] = fmaf(sc[t][0], c01.x, c01.y);
    sc[t][1] = fmaf(sc[t][1], c01.z, c01.w);
    sc[t][2] = fmaf(sc[t][2], c23.x, c23.y);
    sc[t][3] = fmaf(sc[t][3], c23.z, c23.w);
  }
}

// One workgroup per (batch, head): every live block pair of the sequence runs in one software
// pipeline (query blocks in order, key blocks inner), so the staging of a new query block
// hides behind the previous pair, and the workgroup start (δ table, sequence end, first
// staging) is paid once per head instead of once per query block.
template <bool EVEN>
__global__ __launch_bounds__(256, 2) void dis_fwd_bh_kernel(DisArgs a) {
  __shared__ __attribute__((aligned(16))) QSide L;
  __shared__ int s_end;
  const BH id = bh_of(a);
  const int h = id.h, b = id.b;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int S = a.S;
  const int64_t rowb = (int64_t)b * S;
  const int64_t bh = (int64_t)b * a.nh + h;
  const DropKeys dk = resolve_drop(a.drop);
  load_delta(L.sDel, a);
  const int send = seq_end(a, rowb, &s_end);
  const int nlive = (send + 63) / 64;
  for (int qb = nlive; qb < a.nqb; ++qb) {   // padded query blocks: finite placeholder outputs
    const int i = qb * 64 + 16 * w + li;
    if (i >= S) break;
    bf16_t* dst = a.ctx + (rowb + i) * a.ldctx + h * DH;
#pragma unroll
    for (int u = 0; u < 4; ++u) st_bf4(reinterpret_cast<char*>(dst + 16 * u + 4 * lg), f32x4_t{0.f, 0.f, 0.f, 0.f});
    if (lg == 0) a.lse[bh * S + i] = 0.f;
  }
  if (nlive == 0) return;
  const float c = a.inv_scale * LOG2E;
  const bf16_t* qbase = a.q + rowb * a.ldqkv + h * DH;
  // query block 0
  int i = 16 * w + li;
  bool qvalid = i < S && a.mask[rowb + min(i, S - 1)] != 0;
  uint4 qf[2] = {fglob(qbase, a.ldqkv, i, S, 0, lane), fglob(qbase, a.ldqkv, i, S, 1, lane)};
  qside_prologue(L, a, rowb, h, 0, c, tid);
  float m_run = -INFINITY, l_run = 0.f;
  f32x4_t o[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) o[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  int qb = 0, kb = 0;
  const int npairs = nlive * nlive;
  for (int p = 0; p < npairs; ++p) {
    const int i0 = qb * 64, j0 = kb * 64;
    const bool last_k = kb + 1 == nlive;
    const int qbn = last_k ? qb + 1 : qb, kbn = last_k ? 0 : kb + 1;
    const bool more = p + 1 < npairs;
    __syncthreads();                      // staging of pair (i0, j0) is in LDS
    // next pair's staging and the next query block's rows (all unconditional, clamped)
    QRows nx;
    u32x4 nwk[4], nwq[4];
    qrows_load(nx, a, rowb, h, kbn * 64, tid);
    pf_win(nwk, L.sDel, a.posk + h * DH, a.ldpos, qbn * 64 - kbn * 64 - 63, S, tid);
    pf_win(nwq, L.sDel, a.posq + h * DH, a.ldpos, qbn * 64 - kbn * 64 - 63, S, tid);
    const int in_ = qbn * 64 + 16 * w + li;
    const uint4 nqf0 = fglob(qbase, a.ldqkv, in_, S, 0, lane), nqf1 = fglob(qbase, a.ldqkv, in_, S, 1, lane);
    const int64_t nqm = a.mask[rowb + min(in_, S - 1)];
    // shared p2c: this wave's 16 keys against PQexp
    win_product(L.sPQ, fk<TP>(L.sK, 16 * w, 0, lane), fk<TP>(L.sK, 16 * w, 1, lane),
                L.sX + 16 * w * WP, lane);
    __syncthreads();
    f32x4_t sc[4];
    qside_raw(L, qf, w, lane, sc);
    apply_cols(L.sCol[qvalid ? 0 : 1], lg, sc);
    float rmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t) rmax = fmaxf(fmaxf(rmax, fmaxf(sc[t][0], sc[t][1])), fmaxf(sc[t][2], sc[t][3]));
    rmax = fmaxf(rmax, __shfl_xor(rmax, 16, 64));
    rmax = fmaxf(rmax, __shfl_xor(rmax, 32, 64));
    const float m_new = fmaxf(m_run, rmax);
    const float corr = __builtin_amdgcn_exp2f(m_run - m_new);
    float rsum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sc[t][e] = __builtin_amdgcn_exp2f(sc[t][e] - m_new);
        rsum += sc[t][e];
      }
    if (dk.on) {
      const uint32_t dbase = (uint32_t)((bh * S + i) * S) + 4 * lg + j0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float kp[4];
        keep4_row<EVEN>(dk, dbase + (uint32_t)(16 * t), kp);
#pragma unroll
        for (int e = 0; e < 4; ++e) sc[t][e] *= kp[e];
      }
    }
    rsum += __shfl_xor(rsum, 16, 64);
    rsum += __shfl_xor(rsum, 32, 64);
    l_run = l_run * corr + rsum;
    m_run = m_new;
#pragma unroll
    for (int u = 0; u < 4; ++u) o[u] *= corr;
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const uint4 af = freg(sc[2 * cc], sc[2 * cc + 1]);
#pragma unroll
      for (int u = 0; u < 4; ++u) Mma<bf16_t>::run(o[u], ft<TP>(L.sV, 16 * u, cc, lane), af);
    }
    if (last_k) {                         // query block done: write it, move to the next one
      if (i < S) {
        const float inv = 1.f / l_run;
        bf16_t* dst = a.ctx + (rowb + i) * a.ldctx + h * DH;
#pragma unroll
        for (int u = 0; u < 4; ++u) st_bf4(reinterpret_cast<char*>(dst + 16 * u + 4 * lg), o[u] * inv);
        if (lg == 0) a.lse[bh * S + i] = m_run + __log2f(l_run);
      }
      m_run = -INFINITY;
      l_run = 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u) o[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      i = in_;
      qvalid = in_ < S && nqm != 0;
      qf[0] = nqf0;
      qf[1] = nqf1;
    }
    __syncthreads();                      // every wave is done with this pair's LDS
    if (more) {
      qrows_store(nx, L, S, kbn * 64, c, tid);
      put_win(L.sPK, nwk, tid);
      put_win(L.sPQ, nwq, tid);
    }
    qb = qbn;
    kb = kbn;
    (void)i0;
  }
}

// Query-side backward, one workgroup per (batch, head) like dis_fwd_bh_kernel.  At the start
// every thread computes D_i = dO_i·O_i of one row of the head (written to dsum for dis_dkv and
// kept in LDS with the row's lse), so moving to the next query block needs only its Q / dO
// fragments, which are prefetched with each pair's staging.
struct QRowData {
  float lse_s[MAXS];      // lse - log2 inv_scale (log2 units), +inf for padded rows
  float d[MAXS];          // D_i
};
template <bool EVEN>
__global__ __launch_bounds__(256, 2) void dis_dq_kernel(DisArgs a) {
  __shared__ __attribute__((aligned(16))) QSide L;
  __shared__ QRowData R;
  __shared__ int s_end;
  const BH id = bh_of(a);
  const int h = id.h, b = id.b;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int S = a.S;
  const int64_t rowb = (int64_t)b * S;
  const int64_t bh = (int64_t)b * a.nh + h;
  const DropKeys dk = resolve_drop(a.drop);
  const float l2s = __log2f(a.inv_scale);
  load_delta(L.sDel, a);
  // D and lse of every row of this head: four lanes per row (16 columns each, coalesced
  // 128-byte rows), reduced with two lane swaps
  for (int r0 = 0; r0 < S; r0 += 64) {
    const int r = r0 + (tid >> 2), q = tid & 3, rc = min(r, S - 1);
    const bf16_t* o = a.ctx + (rowb + rc) * a.ldctx + h * DH + 16 * q;
    const bf16_t* go = a.dctx + (rowb + rc) * a.lddctx + h * DH + 16 * q;
    float acc = 0.f;
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      float x[8], y[8];
      unpack8(*reinterpret_cast<const uint4*>(o + 8 * cc), x);
      unpack8(*reinterpret_cast<const uint4*>(go + 8 * cc), y);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += x[e] * y[e];
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    const bool qv = a.mask[rowb + rc] != 0;
    const float lse = a.lse[bh * S + rc];
    if (q == 0 && r < S) {
      a.dsum[bh * S + r] = acc;
      R.d[r] = acc;
      R.lse_s[r] = qv ? lse - l2s : INFINITY;
    }
  }
  const int send = seq_end(a, rowb, &s_end);
  const int nlive = (send + 63) / 64;
  for (int qb = nlive; qb < a.nqb; ++qb) {   // padded query block: dS = 0, so dQ = 0
    const int i = qb * 64 + 16 * w + li;
    if (i >= S) break;
    bf16_t* dst = a.dq + (rowb + i) * a.lddqkv + h * DH;
#pragma unroll
    for (int u = 0; u < 4; ++u) st_bf4(reinterpret_cast<char*>(dst + 16 * u + 4 * lg), f32x4_t{0.f, 0.f, 0.f, 0.f});
  }
  if (nlive == 0) return;
  const float c = a.inv_scale * LOG2E;
  const bf16_t* qbase = a.q + rowb * a.ldqkv + h * DH;
  const bf16_t* obase = a.dctx + rowb * a.lddctx + h * DH;
  int i = 16 * w + li;
  uint4 qf[2] = {fglob(qbase, a.ldqkv, i, S, 0, lane), fglob(qbase, a.ldqkv, i, S, 1, lane)};
  uint4 of[2] = {fglob(obase, a.lddctx, i, S, 0, lane), fglob(obase, a.lddctx, i, S, 1, lane)};
  qside_prologue(L, a, rowb, h, 0, c, tid);
  f32x4_t dq[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) dq[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  char* priv = L.sPQ + 16 * w * WP;
  int qb = 0, kb = 0;
  const int npairs = nlive * nlive;
  for (int p = 0; p < npairs; ++p) {
    const int j0 = kb * 64;
    const bool last_k = kb + 1 == nlive;
    const int qbn = last_k ? qb + 1 : qb, kbn = last_k ? 0 : kb + 1;
    const bool more = p + 1 < npairs;
    __syncthreads();                      // staging of the pair is in LDS (and R, at p = 0)
    QRows nx;
    qrows_load(nx, a, rowb, h, kbn * 64, tid);   // clamped: valid on the last pair too
    const int in_ = qbn * 64 + 16 * w + li;
    const uint4 nqf0 = fglob(qbase, a.ldqkv, in_, S, 0, lane), nqf1 = fglob(qbase, a.ldqkv, in_, S, 1, lane);
    const uint4 nof0 = fglob(obase, a.lddctx, in_, S, 0, lane), nof1 = fglob(obase, a.lddctx, in_, S, 1, lane);
    win_product(L.sPQ, fk<TP>(L.sK, 16 * w, 0, lane), fk<TP>(L.sK, 16 * w, 1, lane),
                L.sX + 16 * w * WP, lane);
    __syncthreads();
    const int ic = min(i, S - 1);
    const float lse_s = i < S ? R.lse_s[ic] : INFINITY;   // p·inv_scale = 2^(s - lse_s)
    const float Di = i < S ? R.d[ic] : 0.f;
    uint4 dsf[2];                         // dS as bf16 MFMA operands (16 scores per lane)
    {
      f32x4_t sc[4], dp[4];
      qside_raw(L, qf, w, lane, sc);
      apply_cols(L.sCol[0], lg, sc);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        dp[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        Mma<bf16_t>::run(dp[t], fk<TP>(L.sV, 16 * t, 0, lane), of[0]);
        Mma<bf16_t>::run(dp[t], fk<TP>(L.sV, 16 * t, 1, lane), of[1]);
      }
      const uint32_t dbase = (uint32_t)((bh * S + i) * S) + 4 * lg + j0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float kp[4] = {1.f, 1.f, 1.f, 1.f};
        if (dk.on) keep4_row<EVEN>(dk, dbase + (uint32_t)(16 * t), kp);
#pragma unroll
        for (int e = 0; e < 4; ++e)       // d raw score = p·(dP·keep - D)·inv_scale
          sc[t][e] = __builtin_amdgcn_exp2f(sc[t][e] - lse_s) * fmaf(dp[t][e], kp[e], -Di);
      }
      dsf[0] = freg(sc[0], sc[1]);
      dsf[1] = freg(sc[2], sc[3]);
    }
    // dQ += dS·K
#pragma unroll
    for (int cc = 0; cc < 2; ++cc)
#pragma unroll
      for (int u = 0; u < 4; ++u) Mma<bf16_t>::run(dq[u], ft<TP>(L.sK, 16 * u, cc, lane), dsf[cc]);
    u32x4 nwk[4], nwq[4];                 // next pair's windows (clamped: valid on the last pair)
    pf_win(nwk, L.sDel, a.posk + h * DH, a.ldpos, qbn * 64 - kbn * 64 - 63, S, tid);
    pf_win(nwq, L.sDel, a.posq + h * DH, a.ldpos, qbn * 64 - kbn * 64 - 63, S, tid);
    // SkewQ[il][r] = dS[il][il - r + 63] (private image, after this wave's c2p reads)
    zero_rows16(priv, lane);
    {
      bf16_t* pr = reinterpret_cast<bf16_t*>(priv) + li * (WP / 2);
      const int il = 16 * w + li;
      const uint32_t wv[8] = {dsf[0].x, dsf[0].y, dsf[0].z, dsf[0].w, dsf[1].x, dsf[1].y, dsf[1].z, dsf[1].w};
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t x = wv[2 * t + (e >> 1)];
          pr[il - (16 * t + 4 * lg + e) + 63] = (bf16_t)((e & 1) ? x >> 16 : x & 0xFFFFu);
        }
    }
    // dQ += SkewQ·PKexp
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      const uint4 af = fk<WP>(priv, 0, cc, lane);
#pragma unroll
      for (int u = 0; u < 4; ++u) Mma<bf16_t>::run(dq[u], ft<TP>(L.sPK, 16 * u, cc, lane), af);
    }
    if (last_k) {                         // query block done: write dQ, move to the next one
      if (i < S) {
        bf16_t* dst = a.dq + (rowb + i) * a.lddqkv + h * DH;
#pragma unroll
        for (int u = 0; u < 4; ++u) st_bf4(reinterpret_cast<char*>(dst + 16 * u + 4 * lg), dq[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) dq[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      i = in_;
      qf[0] = nqf0; qf[1] = nqf1;
      of[0] = nof0; of[1] = nof1;
    }
    __syncthreads();
    if (more) {
      qrows_store(nx, L, S, kbn * 64, c, tid);
      put_win(L.sPK, nwk, tid);
      put_win(L.sPQ, nwq, tid);
    }
    qb = qbn;
    kb = kbn;
  }
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
  float sRowA[64], sRowD[64];   // per query row: -lse (log2; -inf for padded rows), D
  int16_t sDel[2 * MAXS];
};
static_assert(4 * 16 * WP <= WIN * TP, "private images must fit the PKexp window");
static_assert(sizeof(KSide) <= 80 * 1024, "two workgroups per CU");

// The next pair's staging, held in registers across a block pair: query rows, dO rows and
// the per-row softmax data (loaded right after the staging barrier), then both windows and
// Uexp (loaded after the score phase, when fewer registers are live).
struct KRows {
  u32x4 q[2], o[2];
  float lse, d;           // query row i0 + tid (tid < 64)
  int64_t qm;
};
struct KWins {
  u32x4 pk[4], pq[4];
  float4 u;               // Uexp row tid >> 1, columns 4·(tid & 1) ..
};
TTMI_DEV void krows_load(KRows& st, const DisArgs& a, int64_t rowb, int64_t bh, int h, int i0, int tid) {
  pf_rows(st.q, a.q + rowb * a.ldqkv + h * DH, a.ldqkv, i0, a.S, tid);
  pf_rows(st.o, a.dctx + rowb * a.lddctx + h * DH, a.lddctx, i0, a.S, tid);
  const int ic = min(i0 + (tid & 63), a.S - 1);    // unconditional loads (see qrows_load)
  st.lse = a.lse[bh * a.S + ic];
  st.d = a.dsum[bh * a.S + ic];
  st.qm = a.mask[rowb + ic];
}
TTMI_DEV void load_u(float4& u, const int16_t* sdel, const DisArgs& a, int rel0, int tid) {
  const int rel = min(max(rel0 + (tid >> 1), -(a.S - 1)), a.S - 1);
  u = *reinterpret_cast<const float4*>(a.u + (int64_t)sdel[rel + a.S - 1] * 8 + (tid & 1) * 4);
}
TTMI_DEV void kwins_load(KWins& st, const KSide& L, const DisArgs& a, int h, int i0, int j0, bool lora,
                         int tid) {
  const int rel0 = i0 - j0 - 63;
  pf_win(st.pk, L.sDel, a.posk + h * DH, a.ldpos, rel0, a.S, tid);
  pf_win(st.pq, L.sDel, a.posq + h * DH, a.ldpos, rel0, a.S, tid);
  if (lora) load_u(st.u, L.sDel, a, rel0, tid);
}
TTMI_DEV void put_u(KSide& L, const float4& u, int tid) {
  uint32_t* row = reinterpret_cast<uint32_t*>(L.sU + (tid >> 1) * UP) + (tid & 1) * 2;
  row[0] = pk2(u.x, u.y);
  row[1] = pk2(u.z, u.w);
  row[4] = 0u;
  row[5] = 0u;
}
TTMI_DEV void krows_store(const KRows& st, KSide& L, int S, int i0, int tid) {
  put_rows(L.sQ, st.q, i0, S, tid);
  put_rows(L.sdO, st.o, i0, S, tid);
  if (tid < 64) {
    // valid query row: p = 2^(s - lse); padded rows (dO = 0 there) and rows past S: p = 0
    const bool ok = i0 + tid < S && st.qm != 0;
    L.sRowA[tid] = ok ? -st.lse : -INFINITY;
    L.sRowD[tid] = ok ? st.d : 0.f;
  }
}
TTMI_DEV void kwins_store(const KWins& st, KSide& L, bool lora, int tid) {
  put_win(L.sPK, st.pk, tid);
  put_win(L.sPQ, st.pq, tid);
  if (lora) put_u(L, st.u, tid);
}
TTMI_DEV void kside_prologue(KSide& L, const DisArgs& a, int64_t rowb, int64_t bh, int h, int j0,
                             bool lora, int tid) {
  KRows st;
  krows_load(st, a, rowb, bh, h, 0, tid);
  u32x4 pk[4], pq[4];
  float4 u;
  pf_win(pk, L.sDel, a.posk + h * DH, a.ldpos, -j0 - 63, a.S, tid);
  pf_win(pq, L.sDel, a.posq + h * DH, a.ldpos, -j0 - 63, a.S, tid);
  if (lora) load_u(u, L.sDel, a, -j0 - 63, tid);
  krows_store(st, L, a.S, 0, tid);
  put_win(L.sPK, pk, tid);
  put_win(L.sPQ, pq, tid);
  if (lora) put_u(L, u, tid);
}

// PBexp of a skipped (query block, key block) pair: zero (dis_pb sums every pair).
TTMI_DEV void zero_pbx(const DisArgs& a, int64_t bh, int qb, int kb) {
  float* dst = a.pbx + ((bh * a.nqb + qb) * a.nqb + kb) * WIN * 8;
  for (int t = threadIdx.x; t < WIN * 8 / 4; t += blockDim.x)
    reinterpret_cast<float4*>(dst)[t] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// Key-side backward, one workgroup per (batch, head): key blocks outer, query blocks inner,
// one software pipeline over every live pair (the next pair's Q / dO rows, row data and
// windows prefetched into registers).  A new key block loads its K / V fragments and, with
// LoRA, forms KB = K·Bq_h with two MFMAs (Bq_h fragments are built once per workgroup).
template <bool EVEN>
__global__ __launch_bounds__(256, 2) void dis_dkv_kernel(DisArgs a) {
  __shared__ __attribute__((aligned(16))) KSide L;
  __shared__ int s_end;
  const BH id = bh_of(a);
  const int h = id.h, b = id.b;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lg = lane >> 4;
  const int S = a.S, jl = 16 * w + li;
  const int64_t rowb = (int64_t)b * S;
  const int64_t bh = (int64_t)b * a.nh + h;
  const DropKeys dk = resolve_drop(a.drop);
  const bool lora = a.u != nullptr;
  load_delta(L.sDel, a);
  const int send = seq_end(a, rowb, &s_end);
  const int nlive = (send + 63) / 64;    // live blocks (query and key): < nlive
  if (lora)                              // pairs with a padded block: dS = 0
    for (int kb = 0; kb < a.nqb; ++kb)
      for (int qb = 0; qb < a.nqb; ++qb)
        if (qb >= nlive || kb >= nlive) zero_pbx(a, bh, qb, kb);
  for (int kb = nlive; kb < a.nqb; ++kb) {   // padded key blocks: masked for every valid query
    const int j = kb * 64 + jl;
    if (j >= S) break;
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
  }
  if (nlive == 0) return;
  const float c = a.inv_scale * LOG2E;
  const float l2s = __log2f(a.inv_scale);
  const bf16_t* kbase = a.k + rowb * a.ldqkv + h * DH;
  const bf16_t* vbase = a.v + rowb * a.ldqkv + h * DH;
  // Bq_h as the MFMA B operand (column = lane & 15 < 8, k = d in the fk permutation), bf16
  uint4 bqf[2] = {make_uint4(0u, 0u, 0u, 0u), make_uint4(0u, 0u, 0u, 0u)};
  if (lora && li < 8) {
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int d = cc * 32 + (e >> 2) * 16 + 4 * lg + (e & 3);
        v[e] = a.bq[(h * DH + d) * 8 + li];
      }
      bqf[cc] = make_uint4(pk2(v[0], v[1]), pk2(v[2], v[3]), pk2(v[4], v[5]), pk2(v[6], v[7]));
    }
  }
  kside_prologue(L, a, rowb, bh, h, 0, lora, tid);
  f32x4_t dka[4], dva[4], hua;
#pragma unroll
  for (int u = 0; u < 4; ++u) dka[u] = dva[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  hua = f32x4_t{0.f, 0.f, 0.f, 0.f};
  uint4 kf[2], vf[2];
  float kbias = 0.f;
  char* priv = L.sPK + 16 * w * WP;
  const bool odd_lane = li & 1;
  int qb = 0, kb = 0;
  const int npairs = nlive * nlive;
  for (int p = 0; p < npairs; ++p) {
    const int i0 = qb * 64, j0 = kb * 64, j = j0 + jl;
    const bool last_q = qb + 1 == nlive;
    const int qbn = last_q ? 0 : qb + 1, kbn = last_q ? kb + 1 : kb;
    const bool more = p + 1 < npairs;
    if (qb == 0) {                        // new key block: own key / value fragments, KB
      kf[0] = fglob(kbase, a.ldqkv, j, S, 0, lane);
      kf[1] = fglob(kbase, a.ldqkv, j, S, 1, lane);
      vf[0] = fglob(vbase, a.ldqkv, j, S, 0, lane);
      vf[1] = fglob(vbase, a.ldqkv, j, S, 1, lane);
      kbias = (j < S && a.mask[rowb + min(j, S - 1)] != 0) ? 0.f : -INFINITY;   // masked key: p = 0
      if (lora) {                         // KB[jl][c] = K_j · Bq[h·64 + :, c] (columns 8-15 zero)
        f32x4_t kbv = f32x4_t{0.f, 0.f, 0.f, 0.f};
        Mma<bf16_t>::run(kbv, kf[0], bqf[0]);
        Mma<bf16_t>::run(kbv, kf[1], bqf[1]);
        bf16_t* dst = reinterpret_cast<bf16_t*>(L.sKB) + (16 * w + 4 * lg) * (UP / 2) + li;
#pragma unroll
        for (int e = 0; e < 4; ++e) dst[e * (UP / 2)] = f2bf(kbv[e]);
      }
    }
    __syncthreads();                      // staging of pair (i0, j0) is in LDS
    KRows nx;
    krows_load(nx, a, rowb, bh, h, qbn * 64, tid);     // clamped: valid on the last pair too
    // shared c2p: this wave's 16 queries against PKexp
    win_product(L.sPK, fk<TP>(L.sQ, 16 * w, 0, lane), fk<TP>(L.sQ, 16 * w, 1, lane),
                L.sX + 16 * w * WP, lane);
    __syncthreads();
    // private p2c: own 16 keys against PQexp (into the dead PKexp window)
    win_product(L.sPQ, kf[0], kf[1], priv, lane);
    uint4 pdf[2], dsf[2];                 // P·keep and dS as bf16 MFMA operands
    {
      f32x4_t sc[4], dp[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        sc[t] = dp[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        Mma<bf16_t>::run(sc[t], fk<TP>(L.sQ, 16 * t, 0, lane), kf[0]);
        Mma<bf16_t>::run(sc[t], fk<TP>(L.sQ, 16 * t, 1, lane), kf[1]);
        Mma<bf16_t>::run(dp[t], fk<TP>(L.sdO, 16 * t, 0, lane), vf[0]);
        Mma<bf16_t>::run(dp[t], fk<TP>(L.sdO, 16 * t, 1, lane), vf[1]);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float4 ra = *reinterpret_cast<const float4*>(L.sRowA + 16 * t + 4 * lg);
        const float4 rd = *reinterpret_cast<const float4*>(L.sRowD + 16 * t + 4 * lg);
        const float ra_[4] = {ra.x, ra.y, ra.z, ra.w}, rd_[4] = {rd.x, rd.y, rd.z, rd.w};
        float kp[4] = {1.f, 1.f, 1.f, 1.f};
        if (dk.on)
          keep4_col<EVEN>(dk, (uint32_t)((bh * S + i0 + 16 * t + 4 * lg) * S + j), (uint32_t)S, odd_lane, kp);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int il = 16 * t + 4 * lg + e, r = il - jl + 63;
          const float raw = sc[t][e] + lds_bf(L.sX, il * (WP / 2) + r) + lds_bf(priv, li * (WP / 2) + r);
          const float arg = fmaf(raw, c, ra_[e] + kbias);
          const float pr = __builtin_amdgcn_exp2f(arg);
          // d raw score = p·(dP·keep - D)·inv_scale
          sc[t][e] = __builtin_amdgcn_exp2f(arg + l2s) * fmaf(dp[t][e], kp[e], -rd_[e]);
          dp[t][e] = pr * kp[e];
        }
      }
      pdf[0] = freg(dp[0], dp[1]);
      pdf[1] = freg(dp[2], dp[3]);
      dsf[0] = freg(sc[0], sc[1]);
      dsf[1] = freg(sc[2], sc[3]);
    }
    // dV += Pdᵀ·dO, dK += dSᵀ·Q
#pragma unroll
    for (int cc = 0; cc < 2; ++cc)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        Mma<bf16_t>::run(dva[u], ft<TP>(L.sdO, 16 * u, cc, lane), pdf[cc]);
        Mma<bf16_t>::run(dka[u], ft<TP>(L.sQ, 16 * u, cc, lane), dsf[cc]);
      }
    KWins nw;
    kwins_load(nw, L, a, h, qbn * 64, kbn * 64, lora, tid);   // clamped: valid on the last pair
    __syncthreads();                      // every wave is done reading the shared c2p image
    // SkewK[jl][r] = dS[jl + r - 63][jl] (own rows of sX)
    char* skew = L.sX + 16 * w * WP;
    zero_rows16(skew, lane);
    {
      bf16_t* pr = reinterpret_cast<bf16_t*>(skew) + li * (WP / 2);
      const uint32_t wv[8] = {dsf[0].x, dsf[0].y, dsf[0].z, dsf[0].w, dsf[1].x, dsf[1].y, dsf[1].z, dsf[1].w};
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t x = wv[2 * t + (e >> 1)];
          pr[16 * t + 4 * lg + e - jl + 63] = (bf16_t)((e & 1) ? x >> 16 : x & 0xFFFFu);
        }
    }
    // dK += SkewK·PQexp;  HU += SkewK·Uexp
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      const uint4 af = fk<WP>(skew, 0, cc, lane);
#pragma unroll
      for (int u = 0; u < 4; ++u) Mma<bf16_t>::run(dka[u], ft<TP>(L.sPQ, 16 * u, cc, lane), af);
      if (lora) Mma<bf16_t>::run(hua, ft<UP>(L.sU, 0, cc, lane), af);
    }
    if (lora) {
      __syncthreads();                    // all SkewK rows written
      // PBexp[r][c] = Σ_jl SkewK[jl][r]·KB[jl][c]: this wave's r tiles 2w, 2w+1
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int rt = 2 * w + q;
        f32x4_t pbv = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) Mma<bf16_t>::run(pbv, ft<UP>(L.sKB, 0, cc, lane), ft<WP>(L.sX, 16 * rt, cc, lane));
        if (lg < 2) {
          float* dst = a.pbx + (((bh * a.nqb + qb) * a.nqb + kb) * WIN + 16 * rt + li) * 8 + 4 * lg;
          *reinterpret_cast<float4*>(dst) = make_float4(pbv[0], pbv[1], pbv[2], pbv[3]);
        }
      }
    }
    if (last_q) {                         // key block done: write dK, dV, HU
      if (j < S) {
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
#pragma unroll
      for (int u = 0; u < 4; ++u) dka[u] = dva[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      hua = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
    if (more) {
      krows_store(nx, L, S, qbn * 64, tid);
      kwins_store(nw, L, lora, tid);
    }
    qb = qbn;
    kb = kbn;
  }
}

// PB[δ][c] = Σ_{b,h} Σ_pairs Σ_{r: δ(i0 - j0 - 63 + r) = δ} PBexp[b,h][pair][r][c]: each thread
// sums one PBexp column over a chunk of (b,h) rows (coalesced 1 KB rows), then adds it to its
// δ row (the r -> δ map depends only on the pair) with an int64 fixed-point add (several
// chunks and several r land on one δ row: integer adds make the sum order-independent);
// the launcher zeroes the accumulator and converts it into PB.
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
  if (rel > -a.S && rel < a.S) fx_add(a.pbacc + win_row(a, rel) * 8 + c, v, TTMI_FX_GRAD);
}

__global__ __launch_bounds__(256) void dis_pb_out_kernel(int n, const int64_t* __restrict__ acc,
                                                         float* __restrict__ pb) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) pb[i] = fx_to_f(acc[i], TTMI_FX_GRAD);
}

}  // namespace

static int64_t pbx_base_floats(int B, int S, int nh) {
  const int64_t nb = (S + 63) / 64;
  return (int64_t)B * nh * nb * nb * WIN * 8;
}

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
  TTMI_REQUIRE(d->ldqkv < (1 << 23) && d->ldpos < (1 << 23) && d->ldctx < (1 << 23) &&
               d->lddctx < (1 << 23), "ttmi_dis_attn: leading dimensions must be < 2^23");
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
  a.pbacc = d->lora_pbx ? reinterpret_cast<int64_t*>(d->lora_pbx + pbx_base_floats(d->B, d->S, d->nh)) : nullptr;
  a.order = d->order;
  return a;
}

namespace {
// Counting sort of the batch rows by live block count (descending); one workgroup.
__global__ __launch_bounds__(1024) void dis_order_kernel(const int64_t* mask, int B, int S, int32_t* order) {
  __shared__ int cnt[MAXS / 64 + 2], base[MAXS / 64 + 2];
  const int nq = (S + 63) / 64;
  if (threadIdx.x <= nq) cnt[threadIdx.x] = 0;
  __syncthreads();
  // one wave per batch row: live blocks = ceil(end / 64), end = 1 + last set position
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int b = wv; b < B; b += nw) {
    int e = 0;
    for (int t = lane; t < S; t += 64)
      if (mask[(int64_t)b * S + t] != 0) e = t + 1;
    for (int o = 32; o > 0; o >>= 1) e = max(e, __shfl_xor(e, o, 64));
    if (lane == 0) atomicAdd(&cnt[(e + 63) / 64], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {                // descending: the most live blocks first
    int acc = 0;
    for (int n = nq; n >= 0; --n) { base[n] = acc; acc += cnt[n]; }
  }
  __syncthreads();
  for (int b = wv; b < B; b += nw) {
    int e = 0;
    for (int t = lane; t < S; t += 64)
      if (mask[(int64_t)b * S + t] != 0) e = t + 1;
    for (int o = 32; o > 0; o >>= 1) e = max(e, __shfl_xor(e, o, 64));
    if (lane == 0) order[atomicAdd(&base[(e + 63) / 64], 1)] = b;
  }
}
}  // namespace

extern "C" int ttmi_dis_attn_order(const int64_t* mask, int B, int S, int32_t* order, hipStream_t s) {
  TTMI_REQUIRE(mask && order && B > 0 && S > 0 && S <= MAXS, "ttmi_dis_attn_order: bad arguments (S <= %d)", MAXS);
  hipLaunchKernelGGL(dis_order_kernel, dim3(1), dim3(1024), 0, s, mask, B, S, order);
  return ttmi_check_launch("ttmi_dis_attn_order");
}

extern "C" int64_t ttmi_dis_attn_pbx_floats(int B, int S, int nh) {
  return pbx_base_floats(B, S, nh) + 2 * 512 * 8;    // + the int64 PB accumulator (npos <= 512)
}

extern "C" int ttmi_dis_attn_fwd(const ttmi_dis_attn_desc* d, hipStream_t s) {
  int rc = dis_check(d);
  if (rc) return rc;
  const DisArgs a = dis_args(d);
  const dim3 grid((unsigned)(d->nh * d->B));
  if (d->S % 2 == 0) hipLaunchKernelGGL(dis_fwd_bh_kernel<true>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(dis_fwd_bh_kernel<false>, grid, dim3(256), 0, s, a);
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
  const dim3 grid((unsigned)(d->nh * d->B));
  if (d->S % 2 == 0) {
    hipLaunchKernelGGL(dis_dq_kernel<true>, grid, dim3(256), 0, s, a);
    hipLaunchKernelGGL(dis_dkv_kernel<true>, grid, dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL(dis_dq_kernel<false>, grid, dim3(256), 0, s, a);
    hipLaunchKernelGGL(dis_dkv_kernel<false>, grid, dim3(256), 0, s, a);
  }
  if (d->lora_u) {
    if (hipMemsetAsync(a.pbacc, 0, (size_t)d->npos * 8 * sizeof(int64_t), s) != hipSuccess)
      return ttmi_check_launch("ttmi_dis_attn_bwd (pb memset)");
    const int ncol = a.nqb * a.nqb * WIN * 8;
    const int64_t rows = (int64_t)d->B * d->nh;
    hipLaunchKernelGGL(dis_pb_kernel, dim3((unsigned)((ncol + 255) / 256), (unsigned)((rows + PB_ROWS - 1) / PB_ROWS)),
                       dim3(256), 0, s, a);
    hipLaunchKernelGGL(dis_pb_out_kernel, dim3((unsigned)((d->npos * 8 + 255) / 256)), dim3(256), 0, s,
                       d->npos * 8, a.pbacc, d->lora_pb);
  }
  return ttmi_check_launch("ttmi_dis_attn_bwd");
}
