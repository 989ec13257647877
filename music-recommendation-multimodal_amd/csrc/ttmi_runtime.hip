// ttmi_runtime.hip — error reporting, version, elementwise helpers and the fused AdamW.
#include <cstdarg>
#include <cstdio>

#include "ttmi_common.h"

namespace {
thread_local char g_err[512] = "";
}

void ttmi_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int ttmi_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    ttmi_set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return TTMI_ERR_LAUNCH;
  }
  return TTMI_OK;
}

extern "C" const char* ttmi_last_error(void) { return g_err; }

extern "C" int ttmi_abi_version(void) { return 22; }

namespace {

__global__ void cast_kernel(int64_t n, const float* __restrict__ src, bf16_t* __restrict__ dst) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 4 <= n) {
      float4 v = *reinterpret_cast<const float4*>(src + i);
      ushort4 o;
      o.x = f2bf(v.x); o.y = f2bf(v.y); o.z = f2bf(v.z); o.w = f2bf(v.w);
      *reinterpret_cast<ushort4*>(dst + i) = o;
    } else {
      for (int64_t j = i; j < n; ++j) dst[j] = f2bf(src[j]);
    }
  }
}

// AdamW (torch.optim.AdamW, non-amsgrad, maximize=False) over flat fp32 buffers.  A thread
// owns ADAM_U float4 groups (stride = the grid's thread count, so every access is coalesced)
// and issues all their p / g / m / v loads before any arithmetic: 4·ADAM_U independent
// 16-byte loads in flight per thread instead of 4.
#ifndef TTMI_ADAM_U
#define TTMI_ADAM_U 2
#endif
constexpr int ADAM_U = TTMI_ADAM_U;
// fx (optional): the gradient of the float4 range [fx_lo, fx_hi) is not in g but in an int64
// fixed-point accumulator (2^-fx_shift; the item-embedding rows of ttmi_seq_embed_bwd): it is
// read from there, converted, and the accumulator cleared instead of g (the fold that would
// otherwise convert it into g is skipped: ~31 MB of traffic per cfg-2 step).
__global__ __launch_bounds__(256) void adamw_kernel(int64_t n, float* __restrict__ p, float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    bf16_t* __restrict__ pb, const double* __restrict__ hyper,
                                                    const int32_t* __restrict__ step, int zero_grad,
                                                    int64_t* __restrict__ fx, int64_t fx_lo, int64_t fx_hi,
                                                    int fx_shift, const int32_t* __restrict__ skip_if) {
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n4 = n / 4;
  float4 pp[ADAM_U], gg[ADAM_U], mm[ADAM_U], vv[ADAM_U];
#pragma unroll
  for (int u = 0; u < ADAM_U; ++u) {
    const int64_t q = min(t0 + u * T, max<int64_t>(n4 - 1, 0));   // clamped: loads unconditional
    if (n4 > 0) {
      pp[u] = reinterpret_cast<const float4*>(p)[q];
      if (fx != nullptr && q >= fx_lo && q < fx_hi) {
        const longlong2 a = reinterpret_cast<const longlong2*>(fx)[2 * (q - fx_lo)];
        const longlong2 b = reinterpret_cast<const longlong2*>(fx)[2 * (q - fx_lo) + 1];
        gg[u] = make_float4(fx_to_f(a.x, fx_shift), fx_to_f(a.y, fx_shift), fx_to_f(b.x, fx_shift),
                            fx_to_f(b.y, fx_shift));
      } else {
        gg[u] = reinterpret_cast<const float4*>(g)[q];
      }
      mm[u] = reinterpret_cast<const float4*>(m)[q];
      vv[u] = reinterpret_cast<const float4*>(v)[q];
    }
  }
  const AdamScalars as = adam_scalars(hyper, step);
  // a step whose lookups met an id outside a table leaves p, m, v untouched (skip_if, ABI 22);
  // its gradient is still cleared
  const bool keep = !id_err_raised(skip_if);
  auto upd = [&](float& P, float G, float& Mv, float& Vv) { adam_upd(as, P, G, Mv, Vv); };
#pragma unroll
  for (int u = 0; u < ADAM_U; ++u) {
    const int64_t q = t0 + u * T;
    if (q >= n4) break;
    upd(pp[u].x, gg[u].x, mm[u].x, vv[u].x);
    upd(pp[u].y, gg[u].y, mm[u].y, vv[u].y);
    upd(pp[u].z, gg[u].z, mm[u].z, vv[u].z);
    upd(pp[u].w, gg[u].w, mm[u].w, vv[u].w);
    if (keep) {
      reinterpret_cast<float4*>(p)[q] = pp[u];
      reinterpret_cast<float4*>(m)[q] = mm[u];
      reinterpret_cast<float4*>(v)[q] = vv[u];
    }
    if (fx != nullptr && q >= fx_lo && q < fx_hi) {
      reinterpret_cast<longlong2*>(fx)[2 * (q - fx_lo)] = make_longlong2(0, 0);
      reinterpret_cast<longlong2*>(fx)[2 * (q - fx_lo) + 1] = make_longlong2(0, 0);
    } else if (zero_grad) {
      reinterpret_cast<float4*>(g)[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (pb && keep) {
      ushort4 o;
      o.x = f2bf(pp[u].x); o.y = f2bf(pp[u].y); o.z = f2bf(pp[u].z); o.w = f2bf(pp[u].w);
      reinterpret_cast<ushort4*>(pb)[q] = o;
    }
  }
  if (t0 == 0) {                                  // the n % 4 tail
    for (int64_t j = 4 * n4; j < n; ++j) {
      float pj = p[j], mj = m[j], vj = v[j];
      upd(pj, g[j], mj, vj);
      if (keep) {
        p[j] = pj; m[j] = mj; v[j] = vj;
        if (pb) pb[j] = f2bf(pj);
      }
      if (zero_grad) g[j] = 0.f;
    }
  }
}

__global__ void step_inc_kernel(int32_t* step) { step[0] += 1; }

TTMI_DEV uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// seeds[s] = splitmix64(splitmix64(base) ^ (step*64 + s)) — functional.site_seeds restates it.
// With inc, the step counter is incremented first (ttmi_step_inc folded in: one launch).
__global__ void dropout_seeds_kernel(uint64_t base, int32_t* step, uint64_t* seeds, int n, int inc) {
  const int s = threadIdx.x;
  const int32_t t = step[0] + (inc ? 1 : 0);
  if (s < n) seeds[s] = splitmix64(splitmix64(base) ^ ((uint64_t)(int64_t)t * 64ull + (uint64_t)s));
  __syncthreads();                        // every thread has read the old count
  if (inc && s == 0) step[0] = t;
}

// Column-reduction layout shared by dropout_bwd / colsum: each thread owns 4 consecutive
// columns (16-byte loads), tpr = N/4 threads cover a row, 256/tpr rows per pass; a block
// walks `rpb` rows, reduces its column sums through LDS and adds them with one atomic per
// column.  Needs N % 4 == 0 and N <= 1024 (callers fall back to the scalar kernels).
template <typename T>
TTMI_DEV void store4(T* p, float a, float b, float c, float d);
template <> TTMI_DEV void store4<float>(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}
template <> TTMI_DEV void store4<bf16_t>(bf16_t* p, float a, float b, float c, float d) {
  ushort4 q;
  q.x = f2bf(a); q.y = f2bf(b); q.z = f2bf(c); q.w = f2bf(d);
  *reinterpret_cast<ushort4*>(p) = q;
}
template <typename T>
TTMI_DEV float4 load4(const T* p);
template <> TTMI_DEV float4 load4<float>(const float* p) { return *reinterpret_cast<const float4*>(p); }
template <> TTMI_DEV float4 load4<bf16_t>(const bf16_t* p) {
  const ushort4 q = *reinterpret_cast<const ushort4*>(p);
  return make_float4(bf2f(q.x), bf2f(q.y), bf2f(q.z), bf2f(q.w));
}

TTMI_DEV void colsum_block_reduce(float (&s)[4], int N, int tpr, int rpp, float* red,
                                  float* colsum) {
  const int t = threadIdx.x, cg = t % tpr, rg = t / tpr;
  if (rg < rpp) {
#pragma unroll
    for (int e = 0; e < 4; ++e) red[rg * N + cg * 4 + e] = s[e];
  }
  __syncthreads();
  for (int c = t; c < N; c += blockDim.x) {
    float acc = 0.f;
    for (int k = 0; k < rpp; ++k) acc += red[k * N + c];
    atomicAdd(colsum + c, acc);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void dropout_bwd_vec_kernel(int64_t M, int N,
                                                              const float* __restrict__ dx,
                                                              int64_t ldx, DropParams d,
                                                              int64_t ld_drop,
                                                              const int32_t* __restrict__ drows,
                                                              T* __restrict__ dy,
                                                              int64_t ldy, float* __restrict__ colsum,
                                                              int64_t rpb) {
  __shared__ float red[1024];
  const int tpr = N >> 2, rpp = 256 / tpr;
  const int t = threadIdx.x, cg = t % tpr, rg = t / tpr;
  const DropKeys dk = resolve_drop(d);
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (rg < rpp) {
    const int n = cg * 4;
    for (int64_t m = r0 + rg; m < r1; m += rpp) {
      float4 v = *reinterpret_cast<const float4*>(dx + m * ldx + n);
      float* pv = &v.x;
      if (dk.on) {
        const int64_t dr = drows ? (int64_t)drows[m] : m;
        drop_apply_vec<4>(dk, (uint32_t)(dr * ld_drop + n), pv);
      }
      store4<T>(dy + m * ldy + n, v.x, v.y, v.z, v.w);
#pragma unroll
      for (int e = 0; e < 4; ++e) s[e] += pv[e];
    }
  }
  if (colsum) colsum_block_reduce(s, N, tpr, rpp, red, colsum);
}

// Without a column sum the op is a pure stream: flat over (row, 4-column group), grid-stride,
// enough workgroups to fill every CU (the column-reduction layout above launches ~512
// workgroups with N/4 of 256 threads busy, ~2.9 TB/s on the text encoder's 65,536 x 768).
template <typename T>
__global__ __launch_bounds__(256) void dropout_flat_kernel(int64_t M, int N, const float* __restrict__ dx,
                                                           int64_t ldx, DropParams d, int64_t ld_drop,
                                                           const int32_t* __restrict__ drows,
                                                           T* __restrict__ dy, int64_t ldy) {
  const int n4 = N >> 2;
  const int64_t total = M * n4;
  const DropKeys dk = resolve_drop(d);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / n4;
    const int n = (int)(i - m * n4) * 4;
    float4 v = *reinterpret_cast<const float4*>(dx + m * ldx + n);
    if (dk.on) {
      const int64_t dr = drows ? (int64_t)drows[m] : m;
      drop_apply_vec<4>(dk, (uint32_t)(dr * ld_drop + n), &v.x);
    }
    store4<T>(dy + m * ldy + n, v.x, v.y, v.z, v.w);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void colsum_vec_kernel(int64_t M, int N, const T* __restrict__ x,
                                                         int64_t ldx, float* __restrict__ colsum,
                                                         int64_t rpb) {
  __shared__ float red[1024];
  const int tpr = N >> 2, rpp = 256 / tpr;
  const int t = threadIdx.x, cg = t % tpr, rg = t / tpr;
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (rg < rpp) {
    for (int64_t m = r0 + rg; m < r1; m += rpp) {
      const float4 v = load4<T>(x + m * ldx + cg * 4);
      s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
    }
  }
  colsum_block_reduce(s, N, tpr, rpp, red, colsum);
}

// Scalar fallbacks (any N): each thread owns one column.
template <typename T>
__global__ void dropout_bwd_kernel(int64_t M, int N, const float* __restrict__ dx, int64_t ldx,
                                   DropParams d, int64_t ld_drop,
                                   const int32_t* __restrict__ drows, T* __restrict__ dy,
                                   int64_t ldy, float* __restrict__ colsum, int rows_per_block) {
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  const DropKeys dk = resolve_drop(d);
  for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < N; n += gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int64_t m = r0; m < r1; ++m) {
      float v = dx[m * ldx + n];
      const int64_t dr = drows ? (int64_t)drows[m] : m;
      if (dk.on) v = drop_keep(dk, (uint32_t)(dr * ld_drop + n)) ? v * dk.scale : 0.f;
      stf<T>(dy, m * ldy + n, v);
      s += v;
    }
    if (colsum) atomicAdd(colsum + n, s);
  }
}

template <typename T>
__global__ void colsum_kernel(int64_t M, int N, const T* __restrict__ x, int64_t ldx,
                              float* __restrict__ colsum, int rows_per_block) {
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < N; n += gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int64_t m = r0; m < r1; ++m) s += ldf<T>(x, m * ldx + n);
    atomicAdd(colsum + n, s);
  }
}

bool vec_ok(int N, int64_t ld, const void* a, const void* b) {
  return N % 4 == 0 && N <= 1024 && ld % 4 == 0 && ((uintptr_t)a & 15) == 0 &&
         ((uintptr_t)b & 7) == 0;
}
int64_t vec_rows_per_block(int64_t M, int N) {
  const int rpp = 256 / (N / 4);
  int64_t rpb = (M + 511) / 512;
  rpb = (rpb + rpp - 1) / rpp * rpp;
  return std::max<int64_t>(rpb, rpp);
}

constexpr int MAX_COPIES = 16;
struct CopyList {
  char* dst[MAX_COPIES];
  const char* src[MAX_COPIES];
  int64_t bytes[MAX_COPIES];
  int n;
};

// Tensor t, block bx of gx: 16-byte vectors when both ends are aligned, bytes otherwise.
TTMI_DEV void copy_body(const CopyList& cl, int t, int bx, int gx) {
  char* dst = cl.dst[t];
  const char* src = cl.src[t];
  const int64_t nb = cl.bytes[t];
  const int64_t tid = (int64_t)bx * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gx * blockDim.x;
  if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
    const int64_t nv = nb / 16;
    for (int64_t i = tid; i < nv; i += stride)
      reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
    for (int64_t i = nv * 16 + tid; i < nb; i += stride) dst[i] = src[i];
  } else {
    for (int64_t i = tid; i < nb; i += stride) dst[i] = src[i];
  }
}
// blockIdx.y = tensor.
__global__ void batch_copy_kernel(CopyList cl) { copy_body(cl, blockIdx.y, blockIdx.x, gridDim.x); }

int grid_for(int64_t n, int per_thread) {
  int64_t b = (n + 256 * per_thread - 1) / (256 * per_thread);
  return (int)std::min<int64_t>(std::max<int64_t>(b, 1), 4096);
}

}  // namespace

extern "C" int ttmi_cast_f32_bf16(int64_t n, const float* src, uint16_t* dst, hipStream_t s) {
  TTMI_REQUIRE(n >= 0 && (n == 0 || (src && dst)), "ttmi_cast_f32_bf16: bad args");
  TTMI_REQUIRE(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 7) == 0,
               "ttmi_cast_f32_bf16: src must be 16-B and dst 8-B aligned");
  if (n == 0) return TTMI_OK;
  hipLaunchKernelGGL(cast_kernel, dim3(grid_for(n, 4)), dim3(256), 0, s, n, src, dst);
  return ttmi_check_launch("ttmi_cast_f32_bf16");
}

extern "C" int ttmi_adamw_fx(int64_t n, float* p, float* g, float* m, float* v,
                             uint16_t* p_bf16, const double* hyper, const int32_t* step,
                             int zero_grad, int64_t* fx, int64_t fx_off, int64_t fx_len,
                             int fx_shift, const int32_t* skip_if, hipStream_t s) {
  TTMI_REQUIRE(n >= 0 && p && g && m && v && hyper && step, "ttmi_adamw: null argument");
  TTMI_REQUIRE(((uintptr_t)p & 15) == 0 && ((uintptr_t)g & 15) == 0 && ((uintptr_t)m & 15) == 0 &&
               ((uintptr_t)v & 15) == 0 && ((uintptr_t)p_bf16 & 7) == 0,
               "ttmi_adamw: buffers must be 16-B aligned (bf16 mirror 8-B)");
  TTMI_REQUIRE(!fx || (fx_off >= 0 && fx_len >= 0 && fx_off % 4 == 0 && fx_len % 4 == 0 &&
                       fx_off + fx_len <= n - n % 4 && ((uintptr_t)fx & 15) == 0 &&
                       fx_shift > 0 && fx_shift < 63),
               "ttmi_adamw_fx: the fixed-point range must be float4-aligned, inside [0, n)");
  if (n == 0) return TTMI_OK;
  const int64_t groups = std::max<int64_t>(n / 4, 1);
  const int blocks = (int)std::max<int64_t>((groups + 256 * ADAM_U - 1) / (256 * ADAM_U), 1);
  hipLaunchKernelGGL(adamw_kernel, dim3(blocks), dim3(256), 0, s, n, p, g, m, v, (bf16_t*)p_bf16,
                     hyper, step, zero_grad, fx, fx ? fx_off / 4 : 0, fx ? (fx_off + fx_len) / 4 : 0,
                     fx_shift, skip_if);
  return ttmi_check_launch("ttmi_adamw");
}

extern "C" int ttmi_adamw(int64_t n, float* p, float* g, float* m, float* v,
                          uint16_t* p_bf16, const double* hyper, const int32_t* step,
                          int zero_grad, const int32_t* skip_if, hipStream_t s) {
  return ttmi_adamw_fx(n, p, g, m, v, p_bf16, hyper, step, zero_grad, nullptr, 0, 0, 0, skip_if, s);
}


// ------------------------------------------------------------ batched bf16 transpose
// dst_i[c][r] = src_i[r][c] for up to MAX_COPIES row-major matrices in one launch (the
// transposed weight mirrors that make input-grad GEMMs k-major).  64x64 tiles through LDS
// (pitch 65 elements); 16-bit loads/stores, each weight is at most a few hundred KB.
struct TransposeList {
  uint16_t* dst[MAX_COPIES];
  const uint16_t* src[MAX_COPIES];
  int rows[MAX_COPIES], cols[MAX_COPIES];
  int tile0[MAX_COPIES + 1];        // prefix sums of 64x64 tile counts
  int n;
};

// Optional side job of the same launch: the step's dropout seeds (dropout_seeds_kernel's body
// in one extra workgroup), so a step that refreshes its mirrors and draws its seeds pays one
// launch for both.
struct SeedJob {
  uint64_t base;
  int32_t* step;
  uint64_t* seeds;
  int n, inc;
};

TTMI_DEV void transpose_body(const TransposeList& tl, const SeedJob& sj, int bid) {
  __shared__ uint16_t t[64][65];
  if (bid == tl.tile0[tl.n]) {                     // the seed workgroup (sj.n > 0 or sj.inc)
    const int s = threadIdx.x;
    const int32_t st = sj.step[0] + (sj.inc ? 1 : 0);
    if (s < sj.n) sj.seeds[s] = splitmix64(splitmix64(sj.base) ^ ((uint64_t)(int64_t)st * 64ull + (uint64_t)s));
    __syncthreads();                               // every thread has read the old count
    if (sj.inc && s == 0) sj.step[0] = st;
    return;
  }
  int i = 0;
  while (i + 1 < tl.n && bid >= tl.tile0[i + 1]) ++i;
  const int local = bid - tl.tile0[i];
  const int R = tl.rows[i], C = tl.cols[i];
  const int tcol = (C + 63) / 64;
  const int r0 = (local / tcol) * 64, c0 = (local % tcol) * 64;
  const uint16_t* src = tl.src[i];
  uint16_t* dst = tl.dst[i];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  // all 16 loads first, from clamped addresses (a guarded load is a branch + vmcnt(0) each:
  // 16 round trips in a row); elements past the edge are never stored
  uint16_t v[16];
  const int cc = min(c0 + tx, C - 1);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = src[(int64_t)min(r0 + ty + 4 * k, R - 1) * C + cc];
#pragma unroll
  for (int k = 0; k < 16; ++k) t[ty + 4 * k][tx] = v[k];
  __syncthreads();
  for (int c = ty; c < 64; c += 4)
    if (c0 + c < C && r0 + tx < R) dst[(int64_t)(c0 + c) * R + r0 + tx] = t[tx][c];
}
__global__ __launch_bounds__(256) void transpose_batch_kernel(TransposeList tl, SeedJob sj) {
  transpose_body(tl, sj, (int)blockIdx.x);
}
// The train step's prologue in one launch (ABI 22): the batch staging copies (blocks
// [0, cgx·cl.n)), then the transposed weight mirrors, then the seed / step-count workgroup.
__global__ __launch_bounds__(256) void step_prologue_kernel(CopyList cl, int cgx, TransposeList tl, SeedJob sj) {
  const int nc = cgx * cl.n;
  const int b = (int)blockIdx.x;
  if (b < nc) {
    copy_body(cl, b / cgx, b % cgx, cgx);
    return;
  }
  transpose_body(tl, sj, b - nc);
}

namespace {
int transpose_list(int n, void* const* dst, const void* const* src, const int64_t* rows,
                   const int64_t* cols, TransposeList& tl) {
  TTMI_REQUIRE(n >= 0 && n <= MAX_COPIES, "ttmi_transpose_bf16_batch: at most %d matrices", MAX_COPIES);
  TTMI_REQUIRE(n == 0 || (dst && src && rows && cols), "ttmi_transpose_bf16_batch: null argument");
  tl.n = n;
  tl.tile0[0] = 0;
  for (int i = 0; i < n; ++i) {
    TTMI_REQUIRE(rows[i] >= 0 && cols[i] >= 0 && rows[i] < (1 << 30) && cols[i] < (1 << 30),
                 "ttmi_transpose_bf16_batch: bad shape %d", i);
    TTMI_REQUIRE(rows[i] * cols[i] == 0 || (dst[i] && src[i]), "ttmi_transpose_bf16_batch: null entry %d", i);
    tl.dst[i] = static_cast<uint16_t*>(dst[i]);
    tl.src[i] = static_cast<const uint16_t*>(src[i]);
    tl.rows[i] = (int)rows[i];
    tl.cols[i] = (int)cols[i];
    const int64_t tiles = ((rows[i] + 63) / 64) * ((cols[i] + 63) / 64);
    TTMI_REQUIRE(tl.tile0[i] + tiles < (1 << 30), "ttmi_transpose_bf16_batch: too large");
    tl.tile0[i + 1] = tl.tile0[i] + (int)tiles;
  }
  return TTMI_OK;
}
int copy_list(int n, void* const* dst, const void* const* src, const int64_t* nbytes, CopyList& cl,
              int& gx) {
  TTMI_REQUIRE(n >= 0 && n <= MAX_COPIES, "ttmi_batch_copy: at most %d tensors", MAX_COPIES);
  TTMI_REQUIRE(n == 0 || (dst && src && nbytes), "ttmi_batch_copy: null argument");
  int64_t mx = 0;
  for (int i = 0; i < n; ++i) {
    TTMI_REQUIRE(nbytes[i] >= 0 && (nbytes[i] == 0 || (dst[i] && src[i])), "ttmi_batch_copy: bad entry %d", i);
    cl.dst[i] = static_cast<char*>(dst[i]);
    cl.src[i] = static_cast<const char*>(src[i]);
    cl.bytes[i] = nbytes[i];
    mx = std::max(mx, nbytes[i]);
  }
  cl.n = n;
  gx = (int)std::min<int64_t>(std::max<int64_t>((mx / 16 + 255) / 256, 1), 256);
  return TTMI_OK;
}
}  // namespace

extern "C" int ttmi_transpose_bf16_batch_seeds(int n, void* const* dst, const void* const* src,
                                               const int64_t* rows, const int64_t* cols,
                                               uint64_t seed_base, int32_t* step, uint64_t* seeds,
                                               int n_seeds, int inc_step, hipStream_t s) {
  TTMI_REQUIRE(n_seeds >= 0 && n_seeds <= 256 && (n_seeds == 0 || (step && seeds)),
               "ttmi_transpose_bf16_batch_seeds: bad seed arguments");
  SeedJob sj{seed_base, step, seeds, n_seeds, inc_step};
  if (n == 0 && n_seeds == 0) return TTMI_OK;
  TransposeList tl;
  int rc = transpose_list(n, dst, src, rows, cols, tl);
  if (rc) return rc;
  const int blocks = tl.tile0[n] + (n_seeds > 0 ? 1 : 0);
  if (blocks == 0) return TTMI_OK;
  hipLaunchKernelGGL(transpose_batch_kernel, dim3(blocks), dim3(256), 0, s, tl, sj);
  return ttmi_check_launch("ttmi_transpose_bf16_batch");
}

extern "C" int ttmi_step_prologue(int n_copy, void* const* cdst, const void* const* csrc,
                                  const int64_t* nbytes, int n_tr, void* const* tdst,
                                  const void* const* tsrc, const int64_t* rows, const int64_t* cols,
                                  uint64_t seed_base, int32_t* step, uint64_t* seeds, int n_seeds,
                                  int inc_step, hipStream_t s) {
  TTMI_REQUIRE(n_seeds >= 0 && n_seeds <= 256 && (n_seeds == 0 || seeds) && ((n_seeds == 0 && !inc_step) || step),
               "ttmi_step_prologue: bad seed arguments");
  CopyList cl;
  int cgx = 1;
  int rc = copy_list(n_copy, cdst, csrc, nbytes, cl, cgx);
  if (rc) return rc;
  TransposeList tl;
  rc = transpose_list(n_tr, tdst, tsrc, rows, cols, tl);
  if (rc) return rc;
  SeedJob sj{seed_base, step, seeds, n_seeds, inc_step};
  const int64_t blocks = (int64_t)cgx * n_copy + tl.tile0[n_tr] + ((n_seeds > 0 || inc_step) ? 1 : 0);
  TTMI_REQUIRE(blocks < (1 << 30), "ttmi_step_prologue: too large");
  if (blocks == 0) return TTMI_OK;
  hipLaunchKernelGGL(step_prologue_kernel, dim3((unsigned)blocks), dim3(256), 0, s, cl, cgx, tl, sj);
  return ttmi_check_launch("ttmi_step_prologue");
}

extern "C" int ttmi_batch_copy(int n, void* const* dst, const void* const* src,
                               const int64_t* nbytes, hipStream_t s) {
  if (n == 0) return TTMI_OK;
  CopyList cl;
  int gx = 1;
  const int rc = copy_list(n, dst, src, nbytes, cl, gx);
  if (rc) return rc;
  hipLaunchKernelGGL(batch_copy_kernel, dim3(gx, n), dim3(256), 0, s, cl);
  return ttmi_check_launch("ttmi_batch_copy");
}

extern "C" int ttmi_transpose_bf16_batch(int n, void* const* dst, const void* const* src,
                                         const int64_t* rows, const int64_t* cols,
                                         hipStream_t s) {
  return ttmi_transpose_bf16_batch_seeds(n, dst, src, rows, cols, 0, nullptr, nullptr, 0, 0, s);
}

extern "C" int ttmi_step_inc(int32_t* step, hipStream_t s) {
  TTMI_REQUIRE(step, "ttmi_step_inc: null step");
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, s, step);
  return ttmi_check_launch("ttmi_step_inc");
}

extern "C" int ttmi_dropout_seeds(uint64_t base, int32_t* step, uint64_t* seeds, int n, int inc_step,
                                  hipStream_t s) {
  TTMI_REQUIRE(step && seeds && n > 0 && n <= 256, "ttmi_dropout_seeds: bad args");
  hipLaunchKernelGGL(dropout_seeds_kernel, dim3(1), dim3(256), 0, s, base, step, seeds, n, inc_step);
  return ttmi_check_launch("ttmi_dropout_seeds");
}

extern "C" int ttmi_dropout_bwd(int dtype, int64_t M, int N, const float* dx, int64_t ldx,
                                float drop_p, const uint64_t* drop_seed, int64_t ld_drop,
                                const int32_t* drop_rows, void* dy, int64_t ldy, float* colsum,
                                hipStream_t s) {
  TTMI_REQUIRE(dtype == TTMI_F32 || dtype == TTMI_BF16, "ttmi_dropout_bwd: bad dtype");
  TTMI_REQUIRE(M >= 0 && N > 0 && dx && dy && ldx >= N && ldy >= N, "ttmi_dropout_bwd: bad args");
  TTMI_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "ttmi_dropout_bwd: drop_p out of [0,1)");
  TTMI_REQUIRE(drop_p == 0.f || drop_seed, "ttmi_dropout_bwd: dropout needs a seed pointer");
  if (M == 0) return TTMI_OK;
  DropParams d = make_drop(drop_p, drop_seed);
  if (ld_drop == 0) ld_drop = N;
  if (!colsum && N % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && ((uintptr_t)dx & 15) == 0 &&
      ((uintptr_t)dy & (dtype == TTMI_BF16 ? 7 : 15)) == 0) {
    const int64_t total = M * (N / 4);
    const dim3 fg((unsigned)std::min<int64_t>((total + 255) / 256, 16384));
    if (dtype == TTMI_BF16)
      hipLaunchKernelGGL(dropout_flat_kernel<bf16_t>, fg, dim3(256), 0, s, M, N, dx, ldx, d, ld_drop,
                         drop_rows, (bf16_t*)dy, ldy);
    else
      hipLaunchKernelGGL(dropout_flat_kernel<float>, fg, dim3(256), 0, s, M, N, dx, ldx, d, ld_drop,
                         drop_rows, (float*)dy, ldy);
    return ttmi_check_launch("ttmi_dropout_bwd");
  }
  if (vec_ok(N, ldx, dx, dy) && ldy % 4 == 0) {
    const int64_t rpb = vec_rows_per_block(M, N);
    dim3 vg((unsigned)((M + rpb - 1) / rpb));
    if (dtype == TTMI_BF16)
      hipLaunchKernelGGL(dropout_bwd_vec_kernel<bf16_t>, vg, dim3(256), 0, s, M, N, dx, ldx, d,
                         ld_drop, drop_rows, (bf16_t*)dy, ldy, colsum, rpb);
    else
      hipLaunchKernelGGL(dropout_bwd_vec_kernel<float>, vg, dim3(256), 0, s, M, N, dx, ldx, d,
                         ld_drop, drop_rows, (float*)dy, ldy, colsum, rpb);
    return ttmi_check_launch("ttmi_dropout_bwd");
  }
  const int rpb = 64;
  dim3 grid((N + 255) / 256, (unsigned)((M + rpb - 1) / rpb));
  if (dtype == TTMI_BF16)
    hipLaunchKernelGGL(dropout_bwd_kernel<bf16_t>, grid, dim3(256), 0, s, M, N, dx, ldx, d, ld_drop,
                       drop_rows, (bf16_t*)dy, ldy, colsum, rpb);
  else
    hipLaunchKernelGGL(dropout_bwd_kernel<float>, grid, dim3(256), 0, s, M, N, dx, ldx, d, ld_drop,
                       drop_rows, (float*)dy, ldy, colsum, rpb);
  return ttmi_check_launch("ttmi_dropout_bwd");
}

extern "C" int ttmi_colsum(int dtype, int64_t M, int N, const void* x, int64_t ldx, float* colsum,
                           hipStream_t s) {
  TTMI_REQUIRE(dtype == TTMI_F32 || dtype == TTMI_BF16, "ttmi_colsum: bad dtype");
  TTMI_REQUIRE(M >= 0 && N > 0 && x && colsum && ldx >= N, "ttmi_colsum: bad args");
  if (M == 0) return TTMI_OK;
  if (vec_ok(N, ldx, x, x)) {
    const int64_t rpb = vec_rows_per_block(M, N);
    dim3 vg((unsigned)((M + rpb - 1) / rpb));
    if (dtype == TTMI_BF16)
      hipLaunchKernelGGL(colsum_vec_kernel<bf16_t>, vg, dim3(256), 0, s, M, N, (const bf16_t*)x, ldx,
                         colsum, rpb);
    else
      hipLaunchKernelGGL(colsum_vec_kernel<float>, vg, dim3(256), 0, s, M, N, (const float*)x, ldx,
                         colsum, rpb);
    return ttmi_check_launch("ttmi_colsum");
  }
  const int rpb = 64;
  dim3 grid((N + 255) / 256, (unsigned)((M + rpb - 1) / rpb));
  if (dtype == TTMI_BF16)
    hipLaunchKernelGGL(colsum_kernel<bf16_t>, grid, dim3(256), 0, s, M, N, (const bf16_t*)x, ldx,
                       colsum, rpb);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, s, M, N, (const float*)x, ldx,
                       colsum, rpb);
  return ttmi_check_launch("ttmi_colsum");
}
