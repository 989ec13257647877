// ttmi_prep.hip — input-side preprocessing of the item modalities on the GPU (SURVEY §8(f)
// rank 1: the batch contract of the reference's missing src/data/dataset.py, whose transforms
// report/chapters/dataset.tex:23 and :38 describe):
//
//   mel_power      per STFT frame: zero-padded (center=True, librosa 0.11 pad_mode='constant')
//                  periodic-Hann window, 2048-point FFT in LDS (radix-2, precomputed twiddles),
//                  |X|² for the 1025 rfft bins, then the sparse Slaney mel filterbank ->
//                  mel power [B, n_mels, F]   (librosa.feature.melspectrogram, power 2)
//   mel_db_minmax  per clip: power_to_db(ref = max, amin 1e-10, top_db 80), then min-max to
//                  [0, 1]  (dataset.tex:23)
//   cover_prep     uint8 HWC album covers -> antialiased bilinear resize (torch / PIL
//                  triangle filter, align_corners = False) -> ImageNet normalisation ->
//                  fp32 NCHW (the batch's target_image) or bf16 NHWC with C padded to 8 (the
//                  ResNet stem's operand layout, skipping the separate layout pass)
//
// All three are HBM/latency-bound byte work (a few KB per frame or pixel row): no MFMA.
#include "ttmi_common.h"

namespace {

constexpr int NFFT = 2048;
constexpr int NBIN = NFFT / 2 + 1;

struct MelArgs {
  int B, F, n_mels, hop;
  int64_t N, ldx;
  const float* x;           // [B, ldx] waveform
  const float* window;      // [2048] periodic Hann
  const float2* twiddle;    // [1024] exp(-2πi k / 2048)
  const int* band_start;    // [n_mels] first nonzero rfft bin of each band
  const int* band_len;      // [n_mels]
  const int* band_off;      // [n_mels] offset of the band's weights in band_w
  const float* band_w;      // packed nonzero filterbank weights
  float* out;               // [B, n_mels, F]
};

TTMI_DEV int bitrev11(int v) { return (int)(__builtin_bitreverse32((uint32_t)v) >> 21); }

// One workgroup per frame: in-place radix-2 DIT FFT of 2048 points in LDS.
__global__ __launch_bounds__(256) void mel_power_kernel(MelArgs a) {
  __shared__ float2 buf[NFFT];
  __shared__ float2 tw[NFFT / 2];
  __shared__ float pw[NBIN + 3];
  const int64_t fid = blockIdx.x;
  const int b = (int)(fid / a.F), f = (int)(fid % a.F);
  const int tid = threadIdx.x;
  const float* x = a.x + (int64_t)b * a.ldx;
  const int64_t t0 = (int64_t)f * a.hop - NFFT / 2;          // center=True
  for (int k = tid; k < NFFT / 2; k += 256) tw[k] = a.twiddle[k];
  for (int n = tid; n < NFFT; n += 256) {
    const int64_t t = t0 + n;
    const float v = (t >= 0 && t < a.N) ? x[t] : 0.f;        // pad_mode='constant'
    buf[bitrev11(n)] = make_float2(v * a.window[n], 0.f);
  }
  __syncthreads();
#pragma unroll 1
  for (int s = 1; s <= 11; ++s) {
    const int half = 1 << (s - 1), tstep = NFFT >> s;
    for (int k = tid; k < NFFT / 2; k += 256) {
      const int j = k & (half - 1), i0 = ((k >> (s - 1)) << s) + j, i1 = i0 + half;
      const float2 w = tw[j * tstep], u = buf[i0], v = buf[i1];
      const float2 t = make_float2(w.x * v.x - w.y * v.y, w.x * v.y + w.y * v.x);
      buf[i0] = make_float2(u.x + t.x, u.y + t.y);
      buf[i1] = make_float2(u.x - t.x, u.y - t.y);
    }
    __syncthreads();
  }
  for (int k = tid; k < NBIN; k += 256) {
    const float2 z = buf[k];
    pw[k] = z.x * z.x + z.y * z.y;
  }
  __syncthreads();
  for (int m = tid; m < a.n_mels; m += 256) {
    const int s0 = a.band_start[m], len = a.band_len[m];
    const float* w = a.band_w + a.band_off[m];
    float acc = 0.f;
    for (int k = 0; k < len; ++k) acc += w[k] * pw[s0 + k];
    a.out[((int64_t)b * a.n_mels + m) * a.F + f] = acc;
  }
}

TTMI_DEV float block_reduce(float v, float* red, bool is_max) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = is_max ? wave_max(v) : wave_sum(v);
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = is_max ? fmaxf(r, red[i]) : r + red[i];
  __syncthreads();
  return r;
}

// One workgroup per clip: power_to_db(S, ref=np.max, amin, top_db) then min-max to [0, 1].
__global__ __launch_bounds__(256) void mel_db_minmax_kernel(int64_t n, float amin, float top_db,
                                                            float* __restrict__ mel) {
  __shared__ float red[4];
  float* s = mel + (int64_t)blockIdx.x * n;
  float mx = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 256) mx = fmaxf(mx, s[i]);
  mx = block_reduce(mx, red, true);
  const float ref_db = 10.f * log10f(fmaxf(amin, mx));
  // log_spec max is 0 when mx >= amin; the top_db floor is relative to the log-spectrum max
  float lmax = -INFINITY;
  for (int64_t i = threadIdx.x; i < n; i += 256) {
    const float v = 10.f * log10f(fmaxf(amin, s[i])) - ref_db;
    s[i] = v;
    lmax = fmaxf(lmax, v);
  }
  lmax = block_reduce(lmax, red, true);
  const float floor_db = lmax - top_db;
  float lmin = INFINITY;
  for (int64_t i = threadIdx.x; i < n; i += 256) {
    const float v = fmaxf(s[i], floor_db);
    s[i] = v;
    lmin = fminf(lmin, v);
  }
  lmin = -block_reduce(-lmin, red, true);
  const float span = lmax - lmin;
  const float inv = span > 0.f ? 1.f / span : 0.f;             // silent clip -> all zeros
  for (int64_t i = threadIdx.x; i < n; i += 256) s[i] = (s[i] - lmin) * inv;
}

// Antialiased bilinear taps of output index o (torch _compute_indices_min_size_weights_aa,
// align_corners = False; PIL's triangle filter with the support widened by the downscale).
constexpr int MAXTAP = 16;
TTMI_DEV int aa_taps(int o, int in, float scale, int* x0, float* w) {
  const float support = scale >= 1.f ? scale : 1.f;
  const float invs = scale >= 1.f ? 1.f / scale : 1.f;
  const float center = scale * (o + 0.5f);
  const int xmin = max((int)(center - support + 0.5f), 0);
  const int xmax = min((int)(center + support + 0.5f), in);
  const int n = min(xmax - xmin, MAXTAP);
  float tot = 0.f;
  for (int j = 0; j < n; ++j) {
    const float d = fabsf((j + xmin - center + 0.5f) * invs);
    w[j] = d < 1.f ? 1.f - d : 0.f;
    tot += w[j];
  }
  const float inv = tot != 0.f ? 1.f / tot : 0.f;
  for (int j = 0; j < n; ++j) w[j] *= inv;
  *x0 = xmin;
  return n;
}

struct CoverArgs {
  int B, H, W, OH, OW;
  int64_t ld_img;                   // bytes per image (H·W·3 for packed covers)
  const uint8_t* img;               // [B] x [H, W, 3] uint8
  float mean[3], inv_std[3];
  float* out_nchw;                  // fp32 [B, 3, OH, OW] or NULL
  bf16_t* out_nhwc8;                // bf16 [B, OH, OW, 8] (channels 3..7 zero) or NULL
};

__global__ __launch_bounds__(256) void cover_prep_kernel(CoverArgs a) {
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t per = (int64_t)a.OH * a.OW;
  if (id >= (int64_t)a.B * per) return;
  const int b = (int)(id / per), p = (int)(id % per), oy = p / a.OW, ox = p % a.OW;
  int x0, y0;
  float wx[MAXTAP], wy[MAXTAP];
  const int nx = aa_taps(ox, a.W, (float)a.W / a.OW, &x0, wx);
  const int ny = aa_taps(oy, a.H, (float)a.H / a.OH, &y0, wy);
  const uint8_t* src = a.img + (int64_t)b * a.ld_img;
  float acc[3] = {0.f, 0.f, 0.f};
  for (int j = 0; j < ny; ++j) {
    const uint8_t* row = src + ((int64_t)(y0 + j) * a.W + x0) * 3;
    float r[3] = {0.f, 0.f, 0.f};
    for (int i = 0; i < nx; ++i) {
      r[0] += wx[i] * row[3 * i];
      r[1] += wx[i] * row[3 * i + 1];
      r[2] += wx[i] * row[3 * i + 2];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) acc[c] += wy[j] * r[c];
  }
  float v[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) v[c] = (acc[c] * (1.f / 255.f) - a.mean[c]) * a.inv_std[c];
  if (a.out_nchw) {
#pragma unroll
    for (int c = 0; c < 3; ++c) a.out_nchw[((int64_t)b * 3 + c) * per + p] = v[c];
  }
  if (a.out_nhwc8) {
    uint4 q;
    q.x = pk_bf2(v[0], v[1]);
    q.y = (uint32_t)f2bf(v[2]);
    q.z = 0u;
    q.w = 0u;
    reinterpret_cast<uint4*>(a.out_nhwc8)[id] = q;
  }
}

}  // namespace

extern "C" int ttmi_mel_power(int B, int64_t N, const float* x, int64_t ldx, int hop, int n_mels,
                              const float* window, const float* twiddle, const int* band_start,
                              const int* band_len, const int* band_off, const float* band_w, float* out,
                              hipStream_t s) {
  TTMI_REQUIRE(B > 0 && N > 0 && hop > 0 && n_mels > 0 && ldx >= N, "ttmi_mel_power: bad size");
  TTMI_REQUIRE(x && window && twiddle && band_start && band_len && band_off && band_w && out,
               "ttmi_mel_power: null argument");
  MelArgs a;
  a.B = B; a.N = N; a.ldx = ldx; a.hop = hop; a.n_mels = n_mels;
  a.F = (int)(1 + N / hop);
  a.x = x; a.window = window; a.twiddle = reinterpret_cast<const float2*>(twiddle);
  a.band_start = band_start; a.band_len = band_len; a.band_off = band_off; a.band_w = band_w; a.out = out;
  hipLaunchKernelGGL(mel_power_kernel, dim3((unsigned)((int64_t)B * a.F)), dim3(256), 0, s, a);
  return ttmi_check_launch("ttmi_mel_power");
}

extern "C" int ttmi_mel_db_minmax(int B, int64_t n, float amin, float top_db, float* mel, hipStream_t s) {
  TTMI_REQUIRE(B > 0 && n > 0 && mel && amin > 0.f && top_db > 0.f, "ttmi_mel_db_minmax: bad argument");
  hipLaunchKernelGGL(mel_db_minmax_kernel, dim3((unsigned)B), dim3(256), 0, s, n, amin, top_db, mel);
  return ttmi_check_launch("ttmi_mel_db_minmax");
}

extern "C" int ttmi_cover_prep(int B, int H, int W, const uint8_t* img, int64_t ld_img, int OH, int OW,
                               const float* mean, const float* std, float* out_nchw,
                               uint16_t* out_nhwc8, hipStream_t s) {
  TTMI_REQUIRE(B > 0 && H > 0 && W > 0 && OH > 0 && OW > 0 && img && mean && std,
               "ttmi_cover_prep: bad argument");
  TTMI_REQUIRE(out_nchw || out_nhwc8, "ttmi_cover_prep: no output");
  TTMI_REQUIRE(ld_img >= (int64_t)H * W * 3, "ttmi_cover_prep: ld_img < H·W·3");
  TTMI_REQUIRE((float)H / OH < MAXTAP / 2 - 1 && (float)W / OW < MAXTAP / 2 - 1,
               "ttmi_cover_prep: downscale factor too large (> %d)", MAXTAP / 2 - 1);
  TTMI_REQUIRE(!out_nhwc8 || (uintptr_t)out_nhwc8 % 16 == 0, "ttmi_cover_prep: NHWC8 output must be 16-byte aligned");
  CoverArgs a;
  a.B = B; a.H = H; a.W = W; a.OH = OH; a.OW = OW; a.ld_img = ld_img; a.img = img;
  for (int c = 0; c < 3; ++c) { a.mean[c] = mean[c]; a.inv_std[c] = 1.f / std[c]; }
  a.out_nchw = out_nchw; a.out_nhwc8 = (bf16_t*)out_nhwc8;
  const int64_t n = (int64_t)B * OH * OW;
  hipLaunchKernelGGL(cover_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  return ttmi_check_launch("ttmi_cover_prep");
}
