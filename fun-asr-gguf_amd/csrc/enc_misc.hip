// Encoder-side memory-bound kernels: frontend (F1, F4), LayerNorm (E1 + E5 mask sweep),
// FSMN depthwise memory (E4), and the wavefront CTC greedy collapse (C2).
#include "common.h"
#include "kernels.h"

namespace fa {

// fp16 encoder mode (C5): op outputs are fp16 values, held in f32
__device__ __forceinline__ float r16e(float v, int r16) { return r16 ? __half2float(__float2half_rn(v)) : v; }

// ---------------- F1: mean over valid samples (model_definition.py:277-278), partial sums per block
constexpr int MEAN_PARTS = 64;

__global__ void k_mean_partial(const float* __restrict__ pcm, int64_t stride, const int64_t* __restrict__ n_samples,
                               float* __restrict__ partial, int r16) {
  const int b = blockIdx.y, p = blockIdx.x;
  const int64_t n = n_samples[b];
  const int64_t chunk = (n + MEAN_PARTS - 1) / MEAN_PARTS;
  const int64_t lo = p * chunk, hi = min(n, lo + chunk);
  const float* x = pcm + b * stride;
  float acc = 0.f;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) acc += r16e(x[i], r16);
  __shared__ float red[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[b * MEAN_PARTS + p] = red[0] + red[1] + red[2] + red[3];
}

// pre-emphasis into the 200/200 zero-padded STFT input xp[b][0 .. xp_stride) (model_definition.py:279-282, 255)
__global__ void k_preemph_pad(const float* __restrict__ pcm, int64_t stride, const int64_t* __restrict__ n_samples,
                              const float* __restrict__ partial, float* __restrict__ xp, int64_t xp_stride, int r16) {
  const int b = blockIdx.y;
  __shared__ float s_mean;
  if (threadIdx.x < 64) {
    float v = threadIdx.x < MEAN_PARTS ? partial[b * MEAN_PARTS + threadIdx.x] : 0.f;
    v = wave_sum(v);
    if (threadIdx.x == 0) s_mean = r16e(v / (float)n_samples[b], r16);
  }
  __syncthreads();
  const float mean = s_mean;
  const int64_t n = n_samples[b];
  const float* x = pcm + b * stride;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < xp_stride; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t t = i - 200;
    float v = 0.f;
    if (t >= 0 && t < n) {
      const float a = r16e(r16e(x[t], r16) - mean, r16);
      v = t == 0 ? a : r16e(a - r16e(0.97f * r16e(r16e(x[t - 1], r16) - mean, r16), r16), r16);
    }
    xp[b * xp_stride + i] = v;
  }
}

void frontend_preemph(const float* pcm, int64_t stride, const int64_t* d_n_samples, int batch, float* partial,
                      float* xp, int64_t xp_stride, hipStream_t s, int r16) {
  hipLaunchKernelGGL(k_mean_partial, dim3(MEAN_PARTS, batch), dim3(256), 0, s, pcm, stride, d_n_samples, partial, r16);
  hipLaunchKernelGGL(k_preemph_pad, dim3(cdiv(xp_stride, 256 * 8), batch), dim3(256), 0, s, pcm, stride, d_n_samples,
                     partial, xp, xp_stride, r16);
}

// ---------------- F4: LFR (m=7, n=6) with replicate padding, mask, x*sqrt(512) + PE (model_definition.py:290-311, 206)
// x[b, i, j*80 + c] = mel[b, clamp(6i + j - 3, 0, t_mel_valid-1), c] for i < t_lfr_valid else 0; then *22.627417 + pe[i].
__global__ void k_lfr_pe(const float* __restrict__ mel, int mel_stride, const int* __restrict__ t_mel_valid,
                         const int* __restrict__ t_lfr_valid, const float* __restrict__ pe, float* __restrict__ x,
                         int t_stride, int n_mels, int lfr_m, int lfr_n, int r16) {
  const int b = blockIdx.y;
  const int d_in = n_mels * lfr_m;
  const int64_t total = (int64_t)t_stride * d_in;
  const int tmv = t_mel_valid[b], tlv = t_lfr_valid[b];
  const float sq = 22.627416997969522f;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    int i = (int)(e / d_in), jc = (int)(e - (int64_t)i * d_in);
    int j = jc / n_mels, c = jc - j * n_mels;
    float v = 0.f;
    if (i < tlv) {
      int p = i * lfr_n + j - (lfr_m - 1) / 2;
      p = p < 0 ? 0 : (p > tmv - 1 ? tmv - 1 : p);
      v = mel[((int64_t)b * mel_stride + p) * n_mels + c];
    }
    x[((int64_t)b * t_stride + i) * d_in + jc] =
        r16e(r16e(v * r16e(sq, r16), r16) + r16e(pe[(int64_t)i * d_in + jc], r16), r16);
  }
}

void frontend_lfr(const float* mel, int mel_stride, const int* t_mel_valid, const int* t_lfr_valid, const float* pe,
                  float* x, int batch, int t_stride, int n_mels, int lfr_m, int lfr_n, hipStream_t s, int r16) {
  int64_t total = (int64_t)t_stride * n_mels * lfr_m;
  hipLaunchKernelGGL(k_lfr_pe, dim3(std::min(cdiv(total, 256), 4096), batch), dim3(256), 0, s, mel, mel_stride,
                     t_mel_valid, t_lfr_valid, pe, x, t_stride, n_mels, lfr_m, lfr_n, r16);
}

// ---------------- E1: LayerNorm, one wave per row, optional row-mask sweep (model_definition.py:209-213)
template <int PER>
__global__ void k_layernorm(const float* __restrict__ x, int64_t ldx, float* __restrict__ y, int64_t ldy,
                            const float* __restrict__ w, const float* __restrict__ bb, int rows, int D, float eps,
                            const int* __restrict__ lens, int t_stride, int r16, APlanesD yp) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + (int64_t)row * ldx;
  float v[PER];
  float s = 0.f;
  // D == 64 PER with 16-B aligned rows: each lane owns PER contiguous columns (PER / 4 float4 loads, not PER dwords)
  const bool vec = PER % 4 == 0 && D == 64 * PER && (ldx & 3) == 0 && (ldy & 3) == 0 &&
                   ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(w) |
                     reinterpret_cast<uintptr_t>(bb)) & 15) == 0;
  if (vec) {
#pragma unroll
    for (int i = 0; i < PER; i += 4) {
      const float4 f = *reinterpret_cast<const float4*>(xr + lane * PER + i);
      v[i] = f.x; v[i + 1] = f.y; v[i + 2] = f.z; v[i + 3] = f.w;
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) s += v[i];
  } else {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int c = lane + i * 64;
      v[i] = c < D ? xr[c] : 0.f;
      s += v[i];
    }
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    int c = vec ? lane * PER + i : lane + i * 64;
    float dv = c < D ? v[i] - mean : 0.f;
    q += dv * dv;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
  float mk = 1.0f;
  if (lens) {
    int b = row / t_stride, t = row - b * t_stride;
    mk = t < lens[b] ? 1.0f : 0.0f;
  }
  const int64_t yo = (int64_t)row * ldy;
  if (vec) {
    float4 o[PER / 4];
#pragma unroll
    for (int i = 0; i < PER; i += 4) {
      const int c = lane * PER + i;
      const float4 wv = *reinterpret_cast<const float4*>(w + c), bv = *reinterpret_cast<const float4*>(bb + c);
      o[i / 4] = make_float4(r16e((v[i] - mean) * rstd * wv.x + bv.x, r16) * mk,
                             r16e((v[i + 1] - mean) * rstd * wv.y + bv.y, r16) * mk,
                             r16e((v[i + 2] - mean) * rstd * wv.z + bv.z, r16) * mk,
                             r16e((v[i + 3] - mean) * rstd * wv.w + bv.w, r16) * mk);
      if (!yp.hi) *reinterpret_cast<float4*>(y + yo + c) = o[i / 4];
    }
    if (yp.hi) {  // bf16x3 consumer only: the planes its staging would form from these f32 values, 16 B per store
      typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
#pragma unroll
      for (int i = 0; i < PER; i += 8) {
        bf16x4_t h0, l0, h1, l1;
        split_bf16x4(o[i / 4], h0, l0);
        if (i + 4 < PER) split_bf16x4(o[i / 4 + 1], h1, l1);
        const int c = lane * PER + i;
        if (i + 8 <= PER) {
          *reinterpret_cast<bf16x8_t*>(yp.hi + yo + c) = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
          *reinterpret_cast<bf16x8_t*>(yp.lo + yo + c) = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
        } else {
          *reinterpret_cast<bf16x4_t*>(yp.hi + yo + c) = h0;
          *reinterpret_cast<bf16x4_t*>(yp.lo + yo + c) = l0;
        }
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int c = lane + i * 64;
      if (c >= D) continue;
      const float o = r16e((v[i] - mean) * rstd * w[c] + bb[c], r16) * mk;
      if (yp.hi) split_bf16(o, yp.hi[yo + c], yp.lo[yo + c]);
      else y[yo + c] = o;
    }
  }
}

void layernorm(const float* x, int64_t ldx, float* y, int64_t ldy, const float* w, const float* b, int rows, int D,
               float eps, const int* lens, int t_stride, hipStream_t s, int r16, APlanes yp) {
  dim3 grid(cdiv(rows, 4));
  const APlanesD yd{reinterpret_cast<__bf16*>(yp.hi), reinterpret_cast<__bf16*>(yp.lo)};
  if (D <= 512) hipLaunchKernelGGL(k_layernorm<8>, grid, dim3(256), 0, s, x, ldx, y, ldy, w, b, rows, D, eps, lens, t_stride, r16, yd);
  else if (D <= 640) hipLaunchKernelGGL(k_layernorm<10>, grid, dim3(256), 0, s, x, ldx, y, ldy, w, b, rows, D, eps, lens, t_stride, r16, yd);
  else if (D <= 1024) hipLaunchKernelGGL(k_layernorm<16>, grid, dim3(256), 0, s, x, ldx, y, ldy, w, b, rows, D, eps, lens, t_stride, r16, yd);
  else FA_REQUIRE(false, "layernorm: D > 1024");
}

// ---------------- E4: FSMN memory = depthwise conv_k(v*m) (zero pad (k-1)/2) + v*m (model_definition.py:60-66)
// A lane owns one channel for FR consecutive rows: the FR + K - 1 input rows it needs are loaded once into
// registers (a wave reads 64 consecutive channels = 256 B per row), the K taps stay in registers, and each output
// row sums only inputs of its own clip that are inside the clip's valid length (the v*m mask + per-clip zero pad).
// FSMN_R rows per wave: 32 for batched encodes; 8 for one clip (T 1001 x 512 channels: 64 -> 256 blocks, 14 -> 5 us)
constexpr int FSMN_K = 11;
template <int FSMN_R>
__global__ __launch_bounds__(256) void k_fsmn(const float* __restrict__ v, int64_t ldv, const float* __restrict__ w,
                                              float* __restrict__ out, int64_t ldo, int rows, int C,
                                              const int* __restrict__ lens, int t_stride, int r16) {
  constexpr int LP = (FSMN_K - 1) / 2, NW = FSMN_R + FSMN_K - 1;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r0 = (blockIdx.y * 4 + (threadIdx.x >> 6)) * FSMN_R;
  if (c >= C || r0 >= rows) return;
  float wk[FSMN_K], win[NW];
#pragma unroll
  for (int j = 0; j < FSMN_K; ++j) wk[j] = r16e(w[c * FSMN_K + j], r16);
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int q = min(max(r0 - LP + i, 0), rows - 1);  // clamped address; out-of-clip taps are skipped below
    win[i] = v[(int64_t)q * ldv + c];
  }
#pragma unroll
  for (int i = 0; i < FSMN_R; ++i) {
    const int r = r0 + i;
    if (r >= rows) break;
    const int b = r / t_stride, lo = b * t_stride, hi = lo + (lens ? lens[b] : t_stride);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < FSMN_K; ++j) {
      const int q = r - LP + j;
      acc = fmaf(wk[j], (q >= lo && q < hi) ? win[i + j] : 0.f, acc);
    }
    const float self = r < hi ? win[i + LP] : 0.f;
    out[(int64_t)r * ldo + c] = r16e(r16e(acc, r16) + self, r16);
  }
}

// Batched encodes, 16-B lanes: a lane owns 4 consecutive channels (one float4 per row; a wave reads 1 KB rows as 16 B
// per lane instead of 4), FR rows. The per-channel arithmetic is k_fsmn's (same taps, same fmaf order): bit-identical.
template <int FR>
__global__ __launch_bounds__(256) void k_fsmn4(const float* __restrict__ v, int64_t ldv, const float* __restrict__ w,
                                               float* __restrict__ out, int64_t ldo, int rows, int C,
                                               const int* __restrict__ lens, int t_stride, int r16) {
  constexpr int LP = (FSMN_K - 1) / 2, NW = FR + FSMN_K - 1;
  const int c = 4 * (blockIdx.x * 64 + (threadIdx.x & 63));
  const int r0 = (blockIdx.y * 4 + (threadIdx.x >> 6)) * FR;
  if (c >= C || r0 >= rows) return;
  float4 wk[FSMN_K], win[NW];
#pragma unroll
  for (int j = 0; j < FSMN_K; ++j)
    wk[j] = make_float4(r16e(w[c * FSMN_K + j], r16), r16e(w[(c + 1) * FSMN_K + j], r16),
                        r16e(w[(c + 2) * FSMN_K + j], r16), r16e(w[(c + 3) * FSMN_K + j], r16));
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int q = min(max(r0 - LP + i, 0), rows - 1);  // clamped address; out-of-clip taps are skipped below
    win[i] = *reinterpret_cast<const float4*>(v + (int64_t)q * ldv + c);
  }
#pragma unroll
  for (int i = 0; i < FR; ++i) {
    const int r = r0 + i;
    if (r >= rows) break;
    const int b = r / t_stride, lo = b * t_stride, hi = lo + (lens ? lens[b] : t_stride);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < FSMN_K; ++j) {
      const int q = r - LP + j;
      const bool in = q >= lo && q < hi;
      acc.x = fmaf(wk[j].x, in ? win[i + j].x : 0.f, acc.x);
      acc.y = fmaf(wk[j].y, in ? win[i + j].y : 0.f, acc.y);
      acc.z = fmaf(wk[j].z, in ? win[i + j].z : 0.f, acc.z);
      acc.w = fmaf(wk[j].w, in ? win[i + j].w : 0.f, acc.w);
    }
    const bool sv = r < hi;
    const float4 self = win[i + LP];
    *reinterpret_cast<float4*>(out + (int64_t)r * ldo + c) =
        make_float4(r16e(r16e(acc.x, r16) + (sv ? self.x : 0.f), r16), r16e(r16e(acc.y, r16) + (sv ? self.y : 0.f), r16),
                    r16e(r16e(acc.z, r16) + (sv ? self.z : 0.f), r16), r16e(r16e(acc.w, r16) + (sv ? self.w : 0.f), r16));
  }
}

int g_fsmn_vec = 1;  // FUNASR_FSMN_VEC=0: the 4-B-lane kernel for batched encodes too (A/B)

void fsmn(const float* v, int64_t ldv, const float* w, float* out, int64_t ldo, int rows, int C, int ksize,
          const int* lens, int t_stride, hipStream_t s, int r16) {
  FA_REQUIRE(ksize == FSMN_K, "fsmn: kernel size 11 (SenseVoiceSmall sanm_shfit 0, kernel_size 11)");
  const bool vec = g_fsmn_vec && C % 256 == 0 && ldv % 4 == 0 && ldo % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(out)) % 16 == 0;
  if (vec && (int64_t)cdiv(C, 256) * cdiv(rows, 4 * 16) >= 512) {
    hipLaunchKernelGGL(k_fsmn4<16>, dim3(cdiv(C, 256), cdiv(rows, 4 * 16)), dim3(256), 0, s, v, ldv, w, out, ldo, rows,
                       C, lens, t_stride, r16);
    return;
  }
  if ((int64_t)cdiv(C, 64) * cdiv(rows, 4 * 32) >= 512)
    hipLaunchKernelGGL(k_fsmn<32>, dim3(cdiv(C, 64), cdiv(rows, 4 * 32)), dim3(256), 0, s, v, ldv, w, out, ldo, rows, C,
                       lens, t_stride, r16);
  else
    hipLaunchKernelGGL(k_fsmn<8>, dim3(cdiv(C, 64), cdiv(rows, 4 * 8)), dim3(256), 0, s, v, ldv, w, out, ldo, rows, C,
                       lens, t_stride, r16);
}

// ---------------- C2: CTC greedy collapse (nano_ctc.py:65-104): keep frame i iff id != blank and
// (i == 0 or id != id[i-1]); block-wide ballot + prefix sum compaction, one block per clip.
__global__ void k_ctc_collapse(const int* __restrict__ ids, int64_t ids_stride, const int* __restrict__ lens, int blank,
                               int* __restrict__ out_ids, int* __restrict__ out_frames, int64_t out_stride,
                               int* __restrict__ n_out) {
  const int b = blockIdx.x;
  const int n = lens[b];
  const int* x = ids + (int64_t)b * ids_stride;
  __shared__ int wave_cnt[16];
  __shared__ int base;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int c0 = 0; c0 < n; c0 += blockDim.x) {
    int i = c0 + threadIdx.x;
    bool keep = false;
    int id = 0;
    if (i < n) {
      id = x[i];
      keep = id != blank && (i == 0 || x[i - 1] != id);
    }
    unsigned long long bal = __ballot(keep);
    int pre = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wave_cnt[wave] = __popcll(bal);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wave; ++w) off += wave_cnt[w];
    if (keep) {
      out_ids[(int64_t)b * out_stride + off + pre] = id;
      out_frames[(int64_t)b * out_stride + off + pre] = i;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int w = 0; w < nw; ++w) tot += wave_cnt[w];
      base += tot;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) n_out[b] = base;
}

void ctc_collapse(const int* ids, int64_t ids_stride, const int* lens, int batch, int blank, int* out_ids,
                  int* out_frames, int64_t out_stride, int* n_out, hipStream_t s) {
  hipLaunchKernelGGL(k_ctc_collapse, dim3(batch), dim3(1024), 0, s, ids, ids_stride, lens, blank, out_ids, out_frames,
                     out_stride, n_out);
}

}  // namespace fa
