// FP32 GEMM on CDNA4 matrix cores: C[M,N] = epilogue(A[M,K] . W[N,K]^T)  (nn.Linear layout).
//
// v_mfma_f32_32x32x2_f32 (exact f32 fma chain, 157 TF/s dense peak on MI355X): lane l holds
// A[i=l&31][k=l>>5], B[k=l>>5][j=l&31]; accumulator reg r -> row (r&3)+8(r>>2)+4(l>>5), col l&31.
// Block tiles 64x64 or 128x128 (x32 in k), 4 waves, row-major LDS double-buffered (see Tile below).
// Used for every encoder/adaptor/CTC projection, the STFT-as-DFT-GEMM (F2) with a
// power epilogue (F3), the mel projection with a log epilogue, and the CTC projection with a fused
// row-argmax epilogue (C1) so the [T, 60515] logits never reach HBM.
#include <algorithm>
#include <type_traits>
#include "common.h"
#include "kernels.h"

namespace fa {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// fp16 encoder mode (C5, the reference's float16 ONNX graphs): every op's output is an fp16 value; held in f32
__device__ __forceinline__ float r16v(float v, int r16) { return r16 ? __half2float(__float2half_rn(v)) : v; }

constexpr int BK = 32;
int g_gemm_f32_split = 1;  // 0: no K splits (A/B)

// Block tile (64 WM) x (64 WN) x 32: 2x2 waves, each wave 32WM x 32WN = WM x WN accumulators of 32x32.
// LDS is row-major [row][k] with row stride 34 floats: the MFMA operand read of lane (r, h) hits bank
// (34 r + 2 kk + h) mod 64 = 2 (17 r mod 32) + h -> 64 distinct banks (17 is odd); each thread stores its
// 16-B global chunk as two aligned 8-B writes. Global loads cover 8 rows x 128 B per wave instruction.
// KB (the k depth of a stage) is 32, 64 or 128: row stride KB + 2 keeps (KB + 2) / 2 odd, so the bank argument holds.
template <int WM, int WN, int KB = BK>
struct Tile {
  static constexpr int BM = 64 * WM, BN = 64 * WN;
  static constexpr int LDK = KB + 2;
  static constexpr int R4 = KB / 4;                                     // float4 per tile row
  static constexpr int NA = BM * KB / 4 / 256, NB = BN * KB / 4 / 256;  // float4 per thread
  static constexpr int STAGE = (BM + BN) * LDK;                         // floats per LDS stage
};

struct ALoadPlain {
  const float* A;
  int64_t lda;
  __device__ __forceinline__ float4 load4(int row, int k, int M, int K) const {
    if (row >= M) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float* p = A + (int64_t)row * lda + k;
    if (k + 3 < K) return *reinterpret_cast<const float4*>(p);
    float4 r;
    r.x = k < K ? p[0] : 0.f;
    r.y = k + 1 < K ? p[1] : 0.f;
    r.z = k + 2 < K ? p[2] : 0.f;
    r.w = k + 3 < K ? p[3] : 0.f;
    return r;
  }
};

// bf16x3 A operand already split by its producer (APlanes): 8 k of one plane per 16-B load, lda % 8 == 0, K % 8 == 0
struct ALoadPlanes {
  const uint16_t* hi;
  const uint16_t* lo;
  int64_t lda;
  __device__ __forceinline__ void load8(int row, int k, int M, int K, uint4& h, uint4& l) const {
    if (row >= M || k >= K) {
      h = l = make_uint4(0, 0, 0, 0);
      return;
    }
    const int64_t o = (int64_t)row * lda + k;
    h = *reinterpret_cast<const uint4*>(hi + o);
    l = *reinterpret_cast<const uint4*>(lo + o);
  }
};
template <class AL>
struct IsPlanes {
  static constexpr bool value = false;
};
template <>
struct IsPlanes<ALoadPlanes> {
  static constexpr bool value = true;
};

// STFT framing (model_definition.py:255 F.pad + conv1d stride 160): row = clip*t_stride + t reads
// xp[clip][160 t + k] from the 200/200 zero-padded, pre-emphasised signal.
struct ALoadFrames {
  const float* xp;
  int64_t xp_stride;
  int t_stride, hop;
  __device__ __forceinline__ float4 load4(int row, int k, int M, int K) const {
    if (row >= M || k >= K) return make_float4(0.f, 0.f, 0.f, 0.f);  // K % 4 == 0
    int b = row / t_stride, t = row - b * t_stride;
    return *reinterpret_cast<const float4*>(xp + (int64_t)b * xp_stride + (int64_t)t * hop + k);
  }
};

__device__ __forceinline__ float4 load_w4(const float* __restrict__ W, int64_t ldw, int n, int k, int N, int K) {
  if (n >= N) return make_float4(0.f, 0.f, 0.f, 0.f);
  const float* p = W + (int64_t)n * ldw + k;
  if (k + 3 < K) return *reinterpret_cast<const float4*>(p);
  float4 r;
  r.x = k < K ? p[0] : 0.f;
  r.y = k + 1 < K ? p[1] : 0.f;
  r.z = k + 2 < K ? p[2] : 0.f;
  r.w = k + 3 < K ? p[3] : 0.f;
  return r;
}

template <int WM, int WN, int KB, class AL>
__device__ __forceinline__ void load_tiles(const AL& al, const float* __restrict__ W, int64_t ldw, int m0, int n0,
                                           int k0, int M, int N, int K, float4 (&ra)[Tile<WM, WN, KB>::NA],
                                           float4 (&rb)[Tile<WM, WN, KB>::NB]) {
  using T = Tile<WM, WN, KB>;
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < T::NA; ++i) {
    const int idx = t + i * 256;  // (row idx / R4, k4 idx % R4)
    ra[i] = al.load4(m0 + idx / T::R4, k0 + 4 * (idx % T::R4), M, K);
  }
#pragma unroll
  for (int i = 0; i < T::NB; ++i) {
    const int idx = t + i * 256;
    rb[i] = load_w4(W, ldw, n0 + idx / T::R4, k0 + 4 * (idx % T::R4), N, K);
  }
}

template <int WM, int WN, int KB>
__device__ __forceinline__ void store_tiles(float* As, float* Bs, const float4 (&ra)[Tile<WM, WN, KB>::NA],
                                            const float4 (&rb)[Tile<WM, WN, KB>::NB]) {
  using T = Tile<WM, WN, KB>;
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < T::NA; ++i) {
    const int idx = t + i * 256;
    float* d = As + (idx / T::R4) * T::LDK + 4 * (idx % T::R4);
    reinterpret_cast<float2*>(d)[0] = make_float2(ra[i].x, ra[i].y);
    reinterpret_cast<float2*>(d)[1] = make_float2(ra[i].z, ra[i].w);
  }
#pragma unroll
  for (int i = 0; i < T::NB; ++i) {
    const int idx = t + i * 256;
    float* d = Bs + (idx / T::R4) * T::LDK + 4 * (idx % T::R4);
    reinterpret_cast<float2*>(d)[0] = make_float2(rb[i].x, rb[i].y);
    reinterpret_cast<float2*>(d)[1] = make_float2(rb[i].z, rb[i].w);
  }
}

// ---------------------------------------------------------------------------------------------
// Epilogues. `apply` receives the wave's 32x32 accumulator at (row0, col0).
struct EpiLinear {
  float* C;
  int64_t ldc;
  const float* bias;
  const float* add1;  // residual (added last)
  int64_t ld1;
  const float* add2;  // e.g. FSMN memory (added before the residual, model_definition.py:90,109)
  int64_t ld2;
  int relu;
  int r16;            // fp16 mode: Gemm (+bias) output, then each Add, rounded to fp16
  __bf16* ph = nullptr;  // bf16x3 consumer only (ffn1 -> ffn2): C written as its hi / lo planes (ldc) instead of f32
  __bf16* pl = nullptr;
  __device__ __forceinline__ void finish(int, int, int, int, float*) const {}  // after every apply of the block
  // Row by row: each row's residual / memory operands are loaded behind the previous row's store (C may alias add1),
  // one memory round trip per row. Measured faster than EpiLinearG's four-row groups on the batched encoder's
  // 128x128 / 256x256 tiles (batch 6 / 32 encodes 27.8 / 98.1 vs 29.3 / 101.0 ms); the one-clip launches take
  // EpiLinearG.
  __device__ __forceinline__ void apply(const f32x16& acc, int row0, int col0, int M, int N, float* lds) const {
    int lane = threadIdx.x & 63;
    int col = col0 + (lane & 31);
    if (ph) {  // planes (host: N even): lane pairs swap values so the even lane stores the hi pair, the odd the lo pair
      const bool cin = col < N;
      const float b = bias && cin ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const bool in = cin && row < M;
        float v = acc[r] + b;
        if (relu) v = fmaxf(v, 0.f);
        if (add2 && in) v = v + add2[(int64_t)row * ld2 + col];
        if (add1 && in) v = add1[(int64_t)row * ld1 + col] + v;
        __bf16 h, l;
        split_bf16(v, h, l);
        const float mine = __uint_as_float(((uint32_t)__builtin_bit_cast(unsigned short, l) << 16) | __builtin_bit_cast(unsigned short, h));
        const uint32_t other = __float_as_uint(__shfl_xor(mine, 1, 64));  // the neighbour column's (hi, lo)
        const uint32_t me = __float_as_uint(mine);
        // even lane: (hi[col], hi[col + 1]); odd lane: (lo[col - 1], lo[col])
        const uint32_t word = (lane & 1) ? ((other >> 16) | (me & 0xffff0000u)) : ((me & 0xffffu) | (other << 16));
        if (in) *reinterpret_cast<uint32_t*>((lane & 1) ? pl + (int64_t)row * ldc + col - 1 : ph + (int64_t)row * ldc + col) = word;
      }
      return;
    }
    if (col >= N) return;
    float b = bias ? r16v(bias[col], r16) : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < M) {
        float v = r16v(acc[r] + b, r16);
        if (relu) v = fmaxf(v, 0.f);
        if (add2) v = r16v(v + add2[(int64_t)row * ld2 + col], r16);
        if (add1) v = r16v(add1[(int64_t)row * ld1 + col] + v, r16);
        C[(int64_t)row * ldc + col] = v;
      }
    }
  }
  // Four rows at a time (apply4: their residual / memory operands loaded first, then the arithmetic and stores),
  // the bias loaded once: EpiLinearG's apply (one-clip launches: 4-5 % faster one-clip encode)
  __device__ __forceinline__ void apply_grouped(const f32x16& acc, int row0, int col0, int M, int N) const {
    const float b = bias_of(col0 + (threadIdx.x & 31), N);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      apply4(f32x4_t{acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]}, q, row0, col0, M, N, b);
  }
  // the bias term of column col as apply4 adds it (planes: raw f32; f32 output: rounded in fp16 mode)
  __device__ __forceinline__ float bias_of(int col, int N) const {
    if (!bias || col >= N) return 0.f;
    return ph ? bias[col] : r16v(bias[col], r16);
  }
  // registers 4 q .. 4 q + 3 of a 32x32 accumulator (rows row0 + 8 q + {0..3} + 4 (lane >> 5)); also k_gemm_sk_reduce's
  // unit (one wave per quarter of an accumulator)
  __device__ __forceinline__ void apply4(const f32x4_t& a, int q, int row0, int col0, int M, int N, float b) const {
    const int lane = threadIdx.x & 63;
    const int col = col0 + (lane & 31);
    const int rb = row0 + 8 * q + 4 * (lane >> 5), cl = min(col, N - 1);
    float a2[4], a1[4];  // loaded first
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int64_t row = min(rb + t, M - 1);
      a2[t] = add2 ? add2[row * ld2 + cl] : 0.f;
      a1[t] = add1 ? add1[row * ld1 + cl] : 0.f;
    }
    if (ph) {
      const bool cin = col < N;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int row = rb + t;
        const bool in = cin && row < M;
        float v = a[t] + b;
        if (relu) v = fmaxf(v, 0.f);
        if (add2 && in) v = v + a2[t];
        if (add1 && in) v = a1[t] + v;
        __bf16 h, l;
        split_bf16(v, h, l);
        const float mine = __uint_as_float(((uint32_t)__builtin_bit_cast(unsigned short, l) << 16) | __builtin_bit_cast(unsigned short, h));
        const uint32_t other = __float_as_uint(__shfl_xor(mine, 1, 64));
        const uint32_t me = __float_as_uint(mine);
        const uint32_t word = (lane & 1) ? ((other >> 16) | (me & 0xffff0000u)) : ((me & 0xffffu) | (other << 16));
        if (in) *reinterpret_cast<uint32_t*>((lane & 1) ? pl + (int64_t)row * ldc + col - 1 : ph + (int64_t)row * ldc + col) = word;
      }
      return;
    }
    if (col >= N) return;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int row = rb + t;
      if (row < M) {
        float v = r16v(a[t] + b, r16);
        if (relu) v = fmaxf(v, 0.f);
        if (add2) v = r16v(v + a2[t], r16);
        if (add1) v = r16v(a1[t] + v, r16);
        C[(int64_t)row * ldc + col] = v;
      }
    }
  }
};

// EpiLinear with the four-row grouped apply (one-clip launches, gemm_linear's M <= G_ROWS_MAX): the same arithmetic
struct EpiLinearG : EpiLinear {
  __device__ __forceinline__ void apply(const f32x16& acc, int row0, int col0, int M, int N, float* lds) const {
    apply_grouped(acc, row0, col0, M, N);
  }
};
constexpr int G_ROWS_MAX = 2048;
int g_gemm_epi_grouped = 1;  // 0: every launch on the row-by-row epilogue (FUNASR_EPI_GROUPED; A/B)

// STFT: W rows interleave (cos_f, -sin_f); power[row][f] = re^2 + im^2 (model_definition.py:287).
struct EpiPower {
  float* P;
  int64_t ldp;
  int r16;
  __device__ __forceinline__ void finish(int, int, int, int, float*) const {}  // after every apply of the block
  __device__ __forceinline__ void apply(const f32x16& acc, int row0, int col0, int M, int N, float* lds) const {
    int lane = threadIdx.x & 63;
    int col = col0 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float v = acc[r];
      float o = __shfl_xor(v, 1, 64);
      int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (!(lane & 1) && row < M && col < N) {
        const float re = r16v(v, r16), im = r16v(o, r16);
        P[(int64_t)row * ldp + (col >> 1)] = r16v(r16v(re * re, r16) + r16v(im * im, r16), r16);
      }
    }
  }
};

// mel = log(fbank . power + 1e-7)
struct EpiLog {
  float* C;
  int64_t ldc;
  int r16;
  __device__ __forceinline__ void finish(int, int, int, int, float*) const {}  // after every apply of the block
  __device__ __forceinline__ void apply(const f32x16& acc, int row0, int col0, int M, int N, float* lds) const {
    int lane = threadIdx.x & 63;
    int col = col0 + (lane & 31);
    if (col >= N) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < M) C[(int64_t)row * ldc + col] = r16v(logf(r16v(r16v(acc[r], r16) + r16v(1e-7f, r16), r16)), r16);
    }
  }
};

// CTC projection + bias + row argmax over this block's 64 columns -> partial (value, index).
struct EpiArgmax {
  const float* bias;
  float* pval;   // [M][n_tiles]
  int* pidx;
  int n_tiles;
  int r16;  // fp16 mode: argmax over fp16 logits (ties resolve to the first index, as on the rounded values)
  __device__ __forceinline__ void finish(int, int, int, int, float*) const {}  // after every apply of the block
  __device__ __forceinline__ void apply(const f32x16& acc, int row0, int col0, int M, int N, float* lds) const {
    int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int col = col0 + (lane & 31);
    float b = col < N ? r16v(bias[col], r16) : 0.f;
    float* sv = lds;                              // [64 rows][2]
    int* si = reinterpret_cast<int*>(lds + 128);  // [64][2]
    int wr = wave >> 1, wc = wave & 1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float v = col < N ? r16v(acc[r] + b, r16) : -INFINITY;
      int i = col < N ? col : 0x7fffffff;
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) {
        float v2 = __shfl_xor(v, o, 32);
        int i2 = __shfl_xor(i, o, 32);
        argmax_combine(v, i, v2, i2);
      }
      if ((lane & 31) == 0) {
        int lr = wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        sv[lr * 2 + wc] = v;
        si[lr * 2 + wc] = i;
      }
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      int lr = threadIdx.x;
      int row = (row0 - (row0 % 64)) + lr;  // block row base
      float v = sv[lr * 2];
      int i = si[lr * 2];
      argmax_combine(v, i, sv[lr * 2 + 1], si[lr * 2 + 1]);
      int tile = col0 / 64;
      if (row < M) {
        pval[(int64_t)row * n_tiles + tile] = v;
        pidx[(int64_t)row * n_tiles + tile] = i;
      }
    }
  }
};

// CTC projection + bias + row argmax over a 128x128 block's columns (2x2 waves x 2x2 accumulators): every apply
// leaves its 32-column winners in LDS, finish merges the block's 4 column slices per row in column order ->
// partial (value, index) per (row, 128-column tile).
struct EpiArgmax128 {
  const float* bias;
  float* pval;   // [M][n_tiles]
  int* pidx;
  int n_tiles;
  int r16 = 0;  // fp16 mode: argmax over fp16 logits (Gemm + bias output rounded to fp16)
  // the wave's 32x32 sub-tile goes through LDS (a per-wave [32][33] scratch after the [128][4] winners) so each row's
  // 32 columns are scanned in registers by a lane pair (16 each) instead of a 5-step shuffle butterfly per row:
  // the epilogue was as long as the K = 512 main loop (CTC GEMM 12.3 ms per 32 clips vs 7.3 ms for a linear
  // epilogue of the same FLOPs)
  __device__ __forceinline__ void apply(const f32x16& acc, int row0, int col0, int M, int N, float* lds) const {
    const int lane = threadIdx.x & 63, wave = (threadIdx.x >> 6) & 3;
    const int col = col0 + (lane & 31);
    const float b = col < N ? r16v(bias[col], r16) : 0.f;
    float* sv = lds;                              // [128 rows][4 slices]
    int* si = reinterpret_cast<int*>(lds + 512);  // [128][4]
    float* scr = lds + 1024 + wave * (32 * 33);   // [32 rows][33]
    const int slice = (col0 & 127) >> 5, rb = row0 & 127;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      scr[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * 33 + (lane & 31)] = col < N ? r16v(acc[r] + b, r16) : -INFINITY;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int lr = lane >> 1, c0 = 16 * (lane & 1);  // lane pair -> row lr, columns [c0, c0 + 16)
    float v = scr[lr * 33 + c0];
    int i = col0 + c0 < N ? col0 + c0 : 0x7fffffff;
#pragma unroll
    for (int c = 1; c < 16; ++c) {
      const int cc = col0 + c0 + c;
      argmax_combine(v, i, scr[lr * 33 + c0 + c], cc < N ? cc : 0x7fffffff);
    }
    argmax_combine(v, i, __shfl_xor(v, 1, 64), __shfl_xor(i, 1, 64));
    if ((lane & 1) == 0) {
      sv[(rb + lr) * 4 + slice] = v;
      si[(rb + lr) * 4 + slice] = i;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the scratch is rewritten by the next sub-tile
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  __device__ __forceinline__ void finish(int m0, int n0, int M, int N, float* lds) const {
    const float* sv = lds;
    const int* si = reinterpret_cast<const int*>(lds + 512);
    __syncthreads();
    if (threadIdx.x < 128 && m0 + (int)threadIdx.x < M) {
      const int lr = threadIdx.x;
      float v = sv[lr * 4];
      int i = si[lr * 4];
#pragma unroll
      for (int c = 1; c < 4; ++c) argmax_combine(v, i, sv[lr * 4 + c], si[lr * 4 + c]);
      pval[(int64_t)(m0 + lr) * n_tiles + n0 / 128] = v;
      pidx[(int64_t)(m0 + lr) * n_tiles + n0 / 128] = i;
    }
  }
};

// The same for the 256x256 tile (8 waves as 2 x 4, each 4 x 2 sub-tiles): [256 rows][8 slices] winners, per-wave
// scratch, partial (value, index) per (row, 256-column tile). argmax_combine is associative with the lower index
// winning ties, so the winners equal the 128-column tiling's.
struct EpiArgmax256 {
  const float* bias;
  float* pval;   // [M][n_tiles]
  int* pidx;
  int n_tiles;
  int r16 = 0;  // fp16 mode: argmax over fp16 logits (Gemm + bias output rounded to fp16)
  __device__ __forceinline__ void apply(const f32x16& acc, int row0, int col0, int M, int N, float* lds) const {
    const int lane = threadIdx.x & 63, wave = (threadIdx.x >> 6) & 7;
    const int col = col0 + (lane & 31);
    const float b = col < N ? r16v(bias[col], r16) : 0.f;
    float* sv = lds;                               // [256 rows][8 slices]
    int* si = reinterpret_cast<int*>(lds + 2048);  // [256][8]
    float* scr = lds + 4096 + wave * (32 * 33);    // [32 rows][33]
    const int slice = (col0 & 255) >> 5, rb = row0 & 255;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      scr[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * 33 + (lane & 31)] = col < N ? r16v(acc[r] + b, r16) : -INFINITY;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int lr = lane >> 1, c0 = 16 * (lane & 1);  // lane pair -> row lr, columns [c0, c0 + 16)
    float v = scr[lr * 33 + c0];
    int i = col0 + c0 < N ? col0 + c0 : 0x7fffffff;
#pragma unroll
    for (int c = 1; c < 16; ++c) {
      const int cc = col0 + c0 + c;
      argmax_combine(v, i, scr[lr * 33 + c0 + c], cc < N ? cc : 0x7fffffff);
    }
    argmax_combine(v, i, __shfl_xor(v, 1, 64), __shfl_xor(i, 1, 64));
    if ((lane & 1) == 0) {
      sv[(rb + lr) * 8 + slice] = v;
      si[(rb + lr) * 8 + slice] = i;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the scratch is rewritten by the next sub-tile
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  __device__ __forceinline__ void finish(int m0, int n0, int M, int N, float* lds) const {
    const float* sv = lds;
    const int* si = reinterpret_cast<const int*>(lds + 2048);
    __syncthreads();
    if (threadIdx.x < 256 && m0 + (int)threadIdx.x < M) {
      const int lr = threadIdx.x;
      float v = sv[lr * 8];
      int i = si[lr * 8];
#pragma unroll
      for (int c = 1; c < 8; ++c) argmax_combine(v, i, sv[lr * 8 + c], si[lr * 8 + c]);
      pval[(int64_t)(m0 + lr) * n_tiles + n0 / 256] = v;
      pidx[(int64_t)(m0 + lr) * n_tiles + n0 / 256] = i;
    }
  }
};

// XCD-aware tile order. Workgroups are dealt round-robin over the 8 XCDs (blocks b and b + 8 share one L2,
// MI355X_MICROARCH.md "Workgroup dispatch"), so block b takes tile id (b % 8) * per + b / 8: each XCD owns one
// contiguous run of tile ids, and ids run through bands of 4 M-tiles (all N-tiles of a band, M fastest), so an XCD's
// blocks share a few A row bands and W column bands in its L2 instead of every XCD streaming all of A and W.
// Placement only decides speed; every tile is computed exactly once either way. false: padding block (no tile).
__device__ __forceinline__ void xcd_tile_of(int t, int nbx, int nby, int& tm, int& tn) {
  const int g = t / (4 * nbx), fm = 4 * g, gs = min(4, nby - fm), r = t - g * 4 * nbx;
  tm = fm + r % gs;
  tn = r / gs;
}
__device__ __forceinline__ bool xcd_tile(int nbx, int nby, int& tm, int& tn) {
  const int T = nbx * nby, per = (T + 7) >> 3, b = blockIdx.x;
  const int t = (b & 7) * per + (b >> 3);
  if (t >= T) return false;
  xcd_tile_of(t, nbx, nby, tm, tn);
  return true;
}
// Persistent form (gridDim.x a multiple of 8, at most one block per CU): block b's it-th tile is local index
// (b >> 3) + it * gridDim.x / 8 of XCD b % 8's contiguous run, so every tile is computed exactly once, on the XCD the
// one-block-per-tile grid would have used, and a block's epilogue stores stay in flight while its next tile's loads
// are issued. false: no tile left for this block.
__device__ __forceinline__ bool xcd_tile_it(int nbx, int nby, int it, bool persist, int& tm, int& tn) {
  if (!persist) return it == 0 && xcd_tile(nbx, nby, tm, tn);
  const int T = nbx * nby, per = (T + 7) >> 3, b = blockIdx.x;
  const int li = (b >> 3) + it * ((int)gridDim.x >> 3);
  const int t = (b & 7) * per + li;
  if (li >= per || t >= T) return false;
  xcd_tile_of(t, nbx, nby, tm, tn);
  return true;
}
inline dim3 xcd_grid(int nbx, int nby, int ks = 1) { return dim3(((nbx * nby + 7) >> 3) << 3, 1, ks); }

// gridDim.z = KS > 1 (64x64 tiles only): split z covers k in [z kper, (z + 1) kper); each split publishes its
// accumulators (sc1), counts its arrival on the tile's counter, and the last one sums all KS partials in split order
// (deterministic) and runs the epilogue (MI355X_MICROARCH.md hand-off table, row 1). Returns false in every block
// but that last one; there acc holds the sum and the counter is re-armed.
__device__ __forceinline__ bool split_combine(f32x16& acc, float* __restrict__ part, int* __restrict__ cnt, int tile) {
  __shared__ int s_last;
  const int KS = gridDim.z;
  float* base = part + (int64_t)tile * KS * 256 * 16;
  const __amdgpu_buffer_rsrc_t rs = buf_rsrc(base, KS * 256 * 16 * 4);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    st_sc1_f4(f32x4_t{acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]}, rs,
              ((blockIdx.z * 4 + q) * 256 + threadIdx.x) * 16);  // one 4-KB run per (split, q): full lines
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(cnt + tile * CNT_LINE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == KS - 1;
  __syncthreads();
  if (!s_last) return false;
  f32x4_t pv[GEMM_F32_KS_MAX][4];
#pragma unroll
  for (int z = 0; z < GEMM_F32_KS_MAX; ++z)  // all in flight; clamped duplicates past KS are not summed
#pragma unroll
    for (int q = 0; q < 4; ++q) pv[z][q] = ld_sc1_f4(rs, ((min(z, KS - 1) * 4 + q) * 256 + threadIdx.x) * 16);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x4_t t = pv[0][q];
#pragma unroll
    for (int z = 1; z < GEMM_F32_KS_MAX; ++z)
      if (z < KS) t += pv[z][q];
    acc[4 * q] = t.x; acc[4 * q + 1] = t.y; acc[4 * q + 2] = t.z; acc[4 * q + 3] = t.w;
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt + tile * CNT_LINE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// K-split factor of a 64x64-tile launch: up to 4 splits while the tiles leave most CUs idle, >= kmin of k per split
// (measured on the f32 kernel: ffn2 of one clip, N 512 K 2048, 60.7 -> 55.8 us; the K = 512 projections lose with 2)
int g_gemm_ks_force = 0;  // microbenchmark hook: K splits of 64x64-tile launches with a workspace (1, 2 or 4)
static int k_splits(int64_t tiles, int K, const GemmF32Work* wk, int kmin) {
  int ks = 1;
  if (wk && wk->part && g_gemm_ks_force && tiles <= wk->cnt_n && tiles * g_gemm_ks_force * 256 * 16 <= wk->part_n)
    return g_gemm_ks_force;
  if (wk && wk->part && g_gemm_f32_split)
    while (ks < GEMM_F32_KS_MAX && tiles * ks * 2 <= 512 && K / (2 * ks) >= kmin && tiles <= wk->cnt_n &&
           tiles * ks * 2 * 256 * 16 <= wk->part_n)
      ks *= 2;
  return ks;
}

// S = 1: write-after-barrier staging (k_gemm_bf3_256 S = 1); same MFMA order
template <class AL, class EPI, int WM, int WN, int KB, bool SPLIT = false, int S = 0>
__global__ __launch_bounds__(256) void k_gemm_f32(AL al, const float* __restrict__ W, int64_t ldw, int M, int N, int K,
                                                  EPI epi, float* __restrict__ part, int* __restrict__ cnt) {
  using T = Tile<WM, WN, KB>;
  constexpr int LDK = T::LDK;
  extern __shared__ float smem[];  // 2 stages x (A [BM][LDK], B [BN][LDK])
  int tm, tn;
  if (!xcd_tile((N + T::BN - 1) / T::BN, (M + T::BM - 1) / T::BM, tm, tn)) return;
  const int m0 = tm * T::BM, n0 = tn * T::BN;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const int r = lane & 31, h = lane >> 5;
  f32x16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x16{};
  float4 ra[T::NA], rb[T::NB];
  const int KS = SPLIT ? gridDim.z : 1;
  const int kper = (K + KB * KS - 1) / (KB * KS) * KB;
  const int kb0 = blockIdx.z * kper, ke = min(K, kb0 + kper);  // this split's k range (zero-filled past ke)
  load_tiles<WM, WN, KB>(al, W, ldw, m0, n0, kb0, M, N, ke, ra, rb);
  store_tiles<WM, WN, KB>(smem, smem + T::BM * LDK, ra, rb);
  const int nk = (ke - kb0 + KB - 1) / KB;
  if (S == 1 && nk > 1) load_tiles<WM, WN, KB>(al, W, ldw, m0, n0, kb0 + KB, M, N, ke, ra, rb);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if constexpr (S == 1) {
      if (kt + 1 < nk)
        store_tiles<WM, WN, KB>(smem + (cur ^ 1) * T::STAGE, smem + (cur ^ 1) * T::STAGE + T::BM * LDK, ra, rb);
      if (kt + 2 < nk) load_tiles<WM, WN, KB>(al, W, ldw, m0, n0, kb0 + (kt + 2) * KB, M, N, ke, ra, rb);
    } else {
      if (kt + 1 < nk) load_tiles<WM, WN, KB>(al, W, ldw, m0, n0, kb0 + (kt + 1) * KB, M, N, ke, ra, rb);
    }
    const float* a = smem + cur * T::STAGE + (wr * 32 * WM + r) * LDK + h;
    const float* b = smem + cur * T::STAGE + T::BM * LDK + (wc * 32 * WN + r) * LDK + h;
#pragma unroll
    for (int kk = 0; kk < KB / 2; ++kk) {
      float av[WM], bv[WN];
#pragma unroll
      for (int i = 0; i < WM; ++i) av[i] = a[32 * i * LDK + 2 * kk];
#pragma unroll
      for (int j = 0; j < WN; ++j) bv[j] = b[32 * j * LDK + 2 * kk];
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (S == 0 && kt + 1 < nk)
      store_tiles<WM, WN, KB>(smem + (cur ^ 1) * T::STAGE, smem + (cur ^ 1) * T::STAGE + T::BM * LDK, ra, rb);
    __syncthreads();
  }
  if constexpr (SPLIT && WM == 1 && WN == 1)
    if (!split_combine(acc[0][0], part, cnt, tm * ((N + T::BN - 1) / T::BN) + tn)) return;
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) epi.apply(acc[i][j], m0 + (wr * WM + i) * 32, n0 + (wc * WN + j) * 32, M, N, smem);
  epi.finish(m0, n0, M, N, smem);
}

int g_gemm_f32_wab = 0;  // exact-f32 tiles: 1 = write-after-barrier staging (FUNASR_F32_WAB)

template <class AL, class EPI, int WM, int WN, int KB, int S>
static void launch_gemm_s(const AL& al, const float* W, int64_t ldw, int M, int N, int K, const EPI& epi, hipStream_t s,
                          const GemmF32Work* wk) {
  using T = Tile<WM, WN, KB>;
  const int ks = WM == 1 && WN == 1 ? k_splits((int64_t)cdiv(N, T::BN) * cdiv(M, T::BM), K, wk, 512) : 1;
  const dim3 grid = xcd_grid(cdiv(N, T::BN), cdiv(M, T::BM), ks);
  const size_t lds = 2 * T::STAGE * sizeof(float);
  static bool attr = false;
  if (!attr && lds > 65536) {
    (void)hipFuncSetAttribute((const void*)k_gemm_f32<AL, EPI, WM, WN, KB, false, S>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)k_gemm_f32<AL, EPI, WM, WN, KB, true, S>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  if (ks > 1)
    hipLaunchKernelGGL((k_gemm_f32<AL, EPI, WM, WN, KB, true, S>), grid, dim3(256), lds, s, al, W, ldw, M, N, K, epi,
                       wk->part, wk->cnt);
  else
    hipLaunchKernelGGL((k_gemm_f32<AL, EPI, WM, WN, KB, false, S>), grid, dim3(256), lds, s, al, W, ldw, M, N, K, epi,
                       nullptr, nullptr);
}

template <class AL, class EPI, int WM, int WN, int KB = BK>
static void launch_gemm(const AL& al, const float* W, int64_t ldw, int M, int N, int K, const EPI& epi, hipStream_t s,
                        const GemmF32Work* wk = nullptr) {
  if (g_gemm_f32_wab) launch_gemm_s<AL, EPI, WM, WN, KB, 1>(al, W, ldw, M, N, K, epi, s, wk);
  else launch_gemm_s<AL, EPI, WM, WN, KB, 0>(al, W, ldw, M, N, K, epi, s, wk);
}

// 128x128 blocks (4 MFMA accumulators per wave: half the LDS reads per MFMA) when they still give every CU
// at least two blocks (batched encoder, C3); 64x64 blocks otherwise (single clip: fill the 256 CUs).
int g_gemm_f32_force = 0;  // microbenchmark hook: 1 = 64x64 blocks, 2 = 128x128 blocks

template <class AL, class EPI>
static void run_gemm(const AL& al, const float* W, int64_t ldw, int M, int N, int K, const EPI& epi, hipStream_t s,
                     bool allow_big = true, const GemmF32Work* wk = nullptr) {
  const bool big = g_gemm_f32_force ? g_gemm_f32_force == 2 : (int64_t)cdiv(M, 128) * cdiv(N, 128) >= 512;
  if (allow_big && big)
    launch_gemm<AL, EPI, 2, 2>(al, W, ldw, M, N, K, epi, s);
  else if (g_gemm_f32_force == 3)
    launch_gemm<AL, EPI, 1, 1, 64>(al, W, ldw, M, N, K, epi, s);
  else if (g_gemm_f32_force == 4)
    launch_gemm<AL, EPI, 1, 1, 128>(al, W, ldw, M, N, K, epi, s);
  else if (g_gemm_f32_force == 1 || (int64_t)cdiv(M, 64) * cdiv(N, 64) > 512)
    launch_gemm<AL, EPI, 1, 1>(al, W, ldw, M, N, K, epi, s, wk);
  else  // up to 2 blocks per CU: stage 64 of k (one clip: 4-8 % faster than 32; 5-12 % slower with many blocks)
    launch_gemm<AL, EPI, 1, 1, 64>(al, W, ldw, M, N, K, epi, s, wk);
}

// ---------------------------------------------------------------------------------------------
// fp16 encoder GEMM (C5): v_mfma_f32_32x32x16_f16, f16 x f16 products exact in the f32 accumulator. A comes from
// the f32 activation buffers (fp16 values in fp16 mode) and is converted while staged; W is the fp16 copy of the
// weight. Lane l holds A[i = l&31][k = 8 (l>>5) + 0..7] (one 16-B LDS read), B likewise; the accumulator layout is
// that of the f32 kernel, so the same epilogues apply. LDS rows of 40 halves (80 B): the 16 rows a 16-lane group
// reads start in 16 distinct 4-bank groups (20 r mod 64), conflict-free.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
constexpr int LDKH = BK + 8;
template <int WM, int WN>
struct Tile16 {
  static constexpr int BM = 64 * WM, BN = 64 * WN;
  static constexpr int NA = BM * BK / 4 / 256;    // float4 of A per thread
  static constexpr int NB = BN * BK / 8 / 256;    // 8 halves of W per thread
  static constexpr int STAGE = (BM + BN) * LDKH;  // halves per LDS stage
};

template <class AL, int WM, int WN>
__device__ __forceinline__ void load16(const AL& al, const __half* __restrict__ W, int64_t ldw, int m0, int n0, int k0,
                                       int M, int N, int K, float4 (&ra)[Tile16<WM, WN>::NA],
                                       uint4 (&rb)[Tile16<WM, WN>::NB]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < Tile16<WM, WN>::NA; ++i) {
    const int idx = t + i * 256;  // (row idx >> 3, k4 idx & 7)
    ra[i] = al.load4(m0 + (idx >> 3), k0 + 4 * (idx & 7), M, K);
  }
#pragma unroll
  for (int i = 0; i < Tile16<WM, WN>::NB; ++i) {
    const int idx = t + i * 256;  // (row idx >> 2, k8 idx & 3); K % 8 == 0
    const int n = n0 + (idx >> 2), k = k0 + 8 * (idx & 3);
    rb[i] = (n < N && k < K) ? *reinterpret_cast<const uint4*>(W + (int64_t)n * ldw + k) : make_uint4(0, 0, 0, 0);
  }
}

template <int WM, int WN>
__device__ __forceinline__ void store16(_Float16* As, _Float16* Bs, const float4 (&ra)[Tile16<WM, WN>::NA],
                                        const uint4 (&rb)[Tile16<WM, WN>::NB]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < Tile16<WM, WN>::NA; ++i) {
    const int idx = t + i * 256;
    const f16x4 v = {(_Float16)ra[i].x, (_Float16)ra[i].y, (_Float16)ra[i].z, (_Float16)ra[i].w};
    *reinterpret_cast<f16x4*>(As + (idx >> 3) * LDKH + 4 * (idx & 7)) = v;
  }
#pragma unroll
  for (int i = 0; i < Tile16<WM, WN>::NB; ++i) {
    const int idx = t + i * 256;
    *reinterpret_cast<uint4*>(Bs + (idx >> 2) * LDKH + 8 * (idx & 3)) = rb[i];
  }
}

template <class AL, class EPI, int WM, int WN>
__global__ __launch_bounds__(256) void k_gemm_f16(AL al, const __half* __restrict__ W, int64_t ldw, int M, int N, int K,
                                                  EPI epi) {
  using T = Tile16<WM, WN>;
  extern __shared__ float smem[];  // 2 stages x (A [BM][LDKH], W [BN][LDKH]) halves; the epilogue reuses it
  _Float16* sh = reinterpret_cast<_Float16*>(smem);
  int tm, tn;
  if (!xcd_tile((N + T::BN - 1) / T::BN, (M + T::BM - 1) / T::BM, tm, tn)) return;
  const int m0 = tm * T::BM, n0 = tn * T::BN;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const int r = lane & 31, h = lane >> 5;
  f32x16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x16{};
  float4 ra[T::NA];
  uint4 rb[T::NB];
  load16<AL, WM, WN>(al, W, ldw, m0, n0, 0, M, N, K, ra, rb);
  store16<WM, WN>(sh, sh + T::BM * LDKH, ra, rb);
  __syncthreads();
  const int nk = (K + BK - 1) / BK;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load16<AL, WM, WN>(al, W, ldw, m0, n0, (kt + 1) * BK, M, N, K, ra, rb);
    const _Float16* a = sh + cur * T::STAGE + (wr * 32 * WM + r) * LDKH + 8 * h;
    const _Float16* b = sh + cur * T::STAGE + T::BM * LDKH + (wc * 32 * WN + r) * LDKH + 8 * h;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      f16x8 av[WM], bv[WN];
#pragma unroll
      for (int i = 0; i < WM; ++i) av[i] = *reinterpret_cast<const f16x8*>(a + 32 * i * LDKH + 16 * kk);
#pragma unroll
      for (int j = 0; j < WN; ++j) bv[j] = *reinterpret_cast<const f16x8*>(b + 32 * j * LDKH + 16 * kk);
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store16<WM, WN>(sh + (cur ^ 1) * T::STAGE, sh + (cur ^ 1) * T::STAGE + T::BM * LDKH, ra, rb);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) epi.apply(acc[i][j], m0 + (wr * WM + i) * 32, n0 + (wc * WN + j) * 32, M, N, smem);
  epi.finish(m0, n0, M, N, smem);
}

template <class AL, class EPI, int WM, int WN>
static void launch_gemm16(const AL& al, const __half* W, int64_t ldw, int M, int N, int K, const EPI& epi,
                          hipStream_t s) {
  using T = Tile16<WM, WN>;
  FA_REQUIRE(K % 8 == 0 && ldw % 8 == 0, "gemm_f16: K and ldw must be multiples of 8");
  const dim3 grid = xcd_grid(cdiv(N, T::BN), cdiv(M, T::BM));
  const size_t lds = std::max<size_t>(2 * T::STAGE * sizeof(_Float16), 1024);  // >= EpiArgmax scratch
  hipLaunchKernelGGL((k_gemm_f16<AL, EPI, WM, WN>), grid, dim3(256), lds, s, al, W, ldw, M, N, K, epi);
}

template <class AL, class EPI>
static void run_gemm16(const AL& al, const __half* W, int64_t ldw, int M, int N, int K, const EPI& epi, hipStream_t s) {
  // 128x128 blocks once they still give every CU two; 64x64 otherwise
  if ((int64_t)cdiv(M, 128) * cdiv(N, 128) >= 512) launch_gemm16<AL, EPI, 2, 2>(al, W, ldw, M, N, K, epi, s);
  else launch_gemm16<AL, EPI, 1, 1>(al, W, ldw, M, N, K, epi, s);
}

// ---------------------------------------------------------------------------------------------
// bf16x3 split GEMM (f32 mode, the default encoder path): x = xh + xl with xh = bf16_rn(x) and xl = bf16_rn(x - xh)
// (x - xh is exact in f32), so x w ~= xh wh + xh wl + xl wh in the f32 accumulator; the dropped xl wl and the rounding
// of xl leave ~2^-16 relative error per product (numpy simulation over the full 10 s encoder golden: 1.7e-5 of the
// output range, CTC ids unchanged on non-tie frames; the GPU tests hold it to the f32 goldens' bars). Three
// v_mfma_f32_32x32x16_bf16 (32 cycles) replace eight v_mfma_f32_32x32x2_f32 (64 cycles) per 16 of k: 5.3x the
// exact-f32 MFMA rate. W is split once when the weights change (hi and lo planes [N][K], launch_split_bf16); A is
// split while it is staged. One LDS stage holds the four planes in rows of KB + 8 bf16 (80 or 144 B): the 16 rows
// one 16-lane group reads start in 16 distinct 4-bank groups, conflict-free. Operand maps and accumulator layout are
// the f16 kernel's, so the same epilogues apply.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
int g_gemm_bf3_pf = 2;     // few-tile bf16x3 shapes: global loads PF k-steps ahead (1 or 2; FUNASR_BF3_PF)
int g_gemm_bf3_force = 0;  // microbenchmark hook: 1 = 64x64x32, 2 = 128x128x32, 3 = 64x64x64, 4 / 5 = 64x64x64 / x32 K halves,
                           // 6 = 256x256x32, 7 = 128x64x32 K halves, 8 = 64x64 K quarters, 9 / 10 = 64x64x128
                           // (10: K halves for fp16)
int g_gemm_bf3_256 = 0;    // 256x256 tiles when a launch has at least this many (0 = off; FUNASR_BF3_256)
int g_gemm_f16_b3 = 1;     // fp16 graph GEMMs on the k_gemm_bf3 kernel family (P = 1); 0: k_gemm_f16 (FUNASR_F16_GEMM, A/B)
int g_gemm_bf3_256_s = 1;  // 256x256 / 128x128 tiles: 1 = write-after-barrier staging (FUNASR_BF3_256_S; A/B at
                           // M = 32032, scripts/ubench/gemm_f32_bench sched: 272-328 vs 185-222 TF/s, bit-identical;
                           // batch-32 encode 128.5-129.2 -> 109.7-109.9 ms)
int g_gemm_f16_deep = 1;   // fp16 graph one-clip shapes on 128-deep stages (FUNASR_F16_DEEP)
int g_gemm_bf3_kw4 = 0;    // few-tile shapes with K >= 2048 (one clip's ffn2): four K groups per block (FUNASR_BF3_KW4;
                           // A/B: ffn2 22.4 vs 23.7 us bf16x3, one-clip encode 10.43-10.63 vs 10.43-10.55 ms bf16x3,
                           // 8.68-8.74 vs 8.77-8.87 ms fp16: within run-to-run noise, not kept)
int g_gemm_bf3_mid = 0;    // 1: one clip's 256-1024-tile shapes (q|k|v, ffn1) on 128x64 tiles (FUNASR_BF3_MID; A/B: one-clip
                           // encode 10.47-10.94 vs 10.49 ms bf16x3, 8.74-8.75 vs 8.79-8.82 ms fp16: not kept)

// P = 3: bf16x3 split operands (two bf16 planes per operand, three MFMAs per 16 of k); P = 1: the fp16 graph (C5):
// one fp16 plane per operand (the activations are fp16 values, converted exactly while staged; W is the fp16 weight
// copy), one v_mfma_f32_32x32x16_f16 per 16 of k, f16 x f16 products exact in the f32 accumulator.
template <int P>
struct PrecB;
template <>
struct PrecB<3> {
  typedef __bf16 E;
  typedef bf16x8 V8;
  typedef bf16x4 V4;
  static constexpr int NPL = 2;
};
template <>
struct PrecB<1> {
  typedef _Float16 E;
  typedef f16x8 V8;
  typedef f16x4 V4;
  static constexpr int NPL = 1;
};
template <int P>
__device__ __forceinline__ f32x16 mfma_pb(const typename PrecB<P>::V8& a, const typename PrecB<P>::V8& b, const f32x16& c) {
  if constexpr (P == 3) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
// one 16-deep k-step of a 32x32 accumulator: bf16x3 lo.hi, hi.lo, hi.hi (this order everywhere); fp16 the one product
template <int P>
__device__ __forceinline__ void mma_step(f32x16& acc, const typename PrecB<P>::V8& ah, const typename PrecB<P>::V8& al,
                                         const typename PrecB<P>::V8& bh, const typename PrecB<P>::V8& bl) {
  if constexpr (P == 3) {
    acc = mfma_pb<3>(al, bh, acc);
    acc = mfma_pb<3>(ah, bl, acc);
  }
  acc = mfma_pb<P>(ah, bh, acc);
}

template <int WM, int WN, int KB, int P = 3>
struct TileB3 {
  static constexpr int BM = 64 * WM, BN = 64 * WN;
  static constexpr int LDK = KB + 8;                    // bf16 / f16 per LDS row
  static constexpr int R4 = KB / 4, R8 = KB / 8;        // float4 of A / 8-element chunks of W per tile row
  static constexpr int NA = BM * KB / 4 / 256;          // float4 of A per thread
  static constexpr int NB = BN * KB / 8 / 256;          // 8-element chunks of each W plane per thread
  static constexpr int PA = BM * LDK, PB = BN * LDK;    // elements per plane
  static constexpr int NPL = PrecB<P>::NPL;
  static constexpr int OB = NPL * PA;                   // W planes after the A planes
  static constexpr int STAGE = NPL * (PA + PB);         // [Ah][Al][Bh][Bl] (P = 1: [Ah][Bh])
};

template <class AL, int WM, int WN, int KB, int P>
__device__ __forceinline__ void load_b3(const AL& al, const typename PrecB<P>::E* __restrict__ Wh,
                                        const typename PrecB<P>::E* __restrict__ Wl, int64_t ldw, int m0, int n0, int k0,
                                        int M, int N, int K, float4 (&ra)[TileB3<WM, WN, KB, P>::NA],
                                        uint4 (&rh)[TileB3<WM, WN, KB, P>::NB], uint4 (&rl)[TileB3<WM, WN, KB, P>::NB],
                                        int t) {
  using T = TileB3<WM, WN, KB, P>;
  if constexpr (IsPlanes<AL>::value) {  // ra[0, NA/2): hi chunks, ra[NA/2, NA): lo chunks (8 k each)
    static_assert(P == 3 && T::NA % 2 == 0, "A planes: bf16x3 only");
    constexpr int NC = T::NA / 2;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int idx = t + i * 256;
      uint4 h, l;
      al.load8(m0 + idx / T::R8, k0 + 8 * (idx % T::R8), M, K, h, l);
      ra[i] = __builtin_bit_cast(float4, h);
      ra[NC + i] = __builtin_bit_cast(float4, l);
    }
  } else {
#pragma unroll
    for (int i = 0; i < T::NA; ++i) {
      const int idx = t + i * 256;
      ra[i] = al.load4(m0 + idx / T::R4, k0 + 4 * (idx % T::R4), M, K);
    }
  }
#pragma unroll
  for (int i = 0; i < T::NB; ++i) {
    const int idx = t + i * 256;  // K % 8 == 0
    const int n = n0 + idx / T::R8, k = k0 + 8 * (idx % T::R8);
    const bool in = n < N && k < K;
    const int64_t o = (int64_t)n * ldw + k;
    rh[i] = in ? *reinterpret_cast<const uint4*>(Wh + o) : make_uint4(0, 0, 0, 0);
    if constexpr (P == 3) rl[i] = in ? *reinterpret_cast<const uint4*>(Wl + o) : make_uint4(0, 0, 0, 0);
  }
}

template <int WM, int WN, int KB, int P, bool AP = false>
__device__ __forceinline__ void store_b3(typename PrecB<P>::E* st, const float4 (&ra)[TileB3<WM, WN, KB, P>::NA],
                                         const uint4 (&rh)[TileB3<WM, WN, KB, P>::NB],
                                         const uint4 (&rl)[TileB3<WM, WN, KB, P>::NB], int t) {
  using T = TileB3<WM, WN, KB, P>;
  typedef typename PrecB<P>::E E;
  typedef typename PrecB<P>::V4 V4;
  if constexpr (AP) {  // A planes (load_b3): whole 16-B chunks per plane, as W
    constexpr int NC = T::NA / 2;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int idx = t + i * 256;
      const int o = (idx / T::R8) * T::LDK + 8 * (idx % T::R8);
      *reinterpret_cast<float4*>(st + o) = ra[i];
      *reinterpret_cast<float4*>(st + T::PA + o) = ra[NC + i];
    }
  } else
#pragma unroll
  for (int i = 0; i < T::NA; ++i) {
    const int idx = t + i * 256;
    const float4 v = ra[i];
    const V4 h = {(E)v.x, (E)v.y, (E)v.z, (E)v.w};
    const int o = (idx / T::R4) * T::LDK + 4 * (idx % T::R4);
    *reinterpret_cast<V4*>(st + o) = h;
    if constexpr (P == 3) {
      const V4 l = {(E)(v.x - (float)h[0]), (E)(v.y - (float)h[1]), (E)(v.z - (float)h[2]), (E)(v.w - (float)h[3])};
      *reinterpret_cast<V4*>(st + T::PA + o) = l;
    }
  }
#pragma unroll
  for (int i = 0; i < T::NB; ++i) {
    const int idx = t + i * 256;
    const int o = (idx / T::R8) * T::LDK + 8 * (idx % T::R8);
    *reinterpret_cast<uint4*>(st + T::OB + o) = rh[i];
    if constexpr (P == 3) *reinterpret_cast<uint4*>(st + T::OB + T::PB + o) = rl[i];
  }
}

// Split-K partial of a 128x128 tile (4 waves as 2 x 2, 2 x 2 accumulators each) for k_gemm_sk_reduce:
// [split gridDim.z][tile][wave][i][j][q][lane] float4, 1 KiB per wave-instruction
__device__ __forceinline__ void sk_store_partial_impl(const f32x16& a, float* __restrict__ part, int64_t o) {
  f32x4_t* dst = reinterpret_cast<f32x4_t*>(part) + o;
#pragma unroll
  for (int q = 0; q < 4; ++q) dst[q * 64] = f32x4_t{a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]};
}
template <int WM, int WN>
__device__ __forceinline__ void sk_store_partial(const f32x16 (&acc)[WM][WN], float* __restrict__ part, int tile,
                                                 int ntiles, int wave, int lane) {
  static_assert(WM == 2 && WN == 2, "split partials: 128x128 tiles of 4 waves");
  const int64_t base = ((int64_t)blockIdx.z * ntiles + tile) * (4 * 4 * 16 * 64 / 4) + wave * 16 * 64 + lane;
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) sk_store_partial_impl(acc[i][j], part, base + (i * WN + j) * 4 * 64);
}

// KW = 2 / 4 (few-tile shapes): KW groups of 4 waves per block split K in equal parts, each with its own LDS stages;
// groups 1..KW-1 hand their accumulators to group 0 through LDS (summed in a fixed order) and group 0 runs the
// epilogue. KW times the waves per CU and 1/KW of the dependent k-steps per wave, with no cross-block split-K seam.
// PF = 2: the global loads run two k-steps ahead (two register sets, the k loop unrolled by two), so a k-step's
// tile has two steps of compute to land instead of one: few-tile shapes (one clip) have too little work per step to
// cover the load latency.
// SPL: gridDim.z splits K (KW = 1, 128x128 tiles): split z covers [z K / KS, (z + 1) K / KS) and stores its
// accumulators for k_gemm_sk_reduce instead of running the epilogue
template <class AL, class EPI, int WM, int WN, int KB, int KW = 1, int PF = 1, int P = 3, bool SPL = false>
__global__ __launch_bounds__(256 * KW) void k_gemm_bf3(AL al, const typename PrecB<P>::E* __restrict__ Wh,
                                                       const typename PrecB<P>::E* __restrict__ Wl, int64_t ldw, int M,
                                                       int N, int K, EPI epi, float* __restrict__ part) {
  using T = TileB3<WM, WN, KB, P>;
  typedef typename PrecB<P>::E E;
  typedef typename PrecB<P>::V8 V8;
  constexpr int LDK = T::LDK;
  extern __shared__ float smem[];  // KW x 2 stages; the epilogue reuses it
  int tm, tn;
  if (!xcd_tile((N + T::BN - 1) / T::BN, (M + T::BM - 1) / T::BM, tm, tn)) return;
  const int m0 = tm * T::BM, n0 = tn * T::BN;
  const int grp = KW > 1 ? (int)(threadIdx.x >> 8) : 0, t = threadIdx.x & 255;
  E* sh = reinterpret_cast<E*>(smem) + grp * 2 * T::STAGE;
  const int wave = t >> 6, lane = t & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const int r = lane & 31, h = lane >> 5;
  f32x16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x16{};
  float4 ra[T::NA];
  uint4 rh[T::NB], rl[T::NB];
  const int kz = SPL ? K / (int)gridDim.z : K;  // host: K % (KS * KB) == 0 when split
  const int kq = kz / KW, kb0 = (SPL ? (int)blockIdx.z * kz : 0) + grp * kq, ke = kb0 + kq;  // K % (KW * KB) == 0, KW > 1
  load_b3<AL, WM, WN, KB, P>(al, Wh, Wl, ldw, m0, n0, kb0, M, N, ke, ra, rh, rl, t);
  store_b3<WM, WN, KB, P, IsPlanes<AL>::value>(sh, ra, rh, rl, t);
  __syncthreads();
  const int nk = (kq + KB - 1) / KB;
  auto compute = [&](const E* stage) {
    const E* a = stage + (wr * 32 * WM + r) * LDK + 8 * h;
    const E* b = stage + T::OB + (wc * 32 * WN + r) * LDK + 8 * h;
#pragma unroll
    for (int kk = 0; kk < KB / 16; ++kk) {
      V8 ah[WM], alo[WM], bh[WN], blo[WN];
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        ah[i] = *reinterpret_cast<const V8*>(a + 32 * i * LDK + 16 * kk);
        if constexpr (P == 3) alo[i] = *reinterpret_cast<const V8*>(a + T::PA + 32 * i * LDK + 16 * kk);
      }
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        bh[j] = *reinterpret_cast<const V8*>(b + 32 * j * LDK + 16 * kk);
        if constexpr (P == 3) blo[j] = *reinterpret_cast<const V8*>(b + T::PB + 32 * j * LDK + 16 * kk);
      }
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j) mma_step<P>(acc[i][j], ah[i], alo[i], bh[j], blo[j]);
    }
  };
  if constexpr (PF == 1) {
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk)
        load_b3<AL, WM, WN, KB, P>(al, Wh, Wl, ldw, m0, n0, kb0 + (kt + 1) * KB, M, N, ke, ra, rh, rl, t);
      compute(sh + cur * T::STAGE);
      if (kt + 1 < nk) store_b3<WM, WN, KB, P, IsPlanes<AL>::value>(sh + (cur ^ 1) * T::STAGE, ra, rh, rl, t);
      __syncthreads();
    }
  } else if constexpr (PF == 3) {
    // write-after-barrier (k_gemm_bf3_256 S = 1): tile kt + 1, loaded a whole step earlier, goes to the free stage at
    // the top of step kt, then the same registers take tile kt + 2's loads
    if (nk > 1) load_b3<AL, WM, WN, KB, P>(al, Wh, Wl, ldw, m0, n0, kb0 + KB, M, N, ke, ra, rh, rl, t);
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) store_b3<WM, WN, KB, P, IsPlanes<AL>::value>(sh + (cur ^ 1) * T::STAGE, ra, rh, rl, t);
      if (kt + 2 < nk)
        load_b3<AL, WM, WN, KB, P>(al, Wh, Wl, ldw, m0, n0, kb0 + (kt + 2) * KB, M, N, ke, ra, rh, rl, t);
      compute(sh + cur * T::STAGE);
      __syncthreads();
    }
  } else {
    // set A (ra, rh, rl) carries the odd k-steps, set B the even ones from step 2 on; step j is loaded right after
    // step j - 2's set was stored, i.e. two compute steps before it is stored itself
    float4 rb[T::NA];
    uint4 rhb[T::NB], rlb[T::NB];
    if (nk > 1) load_b3<AL, WM, WN, KB, P>(al, Wh, Wl, ldw, m0, n0, kb0 + KB, M, N, ke, ra, rh, rl, t);
    if (nk > 2) load_b3<AL, WM, WN, KB, P>(al, Wh, Wl, ldw, m0, n0, kb0 + 2 * KB, M, N, ke, rb, rhb, rlb, t);
    for (int kt = 0; kt < nk; kt += 2) {
      compute(sh);  // step kt (stage 0)
      if (kt + 1 < nk) store_b3<WM, WN, KB, P, IsPlanes<AL>::value>(sh + T::STAGE, ra, rh, rl, t);
      if (kt + 3 < nk)
        load_b3<AL, WM, WN, KB, P>(al, Wh, Wl, ldw, m0, n0, kb0 + (kt + 3) * KB, M, N, ke, ra, rh, rl, t);
      __syncthreads();
      if (kt + 1 >= nk) break;
      compute(sh + T::STAGE);  // step kt + 1 (stage 1)
      if (kt + 2 < nk) store_b3<WM, WN, KB, P, IsPlanes<AL>::value>(sh, rb, rhb, rlb, t);
      if (kt + 4 < nk)
        load_b3<AL, WM, WN, KB, P>(al, Wh, Wl, ldw, m0, n0, kb0 + (kt + 4) * KB, M, N, ke, rb, rhb, rlb, t);
      __syncthreads();
    }
  }
  if constexpr (KW > 1) {
    constexpr int XS = 4 * WM * WN * 16 * 64;  // floats per group
    float* xs = smem;  // [group - 1][wave][i][j][16][64]: groups 1..KW-1's accumulators
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q)
          if (grp > 0) xs[(grp - 1) * XS + (((wave * WM + i) * WN + j) * 16 + q) * 64 + lane] = acc[i][j][q];
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int g = 1; g < KW; ++g)  // fixed order: K quarters ascending
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q)
              acc[i][j][q] += xs[(g - 1) * XS + (((wave * WM + i) * WN + j) * 16 + q) * 64 + lane];
    }
    __syncthreads();  // the epilogue may reuse the LDS
    if (grp > 0) return;
  }
  if constexpr (SPL) {
    static_assert(KW == 1, "split partials: one K group");
    const int nbx = (N + T::BN - 1) / T::BN;
    sk_store_partial<WM, WN>(acc, part, tm * nbx + tn, nbx * ((M + T::BM - 1) / T::BM), wave, lane);
    return;
  }
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) epi.apply(acc[i][j], m0 + (wr * WM + i) * 32, n0 + (wc * WN + j) * 32, M, N, smem);
  epi.finish(m0, n0, M, N, smem);
}

// No K splits: the bf16x3 body is fast enough that the split-K seam (publish + ticket + combine, 5-13 us:
// MI355X_MICROARCH.md splitk-seam) costs more than it saves (one clip, measured: out N 512 K 512 10.8 -> 19.8 us,
// ffn2 N 512 K 2048 32.6 -> 57 us with 2-4 splits).
template <class AL, class EPI, int WM, int WN, int KB, int KW = 1, int PF = 1, int P = 3>
static void launch_gemm_b3(const AL& al, const WSplit& w, int64_t ldw, int M, int N, int K, const EPI& epi,
                           hipStream_t s) {
  using T = TileB3<WM, WN, KB, P>;
  typedef typename PrecB<P>::E E;
  FA_REQUIRE(K % 8 == 0 && ldw % 8 == 0, "gemm_bf3: K and ldw must be multiples of 8");
  FA_REQUIRE(KW == 1 || K % (KW * KB) == 0, "gemm_bf3: K groups need K % (KW * KB) == 0");
  const dim3 grid = xcd_grid(cdiv(N, T::BN), cdiv(M, T::BM));
  // >= EpiArgmax / EpiArgmax128 scratch, >= the KW = 2 accumulator hand-off
  const size_t lds = std::max<size_t>({(size_t)KW * 2 * T::STAGE * 2, (size_t)(1024 + 4 * 32 * 33) * 4,
                                       (size_t)(KW - 1) * 4 * WM * WN * 16 * 64 * 4});
  static bool attr = false;
  if (!attr && lds > 65536) {
    (void)hipFuncSetAttribute((const void*)k_gemm_bf3<AL, EPI, WM, WN, KB, KW, PF, P>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((k_gemm_bf3<AL, EPI, WM, WN, KB, KW, PF, P>), grid, dim3(256 * KW), lds, s, al,
                     reinterpret_cast<const E*>(w.hi), reinterpret_cast<const E*>(w.lo), ldw, M, N, K, epi, nullptr);
}

// 256x256x32 tile (batched encoder, C3; P = 3 bf16x3, P = 1 the fp16 graph): 8 waves as 2 (M) x 4 (N), each wave
// 128 x 64 = 4 x 2 accumulators of 32x32, 512 threads, one block per CU. Per 16 of k a bf16x3 wave reads 12 fragments
// (4 + 2 tiles, two planes) for 24 MFMAs (the 128x128 tile: 8 for 12), and a k-step has 48 MFMAs per wave between
// barriers. Same stage layout, operand maps, per-element MFMA order (lo.hi, hi.lo, hi.hi per 16 of k, k ascending) and
// epilogue calls as k_gemm_bf3: every output is bit-identical to the 128x128 and 64x64 tiles. LDS: two stages of 4
// planes x 256 rows x 80 B = 160 KiB (fp16: 2 planes, 80 KiB).
#ifndef B3B_VARIANT
// A/B only (scripts/gpu_r3_g256b.sh, M = 32032): 1 = MFMA blocks at raised wave priority (275-325 TF/s), 2 = also the
// next stage stored between the k halves (193-229 TF/s); 0 (292-330 TF/s) stays. Diagnostics (wrong results):
// 3 = no global loads after the first stage (LDS reads + MFMAs only), 4 = no MFMAs (loads, stores, LDS reads only)
#define B3B_VARIANT 0
#endif
constexpr int B3B_T = 512, B3B_BM = 256, B3B_BN = 256, B3B_KB = 32, B3B_LDK = B3B_KB + 8;
constexpr int B3B_PA = B3B_BM * B3B_LDK, B3B_PB = B3B_BN * B3B_LDK;  // elements per plane
constexpr int B3B_NA = B3B_BM * B3B_KB / 4 / B3B_T;                  // float4 of A per thread (4)
constexpr int B3B_NB = B3B_BN * B3B_KB / 8 / B3B_T;                  // 8-element chunks of each W plane per thread (2)
template <int P>
struct B3BT {
  static constexpr int NPL = PrecB<P>::NPL;
  static constexpr int OB = NPL * B3B_PA;                            // W planes after the A planes
  static constexpr int STAGE = NPL * (B3B_PA + B3B_PB);              // [Ah][Al][Bh][Bl] (P = 1: [Ah][Bh])
  static constexpr size_t LDS = std::max<size_t>(2 * STAGE * 2, (4096 + 8 * 32 * 33) * 4);  // >= EpiArgmax256
};

template <class AL, int P>
__device__ __forceinline__ void load_b3b(const AL& al, const typename PrecB<P>::E* __restrict__ Wh,
                                         const typename PrecB<P>::E* __restrict__ Wl, int64_t ldw, int m0, int n0, int k0,
                                         int M, int N, int K, float4 (&ra)[B3B_NA], uint4 (&rh)[B3B_NB],
                                         uint4 (&rl)[B3B_NB], int t) {
  constexpr int R4 = B3B_KB / 4, R8 = B3B_KB / 8;
  if constexpr (IsPlanes<AL>::value) {  // as load_b3
    static_assert(P == 3 && B3B_NA % 2 == 0, "A planes: bf16x3 only");
    constexpr int NC = B3B_NA / 2;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int idx = t + i * B3B_T;
      uint4 h, l;
      al.load8(m0 + idx / R8, k0 + 8 * (idx % R8), M, K, h, l);
      ra[i] = __builtin_bit_cast(float4, h);
      ra[NC + i] = __builtin_bit_cast(float4, l);
    }
  } else {
#pragma unroll
    for (int i = 0; i < B3B_NA; ++i) {
      const int idx = t + i * B3B_T;
      ra[i] = al.load4(m0 + idx / R4, k0 + 4 * (idx % R4), M, K);
    }
  }
#pragma unroll
  for (int i = 0; i < B3B_NB; ++i) {
    const int idx = t + i * B3B_T;  // K % 8 == 0
    const int n = n0 + idx / R8, k = k0 + 8 * (idx % R8);
    const bool in = n < N && k < K;
    const int64_t o = (int64_t)n * ldw + k;
    rh[i] = in ? *reinterpret_cast<const uint4*>(Wh + o) : make_uint4(0, 0, 0, 0);
    if constexpr (P == 3) rl[i] = in ? *reinterpret_cast<const uint4*>(Wl + o) : make_uint4(0, 0, 0, 0);
  }
}

template <int P, bool AP = false>
__device__ __forceinline__ void store_b3b(typename PrecB<P>::E* st, const float4 (&ra)[B3B_NA], const uint4 (&rh)[B3B_NB],
                                          const uint4 (&rl)[B3B_NB], int t) {
  constexpr int R4 = B3B_KB / 4, R8 = B3B_KB / 8;
  typedef typename PrecB<P>::E E;
  typedef typename PrecB<P>::V4 V4;
  if constexpr (AP) {  // A planes: whole 16-B chunks per plane
    constexpr int NC = B3B_NA / 2;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int idx = t + i * B3B_T;
      const int o = (idx / R8) * B3B_LDK + 8 * (idx % R8);
      *reinterpret_cast<float4*>(st + o) = ra[i];
      *reinterpret_cast<float4*>(st + B3B_PA + o) = ra[NC + i];
    }
  } else
#pragma unroll
  for (int i = 0; i < B3B_NA; ++i) {
    const int idx = t + i * B3B_T;
    const float4 v = ra[i];
    const V4 h = {(E)v.x, (E)v.y, (E)v.z, (E)v.w};
    const int o = (idx / R4) * B3B_LDK + 4 * (idx % R4);
    *reinterpret_cast<V4*>(st + o) = h;
    if constexpr (P == 3) {
      const V4 l = {(E)(v.x - (float)h[0]), (E)(v.y - (float)h[1]), (E)(v.z - (float)h[2]), (E)(v.w - (float)h[3])};
      *reinterpret_cast<V4*>(st + B3B_PA + o) = l;
    }
  }
#pragma unroll
  for (int i = 0; i < B3B_NB; ++i) {
    const int idx = t + i * B3B_T;
    const int o = (idx / R8) * B3B_LDK + 8 * (idx % R8);
    *reinterpret_cast<uint4*>(st + B3BT<P>::OB + o) = rh[i];
    if constexpr (P == 3) *reinterpret_cast<uint4*>(st + B3BT<P>::OB + B3B_PB + o) = rl[i];
  }
}

// S = 1: write-after-barrier staging (cdna_hip_programming.md T14): step kt first stores the registers holding tile
// kt + 1 (loaded a whole step earlier) into the free stage, re-issues the loads of tile kt + 2 into the same registers,
// then computes tile kt; S = 0 loads tile kt + 1 at the top of step kt and stores it after the compute. Same MFMA order.
template <class AL, class EPI, int P = 3, int S = 0, bool PER = false>
__global__ __launch_bounds__(B3B_T, 1) void k_gemm_bf3_256(AL al, const typename PrecB<P>::E* __restrict__ Wh,
                                                            const typename PrecB<P>::E* __restrict__ Wl, int64_t ldw,
                                                            int M, int N, int K, EPI epi) {
  constexpr int WM = 4, WN = 2, LDK = B3B_LDK;
  constexpr int STAGE = B3BT<P>::STAGE, OB = B3BT<P>::OB;
  typedef typename PrecB<P>::E E;
  typedef typename PrecB<P>::V8 V8;
  extern __shared__ float smem[];  // 2 stages; the epilogue reuses it
  for (int it = 0; it < (PER ? 0x7fffffff : 1); ++it) {
  int tm, tn;
  if (!xcd_tile_it((N + B3B_BN - 1) / B3B_BN, (M + B3B_BM - 1) / B3B_BM, it, PER, tm, tn)) return;
  if (PER && it) __syncthreads();  // the previous tile's epilogue may have used the LDS
  const int m0 = tm * B3B_BM, n0 = tn * B3B_BN;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int wr = wave >> 2, wc = wave & 3;
  const int r = lane & 31, h = lane >> 5;
  E* sh = reinterpret_cast<E*>(smem);
  f32x16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x16{};
  float4 ra[B3B_NA];
  uint4 rh[B3B_NB], rl[B3B_NB];
  load_b3b<AL, P>(al, Wh, Wl, ldw, m0, n0, 0, M, N, K, ra, rh, rl, t);
  store_b3b<P, IsPlanes<AL>::value>(sh, ra, rh, rl, t);
  const int nk = (K + B3B_KB - 1) / B3B_KB;
  if (S == 1 && nk > 1) load_b3b<AL, P>(al, Wh, Wl, ldw, m0, n0, B3B_KB, M, N, K, ra, rh, rl, t);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if constexpr (S == 1) {
      if (kt + 1 < nk) store_b3b<P, IsPlanes<AL>::value>(sh + (cur ^ 1) * STAGE, ra, rh, rl, t);
      if (kt + 2 < nk) load_b3b<AL, P>(al, Wh, Wl, ldw, m0, n0, (kt + 2) * B3B_KB, M, N, K, ra, rh, rl, t);
    }
#if B3B_VARIANT != 3
    if (S == 0 && kt + 1 < nk) load_b3b<AL, P>(al, Wh, Wl, ldw, m0, n0, (kt + 1) * B3B_KB, M, N, K, ra, rh, rl, t);
#endif
    const E* stage = sh + cur * STAGE;
    const E* a = stage + (wr * 32 * WM + r) * LDK + 8 * h;
    const E* b = stage + OB + (wc * 32 * WN + r) * LDK + 8 * h;
#pragma unroll
    for (int kk = 0; kk < B3B_KB / 16; ++kk) {
#if B3B_VARIANT == 2
      if (kk == 1 && kt + 1 < nk) store_b3b<P, IsPlanes<AL>::value>(sh + (cur ^ 1) * STAGE, ra, rh, rl, t);
#endif
      V8 ah[WM], alo[WM], bh[WN], blo[WN];
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        bh[j] = *reinterpret_cast<const V8*>(b + 32 * j * LDK + 16 * kk);
        if constexpr (P == 3) blo[j] = *reinterpret_cast<const V8*>(b + B3B_PB + 32 * j * LDK + 16 * kk);
      }
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        ah[i] = *reinterpret_cast<const V8*>(a + 32 * i * LDK + 16 * kk);
        if constexpr (P == 3) alo[i] = *reinterpret_cast<const V8*>(a + B3B_PA + 32 * i * LDK + 16 * kk);
      }
#if B3B_VARIANT == 1 || B3B_VARIANT == 2
      __builtin_amdgcn_s_setprio(1);
#endif
#if B3B_VARIANT == 4
#pragma unroll
      for (int i = 0; i < WM; ++i) asm volatile("" ::"v"(ah[i]), "v"(alo[i]));
#pragma unroll
      for (int j = 0; j < WN; ++j) asm volatile("" ::"v"(bh[j]), "v"(blo[j]));
#else
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j) mma_step<P>(acc[i][j], ah[i], alo[i], bh[j], blo[j]);
#endif
#if B3B_VARIANT == 1 || B3B_VARIANT == 2
      __builtin_amdgcn_s_setprio(0);
#endif
    }
#if B3B_VARIANT != 2 && B3B_VARIANT != 3
    if (S == 0 && kt + 1 < nk) store_b3b<P, IsPlanes<AL>::value>(sh + (cur ^ 1) * STAGE, ra, rh, rl, t);
#endif
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) epi.apply(acc[i][j], m0 + (wr * WM + i) * 32, n0 + (wc * WN + j) * 32, M, N, smem);
  epi.finish(m0, n0, M, N, smem);
  }
}

int g_gemm_bf3_persist = 0;  // 256x256 tiles: persistent blocks, one per CU (FUNASR_BF3_PERSIST; A/B: batch-32 encode
                             // 105.1-105.9 vs 103.7-104.3 ms on f32 rows, no change on planes)
static int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    FA_HIP(hipGetDevice(&dev));
    FA_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    n = std::max(8, n & ~7);
  }
  return n;
}
// persistent grid: one block per CU (a multiple of 8), never more blocks than the one-block-per-tile grid
static dim3 persist_grid(const dim3& g) { return dim3(std::min<unsigned>(g.x, (unsigned)cu_count()), 1, 1); }

template <class AL, class EPI, int P, int S>
static void launch_gemm_b3_256_s(const AL& al, const WSplit& w, int64_t ldw, int M, int N, int K, const EPI& epi,
                                 hipStream_t s) {
  typedef typename PrecB<P>::E E;
  static bool attr = false;
  if (!attr) {
    FA_HIP(hipFuncSetAttribute((const void*)k_gemm_bf3_256<AL, EPI, P, S>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)B3BT<P>::LDS));
    FA_HIP(hipFuncSetAttribute((const void*)k_gemm_bf3_256<AL, EPI, P, S, true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)B3BT<P>::LDS));
    attr = true;
  }
  const dim3 grid = xcd_grid(cdiv(N, B3B_BN), cdiv(M, B3B_BM));
  if (g_gemm_bf3_persist)
    hipLaunchKernelGGL((k_gemm_bf3_256<AL, EPI, P, S, true>), persist_grid(grid), dim3(B3B_T), B3BT<P>::LDS, s, al,
                       reinterpret_cast<const E*>(w.hi), reinterpret_cast<const E*>(w.lo), ldw, M, N, K, epi);
  else
    hipLaunchKernelGGL((k_gemm_bf3_256<AL, EPI, P, S>), grid, dim3(B3B_T), B3BT<P>::LDS, s, al,
                       reinterpret_cast<const E*>(w.hi), reinterpret_cast<const E*>(w.lo), ldw, M, N, K, epi);
}

// ---- 256x256 bf16x3 tile with both operands as bf16 planes (A from its producer's APlanes), staged by LDS-DMA
// (global_load_lds_dwordx4) into a ring of G_NB 16-deep K-tiles, three K-tiles in flight across each barrier: the
// wait that retires tile kt is a counted `s_waitcnt vmcnt` (4 DMA instructions per wave per K-tile) and the barrier a
// raw s_barrier, so later tiles' DMA stays in flight (cdna_hip_programming.md §5 "Pipelining across barriers"). No
// staging registers, no ds_writes, no A split. Per buffer: 4 planes [Ah][Al][Wh][Wl] of 256 rows x 32 B; a DMA
// wave-instruction fills 32 rows (1 KiB, lane-linear), so the bank swizzle (16-B chunk ^= (row >> 3) & 1, which
// puts every 16-lane group of a fragment read on 16 distinct 16-B slots) is applied to the per-lane SOURCE address
// and undone on the read (§5.4 rule 21). Rows past M / N load row M-1 / N-1 (their products land only in
// accumulator rows / columns the epilogue never stores). Same wave tiling, per-element MFMA order (lo.hi, hi.lo,
// hi.hi per 16 of k, k ascending) and epilogue as k_gemm_bf3_256: bit-identical outputs.
int g_gemm_bf3_dma = 0;  // 1: planes-A 256x256 launches on k_gemm_bf3_256d (FUNASR_BF3_DMA; A/B: batch-32 encode
                         // with planes 109.4 vs 105.8-106.2 ms on register staging, profiles/r05_exp_enc_planes_ab.txt)
constexpr int G_KB = 16, G_NB = 4;
constexpr int G_PLANE = 256 * G_KB;  // bf16 per plane per buffer (8 KiB)
constexpr int G_BUF = 4 * G_PLANE;   // one K-tile: [Ah][Al][Wh][Wl]
constexpr size_t G_LDS = std::max<size_t>((size_t)G_NB * G_BUF * 2, (4096 + 8 * 32 * 33) * 4);  // >= EpiArgmax256

template <class EPI, bool PER = false>
__global__ __launch_bounds__(B3B_T, 1) void k_gemm_bf3_256d(ALoadPlanes al, const __bf16* __restrict__ Wh,
                                                             const __bf16* __restrict__ Wl, int64_t ldw, int M, int N,
                                                             int K, EPI epi) {
  constexpr int WM = 4, WN = 2;
  extern __shared__ float smem[];  // the ring; the epilogue reuses it
  for (int it = 0; it < (PER ? 0x7fffffff : 1); ++it) {
  int tm, tn;
  if (!xcd_tile_it((N + B3B_BN - 1) / B3B_BN, (M + B3B_BM - 1) / B3B_BM, it, PER, tm, tn)) return;
  if (PER && it) __syncthreads();  // the previous tile's epilogue may have used the LDS (no DMA in flight)
  const int m0 = tm * B3B_BM, n0 = tn * B3B_BN;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int wr = wave >> 2, wc = wave & 3;
  const int r = lane & 31, h = lane >> 5;
  __bf16* ring = reinterpret_cast<__bf16*>(smem);
  // DMA: wave w fills plane w >> 1 (0 Ah, 1 Al, 2 Wh, 3 Wl), 32-row chunks c = 4 (w & 1) + i, i < 4; lane s -> row
  // 32 c + (s >> 1), source chunk (s & 1) ^ ((s >> 4) & 1) (= the swizzle of that row)
  const int pl = wave >> 1;
  const int koff = 8 * ((lane & 1) ^ ((lane >> 4) & 1));
  const __bf16* src[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 32 * (4 * (wave & 1) + i) + (lane >> 1);
    if (pl < 2) {
      const int gr = min(m0 + row, M - 1);
      src[i] = reinterpret_cast<const __bf16*>(pl == 0 ? al.hi : al.lo) + (int64_t)gr * al.lda + koff;
    } else {
      const int gr = min(n0 + row, N - 1);
      src[i] = (pl == 2 ? Wh : Wl) + (int64_t)gr * ldw + koff;
    }
  }
  const int ldsw = pl * G_PLANE + 32 * G_KB * 4 * (wave & 1);  // this wave's first chunk in a buffer (elements)
  auto issue = [&](int kt) {
    __bf16* d = ring + (kt % G_NB) * G_BUF + ldsw;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src[i] + kt * G_KB),
                                       (__attribute__((address_space(3))) void*)(d + i * 32 * G_KB), 16, 0, 0);
  };
  f32x16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x16{};
  const int nk = K / G_KB;  // host: K % 16 == 0
  // fragment read offsets (elements): row * 16 + 8 * (h ^ swizzle(row)); rows of a sub-tile differ from r by
  // multiples of 32, so the swizzle bit is (r >> 3) & 1 for all of them
  const int fo = r * G_KB + 8 * (h ^ ((r >> 3) & 1));
  const int fa = (wr * 32 * WM) * G_KB + fo, fb = 2 * G_PLANE + (wc * 32 * WN) * G_KB + fo;
  for (int s = 0; s < G_NB - 1 && s < nk; ++s) issue(s);
  for (int kt = 0; kt < nk; ++kt) {
    // retire this wave's DMA of tile kt (tiles kt + 1, kt + 2 may stay in flight), then the barrier makes every
    // wave's part visible and frees buffer (kt - 1) % G_NB (read in step kt - 1 by all waves) for tile kt + 3
    const int ahead = min(G_NB - 2, nk - 1 - kt);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    if (kt + G_NB - 1 < nk) issue(kt + G_NB - 1);
    const __bf16* b = ring + (kt % G_NB) * G_BUF;
    bf16x8 ah[WM], alo[WM], bh[WN], blo[WN];
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      bh[j] = *reinterpret_cast<const bf16x8*>(b + fb + 32 * j * G_KB);
      blo[j] = *reinterpret_cast<const bf16x8*>(b + fb + G_PLANE + 32 * j * G_KB);
    }
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      ah[i] = *reinterpret_cast<const bf16x8*>(b + fa + 32 * i * G_KB);
      alo[i] = *reinterpret_cast<const bf16x8*>(b + fa + G_PLANE + 32 * i * G_KB);
    }
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) mma_step<3>(acc[i][j], ah[i], alo[i], bh[j], blo[j]);
  }
  __syncthreads();  // every wave's last fragment reads done before an epilogue reuses the LDS (no DMA in flight)
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) epi.apply(acc[i][j], m0 + (wr * WM + i) * 32, n0 + (wc * WN + j) * 32, M, N, smem);
  epi.finish(m0, n0, M, N, smem);
  }
}

template <class EPI>
static void launch_gemm_b3_256d(const ALoadPlanes& al, const WSplit& w, int64_t ldw, int M, int N, int K,
                                const EPI& epi, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    FA_HIP(hipFuncSetAttribute((const void*)k_gemm_bf3_256d<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)G_LDS));
    FA_HIP(hipFuncSetAttribute((const void*)k_gemm_bf3_256d<EPI, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)G_LDS));
    attr = true;
  }
  const dim3 grid = xcd_grid(cdiv(N, B3B_BN), cdiv(M, B3B_BM));
  if (g_gemm_bf3_persist)
    hipLaunchKernelGGL((k_gemm_bf3_256d<EPI, true>), persist_grid(grid), dim3(B3B_T), G_LDS, s, al,
                       reinterpret_cast<const __bf16*>(w.hi), reinterpret_cast<const __bf16*>(w.lo), ldw, M, N, K, epi);
  else
    hipLaunchKernelGGL((k_gemm_bf3_256d<EPI>), grid, dim3(B3B_T), G_LDS, s, al, reinterpret_cast<const __bf16*>(w.hi),
                       reinterpret_cast<const __bf16*>(w.lo), ldw, M, N, K, epi);
}

// ---- few-tile bf16x3 shapes (one clip, M ~ 1000: 32-128 tiles of 128x128): K split over gridDim.z blocks so the
// launch covers the chip with 128x128 tiles instead of 64x64 ones. The 64x64 tile streams 512 B of operand planes per
// k for 64 x 64 outputs and its launch was bound by the per-CU L2 fetch rate (MI355X_MICROARCH.md "Indexed rows":
// 66-73 GB/s per CU; the one-clip ffn2 fetched at ~49 GB/s per CU on half the CUs); the 128x128 tile halves the
// bytes per output. Operands as bf16 planes (A from its producer's APlanes) staged by LDS-DMA into a ring of NB
// 32-deep K-tiles, NB - 2 in flight across each barrier (k_gemm_bf3_256d's pipeline; 4 waves as 2 x 2, each
// 64 x 64 = 2 x 2 accumulators). A DMA wave-instruction fills 16 rows x 64 B (4 lanes per row: a row's 64 B come
// from one line; 16-deep tiles, 32 B per row, measured 4x slower per byte). Split z covers k in [z K / KS,
// (z + 1) K / KS); with KS > 1 every split stores its accumulators (plain stores, accumulator layout) and
// k_gemm_sk_reduce sums them in split order and runs the epilogue: deterministic, no counters, no co-residency (the
// kernel boundary is the hand-off). Per-element MFMA order inside a split: lo.hi, hi.lo, hi.hi per 16 of k, k
// ascending (as every bf16x3 tile), so KS = 1 is bit-identical to the unsplit tiles.
int g_gemm_bf3_sk = 1;  // bf16x3 few-tile K >= 2048 launches split over blocks (k_gemm_bf3_sk / launch_gemm_b3_rs; FUNASR_BF3_SK)
int g_gemm_f16_sk = 1;  // 1: the fp16 graph's few-tile K >= 2048 launches split over blocks (launch_gemm_b3_rs; FUNASR_F16_SK)
int g_gemm_bf3_big = 1024;  // 128x128 register-staged tiles from this many 128x128 tiles (FUNASR_BF3_BIG; batch 6: 64x64 faster)
int g_gemm_f16_pf32 = 1;  // the fp16 graph's batched 128-deep launches on the 32-deep prefetch tile instead (FUNASR_F16_PF32)
int g_gemm_bf3_pf_kb = 0;  // k depth of the 64x64 two-step-prefetch tile: 0 = 32 above G_ROWS_MAX rows, else 64 (FUNASR_BF3_PF_KB)
int g_gemm_bf3_sk_kmin = 2048;  // smallest K split over blocks (FUNASR_BF3_SK_KMIN; A/B)
int g_gemm_bf3_sk_ks = 0;  // microbenchmark hook: force the K split (1, 2, 4, 8)
constexpr int SK_KB = 32;
constexpr int SK_PLANE = 128 * SK_KB;  // bf16 per plane per buffer (8 KiB = 8 DMA wave-instructions)
constexpr int SK_BUF = 4 * SK_PLANE;   // one K-tile: [Ah][Al][Wh][Wl] (32 KiB)
constexpr int SK_KS_MAX = 8;
constexpr int64_t SK_UNIT = 4 * 4 * 16 * 64;  // floats per (tile, split): 4 waves x 4 accumulators x 16 x 64 lanes

__device__ __forceinline__ void sk_wait(int ahead) {  // retire all but `ahead` K-tiles of this wave's DMA (8 each)
  if (ahead >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (ahead == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <class EPI, bool SPLIT>
__global__ __launch_bounds__(256) void k_gemm_bf3_sk(ALoadPlanes al, const __bf16* __restrict__ Wh,
                                                     const __bf16* __restrict__ Wl, int64_t ldw, int M, int N, int K,
                                                     EPI epi, float* __restrict__ part) {
  constexpr int WM = 2, WN = 2, NB = 4;  // 4 x 32 KiB ring, two K-tiles in flight (sk_wait)
  extern __shared__ float smem[];  // the ring; the epilogue reuses it
  const int nbx = (N + 127) / 128, nby = (M + 127) / 128;
  int tm, tn;
  if (!xcd_tile(nbx, nby, tm, tn)) return;
  const int m0 = tm * 128, n0 = tn * 128;
  const int kper = SPLIT ? K / (int)gridDim.z : K;  // host: K % (KS * 32) == 0
  const int kb0 = SPLIT ? (int)blockIdx.z * kper : 0;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const int r = lane & 31, h = lane >> 5;
  __bf16* ring = reinterpret_cast<__bf16*>(smem);
  // DMA: wave w fills plane w (0 Ah, 1 Al, 2 Wh, 3 Wl) in 8 wave-instructions of 16 rows; lane s -> row
  // 16 i + (s >> 2), LDS chunk s & 3 holding source chunk (s & 3) ^ ((s >> 4) & 3) (the bank swizzle of that row,
  // undone on the read: the 16 rows a 16-lane fragment read touches then hit 16 distinct 16-B slots)
  const int koff = 8 * ((lane & 3) ^ ((lane >> 4) & 3));
  const __bf16* base;
  int64_t ld;
  if (wave < 2) {
    base = reinterpret_cast<const __bf16*>(wave == 0 ? al.hi : al.lo);
    ld = al.lda;
  } else {
    base = wave == 2 ? Wh : Wl;
    ld = ldw;
  }
  const int lim = (wave < 2 ? M : N) - 1, r0 = wave < 2 ? m0 : n0;
  const __bf16* src[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)  // rows past M / N: clamped (their products reach no stored output)
    src[i] = base + (int64_t)min(r0 + 16 * i + (lane >> 2), lim) * ld + kb0 + koff;
  auto issue = [&](int kt) {
    __bf16* d = ring + (kt % NB) * SK_BUF + wave * SK_PLANE;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src[i] + kt * SK_KB),
                                       (__attribute__((address_space(3))) void*)(d + i * 16 * SK_KB), 16, 0, 0);
  };
  f32x16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x16{};
  const int nk = kper / SK_KB;
  const int sw = (r >> 2) & 3;  // fragment rows differ from r by multiples of 32: one swizzle for all of them
  const int fa = (wr * 64 + r) * SK_KB, fb = 2 * SK_PLANE + (wc * 64 + r) * SK_KB;
  for (int s = 0; s < NB - 1 && s < nk; ++s) issue(s);
  for (int kt = 0; kt < nk; ++kt) {
    // retire tile kt (tiles kt + 1, kt + 2 stay in flight); the barrier then frees buffer (kt - 1) % NB
    sk_wait(min(NB - 2, nk - 1 - kt));
    asm volatile("s_barrier" ::: "memory");
    if (kt + NB - 1 < nk) issue(kt + NB - 1);
    const __bf16* b = ring + (kt % NB) * SK_BUF;
#pragma unroll
    for (int kk = 0; kk < SK_KB / 16; ++kk) {
      const int c = 8 * ((2 * kk + h) ^ sw);
      bf16x8 ah[WM], alo[WM], bh[WN], blo[WN];
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        bh[j] = *reinterpret_cast<const bf16x8*>(b + fb + 32 * j * SK_KB + c);
        blo[j] = *reinterpret_cast<const bf16x8*>(b + fb + SK_PLANE + 32 * j * SK_KB + c);
      }
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        ah[i] = *reinterpret_cast<const bf16x8*>(b + fa + 32 * i * SK_KB + c);
        alo[i] = *reinterpret_cast<const bf16x8*>(b + fa + SK_PLANE + 32 * i * SK_KB + c);
      }
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j) mma_step<3>(acc[i][j], ah[i], alo[i], bh[j], blo[j]);
    }
  }
  if constexpr (SPLIT) {
    sk_store_partial<WM, WN>(acc, part, tm * nbx + tn, nbx * nby, wave, lane);
  } else {
    __syncthreads();  // every wave's last fragment reads done before an epilogue reuses the LDS (no DMA in flight)
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) epi.apply(acc[i][j], m0 + (wr * WM + i) * 32, n0 + (wc * WN + j) * 32, M, N, smem);
    epi.finish(m0, n0, M, N, smem);
  }
}

// one wave per quarter (4 registers) of a (tile, wave, i, j) accumulator of the split tiles: the KS split partials
// summed in split order, then EpiLinear's arithmetic on the rows / column the unsplit kernel gives those registers
template <class EPI>
__global__ __launch_bounds__(256) void k_gemm_sk_reduce(const float* __restrict__ part, int KS, int nbx, int ntiles,
                                                        int M, int N, EPI epi) {
  // block b -> a unit of a tile the split launch ran on XCD b % 8 (xcd_tile's order): its partials are in that L2
  const int per = (ntiles + 7) >> 3, b = blockIdx.x, u = (b & 7) * per * 16 + (b >> 3);
  if ((b >> 3) >= per * 16 || u >= ntiles * 16) return;
  const int q = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tile = u >> 4, wave = (u >> 2) & 3, ij = u & 3;
  const f32x4_t* src = reinterpret_cast<const f32x4_t*>(part) + ((int64_t)u * 4 + q) * 64 + lane;
  const int64_t zs = (int64_t)ntiles * SK_UNIT / 4;  // float4 per split
  f32x4_t p[SK_KS_MAX];
#pragma unroll
  for (int z = 0; z < SK_KS_MAX; ++z) p[z] = src[min(z, KS - 1) * zs];  // clamped duplicates past KS: not summed
  f32x4_t v = p[0];
#pragma unroll
  for (int z = 1; z < SK_KS_MAX; ++z)
    if (z < KS) v += p[z];
  const int tm = tile / nbx, tn = tile - tm * nbx;
  const int col0 = tn * 128 + (wave & 1) * 64 + (ij & 1) * 32;
  epi.apply4(v, q, tm * 128 + (wave >> 1) * 64 + (ij >> 1) * 32, col0, M, N, epi.bias_of(col0 + (lane & 31), N));
}

// K split of a few-tile launch: the largest power of two <= SK_KS_MAX with tiles x KS <= 256 (one block per CU) and
// >= 64 of k per split; 0 = not this kernel (workspace too small, K not divisible, or enough tiles already)
static int sk_splits(int64_t tiles, int K, const GemmF32Work* wk) {
  int ks = g_gemm_bf3_sk_ks;
  if (!ks) {
    ks = 1;
    while (ks < SK_KS_MAX && tiles * ks * 2 <= 256 && K % (ks * 2 * SK_KB) == 0 && K / (ks * 2) >= 64) ks *= 2;
  }
  if (K % (ks * SK_KB)) return 0;
  if (ks > 1 && (!wk || !wk->part || tiles * ks * SK_UNIT > wk->part_n)) return 0;
  return ks;
}

template <class EPI>
static bool launch_gemm_b3_sk(const ALoadPlanes& al, const WSplit& w, int64_t ldw, int M, int N, int K, const EPI& epi,
                              hipStream_t s, const GemmF32Work* wk) {
  constexpr size_t lds = (size_t)4 * SK_BUF * 2;
  const int nbx = cdiv(N, 128), nby = cdiv(M, 128);
  const int ks = sk_splits((int64_t)nbx * nby, K, wk);
  if (ks == 0) return false;
  static bool attr = false;
  if (!attr) {
    FA_HIP(hipFuncSetAttribute((const void*)k_gemm_bf3_sk<EPI, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds));
    FA_HIP(hipFuncSetAttribute((const void*)k_gemm_bf3_sk<EPI, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds));
    attr = true;
  }
  const auto* wh = reinterpret_cast<const __bf16*>(w.hi);
  const auto* wl = reinterpret_cast<const __bf16*>(w.lo);
  if (ks == 1) {
    hipLaunchKernelGGL((k_gemm_bf3_sk<EPI, false>), xcd_grid(nbx, nby), dim3(256), lds, s, al, wh, wl, ldw, M, N, K,
                       epi, nullptr);
    return true;
  }
  FA_REQUIRE(wk && wk->part && (int64_t)nbx * nby * ks * SK_UNIT <= wk->part_n, "gemm_bf3_sk: split workspace");
  hipLaunchKernelGGL((k_gemm_bf3_sk<EPI, true>), xcd_grid(nbx, nby, ks), dim3(256), lds, s, al, wh, wl, ldw, M, N, K,
                     epi, wk->part);
  hipLaunchKernelGGL(k_gemm_sk_reduce<EPI>, dim3(((nbx * nby + 7) >> 3) * 8 * 16), dim3(256), 0, s, wk->part, ks, nbx,
                     nbx * nby, M, N, epi);
  return true;
}

// the same split over the register-staged 128x128x32 tile (k_gemm_bf3 <2, 2, 32>, write-after-barrier staging): any A
// operand (planes or f32) and both precisions (P = 1: the fp16 graph)
template <class AL, class EPI, int P>
static bool launch_gemm_b3_rs(const AL& al, const WSplit& w, int64_t ldw, int M, int N, int K, const EPI& epi,
                              hipStream_t s, const GemmF32Work* wk) {
  const int nbx = cdiv(N, 128), nby = cdiv(M, 128);
  const int ks = sk_splits((int64_t)nbx * nby, K, wk);
  if (ks == 0) return false;
  if (ks == 1) {  // no split: the unsplit tile and its epilogue (sk_splits sized no workspace for it)
    launch_gemm_b3<AL, EPI, 2, 2, 32, 1, 3, P>(al, w, ldw, M, N, K, epi, s);
    return true;
  }
  using T = TileB3<2, 2, 32, P>;
  typedef typename PrecB<P>::E E;
  const size_t lds = (size_t)2 * T::STAGE * 2;
  static bool attr = false;
  if (!attr && lds > 65536) {
    (void)hipFuncSetAttribute((const void*)k_gemm_bf3<AL, EPI, 2, 2, 32, 1, 3, P, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  FA_REQUIRE(wk && wk->part && (int64_t)nbx * nby * ks * SK_UNIT <= wk->part_n, "gemm_bf3 split: workspace");
  hipLaunchKernelGGL((k_gemm_bf3<AL, EPI, 2, 2, 32, 1, 3, P, true>), xcd_grid(nbx, nby, ks), dim3(256), lds, s, al,
                     reinterpret_cast<const E*>(w.hi), reinterpret_cast<const E*>(w.lo), ldw, M, N, K, epi, wk->part);
  hipLaunchKernelGGL(k_gemm_sk_reduce<EPI>, dim3(((nbx * nby + 7) >> 3) * 8 * 16), dim3(256), 0, s, wk->part, ks, nbx,
                     nbx * nby, M, N, epi);
  return true;
}

template <class AL, class EPI, int P = 3>
static void launch_gemm_b3_256(const AL& al, const WSplit& w, int64_t ldw, int M, int N, int K, const EPI& epi,
                               hipStream_t s) {
  FA_REQUIRE(K % 8 == 0 && ldw % 8 == 0, "gemm_bf3_256: K and ldw must be multiples of 8");
  if constexpr (IsPlanes<AL>::value && P == 3) {
    if (g_gemm_bf3_dma && K % G_KB == 0 && M > 0 && N > 0) {
      launch_gemm_b3_256d<EPI>(al, w, ldw, M, N, K, epi, s);
      return;
    }
  }
  if (g_gemm_bf3_256_s) launch_gemm_b3_256_s<AL, EPI, P, 1>(al, w, ldw, M, N, K, epi, s);
  else launch_gemm_b3_256_s<AL, EPI, P, 0>(al, w, ldw, M, N, K, epi, s);
}

// microbenchmark helper: resident blocks per CU of the 128x128x32 bf16x3 kernel (linear epilogue), its dynamic LDS
int gemm_bf3_occupancy_128() {
  using T = TileB3<2, 2, 32>;
  const size_t lds = 2 * T::STAGE * 2;
  (void)hipFuncSetAttribute((const void*)k_gemm_bf3<ALoadPlain, EpiLinear, 2, 2, 32, 1>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int n = -1;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gemm_bf3<ALoadPlain, EpiLinear, 2, 2, 32, 1>, 256, lds);
  return n;
}

// P = 3: bf16x3 planes (w.hi, w.lo); P = 1: the fp16 graph (w.hi = the fp16 weight copy)
template <class AL, class EPI, int P = 3>
static void run_gemm_b3(const AL& al, const WSplit& w, int64_t ldw, int M, int N, int K, const EPI& epi, hipStream_t s,
                        const GemmF32Work* wk = nullptr) {
  const int f = g_gemm_bf3_force;
  // few-tile linear launches with K >= 2048 (one clip's ffn2): 128x128 tiles, the K split over blocks. Planes-A
  // bf16x3 on the LDS-DMA tile (k_gemm_bf3_sk), f32-A bf16x3 and the fp16 graph on the register-staged one
  // (launch_gemm_b3_rs): both tiles run the same per-element MFMA order and split, so bf16x3 stays bit-identical
  // between planes and f32 rows
  if constexpr (std::is_base_of<EpiLinear, EPI>::value) {
    const bool few = f == 0 && (int64_t)cdiv(M, 128) * cdiv(N, 128) <= 128 && K >= g_gemm_bf3_sk_kmin;
    if (M > 0 && N > 0) {
      if constexpr (IsPlanes<AL>::value && P == 3)
        if ((f == 11 || (few && g_gemm_bf3_sk)) && launch_gemm_b3_sk(al, w, ldw, M, N, K, epi, s, wk)) return;
      const bool rs = few && (P == 1 ? g_gemm_f16_sk != 0 : (g_gemm_bf3_sk != 0 && !IsPlanes<AL>::value));
      if ((f == 12 || rs) && launch_gemm_b3_rs<AL, EPI, P>(al, w, ldw, M, N, K, epi, s, wk)) return;
    }
  }
  const bool big = f ? f == 2 : (int64_t)cdiv(M, 128) * cdiv(N, 128) >= g_gemm_bf3_big;
  const int64_t t64 = (int64_t)cdiv(M, 64) * cdiv(N, 64);
  const bool pf = g_gemm_bf3_pf > 1;
  // 256x256 tiles while they still give most CUs a block (f == 6 forces them)
  if (f == 6 || (f == 0 && g_gemm_bf3_256 && (int64_t)cdiv(M, 256) * cdiv(N, 256) >= g_gemm_bf3_256))
    launch_gemm_b3_256<AL, EPI, P>(al, w, ldw, M, N, K, epi, s);
  else if (big) {
    if (g_gemm_bf3_256_s) launch_gemm_b3<AL, EPI, 2, 2, 32, 1, 3, P>(al, w, ldw, M, N, K, epi, s);
    else launch_gemm_b3<AL, EPI, 2, 2, 32, 1, 1, P>(al, w, ldw, M, N, K, epi, s);
  }
  // fp16 graph, one clip: 128-deep stages (half the k-steps; fp16 planes leave the LDS for them). q|k|v and ffn1 keep
  // their per-element MFMA order (bit-identical to 64-deep stages); ffn2 also splits K in halves. scripts/ubench/
  // gemm_f32_bench kscan, graph-timed: q|k|v 10.1 -> 9.8, ffn1 10.9 -> 10.3, ffn2 14.7 -> 13.8 us (bf16x3: slower)
  else if (P == 1 && f == 0 && g_gemm_f16_deep && t64 > 256 && t64 <= 1024 && K % 128 == 0 &&
           !(g_gemm_f16_pf32 && M > G_ROWS_MAX))
    launch_gemm_b3<AL, EPI, 1, 1, 128, 1, 2, P>(al, w, ldw, M, N, K, epi, s);
  else if (P == 1 && f == 0 && g_gemm_f16_deep && t64 < 256 && K >= 2048 && K % 256 == 0)
    launch_gemm_b3<AL, EPI, 1, 1, 128, P == 1 ? 2 : 1, 2, P>(al, w, ldw, M, N, K, epi, s);
  else if (f == 1) launch_gemm_b3<AL, EPI, 1, 1, 32, 1, 1, P>(al, w, ldw, M, N, K, epi, s);
  // 256 < 64x64 tiles <= 1024 (one clip's q|k|v and ffn1: 384 / 512 tiles, i.e. 1.5-2 rounds of one 147-KiB block per
  // CU): 128x64 tiles, two K groups of 32-deep stages, loads two steps ahead -- one round of twice the work per block
  else if (f == 7 || (f == 0 && g_gemm_bf3_mid && t64 > 256 && t64 <= 1024 && K % 64 == 0))
    launch_gemm_b3<AL, EPI, 2, 1, 32, 2, 2, P>(al, w, ldw, M, N, K, epi, s);
  else if (f == 9) launch_gemm_b3<AL, EPI, 1, 1, 128, 1, 2, P>(al, w, ldw, M, N, K, epi, s);
  else if (f == 10) {  // 128-deep stages in two K groups (fp16: 2 x 2 x 34 KiB of LDS; bf16x3 has no room for it)
    if constexpr (P == 1) launch_gemm_b3<AL, EPI, 1, 1, 128, 2, 2, P>(al, w, ldw, M, N, K, epi, s);
    else launch_gemm_b3<AL, EPI, 1, 1, 128, 1, 2, P>(al, w, ldw, M, N, K, epi, s);
  } else if (f == 8 || (f == 0 && g_gemm_bf3_kw4 && t64 < 256 && K >= 2048 && K % 256 == 0)) {
    // 1024 threads: 16 waves per CU; P = 3 keeps 32-deep stages (4 groups x 2 stages x 20 KiB = 160 KiB)
    if constexpr (P == 1) launch_gemm_b3<AL, EPI, 1, 1, 64, 4, 2, P>(al, w, ldw, M, N, K, epi, s);
    else launch_gemm_b3<AL, EPI, 1, 1, 32, 4, 2, P>(al, w, ldw, M, N, K, epi, s);
  } else if (f == 4 || (f == 0 && t64 < 256 && K % 128 == 0)) {
    if (pf) launch_gemm_b3<AL, EPI, 1, 1, 64, 2, 2, P>(al, w, ldw, M, N, K, epi, s);
    else launch_gemm_b3<AL, EPI, 1, 1, 64, 2, 1, P>(al, w, ldw, M, N, K, epi, s);
  } else if (f == 5) launch_gemm_b3<AL, EPI, 1, 1, 32, 2, 1, P>(al, w, ldw, M, N, K, epi, s);
  // 32-deep k-steps for batched launches (batch 6 encode 27.8 -> 25.5 ms), 64 for one clip (8.2 vs 8.3 ms)
  else if (pf && (g_gemm_bf3_pf_kb == 32 || (g_gemm_bf3_pf_kb == 0 && M > G_ROWS_MAX)))
    launch_gemm_b3<AL, EPI, 1, 1, 32, 1, 2, P>(al, w, ldw, M, N, K, epi, s);
  else if (pf) launch_gemm_b3<AL, EPI, 1, 1, 64, 1, 2, P>(al, w, ldw, M, N, K, epi, s);
  else launch_gemm_b3<AL, EPI, 1, 1, 64, 1, 1, P>(al, w, ldw, M, N, K, epi, s);
}

__global__ void k_split_bf16(const float* __restrict__ w, __bf16* __restrict__ hi, __bf16* __restrict__ lo, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = w[i];
    const __bf16 h = (__bf16)v;
    hi[i] = h;
    lo[i] = (__bf16)(v - (float)h);
  }
}

void launch_split_bf16(const float* w, uint16_t* hi, uint16_t* lo, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  const int blocks = (int)std::min<int64_t>(cdiv(n, 256), 4096);
  hipLaunchKernelGGL(k_split_bf16, dim3(blocks), dim3(256), 0, s, w, reinterpret_cast<__bf16*>(hi),
                     reinterpret_cast<__bf16*>(lo), n);
}

void gemm_linear(const float* A, int64_t lda, const float* W, int64_t ldw, const float* bias, float* C, int64_t ldc,
                 int M, int N, int K, int relu, const float* add1, int64_t ld1, const float* add2, int64_t ld2,
                 hipStream_t s, const __half* W16, const GemmF32Work* wk, WSplit wb, APlanes ap, APlanes cp) {
  ALoadPlain al{A, lda};
  EpiLinear epi{C, ldc, bias, add1, ld1, add2, ld2, relu, W16 ? 1 : 0};
  if (ap.hi || cp.hi) FA_REQUIRE(wb.hi && !W16, "gemm_linear: bf16 activation planes need the bf16x3 mode");
  if (cp.hi) {
    FA_REQUIRE(N % 2 == 0 && ldc % 2 == 0, "gemm_linear: C planes need even N and ldc");
    epi.ph = reinterpret_cast<__bf16*>(cp.hi);
    epi.pl = reinterpret_cast<__bf16*>(cp.lo);
  }
  // one-clip launches (M <= G_ROWS_MAX) take the four-row grouped epilogue (EpiLinearG), batched ones the row-by-row
  // one: the same arithmetic either way
  EpiLinearG epg;
  static_cast<EpiLinear&>(epg) = epi;
  const bool grp = M <= G_ROWS_MAX && g_gemm_epi_grouped;
  if (ap.hi) {
    FA_REQUIRE(lda % 8 == 0 && K % 8 == 0, "gemm_linear: A planes need lda % 8 == 0 and K % 8 == 0");
    const ALoadPlanes alp{ap.hi, ap.lo, lda};
    if (grp) run_gemm_b3(alp, wb, ldw, M, N, K, epg, s, wk);
    else run_gemm_b3(alp, wb, ldw, M, N, K, epi, s, wk);
    return;
  }
  if (W16 && g_gemm_f16_b3) {
    const WSplit w16{reinterpret_cast<const uint16_t*>(W16)};
    if (grp) run_gemm_b3<ALoadPlain, EpiLinearG, 1>(al, w16, ldw, M, N, K, epg, s, wk);
    else run_gemm_b3<ALoadPlain, EpiLinear, 1>(al, w16, ldw, M, N, K, epi, s, wk);
  } else if (W16) {
    run_gemm16(al, W16, ldw, M, N, K, epi, s);
  } else if (wb.hi) {
    if (grp) run_gemm_b3(al, wb, ldw, M, N, K, epg, s, wk);
    else run_gemm_b3(al, wb, ldw, M, N, K, epi, s, wk);
  } else {
    run_gemm(al, W, ldw, M, N, K, epi, s, true, wk);
  }
}

void gemm_stft_power(const float* xp, int64_t xp_stride, int t_stride, int M, const float* basis, float* power,
                     int64_t ldp, hipStream_t s, int r16) {
  ALoadFrames al{xp, xp_stride, t_stride, 160};
  EpiPower epi{power, ldp, r16};
  run_gemm(al, basis, 400, M, 402, 400, epi, s);
}

void gemm_mel_log(const float* power, int64_t ldp, const float* fbank, int64_t ldf, float* mel, int M, int n_mels,
                  int n_freq, hipStream_t s, int r16) {
  ALoadPlain al{power, ldp};
  EpiLog epi{mel, n_mels, r16};
  run_gemm(al, fbank, ldf, M, n_mels, n_freq, epi, s);
}

__global__ void k_argmax_final(const float* __restrict__ pval, const int* __restrict__ pidx, int M, int n_tiles,
                               int* __restrict__ out) {
  int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  if (row >= M) return;
  float v = -INFINITY;
  int i = 0x7fffffff;
  for (int t = lane; t < n_tiles; t += 64) argmax_combine(v, i, pval[(int64_t)row * n_tiles + t], pidx[(int64_t)row * n_tiles + t]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    float v2 = __shfl_xor(v, o, 64);
    int i2 = __shfl_xor(i, o, 64);
    argmax_combine(v, i, v2, i2);
  }
  if (lane == 0) out[row] = i;
}

// ---------------------------------------------------------------------------------------------
// int8-dynamic CTC graph (the reference's default Fun-ASR-Nano-CTC.int8.onnx: 02-Quantize-ONNX.py:38-46, onnxruntime
// quantize_dynamic over every MatMul with a constant weight, per-channel QUInt8 weights, reduce_range off). At run time
// each such MatMul is DynamicQuantizeLinear(x) -> MatMulInteger -> Cast -> Mul(x_scale * w_scale) (ONNX operator
// semantics; the attention's activation x activation MatMuls stay f32):
//   x_min = min(0, min x), x_max = max(0, max x) over the whole [1, T, K] input tensor (one clip's unpadded rows),
//   xs = (x_max - x_min) / 255, xzp = round_half_even(clamp(-x_min / xs, 0, 255)), xq = sat(round_half_even(x / xs) + xzp)
//   y[i][j] = f32(sum_k (xq[i][k] - xzp) (wq[j][k] - wzp[j])) * f32(xs * ws[j]) (+ bias, the Add that follows)
// The integer dot runs on v_mfma_i32_32x32x32_i8 with both operands shifted into int8 (x' = xq - 128, w' = wq - 128):
//   sum (xq - xzp)(wq - wzp) = S' + bz_j rs_i + a cs_j + K a bz_j,  S' = sum x' w', rs_i = sum_k x'[i][k],
//   cs_j = sum_k w'[j][k], a = 128 - xzp, bz_j = 128 - wzp[j]   (exact in int32 for K <= 2^15)
// -> the same integers as MatMulInteger, then the f32 rescale, bias and the existing epilogues (ReLU / residual /
// fused CTC row-argmax).
typedef int i32x4_u __attribute__((ext_vector_type(4)));
typedef int i32x16_u __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float rne_f(float v) { return __builtin_rintf(v); }  // round half to even

// weight prep: ORT uint8 [N][K] + scale / zero point per output channel -> w' = wq - 128 (int8), cs_j, bz_j
__global__ void k_u8w_prep(const uint8_t* __restrict__ q, const float* __restrict__ sc, const uint8_t* __restrict__ zp,
                           int N, int K, int8_t* __restrict__ wq, int* __restrict__ cs, int* __restrict__ bz,
                           float* __restrict__ ws) {
  const int j = blockIdx.x, lane = threadIdx.x;
  if (j >= N) return;
  int sum = 0;
  for (int k = lane; k < K; k += 64) {
    const int v = (int)q[(int64_t)j * K + k] - 128;
    wq[(int64_t)j * K + k] = (int8_t)v;
    sum += v;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
  if (lane == 0) {
    cs[j] = sum;
    bz[j] = 128 - (int)zp[j];
    ws[j] = sc[j];
  }
}

void u8_weight_prep(const uint8_t* q, const float* scale, const uint8_t* zp, int N, int K, int8_t* wq, int* cs, int* bz,
                    float* ws, hipStream_t s) {
  hipLaunchKernelGGL(k_u8w_prep, dim3(N), dim3(64), 0, s, q, scale, zp, N, K, wq, cs, bz, ws);
}

// per-clip min / max partials of x over the clip's valid rows [0, lens[b]) (row base b * ts): grid (DQ_NB, B)
constexpr int DQ_NB = 64;
__global__ __launch_bounds__(256) void k_dq_minmax(const float* __restrict__ x, int64_t ldx, int K,
                                                   const int* __restrict__ lens, int ts, float2* __restrict__ part) {
  const int b = blockIdx.y, len = lens ? lens[b] : ts;
  const int64_t n = (int64_t)len * K;
  float mn = INFINITY, mx = -INFINITY;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)DQ_NB * 256) {
    const int64_t r = i / K, c = i - r * K;
    const float v = x[((int64_t)b * ts + r) * ldx + c];
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  __shared__ float smn[4], smx[4];
  mn = -wave_max(-mn);
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) {
    smn[threadIdx.x >> 6] = mn;
    smx[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    part[b * DQ_NB + blockIdx.x] = make_float2(fminf(fminf(smn[0], smn[1]), fminf(smn[2], smn[3])),
                                               fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3])));
}

// DynamicQuantizeLinear of the clip's rows: one wave per row (grid (cdiv(ts, 4), B)); rows past lens[b] -> zeros.
// xq [rows][K] int8 (xq - 128), rs [rows] = row sums of the int8 values, qp[b] = {xs, a = 128 - xzp}
__global__ __launch_bounds__(256) void k_dq_quant(const float* __restrict__ x, int64_t ldx, int K,
                                                  const int* __restrict__ lens, int ts, const float2* __restrict__ part,
                                                  int8_t* __restrict__ xq, int* __restrict__ rs, float2* __restrict__ qp) {
  const int b = blockIdx.y, len = lens ? lens[b] : ts;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + wave;
  float mn = part[b * DQ_NB + lane].x, mx = part[b * DQ_NB + lane].y;  // DQ_NB == 64: one partial per lane
  mn = -wave_max(-mn);
  mx = wave_max(mx);
  mn = fminf(mn, 0.f);
  mx = fmaxf(mx, 0.f);
  const float xs = mx == mn ? 1.0f : (mx - mn) / 255.0f;
  const float zpf = rne_f(fminf(fmaxf(0.0f - mn / xs, 0.0f), 255.0f));
  if (blockIdx.x == 0 && threadIdx.x == 0) qp[b] = make_float2(xs, 128.0f - zpf);
  if (r >= ts) return;
  const int64_t row = (int64_t)b * ts + r;
  int sum = 0;
  for (int k = 4 * lane; k < K; k += 256) {
    char4 o = make_char4(0, 0, 0, 0);
    if (r < len) {
      const float4 v = *reinterpret_cast<const float4*>(x + row * ldx + k);
      const int q0 = (int)fminf(fmaxf(rne_f(v.x / xs) + zpf, 0.f), 255.f) - 128;
      const int q1 = (int)fminf(fmaxf(rne_f(v.y / xs) + zpf, 0.f), 255.f) - 128;
      const int q2 = (int)fminf(fmaxf(rne_f(v.z / xs) + zpf, 0.f), 255.f) - 128;
      const int q3 = (int)fminf(fmaxf(rne_f(v.w / xs) + zpf, 0.f), 255.f) - 128;
      o = make_char4((char)q0, (char)q1, (char)q2, (char)q3);
      sum += q0 + q1 + q2 + q3;
    }
    *reinterpret_cast<char4*>(xq + row * K + k) = o;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
  if (lane == 0) rs[row] = sum;
}

// integer GEMM tile: 64 WM x 64 WN x 64 (k), 2x2 waves each WM x WN accumulators of 32x32 (v_mfma_i32_32x32x32_i8:
// lane (r, h) holds row r, k 16 h .. 16 h + 15 of A and of B; accumulator reg -> row (reg & 3) + 8 (reg >> 2) + 4 h,
// col r: the f32 kernels' layout, so their epilogues apply). LDS rows of 64 + 16 B: the 16 rows a 16-lane group
// reads start in distinct 4-bank groups. xcd_tile order, no K splits.
constexpr int U8_LD = 80;
template <int WM, int WN>
struct TileU8 {
  static constexpr int BM = 64 * WM, BN = 64 * WN;
  static constexpr int NA = BM * 4 / 256, NB = BN * 4 / 256;  // 16-B chunks per thread
  static constexpr int STAGE = (BM + BN) * U8_LD;              // bytes
};
struct U8Args {
  const int8_t* xq;
  const int* rs;
  const float2* qp;
  const int8_t* wq;
  const int* cs;
  const int* bz;
  const float* ws;
  int ts;  // rows per clip (row -> clip = row / ts)
};

template <class EPI, int WM, int WN>
__global__ __launch_bounds__(256) void k_gemm_u8(U8Args u, int M, int N, int K, EPI epi) {
  using T = TileU8<WM, WN>;
  extern __shared__ float smem[];
  uint8_t* sm = reinterpret_cast<uint8_t*>(smem);
  int tm, tn;
  if (!xcd_tile((N + T::BN - 1) / T::BN, (M + T::BM - 1) / T::BM, tm, tn)) return;
  const int m0 = tm * T::BM, n0 = tn * T::BN;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const int r = lane & 31, h = lane >> 5;
  i32x16_u acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = i32x16_u{};
  i32x4_u ra[T::NA], rb[T::NB];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < T::NA; ++i) {
      const int idx = t + 256 * i, row = idx >> 2, c = idx & 3;
      ra[i] = *reinterpret_cast<const i32x4_u*>(u.xq + (int64_t)min(m0 + row, M - 1) * K + k0 + 16 * c);
    }
#pragma unroll
    for (int i = 0; i < T::NB; ++i) {
      const int idx = t + 256 * i, row = idx >> 2, c = idx & 3;
      rb[i] = *reinterpret_cast<const i32x4_u*>(u.wq + (int64_t)min(n0 + row, N - 1) * K + k0 + 16 * c);
    }
  };
  auto store = [&](uint8_t* st) {
#pragma unroll
    for (int i = 0; i < T::NA; ++i) {
      const int idx = t + 256 * i;
      *reinterpret_cast<i32x4_u*>(st + (idx >> 2) * U8_LD + 16 * (idx & 3)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < T::NB; ++i) {
      const int idx = t + 256 * i;
      *reinterpret_cast<i32x4_u*>(st + (T::BM + (idx >> 2)) * U8_LD + 16 * (idx & 3)) = rb[i];
    }
  };
  const int nk = K / 64;  // host: K % 64 == 0
  load(0);
  store(sm);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load((kt + 1) * 64);
    const uint8_t* st = sm + cur * T::STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      i32x4_u av[WM], bv[WN];
#pragma unroll
      for (int i = 0; i < WM; ++i)
        av[i] = *reinterpret_cast<const i32x4_u*>(st + (wr * 32 * WM + 32 * i + r) * U8_LD + 32 * kk + 16 * h);
#pragma unroll
      for (int j = 0; j < WN; ++j)
        bv[j] = *reinterpret_cast<const i32x4_u*>(st + (T::BM + wc * 32 * WN + 32 * j + r) * U8_LD + 32 * kk + 16 * h);
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store(sm + (cur ^ 1) * T::STAGE);
    __syncthreads();
  }
  // MatMulInteger's integers -> f32 rescale (Cast, Mul by f32(xs * ws_j)), then the epilogue (bias, ReLU, residual,
  // argmax) on the f32 accumulator layout
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int row0 = m0 + (wr * WM + i) * 32, col0 = n0 + (wc * WN + j) * 32;
      const int col = min(col0 + r, N - 1);
      const int cs = u.cs[col], bzj = u.bz[col];
      const float wsj = u.ws[col];
      f32x16 y;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = min(row0 + (q & 3) + 8 * (q >> 2) + 4 * h, M - 1);
        const float2 p = u.qp[row / u.ts];
        const int a = (int)p.y;
        const int tot = acc[i][j][q] + bzj * u.rs[row] + a * cs + K * a * bzj;
        y[q] = __fmul_rn((float)tot, __fmul_rn(p.x, wsj));
      }
      epi.apply(y, row0, col0, M, N, smem);
    }
  epi.finish(m0, n0, M, N, smem);
}

template <class EPI, int WM, int WN>
static void launch_gemm_u8(const U8Args& u, int M, int N, int K, const EPI& epi, hipStream_t s) {
  using T = TileU8<WM, WN>;
  FA_REQUIRE(K % 64 == 0, "gemm_u8: K must be a multiple of 64");
  const size_t lds = std::max<size_t>({(size_t)2 * T::STAGE, (size_t)(1024 + 4 * 32 * 33) * 4});
  static bool attr = false;
  if (!attr && lds > 65536) {
    (void)hipFuncSetAttribute((const void*)k_gemm_u8<EPI, WM, WN>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((k_gemm_u8<EPI, WM, WN>), xcd_grid(cdiv(N, T::BN), cdiv(M, T::BM)), dim3(256), lds, s, u, M, N, K,
                     epi);
}

// DynamicQuantizeLinear of x (B clips of ts rows, lens[b] valid) into the workspace
void dq_quantize(const float* x, int64_t ldx, int K, const int* lens, int ts, int B, U8Work& w, hipStream_t s) {
  FA_REQUIRE(K % 4 == 0 && (int64_t)B * ts * K <= w.xq_n && B <= w.max_clips, "dq_quantize: workspace");
  hipLaunchKernelGGL(k_dq_minmax, dim3(DQ_NB, B), dim3(256), 0, s, x, ldx, K, lens, ts, w.part);
  hipLaunchKernelGGL(k_dq_quant, dim3(cdiv(ts, 4), B), dim3(256), 0, s, x, ldx, K, lens, ts, w.part, w.xq, w.rs, w.qp);
}

void gemm_u8_linear(const U8Work& w, const U8W& wt, const float* bias, float* C, int64_t ldc, int M, int N, int K,
                    int ts, int relu, const float* add1, int64_t ld1, hipStream_t s) {
  const U8Args u{w.xq, w.rs, w.qp, wt.q, wt.cs, wt.bz, wt.ws, ts};
  EpiLinear epi{C, ldc, bias, add1, ld1, nullptr, 0, relu, 0};
  if ((int64_t)cdiv(M, 128) * cdiv(N, 128) >= 256) launch_gemm_u8<EpiLinear, 2, 2>(u, M, N, K, epi, s);
  else launch_gemm_u8<EpiLinear, 1, 1>(u, M, N, K, epi, s);
}

void gemm_u8_ctc_argmax(const U8Work& w, const U8W& wt, const float* bias, int M, int N, int K, int ts, float* pval,
                        int* pidx, int* out, hipStream_t s) {
  const U8Args u{w.xq, w.rs, w.qp, wt.q, wt.cs, wt.bz, wt.ws, ts};
  const int n_tiles = cdiv(N, 128);
  EpiArgmax128 epi{bias, pval, pidx, n_tiles};
  launch_gemm_u8<EpiArgmax128, 2, 2>(u, M, N, K, epi, s);
  hipLaunchKernelGGL(k_argmax_final, dim3(cdiv(M, 4)), dim3(256), 0, s, pval, pidx, M, n_tiles, out);
}

void gemm_ctc_argmax(const float* A, int64_t lda, const float* W, const float* bias, int M, int N, int K, float* pval,
                     int* pidx, int* out, hipStream_t s, const __half* W16, WSplit wb) {
  ALoadPlain al{A, lda};
  int n_tiles = cdiv(N, 64);
  const WSplit w16{reinterpret_cast<const uint16_t*>(W16)};
  if (W16 && g_gemm_f16_b3 && g_gemm_bf3_256 && (int64_t)cdiv(M, 256) * cdiv(N, 256) >= g_gemm_bf3_256) {
    n_tiles = cdiv(N, 256);
    EpiArgmax256 epi{bias, pval, pidx, n_tiles, 1};
    launch_gemm_b3_256<ALoadPlain, EpiArgmax256, 1>(al, w16, K, M, N, K, epi, s);
  } else if (W16 && g_gemm_f16_b3) {
    n_tiles = cdiv(N, 128);
    EpiArgmax128 epi{bias, pval, pidx, n_tiles, 1};
    launch_gemm_b3<ALoadPlain, EpiArgmax128, 2, 2, 32, 1, 1, 1>(al, w16, K, M, N, K, epi, s);
  } else if (wb.hi && g_gemm_bf3_256 && (int64_t)cdiv(M, 256) * cdiv(N, 256) >= g_gemm_bf3_256) {  // batched: 256x256
    n_tiles = cdiv(N, 256);
    EpiArgmax256 epi{bias, pval, pidx, n_tiles};
    launch_gemm_b3_256(al, wb, K, M, N, K, epi, s);
  } else if (wb.hi) {  // bf16x3: 128x128 blocks (one clip: 1001 x 60515 = 3784 tiles; 64x64 measured 606 us)
    n_tiles = cdiv(N, 128);
    EpiArgmax128 epi{bias, pval, pidx, n_tiles};
    launch_gemm_b3<ALoadPlain, EpiArgmax128, 2, 2, 32>(al, wb, K, M, N, K, epi, s);
  } else {
    EpiArgmax epi{bias, pval, pidx, n_tiles, W16 ? 1 : 0};
    // the argmax epilogue reduces 64-column blocks
    if (W16) launch_gemm16<ALoadPlain, EpiArgmax, 1, 1>(al, W16, K, M, N, K, epi, s);
    else run_gemm(al, W, K, M, N, K, epi, s, false);
  }
  hipLaunchKernelGGL(k_argmax_final, dim3(cdiv(M, 4)), dim3(256), 0, s, pval, pidx, M, n_tiles, out);
}

}  // namespace fa
