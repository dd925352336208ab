// Qwen3 decoder kernels with ggml q8_0 x q8_0 numerics (oracle/qwen3.py):
//   activations are RMS-normalised (optional) and quantised per 32-block with the ggml reference
//   quantiser, weight rows are q8_0 (engine layout: int8 qs[O][K] + fp16 d[O][K/32]), each block's
//   integer dot is exact (v_dot4_i32_i8), scaled by f32(dw)*f32(dx) and summed in f32.
// The decode GEMV streams every weight byte exactly once per step for the whole continuous batch
// (HBM-bound: 633 MB/step for Qwen3-0.6B q8_0); one wave covers a K=1024 row with ONE 16 B/lane load.
#include <algorithm>
#include <type_traits>
#include "common.h"
#include "kernels.h"

namespace fa {

// ------------------------------------------------------------------------------------------------
// per-row RMSNorm (ggml_rms_norm: 1/sqrtf(mean(x^2)+eps), then ggml_mul by w) + q8_0 quantisation.
// lane handles 16 consecutive values per 1024-chunk: x[c*1024 + lane*16 + j]; a 32-block = 2 lanes.
template <int NCH>
__device__ __forceinline__ void norm_quant_row(const float* __restrict__ x, const float* __restrict__ w, float eps,
                                               int lane, int8_t* __restrict__ q_out, float* __restrict__ d_out) {
  float v[NCH][16];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const float4* p = reinterpret_cast<const float4*>(x + c * 1024 + lane * 16);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float4 f = p[j];
      v[c][4 * j] = f.x;
      v[c][4 * j + 1] = f.y;
      v[c][4 * j + 2] = f.z;
      v[c][4 * j + 3] = f.w;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) ss += v[c][j] * v[c][j];
  }
  if (w) {
    ss = wave_sum(ss);
    const float mean = ss / (float)(NCH * 1024);
    const float scale = 1.0f / sqrtf(mean + eps);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const float4* wp = reinterpret_cast<const float4*>(w + c * 1024 + lane * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float4 f = wp[j];
        v[c][4 * j] = (v[c][4 * j] * scale) * f.x;
        v[c][4 * j + 1] = (v[c][4 * j + 1] * scale) * f.y;
        v[c][4 * j + 2] = (v[c][4 * j + 2] * scale) * f.z;
        v[c][4 * j + 3] = (v[c][4 * j + 3] * scale) * f.w;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) a = fmaxf(a, fabsf(v[c][j]));
    a = group_max<2>(a);
    const float d = a / 127.0f;
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    int32_t packed[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int b0 = (int)roundf(__fmul_rn(v[c][4 * j], id)) & 0xFF;
      int b1 = (int)roundf(__fmul_rn(v[c][4 * j + 1], id)) & 0xFF;
      int b2 = (int)roundf(__fmul_rn(v[c][4 * j + 2], id)) & 0xFF;
      int b3 = (int)roundf(__fmul_rn(v[c][4 * j + 3], id)) & 0xFF;
      packed[j] = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    }
    *reinterpret_cast<int4*>(q_out + c * 1024 + lane * 16) = make_int4(packed[0], packed[1], packed[2], packed[3]);
    if (!(lane & 1)) d_out[c * 32 + (lane >> 1)] = __half2float(__float2half_rn(d));
  }
}

// Block-cooperative variant (256 threads, one row): thread t owns K/256 consecutive values; a 32-value
// quant block spans 32/(K/256) threads. Same arithmetic as norm_quant_row, the sum of squares is reduced
// over the whole block. Used by the decode GEMV prologue (M == 1) so all 4 waves share the row.
template <int NCH>
__device__ __forceinline__ void norm_quant_row_block(const float* __restrict__ x, const float* __restrict__ w,
                                                     float eps, int8_t* __restrict__ q_out, float* __restrict__ d_out,
                                                     float* __restrict__ s_red) {
  constexpr int PER = NCH * 4;          // values per thread (K = NCH * 1024)
  constexpr int TPB = 32 / PER;         // threads per quant block (8, 4 or 2 for NCH 1, 2, 3 -> NCH 3 uses 12/32)
  // K = 3072: 12 values per thread do not tile 32-blocks; that width uses per-wave chunks (norm_quant_row)
  static_assert(NCH == 1 || NCH == 2, "norm_quant_row_block: K must be 1024 or 2048");
  const int t = threadIdx.x;
  float v[PER];
#pragma unroll
  for (int j = 0; j < PER; j += 4) {
    const float4 f = *reinterpret_cast<const float4*>(x + t * PER + j);
    v[j] = f.x; v[j + 1] = f.y; v[j + 2] = f.z; v[j + 3] = f.w;
  }
  if (w) {
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < PER; ++j) ss += v[j] * v[j];
    ss = wave_sum(ss);
    if ((t & 63) == 0) s_red[t >> 6] = ss;
    __syncthreads();
    ss = s_red[0] + s_red[1] + s_red[2] + s_red[3];
    const float scale = 1.0f / sqrtf(ss / (float)(NCH * 1024) + eps);
#pragma unroll
    for (int j = 0; j < PER; j += 4) {
      const float4 f = *reinterpret_cast<const float4*>(w + t * PER + j);
      v[j] = (v[j] * scale) * f.x;
      v[j + 1] = (v[j + 1] * scale) * f.y;
      v[j + 2] = (v[j + 2] * scale) * f.z;
      v[j + 3] = (v[j + 3] * scale) * f.w;
    }
  }
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) a = fmaxf(a, fabsf(v[j]));
  a = group_max<TPB>(a);
  const float d = a / 127.0f;
  const float id = d != 0.0f ? 1.0f / d : 0.0f;
  int8_t qv[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) qv[j] = (int8_t)roundf(__fmul_rn(v[j], id));
  if (PER == 4) *reinterpret_cast<int32_t*>(q_out + t * PER) = *reinterpret_cast<int32_t*>(qv);
  else *reinterpret_cast<int2*>(q_out + t * PER) = *reinterpret_cast<int2*>(qv);
  if ((t % TPB) == 0) d_out[t / TPB] = __half2float(__float2half_rn(d));
}

// The same two prologues from values already in registers (the GEMV issues its activation loads before its
// weight stream: vmcnt retires in issue order, so activation loads issued after the weights would wait for them).
// Arithmetic identical to norm_quant_row_block / norm_quant_row.
template <int PER>
__device__ __forceinline__ void norm_quant_block_regs(float (&v)[PER], const float (&wv)[PER], bool has_w, float eps,
                                                      int K, int8_t* __restrict__ q_out, float* __restrict__ d_out,
                                                      float* __restrict__ s_red) {
  constexpr int TPB = 32 / PER;
  const int t = threadIdx.x;
  if (has_w) {
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < PER; ++j) ss += v[j] * v[j];
    ss = wave_sum(ss);
    if ((t & 63) == 0) s_red[t >> 6] = ss;
    __syncthreads();
    ss = s_red[0] + s_red[1] + s_red[2] + s_red[3];
    const float scale = 1.0f / sqrtf(ss / (float)K + eps);
#pragma unroll
    for (int j = 0; j < PER; ++j) v[j] = (v[j] * scale) * wv[j];
  }
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) a = fmaxf(a, fabsf(v[j]));
  a = group_max<TPB>(a);
  const float d = a / 127.0f;
  const float id = d != 0.0f ? 1.0f / d : 0.0f;
  int8_t qv[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) qv[j] = (int8_t)roundf(__fmul_rn(v[j], id));
  if (PER == 4) *reinterpret_cast<int32_t*>(q_out + t * PER) = *reinterpret_cast<int32_t*>(qv);
  else *reinterpret_cast<int2*>(q_out + t * PER) = *reinterpret_cast<int2*>(qv);
  if ((t % TPB) == 0) d_out[t / TPB] = __half2float(__float2half_rn(d));
}

// one 1024-chunk per wave, no norm (norm_quant_row<1> with w = nullptr): lane holds x[lane*16 .. +16)
__device__ __forceinline__ void quant_chunk_regs(const float (&v)[16], int lane, int8_t* __restrict__ q_out,
                                                 float* __restrict__ d_out) {
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) a = fmaxf(a, fabsf(v[j]));
  a = group_max<2>(a);
  const float d = a / 127.0f;
  const float id = d != 0.0f ? 1.0f / d : 0.0f;
  int32_t packed[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int b0 = (int)roundf(__fmul_rn(v[4 * j], id)) & 0xFF;
    int b1 = (int)roundf(__fmul_rn(v[4 * j + 1], id)) & 0xFF;
    int b2 = (int)roundf(__fmul_rn(v[4 * j + 2], id)) & 0xFF;
    int b3 = (int)roundf(__fmul_rn(v[4 * j + 3], id)) & 0xFF;
    packed[j] = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
  }
  *reinterpret_cast<int4*>(q_out + lane * 16) = make_int4(packed[0], packed[1], packed[2], packed[3]);
  if (!(lane & 1)) d_out[lane >> 1] = __half2float(__float2half_rn(d));
}

template <int NCH>
__global__ __launch_bounds__(256) void k_prep_q8(const float* __restrict__ x, int64_t ldx, const float* __restrict__ w,
                                                 float eps, int M, int8_t* __restrict__ xq, float* __restrict__ xd) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int K = NCH * 1024;
  norm_quant_row<NCH>(x + (int64_t)row * ldx, w, eps, threadIdx.x & 63, xq + (int64_t)row * K, xd + (int64_t)row * (K / 32));
}

void prep_q8(const float* x, int64_t ldx, const float* w, float eps, int M, int K, int8_t* xq, float* xd, hipStream_t s) {
  dim3 grid(cdiv(M, 4));
  switch (K) {
    case 1024: hipLaunchKernelGGL(k_prep_q8<1>, grid, dim3(256), 0, s, x, ldx, w, eps, M, xq, xd); break;
    case 2048: hipLaunchKernelGGL(k_prep_q8<2>, grid, dim3(256), 0, s, x, ldx, w, eps, M, xq, xd); break;
    case 3072: hipLaunchKernelGGL(k_prep_q8<3>, grid, dim3(256), 0, s, x, ldx, w, eps, M, xq, xd); break;
    default: FA_REQUIRE(false, "prep_q8: K must be 1024/2048/3072");
  }
}

// ------------------------------------------------------------------------------------------------
// q8_0 GEMV / small-M GEMM. Block = 4 waves; block (bx, by) covers rows [bx*4*rpw, ...) and tokens
// [by*MT, by*MT+MT). The activation tile is quantised into LDS by the prologue, either from f32 rows
// (FUSED: rmsnorm+quant recomputed per block, cheap for decode M<=4) or copied from global xq/xd.
// Epilogues: 0 store, 1 residual add (out = res + y, in place allowed), 2 SwiGLU (gate & up rows),
//            3 store + per-wave argmax partial (lm_head, greedy sampling).


__device__ __forceinline__ int dot16(const int4& a, const int4& b, int acc) {
  acc = __builtin_amdgcn_sdot4(a.x, b.x, acc, false);
  acc = __builtin_amdgcn_sdot4(a.y, b.y, acc, false);
  acc = __builtin_amdgcn_sdot4(a.z, b.z, acc, false);
  acc = __builtin_amdgcn_sdot4(a.w, b.w, acc, false);
  return acc;
}

typedef int i32x4_t __attribute__((ext_vector_type(4)));
// streamed-once weights: non-temporal 16 B loads (MI355X_MICROARCH.md row nt-weights)
__device__ __forceinline__ int4 ld_nt16(const int8_t* p) {
  const i32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const i32x4_t*>(p));
  return make_int4(v.x, v.y, v.z, v.w);
}

template <int NCH, int EPI>
struct RowGroup {
  int4 w[4][NCH];
  int4 u[4][NCH];
  float dw[4][NCH];
  float du[4][NCH];
};

// FA_LM_HEAD_NT = 0 (A/B builds only): the LM head's rows (EPI 3) with default-policy loads instead of nt, so that
// they might stay in the Infinity Cache across steps. Graph-replayed batch-1 step (scripts/gpu_r4_l2pf.sh LMT=1):
// 0.4695 vs 0.4740-0.4771 ms without the L2 prefetch blocks, 0.4600 vs 0.4537-0.4549 ms with them: nt stays.
#ifndef FA_LM_HEAD_NT
#define FA_LM_HEAD_NT 1
#endif
template <int NCH, int EPI>
__device__ __forceinline__ void load_group(const GemvArgs& a, int row_base, int r0, int lane, RowGroup<NCH, EPI>& G) {
  constexpr int K = NCH * 1024, NB = K / 32;
  // rows past the matrix/slice are loaded from a clamped valid row and their scales zeroed: no
  // per-row branches around the loads (hipcc would wait vmcnt(0) at each, serialising the stream)
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int row0 = row_base + r0 + rr;
    const bool ok = (r0 + rr < a.rpw) && row0 < a.O;
    const int row = min(row0, a.O - 1);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (EPI == 3 && !FA_LM_HEAD_NT)
        G.w[rr][c] = *reinterpret_cast<const int4*>(a.wq + (int64_t)row * K + c * 1024 + lane * 16);
      else
        G.w[rr][c] = ld_nt16(a.wq + (int64_t)row * K + c * 1024 + lane * 16);
      const float dv = __half2float(a.wd[(int64_t)row * NB + c * 32 + (lane >> 1)]);
      G.dw[rr][c] = ok ? dv : 0.f;
      if (EPI == 2) {
        G.u[rr][c] = ld_nt16(a.wq2 + (int64_t)row * K + c * 1024 + lane * 16);
        const float du = __half2float(a.wd2[(int64_t)row * NB + c * 32 + (lane >> 1)]);
        G.du[rr][c] = ok ? du : 0.f;
      }
    }
  }
}

// the first row group's residual values are loaded with the activations (1; 0: at the epilogue, A/B builds)
#ifndef FA_RES0_PRELOAD
#define FA_RES0_PRELOAD 1
#endif
// One level of a transposed wave reduction: lanes l and l ^ (1 << B) exchange halves of their N partial sums, so every
// lane keeps N / 2 of them, each now summed over both lanes. Levels B = 0..5 add the lanes in exactly wave_sum's
// pairs (xor 1, xor 2, then quads, 8-lane halves, rows 0+1 / 2+3, and the two row pairs: row_half_mirror and
// row_mirror pair the same groups once the lower levels made their lanes equal), so every sum is bit-identical to
// wave_sum of that value, for N values at the cost of about 3 N / 2 instructions instead of 11 N.
template <int N, int B>
__device__ __forceinline__ void tr_level(float (&v)[32], int lane) {
  const bool hi = (lane >> B) & 1;
#pragma unroll
  for (int k = 0; k < N / 2; ++k) {
    const float keep = hi ? v[k + N / 2] : v[k];
    const float send = hi ? v[k] : v[k + N / 2];
    float recv;
    if constexpr (B == 0) recv = dpp_f<DPP_XOR1>(send);
    else if constexpr (B == 1) recv = dpp_f<DPP_XOR2>(send);
    else recv = __shfl_xor(send, 1 << B, 64);
    v[k] = keep + recv;
  }
}

template <int NCH, int MT, int EPI, bool TR = false>
__device__ __forceinline__ void compute_group(const GemvArgs& a, int row_base, int r0, int lane, int m0, int mt,
                                              const int8_t* s_q, const float* s_d, const RowGroup<NCH, EPI>& G,
                                              float (&best_v)[MT], int (&best_i)[MT], const float (&res0)[4]) {
  constexpr int K = NCH * 1024, NB = K / 32;
  if constexpr (TR) {
    static_assert(EPI == 3 && MT > 1 && MT <= 8, "compute_group: transposed reduction for the LM head of 2-8 tokens");
    // LM head of 2-8 tokens: the 4 rows x MT tokens of the group reduced together (slot rr * 8 + m); afterwards lane l
    // (and l ^ 32) holds slot 16 b0 + 8 b1 + 4 b2 + 2 b3 + b4 of its bits, i.e. row rr = 2 b0 + b1 and token
    // m = 4 b2 + 2 b3 + b4, and keeps the running argmax of its (rr, m) in best_v[0] / best_i[0]; the tokens' argmax
    // partials are gathered once per wave after the row loop (argmax_combine is order-free: max, lowest index on ties)
    float v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = 0.f;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (m >= mt) break;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int4 xv = *reinterpret_cast<const int4*>(s_q + m * K + c * 1024 + lane * 16);
        const float xdv = s_d[m * NB + c * 32 + (lane >> 1)];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          int si = dot16(G.w[rr][c], xv, 0);
          si += dpp_i<DPP_XOR1>(si);
          if (!(lane & 1)) v[rr * 8 + m] += (float)si * (G.dw[rr][c] * xdv);
        }
      }
    }
    tr_level<32, 0>(v, lane);
    tr_level<16, 1>(v, lane);
    tr_level<8, 2>(v, lane);
    tr_level<4, 3>(v, lane);
    tr_level<2, 4>(v, lane);
    const float y = v[0] + __shfl_xor(v[0], 32, 64);
    const int rr = 2 * (lane & 1) + ((lane >> 1) & 1), m = 4 * ((lane >> 2) & 1) + 2 * ((lane >> 3) & 1) + ((lane >> 4) & 1);
    const int row = row_base + r0 + rr;
    if (lane < 32 && m < mt && (r0 + rr < a.rpw) && row < a.O) {
      a.out[(int64_t)(m0 + m) * a.ldo + row] = y;
      argmax_combine(best_v[0], best_i[0], y, row);
    }
    return;
  }
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    if (m >= mt) break;
    float acc[4] = {0.f, 0.f, 0.f, 0.f}, acc2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int4 xv = *reinterpret_cast<const int4*>(s_q + m * K + c * 1024 + lane * 16);
      const float xdv = s_d[m * NB + c * 32 + (lane >> 1)];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        int si = dot16(G.w[rr][c], xv, 0);
        si += dpp_i<DPP_XOR1>(si);
        if (!(lane & 1)) acc[rr] += (float)si * (G.dw[rr][c] * xdv);
        if (EPI == 2) {
          int su = dot16(G.u[rr][c], xv, 0);
          su += dpp_i<DPP_XOR1>(su);
          if (!(lane & 1)) acc2[rr] += (float)su * (G.du[rr][c] * xdv);
        }
      }
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = row_base + r0 + rr;
      const float y = wave_sum(acc[rr]);
      const float y2 = EPI == 2 ? wave_sum(acc2[rr]) : 0.f;
      if (lane == 0 && (r0 + rr < a.rpw) && row < a.O) {
        float* op = a.out + (int64_t)(m0 + m) * a.ldo + row;
        if (EPI == 0 || EPI == 3) *op = y;
        else if (EPI == 1) *op = (MT == 1 && r0 == 0 && FA_RES0_PRELOAD ? res0[rr] : a.res[(int64_t)(m0 + m) * a.ldr + row]) + y;
        else *op = (y / (1.0f + expf(-y))) * y2;
        if (EPI == 3) argmax_combine(best_v[m], best_i[m], y, row);
      }
    }
  }
}

// FA_GEMV_STAMPS (microbenchmark builds only): per-block s_memrealtime stamps (100 MHz, chip-wide) of the
// decode GEMV: [start, prologue done, rows done, end] -> g_gstamps[block]
#ifdef FA_GEMV_STAMPS
__device__ unsigned long long g_gstamps[4096][4];
#define GSTAMP(i) do { if (threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.x < 4096) g_gstamps[blockIdx.x][i] = __builtin_amdgcn_s_memrealtime(); } while (0)
void gemv_stamps_read(unsigned long long* host, int n) {
  (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gstamps), (size_t)n * 32, 0, hipMemcpyDeviceToHost);
}
// split-K GEMM: [start, loads landed, reduced in LDS, partial published, arrival counted, end], linear block id
__device__ unsigned long long g_kstamps[4096][6];
#define KSTAMP(i) do { const unsigned bid = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x; \
  if (threadIdx.x == 0 && bid < 4096) g_kstamps[bid][i] = __builtin_amdgcn_s_memrealtime(); } while (0)
void gemm_stamps_read(unsigned long long* host, int n) {
  (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_kstamps), (size_t)n * 48, 0, hipMemcpyDeviceToHost);
}
#else
#define GSTAMP(i) do { } while (0)
#define KSTAMP(i) do { } while (0)
#endif

// PS (fused decode, M = 1, K = 1024): the activation row is first completed as x + psum[0] + ... + psum[7] (the split
// down projection of the previous fused layer), and block 0 stores that row to a.xsum (the residual stream).
// TR: the LM head of 2-8 tokens with the transposed row x token reduction (compute_group; same sums, same argmax)
template <int NCH, int MT, bool FUSED, int EPI, bool PS = false, bool TR = false>
__global__ __launch_bounds__(256) void k_gemv_q8(GemvArgs a) {
  static_assert(!PS || (NCH == 1 && MT == 1 && FUSED), "partial-sum prologue: M = 1, K = 1024 only");
  GSTAMP(0);
  constexpr int K = NCH * 1024, NB = K / 32;
  __shared__ int8_t s_q[MT * K];
  __shared__ float s_d[MT * NB];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int m0 = blockIdx.y * MT;
  const int mt = min(MT, a.M - m0);
  const int row_base = (blockIdx.x * 4 + wave) * a.rpw;
  // ---- activation loads first (a few KB that the whole block waits on; vmcnt retires in issue order, so
  // behind the weight stream they would arrive only with it), then the first weight row group, then the
  // prologue math: the weights stream in while the activations are normalised and quantised
  // (branch-free: a branch here makes the wait-count pass drain the loads at the join, before the weight stream)
  // MT > 1 (small decode batches: every weight row streamed once for all the block's tokens): the same
  // block-cooperative / per-chunk prologue once per token row, so a token's q8_0 input rows are bit-identical to
  // the MT == 1 launch's (continuous batch == single sequence). Rows past mt load a clamped valid row, unused.
  constexpr int PERB = NCH * 4;  // block-cooperative prologue: values per thread
  const bool pro_blk = FUSED && NCH < 3;
  const bool pro_chunk = FUSED && NCH == 3 && !a.norm_w;  // K = 3072, no norm (down projection)
  float xv[MT][NCH < 3 ? PERB : 16], xw[PERB];
  float pv[PS ? FUSED_PARTS : 1][PS ? PERB : 1];
  if constexpr (PS) {
#pragma unroll
    for (int g = 0; g < FUSED_PARTS; ++g) {
      const float4 f = *reinterpret_cast<const float4*>(a.psum + g * 1024 + threadIdx.x * PERB);
      pv[g][0] = f.x; pv[g][1] = f.y; pv[g][2] = f.z; pv[g][3] = f.w;
    }
  }
  if constexpr (FUSED && NCH < 3) {
    const float* wr = (a.norm_w ? a.norm_w : a.x) + threadIdx.x * PERB;  // no norm: a valid dummy row, unused
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const float* xr = a.x + (int64_t)(m0 + min(m, mt - 1)) * a.ldx + threadIdx.x * PERB;
#pragma unroll
      for (int j = 0; j < PERB; j += 4) {
        const float4 f = *reinterpret_cast<const float4*>(xr + j);
        xv[m][j] = f.x; xv[m][j + 1] = f.y; xv[m][j + 2] = f.z; xv[m][j + 3] = f.w;
      }
    }
#pragma unroll
    for (int j = 0; j < PERB; j += 4) {
      const float4 g = *reinterpret_cast<const float4*>(wr + j);
      xw[j] = g.x; xw[j + 1] = g.y; xw[j + 2] = g.z; xw[j + 3] = g.w;
    }
  } else if constexpr (FUSED && NCH == 3) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const float* xr = a.x + (int64_t)(m0 + min(m, mt - 1)) * a.ldx + min(wave, 2) * 1024 + lane * 16;  // wave 3: unused
#pragma unroll
      for (int j = 0; j < 16; j += 4) {
        const float4 f = *reinterpret_cast<const float4*>(xr + j);
        xv[m][j] = f.x; xv[m][j + 1] = f.y; xv[m][j + 2] = f.z; xv[m][j + 3] = f.w;
      }
    }
  }
  // residual epilogue: the first row group's residual values ride with the activation loads (a load after the
  // dot products would be one more serial memory latency at the tail)
  float res0[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (EPI == 1 && MT == 1 && FA_RES0_PRELOAD) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) res0[rr] = a.res[(int64_t)m0 * a.ldr + min(row_base + rr, a.O - 1)];
  }
  __builtin_amdgcn_sched_barrier(0);  // the scheduler would otherwise sink these loads below the weight stream
  RowGroup<NCH, EPI> G0, G1;
  load_group<NCH, EPI>(a, row_base, 0, lane, G0);
  // keep the prologue math below the weight loads: otherwise the scheduler hoists it and waits for the
  // activations (vmcnt(0)) before the weight stream is even issued
  __builtin_amdgcn_sched_barrier(0);
  // ---- prologue: activation tile -> LDS (int8 q + f32 d)
  if constexpr (PS) {
#pragma unroll
    for (int j = 0; j < PERB; ++j) {
      float v = xv[0][j];
#pragma unroll
      for (int g = 0; g < FUSED_PARTS; ++g) v = v + pv[g][j];
      xv[0][j] = v;
    }
    if (a.xsum && blockIdx.x == 0)
      *reinterpret_cast<float4*>(a.xsum + threadIdx.x * PERB) = make_float4(xv[0][0], xv[0][1], xv[0][2], xv[0][3]);
  }
  if (pro_blk) {
    __shared__ float s_red[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (m < mt) {  // block-uniform
        float v[PERB];
#pragma unroll
        for (int j = 0; j < PERB; ++j) v[j] = xv[m][j];
        norm_quant_block_regs<PERB>(v, xw, a.norm_w != nullptr, a.eps, NCH * 1024, s_q + m * K, s_d + m * NB, s_red[m]);
      }
    }
  } else if (pro_chunk) {
    if (wave < NCH) {
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        if (m < mt) {
          float v[16];
#pragma unroll
          for (int j = 0; j < 16; ++j) v[j] = xv[m][j];
          quant_chunk_regs(v, lane, s_q + m * K + wave * 1024, s_d + m * NB + wave * 32);
        }
      }
    }
  } else if (FUSED) {
    for (int m = wave; m < mt; m += 4)
      norm_quant_row<NCH>(a.x + (int64_t)(m0 + m) * a.ldx, a.norm_w, a.eps, lane, s_q + m * K, s_d + m * NB);
  } else {
    const int4* src = reinterpret_cast<const int4*>(a.xq + (int64_t)m0 * K);
    int4* dst = reinterpret_cast<int4*>(s_q);
    for (int i = threadIdx.x; i < mt * K / 16; i += 256) dst[i] = src[i];
    for (int i = threadIdx.x; i < mt * NB; i += 256) s_d[i] = a.xd[(int64_t)m0 * NB + i];
  }
  __syncthreads();
  GSTAMP(1);
  float best_v[MT];
  int best_i[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    best_v[m] = -INFINITY;
    best_i[m] = 0x7fffffff;
  }
  // two-deep register pipeline over 4-row groups (static buffer names, no runtime-indexed arrays)
  for (int r0 = 0; r0 < a.rpw; r0 += 8) {
    if (r0 + 4 < a.rpw) load_group<NCH, EPI>(a, row_base, r0 + 4, lane, G1);
    compute_group<NCH, MT, EPI, TR>(a, row_base, r0, lane, m0, mt, s_q, s_d, G0, best_v, best_i, res0);
    if (r0 + 4 >= a.rpw) break;
    if (r0 + 8 < a.rpw) load_group<NCH, EPI>(a, row_base, r0 + 8, lane, G0);
    compute_group<NCH, MT, EPI, TR>(a, row_base, r0 + 4, lane, m0, mt, s_q, s_d, G1, best_v, best_i, res0);
  }
  GSTAMP(2);
  if constexpr (TR) {  // compute_group's lane-spread argmax: token m's 4 lanes -> lane 0
    const int part = blockIdx.x * 4 + wave;
    const float bv = best_v[0];
    const int bi = best_i[0];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float v = -INFINITY;
      int i = 0x7fffffff;
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // lanes of token m: bits 0-1 = row, bits 2-4 = m's bits 2, 1, 0
        const int l = q + 4 * ((m >> 2) & 1) + 8 * ((m >> 1) & 1) + 16 * (m & 1);
        argmax_combine(v, i, __shfl(bv, l, 64), __shfl(bi, l, 64));
      }
      if (lane == 0 && m < mt) {
        a.pval[(int64_t)(m0 + m) * a.n_part + part] = v;
        a.pidx[(int64_t)(m0 + m) * a.n_part + part] = i;
      }
    }
  } else if (EPI == 3 && lane == 0) {
    const int part = blockIdx.x * 4 + wave;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (m < mt) {
        a.pval[(int64_t)(m0 + m) * a.n_part + part] = best_v[m];
        a.pidx[(int64_t)(m0 + m) * a.n_part + part] = best_i[m];
      }
    }
  }
}

int g_lm_tr = 1;  // LM head of 2-8 tokens: transposed row x token reduction (FUNASR_LM_TR; A/B, scripts/gpu_r4_exp11.sh:
                  // batch-6 decode step 0.933-0.946 -> 0.914-0.931 ms, C4 1038 -> 1051 audio-s/s; bit-identical logits)

template <int NCH, int MT, bool FUSED, int EPI, bool PS = false>
static void launch_gemv(const GemvArgs& a, hipStream_t s) {
  dim3 grid(cdiv(a.O, 4 * a.rpw), cdiv(a.M, MT));
  if constexpr (EPI == 3 && MT > 1 && MT <= 8) {
    if (g_lm_tr) {
      hipLaunchKernelGGL((k_gemv_q8<NCH, MT, FUSED, EPI, PS, true>), grid, dim3(256), 0, s, a);
      return;
    }
  }
  hipLaunchKernelGGL((k_gemv_q8<NCH, MT, FUSED, EPI, PS>), grid, dim3(256), 0, s, a);
}

template <int MT, bool FUSED, int EPI>
static void launch_gemv_k(int K, const GemvArgs& a, hipStream_t s) {
  switch (K) {
    case 1024: launch_gemv<1, MT, FUSED, EPI>(a, s); break;
    case 2048: launch_gemv<2, MT, FUSED, EPI>(a, s); break;
    case 3072: launch_gemv<3, MT, FUSED, EPI>(a, s); break;
    default: FA_REQUIRE(false, "gemv_q8: K must be 1024/2048/3072");
  }
}

// ------------------------------------------------------------------------------------------------
// q8_0 x q8_0 GEMM on the int8 matrix cores (M > 4: prefill and continuous-batch decode). gfx950's
// v_mfma_i32_32x32x32_i8 has K = 32 = one q8_0 block, so each MFMA yields the EXACT integer block dot
// for a 32-row x 32-token tile (the ggml per-block sumi); it is scaled by f32(dw) * f32(dx) and summed in
// f32, as ggml_vec_dot_q8_0_q8_0 does. Operand map (verified with exact integers,
// scripts/ubench/mfma_i8_probe.hip): lane l holds A[l&31][16(l>>5) + j], B[16(l>>5) + j][l&31];
// D: col = l&31 (token), row = (reg&3) + 8(reg>>2) + 4(l>>5) (weight row).
// Block = 4 waves over one 32x32 tile, each wave a contiguous quarter of K; partial tiles are summed in
// LDS in fixed wave order (deterministic). Epilogues as k_gemv_q8.
typedef int i32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// int8 MFMA returning f32: the accumulator starts at 1.5 * 2^23, so every element is the f32 bit pattern of
// 12582912 + dot (|dot| <= 32 * 128 * 128 < 2^22) and as_float(D) - 12582912 == (float)dot exactly (both operands in
// [2^23, 2^24): Sterbenz), two elements per v_pk_add_f32 instead of one v_cvt_f32_i32 each
// (MAGIC = false: the plain conversion, for kernels where the constant's 16 registers would spill)
template <bool MAGIC = true>
__device__ __forceinline__ f32x16 mfma_i8_f32(const i32x4_t& a, const i32x4_t& b) {
  if constexpr (MAGIC) {
    constexpr int M = 0x4B400000;
    const i32x16_t magic = {M, M, M, M, M, M, M, M, M, M, M, M, M, M, M, M};
    const i32x16_t D = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, magic, 0, 0, 0);
    return __builtin_bit_cast(f32x16, D) - 12582912.0f;
  } else {
    const i32x16_t zero = {};
    return __builtin_convertvector(__builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, zero, 0, 0, 0), f32x16);
  }
}

// Scales of NBW consecutive q8_0 blocks of one weight row (fp16, NBW/2 dwords): one load instruction
template <int NBW>
__device__ __forceinline__ void load_scales(const __half* p, uint32_t (&d)[NBW / 2]) {
  if constexpr (NBW == 8) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  } else if constexpr (NBW == 4) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    d[0] = v.x; d[1] = v.y;
  } else {
    d[0] = *reinterpret_cast<const uint32_t*>(p);
  }
}

// SwiGLU epilogue's q8_0 rows: the tile's 32 rows of a token are one q8_0 block of the down projection's input,
// quantised exactly as norm_quant_row does (no prep launch). s_act = tile [token][row]; threads 0..63: token
// t & 31, rows [16 (t >> 5), +16)
template <bool SC1 = false>
__device__ __forceinline__ void swiglu_tile_q8(const float (*s_act)[33], const GemvArgs& a, int t0, int o0) {
  if (threadIdx.x >= 64) return;
  const int tk = threadIdx.x & 31, hh = threadIdx.x >> 5;
  float vv[16], am = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    vv[i] = s_act[tk][16 * hh + i];
    am = fmaxf(am, fabsf(vv[i]));
  }
  am = fmaxf(am, __shfl_xor(am, 32, 64));
  const float d = am / 127.0f;
  const float id = d != 0.0f ? 1.0f / d : 0.0f;
  int32_t pk[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int b0 = (int)roundf(__fmul_rn(vv[4 * j], id)) & 0xFF, b1 = (int)roundf(__fmul_rn(vv[4 * j + 1], id)) & 0xFF;
    const int b2 = (int)roundf(__fmul_rn(vv[4 * j + 2], id)) & 0xFF, b3 = (int)roundf(__fmul_rn(vv[4 * j + 3], id)) & 0xFF;
    pk[j] = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
  }
  if (t0 + tk < a.M) {
    if constexpr (SC1) {  // consumed inside this launch (k_gemm_q8_gu_down): write-through stores, drained by the caller
      const __amdgpu_buffer_rsrc_t rq = buf_rsrc(a.qout, a.M * (int)a.ldo);
      const __amdgpu_buffer_rsrc_t rd = buf_rsrc(a.dout, a.M * (int)(a.ldo / 32) * 4);
      st_sc1_f4(__builtin_bit_cast(f32x4_t, i32x4v_t{pk[0], pk[1], pk[2], pk[3]}), rq,
                (int)((t0 + tk) * a.ldo + o0 + 16 * hh));
      if (hh == 0)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(__half2float(__float2half_rn(d))), rd,
                                              (int)(((t0 + tk) * (a.ldo / 32) + o0 / 32) * 4), 0, CPOL_SC1);
    } else {
      *reinterpret_cast<int4*>(a.qout + (int64_t)(t0 + tk) * a.ldo + o0 + 16 * hh) = make_int4(pk[0], pk[1], pk[2], pk[3]);
      if (hh == 0) a.dout[(int64_t)(t0 + tk) * (a.ldo / 32) + o0 / 32] = __half2float(__float2half_rn(d));
    }
  }
}

// Split-K form (few-tile shapes: batched decode, the o GEMM of prefill). Block = 4 waves over one 32x32 tile and one
// K split of 4 NBW q8_0 blocks (SwiGLU: 2 waves per matrix); every wave issues ALL its weight / activation / scale
// loads before its MFMAs (one memory round trip), and the residual is fetched before the hop. Splits merge by last
// arriver (sc1 partials, MI355X_MICROARCH.md hand-off table row 1) with the KSM partial loads in flight together,
// summed in split order (deterministic).
//
// NRM (batched decode, K = 1024): the input rows come from the previous residual GEMM's epilogue (ssp_out below),
// which quantised z = x * norm_w per 32-block (its tile is one q8_0 block of every token: xq, and the unscaled
// f32 block scales d_z in xd) and left the per-token sum-of-squares partials ssp [M][32]. RMSNorm's per-token factor
// rstd = 1/sqrtf(sum/K + eps) scales every block uniformly, so the q8_0 rows of y = (x * rstd) * w are the same
// integers (up to float rounding at .5 ties) with scale f16(rstd * d_z): this GEMM only applies rstd, and the two
// k_prep_q8 launches per layer (with their kernel boundaries) disappear.
int g_gemm_pf = 7;
int g_gemm_pf_slabs = 4;
int g_gemm_pf_delay = 50;

// L2 prefetch slabs of a batched-decode split-K GEMM (blockIdx.z >= KS): the next GEMM of the layer chain is split-K
// too, with 32-row tiles x on XCD x % 8 (linear block id % 8, tile count a multiple of 8), so XCD g's blocks read
// rows [32 x, +32) for x = g + 8 i in full (every K split of a tile shares its XCD). After pf_delay ticks (this launch's
// own weights have landed) the prefetch blocks on XCD g pull those rows and their scales into g's L2 with LDS-DMA
// loads into a scratch slot, drained before the block ends. Only lines move; no result changes.
// idx: this block's index among the launch's n_pf prefetch blocks (n_pf % 8 == 0; placement: linear block id % 8 ==
// idx % 8, i.e. the launch's compute blocks before them come in multiples of 8)
__device__ __forceinline__ void gemm_l2_prefetch(const GemvArgs& a, int idx, int n_pf) {
  __shared__ __attribute__((aligned(16))) int4 s_pf[4][64];
  const int g = idx & 7, pb = idx >> 3, P = n_pf / 8;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)a.pf_delay) __builtin_amdgcn_s_sleep(4);
  auto* lds = (__attribute__((address_space(3))) void*)&s_pf[threadIdx.x >> 6][0];
  const int T = P * 256, tid = pb * 256 + threadIdx.x, K = a.pf_K;
  for (int x = g; x < a.pf_O / 32; x += 8) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int8_t* q = m ? a.pf_q2 : a.pf_q;
      const __half* d = m ? a.pf_d2 : a.pf_d;
      if (!q) continue;
      const char* qb = (const char*)(q + (int64_t)32 * x * K);  // 32 rows x K bytes
      for (int u = tid; u < 2 * K; u += T) __builtin_amdgcn_global_load_lds((const void*)(qb + (int64_t)u * 16), lds, 16, 0, 0);
      const char* db = (const char*)(d + (int64_t)32 * x * (K / 32));  // 32 rows x K / 32 f16 scales
      for (int u = tid; u < K / 8; u += T) __builtin_amdgcn_global_load_lds((const void*)(db + (int64_t)u * 16), lds, 16, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA write may land after the block's LDS is released
}

// Every in-launch wait is bounded by time, not spin count: SPIN_TICKS of the 100 MHz reference clock (10 ms) from
// the first poll (checked every 16 polls). A group that is not co-resident (another kernel holding CUs) then costs a
// few ms per wait instead of seconds; the timed-out block sets *err and falls through, and fa_llm_generate_end re-runs
// the chunk on the fused layer first and only then on the 5-launch layer (engine.cpp, recover_fused_chunk).
constexpr uint64_t SPIN_TICKS = 1000000;
struct SpinDeadline {
  uint64_t t0 = 0;
  unsigned n = 0;
  __device__ __forceinline__ bool expired() {
    if ((++n & 15) != 1) return false;
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (n == 1) {
      t0 = t;
      return false;
    }
    return t - t0 > SPIN_TICKS;
  }
};

// In-launch fusion of two split-K GEMMs of the batched-decode chain (k_gemm_q8_gu_down): ROLE 1 = a SwiGLU producer
// whose combining block publishes its act tile (sc1 stores, drained) and counts it on arr[tile / tiles_per_split]; ROLE 2
// = a consumer (down projection, K split s = its act columns [32 tiles_per_split s, +32 tiles_per_split)) that issues
// its weight rows and scales first, waits for its split's tiles, then reads the act rows with sc1 loads. The consumer
// blocks of a split count themselves past the wait on dep[s]; the last one re-arms both counters for the next launch
// (every producer of this launch has counted by then, and the next launch starts after this one ends).
struct SkFuse {
  unsigned* arr = nullptr;
  unsigned* dep = nullptr;
  int tiles_per_split = 0;
  int consumers = 0;
  int* err = nullptr;
};

template <int EPI, int NBW, int KSM, bool NRM, int ROLE>
__device__ __forceinline__ void sk_tile(const GemvArgs& a, int K, int KS, int bx, int by, int bz, int gdx,
                                        int8_t* s_ab_mem, const SkFuse& fz) {
  constexpr int WPM = EPI == 2 ? 2 : 4;  // waves per weight matrix
  constexpr int NS = EPI == 2 ? 2 : 1;
  static_assert(!NRM || EPI != 1, "k_gemm_q8_sk: NRM inputs feed q|k|v, gate|up and the LM head");
  const int nb = K >> 5;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int o0 = bx * 32, t0 = by * 32, ks = bz;
  const bool upw = EPI == 2 && wave >= 2;
  const int bw0 = (ks * WPM + (EPI == 2 ? (wave & 1) : wave)) * NBW;  // host: nb == KS * WPM * NBW
  const int8_t* wq = upw ? a.wq2 : a.wq;
  const __half* wd = upw ? a.wd2 : a.wd;
  const int t_b = min(t0 + r, a.M - 1);
  KSTAMP(0);
  float4 sv[NRM ? 8 : 1];
  if constexpr (NRM) {  // this lane's token's 32 partials, issued first (vmcnt retires in issue order)
#pragma unroll
    for (int i = 0; i < 8; ++i) sv[i] = *reinterpret_cast<const float4*>(a.ssp + (int64_t)t_b * 32 + 4 * i);
  }
  i32x4_t A[NBW], B[NBW];
  // coalesced: load instruction i reads RPI rows x RB contiguous bytes of the wave's K slice (weights and activations);
  // the fragments are rebuilt through LDS below (16 B per lane from 32 rows per instruction ran the LM head at a third
  // of the coalesced rate)
  constexpr int RB = NBW * 32, LPR = RB / 16, RPI = 64 / LPR, SLD = RB + 16;
  int8_t(&s_ab)[4][2][32 * SLD] = *reinterpret_cast<int8_t(*)[4][2][32 * SLD]>(s_ab_mem);
  // weight scales: lane (r, h) loads SQ dwords (2 fp16 block scales each) of row o0 + r, blocks [bw0 + 2 SQ h, +2 SQ)
  // (NBW = 2: both halves load the one dword), converted once per wave into LDS below
  constexpr int SQ = NBW >= 4 ? NBW / 4 : 1;
  uint32_t dwr[SQ];
  const __half* wdr = wd + (int64_t)min(o0 + r, a.O - 1) * nb + bw0 + (NBW >= 4 ? 2 * SQ * h : 0);
  float2 dx2[NBW / 2];
  {
    const int rr = lane / LPR, off = bw0 * 32 + 16 * (lane % LPR);
    if constexpr (ROLE == 2) {
      // consumer: weight rows and scales first (they do not depend on the producers), then the wait, then the act
      // rows of this split with sc1 loads (written by other workgroups of this launch, any XCD)
#pragma unroll
      for (int i = 0; i < NBW; ++i)
        A[i] = *reinterpret_cast<const i32x4_t*>(wq + (int64_t)min(o0 + RPI * i + rr, a.O - 1) * K + off);
#pragma unroll
      for (int q = 0; q < SQ; ++q) dwr[q] = *reinterpret_cast<const uint32_t*>(wdr + 2 * q);
      if (threadIdx.x == 0) {
        SpinDeadline dl;
        while ((int)__hip_atomic_load(fz.arr + ks * CNT_LINE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
               fz.tiles_per_split) {
          __builtin_amdgcn_s_sleep(1);
          if (dl.expired()) {
            __hip_atomic_store(fz.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
        if (__hip_atomic_fetch_add(fz.dep + ks * CNT_LINE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            (unsigned)fz.consumers - 1) {
          __hip_atomic_store(fz.arr + ks * CNT_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(fz.dep + ks * CNT_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      __syncthreads();
      const __amdgpu_buffer_rsrc_t rx = buf_rsrc(a.xq, a.M * K);
      const __amdgpu_buffer_rsrc_t rd = buf_rsrc(a.xd, a.M * nb * 4);
#pragma unroll
      for (int i = 0; i < NBW; ++i)
        B[i] = __builtin_bit_cast(i32x4_t, ld_sc1_f4(rx, (min(t0 + RPI * i + rr, a.M - 1) * K + off)));
#pragma unroll
      for (int q = 0; q < NBW / 2; ++q)
        dx2[q] = make_float2(ld_sc1_f1(rd, (t_b * nb + bw0 + 2 * q) * 4), ld_sc1_f1(rd, (t_b * nb + bw0 + 2 * q + 1) * 4));
    } else {
#pragma unroll
      for (int i = 0; i < NBW; ++i) {
        A[i] = *reinterpret_cast<const i32x4_t*>(wq + (int64_t)min(o0 + RPI * i + rr, a.O - 1) * K + off);
        B[i] = *reinterpret_cast<const i32x4_t*>(a.xq + (int64_t)min(t0 + RPI * i + rr, a.M - 1) * K + off);
      }
#pragma unroll
      for (int q = 0; q < SQ; ++q) dwr[q] = *reinterpret_cast<const uint32_t*>(wdr + 2 * q);
#pragma unroll
      for (int q = 0; q < NBW / 2; ++q) dx2[q] = *reinterpret_cast<const float2*>(a.xd + (int64_t)t_b * nb + bw0 + 2 * q);
    }
  }
  if constexpr (NRM) {
    float ss = 0.f;  // the producer's 32 tile partials in tile order
#pragma unroll
    for (int i = 0; i < 8; ++i) ss = (((ss + sv[i].x) + sv[i].y) + sv[i].z) + sv[i].w;
    const float rstd = 1.0f / sqrtf(ss / (float)K + a.eps);
#pragma unroll
    for (int q = 0; q < NBW / 2; ++q) {
      dx2[q].x = __half2float(__float2half_rn(rstd * dx2[q].x));
      dx2[q].y = __half2float(__float2half_rn(rstd * dx2[q].y));
    }
  }
  // this thread finalises regs [4 g, 4 g + 4) of lane l (token col, rows rrow): residual fetched now, used after the hop
  const int l = threadIdx.x & 63, g = threadIdx.x >> 6, col = l & 31, tok = t0 + col;
  // (regs 4 g .. 4 g + 3 of lane l are rows [8 g + 4 (l >> 5), +4) of token col: one 16-B piece; O % 32 == 0)
  float rv[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (EPI == 1) {
    const float4 r4 =
        *reinterpret_cast<const float4*>(a.res + (int64_t)min(tok, a.M - 1) * a.ldr + o0 + 8 * g + 4 * (l >> 5));
    rv[0] = r4.x; rv[1] = r4.y; rv[2] = r4.z; rv[3] = r4.w;
  }
#ifdef FA_GEMV_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  KSTAMP(1);
#endif
  float acc[16];
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) acc[reg] = 0.f;
  const i32x16_t zero = {};
  {  // rows -> LDS, then the MFMA layout: lane (r, h) -> row r, 16 B half h of block j
    const int rr = lane / LPR, cb = 16 * (lane % LPR);
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      *reinterpret_cast<i32x4_t*>(&s_ab[wave][0][(RPI * i + rr) * SLD + cb]) = A[i];
      *reinterpret_cast<i32x4_t*>(&s_ab[wave][1][(RPI * i + rr) * SLD + cb]) = B[i];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      A[j] = *reinterpret_cast<const i32x4_t*>(&s_ab[wave][0][r * SLD + 32 * j + 16 * h]);
      B[j] = *reinterpret_cast<const i32x4_t*>(&s_ab[wave][1][r * SLD + 32 * j + 16 * h]);
    }
  }
  // the wave's weight scales as f32 in LDS, [block][row], in its own staging image past the 4 KB that s_red takes
  // below (its fragments are in registers by now); lane (r, h) reads rows 8 g + 4 h + [0, 4) of block j as a float4
  static_assert(16 * 64 * 4 + NBW * 32 * 4 <= 2 * 32 * SLD, "k_gemm_q8_sk: scales must fit the wave's staging image");
  float4(&s_dw4)[NBW][8] = *reinterpret_cast<float4(*)[NBW][8]>(&s_ab[wave][0][16 * 64 * 4]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // fragment reads before the scale writes
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  {
    float* s_dw = reinterpret_cast<float*>(&s_dw4[0][0]);
#pragma unroll
    for (int q = 0; q < SQ; ++q) {
      const __half* hq = reinterpret_cast<const __half*>(&dwr[q]);
      const int j = (NBW >= 4 ? 2 * SQ * h : 0) + 2 * q;
      s_dw[j * 32 + r] = __half2float(hq[0]);
      s_dw[(j + 1) * 32 + r] = __half2float(hq[1]);
    }
  }
  f32x2_t acc2[8];  // regs 2 p, 2 p + 1
#pragma unroll
  for (int p = 0; p < 8; ++p) acc2[p] = f32x2_t{0.f, 0.f};
#pragma unroll
  for (int j = 0; j < NBW; ++j) {
    // (the 1.5 * 2^23 accumulator start of mfma_i8_f32 measured 1 % slower here)
    const i32x16_t D = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[j], B[j], zero, 0, 0, 0);
    const float dx = (j & 1) ? dx2[j >> 1].y : dx2[j >> 1].x;
    // acc += f32(dot) * (f32(d_w) * d_x): the scalar form's roundings, two values per instruction
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const float4 d4 = s_dw4[j][2 * gq + h];
      const f32x2_t lo = f32x2_t{d4.x, d4.y} * dx, hi = f32x2_t{d4.z, d4.w} * dx;
      acc2[2 * gq] = __builtin_elementwise_fma(f32x2_t{(float)D[4 * gq], (float)D[4 * gq + 1]}, lo, acc2[2 * gq]);
      acc2[2 * gq + 1] =
          __builtin_elementwise_fma(f32x2_t{(float)D[4 * gq + 2], (float)D[4 * gq + 3]}, hi, acc2[2 * gq + 1]);
    }
  }
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) acc[reg] = acc2[reg >> 1][reg & 1];
  // fixed-order reduction over the waves
  // s_red[w] in wave w's own staging image (written after the wave read its fragments, read after the barrier)
  static_assert(16 * 64 * 4 <= 2 * 32 * SLD, "k_gemm_q8_sk: wave partials must fit the wave's staging image");
  float(&s_red)[4][2 * 32 * SLD / 4] = *reinterpret_cast<float(*)[4][2 * 32 * SLD / 4]>(&s_ab[0][0][0]);
#define SRED(w, reg, l) s_red[w][(reg) * 64 + (l)]
  __shared__ float s_act[EPI >= 2 ? 32 : 1][33];  // tile [token][row]: SwiGLU q8_0 epilogue, lm_head argmax
  __shared__ int s_last;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) SRED(wave, reg, lane) = acc[reg];
  __syncthreads();
  KSTAMP(2);
  float y[4], y2[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int reg = 4 * g + q;
    if (EPI == 2) {
      y[q] = SRED(0, reg, l) + SRED(1, reg, l);
      y2[q] = SRED(2, reg, l) + SRED(3, reg, l);
    } else {
      y[q] = ((SRED(0, reg, l) + SRED(1, reg, l)) + SRED(2, reg, l)) + SRED(3, reg, l);
      y2[q] = 0.f;
    }
  }
  if (KSM > 1 && KS > 1) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const int tile = by * gdx + bx;
    float* base = a.kpart + (int64_t)tile * KS * (NS * 1024);
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(base, KS * NS * 1024 * 4);
    st_sc1_f4(f4v{y[0], y[1], y[2], y[3]}, rs, (ks * NS * 1024 + threadIdx.x * 4) * 4);
    if (EPI == 2) st_sc1_f4(f4v{y2[0], y2[1], y2[2], y2[3]}, rs, (ks * NS * 1024 + 1024 + threadIdx.x * 4) * 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    KSTAMP(3);
    if (threadIdx.x == 0)
      s_last = __hip_atomic_fetch_add(a.kcnt + tile * CNT_LINE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == KS - 1;
    __syncthreads();
    if (!s_last) return;
    KSTAMP(4);
    f4v pv[KSM], pv2[EPI == 2 ? KSM : 1];
#pragma unroll
    for (int k2 = 0; k2 < KSM; ++k2) {  // all in flight (clamped duplicates past KS are not summed)
      const int kk = min(k2, KS - 1);
      pv[k2] = ld_sc1_f4(rs, (kk * NS * 1024 + threadIdx.x * 4) * 4);
      if (EPI == 2) pv2[k2] = ld_sc1_f4(rs, (kk * NS * 1024 + 1024 + threadIdx.x * 4) * 4);
    }
    f4v sum = pv[0], sum2 = EPI == 2 ? pv2[0] : f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k2 = 1; k2 < KSM; ++k2) {
      if (k2 < KS) {
        sum += pv[k2];
        if (EPI == 2) sum2 += pv2[k2];
      }
    }
    y[0] = sum.x; y[1] = sum.y; y[2] = sum.z; y[3] = sum.w;
    y2[0] = sum2.x; y2[1] = sum2.y; y2[2] = sum2.z; y2[3] = sum2.w;
    if (threadIdx.x == 0) __hip_atomic_store(a.kcnt + tile * CNT_LINE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  float nv[4], ov[4];  // nv (EPI 1): the new residual values of this thread's 4 consecutive rows [8 g + 4 (l >> 5), +4)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rrow = 8 * g + 4 * (l >> 5) + q;
    nv[q] = rv[q] + y[q];
    float v = 0.f;
    if (EPI == 0 || EPI == 3) v = y[q];
    else if (EPI == 1) v = nv[q];
    else v = (y[q] / (1.0f + expf(-y[q]))) * y2[q];
    ov[q] = v;
    if (EPI == 2) s_act[col][rrow] = v;
    if (EPI == 3) s_act[col][rrow] = o0 + rrow < a.O ? v : -INFINITY;
  }
  if (tok < a.M && o0 + 8 * g + 4 * (l >> 5) < a.O)  // one 16-B store (O % 32 == 0)
    *reinterpret_cast<float4*>(a.out + (int64_t)tok * a.ldo + o0 + 8 * g + 4 * (l >> 5)) =
        make_float4(ov[0], ov[1], ov[2], ov[3]);
  if (EPI == 1 && a.ssp_out) {
    // the next NRM GEMM's input (its K = this GEMM's O = 1024): the tile is one q8_0 block of every token, so it
    // quantises z = x_new * qn_w (block scale d_z = amax / 127 left unrounded in f32, dout) into qout, and leaves the
    // rows' sum of squares (lane halves pair up, then the 4 waves in order) in ssp_out[tok][tile]
    __shared__ float s_ssq[4][32], s_am[4][32];
    const int rb = 8 * g + 4 * (l >> 5);
    float z[4], am = 0.f, ssq = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      ssq += nv[q] * nv[q];
      z[q] = nv[q] * a.qn_w[o0 + rb + q];
      am = fmaxf(am, fabsf(z[q]));
    }
    ssq += __shfl_xor(ssq, 32, 64);
    am = fmaxf(am, __shfl_xor(am, 32, 64));
    if (l < 32) {
      s_ssq[g][l] = ssq;
      s_am[g][l] = am;
    }
    __syncthreads();
    const float amx = fmaxf(fmaxf(s_am[0][col], s_am[1][col]), fmaxf(s_am[2][col], s_am[3][col]));
    const float d = amx / 127.0f;
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    const int b0 = (int)roundf(__fmul_rn(z[0], id)) & 0xFF, b1 = (int)roundf(__fmul_rn(z[1], id)) & 0xFF;
    const int b2 = (int)roundf(__fmul_rn(z[2], id)) & 0xFF, b3 = (int)roundf(__fmul_rn(z[3], id)) & 0xFF;
    if (tok < a.M) {
      *reinterpret_cast<int32_t*>(a.qout + (int64_t)tok * 1024 + o0 + rb) = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
      if (threadIdx.x < 32) {
        a.dout[(int64_t)tok * 32 + bx] = d;
        a.ssp_out[(int64_t)tok * 32 + bx] = ((s_ssq[0][col] + s_ssq[1][col]) + s_ssq[2][col]) + s_ssq[3][col];
      }
    }
  }
  if (EPI == 3) {
    __syncthreads();
    if (threadIdx.x < 32 && t0 + threadIdx.x < a.M) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      for (int rr = 0; rr < 32; ++rr) argmax_combine(bv, bi, s_act[threadIdx.x][rr], o0 + rr);
      a.pval[(int64_t)(t0 + threadIdx.x) * a.n_part + bx] = bv;
      a.pidx[(int64_t)(t0 + threadIdx.x) * a.n_part + bx] = bi;
    }
  }
  if (EPI == 2 && a.qout) {
    __syncthreads();
    swiglu_tile_q8<ROLE == 1>(s_act, a, t0, o0);
    if (ROLE == 1 && threadIdx.x < 64) {  // publish: the tile's sc1 stores drained, then counted for its down split
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (threadIdx.x == 0)
        __hip_atomic_fetch_add(fz.arr + (bx / fz.tiles_per_split) * CNT_LINE, 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  KSTAMP(5);
}
#undef SRED

template <int EPI, int NBW, int KSM, bool NRM = false>
__global__ __launch_bounds__(256) void k_gemm_q8_sk(GemvArgs a, int K, int KS) {
  if ((int)blockIdx.z >= KS) {  // L2 prefetch slabs (host: only with a.pf_q set)
    const int nxy = gridDim.x * gridDim.y;  // host: nxy % 8 == 0
    gemm_l2_prefetch(a, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * (blockIdx.z - KS)), nxy * (gridDim.z - KS));
    return;
  }
  constexpr int SLD = NBW * 32 + 16;
  __shared__ __attribute__((aligned(16))) int8_t s_ab[4 * 2 * 32 * SLD];
  sk_tile<EPI, NBW, KSM, NRM, 0>(a, K, KS, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.x, s_ab, SkFuse{});
}

// Batched LM head (5-32 tokens, K = 1024, the 151936 vocabulary rows): the split-K block kernel's tile arithmetic
// (4 waves x 8 q8_0 blocks of K, fixed-order wave sum, argmax partial per 32-row tile) in a persistent loop over
// tiles, 3 blocks per CU. A block loads its waves' activation blocks and scales (NRM: rstd applied) once for every
// tile. Weight rows are fetched coalesced (each load instruction 4 rows x 256 contiguous B; 16 B per lane from 32
// rows was the old kernel's pattern) and turned into the MFMA fragment layout through LDS; the next tile's loads go out
// before the current tile's math; scales are staged as f32 (no per-product conversion); logits leave through LDS as
// 128-B token rows. scripts/ubench/gemm_batch (M = 32, graph-replayed): 133 -> 44.8 us per launch (3.7 TB/s).
constexpr int LMB_PER_CU = 3;                 // 156 VGPRs, 43 KB of LDS per block
constexpr int LMB_BLOCKS = 256 * LMB_PER_CU;  // every block resident

template <bool NRM>
__global__ __launch_bounds__(256, LMB_PER_CU) void k_lm_head_b(GemvArgs a) {
  constexpr int K = 1024, NB = K / 32, NBW = 8, WLD = 256 + 16;  // LDS weight rows: the wave's 256 B + 16 B pad
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int bw0 = wave * NBW;
  const int t_b = min(r, a.M - 1);
  const int n_tiles = (a.O + 31) >> 5;
  __shared__ __attribute__((aligned(16))) int8_t s_w[4][32 * WLD];  // per wave: its K quarter of the tile's 32 rows
  __shared__ __attribute__((aligned(16))) float s_sc[4][NBW][64];  // per wave: [block j][lane -> row lane & 31], f32
  // s_red[wave] aliases the wave's own weight image: written after the wave has read its A fragments, read between
  // the two barriers, and the image is rewritten only after the second barrier
  static_assert(16 * 64 * 4 <= 32 * WLD, "k_lm_head_b: wave partials must fit the wave's weight image");
  __shared__ float s_act[32][33];  // [token][row]
  // a tile's loads, coalesced: instruction i reads rows 4 i .. 4 i + 3, 256 contiguous bytes each (lanes 16 q .. 16 q
  // + 15 -> row 4 i + q); the scale slab: lane l -> row l & 31, the wave's 8 fp16 scales
  auto load_tile = [&](int tile, i32x4_t (&W)[NBW], uint4& sl) {
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      const int row = min(tile * 32 + 4 * i + (lane >> 4), a.O - 1);
      W[i] = __builtin_nontemporal_load(
          reinterpret_cast<const i32x4_t*>(a.wq + (int64_t)row * K + bw0 * 32 + 16 * (lane & 15)));
    }
    sl = *reinterpret_cast<const uint4*>(a.wd + (int64_t)min(tile * 32 + r, a.O - 1) * NB + bw0);
  };
  i32x4_t W[NBW];
  uint4 sl;
  int tile = blockIdx.x;
  if (tile < n_tiles) load_tile(tile, W, sl);
  float4 sv[NRM ? 8 : 1];
  if constexpr (NRM) {
#pragma unroll
    for (int i = 0; i < 8; ++i) sv[i] = *reinterpret_cast<const float4*>(a.ssp + (int64_t)t_b * 32 + 4 * i);
  }
  i32x4_t B[NBW];
  const int8_t* xb = a.xq + (int64_t)t_b * K + 16 * h + bw0 * 32;
#pragma unroll
  for (int j = 0; j < NBW; ++j) B[j] = *reinterpret_cast<const i32x4_t*>(xb + j * 32);
  float dx[NBW];
#pragma unroll
  for (int q = 0; q < NBW / 2; ++q) {
    const float2 v = *reinterpret_cast<const float2*>(a.xd + (int64_t)t_b * NB + bw0 + 2 * q);
    dx[2 * q] = v.x;
    dx[2 * q + 1] = v.y;
  }
  if constexpr (NRM) {  // as k_gemm_q8_sk<NRM>: the producer's 32 partials in tile order, f16 block scales
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) ss = (((ss + sv[i].x) + sv[i].y) + sv[i].z) + sv[i].w;
    const float rstd = 1.0f / sqrtf(ss / (float)K + a.eps);
#pragma unroll
    for (int j = 0; j < NBW; ++j) dx[j] = __half2float(__float2half_rn(rstd * dx[j]));
  }
  const int l = lane, g = wave, col = l & 31;
  const i32x16_t zero = {};
  // the activation blocks are waited for here, once: inside the loop every vmcnt wait then counts only weight loads
  // (a pending pre-loop load would make each MFMA drain the next tile's prefetch)
#pragma unroll
  for (int j = 0; j < NBW; ++j) asm volatile("" ::"v"(B[j]));
  int8_t* sw = s_w[wave];
  for (; tile < n_tiles; tile += gridDim.x) {
    const int o0 = tile * 32;
    // the landed tile -> LDS (every lane, no branch), then the next tile's loads go out before any math
#pragma unroll
    for (int i = 0; i < NBW; ++i)
      *reinterpret_cast<i32x4_t*>(sw + (4 * i + (lane >> 4)) * WLD + 16 * (lane & 15)) = W[i];
    {  // row r's 8 scales as f32, transposed so a fragment's 16 rows are 4 x 16-B reads (every lane: no branch)
      const uint32_t pr[4] = {sl.x, sl.y, sl.z, sl.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const __half* hp = reinterpret_cast<const __half*>(&pr[k]);
        s_sc[wave][2 * k][lane] = __half2float(hp[0]);
        s_sc[wave][2 * k + 1][lane] = __half2float(hp[1]);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (tile + (int)gridDim.x < n_tiles) load_tile(tile + gridDim.x, W, sl);
    f32x2_t acc2[8];  // regs 2 p, 2 p + 1
#pragma unroll
    for (int p = 0; p < 8; ++p) acc2[p] = f32x2_t{0.f, 0.f};
#pragma unroll
    for (int jp = 0; jp < NBW / 2; ++jp) {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int j = 2 * jp + jj;
        const i32x4_t Aj = *reinterpret_cast<const i32x4_t*>(sw + r * WLD + 32 * j + 16 * h);  // MFMA layout
        const i32x16_t D = __builtin_amdgcn_mfma_i32_32x32x32_i8(Aj, B[j], zero, 0, 0, 0);
        // block j's scales of rows (reg & 3) + 8 (reg >> 2) + 4 h (wave-half broadcast reads); acc += f32(dot) *
        // (d_w * d_x) with the scalar form's roundings, two values per instruction (v_pk_mul_f32 / v_pk_fma_f32)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(&s_sc[wave][j][8 * q + 4 * h]);
          const f32x2_t lo = f32x2_t{v.x, v.y} * dx[j], hi = f32x2_t{v.z, v.w} * dx[j];
          acc2[2 * q] = __builtin_elementwise_fma(f32x2_t{(float)D[4 * q], (float)D[4 * q + 1]}, lo, acc2[2 * q]);
          acc2[2 * q + 1] =
              __builtin_elementwise_fma(f32x2_t{(float)D[4 * q + 2], (float)D[4 * q + 3]}, hi, acc2[2 * q + 1]);
        }
      }
    }
#pragma unroll
    for (int reg = 0; reg < 16; ++reg)
      *reinterpret_cast<float*>(s_w[wave] + (reg * 64 + lane) * 4) = acc2[reg >> 1][reg & 1];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int reg = 4 * g + q;
      auto red = [&](int w) { return *reinterpret_cast<const float*>(s_w[w] + (reg * 64 + l) * 4); };
      const float y = ((red(0) + red(1)) + red(2)) + red(3);
      const int rrow = (reg & 3) + 8 * (reg >> 2) + 4 * (l >> 5);
      s_act[col][rrow] = o0 + rrow < a.O ? y : -INFINITY;
    }
    __syncthreads();
    {  // thread t: token t >> 3, rows [4 (t & 7), +4): logits as 16-B pieces of the token's 128-B row; argmax over 8 lanes
      const int tk = threadIdx.x >> 3, rq = (threadIdx.x & 7) * 4;
      const float4 v = make_float4(s_act[tk][rq], s_act[tk][rq + 1], s_act[tk][rq + 2], s_act[tk][rq + 3]);
      if (tk < a.M && o0 + rq < a.O) *reinterpret_cast<float4*>(a.out + (int64_t)tk * a.ldo + o0 + rq) = v;
      float bv = v.x;
      int bi = o0 + rq;
      argmax_combine(bv, bi, v.y, o0 + rq + 1);
      argmax_combine(bv, bi, v.z, o0 + rq + 2);
      argmax_combine(bv, bi, v.w, o0 + rq + 3);
#pragma unroll
      for (int off = 1; off < 8; off <<= 1) {
        const float ov = __shfl_xor(bv, off, 64);
        const int oi = __shfl_xor(bi, off, 64);
        argmax_combine(bv, bi, ov, oi);
      }
      if ((threadIdx.x & 7) == 0 && tk < a.M) {
        a.pval[(int64_t)tk * a.n_part + tile] = bv;
        a.pidx[(int64_t)tk * a.n_part + tile] = bi;
      }
    }
  }
}

// Small-batch LM head (2-8 tokens, K = 1024, fused rmsnorm + q8_0 prologue): the persistent tile loop of k_lm_head_b
// with the operands swapped (A = the block's token rows from LDS, held in registers for the whole launch; B = the
// tile's weight rows through the LDS image), so a lane's D registers 0-3 are tokens 4 h .. 4 h + 3 of weight row
// lane & 31 and only those four are scaled. Every logit is BIT-IDENTICAL to the batch-1 GEMV's (k_gemv_q8, EPI 3):
// the same prologue (norm_quant_block_regs per token), the same per-block product f32(dot) * (f32(d_w) * d_x) and the
// same balanced tree over the 32 blocks in block order that wave_sum forms (pairs, quads, eights inside a wave's 8
// blocks, then (w0 + w1) + (w2 + w3) across the waves; the GEMV's leaves pass through one + 0.0f, so a pair of -0
// products sums to +0 here too); no contraction into fma. Argmax partial per (token, 32-row tile), as k_lm_head_b.
// Replaces the 3-6 token GEMV (one block row for every token: 63.8 us per launch at 6 tokens) and the two-row-pass
// 2-token GEMV.
constexpr int LMS_PER_CU = 3;
constexpr int LMS_BLOCKS = 256 * LMS_PER_CU;
constexpr int LMS_STEPS = 8;  // tiles per block at most (151936 rows: 4748 tiles over 768 blocks = 7)
int g_lm_head_s = 1;  // FUNASR_LM_HEAD_S: 0 the GEMV forms; 1 k_lm_head_s<1>; 2 k_lm_head_s<2> (A/B)
int g_lm_grid = 0;  // FUNASR_LM_GRID: blocks of the persistent LM-head launches (0: every block resident; A/B)
int g_lm_head_s1 = 0;  // FUNASR_LM_HEAD_S1: the batch-1 fused decode's LM head on k_lm_head_s too (1 / 2 = PF; A/B)

// PF = weight tiles in flight per wave (1: the next tile's loads go out when the current one lands; 2: two ahead, in
// registers, clamped to the last tile so every load is unconditional). PS (M = 1, the fused decode's LM head): the row
// is first completed as x + psum[0] + ... + psum[7], as k_gemv_q8<PS> does.
template <int PF, bool PS>
__global__ __launch_bounds__(256, LMS_PER_CU) void k_lm_head_s(GemvArgs a) {
#pragma clang fp contract(off)
  constexpr int K = 1024, NB = K / 32, NBW = 8, WLD = 256 + 16, PERB = 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, n = lane & 31, h = lane >> 5;
  const int bw0 = wave * NBW;
  const int M = PS ? 1 : a.M;  // 1 .. 8 (host-checked)
  const int n_tiles = (a.O + 31) >> 5;
  __shared__ __attribute__((aligned(16))) int8_t s_w[4][32 * WLD];  // per wave: its K quarter of the tile's 32 rows
  // the token rows (prologue) and, once they are in registers, the per-tile wave partials [parity][wave][reg][lane]
  __shared__ __attribute__((aligned(16))) int8_t s_qr[8 * K];
  __shared__ __attribute__((aligned(16))) float s_dT[NB][8];  // [block][token]: d_x
  __shared__ float s_d[8 * NB];
  __shared__ float s_nred[8][4];
  // the landed scales pass through LDS like the weights (a register copy of a loop-carried load would make the loop
  // latch wait for every load in flight)
  __shared__ __attribute__((aligned(16))) uint4 s_sl[4][64];
  auto load_tile = [&](int tile, i32x4_t (&W)[NBW], uint4& sl) {
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      const int row = min(tile * 32 + 4 * i + (lane >> 4), a.O - 1);
      W[i] = __builtin_nontemporal_load(
          reinterpret_cast<const i32x4_t*>(a.wq + (int64_t)row * K + bw0 * 32 + 16 * (lane & 15)));
    }
    sl = *reinterpret_cast<const uint4*>(a.wd + (int64_t)min(tile * 32 + n, a.O - 1) * NB + bw0);
  };
  // activations first (the whole block waits on them), then the first weight tile(s), then the prologue math
  constexpr int MX = PS ? 1 : 8;
  float xv[MX][PERB], xw[PERB];
  float pv[PS ? FUSED_PARTS : 1][PERB];
  if constexpr (PS) {
#pragma unroll
    for (int g = 0; g < FUSED_PARTS; ++g) {
      const float4 f = *reinterpret_cast<const float4*>(a.psum + g * 1024 + threadIdx.x * PERB);
      pv[g][0] = f.x; pv[g][1] = f.y; pv[g][2] = f.z; pv[g][3] = f.w;
    }
  }
#pragma unroll
  for (int m = 0; m < MX; ++m) {
    const float4 f = *reinterpret_cast<const float4*>(a.x + (int64_t)min(m, M - 1) * a.ldx + threadIdx.x * PERB);
    xv[m][0] = f.x; xv[m][1] = f.y; xv[m][2] = f.z; xv[m][3] = f.w;
  }
  {
    const float4 g = *reinterpret_cast<const float4*>((a.norm_w ? a.norm_w : a.x) + threadIdx.x * PERB);
    xw[0] = g.x; xw[1] = g.y; xw[2] = g.z; xw[3] = g.w;
  }
  __builtin_amdgcn_sched_barrier(0);
  i32x4_t W0[NBW], W1[NBW];
  uint4 sl0, sl1;
  int tile = blockIdx.x;  // < n_tiles: the host launches at most one block per tile
  load_tile(tile, W0, sl0);  // (no branch: the wait-count pass would drain these loads at the join)
  if constexpr (PF == 2) load_tile(tile + (int)gridDim.x < n_tiles ? tile + (int)gridDim.x : tile, W1, sl1);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (PS) {
#pragma unroll
    for (int j = 0; j < PERB; ++j) {
      float v = xv[0][j];
#pragma unroll
      for (int g = 0; g < FUSED_PARTS; ++g) v = v + pv[g][j];
      xv[0][j] = v;
    }
    if (a.xsum && blockIdx.x == 0)
      *reinterpret_cast<float4*>(a.xsum + threadIdx.x * PERB) = make_float4(xv[0][0], xv[0][1], xv[0][2], xv[0][3]);
  }
#pragma unroll
  for (int m = 0; m < MX; ++m) {
    if (m < M) {  // block-uniform
      float v[PERB];
#pragma unroll
      for (int j = 0; j < PERB; ++j) v[j] = xv[m][j];
      norm_quant_block_regs<PERB>(v, xw, a.norm_w != nullptr, a.eps, K, s_qr + m * K, s_d + m * NB, s_nred[m]);
    }
  }
  __syncthreads();
  i32x4_t A[NBW];  // lane: token row min(n, M - 1) (rows past M: a copy, never stored), K bytes 16 h of each block
  {
    const int8_t* xb = s_qr + min(n, M - 1) * K + bw0 * 32 + 16 * h;
#pragma unroll
    for (int j = 0; j < NBW; ++j) A[j] = *reinterpret_cast<const i32x4_t*>(xb + j * 32);
    const int b = threadIdx.x >> 3, t = threadIdx.x & 7;
    s_dT[b][t] = s_d[min(t, M - 1) * NB + b];
  }
  __syncthreads();  // s_qr becomes the partials buffer
  float* s_red = reinterpret_cast<float*>(s_qr);  // [2][4][4][64]
  int8_t* sw = s_w[wave];
  const i32x16_t zero = {};
  auto step = [&](int tile, int par, i32x4_t (&W)[NBW], uint4& sl) {
    const int o0 = tile * 32;
#pragma unroll
    for (int i = 0; i < NBW; ++i)
      *reinterpret_cast<i32x4_t*>(sw + (4 * i + (lane >> 4)) * WLD + 16 * (lane & 15)) = W[i];
    s_sl[wave][lane] = sl;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the tile PF steps ahead, or (past the end) this tile again: unconditional loads keep the wait counts exact
    const int nxt = tile + PF * (int)gridDim.x;
    load_tile(nxt < n_tiles ? nxt : tile, W, sl);
    const uint4 cs = s_sl[wave][lane];
    const uint32_t pr[4] = {cs.x, cs.y, cs.z, cs.w};
    f32x2_t t1[2], t2[2], t3[2];  // tree levels (pairs, quads, the wave's eight blocks), tokens (0, 1) / (2, 3)
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      const i32x4_t Bj = *reinterpret_cast<const i32x4_t*>(sw + n * WLD + 32 * j + 16 * h);
      const i32x16_t D = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[j], Bj, zero, 0, 0, 0);
      const float dw = __half2float(reinterpret_cast<const __half*>(&pr[j >> 1])[j & 1]);
      const float4 dx = *reinterpret_cast<const float4*>(&s_dT[bw0 + j][4 * h]);
      f32x2_t b[2];
      b[0] = f32x2_t{(float)D[0], (float)D[1]} * (f32x2_t{dw, dw} * f32x2_t{dx.x, dx.y});
      b[1] = f32x2_t{(float)D[2], (float)D[3]} * (f32x2_t{dw, dw} * f32x2_t{dx.z, dx.w});
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if ((j & 1) == 0) {
          t1[q] = b[q];
        } else {
          const f32x2_t p = (t1[q] + b[q]) + f32x2_t{0.f, 0.f};
          if ((j & 3) == 1) {
            t2[q] = p;
          } else {
            const f32x2_t p2 = t2[q] + p;
            if (j == 3) t3[q] = p2;
            else t3[q] = t3[q] + p2;
          }
        }
      }
    }
    float* rp = s_red + ((par * 4 + wave) * 4) * 64;
    rp[0 * 64 + lane] = t3[0][0];
    rp[1 * 64 + lane] = t3[0][1];
    rp[2 * 64 + lane] = t3[1][0];
    rp[3 * 64 + lane] = t3[1][1];
    __syncthreads();
    {  // thread: token t = tid >> 5, row o0 + (tid & 31): (w0 + w1) + (w2 + w3), logit out, argmax over the 32 rows
      const int t = threadIdx.x >> 5, rr = threadIdx.x & 31, g = t & 3, ln = rr + 32 * (t >> 2);
      const float* r0 = s_red + (par * 4) * 4 * 64 + g * 64 + ln;
      const float y = (r0[0] + r0[256]) + (r0[512] + r0[768]);
      const int row = o0 + rr;
      if (t < M && row < a.O) a.out[(int64_t)t * a.ldo + row] = y;
      float bv = row < a.O ? y : -INFINITY;
      int bi = row;
#pragma unroll
      for (int off = 1; off < 32; off <<= 1) {
        const float ov = __shfl_xor(bv, off, 64);
        const int oi = __shfl_xor(bi, off, 64);
        argmax_combine(bv, bi, ov, oi);
      }
      if (rr == 0 && t < M) {
        a.pval[(int64_t)t * a.n_part + tile] = bv;
        a.pidx[(int64_t)t * a.n_part + tile] = bi;
      }
    }
  };
  // at most LMS_STEPS tiles per block (host-checked), unrolled: with a loop back-edge the wait-count pass merges the
  // in-flight loads of both register sets and waits for all of them at the loop head
#pragma unroll
  for (int it = 0; it < LMS_STEPS; ++it) {
    const int tl = tile + it * (int)gridDim.x;
    if (tl >= n_tiles) break;
    if (PF == 1 || (it & 1) == 0) step(tl, it & 1, W0, sl0);
    else step(tl, it & 1, W1, sl1);
  }
}

// Same GEMM with K split over the NW waves of ONE block instead of over blocks: no cross-block split-K hop (on
// this chip an in-launch hand-off costs about a kernel boundary: scripts/ubench/edge_chain.hip), and every wave
// issues ALL its loads (NBW q8_0 blocks of weights and activations, their scales) before its MFMAs, so a tile
// costs one memory round trip. Waves are reduced in LDS in fixed order (deterministic). SwiGLU: the first half
// of the waves take the gate matrix, the second half the up matrix. NW = 16 (1024 threads) for the few-tile
// shapes (o and down at batch 32: 32 tiles) so each CU keeps twice the loads in flight.
// NIN (row-local prefill, round 6; the batched decode's NRM form, k_gemm_q8_sk): the input rows come from the previous
// residual GEMM's epilogue (EPI 1 with ssp_out below), which quantised z = x * norm_w per 32-block and left per-token
// sum-of-squares partials; this GEMM applies rstd = 1/sqrtf(sum/K + eps) to the block scales, so the two k_prep_q8
// launches per layer disappear.
template <int EPI, int NW, int NBW, bool NIN = false>
__global__ __launch_bounds__(NW * 64) void k_gemm_q8_kw(GemvArgs a, int K) {
  static_assert(NBW % 2 == 0 && (NW == 8 || (NW == 16 && EPI != 2)), "k_gemm_q8_kw: shapes");
  static_assert(!NIN || EPI == 0 || EPI == 2, "k_gemm_q8_kw: normalised inputs feed q|k|v and gate|up");
  constexpr int NWM = EPI == 2 ? NW / 2 : NW;  // waves per weight matrix
  const int nb = K >> 5;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int o0 = blockIdx.x * 32, t0 = blockIdx.y * 32;
  const bool upw = EPI == 2 && wave >= NWM;
  const int b0 = (EPI == 2 ? wave % NWM : wave) * NBW;  // this wave's q8_0 blocks [b0, b0 + NBW) (host: NBW*NWM == nb)
  const int8_t* wq = upw ? a.wq2 : a.wq;
  const __half* wd = upw ? a.wd2 : a.wd;
  const int8_t* wa = wq + (int64_t)min(o0 + r, a.O - 1) * K + 16 * h + b0 * 32;
  const int t_b = min(t0 + r, a.M - 1);
  const int8_t* xb = a.xq + (int64_t)t_b * K + 16 * h + b0 * 32;
  GSTAMP(0);
  float4 sv[NIN ? 8 : 1];
  if constexpr (NIN) {  // this lane's token's 32 partials, issued first
#pragma unroll
    for (int i = 0; i < 8; ++i) sv[i] = *reinterpret_cast<const float4*>(a.ssp + (int64_t)t_b * 32 + 4 * i);
  }
  i32x4_t A[NBW], B[NBW];
#pragma unroll
  for (int j = 0; j < NBW; ++j) {
    A[j] = *reinterpret_cast<const i32x4_t*>(wa + j * 32);
    B[j] = *reinterpret_cast<const i32x4_t*>(xb + j * 32);
  }
  // weight scales: lane (r, h) loads NBW / 4 dwords (2 fp16 block scales each) of row o0 + r, blocks
  // [b0 + h NBW / 2, +NBW / 2), instead of every lane loading its 16 rows' scales
  constexpr int NQ = NBW / 4;
  uint32_t dwr[NQ];
  {
    const __half* wr = wd + (int64_t)min(o0 + r, a.O - 1) * nb + b0 + h * (NBW / 2);
#pragma unroll
    for (int q = 0; q < NQ; ++q) dwr[q] = *reinterpret_cast<const uint32_t*>(wr + 2 * q);
  }
  float2 dx2[NBW / 2];
#pragma unroll
  for (int q = 0; q < NBW / 2; ++q) dx2[q] = *reinterpret_cast<const float2*>(a.xd + (int64_t)t_b * nb + b0 + 2 * q);
  __builtin_amdgcn_sched_barrier(0);  // every load issued before any use (hipcc would hoist MFMAs between them)
  if constexpr (NIN) {  // k_gemm_q8_sk's NRM arithmetic: the producer's 32 tile partials in tile order
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) ss = (((ss + sv[i].x) + sv[i].y) + sv[i].z) + sv[i].w;
    const float rstd = 1.0f / sqrtf(ss / (float)K + a.eps);
#pragma unroll
    for (int q = 0; q < NBW / 2; ++q) {
      dx2[q].x = __half2float(__float2half_rn(rstd * dx2[q].x));
      dx2[q].y = __half2float(__float2half_rn(rstd * dx2[q].y));
    }
  }
  // the wave's scales as f32 in LDS, [block][row]: each lane then reads its 16 rows' (rows 8 g + 4 h + [0, 4)) of a
  // block as 4 float4, converted once per wave instead of once per lane (wave-private rows: no block barrier)
  __shared__ float4 s_dw4[NW][NBW][8];
  float* s_dw = reinterpret_cast<float*>(s_dw4[wave]);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const __half* hq = reinterpret_cast<const __half*>(&dwr[q]);
    const int j = h * (NBW / 2) + 2 * q;
    s_dw[j * 32 + r] = __half2float(hq[0]);
    s_dw[(j + 1) * 32 + r] = __half2float(hq[1]);
  }
  __builtin_amdgcn_sched_barrier(0);
  f32x2_t acc[8];  // regs 2 p, 2 p + 1
#pragma unroll
  for (int p = 0; p < 8; ++p) acc[p] = f32x2_t{0.f, 0.f};
  const i32x16_t zero = {};
#ifdef FA_GEMV_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  GSTAMP(1);
#endif
#pragma unroll
  for (int j = 0; j < NBW; ++j) {
    const i32x16_t D = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[j], B[j], zero, 0, 0, 0);  // (1.5 * 2^23 start: no gain)
    const float dx = (j & 1) ? dx2[j >> 1].y : dx2[j >> 1].x;
    // acc += f32(dot) * (f32(d_w) * d_x): one rounding per product and per fused add, as the scalar form, two
    // values per instruction (v_pk_mul_f32 / v_pk_fma_f32)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 d4 = s_dw4[wave][j][2 * g + h];
      const f32x2_t lo = f32x2_t{d4.x, d4.y} * dx, hi = f32x2_t{d4.z, d4.w} * dx;
      acc[2 * g] = __builtin_elementwise_fma(f32x2_t{(float)D[4 * g], (float)D[4 * g + 1]}, lo, acc[2 * g]);
      acc[2 * g + 1] = __builtin_elementwise_fma(f32x2_t{(float)D[4 * g + 2], (float)D[4 * g + 3]}, hi, acc[2 * g + 1]);
    }
  }
  // fixed-order reduction over the waves of each matrix (NW = 16: waves w and w + 8 first pair up); thread t then
  // finalises regs [RPT (t>>6), +RPT) of lane t&63
  constexpr int NR = NW == 16 ? 8 : NW;  // partial tiles left for the final sum
  constexpr int NRM = EPI == 2 ? NR / 2 : NR;
  constexpr int RPT = 16 / NW;
  __shared__ float s_red[NR][16][64];
  __shared__ float s_act[EPI >= 1 ? 32 : 1][33];  // tile [token][row]: SwiGLU / NRM q8_0 epilogues, lm_head argmax
  if (NW == 16) {
    if (wave >= 8) {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) s_red[wave - 8][reg][lane] = acc[reg >> 1][reg & 1];
    }
    __syncthreads();
    if (wave < 8) {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) acc[reg >> 1][reg & 1] += s_red[wave][reg][lane];
    }
    __syncthreads();
  }
  if (wave < NR) {
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) s_red[wave][reg][lane] = acc[reg >> 1][reg & 1];
  }
  __syncthreads();
  GSTAMP(2);
  const int l = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int col = l & 31, tok = t0 + col;
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int reg = RPT * g + q;
    float y = 0.f, y2 = 0.f;
#pragma unroll
    for (int w = 0; w < NRM; ++w) y += s_red[w][reg][l];
    if (EPI == 2) {
#pragma unroll
      for (int w = NRM; w < NR; ++w) y2 += s_red[w][reg][l];
    }
    const int rrow = (reg & 3) + 8 * (reg >> 2) + 4 * (l >> 5), row = o0 + rrow;
    float v = 0.f;
    if (row < a.O && tok < a.M) {
      float* op = a.out + (int64_t)tok * a.ldo + row;
      if (EPI == 0 || EPI == 3) *op = v = y;
      else if (EPI == 1) *op = v = a.res[(int64_t)tok * a.ldr + row] + y;
      else *op = v = (y / (1.0f + expf(-y))) * y2;
    }
    if (EPI == 1 || EPI == 2) s_act[col][rrow] = v;
    if (EPI == 3) s_act[col][rrow] = row < a.O ? v : -INFINITY;
  }
  if (EPI == 3) {
    // lm_head: per-token argmax partial of this 32-row tile (first occurrence on ties, rows ascending)
    __syncthreads();
    if (threadIdx.x < 32 && t0 + threadIdx.x < a.M) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      for (int rr = 0; rr < 32; ++rr) argmax_combine(bv, bi, s_act[threadIdx.x][rr], o0 + rr);
      a.pval[(int64_t)(t0 + threadIdx.x) * a.n_part + blockIdx.x] = bv;
      a.pidx[(int64_t)(t0 + threadIdx.x) * a.n_part + blockIdx.x] = bi;
    }
  }
  if (EPI == 2 && a.qout) {
    __syncthreads();
    swiglu_tile_q8(s_act, a, t0, o0);
  }
  if (EPI == 1 && a.ssp_out) {
    // the next NRM GEMM's input (its K = this GEMM's O = 1024): the tile is one q8_0 block of every token; threads
    // 0..63 (token t & 31, rows [16 (t >> 5), +16)) quantise z = x_new * qn_w (block scale amax / 127, unrounded f32)
    // and leave the rows' sum of squares (the two halves added) in ssp_out[tok][tile]
    __syncthreads();
    if (threadIdx.x < 64) {
      const int tk = threadIdx.x & 31, hh = threadIdx.x >> 5, tokq = t0 + tk;
      float z[16], am = 0.f, ssq = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float xv = s_act[tk][16 * hh + i];
        ssq += xv * xv;
        z[i] = xv * a.qn_w[o0 + 16 * hh + i];
        am = fmaxf(am, fabsf(z[i]));
      }
      ssq += __shfl_xor(ssq, 32, 64);
      am = fmaxf(am, __shfl_xor(am, 32, 64));
      const float d = am / 127.0f;
      const float id = d != 0.0f ? 1.0f / d : 0.0f;
      int32_t pk[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q0 = (int)roundf(__fmul_rn(z[4 * j], id)) & 0xFF, q1 = (int)roundf(__fmul_rn(z[4 * j + 1], id)) & 0xFF;
        const int q2 = (int)roundf(__fmul_rn(z[4 * j + 2], id)) & 0xFF, q3 = (int)roundf(__fmul_rn(z[4 * j + 3], id)) & 0xFF;
        pk[j] = q0 | (q1 << 8) | (q2 << 16) | (q3 << 24);
      }
      if (tokq < a.M) {
        *reinterpret_cast<int4*>(a.qout + (int64_t)tokq * 1024 + o0 + 16 * hh) = make_int4(pk[0], pk[1], pk[2], pk[3]);
        if (hh == 0) {
          a.dout[(int64_t)tokq * 32 + blockIdx.x] = d;
          a.ssp_out[(int64_t)tokq * 32 + blockIdx.x] = ssq;
        }
      }
    }
  }
  GSTAMP(3);
}

template <int EPI, int NW, int NBW>
static void launch_gemm_kw(const GemvArgs& a, int K, hipStream_t s) {
  if (a.ssp)
    hipLaunchKernelGGL((k_gemm_q8_kw<EPI == 1 ? 0 : EPI, NW, NBW, true>), dim3(cdiv(a.O, 32), cdiv(a.M, 32)),
                       dim3(NW * 64), 0, s, a, K);
  else
    hipLaunchKernelGGL((k_gemm_q8_kw<EPI, NW, NBW>), dim3(cdiv(a.O, 32), cdiv(a.M, 32)), dim3(NW * 64), 0, s, a, K);
}

// K-in-block GEMM for the shapes it is instantiated for; false otherwise. 8 waves (16 measured slower on the
// few-tile o / down shapes at batch 32: 10.2 / 18.3 vs 8.8 / 14.6 us, register-capped at 128 VGPRs);
// q8_0 blocks per wave NBW = blocks of K per wave.
static bool gemm_q8_kw(const GemvArgs& a, int K, int epi, hipStream_t s, bool force = false) {
  constexpr int nw = 8;
  // batched decode (a few hundred tiles or less) measured 2.6 % faster per step on the split-K block kernel
  // (1.974 vs 2.027 ms at batch 32, same box); prefill-sized grids take this one (row-local prefill: always)
  if (!force && g_gemm_q8_kw < 2 && (int64_t)cdiv(a.O, 32) * cdiv(a.M, 32) < 256) return false;
  const int nb = (K / 32) * (epi == 2 ? 2 : 1);
  if (nb % nw) return false;
  switch (epi * 100 + nb / nw) {
    case 4: launch_gemm_kw<0, nw, 4>(a, K, s); return true;
    case 8: launch_gemm_kw<0, nw, 8>(a, K, s); return true;
    case 12: launch_gemm_kw<0, nw, 12>(a, K, s); return true;
    case 104: launch_gemm_kw<1, nw, 4>(a, K, s); return true;
    case 108: launch_gemm_kw<1, nw, 8>(a, K, s); return true;
    case 112: launch_gemm_kw<1, nw, 12>(a, K, s); return true;
    case 208: launch_gemm_kw<2, nw, 8>(a, K, s); return true;
    default: return false;
  }
}

// ------------------------------------------------------------------------------------------------
// Tiled q8_0 x q8_0 GEMM for large token counts (multi-sequence prefill, M >= g_gemm_t_min_m): 128 weight rows x
// 128 tokens per block, 2x2 waves each owning 2x2 tiles of v_mfma_i32_32x32x32_i8 (the exact per-block integer dot),
// K staged 64 (two q8_0 blocks) at a time through double-buffered LDS: every weight / activation byte a block reads
// feeds 128 tokens / rows (the K-in-block kernel re-reads both per 32x32 tile: 4x the bytes per MAC). The f32 scaling
// per block (acc += f32(dot) * (f32(d_w) * d_x), ggml_vec_dot_q8_0_q8_0) is the VALU work that bounds it. SwiGLU
// (EPI 2) runs gate and up in the same waves and quantises the act rows for the down GEMM in registers (a token's
// 32 rows of a tile are lanes l and l + 32). LDS rows of 64 B + 16 B: 16-B operand reads of 16 rows start in distinct
// 4-bank groups.
constexpr int QT_LD = 80;  // bytes per staged row
template <int EPI>
struct QTile {
  static constexpr int NM = EPI == 2 ? 2 : 1;           // weight matrices (gate, up)
  static constexpr int W = 128 * QT_LD;                 // bytes per staged weight / activation tile
  static constexpr int STAGE = (NM + 1) * W + (NM + 1) * 128 * 2 * 4;  // + f32 scales [m][blk][128]
  static constexpr int BYTES = 2 * STAGE;
};

// The weight scales stay raw fp16 bits in registers until qt_store: converted right after the load (where hipcc put
// the conversion), each k-step began with a vmcnt wait for the NEXT stage's loads, serialising a global round trip with
// every stage's MFMAs.
template <int EPI>
__device__ __forceinline__ void qt_load(const GemvArgs& a, int K, int o0, int t0, int kb, int t, i32x4_t (&rw)[QTile<EPI>::NM][2],
                                        i32x4_t (&rx)[2], unsigned short (&rdw)[QTile<EPI>::NM], float& rdx) {
  const int nb = K >> 5;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int idx = t + 256 * c, row = idx >> 2, k16 = idx & 3;
    const int8_t* xp = a.xq + (int64_t)min(t0 + row, a.M - 1) * K + kb * 32 + 16 * k16;
    rx[c] = *reinterpret_cast<const i32x4_t*>(xp);
#pragma unroll
    for (int m = 0; m < QTile<EPI>::NM; ++m) {
      const int8_t* wp = (m ? a.wq2 : a.wq) + (int64_t)min(o0 + row, a.O - 1) * K + kb * 32 + 16 * k16;
      rw[m][c] = *reinterpret_cast<const i32x4_t*>(wp);
    }
  }
  const int row = t >> 1, blk = t & 1;
#pragma unroll
  for (int m = 0; m < QTile<EPI>::NM; ++m)
    rdw[m] = __half_as_ushort((m ? a.wd2 : a.wd)[(int64_t)min(o0 + row, a.O - 1) * nb + kb + blk]);
  rdx = a.xd[(int64_t)min(t0 + row, a.M - 1) * nb + kb + blk];
}

template <int EPI>
__device__ __forceinline__ void qt_store(uint8_t* st, int t, const i32x4_t (&rw)[QTile<EPI>::NM][2], const i32x4_t (&rx)[2],
                                         const unsigned short (&rdw0)[QTile<EPI>::NM], float rdx) {
  using T = QTile<EPI>;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int idx = t + 256 * c, row = idx >> 2, k16 = idx & 3;
#pragma unroll
    for (int m = 0; m < T::NM; ++m) *reinterpret_cast<i32x4_t*>(st + m * T::W + row * QT_LD + 16 * k16) = rw[m][c];
    *reinterpret_cast<i32x4_t*>(st + T::NM * T::W + row * QT_LD + 16 * k16) = rx[c];
  }
  float* sc = reinterpret_cast<float*>(st + (T::NM + 1) * T::W);  // [m (weights) | NM (tokens)][blk][128]
  const int row = t >> 1, blk = t & 1;
#pragma unroll
  for (int m = 0; m < T::NM; ++m) {
    unsigned short raw = rdw0[m];
    asm volatile("" : "+v"(raw)::"memory");  // convert here, after the stage's compute, not at the load
    sc[(m * 2 + blk) * 128 + row] = __half2float(__ushort_as_half(raw));
  }
  sc[(T::NM * 2 + blk) * 128 + row] = rdx;
}

// S = 1: write-after-barrier staging (the encoder GEMM tiles' schedule): the registers holding K-step kt + 1, loaded a
// whole step earlier, go to the free stage at the top of step kt and then take step kt + 2's loads
// Two blocks per CU (launch bounds): the SwiGLU form held 255 VGPRs + 16 AGPRs and ran one wave per SIMD, with its
// per-block f32 scaling issue-bound (profiles/r05_pmc_sq_stalls.txt); bounded, it fits 256 registers without scratch.
template <int EPI, int S = 0>
__global__ __launch_bounds__(256, 2) void k_gemm_q8_t(GemvArgs a, int K) {
  using T = QTile<EPI>;
  constexpr int NM = T::NM;
  extern __shared__ __attribute__((aligned(16))) uint8_t qsm[];
  const int o0 = blockIdx.x * 128, t0 = blockIdx.y * 128;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63, r = lane & 31, h = lane >> 5;
  const int wr = wave >> 1, wc = wave & 1;
  f32x16 acc[NM][2][2];
#pragma unroll
  for (int m = 0; m < NM; ++m)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[m][i][j] = f32x16{};
  i32x4_t rw[NM][2], rx[2];
  unsigned short rdw[NM];
  float rdx;
  const int nk = K / 64;
  qt_load<EPI>(a, K, o0, t0, 0, t, rw, rx, rdw, rdx);
  qt_store<EPI>(qsm, t, rw, rx, rdw, rdx);
  if (S == 1 && nk > 1) qt_load<EPI>(a, K, o0, t0, 2, t, rw, rx, rdw, rdx);
  __syncthreads();
  const i32x16_t zero = {};
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if constexpr (S == 1) {
      if (kt + 1 < nk) qt_store<EPI>(qsm + (cur ^ 1) * T::STAGE, t, rw, rx, rdw, rdx);
      if (kt + 2 < nk) qt_load<EPI>(a, K, o0, t0, 2 * (kt + 2), t, rw, rx, rdw, rdx);
    } else {
      if (kt + 1 < nk) qt_load<EPI>(a, K, o0, t0, 2 * (kt + 1), t, rw, rx, rdw, rdx);
    }
    const uint8_t* st = qsm + cur * T::STAGE;
    const float* sc = reinterpret_cast<const float*>(st + (NM + 1) * T::W);
#pragma unroll 1
    for (int j = 0; j < 2; ++j) {  // the stage's two q8_0 blocks
      i32x4_t bx[2];
      float dx[2];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int tok = wc * 64 + jj * 32 + r;
        bx[jj] = *reinterpret_cast<const i32x4_t*>(st + NM * T::W + tok * QT_LD + 32 * j + 16 * h);
        dx[jj] = sc[(NM * 2 + j) * 128 + tok];
      }
#pragma unroll
      for (int m = 0; m < NM; ++m)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int rb = wr * 64 + i * 32;
          const i32x4_t aw = *reinterpret_cast<const i32x4_t*>(st + m * T::W + (rb + r) * QT_LD + 32 * j + 16 * h);
          f32x16 dwv;  // this lane's 16 row scales: rows (reg & 3) + 8 (reg >> 2) + 4 h
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const float4 d4 = *reinterpret_cast<const float4*>(sc + (m * 2 + j) * 128 + rb + 8 * g + 4 * h);
            dwv[4 * g + 0] = d4.x;
            dwv[4 * g + 1] = d4.y;
            dwv[4 * g + 2] = d4.z;
            dwv[4 * g + 3] = d4.w;
          }
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const f32x16 D = mfma_i8_f32<EPI != 2>(aw, bx[jj]);  // SwiGLU form: 255 VGPRs already
            // acc += f32(dot) * (f32(d_w) * d_x), one rounding per product and per fused add as before, on 16-wide
            // vectors: v_pk_mul_f32 / v_pk_fma_f32 (two values per instruction; hipcc packed the EPI 0 / 1 forms by
            // itself but not the SwiGLU one)
            acc[m][i][jj] = __builtin_elementwise_fma(D, dwv * dx[jj], acc[m][i][jj]);
          }
          __builtin_amdgcn_sched_barrier(0);  // one (matrix, row tile) at a time: two MFMA results live, not eight
        }
    }
    if (S == 0 && kt + 1 < nk) qt_store<EPI>(qsm + (cur ^ 1) * T::STAGE, t, rw, rx, rdw, rdx);
    __syncthreads();
  }
  // epilogue: lane -> token t0 + wc 64 + jj 32 + r; reg -> row o0 + wr 64 + i 32 + (reg & 3) + 8 (reg >> 2) + 4 h
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int tok = t0 + wc * 64 + jj * 32 + r, rb = o0 + wr * 64 + i * 32;
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float y = acc[0][i][jj][q];
        if constexpr (EPI == 2) {
          const float y2 = acc[NM - 1][i][jj][q];
          v[q] = (y / (1.0f + expf(-y))) * y2;
        } else {
          v[q] = y;
        }
      }
      if (tok < a.M) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int row = rb + (q & 3) + 8 * (q >> 2) + 4 * h;
          if (row < a.O) {
            float* op = a.out + (int64_t)tok * a.ldo + row;
            if (EPI == 1) *op = a.res[(int64_t)tok * a.ldr + row] + v[q];
            else *op = v[q];
          }
        }
      }
      if constexpr (EPI == 2) {
        if (a.qout) {  // the down GEMM's q8_0 input: rows rb .. rb + 31 of this token are one block (swiglu_tile_q8)
          float am = 0.f;
#pragma unroll
          for (int q = 0; q < 16; ++q) am = fmaxf(am, fabsf(v[q]));
          am = fmaxf(am, __shfl_xor(am, 32, 64));
          const float d = am / 127.0f;
          const float id = d != 0.0f ? 1.0f / d : 0.0f;
          if (tok < a.M) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int b0 = (int)roundf(__fmul_rn(v[4 * g], id)) & 0xFF, b1 = (int)roundf(__fmul_rn(v[4 * g + 1], id)) & 0xFF;
              const int b2 = (int)roundf(__fmul_rn(v[4 * g + 2], id)) & 0xFF, b3 = (int)roundf(__fmul_rn(v[4 * g + 3], id)) & 0xFF;
              *reinterpret_cast<int32_t*>(a.qout + (int64_t)tok * a.ldo + rb + 8 * g + 4 * h) =
                  b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
            }
            if (h == 0) a.dout[(int64_t)tok * (a.ldo / 32) + rb / 32] = __half2float(__float2half_rn(d));
          }
        }
      }
    }
}

int g_gemm_t_min_m = 512;  // token count from which prefill GEMMs take the tiled kernel (FUNASR_GEMM_T_MIN_M)

int g_gemm_t_wab = 0;  // k_gemm_q8_t write-after-barrier staging (FUNASR_GEMM_T_WAB)

template <int S>
static void launch_gemm_q8_t(const GemvArgs& a, int K, int epi, dim3 grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_gemm_q8_t<0, S>, hipFuncAttributeMaxDynamicSharedMemorySize, QTile<0>::BYTES);
    (void)hipFuncSetAttribute((const void*)k_gemm_q8_t<1, S>, hipFuncAttributeMaxDynamicSharedMemorySize, QTile<1>::BYTES);
    (void)hipFuncSetAttribute((const void*)k_gemm_q8_t<2, S>, hipFuncAttributeMaxDynamicSharedMemorySize, QTile<2>::BYTES);
    attr = true;
  }
  switch (epi) {
    case 0: hipLaunchKernelGGL((k_gemm_q8_t<0, S>), grid, dim3(256), QTile<0>::BYTES, s, a, K); break;
    case 1: hipLaunchKernelGGL((k_gemm_q8_t<1, S>), grid, dim3(256), QTile<1>::BYTES, s, a, K); break;
    default: hipLaunchKernelGGL((k_gemm_q8_t<2, S>), grid, dim3(256), QTile<2>::BYTES, s, a, K); break;
  }
}

static bool gemm_q8_t(const GemvArgs& a, int K, int epi, hipStream_t s) {
  if (a.M < g_gemm_t_min_m || epi == 3 || K % 64 || a.O % 32) return false;
  const dim3 grid(cdiv(a.O, 128), cdiv(a.M, 128));
  if (g_gemm_t_wab) launch_gemm_q8_t<1>(a, K, epi, grid, s);
  else launch_gemm_q8_t<0>(a, K, epi, grid, s);
  return true;
}

int g_lm_head_b = 1;  // 0: batched LM head on the one-tile-per-block split-K kernel (A/B, FUNASR_LM_HEAD_B=0)
int g_gemm_q8_kw = 1;  // 0: split-K block kernel for every shape (A/B switch, FUNASR_GEMM_KW=0); 2: K-in-block for all

// split-K shape: NBW q8_0 blocks per wave (8, 4 or 2: one load round trip) and KS = nb / (waves per matrix x NBW)
// splits; the largest NBW whose split count fills the chip (>= 256 blocks), else the most splits. lm_head's argmax
// needs whole sums: one split.
// split-K: the fewest blocks a shape must reach before fewer splits are preferred. Measured (graph-replayed decode
// step, full model): 256 / 192 / 128 / 96 -> batch 32 1.213 / 1.191 / 1.186 / 1.202 ms, batch 16 1.101 / 1.084 /
// 1.068 / 1.084 ms: q|k|v and gate|up take one split fewer (the split-K seam costs more than the emptier chip)
int g_sk_min_blocks = 128;
void gemm_sk_shape(int O, int M, int K, int epi, int* nbw, int* ks) {
  const int tiles = cdiv(O, 32) * cdiv(M, 32), nb = K / 32, wpm = epi == 2 ? 2 : 4;
  *nbw = 0;
  *ks = 0;
  for (int c : {8, 4, 2}) {
    if (nb % (wpm * c)) continue;
    const int k = nb / (wpm * c);
    if (k > (epi == 2 ? 4 : 16) || (epi == 3 && k != 1)) continue;
    *nbw = c;
    *ks = k;
    if (tiles * k >= g_sk_min_blocks) return;
  }
}

int gemm_k_splits(int O, int M, int K, int epi) {
  int nbw, ks;
  gemm_sk_shape(O, M, K, epi, &nbw, &ks);
  return ks;
}

int g_lm_rpw = 40;  // rows per wave of the vocabulary-wide GEMV (the LM head); multiple of 4
int gemv_rows_per_wave(int O) {
  // target ~256-1024 blocks of 4 waves
  int rpw = (O + 4 * 256 - 1) / (4 * 256);
  if (rpw > 4) rpw = ((rpw + 3) / 4) * 4;
  if (O >= 65536) rpw = g_lm_rpw;
  return rpw < 1 ? 1 : rpw;
}

// decode batches up to g_gemv_small_max tokens take the fused GEMV (above: the MFMA GEMM with producer-normalised
// inputs); from 3 tokens on, g_gemv_mt tokens share a block (weights streamed once per block for its tokens). Measured
// decode step (full model, graph-replayed, scripts/prof_batch_decode.py, after the coalesced split-K loads): batch
// 2 / 3 / 4 / 5 / 6 / 7 = 0.711 / 0.822 / 0.945 / 1.004 / 1.143 / 1.210 ms on the fused GEMV vs 1.010 / 1.043 / 1.041 /
// 1.038 / 1.063 / 1.081 on the MFMA GEMM: the GEMV up to 5 tokens. More tokens per block serialise more prologue / dot
// work per block than the saved weight re-reads (MT 4 / 8: slower).
int g_gemv_small_max = 5;
int g_gemv_mt = 2;
int g_lm_head_mt6 = 1;  // LM head of 3-6 token batches: one block row for every token (FUNASR_LM_HEAD_MT6=0: pairs)

bool gemv_small(int M) { return M <= g_gemv_small_max; }
// the small-batch MFMA LM head (k_lm_head_s) takes 2-8 tokens of the fused decode path at K = 1024
static bool lm_head_s_takes(int M, int K, int O) {
  return K == 1024 && gemv_small(M) && cdiv(O, 32) <= LMS_STEPS * LMS_BLOCKS &&
         ((g_lm_head_s && M >= 2 && M <= 8) || (g_lm_head_s1 && M == 1));
}

template <int MT>
static void launch_gemv_fused(int K, int epi, const GemvArgs& a, hipStream_t s) {
  switch (epi) {
    case 0: launch_gemv_k<MT, true, 0>(K, a, s); break;
    case 1: launch_gemv_k<MT, true, 1>(K, a, s); break;
    case 2: launch_gemv_k<MT, true, 2>(K, a, s); break;
    case 3: launch_gemv_k<MT, true, 3>(K, a, s); break;
  }
}

void gemv_q8(const GemvArgs& a, int K, int epi, hipStream_t s) {
  const bool fused = a.x != nullptr && a.ssp == nullptr;
  if (a.psum) {  // fused decode layer (M = 1): q|k|v (EPI 0) or the LM head (EPI 3) after a split down projection
    FA_REQUIRE(fused && a.M == 1 && K == 1024 && (epi == 0 || epi == 3), "gemv_q8: partial-sum prologue shape");
    if (epi == 0) {
      launch_gemv<1, 1, true, 0, true>(a, s);
    } else if (lm_head_s_takes(1, K, a.O)) {  // (n_part: lm_head_parts counts the tiles then)
      const dim3 grid(std::min(cdiv(a.O, 32), g_lm_grid > 0 ? std::min(g_lm_grid, LMS_BLOCKS) : LMS_BLOCKS));
      FA_REQUIRE(cdiv(a.O, 32) <= LMS_STEPS * (int)grid.x && a.norm_w, "lm_head_s: vocabulary too large / no norm");
      if (g_lm_head_s1 == 2) hipLaunchKernelGGL((k_lm_head_s<2, true>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((k_lm_head_s<1, true>), grid, dim3(256), 0, s, a);
    } else {
      launch_gemv<1, 1, true, 3, true>(a, s);
    }
    return;
  }
  if (gemv_small(a.M) && fused) {
    FA_REQUIRE(epi != 3 || a.n_part == lm_head_parts(a.O, a.M, K), "gemv_q8: n_part");
    if (epi == 3 && lm_head_s_takes(a.M, K, a.O)) {
      const dim3 grid(std::min(cdiv(a.O, 32), g_lm_grid > 0 ? std::min(g_lm_grid, LMS_BLOCKS) : LMS_BLOCKS));
      FA_REQUIRE(cdiv(a.O, 32) <= LMS_STEPS * (int)grid.x && a.norm_w, "lm_head_s: vocabulary too large / no norm");
      if ((a.M == 1 ? g_lm_head_s1 : g_lm_head_s) == 2) hipLaunchKernelGGL((k_lm_head_s<2, false>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((k_lm_head_s<1, false>), grid, dim3(256), 0, s, a);
      return;
    }
    // decode path: MT tokens per block row (the block's weight rows are streamed once for its MT tokens). The LM head
    // (165 MB of rows) takes all of a 3-6 token batch in one block row: re-streaming it per token pair cost 86 us per
    // launch at 6 tokens. A token's arithmetic does not depend on MT (compute_group runs it per token).
    if (epi == 3 && K == 1024 && a.M >= 3 && a.M <= 6 && g_lm_head_mt6) {
      launch_gemv<1, 6, true, 3>(a, s);
      return;
    }
    const int mt = a.M <= 2 ? 1 : std::min(g_gemv_mt, a.M);
    if (mt <= 1) launch_gemv_fused<1>(K, epi, a, s);
    else launch_gemv_fused<2>(K, epi, a, s);
    return;
  }
  FA_REQUIRE(!fused, "gemv_q8: fused prologue only for M <= g_gemv_small_max");
  if (a.row_local) {  // each token row's arithmetic independent of the token count: the K-in-block kernel only
    FA_REQUIRE(epi != 3, "gemv_q8: row-local rows are prefill layer GEMMs");
    FA_REQUIRE(!a.ssp || (K == 1024 && (epi == 0 || epi == 2) && a.xq && a.xd),
               "gemv_q8: normalised-input rows feed q|k|v / gate|up (K 1024)");
    FA_REQUIRE(!a.ssp_out || (epi == 1 && a.O == 1024 && a.qout && a.dout && a.qn_w),
               "gemv_q8: the normalising residual epilogue needs O 1024, qout / dout and qn_w");
    FA_REQUIRE(gemm_q8_kw(a, K, epi, s, true), "gemv_q8: row-local GEMM shape not instantiated");
    return;
  }
  FA_REQUIRE(K % 1024 == 0 && K <= 3072, "gemm_q8: K must be 1024/2048/3072");
  FA_REQUIRE(epi != 3 || a.n_part == lm_head_parts(a.O, a.M, K), "gemm_q8: n_part");
  if (epi == 3 && K == 1024 && a.M <= 32 && g_lm_head_b) {  // batched LM head: persistent tile loop
    const int nblk = std::min(cdiv(a.O, 32), g_lm_grid > 0 ? std::min(g_lm_grid, LMB_BLOCKS) : LMB_BLOCKS);
    if (a.ssp) hipLaunchKernelGGL(k_lm_head_b<true>, dim3(nblk), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_lm_head_b<false>, dim3(nblk), dim3(256), 0, s, a);
    return;
  }
  if (!a.ssp && gemm_q8_t(a, K, epi, s)) return;
  if (!a.ssp && g_gemm_q8_kw && gemm_q8_kw(a, K, epi, s)) return;
  FA_REQUIRE(a.O % 32 == 0 && a.ldo % 4 == 0 && (!a.res || a.ldr % 4 == 0),
             "gemm_q8: rows must come in whole 32-row tiles with 16-B aligned output / residual rows");
  int NBW, KS;
  gemm_sk_shape(a.O, a.M, K, epi, &NBW, &KS);
  FA_REQUIRE(NBW > 0, "gemm_q8: no split-K shape");
  FA_REQUIRE(!a.ssp || (K == 1024 && epi != 1 && a.xq && a.xd),
             "gemm_q8: rows normalised by their producer's epilogue need K 1024 (a residual GEMM cannot take them)");
  FA_REQUIRE(!a.ssp_out || (epi == 1 && a.O == 1024 && a.qout && a.dout && a.qn_w),
             "gemm_q8: the normalising residual epilogue needs O 1024, qout / dout and qn_w");
  if (KS > 1)
    FA_REQUIRE(a.kpart && a.kcnt && (int64_t)cdiv(a.O, 32) * cdiv(a.M, 32) <= a.kcnt_n &&
                   (int64_t)cdiv(a.O, 32) * cdiv(a.M, 32) * KS * (epi == 2 ? 2 : 1) * 1024 <= a.kpart_n,
               "gemm_q8: split-K workspace too small");
  dim3 grid(cdiv(a.O, 32), cdiv(a.M, 32), KS);
  if (a.pf_q && a.pf_slabs > 0 && grid.x % 8 == 0 && a.pf_O % 256 == 0 && a.pf_K % 128 == 0) grid.z += a.pf_slabs;
  const int ksm = KS == 1 ? 1 : KS <= 4 ? 4 : 16;
  if (a.ssp) {  // batched decode (M <= 32): inputs quantised by the previous residual epilogue, rstd applied here
    switch (epi * 1000 + NBW * 100 + ksm) {
#define SKN(E, N, Q) case E * 1000 + N * 100 + Q: hipLaunchKernelGGL((k_gemm_q8_sk<E, N, Q, true>), grid, dim3(256), 0, s, a, K, KS); return;
      SKN(0, 4, 4) SKN(0, 8, 1) SKN(2, 4, 4) SKN(2, 8, 4) SKN(3, 8, 1)
#undef SKN
      default: FA_REQUIRE(false, "gemm_q8: normalised-input shape not instantiated");
    }
  }
  switch (epi * 1000 + NBW * 100 + ksm) {
#define SK(E, N, Q) case E * 1000 + N * 100 + Q: hipLaunchKernelGGL((k_gemm_q8_sk<E, N, Q>), grid, dim3(256), 0, s, a, K, KS); break;
    SK(0, 2, 1) SK(0, 2, 4) SK(0, 2, 16) SK(0, 4, 1) SK(0, 4, 4) SK(0, 4, 16) SK(0, 8, 1) SK(0, 8, 4) SK(0, 8, 16)
    SK(1, 2, 1) SK(1, 2, 4) SK(1, 2, 16) SK(1, 4, 1) SK(1, 4, 4) SK(1, 4, 16) SK(1, 8, 1) SK(1, 8, 4) SK(1, 8, 16)
    SK(2, 2, 1) SK(2, 2, 4) SK(2, 4, 1) SK(2, 4, 4) SK(2, 8, 1) SK(2, 8, 4)
    SK(3, 8, 1)
#undef SK
    default: FA_REQUIRE(false, "gemm_q8: split-K shape not instantiated");
  }
}

// ---- gate|up + down of a batched-decode layer in ONE launch (FUNASR_GU_DOWN): the SwiGLU split-K blocks first (lower
// block ids, so all of them are dispatched before any consumer can hold a CU), then the down projection's split-K
// blocks, each waiting only for the 96 / KSd act tiles of its own K split (a group-local hand-off, SkFuse), then the
// down GEMM's L2 prefetch slabs (the next layer's q|k|v rows). The down blocks' weight rows are in flight while the
// SwiGLU blocks run, and one kernel boundary per layer disappears. Same per-tile arithmetic and split order as the
// two launches: bit-identical outputs.
template <int NBWG, int KSMG, int NBWD, int KSMD>
__global__ __launch_bounds__(256) void k_gemm_q8_gu_down(GemvArgs g, GemvArgs d, int KSg, int KSd, SkFuse fz, int n_pf) {
  constexpr int SLDG = NBWG * 32 + 16, SLDD = NBWD * 32 + 16;
  __shared__ __attribute__((aligned(16))) int8_t s_ab[4 * 2 * 32 * (SLDG > SLDD ? SLDG : SLDD)];
  const int b = blockIdx.x, tg = g.O >> 5, td = d.O >> 5;  // one 32-token tile (M <= 32)
  const int ng = tg * KSg, nd = td * KSd;
  if (b < ng) {
    sk_tile<2, NBWG, KSMG, true, 1>(g, 1024, KSg, b % tg, 0, b / tg, tg, s_ab, fz);
  } else if (b < ng + nd) {
    const int c = b - ng;
    sk_tile<1, NBWD, KSMD, false, 2>(d, 3072, KSd, c % td, 0, c / td, td, s_ab, fz);
  } else {
    gemm_l2_prefetch(d, b - ng - nd, n_pf);
  }
}

bool gemm_q8_gu_down(const GemvArgs& g0, const GemvArgs& d0, unsigned* cnt, int* err, hipStream_t s) {
  // shapes: Qwen3-0.6B at M <= 32 (E 1024, F 3072), producer-normalised gate|up input, down with K = F
  if (g0.M > 32 || g0.M != d0.M || g0.O != 3072 || d0.O != 1024 || !g0.ssp || !g0.qout || d0.ssp || !g0.kpart ||
      !g0.kcnt)
    return false;
  int nbwg, ksg, nbwd, ksd;
  gemm_sk_shape(g0.O, g0.M, 1024, 2, &nbwg, &ksg);
  gemm_sk_shape(d0.O, d0.M, 3072, 1, &nbwd, &ksd);
  const int tg = g0.O / 32, td = d0.O / 32;
  if (nbwg <= 0 || nbwd <= 0 || tg % ksd || tg % 8 || td % 8) return false;
  const int64_t gpart = (int64_t)tg * ksg * 2 * 1024, dpart = (int64_t)td * ksd * 1024;
  if (tg + td > g0.kcnt_n || gpart + dpart > g0.kpart_n) return false;
  GemvArgs g = g0, d = d0;
  g.pf_q = nullptr;  // the down blocks load their own rows
  d.kpart = g0.kpart + gpart;
  d.kpart_n = dpart;
  d.kcnt = g0.kcnt + tg * CNT_LINE;
  d.kcnt_n = td;
  SkFuse fz;
  fz.arr = cnt;
  fz.dep = cnt + 32 * CNT_LINE;
  fz.tiles_per_split = tg / ksd;
  fz.consumers = td;
  fz.err = err;
  const int n_pf = d.pf_q && d.pf_slabs > 0 && d.pf_O % 256 == 0 && d.pf_K % 128 == 0 ? d.pf_slabs * td : 0;
  if (!n_pf) d.pf_q = nullptr;
  const dim3 grid(tg * ksg + td * ksd + n_pf);
  const int kmg = ksg == 1 ? 1 : ksg <= 4 ? 4 : 16, kmd = ksd == 1 ? 1 : ksd <= 4 ? 4 : 16;
  switch (nbwg * 100000 + kmg * 1000 + nbwd * 100 + kmd) {
#define GD(A, B, C, D)                                                                                     \
  case A * 100000 + B * 1000 + C * 100 + D:                                                                \
    hipLaunchKernelGGL((k_gemm_q8_gu_down<A, B, C, D>), grid, dim3(256), 0, s, g, d, ksg, ksd, fz, n_pf); \
    return true;
    GD(8, 4, 4, 16) GD(4, 4, 4, 16) GD(8, 4, 2, 16) GD(4, 4, 2, 16) GD(8, 4, 8, 4) GD(4, 4, 8, 4)
#undef GD
    default: return false;
  }
}

int lm_head_parts(int O, int M, int K) {
  return gemv_small(M) && !lm_head_s_takes(M, K, O) ? cdiv(O, 4 * gemv_rows_per_wave(O)) * 4 : cdiv(O, 32);
}
int lm_head_chunk(int O, int M, int K) { return gemv_small(M) && !lm_head_s_takes(M, K, O) ? gemv_rows_per_wave(O) : 32; }

// ------------------------------------------------------------------------------------------------
// q/k RMSNorm per head (attn_q_norm/attn_k_norm) + NEOX RoPE + KV-cache store (fp16).
// One wave per (token, head-slot); head slots 0..H-1 = q heads, H..H+KV-1 = k heads, then v heads.
__global__ void k_qk_rope_store(const float* __restrict__ qkv, int M, int H, int KV, float eps,
                                const float* __restrict__ qn, const float* __restrict__ kn,
                                const float* __restrict__ rcos, const float* __restrict__ rsin,
                                const int* __restrict__ tok_seq, const int* __restrict__ tok_pos,
                                float* __restrict__ qout, __half* __restrict__ kc, __half* __restrict__ vc,
                                int64_t seq_stride /* elements per seq per layer */) {
  constexpr int D = 128;
  const int slot = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int m = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int n_slots = H + 2 * KV;
  if (slot >= n_slots || m >= M) return;
  const float* src = qkv + (int64_t)m * (H + 2 * KV) * D + slot * D;
  const int pos = tok_pos[m];
  // head-major cache [seq][kv head][n_ctx][D]: kv head g's rows at cbase + g * (seq_stride / KV)
  const int64_t cbase = (int64_t)tok_seq[m] * seq_stride + (int64_t)pos * D;
  const int64_t hs = seq_stride / KV;
  float x0 = src[lane], x1 = src[lane + 64];
  if (slot >= H + KV) {  // V: store as-is
    const int g = slot - H - KV;
    vc[cbase + g * hs + lane] = __float2half_rn(x0);
    vc[cbase + g * hs + lane + 64] = __float2half_rn(x1);
    return;
  }
  const float* w = slot < H ? qn : kn;
  const float ss = wave_sum(x0 * x0 + x1 * x1);
  const float scale = 1.0f / sqrtf(ss / (float)D + eps);
  x0 = (x0 * scale) * w[lane];
  x1 = (x1 * scale) * w[lane + 64];
  const float c = rcos[(int64_t)pos * 64 + lane], sn = rsin[(int64_t)pos * 64 + lane];
  const float y0 = x0 * c - x1 * sn, y1 = x0 * sn + x1 * c;
  if (slot < H) {
    qout[((int64_t)m * H + slot) * D + lane] = y0;
    qout[((int64_t)m * H + slot) * D + lane + 64] = y1;
  } else {
    const int g = slot - H;
    kc[cbase + g * hs + lane] = __float2half_rn(y0);
    kc[cbase + g * hs + lane + 64] = __float2half_rn(y1);
  }
}

void qk_rope_store(const float* qkv, int M, int H, int KV, float eps, const float* qn, const float* kn, const float* rcos,
                   const float* rsin, const int* tok_seq, const int* tok_pos, float* qout, __half* kc, __half* vc,
                   int64_t seq_stride, hipStream_t s) {
  dim3 grid(cdiv(H + 2 * KV, 4), M);
  hipLaunchKernelGGL(k_qk_rope_store, grid, dim3(256), 0, s, qkv, M, H, KV, eps, qn, kn, rcos, rsin, tok_seq, tok_pos,
                     qout, kc, vc, seq_stride);
}


// ------------------------------------------------------------------------------------------------
// Decode/prefill attention over the fp16 KV cache. Block = (kv head g, token m), 8 waves; wave w takes the
// 64-key chunks w, w+8, ... (lane = key for q.k, 16 lanes x 8 dims x 4 key phases for p.V) with its own
// online softmax; the 8 partial states merge in LDS. Every K/V load of a chunk is issued before any math.
// DECODE mode (each token row its own sequence): wave 0 rms-norms + ropes the group's 2 q heads; the wave
// whose chunk holds the token's position also norms/ropes k, stores K/V of that position to the cache and
// consumes the fresh row from LDS (with the cache's fp16 rounding). PREFILL mode: q comes pre-roped from
// qk_rope_store and the cache is complete.
#ifdef FA_ATTN_STAMPS
// per-block s_memrealtime (100 MHz, chip-wide) stamps of wave 0, lane 0: [i] at the STAMP(i) points
__device__ unsigned long long g_attn_stamps[4096][16];
#define STAMP(i) do { if (threadIdx.x == 0) g_attn_stamps[(blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x][i] = __builtin_amdgcn_s_memrealtime(); } while (0)
void attn_stamps_read(unsigned long long* host, int n_blocks) {
  (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_attn_stamps), (size_t)n_blocks * 128, 0, hipMemcpyDeviceToHost);
}
void attn_stamps_clear() {
  static unsigned long long z[4096][16];
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_attn_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice);
}
#else
#define STAMP(i) do { } while (0)
#endif
constexpr int GQ = 2;     // query heads per kv head (Qwen3-0.6B: 16 / 8)
constexpr int AWV = 4;    // waves per block
int g_attn_blocks = 1024;  // key splits are added while (token, kv head, split) blocks stay within this many
int g_attn_lean = -1;      // -1: lean blocks when a launch needs more than 3 per CU; 0 / 1 force (A/B)
int g_attn_wide = 0;       // decode launches with at least this many (token, kv head) pairs: one 16-wave block each
int g_attn_ldspf = 0;      // ... (off: measured slower, batch-32 step 1.207 -> 1.248 ms, same one block per CU) whose waves pull each next pass's K/V into LDS during the current pass (FUNASR_ATTN_LDSPF)
constexpr int AGI = 16;   // 4-key groups per wave per pass (registers: 16 int4 of K + 16 of V)
constexpr int ASPLIT = ATTN_SPLITS;  // key splits (blocks) per (token, kv head)
#ifndef FA_AMIN_G
#define FA_AMIN_G 8
#endif
constexpr int AMIN_G = FA_AMIN_G;    // minimum 4-key groups per split (32 keys = 16 KB of K+V)
constexpr int APART = ATTN_PART_FLOATS;  // per-split partial: o[GQ][128], m[GQ], l[GQ]
// Within a split, keys are dealt to the waves in 4-key groups, round-robin (group q -> wave q % AWV).
// Lane (kq = lane>>4, dq = lane&15) holds dims [8 dq, 8 dq + 8) of key 4 q + kq: each load instruction
// reads 4 whole 256-B rows. Groups past the wave's share are loaded clamped (valid rows, compute skipped):
// no branches around loads.
// kmax: the last cache row a load may touch. Decode passes pos - 1: row pos is this launch's fresh row, stored by its
// owner wave (which takes its values from LDS) possibly AFTER other waves' clamped loads, so a clamped re-read of it
// would see stale bytes -- bytes a previous buffer left there, possibly NaN / Inf patterns -- and a masked key's
// p = 0 times a NaN V is NaN. Masked keys re-read row pos - 1 instead (written, finite): valid keys are unchanged.
#ifndef FA_KV_CLAMP_OLD  // 1 (A/B builds only): the pre-round-6 clamp to row pos (reproduces the stale-row read)
#define FA_KV_CLAMP_OLD 0
#endif
template <int NI, int AW>
__device__ __forceinline__ void load_kv_groups(const __half* __restrict__ base, int KV, int g0, int kmax, int kq,
                                               int dq, int4 (&t)[NI]) {
  constexpr int D = 128;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int k = min(4 * (g0 + AW * i) + kq, kmax);
    t[i] = *reinterpret_cast<const int4*>(base + (int64_t)k * D + dq * 8);  // head-major cache: rows D apart
  }
}

__device__ __forceinline__ void unpack8(const int4& r, float (&v)[8]) {
  const __half2* hp = reinterpret_cast<const __half2*>(&r);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float2 f = __half22float2(hp[e]);
    v[2 * e] = f.x;
    v[2 * e + 1] = f.y;
  }
}

// RMSNorm (q_norm / k_norm) + NeoX RoPE of one 128-dim head held as (x0 = dim lane, x1 = dim lane + 64).
__device__ __forceinline__ void norm_rope(float x0, float x1, float w0, float w1, float eps, float c, float sn,
                                          float& y0, float& y1) {
  const float sc = 1.0f / sqrtf(wave_sum(x0 * x0 + x1 * x1) / 128.0f + eps);
  x0 = (x0 * sc) * w0;
  x1 = (x1 * sc) * w1;
  y0 = x0 * c - x1 * sn;
  y1 = x0 * sn + x1 * c;
}

// raw per-lane inputs of the q (and fresh k/v) prologue, loaded before the K/V stream is issued
struct AttnQIn {
  float x0[GQ], x1[GQ];             // q heads (dims lane, lane + 64)
  float c, sn, w0, w1;              // rope cos/sin at pos, q_norm weights
  float kx0, kx1, kw0, kw1, v0, v1; // fresh k (pre-norm), k_norm weights, fresh v (owner wave only)
};

// One wave's share of one key split: NI = its 4-key groups per pass rounded up to a power of two (loads of
// the rounded-up slots are clamped duplicates, masked). Issues the K/V stream first, then finishes q while
// it is in flight.
// PIPE: the next pass's K/V loads are issued before this pass's math (2x the K/V registers: non-lean blocks only;
// batch-1 B of the fused layer 7.44 -> 7.32 us, scripts/ubench/decode_step)
// PRE: the first pass's K/V (groups g0 + AW i, i < NI) were loaded by the caller (the first NI of AKV_PRE groups:
// the same clamped addresses load_kv_groups<NI> would use)
constexpr int AKV_PRE = 4;
// LPF (the 16-wave batched-decode blocks, lean passes): the NEXT pass's K/V rows are pulled into this wave's LDS slot
// (slot[0 K / 1 V][i][lane], 16 B per lane, lane-linear as LDS-DMA writes them) while the current pass computes, so a
// context longer than one pass costs one memory round trip instead of one per pass; each lane reads back only the
// bytes its own DMA lane wrote (s_waitcnt vmcnt(0) orders them). Same values, same arithmetic.
template <int NI, int AW, bool PIPE, bool PRE = false, bool LPF = false>
__device__ __forceinline__ void attn_wave(const __half* __restrict__ kb, const __half* __restrict__ vb, int KV, int g0,
                                          int ge, int n_keys, int kq, int dq, int lane, bool decode, bool fresh_here,
                                          int pos, float eps, float scale, const AttnQIn& qi, __half* __restrict__ kd,
                                          __half* __restrict__ vd, float (*s_qw)[128], float* s_kn, float* s_vn,
                                          float (&mx)[GQ], float (&l)[GQ], float (&acc)[GQ][8],
                                          const int4* pk = nullptr, const int4* pv = nullptr, int4* slot = nullptr) {
  constexpr int SD = 128;
  const int kmax = decode && !FA_KV_CLAMP_OLD ? max(pos - 1, 0) : n_keys - 1;  // last cache row a load may touch
  auto lpf_issue = [&](int g1) {  // next pass's groups -> slot (clamped rows as load_kv_groups clamps them)
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int k = min(4 * (g1 + AW * i) + kq, kmax);
      __builtin_amdgcn_global_load_lds((const void*)(kb + (int64_t)k * SD + dq * 8),
                                       (__attribute__((address_space(3))) void*)(slot + i * 64), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(vb + (int64_t)k * SD + dq * 8),
                                       (__attribute__((address_space(3))) void*)(slot + (4 + i) * 64), 16, 0, 0);
    }
  };
  int4 kt[NI], vt[NI];
  if constexpr (PRE) {
    static_assert(NI <= AKV_PRE, "attn_wave: preloaded groups");
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      kt[i] = pk[i];
      vt[i] = pv[i];
    }
  } else {
    load_kv_groups<NI, AW>(kb, KV, g0, kmax, kq, dq, kt);
    load_kv_groups<NI, AW>(vb, KV, g0, kmax, kq, dq, vt);
  }
  if constexpr (LPF) {
    if (g0 + AW * NI < ge) lpf_issue(g0 + AW * NI);
  }
  __builtin_amdgcn_sched_barrier(0);  // the q math below must not be hoisted above the K/V stream's issue
  STAMP(2);
  if (decode) {
#pragma unroll
    for (int j = 0; j < GQ; ++j) {
      float y0, y1;
      norm_rope(qi.x0[j], qi.x1[j], qi.w0, qi.w1, eps, qi.c, qi.sn, y0, y1);
      s_qw[j][lane] = y0 * scale;
      s_qw[j][lane + 64] = y1 * scale;
    }
    if (fresh_here) {  // this wave owns K/V[pos]: store it to the cache and use it from LDS
      float y0, y1;
      norm_rope(qi.kx0, qi.kx1, qi.kw0, qi.kw1, eps, qi.c, qi.sn, y0, y1);
      const __half k0h = __float2half_rn(y0), k1h = __float2half_rn(y1);
      const __half v0h = __float2half_rn(qi.v0), v1h = __float2half_rn(qi.v1);
      kd[lane] = k0h;
      kd[lane + 64] = k1h;
      vd[lane] = v0h;
      vd[lane + 64] = v1h;
      s_kn[lane] = __half2float(k0h);
      s_kn[lane + 64] = __half2float(k1h);
      s_vn[lane] = __half2float(v0h);
      s_vn[lane + 64] = __half2float(v1h);
    }
  } else {
#pragma unroll
    for (int j = 0; j < GQ; ++j) {
      s_qw[j][lane] = qi.x0[j] * scale;
      s_qw[j][lane + 64] = qi.x1[j] * scale;
    }
  }
  __builtin_amdgcn_wave_barrier();
  float q[GQ][8];
#pragma unroll
  for (int j = 0; j < GQ; ++j) {
    const float4 a0 = *reinterpret_cast<const float4*>(&s_qw[j][dq * 8]);
    const float4 a1 = *reinterpret_cast<const float4*>(&s_qw[j][dq * 8 + 4]);
    q[j][0] = a0.x; q[j][1] = a0.y; q[j][2] = a0.z; q[j][3] = a0.w;
    q[j][4] = a1.x; q[j][5] = a1.y; q[j][6] = a1.z; q[j][7] = a1.w;
  }
  STAMP(3);
  const int fresh = fresh_here ? pos : -1;
  int4 kn_[PIPE ? NI : 1], vn_[PIPE ? NI : 1];  // PIPE: the next pass's K/V
  for (;;) {
    if constexpr (PIPE) {
      const int g1 = g0 + AW * NI;
      if (g1 < ge) {
        load_kv_groups<NI, AW>(kb, KV, g1, kmax, kq, dq, kn_);
        load_kv_groups<NI, AW>(vb, KV, g1, kmax, kq, dq, vn_);
      }
    }
    // scores of key 4 (g0 + AW i) + kq: 8-dim partial dot per lane, summed over the row's 16 lanes (DPP)
    float sc[NI][GQ];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int key = 4 * (g0 + AW * i) + kq;
      const bool valid = (g0 + AW * i) < ge && key < n_keys;
      float kv[8];
      unpack8(kt[i], kv);
      if (key == fresh) {
#pragma unroll
        for (int e = 0; e < 8; ++e) kv[e] = s_kn[dq * 8 + e];
      }
#pragma unroll
      for (int j = 0; j < GQ; ++j) {
        float pd = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) pd += kv[e] * q[j][e];
        pd = row_sum16(pd);
        sc[i][j] = valid ? pd : -INFINITY;
      }
    }
    STAMP(4);
    // online softmax: row-local max/sum over i, then across the 4 rows (readlanes)
#pragma unroll
    for (int j = 0; j < GQ; ++j) {
      float cm = sc[0][j];
#pragma unroll
      for (int i = 1; i < NI; ++i) cm = fmaxf(cm, sc[i][j]);
      cm = fmaxf(fmaxf(lane_f(cm, 0), lane_f(cm, 16)), fmaxf(lane_f(cm, 32), lane_f(cm, 48)));
      const float mn = fmaxf(mx[j], cm);
      const float alpha = mx[j] == -INFINITY ? 0.f : __expf(mx[j] - mn);
      float ps = 0.f;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const float p = sc[i][j] == -INFINITY ? 0.f : __expf(sc[i][j] - mn);
        sc[i][j] = p;
        ps += p;
      }
      ps = (lane_f(ps, 0) + lane_f(ps, 16)) + (lane_f(ps, 32) + lane_f(ps, 48));
      l[j] = l[j] * alpha + ps;
      mx[j] = mn;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[j][e] *= alpha;
    }
    STAMP(5);
    // p.V with p still in registers
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int key = 4 * (g0 + AW * i) + kq;
      float v[8];
      unpack8(vt[i], v);
      if (key == fresh) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = s_vn[dq * 8 + e];
      }
#pragma unroll
      for (int j = 0; j < GQ; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[j][e] += sc[i][j] * v[e];
    }
    STAMP(6);
    g0 += AW * NI;
    if (g0 >= ge) break;
    if constexpr (PIPE) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        kt[i] = kn_[PIPE ? i : 0];
        vt[i] = vn_[PIPE ? i : 0];
      }
    } else if constexpr (LPF) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA into its slot has landed
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        kt[i] = slot[i * 64 + lane];
        vt[i] = slot[(4 + i) * 64 + lane];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read back before the slot is refilled
      if (g0 + AW * NI < ge) lpf_issue(g0 + AW * NI);
    } else {
      load_kv_groups<NI, AW>(kb, KV, g0, kmax, kq, dq, kt);
      load_kv_groups<NI, AW>(vb, KV, g0, kmax, kq, dq, vt);
    }
  }
}

// q8_0 quantisation of an attention output row held 4 dims per lane (lanes 8b..8b+7 = one 32-dim block): the
// o projection's input, with the arithmetic of norm_quant_row (no prep launch). e = element index of v.x.
__device__ __forceinline__ void store_q8_row4(int8_t* __restrict__ qout, float* __restrict__ dout, int64_t e, int lane,
                                              float4 v) {
  const float a = group_max<8>(fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  const float d = a / 127.0f;
  const float id = d != 0.0f ? 1.0f / d : 0.0f;
  const int b0 = (int)roundf(__fmul_rn(v.x, id)) & 0xFF, b1 = (int)roundf(__fmul_rn(v.y, id)) & 0xFF;
  const int b2 = (int)roundf(__fmul_rn(v.z, id)) & 0xFF, b3 = (int)roundf(__fmul_rn(v.w, id)) & 0xFF;
  *reinterpret_cast<int32_t*>(qout + e) = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
  if ((lane & 7) == 0) dout[e / 32] = __half2float(__float2half_rn(d));
}

// Decode / causal attention for one (kv head g, token m, key split sp): GQ = 2 query heads share the
// K/V stream. Keys [0, pos] are cut into n_active contiguous splits of >= AMIN_G groups each (one block
// per split, so a long context is fetched by up to ASPLIT CUs instead of one). A single active split writes
// the output directly; otherwise each split stores its (m, l, o) partial with sc1 stores, waits, and adds
// to the (m, g) counter (agent scope); the block whose add comes last combines the partials with sc1
// loads and re-arms the counter (MI355X_MICROARCH.md hand-off table, row 1: no fences needed).
// Prefill mode (decode_mode = 0): q is already normed/roped (qk_rope_store) and K/V[pos] are in the cache.
// (parameter order = kernarg layout: everything the prologue needs sits in the first 64-B line)
// DM = decode_mode as a template constant: a runtime branch between the q loads and the K/V stream made the
// wait-count pass drain the q loads at the join, before the K/V loads were issued
// LEAN (batched decode, several blocks per CU): at most 4 groups per wave pass and a 4-partial combine chunk, so
// the kernel fits 128 VGPRs and 4 blocks share a CU (every block of a batch-32 launch resident at once)
// The decode / causal attention of one (kv head g, key split sp, token m) block up to the merge of its waves:
// returns false for a split past the active ones (block-uniform, nothing computed); otherwise wave 0 leaves the
// split's softmax state in (M, L, o) for lane -> head j = lane >> 5, dims [d0, d0 + 4) (d0 = 4 (lane & 31)).
// Shared by k_attn_block (partials + last-arriver combine) and k_attn_o (fused decode: every split combines, then
// multiplies its slice of the o projection).
template <int DM, int LEAN, bool PRE = false, int NW = AWV, bool LPF = false>
__device__ __forceinline__ bool attn_split_merge(int g, int sp, int m, int pos, int seq, int nsplit, int H, int KV,
                                                 int64_t seq_stride, int64_t head_stride, __half* __restrict__ kc,
                                                 __half* __restrict__ vc, const float* __restrict__ qsrc,
                                                 const float* __restrict__ qn, const float* __restrict__ kn,
                                                 const float* __restrict__ rcos, const float* __restrict__ rsin, float eps,
                                                 float scale, int& n_active_out, int& j, int& d0, float& M, float& L,
                                                 float4& o, const AttnQIn* pre = nullptr, const int4* pk = nullptr,
                                                 const int4* pv = nullptr) {
  static_assert(!PRE || LEAN, "attn_split_merge: preloaded K/V with lean passes only (NI <= 4)");
  constexpr int D = 128;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n_keys = pos + 1;
  const int n_groups = (n_keys + 3) >> 2;
  // groups per split = ceil(n_groups / nsplit) without an integer-division sequence (exact below 2^24)
  const int gps = max(AMIN_G, (int)ceilf((float)n_groups / (float)nsplit));
  // n_active = ceil(n_groups / gps) without an integer-division sequence (gps <= n_groups < 2^24: exact)
  int n_active = (int)ceilf((float)n_groups / (float)gps);
  n_active_out = n_active;
  if (sp >= n_active) return false;                                // uniform over the block
  const int gb = sp * gps, ge = min(n_groups, gb + gps);           // this split's groups [gb, ge)
  STAMP(1);
  __half* kb = kc + (int64_t)seq * seq_stride + g * head_stride;
  __half* vb = vc + (int64_t)seq * seq_stride + g * head_stride;
  __shared__ float s_q[NW][GQ][D];          // per-wave q (scaled, roped) in natural dim order
  __shared__ float s_kn[D], s_vn[D];        // fresh K/V row (decode)
  __shared__ float s_ml[NW][GQ][2];
  static_assert(!LPF || (LEAN && !PRE), "attn_split_merge: LDS prefetch with lean passes only");
  // LPF: per-wave K/V slots [2][4 groups][64 lanes] of 16 B; the per-wave o partials alias them after the passes
  __shared__ __attribute__((aligned(16))) int4 s_slot[LPF ? NW : 1][2 * 4 * 64];
  __shared__ float s_o_own[LPF ? 1 : NW][GQ][D];  // [wave][head][dim], summed over the wave's 4 key rows
  float(*s_o)[GQ][D] = LPF ? reinterpret_cast<float(*)[GQ][D]>(&s_slot[0][0]) : s_o_own;
  static_assert(!LPF || sizeof(s_slot) >= sizeof(float) * NW * GQ * D, "attn_split_merge: o partials fit the slots");
  const int kq = lane >> 4, dq = lane & 15;
  float mx[GQ], l[GQ], acc[GQ][8];
#pragma unroll
  for (int j = 0; j < GQ; ++j) {
    mx[j] = -INFINITY;
    l[j] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[j][e] = 0.f;
  }
  const int fresh_group = DM ? (pos >> 2) : -1;
  const bool fresh_here = fresh_group >= gb && fresh_group < ge && (fresh_group - gb) % NW == wave;
  const int g0 = gb + wave;
  if (g0 < ge) {
    AttnQIn qi;
    if (DM && pre) {  // the caller loaded the pos-independent inputs ahead of its pos read
      qi = *pre;
      if (!PRE) {  // PRE: the caller loaded the rope row with the first pass's K/V
        qi.c = rcos[(int64_t)pos * 64 + lane];
        qi.sn = rsin[(int64_t)pos * 64 + lane];
      }
    } else if (DM) {
      const float* row = qsrc + (int64_t)m * (H + 2 * KV) * D;
#pragma unroll
      for (int j = 0; j < GQ; ++j) {
        qi.x0[j] = row[(g * GQ + j) * D + lane];
        qi.x1[j] = row[(g * GQ + j) * D + lane + 64];
      }
      qi.c = rcos[(int64_t)pos * 64 + lane];
      qi.sn = rsin[(int64_t)pos * 64 + lane];
      qi.w0 = qn[lane];
      qi.w1 = qn[lane + 64];
      // fresh k/v values: loaded by every wave (clamped addresses, no branch), used by the owner only
      qi.kx0 = row[(H + g) * D + lane];
      qi.kx1 = row[(H + g) * D + lane + 64];
      qi.kw0 = kn[lane];
      qi.kw1 = kn[lane + 64];
      qi.v0 = row[(H + KV + g) * D + lane];
      qi.v1 = row[(H + KV + g) * D + lane + 64];
    } else {
#pragma unroll
      for (int j = 0; j < GQ; ++j) {
        const float* qp = qsrc + ((int64_t)m * H + g * GQ + j) * D;
        qi.x0[j] = qp[lane];
        qi.x1[j] = qp[lane + 64];
      }
    }
    __half* kd = kb + (int64_t)pos * D;
    __half* vd = vb + (int64_t)pos * D;
    const int ni = (ge - g0 + NW - 1) / NW;
    int4* slot = LPF ? &s_slot[wave][0] : nullptr;
    if (ni <= 1)
      attn_wave<1, NW, !LEAN, PRE, LPF>(kb, vb, KV, g0, ge, n_keys, kq, dq, lane, DM != 0, fresh_here, pos, eps, scale,
                                        qi, kd, vd, s_q[wave], s_kn, s_vn, mx, l, acc, pk, pv, slot);
    else if (ni <= 2)
      attn_wave<2, NW, !LEAN, PRE, LPF>(kb, vb, KV, g0, ge, n_keys, kq, dq, lane, DM != 0, fresh_here, pos, eps, scale,
                                        qi, kd, vd, s_q[wave], s_kn, s_vn, mx, l, acc, pk, pv, slot);
    else if (ni <= 4 || LEAN)
      attn_wave<4, NW, !LEAN, PRE, LPF>(kb, vb, KV, g0, ge, n_keys, kq, dq, lane, DM != 0, fresh_here, pos, eps, scale,
                                        qi, kd, vd, s_q[wave], s_kn, s_vn, mx, l, acc, pk, pv, slot);
    else
      attn_wave<8, NW, !LEAN>(kb, vb, KV, g0, ge, n_keys, kq, dq, lane, DM != 0, fresh_here, pos, eps, scale, qi, kd, vd,
                       s_q[wave], s_kn, s_vn, mx, l, acc);
  }
  // publish per-wave (m, l) and o summed over the wave's 4 key rows (m is wave-uniform, so the rows add
  // unscaled): permlane32_swap pairs fold rows {r, r^2}, permlane16_swap pairs fold {r, r^1}; afterwards
  // red[k] of a lane in row r holds element t = 4k + 2(r&1) + (r>>1) of acc (t = 8 head + dim-in-lane).
  if constexpr (LPF) {  // the o partials overwrite the slots: no DMA of any wave may still land there
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  float red[4];
  {
    float h8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float a = acc[(2 * i) >> 3][(2 * i) & 7], b = acc[(2 * i + 1) >> 3][(2 * i + 1) & 7];
      const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
      h8[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(h8[2 * k]), __float_as_uint(h8[2 * k + 1]),
                                                      false, false);
      red[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int t = 4 * k + 2 * (kq & 1) + (kq >> 1);
    s_o[wave][t >> 3][dq * 8 + (t & 7)] = red[k];
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < GQ; ++j) {
      s_ml[wave][j][0] = mx[j];
      s_ml[wave][j][1] = l[j];
    }
  }
  STAMP(7);
  __syncthreads();
  if (wave != 0) return true;
  STAMP(8);
  // wave 0 merges the waves: lane -> head j = lane >> 5, dims [4 (lane & 31), +4)
  j = lane >> 5;
  d0 = (lane & 31) * 4;
  M = -INFINITY;
#pragma unroll
  for (int w = 0; w < NW; ++w) M = fmaxf(M, s_ml[w][j][0]);
  L = 0.f;
  o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const float mw = s_ml[w][j][0];
    const float wt = mw == -INFINITY ? 0.f : __expf(mw - M);
    L += wt * s_ml[w][j][1];
    const float4 t = *reinterpret_cast<const float4*>(&s_o[w][j][d0]);
    o.x += wt * t.x;
    o.y += wt * t.y;
    o.z += wt * t.z;
    o.w += wt * t.w;
  }
  return true;
}

// Combine of the n_active split partials (sc1 stores, read with sc1 loads) of one (token, kv head): wave w folds splits
// [4 w, 4 w + 4) (one 4-KB hop per wave rather than a 16-KB hop through one wave: B of the fused layer 7.74 -> 7.45 us),
// wave 0 merges the 4 wave states in wave order and returns the normalised output of head lane >> 5, dims
// [4 (lane & 31), +4) (other waves: unspecified). Every wave of the block must call it. Shared by k_attn_block and
// k_attn_o, so the fused and the 5-launch layers combine identically.
static_assert(ASPLIT == 4 * AWV, "combine_splits: 4 splits per wave");
typedef float cf4v __attribute__((ext_vector_type(4)));
// The fold of combine_splits: pml[t] = {m0, l0, m1, l1}, po[t] = o[head lane >> 5][4 (lane & 31), +4) of split
// 4 wave + t (entries past n_active are ignored). Shared with the granule form of the two-launch layer.
__device__ __forceinline__ float4 combine_fold(const cf4v* pml, const cf4v* po, int n_active, int wave, int lane) {
  typedef cf4v f4v;
  constexpr int SPW = ASPLIT / AWV;
  __shared__ float s_cml[AWV][64][2];
  __shared__ __attribute__((aligned(16))) f4v s_co[AWV][64];
  const int jj = lane >> 5;
  {
    float MM = -INFINITY;
#pragma unroll
    for (int t = 0; t < SPW; ++t)
      if (wave * SPW + t < n_active) MM = fmaxf(MM, jj ? pml[t].z : pml[t].x);
    float LL = 0.f;
    f4v oo = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < SPW; ++t) {
      if (wave * SPW + t < n_active) {
        const float mt = jj ? pml[t].z : pml[t].x;
        const float wt = mt == -INFINITY ? 0.f : __expf(mt - MM);
        LL += wt * (jj ? pml[t].w : pml[t].y);
        oo += wt * po[t];
      }
    }
    s_cml[wave][lane][0] = MM;
    s_cml[wave][lane][1] = LL;
    s_co[wave][lane] = oo;
  }
  __syncthreads();
  float MM = -INFINITY;
#pragma unroll
  for (int w = 0; w < AWV; ++w) MM = fmaxf(MM, s_cml[w][lane][0]);
  float LL = 0.f;
  f4v oo = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int w = 0; w < AWV; ++w) {
    const float mw = s_cml[w][lane][0];
    const float wt = mw == -INFINITY ? 0.f : __expf(mw - MM);
    LL += wt * s_cml[w][lane][1];
    oo += wt * s_co[w][lane];
  }
  return make_float4(oo.x / LL, oo.y / LL, oo.z / LL, oo.w / LL);
}
__device__ __forceinline__ float4 combine_splits(const __amdgpu_buffer_rsrc_t& rs, int n_active, int wave, int lane) {
  constexpr int D = 128, SPW = ASPLIT / AWV;
  const int jj = lane >> 5, dd = (lane & 31) * 4;
  cf4v pml[SPW], po[SPW];
#pragma unroll
  for (int t = 0; t < SPW; ++t) {
    const int tt = min(wave * SPW + t, n_active - 1);  // clamped duplicates past n_active are not folded
    pml[t] = ld_sc1_f4(rs, (tt * APART + GQ * D) * 4);
    po[t] = ld_sc1_f4(rs, (tt * APART + jj * D + dd) * 4);
  }
  return combine_fold(pml, po, n_active, wave, lane);
}

// NW = 16 (batched decode, one block per (token, kv head), n_active == 1 only): the 16 waves of one CU share the key
// range, merged in LDS; no split partials, no combine hop
template <int DM, int LEAN, int NW = AWV, bool LPF = false>
__global__ __launch_bounds__(NW * 64, NW > AWV ? 1 : LEAN ? 4 : 1) void k_attn_block(const int* __restrict__ tok_seq, const int* __restrict__ tok_pos,
                                                         int nsplit, int decode_mode, int H, int KV,
                                                         int64_t seq_stride, int64_t head_stride,
                                                         __half* __restrict__ kc,
                                                         __half* __restrict__ vc, const float* __restrict__ qsrc,
                                                         const float* __restrict__ qn, const float* __restrict__ kn,
                                                         const float* __restrict__ rcos, const float* __restrict__ rsin,
                                                         float eps, float scale, float* __restrict__ out,
                                                         int* __restrict__ counters, float* __restrict__ partials,
                                                         int8_t* __restrict__ qout, float* __restrict__ dout) {
  constexpr int D = 128;
  const int g = blockIdx.x, sp = blockIdx.y, m = blockIdx.z;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int pos = tok_pos[m];
  const int seq = tok_seq[m];
  // pos "depends" on seq and on the pointer arguments: the two index loads and every kernarg line are
  // fetched together, before the first use (otherwise each is a serial scalar-load latency)
  asm volatile("" : "+s"(pos) : "s"(seq), "s"(qsrc), "s"(kc), "s"(vc), "s"(rcos), "s"(rsin), "s"(qn), "s"(kn),
               "s"(seq_stride), "s"(head_stride), "s"(out), "s"(partials));
  STAMP(0);
  int n_active, j, d0;
  float M, L;
  float4 o;
  if (!attn_split_merge<DM, LEAN, false, NW, LPF>(g, sp, m, pos, seq, nsplit, H, KV, seq_stride, head_stride, kc, vc,
                                                   qsrc, qn, kn, rcos, rsin, eps, scale, n_active, j, d0, M, L, o))
    return;
  float* op = out + ((int64_t)m * H + g * GQ + j) * D + d0;  // j, d0: wave 0's lane map
  if (NW != AWV || n_active == 1) {  // NW != AWV: the host launches one split
    if (wave != 0) return;
    const float4 r = make_float4(o.x / L, o.y / L, o.z / L, o.w / L);
    *reinterpret_cast<float4*>(op) = r;
    if (qout) store_q8_row4(qout, dout, (int64_t)m * H * D + (g * GQ + j) * D + d0, lane, r);
    STAMP(9);
    return;
  }
  // split partial -> global (sc1: bypass L1, the combiner reads it from another CU)
  typedef float f4v __attribute__((ext_vector_type(4)));
  float* pbase = partials + ((int64_t)m * KV + g) * ASPLIT * APART;
  const __amdgpu_buffer_rsrc_t rs = buf_rsrc(pbase, ASPLIT * APART * 4);
  __shared__ int s_last;
  if (wave == 0) {
    const f4v ov = {o.x, o.y, o.z, o.w};
    st_sc1_f4(ov, rs, (sp * APART + j * D + d0) * 4);
    const float M1 = lane_f(M, 32), L1 = lane_f(L, 32);  // head 1's (M, L) live in lanes 32..63
    if (lane == 0) {
      const f4v ml = {M, L, M1, L1};
      st_sc1_f4(ml, rs, (sp * APART + GQ * D) * 4);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    STAMP(11);
    if (lane == 0)
      s_last = __hip_atomic_fetch_add(counters + (m * KV + g) * CNT_LINE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               n_active - 1;
  }
  __syncthreads();
  if (!s_last) return;
  STAMP(9);
  // last split: every wave folds a quarter of the partials (combine_splits), wave 0 writes the row
  const float4 r = combine_splits(rs, n_active, wave, lane);
  if (wave != 0) return;
  *reinterpret_cast<float4*>(op) = r;
  if (qout) store_q8_row4(qout, dout, (int64_t)m * H * D + (g * GQ + j) * D + d0, lane, r);
  if (lane == 0) __hip_atomic_store(counters + (m * KV + g) * CNT_LINE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  STAMP(10);
}

// ------------------------------------------------------------------------------------------------
// Prefill attention over query tiles (multi-sequence prefill batches): block = (tile of up to 64 consecutive rows of
// ONE sequence, kv head g); its 2 query heads x 64 rows = 128 query slots share every K/V tile (32 keys, fp16 cache ->
// f32 LDS), so K/V bytes are read once per 64 rows instead of once per row (k_attn_block). Flash style on exact-f32
// MFMA (v_mfma_f32_32x32x2_f32, as the encoder's k_attn_f32): S^T = K . Q^T with the query slot on the lane, online
// softmax in registers, P^T straight into O^T += V^T . P^T. Causal: key k of row r counts iff k <= pos(r). Writes the
// rows (f32) and their q8_0 blocks for the o GEMM. Tiles: int4 {row0, n_rows, seq, 0} from the host.
constexpr int PAQ = 128, PAK = 32, PAD = 128, PAS = PAD + 8;  // query slots, keys per tile, head dim, LDS row stride

__global__ __launch_bounds__(256, 2) void k_attn_prefill(const int4* __restrict__ tiles, const int* __restrict__ tok_pos,
                                                      int H, int KV, int64_t seq_stride, int64_t head_stride,
                                                      const __half* __restrict__ kc, const __half* __restrict__ vc,
                                                      const float* __restrict__ q, float scale, float* __restrict__ out,
                                                      int8_t* __restrict__ qout, float* __restrict__ dout) {
  __shared__ __attribute__((aligned(16))) float smem[2 * 2 * PAK * PAS];  // K, V x 2 stages; O staging reuses it
  __shared__ float s_l[PAQ];
  const int4 td = tiles[blockIdx.x];
  const int row0 = td.x, nr = td.y, seq = td.z, g = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int hh = wave >> 1, rr = (wave & 1) * 32 + r;  // this lane's query slot: head 2 g + hh, tile row rr
  const int rrc = min(rr, nr - 1);
  const int pos = tok_pos[row0 + rrc];
  const int pmax = tok_pos[row0 + nr - 1];             // rows of a tile are consecutive positions
  const __half* kb = kc + (int64_t)seq * seq_stride + g * head_stride;
  const __half* vb = vc + (int64_t)seq * seq_stride + g * head_stride;
  float qreg[PAD / 2];
  {
    const float* p = q + (int64_t)(row0 + rrc) * H * PAD + (2 * g + hh) * PAD + h * (PAD / 2);
#pragma unroll
    for (int d = 0; d < PAD / 2; d += 4) {
      const float4 v = *reinterpret_cast<const float4*>(p + d);
      qreg[d] = v.x * scale; qreg[d + 1] = v.y * scale; qreg[d + 2] = v.z * scale; qreg[d + 3] = v.w * scale;
    }
  }
  // staging: 32 keys x 128 dims fp16 = 512 chunks of 8 halves per K (and per V) tile, 2 per thread
  auto load = [&](int kt, uint4 (&pk)[2], uint4 (&pv)[2]) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int f = threadIdx.x + 256 * c, key = min(kt * PAK + (f >> 4), pmax), d8 = f & 15;
      pk[c] = *reinterpret_cast<const uint4*>(kb + (int64_t)key * PAD + 8 * d8);
      pv[c] = *reinterpret_cast<const uint4*>(vb + (int64_t)key * PAD + 8 * d8);
    }
  };
  auto store = [&](int stage, const uint4 (&pk)[2], const uint4 (&pv)[2]) {
    float* ks_ = smem + stage * 2 * PAK * PAS;
    float* vs_ = ks_ + PAK * PAS;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int f = threadIdx.x + 256 * c, key = f >> 4, d8 = f & 15;
      const __half* hk = reinterpret_cast<const __half*>(&pk[c]);
      const __half* hv = reinterpret_cast<const __half*>(&pv[c]);
      float4 k0, k1, v0, v1;
      k0 = make_float4(__half2float(hk[0]), __half2float(hk[1]), __half2float(hk[2]), __half2float(hk[3]));
      k1 = make_float4(__half2float(hk[4]), __half2float(hk[5]), __half2float(hk[6]), __half2float(hk[7]));
      v0 = make_float4(__half2float(hv[0]), __half2float(hv[1]), __half2float(hv[2]), __half2float(hv[3]));
      v1 = make_float4(__half2float(hv[4]), __half2float(hv[5]), __half2float(hv[6]), __half2float(hv[7]));
      *reinterpret_cast<float4*>(ks_ + key * PAS + 8 * d8) = k0;
      *reinterpret_cast<float4*>(ks_ + key * PAS + 8 * d8 + 4) = k1;
      *reinterpret_cast<float4*>(vs_ + key * PAS + 8 * d8) = v0;
      *reinterpret_cast<float4*>(vs_ + key * PAS + 8 * d8 + 4) = v1;
    }
  };
  f32x16 o[PAD / 32];
#pragma unroll
  for (int i = 0; i < PAD / 32; ++i) o[i] = f32x16{};
  float m_run = -INFINITY, l_run = 0.f;
  const int n_kt = pmax / PAK + 1;
  uint4 pk[2], pv[2];
  load(0, pk, pv);
  store(0, pk, pv);
  __syncthreads();
  for (int kt = 0; kt < n_kt; ++kt) {
    const int stage = kt & 1;
    if (kt + 1 < n_kt) load(kt + 1, pk, pv);
    const float* ks_ = smem + stage * 2 * PAK * PAS;
    const float* vs_ = ks_ + PAK * PAS;
    f32x16 sc = {};
#pragma unroll
    for (int c = 0; c < PAD / 2; c += 4) {
      const float4 kv = *reinterpret_cast<const float4*>(ks_ + r * PAS + h * (PAD / 2) + c);
      sc = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.x, qreg[c], sc, 0, 0, 0);
      sc = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.y, qreg[c + 1], sc, 0, 0, 0);
      sc = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.z, qreg[c + 2], sc, 0, 0, 0);
      sc = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.w, qreg[c + 3], sc, 0, 0, 0);
    }
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int key = kt * PAK + (t & 3) + 8 * (t >> 2) + 4 * h;
      const float v = key <= pos ? sc[t] : -INFINITY;
      sc[t] = v;
      mt = fmaxf(mt, v);
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float m_new = fmaxf(m_run, mt);
    const float alpha = m_run == -INFINITY ? 0.f : __expf(m_run - m_new);
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const float pr = sc[t] == -INFINITY ? 0.f : __expf(sc[t] - m_new);
      sc[t] = pr;
      ls += pr;
    }
    ls += __shfl_xor(ls, 32, 64);
    l_run = l_run * alpha + ls;
    m_run = m_new;
#pragma unroll
    for (int i = 0; i < PAD / 32; ++i) o[i] *= alpha;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int kl = (t & 3) + 8 * (t >> 2) + 4 * h;
#pragma unroll
      for (int i = 0; i < PAD / 32; ++i)
        o[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(vs_[kl * PAS + i * 32 + r], sc[t], o[i], 0, 0, 0);
    }
    if (kt + 1 < n_kt) store(stage ^ 1, pk, pv);
    __syncthreads();
  }
  // O^T (d on registers, slot on lanes) -> LDS [slot][d]; slot = hh 64 + rr
  float* so = smem;  // 128 x (128 + 4) floats = 67.6 KB > the K/V stages: use it in two halves by head
  constexpr int OS = PAD + 4;
  static_assert(64 * OS <= 2 * 2 * PAK * PAS, "k_attn_prefill: O staging per head must fit the K/V stages");
  if (h == 0) s_l[hh * 64 + rr] = l_run;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    if (hh == half) {
#pragma unroll
      for (int i = 0; i < PAD / 32; ++i)
#pragma unroll
        for (int t = 0; t < 16; ++t) so[rr * OS + i * 32 + (t & 3) + 8 * (t >> 2) + 4 * h] = o[i][t];
    }
    __syncthreads();
    // 64 rows x 32 float4 = 2048 float4, 8 per thread; 8 consecutive threads = one 32-dim q8_0 block
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int f = threadIdx.x + 256 * c, row = f >> 5, d4 = f & 31;
      const float inv = 1.0f / s_l[half * 64 + row];
      float4 v = *reinterpret_cast<const float4*>(so + row * OS + 4 * d4);
      v.x *= inv; v.y *= inv; v.z *= inv; v.w *= inv;
      const int orow = row0 + min(row, nr - 1);
      const int64_t e = (int64_t)orow * H * PAD + (2 * g + half) * PAD + 4 * d4;
      if (row < nr) {  // whole 32-thread rows: the 8-lane groups of store_q8_row4 stay together
        *reinterpret_cast<float4*>(out + e) = v;
        if (qout) store_q8_row4(qout, dout, e, threadIdx.x, v);
      }
    }
    __syncthreads();
  }
}

// The same tiles on f16 MFMAs (v_mfma_f32_32x32x16_f16, 16x the f32 MFMA rate): the cache's K and V are fp16 values,
// so they are exact f16 operands. S^T = K . Q^T takes q split into f16 hi + lo (q * d^-0.5, then times 2^8 so the lo
// part stays out of the f16 subnormals; the scores are scaled back by 2^-8, exactly): two MFMAs per 16 dims, products
// exact, q kept to 22 of f32's 24 bits. O^T += V^T . P^T takes P^T straight from the S accumulator split into f16
// hi + lo (as the fp16 encoder attention, attn_f32.hip) with V^T fragments from ds_read_b64_tr_b16. Masking, online
// softmax and the epilogue are k_attn_prefill's; per row the result depends only on its own keys (row-local).
typedef _Float16 f16x8p __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4p __attribute__((ext_vector_type(4)));
typedef short v4i16p __attribute__((ext_vector_type(4)));
typedef float f32x8v __attribute__((ext_vector_type(8)));
constexpr int PHK = PAD + 8, PHV = PAD + 32;  // K rows: 16-B reads of 16 rows on distinct banks; V rows: the tr reads'
constexpr int PH_STAGE = PAK * PHK + PAK * PHV;  // halves per stage (K plane, V plane)

__global__ __launch_bounds__(256, 2) void k_attn_prefill_h(const int4* __restrict__ tiles, const int* __restrict__ tok_pos,
                                                        int H, int KV, int64_t seq_stride, int64_t head_stride,
                                                        const __half* __restrict__ kc, const __half* __restrict__ vc,
                                                        const float* __restrict__ q, float scale, float* __restrict__ out,
                                                        int8_t* __restrict__ qout, float* __restrict__ dout) {
  constexpr int OS = PAD + 4;
  constexpr int SMEM_F = (2 * PH_STAGE / 2 > 64 * OS) ? 2 * PH_STAGE / 2 : 64 * OS;
  __shared__ __attribute__((aligned(16))) float smem[SMEM_F];  // 2 stages of f16 K / V planes; O staging reuses it
  __shared__ float s_l[PAQ];
  const int4 td = tiles[blockIdx.x];
  const int row0 = td.x, nr = td.y, seq = td.z, g = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int hh = wave >> 1, rr = (wave & 1) * 32 + r;  // this lane's query slot: head 2 g + hh, tile row rr
  const int rrc = min(rr, nr - 1);
  const int pos = tok_pos[row0 + rrc];
  const int pmax = tok_pos[row0 + nr - 1];
  const __half* kb = kc + (int64_t)seq * seq_stride + g * head_stride;
  const __half* vb = vc + (int64_t)seq * seq_stride + g * head_stride;
  f16x8p qh[PAD / 16], ql[PAD / 16];  // k-step st: dims 16 st + 8 h + [0, 8) of this lane's slot
  {
    const float* p = q + (int64_t)(row0 + rrc) * H * PAD + (2 * g + hh) * PAD + 8 * h;
#pragma unroll
    for (int st = 0; st < PAD / 16; ++st) {
      const float4 a = *reinterpret_cast<const float4*>(p + 16 * st);
      const float4 b = *reinterpret_cast<const float4*>(p + 16 * st + 4);
      const f32x8v x = f32x8v{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w} * scale * 256.0f;
      qh[st] = __builtin_convertvector(x, f16x8p);
      ql[st] = __builtin_convertvector(x - __builtin_convertvector(qh[st], f32x8v), f16x8p);
    }
  }
  // staging: 32 keys x 128 dims fp16 per K (and V) tile = 512 chunks of 8 halves, 2 per thread (chunk f = t + 256 c:
  // key f >> 4, dims 8 (f & 15) + [0, 8)); plain registers, not arrays (hipcc kept lambda-captured arrays in scratch)
  const int ld_key = threadIdx.x >> 4, ld_d8 = threadIdx.x & 15;
  uint4 pk0, pk1, pv0, pv1;
#define PFH_LOAD(kt)                                                                               \
  do {                                                                                             \
    const int k0_ = min((kt) * PAK + ld_key, pmax), k1_ = min((kt) * PAK + 16 + ld_key, pmax);     \
    pk0 = *reinterpret_cast<const uint4*>(kb + (int64_t)k0_ * PAD + 8 * ld_d8);                    \
    pv0 = *reinterpret_cast<const uint4*>(vb + (int64_t)k0_ * PAD + 8 * ld_d8);                    \
    pk1 = *reinterpret_cast<const uint4*>(kb + (int64_t)k1_ * PAD + 8 * ld_d8);                    \
    pv1 = *reinterpret_cast<const uint4*>(vb + (int64_t)k1_ * PAD + 8 * ld_d8);                    \
  } while (0)
  _Float16* sh = reinterpret_cast<_Float16*>(smem);
#define PFH_STORE(stage)                                                                           \
  do {                                                                                             \
    _Float16* ks_w = sh + (stage) * PH_STAGE;                                                      \
    _Float16* vs_w = ks_w + PAK * PHK;                                                             \
    *reinterpret_cast<uint4*>(ks_w + ld_key * PHK + 8 * ld_d8) = pk0;                              \
    *reinterpret_cast<uint4*>(vs_w + ld_key * PHV + 8 * ld_d8) = pv0;                              \
    *reinterpret_cast<uint4*>(ks_w + (16 + ld_key) * PHK + 8 * ld_d8) = pk1;                       \
    *reinterpret_cast<uint4*>(vs_w + (16 + ld_key) * PHV + 8 * ld_d8) = pv1;                       \
  } while (0)
  f32x16 o[PAD / 32];
#pragma unroll
  for (int i = 0; i < PAD / 32; ++i) o[i] = f32x16{};
  float m_run = -INFINITY, l_run = 0.f;
  const int n_kt = pmax / PAK + 1;
  PFH_LOAD(0);
  PFH_STORE(0);
  __syncthreads();
  for (int kt = 0; kt < n_kt; ++kt) {
    const int stage = kt & 1;
    if (kt + 1 < n_kt) PFH_LOAD(kt + 1);
    const _Float16* ks_ = sh + stage * PH_STAGE;
    const _Float16* vs_ = ks_ + PAK * PHK;
    f32x16 sc = {};
#pragma unroll
    for (int st = 0; st < PAD / 16; ++st) {
      const f16x8p kf = *reinterpret_cast<const f16x8p*>(ks_ + r * PHK + 16 * st + 8 * h);
      sc = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, ql[st], sc, 0, 0, 0);
      sc = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qh[st], sc, 0, 0, 0);
    }
    sc *= 1.0f / 256.0f;
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int key = kt * PAK + (t & 3) + 8 * (t >> 2) + 4 * h;
      const float v = key <= pos ? sc[t] : -INFINITY;
      sc[t] = v;
      mt = fmaxf(mt, v);
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float m_new = fmaxf(m_run, mt);
    const float alpha = m_run == -INFINITY ? 0.f : __expf(m_run - m_new);
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const float pr = sc[t] == -INFINITY ? 0.f : __expf(sc[t] - m_new);
      sc[t] = pr;
      ls += pr;
    }
    ls += __shfl_xor(ls, 32, 64);
    l_run = l_run * alpha + ls;
    m_run = m_new;
#pragma unroll
    for (int i = 0; i < PAD / 32; ++i) o[i] *= alpha;
    // P^T k-step s2 = accumulator registers 8 s2 .. 8 s2 + 7 (keys 16 s2 + 8 (j >> 2) + 4 h + (j & 3))
#pragma unroll
    for (int s2 = 0; s2 < PAK / 16; ++s2) {
      f16x8p ph, pl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ph[j] = (_Float16)sc[8 * s2 + j];
        pl[j] = (_Float16)(sc[8 * s2 + j] - (float)ph[j]);
      }
      const int gq = lane >> 4, key = 16 * s2 + 4 * (gq >> 1) + ((lane >> 2) & 3);
#pragma unroll
      for (int i = 0; i < PAD / 32; ++i) {
        const int off = key * PHV + 32 * i + 16 * (gq & 1) + 4 * (lane & 3);
        const f16x4p h0 = __builtin_bit_cast(
            f16x4p, __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16p*)(vs_ + off)));
        const f16x4p h1 = __builtin_bit_cast(
            f16x4p,
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16p*)(vs_ + off + 8 * PHV)));
        const f16x8p vh = f16x8p{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        o[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, pl, o[i], 0, 0, 0);
        o[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, ph, o[i], 0, 0, 0);
      }
    }
    if (kt + 1 < n_kt) PFH_STORE(stage ^ 1);
    __syncthreads();
  }
#undef PFH_LOAD
#undef PFH_STORE
  // epilogue: k_attn_prefill's (O^T has the same accumulator layout: dims on registers, slots on lanes)
  float* so = smem;
  if (h == 0) s_l[hh * 64 + rr] = l_run;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    if (hh == half) {
#pragma unroll
      for (int i = 0; i < PAD / 32; ++i)
#pragma unroll
        for (int t = 0; t < 16; ++t) so[rr * OS + i * 32 + (t & 3) + 8 * (t >> 2) + 4 * h] = o[i][t];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int f = threadIdx.x + 256 * c, row = f >> 5, d4 = f & 31;
      const float inv = 1.0f / s_l[half * 64 + row];
      float4 v = *reinterpret_cast<const float4*>(so + row * OS + 4 * d4);
      v.x *= inv; v.y *= inv; v.z *= inv; v.w *= inv;
      const int orow = row0 + min(row, nr - 1);
      const int64_t e = (int64_t)orow * H * PAD + (2 * g + half) * PAD + 4 * d4;
      if (row < nr) {
        *reinterpret_cast<float4*>(out + e) = v;
        if (qout) store_q8_row4(qout, dout, e, threadIdx.x, v);
      }
    }
    __syncthreads();
  }
}

int g_attn_pf_f16 = 1;  // query-tiled prefill attention on f16 MFMAs (FUNASR_ATTN_PF_F16; 0: exact-f32 MFMAs)

void attn_prefill(const int4* tiles, int n_tiles, const int* tok_pos, int H, int KV, int64_t seq_stride, const __half* kc,
                  const __half* vc, const float* q, float* out, int8_t* qout, float* dout, hipStream_t s, bool f16) {
  FA_REQUIRE(H == KV * GQ, "attn_prefill: n_head must be 2*n_head_kv");
  if (n_tiles <= 0) return;
  hipLaunchKernelGGL(f16 ? k_attn_prefill_h : k_attn_prefill, dim3(n_tiles, KV), dim3(256), 0, s, tiles,
                     tok_pos, H, KV, seq_stride, seq_stride / KV, kc, vc, q, 1.0f / sqrtf(128.0f), out, qout, dout);
}

void attn_block(const float* qsrc, int decode_mode, const float* qn, const float* kn, float eps, const float* rcos,
                const float* rsin, __half* kc, __half* vc, int M, int H, int KV, const int* tok_seq, const int* tok_pos,
                int64_t seq_stride, float* out, const AttnWork& wk, hipStream_t s, int8_t* qout, float* dout,
                int max_splits) {
  FA_REQUIRE(H == KV * GQ, "attn_block: n_head must be 2*n_head_kv");
  FA_REQUIRE(wk.counters && wk.partials && M <= wk.max_tokens && KV <= wk.max_kv, "attn_block: workspace too small");
  const float scale = 1.0f / sqrtf(128.0f);
  // key splits only while (token, kv head) blocks alone leave the chip idle: 16 at batch 1-4, 4 at batch 32, 1 for
  // prefill. Batch 32 measured 14.7-17.0 us for every target of 256-1024 blocks, lean or not (attn_batch.hip): the
  // K/V stream of 512 (sequence, kv head) pairs comes in at ~2.8 TB/s whatever the block shape.
  if (decode_mode && g_attn_wide > 0 && M * KV >= g_attn_wide) {  // one 16-wave block per (token, kv head)
    if (g_attn_ldspf)
      hipLaunchKernelGGL((k_attn_block<1, 1, 16, true>), dim3(KV, 1, M), dim3(16 * 64), 0, s, tok_seq, tok_pos, 1,
                         decode_mode, H, KV, seq_stride, seq_stride / KV, kc, vc, qsrc, qn, kn, rcos, rsin, eps, scale,
                         out, wk.counters, wk.partials, qout, dout);
    else
      hipLaunchKernelGGL((k_attn_block<1, 1, 16>), dim3(KV, 1, M), dim3(16 * 64), 0, s, tok_seq, tok_pos, 1,
                         decode_mode, H, KV, seq_stride, seq_stride / KV, kc, vc, qsrc, qn, kn, rcos, rsin, eps, scale,
                         out, wk.counters, wk.partials, qout, dout);
    return;
  }
  int ns = 1;
  while (ns < std::min(ASPLIT, max_splits) && (ns + 1) * M * KV <= g_attn_blocks) ++ns;
  FA_REQUIRE(ns == 1 || M <= wk.max_split_tokens, "attn_block: split partials workspace too small");
  const bool lean = g_attn_lean >= 0 ? g_attn_lean != 0 : M * KV * ns > 3 * 256;
  auto kern = lean ? (decode_mode ? k_attn_block<1, 1> : k_attn_block<0, 1>)
                   : (decode_mode ? k_attn_block<1, 0> : k_attn_block<0, 0>);
  hipLaunchKernelGGL(kern, dim3(KV, ns, M), dim3(AWV * 64), 0, s, tok_seq, tok_pos, ns, decode_mode,
                     H, KV, seq_stride, seq_stride / KV, kc, vc, qsrc, qn, kn, rcos, rsin, eps, scale, out, wk.counters, wk.partials,
                     qout, dout);
}

// ------------------------------------------------------------------------------------------------
// D0 embedding rows from q8_0 token_embd. fp16_round: numpy f16 product (llama.py:782-784).
__global__ void k_embed(const int8_t* __restrict__ qs, const __half* __restrict__ d, const int* __restrict__ ids, int n,
                        int E, int fp16_round, float* __restrict__ out) {
  const int m = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n || i >= E) return;
  const int64_t row = ids[m];
  const float dv = __half2float(d[row * (E / 32) + i / 32]);
  float v = dv * (float)qs[row * E + i];
  if (fp16_round) v = __half2float(__float2half_rn(v));
  out[(int64_t)m * E + i] = v;
}

__global__ void k_gather_rows(const float* __restrict__ src, const int* __restrict__ rows, int E, float* __restrict__ dst) {
  const int m = blockIdx.y;
  const int64_t r = rows[m];
  for (int i = (blockIdx.x * blockDim.x + threadIdx.x) * 4; i < E; i += gridDim.x * blockDim.x * 4)
    *reinterpret_cast<float4*>(dst + (int64_t)m * E + i) = *reinterpret_cast<const float4*>(src + r * E + i);
}

void gather_rows(const float* src, const int* rows, int n, int E, float* dst, hipStream_t s) {
  FA_REQUIRE(E % 4 == 0, "gather_rows: E % 4");
  if (n > 0) hipLaunchKernelGGL(k_gather_rows, dim3(1, n), dim3(256), 0, s, src, rows, E, dst);
}

// prompt rows assembled on the device (fa_llm_prefill_rows): code >= 0 is row `code` of the caller's rows (uploaded);
// code < 0 an adaptor output row of the last encode: v = -1 - code, clip v >> 16, row v & 0xffff (clip b's rows start
// at row b * ts). A verbatim copy either way, so the rows equal the host concatenation bit for bit.
__global__ void k_prompt_rows(const float* __restrict__ host, const float* __restrict__ audio, int64_t ts,
                              const int* __restrict__ codes, int E, float* __restrict__ dst) {
  const int m = blockIdx.y;
  const int c = codes[m];
  const float* src;
  if (c >= 0) {
    src = host + (int64_t)c * E;
  } else {
    const int v = -1 - c;
    src = audio + ((int64_t)(v >> 16) * ts + (v & 0xffff)) * E;
  }
  for (int i = threadIdx.x * 4; i < E; i += blockDim.x * 4)
    *reinterpret_cast<float4*>(dst + (int64_t)m * E + i) = *reinterpret_cast<const float4*>(src + i);
}

void prompt_rows(const float* host, const float* audio, int64_t ts, const int* codes, int n, int E, float* dst,
                 hipStream_t s) {
  FA_REQUIRE(E % 4 == 0, "prompt_rows: E % 4");
  if (n > 0) hipLaunchKernelGGL(k_prompt_rows, dim3(1, n), dim3(256), 0, s, host, audio, ts, codes, E, dst);
}

void embed_rows(const int8_t* qs, const __half* d, const int* ids, int n, int E, int fp16_round, float* out,
                hipStream_t s) {
  hipLaunchKernelGGL(k_embed, dim3(cdiv(E, 256), n), dim3(256), 0, s, qs, d, ids, n, E, fp16_round, out);
}

// ------------------------------------------------------------------------------------------------
// D6 sampling: the LlamaSampler chain (llama.py:599-605). temperature <= 0 or top_k == 1: greedy (reduce the
// lm_head's per-wave argmax partials). Otherwise top_k -> top_p (min_keep 1) -> temp -> dist, as llama.cpp's
// chain applies them:
//   * top_k keeps the k largest logits (top_k <= 0: all); ties at the k-th value keep the lowest token ids;
//   * top_p < 1 keeps the shortest prefix of those, sorted by logit, whose softmax mass at temperature 1
//     reaches top_p (at least one token); top_p >= 1 is a no-op;
//   * dist draws by inverse CDF over softmax(l / T) of the kept tokens in sorted order. The uniform u is a
//     counter-based hash of (seed, sequence, position), so every (sequence, position) draws afresh, in every
//     call (llama.cpp seeds an mt19937 per call from np.random, decoder.py:89: nondeterministic, so the
//     distribution is the contract, not the draw).
// Fast path (k <= SAMPLE_CAP): the lm_head's per-chunk maxima bound the k-th largest logit from below (k chunks
// have a maximum >= tau), so ONE pass over the logits gathers a superset of the top-k into LDS, where it is
// sorted (bitonic, by logit desc then id asc). Wide path (top_k <= 0 or > SAMPLE_CAP, or a superset larger
// than SAMPLE_CAP): radix selects of the count (top-k) and mass (top-p) thresholds over the whole row, the draw
// in token-id order; ties AT a threshold value are all kept there (real-valued logits: measure zero).
// Sampling parameters are read from device memory, so one captured decode-step graph serves every setting.
constexpr int SAMPLE_CAP = 4096;
constexpr int SAMPLE_T = 1024;  // threads per row (16 waves)

__device__ __forceinline__ uint32_t hash_u32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}
// order-preserving float -> uint32 map (larger float <-> larger key) and back
__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}
// exclusive prefix of v over the block's threads (1024) in thread order; *total = block sum (block-uniform)
template <typename T>
__device__ T block_excl_scan(T v, T* s_w, T* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const T inc = wave_incl_scan(v);
  if (lane == 63) s_w[wave] = inc;
  __syncthreads();
  T off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < SAMPLE_T / 64; ++w) {
    const T x = s_w[w];
    if (w < wave) off += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return off + inc - v;
}
template <typename T>
__device__ T block_sum(T v, T* s_w) {
  T tot;
  (void)block_excl_scan(v, s_w, &tot);
  return tot;
}

// Radix select, descending: over the items get(i, &key, &w) -> valid (i in [0, n), strided over the block),
// the largest key P with weight(key > P) < need <= weight(key >= P) (need clamped to the total weight: the
// smallest valid key then). T = int: counts (k-th largest); T = float: softmax mass (top-p cut).
template <typename T, typename Get>
__device__ uint32_t radix_select_desc(Get get, int n, T need, T* hist, int* s_dig, T* s_need) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t prefix = 0, mask = 0;
  if (threadIdx.x == 0) *s_need = need;
  for (int sh = 24; sh >= 0; sh -= 8) {
    for (int i = threadIdx.x; i < 256; i += SAMPLE_T) hist[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += SAMPLE_T) {
      uint32_t key;
      T w;
      if (get(i, key, w) && (key & mask) == prefix) atomicAdd(&hist[(key >> sh) & 255], w);
    }
    __syncthreads();
    if (wave == 0) {
      T c[4], s = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c[j] = hist[255 - 4 * lane - j];
        s += c[j];
      }
      const T inc = wave_incl_scan(s);
      const T tot = __shfl(inc, 63, 64);
      T nd = *s_need;
      if (nd > tot) nd = tot;
      const T exc = inc - s;
      if (inc >= nd && exc < nd) {  // exactly one lane (nd > 0); a zero total keeps digit 0
        T acc = exc;
        int d = 255 - 4 * lane - 3;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (acc + c[j] >= nd) { d = 255 - 4 * lane - j; break; }
          acc += c[j];
        }
        *s_dig = d;
        *s_need = nd - acc;
      } else if (lane == 0 && !(tot > 0)) {
        *s_dig = 0;
      }
    }
    __syncthreads();
    prefix |= (uint32_t)(*s_dig) << sh;
    mask |= 0xFFu << sh;
    __syncthreads();
  }
  return prefix;
}

constexpr int SAMPLE_QCAP = 1024;  // fast path: chunks whose maximum reaches tau, scanned (else the whole row)
constexpr int SAMPLE_RANK = 256;   // fast path: candidate lists up to this long are rank-sorted (else bitonic)

struct SampleShared {
  unsigned long long list[SAMPLE_CAP];  // fast path: (~key << 32 | id), sorted ascending = logit desc, id asc
  int qch[SAMPLE_QCAP];
  int nq;
  float hist_f[256];
  int hist_i[256];
  float wf[SAMPLE_T / 64];
  int wi[SAMPLE_T / 64];
  float need_f;
  int need_i, dig, cnt, pick, last_thr;
  float argv[16];
  int argi[16];
};

__global__ __launch_bounds__(SAMPLE_T) void k_sample(const float* __restrict__ logits, int64_t ldl, int V,
                                                     const float* __restrict__ pval, const int* __restrict__ pidx,
                                                     int n_part, int chunk, const SampleParams* __restrict__ sp,
                                                     const int* __restrict__ row_seq, const int* __restrict__ row_pos,
                                                     int* __restrict__ step_ctr, int* __restrict__ tok_out,
                                                     int* __restrict__ tok_hist, int hist_stride, EmbedNext en) {
  __shared__ SampleShared S;
  const int m = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float temperature = sp->temperature, top_p = sp->top_p;
  const int top_k = sp->top_k;
  int tok;
  if (temperature <= 0.f || top_k == 1) {
    float v = -INFINITY;
    int i = 0x7fffffff;
    // partials 4 per thread in flight at once (a plain strided loop waits on each load before the next)
    for (int t0 = 0; t0 < n_part; t0 += 4 * SAMPLE_T) {
      float pv[4];
      int pi[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = min(t0 + u * SAMPLE_T + tid, n_part - 1);  // clamped duplicates: argmax unchanged
        pv[u] = pval[(int64_t)m * n_part + t];
        pi[u] = pidx[(int64_t)m * n_part + t];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) argmax_combine(v, i, pv[u], pi[u]);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      float v2 = __shfl_xor(v, o, 64);
      int i2 = __shfl_xor(i, o, 64);
      argmax_combine(v, i, v2, i2);
    }
    if (lane == 0) { S.argv[wave] = v; S.argi[wave] = i; }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < 16; ++w) argmax_combine(v, i, S.argv[w], S.argi[w]);
      S.argi[0] = i;
    }
    __syncthreads();
    tok = S.argi[0];
  } else {
    const float* lg = logits + (int64_t)m * ldl;
    const int k = (top_k <= 0 || top_k >= V) ? V : top_k;
    uint32_t h = hash_u32(sp->seed ^ 0x5BD1E995u);
    h = hash_u32(h ^ ((uint32_t)row_seq[m] * 0x9E3779B9u));
    h = hash_u32(h ^ ((uint32_t)row_pos[m] * 0x85EBCA6Bu + 0x632BE5ABu));
    const float u = (float)(h >> 8) * 5.9604644775390625e-08f;  // [0, 1)
    bool fast = k <= SAMPLE_CAP && k <= n_part && n_part <= 2 * SAMPLE_CAP;
    if (fast) {
      // tau = k-th largest chunk maximum (keys staged in LDS, reusing the candidate list's space)
      uint32_t* pk = reinterpret_cast<uint32_t*>(S.list);
      for (int i = tid; i < n_part; i += SAMPLE_T) pk[i] = fkey(pval[(int64_t)m * n_part + i]);
      if (tid == 0) { S.cnt = 0; S.nq = 0; }
      __syncthreads();
      const uint32_t tau = radix_select_desc<int>(
          [&](int i, uint32_t& key, int& w) { key = pk[i]; w = 1; return true; }, n_part, k, S.hist_i, &S.dig,
          &S.need_i);
      // every logit >= tau lies in a chunk (rows [chunk t, chunk (t + 1)) of partial t) whose maximum is >= tau:
      // gather those chunks (at least k of them, usually about k) and scan only their rows
      for (int i = tid; i < n_part; i += SAMPLE_T)
        if (pk[i] >= tau) {
          const int slot = atomicAdd(&S.nq, 1);
          if (slot < SAMPLE_QCAP) S.qch[slot] = i;
        }
      __syncthreads();
      const int nq = S.nq;  // the chunk keys (in the list's space) are dead from here on
      if (nq <= SAMPLE_QCAP) {
        for (int p = tid; p < nq * chunk; p += SAMPLE_T) {
          const int i = S.qch[p / chunk] * chunk + p % chunk;
          if (i < V) {
            const uint32_t key = fkey(lg[i]);
            if (key >= tau) {
              const int slot = atomicAdd(&S.cnt, 1);
              if (slot < SAMPLE_CAP) S.list[slot] = ((unsigned long long)(~key) << 32) | (uint32_t)i;
            }
          }
        }
      } else {  // many tied chunk maxima: one pass over the row
        for (int i = tid; i < V; i += SAMPLE_T) {
          const uint32_t key = fkey(lg[i]);
          if (key >= tau) {
            const int slot = atomicAdd(&S.cnt, 1);
            if (slot < SAMPLE_CAP) S.list[slot] = ((unsigned long long)(~key) << 32) | (uint32_t)i;
          }
        }
      }
      __syncthreads();
      fast = S.cnt <= SAMPLE_CAP;  // block-uniform
    }
    if (fast) {
      const int c = S.cnt;
      if (c <= SAMPLE_RANK) {
        // rank sort (entries are distinct: ids differ): entry t moves to its rank among the c entries, in one pass
        unsigned long long x = 0;
        int rank = 0;
        if (tid < c) {
          x = S.list[tid];
          for (int j = 0; j < c; ++j) rank += S.list[j] < x;
        }
        __syncthreads();
        if (tid < c) S.list[rank] = x;
        __syncthreads();
      } else {
        int P = 2;
        while (P < c) P <<= 1;
        for (int i = c + tid; i < P; i += SAMPLE_T) S.list[i] = ~0ull;
        __syncthreads();
        for (int size = 2; size <= P; size <<= 1) {
          for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = tid; i < (P >> 1); i += SAMPLE_T) {
              const int pos = 2 * i - (i & (stride - 1));
              const unsigned long long x = S.list[pos], y = S.list[pos + stride];
              if ((x > y) == ((pos & size) == 0)) { S.list[pos] = y; S.list[pos + stride] = x; }
            }
            __syncthreads();
          }
        }
      }
      int nk = min(k, c);
      const float v0 = fkey_inv(~(uint32_t)(S.list[0] >> 32));
      // thread t holds sorted entries [4t, 4t + 4)
      float lv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * tid + j;
        lv[j] = i < nk ? fkey_inv(~(uint32_t)(S.list[i] >> 32)) : -INFINITY;
      }
      if (top_p < 1.f) {
        float w[4], s = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          w[j] = 4 * tid + j < nk ? expf(lv[j] - v0) : 0.f;
          s += w[j];
        }
        const float z1 = block_sum(s, S.wf);
        float ps = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) { w[j] /= z1; ps += w[j]; }
        float tot;
        float cum = block_excl_scan(ps, S.wf, &tot);
        if (tid == 0) S.pick = nk;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          cum += w[j];
          if (4 * tid + j < nk && cum >= top_p) { atomicMin(&S.pick, 4 * tid + j + 1); break; }
        }
        __syncthreads();
        nk = S.pick;
      }
      float e[4], s = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        e[j] = 4 * tid + j < nk ? expf((lv[j] - v0) / temperature) : 0.f;
        s += e[j];
      }
      float z;
      float cum = block_excl_scan(s, S.wf, &z);
      const float target = u * z;
      if (tid == 0) S.pick = nk - 1;
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cum += e[j];
        if (4 * tid + j < nk && cum > target) { atomicMin(&S.pick, 4 * tid + j); break; }
      }
      __syncthreads();
      tok = (int)(uint32_t)S.list[S.pick];
    } else {
      // wide path over the whole row
      float mx = -INFINITY;
      for (int i = tid; i < V; i += SAMPLE_T) mx = fmaxf(mx, lg[i]);
      mx = wave_max(mx);
      if (lane == 0) S.wf[wave] = mx;
      __syncthreads();
      mx = S.wf[0];
      for (int w = 1; w < SAMPLE_T / 64; ++w) mx = fmaxf(mx, S.wf[w]);
      __syncthreads();
      uint32_t keep = 0;
      if (k < V)
        keep = radix_select_desc<int>([&](int i, uint32_t& key, int& w) { key = fkey(lg[i]); w = 1; return true; },
                                      V, k, S.hist_i, &S.dig, &S.need_i);
      if (top_p < 1.f) {
        float s = 0.f;
        for (int i = tid; i < V; i += SAMPLE_T) s += fkey(lg[i]) >= keep ? expf(lg[i] - mx) : 0.f;
        const float z1 = block_sum(s, S.wf);
        const uint32_t kk = keep;
        keep = radix_select_desc<float>(
            [&](int i, uint32_t& key, float& w) {
              key = fkey(lg[i]);
              w = expf(lg[i] - mx);
              return key >= kk;
            },
            V, top_p * z1, S.hist_f, &S.dig, &S.need_f);
      }
      // draw in token-id order: thread t owns ids [t C, t C + C)
      const int C = (V + SAMPLE_T - 1) / SAMPLE_T;
      const int i0 = min(V, tid * C), i1 = min(V, i0 + C);
      float s = 0.f;
      int lastc = -1;
      for (int i = i0; i < i1; ++i)
        if (fkey(lg[i]) >= keep) { s += expf((lg[i] - mx) / temperature); lastc = i; }
      float z;
      const float excl = block_excl_scan(s, S.wf, &z);
      const float target = u * z;
      if (tid == 0) { S.pick = -1; S.last_thr = -1; }
      __syncthreads();
      if (lastc >= 0) atomicMax(&S.last_thr, tid);
      if (s > 0.f && excl <= target && target < excl + s) {
        float acc = excl;
        int pk = lastc;
        for (int i = i0; i < i1; ++i) {
          if (fkey(lg[i]) >= keep) {
            acc += expf((lg[i] - mx) / temperature);
            if (acc > target) { pk = i; break; }
          }
        }
        atomicMax(&S.pick, pk);
      }
      __syncthreads();
      if (S.pick < 0 && tid == S.last_thr) S.pick = lastc;  // target rounded past the total: last candidate
      __syncthreads();
      tok = S.pick;
    }
  }
  tok = min(max(tok, 0), V - 1);  // the gather below indexes token_embd with it: never out of range, whatever the logits
  if (en.x) {
    // decode step tail: the next step's input row (D0, f32 token_embd row) and the position advance ride along,
    // so a step is forward + this launch (the row was consumed by the lm_head launch before this one)
    const int64_t row = tok;
    for (int i = tid; i < en.E; i += SAMPLE_T)
      en.x[(int64_t)m * en.E + i] = __half2float(en.d[row * (en.E / 32) + i / 32]) * (float)en.qs[row * en.E + i];
  }
  if (tid == 0) {
    tok_out[m] = tok;
    const int c = step_ctr ? step_ctr[m] : 0;
    if (tok_hist) tok_hist[(int64_t)m * hist_stride + c] = tok;
    if (en.x) {
      en.tok_pos[m] += 1;
      step_ctr[m] = c + 1;
    }
  }
}

void sample_tokens(const float* logits, int64_t ldl, int V, const float* pval, const int* pidx, int n_part, int chunk,
                   int M, const SampleParams* d_params, const int* row_seq, const int* row_pos, int* step_ctr,
                   int* tok_out, int* tok_hist, int hist_stride, const EmbedNext* en, hipStream_t s) {
  FA_REQUIRE(!en || (step_ctr && en->tok_pos && en->qs && en->d && en->E % 32 == 0), "sample_tokens: embed-next args");
  FA_REQUIRE(d_params && row_seq && row_pos, "sample_tokens: params / row ids");
  FA_REQUIRE(chunk >= 1 && (int64_t)chunk * n_part >= V, "sample_tokens: partial chunks must cover the row");
  hipLaunchKernelGGL(k_sample, dim3(M), dim3(SAMPLE_T), 0, s, logits, ldl, V, pval, pidx, n_part, chunk, d_params, row_seq,
                     row_pos, step_ctr, tok_out, tok_hist, hist_stride, en ? *en : EmbedNext{});
}

// Profiling aid: one wave spins for `us` microseconds (100 MHz reference clock), so an eager host that
// enqueues a profiled decode step gets ahead of the GPU and the event pairs bracket back-to-back kernels.
__global__ void k_delay(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}
void gpu_delay_us(int us, hipStream_t s) { hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, s, (uint64_t)us * 100); }

// advance per-token positions / counters after a decode step
__global__ void k_advance(int* __restrict__ tok_pos, int* __restrict__ step_ctr, int M) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m < M) { tok_pos[m] += 1; step_ctr[m] += 1; }
}
void advance_positions(int* tok_pos, int* step_ctr, int M, hipStream_t s) {
  hipLaunchKernelGGL(k_advance, dim3(cdiv(M, 64)), dim3(64), 0, s, tok_pos, step_ctr, M);
}


// ------------------------------------------------------------------------------------------------
// Fused batch-1 decode layer: three launches per layer instead of five (M = 1; the C2 critical path).
//   A  q|k|v GEMV (k_gemv_q8 with the PS prologue): x = x_mid + dpart[0] + ... + dpart[7], block 0 stores x;
//   B  k_attn_o: decode attention of (kv head g, split sp) (attn_split_merge), partial published; EVERY split of head
//      g waits for all FS splits (in-launch ticket fan-in), combines them itself, quantises the head pair's 256
//      outputs to q8_0 (ggml's per-32 quantisation of the o projection input) and multiplies them into ITS 64-row
//      slice of the o projection, whose weights it prefetched at kernel start:
//      opart[g][rows] = Wo[rows, 256 g : 256 g + 256] . q8(att_g);
//   C  k_ffn_fused: x_mid = x + opart[0] + ... + opart[7] (block 0 stores it), rmsnorm + q8_0, gate|up GEMV +
//      SwiGLU for the block's 12 rows, published; the 32 blocks of its group (384 act rows = 12 q8_0 blocks) wait
//      for each other, quantise the group's act rows and multiply them into the block's 32-row slice of the down
//      projection (prefetched): dpart[group][rows] = Wdown[rows, 384 group : +384] . q8(act_group).
// The next layer's A (or the LM head) completes the residual. A kernel boundary between two dependent GEMVs costs
// 1.5-1.9 us plus the weight stream's first-byte latency (profiles/); the fan-ins here are 16 / 32 blocks
// deep and the slices' weights are already in registers when their inputs arrive. Every block of a launch is
// resident (128 / 256 blocks, at most 2 per CU); every spin is bounded: a timeout sets *err and falls through.

__device__ __forceinline__ void fanin_wait(unsigned* cnt, unsigned n, int* err) {
  __shared__ unsigned s_target;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 payload stores
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_target = (t / n + 1) * n;  // tickets are consumed n at a time, launch after launch (never re-armed)
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const unsigned target = s_target;
    SpinDeadline dl;
    while ((int)(__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (dl.expired()) {
        if (threadIdx.x == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

constexpr int FO_ROWS = 64;  // o-projection rows per split block (E / ASPLIT, E = 1024)

struct AttnOArgs {
  const int* tok_seq;
  const int* tok_pos;
  int H, KV;
  int64_t seq_stride, head_stride;
  __half* kc;
  __half* vc;
  const float* qkv;
  const float* qn;
  const float* kn;
  const float* rcos;
  const float* rsin;
  float eps, scale;
  const int8_t* wo_q;  // o projection [E][H D], engine layout
  const __half* wo_d;
  int E;
  float* opart;        // [KV][E]
  unsigned* cnt;       // [KV][CNT_LINE]
  float* partials;     // [KV][ASPLIT][APART]
  int* err;
  // QKV (two-launch layer): the q|k|v GEMV of the layer runs in the same launch (k_attn_o<true>)
  const float* x;      // residual row (layer 0: the embedded row; else x_mid of the previous layer)
  const float* psum;   // previous layer's down partials [FUSED_PARTS][E] (layer 0: FusedDecodeWork::pzero)
  float* xsum;         // block (0, 0) stores x + sum psum here (the residual stream); nullptr for layer 0
  const float* norm_w; // attn_norm
  const int8_t* wqkv_q;  // q|k|v [(H + 2 KV) D][E], engine layout
  const __half* wqkv_d;
  unsigned* cnt_qkv;   // [KV][CNT_LINE]
  unsigned long long* gqkv;  // FA_QKV_GRANULE: [(H + 2 KV) D] 8-byte granules {value, tag} (zeroed once)
  int dbg_drop;        // test hook (fa_set_debug bit 1): block (0, 0) publishes no q|k|v granules -> fan-in timeout
  unsigned long long* gpart;  // FA_PART_GRANULE: [KV][ASPLIT][APART] split partials as granules {value, tag}
  L2Prefetch pf;       // l2_prefetch (pf_blocks > 0: the last z slab, pf_blocks blocks per kv head)
  int pf_blocks, pf_delay, pf_mask;  // pf_mask (A/B): 1 the FFN weights, 2 the next q|k|v / o weights, 4 the next K/V
};
// FA_QKV_GRANULE = 1: the q|k|v rows go from the 16 producing blocks of a kv head to the same 16 blocks as
// data-tagged granules (tag = this launch's epoch), polled by every consumer thread for its 2 rows and staged in LDS:
// no drain, no ticket, no read-back (the fused FFN's hand-off). 0: sc1 rows + ticket fan-in + sc1 read-back.
#ifndef FA_QKV_GRANULE
#define FA_QKV_GRANULE 1
#endif
// FA_PART_GRANULE = 1 (two-launch layer, A/B only): the attention split partials of a kv head go to the head's 16
// blocks as data-tagged granules too (each consumer lane polls the 8 values per split it folds), replacing the drained
// sc1 stores + ticket fan-in + sc1 read-back; every block still adds one ticket (not waited on) so the counter keeps
// counting launches (the epoch source). Same fold, same order: bit-identical outputs. Measured (scripts/gpu_r3_pg.sh,
// graph-replayed step): AB 12.5-12.9 vs 9.4-9.7 us -- every poll re-reads the block's 16 KB of partials, and those
// reads queue in the consumer CU's memory pipe (MI355X_MICROARCH.md handoff-1to1: granules pay off up to ~4 KB per
// consumer); the ticket fan-in stays the default.
#ifndef FA_PART_GRANULE
#define FA_PART_GRANULE 0
#endif
// FA_KV_EARLY (two-launch layer): where each wave issues its first attention pass's K/V rows (the cached keys do not
// depend on this launch's q|k|v) and the rope row: 0 = in the attention (after the q|k|v hand-off), 1 = after the
// rmsnorm prologue (behind the q|k|v / o weights, ahead of the GEMV dots), 2 = after the q|k|v rows are published
// (ahead of the hand-off poll). Graph-replayed step (scripts/gpu_r3_kv.sh, n_past 330): 2 = 465.6-466.1 us (AB 9.05-9.13),
// 0 = 474.4-479.3 us (AB 9.50-9.64), 1 = 479.6-488.0 us (the K/V requests delay the GEMV's weight loads).
#ifndef FA_KV_EARLY
#define FA_KV_EARLY 2
#endif
#ifndef FA_QKV_POLL
#define FA_QKV_POLL 0
#endif
// FA_ROPE_EARLY (two-launch layer): the rope row at pos loaded at kernel start with the weights (1) or in kv_early,
// after the q|k|v rows are published (0)
#ifndef FA_ROPE_EARLY
#define FA_ROPE_EARLY 0
#endif

constexpr int FQ_ROWS = 32;  // q|k|v rows per split block in the two-launch layer ((GQ + 2) D / ASPLIT)

// FA_KV_EARLY: the wave's first lean pass of attn_split_merge (groups gb + wave + AWV i, i < AKV_PRE, clamped as
// load_kv_groups clamps them) and the rope row at pos, issued ahead of the attention. Splits past n_active and waves
// without groups load nothing (their registers are never read).
__device__ __forceinline__ void kv_early(const AttnOArgs& a, int g, int sp, int pos, int seq, int wave, int lane,
                                         AttnQIn& qpre, int4 (&pk)[AKV_PRE], int4 (&pv)[AKV_PRE]) {
  const int n_keys = pos + 1, n_groups = (n_keys + 3) >> 2;
  const int gps = max(AMIN_G, (int)ceilf((float)n_groups / (float)ASPLIT));
  const int n_active = (int)ceilf((float)n_groups / (float)gps);
#if !FA_ROPE_EARLY
  qpre.c = a.rcos[(int64_t)pos * 64 + lane];
  qpre.sn = a.rsin[(int64_t)pos * 64 + lane];
#endif
  if (sp >= n_active) return;
  const int g0 = sp * gps + wave, ge = min(n_groups, sp * gps + gps);
  if (g0 >= ge) return;
  const __half* kb = a.kc + (int64_t)seq * a.seq_stride + g * a.head_stride;
  const __half* vb = a.vc + (int64_t)seq * a.seq_stride + g * a.head_stride;
  load_kv_groups<AKV_PRE, AWV>(kb, a.KV, g0, FA_KV_CLAMP_OLD ? pos : max(pos - 1, 0), lane >> 4, lane & 15, pk);
  load_kv_groups<AKV_PRE, AWV>(vb, a.KV, g0, FA_KV_CLAMP_OLD ? pos : max(pos - 1, 0), lane >> 4, lane & 15, pv);
}

int g_l2pf_blocks = 16;
int g_l2pf_delay = 50;
int g_l2pf_max_m = 0;  // > 0 (A/B): the slabs with g_l2pf_mask at every batch up to this width; 0: l2pf_small_mask
// Small decode batches (two-launch layer, M = 2-6, one grid slab per token): which prefetch families pay off depends on
// the batch (scripts/gpu_r5_pfm.sh, profiles/r05_exp_l2pf_small_batches.txt, graph-replayed steps, mask 1 the FFN
// weights, 2 the next layer's q|k|v / o weights, 4 its K/V rows): M = 2 none (0.535 vs 0.568-0.580 ms), 3 mask 3 (0.635
// vs 0.645-0.657), 4 none (0.670-0.678 vs 0.699-0.736), 5 mask 3 (0.778 vs 0.864-0.868), 6 mask 3 (0.860 vs
// 0.902-0.904); the K/V family (4) loses at every M > 1 (it loops over the batch's sequences)
static const int l2pf_small_mask[FUSED_MAX_M + 1] = {0, 7, 0, 3, 0, 3, 3, 0, 0};  // M = 7, 8: not measured
int g_l2pf_mask = 7;

// L2 prefetch blocks of the two-launch layer (the last z slab of k_attn_o<true>, after the M token slabs: block
// (g, pb) with pb < pf_blocks <= ASPLIT; kv head g = blockIdx.x).
// After its weight stream the attention launch is a latency chain (hand-offs, attention, split fan-in, o slice) that
// leaves HBM idle for ~6 us. Extra blocks of the launch, dispatched after the 128 compute blocks and placed on XCD g
// by the same round-robin (linear block id % 8), sleep pf_delay ticks and then pull into THIS XCD's L2 the bytes that
// the next two launches' blocks on XCD g will read: the FFN launch's gate|up rows of blocks b = g + 8 i (rows
// [12 b, +12)) and its down rows of slices bi = g + 8 j (all 8 groups: whole rows [32 bi, +32)); the next layer's
// q|k|v rows of kv head g, the o columns [256 g, +256) and head g's K/V rows [0, pos]. LDS-DMA loads into a scratch slot
// (no VGPR results), drained before the block ends. Bytes and results are untouched: a prefetch only moves lines.
// nseg segments of SU 16-B units, STRIDE bytes apart (compile-time shape: the unit -> address map is a multiply-shift)
// FA_L2PF_AUX (A/B builds): cache-policy bits of the prefetch slabs' LDS-DMA loads (0 default; 2 nt)
#ifndef FA_L2PF_AUX
#define FA_L2PF_AUX 0
#endif
template <int NSEG, int SU, int64_t STRIDE>
__device__ __forceinline__ void pf_family(const void* base, int tid, int T, __attribute__((address_space(3))) void* lds) {
  constexpr int U = NSEG * SU;
  for (int u = tid; u < U; u += T) {
    const int seg = u / SU, off = u - seg * SU;
    __builtin_amdgcn_global_load_lds((const void*)((const char*)base + seg * STRIDE + (int64_t)off * 16), lds, 16, 0,
                                     FA_L2PF_AUX);
  }
}

__device__ __forceinline__ void l2_prefetch(const AttnOArgs& a, int g, int pb, int n_tok) {
  __shared__ __attribute__((aligned(16))) int4 s_pf[AWV][64];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)a.pf_delay) __builtin_amdgcn_s_sleep(4);
  const L2Prefetch& p = a.pf;
  const int T = a.pf_blocks * AWV * 64, tid = pb * AWV * 64 + threadIdx.x;
  auto* lds = (__attribute__((address_space(3))) void*)&s_pf[threadIdx.x >> 6][0];
  // the Qwen3-0.6B shape the fused layer requires (host: qkv_attn_o_fused); FR / DR: FF_ROWS / FD_ROWS of the FFN
  // launch (static_assert with their definitions below)
  constexpr int D = 128, E = 1024, F = 3072, H = 16, KV = 8, FR = 12, DR = 32, NBF = F / FR;
  constexpr int ER = E / 32 * 2, FRB = F / 32 * 2;  // scale bytes per row of K = E / K = F
  if (a.pf_mask & 1) {  // the FFN launch (block b on XCD b % 8)
    pf_family<NBF / 8, FR * E / 16, (int64_t)FR * 8 * E>(p.gq + (int64_t)FR * g * E, tid, T, lds);
    pf_family<NBF / 8, FR * E / 16, (int64_t)FR * 8 * E>(p.uq + (int64_t)FR * g * E, tid, T, lds);
    pf_family<NBF / 8, FR * ER / 16, (int64_t)FR * 8 * ER>((const char*)p.gd + (int64_t)FR * g * ER, tid, T, lds);
    pf_family<NBF / 8, FR * ER / 16, (int64_t)FR * 8 * ER>((const char*)p.ud + (int64_t)FR * g * ER, tid, T, lds);
    pf_family<E / DR / 8, DR * F / 16, (int64_t)DR * 8 * F>(p.dq + (int64_t)DR * g * F, tid, T, lds);
    pf_family<E / DR / 8, DR * FRB / 16, (int64_t)DR * 8 * FRB>((const char*)p.dd + (int64_t)DR * g * FRB, tid, T, lds);
  }
  // the last layer (qkv_q == nullptr): the LM head comes next
  if (p.qkv_q && (a.pf_mask & 2)) {  // the next layer's attention launch (kv head g's 16 blocks on XCD g)
    const int rq = GQ * g * D, rk = (H + g) * D, rv = (H + KV + g) * D;
    pf_family<1, GQ * D * E / 16, 0>(p.qkv_q + (int64_t)rq * E, tid, T, lds);
    pf_family<1, D * E / 16, 0>(p.qkv_q + (int64_t)rk * E, tid, T, lds);
    pf_family<1, D * E / 16, 0>(p.qkv_q + (int64_t)rv * E, tid, T, lds);
    pf_family<1, GQ * D * ER / 16, 0>((const char*)p.qkv_d + (int64_t)rq * ER, tid, T, lds);
    pf_family<1, D * ER / 16, 0>((const char*)p.qkv_d + (int64_t)rk * ER, tid, T, lds);
    pf_family<1, D * ER / 16, 0>((const char*)p.qkv_d + (int64_t)rv * ER, tid, T, lds);
    pf_family<E, GQ * D / 16, (int64_t)H * D>(p.o_q + GQ * D * g, tid, T, lds);
    pf_family<E, GQ * D / 32 * 2 / 16, (int64_t)H * D / 32 * 2>((const char*)p.o_d + GQ * D * g / 32 * 2, tid, T, lds);
  }
  if (p.qkv_q && (a.pf_mask & 4)) {  // ... and its K/V rows [0, pos] of kv head g
    for (int m = 0; m < n_tok; ++m) {  // every token of the launch (its own sequence)
      const int pos = a.tok_pos[m], seq = a.tok_seq[m];
      const int64_t kvo = (int64_t)seq * a.seq_stride + (int64_t)g * a.head_stride;
      const int U = (pos + 1) * D * 2 / 16;
      for (int u = tid; u < U; u += T) {
        __builtin_amdgcn_global_load_lds((const void*)(p.kc + kvo + (int64_t)u * 8), lds, 16, 0, FA_L2PF_AUX);
        __builtin_amdgcn_global_load_lds((const void*)(p.vc + kvo + (int64_t)u * 8), lds, 16, 0, FA_L2PF_AUX);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA write may land after the block's LDS is released
}

// QKV = true: the two-launch batch-1 layer. The 16 split blocks of kv head g first compute the 512 q|k|v rows that
// head's attention reads (q heads GQ g .. GQ g + 1, k head g, v head g), FQ_ROWS each, with the prologue and the
// arithmetic of k_gemv_q8<1, 1, true, 0, PS> (x = x_mid + sum dpart, rmsnorm + q8_0 in LDS, exact block dots, the
// same wave_sum per row: bit-identical q|k|v values), publish them with sc1 stores and pass a 16-block fan-in;
// then the attention + o slice of k_attn_o<false>, with the q|k|v inputs read back with sc1 loads. This replaces
// a kernel boundary (A -> B) by a group-local fan-in whose producers are its consumers.
// Token m = blockIdx.z of a small decode batch (two-launch layer, M <= FUSED_MAX_M): every per-token buffer and
// ticket line is offset by m here, so the body reads as the batch-1 kernel (kernel-uniform pointer arithmetic).
template <bool QKV>
__global__ __launch_bounds__(AWV * 64, 1) void k_attn_o(AttnOArgs a0) {
  constexpr int D = 128, FS = ASPLIT;
  typedef float f4v __attribute__((ext_vector_type(4)));
  const int g = blockIdx.x, sp = blockIdx.y, mt = blockIdx.z;
  if (QKV && a0.pf_blocks > 0 && mt == (int)gridDim.z - 1) {  // the L2 prefetch slab (after the M token slabs)
    if (sp < a0.pf_blocks) l2_prefetch(a0, g, sp, mt);
    return;
  }
  AttnOArgs a = a0;
  {
    const int nq = (a.H + 2 * a.KV) * D;
    a.tok_pos += mt;
    a.tok_seq += mt;
    a.qkv += (int64_t)mt * nq;
    a.opart += (int64_t)mt * a.KV * a.E;
    a.cnt += mt * a.KV * CNT_LINE;
    a.partials += (int64_t)mt * a.KV * FS * APART;
    if constexpr (QKV) {
      a.x += (int64_t)mt * a.E;
      a.psum += (int64_t)mt * FUSED_PARTS * a.E;
      if (a.xsum) a.xsum += (int64_t)mt * a.E;
      a.cnt_qkv += mt * a.KV * CNT_LINE;
      a.gqkv += (int64_t)mt * nq;
      if (a.gpart) a.gpart += (int64_t)mt * a.KV * FS * APART;
    }
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  AttnQIn qpre;
  qpre.c = qpre.sn = 0.f;
  // ---- QKV: activation loads, then this wave's 8 q|k|v weight rows (one 1-KB row per load instruction)
  constexpr int QR = FQ_ROWS / AWV;  // rows per wave
  float xv[4], pv[FUSED_PARTS][4], xw[4];
  int4 wq[QKV ? QR : 1];
  float dq[QKV ? QR : 1];
  int qrow0 = 0;  // global q|k|v row of this block's first row
  unsigned ep_qkv = 0;
  if constexpr (QKV) {
    const float4 x4 = *reinterpret_cast<const float4*>(a.x + threadIdx.x * 4);
    xv[0] = x4.x; xv[1] = x4.y; xv[2] = x4.z; xv[3] = x4.w;
#pragma unroll
    for (int p = 0; p < FUSED_PARTS; ++p) {  // layer 0: a zero block (no branch around the loads)
      const float4 f = *reinterpret_cast<const float4*>(a.psum + p * a.E + threadIdx.x * 4);
      pv[p][0] = f.x; pv[p][1] = f.y; pv[p][2] = f.z; pv[p][3] = f.w;
    }
    const float4 w4 = *reinterpret_cast<const float4*>(a.norm_w + threadIdx.x * 4);
    xw[0] = w4.x; xw[1] = w4.y; xw[2] = w4.z; xw[3] = w4.w;
    __builtin_amdgcn_sched_barrier(0);
    // local rows [FQ_ROWS sp, +FQ_ROWS) of head g's list (q head GQ g, q head GQ g + 1, k head g, v head g)
    const int lr0 = FQ_ROWS * sp, seg = lr0 / D, off = lr0 % D;
    qrow0 = (seg < GQ ? (g * GQ + seg) * D : seg == GQ ? (a.H + g) * D : (a.H + a.KV + g) * D) + off;
#pragma unroll
    for (int r = 0; r < QR; ++r) {
      const int row = qrow0 + QR * wave + r;
      wq[r] = ld_nt16(a.wqkv_q + (int64_t)row * 1024 + lane * 16);
      dq[r] = __half2float(a.wqkv_d[(int64_t)row * 32 + (lane >> 1)]);
    }
    __builtin_amdgcn_sched_barrier(0);
    qpre.w0 = a.qn[lane];
    qpre.w1 = a.qn[lane + 64];
    qpre.kw0 = a.kn[lane];
    qpre.kw1 = a.kn[lane + 64];
    // this launch's epoch: head g's attention fan-in counter (+FS per launch) read before any block of head g can add
    // to it in this launch (an add needs every block's q|k|v granules, each stored after its block read the counter)
    if (FA_QKV_GRANULE || FA_PART_GRANULE)
      ep_qkv = __hip_atomic_load(a.cnt + g * CNT_LINE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) / FS + 1;
  } else {
    // q|k|v row inputs do not depend on the position: issued before the tok_pos / tok_seq read (one round trip less
    // on the critical path than loading them after it)
    const float* row = a.qkv;  // token 0
#pragma unroll
    for (int jh = 0; jh < GQ; ++jh) {
      qpre.x0[jh] = row[(g * GQ + jh) * D + lane];
      qpre.x1[jh] = row[(g * GQ + jh) * D + lane + 64];
    }
    qpre.w0 = a.qn[lane];
    qpre.w1 = a.qn[lane + 64];
    qpre.kx0 = row[(a.H + g) * D + lane];
    qpre.kx1 = row[(a.H + g) * D + lane + 64];
    qpre.kw0 = a.kn[lane];
    qpre.kw1 = a.kn[lane + 64];
    qpre.v0 = row[(a.H + a.KV + g) * D + lane];
    qpre.v1 = row[(a.H + a.KV + g) * D + lane + 64];
  }
  int pos = a.tok_pos[0];
  const int seq = a.tok_seq[0];
  asm volatile("" : "+s"(pos) : "s"(seq));
  STAMP(0);
  int4 kpre[AKV_PRE], vpre[AKV_PRE];  // FA_KV_EARLY: the wave's first-pass K/V
  // this block's o slice: rows [FO_ROWS sp, +FO_ROWS), columns [GQ D g, +GQ D); thread -> row tr, 2 q8_0 blocks tq
  const int KO = a.H * D;
  // coalesced: load k reads rows 16 wave + 4 k + (lane >> 4) of the slice, 256 contiguous bytes each; lane chunk
  // c = lane & 15 is half c & 1 of q8_0 block c >> 1 of the head pair's 256 columns
  const int c16 = lane & 15;
  int4 wk[4];
  float dwk[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int orow = FO_ROWS * sp + 16 * wave + 4 * k + (lane >> 4);
    wk[k] = ld_nt16(a.wo_q + (int64_t)orow * KO + GQ * D * g + 16 * c16);
    dwk[k] = __half2float(a.wo_d[(int64_t)orow * (KO / 32) + (GQ * D * g) / 32 + (c16 >> 1)]);
  }
#if FA_ROPE_EARLY
  if constexpr (QKV) {  // the rope row at pos behind the weight loads (the q norm + rope waited for it in kv_early)
    qpre.c = a.rcos[(int64_t)pos * 64 + lane];
    qpre.sn = a.rsin[(int64_t)pos * 64 + lane];
  }
#endif
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (QKV) {
    // ---- prologue (k_gemv_q8 PS): x = x_mid + sum dpart; block (0, 0) stores it; rmsnorm + q8_0 into LDS
    __shared__ __attribute__((aligned(16))) int8_t s_xq[1024];
    __shared__ float s_xd[32];
    __shared__ float s_red[4];
#pragma unroll
    for (int jv = 0; jv < 4; ++jv) {
      float v = xv[jv];
#pragma unroll
      for (int p = 0; p < FUSED_PARTS; ++p) v = v + pv[p][jv];
      xv[jv] = v;
    }
    if (a.xsum && g == 0 && sp == 0)
      *reinterpret_cast<float4*>(a.xsum + threadIdx.x * 4) = make_float4(xv[0], xv[1], xv[2], xv[3]);
    norm_quant_block_regs<4>(xv, xw, true, a.eps, 1024, s_xq, s_xd, s_red);
    __syncthreads();
    if (FA_KV_EARLY == 1) kv_early(a, g, sp, pos, seq, wave, lane, qpre, kpre, vpre);
    STAMP(12);
    // ---- the wave's QR rows (compute_group<1, 1, 0>'s arithmetic), published as two 16-B sc1 stores
    const int4 xq = *reinterpret_cast<const int4*>(s_xq + lane * 16);
    const float xdv = s_xd[lane >> 1];
    float y[QR];
#pragma unroll
    for (int r = 0; r < QR; ++r) {
      int si = dot16(wq[r], xq, 0);
      si += dpp_i<DPP_XOR1>(si);
      float acc = 0.f;
      if (!(lane & 1)) acc += (float)si * (dq[r] * xdv);
      y[r] = wave_sum(acc);
    }
    static_assert(QR == 8, "two 16-B stores per wave");
#if FA_QKV_GRANULE
    {
      float yv = y[0];
#pragma unroll
      for (int r = 1; r < QR; ++r) yv = lane == r ? y[r] : yv;
      if (lane < QR && !(a.dbg_drop && g == 0 && sp == 0))
        __hip_atomic_store(a.gqkv + qrow0 + QR * wave + lane, ((unsigned long long)ep_qkv << 32) | __float_as_uint(yv),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (FA_KV_EARLY == 2) kv_early(a, g, sp, pos, seq, wave, lane, qpre, kpre, vpre);
    STAMP(13);
    // thread t: head g's local rows 2t, 2t + 1 (q head GQ g, q head GQ g + 1, k head g, v head g; 128 each)
    // (FA_QKV_POLL = 1, A/B builds: wave 0 alone polls all 512 granules, 8 rows per lane, the other waves wait at the
    // barrier: a quarter of the polling traffic in the consumer CU's memory queue)
    __shared__ float s_qkv[(GQ + 2) * D];
#if FA_QKV_POLL
    if (wave == 0) {
      const int lr = 8 * lane, sg = lr / D;
      const int grow = (sg < GQ ? (g * GQ + sg) * D : sg == GQ ? (a.H + g) * D : (a.H + a.KV + g) * D) + lr % D;
      const __amdgpu_buffer_rsrc_t rg = buf_rsrc(a.gqkv, (a.H + 2 * a.KV) * D * 8);
      f4v gv[4];
      SpinDeadline dl;
      for (;;) {
#pragma unroll
        for (int k = 0; k < 4; ++k) gv[k] = ld_sc1_f4(rg, (grow + 2 * k) * 8);
        bool ok = true;
#pragma unroll
        for (int k = 0; k < 4; ++k) ok = ok && __float_as_uint(gv[k].y) == ep_qkv && __float_as_uint(gv[k].w) == ep_qkv;
        if (ok) break;
        if (dl.expired()) {
          __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s_qkv[lr + 2 * k] = gv[k].x;
        s_qkv[lr + 2 * k + 1] = gv[k].z;
      }
    }
#else
    {
      const int lr = 2 * threadIdx.x, sg = lr / D;
      const int grow = (sg < GQ ? (g * GQ + sg) * D : sg == GQ ? (a.H + g) * D : (a.H + a.KV + g) * D) + lr % D;
      const __amdgpu_buffer_rsrc_t rg = buf_rsrc(a.gqkv, (a.H + 2 * a.KV) * D * 8);
      f4v gv;
      SpinDeadline dl;
      for (;;) {
        gv = ld_sc1_f4(rg, grow * 8);
        if (__float_as_uint(gv.y) == ep_qkv && __float_as_uint(gv.w) == ep_qkv) break;
        if (dl.expired()) {
          __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      s_qkv[lr] = gv.x;
      s_qkv[lr + 1] = gv.z;
    }
#endif
    __syncthreads();
    STAMP(14);
#pragma unroll
    for (int jh = 0; jh < GQ; ++jh) {
      qpre.x0[jh] = s_qkv[jh * D + lane];
      qpre.x1[jh] = s_qkv[jh * D + lane + 64];
    }
    qpre.kx0 = s_qkv[GQ * D + lane];
    qpre.kx1 = s_qkv[GQ * D + lane + 64];
    qpre.v0 = s_qkv[(GQ + 1) * D + lane];
    qpre.v1 = s_qkv[(GQ + 1) * D + lane + 64];
#else
    const __amdgpu_buffer_rsrc_t rq = buf_rsrc(a.qkv, (a.H + 2 * a.KV) * D * 4);
    if (lane < 2) {
      const f4v v = lane == 0 ? f4v{y[0], y[1], y[2], y[3]} : f4v{y[4], y[5], y[6], y[7]};
      st_sc1_f4(v, rq, (qrow0 + QR * wave + 4 * lane) * 4);
    }
    STAMP(13);
    fanin_wait(a.cnt_qkv + g * CNT_LINE, FS, a.err);
    STAMP(14);
    // ---- head g's q|k|v inputs, written by the group's blocks (sc1: from L2, never a stale L1 line)
#pragma unroll
    for (int jh = 0; jh < GQ; ++jh) {
      qpre.x0[jh] = ld_sc1_f1(rq, ((g * GQ + jh) * D + lane) * 4);
      qpre.x1[jh] = ld_sc1_f1(rq, ((g * GQ + jh) * D + lane + 64) * 4);
    }
    qpre.kx0 = ld_sc1_f1(rq, ((a.H + g) * D + lane) * 4);
    qpre.kx1 = ld_sc1_f1(rq, ((a.H + g) * D + lane + 64) * 4);
    qpre.v0 = ld_sc1_f1(rq, ((a.H + a.KV + g) * D + lane) * 4);
    qpre.v1 = ld_sc1_f1(rq, ((a.H + a.KV + g) * D + lane + 64) * 4);
#endif
  }
  int n_active = 0, j = 0, d0 = 0;
  float M = -INFINITY, L = 0.f;
  float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
  // QKV: lean passes (at most 4 groups per wave pass, no next-pass prefetch): the GEMV and the preloads need the
  // registers; identical arithmetic to k_attn_o<false> up to 4 groups per wave (n_past < 16 x 4 x 4 x 4 = 1024)
  constexpr bool PRE = QKV && FA_KV_EARLY != 0;
  const bool active = attn_split_merge<1, QKV ? 1 : 0, PRE>(g, sp, 0, pos, seq, FS, a.H, a.KV, a.seq_stride,
                                                            a.head_stride, a.kc, a.vc, a.qkv, a.qn, a.kn, a.rcos,
                                                            a.rsin, a.eps, a.scale, n_active, j, d0, M, L, o, &qpre,
                                                            kpre, vpre);
  float4 r;
  if (QKV && FA_PART_GRANULE) {
    // publish this split's partial as granules tagged with the launch's epoch; poll the n_active splits' granules
    // this lane folds (wave w: splits [4 w, 4 w + 4); head lane >> 5, dims [4 (lane & 31), +4) and the 4 (m, l))
    unsigned long long* gp = a.gpart + (int64_t)g * FS * APART;
    if (active && wave == 0) {
      const float M1 = lane_f(M, 32), L1 = lane_f(L, 32);  // head 1's (M, L) live in lanes 32..63
      const unsigned long long tg = (unsigned long long)ep_qkv << 32;
      unsigned long long* po = gp + sp * APART + j * D + d0;
      __hip_atomic_store(po + 0, tg | __float_as_uint(o.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(po + 1, tg | __float_as_uint(o.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(po + 2, tg | __float_as_uint(o.z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(po + 3, tg | __float_as_uint(o.w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane < 4) {
        const float v = lane == 0 ? M : lane == 1 ? L : lane == 2 ? M1 : L1;
        __hip_atomic_store(gp + sp * APART + GQ * D + lane, tg | __float_as_uint(v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    STAMP(9);
    if (threadIdx.x == 0)  // the launch counter (epoch source): one ticket per block, nobody waits on it
      __hip_atomic_fetch_add(a.cnt + g * CNT_LINE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    constexpr int SPW = FS / AWV;
    const int jj = lane >> 5, dd = (lane & 31) * 4;
    const __amdgpu_buffer_rsrc_t rg = buf_rsrc(gp, FS * APART * 8);
    f4v pml[SPW], pov[SPW];
    SpinDeadline dl;
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int t = 0; t < SPW; ++t) {
        const int tt = min(wave * SPW + t, n_active - 1);  // clamped duplicates past n_active are not folded
        const f4v m0 = ld_sc1_f4(rg, (tt * APART + GQ * D) * 8), m1 = ld_sc1_f4(rg, (tt * APART + GQ * D + 2) * 8);
        const f4v o0 = ld_sc1_f4(rg, (tt * APART + jj * D + dd) * 8);
        const f4v o1 = ld_sc1_f4(rg, (tt * APART + jj * D + dd + 2) * 8);
        pml[t] = f4v{m0.x, m0.z, m1.x, m1.z};
        pov[t] = f4v{o0.x, o0.z, o1.x, o1.z};
        const unsigned e = ep_qkv;
        ok = ok && __float_as_uint(m0.y) == e && __float_as_uint(m0.w) == e && __float_as_uint(m1.y) == e &&
             __float_as_uint(m1.w) == e && __float_as_uint(o0.y) == e && __float_as_uint(o0.w) == e &&
             __float_as_uint(o1.y) == e && __float_as_uint(o1.w) == e;
      }
      if (ok) break;
      if (dl.expired()) {
        __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    STAMP(10);
    r = combine_fold(pml, pov, n_active, wave, lane);
  } else {
    float* pbase = a.partials + (int64_t)g * FS * APART;
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(pbase, FS * APART * 4);
    if (active && wave == 0) {
      const f4v ov = {o.x, o.y, o.z, o.w};
      st_sc1_f4(ov, rs, (sp * APART + j * D + d0) * 4);
      const float M1 = lane_f(M, 32), L1 = lane_f(L, 32);  // head 1's (M, L) live in lanes 32..63
      if (lane == 0) {
        const f4v ml = {M, L, M1, L1};
        st_sc1_f4(ml, rs, (sp * APART + GQ * D) * 4);
      }
    }
    STAMP(9);
    fanin_wait(a.cnt + g * CNT_LINE, FS, a.err);
    STAMP(10);
    // every split combines the n_active partials (combine_splits, as the last arriver of k_attn_block does)
    r = combine_splits(rs, n_active, wave, lane);
  }
  __shared__ __attribute__((aligned(16))) int8_t s_aq[GQ * D];
  __shared__ float s_ad[GQ * D / 32];
  if (wave == 0) {
    const int jj = lane >> 5, dd = (lane & 31) * 4;
    // q8_0 of the o projection's input (lanes 8b..8b+7 hold one 32-dim block), into LDS
    const float am = group_max<8>(fmaxf(fmaxf(fabsf(r.x), fabsf(r.y)), fmaxf(fabsf(r.z), fabsf(r.w))));
    const float d = am / 127.0f;
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    const int b0 = (int)roundf(__fmul_rn(r.x, id)) & 0xFF, b1 = (int)roundf(__fmul_rn(r.y, id)) & 0xFF;
    const int b2 = (int)roundf(__fmul_rn(r.z, id)) & 0xFF, b3 = (int)roundf(__fmul_rn(r.w, id)) & 0xFF;
    *reinterpret_cast<int32_t*>(s_aq + jj * D + dd) = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    if ((lane & 7) == 0) s_ad[(jj * D + dd) / 32] = __half2float(__float2half_rn(d));
  }
  __syncthreads();
  STAMP(11);
  const int4 xc = *reinterpret_cast<const int4*>(s_aq + 16 * c16);
  const float xd = s_ad[c16 >> 1];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int si = dot16(wk[k], xc, 0);
    si += dpp_i<DPP_XOR1>(si);  // the block's two halves: exact integer block dot in both lanes of the pair
    float v = (float)si * (dwk[k] * xd);
    v += dpp_f<DPP_XOR2>(v);  // the 8 blocks of the row (pairs hold duplicates: skip the xor-1 step)
    v += dpp_f<DPP_HALF_MIRROR>(v);
    v += dpp_f<DPP_MIRROR>(v);
    if (c16 == 0) a.opart[(int64_t)g * a.E + FO_ROWS * sp + 16 * wave + 4 * k + (lane >> 4)] = v;
  }
}

void attn_o_fused(const float* qkv, const float* qn, const float* kn, float eps, const float* rcos, const float* rsin,
                  __half* kc, __half* vc, int H, int KV, const int* tok_seq, const int* tok_pos, int64_t seq_stride,
                  const int8_t* wo_q, const __half* wo_d, int E, const AttnWork& wk, const FusedDecodeWork& fw,
                  hipStream_t s) {
  FA_REQUIRE(H == KV * GQ && KV == FUSED_PARTS && E == FO_ROWS * ASPLIT, "attn_o_fused: Qwen3-0.6B head layout");
  FA_REQUIRE(wk.partials && fw.opart && fw.cnt && fw.err, "attn_o_fused: workspace");
  AttnOArgs a{tok_seq, tok_pos, H, KV, seq_stride, seq_stride / KV, kc, vc, qkv, qn, kn, rcos, rsin, eps,
              1.0f / sqrtf(128.0f), wo_q, wo_d, E, fw.opart, fw.cnt, wk.partials, fw.err};
  hipLaunchKernelGGL(k_attn_o<false>, dim3(KV, ASPLIT), dim3(AWV * 64), 0, s, a);
}

void qkv_attn_o_fused(const float* x, const float* psum, float* xsum, const float* norm_w, const int8_t* wqkv_q,
                      const __half* wqkv_d, float* qkv, const float* qn, const float* kn, float eps, const float* rcos,
                      const float* rsin, __half* kc, __half* vc, int H, int KV, const int* tok_seq, const int* tok_pos,
                      int64_t seq_stride, const int8_t* wo_q, const __half* wo_d, int E, const AttnWork& wk,
                      const FusedDecodeWork& fw, hipStream_t s, int M, int dbg_drop, const L2Prefetch* pf) {
  FA_REQUIRE(M >= 1 && M <= FUSED_MAX_M && M <= wk.max_split_tokens, "qkv_attn_o_fused: 1 <= M <= FUSED_MAX_M");
  FA_REQUIRE(H == KV * GQ && KV == FUSED_PARTS && E == FO_ROWS * ASPLIT && E == 1024 &&
                 (GQ + 2) * 128 == FQ_ROWS * ASPLIT,
             "qkv_attn_o_fused: Qwen3-0.6B head layout");
  FA_REQUIRE(wk.partials && fw.opart && fw.cnt && fw.err && x && norm_w, "qkv_attn_o_fused: workspace");
  FA_REQUIRE(psum || fw.pzero, "qkv_attn_o_fused: zero partials for layer 0");
  AttnOArgs a{tok_seq, tok_pos, H, KV, seq_stride, seq_stride / KV, kc, vc, qkv, qn, kn, rcos, rsin, eps,
              1.0f / sqrtf(128.0f), wo_q, wo_d, E, fw.opart, fw.cnt, wk.partials, fw.err,
              x, psum ? psum : fw.pzero, psum ? xsum : nullptr, norm_w, wqkv_q, wqkv_d,
              fw.cnt + 2 * FUSED_MAX_M * FUSED_PARTS * CNT_LINE, fw.gqkv, dbg_drop, fw.gpart};
  FA_REQUIRE(!FA_QKV_GRANULE || fw.gqkv, "qkv_attn_o_fused: granule workspace");
  FA_REQUIRE(!FA_PART_GRANULE || fw.gpart, "qkv_attn_o_fused: partial granule workspace");
  int nz = M;
  const int pf_mask = g_l2pf_max_m > 0 ? (M <= g_l2pf_max_m ? g_l2pf_mask : 0) : M == 1 ? g_l2pf_mask : l2pf_small_mask[M];
  if (pf && pf_mask && g_l2pf_blocks > 0) {
    FA_REQUIRE(pf->F == 3072 && pf->gq && pf->uq && pf->dq && pf->gd && pf->ud && pf->dd &&
                   (!pf->qkv_q || (pf->qkv_d && pf->o_q && pf->o_d && pf->kc && pf->vc)),
               "qkv_attn_o_fused: L2 prefetch set");
    a.pf = *pf;
    a.pf_blocks = std::min(g_l2pf_blocks, ASPLIT);
    a.pf_delay = g_l2pf_delay;
    a.pf_mask = pf_mask;
    nz += 1;
  }
  hipLaunchKernelGGL(k_attn_o<true>, dim3(KV, ASPLIT, nz), dim3(AWV * 64), 0, s, a);
}

// ---- Batched decode at M = 32 (the C3 continuous batch): attention, o projection, residual and the o GEMM's
// normalising epilogue in ONE launch (k_attn_ob), instead of k_attn_block<1, 1, 16> then the split-K o GEMM
// (k_gemm_q8_sk<1, ...>): one dependent launch and the o GEMM's separate weight stream per layer less.
// Block (kv head g, token m), 16 waves (one block per CU, all 256 resident):
//   1. LDS-DMA of the o weights this block will multiply -- rows [32 m, +32) of Wo, columns [256 g, +256) (head g's
//      pair of query heads), 8 KB + 512 B of scales -- issued before anything else, landed by step 3;
//   2. the attention of token m, kv head g, exactly k_attn_block<1, 1, 16>'s (attn_split_merge: same values);
//   3. the head pair's 256 outputs quantised to q8_0 (store_q8_row4's arithmetic: the o GEMM's input), published with
//      sc1 stores; the 32 blocks of head g pass a ticket fan-in (fanin_wait; under the dispatcher's round-robin they
//      are the blocks g + 8 m of XCD g);
//   4. wave 0 multiplies the 32 tokens' rows into its 32 x 32 (row, token) tile on 8 v_mfma_i32_32x32x32_i8 (one q8_0
//      block of K each: exact integer block dots), scaled f32(dot) * (f32(d_w) * d_x) and summed in block order, and
//      publishes the tile partial of head g;
//   5. the last of the 8 head blocks of slice m (last-arriver ticket, re-armed) sums the 8 partials in head order,
//      adds the residual (x updated in place, rows [32 m, +32) of every token) and runs the residual GEMM's NRM
//      epilogue (z = x * ffn_norm per 32-row tile = one q8_0 block of every token, unrounded f32 block scale, sum of
//      squares partial): the gate|up GEMM reads the same inputs as after the o GEMM.
// The o sum runs in another f32 order than the split-K GEMM (above the invariant width both are only bound to the
// oracle). Every spin is bounded (SpinDeadline): a timeout sets *err and fa_llm_generate_end re-runs the chunk on
// the two launches.
// A/B only (FUNASR_ATTN_OB=1; profiles/r06_exp_attn_ob.txt): the graph-replayed batch-32 step is 1.228-1.231 ms
// against 1.154-1.158 ms for the two launches. The launch removes one kernel boundary (MI355X_MICROARCH.md boundary:
// 1.2-1.9 us) but adds a 32-arrival head fan-in with its arrival skew and a cross-XCD last-arriver head sum (two
// sc1 round trips), and the gate|up GEMM loses the L2 prefetch slabs the o GEMM ran for it.
constexpr int OB_M = 32;
struct AttnObArgs {
  const int* tok_seq;
  const int* tok_pos;
  int H, KV;
  int64_t seq_stride, head_stride;
  __half* kc;
  __half* vc;
  const float* qkv;
  const float* qn;
  const float* kn;
  const float* rcos;
  const float* rsin;
  float eps, scale;
  const int8_t* wo_q;  // [E][H D], engine layout
  const __half* wo_d;
  int8_t* aq;          // [M][H D] q8_0 attention rows (published)
  float* ad;           // [M][H D / 32]
  float* opart;        // [32 slices][KV][32 tokens][32 rows]
  unsigned* cnt_g;     // [KV][CNT_LINE] tickets, never re-armed
  unsigned* cnt_s;     // [32][CNT_LINE] last-arriver counters, re-armed
  int* err;
  float* x;            // residual rows [M][E], rows [32 m, +32) rewritten by slice m's last block
  const float* qn_w;   // ffn_norm (the next RMSNorm)
  int8_t* qout;        // [M][E] q8_0 of x * qn_w
  float* dout;         // [M][E / 32] unrounded block scales
  float* ssp_out;      // [M][32] sum-of-squares partials
};

__global__ __launch_bounds__(16 * 64, 1) void k_attn_ob(AttnObArgs a) {
  constexpr int D = 128, NW = 16, E = 1024, KO = 2048, NT = OB_M;  // host: Qwen3-0.6B shapes, M = 32
  const int g = blockIdx.x, m = blockIdx.z;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // 1. o weights -> LDS slots [chunk c][row r] (slot 32 c + r, chunk c = half c & 1 of q8_0 block c >> 1), so the
  //    fragment read of block j (lane (r, h) -> slot 32 (2 j + h) + r) is 1 KB contiguous per wave; scales [row][8]
  __shared__ __attribute__((aligned(16))) int4 s_w[16 * 32];
  __shared__ __attribute__((aligned(16))) __half s_wd[32 * 8];
  int pos = a.tok_pos[m];
  const int seq = a.tok_seq[m];
  asm volatile("" : "+s"(pos) : "s"(seq), "s"(a.qkv), "s"(a.kc), "s"(a.vc), "s"(a.rcos), "s"(a.rsin), "s"(a.qn),
               "s"(a.kn));
  if (threadIdx.x < 512) {
    const int r = threadIdx.x & 31, c = threadIdx.x >> 5;
    __builtin_amdgcn_global_load_lds((const void*)(a.wo_q + (int64_t)(32 * m + r) * KO + 256 * g + 16 * c),
                                     (__attribute__((address_space(3))) void*)&s_w[__builtin_amdgcn_readfirstlane(wave) * 64],
                                     16, 0, 0);
  } else if (threadIdx.x < 512 + 32) {
    const int r = threadIdx.x - 512;
    __builtin_amdgcn_global_load_lds((const void*)(a.wo_d + (int64_t)(32 * m + r) * (KO / 32) + 8 * g),
                                     (__attribute__((address_space(3))) void*)&s_wd[0], 16, 0, 0);
  }
  // 2. attention (one split: the 16 waves share the key range)
  int n_active, j, d0;
  float Mx, L;
  float4 o;
  attn_split_merge<1, 1, false, NW>(g, 0, m, pos, seq, 1, a.H, a.KV, a.seq_stride, a.head_stride, a.kc, a.vc, a.qkv,
                                    a.qn, a.kn, a.rcos, a.rsin, a.eps, a.scale, n_active, j, d0, Mx, L, o);
  const int KH = a.H * D;
  const int r = lane & 31, h = lane >> 5;
  if (wave == 0) {
    // 3. q8_0 of the head pair's outputs, published (sc1: read by the group's other blocks, from L2)
    const float4 v = make_float4(o.x / L, o.y / L, o.z / L, o.w / L);
    const float am = group_max<8>(fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    const float dd = am / 127.0f;
    const float id = dd != 0.0f ? 1.0f / dd : 0.0f;
    const int b0 = (int)roundf(__fmul_rn(v.x, id)) & 0xFF, b1 = (int)roundf(__fmul_rn(v.y, id)) & 0xFF;
    const int b2 = (int)roundf(__fmul_rn(v.z, id)) & 0xFF, b3 = (int)roundf(__fmul_rn(v.w, id)) & 0xFF;
    const int e = m * KH + (g * GQ + j) * D + d0;
    __builtin_amdgcn_raw_buffer_store_b32(b0 | (b1 << 8) | (b2 << 16) | (b3 << 24), buf_rsrc(a.aq, NT * KH), e, 0,
                                          CPOL_SC1);
    if ((lane & 7) == 0)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(__half2float(__float2half_rn(dd))),
                                            buf_rsrc(a.ad, NT * (KH / 32) * 4), (e / 32) * 4, 0, CPOL_SC1);
  }
  fanin_wait(a.cnt_g + g * CNT_LINE, NT, a.err);  // drains every wave's stores and the LDS-DMA loads
  // 4. wave jb < 8 multiplies q8_0 block jb of the 32 tokens' head-pair rows (B: token r, 16 B half h) into the 32 x 32
  //    (row, token) tile: one v_mfma_i32_32x32x32_i8 (the exact integer block dots), scaled f32(dot) * (f32(d_w) * d_x);
  //    wave 0 sums the 8 block products in block order
  __shared__ float s_acc[8][16][64];
  if (wave < 8) {
    const int jb = wave;
    const i32x4_t B = __builtin_bit_cast(i32x4_t, ld_sc1_f4(buf_rsrc(a.aq, NT * KH), r * KH + 256 * g + 32 * jb + 16 * h));
    const float dx = ld_sc1_f1(buf_rsrc(a.ad, NT * (KH / 32) * 4), (r * (KH / 32) + 8 * g + jb) * 4);
    const i32x4_t A = __builtin_bit_cast(i32x4_t, s_w[32 * (2 * jb + h) + r]);
    const i32x16_t zero = {};
    const i32x16_t Dv = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B, zero, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 16; ++q) {  // reg q: row 8 (q >> 2) + 4 h + (q & 3) of the slice, token r
      const int row = 8 * (q >> 2) + 4 * h + (q & 3);
      s_acc[jb][q][lane] = (float)Dv[q] * (__half2float(s_wd[row * 8 + jb]) * dx);
    }
  }
  __syncthreads();
  if (wave != 0) return;
  float acc[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    float v = s_acc[0][q][lane];
#pragma unroll
    for (int jb = 1; jb < 8; ++jb) v += s_acc[jb][q][lane];
    acc[q] = v;
  }
  // 5. the tile partial of head g, then the slice's last arriver sums the 8 heads in order
  typedef float f4v __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rp = buf_rsrc(a.opart + (int64_t)m * a.KV * NT * 32, a.KV * NT * 32 * 4);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    st_sc1_f4(f4v{acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]}, rp, ((g * NT + r) * 32 + 8 * q + 4 * h) * 4);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned t = 0;
  if (lane == 0) t = __hip_atomic_fetch_add(a.cnt_s + m * CNT_LINE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  t = __builtin_amdgcn_readfirstlane(t);
  if (t != (unsigned)a.KV - 1) return;
  // residual rows 32 m + 8 q + 4 h + [0, 4) of token r, loaded with the partials (one round trip)
  float4 xr[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) xr[q] = *reinterpret_cast<const float4*>(a.x + (int64_t)r * E + 32 * m + 8 * q + 4 * h);
  f4v sum[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) sum[q] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int gg = 0; gg < 8; ++gg) {  // head order (host: KV == 8)
    f4v pv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) pv[q] = ld_sc1_f4(rp, ((gg * NT + r) * 32 + 8 * q + 4 * h) * 4);
#pragma unroll
    for (int q = 0; q < 4; ++q) sum[q] += pv[q];
  }
  if (lane == 0) __hip_atomic_store(a.cnt_s + m * CNT_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // residual + NRM epilogue of tile m (k_gemm_q8_sk's EPI 1 with ssp_out: same roundings per value)
  float nv[16], z[16], ssq = 0.f, amx = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    nv[4 * q] = xr[q].x + sum[q].x;
    nv[4 * q + 1] = xr[q].y + sum[q].y;
    nv[4 * q + 2] = xr[q].z + sum[q].z;
    nv[4 * q + 3] = xr[q].w + sum[q].w;
    *reinterpret_cast<float4*>(a.x + (int64_t)r * E + 32 * m + 8 * q + 4 * h) =
        make_float4(nv[4 * q], nv[4 * q + 1], nv[4 * q + 2], nv[4 * q + 3]);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int row = 32 * m + 8 * (q >> 2) + 4 * h + (q & 3);
    ssq += nv[q] * nv[q];
    z[q] = nv[q] * a.qn_w[row];
    amx = fmaxf(amx, fabsf(z[q]));
  }
  ssq += __shfl_xor(ssq, 32, 64);  // the token's other 16 rows (lane r + 32): a + b == b + a, both lanes agree
  amx = fmaxf(amx, __shfl_xor(amx, 32, 64));
  const float dz = amx / 127.0f;
  const float iz = dz != 0.0f ? 1.0f / dz : 0.0f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int q0 = (int)roundf(__fmul_rn(z[4 * q], iz)) & 0xFF, q1 = (int)roundf(__fmul_rn(z[4 * q + 1], iz)) & 0xFF;
    const int q2 = (int)roundf(__fmul_rn(z[4 * q + 2], iz)) & 0xFF, q3 = (int)roundf(__fmul_rn(z[4 * q + 3], iz)) & 0xFF;
    *reinterpret_cast<int32_t*>(a.qout + (int64_t)r * E + 32 * m + 8 * q + 4 * h) = q0 | (q1 << 8) | (q2 << 16) | (q3 << 24);
  }
  if (h == 0) {
    a.dout[(int64_t)r * (E / 32) + m] = dz;
    a.ssp_out[(int64_t)r * 32 + m] = ssq;
  }
}

void attn_o_batched(const float* qkv, const float* qn, const float* kn, float eps, const float* rcos, const float* rsin,
                    __half* kc, __half* vc, int M, int H, int KV, const int* tok_seq, const int* tok_pos,
                    int64_t seq_stride, const int8_t* wo_q, const __half* wo_d, int E, const AttnObWork& w, float* x,
                    const float* qn_w, int8_t* qout, float* dout, float* ssp_out, hipStream_t s) {
  FA_REQUIRE(M == OB_M && H == 16 && KV == 8 && E == 1024, "attn_o_batched: M = 32 rows of the Qwen3-0.6B layer");
  FA_REQUIRE(w.aq && w.ad && w.opart && w.cnt_g && w.cnt_s && w.err && x && qn_w && qout && dout && ssp_out,
             "attn_o_batched: workspace");
  AttnObArgs a{tok_seq, tok_pos, H, KV, seq_stride, seq_stride / KV, kc, vc, qkv, qn, kn, rcos, rsin, eps,
               1.0f / sqrtf(128.0f), wo_q, wo_d, w.aq, w.ad, w.opart, w.cnt_g, w.cnt_s, w.err, x, qn_w, qout, dout,
               ssp_out};
  hipLaunchKernelGGL(k_attn_ob, dim3(KV, 1, M), dim3(16 * 64), 0, s, a);
}

struct FfnArgs {
  const float* x;       // residual stream after A [E]
  const float* opart;   // [FUSED_PARTS][E]
  const float* norm_w;
  float eps;
  float* xmid;          // out (block 0): x + sum opart
  const int8_t* gq;
  const __half* gd;
  const int8_t* uq;
  const __half* ud;
  const int8_t* dq;     // down [E][F]
  const __half* dd;
  float* act;           // [M][F] 8-byte granules {value, launch tag} (hand-off)
  float* dpart;         // [FUSED_PARTS][E]
  unsigned* cnt;        // [FUSED_PARTS][CNT_LINE]
  int* err;
  int E, F;
  const unsigned* epoch;  // the attention launch's fan-in counter of kv head 0: + ASPLIT per launch, never re-armed
};
// The group's act rows are handed over as data-tagged 8-byte granules {f32 value, tag} (one sc1 store each; tag = the
// attention launch's epoch, new every layer and step), and each consumer polls the granules it needs until every tag
// matches: no drain, no ticket atomic, no read-back (MI355X_MICROARCH.md handoff-1to1 vs handoff-flag; measured C 6.08
// -> 5.61 us against the sc1 rows + ticket fan-in + read-back form).

constexpr int FF_ROWS = 12;                        // gate|up rows per block (3 per wave)
constexpr int FF_GROUP_BLOCKS = 32;                // blocks per down-projection group: 384 act rows = 12 q8_0 blocks
constexpr int FF_GROUP_ROWS = FF_ROWS * FF_GROUP_BLOCKS;
constexpr int FD_ROWS = 32;                        // down-projection rows per block (E / FF_GROUP_BLOCKS)
static_assert(FF_ROWS == 12 && FD_ROWS == 32 && FF_GROUP_BLOCKS == 32, "l2_prefetch mirrors the FFN launch's row map");

// CT tokens per block (small decode batches: CT = 2 from 4 tokens on, so every block's weights serve two tokens and
// the token slabs fit the chip at once); tokens m0 = CT blockIdx.y .. m0 + ct - 1 (ct = min(CT, M - m0), block-uniform).
// Per token: x_mid = x + sum opart (block 0 stores it), rmsnorm + q8_0, gate|up + SwiGLU for the block's 12 rows, published
// as granules {value, epoch} (the epoch of that token's attention launch); the group's 384 act rows polled, quantised
// and multiplied into the block's 32-row slice of the down projection. Same arithmetic for every CT.
// CT = 3..6 (round 6, FUNASR_FFN_WIDE): the whole batch in one slab of 256 blocks, one per CU (launch bounds (256, 1):
// the per-token prologue registers of 6 tokens fit), so every block's gate|up and down weight rows are read once for the
// batch and the group fan-ins stay 32 blocks deep with all 256 blocks resident.
template <int CT>
__global__ __launch_bounds__(256, CT > 2 ? 1 : 2) void k_ffn_fused(FfnArgs f, int M) {
  constexpr int K = 1024, NB = K / 32, PER = 4, GB = FF_GROUP_ROWS / 32;
  const int b = blockIdx.x, grp = b / FF_GROUP_BLOCKS, bi = b % FF_GROUP_BLOCKS;
  const int m0 = blockIdx.y * CT, ct = min(CT, M - m0);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, t = threadIdx.x;
  STAMP(0);
  __shared__ __attribute__((aligned(16))) int8_t s_q[CT][K];
  __shared__ float s_d[CT][NB];
  __shared__ float s_red[CT][4];
  __shared__ float s_act[CT][FF_ROWS];
  __shared__ __attribute__((aligned(16))) int8_t s_aq[CT][FF_GROUP_ROWS];
  __shared__ float s_ad[CT][GB];
  // ---- activation loads (x, the 8 o partials per token; the norm weights), then every weight load of the block
  float xv[CT][PER], pv[CT][FUSED_PARTS][PER], wv[PER];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const int m = m0 + min(c, ct - 1);  // a missing second token loads the first's rows (unused)
    const float4 a4 = *reinterpret_cast<const float4*>(f.x + (int64_t)m * f.E + t * PER);
    xv[c][0] = a4.x; xv[c][1] = a4.y; xv[c][2] = a4.z; xv[c][3] = a4.w;
#pragma unroll
    for (int g = 0; g < FUSED_PARTS; ++g) {
      const float4 p4 = *reinterpret_cast<const float4*>(f.opart + ((int64_t)m * FUSED_PARTS + g) * f.E + t * PER);
      pv[c][g][0] = p4.x; pv[c][g][1] = p4.y; pv[c][g][2] = p4.z; pv[c][g][3] = p4.w;
    }
  }
  {
    const float4 w4 = *reinterpret_cast<const float4*>(f.norm_w + t * PER);
    wv[0] = w4.x; wv[1] = w4.y; wv[2] = w4.z; wv[3] = w4.w;
  }
  // the epochs: written by the attention launch's atomics (read past this CU's L1 and the XCD's L2 line); token m's
  // attention fan-in line of kv head 0
  unsigned ep[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c)
    ep[c] = __hip_atomic_load(f.epoch + (m0 + min(c, ct - 1)) * FUSED_PARTS * CNT_LINE, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT) / ASPLIT;  // >= 1 after the layer's attention launch
  __builtin_amdgcn_sched_barrier(0);
  GemvArgs a{};
  a.wq = f.gq; a.wd = f.gd; a.wq2 = f.uq; a.wd2 = f.ud; a.O = f.F; a.rpw = 3;
  const int row_base = (b * 4 + wave) * 3;
  RowGroup<1, 2> G;
  load_group<1, 2>(a, row_base, 0, lane, G);
  // down slice: rows [FD_ROWS bi, +FD_ROWS), K columns [FF_GROUP_ROWS grp, +FF_GROUP_ROWS); thread -> row dr, q8_0
  // blocks dk and (dk < 4) dk + 8 of the group's 12
  // coalesced: load i reads 128 contiguous bytes (chunks 8 i .. 8 i + 7) of each of the wave's 8 rows; lane chunk
  // c = 8 i + (lane & 7) is half c & 1 of the group's q8_0 block c >> 1
  const int drow = FD_ROWS * bi + 8 * wave + (lane >> 3), c8 = lane & 7;
  int4 dwv[3];
  float dsv[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    dwv[i] = ld_nt16(f.dq + (int64_t)drow * f.F + FF_GROUP_ROWS * grp + 16 * (8 * i + c8));
    dsv[i] = __half2float(f.dd[(int64_t)drow * (f.F / 32) + GB * grp + 4 * i + (c8 >> 1)]);
  }
  __builtin_amdgcn_sched_barrier(0);
  // ---- per token: x_mid = x + sum_g opart[g]; rmsnorm + q8_0 into LDS
#pragma unroll
  for (int c = 0; c < CT; ++c) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      float v = xv[c][j];
#pragma unroll
      for (int g = 0; g < FUSED_PARTS; ++g) v = v + pv[c][g][j];
      xv[c][j] = v;
    }
    if (b == 0 && c < ct)
      *reinterpret_cast<float4*>(f.xmid + (int64_t)(m0 + c) * f.E + t * PER) =
          make_float4(xv[c][0], xv[c][1], xv[c][2], xv[c][3]);
    norm_quant_block_regs<PER>(xv[c], wv, true, f.eps, K, s_q[c], s_d[c], s_red[c]);
  }
  __syncthreads();
  STAMP(1);
  // ---- gate|up + SwiGLU for this wave's 3 rows (compute_group's arithmetic), per token
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    float acc[3] = {0.f, 0.f, 0.f}, acc2[3] = {0.f, 0.f, 0.f};
    const int4 xq = *reinterpret_cast<const int4*>(s_q[c] + lane * 16);
    const float xdv = s_d[c][lane >> 1];
#pragma unroll
    for (int rr = 0; rr < 3; ++rr) {
      int si = dot16(G.w[rr][0], xq, 0);
      si += dpp_i<DPP_XOR1>(si);
      if (!(lane & 1)) acc[rr] += (float)si * (G.dw[rr][0] * xdv);
      int su = dot16(G.u[rr][0], xq, 0);
      su += dpp_i<DPP_XOR1>(su);
      if (!(lane & 1)) acc2[rr] += (float)su * (G.du[rr][0] * xdv);
    }
#pragma unroll
    for (int rr = 0; rr < 3; ++rr) {
      const float y = wave_sum(acc[rr]), y2 = wave_sum(acc2[rr]);
      if (lane == 0) s_act[c][wave * 3 + rr] = (y / (1.0f + expf(-y))) * y2;
    }
  }
  __syncthreads();
  typedef float f4v __attribute__((ext_vector_type(4)));
  // ---- publish each token's 12 act rows as granules tagged with its epoch; poll the group's 384 per token
  // (thread t: token t / 96, granules 4 (t % 96) .. +4 of the group)
  if (t < FF_ROWS * ct) {
    const int c = t / FF_ROWS, r = t % FF_ROWS;
    unsigned long long* gact = reinterpret_cast<unsigned long long*>(f.act) + (int64_t)(m0 + c) * f.F;
    __hip_atomic_store(gact + FF_ROWS * b + r, ((unsigned long long)ep[c] << 32) | __float_as_uint(s_act[c][r]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  STAMP(2);
  // thread t < 192 polls 4 granules (act rows 4 pt .. +4 of the group) of tokens pc0, pc0 + 2, ... (NPT of them, all
  // loads of a sweep in flight together)
  constexpr int QT = FF_GROUP_ROWS / 4;  // polling threads per token
  constexpr int NPT = (CT + 1) / 2;      // tokens per polling thread
  const int pc0 = t / QT, pt = t % QT;
  f4v gv0[NPT], gv1[NPT];
  unsigned ek[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    gv0[k] = gv1[k] = f4v{0.f, 0.f, 0.f, 0.f};
    ek[k] = ep[0];
#pragma unroll
    for (int c = 1; c < CT; ++c)
      if (pc0 + 2 * k == c) ek[k] = ep[c];
  }
  if (pc0 < 2 && pc0 < ct) {
    const int off = (FF_GROUP_ROWS * grp + 4 * pt) * 8;
    SpinDeadline dl;
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int pc = pc0 + 2 * k;
        if (pc < ct) {
          const __amdgpu_buffer_rsrc_t ra = buf_rsrc(f.act + (int64_t)(m0 + pc) * 2 * f.F, f.F * 8);
          gv0[k] = ld_sc1_f4(ra, off);
          gv1[k] = ld_sc1_f4(ra, off + 16);
        }
      }
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const unsigned e = ek[k];
        if (pc0 + 2 * k < ct)
          ok = ok && __float_as_uint(gv0[k].y) == e && __float_as_uint(gv0[k].w) == e &&
               __float_as_uint(gv1[k].y) == e && __float_as_uint(gv1[k].w) == e;
      }
      if (ok) break;
      if (dl.expired()) {
        __hip_atomic_store(f.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  STAMP(3);
  // ---- each token's 384 act rows -> q8_0 (8 threads per 32-row block) in LDS
  if (pc0 < 2) {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int pc = pc0 + 2 * k;
      if (pc < CT) {
        const f4v v = {gv0[k].x, gv0[k].z, gv1[k].x, gv1[k].z};
        const float am = group_max<8>(fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        const float d = am / 127.0f;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        const int q0 = (int)roundf(__fmul_rn(v.x, id)) & 0xFF, q1 = (int)roundf(__fmul_rn(v.y, id)) & 0xFF;
        const int q2 = (int)roundf(__fmul_rn(v.z, id)) & 0xFF, q3 = (int)roundf(__fmul_rn(v.w, id)) & 0xFF;
        *reinterpret_cast<int32_t*>(s_aq[pc] + 4 * pt) = q0 | (q1 << 8) | (q2 << 16) | (q3 << 24);
        if ((pt & 7) == 0) s_ad[pc][pt >> 3] = __half2float(__float2half_rn(d));
      }
    }
  }
  __syncthreads();
  STAMP(4);
  // ---- down slice: row drow over the group's 12 q8_0 blocks, 4 per load (8 lanes), loads summed in order; per token
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      int si = dot16(dwv[i], *reinterpret_cast<const int4*>(s_aq[c] + 16 * (8 * i + c8)), 0);
      si += dpp_i<DPP_XOR1>(si);  // the block's two halves: exact integer block dot in both lanes of the pair
      float u = (float)si * (dsv[i] * s_ad[c][4 * i + (c8 >> 1)]);
      u += dpp_f<DPP_XOR2>(u);  // 4 blocks (pairs hold duplicates: no xor-1 step)
      u += dpp_f<DPP_HALF_MIRROR>(u);
      v += u;
    }
    if (c8 == 0 && c < ct) f.dpart[((int64_t)(m0 + c) * FUSED_PARTS + grp) * f.E + drow] = v;
  }
  STAMP(5);
}

// out[m] = xmid[m] + dpart[m][0] + ... + dpart[m][FUSED_PARTS - 1] (the order of the batch-1 partial-sum prologues):
// the residual rows after a small batch's last fused layer, for the LM head
__global__ __launch_bounds__(256) void k_psum_rows(const float* __restrict__ xmid, const float* __restrict__ dpart, int E,
                                                   float* __restrict__ out) {
  const int m = blockIdx.y, e = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (e >= E) return;
  float4 v = *reinterpret_cast<const float4*>(xmid + (int64_t)m * E + e);
#pragma unroll
  for (int p = 0; p < FUSED_PARTS; ++p) {
    const float4 q = *reinterpret_cast<const float4*>(dpart + ((int64_t)m * FUSED_PARTS + p) * E + e);
    v.x = v.x + q.x; v.y = v.y + q.y; v.z = v.z + q.z; v.w = v.w + q.w;
  }
  *reinterpret_cast<float4*>(out + (int64_t)m * E + e) = v;
}

void psum_rows(const float* xmid, const float* dpart, int M, int E, float* out, hipStream_t s) {
  FA_REQUIRE(E % 4 == 0, "psum_rows: E % 4");
  hipLaunchKernelGGL(k_psum_rows, dim3(cdiv(E / 4, 256), M), dim3(256), 0, s, xmid, dpart, E, out);
}

int g_ffn_wide = 0;  // FUNASR_FFN_WIDE: decode batches of 3-6 as one slab of CT = M tokens per block (A/B)
int g_ffn_pair_min_m = 2;  // decode batches from this width run the fused FFN with two tokens per block (round 5,
// profiles/r05_exp_ffn_pairs.txt: graph-replayed steps, pairs vs one token per block, bit-identical: M = 2 0.530-0.538
// vs 0.541 ms, M = 4 0.672 vs 0.727, M = 6 0.885-0.894 vs 0.974; the threshold was 4)
// (three tokens per block, tried in round 4: 184 VGPRs, 2 blocks per CU; at batches 3-6 the in-launch fan-ins timed out
// and every chunk fell back to the 5-launch layer: not kept)

void ffn_fused(const float* x, const float* norm_w, float eps, const int8_t* gq, const __half* gd, const int8_t* uq,
               const __half* ud, const int8_t* dq, const __half* dd, int E, int F, const FusedDecodeWork& fw,
               hipStream_t s, int M) {
  FA_REQUIRE(M >= 1 && M <= FUSED_MAX_M, "ffn_fused: 1 <= M <= FUSED_MAX_M");
  FA_REQUIRE(E == 1024 && F == FF_GROUP_ROWS * FUSED_PARTS && E == FD_ROWS * FF_GROUP_BLOCKS,
             "ffn_fused: Qwen3-0.6B FFN shape (E 1024, F 3072)");
  FA_REQUIRE(fw.opart && fw.dpart && fw.act && fw.xmid && fw.cnt && fw.err, "ffn_fused: workspace");
  FfnArgs f{x, fw.opart, norm_w, eps, fw.xmid, gq, gd, uq, ud, dq, dd, fw.act, fw.dpart,
            fw.cnt + FUSED_MAX_M * FUSED_PARTS * CNT_LINE, fw.err, E, F, fw.cnt};
  if (g_ffn_wide && M >= 3 && M <= 6) {  // the batch in one slab: weights read once, one block per CU
    switch (M) {
      case 3: hipLaunchKernelGGL(k_ffn_fused<3>, dim3(F / FF_ROWS, 1), dim3(256), 0, s, f, M); break;
      case 4: hipLaunchKernelGGL(k_ffn_fused<4>, dim3(F / FF_ROWS, 1), dim3(256), 0, s, f, M); break;
      case 5: hipLaunchKernelGGL(k_ffn_fused<5>, dim3(F / FF_ROWS, 1), dim3(256), 0, s, f, M); break;
      default: hipLaunchKernelGGL(k_ffn_fused<6>, dim3(F / FF_ROWS, 1), dim3(256), 0, s, f, M); break;
    }
  } else if (M >= g_ffn_pair_min_m) {
    hipLaunchKernelGGL(k_ffn_fused<2>, dim3(F / FF_ROWS, cdiv(M, 2)), dim3(256), 0, s, f, M);
  } else {
    hipLaunchKernelGGL(k_ffn_fused<1>, dim3(F / FF_ROWS, M), dim3(256), 0, s, f, M);
  }
}

}  // namespace fa
