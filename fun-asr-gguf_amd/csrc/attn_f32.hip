// Encoder self-attention (SANM / adaptor / CTC-decoder): out = softmax(q*d^-0.5 . k^T + mask) . v
// per head, full-length (non-causal) with the reference's additive key mask (m-1)*1e4
// (model_definition.py:68-78, 122-145). Exact-f32 MFMA (v_mfma_f32_32x32x2_f32), flash-style:
//
//   block = (128-query tile, head, clip, key split); its 4 waves own 32 queries each and share the K/V
//   stream: 32-key tiles are staged through LDS (double-buffered, one barrier per tile), so each K/V byte
//   read from L2 feeds 128 queries. S^T = K . Q^T puts the query on the lane (col) and keys on the 16
//   accumulator registers: the per-query max/sum is an in-register reduction + one cross-half swap, and
//   P^T is directly the B operand of O^T += V^T . P^T.
//   Q/K fragments: lane (r = l&31, h = l>>5) holds row r, dims [h*D/2, h*D/2 + D/2): the dot index is
//   permuted identically on A and B.
//   Key splits (single clip: too few (query tile, head) blocks to cover 256 CUs): each split stores its
//   (m, l, O) with sc1 stores and counts arrivals; the last split merges them in split order
//   (MI355X_MICROARCH.md hand-off table, row 1).
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <cmath>

namespace fa {

// fp16 encoder mode (C5): the attention output (an fp16 tensor in the float16 graph) rounded to fp16
__device__ __forceinline__ float4 round_f16x4(float4 v) {
  return make_float4(__half2float(__float2half_rn(v.x)), __half2float(__float2half_rn(v.y)),
                     __half2float(__float2half_rn(v.z)), __half2float(__float2half_rn(v.w)));
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int AQ = 128;  // queries per block (4 waves x 32)
constexpr int AK = 32;   // keys per tile

template <int D>
struct AttnLds {
  static constexpr int S = D + 8;                    // row stride (floats): S % 16 == 8 -> conflict-free reads
  static constexpr int TILE = AK * S;                // one K or V tile
  static constexpr int BYTES_PIPE = 4 * TILE * 4;    // K, V x 2 stages
  static constexpr int OS = D + 4;                   // output transpose stride
  static constexpr int BYTES_OUT = AQ * OS * 4;
  static constexpr int BYTES = (BYTES_PIPE > BYTES_OUT ? BYTES_PIPE : BYTES_OUT) + 2 * AQ * 4 + 16;
};

// global -> register staging of one K/V tile: float4 f = tid + 256 c -> key f / (D/4), dim4 f % (D/4)
// (row-contiguous, coalesced); keys past the clip are clamped (masked to -inf in the scores)
template <int D>
__device__ __forceinline__ void attn_load_tile(const float* __restrict__ Kp, const float* __restrict__ V, int64_t ldk,
                                               int64_t ldv, int64_t row_base, int head, int t_stride, int kt,
                                               f4v (&pk)[AK * D / 1024], f4v (&pv)[AK * D / 1024]) {
#pragma unroll
  for (int c = 0; c < AK * D / 1024; ++c) {
    const int f = threadIdx.x + 256 * c;
    const int key = min(kt * AK + f / (D / 4), t_stride - 1);
    const int d4 = f % (D / 4);
    pk[c] = *reinterpret_cast<const f4v*>(Kp + (row_base + key) * ldk + head * D + 4 * d4);
    pv[c] = *reinterpret_cast<const f4v*>(V + (row_base + key) * ldv + head * D + 4 * d4);
  }
}
template <int D>
__device__ __forceinline__ void attn_store_tile(float* lds, int stage, const f4v (&pk)[AK * D / 1024],
                                                const f4v (&pv)[AK * D / 1024]) {
  using L = AttnLds<D>;
  float* ks_ = lds + stage * 2 * L::TILE;
  float* vs_ = ks_ + L::TILE;
#pragma unroll
  for (int c = 0; c < AK * D / 1024; ++c) {
    const int f = threadIdx.x + 256 * c;
    const int key = f / (D / 4), d4 = f % (D / 4);
    *reinterpret_cast<f4v*>(ks_ + key * L::S + 4 * d4) = pk[c];
    *reinterpret_cast<f4v*>(vs_ + key * L::S + 4 * d4) = pv[c];
  }
}

// the output row as f32, or (op.hi != nullptr: bf16x3 encoder, output consumed only by the out-projection GEMM) as
// its bf16 hi / lo planes at the same element offsets: hi = bf16_rn(v), lo = bf16_rn(v - hi), the split the GEMM's
// staging would apply to the f32 row (bit-identical products)
__device__ __forceinline__ void store_o4(const float4 v, float* __restrict__ O, const APlanesD& op, int64_t off) {
  if (!op.hi) {
    *reinterpret_cast<float4*>(O + off) = v;
    return;
  }
  bf16x4_t h, l;
  split_bf16x4(v, h, l);
  *reinterpret_cast<bf16x4_t*>(op.hi + off) = h;
  *reinterpret_cast<bf16x4_t*>(op.lo + off) = l;
}

// Merge of a query tile's KS split partials (m, l, O), queries [qa, qa + nq) of the tile: merged max / sum per query
// and each split's weight exp(m_k - m) -> LDS, with every split's (m, l) load in flight at once; then the weighted sum
// of the splits' O, KSM loads per output in flight (clamped duplicates past KS carry weight 0). Shared by the
// last-arriving split (qa = 0, nq = AQ) and k_attn_merge (a slice of the tile per block): the same arithmetic.
template <int D>
__device__ __forceinline__ void attn_merge_rows(const __amdgpu_buffer_rsrc_t rs, float* lds, float* s_l, int qa, int nq,
                                                float* __restrict__ O, int64_t ldo, int64_t row_base, int head, int q0,
                                                int t_stride, int KS, int r16, const APlanesD& op) {
  constexpr int PSZ = AQ * D + 2 * AQ;  // floats per split partial
  constexpr int D4 = D / 4;
  constexpr int KSM = 8;
  float* s_w = lds;  // [KSM][AQ]
  if ((int)threadIdx.x < nq) {
    const int q = qa + threadIdx.x;
    f4v ml[KSM];
#pragma unroll
    for (int k2 = 0; k2 < KSM; ++k2) ml[k2] = ld_sc1_f4(rs, (min(k2, KS - 1) * PSZ + AQ * D + 2 * (q & ~1)) * 4);
    float mm = -INFINITY;
#pragma unroll
    for (int k2 = 0; k2 < KSM; ++k2)
      if (k2 < KS) mm = fmaxf(mm, (q & 1) ? ml[k2].z : ml[k2].x);
    // explicit roundings (no fused multiply-add): the same bits wherever this is inlined (the last split of any
    // attention kernel, or k_attn_merge), whatever the surrounding code lets the compiler contract
    float ll = 0.f;
#pragma unroll
    for (int k2 = 0; k2 < KSM; ++k2) {
      const float mk = (q & 1) ? ml[k2].z : ml[k2].x, lk = (q & 1) ? ml[k2].w : ml[k2].y;
      const float w = (k2 >= KS || mk == -INFINITY) ? 0.f : __expf(__fsub_rn(mk, mm));
      ll = __fadd_rn(ll, __fmul_rn(w, lk));
      s_w[k2 * AQ + q] = w;
    }
    s_l[q] = ll;
  }
  __syncthreads();
  for (int f = threadIdx.x; f < nq * D4; f += 256) {
    const int q = qa + f / D4, d4 = f % D4;
    if (q0 + q >= t_stride) continue;
    f4v pv[KSM];
#pragma unroll
    for (int k2 = 0; k2 < KSM; ++k2) pv[k2] = ld_sc1_f4(rs, (min(k2, KS - 1) * PSZ + q * D + 4 * d4) * 4);
    const float w0 = s_w[q];
    float4 a = make_float4(__fmul_rn(w0, pv[0].x), __fmul_rn(w0, pv[0].y), __fmul_rn(w0, pv[0].z), __fmul_rn(w0, pv[0].w));
#pragma unroll
    for (int k2 = 1; k2 < KSM; ++k2) {
      const float wk = s_w[k2 * AQ + q];
      a.x = __fadd_rn(a.x, __fmul_rn(wk, pv[k2].x));
      a.y = __fadd_rn(a.y, __fmul_rn(wk, pv[k2].y));
      a.z = __fadd_rn(a.z, __fmul_rn(wk, pv[k2].z));
      a.w = __fadd_rn(a.w, __fmul_rn(wk, pv[k2].w));
    }
    const float inv = __frcp_rn(s_l[q]);
    float4 v = make_float4(__fmul_rn(a.x, inv), __fmul_rn(a.y, inv), __fmul_rn(a.z, inv), __fmul_rn(a.w, inv));
    if (r16) v = round_f16x4(v);
    store_o4(v, O, op, (row_base + q0 + q) * ldo + head * D + 4 * d4);
  }
}

// The merge of every key-split tile as its own launch (attn_f32 with g_attn_merge): block (slice, tile) merges AQ / MS
// queries of one tile, so the 512 KB of split partials per tile are read by MS blocks instead of the last split alone
int g_attn_ms = 8;  // query slices per tile (FUNASR_ATTN_MS: 1, 2, 4, 8, 16 or 32)
template <int D>
__global__ __launch_bounds__(256) void k_attn_merge(const float* __restrict__ part, int KS, int n_qt, int n_heads,
                                                    float* __restrict__ O, int64_t ldo, int t_stride, int r16,
                                                    APlanesD op, int ms) {
  __shared__ float lds[8 * AQ + AQ];
  constexpr int PSZ = AQ * D + 2 * AQ;
  const int slice = blockIdx.x % ms, tile = blockIdx.x / ms;
  const int qt = tile % n_qt, head = (tile / n_qt) % n_heads, clip = tile / (n_qt * n_heads);
  const __amdgpu_buffer_rsrc_t rs = buf_rsrc(part + (int64_t)tile * KS * PSZ, KS * PSZ * 4);
  attn_merge_rows<D>(rs, lds, lds + 8 * AQ, slice * (AQ / ms), AQ / ms, O, ldo, (int64_t)clip * t_stride,
                     head, qt * AQ, t_stride, KS, r16, op);
}

// The block's epilogue, shared by the exact-f32 and the bf16x3 kernels: O^T (d on registers, q on lanes) -> LDS [q][d]
// for row-contiguous stores; with key splits, publish (m, l, O) and let the last split merge.
template <int D>
__device__ __forceinline__ void attn_epilogue(const f32x16 (&o)[D / 32], float m_run, float l_run, float* lds,
                                              float* __restrict__ O, int64_t ldo, int64_t row_base, int head, int q0,
                                              int qt, int n_qt, int clip, int t_stride, int KS, int ks, int r16,
                                              float* __restrict__ part, int* __restrict__ cnt, int lds_bytes,
                                              APlanesD op = {}) {
  using L = AttnLds<D>;
  constexpr int NDT = D / 32;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  float* s_m = lds + (lds_bytes - 2 * AQ * 4 - 16) / 4;  // [AQ] merged row max / sum (split path), past the O staging
  float* s_l = s_m + AQ;
  int* s_flag = reinterpret_cast<int*>(s_l + AQ);
  float* so = lds;
#pragma unroll
  for (int i = 0; i < NDT; ++i)
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int d = i * 32 + (t & 3) + 8 * (t >> 2) + 4 * h;
      so[(wave * 32 + r) * L::OS + d] = o[i][t];
    }
  if (h == 0) {
    s_m[wave * 32 + r] = m_run;
    s_l[wave * 32 + r] = l_run;
  }
  __syncthreads();
  constexpr int D4 = D / 4;
  if (KS == 1) {
    for (int f = threadIdx.x; f < AQ * D4; f += 256) {
      const int q = f / D4, d4 = f % D4;
      if (q0 + q < t_stride) {
        const float inv = 1.0f / s_l[q];
        float4 v = *reinterpret_cast<const float4*>(so + q * L::OS + 4 * d4);
        v.x *= inv; v.y *= inv; v.z *= inv; v.w *= inv;
        if (r16) v = round_f16x4(v);
        store_o4(v, O, op, (row_base + q0 + q) * ldo + head * D + 4 * d4);
      }
    }
    return;
  }
  // ---- key split: publish (m, l, O) of this split; the last split merges
  constexpr int PSZ = AQ * D + 2 * AQ;  // floats per split partial
  const int tile = (clip * gridDim.y + head) * n_qt + qt;
  float* pbase = part + (int64_t)tile * KS * PSZ;
  const __amdgpu_buffer_rsrc_t rs = buf_rsrc(pbase, KS * PSZ * 4);
  for (int f = threadIdx.x; f < AQ * D4; f += 256) {
    const int q = f / D4, d4 = f % D4;
    const f4v v = *reinterpret_cast<const f4v*>(so + q * L::OS + 4 * d4);
    st_sc1_f4(v, rs, (ks * PSZ + q * D + 4 * d4) * 4);
  }
  if (threadIdx.x < AQ / 2) {
    const int q = threadIdx.x * 2;
    const f4v v = {s_m[q], s_l[q], s_m[q + 1], s_l[q + 1]};
    st_sc1_f4(v, rs, (ks * PSZ + AQ * D + 2 * q) * 4);
  }
  if (!cnt) return;  // merged by k_attn_merge (the kernel boundary is the hand-off)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    *s_flag = __hip_atomic_fetch_add(cnt + tile * CNT_LINE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == KS - 1;
  __syncthreads();
  if (!*s_flag) return;
  attn_merge_rows<D>(rs, lds, s_l, 0, AQ, O, ldo, row_base, head, q0, t_stride, KS, r16, op);
  if (threadIdx.x == 0) __hip_atomic_store(cnt + tile * CNT_LINE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// two blocks per CU (LDS 70.7 KB per block at D = 128; 234 VGPRs, no AGPRs or scratch), as k_attn_bf3 below
template <int D>
__global__ __launch_bounds__(256, 2) void k_attn_f32(const float* __restrict__ Q, const float* __restrict__ Kp,
                                                  const float* __restrict__ V, int64_t ldq, int64_t ldk, int64_t ldv,
                                                  float* __restrict__ O, int64_t ldo, int t_stride,
                                                  const int* __restrict__ lens, float scale, int KS, int r16,
                                                  float* __restrict__ part, int* __restrict__ cnt) {
  using L = AttnLds<D>;
  constexpr int HD = D / 2;    // dims per lane half
  constexpr int NDT = D / 32;  // output d-tiles
  constexpr int F4 = AK * D / 4 / 256;  // float4 per thread per tile (K or V)
  extern __shared__ float lds[];

  const int n_qt = (t_stride + AQ - 1) / AQ;
  // splits of one (query tile, head, clip) sit 8*k block ids apart: the dispatcher deals blocks round-robin
  // over the 8 XCDs, so they usually share one XCD's L2 with the merging block (speed only: the sc1
  // hand-off is correct at any placement). grid.x = KS * n_qt8, n_qt8 % 8 == 0
  const int n_qt8 = (n_qt + 7) & ~7;
  const int qt = blockIdx.x % n_qt8, ks = blockIdx.x / n_qt8, head = blockIdx.y, clip = blockIdx.z;
  if (qt >= n_qt) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t row_base = (int64_t)clip * t_stride;
  const int len = lens ? lens[clip] : t_stride;
  const int q0 = qt * AQ;
  const int n_kt = (t_stride + AK - 1) / AK;
  const int tpk = (n_kt + KS - 1) / KS;
  const int kt0 = ks * tpk, kt1 = min(n_kt, kt0 + tpk);

  // this wave's 32 queries, pre-scaled (python: q * d_k**-0.5 before the dot)
  float qreg[HD];
  {
    const int q = min(q0 + wave * 32 + r, t_stride - 1);
    const float* p = Q + (row_base + q) * ldq + head * D + h * HD;
#pragma unroll
    for (int s = 0; s < HD; s += 4) {
      const float4 v = *reinterpret_cast<const float4*>(p + s);
      qreg[s] = v.x * scale;
      qreg[s + 1] = v.y * scale;
      qreg[s + 2] = v.z * scale;
      qreg[s + 3] = v.w * scale;
    }
  }
  f32x16 o[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) o[i] = f32x16{};
  float m_run = -INFINITY, l_run = 0.f;
  f4v pk[F4], pv[F4];  // register staging of the next K/V tile
  if (kt0 < kt1) {
    attn_load_tile<D>(Kp, V, ldk, ldv, row_base, head, t_stride, kt0, pk, pv);
    attn_store_tile<D>(lds, 0, pk, pv);
  }
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int stage = (kt - kt0) & 1;
    if (kt + 1 < kt1) attn_load_tile<D>(Kp, V, ldk, ldv, row_base, head, t_stride, kt + 1, pk, pv);  // in flight
    const float* ks_ = lds + stage * 2 * L::TILE;
    const float* vs_ = ks_ + L::TILE;
    const int k0 = kt * AK;
    // S^T[key][q] = sum_d K[key][d] Q[q][d]
    f32x16 s = {};
#pragma unroll
    for (int c = 0; c < HD; c += 4) {
      const float4 kv = *reinterpret_cast<const float4*>(ks_ + r * L::S + h * HD + c);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.x, qreg[c], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.y, qreg[c + 1], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.z, qreg[c + 2], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.w, qreg[c + 3], s, 0, 0, 0);
    }
    // mask + online softmax (per query = per lane column; keys on registers and lane halves)
    // a tile of valid keys only (block-uniform; every tile but a clip's last) needs no mask and holds no -inf score:
    // the same values without the per-score compares and selects
    const bool full = k0 + AK <= min(len, t_stride);
    float mt = -INFINITY;
    if (full) {
#pragma unroll
      for (int t = 0; t < 16; ++t) mt = fmaxf(mt, s[t]);
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int key = k0 + (t & 3) + 8 * (t >> 2) + 4 * h;
        float v = s[t];
        if (key >= t_stride) v = -INFINITY;
        else if (key >= len) v = v + -10000.0f;
        s[t] = v;
        mt = fmaxf(mt, v);
      }
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float m_new = fmaxf(m_run, mt);
    const float alpha = m_run == -INFINITY ? 0.f : __expf(m_run - m_new);
    float ls = 0.f;
    if (full) {
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const float p = __expf(s[t] - m_new);
        s[t] = p;
        ls += p;
      }
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const float p = s[t] == -INFINITY ? 0.f : __expf(s[t] - m_new);
        s[t] = p;
        ls += p;
      }
    }
    ls += __shfl_xor(ls, 32, 64);
    l_run = l_run * alpha + ls;
    m_run = m_new;
#pragma unroll
    for (int i = 0; i < NDT; ++i) o[i] *= alpha;
    // O^T[d][q] += sum_key V[key][d] P^T[key][q]
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int kl = (t & 3) + 8 * (t >> 2) + 4 * h;
#pragma unroll
      for (int i = 0; i < NDT; ++i)
        o[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(vs_[kl * L::S + i * 32 + r], s[t], o[i], 0, 0, 0);
    }
    if (kt + 1 < kt1) attn_store_tile<D>(lds, stage ^ 1, pk, pv);
    __syncthreads();
  }

  attn_epilogue<D>(o, m_run, l_run, lds, O, ldo, row_base, head, q0, qt, n_qt, clip, t_stride, KS, ks, r16, part, cnt,
                   L::BYTES);
}

// ---------------------------------------------------------------------------------------------
// bf16x3 attention (f32 graph in the default bf16x3 GEMM mode): the same flash structure with both products on
// v_mfma_f32_32x32x16_bf16 in split form (x y ~= xh yh + xh yl + xl yh, f32 accumulate, ~2^-16 relative per product;
// 3 x 32 cycles per 32x32x16 step instead of 8 x 64 for the exact-f32 form):
//   S^T = K . Q^T: A = K fragment (lane: key r, dims 16 s + 8 h + 0..7 of k-step s), B = Q^T (lane: query r, the same
//     dims); Q is split once per block, K while staged (planes Kh, Kl [AK][D + 8]);
//   O^T += V^T . P^T: B = P^T straight from the S accumulator (registers 8 s .. 8 s + 7 of lane half h are the keys
//     16 s + 8 (j >> 2) + 4 h + (j & 3): cdna_hip_programming.md "accumulator tile as the next MFMA's operand"), split
//     in registers; A = V^T fragment (lane: dim r, the same 8 keys) read as 8 f32 values from the exact kernel's V tile
//     image (conflict-free, as there) and split in registers: a transposed bf16 V image costs 16-way conflicted
//     2-byte LDS writes in the staging pass (measured at batch 32: 516 vs 412 us per call; exact f32: 679).
//   Softmax, masking, key splits and the epilogue are the exact-f32 kernel's.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8a __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4a __attribute__((ext_vector_type(4)));

// FA_ATTN_TRV = 1: V is split into bf16 planes while staged too ([key][D + 32] rows) and the V^T fragments are read with
// ds_read_b64_tr_b16 (4 keys x 16 dims per 16-lane group, two reads per plane per fragment), instead of 8 f32 LDS
// reads + 8 in-register splits per fragment. Row stride D + 32 bf16 (16 or 48 mod 64 dwords): the two 16-lane groups
// of a 32-lane half read 4 rows x 8 dwords each on 64 distinct banks. Same split values, same MFMA order: outputs
// bit-identical to FA_ATTN_TRV = 0.
#ifndef FA_ATTN_TRV
#define FA_ATTN_TRV 1
#endif
// FA_ATTN_DIAG (microbenchmark builds only; wrong results by construction): 1 = no K/V global loads or LDS stores in
// the key loop, 2 = no S MFMAs, 3 = no PV MFMAs, 4 = no softmax (exp / max / sum)
#ifndef FA_ATTN_DIAG
#define FA_ATTN_DIAG 0
#endif
template <int D>
struct AttnLds3 {
  static constexpr int SK = D + 8;                   // K plane row (bf16): 16-B reads of 16 rows, distinct bank groups
  static constexpr int KP = AK * SK;                 // bf16 per K plane
  static constexpr int VOFF = 2 * KP / 2;            // V tile offset (floats) after the Kh, Kl planes
  static constexpr int SV = D + 32;                  // V plane row (bf16, FA_ATTN_TRV)
  static constexpr int VP = AK * SV;                 // bf16 per V plane
  static constexpr int STAGE = VOFF + (FA_ATTN_TRV ? VP : AttnLds<D>::TILE);  // floats per stage
  static constexpr int BYTES_PIPE = 2 * STAGE * 4;
  static constexpr int BYTES_OUT = AttnLds<D>::BYTES_OUT;
  static constexpr int BYTES = (BYTES_PIPE > BYTES_OUT ? BYTES_PIPE : BYTES_OUT) + 2 * AQ * 4 + 16;
};

template <int D, int P = 3>
__device__ __forceinline__ void attn3_store_tile(float* st, const f4v (&pk)[AK * D / 1024], const f4v (&pv)[AK * D / 1024]) {
  using L = AttnLds3<D>;
  __bf16* kb = reinterpret_cast<__bf16*>(st);
  float* vs_ = st + L::VOFF;
#pragma unroll
  for (int c = 0; c < AK * D / 1024; ++c) {
    const int f = threadIdx.x + 256 * c;
    const int key = f / (D / 4), d4 = f % (D / 4);
    if constexpr (P == 1) {  // fp16 graph: K and V are fp16 values, one exact f16 plane each
      const f4v v = pk[c], w = pv[c];
      _Float16* kh = reinterpret_cast<_Float16*>(st);
      _Float16* vh = reinterpret_cast<_Float16*>(vs_);
      *reinterpret_cast<f16x4a*>(kh + key * L::SK + 4 * d4) = f16x4a{(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
      *reinterpret_cast<f16x4a*>(vh + key * L::SV + 4 * d4) = f16x4a{(_Float16)w.x, (_Float16)w.y, (_Float16)w.z, (_Float16)w.w};
      continue;
    }
    const f4v v = pk[c];
    const bf16x4 hi = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    const bf16x4 lo = {(__bf16)(v.x - (float)hi[0]), (__bf16)(v.y - (float)hi[1]), (__bf16)(v.z - (float)hi[2]),
                       (__bf16)(v.w - (float)hi[3])};
    *reinterpret_cast<bf16x4*>(kb + key * L::SK + 4 * d4) = hi;
    *reinterpret_cast<bf16x4*>(kb + L::KP + key * L::SK + 4 * d4) = lo;
    if constexpr (FA_ATTN_TRV) {
      __bf16* vb = reinterpret_cast<__bf16*>(vs_);
      const f4v w = pv[c];
      const bf16x4 vh = {(__bf16)w.x, (__bf16)w.y, (__bf16)w.z, (__bf16)w.w};
      const bf16x4 vl = {(__bf16)(w.x - (float)vh[0]), (__bf16)(w.y - (float)vh[1]), (__bf16)(w.z - (float)vh[2]),
                         (__bf16)(w.w - (float)vh[3])};
      *reinterpret_cast<bf16x4*>(vb + key * L::SV + 4 * d4) = vh;
      *reinterpret_cast<bf16x4*>(vb + L::VP + key * L::SV + 4 * d4) = vl;
    } else {
      *reinterpret_cast<f4v*>(vs_ + key * AttnLds<D>::S + 4 * d4) = pv[c];
    }
  }
}

// 4 keys x 1 dim per lane from a row-major bf16 [key][SV] plane: lane 4q + p of its 16-lane group supplies row q,
// columns 4p .. 4p + 3 of the group's 4 x 16 block and receives column (lane & 15) of the 4 rows (T10)
typedef short v4i16 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bf16x4 ld_tr4(const __bf16* p) {
  const v4i16 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(p));
  return __builtin_bit_cast(bf16x4, v);
}
__device__ __forceinline__ f16x4a ld_tr4h(const _Float16* p) {
  const v4i16 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(p));
  return __builtin_bit_cast(f16x4a, v);
}

// XCD-aware block order: the blocks that stream the same K/V rows -- the query tiles of one (key split, head, clip)
// group -- are dispatched to one XCD, so that XCD's L2 fetches those rows once, instead of the round-robin dispatch
// (linear block id % 8) sending them to eight L2s. Linear id -> XCD lin % 8, slot lin / 8 -> query tile slot % per of
// group (slot / per) 8 + XCD (per = the grid's query tiles per group); a bijection of the same grid when the group
// count is a multiple of 8 (otherwise the dispatch order stays). Results unchanged.
__device__ __forceinline__ void attn_xcd_coords(int per, int KS, int& qt, int& ks, int& head, int& clip) {
  const int G = KS * gridDim.y * gridDim.z;
  if ((int)gridDim.x != per * KS || (G & 7)) return;
  const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int slot = lin >> 3, grp = (slot / per) * 8 + (lin & 7);
  qt = slot % per;
  ks = grp % KS;
  head = (grp / KS) % gridDim.y;
  clip = grp / (KS * gridDim.y);
}

// P = 1: the fp16 graph's attention (C5) on v_mfma_f32_32x32x16_f16: q, k and v are fp16 values (outputs of the fp16
// q|k|v projection), so S^T = K . Q^T is one f16 MFMA per 16 of k with exact products (d^-0.5 applied to the f32
// scores after the dot), and O^T += V^T . P^T is two (P^T split into f16 hi + lo in registers, V^T exact): the
// attention stays f32 arithmetic on fp16 inputs with its output rounded to fp16, the oracle's contract
// (oracle/encoder_fp16.py); 3 MFMAs per 16 keys x 16 dims instead of the exact-f32 form's 8 x 64 cycles
// S = 1: write-after-barrier staging (as k_gemm_bf3_256 S = 1): the registers holding key tile kt + 1, loaded a whole
// step earlier, go to the free stage at the top of step kt and then take tile kt + 2's loads. Same MFMA order.
// Two blocks per CU (launch bounds; LDS 76.8 KB per block at D = 128): unbounded, hipcc parked 64 values in AGPRs
// beside 254 VGPRs and the kernel ran one wave per SIMD; bounded it fits 256 registers without scratch.
template <int D, int P = 3, int S = 0>
__global__ __launch_bounds__(256, 2) void k_attn_bf3(const float* __restrict__ Q, const float* __restrict__ Kp,
                                                  const float* __restrict__ V, int64_t ldq, int64_t ldk, int64_t ldv,
                                                  float* __restrict__ O, int64_t ldo, int t_stride,
                                                  const int* __restrict__ lens, float scale, int KS,
                                                  float* __restrict__ part, int* __restrict__ cnt, APlanesD op,
                                                  int xcd_order) {
  using L = AttnLds3<D>;
  constexpr int NDT = D / 32;
  constexpr int NKS = D / 16;  // k-steps of the S product
  extern __shared__ float lds[];
  const int n_qt = (t_stride + AQ - 1) / AQ;
  const int n_qt8 = (n_qt + 7) & ~7;
  int qt = blockIdx.x % n_qt8, ks = blockIdx.x / n_qt8, head = blockIdx.y, clip = blockIdx.z;
  if (xcd_order) attn_xcd_coords(KS == 1 ? n_qt : n_qt8, KS, qt, ks, head, clip);
  if (qt >= n_qt) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t row_base = (int64_t)clip * t_stride;
  const int len = lens ? lens[clip] : t_stride;
  const int q0 = qt * AQ;
  const int n_kt = (t_stride + AK - 1) / AK;
  const int tpk = (n_kt + KS - 1) / KS;
  const int kt0 = ks * tpk, kt1 = min(n_kt, kt0 + tpk);
  // this wave's 32 queries, pre-scaled (python: q * d_k**-0.5 before the dot), split into bf16 fragments (P = 1: the
  // fp16 q values as they are, scaled after the dot)
  bf16x8 qh[NKS], ql[NKS];
  f16x8a qf[NKS];
  {
    const int q = min(q0 + wave * 32 + r, t_stride - 1);
    const float* p = Q + (row_base + q) * ldq + head * D + 8 * h;
#pragma unroll
    for (int st = 0; st < NKS; ++st) {
      const float4 a = *reinterpret_cast<const float4*>(p + 16 * st);
      const float4 b = *reinterpret_cast<const float4*>(p + 16 * st + 4);
      if constexpr (P == 1) {
        qf[st] = f16x8a{(_Float16)a.x, (_Float16)a.y, (_Float16)a.z, (_Float16)a.w, (_Float16)b.x, (_Float16)b.y,
                        (_Float16)b.z, (_Float16)b.w};
        continue;
      }
      const float x[8] = {a.x * scale, a.y * scale, a.z * scale, a.w * scale, b.x * scale, b.y * scale, b.z * scale,
                          b.w * scale};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        qh[st][j] = (__bf16)x[j];
        ql[st][j] = (__bf16)(x[j] - (float)qh[st][j]);
      }
    }
  }
  f32x16 o[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) o[i] = f32x16{};
  float m_run = -INFINITY, l_run = 0.f;
  f4v pk[AK * D / 1024], pv[AK * D / 1024];
  if (kt0 < kt1) {
    attn_load_tile<D>(Kp, V, ldk, ldv, row_base, head, t_stride, kt0, pk, pv);
    attn3_store_tile<D, P>(lds, pk, pv);
    if (S == 1 && kt0 + 1 < kt1) attn_load_tile<D>(Kp, V, ldk, ldv, row_base, head, t_stride, kt0 + 1, pk, pv);
  }
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int stage = (kt - kt0) & 1;
    if constexpr (S == 1) {
      if (kt + 1 < kt1) attn3_store_tile<D, P>(lds + (stage ^ 1) * L::STAGE, pk, pv);
      if (kt + 2 < kt1) attn_load_tile<D>(Kp, V, ldk, ldv, row_base, head, t_stride, kt + 2, pk, pv);  // in flight
    } else if (FA_ATTN_DIAG != 1) {
      if (kt + 1 < kt1) attn_load_tile<D>(Kp, V, ldk, ldv, row_base, head, t_stride, kt + 1, pk, pv);  // in flight
    }
    const __bf16* kh_ = reinterpret_cast<const __bf16*>(lds + stage * L::STAGE);
    const float* vs_ = lds + stage * L::STAGE + L::VOFF;
    const int k0 = kt * AK;
    f32x16 s = {};
    if constexpr (P == 1) {
      const _Float16* kf_ = reinterpret_cast<const _Float16*>(kh_);
#pragma unroll
      for (int st = 0; st < NKS; ++st) {
        const f16x8a kf = *reinterpret_cast<const f16x8a*>(kf_ + r * L::SK + 16 * st + 8 * h);
        s = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[st], s, 0, 0, 0);
      }
      s *= scale;
    } else {
#pragma unroll
      for (int st = 0; st < NKS; ++st) {
        const bf16x8 kh = *reinterpret_cast<const bf16x8*>(kh_ + r * L::SK + 16 * st + 8 * h);
        const bf16x8 kl = *reinterpret_cast<const bf16x8*>(kh_ + L::KP + r * L::SK + 16 * st + 8 * h);
#if FA_ATTN_DIAG == 2
        asm volatile("" ::"v"(kh), "v"(kl), "v"(qh[st]), "v"(ql[st]));
        s[st] += (float)kh[0];
#else
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl, qh[st], s, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, ql[st], s, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh, qh[st], s, 0, 0, 0);
#endif
      }
    }
    // mask + online softmax (as k_attn_f32)
#if FA_ATTN_DIAG == 4
    float alpha = 1.f;
    asm volatile("" : "+v"(alpha));
    m_run = 0.f;
#else
    // a tile of valid keys only (block-uniform; every tile but a clip's last) needs no mask and holds no -inf score:
    // the same values without the per-score compares and selects
    const bool full = k0 + AK <= min(len, t_stride);
    float mt = -INFINITY;
    if (full) {
#pragma unroll
      for (int t = 0; t < 16; ++t) mt = fmaxf(mt, s[t]);
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int key = k0 + (t & 3) + 8 * (t >> 2) + 4 * h;
        float v = s[t];
        if (key >= t_stride) v = -INFINITY;
        else if (key >= len) v = v + -10000.0f;
        s[t] = v;
        mt = fmaxf(mt, v);
      }
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float m_new = fmaxf(m_run, mt);
    const float alpha = m_run == -INFINITY ? 0.f : __expf(m_run - m_new);
    float ls = 0.f;
    if (full) {
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const float p = __expf(s[t] - m_new);
        s[t] = p;
        ls += p;
      }
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const float p = s[t] == -INFINITY ? 0.f : __expf(s[t] - m_new);
        s[t] = p;
        ls += p;
      }
    }
    ls += __shfl_xor(ls, 32, 64);
    l_run = l_run * alpha + ls;
    m_run = m_new;
#endif
#pragma unroll
    for (int i = 0; i < NDT; ++i) o[i] *= alpha;
    // O^T[d][q] += V^T[d][key] P^T[key][q]: P^T k-step s2 = registers 8 s2 .. 8 s2 + 7 (keys 16 s2 + kl(j))
#pragma unroll
    for (int s2 = 0; s2 < AK / 16; ++s2) {
      if constexpr (P == 1) {
        f16x8a ph, pl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          ph[j] = (_Float16)s[8 * s2 + j];
          pl[j] = (_Float16)(s[8 * s2 + j] - (float)ph[j]);
        }
        const _Float16* vb = reinterpret_cast<const _Float16*>(vs_);
        const int gq = lane >> 4, key = 16 * s2 + 4 * (gq >> 1) + ((lane >> 2) & 3);
#pragma unroll
        for (int i = 0; i < NDT; ++i) {
          const int off = key * L::SV + 32 * i + 16 * (gq & 1) + 4 * (lane & 3);
          const f16x4a h0 = ld_tr4h(vb + off), h1 = ld_tr4h(vb + off + 8 * L::SV);
          const f16x8a vh = f16x8a{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
          o[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, pl, o[i], 0, 0, 0);
          o[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, ph, o[i], 0, 0, 0);
        }
        continue;
      }
      bf16x8 ph, pl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ph[j] = (__bf16)s[8 * s2 + j];
        pl[j] = (__bf16)(s[8 * s2 + j] - (float)ph[j]);
      }
#pragma unroll
      for (int i = 0; i < NDT; ++i) {
        bf16x8 vh, vl;
        if constexpr (FA_ATTN_TRV) {
          // lane group gq = lane >> 4: keys 16 s2 + 4 (gq >> 1) (+ 8), dims 32 i + 16 (gq & 1) + 0..15; this lane's
          // address: row (lane >> 2) & 3 of the block, columns 4 (lane & 3) .. +3
          const __bf16* vb = reinterpret_cast<const __bf16*>(vs_);
          const int gq = lane >> 4, key = 16 * s2 + 4 * (gq >> 1) + ((lane >> 2) & 3);
          const int off = key * L::SV + 32 * i + 16 * (gq & 1) + 4 * (lane & 3);
          const bf16x4 h0 = ld_tr4(vb + off), h1 = ld_tr4(vb + off + 8 * L::SV);
          const bf16x4 l0 = ld_tr4(vb + L::VP + off), l1 = ld_tr4(vb + L::VP + off + 8 * L::SV);
          vh = bf16x8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
          vl = bf16x8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int key = 16 * s2 + 8 * (j >> 2) + 4 * h + (j & 3);
            const float x = vs_[key * AttnLds<D>::S + i * 32 + r];
            vh[j] = (__bf16)x;
            vl[j] = (__bf16)(x - (float)vh[j]);
          }
        }
#if FA_ATTN_DIAG == 3
        asm volatile("" ::"v"(vh), "v"(vl), "v"(ph), "v"(pl));
        o[i][0] += (float)vh[0];
#else
        o[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vl, ph, o[i], 0, 0, 0);
        o[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, pl, o[i], 0, 0, 0);
        o[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vh, ph, o[i], 0, 0, 0);
#endif
      }
    }
    if (S == 0 && FA_ATTN_DIAG != 1 && kt + 1 < kt1) attn3_store_tile<D, P>(lds + (stage ^ 1) * L::STAGE, pk, pv);
    __syncthreads();
  }
  attn_epilogue<D>(o, m_run, l_run, lds, O, ldo, row_base, head, q0, qt, n_qt, clip, t_stride, KS, ks, P == 1 ? 1 : 0,
                   part, cnt, L::BYTES, op);
}

int g_attn_f32_force_splits = 0;  // test hook (scripts/ubench/attn_f32_check.hip)
int g_attn_f16_mfma = 1;          // fp16 graph attention on f16 MFMAs (k_attn_bf3<D, 1>); 0: exact f32 + rounding (A/B)
int g_attn_wab = 0;               // k_attn_bf3 write-after-barrier staging (S = 1; FUNASR_ATTN_WAB)
int g_attn_xcd = 0;               // k_attn_bf3 XCD-aware block order (FUNASR_ATTN_XCD=1; measured neutral: off)
int g_attn_merge = 1;             // key splits merged by their own launch (k_attn_merge) instead of the last split

template <int D, int P>
static void launch_attn_bf3(dim3 grid, hipStream_t s, const float* Q, const float* K, const float* V, int64_t ldq,
                            int64_t ldk, int64_t ldv, float* O, int64_t ldo, int t_stride, const int* lens, float scale,
                            int KS, const AttnF32Work& wk, APlanesD op = {}) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_attn_bf3<D, P, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, AttnLds3<D>::BYTES);
    (void)hipFuncSetAttribute((const void*)k_attn_bf3<D, P, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, AttnLds3<D>::BYTES);
    attr = true;
  }
  const int xo = g_attn_xcd;
  if (g_attn_wab)
    hipLaunchKernelGGL((k_attn_bf3<D, P, 1>), grid, dim3(256), AttnLds3<D>::BYTES, s, Q, K, V, ldq, ldk, ldv, O, ldo,
                       t_stride, lens, scale, KS, wk.part, wk.cnt, op, xo);
  else
    hipLaunchKernelGGL((k_attn_bf3<D, P, 0>), grid, dim3(256), AttnLds3<D>::BYTES, s, Q, K, V, ldq, ldk, ldv, O, ldo,
                       t_stride, lens, scale, KS, wk.part, wk.cnt, op, xo);
}

int attn_f32_splits(int batch, int t_stride, int n_heads) {
  if (g_attn_f32_force_splits > 0) return g_attn_f32_force_splits;
  const int blocks = cdiv(t_stride, AQ) * n_heads * batch;
  const int n_kt = cdiv(t_stride, AK);
  int ks = 1;
  while (blocks * ks * 2 <= 512 && ks * 2 <= 8 && n_kt >= ks * 2 * 2) ks *= 2;
  return ks;
}

void attn_f32(const float* Q, const float* K, const float* V, int64_t ldq, int64_t ldk, int64_t ldv, float* O,
              int64_t ldo, int batch, int t_stride, int n_heads, int head_dim, const int* lens,
              const AttnF32Work& wk, hipStream_t s, int r16, int bf3, APlanes op) {
  FA_REQUIRE(!op.hi || (bf3 && !r16), "attn_f32: bf16 output planes need the bf16x3 mode");
  const APlanesD opd{reinterpret_cast<__bf16*>(op.hi), reinterpret_cast<__bf16*>(op.lo)};
  const int KS = attn_f32_splits(batch, t_stride, n_heads);
  FA_REQUIRE(KS >= 1 && KS <= 8, "attn_f32: 1-8 key splits (16 measured slower: 60 vs 39 us at T = 1001)");
  const int n_tiles = cdiv(t_stride, AQ) * n_heads * batch;
  if (KS > 1)
    FA_REQUIRE(wk.part && wk.cnt && n_tiles <= wk.cnt_n &&
                   (int64_t)n_tiles * KS * (AQ * head_dim + 2 * AQ) <= wk.part_n,
               "attn_f32: split workspace too small");
  dim3 grid(KS == 1 ? cdiv(t_stride, AQ) : ((cdiv(t_stride, AQ) + 7) & ~7) * KS, n_heads, batch);
  const float scale = (float)std::pow((double)head_dim, -0.5);  // python d_k ** -0.5 rounded to f32
  // g_attn_merge: the splits only publish (no counter: cnt = nullptr) and k_attn_merge merges every tile after them
  const bool sep = KS > 1 && g_attn_merge;
  AttnF32Work wka = wk;
  if (sep) wka.cnt = nullptr;
  auto merge = [&]() {
    if (!sep) return;
    const int n_qt = cdiv(t_stride, AQ);
    const int r16m = r16 ? 1 : 0;
    const int ms = (g_attn_ms >= 1 && g_attn_ms <= 32 && AQ % g_attn_ms == 0) ? g_attn_ms : 8;
    if (head_dim == 128)
      hipLaunchKernelGGL(k_attn_merge<128>, dim3(n_tiles * ms), dim3(256), 0, s, wk.part, KS, n_qt, n_heads, O,
                         ldo, t_stride, r16m, opd, ms);
    else
      hipLaunchKernelGGL(k_attn_merge<64>, dim3(n_tiles * ms), dim3(256), 0, s, wk.part, KS, n_qt, n_heads, O,
                         ldo, t_stride, r16m, opd, ms);
  };
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_attn_f32<128>, hipFuncAttributeMaxDynamicSharedMemorySize, AttnLds<128>::BYTES);
    (void)hipFuncSetAttribute((const void*)k_attn_f32<64>, hipFuncAttributeMaxDynamicSharedMemorySize, AttnLds<64>::BYTES);
    attr_set = true;
  }
  if (r16 && g_attn_f16_mfma) {
    FA_REQUIRE(head_dim == 128 || head_dim == 64, "attn_f32: head_dim must be 64 or 128");
    if (head_dim == 128) launch_attn_bf3<128, 1>(grid, s, Q, K, V, ldq, ldk, ldv, O, ldo, t_stride, lens, scale, KS, wka);
    else launch_attn_bf3<64, 1>(grid, s, Q, K, V, ldq, ldk, ldv, O, ldo, t_stride, lens, scale, KS, wka);
    merge();
    return;
  }
  if (bf3 && !r16) {
    FA_REQUIRE(head_dim == 128 || head_dim == 64, "attn_f32: head_dim must be 64 or 128");
    if (head_dim == 128) launch_attn_bf3<128, 3>(grid, s, Q, K, V, ldq, ldk, ldv, O, ldo, t_stride, lens, scale, KS, wka, opd);
    else launch_attn_bf3<64, 3>(grid, s, Q, K, V, ldq, ldk, ldv, O, ldo, t_stride, lens, scale, KS, wka, opd);
    merge();
    return;
  }
  if (head_dim == 128) {
    hipLaunchKernelGGL(k_attn_f32<128>, grid, dim3(256), AttnLds<128>::BYTES, s, Q, K, V, ldq, ldk, ldv, O, ldo,
                       t_stride, lens, scale, KS, r16, wka.part, wka.cnt);
    merge();
  } else if (head_dim == 64) {
    hipLaunchKernelGGL(k_attn_f32<64>, grid, dim3(256), AttnLds<64>::BYTES, s, Q, K, V, ldq, ldk, ldv, O, ldo,
                       t_stride, lens, scale, KS, r16, wka.part, wka.cnt);
    merge();
  } else {
    FA_REQUIRE(false, "attn_f32: head_dim must be 64 or 128");
  }
}

}  // namespace fa
