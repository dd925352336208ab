// Encoder self-attention (SANM / adaptor / CTC-decoder): out = softmax(q*d^-0.5 . k^T + mask) . v
// per head, full-length (non-causal) with the reference's additive key mask (m-1)*1e4
// (model_definition.py:68-78, 122-145). Exact-f32 MFMA (v_mfma_f32_32x32x2_f32), flash-style:
//
//   block = (32-query tile, head, clip); 4 waves split the key tiles (w, w+4, ...), each keeps its own
//   online-softmax state; partial (m, l, O) are merged through LDS at the end.
//   S^T = K . Q^T so the query index sits on the lane (col) and keys on the 16 accumulator registers:
//   the per-query max/sum is an in-register reduction + one cross-half shuffle, and S^T is directly the
//   B operand of O^T += V^T . P^T (key order permuted consistently on both operands).
// Q/K fragments: lane (r=l&31, h=l>>5) holds row r, dims [h*D/2, h*D/2+D/2) — the dot-product index is
// permuted identically on A and B, so each lane loads D/2 contiguous floats (float4s).
#include "common.h"
#include "kernels.h"

#include <cmath>

namespace fa {

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int D>
__global__ __launch_bounds__(256) void k_attn_f32(const float* __restrict__ Q, const float* __restrict__ Kp,
                                                  const float* __restrict__ V, int64_t ldq, int64_t ldk, int64_t ldv,
                                                  float* __restrict__ O, int64_t ldo, int t_stride,
                                                  const int* __restrict__ lens, float scale) {
  constexpr int HD = D / 2;     // dims per lane half
  constexpr int NDT = D / 32;   // output d-tiles
  extern __shared__ float lds[];
  const int qt = blockIdx.x, head = blockIdx.y, clip = blockIdx.z;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t row_base = (int64_t)clip * t_stride;
  const int len = lens ? lens[clip] : t_stride;
  const int q0 = qt * 32;

  float qreg[HD];
  {
    int q = q0 + r;
    const float* p = Q + (row_base + q) * ldq + head * D + h * HD;
#pragma unroll
    for (int s = 0; s < HD; s += 4) {
      float4 v = q < t_stride ? *reinterpret_cast<const float4*>(p + s) : make_float4(0.f, 0.f, 0.f, 0.f);
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

  const int n_kt = (t_stride + 31) / 32;
  for (int kt = wave; kt < n_kt; kt += 4) {
    const int k0 = kt * 32;
    f32x16 s = {};
    {
      int key = k0 + r;
      const float* p = Kp + (row_base + key) * ldk + head * D + h * HD;
      bool ok = key < t_stride;
#pragma unroll
      for (int c = 0; c < HD; c += 16) {
        float kr[16];
#pragma unroll
        for (int e = 0; e < 16; e += 4) {
          float4 v = ok ? *reinterpret_cast<const float4*>(p + c + e) : make_float4(0.f, 0.f, 0.f, 0.f);
          kr[e] = v.x;
          kr[e + 1] = v.y;
          kr[e + 2] = v.z;
          kr[e + 3] = v.w;
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) s = __builtin_amdgcn_mfma_f32_32x32x2f32(kr[e], qreg[c + e], s, 0, 0, 0);
      }
    }
    // mask + online softmax (per query = per lane column)
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      int key = k0 + (t & 3) + 8 * (t >> 2) + 4 * h;
      float v = s[t];
      if (key >= t_stride) v = -INFINITY;
      else if (key >= len) v = v + -10000.0f;
      s[t] = v;
      mt = fmaxf(mt, v);
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    float m_new = fmaxf(m_run, mt);
    float alpha = m_run == -INFINITY ? 0.f : __expf(m_run - m_new);
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      float p = s[t] == -INFINITY ? 0.f : __expf(s[t] - m_new);
      s[t] = p;
      ls += p;
    }
    ls += __shfl_xor(ls, 32, 64);
    l_run = l_run * alpha + ls;
    m_run = m_new;
#pragma unroll
    for (int i = 0; i < NDT; ++i) o[i] *= alpha;
    // O^T[d][q] += sum_key V[key][d] * P^T[key][q]
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      int key = k0 + (t & 3) + 8 * (t >> 2) + 4 * h;
      const float* vp = V + (row_base + key) * ldv + head * D + r;
      bool ok = key < t_stride;
#pragma unroll
      for (int i = 0; i < NDT; ++i) {
        float vv = ok ? vp[i * 32] : 0.f;
        o[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(vv, s[t], o[i], 0, 0, 0);
      }
    }
  }
  // ---- merge the 4 waves' partial states through LDS
  float* sm = lds;                   // [4][32]
  float* sl = lds + 128;             // [4][32]
  float* so = lds + 256;             // [4][D][32]
  if (h == 0) {
    sm[wave * 32 + r] = m_run;
    sl[wave * 32 + r] = l_run;
  }
#pragma unroll
  for (int i = 0; i < NDT; ++i)
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      int d = i * 32 + (t & 3) + 8 * (t >> 2) + 4 * h;
      so[(wave * D + d) * 32 + r] = o[i][t];
    }
  __syncthreads();
  // 256 threads: thread -> query q = tid & 31, d group
  const int q = threadIdx.x & 31;
  float M = -INFINITY;
#pragma unroll
  for (int w = 0; w < 4; ++w) M = fmaxf(M, sm[w * 32 + q]);
  float wsc[4], L = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    float mw = sm[w * 32 + q];
    wsc[w] = mw == -INFINITY ? 0.f : __expf(mw - M);
    L += wsc[w] * sl[w * 32 + q];
  }
  const float inv = 1.0f / L;
  const int qrow = q0 + q;
  if (qrow < t_stride) {
    float* op = O + (row_base + qrow) * ldo + head * D;
    for (int d = threadIdx.x >> 5; d < D; d += 8) {
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) acc += wsc[w] * so[(w * D + d) * 32 + q];
      op[d] = acc * inv;
    }
  }
}

void attn_f32(const float* Q, const float* K, const float* V, int64_t ldq, int64_t ldk, int64_t ldv, float* O,
              int64_t ldo, int batch, int t_stride, int n_heads, int head_dim, const int* lens, hipStream_t s) {
  dim3 grid(cdiv(t_stride, 32), n_heads, batch);
  const float scale = (float)std::pow((double)head_dim, -0.5);  // python d_k ** -0.5 rounded to f32
  size_t lds = (256 + 4 * head_dim * 32) * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)k_attn_f32<128>, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * 1024);
    hipFuncSetAttribute((const void*)k_attn_f32<64>, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * 1024);
    attr_set = true;
  }
  if (head_dim == 128) {
    hipLaunchKernelGGL(k_attn_f32<128>, grid, dim3(256), lds, s, Q, K, V, ldq, ldk, ldv, O, ldo, t_stride, lens, scale);
  } else if (head_dim == 64) {
    hipLaunchKernelGGL(k_attn_f32<64>, grid, dim3(256), lds, s, Q, K, V, ldq, ldk, ldv, O, ldo, t_stride, lens, scale);
  } else {
    FA_REQUIRE(false, "attn_f32: head_dim must be 64 or 128");
  }
}

}  // namespace fa
