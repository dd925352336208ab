// Device-side deterministic weight generation and q8_0 (de)quantisation / repacking.
//
// Weight hash spec (bit-identical to oracle/synth.py):
//   h = lowbias32(i ^ key); u = f32(h >> 8) * 2^-24 * 2 - 1; w = fl32(fl32(u * scale) + offset)
// q8_0 quantiser = ggml reference quantize_row_q8_0 (gguf/quants.py:378-393, declared bit-exact):
//   d = amax / 127; id = d ? 1/d : 0; q = roundf(x * id); d stored fp16 (RNE).
// Engine layout of a q8_0 matrix [O][K]: qs int8 [O][K] (16-B aligned rows) + d fp16 [O][K/32].
#include "common.h"
#include "kernels.h"

namespace fa {

__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

__global__ void k_synth_fill(float* __restrict__ out, int64_t n, uint32_t key, float scale, float offset) {
  // two IEEE roundings: hipcc fused fl(u * scale) + offset into one fma (the ocml bodies of __fmul_rn / __fadd_rn
  // carry the contract flag), which made ~2% of the offset-1 norm weights differ by 1 ulp from the spec
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    uint32_t h = lowbias32((uint32_t)i ^ key);
    float u = __fsub_rn(__fmul_rn(__fmul_rn((float)(h >> 8), 5.9604644775390625e-08f), 2.0f), 1.0f);
    float w = u * scale;
    asm volatile("" : "+v"(w));  // an opaque hop: the product is rounded before the add (no fma)
    if (offset != 0.0f) w = w + offset;
    out[i] = w;
  }
}

void launch_synth_fill(float* out, int64_t n, uint32_t key, float scale, float offset, hipStream_t s) {
  int grid = (int)std::min<int64_t>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(k_synth_fill, dim3(grid), dim3(256), 0, s, out, n, key, scale, offset);
}

// One 64-lane wave quantises 2 blocks (32 lanes per block, one element per lane).
__global__ void k_quant_q8_0(const float* __restrict__ x, int64_t n_blocks, int8_t* __restrict__ qs,
                             __half* __restrict__ d_out) {
  int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t blk = gid >> 5;
  int lane = threadIdx.x & 31;
  float v = blk < n_blocks ? x[gid] : 0.0f;
  float a = fabsf(v);
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) a = fmaxf(a, __shfl_xor(a, o, 32));
  float d = a / 127.0f;
  float id = d != 0.0f ? 1.0f / d : 0.0f;
  if (blk < n_blocks) {
    qs[gid] = (int8_t)roundf(__fmul_rn(v, id));
    if (lane == 0) d_out[blk] = __float2half_rn(d);
  }
}

void launch_quant_q8_0(const float* x, int64_t n, int8_t* qs, __half* d, hipStream_t s) {
  int64_t nb = n / 32;
  hipLaunchKernelGGL(k_quant_q8_0, dim3(cdiv(nb * 32, 256)), dim3(256), 0, s, x, nb, qs, d);
}

// ggml block layout (34 B: fp16 d + 32 x int8) <-> engine layout.
__global__ void k_unpack_q8_0(const uint8_t* __restrict__ blocks, int64_t n_blocks, int8_t* __restrict__ qs,
                              __half* __restrict__ d) {
  int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t blk = gid >> 5;
  int j = gid & 31;
  if (blk >= n_blocks) return;
  const uint8_t* b = blocks + blk * 34;
  qs[gid] = (int8_t)b[2 + j];
  if (j == 0) {
    uint16_t bits = (uint16_t)b[0] | ((uint16_t)b[1] << 8);
    d[blk] = __ushort_as_half(bits);
  }
}

__global__ void k_pack_q8_0(const int8_t* __restrict__ qs, const __half* __restrict__ d, int64_t n_blocks,
                            uint8_t* __restrict__ blocks) {
  int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t blk = gid >> 5;
  int j = gid & 31;
  if (blk >= n_blocks) return;
  uint8_t* b = blocks + blk * 34;
  b[2 + j] = (uint8_t)qs[gid];
  if (j == 0) {
    uint16_t bits = __half_as_ushort(d[blk]);
    b[0] = bits & 0xFF;
    b[1] = bits >> 8;
  }
}

void launch_unpack_q8_0(const uint8_t* blocks, int64_t n_blocks, int8_t* qs, __half* d, hipStream_t s) {
  hipLaunchKernelGGL(k_unpack_q8_0, dim3(cdiv(n_blocks * 32, 256)), dim3(256), 0, s, blocks, n_blocks, qs, d);
}
void launch_pack_q8_0(const int8_t* qs, const __half* d, int64_t n_blocks, uint8_t* blocks, hipStream_t s) {
  hipLaunchKernelGGL(k_pack_q8_0, dim3(cdiv(n_blocks * 32, 256)), dim3(256), 0, s, qs, d, n_blocks, blocks);
}

// f16 -> f32 (GGUF f16 norm tensors) .
__global__ void k_h2f(const __half* __restrict__ a, float* __restrict__ b, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = __half2float(a[i]);
}
void launch_h2f(const __half* a, float* b, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_h2f, dim3(cdiv(n, 256)), dim3(256), 0, s, a, b, n);
}

// f32 -> f16 as the float16 ONNX converter does for initializers (onnxruntime.transformers.float16,
// 02-Quantize-ONNX.py:21-27: min_positive_val 1e-7, max_finite_val 65504): nonzero magnitudes below 1e-7 become
// +-1e-7, magnitudes above 65504 become +-65504, then round to nearest even. round_only: plain RN (activations).
__global__ void k_f2h(const float* __restrict__ a, __half* __restrict__ b, float* __restrict__ b32, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = a[i];
  const float m = fabsf(v);
  if (m > 0.f && m < 1e-7f) v = copysignf(1e-7f, v);
  if (m > 65504.f) v = copysignf(65504.f, v);
  const __half h = __float2half_rn(v);
  if (b) b[i] = h;
  if (b32) b32[i] = __half2float(h);
}
void launch_f2h_initializer(const float* a, __half* b, float* b32, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_f2h, dim3(cdiv(n, 256)), dim3(256), 0, s, a, b, b32, n);
}

}  // namespace fa
