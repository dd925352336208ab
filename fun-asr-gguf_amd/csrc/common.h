// Shared helpers for the MI355X (gfx950) Fun-ASR engine. Wave = 64 lanes everywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <string>

namespace fa {

void set_error(const std::string& msg);
void log(int level, const std::string& msg);

#define FA_HIP(expr)                                                                          \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) {                                                                   \
      ::fa::set_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " __FILE__ ":" + \
                      std::to_string(__LINE__) + " (" #expr ")");                             \
      throw ::fa::hip_failure();                                                              \
    }                                                                                         \
  } while (0)

struct hip_failure {};
struct arg_failure {};

#define FA_REQUIRE(cond, msg)                      \
  do {                                             \
    if (!(cond)) {                                 \
      ::fa::set_error(std::string("invalid: ") + (msg)); \
      throw ::fa::arg_failure();                   \
    }                                              \
  } while (0)

constexpr int WAVE = 64;

// Wave-wide reductions on DPP (row-local quad_perm / half-mirror / mirror) + 4 readlanes, instead of
// __shfl_xor's ds_bpermute round trips through the LDS crossbar. Result is wave-uniform.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, false);
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;

__device__ __forceinline__ float row_sum16(float v) {  // sum over each 16-lane row, every lane of the row
  v += dpp_f<DPP_XOR1>(v);
  v += dpp_f<DPP_XOR2>(v);
  v += dpp_f<DPP_HALF_MIRROR>(v);
  v += dpp_f<DPP_MIRROR>(v);
  return v;
}
__device__ __forceinline__ float row_max16(float v) {
  v = fmaxf(v, dpp_f<DPP_XOR1>(v));
  v = fmaxf(v, dpp_f<DPP_XOR2>(v));
  v = fmaxf(v, dpp_f<DPP_HALF_MIRROR>(v));
  v = fmaxf(v, dpp_f<DPP_MIRROR>(v));
  return v;
}
// max over aligned groups of N lanes (N = 2, 4, 8, 16), result in every lane of the group
template <int N>
__device__ __forceinline__ float group_max(float v) {
  if (N >= 2) v = fmaxf(v, dpp_f<DPP_XOR1>(v));
  if (N >= 4) v = fmaxf(v, dpp_f<DPP_XOR2>(v));
  if (N >= 8) v = fmaxf(v, dpp_f<DPP_HALF_MIRROR>(v));
  if (N >= 16) v = fmaxf(v, dpp_f<DPP_MIRROR>(v));
  return v;
}
__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wave_sum(float v) {
  v = row_sum16(v);
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
  v = row_max16(v);
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}
__device__ __forceinline__ int wave_sum_i(int v) {
  v += dpp_i<DPP_XOR1>(v);
  v += dpp_i<DPP_XOR2>(v);
  v += dpp_i<DPP_HALF_MIRROR>(v);
  v += dpp_i<DPP_MIRROR>(v);
  return (__builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16)) +
         (__builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48));
}

// 16-B loads/stores with the sc1 cache policy (bypass the CU's L1) through a raw buffer resource, for
// cross-workgroup hand-offs (MI355X_MICROARCH.md hand-off table, row 1). The builtins traffic in int
// vectors: always bit-cast explicitly (an implicit scalar*int-vector promotes the scalar to int).
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef int i32x4v_t __attribute__((ext_vector_type(4)));
constexpr int CPOL_SC1 = 16;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}
__device__ __forceinline__ f32x4_t ld_sc1_f4(__amdgpu_buffer_rsrc_t rs, int byte_off) {
  return __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, CPOL_SC1));
}
__device__ __forceinline__ float ld_sc1_f1(__amdgpu_buffer_rsrc_t rs, int byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, byte_off, 0, CPOL_SC1));
}
__device__ __forceinline__ void st_sc1_f4(f32x4_t v, __amdgpu_buffer_rsrc_t rs, int byte_off) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4v_t, v), rs, byte_off, 0, CPOL_SC1);
}

// bf16x3 encoder activations handed between kernels as their two bf16 planes (APlanes in kernels.h): hi = bf16_rn(v),
// lo = bf16_rn(v - hi), exactly the split the bf16x3 GEMM's staging applies to an f32 A row
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
struct APlanesD {
  __bf16* hi = nullptr;
  __bf16* lo = nullptr;
};
__device__ __forceinline__ void split_bf16x4(const float4 v, bf16x4_t& h, bf16x4_t& l) {
  h = bf16x4_t{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
  l = bf16x4_t{(__bf16)(v.x - (float)h[0]), (__bf16)(v.y - (float)h[1]), (__bf16)(v.z - (float)h[2]),
               (__bf16)(v.w - (float)h[3])};
}
__device__ __forceinline__ void split_bf16(const float v, __bf16& h, __bf16& l) {
  h = (__bf16)v;
  l = (__bf16)(v - (float)h);
}

// (value, index) argmax with torch/numpy semantics: NaN ranks above every number (the first NaN wins, as
// numpy.argmax), then the larger value, then the smaller index on ties. A total order, so the reduction is order-free
// and any input replaces the (-inf, INT_MAX) seed: an all-NaN row still yields a real token id, never the seed's
// out-of-range index (which the sampler's embed-next gather would then read past token_embd with).
__device__ __forceinline__ void argmax_combine(float& v, int& i, float v2, int i2) {
  const bool vn = v != v, v2n = v2 != v2;
  if (v2n ? (!vn || i2 < i) : (!vn && (v2 > v || (v2 == v && i2 < i)))) {
    v = v2;
    i = i2;
  }
}

inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

}  // namespace fa
