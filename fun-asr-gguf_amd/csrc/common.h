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

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// (value, index) argmax with torch/numpy first-occurrence tie-break (smaller index wins on equal value).
__device__ __forceinline__ void argmax_combine(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i) || (v != v)) {
    v = v2;
    i = i2;
  }
}

inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

}  // namespace fa
