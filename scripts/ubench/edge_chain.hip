// Price of one all-to-all activation edge inside a persistent launch vs a kernel boundary, at the decode
// layer's real sizes: 1024 producing waves (256 WGs x 4) each publish NG/1024 f32 values as 8-byte
// {value, tag} granules (sc1 atomic stores); every WG sweeps all NG granules (sc1 16-B buffer loads) until
// every tag matches, stages them in LDS, and consumes one value. A chain of E edges in one launch; per-edge
// time = (t(E) - t(0)) / E. Spins are bounded (s_memrealtime, 0.2 s) and report a timeout word.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int NG>
__global__ __launch_bounds__(256) void k_chain(uint64_t* gbuf, int n_edges, int sweepers, uint32_t* tmo, float* out) {
  __shared__ float s_x[NG];
  __shared__ int s_fail;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + wave;
  constexpr int PER = NG / 1024;
  float acc = 0.f;
  if (threadIdx.x == 0) s_fail = 0;
  __syncthreads();
  for (int e = 0; e < n_edges; ++e) {
    uint64_t* g = gbuf + (size_t)(e & 1) * NG;
    const uint32_t tag = (uint32_t)e + 1;
    if (lane < PER) {
      const float v = acc + (float)(gw + lane);
      const uint64_t x = ((uint64_t)tag << 32) | (uint64_t)__float_as_uint(v);
      __hip_atomic_store(g + gw * PER + lane, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (wave < sweepers) {
      const int per_wave = NG / sweepers;          // granules
      const int nl = per_wave / 128;               // 16-B loads per lane (2 granules each)
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(g, 0, NG * 8, 0x00020000);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      bool ok = false;
      while (!ok) {
        ok = true;
        for (int i = 0; i < nl; ++i) {
          const int gi = wave * per_wave + (i * 64 + lane) * 2;
          const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, gi * 8, 0, 16);
          ok &= ((uint32_t)v.y == tag) && ((uint32_t)v.w == tag);
          s_x[gi] = __int_as_float(v.x);
          s_x[gi + 1] = __int_as_float(v.z);
        }
        ok = __all(ok);
        if (!ok && __builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {
          if (lane == 0) { __hip_atomic_store(tmo, 1u + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); s_fail = 1; }
          break;
        }
      }
    }
    __syncthreads();
    acc += s_x[(gw * 7 + e) % NG] * 1e-3f;
    if (s_fail) break;
  }
  if (lane == 0) out[gw] = acc;
}

// the same edge as a kernel boundary: every WG reads the NG values (plain loads) and writes its own
template <int NG>
__global__ __launch_bounds__(256) void k_step(const float* in, float* outv) {
  __shared__ float s_x[NG];
  for (int i = threadIdx.x; i < NG / 4; i += 256) reinterpret_cast<float4*>(s_x)[i] = reinterpret_cast<const float4*>(in)[i];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + wave;
  constexpr int PER = NG / 1024;
  if (lane < PER) outv[gw * PER + lane] = s_x[(gw * 7) % NG] * 1e-3f + lane;
}

template <int NG>
int run(hipStream_t s, uint64_t* gbuf, uint32_t* tmo, float* out, float* a, float* b) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int sw : {1, 2, 4}) {
    float t[2];
    const int E[2] = {1, 2001};
    for (int r = 0; r < 2; ++r) {
      CK(hipMemsetAsync(gbuf, 0, 2 * NG * 8, s));
      CK(hipMemsetAsync(tmo, 0, 16, s));
      CK(hipEventRecord(e0, s));
      hipLaunchKernelGGL(k_chain<NG>, dim3(256), dim3(256), 0, s, gbuf, E[r], sw, tmo, out);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&t[r], e0, e1));
      uint32_t h;
      CK(hipMemcpy(&h, tmo, 4, hipMemcpyDeviceToHost));
      if (h) { printf("NG %d sweepers %d: TIMEOUT at edge %u\n", NG, sw, h - 1); return 1; }
    }
    printf("persistent edge  NG=%4d (%2d KB granules) sweepers=%d : %.2f us/edge\n", NG, NG * 8 / 1024, sw,
           (t[1] - t[0]) * 1e3 / 2000);
  }
  // kernel-boundary edges in a graph
  hipGraph_t gr; hipGraphExec_t ex;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_step<NG>, dim3(256), dim3(256), 0, s, (i & 1) ? b : a, (i & 1) ? a : b);
  CK(hipStreamEndCapture(s, &gr)); CK(hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0));
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ex, s));
  CK(hipStreamSynchronize(s));
  float ms;
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ex, s));
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("kernel-boundary edge NG=%4d (graph)            : %.2f us/edge\n", NG, ms * 1e3 / 2000);
  hipGraphExecDestroy(ex); hipGraphDestroy(gr);
  return 0;
}

int main() {
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint64_t* gbuf; uint32_t* tmo; float *out, *a, *b;
  CK(hipMalloc(&gbuf, 2 * 3072 * 8)); CK(hipMalloc(&tmo, 16)); CK(hipMalloc(&out, 1024 * 4));
  CK(hipMalloc(&a, 3072 * 4)); CK(hipMalloc(&b, 3072 * 4));
  CK(hipMemset(a, 0, 3072 * 4)); CK(hipMemset(b, 0, 3072 * 4));
  if (run<1024>(s, gbuf, tmo, out, a, b)) return 1;
  if (run<2048>(s, gbuf, tmo, out, a, b)) return 1;
  if (run<3072>(s, gbuf, tmo, out, a, b)) return 1;
  return 0;
}
