// How fast can one workgroup pull a kv head's K/V rows (n_keys x 2 x 256 B) from its XCD's L2 when the 16 workgroups
// of that head (blocks g + 8 sp: one XCD under round-robin placement) all read the same bytes?
// grid (8 heads, 16 blocks per head), 256 threads; every lane loads 16 B per instruction, NI loads in flight.
// modes: 0 = every block reads its head's region in the same order; 1 = block sp starts at a rotated offset
// (sp x region / 16); 2 = distinct regions per block (no sharing; 16x the bytes from HBM/MALL on the first pass);
// 3 = each block reads 1/16 of its head's region (the split form's share).
// Timed: R graph-replayed launches back to back (L2-warm after the first) -> us per launch; also one in-kernel
// s_memrealtime span per block (median / max over blocks).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int NI>
__global__ __launch_bounds__(256) void k_share(const int4* __restrict__ base, int64_t head_stride_v, int n_v, int mode,
                                               float* __restrict__ out, unsigned long long* __restrict__ span) {
  const int g = blockIdx.x, sp = blockIdx.y;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int4* p = base + (mode == 2 ? (int64_t)(g * 16 + sp) : (int64_t)g) * head_stride_v;
  int n = n_v, off0 = 0;
  if (mode == 3) {
    n = n_v / 16;
    p += (int64_t)sp * n;
  }
  if (mode == 1) off0 = (int)((int64_t)sp * n / 16);
  int acc = 0;
  for (int i0 = threadIdx.x; i0 < n; i0 += 256 * NI) {
    int4 v[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      int i = i0 + 256 * j;
      i = i < n ? i : n - 1;
      int k = i + off0;
      k = k >= n ? k - n : k;
      v[j] = p[k];
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) acc += v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  }
  __shared__ int s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  atomicAdd(&s, acc);
  __syncthreads();
  if (threadIdx.x == 0) {
    out[g * 16 + sp] = (float)s;
    span[g * 16 + sp] = __builtin_amdgcn_s_memrealtime() - t0;
  }
}

int main(int argc, char** argv) {
  const int keys = argc > 1 ? atoi(argv[1]) : 330;
  const int64_t bytes = (int64_t)keys * 2 * 256;  // K + V rows of one kv head
  const int n_v = (int)(bytes / 16);
  const int64_t hs = ((bytes + 4095) / 4096) * 4096 / 16;  // int4 per region
  int4* buf;
  CK(hipMalloc(&buf, hs * 16 * 8 * 16));
  CK(hipMemset(buf, 1, hs * 16 * 8 * 16));
  float* out;
  unsigned long long* span;
  CK(hipMalloc(&out, 128 * 4));
  CK(hipMalloc(&span, 128 * 8));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char* names[] = {"shared, same order", "shared, rotated start", "distinct regions", "1/16 share (split form)"};
  for (int ni : {4, 8}) {
    for (int mode = 0; mode < 4; ++mode) {
      hipGraph_t gr;
      hipGraphExec_t ex;
      const int R = 20;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int r = 0; r < R; ++r) {
        if (ni == 4) hipLaunchKernelGGL(k_share<4>, dim3(8, 16), dim3(256), 0, s, buf, hs, n_v, mode, out, span);
        else hipLaunchKernelGGL(k_share<8>, dim3(8, 16), dim3(256), 0, s, buf, hs, n_v, mode, out, span);
      }
      CK(hipStreamEndCapture(s, &gr));
      CK(hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0));
      for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ex, s));
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(a, s));
      for (int w = 0; w < 10; ++w) CK(hipGraphLaunch(ex, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      std::vector<unsigned long long> h(128);
      CK(hipMemcpy(h.data(), span, 128 * 8, hipMemcpyDeviceToHost));
      std::sort(h.begin(), h.end());
      const double per = ms * 1e3 / (10 * R);
      const double rb = mode == 3 ? bytes / 16.0 : (double)bytes;
      printf("keys %d NI %d %-26s: %6.2f us per launch; in-kernel span p50 %.2f max %.2f us -> %.1f GB/s per block (p50)\n",
             keys, ni, names[mode], per, h[64] / 100.0, h[127] / 100.0, rb / (h[64] / 100.0) / 1e3);
      CK(hipGraphExecDestroy(ex));
      CK(hipGraphDestroy(gr));
    }
  }
  return 0;
}
