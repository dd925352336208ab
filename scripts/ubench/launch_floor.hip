// Kernel-boundary floor on this box: back-to-back dependent launches of trivial kernels, eager vs hipGraph,
// 1 block vs 256 blocks, and with/without a global write. Prints microseconds per launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
__global__ void k_empty() {}
__global__ void k_touch(int* p) { if (threadIdx.x == 0) p[blockIdx.x] += 1; }
int main() {
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int* buf; CK(hipMalloc(&buf, 4096 * 4)); CK(hipMemset(buf, 0, 4096 * 4));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const int N = 2000;
  struct V { const char* name; int blocks; bool touch; };
  V vs[] = {{"empty 1x64", 1, false}, {"empty 256x256", 256, false}, {"touch 1x64", 1, true}, {"touch 256x256", 256, true}};
  for (auto& v : vs) {
    dim3 g(v.blocks), t(v.blocks == 1 ? 64 : 256);
    for (int w = 0; w < 100; ++w) { if (v.touch) hipLaunchKernelGGL(k_touch, g, t, 0, s, buf); else hipLaunchKernelGGL(k_empty, g, t, 0, s); }
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int i = 0; i < N; ++i) { if (v.touch) hipLaunchKernelGGL(k_touch, g, t, 0, s, buf); else hipLaunchKernelGGL(k_empty, g, t, 0, s); }
    CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    // graph of 100 launches
    hipGraph_t gr; hipGraphExec_t ex;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < 100; ++i) { if (v.touch) hipLaunchKernelGGL(k_touch, g, t, 0, s, buf); else hipLaunchKernelGGL(k_empty, g, t, 0, s); }
    CK(hipStreamEndCapture(s, &gr)); CK(hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ex, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int i = 0; i < N / 100; ++i) CK(hipGraphLaunch(ex, s));
    CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
    float msg; CK(hipEventElapsedTime(&msg, a, b));
    printf("%-16s eager %.2f us/launch   graph %.2f us/launch\n", v.name, ms * 1e3 / N, msg * 1e3 / N);
    hipGraphExecDestroy(ex); hipGraphDestroy(gr);
  }
  return 0;
}
