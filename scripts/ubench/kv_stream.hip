// Read rate of the batched-decode K/V access pattern without the attention math: 32 sequences x 8 kv heads, K and V
// streams of n_past 200-460 rows x 256 B in the head-major cache, 4 key splits per (sequence, head), 4 waves per block,
// each wave 1 KB (4 rows) per load instruction, 8 instructions of K and 8 of V in flight (as k_attn_block). Compared
// with the same bytes read as one contiguous region by the same grid. Graph-replayed over 28 layer copies.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(256) void k_kv(const int4* __restrict__ kc, const int4* __restrict__ vc, const int* __restrict__ pos,
                                            int64_t seq_stride16, int64_t head_stride16, int nsplit, int* out) {
  const int g = blockIdx.x, sp = blockIdx.y, m = blockIdx.z;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, kq = lane >> 4, dq = lane & 15;
  const int n_keys = pos[m] + 1, n_groups = (n_keys + 3) >> 2;
  const int gps = (n_groups + nsplit - 1) / nsplit;
  const int gb = sp * gps, ge = min(n_groups, gb + gps);
  const int4* kb = kc + m * seq_stride16 + g * head_stride16;
  const int4* vb = vc + m * seq_stride16 + g * head_stride16;
  int acc = 0;
  for (int g0 = gb + wave; g0 < ge; g0 += 32) {
    int4 t[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = min(4 * (g0 + 4 * i) + kq, n_keys - 1);
      t[i] = kb[(int64_t)k * 16 + dq];
      t[8 + i] = vb[(int64_t)k * 16 + dq];
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) acc += t[i].x ^ t[i].w;
  }
  if (acc == 0x7fffffff) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_flat(const int4* __restrict__ src, int64_t n16, int* out) {
  const int64_t nb = (int64_t)gridDim.x * gridDim.y * gridDim.z;
  const int64_t b = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  const int64_t per = (n16 + nb - 1) / nb, beg = b * per, end = min(n16, beg + per);
  int acc = 0;
  for (int64_t i0 = beg + threadIdx.x; i0 < end; i0 += 256 * 16) {
    int4 t[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) t[u] = src[min(i0 + u * 256, end - 1)];
#pragma unroll
    for (int u = 0; u < 16; ++u) acc += t[u].x ^ t[u].w;
  }
  if (acc == 0x7fffffff) out[0] = acc;
}

int main() {
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int M = 32, KV = 8, D = 128, NCTX = 1024, L = 28;
  const int64_t seq_stride = (int64_t)NCTX * KV * D, layer = M * seq_stride;  // halves
  int4 *kc, *vc; int* out;
  CK(hipMalloc(&kc, L * layer * 2)); CK(hipMalloc(&vc, L * layer * 2)); CK(hipMalloc(&out, 4));
  CK(hipMemset(kc, 1, L * layer * 2)); CK(hipMemset(vc, 1, L * layer * 2));
  std::vector<int> hp(M); double keys = 0;
  for (int m = 0; m < M; ++m) { hp[m] = 200 + (m * 97) % 261; keys += hp[m] + 1; }
  int* pos; CK(hipMalloc(&pos, M * 4)); CK(hipMemcpy(pos, hp.data(), M * 4, hipMemcpyHostToDevice));
  const double bytes = keys * KV * 256 * 2;
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto&& body) {
    hipGraph_t g; hipGraphExec_t ex;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal)); for (int l = 0; l < L; ++l) body(l); CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ex, s)); CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s)); for (int i = 0; i < 10; ++i) CK(hipGraphLaunch(ex, s)); CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / (10.0 * L);
    printf("%-44s %7.2f us per launch  %.2f TB/s\n", name, us, bytes / (us * 1e-6) / 1e12);
    CK(hipGraphExecDestroy(ex)); CK(hipGraphDestroy(g));
  };
  for (int ns : {1, 2, 4, 8})
    run(ns == 1 ? "K/V pattern, 1 split" : ns == 2 ? "K/V pattern, 2 splits" : ns == 4 ? "K/V pattern, 4 splits" : "K/V pattern, 8 splits",
        [&](int l) {
          hipLaunchKernelGGL(k_kv, dim3(KV, ns, M), dim3(256), 0, s, kc + l * layer / 8, vc + l * layer / 8, pos,
                             seq_stride / 8, (int64_t)NCTX * D / 8, ns, out);
        });
  const int64_t n16 = (int64_t)(bytes / 16);
  for (int nb : {256, 1024, 4096})
    run(nb == 256 ? "same bytes contiguous, 256 blocks" : nb == 1024 ? "same bytes contiguous, 1024 blocks" : "same bytes contiguous, 4096 blocks",
        [&](int l) { hipLaunchKernelGGL(k_flat, dim3(nb), dim3(256), 0, s, kc + l * layer / 8, n16, out); });
  return 0;
}
