// Encoder f32 GEMM (gemm_linear) per shape and tile variant, graph-timed; plus a CPU spot check.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>
#include "../../fun-asr-gguf_amd/csrc/kernels.h"
namespace fa {
extern int g_gemm_f32_force;
extern int g_gemm_bf3_force;
extern int g_gemm_bf3_256_s;
int gemm_bf3_occupancy_128();
extern int g_gemm_ks_force;
extern int g_gemm_bf3_sk_ks;
void set_error(const std::string& m) { printf("error: %s\n", m.c_str()); }
void log(int, const std::string&) {}
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
using namespace fa;
static hipStream_t s;
static double time_graph(std::function<void()> f, int reps) {
  hipGraph_t g; hipGraphExec_t ex;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < reps; ++i) f();
  CK(hipStreamEndCapture(s, &g)); CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ex, s)); CK(hipStreamSynchronize(s));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s)); for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ex, s)); CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGraphExecDestroy(ex)); CK(hipGraphDestroy(g));
  return ms * 1e3 / (3.0 * reps);
}
int main(int argc, char** argv) {
  const bool ksmode = argc > 1 && std::string(argv[1]) == "ks";  // K-split study on the single-clip shapes
  const int pad = argc > 1 && !ksmode ? atoi(argv[1]) : 0;  // extra floats per A / W row (stride study)
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int Mmax = 32032, Kmax = 2048 + 128, Nmax = 2048;
  float *A, *W, *bias, *C;
  CK(hipMalloc(&A, (size_t)Mmax * Kmax * 4)); CK(hipMalloc(&W, (size_t)Nmax * Kmax * 4));
  CK(hipMalloc(&bias, Nmax * 4)); CK(hipMalloc(&C, (size_t)Mmax * Nmax * 4));
  launch_synth_fill(A, (int64_t)Mmax * Kmax, 1, 1.f, 0.f, s); launch_synth_fill(W, (int64_t)Nmax * Kmax, 2, 0.05f, 0.f, s);
  launch_synth_fill(bias, Nmax, 3, 0.1f, 0.f, s);
  CK(hipStreamSynchronize(s));
  GemmF32Work wk; wk.cnt_n = 512; wk.part_n = (int64_t)512 * 256 * 16;
  CK(hipMalloc(&wk.part, wk.part_n * 4)); CK(hipMalloc(&wk.cnt, wk.cnt_n * CNT_LINE * 4));
  CK(hipMemset(wk.cnt, 0, wk.cnt_n * CNT_LINE * 4));
  {  // spot check: M=100 N=96 K=72 (partial tiles) against the CPU
    const int M = 100, N = 96, K = 72;
    for (int v : {1, 2, 3, 4}) {
      g_gemm_f32_force = v;
      gemm_linear(A, K, W, K, bias, C, N, M, N, K, 0, nullptr, 0, nullptr, 0, s);
      CK(hipStreamSynchronize(s));
      std::vector<float> a((size_t)M * K), w((size_t)N * K), b(N), c((size_t)M * N);
      CK(hipMemcpy(a.data(), A, a.size() * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(w.data(), W, w.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), bias, N * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(c.data(), C, c.size() * 4, hipMemcpyDeviceToHost));
      double err = 0;
      for (int i = 0; i < M; ++i) for (int j = 0; j < N; ++j) {
        double r = b[j]; for (int k = 0; k < K; ++k) r += (double)a[i * K + k] * w[j * K + k];
        err = std::max(err, std::fabs(r - c[i * N + j]));
      }
      printf("check variant %d: max|err| %.3g %s\n", v, err, err < 1e-4 ? "ok" : "FAIL");
    }
  }
  {  // split-K spot check: M=70 N=64 K=2048 (4 splits) against the CPU
    const int M = 70, N = 64, K = 2048;
    g_gemm_f32_force = 1;
    gemm_linear(A, K, W, K, bias, C, N, M, N, K, 0, nullptr, 0, nullptr, 0, s, nullptr, &wk);
    CK(hipStreamSynchronize(s));
    std::vector<float> a((size_t)M * K), w((size_t)N * K), b(N), c((size_t)M * N);
    CK(hipMemcpy(a.data(), A, a.size() * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(w.data(), W, w.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), bias, N * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(c.data(), C, c.size() * 4, hipMemcpyDeviceToHost));
    double err = 0;
    for (int i = 0; i < M; ++i) for (int j = 0; j < N; ++j) {
      double r = b[j]; for (int k = 0; k < K; ++k) r += (double)a[i * K + k] * w[j * K + k];
      err = std::max(err, std::fabs(r - c[i * N + j]));
    }
    printf("check split-K: max|err| %.3g %s\n", err, err < 1e-3 ? "ok" : "FAIL");
  }
  uint16_t *Wh, *Wl;
  CK(hipMalloc(&Wh, (size_t)Nmax * Kmax * 2)); CK(hipMalloc(&Wl, (size_t)Nmax * Kmax * 2));
  launch_split_bf16(W, Wh, Wl, (int64_t)Nmax * Kmax, s);
  WSplit wb; wb.hi = Wh; wb.lo = Wl;
  for (int sk = 0; sk < 3; ++sk) {  // bf16x3 spot checks (M=100 N=96 K=72; M=70 N=64 K=2048; K halves M=100 N=96 K=256)
    const int M = sk == 1 ? 70 : 100, N = sk == 1 ? 64 : 96, K = sk == 1 ? 2048 : sk == 2 ? 256 : 72;
    for (int v : {1, 2, 3, 4, 5, 6, 8, 9, 10}) {
      if ((sk == 1 && v == 2) || (sk < 2 && (v == 4 || v == 5)) || (sk == 2 && v < 4) || (v == 8 && sk != 1)) continue;
      if (v >= 9 && sk == 0) continue;
      g_gemm_bf3_force = v;
      gemm_linear(A, K, W, K, bias, C, N, M, N, K, 0, nullptr, 0, nullptr, 0, s, nullptr, sk ? &wk : nullptr, wb);
      CK(hipStreamSynchronize(s));
      std::vector<float> a((size_t)M * K), w((size_t)N * K), b(N), c((size_t)M * N);
      CK(hipMemcpy(a.data(), A, a.size() * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(w.data(), W, w.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), bias, N * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(c.data(), C, c.size() * 4, hipMemcpyDeviceToHost));
      double err = 0, mag = 0;
      for (int i = 0; i < M; ++i) for (int j = 0; j < N; ++j) {
        double r = b[j], m = std::fabs(b[j]);
        for (int k = 0; k < K; ++k) { r += (double)a[i * K + k] * w[j * K + k]; m += std::fabs((double)a[i * K + k] * w[j * K + k]); }
        err = std::max(err, std::fabs(r - c[i * N + j]) / m);
      }
      printf("check bf16x3 variant %d%s: max|err|/sum|aw| %.3g %s\n", v, sk == 1 ? " K 2048" : sk == 2 ? " K halves" : "", err,
             err < 3e-5 ? "ok" : "FAIL");
    }
  }
  g_gemm_bf3_force = 0;
  if (argc > 1 && std::string(argv[1]) == "sk") {  // few-tile planes-A shapes: 64x64 K groups vs k_gemm_bf3_sk (force 11)
    uint16_t *Ah, *Al;
    CK(hipMalloc(&Ah, (size_t)Mmax * Kmax * 2)); CK(hipMalloc(&Al, (size_t)Mmax * Kmax * 2));
    float* R;  // residual operand (EpiLinear add1)
    CK(hipMalloc(&R, (size_t)Mmax * Nmax * 4));
    launch_synth_fill(R, (int64_t)Mmax * Nmax, 4, 0.5f, 0.f, s);
    GemmF32Work big = wk;  // the engine's workspace after this change: 256 (tile, split) units
    big.part_n = (int64_t)256 * 16 * 1024;
    CK(hipMalloc(&big.part, big.part_n * 4));
    struct Sh { const char* name; int N, K; };
    const Sh sh4[] = {{"sanm qkv", 1536, 512}, {"sanm out", 512, 512}, {"ffn1", 2048, 512}, {"ffn2", 512, 2048}};
    const int Ms[] = {1001, 6006};
    for (int M : Ms)
      for (const Sh& sh : sh4) {
        launch_split_bf16(A, Ah, Al, (int64_t)M * sh.K, s);  // A rows of stride K as planes
        APlanes ap; ap.hi = Ah; ap.lo = Al;
        auto run = [&](int f, int ks) {
          g_gemm_bf3_force = f;
          g_gemm_bf3_sk_ks = ks;
          gemm_linear(nullptr, sh.K, W, sh.K, bias, C, sh.N, M, sh.N, sh.K, 0, R, sh.N, nullptr, 0, s, nullptr, &big, wb, ap);
        };
        std::vector<float> c0((size_t)M * sh.N), c1(c0.size());
        run(0, 0);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(c0.data(), C, c0.size() * 4, hipMemcpyDeviceToHost));
        printf("M=%5d %-9s:", M, sh.name);
        const double t0 = time_graph([&] { run(0, 0); }, 50);
        printf(" default %6.1f us", t0);
        printf("  64x64x64 pf2 %6.1f us", time_graph([&] { run(13, 0); }, 50));  // force 13: no branch -> the last one
        for (int fv : {11, 12})
        for (int ks : {0, 1, 2, 4, 8}) {
          if (ks && sh.K % (ks * 32)) continue;
          CK(hipMemsetAsync(C, 0, c1.size() * 4, s));
          run(fv, ks);
          CK(hipStreamSynchronize(s));
          CK(hipGetLastError());
          CK(hipMemcpy(c1.data(), C, c1.size() * 4, hipMemcpyDeviceToHost));
          double e = 0, mx = 0;
          for (size_t i = 0; i < c0.size(); ++i) { e = std::max(e, (double)std::fabs(c0[i] - c1[i])); mx = std::max(mx, (double)std::fabs(c0[i])); }
          const double us = time_graph([&] { run(fv, ks); }, 50);
          printf("  %s ks%d %6.1f us (dev %.0e%s)", fv == 11 ? "dma" : "reg", ks, us, e / mx, e / mx < 1e-5 ? "" : " FAIL");
        }
        printf("\n");
      }
    g_gemm_bf3_force = 0;
    g_gemm_bf3_sk_ks = 0;
    return 0;
  }
  if (argc > 1 && std::string(argv[1]) == "sched") {  // 256x256 staging schedules A/B, interleaved rounds, M = 32032
    struct Sh { const char* name; int N, K; };
    const Sh sh4[] = {{"sanm qkv", 1536, 512}, {"sanm out", 512, 512}, {"ffn1", 2048, 512}, {"ffn2", 512, 2048}};
    const int M = 32032;
    g_gemm_bf3_force = 6;
    for (const Sh& sh : sh4) {
      std::vector<float> c0((size_t)M * sh.N), c1(c0.size());
      for (int sc = 0; sc < 2; ++sc) {
        g_gemm_bf3_256_s = sc;
        CK(hipMemsetAsync(C, 0, c0.size() * 4, s));
        gemm_linear(A, sh.K, W, sh.K, bias, C, sh.N, M, sh.N, sh.K, 0, nullptr, 0, nullptr, 0, s, nullptr, &wk, wb);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy((sc ? c1 : c0).data(), C, c0.size() * 4, hipMemcpyDeviceToHost));
      }
      size_t nd = 0;
      for (size_t i = 0; i < c0.size(); ++i) nd += c0[i] != c1[i];
      printf("M=%d %-9s: schedule 1 vs 0: %zu outputs differ;", M, sh.name, nd);
      for (int round = 0; round < 3; ++round)
        for (int sc = 0; sc < 2; ++sc) {
          g_gemm_bf3_256_s = sc;
          const double us = time_graph([&] { gemm_linear(A, sh.K, W, sh.K, bias, C, sh.N, M, sh.N, sh.K, 0, nullptr, 0, nullptr, 0,
                                                         s, nullptr, &wk, wb); }, 10);
          printf("  s%d %6.1f us %5.1f TF/s", sc, us, 2.0 * M * sh.N * sh.K / us / 1e6);
        }
      printf("\n");
    }
    g_gemm_bf3_force = 2;  // the 128x128 tile, same A/B
    for (const Sh& sh : sh4) {
      printf("M=%d %-9s 128x128:", M, sh.name);
      for (int round = 0; round < 2; ++round)
        for (int sc = 0; sc < 2; ++sc) {
          g_gemm_bf3_256_s = sc;
          const double us = time_graph([&] { gemm_linear(A, sh.K, W, sh.K, bias, C, sh.N, M, sh.N, sh.K, 0, nullptr, 0, nullptr, 0,
                                                         s, nullptr, &wk, wb); }, 10);
          printf("  s%d %6.1f us %5.1f TF/s", sc, us, 2.0 * M * sh.N * sh.K / us / 1e6);
        }
      printf("\n");
    }
    g_gemm_bf3_256_s = 1;
    g_gemm_bf3_force = 0;
    return 0;
  }
  if (argc > 1 && std::string(argv[1]) == "kscan") {  // fixed vs per-k-step cost of the one-clip GEMMs (M = 1001)
    __half* W16;
    CK(hipMalloc(&W16, (size_t)Nmax * Kmax * 2));
    launch_f2h_initializer(W, W16, nullptr, (int64_t)Nmax * Kmax, s);
    CK(hipStreamSynchronize(s));
    struct Sh { const char* name; int N, K; };
    for (const Sh& sh : {Sh{"sanm qkv", 1536, 512}, Sh{"sanm out", 512, 512}, Sh{"ffn1", 2048, 512}, Sh{"ffn2", 512, 2048}}) {
      printf("M=1001 %-9s:", sh.name);
      for (int v : {0, 9, 10}) {
        g_gemm_bf3_force = v;
        const double b3 = time_graph([&] { gemm_linear(A, sh.K, W, sh.K, bias, C, sh.N, 1001, sh.N, sh.K, 0, nullptr, 0, nullptr, 0,
                                                       s, nullptr, &wk, wb); }, 50);
        const double f16 = time_graph([&] { gemm_linear(A, sh.K, W, sh.K, bias, C, sh.N, 1001, sh.N, sh.K, 0, nullptr, 0, nullptr, 0,
                                                        s, W16, &wk); }, 50);
        CK(hipGetLastError());
        double dev[2];
        for (int p16 = 0; p16 < 2; ++p16) {  // this variant vs the default policy, same precision
          std::vector<float> c0((size_t)1001 * sh.N), c1(c0.size());
          for (int pass = 0; pass < 2; ++pass) {
            g_gemm_bf3_force = pass ? v : 0;
            CK(hipMemsetAsync(C, 0, c0.size() * 4, s));
            gemm_linear(A, sh.K, W, sh.K, bias, C, sh.N, 1001, sh.N, sh.K, 0, nullptr, 0, nullptr, 0, s, p16 ? W16 : nullptr,
                        &wk, p16 ? WSplit{} : wb);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy((pass ? c1 : c0).data(), C, c0.size() * 4, hipMemcpyDeviceToHost));
          }
          double e = 0, mx = 0;
          for (size_t i = 0; i < c0.size(); ++i) { e = std::max(e, (double)std::fabs(c0[i] - c1[i])); mx = std::max(mx, (double)std::fabs(c0[i])); }
          dev[p16] = e / mx;
        }
        g_gemm_bf3_force = v;
        printf("  force %2d: bf16x3 %6.1f fp16 %6.1f us (dev %.0e / %.0e)", v, b3, f16, dev[0], dev[1]);
      }
      g_gemm_bf3_force = 0;
      printf("\n");
    }
    for (int N : {512, 1536}) {
      for (int K : {64, 128, 256, 512, 1024, 2048}) {
        const double b3 = time_graph([&] { gemm_linear(A, K, W, K, bias, C, N, 1001, N, K, 0, nullptr, 0, nullptr, 0, s,
                                                       nullptr, &wk, wb); }, 50);
        const double f16 = time_graph([&] { gemm_linear(A, K, W, K, bias, C, N, 1001, N, K, 0, nullptr, 0, nullptr, 0, s,
                                                        W16, &wk); }, 50);
        CK(hipGetLastError());
        printf("M=1001 N=%4d K=%4d: bf16x3 %6.1f us  fp16 %6.1f us\n", N, K, b3, f16);
      }
    }
    return 0;
  }
  struct Sh { const char* name; int N, K; };
  const Sh shapes[] = {{"sanm qkv", 1536, 512}, {"sanm out", 512, 512}, {"ffn1", 2048, 512}, {"ffn2", 512, 2048}};
  if (ksmode) {
    for (const Sh& sh : shapes) {
      std::vector<float> ref;
      for (int f32 : {1, 0})
        for (int v : {1, 3}) {
          printf("M=1001 %-9s %s %s:", sh.name, f32 ? "f32" : "bf3", v == 1 ? "64x64x32" : "64x64x64");
          for (int ks : {1, 2, 4}) {
            g_gemm_ks_force = ks;
            g_gemm_f32_force = v;
            g_gemm_bf3_force = v;
            const double us = time_graph([&] { gemm_linear(A, sh.K, W, sh.K, bias, C, sh.N, 1001, sh.N, sh.K, 0, nullptr, 0, nullptr, 0, s,
                                                           nullptr, &wk, f32 ? WSplit{} : wb); }, 50);
            CK(hipGetLastError());
            CK(hipMemsetAsync(C, 0, (size_t)1001 * sh.N * 4, s));
            gemm_linear(A, sh.K, W, sh.K, bias, C, sh.N, 1001, sh.N, sh.K, 0, nullptr, 0, nullptr, 0, s, nullptr, &wk,
                        f32 ? WSplit{} : wb);
            CK(hipStreamSynchronize(s));
            std::vector<float> c((size_t)1001 * sh.N);
            CK(hipMemcpy(c.data(), C, c.size() * 4, hipMemcpyDeviceToHost));
            if (ref.size() != c.size()) ref = c;
            double e = 0, mx = 0;
            for (size_t i = 0; i < c.size(); ++i) { e = std::max(e, (double)std::fabs(c[i] - ref[i])); mx = std::max(mx, (double)std::fabs(ref[i])); }
            printf("  ks %d %6.1f us (dev %.1e)", ks, us, e / mx);
          }
          printf("\n");
        }
    }
    return 0;
  }
  for (const Sh& sh : shapes) {  // 256x256 vs 128x128 tiles: same per-element MFMA order -> identical outputs
    const int M = 32032;
    std::vector<float> c2((size_t)M * sh.N), c6((size_t)M * sh.N);
    for (int v : {2, 6}) {
      g_gemm_bf3_force = v;
      CK(hipMemsetAsync(C, 0, (size_t)M * sh.N * 4, s));
      gemm_linear(A, sh.K, W, sh.K, bias, C, sh.N, M, sh.N, sh.K, 0, nullptr, 0, nullptr, 0, s, nullptr, &wk, wb);
      CK(hipStreamSynchronize(s));
      CK(hipMemcpy((v == 2 ? c2 : c6).data(), C, c2.size() * 4, hipMemcpyDeviceToHost));
    }
    size_t nd = 0;
    for (size_t i = 0; i < c2.size(); ++i) nd += c2[i] != c6[i];
    printf("bf3 256x256 vs 128x128, M=%d %s: %zu of %zu outputs differ %s\n", M, sh.name, nd, c2.size(), nd ? "FAIL" : "ok");
  }
  g_gemm_bf3_force = 0;
  printf("bf3 128x128x32: %d resident blocks per CU\n", gemm_bf3_occupancy_128());
  printf("row stride pad %d floats\n", pad);
  for (int M : {1001, 32032}) {
    if (pad && M > 2000) break;
    for (const Sh& sh : shapes) {
      printf("M=%5d %-9s N=%4d K=%4d:", M, sh.name, sh.N, sh.K);
      for (int v : {1, 5, 3, 2, 6}) {
        g_gemm_f32_force = v == 5 ? 1 : v == 6 ? 0 : v;
        const double us = time_graph([&] { gemm_linear(A, sh.K + pad, W, sh.K + pad, bias, C, sh.N, M, sh.N, sh.K, 0, nullptr, 0, nullptr, 0, s,
                                                       nullptr, v >= 5 ? &wk : nullptr); },
                                     M > 2000 ? 10 : 50);
        const char* nm[] = {"", "64x64x32", "128x128x32", "64x64x64", "64x64x128", "64x64x32 split-K", "engine default"};
        printf("  %s %7.1f us %5.1f TF/s", nm[v], us, 2.0 * M * sh.N * sh.K / us / 1e6);
      }
      for (int v : {1, 3, 4, 5, 8, 2, 6, 0}) {
        if ((v == 4 || v == 5) && (M > 2000 || sh.K % 128)) continue;
        if (v == 8 && (M > 2000 || sh.K < 2048)) continue;
        g_gemm_bf3_force = v;
        const double us = time_graph([&] { gemm_linear(A, sh.K + pad, W, sh.K + pad, bias, C, sh.N, M, sh.N, sh.K, 0, nullptr, 0, nullptr, 0, s,
                                                       nullptr, &wk, wb); },
                                     M > 2000 ? 10 : 50);
        const char* nm[] = {"bf3 default", "bf3 64x64x32", "bf3 128x128x32", "bf3 64x64x64", "bf3 64x64x64 K/2", "bf3 64x64x32 K/2",
                            "bf3 256x256x32", "", "bf3 64x64x32 K/4"};
        printf("  %s %7.1f us %5.1f TF/s", nm[v], us, 2.0 * M * sh.N * sh.K / us / 1e6);
      }
      g_gemm_bf3_force = 0;
      printf("\n");
    }
  }
  return 0;
}
