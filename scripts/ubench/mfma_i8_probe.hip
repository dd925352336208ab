// Verifies the operand map of v_mfma_i32_32x32x32_i8 on gfx950 with asymmetric exact-integer data:
// lane l holds A[l&31][16(l>>5)+j] and B[16(l>>5)+j][l&31] (j = 0..15, 16 bytes per lane);
// D: col = lane&31, row = (reg&3) + 8(reg>>2) + 4(lane>>5).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
__global__ void k(const int8_t* A, const int8_t* B, int* D) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; ++j) { a[j] = A[r * 32 + 16 * h + j]; b[j] = B[(16 * h + j) * 32 + r]; }
  i32x4 av = *reinterpret_cast<i32x4*>(a), bv = *reinterpret_cast<i32x4*>(b);
  i32x16 c = {};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
  for (int reg = 0; reg < 16; ++reg) D[((reg & 3) + 8 * (reg >> 2) + 4 * h) * 32 + r] = c[reg];
}
int main() {
  int8_t A[1024], B[1024]; int D[1024], R[1024];
  for (int i = 0; i < 32; ++i) for (int k2 = 0; k2 < 32; ++k2) { A[i * 32 + k2] = (int8_t)((i * 7 + k2 * 3) % 255 - 127); B[k2 * 32 + i] = (int8_t)((k2 * 11 - i * 5 + 300) % 253 - 126); }
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) { int s = 0; for (int k2 = 0; k2 < 32; ++k2) s += A[i * 32 + k2] * B[k2 * 32 + j]; R[i * 32 + j] = s; }
  int8_t *dA, *dB; int* dD;
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dD, 4096);
  hipMemcpy(dA, A, 1024, hipMemcpyHostToDevice); hipMemcpy(dB, B, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(D, dD, 4096, hipMemcpyDeviceToHost);
  int bad = 0; for (int i = 0; i < 1024; ++i) bad += D[i] != R[i];
  printf("mfma_i32_32x32x32_i8 assumed map: %d / 1024 mismatches (D[0]=%d R[0]=%d D[33]=%d R[33]=%d)\n", bad, D[0], R[0], D[33], R[33]);
  return bad != 0;
}
