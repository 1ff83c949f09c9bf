// Layout probe for v_mfma_f32_32x32x16_bf16 on gfx950 (measurement tool, not shipped):
// D = A(32x16) * B(16x32) with exact small integers, then a chained product Y = W(32x32) * D
// taking D's accumulator registers as the B operand in the documented permuted k order.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k_probe(const float* A, const float* B, const float* W, float* D, float* Y) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  bf16x8 a, b;
  for (int j = 0; j < 8; j++) {
    a[j] = (__bf16)A[r * 16 + 8 * h + j];   // A[row r][k = 8h + j]
    b[j] = (__bf16)B[(8 * h + j) * 32 + r]; // B[k = 8h + j][col r]
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int i = 0; i < 16; i++) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * h, col = r;
    D[row * 32 + col] = c[i];
  }
  // Y = W * D: two k-steps s = 0, 1 over D's 32 rows; B fragment element j of half h = D row
  // 16s + 8(j>>2) + 4h + (j&3) = register 8s + j of this lane
  f32x16 y = {};
  for (int s = 0; s < 2; s++) {
    bf16x8 wa, db;
    for (int j = 0; j < 8; j++) {
      const int k = 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
      wa[j] = (__bf16)W[r * 32 + k];
      db[j] = (__bf16)c[8 * s + j];
    }
    y = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, db, y, 0, 0, 0);
  }
  for (int i = 0; i < 16; i++) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    Y[row * 32 + r] = y[i];
  }
}

int main() {
  float hA[32 * 16], hB[16 * 32], hW[32 * 32], hD[32 * 32], hY[32 * 32];
  for (int i = 0; i < 32 * 16; i++) hA[i] = (float)((i * 7) % 5 - 2);
  for (int i = 0; i < 16 * 32; i++) hB[i] = (float)((i * 3) % 7 - 3);
  for (int i = 0; i < 32 * 32; i++) hW[i] = (float)((i * 5) % 3 - 1);
  float *dA, *dB, *dW, *dD, *dY;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dW, sizeof hW);
  hipMalloc(&dD, sizeof hD); hipMalloc(&dY, sizeof hY);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipMemcpy(dW, hW, sizeof hW, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dW, dD, dY);
  hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
  hipMemcpy(hY, dY, sizeof hY, hipMemcpyDeviceToHost);
  int bad = 0, badY = 0;
  for (int i = 0; i < 32; i++)
    for (int j = 0; j < 32; j++) {
      float s = 0;
      for (int k = 0; k < 16; k++) s += hA[i * 16 + k] * hB[k * 32 + j];
      if (s != hD[i * 32 + j]) bad++;
    }
  for (int i = 0; i < 32; i++)
    for (int j = 0; j < 32; j++) {
      float s = 0;
      for (int k = 0; k < 32; k++) s += hW[i * 32 + k] * hD[k * 32 + j];
      if (s != hY[i * 32 + j]) badY++;
    }
  printf("D mismatches %d / 1024, Y (chained) mismatches %d / 1024\n", bad, badY);
  return bad || badY;
}
