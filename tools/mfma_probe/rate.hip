// MFMA issue-rate probe (measurement tool, not shipped): the fp32 MFMA peak the C5 learner's
// roofline is priced against.  Each wave runs CHAINS independent accumulators through ITERS
// rounds of one MFMA kind; grid = 256 CUs x 4 SIMDs x WAVES waves (one 64-thread block per wave,
// waves_per_eu-free kernel).  Prints per case the FLOP rate and the SIMD cycles per MFMA at the
// clock the timing implies (2.4 GHz nominal).
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_probe/rate tools/mfma_probe/rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));

template <int KIND, int CHAINS>
__global__ __launch_bounds__(64) void k_rate(float* out, int iters, float seed) {
  float a = seed + threadIdx.x * 1e-3f, b = 1.0f - seed;
  if constexpr (KIND == 0) {  // v_mfma_f32_32x32x2_f32: 4096 FLOP
    f16v c[CHAINS];
    for (int k = 0; k < CHAINS; k++)
      for (int i = 0; i < 16; i++) c[k][i] = 0.f;
    for (int it = 0; it < iters; it++)
#pragma unroll
      for (int k = 0; k < CHAINS; k++) c[k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c[k], 0, 0, 0);
    float s = 0.f;
    for (int k = 0; k < CHAINS; k++) s += c[k][0] + c[k][15];
    out[blockIdx.x * 64 + threadIdx.x] = s;
  } else if constexpr (KIND == 1) {  // v_mfma_f32_16x16x4_f32: 2048 FLOP
    f4v c[CHAINS];
    for (int k = 0; k < CHAINS; k++)
      for (int i = 0; i < 4; i++) c[k][i] = 0.f;
    for (int it = 0; it < iters; it++)
#pragma unroll
      for (int k = 0; k < CHAINS; k++) c[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[k], 0, 0, 0);
    float s = 0.f;
    for (int k = 0; k < CHAINS; k++) s += c[k][0] + c[k][3];
    out[blockIdx.x * 64 + threadIdx.x] = s;
  } else {  // v_mfma_f32_32x32x16_bf16: 32768 FLOP
    bf8v av, bv;
    for (int j = 0; j < 8; j++) { av[j] = (__bf16)(a + j); bv[j] = (__bf16)(b - j); }
    f16v c[CHAINS];
    for (int k = 0; k < CHAINS; k++)
      for (int i = 0; i < 16; i++) c[k][i] = 0.f;
    for (int it = 0; it < iters; it++)
#pragma unroll
      for (int k = 0; k < CHAINS; k++) c[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, c[k], 0, 0, 0);
    float s = 0.f;
    for (int k = 0; k < CHAINS; k++) s += c[k][0] + c[k][15];
    out[blockIdx.x * 64 + threadIdx.x] = s;
  }
}

template <int KIND, int CHAINS>
static void run(const char* name, double flop, int waves, float* out, bool last) {
  const int blocks = 1024 * waves, iters = 4000 / CHAINS;
  hipLaunchKernelGGL((k_rate<KIND, CHAINS>), dim3(blocks), dim3(64), 0, 0, out, 50, 0.5f);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL((k_rate<KIND, CHAINS>), dim3(blocks), dim3(64), 0, 0, out, iters, 0.5f);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double n = (double)blocks * iters * CHAINS;  // MFMAs
  const double tf = n * flop / (ms * 1e-3) / 1e12;
  // per SIMD: waves * iters * CHAINS MFMAs in ms
  const double cyc = ms * 1e-3 * 2.4e9 / ((double)waves * iters * CHAINS);
  printf("  {\"kind\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"tflops\": %.1f, "
         "\"simd_cycles_per_mfma_at_2.4GHz\": %.1f}%s\n", name, CHAINS, waves, ms, tf, cyc, last ? "" : ",");
}

int main() {
  float* out = nullptr;
  if (hipMalloc(&out, 1024 * 4 * 64 * sizeof(float)) != hipSuccess || !out) return 1;
  printf("{\"cases\": [\n");
  for (int w = 1; w <= 4; w *= 2) {
    run<0, 1>("f32_32x32x2", 4096, w, out, false);
    run<0, 4>("f32_32x32x2", 4096, w, out, false);
    run<1, 1>("f32_16x16x4", 2048, w, out, false);
    run<1, 4>("f32_16x16x4", 2048, w, out, false);
    run<2, 4>("bf16_32x32x16", 32768, w, out, w == 4);
  }
  printf("]}\n");
  return 0;
}
