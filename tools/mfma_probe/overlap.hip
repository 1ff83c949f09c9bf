// Can a SIMD run one wave's fp32 MFMAs and another wave's VALU at the same time?  (measurement
// tool, not shipped; the C5 learner's question)  One 512-thread block per CU:
// waves w = 0..7 sit on SIMD w % 4 (HW_ID checked and reported).  Cases: only the MFMA waves
// (w < 4) work, only the VALU waves (w >= 4) work, both work.  If the mixed time is the max of
// the two, the pipes overlap across waves; if it is the sum, they share the SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_probe/overlap tools/mfma_probe/overlap.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f16v __attribute__((ext_vector_type(16)));

template <int KIND>  // 0: f32 MFMA, 1: bf16 MFMA
__device__ float mfma_work(int iters, float seed) {
  f16v c[4];
  for (int k = 0; k < 4; k++)
    for (int i = 0; i < 16; i++) c[k][i] = 0.f;
  const float a = seed + threadIdx.x * 1e-3f, b = 1.f - seed;
  if constexpr (KIND == 0) {
    for (int it = 0; it < iters; it++)
#pragma unroll
      for (int k = 0; k < 4; k++) c[k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c[k], 0, 0, 0);
  } else {
    typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
    bf8v av, bv;
    for (int j = 0; j < 8; j++) { av[j] = (__bf16)(a + j); bv[j] = (__bf16)(b - j); }
    for (int it = 0; it < iters; it++)
#pragma unroll
      for (int k = 0; k < 4; k++) c[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, c[k], 0, 0, 0);
  }
  float s = 0.f;
  for (int k = 0; k < 4; k++) s += c[k][0] + c[k][15];
  return s;
}

__device__ float valu_work(int iters, float seed) {
  float x0 = seed, x1 = seed + 1, x2 = seed + 2, x3 = seed + 3, x4 = seed + 4, x5 = seed + 5, x6 = seed + 6,
        x7 = seed + 7;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {  // 8 independent chains of v_fma_f32
      x0 = __builtin_fmaf(x0, 0.999f, 0.5f); x1 = __builtin_fmaf(x1, 0.999f, 0.5f);
      x2 = __builtin_fmaf(x2, 0.999f, 0.5f); x3 = __builtin_fmaf(x3, 0.999f, 0.5f);
      x4 = __builtin_fmaf(x4, 0.999f, 0.5f); x5 = __builtin_fmaf(x5, 0.999f, 0.5f);
      x6 = __builtin_fmaf(x6, 0.999f, 0.5f); x7 = __builtin_fmaf(x7, 0.999f, 0.5f);
    }
  }
  return x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

template <int KIND>
__global__ __launch_bounds__(512) void k_overlap(float* out, unsigned* simd, int mode, int mfma_iters, int valu_iters) {
  const int w = threadIdx.x >> 6;
  float s = 0.f;
  if (w < 4 && (mode & 1)) s = mfma_work<KIND>(mfma_iters, 0.25f);
  if (w >= 4 && (mode & 2)) s = valu_work(valu_iters, 0.5f);
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0 && blockIdx.x == 0)
    simd[w] = (__builtin_amdgcn_s_getreg(4 | (31 << 11)) >> 4) & 3;  // HW_ID.SIMD_ID
}

template <int KIND>
static float timed(float* out, unsigned* simd, int mode, int mi, int vi) {
  hipLaunchKernelGGL(k_overlap<KIND>, dim3(256), dim3(512), 0, 0, out, simd, mode, 10, 10);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_overlap<KIND>, dim3(256), dim3(512), 0, 0, out, simd, mode, mi, vi);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  float* out = nullptr;
  unsigned* simd = nullptr;
  if (hipMalloc(&out, 256 * 512 * 4) != hipSuccess || hipMalloc(&simd, 64) != hipSuccess || !out || !simd) return 1;
  printf("{\"cases\": [\n");
  for (int kind = 0; kind < 2; kind++) {
    const int mi = kind == 0 ? 4000 : 8000, vi = 4000;
    float t[4];
    for (int mode = 1; mode <= 3; mode++)
      t[mode] = kind == 0 ? timed<0>(out, simd, mode, mi, vi) : timed<1>(out, simd, mode, mi, vi);
    printf("  {\"mfma\": \"%s\", \"mfma_only_ms\": %.3f, \"valu_only_ms\": %.3f, \"both_ms\": %.3f, "
           "\"both_over_sum\": %.3f, \"both_over_max\": %.3f}%s\n", kind == 0 ? "f32_32x32x2" : "bf16_32x32x16",
           t[1], t[2], t[3], t[3] / (t[1] + t[2]), t[3] / (t[1] > t[2] ? t[1] : t[2]), kind == 0 ? "," : "");
  }
  unsigned h[8];
  (void)hipMemcpy(h, simd, sizeof(h), hipMemcpyDeviceToHost);
  printf("], \"simd_of_wave\": [%u, %u, %u, %u, %u, %u, %u, %u]}\n", h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
  return 0;
}
