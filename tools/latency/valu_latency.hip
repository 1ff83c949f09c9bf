// Issue and latency of the instruction kinds the fused tick is made of, for ONE wave per SIMD
// (C4's 32 768-arena shape) and for two (C3's 65 536), measured with s_memtime around unrolled
// asm blocks (measurement tool, not shipped).  Per kind: cycles per
// instruction of a dependent chain (each instruction reads the previous one's result) and of
// four independent chains interleaved.
//   hipcc --offload-arch=gfx950 -O3 -o tools/latency/valu_latency tools/latency/valu_latency.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

struct Res {
  unsigned long long t;
  unsigned sink;
};

template <int KIND>
__global__ void k_lat(Res* out, int iters) {
  unsigned a = threadIdx.x, b = threadIdx.x * 3u + 1u, c = threadIdx.x ^ 5u, d = threadIdx.x + 7u, one = 1u;
  __shared__ unsigned lds[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) lds[i] = (unsigned)(i + 1) & 1023u;
  __syncthreads();
  unsigned addr = (threadIdx.x * 4u) & 4095u;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (KIND == 0) {  // dependent v_add_u32
      asm volatile(REP64("v_add_u32 %0, %0, %1\n") : "+v"(a) : "v"(one));
    } else if constexpr (KIND == 1) {  // four independent chains
      asm volatile(REP8(REP8("v_add_u32 %0, %0, %4\nv_add_u32 %1, %1, %4\nv_add_u32 %2, %2, %4\nv_add_u32 %3, %3, %4\n"))
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(one));
    } else if constexpr (KIND == 2) {  // dependent v_mov_b32_dpp (pair swap)
      asm volatile(REP64("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\ns_nop 1\n") : "+v"(a));
    } else if constexpr (KIND == 3) {  // dependent v_cmp -> v_cndmask through VCC
      asm volatile(REP64("v_cmp_gt_u32 vcc, %0, %1\nv_cndmask_b32 %0, %1, %0, vcc\n") : "+v"(a) : "v"(b) : "vcc");
    } else if constexpr (KIND == 4) {  // dependent ds_read_b32 (address = previous result)
      asm volatile(REP8("ds_read_b32 %0, %0\ns_waitcnt lgkmcnt(0)\nv_lshlrev_b32 %0, 2, %0\n") : "+v"(addr) :: "memory");
    } else if constexpr (KIND == 5) {  // dependent v_fma_f32
      float x = __builtin_bit_cast(float, a | 0x3f800000u);
      asm volatile(REP64("v_fma_f32 %0, %0, %0, %0\n") : "+v"(x));
      a = __builtin_bit_cast(unsigned, x);
    } else if constexpr (KIND == 6) {  // dependent v_add_f64
      double x = (double)a;
      asm volatile(REP64("v_add_f64 %0, %0, %0\n") : "+v"(x));
      a = (unsigned)x;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0) out[w] = Res{t1 - t0, a + b + c + d + addr};
}

static const char* kNames[] = {"v_add_u32 dependent", "v_add_u32 4 chains", "v_mov_b32_dpp dependent (+s_nop 1)",
                               "v_cmp+v_cndmask via vcc dependent", "ds_read_b32 dependent (+wait, shift)",
                               "v_fma_f32 dependent", "v_add_f64 dependent"};
static const int kPerIter[] = {64, 256, 64, 64, 8, 64, 64};

template <int KIND>
static void run(int waves_per_simd, int cus, Res* d) {
  const int iters = 200;
  const int blocks = cus * waves_per_simd;  // 256 threads = one wave on each of the CU's 4 SIMDs
  hipLaunchKernelGGL(k_lat<KIND>, dim3(blocks), dim3(256), 0, 0, d, iters);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(k_lat<KIND>, dim3(blocks), dim3(256), 0, 0, d, iters);
  hipDeviceSynchronize();
  std::vector<Res> h(blocks * 4);
  hipMemcpy(h.data(), d, h.size() * sizeof(Res), hipMemcpyDeviceToHost);
  double s = 0;
  for (auto& r : h) s += (double)r.t;
  s /= h.size();
  // s_memtime counts at the shader clock's reference (100 MHz on gfx9 parts: scale by the
  // ratio measured below); reported raw per instruction and converted
  printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"memtime_ticks_per_inst\": %.4f}\n", kNames[KIND], waves_per_simd,
         s / (iters * (double)kPerIter[KIND]));
}

int main() {
  int dev = 0, cus = 0, clk = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
  printf("{\"cus\": %d, \"clock_khz\": %d}\n", cus, clk);
  Res* d;
  hipMalloc(&d, sizeof(Res) * cus * 4 * 2);
  for (int w = 1; w <= 2; ++w) {
    run<0>(w, cus, d);
    run<1>(w, cus, d);
    run<2>(w, cus, d);
    run<3>(w, cus, d);
    run<4>(w, cus, d);
    run<5>(w, cus, d);
    run<6>(w, cus, d);
  }
  hipFree(d);
  return 0;
}
