// VALU issue-rate probe for gfx950 (measurement tool, not shipped).
//
// How many wave64 VALU instructions does one SIMD retire per cycle with 1, 2, 4 and 8 waves on
// it?  Every wave runs K blocks of 32 instructions on 4 register chains (each instruction reads
// only its own chain's register and constants, so it waits on nothing issued less than 4
// instructions earlier) and stamps its own shader-clock cycles
// (s_memtime) around the loop.  Per SIMD: instructions retired = waves x K x 32 over the
// slowest wave's cycles.  Instruction kinds: VOP2 (v_add_u32, v_add_f32, v_xor / v_or, v_and /
// v_lshlrev), VOP3 (v_add3_u32, v_bfe_u32), v_pk_add_f32, v_mov_b32_dpp (the pair exchange of
// fs_kernels.hip), v_cndmask_b32 with vcc and with an SGPR-pair mask, v_cmp into vcc, and a mix
// of v_add_u32 with s_add_u32 (does SALU from the partner wave co-issue).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_probe tools/valu_probe/probe.hip
//   /tmp/valu_probe > gpurun_out/valu_probe.json
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define REP4(x) x x x x
#define REP8(x) REP4(x) REP4(x)

template <int KIND>
__global__ __launch_bounds__(256) void k_probe(int iters, unsigned long long* cycles, unsigned* sink) {
  unsigned a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
  unsigned s0 = blockIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
    if constexpr (KIND == 0) {
      asm volatile(REP8("v_add_u32 %0, 1, %0\n v_add_u32 %1, 1, %1\n v_add_u32 %2, 1, %2\n v_add_u32 %3, 1, %3\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if constexpr (KIND == 1) {
      asm volatile(REP8("v_add3_u32 %0, %0, 1, 2\n v_add3_u32 %1, %1, 1, 2\n v_add3_u32 %2, %2, 1, 2\n "
                        "v_add3_u32 %3, %3, 1, 2\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if constexpr (KIND == 2) {
      asm volatile(REP8("v_add_f32 %0, 1.0, %0\n v_add_f32 %1, 1.0, %1\n v_add_f32 %2, 1.0, %2\n v_add_f32 %3, 1.0, %3\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if constexpr (KIND == 3) {
      unsigned long long p = ((unsigned long long)b << 32) | a, q = ((unsigned long long)d << 32) | c;
      unsigned long long r = p ^ 5, u = q ^ 3, k = 0x3f8000003f800000ull;
      asm volatile(REP8("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n "
                        "v_pk_add_f32 %3, %3, %4\n")
                   : "+v"(p), "+v"(q), "+v"(r), "+v"(u) : "v"(k));
      a = (unsigned)(p ^ r), b = (unsigned)((p ^ r) >> 32), c = (unsigned)(q ^ u), d = (unsigned)((q ^ u) >> 32);
    } else if constexpr (KIND == 4) {
      asm volatile(REP8("v_xor_b32 %0, 1, %0\n v_or_b32 %1, 2, %1\n v_xor_b32 %2, 4, %2\n v_or_b32 %3, 8, %3\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if constexpr (KIND == 5) {
      asm volatile(REP8("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n "
                        "v_mov_b32_dpp %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n "
                        "v_mov_b32_dpp %2, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n "
                        "v_mov_b32_dpp %3, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if constexpr (KIND == 7) {  // v_cndmask with independent chains (each reads only itself + a constant)
      const unsigned k = s0 | 1u;
      asm volatile("v_cmp_gt_u32 vcc, %0, %1\n" REP8("v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n "
                                                     "v_cndmask_b32 %2, %2, %4, vcc\n v_cndmask_b32 %3, %3, %4, vcc\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(k) : "vcc");
    } else if constexpr (KIND == 8) {  // the VOP3 form with an SGPR-pair mask
      unsigned long long m;
      asm volatile("v_cmp_gt_u32 %4, %0, %1\n" REP8("v_cndmask_b32_e64 %0, %0, 1, %4\n v_cndmask_b32_e64 %1, %1, 1, %4\n "
                                                    "v_cndmask_b32_e64 %2, %2, 1, %4\n v_cndmask_b32_e64 %3, %3, 1, %4\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "=s"(m));
    } else if constexpr (KIND == 9) {  // VOPC compares writing vcc (no reader)
      asm volatile(REP8("v_cmp_gt_u32 vcc, %0, %1\n v_cmp_gt_u32 vcc, %1, %2\n v_cmp_gt_u32 vcc, %2, %3\n "
                        "v_cmp_gt_u32 vcc, %3, %0\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : : "vcc");
    } else if constexpr (KIND == 10) {  // v_and_b32 / v_lshlrev_b32 (VOP2 integer)
      asm volatile(REP8("v_and_b32 %0, 0x7fffffff, %0\n v_lshlrev_b32 %1, 1, %1\n v_and_b32 %2, 0x7fffffff, %2\n "
                        "v_lshlrev_b32 %3, 1, %3\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if constexpr (KIND == 11) {  // v_bfe_u32 (VOP3 integer)
      asm volatile(REP8("v_bfe_u32 %0, %0, 1, 30\n v_bfe_u32 %1, %1, 1, 30\n v_bfe_u32 %2, %2, 1, 30\n "
                        "v_bfe_u32 %3, %3, 1, 30\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if constexpr (KIND == 12) {  // vcc written by SALU, then 32 e32 cndmasks
      const unsigned k = s0 | 1u;
      asm volatile("s_mov_b64 vcc, exec\n" REP8("v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n "
                                                "v_cndmask_b32 %2, %2, %4, vcc\n v_cndmask_b32 %3, %3, %4, vcc\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(k) : "vcc");
    } else if constexpr (KIND == 13) {  // one v_cmp, then 128 e32 cndmasks (counted as 4 blocks)
      const unsigned k = s0 | 1u;
      asm volatile("v_cmp_gt_u32 vcc, %0, %1\n" REP4(REP8("v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n "
                                                          "v_cndmask_b32 %2, %2, %4, vcc\n v_cndmask_b32 %3, %3, %4, vcc\n"))
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(k) : "vcc");
    } else if constexpr (KIND == 14) {  // e32 cndmask reading vcc, with 3 v_add between each (is it the read?)
      const unsigned k = s0 | 1u;
      asm volatile("v_cmp_gt_u32 vcc, %0, %1\n" REP8("v_cndmask_b32 %0, %0, %4, vcc\n v_add_u32 %1, 1, %1\n "
                                                     "v_add_u32 %2, 1, %2\n v_add_u32 %3, 1, %3\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(k) : "vcc");
    } else if constexpr (KIND == 15) {  // the VOP3 (8-byte) encoding of a plain add: encoding or operation?
      asm volatile(REP8("v_add_u32_e64 %0, %0, 1\n v_add_u32_e64 %1, %1, 1\n v_add_u32_e64 %2, %2, 1\n "
                        "v_add_u32_e64 %3, %3, 1\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if constexpr (KIND == 16) {  // VOP2 with the constant in an SGPR (4 bytes) instead of a literal
      const unsigned m = __builtin_amdgcn_readfirstlane(s0 | 0x7fff0000u);
      asm volatile(REP8("v_and_b32 %0, %4, %0\n v_xor_b32 %1, %4, %1\n v_and_b32 %2, %4, %2\n v_xor_b32 %3, %4, %3\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "s"(m));
    } else if constexpr (KIND == 17) {  // pairs of vcc cndmasks between plain adds
      const unsigned k = s0 | 1u;
      asm volatile("v_cmp_gt_u32 vcc, %0, %1\n" REP8("v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n "
                                                     "v_add_u32 %2, 1, %2\n v_add_u32 %3, 1, %3\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(k) : "vcc");
    } else if constexpr (KIND == 18) {  // VOPC in its VOP3 form, into SGPR pairs (no vcc)
      unsigned long long m0, m1, m2, m3;
      asm volatile(REP8("v_cmp_gt_u32_e64 %4, %0, %1\n v_cmp_gt_u32_e64 %5, %1, %2\n v_cmp_gt_u32_e64 %6, %2, %3\n "
                        "v_cmp_gt_u32_e64 %7, %3, %0\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3));
    } else if constexpr (KIND == 19) {  // v_mov_b32 of a literal (8 bytes)
      asm volatile(REP8("v_mov_b32 %0, 0x12345\n v_mov_b32 %1, 0x23456\n v_mov_b32 %2, 0x34567\n v_mov_b32 %3, 0x45678\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if constexpr (KIND == 20) {  // one v_cmp into vcc, then 3 plain adds
      asm volatile(REP8("v_cmp_gt_u32 vcc, %0, %1\n v_add_u32 %1, 1, %1\n v_add_u32 %2, 1, %2\n v_add_u32 %3, 1, %3\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : : "vcc");
    } else if constexpr (KIND == 21) {  // one v_and with a literal, then 3 plain adds
      asm volatile(REP8("v_and_b32 %0, 0x7fffffff, %0\n v_add_u32 %1, 1, %1\n v_add_u32 %2, 1, %2\n v_add_u32 %3, 1, %3\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else if constexpr (KIND == 22) {  // one VOP3 (v_bfe_u32), then 3 plain adds
      asm volatile(REP8("v_bfe_u32 %0, %0, 1, 30\n v_add_u32 %1, 1, %1\n v_add_u32 %2, 1, %2\n v_add_u32 %3, 1, %3\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    } else {  // 24 VALU + 8 SALU per block of 32
      asm volatile(REP8("v_add_u32 %0, 1, %0\n v_add_u32 %1, 1, %1\n v_add_u32 %2, 1, %2\n s_add_u32 %4, %4, 1\n")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+s"(s0) : : "scc");
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0) cycles[w] = t1 - t0;
  sink[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ s0;
}

template <int KIND>
static void run(const char* name, int cus, int waves_per_simd, int iters, bool first, int per_block = 32) {
  const int blocks = cus * waves_per_simd;  // 256 threads = 4 waves = one per SIMD of a CU
  const int waves = blocks * 4;
  unsigned long long* cyc;
  unsigned* sink;
  hipMalloc(&cyc, waves * sizeof(unsigned long long));
  hipMalloc(&sink, blocks * 256 * sizeof(unsigned));
  hipLaunchKernelGGL(k_probe<KIND>, dim3(blocks), dim3(256), 0, 0, 8, cyc, sink);  // warm
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_probe<KIND>, dim3(blocks), dim3(256), 0, 0, iters, cyc, sink);
  hipEventRecord(e1, 0);
  hipDeviceSynchronize();
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(waves);
  hipMemcpy(h.data(), cyc, waves * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  unsigned long long mx = 0, sum = 0;
  for (auto v : h) { mx = v > mx ? v : mx; sum += v; }
  const double per_wave = (double)iters * per_block;
  // per SIMD: waves_per_simd x per_wave instructions in (about) the slowest wave's cycles
  printf("%s{\"kind\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_instr_per_wave\": %.3f, "
         "\"simd_cycles_per_instr\": %.3f, \"simd_instr_per_cycle\": %.3f, \"kernel_ms\": %.3f, "
         "\"clock_ghz_est\": %.3f}\n",
         first ? " " : ",", name, waves_per_simd, (double)sum / waves / per_wave,
         (double)mx / (waves_per_simd * per_wave), waves_per_simd * per_wave / (double)mx, ms,
         (double)mx / (ms * 1e6));
  hipFree(cyc);
  hipFree(sink);
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  printf("{\"cus\": %d, \"runs\": [\n", cus);
  bool first = true;
  const int iters = 20000;
  for (int w : {1, 2, 4, 8}) {
    run<0>("v_add_u32", cus, w, iters, first); first = false;
    run<1>("v_add3_u32", cus, w, iters, first);
    run<2>("v_add_f32", cus, w, iters, first);
    run<3>("v_pk_add_f32", cus, w, iters, first);
    run<4>("v_xor_b32 / v_or_b32", cus, w, iters, first);
    run<5>("v_mov_b32_dpp", cus, w, iters, first);
    run<6>("3 v_add_u32 + 1 s_add_u32", cus, w, iters, first);
    run<7>("v_cndmask_b32 independent", cus, w, iters, first);
    run<8>("v_cndmask_b32_e64 sgpr mask", cus, w, iters, first);
    run<9>("v_cmp_gt_u32 vcc", cus, w, iters, first);
    run<10>("v_and_b32 / v_lshlrev_b32", cus, w, iters, first);
    run<11>("v_bfe_u32", cus, w, iters, first);
    run<12>("v_cndmask_b32 vcc from s_mov", cus, w, iters, first);
    run<13>("v_cndmask_b32 x128 per v_cmp", cus, w, iters / 4, first, 128);
    run<14>("1 v_cndmask_b32 + 3 v_add_u32", cus, w, iters, first);
    run<15>("v_add_u32_e64 (VOP3 encoding)", cus, w, iters, first);
    run<16>("v_and / v_xor with an SGPR constant", cus, w, iters, first);
    run<17>("2 v_cndmask_b32 vcc + 2 v_add_u32", cus, w, iters, first);
    run<18>("v_cmp_gt_u32_e64 into SGPR pairs", cus, w, iters, first);
    run<19>("v_mov_b32 literal", cus, w, iters, first);
    run<20>("1 v_cmp vcc + 3 v_add_u32", cus, w, iters, first);
    run<21>("1 v_and literal + 3 v_add_u32", cus, w, iters, first);
    run<22>("1 v_bfe_u32 + 3 v_add_u32", cus, w, iters, first);
  }
  printf("]}\n");
  return 0;
}
