// Doorbell round trip for a resident stepping kernel (measurement tool, not shipped; VERDICT r02
// item 6).  A persistent kernel on a side stream polls a doorbell word; the step stream rings it
// (hipStreamWriteValue32, or a one-thread kernel) and waits for the kernel's done word
// (hipStreamWaitValue32).  Per case: microseconds per step over 2000 steps.
// Safety: every wave leaves the poll loop after a 2 s deadline of the constant clock (then the
// done word is set to ~0u, so no stream wait can block), and after the last step.
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_floor/doorbell tools/launch_floor/doorbell.hip
// Every runtime call is checked and the program exits before launching anything on a failed
// allocation (signal memory must be allocated 8 bytes exactly: a failed call leaves the pointer
// unset, and a kernel storing through it faults the card).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

constexpr unsigned long long kDeadline = 200000000ull;  // 2 s of the 100 MHz constant clock

__device__ unsigned ld_sys(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// blocks x 256 threads; block b's waves poll, "tick" (one load + store per thread), then the
// block's count goes into counters[0]; the last block of a step publishes done = step.
__global__ void k_resident(const unsigned* bell, unsigned* done, unsigned* count, unsigned* scratch, int steps) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  __shared__ int quit;
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  for (int s = 1; s <= steps; s++) {
    if (threadIdx.x == 0) {
      int q = 0;
      while (ld_sys(bell) < (unsigned)s) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > kDeadline) { q = 1; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      quit = q;
    }
    __syncthreads();
    if (quit) break;
    scratch[i] = scratch[i] + 1u;  // the step's work stand-in
    __syncthreads();
    if (threadIdx.x == 0) {
      __atomic_thread_fence(__ATOMIC_RELEASE);
      const unsigned old = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (old + 1u == (unsigned)s * gridDim.x)
        __hip_atomic_store(done, (unsigned)s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if (threadIdx.x == 0 && quit) __hip_atomic_store(done, ~0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_ring(unsigned* bell, unsigned v) {
  __hip_atomic_store(bell, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static void run(const char* name, int blocks, bool bell_signal, bool kernel_ring, bool last) {
  const int steps = 2000;
  unsigned *bell = nullptr, *done = nullptr, *count = nullptr, *scratch = nullptr;
  if (bell_signal) CHECK(hipExtMallocWithFlags((void**)&bell, 8, hipMallocSignalMemory));
  else CHECK(hipMalloc(&bell, 64));
  CHECK(hipExtMallocWithFlags((void**)&done, 8, hipMallocSignalMemory));
  CHECK(hipMalloc(&count, 64));
  CHECK(hipMalloc(&scratch, blocks * 256 * 4));
  if (!bell || !done || !count || !scratch) { fprintf(stderr, "null allocation\n"); exit(1); }
  CHECK(hipMemset(bell, 0, 4));
  CHECK(hipMemset(done, 0, 4));
  CHECK(hipMemset(count, 0, 4));
  CHECK(hipMemset(scratch, 0, blocks * 256 * 4));
  CHECK(hipDeviceSynchronize());
  hipStream_t side, st;
  CHECK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipLaunchKernelGGL(k_resident, dim3(blocks), dim3(256), 0, side, bell, done, count, scratch, steps);
  CHECK(hipGetLastError());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int warm = 100;
  for (int s = 1; s <= steps; s++) {
    if (s == warm + 1) CHECK(hipEventRecord(e0, st));
    if (kernel_ring) {
      hipLaunchKernelGGL(k_ring, dim3(1), dim3(1), 0, st, bell, (unsigned)s);
      CHECK(hipGetLastError());
    } else {
      CHECK(hipStreamWriteValue32(st, bell, (unsigned)s, 0));
    }
    CHECK(hipStreamWaitValue32(st, done, (unsigned)s, hipStreamWaitValueGte, 0xFFFFFFFFu));
  }
  CHECK(hipEventRecord(e1, st));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  unsigned d = 0;
  CHECK(hipStreamSynchronize(side));
  CHECK(hipMemcpy(&d, done, 4, hipMemcpyDeviceToHost));
  printf(" \"%s\": {\"us_per_step\": %.3f, \"done\": %u}%s\n", name, 1e3 * ms / (steps - warm), d, last ? "" : ",");
  CHECK(hipStreamDestroy(side));
  CHECK(hipStreamDestroy(st));
  CHECK(hipFree(bell));
  CHECK(hipFree(done));
  CHECK(hipFree(count));
  CHECK(hipFree(scratch));
}

int main() {
  int ok = 0;
  CHECK(hipDeviceGetAttribute(&ok, hipDeviceAttributeCanUseStreamWaitValue, 0));
  if (!ok) { printf("{\"can_use_stream_wait_value\": 0}\n"); return 0; }
  printf("{\"can_use_stream_wait_value\": %d, \"cases\": {\n", ok);
  run("write_value_1block", 1, false, false, false);
  run("write_value_signal_bell_1block", 1, true, false, false);
  run("kernel_ring_1block", 1, false, true, false);
  run("write_value_512blocks", 512, false, false, false);
  run("kernel_ring_512blocks", 512, false, true, true);
  printf("}}\n");
  return 0;
}
