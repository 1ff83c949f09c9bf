// fs_gather.hip -- one packed 40-byte record per arena from the step outputs
// (fs_pack_outputs), the payload of the multi-GPU per-step gather of (obs, reward,
// done) over RCCL (footsies_gym_amd/parallel.py holds the layout):
//   [0,2) guard  [2,4) move  [4,6) action  [6,8) hitstun  [8] terminated  [9] truncated
//   [10,12) pad  [12,20) move_frame f32 x2  [20,28) position f32 x2  [28,32) frame i32
//   [32,40) reward f64
// One thread per arena: pair fields read as one u16 / two-float load, the record written
// as five 8-byte stores (a warp's records are one contiguous 2.5 KB span).
#include <hip/hip_runtime.h>

#include "fs_internal.h"

namespace fsk {

__global__ __launch_bounds__(256) void k_pack_records(DevOutputs o, uint2* dst, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t guard = reinterpret_cast<const uint16_t*>(o.guard)[i];
  const uint32_t move = reinterpret_cast<const uint16_t*>(o.move)[i];
  const uint32_t action = reinterpret_cast<const uint16_t*>(o.action)[i];
  const uint32_t hitstun = reinterpret_cast<const uint16_t*>(o.hitstun)[i];
  const uint2 mf = reinterpret_cast<const uint2*>(o.move_frame)[i];
  const uint2 pos = reinterpret_cast<const uint2*>(o.position)[i];
  const uint32_t flags = (uint32_t)o.terminated[i] | ((uint32_t)o.truncated[i] << 8);
  const uint32_t frame = (uint32_t)o.frame[i];
  const uint64_t rw = __double_as_longlong(o.reward[i]);
  uint2* r = dst + (size_t)i * 5;
  r[0] = make_uint2(guard | (move << 16), action | (hitstun << 16));
  r[1] = make_uint2(flags, mf.x);
  r[2] = make_uint2(mf.y, pos.x);
  r[3] = make_uint2(pos.y, frame);
  r[4] = make_uint2((uint32_t)rw, (uint32_t)(rw >> 32));
}

hipError_t launch_pack_records(const DevOutputs& o, void* dst, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_pack_records, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, o,
                     reinterpret_cast<uint2*>(dst), n);
  return hipGetLastError();
}

}  // namespace fsk
