// fs_delay.hip -- FootsiesEnv's delayed-frame queue on the GPU (frame_delay > 0).
//
// FootsiesEnv keeps deque(maxlen = frame_delay + 1) of states: reset() clears it and
// appends frame_delay copies of state(-1) (FE:493, 502-504); step() appends the new
// state and pops the oldest, whose observation / info is returned while reward and
// termination come from the new state (FE:532-535, 556-566).  Here every arena has a
// ring of d packed records and a head slot: each of its steps reads the record written d of
// its steps ago from the head slot, writes this step's there and advances the head (arenas
// that fs_step_masked leaves idle keep theirs, like separate FootsiesEnvs).  A row whose frame
// is -1 starts an episode (state(-1) is only emitted by a reset): the ring is refilled
// with d copies and the row is left as is.  In same-step auto-reset a terminal row's
// final_* outputs take the delayed record (the popped state) before the refill.
//
// Record (32 B, two uint4):  x: guard0 | guard1 << 8 | move0 << 16 | move1 << 24
//                            y: action0 | action1 << 8 | hitstun0 << 16 | hitstun1 << 24
//                            z: frame                      w: 0
//                            second: move_frame0, move_frame1, position0, position1 (bits)
#include <hip/hip_runtime.h>

#include "fs_internal.h"

namespace fsk {

namespace {

struct Rec {
  uint4 a, b;
};

__device__ __forceinline__ Rec gather(const DevOutputs& o, uint32_t r, bool final_set) {
  const uint8_t* g = final_set ? o.final_guard : o.guard;
  const uint8_t* m = final_set ? o.final_move : o.move;
  const uint8_t* ac = final_set ? o.final_action : o.action;
  const uint8_t* hs = final_set ? o.final_hitstun : o.hitstun;
  const float* mf = final_set ? o.final_move_frame : o.move_frame;
  const float* ps = final_set ? o.final_position : o.position;
  const int32_t* fr = final_set ? o.final_frame : o.frame;
  const uint32_t c = 2 * r;
  Rec R;
  R.a.x = g[c] | (g[c + 1] << 8) | (m[c] << 16) | ((uint32_t)m[c + 1] << 24);
  R.a.y = ac[c] | (ac[c + 1] << 8) | (hs[c] << 16) | ((uint32_t)hs[c + 1] << 24);
  R.a.z = (uint32_t)fr[r];
  R.a.w = 0;
  R.b = make_uint4(__float_as_uint(mf[c]), __float_as_uint(mf[c + 1]), __float_as_uint(ps[c]),
                   __float_as_uint(ps[c + 1]));
  return R;
}

__device__ __forceinline__ void scatter(const DevOutputs& o, uint32_t r, const Rec& R, bool final_set) {
  uint8_t* g = final_set ? o.final_guard : o.guard;
  uint8_t* m = final_set ? o.final_move : o.move;
  uint8_t* ac = final_set ? o.final_action : o.action;
  uint8_t* hs = final_set ? o.final_hitstun : o.hitstun;
  float* mf = final_set ? o.final_move_frame : o.move_frame;
  float* ps = final_set ? o.final_position : o.position;
  int32_t* fr = final_set ? o.final_frame : o.frame;
  const uint32_t c = 2 * r;
  g[c] = (uint8_t)R.a.x;
  g[c + 1] = (uint8_t)(R.a.x >> 8);
  m[c] = (uint8_t)(R.a.x >> 16);
  m[c + 1] = (uint8_t)(R.a.x >> 24);
  ac[c] = (uint8_t)R.a.y;
  ac[c + 1] = (uint8_t)(R.a.y >> 8);
  hs[c] = (uint8_t)(R.a.y >> 16);
  hs[c + 1] = (uint8_t)(R.a.y >> 24);
  fr[r] = (int32_t)R.a.z;
  mf[c] = __uint_as_float(R.b.x);
  mf[c + 1] = __uint_as_float(R.b.y);
  ps[c] = __uint_as_float(R.b.z);
  ps[c + 1] = __uint_as_float(R.b.w);
}

__global__ __launch_bounds__(256) void k_delay(DelayParams p) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= p.n_envs) return;
  const uint32_t N = (uint32_t)p.n_envs;
  const uint32_t row_step = (uint32_t)p.out_stride_steps * N;
  if (p.active && !p.active[a]) return;  // an idle arena: no row, no shift
  auto slot_ptr = [&](uint32_t slot) { return p.ring + 2 * ((size_t)slot * N + (uint32_t)a); };
  uint32_t slot = p.head[a];
  for (int t = 0; t < p.n_steps; t++) {
    const uint32_t r = (uint32_t)t * row_step + (uint32_t)a;
    const Rec cur = gather(p.out, r, false);
    if ((int32_t)cur.a.z == -1) {  // state(-1): the reset refills the queue
      if (!p.refill_only && p.same_step && p.out.terminated[r]) {
        const uint4* q = slot_ptr(slot);
        scatter(p.out, r, Rec{q[0], q[1]}, true);
      }
      for (int j = 0; j < p.delay; j++) {
        uint4* q = slot_ptr((uint32_t)j);
        q[0] = cur.a;
        q[1] = cur.b;
      }
    } else if (!p.refill_only) {
      uint4* q = slot_ptr(slot);
      const Rec old{q[0], q[1]};
      q[0] = cur.a;
      q[1] = cur.b;
      scatter(p.out, r, old, false);
    }
    slot = slot + 1 == (uint32_t)p.delay ? 0u : slot + 1;  // (a refill leaves every slot equal)
  }
  if (!p.refill_only) p.head[a] = (uint8_t)slot;
}

}  // namespace

hipError_t launch_delay(const DelayParams& p, hipStream_t s) {
  if (p.delay <= 0 || p.n_envs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_delay, dim3((unsigned)((p.n_envs + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace fsk
