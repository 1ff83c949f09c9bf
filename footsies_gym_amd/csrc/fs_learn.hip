// fs_learn.hip -- the C5 learner's minibatch gradient (fs_ppo_grad): PPO's clipped-surrogate,
// value and entropy loss of the actor 8-64-64-8 and the critic 8-64-64-1 (tanh MLPs, the
// shapes of footsies_gym_amd/rollout.py make_actor / ppo.py make_critic), forward and backward
// fused into one kernel per network, fp32 throughout.  The torch learner of ppo.py defines the
// values (its loss and autograd's gradients); tests/test_gpu_learn.py compares the two.
//
// One wave per block, 32 samples per tile (kTile), a grid-stride loop over tiles.  Every GEMM runs
// on fp32 MFMA with the tile's activations as rows of an LDS stage (h1, then g1; h2, then g2):
//  1 h1 = tanh(W1 x + b1) and 2 h2 = tanh(W2 h1 + b2) (32 x 32 x 2, hidden units on the rows);
//  3 the actor's logits W3 h2 + b3 (16 x 16 x 4, 8 of 16 rows used) exchanged between lane halves,
//    then (lane = sample) the loss and its gradient g3 (staged); the critic's value on VALU;
//  4 (lane = unit j) dW3[.][j] += g3[s] h2[s][j];
//  5 g2 = (W3^T g3)(1 - h2^2) (actor: 32 x 32 x 2, K = 8) over h2 in place;
//  6 dW2 += G2^T H1 and 7 g1 = (W2^T g2)(1 - h1^2) over h1 in place, W2^T read as rows from a copy
//    k_ppo_t64 writes per call; 8 (lane = unit i) dW1 and db1.
// The gradients accumulate in registers across tiles.  On gfx950 a SIMD does not issue VALU
// while an MFMA executes, not even another wave's (tools/mfma_probe/overlap.hip), so the tile
// time is the sum of the MFMA time (64 cycles per 32x32x2, tools/mfma_probe/rate.hip) and the
// VALU time, not their max.
// Each wave writes its partial gradient to the workspace; k_ppo_reduce sums the partials in a
// fixed order, so the result does not depend on scheduling.  Nothing here is integer game
// state: this is the learner beside the simulator, not part of the bit-exact path.
#include <hip/hip_runtime.h>

#include "fs_internal.h"

namespace fsl {

constexpr int kF = 8;          // features
constexpr int kH = 64;         // hidden units
constexpr int kRow = 12;       // rows: x[8], action, old log-prob, advantage, return
constexpr int kPad = kH + 4;   // LDS row stride of the h1 / h2 stages (b128 writes spread over banks)
// 32 samples per tile: a 19 KB stage, so two waves per SIMD fit the LDS; the MFMA maps (32 x 32
// results, the output layer's two 16-column blocks) are written for it
constexpr int kTile = 32;        // (lanes >= kTile idle in the per-sample phases)
constexpr int kMaxWaves = 2048;  // grid cap: two waves per SIMD
constexpr int kMaxEvalWaves = 4096;  // the forward pass alone: four (fewer registers, ~10 KB of LDS)

template <int OUT>
constexpr int n_params() { return kH * kF + kH + kH * kH + kH + OUT * kH + OUT; }
template <int OUT>
constexpr int partial_stride() { return (n_params<OUT>() + 3 + 31) & ~31; }  // + pg / vf / ent sums; 128-B rows

// parameter offsets in torch's parameters() order: w1, b1, w2, b2, w3, b3
constexpr int kOffB1 = kH * kF, kOffW2 = kOffB1 + kH, kOffB2 = kOffW2 + kH * kH, kOffW3 = kOffB2 + kH;
template <int OUT>
constexpr int off_b3() { return kOffW3 + OUT * kH; }

using CPtr = const __attribute__((address_space(4))) float*;  // scalar (constant) loads
// Weight pointers made opaque per tile (below) lose their address space; as generic pointers their
// loads become flat loads with a 64-bit address add each (flat loads also wait on both counters).
// Cast back to global memory they load with an SGPR base and a 32-bit lane offset.
using GPtr = const __attribute__((address_space(1))) float*;
typedef float F4v __attribute__((ext_vector_type(4)));  // (a native vector: copies from any address space)
using GPtr4 = const __attribute__((address_space(1))) F4v*;
// (an unsigned 32-bit element index: the load can take it as its VGPR offset beside the SGPR base)
__device__ __forceinline__ float4 ld4(GPtr p, uint32_t i) {
  const F4v v = *(GPtr4)(p + i);
  return make_float4(v.x, v.y, v.z, v.w);
}

struct Coef {
  float clip, vf_coef, ent_coef, inv_n;
};

__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

typedef float F16 __attribute__((ext_vector_type(16)));  // a 32 x 32 f32 MFMA accumulator
__device__ __forceinline__ F16 mfma32(float a, float b, F16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
typedef float F4 __attribute__((ext_vector_type(4)));  // a 16 x 16 f32 MFMA accumulator
__device__ __forceinline__ F4 mfma16(float a, float b, F4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// Split-bf16 products (the opt-in FS_PPO_SPLIT_BF16 precision): each fp32 operand x of the three
// 64-wide GEMMs is the pair hi = bf16(x), lo = bf16(x - hi) (x - hi is exact in fp32, so hi + lo
// keeps 16 significant bits), and a product is hi.hi + hi.lo + lo.hi on
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation: lo.lo and the rounding of lo are below
// 2^-15 of the product.  One 32x32x16 bf16 MFMA holds the pipe 32 cycles against the fp32
// 32x32x2's 64, for 8x the K, so a K = 64 block costs 12 instead of 32 MFMAs of pipe time 384
// instead of 2048 cycles.  Operand map (fs_policy.h, checked on the GPU by tools/mfma_probe):
// lane l, r = l & 31, h = l >> 5 holds A[row r][k = 8h + j] and B[k = 8h + j][col r] in element j;
// the 32 x 32 accumulator is laid out as the fp32 32x32x2's (col r, row (q & 3) + 8 (q >> 2) + 4h).
typedef __bf16 BF8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ F16 mfma_bf16(BF8 a, BF8 b, F16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// (as pairs: one v_cvt_pk_bf16_f32 rounds two values and one the two remainders; the library is
// built without SLP vectorization, so the pairs are spelled out)
typedef float F2 __attribute__((ext_vector_type(2)));
typedef __bf16 BF2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split8(const float (&x)[8], BF8& hi, BF8& lo) {
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const F2 v = {x[j], x[j + 1]};
    const BF2 h = __builtin_convertvector(v, BF2);
    const F2 hf = __builtin_convertvector(h, F2);
    // the remainders as two plain subtractions: a v_pk_add_f32 wants its operands in an aligned
    // register pair, which values read from the stages' columns are not (two moves per pair)
    const F2 r = {__fsub_rn(x[j], hf[0]), __fsub_rn(x[j + 1], hf[1])};
    const BF2 l = __builtin_convertvector(r, BF2);
    hi[j] = h[0];
    hi[j + 1] = h[1];
    lo[j] = l[0];
    lo[j + 1] = l[1];
  }
}
// the three products of one K = 16 step, the small ones first
__device__ __forceinline__ F16 mfma_split(BF8 ah, BF8 al, BF8 bh, BF8 bl, F16 c) {
  c = mfma_bf16(ah, bl, c);
  c = mfma_bf16(al, bh, c);
  return mfma_bf16(ah, bh, c);
}
// The same on v_mfma_f32_16x16x32_bf16 (K = 32 in one step): lane l holds A[row l & 15][k = 8 (l >> 4)
// + j] and B[k = 8 (l >> 4) + j][col l & 15] in element j; the 16 x 16 accumulator D[row 4 (l >> 4) +
// i][col l & 15] in its element i.
__device__ __forceinline__ F4 mfma16_split(BF8 ah, BF8 al, BF8 bh, BF8 bl, F4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}
// The weight fragments of the two 64-wide GEMMs with W2 as the A operand, built once per call by
// k_ppo_frag: [mat: 0 = W2, 1 = W2^T][row block][k step][0 = hi, 1 = lo][lane] of 8 bf16 (16 B).
constexpr int kFragsPerNet = 2 * 2 * 4 * 2 * 64;
constexpr int kScaledPerNet = kH * kF + 2 * kH;  // 2 log2 e x (W1, b1, b2) for the split kernels
__device__ __forceinline__ uint32_t frag_at(int mat, int blk, int s, int part, int lane) {  // (unsigned: see ld4)
  return (uint32_t)((((mat * 2 + blk) * 4 + s) * 2 + part) * 64 + lane);
}
// one fragment, loaded through a global-memory pointer
__device__ __forceinline__ BF8 ldfrag(const uint4* frags, uint32_t i) {
  typedef uint32_t U4v __attribute__((ext_vector_type(4)));
  using G4 = const __attribute__((address_space(1))) U4v*;
  return __builtin_bit_cast(BF8, ((G4)frags)[i]);
}

// tanh without branches (the library tanhf runs both of its branches under divergence, ~30
// instructions): |x| < 0.625 the same odd polynomial, above it 1 - 2 / (2^(2|x| log2 e) + 1)
// with the hardware exp2 and reciprocal (within a few ulp of tanhf; 2^+inf -> 1 exactly).
__device__ __forceinline__ float tanh_fast(float x) {
  const float ax = fabsf(x);
  const float e = __builtin_amdgcn_exp2f(ax * 2.8853900817779268f);
  const float big = fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
  const float x2 = x * x;
  float p = fmaf(-0.005700020585209131f, x2, 0.02063407190144062f);  // 0xbbbac73d, 0x3ca908c9
  p = fmaf(x2, p, -0.053737930953502655f);                            // 0xbd5c1c4e
  p = fmaf(x2, p, 0.13331416249275208f);                              // 0x3e088382
  p = fmaf(x2, p, -0.3333328068256378f);                              // 0xbeaaaa99
  const float small = fmaf(x2, ax * p, ax);
  return copysignf(ax < 0.625f ? small : big, x);
}

// The split-bf16 precision's transcendentals: the hardware exp2 and reciprocal alone, without
// tanh_fast's small-|x| polynomial and select or expf's range reduction.  tanh as
// 1 - 2 / (2^(2 x log2 e) + 1) is within 2.5e-7 of tanh absolutely (the cancellation near 0 costs
// relative accuracy, not absolute: far below the bf16 split's 2^-17 per product), exp within a
// few ulp.  The fp32 precision keeps tanh_fast / expf.
__device__ __forceinline__ float tanh_hw(float x) {
  return fmaf(-2.f, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(x * 2.8853900817779268f) + 1.f), 1.f);
}
template <bool HW>
__device__ __forceinline__ float tanh_of(float x) {
  if constexpr (HW) return tanh_hw(x);
  else return tanh_fast(x);
}
// The split-bf16 kernels' hidden layers run on weights and biases pre-scaled by 2 log2 e (W1, b1,
// b2 and W2's layer-2 fragments, written once per call by k_ppo_frag): their pre-activations y are
// already tanh_hw's exp2 argument, so each tanh is exp2, add, reciprocal and fma, one multiply
// fewer (64 per lane and tile).
constexpr float kTanhScale = 2.8853900817779268f;  // 2 log2 e
__device__ __forceinline__ float tanh_prescaled(float y) {
  return fmaf(-2.f, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(y) + 1.f), 1.f);
}
template <bool HW>
__device__ __forceinline__ float tanh_layer(float v) {  // a hidden layer's tanh (HW: of a pre-scaled value)
  if constexpr (HW) return tanh_prescaled(v);
  else return tanh_fast(v);
}
template <bool HW>
__device__ __forceinline__ float exp_of(float x) {
  if constexpr (HW) return __builtin_amdgcn_exp2f(x * 1.4426950408889634f);
  else return expf(x);
}

// PPO's actor loss of one sample (ppo.py update) from its logits z: log_softmax, the clipped
// surrogate and the entropy bonus; g3 = d loss / d z (zero for padding rows, !valid).
template <bool HW>
__device__ __forceinline__ void actor_loss(const float (&z)[8], const float (&tail)[4], bool valid, const Coef& c,
                                           float (&g3)[8], float& pg_sum, float& ent_sum) {
  float m = z[0];
#pragma unroll
  for (int o = 1; o < 8; ++o) m = fmaxf(m, z[o]);
  float se = 0.f;
#pragma unroll
  for (int o = 0; o < 8; ++o) se += exp_of<HW>(z[o] - m);
  const float lse = m + logf(se);
  float lp[8], p[8];
  const int act = (int)tail[0];
  float lp_a = 0.f, ent = 0.f;
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    lp[o] = z[o] - lse;
    p[o] = exp_of<HW>(lp[o]);
    lp_a = o == act ? lp[o] : lp_a;
    ent -= p[o] * lp[o];
  }
  const float adv = tail[2];
  const float rt = exp_of<HW>(lp_a - tail[1]);
  const float s1 = rt * adv, rc = fminf(fmaxf(rt, 1.f - c.clip), 1.f + c.clip), s2 = rc * adv;
  // torch.min's gradient goes to the smaller operand (half to each on a tie); clamp's passes
  // inside [1 - clip, 1 + clip]
  const float inr = (rt >= 1.f - c.clip && rt <= 1.f + c.clip) ? 1.f : 0.f;
  const float wsel = s1 < s2 ? 1.f : (s1 > s2 ? inr : 0.5f + 0.5f * inr);
  const float g_lpa = -(adv * wsel) * c.inv_n * rt;
  const float g_ent = c.ent_coef * c.inv_n;  // d(-ent_coef mean H) / d(exp(lp) lp) per term
  float g_lp[8], gsum = 0.f;
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    g_lp[o] = (o == act ? g_lpa : 0.f) + g_ent * (p[o] * lp[o] + p[o]);
    gsum += g_lp[o];
  }
#pragma unroll
  for (int o = 0; o < 8; ++o) g3[o] = valid ? g_lp[o] - p[o] * gsum : 0.f;  // log_softmax backward
  pg_sum += valid ? -fminf(s1, s2) : 0.f;
  ent_sum += valid ? ent : 0.f;
}

// Accumulator element q of lane (r, hf) is row (q & 3) + 8 (q >> 2) + 4 hf, column r: four runs
// of four consecutive rows.  bias_frag: the accumulator holding b[row] in every column;
// store_rows(_tanh): (tanh of) column r's 16 values into the LDS row `dst` (= stage[r] + 32 block).
__device__ __forceinline__ F16 bias_frag(GPtr b, int hf) {
  F16 v;
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) {
    const float4 x = ld4(b, (uint32_t)(8 * qq + 4 * hf));
    v[4 * qq] = x.x; v[4 * qq + 1] = x.y; v[4 * qq + 2] = x.z; v[4 * qq + 3] = x.w;
  }
  return v;
}
__device__ __forceinline__ void store_rows(float* dst, const F16& v, int hf) {
#pragma unroll
  for (int qq = 0; qq < 4; ++qq)
    *reinterpret_cast<float4*>(dst + 8 * qq + 4 * hf) = make_float4(v[4 * qq], v[4 * qq + 1], v[4 * qq + 2], v[4 * qq + 3]);
}
template <bool HW>
__device__ __forceinline__ void store_rows_tanh(float* dst, const F16& v, int hf) {
#pragma unroll
  for (int qq = 0; qq < 4; ++qq)
    *reinterpret_cast<float4*>(dst + 8 * qq + 4 * hf) = make_float4(tanh_layer<HW>(v[4 * qq]), tanh_layer<HW>(v[4 * qq + 1]),
                                                                    tanh_layer<HW>(v[4 * qq + 2]), tanh_layer<HW>(v[4 * qq + 3]));
}

#ifndef FSL_WAVES
#define FSL_WAVES 2  // and their registers (256 per lane)
#endif
#if FSL_WAVES > 0
#define FSL_OCC __attribute__((amdgpu_waves_per_eu(FSL_WAVES)))
#else
#define FSL_OCC
#endif

// EVAL: the forward pass only (fs_ppo_eval), rows = x [n][8]; the critic writes v per row into
// out, the actor log_softmax(logits)[actions[row]].  Otherwise the gradient, rows [n][12].
template <int OUT, bool EVAL = false, bool SPLIT = false>
__global__ __launch_bounds__(64) FSL_OCC void k_ppo_grad(const float* __restrict__ rows, int64_t n, int64_t tiles,
                                                         const float* __restrict__ w1, const float* __restrict__ b1,
                                                         const float* __restrict__ w2, const float* __restrict__ b2,
                                                         const float* __restrict__ w3, const float* __restrict__ b3,
                                                         Coef c, float* __restrict__ partial,
                                                         const uint8_t* __restrict__ actions = nullptr,
                                                         const float* __restrict__ w2t = nullptr,
                                                         const uint4* __restrict__ frags = nullptr,
                                                         const int64_t* __restrict__ runs = nullptr, int run_shift = 0,
                                                         int64_t n_rows = 0) {
  constexpr int kStride = EVAL ? kF : kRow;
  __shared__ float sX[kTile][kF];
  __shared__ float sH1[kTile][kPad];  // rows: h1 of each sample, then g1
  // (the forward pass alone keeps h2 in h1's stage -- layer 2 reads all of h1 into registers before
  // it writes -- so its blocks need ~10 KB of LDS and four of them fit per SIMD)
  __shared__ float sH2[EVAL ? 1 : kTile][kPad];  // rows: h2, then g2
  __shared__ float sG3[EVAL ? 1 : kTile][8];
  float (*const H2)[kPad] = EVAL ? sH1 : sH2;

  const int lane = threadIdx.x, r = lane & 31, hf = lane >> 5;
  F16 dW2[2][2];  // dW2 as four 32 x 32 MFMA accumulators [i block][k block]
  float dW1[kF], dW3[OUT], dB3[OUT], dB2[2] = {0.f, 0.f};
  float dB1 = 0.f, pg_sum = 0.f, vf_sum = 0.f, ent_sum = 0.f;
  // (split: dW3 and dW1 on 16 x 16 x 32 MFMAs into one set of accumulators, block b = units 16 b ..
  // 16 b + 15 on the rows: columns 0-7 dW3[o][unit] (o < OUT), columns 8-15 dW1[unit][f]; db1 as
  // per-lane partial sums over its 8 samples of each block, added across the lanes at the end)
  F4 dWo[4];
  float dB1p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < 4; ++b) dWo[b] = F4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 16; ++q) dW2[0][0][q] = dW2[0][1][q] = dW2[1][0][q] = dW2[1][1][q] = 0.f;
#pragma unroll
  for (int f = 0; f < kF; ++f) dW1[f] = 0.f;
#pragma unroll
  for (int o = 0; o < OUT; ++o) dW3[o] = dB3[o] = 0.f;

  // (runs: sample i of the minibatch is row runs[i >> run_shift] * 2^run_shift + i mod 2^run_shift of
  // the table, fs_ppo_grad_runs; each lane's run entry is read one tile ahead)
  auto run_of = [&](int64_t t) -> int64_t {
    const int64_t i = t * kTile + lane;
    return (runs && lane < kTile && t < tiles && i < n) ? runs[i >> run_shift] : 0;
  };
  int64_t run_next = run_of(blockIdx.x);
  for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int64_t run_cur = run_next;
    run_next = run_of(tile + gridDim.x);
    // weights re-read every tile (L1 / scalar-cache hits): hoisted out of the loop they would
    // hold ~200 registers; W3 / B3 as wave-uniform scalar loads (constant address space)
    const float *w1v = w1, *b1v = b1, *w2v = w2, *b2v = b2, *w3v = w3, *b3v = b3, *w2tv = w2t;
    asm volatile("" : "+s"(w1v), "+s"(b1v), "+s"(w2v), "+s"(b2v), "+s"(w3v), "+s"(b3v), "+s"(w2tv));
    const CPtr W3 = (CPtr)w3v, B3 = (CPtr)b3v;
    const GPtr w1g = (GPtr)w1v, b1g = (GPtr)b1v, w2g = (GPtr)w2v, b2g = (GPtr)b2v, w3g = (GPtr)w3v, b3g = (GPtr)b3v,
               w2tg = (GPtr)w2tv;
    const int64_t left = n - tile * kTile;
    const int ns = (int)(left < kTile ? left : kTile);
    int64_t row = tile * kTile + lane;
    bool in_table = true;
    if (runs) {  // (a run entry outside the table reads nothing and adds nothing, as a padding row)
      // the run index is bounded before it is shifted: a huge entry (>= 2^(63 - run_shift))
      // would otherwise wrap back into [0, n_rows) and read real rows
      const int64_t mask = ((int64_t)1 << run_shift) - 1;
      in_table = run_cur >= 0 && run_cur <= ((n_rows - 1) >> run_shift);
      row = in_table ? ((run_cur << run_shift) | (row & mask)) : 0;
      in_table = in_table && row < n_rows;
    }
    const bool valid = lane < ns && in_table;  // rows past n: x = 0 and g3 = 0, so they add nothing

    // ---- rows -> x (LDS) and the loss inputs (registers of lanes < kTile) --------------------
    float tail[4] = {0.f, 0.f, 0.f, 0.f};
    if (lane < kTile) {
      const float4* rp = reinterpret_cast<const float4*>(rows + (valid ? row : 0) * kStride);
      float4 r0 = rp[0], r1 = rp[1];
      if constexpr (!EVAL) {
        const float4 r2 = rp[2];
        tail[0] = r2.x; tail[1] = r2.y; tail[2] = r2.z; tail[3] = r2.w;
      }
      if (!valid) r0 = r1 = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(&sX[lane][0]) = r0;
      *reinterpret_cast<float4*>(&sX[lane][4]) = r1;
    }
    __syncthreads();

    // ---- layer 1 on MFMA: H1^T[j][s] = b1[j] + sum_f W1[j][f] X[s][f]; K = 8 as 4 steps of
    // (f = t, t + 4): lane (r, hf) supplies A = W1[32 jb + r][t + 4 hf], B = X[r][t + 4 hf] ----
    // (split: the tanh'd accumulators are also layer 2's B operand, straight from registers: k step
    // 2 jb + u takes registers 8 u .. 8 u + 7 of block jb, units 32 jb + 16 u + 8 (j >> 2) + 4 hf +
    // (j & 3) -- the k order k_ppo_frag gives W2's fragments -- so layer 2 does not wait for h1's
    // trip through LDS; the stage is still written for the backward pass, not for the forward
    // pass alone)
    BF8 bh[4], bl[4];
    {
      const float4 xb = *reinterpret_cast<const float4*>(&sX[r][4 * hf]);
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        const float4 wa = ld4(w1g, (uint32_t)((32 * jb + r) * kF + 4 * hf));
        F16 acc = bias_frag(b1g + 32 * jb, hf);
        acc = mfma32(wa.x, xb.x, acc);
        acc = mfma32(wa.y, xb.y, acc);
        acc = mfma32(wa.z, xb.z, acc);
        acc = mfma32(wa.w, xb.w, acc);
        if constexpr (SPLIT) {
#pragma unroll
          for (int q = 0; q < 16; ++q) acc[q] = tanh_layer<SPLIT>(acc[q]);
          if constexpr (!EVAL) store_rows(&sH1[r][32 * jb], acc, hf);  // (the forward pass alone needs no h1 stage)
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const float v[8] = {acc[8 * u], acc[8 * u + 1], acc[8 * u + 2], acc[8 * u + 3],
                                acc[8 * u + 4], acc[8 * u + 5], acc[8 * u + 6], acc[8 * u + 7]};
            split8(v, bh[2 * jb + u], bl[2 * jb + u]);
          }
        } else {
          store_rows_tanh<SPLIT>(&sH1[r][32 * jb], acc, hf);
        }
      }
    }
    if constexpr (!SPLIT) __syncthreads();

    // ---- layer 2 on MFMA: H2^T[j][s] = b2[j] + sum_k W2[j][k] H1[s][k]; K = 64 as 32 steps of
    // (k = t, t + 32): A = W2[32 jb + r][t + 32 hf] (row loads), B = H1[r][t + 32 hf] (LDS row) ----
    if constexpr (SPLIT) {  // K = 64 as 4 bf16 steps, B from layer 1's registers (above)
#pragma unroll 1
      for (int jb = 0; jb < 2; ++jb) {  // (one block's fragments live at a time)
        F16 acc = bias_frag(b2g + 32 * jb, hf);
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          const BF8 ah = ldfrag(frags, frag_at(0, jb, st, 0, lane));
          const BF8 al = ldfrag(frags, frag_at(0, jb, st, 1, lane));
          acc = mfma_split(ah, al, bh[st], bl[st], acc);
        }
        store_rows_tanh<SPLIT>(&H2[r][32 * jb], acc, hf);
      }
    } else {
      float hb[32];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float4 v = *reinterpret_cast<const float4*>(&sH1[r][32 * hf + 4 * u]);
        hb[4 * u] = v.x; hb[4 * u + 1] = v.y; hb[4 * u + 2] = v.z; hb[4 * u + 3] = v.w;
      }
#pragma unroll 1
      for (int jb = 0; jb < 2; ++jb) {  // (one block's weights live at a time)
        float wa[32];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float4 v = ld4(w2g, (uint32_t)((32 * jb + r) * kH + 32 * hf + 4 * u));
          wa[4 * u] = v.x; wa[4 * u + 1] = v.y; wa[4 * u + 2] = v.z; wa[4 * u + 3] = v.w;
        }
        F16 acc = bias_frag(b2g + 32 * jb, hf);
#pragma unroll
        for (int t = 0; t < 32; ++t) acc = mfma32(wa[t], hb[t], acc);
        store_rows_tanh<SPLIT>(&H2[r][32 * jb], acc, hf);
      }
    }
    __syncthreads();

    if constexpr (EVAL) {  // (lane = sample) the output only
      if (valid) {
        float hv[kH];
#pragma unroll
        for (int k = 0; k < kH; k += 4) {
          const float4 v = *reinterpret_cast<const float4*>(&H2[lane][k]);
          hv[k] = v.x; hv[k + 1] = v.y; hv[k + 2] = v.z; hv[k + 3] = v.w;
        }
        const int64_t srow = tile * kTile + lane;
        if constexpr (OUT == 8) {
          float z[8];
#pragma unroll
          for (int o = 0; o < 8; ++o) {
            float a = B3[o];
#pragma unroll
            for (int j = 0; j < kH; ++j) a = fmaf(W3[o * kH + j], hv[j], a);
            z[o] = a;
          }
          float m = z[0];
#pragma unroll
          for (int o = 1; o < 8; ++o) m = fmaxf(m, z[o]);
          float se = 0.f;
#pragma unroll
          for (int o = 0; o < 8; ++o) se += exp_of<SPLIT>(z[o] - m);
          const int act = actions[srow];
          float za = z[0];
#pragma unroll
          for (int o = 1; o < 8; ++o) za = o == act ? z[o] : za;
          partial[srow] = za - (m + logf(se));
        } else {
          float v = B3[0];
#pragma unroll
          for (int j = 0; j < kH; ++j) v = fmaf(W3[j], hv[j], v);
          partial[srow] = v;
        }
      }
      __syncthreads();
      continue;
    }

    // ---- the output layer and the loss gradient g3 (staged in sG3) ---------------------------
    if constexpr (OUT == 8) {
      // Z^T[o][s] = b3[o] + W3[o] . h2[s] on MFMA 16 x 16 x 4: rows o (8 of 16 used), columns the
      // 16 samples of block nb, K = 64 as 16 steps of k = 16 q + t; lane (c, q) = (lane & 15,
      // lane >> 4) supplies A = W3[c][16 q + t] and B = H2[16 nb + c][16 q + t] and holds rows
      // 4 q .. 4 q + 3 of column c.
      const int c16 = lane & 15, q4 = lane >> 4;
      float wz[16];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 v = c16 < 8 ? ld4(w3g, (uint32_t)(c16 * kH + 16 * q4 + 4 * u))
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
        wz[4 * u] = v.x; wz[4 * u + 1] = v.y; wz[4 * u + 2] = v.z; wz[4 * u + 3] = v.w;
      }
      const float4 bz = q4 < 2 ? ld4(b3g, (uint32_t)(4 * q4)) : make_float4(0.f, 0.f, 0.f, 0.f);
      F4 zacc[2];
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        float hz[16];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float4 v = *reinterpret_cast<const float4*>(&H2[16 * nb + c16][16 * q4 + 4 * u]);
          hz[4 * u] = v.x; hz[4 * u + 1] = v.y; hz[4 * u + 2] = v.z; hz[4 * u + 3] = v.w;
        }
        F4 acc = {bz.x, bz.y, bz.z, bz.w};
#pragma unroll
        for (int t = 0; t < 16; ++t) acc = mfma16(wz[t], hz[t], acc);
        zacc[nb] = acc;
      }
      // lane s < 32 (block nb = s >> 4 = q) holds z[s][4 nb ..]; lane s ^ 16 holds z[s][4 (1 - nb) ..]
      const F4 own = q4 & 1 ? zacc[1] : zacc[0], snd = q4 & 1 ? zacc[0] : zacc[1];
      F4 rcv;
#pragma unroll
      for (int v = 0; v < 4; ++v) rcv[v] = __shfl_xor(snd[v], 16, 64);
      if (lane < kTile) {
        float z[8], g3[8];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          z[v] = q4 ? rcv[v] : own[v];
          z[4 + v] = q4 ? own[v] : rcv[v];
        }
        actor_loss<SPLIT>(z, tail, valid, c, g3, pg_sum, ent_sum);
#pragma unroll
        for (int o = 0; o < 8; ++o) dB3[o] += g3[o];
        *reinterpret_cast<float4*>(&sG3[lane][0]) = make_float4(g3[0], g3[1], g3[2], g3[3]);
        *reinterpret_cast<float4*>(&sG3[lane][4]) = make_float4(g3[4], g3[5], g3[6], g3[7]);
      }
    } else if (lane < kTile) {  // the critic (lane = sample): v = W3 . h2 + b3, the value loss
      float h2[kH];
#pragma unroll
      for (int k = 0; k < kH; k += 4) {
        const float4 v = *reinterpret_cast<const float4*>(&H2[lane][k]);
        h2[k] = v.x; h2[k + 1] = v.y; h2[k + 2] = v.z; h2[k + 3] = v.w;
      }
      float v = B3[0];
#pragma unroll
      for (int j = 0; j < kH; ++j) v = fmaf(W3[j], h2[j], v);
      const float d = v - tail[3];
      const float g3 = valid ? 2.f * d * (c.vf_coef * c.inv_n) : 0.f;
      vf_sum += valid ? d * d : 0.f;
      dB3[0] += g3;
      *reinterpret_cast<float4*>(&sG3[lane][0]) = make_float4(g3, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(&sG3[lane][4]) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();

    // ---- dW3 (split: D[unit][o] += sum_s H2[s][unit] G3[s][o] on 16 x 16 x 32 MFMAs, A = h2's
    // columns, B = g3's rows in columns 0-7; padding samples have g3 = 0; fp32: lane = unit j, dW3's
    // column j from h2's column and g3's rows) ---------------------------------------------------
    if constexpr (SPLIT) {
      const int c16 = lane & 15, g4 = lane >> 4;
      BF8 bh, bl;
      {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = c16 < 8 ? sG3[8 * g4 + j][c16 & 7] : 0.f;
        split8(v, bh, bl);
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = H2[8 * g4 + j][16 * b + c16];
        BF8 ah, al;
        split8(v, ah, al);
        dWo[b] = mfma16_split(ah, al, bh, bl, dWo[b]);
      }
    } else {
      for (int t = 0; t < ns; ++t) {
        const float h2c = H2[t][lane];
#pragma unroll
        for (int o = 0; o < OUT; ++o) dW3[o] = fmaf(sG3[t][o], h2c, dW3[o]);
      }
    }
    __syncthreads();
    if constexpr (OUT == 8) {
      // g2 = (W3^T g3)(1 - h2^2) on MFMA 32 x 32 x 2, K = the 8 outputs as 4 steps of (o = t, t + 4):
      // A = W3[t + 4 hf][32 jb + r], B = G3[r][t + 4 hf]; the result overwrites h2 in place (each
      // lane rewrites only the stage entries it read)
      const float4 gq = *reinterpret_cast<const float4*>(&sG3[r][4 * hf]);
      const float gb[4] = {gq.x, gq.y, gq.z, gq.w};
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        F16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t) acc = mfma32(w3g[(uint32_t)((t + 4 * hf) * kH + 32 * jb + r)], gb[t], acc);
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          float4* hp = reinterpret_cast<float4*>(&H2[r][32 * jb + 8 * qq + 4 * hf]);
          const float4 hv = *hp;
          *hp = make_float4(acc[4 * qq] * (1.f - hv.x * hv.x), acc[4 * qq + 1] * (1.f - hv.y * hv.y),
                            acc[4 * qq + 2] * (1.f - hv.z * hv.z), acc[4 * qq + 3] * (1.f - hv.w * hv.w));
        }
      }
    } else {
      // the critic's g2 = (W3^T g3)(1 - h2^2) = (W3[j] g3[s])(1 - h2^2), in place in the same
      // layout: lane (r, hf) rewrites sample r's units 32 jb + 8 qq + 4 hf .. + 3
      const float g3 = sG3[r][0];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int j = 32 * jb + 8 * qq + 4 * hf;
          const float4 w = ld4(w3g, (uint32_t)j);
          float4* hp = reinterpret_cast<float4*>(&H2[r][j]);
          const float4 hv = *hp;
          *hp = make_float4(fmaf(w.x, g3, 0.f) * (1.f - hv.x * hv.x), fmaf(w.y, g3, 0.f) * (1.f - hv.y * hv.y),
                            fmaf(w.z, g3, 0.f) * (1.f - hv.z * hv.z), fmaf(w.w, g3, 0.f) * (1.f - hv.w * hv.w));
        }
    }
    __syncthreads();

    // ---- dW2[i][k] += sum_s G2[s][i] H1[s][k] on MFMA: K = the tile's samples as 16 steps of
    // (s = t, t + 16): A = G2[t + 16 hf][32 ib + r], B = H1[t + 16 hf][32 kb + r]; db2 alongside ---
    if constexpr (SPLIT) {  // K = 32 samples as 2 bf16 steps of samples 16 st + 8 hf + j
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        BF8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
        for (int ib = 0; ib < 2; ++ib) {
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = H2[16 * st + 8 * hf + j][32 * ib + r];
#pragma unroll
          for (int j = 0; j < 8; ++j) dB2[ib] += v[j];
          split8(v, ah[ib], al[ib]);
        }
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = sH1[16 * st + 8 * hf + j][32 * kb + r];
          split8(v, bh[kb], bl[kb]);
        }
#pragma unroll
        for (int ib = 0; ib < 2; ++ib)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) dW2[ib][kb] = mfma_split(ah[ib], al[ib], bh[kb], bl[kb], dW2[ib][kb]);
      }
    } else {
#pragma unroll
    for (int t = 0; t < kTile / 2; ++t) {
      const int sidx = t + (kTile / 2) * hf;
      const float a0 = H2[sidx][r], a1 = H2[sidx][32 + r];
      const float h0 = sH1[sidx][r], h1v = sH1[sidx][32 + r];
      dB2[0] += a0;
      dB2[1] += a1;
      dW2[0][0] = mfma32(a0, h0, dW2[0][0]);
      dW2[0][1] = mfma32(a0, h1v, dW2[0][1]);
      dW2[1][0] = mfma32(a1, h0, dW2[1][0]);
      dW2[1][1] = mfma32(a1, h1v, dW2[1][1]);
    }
    }
    __syncthreads();

    // ---- backward through W2 on MFMA: gh1^T[i][s] = sum_j W2[j][i] G2[s][j] (A = W2[t + 32 hf][32 ib
    // + r], B = G2[r][t + 32 hf]); g1 = gh1 (1 - h1^2) overwrites h1 where this lane read it ---------
    if constexpr (SPLIT) {  // A = W2^T[32 ib + r][16 s + 8 hf + j] fragments, B = G2[r][16 s + 8 hf + j]
      BF8 gh[4], gl[4];
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const float4 v0 = *reinterpret_cast<const float4*>(&H2[r][16 * st + 8 * hf]);
        const float4 v1 = *reinterpret_cast<const float4*>(&H2[r][16 * st + 8 * hf + 4]);
        const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        split8(v, gh[st], gl[st]);
      }
#pragma unroll 1
      for (int ib = 0; ib < 2; ++ib) {  // (one block's fragments live at a time)
        F16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          const BF8 ah = ldfrag(frags, frag_at(1, ib, st, 0, lane));
          const BF8 al = ldfrag(frags, frag_at(1, ib, st, 1, lane));
          acc = mfma_split(ah, al, gh[st], gl[st], acc);
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {  // rows i = 32 ib + 8 qq + 4 hf + (0..3) of sample r
          float4* hp = reinterpret_cast<float4*>(&sH1[r][32 * ib + 8 * qq + 4 * hf]);
          const float4 hv = *hp;
          *hp = make_float4(acc[4 * qq] * (1.f - hv.x * hv.x), acc[4 * qq + 1] * (1.f - hv.y * hv.y),
                            acc[4 * qq + 2] * (1.f - hv.z * hv.z), acc[4 * qq + 3] * (1.f - hv.w * hv.w));
        }
      }
    } else {
      float gb[32];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float4 v = *reinterpret_cast<const float4*>(&H2[r][32 * hf + 4 * u]);
        gb[4 * u] = v.x; gb[4 * u + 1] = v.y; gb[4 * u + 2] = v.z; gb[4 * u + 3] = v.w;
      }
#pragma unroll 1
      for (int ib = 0; ib < 2; ++ib) {
        float wa[32];  // W2's column 32 ib + r = row 32 ib + r of W2^T (k_ppo_t64), as float4s
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float4 v = ld4(w2tg, (uint32_t)((32 * ib + r) * kH + 32 * hf + 4 * u));
          wa[4 * u] = v.x; wa[4 * u + 1] = v.y; wa[4 * u + 2] = v.z; wa[4 * u + 3] = v.w;
        }
        F16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
        for (int t = 0; t < 32; ++t) acc = mfma32(wa[t], gb[t], acc);
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {  // rows i = 32 ib + 8 qq + 4 hf + (0..3) of sample r
          float4* hp = reinterpret_cast<float4*>(&sH1[r][32 * ib + 8 * qq + 4 * hf]);
          const float4 hv = *hp;
          *hp = make_float4(acc[4 * qq] * (1.f - hv.x * hv.x), acc[4 * qq + 1] * (1.f - hv.y * hv.y),
                            acc[4 * qq + 2] * (1.f - hv.z * hv.z), acc[4 * qq + 3] * (1.f - hv.w * hv.w));
        }
      }
    }
    __syncthreads();

    // ---- dW1 and db1 (split: D[unit][8 + f] += sum_s G1[s][unit] X[s][f] on the same accumulators,
    // A = g1's columns, B = x's rows in columns 8-15; db1 from the A values; fp32: lane = unit i, dW1's
    // row i and db1 from g1's column and x's rows) -----------------------------------------------
    if constexpr (SPLIT) {
      const int c16 = lane & 15, g4 = lane >> 4;
      BF8 bh, bl;
      {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = c16 >= 8 ? sX[8 * g4 + j][c16 & 7] : 0.f;
        split8(v, bh, bl);
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = sH1[8 * g4 + j][16 * b + c16];
        float s8 = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s8 += v[j];
        dB1p[b] += s8;
        BF8 ah, al;
        split8(v, ah, al);
        dWo[b] = mfma16_split(ah, al, bh, bl, dWo[b]);
      }
    }
    if constexpr (!SPLIT) for (int t = 0; t < ns; ++t) {
      const float g = sH1[t][lane];
      dB1 += g;
      const float4 xa = *reinterpret_cast<const float4*>(&sX[t][0]);
      const float4 xb = *reinterpret_cast<const float4*>(&sX[t][4]);
      dW1[0] = fmaf(g, xa.x, dW1[0]);
      dW1[1] = fmaf(g, xa.y, dW1[1]);
      dW1[2] = fmaf(g, xa.z, dW1[2]);
      dW1[3] = fmaf(g, xa.w, dW1[3]);
      dW1[4] = fmaf(g, xb.x, dW1[4]);
      dW1[5] = fmaf(g, xb.y, dW1[5]);
      dW1[6] = fmaf(g, xb.z, dW1[6]);
      dW1[7] = fmaf(g, xb.w, dW1[7]);
    }
    __syncthreads();  // the next tile's stage overwrites what this one read
  }

  if constexpr (EVAL) return;
  // ---- this wave's partial gradient --------------------------------------------------------
  float* out = partial + (size_t)blockIdx.x * partial_stride<OUT>();
  if constexpr (SPLIT) {
    const int c16 = lane & 15, g4 = lane >> 4;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int unit = 16 * b + 4 * g4 + i;
        if (c16 >= 8) out[unit * kF + (c16 - 8)] = dWo[b][i];
        else if (c16 < OUT) out[kOffW3 + c16 * kH + unit] = dWo[b][i];
      }
      // db1 of unit 16 b + c16: the four sample groups' partial sums (lanes c16, c16 + 16, + 32, + 48)
      float d = dB1p[b] + __shfl_xor(dB1p[b], 16, 64);
      d += __shfl_xor(d, 32, 64);
      if (g4 == 0) out[kOffB1 + 16 * b + c16] = d;
    }
  } else {
#pragma unroll
    for (int f = 0; f < kF; ++f) out[lane * kF + f] = dW1[f];
    out[kOffB1 + lane] = dB1;
  }
#pragma unroll
  for (int ib = 0; ib < 2; ++ib)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = 32 * ib + (q & 3) + 8 * (q >> 2) + 4 * hf;  // the accumulator's row map
        out[kOffW2 + i * kH + 32 * kb + r] = dW2[ib][kb][q];
      }
#pragma unroll
  for (int ib = 0; ib < 2; ++ib) {
    const float d = dB2[ib] + __shfl_xor(dB2[ib], 32, 64);  // the two sample halves
    if (hf == 0) out[kOffB2 + 32 * ib + r] = d;
  }
  if constexpr (!SPLIT) {
#pragma unroll
    for (int o = 0; o < OUT; ++o) out[kOffW3 + o * kH + lane] = dW3[o];
  }
#pragma unroll
  for (int o = 0; o < OUT; ++o) dB3[o] = wave_sum(dB3[o]);
  pg_sum = wave_sum(pg_sum);
  vf_sum = wave_sum(vf_sum);
  ent_sum = wave_sum(ent_sum);
  if (lane == 0) {
#pragma unroll
    for (int o = 0; o < OUT; ++o) out[off_b3<OUT>() + o] = dB3[o];
    out[n_params<OUT>() + 0] = pg_sum;
    out[n_params<OUT>() + 1] = vf_sum;
    out[n_params<OUT>() + 2] = ent_sum;
  }
}

// The split-bf16 A fragments of both networks (k_ppo_grad<., ., true>): for mat 0, W2[32 blk + r][16 s
// + 8 h + j]; for mat 1, W2^T[32 blk + r][...] = W2[16 s + 8 h + j][32 blk + r]; hi = bf16(w),
// lo = bf16(w - hi).  One thread per (net, mat, blk, s, lane).
__global__ __launch_bounds__(256) void k_ppo_frag(const float* __restrict__ wa, const float* __restrict__ wc,
                                                 uint4* __restrict__ out, const float* __restrict__ a_w1,
                                                 const float* __restrict__ a_b1, const float* __restrict__ a_b2,
                                                 const float* __restrict__ c_w1, const float* __restrict__ c_b1,
                                                 const float* __restrict__ c_b2, float* __restrict__ scaled) {
  const int t = blockIdx.x * 256 + threadIdx.x;  // < 2 nets x 2 mats x 2 blks x 4 steps x 64 lanes
  if (t < 2 * kScaledPerNet) {  // [net][W1 | b1 | b2] x 2 log2 e (tanh_prescaled); a net passed as null is skipped
    const int net = t / kScaledPerNet, e = t - net * kScaledPerNet;
    const float* w1 = net ? c_w1 : a_w1;
    const float* b1 = net ? c_b1 : a_b1;
    const float* b2 = net ? c_b2 : a_b2;
    if (w1) scaled[t] = kTanhScale * (e < kH * kF ? w1[e] : (e < kH * kF + kH ? b1[e - kH * kF] : b2[e - kH * kF - kH]));
  }
  if (t >= 2 * 2 * 2 * 4 * 64) return;
  const int lane = t & 63, s = (t >> 6) & 3, blk = (t >> 8) & 1, mat = (t >> 9) & 1, net = t >> 10;
  const float* w = net ? wc : wa;
  const int r = lane & 31, h = lane >> 5;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    // mat 0 pairs with layer 1's accumulator as the B operand, whose element j of lane half h in
    // k step s is unit 16 s + 8 (j >> 2) + 4 h + (j & 3) (the 32 x 32 result map), and carries
    // tanh_prescaled's 2 log2 e; mat 1 with G2 rows read in natural order, k = 16 s + 8 h + j
    const int row = 32 * blk + r, k = mat == 0 ? 16 * s + 8 * (j >> 2) + 4 * h + (j & 3) : 16 * s + 8 * h + j;
    v[j] = mat == 0 ? kTanhScale * w[row * kH + k] : w[k * kH + row];
  }
  BF8 hi, lo;
  split8(v, hi, lo);
  uint4* o = out + net * kFragsPerNet;
  o[frag_at(mat, blk, s, 0, lane)] = __builtin_bit_cast(uint4, hi);
  o[frag_at(mat, blk, s, 1, lane)] = __builtin_bit_cast(uint4, lo);
}

// W2^T of both networks into the workspace (64 x 64 each), so the backward pass through W2 reads
// its A operand (a column of W2 per lane) as row vectors, like the forward pass.  The values
// are copied, not recomputed: the products and their order are unchanged.
__global__ __launch_bounds__(256) void k_ppo_t64(const float* __restrict__ wa, const float* __restrict__ wc,
                                                float* __restrict__ out) {
  const float* w = blockIdx.y ? wc : wa;
  float* o = out + blockIdx.y * kH * kH;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < kH * kH; e += gridDim.x * 256) {
    const int i = e >> 6, j = e & 63;  // out[i][j] = w[j][i]
    o[e] = w[j * kH + i];
  }
}

// Sum the partials of `waves` waves in a fixed order, both networks in one launch: blocks
// [0, nba) take the actor's entries, the rest the critic's, 32 entries (one 128-B line of every
// partial row) per block.  Thread (g, p) adds waves g, g + 32, ... of entry p, then thread g = 0
// adds the 32 sums in order.  Entries past a network's parameters are its loss sums; each loss
// term is written by the one network that has it (the actor's policy and entropy, the critic's
// value; the other network's slot is 0), scaled by 1/n.  One launch of ~316 blocks keeps every
// CU loading, where one 83-block launch per network left two thirds of them idle.
constexpr int kRedLanes = 32, kRedGroups = 32;
__global__ __launch_bounds__(1024) void k_ppo_reduce(const float* __restrict__ pa, const float* __restrict__ pc,
                                                     int waves, int nba, float* __restrict__ grad,
                                                     float* __restrict__ loss, float inv_n) {
  __shared__ float sum[kRedGroups][kRedLanes];
  const int pl = threadIdx.x & (kRedLanes - 1), g = threadIdx.x / kRedLanes;
  const bool actor = (int)blockIdx.x < nba;
  const int P = actor ? n_params<8>() : n_params<1>();
  const size_t S = actor ? partial_stride<8>() : partial_stride<1>();
  const float* partial = actor ? pa : pc;
  const int p = ((int)blockIdx.x - (actor ? 0 : nba)) * kRedLanes + pl;
  float a = 0.f;
  if (p < P + 3) {
    // unrolled so sixteen loads are in flight per thread; the additions keep their order
#pragma unroll 16
    for (int w = g; w < waves; w += kRedGroups) a += partial[(size_t)w * S + p];
  }
  sum[g][pl] = a;
  __syncthreads();
  if (g == 0 && p < P + 3) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < kRedGroups; ++i) t += sum[i][pl];
    if (p < P) {
      grad[(actor ? 0 : n_params<8>()) + p] = t;
    } else if ((p - P == 1) != actor) {
      loss[p - P] = 0.f + t * inv_n;
    }
  }
}

// GAE over a [T][N] trajectory (ppo.py gae): one lane per arena walks its ticks backwards, every
// load coalesced across the wave's arenas.  The TD error keeps gae()'s op order, one rounding
// per op (r + (gamma v[t+1]) keep) - v[t]; the recursion is addcmul's fused multiply-add.
// Rewards (f64) and done flags (u8) are read as the trajectory holds them.
__global__ __launch_bounds__(256) void k_ppo_gae(const double* __restrict__ rew, const uint8_t* __restrict__ done,
                                                 const float* __restrict__ val, int T, int64_t N, float gamma,
                                                 float gamma_lam, float* __restrict__ adv, float* __restrict__ ret) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  // ticks in batches of kU, every load of a batch issued before its recursion runs (one wave per
  // SIMD at C5's 65 536 arenas: the loads in flight, not the arithmetic, set the pace); v[t + 1]
  // of tick t is the batch's previous tick's v[t], so val is read once per tick.  The T mod kU
  // ticks left at the start of the trajectory run one by one.
  constexpr int kU = 16;
  float a = 0.f;
  int t = T - 1;
  for (; t + 1 >= kU; t -= kU) {  // ticks t, t - 1, ..., t - kU + 1
    uint8_t d[kU];
    float v[kU + 1];
    double r[kU];
    v[0] = val[(int64_t)(t + 1) * N + n];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = (int64_t)(t - u) * N + n;
      d[u] = done[i];
      v[u + 1] = val[i];
      r[u] = rew[i];
    }
    __builtin_amdgcn_sched_barrier(0);  // (the scheduler would sink each load to its use)
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = (int64_t)(t - u) * N + n;
      const float keep = 1.f - (float)d[u];
      const float delta = ((float)r[u] + (gamma * v[u]) * keep) - v[u + 1];
      a = t - u == T - 1 ? delta : fmaf(gamma_lam * keep, a, delta);
      adv[i] = a;
      ret[i] = a + v[u + 1];
    }
  }
  for (; t >= 0; --t) {
    const int64_t i = (int64_t)t * N + n;
    const float keep = 1.f - (float)done[i];
    const float v0 = val[i];
    const float delta = ((float)rew[i] + (gamma * val[i + N]) * keep) - v0;
    a = t == T - 1 ? delta : fmaf(gamma_lam * keep, a, delta);
    adv[i] = a;
    ret[i] = a + v0;
  }
}

// The update's sample table, one row per sample: x[8], action, old log-prob, the advantage
// normalised as (adv - mean) / (std + 1e-8) with the batch statistics in stats[2], return.
__global__ __launch_bounds__(256) void k_ppo_pack(const float* __restrict__ x, const uint8_t* __restrict__ act,
                                                  const float* __restrict__ old, const float* __restrict__ adv,
                                                  const float* __restrict__ ret, const float* __restrict__ stats,
                                                  int64_t n, float* __restrict__ rows) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  const float4* xs = reinterpret_cast<const float4*>(x + m * kF);
  float4* out = reinterpret_cast<float4*>(rows + m * kRow);
  const float mean = stats[0], den = stats[1] + 1e-8f;
  out[0] = xs[0];
  out[1] = xs[1];
  out[2] = make_float4((float)act[m], old[m], (adv[m] - mean) / den, ret[m]);
}

// obs_features (rollout.py) of n observations: guard / 3, move / 16, move_frame / 55, position / 4.6
// for both fighters, each as torch's division by a host scalar computes it on the GPU: x times the
// f64 reciprocal of the divisor rounded to f32 (neither x / b nor x * (1.0f / b) agrees for 4.6).
__global__ __launch_bounds__(256) void k_ppo_features(const uint8_t* __restrict__ guard, const uint8_t* __restrict__ move,
                                                      const float* __restrict__ move_frame,
                                                      const float* __restrict__ position, int64_t n,
                                                      float* __restrict__ out) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  const uchar2 g = reinterpret_cast<const uchar2*>(guard)[m];
  const uchar2 mv = reinterpret_cast<const uchar2*>(move)[m];
  const float2 f = reinterpret_cast<const float2*>(move_frame)[m];
  const float2 p = reinterpret_cast<const float2*>(position)[m];
  float4* o = reinterpret_cast<float4*>(out + m * kF);
  constexpr float r3 = (float)(1.0 / 3.0), r16 = (float)(1.0 / 16.0), r55 = (float)(1.0 / 55.0), r46 = (float)(1.0 / 4.6);
  o[0] = make_float4((float)g.x * r3, (float)g.y * r3, (float)mv.x * r16, (float)mv.y * r16);
  o[1] = make_float4(f.x * r55, f.y * r55, p.x * r46, p.y * r46);
}

}  // namespace fsl

namespace fsk {

hipError_t launch_ppo_features(const uint8_t* guard, const uint8_t* move, const float* move_frame,
                               const float* position, int64_t n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(fsl::k_ppo_features, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, guard, move, move_frame,
                     position, n, out);
  return hipGetLastError();
}

hipError_t launch_ppo_gae(const double* rew, const uint8_t* done, const float* val, int T, int64_t N, float gamma,
                          float gamma_lam, float* adv, float* ret, hipStream_t s) {
  hipLaunchKernelGGL(fsl::k_ppo_gae, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, rew, done, val, T, N, gamma,
                     gamma_lam, adv, ret);
  return hipGetLastError();
}

hipError_t launch_ppo_pack(const float* x, const uint8_t* act, const float* old, const float* adv, const float* ret,
                           const float* stats, int64_t n, float* rows, hipStream_t s) {
  hipLaunchKernelGGL(fsl::k_ppo_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, act, old, adv, ret,
                     stats, n, rows);
  return hipGetLastError();
}

// workspace: the actor's and the critic's partial gradients, W2^T of both, the split-bf16 fragments
static size_t ppo_frag_offset() {
  return sizeof(float) * ((size_t)fsl::kMaxWaves * (fsl::partial_stride<8>() + fsl::partial_stride<1>()) +
                          2 * fsl::kH * fsl::kH);
}
static size_t ppo_scaled_offset() { return ppo_frag_offset() + sizeof(uint4) * 2 * fsl::kFragsPerNet; }
size_t ppo_workspace_bytes() { return ppo_scaled_offset() + sizeof(float) * 2 * fsl::kScaledPerNet; }

hipError_t launch_ppo_grad(const float* rows, int64_t n, const float* const actor[6], const float* const critic[6],
                           float clip, float vf_coef, float ent_coef, float* grad, float* loss, void* workspace,
                           hipStream_t s, bool split, const int64_t* runs, int run_shift, int64_t n_rows) {
  using namespace fsl;
  const int64_t tiles = (n + kTile - 1) / kTile;
  const int waves = (int)(tiles < kMaxWaves ? tiles : kMaxWaves);
  const Coef c{clip, vf_coef, ent_coef, 1.0f / (float)n};
  float* pa = static_cast<float*>(workspace);
  float* pc = pa + (size_t)kMaxWaves * partial_stride<8>();
  float* w2t = pc + (size_t)kMaxWaves * partial_stride<1>();  // [2][64][64]: actor, critic
  uint4* frags = reinterpret_cast<uint4*>(static_cast<char*>(workspace) + ppo_frag_offset());
  if (split) {  // (W1, b1, b2 as 2 log2 e x their values from the workspace: tanh_prescaled)
    float* sc = reinterpret_cast<float*>(static_cast<char*>(workspace) + ppo_scaled_offset());
    float *sa = sc, *sk = sc + kScaledPerNet;
    hipLaunchKernelGGL(k_ppo_frag, dim3(8), dim3(256), 0, s, actor[2], critic[2], frags, actor[0], actor[1], actor[3],
                       critic[0], critic[1], critic[3], sc);
    hipLaunchKernelGGL((k_ppo_grad<8, false, true>), dim3(waves), dim3(64), 0, s, rows, n, tiles, sa, sa + kH * kF,
                       actor[2], sa + kH * kF + kH, actor[4], actor[5], c, pa, nullptr, nullptr, frags, runs, run_shift,
                       n_rows);
    hipLaunchKernelGGL((k_ppo_grad<1, false, true>), dim3(waves), dim3(64), 0, s, rows, n, tiles, sk, sk + kH * kF,
                       critic[2], sk + kH * kF + kH, critic[4], critic[5], c, pc, nullptr, nullptr, frags + kFragsPerNet,
                       runs, run_shift, n_rows);
  } else {
    hipLaunchKernelGGL(k_ppo_t64, dim3(4, 2), dim3(256), 0, s, actor[2], critic[2], w2t);
    hipLaunchKernelGGL(k_ppo_grad<8>, dim3(waves), dim3(64), 0, s, rows, n, tiles, actor[0], actor[1], actor[2],
                       actor[3], actor[4], actor[5], c, pa, nullptr, w2t, nullptr, runs, run_shift, n_rows);
    hipLaunchKernelGGL(k_ppo_grad<1>, dim3(waves), dim3(64), 0, s, rows, n, tiles, critic[0], critic[1], critic[2],
                       critic[3], critic[4], critic[5], c, pc, nullptr, w2t + kH * kH, nullptr, runs, run_shift, n_rows);
  }
  const int nba = (n_params<8>() + 3 + kRedLanes - 1) / kRedLanes, nbc = (n_params<1>() + 3 + kRedLanes - 1) / kRedLanes;
  hipLaunchKernelGGL(k_ppo_reduce, dim3(nba + nbc), dim3(kRedLanes * kRedGroups), 0, s, pa, pc, waves, nba, grad, loss,
                     c.inv_n);
  return hipGetLastError();
}

hipError_t launch_ppo_eval(const float* x, int64_t n_values, const uint8_t* actions, int64_t n_logp,
                           const float* const actor[6], const float* const critic[6], float* values, float* logp,
                           void* workspace, hipStream_t s, bool split) {
  using namespace fsl;
  const Coef c{0.f, 0.f, 0.f, 0.f};
  uint4* frags = split ? reinterpret_cast<uint4*>(static_cast<char*>(workspace) + ppo_frag_offset()) : nullptr;
  float* sc = split ? reinterpret_cast<float*>(static_cast<char*>(workspace) + ppo_scaled_offset()) : nullptr;
  const bool run_v = values && n_values > 0, run_l = logp && n_logp > 0;
  if (split) {  // (a network not run passes its actor / critic arrays as null: its fragments are not built)
    const float* wa = run_l ? actor[2] : (run_v ? critic[2] : nullptr);
    const float* wc = run_v ? critic[2] : wa;
    const float* const* na = run_l ? actor : nullptr;
    const float* const* nc = run_v ? critic : nullptr;
    if (wa)
      hipLaunchKernelGGL(k_ppo_frag, dim3(8), dim3(256), 0, s, wa, wc, frags, na ? na[0] : nullptr, na ? na[1] : nullptr,
                         na ? na[3] : nullptr, nc ? nc[0] : nullptr, nc ? nc[1] : nullptr, nc ? nc[3] : nullptr, sc);
  }
  if (run_v) {
    const int64_t tiles = (n_values + kTile - 1) / kTile;
    const int waves = (int)(tiles < kMaxEvalWaves ? tiles : kMaxEvalWaves);
    if (split) {
      const float* sk = sc + kScaledPerNet;
      hipLaunchKernelGGL((k_ppo_grad<1, true, true>), dim3(waves), dim3(64), 0, s, x, n_values, tiles, sk, sk + kH * kF,
                         critic[2], sk + kH * kF + kH, critic[4], critic[5], c, values, nullptr, nullptr,
                         frags + kFragsPerNet);
    }
    else
      hipLaunchKernelGGL((k_ppo_grad<1, true>), dim3(waves), dim3(64), 0, s, x, n_values, tiles, critic[0], critic[1],
                         critic[2], critic[3], critic[4], critic[5], c, values, nullptr);
  }
  if (run_l) {
    const int64_t tiles = (n_logp + kTile - 1) / kTile;
    const int waves = (int)(tiles < kMaxEvalWaves ? tiles : kMaxEvalWaves);
    if (split)
      hipLaunchKernelGGL((k_ppo_grad<8, true, true>), dim3(waves), dim3(64), 0, s, x, n_logp, tiles, sc, sc + kH * kF,
                         actor[2], sc + kH * kF + kH, actor[4], actor[5], c, logp, actions, nullptr, frags);
    else
      hipLaunchKernelGGL((k_ppo_grad<8, true>), dim3(waves), dim3(64), 0, s, x, n_logp, tiles, actor[0], actor[1],
                         actor[2], actor[3], actor[4], actor[5], c, logp, actions);
  }
  return hipGetLastError();
}

}  // namespace fsk
