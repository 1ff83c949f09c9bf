// fs_policy.h -- the C5 actor inside the fused tick loop (included by fs_kernels.hip).
//
// P1's action every tick is sampled from an MLP actor on its observation:
//   x (8) = [guard/3, move/16, move_frame/55, position/4.6] of P1, P2   (footsies_gym_amd/rollout.py)
//   logits (8) = W3 tanh(W2 tanh(W1 x + b1) + b2) + b3                  (torch nn.Linear layouts)
//   a ~ softmax(logits) by inverse CDF with one counter-based uniform per (arena, tick)
// The three layers run per wave (32 arenas) on v_mfma_f32_32x32x16_bf16 in the transposed
// orientation: hidden units on the 32 rows, arenas on the lanes.  A 32x32 f32 result then has
// its column (arena) on the lane and its rows in the 16 accumulator registers, which is the B
// fragment of the next product with no data movement (the k order inside a fragment is
// permuted -- element j of lane half h is row 16s + 8(j>>2) + 4h + (j&3) -- so the weight
// fragments are built in that order).  tanh's scale and offset are folded into the weights (see
// kTanhScale), so a hidden value costs v_exp_f32 + v_add + v_rcp_f32 + half a v_cvt_pk_bf16_f32.
// Weights, inputs and the hidden r values are bf16; accumulation is f32.
//
// MFMA operand maps (gfx950, 32x32x16 bf16): lane l, r = l & 31, h = l >> 5 holds
// A[row r][k = 8h + j] and B[k = 8h + j][col r] in element j; C/D: col = r,
// row = (i & 3) + 8 (i >> 2) + 4h for register i.
#pragma once

namespace fsk {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kPolFrags = 17;  // a1[2] | a2[u=2][t,s=4] | a2b[2] | a3[4] | a3b
constexpr int kPolA1 = 0, kPolA2 = 2, kPolA2b = 10, kPolA3 = 12, kPolA3b = 16;
__shared__ bf16x8 sPol[kPolFrags][64];  // every wave of the block reads the same image

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// hidden unit held in element j of a fragment built from accumulator registers 8s..8s+7
__device__ __forceinline__ int acc_row(int s, int j, int h) { return 16 * s + 8 * (j >> 2) + 4 * h + (j & 3); }

// tanh z = 1 - 2 r with r = 1 / (1 + 2^(c z)), c = 2 log2(e).  The affine parts are folded into
// the weights: a layer whose output feeds tanh is pre-scaled by c, so its accumulator is the exp2
// argument; a layer whose input is tanh of the previous one takes r instead, with weights -2 W
// and bias b + sum_k W[., k] (so W (1 - 2 r) + b is unchanged).  What crosses between layers is
// r rounded to bf16.  Biases ride in two k slots as a bf16 hi + lo pair against constant 1s.
constexpr float kTanhScale = 2.8853900817779268f;  // 2 log2(e)

__device__ __forceinline__ void bias_pair(bf16x8& a, float b) {
  const __bf16 hi = (__bf16)b;
  a[0] = hi;
  a[1] = (__bf16)(b - (float)hi);
}

// Build the weight fragments once per block (threads 0..63 write; the caller syncs).
__device__ __forceinline__ void stage_policy(const PolicyParams& P) {
  if (threadIdx.x >= 64) return;
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  for (int t = 0; t < 2; t++) {  // layer 1: row = hidden 32t + r; k = feature 8h + j, bias at k = 8, 9
    bf16x8 a = {};
    const int row = 32 * t + r;
    if (h == 0)
      for (int j = 0; j < 8; j++) a[j] = (__bf16)(kTanhScale * P.w1[row * 8 + j]);
    else
      bias_pair(a, kTanhScale * P.b1[row]);
    sPol[kPolA1 + t][l] = a;
  }
  for (int u = 0; u < 2; u++) {  // layer 2: row = hidden 32u + r; k = hidden 32t + acc_row(s, j, h)
    const int row = 32 * u + r;
    for (int t = 0; t < 2; t++)
      for (int s = 0; s < 2; s++) {
        bf16x8 a;
        for (int j = 0; j < 8; j++) a[j] = (__bf16)(-2.0f * kTanhScale * P.w2[row * 64 + 32 * t + acc_row(s, j, h)]);
        sPol[kPolA2 + 4 * u + 2 * t + s][l] = a;
      }
    float sum = 0.0f;
    for (int k = 0; k < 64; k++) sum += P.w2[row * 64 + k];
    bf16x8 b = {};
    if (h == 0) bias_pair(b, kTanhScale * (P.b2[row] + sum));
    sPol[kPolA2b + u][l] = b;
  }
  for (int u = 0; u < 2; u++)  // layer 3: row = action r (< 8, the rest zero); k = hidden 32u + ...
    for (int s = 0; s < 2; s++) {
      bf16x8 a;
      for (int j = 0; j < 8; j++) a[j] = (__bf16)(r < 8 ? -2.0f * P.w3[r * 64 + 32 * u + acc_row(s, j, h)] : 0.0f);
      sPol[kPolA3 + 2 * u + s][l] = a;
    }
  float sum = 0.0f;
  if (r < 8)
    for (int k = 0; k < 64; k++) sum += P.w3[r * 64 + k];
  bf16x8 b = {};
  if (h == 0 && r < 8) bias_pair(b, P.b3[r] + sum);
  sPol[kPolA3b][l] = b;
}

// e^x on v_exp_f32 (2^x, ~1 ulp) with no denormal range fix-up: the results feed a softmax
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }

// one hidden tile: r = 1 / (1 + 2^d) of the (pre-scaled) accumulator on v_exp_f32 / v_rcp_f32
// (~1 ulp each; saturates through 2^d = inf / 0, no NaN for finite d), packed as the two B
// fragments (k-steps s = 0, 1) of the next layer
__device__ __forceinline__ float tanh_r(float d) { return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(d)); }
__device__ __forceinline__ void activate(const f32x16& d, bf16x8& b0, bf16x8& b1) {
#pragma unroll
  for (int j = 0; j < 8; j++) {
    b0[j] = (__bf16)tanh_r(d[j]);
    b1[j] = (__bf16)tanh_r(d[8 + j]);
  }
}

__device__ __forceinline__ uint32_t lane_read(uint32_t v, int src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}
__device__ __forceinline__ float lane_read(float v, int src_lane) {
  return __uint_as_float(lane_read(__float_as_uint(v), src_lane));
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const __bf16 a = (__bf16)lo, b = (__bf16)hi;
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}

// uniform in [0, 1) of (seed, arena, tick): 24 bits of a splitmix64 finaliser
__device__ __forceinline__ float policy_uniform(uint64_t seed, uint64_t arena, uint64_t t) {
  uint64_t x = seed ^ (arena * 0x9E3779B97F4A7C15ull) ^ (t * 0xD1B54A32D192ED03ull);
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (float)(uint32_t)(x >> 40) * (1.0f / 16777216.0f);
}

struct PolicyOut {
  uint32_t action;
  float logp;
};

// The actor for the wave's 32 arenas.  Called by every lane of the wave in lockstep with the
// wave's pair layout (lane 2a + k = fighter k of local arena a): `d0`, `d1` are this lane's
// fighter features packed as bf16x2 (guard/3 | move/16, move_frame/55 | position/4.6).
// Returns, on every lane, the action and log-probability of its own arena (l >> 1).
// The weight fragments of this lane (sPol[.][lane]), read once per launch into registers: 17 ds_read_b128
// per wave-tick less on the LDS pipe and none on the MFMA's operand path.
struct PolicyWeights {
  bf16x8 f[kPolFrags];
};
__device__ __forceinline__ PolicyWeights policy_weights() {
  PolicyWeights w;
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < kPolFrags; i++) w.f[i] = sPol[i][l];
  return w;
}

__device__ __forceinline__ PolicyOut policy_act(const PolicyWeights& W, uint32_t d0, uint32_t d1, uint64_t seed,
                                                uint64_t arena0, uint64_t t) {
  const int l = threadIdx.x & 63, r = l & 31, h = l >> 5;
  // gather: MFMA lane r takes arena r's two fighters (pair lanes 2r, 2r + 1)
  const uint32_t p1d0 = lane_read(d0, 2 * r), p2d0 = lane_read(d0, 2 * r + 1);
  const uint32_t p1d1 = lane_read(d1, 2 * r), p2d1 = lane_read(d1, 2 * r + 1);
  bf16x8 x;
  {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 v;
    // element order k: g1, g2, m1, m2, mf1, mf2, x1, x2 (rollout.obs_features)
    v.x = __builtin_amdgcn_perm(p2d0, p1d0, 0x05040100u);  // lo halves: g1 | g2
    v.y = __builtin_amdgcn_perm(p2d0, p1d0, 0x07060302u);  // hi halves: m1 | m2
    v.z = __builtin_amdgcn_perm(p2d1, p1d1, 0x05040100u);
    v.w = __builtin_amdgcn_perm(p2d1, p1d1, 0x07060302u);
    const u32x4 one = {0x3F803F80u, 0u, 0u, 0u};  // k = 8, 9: bf16 1.0 (the layer-1 bias pair)
    x = __builtin_bit_cast(bf16x8, h == 0 ? v : one);
  }
  bf16x8 ones = {};  // the bias pair's k slots of layers 2 and 3
  if (h == 0) ones[0] = ones[1] = (__bf16)1.0f;
  const f32x16 zero = {};
  // layer 1
  f32x16 d1a = mfma(W.f[kPolA1 + 0], x, zero), d1b = mfma(W.f[kPolA1 + 1], x, zero);
  bf16x8 h1[2][2];
  activate(d1a, h1[0][0], h1[0][1]);
  activate(d1b, h1[1][0], h1[1][1]);
  // layer 2
  bf16x8 h2[2][2];
#pragma unroll
  for (int u = 0; u < 2; u++) {
    f32x16 acc = mfma(W.f[kPolA2b + u], ones, zero);
#pragma unroll
    for (int tt = 0; tt < 2; tt++)
#pragma unroll
      for (int s = 0; s < 2; s++) acc = mfma(W.f[kPolA2 + 4 * u + 2 * tt + s], h1[tt][s], acc);
    activate(acc, h2[u][0], h2[u][1]);
  }
  // layer 3: logits of actions 4h .. 4h + 3 land in registers 0..3
  f32x16 lg = mfma(W.f[kPolA3b], ones, zero);
#pragma unroll
  for (int u = 0; u < 2; u++)
#pragma unroll
    for (int s = 0; s < 2; s++) lg = mfma(W.f[kPolA3 + 2 * u + s], h2[u][s], lg);
  // softmax over the two halves (partner lane l ^ 32), inverse-CDF sample, log-probability
  const float m_mine = fmaxf(fmaxf(lg[0], lg[1]), fmaxf(lg[2], lg[3]));
  const float m = fmaxf(m_mine, lane_read(m_mine, l ^ 32));
  const float e0 = fast_exp(lg[0] - m), e1 = fast_exp(lg[1] - m), e2 = fast_exp(lg[2] - m), e3 = fast_exp(lg[3] - m);
  const float s_mine = ((e0 + e1) + e2) + e3;
  const float s_other = lane_read(s_mine, l ^ 32);
  const float s_lo = h == 0 ? s_mine : s_other, s_hi = h == 0 ? s_other : s_mine;
  const float total = s_lo + s_hi;
  const float target = policy_uniform(seed, arena0 + (uint64_t)r, t) * total;
  // first action whose cumulative weight exceeds the target (half h = 0 starts at 0, h = 1 at s_lo)
  const float base = h == 0 ? 0.0f : s_lo;
  const float c0 = base + e0, c1 = c0 + e1, c2 = c1 + e2;
  const uint32_t i_mine = target < c0 ? 0u : target < c1 ? 1u : target < c2 ? 2u : 3u;
  const uint32_t i_other = lane_read(i_mine, l ^ 32);
  const bool low = target < s_lo;
  const uint32_t action = low ? (h == 0 ? i_mine : i_other) : 4u + (h == 0 ? i_other : i_mine);
  // the chosen logit lives in half (action >> 2), register (action & 3)
  const uint32_t j = action & 3u;
  const float lg_mine = j == 0 ? lg[0] : j == 1 ? lg[1] : j == 2 ? lg[2] : lg[3];
  const float lg_other = lane_read(lg_mine, l ^ 32);
  const float chosen = ((int)(action >> 2) == h) ? lg_mine : lg_other;
  // back to the pair layout: sim lane l holds arena l >> 1, computed on MFMA lane l >> 1
  PolicyOut o;
  o.action = lane_read(action, l >> 1);
  o.logp = lane_read(chosen - m - __logf(total), l >> 1);
  return o;
}

}  // namespace fsk
