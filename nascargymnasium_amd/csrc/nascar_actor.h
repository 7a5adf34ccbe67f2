// nascar_actor.h -- fused SAC actor inference on MFMA.
//
// The reference's closed-loop drivers run Stable-Baselines3 SAC policies
// (game/control/sac_control_class.py:80-115: model.predict(obs, deterministic=True)):
// MlpPolicy actor  latent = ReLU(W2 ReLU(W1 obs + b1) + b2),  mu = W3 latent + b3,
// action = unscale_action(tanh(mu))  with the Box(-1, 1) action space.
//
// One wave = 32 observations; all three layers run on the MFMA with the batch on the lanes:
//   layer 1  H1^T[256 x 32] = [W1 | b1_hi | b1_lo][256 x 40] . [X | 1 | 1]^T   (bf16 MFMA 32x32x16, fp32
//            acc; 8 tiles x 3 k-steps -- the bias rides in two extra K columns, hi + lo bf16 halves)
//   layer 2  H2^T[256 x 32] = W2[256 x 256] . relu(H1^T) + b2   (the layer-1 accumulator tiles, ReLU'd
//            and packed to bf16 in registers, are the B operands directly -- hidden units sit in the
//            registers -- with W2 pre-permuted on the host into the matching k order; b2 is the
//            accumulator's initial value; W2 staged in LDS per workgroup)
//   layer 3  mu^T[32 x 32] = W3'[32 x 256] . relu(H2^T)  with the same register trick; W3' rows 0-3 are
//            bf16 hi(w3[0]), hi(w3[1]), lo(w3[0]), lo(w3[1]) (rows 4-31 zero), so mu_i = row i + row i+2
//            carries W3 to ~2^-16 relative
// Numerics: bf16 operands X, W1, relu(H1), W2, relu(H2); b1 and W3 as bf16 hi + lo pairs; fp32
// accumulation, b2 and tanh in fp32.  Tolerance vs a PyTorch fp32 forward: tests/test_gpu_actor.py.
#pragma once
#include "nascar_device.h"

namespace nascar {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) short i16x8;
typedef __attribute__((ext_vector_type(2))) float f32x2;

typedef __attribute__((ext_vector_type(2))) short i16x2;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

// two floats -> packed bf16 pair, round-to-nearest-even: one v_cvt_pk_bf16_f32 (converted pairwise --
// hipcc splits wider vector truncations that feed integer ops into per-element converts + v_perm)
__device__ __forceinline__ unsigned cvt_pk_bf16(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(((f32x2){a, b}), bf16x2));
}
// ReLU on a packed bf16 pair's bits (v_pk_max_i16: a negative bf16 is a negative int16)
__device__ __forceinline__ unsigned relu_pk(unsigned p) {
  return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(i16x2, p), (i16x2){}));
}
// relu of registers 8S .. 8S+7 of an accumulator tile as one bf16 B fragment
template <int S>
__device__ __forceinline__ bf16x8 relu_bf16x8(const f32x16& a) {
  const u32x4 u = {relu_pk(cvt_pk_bf16(a[8 * S], a[8 * S + 1])), relu_pk(cvt_pk_bf16(a[8 * S + 2], a[8 * S + 3])),
                   relu_pk(cvt_pk_bf16(a[8 * S + 4], a[8 * S + 5])), relu_pk(cvt_pk_bf16(a[8 * S + 6], a[8 * S + 7]))};
  return __builtin_bit_cast(bf16x8, u);
}

#define ACT_OBS 38
#define ACT_K 40          // layer-1 K: 38 features + the b1 hi/lo columns (row stride of w1p)
#define ACT_H 256
#define ACT_OUT 2
#define ACT_WAVES 8       // waves per workgroup (2 per SIMD); each walks its own 32-observation tiles

struct ActorDev {
  const bf16x8* w1p;   // [256][40] bf16: W1 row | bf16(b1) | bf16(b1 - bf16(b1)), read as 16-B fragments
  const bf16x8* w2p;   // [8 o][8 q][2 s][2 h][32 r] x 8 bf16: W2[32o + r][32q + 16s + 8(j>>2) + 4h + (j&3)]
                       // (lane l = 32h + r reads fragment l of a 1 KB block: conflict-free ds_read_b128)
  const float* b2;     // [256]
  const bf16x8* w3p;   // [8 o][2 s][2 h][4 r] x 8 bf16: W3'[r][32o + 16s + 8(j>>2) + 4h + (j&3)], rows 0-3
  const float* b3;     // [2]
};

// The observations of one 32-row wave tile in the layer-1 B layout: lane (r, h) holds
// obs[row r][16s + 8h .. +7] for s = 0, 1 and, on h = 0 lanes, obs[row r][32 .. 37] (s = 2).
struct ObsFrag { f32x2 v[11]; };

__device__ __forceinline__ void actor_fetch(ObsFrag& f, const float* __restrict__ obs, int N, int tile, int r, int h) {
  // branch-free: the row is clamped (a ragged tile's extra lanes are never stored) and the s = 2
  // loads of h = 1 lanes repeat the h = 0 columns (zeroed at conversion); 8-B aligned float2 loads
  const int row = min(tile * 32 + r, N - 1);
  const f32x2* p = (const f32x2*)(obs + (size_t)row * ACT_OBS);
#pragma unroll
  for (int i = 0; i < 4; ++i) f.v[i] = p[4 * h + i];            // columns 8h .. 8h + 7
#pragma unroll
  for (int i = 0; i < 4; ++i) f.v[4 + i] = p[8 + 4 * h + i];    // columns 16 + 8h .. 23 + 8h
#pragma unroll
  for (int i = 0; i < 3; ++i) f.v[8 + i] = p[16 + i];           // columns 32 .. 37
}

__device__ __forceinline__ bf16x8 to_bf16x8(f32x2 a, f32x2 b, f32x2 c, f32x2 d) {
  const u32x4 u = {cvt_pk_bf16(a.x, a.y), cvt_pk_bf16(b.x, b.y), cvt_pk_bf16(c.x, c.y), cvt_pk_bf16(d.x, d.y)};
  return __builtin_bit_cast(bf16x8, u);
}

// Persistent: one workgroup per CU stages W2 (128 KB), W1' (20 KB), b2 and W3 in LDS once; then each
// wave independently walks 32-observation tiles (no block barriers in the loop), fetching the next
// tile's observations into registers while the current tile computes.  The LDS weight fragments are
// double-buffered in registers one k-step (4 MFMAs) ahead of their use.
__global__ void __launch_bounds__(64 * ACT_WAVES) __attribute__((amdgpu_waves_per_eu(2, 2))) actor_kernel(int N, const float* __restrict__ obs,
                                                               float* __restrict__ act, ActorDev A) {
  __shared__ bf16x8 s_w2[ACT_H * ACT_H / 8];   // 128 KB: the permuted W2 fragments
  __shared__ bf16x8 s_w1[ACT_H * ACT_K / 8];   // 20 KB
  __shared__ float4 s_b2[ACT_H / 4];
  __shared__ bf16x8 s_w3[3 * 8 * 2 * 2 * 4];   // 1 KB of W3' rows 0-3, then 2 KB of zeros read by rows 4-31
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, r = l & 31, h = l >> 5;
  APROF_RT(14);
  APROF(0);
  // W2 and W1' straight into LDS (global_load_lds, 16 B per lane = 1 KB per wave-instruction, all of a
  // wave's in flight together; the barrier below drains them)
#pragma unroll
  for (int i = 0; i < ACT_H * ACT_K / 8 / 64; i += ACT_WAVES) {
    const int chunk = i + wave;
    if (chunk < ACT_H * ACT_K / 8 / 64)
      __builtin_amdgcn_global_load_lds((const void*)(A.w1p + 64 * chunk + l),
                                       (__attribute__((address_space(3))) void*)(s_w1 + 64 * chunk), 16, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < ACT_H * ACT_H / 8 / 64; i += ACT_WAVES) {
    const int chunk = i + wave;
    __builtin_amdgcn_global_load_lds((const void*)(A.w2p + 64 * chunk + l),
                                     (__attribute__((address_space(3))) void*)(s_w2 + 64 * chunk), 16, 0, 0);
  }
  for (int i = tid; i < ACT_H / 4; i += 64 * ACT_WAVES) s_b2[i] = ((const float4*)A.b2)[i];
  for (int i = tid; i < 3 * 8 * 2 * 2 * 4; i += 64 * ACT_WAVES) s_w3[i] = i < 8 * 2 * 2 * 4 ? A.w3p[i] : (bf16x8){};
  const float b30 = A.b3[0], b31 = A.b3[1];
  // contiguous tile ranges per workgroup (the split stays within one tile per CU), round-robin over waves
  const int ntile = (N + 31) / 32;
  const int t_end = (int)((long long)ntile * (blockIdx.x + 1) / gridDim.x);
  int tile = (int)((long long)ntile * blockIdx.x / gridDim.x) + wave;
  ObsFrag cur;
  if (tile < t_end) actor_fetch(cur, obs, N, tile, r, h);
  __syncthreads();
  APROF(1);
  int ntiles_done = 0;
  // lane (r, h)'s A-fragment addresses: W1' row 32p + r (stride 5 fragments), W2 (o, q, s2) blocks
  const bf16x8* w1_lane = s_w1 + r * (ACT_K / 8);
  const bf16x8* w2_lane = s_w2 + l;
  // W3' fragment (o, s2) of lane (r, h) at [8(2o + s2) + 4h + r]; rows 4-31 read the zero block instead
  const bf16x8* w3_lane = s_w3 + (r < 4 ? 4 * h + r : 8 * 2 * 2 * 4);
  for (; tile < t_end; tile += ACT_WAVES) {
    // the LDS weight fragments are tile-invariant: without this clobber LICM hoists them all out of
    // the loop (hundreds of registers) and the kernel spills
    asm volatile("" ::: "memory");
    bf16x8 xf[3];
    xf[0] = to_bf16x8(cur.v[0], cur.v[1], cur.v[2], cur.v[3]);
    xf[1] = to_bf16x8(cur.v[4], cur.v[5], cur.v[6], cur.v[7]);
    xf[2] = to_bf16x8(cur.v[8], cur.v[9], cur.v[10], (f32x2){1.0f, 1.0f});
    if (h) xf[2] = (bf16x8){};
    if (tile + ACT_WAVES < t_end) actor_fetch(cur, obs, N, tile + ACT_WAVES, r, h);   // lands during this tile
    // layer 1 in two halves of 4 accumulator tiles (64 registers live) over 3 k-steps, A fragments
    // one k-step ahead; each half's ReLU output is converted in registers to layer-2 B fragments
    // (register 8 s2 + j of tile p is hidden unit 32p + 16 s2 + 8(j>>2) + 4h + (j&3), the k order w2p
    // was permuted into); the ReLU runs on the packed bf16 bits (v_pk_max_i16: a negative bf16 is a
    // negative int16)
    bf16x8 hf[8][2];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      f32x16 acc[4];
      bf16x8 a1[2][4];
#pragma unroll
      for (int p = 0; p < 4; ++p) a1[0][p] = w1_lane[32 * (4 * half + p) * (ACT_K / 8) + h];
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        if (s < 2) {
#pragma unroll
          for (int p = 0; p < 4; ++p)
            a1[(s + 1) & 1][p] = w1_lane[32 * (4 * half + p) * (ACT_K / 8) + (s == 0 ? 2 + h : 4)];
        }
#pragma unroll
        for (int p = 0; p < 4; ++p)
          acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[s & 1][p], xf[s], s == 0 ? (f32x16){} : acc[p], 0, 0, 0);
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        hf[4 * half + p][0] = relu_bf16x8<0>(acc[p]);
        hf[4 * half + p][1] = relu_bf16x8<1>(acc[p]);
      }
    }
    // layer 2 in two halves of 4 output tiles (64 accumulator registers live, not 128), 16 k-steps
    // each with the next k-step's 4 A fragments in flight, the accumulators starting from b2; each
    // half's relu(H2) is packed to bf16 B fragments and fed straight into layer 3
    f32x16 acc3 = {};
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      f32x16 acc2[4];
#pragma unroll
      for (int o = 0; o < 4; ++o) {   // register reg of tile o is hidden unit 32o + (reg&3) + 8(reg>>2) + 4h
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const float4 b = s_b2[(32 * (4 * half + o) + 8 * q4 + 4 * h) / 4];
          acc2[o][4 * q4] = b.x; acc2[o][4 * q4 + 1] = b.y; acc2[o][4 * q4 + 2] = b.z; acc2[o][4 * q4 + 3] = b.w;
        }
      }
      bf16x8 a2[2][4];
#pragma unroll
      for (int o = 0; o < 4; ++o) a2[0][o] = w2_lane[(4 * half + o) * 8 * 2 * 64];
#pragma unroll
      for (int ks = 0; ks < 16; ++ks) {   // ks = 2q + s2
        if (ks < 15) {
#pragma unroll
          for (int o = 0; o < 4; ++o) a2[(ks + 1) & 1][o] = w2_lane[((4 * half + o) * 16 + ks + 1) * 64];
        }
#pragma unroll
        for (int o = 0; o < 4; ++o)
          acc2[o] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2[ks & 1][o], hf[ks >> 1][ks & 1], acc2[o], 0, 0, 0);
      }
      // layer 3 over this half's 128 hidden units (8 k-steps); W3' fragments are zero past row 3
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        acc3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w3_lane[((4 * half + o) * 2 + 0) * 8], relu_bf16x8<0>(acc2[o]), acc3, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w3_lane[((4 * half + o) * 2 + 1) * 8], relu_bf16x8<1>(acc2[o]), acc3, 0, 0, 0);
      }
    }
    // mu^T rows 0-3 sit in registers 0-3 of the h = 0 lanes (column r = this lane's observation)
    const int row = tile * 32 + r;
    if (row < N && h == 0) {
      // deterministic SAC action tanh(mu), then BasePolicy.unscale_action for Box(-1, 1) in float32:
      // low + 0.5 * (a + 1) * (high - low)
      const float m0 = acc3[0] + acc3[2], m1 = acc3[1] + acc3[3];
      const float a0 = tanhf(m0 + b30), a1v = tanhf(m1 + b31);
      *(f32x2*)&act[2 * (size_t)row] = (f32x2){-1.0f + ((0.5f * (a0 + 1.0f)) * 2.0f), -1.0f + ((0.5f * (a1v + 1.0f)) * 2.0f)};
    }
    ++ntiles_done;
    if (ntiles_done < 6) APROF(1 + ntiles_done);
  }
  APROF_RT(15);
  (void)ntiles_done;
}

// ------------------------------------------------------------------ reference-precision (fp32) actor
// The same SB3 MlpPolicy actor in float32 throughout (fp32 FMAs, fp32 tanh): the precision of the reference's
// model.predict (PyTorch fp32), up to summation order -- |delta action| ~1e-6 against a PyTorch fp32 forward.
// One 256-thread workgroup per 32-observation tile: thread t owns hidden unit t for the tile's 32 rows (32
// accumulators), the tile's observations / ReLU'd activations sit in LDS and are read as broadcasts, the
// weights are read transposed ([k][unit], one coalesced 1 KB row per k, L2-resident), layer 3 on 64 lanes.
// VALU-bound: 151 kFLOP per observation (~2x the bf16 MFMA kernel's time at the fp32 vector peak).
struct ActorF32 {
  const float* w1t;   // [38][256]  W1 transposed
  const float* b1;    // [256]
  const float* w2t;   // [256][256] W2 transposed
  const float* b2;    // [256]
  const float* w3;    // [2][256]   mu.weight
  const float* b3;    // [2]
};
// ------------------------------------------------------------------ reference-precision actor on the f32 MFMA
// The float32 actor (SB3 MlpPolicy: ReLU(W2 ReLU(W1 x + b1) + b2), mu = W3 h + b3, tanh, unscale_action) on
// v_mfma_f32_32x32x2_f32: exact f32 products accumulated as an fmaf chain (bitwise, MI355X_MICROARCH.md
// "FP32-input MFMA"), so the result is the fp32 kernel's up to summation order.  One wave = 32 observations
// (batch on the MFMA N dimension, lane r = l & 31 owns observation r, lane half h = l >> 5):
//   layer 1  H1^T[256 x 32] = W1[256 x 38] . X^T: 8 unit tiles x 19 k-steps; A = W1^T[2s + h][32t + r] (global,
//            coalesced per half), B = X[row r][2s + h] (global);
//   layer 2  H2^T = W2 . relu(H1^T + b1): the layer-1 accumulators are the B operands in place -- k-step
//            (t, q) takes register q of tile t, i.e. hidden unit u = 32t + (q & 3) + 8(q >> 2) + 4h on half h
//            (the 32x32 C/D map) -- and A = W2^T[u][32t' + r] is read from global (L2-resident, coalesced per
//            half): 128 k-steps x 8 output tiles;
//   layer 3  mu_i = W3[i] . relu(H2^T + b2) + b3: per-lane partial sums over the lane's 128 hidden values, the
//            two lane halves added with a cross-half swap, then tanh / unscale_action in f32.
// 1024 + 152 MFMAs of 64 cycles per 32 observations: the f32 matrix rate is the f32 vector rate, and
// the MFMA needs one VGPR per operand where the VALU kernel re-read every activation from LDS.
#define AM_WAVES 4
__global__ void __launch_bounds__(64 * AM_WAVES) __attribute__((amdgpu_waves_per_eu(1)))
actor_mfma32_kernel(int N, const float* __restrict__ obs, float* __restrict__ act, ActorF32 A) {
  __shared__ float s_b1[ACT_H], s_b2[ACT_H], s_w3[2 * ACT_H];
  for (int i = threadIdx.x; i < ACT_H; i += 64 * AM_WAVES) { s_b1[i] = A.b1[i]; s_b2[i] = A.b2[i]; }
  for (int i = threadIdx.x; i < 2 * ACT_H; i += 64 * AM_WAVES) s_w3[i] = A.w3[i];
  __syncthreads();
  const int l = threadIdx.x & 63, r = l & 31, h = l >> 5;
  const int tile = blockIdx.x * AM_WAVES + (threadIdx.x >> 6);
  const int row0 = tile * 32;
  if (row0 >= N) return;
  const int row = row0 + r;
  const float* xr = obs + (size_t)(row < N ? row : N - 1) * ACT_OBS;
  f32x16 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = (f32x16){};
  // layer 1
#pragma unroll
  for (int s = 0; s < ACT_OBS / 2; ++s) {
    const float b = xr[2 * s + h];
    const float* w = A.w1t + (size_t)(2 * s + h) * ACT_H + r;
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(w[32 * t], b, acc[t], 0, 0, 0);
  }
  f32x16 hid[8];   // relu(H1 + b1) as layer 2's B operands
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int u = 32 * t + (q & 3) + 8 * (q >> 2) + 4 * h;
      hid[t][q] = fmaxf(acc[t][q] + s_b1[u], 0.0f);
    }
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = (f32x16){};
  // layer 2
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int u = 32 * t + (q & 3) + 8 * (q >> 2) + 4 * h;
      const float* w = A.w2t + (size_t)u * ACT_H + r;
      const float b = hid[t][q];
#pragma unroll
      for (int o = 0; o < 8; ++o) acc[o] = __builtin_amdgcn_mfma_f32_32x32x2f32(w[32 * o], b, acc[o], 0, 0, 0);
    }
  // layer 3: partial sums of this lane's half, then the two halves of the observation added
  float m0 = 0.0f, m1 = 0.0f;
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int u = 32 * t + (q & 3) + 8 * (q >> 2) + 4 * h;
      const float v = fmaxf(acc[t][q] + s_b2[u], 0.0f);
      m0 = fmaf(s_w3[u], v, m0);
      m1 = fmaf(s_w3[ACT_H + u], v, m1);
    }
  m0 += __shfl_xor(m0, 32);
  m1 += __shfl_xor(m1, 32);
  if (h == 0 && row < N) {
    const float a0 = tanhf(m0 + A.b3[0]), a1 = tanhf(m1 + A.b3[1]);
    *(f32x2*)&act[2 * (size_t)row] = (f32x2){-1.0f + ((0.5f * (a0 + 1.0f)) * 2.0f), -1.0f + ((0.5f * (a1 + 1.0f)) * 2.0f)};
  }
}

#define AF_TILE 32
__global__ void __launch_bounds__(256) actor_fp32_kernel(int N, const float* __restrict__ obs, float* __restrict__ act,
                                                         ActorF32 A) {
  __shared__ float4 xs[ACT_OBS][AF_TILE / 4];   // observations, [feature][row]
  __shared__ float4 hs[ACT_H][AF_TILE / 4];     // relu(H1) then relu(H2), [unit][row]
  const int t = threadIdx.x;
  const float b1 = A.b1[t], b2 = A.b2[t];
  for (int tile = blockIdx.x; tile * AF_TILE < N; tile += gridDim.x) {
    const int row0 = tile * AF_TILE;
    float* xf = (float*)xs;
    for (int i = t; i < AF_TILE * ACT_OBS; i += 256) {
      const int o = i / ACT_OBS, k = i - o * ACT_OBS;
      xf[k * AF_TILE + o] = row0 + o < N ? obs[(size_t)row0 * ACT_OBS + i] : 0.0f;
    }
    __syncthreads();
    float acc[AF_TILE];
#pragma unroll
    for (int o = 0; o < AF_TILE; ++o) acc[o] = 0.0f;
#pragma unroll 2
    for (int k = 0; k < ACT_OBS; ++k) {
      const float w = A.w1t[k * ACT_H + t];
#pragma unroll
      for (int q = 0; q < AF_TILE / 4; ++q) {
        const float4 x = xs[k][q];
        acc[4 * q] = fmaf(x.x, w, acc[4 * q]); acc[4 * q + 1] = fmaf(x.y, w, acc[4 * q + 1]);
        acc[4 * q + 2] = fmaf(x.z, w, acc[4 * q + 2]); acc[4 * q + 3] = fmaf(x.w, w, acc[4 * q + 3]);
      }
    }
#pragma unroll
    for (int q = 0; q < AF_TILE / 4; ++q)
      hs[t][q] = make_float4(fmaxf(acc[4 * q] + b1, 0.0f), fmaxf(acc[4 * q + 1] + b1, 0.0f),
                             fmaxf(acc[4 * q + 2] + b1, 0.0f), fmaxf(acc[4 * q + 3] + b1, 0.0f));
    __syncthreads();
#pragma unroll
    for (int o = 0; o < AF_TILE; ++o) acc[o] = 0.0f;
#pragma unroll 4
    for (int k = 0; k < ACT_H; ++k) {
      const float w = A.w2t[k * ACT_H + t];
#pragma unroll
      for (int q = 0; q < AF_TILE / 4; ++q) {
        const float4 x = hs[k][q];
        acc[4 * q] = fmaf(x.x, w, acc[4 * q]); acc[4 * q + 1] = fmaf(x.y, w, acc[4 * q + 1]);
        acc[4 * q + 2] = fmaf(x.z, w, acc[4 * q + 2]); acc[4 * q + 3] = fmaf(x.w, w, acc[4 * q + 3]);
      }
    }
    __syncthreads();   // every lane has read relu(H1)
#pragma unroll
    for (int q = 0; q < AF_TILE / 4; ++q)
      hs[t][q] = make_float4(fmaxf(acc[4 * q] + b2, 0.0f), fmaxf(acc[4 * q + 1] + b2, 0.0f),
                             fmaxf(acc[4 * q + 2] + b2, 0.0f), fmaxf(acc[4 * q + 3] + b2, 0.0f));
    __syncthreads();
    if (t < 2 * AF_TILE) {
      const int o = t >> 1, i = t & 1;
      const float* hf = (const float*)hs;
      float m = 0.0f;
      for (int k = 0; k < ACT_H; ++k) m = fmaf(A.w3[i * ACT_H + k], hf[k * AF_TILE + o], m);
      const float a = tanhf(m + A.b3[i]);
      if (row0 + o < N) act[2 * (size_t)(row0 + o) + i] = -1.0f + ((0.5f * (a + 1.0f)) * 2.0f);   // unscale_action
    }
    __syncthreads();   // xs / hs are reused by the next tile
  }
}

}  // namespace nascar
