// mlp_core.h — the notebooks' policy / value network body on gfx950 MFMA
// (Actor_Critic_PPO.ipynb:376-424): packed-parameter layout, the per-layer
// MFMA tiles (f32, or f16x3 split operands), LayerNorm + ReLU, the last layer
// and the actor's sampling.  Shared by dd_mlp_forward (policy_mlp.hip) and the
// fused policy rollout (policy_rollout.hip), so both evaluate the network bit
// for bit alike.  The design notes are policy_mlp.hip's header.
#pragma once

#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>

#include "dronestep.h"
#include "philox.h"

namespace dd {
namespace mlp {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kIn = DD_OBS_DIM;  // 15
constexpr int kWaves = 8;  // per block (one block per CU); 12 measured 18.5 -> 22.7 us
constexpr int kThreads = kWaves * 64;
constexpr int kCols = 32;  // drones per wave tile

// k-steps of 2 per layer (K = 16 for the 15 inputs + one zero column).
constexpr int kSteps1 = 8, kSteps2 = 64, kSteps3 = 64;
// Packed buffer (floats).  A sections are [out tile][k-step group of 4][lane][4]
// (DD_MLP_F32) or, in the same space, [out tile][k-step of 16][hi | lo'][lane][8
// halves] (DD_MLP_F16X3, pack_a16); the vector sections are shared.
constexpr int kA1 = 0;
constexpr int kA2 = kA1 + 4 * kSteps1 * 64;
constexpr int kA3 = kA2 + 4 * kSteps2 * 64;
constexpr int kV1 = kA3 + 2 * kSteps3 * 64;  // bias, LN weight, LN bias [3][128]
constexpr int kV2 = kV1 + 3 * 128;
constexpr int kV3 = kV2 + 3 * 128;  // [3][64]
constexpr int kW4 = kV3 + 3 * 64;   // last layer [3][64], rows >= K zero
constexpr int kB4 = kW4 + 3 * 64;   // bias [3], then kFold
constexpr int kFold = kB4 + 3;      // DD_MLP_F16X3: bit L set = LayerNorm L folded (policy_mlp.hip fold_kernel)
constexpr int kTag = kB4 + 4;       // layout tag [4]: pack_tag(compute, K), then the three LayerNorms' eps
constexpr int kEps = kTag + 1;      // eps of LayerNorm 1, 2, 3 (DD_MLP_F16X3: scaled, below)
constexpr int kPacked = kTag + 4;
constexpr size_t kLdsBytes = kPacked * sizeof(float);
static_assert(kPacked % 4 == 0, "packed buffer is read as float4");

// What dd_mlp_pack wrote the buffer for: the A sections' arithmetic
// (DD_MLP_*) and the output width K, as the payload of a quiet NaN (0xDF:
// the late round-5 layout, LayerNorm outputs at per-layer scales below 1).
__host__ __device__ constexpr uint32_t pack_tag(int compute, int out_dim) {
    return 0x7FC0DF00u | ((uint32_t)compute << 4) | (uint32_t)out_dim;
}

// Float4 i of the packed buffer on its way into LDS.  The fragment holding
// the last layer's bias and the LayerNorm eps arrives as NaNs when the
// buffer's tag is not the launch's (packed for another compute or K): every
// output (probability, log-probability, value) comes out NaN instead of a
// number from misread weights.  (A NaN eps alone would not do: ReLU's fmax
// turns the NaN activations into zeros.)
__device__ __forceinline__ f32x4 packed_fragment(const f32x4* src4, int i, uint32_t tag) {
    f32x4 v = src4[i];
    if (i == kB4 / 4 && __float_as_uint(src4[kTag / 4].x) != tag) {
        const float q = __builtin_nanf("");
        v = f32x4{q, q, q, q};
    }
    return v;
}

// The three hidden Linears are packed mean-centred over their outputs
// (policy_mlp.hip weight_at), so the LayerNorm that follows each skips its
// mean pass (the plain weights with a two-pass LayerNorm: 18.6 vs 17.6 us).
constexpr bool kCentered = true;

// Hidden row held in register r of accumulator tile t by lane half h
// (C/D map of the 32x32 MFMAs on gfx950: row = (r&3) + 8(r>>2) + 4h).
__host__ __device__ constexpr int hid(int t, int r, int h) { return 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h; }

// ---- DD_MLP_F16X3: split operands on the f16 MFMA --------------------------
// Every operand is split a = hi + lo, hi = f16(a), lo = f16(a - hi), both
// rounded to nearest-even (a - hi is exact in f32), and a product is
// hi.hi + hi.lo + lo.hi + O(2^-22): three f16 MFMAs per k-step, each
// product exact, all three accumulated into ONE f32 accumulator that starts
// at the Linear's bias — no per-layer rescale pass (round 4's lo' = (a -
// hi) 2^11 needed the cross terms in their own pass, scaled back by 2^-11
// with one FMA per accumulator register: 160 VALU per tile).  The operands
// are scaled by powers of two, which every LayerNorm removes exactly (LN(c x)
// = LN(x) with eps c^2):
//   * hidden weights x kWScale and the layer-1 input x kInScale (in
//     registers), so that their lo halves stay clear of the f16 subnormals;
//   * each LayerNorm's output x kActScale (its weight and bias, packed);
//     ReLU then happens in the split (split_pair_relu): hi rounded toward
//     zero and raised to 0, lo = the residual clamped to [0, 1] (the FMA's
//     clamp modifier), 160 v_max fewer per tile.  Late round 5 tried scaling
//     the outputs below 1 instead, so that ReLU is the affine FMA's clamp:
//     faster still, but the activations' lo halves then sit in the f16
//     subnormals, and a layer whose LayerNorm weights spread over 10^-2..10
//     lost ten times f32's accuracy;
//   * each Linear's bias x kWScale x (its input's scale), each LayerNorm's
//     eps x (that product)^2 (kEps), the last Linear's weights / the last
//     act_scale.
// Operand range: |weights| < 2047 before centring (< 4094 after; MlpNet,
// dronestep.h and fold_kernel check the first), |observations| < 1023
// (f16's 65504).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr float kWScale = 16.0f;    // 2^4
constexpr float kInScale = 64.0f;   // 2^6
constexpr float kActScale = 16.0f;  // 2^4

typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// Two floats -> packed f16 hi and lo halves, each rounded to nearest-even
// (v_cvt_pk_f16_f32).  (Truncating instead, v_cvt_pkrtz, biases lo and
// quadruples the end-to-end error: tools/mlp_split_sim.py --truncate.)  The
// residual a - hi is one v_fma_mix_f32 per element, fma(-hi, 1, a) with hi
// read as f16 straight from the packed register (exact): v_cvt_pk_f16_f32,
// two v_fma_mix_f32, v_cvt_pk_f16_f32 = 4 VALU per pair.
__device__ __forceinline__ void split_pair(float a, float b, uint32_t& hi, uint32_t& lo) {
    uint32_t hp = __builtin_bit_cast(uint32_t, f16x2{(_Float16)a, (_Float16)b});
    asm("" : "+v"(hp));  // widen hi from the packed register (else each half is converted twice)
    f32x2 r;
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r.x) : "v"(hp), "v"(a));
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r.y) : "v"(hp), "v"(b));
    const f16x2 l = {(_Float16)r.x, (_Float16)r.y};
    hi = hp;
    lo = __builtin_bit_cast(uint32_t, l);
}

// split_pair of ReLU(a), ReLU(b), for a LayerNorm's outputs: hi = f16(x)
// rounded toward zero (v_cvt_pkrtz_f16_f32) and raised to 0 (v_pk_max_f16), so
// that for x >= 0 the residual x - hi is >= 0 and for x < 0 it is x itself;
// lo = f16(clamp(x - hi, 0, 1)) (the residual is below 1: x < 2^11 ulp), 0 for
// every x < 0.  RNE on the residual keeps lo unbiased; hi + lo then carries
// about one bit less than split_pair's (tools/mlp_split_sim.py: the notebook
// actor within 4.8e-7 of float64 against 4.4e-7).  4 VALU per pair, the ReLU
// included (it cost two v_max).
__device__ __forceinline__ void split_pair_relu(float a, float b, uint32_t& hi, uint32_t& lo) {
    f16x2 h = __builtin_bit_cast(f16x2, __builtin_amdgcn_cvt_pkrtz(a, b));
    h = __builtin_elementwise_max(h, f16x2{(_Float16)0.0f, (_Float16)0.0f});
    uint32_t hp = __builtin_bit_cast(uint32_t, h);
    asm("" : "+v"(hp));
    f32x2 r;
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0] clamp" : "=v"(r.x) : "v"(hp), "v"(a));
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0] clamp" : "=v"(r.y) : "v"(hp), "v"(b));
    const f16x2 l = {(_Float16)r.x, (_Float16)r.y};
    hi = hp;
    lo = __builtin_bit_cast(uint32_t, l);
}

// Eight consecutive activations (one B fragment of a k-step) -> hi, lo'.
template <bool kRelu = false>
__device__ __forceinline__ void split8(const float* v, f16x8& hi, f16x8& lo) {
    u32x4 h, l;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        uint32_t a, b;
        if constexpr (kRelu)
            split_pair_relu(v[2 * m], v[2 * m + 1], a, b);
        else
            split_pair(v[2 * m], v[2 * m + 1], a, b);
        h[m] = a;
        l[m] = b;
    }
    hi = __builtin_bit_cast(f16x8, h);
    lo = __builtin_bit_cast(f16x8, l);
}

// out^T tiles (NT of 32 rows) = bias + W . in^T over STEPS k-steps; bval(q)
// is the lane's B operand (its column's input at the k of step q); bias_h =
// the layer's bias + 4h (this lane half's rows).
template <int NT, int STEPS, typename BVal>
__device__ __forceinline__ void layer_mfma(const f32x4* __restrict__ a4, int lane, BVal bval, f32x16 (&acc)[NT],
                                           const float* bias_h) {
#pragma unroll
    for (int t = 0; t < NT; ++t)  // the bias is the accumulator's initial value
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = bias_h[hid(t, r, 0)];
#pragma unroll
    for (int g = 0; g < STEPS / 4; ++g) {
        f32x4 a[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) a[t] = a4[(t * (STEPS / 4) + g) * 64 + lane];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float b = bval(4 * g + j);
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t][j], b, acc[t], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep each group's LDS reads next to its MFMAs
    }
}

// The bias as an accumulator's initial value (the lane half's rows).
template <int NT>
__device__ __forceinline__ void bias_init(f32x16 (&acc)[NT], const float* bias_h) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = bias_h[hid(t, r, 0)];
}

// The three f16 MFMAs of one k-step into NT out tiles' accumulators: the two
// small cross terms, then hi.hi.  kWide: each term over the tiles in turn, so
// that consecutive MFMAs write different accumulators (NT hi fragments live);
// otherwise tile by tile (the fused policy rollout, at its register cap).
// blk(t): tile t's k-step fragment block [hi | lo][lane] (each A fragment
// read once).
template <int NT, bool kWide, typename Blk>
__device__ __forceinline__ void mfma3(Blk blk, int lane, const f16x8& bh, const f16x8& bl, f32x16 (&acc)[NT]) {
    if constexpr (!kWide) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const f16x8 ah = __builtin_bit_cast(f16x8, blk(t)[lane]);
            const f16x8 al = __builtin_bit_cast(f16x8, blk(t)[64 + lane]);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[t], 0, 0, 0);
        }
        return;
    }
    f16x8 ah[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        ah[t] = __builtin_bit_cast(f16x8, blk(t)[lane]);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t], bl, acc[t], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, blk(t)[64 + lane]), bh, acc[t], 0,
                                                        0, 0);
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t], bh, acc[t], 0, 0, 0);
}

// out^T tiles (NT of 32 rows) = bias + W . in^T over KS k-steps of 16.  The
// packed A fragments are [tile][k-step][hi | lo][lane] x 16 B (each A
// fragment read once); bh / bl are the lane's B fragments.
template <int NT, int KS, bool kWide>
__device__ __forceinline__ void layer16(const u32x4* __restrict__ a16, int lane, const f16x8 (&bh)[KS],
                                        const f16x8 (&bl)[KS], f32x16 (&acc)[NT], const float* bias_h) {
    bias_init<NT>(acc, bias_h);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        mfma3<NT, kWide>([&](int t) { return a16 + (t * KS + s) * 128; }, lane, bh[s], bl[s], acc);
        __builtin_amdgcn_sched_barrier(0);  // keep each k-step's LDS reads next to its MFMAs
    }
}

// x + (the same register of the other lane half), i.e. x + __shfl_xor(x, 32),
// as one v_permlane32_swap (gfx950) instead of an LDS permute.  Lanes < 32
// get x_l + x_{l+32}, lanes >= 32 x_{l-32} + x_l: the same sum (IEEE
// addition is commutative).
__device__ __forceinline__ float add_other_half(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// LayerNorm over the column's 32*NT rows (biased variance, as nn.LayerNorm),
// then ReLU.  vec = [Linear bias | LN weight | LN bias] of 32*NT each.  Pairs
// of registers hold adjacent rows, so the arithmetic runs as packed f32
// (v_pk_add / v_pk_fma), in torch's form y = (x * rstd - rstd * mean) *
// weight + bias.  kRelu: kReluMax (v_max), kReluClamp (DD_MLP_F32: the affine
// is one v_fma_f32 per row with the clamp modifier, which is the ReLU because
// dd_mlp_pack scaled the LayerNorm's weight and bias by a power of two that
// keeps every output below 1, act_scale in policy_mlp.hip; the same bits, 160
// v_max fewer per tile) or kReluInSplit (emit gets the affine's output and
// splits it with split_pair_relu).
enum { kReluMax = 0, kReluClamp = 1, kReluInSplit = 2 };
template <int NT, typename Emit, bool kBarrier = true, int kRelu = kReluMax, bool kFold = false>
__device__ __forceinline__ void norm_relu_emit(const f32x16 (&acc)[NT], const float* vec, float eps, int h,
                                               Emit emit) {
    constexpr int kRows = 32 * NT;
    const float* gamma = vec + kRows + 4 * h;
    const float* beta = vec + 2 * kRows + 4 * h;
    float mean = 0.0f;  // centred weights: the column's mean is zero to rounding
    if constexpr (!kCentered) {
        f32x2 s2 = {0.0f, 0.0f};
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 16; r += 2) s2 += f32x2{acc[t][r], acc[t][r + 1]};
        mean = add_other_half(s2.x + s2.y) / (float)kRows;
    }
    const f32x2 m2 = {mean, mean};
    f32x2 q2 = {0.0f, 0.0f};
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
            const f32x2 d = kCentered ? f32x2{acc[t][r], acc[t][r + 1]} : f32x2{acc[t][r], acc[t][r + 1]} - m2;
            q2 = __builtin_elementwise_fma(d, d, q2);
        }
    const float sq = add_other_half(q2.x + q2.y);
    // v_rsq_f32 (1 ulp), what torch's LayerNorm kernels use (rsqrtf), instead
    // of an IEEE sqrt and division: ~28 fewer VALU per LayerNorm
    const float rstd = __builtin_amdgcn_rsqf(sq / (float)kRows + eps);
    const f32x2 rs2 = {rstd, rstd}, nb2 = {-rstd * mean, -rstd * mean};
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        float y[16];
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
            const int row = hid(t, r, 0);  // rows row, row + 1 (r even)
            const f32x2 g = *reinterpret_cast<const f32x2*>(gamma + row);
            const f32x2 b = *reinterpret_cast<const f32x2*>(beta + row);
            const f32x2 xn = __builtin_elementwise_fma(f32x2{acc[t][r], acc[t][r + 1]}, rs2, nb2);
            if constexpr (kRelu == kReluClamp) {  // ReLU = clamp to [0, 1] on outputs < 1: v_fma_f32 ... clamp
                y[r] = __builtin_amdgcn_fmed3f(__builtin_fmaf(xn.x, g.x, b.x), 0.0f, 1.0f);
                y[r + 1] = __builtin_amdgcn_fmed3f(__builtin_fmaf(xn.y, g.y, b.y), 0.0f, 1.0f);
            } else {
                // kFold (DD_MLP_F16X3, policy_mlp.hip fold_kernel): the LayerNorm's weight lives in the
                // next layer's columns and its sign in this layer's rows; b = bias / |weight| x kActScale
                const f32x2 v = kFold ? __builtin_elementwise_fma(f32x2{acc[t][r], acc[t][r + 1]}, rs2 * kActScale, b)
                                      : __builtin_elementwise_fma(xn, g, b);
                y[r] = kRelu == kReluMax ? fmaxf(v.x, 0.0f) : v.x;  // ReLU here or in the split
                y[r + 1] = kRelu == kReluMax ? fmaxf(v.y, 0.0f) : v.y;
            }
        }
        emit(t, y);
        if constexpr (kBarrier) __builtin_amdgcn_sched_barrier(0);  // one tile's parameters in registers at a time
    }
}

template <int NT, int kRelu = kReluMax, bool kFold = false>
__device__ __forceinline__ void norm_relu(const f32x16 (&acc)[NT], const float* vec, float eps, int h,
                                          float (&y)[NT][16]) {
    auto keep = [&](int t, const float (&v)[16]) {
#pragma unroll
        for (int r = 0; r < 16; ++r) y[t][r] = v[r];
    };
    norm_relu_emit<NT, decltype(keep), true, kRelu, kFold>(acc, vec, eps, h, keep);
}

// norm_relu straight into the next layer's split B fragments: k-step s takes
// registers 8(s&1)..+7 of tile s>>1 (hidden rows hid(s>>1, 8(s&1)+j, h)),
// the k order pack_a16 assumes.  No f32 copy of the activations stays live.
template <int NT, bool kFold>
__device__ __forceinline__ void norm_relu_split(const f32x16 (&acc)[NT], const float* vec, float eps, int h,
                                                f16x8 (&bh)[2 * NT], f16x8 (&bl)[2 * NT]) {
    auto emit = [&](int t, const float (&v)[16]) {
        split8<true>(&v[0], bh[2 * t], bl[2 * t]);
        split8<true>(&v[8], bh[2 * t + 1], bl[2 * t + 1]);
    };
    norm_relu_emit<NT, decltype(emit), true, kReluInSplit, kFold>(acc, vec, eps, h, emit);
}

// A no-op hook (mlp_body's mid).
struct NoMid {
    __device__ void operator()() const {}
};

// norm_relu_split of a 128-row layer fused with the next layer: as soon as
// hidden tile t is split, the MFMAs of k-steps 2t and 2t + 1 (which read only
// its fragments) are issued, so the split of tile t + 1 can run in their
// shadow (a wave's own VALU does overlap its own MFMAs; another wave's does
// not: tools/micro/mfma_valu_overlap.hip).  Each accumulator sees the same
// MFMAs in the same order as layer16's, so the result is bit-identical.
template <int NTO, bool kFold>
__device__ __forceinline__ void norm_split_next(const f32x16 (&acc)[4], const float* vec, float eps, int h,
                                                const u32x4* __restrict__ a16n, int lane, f16x8 (&bh)[8],
                                                f16x8 (&bl)[8], f32x16 (&out)[NTO], const float* bias_n) {
    bias_init<NTO>(out, bias_n);
    auto emit = [&](int t, const float (&v)[16]) {
        split8<true>(&v[0], bh[2 * t], bl[2 * t]);
        split8<true>(&v[8], bh[2 * t + 1], bl[2 * t + 1]);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int s = 2 * t + q;
            mfma3<NTO, true>([&](int to) { return a16n + (to * 8 + s) * 128; }, lane, bh[s], bl[s], out);
        }
    };
    norm_relu_emit<4, decltype(emit), false, kReluInSplit, kFold>(acc, vec, eps, h, emit);
}

// p(y) of one Bernoulli factor, probabilities clamped to [eps, 1 - eps]
// as torch's Bernoulli does (probs_to_logits, clamp_probs), whose log_prob
// is log p or log(1 - p) (torch evaluates it as -BCE-with-logits of the
// logit; the two agree to float32 rounding).
// Here the factor's probability itself, p or 1 - p (1 - p rounded once: exact
// for p >= 1/2, else within 2^-24 of it); actor_sample takes ONE logf of the
// three factors' product (each >= FLT_EPSILON, so the product is a normal
// float) instead of a logf per factor (round 2 had already cut a select
// between logf and log1pf that evaluated both, ~90 VALU per tile; one logf
// instead of three: 65,536 rows 12.61 -> 12.46 us, lab A/B).
__device__ __forceinline__ float bernoulli_factor(float p, bool on) {
    const float pc = fminf(fmaxf(p, FLT_EPSILON), 1.0f - FLT_EPSILON);
    return on ? pc : 1.0f - pc;
}


// Linear(64, K) of one tile from its LayerNorm'd layer-3 rows: 32 rows per
// lane half, then the other half's.
template <int K>
__device__ __forceinline__ void head_of(const float* lds, int h, const float (&y3)[2][16], float (&z)[K]) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const float* w = lds + kW4 + k * 64 + 4 * h;
        f32x2 s2 = {0.0f, 0.0f};
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; r += 2)
                s2 = __builtin_elementwise_fma(*reinterpret_cast<const f32x2*>(w + hid(t, r, 0)),
                                               f32x2{y3[t][r], y3[t][r + 1]}, s2);
        z[k] = add_other_half(s2.x + s2.y) + lds[kB4 + k];
    }
}

// The network up to the last layer's outputs z (before the actor's Sigmoid)
// for the 32 drones of one wave tile: lane (c, h) holds column c's inputs
// x[q] = obs[c][2q + h] (DD_MLP_F32, k-steps of 2) or obs[c][8h + q]
// (kSplit, one k-step of 16), zero past column 14.  Every lane ends with z
// of its column.  lds: the packed parameters.  mid() runs between layer 1
// and layer 2 (dd_mlp_forward waits there for layers 2-3 of its LDS image).
// kPipe: layer 1's split runs in the shadow of layer 2's MFMAs and layer 2's
// in that of layer 3's (norm_split_next: 65,536 rows 14.33 -> 13.93 us,
// 262,144 rows 46.25 -> 44.21 us for the 1 -> 2 stage, lab A/B); the fused
// policy rollout, at the register cap, pipelines the 2 -> 3 stage only.  Every
// schedule gives the same bits.
// The DD_MLP_F16X3 layers up to the last LayerNorm's output y3 (ReLU'd),
// kFold: every LayerNorm folded (fold_kernel); straight-line code either way.
template <bool kPipe, bool kFold, typename Mid>
__device__ __forceinline__ void split_layers(const float* lds, int lane, const float (&x)[8], float (&y3)[2][16],
                                             Mid mid) {
    const u32x4* a16 = reinterpret_cast<const u32x4*>(lds);
    const int h = lane >> 5;
    const float eps1 = lds[kEps], eps2 = lds[kEps + 1], eps3 = lds[kEps + 2];
    f32x16 acc4[4];
    f32x16 acc2[2];
    f16x8 b1h[1], b1l[1], bh[8], bl[8];
    float xs[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) xs[q] = x[q] * kInScale;  // exact: a power of two
    split8(xs, b1h[0], b1l[0]);
    layer16<4, 1, kPipe>(a16 + kA1 / 4, lane, b1h, b1l, acc4, lds + kV1 + 4 * h);
    if constexpr (kPipe) {  // layer 1's split in the shadow of layer 2's MFMAs, as 2 -> 3 below
        mid();
        f32x16 acc4b[4];
        norm_split_next<4, kFold>(acc4, lds + kV1, eps1, h, a16 + kA2 / 4, lane, bh, bl, acc4b, lds + kV2 + 4 * h);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc4[t] = acc4b[t];
        norm_split_next<2, kFold>(acc4, lds + kV2, eps2, h, a16 + kA3 / 4, lane, bh, bl, acc2, lds + kV3 + 4 * h);
    } else {  // layer 1's LayerNorm + split, then all of layer 2; layer 2's split in layer 3's shadow
        // (the fused rollout, at the register cap: 11.84 -> 11.60 us per frame for the 2 -> 3 stage,
        // 13 VGPRs spilled; the 1 -> 2 stage as well spilled more and ran slower, lab A/B)
        norm_relu_split<4, kFold>(acc4, lds + kV1, eps1, h, bh, bl);
        mid();
        layer16<4, 8, kPipe>(a16 + kA2 / 4, lane, bh, bl, acc4, lds + kV2 + 4 * h);
        norm_split_next<2, kFold>(acc4, lds + kV2, eps2, h, a16 + kA3 / 4, lane, bh, bl, acc2, lds + kV3 + 4 * h);
    }
    norm_relu<2, kReluMax, kFold>(acc2, lds + kV3, eps3, h, y3);  // into the f32 head: ReLU by v_max
}

template <int K, bool kSplit, bool kPipe = true, typename Mid = NoMid>
__device__ __forceinline__ void mlp_body(const float* lds, int lane, const float (&x)[8], float (&z)[K],
                                         Mid mid = {}) {
    const f32x4* lds4 = reinterpret_cast<const f32x4*>(lds);
    const int h = lane >> 5;
    const float eps1 = lds[kEps], eps2 = lds[kEps + 1], eps3 = lds[kEps + 2];
    f32x16 acc4[4];
    f32x16 acc2[2];
    float y3[2][16];
    if constexpr (kSplit) {
        // the LayerNorms folded or not (fold_kernel, all or none): one uniform
        // branch, each side straight-line code of its own
        if (__builtin_amdgcn_readfirstlane(__float_as_uint(lds[kFold])))
            split_layers<kPipe, true>(lds, lane, x, y3, mid);
        else
            split_layers<kPipe, false>(lds, lane, x, y3, mid);
    } else {
        float y1[4][16], y2[4][16];
        layer_mfma<4, kSteps1>(lds4 + kA1 / 4, lane, [&](int q) { return x[q]; }, acc4, lds + kV1 + 4 * h);
        norm_relu<4, kReluClamp>(acc4, lds + kV1, eps1, h, y1);
        mid();
        layer_mfma<4, kSteps2>(lds4 + kA2 / 4, lane, [&](int q) { return y1[q >> 4][q & 15]; }, acc4,
                               lds + kV2 + 4 * h);
        norm_relu<4, kReluClamp>(acc4, lds + kV2, eps2, h, y2);
        layer_mfma<2, kSteps3>(lds4 + kA3 / 4, lane, [&](int q) { return y2[q >> 4][q & 15]; }, acc2,
                               lds + kV3 + 4 * h);
        norm_relu<2, kReluClamp>(acc2, lds + kV3, eps3, h, y3);
    }
    __builtin_amdgcn_sched_barrier(0);
    head_of<K>(lds, h, y3, z);
}

// The actor's head: Sigmoid probabilities of the last layer's outputs, as
// v_rcp_f32(1 + v_exp_f32(-z log2 e)).  Its error grows with |z|: for
// z < 0, p ~ exp(z) and the rounding of z*log2(e) alone is a relative error
// of about |z| * 2^-24, i.e. ~|z| f32 ulps of p (~20 ulps at z = -15, a
// log-probability error near 1e-6); a few ulps for |z| < 2 (torch's 1 / (1 + expf)
// with an IEEE division and a range-reduced expf costs ~40 more VALU per
// drone: 65,536 rows 13.35 -> 13.09 us, lab A/B).
__device__ __forceinline__ void actor_probs(const float (&z)[3], float (&prob)[3]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {  // Sigmoid
        prob[k] = __builtin_amdgcn_rcpf(1.0f + __expf(-z[k]));
    }
}

// The collection loop's sampling for one drone (Actor_Critic_PPO.ipynb:857-859):
// Bernoulli(probs).sample() as the dd_step bitmask (bit j iff u_j < p_j, u_j
// from Philox4x32-10 keyed by (seed; env, step, 0x5A5A5A5A)) and
// log_prob(actions).sum().
__device__ __forceinline__ void actor_sample(const float (&prob)[3], uint64_t env, uint64_t step, uint64_t seed,
                                             uint32_t& bits, float& lp) {
    uint32_t r[4];
    philox4x32_10((uint32_t)env, (uint32_t)(env >> 32), (uint32_t)step, (uint32_t)(step >> 32) ^ 0x5A5A5A5Au,
                  (uint32_t)seed, (uint32_t)(seed >> 32), r);
    bits = 0;
    float pr = 1.0f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float u = (float)(r[k] >> 8) * 0x1p-24f;  // uniform [0, 1), 24 bits
        const bool on = u < prob[k];
        bits |= on ? (1u << k) : 0u;
        pr *= bernoulli_factor(prob[k], on);
    }
    lp = logf(pr);  // log of the product: the sum of the factors' logs to float32 rounding
    // a NaN probability (packed_fragment's poison) makes the log-probability
    // NaN too: the clamped Bernoulli log-probability alone would hide it
    lp = fmaf(prob[0] + prob[1] + prob[2], 0.0f, lp);
}

}  // namespace mlp
}  // namespace dd
