// policy_mlp.hip — the notebooks' policy and value networks on gfx950 MFMA.
//
// DroneGamerBoi / DroneTeacherBoi (reference Actor_Critic_PPO.ipynb:376-424):
//   Linear(15,128) LayerNorm ReLU  Linear(128,128) LayerNorm ReLU
//   Linear(128,64) LayerNorm ReLU  Linear(64,K)  [Sigmoid for the actor]
// plus the collection loop's Bernoulli(probs).sample() and
// .log_prob(actions).sum(dim=1) (:851-859), for N observation rows per call.
//
// Shape of the work: 26.6k multiply-adds per row against 111 KB of weights
// shared by every row, i.e. three small GEMMs per 32-row tile.  They run on
// v_mfma_f32_32x32x2_f32 (f32 in, f32 accumulate, exact fmaf chains; 157 TF
// dense, the same rate as the f32 VALU): the notebook's model is float32 and
// the kernel keeps its precision.
//
//   * The activations are kept TRANSPOSED (hidden x drones): a wave owns 32
//     drones (the MFMA's N) and each layer is out^T = W . in^T.  A 32x32
//     accumulator tile holds hidden row (r&3) + 8(r>>2) + 4h of column
//     lane&31 in register r (h = lane>>5), which is exactly the B-operand
//     slot of the next layer's k-step (t, r) for k = that row.  So layer to
//     layer the activations never leave the registers; the k order this
//     implies is folded into the weights when they are packed.
//   * LayerNorm of a drone's column reduces over its 128 (64) rows: 64 (32)
//     per lane, then one cross-half shuffle.
//   * The packed weights (A operands in MFMA lane order, 16 B per lane per
//     4 k-steps so one ds_read_b128 feeds four MFMAs) live in LDS, loaded
//     once per block of 8 waves (2 per SIMD, 1 block per CU).
//   * The last layer (64 -> K <= 3) and the sampling run on the VALU.
//
// DD_MLP_F16X3 (opt-in) runs the three hidden GEMMs on the f16 MFMA
// (v_mfma_f32_32x32x16_f16, 16x the f32 MFMA's rate) with every operand
// split in two halves, a = hi + lo (hi = f16(a), lo = f16(a - hi), both
// nearest-even): a . b = hi.hi + hi.lo + lo.hi + O(2^-22), three f16 MFMAs
// per k-step of 16 into one f32 accumulator, products exact, so a dot
// product carries about the f32 path's error (the notebook's actor
// probabilities within 4.8e-7 of float64, f32's 2.8e-7-3.6e-7;
// tools/mlp_split_sim.py).  The operands are scaled by powers of two that the
// LayerNorms remove (mlp_core.h), and each LayerNorm's weight folds into the
// next layer when it can (fold_kernel below): hidden weights |w| < 2047,
// observations |obs| < 1023, LayerNorm outputs below 128.

#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>

#include "dronestep.h"
#include "mlp_core.h"
#include "philox.h"

namespace dd {
namespace mlp {

// W[row][col] of layer 1 (cols >= 15 are the zero padding) or layers 2, 3,
// centred over its output rows (kCentered, mlp_core.h): W - 1 (1^T W) / rows,
// in double, rounded once.  Every layer here feeds a LayerNorm, which only
// sees its input minus the input's mean: with centred weights and bias the
// GEMM's output already has (to rounding) zero mean, and norm_relu_emit skips
// the mean pass.
__device__ __forceinline__ float weight_at(const DDMlpParams& p, int base, int row, int col) {
    if (base == kA1 && col >= kIn) return 0.0f;
    const float* w = base == kA1 ? p.w0 : base == kA2 ? p.w3 : p.w6;
    const int cols = base == kA1 ? kIn : 128, rows = base == kA3 ? 64 : 128;
    if (!kCentered) return w[row * cols + col];
    double sum = 0.0;
    for (int r = 0; r < rows; ++r) sum += (double)w[r * cols + col];
    return (float)((double)w[row * cols + col] - sum / rows);
}

// A Linear bias before a LayerNorm, centred like its weights.
__device__ __forceinline__ float bias_at(const float* b, int rows, int o) {
    if (!kCentered) return b[o];
    double sum = 0.0;
    for (int r = 0; r < rows; ++r) sum += (double)b[r];
    return (float)((double)b[o] - sum / rows);
}

// ---- DD_MLP_F16X3: LayerNorm weights folded into the next layer ----------
// gamma_j (xn_j) + beta_j = |gamma_j| (s_j xn_j + beta_j / |gamma_j|) with s_j
// = sign(gamma_j): s_j goes into row j of the Linear before the LayerNorm (its
// output's square sum, all the LayerNorm takes from it, does not change, and
// the centred weights keep the mean at zero), |gamma_j| into column j of the
// Linear after, and the affine is one FMA per activation instead of two
// (norm_relu_emit kFold).  fold_kernel decides, into the packed slot kFold:
// only when for every LayerNorm every |gamma_j| > 0, |beta_j / gamma_j| <= 64
// (the x16 output stays below 2048, split_pair_relu's bound) and the next
// hidden Linear's weights times max|gamma| stay below 2047 (the f16 range
// after centring and x16); otherwise none is folded.
__device__ __forceinline__ const float* ln_weight(const DDMlpParams& p, int L) {
    return L == 0 ? p.ln1_w : L == 1 ? p.ln4_w : p.ln7_w;
}
__device__ __forceinline__ const float* ln_bias(const DDMlpParams& p, int L) {
    return L == 0 ? p.ln1_b : L == 1 ? p.ln4_b : p.ln7_b;
}

__global__ __launch_bounds__(256) void fold_kernel(DDMlpParams p, float* out) {
    __shared__ float red[3][256];
    uint32_t flags = 0;
    for (int L = 0; L < 3; ++L) {
        const float* g = ln_weight(p, L);
        const float* b = ln_bias(p, L);
        const int rows = L == 2 ? 64 : 128;
        float gmin = INFINITY, gmax = 0.0f, ratio = 0.0f, wmax = 0.0f;
        for (int r = threadIdx.x; r < rows; r += 256) {
            const float a = fabsf(g[r]);
            gmin = fminf(gmin, a);
            gmax = fmaxf(gmax, a);
            ratio = fmaxf(ratio, fabsf(b[r]) / a);  // inf or NaN when a == 0: gmin rules that out
        }
        if (L < 2) {  // the next hidden Linear: [64 or 128][128]
            const float* w = L == 0 ? p.w3 : p.w6;
            const int n = (L == 0 ? 128 : 64) * 128;
            for (int i = threadIdx.x; i < n; i += 256) wmax = fmaxf(wmax, fabsf(w[i]));
        }
        red[0][threadIdx.x] = -gmin;
        red[1][threadIdx.x] = fmaxf(gmax, 0.0f);
        red[2][threadIdx.x] = ratio;
        __syncthreads();
        for (int k = 128; k > 0; k >>= 1) {
            if (threadIdx.x < k)
#pragma unroll
                for (int q = 0; q < 3; ++q) red[q][threadIdx.x] = fmaxf(red[q][threadIdx.x], red[q][threadIdx.x + k]);
            __syncthreads();
        }
        const float gmin_all = -red[0][0], gmax_all = red[1][0], ratio_all = red[2][0];
        __syncthreads();
        red[0][threadIdx.x] = wmax;
        __syncthreads();
        for (int k = 128; k > 0; k >>= 1) {
            if (threadIdx.x < k) red[0][threadIdx.x] = fmaxf(red[0][threadIdx.x], red[0][threadIdx.x + k]);
            __syncthreads();
        }
        const float wmax_all = red[0][0];
        __syncthreads();
        const bool ok = gmin_all > 0.0f && ratio_all <= 64.0f && (L == 2 || wmax_all * gmax_all < 2047.0f);
        flags |= ok ? 1u << L : 0u;
    }
    // all or none: the kernels branch once per tile, between two straight-line bodies
    if (threadIdx.x == 0) out[kFold] = __uint_as_float(flags == 7u ? 7u : 0u);
}

// The packed value's fold factors: s_j for row j of the Linear before
// LayerNorm L (L = the layer's own index), |gamma_j| for column j of the
// Linear after LayerNorm L.
__device__ __forceinline__ bool folded(const float* out, int L) {
    return (__float_as_uint(out[kFold]) >> L) & 1u;
}
__device__ __forceinline__ float row_sign(const DDMlpParams& p, const float* out, int L, int row) {
    return folded(out, L) && ln_weight(p, L)[row] < 0.0f ? -1.0f : 1.0f;
}
__device__ __forceinline__ float col_gain(const DDMlpParams& p, const float* out, int L, int col) {
    return folded(out, L) ? fabsf(ln_weight(p, L)[col]) : 1.0f;
}

// DD_MLP_F16X3 A fragments, one packed float = two halves: section
// [tile][k-step][hi | lo'][lane][8 halves]; lane l of k-step s of out tile t
// holds W[32t + (l&31)][k] for its elements j, k = 8h + j (layer 1) or hidden
// row hid(s>>1, 8(s&1) + j, h) (layers 2, 3: the B fragments split_acts makes).
__device__ __forceinline__ float pack_a16(const DDMlpParams& p, const float* out, int i) {
    const int base = i < kA2 ? kA1 : i < kA3 ? kA2 : kA3;
    const int ks = base == kA1 ? 1 : 8;
    const int o = i - base;
    const int blk = o / 512, w = o % 512;
    const int t = blk / ks, s = blk % ks, part = w / 256, l = (w % 256) / 4, m = w % 4;
    const int row = 32 * t + (l & 31), h = l >> 5;
    float v[2];
    for (int e = 0; e < 2; ++e) {
        const int j = 2 * m + e;
        const int col = base == kA1 ? 8 * h + j : hid(s >> 1, 8 * (s & 1) + j, h);
        const int L = base == kA1 ? 0 : base == kA2 ? 1 : 2;  // this Linear feeds LayerNorm L
        float f = row_sign(p, out, L, row);  // and takes LayerNorm L - 1's outputs
        if (L > 0) f *= col_gain(p, out, L - 1, col);
        v[e] = weight_at(p, base, row, col) * f * kWScale;  // kWScale: exact, a power of two
    }
    uint32_t hi, lo;
    split_pair(v[0], v[1], hi, lo);
    return __uint_as_float(part == 0 ? hi : lo);
}

// DD_MLP_F32: the power of two that scales LayerNorm L's output (its weight
// and bias are packed times it) so that every output stays below 1, which
// makes ReLU the clamp modifier of the affine FMA (mlp_core.h norm_relu_emit).
// A LayerNorm output is gamma * xn + beta with |xn| < sqrt(rows) (the
// normalised column has mean square below 1), so |out| < B = max|gamma|
// sqrt(rows) (1 + 2^-8, for rounding) + max|beta|; with B = m 2^x, m in [0.5,
// 1), the scale is 2^-x.  The next LayerNorm removes it exactly (its eps is
// packed at the scale squared).
__device__ __forceinline__ float act_scale(const DDMlpParams& p, int L) {
    const float* g = L == 0 ? p.ln1_w : L == 1 ? p.ln4_w : p.ln7_w;
    const float* b = L == 0 ? p.ln1_b : L == 1 ? p.ln4_b : p.ln7_b;
    const int rows = L == 2 ? 64 : 128;
    float gm = 0.0f, bm = 0.0f;
    for (int r = 0; r < rows; ++r) {
        gm = fmaxf(gm, fabsf(g[r]));
        bm = fmaxf(bm, fabsf(b[r]));
    }
    const float bound = gm * sqrtf((float)rows) * (1.0f + 0x1p-8f) + bm;
    if (!(bound > 0.0f)) return 1.0f;
    int x;
    frexpf(bound, &x);
    return ldexpf(1.0f, -x);
}

// One packed float: which state_dict element (or zero) goes at index i.
__global__ void pack_kernel(DDMlpParams p, int32_t compute, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kPacked) return;
    const bool split = compute == DD_MLP_F16X3;
    float v = 0.0f;
    if (i < kV1 && compute == DD_MLP_F16X3) {
        v = pack_a16(p, out, i);
    } else if (i < kV1) {  // A operands: lane l of k-step q of out tile t holds W[32t + (l&31)][k(q, l>>5)]
        const int base = i < kA2 ? kA1 : i < kA3 ? kA2 : kA3;
        const int steps = i < kA2 ? kSteps1 : i < kA3 ? kSteps2 : kSteps3;
        const int o = i - base;
        const int j = o & 3, l = (o >> 2) & 63, grp = o >> 8;
        const int t = grp / (steps / 4), q = 4 * (grp % (steps / 4)) + j;
        const int row = 32 * t + (l & 31), h = l >> 5;
        // layer 1: natural k order, column 15 is zero; layers 2, 3: k-step
        // (t', r) = q takes hidden row hid(t', r, h)
        const int col = base == kA1 ? 2 * q + h : hid(q >> 4, q & 15, h);
        v = weight_at(p, base, row, col);
    } else if (i < kW4) {  // [bias | LN weight | LN bias] of layers 1-3
        const int L = i < kV2 ? 0 : i < kV3 ? 1 : 2, rows = L == 2 ? 64 : 128;
        const int o = i - (L == 0 ? kV1 : L == 1 ? kV2 : kV3);
        const float* src[3][3] = {{p.b0, p.ln1_w, p.ln1_b}, {p.b3, p.ln4_w, p.ln4_b}, {p.b6, p.ln7_w, p.ln7_b}};
        v = o < rows ? bias_at(src[L][0], rows, o) : src[L][o / rows][o % rows];
        if (split && o < rows) v *= row_sign(p, out, L, o);                       // folded: the row's sign
        if (split && o >= 2 * rows && folded(out, L)) v /= fabsf(src[L][1][o % rows]);  // beta / |gamma|
        // the bias at its GEMM's scale (weights x input); the LN's affine at its output's
        const float in = L == 0 ? (split ? kInScale : 1.0f) : split ? kActScale : act_scale(p, L - 1);
        v *= o < rows ? (split ? kWScale : 1.0f) * in : split ? kActScale : act_scale(p, L);
    } else if (i < kB4) {
        const int o = i - kW4;
        v = (o / 64) < p.out_dim ? p.w9[o] : 0.0f;
        if (split) v *= col_gain(p, out, 2, o % 64);
        v *= 1.0f / (split ? kActScale : act_scale(p, 2));  // the last LayerNorm's output is scaled
    } else if (i == kFold) {  // fold_kernel's flags (DD_MLP_F16X3), none for f32
        if (!split) out[i] = 0.0f;
        return;
    } else if (i < kTag) {
        const int o = i - kB4;
        v = o < p.out_dim ? p.b9[o] : 0.0f;
    } else if (i == kTag) {
        v = __uint_as_float(pack_tag(compute, p.out_dim));
    } else {  // kEps: each LayerNorm's eps at its input's scale squared
        const float sc = split ? kWScale * (i == kEps ? kInScale : kActScale)
                               : (i == kEps ? 1.0f : act_scale(p, i - kEps - 1));
        v = p.ln_eps * sc * sc;
    }
    out[i] = v;
}

struct FwdArgs {
    const float* obs;
    float* out;
    uint8_t* actions;
    float* log_prob;
    uint64_t seed;
    int64_t step;
    int64_t env_id_base;
    int64_t n;
};

// Layer 1's B operands for lane (c, h) of a tile: obs[d][8h + q] (kSplit) or
// obs[d][2q + h], zero past column 14 and past the last row.
template <bool kSplit>
__device__ __forceinline__ void load_inputs_raw(const FwdArgs& p, int64_t tile, int lane, float (&x)[8]) {
    const int h = lane >> 5;
    const int64_t d = tile * kCols + (lane & 31);
    // branch-free: every lane loads from a valid address (row 0, column 14 for
    // the padding), and mask_inputs zeroes what it does not own, so the loads
    // issue back to back (a guarded load per element put each behind its own
    // branch and a vmcnt(0): four HBM round trips in a row)
    const float* row = p.obs + (d < p.n ? d : 0) * kIn;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int k = kSplit ? 8 * h + q : 2 * q + h;
        x[q] = row[k < kIn ? k : kIn - 1];
    }
}

template <bool kSplit>
__device__ __forceinline__ void mask_inputs(const FwdArgs& p, int64_t tile, int lane, float (&x)[8]) {
    const int h = lane >> 5;
    const bool live = tile * kCols + (lane & 31) < p.n;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int k = kSplit ? 8 * h + q : 2 * q + h;
        x[q] = (live && k < kIn) ? x[q] : 0.0f;
    }
}

template <bool kSplit>
__device__ __forceinline__ void load_inputs(const FwdArgs& p, int64_t tile, int lane, float (&x)[8]) {
    load_inputs_raw<kSplit>(p, tile, lane, x);
    mask_inputs<kSplit>(p, tile, lane, x);
}

// The actor's / critic's outputs of one drone (lane h == 0 of its column).
template <int K>
__device__ __forceinline__ void emit_outputs(const FwdArgs& p, int64_t d, const float (&z)[K]) {
    if constexpr (K == 1) {
        if (p.out) p.out[d] = z[0];
    } else {
        float prob[3];
        actor_probs(z, prob);
        if (p.out) {
#pragma unroll
            for (int k = 0; k < K; ++k) p.out[d * K + k] = prob[k];
        }
        if (p.actions || p.log_prob) {
            uint32_t bits;
            float lp;
            actor_sample(prob, (uint64_t)(p.env_id_base + d), (uint64_t)p.step, p.seed, bits, lp);
            if (p.actions) p.actions[d] = (uint8_t)bits;
            if (p.log_prob) p.log_prob[d] = lp;
        }
    }
}

// The LDS image arrives by LDS-DMA (global_load_lds_dwordx4, 1 KB per
// wave-instruction, the LDS image lane-linear like the packed buffer), issued
// right after the first tile's observation loads and before anything waits:
// layer 1's fragments and the vector sections (13 KB) first, then layers 2-3
// (96 KB, [kA2, kV1)).  A vmcnt that leaves the layer 2-3 pieces in flight
// (they complete in issue order) and the block's first barrier release layer
// 1; the second barrier, after a vmcnt(0), comes between layer 1 and layer 2
// of the first tile, so the big part streams in behind layer 1.  Raw
// s_barrier, not __syncthreads() (whose fence would drain the DMA at the first
// barrier).  A buffer packed for another compute or K (its tag, kTag) gives
// NaN outputs.  Round 5 (65,536 rows, lab A/B on one box): register-staging
// the first 13 KB put its load latency and ds_writes ahead of the DMA issue,
// and the observation's guarded loads went out one HBM round trip at a time
// (13.75 -> 13.16 us with the Sigmoid below; a separate wait for layer 3's
// pieces before layer 3 cost 0.4 us: its branch splits the scheduling region).
constexpr size_t kLdsPad = (size_t)((kPacked + 255) / 256 * 256) * sizeof(float);  // whole 1 KB DMA pieces

// The prologue both forward kernels share: the first tile's observation and
// the DMA of the LDS image, then the wait for layer 1 and the vectors and the
// block's first barrier.  x: the first tile's layer-1 B operands.
template <int kW, bool kSplit>
__device__ __forceinline__ void load_image(const float* __restrict__ packed, f32x4* lds4, const FwdArgs& p,
                                           int64_t tile, int wave, int lane, float (&x)[8]) {
    const int h = lane >> 5;
    f32x4 xa, xb;  // DD_MLP_F16X3's first tile: two unaligned 16 B loads, waited for with the early DMA pieces
    if constexpr (kSplit) {
        // columns 8h .. 8h+7 of the row from base column 7h (in bounds for
        // h = 1; shifted down after the wait).  Inline asm so that hipcc,
        // which waits vmcnt(0) at the first use of an ordinary load left
        // outstanding beside an LDS-DMA, does not track them: the vmcnt
        // below covers them (they are older than every piece).
        // CAUTION: gfx9 has no interlock on a VMEM result, and the
        // compiler does not know these registers are pending until that
        // hand-written s_waitcnt; a codegen that copied, spilled or
        // rematerialised xa / xb before it would read stale data.  Any change
        // of compiler (or of this prologue) must re-run the GPU tests
        // test_observations_at_any_offset and test_actor_probs_match_notebook_model
        // (tests/test_gpu_policy.py), which catch exactly that.
        const int64_t d = tile * kCols + (lane & 31);
        const float* rp = p.obs + (d < p.n ? d : 0) * kIn + 7 * h;
        asm volatile("global_load_dwordx4 %0, %2, off\n\tglobal_load_dwordx4 %1, %2, off offset:16"
                     : "=&v"(xa), "=&v"(xb)
                     : "v"(rp)
                     : "memory");
    } else {
        load_inputs<kSplit>(p, tile, lane, x);
        // the observation is waited for before the DMA issue (see above)
        asm volatile("" ::"v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]));
    }
    constexpr int kChunk = 64 * 4;                                 // floats per wave-instruction
    constexpr int kL1 = kA2 / kChunk;                              // layer 1: 8 pieces
    constexpr int kEarly = kL1 + (kPacked - kV1 + kChunk - 1) / kChunk;  // + the vectors: 5, the last partial
    constexpr int kLate = (kV1 - kA2) / kChunk;                    // layers 2-3: 96 pieces
    static_assert(kA2 % kChunk == 0 && (kV1 - kA2) % kChunk == 0, "DMA pieces");
    static_assert(kLate % kW == 0, "the vmcnt below counts kLate / kW late pieces per wave");
    const int swave = __builtin_amdgcn_readfirstlane(wave);  // uniform: scalar branches, M0 from an SGPR
    // The same number of early pieces per wave, so that every wave's vmcnt
    // below counts alike: waves past the last piece load their first piece
    // again, and the last vector piece's lanes past the buffer read its last
    // float4 into the LDS pad (kLdsPad).
#pragma unroll
    for (int j = 0; j < (kEarly + kW - 1) / kW; ++j) {
        const int q = swave + j * kW < kEarly ? swave + j * kW : swave;
        const int off = q < kL1 ? q * kChunk : kV1 + (q - kL1) * kChunk;
        const int src = off + 4 * lane < kPacked ? off + 4 * lane : kPacked - 4;
        __builtin_amdgcn_global_load_lds(packed + src, lds4 + off / 4, 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < kLate / kW; ++j) {
        const int off = kA2 + (swave + j * kW) * kChunk;
        __builtin_amdgcn_global_load_lds(packed + off + 4 * lane, lds4 + off / 4, 16, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kLate / kW) : "memory");  // this wave's early pieces
    __builtin_amdgcn_s_barrier();
    if constexpr (kSplit) {
        asm volatile("" : "+v"(xa), "+v"(xb));  // after the wait
        const float v[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] = h ? (q < 7 ? v[q + 1] : 0.0f) : v[q];
        mask_inputs<kSplit>(p, tile, lane, x);
    }
}

// The second barrier: layers 2-3 in LDS.
__device__ __forceinline__ void wait_layers23() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

template <int K, bool kSplit>
__global__ __launch_bounds__(kThreads) void mlp_kernel(const float* __restrict__ packed, FwdArgs p) {
    extern __shared__ f32x4 lds4[];
    const float* lds = reinterpret_cast<const float*>(lds4);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, c = lane & 31;
    const int64_t tiles = (p.n + kCols - 1) / kCols;
    int64_t tile = (int64_t)blockIdx.x * kWaves + wave;
    float x[8];
    load_image<kWaves, kSplit>(packed, lds4, p, tile, wave, lane, x);
    const bool tag_ok = __float_as_uint(lds[kTag]) == pack_tag(kSplit ? DD_MLP_F16X3 : DD_MLP_F32, K);
    const auto run_tile = [&](auto mid) {
        const int64_t d = tile * kCols + c;  // this lane's drone (column)
        float z[K];
        mlp_body<K, kSplit>(lds, lane, x, z, mid);
        if (d >= p.n || h != 0) return;
        if (!tag_ok)
#pragma unroll
            for (int k = 0; k < K; ++k) z[k] = __builtin_nanf("");
        emit_outputs<K>(p, d, z);
    };
    const auto layers23 = [] { wait_layers23(); };
    // the first tile apart, with the second barrier between its layers 1 and
    // 2; the loop over the others carries no barrier branch (one would split
    // its scheduling regions)
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    if (tile < tiles) {
        run_tile(layers23);
        for (tile += stride; tile < tiles; tile += stride) {
            load_inputs<kSplit>(p, tile, lane, x);
            run_tile(NoMid{});
        }
    } else {
        layers23();  // a wave without a tile still takes its part in the second barrier
    }
}

template <int K, bool kSplit>
hipError_t launch(const float* packed, const FwdArgs& a, hipStream_t s) {
    // the LDS image exceeds the 64 KB default; the attribute is per device, so
    // it is set on every launch (a cheap host call) rather than once per process
    const hipError_t e = hipFuncSetAttribute((const void*)mlp_kernel<K, kSplit>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsPad);
    if (e != hipSuccess) return e;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    const int64_t tiles = (a.n + kCols - 1) / kCols;
    const int64_t want = (tiles + kWaves - 1) / kWaves;
    const unsigned blocks = (unsigned)(want < cus ? want : cus);  // one block per CU, waves loop over tiles
    hipLaunchKernelGGL((mlp_kernel<K, kSplit>), dim3(blocks), dim3(kThreads), kLdsPad, s, packed, a);
    return hipGetLastError();
}

}  // namespace mlp
}  // namespace dd

extern "C" {

int64_t dd_mlp_packed_floats(void) { return dd::mlp::kPacked; }

int dd_mlp_pack(const DDMlpParams* p, int32_t compute, float* packed, void* stream) {
    if (!p || !packed || !(p->out_dim == 1 || p->out_dim == 3) || !(p->ln_eps > 0.0f)) return hipErrorInvalidValue;
    if (reinterpret_cast<uintptr_t>(packed) & 15u) return hipErrorInvalidValue;  // consumers read 16-byte fragments
    if (compute != DD_MLP_F32 && compute != DD_MLP_F16X3) return hipErrorInvalidValue;
    const float* req[] = {p->w0, p->b0, p->ln1_w, p->ln1_b, p->w3, p->b3, p->ln4_w,
                          p->ln4_b, p->w6, p->b6, p->ln7_w, p->ln7_b, p->w9, p->b9};
    for (const float* q : req)
        if (!q) return hipErrorInvalidValue;
    const int threads = 256, blocks = (dd::mlp::kPacked + threads - 1) / threads;
    if (compute == DD_MLP_F16X3)  // which LayerNorms fold into the next layer, before the packing reads it
        hipLaunchKernelGGL(dd::mlp::fold_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, *p, packed);
    hipLaunchKernelGGL(dd::mlp::pack_kernel, dim3(blocks), dim3(threads), 0, (hipStream_t)stream, *p, compute, packed);
    return hipGetLastError();
}

int dd_mlp_forward(const float* packed, int32_t compute, int32_t out_dim, const DDMlpIO* io, int64_t n,
                   void* stream) {
    if (!io || n < 0 || !(out_dim == 1 || out_dim == 3)) return hipErrorInvalidValue;
    if (compute != DD_MLP_F32 && compute != DD_MLP_F16X3) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    if (!packed || !io->obs) return hipErrorInvalidValue;
    if (reinterpret_cast<uintptr_t>(packed) & 15u) return hipErrorInvalidValue;  // 16-byte fragments / LDS-DMA
    if (out_dim == 1 && (io->actions || io->log_prob)) return hipErrorInvalidValue;  // nothing to sample
    const dd::mlp::FwdArgs a{io->obs, io->out, io->actions, io->log_prob, io->seed, io->step, io->env_id_base, n};
    const hipStream_t s = (hipStream_t)stream;
    if (compute == DD_MLP_F16X3)
        return out_dim == 3 ? dd::mlp::launch<3, true>(packed, a, s) : dd::mlp::launch<1, true>(packed, a, s);
    return out_dim == 3 ? dd::mlp::launch<3, false>(packed, a, s) : dd::mlp::launch<1, false>(packed, a, s);
}

}  // extern "C"
