// bmfr_fused_cols.hip -- fused frame kernel K1, column-split form (default for
// the canonical feature lists with half tmp_data, and with f32 tmp_data under
// fast_fit).
//
// Same computation as k_fused (bmfr_fused.hip): accumulate_noisy_data ->
// min/max scaling -> Householder QR -> back substitution -> weighted_sum ->
// temporal blend (bmfr.cl:287-849), one 256-thread work-group per 32x32 block,
// every value rounded exactly as upstream rounds it.  What differs is who
// holds the design matrix during the fit:
//
//   * phase 1: thread (wave w, lane l) computes the features of rows
//     r = l + 64 j, j = 4w..4w+3, and writes them to an LDS matrix;
//   * fit: wave w takes COLUMNS c = 1 + w, 5 + w, 9 + w, ... -- all 1024 rows
//     of each, lane l holding rows l + 64 j, j = 0..15 (8 packed-half
//     registers per column); one copy of the code serves the four waves.  Upstream's fitter work-item t = l + 64 m owns rows t + 256 s,
//     i.e. j = m + 4 s, so each work-item partial and the first tree step
//     (bmfr.cl:32-33) are in one lane and the rest of the tree runs on DPP /
//     permlane swaps (bmfr_wave.h): every dot product, norm, min and max of
//     the fit is a wave-local exact reduction, no LDS round trip, no barrier.
//   * Householder step c needs only u_c, which the owner of column c publishes
//     in LDS (three buffers) as soon as it has applied step c-1 to that
//     column, ahead of its other columns, and announces with an LDS flag: a
//     wave waits only for the pivot it needs -- no block reduction per dot
//     product and no work-group barrier per column.
//   * phase 3 (weighted sum + blend) per pixel again, rows of phase 1.
//
// The R matrix, back substitution and phase-3 code are k_fused's.  Parity:
// tests/test_gpu_parity.py (fused vs stage kernels bit for bit).
#include <type_traits>
#include <utility>

#include "bmfr_launch.h"
#include "bmfr_taa_tile.h"
#include "bmfr_wave.h"

namespace bmfr {
namespace cols {

// Waves per work-group NW = 4 (the default) or 8: 64 NW threads; in phase 1
// and 3 a thread owns kItems = 16 / NW rows of the block.
template <int NW>
constexpr int threads_of() { return 64 * NW; }
template <int NW>
constexpr int items_of() { return 16 / NW; }
constexpr int kSlots = 16;    // rows per lane per column (row = lane + 64 j)
constexpr int kUStride = 20;     // floats per lane in a u buffer: 16 + 4 (conflict-free 16-byte reads)
constexpr int kPre = 2;          // step-0 noise columns per wave prefetched in phase 1

// Householder vectors in flight: the fit's waves wait for each published
// pivot through an LDS flag instead of a barrier per column, so a buffer is
// reused only once every wave has finished the step that read it.
constexpr int kUBufs = 3;
// Phase 1 -> 3, per thread: the previous accumulated filtered colour of its
// four items (12 floats).  Where the matrix area has room beside the u
// buffers (B >= 16) they wait in registers until the fit has loaded its
// columns and then go there, so the work-group's LDS stays within 40 KB (four
// work-groups per CU); otherwise they have their own LDS array.
constexpr int kKeep = 16 * 3 * 64;  // 12 floats per thread at NW = 4, 6 at NW = 8
// F32: f32 tmp_data (USE_HALF_PRECISION_IN_TMP_DATA 0): the design matrix as
// floats -- twice the registers per column (16 per lane, as 8 float pairs),
// the trailing columns never rounded to half.  Only the rows another wave
// needs pass through LDS: wave w computes row quad w of every column in
// phase 1, and the quad of the columns it owns in the fit stays in its
// registers, so LDS holds 12 of each lane's 16 rows (36 KB at B = 13: four
// work-groups per CU, as with half tmp_data; all 16 would be 48 KB, three).
template <bool F32>
constexpr int m_slots() { return F32 ? kSlots - 4 : kSlots; }
constexpr bool keep_in_m(int B, bool F32 = false) {
    return (B - 1) * 64 * (F32 ? 4 * m_slots<true>() : 2 * kSlots) >= (kUBufs * 64 * kUStride + kKeep) * 4;
}
// What the fit writes for back substitution and phase 3: R[x][y][ch] (x =
// column, as k_fused), the weights, per scaled feature min, max,
// 1/(max-min).  Written only once the fit has loaded its columns.
template <int B>
struct FitOut {
    float R[(B - 2) * (B - 2) * 3];
    float weights[(B - 3) * 3];
    float mm[3 * (B - 3)];
};
template <int B, int NW = 4, bool F32 = false>
struct Lds {
    using MT = std::conditional_t<F32, float, _Float16>;
    static constexpr int kMBytes = (B - 1) * 64 * m_slots<F32>() * (F32 ? 4 : 2);
    static constexpr int kUKBytes = (kUBufs * 64 * kUStride + (keep_in_m(B, F32) ? kKeep : 1)) * 4;
    // FitOut in the matrix area's tail, beside the u buffers (and the kept
    // colours), where it has room
    static constexpr bool kTail = kMBytes - kUKBytes >= (int)sizeof(FitOut<B>);
    union {
        // design matrix after phase 1, column c at M[c - 1], [lane * 16 + j]
        // (half pairs swizzled by lane, see run()); F32: [lane * 12 + 4 q' + j % 4],
        // q' the row quad j / 4 among the three its owner wave does not hold
        MT M[B - 1][64 * m_slots<F32>()];
        struct {
            float u[kUBufs][64 * kUStride];  // Householder vectors, u_c in buffer c % kUBufs
            float keep_m[keep_in_m(B, F32) ? kKeep : 1];
            FitOut<B> fo_tail[kTail ? 1 : 0];
        };
    };
    FitOut<B> fo_own[kTail ? 0 : 1];
    __device__ FitOut<B>& fo() {
        if constexpr (kTail) return fo_tail[0];
        else return fo_own[0];
    }
    float keep_s[keep_in_m(B, F32) ? 1 : kKeep];
    __device__ float* keep() { return keep_in_m(B, F32) ? keep_m : keep_s; }  // [(item * 3 + ch) * 64 NW + t]
    float piv[kUBufs][3];               // |u|^2 and RN(1/|u|^2) (fast_fit: 2 RN(1/|u|^2)) of the published vector; fast_fit: u's pivot element
    int pub;                            // highest published pivot column
    int prog[NW];                       // per wave: the last step it has applied
    int timeout;                        // a flag wait of this block gave up (reported once, at the end)
    int max_polls;                      // Params::max_polls (kept here: read only once a flag is not ready)
    int delay;                          // Params::debug_delay (diagnostics, read at the block's end)
    int flag;                           // one-launch frame: index of this block's completion flag
};
static_assert(sizeof(float) * kUBufs * 64 * kUStride <= sizeof(_Float16) * 12 * 64 * kSlots,
              "u buffers must fit in the matrix area (B >= 13)");

template <int... I, class F>
__device__ __forceinline__ void sfor_impl(std::integer_sequence<int, I...>, F&& f) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
    sfor_impl(std::make_integer_sequence<int, N>{}, f);
}

typedef float f2v __attribute__((ext_vector_type(2)));
// A column of the design matrix in one lane: rows l + 64 j, j = 0..15, as 8
// pairs (2k, 2k + 1) -- packed halves (h2) or floats (f2v, F32).
template <bool F32>
using Pair = std::conditional_t<F32, f2v, h2>;
template <class P2>
__device__ __forceinline__ float hget(const P2 (&a)[8], int j) { return (float)a[j >> 1][j & 1]; }
template <class P2>
__device__ __forceinline__ void hset(P2 (&a)[8], int j, float v) {
    if constexpr (std::is_same_v<P2, h2>) a[j >> 1][j & 1] = (_Float16)v;  // vstore_half, round to nearest even
    else a[j >> 1][j & 1] = v;
}

__device__ __forceinline__ float lane_value(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// Phase 1 -> 3 in registers: an item's normal and position as loaded.  f32
// inputs: six floats.  Half inputs: the 12 bytes in three registers (the two
// .xy words and both .z halves in one), not four.
#ifndef BMFR_KEEP_NP_HALF_IN
#define BMFR_KEEP_NP_HALF_IN 0
#endif
#ifndef BMFR_KEEP_NP_F32
#define BMFR_KEEP_NP_F32 0
#endif
template <class IN>
struct KeptNP {
    In3<IN> n, p;
    __device__ __forceinline__ void set(const In3<IN>& nrm, const In3<IN>& wp) {
        n = nrm;
        p = wp;
    }
    __device__ __forceinline__ void get(In3<IN>& nrm, In3<IN>& wp) const {
        nrm = n;
        wp = p;
    }
};
template <>
struct KeptNP<_Float16> {
    uint32_t nxy, pxy, z;  // z: n.z | p.z << 16
    __device__ __forceinline__ void set(const In3<_Float16>& nrm, const In3<_Float16>& wp) {
        nxy = nrm.v.xy;
        pxy = wp.v.xy;
        z = (uint32_t)nrm.v.z | ((uint32_t)wp.v.z << 16);
    }
    __device__ __forceinline__ void get(In3<_Float16>& nrm, In3<_Float16>& wp) const {
        nrm.v.xy = nxy;
        nrm.v.z = (uint16_t)(z & 0xffffu);
        wp.v.xy = pxy;
        wp.v.z = (uint16_t)(z >> 16);
    }
};

// Sum over the wave of upstream work-item partials p[m] (work-item l + 64 m),
// in upstream's association (bmfr.cl:25-44); with FAST (bmfr_config.fast_fit)
// a butterfly instead (wave_reduce_fast).
template <RedOp OP, bool FAST = false>
__device__ __forceinline__ float wave_reduce(const float (&p)[4]) {
    if constexpr (FAST) return wave_reduce_fast<OP>(p);
    else return wave_tree<OP>(step2<OP>(p));
}

// RN(h - q) on one half of a packed pair (f16 -> f32 is exact, one rounding),
// without a separate conversion.  Inline asm (the compiler makes a conversion
// plus a subtraction of fmaf(h, 1, -q)): its operands never come from a DOT or
// transcendental instruction, the producers whose wait states the compiler
// cannot insert for an asm reader -- tools/isa_hazards.py checks the built code.
template <int HI>
__device__ __forceinline__ float sub_h(h2 h, float q) {
    float r;
    if constexpr (HI)
        asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(q));
    else
        asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(q));
    return r;
}

// Column update of Householder step c >= 1 (bmfr.cl:603-653) on one column:
// dot with u over rows >= c, then A -= (2u) dot / |u|^2 on those rows.
// With the fast path, the division is a Markstein step on the shared
// reciprocal (exact for these operand ranges, tests/test_markstein.py);
// non-finite or extreme operands take IEEE division (uniform branch).
// Upstream's per-element operations: the dot's four partial chains as fused
// mixed-precision FMAs (exact products, below), the quotients as packed
// Markstein steps, two rows per instruction (every lane of a packed op rounds
// like the scalar op).
// a_h * b + s in one rounding (the half element widened exactly).  Every
// product the fit forms this way is exact -- a half times a half (22
// significant bits) fits a float -- except the pivot row's u element, which
// only ever enters a chain as its first term (s = 0): so RN(a b + s) equals
// upstream's RN(RN(a b) + s) bit for bit, in one instruction instead of two.
// Written as fmaf on the widened half, which the compiler selects as one
// v_fma_mix_f32 -- NOT as inline asm: gfx950 needs three wait states between
// a DOT instruction writing a VGPR and another VALU instruction reading it
// (fast_fit feeds v_dot2 sums into this FMA), and the compiler's hazard
// recognizer inserts them only for instructions it can see.  As inline asm
// this was the round-3 "ordering bug" that a sched_barrier happened to hide
// (tools/isa_hazards.py, tests/test_isa_hazards.py).
template <int HI>
__device__ __forceinline__ float fma_h(h2 h, float b, float s) {
    return __builtin_fmaf((float)h[HI], b, s);
}

// bmfr_config.fast_fit (not bit-exact): the column update on u as packed
// halves (publish_pivot: the column's own halves, rows <= c zeroed) plus its
// pivot element uc (lane c; 0 elsewhere) in f32.  The dot as v_dot2 pairs
// (half products, f32 sums) and one mixed FMA for the pivot row, summed by
// the butterfly; a - u (2 dot / |u|^2) as one fused mixed-precision FMA per
// element on the uniform factor RN(c2 / |u|^2), instead of upstream's
// RN(a - RN(RN(u c2) / |u|^2)) -- one rounding (to f32, then half as
// upstream) where upstream has three.  (fast_fit also takes the pivot's
// square root, reciprocal and the feature scaling at hardware precision.)
// The update's FMAs are inline asm (the compiler would widen both halves
// first); their operands are u (LDS), the column (a conversion) and sc (a
// multiply) -- never a DOT result, so no hidden wait state is owed.  The pivot
// row's FMA, which reads the v_dot2 chain, is fma_h (compiler-visible).
// The scheduling barrier at the end is a register-footprint knob only
// (-DBMFR_FAST_SCHED_BARRIER=0 builds without it; tests/test_gpu_fast_fit.py
// runs that build against the exact path).
#ifndef BMFR_FAST_SCHED_BARRIER
#define BMFR_FAST_SCHED_BARRIER 1
#endif
template <int c>
__device__ __forceinline__ void update_column_fast(h2 (&a)[8], const h2 (&uh)[8], float uc, float recip2) {
    // one chain per lane: the pivot row's product (lane c) first -- its
    // mixed FMA on 0 starts the chain, no zeroed accumulators -- then the
    // eight v_dot2 pairs
    float s = fma_h<0>(a[0], uc, 0.f);
#pragma unroll
    for (int k = 0; k < 8; ++k) s = __builtin_amdgcn_fdot2(a[k], uh[k], s, false);
    const float sc = wave_reduce_fast<RedOp::Sum>(s) * recip2;  // = RN(RN(2 dot) RN(1/|u|^2)): doubling is exact
#pragma unroll
    for (int k = 0; k < kSlots / 2; ++k) {
        float lo, hi;
        asm("v_fma_mix_f32 %0, -%1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(lo) : "v"(uh[k]), "v"(sc), "v"(a[k]));
        asm("v_fma_mix_f32 %0, -%1, %2, %3 op_sel:[1,0,1] op_sel_hi:[1,0,1]" : "=v"(hi) : "v"(uh[k]), "v"(sc), "v"(a[k]));
        if (k == 0) lo = __builtin_fmaf(-uc, sc, lo);  // rows above the pivot: u = 0, unchanged
        a[k] = __builtin_convertvector((f2v{lo, hi}), h2);
    }
#if BMFR_FAST_SCHED_BARRIER
    __builtin_amdgcn_sched_barrier(0);
#endif
}

template <int c>
__device__ __forceinline__ void update_column(h2 (&a)[8], const float (&u)[kSlots], float ulen2, float recip,
                                              int l) {
    // The dot's four partial chains: chain m sums rows j = m + 4 si in order
    // si = 0..3 (upstream's work-item partials, bmfr.cl:608-617), fused
    // (fma_h: exact products, bit for bit upstream's sums).
    float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int si = 0; si < 4; ++si) {
        p[0] = fma_h<0>(a[2 * si], u[4 * si], p[0]);
        if (si == 0) p[0] = l >= c ? p[0] : 0.f;  // rows above the pivot: skipped
        p[1] = fma_h<1>(a[2 * si], u[4 * si + 1], p[1]);
        p[2] = fma_h<0>(a[2 * si + 1], u[4 * si + 2], p[2]);
        p[3] = fma_h<1>(a[2 * si + 1], u[4 * si + 3], p[3]);
    }
    const float c2 = 2.f * wave_reduce<RedOp::Sum>(p);  // (2u) dot == u (2 dot): same real product, one rounding
    f2v q[kSlots / 2];
    if (fabsf(c2) < 0x1p100f && ulen2 >= 0x1p-100f && ulen2 < 0x1p100f) {
        const f2v vb = {ulen2, ulen2}, vy = {recip, recip};
#pragma unroll
        for (int k = 0; k < kSlots / 2; ++k) {
            const f2v av = f2v{u[2 * k], u[2 * k + 1]} * c2;
            const f2v q0 = av * vy;
            const f2v r = __builtin_elementwise_fma(-q0, vb, av);
            q[k] = __builtin_elementwise_fma(r, vy, q0);
        }
    } else {
        // Cold (never taken on finite data): IEEE division, one row pair per
        // iteration of a rolled loop that rotates u and q by one pair, so the
        // code stays small; after 8 rotations both are back in order.
        float uu[kSlots];
#pragma unroll
        for (int j = 0; j < kSlots; ++j) uu[j] = u[j];
#pragma unroll 1
        for (int k = 0; k < kSlots / 2; ++k) {
            const f2v qk = {(uu[0] * c2) / ulen2, (uu[1] * c2) / ulen2};
            const float u0 = uu[0], u1 = uu[1];
#pragma unroll
            for (int j = 0; j < kSlots - 2; ++j) uu[j] = uu[j + 2];
            uu[kSlots - 2] = u0;
            uu[kSlots - 1] = u1;
#pragma unroll
            for (int i = 0; i < kSlots / 2 - 1; ++i) q[i] = q[i + 1];
            q[kSlots / 2 - 1] = qk;
        }
    }
    q[0].x = l >= c ? q[0].x : 0.f;  // x - (+0) == x: rows above the pivot keep their value
#pragma unroll
    for (int k = 0; k < kSlots / 2; ++k)
        a[k] = __builtin_convertvector((f2v{sub_h<0>(a[k], q[k].x), sub_h<1>(a[k], q[k].y)}), h2);
    __builtin_amdgcn_sched_barrier(0);  // one column in flight: bounds the register footprint
}

// f32 tmp_data (F32): the column update of step c >= 1 on float pairs.  The
// dot's four partial chains are upstream's sums of rounded products
// (bmfr.cl:608-617: tmp * u_vec, then +=) -- chains (0, 1) and (2, 3) as
// packed pairs, every lane rounding as the scalar ops --, reduced in
// upstream's association; then the update of bmfr.cl:646 as in
// update_column (packed Markstein quotients, rows above the pivot kept).
// FAST (fast_fit): fused dot chains, the butterfly sum, and one fused
// multiply-add per element on RN(c2 / |u|^2).
template <int c, bool FAST>
__device__ __forceinline__ void update_column_f32(f2v (&a)[8], const float (&u)[kSlots], float ulen2, float recip,
                                                  int l) {
    f2v p01 = {0.f, 0.f}, p23 = {0.f, 0.f};
#pragma unroll
    for (int si = 0; si < 4; ++si) {
        const f2v u01 = {u[4 * si], u[4 * si + 1]}, u23 = {u[4 * si + 2], u[4 * si + 3]};
        if constexpr (FAST) {  // fused
            p01 = __builtin_elementwise_fma(a[2 * si], u01, p01);
            p23 = __builtin_elementwise_fma(a[2 * si + 1], u23, p23);
        } else {
            p01 = p01 + a[2 * si] * u01;
            p23 = p23 + a[2 * si + 1] * u23;
        }
        if (si == 0) p01.x = l >= c ? p01.x : 0.f;  // rows above the pivot: skipped
    }
    const float p[4] = {p01.x, p01.y, p23.x, p23.y};
    if constexpr (FAST) {  // recip = 2 RN(1/|u|^2) (publish_pivot)
        const float sc = wave_reduce_fast<RedOp::Sum>(p) * recip;
        const f2v vs = {sc, sc};
        const float keep0 = a[0].x;
#pragma unroll
        for (int k = 0; k < kSlots / 2; ++k)
            a[k] = __builtin_elementwise_fma(-f2v{u[2 * k], u[2 * k + 1]}, vs, a[k]);
        a[0].x = l >= c ? a[0].x : keep0;  // rows above the pivot keep their value
        __builtin_amdgcn_sched_barrier(0);
        return;
    }
    const float c2 = 2.f * wave_reduce<RedOp::Sum>(p);
    f2v q[kSlots / 2];
    if (fabsf(c2) < 0x1p100f && ulen2 >= 0x1p-100f && ulen2 < 0x1p100f) {
        const f2v vb = {ulen2, ulen2}, vy = {recip, recip};
#pragma unroll
        for (int k = 0; k < kSlots / 2; ++k) {
            const f2v av = f2v{u[2 * k], u[2 * k + 1]} * c2;
            const f2v q0 = av * vy;
            const f2v r = __builtin_elementwise_fma(-q0, vb, av);
            q[k] = __builtin_elementwise_fma(r, vy, q0);
        }
    } else {
        // Cold (never taken on finite data): IEEE division in a rolled loop
        // rotating u and q by one pair (as update_column: no indexed arrays)
        float uu[kSlots];
#pragma unroll
        for (int j = 0; j < kSlots; ++j) uu[j] = u[j];
#pragma unroll 1
        for (int k = 0; k < kSlots / 2; ++k) {
            const f2v qk = {(uu[0] * c2) / ulen2, (uu[1] * c2) / ulen2};
            const float u0 = uu[0], u1 = uu[1];
#pragma unroll
            for (int j = 0; j < kSlots - 2; ++j) uu[j] = uu[j + 2];
            uu[kSlots - 2] = u0;
            uu[kSlots - 1] = u1;
#pragma unroll
            for (int i = 0; i < kSlots / 2 - 1; ++i) q[i] = q[i + 1];
            q[kSlots / 2 - 1] = qk;
        }
    }
    q[0].x = l >= c ? q[0].x : 0.f;  // x - (+0) == x: rows above the pivot keep their value
#pragma unroll
    for (int k = 0; k < kSlots / 2; ++k) a[k] = a[k] - q[k];
    __builtin_amdgcn_sched_barrier(0);  // one column in flight: bounds the register footprint
}

// Step 0: column 0 is FEATURE_BUFFERS[0] = 1.f, so u = (1 - 32, 1, 1, ...),
// |u|^2 = 1984 and u*x = x exactly (see k_fused's qr_column<0>).  Noise is
// added to feature columns on this first load (bmfr.cl:625-627).
// noise: the column's 1024 noise factors, or null (colour columns get none);
// pre: this lane's 16 of them already loaded (the wave's first column).
// The table holds the float factors (rnd - 0.5f); the term is noise2 * factor
// in double (bmfr.cl:173-182), formed here: 16 floats per lane -- one round
// trip for the column's loads.
template <bool FAST = false, class P2>
__device__ __forceinline__ void update_column0(P2 (&a)[8], int l, const float* __restrict__ noise,
                                               const float (&pre)[kSlots], bool use_pre, double noise2) {
    float x[kSlots];
#pragma unroll
    for (int j = 0; j < kSlots; ++j) x[j] = hget(a, j);
    // upstream adds the noise in double (one rounding to float); fast_fit:
    // one f32 FMA on the rounded amount (within an ulp of x)
    const float noise2f = (float)noise2;
#define BMFR_ADD_NOISE(xv, r) \
    (FAST ? __builtin_fmaf(noise2f, (r), (xv)) : (float)((double)(xv) + noise2 * (double)(r)))
    if (use_pre) {  // wave-uniform
#pragma unroll
        for (int j = 0; j < kSlots; ++j) x[j] = BMFR_ADD_NOISE(x[j], pre[j]);
    } else if (noise) {  // wave-uniform
        float nz[kSlots];
#pragma unroll
        for (int j = 0; j < kSlots; ++j) nz[j] = noise[l + 64 * j];
#pragma unroll
        for (int j = 0; j < kSlots; ++j) x[j] = BMFR_ADD_NOISE(x[j], nz[j]);
    }
#undef BMFR_ADD_NOISE
    if constexpr (FAST) {
        // fast_fit: u.x as a packed pairwise tree (rows 0, 1 | 2, 3 | ...; lane
        // 0's row 0 weighted -31), the subtraction packed
        f2v xp[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) xp[k] = f2v{x[2 * k], x[2 * k + 1]};
        f2v t[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) t[k] = xp[k];
        t[0].x = l == 0 ? x[0] * -31.f : x[0];
#pragma unroll
        for (int w = 4; w >= 1; w >>= 1)
#pragma unroll
            for (int k = 0; k < w; ++k) t[k] = t[k] + t[k + w];
        // the quotients correctly rounded, as upstream (q0 = -31 q instead: 1080p
        // 1.8e-5 -> 3.2e-5 from the strict build, and no faster)
        const float c2 = 2.f * wave_reduce_fast<RedOp::Sum>(t[0].x + t[0].y);
        constexpr float recip = 1.f / 1984.f;
        const float q = div_by_recip(c2, 1984.f, recip), q0 = div_by_recip(-31.f * c2, 1984.f, recip);
        const f2v vq = {q, q};
#pragma unroll
        for (int k = 0; k < 8; ++k) xp[k] = xp[k] - vq;
        xp[0].x = l == 0 ? x[0] - q0 : xp[0].x;
        if constexpr (std::is_same_v<P2, h2>) {
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] = __builtin_convertvector(xp[k], h2);
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] = xp[k];
        }
        __builtin_amdgcn_sched_barrier(0);
        return;
    }
    float p[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        float s = 0.f;
#pragma unroll
        for (int si = 0; si < 4; ++si) {
            const int j = m + 4 * si;
            s = s + (j == 0 && l == 0 ? x[0] * -31.f : x[j]);
        }
        p[m] = s;
    }
    const float c2 = 2.f * wave_reduce<RedOp::Sum>(p);
    constexpr float ulen2 = 1984.f;
    const float recip = 1.f / ulen2;
    float q, q0;
    if (fabsf(c2) < 0x1p100f) {
        q = div_by_recip(c2, ulen2, recip);
        q0 = div_by_recip(-31.f * c2, ulen2, recip);
    } else {
        q = c2 / ulen2;
        q0 = (-31.f * c2) / ulen2;
    }
    float nv[kSlots];
#pragma unroll
    for (int j = 0; j < kSlots; ++j) nv[j] = x[j] - q;
    nv[0] = l == 0 ? x[0] - q0 : nv[0];
#pragma unroll
    for (int j = 0; j < kSlots; ++j) hset(a, j, nv[j]);
    __builtin_amdgcn_sched_barrier(0);
}

// LDS flags of the fit: wave-uniform polls with a short sleep.  A publisher
// waits for lgkmcnt(0) before raising the flag, so the data it wrote is in
// LDS before any wave can see the flag.
// The polls are bounded (mp = Params::max_polls sleeps): a wave that gives up
// marks the block (*timeout), the block reports BMFR_ERROR_SYNC_TIMEOUT
// (report_sync_timeout) and runs to its end -- a scheduling bug gives a
// reported error, never a wave that never finishes nor silently wrong pixels.
template <class LDS>
__device__ __forceinline__ void wait_flag(LDS& L, const int* flag, int c) {
    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= c) return;
    const int mp = L.max_polls;
    for (int k = 0;; ++k) {
        if (k >= mp) {  // wave-uniform
            L.timeout = 1;
            return;
        }
        __builtin_amdgcn_s_sleep(1);
        if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= c) return;
    }
}
template <class LDS>
__device__ __forceinline__ void wait_pub(LDS& L, int c) {
    wait_flag(L, &L.pub, c);
}
template <int NW, class LDS>
__device__ __forceinline__ void wait_all_progress(LDS& L, int c) {
    for (int w = 0; w < NW; ++w) wait_flag(L, &L.prog[w], c);
}

// The owner of pivot column c (>= 1), once steps 0..c-1 are applied to it:
// |x|^2 over rows >= c+1, the Householder vector u and |u|^2 (bmfr.cl:555-601),
// published to LDS with the R column.  FAST (fast_fit): hardware sqrt /
// reciprocal, butterfly sum, fused squares; with half tmp_data u published
// as the column's halves (HALVES), with f32 tmp_data as floats.
template <int c, int B, int NW, bool FAST = false, class P2, class LDS>
__device__ __forceinline__ void publish_pivot(const P2 (&a)[8], LDS& L, int l) {
    constexpr int RE = B - 2;
    constexpr bool F32 = std::is_same_v<P2, f2v>;
    constexpr bool HALVES = FAST && !F32;
    float x[kSlots];
#pragma unroll
    for (int j = 0; j < kSlots; ++j) x[j] = hget(a, j);
    // |x|^2 over rows >= c + 1 (bmfr.cl:555-569): squares of halves are
    // exact, so the fused square-and-add chains are upstream's sums bit for
    // bit; f32 squares are rounded, then added (upstream's strict sequence).
    float p[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        float s = 0.f;
#pragma unroll
        for (int si = 0; si < 4; ++si) {
            const int j = m + 4 * si;
            const float xj = j == 0 && l < c + 1 ? 0.f : x[j];
            if constexpr (F32 && !FAST) s = s + xj * xj;
            else s = __builtin_fmaf(xj, xj, s);
        }
        p[m] = s;
    }
    const float sumsq = wave_reduce<RedOp::Sum, FAST>(p);
    const float ucl = lane_value(x[0], c);  // u_vec[col]: row c is lane c, j = 0
    // fast_fit: the hardware square root and reciprocal (~1 ulp) on the
    // pivot chain instead of the correctly rounded sequences
    const float vlen = FAST ? __builtin_amdgcn_sqrtf(sumsq + ucl * ucl) : sqrtf(sumsq + ucl * ucl);
    const float ucl2 = ucl - vlen;
    const float ulen2 = sumsq + ucl2 * ucl2;
    if (l == c) x[0] = ucl2;
    constexpr int buf = c % kUBufs;
    if constexpr (c >= kUBufs) wait_all_progress<NW>(L, c - kUBufs);  // readers of u_{c-3} done
    if constexpr (HALVES) {  // u as the column's halves, rows <= c zeroed; the pivot element in piv[2]
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = __builtin_bit_cast(uint32_t, a[k]);
        if (l <= c) w[0] &= 0xffff0000u;
        uint4* dst = reinterpret_cast<uint4*>(&L.u[buf][l * kUStride]);
        dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
        dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
    } else {
        float4* dst = reinterpret_cast<float4*>(&L.u[buf][l * kUStride]);
#pragma unroll
        for (int q = 0; q < 4; ++q) dst[q] = make_float4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
    }
    if (l == 0) {
        L.piv[buf][0] = ulen2;
        // fast_fit: 2 RN(1/|u|^2) (the update's factor RN(RN(2 dot) / ...)
        // then takes one multiply: doubling is exact)
        L.piv[buf][1] = FAST ? 2.f * __builtin_amdgcn_rcpf(ulen2) : 1.f / ulen2;
        L.piv[buf][2] = ucl2;
    }
    if (l < c) {  // R column: rows above the diagonal, then the diagonal
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) L.fo().R[(c * RE + l) * 3 + ch] = x[0];
    }
    if (l == c) {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) L.fo().R[(c * RE + c) * 3 + ch] = vlen;
    }
    // u_c and |u_c|^2 in LDS before the flag says so
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    if (l == 0) __hip_atomic_store(&L.pub, c, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The work-group shares data through LDS only, so its barriers need not
// wait for its global loads and stores (__syncthreads() does).
__device__ __forceinline__ void k1_barrier() { lds_barrier(); }

// Wave W's part of the fit: columns c = 1 + W + NW k (slot k); column 0 is
// implicit.  W is a run-time (wave-uniform) value, so the NW waves run one
// copy of the code: column ownership is a scalar branch, while the slot of
// every column a step touches is known at compile time.
template <int NS, int FS, int NW = 4, bool FAST = false, bool F32 = false>
struct WaveFit {
    static constexpr int B = NS + FS + 3;
    // fast_fit (FAST): the fused trailing update, butterfly reductions, f32
    // noise add, hardware sqrt / reciprocals, scaling by the reciprocal; with
    // half tmp_data (FASTR) also u published as halves (the update on v_dot2 /
    // v_fma_mix).
    static constexpr bool FASTR = FAST && !F32;
    using P2 = Pair<F32>;
    static constexpr int NF = B - 3;  // pivot columns
    static constexpr int NSL = (B - 1 + NW - 1) / NW;
    static constexpr int NT = 64 * NW, NI = 16 / NW;  // threads, items (rows) per thread in phases 1 and 3
    using LDS = Lds<B, NW, F32>;
    static __device__ __forceinline__ bool owns(int W, int c) { return c >= 1 && c < B && (c - 1) % NW == W; }
    static constexpr int owner(int c) { return (c - 1) % NW; }
    static constexpr int slot(int c) { return (c - 1) / NW; }
    // Step-0 noise columns prefetched per wave (slots whose column is a
    // feature column for every wave), loaded in phase 1.  B = 16 with four
    // waves: two as well since round 6 (its K1 now has the registers: 108
    // VGPRs with them, no spills; config 5's K1 -1.7 to -2.2 %,
    // profiles/r06_ab_np16.txt); -DBMFR_NP16=0 gives none.
#ifndef BMFR_NP16
#define BMFR_NP16 2
#endif
    static constexpr int NP = B >= 16 && NW == 4 ? BMFR_NP16 : ((NF - 1) / NW < kPre ? (NF - 1) / NW : kPre);
    static_assert(!F32 || NW == 4, "f32 tmp_data: row quad w of wave w");
    static_assert(NP == 0 || NW * NP < NF, "prefetched slots hold feature columns");

    // The first column a wave updates at step 0: a feature column for every wave.
    static __device__ __forceinline__ int first_column(int W) { return 1 + W; }

    template <int c>
    static __device__ __forceinline__ void step(P2 (&a)[NSL][8], LDS& L, int W, int l,
                                                const float* __restrict__ noise, const float (&pre)[kPre][kSlots],
                                                double noise2) {
        constexpr int nxt = c + 1;  // the next pivot column, slot(nxt) of wave owner(nxt)
        const bool publish = nxt < NF && W == owner(nxt);
        if constexpr (c == 0) {
            if (publish) {  // column 1 of wave 0: its first column
                update_column0<FAST>(a[slot(nxt)], l, noise + (nxt - 1) * kBlockPixels, pre[0], NP > 0, noise2);
                publish_pivot<nxt, B, NW, FAST>(a[slot(nxt)], L, l);
            }
            sfor<NSL>([&](auto K) {
                constexpr int k = decltype(K)::value;
                const int fb = 1 + W + NW * k;
                if (owns(W, fb) && !(publish && fb == nxt))  // slots < NP: feature columns, prefetched
                    update_column0<FAST>(a[k], l, fb < NF ? noise + (fb - 1) * kBlockPixels : nullptr,
                                   pre[k < kPre ? k : 0], k < NP, noise2);
            });
        } else {
            if (1 + W + NW * ((B - 2 - W) / NW) > c) {  // this wave's last column is past the pivot
                wait_pub(L, c);
                float u[FASTR ? 1 : kSlots];
                h2 uh[FASTR ? 8 : 1];
                float uc = 0.f;
                if constexpr (FASTR) {
                    const uint4* src = reinterpret_cast<const uint4*>(&L.u[c % kUBufs][l * kUStride]);
                    const uint4 v0 = src[0], v1 = src[1];
                    const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
                    for (int k = 0; k < 8; ++k) uh[k] = __builtin_bit_cast(h2, w[k]);
                    uc = l == c ? L.piv[c % kUBufs][2] : 0.f;
                } else {
                    const float4* src = reinterpret_cast<const float4*>(&L.u[c % kUBufs][l * kUStride]);
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float4 v = src[q];
                        u[4 * q] = v.x;
                        u[4 * q + 1] = v.y;
                        u[4 * q + 2] = v.z;
                        u[4 * q + 3] = v.w;
                    }
                }
                const float ulen2 = L.piv[c % kUBufs][0], recip = L.piv[c % kUBufs][1];
                auto upd = [&](P2 (&col)[8]) {
                    if constexpr (F32) update_column_f32<c, FAST>(col, u, ulen2, recip, l);
                    else if constexpr (FAST) update_column_fast<c>(col, uh, uc, recip);
                    else update_column<c>(col, u, ulen2, recip, l);
                };
                if constexpr (nxt < NF) {
                    if (publish) {  // the next pivot is every wave's critical path: issue it first
                        upd(a[slot(nxt)]);
                        publish_pivot<nxt, B, NW, FAST>(a[slot(nxt)], L, l);
                    }
                }
                sfor<NSL>([&](auto K) {
                    constexpr int k = decltype(K)::value;
                    const int fb = 1 + W + NW * k;
                    if constexpr (NW * k + NW > c) {  // slot k holds columns <= NW k + NW
                        if (owns(W, fb) && fb > c && !(publish && fb == nxt)) upd(a[k]);
                    }
                });
            }
        }
        // this wave is done with u_c (no barrier: a wave waits only for the pivot it needs)
        if (l == 0) __hip_atomic_store(&L.prog[W], c, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }

    template <int... C>
    static __device__ __forceinline__ void steps(P2 (&a)[NSL][8], LDS& L, int W, int l,
                                                 const float* __restrict__ noise, const float (&pre)[kPre][kSlots],
                                                 double noise2, std::integer_sequence<int, C...>) {
        (step<C>(a, L, W, l, noise, pre, noise2), ...);
    }

    // Step 0's noise for the wave's first NP columns (1 + W, 1 + W + NW:
    // feature columns for every wave), loaded while the last items of phase 1
    // finish (the fit's first dependent loads); the other noisy columns load
    // in step 0.
    static __device__ __forceinline__ void prefetch_noise(int W, int l, const float* __restrict__ noise,
                                                          float (&pre)[kPre][kSlots]) {
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            const float* src = noise + (first_column(W) + NW * k - 1) * kBlockPixels + l;
#pragma unroll
            for (int j = 0; j < kSlots; ++j) pre[k][j] = src[64 * j];
        }
    }

    static __device__ __forceinline__ void run(LDS& L, int W, int l, const float* __restrict__ noise,
                                               const float (&pre)[kPre][kSlots], double noise2, int mp,
                                               const float (&kp)[NI][3], const f2v (&own)[NSL][2]) {
        P2 a[NSL][8];
        sfor<NSL>([&](auto K) {
            constexpr int k = decltype(K)::value;
            const int c = 1 + W + NW * k;
            if (owns(W, c)) {
                if constexpr (F32) {
                    // quad W from phase 1's registers, the others from LDS (a lane
                    // stride of 12 floats: conflict-free 16-byte reads)
                    const float4* src = reinterpret_cast<const float4*>(&L.M[c - 1][l * m_slots<true>()]);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        if (i == W) {
                            a[k][2 * i] = own[k][0];
                            a[k][2 * i + 1] = own[k][1];
                        } else {
                            const float4 v = src[i - (i > W)];
                            a[k][2 * i] = f2v{v.x, v.y};
                            a[k][2 * i + 1] = f2v{v.z, v.w};
                        }
                    }
                } else {
                    // pair p of lane l's row slot sits at dword p ^ ((l >> 2) & 7) (see phase 1)
                    const uint32_t* src = reinterpret_cast<const uint32_t*>(&L.M[c - 1][l * kSlots]);
                    const int q = (l >> 2) & 7;
#pragma unroll
                    for (int i = 0; i < 8; ++i) a[k][i] = __builtin_bit_cast(h2, src[i ^ q]);
                }
            }
        });
        if (W == 0 && l < NW + 3) {  // read only after the barrier below
            if (l == 0) L.pub = 0;
            else if (l == NW + 1) L.timeout = 0;
            else if (l == NW + 2) L.max_polls = mp;
            else L.prog[l - 1] = -1;
        }
        k1_barrier();  // the u buffers alias M
        if constexpr (keep_in_m(B, F32)) {  // phase 1's kept colours into the matrix area beside the u buffers
            const int t = W * 64 + l;
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) L.keep_m[(i * 3 + ch) * NT + t] = kp[i][ch];
        }

        // Scale the position features to the block's [min, max] (bmfr.cl:510-542).
        sfor<NSL>([&](auto K) {
            constexpr int k = decltype(K)::value;
            const int c = 1 + W + NW * k;
            if (owns(W, c) && c >= NS && c < NF) {
                float bmax, bmin;
                if constexpr (FASTR) {  // min / max of the packed halves (NaN-free: phase 1 maps NaN to 0)
                    h2 mx = a[k][0], mn = a[k][0];
#pragma unroll
                    for (int i = 1; i < 8; ++i) {
                        mx = __builtin_elementwise_max(mx, a[k][i]);
                        mn = __builtin_elementwise_min(mn, a[k][i]);
                    }
                    bmax = wave_reduce_fast<RedOp::Max>(fmaxf((float)mx[0], (float)mx[1]));
                    bmin = wave_reduce_fast<RedOp::Min>(fminf((float)mn[0], (float)mn[1]));
                } else {
                    float hi[4], lo[4];
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        hi[m] = -INFINITY;
                        lo[m] = INFINITY;
#pragma unroll
                        for (int si = 0; si < 4; ++si) {
                            const float v = hget(a[k], m + 4 * si);
                            hi[m] = fmaxf(v, hi[m]);
                            lo[m] = fminf(v, lo[m]);
                        }
                    }
                    bmax = wave_reduce<RedOp::Max, FAST>(hi);
                    bmin = wave_reduce<RedOp::Min, FAST>(lo);
                }
                const float d = bmax - bmin;
                const bool divide = fabsf(d) > 1.0f;  // scale(), bmfr.cl:200-205
                // fast_fit: the hardware reciprocal, and the scaling as ONE fused
                // multiply-add x s + o, (s, o) = (rcp, RN(-bmin rcp)) or (1, -bmin),
                // in phase 3 as here (fast_scale)
                const float rcp = FAST ? __builtin_amdgcn_rcpf(d) : 1.f / d;
                if (l == 0) {
                    L.fo().mm[3 * (c - NS)] = bmin;
                    L.fo().mm[3 * (c - NS) + 1] = bmax;
                    L.fo().mm[3 * (c - NS) + 2] = rcp;
                }
                if constexpr (FAST) {
                    const float fs = divide ? rcp : 1.f, fo = divide ? -bmin * rcp : -bmin;
                    if constexpr (FASTR) {
#pragma unroll
                        for (int i = 0; i < 8; ++i)
                            a[k][i] = __builtin_convertvector(
                                (f2v{fma_h<0>(a[k][i], fs, fo), fma_h<1>(a[k][i], fs, fo)}), h2);
                    } else {
#pragma unroll
                        for (int i = 0; i < 8; ++i) a[k][i] = __builtin_elementwise_fma(a[k][i], f2v{fs, fs}, f2v{fo, fo});
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < kSlots; ++j) {
                        const float v = hget(a[k], j) - bmin;
                        hset(a[k], j, divide ? div_by_recip(v, d, rcp) : v);
                    }
                }
            }
        });
        if (W == 0 && l < 3) L.fo().R[l] = 32.f;  // R(0,0) = |column 0|

#ifndef BMFR_PROBE_K1_NOQR  // timing probe (wrong results): no Householder steps
        steps(a, L, W, l, noise, pre, noise2, std::make_integer_sequence<int, NF>{});
#endif

        // Right-hand side: rows 0..B-4 of the colour columns (bmfr.cl:596-600).
        sfor<NSL>([&](auto K) {
            constexpr int k = decltype(K)::value;
            const int c = 1 + W + NW * k;
            if (owns(W, c) && c >= NF) {
                if (l < NF) L.fo().R[((B - 3) * (B - 2) + l) * 3 + (c - NF)] = hget(a[k], 0);
            }
        });
    }
};

// Back substitution (bmfr.cl:658-699) in registers of wave 0, one 16-lane
// DPP row per colour channel: lane 16 ch + x holds column x of R (rows
// 0..RE-2) for channel ch.  Every cross-lane value a step needs moves inside
// the row by DPP -- the diagonal by a row broadcast, the right-hand side's
// serial reduction as a scan along the row -- so no step waits on a
// readlane / scalar round trip.  Every element sees upstream's operations in
// upstream's order: row i divided by the diagonal, the right-hand side
// reduced by the already-divided row entries left to right, column i scaled
// by x_i.
template <int K>
__device__ __forceinline__ float row_shl(float v) {  // lane l <- lane l + K of its row
    if constexpr (K == 0) return v;
    else return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x100 + K, 0xf, 0xf, true));
}
template <int N>
__device__ __forceinline__ float row_bcast(float v) {  // every lane <- lane N of its row
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + N, 0xf, 0xf, false));
}
// FAST (fast_fit): the division by the diagonal as a multiply by the
// hardware reciprocal (1 ulp), which shortens the step chain's latency.
#ifndef BMFR_FAST_BACKSUB
#define BMFR_FAST_BACKSUB 1
#endif
template <int B, bool FAST, class LDS>
__device__ __forceinline__ void back_substitute_regs(LDS& L, int t) {
    constexpr int RE = B - 2;
    static_assert(RE <= 16, "one DPP row per channel");
    if (t >= 64) return;
    const int ch = t >> 4, x = t & 15;
    const bool live = ch < 3 && x < RE;
    float col[RE - 1];  // rows 0..RE-2 of column x
#pragma unroll
    for (int y = 0; y < RE - 1; ++y) col[y] = live ? L.fo().R[(x * RE + y) * 3 + ch] : 0.f;
    sfor<RE - 1>([&](auto I) {
        constexpr int i = RE - 2 - decltype(I)::value;
        const float div = row_bcast<i>(col[i]);
        if constexpr (FAST && BMFR_FAST_BACKSUB) {
            const float r = __builtin_amdgcn_rcpf(div);
            if (live && x >= i) col[i] = col[i] * r;
        } else {
            if (live && x >= i) col[i] = col[i] / div;
        }
        const float v = col[i];
        // x_i = ((rhs - v[i+1]) - v[i+2]) ... - v[RE-2], rhs = v[RE-1]: the
        // running value walks from lane i+1 to lane RE-2 (src).
        constexpr int src = i == RE - 2 ? RE - 1 : RE - 2;
        float acc = v;
        if constexpr (i < RE - 2) {
            acc = row_shl<RE - 2 - i>(v) - v;  // lane i+1: rhs - v[i+1]
#pragma unroll
            for (int j = i + 2; j <= RE - 2; ++j) acc = dpp_shr1(acc) - v;  // lane j
        }
        if constexpr (i < RE - 2) {
            const float at_rhs = dpp_shr1(acc);  // lane RE-1 <- lane RE-2
            if (x == RE - 1) col[i] = at_rhs;
        }
        const float xi = row_shl<src - i>(acc);  // lane i <- lane src
        if (x == i) {
#pragma unroll
            for (int y = 0; y <= i; ++y) col[y] = col[y] * xi;
        }
    });
    if (ch < 3 && x == RE - 1) {
#pragma unroll
        for (int y = 0; y < B - 3; ++y) L.fo().weights[y * 3 + ch] = col[y];
    }
}


// One K1 work-group (block g of the launch), on the LDS area L.
// COH: the TAA tiles of the same frame run in this launch: the accumulated
// colour and the reprojected positions they read are stored device-coherent
// and the block publishes done[g] = epoch once they are.
template <int NS, int FS, class IN, bool COH = false, int NW = 4, bool FAST = false, bool F32 = false>
__device__ __forceinline__ void k1_cols_body(const Params& P, const K1Args& A, Lds<NS + FS + 3, NW, F32>& L, int g) {
    constexpr int B = NS + FS + 3;
    constexpr bool FASTR = FAST && !F32;  // WaveFit::FASTR
    using P2 = Pair<F32>;
    constexpr int NT = 64 * NW, NI = 16 / NW;  // threads; items (rows) per thread
    const int t = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int l = t & 63;
    const int frame = A.frame;
#ifdef BMFR_STAMPS
#define BMFR_STAMP(k) \
    if (t == 0 && A.stamps) A.stamps[(size_t)g * 8 + (k)] = __builtin_amdgcn_s_memtime()
#else
#define BMFR_STAMP(k) (void)0
#endif
    BMFR_STAMP(0);
#ifdef BMFR_STAMPS
    if (t == 0 && A.stamps) A.stamps[(size_t)g * 8 + 6] = __builtin_amdgcn_s_memrealtime();  // 100 MHz
#endif
    int bx, by;
    k1_block(P, g, bx, by);
    // COH: this block's completion flag, in the launch's block rectangle (g
    // itself unless the launch is a tiled context's border ring); parked in
    // LDS until the end (fewer scalar registers live across the kernel)
    if constexpr (COH)
        if (t == 0) L.flag = (by - P.by0) * P.nbx + (bx - P.bx0);
    // Item i of wave w: block row pair 2 (NI w + i) (a wave sweeps its own 8
    // rows), or with kInterleave 2 (NW i + w) (the work-group's waves sweep
    // the block together, neighbouring row pairs at a time: their previous-
    // frame taps share cache lines); lanes 0-31 / 32-63 take the pair's rows.
    // The design-matrix row of a pixel (its index in the block) is the same
    // either way: only which thread computes it changes.
    // kInterleave with fast_fit: K1 -1.1 %; on the exact path +1.1 % (its
    // half-at-a-time matrix stores), so not there (profiles/r04_ab_row_interleave.txt).
#ifndef BMFR_K1_INTERLEAVE
#define BMFR_K1_INTERLEAVE (FASTR ? 1 : 0)
#endif
    // 0: own 8 rows; 1: slot NW i + w; 2: item pairs interleaved (slots 2 NW (i / 2) + 2 w + (i & 1):
    // a thread's two items of a pair stay adjacent slots, one 4-byte store per column)
    constexpr int kIlv = F32 ? 0 : BMFR_K1_INTERLEAVE;  // f32: wave w computes row quad w (compacted matrix)
    constexpr bool kInterleave = kIlv == 1;
    auto item_slot = [&](int i) {  // row slot j: rows l + 64 j
        return kIlv == 1 ? NW * i + w : (kIlv == 2 ? 2 * NW * (i / 2) + 2 * w + (i & 1) : NI * w + i);
    };
    const int lx = l & (kEdge - 1);
    auto item_row = [&](int lane, int i) { return (lane >> 5) + 2 * item_slot(i); };

    // ---- accumulate_noisy_data (bmfr.cl:310-484), rows l + 64 (NI w + i) ----
    P2 pk[B];            // features of an item pair, packed for one LDS store per column
    // F32: this wave's row quad of the columns it owns in the fit (slot k:
    // column 1 + w + NW k), never stored to LDS
    f2v own[WaveFit<NS, FS, NW, FAST, F32>::NSL][2];
    uint32_t spps = 0;   // per item i, bits 8i..8i+7: its new spp
    uint32_t ibits = 0;  // per item i, bit i: owner; bit 4 + i: accepted taps with weight > 0
    int over = 0;        // reprojection taps outside the valid state rectangle (tiled contexts)
    // The temporal part of accumulate_filtered_data is read at the noisy
    // accumulation's taps (bmfr.cl:786-842) and parked in LDS for phase 3.
    // Software-pipelined one item deep: item i + 1's current-frame loads go
    // out right behind item i's reprojection taps, so each wait for taps
    // leaves the next item's loads in flight.
    float kp[NI][3];  // keep_in_m(B): the kept colours, in registers until the fit has loaded M
    // fast_fit at B = 13: phase 1's normal / position stay in registers for
    // phase 3 (no second read of those planes: 24 B/px of f32 input; K1
    // -4 %).  The other K1s hold too many registers for it (round 6,
    // profiles/r06_ab_keep_np.txt): the exact fit and f32 tmp_data spill at
    // four work-groups per CU and lose 7-8 % at three; config 5's half inputs
    // (three registers per item, BMFR_KEEP_NP_HALF_IN) spill 7 dwords and tie.
#ifdef BMFR_KEEP_NP_ALL
    constexpr bool kKeepNP = true;
#else
    constexpr bool kKeepNP = FAST && (F32 ? BMFR_KEEP_NP_F32 && B < 16
                                          : B < 16 || (BMFR_KEEP_NP_HALF_IN && sizeof(IN) == 2));
#endif
    KeptNP<IN> keep_np[NI];
    NoisyCur<IN> cur = noisy_load_current<IN>(P, A.in, bx * kEdge + lx, by * kEdge + item_row(l, 0), frame);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const NoisyTaps<IN> tp = noisy_taps_issue<true, IN>(P, A.in, A.cam, cur, frame, A.acc_prev);
        NoisyCur<IN> nxt;
        if (i < NI - 1) nxt = noisy_load_current<IN>(P, A.in, bx * kEdge + lx, by * kEdge + item_row(l, i + 1), frame);
        __builtin_amdgcn_sched_barrier(0);
        const NoisyItem it = noisy_taps_finish<true, IN>(P, cur, tp, frame);
        if constexpr (kKeepNP) keep_np[i].set(cur.nrm, cur.wp);
        {
#pragma unroll
            for (int f = 1; f < B; ++f) {
                float v;
                if (f < B - 3) v = feature_value(f, it.n, it.p);
                else v = f == B - 3 ? it.color.x : (f == B - 2 ? it.color.y : it.color.z);
                // NaN -> 0 (bmfr.cl:468-469), then (half tmp_data) the +-65504
                // clamp (bmfr.cl:471-473) as one med3 (equal to fmax(fmin(v, 65504),
                // -65504) for every non-NaN v)
                if constexpr (F32) v = __builtin_isnan(v) ? 0.0f : v;
                else v = __builtin_isnan(v) ? 0.0f : __builtin_amdgcn_fmed3f(v, -65504.f, 65504.f);
                if constexpr (kInterleave) {  // this item's half of its row-slot pair (XOR-swizzled as below)
                    static_assert(!F32, "f32 tmp_data stores item pairs");
                    const int j = item_slot(i);
                    L.M[f - 1][l * kSlots + 2 * ((j >> 1) ^ ((l >> 2) & 7)) + (j & 1)] = (_Float16)v;
                } else {
                    if constexpr (F32) pk[f][i & 1] = v;
                    else pk[f][i & 1] = (_Float16)v;
                }
            }
            spps |= (uint32_t)it.spp << (8 * i);
            ibits |= ((uint32_t)it.owner << i) | ((uint32_t)it.prev_f_divided << (4 + i));
            over = max(over, it.over);
            if constexpr (keep_in_m(B, F32)) {
                kp[i][0] = it.prev_f.x;
                kp[i][1] = it.prev_f.y;
                kp[i][2] = it.prev_f.z;
            } else {
                L.keep_s[(i * 3 + 0) * NT + t] = it.prev_f.x;
                L.keep_s[(i * 3 + 1) * NT + t] = it.prev_f.y;
                L.keep_s[(i * 3 + 2) * NT + t] = it.prev_f.z;
            }
            // owners only (bmfr.cl:478-484), as branch-free stores (st3_drop)
            st3_drop(drop_plane(A.noisy_out), it.lin, it.owner, it.color);
            st1_drop(drop_plane(A.spp_out), it.lin, it.owner, it.spp);
            st2_drop<COH ? kSc1 : 0>(drop_plane(A.prev_pixel_out), it.lin, it.owner, make_float2(it.pfx, it.pfy));
            if (!kInterleave && (i & 1)) {  // rows j = NI w + i - 1, NI w + i: adjacent halves of lane l's row slot
                if constexpr (F32) {
                    // rows 4 w + i - 1, 4 w + i: half (i - 1) / 2 of quad w; columns of
                    // wave w stay in registers, the others go to compacted quad
                    // w - (w > owner) of the owner's view (see Lds::M)
                    static_assert(kIlv == 0, "f32 tmp_data: wave w computes row quad w");
#pragma unroll
                    for (int f = 1; f < B; ++f) {
                        const int ow = (f - 1) % NW;
                        if (w == ow) own[(f - 1) / NW][i >> 1] = pk[f];
                        else
                            *reinterpret_cast<f2v*>(&L.M[f - 1][l * m_slots<true>() + 4 * (w - (w > ow)) + (i - 1)]) =
                                pk[f];
                    }
                } else {
                    // (pair (NI w + i) / 2; XOR-swizzled by lane so a wave's 4-byte stores hit 32 banks)
                    const int pair = (item_slot(i) / 2) ^ ((l >> 2) & 7);
#pragma unroll
                    for (int f = 1; f < B; ++f)
                        *reinterpret_cast<uint32_t*>(&L.M[f - 1][l * kSlots + 2 * pair]) =
                            __builtin_bit_cast(uint32_t, pk[f]);
                }
            }
        }
        if (i < NI - 1) cur = nxt;
    }
    report_reach(P, A.reach, over);
    float pre[kPre][kSlots];
    WaveFit<NS, FS, NW, FAST, F32>::prefetch_noise(w, l, A.noise, pre);
    k1_barrier();  // matrix in LDS; phase 1's global stores drain in the background
    BMFR_STAMP(1);
    BMFR_STAMP(2);  // scaling runs inside the per-wave fit

    // ---- fit: min/max scaling, Householder QR, right-hand side ----
    if (t == 0) L.delay = P.debug_delay;  // read after the fit's barriers
    WaveFit<NS, FS, NW, FAST, F32>::run(L, w, l, A.noise, pre, P.noise2, P.max_polls, kp, own);
    // Phase 3's loads (normal and position of the NI items, bmfr.cl:725-729)
    // go out now: they land while wave 0 back-substitutes and the others wait.
    int l3 = l;  // opaque copy: recompute phase-1 addresses instead of keeping them live across the fit
    asm volatile("" : "+v"(l3));
    const int2 off = kBlockOffsets[frame & 15];
    uint32_t lin[NI];
    In3<IN> nrm_r[NI], wp_r[NI];  // as loaded: widened after the back substitution
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int px = bx * kEdge + (l3 & (kEdge - 1)) - kEdge / 2 + off.x;
        const int py = by * kEdge + item_row(l3, i) - kEdge / 2 + off.y;
        lin[i] = pix(P, (ibits & (1u << i)) ? px : P.ox, (ibits & (1u << i)) ? py : P.oy);  // margins: a valid pixel, skipped below
        if constexpr (kKeepNP) {
            keep_np[i].get(nrm_r[i], wp_r[i]);
        } else {
            nrm_r[i] = ld3raw<IN>(A.in.n_cur, lin[i]);
            wp_r[i] = ld3raw<IN>(A.in.p_cur, lin[i]);
        }
    }
    k1_barrier();  // R complete (LDS); with LDS-only barriers the loads above stay in flight
    BMFR_STAMP(3);
    back_substitute_regs<B, FAST>(L, t);
    k1_barrier();  // weights complete
    // An exhausted pivot wait: reported here, or (one-launch frame) carried by
    // the block's completion flag to the tiles that read it (fewer values
    // live across the kernel).
    if constexpr (!COH)
        if (t == 0 && L.timeout) report_sync_timeout(A.sync_err, kSyncPivot, frame);
    BMFR_STAMP(4);
    f3 nrm[NI], wp[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        nrm[i] = widen(nrm_r[i]);
        wp[i] = widen(wp_r[i]);
    }

#ifdef BMFR_PROBE_K1_NOP3  // timing probe (wrong results): no weighted sum / blend / stores
    if (frame >= 0) return;
#endif
    // ---- weighted_sum (bmfr.cl:717-750) + temporal blend (bmfr.cl:778-849) ----
    // Items (0, 1) and (2, 3) as packed f32 pairs: every lane rounds as
    // upstream's scalar sequence, each item in feature order.
    constexpr int NPR = NI / 2;  // item pairs
    f2v cp[NPR][3];
#pragma unroll
    for (int h = 0; h < NPR; ++h)
        for (int ch = 0; ch < 3; ++ch) cp[h][ch] = f2v{0.f, 0.f};
    // Item pairs outer where it saves registers: one pair's positions, powers
    // and sums live at a time (features outer keeps every item's in
    // registers: 14-67 dwords of spills at B = 16 with four work-groups per
    // CU; pairs outer: none).  Features outer (each weight and min / max
    // loaded once) at B = 13, where the K1s have the registers for it since
    // round 6 (no spills; K1 -0.3 / -0.5 / -1.3 % headline / exact / f32
    // tmp_data, profiles/r06_ab_np16.txt); -DBMFR_PAIRS_B13=1 keeps pairs
    // outer there too.
#ifndef BMFR_PAIRS_B13
#define BMFR_PAIRS_B13 0
#endif
#ifdef PAIRS_ALL
    constexpr bool kPairs = true;
#else
    constexpr bool kPairs = B >= 16 || (!COH && BMFR_PAIRS_B13) || NPR == 1;
#endif
    constexpr int NH = kPairs ? NPR : 1;
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
#pragma unroll
        for (int f = 0; f < B - 3; ++f) {
            const f2v wv[3] = {f2v{L.fo().weights[3 * f], L.fo().weights[3 * f]},
                               f2v{L.fo().weights[3 * f + 1], L.fo().weights[3 * f + 1]},
                               f2v{L.fo().weights[3 * f + 2], L.fo().weights[3 * f + 2]}};
            float bmin = 0.f, d = 0.f, rcp = 0.f;
            if (f >= NS) {
                bmin = L.fo().mm[3 * (f - NS)];
                d = L.fo().mm[3 * (f - NS) + 1] - bmin;
                rcp = L.fo().mm[3 * (f - NS) + 2];
            }
#pragma unroll
            for (int h = kPairs ? hh : 0; h < (kPairs ? hh + 1 : NPR); ++h) {
                f2v v = {feature_value(f, nrm[2 * h], wp[2 * h]), feature_value(f, nrm[2 * h + 1], wp[2 * h + 1])};
                if (f >= NS && FAST) {  // fast_fit: x s + o, as the fit scaled it
                    const bool divide = fabsf(d) > 1.0f;
                    const float fs = divide ? rcp : 1.f, fo = divide ? -bmin * rcp : -bmin;
                    v = __builtin_elementwise_fma(v, f2v{fs, fs}, f2v{fo, fo});
                } else if (f >= NS) {
                    v = v - f2v{bmin, bmin};
                    if (fabsf(d) > 1.0f) {
                        const f2v q0 = v * f2v{rcp, rcp};
                        const f2v r = __builtin_elementwise_fma(-q0, f2v{d, d}, v);
                        v = __builtin_elementwise_fma(r, f2v{rcp, rcp}, q0);
                    }
                }
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) cp[h][ch] = cp[h][ch] + wv[ch] * v;
            }
            __builtin_amdgcn_sched_barrier(0);  // one feature's weights live at a time
        }
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        if (ibits & (1u << i)) {
            f3 ci{cp[i >> 1][0][i & 1], cp[i >> 1][1][i & 1], cp[i >> 1][2][i & 1]};
            ci.x = ci.x < 0.f ? 0.f : ci.x;
            ci.y = ci.y < 0.f ? 0.f : ci.y;
            ci.z = ci.z < 0.f ? 0.f : ci.z;
            // bmfr.cl:834-849: alpha from the current spp when the taps carried weight
            // 1 / spp with spp in [1, 255]: rcp_nr (exactly 1.f / spp); the
            // one-launch frame kernel keeps the division (rcp_nr's shorter
            // sequence is scheduled early there and spills 14-17 VGPRs)
            const float sp = (float)((spps >> (8 * i)) & 255u);
            const float alpha =
                (ibits & (1u << (4 + i))) ? fmaxf(COH ? 1.f / sp : rcp_nr(sp), P.second_blend_alpha) : 1.f;
            const float beta = 1.f - alpha;
            const int t3 = l3 + 64 * w;
            const float* kb = L.keep();
            const f3 prev{kb[(i * 3) * NT + t3], kb[(i * 3 + 1) * NT + t3], kb[(i * 3 + 2) * NT + t3]};
            const f3 acc{alpha * ci.x + beta * prev.x, alpha * ci.y + beta * prev.y, alpha * ci.z + beta * prev.z};
            if constexpr (COH) st3_coh(coh_plane(A.acc_out), lin[i], acc);
            else st3(A.acc_out, lin[i], acc);
        }
    }
#ifdef BMFR_STAMPS
    __syncthreads();
#endif
    BMFR_STAMP(5);
#ifdef BMFR_STAMPS
    if (t == 0 && A.stamps) A.stamps[(size_t)g * 8 + 7] = __builtin_amdgcn_s_memrealtime();
#endif
#undef BMFR_STAMP
    if constexpr (COH) {
        const int delay = L.delay;
        if (delay > 0 && g % kDelayStride == kDelayPhase)  // diagnostics: tiles really wait
            for (int k = 0; k < delay; ++k) __builtin_amdgcn_s_sleep(127);
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): this wave's stores are performed
        lds_barrier();                       // ... and every wave's
        if (t == 0)
            __hip_atomic_store(&A.done[L.flag], A.epoch | (L.timeout ? kDoneTimeout : 0u), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Waves per work-group of the column-split K1: 4, or 8 with -DBMFR_K1_WAVES=8
// (half the rows per thread in phases 1 and 3, fewer columns per wave in the
// fit, more waves per CU).
#ifndef BMFR_K1_WAVES
#define BMFR_K1_WAVES 4
#endif
constexpr int kNW = BMFR_K1_WAVES;
constexpr int kK1Threads = 64 * kNW;
// Minimum waves per SIMD for the register allocator: 4 work-groups of 4
// waves per CU (128 VGPRs), or 3 of 8 (80); -DBMFR_K1_MIN_WAVES overrides.
// f32 tmp_data: the compacted matrix's LDS allows four work-groups per CU at
// B = 13 (38 KB each), three at B = 16 (48 KB); at B = 13 the exact fit
// needs more than 128 VGPRs (78 spilled at four), so three there.
#ifndef BMFR_F32_WAVES6
#define BMFR_F32_WAVES6 4
#endif
#ifndef BMFR_F32_WAVES6X
#define BMFR_F32_WAVES6X 3
#endif
#ifndef BMFR_F32_WAVES9
#define BMFR_F32_WAVES9 3
#endif
#ifdef BMFR_K1_MIN_WAVES
constexpr int kMinWavesSimd = BMFR_K1_MIN_WAVES;
#else
constexpr int kMinWavesSimd = kNW == 4 ? 4 : 6;
#endif
// Config 5 (B = 16, fast_fit): -DBMFR_K1_WAVES9F=5 asks for five work-groups
// per CU (its LDS allows them since FitOut sits in the matrix area's tail).
#ifndef BMFR_K1_WAVES9F
#define BMFR_K1_WAVES9F kMinWavesSimd
#endif
template <int FS, bool F32, bool FAST>
constexpr int min_waves() {
    return F32 ? (FS == 6 ? (FAST ? BMFR_F32_WAVES6 : BMFR_F32_WAVES6X) : BMFR_F32_WAVES9)
               : (FS == 9 && FAST ? BMFR_K1_WAVES9F : kMinWavesSimd);
}

// FAST: bmfr_config.fast_fit (the fused trailing update, update_column).
template <int NS, int FS, class IN, bool FAST = false, bool F32 = false>
__global__ __launch_bounds__(kK1Threads, (min_waves<FS, F32, FAST>())) void k_fused_cols(Params P, K1Args A) {
    __shared__ Lds<NS + FS + 3, kNW, F32> L;
    k1_cols_body<NS, FS, IN, false, kNW, FAST, F32>(P, A, L, xcd_swizzle(blockIdx.x, gridDim.x));
}

// K1 and K2 (64 x kFrameTaaH tiles) in one launch: work-groups [0, nk1) are K1
// blocks, [nk1p, nk1p + nk2) TAA tiles (nk1p = nk1 rounded up to the 8 XCDs;
// the ones between exit).  The in-order dispatch runs the tiles in K1's
// tail, where its last work-groups leave CUs idle, and a frame costs one
// launch.
//   SAME = false (bmfr_process_sequence): K1 of frame f with K2 of frame
//     f - 1, which reads frame f - 1's state (K1 of f does not write it:
//     double-buffered) and frame f - 2's TAA output.
//   SAME = true (bmfr_process_frame): K1 and K2 of one frame; a tile waits
//     for the K1 blocks under its footprint (completion flags) and reads
//     their outputs device-coherent.  Work-groups of one XCD are dispatched
//     in order, so every K1 block a waiting tile needs has been dispatched:
//     the waits end.
template <int NS, int FS, class IN, bool SAME = false, bool FAST = false, bool F32 = false>
__global__ __launch_bounds__(kK1Threads, (min_waves<FS, F32, FAST>())) void k_fused_cols_taa(Params P, K1Args A, Params P2,
                                                                                    TaaArgs T, int nk1, int nk1p) {
    __shared__ union {
        Lds<NS + FS + 3, kNW, F32> k1;
        FrameTaaLds<kK1Threads> k2;
    } U;
    const int b = blockIdx.x;
    if (b < nk1) k1_cols_body<NS, FS, IN, SAME, kNW, FAST, F32>(P, A, U.k1, xcd_swizzle(b, nk1));
    else if (b >= nk1p) frame_taa_part<IN, SAME, kK1Threads>(P2, T, b, nk1p, U.k2);
}

}  // namespace cols

// The column-split kernels of one tmp_data precision, compiled in their own
// translation unit (bmfr_fused_cols_f32.hip includes this file with
// BMFR_COLS_F32 = 1): K1 alone, the one-launch frame, the sequence launch.
template <bool F32>
hipError_t launch_cols_k1(const Params& P, hipStream_t st, const FusedArgs& A);
template <bool F32>
hipError_t launch_cols_frame_one(const Params& P, hipStream_t st, const FusedArgs& A);
template <bool F32>
hipError_t launch_cols_k1_taa(const Params& P, hipStream_t st, const FusedArgs* A, const Params& P2,
                              const FusedArgs* A2);

#ifndef BMFR_COLS_F32
#define BMFR_COLS_F32 0
#endif
constexpr bool kColsF32 = BMFR_COLS_F32;

// The launchers below differ between the two translation units (kColsF32)
// under the same names: internal linkage, or the linker keeps one TU's copy
// of each inline go() for both.
namespace {

// The column-split kernels' template arguments from the run-time parameters:
// FS (6 or 9 scaled features), the input element type, fast_fit.
// f32 tmp_data runs the exact fit row-split (bmfr_fused.hip: K1 -4 % against
// the column split's, whose exact fit needs 145 VGPRs, three waves per SIMD)
// unless -DBMFR_F32_COLS_EXACT=1; fast_fit column-split (K1 -8 %).
#ifndef BMFR_F32_COLS_EXACT
#define BMFR_F32_COLS_EXACT 0
#endif
constexpr bool kColsExact = !kColsF32 || BMFR_F32_COLS_EXACT;

// false (nothing launched): a configuration this translation unit has no
// kernel for -- the f32 unit compiles only the fast fit, so a strict f32
// context that reached it without fused_cols_supported gets an error, never
// the non-reference fit.
template <template <int, class, bool> class L, class... Args>
bool dispatch_cols(const Params& Q, Args&&... args) {
    if constexpr (kColsExact) {
        if (Q.scaled == 6) {
            if (Q.input_half) Q.fast_fit ? L<6, _Float16, true>::go(args...) : L<6, _Float16, false>::go(args...);
            else Q.fast_fit ? L<6, float, true>::go(args...) : L<6, float, false>::go(args...);
        } else {
            if (Q.input_half) Q.fast_fit ? L<9, _Float16, true>::go(args...) : L<9, _Float16, false>::go(args...);
            else Q.fast_fit ? L<9, float, true>::go(args...) : L<9, float, false>::go(args...);
        }
    } else {
        if (!Q.fast_fit) return false;
        if (Q.scaled == 6) Q.input_half ? L<6, _Float16, true>::go(args...) : L<6, float, true>::go(args...);
        else Q.input_half ? L<9, _Float16, true>::go(args...) : L<9, float, true>::go(args...);
    }
    return true;
}

template <int FS, class IN, bool FAST>
struct LaunchCols {
    static void go(const Params& P, hipStream_t st, const FusedArgs& A) {
        hipLaunchKernelGGL((cols::k_fused_cols<4, FS, IN, FAST, kColsF32>), dim3(k1_blocks(P)),
                           dim3(cols::kK1Threads), 0, st, P, k1_args(A));
    }
};

template <int FS, class IN, bool FAST>
struct LaunchFrameOne {
    static void go(const Params& P, hipStream_t st, const FusedArgs& A) {
        const int nk1 = P.ring < 0 || P.nbx <= 0 || P.nby <= 0 ? 0 : k1_blocks(P), nk1p = (nk1 + 7) & ~7;
        const int nk2 = frame_taa_tiles<cols::kK1Threads>(P);
        hipLaunchKernelGGL((cols::k_fused_cols_taa<4, FS, IN, true, FAST, kColsF32>), dim3(nk1p + nk2),
                           dim3(cols::kK1Threads), 0, st, P, k1_args(A), P, taa_args(A), nk1, nk1p);
    }
};

template <int FS, class IN, bool FAST>
struct LaunchColsTaa {
    static void go(const Params& P, hipStream_t st, const FusedArgs* A, const Params& P2, const FusedArgs* A2) {
        const int nk1 = A ? k1_blocks(P) : 0, nk1p = (nk1 + 7) & ~7;
        const int nk2 = A2 ? frame_taa_tiles<cols::kK1Threads>(P2) : 0;
        if (nk1 + nk2 == 0) return;
        const TaaArgs T = A2 ? taa_args(*A2) : TaaArgs{};
        hipLaunchKernelGGL((cols::k_fused_cols_taa<4, FS, IN, false, FAST, kColsF32>), dim3(nk2 ? nk1p + nk2 : nk1),
                           dim3(cols::kK1Threads), 0, st, A ? P : P2, k1_args(A ? *A : *A2), A2 ? P2 : P, T, nk1,
                           nk1p);
    }
};

}  // namespace

template <>
hipError_t launch_cols_k1<kColsF32>(const Params& P, hipStream_t st, const FusedArgs& A) {
    if (!dispatch_cols<LaunchCols>(P, P, st, A)) return hipErrorInvalidValue;
    return hipGetLastError();
}
template <>
hipError_t launch_cols_frame_one<kColsF32>(const Params& P, hipStream_t st, const FusedArgs& A) {
    if (!dispatch_cols<LaunchFrameOne>(P, P, st, A)) return hipErrorInvalidValue;
    return hipGetLastError();
}
template <>
hipError_t launch_cols_k1_taa<kColsF32>(const Params& P, hipStream_t st, const FusedArgs* A, const Params& P2,
                                        const FusedArgs* A2) {
    if (!dispatch_cols<LaunchColsTaa>(A ? P : P2, P, st, A, P2, A2)) return hipErrorInvalidValue;
    return hipGetLastError();
}

#if !BMFR_COLS_F32
// f32 tmp_data with fast_fit runs the column-split K1 too
// (bmfr_fused_cols_f32.hip); -DBMFR_F32_ROWS=1 keeps the row-split K1 of
// bmfr_fused.hip for it (A/B).
#ifndef BMFR_F32_ROWS
#define BMFR_F32_ROWS 0
#endif
bool fused_cols_supported(const Params& P) {
    return (P.half_tmp || (!BMFR_F32_ROWS && (P.fast_fit || BMFR_F32_COLS_EXACT))) && fused_supported(P);
}

bool seq_fused_supported(const Params& P) { return fused_cols_supported(P) && P.ring == 0; }
// Untiled frames, a tiled context's whole frame and its border launch (the
// ring of K1 blocks + the tile's TAA; the last work-group forwards the reach
// report).
bool frame_fused_supported(const Params& P) { return fused_supported(P); }

hipError_t launch_fused_frame_one(const Params& P, hipStream_t st, const FusedArgs& A) {
    if (!fused_cols_supported(P)) return launch_fused_rows_frame_one(P, st, A);  // f32 tmp_data, BMFR_F32_ROWS
    return P.half_tmp ? launch_cols_frame_one<false>(P, st, A) : launch_cols_frame_one<true>(P, st, A);
}

hipError_t launch_fused_k1_taa(const Params& P, hipStream_t st, const FusedArgs* A, const Params& P2,
                               const FusedArgs* A2) {
    return (A ? P : P2).half_tmp ? launch_cols_k1_taa<false>(P, st, A, P2, A2)
                                 : launch_cols_k1_taa<true>(P, st, A, P2, A2);
}

hipError_t launch_fused_k1_cols(const Params& P, hipStream_t st, const FusedArgs& A) {
    return P.half_tmp ? launch_cols_k1<false>(P, st, A) : launch_cols_k1<true>(P, st, A);
}
#endif

}  // namespace bmfr
