// bmfr_wave.h -- one-wave-per-block building blocks (gfx950).
//
// A 32x32 block is owned by ONE wave64: lane l holds rows r = l + 64*j,
// j = 0..15.  Upstream's fitter work-item t (256 per block, bmfr.cl:487-507)
// owns rows t + 256*s, i.e. t = l + 64*m with j = m + 4*s, so every
// per-work-item partial AND the first tree step (256 -> 64, bmfr.cl:32-33)
// are in-register here.  The remaining steps (64 -> 8 -> 1) run on DPP row
// shifts, gfx950's permlane16/32 swaps and readlanes, in upstream's exact
// association -- no LDS, no barriers.
#pragma once

#include "bmfr_kernels.h"

namespace bmfr {

// Work-group barrier ordering LDS only: __syncthreads() also orders global
// memory, i.e. waits for every outstanding global load of the wave
// (vmcnt(0)) -- this one lets loads stay in flight across the barrier.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// lane l <- lane l+8 within its 16-lane row (valid for l % 16 < 8)
__device__ __forceinline__ float dpp_shl8(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x108, 0xf, 0xf, true));
}
// lane l <- lane l-1 within its 16-lane row (valid for l % 16 > 0)
__device__ __forceinline__ float dpp_shr1(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, true));
}
// lanes 0..15 <- lanes 16..31 (permlane16_swap: odd rows of arg0 <-> even rows of arg1)
__device__ __forceinline__ float swap16_down(float v) {
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
    return __int_as_float(p[1]);
}
// lanes 0..31 <- lanes 32..63
__device__ __forceinline__ float swap32_down(float v) {
    const auto p = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
    return __int_as_float(p[1]);
}

// Step 3 of a sum (64 -> 8, bmfr.cl:35-36) for lanes 0..7:
// s[i] + ((((((s[i+8] + s[i+16]) + s[i+24]) + s[i+32]) + s[i+40]) + s[i+48]) + s[i+56]).
// Rows R0..R3 = lanes 0-15 .. 48-63.  One permlane16 swap gives
// e = (R0, R0, R2, R2) and o = (R1, R1, R3, R3) (s's even rows stay where
// they are, so only one copy of s is made); the running sum is formed on
// lanes 0-7 over R0's upper half and R1, moved to lanes 32-39 to take R2 and
// R3 there, and moved back for s[i]: 7 adds (4 with a fused DPP row shift),
// three permlane swaps, two moves.
__device__ __forceinline__ float sum_step3(float s) {
    const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_int(s), __float_as_int(s), false, false);
    const float e = __int_as_float(sw[0]), o = __int_as_float(sw[1]);
    const float lo = (dpp_shl8(e) + o) + dpp_shl8(o);  // lanes 0-7: (s[i+8] + s[i+16]) + s[i+24]
    const int junk = __builtin_nondeterministic_value(0);
    const float up = __int_as_float(__builtin_amdgcn_permlane32_swap(junk, __float_as_int(lo), false, false)[0]);
    // lanes 32-39: (((lo + s[i+32]) + s[i+40]) + s[i+48]) + s[i+56]
    const float hi = (((up + e) + dpp_shl8(e)) + o) + dpp_shl8(o);
    // (o is dead by now: its lower half takes hi's upper half)
    const float down =
        __int_as_float(__builtin_amdgcn_permlane32_swap(__float_as_int(hi), __float_as_int(o), false, false)[1]);
    return e + down;  // lanes 0-7
}

// Steps 64 -> 8 -> 1 of parallel_reduction_{sum,max,min} (bmfr.cl:35-42,
// 55-63, 77-85) on the 64 step-2 values s (one per lane).  Wave-uniform result.
template <RedOp OP>
__device__ __forceinline__ float wave_tree(float s) {
    if constexpr (OP == RedOp::Sum) {
        // Step 4, ((x0 + x1) + x2) ... + x7 over lanes 0..7, as a serial DPP
        // scan: after pass k, lane k holds the sum of x0..xk (one DPP op per
        // pass, instead of a readlane + a scalar-operand op per term).
        const float x = sum_step3(s);
        float r = x;
#pragma unroll
        for (int k = 1; k < 8; ++k) r = dpp_shr1(r) + x;
        return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r), 7));
    } else {
        // (min / max: a DPP-moved operand of fmaxf / fminf is first
        // canonicalised, so the plain form is as short)
        const float a = dpp_shl8(s);       // s[l+8]
        const float b = swap16_down(s);    // s[l+16]
        const float c = dpp_shl8(b);       // s[l+24]
        const float d = swap32_down(s);    // s[l+32]
        const float e = dpp_shl8(d);       // s[l+40]
        const float f = swap16_down(d);    // s[l+48]
        const float h = dpp_shl8(f);       // s[l+56]
        const float x = red<OP>(red<OP>(red<OP>(red<OP>(red<OP>(red<OP>(red<OP>(s, a), b), c), d), e), f), h);
        float r = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 0));
#pragma unroll
        for (int k = 1; k < 8; ++k) r = red<OP>(r, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), k)));
        return r;
    }
}

// Step 2 (256 -> 64, bmfr.cl:32-33 / 51-53 / 73-75) on the four partials of
// upstream work-items l, l+64, l+128, l+192.
template <RedOp OP>
__device__ __forceinline__ float step2(const float (&p)[4]) {
    if constexpr (OP == RedOp::Sum) return p[0] + ((p[1] + p[2]) + p[3]);
    else return red<OP>(red<OP>(red<OP>(p[0], p[1]), p[2]), p[3]);
}

// bmfr_config.fast_fit: the wave's sum / max / min of the four partials per
// lane as a butterfly -- quad swaps, half-row and row mirrors by DPP, then the
// four rows folded by row-broadcast DPP: 6 dependent steps instead of
// upstream's ~20-step association (wave_tree), so NOT upstream's rounding
// order; the result is lane 63's, as a scalar.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
// Rows folded into lane 63 by two row-broadcast DPP steps (rows 1, 3 take
// lane 15 of the row before; rows 2, 3 take lane 31), read out to a scalar:
// three fewer VALU instructions than permlane swaps, and for a sum the same
// association, (r0 + r1) + (r2 + r3), bit for bit.  Inline asm (the compiler
// keeps a row-masked row_bcast as a separate mov + op), each step carrying
// the two wait states its DPP source needs after a VALU write.
template <RedOp OP>
__device__ __forceinline__ float fold_rows(float s) {
    if constexpr (OP == RedOp::Sum) {
        asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf" : "+v"(s));
        asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf" : "+v"(s));
    } else if constexpr (OP == RedOp::Max) {
        asm("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf" : "+v"(s));
        asm("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf" : "+v"(s));
    } else {
        asm("s_nop 1\n\tv_min_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf" : "+v"(s));
        asm("s_nop 1\n\tv_min_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf" : "+v"(s));
    }
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), 63));
}
template <RedOp OP>
__device__ __forceinline__ float wave_reduce_fast(float s) {
    if constexpr (OP == RedOp::Sum) {  // (the compiler fuses these into v_add_f32_dpp)
        s = s + dpp_mov<0xB1>(s);   // quad_perm [1, 0, 3, 2]
        s = s + dpp_mov<0x4E>(s);   // quad_perm [2, 3, 0, 1]
        s = s + dpp_mov<0x141>(s);  // row_half_mirror
        s = s + dpp_mov<0x140>(s);  // row_mirror: every lane holds its row's sum
    } else {
        // min / max as fused DPP ops in asm: fmaxf / fminf on a DPP-moved
        // operand become mov 0, mov_dpp, canonicalise, op (the operands here
        // are features, never NaN: phase 1 maps NaN to 0)
#define BMFR_DPP_MINMAX(ctrl)                                                                          \
    if constexpr (OP == RedOp::Max) asm("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 " ctrl " row_mask:0xf bank_mask:0xf" \
                                        : "+v"(s));                                                    \
    else asm("s_nop 1\n\tv_min_f32_dpp %0, %0, %0 " ctrl " row_mask:0xf bank_mask:0xf" : "+v"(s))
        BMFR_DPP_MINMAX("quad_perm:[1,0,3,2]");
        BMFR_DPP_MINMAX("quad_perm:[2,3,0,1]");
        BMFR_DPP_MINMAX("row_half_mirror");
        BMFR_DPP_MINMAX("row_mirror");
#undef BMFR_DPP_MINMAX
    }
    return fold_rows<OP>(s);  // uniform: a scalar
}
template <RedOp OP>
__device__ __forceinline__ float wave_reduce_fast(const float (&p)[4]) {
    return wave_reduce_fast<OP>(red<OP>(red<OP>(p[0], p[1]), red<OP>(p[2], p[3])));
}

// K independent sums at once, for one wave: lane l holds the step-2 values
// v[k] (= s[l] of reduction k).  Steps 64 -> 8 -> 1 (bmfr.cl:35-42) run as an
// LDS transpose: lane (k, i) forms e_k[i] = s[i] + (((s[i+8] + s[i+16]) + ...)
// + s[i+56]), lane k forms ((e_k[0] + e_k[1]) + ...) + e_k[7].  About 2K+40
// instructions for all K sums, against ~30 per sum for wave_tree.
// scratch: >= K*72 + K*8 + K floats of LDS.
constexpr int kRowStride = 72;  // 64 + 8: lanes (k, i) of one 32-lane group hit distinct banks
template <int K>
__device__ __forceinline__ void lds_batch_sum(float (&v)[K], float* __restrict__ scratch, int l) {
    float* S = scratch;
    float* E = scratch + K * kRowStride;
    float* R = E + K * 8;
#pragma unroll
    for (int k = 0; k < K; ++k) S[k * kRowStride + l] = v[k];
    __syncthreads();
#pragma unroll
    for (int base = 0; base < K * 8; base += 64) {
        const int idx = base + l;
        if (idx < K * 8) {
            const float* row = S + (idx >> 3) * kRowStride + (idx & 7);
            float acc = row[8];
#pragma unroll
            for (int j = 2; j < 8; ++j) acc = acc + row[8 * j];
            E[idx] = row[0] + acc;
        }
    }
    __syncthreads();
    if (l < K) {
        float r = E[l * 8];
#pragma unroll
        for (int i = 1; i < 8; ++i) r = r + E[l * 8 + i];
        R[l] = r;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = R[k];
}

// Packed-half design matrix: A[f][j] for j = 0..15 in 8 registers per column.
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

template <int B>
struct HalfMatrix {
    h2 v[B][8];
    __device__ __forceinline__ float get(int f, int j) const { return (float)v[f][j >> 1][j & 1]; }
    __device__ __forceinline__ void set(int f, int j, float x) { v[f][j >> 1][j & 1] = (_Float16)x; }
    // Zero-instruction fence: the compiler must assume column f changed, so it
    // re-unpacks it on the next get() instead of keeping f32 copies alive
    // across a reduction (the difference between fitting in VGPRs and spilling).
    __device__ __forceinline__ void fence(int f) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(v[f][i]));
    }
};

}  // namespace bmfr
