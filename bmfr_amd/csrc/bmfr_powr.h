// The tone map's powr(x, 0.454545f) (bmfr.cl:854), correctly rounded.
//
// OpenCL leaves powr's rounding to the device (up to 16 ulp), so the
// reference fixes no bit pattern here; the CPU oracle takes the correctly
// rounded value ((float)pow in double, oracle/bmfr_oracle.c).  This is that
// value, computed in ~20 instructions instead of the device library's ~130
// (the extended-precision log/exp of __ocml_powr_f32), which made the tone
// map 55 % of K2's VALU work:
//   x = m 2^e, m in [0.5, 1):  x^c = 2^(e c) * rc_j^-c * (1 + u)^c,
//   u = m rc_j - 1 (exact, |u| < 2^-8), (1 + u)^c a degree-4 series,
// all in double (relative error < 2^-45), rounded once to float.  A result
// whose double lies within 2^10 double ulps of a float rounding midpoint
// (about one input in 2^18) is recomputed with the device library's f64 pow.
// tools/powr_check.hip checks every float in (0, 1) against (float)pow.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bmfr_powr_tables.h"

extern "C" __device__ double __ocml_pow_f64(double, double);
extern "C" __device__ float __ocml_powr_f32(float, float);

// min(max(powr(max(0, p), 0.454545f), 0), 1) (bmfr.cl:853-855), with the
// tables read from `tE` / `tRP`: kPowrE / kPowrRP in global memory, or a
// work-group's copy in LDS (bmfr_powr_tables_to_lds), which keeps the two
// lookups per channel off the vector-memory path.
// The table part alone: the result when *rare is false; when *rare is true
// (the double lies within 2^10 double ulps of a float rounding midpoint) the
// caller must take gamma_clamped instead.  Branch-free, so a caller can issue
// the lookups of several values back to back and fix the rare ones after.
__device__ __forceinline__ float gamma_table(float p, bool& rare, const double* tE = kPowrE,
                                             const double2* tRP = kPowrRP) {
    const bool pos = p > 0.f, below = p < 1.f;
    const float x = pos && below ? p : 0.5f;
    const float m = __builtin_amdgcn_frexp_mantf(x);
    const int e = __builtin_amdgcn_frexp_expf(x);
    const int j = (int)(__float_as_uint(m) >> (23 - BMFR_POWR_J_BITS)) & ((1 << BMFR_POWR_J_BITS) - 1);
    const double2 rp = tRP[j];
    const double ep = tE[e - BMFR_POWR_E_MIN] * rp.y;
    const double u = __builtin_fma((double)m, rp.x, -1.0);
    double q = __builtin_fma(BMFR_POWR_A4, u, BMFR_POWR_A3);
    q = __builtin_fma(q, u, BMFR_POWR_A2);
    q = __builtin_fma(q, u, BMFR_POWR_A1);
    const double r = __builtin_fma(ep, u * q, ep);
    const uint32_t low = (uint32_t)__double_as_longlong(r) & 0x1FFFFFFFu;
    rare = pos && below && low - (0x10000000u - 1024u) < 2048u;
    return pos ? (below ? (float)r : 1.f) : 0.f;
}

// gamma_table of three values with the six table lookups issued together
// (a scheduling barrier keeps the compiler from spacing them out to save
// registers: each would then wait for its own LDS round trip).  Bit i of
// *rare: value i needs gamma_clamped.
__device__ __forceinline__ void gamma_table3(const float (&p)[3], float (&out)[3], uint32_t& rare,
                                             const double* tE, const double2* tRP) {
    float m[3];
    bool ok[3], pos[3], below[3];
    double2 rp[3];
    double te[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        pos[c] = p[c] > 0.f;
        below[c] = p[c] < 1.f;
        ok[c] = pos[c] && below[c];
        const float x = ok[c] ? p[c] : 0.5f;
        m[c] = __builtin_amdgcn_frexp_mantf(x);
        const int e = __builtin_amdgcn_frexp_expf(x);
        const int j = (int)(__float_as_uint(m[c]) >> (23 - BMFR_POWR_J_BITS)) & ((1 << BMFR_POWR_J_BITS) - 1);
        rp[c] = tRP[j];
        te[c] = tE[e - BMFR_POWR_E_MIN];
    }
    __builtin_amdgcn_sched_barrier(0);
    rare = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double ep = te[c] * rp[c].y;
        const double u = __builtin_fma((double)m[c], rp[c].x, -1.0);
        double q = __builtin_fma(BMFR_POWR_A4, u, BMFR_POWR_A3);
        q = __builtin_fma(q, u, BMFR_POWR_A2);
        q = __builtin_fma(q, u, BMFR_POWR_A1);
        const double r = __builtin_fma(ep, u * q, ep);
        const uint32_t low = (uint32_t)__double_as_longlong(r) & 0x1FFFFFFFu;
        rare |= (uint32_t)(ok[c] && low - (0x10000000u - 1024u) < 2048u) << c;
        out[c] = pos[c] ? (below[c] ? (float)r : 1.f) : 0.f;
    }
}

__device__ __forceinline__ float gamma_clamped(float p, const double* tE = kPowrE, const double2* tRP = kPowrRP) {
    bool rare;
    const float v = gamma_table(p, rare, tE, tRP);
    if (__builtin_expect(rare, 0)) return (float)__ocml_pow_f64((double)p, (double)0.454545f);
    return v;
}

constexpr int kPowrENum = sizeof(kPowrE) / sizeof(double), kPowrRPNum = sizeof(kPowrRP) / sizeof(double2);

// Copy the tables to LDS (all threads of the work-group; a barrier must
// follow before gamma_clamped reads them).
template <int NT>
__device__ __forceinline__ void bmfr_powr_tables_to_lds(double* sE, double2* sRP, int t) {
    for (int i = t; i < kPowrRPNum; i += NT) sRP[i] = kPowrRP[i];
    for (int i = t; i < kPowrENum; i += NT) sE[i] = kPowrE[i];
}
