// bmfr_device.h -- device-side building blocks of the BMFR kernels (gfx950).
//
// Arithmetic contract: every helper here rounds exactly like the reference
// kernels in /root/reference/opencl/bmfr.cl do when compiled for gfx950 with
// IEEE-strict OpenCL options (no contraction of user code, correctly rounded
// division and sqrt).  The library is built with -ffp-contract=off, so an
// expression `a * b + c` is two rounded operations; __builtin_fmaf appears
// only where the reference's OpenCL library itself fuses (dot(), whose ROCm
// device-libs implementation is an fmuladd chain).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bmfr_params.h"

namespace bmfr {

// BLOCK_OFFSETS, bmfr.cl:267-285: per-frame shift of the 32x32 block grid.
__constant__ static const int2 kBlockOffsets[16] = {
    {-14, -14}, {4, -6}, {-8, 14}, {8, 0}, {-10, -8}, {2, 12}, {12, -12}, {-10, 0},
    {12, 14}, {-8, -16}, {6, 6}, {-2, -2}, {6, -14}, {-16, 12}, {14, -4}, {-6, 4}};

struct f3 {
    float x, y, z;
};

// One float3 of an interleaved RGB plane as a single dwordx3 access.
struct __attribute__((packed, aligned(4))) f3mem {
    float x, y, z;
};

// Byte offsets of pixel i in planes of 12- and 6-byte elements: i * 3 as one
// shift-and-add, then a shift -- two full-rate instructions, where the
// compiler turns i * 12 into v_mul_lo_u32 (a multi-pass integer multiply).
// i may reach 2^25 (8K frames), so a 24-bit multiply cannot do it.  Inline
// asm so the shift-and-add is not folded back into a multiply; it reads and
// writes plain integer VGPRs (no DOT / transcendental producer involved).
__device__ __forceinline__ uint32_t times3(uint32_t i) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 1, %1" : "=v"(r) : "v"(i));
    return r;
}
__device__ __forceinline__ uint32_t x12(uint32_t i) { return times3(i) << 2; }
__device__ __forceinline__ uint32_t x6(uint32_t i) { return times3(i) << 1; }

// Device-coherent plane accesses, for data one work-group of a launch hands
// to another that may run on another XCD (each XCD's L2 is write-back and
// not coherent with the others'): raw buffer loads / stores with the sc1
// cache policy, which the memory model uses for agent-scope atomics --
// coherent at device scope without flushing or invalidating any L2.
typedef __amdgpu_buffer_rsrc_t CohPlane;
__device__ __forceinline__ CohPlane coh_plane(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, -1, 0x00020000);
}
#ifdef BMFR_PROBE_NOSC1
constexpr int kSc1 = 0;  // timing probe only (tools/ab.py variants): plain hand-off, results not guaranteed
#else
constexpr int kSc1 = 16;  // buffer instruction cache-policy bit SC1
#endif
__device__ __forceinline__ f3 ld3_coh(CohPlane r, uint32_t i) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b96(r, x12(i), 0, kSc1);
    return f3{__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2])};
}
__device__ __forceinline__ void st3_coh(CohPlane r, uint32_t i, f3 v) {
    typedef unsigned u3 __attribute__((ext_vector_type(3)));
    __builtin_amdgcn_raw_buffer_store_b96(u3{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z)}, r,
                                          x12(i), 0, kSc1);
}
__device__ __forceinline__ float2 ld2_coh(CohPlane r, uint32_t i) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, i * 8u, 0, kSc1);
    return make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
}
__device__ __forceinline__ void st2_coh(CohPlane r, uint32_t i, float2 v) {
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(u2{__float_as_uint(v.x), __float_as_uint(v.y)}, r, i * 8u, 0, kSc1);
}

// Stores only some lanes perform, without a branch: raw buffer stores whose
// discarded lanes get an out-of-range offset (the buffer range check drops
// the write; a plane is far below 4 GiB, validate() in bmfr_capi.hip).  A
// store inside a divergent branch makes the compiler's s_waitcnt for an OLDER
// load after the branch conservative -- the count must hold on the path that
// skipped the stores, so it waits for the stores' acknowledgement too (K1's
// phase 1: each item's owner stores held up the next item's reprojection
// until they were written back).  Issued on every path, they are counted
// exactly.  `sc1`: the cache policy of the device-coherent hand-off (COH).
typedef __amdgpu_buffer_rsrc_t DropPlane;
__device__ __forceinline__ DropPlane drop_plane(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
constexpr uint32_t kDropOff = 0x80000000u;  // any offset past the range
template <int AUX = 0>
__device__ __forceinline__ void st3_drop(DropPlane r, uint32_t i, bool keep, f3 v) {
    typedef unsigned u3 __attribute__((ext_vector_type(3)));
    __builtin_amdgcn_raw_buffer_store_b96(u3{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z)}, r,
                                          keep ? x12(i) : kDropOff, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void st2_drop(DropPlane r, uint32_t i, bool keep, float2 v) {
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(u2{__float_as_uint(v.x), __float_as_uint(v.y)}, r,
                                          keep ? i * 8u : kDropOff, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void st1_drop(DropPlane r, uint32_t i, bool keep, uint8_t v) {
    __builtin_amdgcn_raw_buffer_store_b8(v, r, keep ? i : kDropOff, 0, AUX);
}

// Plane elements by pixel index i.  The address is the plane's base (a kernel
// argument: uniform, in SGPRs) plus a 32-bit byte offset (one VGPR) -- the
// SGPR-base form of the global memory instructions -- so the planes read at
// one pixel share a single offset register and no 64-bit address arithmetic
// is spent per access.  Every plane is under 4 GiB (validate() in
// bmfr_capi.hip bounds the image), so i * element size fits 32 bits.
template <class T>
__device__ __forceinline__ const T* at_byte(const T* b, uint32_t off) {
    return reinterpret_cast<const T*>(reinterpret_cast<const char*>(b) + off);
}
template <class T>
__device__ __forceinline__ T* at_byte(T* b, uint32_t off) {
    return reinterpret_cast<T*>(reinterpret_cast<char*>(b) + off);
}
template <class T>
__device__ __forceinline__ T ld_px(const T* b, uint32_t i) {
    return *at_byte(b, i * (uint32_t)sizeof(T));
}
template <class T>
__device__ __forceinline__ void st_px(T* b, uint32_t i, T v) {
    *at_byte(b, i * (uint32_t)sizeof(T)) = v;
}
__device__ __forceinline__ f3 ld3(const float* __restrict__ b, uint32_t i) {
    const f3mem v = *reinterpret_cast<const f3mem*>(at_byte(b, x12(i)));
    return f3{v.x, v.y, v.z};
}
__device__ __forceinline__ void st3(float* __restrict__ b, uint32_t i, f3 v) {
    *reinterpret_cast<f3mem*>(at_byte(b, x12(i))) = f3mem{v.x, v.y, v.z};
}

// One pixel of an input plane of element type IN (float: the reference's
// float3 layout; _Float16: half3, 6 bytes per pixel), widened exactly to f32.
struct __attribute__((packed, aligned(2))) h3mem {
    _Float16 x, y, z;
};
template <class IN>
__device__ __forceinline__ f3 ld3in(const float* __restrict__ b, uint32_t i) {
    if constexpr (sizeof(IN) == 2) {
        const h3mem v = *reinterpret_cast<const h3mem*>(at_byte(b, x6(i)));
        return f3{(float)v.x, (float)v.y, (float)v.z};
    } else {
        return ld3(b, i);
    }
}

// The same pixel as loaded (In3<float> = f3, In3<_Float16> = the 6 bytes),
// widened by widen() where it is used: a conversion right after a load makes
// the wave wait for that load, so the loads a pipeline stage issues together
// stay raw until the stage consumes them.
template <class IN>
struct In3 {
    f3 v;
};
struct __attribute__((packed, aligned(2))) h3raw {  // h3mem's bytes: x | y << 16, z
    uint32_t xy;
    uint16_t z;
};
template <>
struct In3<_Float16> {
    h3raw v;  // kept whole (not split into halves) until widened
};
template <class IN>
__device__ __forceinline__ In3<IN> ld3raw(const float* __restrict__ b, uint32_t i) {
    if constexpr (sizeof(IN) == 2) return In3<IN>{*reinterpret_cast<const h3raw*>(at_byte(b, x6(i)))};
    else return In3<IN>{ld3(b, i)};
}
// Two horizontally adjacent half3 pixels (i, i + 1) of a plane in one 12-byte
// load: .x = pixel i's x | y << 16, .y = its z | pixel i + 1's x << 16, .z =
// pixel i + 1's y | z << 16.
struct __attribute__((packed, aligned(2))) h3pair {
    uint32_t a, b, c;
};
__device__ __forceinline__ h3pair ld3pair_h(const float* __restrict__ b, uint32_t i) {
    return *reinterpret_cast<const h3pair*>(at_byte(b, x6(i)));
}
__device__ __forceinline__ f3 widen(const In3<float>& r) { return r.v; }
__device__ __forceinline__ f3 widen(const In3<_Float16>& r) {
    return f3{(float)__builtin_bit_cast(_Float16, (uint16_t)(r.v.xy & 0xffffu)),
              (float)__builtin_bit_cast(_Float16, (uint16_t)(r.v.xy >> 16)), (float)__builtin_bit_cast(_Float16, r.v.z)};
}

// OpenCL dot() as ROCm's opencl.bc implements it (fmuladd chain).
__device__ __forceinline__ float dot3(f3 a, f3 b) {
    return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x));
}
__device__ __forceinline__ float dot4(float a0, float a1, float a2, float a3, float b0, float b1,
                                      float b2, float b3) {
    return __builtin_fmaf(a3, b3, __builtin_fmaf(a2, b2, __builtin_fmaf(a1, b1, a0 * b0)));
}

// mirror(), bmfr.cl:207-216.
__device__ __forceinline__ int mirror(int i, int size) {
    return i < 0 ? -i - 1 : (i >= size ? 2 * size - i - 1 : i);
}

// scale(), bmfr.cl:200-205.
__device__ __forceinline__ float scale(float v, float mn, float mx) {
    const float d = mx - mn;
    return fabsf(d) > 1.0f ? (v - mn) / d : v - mn;
}

// vstore_half / vload_half round trip (round to nearest even), bmfr.cl:255-258.
__device__ __forceinline__ float round_half(float v) { return (float)(_Float16)v; }

// random() + add_random(), bmfr.cl:161-182.  NOISE_AMOUNT is a double
// literal upstream, so the noise and the add are double.
__device__ __forceinline__ float hash_random(uint32_t a) {
    a = (a + 0x7ed55d16u) + (a << 12);
    a = (a ^ 0xc761c23cu) ^ (a >> 19);
    a = (a + 0x165667b1u) + (a << 5);
    a = (a + 0xd3a2646cu) ^ (a << 9);
    a = (a + 0xfd7046c5u) + (a << 3);
    a = (a ^ 0xb55a4f09u) ^ (a >> 16);
    return (float)a / 4294967296.0f;  // convert_float(UINT_MAX) == 2^32
}
__device__ __forceinline__ float add_random(float v, double noise2, int seed) {
    const float r = hash_random((uint32_t)seed) - 0.5f;
    return (float)((double)v + noise2 * (double)r);
}

// One FEATURE_BUFFERS entry (bmfr.cl:448-453, 727-729).
__device__ __forceinline__ float feature_value(int code, f3 n, f3 p) {
    switch (code) {
        case kFeatOne: return 1.f;
        case kFeatNx: return n.x;
        case kFeatNy: return n.y;
        case kFeatNz: return n.z;
        case kFeatPx: return p.x;
        case kFeatPy: return p.y;
        case kFeatPz: return p.z;
        case kFeatPx2: return p.x * p.x;
        case kFeatPy2: return p.y * p.y;
        case kFeatPz2: return p.z * p.z;
        case kFeatPx3: return p.x * p.x * p.x;
        case kFeatPy3: return p.y * p.y * p.y;
        case kFeatPz3: return p.z * p.z * p.z;
        default: return 0.f;
    }
}

// RGB <-> YCoCg, bmfr.cl:184-198 (dot-based, hence fma chains).
__device__ __forceinline__ f3 rgb_to_ycocg(f3 c) {
    return f3{dot3(c, f3{1.f, 2.f, 1.f}), dot3(c, f3{2.f, 0.f, -2.f}), dot3(c, f3{-1.f, 2.f, -1.f})};
}
__device__ __forceinline__ f3 ycocg_to_rgb(f3 c) {
    return f3{dot3(c, f3{0.25f, 0.25f, -0.25f}), dot3(c, f3{0.25f, 0.f, 0.25f}),
              dot3(c, f3{0.25f, -0.25f, -0.25f})};
}

// v_min_f32 / v_max_f32 as written.  fminf / fmaxf on values the compiler
// cannot prove canonical (loaded from LDS or memory) get a quieting
// v_max_f32 x, x, x per operand first; the instruction itself already
// returns the other operand for a quiet NaN, and arithmetic never makes a
// signalling one, so results are identical for every value reaching here.
__device__ __forceinline__ float vmin(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vmax(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// min(min(a, b), c) / max(max(a, b), c) in one instruction: bit for bit the
// nested two-operand forms on gfx950 for every input incl. signed zeros,
// infinities, quiet NaNs and denormals (tools/minmax3_check.hip, 64M triples).
__device__ __forceinline__ float vmin3(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float vmax3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// The same with a wave-uniform first operand (a constant kept in an SGPR).
__device__ __forceinline__ float vmin3s(float s, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "s"(s), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float vmax3s(float s, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "s"(s), "v"(b), "v"(c));
    return r;
}


// Correctly rounded a / b given y = RN(1/b): one Markstein correction step
// (r = a - q*b is exact under FMA; q + r*y rounds to RN(a/b) when a, b, 1/b
// and a/b are normal).  Used where one divisor serves several dividends, in
// place of the ~10-instruction generic division.  Callers guarantee finite a
// and finite, nonzero b with a normal reciprocal (see div_shared for the
// guarded form).
__device__ __forceinline__ float div_by_recip(float a, float b, float y) {
    const float q = a * y;
    const float r = __builtin_fmaf(-q, b, a);
    return __builtin_fmaf(r, y, q);
}
// RN(1/x) as the hardware reciprocal plus one FMA Newton step: equal to the
// correctly rounded 1.0f / x for every float with |x| in [2^-125, 2^126)
// (tools/rcp_check.hip, all 4.2e9 such floats on the device) -- three
// instructions instead of the ~10 of IEEE division.  Only for operands
// provably inside that range (the spp blend factors, x in [1, 257)).
__device__ __forceinline__ float rcp_nr(float x) {
    const float y = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(__builtin_fmaf(-x, y, 1.f), y, y);
}

// Guarded form: where the correction step itself breaks down (a infinite,
// b zero or infinite: r becomes NaN) the first quotient q = a * (1/b) already
// is IEEE a / b, so use it.
__device__ __forceinline__ float div_shared(float a, float b, float y) {
    const float q = a * y;
    const float r = __builtin_fmaf(-q, b, a);
    const float q1 = __builtin_fmaf(r, y, q);
    return q1 == q1 ? q1 : q;
}

}  // namespace bmfr
