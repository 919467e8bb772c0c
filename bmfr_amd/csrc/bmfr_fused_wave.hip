// bmfr_fused_wave.hip -- fused frame kernel K1, one wave64 per 32x32 block.
//
// accumulate_noisy_data -> min/max scaling -> Householder QR -> back
// substitution -> weighted_sum -> accumulate_filtered_data (+ tone map) for
// one block of the shifted grid (bmfr.cl:287-857), with the whole half-
// precision design matrix in VGPRs (packed f16 pairs) and every reduction
// done in-wave in upstream's association (bmfr_wave.h).  Bit-identical to the
// stage kernels / the reference; see tests/test_gpu_parity.py.
//
// Specialised for the canonical feature lists (FEATURE_BUFFERS entry f is
// monomial f: the reference defaults and the 3rd-order set) and half
// tmp_data; other configurations use the 4-wave kernel in bmfr_kernels.hip.
#include "bmfr_launch.h"
#include "bmfr_wave.h"

#include <utility>

namespace bmfr {

// One Householder column step (bmfr.cl:549-655) with a compile-time column
// index, so every access to the register-resident matrix is static.
template <int col, int B>
__device__ __forceinline__ void qr_column(HalfMatrix<B>& A, float* __restrict__ Rl, float* __restrict__ red,
                                          int l, const float* __restrict__ noise, double noise2) {
    constexpr int RE = B - 2;
    constexpr int J = 16;
    constexpr int cl = col;  // col_limited (feature columns only)

    // |x|^2 over rows >= cl+1 (bmfr.cl:555-569); row l + 64j.
    float p[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        float sum = 0.f;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int j = m + 4 * s;
            const float v = A.get(col, j);
            if (j > 0 || l >= cl + 1) sum = sum + v * v;
        }
        p[m] = sum;
    }
    const float sumsq = wave_tree<RedOp::Sum>(step2<RedOp::Sum>(p));
    const float ucl = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(A.get(col, 0)), cl));
    const float vlen = sqrtf(sumsq + ucl * ucl);  // bmfr.cl:582-585
    const float ucl2 = ucl - vlen;
    const float ulen2 = sumsq + ucl2 * ucl2;
    // ulen2 > 0 for any block whose columns are not all zero below the
    // diagonal (the noise of bmfr.cl:625-627 ensures it); a zero column is
    // 0/0 upstream and NaN here too.
    const float recip = 1.f / ulen2;

    // R column (bmfr.cl:574-601): rows above the diagonal and the diagonal.
    if (l < col) {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) Rl[(col * RE + l) * 3 + ch] = A.get(col, 0);
    }
    if (l == col) {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) Rl[(col * RE + col) * 3 + ch] = vlen;
    }

    float u[J];
#pragma unroll
    for (int j = 0; j < J; ++j) u[j] = A.get(col, j);
    if (l == cl) u[0] = ucl2;

    if constexpr (col == 0) {
        // Column 0 is FEATURE_BUFFERS' "1.f" (canonical feature list): after
        // the norm above, u = (-31, 1, 1, ...) and |u|^2 = 1984 exactly, so
        // RN(v*u) = v off row 0 and the update quotient RN(RN(u*c2)/1984) is
        // one uniform value per trailing column off row 0.  Same operations,
        // same roundings as the generic step.  The trailing columns get their
        // noise on first load (bmfr.cl:625-627); the noisy f32 values feed the
        // dot and the update, so each column is done on its own.
        const bool row0 = l == 0;
#pragma unroll
        for (int fb = 1; fb < B; ++fb) {
            float v[J];
#pragma unroll
            for (int j = 0; j < J; ++j) {
                v[j] = A.get(fb, j);
                if (fb < B - 3)
                    v[j] = (float)((double)v[j] + noise2 * (double)noise[(fb - 1) * kBlockPixels + l + 64 * j]);
            }
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                float sum = m == 0 ? v[0] * u[0] : v[m];
#pragma unroll
                for (int s = 1; s < 4; ++s) sum = sum + v[m + 4 * s];
                p[m] = sum;
            }
            const float c2 = 2.f * wave_tree<RedOp::Sum>(step2<RedOp::Sum>(p));
            const float q = div_by_recip(c2, ulen2, recip);  // rows with u = 1
            A.set(fb, 0, v[0] - (row0 ? div_by_recip(u[0] * c2, ulen2, recip) : q));
#pragma unroll
            for (int j = 1; j < J; ++j) A.set(fb, j, v[j] - q);
            __builtin_amdgcn_sched_barrier(0);
        }
    } else {
        // All trailing dots first (one reduction each, independent), then all
        // updates; a column's update depends only on its own dot.
        float dot[B - 1 - cl];
#pragma unroll
        for (int k = 0; k < B - 1 - cl; ++k) {
            const int fb = cl + 1 + k;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                float sum = 0.f;
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int j = m + 4 * s;
                    if (j > 0 || l >= cl) sum = sum + A.get(fb, j) * u[j];
                }
                p[m] = sum;
            }
            dot[k] = step2<RedOp::Sum>(p);
        }
#pragma unroll
        for (int fb = cl + 1; fb < B; ++fb) A.fence(fb);
        lds_batch_sum<B - 1 - cl>(dot, red, l);
#pragma unroll
        for (int k = 0; k < B - 1 - cl; ++k) {
            const int fb = cl + 1 + k;
            const float c2 = 2.f * dot[k];
#pragma unroll
            for (int j = 0; j < J; ++j)
                if (j > 0 || l >= cl) A.set(fb, j, A.get(fb, j) - div_by_recip(u[j] * c2, ulen2, recip));
        }
    }
    __builtin_amdgcn_sched_barrier(0);
}

template <int B, int... C>
__device__ __forceinline__ void qr_columns(HalfMatrix<B>& A, float* __restrict__ Rl, float* __restrict__ red,
                                           int l, const float* __restrict__ noise, double noise2,
                                           std::integer_sequence<int, C...>) {
    (qr_column<C, B>(A, Rl, red, l, noise, noise2), ...);
}

template <int NS, int FS>
__global__ __launch_bounds__(64, 3) void k_fused_wave(Params P, NoisyInputs in, Camera cam, int frame,
                                                   const float* __restrict__ albedo,
                                                   const float* __restrict__ acc_prev,
                                                   float* __restrict__ noisy_out,
                                                   uint8_t* __restrict__ spp_out,
                                                   float2* __restrict__ prev_pixel_out,
                                                   float* __restrict__ acc_out,
                                                   float* __restrict__ tone_out,
                                                   const float* __restrict__ noise) {
    constexpr int B = NS + FS + 3;
    constexpr int RE = B - 2;  // R_EDGE
    constexpr int J = 16;      // rows per lane
    __shared__ float Rl[RE * RE * 3];
    __shared__ float Wl[(B - 3) * 3];
    __shared__ float red[(B - 2) * (kRowStride + 9)];  // lds_batch_sum scratch
    __shared__ float mm[3 * (FS > 0 ? FS : 1)];          // block min, max, 1/(max-min)
    __shared__ uint32_t parked[7][64];                     // per-lane phase-1 state kept for phase 3

    const int l = threadIdx.x;
    const int g = blockIdx.x;
    const int bx = g % P.blocks_x, by = g / P.blocks_x;

    HalfMatrix<B> A;
    uint32_t owner = 0;
    uint32_t accept_bits[2] = {0u, 0u};  // 4 bits per row
    uint32_t spp_bytes[4] = {0u, 0u, 0u, 0u};

    // ---- accumulate_noisy_data (bmfr.cl:310-484) for rows l + 64j ----
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int r = l + 64 * j;
        const int gx = bx * kEdge + (r & (kEdge - 1)), gy = by * kEdge + (r >> 5);
        const NoisyItem it = noisy_item(P, in, cam, gx, gy, frame);
#pragma unroll
        for (int f = 0; f < B; ++f) {
            float v;
            if (f < B - 3) v = feature_value(f, it.n, it.p);
            else v = f == B - 3 ? it.color.x : (f == B - 2 ? it.color.y : it.color.z);
            if (__builtin_isnan(v)) v = 0.0f;
            A.set(f, j, fmaxf(fminf(v, 65504.f), -65504.f));
        }
        accept_bits[j >> 3] |= (uint32_t)it.accept << (4 * (j & 7));
        spp_bytes[j >> 2] |= (uint32_t)it.spp << (8 * (j & 3));
        if (it.owner) {
            owner |= 1u << j;
            st3(noisy_out, it.lin, it.color);
            spp_out[it.lin] = it.spp;
            prev_pixel_out[it.lin] = make_float2(it.pfx, it.pfy);
        }
        if (j & 1) __builtin_amdgcn_sched_barrier(0);  // two rows in flight at a time
    }

    parked[0][l] = owner;
    parked[1][l] = accept_bits[0];
    parked[2][l] = accept_bits[1];
#pragma unroll
    for (int i = 0; i < 4; ++i) parked[3 + i][l] = spp_bytes[i];
    __builtin_amdgcn_sched_barrier(0);
    // ---- fitter: scale position features to [min, max] (bmfr.cl:510-542) ----
#pragma unroll
    for (int f = 0; f < FS; ++f) {
        float pmx[4], pmn[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            float hi = -INFINITY, lo = INFINITY;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const float v = A.get(NS + f, m + 4 * s);
                hi = fmaxf(v, hi);
                lo = fminf(v, lo);
            }
            pmx[m] = hi;
            pmn[m] = lo;
        }
        const float bmax = wave_tree<RedOp::Max>(step2<RedOp::Max>(pmx));
        const float bmin = wave_tree<RedOp::Min>(step2<RedOp::Min>(pmn));
        const float d = bmax - bmin;
        const bool divide = fabsf(d) > 1.0f;  // scale(), bmfr.cl:200-205
        const float brcp = 1.f / d;
        if (l == 0) {
            mm[3 * f] = bmin;
            mm[3 * f + 1] = bmax;
            mm[3 * f + 2] = brcp;
        }
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const float v = A.get(NS + f, j) - bmin;
            A.set(NS + f, j, divide ? div_by_recip(v, d, brcp) : v);
        }
        __builtin_amdgcn_sched_barrier(0);
    }

    // ---- Householder QR over the feature columns (bmfr.cl:544-656) ----
    qr_columns<B>(A, Rl, red, l, noise, P.noise2, std::make_integer_sequence<int, B - 3>{});
    __builtin_amdgcn_sched_barrier(0);
    // Right-hand side: rows 0..B-4 of the colour columns (bmfr.cl:596-600).
    if (l < B - 3) {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) Rl[((RE - 1) * RE + l) * 3 + ch] = A.get(B - 3 + ch, 0);
    }
    __syncthreads();

    // ---- back substitution (bmfr.cl:658-699), one lane per channel ----
    if (l < 3) {
        const int ch = l;
        float R[RE][RE];
#pragma unroll
        for (int x = 0; x < RE; ++x)
#pragma unroll
            for (int y = 0; y <= (x < RE - 1 ? x : RE - 2); ++y) R[x][y] = Rl[(x * RE + y) * 3 + ch];
#pragma unroll
        for (int i = RE - 2; i >= 0; --i) {
            const float div = R[i][i];
#pragma unroll
            for (int x = i; x < RE; ++x) R[x][i] = R[x][i] / div;
#pragma unroll
            for (int j = i + 1; j < RE - 1; ++j) R[RE - 1][i] = R[RE - 1][i] - R[j][i];
#pragma unroll
            for (int y = 0; y <= i; ++y) R[i][y] = R[i][y] * R[RE - 1][i];
        }
#pragma unroll
        for (int id = 0; id < B - 3; ++id) Wl[id * 3 + ch] = R[RE - 1][id];
    }
    __syncthreads();

    // ---- weighted_sum + accumulate_filtered_data for owned pixels ----
    float w[(B - 3) * 3];
#pragma unroll
    for (int i = 0; i < (B - 3) * 3; ++i) w[i] = Wl[i];
    float bmin[FS > 0 ? FS : 1], bmax[FS > 0 ? FS : 1], brcp[FS > 0 ? FS : 1];
#pragma unroll
    for (int f = 0; f < FS; ++f) {
        bmin[f] = mm[3 * f];
        bmax[f] = mm[3 * f + 1];
        brcp[f] = mm[3 * f + 2];
    }
    // Derive phase-3 addresses from an opaque copy of the lane id, so the
    // compiler recomputes them instead of keeping phase 1's 64-bit pixel
    // offsets alive (in scratch) across the whole QR.
    int l3 = l;
    asm volatile("" : "+v"(l3));
    owner = parked[0][l];
    accept_bits[0] = parked[1][l];
    accept_bits[1] = parked[2][l];
#pragma unroll
    for (int i = 0; i < 4; ++i) spp_bytes[i] = parked[3 + i][l];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        if (owner & (1u << j)) {
            const int r = l3 + 64 * j;
            const int2 off = kBlockOffsets[frame & 15];
            const int px = bx * kEdge + (r & (kEdge - 1)) - kEdge / 2 + off.x;
            const int py = by * kEdge + (r >> 5) - kEdge / 2 + off.y;
            const long lin = (long)py * P.width + px;
            const f3 n = ld3(in.n_cur, lin), pos = ld3(in.p_cur, lin);
            f3 c{0.f, 0.f, 0.f};
#pragma unroll
            for (int f = 0; f < B - 3; ++f) {
                float v = feature_value(f, n, pos);
                if (f >= NS) {
                    const float d = bmax[f - NS] - bmin[f - NS];
                    v = v - bmin[f - NS];
                    if (fabsf(d) > 1.0f) v = div_by_recip(v, d, brcp[f - NS]);
                }
                c.x = c.x + w[3 * f] * v;
                c.y = c.y + w[3 * f + 1] * v;
                c.z = c.z + w[3 * f + 2] * v;
            }
            c.x = c.x < 0.f ? 0.f : c.x;
            c.y = c.y < 0.f ? 0.f : c.y;
            c.z = c.z < 0.f ? 0.f : c.z;
            const float2 pp = prev_pixel_out[lin];
            f3 tone;
            const f3 acc = accumulate_filtered(P, c, pp.x, pp.y,
                                               (uint8_t)((accept_bits[j >> 3] >> (4 * (j & 7))) & 15u),
                                               (uint8_t)(spp_bytes[j >> 2] >> (8 * (j & 3))),
                                               ld3(albedo, lin), acc_prev, frame, &tone);
            st3(acc_out, lin, acc);
            st3(tone_out, lin, tone);
        }
    }
}

bool fused_wave_supported(const Params& P) {
    if (P.fused_variant == 1 || !P.half_tmp || P.not_scaled != 4 || (P.scaled != 6 && P.scaled != 9)) return false;
    for (int f = 0; f < P.buffers - 3; ++f)
        if (P.codes[f] != f) return false;
    return true;
}

hipError_t launch_fused_wave(const Params& P, hipStream_t st, const FusedArgs& A) {
    const int G = P.blocks_x * P.blocks_y;
    if (P.scaled == 6)
        hipLaunchKernelGGL((k_fused_wave<4, 6>), dim3(G), dim3(64), 0, st, P, A.in, A.cam, A.frame, A.albedo,
                           A.acc_prev, A.noisy_out, A.spp_out, A.prev_pixel_out, A.acc_out, A.tone_out, A.noise_table);
    else
        hipLaunchKernelGGL((k_fused_wave<4, 9>), dim3(G), dim3(64), 0, st, P, A.in, A.cam, A.frame, A.albedo,
                           A.acc_prev, A.noisy_out, A.spp_out, A.prev_pixel_out, A.acc_out, A.tone_out, A.noise_table);
    return hipGetLastError();
}

}  // namespace bmfr
