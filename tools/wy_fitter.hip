// wy_fitter.hip -- EXPERIMENT (tools-only build, not in libbmfr): the BMFR
// fitter stage (bmfr.cl:490-700) with a blocked compact-WY Householder QR
// whose trailing-panel update runs on MFMA (v_mfma_f32_16x16x4_f32), in
// f32-tmp_data mode, for the canonical feature lists B = 13 (FS = 6) and
// B = 16 (FS = 9, BASELINE config 5's 3rd-order set), panels of NB pivot
// columns (4, 8, or all of them: one full-width panel).
//
// Same inputs / outputs as the stage fitter (bmfr_fitter: tmp_data
// [block][B][1024] f32 -> weights [block][B-3][3], mins_maxs [block][FS][2]).
// Scaling and noise are the reference's (exact); the QR reassociates:
//   per panel of nb <= NB pivot columns: unblocked Householder steps on the
//   panel columns (VALU), T of Q = H_0 ... H_{nb-1} = I - V T V^T, then the
//   trailing columns X_t <- X_t - V (T^T (V^T X_t)) with V^T X_t (K = 1024
//   rows) and the rank-nb update V W2 as 16x16x4 f32 MFMAs (ceil(nb / 4)
//   k-steps of 4).
// Back substitution as the reference (bmfr.cl:658-699).  Tolerance-checked
// against the reference (tools/mfma_experiment.py), never bit-exact.
#include <hip/hip_runtime.h>

#include "../bmfr_amd/csrc/bmfr_device.h"

namespace {

constexpr int NS = 4;
constexpr int kRows = 1024, kThreads = 256;

typedef float f4 __attribute__((ext_vector_type(4)));

template <int B, int FS>
struct Lds {
    static constexpr int NF = B - 3, RE = B - 2;
    static constexpr int kX = B | 1;  // LDS row stride of the block matrix (odd: conflict-free row-per-lane access)
    float X[kRows * kX];       // block matrix, row-major
    float red[4][16];          // cross-wave reduction scratch
    float Wp[4][16][16];       // per-wave partial V^T X
    float W2[16][16];          // T^T V^T X
    float T[16][16];
    float gram[16][16];
    float ucl2[NF], ulen2[NF];
    float R[RE * RE * 3];      // R[x][y][ch], x = column
    float weights[NF * 3];
    float mm[2 * FS];
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Block-wide sum of one value per thread (any association: tolerance mode).
template <class L_>
__device__ __forceinline__ float block_sum(float v, L_& L, int t) {
    v = wave_sum(v);
    __syncthreads();
    if ((t & 63) == 0) L.red[t >> 6][0] = v;
    __syncthreads();
    return L.red[0][0] + L.red[1][0] + L.red[2][0] + L.red[3][0];
}

// V[r][c] of the reflector of pivot column c: zero above the pivot, u_c below.
template <class L_>
__device__ __forceinline__ float vval(const L_& L, int r, int c) {
    return r < c ? 0.f : (r == c ? L.ucl2[c] : L.X[r * L_::kX + c]);
}

template <int B, int FS, int NB>
__global__ __launch_bounds__(kThreads) void k_fitter_wy(const float* __restrict__ tmp, float* __restrict__ weights,
                                                        float* __restrict__ mins_maxs, int frame, double noise2) {
    static_assert(B <= 16 && NB <= 16, "16x16 MFMA tiles");
    using L_ = Lds<B, FS>;
    constexpr int NF = L_::NF, RE = L_::RE, kX = L_::kX;
    __shared__ L_ L;
    const int t = threadIdx.x, w = t >> 6, l = t & 63, g = blockIdx.x;
    const float* src = tmp + (size_t)g * B * kRows;
    // ---- load, min/max scaling (bmfr.cl:510-542), noise (bmfr.cl:625-627) ----
    for (int i = t; i < B * kRows; i += kThreads) {
        const int f = i / kRows, r = i % kRows;
        L.X[r * kX + f] = src[i];
    }
    __syncthreads();
    for (int f = NS; f < NF; ++f) {
        float hi = -INFINITY, lo = INFINITY;
        for (int s = 0; s < 4; ++s) {
            const float v = L.X[(t + 256 * s) * kX + f];
            hi = fmaxf(hi, v);
            lo = fminf(lo, v);
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            hi = fmaxf(hi, __shfl_xor(hi, o, 64));
            lo = fminf(lo, __shfl_xor(lo, o, 64));
        }
        __syncthreads();
        if (l == 0) {
            L.red[w][0] = hi;
            L.red[w][1] = lo;
        }
        __syncthreads();
        const float bmax = fmaxf(fmaxf(L.red[0][0], L.red[1][0]), fmaxf(L.red[2][0], L.red[3][0]));
        const float bmin = fminf(fminf(L.red[0][1], L.red[1][1]), fminf(L.red[2][1], L.red[3][1]));
        if (t == 0) {
            L.mm[2 * (f - NS)] = bmin;
            L.mm[2 * (f - NS) + 1] = bmax;
        }
        for (int s = 0; s < 4; ++s) {
            float& x = L.X[(t + 256 * s) * kX + f];
            x = bmfr::scale(x, bmin, bmax);
        }
    }
    __syncthreads();
    for (int s = 0; s < 4; ++s)
        for (int f = 1; f < NF; ++f) {
            float& x = L.X[(t + 256 * s) * kX + f];
            x = bmfr::add_random(x, noise2, t + s * 256 + f * kRows + frame * B * kRows);
        }
    __syncthreads();

    // ---- blocked Householder QR ----
    for (int j0 = 0; j0 < NF; j0 += NB) {
        const int nb = NF - j0 < NB ? NF - j0 : NB;
        // panel factorization, unblocked (VALU)
        for (int c = j0; c < j0 + nb; ++c) {
            float sq = 0.f;
            for (int s = 0; s < 4; ++s) {
                const int r = t + 256 * s;
                const float v = L.X[r * kX + c];
                if (r > c) sq += v * v;
            }
            const float sumsq = block_sum(sq, L, t);
            const float ucl = L.X[c * kX + c];
            const float vlen = sqrtf(sumsq + ucl * ucl);
            const float ucl2 = ucl - vlen;
            const float ulen2 = sumsq + ucl2 * ucl2;
            if (t == 0) {
                L.ucl2[c] = ucl2;
                L.ulen2[c] = ulen2;
            }
            if (t < c)
                for (int ch = 0; ch < 3; ++ch) L.R[(c * RE + t) * 3 + ch] = L.X[t * kX + c];
            if (t == c)
                for (int ch = 0; ch < 3; ++ch) L.R[(c * RE + c) * 3 + ch] = vlen;
            __syncthreads();
            for (int fb = c + 1; fb < j0 + nb; ++fb) {
                float d = 0.f;
                for (int s = 0; s < 4; ++s) {
                    const int r = t + 256 * s;
                    d += vval(L, r, c) * L.X[r * kX + fb];
                }
                const float q = 2.f * block_sum(d, L, t) / ulen2;
                for (int s = 0; s < 4; ++s) {
                    const int r = t + 256 * s;
                    if (r >= c) L.X[r * kX + fb] -= q * vval(L, r, c);
                }
                __syncthreads();
            }
        }
        // Gram V^T V and T (Q = I - V T V^T, T upper triangular, T_ii = 2 / |u_i|^2)
        for (int p = 0; p < nb * nb; ++p) {
            const int i = p / nb, k = p % nb;
            if (k < i) continue;
            float d = 0.f;
            for (int s = 0; s < 4; ++s) {
                const int r = t + 256 * s;
                d += vval(L, r, j0 + i) * vval(L, r, j0 + k);
            }
            const float gsum = block_sum(d, L, t);
            if (t == 0) L.gram[i][k] = L.gram[k][i] = gsum;
        }
        __syncthreads();
        if (t == 0) {
            for (int i = 0; i < 16; ++i)
                for (int k = 0; k < 16; ++k) L.T[i][k] = 0.f;
            for (int i = 0; i < nb; ++i) {
                const float tau = 2.f / L.ulen2[j0 + i];
                L.T[i][i] = tau;
                for (int a = 0; a < i; ++a) {  // T[0:i, i] = -tau T[0:i, 0:i] (V_{0:i}^T v_i)
                    float acc = 0.f;
                    for (int b = a; b < i; ++b) acc += L.T[a][b] * L.gram[b][i];
                    L.T[a][i] = -tau * acc;
                }
            }
        }
        __syncthreads();
        const int jt = j0 + nb;  // first trailing column
        // W = V^T X on MFMA: per wave its 256 rows as 64 k-steps of 4 rows.
        // A (16 x 4): lane l -> V[r][j0 + l % 16] (rows r = r0 + l / 16), zero past nb;
        // B (4 x 16): lane l -> X[r][l % 16], zero past B.
        f4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < 64; ++k) {
            const int r = 256 * w + 4 * k + (l >> 4), j = l & 15;
            const float a = j < nb ? vval(L, r, j0 + j) : 0.f;
            const float b = j < B ? L.X[r * kX + j] : 0.f;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
        }
        // D[i][j]: lane l holds rows i = 4 (l / 16) + e, column j = l % 16
        for (int e = 0; e < 4; ++e) L.Wp[w][4 * (l >> 4) + e][l & 15] = acc[e];
        __syncthreads();
        {  // W2 = -(T^T W) on the trailing columns, zero elsewhere
            const int i = t >> 4, j = t & 15;
            float v = 0.f;
            if (i < nb && j >= jt && j < B)
                for (int k = 0; k <= i; ++k)
                    v += L.T[k][i] * (L.Wp[0][k][j] + L.Wp[1][k][j] + L.Wp[2][k][j] + L.Wp[3][k][j]);
            L.W2[i][j] = -v;
        }
        __syncthreads();
        // X_t += V (-W2) on MFMA, 16-row tiles, ceil(nb / 4) k-steps: A (16 x 4): lane l ->
        // V[r0 + l % 16][j0 + 4 kk + l / 16]; B (4 x 16): lane l -> -W2[4 kk + l / 16][l % 16];
        // C / D: rows r0 + 4 (l / 16) + e, column l % 16.
        if (jt < B)
        for (int tile = w; tile < kRows / 16; tile += 4) {
            const int r0 = 16 * tile, j = l & 15, q = l >> 4;
            f4 d;
            for (int e = 0; e < 4; ++e) d[e] = j < B ? L.X[(r0 + 4 * q + e) * kX + j] : 0.f;
            for (int kk = 0; 4 * kk < nb; ++kk) {
                const int vc = 4 * kk + q;
                const float a = vc < nb ? vval(L, r0 + j, j0 + vc) : 0.f;
                const float b = L.W2[vc][j];
                d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, d, 0, 0, 0);
            }
            // (V reads the panel columns, the writes go to trailing columns of this wave's rows)
            if (j >= jt && j < B)
                for (int e = 0; e < 4; ++e) L.X[(r0 + 4 * q + e) * kX + j] = d[e];
        }
        __syncthreads();
    }
    // right-hand side: rows 0..B-4 of the colour columns (bmfr.cl:596-600)
    if (t < NF)
        for (int ch = 0; ch < 3; ++ch) L.R[((RE - 1) * RE + t) * 3 + ch] = L.X[t * kX + NF + ch];
    __syncthreads();
    // back substitution (bmfr.cl:658-699)
    if (t < 64) {
        const int ch = t % 3, x = t / 3;
        float* R = L.R;
        for (int i = RE - 2; i >= 0; --i) {
            const float div = R[(i * RE + i) * 3 + ch];
            __builtin_amdgcn_wave_barrier();
            if (x < RE && x >= i) R[(x * RE + i) * 3 + ch] = R[(x * RE + i) * 3 + ch] / div;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (x == 0) {
                float rhs = R[((RE - 1) * RE + i) * 3 + ch];
                for (int j = i + 1; j < RE - 1; ++j) rhs = rhs - R[(j * RE + i) * 3 + ch];
                R[((RE - 1) * RE + i) * 3 + ch] = rhs;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const float xi = R[((RE - 1) * RE + i) * 3 + ch];
            if (x <= i && x < RE) R[(i * RE + x) * 3 + ch] = R[(i * RE + x) * 3 + ch] * xi;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        if (x < NF) weights[(size_t)g * NF * 3 + x * 3 + ch] = R[((RE - 1) * RE + x) * 3 + ch];
    }
    if (t < 2 * FS) mins_maxs[(size_t)g * FS * 2 + t] = L.mm[t];
}

}  // namespace

// buffers = B (13 or 16), nb = panel width (4, 8 or 16: the whole QR in one panel).
extern "C" int wy_fitter(int blocks, const float* tmp, float* weights, float* mins_maxs, int frame, double noise2,
                         void* stream, int buffers, int nb) {
    const hipStream_t st = static_cast<hipStream_t>(stream);
#define WY(B_, FS_, NB_)                                                                                 \
    if (buffers == B_ && nb == NB_)                                                                      \
        hipLaunchKernelGGL((k_fitter_wy<B_, FS_, NB_>), dim3(blocks), dim3(kThreads), 0, st, tmp, weights, \
                           mins_maxs, frame, noise2);
    WY(13, 6, 4) WY(13, 6, 8) WY(13, 6, 16) WY(16, 9, 4) WY(16, 9, 8) WY(16, 9, 16)
#undef WY
    return (int)hipGetLastError();
}
