// bmfr_fused.hip -- fused frame kernel K1 for f32 tmp_data
// (USE_HALF_PRECISION_IN_TMP_DATA 0; half tmp_data runs the column-split K1
// of bmfr_fused_cols.hip), one 256-thread work-group per 32x32 block:
// accumulate_noisy_data -> min/max scaling -> Householder QR -> back
// substitution -> weighted_sum -> temporal blend of the filtered colour
// (bmfr.cl:287-849).  Tone mapping and TAA follow in K2 (bmfr_kernels.hip).
//
// Work decomposition: thread t owns rows t + 256*s (s = 0..3) of the
// block's design matrix -- exactly the rows upstream's fitter work-item t
// touches (bmfr.cl:516-563) -- so per-thread partial sums and the
// 256 -> 64 -> 8 -> 1 reduction tree (bmfr.cl:25-87) are reproduced in
// upstream's association.  The matrix stays in VGPRs (f32), so tmp_data
// never touches HBM.  Every arithmetic step is upstream's, rounded
// the same way; parity: tests/test_gpu_parity.py (bit-exact vs the stage
// kernels and the reference kernels).
//
// Specialised for the canonical feature lists (FEATURE_BUFFERS entry f is
// monomial f: the reference defaults and the 3rd-order set); other lists run
// through the stage kernels.
#include <utility>

#include "bmfr_launch.h"
#include "bmfr_taa_tile.h"
#include "bmfr_wave.h"

namespace bmfr {

constexpr int kThreads = 256;
constexpr int kS64Stride = 72;  // 64 + 8: conflict-free transposed reads

// The f32 design matrix, rows t + 256 s of every column.
template <int B, int N>
struct FloatRows {
    float v[B][N];
    __device__ __forceinline__ float get(int f, int j) const { return v[f][j]; }
    __device__ __forceinline__ void set(int f, int j, float x) { v[f][j] = x; }
    __device__ __forceinline__ void fence(int f) {
#pragma unroll
        for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[f][i]));
    }
};

// LDS of one block.
template <int B>
struct K1Lds {
    // Largest batch: the B-1 trailing dots of column 0 or the 2*FS min/max.
    static constexpr int KMAX = (B - 1) > 2 * (B - 7) ? (B - 1) : 2 * (B - 7);
    float part[KMAX * kThreads];         // per-thread partials, [k][t]
    float s64[KMAX * kS64Stride];        // step-2 results, [k][x]
    float e8[KMAX * 8];                  // step-3 results, [k][i]
    float res[KMAX];                     // reduction results
    float bc;                            // broadcast slot
    float R[(B - 2) * (B - 2) * 3];      // R[x][y][ch], x = column
    float weights[(B - 3) * 3];
    float mm[3 * (B - 3)];               // per scaled feature: min, max, 1/(max-min)
    int flag;                            // one-launch frame: index of this block's completion flag
    int delay;                           // Params::debug_delay (diagnostics)
    // Phase 1 -> 3: each row's previous accumulated filtered colour, blended
    // at the noisy accumulation's taps (bmfr.cl:786-842), [(s * 3 + ch) * kThreads + t]
    float keep[kSubs * 3 * kThreads];
};

// ---------------------------------------------------------------------------
// Batched block reductions, upstream association (bmfr.cl:25-87).  v[k] holds
// thread t's partial of reduction k; on return every thread has the results.
// MODE 0: sums.  MODE 1: max for k < SPLIT, min for k >= SPLIT.
// K <= 4: one wave per reduction, steps 3-4 on DPP/permlane (2 barriers).
// K > 4: steps 2, 3, 4 spread over the block through LDS (4 barriers).
// ---------------------------------------------------------------------------
template <int MODE, int SPLIT>
__device__ __forceinline__ float rop(int k, float a, float b) {
    if constexpr (MODE == 0) return a + b;
    else return k < SPLIT ? fmaxf(a, b) : fminf(a, b);
}

template <int K, int MODE = 0, int SPLIT = 0, int B>
__device__ __forceinline__ void block_reduce(float (&v)[K], K1Lds<B>& L, int t) {
    static_assert(K <= K1Lds<B>::KMAX, "reduction batch exceeds the LDS scratch");
#pragma unroll
    for (int k = 0; k < K; ++k) L.part[k * kThreads + t] = v[k];
    __syncthreads();
    const int w = t >> 6, l = t & 63;
    if constexpr (K <= 4) {
        if (w < K) {  // wave-uniform
            const float* p = L.part + w * kThreads;
            float s;
            if constexpr (MODE == 0) {
                s = p[l] + ((p[l + 64] + p[l + 128]) + p[l + 192]);
                s = wave_tree<RedOp::Sum>(s);
            } else if (w < SPLIT) {
                s = wave_tree<RedOp::Max>(fmaxf(fmaxf(fmaxf(p[l], p[l + 64]), p[l + 128]), p[l + 192]));
            } else {
                s = wave_tree<RedOp::Min>(fminf(fminf(fminf(p[l], p[l + 64]), p[l + 128]), p[l + 192]));
            }
            if (l == 0) L.res[w] = s;
        }
        __syncthreads();
    } else {
#pragma unroll
        for (int base = 0; base < K * 64; base += kThreads) {  // 256 -> 64
            const int idx = base + t;
            if (idx < K * 64) {
                const int k = idx >> 6, x = idx & 63;
                const float* p = L.part + k * kThreads + x;
                float s;
                if constexpr (MODE == 0) s = p[0] + ((p[64] + p[128]) + p[192]);
                else s = rop<MODE, SPLIT>(k, rop<MODE, SPLIT>(k, rop<MODE, SPLIT>(k, p[0], p[64]), p[128]), p[192]);
                L.s64[k * kS64Stride + x] = s;
            }
        }
        __syncthreads();
        if (t < K * 8) {  // 64 -> 8
            const int k = t >> 3, i = t & 7;
            const float* row = L.s64 + k * kS64Stride + i;
            float e;
            if constexpr (MODE == 0) {
                float acc = row[8];
#pragma unroll
                for (int j = 2; j < 8; ++j) acc = acc + row[8 * j];
                e = row[0] + acc;
            } else {
                e = row[0];
#pragma unroll
                for (int j = 1; j < 8; ++j) e = rop<MODE, SPLIT>(k, e, row[8 * j]);
            }
            L.e8[t] = e;
        }
        __syncthreads();
        if (t < K) {  // 8 -> 1, left to right
            float r = L.e8[t * 8];
#pragma unroll
            for (int i = 1; i < 8; ++i) r = rop<MODE, SPLIT>(t, r, L.e8[t * 8 + i]);
            L.res[t] = r;
        }
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = L.res[k];
}

// ---------------------------------------------------------------------------
// One Householder column (bmfr.cl:549-655), compile-time column index.
// ---------------------------------------------------------------------------
// FAST: bmfr_config.fast_fit -- the trailing update of steps >= 1 as one
// fused multiply-add on the block-wide factor RN(2 dot / |u|^2) (as
// update_column in bmfr_fused_cols.hip; not bit-exact).
template <int col, int B, bool FAST, class M>
__device__ __forceinline__ void qr_column(M& A, K1Lds<B>& L, int t, const float* __restrict__ noise,
                                          double noise2) {
    constexpr int RE = B - 2;
    constexpr int cl = col;  // col_limited (feature columns only)
    if constexpr (col == 0) {
        // FEATURE_BUFFERS[0] is "1.f": the column is all ones, so the norm step
        // is exact integer arithmetic -- sum over rows >= 1 is 1023, |x| = 32,
        // u = (1 - 32, 1, 1, ...), |u|^2 = 1023 + 961 = 1984 -- and RN(v*u) = v
        // off row 0.  Identical values to running the generic step.
        const float ulen2 = 1984.f;
        const float recip = 1.f / ulen2;
        if (t < 3) L.R[t] = 32.f;  // R(0,0), all channels
        const bool row0 = t == 0;
        // Trailing columns in groups of four: noisy f32 values (noise once, on
        // first load, bmfr.cl:625-627) stay in registers for dot and update.
        constexpr int G = 4;
#pragma unroll
        for (int g0 = 1; g0 < B; g0 += G) {
            constexpr int dummy = 0;
            (void)dummy;
            float vals[G][kSubs];
            float dot[G];
#pragma unroll
            for (int k = 0; k < G; ++k) {
                const int fb = g0 + k;
                dot[k] = 0.f;
                if (fb < B) {
#pragma unroll
                    for (int s = 0; s < kSubs; ++s) {
                        float v = A.get(fb, s);
                        if (fb < B - 3)
                            v = (float)((double)v + noise2 * (double)noise[(fb - 1) * kBlockPixels + t + kLocal * s]);
                        vals[k][s] = v;
                    }
                    float sum = row0 ? vals[k][0] * -31.f : vals[k][0];
#pragma unroll
                    for (int s = 1; s < kSubs; ++s) sum = sum + vals[k][s];
                    dot[k] = sum;
                }
            }
            block_reduce<G>(dot, L, t);
#pragma unroll
            for (int k = 0; k < G; ++k) {
                const int fb = g0 + k;
                if (fb < B) {
                    const float c2 = 2.f * dot[k];
                    const float q = div_by_recip(c2, ulen2, recip);
                    A.set(fb, 0, vals[k][0] - (row0 ? div_by_recip(-31.f * c2, ulen2, recip) : q));
#pragma unroll
                    for (int s = 1; s < kSubs; ++s) A.set(fb, s, vals[k][s] - q);
                }
            }
            __builtin_amdgcn_sched_barrier(0);  // one group's noise loads in flight at a time
        }
    } else {
        // |x|^2 over rows >= cl+1 (bmfr.cl:555-569)
        float sq[1] = {0.f};
#pragma unroll
        for (int s = 0; s < kSubs; ++s) {
            const float v = A.get(col, s);
            if (s > 0 || t >= cl + 1) sq[0] = sq[0] + v * v;
        }
        if (t == cl) L.bc = A.get(col, 0);  // u_vec[col_limited]: row cl is thread cl, s = 0
        block_reduce<1>(sq, L, t);
        const float sumsq = sq[0];
        const float ucl = L.bc;
        const float vlen = sqrtf(sumsq + ucl * ucl);  // bmfr.cl:582-585
        const float ucl2 = ucl - vlen;
        const float ulen2 = sumsq + ucl2 * ucl2;
        // ulen2 > 0 unless the column is zero on and below the diagonal, which
        // is 0/0 upstream as well (then NaN here too).
        const float recip = 1.f / ulen2;
        if (t < col) {  // R column (bmfr.cl:574-601): rows above the diagonal ...
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) L.R[(col * RE + t) * 3 + ch] = A.get(col, 0);
        }
        if (t == col) {  // ... and the diagonal
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) L.R[(col * RE + col) * 3 + ch] = vlen;
        }
        float u[kSubs];
#pragma unroll
        for (int s = 0; s < kSubs; ++s) u[s] = A.get(col, s);
        if (t == cl) u[0] = ucl2;

        // All trailing dots (one batched reduction), then all updates; each
        // column's update depends only on its own dot.
        constexpr int K = B - 1 - cl;
        float dot[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int fb = cl + 1 + k;
            float sum = 0.f;
#pragma unroll
            for (int s = 0; s < kSubs; ++s)
                if (s > 0 || t >= cl) sum = sum + A.get(fb, s) * u[s];
            dot[k] = sum;
        }
#pragma unroll
        for (int fb = cl + 1; fb < B; ++fb) A.fence(fb);
        block_reduce<K>(dot, L, t);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int fb = cl + 1 + k;
            const float c2 = 2.f * dot[k];  // 2*u*dot == u*(2*dot): both exact doublings
            if constexpr (FAST) {
                const float sc = c2 * recip;
#pragma unroll
                for (int s = 0; s < kSubs; ++s)
                    if (s > 0 || t >= cl) A.set(fb, s, __builtin_fmaf(-u[s], sc, A.get(fb, s)));
            } else {
#pragma unroll
                for (int s = 0; s < kSubs; ++s)
                    if (s > 0 || t >= cl) A.set(fb, s, A.get(fb, s) - div_by_recip(u[s] * c2, ulen2, recip));
            }
        }
    }
}

template <int B, bool FAST, class M, int... C>
__device__ __forceinline__ void qr_columns(M& A, K1Lds<B>& L, int t, const float* __restrict__ noise,
                                           double noise2, std::integer_sequence<int, C...>) {
    (qr_column<C, B, FAST>(A, L, t, noise, noise2), ...);
}

// Back substitution (bmfr.cl:658-699) on R in LDS, parallel over elements
// like upstream: lanes (ch, x) of wave 0.  Every element sees upstream's
// operations in upstream's order.
template <int B>
__device__ __forceinline__ void back_substitute(K1Lds<B>& L, int t) {
    constexpr int RE = B - 2;
    if (t >= 64) return;
    const int ch = t % 3, x = t / 3;  // 3 * RE <= 48 lanes
    float* R = L.R;
    for (int i = RE - 2; i >= 0; --i) {
        const float div = R[(i * RE + i) * 3 + ch];
        __builtin_amdgcn_wave_barrier();
        if (x < RE && x >= i) R[(x * RE + i) * 3 + ch] = R[(x * RE + i) * 3 + ch] / div;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (x == 0) {  // one lane per channel: sequential sum (bmfr.cl:675-680)
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
    if (x < B - 3) L.weights[x * 3 + ch] = R[((RE - 1) * RE + x) * 3 + ch];
}

// One K1 work-group (block g of the launch) on the LDS area L.  COH: the TAA
// tiles of the same frame run in this launch (k_fused_rows_taa): the
// accumulated colour and reprojected positions they read are stored
// device-coherent and the block publishes done[...] = epoch once they are
// (the hand-off of bmfr_taa_tile.h wait_k1_blocks).
template <int NS, int FS, class IN, bool COH = false, bool FAST = false>
__device__ __forceinline__ void k1_rows_body(const Params& P, const K1Args& A, K1Lds<NS + FS + 3>& L, int g) {
    constexpr int B = NS + FS + 3;
    const int t = threadIdx.x;
    const int frame = A.frame;
    const NoisyInputs& in = A.in;
    // Diagnostic build only (-DBMFR_STAMPS): per-block phase timestamps.
#ifdef BMFR_STAMPS
#define BMFR_STAMP(k) \
    if (t == 0 && A.stamps) A.stamps[(size_t)g * 8 + (k)] = __builtin_amdgcn_s_memtime()
#else
#define BMFR_STAMP(k) (void)0
#endif
    BMFR_STAMP(0);
    int bx, by;
    k1_block(P, g, bx, by);
    if constexpr (COH) {
        if (t == 0) {
            L.flag = (by - P.by0) * P.nbx + (bx - P.bx0);  // this block's completion flag
            L.delay = P.debug_delay;
        }
    }

    // ---- accumulate_noisy_data (bmfr.cl:310-484) for rows t + 256s ----
    FloatRows<B, kSubs> M;
    int over = 0;
    uint32_t state = 0;  // per s: owner (bit 0), accept bits (1-4), spp (8-15) -> 16 bits each ...
    uint32_t state_hi = 0;
    NoisyCur<IN> cur[kSubs];  // current-frame loads of all four rows go out first
#pragma unroll
    for (int s = 0; s < kSubs; ++s)
        cur[s] = noisy_load_current<IN>(P, in, bx * kEdge + (t & (kEdge - 1)), by * kEdge + (t >> 5) + 8 * s, frame);
#pragma unroll
    for (int s = 0; s < kSubs; ++s) {
        // with accumulate_filtered_data's taps (FILT): the same taps and
        // weights, so phase 3 needs no second gather
        const NoisyItem it = noisy_item_spec<true, IN>(P, in, A.cam, cur[s], frame, A.acc_prev);
        L.keep[(s * 3 + 0) * kThreads + t] = it.prev_f.x;
        L.keep[(s * 3 + 1) * kThreads + t] = it.prev_f.y;
        L.keep[(s * 3 + 2) * kThreads + t] = it.prev_f.z;
        over = max(over, it.over);
#pragma unroll
        for (int f = 0; f < B; ++f) {
            float v;
            if (f < B - 3) v = feature_value(f, it.n, it.p);
            else v = f == B - 3 ? it.color.x : (f == B - 2 ? it.color.y : it.color.z);
            if (__builtin_isnan(v)) v = 0.0f;           // bmfr.cl:468-469
            M.set(f, s, v);
        }
        const uint32_t bits = (uint32_t)it.owner | ((uint32_t)it.accept << 1) | ((uint32_t)it.prev_f_divided << 5) |
                              ((uint32_t)it.spp << 8);
        if (s < 2) state |= bits << (16 * s);
        else state_hi |= bits << (16 * (s - 2));
        // owners only (bmfr.cl:478-484), as branch-free stores (st3_drop)
        st3_drop(drop_plane(A.noisy_out), it.lin, it.owner, it.color);
        st1_drop(drop_plane(A.spp_out), it.lin, it.owner, it.spp);
        st2_drop<COH ? kSc1 : 0>(drop_plane(A.prev_pixel_out), it.lin, it.owner, make_float2(it.pfx, it.pfy));
    }
    report_reach(P, A.reach, over);

    BMFR_STAMP(1);
    // ---- scale the position features to the block's [min, max] (bmfr.cl:510-542) ----
    if constexpr (FS > 0) {
        float mm[2 * FS];
#pragma unroll
        for (int f = 0; f < FS; ++f) {
            float hi = -INFINITY, lo = INFINITY;
#pragma unroll
            for (int s = 0; s < kSubs; ++s) {
                hi = fmaxf(M.get(NS + f, s), hi);
                lo = fminf(M.get(NS + f, s), lo);
            }
            mm[f] = hi;
            mm[FS + f] = lo;
        }
        block_reduce<2 * FS, 1, FS>(mm, L, t);
#pragma unroll
        for (int f = 0; f < FS; ++f) {
            const float bmax = mm[f], bmin = mm[FS + f];
            const float d = bmax - bmin;
            const bool divide = fabsf(d) > 1.0f;  // scale(), bmfr.cl:200-205
            const float rcp = 1.f / d;
            if (t == 0) {
                L.mm[3 * f] = bmin;
                L.mm[3 * f + 1] = bmax;
                L.mm[3 * f + 2] = rcp;
            }
#pragma unroll
            for (int s = 0; s < kSubs; ++s) {
                const float v = M.get(NS + f, s) - bmin;
                M.set(NS + f, s, divide ? div_by_recip(v, d, rcp) : v);
            }
        }
    }

    BMFR_STAMP(2);
    // ---- Householder QR over the feature columns (bmfr.cl:544-656) ----
    qr_columns<B, FAST>(M, L, t, A.noise, P.noise2, std::make_integer_sequence<int, B - 3>{});
    // Right-hand side: rows 0..B-4 of the colour columns, which the colour
    // columns' own Householder steps never touch (bmfr.cl:550, 596-600, 606).
    if (t < B - 3) {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) L.R[((B - 3) * (B - 2) + t) * 3 + ch] = M.get(B - 3 + ch, 0);
    }
    __syncthreads();
    BMFR_STAMP(3);
    back_substitute<B>(L, t);
    __syncthreads();
    BMFR_STAMP(4);

    // ---- weighted_sum (bmfr.cl:717-750) + temporal blend (bmfr.cl:778-849) ----
    int t3 = t;  // opaque copy: recompute phase-1 addresses instead of keeping them live
    asm volatile("" : "+v"(t3));
    const int2 off = kBlockOffsets[frame & 15];
    // The normal and position loads of the four rows first.
    f3 n[kSubs], pos[kSubs];
    uint32_t lin[kSubs];
    uint32_t bits[kSubs];
#pragma unroll
    for (int s = 0; s < kSubs; ++s) {
        bits[s] = (s < 2 ? state >> (16 * s) : state_hi >> (16 * (s - 2))) & 0xffffu;
        const int px = bx * kEdge + (t3 & (kEdge - 1)) - kEdge / 2 + off.x;
        const int py = by * kEdge + (t3 >> 5) + 8 * s - kEdge / 2 + off.y;
        // non-owned rows (margins) read a valid pixel and are then skipped
        lin[s] = pix(P, (bits[s] & 1u) ? px : P.ox, (bits[s] & 1u) ? py : P.oy);
        n[s] = ld3in<IN>(in.n_cur, lin[s]);
        pos[s] = ld3in<IN>(in.p_cur, lin[s]);
    }
#pragma unroll
    for (int s = 0; s < kSubs; ++s) {
        if (bits[s] & 1u) {
            f3 c{0.f, 0.f, 0.f};
#pragma unroll
            for (int f = 0; f < B - 3; ++f) {
                float v = feature_value(f, n[s], pos[s]);
                if (f >= NS) {
                    const float bmin = L.mm[3 * (f - NS)], bmax = L.mm[3 * (f - NS) + 1];
                    const float d = bmax - bmin;
                    v = v - bmin;
                    if (fabsf(d) > 1.0f) v = div_by_recip(v, d, L.mm[3 * (f - NS) + 2]);
                }
                c.x = c.x + L.weights[3 * f] * v;
                c.y = c.y + L.weights[3 * f + 1] * v;
                c.z = c.z + L.weights[3 * f + 2] * v;
            }
            c.x = c.x < 0.f ? 0.f : c.x;
            c.y = c.y < 0.f ? 0.f : c.y;
            c.z = c.z < 0.f ? 0.f : c.z;
            // bmfr.cl:834-849 (blend_filtered's arithmetic, the sums from phase 1):
            // alpha from the current spp when the taps carried weight
            // 1 / spp, spp in [1, 255] (rcp_nr: exactly 1.f / spp)
            const float alpha = (bits[s] & 32u) ? fmaxf(rcp_nr((float)(bits[s] >> 8)), P.second_blend_alpha) : 1.f;
            const float beta = 1.f - alpha;
            const f3 prev{L.keep[(s * 3) * kThreads + t3], L.keep[(s * 3 + 1) * kThreads + t3],
                          L.keep[(s * 3 + 2) * kThreads + t3]};
            const f3 acc{alpha * c.x + beta * prev.x, alpha * c.y + beta * prev.y, alpha * c.z + beta * prev.z};
            if constexpr (COH) st3_coh(coh_plane(A.acc_out), lin[s], acc);
            else st3(A.acc_out, lin[s], acc);
        }
    }
#ifdef BMFR_STAMPS
    __syncthreads();
#endif
    BMFR_STAMP(5);
#undef BMFR_STAMP
    if constexpr (COH) {  // as k1_cols_body: stores performed, then the flag
        const int delay = L.delay;
        if (delay > 0 && g % kDelayStride == kDelayPhase)  // diagnostics: tiles really wait
            for (int k = 0; k < delay; ++k) __builtin_amdgcn_s_sleep(127);
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
        __syncthreads();
        if (t == 0) __hip_atomic_store(&A.done[L.flag], A.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Minimum waves per SIMD for the register allocator at B = 13: four (128
// VGPRs, 12-32 bytes of spills) instead of three (129-130 VGPRs).
#ifndef BMFR_ROWS_MIN_WAVES
#define BMFR_ROWS_MIN_WAVES 4
#endif
constexpr int kRowsMinWaves = BMFR_ROWS_MIN_WAVES;
template <int NS, int FS, class IN, bool FAST = false>
__global__ __launch_bounds__(kThreads, FS == 6 ? kRowsMinWaves : 3) void k_fused(Params P, K1Args A) {
    __shared__ K1Lds<NS + FS + 3> L;
    k1_rows_body<NS, FS, IN, false, FAST>(P, A, L, xcd_swizzle(blockIdx.x, gridDim.x));
}

// The one-launch frame with this K1 (f32 tmp_data): K1 blocks, then the
// frame's TAA tiles waiting on their completion flags (as k_fused_cols_taa,
// bmfr_fused_cols.hip).
template <int NS, int FS, class IN, bool FAST = false>
__global__ __launch_bounds__(kThreads, FS == 6 ? kRowsMinWaves : 3) void k_fused_rows_taa(Params P, K1Args A, TaaArgs T, int nk1, int nk1p) {
    __shared__ union {
        K1Lds<NS + FS + 3> k1;
        FrameTaaLds<kThreads> k2;
    } U;
    const int b = blockIdx.x;
    if (b < nk1) k1_rows_body<NS, FS, IN, true, FAST>(P, A, U.k1, xcd_swizzle(b, nk1));
    else if (b >= nk1p) frame_taa_part<IN, true, kThreads>(P, T, b, nk1p, U.k2);
}

bool fused_supported(const Params& P) {
    if (P.not_scaled != 4 || (P.scaled != 6 && P.scaled != 9)) return false;
    for (int f = 0; f < P.buffers - 3; ++f)
        if (P.codes[f] != f) return false;
    return true;
}

// The row-split kernels' template arguments from the run-time parameters
// (FS, the input element type, fast_fit), as dispatch_cols in bmfr_fused_cols.hip.
template <template <int, class, bool> class L, class... Args>
static void dispatch_rows(const Params& Q, Args&&... args) {
    if (Q.scaled == 6) {
        if (Q.input_half) Q.fast_fit ? L<6, _Float16, true>::go(args...) : L<6, _Float16, false>::go(args...);
        else Q.fast_fit ? L<6, float, true>::go(args...) : L<6, float, false>::go(args...);
    } else {
        if (Q.input_half) Q.fast_fit ? L<9, _Float16, true>::go(args...) : L<9, _Float16, false>::go(args...);
        else Q.fast_fit ? L<9, float, true>::go(args...) : L<9, float, false>::go(args...);
    }
}

template <int FS, class IN, bool FAST>
struct LaunchK1 {
    static void go(const Params& P, hipStream_t st, const FusedArgs& A) {
        hipLaunchKernelGGL((k_fused<4, FS, IN, FAST>), dim3(k1_blocks(P)), dim3(kThreads), 0, st, P, k1_args(A));
    }
};

template <int FS, class IN, bool FAST>
struct LaunchRowsFrame {
    static void go(const Params& P, hipStream_t st, const FusedArgs& A) {
        const int nk1 = P.ring < 0 || P.nbx <= 0 || P.nby <= 0 ? 0 : k1_blocks(P), nk1p = (nk1 + 7) & ~7;
        hipLaunchKernelGGL((k_fused_rows_taa<4, FS, IN, FAST>), dim3(nk1p + frame_taa_tiles<kThreads>(P)),
                           dim3(kThreads), 0, st, P, k1_args(A), taa_args(A), nk1, nk1p);
    }
};

hipError_t launch_fused_rows_frame_one(const Params& P, hipStream_t st, const FusedArgs& A) {
    dispatch_rows<LaunchRowsFrame>(P, P, st, A);
    return hipGetLastError();
}

hipError_t launch_fused_k1(const Params& P, hipStream_t st, const FusedArgs& A) {
    dispatch_rows<LaunchK1>(P, P, st, A);
    return hipGetLastError();
}

}  // namespace bmfr
