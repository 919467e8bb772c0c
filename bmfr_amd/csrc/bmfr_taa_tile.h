// K2's tile body (fused TAA, bmfr.cl:860-974, with the tone map of
// bmfr.cl:851-856): one 64 x TH output tile per 256-thread
// work-group.  The tile's tone-mapped colours and a 1-pixel halo go to LDS
// (Y) once as YCoCg, and the 3x3 neighbourhoods (bmfr.cl:897-920) are read
// from there; each thread keeps the RGB of its own TH / 4 output pixels in
// registers.  Shared by k_fused_taa (bmfr_kernels.hip) and the sequence
// kernel k_fused_cols_taa (bmfr_fused_cols.hip).
#pragma once

#include "bmfr_kernels.h"

namespace bmfr {

struct TaaArgs {
    const float* src;         // accumulated filtered colour (tone-mapped here)
    const float* albedo;      // float3 or half3 (IN)
    const float2* prev_pixel;
    float* result;
    const float* prev_frame;  // previous TAA output
    int frame;
    // Tiled contexts (else null): K1's reprojection-reach word, forwarded by
    // K2 (which runs after every K1 block of the frame) to page-locked host
    // memory -- reach_host[0] = max so far, reach_host[1] = frame + 1 -- and
    // cleared for the next frame.
    unsigned* reach_dev;
    unsigned* reach_host;
    // One-launch frame (COH tiles): K1 block g of this launch has stored its
    // accumulated colour and reprojected positions once done[g] >= epoch.
    const unsigned* done;
    unsigned epoch;
    // Page-locked host words (or null): [kSyncPivot] / [kSyncTile] become
    // nonzero when a K1 pivot wait / a tile's completion-flag wait gave up
    // (include/bmfr.h BMFR_ERROR_SYNC_TIMEOUT).
    unsigned* sync_err;
};

constexpr int kSyncPivot = 0, kSyncTile = 1;
// One-launch frame: done[g] = epoch (< 2^31) | kDoneTimeout when a pivot wait
// of block g gave up; the tiles that read the flag report it.
constexpr unsigned kDoneTimeout = 0x80000000u;
// An exhausted bounded wait: the kernel runs on (every wave must finish), so
// the context reports BMFR_ERROR_SYNC_TIMEOUT for this frame instead of
// handing out its pixels as good.  Cold path: a system-scope vector store to
// page-locked host memory (idempotent, any number of writers).
__device__ __forceinline__ void report_sync_timeout(unsigned* err, int which, int frame) {
    if (err) {
        __hip_atomic_store(err + which, (unsigned)frame + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
    }
}

// A COH tile first waits until every K1 block owning a pixel of the tile or
// its 1-px halo (the blocks of the frame's shifted grid, bmfr.cl:267-285)
// has published: at most 4 x 2 blocks, one lane each.  The polls are bounded
// (4 * P.max_polls sleeps of 128 cycles): a block that never publishes --
// a protocol error, or a block parked by the hardware far longer than any
// frame -- makes the tile report a sync timeout instead of hanging the GPU.
//
// Why the hand-off is safe without release / acquire fences (which on gfx942 /
// gfx950 would write back or invalidate the whole L2 of an XCD): every K1
// output a tile reads (accumulated colour, reprojected positions) is stored
// with SC1 (buffer stores with the sc1 policy: written through to memory,
// the form the AMDGPU memory model uses for agent-scope atomics) and loaded
// with SC1 (served coherently at device scope, never from another XCD's stale
// line); each location is written by exactly one block per launch.  The block
// waits for its own stores to be acknowledged (s_waitcnt vmcnt(0)), meets the
// work-group barrier (an asm with a memory clobber: no store moves across it)
// and only then stores its flag.  A tile that reads the flag >= epoch (agent
// scope, coherent) therefore finds every store of that block performed.  A
// cache line a tile loads may straddle a neighbouring block that has not
// finished; the tile never uses those bytes, and any later read of them in
// the launch is again an SC1 load that does not hit a stale copy.
// One completion flag (bounded poll, one lane).
__device__ __forceinline__ void wait_done(const Params& P, const TaaArgs& T, const unsigned* f) {
    const int limit = 4 * P.max_polls;
    for (int k = 0;; ++k) {
        const unsigned v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((v & ~kDoneTimeout) >= T.epoch) {
            if (v & kDoneTimeout) report_sync_timeout(T.sync_err, kSyncPivot, T.frame);
            return;
        }
        if (k >= limit) {
            report_sync_timeout(T.sync_err, kSyncTile, T.frame);
            return;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// K1 block (bx, by) of launch P runs in this launch (a tiled context's border
// launch holds only the ring outside [rx0, rx1) x [ry0, ry1), none when
// ring < 0; the interior blocks ran in the launch before, complete before
// this one starts).
__device__ __forceinline__ bool k1_in_launch(const Params& P, int bx, int by) {
    if (P.ring <= 0) return P.ring == 0;
    return bx < P.rx0 || bx >= P.rx1 || by < P.ry0 || by >= P.ry1;
}

__device__ __forceinline__ void wait_k1_blocks(const Params& P, const TaaArgs& T, int x0, int y0, int th) {
    const int2 off = kBlockOffsets[T.frame & 15];
    // the tile and its 1-px halo, inside the output rectangle + 1 px (a tiled
    // context's K1 blocks cover exactly that) and the buffer region
    const int xa = max(x0 - 1, P.ox), xb = min(min(x0 + 64, P.tx1), P.ox + P.stride - 1);
    const int ya = max(y0 - 1, P.oy), yb = min(min(y0 + th, P.ty1), P.oy + P.rows - 1);
    const int bxa = (xa + kEdge / 2 - off.x) / kEdge, bxb = (xb + kEdge / 2 - off.x) / kEdge;
    const int bya = (ya + kEdge / 2 - off.y) / kEdge, byb = (yb + kEdge / 2 - off.y) / kEdge;
    const int nx = bxb - bxa + 1, n = nx * (byb - bya + 1);
    const int t = threadIdx.x;
    if (t < n) {
        const int bx = bxa + t % nx, by = bya + t / nx;
        if (k1_in_launch(P, bx, by)) wait_done(P, T, T.done + (by - P.by0) * P.nbx + (bx - P.bx0));
    }
    __syncthreads();
}

// Every K1 block of this launch has published (the reach report is complete).
__device__ __forceinline__ void wait_all_k1_blocks(const Params& P, const TaaArgs& T) {
    for (int i = threadIdx.x; i < P.nbx * P.nby; i += blockDim.x) {
        const int bx = P.bx0 + i % P.nbx, by = P.by0 + i / P.nbx;
        if (k1_in_launch(P, bx, by)) wait_done(P, T, T.done + i);
    }
    __syncthreads();
}

__device__ __forceinline__ void forward_reach(const TaaArgs& T, bool here = true) {
    if (T.reach_dev && here && threadIdx.x == 0) {
        const unsigned v = atomicExch(T.reach_dev, 0u);
        volatile unsigned* h = T.reach_host;
        if (v > h[0]) h[0] = v;
        __threadfence_system();
        h[1] = (unsigned)T.frame + 1u;
        __threadfence_system();
    }
}

#ifndef BMFR_K2_STRIP
#define BMFR_K2_STRIP 1
#endif
constexpr bool kStrip = BMFR_K2_STRIP;

// A tile's geometry: 64 x TH output pixels, NT threads (NT / 64 rows of 64
// per pass, KN output pixels per thread), the tile and a 1-pixel ring in LDS.
template <int TH, int NT, bool ST = false>
struct TileShape {
    static constexpr int RP = NT / 64;  // tile rows per pass
    static_assert(TH % RP == 0 && TH >= RP, "tile height");
    static constexpr int HW = 64 + 2, HH = TH + 2, N = HW * HH;
    static constexpr int RING = N - 64 * TH;  // halo pixels
    static constexpr int KN = TH / RP;        // output pixels per thread
    static_assert(RING <= NT, "one ring pixel per thread");
    // Tile row of thread row ty's k-th output pixel: a strip of KN
    // consecutive rows per thread (its KN 3x3 neighbourhoods overlap: one
    // (KN + 2) x 3 window of LDS reads serves all of them), or with
    // BMFR_K2_STRIP=0 rows ty, ty + RP, ... (a 3x3 read per pixel).  Either
    // way a wave's loads and LDS accesses cover 64 consecutive pixels of a row.
    static __device__ __forceinline__ int row(int ty, int k) { return ST ? ty * KN + k : ty + RP * k; }
};

// A thread's current-frame inputs of one tile, as loaded: the reprojected
// positions of its KN output pixels, and the colour and albedo of those and
// of its ring pixel (k = KN, threads t < RING).
template <class IN, int KN>
struct TileLoads {
    float2 pf[KN];
    f3 v[KN + 1];
    In3<IN> al[KN + 1];  // widened in the tone map
};

// This thread's ring pixel (t < RING), in tile + halo coordinates.
template <int TH, int NT>
__device__ __forceinline__ void ring_pixel(int t, int& hx, int& hy) {
    using S = TileShape<TH, NT>;
    if (t < 2 * S::HW) {
        hx = t % S::HW;
        hy = t < S::HW ? 0 : S::HH - 1;
    } else {
        hx = t < 2 * S::HW + TH ? 0 : S::HW - 1;
        hy = 1 + (t - 2 * S::HW) % TH;
    }
}

// Issue the tile's current-frame loads (reprojected positions first).  COH:
// device-coherent loads of K1's outputs of the same launch.
template <class IN, int TH, bool COH, int NT, bool ST>
__device__ __forceinline__ void tile_issue(const Params& P, const TaaArgs& T, int x0, int y0, int hx, int hy,
                                           TileLoads<IN, TileShape<TH, NT>::KN>& L) {
    using S = TileShape<TH, NT, ST>;
    const int t = threadIdx.x, tx = t & 63, ty = t >> 6;
    const CohPlane c_pp = coh_plane(T.prev_pixel), c_src = coh_plane(T.src);  // (unused unless COH)
#pragma unroll
    for (int k = 0; k < S::KN; ++k) {
        const uint32_t i = pix(P, min(x0 + tx, P.tx1 - 1), min(y0 + S::row(ty, k), P.ty1 - 1));
        if constexpr (COH) L.pf[k] = ld2_coh(c_pp, i);
        else L.pf[k] = ld_px(T.prev_pixel, i);
    }
#pragma unroll
    for (int k = 0; k <= S::KN; ++k) {
        const int lx = k < S::KN ? tx + 1 : hx, ly = k < S::KN ? S::row(ty, k) + 1 : hy;
        if (k == S::KN && t >= S::RING) break;
        // Clamped into the buffer region (= the image when untiled): a tile
        // whose last 64-px column or TH-row band overhangs its output reads
        // no pixel outside the region; such values reach no output pixel.
        const uint32_t lin = pix(P, clamp_rx(P, x0 - 1 + lx), clamp_ry(P, y0 - 1 + ly));
        if constexpr (COH) L.v[k] = ld3_coh(c_src, lin);
        else L.v[k] = ld3(T.src, lin);
        L.al[k] = ld3raw<IN>(T.albedo, lin);
    }
}

// Tone map (bmfr.cl:851-856) of the loaded colours into the LDS window Y as
// YCoCg; me[k]: this thread's own output pixels, tone-mapped RGB.
template <class IN, int TH, int NT, bool ST>
__device__ __forceinline__ void tile_tone(const Params& P, const TileLoads<IN, TileShape<TH, NT>::KN>& L, int hx,
                                          int hy, float4* __restrict__ Y, const double* __restrict__ sE,
                                          const double2* __restrict__ sRP, f3 (&me)[TileShape<TH, NT>::KN]) {
    using S = TileShape<TH, NT, ST>;
    const int t = threadIdx.x, tx = t & 63, ty = t >> 6;
    // The correctly rounded powr's table part for every channel of every
    // pixel, branch-free (gamma_table), so the compiler can issue a pixel's
    // six table lookups together and overlap pixels; the rare values next to
    // a float rounding midpoint (about one in 2^18) are redone afterwards
    // through the whole tone map (gamma_clamped's fallback).  library_powr
    // (uniform): the device library's powr, no fallback needed.
    uint32_t rare = 0;  // bit k: a channel of pixel k needs the fallback
    auto put = [&](int k, const f3& v) {
        const int lx = k < S::KN ? tx + 1 : hx, ly = k < S::KN ? S::row(ty, k) + 1 : hy;
        if (k < S::KN) me[k] = v;
        const f3 yc = rgb_to_ycocg(v);
        Y[ly * S::HW + lx] = make_float4(yc.x, yc.y, yc.z, 0.f);
    };
#ifdef BMFR_PROBE_K2_NOTONE  // timing probe (wrong results): no tone map
#pragma unroll
    for (int k = 0; k <= S::KN; ++k) {
        if (k == S::KN && t >= S::RING) break;
        const f3 a = widen(L.al[k]);
        put(k, f3{L.v[k].x * a.x, L.v[k].y * a.y, L.v[k].z * a.z});
    }
#else
    if (P.library_powr) {
#pragma unroll
        for (int k = 0; k <= S::KN; ++k) {
            if (k == S::KN && t >= S::RING) break;
            put(k, tone_map(P, widen(L.al[k]), L.v[k], sE, sRP));
        }
    } else {
#pragma unroll
        for (int k = 0; k <= S::KN; ++k) {
            if (k == S::KN && t >= S::RING) break;
            // tone_map's arithmetic (bmfr.cl:851-856), the powr by table
            const f3 a = widen(L.al[k]);
            const float p[3] = {a.x * L.v[k].x, a.y * L.v[k].y, a.z * L.v[k].z};
            float g[3];
            uint32_t r;
            gamma_table3(p, g, r, sE, sRP);
            rare |= (r != 0 ? 1u : 0u) << k;
            put(k, f3{g[0], g[1], g[2]});
        }
    }
#endif
    if (__builtin_expect(rare != 0, 0)) {
#pragma unroll
        for (int k = 0; k <= S::KN; ++k)
            if (rare & (1u << k)) put(k, tone_map(P, widen(L.al[k]), L.v[k], sE, sRP));
    }
}

// The previous TAA output's bilinear taps at each output pixel's reprojected
// position (bmfr.cl:929-960).
template <int KN>
__device__ __forceinline__ void tile_taps(const Params& P, const TaaArgs& T, const float2 (&pf)[KN],
                                          f3 (&taps)[KN][4]) {
#pragma unroll
    for (int k = 0; k < KN; ++k) {
#ifdef BMFR_PROBE_K2_NOTAPS  // timing probe (wrong results): no previous-frame taps
        taps[k][0] = taps[k][1] = taps[k][2] = taps[k][3] = f3{pf[k].x, pf[k].y, 0.f};
#else
        taa_load_taps(P, pf[k], T.prev_frame, taps[k]);
#endif
    }
}

// Strip form of the resolve (kStrip): the thread's KN output pixels are KN
// consecutive rows of one column, so their 3x3 neighbourhoods lie in one
// (KN + 2) x 3 window.  Each window row is read from LDS once and reduced to
// its box bounds (min / max of its three values) and its centre value; a
// pixel's box bounds are then the bounds of its three rows' and its cross
// bounds those of the top and bottom centres and the middle row -- the
// sets of bmfr.cl:897-920, grouped differently (exact: taa_clamp_tail).
// CHECK (tiles at the image border): out-of-image neighbours enter as +inf /
// -inf, as in taa_clamp.
template <int TH, int NT, bool CHECK>
__device__ __forceinline__ void resolve_strip(const Params& P, const TaaArgs& T, int x0, int y0,
                                              const float4* __restrict__ Y, const f3 (&me)[TileShape<TH, NT>::KN],
                                              const float2 (&pf)[TileShape<TH, NT>::KN],
                                              const f3 (&hist)[TileShape<TH, NT>::KN]) {
    using S = TileShape<TH, NT, true>;
    const int t = threadIdx.x, tx = t & 63, ty = t >> 6;
    const int r0 = S::row(ty, 0);  // the window's first row is tile row r0 - 1
    struct Row {
        f3 mn, mx;    // box bounds of the row's three neighbours
        f3 clo, chi;  // its centre (as a lower / upper bound: +-inf when out of the image)
    };
    auto reduce_row = [&](int r) {
        f3 lo[3], hi[3];
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
            const float4 q = Y[(r0 + r) * S::HW + tx + dx];
            lo[dx] = hi[dx] = f3{q.x, q.y, q.z};
            if constexpr (CHECK) {
                const int sx = x0 + tx + dx - 1, sy = y0 + r0 + r - 1;
                const bool in = sx >= 0 && sy >= 0 && sx < P.width && sy < P.height;
                lo[dx] = in ? lo[dx] : f3{INFINITY, INFINITY, INFINITY};
                hi[dx] = in ? hi[dx] : f3{-INFINITY, -INFINITY, -INFINITY};
            }
        }
        Row w;
        w.mn = f3{vmin3(lo[0].x, lo[1].x, lo[2].x), vmin3(lo[0].y, lo[1].y, lo[2].y), vmin3(lo[0].z, lo[1].z, lo[2].z)};
        w.mx = f3{vmax3(hi[0].x, hi[1].x, hi[2].x), vmax3(hi[0].y, hi[1].y, hi[2].y), vmax3(hi[0].z, hi[1].z, hi[2].z)};
        w.clo = lo[1];
        w.chi = hi[1];
        return w;
    };
    // min(+inf, a, b, c) / max(-inf, a, b, c): upstream's sets start from +-inf
    auto mn4 = [](float a, float b, float c) { return vmin(vmin3s(INFINITY, a, b), c); };
    auto mx4 = [](float a, float b, float c) { return vmax(vmax3s(-INFINITY, a, b), c); };
    Row w0 = reduce_row(0), w1 = reduce_row(1);
#pragma unroll
    for (int k = 0; k < S::KN; ++k) {
        const Row w2 = reduce_row(k + 2);
        const int x = x0 + tx, y = y0 + r0 + k;
        if (x < P.tx1 && y < P.ty1) {
#ifdef BMFR_PROBE_K2_NORESOLVE  // timing probe (wrong results): no TAA resolve
            const f3 r{me[k].x + w1.mn.x + hist[k].x, me[k].y + w1.mx.y + hist[k].y, me[k].z + w2.clo.z};
#else
            f3 r = me[k];
            if (!taa_offscreen(P, pf[k], T.frame)) {
                const f3 mnb{mn4(w0.mn.x, w1.mn.x, w2.mn.x), mn4(w0.mn.y, w1.mn.y, w2.mn.y),
                             mn4(w0.mn.z, w1.mn.z, w2.mn.z)};
                const f3 mxb{mx4(w0.mx.x, w1.mx.x, w2.mx.x), mx4(w0.mx.y, w1.mx.y, w2.mx.y),
                             mx4(w0.mx.z, w1.mx.z, w2.mx.z)};
                const f3 mnc{mn4(w0.clo.x, w1.mn.x, w2.clo.x), mn4(w0.clo.y, w1.mn.y, w2.clo.y),
                             mn4(w0.clo.z, w1.mn.z, w2.clo.z)};
                const f3 mxc{mx4(w0.chi.x, w1.mx.x, w2.chi.x), mx4(w0.chi.y, w1.mx.y, w2.chi.y),
                             mx4(w0.chi.z, w1.mx.z, w2.chi.z)};
                r = taa_clamp_tail(P, me[k], mnb, mxb, mnc, mxc, hist[k]);
            }
#endif
            st3(T.result, pix(P, x, y), r);
        }
        w0 = w1;
        w1 = w2;
    }
}

// The resolve of the tile's output pixels from the complete window Y
// (bmfr.cl:897-973) and the stores.
template <int TH, int NT, bool ST>
__device__ __forceinline__ void tile_resolve(const Params& P, const TaaArgs& T, int x0, int y0,
                                             const float4* __restrict__ Y, const f3 (&me)[TileShape<TH, NT>::KN],
                                             const float2 (&pf)[TileShape<TH, NT>::KN],
                                             const f3 (&hist)[TileShape<TH, NT>::KN]) {
    using S = TileShape<TH, NT, ST>;
    const int t = threadIdx.x, tx = t & 63, ty = t >> 6;
    // Tiles that reach the image border check every neighbour (bmfr.cl:901);
    // the others have all nine in the image.
    const bool edge = x0 == 0 || y0 == 0 || x0 + 64 >= P.width || y0 + TH >= P.height;
    if constexpr (ST) {
        if (edge) resolve_strip<TH, NT, true>(P, T, x0, y0, Y, me, pf, hist);
        else resolve_strip<TH, NT, false>(P, T, x0, y0, Y, me, pf, hist);
        return;
    }
#pragma unroll
    for (int k = 0; k < S::KN; ++k) {
        const int x = x0 + tx, y = y0 + S::row(ty, k);
        if (x < P.tx1 && y < P.ty1) {
            const int c = (S::row(ty, k) + 1) * S::HW + tx + 1;
            f3 nb[9];
#pragma unroll
            for (int j = 0; j < 9; ++j) {
                const float4 q = Y[c + (j / 3 - 1) * S::HW + (j % 3 - 1)];
                nb[j] = f3{q.x, q.y, q.z};
            }
#ifdef BMFR_PROBE_K2_NORESOLVE  // timing probe (wrong results): no TAA resolve
            f3 r = me[k];
#pragma unroll
            for (int j = 0; j < 9; ++j) r = f3{r.x + nb[j].x, r.y + nb[j].y, r.z + nb[j].z};
            r = f3{r.x + hist[k].x, r.y + hist[k].y, r.z + hist[k].z};
#else
            const f3 r = edge ? taa_clamp<true>(P, x, y, me[k], pf[k], nb, hist[k], T.frame)
                              : taa_clamp<false>(P, x, y, me[k], pf[k], nb, hist[k], T.frame);
#endif
            st3(T.result, pix(P, x, y), r);
        }
    }
}

// One tile.  Y: (64 + 2) * (TH + 2) float4; sE / sRP: the powr tables' LDS
// copies.  COH: the tile runs in the launch that computes its K1 blocks: it
// waits for them and reads their outputs with device-coherent loads.
// Order: current-frame loads, tone map into LDS, then the previous-frame
// taps (their latency under the barrier), each pixel's history as its taps
// arrive (three values live instead of twelve: 89 VGPRs, five waves per
// SIMD, where taps issued before the tone map held 124), the resolve.
template <class IN, int TH, bool COH = false, int NT = 256, bool ST = false>
__device__ __forceinline__ void taa_tile(const Params& P, const TaaArgs& T, int x0, int y0, float4* __restrict__ Y,
                                         double* __restrict__ sE, double2* __restrict__ sRP) {
    using S = TileShape<TH, NT>;
    constexpr int KN = S::KN;
    const int t = threadIdx.x;
    bmfr_powr_tables_to_lds<NT>(sE, sRP, t);
    if constexpr (COH) wait_k1_blocks(P, T, x0, y0, TH);
    int hx = 0, hy = 0;
    ring_pixel<TH, NT>(t, hx, hy);
    TileLoads<IN, KN> L;
    tile_issue<IN, TH, COH, NT, ST>(P, T, x0, y0, hx, hy, L);
    __syncthreads();  // the powr tables are in LDS
    f3 me[KN];
    tile_tone<IN, TH, NT, ST>(P, L, hx, hy, Y, sE, sRP, me);
    f3 taps[KN][4];
    tile_taps<KN>(P, T, L.pf, taps);
    __syncthreads();  // the window is complete
    f3 hist[KN];
#pragma unroll
    for (int k = 0; k < KN; ++k) hist[k] = taa_history(P, L.pf[k], taps[k]);
    tile_resolve<TH, NT, ST>(P, T, x0, y0, Y, me, L.pf, hist);
}

// The TAA part of a one-launch frame kernel (K1 blocks, then the frame's
// TAA tiles; bmfr_fused_cols.hip k_fused_cols_taa, bmfr_fused.hip
// k_fused_rows_taa) of NT threads per work-group: work-group b >= nk1p of
// the launch is tile b - nk1p (64 x frame_taa_h<NT>, XCD-aware order).
// COH: the tiles wait for the K1 blocks of the same launch; a tiled
// context's last work-group then forwards the reach report once every K1
// block of the launch has raised it.
template <int NT>
// Tile height of the one-launch frame's TAA tiles at 256 threads: 16 (four
// output rows per thread; no spills beside K1's registers) against 12: 1080p
// frame -1.2 % (fast_fit), -2.1 % (config 5), -0.4 % (exact); 8: +5 %; 20: 1
// dword of spills, -0.8 %; 24: spills (round 6, profiles/r06_ab_frame_taa_h.txt).
// The standalone K2 keeps 64 x 12 (BMFR_K2_H): its occupancy is its own.
#ifndef BMFR_FRAME_TAA_H
#define BMFR_FRAME_TAA_H 16
#endif
constexpr int frame_taa_h() { return NT == 256 ? BMFR_FRAME_TAA_H : 24; }  // TH / 4 output rows per thread
template <int NT>
struct FrameTaaLds {
    float4 Y[(64 + 2) * (frame_taa_h<NT>() + 2)];
    double sE[kPowrENum];
    double2 sRP[kPowrRPNum];
};
template <class IN, bool COH, int NT>
__device__ __forceinline__ void frame_taa_part(const Params& P2, const TaaArgs& T, int b, int nk1p,
                                               FrameTaaLds<NT>& L) {
    constexpr int TH = frame_taa_h<NT>();
    const int gx = (P2.tx1 - P2.tx0 + 63) / 64, n2 = (int)gridDim.x - nk1p;
    const int gi = xcd_swizzle(b - nk1p, n2);
    taa_tile<IN, TH, COH, NT, kStrip>(P2, T, P2.tx0 + (gi % gx) * 64, P2.ty0 + (gi / gx) * TH, L.Y, L.sE, L.sRP);
    if constexpr (COH) {
        if (T.reach_dev && b == (int)gridDim.x - 1) {
            wait_all_k1_blocks(P2, T);
            forward_reach(T);
        }
    }
}
template <int NT>
inline int frame_taa_tiles(const Params& P) {
    constexpr int TH = frame_taa_h<NT>();
    return ((P.tx1 - P.tx0 + 63) / 64) * ((P.ty1 - P.ty0 + TH - 1) / TH);
}

}  // namespace bmfr
