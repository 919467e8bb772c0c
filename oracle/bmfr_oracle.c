/* bmfr_oracle.c -- CPU restatement of /root/reference/opencl/bmfr.cl.
 *
 * TEST INFRASTRUCTURE ONLY (see bmfr_oracle.h).  Build: oracle/Makefile
 * (gcc -O2 -ffp-contract=off, optional -fopenmp).  The file must be compiled
 * without contraction and without fast-math: every `a*b + c` below is meant as
 * two correctly rounded operations, and fmaf() appears only where the
 * reference's OpenCL library performs a fused multiply-add (dot()).
 *
 * Semantics of the one racy spot in the reference: accumulate_noisy_data's
 * margin work-items read current_noisy at a mirrored pixel while the owner of
 * that pixel overwrites it (bmfr.cl:316-322 vs 478-481).  The oracle defines
 * the race away: every read sees the colour the buffer held before the kernel
 * (SURVEY.md A.4); oracle/ref_wrappers.cl runs the reference the same way
 * (margin work-items first, owners second).
 */
#include "bmfr_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define EDGE 32                 /* BLOCK_EDGE_LENGTH   bmfr.cpp:104 */
#define PIXELS (EDGE * EDGE)    /* BLOCK_PIXELS        bmfr.cpp:105 */
#define LSIZE 256               /* LOCAL_SIZE          bmfr.cpp:116 */
#define SUBS (PIXELS / LSIZE)   /* sub-vectors per work-item in the fitter */

/* BLOCK_OFFSETS, bmfr.cl:267-285: the per-frame shift of the block grid. */
static const int kOffsets[16][2] = {
    {-14, -14}, {4, -6}, {-8, 14}, {8, 0}, {-10, -8}, {2, 12}, {12, -12},
    {-10, 0}, {12, 14}, {-8, -16}, {6, 6}, {-2, -2}, {6, -14}, {-16, 12},
    {14, -4}, {-6, 4}};

/* ---------------------------------------------------------------- sizes -- */
static int buffers(const oracle_cfg *c) { return c->n_not_scaled + c->n_scaled + 3; }
static int workset_w(const oracle_cfg *c) { return EDGE * ((c->width + EDGE - 1) / EDGE); }
static int workset_h(const oracle_cfg *c) { return EDGE * ((c->height + EDGE - 1) / EDGE); }
static int margins_w(const oracle_cfg *c) { return workset_w(c) + EDGE; }
static int margins_h(const oracle_cfg *c) { return workset_h(c) + EDGE; }
int oracle_num_blocks(const oracle_cfg *c) {
    return (margins_w(c) / EDGE) * (margins_h(c) / EDGE); /* FITTER_GLOBAL/256 bmfr.cpp:117 */
}

int oracle_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ----------------------------------------------------------- binary16 -- */
uint16_t oracle_f32_to_f16(float f) {
    /* vstore_half: round to nearest even, overflow to inf (bmfr.cl:258). */
    uint32_t x;
    memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t mag = x & 0x7fffffffu;
    if (mag >= 0x7f800000u) /* inf or nan */
        return (uint16_t)(sign | 0x7c00u | (mag > 0x7f800000u ? 0x200u | ((mag >> 13) & 0x3ffu) : 0u));
    if (mag >= 0x477ff000u) /* >= 65520: rounds to inf */
        return (uint16_t)(sign | 0x7c00u);
    if (mag < 0x38800000u) { /* result subnormal (or zero) in half */
        if (mag < 0x33000000u) /* < 2^-25: rounds to zero (2^-25 exactly ties to even = 0) */
            return (uint16_t)sign;
        uint32_t e = mag >> 23;
        uint32_t m = (mag & 0x7fffffu) | 0x800000u;
        uint32_t shift = 126u - e; /* value = m * 2^(e-150); half ulp 2^-24 */
        uint32_t q = m >> shift;
        uint32_t rem = m & ((1u << shift) - 1u);
        uint32_t halfway = 1u << (shift - 1u);
        if (rem > halfway || (rem == halfway && (q & 1u))) q++;
        return (uint16_t)(sign | q);
    }
    uint32_t e = (mag >> 23) - 112u; /* rebias 127 -> 15 */
    uint32_t m = mag & 0x7fffffu;
    uint32_t q = (e << 10) | (m >> 13);
    uint32_t rem = m & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (q & 1u))) q++;
    return (uint16_t)(sign | q);
}

float oracle_f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1fu;
    uint32_t m = h & 0x3ffu;
    uint32_t x;
    if (e == 0x1fu) {
        x = sign | 0x7f800000u | (m << 13);
    } else if (e == 0) {
        if (m == 0) {
            x = sign;
        } else { /* subnormal half -> normal float */
            int sh = 0;
            while (!(m & 0x400u)) { m <<= 1; sh++; }
            m &= 0x3ffu;
            x = sign | ((uint32_t)(113 - sh) << 23) | (m << 13);
        }
    } else {
        x = sign | ((e + 112u) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

/* LOAD / STORE on tmp_data (bmfr.cl:255-265). */
static float tmp_load(const oracle_cfg *c, const void *tmp, size_t i) {
    return c->half_tmp ? oracle_f16_to_f32(((const uint16_t *)tmp)[i]) : ((const float *)tmp)[i];
}
static void tmp_store(const oracle_cfg *c, void *tmp, size_t i, float v) {
    if (c->half_tmp) ((uint16_t *)tmp)[i] = oracle_f32_to_f16(v);
    else ((float *)tmp)[i] = v;
}

/* ------------------------------------------------------------- helpers -- */
typedef struct { float x, y, z; } f3;

static f3 ld3(const float *b, long i) { f3 r = {b[3 * i], b[3 * i + 1], b[3 * i + 2]}; return r; }
static void st3(float *b, long i, f3 v) { b[3 * i] = v.x; b[3 * i + 1] = v.y; b[3 * i + 2] = v.z; }

/* OpenCL dot() as ROCm device-libs implements it: an fma chain. */
static float dot3(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static float dot4(const float a[4], const float b[4]) {
    return fmaf(a[3], b[3], fmaf(a[2], b[2], fmaf(a[1], b[1], a[0] * b[0])));
}

/* mirror(), bmfr.cl:207-216 (valid for less than one size out of range). */
static int mirror(int i, int size) {
    if (i < 0) return -i - 1;
    if (i >= size) return 2 * size - i - 1;
    return i;
}

/* scale(), bmfr.cl:200-205. */
static float scale(float v, float mn, float mx) {
    if (fabsf(mx - mn) > 1.0f) return (v - mn) / (mx - mn);
    return v - mn;
}

/* random(), bmfr.cl:161-171: integer hash, then a / (float)UINT_MAX. */
static float hash_random(uint32_t a) {
    a = (a + 0x7ed55d16u) + (a << 12);
    a = (a ^ 0xc761c23cu) ^ (a >> 19);
    a = (a + 0x165667b1u) + (a << 5);
    a = (a + 0xd3a2646cu) ^ (a << 9);
    a = (a + 0xfd7046c5u) + (a << 3);
    a = (a ^ 0xb55a4f09u) ^ (a >> 16);
    return (float)a / (float)4294967295u;
}

/* add_random(), bmfr.cl:173-182.  NOISE_AMOUNT is a double literal, so the
 * noise term and the add are double and the result is rounded back to float. */
static float add_random(const oracle_cfg *c, float value, int id, int sub, int feature, int frame) {
    int seed = id + sub * LSIZE + feature * PIXELS + frame * buffers(c) * PIXELS;
    float r = hash_random((uint32_t)seed) - 0.5f;
    double noise = c->noise_amount * (double)2.0f * (double)r;
    return (float)((double)value + noise);
}

/* One FEATURE_BUFFERS entry evaluated on a pixel's normal / position. */
static float feature(int code, f3 n, f3 p) {
    switch (code) {
    case ORACLE_F_ONE: return 1.f;
    case ORACLE_F_NX: return n.x;
    case ORACLE_F_NY: return n.y;
    case ORACLE_F_NZ: return n.z;
    case ORACLE_F_PX: return p.x;
    case ORACLE_F_PY: return p.y;
    case ORACLE_F_PZ: return p.z;
    case ORACLE_F_PX2: return p.x * p.x;
    case ORACLE_F_PY2: return p.y * p.y;
    case ORACLE_F_PZ2: return p.z * p.z;
    case ORACLE_F_PX3: return p.x * p.x * p.x;
    case ORACLE_F_PY3: return p.y * p.y * p.y;
    case ORACLE_F_PZ3: return p.z * p.z * p.z;
    default: return 0.f;
    }
}

/* ---------------------------------------------- accumulate_noisy_data -- */
/* bmfr.cl:287-485.  One call of `item` is one work-item of the
 * (WORKSET+32)x(WORKSET+32) NDRange; new colours of owners are returned in
 * *blended instead of being written back, so that every read in the launch
 * sees the input colours. */
static int noisy_item(const oracle_cfg *c, int gx, int gy, int frame,
    float *out_prev_frame_pixel, uint8_t *accept_bools,
    const float *n_cur, const float *n_prev, const float *p_cur, const float *p_prev,
    const float *noisy_cur, const float *noisy_prev, const uint8_t *spp_prev, uint8_t *spp_cur,
    void *tmp, const float M[16], const float jitter[2], f3 *blended, long *owner_pixel) {
    const int W = c->width, H = c->height, B = buffers(c);
    const int *off = kOffsets[frame % 16];
    const int ux = gx - EDGE / 2 + off[0], uy = gy - EDGE / 2 + off[1]; /* bmfr.cl:314-315 */
    const int px = mirror(ux, W), py = mirror(uy, H);
    const long lin = (long)py * W + px;

    f3 wp = ld3(p_cur, lin);
    f3 nrm = ld3(n_cur, lin);
    f3 cur = ld3(noisy_cur, lin);
    const float wp4[4] = {wp.x, wp.y, wp.z, 1.f};

    float pfx = (float)px, pfy = (float)py;     /* bmfr.cl:325 */
    uint8_t accept = 0;
    float alpha = 1.f;
    f3 prev = {0.f, 0.f, 0.f};
    float sample_spp = 0.f;

    if (frame > 0) {
        /* Column-major VP: .s048c is row 0, .s159d row 1, .s37bf row 3 (bmfr.cl:343-347). */
        const float r0[4] = {M[0], M[4], M[8], M[12]};
        const float r1[4] = {M[1], M[5], M[9], M[13]};
        const float r3[4] = {M[3], M[7], M[11], M[15]};
        float u = dot4(r0, wp4), v = dot4(r1, wp4);
        const float w = dot4(r3, wp4);
        u = u / w; v = v / w;
        u = u + 1.f; v = v + 1.f;
        u = u / 2.f; v = v / 2.f;
        pfx = u * (float)W; pfy = v * (float)H;               /* bmfr.cl:352 */
        pfx = pfx - jitter[0]; pfy = pfy - (1 - jitter[1]);   /* bmfr.cl:353-355 */
        const float flx = floorf(pfx), fly = floorf(pfy);     /* convert_int2_rtn */
        const int ix = (int)flx, iy = (int)fly;
        const float fx = pfx - flx, fy = pfy - fly;
        const float omx = 1.f - fx, omy = 1.f - fy;
        const float wts[4] = {omx * omy, fx * omy, omx * fy, fx * fy};
        float total = 0.f;
        for (int i = 0; i < 4; ++i) {                         /* bmfr.cl:374-419 */
            const int sx = ix + (i & 1), sy = iy + (i >> 1);
            if (sx < 0 || sy < 0 || sx >= W || sy >= H) continue;
            const long s = (long)sy * W + sx;
            f3 pp = ld3(p_prev, s);
            f3 d = {pp.x - wp.x, pp.y - wp.y, pp.z - wp.z};
            if (!(dot3(d, d) < c->position_limit_sq)) continue;
            f3 pn = ld3(n_prev, s);
            f3 dn = {pn.x - nrm.x, pn.y - nrm.y, pn.z - nrm.z};
            if (!(dot3(dn, dn) < c->normal_limit_sq)) continue;
            accept |= (uint8_t)(1 << i);
            sample_spp = sample_spp + wts[i] * (float)spp_prev[s];
            f3 pc = ld3(noisy_prev, s);
            prev.x = prev.x + wts[i] * pc.x;
            prev.y = prev.y + wts[i] * pc.y;
            prev.z = prev.z + wts[i] * pc.z;
            total = total + wts[i];
        }
        if (total > 0.f) {                                    /* bmfr.cl:421-429 */
            prev.x = prev.x / total; prev.y = prev.y / total; prev.z = prev.z / total;
            sample_spp = sample_spp / total;
            alpha = 1.f / (sample_spp + 1.f);
            alpha = fmaxf(alpha, c->blend_alpha);
        }
    }

    uint8_t new_spp = 1;                                      /* bmfr.cl:433-442 */
    if (alpha < 1.f) {
        if (sample_spp > 254.f) new_spp = 255;
        else new_spp = (uint8_t)((int)rintf(sample_spp) + 1);
    }
    spp_cur[lin] = new_spp;

    const float beta = 1.f - alpha;                          /* bmfr.cl:444-445 */
    f3 col = {alpha * cur.x + beta * prev.x, alpha * cur.y + beta * prev.y, alpha * cur.z + beta * prev.z};

    /* Design-matrix row of this work-item (bmfr.cl:448-476). */
    const int bx = gx / EDGE, by = gy / EDGE, xi = gx % EDGE, yi = gy % EDGE;
    const size_t base = ((size_t)by * (margins_w(c) / EDGE) + bx) * (size_t)B * PIXELS
                      + (size_t)yi * EDGE + xi;
    for (int f = 0; f < B; ++f) {
        float v;
        if (f < B - 3) v = feature(c->codes[f], nrm, wp);
        else v = (f == B - 3) ? col.x : (f == B - 2) ? col.y : col.z;
        if (isnan(v)) v = 0.0f;
        if (c->half_tmp) v = fmaxf(fminf(v, 65504.f), -65504.f);
        tmp_store(c, tmp, base + (size_t)f * PIXELS, v);
    }

    if (ux >= 0 && ux < W && uy >= 0 && uy < H) {            /* owners, bmfr.cl:478-484 */
        *blended = col;
        *owner_pixel = lin;
        out_prev_frame_pixel[2 * lin] = pfx;
        out_prev_frame_pixel[2 * lin + 1] = pfy;
        accept_bools[lin] = accept;
        return 1;
    }
    return 0;
}

void oracle_accumulate_noisy_data(const oracle_cfg *c,
    float *out_prev_frame_pixel, uint8_t *accept_bools,
    const float *current_normals, const float *previous_normals,
    const float *current_positions, const float *previous_positions,
    float *current_noisy, const float *previous_noisy,
    const uint8_t *previous_spp, uint8_t *current_spp,
    void *tmp_data, const float M[16], const float jitter[2], int frame) {
    const int MW = margins_w(c), MH = margins_h(c);
    const long items = (long)MW * MH;
    f3 *blended = (f3 *)malloc(sizeof(f3) * (size_t)items);
    long *owner = (long *)malloc(sizeof(long) * (size_t)items);

#pragma omp parallel for schedule(static)
    for (long g = 0; g < items; ++g) {
        owner[g] = -1;
        noisy_item(c, (int)(g % MW), (int)(g / MW), frame, out_prev_frame_pixel, accept_bools,
                   current_normals, previous_normals, current_positions, previous_positions,
                   current_noisy, previous_noisy, previous_spp, current_spp, tmp_data, M, jitter,
                   &blended[g], &owner[g]);
    }
    /* Owners' blended colours land after every read (race-free semantics). */
    for (long g = 0; g < items; ++g)
        if (owner[g] >= 0) st3(current_noisy, owner[g], blended[g]);
    free(blended);
    free(owner);
}

/* ------------------------------------------------------------- fitter -- */
/* parallel_reduction_sum, bmfr.cl:25-44: the exact association of the
 * 256 -> 64 -> 8 -> 1 tree over the per-work-item partials. */
static float tree_sum(const float s_in[LSIZE]) {
    float s[64];
    for (int t = 0; t < 64; ++t) s[t] = s_in[t] + ((s_in[t + 64] + s_in[t + 128]) + s_in[t + 192]);
    float e[8];
    for (int t = 0; t < 8; ++t) {
        float a = s[t + 8];
        for (int k = 2; k < 8; ++k) a = a + s[t + 8 * k];
        e[t] = s[t] + a;
    }
    float r = e[0];
    for (int t = 1; t < 8; ++t) r = r + e[t];
    return r;
}

static float tree_max(const float s_in[LSIZE]) {   /* bmfr.cl:68-87 */
    float s[64];
    for (int t = 0; t < 64; ++t)
        s[t] = fmaxf(fmaxf(fmaxf(s_in[t], s_in[t + 64]), s_in[t + 128]), s_in[t + 192]);
    float e[8];
    for (int t = 0; t < 8; ++t) {
        float a = s[t];
        for (int k = 1; k < 8; ++k) a = fmaxf(a, s[t + 8 * k]);
        e[t] = a;
    }
    float r = e[0];
    for (int t = 1; t < 8; ++t) r = fmaxf(r, e[t]);
    return r;
}

static float tree_min(const float s_in[LSIZE]) {   /* bmfr.cl:46-66 */
    float s[64];
    for (int t = 0; t < 64; ++t)
        s[t] = fminf(fminf(fminf(s_in[t], s_in[t + 64]), s_in[t + 128]), s_in[t + 192]);
    float e[8];
    for (int t = 0; t < 8; ++t) {
        float a = s[t];
        for (int k = 1; k < 8; ++k) a = fminf(a, s[t + 8 * k]);
        e[t] = a;
    }
    float r = e[0];
    for (int t = 1; t < 8; ++t) r = fminf(r, e[t]);
    return r;
}

/* Experiment hook, off in the oracle (tools/panel_rounding.py builds a
 * separate library with -DORACLE_PANEL_EXPERIMENT): with a panel width
 * g_panel > 0, a trailing column beyond the current panel of pivot columns is
 * rounded to half only at the panel's last step -- the arithmetic of a blocked
 * (compact-WY) trailing update -- instead of after every step (bmfr.cl:651). */
#ifdef ORACLE_PANEL_EXPERIMENT
static int g_panel = 0;
void oracle_set_panel(int nb) { g_panel = nb; }
static int panel_rounds(int col, int fb, int B) {
    if (g_panel <= 0 || col >= B - 3) return 1;  /* g_panel < 0: dots-only mode, below */
    int end = (col / g_panel + 1) * g_panel;
    if (end > B - 3) end = B - 3;
    return fb < end || col == end - 1;
}
#define PANEL_ROUNDS(col, fb, B) panel_rounds(col, fb, B)
#else
#define PANEL_ROUNDS(col, fb, B) 1
#endif

/* One fitter work-group (bmfr.cl:490-700) on block g.  The block's design
 * matrix is kept as A[feature][row], row = y*32 + x; work-item t of the
 * reference owns rows t + 256*s, s = 0..3. */
static void fit_block(const oracle_cfg *c, float *weights, float *mins_maxs, void *tmp, int frame, int g) {
    const int B = buffers(c), NS = c->n_not_scaled, FS = c->n_scaled;
    const int RE = B - 2;                          /* R_EDGE, bmfr.cpp:221 */
    const size_t base = (size_t)g * B * PIXELS;
    float A[ORACLE_MAX_FEATURES + 3][PIXELS];
    float part[LSIZE];
    float u[PIXELS];
    /* R[x][y]: column x, row y, float3 channels (plain upper-triangular; the
     * compressed-R aliasing of the reference only touches slots rewritten
     * before use or never read). */
    float R[ORACLE_MAX_FEATURES + 1][ORACLE_MAX_FEATURES + 1][3];
    memset(R, 0, sizeof(R));
#ifdef ORACLE_PANEL_EXPERIMENT
    static _Thread_local float Sh[ORACLE_MAX_FEATURES + 3][PIXELS];
#endif

    for (int f = 0; f < B; ++f)
        for (int r = 0; r < PIXELS; ++r) A[f][r] = tmp_load(c, tmp, base + (size_t)f * PIXELS + r);

    /* Scale the position features to the block's min..max (bmfr.cl:510-542). */
    for (int f = NS; f < B - 3; ++f) {
        float pmax[LSIZE], pmin[LSIZE];
        for (int t = 0; t < LSIZE; ++t) {
            float mx = -INFINITY, mn = INFINITY;
            for (int s = 0; s < SUBS; ++s) {
                const float v = A[f][t + s * LSIZE];
                mx = fmaxf(v, mx);
                mn = fminf(v, mn);
            }
            pmax[t] = mx; pmin[t] = mn;
        }
        const float bmax = tree_max(pmax), bmin = tree_min(pmin);
        const int idx = (g * FS + f - NS) * 2;
        mins_maxs[idx + 0] = bmin;
        mins_maxs[idx + 1] = bmax;
        for (int r = 0; r < PIXELS; ++r) {
            const float v = scale(A[f][r], bmin, bmax);
            A[f][r] = c->half_tmp ? oracle_f16_to_f32(oracle_f32_to_f16(v)) : v;
        }
    }

    /* Householder QR, one column at a time (bmfr.cl:544-656). */
    for (int col = 0; col < B; ++col) {
        const int cl = col < B - 3 ? col : B - 3;   /* col_limited */
        for (int t = 0; t < LSIZE; ++t) {
            float sum = 0.f;
            for (int s = 0; s < SUBS; ++s) {
                const int i = t + s * LSIZE;
                const float v = A[col][i];
                u[i] = v;
                if (i >= cl + 1) sum = sum + v * v;
            }
            part[t] = sum;
        }
        const float sumsq = tree_sum(part);
        /* Work-item `col` (bmfr.cl:580-588). */
        float ulen2 = sumsq;
        const float vlen = sqrtf(sumsq + u[cl] * u[cl]);
        u[cl] = u[cl] - vlen;
        ulen2 = ulen2 + u[cl] * u[cl];
        /* R column (bmfr.cl:574-601); only slots read later are kept. */
        if (col < B - 3) {
            for (int y = 0; y < col; ++y) R[cl][y][0] = R[cl][y][1] = R[cl][y][2] = A[col][y];
            R[cl][col][0] = R[cl][col][1] = R[cl][col][2] = vlen;
        } else {
            const int ch = col - (B - 3);
            for (int y = 0; y < B - 3; ++y) R[cl][y][ch] = A[col][y];
        }
        /* Transform the trailing columns (bmfr.cl:606-655). */
#ifdef ORACLE_PANEL_EXPERIMENT
        /* dots-only mode (g_panel < 0): the trailing columns' dot products from
         * an unrounded shadow, as V^T X with the WY identity would give them;
         * the updates still rounded every step */
        if (g_panel < 0 && col < B - 3 && col % -g_panel == 0)
            for (int f = 0; f < B; ++f)
                for (int r = 0; r < PIXELS; ++r) Sh[f][r] = A[f][r];
#endif
        for (int fb = cl + 1; fb < B; ++fb) {
            float cache[LSIZE][SUBS];
#ifdef ORACLE_PANEL_EXPERIMENT
            const int shadow = g_panel < 0 && col < B - 3 && fb >= (col / -g_panel + 1) * -g_panel;
#endif
            for (int t = 0; t < LSIZE; ++t) {
                float sum = 0.f;
                for (int s = 0; s < SUBS; ++s) {
                    const int i = t + s * LSIZE;
                    if (i >= cl) {
                        float v = A[fb][i];
                        if (col == 0 && fb < B - 3) v = add_random(c, v, t, s, fb, frame);
                        cache[t][s] = v;
#ifdef ORACLE_PANEL_EXPERIMENT
                        if (shadow) {
                            float w = Sh[fb][i];
                            if (col == 0 && fb < B - 3) w = add_random(c, w, t, s, fb, frame);
                            sum = sum + w * u[i];
                            continue;
                        }
#endif
                        sum = sum + v * u[i];
                    }
                }
                part[t] = sum;
            }
            const float dot = tree_sum(part);
            for (int t = 0; t < LSIZE; ++t)
                for (int s = 0; s < SUBS; ++s) {
                    const int i = t + s * LSIZE;
                    if (i >= cl) {
                        float v = cache[t][s];
#ifdef ORACLE_PANEL_EXPERIMENT
                        if (shadow) {
                            float w = Sh[fb][i];
                            if (col == 0 && fb < B - 3) w = add_random(c, w, t, s, fb, frame);
                            Sh[fb][i] = w - 2 * u[i] * dot / ulen2;
                        }
#endif
                        v = v - 2 * u[i] * dot / ulen2;
                        A[fb][i] = c->half_tmp && PANEL_ROUNDS(col, fb, B) ? oracle_f16_to_f32(oracle_f32_to_f16(v)) : v;
                    }
                }
        }
    }

    /* Back substitution (bmfr.cl:658-692); RHS lives in column R_EDGE-1. */
    for (int i = RE - 2; i >= 0; --i) {
        float div[3] = {R[i][i][0], R[i][i][1], R[i][i][2]};
        for (int x = i; x < RE; ++x)
            for (int k = 0; k < 3; ++k) R[x][i][k] = R[x][i][k] / div[k];
        for (int j = i + 1; j < RE - 1; ++j)
            for (int k = 0; k < 3; ++k) R[RE - 1][i][k] = R[RE - 1][i][k] - R[j][i][k];
        for (int y = 0; y <= i; ++y)
            for (int k = 0; k < 3; ++k) R[i][y][k] = R[i][y][k] * R[RE - 1][i][k];
    }
    for (int id = 0; id < B - 3; ++id)              /* bmfr.cl:694-699 */
        for (int k = 0; k < 3; ++k) weights[((size_t)g * (B - 3) + id) * 3 + k] = R[RE - 1][id][k];

    for (int f = 0; f < B; ++f)                     /* tmp_data ends as the reference leaves it */
        for (int r = 0; r < PIXELS; ++r) tmp_store(c, tmp, base + (size_t)f * PIXELS + r, A[f][r]);
}

void oracle_fitter(const oracle_cfg *c, float *weights, float *mins_maxs, void *tmp_data, int frame) {
    const int G = oracle_num_blocks(c);
#pragma omp parallel for schedule(dynamic, 1)
    for (int g = 0; g < G; ++g) fit_block(c, weights, mins_maxs, tmp_data, frame, g);
}

/* ------------------------------------------------------- weighted_sum -- */
void oracle_weighted_sum(const oracle_cfg *c, const float *weights, const float *mins_maxs,
    float *output, const float *current_normals, const float *current_positions, int frame) {
    const int W = c->width, H = c->height, B = buffers(c), NS = c->n_not_scaled, FS = c->n_scaled;
    const int *off = kOffsets[frame % 16];
    const int gw = margins_w(c) / EDGE;
#pragma omp parallel for schedule(static)
    for (long lin = 0; lin < (long)W * H; ++lin) {   /* bmfr.cl:703-758 */
        const int x = (int)(lin % W), y = (int)(lin / W);
        const int g = (x + EDGE / 2 - off[0]) / EDGE + ((y + EDGE / 2 - off[1]) / EDGE) * gw;
        f3 p = ld3(current_positions, lin), n = ld3(current_normals, lin);
        f3 col = {0.f, 0.f, 0.f};
        for (int f = 0; f < B - 3; ++f) {
            float v = feature(c->codes[f], n, p);
            if (f >= NS) {
                const int mi = (g * FS + f - NS) * 2;
                v = scale(v, mins_maxs[mi], mins_maxs[mi + 1]);
            }
            f3 w = ld3(weights, (long)g * (B - 3) + f);
            col.x = col.x + w.x * v;
            col.y = col.y + w.y * v;
            col.z = col.z + w.z * v;
        }
        col.x = col.x < 0.f ? 0.f : col.x;           /* bmfr.cl:750 */
        col.y = col.y < 0.f ? 0.f : col.y;
        col.z = col.z < 0.f ? 0.f : col.z;
        st3(output, lin, col);
    }
}

/* ------------------------------------------- accumulate_filtered_data -- */
/* bmfr.cl:761-857.  powr(x, 0.454545f) is evaluated as the correctly rounded
 * pow in double; the GPU library's powr may differ from it in the last bit, so
 * tone_mapped (and TAA after it) are compared with a tolerance, not bitwise. */
static float powr_f(float x, float y) { return (float)pow((double)x, (double)y); }

void oracle_accumulate_filtered_data(const oracle_cfg *c,
    const float *filtered, const float *in_prev_frame_pixel, const uint8_t *accept_bools,
    const float *albedo, float *tone_mapped, const uint8_t *current_spp,
    const float *acc_prev, float *acc, int frame) {
    const int W = c->width, H = c->height;
#pragma omp parallel for schedule(static)
    for (long lin = 0; lin < (long)W * H; ++lin) {
        f3 fc = ld3(filtered, lin);
        f3 prev = {0.f, 0.f, 0.f};
        float alpha = 1.f;
        if (frame > 0) {
            const uint8_t accept = accept_bools[lin];
            if (accept > 0) {
                const float pfx = in_prev_frame_pixel[2 * lin], pfy = in_prev_frame_pixel[2 * lin + 1];
                const float flx = floorf(pfx), fly = floorf(pfy);
                const int ix = (int)flx, iy = (int)fly;
                const float fx = pfx - flx, fy = pfy - fly;
                const float omx = 1.f - fx, omy = 1.f - fy;
                const float wts[4] = {omx * omy, fx * omy, omx * fy, fx * fy};
                float total = 0.f;
                for (int i = 0; i < 4; ++i) {
                    if (!(accept & (1 << i))) continue;
                    total = total + wts[i];
                    const long s = (long)(iy + (i >> 1)) * W + ix + (i & 1);
                    f3 pc = ld3(acc_prev, s);
                    prev.x = prev.x + wts[i] * pc.x;
                    prev.y = prev.y + wts[i] * pc.y;
                    prev.z = prev.z + wts[i] * pc.z;
                }
                if (total > 0.f) {
                    alpha = 1.f / (float)current_spp[lin];
                    alpha = fmaxf(alpha, c->second_blend_alpha);
                    prev.x = prev.x / total; prev.y = prev.y / total; prev.z = prev.z / total;
                }
            }
        }
        const float beta = 1.f - alpha;
        f3 a = {alpha * fc.x + beta * prev.x, alpha * fc.y + beta * prev.y, alpha * fc.z + beta * prev.z};
        st3(acc, lin, a);
        f3 al = ld3(albedo, lin);
        const float g = 0.454545f;
        f3 t = {fmaxf(0.f, al.x * a.x), fmaxf(0.f, al.y * a.y), fmaxf(0.f, al.z * a.z)};
        t.x = fminf(fmaxf(powr_f(t.x, g), 0.f), 1.f);
        t.y = fminf(fmaxf(powr_f(t.y, g), 0.f), 1.f);
        t.z = fminf(fmaxf(powr_f(t.z, g), 0.f), 1.f);
        st3(tone_mapped, lin, t);
    }
}

/* ---------------------------------------------------------------- taa -- */
static f3 to_ycocg(f3 c) {                  /* bmfr.cl:184-190 */
    const f3 a = {1.f, 2.f, 1.f}, b = {2.f, 0.f, -2.f}, d = {-1.f, 2.f, -1.f};
    f3 r = {dot3(c, a), dot3(c, b), dot3(c, d)};
    return r;
}
static f3 from_ycocg(f3 c) {                /* bmfr.cl:192-198 */
    const f3 a = {0.25f, 0.25f, -0.25f}, b = {0.25f, 0.f, 0.25f}, d = {0.25f, -0.25f, -0.25f};
    f3 r = {dot3(c, a), dot3(c, b), dot3(c, d)};
    return r;
}

void oracle_taa(const oracle_cfg *c, const float *in_prev_frame_pixel, const float *new_frame,
    float *result_frame, const float *prev_frame, int frame) {
    const int W = c->width, H = c->height;
#pragma omp parallel for schedule(static)
    for (long lin = 0; lin < (long)W * H; ++lin) {   /* bmfr.cl:860-974 */
        const int x = (int)(lin % W), y = (int)(lin / W);
        f3 me = ld3(new_frame, lin);
        const float pfx = in_prev_frame_pixel[2 * lin], pfy = in_prev_frame_pixel[2 * lin + 1];
        const float flx = floorf(pfx), fly = floorf(pfy);
        const int ix = (int)flx, iy = (int)fly;
        if (frame == 0 || ix < -1 || iy < -1 || ix >= W || iy >= H) {
            st3(result_frame, lin, me);
            continue;
        }
        f3 mnb = {INFINITY, INFINITY, INFINITY}, mnc = mnb;
        f3 mxb = {-INFINITY, -INFINITY, -INFINITY}, mxc = mxb;
        for (int dy = -1; dy < 2; ++dy)
            for (int dx = -1; dx < 2; ++dx) {
                const int sx = x + dx, sy = y + dy;
                if (sx < 0 || sy < 0 || sx >= W || sy >= H) continue;
                f3 s = (dx == 0 && dy == 0) ? me : ld3(new_frame, (long)sy * W + sx);
                s = to_ycocg(s);
                if (dx == 0 || dy == 0) {
                    mnc.x = fminf(mnc.x, s.x); mnc.y = fminf(mnc.y, s.y); mnc.z = fminf(mnc.z, s.z);
                    mxc.x = fmaxf(mxc.x, s.x); mxc.y = fmaxf(mxc.y, s.y); mxc.z = fmaxf(mxc.z, s.z);
                }
                mnb.x = fminf(mnb.x, s.x); mnb.y = fminf(mnb.y, s.y); mnb.z = fminf(mnb.z, s.z);
                mxb.x = fmaxf(mxb.x, s.x); mxb.y = fmaxf(mxb.y, s.y); mxb.z = fmaxf(mxb.z, s.z);
            }
        f3 prev = {0.f, 0.f, 0.f};
        float total = 0;
        const float fx = pfx - flx, fy = pfy - fly;
        const float omx = 1.f - fx, omy = 1.f - fy;
        /* Taps in the reference's order (bmfr.cl:929-960). */
        const int tx[4] = {ix, ix + 1, ix, ix + 1}, ty[4] = {iy, iy, iy + 1, iy + 1};
        const float tw[4] = {omx * omy, fx * omy, omx * fy, fx * fy};
        for (int i = 0; i < 4; ++i) {
            const int okx = (i & 1) ? (ix < W - 1) : (ix >= 0);
            const int oky = (i >> 1) ? (iy < H - 1) : (iy >= 0);
            if (!(okx && oky)) continue;
            f3 pc = ld3(prev_frame, (long)ty[i] * W + tx[i]);
            prev.x = prev.x + tw[i] * pc.x;
            prev.y = prev.y + tw[i] * pc.y;
            prev.z = prev.z + tw[i] * pc.z;
            total = total + tw[i];
        }
        prev.x = prev.x / total; prev.y = prev.y / total; prev.z = prev.z / total;
        f3 py = to_ycocg(prev);
        f3 lo = {(mnb.x + mnc.x) / 2.f, (mnb.y + mnc.y) / 2.f, (mnb.z + mnc.z) / 2.f};
        f3 hi = {(mxb.x + mxc.x) / 2.f, (mxb.y + mxc.y) / 2.f, (mxb.z + mxc.z) / 2.f};
        f3 cl = {fminf(fmaxf(py.x, lo.x), hi.x), fminf(fmaxf(py.y, lo.y), hi.y), fminf(fmaxf(py.z, lo.z), hi.z)};
        f3 pr = from_ycocg(cl);
        const float a = c->taa_blend_alpha, b = 1.f - a;
        f3 out = {a * me.x + b * pr.x, a * me.y + b * pr.y, a * me.z + b * pr.z};
        st3(result_frame, lin, out);
    }
}
