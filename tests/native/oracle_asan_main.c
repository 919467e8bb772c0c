/* Sanitizer driver for the CPU restatement oracle/bmfr_oracle.c (TEST
 * INFRASTRUCTURE): built with
 * -fsanitize=address,undefined by tests/test_sanitizers.py, it runs the five
 * stages over a few frames of seeded random inputs for several
 * configurations (padded sizes, both tmp_data precisions, B = 7 / 13 / 16),
 * so every indexing path of the restatement runs under the sanitizers. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bmfr_oracle.h"

static uint32_t rng = 0x424D4652u;
static float frand(float lo, float hi) {
    rng = rng * 1664525u + 1013904223u;
    return lo + (hi - lo) * (float)(rng >> 8) / 16777216.0f;
}

static void fill(float* p, size_t n, float lo, float hi) {
    for (size_t i = 0; i < n; ++i) p[i] = frand(lo, hi);
}

static int run(int W, int H, int ns, int fs, int half, int frames) {
    oracle_cfg c;
    memset(&c, 0, sizeof c);
    c.width = W;
    c.height = H;
    c.n_not_scaled = ns;
    c.n_scaled = fs;
    for (int i = 0; i < ns + fs; ++i) c.codes[i] = i < ns ? i : 4 + (i - ns);
    c.noise_amount = 1e-2;
    c.blend_alpha = 0.2f;
    c.second_blend_alpha = 0.1f;
    c.taa_blend_alpha = 0.2f;
    c.position_limit_sq = 0.01f;
    c.normal_limit_sq = 0.1f;
    c.half_tmp = half;
    const int B = ns + fs + 3, G = oracle_num_blocks(&c);
    const size_t px = (size_t)W * H, ws = (size_t)(32 * ((W + 31) / 32)) * (32 * ((H + 31) / 32));
    const size_t tmp = (size_t)G * B * 1024 * (half ? 2 : 4);
    float *n[2], *p[2], *noisy[2], *out[2], *res[2];
    uint8_t* spp[2];
    for (int k = 0; k < 2; ++k) {
        n[k] = malloc(px * 12);
        p[k] = malloc(px * 12);
        noisy[k] = malloc(px * 12);
        out[k] = malloc(px * 12);
        res[k] = malloc(px * 12);
        spp[k] = malloc(px);
    }
    float* alb = malloc(px * 12);
    float* filt = malloc(px * 12);
    float* tone = malloc(px * 12);
    float* pp = malloc(px * 8);
    uint8_t* acc = malloc(px);
    void* td = malloc(tmp);
    float* wts = malloc((size_t)G * (B - 3) * 12);
    float* mm = malloc((size_t)G * (fs > 0 ? fs : 1) * 8);
    (void)ws;
    double sum = 0;
    for (int f = 0; f < frames; ++f) {
        const int cur = f & 1, prv = 1 - cur;
        fill(n[cur], px * 3, -1, 1);
        fill(p[cur], px * 3, -4, 4);
        fill(noisy[cur], px * 3, 0, 2);
        fill(alb, px * 3, 0.1f, 0.9f);
        float vp[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0.1f, 0.01f * f, 0, 0, 1}, jit[2] = {0.5f, 0.25f};
        oracle_accumulate_noisy_data(&c, pp, acc, n[cur], n[prv], p[cur], p[prv], noisy[cur], noisy[prv], spp[prv],
                                     spp[cur], td, vp, jit, f);
        oracle_fitter(&c, wts, mm, td, f);
        oracle_weighted_sum(&c, wts, mm, filt, n[cur], p[cur], f);
        oracle_accumulate_filtered_data(&c, filt, pp, acc, alb, tone, spp[cur], out[prv], out[cur], f);
        oracle_taa(&c, pp, tone, res[cur], res[prv], f);
        for (size_t i = 0; i < px * 3; ++i) sum += isfinite(res[cur][i]) ? res[cur][i] : 0;
    }
    printf("%dx%d ns=%d fs=%d half=%d: checksum %.6f\n", W, H, ns, fs, half, sum);
    for (int k = 0; k < 2; ++k) {
        free(n[k]);
        free(p[k]);
        free(noisy[k]);
        free(out[k]);
        free(res[k]);
        free(spp[k]);
    }
    free(alb);
    free(filt);
    free(tone);
    free(pp);
    free(acc);
    free(td);
    free(wts);
    free(mm);
    return 0;
}

int main(void) {
    run(48, 48, 4, 6, 1, 3);
    run(100, 72, 4, 9, 0, 3);
    run(70, 48, 1, 3, 1, 3);  /* sizes obey the reference's mirror() range: WORKSET + 30 <= 2 * size */
    run(64, 64, 4, 0, 0, 2);
    return 0;
}
