/* Sanitizer driver for the CPU restatement (oracle/mim_oracle.c, oracle/sift_oracle.c): SURVEY.md §5's
 * host sanitizers.  tests/test_sanitizers.py builds it twice — plain and with
 * -fsanitize=address,undefined — runs both and requires a clean exit and identical output.
 *
 * Exercises every entry point the tests and the bench use: the kNN (2 threads, an empty train set,
 * ties), the ratio filter, findHomography on planted points and on degenerate input (n = 4 collinear),
 * one whole problem (orc_match_problem), Jacobi, resize at the reference's scales, SIFT with and
 * without a mask, and an image too small for any octave. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/mim_oracle.h"
#include "../../oracle/sift_oracle.h"

static uint64_t g_s = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
    g_s ^= g_s << 13;
    g_s ^= g_s >> 7;
    g_s ^= g_s << 17;
    return (uint32_t)(g_s >> 11);
}
static float urand(float lo, float hi) { return lo + (hi - lo) * (float)(rnd() & 0xFFFFFF) / 16777216.0f; }

static uint64_t fnv(uint64_t h, const void* p, size_t n) {
    const unsigned char* b = (const unsigned char*)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001B3ull;
    return h;
}

static void sift_like(float* d, int n) {
    for (int i = 0; i < n * 128; ++i) d[i] = (float)((rnd() % 7 == 0) ? rnd() % 120 : rnd() % 12);
}

static void apply_h(const double H[9], float x, float y, float* u, float* v) {
    const double w = H[6] * x + H[7] * y + H[8];
    *u = (float)((H[0] * x + H[1] * y + H[2]) / w);
    *v = (float)((H[3] * x + H[4] * y + H[5]) / w);
}

static void matching(void) {
    const int nq = 300, nt = 700;
    float* q = malloc(sizeof(float) * nq * 128);
    float* t = malloc(sizeof(float) * nt * 128);
    float* qkp = malloc(sizeof(float) * nq * 2);
    float* tkp = malloc(sizeof(float) * nt * 2);
    sift_like(q, nq);
    sift_like(t, nt);
    const double Ht[9] = {0.95, -0.1, 20, 0.08, 1.02, -12, 1e-5, -2e-5, 1};
    for (int i = 0; i < nq; ++i) {
        qkp[2 * i] = urand(0, 640);
        qkp[2 * i + 1] = urand(0, 480);
    }
    for (int i = 0; i < nt; ++i) {
        tkp[2 * i] = urand(0, 640);
        tkp[2 * i + 1] = urand(0, 480);
    }
    for (int i = 0; i < 120; ++i) {  /* planted copies; every other one at H(model point) */
        const int j = 3 * i + 1;
        memcpy(t + (size_t)j * 128, q + (size_t)i * 128, sizeof(float) * 128);
        t[(size_t)j * 128 + (i % 128)] += 1.0f;
        if (i % 2 == 0) apply_h(Ht, qkp[2 * i], qkp[2 * i + 1], &tkp[2 * j], &tkp[2 * j + 1]);
    }
    memcpy(t + 5 * 128, t + 4 * 128, sizeof(float) * 128); /* an exact tie */
    int32_t* idx = malloc(sizeof(int32_t) * nq * 2);
    float* dist = malloc(sizeof(float) * nq * 2);
    orc_knn2_l2(q, nq, t, nt, 128, idx, dist, 2);
    uint64_t h = fnv(0xCBF29CE484222325ull, idx, sizeof(int32_t) * nq * 2);
    h = fnv(h, dist, sizeof(float) * nq * 2);
    orc_knn2_l2(q, nq, t, 0, 128, idx, dist, 1); /* empty train set: no matches */
    h = fnv(h, idx, sizeof(int32_t) * nq * 2);
    orc_knn2_l2(q, nq, t, nt, 128, idx, dist, 1);
    int32_t* gq = malloc(sizeof(int32_t) * nq);
    int32_t* gt = malloc(sizeof(int32_t) * nq);
    const int ng = orc_ratio_filter(idx, dist, nq, 0.9f, gq, gt);
    h = fnv(h, gq, sizeof(int32_t) * ng);
    printf("knn %016llx good %d\n", (unsigned long long)h, ng);

    float* src = malloc(sizeof(float) * 2 * (ng + 4));
    float* dst = malloc(sizeof(float) * 2 * (ng + 4));
    for (int i = 0; i < ng; ++i) {
        src[2 * i] = qkp[2 * gq[i]];
        src[2 * i + 1] = qkp[2 * gq[i] + 1];
        dst[2 * i] = tkp[2 * gt[i]];
        dst[2 * i + 1] = tkp[2 * gt[i] + 1];
    }
    double H[9];
    uint8_t* mask = calloc(ng + 4, 1);
    const int ok = orc_find_homography(src, dst, ng, 5.0, 2000, 0.995, H, mask);
    printf("homography %d %016llx\n", ok, (unsigned long long)fnv(fnv(0, H, sizeof H), mask, ng));
    float line[8] = {0, 0, 1, 1, 2, 2, 3, 3};
    const int ok2 = orc_find_homography(line, line, 4, 5.0, 2000, 0.995, H, mask);
    printf("collinear %d\n", ok2);

    orc_params prm;
    orc_default_params(&prm);
    orc_result res;
    uint8_t* m2 = calloc(nq, 1);
    orc_match_problem(q, qkp, nq, t, tkp, nt, 128, &prm, 2, &res, m2, gq, gt);
    printf("problem n_good %d n_inl %d status %d iters %d %016llx\n", res.n_good, res.n_inl, res.status, res.iters,
           (unsigned long long)fnv(fnv(0, res.H, sizeof res.H), m2, res.n_good));

    double A[81], W[9], V[81];
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j <= i; ++j) A[9 * i + j] = A[9 * j + i] = urand(-1, 1);
    orc_jacobi(A, W, V, 9);
    printf("jacobi %016llx\n", (unsigned long long)fnv(fnv(0, W, sizeof W), V, sizeof V));
    free(q); free(t); free(qkp); free(tkp); free(idx); free(dist); free(gq); free(gt); free(src); free(dst);
    free(mask); free(m2);
}

static void features(void) {
    const int R = 120, C = 160;
    uint8_t* img = malloc(R * C);
    for (int y = 0; y < R; ++y)
        for (int x = 0; x < C; ++x) {
            double v = 100;
            for (int k = 0; k < 8; ++k) {
                const double cy = 15 + 13 * k, cx = 20 + 17 * k, s = 3 + k;
                v += (k % 2 ? 70 : -60) * exp(-((y - cy) * (y - cy) + (x - cx) * (x - cx)) / (2 * s * s));
            }
            v += (double)(rnd() % 7) - 3;
            img[y * C + x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : lrint(v));
        }
    uint64_t h = 0;
    const double sc[5] = {0.7, 0.85, 1.0, 1.15, 1.3};
    for (int i = 0; i < 5; ++i) {
        const float f = (float)sc[i];
        const int dr = (int)lrint(R * (double)f), dc = (int)lrint(C * (double)f);
        uint8_t* d = malloc((size_t)dr * dc);
        orc_resize_linear_u8(img, R, C, d, dr, dc, (double)f, (double)f);
        h = fnv(h, d, (size_t)dr * dc);
        free(d);
    }
    printf("resize %016llx\n", (unsigned long long)h);
    const int cap = 4096;
    orc_keypoint* kp = malloc(sizeof(orc_keypoint) * cap);
    float* desc = malloc(sizeof(float) * 128 * cap);
    int n = orc_sift_detect_compute(img, R, C, NULL, cap, kp, desc);
    printf("sift %d %016llx\n", n, (unsigned long long)fnv(fnv(0, kp, sizeof(orc_keypoint) * n), desc, sizeof(float) * 128 * n));
    uint8_t* mask = calloc(R * C, 1);
    for (int y = 20; y < 100; ++y) memset(mask + y * C + 30, 255, 100);
    n = orc_sift_detect_compute(img, R, C, mask, cap, kp, desc);
    printf("sift-mask %d %016llx\n", n, (unsigned long long)fnv(fnv(0, kp, sizeof(orc_keypoint) * n), desc, sizeof(float) * 128 * n));
    n = orc_sift_detect_compute(img, R, C, NULL, 3, kp, desc); /* capacity below the count */
    printf("sift-cap %d\n", n);
    n = orc_sift_detect_compute(img, 3, 5, NULL, cap, kp, desc); /* no octave */
    printf("sift-tiny %d\n", n);
    free(img); free(kp); free(desc); free(mask);
}

int main(void) {
    matching();
    features();
    printf("OK\n");
    return 0;
}
