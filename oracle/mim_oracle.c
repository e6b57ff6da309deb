/*
 * mim_oracle.c — CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY; see
 * mim_oracle.h for who may load it and for the parity-pinning status).
 *
 * Compiled with -O2 -ffp-contract=off (oracle/Makefile): scalar IEEE fp32/fp64 on x86-64 SSE,
 * no FMA contraction, correctly rounded division and sqrt — the floating-point environment of a
 * distro OpenCV build's calib3d code.
 *
 * Every function names the reference call site it serves and the OpenCV routine it restates.
 * OpenCV routines are cited by file (OpenCV 4.5.4, not present in this image).
 */
#include "mim_oracle.h"
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ------------------------------------------------------------------------------------------ */
/* cv::RNG — core/include/opencv2/core/operations.hpp (RNG::next, RNG::uniform(int,int)).      */
/* RANSACPointSetRegistrator::run seeds RNG((uint64)-1) on every call (calib3d/src/ptsetreg.cpp) */
/* ------------------------------------------------------------------------------------------ */
#define ORC_RNG_COEF 4164903690U

uint32_t orc_rng_next(uint64_t* state) {
    *state = (uint64_t)(uint32_t)(*state) * ORC_RNG_COEF + (uint32_t)(*state >> 32);
    return (uint32_t)(*state);
}

void orc_rng_stream(uint64_t seed, uint32_t* out, int64_t n) {
    uint64_t s = seed ? seed : 0xffffffffULL; /* RNG::RNG(uint64) */
    for (int64_t i = 0; i < n; ++i) out[i] = orc_rng_next(&s);
}

static inline int rng_uniform(uint64_t* s, int a, int b, int64_t* used) {
    /* RNG::uniform(int a, int b): a == b ? a : (int)(next() % (b - a) + a) */
    if (a == b) return a;
    ++*used;
    return (int)(orc_rng_next(s) % (unsigned)(b - a) + (unsigned)a);
}

/* ------------------------------------------------------------------------------------------ */
/* knnMatch(k=2) — TestsDetector.cpp:36,60 -> features2d/src/matchers.cpp BFMatcher::knnMatchImpl */
/* -> core/src/batch_distance.cpp batchDistance(NORM_L2, K=2) / BatchDistInvoker              */
/* -> batchDistL2_32f -> hal::normL2Sqr_ (core/src/norm.cpp, SSE path: 4 accumulators x 4 lanes)*/
/* ------------------------------------------------------------------------------------------ */
static float l2sqr_sse_order(const float* a, const float* b, int n) {
    int j = 0;
    float d = 0.f;
    float acc[4][4] = {{0}};
    for (; j <= n - 16; j += 16) {
        for (int v = 0; v < 4; ++v)
            for (int l = 0; l < 4; ++l) {
                float t = a[j + 4 * v + l] - b[j + 4 * v + l];
                acc[v][l] = t * t + acc[v][l]; /* v_muladd without FMA: mul then add */
            }
    }
    if (j > 0) {
        float s[4];
        for (int l = 0; l < 4; ++l) s[l] = ((acc[0][l] + acc[1][l]) + acc[2][l]) + acc[3][l];
        d = (s[0] + s[2]) + (s[1] + s[3]); /* v_reduce_sum (SSE: movehl + add_ss) */
    }
    for (; j < n; ++j) {
        float t = a[j] - b[j];
        d += t * t;
    }
    return d;
}

typedef struct {
    const float *q, *t;
    int nq, nt, dim, row0, row1;
    int32_t* idx;
    float* dist;
} knn_job;

static void* knn_worker(void* arg) {
    knn_job* jb = (knn_job*)arg;
    for (int i = jb->row0; i < jb->row1; ++i) {
        const float* qi = jb->q + (size_t)i * jb->dim;
        int32_t nidx[2] = {-1, -1};
        float fmax = FLT_MAX;
        int32_t dist[2];
        memcpy(&dist[0], &fmax, 4);
        memcpy(&dist[1], &fmax, 4);
        for (int j = 0; j < jb->nt; ++j) {
            float df = sqrtf(l2sqr_sse_order(qi, jb->t + (size_t)j * jb->dim, jb->dim));
            int32_t d;
            memcpy(&d, &df, 4); /* non-negative floats compared as int bit patterns */
            if (d < dist[1]) {
                int k;
                for (k = 0; k >= 0 && dist[k] > d; --k) {
                    nidx[k + 1] = nidx[k];
                    dist[k + 1] = dist[k];
                }
                nidx[k + 1] = j;
                dist[k + 1] = d;
            }
        }
        for (int k = 0; k < 2; ++k) {
            jb->idx[2 * (size_t)i + k] = nidx[k];
            memcpy(&jb->dist[2 * (size_t)i + k], &dist[k], 4);
        }
    }
    return NULL;
}

void orc_knn2_l2(const float* q, int nq, const float* t, int nt, int dim, int32_t* idx, float* dist,
                 int nthreads) {
    if (nq <= 0) return;
    if (nthreads <= 0) nthreads = (int)sysconf(_SC_NPROCESSORS_ONLN);
    if (nthreads > nq) nthreads = nq;
    if (nthreads < 1) nthreads = 1;
    knn_job* jobs = (knn_job*)calloc((size_t)nthreads, sizeof(knn_job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int w = 0; w < nthreads; ++w) {
        jobs[w] = (knn_job){q, t, nq, nt, dim, (int)((long)nq * w / nthreads),
                            (int)((long)nq * (w + 1) / nthreads), idx, dist};
        if (nthreads == 1) knn_worker(&jobs[w]);
        else pthread_create(&th[w], NULL, knn_worker, &jobs[w]);
    }
    if (nthreads > 1)
        for (int w = 0; w < nthreads; ++w) pthread_join(th[w], NULL);
    free(jobs);
    free(th);
}

/* TestsDetector.cpp:66-72 */
int orc_ratio_filter(const int32_t* idx, const float* dist, int nq, float ratio, int32_t* q_out,
                     int32_t* t_out) {
    int n = 0;
    for (int i = 0; i < nq; ++i) {
        if (idx[2 * i] < 0 || idx[2 * i + 1] < 0) continue; /* m.size() == 2 */
        if (dist[2 * i] < ratio * dist[2 * i + 1]) {
            if (q_out) q_out[n] = i;
            if (t_out) t_out[n] = idx[2 * i];
            ++n;
        }
    }
    return n;
}

/* ------------------------------------------------------------------------------------------ */
/* calib3d/src/ptsetreg.cpp : RANSACUpdateNumIters                                           */
/* ------------------------------------------------------------------------------------------ */
int orc_update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = p > 0. ? p : 0.;
    p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.;
    ep = ep < 1. ? ep : 1.;
    double num = 1. - p;
    if (num < DBL_MIN) num = DBL_MIN;
    double denom = 1. - pow(1. - ep, model_points);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    if (denom >= 0 || -num >= max_iters * (-denom)) return max_iters;
    return (int)lrint(num / denom); /* cvRound: round half to even */
}

/* ------------------------------------------------------------------------------------------ */
/* calib3d/src/fundam.cpp : haveCollinearPoints, HomographyEstimatorCallback::checkSubset       */
/* ------------------------------------------------------------------------------------------ */
int orc_have_collinear(const float* xy, int count) {
    int i = count - 1;
    for (int j = 0; j < i; ++j) {
        double dx1 = (double)(xy[2 * j] - xy[2 * i]); /* float subtraction, then widened */
        double dy1 = (double)(xy[2 * j + 1] - xy[2 * i + 1]);
        for (int k = 0; k < j; ++k) {
            double dx2 = (double)(xy[2 * k] - xy[2 * i]);
            double dy2 = (double)(xy[2 * k + 1] - xy[2 * i + 1]);
            if (fabs(dx2 * dy1 - dy2 * dx1) <=
                FLT_EPSILON * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
                return 1;
        }
    }
    return 0;
}

static double det3_rows(double a00, double a01, double a02, double a10, double a11, double a12,
                        double a20, double a21, double a22) {
    /* Matx_DetOp<double,3> (core/include/opencv2/core/matx.inl.hpp) */
    return a00 * (a11 * a22 - a21 * a12) - a01 * (a10 * a22 - a20 * a12) +
           a02 * (a10 * a21 - a20 * a11);
}

int orc_check_subset(const float* s, const float* d) {
    if (orc_have_collinear(s, 4) || orc_have_collinear(d, 4)) return 0;
    static const int tt[4][3] = {{0, 1, 2}, {1, 2, 3}, {0, 2, 3}, {0, 1, 3}};
    int negative = 0;
    for (int i = 0; i < 4; ++i) {
        const int* t = tt[i];
        double dA = det3_rows(s[2 * t[0]], s[2 * t[0] + 1], 1., s[2 * t[1]], s[2 * t[1] + 1], 1.,
                              s[2 * t[2]], s[2 * t[2] + 1], 1.);
        double dB = det3_rows(d[2 * t[0]], d[2 * t[0] + 1], 1., d[2 * t[1]], d[2 * t[1] + 1], 1.,
                              d[2 * t[2]], d[2 * t[2] + 1], 1.);
        negative += dA * dB < 0;
    }
    return !(negative != 0 && negative != 4);
}

/* ------------------------------------------------------------------------------------------ */
/* core/src/lapack.cpp : hypot<double>, JacobiImpl_<double> (the cv::eigen path of a build     */
/* without HAVE_EIGEN; also what cv::solve(DECOMP_EIG) always uses).                           */
/* ------------------------------------------------------------------------------------------ */
static double orc_hypot(double a, double b) {
    a = fabs(a);
    b = fabs(b);
    if (a > b) {
        b /= a;
        return a * sqrt(1 + b * b);
    }
    if (b > 0) {
        a /= b;
        return b * sqrt(1 + a * a);
    }
    return 0;
}

void orc_jacobi(double* A, double* W, double* V, int n) {
    const double eps = DBL_EPSILON;
    int i, j, k, m, iters, maxIters = n * n * 30;
    int indR[16], indC[16];
    double mv = 0;
    for (i = 0; i < n; ++i) {
        for (j = 0; j < n; ++j) V[i * n + j] = 0;
        V[i * n + i] = 1;
    }
    for (k = 0; k < n; ++k) {
        W[k] = A[(n + 1) * k];
        if (k < n - 1) {
            for (m = k + 1, mv = fabs(A[n * k + m]), i = k + 2; i < n; i++) {
                double val = fabs(A[n * k + i]);
                if (mv < val) mv = val, m = i;
            }
            indR[k] = m;
        }
        if (k > 0) {
            for (m = 0, mv = fabs(A[k]), i = 1; i < k; i++) {
                double val = fabs(A[n * i + k]);
                if (mv < val) mv = val, m = i;
            }
            indC[k] = m;
        }
    }
    if (n > 1)
        for (iters = 0; iters < maxIters; iters++) {
            for (k = 0, mv = fabs(A[indR[0]]), i = 1; i < n - 1; i++) {
                double val = fabs(A[n * i + indR[i]]);
                if (mv < val) mv = val, k = i;
            }
            int l = indR[k];
            for (i = 1; i < n; i++) {
                double val = fabs(A[n * indC[i] + i]);
                if (mv < val) mv = val, k = indC[i], l = i;
            }
            double p = A[n * k + l];
            if (fabs(p) <= eps) break;
            double y = (double)((W[l] - W[k]) * 0.5);
            double t = fabs(y) + orc_hypot(p, y);
            double s = orc_hypot(p, t);
            double c = t / s;
            s = p / s;
            t = (p / t) * p;
            if (y < 0) s = -s, t = -t;
            A[n * k + l] = 0;
            W[k] -= t;
            W[l] += t;
            double a0, b0;
#define ORC_ROT(v0, v1) a0 = v0, b0 = v1, v0 = a0 * c - b0 * s, v1 = a0 * s + b0 * c
            for (i = 0; i < k; i++) ORC_ROT(A[n * i + k], A[n * i + l]);
            for (i = k + 1; i < l; i++) ORC_ROT(A[n * k + i], A[n * i + l]);
            for (i = l + 1; i < n; i++) ORC_ROT(A[n * k + i], A[n * l + i]);
            for (i = 0; i < n; i++) ORC_ROT(V[n * k + i], V[n * l + i]);
#undef ORC_ROT
            for (j = 0; j < 2; j++) {
                int idx = j == 0 ? k : l;
                if (idx < n - 1) {
                    for (m = idx + 1, mv = fabs(A[n * idx + m]), i = idx + 2; i < n; i++) {
                        double val = fabs(A[n * idx + i]);
                        if (mv < val) mv = val, m = i;
                    }
                    indR[idx] = m;
                }
                if (idx > 0) {
                    for (m = 0, mv = fabs(A[idx]), i = 1; i < idx; i++) {
                        double val = fabs(A[n * i + idx]);
                        if (mv < val) mv = val, m = i;
                    }
                    indC[idx] = m;
                }
            }
        }
    for (k = 0; k < n - 1; k++) {
        m = k;
        for (i = k + 1; i < n; i++)
            if (W[m] < W[i]) m = i;
        if (k != m) {
            double tmp = W[m];
            W[m] = W[k];
            W[k] = tmp;
            for (i = 0; i < n; i++) {
                tmp = V[n * m + i];
                V[n * m + i] = V[n * k + i];
                V[n * k + i] = tmp;
            }
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* calib3d/src/fundam.cpp : HomographyEstimatorCallback::runKernel (normalized DLT).           */
/* src = M (model/object points), dst = m (scene points), TestsDetector.cpp:78 argument order.  */
/* ------------------------------------------------------------------------------------------ */
static void mat3_mul(const double* a, const double* b, double* c) {
    /* cv::gemm of two 3x3 CV_64F: dot products in k order */
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            c[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
}

int orc_run_kernel(const float* M, const float* m, int count, double H[9]) {
    double LtL[81], W[9], V[81];
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0, sMx = 0, sMy = 0, smx = 0, smy = 0;
    int i;
    for (i = 0; i < count; i++) {
        cmx += m[2 * i];
        cmy += m[2 * i + 1];
        cMx += M[2 * i];
        cMy += M[2 * i + 1];
    }
    cmx /= count;
    cmy /= count;
    cMx /= count;
    cMy /= count;
    for (i = 0; i < count; i++) {
        smx += fabs(m[2 * i] - cmx);
        smy += fabs(m[2 * i + 1] - cmy);
        sMx += fabs(M[2 * i] - cMx);
        sMy += fabs(M[2 * i + 1] - cMy);
    }
    if (fabs(smx) < DBL_EPSILON || fabs(smy) < DBL_EPSILON || fabs(sMx) < DBL_EPSILON ||
        fabs(sMy) < DBL_EPSILON)
        return 0;
    smx = count / smx;
    smy = count / smy;
    sMx = count / sMx;
    sMy = count / sMy;
    double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    memset(LtL, 0, sizeof LtL);
    for (i = 0; i < count; i++) {
        double x = (m[2 * i] - cmx) * smx, y = (m[2 * i + 1] - cmy) * smy;
        double X = (M[2 * i] - cMx) * sMx, Y = (M[2 * i + 1] - cMy) * sMy;
        double Lx[9] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
        double Ly[9] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
        for (int j = 0; j < 9; j++)
            for (int k = j; k < 9; k++) LtL[9 * j + k] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
    }
    for (int j = 0; j < 9; j++) /* completeSymm (upper -> lower) */
        for (int k = 0; k < j; k++) LtL[9 * j + k] = LtL[9 * k + j];
    orc_jacobi(LtL, W, V, 9);
    double Htemp[9], H0[9];
    mat3_mul(invHnorm, &V[72], Htemp);
    mat3_mul(Htemp, Hnorm2, H0);
    double sc = 1. / H0[8]; /* convertTo(_model, type, 1./H0(2,2)) */
    for (i = 0; i < 9; ++i) H[i] = H0[i] * sc;
    return 1;
}

/* HomographyEstimatorCallback::computeError (fp32, Hf = (float)H) */
void orc_compute_error(const float* M, const float* m, int count, const double H[9], float* err) {
    float Hf[8];
    for (int i = 0; i < 8; ++i) Hf[i] = (float)H[i];
    for (int i = 0; i < count; i++) {
        float x = M[2 * i], y = M[2 * i + 1];
        float ww = 1.f / (Hf[6] * x + Hf[7] * y + 1.f);
        float dx = (Hf[0] * x + Hf[1] * y + Hf[2]) * ww - m[2 * i];
        float dy = (Hf[3] * x + Hf[4] * y + Hf[5]) * ww - m[2 * i + 1];
        err[i] = dx * dx + dy * dy;
    }
}

/* RANSACPointSetRegistrator::findInliers */
static int find_inliers(const float* M, const float* m, int count, const double* H, float* err,
                        uint8_t* mask, double thresh) {
    orc_compute_error(M, m, count, H, err);
    float t = (float)(thresh * thresh);
    int nz = 0;
    for (int i = 0; i < count; i++) {
        int f = err[i] <= t;
        mask[i] = (uint8_t)f;
        nz += f;
    }
    return nz;
}

/* RANSACPointSetRegistrator::getSubset (modelPoints = 4) */
static int get_subset(const float* M, const float* m, int count, float* ms1, float* ms2,
                      uint64_t* rng, int max_attempts, int64_t* used) {
    int idx[4];
    for (int iters = 0; iters < max_attempts; ++iters) {
        int i;
        for (i = 0; i < 4; ++i) {
            int idx_i;
            for (;;) {
                idx_i = rng_uniform(rng, 0, count, used);
                int j;
                for (j = 0; j < i; ++j)
                    if (idx[j] == idx_i) break;
                if (j == i) break;
            }
            idx[i] = idx_i;
            ms1[2 * i] = M[2 * idx_i];
            ms1[2 * i + 1] = M[2 * idx_i + 1];
            ms2[2 * i] = m[2 * idx_i];
            ms2[2 * i + 1] = m[2 * idx_i + 1];
        }
        if (orc_check_subset(ms1, ms2)) return 1;
    }
    return 0;
}

/* Study knob (tools/eigen_gap.py), off by default: OpenCV built HAVE_EIGEN solves runKernel's 9x9
 * eigenproblem with Eigen's SelfAdjointEigenSolver instead of JacobiImpl_, so its minimal-sample models
 * can differ from this restatement's in the last bits.  With ulps > 0 every minimal-sample model of
 * orc_ransac gets each of h0..h7 moved by a pseudo-random k in [-ulps, ulps] ulp (splitmix64 of seed,
 * iteration, element), to measure how often such a difference changes the RANSAC outcome. */
static int g_perturb_ulps = 0;
static uint64_t g_perturb_seed = 0;

void orc_set_model_perturbation(int ulps, uint64_t seed) {
    g_perturb_ulps = ulps;
    g_perturb_seed = seed;
}

static uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

/* Study knob: record every iteration's inlier count (-1: runKernel rejected the sample) */
static int* g_count_trace = NULL;
static int g_count_cap = 0;

void orc_set_count_trace(int* counts, int cap) {
    g_count_trace = counts;
    g_count_cap = counts ? cap : 0;
}

static void perturb_model(double H[9], int iter) {
    for (int i = 0; i < 8; ++i) {
        const uint64_t r = splitmix64(g_perturb_seed ^ ((uint64_t)iter << 8) ^ (uint64_t)i);
        const int64_t k = (int64_t)(r % (uint64_t)(2 * (int64_t)g_perturb_ulps + 1)) - g_perturb_ulps;
        if (k > -8 && k < 8) {  /* exact ulp steps */
            for (int64_t j = k; j > 0; --j) H[i] = nextafter(H[i], INFINITY);
            for (int64_t j = k; j < 0; ++j) H[i] = nextafter(H[i], -INFINITY);
        } else {  /* large levels: k times the element's ulp */
            H[i] += (double)k * (nextafter(H[i], INFINITY) - H[i]);
        }
    }
}

/* RANSACPointSetRegistrator::run (calib3d/src/ptsetreg.cpp) */
int orc_ransac(const float* M, const float* m, int count, double thresh, double conf, int max_iters,
               double Hbest[9], uint8_t* bestMask, int* n_iters, int* best_iter,
               int64_t* stream_used) {
    int niters = max_iters > 1 ? max_iters : 1, maxGoodCount = 0, iter;
    uint64_t rng = 0xffffffffffffffffULL;
    int64_t used = 0;
    float ms1[8], ms2[8];
    double model[9];
    if (n_iters) *n_iters = 0;
    if (best_iter) *best_iter = -1;
    if (count < 4) return 0;
    if (count == 4) {
        if (orc_run_kernel(M, m, 4, Hbest) <= 0) return 0;
        memset(bestMask, 1, 4);
        return 1;
    }
    float* err = (float*)malloc(sizeof(float) * (size_t)count);
    uint8_t* mask = (uint8_t*)malloc((size_t)count);
    for (iter = 0; iter < niters; iter++) {
        if (!get_subset(M, m, count, ms1, ms2, &rng, 10000, &used)) {
            if (iter == 0) {
                free(err);
                free(mask);
                if (stream_used) *stream_used = used;
                return 0;
            }
            break;
        }
        if (orc_run_kernel(ms1, ms2, 4, model) <= 0) {
            if (iter < g_count_cap) g_count_trace[iter] = -1;
            continue;
        }
        if (g_perturb_ulps > 0) perturb_model(model, iter);
        int goodCount = find_inliers(M, m, count, model, err, mask, thresh);
        if (iter < g_count_cap) g_count_trace[iter] = goodCount;
        if (goodCount > (maxGoodCount > 3 ? maxGoodCount : 3)) {
            memcpy(bestMask, mask, (size_t)count);
            memcpy(Hbest, model, sizeof model);
            maxGoodCount = goodCount;
            if (best_iter) *best_iter = iter;
            niters = orc_update_num_iters(conf, (double)(count - goodCount) / count, 4, niters);
        }
    }
    free(err);
    free(mask);
    if (n_iters) *n_iters = iter;
    if (stream_used) *stream_used = used;
    return maxGoodCount > 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Levenberg-Marquardt refine: calib3d/src/fundam.cpp HomographyRefineCallback +               */
/* calib3d/src/levmarq.cpp LMSolverImpl (4.5.x), cv::solve/invert(DECOMP_EIG) + SVBkSb          */
/* (core/src/lapack.cpp).  Contract with the real OpenCV is |dH| <= 1e-4, not bits (A.12).      */
/* ------------------------------------------------------------------------------------------ */
static void refine_compute(const float* M, const float* m, int count, const double* h, double* err,
                           double* J) {
    for (int i = 0; i < count; i++) {
        double Mx = M[2 * i], My = M[2 * i + 1];
        double ww = h[6] * Mx + h[7] * My + 1.;
        ww = fabs(ww) > DBL_EPSILON ? 1. / ww : 0;
        double xi = (h[0] * Mx + h[1] * My + h[2]) * ww;
        double yi = (h[3] * Mx + h[4] * My + h[5]) * ww;
        err[i * 2] = xi - m[2 * i];
        err[i * 2 + 1] = yi - m[2 * i + 1];
        if (J) {
            double* Jp = J + 16 * i;
            Jp[0] = Mx * ww;
            Jp[1] = My * ww;
            Jp[2] = ww;
            Jp[3] = Jp[4] = Jp[5] = 0.;
            Jp[6] = -Mx * ww * xi;
            Jp[7] = -My * ww * xi;
            Jp[8] = Jp[9] = Jp[10] = 0.;
            Jp[11] = Mx * ww;
            Jp[12] = My * ww;
            Jp[13] = ww;
            Jp[14] = -Mx * ww * yi;
            Jp[15] = -My * ww * yi;
        }
    }
}

/* A = J^T J, v = J^T r (mulTransposed / gemm GEMM_1_T: sums over rows in order) */
static void normal_eq(const double* J, const double* r, int rows, double* A, double* v) {
    for (int a = 0; a < 8; ++a) {
        for (int b = a; b < 8; ++b) {
            double s = 0;
            for (int k = 0; k < rows; ++k) s += J[8 * k + a] * J[8 * k + b];
            A[8 * a + b] = A[8 * b + a] = s;
        }
        double s = 0;
        for (int k = 0; k < rows; ++k) s += J[8 * k + a] * r[k];
        v[a] = s;
    }
}

/* solve(Ap, v, d, DECOMP_EIG): Jacobi + SVBkSb(eps = 2*DBL_EPSILON), u = v = eigvec rows */
static void solve_eig8(const double* Ain, const double* b, double* x) {
    double a[64], w[8], V[64];
    memcpy(a, Ain, sizeof a);
    orc_jacobi(a, w, V, 8);
    double threshold = 0;
    for (int i = 0; i < 8; i++) threshold += w[i];
    threshold *= DBL_EPSILON * 2;
    for (int j = 0; j < 8; j++) x[j] = 0;
    for (int i = 0; i < 8; i++) {
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        double s = 0;
        for (int j = 0; j < 8; j++) s += V[8 * i + j] * b[j];
        s *= wi;
        for (int j = 0; j < 8; j++) x[j] = x[j] + s * V[8 * i + j];
    }
}

/* invert(A, Ai, DECOMP_EIG) diagonal only (LMSolverImpl uses max |Ai(i,i)|) */
static double inv_diag_max8(const double* Ain) {
    double a[64], w[8], V[64];
    memcpy(a, Ain, sizeof a);
    orc_jacobi(a, w, V, 8);
    double threshold = 0;
    for (int i = 0; i < 8; i++) threshold += w[i];
    threshold *= DBL_EPSILON * 2;
    double maxval = DBL_EPSILON;
    for (int c = 0; c < 8; ++c) {
        double diag = 0;
        for (int i = 0; i < 8; i++) {
            double wi = w[i];
            if (fabs(wi) <= threshold) continue;
            diag += V[8 * i + c] * V[8 * i + c] / wi;
        }
        double ad = fabs(diag);
        if (ad > maxval) maxval = ad;
    }
    return maxval;
}

static double sumsq(const double* r, int n) {
    double s = 0;
    for (int i = 0; i < n; ++i) s += r[i] * r[i];
    return s;
}
static double norm_inf(const double* r, int n) {
    double s = 0;
    for (int i = 0; i < n; ++i) s = fabs(r[i]) > s ? fabs(r[i]) : s;
    return s;
}

static void lm_refine(const float* M, const float* m, int count, double* x /* 8 */) {
    const int maxIters = 10;
    const double eps = FLT_EPSILON;
    int rows = 2 * count;
    double* r = (double*)malloc(sizeof(double) * rows);
    double* rd = (double*)malloc(sizeof(double) * rows);
    double* J = (double*)malloc(sizeof(double) * rows * 8);
    double A[64], Ap[64], v[8], D[8], d[8], xd[8], temp_d[8];
    refine_compute(M, m, count, x, r, J);
    double S = sumsq(r, rows);
    normal_eq(J, r, rows, A, v);
    for (int i = 0; i < 8; ++i) D[i] = A[9 * i];
    const double Rlo = 0.25, Rhi = 0.75;
    double lambda = 1, lc = 0.75;
    int iter = 0;
    for (;;) {
        memcpy(Ap, A, sizeof A);
        for (int i = 0; i < 8; i++) Ap[9 * i] += lambda * D[i];
        solve_eig8(Ap, v, d);
        for (int i = 0; i < 8; ++i) xd[i] = x[i] - d[i];
        refine_compute(M, m, count, xd, rd, NULL);
        double Sd = sumsq(rd, rows);
        /* gemm(A, d, -1, v, 2, temp_d): temp_d = -A d + 2 v */
        for (int i = 0; i < 8; ++i) {
            double s = 0;
            for (int j = 0; j < 8; ++j) s += A[8 * i + j] * d[j];
            temp_d[i] = -s + 2 * v[i];
        }
        double dS = 0;
        for (int i = 0; i < 8; ++i) dS += d[i] * temp_d[i];
        double R = (S - Sd) / (fabs(dS) > DBL_EPSILON ? dS : 1);
        if (R > Rhi) {
            lambda *= 0.5;
            if (lambda < lc) lambda = 0;
        } else if (R < Rlo) {
            double t = 0;
            for (int i = 0; i < 8; ++i) t += d[i] * v[i];
            double nu = (Sd - S) / (fabs(t) > DBL_EPSILON ? t : 1) + 2;
            nu = nu < 2. ? 2. : (nu > 10. ? 10. : nu);
            if (lambda == 0) {
                double maxval = inv_diag_max8(A);
                lambda = lc = 1. / maxval;
                nu *= 0.5;
            }
            lambda *= nu;
        }
        if (Sd < S) {
            S = Sd;
            memcpy(x, xd, sizeof xd);
            refine_compute(M, m, count, x, r, J);
            normal_eq(J, r, rows, A, v);
        }
        iter++;
        int proceed = iter < maxIters && norm_inf(d, 8) >= eps && norm_inf(r, rows) >= eps;
        if (!proceed) break;
    }
    free(r);
    free(rd);
    free(J);
}

/* cv::findHomography (calib3d/src/fundam.cpp), method = RANSAC */
int orc_find_homography(const float* src, const float* dst, int n, double thresh, int max_iters,
                        double conf, double H[9], uint8_t* mask) {
    if (n < 4) return -1; /* CV_Error(StsVecLengthErr) — never reached: TestsDetector.cpp:74 */
    if (thresh <= 0) thresh = 3;
    int result;
    if (n == 4) {
        memset(mask, 1, 4);
        result = orc_run_kernel(src, dst, 4, H) > 0;
    } else {
        result = orc_ransac(src, dst, n, thresh, conf, max_iters, H, mask, NULL, NULL, NULL);
    }
    if (result && n > 4) {
        float* s2 = (float*)malloc(sizeof(float) * 2 * n);
        float* d2 = (float*)malloc(sizeof(float) * 2 * n);
        int k = 0;
        for (int i = 0; i < n; ++i)
            if (mask[i]) { /* compressElems */
                s2[2 * k] = src[2 * i];
                s2[2 * k + 1] = src[2 * i + 1];
                d2[2 * k] = dst[2 * i];
                d2[2 * k + 1] = dst[2 * i + 1];
                ++k;
            }
        if (k > 0) {
            orc_run_kernel(s2, d2, k, H); /* returns 0 on degenerate spread: H kept */
            lm_refine(s2, d2, k, H);      /* H8 = first 8 entries, H22 stays */
        }
        free(s2);
        free(d2);
    }
    if (!result) memset(mask, 0, (size_t)n);
    return result;
}

/* ------------------------------------------------------------------------------------------ */
/* One problem of the detectAtScale view loop, TestsDetector.cpp:58-95                        */
/* ------------------------------------------------------------------------------------------ */
void orc_default_params(orc_params* p) {
    p->ratio = 0.9f;
    p->min_good = 4;
    p->min_inliers = 4;
    p->ransac_thresh = 5.0;
    p->max_iters = 2000;
    p->confidence = 0.995;
    p->det_lo = (double)0.1f; /* constexpr float HOMOGRAPHY_DET_THRESHOLD = 0.1 */
    p->det_hi = (double)10.0f;
}

static double det3(const double* H) {
    /* cv::determinant for a 3x3 CV_64F Mat (core/src/lapack.cpp) */
    double t = H[0] * (H[4] * H[8] - H[5] * H[7]);
    t -= H[1] * (H[3] * H[8] - H[5] * H[6]);
    t += H[2] * (H[3] * H[7] - H[4] * H[6]);
    return t;
}

void orc_match_problem(const float* qdesc, const float* qkp, int nq, const float* tdesc,
                       const float* tkp, int nt, int dim, const orc_params* prm, int knn_threads,
                       orc_result* res, uint8_t* mask_out, int32_t* good_q, int32_t* good_t) {
    memset(res, 0, sizeof *res);
    int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * 2 * (nq > 0 ? nq : 1));
    float* dist = (float*)malloc(sizeof(float) * 2 * (nq > 0 ? nq : 1));
    int32_t* gq = good_q ? good_q : (int32_t*)malloc(sizeof(int32_t) * (nq > 0 ? nq : 1));
    int32_t* gt = good_t ? good_t : (int32_t*)malloc(sizeof(int32_t) * (nq > 0 ? nq : 1));
    orc_knn2_l2(qdesc, nq, tdesc, nt, dim, idx, dist, knn_threads);
    int ng = nq > 0 ? orc_ratio_filter(idx, dist, nq, prm->ratio, gq, gt) : 0;
    res->n_good = ng;
    if (ng < prm->min_good) {
        res->status = 1;
    } else {
        float* src = (float*)malloc(sizeof(float) * 2 * ng);
        float* dst = (float*)malloc(sizeof(float) * 2 * ng);
        uint8_t* mask = (uint8_t*)malloc((size_t)ng);
        for (int i = 0; i < ng; ++i) {
            src[2 * i] = qkp[2 * gq[i]];
            src[2 * i + 1] = qkp[2 * gq[i] + 1];
            dst[2 * i] = tkp[2 * gt[i]];
            dst[2 * i + 1] = tkp[2 * gt[i] + 1];
        }
        int ok;
        if (ng == 4) {
            memset(mask, 1, 4);
            ok = orc_run_kernel(src, dst, 4, res->H) > 0;
            res->iters = 0;
        } else {
            int it = 0;
            ok = orc_ransac(src, dst, ng, prm->ransac_thresh, prm->confidence, prm->max_iters,
                            res->H, mask, &it, NULL, NULL);
            res->iters = it;
            if (ok) {
                int k = 0;
                for (int i = 0; i < ng; ++i)
                    if (mask[i]) {
                        src[2 * k] = src[2 * i];
                        src[2 * k + 1] = src[2 * i + 1];
                        dst[2 * k] = dst[2 * i];
                        dst[2 * k + 1] = dst[2 * i + 1];
                        ++k;
                    }
                if (k > 0) {
                    orc_run_kernel(src, dst, k, res->H);
                    lm_refine(src, dst, k, res->H);
                }
            } else {
                memset(mask, 0, (size_t)ng);
            }
        }
        int ninl = 0;
        for (int i = 0; i < ng; ++i) ninl += mask[i] != 0;
        res->n_inl = ninl;
        if (!ok) {
            res->status = 2;
            memset(res->H, 0, sizeof res->H);
        } else if (ninl < prm->min_inliers) {
            res->status = 3;
        } else {
            res->det = det3(res->H);
            double ad = fabs(res->det);
            res->status = (ad < prm->det_lo || ad > prm->det_hi) ? 4 : 0;
        }
        if (ok && res->status != 3) res->det = det3(res->H);
        if (mask_out) memcpy(mask_out, mask, (size_t)ng);
        free(src);
        free(dst);
        free(mask);
    }
    free(idx);
    free(dist);
    if (!good_q) free(gq);
    if (!good_t) free(gt);
}
