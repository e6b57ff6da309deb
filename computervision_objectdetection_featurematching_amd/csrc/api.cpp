// api.cpp — the C ABI of include/mim.h: context, descriptor sets, batch orchestration.
//
// Host side of the drop-in boundary for TestsDetector.cpp:58-95.  Everything numeric runs in the
// HIP kernels of knn.hip / ransac.hip; this file only allocates, builds problem tables and
// enqueues launches on the ctx stream.  There is no CPU compute path: a missing device or a
// failed launch is reported as MIM_EDEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mim.h"
#include "../../include/mim_detect.hpp"
#include "mim_internal.h"

namespace mim {
void launch_prep_batch(const PrepJob* jobs, int njobs, int total_tiles, hipStream_t st);
void launch_knn(const ProbDev* probs, const KnnWork* works, int n_works, const int* seg_start, int n_blocks, Top2* parts,
                int* dyn_ctr, hipStream_t st);
int knn_blocks_per_cu();
void launch_ratio(const ProbDev* probs, int n_probs, const Top2* parts, float ratio, int32_t* good_q,
                  int32_t* good_t, float4* pts, int* n_good, int32_t* knn_idx, float* knn_dist,
                  hipStream_t st);
void launch_knn_emit(const ProbDev* probs, int nq, const Top2* parts, int32_t* knn_idx, float* knn_dist,
                     hipStream_t st);
void launch_inlier_gather(const ProbDev* probs, int n, const mim_result* res, const int32_t* good_t,
                          const uint8_t* masks, const long long* offs, const float* scales, float2* out, hipStream_t st);
size_t ransac_chain_bytes();
void launch_rng_stream(const unsigned long long* seg_state, uint32_t* out, long long len, int seg, int n_seg,
                       hipStream_t s);
void ransac_enqueue(const RansacParams& prm, int n_probs, const ProbDev* probs, const float4* pts,
                    const int* n_good, const RansacBufs& b, uint8_t* masks, mim_result* results, int raw,
                    hipStream_t s, void (*mark)(void*, const char*, hipStream_t), void* mark_ctx, int exact_all);
}  // namespace mim

using namespace mim;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max(bytes, (size_t)4096);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

// Bump arena for per-set device storage; mim_sets_clear() rewinds it without freeing.
struct Arena {
    std::vector<std::pair<char*, size_t>> chunks;
    size_t chunk_i = 0, off = 0;
    hipError_t alloc(size_t bytes, void** out) {
        bytes = (bytes + 255) & ~size_t(255);
        while (chunk_i < chunks.size() && off + bytes > chunks[chunk_i].second) {
            ++chunk_i;
            off = 0;
        }
        if (chunk_i == chunks.size()) {
            size_t sz = std::max(bytes, (size_t)256 << 20);
            char* p = nullptr;
            hipError_t e = hipMalloc(&p, sz);
            if (e != hipSuccess) return e;
            chunks.push_back({p, sz});
            off = 0;
        }
        *out = chunks[chunk_i].first + off;
        off += bytes;
        return hipSuccess;
    }
    void rewind() { chunk_i = 0; off = 0; }
    struct Mark {
        size_t chunk_i, off;
        bool operator<(const Mark& o) const { return chunk_i < o.chunk_i || (chunk_i == o.chunk_i && off < o.off); }
    };
    Mark pos() const { return Mark{chunk_i, off}; }
    void seek(Mark m) { chunk_i = m.chunk_i; off = m.off; }
    void release() {
        for (auto& c : chunks) (void)hipFree(c.first);
        chunks.clear();
        rewind();
    }
};

struct SetRec {
    SetDev d;
    Arena::Mark mark;  // the arena before the set's storage (mim_sets_truncate)
};

// Pinned staging for the per-batch tables, two generations: a batch's host->device table copies
// are stream-ordered, so the host never waits for the previous batch; a generation is rewritten
// only after the event of its last copy (two batches back) has completed.
struct PinnedStage {
    char* p[2] = {nullptr, nullptr};
    size_t cap[2] = {0, 0};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool used[2] = {false, false};
    int par = 0;
    hipError_t acquire(size_t bytes, char** out) {
        par ^= 1;
        if (used[par]) {
            hipError_t e = hipEventSynchronize(ev[par]);
            if (e != hipSuccess) return e;
        }
        if (!ev[par]) {
            hipError_t e = hipEventCreateWithFlags(&ev[par], hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        if (bytes > cap[par]) {
            if (p[par]) (void)hipHostFree(p[par]);
            p[par] = nullptr;
            cap[par] = 0;
            hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p[par]), std::max(bytes, (size_t)1 << 16));
            if (e != hipSuccess) return e;
            cap[par] = std::max(bytes, (size_t)1 << 16);
        }
        *out = p[par];
        return hipSuccess;
    }
    hipError_t release_after(hipStream_t s) {  // the copies from the current generation are enqueued
        used[par] = true;
        return hipEventRecord(ev[par], s);
    }
    void destroy() {
        for (int i = 0; i < 2; ++i) {
            if (ev[i]) (void)hipEventSynchronize(ev[i]);
            if (p[i]) (void)hipHostFree(p[i]);
            if (ev[i]) (void)hipEventDestroy(ev[i]);
            p[i] = nullptr;
            ev[i] = nullptr;
        }
    }
};

}  // namespace

namespace mim {
// RANSAC workspace (definition shared with ransac.hip through this layout)
struct RansacWs {
    DevBuf state, samples, hyp, counts, bounds, flags, irr_bits, irr, irr_cnt, pass_bits, defer, defer_n, chains, best_h, cand, ncand, cex, cH, decided, stream,
        scratch, inl, tiles, err;
    long long stream_len = 0;
};
}  // namespace mim

struct mim_ctx {
    int device = 0;
    hipStream_t own = nullptr, stream = nullptr;
    std::mutex mu;
    std::string err;
    Arena arena;
    std::vector<SetRec> sets;
    // batch workspace
    DevBuf probs, works, parts, good_q, good_t, pts, n_good, results, masks, knn_idx, knn_dist, inl_tab, inl_out, knn_ctr;
    RansacWs rws;
    std::vector<ProbDev> h_probs;
    int n_works = 0;  // distance segments of the current batch (works, then the per-block segment starts)
    std::vector<long long> h_good_off;
    PinnedStage stage;
    // sets created since the last batch: their prep runs as one launch at the next build_tables
    std::vector<PrepJob> pend;
    std::vector<int> pend_set;
    // per prep flush: the lowest set id it covered and the arena after its flags block
    std::vector<std::pair<int, Arena::Mark>> flushes;
    PinnedStage prep_stage;
    DevBuf prep_jobs;
    int last_n = 0;
    // the last mim_batch_run, kept so that mim_batch_results can re-run it on a longer RNG stream
    // (possible while its sets are intact: sets_gen unchanged since the batch)
    std::vector<mim_problem> last_problems;
    mim_params last_params{};
    long long sets_gen = 0, last_gen = -1;
    // the last batch is mim_find_homography's one record (no set table: no inlier points to gather)
    bool last_fh = false;
    // MIM_CAND_CAP: candidate-list capacity override (test knob for the replay's overflow rescan)
    int cand_cap = 0;
    // MIM_ATTEMPT_REP_CAP: the attempt kernel's redraw-list capacity (test knob for its in-place path)
    int rep_cap = 0;
    // MIM_STREAM_DRAWS: initial RNG stream length (test knob for the grow-and-re-run path)
    long long stream_draws = 0;
    // MIM_RANSAC_EXACT=1: evaluate every hypothesis exactly (reference mode for cross-checks)
    int exact_all = 0;
    int knn_grid = 0;      // resident distance-kernel blocks on the device (first batch)
    int n_knn_blocks = 0;  // distance-kernel blocks of the current batch (<= knn_grid)
    bool knn_dyn = false;  // current batch's distance work as 8 per-XCD lists pulled dynamically
    hipStream_t cur = nullptr;  // stream the enqueue helpers launch on
    // sampler stream (RansacBufs::s2): the next chunk's getSubset replay beside this chunk's
    // selection kernels (MIM_SAMPLER_STREAM=0: one stream)
    hipStream_t samp = nullptr;
    hipEvent_t ev_samp_fork = nullptr, ev_samp[2] = {nullptr, nullptr};
    int samp_on = -1;
    // timing: events per stream, durations summed per kernel name over the streams
    bool timing = false;
    struct Ev {
        std::string name;
        hipStream_t s;
        hipEvent_t e;
        int seq;  // batch the event belongs to: spans are taken within one batch only
    };
    int ev_seq = 0;
    std::vector<Ev> evs;
    std::vector<hipEvent_t> ev_pool;  // recycled events (creating one per mark costs host time)
    std::map<std::string, double> last_ms;
    mim::SiftWs* sift = nullptr;
    std::vector<mim::SiftWs*> sift_scales;  // mim_sift_detect_compute_scales: one per scale + the scene  // SIFT pyramid / candidate / descriptor workspace (first use)
};

static mim_status fail(mim_ctx* c, mim_status code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}

#define HIPCHK(c, expr)                                                                          \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return fail((c), e_ == hipErrorOutOfMemory ? MIM_ENOMEM : MIM_EDEVICE, "%s: %s (%s:%d)", \
                        #expr, hipGetErrorString(e_), __FILE__, __LINE__);                       \
    } while (0)

extern "C" {

const char* mim_version(void) { return "mim 0.1.0 (gfx950)"; }

void mim_default_params(mim_params* p) {
    p->ratio = 0.9f;          // TestsDetector.cpp:21
    p->min_good = 4;          // :22, :74
    p->min_inliers = 4;       // :22, :81
    p->ransac_thresh = 5.0;   // :23
    p->max_iters = 2000;      // findHomography default
    p->confidence = 0.995;    // findHomography default
    p->det_lo = (double)0.1f; // :24 (constexpr float)
    p->det_hi = (double)10.0f;  // :25
}

mim_status mim_ctx_create(int device, mim_ctx** out) {
    if (!out) return MIM_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MIM_EDEVICE;
    if (device < 0 || device >= ndev) return MIM_EINVAL;
    if (hipSetDevice(device) != hipSuccess) return MIM_EDEVICE;
    mim_ctx* c = new mim_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return MIM_EDEVICE;
    }
    c->stream = c->own;
    c->cur = c->own;
    const char* ex = getenv("MIM_RANSAC_EXACT");
    c->exact_all = (ex && ex[0] == '1') ? 1 : 0;
    const char* cc = getenv("MIM_CAND_CAP");
    c->cand_cap = cc ? std::max(1, atoi(cc)) : 0;
    const char* rc = getenv("MIM_ATTEMPT_REP_CAP");
    c->rep_cap = rc ? std::max(1, atoi(rc)) : 0;
    const char* sd = getenv("MIM_STREAM_DRAWS");
    c->stream_draws = sd ? std::max(4096LL, atoll(sd)) : 0;
    *out = c;
    return MIM_OK;
}

void mim_ctx_destroy(mim_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto& e : c->evs) (void)hipEventDestroy(e.e);
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->samp) (void)hipStreamSynchronize(c->samp);
    if (c->ev_samp_fork) (void)hipEventDestroy(c->ev_samp_fork);
    for (auto e : c->ev_samp)
        if (e) (void)hipEventDestroy(e);
    if (c->samp) (void)hipStreamDestroy(c->samp);
    mim::sift_ws_destroy(c->sift);
    for (mim::SiftWs* w : c->sift_scales) mim::sift_ws_destroy(w);
    c->stage.destroy();
    c->prep_stage.destroy();
    c->arena.release();
    for (DevBuf* b : {&c->probs, &c->works, &c->parts, &c->good_q, &c->good_t, &c->pts, &c->n_good,
                      &c->results, &c->masks, &c->knn_idx, &c->knn_dist, &c->inl_tab, &c->inl_out, &c->knn_ctr, &c->rws.state, &c->rws.samples,
                      &c->rws.hyp, &c->rws.counts, &c->rws.bounds, &c->rws.flags, &c->rws.irr_bits, &c->rws.irr, &c->rws.irr_cnt, &c->rws.pass_bits, &c->rws.defer, &c->rws.defer_n, &c->rws.chains, &c->rws.best_h, &c->rws.cand, &c->rws.ncand, &c->rws.cex, &c->rws.cH, &c->rws.decided, &c->rws.stream, &c->rws.scratch, &c->rws.inl, &c->rws.tiles, &c->rws.err, &c->prep_jobs})
        b->release();
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

const char* mim_last_error(const mim_ctx* c) { return c ? c->err.c_str() : "null ctx"; }

mim_status mim_ctx_set_stream(mim_ctx* c, void* stream) {
    if (!c) return MIM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    c->stream = stream ? (hipStream_t)stream : c->own;
    return MIM_OK;
}

mim_status mim_ctx_set_sampler_stream(mim_ctx* c, int32_t on) {
    if (!c) return MIM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    c->samp_on = on != 0;  // the stream itself is created on the first batch that uses it
    return MIM_OK;
}

void* mim_ctx_get_stream(const mim_ctx* c) { return c ? (void*)c->stream : nullptr; }

mim_status mim_synchronize(mim_ctx* c) {
    if (!c) return MIM_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MIM_OK;
}

mim_status mim_set_timing(mim_ctx* c, int32_t enable) {
    if (!c) return MIM_EINVAL;
    c->timing = enable != 0;
    return MIM_OK;
}

double mim_last_kernel_ms(mim_ctx* c, const char* name) {
    if (!c || !name) return -1;
    auto it = c->last_ms.find(name);
    return it == c->last_ms.end() ? -1 : it->second;
}

// sync: wait for the copies of host rows before returning (false: the caller waits once for several)
static mim_status set_create_locked(mim_ctx* c, const float* desc, const float* kp, int32_t n, int32_t dim,
                                    int32_t on_device, int32_t* set_id, bool sync = true) {
    if (!set_id || n < 0 || (n > 0 && (!desc || !kp))) return fail(c, MIM_EINVAL, "set_create: bad arguments");
    if (dim != kDim) return fail(c, MIM_EINVAL, "set_create: dim must be %d (got %d)", kDim, dim);
    HIPCHK(c, hipSetDevice(c->device));
    SetRec r{};
    r.mark = c->arena.pos();
    r.d.n = n;
    r.d.n_tiles = (n + 63) / 64;
    const size_t tiles = (size_t)std::max(r.d.n_tiles, 1);
    void *frag, *norm;
    HIPCHK(c, c->arena.alloc(tiles * kTileBytes, &frag));
    HIPCHK(c, c->arena.alloc(tiles * kNormWords * sizeof(int), &norm));
    const float* f32 = desc;
    const float* kpd = kp;
    if (!on_device && n > 0) {
        void *df, *dk;
        HIPCHK(c, c->arena.alloc((size_t)n * kDim * sizeof(float), &df));
        HIPCHK(c, c->arena.alloc((size_t)n * 2 * sizeof(float), &dk));
        HIPCHK(c, hipMemcpyAsync(df, desc, (size_t)n * kDim * sizeof(float), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(dk, kp, (size_t)n * 2 * sizeof(float), hipMemcpyHostToDevice, c->stream));
        f32 = (const float*)df;
        kpd = (const float*)dk;
    }
    r.d.frag = (const int8_t*)frag;
    r.d.norm = (const int*)norm;
    r.d.f32 = f32;
    r.d.kp = (const float2*)kpd;
    r.d.flags = nullptr;  // assigned when the prep is flushed
    if (!on_device && sync) HIPCHK(c, hipStreamSynchronize(c->stream));  // host buffers may go away
    *set_id = (int32_t)c->sets.size();
    c->pend.push_back(PrepJob{f32, (int8_t*)frag, (int*)norm, nullptr, n, 0});
    c->pend_set.push_back(*set_id);
    c->sets.push_back(r);
    return MIM_OK;
}

// Preps of the sets created since the last flush: one flags block, one memset, one launch.
static mim_status flush_preps(mim_ctx* c) {
    const int nj = (int)c->pend.size();
    if (nj == 0) return MIM_OK;
    void* flags;
    HIPCHK(c, c->arena.alloc(sizeof(int) * 4 * (size_t)nj, &flags));
    HIPCHK(c, hipMemsetAsync(flags, 0, sizeof(int) * 4 * (size_t)nj, c->stream));
    int tiles = 0;
    for (int j = 0; j < nj; ++j) {
        PrepJob& J = c->pend[j];
        J.flags = static_cast<int*>(flags) + 4 * j;
        J.tile0 = tiles;
        tiles += (J.n + 63) / 64;
        c->sets[c->pend_set[j]].d.flags = J.flags;
    }
    const size_t bytes = sizeof(PrepJob) * nj;
    HIPCHK(c, c->prep_jobs.ensure(bytes));
    char* st = nullptr;
    HIPCHK(c, c->prep_stage.acquire(bytes, &st));
    memcpy(st, c->pend.data(), bytes);
    HIPCHK(c, hipMemcpyAsync(c->prep_jobs.p, st, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, c->prep_stage.release_after(c->stream));
    launch_prep_batch(c->prep_jobs.as<PrepJob>(), nj, tiles, c->stream);
    HIPCHK(c, hipGetLastError());
    c->flushes.push_back({*std::min_element(c->pend_set.begin(), c->pend_set.end()), c->arena.pos()});
    c->pend.clear();
    c->pend_set.clear();
    return MIM_OK;
}

mim_status mim_set_create(mim_ctx* c, const float* desc, const float* kp, int32_t n, int32_t dim,
                          int32_t on_device, int32_t* set_id) {
    if (!c) return MIM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    return set_create_locked(c, desc, kp, n, dim, on_device, set_id);
}

static void sets_truncate_locked(mim_ctx* c, int n_keep);

mim_status mim_sets_create(mim_ctx* c, int32_t count, const float* const* desc, const float* const* kp,
                           const int32_t* rows, int32_t dim, int32_t on_device, int32_t* first_id) {
    if (!c) return MIM_EINVAL;
    if (count < 0 || !first_id || (count > 0 && (!desc || !kp || !rows)))
        return fail(c, MIM_EINVAL, "sets_create: bad arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    const int n0 = (int)c->sets.size();
    const Arena::Mark m0 = c->arena.pos();
    // all or nothing: the sets of this call go, and so does the storage a set that failed part-way
    // took (it is not in `sets` yet, so only the arena mark of the call's start covers it)
    auto undo = [&](mim_status st) {
        if (!on_device) (void)hipStreamSynchronize(c->stream);  // copies already enqueued read the host rows
        if ((int)c->sets.size() > n0) sets_truncate_locked(c, n0);
        c->arena.seek(m0);
        return st;
    };
    for (int i = 0; i < count; ++i) {
        int32_t id = -1;
        const mim_status st = set_create_locked(c, desc[i], kp[i], rows[i], dim, on_device, &id, false);
        if (st != MIM_OK) return undo(st);
    }
    // host rows: every copy enqueued, one wait for all of them (the host buffers may go away after)
    if (!on_device && count > 0) {
        const hipError_t e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) return undo(fail(c, MIM_EDEVICE, "sets_create: hipStreamSynchronize: %s", hipGetErrorString(e)));
    }
    *first_id = n0;
    return MIM_OK;
}

mim_status mim_sets_clear(mim_ctx* c) {
    if (!c) return MIM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    // no host wait: every write into the arena (prep kernels, copies of host rows) is ordered on the
    // ctx stream after the previous batch, whose groups join back into that stream
    c->sets.clear();
    c->pend.clear();
    c->pend_set.clear();
    c->flushes.clear();
    c->arena.rewind();
    ++c->sets_gen;
    return MIM_OK;
}

// drops the sets with ids >= n_keep (0 <= n_keep <= sets.size(), checked by the callers) and
// rewinds the arena to the first dropped set's storage; with the lock held
static void sets_truncate_locked(mim_ctx* c, int n_keep) {
    // the dropped sets' pending preps go; their storage (and prep flags blocks that cover only dropped
    // sets) is reused by later sets, ordered on the ctx stream after the work already enqueued, as
    // for mim_sets_clear
    size_t m = 0;
    for (size_t j = 0; j < c->pend.size(); ++j)
        if (c->pend_set[j] < n_keep) {
            c->pend[m] = c->pend[j];
            c->pend_set[m++] = c->pend_set[j];
        }
    c->pend.resize(m);
    c->pend_set.resize(m);
    Arena::Mark target = c->sets[n_keep].mark;
    for (const auto& f : c->flushes)
        if (f.first < n_keep && target < f.second) target = f.second;  // a kept set's flags lie beyond
    c->flushes.erase(std::remove_if(c->flushes.begin(), c->flushes.end(),
                                    [n_keep](const std::pair<int, Arena::Mark>& f) { return f.first >= n_keep; }),
                     c->flushes.end());
    c->arena.seek(target);
    c->sets.resize(n_keep);
    ++c->sets_gen;
}

mim_status mim_sets_truncate(mim_ctx* c, int32_t n_keep) {
    if (!c) return MIM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (n_keep < 0 || n_keep > (int)c->sets.size())
        return fail(c, MIM_EINVAL, "sets_truncate: %d sets registered, %d to keep", (int)c->sets.size(), n_keep);
    if (n_keep == (int)c->sets.size()) return MIM_OK;
    HIPCHK(c, hipSetDevice(c->device));
    sets_truncate_locked(c, n_keep);
    return MIM_OK;
}

mim_status mim_sets_info(mim_ctx* c, int32_t* n_sets, int64_t* generation) {
    if (!c) return MIM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (n_sets) *n_sets = (int32_t)c->sets.size();
    if (generation) *generation = (int64_t)c->sets_gen;
    return MIM_OK;
}

mim_status mim_set_rows(mim_ctx* c, int32_t set_id, int32_t cap, float* desc, float* kp_xy, int32_t* n_rows) {
    if (!c) return MIM_EINVAL;
    if (!n_rows || cap < 0) return fail(c, MIM_EINVAL, "set_rows: bad arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_id < 0 || set_id >= (int)c->sets.size())
        return fail(c, MIM_EINVAL, "set_rows: set %d not registered (%d sets)", set_id, (int)c->sets.size());
    HIPCHK(c, hipSetDevice(c->device));
    const SetDev& d = c->sets[set_id].d;
    *n_rows = d.n;
    const int m = std::min(d.n, cap);
    if (m > 0 && desc && d.f32)
        HIPCHK(c, hipMemcpyAsync(desc, d.f32, sizeof(float) * kDim * m, hipMemcpyDeviceToHost, c->stream));
    if (m > 0 && kp_xy && d.kp)
        HIPCHK(c, hipMemcpyAsync(kp_xy, d.kp, sizeof(float2) * m, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MIM_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// Problem table + distance work list.  Work items of one problem are placed at block indices
// with equal (index % 8) so they share one XCD's L2 under round-robin dispatch (speed only).
// ---------------------------------------------------------------------------------------------
static mim_status build_tables(mim_ctx* c, const mim_problem* problems, int n, int max_iters) {
    mim_status fs = flush_preps(c);  // the sets' device tiles and flags, before ProbDev copies them
    if (fs != MIM_OK) return fs;
    if (c->knn_grid == 0) {  // resident distance-kernel blocks: CUs x blocks per CU (occupancy query)
        hipDeviceProp_t prop;
        HIPCHK(c, hipGetDeviceProperties(&prop, c->device));
        c->knn_grid = std::max(1, prop.multiProcessorCount * std::max(1, knn_blocks_per_cu()));
    }
    c->h_probs.assign(n, ProbDev{});
    long long part = 0, good = 0, it = 0, units = 0;
    for (int i = 0; i < n; ++i) {
        const int qs = problems[i].query_set, ts = problems[i].train_set;
        if (qs < 0 || qs >= (int)c->sets.size() || ts < 0 || ts >= (int)c->sets.size())
            return fail(c, MIM_EINVAL, "problem %d: bad set id (%d, %d)", i, qs, ts);
        if (c->sets[ts].d.n >= (1 << 18))  // BFMatcher::knnMatchImpl: train rows < 1 << 18 (IMGIDX_SHIFT)
            return fail(c, MIM_EINVAL, "problem %d: train set of %d rows exceeds OpenCV's 2^18 limit", i,
                        c->sets[ts].d.n);
        units += (long long)((c->sets[qs].d.n + kKnnBlockQ - 1) / kKnnBlockQ) * c->sets[ts].d.n_tiles;
    }
    // Balanced distance schedule.  The (problem, query block, train tile) units are cut into equal
    // sub-chunks, every resident block of the single wave of blocks doing the same number of tiles
    // (no tail wave).  A query block cut into k pieces gets k train splits (partial top-2 lists merged
    // by the ratio kernel); a problem's split count is the largest over its query blocks, and the
    // missing splits of the others are empty work items (sentinel lists).
    // L2 locality (MIM_KNN_SUB = s > 0, tiles): with the chunk of a block longer than s, the block
    // does R = ceil(chunk / s) sub-chunks of ~s tiles in rounds, and a problem's train tiles are
    // ordered in segments of <= s tiles (units: problem, segment, query block, tile), so the blocks
    // running at one time on an XCD sweep the same few segments of the same one or two problems.
    // Placement: workgroups are dispatched round-robin over the 8 XCDs (block b on XCD b % 8), and
    // XCD x gets the x-th eighth of the sub-chunks.  MIM_KNN_SUB = 0: segments of <= chunk tiles, one
    // round; < 0: whole query-block sweeps, one round.
    const char* sub_env = getenv("MIM_KNN_SUB");  // read per batch (tests switch it)
    const int sub_target = sub_env ? atoi(sub_env) : kKnnSubTiles;
    // Dynamic mode (whole sweeps pulled from per-XCD lists) when the batch has at least one query-block
    // sweep per resident block: fewer pieces (no early tiles and prologue per split) and a block that
    // starts late under other batches' kernels takes less (measured: C3 isolated kNN 1.39 -> 1.32 ms,
    // pipelined C3 +2.5 %, 32-problem shards +3.8 %, C4 even; profiles/r03_knn_variants.txt, r03ac).
    // Fewer sweeps than blocks (C5's one problem, a scene's small views): the static balanced chunks.
    // MIM_KNN_DYN=0 / 1 forces either.
    long long n_sweeps = 0;
    for (int i = 0; i < n; ++i)
        n_sweeps += (c->sets[problems[i].query_set].d.n + kKnnBlockQ - 1) / kKnnBlockQ;
    const char* dyn_env = getenv("MIM_KNN_DYN");
    const bool dyn = dyn_env ? atoi(dyn_env) != 0 : n_sweeps >= c->knn_grid;
    const long long G = c->knn_grid;
    const long long chunk = std::max<long long>(kKnnMinChunk, (units + G - 1) / G);
    const long long R = (sub_target > 0 && chunk > sub_target) ? (chunk + sub_target - 1) / sub_target : 1;
    const long long sub = std::max<long long>(kKnnMinChunk, (chunk + R - 1) / R);
    const long long NS = std::max<long long>(1, (units + sub - 1) / sub);  // sub-chunks
    const long long per_x = (NS + 7) / 8;
    const int m = (int)std::max<long long>(1, (per_x + R - 1) / R);  // blocks per XCD
    const int nphys = NS < 8 ? (int)NS : 8 * m;
    auto owner = [&](long long j) -> int {
        if (NS < 8) return (int)j;
        const long long x = j / per_x, jj = j % per_x;
        return (int)(8 * (jj % m) + x);
    };
    std::vector<std::vector<KnnWork>> blk(nphys);
    long long pos = 0;
    struct Piece { int b, t0, t1, k, owner; };
    std::vector<Piece> pieces;
    std::vector<int> cnt, last_owner;
    for (int i = 0; i < n; ++i) {
        ProbDev& P = c->h_probs[i];
        P.q = c->sets[problems[i].query_set].d;
        P.t = c->sets[problems[i].train_set].d;
        const int qb = (P.q.n + kKnnBlockQ - 1) / kKnnBlockQ, nt = P.t.n_tiles;
        const int nseg = (sub_target >= 0 && nt > sub) ? (int)((nt + sub - 1) / sub) : 1;
        const int lseg = nseg > 1 ? (nt + nseg - 1) / nseg : nt;
        pieces.clear();
        cnt.assign(qb, 0);
        last_owner.assign(qb, owner(std::min(NS - 1, pos / sub)));
        for (int sg = 0; sg < nseg; ++sg) {
            const int s0 = sg * lseg, s1 = std::min(nt, s0 + lseg);
            for (int b = 0; b < qb && s0 < s1; ++b) {
                const long long u0 = pos, u1 = pos + (s1 - s0);
                for (long long a = u0; a < u1;) {
                    const long long e = std::min(u1, (a / sub + 1) * sub);
                    const int o = owner(std::min(NS - 1, a / sub));
                    pieces.push_back(Piece{b, s0 + (int)(a - u0), s0 + (int)(e - u0), cnt[b]++, o});
                    last_owner[b] = o;
                    a = e;
                }
                pos = u1;
            }
        }
        int nsplit = 1;
        for (int b = 0; b < qb; ++b) nsplit = std::max(nsplit, cnt[b]);
        P.nsplit = nsplit;
        P.q_pad = qb * kKnnBlockQ;
        P.part_off = part;
        part += (long long)nsplit * P.q_pad;
        P.good_off = good;
        good += (std::max(P.q.n, 1) + 31) & ~31;  // 32-aligned: the MFMA bound's point tiles
        P.it_off = it;
        it += std::max(max_iters, 1);
        for (const Piece& pc : pieces) blk[pc.owner].push_back(KnnWork{i, pc.b * kKnnBlockQ, pc.t0, pc.t1, pc.k});
        for (int b = 0; b < qb; ++b)
            for (int k = cnt[b]; k < nsplit; ++k)
                blk[last_owner[b]].push_back(KnnWork{i, b * kKnnBlockQ, nt, nt, k});  // empty split
    }
    std::vector<KnnWork> works;
    std::vector<int> seg;
    int n_launch = nphys;
    if (dyn) {
        // MIM_KNN_DYN=1: whole query-block sweeps (one split per problem), in unit order, as 8 contiguous
        // lists of about equal work (one per XCD); the resident blocks pull them (knn2_i8_kernel).
        // The tail: when the sweeps do not fill the last round of the G resident blocks (a per-GPU shard
        // of 32 C4 problems is 640 sweeps over 512 blocks: two rounds, the second a quarter full), the
        // trailing problems covering that remainder are cut into k train-tile pieces per query block
        // (k ~ G / their sweeps, <= 8), which every list holds after its whole sweeps: the blocks
        // that finish early pull pieces and the kernel ends near sweeps / G rounds instead of the
        // ceiling (each piece repeats the keyed early tiles and the prologue, a few per cent of a
        // sweep; partial top-2 lists merged by the ratio kernel).  Opt-in (MIM_KNN_TAIL=1): it shortens a
        // batch alone (32-problem shard: 0.48 -> 0.45 ms) but costs throughput once batches overlap (the
        // pieces' extra early tiles and merge work: 32-problem shard with 12 in flight 26.8k -> 25.5k
        // problems/s, profiles/r05i_*), and the bench keeps batches in flight.
        works.clear();
        const char* tail_env = getenv("MIM_KNN_TAIL");
        const long long rem = n_sweeps % G;
        int tail_from = n, ksplit = 1;
        if (tail_env && atoi(tail_env) != 0 && n_sweeps > G && rem > 0) {
            long long ts = 0;
            while (tail_from > 0 && ts < rem) ts += c->h_probs[--tail_from].q_pad / kKnnBlockQ;
            ksplit = (int)std::max<long long>(2, std::min<long long>(8, (G + ts / 2) / ts));
        }
        long long total = 0, total_t = 0;
        for (int i = 0; i < n; ++i) {
            ProbDev& P = c->h_probs[i];
            const int qb = P.q_pad / kKnnBlockQ;
            P.nsplit = 1;
            if (i >= tail_from) continue;
            for (int b = 0; b < qb; ++b) works.push_back(KnnWork{i, b * kKnnBlockQ, 0, P.t.n_tiles, 0});
            total += (long long)qb * P.t.n_tiles;
        }
        std::vector<KnnWork> tail;
        for (int i = tail_from; i < n; ++i) {  // pieces in (problem, tile range, query block) order
            ProbDev& P = c->h_probs[i];
            const int qb = P.q_pad / kKnnBlockQ, nt = P.t.n_tiles, k = std::min(ksplit, std::max(nt, 1));
            P.nsplit = k;
            for (int j = 0; j < k; ++j)
                for (int b = 0; b < qb; ++b) tail.push_back(KnnWork{i, b * kKnnBlockQ, j * nt / k, (j + 1) * nt / k, j});
            total_t += (long long)qb * nt;
        }
        part = 0;
        for (int i = 0; i < n; ++i) {
            c->h_probs[i].part_off = part;
            part += (long long)c->h_probs[i].nsplit * c->h_probs[i].q_pad;
        }
        // 8 lists, each [its eighth of the whole sweeps | its eighth of the pieces], equal work per part
        auto cuts = [&](const std::vector<KnnWork>& v, long long tot) {
            std::vector<int> cut(9, (int)v.size());
            cut[0] = 0;
            long long acc = 0;
            int x = 1;
            for (size_t k = 0; k < v.size() && x < 8; ++k) {
                acc += v[k].tile1 - v[k].tile0;
                while (x < 8 && acc * 8 >= tot * x) cut[x++] = (int)k + 1;
            }
            return cut;
        };
        const std::vector<int> cw = cuts(works, total), ct = cuts(tail, total_t);
        std::vector<KnnWork> all;
        all.reserve(works.size() + tail.size());
        seg.assign(9, 0);
        for (int x = 0; x < 8; ++x) {
            seg[x] = (int)all.size();
            all.insert(all.end(), works.begin() + cw[x], works.begin() + cw[x + 1]);
            all.insert(all.end(), tail.begin() + ct[x], tail.begin() + ct[x + 1]);
        }
        seg[8] = (int)all.size();
        works.swap(all);
        n_launch = (int)std::min<long long>(G, std::max<size_t>(works.size(), 8));
        n_launch = std::max(8, n_launch / 8 * 8);
    } else {
        seg.assign(nphys + 1, 0);
        for (int b = 0; b < nphys; ++b) {
            seg[b] = (int)works.size();
            works.insert(works.end(), blk[b].begin(), blk[b].end());
        }
        seg[nphys] = (int)works.size();
    }
    HIPCHK(c, c->probs.ensure(sizeof(ProbDev) * std::max(n, 1)));
    HIPCHK(c, c->works.ensure(sizeof(KnnWork) * std::max<size_t>(works.size(), 1) + sizeof(int) * seg.size()));
    HIPCHK(c, c->parts.ensure(sizeof(Top2) * std::max<long long>(part, 1)));
    HIPCHK(c, c->good_q.ensure(sizeof(int32_t) * good));
    HIPCHK(c, c->good_t.ensure(sizeof(int32_t) * good));
    HIPCHK(c, c->pts.ensure(sizeof(float4) * good));
    HIPCHK(c, c->n_good.ensure(sizeof(int) * std::max(n, 1)));
    HIPCHK(c, c->masks.ensure(good));
    // the device tables are rewritten in stream order (after the previous batch's kernels)
    const size_t pb = sizeof(ProbDev) * n, wb = sizeof(KnnWork) * works.size(), sb = sizeof(int) * seg.size();
    char* st = nullptr;
    HIPCHK(c, c->stage.acquire(pb + wb + sb, &st));
    memcpy(st, c->h_probs.data(), pb);
    memcpy(st + pb, works.data(), wb);
    memcpy(st + pb + wb, seg.data(), sb);
    HIPCHK(c, hipMemcpyAsync(c->probs.p, st, pb, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->works.p, st + pb, wb + sb, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, c->stage.release_after(c->stream));
    c->h_good_off.resize(n);
    for (int i = 0; i < n; ++i) c->h_good_off[i] = c->h_probs[i].good_off;
    c->last_n = n;
    c->n_works = (int)works.size();
    c->n_knn_blocks = n_launch;
    c->knn_dyn = dyn;
    if (dyn) HIPCHK(c, c->knn_ctr.ensure(8 * sizeof(int)));
    return MIM_OK;
}

// Kernel timing: an event after every launch on the stream it ran on; a kernel's time is the gap to
// the previous event of the same stream (with pipelined groups these are the kernels' own spans,
// overlap with other groups included).
static void ev_mark(mim_ctx* c, const char* name) {
    if (!c->timing) return;
    hipEvent_t e;
    if (!c->ev_pool.empty()) {
        e = c->ev_pool.back();
        c->ev_pool.pop_back();
    } else if (hipEventCreate(&e) != hipSuccess) {
        return;
    }
    (void)hipEventRecord(e, c->cur);
    if (!strcmp(name, "begin")) ++c->ev_seq;
    c->evs.push_back({name, c->cur, e, c->ev_seq});
}

static void ev_collect(mim_ctx* c) {
    if (c->evs.empty()) return;
    for (auto& e : c->evs) (void)hipEventSynchronize(e.e);
    c->last_ms.clear();
    // kernel time summed over every batch since the last collection
    std::map<hipStream_t, const mim_ctx::Ev*> prev;
    for (auto& e : c->evs) {
        auto it = prev.find(e.s);
        if (it != prev.end() && it->second->seq == e.seq) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, it->second->e, e.e);
            c->last_ms[e.name] += ms;
        }
        prev[e.s] = &e;
    }
    for (auto& e : c->evs) c->ev_pool.push_back(e.e);
    c->evs.clear();
}

static void knn_launch(mim_ctx* c) {
    const KnnWork* w = c->works.as<KnnWork>();
    launch_knn(c->probs.as<ProbDev>(), w, c->n_works, reinterpret_cast<const int*>(w + c->n_works), c->n_knn_blocks,
               c->parts.as<Top2>(), c->knn_dyn ? c->knn_ctr.as<int>() : nullptr, c->cur);
}

// distance + ratio kernels of the batch's problems
static mim_status knn_ratio_locked(mim_ctx* c, int n, float ratio, bool emit_knn) {
    c->cur = c->stream;
    ev_mark(c, "begin");
    knn_launch(c);
    HIPCHK(c, hipGetLastError());
    ev_mark(c, "knn");
    launch_ratio(c->probs.as<ProbDev>(), n, c->parts.as<Top2>(), ratio, c->good_q.as<int32_t>(), c->good_t.as<int32_t>(),
                 c->pts.as<float4>(), c->n_good.as<int>(), emit_knn ? c->knn_idx.as<int32_t>() : nullptr,
                 emit_knn ? c->knn_dist.as<float>() : nullptr, c->cur);
    HIPCHK(c, hipGetLastError());
    ev_mark(c, "ratio");
    return MIM_OK;
}

extern "C" {

mim_status mim_knn2_l2(mim_ctx* c, const float* q, int32_t nq, const float* t, int32_t nt, int32_t dim,
                       int32_t* idx, float* dist) {
    if (!c) return MIM_EINVAL;
    if (nq < 0 || nt < 0 || (nq > 0 && (!q || !idx || !dist)) || (nt > 0 && !t))
        return fail(c, MIM_EINVAL, "knn2_l2: bad arguments");
    if (dim != kDim) return fail(c, MIM_EINVAL, "knn2_l2: dim must be %d", kDim);
    if (nq == 0) return MIM_OK;  // knnMatch on an empty query returns no rows
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    // private sets appended after the user's sets, removed afterwards
    const size_t base = c->sets.size();
    std::vector<float> kp0((size_t)std::max(nq, nt) * 2, 0.f);
    int32_t sq, st;
    mim_status s = set_create_locked(c, q, kp0.data(), nq, dim, 0, &sq);
    if (s != MIM_OK) return s;
    s = set_create_locked(c, t ? t : kp0.data(), kp0.data(), nt, dim, 0, &st);
    if (s != MIM_OK) return s;
    mim_problem pr{sq, st};
    s = build_tables(c, &pr, 1, 1);
    if (s != MIM_OK) return s;
    HIPCHK(c, c->knn_idx.ensure(sizeof(int32_t) * 2 * nq));
    HIPCHK(c, c->knn_dist.ensure(sizeof(float) * 2 * nq));
    s = knn_ratio_locked(c, 1, 0.9f, true);
    if (s != MIM_OK) return s;
    HIPCHK(c, hipMemcpyAsync(idx, c->knn_idx.p, sizeof(int32_t) * 2 * nq, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(dist, c->knn_dist.p, sizeof(float) * 2 * nq, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    ev_collect(c);
    c->sets.resize(base);  // arena space is reclaimed at the next mim_sets_clear
    c->last_n = 0;         // no RANSAC records: the previous batch's are invalidated (mim.h)
    c->last_gen = -1;
    c->last_fh = false;
    return MIM_OK;
}

mim_status mim_ratio_filter(mim_ctx* c, const int32_t* idx, const float* dist, int32_t nq, float ratio,
                            int32_t* q_out, int32_t* t_out, int32_t* n_good) {
    if (!c) return MIM_EINVAL;
    if (nq < 0 || !n_good || (nq > 0 && (!idx || !dist))) return fail(c, MIM_EINVAL, "ratio_filter: bad arguments");
    *n_good = 0;
    if (nq == 0) return MIM_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // knnMatch rows -> one train split of Top2 partials, then the device ratio/compaction kernel
    int max_t = 0;
    std::vector<Top2> parts(nq);
    for (int i = 0; i < nq; ++i) {
        const int a = idx[2 * i], b = idx[2 * i + 1];
        parts[i] = Top2{a < 0 ? FLT_MAX : dist[2 * i], a < 0 ? INT_MAX : a, b < 0 ? FLT_MAX : dist[2 * i + 1],
                        b < 0 ? INT_MAX : b};
        max_t = std::max(max_t, std::max(a, b));
    }
    const int q_pad = (nq + kKnnBlockQ - 1) / kKnnBlockQ * kKnnBlockQ;
    const size_t nkp = (size_t)std::max(nq, max_t + 1);
    HIPCHK(c, c->parts.ensure(sizeof(Top2) * q_pad));
    HIPCHK(c, c->rws.scratch.ensure(sizeof(float2) * nkp));
    HIPCHK(c, c->good_q.ensure(sizeof(int32_t) * nq));
    HIPCHK(c, c->good_t.ensure(sizeof(int32_t) * nq));
    HIPCHK(c, c->pts.ensure(sizeof(float4) * nq));
    HIPCHK(c, c->n_good.ensure(sizeof(int)));
    HIPCHK(c, c->probs.ensure(sizeof(ProbDev)));
    HIPCHK(c, hipMemsetAsync(c->rws.scratch.p, 0, sizeof(float2) * nkp, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->parts.p, parts.data(), sizeof(Top2) * nq, hipMemcpyHostToDevice, c->stream));
    ProbDev P{};
    P.q.n = nq;
    P.q.kp = c->rws.scratch.as<float2>();
    P.t.kp = c->rws.scratch.as<float2>();
    P.nsplit = 1;
    P.q_pad = q_pad;
    HIPCHK(c, hipMemcpyAsync(c->probs.p, &P, sizeof P, hipMemcpyHostToDevice, c->stream));
    launch_ratio(c->probs.as<ProbDev>(), 1, c->parts.as<Top2>(), ratio, c->good_q.as<int32_t>(),
                 c->good_t.as<int32_t>(), c->pts.as<float4>(), c->n_good.as<int>(), nullptr, nullptr, c->stream);
    HIPCHK(c, hipGetLastError());
    int ng = 0;
    HIPCHK(c, hipMemcpyAsync(&ng, c->n_good.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (ng > 0) {
        if (q_out) HIPCHK(c, hipMemcpy(q_out, c->good_q.p, sizeof(int32_t) * ng, hipMemcpyDeviceToHost));
        if (t_out) HIPCHK(c, hipMemcpy(t_out, c->good_t.p, sizeof(int32_t) * ng, hipMemcpyDeviceToHost));
    }
    *n_good = ng;
    c->last_n = 0;
    c->last_gen = -1;
    c->last_fh = false;
    return MIM_OK;
}

mim_status mim_knn2_sets_dev(mim_ctx* c, int32_t query_set, int32_t train_set, int32_t* idx_dev,
                             float* dist_dev) {
    if (!c || !idx_dev || !dist_dev) return MIM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    mim_problem pr{query_set, train_set};
    mim_status s = build_tables(c, &pr, 1, 1);
    if (s != MIM_OK) return s;
    c->cur = c->stream;
    ev_mark(c, "begin");
    knn_launch(c);
    HIPCHK(c, hipGetLastError());
    ev_mark(c, "knn");
    launch_knn_emit(c->probs.as<ProbDev>(), c->h_probs[0].q.n, c->parts.as<Top2>(), idx_dev, dist_dev, c->stream);
    HIPCHK(c, hipGetLastError());
    ev_mark(c, "ratio");
    c->last_n = 0;  // no RANSAC records (mim.h)
    c->last_gen = -1;
    c->last_fh = false;
    return MIM_OK;
}

void mim_default_box_params(mim_box_params* p) {
    const mim::BoxParams d;
    p->cluster_distance = d.cluster_distance;
    p->min_points_per_cluster = d.min_points_per_cluster;
    p->box_merge_distance = d.box_merge_distance;
    p->min_box_area = d.min_box_area;
    p->dynamic_margin = d.dynamic_margin;
}

mim_status mim_detect_boxes(const float* pts_xy, int32_t n, const mim_box_params* bp, mim_rect* boxes, int32_t cap,
                            int32_t* n_boxes) {
    if (n < 0 || (n > 0 && !pts_xy) || !n_boxes || cap < 0 || (cap > 0 && !boxes)) return MIM_EINVAL;
    mim::BoxParams p;
    if (bp) {
        p.cluster_distance = bp->cluster_distance;
        p.min_points_per_cluster = bp->min_points_per_cluster;
        p.box_merge_distance = bp->box_merge_distance;
        p.min_box_area = bp->min_box_area;
        p.dynamic_margin = bp->dynamic_margin;
    }
    try {
        std::vector<mim::Point2f> pts(n);
        for (int32_t i = 0; i < n; ++i) pts[i] = {pts_xy[2 * i], pts_xy[2 * i + 1]};
        mim::Detections dets;
        mim::boxes_for_model(pts, "", dets, p);
        *n_boxes = (int32_t)dets.size();
        for (int32_t i = 0; i < std::min(cap, *n_boxes); ++i)
            boxes[i] = mim_rect{dets[i].first.x, dets[i].first.y, dets[i].first.width, dets[i].first.height};
    } catch (const std::bad_alloc&) {
        return MIM_ENOMEM;
    }
    return MIM_OK;
}

mim_status mim_sift_detect_compute(mim_ctx* c, const uint8_t* gray, int32_t rows, int32_t cols, int64_t step,
                                   const uint8_t* mask, int64_t mask_step, int32_t max_kp, mim_keypoint* kps,
                                   float* desc, int32_t* n_kp) {
    if (!c) return MIM_EINVAL;
    if (!gray || !n_kp || rows <= 0 || cols <= 0 || step < cols || max_kp < 0 || (max_kp > 0 && (!kps || !desc)) ||
        (mask && mask_step < cols))
        return fail(c, MIM_EINVAL, "sift_detect_compute: bad arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->sift) c->sift = mim::sift_ws_create();
    int n = 0;
    const int r = mim::sift_detect_compute(c->sift, c->stream, gray, rows, cols, step, mask, mask_step, max_kp, kps,
                                           desc, &n, c->err);
    *n_kp = n;
    if (r == -1) return MIM_EDEVICE;
    if (r == -2) return MIM_ERANGE;
    if (r == -4) return MIM_ELIMIT;
    return MIM_OK;
}

mim_status mim_sift_detect_compute_scales(mim_ctx* c, const uint8_t* gray, int32_t rows, int32_t cols, int64_t step,
                                          int32_t n_scales, const float* scales, int32_t max_kp, mim_keypoint* kps,
                                          float* desc, int32_t* n_kp) {
    if (!c) return MIM_EINVAL;
    if (!gray || !n_kp || !scales || n_scales <= 0 || n_scales > 64 || rows <= 0 || cols <= 0 || step < cols ||
        max_kp < 0 || (max_kp > 0 && (!kps || !desc)))
        return fail(c, MIM_EINVAL, "sift_detect_compute_scales: bad arguments");
    for (int i = 0; i < n_scales; ++i)
        if (!(scales[i] > 0)) return fail(c, MIM_EINVAL, "sift_detect_compute_scales: scale %d is not > 0", i);
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    std::vector<int> n(n_scales, 0);
    const int r = mim::sift_detect_compute_scales(c->sift_scales, c->stream, gray, rows, cols, step, n_scales, scales,
                                                  max_kp, kps, desc, n.data(), c->err);
    for (int i = 0; i < n_scales; ++i) n_kp[i] = n[i];
    if (r == -1) return MIM_EDEVICE;
    if (r == -2) return MIM_ERANGE;
    if (r == -3) return MIM_EINVAL;
    if (r == -4) return MIM_ELIMIT;
    return MIM_OK;
}

// mim_sift_scales_sets' registration of the scales as sets (lock held); total = keypoints of all scales
static mim_status scales_sets_register(mim_ctx* c, const mim::SiftDevOut* out, int n_scales, int32_t* set_ids,
                                       int32_t* n_kp, long long& total) {
    std::vector<float*> ddesc(n_scales, nullptr);
    std::vector<float2*> dkp(n_scales, nullptr);
    for (int i = 0; i < n_scales; ++i) {
        const int n = out[i].n;
        n_kp[i] = n;
        total += n;
        SetRec rec{};
        rec.mark = c->arena.pos();
        rec.d.n = n;
        rec.d.n_tiles = (n + 63) / 64;
        const size_t tiles = (size_t)std::max(rec.d.n_tiles, 1);
        void *frag, *norm, *df = nullptr, *dk = nullptr;
        HIPCHK(c, c->arena.alloc(tiles * kTileBytes, &frag));
        HIPCHK(c, c->arena.alloc(tiles * kNormWords * sizeof(int), &norm));
        if (n > 0) {
            HIPCHK(c, c->arena.alloc((size_t)n * kDim * sizeof(float), &df));
            HIPCHK(c, c->arena.alloc((size_t)n * 2 * sizeof(float), &dk));
        }
        ddesc[i] = (float*)df;
        dkp[i] = (float2*)dk;
        rec.d.frag = (const int8_t*)frag;
        rec.d.norm = (const int*)norm;
        rec.d.f32 = (const float*)df;
        rec.d.kp = (const float2*)dk;
        rec.d.flags = nullptr;
        set_ids[i] = (int32_t)c->sets.size();
        c->pend.push_back(PrepJob{(const float*)df, (int8_t*)frag, (int*)norm, nullptr, n, 0});
        c->pend_set.push_back(set_ids[i]);
        c->sets.push_back(rec);
    }
    // every scale's rows and KeyPoint::pt (the first two floats of each mim_keypoint) in one launch
    if (mim::sift_copy_sets(out, n_scales, ddesc.data(), dkp.data(), c->stream) != 0)
        return fail(c, MIM_EDEVICE, "sift_scales_sets: set copy launch failed");
    return MIM_OK;
}

mim_status mim_sift_scales_sets(mim_ctx* c, const uint8_t* gray, int32_t rows, int32_t cols, int64_t step,
                                int32_t n_scales, const float* scales, int32_t* set_ids, int32_t* n_kp, int32_t max_kp,
                                mim_keypoint* kps) {
    if (!c) return MIM_EINVAL;
    if (!gray || !set_ids || !n_kp || !scales || n_scales <= 0 || n_scales > 8 || rows <= 0 || cols <= 0 ||
        step < cols || max_kp < 0 || (max_kp > 0 && !kps))
        return fail(c, MIM_EINVAL, "sift_scales_sets: bad arguments");
    for (int i = 0; i < n_scales; ++i)
        if (!(scales[i] > 0)) return fail(c, MIM_EINVAL, "sift_scales_sets: scale %d is not > 0", i);
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    std::vector<mim::SiftDevOut> out(n_scales);
    const int r = mim::sift_scales_device(c->sift_scales, c->stream, gray, rows, cols, step, n_scales, scales, out.data(),
                                          c->err);
    if (r == -1) return MIM_EDEVICE;
    if (r == -3) return MIM_EINVAL;
    if (r == -4) return MIM_ELIMIT;
    if (r != 0) return MIM_ERANGE;
    // each scale's rows and keypoint positions copied on the device into the set arena (the SIFT
    // workspaces are overwritten by the next SIFT call), the set registered as by mim_set_create; a
    // failure part-way (arena allocation, copy) drops the scales registered so far, so the ctx is left
    // as before the call
    const int n0 = (int)c->sets.size();
    const Arena::Mark mark0 = c->arena.pos();
    long long total = 0;
    const mim_status rs = scales_sets_register(c, out.data(), n_scales, set_ids, n_kp, total);
    if (rs != MIM_OK) {
        if ((int)c->sets.size() > n0)
            sets_truncate_locked(c, n0);
        else
            c->arena.seek(mark0);
        return rs;
    }
    if (kps && max_kp > 0) {  // the keypoints on the host too, concatenated in scale order
        long long used = 0;
        for (int i = 0; i < n_scales && used < max_kp; ++i) {
            const long long m = std::min<long long>(out[i].n, max_kp - used);
            if (m > 0)
                HIPCHK(c, hipMemcpyAsync(kps + used, out[i].kp, sizeof(mim_keypoint) * m, hipMemcpyDeviceToHost, c->stream));
            used += m;
        }
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    if (kps && total > max_kp) return fail(c, MIM_ERANGE, "sift_scales_sets: %lld keypoints, buffer holds %d", total, max_kp);
    return MIM_OK;
}

mim_status mim_resize_linear_u8(mim_ctx* c, const uint8_t* src, int32_t rows, int32_t cols, int64_t step,
                                uint8_t* dst, int32_t drows, int32_t dcols, double fx, double fy) {
    if (!c) return MIM_EINVAL;
    if (!src || !dst || rows <= 0 || cols <= 0 || step < cols || drows <= 0 || dcols <= 0 || fx < 0 || fy < 0 ||
        (fx > 0) != (fy > 0))
        return fail(c, MIM_EINVAL, "resize_linear_u8: bad arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->sift) c->sift = mim::sift_ws_create();
    if (mim::sift_resize_u8(c->sift, c->stream, src, rows, cols, step, dst, drows, dcols, fx, fy, c->err) != 0)
        return MIM_EDEVICE;
    return MIM_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// RANSAC: RNG stream, workspace, batch entry points
// ---------------------------------------------------------------------------------------------
static void mark_cb(void* vc, const char* name, hipStream_t st) {
    mim_ctx* c = (mim_ctx*)vc;
    const hipStream_t keep = c->cur;
    c->cur = st;
    ev_mark(c, name);
    c->cur = keep;
}

// cv::RNG((uint64)-1).next() stream (core/include/opencv2/core/operations.hpp).  Every
// findHomography call re-seeds, so one stream serves all problems of a ctx.  Generated on the
// device: the MWC state s' = (u32)s * a + (s >> 32) (a = 4164903690) is, from the second state on,
// the Lehmer sequence s_{n+1} = a * s_n mod (a * 2^32 - 1), so each 4096-draw segment starts from
// a * ... jump-ahead computed here in 128-bit arithmetic and the device expands the segments.
constexpr long long kStreamMin = 1LL << 23, kStreamCap = 1LL << 30;  // draws (the cap: 4 GiB)
constexpr int kStreamSeg = 4096;

static inline unsigned long long mwc_next(unsigned long long s) {
    return (unsigned long long)(uint32_t)s * 4164903690ULL + (s >> 32);
}
static inline unsigned long long mulmod(unsigned long long x, unsigned long long y, unsigned long long m) {
    return (unsigned long long)(((unsigned __int128)x * y) % m);
}

static mim_status ensure_stream(mim_ctx* c, long long need) {
    if (c->rws.stream_len >= need) return MIM_OK;
    long long len = std::max(need, kStreamMin);
    if (c->stream_draws && c->rws.stream_len == 0) len = c->stream_draws;  // test knob: first stream only
    if (len > kStreamCap) return fail(c, MIM_ERANGE, "RNG stream of %lld draws exceeds the 2^30 cap", len);
    len = (len + kStreamSeg - 1) / kStreamSeg * kStreamSeg;
    const int n_seg = (int)(len / kStreamSeg);
    const unsigned long long a = 4164903690ULL, m = a * 4294967296ULL - 1;
    std::vector<unsigned long long> seg((size_t)n_seg);
    const unsigned long long s0 = mwc_next(~0ULL), s1 = mwc_next(s0);
    // a^(kStreamSeg) and a^(kStreamSeg - 1) mod m
    unsigned long long J = 1, Jm1 = 1;
    for (int k = 0; k < kStreamSeg; ++k) {
        Jm1 = J;
        J = mulmod(J, a, m);
    }
    seg[0] = s0;
    if (n_seg > 1) seg[1] = mulmod(Jm1, s1, m);  // s_{4096} = a^4095 s_1
    for (int i = 2; i < n_seg; ++i) seg[(size_t)i] = mulmod(seg[(size_t)i - 1], J, m);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // 64 zero draws of padding: the draw prefetches of resolve_at may read up to 7 past the end
    HIPCHK(c, c->rws.stream.ensure(sizeof(uint32_t) * (len + 64)));
    DevBuf segs;
    HIPCHK(c, segs.ensure(sizeof(unsigned long long) * n_seg));
    HIPCHK(c, hipMemcpy(segs.p, seg.data(), sizeof(unsigned long long) * n_seg, hipMemcpyHostToDevice));
    launch_rng_stream(segs.as<unsigned long long>(), c->rws.stream.as<uint32_t>(), len, kStreamSeg, n_seg,
                      c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemsetAsync((uint32_t*)c->rws.stream.p + len, 0, sizeof(uint32_t) * 64, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    segs.release();
    c->rws.stream_len = len;
    return MIM_OK;
}

// Longer stream after a batch ran out (status MIM_STREAM_SHORT): x8, up to the cap.
static mim_status grow_stream(mim_ctx* c) {
    if (c->rws.stream_len >= kStreamCap)
        return fail(c, MIM_ERANGE, "RANSAC consumed the whole RNG stream (%lld draws, the cap)", c->rws.stream_len);
    return ensure_stream(c, std::min(kStreamCap, c->rws.stream_len * 8));
}

// Buffers and parameters of one RANSAC batch over n problems (allocation only: call before any
// launch of the batch, a reallocation synchronises the device).
static mim_status ransac_prepare(mim_ctx* c, int n, const mim_params* prm, RansacBufs& b, RansacParams& rp,
                                 long long& flag_per) {
    const int max_iters = std::max(prm->max_iters, 1);
    mim_status s = ensure_stream(c, (long long)max_iters * 64 + 40000 * 4);
    if (s != MIM_OK) return s;
    long long it_total = 0, good_total = 0;
    for (int i = 0; i < n; ++i) {
        it_total = std::max(it_total, c->h_probs[i].it_off + max_iters);
        good_total = std::max(good_total, c->h_probs[i].good_off + std::max(c->h_probs[i].q.n, 1));
    }
    HIPCHK(c, c->rws.state.ensure(sizeof(RansacState) * std::max(n, 1)));
    HIPCHK(c, c->rws.samples.ensure(sizeof(int4) * it_total));
    HIPCHK(c, c->rws.hyp.ensure(sizeof(float) * 8 * it_total));
    HIPCHK(c, c->rws.counts.ensure(sizeof(int) * it_total));
    HIPCHK(c, c->rws.bounds.ensure(sizeof(int2) * it_total));
    // attempt-outcome windows: largest chunk x 28 draws per problem, 64-byte granular per problem
    const long long chunk_max = std::min<long long>(max_iters, 1 << 18);
    flag_per = (chunk_max * 28 + 4096 + 63) & ~63LL;
    const long long flag_cap = (long long)std::max(n, 1) * flag_per;
    HIPCHK(c, c->rws.flags.ensure((size_t)flag_cap));
    HIPCHK(c, c->rws.irr_bits.ensure((size_t)flag_cap / 8));
    const int irr_blocks = (int)((flag_per + kIrrBlock - 1) / kIrrBlock);
    HIPCHK(c, c->rws.irr.ensure(sizeof(int) * (size_t)std::max(n, 1) * irr_blocks * kIrrCap));
    HIPCHK(c, c->rws.irr_cnt.ensure(sizeof(int) * (size_t)std::max(n, 1) * irr_blocks));
    HIPCHK(c, c->rws.pass_bits.ensure((size_t)flag_cap / 8));
    // deferred-attempt lists of the check rounds: a chain holds at most ~window / 4 attempts
    const int def_rounds = (int)((flag_per / 4 + 2 * kRansacDefRoundAttempts) / kRansacDefRoundAttempts);
    HIPCHK(c, c->rws.defer.ensure(sizeof(int2) * kRansacDefSlots * (size_t)std::max(n, 1) * def_rounds));
    HIPCHK(c, c->rws.defer_n.ensure(sizeof(int) * (size_t)std::max(n, 1) * def_rounds));
    HIPCHK(c, c->rws.chains.ensure(ransac_chain_bytes() * (size_t)std::max(n, 1)));
    HIPCHK(c, c->rws.best_h.ensure(sizeof(double) * 9 * std::max(n, 1)));
    // two candidate lists per problem: chunk 1's (kept when its exact pass is deferred) and chunk 2's
    const size_t cap = (size_t)std::max(n, 1) * 2 * kCandPerProblem;
    HIPCHK(c, c->rws.cand.ensure(sizeof(int) * cap));
    HIPCHK(c, c->rws.ncand.ensure(sizeof(int) * 2 * std::max(n, 1)));
    HIPCHK(c, c->rws.cex.ensure(sizeof(int) * cap));
    HIPCHK(c, c->rws.cH.ensure(sizeof(double) * 9 * cap));
    HIPCHK(c, c->rws.decided.ensure(sizeof(int) * cap));
    HIPCHK(c, c->rws.inl.ensure(sizeof(float4) * good_total));
    HIPCHK(c, c->rws.tiles.ensure(sizeof(uint4) * 128 * ((good_total + 31) / 32)));
    HIPCHK(c, c->rws.err.ensure(sizeof(int) * 4));
    HIPCHK(c, c->results.ensure(sizeof(mim_result) * std::max(n, 1)));
    HIPCHK(c, c->masks.ensure(good_total));
    HIPCHK(c, hipMemsetAsync(c->rws.err.p, 0, sizeof(int) * 4, c->stream));
    b = RansacBufs{};
    b.state = c->rws.state.as<RansacState>();
    b.samples = c->rws.samples.as<int4>();
    b.hyp = c->rws.hyp.as<float>();
    b.counts = c->rws.counts.as<int>();
    b.bounds = c->rws.bounds.as<int2>();
    b.flags = c->rws.flags.as<uint8_t>();
    b.irr_bits = c->rws.irr_bits.as<uint8_t>();
    b.best_h = c->rws.best_h.as<double>();
    b.cand = c->rws.cand.as<int>();
    b.ncand = c->rws.ncand.as<int>();
    b.cex = c->rws.cex.as<int>();
    b.cH = c->rws.cH.as<double>();
    b.decided = c->rws.decided.as<int>();
    b.flag_cap = flag_cap;
    b.irr = c->rws.irr.as<int>();
    b.irr_cnt = c->rws.irr_cnt.as<int>();
    b.pass_bits = c->rws.pass_bits.as<uint32_t>();
    b.defer = c->rws.defer.as<int2>();
    b.defer_n = c->rws.defer_n.as<int>();
    // MIM_CHECK_DEFER=0: every deferred attempt decided inside the check kernel (test knob)
    const char* cde = getenv("MIM_CHECK_DEFER");
    b.def_rounds = (cde && cde[0] == '0') ? 0 : def_rounds;
    b.irr_blocks = irr_blocks;
    b.chains = c->rws.chains.p;
    b.stream = c->rws.stream.as<uint32_t>();
    b.stream_len = c->rws.stream_len;
    b.inl = c->rws.inl.as<float4>();
    b.tiles = c->rws.tiles.as<uint4>();
    b.err = c->rws.err.as<int>();
    if (c->samp_on < 0) {
        const char* e = getenv("MIM_SAMPLER_STREAM");
        c->samp_on = (e && e[0] == '0') ? 0 : 1;
    }
    if (c->samp_on && !c->samp) {
        HIPCHK(c, hipStreamCreateWithFlags(&c->samp, hipStreamNonBlocking));
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_samp_fork, hipEventDisableTiming));
        for (auto& e : c->ev_samp) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    b.s2 = c->samp_on ? c->samp : nullptr;
    b.ev_fork = c->ev_samp_fork;
    b.ev_samp[0] = c->ev_samp[0];
    b.ev_samp[1] = c->ev_samp[1];
    rp = RansacParams{};
    rp.thresh = prm->ransac_thresh > 0 ? prm->ransac_thresh : 3.0;  // findHomography: thresh <= 0 -> 3
    rp.conf = prm->confidence;
    rp.max_iters = max_iters;
    rp.ratio = prm->ratio;
    rp.min_good = prm->min_good;
    rp.min_inliers = prm->min_inliers;
    rp.det_lo = prm->det_lo;
    rp.det_hi = prm->det_hi;
    rp.cand_cap = c->cand_cap;
    rp.rep_cap = c->rep_cap;
    return MIM_OK;
}

// RANSAC kernels for problems [p0, p0 + np) on c->cur: per-problem buffers are offset to the range
// (problem-indexed ones by p0, the iteration/point-indexed ones use the global it_off/good_off).
static mim_status ransac_enqueue_range(mim_ctx* c, int p0, int np, const RansacBufs& b, const RansacParams& rp,
                                       long long flag_per, int raw) {
    RansacBufs g = b;
    g.state += p0;
    g.flags += (long long)p0 * flag_per;
    g.irr_bits += (long long)p0 * flag_per / 8;
    g.flag_cap = (long long)np * flag_per;
    g.irr += (long long)p0 * b.irr_blocks * kIrrCap;
    g.irr_cnt += (long long)p0 * b.irr_blocks;
    g.pass_bits += (long long)p0 * flag_per / 32;
    g.defer += (long long)p0 * b.def_rounds * kRansacDefSlots;
    g.defer_n += (long long)p0 * b.def_rounds;
    g.chains = static_cast<char*>(b.chains) + (size_t)p0 * ransac_chain_bytes();
    g.best_h += 9LL * p0;
    g.cand += (long long)p0 * 2 * kCandPerProblem;
    g.ncand += 2 * p0;
    g.cex += (long long)p0 * 2 * kCandPerProblem;
    g.cH += 9LL * p0 * 2 * kCandPerProblem;
    g.decided += (long long)p0 * 2 * kCandPerProblem;
    ransac_enqueue(rp, np, c->probs.as<ProbDev>() + p0, c->pts.as<float4>(), c->n_good.as<int>() + p0, g,
                   c->masks.as<uint8_t>(), c->results.as<mim_result>() + p0, raw, c->cur, mark_cb, c, c->exact_all);
    HIPCHK(c, hipGetLastError());
    return MIM_OK;
}

static mim_status ransac_locked(mim_ctx* c, int n, const mim_params* prm, int raw) {
    RansacBufs b;
    RansacParams rp;
    long long flag_per = 0;
    mim_status s = ransac_prepare(c, n, prm, b, rp, flag_per);
    if (s != MIM_OK) return s;
    c->cur = c->stream;
    return ransac_enqueue_range(c, 0, n, b, rp, flag_per, raw);
}

static mim_status check_params(mim_ctx* c, const mim_params* p) {
    if (!p) return fail(c, MIM_EINVAL, "null params");
    if (!(p->confidence > 0 && p->confidence < 1)) return fail(c, MIM_EINVAL, "confidence must be in (0,1)");
    if (p->max_iters > 10000000) return fail(c, MIM_EINVAL, "max_iters too large");
    return MIM_OK;
}

extern "C" {

}  // extern "C"

static mim_status batch_run_locked(mim_ctx* c, const mim_problem* problems, int32_t n, const mim_params* params) {
    HIPCHK(c, hipSetDevice(c->device));
    c->last_problems.assign(problems, problems + n);
    c->last_params = *params;
    c->last_gen = c->sets_gen;
    c->last_fh = false;
    if (n == 0) { c->last_n = 0; return MIM_OK; }
    mim_status s = build_tables(c, problems, n, std::max(params->max_iters, 1));
    if (s != MIM_OK) return s;
    RansacBufs b;
    RansacParams rp;
    long long flag_per = 0;
    s = ransac_prepare(c, n, params, b, rp, flag_per);
    if (s != MIM_OK) return s;
    s = knn_ratio_locked(c, n, params->ratio, false);
    if (s != MIM_OK) return s;
    return ransac_enqueue_range(c, 0, n, b, rp, flag_per, 0);
}

// Waits for the last batch; if a problem ran out of RNG draws (status MIM_STREAM_SHORT: OpenCV's
// loop consumed more than the stream holds), grows the stream and re-runs the batch, which is
// possible while its sets are intact.  `res` receives the final records.
static mim_status finish_batch_locked(mim_ctx* c, std::vector<mim_result>& res) {
    for (;;) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        ev_collect(c);
        res.resize((size_t)c->last_n);
        if (c->last_n > 0)
            HIPCHK(c, hipMemcpy(res.data(), c->results.p, sizeof(mim_result) * c->last_n, hipMemcpyDeviceToHost));
        bool short_ = false;
        for (const mim_result& r : res) short_ |= r.status == MIM_STREAM_SHORT;
        if (!short_) return MIM_OK;
        if (c->last_gen != c->sets_gen || c->last_problems.size() != res.size())
            return fail(c, MIM_ERANGE, "a problem ran out of RNG draws (%lld) and its sets were cleared: re-run the "
                                       "batch", c->rws.stream_len);
        mim_status s = grow_stream(c);
        if (s != MIM_OK) return s;
        const std::vector<mim_problem> probs = c->last_problems;
        const mim_params prm = c->last_params;
        s = batch_run_locked(c, probs.data(), (int32_t)probs.size(), &prm);
        if (s != MIM_OK) return s;
    }
}

extern "C" {

mim_status mim_batch_run(mim_ctx* c, const mim_problem* problems, int32_t n, const mim_params* params) {
    if (!c) return MIM_EINVAL;
    if (n < 0 || (n > 0 && !problems)) return fail(c, MIM_EINVAL, "batch_run: bad arguments");
    mim_status s = check_params(c, params);
    if (s != MIM_OK) return s;
    std::lock_guard<std::mutex> lk(c->mu);
    return batch_run_locked(c, problems, n, params);
}

mim_status mim_batch_results(mim_ctx* c, mim_result* out) {
    if (!c) return MIM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    std::vector<mim_result> res;
    mim_status s = finish_batch_locked(c, res);
    if (s != MIM_OK) return s;
    if (out && !res.empty()) memcpy(out, res.data(), sizeof(mim_result) * res.size());
    return MIM_OK;
}

const mim_result* mim_batch_results_dev(mim_ctx* c) { return c ? c->results.as<mim_result>() : nullptr; }

mim_status mim_batch_results_copy(mim_ctx* c, void* dst, int32_t dst_on_device) {
    if (!c || !dst) return MIM_EINVAL;
    if (!dst_on_device) return mim_batch_results(c, (mim_result*)dst);
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    if (c->last_n > 0)
        HIPCHK(c, hipMemcpyAsync(dst, c->results.p, sizeof(mim_result) * c->last_n, hipMemcpyDeviceToDevice, c->stream));
    return MIM_OK;
}

mim_status mim_batch_problem_detail(mim_ctx* c, int32_t i, int32_t* q_idx, int32_t* t_idx, uint8_t* mask) {
    if (!c) return MIM_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (i < 0 || i >= c->last_n) return fail(c, MIM_EINVAL, "problem %d out of range", i);
    HIPCHK(c, hipSetDevice(c->device));
    // the final records first: a batch cut short by the RNG stream is re-run here, as in
    // mim_batch_results, so the mask is never that of an unfinished RANSAC
    std::vector<mim_result> res;
    mim_status fs = finish_batch_locked(c, res);
    if (fs != MIM_OK) return fs;
    int ng = 0;
    HIPCHK(c, hipMemcpy(&ng, c->n_good.as<int>() + i, sizeof(int), hipMemcpyDeviceToHost));
    const long long o = c->h_good_off[i];
    if (ng > 0) {
        if (q_idx) HIPCHK(c, hipMemcpy(q_idx, c->good_q.as<int32_t>() + o, sizeof(int32_t) * ng, hipMemcpyDeviceToHost));
        if (t_idx) HIPCHK(c, hipMemcpy(t_idx, c->good_t.as<int32_t>() + o, sizeof(int32_t) * ng, hipMemcpyDeviceToHost));
        if (mask) HIPCHK(c, hipMemcpy(mask, c->masks.as<uint8_t>() + o, ng, hipMemcpyDeviceToHost));
    }
    return MIM_OK;
}

mim_status mim_batch_inlier_points(mim_ctx* c, const float* scales, float* out_xy, int64_t cap, int64_t* offsets) {
    if (!c) return MIM_EINVAL;
    if (!offsets || cap < 0) return fail(c, MIM_EINVAL, "batch_inlier_points: bad arguments");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    std::vector<mim_result> res;
    mim_status fs = finish_batch_locked(c, res);  // waits; re-runs a batch cut short by the RNG stream
    if (fs != MIM_OK) return fs;
    const int n = c->last_n;
    // the gather reads the scene keypoints through the batch's set table: sets cleared or truncated
    // since mim_batch_run have had their storage rewound and possibly reused by newer sets
    if (n > 0 && c->last_fh)
        return fail(c, MIM_EINVAL, "batch_inlier_points: the last call was mim_find_homography, whose record has "
                                   "no scene set to gather from (read its mask instead)");
    if (n > 0 && c->last_gen != c->sets_gen)
        return fail(c, MIM_EINVAL, "batch_inlier_points: the batch's sets were cleared or truncated since "
                                   "mim_batch_run");
    offsets[0] = 0;
    for (int i = 0; i < n; ++i)  // TestsDetector.cpp:79-84: only accepted problems contribute
        offsets[i + 1] = offsets[i] + (res[i].status == MIM_ACCEPTED ? res[i].n_inl : 0);
    const long long total = n ? offsets[n] : 0;
    if (!out_xy || total == 0) return MIM_OK;
    if (total > cap) return fail(c, MIM_ERANGE, "batch_inlier_points: %lld points, buffer holds %lld", total, (long long)cap);
    // table: offsets (n + 1) then the scales (n), one copy; the gather; one copy of the points back
    const size_t tb = sizeof(long long) * (n + 1) + (scales ? sizeof(float) * n : 0);
    HIPCHK(c, c->inl_tab.ensure(tb));
    HIPCHK(c, c->inl_out.ensure(sizeof(float2) * total));
    char* st = nullptr;
    HIPCHK(c, c->stage.acquire(tb, &st));
    memcpy(st, offsets, sizeof(long long) * (n + 1));
    if (scales) memcpy(st + sizeof(long long) * (n + 1), scales, sizeof(float) * n);
    HIPCHK(c, hipMemcpyAsync(c->inl_tab.p, st, tb, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, c->stage.release_after(c->stream));
    const long long* offs = c->inl_tab.as<long long>();
    launch_inlier_gather(c->probs.as<ProbDev>(), n, c->results.as<mim_result>(), c->good_t.as<int32_t>(),
                         c->masks.as<uint8_t>(), offs,
                         scales ? reinterpret_cast<const float*>(offs + n + 1) : nullptr, c->inl_out.as<float2>(),
                         c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(out_xy, c->inl_out.p, sizeof(float2) * total, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return MIM_OK;
}

mim_status mim_find_homography(mim_ctx* c, const float* src, const float* dst, int32_t n, double thresh,
                               int32_t max_iters, double conf, double H[9], uint8_t* mask) {
    if (!c) return MIM_EINVAL;
    if (!src || !dst || !H || !mask) return fail(c, MIM_EINVAL, "find_homography: null pointer");
    if (n < 4)  // CV_Error(StsVecLengthErr) in cv::findHomography
        return fail(c, MIM_EINVAL, "The input arrays should have at least 4 corresponding point sets");
    mim_params prm;
    mim_default_params(&prm);
    prm.ransac_thresh = thresh;
    prm.max_iters = max_iters;
    prm.confidence = conf;
    prm.min_good = 4;
    prm.min_inliers = 0;
    mim_status s = check_params(c, &prm);
    if (s != MIM_OK) return s;
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<float4> pts(n);
    for (int i = 0; i < n; ++i) pts[i] = make_float4(src[2 * i], src[2 * i + 1], dst[2 * i], dst[2 * i + 1]);
    HIPCHK(c, c->pts.ensure(sizeof(float4) * n));
    HIPCHK(c, c->n_good.ensure(sizeof(int)));
    HIPCHK(c, c->probs.ensure(sizeof(ProbDev)));
    HIPCHK(c, hipMemcpy(c->pts.p, pts.data(), sizeof(float4) * n, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->n_good.p, &n, sizeof(int), hipMemcpyHostToDevice));
    ProbDev P{};
    P.q.n = n;
    P.good_off = 0;
    P.it_off = 0;
    HIPCHK(c, hipMemcpy(c->probs.p, &P, sizeof P, hipMemcpyHostToDevice));
    c->h_probs.assign(1, P);
    c->h_good_off.assign(1, 0);
    c->last_n = 1;  // mim_batch_results returns this call's record (mim.h)
    c->last_gen = -1;
    c->last_fh = true;
    c->last_problems.clear();
    mim_result r;
    for (;;) {  // a run out of RNG draws is re-run on a longer stream
        c->cur = c->stream;
        ev_mark(c, "begin");
        s = ransac_locked(c, 1, &prm, 1);
        if (s != MIM_OK) return s;
        HIPCHK(c, hipStreamSynchronize(c->stream));
        ev_collect(c);
        HIPCHK(c, hipMemcpy(&r, c->results.p, sizeof r, hipMemcpyDeviceToHost));
        if (r.status != MIM_STREAM_SHORT) break;
        s = grow_stream(c);
        if (s != MIM_OK) return s;
    }
    HIPCHK(c, hipMemcpy(mask, c->masks.p, n, hipMemcpyDeviceToHost));
    if (r.status == MIM_EMPTY_H) {
        for (int i = 0; i < 9; ++i) H[i] = 0;
        memset(mask, 0, n);
        return MIM_ENOMODEL;
    }
    for (int i = 0; i < 9; ++i) H[i] = r.H[i];
    return MIM_OK;
}

}  // extern "C"
