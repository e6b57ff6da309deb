// group.cpp — several GPUs of one node behind the C ABI (include/mim.h, "several GPUs"):
// scene-batch data parallelism with one RCCL all-gather of the result records.
//
// The reference's process loops over the test scenes (processAllTestImages, /root/reference/src/
// Output.cpp:23-57) into detectObjects (/root/reference/src/TestsDetector.cpp:58-95), and no problem
// depends on another.  A mim_group holds one mim_ctx per device and an RCCL communicator over them
// (ncclCommInitAll: one process, every GPU); a scene batch is split into contiguous scene ranges
// (sizes differ by at most one, as shard.shard_range), each device uploads and matches only its own
// scenes on its own ctx, and one ncclAllGather over xGMI puts every device's fixed-size mim_result
// records (padded to the largest range) on every device.  The query (model view) sets are replicated:
// registered once per device, before the scene batches.  No descriptor crosses devices.
//
// Built only on the public C ABI of api.cpp (one ctx per device), plus HIP streams/events and RCCL.
// A group whose device list repeats a device (two ctxs on one GPU: the test mode of a one-GPU box)
// cannot hold an RCCL communicator (RCCL refuses two ranks on one device); it gathers with
// device-to-device copies ordered by events instead, the same records in the same places.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mim.h"

struct mim_group {
    std::vector<int> dev;
    std::vector<mim_ctx*> ctx;
    std::vector<ncclComm_t> comm;  // empty: the device list repeats a device (copy gather)
    std::vector<void*> send, recv;  // per rank: its padded records / the world's gathered records
    std::vector<hipEvent_t> ev;     // per rank: its records copied into `send` (copy gather)
    size_t cap = 0;                 // records per rank the buffers hold
    int base_sets = 0;              // replicated (query) sets registered on every ctx
    // the last scene batch
    int n_scenes = 0, n_tmpl = 0, pad = 0;
    std::vector<int> first, count;
    bool pending = false;
    std::string err;
};

static mim_status gfail(mim_group* g, mim_status code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (g) g->err = buf;
    return code;
}

#define GHIP(g, expr)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess)                                                                           \
            return gfail((g), e_ == hipErrorOutOfMemory ? MIM_ENOMEM : MIM_EDEVICE, "%s: %s (%s:%d)", #expr, \
                         hipGetErrorString(e_), __FILE__, __LINE__);                                    \
    } while (0)

#define GNCCL(g, expr)                                                                                  \
    do {                                                                                                \
        ncclResult_t r_ = (expr);                                                                       \
        if (r_ != ncclSuccess)                                                                          \
            return gfail((g), MIM_EDEVICE, "%s: %s (%s:%d)", #expr, ncclGetErrorString(r_), __FILE__, __LINE__); \
    } while (0)

static mim_status ctx_fail(mim_group* g, int rank, mim_status s, const char* what) {
    return gfail(g, s, "rank %d (device %d): %s: %s", rank, g->dev[rank], what, mim_last_error(g->ctx[rank]));
}

static void release_buffers(mim_group* g) {
    for (size_t r = 0; r < g->dev.size(); ++r) {
        (void)hipSetDevice(g->dev[r]);
        if (r < g->send.size() && g->send[r]) (void)hipFree(g->send[r]);
        if (r < g->recv.size() && g->recv[r]) (void)hipFree(g->recv[r]);
    }
    g->send.assign(g->dev.size(), nullptr);
    g->recv.assign(g->dev.size(), nullptr);
    g->cap = 0;
}

extern "C" {

mim_status mim_group_shard(int32_t n_items, int32_t world, int32_t rank, int32_t* first, int32_t* count) {
    if (n_items < 0 || world < 1 || rank < 0 || rank >= world || !first || !count) return MIM_EINVAL;
    const int32_t base = n_items / world, extra = n_items % world;
    *first = rank * base + std::min(rank, extra);
    *count = base + (rank < extra ? 1 : 0);
    return MIM_OK;
}

void mim_group_destroy(mim_group* g) {
    if (!g) return;
    for (size_t r = 0; r < g->ctx.size(); ++r)
        if (g->ctx[r]) (void)mim_synchronize(g->ctx[r]);
    for (ncclComm_t c : g->comm)
        if (c) (void)ncclCommDestroy(c);
    release_buffers(g);
    for (size_t r = 0; r < g->ev.size(); ++r) {
        (void)hipSetDevice(g->dev[r]);
        if (g->ev[r]) (void)hipEventDestroy(g->ev[r]);
    }
    for (mim_ctx* c : g->ctx) mim_ctx_destroy(c);
    delete g;
}

mim_status mim_group_create(const int32_t* devices, int32_t n_devices, mim_group** out) {
    if (!out) return MIM_EINVAL;
    *out = nullptr;
    if (!devices || n_devices < 1) return MIM_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MIM_EDEVICE;
    for (int i = 0; i < n_devices; ++i)
        if (devices[i] < 0 || devices[i] >= ndev) return MIM_EINVAL;
    mim_group* g = new mim_group();
    g->dev.assign(devices, devices + n_devices);
    g->ctx.assign(n_devices, nullptr);
    g->ev.assign(n_devices, nullptr);
    g->send.assign(n_devices, nullptr);
    g->recv.assign(n_devices, nullptr);
    for (int r = 0; r < n_devices; ++r) {
        const mim_status s = mim_ctx_create(g->dev[r], &g->ctx[r]);
        if (s != MIM_OK) {
            mim_group_destroy(g);
            return s;
        }
        // the batches of the ranks already overlap one another (one per device): one stream per ctx
        (void)mim_ctx_set_sampler_stream(g->ctx[r], 0);
        if (hipSetDevice(g->dev[r]) != hipSuccess ||
            hipEventCreateWithFlags(&g->ev[r], hipEventDisableTiming) != hipSuccess) {
            mim_group_destroy(g);
            return MIM_EDEVICE;
        }
    }
    std::vector<int> sorted = g->dev;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (distinct) {
        g->comm.assign(n_devices, nullptr);
        if (ncclCommInitAll(g->comm.data(), n_devices, g->dev.data()) != ncclSuccess) {
            g->comm.clear();
            mim_group_destroy(g);
            return MIM_EDEVICE;
        }
    }
    *out = g;
    return MIM_OK;
}

int32_t mim_group_size(const mim_group* g) { return g ? (int32_t)g->dev.size() : 0; }

int32_t mim_group_uses_rccl(const mim_group* g) { return g && !g->comm.empty() ? 1 : 0; }

mim_ctx* mim_group_ctx(mim_group* g, int32_t rank) {
    return g && rank >= 0 && rank < (int32_t)g->ctx.size() ? g->ctx[rank] : nullptr;
}

const char* mim_group_last_error(const mim_group* g) { return g ? g->err.c_str() : "null group"; }

mim_status mim_group_set_create(mim_group* g, const float* desc, const float* kp_xy, int32_t n, int32_t dim,
                                int32_t* set_id) {
    if (!g) return MIM_EINVAL;
    if (!set_id) return gfail(g, MIM_EINVAL, "group_set_create: null set_id");
    int32_t id0 = -1;
    for (size_t r = 0; r < g->ctx.size(); ++r) {
        int32_t n_sets = 0;
        mim_status s = mim_sets_info(g->ctx[r], &n_sets, nullptr);
        if (s == MIM_OK && n_sets != g->base_sets) s = mim_sets_truncate(g->ctx[r], g->base_sets);  // scene sets go
        if (s != MIM_OK) return ctx_fail(g, (int)r, s, "sets_truncate");
        int32_t id = -1;
        s = mim_set_create(g->ctx[r], desc, kp_xy, n, dim, 0, &id);
        if (s != MIM_OK) {
            for (size_t q = 0; q < r; ++q) (void)mim_sets_truncate(g->ctx[q], g->base_sets);  // all or nothing
            return ctx_fail(g, (int)r, s, "set_create");
        }
        if (r == 0) id0 = id;
        if (id != id0) return gfail(g, MIM_EINVAL, "group_set_create: set ids diverged across devices");
    }
    g->base_sets = id0 + 1;
    *set_id = id0;
    return MIM_OK;
}

// One rank's part of a scene batch: its scenes' sets uploaded to its device, its problems enqueued,
// its records copied into `send` (padded with zero records past its own).  Runs on its own host
// thread per rank, so the uploads of the devices overlap; errors go to the rank's own string.
static mim_status rank_run(mim_group* g, int r, int sets_per_scene, const mim_host_set* scene_sets, int n_tmpl,
                           const mim_problem* tmpl, const mim_params* params, std::string& err) {
    mim_ctx* c = g->ctx[r];
    auto cfail = [&](mim_status s, const char* what) {
        err = std::string("rank ") + std::to_string(r) + " (device " + std::to_string(g->dev[r]) + "): " + what + ": " +
              mim_last_error(c);
        return s;
    };
    auto hfail = [&](hipError_t e, const char* what) {
        err = std::string("rank ") + std::to_string(r) + ": " + what + ": " + hipGetErrorString(e);
        return e == hipErrorOutOfMemory ? (mim_status)MIM_ENOMEM : (mim_status)MIM_EDEVICE;
    };
    mim_status s = mim_sets_truncate(c, g->base_sets);
    if (s != MIM_OK) return cfail(s, "sets_truncate");
    const int ns = g->count[r] * sets_per_scene;
    std::vector<const float*> desc(ns), kp(ns);
    std::vector<int32_t> rows(ns);
    for (int i = 0; i < ns; ++i) {
        const mim_host_set& hs = scene_sets[(size_t)g->first[r] * sets_per_scene + i];
        desc[i] = hs.desc;
        kp[i] = hs.kp_xy;
        rows[i] = hs.n;
    }
    int32_t first_id = 0;
    if (ns > 0) {
        s = mim_sets_create(c, ns, desc.data(), kp.data(), rows.data(), 128, 0, &first_id);
        if (s != MIM_OK) return cfail(s, "sets_create");
    }
    std::vector<mim_problem> probs((size_t)g->count[r] * n_tmpl);
    for (int j = 0; j < g->count[r]; ++j)
        for (int k = 0; k < n_tmpl; ++k)
            probs[(size_t)j * n_tmpl + k] = mim_problem{tmpl[k].query_set, first_id + j * sets_per_scene + tmpl[k].train_set};
    s = mim_batch_run(c, probs.data(), (int32_t)probs.size(), params);
    if (s != MIM_OK) return cfail(s, "batch_run");
    hipError_t e = hipSetDevice(g->dev[r]);
    if (e != hipSuccess) return hfail(e, "hipSetDevice");
    hipStream_t st = (hipStream_t)mim_ctx_get_stream(c);
    e = hipMemsetAsync(g->send[r], 0, sizeof(mim_result) * (size_t)g->pad, st);
    if (e != hipSuccess) return hfail(e, "hipMemsetAsync");
    s = mim_batch_results_copy(c, g->send[r], 1);
    if (s != MIM_OK) return cfail(s, "batch_results_copy");
    e = hipEventRecord(g->ev[r], st);
    if (e != hipSuccess) return hfail(e, "hipEventRecord");
    return MIM_OK;
}

mim_status mim_group_scene_batch_run(mim_group* g, int32_t n_scenes, int32_t sets_per_scene,
                                     const mim_host_set* scene_sets, int32_t n_tmpl, const mim_problem* tmpl,
                                     const mim_params* params) {
    if (!g) return MIM_EINVAL;
    if (n_scenes < 0 || sets_per_scene < 1 || n_tmpl < 0 || !params || (n_scenes > 0 && !scene_sets) ||
        (n_tmpl > 0 && !tmpl))
        return gfail(g, MIM_EINVAL, "group_scene_batch_run: bad arguments");
    for (int k = 0; k < n_tmpl; ++k)
        if (tmpl[k].query_set < 0 || tmpl[k].query_set >= g->base_sets || tmpl[k].train_set < 0 ||
            tmpl[k].train_set >= sets_per_scene)
            return gfail(g, MIM_EINVAL, "group_scene_batch_run: template %d names set (%d, %d); %d replicated sets, %d "
                                        "sets per scene", k, tmpl[k].query_set, tmpl[k].train_set, g->base_sets,
                         sets_per_scene);
    if (g->pending) {  // the previous batch's gather still reads `send`: finish it first
        mim_status s = mim_group_results(g, nullptr);
        if (s != MIM_OK) return s;
    }
    const int W = (int)g->dev.size();
    g->first.assign(W, 0);
    g->count.assign(W, 0);
    int maxc = 0;
    for (int r = 0; r < W; ++r) {
        mim_group_shard(n_scenes, W, r, &g->first[r], &g->count[r]);
        maxc = std::max(maxc, g->count[r]);
    }
    g->n_scenes = n_scenes;
    g->n_tmpl = n_tmpl;
    g->pad = std::max(1, maxc * n_tmpl);
    if ((size_t)g->pad > g->cap) {
        release_buffers(g);
        for (int r = 0; r < W; ++r) {
            GHIP(g, hipSetDevice(g->dev[r]));
            GHIP(g, hipMalloc(&g->send[r], sizeof(mim_result) * (size_t)g->pad));
            GHIP(g, hipMalloc(&g->recv[r], sizeof(mim_result) * (size_t)g->pad * W));
        }
        g->cap = (size_t)g->pad;
    }
    std::vector<mim_status> st(W, MIM_OK);
    std::vector<std::string> errs(W);
    if (W == 1) {
        st[0] = rank_run(g, 0, sets_per_scene, scene_sets, n_tmpl, tmpl, params, errs[0]);
    } else {
        std::vector<std::thread> th;
        for (int r = 0; r < W; ++r)
            th.emplace_back([&, r] { st[r] = rank_run(g, r, sets_per_scene, scene_sets, n_tmpl, tmpl, params, errs[r]); });
        for (auto& t : th) t.join();
    }
    for (int r = 0; r < W; ++r)
        if (st[r] != MIM_OK) {
            g->err = errs[r];
            return st[r];
        }
    const size_t bytes = sizeof(mim_result) * (size_t)g->pad;
    if (!g->comm.empty()) {
        // one all-gather over xGMI: every device receives every rank's padded records, rank-major
        GNCCL(g, ncclGroupStart());
        for (int r = 0; r < W; ++r) {
            hipStream_t s = (hipStream_t)mim_ctx_get_stream(g->ctx[r]);
            const ncclResult_t e = ncclAllGather(g->send[r], g->recv[r], bytes, ncclUint8, g->comm[r], s);
            if (e != ncclSuccess) {
                (void)ncclGroupEnd();
                return gfail(g, MIM_EDEVICE, "ncclAllGather (rank %d): %s", r, ncclGetErrorString(e));
            }
        }
        GNCCL(g, ncclGroupEnd());
    } else {
        for (int r = 0; r < W; ++r) {
            GHIP(g, hipSetDevice(g->dev[r]));
            hipStream_t s = (hipStream_t)mim_ctx_get_stream(g->ctx[r]);
            for (int q = 0; q < W; ++q) {
                if (q != r) GHIP(g, hipStreamWaitEvent(s, g->ev[q], 0));
                GHIP(g, hipMemcpyAsync((char*)g->recv[r] + bytes * q, g->send[q], bytes, hipMemcpyDeviceToDevice, s));
            }
        }
    }
    g->pending = true;
    return MIM_OK;
}

mim_status mim_group_results(mim_group* g, mim_result* out) {
    if (!g) return MIM_EINVAL;
    const int W = (int)g->dev.size();
    const size_t pad = (size_t)g->pad;
    std::vector<mim_result> all(pad * W);
    for (int r = 0; r < W; ++r) {  // every rank's gather (rank 0's buffer is read below)
        mim_status s = mim_synchronize(g->ctx[r]);
        if (s != MIM_OK) return ctx_fail(g, r, s, "synchronize");
    }
    if (g->n_scenes > 0 && g->n_tmpl > 0) {
        GHIP(g, hipSetDevice(g->dev[0]));
        GHIP(g, hipMemcpy(all.data(), g->recv[0], sizeof(mim_result) * pad * W, hipMemcpyDeviceToHost));
    }
    g->pending = false;
    if (!out) return MIM_OK;
    std::vector<mim_result> fix;
    for (int r = 0; r < W; ++r) {
        const size_t m = (size_t)g->count[r] * g->n_tmpl;
        const mim_result* src = all.data() + pad * r;
        bool short_ = false;
        for (size_t i = 0; i < m; ++i) short_ |= src[i].status == MIM_STREAM_SHORT;
        if (short_) {  // a problem ran out of RNG draws: the rank's ctx grows its stream and re-runs the batch
            fix.resize(m);
            mim_status s = mim_batch_results(g->ctx[r], fix.data());
            if (s != MIM_OK) return ctx_fail(g, r, s, "batch_results");
            src = fix.data();
        }
        if (m > 0) memcpy(out + (size_t)g->first[r] * g->n_tmpl, src, sizeof(mim_result) * m);
    }
    return MIM_OK;
}

}  // extern "C"
