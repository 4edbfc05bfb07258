// multi.cpp — single-process multi-GPU part scheduler (cec_multi_*).
//
// The reference writes and reads a file from ONE process: FileWriteBuilder::write runs up to
// `concurrency` part tasks (src/file/writer.rs:117-255, semaphore :130, spawn :208) and the
// reader streams parts with buffered(5) (src/file/reader.rs:63); resilver uses buffered(10)
// (file_reference.rs:109).  Parts are independent, so on a GPU node the natural form is part-wise
// sharding over the devices with no exchange: a job of n parts in file order is
// split into contiguous ranges [g*n/G, (g+1)*n/G), one per shard, and every result lands at its
// part's own position, so results come back in file order without any reordering.
//
// One worker thread per shard (a device may carry several shards).  Each worker binds itself to
// its device's NUMA node (hostmem.cpp) before allocating anything, owns a write and a read
// pipeline of `depth` slots (pipeline.cpp, CEC_PIPE_EXTERNAL), and streams its range batch by
// batch: caller buffers that are page-locked (cec_host_alloc) are DMA'd directly; pageable ones
// go through the worker's own NUMA-local pinned staging.  Jobs are queued and run in submission
// order; a worker keeps its batches in flight across job boundaries: with its queue empty it
// completes batches as their events fire while watching the queue, so the next job of a stream
// is queued behind the batches still running instead of after a drain (no bubble).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "chunky_ec.h"
#include "hostmem.hpp"
#include "knobs.hpp"

namespace {

thread_local std::string g_multi_error;

enum class Kind { Write, Read };

struct Job {
    uint64_t id = 0;
    Kind kind = Kind::Write;
    size_t n = 0;
    unsigned flags = 0;
    // write
    const uint8_t* data = nullptr;
    uint8_t* parity = nullptr;
    uint8_t* digests = nullptr;
    // read
    const uint8_t* chunks = nullptr;
    const uint8_t* present = nullptr;
    const uint8_t* expected = nullptr;
    uint8_t* out_data = nullptr;
    uint8_t* verified = nullptr;
    int* status = nullptr;
    const uint8_t** data_ptrs = nullptr;
    bool resilver = false;  // FilePart::resilver's compute: output [n][t][L], t pointers a part
    bool verify_only = false;  // FilePart::verify's compute: verified flags only
    // completion
    size_t remaining = 0;  // parts not yet finished (guarded by cec_multi::mu)
    int result = CEC_OK;
    std::string error;
};

// Pinned staging of one slot (pageable caller buffers only), NUMA-local to the worker.
struct Staging {
    uint8_t* in = nullptr;   // write: [P][d][L]; read: [P][t][L]
    uint8_t* out = nullptr;  // write: [P][p][L]; read: [P][d][L]
    size_t in_cap = 0, out_cap = 0;
    void release() {
        if (in) (void)hipHostFree(in);
        if (out) (void)hipHostFree(out);
        in = out = nullptr;
        in_cap = out_cap = 0;
    }
    hipError_t reserve(size_t in_bytes, size_t out_bytes, int device) {
        hipError_t e = hipSuccess;
        if (in_cap < in_bytes) {
            if (in) (void)hipHostFree(in);
            in = nullptr;
            in_cap = 0;
            e = cec::host_malloc_near(reinterpret_cast<void**>(&in), in_bytes,
                                      hipHostMallocDefault, device);
            if (e != hipSuccess) return e;
            in_cap = in_bytes;
        }
        if (out_cap < out_bytes) {
            if (out) (void)hipHostFree(out);
            out = nullptr;
            out_cap = 0;
            e = cec::host_malloc_near(reinterpret_cast<void**>(&out), out_bytes,
                                      hipHostMallocDefault, device);
            if (e != hipSuccess) return e;
            out_cap = out_bytes;
        }
        return hipSuccess;
    }
};

// Host threads per shard for its staging copies (CEC_MULTI_COPY_THREADS, default 4): one
// thread's memcpy (~10 GB/s) is below the ~55 GB/s a GPU's PCIe link takes.
size_t copy_threads() { return cec::knobs().multi_copy_threads; }

// fn(i) for i in [0, n) split in contiguous ranges over copy_threads() threads (inline when the
// work is small).
template <typename Fn>
void parallel_for(size_t n, size_t bytes, Fn fn) {
    const size_t w = std::min(copy_threads(), n);
    if (w <= 1 || bytes < (size_t(16) << 20)) {
        for (size_t i = 0; i < n; ++i) fn(i);
        return;
    }
    std::vector<std::thread> pool;
    pool.reserve(w - 1);
    for (size_t k = 1; k < w; ++k)
        pool.emplace_back([&, k] {
            for (size_t i = n * k / w; i < n * (k + 1) / w; ++i) fn(i);
        });
    for (size_t i = 0; i < n / w; ++i) fn(i);
    for (auto& th : pool) th.join();
}

void parallel_copy(uint8_t* dst, const uint8_t* src, size_t n) {
    constexpr size_t kGrain = size_t(1) << 20;
    parallel_for((n + kGrain - 1) / kGrain, n, [&](size_t i) {
        const size_t off = i * kGrain;
        std::memcpy(dst + off, src + off, std::min(kGrain, n - off));
    });
}

// A batch in flight on one slot of a shard's pipeline.
struct InFlight {
    Job* job = nullptr;
    size_t first = 0, n = 0;  // parts [first, first + n) of the job
    bool staged_in = false, staged_out = false;
    bool direct_dig = false;  // write: digests DMA'd straight into the job's buffer
};

}  // namespace

struct cec_multi;

namespace {

struct Shard {
    cec_multi* owner = nullptr;
    size_t index = 0;
    int device = 0;
    int numa = -1;
    bool bound = false;
    std::thread th;
    std::deque<Job*> queue;  // guarded by cec_multi::mu
    std::atomic<uint64_t> parts{0};
    // worker-thread state
    cec_pipeline* wp = nullptr;
    cec_read_pipeline* rp = nullptr;
    unsigned rp_flags = 0;
    Kind active = Kind::Write;
    std::vector<InFlight> wslots, rslots;
    std::deque<size_t> worder, rorder;  // slots in flight, oldest first
    std::vector<Staging> wstage, rstage;
    std::vector<const uint8_t*> ptrs;  // read: data chunk locations of one batch
};

}  // namespace

struct cec_multi {
    const cec_codec* codec = nullptr;
    size_t d = 0, p = 0, t = 0, L = 0, P = 0, depth = 0;
    std::vector<std::unique_ptr<Shard>> shards;
    std::mutex mu;
    std::condition_variable work_cv, done_cv;
    bool stop = false;
    uint64_t next_id = 1;
    std::map<uint64_t, std::unique_ptr<Job>> jobs;  // submitted, not yet waited for

    // ---- completion (worker threads) ----
    void finish_parts(Job* job, size_t n, int st, const std::string& err) {
        std::lock_guard<std::mutex> lk(mu);
        if (st != CEC_OK && job->result == CEC_OK) {
            job->result = st;
            job->error = err;
        }
        job->remaining -= n;
        if (job->remaining == 0) done_cv.notify_all();
    }

    // ---- per-shard work ----
    int ensure_write_pipe(Shard& s) {
        if (s.wp) return CEC_OK;
        int st = cec_pipeline_new_ex(codec, L, P, depth, CEC_PIPE_EXTERNAL, &s.wp);
        if (st != CEC_OK) g_multi_error = cec_pipeline_last_error();
        s.wslots.assign(depth, InFlight{});
        s.wstage.resize(depth);
        return st;
    }

    int ensure_read_pipe(Shard& s, unsigned flags, bool resilver, bool verify_only) {
        const unsigned want = (flags & CEC_READ_REBUILT_ONLY) | CEC_PIPE_EXTERNAL |
                              (resilver ? CEC_READ_RESILVER : 0u) |
                              (verify_only ? CEC_READ_VERIFY_ONLY : 0u);
        if (s.rp && s.rp_flags == want) return CEC_OK;
        if (s.rp) {
            drain_read(s);
            cec_read_pipeline_free(s.rp);
            s.rp = nullptr;
        }
        int st = cec_read_pipeline_new_ex(codec, L, P, depth, want, &s.rp);
        if (st != CEC_OK) g_multi_error = cec_pipeline_last_error();
        s.rp_flags = want;
        s.rslots.assign(depth, InFlight{});
        s.rstage.resize(depth);
        return st;
    }

    void finish_write(Shard& s, size_t slot) {
        InFlight& f = s.wslots[slot];
        if (!f.job) return;
        auto wo = std::find(s.worder.begin(), s.worder.end(), slot);
        if (wo != s.worder.end()) s.worder.erase(wo);
        const uint8_t *par = nullptr, *dig = nullptr;
        size_t got = 0;
        int st = cec_pipeline_wait(s.wp, slot, &par, &dig, &got);
        std::string err = st == CEC_OK ? std::string() : cec_pipeline_last_error();
        Job* job = f.job;
        if (st == CEC_OK) {
            if (f.staged_out) parallel_copy(job->parity + f.first * p * L, par, f.n * p * L);
            if (!f.direct_dig) std::memcpy(job->digests + f.first * t * 32, dig, f.n * t * 32);
        }
        s.parts.fetch_add(f.n, std::memory_order_relaxed);
        const size_t n = f.n;
        f = InFlight{};
        finish_parts(job, n, st, err);
    }

    void finish_read(Shard& s, size_t slot) {
        InFlight& f = s.rslots[slot];
        if (!f.job) return;
        auto ro = std::find(s.rorder.begin(), s.rorder.end(), slot);
        if (ro != s.rorder.end()) s.rorder.erase(ro);
        const uint8_t *data = nullptr, *ver = nullptr;
        const int* status = nullptr;
        size_t got = 0;
        Job* job = f.job;
        // chunks per part in the output / pointer table: d (read) or t (resilver)
        const size_t W = (s.rp_flags & CEC_READ_RESILVER) ? t : d;
        const bool verify_only = (s.rp_flags & CEC_READ_VERIFY_ONLY) != 0;
        int st = cec_read_pipeline_wait(s.rp, slot, &data, &ver, &status, &got);
        if (st == CEC_OK && !verify_only) {
            s.ptrs.resize(f.n * W);
            st = cec_read_pipeline_data_chunks(s.rp, slot, s.ptrs.data());
        }
        std::string err = st == CEC_OK ? std::string() : cec_pipeline_last_error();
        if (st == CEC_OK && verify_only) {
            std::memcpy(job->verified + f.first * t, ver, f.n * t);
        } else if (st == CEC_OK) {
            std::memcpy(job->verified + f.first * t, ver, f.n * t);
            std::memcpy(job->status + f.first, status, f.n * sizeof(int));
            const bool staged = f.staged_in || f.staged_out;
            parallel_for(f.n, staged ? f.n * W * L : 0, [&](size_t k) {
                for (size_t j = 0; j < W; ++j) {
                    const size_t q = (f.first + k) * W + j;
                    const uint8_t* src = s.ptrs[k * W + j];
                    uint8_t* dst = job->out_data + q * L;
                    if (staged) {
                        // staging is reused by the next batch: the bytes move to the caller (a
                        // part that could not be decoded has no bytes: its pointers are null)
                        if (status[k] == CEC_OK && src != dst) std::memcpy(dst, src, L);
                        src = status[k] == CEC_OK ? dst : nullptr;
                    }
                    if (job->data_ptrs) job->data_ptrs[q] = src;
                }
            });
        }
        s.parts.fetch_add(f.n, std::memory_order_relaxed);
        const size_t n = f.n;
        f = InFlight{};
        finish_parts(job, n, st, err);
    }

    void drain_write(Shard& s) {
        if (!s.wp) return;
        for (size_t i = 0; i < s.wslots.size(); ++i) finish_write(s, i);
    }
    void drain_read(Shard& s) {
        if (!s.rp) return;
        for (size_t i = 0; i < s.rslots.size(); ++i) finish_read(s, i);
    }
    void drain(Shard& s) {
        drain_write(s);
        drain_read(s);
    }
    bool in_flight(const Shard& s) const { return !s.worder.empty() || !s.rorder.empty(); }

    // Finish the oldest batch in flight if it is complete; never blocks.  False when it is still
    // running (or nothing is in flight).
    bool finish_oldest_if_done(Shard& s) {
        if (!s.worder.empty()) {
            const size_t slot = s.worder.front();
            if (cec_pipeline_query(s.wp, slot) != 1) return false;
            finish_write(s, slot);
            return true;
        }
        if (!s.rorder.empty()) {
            const size_t slot = s.rorder.front();
            if (cec_read_pipeline_query(s.rp, slot) != 1) return false;
            finish_read(s, slot);
            return true;
        }
        return false;
    }

    void run_write(Shard& s, Job* job, size_t lo, size_t hi) {
        int st = ensure_write_pipe(s);
        if (st != CEC_OK) return finish_parts(job, hi - lo, st, g_multi_error);
        if (s.active != Kind::Write) drain_read(s);
        s.active = Kind::Write;
        const size_t dw = d * L, pw = p * L;
        for (size_t first = lo; first < hi; first += P) {
            const size_t n = std::min(P, hi - first);
            size_t slot = 0;
            uint8_t* unused = nullptr;
            st = cec_pipeline_acquire(s.wp, &slot, &unused);
            if (st != CEC_OK) {
                finish_parts(job, hi - first, st, cec_pipeline_last_error());
                return;
            }
            finish_write(s, slot);  // the slot's previous batch (possibly of an earlier job)
            InFlight f;
            f.job = job;
            f.first = first;
            f.n = n;
            const uint8_t* src = job->data + first * dw;
            uint8_t* par = job->parity + first * pw;
            uint8_t* dig = job->digests + first * t * 32;
            f.staged_in = !cec::pinned_range(src, n * dw);
            f.staged_out = !cec::pinned_range(par, n * pw);
            f.direct_dig = cec::pinned_range(dig, n * t * 32);
            Staging& sg = s.wstage[slot];
            if (f.staged_in || f.staged_out) {
                // every slot's staging at once: pinning costs ~0.35 s per GiB, so it happens on
                // the first pageable job, not whenever a later job first reaches a slot
                hipError_t e = hipSuccess;
                for (Staging& each : s.wstage)
                    if (e == hipSuccess)
                        e = each.reserve(f.staged_in ? P * dw : 0, f.staged_out ? P * pw : 0,
                                         s.device);
                if (e != hipSuccess) {
                    finish_parts(job, hi - first, CEC_ERR_OUT_OF_MEMORY,
                                 std::string("multi staging: ") + hipGetErrorString(e));
                    return;
                }
            }
            if (f.staged_in) {
                parallel_copy(sg.in, src, n * dw);
                src = sg.in;
            }
            st = cec_pipeline_submit_from(s.wp, slot, src, n, f.staged_out ? sg.out : par,
                                          f.direct_dig ? dig : nullptr);
            if (st != CEC_OK) {
                finish_parts(job, hi - first, st, cec_pipeline_last_error());
                return;
            }
            s.wslots[slot] = f;
            s.worder.push_back(slot);
        }
    }

    void run_read(Shard& s, Job* job, size_t lo, size_t hi) {
        int st = ensure_read_pipe(s, job->flags, job->resilver, job->verify_only);
        if (st != CEC_OK) return finish_parts(job, hi - lo, st, g_multi_error);
        if (s.active != Kind::Read) drain_write(s);
        s.active = Kind::Read;
        const size_t cw = t * L, dw = (job->resilver ? t : d) * L;  // output per part
        for (size_t first = lo; first < hi; first += P) {
            const size_t n = std::min(P, hi - first);
            size_t slot = 0;
            uint8_t *c = nullptr, *pr = nullptr, *ex = nullptr;
            st = cec_read_pipeline_acquire(s.rp, &slot, &c, &pr, &ex);
            if (st != CEC_OK) {
                finish_parts(job, hi - first, st, cec_pipeline_last_error());
                return;
            }
            finish_read(s, slot);
            InFlight f;
            f.job = job;
            f.first = first;
            f.n = n;
            const uint8_t* src = job->chunks + first * cw;
            uint8_t* dst = job->verify_only ? nullptr : job->out_data + first * dw;
            f.staged_in = !cec::pinned_range(src, n * cw);
            f.staged_out = !job->verify_only && !cec::pinned_range(dst, n * dw);
            Staging& sg = s.rstage[slot];
            if (f.staged_in || f.staged_out) {
                hipError_t e = hipSuccess;  // every slot at once (see run_write)
                for (Staging& each : s.rstage)
                    if (e == hipSuccess)
                        e = each.reserve(f.staged_in ? P * cw : 0, f.staged_out ? P * dw : 0,
                                         s.device);
                if (e != hipSuccess) {
                    finish_parts(job, hi - first, CEC_ERR_OUT_OF_MEMORY,
                                 std::string("multi staging: ") + hipGetErrorString(e));
                    return;
                }
            }
            if (f.staged_in) {
                // only the loaded chunks are staged, packed back to back (part by part, index
                // ascending): the batch then goes up as one copy (submit_packed)
                const uint8_t* prs = job->present + first * t;
                std::vector<size_t> at(n + 1, 0);
                for (size_t k = 0; k < n; ++k)
                    at[k + 1] = at[k] + size_t(std::count_if(prs + k * t, prs + (k + 1) * t,
                                                             [](uint8_t x) { return x != 0; }));
                const uint8_t* from = src;
                uint8_t* to = sg.in;
                parallel_for(n, n * cw, [&](size_t k) {
                    size_t pos = at[k];
                    for (size_t i = k * t; i < (k + 1) * t; ++i)
                        if (prs[i]) std::memcpy(to + (pos++) * L, from + i * L, L);
                });
                st = cec_read_pipeline_submit_packed(s.rp, slot, sg.in, prs,
                                                     job->expected + first * t * 32, n,
                                                     f.staged_out ? sg.out : dst);
            } else {
                st = cec_read_pipeline_submit_from(s.rp, slot, src, job->present + first * t,
                                                   job->expected + first * t * 32, n,
                                                   f.staged_out ? sg.out : dst);
            }
            if (st != CEC_OK) {
                finish_parts(job, hi - first, st, cec_pipeline_last_error());
                return;
            }
            s.rslots[slot] = f;
            s.rorder.push_back(slot);
        }
    }

    void worker(Shard& s) {
        s.bound = cec::bind_thread_to_device_node(s.device);
        if (hipSetDevice(s.device) != hipSuccess) (void)hipGetLastError();
        const size_t G = shards.size();
        for (;;) {
            Job* job = nullptr;
            {
                std::unique_lock<std::mutex> lk(mu);
                // Nothing queued: complete batches as they finish (polling their events, 100 us
                // apart) while watching the queue, so a job submitted meanwhile (the next segment
                // of a stream) is queued behind the batches still running, never behind a drain;
                // sleep on the queue alone only when nothing is in flight.
                while (s.queue.empty() && in_flight(s)) {
                    lk.unlock();
                    while (finish_oldest_if_done(s)) {
                    }
                    lk.lock();
                    if (!s.queue.empty() || !in_flight(s)) break;
                    work_cv.wait_for(lk, std::chrono::microseconds(100));
                }
                work_cv.wait(lk, [&] { return stop || !s.queue.empty(); });
                if (s.queue.empty()) break;  // stop requested and nothing left
                job = s.queue.front();
                s.queue.pop_front();
            }
            const size_t lo = job->n * s.index / G, hi = job->n * (s.index + 1) / G;
            if (hi > lo) {
                if (job->kind == Kind::Write) run_write(s, job, lo, hi);
                else run_read(s, job, lo, hi);
            }
        }
        drain(s);
        if (s.wp) cec_pipeline_free(s.wp);
        if (s.rp) cec_read_pipeline_free(s.rp);
        for (auto& sg : s.wstage) sg.release();
        for (auto& sg : s.rstage) sg.release();
        s.wp = nullptr;
        s.rp = nullptr;
    }

    int submit(std::unique_ptr<Job> job, uint64_t* id) {
        std::lock_guard<std::mutex> lk(mu);
        job->id = next_id++;
        job->remaining = job->n;
        *id = job->id;
        Job* raw = job.get();
        jobs.emplace(raw->id, std::move(job));
        if (raw->n == 0) return CEC_OK;
        // Only shards with a non-empty range get the job: once the others have finished, the
        // caller may free it, and a shard popping it later would read freed memory.
        const size_t G = shards.size();
        for (size_t g = 0; g < G; ++g)
            if (raw->n * (g + 1) / G > raw->n * g / G) shards[g]->queue.push_back(raw);
        work_cv.notify_all();
        return CEC_OK;
    }

    ~cec_multi() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        work_cv.notify_all();
        for (auto& s : shards)
            if (s->th.joinable()) s->th.join();
    }
};

extern "C" {

const char* cec_multi_last_error(void) { return g_multi_error.c_str(); }

int cec_multi_new(const cec_codec* codec, size_t chunk_len, size_t parts_per_batch, size_t depth,
                  const int* devices, size_t n_devices, cec_multi** out) {
    if (!codec || !out || chunk_len == 0 || parts_per_batch == 0 || depth == 0 || depth > 16 ||
        !devices || n_devices == 0 || n_devices > 64)
        return CEC_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    const int count = cec_device_count();
    if (count <= 0) return CEC_ERR_NO_DEVICE;
    for (size_t g = 0; g < n_devices; ++g)
        if (devices[g] < 0 || devices[g] >= count) return CEC_ERR_INVALID_ARGUMENT;
    auto m = std::make_unique<cec_multi>();
    m->codec = codec;
    m->d = cec_codec_data_shards(codec);
    m->p = cec_codec_parity_shards(codec);
    m->t = m->d + m->p;
    m->L = chunk_len;
    m->P = parts_per_batch;
    m->depth = depth;
    for (size_t g = 0; g < n_devices; ++g) {
        auto s = std::make_unique<Shard>();
        s->owner = m.get();
        s->index = g;
        s->device = devices[g];
        s->numa = cec::device_numa_node(devices[g]);
        m->shards.push_back(std::move(s));
    }
    for (auto& s : m->shards) {
        Shard* sp = s.get();
        cec_multi* mp = m.get();
        sp->th = std::thread([mp, sp] { mp->worker(*sp); });
    }
    *out = m.release();
    return CEC_OK;
}

void cec_multi_free(cec_multi* m) { delete m; }

size_t cec_multi_shards(const cec_multi* m) { return m ? m->shards.size() : 0; }

int cec_multi_shard_info(cec_multi* m, size_t g, int* device, int* numa_node, uint64_t* parts) {
    if (!m || g >= m->shards.size()) return CEC_ERR_INVALID_ARGUMENT;
    const Shard& s = *m->shards[g];
    if (device) *device = s.device;
    if (numa_node) *numa_node = s.numa;
    if (parts) *parts = s.parts.load();
    return CEC_OK;
}

int cec_multi_encode_hash(cec_multi* m, const uint8_t* data, size_t n_parts, uint8_t* parity,
                          uint8_t* digests, uint64_t* job) {
    if (!m || !job || (n_parts && (!data || !parity || !digests))) return CEC_ERR_INVALID_ARGUMENT;
    auto j = std::make_unique<Job>();
    j->kind = Kind::Write;
    j->n = n_parts;
    j->data = data;
    j->parity = parity;
    j->digests = digests;
    return m->submit(std::move(j), job);
}

int cec_multi_read(cec_multi* m, const uint8_t* chunks, const uint8_t* present,
                   const uint8_t* expected, size_t n_parts, uint8_t* data, uint8_t* verified,
                   int* part_status, const uint8_t** data_ptrs, unsigned flags, uint64_t* job) {
    if (!m || !job || (flags & ~unsigned(CEC_READ_REBUILT_ONLY))) return CEC_ERR_INVALID_ARGUMENT;
    if (n_parts && (!chunks || !present || !expected || !data || !verified || !part_status))
        return CEC_ERR_INVALID_ARGUMENT;
    if ((flags & CEC_READ_REBUILT_ONLY) && !data_ptrs) return CEC_ERR_INVALID_ARGUMENT;
    auto j = std::make_unique<Job>();
    j->kind = Kind::Read;
    j->n = n_parts;
    j->flags = flags;
    j->chunks = chunks;
    j->present = present;
    j->expected = expected;
    j->out_data = data;
    j->verified = verified;
    j->status = part_status;
    j->data_ptrs = data_ptrs;
    return m->submit(std::move(j), job);
}

int cec_multi_resilver(cec_multi* m, const uint8_t* chunks, const uint8_t* present,
                       const uint8_t* expected, size_t n_parts, uint8_t* rebuilt,
                       uint8_t* verified, int* part_status, const uint8_t** chunk_ptrs,
                       uint64_t* job) {
    if (!m || !job) return CEC_ERR_INVALID_ARGUMENT;
    if (n_parts && (!chunks || !present || !expected || !rebuilt || !verified || !part_status))
        return CEC_ERR_INVALID_ARGUMENT;
    auto j = std::make_unique<Job>();
    j->kind = Kind::Read;
    j->resilver = true;
    j->n = n_parts;
    j->chunks = chunks;
    j->present = present;
    j->expected = expected;
    j->out_data = rebuilt;
    j->verified = verified;
    j->status = part_status;
    j->data_ptrs = chunk_ptrs;
    return m->submit(std::move(j), job);
}

int cec_multi_verify(cec_multi* m, const uint8_t* chunks, const uint8_t* present,
                     const uint8_t* expected, size_t n_parts, uint8_t* verified, uint64_t* job) {
    if (!m || !job) return CEC_ERR_INVALID_ARGUMENT;
    if (n_parts && (!chunks || !present || !expected || !verified)) return CEC_ERR_INVALID_ARGUMENT;
    auto j = std::make_unique<Job>();
    j->kind = Kind::Read;
    j->verify_only = true;
    j->n = n_parts;
    j->chunks = chunks;
    j->present = present;
    j->expected = expected;
    j->verified = verified;
    return m->submit(std::move(j), job);
}

int cec_multi_wait(cec_multi* m, uint64_t job) {
    if (!m) return CEC_ERR_INVALID_ARGUMENT;
    std::unique_lock<std::mutex> lk(m->mu);
    auto it = m->jobs.find(job);
    if (it == m->jobs.end()) return CEC_ERR_INVALID_ARGUMENT;
    Job* j = it->second.get();
    m->done_cv.wait(lk, [&] { return j->remaining == 0; });
    const int st = j->result;
    if (st != CEC_OK) g_multi_error = j->error;
    m->jobs.erase(it);
    return st;
}

}  // extern "C"
