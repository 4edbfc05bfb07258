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
// its device's NUMA node (hostmem.cpp), then makes its write and read pipelines of `depth` slots
// (pipeline.cpp, CEC_PIPE_EXTERNAL) ONCE, before cec_multi_new returns: nothing creates streams
// or device buffers while another shard's batches run (the round-5 deadlock, profiles/HISTORY.md).
// Read, resilver and verify jobs use the same read pipeline, the mode picked per submit.  A worker
// streams its share batch by batch: caller buffers that are page-locked (cec_host_alloc) are
// DMA'd directly; pageable ones go through the worker's own NUMA-local pinned staging.  Jobs are
// queued and run in submission order, except that a read job flagged CEC_MULTI_AHEAD (a reader's
// retry round: a few parts whose window waits for them) goes ahead of the queued jobs that have
// not started, behind earlier such jobs; a worker keeps its batches in flight across job
// boundaries: with its queue empty it completes batches as their events fire while watching the
// queue, so the next job of a stream is queued behind the batches still running instead of after
// a drain (no bubble).
//
// Read retries keep their verified chunks on the device (file_part.rs:92-107 keeps them in
// memory): the read pipeline's carry pool stashes the verified chunks of every part reported
// TooFewShardsPresent; a job given carry_out gets an id per such part (shard << 20 | entry), and a
// retry job given those ids as carry_in sends each carried part to the shard holding its chunks
// and uploads only its new chunks.
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
#include "pipeline_internal.hpp"

namespace {

thread_local std::string g_multi_error;

// scheduler carry id = shard << kCarryShift | the shard read pipeline's entry
constexpr int kCarryShift = 20;
constexpr int32_t kCarryEntryMask = (int32_t(1) << kCarryShift) - 1;

enum class Kind { Write, Read };

struct Job {
    uint64_t id = 0;
    Kind kind = Kind::Write;
    size_t n = 0;
    unsigned mode = 0;  // read: the read pipeline's mode bits for this job's submits
    bool ahead = false;  // CEC_MULTI_AHEAD: queued ahead of the jobs not yet started
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
    const int32_t* carry_in = nullptr;  // [n] scheduler carry ids (-1 none), nullable
    int32_t* carry_out = nullptr;       // [n] out, nullable
    // per shard, the parts it runs (a job with carry_in: a carried part goes to the shard holding
    // its chunks); empty: the contiguous ranges
    std::vector<std::vector<uint32_t>> share;
    // completion
    size_t remaining = 0;  // parts not yet finished (guarded by cec_multi::mu)
    int result = CEC_OK;
    std::string error;
};

size_t out_chunks(unsigned mode, size_t d, size_t t) {
    return (mode & CEC_READ_VERIFY_ONLY) ? 0 : (mode & CEC_READ_RESILVER) ? t : d;
}

// Pinned staging of one slot (pageable caller buffers only), NUMA-local to the worker.
struct Staging {
    uint8_t* in = nullptr;   // write: [P][d][L]; read: the packed uploaded chunks
    uint8_t* out = nullptr;  // write: [P][p][L]; read: [P][d or d+p][L]
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
    size_t first = 0, n = 0;        // parts [first, first + n) of the job (idx == nullptr)
    const uint32_t* idx = nullptr;  // else: the job's parts idx[0..n)
    bool staged_in = false, staged_out = false;
    bool direct_dig = false;  // write: digests DMA'd straight into the job's buffer
    size_t pos(size_t k) const { return idx ? idx[k] : first + k; }
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
    std::deque<Job*> queue;         // guarded by cec_multi::mu
    std::vector<int32_t> releases;  // carry entries to give back (guarded by cec_multi::mu)
    std::atomic<uint64_t> parts{0};
    std::atomic<uint64_t> pipelines_made{0};
    std::atomic<uint64_t> chunks_uploaded{0};
    std::atomic<uint64_t> chunks_carried{0};
    std::atomic<uint64_t> carry_held{0};
    // worker-thread state
    cec_pipeline* wp = nullptr;
    cec_read_pipeline* rp = nullptr;
    Kind active = Kind::Write;
    std::vector<InFlight> wslots, rslots;
    std::deque<size_t> worder, rorder;  // slots in flight, oldest first
    size_t rnext = 0;                   // read: where the search for a free slot starts
    std::vector<Staging> wstage, rstage;
    std::vector<const uint8_t*> ptrs;  // read: output chunk locations of one batch
    std::vector<int32_t> ids;          // read: carry ids of one batch
    // gathered per-batch arrays of a non-contiguous batch (copied in at submit)
    std::vector<uint8_t> g_present, g_expected;
    std::vector<int32_t> g_carry;
};

}  // namespace

struct cec_multi {
    const cec_codec* codec = nullptr;
    size_t d = 0, p = 0, t = 0, L = 0, P = 0, depth = 0;
    unsigned kinds = 0;  // CEC_MULTI_WRITE | CEC_MULTI_READ
    std::vector<std::unique_ptr<Shard>> shards;
    std::mutex mu;
    std::condition_variable work_cv, done_cv, ready_cv;
    bool stop = false;
    size_t ready = 0;  // workers done making their pipelines (guarded by mu)
    int init_status = CEC_OK;
    std::string init_error;
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

    // ---- the shard's pipelines, made once when the worker starts ----
    int make_pipelines(Shard& s, std::string& err) {
        if (kinds & CEC_MULTI_WRITE) {
            const int st = cec_pipeline_new_ex(codec, L, P, depth, CEC_PIPE_EXTERNAL, &s.wp);
            if (st != CEC_OK) {
                err = std::string("write pipeline: ") + cec_pipeline_last_error();
                return st;
            }
            s.pipelines_made.fetch_add(1);
            s.wslots.assign(depth, InFlight{});
            s.wstage.resize(depth);
        }
        if (kinds & CEC_MULTI_READ) {
            // up to 3 slots more than depth (pipelines hold at most 16) kept for CEC_MULTI_AHEAD
            // batches: a retry round need not wait for a window's batch to free a slot, and the
            // rounds of several windows run together (each is one SHA-256 chain long)
            const size_t rd = read_slots();
            const int st = cec_read_pipeline_new_ex(codec, L, P, rd,
                                                    CEC_PIPE_EXTERNAL | CEC_READ_CARRY, &s.rp);
            if (st != CEC_OK) {
                err = std::string("read pipeline: ") + cec_pipeline_last_error();
                return st;
            }
            s.pipelines_made.fetch_add(1);
            for (size_t a = depth; a < rd; ++a) {
                const int pst = cec::read_pipeline_priority_slot(s.rp, a);
                if (pst != CEC_OK) {
                    err = std::string("read pipeline AHEAD slot: ") + cec_pipeline_last_error();
                    return pst;
                }
            }
            s.rslots.assign(rd, InFlight{});
            s.rstage.resize(rd);
        }
        return CEC_OK;
    }

    // ---- per-shard work ----
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
        const size_t W = out_chunks(job->mode, d, t);  // output chunks per part
        int st = cec_read_pipeline_wait(s.rp, slot, &data, &ver, &status, &got);
        if (st == CEC_OK && W) {
            s.ptrs.resize(f.n * W);
            st = cec_read_pipeline_data_chunks(s.rp, slot, s.ptrs.data(), s.ptrs.size());
        }
        // a read job given carry_out takes its parts' carry entries (the others go back when the
        // slot is submitted again)
        if (st == CEC_OK && job->carry_out) {
            s.ids.assign(f.n, -1);
            st = cec_read_pipeline_carry_ids(s.rp, slot, s.ids.data(), s.ids.size());
            for (size_t k = 0; st == CEC_OK && k < f.n; ++k)
                job->carry_out[f.pos(k)] =
                    s.ids[k] < 0 ? -1 : int32_t(s.index << kCarryShift) | s.ids[k];
        }
        std::string err = st == CEC_OK ? std::string() : cec_pipeline_last_error();
        if (st == CEC_OK) {
            for (size_t k = 0; k < f.n; ++k) {
                std::memcpy(job->verified + f.pos(k) * t, ver + k * t, t);
                if (job->status) job->status[f.pos(k)] = status[k];
            }
        }
        if (st == CEC_OK && W) {
            const bool staged = f.staged_in || f.staged_out;
            parallel_for(f.n, staged ? f.n * W * L : 0, [&](size_t k) {
                for (size_t j = 0; j < W; ++j) {
                    const size_t q = f.pos(k) * W + j;
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
        s.carry_held.store(cec_read_pipeline_carry_held(s.rp), std::memory_order_relaxed);
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

    // Carry entries the caller gave back (cec_multi_carry_release), applied on the worker: the
    // pipeline is the worker's alone.
    void apply_releases(Shard& s) {
        std::vector<int32_t> ids;
        {
            std::lock_guard<std::mutex> lk(mu);
            ids.swap(s.releases);
        }
        if (ids.empty() || !s.rp) return;
        for (int32_t id : ids) (void)cec_read_pipeline_carry_release(s.rp, id);
        s.carry_held.store(cec_read_pipeline_carry_held(s.rp), std::memory_order_relaxed);
    }

    size_t read_slots() const { return std::min<size_t>(depth + 3, 16); }

    // Finish every batch in flight that is complete, in any order (a retry round finishes while
    // older windows' batches still run, and its job completes then); never blocks.
    void finish_done(Shard& s) {
        for (size_t i = 0; i < s.worder.size();) {
            const size_t slot = s.worder[i];
            if (cec_pipeline_query(s.wp, slot) == 1) finish_write(s, slot);  // erases it
            else ++i;
        }
        for (size_t i = 0; i < s.rorder.size();) {
            const size_t slot = s.rorder[i];
            if (cec_read_pipeline_query(s.rp, slot) == 1) finish_read(s, slot);  // erases it
            else ++i;
        }
    }

    // A read slot for the next batch: one with no batch in flight -- an AHEAD slot first for an
    // AHEAD job, which may also take a depth slot; the others never take an AHEAD slot.  None
    // free: the complete batches are finished (their jobs complete as soon as their batches
    // are done, not behind older ones) and the slots polled again 50 us later.
    int read_slot(Shard& s, bool ahead, size_t* slot, uint8_t** c, uint8_t** pr, uint8_t** ex) {
        const size_t n = s.rslots.size(), nd = std::min(n, depth);
        for (;;) {
            finish_done(s);
            size_t pick = n;
            for (size_t a = nd; ahead && pick == n && a < n; ++a)
                if (!s.rslots[a].job) pick = a;
            for (size_t k = 0; pick == n && k < nd; ++k) {
                const size_t i = (s.rnext + k) % nd;
                if (!s.rslots[i].job) pick = i;
            }
            if (pick < n) {
                if (pick < nd) s.rnext = (pick + 1) % nd;
                *slot = pick;
                return cec::read_pipeline_acquire_slot(s.rp, pick, c, pr, ex);
            }
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    }

    void run_write(Shard& s, Job* job, size_t lo, size_t hi) {
        if (s.active != Kind::Write) drain_read(s);
        s.active = Kind::Write;
        const size_t dw = d * L, pw = p * L;
        for (size_t first = lo; first < hi; first += P) {
            const size_t n = std::min(P, hi - first);
            size_t slot = 0;
            uint8_t* unused = nullptr;
            int st = cec_pipeline_acquire(s.wp, &slot, &unused);
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

    // The shard's parts of a read job: the list of a carried job, else [lo, hi).
    void run_read(Shard& s, Job* job, size_t lo, size_t hi) {
        apply_releases(s);
        if (s.active != Kind::Read) drain_write(s);
        s.active = Kind::Read;
        const std::vector<uint32_t>* list = job->share.empty() ? nullptr : &job->share[s.index];
        const size_t count = list ? list->size() : hi - lo;
        const size_t W = out_chunks(job->mode, d, t);
        const size_t cw = t * L, dw = W * L;  // input / output bytes per part
        for (size_t at = 0; at < count; at += P) {
            const size_t n = std::min(P, count - at);
            size_t slot = 0;
            uint8_t *c = nullptr, *pr = nullptr, *ex = nullptr;
            int st = read_slot(s, job->ahead, &slot, &c, &pr, &ex);
            if (st != CEC_OK) {
                finish_parts(job, count - at, st, cec_pipeline_last_error());
                return;
            }
            InFlight f;
            f.job = job;
            f.n = n;
            const uint32_t* ix = list ? list->data() + at : nullptr;
            const bool contiguous = !ix || size_t(ix[n - 1] - ix[0]) == n - 1;
            f.first = ix ? ix[0] : lo + at;
            f.idx = contiguous ? nullptr : ix;
            // the batch's flags and digests: the job's own rows, or gathered for a list batch
            const uint8_t* prs = job->present + f.first * t;
            const uint8_t* exs = job->expected + f.first * t * 32;
            if (!contiguous) {
                s.g_present.resize(n * t);
                s.g_expected.resize(n * t * 32);
                for (size_t k = 0; k < n; ++k) {
                    std::memcpy(s.g_present.data() + k * t, job->present + f.pos(k) * t, t);
                    std::memcpy(s.g_expected.data() + k * t * 32,
                                job->expected + f.pos(k) * t * 32, t * 32);
                }
                prs = s.g_present.data();
                exs = s.g_expected.data();
            }
            // carry ids of this shard's entries (routing sent every carried part here)
            const int32_t* cin = nullptr;
            if (job->carry_in) {
                s.g_carry.assign(n, -1);
                for (size_t k = 0; k < n; ++k) {
                    const int32_t id = job->carry_in[f.pos(k)];
                    if (id >= 0) {
                        s.g_carry[k] = id & kCarryEntryMask;
                        cin = s.g_carry.data();
                    }
                }
            }
            auto carried = [&](size_t k) { return cin && cin[k] >= 0; };
            auto uploaded = [&](size_t k, size_t i) {
                const uint8_t fl = prs[k * t + i];
                return fl && !(carried(k) && fl == CEC_PRESENT_VERIFIED);
            };
            const uint8_t* src = job->chunks + f.first * cw;
            uint8_t* dst = W ? job->out_data + f.first * dw : nullptr;
            f.staged_in = !contiguous || !cec::pinned_range(src, n * cw);
            f.staged_out = W && (!contiguous || !cec::pinned_range(dst, n * dw));
            Staging& sg = s.rstage[slot];
            if (f.staged_in || f.staged_out) {
                // every depth slot at once (see run_write); an AHEAD slot's when it is used
                hipError_t e = hipSuccess;
                for (size_t i = 0; i < s.rstage.size(); ++i)
                    if (e == hipSuccess && (i < depth || i == slot))
                        e = s.rstage[i].reserve(f.staged_in ? P * cw : 0,
                                                f.staged_out ? P * dw : 0, s.device);
                if (e != hipSuccess) {
                    finish_parts(job, count - at, CEC_ERR_OUT_OF_MEMORY,
                                 std::string("multi staging: ") + hipGetErrorString(e));
                    return;
                }
            }
            size_t up = 0, kept = 0;
            for (size_t k = 0; k < n; ++k)
                for (size_t i = 0; i < t; ++i) {
                    up += uploaded(k, i) ? 1 : 0;
                    kept += carried(k) && prs[k * t + i] == CEC_PRESENT_VERIFIED ? 1 : 0;
                }
            cec_read_submit a{src, prs, exs, n, f.staged_out ? sg.out : dst, cin, job->mode};
            if (f.staged_in) {
                // only the uploaded chunks are staged, packed back to back (part by part, index
                // ascending): the batch then goes up as one copy (CEC_SUBMIT_PACKED)
                std::vector<size_t> at_k(n + 1, 0);
                for (size_t k = 0; k < n; ++k) {
                    size_t m = 0;
                    for (size_t i = 0; i < t; ++i) m += uploaded(k, i) ? 1 : 0;
                    at_k[k + 1] = at_k[k] + m;
                }
                uint8_t* to = sg.in;
                parallel_for(n, n * cw, [&](size_t k) {
                    size_t q = at_k[k];
                    const uint8_t* from = job->chunks + f.pos(k) * cw;
                    for (size_t i = 0; i < t; ++i)
                        if (uploaded(k, i)) std::memcpy(to + (q++) * L, from + i * L, L);
                });
                a.chunks = sg.in;
                a.flags |= CEC_SUBMIT_PACKED;
            }
            st = cec_read_pipeline_submit_ex(s.rp, slot, &a);
            if (st != CEC_OK) {
                finish_parts(job, count - at, st, cec_pipeline_last_error());
                return;
            }
            s.chunks_uploaded.fetch_add(up, std::memory_order_relaxed);
            s.chunks_carried.fetch_add(kept, std::memory_order_relaxed);
            s.carry_held.store(cec_read_pipeline_carry_held(s.rp), std::memory_order_relaxed);
            s.rslots[slot] = f;
            s.rorder.push_back(slot);
        }
    }

    void worker(Shard& s) {
        s.bound = cec::bind_thread_to_device_node(s.device);
        std::string err;
        int st = hipSetDevice(s.device) == hipSuccess ? CEC_OK : CEC_ERR_HIP;
        if (st != CEC_OK) err = "hipSetDevice failed";
        if (st == CEC_OK) st = make_pipelines(s, err);
        {
            std::lock_guard<std::mutex> lk(mu);
            ++ready;
            if (st != CEC_OK && init_status == CEC_OK) {
                init_status = st;
                init_error = err;
            }
        }
        ready_cv.notify_all();
        const size_t G = shards.size();
        for (;;) {
            if (st != CEC_OK) break;  // cec_multi_new fails and frees the scheduler
            Job* job = nullptr;
            {
                std::unique_lock<std::mutex> lk(mu);
                // Nothing queued: complete batches as they finish (polling their events, 100 us
                // apart) while watching the queue, so a job submitted meanwhile (the next segment
                // of a stream) is queued behind the batches still running, never behind a drain;
                // sleep on the queue alone only when nothing is in flight.
                while (s.queue.empty() && in_flight(s)) {
                    lk.unlock();
                    finish_done(s);
                    lk.lock();
                    if (!s.queue.empty() || !in_flight(s)) break;
                    work_cv.wait_for(lk, std::chrono::microseconds(100));
                }
                work_cv.wait(lk, [&] { return stop || !s.queue.empty() || !s.releases.empty(); });
                if (s.queue.empty() && !stop) {  // carry ids given back while idle
                    lk.unlock();
                    apply_releases(s);
                    continue;
                }
                if (s.queue.empty()) break;  // stop requested and nothing left
                job = s.queue.front();
                s.queue.pop_front();
            }
            const size_t lo = job->n * s.index / G, hi = job->n * (s.index + 1) / G;
            if (job->kind == Kind::Write) run_write(s, job, lo, hi);
            else run_read(s, job, lo, hi);
        }
        drain(s);  // the pipelines are freed by ~cec_multi, one shard after another
    }

    // A shard's pipelines and staging, freed on the destroying thread once every worker has
    // exited: no HIP stream, event or buffer is destroyed while another shard's are (two shards
    // of one device tearing down their priority streams at once ended one run of the GPU suite
    // in an abort inside cec_multi_free, cause not isolated; the creation side is the round-5
    // deadlock, profiles/HISTORY.md).
    static void free_shard(Shard& s) {
        if (s.wp) cec_pipeline_free(s.wp);
        if (s.rp) cec_read_pipeline_free(s.rp);
        for (auto& sg : s.wstage) sg.release();
        for (auto& sg : s.rstage) sg.release();
        s.wp = nullptr;
        s.rp = nullptr;
    }

    // The shard of part k under the contiguous split of an n-part job.
    size_t range_shard(size_t k, size_t n) const {
        const size_t G = shards.size();
        size_t g = k * G / n;
        while (g + 1 < G && n * (g + 1) / G <= k) ++g;
        while (g > 0 && n * g / G > k) --g;
        return g;
    }

    int submit(std::unique_ptr<Job> job, uint64_t* id) {
        const size_t G = shards.size();
        if (job->carry_in && job->n) {
            // a carried part runs on the shard whose pool holds its chunks; the others as usual
            job->share.assign(G, {});
            for (size_t k = 0; k < job->n; ++k) {
                const int32_t c = job->carry_in[k];
                const size_t g = c >= 0 ? size_t(c >> kCarryShift) : range_shard(k, job->n);
                if (g >= G) {
                    g_multi_error = "carry id of no shard of this scheduler";
                    return CEC_ERR_INVALID_ARGUMENT;
                }
                job->share[g].push_back(uint32_t(k));
            }
        }
        std::lock_guard<std::mutex> lk(mu);
        job->id = next_id++;
        job->remaining = job->n;
        *id = job->id;
        Job* raw = job.get();
        jobs.emplace(raw->id, std::move(job));
        if (raw->n == 0) return CEC_OK;
        // Only shards with parts get the job: once the others have finished, the caller may free
        // it, and a shard popping it later would read freed memory.
        for (size_t g = 0; g < G; ++g) {
            const bool any = raw->share.empty() ? raw->n * (g + 1) / G > raw->n * g / G
                                                : !raw->share[g].empty();
            if (!any) continue;
            std::deque<Job*>& q = shards[g]->queue;
            auto at = q.end();
            if (raw->ahead)  // behind the AHEAD jobs already queued, ahead of the others
                at = std::find_if(q.begin(), q.end(), [](const Job* x) { return !x->ahead; });
            q.insert(at, raw);
        }
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
        for (auto& s : shards) free_shard(*s);
    }
};

extern "C" {

const char* cec_multi_last_error(void) { return g_multi_error.c_str(); }

int cec_multi_new_ex(const cec_codec* codec, size_t chunk_len, size_t parts_per_batch,
                     size_t depth, const int* devices, size_t n_devices, unsigned flags,
                     cec_multi** out) {
    if (!codec || !out || chunk_len == 0 || parts_per_batch == 0 || depth == 0 || depth > 16 ||
        !devices || n_devices == 0 || n_devices > 64 || flags == 0 ||
        (flags & ~unsigned(CEC_MULTI_WRITE | CEC_MULTI_READ)))
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
    m->kinds = flags;
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
    // every worker has made its pipelines (or failed) before the scheduler is handed out
    int st = CEC_OK;
    {
        std::unique_lock<std::mutex> lk(m->mu);
        m->ready_cv.wait(lk, [&] { return m->ready == m->shards.size(); });
        st = m->init_status;
        if (st != CEC_OK) g_multi_error = m->init_error;
    }
    if (st != CEC_OK) return st;  // m's destructor stops and joins the workers
    *out = m.release();
    return CEC_OK;
}

int cec_multi_new(const cec_codec* codec, size_t chunk_len, size_t parts_per_batch, size_t depth,
                  const int* devices, size_t n_devices, cec_multi** out) {
    return cec_multi_new_ex(codec, chunk_len, parts_per_batch, depth, devices, n_devices,
                            CEC_MULTI_WRITE | CEC_MULTI_READ, out);
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

int cec_multi_shard_stats(cec_multi* m, size_t g, cec_multi_stats* out) {
    if (!m || !out || g >= m->shards.size()) return CEC_ERR_INVALID_ARGUMENT;
    const Shard& s = *m->shards[g];
    out->device = s.device;
    out->numa_node = s.numa;
    out->parts = s.parts.load();
    out->pipelines_made = s.pipelines_made.load();
    out->chunks_uploaded = s.chunks_uploaded.load();
    out->chunks_carried = s.chunks_carried.load();
    out->carry_held = s.carry_held.load();
    return CEC_OK;
}

int cec_multi_encode_hash(cec_multi* m, const uint8_t* data, size_t n_parts, uint8_t* parity,
                          uint8_t* digests, uint64_t* job) {
    if (!m || !job || (n_parts && (!data || !parity || !digests))) return CEC_ERR_INVALID_ARGUMENT;
    if (!(m->kinds & CEC_MULTI_WRITE)) {
        g_multi_error = "scheduler made without CEC_MULTI_WRITE";
        return CEC_ERR_INVALID_ARGUMENT;
    }
    auto j = std::make_unique<Job>();
    j->kind = Kind::Write;
    j->n = n_parts;
    j->data = data;
    j->parity = parity;
    j->digests = digests;
    return m->submit(std::move(j), job);
}

int cec_multi_read_carry(cec_multi* m, const uint8_t* chunks, const uint8_t* present,
                         const uint8_t* expected, size_t n_parts, uint8_t* data, uint8_t* verified,
                         int* part_status, const uint8_t** data_ptrs, unsigned flags,
                         const int32_t* carry_in, int32_t* carry_out, uint64_t* job) {
    if (!m || !job || (flags & ~unsigned(CEC_READ_REBUILT_ONLY | CEC_MULTI_AHEAD)))
        return CEC_ERR_INVALID_ARGUMENT;
    if (n_parts && (!chunks || !present || !expected || !data || !verified || !part_status))
        return CEC_ERR_INVALID_ARGUMENT;
    if ((flags & CEC_READ_REBUILT_ONLY) && !data_ptrs) return CEC_ERR_INVALID_ARGUMENT;
    if (!(m->kinds & CEC_MULTI_READ)) {
        g_multi_error = "scheduler made without CEC_MULTI_READ";
        return CEC_ERR_INVALID_ARGUMENT;
    }
    auto j = std::make_unique<Job>();
    j->kind = Kind::Read;
    j->n = n_parts;
    j->mode = flags & CEC_READ_REBUILT_ONLY;
    j->ahead = (flags & CEC_MULTI_AHEAD) != 0;
    j->chunks = chunks;
    j->present = present;
    j->expected = expected;
    j->out_data = data;
    j->verified = verified;
    j->status = part_status;
    j->data_ptrs = data_ptrs;
    j->carry_in = carry_in;
    j->carry_out = carry_out;
    if (carry_out)
        for (size_t k = 0; k < n_parts; ++k) carry_out[k] = -1;
    return m->submit(std::move(j), job);
}

int cec_multi_read(cec_multi* m, const uint8_t* chunks, const uint8_t* present,
                   const uint8_t* expected, size_t n_parts, uint8_t* data, uint8_t* verified,
                   int* part_status, const uint8_t** data_ptrs, unsigned flags, uint64_t* job) {
    return cec_multi_read_carry(m, chunks, present, expected, n_parts, data, verified, part_status,
                                data_ptrs, flags, nullptr, nullptr, job);
}

int cec_multi_carry_release(cec_multi* m, int32_t id) {
    if (!m || id < 0 || size_t(id >> kCarryShift) >= m->shards.size())
        return CEC_ERR_INVALID_ARGUMENT;
    {
        std::lock_guard<std::mutex> lk(m->mu);
        m->shards[size_t(id >> kCarryShift)]->releases.push_back(id & kCarryEntryMask);
    }
    m->work_cv.notify_all();
    return CEC_OK;
}

int cec_multi_resilver(cec_multi* m, const uint8_t* chunks, const uint8_t* present,
                       const uint8_t* expected, size_t n_parts, uint8_t* rebuilt,
                       uint8_t* verified, int* part_status, const uint8_t** chunk_ptrs,
                       uint64_t* job) {
    if (!m || !job) return CEC_ERR_INVALID_ARGUMENT;
    if (n_parts && (!chunks || !present || !expected || !rebuilt || !verified || !part_status))
        return CEC_ERR_INVALID_ARGUMENT;
    if (!(m->kinds & CEC_MULTI_READ)) {
        g_multi_error = "scheduler made without CEC_MULTI_READ";
        return CEC_ERR_INVALID_ARGUMENT;
    }
    auto j = std::make_unique<Job>();
    j->kind = Kind::Read;
    j->mode = CEC_READ_RESILVER;
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
    if (!(m->kinds & CEC_MULTI_READ)) {
        g_multi_error = "scheduler made without CEC_MULTI_READ";
        return CEC_ERR_INVALID_ARGUMENT;
    }
    auto j = std::make_unique<Job>();
    j->kind = Kind::Read;
    j->mode = CEC_READ_VERIFY_ONLY;
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

int cec_multi_query(cec_multi* m, uint64_t job) {
    if (!m) return CEC_ERR_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> lk(m->mu);
    auto it = m->jobs.find(job);
    if (it == m->jobs.end()) return CEC_ERR_INVALID_ARGUMENT;
    return it->second->remaining == 0 ? 1 : 0;
}

}  // extern "C"
