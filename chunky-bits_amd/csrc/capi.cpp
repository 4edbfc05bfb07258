// capi.cpp — implementation of include/chunky_ec.h.
//
// Host responsibilities only: argument checks in the crate's order, coding/decode matrices
// (tiny), erasure-pattern grouping, staging, and kernel launches.  Every shard byte is
// processed by the gfx950 kernels in kernels.hip; there is no CPU compute path.
#include "chunky_ec.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "gf256.hpp"
#include "hostmem.hpp"
#include "kernels.hpp"
#include "knobs.hpp"

using namespace cec;

namespace {

thread_local std::string g_last_error;

int hip_fail(hipError_t e, const char* what) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return e == hipErrorOutOfMemory ? CEC_ERR_OUT_OF_MEMORY : CEC_ERR_HIP;
}

#define HIP_TRY(expr)                                        \
    do {                                                     \
        hipError_t _e = (expr);                              \
        if (_e != hipSuccess) return hip_fail(_e, #expr);    \
    } while (0)

#define CEC_TRY(expr)              \
    do {                           \
        int _s = (expr);           \
        if (_s != CEC_OK) return _s; \
    } while (0)

int current_device(int* dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        g_last_error = "no HIP device";
        return CEC_ERR_NO_DEVICE;
    }
    HIP_TRY(hipGetDevice(dev));
    return CEC_OK;
}

constexpr size_t kChunkAlign = 256;
size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

bool aligned16(const void* p, size_t a, size_t b) {
    return (reinterpret_cast<uintptr_t>(p) % 16 == 0) && (a % 16 == 0) && (b % 16 == 0);
}

// ------------------------------------------------------------------------------------------
// Small per-launch device buffers (decode pattern records, verify item lists, flag arrays).
//
// Not hipMallocAsync / hipFreeAsync: with them, read and resilver batches came back with chunks
// the decode had not (re)written (round 2: the C++ mirror's batched verify/resilver and streamed
// reads, 4 of 4 runs).  tools/repro_free_async.hip shows why, with no engine code: on this
// ROCm, memory hipMallocAsync maps fresh (the default pool trimmed) is, on some boxes and every
// other allocation, zeroed AFTER the stream's first writes to it -- a kernel that filled it reads
// zeros on its later passes, and metadata words uploaded into it read as zeros (round 2's
// fork/join read shape loses whole outputs the same way, with the free queued behind the work
// or only after a sync).  hipMalloc'd memory never showed it (profiles/r3_repro/).
// Instead a process-wide pool of device buffers, each with a page-locked host mirror
// and an event: a buffer is handed out only once the event recorded after its last use has
// completed, the words go up from the mirror (a truly asynchronous copy, no host lifetime to
// manage), and its release records the event on the stream of the work that used it.
// ------------------------------------------------------------------------------------------
class ScratchPool {
   public:
    struct Buf {
        int device = 0;
        uint8_t* dev = nullptr;
        uint8_t* host = nullptr;  // page-locked mirror of the same size
        size_t cap = 0;
        hipEvent_t done = nullptr;
        bool in_use = false;   // handed out, release not called yet
        bool pending = false;  // released: `done` marks the end of its last use
    };

    // A buffer of >= bytes on `device` whose last use has completed.
    hipError_t acquire(int device, size_t bytes, Buf** out) {
        std::unique_lock<std::mutex> lk(mu_);
        Buf* best = nullptr;
        for (Buf* b : bufs_) {
            if (b->device != device || b->in_use) continue;
            if (b->pending) {
                const hipError_t q = hipEventQuery(b->done);
                if (q == hipErrorNotReady) {
                    (void)hipGetLastError();
                    continue;
                }
                if (q != hipSuccess) {  // unknown state (e.g. its stream was destroyed): wait
                    (void)hipGetLastError();
                    if (hipEventSynchronize(b->done) != hipSuccess) {
                        (void)hipGetLastError();
                        continue;  // never reused
                    }
                }
                b->pending = false;
            }
            if (b->cap >= bytes && (!best || b->cap < best->cap)) best = b;
        }
        if (best) {
            best->in_use = true;
            *out = best;
            return hipSuccess;
        }
        // None free: a new buffer, made outside the lock (allocations are slow).
        lk.unlock();
        auto* b = new Buf();
        b->device = device;
        b->cap = std::max<size_t>(size_t(64) << 10, size_t(1) << (64 - __builtin_clzll(bytes | 1)));
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&b->dev), b->cap);
        if (e == hipSuccess)
            e = hipHostMalloc(reinterpret_cast<void**>(&b->host), b->cap, hipHostMallocDefault);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&b->done, hipEventDisableTiming);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            if (b->dev) (void)hipFree(b->dev);
            if (b->host) (void)hipHostFree(b->host);
            delete b;
            return e;
        }
        b->in_use = true;
        lk.lock();
        bufs_.push_back(b);
        *out = b;
        return hipSuccess;
    }

    // The work that uses `b` has been queued on `s`: reusable once it completes.
    void release(Buf* b, hipStream_t s) {
        const hipError_t e = hipEventRecord(b->done, s);
        if (e != hipSuccess) {  // no marker: wait for the stream instead
            (void)hipGetLastError();
            (void)hipStreamSynchronize(s);
            (void)hipGetLastError();
        }
        std::lock_guard<std::mutex> lk(mu_);
        b->pending = e == hipSuccess;
        b->in_use = false;
    }

   private:
    std::mutex mu_;
    std::vector<Buf*> bufs_;  // never freed: the pool lives as long as the process
};

ScratchPool& scratch_pool() {
    static auto* pool = new ScratchPool();
    return *pool;
}

// One scratch buffer for the launches of one call: acquire, fill / upload, launch, and the
// destructor releases it on the stream those launches went to (error paths included).
class Scratch {
   public:
    Scratch() = default;
    Scratch(const Scratch&) = delete;
    Scratch& operator=(const Scratch&) = delete;
    ~Scratch() {
        if (buf_) scratch_pool().release(buf_, stream_);
    }
    int acquire(size_t bytes, hipStream_t s) {
        int dev = 0;
        CEC_TRY(current_device(&dev));
        HIP_TRY(scratch_pool().acquire(dev, bytes, &buf_));
        stream_ = s;
        return CEC_OK;
    }
    uint8_t* dev() const { return buf_->dev; }
    uint8_t* host() const { return buf_->host; }

   private:
    ScratchPool::Buf* buf_ = nullptr;
    hipStream_t stream_ = nullptr;
};

// Upload `words` into `sc` (acquired here) on stream s; *dptr = their device copy.
int upload_words(const std::vector<uint32_t>& words, hipStream_t s, Scratch& sc, uint32_t** dptr) {
    const size_t bytes = std::max<size_t>(words.size() * sizeof(uint32_t), 4);
    CEC_TRY(sc.acquire(bytes, s));
    std::memcpy(sc.host(), words.data(), words.size() * sizeof(uint32_t));
    HIP_TRY(hipMemcpyAsync(sc.dev(), sc.host(), words.size() * sizeof(uint32_t),
                           hipMemcpyHostToDevice, s));
    *dptr = reinterpret_cast<uint32_t*>(sc.dev());
    return CEC_OK;
}

// ------------------------------------------------------------------------------------------
// Staging contexts for the host-buffer API: a stream + a device buffer, leased per call from a
// bounded per-device pool (not thread_local: the reference calls the crate from tokio's
// blocking pool, whose threads come and go, file_part.rs:128,161 / any.rs:19-24, so per-thread
// resources would leak with every retired thread).  At most kMaxIdleCtx contexts per device
// stay alive between calls, holding at most CEC_IDLE_STAGING_MIB (default 1 GiB) of device
// buffers together; cec_release_cached() frees the idle ones.
// ------------------------------------------------------------------------------------------
struct StageCtx {
    int device = 0;
    hipStream_t stream = nullptr;
    uint8_t* dbuf = nullptr;
    size_t dcap = 0;
    void release_buffer() {
        if (dbuf) (void)hipFree(dbuf);
        dbuf = nullptr;
        dcap = 0;
    }
    void destroy() {  // on `device` (callers set it)
        if (stream) {
            (void)hipStreamSynchronize(stream);
            (void)hipStreamDestroy(stream);
        }
        stream = nullptr;
        release_buffer();
    }
};

// Stream + device staging of at least device_bytes (grown, never shrunk while leased).
int ctx_reserve(StageCtx& c, size_t device_bytes) {
    if (!c.stream) HIP_TRY(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    if (c.dcap < device_bytes) {
        c.release_buffer();
        const size_t cap = round_up(std::max<size_t>(device_bytes, 1 << 20), 1 << 20);
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c.dbuf), cap));
        c.dcap = cap;
    }
    return CEC_OK;
}

constexpr size_t kMaxIdleCtx = 8;
// Device bytes idle contexts may hold per device (knobs().idle_staging_bytes, the
// CEC_IDLE_STAGING_MIB knob, default 1 GiB).  Bounding the total (not each buffer) keeps a
// steady stream of large per-call requests (e.g. RS(10,4) at 8 MiB chunks: 112 MiB per part)
// from paying a hipMalloc + a device-synchronizing hipFree on every call.

class CtxPool {
   public:
    // An idle context of `device` whose buffer already holds `device_bytes` (the smallest such),
    // else the one with the largest buffer (grown by ctx_reserve), else a new one.
    std::unique_ptr<StageCtx> take(int device, size_t device_bytes) {
        std::lock_guard<std::mutex> lk(mu_);
        auto& v = idle_[device];
        if (v.empty()) {
            auto c = std::make_unique<StageCtx>();
            c->device = device;
            return c;
        }
        size_t best = 0;
        for (size_t i = 1; i < v.size(); ++i) {
            const size_t a = v[i]->dcap, b = v[best]->dcap;
            const bool fits_a = a >= device_bytes, fits_b = b >= device_bytes;
            if (fits_a != fits_b ? fits_a : (fits_a ? a < b : a > b)) best = i;
        }
        auto c = std::move(v[best]);
        v.erase(v.begin() + std::ptrdiff_t(best));
        idle_bytes_[device] -= c->dcap;
        return c;
    }
    // The caller's current device is the context's (leases never cross devices).
    void give(std::unique_ptr<StageCtx> c) {
        if (!c) return;
        if (c->stream) (void)hipStreamSynchronize(c->stream);
        bool drop_buffer = false;
        {
            std::lock_guard<std::mutex> lk(mu_);
            auto& v = idle_[c->device];
            if (v.size() < kMaxIdleCtx) {
                size_t& held = idle_bytes_[c->device];
                if (held + c->dcap <= knobs().idle_staging_bytes) {
                    held += c->dcap;
                    v.push_back(std::move(c));
                    return;
                }
                drop_buffer = true;  // over the budget: keep the stream, free the buffer below
            }
        }
        if (!drop_buffer) {
            c->destroy();
            return;
        }
        c->release_buffer();
        std::lock_guard<std::mutex> lk(mu_);
        auto& v = idle_[c->device];
        if (v.size() < kMaxIdleCtx) v.push_back(std::move(c));
        // (else another thread filled the pool meanwhile: c's stream is destroyed with it)
    }

    // Destroys the idle contexts of `device` (every device if < 0): their streams and device
    // buffers are freed; leased contexts are untouched.  Returns the device bytes released.
    size_t trim(int device) {
        std::vector<std::unique_ptr<StageCtx>> out;
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (auto& [dev, v] : idle_) {
                if (device >= 0 && dev != device) continue;
                for (auto& c : v) out.push_back(std::move(c));
                v.clear();
                idle_bytes_[dev] = 0;
            }
        }
        size_t bytes = 0;
        int cur = 0;
        const bool have_cur = hipGetDevice(&cur) == hipSuccess;
        for (auto& c : out) {
            bytes += c->dcap;
            if (hipSetDevice(c->device) == hipSuccess) c->destroy();
            (void)hipGetLastError();
        }
        if (have_cur) (void)hipSetDevice(cur);
        return bytes;
    }

   private:
    std::mutex mu_;
    std::map<int, std::vector<std::unique_ptr<StageCtx>>> idle_;
    std::map<int, size_t> idle_bytes_;
};

// Leaked on purpose: destroying HIP objects from a static destructor races the runtime's own
// teardown at process exit.
CtxPool& ctx_pool() {
    static CtxPool* pool = new CtxPool();
    return *pool;
}

// RAII lease of a staging context on the current device.
class CtxLease {
   public:
    CtxLease() = default;
    CtxLease(const CtxLease&) = delete;
    CtxLease& operator=(const CtxLease&) = delete;
    ~CtxLease() { ctx_pool().give(std::move(c_)); }
    int acquire(size_t device_bytes) {
        int dev = 0;
        CEC_TRY(current_device(&dev));
        c_ = ctx_pool().take(dev, device_bytes);
        return ctx_reserve(*c_, device_bytes);
    }
    StageCtx* operator->() { return c_.get(); }

   private:
    std::unique_ptr<StageCtx> c_;
};

// Erasure-pattern key: present bitset (<= 256 shards) + data_only.
struct PatternKey {
    std::array<uint64_t, 4> bits{};
    bool data_only = false;
    bool operator<(const PatternKey& o) const {
        if (bits != o.bits) return bits < o.bits;
        return data_only < o.data_only;
    }
};

}  // namespace

// ------------------------------------------------------------------------------------------
// Codec
// ------------------------------------------------------------------------------------------
struct cec_codec {
    size_t d = 0, p = 0;
    ByteMatrix m;                  // (d+p) x d
    std::vector<uint32_t> enc;     // pattern record: parity rows over the d data chunks
    bool bs = false;               // parity rows = a compiled bit-sliced shape (bs_encode_matches)
    std::mutex mu;
    std::unordered_map<int, uint32_t*> dev_enc;  // encode record per device
    // Decode records, least recently used first out once kDecCacheCap patterns are cached (every
    // 1..4-erasure pattern of RS(10,4), both modes, is 2 940).
    static constexpr size_t kDecCacheCap = 4096;
    using Record = std::shared_ptr<const std::vector<uint32_t>>;
    std::list<PatternKey> dec_lru;  // front = most recent
    std::map<PatternKey, std::pair<Record, std::list<PatternKey>::iterator>> dec_cache;

    ~cec_codec() {
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) return;
        for (auto& kv : dev_enc) {
            if (hipSetDevice(kv.first) == hipSuccess) (void)hipFree(kv.second);
        }
        (void)hipSetDevice(cur);
    }

    // Device copy of the encode record on the current device.
    int encode_record(uint32_t** out) {
        int dev = 0;
        CEC_TRY(current_device(&dev));
        std::lock_guard<std::mutex> lk(mu);
        auto it = dev_enc.find(dev);
        if (it != dev_enc.end()) {
            *out = it->second;
            return CEC_OK;
        }
        uint32_t* ptr = nullptr;
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&ptr), enc.size() * sizeof(uint32_t)));
        HIP_TRY(hipMemcpy(ptr, enc.data(), enc.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        dev_enc[dev] = ptr;
        *out = ptr;
        return CEC_OK;
    }

    // Decode record for a present set: inputs = first d present chunks (the crate's choice,
    // reconstruct_internal), outputs = missing data (+ missing parity unless data_only).
    // Missing data rows = rows of inv(M[valid]); missing parity rows = M[r] * inv(M[valid]),
    // i.e. the crate's "recompute parity from the rebuilt data" folded into one pass
    // (identical bytes: GF(2^8) arithmetic is exact).
    std::shared_ptr<const std::vector<uint32_t>> decode_record(const PatternKey& key) {
        std::lock_guard<std::mutex> lk(mu);
        auto it = dec_cache.find(key);
        if (it != dec_cache.end()) {
            dec_lru.splice(dec_lru.begin(), dec_lru, it->second.second);
            return it->second.first;
        }
        const size_t t = d + p;
        std::vector<uint32_t> in_idx, out_idx;
        std::vector<size_t> miss_par;
        for (size_t i = 0; i < t; ++i) {
            const bool present = (key.bits[i / 64] >> (i % 64)) & 1;
            if (present) {
                if (in_idx.size() < d) in_idx.push_back(uint32_t(i));
            } else if (i < d) {
                out_idx.push_back(uint32_t(i));
            } else if (!key.data_only) {
                miss_par.push_back(i);
            }
        }
        for (size_t i : miss_par) out_idx.push_back(uint32_t(i));
        ByteMatrix sub(d, d), dec;
        for (size_t r = 0; r < d; ++r)
            for (size_t c = 0; c < d; ++c) sub.at(r, c) = m.at(in_idx[r], c);
        invert(sub, dec);  // any d rows of M are independent (distinct Vandermonde points)
        ByteMatrix rows(out_idx.size(), d);
        for (size_t k = 0; k < out_idx.size(); ++k) {
            const size_t o = out_idx[k];
            if (o < d) {
                for (size_t c = 0; c < d; ++c) rows.at(k, c) = dec.at(o, c);
            } else {
                const Gf256& g = Gf256::get();
                for (size_t c = 0; c < d; ++c) {
                    uint8_t acc = 0;
                    for (size_t q = 0; q < d; ++q) acc ^= g.mul(m.at(o, q), dec.at(q, c));
                    rows.at(k, c) = acc;
                }
            }
        }
        auto rec = std::make_shared<std::vector<uint32_t>>(pattern_words(d, out_idx.size()));
        write_pattern(rec->data(), d, in_idx, out_idx, rows);
        if (dec_cache.size() >= kDecCacheCap) {
            dec_cache.erase(dec_lru.back());
            dec_lru.pop_back();
        }
        dec_lru.push_front(key);
        dec_cache.emplace(key, std::make_pair(Record(rec), dec_lru.begin()));
        return rec;
    }

    size_t cached_patterns() {
        std::lock_guard<std::mutex> lk(mu);
        return dec_cache.size();
    }
};

namespace {

// Crate checks shared by the per-part reconstruct entry points.  Returns CEC_OK with *len set
// and *work = true if something must be rebuilt.
int check_reconstruct(const cec_codec* c, const size_t* lens, const uint8_t* present,
                      size_t n_shards, size_t* len, bool* work) {
    const size_t t = c->d + c->p;
    if (n_shards < t) return CEC_TOO_FEW_SHARDS;
    if (n_shards > t) return CEC_TOO_MANY_SHARDS;
    size_t n_present = 0;
    bool have = false;
    for (size_t i = 0; i < t; ++i) {
        if (!present[i]) continue;
        if (lens[i] == 0) return CEC_EMPTY_SHARD;
        ++n_present;
        if (have && lens[i] != *len) return CEC_INCORRECT_SHARD_SIZE;
        *len = lens[i];
        have = true;
    }
    *work = n_present != t;
    if (!*work) return CEC_OK;
    if (n_present < c->d) return CEC_TOO_FEW_SHARDS_PRESENT;
    return CEC_OK;
}

PatternKey make_key(const uint8_t* present, size_t t, bool data_only) {
    PatternKey k;
    for (size_t i = 0; i < t; ++i)
        if (present[i]) k.bits[i / 64] |= uint64_t(1) << (i % 64);
    k.data_only = data_only;
    return k;
}

int reconstruct_host(const cec_codec* cc, uint8_t* const* shards, const size_t* lens,
                     uint8_t* present, size_t n_shards, bool data_only) {
    if (!cc || !shards || !lens || !present) return CEC_ERR_INVALID_ARGUMENT;
    cec_codec* c = const_cast<cec_codec*>(cc);
    size_t len = 0;
    bool work = false;
    CEC_TRY(check_reconstruct(c, lens, present, n_shards, &len, &work));
    if (!work) return CEC_OK;
    const size_t t = c->d + c->p;
    auto rec = c->decode_record(make_key(present, t, data_only));
    const size_t n_out = (*rec)[0];
    const uint32_t* out_idx = rec->data() + 1 + c->d;
    for (size_t k = 0; k < n_out; ++k) {
        const size_t o = out_idx[k];
        if (!shards[o] || lens[o] < len) {
            g_last_error = "missing shard buffer too small";
            return CEC_ERR_INVALID_ARGUMENT;
        }
    }
    if (n_out == 0) return CEC_OK;  // data_only with only parity missing
    const size_t cs = round_up(len, kChunkAlign);
    const size_t rec_bytes = round_up(rec->size() * sizeof(uint32_t), kChunkAlign);
    CtxLease ctx;
    CEC_TRY(ctx.acquire(rec_bytes + t * cs));
    uint32_t* drec = reinterpret_cast<uint32_t*>(ctx->dbuf);
    uint8_t* dbase = ctx->dbuf + rec_bytes;
    HIP_TRY(hipMemcpyAsync(drec, rec->data(), rec->size() * sizeof(uint32_t),
                           hipMemcpyHostToDevice, ctx->stream));
    const uint32_t* in_idx = rec->data() + 1;
    for (size_t j = 0; j < c->d; ++j)
        HIP_TRY(hipMemcpyAsync(dbase + in_idx[j] * cs, shards[in_idx[j]], len,
                               hipMemcpyHostToDevice, ctx->stream));
    ApplyParams a{};
    a.base = dbase;
    a.part_stride = t * cs;
    a.chunk_stride = cs;
    a.len = len;
    a.pat = drec;
    a.n_parts = 1;
    a.d = uint32_t(c->d);
    a.n_rows = uint32_t(n_out);
    HIP_TRY(launch_rs_apply(a, true, ctx->stream));
    for (size_t k = 0; k < n_out; ++k)
        HIP_TRY(hipMemcpyAsync(shards[out_idx[k]], dbase + out_idx[k] * cs, len,
                               hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    for (size_t k = 0; k < n_out; ++k) present[out_idx[k]] = 1;
    return CEC_OK;
}

// Fused encode+hash kernel or encode kernel + SHA kernel for a batch of `chunks` chunks (d+p per
// part).  The fused kernel reads every byte once and wins when the SHA lanes fill the chip; a
// small batch leaves most SIMDs idle, and the split SHA kernel's lower per-chain latency (31 vs
// 42 ms per MiB) wins while the encode's extra pass is negligible.  CEC_FUSED (A/B knob): 0 =
// always separate, 1 = always fused where supported.
bool prefer_fused(size_t chunks) {
    const int f = knobs().fused;
    return f >= 0 ? f == 1 : !use_split(chunks);
}

// ------------------------------------------------------------------------------------------
// Per-call coalescing ("a batch queue behind the per-part call").
//
// A GPU SHA-256 lane hashes one chunk as a serial chain (~42 ms per MiB), so one part per
// launch leaves the chip idle and the reference's own concurrency (≤10 part tasks,
// writer.rs:130; `concurrency` is a builder knob) only helps if concurrent calls share a
// launch.  cec_part_encode / cec_sha256(_many) therefore go through a leader/follower queue:
// the first caller to find no batch in progress becomes the leader, waits up to
// CEC_COALESCE_US microseconds (default 200; only when calls are concurrent) for more requests
// with its key (codec, chunk length, device), and runs them as ONE batch:
//   1. copy-in   every caller copies its own (pageable) input into the queue's pinned staging,
//                in parallel on its own thread;
//   2. launch    the leader moves the whole batch with one H2D copy, runs the fused
//                encode+hash (or the SHA) kernel over every part, and brings parity and
//                digests back with one D2H copy into pinned staging;
//   3. copy-out  every caller copies its results out into its own buffers, in parallel.
// Batches are capped at CEC_COALESCE_MAX_MIB of input (default 1024).  Results are
// bit-identical to one call per launch (same kernels, same inputs).
// ------------------------------------------------------------------------------------------
std::atomic<uint64_t> g_calls{0}, g_launches{0};

uint32_t coalesce_window_us() { return knobs().coalesce_us; }

size_t coalesce_max_bytes() { return knobs().coalesce_max_bytes; }

bool coalesce_trace() { return knobs().coalesce_trace; }

// Pinned host staging, never shrunk.  Pinning costs ~0.35 s per GiB, so the first growth
// past 64 MiB goes straight to the batch cap (one pinning per process, not one per size step).
struct PinnedBuf {
    uint8_t* ptr = nullptr;
    size_t cap = 0;
    int reserve(size_t bytes, size_t cap_hint) {
        if (cap >= bytes) return CEC_OK;
        if (ptr) HIP_TRY(hipHostFree(ptr));
        ptr = nullptr;
        cap = 0;
        const size_t want =
            round_up(bytes <= (size_t(64) << 20) ? std::max(bytes, size_t(64) << 20)
                                                 : std::max(bytes, cap_hint),
                     1 << 20);
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ptr), want, hipHostMallocDefault));
        cap = want;
        return CEC_OK;
    }
};

struct Arena {
    StageCtx dev;  // stream + device staging
    PinnedBuf in, out;
    // CEC_COALESCE_EARLY_D2H: the parity comes back on a side stream as soon as the encode is
    // done, beside the SHA-256 chains (made on first use; arenas live as long as the process)
    hipStream_t side = nullptr;
    hipEvent_t encoded = nullptr;
};

// How the early parity download waits for the encode: on the host (the leader blocks on the
// event, then queues the copy: the default, round 2's form, adopted after a 256-caller hang on
// an earlier device-side form) or on the device (the side stream waits on the encode's event:
// CEC_COALESCE_D2H_WAIT=device, kept for the A/B).  Both are deadlock-free (see the wait
// itself), and DESIGN.md §4.7's A/B put them within run-to-run spread, so the default is the
// form with the longer record.
bool coalesce_d2h_host_wait() { return knobs().coalesce_d2h_host_wait; }

bool coalesce_early_d2h() {  // default on (profiles/r2_early_d2h/); =0 for A/B
    return knobs().coalesce_early_d2h;
}

struct CoalesceKey {
    const void* codec;
    size_t len;
    int device;
    bool operator==(const CoalesceKey& o) const {
        return codec == o.codec && len == o.len && device == o.device;
    }
};

enum class Phase { Queued, CopyIn, Staged, CopyOut, Finished };

struct ReqBase {
    int device = 0;
    int status = CEC_OK;
    std::string err;
    Phase phase = Phase::Queued;
    size_t slot = 0;        // index in the batch
    size_t in_off = 0;      // byte offset in the pinned input staging
    size_t item0 = 0;       // sha: first item index; parts: parts in the batch
    Arena* arena = nullptr;
    struct Batch* batch = nullptr;  // the batch this request runs in
    std::condition_variable cv;     // this caller's wake-ups
};

// Impl: bytes(r) = input bytes; prepare(batch, arena) lays out + reserves; copy_in(r);
// run(batch, arena) launches and waits; copy_out(r).
// Wake-ups are targeted (one condition variable per request plus one for the leader) so a
// batch of hundreds of callers costs O(batch) wake-ups, not O(batch^2).
// One batch in flight: its size and copy counters, and the leader's wake-ups.
struct Batch {
    size_t size = 0, staged = 0, finished = 0;
    std::condition_variable cv;
};

// Batches on the GPU at once (CEC_COALESCE_INFLIGHT, 1..16; default 2).  A second batch starts
// while one runs only when the batch before it overflowed the cap (callers of its key were left
// queued): otherwise a leader would start as soon as an arena is free, and since a launch costs
// one chunk's SHA chain whatever its size, the callers would split into ever smaller batches that
// each pay it (round 1, unconditional: 100 threads 7.1-8.2 GB/s with 1 vs 3.6-3.8 with 4,
// profiles/r1y_percall_ab.log).  Overflowing callers (256 pageable parts vs a 1 GiB cap) then
// copy in while the first batch runs: 13.9 -> ~26 GB/s (profiles/r2_percall/).
// CEC_COALESCE_ADAPT=0 (A/B knob): fixed CEC_COALESCE_US window, no early exit.
bool coalesce_adaptive() { return knobs().coalesce_adaptive; }

uint32_t coalesce_inflight() { return knobs().coalesce_inflight; }

template <typename Req, typename Impl>
class Coalescer {
   public:
    int submit(Req* r) {
        g_calls.fetch_add(1, std::memory_order_relaxed);
        std::unique_lock<std::mutex> lk(mu_);
        peak_ = std::max(peak_, ++callers_);
        queue_.push_back(r);
        if (gathering_) gather_cv_.notify_one();  // the gathering leader re-checks its batch
        for (;;) {
            if (r->phase == Phase::CopyIn) {
                lk.unlock();
                Impl::copy_in(*r);
                lk.lock();
                r->phase = Phase::Staged;
                if (++r->batch->staged == r->batch->size) r->batch->cv.notify_one();
            } else if (r->phase == Phase::CopyOut) {
                lk.unlock();
                if (r->status == CEC_OK) Impl::copy_out(*r);
                lk.lock();
                r->phase = Phase::Finished;
                if (++r->batch->finished == r->batch->size) r->batch->cv.notify_one();
                break;
            } else if (r->phase == Phase::Queued && r->batch == nullptr && !gathering_ &&
                       (active_ == 0 || (overflow_ && active_ < coalesce_inflight()))) {
                // r->batch: a caller already taken into a batch stays Queued until its leader
                // has prepared the arena (lock released meanwhile); woken in that window (a
                // wake-up sent before the batch formed) it must not lead a batch of its own, or
                // it never copies in and its leader waits forever — seen with two batches in
                // flight at 256 pageable callers.
                lead(r, lk);
                break;
            } else {
                r->cv.wait(lk);
            }
        }
        --callers_;
        lk.unlock();
        if (r->status != CEC_OK) g_last_error = r->err;
        return r->status;
    }

   private:
    // Wake the oldest queued request so it can lead the next batch (if a slot is free).
    void wake_next() {
        if (!queue_.empty()) queue_.front()->cv.notify_one();
    }

    // Called with lk held; returns with r finished.  Up to coalesce_inflight() leaders run their
    // batches at once (one arena = pinned staging + device buffer + stream each), so the next
    // batch gathers, copies and launches while earlier ones are still on the GPU.
    void lead(Req* r, std::unique_lock<std::mutex>& lk) {
        ++active_;
        gathering_ = true;
        const auto key = r->key();
        auto matching_bytes = [&] {
            size_t b = 0;
            for (Req* q : queue_)
                if (q->key() == key) b += Impl::cap_bytes(*q);
            return b;
        };
        auto matching_count = [&] {
            size_t n = 0;
            for (Req* q : queue_) n += q->key() == key ? 1 : 0;
            return n;
        };
        if (last_batch_ > 1 || queue_.size() > 1) {
            // Wait for company only when calls are actually concurrent (the last batch had several
            // callers, or others are queued now): a lone caller's calls never pay the window.
            // The window scales with the last launch (1/8 of its run time, at least
            // CEC_COALESCE_US): callers of the batch that just finished are still copying their
            // results out and come back a few ms later; a short window splits the callers into
            // two alternating groups, each paying a full launch (10 threads: 5 parts per launch).
            // It ends early once as many callers are queued as were ever inside at once lately.
            uint64_t window = coalesce_window_us();
            if (coalesce_adaptive()) window = std::max<uint64_t>(window, last_run_us_ / 8);
            const auto until =
                std::chrono::steady_clock::now() + std::chrono::microseconds(window);
            gather_cv_.wait_until(lk, until, [&] {
                return matching_bytes() >= coalesce_max_bytes() ||
                       (coalesce_adaptive() && matching_count() >= peak_);
            });
        }
        Batch batch_state;
        std::vector<Req*> batch{r};
        size_t bytes = Impl::cap_bytes(*r);
        for (auto it = queue_.begin(); it != queue_.end();) {
            if (*it == r) {
                it = queue_.erase(it);
            } else if ((*it)->key() == key &&
                       bytes + Impl::cap_bytes(**it) <= coalesce_max_bytes()) {
                bytes += Impl::cap_bytes(**it);
                batch.push_back(*it);
                it = queue_.erase(it);
            } else {
                ++it;
            }
        }
        for (Req* q : batch) q->batch = &batch_state;
        batch_state.size = batch.size();
        last_batch_ = batch.size();
        overflow_ = false;  // callers of this key left behind by the cap
        for (Req* q : queue_) overflow_ = overflow_ || q->key() == key;
        if (++batches_since_peak_ >= 32) {  // forget an old burst of callers
            peak_ = callers_;
            batches_since_peak_ = 0;
        }
        Arena* arena = take_arena(key.device);
        gathering_ = false;
        if (coalesce_trace())
            std::fprintf(stderr, "[cec coalesce] lead arena %p: %zu callers, %u active, %zu queued\n",
                         (void*)arena, batch.size(), active_, queue_.size());
        wake_next();  // the next batch can gather while this one runs
        lk.unlock();
        const auto t0 = std::chrono::steady_clock::now();
        auto t1 = t0, t2 = t0, t3 = t0;
        int st = Impl::prepare(batch, *arena);
        if (coalesce_trace())
            std::fprintf(stderr, "[cec coalesce] arena %p: prepared (%d)\n", (void*)arena, st);
        if (st == CEC_OK) {
            lk.lock();
            batch_state.staged = 1;  // the leader's own copy, done below
            for (Req* q : batch)
                if (q != r) {
                    q->phase = Phase::CopyIn;
                    q->cv.notify_one();
                }
            t1 = std::chrono::steady_clock::now();
            lk.unlock();
            Impl::copy_in(*r);
            lk.lock();
            batch_state.cv.wait(lk, [&] { return batch_state.staged == batch_state.size; });
            lk.unlock();
            if (coalesce_trace())
                std::fprintf(stderr, "[cec coalesce] arena %p: staged\n", (void*)arena);
            t2 = std::chrono::steady_clock::now();
            g_launches.fetch_add(1, std::memory_order_relaxed);
            st = Impl::run(batch, *arena);
            t3 = std::chrono::steady_clock::now();
        }
        const std::string err = st == CEC_OK ? std::string() : g_last_error;
        lk.lock();
        last_run_us_ = uint64_t(std::chrono::duration_cast<std::chrono::microseconds>(t3 - t2).count());
        batch_state.finished = 1;
        for (Req* q : batch) {
            q->status = st;
            q->err = err;
            if (q != r) {
                q->phase = Phase::CopyOut;
                q->cv.notify_one();
            }
        }
        lk.unlock();
        if (st == CEC_OK) Impl::copy_out(*r);
        lk.lock();
        // the arena is reused by a later batch: wait for every copy-out
        batch_state.cv.wait(lk, [&] { return batch_state.finished == batch_state.size; });
        if (coalesce_trace()) {
            auto ms = [](auto a, auto b) {
                return std::chrono::duration<double, std::milli>(b - a).count();
            };
            std::fprintf(stderr,
                         "[cec coalesce] batch %zu (%zu B): prepare %.2f ms, copy-in %.2f ms, "
                         "run %.2f ms, copy-out %.2f ms\n",
                         batch.size(), bytes, ms(t0, t1), ms(t1, t2), ms(t2, t3),
                         ms(t3, std::chrono::steady_clock::now()));
        }
        r->phase = Phase::Finished;
        free_[key.device].push_back(arena);
        --active_;
        wake_next();
    }

    // A free arena of `device` (called with mu_ held; at most coalesce_inflight() are in use).
    Arena* take_arena(int device) {
        auto& free_list = free_[device];
        if (free_list.empty()) {
            arenas_.push_back(std::make_unique<Arena>());
            return arenas_.back().get();
        }
        Arena* a = free_list.back();
        free_list.pop_back();
        return a;
    }

    std::mutex mu_;
    std::condition_variable gather_cv_;
    std::deque<Req*> queue_;
    bool gathering_ = false;
    uint32_t active_ = 0;
    bool overflow_ = false;          // the last batch formed left callers of its key queued
    size_t last_batch_ = 0;
    size_t callers_ = 0;             // submit() calls in progress
    size_t peak_ = 0;                // most callers in progress at once, lately
    uint32_t batches_since_peak_ = 0;
    uint64_t last_run_us_ = 0;       // launch-to-results time of the last batch
    std::vector<std::unique_ptr<Arena>> arenas_;  // owned; free lists per device below
    std::map<int, std::vector<Arena*>> free_;
};

// ---- cec_sha256(_many): one request = n buffers ----
struct ShaReq : ReqBase {
    const uint8_t* const* bufs = nullptr;
    const size_t* lens = nullptr;
    size_t n = 0;
    uint8_t* out = nullptr;
    CoalesceKey key() const { return {nullptr, 0, device}; }
};

struct ShaImpl {
    static size_t item_bytes(size_t len) { return round_up(std::max<size_t>(len, 1), kChunkAlign); }
    static size_t bytes(const ShaReq& r) {
        size_t b = 0;
        for (size_t i = 0; i < r.n; ++i) b += item_bytes(r.lens[i]);
        return b;
    }
    static size_t cap_bytes(const ShaReq& r) { return bytes(r); }
    static int prepare(std::vector<ShaReq*>& batch, Arena& a) {
        size_t off = 0, items = 0;
        for (ShaReq* r : batch) {
            r->arena = &a;
            r->in_off = off;
            r->item0 = items;
            off += bytes(*r);
            items += r->n;
        }
        CEC_TRY(a.in.reserve(off, coalesce_max_bytes()));
        CEC_TRY(a.out.reserve(items * 32, coalesce_max_bytes() / 8));
        const size_t meta = round_up(2 * items * sizeof(uint64_t), kChunkAlign);
        return ctx_reserve(a.dev, meta + round_up(items * 32, kChunkAlign) + off);
    }
    static void copy_in(ShaReq& r) {
        size_t off = r.in_off;
        for (size_t i = 0; i < r.n; ++i) {
            if (r.lens[i]) std::memcpy(r.arena->in.ptr + off, r.bufs[i], r.lens[i]);
            off += item_bytes(r.lens[i]);
        }
    }
    static int run(std::vector<ShaReq*>& batch, Arena& a) {
        size_t items = 0, total = 0;
        for (ShaReq* r : batch) {
            items += r->n;
            total += bytes(*r);
        }
        const size_t meta = round_up(2 * items * sizeof(uint64_t), kChunkAlign);
        const size_t dig = round_up(items * 32, kChunkAlign);
        uint64_t* dptrs = reinterpret_cast<uint64_t*>(a.dev.dbuf);
        uint8_t* ddig = a.dev.dbuf + meta;
        uint8_t* ddata = ddig + dig;
        std::vector<uint64_t> hmeta(2 * items);
        size_t k = 0, off = 0;
        for (ShaReq* r : batch)
            for (size_t i = 0; i < r->n; ++i, ++k) {
                hmeta[k] = reinterpret_cast<uint64_t>(ddata + off);
                hmeta[items + k] = r->lens[i];
                off += item_bytes(r->lens[i]);
            }
        hipStream_t s = a.dev.stream;
        HIP_TRY(hipMemcpyAsync(ddata, a.in.ptr, total, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(dptrs, hmeta.data(), hmeta.size() * sizeof(uint64_t),
                               hipMemcpyHostToDevice, s));
        ShaParams h{};
        h.ptrs = dptrs;
        h.lens = dptrs + items;
        h.n_parts = uint32_t(items);
        h.n_chunks = 1;
        h.digests = ddig;
        HIP_TRY(launch_sha256(h, true, s));
        HIP_TRY(hipMemcpyAsync(a.out.ptr, ddig, items * 32, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        return CEC_OK;
    }
    static void copy_out(ShaReq& r) {
        std::memcpy(r.out, r.arena->out.ptr + r.item0 * 32, r.n * 32);
    }
};

// ---- cec_part_encode: one request = one part (d*L bytes of data_buf) ----
struct PartReq : ReqBase {
    cec_codec* codec = nullptr;
    const uint8_t* data_buf = nullptr;  // d*L bytes
    size_t L = 0;
    uint8_t* parity_out = nullptr;      // p*L bytes
    uint8_t* digests_out = nullptr;     // (d+p)*32 bytes
    // Page-locked caller buffers (cec_host_alloc): DMA'd directly, no copy-in / copy-out.
    bool in_pinned = false, out_pinned = false;
    size_t out_off = 0;                 // parity offset in the pinned output staging
    // Early upload (CEC_COALESCE_EARLY_H2D): the caller queues its own part's H2D right after its
    // copy-in, so the uploads overlap the other callers' copies instead of following them all.
    bool early = false;
    uint8_t* dev_dst = nullptr;         // this part's place in the device batch
    hipStream_t stream = nullptr;       // the batch's stream
    hipError_t early_err = hipSuccess;
    CoalesceKey key() const { return {codec, L, device}; }
};

bool coalesce_early_h2d() { return knobs().coalesce_early_h2d; }

// Pinned layout: input [part][d][cs] (staged parts only, at in_off), output [part][p][cs]
// (staged parts only, at out_off) then digests [part][d+p][32]; device batch [part][d+p][cs]
// (cs = L rounded up to 256 B).  A batch with no page-locked caller buffer moves with one
// 2-D copy each way; otherwise every part is copied on its own (pinned ones straight from /
// into the caller's memory).
struct PartImpl {
    static size_t cs_of(const PartReq& r) { return round_up(r.L, kChunkAlign); }
    static size_t bytes(const PartReq& r) { return r.codec->d * cs_of(r); }
    // Weight against CEC_COALESCE_MAX_MIB: the cap bounds the pinned staging a batch needs; a
    // page-locked caller needs none, so its part counts a quarter (its batch is bounded by the
    // device buffer, 4x the staging cap).
    // (A/B at 256 page-locked callers, profiles/r2_percall/pinned_cap_*: full weight 26.0 GB/s,
    // half 23.6, quarter 24.8 — noise; the quarter keeps them in one launch.)
    static size_t cap_bytes(const PartReq& r) { return r.in_pinned ? bytes(r) / 4 : bytes(r); }
    static bool any_pinned(const std::vector<PartReq*>& batch) {
        for (const PartReq* r : batch)
            if (r->in_pinned || r->out_pinned) return true;
        return false;
    }
    static size_t digest_base(const std::vector<PartReq*>& batch) {
        size_t off = 0;
        for (const PartReq* r : batch)
            if (!r->out_pinned) off += r->codec->p * cs_of(*r);
        return off;
    }
    static int prepare(std::vector<PartReq*>& batch, Arena& a) {
        const cec_codec* c = batch[0]->codec;
        const size_t d = c->d, p = c->p, t = d + p, B = batch.size(), cs = cs_of(*batch[0]);
        size_t in_bytes = 0, out_bytes = 0;
        for (size_t k = 0; k < B; ++k) {
            PartReq* r = batch[k];
            r->arena = &a;
            r->slot = k;
            r->in_off = in_bytes;
            r->out_off = out_bytes;
            if (!r->in_pinned) in_bytes += d * cs;
            if (!r->out_pinned) out_bytes += p * cs;
        }
        const size_t dig0 = out_bytes;
        for (PartReq* r : batch) r->item0 = dig0;  // locates the digest block
        CEC_TRY(a.in.reserve(std::max<size_t>(in_bytes, 1), coalesce_max_bytes()));
        CEC_TRY(a.out.reserve(out_bytes + B * t * 32,
                              coalesce_max_bytes() / d * p + coalesce_max_bytes() / cs * t * 32));
        CEC_TRY(ctx_reserve(a.dev, round_up(B * t * 32, kChunkAlign) + B * t * cs));
        const bool early = coalesce_early_h2d();
        uint8_t* dbase = a.dev.dbuf + round_up(B * t * 32, kChunkAlign);
        for (PartReq* r : batch) {
            r->early = early;
            r->dev_dst = dbase + r->slot * t * cs;
            r->stream = a.dev.stream;
            r->early_err = hipSuccess;
        }
        return CEC_OK;
    }
    // This part's upload into the device batch (from the caller's page-locked buffer or from its
    // copy in the pinned staging).
    static hipError_t upload(PartReq& r) {
        const size_t d = r.codec->d, cs = cs_of(r);
        if (r.in_pinned && cs == r.L)
            return hipMemcpyAsync(r.dev_dst, r.data_buf, d * r.L, hipMemcpyHostToDevice, r.stream);
        if (r.in_pinned)
            return hipMemcpy2DAsync(r.dev_dst, cs, r.data_buf, r.L, r.L, d, hipMemcpyHostToDevice,
                                    r.stream);
        return hipMemcpyAsync(r.dev_dst, r.arena->in.ptr + r.in_off, d * cs, hipMemcpyHostToDevice,
                              r.stream);
    }
    static void copy_in(PartReq& r) {
        if (!r.in_pinned) {
            const size_t d = r.codec->d, cs = cs_of(r);
            uint8_t* dst = r.arena->in.ptr + r.in_off;
            for (size_t j = 0; j < d; ++j) std::memcpy(dst + j * cs, r.data_buf + j * r.L, r.L);
        }
        if (r.early) {
            r.early_err = upload(r);
            if (r.early_err != hipSuccess) (void)hipGetLastError();
        }
    }
    static int run(std::vector<PartReq*>& batch, Arena& a) {
        cec_codec* c = batch[0]->codec;
        const size_t d = c->d, p = c->p, t = d + p, B = batch.size();
        const size_t L = batch[0]->L, cs = cs_of(*batch[0]);
        const bool per_part = any_pinned(batch);
        uint32_t* drec = nullptr;
        CEC_TRY(c->encode_record(&drec));
        uint8_t* ddig = a.dev.dbuf;
        uint8_t* dbase = a.dev.dbuf + round_up(B * t * 32, kChunkAlign);
        hipStream_t s = a.dev.stream;
        if (batch[0]->early) {  // every caller queued its own upload after its copy-in
            for (const PartReq* r : batch) HIP_TRY(r->early_err);
        } else if (!per_part) {
            HIP_TRY(hipMemcpy2DAsync(dbase, t * cs, a.in.ptr, d * cs, d * cs, B,
                                     hipMemcpyHostToDevice, s));
        } else {
            for (PartReq* r : batch) HIP_TRY(upload(*r));  // pinned ones straight from the caller
        }
        // the parity of every part back to its caller (or the staging) on stream `q`
        auto parity_down = [&](hipStream_t q) -> int {
            if (!per_part) {
                HIP_TRY(hipMemcpy2DAsync(a.out.ptr, p * cs, dbase + d * cs, t * cs, p * cs, B,
                                         hipMemcpyDeviceToHost, q));
                return CEC_OK;
            }
            for (const PartReq* r : batch) {
                const uint8_t* src = dbase + r->slot * t * cs + d * cs;
                if (r->out_pinned && cs == L)  // straight into the caller's parity buffer
                    HIP_TRY(hipMemcpyAsync(r->parity_out, src, p * L, hipMemcpyDeviceToHost, q));
                else if (r->out_pinned)  // p rows of L bytes out of the padded chunk stride
                    HIP_TRY(hipMemcpy2DAsync(r->parity_out, r->L, src, cs, r->L, p,
                                             hipMemcpyDeviceToHost, q));
                else
                    HIP_TRY(hipMemcpyAsync(a.out.ptr + r->out_off, src, p * cs,
                                           hipMemcpyDeviceToHost, q));
            }
            return CEC_OK;
        };
        bool parity_sent = false;
        // an error return after the side-stream download was queued must not leave it writing
        // into the callers' buffers: wait for it on every exit
        struct SideWait {
            hipStream_t q = nullptr;
            ~SideWait() {
                if (q) (void)hipStreamSynchronize(q);
            }
        } side_wait;
        if (fused_covers(uint32_t(d), uint32_t(p), L) && prefer_fused(B * t)) {
            FusedParams f{};
            f.base = dbase;
            f.part_stride = t * cs;
            f.chunk_stride = cs;
            f.len = L;
            f.pat = drec;
            f.digests = ddig;
            f.n_parts = uint32_t(B);
            f.d = uint32_t(d);
            f.p = uint32_t(p);
            HIP_TRY(launch_encode_hash(f, true, s));
        } else {
            ApplyParams ap{};
            ap.base = dbase;
            ap.part_stride = t * cs;
            ap.chunk_stride = cs;
            ap.len = L;
            ap.pat = drec;
            ap.n_parts = uint32_t(B);
            ap.d = uint32_t(d);
            ap.n_rows = uint32_t(p);
            ap.std_encode = c->bs ? 1u : 0u;
            HIP_TRY(launch_rs_encode(ap, true, s));
            const bool early = coalesce_early_d2h();
            if (early) {
                if (!a.side) HIP_TRY(hipStreamCreateWithFlags(&a.side, hipStreamNonBlocking));
                if (!a.encoded) HIP_TRY(hipEventCreateWithFlags(&a.encoded, hipEventDisableTiming));
                HIP_TRY(hipEventRecord(a.encoded, s));
            }
            ShaParams h{};
            h.base = dbase;
            h.part_stride = t * cs;
            h.chunk_stride = cs;
            h.len = L;
            h.n_parts = uint32_t(B);
            h.first_chunk = 0;
            h.n_chunks = uint32_t(t);
            h.digests = ddig;
            HIP_TRY(launch_sha256(h, true, s));
            if (early) {
                // Parity down beside the SHA-256 chains (both only read the batch): the side
                // stream waits on the device for the encode's event.  A wait on an event that
                // was recorded before the wait is queued cannot deadlock, even when two streams
                // share one in-order hardware queue (more streams than GPU_MAX_HW_QUEUES): the
                // event's marker precedes the waiting packet in any queue order.  (Round 2 had
                // the host block on the event here, blaming a 256-caller hang on such waits;
                // that hang was the stranded-caller race fixed below, and the host hand-over
                // build hung the same way before that fix.)
                if (coalesce_d2h_host_wait())
                    HIP_TRY(hipEventSynchronize(a.encoded));
                else
                    HIP_TRY(hipStreamWaitEvent(a.side, a.encoded, 0));
                side_wait.q = a.side;
                CEC_TRY(parity_down(a.side));
                parity_sent = true;
            }
        }
        const size_t dig0 = batch[0]->item0;
        if (!parity_sent) CEC_TRY(parity_down(s));
        HIP_TRY(hipMemcpyAsync(a.out.ptr + dig0, ddig, B * t * 32, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (parity_sent) HIP_TRY(hipStreamSynchronize(a.side));
        return CEC_OK;
    }
    static void copy_out(PartReq& r) {
        const size_t d = r.codec->d, p = r.codec->p, t = d + p, cs = cs_of(r);
        if (!r.out_pinned) {
            const uint8_t* par = r.arena->out.ptr + r.out_off;
            for (size_t i = 0; i < p; ++i) std::memcpy(r.parity_out + i * r.L, par + i * cs, r.L);
        }
        std::memcpy(r.digests_out, r.arena->out.ptr + r.item0 + r.slot * t * 32, t * 32);
    }
};

Coalescer<ShaReq, ShaImpl> g_sha_queue;
Coalescer<PartReq, PartImpl> g_part_queue;

int sha256_coalesced(const uint8_t* const* bufs, const size_t* lens, size_t n, uint8_t* out) {
    ShaReq r;
    CEC_TRY(current_device(&r.device));
    r.bufs = bufs;
    r.lens = lens;
    r.n = n;
    r.out = out;
    return g_sha_queue.submit(&r);
}

int part_encode_coalesced(cec_codec* c, const uint8_t* data_buf, size_t L, uint8_t* parity_out,
                          uint8_t* digests_out) {
    PartReq r;
    CEC_TRY(current_device(&r.device));
    r.codec = c;
    r.data_buf = data_buf;
    r.L = L;
    r.parity_out = parity_out;
    r.digests_out = digests_out;
    r.in_pinned = pinned_range(data_buf, c->d * L);
    r.out_pinned = pinned_range(parity_out, c->p * L);
    return g_part_queue.submit(&r);
}

void coalesce_stats(uint64_t* calls, uint64_t* launches) {
    if (calls) *calls = g_calls.load();
    if (launches) *launches = g_launches.load();
}

int batch_ok(const cec_part_batch* b) {
    if (!b || !b->base) return CEC_ERR_INVALID_ARGUMENT;
    return CEC_OK;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// Library
// ------------------------------------------------------------------------------------------
extern "C" {

int cec_abi_version(void) { return CEC_ABI_VERSION; }

const char* cec_build_info(void) {
#ifdef CEC_AB_TOOLS
    return "chunky_ec gfx950 ab_tools=1 (A/B attribution build: CEC_FUSED_MODE 1/2 and "
           "CEC_SHA_VARIANT 7/8 produce wrong outputs by design; not for production)";
#else
    return "chunky_ec gfx950 ab_tools=0";
#endif
}

const char* cec_status_name(int s) {
    switch (s) {
        case CEC_OK: return "Ok";
        case CEC_TOO_FEW_SHARDS: return "TooFewShards";
        case CEC_TOO_MANY_SHARDS: return "TooManyShards";
        case CEC_TOO_FEW_DATA_SHARDS: return "TooFewDataShards";
        case CEC_TOO_MANY_DATA_SHARDS: return "TooManyDataShards";
        case CEC_TOO_FEW_PARITY_SHARDS: return "TooFewParityShards";
        case CEC_TOO_MANY_PARITY_SHARDS: return "TooManyParityShards";
        case CEC_TOO_FEW_BUFFER_SHARDS: return "TooFewBufferShards";
        case CEC_TOO_MANY_BUFFER_SHARDS: return "TooManyBufferShards";
        case CEC_INCORRECT_SHARD_SIZE: return "IncorrectShardSize";
        case CEC_TOO_FEW_SHARDS_PRESENT: return "TooFewShardsPresent";
        case CEC_EMPTY_SHARD: return "EmptyShard";
        case CEC_INVALID_SHARD_FLAGS: return "InvalidShardFlags";
        case CEC_INVALID_INDEX: return "InvalidIndex";
        case CEC_ERR_INVALID_ARGUMENT: return "InvalidArgument";
        case CEC_ERR_HIP: return "HipError";
        case CEC_ERR_NO_DEVICE: return "NoDevice";
        case CEC_ERR_OUT_OF_MEMORY: return "OutOfMemory";
        default: return "Unknown";
    }
}

const char* cec_last_error(void) { return g_last_error.c_str(); }

int cec_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// ------------------------------------------------------------------------------------------
// Codec
// ------------------------------------------------------------------------------------------

int cec_codec_new(size_t d, size_t p, cec_codec** out) {
    if (!out) return CEC_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    // ReedSolomon::new order of checks.
    if (d == 0) return CEC_TOO_FEW_DATA_SHARDS;
    if (p == 0) return CEC_TOO_FEW_PARITY_SHARDS;
    if (d + p > 256) return CEC_TOO_MANY_SHARDS;
    auto c = std::make_unique<cec_codec>();
    c->d = d;
    c->p = p;
    c->m = build_coding_matrix(d, p);
    ByteMatrix rows(p, d);
    std::vector<uint32_t> in_idx(d), out_idx(p);
    for (size_t j = 0; j < d; ++j) in_idx[j] = uint32_t(j);
    for (size_t i = 0; i < p; ++i) {
        out_idx[i] = uint32_t(d + i);
        for (size_t j = 0; j < d; ++j) rows.at(i, j) = c->m.at(d + i, j);
    }
    c->enc.resize(pattern_words(d, p));
    write_pattern(c->enc.data(), d, in_idx, out_idx, rows);
    c->bs = d <= 0xFFFFFFFFull && p <= 0xFFFFFFFFull &&
            bs_encode_matches(uint32_t(d), uint32_t(p), rows.v.data());
    *out = c.release();
    return CEC_OK;
}

void cec_codec_free(cec_codec* c) { delete c; }
size_t cec_codec_data_shards(const cec_codec* c) { return c ? c->d : 0; }
size_t cec_codec_parity_shards(const cec_codec* c) { return c ? c->p : 0; }
size_t cec_codec_total_shards(const cec_codec* c) { return c ? c->d + c->p : 0; }
size_t cec_codec_cached_patterns(const cec_codec* c) {
    return c ? const_cast<cec_codec*>(c)->cached_patterns() : 0;
}

int cec_codec_matrix(const cec_codec* c, uint8_t* out, size_t out_len) {
    if (!c || !out || out_len < c->m.v.size()) return CEC_ERR_INVALID_ARGUMENT;
    std::memcpy(out, c->m.v.data(), c->m.v.size());
    return CEC_OK;
}

// ------------------------------------------------------------------------------------------
// Host-buffer API
// ------------------------------------------------------------------------------------------

int cec_encode_sep(const cec_codec* cc, const uint8_t* const* data, const size_t* data_lens,
                   size_t n_data, uint8_t* const* parity, const size_t* parity_lens,
                   size_t n_parity) {
    if (!cc) return CEC_ERR_INVALID_ARGUMENT;
    cec_codec* c = const_cast<cec_codec*>(cc);
    // check_piece_count!(data), check_piece_count!(parity)
    if (n_data < c->d) return CEC_TOO_FEW_DATA_SHARDS;
    if (n_data > c->d) return CEC_TOO_MANY_DATA_SHARDS;
    if (n_parity < c->p) return CEC_TOO_FEW_PARITY_SHARDS;
    if (n_parity > c->p) return CEC_TOO_MANY_PARITY_SHARDS;
    if (!data || !data_lens || !parity || !parity_lens) return CEC_ERR_INVALID_ARGUMENT;
    // check_slices!(multi => data, multi => parity)
    const size_t len = data_lens[0];
    if (len == 0) return CEC_EMPTY_SHARD;
    for (size_t j = 0; j < n_data; ++j)
        if (data_lens[j] != len) return CEC_INCORRECT_SHARD_SIZE;
    if (parity_lens[0] == 0) return CEC_EMPTY_SHARD;
    for (size_t i = 0; i < n_parity; ++i)
        if (parity_lens[i] != parity_lens[0]) return CEC_INCORRECT_SHARD_SIZE;
    if (parity_lens[0] != len) return CEC_INCORRECT_SHARD_SIZE;

    const size_t t = c->d + c->p, cs = round_up(len, kChunkAlign);
    uint32_t* drec = nullptr;
    CEC_TRY(c->encode_record(&drec));
    CtxLease ctx;
    CEC_TRY(ctx.acquire(t * cs));
    for (size_t j = 0; j < c->d; ++j)
        HIP_TRY(hipMemcpyAsync(ctx->dbuf + j * cs, data[j], len, hipMemcpyHostToDevice,
                               ctx->stream));
    ApplyParams a{};
    a.base = ctx->dbuf;
    a.part_stride = t * cs;
    a.chunk_stride = cs;
    a.len = len;
    a.pat = drec;
    a.n_parts = 1;
    a.d = uint32_t(c->d);
    a.n_rows = uint32_t(c->p);
    a.std_encode = c->bs ? 1u : 0u;
    HIP_TRY(launch_rs_encode(a, true, ctx->stream));
    for (size_t i = 0; i < c->p; ++i)
        HIP_TRY(hipMemcpyAsync(parity[i], ctx->dbuf + (c->d + i) * cs, len,
                               hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return CEC_OK;
}

int cec_reconstruct(const cec_codec* c, uint8_t* const* shards, const size_t* lens,
                    uint8_t* present, size_t n) {
    return reconstruct_host(c, shards, lens, present, n, false);
}

int cec_reconstruct_data(const cec_codec* c, uint8_t* const* shards, const size_t* lens,
                         uint8_t* present, size_t n) {
    return reconstruct_host(c, shards, lens, present, n, true);
}

int cec_sha256_many(const uint8_t* const* bufs, const size_t* lens, size_t n, uint8_t* out) {
    if (n == 0) return CEC_OK;
    if (!bufs || !lens || !out) return CEC_ERR_INVALID_ARGUMENT;
    for (size_t i = 0; i < n; ++i)
        if (lens[i] && !bufs[i]) return CEC_ERR_INVALID_ARGUMENT;
    return sha256_coalesced(bufs, lens, n, out);
}

int cec_sha256(const uint8_t* buf, size_t len, uint8_t* out32) {
    return cec_sha256_many(&buf, &len, 1, out32);
}

int cec_part_encode(const cec_codec* cc, const uint8_t* data_buf, size_t length,
                    uint8_t* parity_out, uint8_t* digests_out, size_t* chunksize) {
    if (!cc || !parity_out || !digests_out || !chunksize) return CEC_ERR_INVALID_ARGUMENT;
    if (length == 0) return CEC_EMPTY_SHARD;
    if (!data_buf) return CEC_ERR_INVALID_ARGUMENT;
    const size_t L = (length + cc->d - 1) / cc->d;
    CEC_TRY(part_encode_coalesced(const_cast<cec_codec*>(cc), data_buf, L, parity_out,
                                  digests_out));
    *chunksize = L;
    return CEC_OK;
}

void cec_coalesce_stats(uint64_t* calls, uint64_t* launches) {
    coalesce_stats(calls, launches);
}

size_t cec_release_cached(int device) { return ctx_pool().trim(device); }

int cec_encode_batch(const cec_codec* cc, const cec_part_batch* b, void* stream) {
    if (!cc) return CEC_ERR_INVALID_ARGUMENT;
    CEC_TRY(batch_ok(b));
    if (b->n_parts == 0) return CEC_OK;
    if (b->chunk_len == 0) return CEC_EMPTY_SHARD;
    if (b->n_parts > 0xFFFFFFFFull) return CEC_ERR_INVALID_ARGUMENT;
    cec_codec* c = const_cast<cec_codec*>(cc);
    uint32_t* drec = nullptr;
    CEC_TRY(c->encode_record(&drec));
    ApplyParams a{};
    a.base = b->base;
    a.part_stride = b->part_stride;
    a.chunk_stride = b->chunk_stride;
    a.len = b->chunk_len;
    a.pat = drec;
    a.n_parts = uint32_t(b->n_parts);
    a.d = uint32_t(c->d);
    a.n_rows = uint32_t(c->p);
    a.std_encode = c->bs ? 1u : 0u;
    HIP_TRY(launch_rs_encode(a, aligned16(b->base, b->part_stride, b->chunk_stride),
                            static_cast<hipStream_t>(stream)));
    return CEC_OK;
}

int cec_sha256_batch(const cec_part_batch* b, size_t first_chunk, size_t n_chunks,
                     uint8_t* digests, void* stream) {
    CEC_TRY(batch_ok(b));
    if (!digests) return CEC_ERR_INVALID_ARGUMENT;
    if (b->n_parts == 0 || n_chunks == 0) return CEC_OK;
    if (b->n_parts * n_chunks > 0xFFFFFFFFull) return CEC_ERR_INVALID_ARGUMENT;
    ShaParams h{};
    h.base = b->base;
    h.part_stride = b->part_stride;
    h.chunk_stride = b->chunk_stride;
    h.len = b->chunk_len;
    h.n_parts = uint32_t(b->n_parts);
    h.first_chunk = uint32_t(first_chunk);
    h.n_chunks = uint32_t(n_chunks);
    h.digests = digests;
    HIP_TRY(launch_sha256(h, aligned16(b->base, b->part_stride, b->chunk_stride),
                          static_cast<hipStream_t>(stream)));
    return CEC_OK;
}

int cec_encode_hash_batch(const cec_codec* cc, const cec_part_batch* b, uint8_t* digests,
                          void* stream) {
    if (!cc || !digests) return CEC_ERR_INVALID_ARGUMENT;
    CEC_TRY(batch_ok(b));
    if (b->n_parts == 0) return CEC_OK;
    if (b->chunk_len == 0) return CEC_EMPTY_SHARD;
    if (b->n_parts * (cc->d + cc->p) > 0xFFFFFFFFull) return CEC_ERR_INVALID_ARGUMENT;
    cec_codec* c = const_cast<cec_codec*>(cc);
    const bool fused = fused_covers(uint32_t(c->d), uint32_t(c->p), b->chunk_len) &&
                       aligned16(b->base, b->part_stride, b->chunk_stride) &&
                       prefer_fused(b->n_parts * (c->d + c->p));
    if (!fused) {
        CEC_TRY(cec_encode_batch(c, b, stream));
        return cec_sha256_batch(b, 0, c->d + c->p, digests, stream);
    }
    uint32_t* drec = nullptr;
    CEC_TRY(c->encode_record(&drec));
    FusedParams f{};
    f.base = b->base;
    f.part_stride = b->part_stride;
    f.chunk_stride = b->chunk_stride;
    f.len = b->chunk_len;
    f.pat = drec;
    f.digests = digests;
    f.n_parts = uint32_t(b->n_parts);
    f.d = uint32_t(c->d);
    f.p = uint32_t(c->p);
    HIP_TRY(launch_encode_hash(f, aligned16(b->base, b->part_stride, b->chunk_stride),
                               static_cast<hipStream_t>(stream)));
    return CEC_OK;
}

// cec_reconstruct_batch with each decode block reserving lds_reserve bytes of LDS (see
// ApplyParams::lds_reserve).
static int reconstruct_batch(const cec_codec* cc, const cec_part_batch* b, const uint8_t* present,
                             int data_only, void* stream, uint32_t lds_reserve) {
    if (!cc || !present) return CEC_ERR_INVALID_ARGUMENT;
    CEC_TRY(batch_ok(b));
    if (b->n_parts == 0) return CEC_OK;
    if (b->chunk_len == 0) return CEC_EMPTY_SHARD;
    if (b->n_parts > 0xFFFFFFFFull) return CEC_ERR_INVALID_ARGUMENT;
    cec_codec* c = const_cast<cec_codec*>(cc);
    const size_t d = c->d, t = c->d + c->p;
    // Validate every part before launching anything.
    for (size_t k = 0; k < b->n_parts; ++k) {
        size_t n_present = 0;
        for (size_t i = 0; i < t; ++i) n_present += present[k * t + i] ? 1 : 0;
        if (n_present != t && n_present < d) return CEC_TOO_FEW_SHARDS_PRESENT;
    }
    // Group parts by pattern; bucket patterns by output-row count.
    std::map<PatternKey, std::pair<uint32_t, std::vector<uint32_t>>> groups;  // key -> (n_out, parts)
    for (size_t k = 0; k < b->n_parts; ++k) {
        const uint8_t* pr = present + k * t;
        size_t n_present = 0;
        for (size_t i = 0; i < t; ++i) n_present += pr[i] ? 1 : 0;
        if (n_present == t) continue;
        PatternKey key = make_key(pr, t, data_only != 0);
        auto& g = groups[key];
        g.second.push_back(uint32_t(k));
    }
    if (groups.empty()) return CEC_OK;
    // words = [records...][launch lists: part_ids..., part_pat...].  Patterns of up to
    // max_var_rows() rows (every RS(10,4) erasure set) share ONE launch that dispatches on each
    // part's row count; wider patterns get a row-group launch per row count.
    std::vector<uint32_t> words;
    std::map<uint32_t, std::pair<std::vector<uint32_t>, std::vector<uint32_t>>> buckets;
    uint32_t var_rows = 0;  // the shared launch's widest pattern: its kernel's row class
    for (auto& kv : groups) {
        auto rec = c->decode_record(kv.first);
        const uint32_t n_out = (*rec)[0];
        if (n_out == 0) continue;  // data_only: only parity missing, nothing to do
        if (n_out <= max_var_rows()) var_rows = std::max(var_rows, n_out);
        const uint32_t off = uint32_t(words.size());
        words.insert(words.end(), rec->begin(), rec->end());
        auto& bk = buckets[n_out <= max_var_rows() ? 0u : n_out];  // 0 = the shared launch
        for (uint32_t part : kv.second.second) {
            bk.first.push_back(part);
            bk.second.push_back(off);
        }
    }
    if (buckets.empty()) return CEC_OK;
    struct Launch {
        uint32_t n_out;  // 0: per-part row counts (launch_rs_apply_var)
        size_t ids;      // word offset of part_ids
        size_t count;
    };
    std::vector<Launch> launches;
    for (auto& kv : buckets) {
        launches.push_back({kv.first, words.size(), kv.second.first.size()});
        words.insert(words.end(), kv.second.first.begin(), kv.second.first.end());
        words.insert(words.end(), kv.second.second.begin(), kv.second.second.end());
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    uint32_t* dwords = nullptr;
    Scratch scratch;  // released on s behind the launches below
    CEC_TRY(upload_words(words, s, scratch, &dwords));
    const bool vec = aligned16(b->base, b->part_stride, b->chunk_stride);
    int status = CEC_OK;
    for (size_t i = 0; i < launches.size() && status == CEC_OK; ++i) {
        ApplyParams a{};
        a.base = b->base;
        a.part_stride = b->part_stride;
        a.chunk_stride = b->chunk_stride;
        a.len = b->chunk_len;
        a.pat = dwords;
        a.part_ids = dwords + launches[i].ids;
        a.part_pat = dwords + launches[i].ids + launches[i].count;
        a.n_parts = uint32_t(launches[i].count);
        a.d = uint32_t(d);
        a.n_rows = launches[i].n_out ? launches[i].n_out : var_rows;
        if (!launches[i].n_out) {
            // the shared launch's row class must cover every record it lists (the kernel skips
            // a wider pattern without writing its chunks: kernels.hpp launch_rs_apply_var)
            const uint32_t* pat_off = words.data() + launches[i].ids + launches[i].count;
            for (size_t q = 0; q < launches[i].count; ++q)
                if (words[pat_off[q]] == 0 || words[pat_off[q]] > a.n_rows) {
                    g_last_error = "reconstruct_batch: a listed pattern is wider than its launch";
                    return CEC_ERR_INVALID_ARGUMENT;
                }
        }
        a.lds_reserve = lds_reserve;
        hipError_t e = launches[i].n_out ? launch_rs_apply(a, vec, s)
                                         : launch_rs_apply_var(a, vec, s);
        if (e != hipSuccess) status = hip_fail(e, "launch_rs_apply");
    }
    return status;
}

int cec_reconstruct_batch(const cec_codec* c, const cec_part_batch* b, const uint8_t* present,
                          int data_only, void* stream) {
    return reconstruct_batch(c, b, present, data_only, stream, 0);
}

int cec_verify_batch(const cec_part_batch* b, size_t first_chunk, size_t n_chunks,
                     const uint8_t* present, const uint8_t* expected, uint8_t* ok, void* stream) {
    CEC_TRY(batch_ok(b));
    if (!expected || !ok) return CEC_ERR_INVALID_ARGUMENT;
    if (b->n_parts == 0 || n_chunks == 0) return CEC_OK;
    if (b->n_parts * n_chunks > 0xFFFFFFFFull) return CEC_ERR_INVALID_ARGUMENT;
    ShaParams h{};
    h.base = b->base;
    h.part_stride = b->part_stride;
    h.chunk_stride = b->chunk_stride;
    h.len = b->chunk_len;
    h.n_parts = uint32_t(b->n_parts);
    h.first_chunk = uint32_t(first_chunk);
    h.n_chunks = uint32_t(n_chunks);
    h.present = present;
    h.expected = expected;
    h.ok = ok;
    HIP_TRY(launch_sha256(h, aligned16(b->base, b->part_stride, b->chunk_stride),
                          static_cast<hipStream_t>(stream)));
    return CEC_OK;
}

}  // extern "C"

namespace {

// Side stream of the speculative decode in cec_read_batch / cec_resilver_batch, with the
// fork/join events that order it against the caller's stream: leased per call from a bounded
// per-device pool (see CtxPool for why not thread_local).
struct SideCtx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    void destroy() {
        if (stream) {
            (void)hipStreamSynchronize(stream);
            (void)hipStreamDestroy(stream);
        }
        if (fork) (void)hipEventDestroy(fork);
        if (join) (void)hipEventDestroy(join);
        stream = nullptr;
        fork = join = nullptr;
    }
};

class SidePool {
   public:
    std::unique_ptr<SideCtx> take(int device) {
        std::lock_guard<std::mutex> lk(mu_);
        auto& v = idle_[device];
        if (v.empty()) {
            auto c = std::make_unique<SideCtx>();
            c->device = device;
            return c;
        }
        auto c = std::move(v.back());
        v.pop_back();
        return c;
    }
    void give(std::unique_ptr<SideCtx> c) {
        if (!c) return;
        {
            std::lock_guard<std::mutex> lk(mu_);
            auto& v = idle_[c->device];
            if (v.size() < kMaxIdleCtx) {
                v.push_back(std::move(c));
                return;
            }
        }
        c->destroy();
    }

   private:
    std::mutex mu_;
    std::map<int, std::vector<std::unique_ptr<SideCtx>>> idle_;
};

SidePool& side_pool() {
    static SidePool* pool = new SidePool();  // leaked: see ctx_pool()
    return *pool;
}

class SideLease {
   public:
    SideLease() = default;
    SideLease(const SideLease&) = delete;
    SideLease& operator=(const SideLease&) = delete;
    ~SideLease() { side_pool().give(std::move(c_)); }
    int acquire() {
        int dev = 0;
        CEC_TRY(current_device(&dev));
        c_ = side_pool().take(dev);
        if (!c_->stream) HIP_TRY(hipStreamCreateWithFlags(&c_->stream, hipStreamNonBlocking));
        if (!c_->fork) HIP_TRY(hipEventCreateWithFlags(&c_->fork, hipEventDisableTiming));
        if (!c_->join) HIP_TRY(hipEventCreateWithFlags(&c_->join, hipEventDisableTiming));
        return CEC_OK;
    }
    SideCtx* get() { return c_.get(); }

   private:
    std::unique_ptr<SideCtx> c_;
};

// LDS each speculative-decode block reserves (A/B knob CEC_SPEC_LDS_KIB).  100 KiB keeps decode
// blocks off the CUs holding SHA workgroups (>= 64 KiB each) and runs one per free CU: a
// low-intensity decode spread under the SHA chains.  Measured on the c3r read (4 096 parts,
// RS(10,4), d loaded, tools/c3r_ab.sh): 43.2 ms vs 45.3 (65 KiB: two per free CU) vs 46.5 (none:
// decode everywhere, done in 17 ms, but the SHA chains slow from 42.6 to 46.4 ms beside it) vs
// 53.0 ms without speculation.
uint32_t decode_lds() { return knobs().spec_lds; }

// CEC_READ_SPECULATE=0 (A/B knob): verify, wait, then decode from the verified chunks only.
bool read_speculate() { return knobs().read_speculate; }

// A loaded chunk is hashed unless the caller marked it CEC_PRESENT_VERIFIED (a read retry's
// chunks that an earlier pass already verified).
inline bool needs_hash(uint8_t f) { return f != 0 && f != CEC_PRESENT_VERIFIED; }

// DataVerifier::verify of the loaded chunks (present_host[k*t + i] != 0) of a batch: ok[item] =
// digest matches (ok of the others is left as is).  The loaded chunks are packed into a
// compacted item list, so a read with d of d+p chunks loaded runs d/(d+p) of the waves of a
// strided launch with skipped lanes (a SHA wave costs the same with idle lanes), which leaves
// SIMDs free for the decode running beside it.
int verify_loaded(const cec_part_batch* b, size_t t, const uint8_t* present_host,
                  const uint8_t* expected, uint8_t* ok, hipStream_t s) {
    const size_t n = b->n_parts * t;
    if (!knobs().verify_compact) {  // A/B: strided launch with the skipped lanes
        std::vector<uint32_t> mask(n);  // chunks to hash: loaded, not already verified
        for (size_t i = 0; i < n; ++i) mask[i] = needs_hash(present_host[i]) ? 1u : 0u;
        std::vector<uint8_t> bytes(n);
        for (size_t i = 0; i < n; ++i) bytes[i] = uint8_t(mask[i]);
        Scratch sc;
        CEC_TRY(sc.acquire(n, s));
        std::memcpy(sc.host(), bytes.data(), n);
        HIP_TRY(hipMemcpyAsync(sc.dev(), sc.host(), n, hipMemcpyHostToDevice, s));
        CEC_TRY(cec_verify_batch(b, 0, t, sc.dev(), expected, ok, s));
        return CEC_OK;
    }
    std::vector<uint32_t> items;
    items.reserve(n);
    for (size_t i = 0; i < n; ++i)
        if (needs_hash(present_host[i])) items.push_back(uint32_t(i));
    if (items.empty()) return CEC_OK;
    const uint32_t n_items = uint32_t(items.size());
    uint32_t* ditems = nullptr;
    Scratch sc;  // released on s behind the verification launch
    CEC_TRY(upload_words(items, s, sc, &ditems));
    ShaParams h{};
    h.base = b->base;
    h.part_stride = b->part_stride;
    h.chunk_stride = b->chunk_stride;
    h.len = b->chunk_len;
    h.n_parts = uint32_t(b->n_parts);
    h.first_chunk = 0;
    h.n_chunks = uint32_t(t);
    h.expected = expected;
    h.ok = ok;
    h.items = ditems;
    h.n_items = n_items;
    hipError_t e = launch_sha256(h, aligned16(b->base, b->part_stride, b->chunk_stride), s);
    if (e != hipSuccess) return hip_fail(e, "launch_sha256 (verify)");
    return CEC_OK;
}

// Shared body of cec_read_batch / cec_resilver_batch.  The result is the reference's: rebuild
// from the first d VERIFIED chunks of each part (file_part.rs:98-128 keeps only chunks whose hash
// matched).  The decode does not wait for the verdict: the pattern is known from the loaded
// flags, so it runs speculatively from the first d LOADED chunks on a side stream, concurrently
// with the SHA-256 verification (which leaves 384 of 1 024 SIMDs idle on a 4 096-part RS(10,4)
// read: 40 960 chains = 640 waves).  Both only read the loaded chunks and the decode writes only
// chunks that were not loaded, so they do not race.  When every loaded chunk verifies (the
// common case) the speculative result is the final one; a part with a loaded chunk that failed
// is decoded again from its verified chunks, which rewrites every chunk the first pass wrote.
int verify_then_reconstruct(const cec_codec* c, const cec_part_batch* b,
                            const uint8_t* present_host, const uint8_t* expected,
                            uint8_t* verified_host, int* part_status, bool data_only,
                            hipStream_t s) {
    if (!c || !present_host || !expected || !verified_host || !part_status)
        return CEC_ERR_INVALID_ARGUMENT;
    CEC_TRY(batch_ok(b));
    if (b->n_parts == 0) return CEC_OK;
    if (b->chunk_len == 0) return CEC_EMPTY_SHARD;
    const size_t d = c->d, t = c->d + c->p, n = b->n_parts * t;
    if (n > 0xFFFFFFFFull) return CEC_ERR_INVALID_ARGUMENT;
    const bool speculate = read_speculate();
    Scratch ok_buf;  // device verification flags, released on s behind the readback
    CEC_TRY(ok_buf.acquire(n, s));
    uint8_t* ok = ok_buf.dev();
    HIP_TRY(hipMemsetAsync(ok, 0, n, s));
    // Fork point: the caller's work on s so far (the chunks).  The side stream waits for it and
    // s later waits for the side stream's join, each on an event recorded before the wait is
    // queued: safe in shared in-order hardware queues (the rule of the coalescer's early parity
    // download above).
    SideLease lease;
    SideCtx* side = nullptr;
    if (speculate) {
        CEC_TRY(lease.acquire());
        side = lease.get();
        HIP_TRY(hipEventRecord(side->fork, s));
    }
    // Verification goes first so its long-lived workgroups claim their CUs (one or two per CU)
    // before the decode's blocks take the CUs left free.
    int st = verify_loaded(b, t, present_host, expected, ok, s);
    if (st == CEC_OK && speculate) {
        // Parts with fewer than d loaded chunks cannot be decoded: left out (mask all ones).
        std::vector<uint8_t> spec(present_host, present_host + n);
        for (size_t k = 0; k < b->n_parts; ++k) {
            const size_t loaded =
                size_t(std::count_if(spec.begin() + k * t, spec.begin() + (k + 1) * t,
                                     [](uint8_t f) { return f != 0; }));
            if (loaded < d) std::fill(spec.begin() + k * t, spec.begin() + (k + 1) * t, uint8_t(1));
        }
        hipError_t e = hipStreamWaitEvent(side->stream, side->fork, 0);
        if (e != hipSuccess) st = hip_fail(e, "speculative decode fork");
        if (st == CEC_OK)
            st = reconstruct_batch(c, b, spec.data(), data_only ? 1 : 0, side->stream,
                                   decode_lds());
        if (st == CEC_OK) {
            e = hipEventRecord(side->join, side->stream);
            if (e == hipSuccess) e = hipStreamWaitEvent(s, side->join, 0);
            if (e != hipSuccess) st = hip_fail(e, "speculative decode join");
        }
        // On failure nothing joins the side stream: let what it launched finish before the
        // caller gets its buffers back.
        if (st != CEC_OK) (void)hipStreamSynchronize(side->stream);
    }
    if (st == CEC_OK) {
        hipError_t e = hipMemcpyAsync(verified_host, ok, n, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) st = hip_fail(e, "verify readback");
    }
    if (st != CEC_OK) return st;
    for (size_t i = 0; i < n; ++i)  // verified by an earlier pass: trusted, not hashed again
        if (present_host[i] == CEC_PRESENT_VERIFIED) verified_host[i] = 1;
    // Parts with fewer than d verified chunks cannot be decoded (the reference's read returns
    // the part short / resilver reports it).  Decode (again) the parts whose loaded chunks did
    // not all verify — or every part, without speculation.
    std::vector<uint8_t> pres(n, uint8_t(1));
    bool any = false;
    for (size_t k = 0; k < b->n_parts; ++k) {
        size_t good = 0;
        bool bad = false;
        for (size_t i = 0; i < t; ++i) {
            good += verified_host[k * t + i] ? 1 : 0;
            bad |= present_host[k * t + i] && !verified_host[k * t + i];
        }
        part_status[k] = good >= d ? CEC_OK : CEC_TOO_FEW_SHARDS_PRESENT;
        if (good >= d && (bad || !speculate)) {
            std::copy(verified_host + k * t, verified_host + (k + 1) * t, pres.begin() + k * t);
            any = true;
        }
    }
    return any ? cec_reconstruct_batch(c, b, pres.data(), data_only ? 1 : 0, s) : CEC_OK;
}

}  // namespace

extern "C" {

int cec_read_batch(const cec_codec* c, const cec_part_batch* b, const uint8_t* present,
                   const uint8_t* expected, uint8_t* verified, int* part_status, void* stream) {
    return verify_then_reconstruct(c, b, present, expected, verified, part_status, true,
                                   static_cast<hipStream_t>(stream));
}

int cec_resilver_batch(const cec_codec* c, const cec_part_batch* b, const uint8_t* present,
                       const uint8_t* expected, uint8_t* verified, int* part_status,
                       void* stream) {
    return verify_then_reconstruct(c, b, present, expected, verified, part_status, false,
                                   static_cast<hipStream_t>(stream));
}

// ------------------------------------------------------------------------------------------
// Utilities
// ------------------------------------------------------------------------------------------

int cec_fill_synthetic(const cec_part_batch* b, size_t n_chunks, uint64_t seed, void* stream) {
    CEC_TRY(batch_ok(b));
    if (b->n_parts > 0xFFFFFFFFull || n_chunks > 0xFFFFFFFFull) return CEC_ERR_INVALID_ARGUMENT;
    FillParams f{};
    f.base = b->base;
    f.part_stride = b->part_stride;
    f.chunk_stride = b->chunk_stride;
    f.len = b->chunk_len;
    f.seed = seed;
    f.n_parts = uint32_t(b->n_parts);
    f.n_chunks = uint32_t(n_chunks);
    HIP_TRY(launch_fill(f, static_cast<hipStream_t>(stream)));
    return CEC_OK;
}

uint8_t cec_synth_byte(uint64_t seed, uint64_t part, uint64_t chunk, uint64_t offset) {
    return synth_byte(seed, part, chunk, offset);
}

}  // extern "C"
