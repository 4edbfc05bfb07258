// pipeline.cpp — host-staged write pipeline (cec_pipeline_*): the batched form of
// FileWriteBuilder::write's part loop (reference src/file/writer.rs:166-231: read d*chunk_size
// bytes per part, encode + hash each part, hand back parity and digests in order).
//
// A pipeline owns `depth` slots on one GPU.  Each slot has a device batch, its own HIP stream
// and (unless created with CEC_PIPE_EXTERNAL) pinned host buffers the caller writes part data
// straight into.  H2D (one 2-D copy scattering [part][d][L] into the device's [part][d+p][L]),
// the fused encode_hash kernel, and D2H of parity + digests are queued on the slot's stream, so
// the copies of one slot overlap the kernels of the others.  A batch's kernel time is the
// per-chunk serial SHA-256 time whatever its part count (sha256_kernels.hip), so several modest
// batches in flight on separate streams (their workgroups run on disjoint CUs) keep the PCIe link
// busy.  submit_from takes the caller's own (ideally pinned: cec_host_alloc) buffers instead of
// the slot's, so the copy engines DMA straight from / into them with no host copy at all.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <deque>
#include <cstring>
#include <string>
#include <vector>

#include "chunky_ec.h"
#include "hostmem.hpp"
#include "kernels.hpp"
#include "pipeline_internal.hpp"

namespace {

thread_local std::string g_pipe_error;

int pipe_fail(hipError_t e, const char* what) {
    g_pipe_error = std::string(what) + ": " + hipGetErrorString(e);
    return e == hipErrorOutOfMemory ? CEC_ERR_OUT_OF_MEMORY : CEC_ERR_HIP;
}

#define PIPE_TRY(expr)                                      \
    do {                                                    \
        hipError_t _e = (expr);                             \
        if (_e != hipSuccess) return pipe_fail(_e, #expr);  \
    } while (0)

// Makes `device` current for a scope and restores the caller's device on every exit path
// (early error returns included).
class DeviceGuard {
   public:
    explicit DeviceGuard(int device) {
        err_ = hipGetDevice(&prev_);
        if (err_ == hipSuccess && prev_ != device) {
            err_ = hipSetDevice(device);
            switched_ = err_ == hipSuccess;
        }
    }
    ~DeviceGuard() {
        if (switched_) (void)hipSetDevice(prev_);
    }
    hipError_t status() const { return err_; }

   private:
    int prev_ = 0;
    bool switched_ = false;
    hipError_t err_ = hipSuccess;
};

// A slot's stream: a plain non-blocking stream.  HIP maps streams onto GPU_MAX_HW_QUEUES (4 by
// default) hardware queues per process, so two slots can share a queue; the carry stash is queued
// in the batch's own stream for that reason (see cec_read_pipeline::carry_stash).  Streams are
// made only when a pipeline is made, and a cec_multi makes its pipelines before any job runs
// (multi.cpp): making streams while other queues of the process were busy is what deadlocked the
// round-5 scheduler (profiles/HISTORY.md, "slot queues").
hipError_t slot_stream(hipStream_t* stream) {
    return hipStreamCreateWithFlags(stream, hipStreamNonBlocking);
}

// Pipelines made by this process (both kinds): tests check that a scheduler makes its pipelines
// once, up front (cec_pipelines_made).
std::atomic<uint64_t> g_pipelines_made{0};

struct Slot {
    uint8_t* h_data = nullptr;    // pinned [parts][d][L] (null with CEC_PIPE_EXTERNAL)
    uint8_t* h_parity = nullptr;  // pinned [parts][p][L] (null with CEC_PIPE_EXTERNAL)
    uint8_t* h_dig = nullptr;     // pinned [parts][d+p][32]
    uint8_t* d_buf = nullptr;     // device [parts][d+p][cs]
    uint8_t* d_dig = nullptr;     // device [parts][d+p][32]
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    bool in_flight = false;
    size_t n_parts = 0;
    uint8_t* out_parity = nullptr;  // where this batch's parity / digests go
    uint8_t* out_dig = nullptr;
};

}  // namespace

struct cec_pipeline {
    const cec_codec* codec = nullptr;
    int device = 0;
    size_t d = 0, p = 0, t = 0, L = 0, cs = 0, parts = 0;
    bool external = false;
    std::vector<Slot> slots;
    size_t next = 0;

    ~cec_pipeline() {
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) return;
        (void)hipSetDevice(device);
        for (Slot& s : slots) {
            if (s.stream) (void)hipStreamSynchronize(s.stream);
            if (s.done) (void)hipEventDestroy(s.done);
            if (s.stream) (void)hipStreamDestroy(s.stream);
            if (s.d_buf) (void)hipFree(s.d_buf);
            if (s.d_dig) (void)hipFree(s.d_dig);
            if (s.h_data) (void)hipHostFree(s.h_data);
            if (s.h_parity) (void)hipHostFree(s.h_parity);
            if (s.h_dig) (void)hipHostFree(s.h_dig);
        }
        (void)hipSetDevice(cur);
    }

    // Queue one batch: data [n][d][L] host -> device, encode + hash, parity [n][p][L] and
    // digests [n][d+p][32] back to host.
    int submit(Slot& s, const uint8_t* data, size_t n_parts, uint8_t* parity, uint8_t* dig) {
        DeviceGuard guard(device);
        PIPE_TRY(guard.status());
        const size_t dw = d * L, pitch = t * cs;
        if (cs == L) {
            PIPE_TRY(hipMemcpy2DAsync(s.d_buf, pitch, data, dw, dw, n_parts, hipMemcpyHostToDevice,
                                      s.stream));
        } else {  // chunk stride padded past L: one 2-D copy per data chunk column
            for (size_t j = 0; j < d; ++j)
                PIPE_TRY(hipMemcpy2DAsync(s.d_buf + j * cs, pitch, data + j * L, dw, L, n_parts,
                                          hipMemcpyHostToDevice, s.stream));
        }
        cec_part_batch b{s.d_buf, pitch, cs, n_parts, L};
        int st = cec_encode_hash_batch(codec, &b, s.d_dig, s.stream);
        if (st != CEC_OK) {
            g_pipe_error = cec_last_error();
            return st;
        }
        const size_t pw = p * L;
        if (cs == L) {
            PIPE_TRY(hipMemcpy2DAsync(parity, pw, s.d_buf + dw, pitch, pw, n_parts,
                                      hipMemcpyDeviceToHost, s.stream));
        } else {
            for (size_t i = 0; i < p; ++i)
                PIPE_TRY(hipMemcpy2DAsync(parity + i * L, pw, s.d_buf + (d + i) * cs, pitch, L,
                                          n_parts, hipMemcpyDeviceToHost, s.stream));
        }
        PIPE_TRY(hipMemcpyAsync(dig, s.d_dig, n_parts * t * 32, hipMemcpyDeviceToHost, s.stream));
        PIPE_TRY(hipEventRecord(s.done, s.stream));
        s.in_flight = true;
        s.n_parts = n_parts;
        s.out_parity = parity;
        s.out_dig = dig;
        return CEC_OK;
    }
};

extern "C" {

const char* cec_pipeline_last_error(void) { return g_pipe_error.c_str(); }

int cec_pipeline_new(const cec_codec* codec, size_t chunk_len, size_t parts_per_batch,
                     size_t depth, cec_pipeline** out) {
    return cec_pipeline_new_ex(codec, chunk_len, parts_per_batch, depth, 0u, out);
}

int cec_pipeline_new_ex(const cec_codec* codec, size_t chunk_len, size_t parts_per_batch,
                        size_t depth, unsigned flags, cec_pipeline** out) {
    if (!codec || !out || chunk_len == 0 || parts_per_batch == 0 || depth == 0 || depth > 16 ||
        (flags & ~unsigned(CEC_PIPE_EXTERNAL)))
        return CEC_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    if (cec_device_count() <= 0) return CEC_ERR_NO_DEVICE;
    auto* pl = new cec_pipeline();
    pl->codec = codec;
    PIPE_TRY(hipGetDevice(&pl->device));
    pl->d = cec_codec_data_shards(codec);
    pl->p = cec_codec_parity_shards(codec);
    pl->t = pl->d + pl->p;
    pl->L = chunk_len;
    pl->cs = (chunk_len + 255) / 256 * 256;
    pl->parts = parts_per_batch;
    pl->external = (flags & CEC_PIPE_EXTERNAL) != 0;
    pl->slots.resize(depth);
    for (Slot& s : pl->slots) {
        hipError_t e = hipSuccess;
        auto host = [&](uint8_t** ptr, size_t bytes) {  // pinned, on the device's NUMA node
            if (e == hipSuccess)
                e = cec::host_malloc_near(reinterpret_cast<void**>(ptr), bytes,
                                          hipHostMallocDefault, pl->device);
        };
        if (!pl->external) {
            host(&s.h_data, pl->parts * pl->d * pl->L);
            host(&s.h_parity, pl->parts * pl->p * pl->L);
        }
        host(&s.h_dig, pl->parts * pl->t * 32);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s.d_buf), pl->parts * pl->t * pl->cs);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s.d_dig), pl->parts * pl->t * 32);
        if (e == hipSuccess) e = slot_stream(&s.stream);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
        if (e != hipSuccess) {
            delete pl;
            return pipe_fail(e, "cec_pipeline_new allocation");
        }
    }
    g_pipelines_made.fetch_add(1, std::memory_order_relaxed);
    *out = pl;
    return CEC_OK;
}

uint64_t cec_pipelines_made(void) { return g_pipelines_made.load(std::memory_order_relaxed); }

void cec_pipeline_free(cec_pipeline* pl) { delete pl; }

size_t cec_pipeline_depth(const cec_pipeline* pl) { return pl ? pl->slots.size() : 0; }

// Next slot in round-robin order; waits for that slot's previous batch to finish, after which
// its previous results are no longer valid.  *data receives the pinned [parts][d][L] buffer
// (null for a CEC_PIPE_EXTERNAL pipeline: use submit_from).
int cec_pipeline_acquire(cec_pipeline* pl, size_t* slot, uint8_t** data) {
    if (!pl || !slot || !data) return CEC_ERR_INVALID_ARGUMENT;
    const size_t i = pl->next;
    pl->next = (pl->next + 1) % pl->slots.size();
    Slot& s = pl->slots[i];
    if (s.in_flight) {
        PIPE_TRY(hipEventSynchronize(s.done));
        s.in_flight = false;
    }
    *slot = i;
    *data = s.h_data;
    return CEC_OK;
}

// Queue one batch of n_parts (<= parts_per_batch) parts whose data the caller wrote into the
// slot's pinned buffer: H2D, fused encode + SHA-256 of all d+p chunks, D2H parity + digests.
int cec_pipeline_submit(cec_pipeline* pl, size_t slot, size_t n_parts) {
    if (!pl || slot >= pl->slots.size() || n_parts == 0 || n_parts > pl->parts || pl->external)
        return CEC_ERR_INVALID_ARGUMENT;
    Slot& s = pl->slots[slot];
    return pl->submit(s, s.h_data, n_parts, s.h_parity, s.h_dig);
}

int cec_pipeline_submit_from(cec_pipeline* pl, size_t slot, const uint8_t* data, size_t n_parts,
                             uint8_t* parity_out, uint8_t* digests_out) {
    if (!pl || slot >= pl->slots.size() || !data || n_parts == 0 || n_parts > pl->parts)
        return CEC_ERR_INVALID_ARGUMENT;
    Slot& s = pl->slots[slot];
    if (!parity_out && !s.h_parity) return CEC_ERR_INVALID_ARGUMENT;
    return pl->submit(s, data, n_parts, parity_out ? parity_out : s.h_parity,
                      digests_out ? digests_out : s.h_dig);
}

// Wait for a submitted slot; *parity = [parts][p][L], *digests = [parts][d+p][32] (chunks in
// order) where submit / submit_from put them.  Valid until the slot is acquired again.
int cec_pipeline_wait(cec_pipeline* pl, size_t slot, const uint8_t** parity,
                      const uint8_t** digests, size_t* n_parts) {
    if (!pl || slot >= pl->slots.size()) return CEC_ERR_INVALID_ARGUMENT;
    Slot& s = pl->slots[slot];
    if (s.in_flight) {
        PIPE_TRY(hipEventSynchronize(s.done));
        s.in_flight = false;
    }
    if (parity) *parity = s.out_parity ? s.out_parity : s.h_parity;
    if (digests) *digests = s.out_dig ? s.out_dig : s.h_dig;
    if (n_parts) *n_parts = s.n_parts;
    return CEC_OK;
}

// 1 when the slot's batch is complete (or none is in flight), 0 while it runs; never blocks.
int cec_pipeline_query(cec_pipeline* pl, size_t slot) {
    if (!pl || slot >= pl->slots.size()) return CEC_ERR_INVALID_ARGUMENT;
    Slot& s = pl->slots[slot];
    if (!s.in_flight) return 1;
    const hipError_t e = hipEventQuery(s.done);
    (void)hipGetLastError();
    return e == hipErrorNotReady ? 0 : 1;
}

// Wait for every slot.
int cec_pipeline_drain(cec_pipeline* pl) {
    if (!pl) return CEC_ERR_INVALID_ARGUMENT;
    for (Slot& s : pl->slots) {
        if (s.in_flight) {
            PIPE_TRY(hipEventSynchronize(s.done));
            s.in_flight = false;
        }
    }
    return CEC_OK;
}

}  // extern "C"


// ------------------------------------------------------------------------------------------
// Read pipeline (cec_read_pipeline_*): the batched form of FileReadBuilder's part loop
// (reference src/file/reader.rs:40-75, buffered(5) reads of FilePart::read_with_context,
// file_part.rs:73-135): per part, the chunks the caller could load, verified against their
// metadata digests, and the d data chunks rebuilt from the verified ones.
//
// Per slot, asynchronously on the slot's stream: the loaded chunks go up (one copy per run of
// consecutive loaded chunks, or one copy of a packed batch), the SHA-256 kernel verifies every
// loaded chunk against its expected digest, and the missing data chunks are rebuilt
// SPECULATIVELY from the first d loaded chunks (the pattern is known at submit time, so no host
// round trip sits between verification and decode); the d data chunks and the verification flags
// come back.  wait() checks the flags: a part whose loaded chunks all verified is done (the
// common case); a part with a chunk that failed is decoded again from its verified chunks only
// (or reported TooFewShardsPresent when fewer than d verify) before wait() returns.
//
// The mode (read, REBUILT_ONLY, RESILVER, VERIFY_ONLY) is a property of each SUBMIT (the
// pipeline's creation flags are only the default of the older entry points): the device buffers
// are the same for every mode, so one pipeline serves FilePart's verify, resilver and read in
// turn without being rebuilt (file_part.rs:228-390 runs them on the same parts).
// ------------------------------------------------------------------------------------------

namespace {

constexpr unsigned kModeBits = CEC_READ_REBUILT_ONLY | CEC_READ_RESILVER | CEC_READ_VERIFY_ONLY;

struct ReadSlot {
    uint8_t* h_chunks = nullptr;    // pinned [parts][t][L]   (caller: loaded chunk bytes)
    uint8_t* h_present = nullptr;   // pinned [parts][t]      (caller: nonzero = loaded)
    uint8_t* h_expected = nullptr;  // pinned [parts][t][32]  (caller: metadata digests)
    uint8_t* h_data = nullptr;      // pinned [parts][out][L] (result: data / rebuilt chunks)
    uint8_t* h_ok = nullptr;        // pinned [parts][t]      (result: verified flags)
    uint8_t* h_hash = nullptr;      // pinned [parts][t]      chunks to hash (loaded, not
                                    //                        CEC_PRESENT_VERIFIED)
    int* h_status = nullptr;        // host [parts]
    uint8_t* d_buf = nullptr;       // device [parts][t][cs]
    uint8_t* d_expected = nullptr;  // device [parts][t][32]
    uint8_t* d_flags = nullptr;     // device [parts][t] present, then [parts][t] ok
    uint8_t* d_pack = nullptr;      // device [parts*t][L]  packed upload (submit_packed; lazy)
    uint32_t* h_ids = nullptr;      // pinned [parts*t]     batch position of packed chunk j
    uint32_t* d_ids = nullptr;      // device [parts*t]
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    bool in_flight = false;
    bool checked = false;
    unsigned mode = 0;     // this batch's mode bits (kModeBits)
    bool stashed = false;  // this batch queued a carry stash
    size_t n_parts = 0;
    const uint8_t* src_chunks = nullptr;  // this batch's chunk bytes (h_chunks or the caller's)
    uint8_t* dst_data = nullptr;          // this batch's data output (h_data or the caller's)
    std::vector<uint8_t> decode_mask;  // present mask the speculative decode used
    std::vector<const uint8_t*> data_ptrs;  // [parts][out]: where each output chunk is
    std::vector<size_t> src_off;  // [parts][t]: byte offset of a loaded chunk in src_chunks
    // CEC_READ_CARRY: per part of this batch, the carry entry its verified chunks were kept in
    // (-1: none), and whether its CEC_PRESENT_VERIFIED chunks came from the carry pool at submit
    // (not from the caller's buffer: they are copied back like rebuilt ones)
    std::vector<int32_t> carry_ids;
    std::vector<uint8_t> carried;
    // pool entries this batch's stash may fill (kReserved); after wait, the entries of its
    // TooFewShardsPresent parts until the caller claims them (cec_read_pipeline_carry_ids) or
    // the slot's next submit gives them back
    std::vector<int32_t> reserved;
    // made with the pipeline: the consume's index lists ([0, parts*t) batch positions, then
    // pool positions), the reserved entries, the stash's part -> entry map, the loaded flags
    uint32_t* h_cids = nullptr;
    uint32_t* d_cids = nullptr;
    uint32_t* h_res = nullptr;
    uint32_t* d_res = nullptr;
    int32_t* h_map = nullptr;
    int32_t* d_map = nullptr;
    uint8_t* d_present = nullptr;
};

}  // namespace

struct cec_read_pipeline {
    const cec_codec* codec = nullptr;
    int device = 0;
    size_t d = 0, p = 0, t = 0, L = 0, cs = 0, parts = 0;
    // The creation flags' mode: what cec_read_pipeline_submit / submit_from / submit_packed /
    // submit_carried use.  Mode bits (per submit, cec_read_pipeline_submit_ex):
    //  CEC_READ_REBUILT_ONLY -- D2H only the data chunks rebuilt;
    //  CEC_READ_RESILVER     -- FilePart::resilver's compute (file_part.rs:253-308): every chunk
    //                           that did not verify (data AND parity) is rebuilt and comes back,
    //                           in a [parts][t][L] output; the verified ones stay where read;
    //  CEC_READ_VERIFY_ONLY  -- FilePart::verify's compute (file_part.rs:228-251): the loaded
    //                           chunks are hashed and compared, nothing is decoded or copied back.
    unsigned default_mode = 0;
    size_t h_out_chunks = 0;  // output chunks per part the slots' own h_data holds (0: none)
    bool external = false;    // CEC_PIPE_EXTERNAL: no pinned chunk / data slot buffers
    std::vector<ReadSlot> slots;
    size_t next = 0;
    // CEC_READ_CARRY: device pool of `carry_cap` entries of [t][cs] bytes (made with the
    // pipeline: a fresh multi-GiB allocation is cleared by the driver in the background, which
    // would compete with the uploads if it were made mid-stream) holding the verified chunks of
    // parts reported CEC_TOO_FEW_SHARDS_PRESENT until their retry takes them (or the caller
    // releases them).  Each batch reserves up to `carry_batch` free entries at submit and its
    // stash kernels fill them in the batch's own stream, right after the verification: the stash
    // needs no host round trip, and nothing the next uploads depend on is queued behind another
    // slot's batch (slot streams can share a hardware queue, where a kernel waits for every
    // packet queued before it).  Per entry an event after its last stash or consumption, so
    // reusing an entry waits for its previous copies.  carry_used: kFree, kHeld (a carry id the
    // caller has), kReserved (by a batch: in flight, or waited for and not yet claimed).  Per
    // entry, the chunks its stash kept (carry_mask [cap][t]) and the part's metadata digests
    // (carry_exp [cap][t][32]): a retry may take an entry only for the part it was kept for.
    static constexpr uint8_t kFree = 0, kHeld = 1, kReserved = 2;
    bool carry = false;
    size_t carry_batch = 0;
    size_t carry_cap = 0;
    uint8_t* d_carry = nullptr;
    std::vector<hipEvent_t> carry_ready;
    std::vector<uint8_t> carry_used;
    std::vector<uint8_t> carry_mask;
    std::vector<uint8_t> carry_exp;
    std::deque<int32_t> carry_free;

    static size_t out_chunks(unsigned mode, size_t d, size_t t) {
        return (mode & CEC_READ_VERIFY_ONLY) ? 0 : (mode & CEC_READ_RESILVER) ? t : d;
    }

    ~cec_read_pipeline() {
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) return;
        (void)hipSetDevice(device);
        for (ReadSlot& s : slots) {
            if (s.stream) (void)hipStreamSynchronize(s.stream);
            if (s.done) (void)hipEventDestroy(s.done);
            if (s.stream) (void)hipStreamDestroy(s.stream);
            for (void* dptr : {static_cast<void*>(s.d_buf), static_cast<void*>(s.d_expected),
                               static_cast<void*>(s.d_flags), static_cast<void*>(s.d_pack),
                               static_cast<void*>(s.d_ids), static_cast<void*>(s.d_cids),
                               static_cast<void*>(s.d_res), static_cast<void*>(s.d_map),
                               static_cast<void*>(s.d_present)})
                if (dptr) (void)hipFree(dptr);
            for (void* hptr : {static_cast<void*>(s.h_ids), static_cast<void*>(s.h_cids),
                               static_cast<void*>(s.h_res), static_cast<void*>(s.h_map)})
                if (hptr) (void)hipHostFree(hptr);
            for (uint8_t* hptr : {s.h_chunks, s.h_present, s.h_expected, s.h_data, s.h_ok, s.h_hash})
                if (hptr) (void)hipHostFree(hptr);
            delete[] s.h_status;
        }
        for (hipEvent_t ev : carry_ready)
            if (ev) (void)hipEventDestroy(ev);
        if (d_carry) (void)hipFree(d_carry);
        (void)hipSetDevice(cur);
    }

    // The carry pool, its events and every slot's carry buffers (at creation).
    hipError_t make_carry_pool() {
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&d_carry), carry_cap * t * cs);
        if (e != hipSuccess) {
            d_carry = nullptr;
            return e;
        }
        // touched once here, not by the first stashes mid-stream
        e = hipMemset(d_carry, 0, carry_cap * t * cs);
        if (e != hipSuccess) return e;
        carry_ready.assign(carry_cap, nullptr);
        for (auto& ev : carry_ready) {
            e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        carry_used.assign(carry_cap, kFree);
        carry_mask.assign(carry_cap * t, 0);
        carry_exp.assign(carry_cap * t * 32, 0);
        carry_free.clear();
        for (size_t i = 0; i < carry_cap; ++i) carry_free.push_back(int32_t(i));
        for (ReadSlot& s : slots) {
            auto dev = [&](void** ptr, size_t bytes) {
                if (e == hipSuccess) e = hipMalloc(ptr, bytes);
            };
            auto host = [&](void** ptr, size_t bytes) {
                if (e == hipSuccess) e = cec::host_malloc_near(ptr, bytes, hipHostMallocDefault, device);
            };
            dev(reinterpret_cast<void**>(&s.d_cids), 2 * parts * t * sizeof(uint32_t));
            host(reinterpret_cast<void**>(&s.h_cids), 2 * parts * t * sizeof(uint32_t));
            dev(reinterpret_cast<void**>(&s.d_res), carry_batch * sizeof(uint32_t));
            host(reinterpret_cast<void**>(&s.h_res), carry_batch * sizeof(uint32_t));
            dev(reinterpret_cast<void**>(&s.d_map), parts * sizeof(int32_t));
            host(reinterpret_cast<void**>(&s.h_map), parts * sizeof(int32_t));
            dev(reinterpret_cast<void**>(&s.d_present), parts * t);
        }
        return e;
    }

    // Entries the slot still reserves (its stash did not fill them, or the caller did not claim
    // them after wait) go back to the free list.
    void carry_unreserve(ReadSlot& s) {
        for (int32_t id : s.reserved)
            if (carry_used[size_t(id)] == kReserved) carry_give_back(id);
        s.reserved.clear();
    }
    void carry_give_back(int32_t id) {
        carry_used[size_t(id)] = kFree;
        carry_free.push_back(id);
    }
    bool carry_valid(int32_t id) const {  // a carry id the caller holds
        return id >= 0 && size_t(id) < carry_used.size() && carry_used[size_t(id)] == kHeld;
    }
    size_t held_entries() const {
        return size_t(std::count(carry_used.begin(), carry_used.end(), kHeld));
    }

    // Whether carry entry `id` was kept for part k of slot s as the slot's present / expected
    // arrays now describe it: the part's metadata digests are the ones stashed with the entry,
    // and every chunk it flags CEC_PRESENT_VERIFIED is one the stash kept.  Anything else would
    // decode stale bytes that are never hashed again.
    bool carry_matches(const ReadSlot& s, size_t k, int32_t id) const {
        const uint8_t* pr = s.h_present + k * t;
        const uint8_t* mask = carry_mask.data() + size_t(id) * t;
        for (size_t i = 0; i < t; ++i)
            if (pr[i] == CEC_PRESENT_VERIFIED && !mask[i]) return false;
        return std::memcmp(s.h_expected + k * t * 32, carry_exp.data() + size_t(id) * t * 32,
                           t * 32) == 0;
    }

    // The retry's consume: pairs[j] = (batch position, pool position), one move kernel launch
    // (pool -> d_buf) after the index lists go up, on the slot's stream.
    int carry_consume(ReadSlot& s, const std::vector<std::pair<uint32_t, uint32_t>>& pairs) const {
        const size_t m = pairs.size();
        if (!m) return CEC_OK;
        for (size_t j = 0; j < m; ++j) {
            s.h_cids[j] = pairs[j].first;
            s.h_cids[m + j] = pairs[j].second;
        }
        PIPE_TRY(hipMemcpyAsync(s.d_cids, s.h_cids, 2 * m * sizeof(uint32_t), hipMemcpyHostToDevice,
                                s.stream));
        cec::MoveParams mv{s.d_buf, t * cs, cs, uint32_t(t), d_carry, cs, s.d_cids, uint32_t(m), 1u,
                           s.d_cids + m};
        PIPE_TRY(cec::launch_move_chunks(mv, s.stream));
        return CEC_OK;
    }

    // The batch's stash (CEC_READ_CARRY, read modes), queued after its verification: reserve up
    // to carry_batch free entries (each waits for its last copies), let the stash kernels fill
    // them with the verified chunks of the parts that will come back TooFewShardsPresent, and
    // bring the part -> entry map back with the batch.
    int carry_stash(ReadSlot& s, size_t n_parts) {
        carry_unreserve(s);
        while (s.reserved.size() < carry_batch && !carry_free.empty()) {
            const int32_t id = carry_free.front();  // the entry freed longest ago first (FIFO)
            carry_free.pop_front();
            carry_used[size_t(id)] = kReserved;
            s.h_res[s.reserved.size()] = uint32_t(id);
            s.reserved.push_back(id);
            PIPE_TRY(hipStreamWaitEvent(s.stream, carry_ready[size_t(id)], 0));
        }
        const size_t n = n_parts * t;
        PIPE_TRY(hipMemcpyAsync(s.d_present, s.h_present, n, hipMemcpyHostToDevice, s.stream));
        if (!s.reserved.empty())
            PIPE_TRY(hipMemcpyAsync(s.d_res, s.h_res, s.reserved.size() * sizeof(uint32_t),
                                    hipMemcpyHostToDevice, s.stream));
        cec::CarryStashParams cp{s.d_buf, t * cs, cs, uint32_t(t), uint32_t(d), uint32_t(n_parts),
                                 d_carry, cs, s.d_present, s.d_flags + n, s.d_res,
                                 uint32_t(s.reserved.size()), s.d_map};
        PIPE_TRY(cec::launch_carry_stash(cp, s.stream));
        for (int32_t id : s.reserved) PIPE_TRY(hipEventRecord(carry_ready[size_t(id)], s.stream));
        PIPE_TRY(hipMemcpyAsync(s.h_map, s.d_map, n_parts * sizeof(int32_t), hipMemcpyDeviceToHost,
                                s.stream));
        s.stashed = true;
        return CEC_OK;
    }

    cec_part_batch batch(ReadSlot& s, size_t n) const {
        return cec_part_batch{s.d_buf, t * cs, cs, n, L};
    }

    // D2H of the data chunks of part k that were not loaded (the speculative decode rebuilt
    // them) into their data slots: one copy per run of consecutive missing data chunks.
    int copy_rebuilt_back(ReadSlot& s, size_t k) const {
        const uint8_t* pr = s.h_present + k * t;
        const bool carried = !s.carried.empty() && s.carried[k];
        // in the caller's buffer: loaded chunks, except those a carried part took from the pool
        auto held = [&](size_t j) { return pr[j] && !(carried && pr[j] == CEC_PRESENT_VERIFIED); };
        for (size_t j = 0; j < d;) {
            if (held(j)) {
                ++j;
                continue;
            }
            size_t e = j;
            while (e < d && !held(e)) ++e;
            uint8_t* dst = s.dst_data + (k * d + j) * L;
            const uint8_t* src = s.d_buf + (k * t + j) * cs;
            if (cs == L)
                PIPE_TRY(hipMemcpyAsync(dst, src, (e - j) * L, hipMemcpyDeviceToHost, s.stream));
            else
                PIPE_TRY(hipMemcpy2DAsync(dst, L, src, cs, L, e - j, hipMemcpyDeviceToHost,
                                          s.stream));
            j = e;
        }
        return CEC_OK;
    }

    // Resilver: D2H of the chunks of part k whose flag in `have` is 0 (rebuilt) into their
    // [t] output slots, one copy per run.
    int copy_missing_back(ReadSlot& s, size_t k, const uint8_t* have) const {
        for (size_t i = 0; i < t;) {
            if (have[i]) {
                ++i;
                continue;
            }
            size_t e = i;
            while (e < t && !have[e]) ++e;
            uint8_t* dst = s.dst_data + (k * t + i) * L;
            const uint8_t* src = s.d_buf + (k * t + i) * cs;
            if (cs == L)
                PIPE_TRY(hipMemcpyAsync(dst, src, (e - i) * L, hipMemcpyDeviceToHost, s.stream));
            else
                PIPE_TRY(hipMemcpy2DAsync(dst, L, src, cs, L, e - i, hipMemcpyDeviceToHost,
                                          s.stream));
            i = e;
        }
        return CEC_OK;
    }

    // D2H of the d data chunks of parts [k0, k0 + n) into the data output.
    int copy_data_back(ReadSlot& s, size_t k0, size_t n) const {
        const size_t pitch = t * cs, dw = d * L;
        if (cs == L) {
            PIPE_TRY(hipMemcpy2DAsync(s.dst_data + k0 * dw, dw, s.d_buf + k0 * pitch, pitch, dw, n,
                                      hipMemcpyDeviceToHost, s.stream));
        } else {
            for (size_t j = 0; j < d; ++j)
                PIPE_TRY(hipMemcpy2DAsync(s.dst_data + k0 * dw + j * L, dw,
                                          s.d_buf + k0 * pitch + j * cs, pitch, L, n,
                                          hipMemcpyDeviceToHost, s.stream));
        }
        return CEC_OK;
    }

    // Device / pinned buffers of the packed upload, made on a slot's first packed batch.
    int ensure_packed(ReadSlot& s) const {
        const size_t n = parts * t;
        hipError_t e = hipSuccess;  // each buffer made once (a failed call leaves the others)
        if (!s.d_ids) e = hipMalloc(reinterpret_cast<void**>(&s.d_ids), n * sizeof(uint32_t));
        if (e == hipSuccess && !s.h_ids)
            e = cec::host_malloc_near(reinterpret_cast<void**>(&s.h_ids), n * sizeof(uint32_t),
                                      hipHostMallocDefault, device);
        if (e == hipSuccess && !s.d_pack) e = hipMalloc(reinterpret_cast<void**>(&s.d_pack), n * L);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return pipe_fail(e, "read pipeline packed buffers");
        }
        return CEC_OK;
    }

    // Queue one batch whose present flags / expected digests are in the slot's pinned arrays.
    // packed: `chunks` holds the uploaded chunks back to back (part by part, ascending chunk
    // index), uploaded with ONE copy and placed by the move kernel; else chunk (k, i) is at
    // chunks + (k*t + i)*L and goes up with one copy per run of consecutive uploaded chunks.
    // carry_ids (CEC_READ_CARRY, nullable): per part, a carry entry whose chunks replace the
    // part's CEC_PRESENT_VERIFIED chunks (copied on the device; the caller's buffer need not hold
    // them, and a packed buffer leaves them out), or -1.
    int submit(ReadSlot& s, const uint8_t* chunks, size_t n_parts, uint8_t* data_out,
               unsigned mode, bool packed, const int32_t* carry_ids) {
        DeviceGuard guard(device);
        PIPE_TRY(guard.status());
        if (s.in_flight) {  // the slot's pinned arrays may still be read by its last batch
            PIPE_TRY(hipEventSynchronize(s.done));
            s.in_flight = false;
        }
        // a new batch on the slot: entries of its last one the caller did not claim go back
        if (carry) carry_unreserve(s);
        s.stashed = false;
        s.n_parts = 0;  // nothing valid on the slot until this batch is queued
        if ((mode & ~kModeBits) || ((mode & CEC_READ_RESILVER) && (mode & CEC_READ_VERIFY_ONLY))) {
            g_pipe_error = "invalid read mode";
            return CEC_ERR_INVALID_ARGUMENT;
        }
        const size_t out = out_chunks(mode, d, t);
        if (out && !data_out) {
            g_pipe_error = "no output buffer for this mode";
            return CEC_ERR_INVALID_ARGUMENT;
        }
        if (out && data_out == s.h_data && out > h_out_chunks) {
            g_pipe_error = "the slot's own output holds fewer chunks per part than this mode "
                           "writes: pass data_out";
            return CEC_ERR_INVALID_ARGUMENT;
        }
        const bool read_mode = !(mode & (CEC_READ_RESILVER | CEC_READ_VERIFY_ONLY));
        const size_t n = n_parts * t;
        s.carried.assign(carry_ids ? n_parts : 0, 0);
        if (carry_ids) {
            if (!carry || !read_mode) {
                g_pipe_error = "carry ids need CEC_READ_CARRY and a read mode";
                return CEC_ERR_INVALID_ARGUMENT;
            }
            for (size_t k = 0; k < n_parts; ++k) {
                if (carry_ids[k] < 0) continue;
                if (!carry_valid(carry_ids[k])) {
                    g_pipe_error = "carry id not held (already used or released)";
                    return CEC_ERR_INVALID_ARGUMENT;
                }
                for (size_t q = 0; q < k; ++q)
                    if (carry_ids[q] == carry_ids[k]) {
                        g_pipe_error = "carry id given twice";
                        return CEC_ERR_INVALID_ARGUMENT;
                    }
                if (!carry_matches(s, k, carry_ids[k])) {
                    g_pipe_error = "carry id was kept for another part (digests or verified "
                                   "chunks differ)";
                    return CEC_ERR_INVALID_ARGUMENT;
                }
                s.carried[k] = 1;
            }
        }
        s.mode = mode;
        s.src_chunks = chunks;
        s.dst_data = data_out;
        s.src_off.assign(n, 0);
        // chunks that come from the caller's buffer: loaded ones, except the verified chunks of
        // a carried part (those come from the carry pool, below)
        auto uploaded = [&](size_t x) {
            const uint8_t f = s.h_present[x];
            return f && !(!s.carried.empty() && s.carried[x / t] && f == CEC_PRESENT_VERIFIED);
        };
        if (packed) {
            const int est = ensure_packed(s);
            if (est != CEC_OK) return est;
            size_t m = 0;
            for (size_t x = 0; x < n; ++x)
                if (uploaded(x)) {
                    s.h_ids[m] = uint32_t(x);
                    s.src_off[x] = m * L;
                    ++m;
                }
            if (m) {
                PIPE_TRY(hipMemcpyAsync(s.d_pack, chunks, m * L, hipMemcpyHostToDevice, s.stream));
                PIPE_TRY(hipMemcpyAsync(s.d_ids, s.h_ids, m * sizeof(uint32_t),
                                        hipMemcpyHostToDevice, s.stream));
                cec::MoveParams mv{s.d_buf, t * cs, cs, uint32_t(t), s.d_pack, L, s.d_ids,
                                   uint32_t(m), 1u};
                PIPE_TRY(cec::launch_move_chunks(mv, s.stream));
            }
        } else {
            for (size_t x = 0; x < n; ++x) s.src_off[x] = x * L;
            // one copy per run of consecutive uploaded chunks of a part
            for (size_t k = 0; k < n_parts; ++k) {
                for (size_t i = 0; i < t;) {
                    if (!uploaded(k * t + i)) {
                        ++i;
                        continue;
                    }
                    size_t j = i;
                    while (j < t && uploaded(k * t + j)) ++j;
                    const uint8_t* src = chunks + (k * t + i) * L;
                    uint8_t* dst = s.d_buf + (k * t + i) * cs;
                    if (cs == L)
                        PIPE_TRY(hipMemcpyAsync(dst, src, (j - i) * L, hipMemcpyHostToDevice,
                                                s.stream));
                    else
                        PIPE_TRY(hipMemcpy2DAsync(dst, cs, src, L, L, j - i, hipMemcpyHostToDevice,
                                                  s.stream));
                    i = j;
                }
            }
        }
        // carried parts: their verified chunks come from the pool, one move launch queued after
        // the uploads (it writes only positions they do not); each entry waits for its stash and
        // is free again once this move has run
        if (!s.carried.empty()) {
            std::vector<std::pair<uint32_t, uint32_t>> pairs;
            for (size_t k = 0; k < n_parts; ++k) {
                if (!s.carried[k]) continue;
                const int32_t id = carry_ids[k];
                PIPE_TRY(hipStreamWaitEvent(s.stream, carry_ready[size_t(id)], 0));
                const uint8_t* pr = s.h_present + k * t;
                for (size_t i = 0; i < t; ++i)
                    if (pr[i] == CEC_PRESENT_VERIFIED)
                        pairs.emplace_back(uint32_t(k * t + i), uint32_t(size_t(id) * t + i));
            }
            const int mst = carry_consume(s, pairs);
            if (mst != CEC_OK) return mst;
            for (size_t k = 0; k < n_parts; ++k)
                if (s.carried[k]) {
                    PIPE_TRY(hipEventRecord(carry_ready[size_t(carry_ids[k])], s.stream));
                    carry_give_back(carry_ids[k]);
                }
        }
        return submit_compute(s, n_parts);
    }

    int submit_compute(ReadSlot& s, size_t n_parts) {
        const size_t n = n_parts * t;
        const bool verify_only = (s.mode & CEC_READ_VERIFY_ONLY) != 0;
        const bool resilver = (s.mode & CEC_READ_RESILVER) != 0;
        // hash every loaded chunk except those an earlier pass verified (read retries)
        for (size_t i = 0; i < n; ++i)
            s.h_hash[i] = s.h_present[i] != 0 && s.h_present[i] != CEC_PRESENT_VERIFIED;
        PIPE_TRY(hipMemcpyAsync(s.d_expected, s.h_expected, n * 32, hipMemcpyHostToDevice, s.stream));
        PIPE_TRY(hipMemcpyAsync(s.d_flags, s.h_hash, n, hipMemcpyHostToDevice, s.stream));
        cec_part_batch b = batch(s, n_parts);
        int st = cec_verify_batch(&b, 0, t, s.d_flags, s.d_expected, s.d_flags + n, s.stream);
        if (verify_only) {
            if (st != CEC_OK) {
                g_pipe_error = cec_last_error();
                return st;
            }
            for (size_t k = 0; k < n_parts; ++k) s.h_status[k] = CEC_OK;
            PIPE_TRY(hipMemcpyAsync(s.h_ok, s.d_flags + n, n, hipMemcpyDeviceToHost, s.stream));
            PIPE_TRY(hipEventRecord(s.done, s.stream));
            s.in_flight = true;
            s.checked = false;
            s.n_parts = n_parts;
            return CEC_OK;
        }
        // speculative decode from the loaded chunks; parts with fewer than d loaded are skipped
        // (reported at wait).  Any nonzero flag means loaded, as everywhere else.
        s.decode_mask.assign(s.h_present, s.h_present + n);
        for (size_t k = 0; k < n_parts; ++k) {
            const size_t loaded = size_t(std::count_if(
                s.decode_mask.begin() + k * t, s.decode_mask.begin() + (k + 1) * t,
                [](uint8_t f) { return f != 0; }));
            s.h_status[k] = loaded >= d ? CEC_OK : CEC_TOO_FEW_SHARDS_PRESENT;
            if (loaded < d)
                std::fill(s.decode_mask.begin() + k * t, s.decode_mask.begin() + (k + 1) * t,
                          uint8_t(1));
        }
        if (st == CEC_OK)
            st = cec_reconstruct_batch(codec, &b, s.decode_mask.data(), resilver ? 0 : 1, s.stream);
        if (st != CEC_OK) {
            g_pipe_error = cec_last_error();
            return st;
        }
        if (resilver) {
            for (size_t k = 0; k < n_parts && st == CEC_OK; ++k)
                if (s.h_status[k] == CEC_OK) st = copy_missing_back(s, k, s.h_present + k * t);
        } else if (s.mode & CEC_READ_REBUILT_ONLY) {
            for (size_t k = 0; k < n_parts && st == CEC_OK; ++k)
                if (s.h_status[k] == CEC_OK) st = copy_rebuilt_back(s, k);
        } else {
            st = copy_data_back(s, 0, n_parts);
        }
        if (st != CEC_OK) return st;
        if (carry && !resilver) {
            const int cst = carry_stash(s, n_parts);
            if (cst != CEC_OK) return cst;
        }
        PIPE_TRY(hipMemcpyAsync(s.h_ok, s.d_flags + n, n, hipMemcpyDeviceToHost, s.stream));
        PIPE_TRY(hipEventRecord(s.done, s.stream));
        s.in_flight = true;
        s.checked = false;
        s.n_parts = n_parts;
        return CEC_OK;
    }

    // wait's host side for a completed batch (run once per batch).
    int check(ReadSlot& s) {
        const size_t n = s.n_parts;
        for (size_t i = 0; i < n * t; ++i)  // verified by an earlier pass: trusted
            if (s.h_present[i] == CEC_PRESENT_VERIFIED) s.h_ok[i] = 1;
        if (s.mode & CEC_READ_VERIFY_ONLY) {
            s.data_ptrs.clear();
            s.carry_ids.assign(n, -1);
            s.checked = true;
            return CEC_OK;
        }
        const bool resilver = (s.mode & CEC_READ_RESILVER) != 0;
        // parts whose loaded chunks did not all verify: decode again from the verified ones
        std::vector<uint8_t> mask(n * t, 1);
        std::vector<size_t> redo;
        for (size_t k = 0; k < n; ++k) {
            if (s.h_status[k] != CEC_OK) continue;
            bool bad = false;
            size_t good = 0;
            for (size_t i = 0; i < t; ++i) {
                bad |= s.h_present[k * t + i] && !s.h_ok[k * t + i];
                good += s.h_ok[k * t + i] ? 1 : 0;
            }
            if (!bad) continue;
            if (good < d) {
                s.h_status[k] = CEC_TOO_FEW_SHARDS_PRESENT;
                continue;
            }
            std::copy(s.h_ok + k * t, s.h_ok + (k + 1) * t, mask.begin() + k * t);
            redo.push_back(k);
        }
        if (!redo.empty()) {
            DeviceGuard guard(device);
            PIPE_TRY(guard.status());
            cec_part_batch b = batch(s, n);
            int st = cec_reconstruct_batch(codec, &b, mask.data(), resilver ? 0 : 1, s.stream);
            if (st != CEC_OK) {
                g_pipe_error = cec_last_error();
                return st;
            }
            for (size_t k : redo) {
                st = resilver ? copy_missing_back(s, k, s.h_ok + k * t) : copy_data_back(s, k, 1);
                if (st != CEC_OK) return st;
            }
            PIPE_TRY(hipStreamSynchronize(s.stream));
        }
        // CEC_READ_CARRY: the stash kept the verified chunks of every part with fewer than d of
        // them (exactly the parts reported TooFewShardsPresent) in a reserved entry, while
        // reservations lasted.  Those entries stay reserved for the caller to claim
        // (cec_read_pipeline_carry_ids); the rest go back now.  Each records what it holds.
        s.carry_ids.assign(n, -1);
        if (s.stashed) {
            std::vector<int32_t> keep;
            for (size_t k = 0; k < n; ++k) {
                const int32_t id = s.h_map[k];
                if (id < 0 || s.h_status[k] != CEC_TOO_FEW_SHARDS_PRESENT) continue;
                if (size_t(id) >= carry_cap || carry_used[size_t(id)] != kReserved) {
                    g_pipe_error = "carry stash returned an entry the batch did not reserve";
                    return CEC_ERR_HIP;
                }
                s.carry_ids[k] = id;
                keep.push_back(id);
                for (size_t i = 0; i < t; ++i)
                    carry_mask[size_t(id) * t + i] = s.h_present[k * t + i] && s.h_ok[k * t + i];
                std::memcpy(carry_exp.data() + size_t(id) * t * 32, s.h_expected + k * t * 32,
                            t * 32);
            }
            for (int32_t id : s.reserved)
                if (std::find(keep.begin(), keep.end(), id) == keep.end() &&
                    carry_used[size_t(id)] == kReserved)
                    carry_give_back(id);
            s.reserved = keep;
        }
        // Where each output chunk is: re-decoded parts and (without REBUILT_ONLY) every part in
        // the data output; otherwise a loaded chunk stays in the chunk buffer it was read from (it
        // verified: parts with a failed chunk were re-decoded) and a rebuilt one came back into
        // the data output -- as did a carried part's verified data chunks (the caller's buffer
        // does not hold them).
        std::vector<uint8_t> redone(n, 0);
        for (size_t k : redo) redone[k] = 1;
        if (resilver) {  // [parts][t]: verified chunks where they were read, others rebuilt
            s.data_ptrs.resize(n * t);
            for (size_t k = 0; k < n; ++k)
                for (size_t i = 0; i < t; ++i)
                    s.data_ptrs[k * t + i] = s.h_ok[k * t + i] ? s.src_chunks + s.src_off[k * t + i]
                                                               : s.dst_data + (k * t + i) * L;
        } else {
            const bool rebuilt_only = (s.mode & CEC_READ_REBUILT_ONLY) != 0;
            s.data_ptrs.resize(n * d);
            for (size_t k = 0; k < n; ++k)
                for (size_t j = 0; j < d; ++j) {
                    const uint8_t f = s.h_present[k * t + j];
                    const bool from_pool = !s.carried.empty() && s.carried[k] &&
                                           f == CEC_PRESENT_VERIFIED;
                    const bool in_place = rebuilt_only && !redone[k] && f && !from_pool;
                    s.data_ptrs[k * d + j] = in_place ? s.src_chunks + s.src_off[k * t + j]
                                                      : s.dst_data + (k * d + j) * L;
                }
        }
        s.checked = true;
        return CEC_OK;
    }

    int finish(ReadSlot& s) {
        if (s.in_flight) {
            PIPE_TRY(hipEventSynchronize(s.done));
            s.in_flight = false;
        }
        if (!s.checked && s.n_parts) return check(s);
        return CEC_OK;
    }
};

extern "C" {

int cec_read_pipeline_new(const cec_codec* codec, size_t chunk_len, size_t parts_per_batch,
                          size_t depth, cec_read_pipeline** out) {
    return cec_read_pipeline_new_ex(codec, chunk_len, parts_per_batch, depth, 0u, out);
}

int cec_read_pipeline_new_ex(const cec_codec* codec, size_t chunk_len, size_t parts_per_batch,
                             size_t depth, unsigned flags, cec_read_pipeline** out) {
    if (!codec || !out || chunk_len == 0 || parts_per_batch == 0 || depth == 0 || depth > 16 ||
        (flags & ~unsigned(kModeBits | CEC_PIPE_EXTERNAL | CEC_READ_CARRY)) ||
        ((flags & CEC_READ_RESILVER) && (flags & CEC_READ_VERIFY_ONLY)))
        return CEC_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    if (cec_device_count() <= 0) return CEC_ERR_NO_DEVICE;
    auto* pl = new cec_read_pipeline();
    pl->codec = codec;
    PIPE_TRY(hipGetDevice(&pl->device));
    pl->d = cec_codec_data_shards(codec);
    pl->p = cec_codec_parity_shards(codec);
    pl->t = pl->d + pl->p;
    pl->L = chunk_len;
    pl->cs = (chunk_len + 255) / 256 * 256;
    pl->parts = parts_per_batch;
    pl->default_mode = flags & kModeBits;
    pl->external = (flags & CEC_PIPE_EXTERNAL) != 0;
    pl->carry = (flags & CEC_READ_CARRY) != 0;
    pl->h_out_chunks = pl->external ? 0 : cec_read_pipeline::out_chunks(pl->default_mode, pl->d, pl->t);
    // a quarter of a batch's parts per batch (a 1 % damaged-fetch rate fails ~10 % of RS(10,4)
    // parts): entries for every batch in flight plus one batch's retries
    pl->carry_batch = pl->carry ? std::min<size_t>(parts_per_batch, std::max<size_t>(8, parts_per_batch / 4)) : 0;
    pl->carry_cap = pl->carry_batch * (depth + 1);
    pl->slots.resize(depth);
    const size_t P = pl->parts, t = pl->t;
    for (ReadSlot& s : pl->slots) {
        hipError_t e = hipSuccess;
        auto host = [&](uint8_t** ptr, size_t bytes) {  // pinned, on the device's NUMA node
            if (e == hipSuccess)
                e = cec::host_malloc_near(reinterpret_cast<void**>(ptr), bytes,
                                          hipHostMallocDefault, pl->device);
        };
        auto dev = [&](uint8_t** ptr, size_t bytes) {
            if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(ptr), bytes);
        };
        if (!pl->external) {
            host(&s.h_chunks, P * t * pl->L);
            if (pl->h_out_chunks) host(&s.h_data, P * pl->h_out_chunks * pl->L);
        }
        host(&s.h_present, P * t);
        host(&s.h_expected, P * t * 32);
        host(&s.h_ok, P * t);
        host(&s.h_hash, P * t);
        dev(&s.d_buf, P * t * pl->cs);
        dev(&s.d_expected, P * t * 32);
        dev(&s.d_flags, 2 * P * t);
        if (e == hipSuccess) e = slot_stream(&s.stream);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
        s.h_status = new int[P];
        if (e != hipSuccess) {
            delete pl;
            return pipe_fail(e, "cec_read_pipeline_new allocation");
        }
        std::memset(s.h_present, 0, P * t);
    }
    if (pl->carry) {
        const hipError_t e = pl->make_carry_pool();
        if (e != hipSuccess) {
            (void)hipGetLastError();
            delete pl;
            return pipe_fail(e, "cec_read_pipeline_new carry pool");
        }
    }
    g_pipelines_made.fetch_add(1, std::memory_order_relaxed);
    *out = pl;
    return CEC_OK;
}

void cec_read_pipeline_free(cec_read_pipeline* pl) { delete pl; }

size_t cec_read_pipeline_depth(const cec_read_pipeline* pl) { return pl ? pl->slots.size() : 0; }

}  // extern "C"

namespace {

int read_acquire(cec_read_pipeline* pl, size_t i, size_t* slot, uint8_t** chunks,
                 uint8_t** present, uint8_t** expected) {
    pl->next = (i + 1) % pl->slots.size();
    ReadSlot& s = pl->slots[i];
    if (s.in_flight) {
        PIPE_TRY(hipEventSynchronize(s.done));
        s.in_flight = false;
    }
    *slot = i;
    *chunks = s.h_chunks;
    *present = s.h_present;
    *expected = s.h_expected;
    return CEC_OK;
}

}  // namespace

int cec::read_pipeline_acquire_slot(cec_read_pipeline* pl, size_t slot, uint8_t** chunks,
                                    uint8_t** present, uint8_t** expected) {
    if (!pl || slot >= pl->slots.size() || !chunks || !present || !expected)
        return CEC_ERR_INVALID_ARGUMENT;
    size_t unused = 0;
    return read_acquire(pl, slot, &unused, chunks, present, expected);
}

int cec::read_pipeline_priority_slot(cec_read_pipeline* pl, size_t slot) {
    if (!pl || slot >= pl->slots.size() || pl->slots[slot].in_flight)
        return CEC_ERR_INVALID_ARGUMENT;
    ReadSlot& s = pl->slots[slot];
    DeviceGuard guard(pl->device);
    PIPE_TRY(guard.status());
    int least = 0, greatest = 0;
    PIPE_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    if (least == greatest) return CEC_OK;
    hipStream_t high = nullptr;
    PIPE_TRY(hipStreamCreateWithPriority(&high, hipStreamNonBlocking, greatest));
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s.stream = high;
    return CEC_OK;
}

extern "C" {

int cec_read_pipeline_acquire(cec_read_pipeline* pl, size_t* slot, uint8_t** chunks,
                              uint8_t** present, uint8_t** expected) {
    if (!pl || !slot || !chunks || !present || !expected) return CEC_ERR_INVALID_ARGUMENT;
    return read_acquire(pl, pl->next, slot, chunks, present, expected);
}

int cec_read_pipeline_acquire_idle(cec_read_pipeline* pl, size_t* slot, uint8_t** chunks,
                                   uint8_t** present, uint8_t** expected) {
    if (!pl || !slot || !chunks || !present || !expected) return CEC_ERR_INVALID_ARGUMENT;
    // the first slot from the round-robin position on whose batch is done (or that has none);
    // all busy: the round-robin slot, waited for
    const size_t n = pl->slots.size();
    for (size_t k = 0; k < n; ++k) {
        const size_t i = (pl->next + k) % n;
        if (cec_read_pipeline_query(pl, i) == 1)
            return read_acquire(pl, i, slot, chunks, present, expected);
    }
    return read_acquire(pl, pl->next, slot, chunks, present, expected);
}

int cec_read_pipeline_submit_ex(cec_read_pipeline* pl, size_t slot, const cec_read_submit* a) {
    if (!pl || !a || slot >= pl->slots.size() || a->n_parts == 0 || a->n_parts > pl->parts ||
        (a->flags & ~unsigned(kModeBits | CEC_SUBMIT_PACKED)))
        return CEC_ERR_INVALID_ARGUMENT;
    ReadSlot& s = pl->slots[slot];
    const uint8_t* chunks = a->chunks ? a->chunks : s.h_chunks;
    if (!chunks) return CEC_ERR_INVALID_ARGUMENT;  // CEC_PIPE_EXTERNAL: the caller's chunks
    if (s.in_flight && (a->present || a->expected)) {
        // the arrays below are read by the slot's last batch until it completes
        DeviceGuard guard(pl->device);
        PIPE_TRY(guard.status());
        PIPE_TRY(hipEventSynchronize(s.done));
        s.in_flight = false;
    }
    const size_t n = a->n_parts * pl->t;
    if (a->present) std::memcpy(s.h_present, a->present, n);
    if (a->expected) std::memcpy(s.h_expected, a->expected, n * 32);
    const unsigned mode = a->flags & kModeBits;
    return pl->submit(s, chunks, a->n_parts, a->data_out ? a->data_out : s.h_data, mode,
                      (a->flags & CEC_SUBMIT_PACKED) != 0, a->carry_ids);
}

int cec_read_pipeline_submit(cec_read_pipeline* pl, size_t slot, size_t n_parts) {
    if (!pl || pl->external) return CEC_ERR_INVALID_ARGUMENT;
    cec_read_submit a{nullptr, nullptr, nullptr, n_parts, nullptr, nullptr, pl->default_mode};
    return cec_read_pipeline_submit_ex(pl, slot, &a);
}

int cec_read_pipeline_submit_from(cec_read_pipeline* pl, size_t slot, const uint8_t* chunks,
                                  const uint8_t* present, const uint8_t* expected, size_t n_parts,
                                  uint8_t* data_out) {
    if (!pl || !chunks) return CEC_ERR_INVALID_ARGUMENT;
    cec_read_submit a{chunks, present, expected, n_parts, data_out, nullptr, pl->default_mode};
    return cec_read_pipeline_submit_ex(pl, slot, &a);
}

int cec_read_pipeline_submit_packed(cec_read_pipeline* pl, size_t slot, const uint8_t* chunks,
                                    const uint8_t* present, const uint8_t* expected,
                                    size_t n_parts, uint8_t* data_out) {
    if (!pl || !chunks) return CEC_ERR_INVALID_ARGUMENT;
    cec_read_submit a{chunks, present, expected, n_parts, data_out, nullptr,
                      pl->default_mode | CEC_SUBMIT_PACKED};
    return cec_read_pipeline_submit_ex(pl, slot, &a);
}

int cec_read_pipeline_submit_carried(cec_read_pipeline* pl, size_t slot, size_t n_parts,
                                     const int32_t* carry_ids) {
    if (!pl || pl->external || !carry_ids) return CEC_ERR_INVALID_ARGUMENT;
    cec_read_submit a{nullptr, nullptr, nullptr, n_parts, nullptr, carry_ids, pl->default_mode};
    return cec_read_pipeline_submit_ex(pl, slot, &a);
}

int cec_read_pipeline_wait(cec_read_pipeline* pl, size_t slot, const uint8_t** data,
                           const uint8_t** verified, const int** part_status, size_t* n_parts) {
    if (!pl || slot >= pl->slots.size()) return CEC_ERR_INVALID_ARGUMENT;
    ReadSlot& s = pl->slots[slot];
    const int st = pl->finish(s);
    if (st != CEC_OK) return st;
    if (data) *data = s.dst_data ? s.dst_data : s.h_data;
    if (verified) *verified = s.h_ok;
    if (part_status) *part_status = s.h_status;
    if (n_parts) *n_parts = s.n_parts;
    return CEC_OK;
}

int cec_read_pipeline_data_chunks(cec_read_pipeline* pl, size_t slot, const uint8_t** ptrs,
                                  size_t capacity) {
    if (!pl || slot >= pl->slots.size() || !ptrs) return CEC_ERR_INVALID_ARGUMENT;
    ReadSlot& s = pl->slots[slot];
    const int st = pl->finish(s);
    if (st != CEC_OK) return st;
    if (s.data_ptrs.size() > capacity) {
        g_pipe_error = "data_chunks: the batch has more chunk pointers than the output holds";
        return CEC_ERR_INVALID_ARGUMENT;
    }
    std::copy(s.data_ptrs.begin(), s.data_ptrs.end(), ptrs);
    return CEC_OK;
}

int cec_read_pipeline_carry_ids(cec_read_pipeline* pl, size_t slot, int32_t* ids,
                                size_t capacity) {
    if (!pl || slot >= pl->slots.size() || !ids || !pl->carry) return CEC_ERR_INVALID_ARGUMENT;
    ReadSlot& s = pl->slots[slot];
    const int st = pl->finish(s);
    if (st != CEC_OK) return st;
    if (s.n_parts > capacity) {
        g_pipe_error = "carry_ids: the batch has more parts than the output holds";
        return CEC_ERR_INVALID_ARGUMENT;
    }
    // the caller now holds these entries (until it submits them or releases them)
    for (int32_t id : s.reserved)
        if (pl->carry_used[size_t(id)] == pl->kReserved) pl->carry_used[size_t(id)] = pl->kHeld;
    s.reserved.clear();
    for (size_t k = 0; k < s.n_parts; ++k) ids[k] = k < s.carry_ids.size() ? s.carry_ids[k] : -1;
    return CEC_OK;
}

int cec_read_pipeline_carry_release(cec_read_pipeline* pl, int32_t id) {
    if (!pl || !pl->carry_valid(id)) return CEC_ERR_INVALID_ARGUMENT;
    pl->carry_give_back(id);
    return CEC_OK;
}

size_t cec_read_pipeline_carry_held(const cec_read_pipeline* pl) {
    return pl ? pl->held_entries() : 0;
}

int cec_read_pipeline_query(cec_read_pipeline* pl, size_t slot) {
    if (!pl || slot >= pl->slots.size()) return CEC_ERR_INVALID_ARGUMENT;
    ReadSlot& s = pl->slots[slot];
    if (!s.in_flight) return 1;
    const hipError_t e = hipEventQuery(s.done);
    (void)hipGetLastError();
    return e == hipErrorNotReady ? 0 : 1;
}

int cec_read_pipeline_drain(cec_read_pipeline* pl) {
    if (!pl) return CEC_ERR_INVALID_ARGUMENT;
    for (ReadSlot& s : pl->slots)
        if (s.in_flight) {
            const int st = pl->finish(s);
            if (st != CEC_OK) return st;
        }
    return CEC_OK;
}

}  // extern "C"
