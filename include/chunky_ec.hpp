// chunky_ec.hpp — C++17 host layer over the C-ABI (chunky_ec.h) that mirrors the interface of
// the reference's part layer for this path, so host code and tests read like the reference's
// own (Rust) code.  Header-only; every computation goes through libchunky_ec.so on the GPU.
//
//   reference (Rust)                                   here
//   reed_solomon_erasure::ReedSolomon<galois_8::Field> chunky_ec::ReedSolomon
//     ::new / encode_sep / reconstruct / reconstruct_data   (same names, same argument meaning)
//   reed_solomon_erasure::Error (13 variants)          chunky_ec::Error + ErasureError exception
//   file::hash::Sha256Hash (sha256.rs:14-47)           chunky_ec::Sha256Hash
//     from_buf / verify / Display (lower-case hex)        from_buf / verify / to_string
//   file::Chunk (chunk.rs:10-17)                       chunky_ec::Chunk (hash + locations: keys
//                                                        of a ChunkStore, below)
//   file::FilePart (file_part.rs:57-390)               chunky_ec::FilePart
//     write_with_encoder (137-225)                        write_with_encoder
//     read_with_context (73-135)                          read_with_context
//     verify (228-251) / resilver (253-390)               verify / resilver
//   file::FileWriteBuilder (writer.rs:88-255)          chunky_ec::FileWriteBuilder
//   file::FileReference (file_reference.rs)            chunky_ec::FileReference
//
// Storage, placement and networking are out of scope: a ChunkStore stands in
// for the locations (location -> bytes; shards written as `sha256-<hex>`, location.rs:612).  Rust's
// `Result<_, Error>` + `?` becomes a thrown ErasureError carrying the same variant; engine
// failures (no GPU, HIP errors) throw EngineError and are never disguised as crate errors.
#ifndef CHUNKY_EC_HPP
#define CHUNKY_EC_HPP

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <future>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "chunky_ec.h"

namespace chunky_ec {

using Bytes = std::vector<uint8_t>;
// &mut [Option<Vec<u8>>] of reconstruct / reconstruct_data
using Shards = std::vector<std::optional<Bytes>>;

// reed_solomon_erasure::Error, declaration order (cec_status 1..13).
enum class Error {
    TooFewShards = CEC_TOO_FEW_SHARDS,
    TooManyShards = CEC_TOO_MANY_SHARDS,
    TooFewDataShards = CEC_TOO_FEW_DATA_SHARDS,
    TooManyDataShards = CEC_TOO_MANY_DATA_SHARDS,
    TooFewParityShards = CEC_TOO_FEW_PARITY_SHARDS,
    TooManyParityShards = CEC_TOO_MANY_PARITY_SHARDS,
    TooFewBufferShards = CEC_TOO_FEW_BUFFER_SHARDS,
    TooManyBufferShards = CEC_TOO_MANY_BUFFER_SHARDS,
    IncorrectShardSize = CEC_INCORRECT_SHARD_SIZE,
    TooFewShardsPresent = CEC_TOO_FEW_SHARDS_PRESENT,
    EmptyShard = CEC_EMPTY_SHARD,
    InvalidShardFlags = CEC_INVALID_SHARD_FLAGS,
    InvalidIndex = CEC_INVALID_INDEX,
};

// A crate error (FileWriteError::Erasure / FileReadError::Erasure in the reference).
class ErasureError : public std::runtime_error {
   public:
    explicit ErasureError(Error e) : std::runtime_error(cec_status_name(int(e))), error_(e) {}
    Error error() const { return error_; }

   private:
    Error error_;
};

// Engine failure with no crate equivalent.
class EngineError : public std::runtime_error {
   public:
    EngineError(int code, const std::string& what) : std::runtime_error(what), code_(code) {}
    int code() const { return code_; }

   private:
    int code_;
};

namespace detail {
inline void check(int status) {
    if (status == CEC_OK) return;
    if (status >= CEC_TOO_FEW_SHARDS && status <= CEC_INVALID_INDEX)
        throw ErasureError(static_cast<Error>(status));
    throw EngineError(status, std::string(cec_status_name(status)) + ": " + cec_last_error());
}

// Pipeline calls keep their messages in cec_pipeline_last_error().
inline void check_pipe(int status) {
    if (status == CEC_OK) return;
    if (status >= CEC_TOO_FEW_SHARDS && status <= CEC_INVALID_INDEX)
        throw ErasureError(static_cast<Error>(status));
    throw EngineError(status, std::string(cec_status_name(status)) + ": " + cec_pipeline_last_error());
}

// Host threads for the batched paths' copies into / out of pinned staging (CEC_HOST_COPY_THREADS,
// default 8).  One thread's memcpy (~10-20 GB/s) is below the PCIe rate the pipelines reach.
inline size_t copy_threads() {
    static const size_t n = [] {
        const char* e = std::getenv("CEC_HOST_COPY_THREADS");
        const long v = e ? std::atol(e) : 8;
        return size_t(std::min<long>(std::max<long>(v, 1), 64));
    }();
    return n;
}

// fn(i) for i in [0, n) over copy_threads() threads (contiguous ranges; inline when small).
template <typename Fn>
inline void parallel_for(size_t n, Fn fn) {
    const size_t w = std::min(copy_threads(), n);
    if (w <= 1) {
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

// memcpy of n bytes split over copy_threads() threads (1 MiB grain).
inline void parallel_copy(uint8_t* dst, const uint8_t* src, size_t n) {
    constexpr size_t kGrain = size_t(1) << 20;
    const size_t pieces = (n + kGrain - 1) / kGrain;
    parallel_for(pieces, [&](size_t i) {
        const size_t off = i * kGrain;
        std::memcpy(dst + off, src + off, std::min(kGrain, n - off));
    });
}

inline char hex_digit(unsigned v) { return char(v < 10 ? '0' + v : 'a' + (v - 10)); }

inline int hex_value(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}
}  // namespace detail

// ReedSolomon<galois_8::Field>.  Immutable after construction; share it like the reference's
// Arc<ReedSolomon> (writer.rs:131,200): every method is const and thread-safe.
class ReedSolomon {
   public:
    ReedSolomon(size_t data_shards, size_t parity_shards) {
        cec_codec* raw = nullptr;
        detail::check(cec_codec_new(data_shards, parity_shards, &raw));
        raw_ = std::shared_ptr<cec_codec>(raw, Free{});
    }

    size_t data_shard_count() const { return cec_codec_data_shards(raw_.get()); }
    size_t parity_shard_count() const { return cec_codec_parity_shards(raw_.get()); }
    size_t total_shard_count() const { return cec_codec_total_shards(raw_.get()); }

    // The (d+p) x d coding matrix, row major (top d x d = identity).
    std::vector<Bytes> matrix() const {
        const size_t d = data_shard_count(), t = total_shard_count();
        Bytes flat(t * d);
        detail::check(cec_codec_matrix(raw_.get(), flat.data(), flat.size()));
        std::vector<Bytes> rows(t);
        for (size_t r = 0; r < t; ++r) rows[r].assign(flat.begin() + r * d, flat.begin() + (r + 1) * d);
        return rows;
    }

    // encode_sep(&data, &mut parity): parity slices are overwritten.
    void encode_sep(const std::vector<std::pair<const uint8_t*, size_t>>& data,
                    std::vector<Bytes>& parity) const {
        std::vector<const uint8_t*> dp;
        std::vector<size_t> dl;
        for (const auto& s : data) {
            dp.push_back(s.first);
            dl.push_back(s.second);
        }
        std::vector<uint8_t*> pp;
        std::vector<size_t> pl;
        for (auto& v : parity) {
            pp.push_back(v.data());
            pl.push_back(v.size());
        }
        detail::check(cec_encode_sep(raw_.get(), dp.data(), dl.data(), dp.size(), pp.data(),
                                     pl.data(), pp.size()));
    }

    void encode_sep(const std::vector<Bytes>& data, std::vector<Bytes>& parity) const {
        std::vector<std::pair<const uint8_t*, size_t>> views;
        for (const auto& v : data) views.emplace_back(v.data(), v.size());
        encode_sep(views, parity);
    }

    // reconstruct(&mut shards): rebuilds every missing shard (data and parity).
    void reconstruct(Shards& shards) const { reconstruct_inner(shards, false); }
    // reconstruct_data(&mut shards): rebuilds missing data shards only.
    void reconstruct_data(Shards& shards) const { reconstruct_inner(shards, true); }

    const cec_codec* raw() const { return raw_.get(); }

   private:
    struct Free {
        void operator()(cec_codec* c) const { cec_codec_free(c); }
    };
    std::shared_ptr<cec_codec> raw_{nullptr, Free{}};

    void reconstruct_inner(Shards& shards, bool data_only) const {
        // The crate allocates missing slots zeroed at the present length: do the same so the
        // engine writes straight into the caller's vectors.
        size_t len = 0;
        for (const auto& s : shards)
            if (s && !s->empty()) {
                len = s->size();
                break;
            }
        const size_t d = data_shard_count();
        std::vector<uint8_t> present(shards.size());
        Shards scratch(shards.size());
        std::vector<uint8_t*> ptrs(shards.size(), nullptr);
        std::vector<size_t> lens(shards.size(), 0);
        for (size_t i = 0; i < shards.size(); ++i) {
            present[i] = shards[i].has_value();
            if (shards[i]) {
                ptrs[i] = shards[i]->data();
                lens[i] = shards[i]->size();
            } else if (!(data_only && i >= d)) {
                scratch[i].emplace(len, 0);
                ptrs[i] = scratch[i]->data();
                lens[i] = len;
            }
        }
        auto f = data_only ? cec_reconstruct_data : cec_reconstruct;
        detail::check(f(raw_.get(), ptrs.data(), lens.data(), present.data(), shards.size()));
        for (size_t i = 0; i < shards.size(); ++i)
            if (!shards[i] && present[i]) shards[i] = std::move(scratch[i]);
    }
};

namespace detail {
// Multi-GPU scheduler calls keep their messages in cec_multi_last_error().
inline void check_multi(int status) {
    if (status == CEC_OK) return;
    if (status >= CEC_TOO_FEW_SHARDS && status <= CEC_INVALID_INDEX)
        throw ErasureError(static_cast<Error>(status));
    throw EngineError(status, std::string(cec_status_name(status)) + ": " + cec_multi_last_error());
}

// Page-locked host buffer (cec_host_alloc, pages on `device`'s NUMA node), grown on demand:
// the engine DMAs it directly.
class PinnedBuf {
   public:
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() { release(); }
    uint8_t* reserve(size_t n, int device) {
        if (n > cap_) {
            release();
            void* q = nullptr;
            check(cec_host_alloc(n, device, &q));
            p_ = static_cast<uint8_t*>(q);
            cap_ = n;
        }
        return p_;
    }
    void release() {
        if (p_) cec_host_free(p_);
        p_ = nullptr;
        cap_ = 0;
    }

   private:
    uint8_t* p_ = nullptr;
    size_t cap_ = 0;
};

// fn(k) for k in [0, n) with at most `window` calls in flight, sink(k, result) in order of k —
// the reference's `buffered(window)` / FuturesOrdered over part futures.  A call's exception
// reaches the caller at its turn (the calls still in flight finish first).
template <typename Fn, typename Sink>
void ordered_concurrent(size_t n, size_t window, Fn fn, Sink sink) {
    using R = decltype(fn(size_t(0)));
    std::deque<std::future<R>> q;
    size_t next = 0, done = 0;
    window = std::max<size_t>(window, 1);
    while (done < n) {
        while (next < n && q.size() < window) q.push_back(std::async(std::launch::async, fn, next++));
        sink(done++, q.front().get());
        q.pop_front();
    }
}

inline std::vector<int> devices_or_current(const std::vector<int>& devices) {
    if (!devices.empty()) return devices;
    int dev = 0;
    (void)cec_current_device(&dev);
    return {dev};
}

// The batched paths run through the multi-GPU scheduler (cec_multi: one worker thread and
// pipeline per shard).  Its pipelines and staging pin host memory (~0.35 s per GiB), so the most
// recent scheduler is kept per thread and reused by every later write/read of the same shape and
// device list; a new shape frees the old one first, so the pinned total stays bounded.
struct CachedMulti {
    std::vector<size_t> key;
    std::shared_ptr<ReedSolomon> codec;
    std::shared_ptr<cec_multi> multi;
};

// Batched read retries leave their verified chunks on the GPU (cec_multi_read_carry) unless this
// is false (then they are sent again): the with / without figure of tools/cp_bench.
inline std::atomic<bool>& read_carry() {
    static std::atomic<bool> on{true};
    return on;
}

// Where this thread's batched reads spent their time (seconds; tools/cp_bench prints them):
// loading windows from the store, waiting for read jobs, building and waiting for retry rounds,
// and in the sink.
struct ReadTimes {
    double load = 0, wait_job = 0, retry_build = 0, wait_retry = 0, emit = 0;
    // submission to the loop seeing the job done, summed: windows' read jobs, retry rounds
    double job_latency = 0, round_latency = 0;
    uint64_t windows = 0, retry_rounds = 0, retry_parts = 0, later_rounds = 0;
};
inline ReadTimes& read_times() {
    thread_local ReadTimes t;
    return t;
}
// Adds the seconds from construction to destruction to `acc`.
struct Timed {
    double& acc;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    explicit Timed(double& a) : acc(a) {}
    ~Timed() { acc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); }
};

inline CachedMulti& cached_multi_entry() {
    thread_local CachedMulti e;
    return e;
}

inline cec_multi* cached_multi(size_t d, size_t p, size_t L, size_t parts, size_t depth,
                               const std::vector<int>& devices) {
    CachedMulti& e = cached_multi_entry();
    std::vector<size_t> key{d, p, L, parts, depth};
    for (int dv : devices) key.push_back(size_t(dv));
    if (!e.multi || e.key != key) {
        e.multi.reset();
        e.codec = std::make_shared<ReedSolomon>(d, p);
        cec_multi* raw = nullptr;
        check_multi(cec_multi_new(e.codec->raw(), L, parts, depth, devices.data(), devices.size(),
                                  &raw));
        e.multi = std::shared_ptr<cec_multi>(raw, cec_multi_free);
        e.key = key;
    }
    return e.multi.get();
}
}  // namespace detail

// file::hash::Sha256Hash.
class Sha256Hash {
   public:
    Sha256Hash() = default;
    explicit Sha256Hash(const std::array<uint8_t, 32>& digest) : digest_(digest) {}

    static Sha256Hash from_buf(const uint8_t* buf, size_t len) {
        std::array<uint8_t, 32> d{};
        detail::check(cec_sha256(buf, len, d.data()));
        return Sha256Hash(d);
    }
    static Sha256Hash from_buf(const Bytes& buf) { return from_buf(buf.data(), buf.size()); }
    static Sha256Hash from_buf(const std::string& s) {
        return from_buf(reinterpret_cast<const uint8_t*>(s.data()), s.size());
    }

    // Many digests in one launch (DataHasher over a part's chunks).
    static std::vector<Sha256Hash> from_bufs(const std::vector<const Bytes*>& bufs) {
        std::vector<const uint8_t*> p;
        std::vector<size_t> l;
        for (const Bytes* b : bufs) {
            p.push_back(b->data());
            l.push_back(b->size());
        }
        std::vector<uint8_t> out(32 * bufs.size());
        if (!bufs.empty()) detail::check(cec_sha256_many(p.data(), l.data(), p.size(), out.data()));
        std::vector<Sha256Hash> r(bufs.size());
        for (size_t i = 0; i < bufs.size(); ++i) std::memcpy(r[i].digest_.data(), &out[32 * i], 32);
        return r;
    }

    // Display: lower-case hex (the metadata's `sha256: <hex>` and `sha256-<hex>` file names).
    std::string to_string() const {
        std::string s(64, '0');
        for (size_t i = 0; i < 32; ++i) {
            s[2 * i] = detail::hex_digit(digest_[i] >> 4);
            s[2 * i + 1] = detail::hex_digit(digest_[i] & 15);
        }
        return s;
    }

    static Sha256Hash from_str(const std::string& hex) {
        if (hex.size() != 64) throw std::invalid_argument("sha256 hex must be 64 digits");
        std::array<uint8_t, 32> d{};
        for (size_t i = 0; i < 32; ++i) {
            const int hi = detail::hex_value(hex[2 * i]), lo = detail::hex_value(hex[2 * i + 1]);
            if (hi < 0 || lo < 0) throw std::invalid_argument("bad sha256 hex digit");
            d[i] = uint8_t(hi * 16 + lo);
        }
        return Sha256Hash(d);
    }

    // DataVerifier::verify: digest of buf equals this hash.
    bool verify(const uint8_t* buf, size_t len) const { return from_buf(buf, len) == *this; }
    bool verify(const Bytes& buf) const { return verify(buf.data(), buf.size()); }
    bool verify(const std::string& s) const {
        return verify(reinterpret_cast<const uint8_t*>(s.data()), s.size());
    }

    const std::array<uint8_t, 32>& digest() const { return digest_; }
    bool operator==(const Sha256Hash& o) const { return digest_ == o.digest_; }
    bool operator!=(const Sha256Hash& o) const { return !(*this == o); }
    bool operator<(const Sha256Hash& o) const { return digest_ < o.digest_; }

   private:
    std::array<uint8_t, 32> digest_{};
};

// file::Location (location.rs:61-68): where one copy of a chunk lives.  The reference's are file
// paths and URLs; here they are keys of a ChunkStore.
using Location = std::string;

// Chunk storage standing in for the reference's locations: location -> bytes.  A shard written
// through write_shard lands at "sha256-<hex>" (location.rs:605-616: one destination directory;
// OnConflict::Overwrite, the default outside clusters, location.rs:505) and that location is
// returned, as ShardWriter::write_shard returns the locations it wrote.  Reads of different
// locations may run concurrently; writes need the caller's lock.
class ChunkStore {
   public:
    ChunkStore() = default;
    // A sink that records nothing (shards to /dev/null): for measuring the write path alone.
    static ChunkStore discard() {
        ChunkStore s;
        s.discard_ = true;
        return s;
    }
    bool discards() const { return discard_; }
    static Location location_of(const Sha256Hash& hash) { return "sha256-" + hash.to_string(); }
    Location write_shard(const Sha256Hash& hash, Bytes bytes) {
        Location loc = location_of(hash);
        if (!discard_) store_[loc] = std::move(bytes);
        return loc;
    }
    Location write_shard(const Sha256Hash& hash, const uint8_t* bytes, size_t n) {
        if (discard_) return location_of(hash);  // no copy of bytes nobody keeps
        return write_shard(hash, Bytes(bytes, bytes + n));
    }
    // Put bytes at any location (a replica elsewhere, a stale copy in tests).
    void put(const Location& loc, Bytes bytes) { store_[loc] = std::move(bytes); }
    std::optional<Bytes> read(const Location& loc) const {
        auto it = store_.find(loc);
        if (it == store_.end()) return std::nullopt;
        return it->second;
    }
    // The stored bytes without a copy (nullptr if the location does not read); valid until that
    // location is written or erased.
    const Bytes* find(const Location& loc) const {
        auto it = store_.find(loc);
        return it == store_.end() ? nullptr : &it->second;
    }
    bool erase(const Location& loc) { return store_.erase(loc) > 0; }
    // Flip a bit of the copy at `loc` (bit rot / tampering in tests).
    bool corrupt(const Location& loc, size_t offset) {
        auto it = store_.find(loc);
        if (it == store_.end() || offset >= it->second.size()) return false;
        it->second[offset] ^= 0x01;
        return true;
    }
    size_t size() const { return store_.size(); }

   private:
    std::map<Location, Bytes> store_;
    bool discard_ = false;
};

// file::Chunk (chunk.rs:10-17): the hash of one chunk and the locations of its copies, in order.
struct Chunk {
    Sha256Hash hash;
    std::vector<Location> locations;
};

// LocationIntegrity (file_part.rs:397-403), in the reference's order (chunk_integrity keeps the
// smallest).
enum class LocationIntegrity { Valid, Resilvered, Invalid, Unavailable };

// VerifyPartReport / ResilverPartReport (file_part.rs:570-811).  locations: the result of every
// location of every chunk (read_results: Valid, Invalid, or Unavailable when it does not read).
// chunks: each chunk's integrity (chunk_integrity, :599-613: Valid when a location is, else the
// best of its locations; no location at all is Unavailable), Resilvered for a chunk resilver
// rebuilt and wrote.  new_locations: resilver's writes, appended to the chunks' location lists
// (:340-347).  write_error: the reconstruct failure of this part (TooFewShardsPresent when fewer
// than d chunks have a valid copy, :296-308); the other parts of the file are still resilvered.
struct PartReport {
    std::vector<std::vector<LocationIntegrity>> locations;  // [chunk][location], d data then p
    std::vector<LocationIntegrity> chunks;                  // d data then p parity
    std::vector<Location> new_locations;
    std::optional<Error> write_error;
    bool is_ideal() const {
        if (write_error) return false;
        for (auto c : chunks)
            if (c != LocationIntegrity::Valid && c != LocationIntegrity::Resilvered) return false;
        return true;
    }
    size_t count(LocationIntegrity what) const {
        size_t n = 0;
        for (auto c : chunks) n += c == what;
        return n;
    }
    size_t unavailable_locations() const { return count_locations(LocationIntegrity::Unavailable); }
    size_t invalid_locations() const { return count_locations(LocationIntegrity::Invalid); }
    size_t count_locations(LocationIntegrity what) const {
        size_t n = 0;
        for (const auto& c : locations)
            for (auto l : c) n += l == what;
        return n;
    }
    // chunks[] from locations[] (chunk_integrity).
    void summarize() {
        chunks.assign(locations.size(), LocationIntegrity::Unavailable);
        for (size_t i = 0; i < locations.size(); ++i)
            for (auto l : locations[i]) chunks[i] = std::min(chunks[i], l);
    }
};

namespace detail {
// file_part.rs:100-107's walk over a chunk's locations, one step: the first location from `start`
// on that reads and holds `size` bytes (a copy of another size cannot hash to the digest; the
// reference hashes it and moves on); *next = the index after it.  nullptr when none is left.
inline const Bytes* next_copy(const ChunkStore& src, const Chunk& c, size_t start, size_t size,
                              size_t* next) {
    for (size_t j = start; j < c.locations.size(); ++j) {
        const Bytes* b = src.find(c.locations[j]);
        if (b && b->size() == size) {
            *next = j + 1;
            return b;
        }
    }
    *next = c.locations.size();
    return nullptr;
}

// Chunks to load next for a part short of d verified chunks: those whose copy failed first (at
// their next location: the reference walks a chunk's locations before it draws another chunk),
// then the untried ones.
inline std::vector<size_t> draw_order(const uint8_t* good, const uint8_t* tried,
                                      const uint8_t* exhausted, size_t t) {
    std::vector<size_t> order;
    for (size_t i = 0; i < t; ++i)
        if (tried[i] && !good[i] && !exhausted[i]) order.push_back(i);
    for (size_t i = 0; i < t; ++i)
        if (!tried[i] && !exhausted[i]) order.push_back(i);
    return order;
}
}  // namespace detail

// file::FilePart.
struct FilePart {
    size_t chunksize = 0;
    std::vector<Chunk> data;
    std::vector<Chunk> parity;

    size_t len_bytes() const { return chunksize * data.size(); }

    // write_with_encoder (file_part.rs:137-225): L = ceil(length/d); data chunk j =
    // data_buf[L*j .. L*(j+1)] (data_buf zero padded to d*L, writer.rs:172); parity from
    // encode_sep; every chunk hashed, in order, and written to `dest`, its location recorded.
    // dest_mu (optional): held while the chunks go into `dest` (several parts written at once,
    // FileWriteBuilder::concurrency); the GPU work runs outside it.
    static FilePart write_with_encoder(const ReedSolomon& encoder, ChunkStore& dest,
                                       const Bytes& data_buf, size_t length,
                                       std::mutex* dest_mu = nullptr) {
        const size_t d = encoder.data_shard_count(), p = encoder.parity_shard_count();
        if (length > data_buf.size()) throw std::invalid_argument("length > data_buf.len()");
        const size_t L = (length + d - 1) / d;
        if (data_buf.size() < d * L) throw std::invalid_argument("data_buf shorter than d*L");
        Bytes parity(p * L);
        std::vector<uint8_t> digests(32 * (d + p));
        size_t chunksize = 0;
        detail::check(cec_part_encode(encoder.raw(), data_buf.data(), length, parity.data(),
                                      digests.data(), &chunksize));
        FilePart part;
        part.chunksize = chunksize;
        std::unique_lock<std::mutex> lk;
        if (dest_mu) lk = std::unique_lock<std::mutex>(*dest_mu);
        for (size_t i = 0; i < d + p; ++i) {
            std::array<uint8_t, 32> h{};
            std::memcpy(h.data(), &digests[32 * i], 32);
            Chunk c{Sha256Hash(h), {}};
            const uint8_t* src = i < d ? &data_buf[i * L] : &parity[(i - d) * L];
            c.locations.push_back(dest.write_shard(c.hash, src, L));
            (i < d ? part.data : part.parity).push_back(std::move(c));
        }
        return part;
    }

    // read_with_context (file_part.rs:73-135): chunks drawn until d verify (data chunks first
    // here, so an intact part needs no rebuild; the reference samples at random, and any d
    // verified chunks decode to the same bytes), each at its first copy whose hash verifies --
    // a failed copy is followed by the same chunk's next location before another chunk is drawn
    // (:100-107) -- one hashing launch per round; missing data rebuilt with reconstruct_data
    // (TooFewShardsPresent when the copies run out); the d data chunks concatenated.
    Bytes read_with_context(const ChunkStore& src) const {
        const size_t d = data.size(), t = d + parity.size();
        std::vector<uint8_t> good(t), tried(t), exhausted(t);
        std::vector<size_t> cursor(t);
        Shards all(t);
        size_t have = 0;
        while (have < d) {
            std::vector<size_t> idx;
            std::vector<const Bytes*> copies;
            for (size_t i : detail::draw_order(good.data(), tried.data(), exhausted.data(), t)) {
                if (have + idx.size() >= d) break;
                tried[i] = 1;
                const Bytes* b = detail::next_copy(src, chunk(i), cursor[i], chunksize, &cursor[i]);
                if (!b) {
                    exhausted[i] = 1;
                    continue;
                }
                idx.push_back(i);
                copies.push_back(b);
            }
            if (idx.empty()) throw ErasureError(Error::TooFewShardsPresent);
            const std::vector<Sha256Hash> got = Sha256Hash::from_bufs(copies);  // one launch
            for (size_t k = 0; k < idx.size(); ++k)
                if (got[k] == chunk(idx[k]).hash) {
                    good[idx[k]] = 1;
                    all[idx[k]] = *copies[k];
                    ++have;
                }
        }
        bool complete = true;
        for (size_t i = 0; i < d; ++i) complete = complete && all[i].has_value();
        if (!complete) ReedSolomon(d, parity.size()).reconstruct_data(all);
        Bytes out;
        out.reserve(len_bytes());
        for (size_t i = 0; i < d; ++i) out.insert(out.end(), all[i]->begin(), all[i]->end());
        return out;
    }

    // verify (file_part.rs:228-251): every location of every chunk read and its copy checked
    // against the chunk's hash (one hashing launch).
    PartReport verify(const ChunkStore& src) const {
        PartReport rep;
        check_locations(src, rep, nullptr, nullptr);
        rep.summarize();
        return rep;
    }

    // resilver (file_part.rs:253-390): every location of every chunk read and checked; each
    // chunk's first valid copy kept; if a chunk has none, reconstruct (data AND parity), then
    // every such chunk written to `dest` and the new location APPENDED to the chunk's list
    // (chunk.locations.extend, :346).  A chunk with a bad copy and a valid one is not rewritten.
    // Rebuilt chunks report Resilvered.  dest_mu (optional): held while reading from and writing
    // to `dest` (several parts resilvered at once, FileReference::resilver); the GPU work runs
    // outside it.
    PartReport resilver(ChunkStore& dest, std::mutex* dest_mu = nullptr) {
        PartReport rep;
        const size_t d = data.size(), t = d + parity.size();
        Shards all(t);
        check_locations(dest, rep, &all, dest_mu);
        rep.summarize();
        bool any_missing = false;
        for (const auto& s : all) any_missing = any_missing || !s;
        if (!any_missing) return rep;
        try {
            ReedSolomon(d, parity.size()).reconstruct(all);
        } catch (const ErasureError& e) {  // recorded in the report, as write_error
            rep.write_error = e.error();
            return rep;
        }
        std::unique_lock<std::mutex> lk;
        if (dest_mu) lk = std::unique_lock<std::mutex>(*dest_mu);
        for (size_t i = 0; i < t; ++i) {
            if (rep.chunks[i] == LocationIntegrity::Valid) continue;
            Chunk& c = chunk_mut(i);
            c.locations.push_back(dest.write_shard(c.hash, *all[i]));
            rep.new_locations.push_back(c.locations.back());
            rep.chunks[i] = LocationIntegrity::Resilvered;
        }
        return rep;
    }

    const Chunk& chunk(size_t i) const { return i < data.size() ? data[i] : parity[i - data.size()]; }
    Chunk& chunk_mut(size_t i) { return i < data.size() ? data[i] : parity[i - data.size()]; }

   private:
    // Every location's copy of every chunk hashed in one launch: rep.locations filled; with
    // `first_valid`, each chunk's first valid copy is copied there.  The copies are taken under
    // `mu` (a resilver elsewhere may be writing the store).
    void check_locations(const ChunkStore& src, PartReport& rep, Shards* first_valid,
                         std::mutex* mu) const {
        const size_t t = data.size() + parity.size();
        rep.locations.assign(t, {});
        std::vector<Bytes> held;  // copies taken under the lock
        std::vector<const Bytes*> copies;
        std::vector<std::pair<size_t, size_t>> at;
        {
            std::unique_lock<std::mutex> lk;
            if (mu) lk = std::unique_lock<std::mutex>(*mu);
            held.reserve(64);
            for (size_t i = 0; i < t; ++i) {
                const Chunk& c = chunk(i);
                rep.locations[i].assign(c.locations.size(), LocationIntegrity::Unavailable);
                for (size_t j = 0; j < c.locations.size(); ++j) {
                    const Bytes* b = src.find(c.locations[j]);
                    if (!b) continue;
                    if (b->size() != chunksize) {  // cannot hash to the digest
                        rep.locations[i][j] = LocationIntegrity::Invalid;
                        continue;
                    }
                    at.emplace_back(i, j);
                    if (mu) held.push_back(*b);
                    else copies.push_back(b);
                }
            }
        }
        if (mu)
            for (const Bytes& b : held) copies.push_back(&b);
        const std::vector<Sha256Hash> got = Sha256Hash::from_bufs(copies);  // one launch
        for (size_t k = 0; k < at.size(); ++k) {
            const auto [i, j] = at[k];
            const bool ok = got[k] == chunk(i).hash;
            rep.locations[i][j] = ok ? LocationIntegrity::Valid : LocationIntegrity::Invalid;
            if (ok && first_valid && !(*first_valid)[i]) (*first_valid)[i] = *copies[k];
        }
    }
};

// file::FileReference: total length + parts (the metadata document).
void release_thread_buffers();

struct FileReference {
    friend void release_thread_buffers();
    std::optional<uint64_t> length;
    std::vector<FilePart> parts;
    // Part futures in flight on the per-part paths, as the reference: FileReadBuilder's default
    // buffer (reader.rs), verify's FuturesOrdered over every part (capped here at 64 threads),
    // resilver's buffered(10).
    static constexpr size_t kReadBuffer = 5, kVerifyBuffer = 64, kResilverBuffer = 10;

    // FileReference::read: every part's data, truncated to `length` (file_reference.rs:49-56).
    // parts_per_batch > 0: runs of parts of one shape go through the multi-GPU scheduler
    // (cec_multi: a whole window of parts verified + rebuilt per launch, sharded over `devices`,
    // default the current device) the way the reference reads (file_part.rs:86-122): d chunks
    // loaded per part, and for a part whose loaded chunks do not all verify, the failed chunks'
    // next locations and then more chunks loaded and the part resubmitted (CEC_PRESENT_VERIFIED
    // marks the chunks already verified) until d verify or the copies run out
    // (TooFewShardsPresent).  Same bytes and the same failure as the per-part path.
    Bytes read(const ChunkStore& src, size_t parts_per_batch = 0, size_t depth = 4,
               const std::vector<int>& devices = {}) const {
        uint64_t total = 0;
        for (const FilePart& part : parts) total += part.len_bytes();
        if (length && *length < total) total = *length;
        Bytes out(static_cast<size_t>(total));
        size_t at = 0;
        read_to(
            src,
            [&](const uint8_t* p, size_t n) {
                detail::parallel_copy(out.data() + at, p, n);
                at += n;
            },
            parts_per_batch, depth, devices);
        return out;
    }
    // FileReadBuilder's reader (reader.rs:40-75) as a stream: the file's bytes in order (the
    // last part truncated to `length`, file_reference.rs:49-56) handed to sink(bytes, n) piece by
    // piece — a batched window of parts at a time, straight from the page-locked buffer the
    // GPU's output landed in (valid during the call only).  Same bytes and failures as read().
    template <typename Sink>
    void read_to(const ChunkStore& src, Sink&& sink, size_t parts_per_batch = 0, size_t depth = 4,
                 const std::vector<int>& devices = {}) const {
        read_span_to(src, 0, parts.size(), 0, len_bytes(), sink, parts_per_batch, depth, devices);
    }
    // FileReference::len_bytes (file_reference.rs:49-56): `length`, else the parts' bytes.
    uint64_t len_bytes() const {
        if (length) return *length;
        uint64_t total = 0;
        for (const FilePart& part : parts) total += part.len_bytes();
        return total;
    }
    // Parts [k_begin, k_end) read as read_to reads them; of their bytes (d*L per part, the
    // padding of a short part included) the first `skip` are dropped and at most `limit` go to
    // the sink -- reader.rs:40-67's read_skip and bytes_remaining (FileReadBuilder below).
    template <typename Sink>
    void read_span_to(const ChunkStore& src, size_t k_begin, size_t k_end, uint64_t skip,
                      uint64_t limit, Sink&& sink, size_t parts_per_batch = 0, size_t depth = 4,
                      const std::vector<int>& devices = {}, size_t buffer = kReadBuffer) const {
        k_end = std::min(k_end, parts.size());
        if (k_begin >= k_end) return;
        auto emit = [&](const uint8_t* p, size_t n) {
            const size_t s = size_t(std::min<uint64_t>(n, skip));
            p += s;
            n -= s;
            skip -= s;
            const size_t m = size_t(std::min<uint64_t>(n, limit));
            if (m) sink(p, m);
            limit -= m;
        };
        if (!parts_per_batch) {  // FileReadBuilder: part reads buffered(buffer) (reader.rs:63)
            detail::ordered_concurrent(
                k_end - k_begin, buffer,
                [&](size_t k) { return parts[k_begin + k].read_with_context(src); },
                [&](size_t, const Bytes& b) { emit(b.data(), b.size()); });
            return;
        }
        for_runs(parts_per_batch, [&](size_t k0, size_t n) {
            // a run shares one scheduler, so its parts share the whole shape: the metadata allows
            // a different d/p per part (file_part.rs:77 builds a codec per part)
            if (n < 2) {
                const Bytes b = parts[k0].read_with_context(src);
                emit(b.data(), b.size());
            } else {
                read_run(src, k0, n, parts_per_batch, depth, devices, emit);
            }
        }, k_begin, k_end);
    }
    // FileReference::verify / resilver (file_reference.rs:78-113 over FilePart::verify /
    // resilver, file_part.rs:228-390).  parts_per_batch > 0: runs of parts of one shape go
    // through the multi-GPU scheduler (cec_multi_verify / cec_multi_resilver over `devices`):
    // every location of every chunk hashed against its metadata digest, and (resilver) every
    // chunk with no valid copy rebuilt, written back and its new location appended.  Same
    // reports as the per-part calls: a part that cannot be rebuilt gets write_error in its
    // report and the remaining parts are still resilvered (file_reference.rs:103-110 collects
    // every report).
    std::vector<PartReport> verify(const ChunkStore& src, size_t parts_per_batch = 0,
                                   size_t depth = 4, const std::vector<int>& devices = {}) const {
        std::vector<PartReport> r(parts.size());
        if (!parts_per_batch) {  // every part at once (FuturesOrdered, file_reference.rs:78-86)
            detail::ordered_concurrent(
                parts.size(), kVerifyBuffer, [&](size_t k) { return parts[k].verify(src); },
                [&](size_t k, PartReport rep) { r[k] = std::move(rep); });
            return r;
        }
        for_runs(parts_per_batch, [&](size_t k0, size_t n) {
            if (n < 2) r[k0] = parts[k0].verify(src);
            else check_run(const_cast<ChunkStore&>(src), k0, n, parts_per_batch, depth, devices,
                           nullptr, r);  // verify only reads the store
        });
        return r;
    }
    std::vector<PartReport> resilver(ChunkStore& dest, size_t parts_per_batch = 0,
                                     size_t depth = 4, const std::vector<int>& devices = {}) {
        std::vector<PartReport> r(parts.size());
        if (!parts_per_batch) {  // buffered(10) (file_reference.rs:103-110)
            std::mutex dest_mu;
            detail::ordered_concurrent(
                parts.size(), kResilverBuffer,
                [&](size_t k) { return parts[k].resilver(dest, &dest_mu); },
                [&](size_t k, PartReport rep) { r[k] = std::move(rep); });
            return r;
        }
        for_runs(parts_per_batch, [&](size_t k0, size_t n) {
            if (n < 2) r[k0] = parts[k0].resilver(dest);
            else check_run(dest, k0, n, parts_per_batch, depth, devices, &parts, r);
        });
        return r;
    }

   private:
    // fn(k0, n) over runs of parts of one shape (whole shape: chunk size, d and p) among parts
    // [k_begin, k_end); runs of one part when batching is off.
    template <typename Fn>
    void for_runs(size_t parts_per_batch, Fn fn, size_t k_begin = 0,
                  size_t k_end = std::numeric_limits<size_t>::max()) const {
        k_end = std::min(k_end, parts.size());
        size_t k = k_begin;
        while (k < k_end) {
            size_t run = 1;
            while (parts_per_batch && k + run < k_end &&
                   parts[k + run].chunksize == parts[k].chunksize &&
                   parts[k + run].data.size() == parts[k].data.size() &&
                   parts[k + run].parity.size() == parts[k].parity.size())
                ++run;
            fn(k, run);
            k += run;
        }
    }

    // One verify / resilver window in flight.
    struct CheckWindow {
        size_t first = 0, n = 0;
        uint64_t job = 0;
        bool live = false;
        // [W][t][L] the copies (DMA'd directly); verify grows it when a window has more copies
        // than chunks (chunks with several locations), and keeps it for the next windows
        detail::PinnedBuf chunks;
        detail::PinnedBuf rebuilt;  // [W][t][L] resilver: the rebuilt chunks
        detail::PinnedBuf prepass;  // resilver: the copies of chunks with several locations
        std::vector<uint8_t> present, expected, verified;
        std::vector<int> status;
        // verify: one item per copy hashed, (window part, chunk, location); resilver: the chunks
        // whose lone copy the resilver job hashes
        std::vector<std::array<uint32_t, 3>> items;
    };
    static std::array<CheckWindow, 8>& check_windows() {
        thread_local std::array<CheckWindow, 8> win;
        return win;
    }

    // verify / resilver of parts [k0, k0 + n) (one shape) through cec_multi: windows of one
    // pipeline batch per shard (ppb x shards parts), up to `depth` in flight, so loading the next
    // windows overlaps the GPU work; reports (and resilver's write-backs) are made window by
    // window in file order.  verify: every copy of the window is one item of a cec_multi_verify
    // job, d + p items per scheduler row whatever chunk they belong to.  resilver: a window whose
    // chunks have one location each is one cec_multi_resilver job; the copies of chunks with
    // several locations are hashed first (a verify job) and their first valid copy goes to the
    // resilver job flagged CEC_PRESENT_VERIFIED: every copy is hashed exactly once.
    // rebuilt_into: resilver (its parts get the new locations); nullptr: verify.
    void check_run(ChunkStore& store, size_t k0, size_t n, size_t ppb, size_t depth,
                   const std::vector<int>& devices, std::vector<FilePart>* rebuilt_into,
                   std::vector<PartReport>& reports) const {
        const bool resilver = rebuilt_into != nullptr;
        const FilePart& first = parts[k0];
        const size_t d = first.data.size(), t = d + first.parity.size(), L = first.chunksize;
        const std::vector<int> devs = detail::devices_or_current(devices);
        cec_multi* m = detail::cached_multi(d, t - d, L, ppb, depth, devs);
        const size_t W = ppb * devs.size();
        std::array<CheckWindow, 8>& win = check_windows();
        const size_t nwin = std::min<size_t>(std::max<size_t>(depth, 2), win.size());
        // the report skeleton of window part q: Unavailable where a location does not read,
        // Invalid where its copy has the wrong size, Valid (to be checked) otherwise
        auto skeleton = [&](size_t at, size_t cnt) {
            for (size_t q = 0; q < cnt; ++q) {
                const FilePart& part = parts[k0 + at + q];
                PartReport& rep = reports[k0 + at + q];
                rep = PartReport{};
                rep.locations.assign(t, {});
                for (size_t i = 0; i < t; ++i) {
                    const Chunk& c = part.chunk(i);
                    rep.locations[i].assign(c.locations.size(), LocationIntegrity::Unavailable);
                    for (size_t j = 0; j < c.locations.size(); ++j) {
                        const Bytes* b = store.find(c.locations[j]);
                        if (b) rep.locations[i][j] = b->size() == L ? LocationIntegrity::Valid
                                                                    : LocationIntegrity::Invalid;
                    }
                }
            }
        };
        // a verify job over `items` of window [at, at + cnt): copies into buf (g rows of t),
        // flags into `verified`; returns the job
        auto verify_items = [&](const std::vector<std::array<uint32_t, 3>>& items, size_t at,
                                uint8_t* buf, std::vector<uint8_t>& present,
                                std::vector<uint8_t>& expected, std::vector<uint8_t>& verified) {
            const size_t g = (items.size() + t - 1) / t;
            present.assign(g * t, 0);
            expected.assign(g * t * 32, 0);
            verified.assign(g * t, 0);
            detail::parallel_for(items.size(), [&](size_t x) {
                const auto& it = items[x];
                const Chunk& c = parts[k0 + at + it[0]].chunk(it[1]);
                std::memcpy(buf + x * L, store.find(c.locations[it[2]])->data(), L);
                std::memcpy(&expected[x * 32], c.hash.digest().data(), 32);
                present[x] = 1;
            });
            uint64_t job = 0;
            detail::check_multi(cec_multi_verify(m, buf, present.data(), expected.data(), g,
                                                 verified.data(), &job));
            return job;
        };
        auto submit = [&](CheckWindow& w, size_t at, size_t cnt) {
            skeleton(at, cnt);
            uint8_t* chunks = w.chunks.reserve(W * t * L, devs[0]);
            w.items.clear();
            if (!resilver) {
                for (size_t q = 0; q < cnt; ++q)
                    for (size_t i = 0; i < t; ++i) {
                        const auto& locs = reports[k0 + at + q].locations[i];
                        for (size_t j = 0; j < locs.size(); ++j)
                            if (locs[j] == LocationIntegrity::Valid)
                                w.items.push_back({uint32_t(q), uint32_t(i), uint32_t(j)});
                    }
                // page-locked whatever the count: a pageable spill would go through the
                // scheduler's staging copies, into memory touched for the first time
                uint8_t* buf = w.items.size() > W * t ? w.chunks.reserve(w.items.size() * L, devs[0])
                                                      : chunks;
                w.job = w.items.empty() ? 0 : verify_items(w.items, at, buf, w.present,
                                                          w.expected, w.verified);
            } else {
                // chunks with several locations: every copy hashed first (file_part.rs:277-289)
                std::vector<std::array<uint32_t, 3>> multi;
                for (size_t q = 0; q < cnt; ++q)
                    for (size_t i = 0; i < t; ++i) {
                        const auto& locs = reports[k0 + at + q].locations[i];
                        if (locs.size() < 2) continue;
                        for (size_t j = 0; j < locs.size(); ++j)
                            if (locs[j] == LocationIntegrity::Valid)
                                multi.push_back({uint32_t(q), uint32_t(i), uint32_t(j)});
                    }
                if (!multi.empty()) {
                    uint8_t* buf = w.prepass.reserve(((multi.size() + t - 1) / t) * t * L, devs[0]);
                    std::vector<uint8_t> pr, ex, ver;
                    const uint64_t job = verify_items(multi, at, buf, pr, ex, ver);
                    detail::check_multi(cec_multi_wait(m, job));
                    for (size_t x = 0; x < multi.size(); ++x)
                        reports[k0 + at + multi[x][0]].locations[multi[x][1]][multi[x][2]] =
                            ver[x] ? LocationIntegrity::Valid : LocationIntegrity::Invalid;
                }
                uint8_t* rebuilt = w.rebuilt.reserve(W * t * L, devs[0]);
                w.present.assign(cnt * t, 0);
                w.expected.resize(cnt * t * 32);
                w.verified.assign(cnt * t, 0);
                w.status.assign(cnt, 0);
                for (size_t q = 0; q < cnt; ++q)
                    for (size_t i = 0; i < t; ++i) {
                        const auto& locs = reports[k0 + at + q].locations[i];
                        if (locs.size() == 1 && locs[0] == LocationIntegrity::Valid)
                            w.items.push_back({uint32_t(q), uint32_t(i), 0});
                    }
                detail::parallel_for(cnt, [&](size_t q) {
                    const FilePart& part = parts[k0 + at + q];
                    const auto& rl = reports[k0 + at + q].locations;
                    for (size_t i = 0; i < t; ++i) {
                        const Chunk& c = part.chunk(i);
                        std::memcpy(&w.expected[(q * t + i) * 32], c.hash.digest().data(), 32);
                        const auto& locs = rl[i];
                        const auto valid = std::find(locs.begin(), locs.end(),
                                                     LocationIntegrity::Valid);
                        if (valid == locs.end()) continue;
                        const size_t j = size_t(valid - locs.begin());
                        std::memcpy(chunks + (q * t + i) * L, store.find(c.locations[j])->data(), L);
                        // a lone copy is hashed by the resilver job; one from a chunk with several
                        // locations was verified above
                        w.present[q * t + i] = locs.size() == 1 ? 1 : CEC_PRESENT_VERIFIED;
                    }
                });
                detail::check_multi(cec_multi_resilver(m, chunks, w.present.data(),
                                                       w.expected.data(), cnt, rebuilt,
                                                       w.verified.data(), w.status.data(), nullptr,
                                                       &w.job));
            }
            w.first = at;
            w.n = cnt;
            w.live = true;
        };
        auto collect = [&](CheckWindow& w) {
            w.live = false;
            if (!resilver) {
                if (!w.items.empty()) detail::check_multi(cec_multi_wait(m, w.job));
                for (size_t x = 0; x < w.items.size(); ++x) {
                    const auto& it = w.items[x];
                    reports[k0 + w.first + it[0]].locations[it[1]][it[2]] =
                        w.verified[x] ? LocationIntegrity::Valid : LocationIntegrity::Invalid;
                }
                for (size_t q = 0; q < w.n; ++q) reports[k0 + w.first + q].summarize();
                return;
            }
            detail::check_multi(cec_multi_wait(m, w.job));
            for (const auto& it : w.items)  // the lone copies the resilver job hashed
                reports[k0 + w.first + it[0]].locations[it[1]][0] =
                    w.verified[it[0] * t + it[1]] ? LocationIntegrity::Valid
                                                  : LocationIntegrity::Invalid;
            const uint8_t* rebuilt = w.rebuilt.reserve(W * t * L, devs[0]);
            for (size_t q = 0; q < w.n; ++q) {
                PartReport& rep = reports[k0 + w.first + q];
                rep.summarize();
                bool missing = false;
                for (size_t i = 0; i < t; ++i) missing = missing || !w.verified[q * t + i];
                if (!missing) continue;
                if (w.status[q] != CEC_OK) {  // this part's write_error; the others go on
                    if (w.status[q] >= CEC_TOO_FEW_SHARDS && w.status[q] <= CEC_INVALID_INDEX)
                        rep.write_error = static_cast<Error>(w.status[q]);
                    else
                        detail::check(w.status[q]);  // an engine failure is the job's
                    continue;
                }
                FilePart& part = (*rebuilt_into)[k0 + w.first + q];
                for (size_t i = 0; i < t; ++i) {
                    if (w.verified[q * t + i]) continue;
                    Chunk& c = part.chunk_mut(i);
                    c.locations.push_back(store.write_shard(c.hash, rebuilt + (q * t + i) * L, L));
                    rep.new_locations.push_back(c.locations.back());
                    rep.chunks[i] = LocationIntegrity::Resilvered;
                }
            }
        };
        try {
            size_t at = 0;
            for (size_t i = 0; at < n || std::any_of(win.begin(), win.begin() + nwin,
                                                     [](const CheckWindow& w) { return w.live; });
                 ++i) {
                CheckWindow& w = win[i % nwin];  // collected in submission order
                if (w.live) collect(w);
                if (at < n) {
                    const size_t cnt = std::min(W, n - at);
                    submit(w, at, cnt);
                    at += cnt;
                }
            }
        } catch (...) {
            for (auto& w : win)  // no job may still write into the window buffers
                if (w.live) {
                    if (resilver || !w.items.empty()) (void)cec_multi_wait(m, w.job);
                    w.live = false;
                }
            throw;
        }
    }

    // The retry of a window's failed parts (file_part.rs:92-107), kept with the window so its
    // first round runs on the GPU while the reader loads and submits the next window.
    struct ReadRetry {
        bool active = false;     // the window has failed parts to finish
        bool in_flight = false;  // a round's job is queued
        uint64_t job = 0;
        size_t f = 0, g = 0;  // failed parts; parts in the round in flight
        std::vector<size_t> failed, open;
        std::vector<uint8_t> tried, good, exhausted;  // [f][t]
        std::vector<size_t> cursor;                   // [f][t]
        std::vector<const Bytes*> held;  // [f][t] the copy each chunk verified with
        std::vector<int32_t> cid;        // [f] carry id of the part's verified chunks (-1 none)
        // the round's job: [g][t] chunks (page-locked: they go up without staging), flags,
        // digests, results, carry ids
        detail::PinnedBuf chunks, data;
        std::vector<uint8_t> present, expected, verified;
        std::vector<int> status;
        std::vector<int32_t> carry_in, carry_out;
    };

    // One window of a run in flight: its parts, loaded chunk buffers and results.
    struct ReadWindow {
        size_t first = 0, n = 0;
        uint64_t job = 0;
        std::chrono::steady_clock::time_point sent;  // when the job (or the last round) went out
        bool live = false;     // its read job was submitted and its parts not yet emitted
        bool checked = false;  // its read job was waited for (and its retry started)
        detail::PinnedBuf chunks;  // [W][t][L] loaded chunk bytes (DMA'd directly)
        detail::PinnedBuf out;     // [W][d][L] rebuilt data chunks and retried parts' data
        std::vector<const uint8_t*> ptrs;  // [n][d] where each data chunk of each part is
        std::vector<uint8_t> present, expected, verified, exhausted;
        std::vector<size_t> cursor;  // per chunk: the next location to read
        std::vector<int> status;
        std::vector<int32_t> carry;  // per part: the scheduler's carry id of its verified chunks
        ReadRetry retry;
    };
    static constexpr size_t kMaxReadWindows = 8;
    // The windows (and their page-locked buffers) of this thread, shared by every read_run
    // instantiation: a thread_local inside the template would pin a new set per sink type.
    static std::array<ReadWindow, kMaxReadWindows>& read_windows() {
        thread_local std::array<ReadWindow, kMaxReadWindows> win;
        return win;
    }

    // Parts [k0, k0 + n) (one shape) through cec_multi in windows of one pipeline batch per
    // shard (ppb x shards parts), up to `depth` windows' read jobs in flight, so loading the next
    // windows overlaps the GPU work and the output of the earlier ones; each window's data goes to
    // emit() in file order (the loaded data chunks straight from the window's chunk buffer, the
    // rebuilt ones from its output: CEC_READ_REBUILT_ONLY).  Every window is polled: checked (its
    // job waited for, the first round of its failed parts' retry queued as a CEC_MULTI_AHEAD job)
    // as soon as its job is done, and its next retry round queued as soon as the last one is, so
    // retries run beside the loading of the next windows: depth + 1 window buffers.
    template <typename Emit>
    void read_run(const ChunkStore& src, size_t k0, size_t n, size_t ppb, size_t depth,
                  const std::vector<int>& devices, Emit& emit) const {
        const FilePart& first = parts[k0];
        const size_t d = first.data.size(), t = d + first.parity.size(), L = first.chunksize;
        const std::vector<int> devs = detail::devices_or_current(devices);
        cec_multi* m = detail::cached_multi(d, t - d, L, ppb, depth, devs);
        const size_t W = ppb * devs.size();
        const size_t nwin = std::min(std::max<size_t>(depth, 2), kMaxReadWindows - 1);
        const size_t R = nwin + 1;
        std::array<ReadWindow, kMaxReadWindows>& win = read_windows();
        auto submit = [&](ReadWindow& w, size_t at, size_t cnt) {
            uint8_t* ch = w.chunks.reserve(W * t * L, devs[0]);
            uint8_t* out = w.out.reserve(W * d * L, devs[0]);
            w.present.assign(cnt * t, 0);
            w.expected.resize(cnt * t * 32);
            w.verified.assign(cnt * t, 0);
            w.exhausted.assign(cnt * t, 0);
            w.cursor.assign(cnt * t, 0);
            w.status.assign(cnt, 0);
            w.carry.assign(cnt, -1);
            w.ptrs.assign(cnt * d, nullptr);
            // The reference loads d chunks per part (file_part.rs:86-107): the first d that have
            // a copy here (data chunks first: no rebuild when they are all there), each at its
            // first location that reads.
            detail::ReadTimes& times = detail::read_times();
            ++times.windows;
            detail::Timed load_time(times.load);
            detail::parallel_for(cnt, [&](size_t q) {
                const FilePart& part = parts[k0 + at + q];
                size_t loaded = 0;
                for (size_t i = 0; i < t; ++i) {
                    std::memcpy(&w.expected[(q * t + i) * 32], part.chunk(i).hash.digest().data(), 32);
                    if (loaded == d) continue;
                    const Bytes* bytes =
                        detail::next_copy(src, part.chunk(i), 0, L, &w.cursor[q * t + i]);
                    if (!bytes) {
                        w.exhausted[q * t + i] = 1;
                        continue;
                    }
                    std::memcpy(ch + (q * t + i) * L, bytes->data(), L);
                    w.present[q * t + i] = 1;
                    ++loaded;
                }
            });
            // REBUILT_ONLY: only the rebuilt data chunks come down; a loaded one is emitted from
            // the window's chunk buffer it went up from (w.ptrs says which)
            detail::check_multi(cec_multi_read_carry(m, ch, w.present.data(), w.expected.data(),
                                                     cnt, out, w.verified.data(), w.status.data(),
                                                     w.ptrs.data(), CEC_READ_REBUILT_ONLY, nullptr,
                                                     detail::read_carry() ? w.carry.data() : nullptr,
                                                     &w.job));
            w.sent = std::chrono::steady_clock::now();
            w.first = at;
            w.n = cnt;
            w.live = true;
            w.checked = false;
            w.retry.active = w.retry.in_flight = false;
        };
        auto check = [&](ReadWindow& w) {
            w.checked = true;
            detail::check_multi(cec_multi_wait(m, w.job));
            detail::read_times().job_latency +=
                std::chrono::duration<double>(std::chrono::steady_clock::now() - w.sent).count();
            std::vector<size_t> failed;
            for (size_t q = 0; q < w.n; ++q)
                if (w.status[q] != CEC_OK) failed.push_back(q);
            if (!failed.empty()) retry_start(src, m, k0, d, t, L, w, std::move(failed));
        };
        // Every live window but `skip`: checked as soon as its job is done and its retry's next
        // round queued as soon as the last one is (cec_multi_query never blocks), so retries run
        // on the GPUs while windows load and while the loop waits for another window (a round
        // costs one SHA-256 chain, ~33 ms for 1 MiB chunks, whatever its size).  all: check every
        // window whatever its state (nothing is left to load: the last retries run together).
        size_t at = 0;
        auto poll = [&](size_t first, const ReadWindow* skip, bool all) {
            for (size_t a = 0; a < R; ++a) {
                ReadWindow& x = win[(first + a) % R];
                if (!x.live || &x == skip) continue;
                if (!x.checked) {
                    if (all || cec_multi_query(m, x.job) == 1) check(x);
                } else if (x.retry.in_flight && cec_multi_query(m, x.retry.job) == 1) {
                    retry_collect(src, m, k0, d, t, L, x, x.out.reserve(W * d * L, devs[0]));
                }
            }
        };
        auto finish = [&](ReadWindow& w, size_t i) {
            uint8_t* out = w.out.reserve(W * d * L, devs[0]);
            // w's job, then its retry rounds, polling the other windows meanwhile
            detail::ReadTimes& times = detail::read_times();
            for (;;) {
                if (!w.checked && cec_multi_query(m, w.job) == 1) check(w);
                if (w.checked && w.retry.in_flight && cec_multi_query(m, w.retry.job) == 1)
                    retry_collect(src, m, k0, d, t, L, w, out);
                if (w.checked && !w.retry.in_flight) break;
                detail::Timed waited(w.checked ? times.wait_retry : times.wait_job);
                poll(i + 1, &w, at >= n);
                std::this_thread::sleep_for(std::chrono::microseconds(100));
            }
            w.retry.active = false;
            w.live = false;
            detail::Timed emit_time(detail::read_times().emit);
            // the parts' data chunks in order, runs of adjacent chunks as one piece
            const uint8_t* run = nullptr;
            size_t len = 0;
            for (const uint8_t* p : w.ptrs) {
                if (run && p == run + len) {
                    len += L;
                    continue;
                }
                if (run) emit(run, len);
                run = p;
                len = L;
            }
            if (run) emit(run, len);
        };
        try {
            for (size_t i = 0;; ++i) {
                // windows are emitted in submission order: win[i % R] was submitted R steps ago
                poll(i + 1, nullptr, at >= n);
                ReadWindow& w = win[i % R];
                if (w.live) finish(w, i);
                if (at < n) {
                    const size_t cnt = std::min(W, n - at);
                    submit(w, at, cnt);
                    at += cnt;
                } else if (std::none_of(win.begin(), win.begin() + R,
                                        [](const ReadWindow& x) { return x.live; })) {
                    break;
                }
            }
        } catch (...) {
            for (size_t x = 0; x < R; ++x) {  // no job may still write into the window buffers
                ReadWindow& w = win[x];
                if (w.live && !w.checked) (void)cec_multi_wait(m, w.job);
                if (w.retry.in_flight && cec_multi_wait(m, w.retry.job) == CEC_OK)
                    // the round's ids for its parts still short of d: nobody collects them now
                    for (size_t q = 0; q < w.retry.g && q < w.retry.carry_out.size(); ++q)
                        if (w.retry.carry_out[q] >= 0)
                            (void)cec_multi_carry_release(m, w.retry.carry_out[q]);
                if (w.live)  // carry ids the failed read will not use go back to their GPUs
                    for (int32_t id : w.carry)
                        if (id >= 0) (void)cec_multi_carry_release(m, id);
                if (w.retry.active)
                    for (int32_t id : w.retry.cid)
                        if (id >= 0) (void)cec_multi_carry_release(m, id);
                w.live = w.retry.active = w.retry.in_flight = false;
            }
            throw;
        }
    }

    // file_part.rs:92-107: a copy whose hash fails is dropped and the same chunk's next location
    // read, and a chunk with no valid copy left is replaced by another chunk.  The failed parts of
    // a window are resubmitted with the chunks that verified (marked CEC_PRESENT_VERIFIED: not
    // hashed again) plus, up to d, the failed chunks' next copies and then untried chunks, until
    // they decode or no copy is left (TooFewShardsPresent, as the reference's read).  The
    // verified chunks of a part the scheduler kept on its GPU (its carry id) are not sent again;
    // the others are re-sent from their verified copies.  retry_start queues the first round;
    // retry_collect takes a round's results (the rebuilt data of window part q going to
    // out + q*d*L) and queues the next round for the parts still short of d.
    void retry_start(const ChunkStore& src, cec_multi* m, size_t k0, size_t d, size_t t,
                     size_t L, ReadWindow& w, std::vector<size_t> failed) const {
        ReadRetry& r = w.retry;
        const size_t f = failed.size();
        r.f = f;
        r.g = 0;  // no round yet
        r.failed = std::move(failed);
        r.tried.assign(f * t, 0);
        r.good.assign(f * t, 0);
        r.exhausted.assign(f * t, 0);
        r.cursor.assign(f * t, 0);
        r.held.assign(f * t, nullptr);
        r.cid.assign(f, -1);
        for (size_t j = 0; j < f; ++j) {
            const size_t q = r.failed[j];
            r.cid[j] = w.carry[q];  // the retry holds the id now
            w.carry[q] = -1;
            for (size_t i = 0; i < t; ++i) {
                const size_t x = q * t + i;
                r.tried[j * t + i] = w.present[x] != 0;
                r.good[j * t + i] = w.verified[x] != 0;
                r.exhausted[j * t + i] = w.exhausted[x];
                r.cursor[j * t + i] = w.cursor[x];
            }
        }
        // the copies that verified in the window's pass: the location before each cursor
        for (size_t j = 0; j < f; ++j) {
            const FilePart& part = parts[k0 + w.first + r.failed[j]];
            for (size_t i = 0; i < t; ++i)
                if (r.good[j * t + i])
                    r.held[j * t + i] = src.find(part.chunk(i).locations[r.cursor[j * t + i] - 1]);
        }
        r.open.resize(f);
        for (size_t j = 0; j < f; ++j) r.open[j] = j;
        r.active = true;
        retry_round(src, m, k0, d, t, L, w);
    }

    // Builds and queues one round over the window's still-open failed parts.
    void retry_round(const ChunkStore& src, cec_multi* m, size_t k0, size_t d, size_t t,
                     size_t L, ReadWindow& w) const {
        ReadRetry& r = w.retry;
        const size_t g = r.open.size();
        ++detail::read_times().retry_rounds;
        detail::read_times().retry_parts += g;
        if (g && r.g) ++detail::read_times().later_rounds;  // a round after the first
        detail::Timed build_time(detail::read_times().retry_build);
        // kept page-locked between retries: fresh zeroed buffers cost ~200 ms of page faults
        // per retry of a dozen RS(10,4) 1 MiB parts (profiles/r6/cp_bench_*.log)
        uint8_t* chunks = r.chunks.reserve(r.f * t * L, -1);
        r.data.reserve(r.f * d * L, -1);
        r.present.assign(g * t, 0);
        r.expected.resize(g * t * 32);
        r.verified.assign(g * t, 0);
        r.status.assign(g, 0);
        r.carry_in.assign(g, -1);
        r.carry_out.assign(g, -1);
        for (size_t q = 0; q < g; ++q) {
            const size_t j = r.open[q];
            const FilePart& part = parts[k0 + w.first + r.failed[j]];
            size_t have = 0, added = 0;
            r.carry_in[q] = r.cid[j];
            for (size_t i = 0; i < t; ++i) {
                std::memcpy(&r.expected[(q * t + i) * 32], part.chunk(i).hash.digest().data(), 32);
                if (!r.good[j * t + i]) continue;
                ++have;
                if (r.cid[j] < 0)  // not kept on the GPU: send the copy that verified
                    std::memcpy(&chunks[(q * t + i) * L], r.held[j * t + i]->data(), L);
                r.present[q * t + i] = CEC_PRESENT_VERIFIED;
            }
            for (size_t i : detail::draw_order(&r.good[j * t], &r.tried[j * t], &r.exhausted[j * t], t)) {
                if (!(have + added < d)) break;
                r.tried[j * t + i] = 1;
                const Bytes* bytes = detail::next_copy(src, part.chunk(i), r.cursor[j * t + i], L,
                                                       &r.cursor[j * t + i]);
                if (!bytes) {
                    r.exhausted[j * t + i] = 1;
                    continue;
                }
                r.held[j * t + i] = bytes;
                std::memcpy(&chunks[(q * t + i) * L], bytes->data(), L);
                r.present[q * t + i] = 1;
                ++added;
            }
            if (added == 0) throw ErasureError(Error::TooFewShardsPresent);
        }
        detail::check_multi(cec_multi_read_carry(
            m, chunks, r.present.data(), r.expected.data(), g, r.data.reserve(r.f * d * L, -1),
            r.verified.data(), r.status.data(), nullptr, CEC_MULTI_AHEAD, r.carry_in.data(),
            detail::read_carry() ? r.carry_out.data() : nullptr, &r.job));
        for (size_t q = 0; q < g; ++q) r.cid[r.open[q]] = -1;  // the job's ids now
        w.sent = std::chrono::steady_clock::now();
        r.g = g;
        r.in_flight = true;
    }

    // Waits for the round in flight: the parts that decoded go to out, the others go again in
    // the next round, queued here.
    void retry_collect(const ChunkStore& src, cec_multi* m, size_t k0, size_t d, size_t t,
                       size_t L, ReadWindow& w, uint8_t* out) const {
        ReadRetry& r = w.retry;
        {
            r.in_flight = false;
            detail::check_multi(cec_multi_wait(m, r.job));
            detail::read_times().round_latency +=
                std::chrono::duration<double>(std::chrono::steady_clock::now() - w.sent).count();
            const uint8_t* data = r.data.reserve(r.f * d * L, -1);
            std::vector<size_t> still;
            for (size_t q = 0; q < r.g; ++q) {
                const size_t j = r.open[q];
                for (size_t i = 0; i < t; ++i) r.good[j * t + i] = r.verified[q * t + i] != 0;
                if (r.status[q] == CEC_OK) {
                    const size_t part = r.failed[j];
                    std::memcpy(out + part * d * L, data + q * d * L, d * L);
                    for (size_t i = 0; i < d; ++i) w.ptrs[part * d + i] = out + (part * d + i) * L;
                } else {
                    r.cid[j] = r.carry_out[q];
                    still.push_back(j);
                }
            }
            r.open.swap(still);
            if (!r.open.empty()) retry_round(src, m, k0, d, t, L, w);
            else r.active = false;
        }
    }
};

// file::FileWriteBuilder (writer.rs:88-255): the part loop of write().  Parts are
// d*chunk_size bytes of the input (the last one shorter), each zero padded and handed to
// FilePart::write_with_encoder with one shared codec.
// FileReadBuilder (reader.rs:22-173): a file's bytes from `seek` on, `take` of them (0: to the
// end), read from the parts that hold them -- the HTTP gateway's range reads (http.rs:37-56).
// Parts wholly before `seek` are not read and the first part's leading bytes are dropped, as the
// reference does (reader.rs:44-65).  Parts wholly past the range are not read either: the
// reference still reads every part after it and empties its bytes (the stream's map,
// reader.rs:67-75), so an undecodable part past the range fails its read and not this one; the
// range's bytes are the same.  batch() / devices() pick the batched path (FileReference::read_to).
class FileReadBuilder {
   public:
    explicit FileReadBuilder(const FileReference& file) : file_(&file) {}
    FileReadBuilder& seek(uint64_t s) {
        seek_ = s;
        return *this;
    }
    FileReadBuilder& take(uint64_t n) {
        take_ = n;
        return *this;
    }
    // Part reads in flight on the per-part path (reader.rs:111-114, default 5), or as many parts
    // as `bytes` hold, rounded, at least 1 (buffer_bytes, reader.rs:117-126).
    FileReadBuilder& buffer(size_t parts) {
        buffer_ = parts;
        return *this;
    }
    FileReadBuilder& buffer_bytes(size_t bytes) {
        if (!file_->parts.empty()) {
            const size_t part_len = file_->parts.front().len_bytes();
            buffer_ = std::max<size_t>((bytes + part_len / 2) / std::max<size_t>(part_len, 1), 1);
        }
        return *this;
    }
    size_t get_buffer() const { return buffer_; }
    FileReadBuilder& batch(size_t parts_per_batch, size_t depth = 4) {
        batch_ = parts_per_batch;
        depth_ = depth;
        return *this;
    }
    FileReadBuilder& devices(std::vector<int> devs) {
        devices_ = std::move(devs);
        return *this;
    }
    uint64_t get_seek() const { return seek_; }
    const FileReference& file_reference() const { return *file_; }
    // reader.rs:129-138 (a seek past the end gives 0 here; the reference's u64 subtraction would
    // underflow there).
    uint64_t len_bytes() const {
        const uint64_t length = file_->len_bytes();
        if (seek_ >= length) return 0;
        return take_ == 0 ? length - seek_ : std::min(take_, length - seek_);
    }
    template <typename Sink>
    void read_to(const ChunkStore& src, Sink&& sink) const {
        const uint64_t want = len_bytes();
        if (want == 0) return;
        const std::vector<FilePart>& parts = file_->parts;
        size_t k = 0;
        uint64_t skip = seek_;
        while (k < parts.size() && skip >= parts[k].len_bytes()) skip -= parts[k++].len_bytes();
        size_t end = k;
        for (uint64_t covered = 0; end < parts.size() && covered < skip + want; ++end)
            covered += parts[end].len_bytes();
        file_->read_span_to(src, k, end, skip, want, sink, batch_, depth_, devices_, buffer_);
    }
    Bytes read(const ChunkStore& src) const {
        Bytes out;
        out.reserve(size_t(len_bytes()));
        read_to(src, [&](const uint8_t* p, size_t n) { out.insert(out.end(), p, p + n); });
        return out;
    }

   private:
    const FileReference* file_;
    uint64_t seek_ = 0, take_ = 0;
    size_t buffer_ = FileReference::kReadBuffer, batch_ = 0, depth_ = 4;
    std::vector<int> devices_;
};

class FileWriteBuilder {
   public:
    FileWriteBuilder& chunk_size(size_t n) {
        chunk_size_ = n;
        return *this;
    }
    FileWriteBuilder& data_chunks(size_t n) {
        data_ = n;
        return *this;
    }
    FileWriteBuilder& parity_chunks(size_t n) {
        parity_ = n;
        return *this;
    }
    // Part tasks in flight for the per-part path (writer.rs:106-110 `concurrency`, default 10,
    // semaphore at :130; write() requires > 1 like writer.rs:128): that many parts are encoded
    // and hashed at once, so their per-call GPU work shares coalesced launches (DESIGN.md §4.7:
    // raise it to >= 64 for the swap to pay).  Parts still come out in file order.
    FileWriteBuilder& concurrency(size_t n) {
        concurrency_ = n;
        return *this;
    }

    // Parts per batch and batches in flight per device for the batched path (the multi-GPU
    // scheduler, cec_multi); 0 = one write_with_encoder call per part (the reference's shape).
    FileWriteBuilder& batch(size_t parts_per_batch, size_t depth = 4) {
        batch_ = parts_per_batch;
        depth_ = depth;
        return *this;
    }
    // Devices the batched path shards over (one shard per entry; default: the current device).
    FileWriteBuilder& devices(std::vector<int> devs) {
        devices_ = std::move(devs);
        return *this;
    }

    FileReference write(const uint8_t* bytes, size_t n, ChunkStore& dest) const {
        if (concurrency_ <= 1) throw std::invalid_argument("concurrency must be > 1");  // :128
        const ReedSolomon encoder(data_, parity_);  // writer.rs:131
        FileReference file;
        const size_t part_cap = data_ * chunk_size_;
        const size_t full = n / part_cap;
        size_t off = 0;
        if (batch_ && full >= 2) {  // full parts: L = chunk_size for every one of them
            write_full_parts(encoder, bytes, full, dest, file);
            off = full * part_cap;
        }
        std::vector<size_t> offs;
        for (; off < n; off += part_cap) offs.push_back(off);
        auto one_part = [&](size_t k, std::mutex* mu) {
            const size_t bytes_read = std::min(part_cap, n - offs[k]);
            Bytes data_buf(part_cap, 0);  // vec![0; data * chunk_size] (writer.rs:172)
            std::memcpy(data_buf.data(), bytes + offs[k], bytes_read);
            return FilePart::write_with_encoder(encoder, dest, data_buf, bytes_read, mu);
        };
        const size_t workers = std::min(concurrency_, offs.size());
        if (workers <= 1) {
            for (size_t k = 0; k < offs.size(); ++k) file.parts.push_back(one_part(k, nullptr));
        } else {  // `workers` part tasks at once (writer.rs:200-210), results in file order
            std::vector<FilePart> parts(offs.size());
            std::mutex dest_mu, err_mu;
            std::atomic<size_t> next{0};
            std::exception_ptr err;
            auto task = [&] {
                for (size_t k; (k = next.fetch_add(1)) < offs.size();) {
                    try {
                        parts[k] = one_part(k, &dest_mu);
                    } catch (...) {  // the first failure is the write's; stop taking parts
                        std::lock_guard<std::mutex> lk(err_mu);
                        if (!err) err = std::current_exception();
                        next.store(offs.size());
                    }
                }
            };
            std::vector<std::thread> pool;
            for (size_t w = 0; w < workers; ++w) pool.emplace_back(task);
            for (auto& th : pool) th.join();
            if (err) std::rethrow_exception(err);
            for (auto& part : parts) file.parts.push_back(std::move(part));
        }
        file.length = n;
        return file;
    }
    FileReference write(const Bytes& b, ChunkStore& dest) const { return write(b.data(), b.size(), dest); }

   public:
    // The page-locked windows of the calling thread's batched writes (see release_thread_buffers).
    struct WriteWindow {
        size_t first = 0, n = 0;
        uint64_t job = 0;
        bool live = false;
        detail::PinnedBuf parity, digests;
    };
    static std::array<WriteWindow, 2>& write_windows() {
        thread_local std::array<WriteWindow, 2> win;
        return win;
    }

   private:
    size_t chunk_size_ = size_t(1) << 20;
    size_t data_ = 3;
    size_t parity_ = 2;
    size_t batch_ = 0;
    size_t depth_ = 4;
    size_t concurrency_ = 10;  // the reference's default (writer.rs:56)
    std::vector<int> devices_;

    // The `full` parts of d*chunk_size bytes through the multi-GPU scheduler, in windows of
    // batch * depth * shards parts with two windows in flight: same FileParts and stored chunks as
    // write_with_encoder part by part.  The input bytes are already [part][d][L] (a full part is
    // d*chunk_size contiguous bytes), so each window is one job straight from them; parity and
    // digests come back into page-locked buffers.
    void write_full_parts(const ReedSolomon& encoder, const uint8_t* bytes, size_t full,
                          ChunkStore& dest, FileReference& file) const {
        (void)encoder;
        const size_t d = data_, p = parity_, t = d + p, L = chunk_size_;
        const std::vector<int> devs = detail::devices_or_current(devices_);
        cec_multi* m = detail::cached_multi(d, p, L, batch_, depth_, devs);
        const size_t W = batch_ * depth_ * devs.size();
        std::array<WriteWindow, 2>& win = write_windows();
        auto collect = [&](WriteWindow& w) {
            w.live = false;
            detail::check_multi(cec_multi_wait(m, w.job));
            const uint8_t* par = w.parity.reserve(W * p * L, devs[0]);
            const uint8_t* dig = w.digests.reserve(W * t * 32, devs[0]);
            for (size_t k = 0; k < w.n; ++k) {
                FilePart part;
                part.chunksize = L;
                for (size_t i = 0; i < t; ++i) {
                    std::array<uint8_t, 32> h{};
                    std::memcpy(h.data(), dig + (k * t + i) * 32, 32);
                    Chunk c{Sha256Hash(h), {}};
                    const uint8_t* src = i < d ? bytes + ((w.first + k) * d + i) * L
                                               : par + (k * p + (i - d)) * L;
                    c.locations.push_back(dest.write_shard(c.hash, src, L));
                    (i < d ? part.data : part.parity).push_back(std::move(c));
                }
                file.parts.push_back(std::move(part));
            }
        };
        try {
            size_t at = 0;
            int cur = 0;
            while (at < full || win[0].live || win[1].live) {
                WriteWindow& w = win[cur];
                if (w.live) collect(w);  // oldest window first: parts stay in file order
                if (at < full) {
                    const size_t cnt = std::min(W, full - at);
                    detail::check_multi(cec_multi_encode_hash(
                        m, bytes + at * d * L, cnt, w.parity.reserve(W * p * L, devs[0]),
                        w.digests.reserve(W * t * 32, devs[0]), &w.job));
                    w.first = at;
                    w.n = cnt;
                    w.live = true;
                    at += cnt;
                }
                cur ^= 1;
            }
        } catch (...) {
            for (auto& w : win)  // no job may still write into the window buffers
                if (w.live) {
                    (void)cec_multi_wait(m, w.job);
                    w.live = false;
                }
            throw;
        }
    }
};

// The batched paths keep, per thread, the most recent scheduler and the page-locked windows of
// the last writes / reads / verifies (reused by the next call: pinning costs ~0.35 s per GiB).
// A thread that is done with large files can hand them back here; the next batched call makes
// them again.  Must not be called while that thread has a batched call running (it never does
// by construction: the calls are synchronous).
inline void release_thread_buffers() {
    for (auto& w : FileWriteBuilder::write_windows()) {
        w.parity.release();
        w.digests.release();
    }
    for (auto& w : FileReference::read_windows()) {
        w.chunks.release();
        w.out.release();
        w.retry.chunks.release();
        w.retry.data.release();
    }
    for (auto& w : FileReference::check_windows()) {
        w.chunks.release();
        w.rebuilt.release();
        w.prepass.release();
    }
    detail::cached_multi_entry() = detail::CachedMulti{};
}

}  // namespace chunky_ec

#endif  // CHUNKY_EC_HPP
