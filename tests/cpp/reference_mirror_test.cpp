// reference_mirror_test.cpp — the reference's own tests for this path, restated against the C++
// host layer (include/chunky_ec.hpp) so they read like the Rust originals:
//
//   sha256                      tests/hash.rs:10-16        Hello World KAT, Display, verify
//   test_file_write             tests/file.rs:26-56        zeros (2^23 + 7 B), d,p in 1..3:
//                                                          part count and length
//   test_resilver               tests/cluster.rs:145-190   tests/cluster.rs generator (d=3, p=2,
//                                                          2^10-byte chunks): delete 1 data + 1
//                                                          parity chunk per part, verify, resilver,
//                                                          verify ideal, read back bit-exact
//   test_cluster_digests        golden fixture of the same write (tests/golden, pinned oracle)
//   test_cp_50mib               BASELINE configs[0]: `cp` of a 50 MiB file, d=3 p=2, 1 MiB
//                               chunks: 17 parts, last chunksize 699 051, read back bit-exact
//   test_range_reads            FileReadBuilder::seek / take (reader.rs:22-173) over the same
//                               file: the gateway's range reads, per part and batched
//   test_batched_paths          FileWriteBuilder::batch / FileReference::read batched through
//                               the host-staged pipelines == the per-part path, bit-exact
//   test_locations_bad_then_good  chunks listed [bad copy, good copy]: read walks the locations,
//                               verify flags exactly the bad ones, resilver appends
//   test_one_encode             JavaReedSolomon testOneEncode RS(5,5) (crate KAT)
//   test_matrix_rows            SURVEY.md Appendix A RS(3,2) / RS(10,4) parity rows
//   test_errors                 reed_solomon_erasure::Error variants of ReedSolomon::new,
//                               encode_sep and reconstruct argument checks
//   test_reconstruct_every_pattern  every 1..p erasure set of RS(4,3), data+parity
//
// Runs on a GPU (every computation goes through libchunky_ec.so).  `--list` prints the test
// names without touching the GPU.  Exit status 0 iff every test passed.
#include <array>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "chunky_ec.hpp"

namespace {

using namespace chunky_ec;

#include "golden_cluster.inc"

int g_failures = 0;

#define CHECK(cond)                                                                   \
    do {                                                                              \
        if (!(cond)) {                                                                \
            std::fprintf(stderr, "  CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++g_failures;                                                             \
            return;                                                                   \
        }                                                                             \
    } while (0)

template <typename F>
bool throws_erasure(F&& f, Error want) {
    try {
        f();
    } catch (const ErasureError& e) {
        return e.error() == want;
    }
    return false;
}

// tests/cluster.rs:95-102: 80 blocks of 256 bytes, byte x of block i = (x % 128) + i.
Bytes cluster_reader_bytes() {
    Bytes b;
    for (int i = 0; i < 80; ++i)
        for (int x = 0; x < 256; ++x) b.push_back(uint8_t((x % 128) + i));
    return b;
}

// tests/hash.rs
void sha256() {
    const std::string payload = "Hello World";
    const Sha256Hash hash = Sha256Hash::from_buf(payload);
    CHECK(hash.to_string() == "a591a6d40bf420404a011733cfb7b190d62c65bf0bcda32b57b277d9ad9f146e");
    CHECK(hash.verify(payload));
    CHECK(!hash.verify(std::string("Hello World!")));
    CHECK(Sha256Hash::from_str(hash.to_string()) == hash);
}

// tests/file.rs:26-56
void test_file_write() {
    const size_t length = (size_t(1) << 23) + 7;  // not divisible by d+p
    const size_t chunk_size = size_t(1) << 20;
    const Bytes zeros(length, 0);
    const std::string zero_mib = "30e14955ebf1352266dc2ff8067e68104607e750abb9d3b36582b8af909fcb58";
    for (size_t data = 1; data <= 3; ++data) {
        for (size_t parity = 1; parity <= 3; ++parity) {
            ChunkStore store;
            const FileReference file_ref =
                FileWriteBuilder().chunk_size(chunk_size).data_chunks(data).parity_chunks(parity).write(
                    zeros, store);
            CHECK(file_ref.length && *file_ref.length == length);
            const size_t part_size = chunk_size * data;
            CHECK(file_ref.parts.size() == (length + part_size - 1) / part_size);
            // full parts: every chunk (data and parity of zeros) is 1 MiB of zeros
            CHECK(file_ref.parts.front().data[0].hash.to_string() == zero_mib);
            CHECK(file_ref.parts.front().parity.back().hash.to_string() == zero_mib);
            CHECK(file_ref.read(store) == zeros);
        }
    }
}

// tests/cluster.rs:145-190 (test_resilver)
void test_resilver() {
    ChunkStore store;
    const Bytes input = cluster_reader_bytes();
    FileReference file_ref =
        FileWriteBuilder().chunk_size(size_t(1) << 10).data_chunks(3).parity_chunks(2).write(input, store);
    // File should be 100% valid
    for (const auto& r : file_ref.verify(store)) CHECK(r.is_ideal());
    size_t deleted_chunks = 0;
    for (const auto& part : file_ref.parts) {
        const Location& d0 = part.data.front().locations.front();  // delete 1 / 3 data chunks
        CHECK(store.erase(d0));
        CHECK(!store.read(d0));
        const Location& p0 = part.parity.front().locations.front();  // delete 1 / 2 parity chunks
        CHECK(store.erase(p0));
        CHECK(!store.read(p0));
        deleted_chunks += 2;
    }
    // File should not be 100% valid, but still available
    size_t unavailable = 0;
    for (const auto& r : file_ref.verify(store)) {
        CHECK(!r.is_ideal());
        unavailable += r.unavailable_locations();  // verify_report.unavailable_locations()
    }
    CHECK(unavailable == deleted_chunks);
    CHECK(file_ref.read(store) == input);  // reads decode around the holes
    size_t new_locations = 0;
    for (const auto& r : file_ref.resilver(store)) {
        CHECK(r.is_ideal());
        new_locations += r.new_locations.size();  // resilver_report.new_locations()
    }
    CHECK(new_locations == deleted_chunks);
    // the new locations are appended (file_part.rs:346): [the deleted one, the rewritten one]
    for (const auto& part : file_ref.parts) CHECK(part.data.front().locations.size() == 2);
    for (const auto& r : file_ref.verify(store)) CHECK(r.is_ideal());
    CHECK(file_ref.read(store) == input);
    // a corrupted chunk is not trusted: it verifies Invalid and is rebuilt by resilver
    const Location victim = file_ref.parts[2].data[1].locations.front();
    CHECK(store.corrupt(victim, 17));
    CHECK(file_ref.parts[2].verify(store).count(LocationIntegrity::Invalid) == 1);
    CHECK(file_ref.read(store) == input);
    CHECK(file_ref.parts[2].resilver(store).count(LocationIntegrity::Resilvered) == 1);
    CHECK(file_ref.parts[2].verify(store).is_ideal());
}

// Golden digests of the tests/cluster.rs write (tests/golden/golden_vectors.json "cluster").
void test_cluster_digests() {
    ChunkStore store;
    const Bytes input = cluster_reader_bytes();
    CHECK(input.size() == kClusterTotal);
    CHECK(Sha256Hash::from_buf(input).to_string() == kClusterDataSha256);
    const FileReference file_ref = FileWriteBuilder()
                                       .chunk_size(kClusterChunk)
                                       .data_chunks(kClusterD)
                                       .parity_chunks(kClusterP)
                                       .write(input, store);
    const size_t n = sizeof(kClusterParts) / sizeof(kClusterParts[0]);
    CHECK(file_ref.parts.size() == n);
    for (size_t k = 0; k < n; ++k) {
        const FilePart& part = file_ref.parts[k];
        CHECK(part.chunksize == kClusterParts[k].chunksize);
        for (size_t i = 0; i < kClusterD + kClusterP; ++i)
            CHECK(part.chunk(i).hash.to_string() == kClusterParts[k].sha256[i]);
    }
}

// n bytes of a splitmix64 stream (no repeated chunks: the store is content-addressed).
Bytes random_bytes(size_t n, uint64_t seed) {
    Bytes out(n);
    uint64_t z = seed * 0x2545F4914F6CDD1Dull + 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < n; i += 8) {
        z += 0x9E3779B97F4A7C15ull;
        uint64_t v = z;
        v = (v ^ (v >> 30)) * 0xBF58476D1CE4E5B9ull;
        v = (v ^ (v >> 27)) * 0x94D049BB133111EBull;
        v ^= v >> 31;
        std::memcpy(&out[i], &v, std::min<size_t>(8, n - i));
    }
    return out;
}

// BASELINE.json configs[0] (`chunky-bits cp` of 50 MiB into a d=3, p=2, 1 MiB-chunk cluster),
// compute part: 16 full parts + one of 2 MiB (L = ceil(2 MiB / 3) = 699 051), every chunk
// stored under its digest, the file read back bit-exact after losing 2 chunks per part.
void test_cp_50mib() {
    const size_t length = size_t(50) << 20;
    const Bytes input = random_bytes(length, 50);
    ChunkStore store;
    const FileReference f =
        FileWriteBuilder().chunk_size(size_t(1) << 20).data_chunks(3).parity_chunks(2).write(input, store);
    CHECK(f.parts.size() == 17);
    CHECK(f.parts[0].chunksize == (size_t(1) << 20));
    CHECK(f.parts[16].chunksize == 699051);
    CHECK(store.size() == 17 * 5);
    CHECK(Sha256Hash::from_buf(&input[0], size_t(1) << 20) == f.parts[0].data[0].hash);
    CHECK(Sha256Hash::from_buf(&input[size_t(48) << 20], 699051) == f.parts[16].data[0].hash);
    for (const auto& part : f.parts) {
        store.erase(part.data[2].locations[0]);
        store.erase(part.parity[1].locations[0]);
    }
    CHECK(f.read(store) == input);
}

// FileReadBuilder::seek / take (reader.rs:22-173), the gateway's Range / Prefix / Suffix reads
// (http.rs:37-56) of the 50 MiB cp file, holes in every part: the range's bytes, per part and
// batched (one and two scheduler shards); len_bytes as reader.rs:129-138.
void test_range_reads() {
    const size_t length = size_t(50) << 20, part = size_t(3) << 20;
    const Bytes input = random_bytes(length, 51);
    ChunkStore store;
    const FileReference f =
        FileWriteBuilder().chunk_size(size_t(1) << 20).data_chunks(3).parity_chunks(2).write(input, store);
    for (const auto& pt : f.parts) store.erase(pt.data[1].locations[0]);
    const uint64_t ranges[][2] = {{0, 0},           {0, 10},          {part - 1, 2},
                                  {part, part},     {5 * part + 7, 0}, {length - 699051, 0},
                                  {length - 1, 0},  {length - 100, 1000}, {length, 0},
                                  {1234567, 20 << 20}};
    for (const auto& r : ranges) {
        const uint64_t want = r[0] >= length ? 0 : r[1] == 0 ? length - r[0]
                                                             : std::min<uint64_t>(r[1], length - r[0]);
        for (size_t batch : {size_t(0), size_t(4), size_t(3)}) {
            FileReadBuilder rb(f);
            rb.seek(r[0]).take(r[1]).batch(batch);
            if (batch == 3) rb.devices({0, 0});  // two scheduler shards on one GPU
            CHECK(rb.len_bytes() == want && rb.get_seek() == r[0]);
            const Bytes got = rb.read(store);
            CHECK(got.size() == want);
            CHECK(std::equal(got.begin(), got.end(), input.begin() + std::ptrdiff_t(std::min<uint64_t>(r[0], length))));
        }
    }
}

// FileWriteBuilder::concurrency (writer.rs:106-130): 2 and 64 part tasks at once give the
// same FileParts, in file order, and the same stored chunks as the default 10; 1 is refused like
// the reference's assert.
void test_write_concurrency() {
    const size_t length = size_t(40) << 20;
    const Bytes input = random_bytes(length, 77);
    const auto b = FileWriteBuilder().chunk_size(size_t(1) << 18).data_chunks(10).parity_chunks(4);
    ChunkStore s10, s2, s64;
    const FileReference f10 = FileWriteBuilder(b).write(input, s10);
    const FileReference f2 = FileWriteBuilder(b).concurrency(2).write(input, s2);
    const FileReference f64 = FileWriteBuilder(b).concurrency(64).write(input, s64);
    CHECK(f10.parts.size() == 16 && f2.parts.size() == 16 && f64.parts.size() == 16);
    for (size_t k = 0; k < f10.parts.size(); ++k)
        for (size_t i = 0; i < 14; ++i) {
            CHECK(f10.parts[k].chunk(i).hash == f2.parts[k].chunk(i).hash);
            CHECK(f10.parts[k].chunk(i).hash == f64.parts[k].chunk(i).hash);
        }
    CHECK(s10.size() == s2.size() && s10.size() == s64.size());
    CHECK(f64.read(s64) == input);
    bool refused = false;
    try {
        ChunkStore s1;
        FileWriteBuilder(b).concurrency(1).write(input, s1);
    } catch (const std::invalid_argument&) {
        refused = true;
    }
    CHECK(refused);
}

// The host-staged pipelines behind FileWriteBuilder::batch and FileReference::read(src, n):
// identical FileParts, identical stored chunks, identical bytes read back (with holes).
void test_batched_paths() {
    for (const auto& shape : std::vector<std::array<size_t, 4>>{
             {10, 4, size_t(1) << 16, 37}, {3, 2, 1024, 20}, {20, 8, 4096, 9}}) {
        const size_t d = shape[0], p = shape[1], chunk = shape[2], n_parts = shape[3];
        const size_t length = d * chunk * (n_parts - 1) + 12345 % (d * chunk - 1) + 1;  // short last
        const Bytes input = random_bytes(length, d * 1000 + chunk);
        ChunkStore per_part, batched;
        const auto b = FileWriteBuilder().chunk_size(chunk).data_chunks(d).parity_chunks(p);
        const FileReference a = b.write(input, per_part);
        const FileReference c = FileWriteBuilder(b).batch(8, 3).write(input, batched);
        CHECK(a.parts.size() == n_parts && c.parts.size() == n_parts);
        CHECK(per_part.size() == batched.size());
        for (size_t k = 0; k < n_parts; ++k) {
            CHECK(a.parts[k].chunksize == c.parts[k].chunksize);
            for (size_t i = 0; i < d + p; ++i) {
                CHECK(a.parts[k].chunk(i).hash == c.parts[k].chunk(i).hash);
                CHECK(batched.read(c.parts[k].chunk(i).locations[0]) ==
                      per_part.read(a.parts[k].chunk(i).locations[0]));
            }
        }
        // holes: one data + one parity chunk per part, then (where p leaves room) a corrupted
        // chunk in part 3 that the read must not trust
        for (const auto& part : c.parts) {
            batched.erase(part.data[1 % d].locations[0]);
            batched.erase(part.parity[0].locations[0]);
        }
        if (p >= 3) CHECK(batched.corrupt(c.parts[3].data[0].locations[0], 5));
        CHECK(c.read(batched, 8, 3) == input);
        CHECK(c.read(batched) == input);
        // streamed (reader.rs:40-75): the same bytes in order, piece by piece, the last part cut
        // at the file length; depth 1..5 windows in flight (2..5 rings)
        for (size_t depth : {1, 3, 5}) {
            Bytes streamed;
            size_t pieces = 0;
            c.read_to(batched, [&](const uint8_t* q, size_t m) {
                streamed.insert(streamed.end(), q, q + m);
                ++pieces;
            }, 4, depth);
            if (streamed != input) {
                size_t bad = 0;
                while (bad < std::min(streamed.size(), input.size()) && streamed[bad] == input[bad]) ++bad;
                std::printf("  streamed read, depth %zu: %zu of %zu bytes, first difference at %zu "
                            "(part %zu)\n", depth, streamed.size(), input.size(), bad,
                            bad / (d * chunk));
            }
            CHECK(streamed == input);
            CHECK(pieces >= 2);
        }
        // a part with fewer than d usable chunks fails like the per-part read
        for (size_t i = 2; i < d + p; ++i) batched.erase(c.parts[5].chunk(i).locations[0]);
        CHECK(batched.corrupt(c.parts[5].chunk(0).locations[0], 1));
        CHECK(throws_erasure([&] { c.read(batched, 8, 3); }, Error::TooFewShardsPresent));
    }
}

// The batched paths sharded over several devices in one process (cec_multi): two shards on the
// first GPU (and one per GPU when more are visible), identical parts, chunks and bytes; a read
// whose d loaded chunks include a corrupted one is retried with another chunk (file_part.rs:92-107).
void test_multi_device_paths() {
    int n_dev = cec_device_count();
    std::vector<std::vector<int>> lists = {{0, 0}};
    if (n_dev > 1) {
        std::vector<int> all;
        for (int i = 0; i < n_dev; ++i) all.push_back(i);
        lists.push_back(all);
    }
    const size_t d = 10, p = 4, chunk = size_t(1) << 14, n_parts = 29;
    const size_t length = d * chunk * (n_parts - 1) + 777;
    const Bytes input = random_bytes(length, 4242);
    ChunkStore per_part;
    const auto b = FileWriteBuilder().chunk_size(chunk).data_chunks(d).parity_chunks(p);
    const FileReference a = b.write(input, per_part);
    for (const auto& devs : lists) {
        ChunkStore store;
        const FileReference c = FileWriteBuilder(b).batch(3, 2).devices(devs).write(input, store);
        CHECK(c.parts.size() == n_parts);
        for (size_t k = 0; k < n_parts; ++k)
            for (size_t i = 0; i < d + p; ++i) CHECK(a.parts[k].chunk(i).hash == c.parts[k].chunk(i).hash);
        CHECK(c.read(store, 3, 2, devs) == input);
        // data chunk 0 corrupted in every other part: the d-chunk first pass fails its hash,
        // the retry loads the next stored chunk
        for (size_t k = 0; k < n_parts; k += 2) CHECK(store.corrupt(c.parts[k].data[0].locations[0], 9));
        CHECK(c.read(store, 3, 2, devs) == input);
        // and a part whose usable chunks run out
        for (size_t i = 1; i < d + p - (d - 2); ++i) store.erase(c.parts[7].chunk(i).locations[0]);
        CHECK(throws_erasure([&] { c.read(store, 3, 2, devs); }, Error::TooFewShardsPresent));
        // the failed read (other parts' retry rounds in flight) left the thread's scheduler sound:
        // no carry entry held, and another file of the shape reads back through it
        cec_multi* m = detail::cached_multi_entry().multi.get();
        for (size_t g = 0; m && g < cec_multi_shards(m); ++g) {
            cec_multi_stats st{};
            CHECK(cec_multi_shard_stats(m, g, &st) == CEC_OK && st.carry_held == 0);
        }
        CHECK(a.read(per_part, 3, 2, devs) == input);
    }
}

// tests/cluster.rs:145-231 through the batched verify / resilver (cec_multi_verify /
// cec_multi_resilver): delete data[0] and parity[0] of every part, corrupt another chunk of some
// parts, verify reports them, resilver rebuilds exactly those chunks, verify is ideal again, and
// the file reads back bit-exact.
void test_batched_verify_resilver() {
    const size_t d = 3, p = 3, chunk = 1024;  // 2 lost + 1 corrupt leaves exactly d
    const Bytes input = random_bytes(d * chunk * 11 + 500, 99);
    ChunkStore store;
    FileReference f =
        FileWriteBuilder().chunk_size(chunk).data_chunks(d).parity_chunks(p).write(input, store);
    for (const auto& devs : std::vector<std::vector<int>>{{}, {0, 0}}) {
        for (size_t k = 0; k < f.parts.size(); ++k) {
            store.erase(f.parts[k].data[0].locations[0]);
            store.erase(f.parts[k].parity[0].locations[0]);
            if (k % 3 == 1) CHECK(store.corrupt(f.parts[k].data[2].locations[0], 7));
        }
        auto before = f.verify(store, 4, 2, devs);
        CHECK(before.size() == f.parts.size());
        for (size_t k = 0; k < f.parts.size(); ++k) {
            CHECK(!before[k].is_ideal());
            CHECK(before[k].chunks[0] == LocationIntegrity::Unavailable);
            CHECK(before[k].chunks[d] == LocationIntegrity::Unavailable);
            CHECK(before[k].chunks[2] ==
                  (k % 3 == 1 ? LocationIntegrity::Invalid : LocationIntegrity::Valid));
        }
        // the per-part verify reports the same
        const auto per_part = f.verify(store);
        for (size_t k = 0; k < f.parts.size(); ++k) {
            CHECK(per_part[k].chunks == before[k].chunks);
            CHECK(per_part[k].locations == before[k].locations);
        }
        const auto rep = f.resilver(store, 4, 2, devs);
        for (size_t k = 0; k < f.parts.size(); ++k) {
            CHECK(rep[k].chunks[0] == LocationIntegrity::Resilvered);
            CHECK(rep[k].chunks[d] == LocationIntegrity::Resilvered);
            CHECK(rep[k].chunks[2] ==
                  (k % 3 == 1 ? LocationIntegrity::Resilvered : LocationIntegrity::Valid));
        }
        {
            const auto after = f.verify(store, 4, 2, devs);
            for (size_t k = 0; k < after.size(); ++k)
                if (!after[k].is_ideal())
                    for (size_t i = 0; i < d + p; ++i)
                        if (after[k].chunks[i] != LocationIntegrity::Valid)
                            std::printf("  after resilver (%zu devices): part %zu chunk %zu state %d\n",
                                        devs.size(), k, i, int(after[k].chunks[i]));
            for (const auto& r : after) CHECK(r.is_ideal());
        }
        CHECK(f.read(store, 4, 2, devs) == input);
        // the thread's scheduler and page-locked windows handed back: the next call remakes them
        release_thread_buffers();
        CHECK(f.read(store, 4, 2, devs) == input);
        for (const auto& r : f.verify(store, 4, 2, devs)) CHECK(r.is_ideal());
    }
    // a part with fewer than d usable chunks: its report carries the reconstruct error
    // (ResilverPartReport::write_error) and the other parts are still resilvered, batched and
    // per part alike
    for (size_t i = 1; i < d + p; ++i) store.erase(f.parts[4].chunk(i).locations[0]);
    for (const size_t ppb : {size_t(4), size_t(0)}) {
        store.erase(f.parts[7].data[1].locations[0]);  // a repairable hole in another part
        const auto rep = f.resilver(store, ppb, 2);
        CHECK(rep.size() == f.parts.size());
        CHECK(rep[4].write_error && *rep[4].write_error == Error::TooFewShardsPresent);
        CHECK(rep[4].count(LocationIntegrity::Resilvered) == 0 && !rep[4].is_ideal());
        CHECK(!rep[7].write_error && rep[7].chunks[1] == LocationIntegrity::Resilvered);
        for (size_t k = 0; k < f.parts.size(); ++k)
            if (k != 4) CHECK(!rep[k].write_error && rep[k].is_ideal());
    }
}

// A store a resilver has touched lists chunks as [bad copy, good copy] (resilver appends the
// rebuilt copy's location, file_part.rs:346).  p + 1 chunks of every part get a stale copy listed
// first, so fewer than d first copies verify: the read succeeds only by walking each chunk's
// locations before drawing another chunk (file_part.rs:100-107), per part and batched over one
// and two shards; verify flags exactly the stale locations (file_part.rs:236-243); resilver
// rebuilds nothing (every chunk has a valid copy) -- until a chunk's every copy is bad, when it
// is rebuilt and its location appended.
void test_locations_bad_then_good() {
    for (const auto& shape : std::vector<std::array<size_t, 3>>{{3, 2, 4096}, {10, 4, 2048}}) {
        const size_t d = shape[0], p = shape[1], chunk = shape[2], t = d + p;
        const Bytes input = random_bytes(d * chunk * 13 + 211, d * 7 + 1);
        ChunkStore store;
        FileReference f =
            FileWriteBuilder().chunk_size(chunk).data_chunks(d).parity_chunks(p).write(input, store);
        size_t stale = 0;
        for (size_t k = 0; k < f.parts.size(); ++k)
            for (size_t m = 0; m <= p; ++m) {
                Chunk& c = f.parts[k].chunk_mut((k + 2 * m) % t);
                Bytes bad = *store.read(c.locations[0]);
                bad[bad.size() / 2] ^= 0x10;
                const Location loc = "stale/" + ChunkStore::location_of(c.hash);
                store.put(loc, bad);
                c.locations.insert(c.locations.begin(), loc);
                ++stale;
            }
        CHECK(f.read(store) == input);
        for (const auto& devs : std::vector<std::vector<int>>{{}, {0, 0}}) {
            CHECK(f.read(store, 3, 2, devs) == input);
            for (const auto& reps : {f.verify(store), f.verify(store, 3, 2, devs)}) {
                size_t invalid = 0;
                for (size_t k = 0; k < reps.size(); ++k) {
                    CHECK(reps[k].is_ideal());  // every chunk has a valid copy
                    for (size_t i = 0; i < t; ++i) {
                        const auto& locs = reps[k].locations[i];
                        const bool has_stale = f.parts[k].chunk(i).locations.size() == 2;
                        CHECK(locs.size() == (has_stale ? 2u : 1u));
                        CHECK(locs.back() == LocationIntegrity::Valid);
                        if (has_stale) CHECK(locs[0] == LocationIntegrity::Invalid);
                    }
                    invalid += reps[k].invalid_locations();
                }
                CHECK(invalid == stale);
            }
        }
        // resilver: nothing to rebuild (per part and batched)
        for (const size_t ppb : {size_t(0), size_t(3)})
            for (const auto& r : f.resilver(store, ppb, 2)) CHECK(r.new_locations.empty() && r.is_ideal());
        // part 4: a chunk whose copies are both bad is rebuilt, its location appended
        Chunk& victim = f.parts[4].chunk_mut(4 % t);
        CHECK(victim.locations.size() == 2);
        CHECK(store.corrupt(victim.locations[1], 3));
        const auto rep = f.resilver(store, 3, 2);
        CHECK(rep[4].new_locations.size() == 1 && victim.locations.size() == 3);
        CHECK(rep[4].chunks[4 % t] == LocationIntegrity::Resilvered);
        CHECK(victim.locations[2] == ChunkStore::location_of(victim.hash));
        for (const auto& r : f.verify(store, 3, 2)) CHECK(r.is_ideal());
        CHECK(f.read(store, 3, 2) == input);
    }
}

// A FileReference whose parts have different shapes (the metadata allows a d/p per part;
// file_part.rs:77 builds a codec per part): batched reads group only parts of one shape.
void test_mixed_shape_read() {
    const size_t chunk = 2048;
    const Bytes in1 = random_bytes(3 * chunk * 4, 11), in2 = random_bytes(5 * chunk * 3 + 17, 12);
    ChunkStore store;
    const FileReference f1 = FileWriteBuilder().chunk_size(chunk).data_chunks(3).parity_chunks(2).write(in1, store);
    const FileReference f2 = FileWriteBuilder().chunk_size(chunk).data_chunks(5).parity_chunks(3).write(in2, store);
    FileReference mixed;
    mixed.parts = f1.parts;
    mixed.parts.insert(mixed.parts.end(), f2.parts.begin(), f2.parts.end());
    // f2's last part is short (chunksize < chunk): its bytes are that part's d*chunksize
    Bytes expect = in1;
    for (const auto& part : f2.parts) {
        const Bytes b = part.read_with_context(store);
        expect.insert(expect.end(), b.begin(), b.end());
    }
    mixed.length = expect.size();
    CHECK(mixed.read(store, 2, 2) == expect);
    CHECK(mixed.read(store) == expect);
}

// JavaReedSolomon testOneEncode / reed-solomon-erasure test_encoding (RS(5,5)).
void test_one_encode() {
    const ReedSolomon rs(5, 5);
    const std::vector<Bytes> data = {{0, 1}, {4, 5}, {2, 3}, {6, 7}, {8, 9}};
    std::vector<Bytes> parity(5, Bytes(2, 0xEE));
    rs.encode_sep(data, parity);
    const std::vector<Bytes> want = {{12, 13}, {10, 11}, {14, 15}, {90, 91}, {94, 95}};
    CHECK(parity == want);
}

// M = V * inv(V[0..d]) over GF(2^8)/0x11D, parity rows.
void test_matrix_rows() {
    const auto m32 = ReedSolomon(3, 2).matrix();
    CHECK((m32[3] == Bytes{1, 1, 1}));
    CHECK((m32[4] == Bytes{15, 8, 6}));
    const auto m = ReedSolomon(10, 4).matrix();
    CHECK((m[10] == Bytes{129, 150, 175, 184, 210, 196, 254, 232, 3, 2}));
    CHECK((m[11] == Bytes{150, 129, 184, 175, 196, 210, 232, 254, 2, 3}));
    CHECK((m[12] == Bytes{191, 214, 98, 10, 6, 111, 223, 183, 5, 4}));
    CHECK((m[13] == Bytes{214, 191, 10, 98, 111, 6, 183, 223, 4, 5}));
    for (size_t r = 0; r < 10; ++r)
        for (size_t c = 0; c < 10; ++c) CHECK(m[r][c] == (r == c ? 1 : 0));
}

void test_errors() {
    CHECK(throws_erasure([] { ReedSolomon(0, 1); }, Error::TooFewDataShards));
    CHECK(throws_erasure([] { ReedSolomon(1, 0); }, Error::TooFewParityShards));
    CHECK(throws_erasure([] { ReedSolomon(200, 57); }, Error::TooManyShards));
    const ReedSolomon rs(3, 2);
    CHECK(throws_erasure(
        [&] {
            std::vector<Bytes> parity(2, Bytes(4));
            rs.encode_sep(std::vector<Bytes>(2, Bytes(4)), parity);
        },
        Error::TooFewDataShards));
    CHECK(throws_erasure(
        [&] {
            std::vector<Bytes> parity(2, Bytes(4));
            rs.encode_sep(std::vector<Bytes>{Bytes(4), Bytes(4), Bytes(5)}, parity);
        },
        Error::IncorrectShardSize));
    CHECK(throws_erasure(
        [&] {
            std::vector<Bytes> parity(2, Bytes(0));
            rs.encode_sep(std::vector<Bytes>(3, Bytes(0)), parity);
        },
        Error::EmptyShard));
    CHECK(throws_erasure(
        [&] {
            Shards s = {Bytes(8, 1), std::nullopt, std::nullopt, std::nullopt, Bytes(8, 2)};
            rs.reconstruct(s);
        },
        Error::TooFewShardsPresent));
    // FilePart::read_with_context with fewer than d verifiable chunks
    ChunkStore store;
    const FileReference f = FileWriteBuilder().chunk_size(1024).data_chunks(3).parity_chunks(2).write(
        Bytes(3000, 7), store);
    for (size_t i = 0; i < 3; ++i) store.erase(f.parts[0].chunk(i).locations[0]);
    CHECK(throws_erasure([&] { f.read(store); }, Error::TooFewShardsPresent));
}

void test_reconstruct_every_pattern() {
    const size_t d = 4, p = 3, t = d + p, L = 1000 + 3;
    const ReedSolomon rs(d, p);
    std::vector<Bytes> data(d, Bytes(L));
    for (size_t j = 0; j < d; ++j)
        for (size_t x = 0; x < L; ++x) data[j][x] = uint8_t(x * 31 + j * 7 + (x >> 5));
    std::vector<Bytes> parity(p, Bytes(L));
    rs.encode_sep(data, parity);
    std::vector<Bytes> full = data;
    full.insert(full.end(), parity.begin(), parity.end());
    for (uint32_t mask = 1; mask < (1u << t); ++mask) {
        if (size_t(__builtin_popcount(mask)) > p) continue;
        for (int data_only = 0; data_only < 2; ++data_only) {
            Shards s(t);
            for (size_t i = 0; i < t; ++i)
                if (!(mask >> i & 1)) s[i] = full[i];
            if (data_only) rs.reconstruct_data(s);
            else rs.reconstruct(s);
            for (size_t i = 0; i < t; ++i) {
                if (data_only && i >= d && (mask >> i & 1)) {
                    CHECK(!s[i]);  // reconstruct_data leaves missing parity None
                } else {
                    CHECK(s[i] && *s[i] == full[i]);
                }
            }
        }
    }
}

struct Test {
    const char* name;
    void (*fn)();
};

const Test kTests[] = {
    {"sha256", sha256},
    {"test_file_write", test_file_write},
    {"test_resilver", test_resilver},
    {"test_cluster_digests", test_cluster_digests},
    {"test_cp_50mib", test_cp_50mib},
    {"test_range_reads", test_range_reads},
    {"test_write_concurrency", test_write_concurrency},
    {"test_batched_paths", test_batched_paths},
    {"test_multi_device_paths", test_multi_device_paths},
    {"test_mixed_shape_read", test_mixed_shape_read},
    {"test_batched_verify_resilver", test_batched_verify_resilver},
    {"test_locations_bad_then_good", test_locations_bad_then_good},
    {"test_one_encode", test_one_encode},
    {"test_matrix_rows", test_matrix_rows},
    {"test_errors", test_errors},
    {"test_reconstruct_every_pattern", test_reconstruct_every_pattern},
};

}  // namespace

int main(int argc, char** argv) {
    if (argc > 1 && std::strcmp(argv[1], "--list") == 0) {
        for (const Test& t : kTests) std::printf("%s\n", t.name);
        return 0;
    }
    int failed_tests = 0;
    for (const Test& t : kTests) {
        if (argc > 1 && std::strcmp(argv[1], t.name) != 0) continue;
        const int before = g_failures;
        try {
            t.fn();
        } catch (const std::exception& e) {
            std::fprintf(stderr, "  exception: %s\n", e.what());
            ++g_failures;
        }
        const bool ok = g_failures == before;
        failed_tests += ok ? 0 : 1;
        std::printf("%s ... %s\n", t.name, ok ? "ok" : "FAILED");
        std::fflush(stdout);
    }
    std::printf("%s\n", failed_tests ? "FAILED" : "all passed");
    return failed_tests ? 1 : 0;
}
