// End-to-end `cp` through the C++ host layer (dev tool): FileWriteBuilder::write of an in-memory
// file into a ChunkStore (RAM stand-in for the locations), then FileReference::read back after
// losing one data + one parity chunk per part — per-part calls (the reference's shape) vs the
// batched paths (FileWriteBuilder::batch / read(src, parts_per_batch) through the multi-GPU
// scheduler, sharded over `devices`: default the current GPU; e.g. 0,0 = two shards on GPU 0).
// Batched only, last: the read with `damage` (default 1 %) of the stored chunk copies flipped,
// so parts retry (file_part.rs:92-107), with the retries' verified chunks kept on the GPU
// (carry) and sent again (no carry): time and chunks sent to the GPUs.
//   make -C chunky-bits_amd/csrc cp_bench ; tools/cp_bench [GiB] [devices] [damage] [depth]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <string>

#include "chunky_ec.hpp"

using namespace chunky_ec;

int main(int argc, char** argv) {
    const double gib = argc > 1 ? std::atof(argv[1]) : 4.0;
    const double damage = argc > 3 ? std::atof(argv[3]) : 0.01;
    const size_t depth = argc > 4 ? size_t(std::atoi(argv[4])) : 4;  // scheduler depth (read windows: depth + 1)
    std::vector<int> devices;
    if (argc > 2) {
        std::stringstream ss(argv[2]);
        std::string tok;
        while (std::getline(ss, tok, ',')) devices.push_back(std::atoi(tok.c_str()));
    }
    const size_t d = 10, p = 4, chunk = size_t(1) << 20;
    const size_t length = size_t(gib * double(size_t(1) << 30)) / (d * chunk) * (d * chunk) + 4321;
    Bytes input(length);
    uint64_t z = 7;
    for (size_t i = 0; i + 8 <= length; i += 8) {
        z += 0x9E3779B97F4A7C15ull;
        uint64_t v = z;
        v = (v ^ (v >> 30)) * 0xBF58476D1CE4E5B9ull;
        v = (v ^ (v >> 27)) * 0x94D049BB133111EBull;
        v ^= v >> 31;
        std::memcpy(&input[i], &v, 8);
    }
    auto secs = [](auto t0) {
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    // where the batched read loop's time went since the last call (detail::read_times)
    auto times = [] {
        detail::ReadTimes& t = detail::read_times();
        char buf[384];
        std::snprintf(buf, sizeof buf,
                      "[%llu windows: load %.3f s, wait job %.3f s (job latency %.1f ms), %llu retry "
                      "rounds (%llu after a first, %llu parts, latency %.1f ms): build %.3f s, wait "
                      "%.3f s; sink %.3f s]",
                      static_cast<unsigned long long>(t.windows), t.load, t.wait_job,
                      t.windows ? t.job_latency / double(t.windows) * 1e3 : 0.0,
                      static_cast<unsigned long long>(t.retry_rounds),
                      static_cast<unsigned long long>(t.later_rounds),
                      static_cast<unsigned long long>(t.retry_parts),
                      t.retry_rounds ? t.round_latency / double(t.retry_rounds) * 1e3 : 0.0,
                      t.retry_build,
                      t.wait_retry, t.emit);
        t = detail::ReadTimes{};
        return std::string(buf);
    };
    const auto builder = FileWriteBuilder().chunk_size(chunk).data_chunks(d).parity_chunks(p);
    for (int batched = 1; batched >= 0; --batched) {
        const size_t n = batched ? length : std::min(length, size_t(64) * d * chunk);
        auto write = [&](ChunkStore& store) {
            return batched ? FileWriteBuilder(builder).batch(128, depth).devices(devices).write(
                                 input.data(), n, store)
                           : builder.write(input.data(), n, store);
        };
        // write path alone (shards discarded, as if written to /dev/null); the first write
        // of a shape pins the pipeline's host buffers (made once per thread and shape)
        ChunkStore sink = ChunkStore::discard();
        write(sink);
        auto t0 = std::chrono::steady_clock::now();
        write(sink);
        const double w = secs(t0);
        // write into RAM, lose one data + one parity chunk per part, read back
        ChunkStore store;
        t0 = std::chrono::steady_clock::now();
        FileReference f = write(store);
        const double w_ram = secs(t0);
        if (batched) {  // pins the verify / resilver windows (nothing to rebuild yet)
            (void)f.resilver(store, 128, depth, devices);
            (void)f.verify(store, 128, depth, devices);
        }
        for (const auto& part : f.parts) {
            store.erase(part.data[3].locations[0]);
            store.erase(part.parity[1].locations[0]);
        }
        if (batched) (void)f.read(store, 128, depth, devices);  // pins the read windows
        t0 = std::chrono::steady_clock::now();
        const Bytes back = batched ? f.read(store, 128, depth, devices) : f.read(store);
        const double r = secs(t0);
        bool ok = back.size() == n && std::memcmp(back.data(), input.data(), n) == 0;
        // the same read streamed to a sink (FileReadBuilder's reader, reader.rs:40-75) that
        // discards the bytes, as if written to /dev/null (read() above checked them)
        size_t at = 0;
        (void)times();
        t0 = std::chrono::steady_clock::now();
        if (batched)
            f.read_to(store, [&](const uint8_t*, size_t m) { at += m; }, 128, depth, devices);
        else
            f.read_to(store, [&](const uint8_t*, size_t m) { at += m; });
        const double r_sink = secs(t0);
        const std::string r_times = times();
        ok = ok && at == n;
        // resilver (rebuild the two lost chunks of every part and write them back), then verify
        // (every stored chunk hashed)
        t0 = std::chrono::steady_clock::now();
        const auto rep = batched ? f.resilver(store, 128, depth, devices) : f.resilver(store);
        const double rs = secs(t0);
        // the two repaired chunks of every part now list two locations (the lost one and the new
        // copy, file_part.rs:346; both "sha256-<hex>" here, so both read): 16 copies per part to
        // hash, more than the 14-chunk windows hold, so the first such verify of a thread grows
        // its page-locked windows -- once, like the first call's pinning above
        if (batched) (void)f.verify(store, 128, depth, devices);
        t0 = std::chrono::steady_clock::now();
        const auto ver = batched ? f.verify(store, 128, depth, devices) : f.verify(store);
        const double vs = secs(t0);
        for (const auto& r : ver) ok = ok && r.is_ideal();
        for (const auto& r : rep)
            ok = ok && r.chunks[3] == LocationIntegrity::Resilvered &&
                 r.chunks[d + 1] == LocationIntegrity::Resilvered;
        std::printf("%-9s %6.2f GiB, %zu parts, %zu shard(s): write %6.2f GB/s (%6.2f GB/s into "
                    "the RAM store), read with 2 holes/part %6.2f GB/s (%6.2f GB/s streamed to a "
                    "sink), resilver %6.2f GB/s, verify %6.2f GB/s, bit-exact %s\n",
                    batched ? "batched" : "per-part", double(n) / double(size_t(1) << 30),
                    f.parts.size(), batched ? std::max<size_t>(devices.size(), 1) : size_t(0),
                    double(n) / w / 1e9, double(n) / w_ram / 1e9,
                    double(n) / r / 1e9, double(n) / r_sink / 1e9, double(n) / rs / 1e9,
                    double(n) / vs / 1e9, ok ? "yes" : "NO");
        if (batched) std::printf("          read to a sink: %s\n", r_times.c_str());
        std::fflush(stdout);
        if (!ok) return 1;
        if (!batched) continue;
        // the damaged read: a seeded `damage` fraction of the data chunks' copies flipped (a
        // reader loads the data chunks first, so each flip makes its part retry)
        uint64_t x = 99;
        size_t flipped = 0;
        for (const auto& part : f.parts)
            for (size_t j = 0; j < d; ++j) {
                x = x * 6364136223846793005ull + 1442695040888963407ull;
                if (double(x >> 11) / double(1ull << 53) < damage)
                    flipped += store.corrupt(part.data[j].locations[0], (x >> 7) % chunk) ? 1 : 0;
            }
        cec_multi* m = detail::cached_multi_entry().multi.get();
        auto uploaded = [&] {
            uint64_t u = 0;
            for (size_t g = 0; g < cec_multi_shards(m); ++g) {
                cec_multi_stats st{};
                if (cec_multi_shard_stats(m, g, &st) == CEC_OK) u += st.chunks_uploaded;
            }
            return u;
        };
        for (int carry = 1; carry >= 0; --carry) {  // checked (and warms the windows)
            detail::read_carry() = carry != 0;
            const Bytes dmg = f.read(store, 128, depth, devices);
            ok = ok && dmg.size() == n && std::memcmp(dmg.data(), input.data(), n) == 0;
        }
        // timed: streamed to a sink that discards the bytes, as read_to above; the two modes
        // alternate, 3 runs each, best of each kept (one run is ~1 s: box noise is ±15 %)
        double best[2] = {0, 0};
        uint64_t sent[2] = {0, 0};
        std::string best_times[2];
        for (int rep = 0; rep < 3; ++rep)
            for (int carry = 1; carry >= 0; --carry) {
                detail::read_carry() = carry != 0;
                const uint64_t u0 = uploaded();
                size_t got = 0;
                (void)times();
                t0 = std::chrono::steady_clock::now();
                f.read_to(store, [&](const uint8_t*, size_t m) { got += m; }, 128, depth, devices);
                const double rate = double(n) / secs(t0) / 1e9;
                if (rate > best[carry]) best_times[carry] = times();
                best[carry] = std::max(best[carry], rate);
                sent[carry] = uploaded() - u0;
                ok = ok && got == n;
            }
        for (int carry = 1; carry >= 0; --carry)
            std::printf("batched   read with %.2f %% of data copies damaged (%zu flipped) + the "
                        "lost chunks, %s: %6.2f GB/s streamed to a sink (best of 3), %llu chunks "
                        "sent to the GPU, bit-exact %s\n",
                        damage * 100, flipped, carry ? "carry   " : "no carry", best[carry],
                        static_cast<unsigned long long>(sent[carry]), ok ? "yes" : "NO");
        for (int carry = 1; carry >= 0; --carry)
            std::printf("          %s: %s\n", carry ? "carry   " : "no carry", best_times[carry].c_str());
        std::fflush(stdout);
        if (!ok) return 1;
        detail::read_carry() = true;
    }
    return 0;
}
