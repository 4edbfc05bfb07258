// Per-call tier throughput (dev tool): the drop-in host-buffer calls made the way the reference
// makes them — one part per call from ordinary (pageable) Vec<u8>-like buffers, up to 10 part
// tasks in flight (writer.rs:130 concurrency) — through the C++ host layer.
//   encode_sep   ReedSolomon::encode_sep of RS(10,4), 1 MiB chunks (file_part.rs:161-165)
//   part_encode  FilePart::write_with_encoder's compute: encode + SHA-256 of the 14 chunks
// Build: make -C chunky-bits_amd/csrc percall   (-> tools/percall_bench)
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

#include "chunky_ec.hpp"

using namespace chunky_ec;

namespace {

double run(int threads, int calls_per_thread, bool hashed, const ReedSolomon& rs) {
    const size_t d = 10, p = 4, L = size_t(1) << 20;
    std::vector<std::thread> pool;
    auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < threads; ++t) {
        pool.emplace_back([&, t] {
            std::vector<Bytes> data(d, Bytes(L, uint8_t(t)));
            std::vector<Bytes> parity(p, Bytes(L));
            Bytes data_buf(d * L, uint8_t(t));
            ChunkStore sink;
            for (int i = 0; i < calls_per_thread; ++i) {
                if (hashed) {
                    ChunkStore store;
                    FilePart::write_with_encoder(rs, store, data_buf, d * L);
                } else {
                    rs.encode_sep(data, parity);
                }
            }
        });
    }
    for (auto& th : pool) th.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return double(threads) * calls_per_thread * d * L / s / 1e9;
}

}  // namespace

int main() {
    const ReedSolomon rs(10, 4);
    run(1, 2, false, rs);  // warm up: device contexts, staging buffers
    run(1, 1, true, rs);
    for (int threads : {1, 10}) {
        std::printf("encode_sep  RS(10,4) 1 MiB, %2d thread(s): %6.2f GB/s of data\n", threads,
                    run(threads, 20, false, rs));
        std::fflush(stdout);
    }
    for (int threads : {1, 10, 100, 400}) {
        run(threads, 1, true, rs);  // warm: pinned staging grown to this batch size
        uint64_t c0, l0, c1, l1;
        cec_coalesce_stats(&c0, &l0);
        const double gbs = run(threads, 3, true, rs);
        cec_coalesce_stats(&c1, &l1);
        std::printf("part_encode RS(10,4) 1 MiB, %3d thread(s): %6.2f GB/s of data "
                    "(%llu calls in %llu launches)\n",
                    threads, gbs, (unsigned long long)(c1 - c0), (unsigned long long)(l1 - l0));
        std::fflush(stdout);
    }
    return 0;
}
