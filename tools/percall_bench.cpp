// Per-call tier throughput (dev tool): the drop-in host-buffer calls made the way the reference
// makes them — one part per call, many part tasks in flight (writer.rs:130 `concurrency`).
//   encode_sep   ReedSolomon::encode_sep of RS(10,4), 1 MiB chunks (file_part.rs:161-165)
//   part_encode  FilePart::write_with_encoder's compute: encode + SHA-256 of the 14 chunks
//                (cec_part_encode), from ordinary pageable buffers (the reference's
//                vec![0; d*chunk_size], writer.rs:172) or from page-locked cec_host_alloc
//                buffers, which the engine DMAs directly (no staging copies).
//   literal      the swap made literally at each call site ("literal"):
//                encode_sep (file_part.rs:161-165), then Sha256Hash::from_buf of each of the 14
//                chunks one after the other, as the reference's FuturesOrdered polls them inside
//                one part task (file_part.rs:177-197) -- beside part_encode at the same counts
// Build: make -C chunky-bits_amd/csrc percall   (-> tools/percall_bench)
// Usage: tools/percall_bench [threads...]   (default 1 10 100 256 400)
//        tools/percall_bench --literal [threads...]   (default 10 64)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "chunky_ec.hpp"

using namespace chunky_ec;

namespace {

constexpr size_t kD = 10, kP = 4, kL = size_t(1) << 20;

// One part's caller buffers: pageable vectors or page-locked host memory.
struct PartBufs {
    bool pinned = false;
    uint8_t* data = nullptr;
    uint8_t* parity = nullptr;
    std::vector<uint8_t> vdata, vparity;
    explicit PartBufs(bool pin, uint8_t fill) : pinned(pin) {
        if (pin) {
            void *a = nullptr, *b = nullptr;
            if (cec_host_alloc(kD * kL, -1, &a) != CEC_OK || cec_host_alloc(kP * kL, -1, &b) != CEC_OK) {
                std::fprintf(stderr, "cec_host_alloc failed\n");
                std::exit(1);
            }
            data = static_cast<uint8_t*>(a);
            parity = static_cast<uint8_t*>(b);
            std::memset(data, fill, kD * kL);
        } else {
            vdata.assign(kD * kL, fill);
            vparity.assign(kP * kL, 0);
            data = vdata.data();
            parity = vparity.data();
        }
    }
    ~PartBufs() {
        if (pinned) {
            cec_host_free(data);
            cec_host_free(parity);
        }
    }
};

double run_encode(int threads, int calls, const ReedSolomon& rs) {
    std::vector<std::thread> pool;
    auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < threads; ++t)
        pool.emplace_back([&, t] {
            std::vector<Bytes> data(kD, Bytes(kL, uint8_t(t)));
            std::vector<Bytes> parity(kP, Bytes(kL));
            for (int i = 0; i < calls; ++i) rs.encode_sep(data, parity);
        });
    for (auto& th : pool) th.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return double(threads) * calls * kD * kL / s / 1e9;
}

double run_part(int threads, int calls, bool pinned, const ReedSolomon& rs) {
    std::vector<std::unique_ptr<PartBufs>> bufs;
    for (int t = 0; t < threads; ++t) bufs.push_back(std::make_unique<PartBufs>(pinned, uint8_t(t)));
    std::vector<std::thread> pool;
    auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < threads; ++t)
        pool.emplace_back([&, t] {
            uint8_t digests[32 * (kD + kP)];
            size_t cs = 0;
            for (int i = 0; i < calls; ++i)
                if (cec_part_encode(rs.raw(), bufs[t]->data, kD * kL, bufs[t]->parity, digests,
                                    &cs) != CEC_OK) {
                    std::fprintf(stderr, "cec_part_encode: %s\n", cec_last_error());
                    std::exit(1);
                }
        });
    for (auto& th : pool) th.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return double(threads) * calls * kD * kL / s / 1e9;
}

// The literal per-call wiring: per part, encode_sep, then the d + p digests one call at a time.
double run_literal(int threads, int calls, const ReedSolomon& rs) {
    std::vector<std::thread> pool;
    auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < threads; ++t)
        pool.emplace_back([&, t] {
            std::vector<Bytes> data(kD, Bytes(kL, uint8_t(t)));
            std::vector<Bytes> parity(kP, Bytes(kL));
            for (int i = 0; i < calls; ++i) {
                rs.encode_sep(data, parity);
                for (const Bytes& c : data) (void)Sha256Hash::from_buf(c);
                for (const Bytes& c : parity) (void)Sha256Hash::from_buf(c);
            }
        });
    for (auto& th : pool) th.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return double(threads) * calls * kD * kL / s / 1e9;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "--literal") {
        std::vector<int> counts;
        for (int i = 2; i < argc; ++i) counts.push_back(std::atoi(argv[i]));
        if (counts.empty()) counts = {10, 64};
        const ReedSolomon rs(kD, kP);
        run_literal(2, 1, rs);  // warm up
        for (int threads : counts) {
            run_literal(threads, 1, rs);
            uint64_t c0, l0, c1, l1;
            cec_coalesce_stats(&c0, &l0);
            const double lit = run_literal(threads, 2, rs);
            cec_coalesce_stats(&c1, &l1);
            std::printf("literal     RS(10,4) 1 MiB, pageable, %3d part task(s): %6.2f GB/s of data "
                        "(encode_sep + 14 serial sha256 per part; %llu hashing calls in %llu "
                        "launches)\n", threads, lit, (unsigned long long)(c1 - c0),
                        (unsigned long long)(l1 - l0));
            run_part(threads, 1, false, rs);
            const double part = run_part(threads, 3, false, rs);
            std::printf("part_encode RS(10,4) 1 MiB, pageable, %3d part task(s): %6.2f GB/s of data\n",
                        threads, part);
            std::fflush(stdout);
        }
        return 0;
    }
    std::vector<int> counts;
    for (int i = 1; i < argc; ++i) counts.push_back(std::atoi(argv[i]));
    if (counts.empty()) counts = {1, 10, 100, 256, 400};
    const ReedSolomon rs(kD, kP);
    run_encode(1, 2, rs);  // warm up: device contexts, staging buffers
    for (int threads : {1, 10}) {
        std::printf("encode_sep  RS(10,4) 1 MiB, %3d thread(s): %6.2f GB/s of data\n", threads,
                    run_encode(threads, 20, rs));
        std::fflush(stdout);
    }
    for (bool pinned : {false, true}) {
        for (int threads : counts) {
            run_part(threads, 1, pinned, rs);  // warm: staging grown to this batch size
            uint64_t c0, l0, c1, l1;
            cec_coalesce_stats(&c0, &l0);
            const double gbs = run_part(threads, 3, pinned, rs);
            cec_coalesce_stats(&c1, &l1);
            std::printf("part_encode RS(10,4) 1 MiB, %-8s %3d thread(s): %6.2f GB/s of data "
                        "(%llu calls in %llu launches)\n",
                        pinned ? "pinned," : "pageable,", threads, gbs,
                        (unsigned long long)(c1 - c0), (unsigned long long)(l1 - l0));
            std::fflush(stdout);
        }
    }
    return 0;
}
