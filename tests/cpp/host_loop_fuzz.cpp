// host_loop_fuzz.cpp — the C++ host layer's batched loops (include/chunky_ec.hpp: the write's
// write_full_parts, the read's read_run / retry_start / retry_round / retry_collect, verify and
// resilver's check_run) on the CPU, with the scheduler replaced by a stand-in that keeps the
// C-ABI's job contract and computes with the oracle (test infrastructure: this binary is built and
// run only by tests/test_cpp_loop_fuzz.py).
//
// The stand-in (cec_multi_* below) computes a job only when it completes: after a seeded number
// of cec_multi_query calls, or at cec_multi_wait.  So jobs finish out of order, and a loop that
// touched a job's buffers before the job was done, or read its results early, gets wrong bytes.
// Carry ids follow the ABI (include/chunky_ec.h: kept for one part, used once, refused for
// another part's digests).
//
// Each seed: (1) writes a file through the batched and the per-part write paths (same parts,
// digests, locations and stored bytes); (2) builds a store of random location mixes (good;
// [bad, good]; [gone, short, good]; [bad, bad]; bad; gone -- file_part.rs:92-107's location
// walk) and reads it with a random window size, depth, shard list and carry switch: the bytes out
// are the file's, in order, up to the first part with fewer than d good chunks, which fails the
// read with TooFewShardsPresent, and afterwards no job is left unwaited and no carry id held;
// (3) runs verify and resilver batched and per part on copies of the file and store: same
// reports, same write-backs, and the resilvered file reads back whole.  Some seeds first read
// with a sink that fails part way: nothing may be left behind.  No job may break the
// contract.  Usage: host_loop_fuzz FIRST_SEED N_SEEDS; exit status 0 iff every seed passed.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "chunky_ec.hpp"

extern "C" {
// oracle/cec_oracle.c
void or_sha256(const uint8_t* buf, size_t len, uint8_t out[32]);
int or_rs_encode_sep(size_t d, size_t p, const uint8_t* const* data, const size_t* data_lens,
                     size_t n_data, uint8_t* const* parity, const size_t* parity_lens,
                     size_t n_parity);
int or_rs_reconstruct(size_t d, size_t p, uint8_t* const* shards, const size_t* lens,
                      uint8_t* present, size_t n_shards, int data_only);
}

namespace {

std::mt19937_64 g_poll_rng;  // how many queries a job takes to report done
int g_violations = 0;        // contract breaches seen by the stand-in

void violation(const char* what) {
    std::fprintf(stderr, "  contract: %s\n", what);
    ++g_violations;
}

}  // namespace

// Parity and the d+p digests of one part whose d data chunks are data[0 .. d*L).
void encode_part(size_t d, size_t p, size_t L, const uint8_t* data, uint8_t* parity,
                 uint8_t* digests) {
    std::vector<const uint8_t*> dp(d);
    std::vector<uint8_t*> pp(p);
    std::vector<size_t> dl(d, L), pl(p, L);
    for (size_t i = 0; i < d; ++i) dp[i] = data + i * L;
    for (size_t i = 0; i < p; ++i) pp[i] = parity + i * L;
    if (or_rs_encode_sep(d, p, dp.data(), dl.data(), d, pp.data(), pl.data(), p) != 0)
        violation("oracle encode failed");
    for (size_t i = 0; i < d + p; ++i) or_sha256(i < d ? dp[i] : pp[i - d], L, digests + 32 * i);
}

struct cec_codec {
    size_t d, p;
};

struct cec_multi {
    size_t d, p, L, shards;
    struct Job {
        const uint8_t *chunks, *present, *expected;
        size_t n;
        uint8_t *data, *verified;
        int* status;
        const uint8_t** ptrs;
        unsigned flags;
        const int32_t* carry_in;
        int32_t* carry_out;
        int polls_left;
        bool done = false;
        int result = CEC_OK;
        enum { READ, VERIFY, RESILVER, WRITE } kind = READ;
    };
    struct Entry {
        std::vector<uint8_t> mask, expected, bytes;  // [t], [t][32], [t][L]
    };
    std::map<uint64_t, Job> jobs;  // submitted, not yet waited for
    std::map<int32_t, Entry> pool;
    uint64_t next_job = 1;
    int32_t next_carry = 0;
    uint64_t uploaded = 0, carried = 0;

    // The job's compute, run at completion (file_part.rs:86-122 per part: verify the loaded
    // chunks, decode from d verified ones, or TooFewShardsPresent with the verified ones kept).
    void run(Job& j) {
        const size_t t = d + p;
        if (j.kind == Job::WRITE) {  // write_with_encoder's compute: parity + every digest
            for (size_t k = 0; k < j.n; ++k)
                encode_part(d, p, L, j.chunks + k * d * L, j.data + k * p * L,
                            j.verified + k * t * 32);
            return;
        }
        if (j.kind == Job::VERIFY) {  // every loaded row hashed, nothing decoded
            for (size_t x = 0; x < j.n * t; ++x) {
                uint8_t h[32];
                if (j.present[x]) or_sha256(j.chunks + x * L, L, h);
                j.verified[x] = j.present[x] && std::memcmp(h, j.expected + x * 32, 32) == 0;
            }
            return;
        }
        if (j.kind == Job::RESILVER) {  // file_part.rs:253-308: every chunk without a valid copy
            for (size_t k = 0; k < j.n; ++k) {
                std::vector<uint8_t> buf(t * L), present(t);
                std::vector<uint8_t*> ptr(t);
                std::vector<size_t> lens(t, L);
                size_t good = 0;
                for (size_t i = 0; i < t; ++i) {
                    const size_t x = k * t + i;
                    ptr[i] = &buf[i * L];
                    uint8_t h[32];
                    if (j.present[x] && j.present[x] != CEC_PRESENT_VERIFIED)
                        or_sha256(j.chunks + x * L, L, h);
                    j.verified[x] = j.present[x] == CEC_PRESENT_VERIFIED ||
                                    (j.present[x] && std::memcmp(h, j.expected + x * 32, 32) == 0);
                    if (j.verified[x]) std::memcpy(ptr[i], j.chunks + x * L, L);
                    present[i] = j.verified[x];
                    good += present[i];
                }
                if (good < d) {
                    j.status[k] = CEC_TOO_FEW_SHARDS_PRESENT;
                    continue;
                }
                if (or_rs_reconstruct(d, p, ptr.data(), lens.data(), present.data(), t, 0) != 0) {
                    violation("oracle reconstruct failed");
                    j.result = CEC_ERR_INVALID_ARGUMENT;
                    return;
                }
                for (size_t i = 0; i < t; ++i)
                    if (!j.verified[k * t + i]) std::memcpy(j.data + (k * t + i) * L, ptr[i], L);
                j.status[k] = CEC_OK;
            }
            return;
        }
        for (size_t k = 0; k < j.n; ++k) {
            const uint8_t* pres = j.present + k * t;
            const uint8_t* exp = j.expected + k * t * 32;
            std::vector<std::vector<uint8_t>> ch(t);
            const int32_t cid = j.carry_in ? j.carry_in[k] : -1;
            const Entry* kept = nullptr;
            if (cid >= 0) {
                auto it = pool.find(cid);
                if (it == pool.end()) {
                    violation("carry id not held");
                    j.result = CEC_ERR_INVALID_ARGUMENT;
                    return;
                }
                kept = &it->second;
                if (std::memcmp(kept->expected.data(), exp, t * 32) != 0) {
                    violation("carry id of another part");
                    j.result = CEC_ERR_INVALID_ARGUMENT;
                    return;
                }
                for (size_t i = 0; i < t; ++i)
                    if (pres[i] == CEC_PRESENT_VERIFIED && !kept->mask[i]) {
                        violation("verified chunk not in the carry entry");
                        j.result = CEC_ERR_INVALID_ARGUMENT;
                        return;
                    }
            }
            uint8_t* ver = j.verified + k * t;
            size_t good = 0;
            bool redone = false;
            for (size_t i = 0; i < t; ++i) {
                ver[i] = 0;
                if (!pres[i]) continue;
                if (kept && pres[i] == CEC_PRESENT_VERIFIED) {
                    ch[i].assign(kept->bytes.begin() + i * L, kept->bytes.begin() + (i + 1) * L);
                    ++carried;
                } else {
                    ch[i].assign(j.chunks + (k * t + i) * L, j.chunks + (k * t + i + 1) * L);
                    ++uploaded;
                }
                if (pres[i] == CEC_PRESENT_VERIFIED) {
                    ver[i] = 1;
                } else {
                    uint8_t h[32];
                    or_sha256(ch[i].data(), L, h);
                    ver[i] = std::memcmp(h, exp + i * 32, 32) == 0;
                    redone = redone || !ver[i];
                }
                good += ver[i];
            }
            if (cid >= 0) pool.erase(cid);  // used once
            if (j.carry_out) j.carry_out[k] = -1;
            if (j.ptrs)
                for (size_t i = 0; i < d; ++i) j.ptrs[k * d + i] = nullptr;
            if (good < d) {
                j.status[k] = CEC_TOO_FEW_SHARDS_PRESENT;
                if (j.carry_out && good) {
                    Entry e;
                    e.mask.assign(ver, ver + t);
                    e.expected.assign(exp, exp + t * 32);
                    e.bytes.assign(t * L, 0);
                    for (size_t i = 0; i < t; ++i)
                        if (ver[i]) std::memcpy(&e.bytes[i * L], ch[i].data(), L);
                    pool[next_carry] = std::move(e);
                    j.carry_out[k] = next_carry++;
                }
                continue;
            }
            std::vector<uint8_t> present(t), buf(t * L);
            std::vector<uint8_t*> ptr(t);
            std::vector<size_t> lens(t, L);
            for (size_t i = 0; i < t; ++i) {
                ptr[i] = &buf[i * L];
                present[i] = ver[i];
                if (ver[i]) std::memcpy(ptr[i], ch[i].data(), L);
            }
            if (or_rs_reconstruct(d, p, ptr.data(), lens.data(), present.data(), t, 1) != 0) {
                violation("oracle reconstruct failed");
                j.result = CEC_ERR_INVALID_ARGUMENT;
                return;
            }
            const bool rebuilt_only = (j.flags & CEC_READ_REBUILT_ONLY) != 0;
            for (size_t i = 0; i < d; ++i) {
                // REBUILT_ONLY: a loaded data chunk stays where the caller's buffer holds it
                const bool in_place = rebuilt_only && !redone && pres[i] &&
                                      !(kept && pres[i] == CEC_PRESENT_VERIFIED);
                if (in_place) {
                    j.ptrs[k * d + i] = j.chunks + (k * t + i) * L;
                } else {
                    std::memcpy(j.data + (k * d + i) * L, ptr[i], L);
                    if (j.ptrs) j.ptrs[k * d + i] = j.data + (k * d + i) * L;
                }
            }
            j.status[k] = CEC_OK;
        }
    }
    void complete(Job& j) {
        if (!j.done) {
            j.done = true;
            run(j);
        }
    }
};

extern "C" {

const char* cec_status_name(int) { return "status"; }
const char* cec_last_error(void) { return ""; }
const char* cec_multi_last_error(void) { return "fake scheduler"; }
int cec_current_device(int* device) {
    *device = 0;
    return CEC_OK;
}

int cec_codec_new(size_t d, size_t p, cec_codec** out) {
    if (!d || !p || d + p > 256) return CEC_TOO_MANY_SHARDS;
    *out = new cec_codec{d, p};
    return CEC_OK;
}
void cec_codec_free(cec_codec* c) { delete c; }
size_t cec_codec_data_shards(const cec_codec* c) { return c->d; }
size_t cec_codec_parity_shards(const cec_codec* c) { return c->p; }
size_t cec_codec_total_shards(const cec_codec* c) { return c->d + c->p; }

// The per-part path's calls (a run of one part reads through read_with_context).
int cec_sha256_many(const uint8_t* const* bufs, const size_t* lens, size_t n, uint8_t* out) {
    for (size_t i = 0; i < n; ++i) or_sha256(bufs[i], lens[i], out + 32 * i);
    return CEC_OK;
}
static int reconstruct(const cec_codec* c, uint8_t* const* shards, const size_t* lens,
                       uint8_t* present, size_t n, int data_only) {
    return or_rs_reconstruct(c->d, c->p, shards, lens, present, n, data_only);
}
int cec_reconstruct(const cec_codec* c, uint8_t* const* shards, const size_t* lens,
                    uint8_t* present, size_t n) {
    return reconstruct(c, shards, lens, present, n, 0);
}
int cec_reconstruct_data(const cec_codec* c, uint8_t* const* shards, const size_t* lens,
                         uint8_t* present, size_t n) {
    return reconstruct(c, shards, lens, present, n, 1);
}

int cec_part_encode(const cec_codec* c, const uint8_t* data_buf, size_t length, uint8_t* parity,
                    uint8_t* digests, size_t* chunksize) {
    if (!length) return CEC_EMPTY_SHARD;
    const size_t L = (length + c->d - 1) / c->d;
    encode_part(c->d, c->p, L, data_buf, parity, digests);
    *chunksize = L;
    return CEC_OK;
}

int cec_host_alloc(size_t bytes, int, void** out) {
    *out = std::malloc(bytes ? bytes : 1);
    return *out ? CEC_OK : CEC_ERR_INVALID_ARGUMENT;
}
void cec_host_free(void* p) { std::free(p); }

int cec_multi_new(const cec_codec* codec, size_t chunk_len, size_t, size_t, const int*,
                  size_t n_devices, cec_multi** out) {
    *out = new cec_multi{codec->d, codec->p, chunk_len, n_devices};
    return CEC_OK;
}
void cec_multi_free(cec_multi* m) {
    if (!m->jobs.empty()) violation("scheduler freed with jobs not waited for");
    delete m;
}

int cec_multi_read_carry(cec_multi* m, const uint8_t* chunks, const uint8_t* present,
                         const uint8_t* expected, size_t n, uint8_t* data, uint8_t* verified,
                         int* status, const uint8_t** ptrs, unsigned flags,
                         const int32_t* carry_in, int32_t* carry_out, uint64_t* job) {
    if ((flags & CEC_READ_REBUILT_ONLY) && !ptrs) return CEC_ERR_INVALID_ARGUMENT;
    if ((flags & CEC_MULTI_AHEAD) != (carry_in ? CEC_MULTI_AHEAD : 0u))
        violation("retry rounds (and only they) go AHEAD");
    cec_multi::Job j{chunks, present, expected, n,     data,      verified, status,
                     ptrs,   flags,   carry_in, carry_out, int(g_poll_rng() % 6)};
    *job = m->next_job++;
    m->jobs.emplace(*job, j);
    return CEC_OK;
}
int cec_multi_encode_hash(cec_multi* m, const uint8_t* data, size_t n, uint8_t* parity,
                          uint8_t* digests, uint64_t* job) {
    cec_multi::Job j{data, nullptr, nullptr, n, parity, digests, nullptr, nullptr, 0u,
                     nullptr, nullptr, int(g_poll_rng() % 6)};
    j.kind = cec_multi::Job::WRITE;
    *job = m->next_job++;
    m->jobs.emplace(*job, j);
    return CEC_OK;
}
int cec_multi_verify(cec_multi* m, const uint8_t* chunks, const uint8_t* present,
                     const uint8_t* expected, size_t n, uint8_t* verified, uint64_t* job) {
    cec_multi::Job j{chunks, present, expected, n, nullptr, verified, nullptr, nullptr, 0u,
                     nullptr, nullptr, int(g_poll_rng() % 6)};
    j.kind = cec_multi::Job::VERIFY;
    *job = m->next_job++;
    m->jobs.emplace(*job, j);
    return CEC_OK;
}
int cec_multi_resilver(cec_multi* m, const uint8_t* chunks, const uint8_t* present,
                       const uint8_t* expected, size_t n, uint8_t* rebuilt, uint8_t* verified,
                       int* status, const uint8_t** chunk_ptrs, uint64_t* job) {
    if (chunk_ptrs) return CEC_ERR_INVALID_ARGUMENT;  // the loop passes none
    cec_multi::Job j{chunks, present, expected, n, rebuilt, verified, status, nullptr, 0u,
                     nullptr, nullptr, int(g_poll_rng() % 6)};
    j.kind = cec_multi::Job::RESILVER;
    *job = m->next_job++;
    m->jobs.emplace(*job, j);
    return CEC_OK;
}
int cec_multi_query(cec_multi* m, uint64_t job) {
    auto it = m->jobs.find(job);
    if (it == m->jobs.end()) return CEC_ERR_INVALID_ARGUMENT;
    if (it->second.polls_left-- > 0) return 0;
    m->complete(it->second);
    return 1;
}
int cec_multi_wait(cec_multi* m, uint64_t job) {
    auto it = m->jobs.find(job);
    if (it == m->jobs.end()) {
        violation("wait on a job not submitted or already waited for");
        return CEC_ERR_INVALID_ARGUMENT;
    }
    m->complete(it->second);
    const int r = it->second.result;
    m->jobs.erase(it);
    return r;
}
int cec_multi_carry_release(cec_multi* m, int32_t id) {
    if (!m->pool.erase(id)) {
        violation("release of an id not held");
        return CEC_ERR_INVALID_ARGUMENT;
    }
    return CEC_OK;
}

}  // extern "C"

namespace {

using namespace chunky_ec;

// One seed: a store, a read, the checks.  Returns true iff it passed.
bool run_seed(uint64_t seed) {
    std::mt19937_64 rng(seed);
    auto uni = [&](size_t lo, size_t hi) { return lo + size_t(rng() % (hi - lo + 1)); };
    const size_t d = uni(2, 5), p = uni(1, 3), t = d + p, L = 64 * uni(1, 8);
    const size_t n = uni(5, 40);
    g_poll_rng.seed(seed * 7919 + 1);

    // write (writer.rs:117-255): the batched path (FileWriteBuilder::batch over cec_multi jobs)
    // and the per-part path give the same parts, digests, locations and stored bytes, the short
    // last part included
    {
        const size_t cap = d * L, parts = uni(2, 12);
        Bytes file_bytes(parts * cap - (rng() % 2 ? uni(1, cap - 1) : 0));
        for (auto& b : file_bytes) b = uint8_t(rng());
        ChunkStore sa, sb;
        auto builder = [&] {
            FileWriteBuilder w;
            w.chunk_size(L).data_chunks(d).parity_chunks(p).concurrency(uni(2, 10));
            return w;
        };
        const FileReference fa = builder().write(file_bytes, sa);
        FileWriteBuilder wb = builder();
        wb.batch(uni(1, 3), uni(1, 4)).devices(rng() % 2 ? std::vector<int>{0} : std::vector<int>{0, 0});
        const FileReference fb = wb.write(file_bytes, sb);
        bool same = fa.parts.size() == fb.parts.size() && fa.length == fb.length &&
                    sa.size() == sb.size();
        for (size_t k = 0; same && k < fa.parts.size(); ++k)
            for (size_t i = 0; same && i < t; ++i) {
                const Chunk &ca = fa.parts[k].chunk(i), &cb = fb.parts[k].chunk(i);
                same = fa.parts[k].chunksize == fb.parts[k].chunksize && ca.hash == cb.hash &&
                       ca.locations == cb.locations && *sa.find(ca.locations[0]) == *sb.find(cb.locations[0]);
            }
        Bytes back;
        fb.read_to(sb, [&](const uint8_t* b, size_t len) { back.insert(back.end(), b, b + len); });
        if (!same || back != file_bytes) {
            std::fprintf(stderr, "seed %llu: batched write differs from the per-part write\n",
                         (unsigned long long)seed);
            return false;
        }
    }

    ChunkStore st;
    FileReference file;
    Bytes want;
    size_t first_short = n;
    std::vector<size_t> short_parts;
    for (size_t k = 0; k < n; ++k) {
        std::vector<Bytes> c(t, Bytes(L));
        for (size_t i = 0; i < d; ++i)
            for (auto& b : c[i]) b = uint8_t(rng());
        std::vector<const uint8_t*> dp(d);
        std::vector<uint8_t*> pp(p);
        std::vector<size_t> dl(d, L), pl(p, L);
        for (size_t i = 0; i < d; ++i) dp[i] = c[i].data();
        for (size_t i = 0; i < p; ++i) pp[i] = c[d + i].data();
        if (or_rs_encode_sep(d, p, dp.data(), dl.data(), d, pp.data(), pl.data(), p) != 0) return false;
        for (size_t i = 0; i < d; ++i) want.insert(want.end(), c[i].begin(), c[i].end());
        FilePart part;
        part.chunksize = L;
        size_t good = 0;
        for (size_t i = 0; i < t; ++i) {
            std::array<uint8_t, 32> h{};
            or_sha256(c[i].data(), L, h.data());
            Chunk ch{Sha256Hash(h), {}};
            const double u = double(rng() % 1000) / 1000.0;
            const char* spec = u < 0.7    ? "G"
                               : u < 0.78 ? "BG"
                               : u < 0.83 ? "XSG"
                               : u < 0.88 ? "BB"
                               : u < 0.94 ? "B"
                                          : "X";
            for (size_t j = 0; spec[j]; ++j) {
                const Location loc = std::to_string(k) + "/" + std::to_string(i) + "/" + std::to_string(j);
                ch.locations.push_back(loc);
                Bytes b = c[i];
                switch (spec[j]) {
                    case 'G': st.put(loc, b); ++good; break;
                    case 'B': b[rng() % L] ^= uint8_t(1 + rng() % 255); st.put(loc, b); break;
                    case 'S': b.resize(L / 2); st.put(loc, b); break;
                    default: break;  // 'X': the location does not read
                }
            }
            (i < d ? part.data : part.parity).push_back(std::move(ch));
        }
        if (good < d && first_short == n) first_short = k;
        if (good < d) short_parts.push_back(k);
        file.parts.push_back(std::move(part));
    }
    file.length = want.size();

    const size_t ppb = uni(1, 4), depth = uni(1, 7);
    const std::vector<int> devices = rng() % 2 ? std::vector<int>{0} : std::vector<int>{0, 0};
    detail::read_carry() = rng() % 2 == 0;
    if (rng() % 3 == 0) {
        // a sink that fails part way (FileReadBuilder's consumer gone): the read ends with its
        // error, every job waited for and every carry id given back; the read below reuses the
        // same windows
        const size_t stop_at = rng() % want.size();
        size_t seen = 0;
        bool thrown = false;
        try {
            file.read_to(st, [&](const uint8_t*, size_t len) {
                seen += len;
                if (seen > stop_at) throw std::runtime_error("sink closed");
            }, ppb, depth, devices);
        } catch (const ErasureError&) {  // a short part came first
        } catch (const std::runtime_error&) {
            thrown = true;
        }
        const cec_multi* m0 = detail::cached_multi_entry().multi.get();
        if (!m0 || !m0->jobs.empty() || !m0->pool.empty() || (!thrown && first_short == n)) {
            std::fprintf(stderr, "seed %llu: a failed sink left a job or carry id behind\n",
                         (unsigned long long)seed);
            return false;
        }
    }
    Bytes got;
    bool failed = false;
    try {
        file.read_to(st, [&](const uint8_t* b, size_t len) { got.insert(got.end(), b, b + len); },
                     ppb, depth, devices);
    } catch (const ErasureError& e) {
        failed = e.error() == Error::TooFewShardsPresent;
        if (!failed) {
            std::fprintf(stderr, "seed %llu: unexpected erasure error\n", (unsigned long long)seed);
            return false;
        }
    }
    const cec_multi* m = detail::cached_multi_entry().multi.get();
    bool ok = true;
    auto expect = [&](bool c, const char* what) {
        if (!c) {
            std::fprintf(stderr, "seed %llu (d=%zu p=%zu L=%zu n=%zu ppb=%zu depth=%zu shards=%zu): %s\n",
                         (unsigned long long)seed, d, p, L, n, ppb, depth, devices.size(), what);
            ok = false;
        }
    };
    expect(got.size() <= want.size() && std::equal(got.begin(), got.end(), want.begin()),
           "bytes out differ from the file");
    expect(got.size() % (d * L) == 0 || got.size() == want.size(), "a part cut short");
    if (first_short < n) {
        expect(failed, "a part without d good chunks did not fail the read");
        expect(got.size() <= first_short * d * L, "parts after the failing one came out");
    } else {
        expect(!failed && got.size() == want.size(), "the read did not return the whole file");
    }
    expect(m && m->jobs.empty(), "jobs left unwaited");
    expect(m && m->pool.empty(), "carry ids left held");

    // range reads (FileReadBuilder::seek / take, reader.rs:22-173; the gateway's Range requests):
    // the range's bytes, read from the parts that hold them -- a part without d good chunks fails
    // the read only when the range reaches into it
    for (int r = 0; r < 3; ++r) {
        // a third of the seeks on a part boundary (the part before must not be read)
        const uint64_t seek = rng() % 3 == 0 ? (rng() % (n + 1)) * d * L : rng() % (want.size() + 2);
        const uint64_t take = rng() % 3 == 0   ? 0
                              : rng() % 6 == 0 ? std::numeric_limits<uint64_t>::max()
                                               : rng() % (want.size() + 2);
        FileReadBuilder rb(file);
        rb.seek(seek).take(take);
        if (rng() % 2) rb.batch(ppb, depth).devices(devices);
        else if (rng() % 2) rb.buffer_bytes(rng() % (4 * d * L));  // 1..4 part reads in flight
        if (rb.get_buffer() < 1) {
            std::fprintf(stderr, "seed %llu: buffer_bytes gave 0\n", (unsigned long long)seed);
            return false;
        }
        const uint64_t len = rb.len_bytes();
        const uint64_t exp_len = seek >= want.size() ? 0 : take == 0 ? want.size() - seek
                                                                   : std::min<uint64_t>(take, want.size() - seek);
        expect(len == exp_len, "len_bytes differs from reader.rs:129-138");
        const size_t k_lo = size_t(seek / (d * L)), k_hi = size_t((seek + len + d * L - 1) / (d * L));
        const bool reaches_short = len && std::any_of(short_parts.begin(), short_parts.end(),
                                                      [&](size_t k) { return k >= k_lo && k < k_hi; });
        Bytes part_bytes;
        bool range_failed = false;
        try {
            part_bytes = rb.read(st);
        } catch (const ErasureError&) {
            range_failed = true;
        }
        expect(range_failed == reaches_short, "range read failed or passed unexpectedly");
        if (!range_failed)
            expect(part_bytes.size() == len &&
                   std::equal(part_bytes.begin(), part_bytes.end(), want.begin() + std::ptrdiff_t(std::min<uint64_t>(seek, want.size()))),
                   "range bytes differ from the file's");
        m = detail::cached_multi_entry().multi.get();
        expect(m && m->jobs.empty() && m->pool.empty(), "a range read left a job or carry id");
    }

    // verify and resilver (file_part.rs:228-390): the batched loops' reports and write-backs
    // equal the per-part calls' on copies of the same file and store
    FileReference fa = file, fb = file;
    ChunkStore sa = st, sb = st;
    auto same = [](const std::vector<PartReport>& a, const std::vector<PartReport>& b) {
        if (a.size() != b.size()) return false;
        for (size_t k = 0; k < a.size(); ++k)
            if (a[k].locations != b[k].locations || a[k].chunks != b[k].chunks ||
                a[k].new_locations != b[k].new_locations || a[k].write_error != b[k].write_error)
                return false;
        return true;
    };
    expect(same(fa.verify(sa), fb.verify(sb, ppb, depth, devices)), "batched verify reports differ");
    const std::vector<PartReport> rb = fb.resilver(sb, ppb, depth, devices);
    expect(same(fa.resilver(sa), rb), "batched resilver reports differ");
    bool same_store = true, unrepaired = false;
    for (size_t k = 0; k < n; ++k) {
        unrepaired = unrepaired || rb[k].write_error.has_value();
        for (size_t i = 0; i < t; ++i) {
            const Chunk &ca = fa.parts[k].chunk(i), &cb = fb.parts[k].chunk(i);
            same_store = same_store && ca.locations == cb.locations;
            for (const Location& loc : ca.locations) {
                const Bytes *x = sa.find(loc), *y = sb.find(loc);
                same_store = same_store && (x && y ? *x == *y : x == y);
            }
        }
    }
    expect(same_store, "batched resilver wrote other locations or bytes");
    expect(unrepaired == (first_short < n), "a part without d good chunks was rebuilt, or one with d was not");
    // the resilvered file reads back whole, up to a part resilver could not rebuild
    Bytes back;
    bool failed_again = false;
    try {
        fb.read_to(sb, [&](const uint8_t* b, size_t len) { back.insert(back.end(), b, b + len); },
                   ppb, depth, devices);
    } catch (const ErasureError&) {
        failed_again = true;
    }
    expect(failed_again == unrepaired, "read after resilver failed or passed unexpectedly");
    expect(unrepaired || back == want, "read after resilver differs from the file");
    m = detail::cached_multi_entry().multi.get();
    expect(m && m->jobs.empty() && m->pool.empty(), "verify / resilver left a job or carry id");
    return ok;
}

}  // namespace

int main(int argc, char** argv) {
    const uint64_t first = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 0;
    const uint64_t count = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 200;
    size_t bad = 0;
    for (uint64_t s = first; s < first + count; ++s) {
        const int before = g_violations;
        bool ok = false;
        try {
            ok = run_seed(s);
        } catch (const std::exception& e) {
            std::fprintf(stderr, "seed %llu: uncaught %s\n", (unsigned long long)s, e.what());
        }
        if (!ok || g_violations != before) ++bad;
    }
    std::printf("%llu seeds, %zu failed, %d contract violations\n", (unsigned long long)count, bad,
                g_violations);
    return bad == 0 ? 0 : 1;
}
