// chunky-shards — the reference CLI's `encode-shards` / `decode-shards` subcommands
// (src/bin/chunky-bits/main.rs:235-312, argument checks in get_shard_encoder at :521-559) over
// the engine's per-call C-ABI: the one direct use of the erasure crate outside FilePart, where
// the swap is `encoder.encode_sep` -> cec_encode_sep and `encoder.reconstruct_data` ->
// cec_reconstruct_data (through chunky_ec::ReedSolomon).
//
//   chunky-shards [--data-chunks D] --parity-chunks P encode-shards SOURCE TARGET...
//   chunky-shards [--data-chunks D] --parity-chunks P decode-shards TARGET...
//
// Locations are local paths or `-` (stdin / stdout), the `Other(Local)` and `Stdio` cases of
// ClusterLocation (cluster_location.rs:653-702); cluster and HTTP locations are out of scope
// (DESIGN.md §7).  Behaviour follows the reference:
//   - P is required for both commands ("Parity Chunk Count must be known to decode shards");
//     D, when given, must make D+P equal the target count, else D = targets - P (> 0);
//   - encode: the whole source is read, padded with zeros to D*ceil(len/D), cut into D data
//     shards, P parity shards are computed, and shard i is written to target i (data first);
//     a target that cannot be written prints "Error <target>: <err>" and the rest go on;
//   - decode: every target is read (an unreadable one prints "Error <target>: <err>" and counts
//     as missing), missing data shards are rebuilt, and the D data shards (padding included,
//     as the reference does not truncate) go to stdout;
//   - crate errors and argument errors print one line on stderr and exit 1; a malformed option
//     value exits 2 like clap, with the SizeError text of cluster/sized_int.rs:34-42.
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "chunky_ec.hpp"

using chunky_ec::Bytes;

namespace {

struct Fail {
    std::string msg;
    int code;
};

// std::io::Error's Display: "<strerror> (os error N)".
std::string os_error(int e) { return std::string(std::strerror(e)) + " (os error " + std::to_string(e) + ")"; }

// Whole contents of a location ("-" = stdin).
bool read_all(const std::string& loc, Bytes& out, std::string& err) {
    FILE* f = loc == "-" ? stdin : std::fopen(loc.c_str(), "rb");
    if (!f) {
        err = os_error(errno);
        return false;
    }
    out.clear();
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) out.insert(out.end(), buf, buf + n);
    const bool bad = std::ferror(f);
    const int e = errno;
    if (f != stdin) std::fclose(f);
    if (bad) err = os_error(e);
    return !bad;
}

bool write_all(const std::string& loc, const uint8_t* p, size_t n, std::string& err) {
    FILE* f = loc == "-" ? stdout : std::fopen(loc.c_str(), "wb");
    if (!f) {
        err = os_error(errno);
        return false;
    }
    const bool ok = (n == 0 || std::fwrite(p, 1, n, f) == n) && std::fflush(f) == 0;
    const int e = errno;
    if (f != stdout && std::fclose(f) != 0 && ok) {
        err = os_error(errno);
        return false;
    }
    if (!ok) err = os_error(e);
    return ok;
}

// DataChunkCount (1..=255) / ParityChunkCount (0..=255): parsed as u8 then range-checked.
size_t parse_count(const std::string& flag, const std::string& v, size_t min, const char* name) {
    bool digits = !v.empty() && v.size() <= 3;
    for (char c : v) digits = digits && c >= '0' && c <= '9';
    const long x = digits ? std::stol(v) : -1;
    if (x < long(min) || x > 255) {
        std::string upper = flag.substr(2);
        for (auto& c : upper) c = c == '-' ? '_' : char(std::toupper(static_cast<unsigned char>(c)));
        throw Fail{"error: invalid value '" + v + "' for '" + flag + " <" + upper + ">': " + name +
                       " must be greater than " + std::to_string(min) + " and less than 256",
                   2};
    }
    return size_t(x);
}

// get_shard_encoder (main.rs:521-559).
size_t shard_data_count(bool have_d, size_t d, bool have_p, size_t p, size_t targets) {
    if (!have_p) throw Fail{"Parity Chunk Count must be known to decode shards", 1};
    if (have_d) {
        if (targets != d + p)
            throw Fail{"Invalid targets: Expected " + std::to_string(d + p) + " targets but got " +
                           std::to_string(targets),
                       1};
        return d;
    }
    if (targets <= p)
        throw Fail{"Invalid targets: Expected more than " + std::to_string(p) + " targets but got " +
                       std::to_string(targets),
                   1};
    return targets - p;
}

int encode_shards(const chunky_ec::ReedSolomon& rs, const std::string& source,
                  const std::vector<std::string>& targets) {
    const size_t d = rs.data_shard_count(), p = rs.parity_shard_count();
    Bytes data;
    std::string err;
    if (!read_all(source, data, err)) throw Fail{source + ": " + err, 1};
    const size_t len = (data.size() + d - 1) / d;  // buf_length (main.rs:280)
    data.resize(len * d, 0);
    std::vector<std::pair<const uint8_t*, size_t>> views;
    for (size_t j = 0; j < d; ++j) views.emplace_back(data.data() + j * len, len);
    std::vector<Bytes> parity(p, Bytes(len, 0));
    rs.encode_sep(views, parity);
    for (size_t i = 0; i < targets.size(); ++i) {
        const uint8_t* src = i < d ? views[i].first : parity[i - d].data();
        if (!write_all(targets[i], src, len, err))
            std::fprintf(stderr, "Error %s: %s\n", targets[i].c_str(), err.c_str());
    }
    return 0;
}

int decode_shards(const chunky_ec::ReedSolomon& rs, const std::vector<std::string>& targets) {
    const size_t d = rs.data_shard_count();
    chunky_ec::Shards shards(targets.size());
    for (size_t i = 0; i < targets.size(); ++i) {
        Bytes b;
        std::string err;
        if (read_all(targets[i], b, err))
            shards[i] = std::move(b);
        else  // get_reader's prefix_err (error_message.rs:16-21) names the target once more
            std::fprintf(stderr, "Error %s: %s: %s\n", targets[i].c_str(), targets[i].c_str(),
                         err.c_str());
    }
    rs.reconstruct_data(shards);
    for (size_t j = 0; j < d; ++j) {
        if (!shards[j]) continue;
        std::string err;
        if (!write_all("-", shards[j]->data(), shards[j]->size(), err)) throw Fail{err, 1};
    }
    return 0;
}

int usage() {
    std::fprintf(stderr,
                 "usage: chunky-shards [--data-chunks D] --parity-chunks P encode-shards SOURCE "
                 "TARGET...\n"
                 "       chunky-shards [--data-chunks D] --parity-chunks P decode-shards TARGET...\n");
    return 2;
}

}  // namespace

int main(int argc, char** argv) {
    try {
        bool have_d = false, have_p = false;
        size_t d = 0, p = 0;
        int i = 1;
        // Global options (Opt, main.rs:78-92); --config / --chunk-size do not affect these two
        // commands and are accepted for command-line compatibility.
        for (; i < argc && std::strncmp(argv[i], "--", 2) == 0; ++i) {
            std::string flag = argv[i], val;
            const size_t eq = flag.find('=');
            if (eq != std::string::npos) {
                val = flag.substr(eq + 1);
                flag = flag.substr(0, eq);
            } else if (i + 1 < argc) {
                val = argv[++i];
            } else {
                return usage();
            }
            if (flag == "--data-chunks") {
                d = parse_count(flag, val, 1, "DataChunkCount");
                have_d = true;
            } else if (flag == "--parity-chunks") {
                p = parse_count(flag, val, 0, "ParityChunkCount");
                have_p = true;
            } else if (flag != "--config" && flag != "--chunk-size") {
                return usage();
            }
        }
        if (i >= argc) return usage();
        const std::string cmd = argv[i++];
        std::vector<std::string> rest(argv + i, argv + argc);
        if (cmd == "encode-shards") {
            if (rest.size() < 2) return usage();
            const std::string source = rest.front();
            const std::vector<std::string> targets(rest.begin() + 1, rest.end());
            const size_t data = shard_data_count(have_d, d, have_p, p, targets.size());
            return encode_shards(chunky_ec::ReedSolomon(data, p), source, targets);
        }
        if (cmd == "decode-shards") {
            if (rest.empty()) return usage();
            const size_t data = shard_data_count(have_d, d, have_p, p, rest.size());
            return decode_shards(chunky_ec::ReedSolomon(data, p), rest);
        }
        return usage();
    } catch (const Fail& f) {
        std::fprintf(stderr, "%s\n", f.msg.c_str());
        return f.code;
    } catch (const std::exception& e) {  // ErasureError (crate variant name) / EngineError
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
}
