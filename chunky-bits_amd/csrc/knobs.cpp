// Environment knobs, parsed once into an immutable snapshot (knobs.hpp).
#include "knobs.hpp"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "chunky_ec.h"

namespace cec {

namespace {

// "0" -> false, anything else set -> true, unset -> dflt
bool flag(const char* name, bool dflt) {
    const char* e = std::getenv(name);
    return e ? !(e[0] == '0') : dflt;
}

unsigned long long number(const char* name, unsigned long long dflt) {
    const char* e = std::getenv(name);
    return e ? std::strtoull(e, nullptr, 10) : dflt;
}

Knobs* parse() {
    auto* k = new Knobs();
    // Product knobs: capacities and diagnostics, and the test knobs that force one of the
    // product's own paths at test sizes (both arms are product code, picked by shape or size).
    k->apply_bs = flag("CEC_APPLY_BS", true);
    k->apply_max_blocks = number("CEC_APPLY_MAX_BLOCKS", 0);
    if (const char* e = std::getenv("CEC_SHA_VARIANT")) k->sha_variant = std::atoi(e);
    if (const char* e = std::getenv("CEC_FUSED_MODE")) k->fused_mode = std::atoi(e);
    if (const char* e = std::getenv("CEC_FUSED"))
        k->fused = e[0] == '0' ? 0 : e[0] == '1' ? 1 : -1;
    k->coalesce_us = uint32_t(number("CEC_COALESCE_US", 200));
    k->coalesce_max_bytes = std::max<size_t>(size_t(number("CEC_COALESCE_MAX_MIB", 1024)), 1)
                            << 20;
    k->coalesce_trace = std::getenv("CEC_COALESCE_TRACE") != nullptr;
    k->coalesce_inflight =
        uint32_t(std::min<unsigned long long>(std::max(number("CEC_COALESCE_INFLIGHT", 2), 1ull), 16ull));
    if (std::getenv("CEC_IDLE_STAGING_MIB"))
        k->idle_staging_bytes = size_t(number("CEC_IDLE_STAGING_MIB", 1024)) << 20;
    k->multi_copy_threads = unsigned(
        std::min<unsigned long long>(std::max(number("CEC_MULTI_COPY_THREADS", 4), 1ull), 32ull));
#ifdef CEC_AB_TOOLS
    // The losing arms of finished A/B experiments (profiles/HISTORY.md): read only
    // by the A/B build (`make ab`, tools/ab/libchunky_ec.so); the product library keeps every
    // one of them at the measured winner.
    if (const char* e = std::getenv("CEC_APPLY_TUNE"))
        k->apply_tune = (std::strstr(e, "nt") ? 1 : 0) | (std::strstr(e, "g8") ? 2 : 0) |
                        (std::strstr(e, "v1") ? 4 : 0);
    k->apply_xcd = flag("CEC_APPLY_XCD", true);
    if (const char* e = std::getenv("CEC_APPLY_BLOCKS_PER_CU")) k->apply_blocks_per_cu = std::atoi(e);
    k->apply_rg_classes = flag("CEC_APPLY_RGCLS", true);
    k->apply_cd = flag("CEC_APPLY_CD", true);
    k->apply_tile = number("CEC_APPLY_TILE", 0);
    if (const char* e = std::getenv("CEC_FUSED_PRIO"))
        if (e[0] >= '0' && e[0] <= '2') k->fused_prio = e[0] - '0';
    if (const char* e = std::getenv("CEC_FUSED_BE"))
        if (e[0] == '0' || e[0] == '1') k->fused_be = e[0] - '0';
    k->fused_enc3 = flag("CEC_FUSED_ENC3", true);
    if (const char* e = std::getenv("CEC_COALESCE_D2H_WAIT"))
        k->coalesce_d2h_host_wait = std::strcmp(e, "device") != 0;
    k->coalesce_early_d2h = flag("CEC_COALESCE_EARLY_D2H", true);
    if (const char* e = std::getenv("CEC_COALESCE_EARLY_H2D")) k->coalesce_early_h2d = e[0] == '1';
    k->coalesce_adaptive = flag("CEC_COALESCE_ADAPT", true);
    if (const char* e = std::getenv("CEC_SPEC_LDS_KIB")) k->spec_lds = uint32_t(std::atoi(e)) * 1024u;
    k->read_speculate = flag("CEC_READ_SPECULATE", true);
    k->verify_compact = flag("CEC_VERIFY_COMPACT", true);
#endif
    return k;
}

std::atomic<const Knobs*> g_knobs{nullptr};
std::mutex g_parse_mu;

}  // namespace

const Knobs& knobs() {
    const Knobs* k = g_knobs.load(std::memory_order_acquire);
    if (k) return *k;
    std::lock_guard<std::mutex> lk(g_parse_mu);
    k = g_knobs.load(std::memory_order_acquire);
    if (!k) {
        k = parse();
        g_knobs.store(k, std::memory_order_release);
    }
    return *k;
}

void reload_knobs() {
    std::lock_guard<std::mutex> lk(g_parse_mu);
    // the old snapshot stays allocated: a launch on another thread may still be reading it
    g_knobs.store(parse(), std::memory_order_release);
}

}  // namespace cec

extern "C" void cec_reload_knobs(void) { cec::reload_knobs(); }
