// Environment knobs of the engine, read ONCE per process.
//
// Every knob is parsed into one immutable snapshot on first use; the launch paths read the
// snapshot, never the environment.  The product library reads only capacity / diagnostic knobs
// and the test knobs that force one of its own paths (CEC_APPLY_BS, CEC_APPLY_MAX_BLOCKS,
// CEC_SHA_VARIANT 1/2, CEC_FUSED_MODE 3, CEC_FUSED, CEC_COALESCE_US / _MAX_MIB / _INFLIGHT /
// _TRACE, CEC_IDLE_STAGING_MIB, CEC_MULTI_COPY_THREADS); the losing arms of finished A/B
// experiments (the other fields below) are read only by the A/B build (-DCEC_AB_TOOLS).
// The reference calls the hot path from tokio worker threads (writer.rs:200-210 spawns a task
// per part; file_part.rs:161 runs the encode inside block_in_place), and getenv racing a setenv
// elsewhere in the host process is undefined behaviour; a snapshot read is a plain load.
//
// cec_reload_knobs() (include/chunky_ec.h, test-only) re-reads the environment into a fresh
// snapshot: the tests that flip a knob set the variable, reload, and reload again after
// restoring it.  Snapshots are never freed (a launch on another thread may still hold the old
// one); a reload costs one small allocation.
#pragma once

#include <cstddef>
#include <cstdint>

namespace cec {

struct Knobs {
    // rs_kernels.hip (meanings at each knob's use)
    int apply_tune = 1;             // CEC_APPLY_TUNE: bit 0 nt, bit 1 g8, bit 2 v1
    bool apply_xcd = true;          // CEC_APPLY_XCD
    int apply_blocks_per_cu = -1;   // CEC_APPLY_BLOCKS_PER_CU (-1: unset, per-kernel default)
    bool apply_rg_classes = true;   // CEC_APPLY_RGCLS
    bool apply_cd = true;           // CEC_APPLY_CD
    uint64_t apply_tile = 0;        // CEC_APPLY_TILE (0: unset)
    uint64_t apply_max_blocks = 0;  // CEC_APPLY_MAX_BLOCKS (0: unset)
    bool apply_bs = true;           // CEC_APPLY_BS
    // sha256_kernels.hip / fused_kernels.hip
    int sha_variant = 0;            // CEC_SHA_VARIANT (raw value; the product build filters it)
    int fused_prio = -1;            // CEC_FUSED_PRIO 0/1/2 (-1: the build's default)
    int fused_be = -1;              // CEC_FUSED_BE 0/1 (-1: the build's default)
    bool fused_enc3 = true;         // CEC_FUSED_ENC3
    int fused_mode = 0;             // CEC_FUSED_MODE (raw value; the product build filters it)
    // capi.cpp
    int fused = -1;                 // CEC_FUSED 0/1 (-1: by batch size)
    uint32_t coalesce_us = 200;     // CEC_COALESCE_US
    size_t coalesce_max_bytes = size_t(1024) << 20;  // CEC_COALESCE_MAX_MIB
    bool coalesce_trace = false;    // CEC_COALESCE_TRACE
    bool coalesce_d2h_host_wait = true;  // CEC_COALESCE_D2H_WAIT (host | device)
    bool coalesce_early_d2h = true;      // CEC_COALESCE_EARLY_D2H
    bool coalesce_early_h2d = false;     // CEC_COALESCE_EARLY_H2D
    bool coalesce_adaptive = true;       // CEC_COALESCE_ADAPT
    uint32_t coalesce_inflight = 2;      // CEC_COALESCE_INFLIGHT (1..16)
    uint32_t spec_lds = 100u * 1024u;    // CEC_SPEC_LDS_KIB
    bool read_speculate = true;          // CEC_READ_SPECULATE
    bool verify_compact = true;          // CEC_VERIFY_COMPACT
    size_t idle_staging_bytes = size_t(1) << 30;  // CEC_IDLE_STAGING_MIB (per device)
    // multi.cpp
    unsigned multi_copy_threads = 4;     // CEC_MULTI_COPY_THREADS (1..32)
};

// The current snapshot (parsed on first call).
const Knobs& knobs();
// Parse the environment into a new snapshot and make it current.
void reload_knobs();

}  // namespace cec
