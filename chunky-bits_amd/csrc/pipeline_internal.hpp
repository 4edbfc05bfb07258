// pipeline_internal.hpp — read-pipeline entry points the scheduler (multi.cpp) uses beyond the
// C-ABI.  Not exported.
#pragma once
#include <cstddef>
#include <cstdint>

#include "chunky_ec.h"

namespace cec {

// As cec_read_pipeline_acquire, for slot `slot` (waits for its batch if one is in flight): the
// scheduler picks its slots itself (a free one; an AHEAD slot for a retry round).
int read_pipeline_acquire_slot(cec_read_pipeline* pl, size_t slot, uint8_t** chunks,
                               uint8_t** present, uint8_t** expected);

// Gives slot `slot` (no batch in flight) a stream of the device's greatest priority instead of
// its plain one.  HIP pools the streams of each priority onto their own GPU_MAX_HW_QUEUES hardware
// queues, so the scheduler's AHEAD slots do not share an in-order queue with a window's batch
// (a retry round queued behind a whole window batch waits for it).  Called when the pipeline is
// made, before any batch.  A device without priorities keeps the plain stream.
int read_pipeline_priority_slot(cec_read_pipeline* pl, size_t slot);

}  // namespace cec
