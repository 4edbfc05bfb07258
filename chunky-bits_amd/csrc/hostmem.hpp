// hostmem.hpp — page-locked host memory and NUMA placement shared by the pipelines, the
// per-call coalescer and the multi-GPU scheduler (hostmem.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace cec {

// [p, p + n) lies inside one page-locked host allocation (cec_host_alloc, or any hipHostMalloc /
// hipHostRegister range HIP reports), so a copy engine can DMA it directly (no staging copy).
bool pinned_range(const void* p, size_t n);

// NUMA node of a HIP device's PCIe root (-1 when unknown), from sysfs via its PCI bus id.
int device_numa_node(int device);

// Restrict the calling thread to the CPUs of `device`'s NUMA node (intersected with the CPUs it
// may use now).  Returns false (and leaves the affinity alone) when that is not possible.
bool bind_thread_to_device_node(int device);

// hipHostMalloc(bytes, flags) with the pages preferred on `device`'s NUMA node (device < 0 or
// node unknown: the default placement).  Used for every pinned buffer the engine allocates
// itself (pipeline slots, scheduler staging) and by cec_host_alloc.
hipError_t host_malloc_near(void** out, size_t bytes, unsigned flags, int device);

}  // namespace cec
