// hostmem.cpp — page-locked host buffers (cec_host_alloc / cec_host_free), pinned-range
// detection, and NUMA placement of the staging a GPU's copies go through.
//
// The reference allocates each part's data buffer with `vec![0; d*chunk_size]`
// (src/file/writer.rs:172) and the parity with `vec![vec![0; L]; p]` (file_part.rs:158).  On a
// GPU those bytes cross PCIe, and the copy engines only stream at full rate from page-locked
// memory: pageable buffers cost an extra host copy into pinned staging.  cec_host_alloc gives
// the caller pinned, portable (every device may DMA it) memory placed on the NUMA node of the
// device that will read it, so the engine can DMA straight from / into the caller's buffers.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "chunky_ec.h"
#include "hostmem.hpp"

namespace cec {
namespace {

std::mutex g_reg_mu;
std::map<uintptr_t, size_t>& registry() {  // base -> bytes of every live cec_host_alloc
    static auto* m = new std::map<uintptr_t, size_t>();
    return *m;
}

bool in_registry(const void* p, size_t n) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto& reg = registry();
    auto it = reg.upper_bound(a);
    if (it == reg.begin()) return false;
    --it;
    return a >= it->first && a + n <= it->first + it->second;
}

// CPUs listed in a sysfs cpulist ("0-15,32-47").
std::vector<int> parse_cpulist(const std::string& s) {
    std::vector<int> cpus;
    std::stringstream ss(s);
    std::string part;
    while (std::getline(ss, part, ',')) {
        if (part.empty()) continue;
        const size_t dash = part.find('-');
        const int lo = std::atoi(part.c_str());
        const int hi = dash == std::string::npos ? lo : std::atoi(part.c_str() + dash + 1);
        for (int c = lo; c <= hi && c >= 0; ++c) cpus.push_back(c);
    }
    return cpus;
}

std::string read_line(const std::string& path) {
    std::ifstream f(path);
    std::string line;
    if (f) std::getline(f, line);
    return line;
}

// set_mempolicy(2) / get_mempolicy(2) without libnuma.
constexpr int kMpolPreferred = 1;
constexpr unsigned long kMaxNodes = 1024;  // node mask bits saved / restored
long set_mempolicy_raw(int mode, const unsigned long* mask, unsigned long maxnode) {
    return syscall(SYS_set_mempolicy, mode, mask, maxnode);
}
long get_mempolicy_raw(int* mode, unsigned long* mask, unsigned long maxnode) {
    return syscall(SYS_get_mempolicy, mode, mask, maxnode, nullptr, 0ul);
}

}  // namespace

bool pinned_range(const void* p, size_t n) {
    if (!p) return false;
    if (n == 0) n = 1;
    if (in_registry(p, n)) return true;
    // Memory pinned elsewhere (hipHostMalloc / hipHostRegister / torch pin_memory): one
    // allocation must cover the whole range.
    hipPointerAttribute_t attr{};
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: not an error for the caller
        return false;
    }
    if (attr.type != hipMemoryTypeHost) return false;
    void* start = nullptr;
    size_t size = 0;
    hipDeviceptr_t dp = reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(p));
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, dp) != hipSuccess ||
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, dp) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    const uintptr_t a = reinterpret_cast<uintptr_t>(p), s = reinterpret_cast<uintptr_t>(start);
    return a >= s && a + n <= s + size;
}

int device_numa_node(int device) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    std::string id(bus);
    for (auto& c : id) c = char(std::tolower(static_cast<unsigned char>(c)));
    const std::string line = read_line("/sys/bus/pci/devices/" + id + "/numa_node");
    if (line.empty()) return -1;
    return std::atoi(line.c_str());
}

bool bind_thread_to_device_node(int device) {
    const int node = device_numa_node(device);
    if (node < 0) return false;
    const std::vector<int> cpus =
        parse_cpulist(read_line("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist"));
    if (cpus.empty()) return false;
    cpu_set_t now, want;
    CPU_ZERO(&now);
    CPU_ZERO(&want);
    if (sched_getaffinity(0, sizeof(now), &now) != 0) return false;
    int n = 0;
    for (int c : cpus)
        if (c < CPU_SETSIZE && CPU_ISSET(c, &now)) {
            CPU_SET(c, &want);
            ++n;
        }
    if (n == 0) return false;  // the node's CPUs are outside this process's cpuset
    return sched_setaffinity(0, sizeof(want), &want) == 0;
}

hipError_t host_malloc_near(void** out, size_t bytes, unsigned flags, int device) {
    // Pages land on the device's NUMA node: prefer that node for this thread while HIP pins them
    // (hipHostMallocNumaUser: HIP follows the thread's policy), then restore the thread's own
    // policy (a caller under `numactl --membind` keeps it).
    const int node = device >= 0 ? device_numa_node(device) : -1;
    constexpr size_t kWords = kMaxNodes / (8 * sizeof(unsigned long));
    unsigned long saved_mask[kWords] = {};
    int saved_mode = 0;
    bool policy = false;
    if (node >= 0 && node < 64 && get_mempolicy_raw(&saved_mode, saved_mask, kMaxNodes) == 0) {
        const unsigned long mask = 1ul << node;
        policy = set_mempolicy_raw(kMpolPreferred, &mask, 64) == 0;
    }
    const hipError_t e = hipHostMalloc(out, bytes, flags | (policy ? hipHostMallocNumaUser : 0u));
    if (policy) (void)set_mempolicy_raw(saved_mode, saved_mask, kMaxNodes);
    return e;
}

}  // namespace cec

using namespace cec;

extern "C" {

int cec_current_device(int* device) {
    if (!device) return CEC_ERR_INVALID_ARGUMENT;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        *device = 0;
        return CEC_ERR_NO_DEVICE;
    }
    return hipGetDevice(device) == hipSuccess ? CEC_OK : CEC_ERR_HIP;
}

int cec_set_device(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        return CEC_ERR_NO_DEVICE;
    }
    if (device < 0 || device >= n) return CEC_ERR_INVALID_ARGUMENT;
    return hipSetDevice(device) == hipSuccess ? CEC_OK : CEC_ERR_HIP;
}

int cec_device_numa_node(int device) { return device_numa_node(device); }

int cec_host_alloc(size_t bytes, int device, void** out) {
    if (!out || bytes == 0) return CEC_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        return CEC_ERR_NO_DEVICE;
    }
    if (device >= n) return CEC_ERR_INVALID_ARGUMENT;
    void* p = nullptr;
    const hipError_t e = host_malloc_near(&p, bytes, hipHostMallocPortable, device);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return e == hipErrorOutOfMemory ? CEC_ERR_OUT_OF_MEMORY : CEC_ERR_HIP;
    }
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        registry()[reinterpret_cast<uintptr_t>(p)] = bytes;
    }
    *out = p;
    return CEC_OK;
}

void cec_host_free(void* p) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        registry().erase(reinterpret_cast<uintptr_t>(p));
    }
    (void)hipHostFree(p);
}

int cec_host_is_pinned(const void* p, size_t bytes) { return pinned_range(p, bytes) ? 1 : 0; }

int cec_bind_thread_to_device_node(int device) { return bind_thread_to_device_node(device) ? 1 : 0; }

int cec_host_numa_node(const void* p) {
    // move_pages(2) in query mode (nodes == NULL) reports the node of each page.
    void* page = reinterpret_cast<void*>(reinterpret_cast<uintptr_t>(p) &
                                         ~uintptr_t(sysconf(_SC_PAGESIZE) - 1));
    int status = -1;
    if (syscall(SYS_move_pages, 0, 1ul, &page, nullptr, &status, 0) != 0) return -1;
    return status >= 0 ? status : -1;  // a page not resident / not mapped: -ENOENT, -EFAULT
}

}  // extern "C"
