// numa_affinity.hip -- bind host worker threads to their GPU's share of its NUMA
// node (one worker pool per GPU, cores split per GPU, NUMA-local).
// Linux sysfs only; everything degrades to "no binding" when a file is absent.
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "hjd.h"
#include "hjd_host.h"
#include "hjd_internal.h"

namespace {

std::vector<int> parse_cpulist(const std::string& s)
{
    std::vector<int> out;
    size_t i = 0;
    while (i < s.size()) {
        while (i < s.size() && (s[i] == ',' || s[i] == ' ' || s[i] == '\n')) ++i;
        if (i >= s.size()) break;
        int a = 0, b = -1;
        size_t k = i;
        while (k < s.size() && s[k] >= '0' && s[k] <= '9') a = a * 10 + (s[k++] - '0');
        if (k == i) break;
        if (k < s.size() && s[k] == '-') {
            b = 0;
            size_t m = ++k;
            while (k < s.size() && s[k] >= '0' && s[k] <= '9') b = b * 10 + (s[k++] - '0');
            if (k == m) b = a;
        } else {
            b = a;
        }
        for (int c = a; c <= b && c < CPU_SETSIZE; ++c) out.push_back(c);
        i = k;
    }
    return out;
}

std::string read_file(const std::string& path)
{
    FILE* f = fopen(path.c_str(), "r");
    if (!f) return {};
    char buf[4096];
    const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[n] = 0;
    return buf;
}

std::string lower(std::string s)
{
    for (char& c : s)
        if (c >= 'A' && c <= 'F') c = static_cast<char>(c - 'A' + 'a');
    return s;
}

std::vector<int> allowed_only(std::vector<int> cpus)
{
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return cpus;
    std::vector<int> keep;
    for (int c : cpus)
        if (CPU_ISSET(c, &allowed)) keep.push_back(c);
    return keep;
}

int numa_node_of(const std::string& root, const std::string& bus)
{
    const std::string node = read_file(root + "/sys/bus/pci/devices/" + lower(bus) + "/numa_node");
    return node.empty() ? -1 : atoi(node.c_str());
}

// The host CPUs for the worker pool of the GPU at PCI address `bus`, among
// the GPUs `gpus` this process sees (one pool per GPU, the
// cores split per GPU, NUMA-local).  The GPUs on the same NUMA node, in bus
// order, split that node's CPUs into equal contiguous slices (the first
// node_cpus % k GPUs take one more); with fewer CPUs than GPUs every GPU of the
// node shares all of them.  Unknown topology: empty (no binding).  `root` is
// "" for the real sysfs (a test passes a fake tree); `only_allowed` intersects
// the node's CPUs with this process's affinity first.
std::vector<int> split_worker_cpus(const std::string& root, const std::string& bus,
                                   const std::vector<std::string>& gpus, bool only_allowed)
{
    const int node = numa_node_of(root, bus);
    if (node < 0) return {};
    std::vector<int> cpus =
        parse_cpulist(read_file(root + "/sys/devices/system/node/node" + std::to_string(node) + "/cpulist"));
    if (only_allowed) cpus = allowed_only(cpus);
    std::vector<std::string> peers;
    for (const std::string& g : gpus)
        if (numa_node_of(root, g) == node) peers.push_back(lower(g));
    std::sort(peers.begin(), peers.end());
    peers.erase(std::unique(peers.begin(), peers.end()), peers.end());
    const auto it = std::find(peers.begin(), peers.end(), lower(bus));
    const int k = static_cast<int>(peers.size());
    if (it == peers.end() || k <= 1 || static_cast<int>(cpus.size()) < k) return cpus;
    const int i = static_cast<int>(it - peers.begin());
    const int n = static_cast<int>(cpus.size()), q = n / k, r = n % k;
    const int b0 = i * q + std::min(i, r), b1 = b0 + q + (i < r ? 1 : 0);
    return std::vector<int>(cpus.begin() + b0, cpus.begin() + b1);
}

std::string bus_id(int device)
{
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) {
        (void)hipGetLastError();
        return {};
    }
    return bus;
}

}  // namespace

hjd_internal::CpuSet hjd_internal::device_local_cpus(int device)
{
    CpuSet s;
    const std::string mine = bus_id(device);
    if (mine.empty()) return s;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        n = 0;
    }
    std::vector<std::string> gpus;
    for (int d = 0; d < n; ++d) {
        const std::string b = bus_id(d);
        if (!b.empty()) gpus.push_back(b);
    }
    s.cpus = split_worker_cpus("", mine, gpus, true);
    return s;
}

extern "C" int hjd_device_worker_cpus(int device, int32_t* cpus, int capacity, int32_t* ncpus)
{
    if (capacity < 0 || (!cpus && capacity > 0) || !ncpus) return hjd_internal::set_error(HJD_E_INVALID, "invalid arguments");
    const hjd_internal::CpuSet s = hjd_internal::device_local_cpus(device);
    *ncpus = static_cast<int32_t>(s.cpus.size());
    for (int i = 0; i < static_cast<int>(s.cpus.size()) && i < capacity; ++i) cpus[i] = s.cpus[i];
    return 0;
}

int hjd_internal::default_worker_threads(int device)
{
    const int share = hjd_host_cpu_share();
    const int slice = static_cast<int>(device_local_cpus(device).cpus.size());
    return slice > 0 ? std::min(share, slice) : share;
}

extern "C" int hjd_debug_worker_cpus(const char* sysfs_root, const char* bus, const char* const* gpus, int ngpus,
                                     int only_allowed, int32_t* cpus, int capacity, int32_t* ncpus)
{
    if (!bus || (!gpus && ngpus > 0) || ngpus < 0 || capacity < 0 || (!cpus && capacity > 0) || !ncpus)
        return hjd_internal::set_error(HJD_E_INVALID, "invalid arguments");
    std::vector<std::string> g;
    for (int i = 0; i < ngpus; ++i) g.push_back(gpus[i] ? gpus[i] : "");
    const std::vector<int> r = split_worker_cpus(sysfs_root ? sysfs_root : "", bus, g, only_allowed != 0);
    *ncpus = static_cast<int32_t>(r.size());
    for (int i = 0; i < static_cast<int>(r.size()) && i < capacity; ++i) cpus[i] = r[i];
    return 0;
}

std::vector<int> hjd_internal::bind_current_thread(const CpuSet& s)
{
    std::vector<int> prev;
    cpu_set_t cur;
    CPU_ZERO(&cur);
    if (pthread_getaffinity_np(pthread_self(), sizeof(cur), &cur) == 0)
        for (int c = 0; c < CPU_SETSIZE; ++c)
            if (CPU_ISSET(c, &cur)) prev.push_back(c);
    if (s.cpus.empty()) return prev;
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int c : s.cpus) CPU_SET(c, &set);
    (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    return prev;
}

void hjd_internal::restore_current_thread(const std::vector<int>& prev)
{
    if (prev.empty()) return;
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int c : prev) CPU_SET(c, &set);
    (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

hjd_internal::CpuSet hjd_internal::node_cpus(int node)
{
    CpuSet s;
    if (node < 0) return s;
    s.cpus = allowed_only(parse_cpulist(read_file("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist")));
    return s;
}
