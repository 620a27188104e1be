// numa_affinity.hip -- bind host worker threads to the NUMA node of their GPU
// (one worker pool per GPU, cores split per GPU, NUMA-local).
// Linux sysfs only; everything degrades to "no binding" when a file is absent.
#include <pthread.h>
#include <sched.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

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

}  // namespace

hjd_internal::CpuSet hjd_internal::device_local_cpus(int device)
{
    CpuSet s;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return s;
    for (char* p = bus; *p; ++p)
        if (*p >= 'A' && *p <= 'F') *p = static_cast<char>(*p - 'A' + 'a');
    const std::string node = read_file(std::string("/sys/bus/pci/devices/") + bus + "/numa_node");
    if (node.empty()) return s;
    const int n = atoi(node.c_str());
    if (n < 0) return s;
    std::vector<int> cpus = parse_cpulist(read_file("/sys/devices/system/node/node" + std::to_string(n) + "/cpulist"));
    // only CPUs this process may run on (container cpusets, taskset)
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) == 0) {
        std::vector<int> keep;
        for (int c : cpus)
            if (CPU_ISSET(c, &allowed)) keep.push_back(c);
        cpus.swap(keep);
    }
    s.cpus = cpus;
    return s;
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
    std::vector<int> cpus =
        parse_cpulist(read_file("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist"));
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) == 0) {
        std::vector<int> keep;
        for (int c : cpus)
            if (CPU_ISSET(c, &allowed)) keep.push_back(c);
        cpus.swap(keep);
    }
    s.cpus = cpus;
    return s;
}
