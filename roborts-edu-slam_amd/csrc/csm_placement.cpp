// csm_placement.cpp — where a context's host worker pool runs (include/csm.h
// csm_host_plan). The reference matches scans on one host thread
// (correlate_scan_matcher.h has no threading), so this has no
// reference counterpart: it sizes the pool that plans and completes the
// windows (csm_driver.cpp) for one process per GPU. Each
// local rank gets a disjoint slice of the CPUs it may run on near its GPU,
// and as many threads as its share of the cgroup's CPU quota: eight ranks on
// one node no longer start 8 x 16 pool threads on a 16-CPU quota.
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "csm.h"

namespace csmh {

constexpr int kHostThreadsMax = 16;  // more measured no faster

// "0-7,16-23" -> {0..7, 16..23}
std::vector<int> parse_cpulist(const char* s) {
  std::vector<int> out;
  while (s && *s) {
    char* end = nullptr;
    const long a = std::strtol(s, &end, 10);
    if (end == s) break;
    long b = a;
    s = end;
    if (*s == '-') {
      b = std::strtol(s + 1, &end, 10);
      s = end;
    }
    for (long c = a; c <= b && c < 65536; ++c) out.push_back((int)c);
    while (*s == ',' || *s == '\n' || *s == ' ') ++s;
  }
  return out;
}

namespace {

std::string read_file(const char* path) {
  std::string out;
  if (FILE* f = std::fopen(path, "r")) {
    char buf[4096];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) out.append(buf, n);
    std::fclose(f);
  }
  return out;
}

// the cgroup's CPU quota in whole CPUs (v2 cpu.max, then v1), -1 when none
int cgroup_quota_cpus() {
  const std::string v2 = read_file("/sys/fs/cgroup/cpu.max");
  if (!v2.empty()) {
    char q[32] = {0};
    long per = 0;
    if (std::sscanf(v2.c_str(), "%31s %ld", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0)
      return (int)std::max(1L, std::atol(q) / per);
    return -1;
  }
  const std::string q1 = read_file("/sys/fs/cgroup/cpu/cpu.cfs_quota_us");
  const std::string p1 = read_file("/sys/fs/cgroup/cpu/cpu.cfs_period_us");
  const long q = q1.empty() ? -1 : std::atol(q1.c_str()), p = p1.empty() ? 0 : std::atol(p1.c_str());
  return (q > 0 && p > 0) ? (int)std::max(1L, q / p) : -1;
}

std::vector<int> affinity_cpus() {
  std::vector<int> out;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0)
    for (int c = 0; c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &set)) out.push_back(c);
  return out;
}

std::vector<int> node_cpus(int node) {
  if (node < 0) return {};
  char path[96];
  std::snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
  return parse_cpulist(read_file(path).c_str());
}

}  // namespace

// The plan itself (csm_host_plan_compute). numa_of: each local rank's NUMA
// node (-1 unknown; null: all unknown). quota: cgroup CPUs (-1 none).
void host_plan(int rank, int world, const int32_t* numa_of, int quota, const std::vector<int>& aff,
               csm_host_plan* out) {
  std::memset(out, 0, sizeof(*out));
  world = std::max(1, world);
  rank = std::min(std::max(0, rank), world - 1);
  const int my = numa_of ? numa_of[rank] : -1;
  out->numa_node = my;
  out->quota_cpus = quota;
  out->affinity_cpus = (int32_t)aff.size();
  // the CPUs near the device that the process may use, shared by the local
  // ranks on the same node; without a node (or none of its CPUs allowed) the
  // whole mask, shared by every local rank
  std::vector<int> pool;
  int peers = world, index = rank;
  if (my >= 0) {
    const std::vector<int> nc = node_cpus(my);
    for (int c : aff)
      if (std::find(nc.begin(), nc.end(), c) != nc.end()) pool.push_back(c);
    if (!pool.empty()) {
      peers = 0;
      index = 0;
      for (int r = 0; r < world; ++r)
        if (numa_of[r] == my) {
          if (r < rank) ++index;
          ++peers;
        }
    }
  }
  if (pool.empty()) pool = aff;
  std::vector<int> mine;
  if ((int)pool.size() >= peers) {  // disjoint contiguous slices
    const size_t a = pool.size() * (size_t)index / (size_t)peers, b = pool.size() * (size_t)(index + 1) / (size_t)peers;
    mine.assign(pool.begin() + (long)a, pool.begin() + (long)b);
  } else if (!pool.empty()) {  // fewer CPUs than ranks: one each, shared
    mine.push_back(pool[(size_t)index % pool.size()]);
  }
  int threads = std::max(1, (int)mine.size());
  if (quota > 0) threads = std::min(threads, std::max(1, quota / world));
  threads = std::min(threads, kHostThreadsMax);
  out->threads = threads;
  out->n_cpus = (int32_t)std::min<size_t>(mine.size(), CSM_HOST_PLAN_MAX_CPUS);
  for (int i = 0; i < out->n_cpus; ++i) out->cpus[i] = mine[(size_t)i];
}

// A device's NUMA node from its PCI address (sysfs), -1 when unknown.
int device_numa_node(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return -1;
  for (char* p = bus; *p; ++p) *p = (char)std::tolower((unsigned char)*p);
  char path[160];
  std::snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
  const std::string s = read_file(path);
  return s.empty() ? -1 : std::atoi(s.c_str());
}

// The plan of a context on `device`, local rank `rank` of `world`. The local
// ranks' NUMA nodes: CSM_LOCAL_NUMA (comma-separated, one per local rank) when
// set; else, when every local rank's device is visible here, local rank r
// drives device r (the one-process-per-GPU launch, bench.py / torchrun's
// LOCAL_RANK). When the ranks outnumber the visible devices (each rank's
// HIP_VISIBLE_DEVICES shows its own GPU only) the peers' nodes are unknown:
// the plan then keeps this rank's node and thread share but pins nothing,
// rather than guess which ranks share the node and pin them to overlapping or
// too-small slices.
void context_host_plan(int device, int rank, int world, csm_host_plan* out) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
  world = std::max(1, world);
  rank = std::min(std::max(0, rank), world - 1);
  std::vector<int32_t> numa((size_t)world, -1);
  bool known = false;
  if (const char* env = std::getenv("CSM_LOCAL_NUMA")) {
    int r = 0;
    for (const char* p = env; *p && r < world; ++r) {
      numa[(size_t)r] = (int32_t)std::strtol(p, nullptr, 10);
      while (*p && *p != ',') ++p;
      if (*p == ',') ++p;
    }
    known = r == world;
  }
  if (!known && count >= world) {
    for (int r = 0; r < world; ++r) numa[(size_t)r] = device_numa_node(r);
    known = true;
  }
  if (!known) {
    std::fill(numa.begin(), numa.end(), -1);
    numa[(size_t)rank] = device_numa_node(device);
  }
  host_plan(rank, world, numa.data(), cgroup_quota_cpus(), affinity_cpus(), out);
  if (!known && world > 1) {
    // this rank's node CPUs, shared with an unknown number of peers: the
    // quota's per-rank share of threads, unpinned
    out->n_cpus = 0;
    out->threads = std::max(1, std::min(out->threads, (int)std::max<size_t>(1, affinity_cpus().size() / (size_t)world)));
  }
}

// Pin the calling (worker) thread to a plan's CPUs; nothing when it has none.
void pin_to_plan(const csm_host_plan& p) {
  if (p.n_cpus <= 0) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int i = 0; i < p.n_cpus; ++i)
    if (p.cpus[i] >= 0 && p.cpus[i] < CPU_SETSIZE) CPU_SET(p.cpus[i], &set);
  (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

}  // namespace csmh

extern "C" int csm_host_plan_compute(int32_t local_rank, int32_t local_world, const int32_t* numa_of_rank,
                                     int32_t quota_cpus, csm_host_plan* out) {
  if (!out || local_world <= 0 || local_rank < 0 || local_rank >= local_world) return CSM_ERR_INVALID_ARG;
  csmh::host_plan(local_rank, local_world, numa_of_rank, quota_cpus == 0 ? csmh::cgroup_quota_cpus() : quota_cpus,
                  csmh::affinity_cpus(), out);
  return CSM_OK;
}
