// Internal interface of the host SHA-256 (sha256_host.cpp) for the pipeline and the C ABI.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <mutex>

#include "../../include/cess_ec.h"

namespace hsha {

// n chains of `len` bytes: chain i reads bufs[i]; its hex goes to
// hex + ((i / per) * hex_outer + i % per) * 64, and with prefix_len (a multiple of 64) the hex of
// its first prefix_len bytes to prefix_hex + ((i / per) * prefix_outer + i % per) * 64.
struct Job {
  const uint8_t* const* bufs = nullptr;
  size_t n = 0, len = 0;
  uint8_t* hex = nullptr;
  size_t per = 1, hex_outer = 1;
  size_t prefix_len = 0;
  uint8_t* prefix_hex = nullptr;
  size_t prefix_outer = 1;
  // optional: the 8 state words of chain i after its full blocks (before the padding) to
  // state_out + 8 i (a segment chain resumed elsewhere after its first len bytes)
  uint32_t* state_out = nullptr;
};

struct JobState {
  Job job;
  int form = 0;
  size_t next = 0;      // next chain to hand out (under the pool's lock)
  size_t per_task = 1;  // groups per task (forms other than x16)
  std::atomic<int> left{0};  // chains (x16) or tasks not yet finished
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
};

void hash_range(const Job& j, size_t c0, size_t n, int form);
// Queue a job on the process-wide pool (grown to `threads` workers). The job's pointers must stay
// valid until it is ready.
std::shared_ptr<JobState> submit(const Job& job, int threads);
bool ready(const std::shared_ptr<JobState>& js);
// Block until the job is done (the second argument is unused: the workers do all hashing).
void wait(const std::shared_ptr<JobState>& js, bool help);

// Thread reservations of long-lived users (a host-hashing pipeline reserves its host_threads at
// creation, releases them at destruction): the pool grows to the sum of the live reservations.
void reserve_threads(int n);
void release_threads(int n);
int pool_threads();

// Cumulative counters of the pool's workers (diagnostics: the pipeline's CEC_PIPELINE_TRACE).
struct PoolStats {
  double busy_s = 0;          // worker time spent hashing
  uint64_t lane_blocks = 0;   // blocks hashed by lane steps (x16 and SHA-NI lane steps)
  uint64_t x16_steps = 0, ni_steps = 0, x16_lane_steps = 0;  // steps, and lanes used by x16 ones
  uint64_t spilled = 0;       // chains given back to idle workers
};
PoolStats stats();

}  // namespace hsha
