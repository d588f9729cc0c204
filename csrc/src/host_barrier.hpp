// Host-side agreement of the ranks of one device communicator, over one POSIX shared-memory page.
//
// Every rank of a device communicator is a process on the same host (flexar_comm_connect refuses
// anything else), so a page of per-rank monotonic counters is an agreement that needs neither the
// device protocol nor the caller's bootstrap (torch.distributed, MPI, a Store). It keeps working after
// the peers' IPC mappings are closed, which is exactly what the collective teardown needs
// (flexar_comm_destroy: quiesce -> agree -> unmap -> agree -> free; docs/DESIGN.md §21).
//
// Reference counterpart: the reference never frees its scratch (allreduce_over_mpi/mpi_mod.hpp:931-950,
// grow-only and never deleted while in use), so it has no teardown to agree on. Here workspaces are
// freed per communicator; the agreement guarantees that no peer still maps a buffer when it is freed
// and its virtual address can be handed out (and exported) again.
#pragma once

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <string>

#include "flexar/program.hpp"

namespace flexar {

class HostBarrier {
 public:
  static constexpr size_t kPageBytes = 4096;
  struct Page {
    std::atomic<uint64_t> arrived[kMaxRanks];   // phases rank r has reached (1 = joined)
    std::atomic<uint64_t> value[2][kMaxRanks];  // exchange_max payload of rank r, by phase parity
    std::atomic<uint64_t> ident[kMaxRanks];     // mark(): rank r's proof that it wrote into THIS page
  };
  static_assert(sizeof(Page) <= kPageBytes, "one page");
  static_assert(std::atomic<uint64_t>::is_always_lock_free, "cross-process atomics need lock-free words");

  HostBarrier() = default;
  HostBarrier(const HostBarrier&) = delete;
  HostBarrier& operator=(const HostBarrier&) = delete;
  ~HostBarrier() {
    if (page_) munmap(page_, kPageBytes);
  }

  // Opens (creating if needed) the page `name` shared by `nranks` ranks and marks this rank joined.
  bool join(const std::string& name, int rank, int nranks, std::string* err) {
    name_ = name;
    rank_ = rank;
    nranks_ = nranks;
    const int fd = shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0) {
      if (err) *err = "shm_open(" + name + ") failed";
      return false;
    }
    // every rank extends the file to one page; extending to the same size never clears what a faster
    // rank already wrote, and a new file reads as zeros
    if (ftruncate(fd, (off_t)kPageBytes) != 0) {
      close(fd);
      if (err) *err = "ftruncate(" + name + ") failed";
      return false;
    }
    void* p = mmap(nullptr, kPageBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
      if (err) *err = "mmap(" + name + ") failed";
      return false;
    }
    page_ = static_cast<Page*>(p);
    phase_ = 1;
    page_->arrived[rank_].store(phase_, std::memory_order_release);
    return true;
  }

  bool joined() const { return page_ != nullptr; }

  // Is the page really shared by every rank? (One container per rank, or a private /dev/shm, gives each
  // rank its own page of the same name: every agreement would then wait out its timeout at the worst
  // moment, teardown.) Two steps around one bootstrap barrier, so the answer is immediate, not a timeout:
  // mark() writes this rank's identity word (`token`, the same on every rank, mixed with the rank);
  // after every rank has marked (the caller's barrier), shared() checks every rank's word.
  static uint64_t ident_of(uint64_t token, int rank) { return token ^ (0x9E3779B97F4A7C15ull * (uint64_t)(rank + 1)); }
  void mark(uint64_t token) {
    if (page_) page_->ident[rank_].store(ident_of(token, rank_), std::memory_order_release);
  }
  bool shared(uint64_t token, int* missing) const {
    if (!page_) return false;
    for (int r = 0; r < nranks_; ++r)
      if (page_->ident[r].load(std::memory_order_acquire) != ident_of(token, r)) {
        if (missing) *missing = r;
        return false;
      }
    return true;
  }
  const std::string& name() const { return name_; }

  // Next phase: this rank arrives, then waits until every rank has arrived. false = timed out
  // (`*straggler` = the lowest rank that had not arrived). A timed-out barrier leaves this rank's
  // counter advanced, so a late peer passes the phase without waiting for anyone.
  bool arrive_and_wait(uint64_t timeout_ms, int* straggler) {
    if (!page_) return false;
    ++phase_;
    page_->arrived[rank_].store(phase_, std::memory_order_release);
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
      int late = -1;
      for (int r = 0; r < nranks_ && late < 0; ++r)
        if (page_->arrived[r].load(std::memory_order_acquire) < phase_) late = r;
      if (late < 0) return true;
      if (straggler) *straggler = late;
      if (spin < 64) {
        sched_yield();
        continue;
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) return false;
      const timespec ts{0, 20000};  // 20 us: teardown is not latency-critical
      nanosleep(&ts, nullptr);
    }
  }

  // A barrier that also combines one value per rank: the maximum (bor = false) or the bitwise OR (bor =
  // true). The value is published before this rank arrives (release) and read after every rank has
  // (acquire); a rank cannot be two phases ahead of another, so one slot per phase parity never holds a
  // value someone still has to read.
  bool exchange(uint64_t mine, uint64_t* out, uint64_t timeout_ms, int* straggler, bool bor = false) {
    if (!page_) return false;
    const int par = (int)((phase_ + 1) & 1);
    page_->value[par][rank_].store(mine, std::memory_order_relaxed);
    if (!arrive_and_wait(timeout_ms, straggler)) return false;
    uint64_t m = 0;
    for (int r = 0; r < nranks_; ++r) {
      const uint64_t v = page_->value[par][r].load(std::memory_order_relaxed);
      m = bor ? (m | v) : std::max<uint64_t>(m, v);
    }
    if (out) *out = m;
    return true;
  }
  bool exchange_max(uint64_t mine, uint64_t* out, uint64_t timeout_ms, int* straggler) {
    return exchange(mine, out, timeout_ms, straggler, false);
  }

  // Removes the name (existing mappings stay valid); safe to call more than once and from every rank.
  void unlink() {
    if (!name_.empty() && !unlinked_) {
      (void)shm_unlink(name_.c_str());
      unlinked_ = true;
    }
  }

 private:
  Page* page_ = nullptr;
  std::string name_;
  int rank_ = 0, nranks_ = 0;
  uint64_t phase_ = 0;
  bool unlinked_ = false;
};

}  // namespace flexar
