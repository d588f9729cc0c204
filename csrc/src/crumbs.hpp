// Launch breadcrumbs and the fatal-signal report.
//
// Every kernel launch, copy, RCCL group and start-up phase of this process appends one fixed-size record to
// a lock-free host ring (the last kCrumbs events). On a fatal signal (SIGSEGV, SIGBUS, SIGFPE, SIGILL,
// SIGABRT) or std::terminate - e.g. torch's ProcessGroupNCCL watchdog rethrowing an asynchronous
// hipErrorIllegalAddress, which is how the round-4 rehearsal fault surfaced - the handler writes the ring and
// every live communicator's device progress words to stderr with write(2) and then chains to the previous
// handler. The device progress words are host-mapped: workgroup 0 of every executor launch stores the epoch
// it starts and the epoch it finishes, so the report tells which launch was on the device when the process
// died, not only which one was issued last.
//
// Reference counterpart: glog's InstallFailureSignalHandler in the benchmark driver
// (allreduce_over_mpi/benchmark.cpp:62), which prints a stack on a fatal signal; the reference has no
// asynchronous device work, so a stack was enough there.
#pragma once

#include <stdint.h>

namespace flexar {

enum CrumbType : uint8_t { CRUMB_PHASE = 0, CRUMB_LAUNCH = 1, CRUMB_COPY = 2, CRUMB_RCCL = 3, CRUMB_HOST = 4 };

struct CrumbArgs {
  uint8_t type = CRUMB_PHASE;
  uint8_t launch_kind = 0;  // LaunchKind (CRUMB_LAUNCH)
  uint8_t proto = 0;        // executor protocol mode
  uint8_t wire = 0;         // typed program wire
  int16_t rank = -1, nranks = 0;
  int16_t dtype = -1, op = -1;
  uint32_t grid = 0;
  uint64_t epoch = 0;  // device epoch the launch runs as (communicator launch counter + 1), 0 = n/a
  uint64_t bytes = 0;
  const char* what = nullptr;   // kernel or phase name (static string)
  const char* label = nullptr;  // spec / detail (copied, at most 63 bytes)
};

// Appends one record (thread-safe, lock-free, ~50 ns).
void crumb(const CrumbArgs& a);
// Phase shorthand.
void crumb_phase(const char* what, const char* label, int rank = -1, int nranks = 0);

// Live communicators whose host-mapped progress words the report prints: `progress` points at two uint64
// words (workgroup 0's started / finished epoch). Returns the slot (or -1 when the table is full).
int crumb_register_comm(int rank, int nranks, int device, const volatile uint64_t* progress);
void crumb_unregister_comm(int slot);

// FLEXAR_CRASH_REPORT unset or non-zero: breadcrumbs, launch progress words and the report are on.
bool crumbs_on();
// Installs the fatal-signal and terminate handlers once per process (FLEXAR_CRASH_REPORT=0: never).
void crash_report_install();
// Writes the report to fd 2 now (tests, explicit dumps); `why` is printed in the header.
void crash_report_write(const char* why);

}  // namespace flexar
