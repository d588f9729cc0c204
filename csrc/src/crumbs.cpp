// Launch breadcrumbs and the fatal-signal report (crumbs.hpp). Host-only; everything the handlers call is
// async-signal-safe: write(2), clock_gettime, atomics and a hand-written integer formatter (no stdio, no
// allocation), so the report also comes out of a SIGSEGV or an abort() inside another library.
#include "crumbs.hpp"

#include <signal.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <exception>

#include "flexar/flexar.h"
#include "flexar/types.hpp"

namespace flexar {

namespace {

constexpr uint32_t kCrumbs = 256;      // ring size (a power of two)
constexpr uint32_t kReportLast = 48;   // records printed, newest last
constexpr int kMaxLiveComms = 64;

struct Crumb {
  std::atomic<uint64_t> seq;  // 0 = empty / being written; written last (release)
  uint64_t t_ns;
  uint32_t tid;
  uint8_t type, launch_kind, proto, wire;
  int16_t rank, nranks, dtype, op;
  uint32_t grid;
  uint64_t epoch, bytes;
  const char* what;
  char label[64];
};

Crumb g_ring[kCrumbs];
std::atomic<uint64_t> g_next{1};

struct LiveComm {
  std::atomic<const volatile uint64_t*> progress{nullptr};
  int rank = 0, nranks = 0, device = 0;
};
LiveComm g_live[kMaxLiveComms];

uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// ---- async-signal-safe output ---------------------------------------------------------------------
struct Out {
  char buf[512];
  size_t n = 0;
  void flush() {
    size_t off = 0;
    while (off < n) {
      const ssize_t w = ::write(2, buf + off, n - off);
      if (w <= 0) break;
      off += (size_t)w;
    }
    n = 0;
  }
  Out& s(const char* x) {
    if (!x) x = "(null)";
    for (; *x; ++x) {
      if (n == sizeof(buf)) flush();
      buf[n++] = *x;
    }
    return *this;
  }
  Out& u(uint64_t v) {
    char t[24];
    int k = 0;
    do { t[k++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (k) {
      if (n == sizeof(buf)) flush();
      buf[n++] = t[--k];
    }
    return *this;
  }
  Out& i(int64_t v) {
    if (v < 0) { s("-"); return u((uint64_t)(-v)); }
    return u((uint64_t)v);
  }
  // milliseconds with three decimals
  Out& ms(uint64_t ns) {
    u(ns / 1000000ull).s(".");
    const uint64_t f = (ns / 1000ull) % 1000ull;
    if (f < 100) s("0");
    if (f < 10) s("0");
    return u(f);
  }
};

const char* launch_kind_name(int k) {
  static const char* n[] = {"exec", "exec-group", "reduce", "ll", "ll-group", "query"};
  return (k >= 0 && k < 6) ? n[k] : "?";
}
const char* proto_name(int p) { return p == 2 ? "wt" : p == 1 ? "nts" : "fence"; }
const char* type_name(int t) {
  static const char* n[] = {"phase", "launch", "copy", "rccl", "host"};
  return (t >= 0 && t < 5) ? n[t] : "?";
}

std::atomic<int> g_reported{0};
std::atomic<int> g_installed{0};
struct sigaction g_old[32];
std::terminate_handler g_old_terminate = nullptr;
const int kSignals[] = {SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGABRT};

const char* signal_name(int sig) {
  switch (sig) {
    case SIGSEGV: return "SIGSEGV";
    case SIGBUS: return "SIGBUS";
    case SIGFPE: return "SIGFPE";
    case SIGILL: return "SIGILL";
    case SIGABRT: return "SIGABRT";
    default: return "signal";
  }
}

void report_once(const char* why) {
  int expected = 0;
  if (!g_reported.compare_exchange_strong(expected, 1)) return;  // one report per process
  crash_report_write(why);
}

void on_signal(int sig, siginfo_t* info, void* uctx) {
  report_once(signal_name(sig));
  // chain: the previous handler (Python's faulthandler, a sanitizer, the default action)
  struct sigaction& old = g_old[sig];
  if (old.sa_flags & SA_SIGINFO) {
    if (old.sa_sigaction) {
      old.sa_sigaction(sig, info, uctx);
      return;
    }
  } else if (old.sa_handler != SIG_DFL && old.sa_handler != SIG_IGN) {
    old.sa_handler(sig);
    return;
  }
  // default action: restore it and re-raise (delivered when this handler returns)
  struct sigaction dfl;
  memset(&dfl, 0, sizeof(dfl));
  dfl.sa_handler = SIG_DFL;
  sigemptyset(&dfl.sa_mask);
  sigaction(sig, &dfl, nullptr);
  raise(sig);
}

void on_terminate() {
  report_once("std::terminate (an uncaught C++ exception, e.g. torch's ProcessGroupNCCL watchdog)");
  if (g_old_terminate) g_old_terminate();
  std::abort();
}

// A per-thread alternate signal stack: the handlers are installed with SA_ONSTACK, and a
// SIGSEGV from a stack overflow cannot run on the stack that overflowed. The installing thread gets one in
// crash_report_install and every thread that records a breadcrumb (every thread that launches flexar work)
// lazily in crumb(); a thread that already has one (Python's faulthandler, a sanitizer) keeps it. Freed at
// thread exit. 64 KiB: the report needs a few hundred bytes of frames plus its 512-byte line buffer.
struct AltStack {
  void* mem = nullptr;
  ~AltStack() {
    if (!mem) return;
    stack_t cur;
    if (sigaltstack(nullptr, &cur) == 0 && cur.ss_sp == mem) {
      stack_t off;
      memset(&off, 0, sizeof(off));
      off.ss_flags = SS_DISABLE;
      sigaltstack(&off, nullptr);
    }
    free(mem);
  }
};
void ensure_altstack() {
  static thread_local bool done = false;
  static thread_local AltStack mine;
  if (done) return;
  done = true;
  stack_t cur;
  if (sigaltstack(nullptr, &cur) == 0 && !(cur.ss_flags & SS_DISABLE)) return;  // the thread has one already
  constexpr size_t kAltStackBytes = 64 * 1024;
  void* m = malloc(kAltStackBytes);
  if (!m) return;
  stack_t ss;
  memset(&ss, 0, sizeof(ss));
  ss.ss_sp = m;
  ss.ss_size = kAltStackBytes;
  if (sigaltstack(&ss, nullptr) == 0) mine.mem = m;
  else free(m);
}

}  // namespace

bool crumbs_on() {
  static const bool on = [] {
    const char* e = getenv("FLEXAR_CRASH_REPORT");
    return !(e && *e == '0');
  }();
  return on;
}

void crumb(const CrumbArgs& a) {
  if (!crumbs_on()) return;  // FLEXAR_CRASH_REPORT=0: no ring, no report
  if (g_installed.load(std::memory_order_relaxed)) ensure_altstack();
  const uint64_t s = g_next.fetch_add(1, std::memory_order_relaxed);
  Crumb& c = g_ring[s & (kCrumbs - 1)];
  c.seq.store(0, std::memory_order_relaxed);
  std::atomic_signal_fence(std::memory_order_seq_cst);
  c.t_ns = now_ns();
  static thread_local const uint32_t tid = (uint32_t)syscall(SYS_gettid);  // once per thread: no syscall per launch
  c.tid = tid;
  c.type = a.type;
  c.launch_kind = a.launch_kind;
  c.proto = a.proto;
  c.wire = a.wire;
  c.rank = a.rank;
  c.nranks = a.nranks;
  c.dtype = a.dtype;
  c.op = a.op;
  c.grid = a.grid;
  c.epoch = a.epoch;
  c.bytes = a.bytes;
  c.what = a.what;
  size_t k = 0;
  if (a.label)
    for (; k + 1 < sizeof(c.label) && a.label[k]; ++k) c.label[k] = a.label[k];
  c.label[k] = 0;
  c.seq.store(s, std::memory_order_release);
}

void crumb_phase(const char* what, const char* label, int rank, int nranks) {
  CrumbArgs a;
  a.type = CRUMB_PHASE;
  a.what = what;
  a.label = label;
  a.rank = (int16_t)rank;
  a.nranks = (int16_t)nranks;
  crumb(a);
}

// A slot is claimed with a sentinel first (a concurrent registration cannot claim it too), then filled, then
// published with a release store - the report (which skips the sentinel) never pairs one communicator's
// progress words with another's rank / device.
static const volatile uint64_t kClaimed[2] = {0, 0};
int crumb_register_comm(int rank, int nranks, int device, const volatile uint64_t* progress) {
  for (int i = 0; i < kMaxLiveComms; ++i) {
    const volatile uint64_t* expected = nullptr;
    if (g_live[i].progress.load(std::memory_order_relaxed) != nullptr) continue;
    if (!g_live[i].progress.compare_exchange_strong(expected, kClaimed, std::memory_order_acquire)) continue;
    g_live[i].rank = rank;
    g_live[i].nranks = nranks;
    g_live[i].device = device;
    g_live[i].progress.store(progress, std::memory_order_release);
    return i;
  }
  return -1;
}

void crumb_unregister_comm(int slot) {
  if (slot >= 0 && slot < kMaxLiveComms) g_live[slot].progress.store(nullptr, std::memory_order_release);
}

void crash_report_write(const char* why) {
  Out o;
  const uint64_t t = now_ns();
  o.s("\n[flexar crash report] pid ").u((uint64_t)getpid()).s(": ").s(why).s("\n");
  // device progress of every live communicator (host-mapped words written by executor workgroup 0)
  for (int i = 0; i < kMaxLiveComms; ++i) {
    const volatile uint64_t* p = g_live[i].progress.load(std::memory_order_acquire);
    if (!p || p == kClaimed) continue;
    o.s("[flexar crash report]   communicator rank ").i(g_live[i].rank).s("/").i(g_live[i].nranks).s(" device ")
        .i(g_live[i].device).s(": executor workgroup 0 started epoch ").u(p[0]).s(", finished epoch ").u(p[1])
        .s(" (launches of >= FLEXAR_PROGRESS_MIN_BYTES, default 1 MiB)\n");
  }
  // newest records: find the highest sequence, walk back
  uint64_t hi = g_next.load(std::memory_order_acquire);
  const uint64_t lo = hi > kReportLast ? hi - kReportLast : 1;
  if (hi <= 1) o.s("[flexar crash report]   no flexar events recorded in this process\n");
  else o.s("[flexar crash report]   last flexar events, oldest first (age = ms before this report):\n");
  for (uint64_t s = lo; s < hi; ++s) {
    const Crumb& c = g_ring[s & (kCrumbs - 1)];
    if (c.seq.load(std::memory_order_acquire) != s) continue;  // overwritten or being written
    o.s("[flexar crash report]   #").u(s).s(" -").ms(t > c.t_ns ? t - c.t_ns : 0).s(" ms tid ").u(c.tid).s(" ")
        .s(type_name(c.type));
    if (c.rank >= 0) o.s(" rank ").i(c.rank).s("/").i(c.nranks);
    o.s(" ").s(c.what ? c.what : "");
    if (c.type == CRUMB_LAUNCH) {
      o.s(" kernel=").s(launch_kind_name(c.launch_kind)).s(" proto=").s(proto_name(c.proto));
      if (c.wire) o.s(" wire=").u(c.wire);
      if (c.dtype >= 0) o.s(" ").s(dtype_name(c.dtype)).s("/").s(op_name(c.op));
      o.s(" grid=").u(c.grid);
    }
    if (c.epoch) o.s(" epoch=").u(c.epoch);
    if (c.bytes) o.s(" bytes=").u(c.bytes);
    if (c.label[0]) o.s(" [").s(c.label).s("]");
    o.s("\n");
  }
  o.s("[flexar crash report] end\n");
  o.flush();
}

void crash_report_install() {
  int expected = 0;
  if (!g_installed.compare_exchange_strong(expected, 1)) return;
  if (!crumbs_on()) return;
  ensure_altstack();
  for (int sig : kSignals) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = on_signal;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(sig, &sa, &g_old[sig]);
  }
  g_old_terminate = std::set_terminate(on_terminate);
}

}  // namespace flexar

extern "C" {

void flexar_crumb(const char* what, const char* label, int rank, int nranks, uint64_t epoch, uint64_t bytes) {
  flexar::CrumbArgs a;
  a.type = flexar::CRUMB_PHASE;
  a.what = nullptr;
  // the caller's `what` may be a temporary (Python bytes): keep it in the copied label
  char buf[64];
  size_t k = 0;
  for (const char* p = what; p && *p && k + 1 < sizeof(buf); ++p) buf[k++] = *p;
  if (label && *label && k + 3 < sizeof(buf)) {
    buf[k++] = ':';
    buf[k++] = ' ';
    for (const char* p = label; *p && k + 1 < sizeof(buf); ++p) buf[k++] = *p;
  }
  buf[k] = 0;
  a.label = buf;
  a.rank = (int16_t)rank;
  a.nranks = (int16_t)nranks;
  a.epoch = epoch;
  a.bytes = bytes;
  flexar::crumb(a);
}

void flexar_crash_report_install(void) { flexar::crash_report_install(); }

void flexar_crash_report_dump(const char* why) { flexar::crash_report_write(why ? why : "explicit dump"); }

// Tests only: end the process the way an uncaught C++ exception (kind 0: std::terminate) or abort() (1) does.
// kind 2: a stack overflow by unbounded recursion (the SIGSEGV then arrives on an exhausted stack).
static int overflow_stack(volatile int depth) {
  volatile char pad[4096];
  pad[0] = (char)depth;
  pad[sizeof(pad) - 1] = (char)(depth >> 8);
  return overflow_stack(depth + 1) + pad[0] + pad[sizeof(pad) - 1];  // not a tail call
}
void flexar_test_fatal(int kind) {
  if (kind == 0) std::terminate();
  if (kind == 2) (void)overflow_stack(0);
  std::abort();
}

}  // extern "C"
