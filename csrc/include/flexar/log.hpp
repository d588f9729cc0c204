// Minimal logger (reference used glog: LOG / LOG_IF / CHECK_GE, benchmark.cpp:58-62, and raw
// std::cout under FT_DEBUG, mpi_mod.hpp:32). Level from FLEXAR_LOG_LEVEL=error|warn|info|debug
// (default warn); messages go to stderr prefixed with the rank.
#pragma once

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace flexar {

enum LogLevel { LOG_ERROR = 0, LOG_WARN = 1, LOG_INFO = 2, LOG_DEBUG = 3 };

inline int log_level() {
  static int lvl = [] {
    const char* e = getenv("FLEXAR_LOG_LEVEL");
    if (!e) return (int)LOG_WARN;
    if (!strcmp(e, "error")) return (int)LOG_ERROR;
    if (!strcmp(e, "info")) return (int)LOG_INFO;
    if (!strcmp(e, "debug")) return (int)LOG_DEBUG;
    return (int)LOG_WARN;
  }();
  return lvl;
}

inline void logf(int level, int rank, const char* fmt, ...) {
  if (level > log_level()) return;
  static const char* tag[] = {"E", "W", "I", "D"};
  char buf[2048];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  fprintf(stderr, "[flexar %s r%d] %s\n", tag[level], rank, buf);
}

}  // namespace flexar
