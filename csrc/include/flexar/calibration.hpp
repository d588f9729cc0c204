// Connect-time calibration of the runtime selector: the cost model's constants
// theta = (alpha_launch_us, alpha_sync_us, 1 / link_gbps, 1 / hbm_gbps) are fitted to executor schedules
// timed on THIS node right after the connect-time self-test, max over ranks, and cached on disk per node
// shape so later processes skip the measurement.
//
// Reference: cost_model/CostModel.h:82-119 scores topologies with hand-set constants (lo, co, bo, o) that
// nothing ever measures, and cost_model/main.cpp prints the argmin for a human to export as FT_TOPO. Here
// the model is the runtime selector itself and its constants come from the machine it runs on.
//
// Host-only (unit-tested on the CPU, tests/test_calibration.py); the device measurement that feeds it is
// flexar_comm_calibrate (csrc/src/comm_connect.hip).
#pragma once

#include <stdint.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "flexar/cost_model.hpp"
#include "flexar/readiness.hpp"

namespace flexar {

// The fixed measurement set: enough distinct (hand-offs, link bytes, HBM bytes) mixes to identify the four
// constants - latency-bound single-hand-off and many-hand-off calls (oneshot, ring at 256 KiB separate
// alpha_launch from alpha_sync), and bandwidth-bound flat / ring / oneshot calls whose link-to-HBM byte
// ratios differ (flat: ~S/N per link per phase, 4.75 S of HBM at N = 8; oneshot: S per link, 2N S of HBM).
struct CalibPoint {
  std::string spec;
  double bytes;
};

// Every schedule family the selector can pick appears at a bandwidth-bound size too: a oneshot measured
// only where it is latency-bound leaves its extra HBM bytes (every rank reduces the whole buffer: (2N + 1) S
// against flat's ~4 S) unpriced, and the selector then picks it for 256 MiB (round-3 rehearsal, N = 2:
// oneshot 533 us where flat+pull takes 430 us).
inline std::vector<CalibPoint> calib_points(int nranks) {
  std::vector<CalibPoint> p = {{"oneshot", 64 << 10},  {"flat+pull", 64 << 10}, {"ring", 256 << 10},
                               {"oneshot", 1 << 20},   {"flat+pull", 4 << 20},  {"flat+pull", 32 << 20},
                               {"ring", 32 << 20},     {"flat+push", 32 << 20}, {"oneshot", 32 << 20}};
  if (nranks > 2 && !(nranks & (nranks - 1))) p.push_back({"rhd+pull", 32 << 20});
  return p;
}

struct CalibRow {
  std::string spec;
  double bytes;
  double us;
};

struct CalibFit {
  double theta[4] = {0, 0, 0, 0};  // alpha_launch_us, alpha_sync_us, 1/link_gbps, 1/hbm_gbps
  double median_rel_err = 0, max_rel_err = 0;
  int rows = 0;
  bool ok = false;
};

// A physical prior on the HBM term: no schedule streams HBM faster than the part's peak (MI355X HBM3E,
// 8 TB/s), so 1 / hbm_gbps >= 1 / kHbmPeakGBps. Without it, calls whose link and HBM byte counts are nearly
// proportional (ranks sharing one device: the "links" ARE the HBM) leave the split between the two terms
// unidentified and the fit may report an unphysical HBM rate (a round-3 rehearsal fitted 12.8 TB/s).
constexpr double kHbmPeakGBps = 8000.0;

// Least squares with theta >= lb on the rows' RELATIVE errors (rows weighted by 1 / measured us): the
// non-negative optimum is the unconstrained optimum of the best support, so with four unknowns every
// support (15 of them) is solved and the best feasible one kept. Columns are scaled to unit max for
// conditioning. Deterministic: every rank fitting the same rows gets bit-identical theta.
inline CalibFit fit_theta(const std::vector<CalibRow>& rows, const XgmiModel& base, int nranks, uint32_t esize = 4) {
  CalibFit out;
  std::vector<std::array<double, 4>> A;
  std::vector<double> y;
  for (const CalibRow& r : rows) {
    if (!(r.us > 0)) continue;
    AlgoSpec s;
    std::string err;
    if (!parse_algo(r.spec, nranks, &s, &err)) continue;
    if (s.kind == AlgoKind::TREE && s.ag == AgMode::AUTO) s.ag = AgMode::PULL;
    double f[4];
    if (!base.features(s, nranks, r.bytes, f, esize)) continue;
    A.push_back({f[0] / r.us, f[1] / r.us, f[2] / r.us, f[3] / r.us});
    y.push_back(1.0);
  }
  out.rows = (int)A.size();
  if (out.rows < 4) return out;
  double scale[4] = {0, 0, 0, 0};
  for (auto& a : A)
    for (int j = 0; j < 4; ++j) scale[j] = std::max(scale[j], std::fabs(a[j]));
  for (int j = 0; j < 4; ++j)
    if (scale[j] <= 0) scale[j] = 1;
  for (auto& a : A)
    for (int j = 0; j < 4; ++j) a[j] /= scale[j];
  // theta = lb + phi with phi >= 0: the lower bounds move to the right-hand side
  const double lb[4] = {0, 0, 0, 1.0 / kHbmPeakGBps};
  for (size_t i = 0; i < A.size(); ++i)
    for (int j = 0; j < 4; ++j) y[i] -= A[i][j] * lb[j] * scale[j];
  double best_res = 1e300;
  for (int mask = 0; mask < 16; ++mask) {
    int idx[4], k = 0;
    for (int j = 0; j < 4; ++j)
      if (mask & (1 << j)) idx[k++] = j;
    // normal equations (k x k) by Gaussian elimination with partial pivoting
    double M[4][5] = {};
    for (size_t i = 0; i < A.size(); ++i)
      for (int a = 0; a < k; ++a) {
        for (int b = 0; b < k; ++b) M[a][b] += A[i][idx[a]] * A[i][idx[b]];
        M[a][k] += A[i][idx[a]] * y[i];
      }
    bool singular = false;
    for (int c = 0; c < k && !singular; ++c) {
      int piv = c;
      for (int r = c + 1; r < k; ++r)
        if (std::fabs(M[r][c]) > std::fabs(M[piv][c])) piv = r;
      if (std::fabs(M[piv][c]) < 1e-14) { singular = true; break; }
      for (int j = 0; j <= k; ++j) std::swap(M[c][j], M[piv][j]);
      for (int r = 0; r < k; ++r) {
        if (r == c) continue;
        const double m = M[r][c] / M[c][c];
        for (int j = c; j <= k; ++j) M[r][j] -= m * M[c][j];
      }
    }
    if (singular) continue;
    double t[4] = {0, 0, 0, 0};  // phi (scaled)
    bool feasible = true;
    for (int a = 0; a < k; ++a) {
      t[idx[a]] = M[a][k] / M[a][a];
      if (t[idx[a]] < 0) feasible = false;
    }
    if (!feasible) continue;
    double res = 0;
    for (size_t i = 0; i < A.size(); ++i) {
      double p = 0;
      for (int j = 0; j < 4; ++j) p += A[i][j] * t[j];
      res += (p - y[i]) * (p - y[i]);
    }
    if (res < best_res) {
      best_res = res;
      for (int j = 0; j < 4; ++j) out.theta[j] = lb[j] + t[j] / scale[j];
      out.ok = true;
    }
  }
  if (!out.ok) return out;
  std::vector<double> rel;
  for (size_t i = 0; i < A.size(); ++i) {
    double p = 0;
    for (int j = 0; j < 4; ++j) p += A[i][j] * scale[j] * out.theta[j];  // = predicted / measured
    rel.push_back(std::fabs(p - 1.0));
  }
  std::sort(rel.begin(), rel.end());
  out.median_rel_err = rel[rel.size() / 2];
  out.max_rel_err = rel.back();
  return out;
}

// theta -> the model's parameters (a constant the data never exercised, fitted to 0, keeps a finite
// bandwidth); links and the copy-engine terms stay as they were.
inline XgmiModel model_with_theta(XgmiModel m, const double theta[4]) {
  m.alpha_launch_us = theta[0];
  m.alpha_sync_us = theta[1];
  m.link_gbps = theta[2] > 1e-12 ? 1.0 / theta[2] : 1e6;
  m.hbm_gbps = theta[3] > 1e-12 ? 1.0 / theta[3] : 1e6;
  return m;
}

// ---- on-disk cache -------------------------------------------------------------------------------
// Keyed by what the constants depend on: GPU architecture, world size, the agreed link count, the link
// classes seen (ranks sharing a device time the shared HBM, not links), the protocol families the
// self-test disabled, the library version and the measurement set's revision.
constexpr int kCalibRevision = 3;  // 2: oneshot at 32 MiB joined the set; 3: HBM term bounded by the peak

inline std::string calib_key(const std::string& arch, int nranks, int links, const std::string& link_classes,
                             uint32_t disabled, const std::string& version) {
  std::ostringstream k;
  k << "arch=" << arch << ";n=" << nranks << ";links=" << links << ";classes=" << link_classes
    << ";disabled=" << disabled << ";flexar=" << version << ";rev=" << kCalibRevision;
  return k.str();
}

// FLEXAR_CALIB_DIR, else $XDG_CACHE_HOME/flexar, else $HOME/.cache/flexar ("" = no cache directory)
inline std::string calib_dir() {
  if (const char* d = getenv("FLEXAR_CALIB_DIR")) return d;
  if (const char* x = getenv("XDG_CACHE_HOME")) if (*x) return std::string(x) + "/flexar";
  if (const char* h = getenv("HOME")) if (*h) return std::string(h) + "/.cache/flexar";
  return "";
}

inline std::string calib_path(const std::string& dir, const std::string& key) {
  char name[64];
  snprintf(name, sizeof(name), "calib-%016llx.txt", (unsigned long long)fnv1a(key));
  return dir + "/" + name;
}

// File: line 1 the key, line 2 the four theta values (%.17g: bit-exact round trip), then the rows as
// "spec bytes us" for the record. A key mismatch (hash collision, edited file) is a miss.
inline bool calib_load(const std::string& path, const std::string& key, double theta[4]) {
  std::ifstream f(path);
  if (!f) return false;
  std::string k, vals;
  if (!std::getline(f, k) || k != key || !std::getline(f, vals)) return false;
  std::istringstream ss(vals);
  double t[4];
  for (int j = 0; j < 4; ++j)
    if (!(ss >> t[j]) || !std::isfinite(t[j]) || t[j] < 0) return false;
  for (int j = 0; j < 4; ++j) theta[j] = t[j];
  return true;
}

inline bool calib_store(const std::string& path, const std::string& key, const double theta[4],
                        const std::vector<CalibRow>& rows) {
  const size_t slash = path.rfind('/');
  if (slash != std::string::npos) {  // mkdir -p
    std::string d = path.substr(0, slash);
    for (size_t i = 1; i <= d.size(); ++i)
      if (i == d.size() || d[i] == '/') (void)mkdir(d.substr(0, i).c_str(), 0755);
  }
  const std::string tmp = path + ".tmp." + std::to_string((long)getpid());
  {
    std::ofstream f(tmp);
    if (!f) return false;
    char line[256];
    f << key << "\n";
    snprintf(line, sizeof(line), "%.17g %.17g %.17g %.17g\n", theta[0], theta[1], theta[2], theta[3]);
    f << line;
    for (const CalibRow& r : rows) {
      snprintf(line, sizeof(line), "%s %.0f %.6g\n", r.spec.c_str(), r.bytes, r.us);
      f << line;
    }
    if (!f) return false;
  }
  return rename(tmp.c_str(), path.c_str()) == 0;  // atomic: a concurrent reader sees the old file or the new
}

}  // namespace flexar
