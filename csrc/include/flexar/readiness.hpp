// Connect-time readiness of a communicator: which device protocol families passed the exact
// self-test, how a requested algorithm is rewritten onto a verified family (the downgrade chain),
// the per-peer link classes found by the topology probe, and the fingerprint of the settings every
// rank must agree on.
//
// Reference counterpart: the per-communicator setup of FlexTree_Context (allreduce_over_mpi/
// mpi_mod.hpp:216-243) reads the communicator shape and trusts the transport. MPI_Isend/Irecv never
// fail silently; the device protocols here can (a cross-device visibility bug would corrupt sums
// without hanging), so every protocol family is verified on the real links before a production call
// may use it, and the machine shape (the reference's hostfile and fan-in penalty,
// mpi_config_file:1-16, cost_model/CostModel.h:1-20) is probed instead of assumed.
// Host-only: unit-tested on the CPU (tests/test_readiness.py).
#pragma once

#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>

#include "flexar/topology.hpp"

namespace flexar {

// Protocol families. Every algorithm runs on exactly one of them.
enum : uint32_t {
  PF_FENCE = 1,  // executor, plain stores + system release/acquire (default, "+nts" included)
  PF_WT = 2,     // executor, write-through payload ("+wt")
  PF_LL = 4,     // flag-free {data, epoch} granules ("ll")
  PF_DMA = 8,    // copy engines + stream-ordered flag writes ("dma")
  PF_ALL = 15,
  PF_MSG = 16    // message transport: RCCL send/recv + local executor segments ("+rccl")
};

inline uint32_t proto_family(const AlgoSpec& s) {
  if (s.msg) return PF_MSG;
  switch (s.kind) {
    case AlgoKind::LL: return PF_LL;
    case AlgoKind::DMA: return PF_DMA;
    default: return s.wt ? PF_WT : PF_FENCE;
  }
}

inline std::string family_names(uint32_t mask) {
  static const char* n[] = {"fence", "wt", "ll", "dma", "rccl"};
  std::string s;
  for (int i = 0; i < 5; ++i)
    if (mask & (1u << i)) s += (s.empty() ? "" : ",") + std::string(n[i]);
  return s.empty() ? "none" : s;
}

// Rewrite `s` onto a family that is not in `disabled`, keeping the schedule where possible:
//   ll    -> oneshot (same single hop, flag hand-off instead of granules)
//   fence -> the same schedule with "+wt"
//   wt    -> dma (the flat exchange on the copy engines) when the spec is an allreduce schedule
//   dma   -> flat+pull on the executor (fence, then wt)
//   any IPC family -> the same schedule over the message transport when every IPC route is gone and
//   the transport exists (allow_msg)
// Returns false (and says why) when no verified family is left for this call.
inline bool downgrade_spec(AlgoSpec* s, int nranks, uint32_t disabled, bool allow_dma, std::string* why,
                           bool allow_msg = false) {
  disabled &= PF_ALL | PF_MSG;
  const AlgoSpec orig = *s;
  for (int hop = 0; hop < 6; ++hop) {
    const uint32_t f = proto_family(*s);
    if (!(disabled & f)) return true;
    if (f == PF_MSG) break;
    if (allow_msg && !(disabled & PF_MSG) && (disabled & (PF_FENCE | PF_WT)) == (PF_FENCE | PF_WT) &&
        (!allow_dma || (disabled & PF_DMA))) {
      *s = orig;  // every peer-memory route failed: same schedule, bytes over send/recv
      s->msg = true;
      s->wt = s->nts = false;
      if (s->kind == AlgoKind::LL) s->kind = AlgoKind::ONESHOT;
      if (s->kind == AlgoKind::DMA) *s = AlgoSpec(), s->kind = AlgoKind::TREE, s->widths = {nranks}, s->msg = true;
      return true;
    }
    switch (f) {
      case PF_LL: s->kind = AlgoKind::ONESHOT; break;
      case PF_FENCE: s->wt = true; s->nts = false; break;
      case PF_WT:
        if (allow_dma && !(disabled & PF_DMA)) {
          *s = AlgoSpec();
          s->kind = AlgoKind::DMA;
        } else {
          if (why) *why = "no verified device protocol for " + s->str() + " (failed self-test: " +
                          family_names(disabled) + ")";
          return false;
        }
        break;
      case PF_DMA:
        *s = AlgoSpec();
        s->kind = AlgoKind::TREE;
        s->ag = AgMode::PULL;
        s->widths = {nranks};
        break;
    }
  }
  if (why) *why = "no verified device protocol (failed self-test: " + family_names(disabled) + ")";
  return false;
}

// ---- per-peer link classes (topology probe) ----------------------------------------------------
enum : int32_t {
  LINK_UNKNOWN = 0,  // peer device not visible in this process (e.g. HIP_VISIBLE_DEVICES): IPC only
  LINK_SAME = 1,     // the same GPU (ranks sharing a device: one HBM, no link)
  LINK_XGMI = 2,     // xGMI, hop count in `hops`
  LINK_PCIE = 3,     // PCIe peer-to-peer
  LINK_OTHER = 4
};

inline const char* link_name(int32_t k) {
  switch (k) {
    case LINK_SAME: return "same-device";
    case LINK_XGMI: return "xgmi";
    case LINK_PCIE: return "pcie";
    case LINK_OTHER: return "other";
    default: return "unknown";
  }
}

// HSA link types (hsa_ext_amd.h HSA_AMD_LINK_INFO_TYPE_*) reported by hipExtGetLinkTypeAndHopCount.
inline int32_t link_class_of_hsa(uint32_t hsa_type) {
  switch (hsa_type) {
    case 4: return LINK_XGMI;
    case 2: return LINK_PCIE;
    default: return LINK_OTHER;
  }
}

// Direct xGMI links to drive concurrently for the cost model: the number of peers one xGMI hop away
// (7 on a fully connected 8-GPU node), at least 1. Ranks on the same device count as one "link"
// (the shared HBM); unknown peers count as direct links.
inline int direct_links(const int32_t* cls, const int32_t* hops, int n, int self) {
  int x = 0;
  for (int p = 0; p < n; ++p) {
    if (p == self) continue;
    if ((cls[p] == LINK_XGMI && hops[p] <= 1) || cls[p] == LINK_UNKNOWN) ++x;
  }
  return x < 1 ? 1 : x;
}

// ---- probe agreement ----------------------------------------------------------
// The link count that prices schedules comes from each rank's OWN probe. The reference derives its
// geometry from the communicator alone, identically on every rank (mpi_mod.hpp:216-243); here the probe
// results are exchanged after connect and agreed on, so ranks cannot select different schedules (which
// would surface as a device watchdog timeout in the first collective):
//  * every rank installs the MINIMUM of the ranks' direct-link counts (a conservative, identical value);
//  * the link classes must be symmetric - rank r's view of rank p equals p's view of r wherever both
//    see each other (UNKNOWN = not visible in that process: no claim) - and a rank that sees a peer as
//    the same device must be seen the same way; anything else is a real disagreement about the machine
//    and connect fails with a message naming both ranks and both views;
//  * the post-probe settings fingerprint must match (FLEXAR_MODEL fixing the link count included).
struct ProbeBlob {
  uint32_t magic;
  int32_t rank;
  int32_t links;          // this rank's direct_links()
  int32_t links_fixed;    // FLEXAR_MODEL fixed the link count (the probe does not override it)
  uint64_t fingerprint;   // settings fingerprint, recomputed after the probe
  int8_t cls[16];         // link class of every peer as this rank sees it
  int8_t hops[16];
  int32_t resident;       // executor workgroups this rank's GPU keeps resident (0 = unknown)
  int32_t reserved;
};
constexpr uint32_t kProbeMagic = 0xF1E8B10Bu;

// Returns true and the agreed link count, or false with a message naming the disagreement.
// `resident_out` (optional): the minimum of the ranks' known resident-workgroup counts (0 = none known) -
// the grid clamp must be the same on every rank, or the per-workgroup flag protocol pairs workgroups that
// do not exist on the peer.
inline bool probe_agree(const ProbeBlob* all, int nranks, int* links_out, std::string* why,
                        int* resident_out = nullptr) {
  int links = 1 << 30, resident = 0;
  for (int r = 0; r < nranks; ++r) {
    const ProbeBlob& a = all[r];
    if (a.magic != kProbeMagic || a.rank != r) {
      if (why) *why = "probe summary of rank " + std::to_string(r) + " is malformed";
      return false;
    }
    if (a.fingerprint != all[0].fingerprint || a.links_fixed != all[0].links_fixed) {
      if (why) *why = "rank " + std::to_string(r) + " resolves calls with different settings than rank 0 after the "
                      "topology probe (FLEXAR_MODEL, FLEXAR_PARTIALS or another selector setting differs)";
      return false;
    }
    links = std::min(links, (int)a.links);
    if (a.resident > 0) resident = resident ? std::min(resident, (int)a.resident) : (int)a.resident;
    for (int p = 0; p < nranks; ++p) {
      if (p == r) continue;
      const int8_t rp = a.cls[p], pr = all[p].cls[r];
      if (rp == LINK_UNKNOWN || pr == LINK_UNKNOWN) continue;
      if (rp != pr) {
        if (why)
          *why = "ranks disagree on the machine shape: rank " + std::to_string(r) + " sees rank " + std::to_string(p) +
                 " over " + link_name(rp) + " but rank " + std::to_string(p) + " sees rank " + std::to_string(r) +
                 " over " + link_name(pr);
        return false;
      }
    }
  }
  if (links_out) *links_out = links < 1 ? 1 : links;
  if (resident_out) *resident_out = resident;
  return true;
}

// ---- settings fingerprint ----------------------------------------------------------------------
// Every rank must resolve a call to the same schedule, pieces and grid. Those follow from these
// settings (plus the loaded tune table, hashed by the caller as `extra`); a difference is rejected at
// connect time instead of surfacing as a device timeout in the first collective (FNV-1a over
// "name=value;").
inline uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}
inline const char* const* fingerprint_vars() {
  static const char* v[] = {"FLEXAR_ALGO",     "FT_TOPO",          "FLEXAR_CHUNK_BYTES", "FLEXAR_NCHANNELS",
                            "FLEXAR_MAX_GRID", "FLEXAR_MIN_BLOCK_BYTES", "FLEXAR_MODEL",
                            "FLEXAR_SELFTEST", "FLEXAR_ZC_AUTO", "FLEXAR_PARTIALS", "FLEXAR_CALIB",
                            "FLEXAR_EXEC_INTERLEAVE", nullptr};
  return v;
}
// FLEXAR_CALIB as the mode it selects: unset and "1" behave the same, "off" is "0", "2" is "force".
inline std::string calib_mode_name(const char* e) {
  const std::string v = e ? e : "";
  if (v == "0" || v == "off") return "0";
  if (v == "force" || v == "2") return "force";
  return "1";
}
// `with_calib` = false: the fingerprint the calibration cache is keyed by - the calibration mode decides
// whether the cache is read, not what a schedule costs, so a forced run writes the cache default runs read
// (ADVICE r3). Ranks still agree on the (normalised) mode through the connect-time fingerprint.
inline uint64_t env_fingerprint(const std::string& extra, bool with_calib = true) {
  uint64_t h = fnv1a(extra);
  for (const char* const* v = fingerprint_vars(); *v; ++v) {
    const bool calib = !strcmp(*v, "FLEXAR_CALIB");
    if (calib && !with_calib) continue;
    const char* e = getenv(*v);
    h = fnv1a(std::string(*v) + "=" + (calib ? calib_mode_name(e) : std::string(e ? e : "")) + ";", h);
  }
  return h;
}

}  // namespace flexar
