// flexar MPI compatibility layer: MPI_Allreduce_FT for MPI applications.
//
// Reference: allreduce_over_mpi/mpi_mod.hpp (the whole header), whose entry
//   int MPI_Allreduce_FT(const void*, void*, int, MPI_Datatype, MPI_Op, MPI_Comm)
// (mpi_mod.hpp:1167-1221) reduces HOST buffers with MPI_Isend/Irecv +
// MPI_Barrier per stage + an OpenMP reduce, topology from FT_TOPO.
//
// Same signature and FT_TOPO semantics here, new mechanics:
//  * DEVICE buffers (hipMalloc'd): routed to the flexar GPU communicator —
//    workspaces exchanged once with MPI_Allgather, then one executor kernel
//    per call over xGMI (see flexar.h). Cached per MPI_Comm (attribute).
//  * HOST buffers, all ranks on one node: the same op programs executed by the
//    host engine (host_exec.hpp) over an MPI-3 shared-memory window — direct
//    loads/stores into peers' staging + atomic epoch flags; no barriers.
//  * HOST buffers across nodes: the push-form op program translated to
//    point-to-point messages, ONE coalesced message per (peer, stage) instead
//    of one MPI_Isend per block (reference defect: mpi_mod.hpp:679-702).
// Fixed reference defects: D1 (leaked requests), D2 (OOB src table), D3
// (fan-in > 20 garbage), D4 (FT_TOPO trailing separator), D7 (count is still
// `int` in the compatible signature; MPI_Allreduce_FT_large takes size_t),
// D8 (per-call allocations/getenv: plans and windows are cached).
// Define FLEXAR_MPI_INTERPOSE before including to also shadow MPI_Allreduce
// in this translation unit (the reference's default integration mode).
#pragma once

#include <mpi.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <set>
#include <vector>

#include "flexar/cost_model.hpp"
#include "flexar/flexar.h"
#include "flexar/host_exec.hpp"
#include "flexar/msg_plan.hpp"
#include "flexar/planner.hpp"
#include "flexar/readiness.hpp"

extern "C" int flexar_pointer_is_device(const void* p);  // libflexar: hipPointerGetAttributes
extern "C" int flexar_copy_device_host(void* dst, const void* src, size_t bytes);  // synchronous hipMemcpy
extern "C" void* flexar_device_alloc(size_t bytes);
extern "C" void flexar_device_free(void* p);

// Feature probe (reference mpi_mod.hpp:8-12 printed "FlexTree enabled").
static inline int FT_enabled() {
  fprintf(stdout, "FlexTree enabled (flexar %s, MI355X-native)\n", flexar_version());
  return 0;
}

namespace flexar {
namespace mpi {

inline int dtype_of(MPI_Datatype dt) {
  if (dt == MPI_FLOAT) return FLEXAR_FLOAT32;
  if (dt == MPI_DOUBLE) return FLEXAR_FLOAT64;
  if (dt == MPI_INT8_T || dt == MPI_SIGNED_CHAR || dt == MPI_CHAR) return FLEXAR_INT8;
  if (dt == MPI_UINT8_T || dt == MPI_UNSIGNED_CHAR || dt == MPI_BYTE) return FLEXAR_UINT8;
  if (dt == MPI_INT16_T || dt == MPI_SHORT) return FLEXAR_INT16;
  if (dt == MPI_UINT16_T || dt == MPI_UNSIGNED_SHORT) return FLEXAR_UINT16;
  if (dt == MPI_INT32_T || dt == MPI_INT) return FLEXAR_INT32;
  if (dt == MPI_UINT32_T || dt == MPI_UNSIGNED) return FLEXAR_UINT32;
  if (dt == MPI_INT64_T || dt == MPI_LONG_LONG_INT || dt == MPI_LONG_LONG || dt == MPI_LONG) return FLEXAR_INT64;
  if (dt == MPI_UINT64_T || dt == MPI_UNSIGNED_LONG_LONG || dt == MPI_UNSIGNED_LONG) return FLEXAR_UINT64;
  if (dt == MPI_C_BOOL) return FLEXAR_BOOL;
  return -1;
}

inline int op_of(MPI_Op op) {
  if (op == MPI_SUM) return FLEXAR_SUM;
  if (op == MPI_PROD) return FLEXAR_PROD;
  if (op == MPI_MAX) return FLEXAR_MAX;
  if (op == MPI_MIN) return FLEXAR_MIN;
  if (op == MPI_BAND) return FLEXAR_BAND;
  if (op == MPI_BOR) return FLEXAR_BOR;
  if (op == MPI_BXOR) return FLEXAR_BXOR;
  return -1;
}

// Persistent worker pool: workgroup g (1..G-1) of the host engine runs on worker g-1.
class Pool {
 public:
  explicit Pool(int n) : n_(n) {
    for (int i = 0; i < n_; ++i) th_.emplace_back([this, i] { loop(i); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return n_; }
  // run fn(i) on workers 0..k-1 and fn(k) on the caller... caller passes its own share separately
  template <typename F>
  void run(int k, F&& fn) {
    {
      std::lock_guard<std::mutex> lk(m_);
      job_ = fn;
      active_ = k;
      pending_ = k;
      ++gen_;
    }
    cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
  }

 private:
  void loop(int i) {
    int seen = 0;
    for (;;) {
      std::function<void(int)> job;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        if (i >= active_) continue;
        job = job_;
      }
      job(i);
      {
        std::lock_guard<std::mutex> lk(m_);
        if (--pending_ == 0) done_cv_.notify_all();
      }
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  std::function<void(int)> job_;
  int gen_ = 0, active_ = 0, pending_ = 0;
  bool stop_ = false;
};

constexpr uint32_t kHostMaxGrid = 16;

// Per-rank translation of the push-form program into coalesced p2p messages.
struct P2PPlan {
  // for every peer: the (off, len) STG regions it writes into this rank, grouped by the slot of
  // the SIGNAL that publishes them, in program order (the payload order of its message).
  std::map<std::pair<int, uint32_t>, std::vector<std::pair<uint64_t, uint64_t>>> incoming;
  std::map<std::pair<int, uint32_t>, uint64_t> incoming_elems;
  std::map<std::pair<int, uint32_t>, uint64_t> outgoing_elems;
};

struct HostComm {
  MPI_Comm comm = MPI_COMM_NULL;
  int rank = 0, size = 1;
  bool shared = false;
  MPI_Win win = MPI_WIN_NULL;
  size_t cap = 0;           // staging bytes per parity
  size_t flag_bytes = 0;
  std::vector<char*> stg;   // per rank staging base (shared mode)
  std::vector<std::atomic<uint64_t>*> flags;
  uint64_t epoch = 0;  // one epoch per call for every host workgroup: uniform staging parity per call
  std::map<std::string, std::unique_ptr<Program>> plans;
  std::map<std::string, std::unique_ptr<P2PPlan>> p2p;
  std::vector<char> p2p_stg, outbox, inbox, host_stage;
  // node structure for device buffers across nodes (FLEXAR_NODE_SIZE=k forces virtual nodes of k ranks)
  MPI_Comm local = MPI_COMM_NULL, cross = MPI_COMM_NULL;
  int nodes = 1;
  void* shard_dev = nullptr;
  size_t shard_cap = 0;
  std::unique_ptr<Pool> pool;
  XgmiModel model = XgmiModel::from_env();
  std::map<double, AlgoSpec> auto_choice;  // the selector's pick per call size ("auto": priced once, not per call)
  int threads = 1;

  ~HostComm() {
    if (shard_dev) flexar_device_free(shard_dev);
    if (local != MPI_COMM_NULL) MPI_Comm_free(&local);
    if (cross != MPI_COMM_NULL) MPI_Comm_free(&cross);
    if (win != MPI_WIN_NULL) MPI_Win_free(&win);
    if (comm != MPI_COMM_NULL) MPI_Comm_free(&comm);
  }

  void init(MPI_Comm parent) {
    MPI_Comm_dup(parent, &comm);
    MPI_Comm_rank(comm, &rank);
    MPI_Comm_size(comm, &size);
    MPI_Comm node;
    MPI_Comm_split_type(comm, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &node);
    int nsz = 0;
    MPI_Comm_size(node, &nsz);
    MPI_Comm_free(&node);
    shared = (nsz == size) && getenv("FLEXAR_MPI_P2P") == nullptr;
    // node split: physical shared-memory domains, or virtual nodes of FLEXAR_NODE_SIZE ranks
    const char* ns = getenv("FLEXAR_NODE_SIZE");
    int k = ns ? atoi(ns) : 0;
    if (k > 0 && size % k == 0) {
      MPI_Comm_split(comm, rank / k, rank, &local);
    } else {
      MPI_Comm_split_type(comm, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &local);
    }
    int lr = 0, ls = 1;
    MPI_Comm_rank(local, &lr);
    MPI_Comm_size(local, &ls);
    MPI_Comm_split(comm, lr, rank, &cross);
    MPI_Comm_size(cross, &nodes);
    // reduce threads per rank: FLEXAR_HOST_THREADS, else this rank's share of the node's hardware threads
    // (the reference runs a fixed 14-thread OpenMP team per reduce call, mpi_mod.hpp:253, oversubscribing
    // a node whenever more than one rank shares it). Calls below 1 MiB per thread stay single-threaded.
    const char* t = getenv("FLEXAR_HOST_THREADS");
    const int hw = (int)std::thread::hardware_concurrency();
    threads = t ? atoi(t) : std::max(1, hw / std::max(1, ls));
    if (threads < 1) threads = 1;
    if (threads > (int)kHostMaxGrid) threads = kHostMaxGrid;
    if (threads > 1) pool.reset(new Pool(threads - 1));
  }

  // (Re)allocate the shared window so one parity half holds `need` bytes. Collective.
  void ensure_window(size_t need) {
    if (!shared || (win != MPI_WIN_NULL && need <= cap)) return;
    if (win != MPI_WIN_NULL) MPI_Win_free(&win);
    cap = std::max<size_t>(need, size_t(1) << 20);
    cap = (cap + 4095) / 4096 * 4096;
    flag_bytes = (size_t)kMaxSlots * size * kHostMaxGrid * sizeof(uint64_t);
    flag_bytes = (flag_bytes + 4095) / 4096 * 4096;
    char* base = nullptr;
    MPI_Win_allocate_shared((MPI_Aint)(flag_bytes + 2 * cap), 1, MPI_INFO_NULL, comm, &base, &win);
    memset(base, 0, flag_bytes);
    stg.assign(size, nullptr);
    flags.assign(size, nullptr);
    for (int r = 0; r < size; ++r) {
      MPI_Aint sz;
      int du;
      char* p = nullptr;
      MPI_Win_shared_query(win, r, &sz, &du, &p);
      flags[r] = reinterpret_cast<std::atomic<uint64_t>*>(p);
      stg[r] = p + flag_bytes;
    }
    epoch = 0;
    MPI_Barrier(comm);  // flags zeroed everywhere before anyone signals
  }
};

inline std::string plan_key(const AlgoSpec& s, size_t count, size_t es, float fs) {
  char b[256];
  uint32_t u;
  memcpy(&u, &fs, 4);
  snprintf(b, sizeof(b), "%s|%zu|%zu|%08x", s.str().c_str(), count, es, u);
  return b;
}

inline int resolve_algo(HostComm& h, double bytes, AlgoSpec* s) {
  std::string err;
  const char* a = getenv("FLEXAR_ALGO");
  if (a && *a) {
    if (!parse_algo(a, h.size, s, &err)) { fprintf(stderr, "[flexar] bad FLEXAR_ALGO: %s\n", err.c_str()); return 1; }
  } else if (!parse_ft_topo(getenv("FT_TOPO"), h.size, s, &err)) {  // reference semantics, read per call
    fprintf(stderr, "[flexar] %s\n", err.c_str());
    return 1;
  }
  if (s->kind == AlgoKind::AUTO) {
    auto it = h.auto_choice.find(bytes);
    if (it == h.auto_choice.end()) {
      if (h.auto_choice.size() > 4096) h.auto_choice.clear();
      it = h.auto_choice.emplace(bytes, select_plan(h.model, h.size, bytes)).first;
    }
    *s = it->second;
  }
  if (s->kind == AlgoKind::LL) s->kind = AlgoKind::ONESHOT;  // LL granules are a device protocol
  if (s->kind == AlgoKind::DMA) s->kind = AlgoKind::TREE, s->widths = {h.size};  // copy engines: device only
  if (s->kind == AlgoKind::TREE && (!h.shared || s->ag == AgMode::AUTO)) s->ag = AgMode::PUSH;
  s->wire = 0;  // typed staging is a device-executor feature: the host engines run the dtype throughout
  s->zc = false;  // so are registered (zero-copy) device buffers
  s->put = false;
  if (!h.shared) s->bidir = false;  // the p2p engine carries messages: no peer reads
  return 0;
}

template <typename T, typename OP>
struct ShmRun {
  static int run(HostComm& h, const Program& P, const void* in, void* out, int grid) {
    HostExecCtx c;
    c.rank = h.rank;
    c.local[BUF_IN] = (char*)in;
    c.local[BUF_OUT] = (char*)out;
    c.local[BUF_STG] = h.stg[h.rank];
    c.peer_stg = h.stg;
    c.peer_flags = h.flags;
    c.ranks_stride = h.size;
    c.blocks_stride = kHostMaxGrid;
    c.stg_half_bytes = h.cap;
    std::atomic<int> rc{0};
    const uint64_t e = ++h.epoch;
    auto body = [&](int g) {
      int x = HostExec<T, OP>::run(P, c, (uint32_t)g, (uint32_t)grid, e);
      if (x) rc.store(x);
    };
    if (grid > 1) h.pool->run(grid - 1, [&](int i) { body(i + 1); });
    body(0);
    if (grid > 1) h.pool->wait();
    return rc.load();
  }
};

// Build the p2p message plan for rank h.rank: replay every peer's program to learn what it
// writes into us and under which SIGNAL slot it publishes it.
// The coalescing is the message transport's (msg_plan.hpp msg_regions): one message per (peer, SIGNAL).
inline std::unique_ptr<P2PPlan> build_p2p(HostComm& h, const AlgoSpec& s, size_t count, size_t es, float fs) {
  std::unique_ptr<P2PPlan> pp(new P2PPlan);
  std::string err;
  for (int p = 0; p < h.size; ++p) {
    Program Q;
    Planner pl(h.size, p, count, (uint32_t)es, fs);
    pl.build(s, &Q, &err);
    for (int q = 0; q < h.size; ++q) {
      if (q == p || (p != h.rank && q != h.rank)) continue;
      for (const MsgRegions& m : msg_regions(Q, (uint32_t)p, (uint32_t)q)) {
        uint64_t tot = 0;
        for (auto& rg : m.regions) tot += rg.second;
        if (q == h.rank) {
          pp->incoming[{p, m.slot}] = m.regions;
          pp->incoming_elems[{p, m.slot}] = tot;
        }
        if (p == h.rank) pp->outgoing_elems[{q, m.slot}] = tot;
      }
    }
  }
  return pp;
}

template <typename T, typename OP>
struct P2PRun {
  static int run(HostComm& h, const Program& P, const P2PPlan& pp, const void* in, void* out) {
    const size_t es = sizeof(T);
    char* stg = h.p2p_stg.data();
    auto addr = [&](const Loc& l) -> char* {
      if (l.buf == BUF_STG) return stg + l.off * es;
      return (l.buf == BUF_IN ? (char*)in : (char*)out) + l.off * es;
    };
    // outbox: per-peer running buffers (sized by the plan), kept alive until Waitall
    std::map<int, std::vector<char>> box;
    std::vector<MPI_Request> reqs;
    std::vector<std::vector<char>> sent;
    for (const Op& o : P.ops) {
      if (o.kind == OP_XFER) {
        const T* srcs[kMaxSrc];
        T* dsts[kMaxDst];
        int nloc = 0;
        for (int k = 0; k < o.nsrc; ++k) srcs[k] = (const T*)addr(o.src[k]);
        std::vector<int> remote;
        for (int d = 0; d < o.ndst; ++d) {
          if (o.dst[d].rank == (uint16_t)h.rank) dsts[nloc++] = (T*)addr(o.dst[d]);
          else remote.push_back(o.dst[d].rank);
        }
        for (int q : remote) {
          auto& b = box[q];
          size_t at = b.size();
          b.resize(at + o.len * es);
          dsts[nloc++] = (T*)(b.data() + at);
        }
        host_reduce_span<T, OP>(dsts, nloc, srcs, o.nsrc, o.len, o.scale);
      } else if (o.kind == OP_SIGNAL) {
        for (int k = 0; k < o.npeers; ++k) {
          int q = o.peers[k];
          sent.emplace_back(std::move(box[q]));
          box[q].clear();
          reqs.emplace_back();
          MPI_Isend(sent.back().data(), (int)sent.back().size(), MPI_BYTE, q, (int)o.slot, h.comm, &reqs.back());
        }
      } else if (o.kind == OP_WAIT) {
        for (int k = 0; k < o.npeers; ++k) {
          int p = o.peers[k];
          auto key = std::make_pair(p, o.slot);
          auto it = pp.incoming.find(key);
          uint64_t tot = pp.incoming_elems.count(key) ? pp.incoming_elems.at(key) : 0;
          h.inbox.resize(std::max<size_t>(h.inbox.size(), tot * es + 1));
          MPI_Recv(h.inbox.data(), (int)(tot * es), MPI_BYTE, p, (int)o.slot, h.comm, MPI_STATUS_IGNORE);
          if (it != pp.incoming.end()) {
            size_t at = 0;
            for (auto& rg : it->second) {
              memcpy(stg + rg.first * es, h.inbox.data() + at, rg.second * es);
              at += rg.second * es;
            }
          }
        }
      }
    }
    if (!reqs.empty()) MPI_Waitall((int)reqs.size(), reqs.data(), MPI_STATUSES_IGNORE);  // D1: every send completed
    return 0;
  }
};

struct Dispatch {
  template <typename T, typename OP>
  static int run(HostComm& h, const Program& P, const P2PPlan* pp, const void* in, void* out, int grid) {
    if (pp) return P2PRun<T, OP>::run(h, P, *pp, in, out);
    return ShmRun<T, OP>::run(h, P, in, out, grid);
  }
};

inline int keyval() {
  static int kv = MPI_KEYVAL_INVALID;
  if (kv == MPI_KEYVAL_INVALID) {
    auto del = [](MPI_Comm, int, void* attr, void*) -> int {
      delete static_cast<HostComm*>(attr);
      return MPI_SUCCESS;
    };
    MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, del, &kv, nullptr);
  }
  return kv;
}

inline HostComm* host_comm(MPI_Comm comm) {
  int flag = 0;
  void* v = nullptr;
  MPI_Comm_get_attr(comm, keyval(), &v, &flag);
  if (flag) return static_cast<HostComm*>(v);
  HostComm* h = new HostComm;
  h->init(comm);
  MPI_Comm_set_attr(comm, keyval(), h);
  return h;
}

// ---- device buffers: flexar GPU communicator bootstrapped over MPI ------------------------------
// Deleted by MPI when the communicator's attributes go (MPI_Comm_free / MPI_Finalize, collective): the
// device communicator's teardown agrees with its peers by itself (flexar_comm_destroy, host_barrier.hpp).
struct DevHolder {
  flexar_comm_t c = nullptr;
  // zero copy through the MPI entry points (zc_prepare): buffers whose registration was refused on some rank
  // (e.g. an allocation above FLEXAR_REG_MAX_ALLOC) are not tried again; past 64 refusals nothing is
  std::set<std::pair<uintptr_t, size_t>> zc_refused;
  bool zc_closed = false;
  ~DevHolder() {
    if (c) flexar_comm_destroy(c);
  }
};
inline int dev_keyval() {
  static int kv = MPI_KEYVAL_INVALID;
  if (kv == MPI_KEYVAL_INVALID) {
    auto del = [](MPI_Comm, int, void* attr, void*) -> int {
      delete static_cast<DevHolder*>(attr);
      return MPI_SUCCESS;
    };
    MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, del, &kv, nullptr);
  }
  return kv;
}
extern "C" int flexar_current_device(void);
inline DevHolder* dev_holder(MPI_Comm comm) {
  int flag = 0;
  void* v = nullptr;
  MPI_Comm_get_attr(comm, dev_keyval(), &v, &flag);
  return flag ? static_cast<DevHolder*>(v) : nullptr;
}
inline flexar_comm_t device_comm(MPI_Comm comm) {
  if (DevHolder* h = dev_holder(comm)) return h->c;
  int rank, size;
  MPI_Comm_rank(comm, &rank);
  MPI_Comm_size(comm, &size);
  DevHolder* d = new DevHolder;
  int rc = flexar_comm_create(rank, size, flexar_current_device(), 0, &d->c);
  if (rc) { fprintf(stderr, "[flexar] comm_create: %s\n", flexar_last_error()); abort(); }
  size_t hs = flexar_handle_size();
  std::vector<char> mine(hs), all(hs * size);
  flexar_comm_export(d->c, mine.data());
  MPI_Allgather(mine.data(), (int)hs, MPI_BYTE, all.data(), (int)hs, MPI_BYTE, comm);
  int ok = flexar_comm_connect(d->c, all.data()) == 0, all_ok = 0;
  if (!ok) fprintf(stderr, "[flexar] rank %d connect: %s\n", rank, flexar_last_error());
  MPI_Allreduce(&ok, &all_ok, 1, MPI_INT, MPI_MIN, comm);
  if (!all_ok) abort();
  // probe agreement (readiness.hpp probe_agree): the minimum link count on every rank, or a named error
  if (size > 1) {
    std::vector<char> pb(flexar_probe_blob_size()), pall(pb.size() * size);
    flexar_comm_probe_export(d->c, pb.data());
    MPI_Allgather(pb.data(), (int)pb.size(), MPI_BYTE, pall.data(), (int)pb.size(), MPI_BYTE, comm);
    if (flexar_comm_probe_agree(d->c, pall.data())) {
      fprintf(stderr, "[flexar] rank %d: %s\n", rank, flexar_last_error());
      abort();
    }
  }
  // connect-time self-test (readiness.hpp): a protocol family that failed on any rank is disabled on all
  if (size > 1 && !(getenv("FLEXAR_SELFTEST") && strcmp(getenv("FLEXAR_SELFTEST"), "0") == 0)) {
    // one family at a time behind a barrier, and a failed family once more before it is disabled (a rank
    // arriving past its peers' short watchdog must not shift every later family out of step)
    // A HIP error on one rank fails that family there (named by flexar_comm_selftest_note) and the
    // downgrade chain goes on; only an error that left a device unusable (non-zero rc, agreed on) ends here
    auto run = [&](uint32_t fam) -> uint32_t {
      uint32_t failed = 0, any = 0;
      MPI_Barrier(comm);
      int rc = flexar_comm_selftest(d->c, fam, &failed), worst = 0;
      if (rc) fprintf(stderr, "[flexar] rank %d self-test: %s\n", rank, flexar_last_error());
      MPI_Allreduce(&rc, &worst, 1, MPI_INT, MPI_MAX, comm);
      if (worst) abort();
      if (failed) {
        char note[512];
        flexar_comm_selftest_note(d->c, note, sizeof(note));
        fprintf(stderr, "[flexar] rank %d self-test: %s\n", rank, note);
      }
      MPI_Allreduce(&failed, &any, 1, MPI_UINT32_T, MPI_BOR, comm);
      if (any) {  // every rank is past this family's calls: reset the protocol state, then start together
        flexar_comm_resync(d->c);
        MPI_Barrier(comm);
      }
      return any;
    };
    uint32_t any = 0;
    for (uint32_t fam = 1; fam & PF_ALL; fam <<= 1) any |= run(fam);
    if (any) {
      uint32_t again = 0;
      for (uint32_t fam = 1; fam & PF_ALL; fam <<= 1)
        if (any & fam) again |= run(fam);
      any = again;
    }
    if (any) {
      flexar_comm_set_disabled(d->c, any);
      fprintf(stderr, "[flexar] rank %d: protocol families failing the self-test disabled: %s\n", rank,
              family_names(any).c_str());
      if (any == PF_ALL) abort();
    }
  }
  // connect-time calibration of the cost model (FLEXAR_CALIB=0 | 1 | force; calibration.hpp): the cached
  // constants of this node shape or a short measurement, identical on every rank; ranks whose models end
  // up different all fall back to the default model
  if (size > 1) {
    const char* cm = getenv("FLEXAR_CALIB");
    const int mode = !cm ? 1 : (!strcmp(cm, "0") || !strcmp(cm, "off")) ? 0 : !strcmp(cm, "force") ? 2 : 1;
    MPI_Barrier(comm);
    const int crc = flexar_comm_calibrate(d->c, mode, nullptr, 0);
    unsigned long long h[2] = {crc ? 0ull : (unsigned long long)flexar_comm_model_hash(d->c), 0}, lo = 0, hi = 0;
    h[1] = h[0];
    MPI_Allreduce(&h[0], &lo, 1, MPI_UNSIGNED_LONG_LONG, MPI_MIN, comm);
    MPI_Allreduce(&h[1], &hi, 1, MPI_UNSIGNED_LONG_LONG, MPI_MAX, comm);
    if (lo != hi || lo == 0) {
      flexar_comm_clear_error(d->c);
      flexar_comm_reset_model(d->c);
    }
  }
  MPI_Barrier(comm);
  MPI_Comm_set_attr(comm, dev_keyval(), d);
  return d->c;
}

inline int allreduce(const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype datatype, MPI_Op mop,
                     MPI_Comm comm);

// Zero copy through the MPI entry points. The zero-copy schedules read / write the peers'
// buffers directly, so a call's buffers must be registered on every rank (collective, cached per range).
//  * FORCE (FLEXAR_ALGO names "+zc"): every device call registers its buffers first (ensure_registered);
//  * AUTO (default: FLEXAR_ALGO unset or "auto", FLEXAR_MPI_ZC unset or 1): device calls of at least
//    FLEXAR_MPI_ZC_MIN_BYTES (1 MiB) take part in one agreement per call (a 2-int MPI_Allreduce MIN): "both
//    buffers registered and fresh on every rank" runs the cost model's choice with zero copy allowed (the
//    flat schedule becomes "+zc+push", zc_policy.hpp); otherwise, while registrations are below
//    FLEXAR_MPI_ZC_MAX_REGS (64) and this buffer's registration was not refused before, the buffers are
//    registered collectively (a stale registration - freed, address reused - is replaced) and the call runs
//    zero copy; else it runs staging
//    with zero copy disallowed on every rank (flexar_comm_set_zc_auto), so a registration that is fresh on
//    one rank and stale on another can never split the ranks between two schedules. The c10d backend's
//    probe window (parallel/backend.py) closes after idle agreements because it sits on DDP's issue path;
//    an MPI call already synchronises the device, and only the per-call agreement catches a freed and
//    reused address, so here it stays;
//  * OFF: FLEXAR_ALGO set to a spec without "+zc" (the user chose the schedule), FLEXAR_MPI_ZC=0 or
//    FLEXAR_ZC_AUTO=0.
// Reference entry point: allreduce_over_mpi/mpi_mod.hpp:1167-1221 (MPI_Allreduce_FT), driven by
// benchmark.cpp:147-159.
enum class ZcMode { OFF = 0, AUTO = 1, FORCE = 2 };
inline ZcMode zc_mode_of(const char* algo, const char* mpi_zc, const char* zc_auto = nullptr) {
  if (algo && strstr(algo, "+zc")) return ZcMode::FORCE;
  if ((mpi_zc && !strcmp(mpi_zc, "0")) || (zc_auto && !strcmp(zc_auto, "0"))) return ZcMode::OFF;
  if (algo && *algo && strcmp(algo, "auto") != 0) return ZcMode::OFF;
  return ZcMode::AUTO;
}
inline ZcMode zc_mode() {
  static const ZcMode m = zc_mode_of(getenv("FLEXAR_ALGO"), getenv("FLEXAR_MPI_ZC"), getenv("FLEXAR_ZC_AUTO"));
  return m;
}
inline bool zc_requested() { return zc_mode() == ZcMode::FORCE; }
inline int ensure_registered(flexar_comm_t c, MPI_Comm comm, const void* p, size_t bytes) {
  int mine = flexar_reg_find(c, p, bytes) > 0 ? 1 : 0, all = 0;
  MPI_Allreduce(&mine, &all, 1, MPI_INT, MPI_MIN, comm);
  if (all) return MPI_SUCCESS;
  int size = 1;
  MPI_Comm_size(comm, &size);
  const size_t hs = flexar_reg_handle_size();
  std::vector<char> blob(hs, 0), blobs(hs * size);
  int ok = flexar_reg_export(c, p, bytes, blob.data()) == 0 ? 1 : 0, all_ok = 0;
  if (!ok) fprintf(stderr, "[flexar] register: %s\n", flexar_last_error());
  MPI_Allgather(blob.data(), (int)hs, MPI_BYTE, blobs.data(), (int)hs, MPI_BYTE, comm);
  MPI_Allreduce(&ok, &all_ok, 1, MPI_INT, MPI_MIN, comm);
  if (!all_ok) return MPI_ERR_OTHER;
  int id = 0;
  ok = flexar_reg_open(c, p, bytes, blobs.data(), &id) == 0 ? 1 : 0;
  if (!ok) fprintf(stderr, "[flexar] register: %s\n", flexar_last_error());
  MPI_Allreduce(&ok, &all_ok, 1, MPI_INT, MPI_MIN, comm);
  return all_ok ? MPI_SUCCESS : MPI_ERR_OTHER;
}

// Registration / zero-copy decision for one device call on `comm` (see zc_mode). Collective over `comm` for
// FORCE and for AUTO calls of at least the minimum size (every rank passes the same count); returns true
// when the call may run zero copy.
inline bool zc_prepare(MPI_Comm comm, const void* in, const void* out, size_t bytes) {
  const ZcMode m = zc_mode();
  DevHolder* d = dev_holder(comm);
  if (!d) return false;
  flexar_comm_t c = d->c;
  if (m == ZcMode::OFF) return false;
  if (m == ZcMode::FORCE) {
    // a registration refused on any rank (all agree) leaves the buffers unregistered: the call then runs
    // the staging schedule (comm.hip falls back from a default "+zc" spec for unregistered buffers)
    int e = ensure_registered(c, comm, in, bytes);
    if (e == MPI_SUCCESS && in != out) e = ensure_registered(c, comm, out, bytes);
    return e == MPI_SUCCESS;
  }
  static const uint64_t min_bytes = [] {
    const char* e = getenv("FLEXAR_MPI_ZC_MIN_BYTES");
    return e && *e ? strtoull(e, nullptr, 10) : (1ull << 20);
  }();
  static const int max_regs = [] {
    const char* e = getenv("FLEXAR_MPI_ZC_MAX_REGS");
    return e && *e ? atoi(e) : 64;
  }();
  if (bytes < min_bytes) {  // the same on every rank: no agreement, never zero copy
    flexar_comm_set_zc_auto(c, 0);
    return false;
  }
  auto fresh = [&](const void* p) { return flexar_reg_find(c, p, bytes) > 0; };
  const bool aligned = (((uintptr_t)in | (uintptr_t)out) & 15) == 0;
  const bool refused = d->zc_refused.count({(uintptr_t)in, bytes}) || d->zc_refused.count({(uintptr_t)out, bytes});
  int v[2] = {fresh(in) && (in == out || fresh(out)) ? 1 : 0,
              aligned && !refused && !d->zc_closed && flexar_reg_count(c) + 2 <= max_regs ? 1 : 0};
  MPI_Allreduce(MPI_IN_PLACE, v, 2, MPI_INT, MPI_MIN, comm);
  bool use = v[0] != 0;
  if (!use && v[1]) {
    int e = ensure_registered(c, comm, in, bytes);  // agreed result on every rank
    if (e == MPI_SUCCESS && in != out) e = ensure_registered(c, comm, out, bytes);
    if (e == MPI_SUCCESS) {
      use = true;
    } else {  // refused on some rank (agreed): remember this buffer, give up after many
      d->zc_refused.insert({(uintptr_t)in, bytes});
      d->zc_refused.insert({(uintptr_t)out, bytes});
      if (d->zc_refused.size() > 64) d->zc_closed = true;
    }
  }
  flexar_comm_set_zc_auto(c, use ? 1 : 0);
  return use;
}

// Device buffers spanning nodes: intra-node reduce-scatter over xGMI (flexar), inter-node allreduce
// of each rank's 1/L shard through host memory (p2p engine over the cross-node communicator of the
// ranks with the same node-local index), intra-node all-gather over xGMI. Each rank ships only 1/L of
// the buffer across nodes — the hierarchical form of the reference's multi-host FlexTree.
inline int hierarchical_device_allreduce(HostComm& hc, const void* in, void* out, size_t count, MPI_Datatype datatype,
                                         MPI_Op mop, int dt, int op) {
  int L = 1;
  MPI_Comm_size(hc.local, &L);
  const size_t es = dtype_size(dt);
  const size_t m = count / L, main = m * L, rem = count - main;
  flexar_comm_t dc = device_comm(hc.local);
  int rc = MPI_SUCCESS;
  if (m > 0) {
    if (hc.shard_cap < m * es) {
      if (hc.shard_dev) flexar_device_free(hc.shard_dev);
      hc.shard_dev = flexar_device_alloc(m * es);
      hc.shard_cap = hc.shard_dev ? m * es : 0;
      if (!hc.shard_dev) return MPI_ERR_NO_MEM;
    }
    if (flexar_reduce_scatter(dc, in, hc.shard_dev, m, dt, op, nullptr, nullptr)) {
      fprintf(stderr, "[flexar] reduce_scatter: %s\n", flexar_last_error());
      return MPI_ERR_OTHER;
    }
    hc.host_stage.resize(m * es);
    if (flexar_copy_device_host(hc.host_stage.data(), hc.shard_dev, m * es)) return MPI_ERR_OTHER;
    rc = allreduce(MPI_IN_PLACE, hc.host_stage.data(), m, datatype, mop, hc.cross);
    if (rc != MPI_SUCCESS) return rc;
    if (flexar_copy_device_host(hc.shard_dev, hc.host_stage.data(), m * es)) return MPI_ERR_OTHER;
    if (flexar_all_gather(dc, hc.shard_dev, out, m, dt, nullptr, nullptr)) {
      fprintf(stderr, "[flexar] all_gather: %s\n", flexar_last_error());
      return MPI_ERR_OTHER;
    }
  }
  if (rem > 0) {  // fewer than L trailing elements: whole-communicator host allreduce
    std::vector<char> tail(rem * es);
    if (flexar_copy_device_host(tail.data(), (const char*)in + main * es, rem * es)) return MPI_ERR_OTHER;
    rc = allreduce(MPI_IN_PLACE, tail.data(), rem, datatype, mop, hc.comm);
    if (rc == MPI_SUCCESS && flexar_copy_device_host((char*)out + main * es, tail.data(), rem * es)) rc = MPI_ERR_OTHER;
  }
  return rc;
}

inline int allreduce(const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype datatype, MPI_Op mop,
                     MPI_Comm comm) {
  const int dt = dtype_of(datatype), op = op_of(mop);
  if (dt < 0 || op < 0 || !op_supported(dt, op)) {
    fprintf(stderr, "[flexar] MPI_Allreduce_FT: unsupported datatype/op\n");
    return MPI_ERR_OP;
  }
  const bool in_place = (sendbuf == MPI_IN_PLACE);
  const void* in = in_place ? recvbuf : sendbuf;
  int size;
  MPI_Comm_size(comm, &size);
  const size_t es = dtype_size(dt);
  if (count == 0) return MPI_SUCCESS;
  const bool dev_out = flexar_pointer_is_device(recvbuf) != 0;
  if (!in_place && in != recvbuf && (flexar_pointer_is_device(in) != 0) != dev_out) {
    // mixed host/device pair: bring the input to recvbuf's side, then run in place there
    if (flexar_copy_device_host(recvbuf, in, count * es)) return MPI_ERR_OTHER;
    in = recvbuf;
  }
  if (dev_out) {
    HostComm* hc = host_comm(comm);
    if (hc->nodes > 1 && getenv("FLEXAR_MPI_FLAT_STAGING") == nullptr)
      return hierarchical_device_allreduce(*hc, in, recvbuf, count, datatype, mop, dt, op);
    if (hc->nodes == 1 || size <= 1) {  // one node: xGMI/IPC GPU engine
      flexar_comm_t c = device_comm(comm);
      if (size > 1) zc_prepare(comm, in, recvbuf, count * es);
      int rc = flexar_allreduce(c, in, recvbuf, count, dt, op, nullptr);
      // MPI semantics: recvbuf holds the result when the call returns (a NIC, MPI_Send or another stream
      // may read it next), and a device watchdog timeout is this call's error, not the next one's
      if (!rc) rc = flexar_device_synchronize();
      if (!rc) rc = flexar_comm_check(c);
      if (rc) { fprintf(stderr, "[flexar] allreduce: %s\n", flexar_last_error()); return MPI_ERR_OTHER; }
      return MPI_SUCCESS;
    }
    // ranks on several nodes: IPC cannot span nodes -> stage through host memory and run the p2p engine
    hc->host_stage.resize(count * es);
    if (flexar_copy_device_host(hc->host_stage.data(), in, count * es)) return MPI_ERR_OTHER;
    int rc = allreduce(MPI_IN_PLACE, hc->host_stage.data(), count, datatype, mop, comm);
    if (rc == MPI_SUCCESS && flexar_copy_device_host(recvbuf, hc->host_stage.data(), count * es)) rc = MPI_ERR_OTHER;
    return rc;
  }
  if (size <= 1) {  // reference: memcpy unless in place (mpi_mod.hpp:1181-1188)
    if (!in_place) memcpy(recvbuf, sendbuf, count * es);
    return MPI_SUCCESS;
  }
  HostComm* h = host_comm(comm);
  AlgoSpec s;
  if (resolve_algo(*h, (double)count * es, &s)) return MPI_ERR_ARG;
  const std::string key = plan_key(s, count, es, 1.0f);
  auto it = h->plans.find(key);
  if (it == h->plans.end()) {
    std::unique_ptr<Program> P(new Program);
    Planner pl(h->size, h->rank, count, (uint32_t)es, 1.0f);
    std::string err;
    if (!pl.build(s, P.get(), &err)) { fprintf(stderr, "[flexar] %s\n", err.c_str()); return MPI_ERR_ARG; }
    it = h->plans.emplace(key, std::move(P)).first;
  }
  const Program& P = *it->second;
  const P2PPlan* pp = nullptr;
  int grid = 1;
  if (h->shared) {
    h->ensure_window(P.stg_elems * es);
    uint64_t bytes = count * es;
    grid = h->threads;
    while (grid > 1 && bytes / grid < (1u << 20)) --grid;  // >= 1 MiB per host workgroup
    // whole channels, and never more host workgroups than the flag layout has per rank
    // (host_flag_index strides blocks by kHostMaxGrid: a larger grid would alias another rank's flags)
    if (P.nchan > kHostMaxGrid) {
      fprintf(stderr, "[flexar] %s needs %u channels; the host engine runs at most %u\n", s.str().c_str(), P.nchan,
              kHostMaxGrid);
      return MPI_ERR_ARG;
    }
    grid = std::max<int>(grid, (int)P.nchan);
    grid = (grid + P.nchan - 1) / P.nchan * P.nchan;
    if (grid > (int)kHostMaxGrid) grid = (int)(kHostMaxGrid / P.nchan * P.nchan);
    if (grid > 1 && (!h->pool || h->pool->size() < grid - 1)) h->pool.reset(new Pool(grid - 1));
  } else {
    auto jt = h->p2p.find(key);
    if (jt == h->p2p.end()) jt = h->p2p.emplace(key, build_p2p(*h, s, count, es, 1.0f)).first;
    pp = jt->second.get();
    h->p2p_stg.resize(std::max<size_t>(h->p2p_stg.size(), P.stg_elems * es + 64));
  }
  int rc = dispatch_dtype_op<Dispatch>(dt, op, *h, P, pp, in, recvbuf, grid);
  return rc == 0 ? MPI_SUCCESS : MPI_ERR_OTHER;
}

}  // namespace mpi
}  // namespace flexar

// ---- public entry points ----------------------------------------------------------------------
inline int MPI_Allreduce_FT(const void* sendbuf, void* recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                            MPI_Comm comm) {
  if (count < 0) return MPI_ERR_COUNT;
  return flexar::mpi::allreduce(sendbuf, recvbuf, (size_t)count, datatype, op, comm);
}
// size_t count: a 4 GiB bf16 tensor fits (defect D7).
inline int MPI_Allreduce_FT_large(const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype datatype,
                                  MPI_Op op, MPI_Comm comm) {
  return flexar::mpi::allreduce(sendbuf, recvbuf, count, datatype, op, comm);
}

#ifdef FLEXAR_MPI_INTERPOSE
// Route this translation unit's MPI_Allreduce calls to flexar (reference mpi_mod.hpp:1169-1171 shadowed
// the symbol with a static function, which conflicts with mpi.h's extern declaration; a macro does not).
#define MPI_Allreduce MPI_Allreduce_FT
#endif
