// flexar_bench — MPI benchmark driver, CLI-compatible with the reference's
// allreduce_over_mpi/benchmark.cpp (flags --size --repeat --to-file
// --comm-type --tag --version, same banner / CHECK / DONE lines and per-repeat
// time file), extended for MI355X:
//   --mem device|host      buffers in HBM (default when a GPU is present) or host memory
//   --comm-type flextree|flexar|mpi|rccl   flexar (FlexTree successor), vendor MPI_Allreduce,
//                          or ncclAllReduce (RCCL) as the GPU comparator
//   --dtype float32|bfloat16|float16|int32|...   --op sum|max|...   --algo <flexar spec>
//   --sweep MIN:MAX        busbw table over sizes (bytes, x2 steps), rccl-tests columns
//   --check                reset inputs every repeat and verify the result exactly
// Fixed reference defects (D12): CHECK never reads out of bounds, repeats do not
// compound in --check mode, and the reported time is the MAX over ranks.
#include <hip/hip_runtime.h>
#include <mpi.h>
#include <rccl/rccl.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "flexar/timer.hpp"
#include "flexar/mpi_mod.hpp"

#ifndef FLEXAR_GIT_VERSION
#define FLEXAR_GIT_VERSION "unknown"
#endif

namespace {

struct Args {
  size_t size = 35;  // elements (reference default)
  int repeat = 1;
  bool to_file = false;
  std::string comm = "flexar";
  std::string tag;
  std::string mem = "auto";
  std::string dtype = "float32";
  std::string op = "sum";
  std::string algo;
  size_t sweep_min = 0, sweep_max = 0;
  bool check = false;
  int warmup = 2;
};

int fx_dtype(const std::string& s) {
  static const char* n[] = {"float32", "float16", "bfloat16", "float64", "fp8_e4m3", "fp8_e5m2", "int8", "uint8",
                            "int16", "uint16", "int32", "uint32", "int64", "uint64", "bool"};
  for (int i = 0; i < FLEXAR_NUM_DTYPES; ++i)
    if (s == n[i]) return i;
  return -1;
}
int fx_op(const std::string& s) {
  static const char* n[] = {"sum", "prod", "max", "min", "avg", "band", "bor", "bxor"};
  for (int i = 0; i < FLEXAR_NUM_OPS; ++i)
    if (s == n[i]) return i;
  return -1;
}
MPI_Datatype mpi_dtype(int dt) {
  switch (dt) {
    case FLEXAR_FLOAT32: return MPI_FLOAT;
    case FLEXAR_FLOAT64: return MPI_DOUBLE;
    case FLEXAR_INT8: return MPI_INT8_T;
    case FLEXAR_UINT8: return MPI_UINT8_T;
    case FLEXAR_INT16: return MPI_INT16_T;
    case FLEXAR_UINT16: return MPI_UINT16_T;
    case FLEXAR_INT32: return MPI_INT32_T;
    case FLEXAR_UINT32: return MPI_UINT32_T;
    case FLEXAR_INT64: return MPI_INT64_T;
    case FLEXAR_UINT64: return MPI_UINT64_T;
    default: return MPI_DATATYPE_NULL;
  }
}
MPI_Op mpi_op(int op) {
  switch (op) {
    case FLEXAR_SUM: return MPI_SUM;
    case FLEXAR_PROD: return MPI_PROD;
    case FLEXAR_MAX: return MPI_MAX;
    case FLEXAR_MIN: return MPI_MIN;
    case FLEXAR_BAND: return MPI_BAND;
    case FLEXAR_BOR: return MPI_BOR;
    case FLEXAR_BXOR: return MPI_BXOR;
    default: return MPI_OP_NULL;
  }
}
ncclDataType_t nccl_dtype(int dt) {
  switch (dt) {
    case FLEXAR_FLOAT32: return ncclFloat32;
    case FLEXAR_FLOAT16: return ncclFloat16;
    case FLEXAR_BFLOAT16: return ncclBfloat16;
    case FLEXAR_FLOAT64: return ncclFloat64;
    case FLEXAR_INT8: return ncclInt8;
    case FLEXAR_UINT8: return ncclUint8;
    case FLEXAR_INT32: return ncclInt32;
    case FLEXAR_UINT32: return ncclUint32;
    case FLEXAR_INT64: return ncclInt64;
    case FLEXAR_UINT64: return ncclUint64;
    default: return ncclFloat32;
  }
}

[[noreturn]] void die(const std::string& m) {
  fprintf(stderr, "flexar_bench: %s\n", m.c_str());
  MPI_Abort(MPI_COMM_WORLD, 1);
  exit(1);
}

size_t parse_size(const std::string& s) {
  double v = atof(s.c_str());
  char u = s.empty() ? 0 : s.back();
  if (u == 'K' || u == 'k') v *= 1024;
  if (u == 'M' || u == 'm') v *= 1024 * 1024;
  if (u == 'G' || u == 'g') v *= 1024.0 * 1024 * 1024;
  return (size_t)v;
}

// fill element i with the small integer (i % 64) + rank_mix, exactly representable in every dtype we test
void fill_host(std::vector<char>& h, int dt, size_t n, int rank) {
  size_t es = flexar_dtype_size(dt);
  h.resize(n * es);
  for (size_t i = 0; i < n; ++i) {
    double v = (double)((i + rank) % 8);
    char* p = h.data() + i * es;
    switch (dt) {
      case FLEXAR_FLOAT32: { float f = (float)v; memcpy(p, &f, 4); break; }
      case FLEXAR_FLOAT64: { memcpy(p, &v, 8); break; }
      case FLEXAR_FLOAT16: { uint16_t b = flexar::f32_to_f16((float)v); memcpy(p, &b, 2); break; }
      case FLEXAR_BFLOAT16: { uint16_t b = flexar::f32_to_bf16((float)v); memcpy(p, &b, 2); break; }
      case FLEXAR_INT32: case FLEXAR_UINT32: { uint32_t x = (uint32_t)v; memcpy(p, &x, 4); break; }
      case FLEXAR_INT64: case FLEXAR_UINT64: { uint64_t x = (uint64_t)v; memcpy(p, &x, 8); break; }
      case FLEXAR_INT16: case FLEXAR_UINT16: { uint16_t x = (uint16_t)v; memcpy(p, &x, 2); break; }
      default: { uint8_t x = (uint8_t)v; memcpy(p, &x, 1); break; }
    }
  }
}
double host_val(const std::vector<char>& h, int dt, size_t i) {
  size_t es = flexar_dtype_size(dt);
  const char* p = h.data() + i * es;
  switch (dt) {
    case FLEXAR_FLOAT32: { float f; memcpy(&f, p, 4); return f; }
    case FLEXAR_FLOAT64: { double d; memcpy(&d, p, 8); return d; }
    case FLEXAR_FLOAT16: { uint16_t b; memcpy(&b, p, 2); return flexar::f16_to_f32(b); }
    case FLEXAR_BFLOAT16: { uint16_t b; memcpy(&b, p, 2); return flexar::bf16_to_f32(b); }
    case FLEXAR_INT32: { int32_t x; memcpy(&x, p, 4); return x; }
    case FLEXAR_UINT32: { uint32_t x; memcpy(&x, p, 4); return x; }
    case FLEXAR_INT64: { int64_t x; memcpy(&x, p, 8); return (double)x; }
    case FLEXAR_UINT64: { uint64_t x; memcpy(&x, p, 8); return (double)x; }
    case FLEXAR_INT16: { int16_t x; memcpy(&x, p, 2); return x; }
    case FLEXAR_UINT16: { uint16_t x; memcpy(&x, p, 2); return x; }
    case FLEXAR_INT8: { int8_t x; memcpy(&x, p, 1); return x; }
    default: { uint8_t x; memcpy(&x, p, 1); return x; }
  }
}

}  // namespace

int main(int argc, char** argv) {
  int provided = 0;
  MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &provided);
  int rank, nranks;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &nranks);

  Args a;
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) die("missing value for " + s);
      return argv[++i];
    };
    if (s == "--size") a.size = parse_size(next());
    else if (s == "--repeat") a.repeat = atoi(next().c_str());
    else if (s == "--to-file") a.to_file = true;
    else if (s == "--comm-type") a.comm = next();
    else if (s == "--tag") a.tag = next();
    else if (s == "--mem") a.mem = next();
    else if (s == "--dtype") a.dtype = next();
    else if (s == "--op") a.op = next();
    else if (s == "--algo") a.algo = next();
    else if (s == "--warmup") a.warmup = atoi(next().c_str());
    else if (s == "--check") a.check = true;
    else if (s == "--sweep") {
      std::string v = next();
      size_t c = v.find(':');
      if (c == std::string::npos) die("--sweep MIN:MAX");
      a.sweep_min = parse_size(v.substr(0, c));
      a.sweep_max = parse_size(v.substr(c + 1));
    } else if (s == "--version") {
      if (rank == 0)
        printf("----------\nflexar standalone benchmark\nversion: %s (library %s)\n", FLEXAR_GIT_VERSION,
               flexar_version());
      MPI_Finalize();
      return 0;
    } else {
      die("unknown parameter: " + s);  // reference: LOG(FATAL)
    }
  }
  if (a.comm == "flextree") a.comm = "flexar";
  if (a.comm != "flexar" && a.comm != "mpi" && a.comm != "rccl") die("unknown comm type: " + a.comm);
  const int dt = fx_dtype(a.dtype), op = fx_op(a.op);
  if (dt < 0 || op < 0) die("bad --dtype/--op");
  int ngpu = 0;
  if (hipGetDeviceCount(&ngpu) != hipSuccess) ngpu = 0;
  bool device = a.mem == "device" || (a.mem == "auto" && ngpu > 0);
  if (device && ngpu == 0) die("--mem device needs a GPU");
  if (a.comm == "rccl" && !device) die("rccl needs device buffers");
  if (device) {
    MPI_Comm local;
    MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &local);
    int lr;
    MPI_Comm_rank(local, &lr);
    MPI_Comm_free(&local);
    (void)hipSetDevice(lr % ngpu);
  }
  if (!a.algo.empty()) setenv("FLEXAR_ALGO", a.algo.c_str(), 1);
  const size_t es = flexar_dtype_size(dt);

  ncclComm_t nc = nullptr;
  if (a.comm == "rccl") {
    ncclUniqueId id;
    if (rank == 0) ncclGetUniqueId(&id);
    MPI_Bcast(&id, sizeof(id), MPI_BYTE, 0, MPI_COMM_WORLD);
    if (ncclCommInitRank(&nc, nranks, id, rank) != ncclSuccess) die("ncclCommInitRank failed");
  }

  std::vector<size_t> sizes;
  if (a.sweep_max) {
    for (size_t b = std::max<size_t>(a.sweep_min, es); b <= a.sweep_max; b *= 2) sizes.push_back(b / es);
  } else {
    sizes.push_back(a.size);
  }

  if (rank == 0) {
    std::ostringstream ss;
    ss << "configuration: \n  - total_peers: " << nranks << "\n  - data_size: " << a.size << "\n  - repeat: " << a.repeat
       << "\n  - to_file: " << (a.to_file ? "true" : "false");
    if (a.to_file && !a.tag.empty()) ss << "\n  - file tag: " << a.tag;
    ss << "\n  - communication method: " << a.comm << "\n  - memory: " << (device ? "device (HBM)" : "host")
       << "\n  - dtype/op: " << a.dtype << "/" << a.op;
    const char* ft = getenv("FT_TOPO");
    if (a.comm == "flexar")
      ss << "\n  - algorithm: " << (getenv("FLEXAR_ALGO") ? getenv("FLEXAR_ALGO") : (ft ? (std::string("FT_TOPO=") + ft).c_str() : "auto"));
    fprintf(stderr, "%s\n", ss.str().c_str());
    if (a.sweep_max)
      printf("%12s %12s %10s %10s %10s %10s\n", "size(B)", "count", "time(us)", "min(us)", "algbw", "busbw");
  }

  std::vector<double> times;
  double last_avg = 0, last_min = 0;
  std::vector<char> hsrc, hres;
  for (size_t n : sizes) {
    fill_host(hsrc, dt, n, rank);
    void* buf = nullptr;
    if (device) {
      if (hipMalloc(&buf, std::max<size_t>(n * es, 16)) != hipSuccess) die("hipMalloc failed");
      (void)hipMemcpy(buf, hsrc.data(), n * es, hipMemcpyHostToDevice);
    } else {
      buf = malloc(std::max<size_t>(n * es, 16));
      memcpy(buf, hsrc.data(), n * es);
    }
    auto reset = [&] {
      if (device) (void)hipMemcpy(buf, hsrc.data(), n * es, hipMemcpyHostToDevice);
      else memcpy(buf, hsrc.data(), n * es);
    };
    auto run_once = [&] {
      int rc = MPI_SUCCESS;
      if (a.comm == "flexar") {
        if (mpi_dtype(dt) != MPI_DATATYPE_NULL && mpi_op(op) != MPI_OP_NULL) {
          rc = MPI_Allreduce_FT_large(MPI_IN_PLACE, buf, n, mpi_dtype(dt), mpi_op(op), MPI_COMM_WORLD);
        } else {  // bf16/fp16/fp8 or AVG have no MPI handle: call the flexar C API directly
          if (!device) die("this dtype/op needs --mem device");
          static flexar_comm_t dc = flexar::mpi::device_comm(MPI_COMM_WORLD);
          if (nranks > 1)  // registration / zero-copy agreement, as MPI_Allreduce_FT does (mpi_mod.hpp zc_prepare)
            (void)flexar::mpi::zc_prepare(MPI_COMM_WORLD, buf, buf, n * es);
          rc = flexar_allreduce(dc, buf, buf, n, dt, op, nullptr);
        }
      } else if (a.comm == "mpi") {
        if (device) die("vendor MPI_Allreduce is not GPU-aware here: use --comm-type rccl");
        rc = MPI_Allreduce(MPI_IN_PLACE, buf, (int)n, mpi_dtype(dt), mpi_op(op), MPI_COMM_WORLD);
      } else {
        rc = ncclAllReduce(buf, buf, n, nccl_dtype(dt), (ncclRedOp_t)(op == FLEXAR_AVG ? ncclAvg : op), nc, nullptr);
      }
      if (device) (void)hipDeviceSynchronize();
      if (rc != 0) die("allreduce failed");
    };
    for (int w = 0; w < a.warmup; ++w) {
      if (a.check) reset();
      run_once();
    }
    times.clear();
    double sum = 0, mn = 1e30;
    for (int i = 0; i < a.repeat; ++i) {
      if (a.check) reset();
      MPI_Barrier(MPI_COMM_WORLD);
      flexar::HostTimer tm;  // steady_clock (the reference uses MPI_Wtime, benchmark.cpp:152-154)
      run_once();
      double t = tm.seconds(), tmax = 0;
      MPI_Allreduce(&t, &tmax, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);  // D12: max over ranks
      times.push_back(tmax);
      sum += tmax;
      mn = std::min(mn, tmax);
    }
    last_avg = sum / std::max(1, a.repeat);
    last_min = mn;
    if (a.check) {
      reset();
      run_once();
      hres.resize(n * es);
      if (device) (void)hipMemcpy(hres.data(), buf, n * es, hipMemcpyDeviceToHost);
      else memcpy(hres.data(), buf, n * es);
      size_t bad = 0;
      for (size_t i = 0; i < n; ++i) {
        double want = 0;
        for (int r = 0; r < nranks; ++r) {
          double v = (double)((i + r) % 8);
          if (op == FLEXAR_SUM || op == FLEXAR_AVG) want += v;
          else if (op == FLEXAR_MAX) want = r ? std::max(want, v) : v;
          else if (op == FLEXAR_MIN) want = r ? std::min(want, v) : v;
          else want = r ? want : v;  // other ops: only checked via tests
        }
        if (op == FLEXAR_AVG) want /= nranks;
        if ((op <= FLEXAR_AVG && op != FLEXAR_PROD) && std::fabs(host_val(hres, dt, i) - want) > 1e-3 * std::max(1.0, want)) ++bad;
      }
      size_t tot = 0;
      MPI_Allreduce(&bad, &tot, 1, MPI_UNSIGNED_LONG, MPI_SUM, MPI_COMM_WORLD);
      if (rank == 0) fprintf(stderr, "check n=%zu: %s (%zu wrong elements over all ranks)\n", n, tot ? "FAILED" : "ok", tot);
      if (tot) die("verification failed");
    }
    if (!a.check) {  // the reference's CHECK line prints the final buffer (benchmark.cpp:180-189)
      hres.resize(n * es);
      if (device) (void)hipMemcpy(hres.data(), buf, n * es, hipMemcpyDeviceToHost);
      else memcpy(hres.data(), buf, n * es);
    }
    if (a.comm == "flexar" && device && rank == 0) {  // the schedule the last call ran (zero copy or staging)
      char spec[256] = {0};
      if (flexar::mpi::dev_holder(MPI_COMM_WORLD) &&
          flexar_comm_last_spec(flexar::mpi::dev_holder(MPI_COMM_WORLD)->c, spec, sizeof(spec)) == 0 && spec[0])
        fprintf(stderr, "schedule n=%zu: %s\n", n, spec);
    }
    if (a.sweep_max && rank == 0) {
      double bytes = (double)n * es;
      double alg = bytes / last_avg / 1e9;
      printf("%12.0f %12zu %10.2f %10.2f %10.2f %10.2f\n", bytes, n, last_avg * 1e6, last_min * 1e6, alg,
             alg * 2.0 * (nranks - 1) / nranks);
      fflush(stdout);
    }
    if (device) (void)hipFree(buf);
    else free(buf);
  }

  // reference CHECK print (benchmark.cpp:180-189) without the out-of-bounds read for small sizes
  if (!a.sweep_max) {
    for (int r = 0; r <= nranks; ++r) {
      MPI_Barrier(MPI_COMM_WORLD);
      if (r == rank + 1 && hres.size()) {
        std::ostringstream ss;
        ss << "CHECK " << rank << ": ";
        for (size_t i = 9; i < std::min<size_t>(20, a.size); ++i) ss << host_val(hres, dt, i) << " ";
        printf("%s\n", ss.str().c_str());
        fflush(stdout);
      }
    }
  }
  if (rank == 0 && a.to_file) {
    std::ostringstream ss;
    if (!a.tag.empty()) ss << a.tag << ".";
    ss << nranks << "." << a.size << ".";
    if (a.comm == "flexar") ss << (getenv("FLEXAR_ALGO") ? getenv("FLEXAR_ALGO") : (getenv("FT_TOPO") ? getenv("FT_TOPO") : "auto"));
    else ss << a.comm;
    ss << ".ar_test." << time(nullptr) << ".txt";
    std::ofstream f(ss.str());
    for (double t : times) f << t << "\n";
  }
  if (rank == 0)
    fprintf(stderr, "\nDONE, average time: %g, min time: %g\n", last_avg, last_min);
  if (nc) ncclCommDestroy(nc);
  MPI_Finalize();
  return 0;
}
