// flexar copy-engine ("dma") allreduce and the standalone reduction chain.
#include "comm_internal.hpp"

namespace flexar {

// dst (and dst2, if given) = scale * OP(srcs[0..nsrc)) over `count` elements: groups of kMaxSrc
// sources chain through dst (fan-in > 8: dst joins the next group; only the last group scales and
// writes dst2).
int reduce_chain(char* dst, char* dst2, const char* const* srcs, int nsrc, uint64_t count, int dtype,
                        int op, float fs, hipStream_t st, int proto) {
  const size_t es = dtype_size(dtype);
  // FLEXAR_REDUCE_GRID: workgroup cap of the standalone reduction (A/B; default 1024, one per 64 KiB below it)
  static const uint64_t cap = std::max<uint64_t>(1, std::min<uint64_t>(env_u64("FLEXAR_REDUCE_GRID", 1024), 65535));
  int grid = (int)std::min<uint64_t>(cap, std::max<uint64_t>(1, count * es / (64 * 1024)));
  int done = 0;
  while (done < nsrc) {
    SrcTable t;
    memset(&t, 0, sizeof(t));
    int k = 0;
    if (done > 0) t.p[k++] = dst;
    while (k < (int)kMaxSrc && done < nsrc) t.p[k++] = srcs[done++];
    const bool last = done >= nsrc;
    uintptr_t al = (uintptr_t)dst | (last && dst2 ? (uintptr_t)dst2 : 0);
    for (int i = 0; i < k; ++i) al |= (uintptr_t)t.p[i];
    LaunchArgs la;
    la.kind = LAUNCH_REDUCE;
    la.srcs = t;
    la.nsrc = k;
    la.dst = dst;
    la.dst2 = last ? dst2 : nullptr;
    la.n = count;
    la.scale = last ? fs : 1.0f;
    // the standalone reduction takes the grid-interleaved form (device_exec.hpp reduce_interleaved);
    // FLEXAR_REDUCE_SLICES=1 keeps per-workgroup slices (A/B)
    static const bool slices = env_u64("FLEXAR_REDUCE_SLICES", 0) != 0;
    la.vec = (vec_ok_for(al) ? 1 : 0) | (proto != PM_WT && !slices ? 2 : 0);
    la.grid = grid;
    la.stream = st;
    la.proto = proto;
    la.tag = proto == PM_WT ? "dma: reduce of the landed blocks" : "flexar_reduce";
    la.bytes = count * es;
    int rc = launch_dtype(dtype, op, la);
    if (rc) return rc;
  }
  return 0;
}

// ---- copy-engine ("dma") allreduce ------------------------------------------------------------
// The flat two-shot exchange with the bytes moved by copy engines instead of CUs, so an allreduce
// overlapped with compute (DDP backward) takes no CUs beyond a short reduce (SURVEY.md §5.8 (a),
// the reference's MPI_Isend/Irecv per block, mpi_mod.hpp:662-765, as one peer copy per peer). A call is
// split into pieces whose N landing slots + 1 result slot fit one staging parity half; piece k runs
//   RS   on peer p's reduce-scatter stream: copy my block p of piece k into p's landing slot r, then write
//        flag (kDmaSlotRS, r) = e_k into p's flags (stream-ordered after the copy);
//   RED  on the caller's stream: wait for every peer's RS flag e_k, reduce my block (write-through) into
//        OUT and my result slot, write flag (kDmaSlotAG, r) = e_k to every peer;
//   AG   on peer q's all-gather stream: wait for q's AG flag e_k, copy q's result slot into OUT block q.
// Pipelined: the reference serialises send -> recv -> reduce per stage
// (mpi_mod.hpp:988-1029); here the streams of different phases run concurrently, so the SDMA copies of
// piece k+1 overlap the reduce of piece k and the all-gather copies of piece k overlap the reduce-scatter
// copies of piece k+1. Pieces alternate staging halves (parity = epoch & 1); reusing a half is safe
// because piece k+2's RS copy into p waits for my AG copy of piece k from p (event per peer and parity),
// which followed p's AG flag, which p wrote after reducing piece k out of that half - and p reduces piece
// k+2 (overwriting its result slot) only after my RS flag of k+2. The host enqueues RS(k), RED(k),
// AG(k), RS(k+1), ...: every wait depends only on earlier-enqueued work of some rank, so hardware queues
// shared by several streams cannot deadlock.
static int dma_init(flexar_comm* c) {
  if (c->dma_ready) return 0;
  FX_HIP(hipSetDevice(c->device));
  for (int p = 0; p < c->nranks; ++p) {
    if (p == c->rank) continue;
    FX_HIP(hipStreamCreateWithFlags(&c->dma_st[p], hipStreamNonBlocking));
    FX_HIP(hipStreamCreateWithFlags(&c->dma_ag[p], hipStreamNonBlocking));
    FX_HIP(hipEventCreateWithFlags(&c->dma_join[p], hipEventDisableTiming));
    FX_HIP(hipEventCreateWithFlags(&c->dma_rs_end[p], hipEventDisableTiming));
    FX_HIP(hipEventCreateWithFlags(&c->dma_ag_done[p][0], hipEventDisableTiming));
    FX_HIP(hipEventCreateWithFlags(&c->dma_ag_done[p][1], hipEventDisableTiming));
  }
  FX_HIP(hipEventCreateWithFlags(&c->dma_fork, hipEventDisableTiming));
  c->dma_ready = true;
  return 0;
}

// elements per dma piece: N + 1 block slots must fit one parity half (FLEXAR_CHUNK_BYTES caps it too)
static uint64_t dma_piece(flexar_comm* c, uint64_t count, uint32_t es) {
  const uint64_t slot = c->exec_half / (uint64_t)(c->nranks + 1) / kStageAlignBytes * kStageAlignBytes;
  uint64_t per_block = std::max<uint64_t>(1, slot / es);
  if (c->chunk_bytes) per_block = std::max<uint64_t>(1, std::min<uint64_t>(per_block, c->chunk_bytes / es / c->nranks));
  return std::min<uint64_t>(count, per_block * (uint64_t)c->nranks);
}

static int dma_wait(flexar_comm* c, uint32_t slot, const int* srcs, int n, uint64_t e, hipStream_t st) {
  DmaWait w;
  memset(&w, 0, sizeof(w));
  w.flags = c->flags;
  for (int i = 0; i < n; ++i) {
    w.idx[i] = (uint32_t)flag_index(slot, (uint32_t)srcs[i], 0);
    w.src[i] = (uint32_t)srcs[i];
  }
  w.n = (uint32_t)n;
  w.slot = slot;
  w.value = e;
  w.timeout_ticks = c->timeout_ticks;
  w.err = c->err_dev;
  CrumbArgs ca;
  ca.type = CRUMB_LAUNCH;
  ca.what = "dma_wait_kernel";
  ca.rank = (int16_t)c->rank;
  ca.nranks = (int16_t)c->nranks;
  ca.epoch = e;
  ca.label = slot == kDmaSlotRS ? "dma: wait for the peers' reduce-scatter flags" : "dma: wait for a peer's all-gather flag";
  crumb(ca);
  hipLaunchKernelGGL(dma_wait_kernel, dim3(1), dim3(64), 0, st, w);
  FX_HIP(hipGetLastError());
  return 0;
}

// phase: 0 = fork (first piece only), 1 = RS copies of the piece, 2 = reduce, 3 = AG, 4 = join (after the
// last piece). `e` is the piece's epoch.
static int dma_phase(flexar_comm* c, int phase, const char* in, char* out, uint64_t count, int dtype, int op,
                     float fs, hipStream_t st, uint64_t e) {
  const int N = c->nranks, r = c->rank;
  const uint64_t es = dtype_size(dtype);
  const uint64_t B = (count + N - 1) / N;
  const uint64_t Bb = (B * es + kStageAlignBytes - 1) / kStageAlignBytes * kStageAlignBytes;
  const uint64_t par = (e & 1) ? c->half_bytes : 0;
  auto len = [&](int i) -> uint64_t {
    const uint64_t s0 = (uint64_t)i * B;
    return s0 >= count ? 0 : std::min<uint64_t>(B, count - s0);
  };
  {
    CrumbArgs ca;
    ca.type = CRUMB_COPY;
    ca.what = "dma phase";
    ca.rank = (int16_t)r;
    ca.nranks = (int16_t)N;
    ca.epoch = e;
    ca.bytes = count * es;
    static const char* names[] = {"fork", "reduce-scatter copies (hipMemcpyAsync into peers' staging) + flag writes",
                                  "wait + reduce + all-gather flag writes", "all-gather copies from peers' result slots",
                                  "join + epoch_set_kernel"};
    ca.label = names[phase < 0 || phase > 4 ? 0 : phase];
    crumb(ca);
  }
  if (phase == 0) {  // the streams start after everything the caller enqueued before this call
    FX_HIP(hipEventRecord(c->dma_fork, st));
    for (int p = 0; p < N; ++p) {
      if (p == r) continue;
      FX_HIP(hipStreamWaitEvent(c->dma_st[p], c->dma_fork, 0));
      FX_HIP(hipStreamWaitEvent(c->dma_ag[p], c->dma_fork, 0));
    }
  } else if (phase == 1) {
    for (int j = 1; j < N; ++j) {
      const int p = (r + j) % N;
      hipStream_t s = c->dma_st[p];
      // p's landing slots / result slot of this parity were last used two pieces ago: my AG copy of that
      // piece from p (after p's AG flag, i.e. after p reduced it) must be complete
      FX_HIP(hipStreamWaitEvent(s, c->dma_ag_done[p][e & 1], 0));
      if (len(p))
        FX_HIP(hipMemcpyAsync(c->peer_stg[p] + par + (uint64_t)r * Bb, in + (uint64_t)p * B * es, len(p) * es,
                              hipMemcpyDeviceToDevice, s));
      FX_HIP(hipStreamWriteValue64(s, c->peer_flags[p] + flag_index(kDmaSlotRS, (uint32_t)r, 0), e, 0));
    }
  } else if (phase == 2) {
    int peers[kMaxRanks], np = 0;
    for (int j = 1; j < N; ++j) peers[np++] = (r + j) % N;
    int rc = dma_wait(c, kDmaSlotRS, peers, np, e, st);
    if (rc) return rc;
    if (len(r)) {
      const char* srcs[kMaxRanks];
      int ns = 0;
      srcs[ns++] = in + (uint64_t)r * B * es;
      for (int j = 0; j < np; ++j) srcs[ns++] = c->stg + par + (uint64_t)peers[j] * Bb;
      rc = reduce_chain(out + (uint64_t)r * B * es, c->stg + par + (uint64_t)N * Bb, srcs, ns, len(r), dtype, op, fs,
                        st, PM_WT);
      if (rc) return rc;
    }
    for (int j = 0; j < np; ++j)
      FX_HIP(hipStreamWriteValue64(st, c->peer_flags[peers[j]] + flag_index(kDmaSlotAG, (uint32_t)r, 0), e, 0));
  } else if (phase == 3) {
    for (int j = 1; j < N; ++j) {
      const int q = (r + j) % N;
      hipStream_t s = c->dma_ag[q];
      // q's AG flag: q reduced this piece, which needed my RS flag, which followed my RS copy out of an
      // in-place OUT block q - so the copy below cannot overwrite data my RS copy still reads
      int rc = dma_wait(c, kDmaSlotAG, &q, 1, e, s);
      if (rc) return rc;
      if (len(q))
        FX_HIP(hipMemcpyAsync(out + (uint64_t)q * B * es, c->peer_stg[q] + par + (uint64_t)N * Bb, len(q) * es,
                              hipMemcpyDeviceToDevice, s));
      FX_HIP(hipEventRecord(c->dma_ag_done[q][e & 1], s));
    }
    c->launches = e;
  } else {  // join: the caller's stream continues after every copy of the call; epochs advance to e
    for (int j = 1; j < N; ++j) {
      const int q = (r + j) % N;
      FX_HIP(hipEventRecord(c->dma_join[q], c->dma_ag[q]));
      FX_HIP(hipEventRecord(c->dma_rs_end[q], c->dma_st[q]));
      FX_HIP(hipStreamWaitEvent(st, c->dma_join[q], 0));
      FX_HIP(hipStreamWaitEvent(st, c->dma_rs_end[q], 0));
    }
    hipLaunchKernelGGL(epoch_set_kernel, dim3(1), dim3(256), 0, st, c->epochs, e);
    FX_HIP(hipGetLastError());
  }
  return 0;
}

int run_dma(flexar_comm* const* cs, int ncomm, const char* const* ins, char* const* outs, uint64_t count,
                   int dtype, int op, float fs, hipStream_t st) {
  const uint32_t es = (uint32_t)dtype_size(dtype);
  for (int i = 0; i < ncomm; ++i) {
    int rc = dma_init(cs[i]);
    if (rc) return rc;
  }
  const uint64_t piece = dma_piece(cs[0], count, es);
  const uint64_t e0 = cs[0]->launches;
  auto each = [&](int phase, uint64_t off, uint64_t n, uint64_t e) {
    // phase by phase across the group: a rank's waits are enqueued after every rank's signals
    for (int i = 0; i < ncomm; ++i) {
      int rc = dma_phase(cs[i], phase, ins[i] + off * es, outs[i] + off * es, n, dtype, op, fs, st, e);
      if (rc) return rc;
    }
    return 0;
  };
  // FLEXAR_DMA_SERIAL=1: join + fork around every piece (the round-1 serial schedule, for A/B measurements)
  static const bool serial = env_u64("FLEXAR_DMA_SERIAL", 0) != 0;
  int rc = each(0, 0, count, e0 + 1);
  uint64_t e = e0;
  for (uint64_t off = 0; off < count && !rc; off += piece) {
    const uint64_t n = std::min<uint64_t>(piece, count - off);
    ++e;
    if (serial && off) rc = each(4, 0, count, e - 1) || each(0, 0, count, e);
    for (int phase = 1; phase <= 3 && !rc; ++phase) rc = each(phase, off, n, e);
  }
  if (!rc) rc = each(4, 0, count, e);
  return rc;
}

}  // namespace flexar

