// flexar registered buffers (zero copy "+zc"): IPC mappings of the callers' buffers.
#include "comm_internal.hpp"

extern "C" {

// ---- registered buffers (zero-copy "+zc") --------------------------------------------------------
// Registration blob: the IPC handle of the allocation holding the buffer and the buffer's place in it.
struct RegBlob {
  hipIpcMemHandle_t h;
  uint64_t offset;  // buffer start - allocation base
  uint64_t bytes;
  int32_t device, pad;
};
static_assert(sizeof(RegBlob) <= FLEXAR_REG_HANDLE_BYTES, "registration blob size");

size_t flexar_reg_handle_size(void) { return FLEXAR_REG_HANDLE_BYTES; }

static uint64_t buffer_id(const void* p) {
  unsigned long long id = 0;
  if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return (uint64_t)id;
}

// Drop registration i: its peer mappings close once no other registration uses them (caller holds mu
// and has synchronised the device).
static void reg_drop(flexar_comm* c, size_t i) {
  for (int p = 0; p < c->nranks; ++p) {
    if (p == c->rank) continue;
    auto it = c->ipc_maps.find(c->regs[i].key[p]);
    if (it == c->ipc_maps.end()) continue;
    if (--it->second.second == 0) {
      (void)hipIpcCloseMemHandle(it->second.first);
      c->ipc_maps.erase(it);
    }
  }
  c->regs.erase(c->regs.begin() + (long)i);
  (void)hipGetLastError();  // an ignored close failure must not surface in the caller's next launch
}

int flexar_reg_export(flexar_comm_t c, const void* ptr, size_t bytes, void* out) {
  if (!c || !ptr || !out || !bytes) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  FX_HIP(hipSetDevice(c->device));
  RegBlob b;
  memset(&b, 0, sizeof(b));
  if (c->nranks > 1 && !c->group_member) {
    void* base = nullptr;
    size_t size = 0;
    FX_HIP(hipMemGetAddressRange(&base, &size, const_cast<void*>(ptr)));
    if ((const char*)ptr + bytes > (const char*)base + size) {
      set_error("registered range exceeds its allocation");
      return FLEXAR_ERR_INVALID;
    }
    // Importing a peer allocation larger than ~1 GiB through HIP IPC after other imports hangs in
    // hipIpcOpenMemHandle on this platform (ROCm 7, dmabuf IPC; reproduced with hipMalloc'd and torch
    // allocations of 2 GiB+, bench/reg_repro.py), so such allocations are refused up front instead
    // (every rank then keeps the staging schedules). FLEXAR_REG_MAX_ALLOC overrides the cap.
    const uint64_t cap = env_u64("FLEXAR_REG_MAX_ALLOC", 1ull << 30);
    if (size > cap) {
      set_error("registering: the buffer lies in an allocation of " + std::to_string(size) + " bytes, above the " +
                std::to_string(cap) + "-byte cap for IPC-mapped registrations (allocate it on its own)");
      return FLEXAR_ERR_UNSUPPORTED;
    }
    FX_HIP(hipIpcGetMemHandle(&b.h, base));
    b.offset = (uint64_t)((const char*)ptr - (const char*)base);
    logf(LOG_DEBUG, c->rank, "registering: buffer %p (%zu bytes) lies in allocation %p (%zu bytes) at +%llu", ptr,
         bytes, base, size, (unsigned long long)b.offset);
  }
  b.bytes = bytes;
  b.device = c->device;
  memset(out, 0, FLEXAR_REG_HANDLE_BYTES);
  memcpy(out, &b, sizeof(b));
  return 0;
}

// Collective in effect: every rank opens the blobs of all ranks (rank-major, flexar_reg_handle_size()
// bytes each) for its own buffer of the same size.
int flexar_reg_open(flexar_comm_t c, const void* ptr, size_t bytes, const void* all, int* id_out) {
  if (!c || !ptr || !all || !id_out) { set_error("null argument"); return FLEXAR_ERR_INVALID; }
  if (!c->connected && c->nranks > 1) { set_error("communicator not connected"); return FLEXAR_ERR_STATE; }
  if (c->nranks > 1 && !c->ipc) { set_error("zero-copy needs IPC peer access (this communicator runs RCCL messages)"); return FLEXAR_ERR_UNSUPPORTED; }
  if (c->group_member) {
    set_error("in-process groups address every rank's buffers directly: no registration needed");
    return FLEXAR_ERR_INVALID;
  }
  std::lock_guard<std::mutex> lk(c->mu);
  FX_HIP(hipSetDevice(c->device));
  // a new registration replaces an overlapping old one whose allocation is gone (freed, address reused:
  // stale peer mappings) or which it contains (a call outgrew it); every rank registers together, so
  // every rank drops it. Other overlaps (a tensor inside a registered arena) coexist.
  logf(LOG_DEBUG, c->rank, "registering %zu bytes at %p (%zu registrations)", bytes, ptr, c->regs.size());
  bool synced = false;
  for (size_t i = c->regs.size(); i-- > 0;) {
    const flexar_comm::Reg& o = c->regs[i];
    const bool overlap = (const char*)ptr < o.base + o.bytes && o.base < (const char*)ptr + bytes;
    const bool contains = (const char*)ptr <= o.base && o.base + o.bytes <= (const char*)ptr + bytes;
    const bool stale = o.bufid && buffer_id(o.base) != o.bufid;
    if (overlap && (contains || stale)) {
      if (!synced) FX_HIP(hipDeviceSynchronize());
      synced = true;
      reg_drop(c, i);
    }
  }
  flexar_comm::Reg g;
  g.id = c->next_reg++;
  g.bufid = c->nranks > 1 && !c->group_member ? buffer_id(ptr) : 0;
  g.base = (char*)ptr;
  g.bytes = bytes;
  g.aligned = ((uintptr_t)ptr & 15) == 0;
  for (int p = 0; p < kMaxRanks; ++p) g.peer[p] = nullptr;
  std::vector<std::string> opened;
  auto undo = [&]() {
    for (const std::string& k : opened) {
      auto it = c->ipc_maps.find(k);
      if (it != c->ipc_maps.end() && --it->second.second == 0) {
        (void)hipIpcCloseMemHandle(it->second.first);
        c->ipc_maps.erase(it);
      }
    }
    (void)hipGetLastError();  // the failed open (and any close) must not stay the thread's sticky error
  };
  for (int p = 0; p < c->nranks; ++p) {
    RegBlob b;
    memcpy(&b, (const char*)all + (size_t)p * FLEXAR_REG_HANDLE_BYTES, sizeof(b));
    if (b.bytes != bytes) {
      undo();
      set_error("rank " + std::to_string(p) + " registered " + std::to_string(b.bytes) + " bytes, this rank " +
                std::to_string(bytes) + " (corresponding buffers must have the same size)");
      return FLEXAR_ERR_INVALID;
    }
    if (p == c->rank) { g.peer[p] = (char*)ptr; continue; }
    if (b.offset & 15) g.aligned = false;
    const std::string key = std::to_string(p) + ":" + std::string((const char*)&b.h, sizeof(b.h));
    auto it = c->ipc_maps.find(key);
    char* mapped = nullptr;
    if (it != c->ipc_maps.end()) {
      mapped = it->second.first;
      it->second.second++;
    } else {
      void* q = nullptr;
      logf(LOG_DEBUG, c->rank, "registering: opening rank %d's allocation (buffer at +%llu, %zu bytes)", p,
           (unsigned long long)b.offset, bytes);
      hipError_t e = hipIpcOpenMemHandle(&q, b.h, hipIpcMemLazyEnablePeerAccess);
      logf(LOG_DEBUG, c->rank, "registering: rank %d's allocation mapped (%s)", p, hipGetErrorString(e));
      if (e != hipSuccess) {
        undo();
        set_error("registering: mapping rank " + std::to_string(p) + "'s buffer failed: hipIpcOpenMemHandle: " +
                  hipGetErrorString(e));
        return FLEXAR_ERR_HIP;
      }
      mapped = (char*)q;
      c->ipc_maps[key] = {mapped, 1};
    }
    opened.push_back(key);
    g.key[p] = key;
    g.peer[p] = mapped + b.offset;
  }
  c->regs.push_back(g);
  *id_out = g.id;
  logf(LOG_INFO, c->rank, "registered buffer %d: %zu bytes (%zu registrations, %zu peer mappings)", g.id, bytes,
       c->regs.size(), c->ipc_maps.size());
  return 0;
}

// Drop a registration (every rank, after the calls using it completed): its peer mappings are closed
// once no other registration uses them.
int flexar_reg_close(flexar_comm_t c, int id) {
  if (!c) return FLEXAR_ERR_INVALID;
  std::lock_guard<std::mutex> lk(c->mu);
  for (size_t i = 0; i < c->regs.size(); ++i) {
    if (c->regs[i].id != id) continue;
    FX_HIP(hipSetDevice(c->device));
    FX_HIP(hipDeviceSynchronize());  // no call of ours still reads through the mappings
    reg_drop(c, i);
    return 0;
  }
  set_error("no registration " + std::to_string(id));
  return FLEXAR_ERR_INVALID;
}

// The registration holding [p, p + bytes): its id, 0 if none, -1 if the allocation behind the registered
// address is not the one registered any more (freed and reused: the peers' mappings are stale).
int flexar_reg_find(flexar_comm_t c, const void* p, size_t bytes) {
  if (!c || !p) return 0;
  std::lock_guard<std::mutex> lk(c->mu);
  const flexar_comm::Reg* r = reg_lookup(c, p, bytes);
  if (!r) return 0;
  if (r->bufid && buffer_id(p) != r->bufid) return -1;
  return r->id;
}

int flexar_reg_count(flexar_comm_t c) { return c ? (int)c->regs.size() : -1; }

int flexar_reg_ids(flexar_comm_t c, int* out, int max) {
  if (!c) return -1;
  std::lock_guard<std::mutex> lk(c->mu);
  int n = 0;
  for (const auto& r : c->regs)
    if (n < max && out) out[n++] = r.id;
  return (int)c->regs.size();
}

}  // extern "C"
