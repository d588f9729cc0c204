// Stand-alone probe of the stream primitives the copy-engine (dma) allreduce relies on:
// hipStreamWriteValue64 into uncached device memory, a polling wait kernel on another stream,
// and copy -> write ordering. Every step is bounded (device watchdog + alarm()).
#include <hip/hip_runtime.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>
#include <chrono>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("FAIL %s: %s\n", #x, hipGetErrorString(e_)); exit(2); } } while (0)

__global__ void wait_kernel(uint64_t* f, uint64_t v, uint32_t* timed_out) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < v) {
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 300000000ull) { *timed_out = 1; return; }  // 3 s
  }
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  alarm(60);
  uint64_t* flag;
  CK(hipExtMallocWithFlags((void**)&flag, 4096, hipDeviceMallocUncached));
  CK(hipMemset(flag, 0, 4096));
  uint32_t* to;
  CK(hipHostMalloc((void**)&to, 64, hipHostMallocMapped));
  *to = 0;
  uint32_t* to_d;
  CK(hipHostGetDevicePointer((void**)&to_d, to, 0));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));

  // T1: write value, read back
  double t = now_ms();
  CK(hipStreamWriteValue64(a, flag, 5, 0));
  CK(hipStreamSynchronize(a));
  uint64_t h = 0;
  CK(hipMemcpy(&h, flag, 8, hipMemcpyDeviceToHost));
  printf("T1 writevalue readback=%llu (%.3f ms)\n", (unsigned long long)h, now_ms() - t);
  fflush(stdout);

  // T2: wait kernel on b released by a write on a (write enqueued AFTER the wait)
  t = now_ms();
  hipLaunchKernelGGL(wait_kernel, dim3(1), dim3(1), 0, b, flag + 1, 7ull, to_d);
  CK(hipStreamWriteValue64(a, flag + 1, 7, 0));
  CK(hipStreamSynchronize(a));
  CK(hipStreamSynchronize(b));
  printf("T2 wait-kernel released by writevalue: timed_out=%u (%.3f ms)\n", *to, now_ms() - t);
  fflush(stdout);

  // T3: copy then write on a; b waits then copies back; check data
  const size_t n = 1 << 20;
  char *src, *mid, *dst;
  CK(hipMalloc(&src, n)); CK(hipMalloc(&mid, n)); CK(hipMalloc(&dst, n));
  CK(hipMemset(src, 0x5a, n)); CK(hipMemset(mid, 0, n)); CK(hipMemset(dst, 0, n));
  CK(hipDeviceSynchronize());
  *to = 0;
  t = now_ms();
  hipLaunchKernelGGL(wait_kernel, dim3(1), dim3(1), 0, b, flag + 2, 9ull, to_d);
  CK(hipMemcpyAsync(dst, mid, n, hipMemcpyDeviceToDevice, b));
  CK(hipMemcpyAsync(mid, src, n, hipMemcpyDeviceToDevice, a));
  CK(hipStreamWriteValue64(a, flag + 2, 9, 0));
  CK(hipStreamSynchronize(a));
  CK(hipStreamSynchronize(b));
  char* hb = (char*)malloc(n);
  CK(hipMemcpy(hb, dst, n, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < n; ++i) bad += hb[i] != 0x5a;
  printf("T3 copy->write->wait->copy: timed_out=%u bad=%zu (%.3f ms)\n", *to, bad, now_ms() - t);
  fflush(stdout);

  // T4: many streams (more than hardware queues) each waiting, released in reverse order
  const int S = 16;
  hipStream_t ss[S];
  for (int i = 0; i < S; ++i) CK(hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking));
  *to = 0;
  t = now_ms();
  for (int i = 0; i < S; ++i) hipLaunchKernelGGL(wait_kernel, dim3(1), dim3(1), 0, ss[i], flag + 16 + i, 3ull, to_d);
  for (int i = S - 1; i >= 0; --i) CK(hipStreamWriteValue64(ss[(i + 1) % S], flag + 16 + i, 3, 0));
  for (int i = 0; i < S; ++i) CK(hipStreamSynchronize(ss[i]));
  printf("T4 %d streams cross-released: timed_out=%u (%.3f ms)\n", S, *to, now_ms() - t);
  fflush(stdout);

  // T5: latency of write -> wait hand-off (100 round trips on two streams)
  t = now_ms();
  *to = 0;
  for (int i = 0; i < 100; ++i) {
    hipLaunchKernelGGL(wait_kernel, dim3(1), dim3(1), 0, b, flag + 40, (uint64_t)(i + 1), to_d);
    CK(hipStreamWriteValue64(a, flag + 40, (uint64_t)(i + 1), 0));
  }
  CK(hipStreamSynchronize(a));
  CK(hipStreamSynchronize(b));
  printf("T5 100 hand-offs: timed_out=%u (%.3f ms)\n", *to, now_ms() - t);
  printf("done\n");
  return 0;
}
