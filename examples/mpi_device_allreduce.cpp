// Drop-in MPI_Allreduce_FT on HBM buffers (the reference's API, allreduce_over_mpi/mpi_mod.hpp:1167-1221).
//
//   g++ -std=c++17 -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Icsrc/include -I$MPI/include \
//       examples/mpi_device_allreduce.cpp -o mpi_device_allreduce \
//       -Lallreduce_over_mpi_amd/_lib -lflexar -L/opt/rocm/lib -lamdhip64 -L$MPI/lib -lmpi
//   mpirun -np 8 ./mpi_device_allreduce
//
// One rank per GPU: the device buffer is reduced by the flexar executor over xGMI (workspaces mapped
// once through MPI_Allgather of IPC handles); FT_TOPO / FLEXAR_ALGO pick the algorithm as in the reference.
#include <hip/hip_runtime.h>
#include <mpi.h>

#include <cstdio>
#include <vector>

#include "flexar/mpi_mod.hpp"

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank, size, ngpu = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  (void)hipGetDeviceCount(&ngpu);
  (void)hipSetDevice(ngpu ? rank % ngpu : 0);
  const int n = 1 << 24;  // 64 MiB of fp32
  std::vector<float> h(n, (float)(rank + 1));
  float* d = nullptr;
  (void)hipMalloc(&d, n * sizeof(float));
  (void)hipMemcpy(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice);
  MPI_Allreduce_FT(MPI_IN_PLACE, d, n, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD);  // stream-ordered on stream 0
  (void)hipMemcpy(h.data(), d, n * sizeof(float), hipMemcpyDeviceToHost);
  const float want = size * (size + 1) / 2.0f;
  size_t bad = 0;
  for (int i = 0; i < n; ++i) bad += h[i] != want;
  if (rank == 0) printf("MPI_Allreduce_FT on device buffers: %s (%zu wrong)\n", bad ? "FAILED" : "ok", bad);
  (void)hipFree(d);
  MPI_Finalize();
  return bad ? 1 : 0;
}
