// latency_floor.hip — where the single-instance callback time goes (scripts only).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/latency_floor.hip -Iinclude
//        -Lcentroidalplanner_amd -lcpl_mi355x -Wl,-rpath,$PWD/centroidalplanner_amd -o build/latency_floor
// Times (µs per call, best-of-5 means over 2000 calls): an empty kernel + hipStreamSynchronize; an
// empty kernel reading 40 doubles from and writing 200 doubles to pinned coherent host memory; the
// eval with device buffers (B = 1) + sync; the same with pinned host buffers as device pointers;
// cpl_eval_batch_host (B = 1, pageable arrays); the library's host-side work alone (a B = 0 call).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

#include "cpl_mi355x.h"

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));            \
      return 1;                                                                                 \
    }                                                                                           \
  } while (0)
#define CC(x)                                                                                   \
  do {                                                                                          \
    int32_t s_ = (x);                                                                           \
    if (s_ != CPL_OK) {                                                                         \
      std::fprintf(stderr, "%s:%d cpl status %d: %s\n", __FILE__, __LINE__, s_, cpl_last_error()); \
      return 1;                                                                                 \
    }                                                                                           \
  } while (0)

__global__ void k_empty() {}
struct Big {
  double v[250];  // a kernel-argument block of the eval kernel's size (~2 KiB)
};
__global__ void k_big(const Big b, double* y) {
  if (threadIdx.x == 0 && b.v[0] == 12345.0) y[0] = b.v[1];
}
__global__ void k_touch(const double* __restrict__ x, double* __restrict__ y, int nx, int ny) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nx; i += blockDim.x) s += x[i];
  for (int i = threadIdx.x; i < ny; i += blockDim.x) y[i] = s + i;
}

static double time_us(const std::function<int()>& f, int reps = 2000) {
  double best = 1e30;
  for (int round = 0; round < 5; ++round) {
    for (int i = 0; i < 50; ++i) f();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) f();
    const auto t1 = std::chrono::steady_clock::now();
    best = std::min(best, std::chrono::duration<double, std::micro>(t1 - t0).count() / reps);
  }
  return best;
}

int main() {
  cpl_problem_desc d;
  CC(cpl_desc_init(&d, 4, CPL_ENV_GROUND, 100.0));
  int32_t n, m, nnz;
  CC(cpl_dims(&d, &n, &m, &nnz));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  double *dx, *dg, *dj, *hx, *hg, *hj;
  CK(hipMalloc(&dx, 8 * n));
  CK(hipMalloc(&dg, 8 * m));
  CK(hipMalloc(&dj, 8 * nnz));
  CK(hipHostMalloc(&hx, 8 * n, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc(&hg, 8 * m, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc(&hj, 8 * nnz, hipHostMallocCoherent | hipHostMallocMapped));
  std::vector<double> x(n, 0.5), g(m), j(nnz);
  for (int i = 0; i < n; ++i) hx[i] = x[i];
  CK(hipMemcpy(dx, x.data(), 8 * n, hipMemcpyHostToDevice));

  int bad = 0;
  auto chk = [&](hipError_t e) { bad |= e != hipSuccess; return 0; };
  const double empty = time_us([&] {
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
    return chk(hipStreamSynchronize(s));
  });
  Big big{};
  const double empty_big = time_us([&] {
    hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, big, dg);
    return chk(hipStreamSynchronize(s));
  });
  const double touch = time_us([&] {
    hipLaunchKernelGGL(k_touch, dim3(1), dim3(256), 0, s, hx, hj, n, m + nnz);
    return chk(hipStreamSynchronize(s));
  });
  const double dev_eval = time_us([&] {
    bad |= cpl_eval_batch(&d, 1, dx, nullptr, nullptr, dg, dj, nullptr, nullptr, s) != CPL_OK;
    return chk(hipStreamSynchronize(s));
  });
  const double pinned_eval = time_us([&] {
    bad |= cpl_eval_batch(&d, 1, hx, nullptr, nullptr, hg, hj, nullptr, nullptr, s) != CPL_OK;
    return chk(hipStreamSynchronize(s));
  });
  const double host_entry = time_us([&] {
    bad |= cpl_eval_batch_host(&d, 1, x.data(), nullptr, nullptr, g.data(), j.data(), nullptr, nullptr, nullptr, 0) !=
           CPL_OK;
    return 0;
  });
  const double host_side = time_us([&] {
    bad |= cpl_eval_batch(&d, 0, dx, nullptr, nullptr, dg, dj, nullptr, nullptr, s) != CPL_OK;
    return 0;
  });
  // the same device-buffer eval with the tile-stationary kernel forced (cpl_set_tuning variant 3)
  CC(cpl_set_tuning(3, 0, 256, 1, 0));
  const double dev_eval_tile = time_us([&] {
    bad |= cpl_eval_batch(&d, 1, dx, nullptr, nullptr, dg, dj, nullptr, nullptr, s) != CPL_OK;
    return chk(hipStreamSynchronize(s));
  });
  CC(cpl_set_tuning(0, 0, 256, 1, 0));
  const double launch_only = time_us([&] {
    bad |= cpl_eval_batch(&d, 1, dx, nullptr, nullptr, dg, dj, nullptr, nullptr, s) != CPL_OK;
    return 0;
  }, 200);
  CK(hipStreamSynchronize(s));
  std::printf(
      "{\"empty_kernel_sync_us\": %.2f, \"host_memory_touch_kernel_sync_us\": %.2f, \"eval_device_buffers_sync_us\": "
      "%.2f, \"eval_pinned_host_buffers_sync_us\": %.2f, \"cpl_eval_batch_host_us\": %.2f, \"eval_b0_host_side_us\": "
      "%.2f, \"eval_launch_enqueue_us\": %.2f, \"eval_device_buffers_tile_kernel_sync_us\": %.2f, "
      "\"empty_kernel_2kib_args_sync_us\": %.2f, \"errors\": %d}\n",
      empty, touch, dev_eval, pinned_eval, host_entry, host_side, launch_only, dev_eval_tile, empty_big, bad);
  return bad;
}
