// kkt_probe.hip — phase timing of cpl_kkt_kernel (scripts only, not part of the library).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DCPL_KKT_PROFILE scripts/kkt_probe.hip -o scripts/kkt_probe
// Random SPD-plus-structure systems (nw = 47, m = 30 by default: the 4-contact solve loop's size),
// batch 8192; prints the kernel time (HIP events, mode 0 and mode 1) and the mean clock64 cycles
// per phase (QR | Q accumulation | reduced Hessian | inertia/Cholesky | solve | refinement | store).
#include "../centroidalplanner_amd/csrc/cpl_kkt.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

namespace cpl {
int32_t fail(int32_t status, const std::string& msg) {
  std::fprintf(stderr, "fail %d: %s\n", status, msg.c_str());
  return status;
}
}  // namespace cpl

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

int main(int argc, char** argv) {
  const int B = argc > 1 ? std::atoi(argv[1]) : 8192;
  const int nw = argc > 2 ? std::atoi(argv[2]) : 47;
  const int m = argc > 3 ? std::atoi(argv[3]) : 30;
  std::mt19937_64 rng(7);
  std::normal_distribution<double> N(0.0, 1.0);
  std::vector<double> M((size_t)B * nw * nw), A((size_t)B * m * nw), r1((size_t)B * nw), r2((size_t)B * m),
      mu(B, 0.1), last(B, 0.0);
  for (int b = 0; b < B; ++b) {
    std::vector<double> X((size_t)nw * nw);
    for (auto& v : X) v = N(rng);
    for (int i = 0; i < nw; ++i)
      for (int j = 0; j < nw; ++j) {
        double s = 0.0;
        for (int k = 0; k < nw; ++k) s += X[i * nw + k] * X[j * nw + k];
        M[(size_t)b * nw * nw + i * nw + j] = s / nw + (i == j ? 0.1 : 0.0);
      }
    for (int i = 0; i < m * nw; ++i) A[(size_t)b * m * nw + i] = N(rng);
    for (int i = 0; i < nw; ++i) r1[(size_t)b * nw + i] = N(rng);
    for (int i = 0; i < m; ++i) r2[(size_t)b * m + i] = N(rng);
  }
  double *dM, *dA, *dr1, *dr2, *dmu, *dlast, *ddw, *ddy, *ddW, *ddC, *dws;
  int32_t* dinfo;
  long long* dprof;
  const int64_t per = kkt_ws_per(nw, m);
  CK(hipMalloc(&dM, M.size() * 8));
  CK(hipMalloc(&dA, A.size() * 8));
  CK(hipMalloc(&dr1, r1.size() * 8));
  CK(hipMalloc(&dr2, r2.size() * 8));
  CK(hipMalloc(&dmu, B * 8));
  CK(hipMalloc(&dlast, B * 8));
  CK(hipMalloc(&ddw, (size_t)B * nw * 8));
  CK(hipMalloc(&ddy, (size_t)B * m * 8));
  CK(hipMalloc(&ddW, B * 8));
  CK(hipMalloc(&ddC, B * 8));
  CK(hipMalloc(&dinfo, B * 4));
  CK(hipMalloc(&dws, (size_t)B * per * 8));
  CK(hipMalloc(&dprof, (size_t)B * 8 * 8));
  CK(hipMemcpy(dM, M.data(), M.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dr1, r1.data(), r1.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dr2, r2.data(), r2.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dmu, mu.data(), B * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dlast, last.data(), B * 8, hipMemcpyHostToDevice));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_kkt_prof), &dprof, sizeof(dprof)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int mode = 0; mode < 2; ++mode) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(e0));
      int st = cpl_kkt_solve(mode, B, nw, m, dM, dA, dr1, dr2, dmu, dlast, nullptr, ddw, ddy, ddW, ddC, dinfo, dws,
                             nullptr);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      if (st) return 2;
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    std::printf("mode %d: %.3f ms for %d systems (nw %d, m %d)\n", mode, best, B, nw, m);
    {  // FNV-1a of the outputs' bit patterns: variants of the kernel compare bit for bit
      std::vector<double> ow((size_t)B * nw), oy((size_t)B * m);
      CK(hipMemcpy(ow.data(), ddw, ow.size() * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(oy.data(), ddy, oy.size() * 8, hipMemcpyDeviceToHost));
      unsigned long long h = 1469598103934665603ull;
      for (const auto* v : {&ow, &oy})
        for (double d : *v) {
          unsigned long long bits;
          std::memcpy(&bits, &d, 8);
          h = (h ^ bits) * 1099511628211ull;
        }
      std::printf("  outputs hash %016llx\n", h);
    }
    if (mode == 0) {
      std::vector<long long> prof((size_t)B * 8);
      CK(hipMemcpy(prof.data(), dprof, prof.size() * 8, hipMemcpyDeviceToHost));
      const char* block_names[7] = {"QR", "Q accumulation", "rank + Z^T M Z", "inertia/Cholesky", "solve",
                                    "refinement", "store factors"};
      const char* wave_names[7] = {"QR", "Z accumulation", "rank + Z^T M Z", "inertia/Cholesky", "solve",
                                   "refinement", "store factors"};
      const char* const* names = kkt_wave_kernel_for(nw, m) ? wave_names : block_names;
      std::printf("  (%s kernel)\n", kkt_wave_kernel_for(nw, m) ? "one-wave" : "workgroup");
      for (int p = 0; p < 7; ++p) {
        double s = 0.0;
        for (int b = 0; b < B; ++b) s += (double)(prof[(size_t)b * 8 + p + 1] - prof[(size_t)b * 8 + p]);
        std::printf("  %-18s %9.0f cycles\n", names[p], s / B);
      }
    }
  }
  // occupancy sweep: the same mode-0 launch with extra dynamic LDS (argv[4..]: pad bytes), to see
  // how the kernel's time scales with resident workgroups per CU
  for (int a = 4; a < argc; ++a) {
    const size_t pad = (size_t)std::atol(argv[a]);
    const size_t lds = sizeof(double) * (size_t)kkt_launch_lds_doubles(nw, m, 0) + pad;
    int per_cu = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kkt_kernel_for(nw, m)),
                                                    KKT_THREADS, lds));
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(kkt_kernel_for(nw, m), dim3((unsigned)B), dim3(KKT_THREADS), lds, 0, 0, (int64_t)B, nw, m, dM, dA,
                         dr1, dr2, dmu, dlast, nullptr, ddw, ddy, ddW, ddC, dinfo, dws);
      CK(hipGetLastError());
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    std::printf("pad %zu B: LDS %zu B, %d workgroups/CU: mode 0 %.3f ms\n", pad, lds, per_cu, best);
  }
  return 0;
}
