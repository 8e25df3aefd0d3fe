// kkt_ab.hip — the one-wave-per-system KKT kernel against the workgroup kernel (scripts only).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/kkt_ab.hip -o build/kkt_ab
// Random symmetric-positive-definite-plus-shift M, random A (full rank), nw = 47, m = 30 by default
// (argv: B nw m [rank_deficient_rows]); times mode 0 / mode 1 of both kernels (HIP events, best of
// 7) and reports the KKT residual of each solution and their difference.
#include "../centroidalplanner_amd/csrc/cpl_kkt.hip"

#include <cstdio>
#include <cstdlib>
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
  const int defrows = argc > 4 ? std::atoi(argv[4]) : 0;  // rows of A duplicated (rank deficiency)
  std::mt19937_64 rng(7);
  std::normal_distribution<double> N(0.0, 1.0);
  std::vector<double> M((size_t)B * nw * nw), A((size_t)B * m * nw), r1((size_t)B * nw), r2((size_t)B * m),
      mu(B, 0.1), last(B, 0.0);
  for (int b = 0; b < B; ++b) {
    std::vector<double> X((size_t)nw * nw);
    for (auto& v : X) v = N(rng);
    // indefinite on a few directions for some instances: exercises the delta_w retries
    const double shift = (b % 3 == 0) ? -0.5 : 0.1;
    for (int i = 0; i < nw; ++i)
      for (int j = 0; j <= i; ++j) {
        double s = 0.0;
        for (int k = 0; k < nw; ++k) s += X[i * nw + k] * X[j * nw + k];
        const double v = s / nw + (i == j ? shift : 0.0);
        M[(size_t)b * nw * nw + i * nw + j] = v;
        M[(size_t)b * nw * nw + j * nw + i] = v;
      }
    for (int i = 0; i < m * nw; ++i) A[(size_t)b * m * nw + i] = N(rng);
    for (int r = 0; r < defrows && r + 1 < m; ++r)
      for (int i = 0; i < nw; ++i) A[(size_t)b * m * nw + (r + 1) * nw + i] = A[(size_t)b * m * nw + i];
    for (int i = 0; i < nw; ++i) r1[(size_t)b * nw + i] = N(rng);
    for (int i = 0; i < m; ++i) r2[(size_t)b * m + i] = N(rng);
  }
  double *dM, *dA, *dr1, *dr2, *dmu, *dlast, *dws;
  double *dw[2], *dy[2], *dW[2], *dC[2];
  int32_t* info[2];
  const int64_t per = kkt_ws_per(nw, m);
  CK(hipMalloc(&dM, M.size() * 8));
  CK(hipMalloc(&dA, A.size() * 8));
  CK(hipMalloc(&dr1, r1.size() * 8));
  CK(hipMalloc(&dr2, r2.size() * 8));
  CK(hipMalloc(&dmu, B * 8));
  CK(hipMalloc(&dlast, B * 8));
  CK(hipMalloc(&dws, (size_t)B * per * 8));
  for (int v = 0; v < 2; ++v) {
    CK(hipMalloc(&dw[v], (size_t)B * nw * 8));
    CK(hipMalloc(&dy[v], (size_t)B * m * 8));
    CK(hipMalloc(&dW[v], B * 8));
    CK(hipMalloc(&dC[v], B * 8));
    CK(hipMalloc(&info[v], B * 4));
  }
  CK(hipMemcpy(dM, M.data(), M.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dr1, r1.data(), r1.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dr2, r2.data(), r2.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dmu, mu.data(), B * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dlast, last.data(), B * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[2] = {"block", "wave"};
  for (int v = 0; v < 2; ++v) {
    for (int mode = 0; mode < 2; ++mode) {
      float best = 1e30f;
      for (int rep = 0; rep < 7; ++rep) {
        CK(hipEventRecord(e0));
        if (v == 0) {
          const size_t lds = sizeof(double) * (size_t)kkt_launch_lds_doubles(nw, m, mode);
          hipLaunchKernelGGL(kkt_kernel_for(nw, m), dim3((unsigned)B), dim3(KKT_THREADS), lds, 0, mode, (int64_t)B, nw,
                             m, dM, dA, dr1, dr2, dmu, dlast, nullptr, dw[v], dy[v], dW[v], dC[v], info[v], dws);
        } else {
          const size_t lds = sizeof(double) * (size_t)kktw_lds_doubles(nw, m);
          hipLaunchKernelGGL(kkt_wave_kernel_for(nw, m, 1 << 30), dim3((unsigned)B), dim3(64), lds, 0, mode, (int64_t)B, dM, dA,
                             dr1, dr2, dmu, dlast, nullptr, dw[v], dy[v], dW[v], dC[v], info[v], dws);
        }
        CK(hipGetLastError());
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
      }
      int per_cu = 0;
      if (v == 0)
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kkt_kernel_for(nw, m)),
                                                        KKT_THREADS, sizeof(double) * kkt_launch_lds_doubles(nw, m, mode)));
      else
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kkt_wave_kernel_for(nw, m, 1 << 30)),
                                                        64, sizeof(double) * kktw_lds_doubles(nw, m)));
      std::printf("%-5s mode %d: %.3f ms for %d systems (nw %d, m %d), %d workgroups/CU\n", names[v], mode, best, B, nw,
                  m, per_cu);
    }
    // leave the mode-0 result (mode 1 re-solved with the same rhs: must equal it up to refinement)
    if (v == 0) {
      const size_t lds = sizeof(double) * (size_t)kkt_launch_lds_doubles(nw, m, 0);
      hipLaunchKernelGGL(kkt_kernel_for(nw, m), dim3((unsigned)B), dim3(KKT_THREADS), lds, 0, 0, (int64_t)B, nw, m, dM,
                         dA, dr1, dr2, dmu, dlast, nullptr, dw[v], dy[v], dW[v], dC[v], info[v], dws);
    } else {
      const size_t lds = sizeof(double) * (size_t)kktw_lds_doubles(nw, m);
      hipLaunchKernelGGL(kkt_wave_kernel_for(nw, m, 1 << 30), dim3((unsigned)B), dim3(64), lds, 0, 0, (int64_t)B, dM, dA, dr1,
                         dr2, dmu, dlast, nullptr, dw[v], dy[v], dW[v], dC[v], info[v], dws);
    }
    CK(hipDeviceSynchronize());
  }
  // compare: KKT residuals of both, the difference, delta_w / delta_c agreement
  std::vector<double> hw[2], hy[2], hW[2], hC[2];
  std::vector<int32_t> hi[2];
  for (int v = 0; v < 2; ++v) {
    hw[v].resize((size_t)B * nw);
    hy[v].resize((size_t)B * m);
    hW[v].resize(B);
    hC[v].resize(B);
    hi[v].resize(B);
    CK(hipMemcpy(hw[v].data(), dw[v], hw[v].size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hy[v].data(), dy[v], hy[v].size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hW[v].data(), dW[v], B * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hC[v].data(), dC[v], B * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hi[v].data(), info[v], B * 4, hipMemcpyDeviceToHost));
  }
  double res[2] = {0, 0}, dmax = 0.0;
  int dW_diff = 0, dC_diff = 0, info_diff = 0;
  for (int b = 0; b < B; ++b) {
    for (int v = 0; v < 2; ++v) {
      const double* Mb = &M[(size_t)b * nw * nw];
      const double* Ab = &A[(size_t)b * m * nw];
      const double* x = &hw[v][(size_t)b * nw];
      const double* y = &hy[v][(size_t)b * m];
      double rn = 0.0, qn = 0.0;
      for (int i = 0; i < nw; ++i) {
        double s = (hW[v][b]) * x[i];
        for (int k = 0; k < nw; ++k) s += Mb[i * nw + k] * x[k];
        for (int k = 0; k < m; ++k) s += Ab[k * nw + i] * y[k];
        rn = std::max(rn, std::fabs(s - r1[(size_t)b * nw + i]));
        qn = std::max(qn, std::fabs(r1[(size_t)b * nw + i]));
      }
      for (int k = 0; k < m; ++k) {
        double s = 0.0;
        for (int i = 0; i < nw; ++i) s += Ab[k * nw + i] * x[i];
        rn = std::max(rn, std::fabs(s - r2[(size_t)b * m + k]));
      }
      res[v] = std::max(res[v], rn / std::max(qn, 1.0));
    }
    if (hW[0][b] != hW[1][b]) ++dW_diff;
    if (hC[0][b] != hC[1][b]) ++dC_diff;
    if (hi[0][b] != hi[1][b]) ++info_diff;
    if (hW[0][b] == hW[1][b]) {
      double xn = 0.0, dn = 0.0;
      for (int i = 0; i < nw; ++i) {
        xn = std::max(xn, std::fabs(hw[0][(size_t)b * nw + i]));
        dn = std::max(dn, std::fabs(hw[0][(size_t)b * nw + i] - hw[1][(size_t)b * nw + i]));
      }
      dmax = std::max(dmax, dn / std::max(xn, 1e-300));
    }
  }
  std::printf("max relative KKT residual: block %.3e, wave %.3e (with each kernel's delta_w on M)\n", res[0], res[1]);
  std::printf("max relative |dw_block - dw_wave| (same delta_w): %.3e\n", dmax);
  std::printf("instances with different delta_w: %d, delta_c: %d, info: %d (of %d)\n", dW_diff, dC_diff, info_diff, B);
  return 0;
}
