// cpl_check.hip — host-buffer evaluation (cpl_eval_batch_host) and the batched first-order
// derivative checker (cpl_derivative_test).
//
// The derivative checker restates IPOPT's "derivative_test = first-order" (TNLPAdapter::
// CheckDerivatives, IPOPT 3.x; IPOPT is an un-vendored dependency of the reference, enabled for
// every solve by src/CentroidalPlanner.cpp:26): forward differences of g and f along each variable,
// perturbation h_j = derivative_test_perturbation * max(1, |x_j|), compared entry by entry with the
// Jacobian / objective gradient the callbacks return, flagged above derivative_test_tol.  On the GPU
// the batch * n perturbed points are ONE more batch for the eval kernel: the checker costs one
// launch over n times the instances, plus two small kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <mutex>
#include <vector>

#include "cpl_layout.hpp"
#include "cpl_status.hpp"

namespace cpl {

static int32_t hfail(hipError_t e, const char* what) {
  return fail(CPL_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// ------------------------------------------------------------------------------------------
// host-buffer staging
// ------------------------------------------------------------------------------------------
struct HostIo {
  std::mutex mu;
  hipStream_t stream = nullptr;
  void* buf = nullptr;  // device workspace (batches past the zero-copy limit)
  size_t bytes = 0;
  void* pin = nullptr;  // pinned, device-mapped host staging (small batches: the kernel reads and writes it)
  size_t pin_bytes = 0;
};
// Small batches (the single-instance TNLP callback path) skip the DMA copies: the host arrays are
// memcpy'd into library-owned coherent pinned memory, the eval kernel reads x and writes g / jac there
// directly over the host link, and the outputs are memcpy'd back after the stream drains — one launch
// and one wait instead of 2 + #outputs DMA transfers (each a pageable-memory staging round trip):
// 22.5 us per single-instance eval_g + eval_jac_g (Ground N = 4) against 31 us for the DMA-staged
// path.  (Polling hipStreamQuery instead of hipStreamSynchronize measured 4 us slower.)
constexpr size_t ZERO_COPY_MAX = (size_t)1 << 20;
static std::mutex g_hostio_mutex;
static HostIo* g_hostio[64] = {nullptr};  // per device, never freed (process lifetime)

static int32_t hostio_for_device(HostIo** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hfail(e, "hipGetDevice");
  if (dev < 0 || dev >= 64) return fail(CPL_ERR_UNSUPPORTED, "device index out of range");
  std::lock_guard<std::mutex> lk(g_hostio_mutex);
  if (!g_hostio[dev]) {
    HostIo* h = new HostIo();
    e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      delete h;
      return hfail(e, "hipStreamCreate");
    }
    g_hostio[dev] = h;
  }
  *out = g_hostio[dev];
  return CPL_OK;
}

static size_t up256(size_t b) { return (b + 255) & ~(size_t)255; }

// ------------------------------------------------------------------------------------------
// derivative checker kernels
// ------------------------------------------------------------------------------------------

// Xp[(b*n + j)*n + k] = x[b,k] (+ h_bj at k == j); mass / tag repeated n times.
__global__ __launch_bounds__(256) void k_dt_perturb(int64_t C, int n, const double* __restrict__ x,
                                                     const double* __restrict__ mass,
                                                     const uint8_t* __restrict__ tag, double pert,
                                                     double* __restrict__ xp, double* __restrict__ h,
                                                     double* __restrict__ massp, uint8_t* __restrict__ tagp) {
  const int64_t total = C * n * n;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t bj = e / n;
    const int k = (int)(e - bj * n);
    const int64_t b = bj / n;
    const int j = (int)(bj - b * n);
    const double xv = x[b * n + k];
    if (k == j) {
      const double hv = pert * fmax(1.0, fabs(xv));
      xp[e] = xv + hv;
      h[bj] = hv;
      if (mass) massp[bj] = mass[b];
      if (tag) tagp[bj] = tag[b];
    } else {
      xp[e] = xv;
    }
  }
}

// One thread per (instance, variable): walk the m constraint rows and the objective.
// amap[i*n + j] = CSR position of (i, j), -1 outside the structure.
__global__ __launch_bounds__(256) void k_dt_compare(int64_t C, int n, int m, int nnz, const int32_t* __restrict__ amap,
                                                     const double* __restrict__ g0, const double* __restrict__ jac,
                                                     const double* __restrict__ f0, const double* __restrict__ grad,
                                                     const double* __restrict__ gp, const double* __restrict__ fp,
                                                     const double* __restrict__ h, double tol,
                                                     int32_t* __restrict__ cnt, double* __restrict__ worst,
                                                     int32_t* __restrict__ worst_row, double* __restrict__ wex,
                                                     double* __restrict__ wap) {
  const int64_t bj = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (bj >= C * n) return;
  const int64_t b = bj / n;
  const int j = (int)(bj - b * n);
  const double hv = h[bj];
  int c = 0;
  double wr = -1.0, we = 0.0, wa = 0.0;
  int wrow = -2;
  auto check = [&](double approx, double exact, int row) {
    const double rel = fabs(approx - exact) / fmax(fabs(approx), tol);
    if (!(rel <= tol)) ++c;  // NaN counts as flagged
    if (rel > wr || (rel != rel && wr == wr)) {
      wr = rel;
      wrow = row;
      we = exact;
      wa = approx;
    }
  };
  // objective gradient first (IPOPT checks grad_f before jac_g)
  check((fp[bj] - f0[b]) / hv, grad[b * n + j], -1);
  for (int i = 0; i < m; ++i) {
    const int q = amap[i * n + j];
    const double exact = q >= 0 ? jac[b * nnz + q] : 0.0;
    check((gp[bj * m + i] - g0[b * m + i]) / hv, exact, i);
  }
  cnt[bj] = c;
  worst[bj] = wr;
  worst_row[bj] = wrow;
  wex[bj] = we;
  wap[bj] = wa;
}

// per instance: sum the n counts, pick the worst variable (first on ties)
__global__ __launch_bounds__(64) void k_dt_instance(int64_t C, int n, const int32_t* __restrict__ cnt,
                                                     const double* __restrict__ worst, int32_t* __restrict__ icnt,
                                                     int32_t* __restrict__ iworst_j, double* __restrict__ iworst) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= C) return;
  int s = 0, wj = 0;
  double w = -1.0;
  for (int j = 0; j < n; ++j) {
    s += cnt[b * n + j];
    const double v = worst[b * n + j];
    if (v > w || (v != v && w == w)) {
      w = v;
      wj = j;
    }
  }
  icnt[b] = s;
  iworst_j[b] = wj;
  iworst[b] = w;
}

}  // namespace cpl

using namespace cpl;

extern "C" {

int32_t cpl_eval_batch_host(const cpl_problem_desc* d, int64_t batch, const double* h_x, const double* h_mass,
                            const uint8_t* h_env_tag, double* h_g, double* h_jac, double* h_f, double* h_grad,
                            double* h_norms, int32_t flags) {
  int32_t st = validate_desc(d);
  if (st) return st;
  if (batch < 0) return fail(CPL_ERR_INVALID_ARGUMENT, "negative batch");
  if (batch > 0 && !h_x) return fail(CPL_ERR_INVALID_ARGUMENT, "x is required");
  if (h_norms && !h_g) return fail(CPL_ERR_INVALID_ARGUMENT, "residual norms need the g output");
  int32_t n, m, nnz;
  if ((st = cpl_dims(d, &n, &m, &nnz))) return st;
  if (flags & CPL_EVAL_JAC_FOLDED) {
    if ((st = cpl_jac_fold_info(d, &nnz, nullptr, nullptr, nullptr, nullptr))) return st;
  }
  const bool mixed = d->env_kind == CPL_ENV_MIXED;
  if (mixed && batch > 0 && !h_env_tag)
    return fail(CPL_ERR_INVALID_ARGUMENT, "mixed environment batch needs a per-instance env tag array");
  HostIo* io = nullptr;
  if ((st = hostio_for_device(&io))) return st;
  std::lock_guard<std::mutex> lk(io->mu);
  const size_t B = (size_t)batch;
  const size_t sx = up256(8 * B * n), sm = h_mass ? up256(8 * B) : 0, st8 = mixed ? up256(B) : 0;
  const size_t sg = h_g ? up256(8 * B * m) : 0, sj = h_jac ? up256(8 * B * nnz) : 0;
  const size_t sf = h_f ? up256(8 * B) : 0, sd = h_grad ? up256(8 * B * n) : 0, sn = h_norms ? 256 : 0;
  const size_t need = sx + sm + st8 + sg + sj + sf + sd + sn;
  hipError_t e;
  if (need <= ZERO_COPY_MAX) {
    if (need > io->pin_bytes) {
      if (io->pin) {
        if ((e = hipStreamSynchronize(io->stream)) != hipSuccess) return hfail(e, "hipStreamSynchronize");
        (void)hipHostFree(io->pin);
        io->pin = nullptr;
        io->pin_bytes = 0;
      }
      const size_t cap = std::max(need, (size_t)64 << 10);
      if ((e = hipHostMalloc(&io->pin, cap, hipHostMallocCoherent | hipHostMallocMapped)) != hipSuccess)
        return hfail(e, "hipHostMalloc host-io staging");
      io->pin_bytes = cap;
    }
    void* dpin = nullptr;  // the device's address of the staging (the same address on this platform)
    if ((e = hipHostGetDevicePointer(&dpin, io->pin, 0)) != hipSuccess) return hfail(e, "hipHostGetDevicePointer");
    char* hp = static_cast<char*>(io->pin);
    char* dp = static_cast<char*>(dpin);
    size_t off = 0;
    auto carve = [&](size_t sz, const void* src, size_t copy) {
      if (!sz) return (void*)nullptr;
      if (src && copy) memcpy(hp + off, src, copy);
      void* r = dp + off;
      off += sz;
      return r;
    };
    const double* px = static_cast<const double*>(carve(sx, h_x, 8 * B * n));
    const double* pm = static_cast<const double*>(carve(sm, h_mass, 8 * B));
    const uint8_t* pt = static_cast<const uint8_t*>(carve(st8, h_env_tag, B));
    const size_t og = off;
    double* pg = static_cast<double*>(carve(sg, nullptr, 0));
    const size_t oj = off;
    double* pj = static_cast<double*>(carve(sj, nullptr, 0));
    const size_t of = off;
    double* pf = static_cast<double*>(carve(sf, nullptr, 0));
    const size_t od = off;
    double* pd = static_cast<double*>(carve(sd, nullptr, 0));
    const size_t on = off;
    double* pn = static_cast<double*>(carve(sn, nullptr, 0));
    if ((st = cpl_eval_batch_ex(d, batch, px, pm, pt, pg, pj, pf, pd, pn, flags, io->stream))) return st;
    if ((e = hipStreamSynchronize(io->stream)) != hipSuccess) return hfail(e, "hipStreamSynchronize");
    if (pg) memcpy(h_g, hp + og, 8 * B * m);
    if (pj) memcpy(h_jac, hp + oj, 8 * B * nnz);
    if (pf) memcpy(h_f, hp + of, 8 * B);
    if (pd) memcpy(h_grad, hp + od, 8 * B * n);
    if (pn) memcpy(h_norms, hp + on, 16);
    return CPL_OK;
  }
  if (need > io->bytes) {
    if (io->buf) {
      e = hipStreamSynchronize(io->stream);
      if (e != hipSuccess) return hfail(e, "hipStreamSynchronize");
      (void)hipFree(io->buf);
      io->buf = nullptr;
      io->bytes = 0;
    }
    e = hipMalloc(&io->buf, need);
    if (e != hipSuccess) return hfail(e, "hipMalloc host-io workspace");
    io->bytes = need;
  }
  char* p = static_cast<char*>(io->buf);
  double* dx = reinterpret_cast<double*>(p); p += sx;
  double* dm = h_mass ? reinterpret_cast<double*>(p) : nullptr; p += sm;
  uint8_t* dt = mixed ? reinterpret_cast<uint8_t*>(p) : nullptr; p += st8;
  double* dg = h_g ? reinterpret_cast<double*>(p) : nullptr; p += sg;
  double* dj = h_jac ? reinterpret_cast<double*>(p) : nullptr; p += sj;
  double* df = h_f ? reinterpret_cast<double*>(p) : nullptr; p += sf;
  double* dd = h_grad ? reinterpret_cast<double*>(p) : nullptr; p += sd;
  double* dn = h_norms ? reinterpret_cast<double*>(p) : nullptr;
  hipStream_t s = io->stream;
  if (B) {
    if ((e = hipMemcpyAsync(dx, h_x, 8 * B * n, hipMemcpyHostToDevice, s)) != hipSuccess) return hfail(e, "H2D x");
    if (dm && (e = hipMemcpyAsync(dm, h_mass, 8 * B, hipMemcpyHostToDevice, s)) != hipSuccess) return hfail(e, "H2D mass");
    if (dt && (e = hipMemcpyAsync(dt, h_env_tag, B, hipMemcpyHostToDevice, s)) != hipSuccess) return hfail(e, "H2D tag");
  }
  if ((st = cpl_eval_batch_ex(d, batch, dx, dm, dt, dg, dj, df, dd, dn, flags, s))) return st;
  if (B) {
    if (dg && (e = hipMemcpyAsync(h_g, dg, 8 * B * m, hipMemcpyDeviceToHost, s)) != hipSuccess) return hfail(e, "D2H g");
    if (dj && (e = hipMemcpyAsync(h_jac, dj, 8 * B * nnz, hipMemcpyDeviceToHost, s)) != hipSuccess) return hfail(e, "D2H jac");
    if (df && (e = hipMemcpyAsync(h_f, df, 8 * B, hipMemcpyDeviceToHost, s)) != hipSuccess) return hfail(e, "D2H f");
    if (dd && (e = hipMemcpyAsync(h_grad, dd, 8 * B * n, hipMemcpyDeviceToHost, s)) != hipSuccess) return hfail(e, "D2H grad");
  }
  if (dn && (e = hipMemcpyAsync(h_norms, dn, 16, hipMemcpyDeviceToHost, s)) != hipSuccess) return hfail(e, "D2H norms");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hfail(e, "hipStreamSynchronize");
  return CPL_OK;
}

int32_t cpl_derivative_test(const cpl_problem_desc* d, int64_t batch, const double* d_x, const double* d_mass,
                            const uint8_t* d_env_tag, double perturbation, double tol, int32_t* d_inst_flagged,
                            cpl_derivative_report* report, void* stream) {
  int32_t st = validate_desc(d);
  if (st) return st;
  if (!report) return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_derivative_test: report is required");
  if (batch < 0) return fail(CPL_ERR_INVALID_ARGUMENT, "negative batch");
  if (!(perturbation > 0.0) || !(tol > 0.0))
    return fail(CPL_ERR_INVALID_ARGUMENT, "cpl_derivative_test: perturbation and tol must be > 0");
  if (batch > 0 && !d_x) return fail(CPL_ERR_INVALID_ARGUMENT, "x is required");
  const bool mixed = d->env_kind == CPL_ENV_MIXED;
  if (mixed && batch > 0 && !d_env_tag)
    return fail(CPL_ERR_INVALID_ARGUMENT, "mixed environment batch needs a per-instance env tag array");
  int32_t n, m, nnz;
  if ((st = cpl_dims(d, &n, &m, &nnz))) return st;
  *report = cpl_derivative_report{0, 0, 0.0, -1, -2, -1, 0.0, 0.0};
  report->n_checked = batch * (int64_t)n * (m + 1);
  if (batch == 0) return CPL_OK;

  // dense (row, col) -> CSR position map of the structure
  std::vector<int32_t> iRow(nnz), jCol(nnz), amap((size_t)m * n, -1);
  if ((st = cpl_structure(d, iRow.data(), jCol.data(), nullptr))) return st;
  for (int32_t k = 0; k < nnz; ++k) amap[(size_t)iRow[k] * n + jCol[k]] = k;

  // chunk so that the perturbed batch's x and g stay within ~512 MiB
  const int64_t per_inst = (int64_t)n * (n + m + 8) + m + nnz + n + 4;
  int64_t C = std::max<int64_t>(1, ((int64_t)64 << 20) / per_inst);
  C = std::min<int64_t>(C, batch);
  const size_t Cn = (size_t)C * n;
  const size_t bytes = up256(4 * (size_t)m * n) + up256(8 * Cn * n) + 3 * up256(8 * Cn) + up256(Cn) +
                       up256(8 * Cn * m) + up256(8 * (size_t)C * m) + up256(8 * (size_t)C * nnz) +
                       up256(8 * (size_t)C) + up256(8 * Cn) + up256(4 * Cn) * 2 + up256(8 * Cn) * 3 +
                       up256(4 * (size_t)C) * 2 + up256(8 * (size_t)C);
  hipStream_t s = (hipStream_t)stream;
  void* ws = nullptr;
  hipError_t e = hipMalloc(&ws, bytes);
  if (e != hipSuccess) return hfail(e, "hipMalloc derivative-test workspace");
  char* p = static_cast<char*>(ws);
  auto take = [&](size_t b) { char* r = p; p += up256(b); return r; };
  int32_t* damap = reinterpret_cast<int32_t*>(take(4 * (size_t)m * n));
  double* xp = reinterpret_cast<double*>(take(8 * Cn * n));
  double* h = reinterpret_cast<double*>(take(8 * Cn));
  double* massp = reinterpret_cast<double*>(take(8 * Cn));
  double* fp = reinterpret_cast<double*>(take(8 * Cn));
  uint8_t* tagp = reinterpret_cast<uint8_t*>(take(Cn));
  double* gp = reinterpret_cast<double*>(take(8 * Cn * m));
  double* g0 = reinterpret_cast<double*>(take(8 * (size_t)C * m));
  double* jac = reinterpret_cast<double*>(take(8 * (size_t)C * nnz));
  double* f0 = reinterpret_cast<double*>(take(8 * (size_t)C));
  double* grad = reinterpret_cast<double*>(take(8 * Cn));
  int32_t* cnt = reinterpret_cast<int32_t*>(take(4 * Cn));
  int32_t* wrow = reinterpret_cast<int32_t*>(take(4 * Cn));
  double* worst = reinterpret_cast<double*>(take(8 * Cn));
  double* wex = reinterpret_cast<double*>(take(8 * Cn));
  double* wap = reinterpret_cast<double*>(take(8 * Cn));
  int32_t* icnt = reinterpret_cast<int32_t*>(take(4 * (size_t)C));
  int32_t* iwj = reinterpret_cast<int32_t*>(take(4 * (size_t)C));
  double* iwv = reinterpret_cast<double*>(take(8 * (size_t)C));

  std::vector<int32_t> h_icnt(C), h_iwj(C);
  std::vector<double> h_iwv(C);
  int32_t rc = CPL_OK;
  e = hipMemcpyAsync(damap, amap.data(), 4 * (size_t)m * n, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) rc = hfail(e, "H2D structure map");
  for (int64_t b0 = 0; rc == CPL_OK && b0 < batch; b0 += C) {
    const int64_t c = std::min<int64_t>(C, batch - b0);
    const double* xb = d_x + b0 * n;
    const double* mb = d_mass ? d_mass + b0 : nullptr;
    const uint8_t* tb = mixed ? d_env_tag + b0 : nullptr;
    if ((rc = cpl_eval_batch(d, c, xb, mb, tb, g0, jac, f0, grad, s))) break;
    const int64_t total = c * n * n;
    const unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(k_dt_perturb, dim3(grid), dim3(256), 0, s, c, n, xb, mb, tb, perturbation, xp, h,
                       mb ? massp : nullptr, tb ? tagp : nullptr);
    if ((e = hipGetLastError()) != hipSuccess) { rc = hfail(e, "k_dt_perturb launch"); break; }
    if ((rc = cpl_eval_batch(d, c * n, xp, mb ? massp : nullptr, tb ? tagp : nullptr, gp, nullptr, fp, nullptr, s)))
      break;
    hipLaunchKernelGGL(k_dt_compare, dim3((unsigned)((c * n + 255) / 256)), dim3(256), 0, s, c, n, m, nnz, damap, g0,
                       jac, f0, grad, gp, fp, h, tol, cnt, worst, wrow, wex, wap);
    if ((e = hipGetLastError()) != hipSuccess) { rc = hfail(e, "k_dt_compare launch"); break; }
    hipLaunchKernelGGL(k_dt_instance, dim3((unsigned)((c + 63) / 64)), dim3(64), 0, s, c, n, cnt, worst, icnt, iwj, iwv);
    if ((e = hipGetLastError()) != hipSuccess) { rc = hfail(e, "k_dt_instance launch"); break; }
    if (d_inst_flagged &&
        (e = hipMemcpyAsync(d_inst_flagged + b0, icnt, 4 * (size_t)c, hipMemcpyDeviceToDevice, s)) != hipSuccess) {
      rc = hfail(e, "copy per-instance counts");
      break;
    }
    if ((e = hipMemcpyAsync(h_icnt.data(), icnt, 4 * (size_t)c, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipMemcpyAsync(h_iwj.data(), iwj, 4 * (size_t)c, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipMemcpyAsync(h_iwv.data(), iwv, 8 * (size_t)c, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess) {
      rc = hfail(e, "D2H derivative-test counts");
      break;
    }
    // the chunk's worst instance (first on ties; a NaN deviation wins and stays)
    int64_t wb = -1;
    double wv = report->max_rel_error;
    for (int64_t b = 0; b < c; ++b) report->n_flagged += h_icnt[b];
    if (report->worst_instance < 0 || wv == wv) {
      for (int64_t b = 0; b < c; ++b) {
        const double v = h_iwv[b];
        if (v > wv || (v != v && wv == wv) || (report->worst_instance < 0 && wb < 0)) {
          wv = v;
          wb = b;
        }
      }
    }
    if (wb >= 0) {
      const size_t at = (size_t)wb * n + h_iwj[wb];
      int32_t r = -2;
      double ex = 0.0, ap = 0.0;
      if ((e = hipMemcpy(&r, wrow + at, 4, hipMemcpyDeviceToHost)) != hipSuccess ||
          (e = hipMemcpy(&ex, wex + at, 8, hipMemcpyDeviceToHost)) != hipSuccess ||
          (e = hipMemcpy(&ap, wap + at, 8, hipMemcpyDeviceToHost)) != hipSuccess) {
        rc = hfail(e, "D2H worst entry");
        break;
      }
      report->max_rel_error = wv;
      report->worst_instance = b0 + wb;
      report->worst_row = r;
      report->worst_col = h_iwj[wb];
      report->worst_exact = ex;
      report->worst_approx = ap;
    }
  }
  (void)hipStreamSynchronize(s);
  (void)hipFree(ws);
  return rc;
}

}  // extern "C"
