// Host side of the native solve engine: solver::BatchSolver (many instances, host arrays) and
// solver::NativeSolver (CentroidalPlanner's default NlpSolver: a batch of one) over the C-ABI
// cpl_solver_* (csrc/cpl_solver.hip).  Reference: the IPOPT solve behind
// src/CentroidalPlanner.cpp:22-34 (ifopt::IpoptSolver::Solve), with IFOPT's defaults.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>

#include "cpl/CentroidalPlanner.hpp"

namespace cpl {
namespace solver {

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

static void engine_check(int32_t st) {
  if (st != CPL_OK) throw std::runtime_error(std::string("cpl_solver: ") + cpl_last_error());
}

BatchSolver::BatchSolver(CplProblem::Ptr problem, int64_t batch, const SolveOptions& opt)
    : _problem(std::move(problem)), _batch(batch) {
  const size_t B = (size_t)batch, n = (size_t)_problem->n(), m = (size_t)_problem->m();
  engine_check(cpl_solver_create(&_problem->Desc(), batch, &opt, &_solver));
  try {
    hipStream_t s = nullptr;
    hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    _stream = s;
    hip_check(hipMalloc(&_dx0, 8 * B * n), "hipMalloc");
    hip_check(hipMalloc(&_dmass, 8 * B), "hipMalloc");
    hip_check(hipMalloc(&_dx, 8 * B * n), "hipMalloc");
    hip_check(hipMalloc(&_dy, 8 * B * m), "hipMalloc");
    hip_check(hipMalloc(&_dobj, 8 * B), "hipMalloc");
    hip_check(hipMalloc(&_dpinf, 8 * B), "hipMalloc");
    hip_check(hipMalloc(&_dstatus, 4 * B), "hipMalloc");
    hip_check(hipMalloc(&_diters, 4 * B), "hipMalloc");
    hip_check(hipMalloc(&_dnan, 4 * B), "hipMalloc");
  } catch (...) {
    release();  // (the destructor does not run for a constructor that throws)
    throw;
  }
}

BatchSolver::~BatchSolver() { release(); }

void BatchSolver::release() {
  for (void* p : {(void*)_dx0, (void*)_dmass, (void*)_dx, (void*)_dy, (void*)_dobj, (void*)_dpinf, (void*)_dstatus,
                  (void*)_diters, (void*)_dnan})
    if (p) (void)hipFree(p);
  _dx0 = _dmass = _dx = _dy = _dobj = _dpinf = nullptr;
  _dstatus = _diters = _dnan = nullptr;
  if (_stream) (void)hipStreamDestroy((hipStream_t)_stream);
  _stream = nullptr;
  if (_solver) cpl_solver_destroy(_solver);
  _solver = nullptr;
}

bool BatchSolver::graph_captured() const {
  int32_t g = 0;
  return _solver && cpl_solver_dims(_solver, nullptr, nullptr, &g) == CPL_OK && g;
}

void BatchSolver::Solve(const double* x0, const double* mass, double* x, double* y, int32_t* status,
                        int32_t* iterations, double* objective, double* primal_inf) {
  const size_t B = (size_t)_batch, n = (size_t)_problem->n(), m = (size_t)_problem->m();
  hipStream_t s = (hipStream_t)_stream;
  hip_check(hipMemcpyAsync(_dx0, x0, 8 * B * n, hipMemcpyHostToDevice, s), "hipMemcpyAsync x0");
  if (mass) hip_check(hipMemcpyAsync(_dmass, mass, 8 * B, hipMemcpyHostToDevice, s), "hipMemcpyAsync mass");
  engine_check(cpl_solver_solve(_solver, _dx0, mass ? _dmass : nullptr, nullptr, _dx, _dy, _dstatus, _diters, _dobj,
                                _dpinf, nullptr, &_iterations_run, nullptr, s));
  if (x) hip_check(hipMemcpyAsync(x, _dx, 8 * B * n, hipMemcpyDeviceToHost, s), "hipMemcpyAsync x");
  if (y) hip_check(hipMemcpyAsync(y, _dy, 8 * B * m, hipMemcpyDeviceToHost, s), "hipMemcpyAsync y");
  if (status) hip_check(hipMemcpyAsync(status, _dstatus, 4 * B, hipMemcpyDeviceToHost, s), "hipMemcpyAsync status");
  if (iterations) hip_check(hipMemcpyAsync(iterations, _diters, 4 * B, hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
  if (objective) hip_check(hipMemcpyAsync(objective, _dobj, 8 * B, hipMemcpyDeviceToHost, s), "hipMemcpyAsync obj");
  if (primal_inf) hip_check(hipMemcpyAsync(primal_inf, _dpinf, 8 * B, hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
}

void BatchSolver::NanJacobian(int32_t* counts) const {
  // (into the buffer allocated with the solver's others: a hipMalloc / hipFree per Solve() sat on the
  // single-instance latency path, and hipFree can synchronise the device)
  const size_t B = (size_t)_batch;
  const hipStream_t s = (hipStream_t)_stream;
  const int32_t st = cpl_solver_nan_jacobian(_solver, _dnan, s);
  hipError_t e = st == CPL_OK ? hipMemcpyAsync(counts, _dnan, 4 * B, hipMemcpyDeviceToHost, s) : hipSuccess;
  if (e == hipSuccess && st == CPL_OK) e = hipStreamSynchronize(s);
  engine_check(st);
  hip_check(e, "hipMemcpyAsync nan_jacobian");
}

bool NativeSolver::Solve(CplTNLP& nlp) {
  const CplProblem::Ptr& prob = nlp.problem();
  const int32_t n = prob->n(), m = prob->m();
  std::vector<double> x0(n), x(n);
  nlp.get_starting_point(n, true, x0.data());
  {  // the derivative test runs where the solve starts: x0 inside the variable bounds
    std::vector<double> xl(n), xu(n), gl(m), gu(m);
    nlp.get_bounds_info(n, xl.data(), xu.data(), m, gl.data(), gu.data());
    for (int32_t j = 0; j < n; ++j) x0[j] = std::fmin(std::fmax(x0[j], xl[j]), xu[j]);
  }
  _dreport = cpl_derivative_report{};
  if (_opt.derivative_test) {  // IPOPT checks the first derivatives before it iterates
    double* dx = nullptr;
    hip_check(hipMalloc(&dx, 8 * (size_t)n), "hipMalloc");
    hipError_t e = hipMemcpy(dx, x0.data(), 8 * (size_t)n, hipMemcpyHostToDevice);
    const int32_t st = e == hipSuccess ? cpl_derivative_test(&prob->Desc(), 1, dx, nullptr, nullptr,
                                                             _opt.derivative_test_perturbation,
                                                             _opt.derivative_test_tol, nullptr, &_dreport, nullptr)
                                       : CPL_OK;
    (void)hipFree(dx);
    hip_check(e, "hipMemcpy x0");
    engine_check(st);
  }
  // the engine handle (device buffers, captured iteration graphs) is kept between solves of the same
  // problem template; a changed template (any setter since the last solve) gets a new one
  if (!_bs || _bs_problem != prob.get() || std::memcmp(&_bs_desc, &prob->Desc(), sizeof(_bs_desc)) != 0) {
    _bs.reset();
    _bs.reset(new BatchSolver(prob, 1, _opt));
    _bs_problem = prob.get();
    _bs_desc = prob->Desc();
  }
  _bs->Solve(x0.data(), nullptr, x.data(), nullptr, &_status, &_iterations, nullptr, &_primal_inf);
  // NaN Jacobian entries at the start point (the 0/0 of a cone at F_t = 0), counted by the engine's
  // own start-point evaluation
  _bs->NanJacobian(&_nan_jac_start);
  nlp.finalize_solution(n, x.data());
  return _status == CPL_SOLVE_OPTIMAL || _status == CPL_SOLVE_ACCEPTABLE;
}

}  // namespace solver
}  // namespace cpl
