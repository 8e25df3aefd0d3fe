// cpl/BatchBroker.hpp — the batched TNLP broker (SURVEY.md §8(b) caller 2, §8(f) rank 1).
//
// Many concurrent solver instances of one problem template (IPOPT instances, or a built-in
// driver's iterates) each deposit their x in a pinned host slot; Evaluate() moves the whole batch
// to HBM in one copy, runs ONE fused cpl_eval_batch launch for all of them and brings the
// requested outputs back in one copy, after which each instance reads its own g / jac / f / grad
// slot.  This replaces the reference's one-callback-per-instance IpoptAdapter traffic
// (src/CentroidalPlanner.cpp:29 -> IFOPT IpoptAdapter::eval_* [IFOPT-ext]) with one launch per
// solver iteration across the batch.  Device-resident callers skip the host slots entirely and
// use cpl_eval_batch on their own device arrays.
#pragma once

#include <cstdint>

#include "cpl/CplProblem.hpp"

namespace cpl {
namespace solver {

class BatchBroker {
 public:
  enum Output : unsigned { G = 1u, JAC = 2u, F = 4u, GRAD = 8u };

  BatchBroker(CplProblem::Ptr problem, int64_t capacity, int device = -1);
  ~BatchBroker();
  BatchBroker(const BatchBroker&) = delete;
  BatchBroker& operator=(const BatchBroker&) = delete;

  int64_t capacity() const { return _cap; }
  const CplProblem& problem() const { return *_problem; }

  // host (pinned) slots, instance i in [0, capacity)
  double* x(int64_t i) { return _hx + i * _n; }
  double& mass(int64_t i) { return _hmass[i]; }  // per-instance robot mass (default: the problem's)
  uint8_t& env_tag(int64_t i) { return _htag[i]; }  // mixed environment only
  const double* g(int64_t i) const { return _hg + i * _m; }
  const double* jac(int64_t i) const { return _hjac + i * _nnz; }
  double f(int64_t i) const { return _hf[i]; }
  const double* grad(int64_t i) const { return _hgrad + i * _n; }

  // evaluates instances [0, count): one H2D copy, one launch, one D2H copy per requested output
  void Evaluate(int64_t count, unsigned outputs = G | JAC | F | GRAD);
  // [max violation, sum of squared violations] of the last evaluated g over [0, count)
  void ResidualNorms(int64_t count, double out[2]);

  int64_t launches() const { return _launches; }

 private:
  CplProblem::Ptr _problem;
  int64_t _cap;
  int32_t _n, _m, _nnz;
  void* _stream = nullptr;
  double *_hx = nullptr, *_hmass = nullptr, *_hg = nullptr, *_hjac = nullptr, *_hf = nullptr, *_hgrad = nullptr;
  uint8_t* _htag = nullptr;
  double *_dx = nullptr, *_dmass = nullptr, *_dg = nullptr, *_djac = nullptr, *_df = nullptr, *_dgrad = nullptr,
         *_dnorm = nullptr;
  uint8_t* _dtag = nullptr;
  int64_t _launches = 0;
};

}  // namespace solver
}  // namespace cpl
