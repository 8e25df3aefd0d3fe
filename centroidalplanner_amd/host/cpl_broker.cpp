// Batched TNLP broker: pinned host slots <-> one fused launch per batch (include/cpl/BatchBroker.hpp).
#include <hip/hip_runtime_api.h>

#include <stdexcept>
#include <string>

#include "cpl/BatchBroker.hpp"

namespace cpl {
namespace solver {

namespace {
void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
template <class T>
void host_alloc(T** p, size_t count) {
  hip_check(hipHostMalloc(reinterpret_cast<void**>(p), sizeof(T) * (count ? count : 1), hipHostMallocDefault),
            "hipHostMalloc");
}
template <class T>
void dev_alloc(T** p, size_t count) {
  hip_check(hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * (count ? count : 1)), "hipMalloc");
}
}  // namespace

BatchBroker::BatchBroker(CplProblem::Ptr problem, int64_t capacity, int device)
    : _problem(std::move(problem)), _cap(capacity) {
  if (!_problem) throw std::invalid_argument("BatchBroker needs a problem");
  if (capacity < 1) throw std::invalid_argument("BatchBroker capacity must be >= 1");
  if (device >= 0) hip_check(hipSetDevice(device), "hipSetDevice");
  _n = _problem->n();
  _m = _problem->m();
  _nnz = _problem->nnz();
  const size_t B = (size_t)capacity;
  hipStream_t s = nullptr;
  hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  _stream = s;
  host_alloc(&_hx, B * _n);
  host_alloc(&_hmass, B);
  host_alloc(&_htag, B);
  host_alloc(&_hg, B * _m);
  host_alloc(&_hjac, B * _nnz);
  host_alloc(&_hf, B);
  host_alloc(&_hgrad, B * _n);
  dev_alloc(&_dx, B * _n);
  dev_alloc(&_dmass, B);
  dev_alloc(&_dtag, B);
  dev_alloc(&_dg, B * _m);
  dev_alloc(&_djac, B * _nnz);
  dev_alloc(&_df, B);
  dev_alloc(&_dgrad, B * _n);
  dev_alloc(&_dnorm, 2);
  const double m0 = _problem->Desc().mass;
  for (size_t i = 0; i < B; ++i) {
    _hmass[i] = m0;
    _htag[i] = CPL_ENV_GROUND;
  }
  for (size_t i = 0; i < B * _n; ++i) _hx[i] = 0.0;
}

BatchBroker::~BatchBroker() {
  for (void* p : {(void*)_hx, (void*)_hmass, (void*)_htag, (void*)_hg, (void*)_hjac, (void*)_hf, (void*)_hgrad})
    if (p) (void)hipHostFree(p);
  for (void* p : {(void*)_dx, (void*)_dmass, (void*)_dtag, (void*)_dg, (void*)_djac, (void*)_df, (void*)_dgrad,
                  (void*)_dnorm})
    if (p) (void)hipFree(p);
  if (_stream) (void)hipStreamDestroy(static_cast<hipStream_t>(_stream));
}

void BatchBroker::Evaluate(int64_t count, unsigned outputs) {
  if (count < 0 || count > _cap) throw std::out_of_range("BatchBroker::Evaluate: count out of range");
  if (count == 0) return;
  hipStream_t s = static_cast<hipStream_t>(_stream);
  const cpl_problem_desc& d = _problem->Desc();
  const size_t B = (size_t)count;
  hip_check(hipMemcpyAsync(_dx, _hx, sizeof(double) * B * _n, hipMemcpyHostToDevice, s), "H2D x");
  hip_check(hipMemcpyAsync(_dmass, _hmass, sizeof(double) * B, hipMemcpyHostToDevice, s), "H2D mass");
  const bool mixed = d.env_kind == CPL_ENV_MIXED;
  if (mixed) hip_check(hipMemcpyAsync(_dtag, _htag, B, hipMemcpyHostToDevice, s), "H2D env tag");
  ThrowOnError(cpl_eval_batch(&d, count, _dx, _dmass, mixed ? _dtag : nullptr, (outputs & G) ? _dg : nullptr,
                              (outputs & JAC) ? _djac : nullptr, (outputs & F) ? _df : nullptr,
                              (outputs & GRAD) ? _dgrad : nullptr, s));
  if (outputs & G) hip_check(hipMemcpyAsync(_hg, _dg, sizeof(double) * B * _m, hipMemcpyDeviceToHost, s), "D2H g");
  if (outputs & JAC)
    hip_check(hipMemcpyAsync(_hjac, _djac, sizeof(double) * B * _nnz, hipMemcpyDeviceToHost, s), "D2H jac");
  if (outputs & F) hip_check(hipMemcpyAsync(_hf, _df, sizeof(double) * B, hipMemcpyDeviceToHost, s), "D2H f");
  if (outputs & GRAD)
    hip_check(hipMemcpyAsync(_hgrad, _dgrad, sizeof(double) * B * _n, hipMemcpyDeviceToHost, s), "D2H grad");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  ++_launches;
}

void BatchBroker::ResidualNorms(int64_t count, double out[2]) {
  if (count < 0 || count > _cap) throw std::out_of_range("BatchBroker::ResidualNorms: count out of range");
  hipStream_t s = static_cast<hipStream_t>(_stream);
  ThrowOnError(cpl_residual_norms(&_problem->Desc(), count, _dg, _dnorm, s));
  hip_check(hipMemcpyAsync(out, _dnorm, sizeof(double) * 2, hipMemcpyDeviceToHost, s), "D2H norms");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
}

}  // namespace solver
}  // namespace cpl
