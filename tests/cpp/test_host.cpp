// C++ host-facade tests (tests/test_host_cpp.py builds and runs this).
//
//   test_host          CPU cases: API mirror of src/CentroidalPlanner.cpp / src/CoMPlanner.cpp /
//                      src/CplProblem.cpp (validation, exception types, threshold gate, lifting
//                      contacts, map-order solution, printing) — no GPU call.
//   test_host --gpu    GPU cases: CplTNLP callbacks and the BatchBroker against the CPU oracle
//                      (oracle/_build/libcpl_oracle.so, test infrastructure) on seeded inputs.
#include <dlfcn.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "cpl/BatchBroker.hpp"
#include "cpl/CentroidalPlanner.hpp"

using namespace cpl;

static int g_fail = 0, g_pass = 0;
#define CHECK(cond)                                                           \
  do {                                                                        \
    if (!(cond)) {                                                            \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);    \
      ++g_fail;                                                               \
    } else {                                                                  \
      ++g_pass;                                                               \
    }                                                                         \
  } while (0)

template <class E>
static bool throws(const std::function<void()>& f, const char* needle = nullptr) {
  try {
    f();
  } catch (const E& e) {
    return !needle || std::string(e.what()).find(needle) != std::string::npos;
  } catch (...) {
    return false;
  }
  return false;
}

static const std::vector<std::string> NAMES = {"contact1", "contact2", "contact3", "contact4"};

// ---------------------------------------------------------------------------------------------
static void test_planner_api() {
  CHECK(throws<std::invalid_argument>([] { CentroidalPlanner(NAMES, 0.0, std::make_shared<env::Ground>()); },
                                      "Invalid robot mass"));
  auto ground = std::make_shared<env::Ground>();
  CentroidalPlanner cpl(NAMES, 80.0, ground);
  CHECK(throws<std::invalid_argument>([&] { cpl.SetForceBounds("nope", {0, 0, 0}, {1, 1, 1}); },
                                      "Invalid contact name: 'nope'"));
  CHECK(throws<std::invalid_argument>([&] { cpl.GetPosRef("nope"); }, "Invalid contact name"));
  CHECK(throws<std::invalid_argument>([&] { cpl.SetCoMWeight(-1.0); }, "Invalid weight"));
  CHECK(throws<std::invalid_argument>([&] { cpl.SetContactForceWeight("contact2", -1.0); }, "Invalid weight"));
  CHECK(throws<std::invalid_argument>([&] { cpl.SetForceThreshold("contact1", -1.0); }, "Invalid force threshold"));
  CHECK(throws<std::invalid_argument>([&] { cpl.SetForceBounds("contact1", {0, 0, 1}, {1, 1, 0}); },
                                      "Inconsistent bounds"));
  cpl.SetPosWeight(3.0);
  cpl.SetContactForceWeight("contact3", 0.5);
  for (const auto& e : cpl.GetPosWeight()) CHECK(e.second == 3.0);
  CHECK(cpl.GetForceWeight().at("contact3") == 0.5);
  cpl.SetForceThreshold("contact2", 15.0);
  CHECK(cpl.GetForceThreshold("contact2") == 15.0);
  // src/CentroidalPlanner.cpp:340 — zero force bounds keep the threshold untouched
  cpl.SetForceBounds("contact1", {0, 0, 0}, {0, 0, 0});
  cpl.SetForceThreshold("contact1", 15.0);
  CHECK(cpl.GetForceThreshold("contact1") == 0.0);
  Vector3d lb, ub;
  cpl.SetPosBounds("contact2", {-1, -2, -3}, {1, 2, 3});
  cpl.GetPosBounds("contact2", lb, ub);
  CHECK((lb == Vector3d{-1, -2, -3}) && (ub == Vector3d{1, 2, 3}));
  cpl.GetNormalBounds("contact4", lb, ub);
  CHECK((lb == Vector3d{-1e3, -1e3, -1e3}) && (ub == Vector3d{1e3, 1e3, 1e3}));  // Variable3D.cpp:12-13
  CHECK((cpl.GetCoMRef() == Vector3d{0, 0, 1}));  // MinimizeCentroidalVariables.cpp:11-25
  CHECK(throws<std::invalid_argument>([&] { cpl.SetManipulationWrench({1, 2, 3}); }));
  cpl.SetManipulationWrench({100, 0, 0, 0, 0, 100});
  CHECK(cpl.GetManipulationWrench()[5] == 100.0);
  // shared environment: SetMu on the env is seen by every planner (src/CplProblem.cpp:275-287)
  CentroidalPlanner other({"a", "b"}, 60.0, ground);
  ground->SetMu(0.3);
  CHECK(cpl.GetMu() == 0.3 && other.GetMu() == 0.3);
  CHECK(throws<std::invalid_argument>([&] { ground->SetMu(0.0); }, "Invalid friction coefficient"));
}

// without a GPU the default solver (the native engine) cannot run: a HIP failure is a runtime_error
static void test_solve_without_gpu() {
  CentroidalPlanner cpl(NAMES, 100.0, std::make_shared<env::Ground>());
  CHECK(throws<std::runtime_error>([&] { cpl.Solve(); }));
}

static void test_environment() {
  env::Superquadric sq;
  CHECK(throws<std::invalid_argument>([&] { sq.SetParameters({0, 0, 0}, {1, -1, 1}, {2, 2, 2}); }, "radii"));
  CHECK(throws<std::invalid_argument>([&] { sq.SetParameters({0, 0, 0}, {1, 1, 1}, {2, 1.9, 2}); }, "curvatures"));
  Vector3d C, R, P;
  sq.GetParameters(C, R, P);
  CHECK((C == Vector3d{0, 0, 10}) && (R == Vector3d{10, 10, 10}) && (P == Vector3d{10, 10, 10}));
  sq.SetParameters({0, 0, 1}, {0.3, 0.3, 10}, {10, 10, 10});
  sq.GetParameters(C, R, P);
  CHECK(R[0] == 0.3 && C[2] == 1.0);
}

static void test_problem_layout() {
  auto sq = std::make_shared<env::Superquadric>();
  sq->SetParameters({0, 0, 1}, {0.3, 0.3, 10}, {10, 10, 10});
  auto prob = std::make_shared<solver::CplProblem>(NAMES, 100.0, sq);
  CHECK(prob->n() == 39 && prob->m() == 30 && prob->nnz() == 174);  // SURVEY.md §8 [probe]
  CHECK(prob->Desc().sq_R[0] == 0.3 && prob->Desc().env_kind == CPL_ENV_SUPERQUADRIC);
  CHECK(throws<std::out_of_range>([&] { prob->SetForceThreshold("missing", 1.0); }));
  auto none = std::make_shared<solver::CplProblem>(NAMES, 100.0, nullptr);
  CHECK(none->m() == 14 && none->nnz() == 114);
  // N >= 10: variable order follows the vector, solution/constraint order the std::map
  std::vector<std::string> many;
  for (int i = 1; i <= 12; ++i) many.push_back("contact" + std::to_string(i));
  solver::CplProblem big(many, 100.0, std::make_shared<env::Ground>());
  VectorXd x(big.n());
  for (int i = 0; i < big.n(); ++i) x[i] = i;
  big.SetVariables(x);
  solver::Solution sol;
  big.GetSolution(sol);
  CHECK(sol.contact_values_map.begin()->first == "contact1");
  CHECK(std::next(sol.contact_values_map.begin())->first == "contact10");
  CHECK(sol.contact_values_map.at("contact10").force_value[0] == 3 + 9 * 9);
  std::ostringstream os;
  os << sol;
  CHECK(os.str().rfind("CoM: 0 1 2\n", 0) == 0);
  CHECK(os.str().find("F_contact10: 84 85 86\n") != std::string::npos);
}

static void test_com_planner() {
  CoMPlanner cpl(NAMES, 100.0);
  for (const auto& e : cpl.GetPosWeight()) CHECK(e.second == 0.0);
  CHECK((cpl.GetContactNormal("contact3") == Vector3d{0, 0, 1}));
  CHECK(throws<std::runtime_error>([&] { cpl.GetContactPosition("contact1"); }, "not set"));
  cpl.SetContactPosition("contact1", {1, 1, 0});
  CHECK((cpl.GetContactPosition("contact1") == Vector3d{1, 1, 0}));
  CHECK(throws<std::invalid_argument>([&] { cpl.SetMu(-0.1); }, "Invalid friction coefficient"));
  cpl.SetForceThreshold("contact2", 20.0);
  cpl.SetLiftingContact("contact2");
  CHECK(cpl.GetLiftingContacts() == std::vector<std::string>{"contact2"});
  CHECK(cpl.GetForceThreshold("contact2") == 0.0);
  CHECK(throws<std::runtime_error>([&] { cpl.ResetLiftingContact("contact1"); }, "is not a lifting contact"));
  cpl.ResetLiftingContact("contact2");
  CHECK(cpl.GetLiftingContacts().empty());
  CHECK(cpl.GetForceThreshold("contact2") == 20.0);
  CHECK(throws<std::invalid_argument>([&] { cpl.SetLiftingContact("nope"); }, "Invalid contact name"));
}

// ---------------------------------------------------------------------------------------------
// GPU cases
// ---------------------------------------------------------------------------------------------
typedef int (*oracle_eval_t)(const cpl_problem_desc*, int64_t, const double*, const double*, const uint8_t*,
                             double*, double*, double*, double*, int);
static oracle_eval_t g_oracle = nullptr;

static void load_oracle(const char* path) {
  void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) throw std::runtime_error(std::string("cannot load oracle: ") + dlerror());
  g_oracle = reinterpret_cast<oracle_eval_t>(dlsym(h, "cplo_eval_batch"));
  if (!g_oracle) throw std::runtime_error("oracle has no cplo_eval_batch");
}

// seeded instances in the style of SURVEY.md §8(d): CoM box, forces inside the cone, contacts on
// the surface neighbourhood
static void fill_instance(std::mt19937_64& rng, int N, bool sq, double* x, double& mass) {
  std::uniform_real_distribution<double> U(0.0, 1.0);
  auto u = [&](double a, double b) { return a + (b - a) * U(rng); };
  x[0] = u(-0.2, 0.2);
  x[1] = u(-0.2, 0.2);
  x[2] = u(0.8, 1.2);
  mass = u(20.0, 150.0);
  for (int i = 0; i < N; ++i) {
    double* q = x + 3 + 9 * i;
    const double fn = u(0.2, 2.0) * mass * 9.81 / N;
    q[0] = u(-0.3, 0.3) * fn;
    q[1] = u(-0.3, 0.3) * fn;
    q[2] = fn;
    q[3] = u(-0.3, 0.3);
    q[4] = u(-0.3, 0.3);
    q[5] = sq ? u(0.5, 1.5) : 0.1 + u(-1e-3, 1e-3);
    q[6] = u(-1e-3, 1e-3);
    q[7] = u(-1e-3, 1e-3);
    q[8] = 1.0;
  }
}

static bool close(double a, double b, double rtol) {
  if (std::isnan(a) || std::isnan(b)) return std::isnan(a) && std::isnan(b);
  if (rtol == 0.0) return a == b;
  return std::fabs(a - b) <= rtol * std::max(1.0, std::fabs(b));
}

static void test_tnlp(env::EnvironmentClass::Ptr e, double rtol) {
  auto prob = std::make_shared<solver::CplProblem>(NAMES, 100.0, e);
  prob->SetForceThreshold("contact3", 20.0);
  prob->SetManipulationWrench({100, 0, 0, 0, 0, 100});
  solver::CplTNLP nlp(prob);
  int32_t n, m, nnz, nh;
  CHECK(nlp.get_nlp_info(n, m, nnz, nh) && n == prob->n() && nh == n * n);
  std::vector<double> xl(n), xu(n), gl(m), gu(m);
  CHECK(nlp.get_bounds_info(n, xl.data(), xu.data(), m, gl.data(), gu.data()));
  CHECK(gl[0] == 0.0 && gu[0] == 0.0 && xl[0] == -1e3);
  std::vector<double> x(n);
  CHECK(nlp.get_starting_point(n, true, x.data()) && x[5] == 0.0);
  std::mt19937_64 rng(0xC910 + 1);
  double mass;
  const bool sq = e && e->Kind() == CPL_ENV_SUPERQUADRIC;
  fill_instance(rng, 4, sq, x.data(), mass);
  std::vector<double> g(m), jac(nnz), grad(n);
  std::vector<int32_t> iRow(nnz), jCol(nnz);
  double f = 0;
  CHECK(nlp.eval_f(n, x.data(), true, f));
  CHECK(nlp.eval_grad_f(n, x.data(), false, grad.data()));
  CHECK(nlp.eval_g(n, x.data(), false, m, g.data()));
  CHECK(nlp.eval_jac_g(n, x.data(), false, m, nnz, iRow.data(), jCol.data(), nullptr));
  CHECK(nlp.eval_jac_g(n, x.data(), false, m, nnz, nullptr, nullptr, jac.data()));
  CHECK(nlp.launches() == 1);  // one fused launch served every callback of this x
  for (int k = 1; k < nnz; ++k)
    CHECK(iRow[k] > iRow[k - 1] || (iRow[k] == iRow[k - 1] && jCol[k] > jCol[k - 1]));  // RowMajor CSR
  std::vector<double> rg(m), rj(nnz), rgrad(n);
  double rf;
  CHECK(g_oracle(&prob->Desc(), 1, x.data(), nullptr, nullptr, rg.data(), rj.data(), &rf, rgrad.data(), 1) == 0);
  bool ok = close(f, rf, rtol);
  for (int i = 0; i < m; ++i) ok = ok && close(g[i], rg[i], rtol);
  for (int i = 0; i < nnz; ++i) ok = ok && close(jac[i], rj[i], rtol);
  for (int i = 0; i < n; ++i) ok = ok && close(grad[i], rgrad[i], rtol);
  CHECK(ok);
  x[0] += 0.01;
  CHECK(nlp.eval_g(n, x.data(), true, m, g.data()) && nlp.launches() == 2);
  nlp.finalize_solution(n, x.data());
  CHECK(prob->GetVariables()[0] == x[0]);
}

static void test_broker(env::EnvironmentClass::Ptr e, int64_t B, double rtol) {
  auto prob = std::make_shared<solver::CplProblem>(NAMES, 100.0, e);
  solver::BatchBroker broker(prob, B);
  const int n = prob->n(), m = prob->m(), nnz = prob->nnz();
  std::mt19937_64 rng(0xC910 + 5);
  const bool sq = e && e->Kind() == CPL_ENV_SUPERQUADRIC;
  std::vector<double> xs(B * n), ms(B);
  for (int64_t b = 0; b < B; ++b) {
    fill_instance(rng, 4, sq, xs.data() + b * n, ms[b]);
    std::memcpy(broker.x(b), xs.data() + b * n, sizeof(double) * n);
    broker.mass(b) = ms[b];
  }
  broker.Evaluate(B);
  std::vector<double> rg(B * m), rj(B * nnz), rf(B), rgrad(B * n);
  CHECK(g_oracle(&prob->Desc(), B, xs.data(), ms.data(), nullptr, rg.data(), rj.data(), rf.data(), rgrad.data(), 4) ==
        0);
  bool ok = true;
  for (int64_t b = 0; b < B; ++b) {
    ok = ok && close(broker.f(b), rf[b], rtol);
    for (int i = 0; i < m; ++i) ok = ok && close(broker.g(b)[i], rg[b * m + i], rtol);
    for (int i = 0; i < nnz; ++i) ok = ok && close(broker.jac(b)[i], rj[b * nnz + i], rtol);
    for (int i = 0; i < n; ++i) ok = ok && close(broker.grad(b)[i], rgrad[b * n + i], rtol);
  }
  CHECK(ok);
  CHECK(broker.launches() == 1);
  double norms[2];
  broker.ResidualNorms(B, norms);
  CHECK(norms[0] >= 0.0 && norms[1] >= norms[0] * norms[0] * 0.999999);
}

// a stand-in NLP solver: checks Solve() plumbing (TNLP hooks reached, finalize_solution stored)
struct FixedPointSolver : solver::NlpSolver {
  bool Solve(solver::CplTNLP& nlp) override {
    int32_t n, m, nnz, nh;
    nlp.get_nlp_info(n, m, nnz, nh);
    std::vector<double> x(n, 0.0), g(m);
    nlp.get_starting_point(n, true, x.data());
    x[2] = 1.0;
    if (!nlp.eval_g(n, x.data(), true, m, g.data())) return false;
    nlp.finalize_solution(n, x.data());
    return true;
  }
};

static void test_solve_plumbing() {
  CentroidalPlanner cpl(NAMES, 100.0, std::make_shared<env::Ground>());
  cpl.SetSolver(std::make_shared<FixedPointSolver>());
  solver::Solution sol = cpl.Solve();
  CHECK(cpl.LastSolveSucceeded());
  CHECK(sol.com_sol[2] == 1.0 && sol.contact_values_map.size() == 4);
}

// ---- TestBasic (tests/TestBasic.cpp) through the C++ facade with its default solver — the native
// engine (IPOPT's method, IFOPT's defaults: limited-memory Hessian, max_iter 3000), from the
// reference's own start point x = 0 (Variable3D's initial value, src/Variable3D.cpp:8-10; no warm
// start) — with TestBasic's own assertions and tolerances.  The solver object is the default one
// (NativeSolver with default SolveOptions), held here only to read its status and derivative report.
static Vector3d cross3(const Vector3d& a, const Vector3d& b) {
  return {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
}
static double dot3(const Vector3d& a, const Vector3d& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static double norm3(const Vector3d& a) { return std::sqrt(dot3(a, a)); }
#define NEAR(a, b, tol) CHECK(std::fabs((a) - (b)) <= (tol))

static void check_balance(const solver::Solution& sol, double mass, const std::vector<double>& w, double mu,
                          double ttol) {
  Vector3d F{0, 0, 0}, T{0, 0, 0};
  for (const auto& e : sol.contact_values_map) {
    const auto& v = e.second;
    Vector3d r{v.position_value[0] - sol.com_sol[0], v.position_value[1] - sol.com_sol[1],
               v.position_value[2] - sol.com_sol[2]};
    const Vector3d t = cross3(r, v.force_value);
    for (int k = 0; k < 3; ++k) { F[k] += v.force_value[k]; T[k] += t[k]; }
    const double fn = dot3(v.force_value, v.normal_value);
    Vector3d ft;
    for (int k = 0; k < 3; ++k) ft[k] = v.force_value[k] - fn * v.normal_value[k];
    CHECK(-fn <= 0.0);                            // TestBasic.cpp:122-123 (cone signs, as asserted there)
    CHECK(norm3(ft) - mu * fn <= 0.0);
  }
  NEAR(F[0], w[0], 1e-6);
  NEAR(F[1], w[1], 1e-6);
  NEAR(F[2], mass * 9.81 + w[2], 1e-6);
  NEAR(T[0], w[3], ttol);
  NEAR(T[1], w[4], ttol);
  NEAR(T[2], w[5], ttol);
}

static void test_testbasic_native() {
  const double mass = 100.0, g = -9.81;
  {  // testSimpleProblem (TestBasic.cpp:28-61): default settings, from x = 0
    auto ground = std::make_shared<env::Ground>();
    ground->SetGroundZ(0.1);
    CentroidalPlanner cpl({"contact1"}, mass, ground);
    solver::Solution sol = cpl.Solve();
    double Fz = 0.0;
    for (const auto& e : sol.contact_values_map) {
      Fz += e.second.force_value[2];
      NEAR(e.second.position_value[2], 0.1, 1e-6);
      NEAR(norm3(e.second.normal_value), 1.0, 1e-6);
      NEAR(e.second.normal_value[2], 1.0, 1e-6);
    }
    NEAR(Fz, -mass * g, 1e-6);
  }
  {  // the same with IPOPT's Jacobian regularisation (SolveOptions::jacobian_regularization = 1): every
     // Newton system here is rank deficient; the regularised form converges
    auto ground = std::make_shared<env::Ground>();
    ground->SetGroundZ(0.1);
    CentroidalPlanner cpl({"contact1"}, mass, ground);
    solver::SolveOptions opt;
    opt.jacobian_regularization = 1;
    auto ns = std::make_shared<solver::NativeSolver>(opt);
    cpl.SetSolver(ns);
    solver::Solution sol = cpl.Solve();
    std::printf("testSimpleProblem (IPOPT's Jacobian regularisation): status %d after %d iterations\n", ns->status(),
                ns->iterations());
    CHECK(ns->status() == CPL_SOLVE_OPTIMAL && ns->iterations() <= 20);
    double Fz = 0.0;
    for (const auto& e : sol.contact_values_map) Fz += e.second.force_value[2];
    NEAR(Fz, -mass * g, 1e-6);
  }
  const std::vector<double> wrench = {100, 0, 0, 0, 0, 100};
  {  // testGroundEnv (TestBasic.cpp:64-135): ends at the iteration limit (the unloaded contacts' cone
     // apex); the returned point is checked, as TestBasic does
    auto ground = std::make_shared<env::Ground>();
    ground->SetGroundZ(0.1);
    ground->SetMu(0.5);
    CentroidalPlanner cpl(NAMES, mass, ground);
    cpl.SetCoMWeight(2.0);
    cpl.SetForceWeight(0.0);
    for (const auto& c : NAMES) cpl.SetPosBounds(c, {-0.3, -0.3, 0.0}, {0.3, 0.3, 1.0});
    cpl.SetManipulationWrench(wrench);
    auto ns = std::make_shared<solver::NativeSolver>();
    cpl.SetSolver(ns);
    solver::Solution sol = cpl.Solve();
    {  // derivative_test = first-order ran at the start point (src/CentroidalPlanner.cpp:26)
      const cpl_derivative_report& dr = ns->derivative_report();
      CHECK(dr.n_checked == 39 * (30 + 1));
      CHECK(dr.worst_row >= -1 && dr.worst_col >= 0);
    }
    // x = 0: every cone's Jacobian row is 0/0 (FrictionCone.cpp:85-87), reported as substituted
    CHECK(ns->nan_jacobian_at_start() > 0);
    std::printf("testGroundEnv: status %d after %d iterations (%d NaN Jacobian entries at the start)\n", ns->status(),
                ns->iterations(), ns->nan_jacobian_at_start());
    for (const auto& e : sol.contact_values_map) {
      NEAR(e.second.position_value[2], 0.1, 1e-6);
      NEAR(norm3(e.second.normal_value), 1.0, 1e-6);
      NEAR(e.second.normal_value[2], 1.0, 1e-6);
    }
    check_balance(sol, mass, wrench, 0.5, 1e-5);
  }
  {  // testSuperquadricEnv (TestBasic.cpp:138-222)
    auto sq = std::make_shared<env::Superquadric>();
    sq->SetMu(0.5);
    sq->SetParameters({0, 0, 1}, {0.3, 0.3, 10}, {10, 10, 10});
    CentroidalPlanner cpl(NAMES, mass, sq);
    cpl.SetForceWeight(0.0);
    for (const auto& c : NAMES) cpl.SetPosBounds(c, {-0.5, -0.5, 0.5}, {0.5, 0.5, 1.5});
    cpl.SetManipulationWrench(wrench);
    auto ns = std::make_shared<solver::NativeSolver>();
    cpl.SetSolver(ns);
    solver::Solution sol = cpl.Solve();
    std::printf("testSuperquadricEnv: status %d after %d iterations\n", ns->status(), ns->iterations());
    CHECK(cpl.LastSolveSucceeded());
    for (const auto& e : sol.contact_values_map) {
      const Vector3d& p = e.second.position_value;
      const double C[3] = {0, 0, 1}, R[3] = {0.3, 0.3, 10};
      double v = 0.0;
      for (int k = 0; k < 3; ++k) v += std::pow((p[k] - C[k]) / R[k], 10.0);
      NEAR(v, 1.0, 1e-4);
      NEAR(norm3(e.second.normal_value), 1.0, 1e-6);
      CHECK(p[0] >= -0.5 && p[0] <= 0.5 && p[1] >= -0.5 && p[1] <= 0.5 && p[2] >= 0.5 && p[2] <= 1.5);
    }
    check_balance(sol, mass, wrench, 0.5, 1e-4);
  }
  {  // testCoMPlanner (TestBasic.cpp:225-292)
    CoMPlanner cpl(NAMES, mass);
    cpl.SetMu(0.5);
    cpl.SetContactPosition("contact1", {1.0, 1.0, 0.0});
    cpl.SetContactPosition("contact2", {-1.0, 1.0, 0.0});
    cpl.SetContactPosition("contact3", {-1.0, -1.0, 0.0});
    cpl.SetContactPosition("contact4", {1.0, -1.0, 0.0});
    cpl.SetLiftingContact("contact4");
    for (const auto& c : NAMES) cpl.SetForceThreshold(c, 20.0);
    auto ns = std::make_shared<solver::NativeSolver>();
    cpl.SetSolver(ns);
    solver::Solution sol = cpl.Solve();
    std::printf("testCoMPlanner: status %d after %d iterations\n", ns->status(), ns->iterations());
    CHECK(cpl.LastSolveSucceeded());
    check_balance(sol, mass, std::vector<double>(6, 0.0), 0.5, 1e-4);
  }
}

// the batched engine from C++: many instances, host arrays (configs[4]'s problem)
static void test_batch_solver() {
  auto ground = std::make_shared<env::Ground>();
  ground->SetGroundZ(0.1);
  ground->SetMu(0.5);
  auto prob = std::make_shared<solver::CplProblem>(NAMES, 100.0, ground);
  prob->SetCoMWeight(2.0);
  for (const auto& c : NAMES) prob->SetPosBounds(c, {-0.3, -0.3, 0.0}, {0.3, 0.3, 1.0});
  prob->SetManipulationWrench({100, 0, 0, 0, 0, 100});
  const int64_t B = 64;
  const int n = prob->n();
  std::vector<double> x0(B * n, 0.0), mass(B), x(B * n), obj(B), pinf(B);
  std::vector<int32_t> status(B), its(B);
  for (int64_t b = 0; b < B; ++b) {
    mass[b] = 80.0 + 70.0 * (double)b / (double)(B - 1);
    double* xb = &x0[b * n];
    xb[2] = 1.0;
    for (int i = 0; i < 4; ++i) {
      const double ang = 2.0 * M_PI * (i + 0.125) / 4;
      double* q = xb + 3 + 9 * i;
      q[0] = 1.0; q[1] = 1.0; q[2] = mass[b] * 9.81 / 4;
      q[3] = 0.2 * std::cos(ang); q[4] = 0.2 * std::sin(ang); q[5] = 0.05;
      q[8] = 1.0;
    }
  }
  solver::SolveOptions opt;
  opt.hessian = CPL_HESSIAN_EXACT;
  solver::BatchSolver bs(prob, B, opt);
  for (int rep = 0; rep < 2; ++rep) {  // the second solve replays the captured iteration
    bs.Solve(x0.data(), mass.data(), x.data(), nullptr, status.data(), its.data(), obj.data(), pinf.data());
    CHECK(bs.graph_captured());
    double worst = 0.0;
    for (int64_t b = 0; b < B; ++b) {
      CHECK(status[b] == CPL_SOLVE_OPTIMAL || status[b] == CPL_SOLVE_ACCEPTABLE);
      worst = std::fmax(worst, pinf[b]);
      // force balance against this instance's mass (TestBasic.cpp:126-128 tolerance)
      double Fz = 0.0;
      for (int i = 0; i < 4; ++i) Fz += x[b * n + 5 + 9 * i];
      NEAR(Fz, mass[b] * 9.81, 1e-6);
    }
    std::printf("batch solver: %d lock-step iterations, worst primal infeasibility %.3g\n", bs.iterations_run(), worst);
    CHECK(worst <= 1e-4);  // IPOPT constr_viol_tol
  }
}

int main(int argc, char** argv) {
  bool gpu = false;
  const char* oracle = nullptr;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--gpu")) gpu = true;
    if (!std::strcmp(argv[i], "--oracle") && i + 1 < argc) oracle = argv[++i];
  }
  try {
    test_planner_api();
    test_environment();
    test_problem_layout();
    test_com_planner();
    if (!gpu) test_solve_without_gpu();
    if (gpu) {
      if (!oracle) throw std::runtime_error("--gpu needs --oracle <libcpl_oracle.so>");
      load_oracle(oracle);
      auto sq = std::make_shared<env::Superquadric>();
      sq->SetParameters({0, 0, 1}, {0.3, 0.3, 10}, {10, 10, 10});
      auto ground = std::make_shared<env::Ground>();
      ground->SetGroundZ(0.1);
      test_tnlp(ground, 0.0);   // bitwise
      test_tnlp(nullptr, 0.0);  // bitwise
      test_tnlp(sq, 1e-9);      // pow entries: the Python suite holds the conditioning-aware policy
      test_broker(ground, 3001, 0.0);
      test_broker(sq, 1001, 1e-9);
      test_solve_plumbing();
      test_testbasic_native();
      test_batch_solver();
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "FAIL: uncaught exception: %s\n", e.what());
    ++g_fail;
  }
  std::printf("%d passed, %d failed\n", g_pass, g_fail);
  return g_fail ? 1 : 0;
}
