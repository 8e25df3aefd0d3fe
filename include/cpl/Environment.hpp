// cpl/Environment.hpp — host-side environment classes of the MI355X engine.
//
// Mirrors include/CentroidalPlanner/Environment/{Environment,Ground,Superquadric}.h of the
// reference: same class names, setters/getters, defaults and exceptions.  The per-point
// evaluation virtuals of the reference (GetEnvironmentValue / GetEnvironmentJacobian /
// GetNormalValue / GetNormalJacobian, Environment.h:30-40) are not host methods here: the
// environment is evaluated inside the batched HIP kernels only (cpl_eval_batch), and a host class
// contributes its parameters to the problem descriptor instead (FillDesc).
#pragma once

#include <array>
#include <memory>
#include <stdexcept>

#include "cpl_mi355x.h"

namespace cpl {

using Vector3d = std::array<double, 3>;

namespace env {

// include/CentroidalPlanner/Environment/Environment.h:13-48
class EnvironmentClass {
 public:
  typedef std::shared_ptr<EnvironmentClass> Ptr;

  // Environment.h:19-26
  void SetMu(const double& mu) {
    if (mu <= 0.0) throw std::invalid_argument("Invalid friction coefficient");
    _mu = mu;
  }
  double GetMu() const { return _mu; }

  // descriptor kind (CPL_ENV_GROUND / CPL_ENV_SUPERQUADRIC / CPL_ENV_MIXED)
  virtual int32_t Kind() const = 0;
  // folds the environment's current state (mu and shape parameters) into a descriptor
  virtual void FillDesc(cpl_problem_desc& d) const { d.mu = _mu; }

  virtual ~EnvironmentClass() = default;

 protected:
  double _mu = 1.0;  // Environment.h:46
};

// include/CentroidalPlanner/Environment/Ground.h, src/Ground.cpp
class Ground : public EnvironmentClass {
 public:
  typedef std::shared_ptr<Ground> Ptr;
  Ground() = default;
  void SetGroundZ(const double& ground_z) { _ground_z = ground_z; }
  double GetGroundZ() const { return _ground_z; }
  int32_t Kind() const override { return CPL_ENV_GROUND; }
  void FillDesc(cpl_problem_desc& d) const override {
    EnvironmentClass::FillDesc(d);
    d.ground_z = _ground_z;
  }

 private:
  double _ground_z = 0.0;  // src/Ground.cpp:7
};

// include/CentroidalPlanner/Environment/Superquadric.h, src/Superquadric.cpp
class Superquadric : public EnvironmentClass {
 public:
  typedef std::shared_ptr<Superquadric> Ptr;
  Superquadric() = default;
  // src/Superquadric.cpp:12-29; throws std::invalid_argument for R <= 0 or P < 2
  void SetParameters(const Vector3d& C, const Vector3d& R, const Vector3d& P);
  void GetParameters(Vector3d& C, Vector3d& R, Vector3d& P) const {
    C = _C;
    R = _R;
    P = _P;
  }
  int32_t Kind() const override { return CPL_ENV_SUPERQUADRIC; }
  void FillDesc(cpl_problem_desc& d) const override;

 private:
  Vector3d _C{0.0, 0.0, 10.0};  // src/Superquadric.cpp:7-9
  Vector3d _R{10.0, 10.0, 10.0};
  Vector3d _P{10.0, 10.0, 10.0};
};

// Not a reference class: a batch whose instances are each on the Ground or on the Superquadric,
// selected per instance by the env_tag array of cpl_eval_batch.
class MixedEnvironment : public EnvironmentClass {
 public:
  typedef std::shared_ptr<MixedEnvironment> Ptr;
  MixedEnvironment(Ground::Ptr ground, Superquadric::Ptr superquadric)
      : _ground(std::move(ground)), _sq(std::move(superquadric)) {
    if (!_ground || !_sq) throw std::invalid_argument("MixedEnvironment needs a ground and a superquadric");
    _mu = _ground->GetMu();
  }
  int32_t Kind() const override { return CPL_ENV_MIXED; }
  void FillDesc(cpl_problem_desc& d) const override {
    _sq->FillDesc(d);
    _ground->FillDesc(d);
    d.mu = _mu;
  }

 private:
  Ground::Ptr _ground;
  Superquadric::Ptr _sq;
};

}  // namespace env
}  // namespace cpl
