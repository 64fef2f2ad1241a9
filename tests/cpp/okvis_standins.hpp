// Stand-ins for the okvis functor classes whose protected members the facade's accessors
// (include/okvisgpu_problem.hpp, namespace okvisgpu::okvis_access) read and write. Eigen, Ceres and
// okvis are not in this image, so these mirror the reference headers' member NAMES, TYPES (through
// a minimal Eigen-shaped matrix / quaternion: column-major storage, m(r, c), v(i), q.x() ...),
// `mutable` qualifiers and access levels, plus the public getters the adapters use:
//   okvis::ceres::ImuError                      okvis_ceres/include/okvis/ceres/ImuError.hpp:123-306
//   okvis::ceres::TwoPoseGraphError (base part) TwoPoseGraphError.hpp:130-179
//   okvis::ceres::TwoPoseStandardGraphError     TwoPoseGraphError.hpp:278-284
//   okvis::ceres::TwoPoseStandardGraphErrorConst TwoPoseGraphError.hpp:294-373
//   okvis::ceres::RelativePoseError             RelativePoseError.hpp:148-150
//   okvis::ceres::PoseError                     PoseError.hpp:166-170 (+ PoseError.cpp:34-39,57-63)
//   okvis::ceres::SpeedAndBiasError             SpeedAndBiasError.hpp:163-168
// Test infrastructure only.
#pragma once

#include <cmath>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

namespace mini {  // the Eigen subset the adapters touch
template <int R, int C>
struct Matrix {
  double a[R * C] = {};  // column-major, as Eigen's default
  double& operator()(int r, int c) { return a[c * R + r]; }
  double operator()(int r, int c) const { return a[c * R + r]; }
  double& operator()(int i) { return a[i]; }
  double operator()(int i) const { return a[i]; }
  double& operator[](int i) { return a[i]; }
  double operator[](int i) const { return a[i]; }
  static Matrix Zero() { return Matrix(); }
  static Matrix Identity() {
    Matrix m;
    for (int i = 0; i < (R < C ? R : C); ++i) m(i, i) = 1.0;
    return m;
  }
};
struct Quaterniond {  // Eigen::Quaterniond(w, x, y, z) constructor order, coeffs x y z w
  double c[4] = {0, 0, 0, 1};
  Quaterniond() = default;
  Quaterniond(double w, double x, double y, double z) : c{x, y, z, w} {}
  double& x() { return c[0]; }
  double& y() { return c[1]; }
  double& z() { return c[2]; }
  double& w() { return c[3]; }
  double x() const { return c[0]; }
  double y() const { return c[1]; }
  double z() const { return c[2]; }
  double w() const { return c[3]; }
};
template <class T>
using AlignedVector = std::vector<T>;
}  // namespace mini

namespace okvis {
struct Time {  // okvis::Time (okvis_time/include/okvis/Time.hpp): sec / nsec
  uint32_t sec = 0, nsec = 0;
  Time() = default;
  static Time fromNSec(int64_t ns) {
    Time t;
    t.sec = (uint32_t)(ns / 1000000000);
    t.nsec = (uint32_t)(ns % 1000000000);
    return t;
  }
  uint64_t toNSec() const { return (uint64_t)sec * 1000000000ull + nsec; }
};
struct ImuSensorReadings {
  mini::Matrix<3, 1> gyroscopes, accelerometers;
};
template <class M>
struct Measurement {
  Time timeStamp;
  M measurement;
};
using ImuMeasurement = Measurement<ImuSensorReadings>;
using ImuMeasurementDeque = std::deque<ImuMeasurement>;
struct ImuParameters {  // okvis_util/include/okvis/Parameters.hpp (the fields the factor uses)
  double a_max = 200.0, g_max = 10.0, sigma_g_c = 12e-4, sigma_a_c = 8e-3, sigma_bg = 0.01, sigma_ba = 0.1,
         sigma_gw_c = 4e-6, sigma_aw_c = 4e-5, g = 9.81;
};
using SpeedAndBias = mini::Matrix<9, 1>;

namespace kinematics {
class Transformation {  // parameters [r_AB, q_AB xyzw] (Transformation.hpp:92-123)
 public:
  Transformation() { c_(6) = 1.0; }
  explicit Transformation(const double* coeffs) {
    for (int i = 0; i < 7; ++i) c_(i) = coeffs[i];
  }
  const mini::Matrix<7, 1>& coeffs() const { return c_; }

 private:
  mini::Matrix<7, 1> c_;
};
}  // namespace kinematics

namespace ceres {
class ImuError {
 public:
  typedef mini::Matrix<15, 15> information_t;
  ImuError() = default;
  ImuError(const ImuMeasurementDeque& m, const ImuParameters& p, const Time& t0, const Time& t1)
      : imuParameters_(p), imuMeasurements_(m), t0_(t0), t1_(t1) {}
  virtual ~ImuError() = default;
  Time t0() const { return t0_; }
  Time t1() const { return t1_; }
  void setT1(const Time& t) { t1_ = t; }
  const ImuParameters& imuParameters() const { return imuParameters_; }
  const ImuMeasurementDeque& imuMeasurements() const { return imuMeasurements_; }
  void setImuMeasurements(const ImuMeasurementDeque& m) { imuMeasurements_ = m; }
  std::string typeInfo() const { return "ImuError"; }

 protected:
  ImuParameters imuParameters_;
  ImuMeasurementDeque imuMeasurements_;
  mutable std::mutex preintegrationMutex_;
  mutable mini::Quaterniond Delta_q_ = mini::Quaterniond(1, 0, 0, 0);
  mutable mini::Matrix<3, 3> C_integral_ = mini::Matrix<3, 3>::Zero();
  mutable mini::Matrix<3, 3> C_doubleintegral_ = mini::Matrix<3, 3>::Zero();
  mutable mini::Matrix<3, 1> acc_integral_ = mini::Matrix<3, 1>::Zero();
  mutable mini::Matrix<3, 1> acc_doubleintegral_ = mini::Matrix<3, 1>::Zero();
  mutable mini::Matrix<3, 3> cross_ = mini::Matrix<3, 3>::Zero();
  mutable mini::Matrix<3, 3> dalpha_db_g_ = mini::Matrix<3, 3>::Zero();
  mutable mini::Matrix<3, 3> dv_db_g_ = mini::Matrix<3, 3>::Zero();
  mutable mini::Matrix<3, 3> dp_db_g_ = mini::Matrix<3, 3>::Zero();
  mutable mini::Matrix<15, 15> P_delta_ = mini::Matrix<15, 15>::Zero();
  mutable SpeedAndBias speedAndBiases_ref_ = SpeedAndBias::Zero();
  mutable bool redo_ = true;
  mutable int redoCounter_ = 0;
  mutable information_t information_;
  mutable information_t squareRootInformation_;
  mutable mini::AlignedVector<mini::Matrix<15, 15>> dPdsigma_;
  Time t0_, t1_;  // ImuErrorBase (ImuError.hpp:116-119)
};

class TwoPoseGraphError {  // the base part the standard error inherits (TwoPoseGraphError.hpp:130-179)
 public:
  virtual ~TwoPoseGraphError() = default;

 protected:
  bool errorComputationValid_ = false;
  bool isComputed_ = false;
  kinematics::Transformation linearisationPoint_T_S0S1_;
};
class TwoPoseStandardGraphError : public TwoPoseGraphError {
 public:
  // (the reference fills these in compute(); the stand-in takes them directly)
  TwoPoseStandardGraphError(const double* dx, const double* J_rowmajor, const double* lp) {
    for (int i = 0; i < 6; ++i) DeltaX_(i) = dx[i];
    for (int r = 0; r < 6; ++r)
      for (int c = 0; c < 6; ++c) J_(r, c) = J_rowmajor[6 * r + c];
    linearisationPoint_T_S0S1_ = kinematics::Transformation(lp);
    isComputed_ = true;
  }
  std::string typeInfo() const { return "TwoPoseStandardGraphError"; }

 protected:
  mini::Matrix<6, 6> H00_;
  mini::Matrix<6, 1> b0_;
  mini::Matrix<6, 1> DeltaX_;
  mini::Matrix<6, 6> J_;
};
class TwoPoseStandardGraphErrorConst {
 public:
  TwoPoseStandardGraphErrorConst() = delete;
  TwoPoseStandardGraphErrorConst(const mini::Matrix<6, 1>& DeltaX, const mini::Matrix<6, 6>& J,
                                 const kinematics::Transformation& lp)
      : DeltaX_(DeltaX), J_(J), linearisationPoint_T_S0S1_(lp) {}
  virtual ~TwoPoseStandardGraphErrorConst() = default;
  std::string typeInfo() const { return "TwoPoseStandardGraphErrorConst"; }

 protected:
  mini::Matrix<6, 1> DeltaX_;
  mini::Matrix<6, 6> J_;
  kinematics::Transformation linearisationPoint_T_S0S1_;
};

class RelativePoseError {
 public:
  // (information, T_AB); the stand-in takes the square root directly
  RelativePoseError(const double* sqrt_rowmajor, const kinematics::Transformation& T_AB) : T_AB_(T_AB) {
    for (int r = 0; r < 6; ++r)
      for (int c = 0; c < 6; ++c) squareRootInformation_(r, c) = sqrt_rowmajor[6 * r + c];
  }
  virtual ~RelativePoseError() = default;
  std::string typeInfo() const { return "RelativePoseError"; }

 protected:
  kinematics::Transformation T_AB_;
  mini::Matrix<6, 6> information_;
  mini::Matrix<6, 6> squareRootInformation_;
};

class PoseError {
 public:
  // PoseError(measurement, translationVariance, rotationVariance)-style diagonal constructor
  // (PoseError.cpp:28-39): squareRootInformation_ = sqrt(diag(information))
  PoseError(const kinematics::Transformation& m, const double* infoDiag) : measurement_(m) {
    for (int i = 0; i < 6; ++i) {
      information_(i, i) = infoDiag[i];
      squareRootInformation_(i, i) = std::sqrt(infoDiag[i]);
    }
  }
  // full square root (the LLT constructor's result, PoseError.cpp:57-63, given directly)
  PoseError(const kinematics::Transformation& m, const double* sqrt_rowmajor, int) : measurement_(m) {
    for (int r = 0; r < 6; ++r)
      for (int c = 0; c < 6; ++c) squareRootInformation_(r, c) = sqrt_rowmajor[6 * r + c];
  }
  virtual ~PoseError() = default;
  std::string typeInfo() const { return "PoseError"; }

 protected:
  kinematics::Transformation measurement_;
  mini::Matrix<6, 6> information_;
  mini::Matrix<6, 6> squareRootInformation_;
};

class SpeedAndBiasError {
 public:
  SpeedAndBiasError(const SpeedAndBias& m, const double* sqrt_rowmajor) : measurement_(m) {
    for (int r = 0; r < 9; ++r)
      for (int c = 0; c < 9; ++c) squareRootInformation_(r, c) = sqrt_rowmajor[9 * r + c];
  }
  virtual ~SpeedAndBiasError() = default;
  std::string typeInfo() const { return "SpeedAndBiasError"; }

 protected:
  SpeedAndBias measurement_;
  mini::Matrix<9, 9> information_;
  mini::Matrix<9, 9> squareRootInformation_;
  mini::Matrix<9, 9> covariance_;
};
}  // namespace ceres
}  // namespace okvis
