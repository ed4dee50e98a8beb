// fdtd3d -- standalone native driver (no Python): command line -> device
// fields -> HIP kernels -> timing report, the counterpart of the reference's
// Source/main.cpp built directly on libfdtd3d_hip's C ABI.
//
// Covers the plain Yee solvers (1D, 2D TMz/TEz, 3D) on one GPU with the
// vacuum / dielectric-sphere scenes and the hard point source, fp32 or fp64,
// fused or split 3D kernels, CPML absorbing layers in 3D fp32 (--use-pml
// --pml-type cpml; with hybrid passes -- blocked core, stepped shell -- like
// the Python driver's automatic plan), the UPML in the reference's D/B form and Drude / Lorentz
// spheres (--use-metamaterials, scene drude-sphere) in 3D through the fused
// chain kernel, TF/SF plane waves in 3D, the NTFF scattered power diagram
// (--use-ntff) and DAT/BMP output of the final fields (native_physics.h).
// 2D TF/SF / PML, amplitude mode and multi-GPU runs go through the Python
// driver (python -m fdtd3d_amd), which shares the kernels; asking this
// binary for them is an error, never a silent fallback.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "capi.h"
#include "host_native.h"
#include "native_physics.h"
#include "settings_native.h"

namespace {

constexpr double kC = 2.99792458e8;
constexpr double kEps0 = 8.8541878176203892e-12;
constexpr double kMu0 = 1.2566370614359173e-6;
constexpr double kPi = 3.14159265358979323846;

#define HIP_OK(x)                                                                       \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

#define K_OK(x)                                                              \
  do {                                                                       \
    int r_ = (x);                                                            \
    if (r_ != 0) {                                                           \
      std::fprintf(stderr, "kernel launch failed (%d) at %s:%d\n", r_, __FILE__, __LINE__); \
      std::exit(1);                                                          \
    }                                                                        \
  } while (0)

double sphere_eps(double x, double y, double z, const double c[3], double r, double eps) {
  // linear sub-cell smoothing (reference Approximation.cpp:286-314)
  const double d = std::sqrt((x - c[0]) * (x - c[0]) + (y - c[1]) * (y - c[1]) + (z - c[2]) * (z - c[2]));
  const double diff = d - r;
  if (diff < -0.5) return eps;
  if (diff > 0.5) return 1.0;
  const double p = 0.5 - diff;
  return p * eps + (1 - p) * 1.0;
}

template <typename T>
struct Dev {
  T* p = nullptr;
  size_t n = 0;
  void alloc(size_t count) {
    n = count;
    HIP_OK(hipMalloc(&p, n * sizeof(T)));
    HIP_OK(hipMemset(p, 0, n * sizeof(T)));
  }
  ~Dev() {
    if (p) (void)hipFree(p);
  }
};

template <typename T>
struct Api;
template <>
struct Api<float> {
  static constexpr const char* name = "float";
};
template <>
struct Api<double> {
  static constexpr const char* name = "double";
};

int e3d(float* a, float* b, float* c, const float* d, const float* e, const float* f, const float* g,
        const float* h, const float* i, double cb, int nx, int ny, int nz, const int* bx, int xc, void* s, bool v4) {
  return v4 ? fdtd_update_e3d_v4_f32(a, b, c, d, e, f, g, h, i, cb, nx, ny, nz, bx, xc, s)
            : fdtd_update_e3d_f32(a, b, c, d, e, f, g, h, i, cb, nx, ny, nz, bx, xc, s);
}
int e3d(double* a, double* b, double* c, const double* d, const double* e, const double* f, const double* g,
        const double* h, const double* i, double cb, int nx, int ny, int nz, const int* bx, int xc, void* s, bool) {
  return fdtd_update_e3d_f64(a, b, c, d, e, f, g, h, i, cb, nx, ny, nz, bx, xc, s);
}
int h3d(float* a, float* b, float* c, const float* d, const float* e, const float* f, const float* g,
        const float* h, const float* i, double cb, int nx, int ny, int nz, const int* bx, int xc, void* s, bool v4) {
  return v4 ? fdtd_update_h3d_v4_f32(a, b, c, d, e, f, g, h, i, cb, nx, ny, nz, bx, xc, s)
            : fdtd_update_h3d_f32(a, b, c, d, e, f, g, h, i, cb, nx, ny, nz, bx, xc, s);
}
int h3d(double* a, double* b, double* c, const double* d, const double* e, const double* f, const double* g,
        const double* h, const double* i, double cb, int nx, int ny, int nz, const int* bx, int xc, void* s, bool) {
  return fdtd_update_h3d_f64(a, b, c, d, e, f, g, h, i, cb, nx, ny, nz, bx, xc, s);
}
int fused(const float* const* ei, const float* const* hi, float* const* eo, float* const* ho,
          const float* const* cbs, const float* const* dbs, double cb, double db, int nx, int ny, int nz,
          const int* bx, long long so, int sc, double sv, void* s, bool v4) {
  return v4 ? fdtd_fused3d_v4_f32(ei, hi, eo, ho, cbs, dbs, cb, db, nx, ny, nz, bx, 0, so, sc, sv, s)
            : fdtd_fused3d_f32(ei, hi, eo, ho, cbs, dbs, cb, db, nx, ny, nz, bx, 0, so, sc, sv, s);
}
int fused(const double* const* ei, const double* const* hi, double* const* eo, double* const* ho,
          const double* const* cbs, const double* const* dbs, double cb, double db, int nx, int ny, int nz,
          const int* bx, long long so, int sc, double sv, void* s, bool) {
  return fdtd_fused3d_f64(ei, hi, eo, ho, cbs, dbs, cb, db, nx, ny, nz, bx, 0, so, sc, sv, s);
}
// temporally blocked pass (fp32: yee3d_tb.hip, fp64: yee3d_tb64.hip)
// fp32: a sparse float4 box of the E coefficients (ce4 over ebox, scalar cb
// elsewhere, scalar db) takes the multi-row kernel; otherwise per-kind arrays
int tb3d(const float* const* ei, const float* const* hi, float* const* eo, float* const* ho, const float* const* cbs,
         const float* const* dbs, double cb, double db, int nx, int ny, int nz, const int* bx, int T,
         const int* src, const double* vals, void* s, const void* ce4 = nullptr, const int* ebox = nullptr,
         const int* obox = nullptr) {
  const int whole[6] = {0, 0, 0, nx, ny, nz};
  const int* ob = obox ? obox : whole;
  if (ce4) {
    const int none[6] = {0, 0, 0, 0, 0, 0};
    return fdtd_tb3d_ext_f32(ei, hi, eo, ho, ce4, ebox, nullptr, none, cb, db, nx, ny, nz, bx, ob, 0, T, src, vals,
                             nullptr, nullptr, s);
  }
  return fdtd_tb3d_v4_f32(ei, hi, eo, ho, cbs, dbs, cb, db, nx, ny, nz, bx, ob, 0, T, src, vals, s);
}
int tb3d(const double* const* ei, const double* const* hi, double* const* eo, double* const* ho,
         const double* const* cbs, const double* const* dbs, double cb, double db, int nx, int ny, int nz,
         const int* bx, int T, const int* src, const double* vals, void* s, const void* = nullptr,
         const int* = nullptr) {
  const int ob[6] = {0, 0, 0, nx, ny, nz};
  return fdtd_tb3d_f64(ei, hi, eo, ho, cbs, dbs, cb, db, nx, ny, nz, bx, ob, 0, T, src, vals, s);
}
int tb2d(int mode, const float* const* ei, const float* const* hi, float* const* eo, float* const* ho,
         const float* const* cs, double cb, double db, int nx, int ny, const int* bx, const int* ob, int T,
         const int* src, const double* vals, void* s) {
  return fdtd_tb2d_f32(mode, ei, hi, eo, ho, cs, cb, db, nx, ny, bx, ob, 0, T, src, vals, s);
}
int tb2d(int mode, const double* const* ei, const double* const* hi, double* const* eo, double* const* ho,
         const double* const* cs, double cb, double db, int nx, int ny, const int* bx, const int* ob, int T,
         const int* src, const double* vals, void* s) {
  return fdtd_tb2d_f64(mode, ei, hi, eo, ho, cs, cb, db, nx, ny, bx, ob, 0, T, src, vals, s);
}
int res1d(float* ez, float* hy, const float* ce, const float* ch, double cb, double db, int n, const int* bx, int steps,
          int si, const float* vals, void* s) {
  return fdtd_res1d_f32(ez, hy, ce, ch, cb, db, n, bx, steps, si, vals, s);
}
int res1d(double* ez, double* hy, const double* ce, const double* ch, double cb, double db, int n, const int* bx,
          int steps, int si, const double* vals, void* s) {
  return fdtd_res1d_f64(ez, hy, ce, ch, cb, db, n, bx, steps, si, vals, s);
}
int setv(float* f, long long off, double v, void* s) { return fdtd_set_value_f32(f, off, v, s); }
int setv(double* f, long long off, double v, void* s) { return fdtd_set_value_f64(f, off, v, s); }
int tmz_e(float* a, const float* b, const float* c, const float* d, double cb, int nx, int ny, const int* bx, void* s) {
  return fdtd_tmz_e_f32(a, b, c, d, cb, nx, ny, bx, 0, s);
}
int tmz_e(double* a, const double* b, const double* c, const double* d, double cb, int nx, int ny, const int* bx,
          void* s) {
  return fdtd_tmz_e_f64(a, b, c, d, cb, nx, ny, bx, 0, s);
}
int tmz_h(float* a, float* b, const float* c, const float* d, const float* e, double db, int nx, int ny,
          const int* bx, void* s) {
  return fdtd_tmz_h_f32(a, b, c, d, e, db, nx, ny, bx, 0, s);
}
int tmz_h(double* a, double* b, const double* c, const double* d, const double* e, double db, int nx, int ny,
          const int* bx, void* s) {
  return fdtd_tmz_h_f64(a, b, c, d, e, db, nx, ny, bx, 0, s);
}
int tez_e(float* a, float* b, const float* c, const float* d, const float* e, double cb, int nx, int ny,
          const int* bx, void* s) {
  return fdtd_tez_e_f32(a, b, c, d, e, cb, nx, ny, bx, 0, s);
}
int tez_e(double* a, double* b, const double* c, const double* d, const double* e, double cb, int nx, int ny,
          const int* bx, void* s) {
  return fdtd_tez_e_f64(a, b, c, d, e, cb, nx, ny, bx, 0, s);
}
int tez_h(float* a, const float* b, const float* c, const float* d, double db, int nx, int ny, const int* bx, void* s) {
  return fdtd_tez_h_f32(a, b, c, d, db, nx, ny, bx, 0, s);
}
int tez_h(double* a, const double* b, const double* c, const double* d, double db, int nx, int ny, const int* bx,
          void* s) {
  return fdtd_tez_h_f64(a, b, c, d, db, nx, ny, bx, 0, s);
}
int e1d(float* a, const float* b, const float* c, double cb, int lo, int hi, void* s) {
  return fdtd_1d_e_f32(a, b, c, cb, lo, hi, s);
}
int e1d(double* a, const double* b, const double* c, double cb, int lo, int hi, void* s) {
  return fdtd_1d_e_f64(a, b, c, cb, lo, hi, s);
}
int h1d(float* a, const float* b, const float* c, double db, int lo, int hi, void* s) {
  return fdtd_1d_h_f32(a, b, c, db, lo, hi, s);
}
int h1d(double* a, const double* b, const double* c, double db, int lo, int hi, void* s) {
  return fdtd_1d_h_f64(a, b, c, db, lo, hi, s);
}

// CPML (3D, fp32 float4 kernels): profiles, psi slabs and the per-kind term
// tables of yee3d_cpml.hip -- the same slabs and profiles as
// fdtd3d_amd/models/cpml.py (polynomial grading m = 4, R = 1e-8, kappa and
// alpha from --cpml-kappa-max / --cpml-alpha-max, each component's own
// staggered position).
// ---- boxes (lo[3], hi[3]) for the hybrid passes
struct IBox {
  int lo[3], hi[3];
  bool empty() const { return hi[0] <= lo[0] || hi[1] <= lo[1] || hi[2] <= lo[2]; }
  long long volume() const { return empty() ? 0 : (long long)(hi[0] - lo[0]) * (hi[1] - lo[1]) * (hi[2] - lo[2]); }
};

IBox box_and(const IBox& a, const IBox& b) {
  IBox r;
  for (int d = 0; d < 3; ++d) {
    r.lo[d] = std::max(a.lo[d], b.lo[d]);
    r.hi[d] = std::min(a.hi[d], b.hi[d]);
  }
  return r;
}

// a minus b as up to six disjoint slabs (x first, then y, then z)
std::vector<IBox> box_minus(const IBox& a, const IBox& b) {
  std::vector<IBox> out;
  const IBox c = box_and(a, b);
  if (c.empty()) {
    out.push_back(a);
    return out;
  }
  IBox rest = a;
  for (int d = 0; d < 3; ++d) {
    if (rest.lo[d] < c.lo[d]) {
      IBox s = rest;
      s.hi[d] = c.lo[d];
      out.push_back(s);
    }
    if (c.hi[d] < rest.hi[d]) {
      IBox s = rest;
      s.lo[d] = c.hi[d];
      out.push_back(s);
    }
    rest.lo[d] = c.lo[d];
    rest.hi[d] = c.hi[d];
  }
  return out;
}

struct NativeCpml {
  std::vector<Dev<float>*> keep;       // psi slabs and profile arrays
  std::vector<const void*> P[2];       // per kind (E, H): 9 x 5 pointers
  std::vector<int> I[2];               // per kind: 9 x 4 ints
  ~NativeCpml() {
    for (auto* d : keep) delete d;
  }
  float* upload(const std::vector<float>& h) {
    auto* d = new Dev<float>();
    d->alloc(h.size());
    HIP_OK(hipMemcpy(d->p, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
    keep.push_back(d);
    return d->p;
  }
  float* zeros(size_t n) {
    auto* d = new Dev<float>();
    d->alloc(n);
    keep.push_back(d);
    return d->p;
  }
};

void setup_cpml(NativeCpml& cp, const fdtd::Settings& s, const fdtd::Int3& N, const std::vector<int>& active,
                double dt, double dx) {
  // staggered offset of each component inside its cell (layout/yee.py MIN_COORD_FP)
  static const double mco[6][3] = {{1.0, 0.5, 0.5}, {0.5, 1.0, 0.5}, {0.5, 0.5, 1.0},
                                   {0.5, 1.0, 1.0}, {1.0, 0.5, 1.0}, {1.0, 1.0, 0.5}};
  const int Ps[3] = {s.pmlSizeX, s.pmlSizeY, s.pmlSizeZ};
  const double eta = std::sqrt(kMu0 / kEps0);
  const double kmax = s.cpmlKappaMax, amax = s.cpmlAlphaMax;
  for (int kind = 0; kind < 2; ++kind) {
    cp.P[kind].assign(45, nullptr);
    cp.I[kind].assign(36, 0);
    for (int cc = 0; cc < 3; ++cc) {
      const int c = 3 * kind + cc;
      fdtd::Int3 glo, ghi;
      fdtd::global_range(c, N, active, glo, ghi);
      for (int a = 0; a < 3; ++a) {
        // a component's two curl terms differentiate along the other two axes
        const int P = Ps[a];
        if (a == cc || P <= 0 || std::find(active.begin(), active.end(), a) == active.end()) continue;
        const int n = N[a];
        const double m = mco[c][a];
        const double sig_max = -(4 + 1) * std::log(1e-8) / (2 * eta * P * dx);
        std::vector<float> b(n, 1.f), cv(n, 0.f), kk(n, 0.f);
        const void* psi[2] = {nullptr, nullptr};
        int rng[2][2] = {{0, 0}, {0, 0}};
        for (int side = 0; side < 2; ++side) {
          int lo = glo[a], hi = ghi[a];
          if (side == 0)
            hi = std::min(hi, (int)std::ceil(P - m));
          else
            lo = std::max(lo, (int)std::floor(N[a] - P - m) + 1);
          bool empty = hi <= lo;
          for (int d = 0; d < 3; ++d) empty = empty || ghi[d] <= glo[d];
          if (empty) continue;
          if (a == 2 && N[2] % 4 == 0) {  // z slabs padded to whole float4 groups (c = 0 there)
            lo &= ~3;
            hi = std::min(N[2], (hi + 3) & ~3);
          }
          for (int v = lo; v < hi; ++v) {
            const double idx = v + m;
            double depth = side == 0 ? (P - idx) / P : (idx - (N[a] - P)) / P;
            depth = std::min(1.0, std::max(0.0, depth));
            const double d4 = depth * depth * depth * depth;
            const double sig = sig_max * d4, kap = 1.0 + (kmax - 1.0) * d4, alp = amax * (1.0 - depth);
            const double bc = std::exp(-(sig / kap + alp) * dt / kEps0);
            const double den = sig * kap + kap * kap * alp;
            b[v] = (float)bc;
            cv[v] = (float)(den > 0 ? sig / den * (bc - 1.0) : 0.0);
            kk[v] = (float)(1.0 / kap - 1.0);
          }
          // psi storage: the slab's range along a x the full extents of the other two
          size_t vol = (size_t)(hi - lo);
          for (int d = 0; d < 3; ++d)
            if (d != a) vol *= (size_t)N[d];
          psi[side] = cp.zeros(vol);
          rng[side][0] = lo;
          rng[side][1] = hi;
        }
        const int t = 3 * cc + a;
        cp.P[kind][5 * t] = psi[0];
        cp.P[kind][5 * t + 1] = psi[1];
        cp.P[kind][5 * t + 2] = cp.upload(b);
        cp.P[kind][5 * t + 3] = cp.upload(cv);
        cp.P[kind][5 * t + 4] = cp.upload(kk);
        cp.I[kind][4 * t] = rng[0][0];
        cp.I[kind][4 * t + 1] = rng[0][1];
        cp.I[kind][4 * t + 2] = rng[1][0];
        cp.I[kind][4 * t + 3] = rng[1][1];
      }
    }
  }
}

// ------------------------------------------------------------------ TF/SF
// Plane-wave injection through a total-field / scattered-field box, 3D: the
// 1D incident line (k_inc_e / k_inc_h) and per-component correction tables
// applied after each half step (k_tfsf_apply) -- the tables of
// fdtd3d_amd/models/tfsf.py build_tfsf_tables, built here on the host.

// numerical phase velocity of a plane wave on the Yee grid (Taflove;
// reference Approximation.cpp:212-269, layout/approximation.py)
double phase_velocity_3d(double delta, double wl, double courant, double nl, double theta, double phi) {
  const double half = kPi / 2;
  if (theta == half && (phi == 0.0 || phi == half || phi == kPi || phi == 3 * half))
    return kC * kPi / (nl * std::asin(std::sin(kPi * courant / nl) / courant));
  if (theta == half && (phi == kPi / 4 || phi == 3 * kPi / 4 || phi == 5 * kPi / 4 || phi == 7 * kPi / 4)) {
    const double s2 = std::sqrt(2.0);
    return kC * kPi / (nl * s2 * std::asin(std::sin(kPi * courant / nl) / (courant * s2)));
  }
  const double acc = 1e-7;  // Approximation.cpp:7
  double k = 2 * kPi, kp = k + acc;
  const double nd = delta / wl;
  const double A = nd * std::sin(theta) * std::cos(phi) / 2, B = nd * std::sin(theta) * std::sin(phi) / 2;
  const double C = nd * std::cos(theta) / 2;
  const double D = std::pow(std::sin(kPi * courant / nl), 2) / (courant * courant);
  for (int it = 0; (kp - k) * (kp - k) >= acc && it < 1000; ++it) {
    kp = k;
    const double f = std::pow(std::sin(A * k), 2) + std::pow(std::sin(B * k), 2) + std::pow(std::sin(C * k), 2) - D;
    const double df = A * std::sin(2 * A * k) + B * std::sin(2 * B * k) + C * std::sin(2 * C * k);
    k -= f / df;
  }
  return kC * 2 * kPi / k;
}

// (component, direction) -> per-axis open interval (ref lo, offset, ref hi,
// offset), ref 0 = the box's left border L, 1 = its right border R; directions
// L R D U B F (x low / high, y low / high, z low / high) -- models/tfsf.py
struct TfsfPred {
  int comp, dir;
  struct {
    int ra;
    double oa;
    int rb;
    double ob;
  } iv[3];
};
const TfsfPred kTfsfPred[24] = {
    {0, 2, {{0, -0.5, 1, 0.5}, {0, -1.0, 0, 0.0}, {0, 0.0, 1, 0.0}}},
    {0, 3, {{0, -0.5, 1, 0.5}, {1, 0.0, 1, 1.0}, {0, 0.0, 1, 0.0}}},
    {0, 4, {{0, -0.5, 1, 0.5}, {0, 0.0, 1, 0.0}, {0, -1.0, 0, 0.0}}},
    {0, 5, {{0, -0.5, 1, 0.5}, {0, 0.0, 1, 0.0}, {1, 0.0, 1, 1.0}}},
    {1, 0, {{0, -1.0, 0, 0.0}, {0, -0.5, 1, 0.5}, {0, 0.0, 1, 0.0}}},
    {1, 1, {{1, 0.0, 1, 1.0}, {0, -0.5, 1, 0.5}, {0, 0.0, 1, 0.0}}},
    {1, 4, {{0, 0.0, 1, 0.0}, {0, -0.5, 1, 0.5}, {0, -1.0, 0, 0.0}}},
    {1, 5, {{0, 0.0, 1, 0.0}, {0, -0.5, 1, 0.5}, {1, 0.0, 1, 1.0}}},
    {2, 0, {{0, -1.0, 0, 0.0}, {0, 0.0, 1, 0.0}, {0, -0.5, 1, 0.5}}},
    {2, 1, {{1, 0.0, 1, 1.0}, {0, 0.0, 1, 0.0}, {0, -0.5, 1, 0.5}}},
    {2, 2, {{0, 0.0, 1, 0.0}, {0, -1.0, 0, 0.0}, {0, -0.5, 1, 0.5}}},
    {2, 3, {{0, 0.0, 1, 0.0}, {1, 0.0, 1, 1.0}, {0, -0.5, 1, 0.5}}},
    {3, 2, {{0, 0.0, 1, 0.0}, {0, -0.5, 0, 0.5}, {0, -0.5, 1, 0.5}}},
    {3, 3, {{0, 0.0, 1, 0.0}, {1, -0.5, 1, 0.5}, {0, -0.5, 1, 0.5}}},
    {3, 4, {{0, 0.0, 1, 0.0}, {0, -0.5, 1, 0.5}, {0, -0.5, 0, 0.5}}},
    {3, 5, {{0, 0.0, 1, 0.0}, {0, -0.5, 1, 0.5}, {1, -0.5, 1, 0.5}}},
    {4, 0, {{0, -0.5, 0, 0.5}, {0, 0.0, 1, 0.0}, {0, -0.5, 1, 0.5}}},
    {4, 1, {{1, -0.5, 1, 0.5}, {0, 0.0, 1, 0.0}, {0, -0.5, 1, 0.5}}},
    {4, 4, {{0, -0.5, 1, 0.5}, {0, 0.0, 1, 0.0}, {0, -0.5, 0, 0.5}}},
    {4, 5, {{0, -0.5, 1, 0.5}, {0, 0.0, 1, 0.0}, {1, -0.5, 1, 0.5}}},
    {5, 0, {{0, -0.5, 0, 0.5}, {0, -0.5, 1, 0.5}, {0, 0.0, 1, 0.0}}},
    {5, 1, {{1, -0.5, 1, 0.5}, {0, -0.5, 1, 0.5}, {0, 0.0, 1, 0.0}}},
    {5, 2, {{0, -0.5, 1, 0.5}, {0, -0.5, 0, 0.5}, {0, 0.0, 1, 0.0}}},
    {5, 3, {{0, -0.5, 1, 0.5}, {1, -0.5, 1, 0.5}, {0, 0.0, 1, 0.0}}},
};
// curl terms (source component, derivative axis, sign) of each component (layout/yee.py CURL_TERMS)
const int kCurl[6][2][3] = {{{5, 1, +1}, {4, 2, -1}}, {{3, 2, +1}, {5, 0, -1}}, {{4, 0, +1}, {3, 1, -1}},
                            {{1, 2, +1}, {2, 1, -1}}, {{2, 0, +1}, {0, 2, -1}}, {{0, 1, +1}, {1, 0, -1}}};
// staggered offset of each component inside its cell (layout/yee.py MIN_COORD_FP)
const double kMinFP[6][3] = {{1.0, 0.5, 0.5}, {0.5, 1.0, 0.5}, {0.5, 0.5, 1.0},
                             {0.5, 1.0, 1.0}, {1.0, 0.5, 1.0}, {1.0, 1.0, 0.5}};

template <typename T>
struct TfsfLayer {
  Dev<long long> off, i0;
  Dev<T> w0, w1, coef;
  int n = 0;
};

template <typename T>
struct NativeTfsf {
  std::vector<TfsfLayer<T>*> tab[6];
  Dev<T> einc, hinc;
  int nline = 0;
  double ce = 0, ch = 0;
  ~NativeTfsf() {
    for (auto& v : tab)
      for (auto* l : v) delete l;
  }
};

// incident-wave projection onto a component (YeeGridLayout.cpp:811-845)
double inc_projection(int c, double t, double p, double q) {
  switch (c) {
    case 0: return std::cos(q) * std::sin(p) - std::sin(q) * std::cos(t) * std::cos(p);
    case 1: return -std::cos(q) * std::cos(p) - std::sin(q) * std::cos(t) * std::sin(p);
    case 2: return std::sin(q) * std::sin(t);
    case 3: return std::sin(q) * std::sin(p) + std::cos(q) * std::cos(t) * std::cos(p);
    case 4: return -std::sin(q) * std::cos(p) + std::cos(q) * std::cos(t) * std::sin(p);
    default: return -(std::cos(q) * std::sin(t));
  }
}

template <typename T>
bool setup_tfsf(NativeTfsf<T>& tf, const fdtd::Settings& s, const fdtd::Int3& N, const int* boxes,
                const Dev<T>* Cc, double cb, double db, double dt, double dx, double freq) {
  const double th = s.incidentWaveAngle1 * (kPi / 180.0), ph = s.incidentWaveAngle2 * (kPi / 180.0);
  const double ps = s.incidentWaveAngle3 * (kPi / 180.0);
  if (!(th >= 0 && th <= kPi / 2 + 1e-12 && ph >= 0 && ph <= kPi / 2 + 1e-12)) {
    std::fprintf(stderr, "fdtd3d (native): TF/SF incident angles must lie in [0, 90] degrees\n");
    return false;
  }
  const double wl = kC / freq, nl = wl / dx, courant = s.courantNum;
  const double rel = phase_velocity_3d(dx, wl, courant, nl, kPi / 2, 0.0) /
                     phase_velocity_3d(dx, wl, courant, nl, th, ph);
  tf.ce = dt / (rel * kEps0 * dx);
  tf.ch = dt / (rel * kMu0 * dx);
  tf.nline = 100 * (N[0] + N[1] + N[2]);
  tf.einc.alloc(tf.nline);
  tf.hinc.alloc(tf.nline);
  const double L[3] = {(double)s.tfsfSizeX, (double)s.tfsfSizeY, (double)s.tfsfSizeZ};
  const double R[3] = {N[0] - L[0], N[1] - L[1], N[2] - L[2]};
  const double dir[3] = {std::sin(th) * std::cos(ph), std::sin(th) * std::sin(ph), std::cos(th)};
  const double zero[3] = {L[0] - 2.5 * std::sin(th) * std::cos(ph), L[1] - 2.5 * std::sin(th) * std::sin(ph),
                          L[2] - 2.5 * std::cos(th)};
  const int dir_axis[6] = {0, 0, 1, 1, 2, 2};
  const bool dir_low[6] = {true, false, true, false, true, false};
  std::vector<T> hc((size_t)N[0] * N[1] * N[2]);
  for (int c = 0; c < 6; ++c) {
    const int* bx = boxes + 6 * c;
    if (bx[3] <= bx[0] || bx[4] <= bx[1] || bx[5] <= bx[2]) continue;
    const bool kind_e = c < 3;
    const bool pc = Cc[c].p != nullptr;
    if (pc) HIP_OK(hipMemcpy(hc.data(), Cc[c].p, hc.size() * sizeof(T), hipMemcpyDeviceToHost));
    struct Ent {
      long long flat, i0;
      double w0, w1, cv;
      size_t seq;
    };
    std::vector<Ent> ents;
    for (int t = 0; t < 2; ++t) {
      const int src = kCurl[c][t][0], axis = kCurl[c][t][1], sign = kCurl[c][t][2];
      const double proj = inc_projection(src, th, ph, ps);
      for (int d = 0; d < 6; ++d) {
        if (dir_axis[d] != axis) continue;
        const TfsfPred* pr = nullptr;
        for (const auto& q : kTfsfPred)
          if (q.comp == c && q.dir == d) pr = &q;
        if (!pr) continue;
        std::vector<int> sel[3];
        for (int a = 0; a < 3; ++a) {
          const double lo = (pr->iv[a].ra ? R[a] : L[a]) + pr->iv[a].oa;
          const double hi = (pr->iv[a].rb ? R[a] : L[a]) + pr->iv[a].ob;
          for (int v = bx[a]; v < bx[3 + a]; ++v) {
            const double g = v + kMinFP[c][a];
            if (g > lo && g < hi) sel[a].push_back(v);
          }
        }
        const int nb = kind_e ? (dir_low[d] ? 0 : -1) : (dir_low[d] ? 0 : 1);
        const int tsign = dir_low[d] ? -sign : sign;
        for (int i : sel[0])
          for (int j : sel[1])
            for (int k : sel[2]) {
              int ni[3] = {i, j, k};
              ni[axis] += nb;
              double dd = 0.0;
              for (int a = 0; a < 3; ++a) dd += (ni[a] + kMinFP[src][a] - zero[a]) * dir[a];
              dd -= kind_e ? 0.5 : 0.0;
              const long long i0 = (long long)std::floor(dd);
              if (i0 < 0 || i0 + 1 >= tf.nline) {
                std::fprintf(stderr, "fdtd3d (native): TF/SF box does not fit the incident line\n");
                return false;
              }
              const long long flat = ((long long)i * N[1] + j) * N[2] + k;
              const double cf = pc ? (double)hc[flat] : (kind_e ? cb : db);
              const double w1 = dd - (double)i0;
              ents.push_back({flat, i0, 1.0 - w1, w1, cf * tsign * proj, ents.size()});
            }
      }
    }
    if (ents.empty()) continue;
    // layers of unique targets (k_tfsf_apply has no atomics): stable order, the
    // r-th entry of a target goes to layer r
    std::stable_sort(ents.begin(), ents.end(), [](const Ent& a, const Ent& b) { return a.flat < b.flat; });
    std::vector<int> rank(ents.size(), 0);
    int maxr = 0;
    for (size_t q = 1; q < ents.size(); ++q)
      if (ents[q].flat == ents[q - 1].flat) maxr = std::max(maxr, rank[q] = rank[q - 1] + 1);
    for (int r = 0; r <= maxr; ++r) {
      std::vector<long long> off, i0;
      std::vector<T> w0, w1, cv;
      for (size_t q = 0; q < ents.size(); ++q)
        if (rank[q] == r) {
          off.push_back(ents[q].flat);
          i0.push_back(ents[q].i0);
          w0.push_back((T)ents[q].w0);
          w1.push_back((T)ents[q].w1);
          cv.push_back((T)ents[q].cv);
        }
      auto* l = new TfsfLayer<T>();
      l->n = (int)off.size();
      l->off.alloc(off.size());
      l->i0.alloc(i0.size());
      l->w0.alloc(w0.size());
      l->w1.alloc(w1.size());
      l->coef.alloc(cv.size());
      HIP_OK(hipMemcpy(l->off.p, off.data(), off.size() * sizeof(long long), hipMemcpyHostToDevice));
      HIP_OK(hipMemcpy(l->i0.p, i0.data(), i0.size() * sizeof(long long), hipMemcpyHostToDevice));
      HIP_OK(hipMemcpy(l->w0.p, w0.data(), w0.size() * sizeof(T), hipMemcpyHostToDevice));
      HIP_OK(hipMemcpy(l->w1.p, w1.data(), w1.size() * sizeof(T), hipMemcpyHostToDevice));
      HIP_OK(hipMemcpy(l->coef.p, cv.data(), cv.size() * sizeof(T), hipMemcpyHostToDevice));
      tf.tab[c].push_back(l);
    }
  }
  return true;
}

int inc_e(float* e, const float* h, int n, double c, double v, void* s) { return fdtd_inc_e_f32(e, h, n, c, v, s); }
int inc_e(double* e, const double* h, int n, double c, double v, void* s) { return fdtd_inc_e_f64(e, h, n, c, v, s); }
int inc_h(const float* e, float* h, int n, double c, void* s) { return fdtd_inc_h_f32(e, h, n, c, s); }
int inc_h(const double* e, double* h, int n, double c, void* s) { return fdtd_inc_h_f64(e, h, n, c, s); }
int tfsf_apply(float* t, const TfsfLayer<float>& l, const float* inc, const int* box, void* s) {
  return fdtd_tfsf_apply_f32(t, l.off.p, l.i0.p, l.w0.p, l.w1.p, l.coef.p, nullptr, l.n, inc, box, s);
}
int tfsf_apply(double* t, const TfsfLayer<double>& l, const double* inc, const int* box, void* s) {
  return fdtd_tfsf_apply_f64(t, l.off.p, l.i0.p, l.w0.p, l.w1.p, l.coef.p, nullptr, l.n, inc, box, s);
}

template <typename T>
int run(const fdtd::Settings& s) {
  const int dim = s.dimension;
  std::string scheme = dim == 3 ? "3d" : (dim == 2 ? s.mode2D : "1d");
  fdtd::Int3 N = {s.sizeX, dim >= 2 ? s.sizeY : 1, dim == 3 ? s.sizeZ : 1};
  std::vector<int> active = dim == 3 ? std::vector<int>{0, 1, 2} : (dim == 2 ? std::vector<int>{0, 1} : std::vector<int>{0});
  const size_t cells = (size_t)N[0] * N[1] * N[2];
  const double dx = s.gridStep, courant = s.courantNum;
  const double dt = dx * courant / kC;
  const double freq = kC / s.sourceWaveLength;
  // eps = 1 everywhere (a Drude sphere's eps_inf is 1 too: layout/materials.py Scene.eps)
  const bool vacuum = s.scene == "vacuum" || s.scene == "drude-sphere" || (s.scene == "reference" && dim != 3);
  const bool v4 = sizeof(T) == 4 && N[2] % 4 == 0 && dim == 3;
  // fused / blocked / resident kernels unless --split-kernels (3D fused E+H
  // and blocked passes, 2D blocked passes, 1D one-launch resident run)
  // CPML runs step through the float4 split kernels with the psi terms folded
  // in; TF/SF runs apply their corrections between the split half steps
  const bool upml = (s.doUsePML && s.pmlType == "upml") || s.doUseMetamaterials;  // the D/B chain
  const bool cpml = s.doUsePML && !upml;
  const bool tfsf = s.doUseTFSF;
  const bool ntff = s.doUseNTFF && dim == 3;
  const bool use_fused = !s.doUseSplitKernels && !cpml && !tfsf && !upml;
  hipStream_t st;
  HIP_OK(hipStreamCreate(&st));

  // components present: 0..2 E, 3..5 H
  bool present[6];
  for (int c = 0; c < 6; ++c) present[c] = dim == 3;
  if (scheme == "tmz") present[2] = present[3] = present[4] = true;
  if (scheme == "tez") present[0] = present[1] = present[5] = true;
  if (scheme == "1d") present[2] = present[4] = true;
  Dev<T> F[6], G[6], C[6];
  Dev<float> CE4;  // fp32 3D per-cell: sparse E coefficients of the blocked kernel
  int ebox[6] = {0, 0, 0, 0, 0, 0};
  for (int c = 0; c < 6; ++c)
    if (present[c]) {
      F[c].alloc(cells);
      if (use_fused) G[c].alloc(cells);
    }
  double cb = dt / (kEps0 * dx), db = dt / (kMu0 * dx);
  const bool percell = !vacuum;
  if (percell) {
    // per-component averaged eps on the eps layout (2-point E averaging,
    // YeeGridLayout.h:1007-1263); mu = 1 -> constant H arrays
    const double ctr[3] = {s.sphereCenterX, s.sphereCenterY, s.sphereCenterZ};
    auto eps_at = [&](int i, int j, int k) {
      return sphere_eps(i + 0.5, j + 0.5, dim == 3 ? k + 0.5 : ctr[2], ctr, s.sphereRadius, s.sphereEps);
    };
    std::vector<T> host(cells);
    for (int c = 0; c < 6; ++c) {
      if (!present[c]) continue;
      for (int i = 0; i < N[0]; ++i)
        for (int j = 0; j < N[1]; ++j)
          for (int k = 0; k < N[2]; ++k) {
            double v;
            if (c < 3) {
              const int di = c == 0, dj = c == 1 && dim >= 2, dk = c == 2 && dim == 3;
              v = cb * 2.0 / (eps_at(i, j, k) + eps_at(i + di, j + dj, k + dk));
            } else {
              v = db;
            }
            host[((size_t)i * N[1] + j) * N[2] + k] = (T)v;
          }
      C[c].alloc(cells);
      HIP_OK(hipMemcpy(C[c].p, host.data(), cells * sizeof(T), hipMemcpyHostToDevice));
    }
    if (sizeof(T) == 4 && dim == 3) {
      // sparse form for the blocked kernel: the E coefficients of the cells
      // around the sphere (its bounding box + 2 cells; every other cell has
      // eps = 1 on both averaging points, i.e. exactly cb) as one float4 per
      // cell; mu = 1, so H stays on the scalar db
      for (int a = 0; a < 3; ++a) {
        ebox[a] = std::max(0, (int)std::floor(ctr[a] - s.sphereRadius) - 2);
        ebox[3 + a] = std::min(N[a], (int)std::ceil(ctr[a] + s.sphereRadius) + 3);
      }
      const size_t bn = (size_t)std::max(0, ebox[3] - ebox[0]) * std::max(0, ebox[4] - ebox[1]) *
                        std::max(0, ebox[5] - ebox[2]);
      if (bn > 0) {
        std::vector<float> h4(4 * bn, 0.f);
        size_t q = 0;
        for (int i = ebox[0]; i < ebox[3]; ++i)
          for (int j = ebox[1]; j < ebox[4]; ++j)
            for (int k = ebox[2]; k < ebox[5]; ++k, ++q)
              for (int c = 0; c < 3; ++c) {
                const int di = c == 0, dj = c == 1, dk = c == 2;
                h4[4 * q + c] = (float)(cb * 2.0 / (eps_at(i, j, k) + eps_at(i + di, j + dj, k + dk)));
              }
        CE4.alloc(4 * bn);
        HIP_OK(hipMemcpy(CE4.p, h4.data(), 4 * bn * sizeof(float), hipMemcpyHostToDevice));
      }
    }
  }
  int boxes[36];
  for (int c = 0; c < 6; ++c) {
    fdtd::Int3 lo, hi;
    fdtd::global_range(c, N, active, lo, hi);
    for (int a = 0; a < 3; ++a) {
      boxes[6 * c + a] = lo[a];
      boxes[6 * c + 3 + a] = hi[a];
    }
  }
  // point source (reference Scheme3D.cpp:2011-2022, SchemeTMz.cpp:1345)
  int src_comp = 2;
  fdtd::Int3 sp = {N[0] / 2, N[1] / 2, N[2] / 2};
  if (scheme == "tmz") sp = {N[0] > 140 ? 70 : N[0] / 2, N[1] / 2, 0};
  if (scheme == "tez") src_comp = 5;
  if (scheme == "1d") sp = {N[0] / 2, 0, 0};
  const long long src_off = ((long long)sp[0] * N[1] + sp[1]) * N[2] + sp[2];
  auto src_val = [&](int t) {
    if (s.sourceType == "gaussian") return std::exp(-std::pow((t - s.gaussianDelay) / s.gaussianWidth, 2));
    return std::sin(dt * t * 2 * kPi * freq);
  };
  NativeCpml cpt;
  if (cpml) setup_cpml(cpt, s, N, active, dt, dx);
  native_phys::Upml<T> upt;
  if (upml) {
    native_phys::UpmlScene sc;
    sc.pml[0] = s.pmlSizeX;
    sc.pml[1] = s.pmlSizeY;
    sc.pml[2] = s.pmlSizeZ;
    sc.use_pml = s.doUsePML;
    sc.metamaterials = s.doUseMetamaterials;
    sc.lorentz = s.dispersion == "lorentz";
    sc.lorentz_ratio = s.lorentzOmega0Ratio;
    sc.freq = freq;
    sc.sphere_eps = s.scene == "sphere";
    sc.drude_sphere = s.scene == "drude-sphere";
    sc.ctr[0] = s.sphereCenterX;
    sc.ctr[1] = s.sphereCenterY;
    sc.ctr[2] = s.sphereCenterZ;
    sc.radius = s.sphereRadius;
    sc.eps_in = s.sphereEps;
    native_phys::setup_upml<T>(upt, N, sc, dt, dx);
  }
  T* Fp[6];
  auto fptrs = [&]() {
    for (int c = 0; c < 6; ++c) Fp[c] = F[c].p;
  };
  int (*chain_fn)(const void* const*, const double*, const int*, int, int, int, int, void*) =
      sizeof(T) == 4 ? fdtd_chain3d_f32 : fdtd_chain3d_f64;
  NativeTfsf<T> tft;
  if (tfsf && !setup_tfsf(tft, s, N, boxes, C, percell ? 1.0 : cb, percell ? 1.0 : db, dt, dx, freq)) return 1;
  const bool point_src = !tfsf || s.doUsePointSource;
  const int whole[6] = {0, 0, 0, N[0], N[1], N[2]};
  auto tfsf_kind = [&](int kind) {
    for (int c = 3 * kind; c < 3 * kind + 3; ++c)
      for (auto* l : tft.tab[c]) K_OK(tfsf_apply(F[c].p, *l, kind == 0 ? tft.hinc.p : tft.einc.p, whole, st));
  };

  // one time step (t) through the configured kernels
  auto step = [&](int t) {
    const double sv = src_val(t);
    if (scheme == "3d") {
      if (use_fused) {
        const T* ei[3] = {F[0].p, F[1].p, F[2].p};
        const T* hi[3] = {F[3].p, F[4].p, F[5].p};
        T* eo[3] = {G[0].p, G[1].p, G[2].p};
        T* ho[3] = {G[3].p, G[4].p, G[5].p};
        const T* cbs[3] = {C[0].p, C[1].p, C[2].p};
        const T* dbs[3] = {C[3].p, C[4].p, C[5].p};
        K_OK(fused(ei, hi, eo, ho, cbs, dbs, percell ? 1.0 : cb, percell ? 1.0 : db, N[0], N[1], N[2], boxes,
                   src_off, src_comp, sv, st, v4));
        for (int c = 0; c < 6; ++c) std::swap(F[c].p, G[c].p);
      } else {
        // split half steps: [incident line E] E update [TF/SF on E] [source]
        // [incident line H] H update [TF/SF on H] -- the order of scheme.step
        if (tfsf) K_OK(inc_e(tft.einc.p, tft.hinc.p, tft.nline, tft.ce, sv, st));
        if (upml) {
          fptrs();
          K_OK(native_phys::upml_kind<T>(upt, Fp, boxes, 0, N[1], N[2], st, chain_fn));
        } else if (cpml) {
          if constexpr (sizeof(T) == 4)
            K_OK(fdtd_update_e3d_cpml_v4_f32(F[0].p, F[1].p, F[2].p, F[3].p, F[4].p, F[5].p, C[0].p, C[1].p, C[2].p,
                                             percell ? 1.0 : cb, N[0], N[1], N[2], boxes, 0, cpt.P[0].data(),
                                             cpt.I[0].data(), st));
        } else {
          K_OK(e3d(F[0].p, F[1].p, F[2].p, F[3].p, F[4].p, F[5].p, C[0].p, C[1].p, C[2].p, percell ? 1.0 : cb,
                   N[0], N[1], N[2], boxes, 0, st, v4));
        }
        if (tfsf) tfsf_kind(0);
        if (point_src) K_OK(setv(F[src_comp].p, src_off, sv, st));
        if (tfsf) K_OK(inc_h(tft.einc.p, tft.hinc.p, tft.nline, tft.ch, st));
        if (upml) {
          fptrs();
          K_OK(native_phys::upml_kind<T>(upt, Fp, boxes, 1, N[1], N[2], st, chain_fn));
        } else if (cpml) {
          if constexpr (sizeof(T) == 4)
            K_OK(fdtd_update_h3d_cpml_v4_f32(F[3].p, F[4].p, F[5].p, F[0].p, F[1].p, F[2].p, C[3].p, C[4].p, C[5].p,
                                             percell ? 1.0 : db, N[0], N[1], N[2], boxes + 18, 0, cpt.P[1].data(),
                                             cpt.I[1].data(), st));
        } else {
          K_OK(h3d(F[3].p, F[4].p, F[5].p, F[0].p, F[1].p, F[2].p, C[3].p, C[4].p, C[5].p, percell ? 1.0 : db,
                   N[0], N[1], N[2], boxes + 18, 0, st, v4));
        }
        if (tfsf) tfsf_kind(1);
      }
    } else if (scheme == "tmz") {
      K_OK(tmz_e(F[2].p, F[3].p, F[4].p, C[2].p, percell ? 1.0 : cb, N[0], N[1], boxes + 12, st));
      K_OK(setv(F[2].p, src_off, sv, st));
      int hb[12];
      std::memcpy(hb, boxes + 18, 12 * sizeof(int));
      K_OK(tmz_h(F[3].p, F[4].p, F[2].p, C[3].p, C[4].p, percell ? 1.0 : db, N[0], N[1], hb, st));
    } else if (scheme == "tez") {
      K_OK(tez_e(F[0].p, F[1].p, F[5].p, C[0].p, C[1].p, percell ? 1.0 : cb, N[0], N[1], boxes, st));
      K_OK(setv(F[5].p, src_off, sv, st));  // hard source between the E and H updates
      K_OK(tez_h(F[5].p, F[0].p, F[1].p, C[5].p, percell ? 1.0 : db, N[0], N[1], boxes + 30, st));
    } else {
      K_OK(e1d(F[2].p, F[4].p, C[2].p, percell ? 1.0 : cb, boxes[12], boxes[15], st));
      K_OK(setv(F[2].p, src_off, sv, st));
      K_OK(h1d(F[4].p, F[2].p, C[4].p, percell ? 1.0 : db, boxes[24], boxes[27], st));
    }
  };
  // --time-block T: T steps per HBM pass through the blocked kernel
  // 0: automatic (5 steps per pass in fp32, 4 in fp64)
  const int T_req = s.timeBlock <= 0 ? (sizeof(T) == 4 ? 5 : 4) : s.timeBlock;
  const int T_max = sizeof(T) == 4 ? fdtd_tb_max_steps() : fdtd_tb64_max_steps();
  const int T_blk = (scheme == "3d" && use_fused && (v4 || sizeof(T) == 8)) ? std::max(1, std::min(T_max, T_req)) : 1;
  // 2D: yee2d_tb.hip passes (automatic 7 steps), rows of whole 16-byte lanes
  const int T2_max = sizeof(T) == 4 ? fdtd_tb2d_max_steps() : fdtd_tb2d64_max_steps();
  const int T2_blk = (dim == 2 && use_fused && N[1] % (16 / (int)sizeof(T)) == 0)
                         ? std::max(1, std::min(T2_max, s.timeBlock <= 0 ? 7 : s.timeBlock))
                         : 1;
  // 1D: the whole run in one launch of the register-resident kernel
  const bool res1 = dim == 1 && use_fused && N[0] <= fdtd_res1d_max_cells((int)sizeof(T));
  // Hybrid passes for 3D fp32 CPML runs (+ TF/SF, point source) -- the plan
  // the Python driver picks automatically (models/blocking.py _hybrid_plan):
  // every T steps the blocked kernel advances the core (cells at least T + 2
  // beyond every CPML slab and TF/SF target) by T steps F -> G; the shell is
  // stepped in place in F with a band T - s deep into the core at step s
  // (stale core values corrupt one band cell per step, so the shell itself
  // stays exact), copied into G, and the buffers swap.
  const int T_h_req = s.hybridBlock == 0 ? 5 : s.hybridBlock;
  IBox hcore = {{0, 0, 0}, {0, 0, 0}};
  std::vector<IBox> hshell[8], hcopy;
  int T_h = 1;
  if (scheme == "3d" && sizeof(T) == 4 && v4 && cpml && !percell && T_h_req > 1 && T_h_req <= fdtd_tb_max_steps()) {
    const int pml[3] = {s.pmlSizeX, s.pmlSizeY, s.pmlSizeZ};
    const int tfs[3] = {s.tfsfSizeX, s.tfsfSizeY, s.tfsfSizeZ};
    IBox K;
    for (int a = 0; a < 3; ++a) {
      const int edge = std::max(pml[a], tfsf ? tfs[a] + 1 : 0);
      K.lo[a] = edge + T_h_req + 2;
      K.hi[a] = N[a] - edge - T_h_req - 2;
    }
    if (!K.empty() && K.volume() >= (long long)cells / 4) {
      T_h = T_h_req;
      hcore = K;
      const IBox alloc = {{0, 0, 0}, {N[0], N[1], N[2]}};
      for (int q = 0; q < T_h; ++q) {
        IBox Kd = K;
        for (int a = 0; a < 3; ++a) {
          Kd.lo[a] += T_h - q;
          Kd.hi[a] -= T_h - q;
        }
        hshell[q] = box_minus(alloc, Kd);
      }
      hcopy = box_minus(alloc, K);
      for (int c = 0; c < 6; ++c)
        if (present[c] && !G[c].p) G[c].alloc(cells);
    }
  }
  auto window_boxes = [&](const IBox& w, int c0, int* out) {
    for (int c = c0; c < c0 + 3; ++c) {
      IBox b;
      for (int a = 0; a < 3; ++a) {
        b.lo[a] = boxes[6 * c + a];
        b.hi[a] = boxes[6 * c + 3 + a];
      }
      b = box_and(b, w);
      for (int a = 0; a < 3; ++a) {
        out[6 * (c - c0) + a] = b.empty() ? 0 : b.lo[a];
        out[6 * (c - c0) + 3 + a] = b.empty() ? 0 : b.hi[a];
      }
    }
  };
  auto hybrid_pass = [&](int t) {
    if constexpr (sizeof(T) == 4) {
      const T* ei[3] = {F[0].p, F[1].p, F[2].p};
      const T* hi[3] = {F[3].p, F[4].p, F[5].p};
      T* eo[3] = {G[0].p, G[1].p, G[2].p};
      T* ho[3] = {G[3].p, G[4].p, G[5].p};
      const T* none3[3] = {nullptr, nullptr, nullptr};
      bool in_core = true;
      for (int a = 0; a < 3; ++a) in_core = in_core && sp[a] >= hcore.lo[a] && sp[a] < hcore.hi[a];
      const int src[4] = {sp[0], sp[1], sp[2], point_src && in_core ? src_comp : -1};
      double vals[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int l = 0; l < T_h; ++l) vals[l] = src_val(t + l);
      const int ob[6] = {hcore.lo[0], hcore.lo[1], hcore.lo[2], hcore.hi[0], hcore.hi[1], hcore.hi[2]};
      K_OK(tb3d(ei, hi, eo, ho, none3, none3, cb, db, N[0], N[1], N[2], boxes, T_h, src, vals, st, nullptr, nullptr,
                ob));
      for (int q = 0; q < T_h; ++q) {
        const double sv = src_val(t + q);
        int wb[18];
        if (tfsf) K_OK(inc_e(tft.einc.p, tft.hinc.p, tft.nline, tft.ce, sv, st));
        for (const IBox& w : hshell[q]) {
          window_boxes(w, 0, wb);
          K_OK(fdtd_update_e3d_cpml_v4_f32(F[0].p, F[1].p, F[2].p, F[3].p, F[4].p, F[5].p, nullptr, nullptr, nullptr,
                                           cb, N[0], N[1], N[2], wb, 0, cpt.P[0].data(), cpt.I[0].data(), st));
        }
        if (tfsf) tfsf_kind(0);
        if (point_src) K_OK(setv(F[src_comp].p, src_off, sv, st));
        if (tfsf) K_OK(inc_h(tft.einc.p, tft.hinc.p, tft.nline, tft.ch, st));
        for (const IBox& w : hshell[q]) {
          window_boxes(w, 3, wb);
          K_OK(fdtd_update_h3d_cpml_v4_f32(F[3].p, F[4].p, F[5].p, F[0].p, F[1].p, F[2].p, nullptr, nullptr, nullptr,
                                           db, N[0], N[1], N[2], wb, 0, cpt.P[1].data(), cpt.I[1].data(), st));
        }
        if (tfsf) tfsf_kind(1);
      }
      float* src6[6] = {F[0].p, F[1].p, F[2].p, F[3].p, F[4].p, F[5].p};
      float* dst6[6] = {G[0].p, G[1].p, G[2].p, G[3].p, G[4].p, G[5].p};
      for (const IBox& b : hcopy) {
        const int bx[6] = {b.lo[0], b.lo[1], b.lo[2], b.hi[0], b.hi[1], b.hi[2]};
        K_OK(fdtd_box_xfer_f32(src6, dst6, 6, N[1], N[2], bx, st));
      }
      for (int c = 0; c < 6; ++c) std::swap(F[c].p, G[c].p);
    }
  };
  auto advance = [&](int t0, int n) {
    int t = t0;
    while (T_h > 1 && n >= T_h) {
      hybrid_pass(t);
      t += T_h;
      n -= T_h;
    }
    if (res1 && n > 0) {
      std::vector<T> hv(n);
      for (int l = 0; l < n; ++l) hv[l] = (T)src_val(t + l);
      Dev<T> dv;
      dv.alloc(n);
      HIP_OK(hipMemcpyAsync(dv.p, hv.data(), n * sizeof(T), hipMemcpyHostToDevice, st));
      const int b1[4] = {boxes[12], boxes[15], boxes[24], boxes[27]};
      K_OK(res1d(F[2].p, F[4].p, C[2].p, C[4].p, percell ? 1.0 : cb, percell ? 1.0 : db, N[0], b1, n, sp[0], dv.p,
                 st));
      HIP_OK(hipStreamSynchronize(st));  // the table is freed on return
      return;
    }
    while (n > 0) {
      if (T2_blk > 1) {
        // component order: TMz Ez Hx Hy, TEz Ex Ey Hz
        const int ord[2][3] = {{2, 3, 4}, {0, 1, 5}};
        const int m = scheme == "tmz" ? 0 : 1;
        const int* o = ord[m];
        const T* ei[2] = {F[o[0]].p, m ? F[o[1]].p : nullptr};
        const T* hi[2] = {F[m ? o[2] : o[1]].p, m ? nullptr : F[o[2]].p};
        T* eo[2] = {G[o[0]].p, m ? G[o[1]].p : nullptr};
        T* ho[2] = {G[m ? o[2] : o[1]].p, m ? nullptr : G[o[2]].p};
        const T* cs[3] = {C[o[0]].p, C[o[1]].p, C[o[2]].p};
        int b2[18];
        for (int q = 0; q < 3; ++q) std::memcpy(b2 + 6 * q, boxes + 6 * o[q], 6 * sizeof(int));
        const int ob[6] = {0, 0, 0, N[0], N[1], 1};
        const int src[3] = {sp[0], sp[1], m ? 2 : 0};
        const int k = std::min(T2_blk, n);
        double vals[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int l = 0; l < k; ++l) vals[l] = src_val(t + l);
        K_OK(tb2d(m, ei, hi, eo, ho, cs, percell ? 1.0 : cb, percell ? 1.0 : db, N[0], N[1], b2, ob, k, src, vals,
                  st));
        for (int q = 0; q < 3; ++q) std::swap(F[o[q]].p, G[o[q]].p);
        t += k;
        n -= k;
        continue;
      }
      if (T_blk > 1 && n >= T_blk) {
        const T* ei[3] = {F[0].p, F[1].p, F[2].p};
        const T* hi[3] = {F[3].p, F[4].p, F[5].p};
        T* eo[3] = {G[0].p, G[1].p, G[2].p};
        T* ho[3] = {G[3].p, G[4].p, G[5].p};
        const T* cbs[3] = {C[0].p, C[1].p, C[2].p};
        const T* dbs[3] = {C[3].p, C[4].p, C[5].p};
        const int src[4] = {sp[0], sp[1], sp[2], src_comp};
        double vals[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int l = 0; l < T_blk; ++l) vals[l] = src_val(t + l);
        if (CE4.p)
          K_OK(tb3d(ei, hi, eo, ho, cbs, dbs, cb, db, N[0], N[1], N[2], boxes, T_blk, src, vals, st, CE4.p, ebox));
        else
          K_OK(tb3d(ei, hi, eo, ho, cbs, dbs, percell ? 1.0 : cb, percell ? 1.0 : db, N[0], N[1], N[2], boxes, T_blk,
                    src, vals, st));
        for (int c = 0; c < 6; ++c) std::swap(F[c].p, G[c].p);
        t += T_blk;
        n -= T_blk;
      } else {
        step(t);
        ++t;
        --n;
      }
    }
  };

  // NTFF diagram after every step t with (t - 1) % ntffStep == 0, for the
  // fields of step t - 1 (the Python driver's periodic hook, runner.py)
  const int nstep = std::max(1, s.ntffStep);
  const int nbox[3] = {s.ntffSizeX, s.ntffSizeY, s.ntffSizeZ};
  auto ntff_report = [&](int t) {
    HIP_OK(hipStreamSynchronize(st));
    fptrs();
    const std::vector<double> phis = native_phys::reference_angles();
    const std::vector<double> p =
        native_phys::ntff_power<T>(Fp, N, nbox, dx, s.sourceWaveLength, s.incidentWaveAngle1 * (kPi / 180.0), phis);
    for (size_t q = 0; q < phis.size(); ++q)
      std::printf("=== t=%u, inc angle=%f; angle %f === %.17g \n", (unsigned)t, s.incidentWaveAngle2 * (kPi / 180.0),
                  phis[q], p[q]);
  };
  auto run_steps = [&](int t0, int n) {
    if (!ntff) {
      advance(t0, n);
      return;
    }
    int t = t0;
    const int end = t0 + n;
    while (t < end) {
      const int nxt = std::min(end, t + 1 + ((1 - (t + 1)) % nstep + nstep) % nstep);
      advance(t, nxt - t);
      t = nxt;
      if ((t - 1) % nstep == 0) ntff_report(t - 1);
    }
  };

  const int steps = s.numTimeSteps;
  const int warm = std::max(0, std::min(s.warmupSteps, steps));
  run_steps(0, warm);  // untimed (they advance the simulation)
  HIP_OK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  HIP_OK(hipEventRecord(e0, st));
  run_steps(warm, steps - warm);
  HIP_OK(hipEventRecord(e1, st));
  HIP_OK(hipEventSynchronize(e1));
  HIP_OK(hipGetLastError());
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  const double sec = ms / 1e3;

  std::printf("Total time = %f seconds\n", sec);
  std::printf("Dimension: %d\n", dim);
  if (dim == 3)
    std::printf("Grid size: %dx%dx%d\n", N[0], N[1], N[2]);
  else if (dim == 2)
    std::printf("Grid size: %dx%d\n", N[0], N[1]);
  else
    std::printf("Grid size: %d\n", N[0]);
  const int timed = steps - warm;
  std::printf("Number of time steps: %d (%d timed after %d warm-up)\n\n", steps, timed, warm);
  std::printf("Value type: %s\n", Api<T>::name);
  std::printf("\n-------- Details --------\n");
  std::printf("Parallel grid: 0\n");
  if (T_h > 1)
    std::printf("Backend: native HIP, hybrid passes (blocked core, %d steps per pass; stepped CPML%s shell)\n", T_h,
                tfsf ? " + TF/SF" : "");
  else if (T_blk > 1 || T2_blk > 1)
    std::printf("Backend: native HIP, temporally blocked kernel (%d steps per pass)\n", std::max(T_blk, T2_blk));
  else if (res1)
    std::printf("Backend: native HIP, register-resident 1D kernel (one launch per run)\n");
  else if (cpml || tfsf || upml)
    std::printf("Backend: native HIP, split kernels%s%s%s\n", cpml ? " with the CPML terms folded in" : "",
                upml ? " with the UPML / dispersive chain" : "", tfsf ? " + TF/SF corrections" : "");
  else
    std::printf("Backend: native HIP, %s kernels%s\n", use_fused ? "fused E+H" : "split", v4 ? " (float4)" : "");
  std::printf("Throughput: %.1f Mcells/s\n", cells * (double)timed / sec / 1e6);
  if (s.doPrintJson)
    std::printf("{\"seconds\": %.6f, \"steps\": %d, \"mcells_per_s\": %.3f}\n", sec, timed,
                cells * (double)timed / sec / 1e6);

  if (s.doSaveRes) {
    const char* names[6] = {"Ex", "Ey", "Ez", "Hx", "Hy", "Hz"};
    std::vector<T> host(cells);
    for (int c = 0; c < 6; ++c) {
      if (!present[c]) continue;
      HIP_OK(hipMemcpy(host.data(), F[c].p, cells * sizeof(T), hipMemcpyDeviceToHost));
      const std::string base = fdtd::grid_file_name(steps, 0, names[c], s.outputDir == "." ? "" : s.outputDir);
      if (s.saveAsDAT) fdtd::write_dat(base + ".dat", host.data(), cells * sizeof(T));
      if (s.saveAsBMP || !s.saveAsDAT) {
        // middle slice along z (3D) or the plane (2D) / line (1D)
        const int w = N[0], h = N[1];
        const int kz = dim == 3 ? N[2] / 2 : 0;
        std::vector<double> v((size_t)w * h);
        for (int i = 0; i < w; ++i)
          for (int j = 0; j < h; ++j) v[(size_t)i * h + j] = host[((size_t)i * N[1] + j) * N[2] + kz];
        const std::string name = dim == 3 ? base + std::to_string(kz) + "-Re.bmp" : base + "-Re.bmp";
        fdtd::write_bmp(name, v, w, h, s.dumperPalette);
      }
    }
  }
  HIP_OK(hipStreamDestroy(st));
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  fdtd::Settings s;
  int st = s.parse(argc, argv, true, 1);
  if (st == fdtd::SETTINGS_BREAK) {
    std::fputs(s.message.c_str(), stdout);
    return 0;
  }
  if (st != fdtd::SETTINGS_OK) {
    std::fputs(s.message.c_str(), stdout);
    return st;
  }
  if (s.validate() != fdtd::SETTINGS_OK) {
    std::fprintf(stdout, "ERROR: %s\n", s.message.c_str());
    return 1;
  }
  // CPML absorbing layers: 3D fp32 with whole float4 z rows (the folded float4 kernels)
  const bool cpml_ok = s.doUsePML && s.pmlType == "cpml" && !s.doUseMetamaterials && s.dimension == 3 &&
                       s.valueType == "f32" && s.sizeZ % 4 == 0;
  // UPML (D/B chain) and Drude / Lorentz spheres: 3D, any precision
  const bool upml_ok = s.doUsePML && (s.pmlType == "upml" || s.doUseMetamaterials) && s.dimension == 3;
  const bool meta_ok = !s.doUseMetamaterials || (s.dimension == 3 && s.scene == "drude-sphere");
  // TF/SF plane waves: 3D (any precision), with the CPML or the UPML; with the
  // UPML the corrections take the E form, exact where every sigma vanishes:
  // the TF/SF box must lie inside the absorbing layers' interior
  bool tfsf_ok = s.doUseTFSF && s.dimension == 3;
  if (tfsf_ok && s.doUsePML && (s.pmlType == "upml" || s.doUseMetamaterials))
    tfsf_ok = s.tfsfSizeX > s.pmlSizeX + 1 && s.tfsfSizeY > s.pmlSizeY + 1 && s.tfsfSizeZ > s.pmlSizeZ + 1;
  const bool ntff_ok = !s.doUseNTFF || s.dimension == 3;
  if ((s.doUsePML && !cpml_ok && !upml_ok) || (s.doUseTFSF && !tfsf_ok) || !meta_ok || !ntff_ok ||
      s.doUseAmplitudeMode || s.doUseComplexFieldValues || s.doUseParallelGrid || s.doUseDoubleMaterialPrecision ||
      !s.loadFromFile.empty()) {
    std::fprintf(stderr,
                 "fdtd3d (native): CPML outside 3D fp32 float4 rows, PML / TF/SF / NTFF outside 3D, TF/SF boxes "
                 "reaching the UPML, metamaterials outside the drude-sphere scene, amplitude mode, complex fields, "
                 "parallel grids and resume run through the Python driver: python -m fdtd3d_amd <same options>\n");
    return 2;
  }
  int ndev = 0;
  HIP_OK(hipGetDeviceCount(&ndev));
  if (ndev < 1) {
    std::fprintf(stderr, "no HIP device\n");
    return 1;
  }
  HIP_OK(hipSetDevice(0 % (s.numCudaGPUs > 0 ? s.numCudaGPUs : 1)));
  return s.valueType == "f32" ? run<float>(s) : run<double>(s);
}
