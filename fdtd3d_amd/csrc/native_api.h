// native_api.h -- the native driver's physical constants, status macros, device buffers and
// the typed (fp32 / fp64 overloaded) wrappers over libfdtd3d_hip's C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "capi.h"

// Part of the native driver: included by main.cpp only (one translation unit),
// hence the unnamed namespace.
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
  void reset() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  ~Dev() { reset(); }
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
         const int* = nullptr, const int* obox = nullptr) {
  const int whole[6] = {0, 0, 0, nx, ny, nz};
  return fdtd_tb3d_f64(ei, hi, eo, ho, cbs, dbs, cb, db, nx, ny, nz, bx, obox ? obox : whole, 0, T, src, vals, s);
}
// the Drude pass of a hybrid pass (fp32: tb3d_mr.h DrDev, fp64: yee3d_tb64.hip DrDev64)
int drude3d(const float* const* ei, const float* const* hi, float* const* eo, float* const* ho, double cb, double db,
            int nx, int ny, int nz, const int* bx, const int* ob, int T, const int* src, const double* vals,
            const int* bb, void* const* sin, void* const* sout, const float* lut, int nid, double cbd, void* s) {
  return fdtd_tb3d_drude_f32(ei, hi, eo, ho, cb, db, nx, ny, nz, bx, ob, 0, T, src, vals, bb, sin, sout, lut, nid,
                             cbd, s);
}
int drude3d(const double* const* ei, const double* const* hi, double* const* eo, double* const* ho, double cb,
            double db, int nx, int ny, int nz, const int* bx, const int* ob, int T, const int* src, const double* vals,
            const int* bb, void* const* sin, void* const* sout, const double* lut, int nid, double cbd, void* s) {
  return fdtd_tb3d_drude_f64(ei, hi, eo, ho, cb, db, nx, ny, nz, bx, ob, 0, T, src, vals, bb, sin, sout, lut, nid,
                             cbd, s);
}
// CPML half steps with the psi terms folded in (yee3d_cpml.hip, 4-cell z lanes)
int cpml_e3d(float* const* F, const float* const* C, double cb, int nx, int ny, int nz, const int* bx,
             const void* const* P, const int* I, void* s) {
  return fdtd_update_e3d_cpml_v4_f32(F[0], F[1], F[2], F[3], F[4], F[5], C[0], C[1], C[2], cb, nx, ny, nz, bx, 0, P,
                                     I, s);
}
int cpml_e3d(double* const* F, const double* const* C, double cb, int nx, int ny, int nz, const int* bx,
             const void* const* P, const int* I, void* s) {
  return fdtd_update_e3d_cpml_v4_f64(F[0], F[1], F[2], F[3], F[4], F[5], C[0], C[1], C[2], cb, nx, ny, nz, bx, 0, P,
                                     I, s);
}
int cpml_h3d(float* const* F, const float* const* C, double db, int nx, int ny, int nz, const int* bx,
             const void* const* P, const int* I, void* s) {
  return fdtd_update_h3d_cpml_v4_f32(F[3], F[4], F[5], F[0], F[1], F[2], C[3], C[4], C[5], db, nx, ny, nz, bx, 0, P,
                                     I, s);
}
int cpml_h3d(double* const* F, const double* const* C, double db, int nx, int ny, int nz, const int* bx,
             const void* const* P, const int* I, void* s) {
  return fdtd_update_h3d_cpml_v4_f64(F[3], F[4], F[5], F[0], F[1], F[2], C[3], C[4], C[5], db, nx, ny, nz, bx, 0, P,
                                     I, s);
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
int box_pack(float* const* f, float* buf, int n, int ny, int nz, const int* box, void* s) {
  return fdtd_box_pack_f32(f, buf, n, ny, nz, box, s);
}
int box_pack(double* const* f, double* buf, int n, int ny, int nz, const int* box, void* s) {
  return fdtd_box_pack_f64(f, buf, n, ny, nz, box, s);
}
int box_unpack(float* const* f, const float* buf, int n, int ny, int nz, const int* box, void* s) {
  return fdtd_box_unpack_f32(f, buf, n, ny, nz, box, s);
}
int box_unpack(double* const* f, const double* buf, int n, int ny, int nz, const int* box, void* s) {
  return fdtd_box_unpack_f64(f, buf, n, ny, nz, box, s);
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
int xfer(float* const* a, float* const* b, int n, int ny, int nz, const int* bx, void* s) {
  return fdtd_box_xfer_f32(a, b, n, ny, nz, bx, s);
}
int xfer(double* const* a, double* const* b, int n, int ny, int nz, const int* bx, void* s) {
  return fdtd_box_xfer_f64(a, b, n, ny, nz, bx, s);
}
int setvs(float* f, const long long* o, int n, double v, void* s) { return fdtd_set_values_f32(f, o, n, v, s); }
int setvs(double* f, const long long* o, int n, double v, void* s) { return fdtd_set_values_f64(f, o, n, v, s); }
int curl_gen(float* out, const float* inp, const float* const* srcs, const int* axes, const int* signs, int nt,
             int ke, const void* const* ca, const void* const* cbp, int ny, int nz, const int* box, void* s) {
  return fdtd_curl_general_f32(out, inp, srcs, axes, signs, nt, ke, 1.0, ca, 1.0, cbp, ny, nz, box, s);
}
int curl_gen(double* out, const double* inp, const double* const* srcs, const int* axes, const int* signs, int nt,
             int ke, const void* const* ca, const void* const* cbp, int ny, int nz, const int* box, void* s) {
  return fdtd_curl_general_f64(out, inp, srcs, axes, signs, nt, ke, 1.0, ca, 1.0, cbp, ny, nz, box, s);
}
int lincomb(float* out, int nt, const double* sc, const void* const* p, const float* const* xs, int ny, int nz,
            const int* box, void* s) {
  return fdtd_lincomb_f32(out, nt, sc, p, xs, ny, nz, box, s);
}
int lincomb(double* out, int nt, const double* sc, const void* const* p, const double* const* xs, int ny, int nz,
            const int* box, void* s) {
  return fdtd_lincomb_f64(out, nt, sc, p, xs, ny, nz, box, s);
}
int cpml_apply(float* t, const float* src, float* psi, int axis, int sign, int ke, const float* b, const float* c,
               const float* k, double cbs, const void* const* cbp, int ny, int nz, const int* box, const int* pb,
               void* s) {
  return fdtd_cpml_apply_f32(t, src, psi, axis, sign, ke, b, c, k, cbs, cbp, ny, nz, box, pb, s);
}
int cpml_apply(double* t, const double* src, double* psi, int axis, int sign, int ke, const double* b,
               const double* c, const double* k, double cbs, const void* const* cbp, int ny, int nz, const int* box,
               const int* pb, void* s) {
  return fdtd_cpml_apply_f64(t, src, psi, axis, sign, ke, b, c, k, cbs, cbp, ny, nz, box, pb, s);
}
int amp_many(const float* const* f, float* const* a, int n, int ny, int nz, const int* bx, long long xs, double acc,
             unsigned* cnt, void* s) {
  return fdtd_amplitude_many_f32((const void* const*)f, (void* const*)a, n, ny, nz, bx, xs, acc, cnt, s);
}
int amp_many(const double* const* f, double* const* a, int n, int ny, int nz, const int* bx, long long xs,
             double acc, unsigned* cnt, void* s) {
  return fdtd_amplitude_many_f64((const void* const*)f, (void* const*)a, n, ny, nz, bx, xs, acc, cnt, s);
}

}  // namespace
