// Native driver physics beyond the plain Yee update (csrc/main.cpp): the UPML
// in the reference's D/B form, Drude / Lorentz dispersive media and the
// near-to-far-field scattered power diagram -- host set-up of the same
// profiles, coefficient tables and surface sums as the Python driver
// (models/scheme.py _init_upml, layout/materials.py, models/ntff.py), on top of
// libfdtd3d_hip's chain kernel (chain_kernels.hip) through its C ABI.
//
// Reference: UPML Scheme3D.cpp:266-416 and 3659-3818 (profiles), Drude
// Kernels.h:103-107 / Scheme3D.cpp:326-364, NTFF Scheme3D.cpp:2263-2307 and
// 4093-4509.
#pragma once

#include <array>

#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstdio>
#include <string>
#include <vector>

#include "capi.h"
#include "host_native.h"

namespace native_phys {

constexpr double kC = 2.99792458e8;
constexpr double kEps0 = 8.8541878176203892e-12;
constexpr double kMu0 = 1.2566370614359173e-6;
constexpr double kPi = 3.14159265358979323846;

// material averaging stencils (eps-layout offsets, pairwise order; layout/yee.py MATERIAL_STENCIL)
const int kStencilN[6] = {2, 2, 2, 4, 4, 4};
const int kStencil[6][4][3] = {{{0, 0, 0}, {1, 0, 0}},
                               {{0, 0, 0}, {0, 1, 0}},
                               {{0, 0, 0}, {0, 0, 1}},
                               {{0, 0, 0}, {0, 0, 1}, {0, 1, 0}, {0, 1, 1}},
                               {{0, 0, 0}, {0, 0, 1}, {1, 0, 0}, {1, 0, 1}},
                               {{0, 0, 0}, {0, 1, 0}, {1, 0, 0}, {1, 1, 0}}};
// UPML axes (aD, aCa, aCb) per component (layout/yee.py UPML_AXES)
const int kUpmlAxes[6][3] = {{1, 2, 0}, {2, 0, 1}, {0, 1, 2}, {1, 2, 0}, {2, 0, 1}, {0, 1, 2}};
// curl terms (source component, axis, sign) (layout/yee.py CURL_TERMS)
const int kCurlT[6][2][3] = {{{5, 1, +1}, {4, 2, -1}}, {{3, 2, +1}, {5, 0, -1}}, {{4, 0, +1}, {3, 1, -1}},
                             {{1, 2, +1}, {2, 1, -1}}, {{2, 0, +1}, {0, 2, -1}}, {{0, 1, +1}, {1, 0, -1}}};

// pairwise-hierarchical mean of 2 or 4 values (Approximation.cpp:15-32)
inline double approx_mean(const double* v, int n) {
  if (n == 2) return (v[0] + v[1]) / 2.0;
  return ((v[0] + v[1]) / 2.0 + (v[2] + v[3]) / 2.0) / 2.0;
}

// polynomially graded UPML sigma on the eps layout of one axis (grading m = 6,
// reflection 1e-16, integrated per cell; layout/materials.py sigma_profile_1d)
inline std::vector<double> sigma_profile(int n_eps, int pml, double dx) {
  std::vector<double> out(n_eps, 0.0);
  if (pml <= 0) return out;
  const double boundary = pml * dx;
  const int m = 6;
  const double sigma_max = -std::log(1e-16) * (m + 1.0) / (2.0 * std::sqrt(kMu0 / kEps0) * boundary);
  const double factor = sigma_max / (dx * std::pow(boundary, m) * (m + 1));
  for (int idx = 0; idx < n_eps; ++idx) {
    const double pos = idx + 0.5;
    int dist = -1;
    if (pos < pml)
      dist = (int)(pml - pos);
    else if (pos >= (n_eps + 0.5) - pml)
      dist = (int)(pos - ((n_eps + 0.5) - pml));
    if (dist < 0) continue;
    const double x1 = (dist + 1) * dx, x2 = dist * dx;
    out[idx] = factor * (std::pow(x1, m + 1) - std::pow(x2, m + 1));
  }
  return out;
}

// (b0, b1, b2, ma1, ma2) of the dispersive ADE (models/scheme.py _drude_coefs:
// the same expression order, so the fp64 values agree bit for bit)
inline void drude_coefs(double dt, double e0, double eps, double w, double g, double q, double* o) {
  const double A = 4 * e0 * eps + 2 * dt * e0 * eps * g + e0 * (dt * dt * w * w + q * eps);
  o[0] = (4 + 2 * dt * g + q) / A;
  o[1] = (-8.0 + 2 * q) / A;
  o[2] = (4 - 2 * dt * g + q) / A;
  o[3] = -(2 * e0 * (dt * dt * w * w + q * eps) - 8 * e0 * eps) / A;
  o[4] = -(4 * e0 * eps - 2 * dt * e0 * eps * g + e0 * (dt * dt * w * w + q * eps)) / A;
}

inline void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "HIP error %s (%s)\n", hipGetErrorString(e), what);
    std::exit(1);
  }
}

template <typename T>
T* dev_upload(const std::vector<T>& h, std::vector<void*>& keep) {
  void* p = nullptr;
  hip_ok(hipMalloc(&p, (h.empty() ? 1 : h.size()) * sizeof(T)), "malloc");
  if (!h.empty()) hip_ok(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice), "upload");
  keep.push_back(p);
  return (T*)p;
}

template <typename T>
T* dev_zeros(size_t n, std::vector<void*>& keep) {
  void* p = nullptr;
  hip_ok(hipMalloc(&p, n * sizeof(T)), "malloc");
  hip_ok(hipMemset(p, 0, n * sizeof(T)), "memset");
  keep.push_back(p);
  return (T*)p;
}

// ---------------------------------------------------------------- UPML / Drude
// Per component: the six factored profiles along (aD, aD, aCa, aCa, aCb, aCb),
// the E-from-D scalar and optional per-cell 1/(eps eps0), D levels (new level
// last: [cur, new] or, dispersive, [cur, prev, new]) and for dispersive
// components D1 levels + the uint8 material index and coefficient table.
template <typename T>
struct Upml {
  std::vector<void*> keep;
  const T* prof[6][6] = {};
  T* cell[6] = {};
  double s[6] = {};
  // D / D1 levels region-local (models/regions.py): D[c][l][q] = level l of
  // component c over chain region q (lo[3] hi[3] in rbox[q], x-major, z
  // fastest); only chain cells ever read their levels
  std::vector<std::vector<T*>> D[6], D1[6];
  std::vector<std::array<int, 6>> rbox;
  std::vector<size_t> rvol;
  bool disp[6] = {};
  unsigned char* ids[6] = {};
  T* lut[6] = {};
  int nlut[6] = {};  // rows of lut[c]
  ~Upml() {
    for (void* p : keep) (void)hipFree(p);
  }
};

struct UpmlScene {
  int pml[3];
  bool use_pml;
  bool metamaterials;
  bool lorentz;
  double lorentz_ratio;
  double freq;
  // dielectric sphere (per-cell eps) or the dispersive sphere
  bool sphere_eps;
  bool drude_sphere;
  double ctr[3], radius, eps_in;
};

// eps at an eps-layout point (linear sub-cell smoothing, Approximation.cpp:286-314)
inline double sphere_eps_at(double x, double y, double z, const UpmlScene& sc) {
  const double d = std::sqrt((x - sc.ctr[0]) * (x - sc.ctr[0]) + (y - sc.ctr[1]) * (y - sc.ctr[1]) +
                             (z - sc.ctr[2]) * (z - sc.ctr[2]));
  const double diff = d - sc.radius;
  if (diff < -0.5) return sc.eps_in;
  if (diff > 0.5) return 1.0;
  const double p = 0.5 - diff;
  return p * sc.eps_in + (1 - p) * 1.0;
}

// (decomposed runs: the rank's arrays -- allocated box at global origin `org`,
// extents `ext` -- with the profiles, materials and ids at the global
// positions; `all_disp`: every E component takes the dispersive form wherever
// the global sphere makes it dispersive, so every rank's chain launches agree
// on the form -- a rank the sphere misses gets the omega = 0 row)
template <typename T>
void setup_upml(Upml<T>& U, const fdtd::Int3& N, const UpmlScene& sc, double dt, double dx,
                const int* org = nullptr, const int* ext = nullptr, bool all_disp = false) {
  const int o0[3] = {0, 0, 0};
  const int n0[3] = {N[0], N[1], N[2]};
  if (!org) org = o0;
  if (!ext) ext = n0;
  const size_t cells = (size_t)ext[0] * ext[1] * ext[2];
  std::vector<double> sig[3];
  for (int a = 0; a < 3; ++a) sig[a] = sigma_profile(N[a] + 1, sc.use_pml ? sc.pml[a] : 0, dx);
  // omega_p of the dispersive sphere on the eps layout (float32 sqrt(2), as the reference)
  const double wp = (double)std::sqrt(2.0f) * 2 * kPi * sc.freq;
  const double w0 = sc.lorentz ? sc.lorentz_ratio * 2 * kPi * sc.freq : 0.0;
  const double q = dt * dt * w0 * w0;
  auto in_sphere = [&](int i, int j, int k) {
    const double x = i + 0.5, y = j + 0.5, z = k + 0.5;
    return (x - sc.ctr[0]) * (x - sc.ctr[0]) + (y - sc.ctr[1]) * (y - sc.ctr[1]) +
               (z - sc.ctr[2]) * (z - sc.ctr[2]) < sc.radius * sc.radius;
  };
  for (int c = 0; c < 6; ++c) {
    const int aD = kUpmlAxes[c][0], aA = kUpmlAxes[c][1], aB = kUpmlAxes[c][2];
    const double base = c < 3 ? kEps0 : kMu0;
    auto avg_prof = [&](int a) {
      std::vector<double> out(ext[a]);
      double v[4];
      for (int n = 0; n < ext[a]; ++n) {
        for (int p = 0; p < kStencilN[c]; ++p) v[p] = sig[a][org[a] + n + kStencil[c][p][a]];
        out[n] = approx_mean(v, kStencilN[c]);
      }
      return out;
    };
    const std::vector<double> sD = avg_prof(aD), sA = avg_prof(aA), sB = avg_prof(aB);
    const double two = 2 * kEps0;  // H-side sigma normalised by eps0 too (Scheme3D.cpp:1198-1201)
    std::vector<T> caD(ext[aD]), cbD(ext[aD]), caE(ext[aA]), ica(ext[aA]), cbEa(ext[aB]), ccEa(ext[aB]);
    for (int n = 0; n < ext[aD]; ++n) {
      caD[n] = (T)((two - sD[n] * dt) / (two + sD[n] * dt));
      cbD[n] = (T)((two * dt / dx) / (two + sD[n] * dt));
    }
    for (int n = 0; n < ext[aA]; ++n) {
      caE[n] = (T)((two - sA[n] * dt) / (two + sA[n] * dt));
      ica[n] = (T)(1.0 / (two + sA[n] * dt));
    }
    for (int n = 0; n < ext[aB]; ++n) {
      cbEa[n] = (T)(two + sB[n] * dt);
      ccEa[n] = (T)(-(two - sB[n] * dt));
    }
    const std::vector<T>* pv[6] = {&caD, &cbD, &caE, &ica, &cbEa, &ccEa};
    for (int p = 0; p < 6; ++p) U.prof[c][p] = dev_upload(*pv[p], U.keep);
    U.s[c] = 1.0 / base;
    // dispersive component: omega_p averaged at the component (sqrt of the
    // plain mean of squares, approximate_drude), coefficient table by value
    U.disp[c] = false;
    if (sc.metamaterials && sc.drude_sphere && c < 3) {
      std::vector<double> vals;
      std::vector<unsigned char> id(cells);
      for (int li = 0; li < ext[0]; ++li)
        for (int lj = 0; lj < ext[1]; ++lj)
          for (int lk = 0; lk < ext[2]; ++lk) {
            const int i = org[0] + li, j = org[1] + lj, k = org[2] + lk;
            double sq = 0.0;
            for (int p = 0; p < kStencilN[c]; ++p) {
              const double w = in_sphere(i + kStencil[c][p][0], j + kStencil[c][p][1], k + kStencil[c][p][2]) ? wp
                                                                                                                 : 0.0;
              sq += w * w;
            }
            const double w = std::sqrt(sq / (double)kStencilN[c]);
            size_t q2 = 0;
            while (q2 < vals.size() && vals[q2] != w) ++q2;
            if (q2 == vals.size()) vals.push_back(w);
            id[((size_t)li * ext[1] + lj) * ext[2] + lk] = (unsigned char)q2;
          }
      if (vals.size() > 256) {
        std::fprintf(stderr, "fdtd3d (native): more than 256 distinct Drude tuples\n");
        std::exit(1);
      }
      bool any = all_disp && sc.radius > 0;
      for (double w : vals) any = any || w != 0.0;
      if (any) {
        U.disp[c] = true;
        std::vector<T> tab(5 * vals.size());
        for (size_t q2 = 0; q2 < vals.size(); ++q2) {
          double o[5];
          drude_coefs(dt, base, 1.0, vals[q2], 0.0, q, o);
          for (int e = 0; e < 5; ++e) tab[5 * q2 + e] = (T)o[e];
        }
        U.lut[c] = dev_upload(tab, U.keep);
        U.nlut[c] = (int)vals.size();
        U.ids[c] = dev_upload(id, U.keep);
        U.s[c] = 1.0;  // E from D1 (D1 already carries 1/(eps eps0))
      }
    } else if (sc.sphere_eps && c < 3) {
      // per-cell 1/(eps eps0) with eps averaged at the component (E only; mu = 1)
      std::vector<T> cl(cells);
      for (int li = 0; li < ext[0]; ++li)
        for (int lj = 0; lj < ext[1]; ++lj)
          for (int lk = 0; lk < ext[2]; ++lk) {
            const int i = org[0] + li, j = org[1] + lj, k = org[2] + lk;
            double v[2];
            for (int p = 0; p < 2; ++p)
              v[p] = sphere_eps_at(i + kStencil[c][p][0] + 0.5, j + kStencil[c][p][1] + 0.5,
                                   k + kStencil[c][p][2] + 0.5, sc);
            cl[((size_t)li * ext[1] + lj) * ext[2] + lk] = (T)(1.0 / (approx_mean(v, 2) * base));
          }
      U.cell[c] = dev_upload(cl, U.keep);
      U.s[c] = 1.0;
    }
  }
}

// the level storage over the chain regions (after the plan knows them):
// ``disp_reg[q]`` -- region q runs the dispersive form (D1 levels there)
template <typename T>
void alloc_levels(Upml<T>& U, const std::vector<std::array<int, 6>>& regs, const std::vector<bool>& disp_reg) {
  U.rbox = regs;
  U.rvol.clear();
  for (const auto& b : regs)
    U.rvol.push_back((size_t)std::max(0, b[3] - b[0]) * std::max(0, b[4] - b[1]) * std::max(0, b[5] - b[2]));
  for (int c = 0; c < 6; ++c) {
    const int nlev = U.disp[c] ? 3 : 2;
    U.D[c].assign(nlev, std::vector<T*>(regs.size(), nullptr));
    U.D1[c].assign(U.disp[c] ? 3 : 0, std::vector<T*>(regs.size(), nullptr));
    for (int l = 0; l < nlev; ++l)
      for (size_t q = 0; q < regs.size(); ++q) U.D[c][l][q] = dev_zeros<T>(std::max<size_t>(1, U.rvol[q]), U.keep);
    if (U.disp[c])
      for (int l = 0; l < 3; ++l)
        for (size_t q = 0; q < regs.size(); ++q)
          if (disp_reg[q]) U.D1[c][l][q] = dev_zeros<T>(std::max<size_t>(1, U.rvol[q]), U.keep);
  }
}

// one chain launch for the three components of a kind (kind 0 = E): the whole
// update boxes; dispersive components take the ADE form
// level rotation of a kind's components: new -> cur (-> prev)
template <typename T>
void upml_rotate(Upml<T>& U, int kind) {
  for (int cc = 0; cc < 3; ++cc) {
    const int c = 3 * kind + cc;
    auto& D = U.D[c];
    if (D.size() == 3) {
      std::swap(D[2], D[1]);
      std::swap(D[1], D[0]);  // (new, cur, prev) -> (old prev, new, cur)
      auto& E1 = U.D1[c];
      std::swap(E1[2], E1[1]);
      std::swap(E1[1], E1[0]);
    } else if (D.size() == 2) {
      std::swap(D[0], D[1]);
    }
  }
}

template <typename T>
int upml_kind(Upml<T>& U, T* const* F, const int* boxes, int kind, int ny, int nz, void* stream,
              int (*chain)(const void* const*, const double*, const int*, int, int, int, int, void*),
              bool rotate = true, bool plain_form = false, const int* pboxes = nullptr, double pcb = 1.0,
              int region = 0) {
  // pboxes (36 ints, per component lo[3] hi[3]): plain Yee cells folded into
  // the launch, F += pcb curl (a thin shell window on the z side of a z slab)
  // plain_form: dispersive components take the non-dispersive chain (E from D
  // through 1/eps0) -- the launches over boxes without dispersive cells (the
  // PML slabs around an interior sphere)
  if (fdtd_chain_ints_per_comp() != 25 || fdtd_chain_ptrs_per_comp() != 24) return (int)hipErrorInvalidValue;
  const void* P[72] = {};
  double S[6] = {};
  int I[75] = {};  // 25 per component (chain_kernels.hip CI_PER); plain and storage boxes empty
  int drude = 0;
  for (int cc = 0; cc < 3; ++cc) {
    const int c = 3 * kind + cc;
    const void** p = P + 24 * cc;
    const bool d = U.disp[c] && !plain_form;
    drude = drude || d;
    const auto& D = U.D[c];
    const int q = region;
    p[0] = F[c];
    p[1] = D.back()[q];
    p[2] = D[0][q];
    p[3] = d ? D[1][q] : nullptr;
    if (d) {
      p[4] = U.D1[c][2][q];
      p[5] = U.D1[c][0][q];
      p[6] = U.D1[c][1][q];
      if (!p[4] || !p[5] || !p[6]) return (int)hipErrorInvalidValue;
    }
    p[7] = F[kCurlT[c][0][0]];
    p[8] = F[kCurlT[c][1][0]];
    for (int q = 0; q < 6; ++q) p[9 + q] = U.prof[c][q];
    p[15] = U.cell[c];
    p[21] = U.ids[c];
    p[22] = U.lut[c];
    S[2 * cc] = (U.disp[c] && !d) ? 1.0 / (c < 3 ? kEps0 : kMu0) : U.s[c];
    S[2 * cc + 1] = pcb;
    int* in = I + 25 * cc;
    in[0] = kCurlT[c][0][1];
    in[1] = kCurlT[c][1][1];
    in[2] = kCurlT[c][0][2];
    in[3] = kCurlT[c][1][2];
    in[4] = kUpmlAxes[c][0];
    in[5] = kUpmlAxes[c][1];
    in[6] = kUpmlAxes[c][2];
    for (int q = 0; q < 6; ++q) in[7 + q] = boxes[6 * c + q];
    if (pboxes)
      for (int e = 0; e < 6; ++e) in[13 + e] = pboxes[6 * c + e];
    for (int e = 0; e < 6; ++e) in[19 + e] = U.rbox[q][e];  // the storage box of the levels
  }
  // a kind launches in one form: every component dispersive, or none
  for (int cc = 0; cc < 3; ++cc)
    if ((U.disp[3 * kind + cc] && !plain_form) != (drude != 0)) return (int)hipErrorInvalidValue;
  const int rc = chain(P, S, I, drude, kind == 0 ? 1 : 0, ny, nz, stream);
  if (rc) return rc;
  if (rotate) upml_rotate(U, kind);
  return 0;
}

// ------------------------------------------------------------------- NTFF
// Scattered power diagram over the box ntff cells inside every border
// (models/ntff.py): tangential fields averaged to the face-cell centres,
// equivalent currents J = n x H, M = -n x E, radiation vectors N, L summed
// with separable phases, P = k^2 / (8 pi eta0) (|L_ph + eta0 N_th|^2 +
// |L_th - eta0 N_ph|^2) normalised by 1 / eta0.  Real fields (zero imaginary
// part) -- the native driver has no complex mode.
const double kMinFPn[6][3] = {{1.0, 0.5, 0.5}, {0.5, 1.0, 0.5}, {0.5, 0.5, 1.0},
                              {0.5, 1.0, 1.0}, {1.0, 0.5, 1.0}, {1.0, 1.0, 0.5}};

struct Plan {
  int base[3], n[3], noff[3];
};

inline Plan sample_plan(int comp, int axis, double x0, const double* lo, const double* hi) {
  Plan P;
  for (int a = 0; a < 3; ++a) {
    const double t0 = a == axis ? x0 : lo[a] + 0.5;
    P.n[a] = a == axis ? 1 : (int)std::lround(hi[a] - lo[a]);
    const double first = t0 - kMinFPn[comp][a];
    if (std::fabs(first - std::round(first)) < 1e-9) {
      P.noff[a] = 1;
      P.base[a] = (int)std::lround(first);
    } else {
      P.noff[a] = 2;
      P.base[a] = (int)std::floor(first);
    }
  }
  return P;
}

// face-centre values of a component (row-major over the two other axes)
template <typename T>
std::vector<double> sample_face(const T* dev, const fdtd::Int3& N, int comp, int axis, double x0, const double* lo,
                                const double* hi) {
  const Plan P = sample_plan(comp, axis, x0, lo, hi);
  int ext[3];
  for (int a = 0; a < 3; ++a) ext[a] = P.n[a] + P.noff[a] - 1;
  // the slab the plan reads, copied row block by row block
  std::vector<T> box((size_t)ext[0] * ext[1] * ext[2]);
  for (int i = 0; i < ext[0]; ++i) {
    const T* src = dev + ((size_t)(P.base[0] + i) * N[1] + P.base[1]) * N[2] + P.base[2];
    hip_ok(hipMemcpy2D(box.data() + (size_t)i * ext[1] * ext[2], ext[2] * sizeof(T), src, N[2] * sizeof(T),
                       ext[2] * sizeof(T), ext[1], hipMemcpyDeviceToHost),
           "ntff slab");
  }
  std::vector<double> out((size_t)P.n[0] * P.n[1] * P.n[2]);
  const int cnt = P.noff[0] * P.noff[1] * P.noff[2];
  for (int i = 0; i < P.n[0]; ++i)
    for (int j = 0; j < P.n[1]; ++j)
      for (int k = 0; k < P.n[2]; ++k) {
        double acc = 0.0;
        bool first = true;
        for (int ox = 0; ox < P.noff[0]; ++ox)
          for (int oy = 0; oy < P.noff[1]; ++oy)
            for (int oz = 0; oz < P.noff[2]; ++oz) {
              const double v = (double)box[((size_t)(i + ox) * ext[1] + (j + oy)) * ext[2] + (k + oz)];
              acc = first ? v : acc + v;
              first = false;
            }
        out[((size_t)i * P.n[1] + j) * P.n[2] + k] = acc / cnt;
      }
  return out;
}

template <typename T>
std::vector<double> ntff_power(T* const* F, const fdtd::Int3& N, const int* ntff, double dx, double wavelength,
                               double theta, const std::vector<double>& phis) {
  using cd = std::complex<double>;
  const double eta0 = std::sqrt(kMu0 / kEps0);
  const double k = 2 * kPi / wavelength;
  double L[3], R[3];
  for (int a = 0; a < 3; ++a) {
    L[a] = ntff[a];
    R[a] = N[a] - ntff[a];
  }
  const double center = N[0] / 2.0;
  const size_t A = phis.size();
  const double st = std::sin(theta), ct = std::cos(theta);
  std::vector<double> rh[3];
  for (int a = 0; a < 3; ++a) rh[a].resize(A);
  for (size_t q = 0; q < A; ++q) {
    rh[0][q] = st * std::cos(phis[q]);
    rh[1][q] = st * std::sin(phis[q]);
    rh[2][q] = ct;
  }
  std::vector<cd> Nv(3 * A, cd(0, 0)), Lv(3 * A, cd(0, 0));
  const cd I1(0.0, 1.0);
  for (int axis = 0; axis < 3; ++axis) {
    for (int side = 0; side < 2; ++side) {
      const double x0 = side ? R[axis] : L[axis];
      const double s = side ? 1.0 : -1.0;
      int others[2], m = 0;
      for (int a = 0; a < 3; ++a)
        if (a != axis) others[m++] = a;
      const int a1 = others[0], a2 = others[1];
      std::vector<double> Ht[3], Et[3];
      for (int a : others) {
        Ht[a] = sample_face(F[3 + a], N, 3 + a, axis, x0, L, R);
        Et[a] = sample_face(F[a], N, a, axis, x0, L, R);
      }
      const double cyc = ((a1 - axis + 3) % 3 == 1) ? 1.0 : -1.0;
      const int nu = (int)std::lround(R[a1] - L[a1]), nv = (int)std::lround(R[a2] - L[a2]);
      // currents: (target vector, component, sign, source)
      struct Cur {
        std::vector<cd>* acc;
        int ca;
        double sg;
        const std::vector<double>* v;
      } cur[4] = {{&Nv, a2, s * cyc, &Ht[a1]}, {&Nv, a1, -s * cyc, &Ht[a2]},
                  {&Lv, a2, -s * cyc, &Et[a1]}, {&Lv, a1, s * cyc, &Et[a2]}};
      std::vector<cd> eu((size_t)A * nu), ev((size_t)A * nv), e0(A);
      for (size_t q = 0; q < A; ++q) {
        for (int u = 0; u < nu; ++u)
          eu[q * nu + u] = std::exp(-I1 * (k * (rh[a1][q] * ((u + L[a1] + 0.5 - center) * dx))));
        for (int v = 0; v < nv; ++v)
          ev[q * nv + v] = std::exp(-I1 * (k * (rh[a2][q] * ((v + L[a2] + 0.5 - center) * dx))));
        e0[q] = std::exp(-I1 * (k * (rh[axis][q] * ((x0 - center) * dx)))) * (dx * dx);
      }
      for (const Cur& C : cur) {
        for (size_t q = 0; q < A; ++q) {
          cd sum(0, 0);
          for (int u = 0; u < nu; ++u) {
            cd t1(0, 0);
            for (int v = 0; v < nv; ++v) t1 += (*C.v)[(size_t)u * nv + v] * ev[q * nv + v];
            sum += t1 * eu[q * nu + u];
          }
          (*C.acc)[3 * q + C.ca] += C.sg * sum * e0[q];
        }
      }
    }
  }
  std::vector<double> out(A);
  for (size_t q = 0; q < A; ++q) {
    const double cp = std::cos(phis[q]), sp = std::sin(phis[q]);
    const cd N_th = Nv[3 * q] * (ct * cp) + Nv[3 * q + 1] * (ct * sp) - Nv[3 * q + 2] * st;
    const cd N_ph = -Nv[3 * q] * sp + Nv[3 * q + 1] * cp;
    const cd L_th = Lv[3 * q] * (ct * cp) + Lv[3 * q + 1] * (ct * sp) - Lv[3 * q + 2] * st;
    const cd L_ph = -Lv[3 * q] * sp + Lv[3 * q + 1] * cp;
    const double p = (k * k) / (8 * kPi * eta0) * (std::norm(L_ph + eta0 * N_th) + std::norm(L_th - eta0 * N_ph));
    out[q] = p / (1.0 / eta0);
  }
  return out;
}

// phi in [0, 2 pi + pi/180] step pi/90 (Scheme3D.cpp:2283, models/ntff.py reference_angles)
inline std::vector<double> reference_angles() {
  std::vector<double> out;
  for (double a = 0.0; a <= 2 * kPi + kPi / 180; a += kPi / 90) out.push_back(a);
  return out;
}

}  // namespace native_phys
