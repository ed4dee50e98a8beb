// native_setup.h -- host-side set-up of the native driver's physics: hybrid-pass boxes,
// 3D / 2D CPML and UPML profiles, TF/SF tables (models/cpml.py, models/tfsf.py twins).
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
#include "host_native.h"
#include "native_physics.h"
#include "settings_native.h"
#include "native_api.h"

// Part of the native driver: included by main.cpp only (one translation unit),
// hence the unnamed namespace.
namespace {

// CPML (3D, 4-cell z lanes: fp32 float4 / fp64 double4): profiles, psi slabs and the per-kind term
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

template <typename T>
struct NativeCpml {
  std::vector<Dev<T>*> keep;           // psi slabs and profile arrays
  std::vector<const void*> P[2];       // per kind (E, H): 9 x 5 pointers
  std::vector<int> I[2];               // per kind: 9 x 4 ints
  ~NativeCpml() {
    for (auto* d : keep) delete d;
  }
  T* upload(const std::vector<T>& h) {
    auto* d = new Dev<T>();
    d->alloc(h.size());
    HIP_OK(hipMemcpy(d->p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    keep.push_back(d);
    return d->p;
  }
  T* zeros(size_t n) {
    auto* d = new Dev<T>();
    d->alloc(n);
    keep.push_back(d);
    return d->p;
  }
};

// (decomposed runs: `own` = the rank's owned cells [lo, hi) in global
// indices, `org` / `nl` = its allocated box's global origin and extents; the
// profiles follow the global position, psi and ranges are in the rank's own
// array indices)
template <typename T>
void setup_cpml(NativeCpml<T>& cp, const fdtd::Settings& s, const fdtd::Int3& N, const std::vector<int>& active,
                double dt, double dx, const int* own = nullptr, const int* org = nullptr, const int* nl = nullptr) {
  const int o0[3] = {0, 0, 0};
  const int n0[3] = {N[0], N[1], N[2]};
  if (!org) org = o0;
  if (!nl) nl = n0;
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
      if (own)
        for (int a = 0; a < 3; ++a) {
          glo[a] = std::max(glo[a], own[a]);
          ghi[a] = std::min(ghi[a], own[3 + a]);
        }
      for (int a = 0; a < 3; ++a) {
        // a component's two curl terms differentiate along the other two axes
        const int P = Ps[a];
        if (a == cc || P <= 0 || std::find(active.begin(), active.end(), a) == active.end()) continue;
        const int n = nl[a];
        const double m = mco[c][a];
        const double sig_max = -(4 + 1) * std::log(1e-8) / (2 * eta * P * dx);
        std::vector<T> b(n, T(1)), cv(n, T(0)), kk(n, T(0));
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
          lo -= org[a];  // the rank's array indices
          hi -= org[a];
          if (a == 2 && nl[2] % 4 == 0) {  // z slabs padded to whole float4 groups (c = 0 there)
            lo &= ~3;
            hi = std::min(nl[2], (hi + 3) & ~3);
          }
          for (int v = lo; v < hi; ++v) {
            const double idx = v + org[a] + m;
            double depth = side == 0 ? (P - idx) / P : (idx - (N[a] - P)) / P;
            depth = std::min(1.0, std::max(0.0, depth));
            const double d4 = depth * depth * depth * depth;
            const double sig = sig_max * d4, kap = 1.0 + (kmax - 1.0) * d4, alp = amax * (1.0 - depth);
            const double bc = std::exp(-(sig / kap + alp) * dt / kEps0);
            const double den = sig * kap + kap * kap * alp;
            b[v] = (T)bc;
            cv[v] = (T)(den > 0 ? sig / den * (bc - 1.0) : 0.0);
            kk[v] = (T)(1.0 / kap - 1.0);
          }
          // psi storage: the slab's range along a x the full extents of the other two
          size_t vol = (size_t)(hi - lo);
          for (int d = 0; d < 3; ++d)
            if (d != a) vol *= (size_t)nl[d];
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

// ------------------------------------------------------------- 2D PML
// Absorbing layers of the 2D schemes (TMz / TEz, fp32 / fp64) on the generic
// one-thread-per-cell kernels of generic_kernels.hip, whose flattened (y, z)
// plane keeps every lane busy at nz = 1:
//  * CPML: the plain 2D update runs on every cell, then each (component, curl
//    term, side) slab updates its psi and adds its term (models/cpml.py);
//  * UPML (the reference's 2D PML, SchemeTMz.cpp:1896-1945): every component
//    runs the D/B chain on its update box -- D_new = caD D + cbD curl
//    (curl_general), E = caE E + s cell ica (cbEa D_new + ccEa D) (lincomb),
//    the factored profiles of models/scheme.py _init_upml; where every sigma
//    vanishes this is the plain update to round-off.
template <typename T>
struct Slab2d {
  int comp, src, axis, sign;
  int box[6], pbox[6];
  T *psi, *b, *c, *k;
};

template <typename T>
struct Pml2d {
  std::vector<void*> keep;
  std::vector<Slab2d<T>> slabs;
  // UPML: D levels [cur, new] and the coefficient pointer sets per component
  T* D[6][2] = {};
  const void* ca[6][4] = {};
  const void* cbp[6][4] = {};
  const void* lin[6][12] = {};
  double s[6] = {};
  ~Pml2d() {
    for (void* p : keep) (void)hipFree(p);
  }
};

// (decomposed runs: `own` = the rank's owned cells in global indices, `org` /
// `ext` = its allocated box's origin and extents; slabs and psi in the rank's
// array indices, profiles at the global positions)
template <typename T>
void setup_cpml2d(Pml2d<T>& P, const fdtd::Settings& s, const fdtd::Int3& N, const std::vector<int>& active,
                  const bool* present, double dt, double dx, const int* own = nullptr, const int* org = nullptr,
                  const int* ext = nullptr) {
  const int o0[3] = {0, 0, 0};
  const int n0[3] = {N[0], N[1], N[2]};
  if (!org) org = o0;
  if (!ext) ext = n0;
  // (3D -- three active axes -- the generic slabs of 3D CPML runs whose z rows
  // are not whole 4-cell lanes)
  const int Ps[3] = {s.pmlSizeX, s.pmlSizeY, active.size() == 3 ? s.pmlSizeZ : 0};
  const int nact = (int)active.size();
  const double eta = std::sqrt(kMu0 / kEps0);
  const double kmax = s.cpmlKappaMax, amax = s.cpmlAlphaMax;
  for (int c = 0; c < 6; ++c) {
    if (!present[c]) continue;
    fdtd::Int3 glo, ghi;
    fdtd::global_range(c, N, active, glo, ghi);
    if (own)
      for (int a = 0; a < 3; ++a) {
        glo[a] = std::max(glo[a], own[a]);
        ghi[a] = std::min(ghi[a], own[3 + a]);
      }
    for (int t = 0; t < 2; ++t) {
      const int src = kCurl[c][t][0], axis = kCurl[c][t][1], sign = kCurl[c][t][2];
      if (!present[src] || axis >= std::max(2, nact) || Ps[axis] <= 0) continue;
      const int Pa = Ps[axis], n = N[axis];
      const double m = kMinFP[c][axis];
      const double sig_max = -(4 + 1) * std::log(1e-8) / (2 * eta * Pa * dx);
      for (int side = 0; side < 2; ++side) {
        int lo = glo[axis], hi = ghi[axis];
        if (side == 0)
          hi = std::min(hi, (int)std::ceil(Pa - m));
        else
          lo = std::max(lo, (int)std::floor(n - Pa - m) + 1);
        bool empty = hi <= lo;
        for (int d = 0; d < 3; ++d) empty = empty || ghi[d] <= glo[d];
        if (empty) continue;
        // profiles over the whole axis with this side's clamped depth (models/cpml.py)
        const int ne = ext[axis];
        std::vector<T> b(ne), cv(ne), kk(ne);
        for (int v = 0; v < ne; ++v) {
          const double idx = v + org[axis] + m;
          double depth = side == 0 ? (Pa - idx) / Pa : (idx - (n - Pa)) / Pa;
          depth = std::min(1.0, std::max(0.0, depth));
          const double d4 = depth * depth * depth * depth;
          const double sig = sig_max * d4, kap = 1.0 + (kmax - 1.0) * d4, alp = amax * (1.0 - depth);
          const double bc = std::exp(-(sig / kap + alp) * dt / kEps0);
          const double den = sig * kap + kap * kap * alp;
          b[v] = (T)bc;
          cv[v] = (T)(den > 0 ? sig / den * (bc - 1.0) : 0.0);
          kk[v] = (T)(1.0 / kap - 1.0);
        }
        Slab2d<T> sl;
        sl.comp = c;
        sl.src = src;
        sl.axis = axis;
        sl.sign = sign;
        size_t vol = 1;
        for (int d = 0; d < 3; ++d) {
          sl.box[d] = (d == axis ? lo : glo[d]) - org[d];
          sl.box[3 + d] = (d == axis ? hi : ghi[d]) - org[d];
          sl.pbox[d] = d == axis ? lo - org[d] : 0;
          sl.pbox[3 + d] = d == axis ? hi - org[d] : ext[d];
          vol *= (size_t)(sl.pbox[3 + d] - sl.pbox[d]);
        }
        sl.psi = native_phys::dev_zeros<T>(vol, P.keep);
        sl.b = native_phys::dev_upload(b, P.keep);
        sl.c = native_phys::dev_upload(cv, P.keep);
        sl.k = native_phys::dev_upload(kk, P.keep);
        P.slabs.push_back(sl);
      }
    }
  }
}

// 2D UPML coefficients; ``cell_inv`` (optional, per present E component):
// 1 / (eps eps0) per cell of a dielectric scene
// (decomposed runs: the rank's arrays at global origin `org`, extents `ext`,
// the profiles at the global positions; `cell_inv` over the rank's cells)
template <typename T>
void setup_upml2d(Pml2d<T>& P, const fdtd::Settings& s, const fdtd::Int3& N, const bool* present, double dt,
                  double dx, std::vector<T>* cell_inv, const int* org = nullptr, const int* ext = nullptr) {
  const int o0[3] = {0, 0, 0};
  const int n0[3] = {N[0], N[1], N[2]};
  if (!org) org = o0;
  if (!ext) ext = n0;
  const size_t cells = (size_t)ext[0] * ext[1] * ext[2];
  std::vector<double> sig[3];
  const int pml[3] = {s.pmlSizeX, s.pmlSizeY, 0};
  for (int a = 0; a < 3; ++a) sig[a] = native_phys::sigma_profile(N[a] + 1, pml[a], dx);
  for (int c = 0; c < 6; ++c) {
    if (!present[c]) continue;
    const int aD = native_phys::kUpmlAxes[c][0], aA = native_phys::kUpmlAxes[c][1], aB = native_phys::kUpmlAxes[c][2];
    auto avg = [&](int a) {
      std::vector<double> out(ext[a]);
      double v[4];
      for (int n = 0; n < ext[a]; ++n) {
        for (int p = 0; p < native_phys::kStencilN[c]; ++p)
          v[p] = sig[a][org[a] + n + native_phys::kStencil[c][p][a]];
        out[n] = native_phys::approx_mean(v, native_phys::kStencilN[c]);
      }
      return out;
    };
    const std::vector<double> sD = avg(aD), sA = avg(aA), sB = avg(aB);
    const double two = 2 * kEps0;
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
    const T* cell = nullptr;
    P.s[c] = 1.0 / (c < 3 ? kEps0 : kMu0);
    if (cell_inv && c < 3 && !cell_inv[c].empty()) {
      cell = native_phys::dev_upload(cell_inv[c], P.keep);
      P.s[c] = 1.0;
    }
    P.ca[c][aD] = native_phys::dev_upload(caD, P.keep);
    P.cbp[c][aD] = native_phys::dev_upload(cbD, P.keep);
    const T* caEd = native_phys::dev_upload(caE, P.keep);
    const T* icad = native_phys::dev_upload(ica, P.keep);
    const T* cbEd = native_phys::dev_upload(cbEa, P.keep);
    const T* ccEd = native_phys::dev_upload(ccEa, P.keep);
    // lincomb terms: (caE, E), (s ica cbEa cell, D_new), (s ica ccEa cell, D)
    P.lin[c][aA] = caEd;
    P.lin[c][4 + aA] = icad;
    P.lin[c][4 + aB] = cbEd;
    P.lin[c][4 + 3] = cell;
    P.lin[c][8 + aA] = icad;
    P.lin[c][8 + aB] = ccEd;
    P.lin[c][8 + 3] = cell;
    for (int l = 0; l < 2; ++l) P.D[c][l] = native_phys::dev_zeros<T>(cells, P.keep);
  }
}

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

// incident-wave projection onto a component (YeeGridLayout.cpp:811-845);
// projections zero in exact arithmetic (cos(pi/2) = 6e-17) are zero, as in
// layout/yee.py incident_projection
double inc_projection(int c, double t, double p, double q) {
  double v;
  switch (c) {
    case 0: v = std::cos(q) * std::sin(p) - std::sin(q) * std::cos(t) * std::cos(p); break;
    case 1: v = -std::cos(q) * std::cos(p) - std::sin(q) * std::cos(t) * std::sin(p); break;
    case 2: v = std::sin(q) * std::sin(t); break;
    case 3: v = std::sin(q) * std::sin(p) + std::cos(q) * std::cos(t) * std::cos(p); break;
    case 4: v = -std::sin(q) * std::cos(p) + std::cos(q) * std::cos(t) * std::sin(p); break;
    default: v = -(std::cos(q) * std::sin(t));
  }
  return std::fabs(v) < 1e-12 ? 0.0 : v;
}

template <typename T>
bool setup_tfsf(NativeTfsf<T>& tf, const fdtd::Settings& s, const fdtd::Int3& N, const int* boxes,
                const Dev<T>* Cc, double cb, double db, double dt, double dx, double freq, int dim,
                const bool* present, const int* org = nullptr, const int* ext = nullptr) {
  // (decomposed runs: `boxes` = the rank's owned part of every component's
  // range in global indices, targets at the rank's array offsets -- allocated
  // box at global origin `org`, extents `ext`; the incident line is global)
  const int o0[3] = {0, 0, 0};
  const int n0[3] = {N[0], N[1], N[2]};
  if (!org) org = o0;
  if (!ext) ext = n0;
  // 2D (TMz / TEz): propagation in the xy plane, theta = pi / 2, the line
  // 100 (Nx + Ny) long (SchemeTMz.h:186), z never bounds the TF box
  const bool d2 = dim == 2;
  const double th = d2 ? kPi / 2 : s.incidentWaveAngle1 * (kPi / 180.0), ph = s.incidentWaveAngle2 * (kPi / 180.0);
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
  tf.nline = 100 * (N[0] + N[1] + (d2 ? 0 : N[2]));
  tf.einc.alloc(tf.nline);
  tf.hinc.alloc(tf.nline);
  const double L[3] = {(double)s.tfsfSizeX, (double)s.tfsfSizeY, (double)s.tfsfSizeZ};
  const double R[3] = {N[0] - L[0], N[1] - L[1], N[2] - L[2]};
  const double dir[3] = {std::sin(th) * std::cos(ph), std::sin(th) * std::sin(ph), d2 ? 0.0 : std::cos(th)};
  const double zero[3] = {L[0] - 2.5 * std::sin(th) * std::cos(ph), L[1] - 2.5 * std::sin(th) * std::sin(ph),
                          d2 ? 0.0 : L[2] - 2.5 * std::cos(th)};
  const int dir_axis[6] = {0, 0, 1, 1, 2, 2};
  const bool dir_low[6] = {true, false, true, false, true, false};
  std::vector<T> hc((size_t)ext[0] * ext[1] * ext[2]);
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
      if (!present[src] || axis >= dim) continue;  // the scheme's own curl terms only
      const double proj = inc_projection(src, th, ph, ps);
      if (proj == 0.0) continue;  // no such incident component: nothing to correct
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
            if (a >= dim || (g > lo && g < hi)) sel[a].push_back(v);
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
              const long long flat = ((long long)(i - org[0]) * ext[1] + (j - org[1])) * ext[2] + (k - org[2]);
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

// The options this binary runs (everything else goes through the Python
// driver, never a silent fallback).
bool native_supported(const fdtd::Settings& s) {
  // CPML absorbing layers: 3D (the folded float4 / double4 kernels on whole
  // 4-cell z rows, else the plain kernels + generic slab kernels), 2D in
  // either precision (generic slab kernels)
  const bool cpml_ok = s.doUsePML && s.pmlType == "cpml" && !s.doUseMetamaterials && s.dimension >= 2 &&
                       (s.dimension == 2 || s.sizeZ % 4 == 0 || !s.doUseParallelGrid);
  // UPML (D/B chain) and Drude / Lorentz spheres: 3D, any precision; the 2D UPML without dispersive media
  const bool upml_ok = s.doUsePML && (s.pmlType == "upml" || s.doUseMetamaterials) &&
                       (s.dimension == 3 || (s.dimension == 2 && !s.doUseMetamaterials));
  const bool meta_ok = !s.doUseMetamaterials || (s.dimension == 3 && s.scene == "drude-sphere");
  // TF/SF plane waves: 3D and 2D (any precision), with the CPML or the UPML;
  // with the UPML the corrections take the E form, exact where every sigma
  // vanishes: the TF/SF box must lie inside the absorbing layers' interior
  bool tfsf_ok = s.doUseTFSF && s.dimension >= 2;
  if (tfsf_ok && s.doUsePML && (s.pmlType == "upml" || s.doUseMetamaterials))
    tfsf_ok = s.tfsfSizeX > s.pmlSizeX + 1 && s.tfsfSizeY > s.pmlSizeY + 1 &&
              (s.dimension == 2 || s.tfsfSizeZ > s.pmlSizeZ + 1);
  const bool ntff_ok = !s.doUseNTFF || s.dimension == 3;
  // amplitude mode: any scheme, not with the NTFF diagram
  const bool amp_ok = !s.doUseAmplitudeMode || !s.doUseNTFF;
  // parallel grids: 3D (any rank grid) / 2D (x / y) / 1D (x) -- 3D plain media on blocked passes; CPML, the UPML, Drude / Lorentz spheres
  // and TF/SF (point source optional) on the split half steps, the NTFF diagram from the gathered grid
  // (native_multi.h), amplitude mode on the split half steps
  const bool par_phys = s.doUsePML || s.doUseTFSF || s.doUseMetamaterials;
  const bool par_ok = !s.doUseParallelGrid ||
                      (s.dimension >= 1 &&
                       (s.scene == "vacuum" || s.scene == "sphere" || s.scene == "drude-sphere") &&
                       (par_phys || s.doUseMetamaterials || !s.doUseSplitKernels));
  // checkpoints / resume: plain media (state = the field components)
  const bool ckpt = !s.checkpointDir.empty() || !s.loadFromFile.empty();
  // (parallel grids: the gathered grid in the serial form, scattered over the ranks on resume)
  const bool ckpt_ok = !ckpt || (!s.doUsePML && !s.doUseTFSF && !s.doUseMetamaterials && !s.doUseAmplitudeMode &&
                                 !s.doUseNTFF && (!s.doUseParallelGrid || s.dimension == 3));
  return !((s.doUsePML && !cpml_ok && !upml_ok) || (s.doUseTFSF && !tfsf_ok) || !meta_ok || !ntff_ok || !amp_ok ||
           !par_ok || !ckpt_ok || s.doUseDoubleMaterialPrecision ||
           // complex fields: two real planes of one-GPU runs (main.cpp run)
           (s.doUseComplexFieldValues && (s.doUseAmplitudeMode || s.doUseNTFF || s.doUseParallelGrid || ckpt)));
}

}  // namespace
