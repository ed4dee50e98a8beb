// native_lowdim.h -- the native driver's 2D (TMz / TEz) half steps on boxes:
// the plain 2D kernels clipped to a region, the CPML corrections and the UPML
// D/B chain on the four PML strips (models/scheme.py _update for 2D schemes).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>

#include "capi.h"
#include "host_native.h"
#include "settings_native.h"
#include "native_api.h"
#include "native_setup.h"

// Part of the native driver: included by main.cpp only (one translation unit),
// hence the unnamed namespace.
namespace {

template <typename T>
struct Lowdim2d {
  Dev<T>* F;  // the current field buffers (pointer swaps are seen at every call)
  Dev<T>* C;
  const int* boxes;
  fdtd::Int3 N;
  const bool* present;
  Pml2d<T>& p2;
  bool tm, percell;
  double cb, db;
  hipStream_t st;
  // UPML: the inner box (every sigma vanishes, the chain is the plain update
  // to round-off) and the four PML strips (one cell of staggering slack inside)
  IBox inner, strips[4];

  // (decomposed runs: N_ = the rank's array extents, `G` = the global grid,
  // `org` = the rank's global origin: the strips are the global ones in the
  // rank's indices; `boxes` hold its owned update boxes)
  Lowdim2d(const fdtd::Settings& s, Dev<T>* F_, Dev<T>* C_, const int* boxes_, const fdtd::Int3& N_,
           const bool* present_, Pml2d<T>& p2_, bool tm_, bool percell_, double cb_, double db_, hipStream_t st_,
           const fdtd::Int3* G = nullptr, const int* org = nullptr)
      : F(F_), C(C_), boxes(boxes_), N(N_), present(present_), p2(p2_), tm(tm_), percell(percell_), cb(cb_), db(db_),
        st(st_) {
    const fdtd::Int3 M = G ? *G : N;
    const int o[3] = {org ? org[0] : 0, org ? org[1] : 0, org ? org[2] : 0};
    const int ppx = s.pmlSizeX + 1, ppy = s.pmlSizeY + 1;
    inner = {{ppx, ppy, 0}, {M[0] - ppx, M[1] - ppy, M[2]}};
    strips[0] = {{0, 0, 0}, {std::min(ppx, M[0]), M[1], M[2]}};
    strips[1] = {{std::max(0, M[0] - ppx), 0, 0}, {M[0], M[1], M[2]}};
    strips[2] = {{ppx, 0, 0}, {M[0] - ppx, std::min(ppy, M[1]), M[2]}};
    strips[3] = {{ppx, std::max(0, M[1] - ppy), 0}, {M[0] - ppx, M[1], M[2]}};
    for (IBox* b : {&inner, &strips[0], &strips[1], &strips[2], &strips[3]})
      for (int a = 0; a < 3; ++a) {
        b->lo[a] -= o[a];
        b->hi[a] -= o[a];
      }
  }

  // 2D CPML corrections of one kind (0 = E) after the plain update
  void cpml(int kind) {
    for (const Slab2d<T>& sl : p2.slabs) {
      if ((sl.comp < 3) != (kind == 0)) continue;
      const void* cp[4] = {nullptr, nullptr, nullptr, percell ? (const void*)C[sl.comp].p : nullptr};
      K_OK(cpml_apply(F[sl.comp].p, F[sl.src].p, sl.psi, sl.axis, sl.sign, kind == 0 ? 1 : 0, sl.b, sl.c, sl.k,
                      percell ? 1.0 : (kind == 0 ? cb : db), cp, N[1], N[2], sl.box, sl.pbox, st));
    }
  }

  // the plain 2D kernels of one kind over the per-component update boxes
  // clipped to `region`
  void plain(int kind, const IBox& region) {
    int ib[36];
    for (int c = 0; c < 6; ++c) {
      IBox ub;
      for (int a = 0; a < 3; ++a) {
        ub.lo[a] = boxes[6 * c + a];
        ub.hi[a] = boxes[6 * c + 3 + a];
      }
      const IBox b = box_and(ub, region);
      for (int a = 0; a < 3; ++a) {
        ib[6 * c + a] = b.empty() ? 0 : b.lo[a];
        ib[6 * c + 3 + a] = b.empty() ? 0 : b.hi[a];
      }
    }
    if (kind == 0) {
      if (tm)
        K_OK(tmz_e(F[2].p, F[3].p, F[4].p, C[2].p, percell ? 1.0 : cb, N[0], N[1], ib + 12, st));
      else
        K_OK(tez_e(F[0].p, F[1].p, F[5].p, C[0].p, C[1].p, percell ? 1.0 : cb, N[0], N[1], ib, st));
    } else {
      if (tm)
        K_OK(tmz_h(F[3].p, F[4].p, F[2].p, C[3].p, C[4].p, percell ? 1.0 : db, N[0], N[1], ib + 18, st));
      else
        K_OK(tez_h(F[5].p, F[0].p, F[1].p, C[5].p, percell ? 1.0 : db, N[0], N[1], ib + 30, st));
    }
  }

  // the D/B chain of one kind on the PML strips (+ level rotation)
  void upml_chain(int kind) {
    for (int c = 3 * kind; c < 3 * kind + 3; ++c) {
      if (!present[c]) continue;
      const T* srcs[2];
      int axes[2], signs[2], nt = 0;
      for (int q = 0; q < 2; ++q) {
        const int sc = kCurl[c][q][0], ax = kCurl[c][q][1];
        if (!present[sc] || ax >= 2) continue;
        srcs[nt] = F[sc].p;
        axes[nt] = ax;
        signs[nt++] = kCurl[c][q][2];
      }
      IBox ub;
      for (int a = 0; a < 3; ++a) {
        ub.lo[a] = boxes[6 * c + a];
        ub.hi[a] = boxes[6 * c + 3 + a];
      }
      const double sc3[3] = {1.0, p2.s[c], p2.s[c]};
      const T* xs[3] = {F[c].p, p2.D[c][1], p2.D[c][0]};
      for (const IBox& sb : strips) {
        const IBox b = box_and(sb, ub);
        if (b.empty()) continue;
        const int bx[6] = {b.lo[0], b.lo[1], b.lo[2], b.hi[0], b.hi[1], b.hi[2]};
        K_OK(curl_gen(p2.D[c][1], p2.D[c][0], srcs, axes, signs, nt, kind == 0 ? 1 : 0, p2.ca[c], p2.cbp[c], N[1],
                      N[2], bx, st));
        K_OK(lincomb(F[c].p, 3, sc3, p2.lin[c], xs, N[1], N[2], bx, st));
      }
      std::swap(p2.D[c][0], p2.D[c][1]);
    }
  }

  // UPML half step: the chain on the strips, the plain kernel on the inner box
  void upml(int kind) {
    upml_chain(kind);
    plain(kind, inner);
  }
};

}  // namespace
