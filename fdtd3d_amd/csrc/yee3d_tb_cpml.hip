// Multi-step CPML variants of the multi-row blocked kernel (tb3d_mr.h):
// one instantiation per (CPML axes of the box's dependency cone, TF/SF on /
// off) at 4 steps per pass (5 measured no faster and doubles the build), in a
// translation unit of their own.  A hybrid pass
// (models/blocking.py _hybrid3_plan) advances every shell box T steps with
// the variant of its class while the plain kernel advances the core.

#include "tb3d_mr.h"

namespace tb3d {

namespace {

const int kNone[6] = {0, 0, 0, 0, 0, 0};

template <int T>
int cpml_sel(int fx, const float* const* ein, const float* const* hin, float* const* eout, float* const* hout,
             float cb, float db, int nx, int ny, int nz, const Box3* b, const Box3& O, int xchunk, const int* src,
             const TbSrc& sv, const TfDev* tf, const float* gtab, const CpmlDev* cp, float* pscr, hipStream_t s) {
  const Box3 nb = make_box(kNone);
#define CPML_CASE(F)                                                                                            \
  case F:                                                                                                     \
    return launch_tb_mr<T, 1, CPML_R, F, CPML_NW>(ein, hin, eout, hout, nullptr, nullptr, nb, nb, cb, db, nx, ny, \
                                                  nz, b, O, xchunk, src, sv, tf, gtab, cp, pscr, s);
  if constexpr (T == 4) {
    // face classes: psi through LDS, the plain kernel's 16-wave x 2-row tile
#define FACE_CASE(F)                                                                                          \
  case F:                                                                                                     \
    return launch_tb_mr<T, 1, 2, F, 16>(ein, hin, eout, hout, nullptr, nullptr, nb, nb, cb, db, nx, ny, nz, b, O, \
                                        xchunk, src, sv, tf, gtab, cp, pscr, s);
    switch (fx) {
      FACE_CASE(8)
      FACE_CASE(12)
      FACE_CASE(16)
      FACE_CASE(20)
      FACE_CASE(32)
      FACE_CASE(36)
    }
#undef FACE_CASE
  }
  switch (fx) {
    CPML_CASE(8)
    CPML_CASE(12)
    CPML_CASE(16)
    CPML_CASE(20)
    CPML_CASE(24)
    CPML_CASE(28)
    CPML_CASE(32)
    CPML_CASE(36)
    CPML_CASE(40)
    CPML_CASE(44)
    CPML_CASE(48)
    CPML_CASE(52)
    CPML_CASE(56)
    CPML_CASE(60)
  }
#undef CPML_CASE
  return (int)hipErrorInvalidValue;
}

}  // namespace

int launch_tb_mr_cpml(int T, int fx, const float* const* ein, const float* const* hin, float* const* eout,
                      float* const* hout, float cb, float db, int nx, int ny, int nz, const Box3* b, const Box3& O,
                      int xchunk, const int* src, const TbSrc& sv, const TfDev* tf, const float* gtab,
                      const CpmlDev* cp, float* pscr, hipStream_t s) {
  switch (T) {
    case 4: return cpml_sel<4>(fx, ein, hin, eout, hout, cb, db, nx, ny, nz, b, O, xchunk, src, sv, tf, gtab, cp, pscr, s);
  }
  return (int)hipErrorInvalidValue;
}

}  // namespace tb3d
