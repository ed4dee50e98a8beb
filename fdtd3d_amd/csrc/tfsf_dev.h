// TF/SF set table of the blocked kernels (fp32 tb3d_mr.h, fp64 yee3d_tb64.hip)
#pragma once

namespace tb3d {

// TF/SF plane-wave corrections folded into the blocked passes (fdtd3d_amd/
// models/tfsf.py TfsfSets).  A set is one (component, TF/SF face) pair of the
// reference's border tests (Scheme3D.cpp:138-208, YeeGridLayout.cpp:327-809):
// a box of target cells, one cell thick across the face.  For an incident
// direction along x or y the incident value a target sees depends on its
// index along that axis only (`va`), so each pass precomputes, per level,
// g = sign * projection * interpolated incident line at every index of a set
// (k_tfsf_pass in yee3d_tb.hip).  Inside the kernel the index along `va` is
// the plane (va = 0) or the row (va = 1) -- both wave-uniform -- so a
// correction is ONE value per (set, level, plane or row), added to the new
// value after the update (E + c (curl + g) = (E + c curl) + c g).  Each wave
// numbers the sets that touch it as slots; their metadata sit in VGPR lanes
// and the g values of a trip arrive with one vector load per kind issued
// before the field prefetch, so the level loop reads everything with
// readlane (no memory round trip) and a wave away from every face pays a few
// scalar compares per level.  (Round 4 parked 6 slots per kind and unrolled
// them at every level and row: twice the plain kernel's VALU work; the first
// round-5 form read the set table with scalar loads inside the level loop:
// +55% on the face tiles, which bound the pass.  profiles/tfsf_cost_r5.md.)
constexpr int TF_MAX_SETS = 24;
struct TfSet {
  int n;          // component 0..5 = Ex Ey Ez Hx Hy Hz
  int fa;         // axis the face is perpendicular to
  int lo[3], hi[3];
  int va;         // table axis (0 x, 1 y)
  int goff;       // first g entry of the set inside one level
};
struct TfDev {
  int nsets;
  int ld;                   // g entries per level
  int xpl[2][2];            // [E / H][low / high] x-face planes (-1: none)
  TfSet s[TF_MAX_SETS];
};

}  // namespace tb3d
