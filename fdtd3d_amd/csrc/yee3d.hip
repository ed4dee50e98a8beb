// 3D Yee leapfrog kernels for MI355X (gfx950).
//
// Replaces the reference's per-component CUDA kernels
// (Source/Cuda/CudaGlobalKernels.cu:195-439) and the CPU triple loops
// (Source/Scheme/Scheme3D.cpp:211-263 etc.) with two fused launches per step:
// one updates Ex, Ey, Ez together, one updates Hx, Hy, Hz together, so every
// H (E) value is read from HBM once per half step instead of once per
// component.
//
// Mapping (wave64-first):
//   * threadIdx.x (64 lanes) walks z, the contiguous axis: one wave = one
//     256-byte (fp32) row, fully coalesced;
//   * threadIdx.y (4 waves) walks y; the j-1 / j+1 neighbour rows are rows of
//     the same workgroup, so they hit L1;
//   * each thread marches along x over XCHUNK planes keeping the x-1 (E pass)
//     or x+1 (H pass) plane values in registers: the x-neighbour costs no load.
// With 1024^3 cells this launches 16 x 256 x (1024/XCHUNK) workgroups: far
// more than the 256 CUs x 8 resident workgroups.
//
// Coefficients: either one scalar (vacuum/homogeneous: Cb = dt/(eps eps0 dx))
// or per-cell arrays (dielectric scenes, Scheme3D.cpp:222-259).
// Each component is only written inside its own computation box (reference
// YeeGridLayout.h:131-182), so PEC borders and decomposed chunks behave
// exactly like the serial reference.

#include "common.h"

namespace {

constexpr int TX = 64;
constexpr int TY = 4;

template <typename T, bool PERCELL>
__global__ __launch_bounds__(TX * TY) void k_update_e3d(
    T* __restrict__ ex, T* __restrict__ ey, T* __restrict__ ez,
    const T* __restrict__ hx, const T* __restrict__ hy, const T* __restrict__ hz,
    const T* __restrict__ cbx, const T* __restrict__ cby, const T* __restrict__ cbz,
    T cb, int nx, int ny, int nz, Box3 bx, Box3 by, Box3 bz, Box3 bu, int xchunk) {
  const int k = bu.lo[2] + blockIdx.x * TX + threadIdx.x;
  const int j = bu.lo[1] + blockIdx.y * TY + threadIdx.y;
  if (k >= bu.hi[2] || j >= bu.hi[1]) return;
  const int i0 = bu.lo[0] + blockIdx.z * xchunk;
  const int i1 = min(i0 + xchunk, bu.hi[0]);
  const size_t plane = (size_t)ny * nz;
  const size_t row = (size_t)j * nz + k;
  // x-1 plane values carried in registers
  T hz_m = 0, hy_m = 0;
  if (i0 > 0) {
    hz_m = hz[(size_t)(i0 - 1) * plane + row];
    hy_m = hy[(size_t)(i0 - 1) * plane + row];
  }
  for (int i = i0; i < i1; ++i) {
    const size_t off = (size_t)i * plane + row;
    const T hxc = hx[off];
    const T hyc = hy[off];
    const T hzc = hz[off];
    if (in_box(bx, i, j, k)) {
      const T c = PERCELL ? cbx[off] : cb;
      ex[off] += c * ((hzc - hz[off - nz]) - (hyc - hy[off - 1]));
    }
    if (in_box(by, i, j, k)) {
      const T c = PERCELL ? cby[off] : cb;
      ey[off] += c * ((hxc - hx[off - 1]) - (hzc - hz_m));
    }
    if (in_box(bz, i, j, k)) {
      const T c = PERCELL ? cbz[off] : cb;
      ez[off] += c * ((hyc - hy_m) - (hxc - hx[off - nz]));
    }
    hz_m = hzc;
    hy_m = hyc;
  }
}

template <typename T, bool PERCELL>
__global__ __launch_bounds__(TX * TY) void k_update_h3d(
    T* __restrict__ hx, T* __restrict__ hy, T* __restrict__ hz,
    const T* __restrict__ ex, const T* __restrict__ ey, const T* __restrict__ ez,
    const T* __restrict__ dbx, const T* __restrict__ dby, const T* __restrict__ dbz,
    T db, int nx, int ny, int nz, Box3 bx, Box3 by, Box3 bz, Box3 bu, int xchunk) {
  const int k = bu.lo[2] + blockIdx.x * TX + threadIdx.x;
  const int j = bu.lo[1] + blockIdx.y * TY + threadIdx.y;
  if (k >= bu.hi[2] || j >= bu.hi[1]) return;
  const int i0 = bu.lo[0] + blockIdx.z * xchunk;
  const int i1 = min(i0 + xchunk, bu.hi[0]);
  const size_t plane = (size_t)ny * nz;
  const size_t row = (size_t)j * nz + k;
  if (i0 >= i1) return;
  T ey_c = ey[(size_t)i0 * plane + row];
  T ez_c = ez[(size_t)i0 * plane + row];
  for (int i = i0; i < i1; ++i) {
    const size_t off = (size_t)i * plane + row;
    const T exc = ex[off];
    T ey_n = 0, ez_n = 0;
    if (i + 1 < nx) {
      ey_n = ey[off + plane];
      ez_n = ez[off + plane];
    }
    if (in_box(bx, i, j, k)) {
      const T c = PERCELL ? dbx[off] : db;
      hx[off] += c * ((ey[off + 1] - ey_c) - (ez[off + nz] - ez_c));
    }
    if (in_box(by, i, j, k)) {
      const T c = PERCELL ? dby[off] : db;
      hy[off] += c * ((ez_n - ez_c) - (ex[off + 1] - exc));
    }
    if (in_box(bz, i, j, k)) {
      const T c = PERCELL ? dbz[off] : db;
      hz[off] += c * ((ex[off + nz] - exc) - (ey_n - ey_c));
    }
    ey_c = ey_n;
    ez_c = ez_n;
  }
}

template <typename T>
int launch_e3d(T* ex, T* ey, T* ez, const T* hx, const T* hy, const T* hz,
               const T* cbx, const T* cby, const T* cbz, double cb,
               int nx, int ny, int nz, const int* boxes, int xchunk, hipStream_t s) {
  Box3 bx = make_box(boxes), by = make_box(boxes + 6), bz = make_box(boxes + 12);
  Box3 bu = box_union(box_union(bx, by), bz);
  if (box_empty(bu)) return 0;
  if (xchunk <= 0) xchunk = 32;
  dim3 block(TX, TY, 1);
  dim3 grid(cdiv(bu.hi[2] - bu.lo[2], TX), cdiv(bu.hi[1] - bu.lo[1], TY), cdiv(bu.hi[0] - bu.lo[0], xchunk));
  if (cbx != nullptr) {
    k_update_e3d<T, true><<<grid, block, 0, s>>>(ex, ey, ez, hx, hy, hz, cbx, cby, cbz, (T)cb, nx, ny, nz,
                                                  bx, by, bz, bu, xchunk);
  } else {
    k_update_e3d<T, false><<<grid, block, 0, s>>>(ex, ey, ez, hx, hy, hz, cbx, cby, cbz, (T)cb, nx, ny, nz,
                                                   bx, by, bz, bu, xchunk);
  }
  FDTD_RETURN_LAUNCH_STATUS();
}

template <typename T>
int launch_h3d(T* hx, T* hy, T* hz, const T* ex, const T* ey, const T* ez,
               const T* dbx, const T* dby, const T* dbz, double db,
               int nx, int ny, int nz, const int* boxes, int xchunk, hipStream_t s) {
  Box3 bx = make_box(boxes), by = make_box(boxes + 6), bz = make_box(boxes + 12);
  Box3 bu = box_union(box_union(bx, by), bz);
  if (box_empty(bu)) return 0;
  if (xchunk <= 0) xchunk = 32;
  dim3 block(TX, TY, 1);
  dim3 grid(cdiv(bu.hi[2] - bu.lo[2], TX), cdiv(bu.hi[1] - bu.lo[1], TY), cdiv(bu.hi[0] - bu.lo[0], xchunk));
  if (dbx != nullptr) {
    k_update_h3d<T, true><<<grid, block, 0, s>>>(hx, hy, hz, ex, ey, ez, dbx, dby, dbz, (T)db, nx, ny, nz,
                                                  bx, by, bz, bu, xchunk);
  } else {
    k_update_h3d<T, false><<<grid, block, 0, s>>>(hx, hy, hz, ex, ey, ez, dbx, dby, dbz, (T)db, nx, ny, nz,
                                                   bx, by, bz, bu, xchunk);
  }
  FDTD_RETURN_LAUNCH_STATUS();
}

}  // namespace

// boxes: 18 ints = 3 boxes (x, y, z component) of (lo0, lo1, lo2, hi0, hi1, hi2)
FDTD_API int fdtd_update_e3d_f32(float* ex, float* ey, float* ez, const float* hx, const float* hy,
                                 const float* hz, const float* cbx, const float* cby, const float* cbz,
                                 double cb, int nx, int ny, int nz, const int* boxes, int xchunk,
                                 void* stream) {
  return launch_e3d<float>(ex, ey, ez, hx, hy, hz, cbx, cby, cbz, cb, nx, ny, nz, boxes, xchunk,
                           (hipStream_t)stream);
}

FDTD_API int fdtd_update_e3d_f64(double* ex, double* ey, double* ez, const double* hx, const double* hy,
                                 const double* hz, const double* cbx, const double* cby, const double* cbz,
                                 double cb, int nx, int ny, int nz, const int* boxes, int xchunk,
                                 void* stream) {
  return launch_e3d<double>(ex, ey, ez, hx, hy, hz, cbx, cby, cbz, cb, nx, ny, nz, boxes, xchunk,
                            (hipStream_t)stream);
}

FDTD_API int fdtd_update_h3d_f32(float* hx, float* hy, float* hz, const float* ex, const float* ey,
                                 const float* ez, const float* dbx, const float* dby, const float* dbz,
                                 double db, int nx, int ny, int nz, const int* boxes, int xchunk,
                                 void* stream) {
  return launch_h3d<float>(hx, hy, hz, ex, ey, ez, dbx, dby, dbz, db, nx, ny, nz, boxes, xchunk,
                           (hipStream_t)stream);
}

FDTD_API int fdtd_update_h3d_f64(double* hx, double* hy, double* hz, const double* ex, const double* ey,
                                 const double* ez, const double* dbx, const double* dby, const double* dbz,
                                 double db, int nx, int ny, int nz, const int* boxes, int xchunk,
                                 void* stream) {
  return launch_h3d<double>(hx, hy, hz, ex, ey, ez, dbx, dby, dbz, db, nx, ny, nz, boxes, xchunk,
                            (hipStream_t)stream);
}
