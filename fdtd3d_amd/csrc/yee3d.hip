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
      const T c = (PERCELL && cbx) ? cbx[off] : cb;
      ex[off] += c * ((hzc - hz[off - nz]) - (hyc - hy[off - 1]));
    }
    if (in_box(by, i, j, k)) {
      const T c = (PERCELL && cby) ? cby[off] : cb;
      ey[off] += c * ((hxc - hx[off - 1]) - (hzc - hz_m));
    }
    if (in_box(bz, i, j, k)) {
      const T c = (PERCELL && cbz) ? cbz[off] : cb;
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
      const T c = (PERCELL && dbx) ? dbx[off] : db;
      hx[off] += c * ((ey[off + 1] - ey_c) - (ez[off + nz] - ez_c));
    }
    if (in_box(by, i, j, k)) {
      const T c = (PERCELL && dby) ? dby[off] : db;
      hy[off] += c * ((ez_n - ez_c) - (ex[off + 1] - exc));
    }
    if (in_box(bz, i, j, k)) {
      const T c = (PERCELL && dbz) ? dbz[off] : db;
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
  xchunk = split_xchunk(bu.hi[0] - bu.lo[0], (long long)cdiv(bu.hi[2] - bu.lo[2], TX) * cdiv(bu.hi[1] - bu.lo[1], TY),
                        xchunk, 32);
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
  xchunk = split_xchunk(bu.hi[0] - bu.lo[0], (long long)cdiv(bu.hi[2] - bu.lo[2], TX) * cdiv(bu.hi[1] - bu.lo[1], TY),
                        xchunk, 32);
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

// ===========================================================================
// Fused leapfrog step (E then H in ONE pass, ping-pong buffers).
//
// The split kernels above move 72 B/cell/step in fp32 (E pass: read E,H
// write E; H pass: read H,E write H).  Reading old E/H from one buffer pair
// and writing new E/H to the other lets one workgroup do both half steps on a
// tile before moving on: 48 B/cell/step.  Per workgroup: a (TY x 64) tile in
// (y, z) marching along x.  At plane x it computes E_new(x) on the tile plus
// one halo row (wave TY) and one halo column (extra Ex/Ey at k+64 by lane 63)
// -- exactly the E values H_new(x-1) needs -- keeps three E planes in LDS
// (3 buffers, one barrier per plane) and then writes H_new(x-1).  Halo E
// values are recomputed, never exchanged, so there are no inter-workgroup
// dependencies.  The hard point source is applied inside the kernel so H
// sees the sourced E, as in the reference loop (Scheme3D.cpp:2003-2024).
// ===========================================================================
namespace {

template <typename T, bool PERCELL, int TY>
__global__ __launch_bounds__(64 * (TY + 1)) void k_fused3d(
    const T* __restrict__ exi, const T* __restrict__ eyi, const T* __restrict__ ezi,
    const T* __restrict__ hxi, const T* __restrict__ hyi, const T* __restrict__ hzi,
    T* __restrict__ exo, T* __restrict__ eyo, T* __restrict__ ezo,
    T* __restrict__ hxo, T* __restrict__ hyo, T* __restrict__ hzo,
    const T* __restrict__ cbx, const T* __restrict__ cby, const T* __restrict__ cbz,
    const T* __restrict__ dbx, const T* __restrict__ dby, const T* __restrict__ dbz, T cb, T db,
    int nx, int ny, int nz, Box3 bex, Box3 bey, Box3 bez, Box3 bhx, Box3 bhy, Box3 bhz, Box3 R, int xchunk,
    long long src_off, int src_comp, T src_val) {
  __shared__ T sE[3][3][TY + 1][65];  // [buffer][component][row][lane (+1 halo column)]
  const int lane = threadIdx.x;
  const int w = threadIdx.y;
  const int k = R.lo[2] + blockIdx.x * 64 + lane;
  const int j = R.lo[1] + blockIdx.y * TY + w;
  const int i0 = R.lo[0] + blockIdx.z * xchunk;
  const int i1 = min(i0 + xchunk, R.hi[0]);
  const bool owned = (w < TY) && (j < R.hi[1]) && (k < R.hi[2]);
  const bool valid = (j < ny) && (k < nz);           // may compute E here (halo included)
  const bool extra = (lane == 63) && (w < TY) && (j < ny) && (k + 1 < nz);  // E at k+1
  const size_t plane = (size_t)ny * nz;
  const size_t row = (size_t)j * nz + k;

  // plane x-1 values carried in registers
  T hxp = 0, hyp = 0, hzp = 0, hz_p1 = 0;  // hz_p1: Hz(x-1, j, k+1) for the extra column
  if (valid && i0 > 0) {
    const size_t o = (size_t)(i0 - 1) * plane + row;
    hxp = hxi[o];
    hyp = hyi[o];
    hzp = hzi[o];
    if (extra) hz_p1 = hzi[o + 1];
  }
  for (int x = i0; x <= i1; ++x) {
    const int buf = (x - i0) % 3;
    T hxc = 0, hyc = 0, hzc = 0;
    T exn = 0, eyn = 0, ezn = 0;
    if (valid && x < nx) {
      const size_t off = (size_t)x * plane + row;
      hxc = hxi[off];
      hyc = hyi[off];
      hzc = hzi[off];
      exn = exi[off];
      eyn = eyi[off];
      ezn = ezi[off];
      if (in_box(bex, x, j, k)) {
        const T c = (PERCELL && cbx) ? cbx[off] : cb;
        exn += c * ((hzc - hzi[off - nz]) - (hyc - hyi[off - 1]));
      }
      if (in_box(bey, x, j, k)) {
        const T c = (PERCELL && cby) ? cby[off] : cb;
        eyn += c * ((hxc - hxi[off - 1]) - (hzc - hzp));
      }
      if (in_box(bez, x, j, k)) {
        const T c = (PERCELL && cbz) ? cbz[off] : cb;
        ezn += c * ((hyc - hyp) - (hxc - hxi[off - nz]));
      }
      if (src_comp >= 0 && (long long)off == src_off) {
        if (src_comp == 0) exn = src_val;
        if (src_comp == 1) eyn = src_val;
        if (src_comp == 2) ezn = src_val;
      }
      // only cells inside a component's box are written: launches on
      // overlapping regions (interior / boundary shell) never clobber each other
      if (owned && x < i1) {
        if (in_box(bex, x, j, k)) exo[off] = exn;
        if (in_box(bey, x, j, k)) eyo[off] = eyn;
        if (in_box(bez, x, j, k)) ezo[off] = ezn;
      }
    }
    sE[buf][0][w][lane] = exn;
    sE[buf][1][w][lane] = eyn;
    sE[buf][2][w][lane] = ezn;
    T hz_c1 = 0;
    if (extra && x < nx) {
      // Ex, Ey at (x, j, k+1): the halo column the H update of lane 63 needs
      const size_t off = (size_t)x * plane + row + 1;
      const int k1 = k + 1;
      T ex1 = exi[off], ey1 = eyi[off];
      hz_c1 = hzi[off];
      if (in_box(bex, x, j, k1)) {
        const T c = (PERCELL && cbx) ? cbx[off] : cb;
        ex1 += c * ((hz_c1 - hzi[off - nz]) - (hyi[off] - hyi[off - 1]));
      }
      if (in_box(bey, x, j, k1)) {
        const T c = (PERCELL && cby) ? cby[off] : cb;
        ey1 += c * ((hxi[off] - hxi[off - 1]) - (hz_c1 - hz_p1));
      }
      if (src_comp >= 0 && (long long)off == src_off) {
        if (src_comp == 0) ex1 = src_val;
        if (src_comp == 1) ey1 = src_val;
      }
      sE[buf][0][w][64] = ex1;
      sE[buf][1][w][64] = ey1;
    }
    __syncthreads();
    if (x > i0 && owned) {
      // H_new at plane xm = x-1 from E_new planes xm (buffer pb) and x (buffer buf)
      const int xm = x - 1;
      const int pb = (x - 1 - i0) % 3;
      const size_t off = (size_t)xm * plane + row;
      const T ex_c = sE[pb][0][w][lane], ey_c = sE[pb][1][w][lane], ez_c = sE[pb][2][w][lane];
      const T ey_kp = sE[pb][1][w][lane + 1], ex_kp = sE[pb][0][w][lane + 1];
      const T ez_jp = sE[pb][2][w + 1][lane], ex_jp = sE[pb][0][w + 1][lane];
      const T ez_ip = sE[buf][2][w][lane], ey_ip = sE[buf][1][w][lane];
      T hxn = hxp, hyn = hyp, hzn = hzp;
      if (in_box(bhx, xm, j, k)) {
        const T c = (PERCELL && dbx) ? dbx[off] : db;
        hxn += c * ((ey_kp - ey_c) - (ez_jp - ez_c));
      }
      if (in_box(bhy, xm, j, k)) {
        const T c = (PERCELL && dby) ? dby[off] : db;
        hyn += c * ((ez_ip - ez_c) - (ex_kp - ex_c));
      }
      if (in_box(bhz, xm, j, k)) {
        const T c = (PERCELL && dbz) ? dbz[off] : db;
        hzn += c * ((ex_jp - ex_c) - (ey_ip - ey_c));
      }
      if (in_box(bhx, xm, j, k)) hxo[off] = hxn;
      if (in_box(bhy, xm, j, k)) hyo[off] = hyn;
      if (in_box(bhz, xm, j, k)) hzo[off] = hzn;
    }
    hxp = hxc;
    hyp = hyc;
    hzp = hzc;
    hz_p1 = hz_c1;
  }
}

template <typename T, int TY>
int launch_fused(const T* const* ein, const T* const* hin, T* const* eout, T* const* hout, const T* const* cbs,
                 const T* const* dbs, double cb, double db, int nx, int ny, int nz, const int* boxes, int xchunk,
                 long long src_off, int src_comp, double src_val, hipStream_t s) {
  Box3 b[6];
  for (int n = 0; n < 6; ++n) b[n] = make_box(boxes + 6 * n);
  Box3 R = b[0];
  for (int n = 1; n < 6; ++n) R = box_union(R, b[n]);
  if (box_empty(R)) return 0;
  if (xchunk <= 0) xchunk = 32;
  dim3 block(64, TY + 1, 1);
  dim3 grid(cdiv(R.hi[2] - R.lo[2], 64), cdiv(R.hi[1] - R.lo[1], TY), cdiv(R.hi[0] - R.lo[0], xchunk));
  if (cbs[0] != nullptr || dbs[0] != nullptr)  // a null kind uses its scalar
    k_fused3d<T, true, TY><<<grid, block, 0, s>>>(ein[0], ein[1], ein[2], hin[0], hin[1], hin[2], eout[0], eout[1],
                                                  eout[2], hout[0], hout[1], hout[2], cbs[0], cbs[1], cbs[2], dbs[0],
                                                  dbs[1], dbs[2], (T)cb, (T)db, nx, ny, nz, b[0], b[1], b[2], b[3],
                                                  b[4], b[5], R, xchunk, src_off, src_comp, (T)src_val);
  else
    k_fused3d<T, false, TY><<<grid, block, 0, s>>>(ein[0], ein[1], ein[2], hin[0], hin[1], hin[2], eout[0], eout[1],
                                                   eout[2], hout[0], hout[1], hout[2], cbs[0], cbs[1], cbs[2], dbs[0],
                                                   dbs[1], dbs[2], (T)cb, (T)db, nx, ny, nz, b[0], b[1], b[2], b[3],
                                                   b[4], b[5], R, xchunk, src_off, src_comp, (T)src_val);
  FDTD_RETURN_LAUNCH_STATUS();
}

}  // namespace

// ein/hin/eout/hout/cbs/dbs: arrays of 3 pointers; boxes: 6 boxes (Ex,Ey,Ez,Hx,Hy,Hz)
FDTD_API int fdtd_fused3d_f32(const float* const* ein, const float* const* hin, float* const* eout,
                              float* const* hout, const float* const* cbs, const float* const* dbs, double cb,
                              double db, int nx, int ny, int nz, const int* boxes, int xchunk, long long src_off,
                              int src_comp, double src_val, void* s) {
  return launch_fused<float, 7>(ein, hin, eout, hout, cbs, dbs, cb, db, nx, ny, nz, boxes, xchunk, src_off,
                                src_comp, src_val, (hipStream_t)s);
}

FDTD_API int fdtd_fused3d_f64(const double* const* ein, const double* const* hin, double* const* eout,
                              double* const* hout, const double* const* cbs, const double* const* dbs, double cb,
                              double db, int nx, int ny, int nz, const int* boxes, int xchunk, long long src_off,
                              int src_comp, double src_val, void* s) {
  return launch_fused<double, 7>(ein, hin, eout, hout, cbs, dbs, cb, db, nx, ny, nz, boxes, xchunk, src_off,
                                 src_comp, src_val, (hipStream_t)s);
}
