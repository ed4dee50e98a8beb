// 2D (TMz, TEz) and 1D Yee kernels.
//
// The reference's 2D schemes (Source/Scheme/SchemeTMz.cpp:162-1309,
// SchemeTEz.cpp:109-1025) and its CUDA TMz kernels
// (Source/Cuda/CudaGlobalKernels.cu:5-153) update one component per launch
// with one thread per cell.  Here each half step is one launch; lanes walk the
// contiguous y axis (arrays are (nx, ny, 1), y fastest) and each thread
// marches along x carrying the x-neighbour in a register, as in yee3d.hip.
// The 1D scheme (Ez/Hy along x) is new: the reference lists 1D as NYI
// (Source/Settings/Settings.cpp:29).

#include "common.h"

namespace {

constexpr int TX = 64;
constexpr int TY = 4;

// Up to 8 disjoint windows of one half step in ONE launch (the hybrid
// shell's strips: models/scheme.py _update): blocks are numbered window by
// window (start[w] .. start[w + 1]), each window a (gx x gy) block grid over
// its union box bu with its own x chunk.  b0 / b1: the per-component update
// boxes (one component: b0 only).
constexpr int MAXW2 = 8;
struct Win2 {
  Box3 b0[MAXW2], b1[MAXW2], bu[MAXW2];
  int xc[MAXW2], gx[MAXW2], start[MAXW2 + 1];
  int n;
};

// window of this block (wave-uniform) and its block coordinates in it
__device__ __forceinline__ int win_of(const Win2& W, int& bx, int& by) {
  const int id = (int)blockIdx.x;
  int w = 0;
#pragma unroll
  for (int q = 1; q < MAXW2; ++q) w += (q < W.n && id >= W.start[q]) ? 1 : 0;
  const int loc = id - W.start[w];
  bx = loc % W.gx[w];
  by = loc / W.gx[w];
  return w;
}

// TMz: Ez += cb*((Hy[i]-Hy[i-1]) - (Hx[j]-Hx[j-1]))   (Kernels.h:64-74)
template <typename T, bool PERCELL>
__global__ __launch_bounds__(TX * TY) void k_tmz_e(T* __restrict__ ez, const T* __restrict__ hx,
                                                   const T* __restrict__ hy, const T* __restrict__ cbz, T cb,
                                                   int nx, int ny, Win2 W) {
  int bxi, byi;
  const int w = win_of(W, bxi, byi);
  const Box3 bz = W.b0[w];
  const int xchunk = W.xc[w];
  const int j = bz.lo[1] + bxi * TX + threadIdx.x;
  if (j >= bz.hi[1]) return;
  const int i0 = bz.lo[0] + (byi * TY + threadIdx.y) * xchunk;
  const int i1 = min(i0 + xchunk, bz.hi[0]);
  if (i0 >= i1) return;
  T hy_m = hy[(size_t)(i0 - 1) * ny + j];
  for (int i = i0; i < i1; ++i) {
    const size_t off = (size_t)i * ny + j;
    const T hyc = hy[off];
    const T c = PERCELL ? cbz[off] : cb;
    ez[off] += c * ((hyc - hy_m) - (hx[off] - hx[off - 1]));
    hy_m = hyc;
  }
}

// TMz: Hx += db*(-(Ez[j+1]-Ez[j])), Hy += db*(Ez[i+1]-Ez[i])
template <typename T, bool PERCELL>
__global__ __launch_bounds__(TX * TY) void k_tmz_h(T* __restrict__ hx, T* __restrict__ hy,
                                                   const T* __restrict__ ez, const T* __restrict__ dbx,
                                                   const T* __restrict__ dby, T db, int nx, int ny, Win2 W) {
  int bxi, byi;
  const int w = win_of(W, bxi, byi);
  const Box3 bx = W.b0[w], by = W.b1[w], bu = W.bu[w];
  const int xchunk = W.xc[w];
  const int j = bu.lo[1] + bxi * TX + threadIdx.x;
  if (j >= bu.hi[1]) return;
  const int i0 = bu.lo[0] + (byi * TY + threadIdx.y) * xchunk;
  const int i1 = min(i0 + xchunk, bu.hi[0]);
  if (i0 >= i1) return;
  T ez_c = ez[(size_t)i0 * ny + j];
  for (int i = i0; i < i1; ++i) {
    const size_t off = (size_t)i * ny + j;
    const T ez_n = (i + 1 < nx) ? ez[off + ny] : T(0);
    if (in_box(bx, i, j, 0)) {
      const T c = PERCELL ? dbx[off] : db;
      hx[off] += c * (-(ez[off + 1] - ez_c));
    }
    if (in_box(by, i, j, 0)) {
      const T c = PERCELL ? dby[off] : db;
      hy[off] += c * (ez_n - ez_c);
    }
    ez_c = ez_n;
  }
}

// TEz: Ex += cb*(Hz[j]-Hz[j-1]), Ey += cb*(-(Hz[i]-Hz[i-1]))
template <typename T, bool PERCELL>
__global__ __launch_bounds__(TX * TY) void k_tez_e(T* __restrict__ ex, T* __restrict__ ey,
                                                   const T* __restrict__ hz, const T* __restrict__ cbx,
                                                   const T* __restrict__ cby, T cb, int nx, int ny, Win2 W) {
  int bxi, byi;
  const int w = win_of(W, bxi, byi);
  const Box3 bx = W.b0[w], by = W.b1[w], bu = W.bu[w];
  const int xchunk = W.xc[w];
  const int j = bu.lo[1] + bxi * TX + threadIdx.x;
  if (j >= bu.hi[1]) return;
  const int i0 = bu.lo[0] + (byi * TY + threadIdx.y) * xchunk;
  const int i1 = min(i0 + xchunk, bu.hi[0]);
  if (i0 >= i1) return;
  T hz_m = i0 > 0 ? hz[(size_t)(i0 - 1) * ny + j] : T(0);
  for (int i = i0; i < i1; ++i) {
    const size_t off = (size_t)i * ny + j;
    const T hzc = hz[off];
    if (in_box(bx, i, j, 0)) {
      const T c = PERCELL ? cbx[off] : cb;
      ex[off] += c * (hzc - hz[off - 1]);
    }
    if (in_box(by, i, j, 0)) {
      const T c = PERCELL ? cby[off] : cb;
      ey[off] += c * (-(hzc - hz_m));
    }
    hz_m = hzc;
  }
}

// TEz: Hz += db*((Ex[j+1]-Ex[j]) - (Ey[i+1]-Ey[i]))
template <typename T, bool PERCELL>
__global__ __launch_bounds__(TX * TY) void k_tez_h(T* __restrict__ hz, const T* __restrict__ ex,
                                                   const T* __restrict__ ey, const T* __restrict__ dbz, T db,
                                                   int nx, int ny, Win2 W) {
  int bxi, byi;
  const int w = win_of(W, bxi, byi);
  const Box3 bz = W.b0[w];
  const int xchunk = W.xc[w];
  const int j = bz.lo[1] + bxi * TX + threadIdx.x;
  if (j >= bz.hi[1]) return;
  const int i0 = bz.lo[0] + (byi * TY + threadIdx.y) * xchunk;
  const int i1 = min(i0 + xchunk, bz.hi[0]);
  if (i0 >= i1) return;
  T ey_c = ey[(size_t)i0 * ny + j];
  for (int i = i0; i < i1; ++i) {
    const size_t off = (size_t)i * ny + j;
    const T ey_n = ey[off + ny];
    const T c = PERCELL ? dbz[off] : db;
    hz[off] += c * ((ex[off + 1] - ex[off]) - (ey_n - ey_c));
    ey_c = ey_n;
  }
}

// 1D: Ez += cb*(Hy[i]-Hy[i-1]) on [lo, hi); Hy += db*(Ez[i+1]-Ez[i])
template <typename T, bool PERCELL>
__global__ void k_1d_e(T* __restrict__ ez, const T* __restrict__ hy, const T* __restrict__ cbz, T cb, int lo,
                       int hi) {
  const int i = lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= hi) return;
  const T c = PERCELL ? cbz[i] : cb;
  ez[i] += c * (hy[i] - hy[i - 1]);
}

template <typename T, bool PERCELL>
__global__ void k_1d_h(T* __restrict__ hy, const T* __restrict__ ez, const T* __restrict__ dby, T db, int lo,
                       int hi) {
  const int i = lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= hi) return;
  const T c = PERCELL ? dby[i] : db;
  hy[i] += c * (ez[i + 1] - ez[i]);
}

// rows per thread along x: 16, fewer on thin windows (hybrid shell, PML
// slabs) until the launch holds >= 2048 workgroups
inline int xchunk2d(const Box3& b, int req) {
  if (req > 0) return req;
  int xc = 16;
  while (xc > 1 && (long long)cdiv(b.hi[1] - b.lo[1], TX) * cdiv(cdiv(b.hi[0] - b.lo[0], xc), TY) < 2048) xc /= 2;
  return xc;
}

// the window table of n windows: `boxes` holds per window `per` boxes of 6
// ints (one per component); empty windows are dropped.  Returns the block
// count (0: nothing to do).
inline unsigned win2(Win2& W, const int* boxes, int n, int per, int xchunk) {
  W.n = 0;
  W.start[0] = 0;
  for (int q = 0; q < n && W.n < MAXW2; ++q) {
    const Box3 b0 = make_box(boxes + 6 * per * q);
    const Box3 b1 = per > 1 ? make_box(boxes + 6 * per * q + 6) : b0;
    const Box3 bu = box_union(b0, b1);
    if (box_empty(bu)) continue;
    const int w = W.n++;
    W.b0[w] = b0;
    W.b1[w] = b1;
    W.bu[w] = bu;
    W.xc[w] = xchunk2d(bu, xchunk);
    W.gx[w] = cdiv(bu.hi[1] - bu.lo[1], TX);
    W.start[w + 1] = W.start[w] + W.gx[w] * cdiv(cdiv(bu.hi[0] - bu.lo[0], W.xc[w]), TY);
  }
  for (int w = W.n; w < MAXW2; ++w) W.start[w + 1] = W.start[W.n];
  return (unsigned)W.start[W.n];
}

template <typename T>
int tmz_e(T* ez, const T* hx, const T* hy, const T* cbz, double cb, int nx, int ny, const int* box, int n,
          int xchunk, hipStream_t s) {
  Win2 W;
  const unsigned g = win2(W, box, n, 1, xchunk);
  if (!g) return 0;
  if (cbz)
    k_tmz_e<T, true><<<g, dim3(TX, TY), 0, s>>>(ez, hx, hy, cbz, (T)cb, nx, ny, W);
  else
    k_tmz_e<T, false><<<g, dim3(TX, TY), 0, s>>>(ez, hx, hy, cbz, (T)cb, nx, ny, W);
  FDTD_RETURN_LAUNCH_STATUS();
}

template <typename T>
int tmz_h(T* hx, T* hy, const T* ez, const T* dbx, const T* dby, double db, int nx, int ny, const int* boxes, int n,
          int xchunk, hipStream_t s) {
  Win2 W;
  const unsigned g = win2(W, boxes, n, 2, xchunk);
  if (!g) return 0;
  if (dbx)
    k_tmz_h<T, true><<<g, dim3(TX, TY), 0, s>>>(hx, hy, ez, dbx, dby, (T)db, nx, ny, W);
  else
    k_tmz_h<T, false><<<g, dim3(TX, TY), 0, s>>>(hx, hy, ez, dbx, dby, (T)db, nx, ny, W);
  FDTD_RETURN_LAUNCH_STATUS();
}

template <typename T>
int tez_e(T* ex, T* ey, const T* hz, const T* cbx, const T* cby, double cb, int nx, int ny, const int* boxes, int n,
          int xchunk, hipStream_t s) {
  Win2 W;
  const unsigned g = win2(W, boxes, n, 2, xchunk);
  if (!g) return 0;
  if (cbx)
    k_tez_e<T, true><<<g, dim3(TX, TY), 0, s>>>(ex, ey, hz, cbx, cby, (T)cb, nx, ny, W);
  else
    k_tez_e<T, false><<<g, dim3(TX, TY), 0, s>>>(ex, ey, hz, cbx, cby, (T)cb, nx, ny, W);
  FDTD_RETURN_LAUNCH_STATUS();
}

template <typename T>
int tez_h(T* hz, const T* ex, const T* ey, const T* dbz, double db, int nx, int ny, const int* box, int n,
          int xchunk, hipStream_t s) {
  Win2 W;
  const unsigned g = win2(W, box, n, 1, xchunk);
  if (!g) return 0;
  if (dbz)
    k_tez_h<T, true><<<g, dim3(TX, TY), 0, s>>>(hz, ex, ey, dbz, (T)db, nx, ny, W);
  else
    k_tez_h<T, false><<<g, dim3(TX, TY), 0, s>>>(hz, ex, ey, dbz, (T)db, nx, ny, W);
  FDTD_RETURN_LAUNCH_STATUS();
}

template <typename T>
int oned_e(T* ez, const T* hy, const T* cbz, double cb, int lo, int hi, hipStream_t s) {
  if (hi <= lo) return 0;
  if (cbz)
    k_1d_e<T, true><<<cdiv(hi - lo, 256), 256, 0, s>>>(ez, hy, cbz, (T)cb, lo, hi);
  else
    k_1d_e<T, false><<<cdiv(hi - lo, 256), 256, 0, s>>>(ez, hy, cbz, (T)cb, lo, hi);
  FDTD_RETURN_LAUNCH_STATUS();
}

template <typename T>
int oned_h(T* hy, const T* ez, const T* dby, double db, int lo, int hi, hipStream_t s) {
  if (hi <= lo) return 0;
  if (dby)
    k_1d_h<T, true><<<cdiv(hi - lo, 256), 256, 0, s>>>(hy, ez, dby, (T)db, lo, hi);
  else
    k_1d_h<T, false><<<cdiv(hi - lo, 256), 256, 0, s>>>(hy, ez, dby, (T)db, lo, hi);
  FDTD_RETURN_LAUNCH_STATUS();
}

}  // namespace

#define FDTD_LOWDIM_API(SUF, T)                                                                                \
  FDTD_API int fdtd_tmz_e_##SUF(T* ez, const T* hx, const T* hy, const T* cbz, double cb, int nx, int ny,      \
                                const int* box, int xchunk, void* s) {                                         \
    return tmz_e<T>(ez, hx, hy, cbz, cb, nx, ny, box, 1, xchunk, (hipStream_t)s);                                 \
  }                                                                                                            \
  FDTD_API int fdtd_tmz_h_##SUF(T* hx, T* hy, const T* ez, const T* dbx, const T* dby, double db, int nx,      \
                                int ny, const int* boxes, int xchunk, void* s) {                               \
    return tmz_h<T>(hx, hy, ez, dbx, dby, db, nx, ny, boxes, 1, xchunk, (hipStream_t)s);                          \
  }                                                                                                            \
  FDTD_API int fdtd_tez_e_##SUF(T* ex, T* ey, const T* hz, const T* cbx, const T* cby, double cb, int nx,      \
                                int ny, const int* boxes, int xchunk, void* s) {                               \
    return tez_e<T>(ex, ey, hz, cbx, cby, cb, nx, ny, boxes, 1, xchunk, (hipStream_t)s);                          \
  }                                                                                                            \
  FDTD_API int fdtd_tez_h_##SUF(T* hz, const T* ex, const T* ey, const T* dbz, double db, int nx, int ny,      \
                                const int* box, int xchunk, void* s) {                                         \
    return tez_h<T>(hz, ex, ey, dbz, db, nx, ny, box, 1, xchunk, (hipStream_t)s);                                 \
  }                                                                                                            \
  /* the same over n <= 8 disjoint windows in one launch (boxes: per window the component boxes) */            \
  FDTD_API int fdtd_tmz_e_multi_##SUF(T* ez, const T* hx, const T* hy, const T* cbz, double cb, int nx, int ny, \
                                      const int* boxes, int n, void* s) {                                       \
    return tmz_e<T>(ez, hx, hy, cbz, cb, nx, ny, boxes, n, 0, (hipStream_t)s);                                  \
  }                                                                                                             \
  FDTD_API int fdtd_tmz_h_multi_##SUF(T* hx, T* hy, const T* ez, const T* dbx, const T* dby, double db, int nx, \
                                      int ny, const int* boxes, int n, void* s) {                               \
    return tmz_h<T>(hx, hy, ez, dbx, dby, db, nx, ny, boxes, n, 0, (hipStream_t)s);                             \
  }                                                                                                             \
  FDTD_API int fdtd_tez_e_multi_##SUF(T* ex, T* ey, const T* hz, const T* cbx, const T* cby, double cb, int nx, \
                                      int ny, const int* boxes, int n, void* s) {                               \
    return tez_e<T>(ex, ey, hz, cbx, cby, cb, nx, ny, boxes, n, 0, (hipStream_t)s);                             \
  }                                                                                                             \
  FDTD_API int fdtd_tez_h_multi_##SUF(T* hz, const T* ex, const T* ey, const T* dbz, double db, int nx, int ny, \
                                      const int* boxes, int n, void* s) {                                       \
    return tez_h<T>(hz, ex, ey, dbz, db, nx, ny, boxes, n, 0, (hipStream_t)s);                                  \
  }                                                                                                             \
  FDTD_API int fdtd_1d_e_##SUF(T* ez, const T* hy, const T* cbz, double cb, int lo, int hi, void* s) {         \
    return oned_e<T>(ez, hy, cbz, cb, lo, hi, (hipStream_t)s);                                                 \
  }                                                                                                            \
  FDTD_API int fdtd_1d_h_##SUF(T* hy, const T* ez, const T* dby, double db, int lo, int hi, void* s) {         \
    return oned_h<T>(hy, ez, dby, db, lo, hi, (hipStream_t)s);                                                 \
  }

FDTD_LOWDIM_API(f32, float)
FDTD_LOWDIM_API(f64, double)
