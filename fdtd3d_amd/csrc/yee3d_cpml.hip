// 3D Yee half-step kernels with the CPML folded in, 4 z cells per lane (fp32
// float4 / fp64 double4: one template).
//
// The reference absorbs with a UPML that runs three sweeps per component over
// the whole grid (Scheme3D.cpp:266-416).  The CPML here (models/cpml.py) keeps
// the plain update and adds, inside each absorbing slab, the convolution
// auxiliary of every curl term whose derivative crosses the slab:
//     psi = b[n] psi + c[n] d        d = the term's finite difference
//     F  += Cb * sign * ((1/kappa[n] - 1) d + psi)
// This kernel does both in ONE pass: the differences it needs for the curl are
// already in registers, so a slab cell costs only its psi read + write on top
// of the plain update (a separate correction launch re-reads the field, its
// source and its coefficient: 24 launches per step at 512^3 in the first
// version).  Slabs along x / y are uniform per plane / wave row and use float4
// psi rows; z slabs cover a few lanes at both row ends and go per element.
//
// psi layout of a slab along axis a: the slab's extent along a times the full
// local extents of the other two axes, z fastest (z slabs padded to float4
// groups).

#include "common.h"
#include "vec4.h"

namespace {

constexpr int TY = 4;

template <typename T>
struct CpmlT {          // one curl term of one component
  T* psi[2];            // low / high slab (nullptr: no slab on that side)
  int lo[2], hi[2];     // slab range along the term axis (local index)
  const T* b;           // profiles along the axis (identity outside the slabs)
  const T* c;
  const T* k;           // 1/kappa - 1
};

template <typename T>
struct CpmlK {
  CpmlT<T> t[3][3];     // [component][term axis] (diagonal unused)
};

template <typename V>
__device__ __forceinline__ V sub4(const V& a, const V& b) {
  V r;
  r.x = a.x - b.x;
  r.y = a.y - b.y;
  r.z = a.z - b.z;
  r.w = a.w - b.w;
  return r;
}

template <typename V, typename T>
__device__ __forceinline__ V zm1(const V& v, T s) {
  V r;
  r.x = s;
  r.y = v.x;
  r.z = v.y;
  r.w = v.z;
  return r;
}
template <typename V, typename T>
__device__ __forceinline__ V zp1(const V& v, T s) {
  V r;
  r.x = v.y;
  r.y = v.z;
  r.z = v.w;
  r.w = s;
  return r;
}

template <typename T>
__device__ __forceinline__ typename Vec4<T>::type bc4(T v) {
  return Vec4<T>::make(v, v, v, v);
}

// CPML contribution of one term (without the term sign) for the lane's 4 cells
template <int AXIS, typename T, typename V = typename Vec4<T>::type>
__device__ __forceinline__ V cpml_term(const CpmlT<T>& t, const V& d, int i, int j, int kb, int ny, int nz,
                                       unsigned mask) {
  V r = bc4<T>(T(0));
  if (AXIS < 2) {
    const int n = AXIS == 0 ? i : j;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (t.psi[s] && n >= t.lo[s] && n < t.hi[s]) {
        const int w = t.hi[s] - t.lo[s];
        const size_t po = AXIS == 0 ? ((size_t)(n - t.lo[s]) * ny + j) * nz + kb
                                    : ((size_t)i * w + (n - t.lo[s])) * nz + kb;
        const T bn = t.b[n], cn = t.c[n], kn = t.k[n];
        V p = ld4(t.psi[s], po);
        p = Vec4<T>::make(bn * p.x + cn * d.x, bn * p.y + cn * d.y, bn * p.z + cn * d.z, bn * p.w + cn * d.w);
        if (mask == 0xFu) {
          st4(t.psi[s], po, p);
        } else {
          st4m(t.psi[s], po, p, mask);
        }
        r = Vec4<T>::make(kn * d.x + p.x, kn * d.y + p.y, kn * d.z + p.z, kn * d.w + p.w);
      }
    }
  } else {
    // z slabs: ranges are whole float4 groups (models/cpml.py pads them) and
    // the profiles are the identity outside the slab, so a lane is either
    // fully outside or takes one float4 psi read/write
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (t.psi[s] && kb >= t.lo[s] && kb < t.hi[s]) {
        const int w = t.hi[s] - t.lo[s];
        const size_t po = ((size_t)i * ny + j) * w + (kb - t.lo[s]);
        const V bn = ld4(t.b, kb), cn = ld4(t.c, kb), kn = ld4(t.k, kb);
        V p = ld4(t.psi[s], po);
        p = Vec4<T>::make(bn.x * p.x + cn.x * d.x, bn.y * p.y + cn.y * d.y, bn.z * p.z + cn.z * d.z,
                          bn.w * p.w + cn.w * d.w);
        st4m(t.psi[s], po, p, mask);
        r = Vec4<T>::make(kn.x * d.x + p.x, kn.y * d.y + p.y, kn.z * d.z + p.z, kn.w * d.w + p.w);
      }
    }
  }
  return r;
}

// F += c * (sa*da + sb*db + sa*corr_a + sb*corr_b) on the masked elements
// Several disjoint windows of one half step in ONE launch (the hybrid shell:
// its windows are independent; one launch per row layout instead of one per
// window): per window its three component boxes, their union, x chunk and
// block grid; blocks numbered window by window (start[w]).
constexpr int MAXW3 = 8;
struct Win3 {
  Box3 bx[MAXW3], by[MAXW3], bz[MAXW3], bu[MAXW3];
  int xc[MAXW3], gx[MAXW3], gy[MAXW3], start[MAXW3 + 1];
  int n;
};

// window of this block (wave-uniform) and its block coordinates in it
__device__ __forceinline__ int win3_of(const Win3& W, int& gbx, int& gby, int& gbz) {
  const int id = (int)blockIdx.x;
  int w = 0;
#pragma unroll
  for (int q = 1; q < MAXW3; ++q) w += (q < W.n && id >= W.start[q]) ? 1 : 0;
  const int loc = id - W.start[w];
  gbx = loc % W.gx[w];
  gby = (loc / W.gx[w]) % W.gy[w];
  gbz = loc / (W.gx[w] * W.gy[w]);
  return w;
}

template <typename V>
__device__ __forceinline__ void apply4(V& f, const V& c, const V& v, unsigned m) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (m & (1u << q)) f4set(f, q, f4(f, q) + f4(c, q) * f4(v, q));
}

template <typename V>
__device__ __forceinline__ V comb(const V& da, const V& ca, const V& db, const V& cb_) {
  // (da + ca) - (db + cb): term a has sign +1, term b sign -1 (CURL_TERMS)
  V r;
  r.x = (da.x + ca.x) - (db.x + cb_.x);
  r.y = (da.y + ca.y) - (db.y + cb_.y);
  r.z = (da.z + ca.z) - (db.z + cb_.z);
  r.w = (da.w + ca.w) - (db.w + cb_.w);
  return r;
}

template <typename T, bool PERCELL, int LZ>
__device__ __forceinline__ void e3d_cpml_body(
    T* __restrict__ ex, T* __restrict__ ey, T* __restrict__ ez, const T* __restrict__ hx,
    const T* __restrict__ hy, const T* __restrict__ hz, const T* __restrict__ cbx,
    const T* __restrict__ cby, const T* __restrict__ cbz, T cb, int nx, int ny, int nz, const Box3& bx, const Box3& by,
    const Box3& bz, const Box3& bu, int xchunk, int gbx, int gby, int gbz, const CpmlK<T>& P) {
  // LZ lanes per z row, 64 / LZ rows per wave (LZ < 64 for z-thin boxes)
  const int zl = threadIdx.x % LZ;
  const int kb = (bu.lo[2] & ~3) + 4 * (gbx * LZ + zl);
  const int j = bu.lo[1] + (gby * TY + threadIdx.y) * (64 / LZ) + threadIdx.x / LZ;
  const bool act = (kb < bu.hi[2]) && (j < bu.hi[1]);
  const int i0 = bu.lo[0] + gbz * xchunk;
  const int i1 = min(i0 + xchunk, bu.hi[0]);
  const size_t plane = (size_t)ny * nz;
  const size_t row = act ? (size_t)j * nz + kb : 0;
  const unsigned mx = act ? kmask(bx, j, kb) : 0u;
  const unsigned my = act ? kmask(by, j, kb) : 0u;
  const unsigned mz = act ? kmask(bz, j, kb) : 0u;
  using V = typename Vec4<T>::type;
  V hz_m = bc4<T>(T(0)), hy_m = hz_m;
  if (act && i0 > 0 && (my | mz)) {
    hz_m = ld4(hz, (size_t)(i0 - 1) * plane + row);
    hy_m = ld4(hy, (size_t)(i0 - 1) * plane + row);
  }
  for (int i = i0; i < i1; ++i) {
    const size_t off = (size_t)i * plane + row;
    V hxc = bc4<T>(T(0)), hyc = hxc, hzc = hxc;
    if (act) {
      hxc = ld4(hx, off);
      hyc = ld4(hy, off);
      hzc = ld4(hz, off);
    }
    T hy_k0 = __shfl_up(hyc.w, 1, LZ);
    T hx_k0 = __shfl_up(hxc.w, 1, LZ);
    if (zl == 0 && act && kb > 0) {
      hy_k0 = hy[off - 1];
      hx_k0 = hx[off - 1];
    }
    const unsigned ux = (i >= bx.lo[0] && i < bx.hi[0]) ? mx : 0u;
    const unsigned uy = (i >= by.lo[0] && i < by.hi[0]) ? my : 0u;
    const unsigned uz = (i >= bz.lo[0] && i < bz.hi[0]) ? mz : 0u;
    if (ux) {  // Ex: (Hz, y, +) (Hy, z, -)
      V e = ld4(ex, off);
      const V da = sub4(hzc, ld4(hz, off - nz));
      const V db = sub4(hyc, zm1(hyc, hy_k0));
      const V ca = cpml_term<1>(P.t[0][1], da, i, j, kb, ny, nz, ux);
      const V cb2 = cpml_term<2>(P.t[0][2], db, i, j, kb, ny, nz, ux);
      const V c4 = PERCELL ? ld4(cbx, off) : bc4<T>(cb);
      apply4(e, c4, comb(da, ca, db, cb2), ux);
      st4m(ex, off, e, ux);
    }
    if (uy) {  // Ey: (Hx, z, +) (Hz, x, -)
      V e = ld4(ey, off);
      const V da = sub4(hxc, zm1(hxc, hx_k0));
      const V db = sub4(hzc, hz_m);
      const V ca = cpml_term<2>(P.t[1][2], da, i, j, kb, ny, nz, uy);
      const V cb2 = cpml_term<0>(P.t[1][0], db, i, j, kb, ny, nz, uy);
      const V c4 = PERCELL ? ld4(cby, off) : bc4<T>(cb);
      apply4(e, c4, comb(da, ca, db, cb2), uy);
      st4m(ey, off, e, uy);
    }
    if (uz) {  // Ez: (Hy, x, +) (Hx, y, -)
      V e = ld4(ez, off);
      const V da = sub4(hyc, hy_m);
      const V db = sub4(hxc, ld4(hx, off - nz));
      const V ca = cpml_term<0>(P.t[2][0], da, i, j, kb, ny, nz, uz);
      const V cb2 = cpml_term<1>(P.t[2][1], db, i, j, kb, ny, nz, uz);
      const V c4 = PERCELL ? ld4(cbz, off) : bc4<T>(cb);
      apply4(e, c4, comb(da, ca, db, cb2), uz);
      st4m(ez, off, e, uz);
    }
    hz_m = hzc;
    hy_m = hyc;
  }
}

template <typename T, bool PERCELL, int LZ>
__global__ __launch_bounds__(64 * TY) void k_update_e3d_cpml_v4(
    T* __restrict__ ex, T* __restrict__ ey, T* __restrict__ ez, const T* __restrict__ hx,
    const T* __restrict__ hy, const T* __restrict__ hz, const T* __restrict__ cbx,
    const T* __restrict__ cby, const T* __restrict__ cbz, T cb, int nx, int ny, int nz, Box3 bx,
    Box3 by, Box3 bz, Box3 bu, int xchunk, CpmlK<T> P) {
  e3d_cpml_body<T, PERCELL, LZ>(ex, ey, ez, hx, hy, hz, cbx, cby, cbz, cb, nx, ny, nz, bx, by, bz, bu, xchunk,
                                blockIdx.x, blockIdx.y, blockIdx.z, P);
}

template <typename T, bool PERCELL, int LZ>
__global__ __launch_bounds__(64 * TY) void k_update_e3d_cpml_multi(
    T* __restrict__ ex, T* __restrict__ ey, T* __restrict__ ez, const T* __restrict__ hx,
    const T* __restrict__ hy, const T* __restrict__ hz, const T* __restrict__ cbx,
    const T* __restrict__ cby, const T* __restrict__ cbz, T cb, int nx, int ny, int nz, Win3 W,
    CpmlK<T> P) {
  int gbx, gby, gbz;
  const int w = win3_of(W, gbx, gby, gbz);
  e3d_cpml_body<T, PERCELL, LZ>(ex, ey, ez, hx, hy, hz, cbx, cby, cbz, cb, nx, ny, nz, W.bx[w], W.by[w], W.bz[w],
                                W.bu[w], W.xc[w], gbx, gby, gbz, P);
}

template <typename T, bool PERCELL, int LZ>
__device__ __forceinline__ void h3d_cpml_body(
    T* __restrict__ hx, T* __restrict__ hy, T* __restrict__ hz, const T* __restrict__ ex,
    const T* __restrict__ ey, const T* __restrict__ ez, const T* __restrict__ dbx,
    const T* __restrict__ dby, const T* __restrict__ dbz, T db, int nx, int ny, int nz, const Box3& bx, const Box3& by,
    const Box3& bz, const Box3& bu, int xchunk, int gbx, int gby, int gbz, const CpmlK<T>& P) {
  // LZ lanes per z row, 64 / LZ rows per wave (LZ < 64 for z-thin boxes)
  const int zl = threadIdx.x % LZ;
  const int kb = (bu.lo[2] & ~3) + 4 * (gbx * LZ + zl);
  const int j = bu.lo[1] + (gby * TY + threadIdx.y) * (64 / LZ) + threadIdx.x / LZ;
  const bool act = (kb < bu.hi[2]) && (j < bu.hi[1]);
  const bool ld_ok = (kb < nz) && (j < ny);
  const int i0 = bu.lo[0] + gbz * xchunk;
  const int i1 = min(i0 + xchunk, bu.hi[0]);
  const size_t plane = (size_t)ny * nz;
  const size_t row = ld_ok ? (size_t)j * nz + kb : 0;
  const unsigned mx = act ? kmask(bx, j, kb) : 0u;
  const unsigned my = act ? kmask(by, j, kb) : 0u;
  const unsigned mz = act ? kmask(bz, j, kb) : 0u;
  using V = typename Vec4<T>::type;
  V ey_c = bc4<T>(T(0)), ez_c = ey_c;
  if (ld_ok && i0 < i1) {
    ey_c = ld4(ey, (size_t)i0 * plane + row);
    ez_c = ld4(ez, (size_t)i0 * plane + row);
  }
  for (int i = i0; i < i1; ++i) {
    const size_t off = (size_t)i * plane + row;
    V exc = bc4<T>(T(0)), ey_n = exc, ez_n = exc;
    if (ld_ok) {
      exc = ld4(ex, off);
      if (i + 1 < nx) {
        ey_n = ld4(ey, off + plane);
        ez_n = ld4(ez, off + plane);
      }
    }
    T ey_k3 = __shfl_down(ey_c.x, 1, LZ);
    T ex_k3 = __shfl_down(exc.x, 1, LZ);
    if (zl == LZ - 1 && act && kb + 4 < nz) {
      ey_k3 = ey[off + 4];
      ex_k3 = ex[off + 4];
    }
    const unsigned ux = (i >= bx.lo[0] && i < bx.hi[0]) ? mx : 0u;
    const unsigned uy = (i >= by.lo[0] && i < by.hi[0]) ? my : 0u;
    const unsigned uz = (i >= bz.lo[0] && i < bz.hi[0]) ? mz : 0u;
    if (ux) {  // Hx: (Ey, z, +) (Ez, y, -)
      V h = ld4(hx, off);
      const V da = sub4(zp1(ey_c, ey_k3), ey_c);
      const V dd = sub4(ld4(ez, off + nz), ez_c);
      const V ca = cpml_term<2>(P.t[0][2], da, i, j, kb, ny, nz, ux);
      const V cb2 = cpml_term<1>(P.t[0][1], dd, i, j, kb, ny, nz, ux);
      const V c4 = PERCELL ? ld4(dbx, off) : bc4<T>(db);
      apply4(h, c4, comb(da, ca, dd, cb2), ux);
      st4m(hx, off, h, ux);
    }
    if (uy) {  // Hy: (Ez, x, +) (Ex, z, -)
      V h = ld4(hy, off);
      const V da = sub4(ez_n, ez_c);
      const V dd = sub4(zp1(exc, ex_k3), exc);
      const V ca = cpml_term<0>(P.t[1][0], da, i, j, kb, ny, nz, uy);
      const V cb2 = cpml_term<2>(P.t[1][2], dd, i, j, kb, ny, nz, uy);
      const V c4 = PERCELL ? ld4(dby, off) : bc4<T>(db);
      apply4(h, c4, comb(da, ca, dd, cb2), uy);
      st4m(hy, off, h, uy);
    }
    if (uz) {  // Hz: (Ex, y, +) (Ey, x, -)
      V h = ld4(hz, off);
      const V da = sub4(ld4(ex, off + nz), exc);
      const V dd = sub4(ey_n, ey_c);
      const V ca = cpml_term<1>(P.t[2][1], da, i, j, kb, ny, nz, uz);
      const V cb2 = cpml_term<0>(P.t[2][0], dd, i, j, kb, ny, nz, uz);
      const V c4 = PERCELL ? ld4(dbz, off) : bc4<T>(db);
      apply4(h, c4, comb(da, ca, dd, cb2), uz);
      st4m(hz, off, h, uz);
    }
    ey_c = ey_n;
    ez_c = ez_n;
  }
}

template <typename T, bool PERCELL, int LZ>
__global__ __launch_bounds__(64 * TY) void k_update_h3d_cpml_v4(
    T* __restrict__ hx, T* __restrict__ hy, T* __restrict__ hz, const T* __restrict__ ex,
    const T* __restrict__ ey, const T* __restrict__ ez, const T* __restrict__ dbx,
    const T* __restrict__ dby, const T* __restrict__ dbz, T db, int nx, int ny, int nz, Box3 bx,
    Box3 by, Box3 bz, Box3 bu, int xchunk, CpmlK<T> P) {
  h3d_cpml_body<T, PERCELL, LZ>(hx, hy, hz, ex, ey, ez, dbx, dby, dbz, db, nx, ny, nz, bx, by, bz, bu, xchunk,
                                blockIdx.x, blockIdx.y, blockIdx.z, P);
}

template <typename T, bool PERCELL, int LZ>
__global__ __launch_bounds__(64 * TY) void k_update_h3d_cpml_multi(
    T* __restrict__ hx, T* __restrict__ hy, T* __restrict__ hz, const T* __restrict__ ex,
    const T* __restrict__ ey, const T* __restrict__ ez, const T* __restrict__ dbx,
    const T* __restrict__ dby, const T* __restrict__ dbz, T db, int nx, int ny, int nz, Win3 W,
    CpmlK<T> P) {
  int gbx, gby, gbz;
  const int w = win3_of(W, gbx, gby, gbz);
  h3d_cpml_body<T, PERCELL, LZ>(hx, hy, hz, ex, ey, ez, dbx, dby, dbz, db, nx, ny, nz, W.bx[w], W.by[w], W.bz[w],
                                W.bu[w], W.xc[w], gbx, gby, gbz, P);
}

template <typename T>
CpmlK<T> make_cpml(const void* const* P, const int* I) {
  // per (component c, axis a): P[5 (3c + a) ..] = psi_lo psi_hi b c k; I[4 (3c + a) ..] = lo0 hi0 lo1 hi1
  CpmlK<T> K;
  for (int c = 0; c < 3; ++c)
    for (int a = 0; a < 3; ++a) {
      const int n = 3 * c + a;
      CpmlT<T>& t = K.t[c][a];
      t.psi[0] = (T*)P[5 * n];
      t.psi[1] = (T*)P[5 * n + 1];
      t.b = (const T*)P[5 * n + 2];
      t.c = (const T*)P[5 * n + 3];
      t.k = (const T*)P[5 * n + 4];
      t.lo[0] = I[4 * n];
      t.hi[0] = I[4 * n + 1];
      t.lo[1] = I[4 * n + 2];
      t.hi[1] = I[4 * n + 3];
    }
  return K;
}

// lanes per z row for a box: full 64-lane (256-cell) rows unless the box is
// z-thin (PML / shell slabs normal to z), where short rows stacked 64 / LZ
// per wave keep the lanes busy
inline int lanes_z(const Box3& bu) {
  const int kspan = bu.hi[2] - (bu.lo[2] & ~3);
  // the widest row layout whose padding wastes at most 15% of the lanes (a
  // 272-cell window row: 256-cell rows run 2 x 256 = 53% busy, 32-cell rows
  // 9 x 32 = 94%); thin rows fall through to the 32-cell layout
  for (int lz = 64; lz > 8; lz /= 4) {
    const int seg = 4 * lz;
    if (20 * kspan >= 17 * (cdiv(kspan, seg) * seg)) return lz;
  }
  return 8;
}

inline dim3 grid_c(const Box3& bu, int xchunk, int lz) {
  const int kspan = bu.hi[2] - (bu.lo[2] & ~3);
  return dim3(cdiv(kspan, 4 * lz), cdiv(bu.hi[1] - bu.lo[1], TY * (64 / lz)), cdiv(bu.hi[0] - bu.lo[0], xchunk));
}

// launch one split-kernel instantiation with the box's lane layout
#define LAUNCH_LZ(KERNEL, T, PC, ...)                                                          \
  do {                                                                                         \
    const int lz_ = lanes_z(bu);                                                               \
    if (lz_ == 8)                                                                              \
      KERNEL<T, PC, 8><<<grid_c(bu, xchunk, 8), dim3(64, TY), 0, (hipStream_t)s>>>(__VA_ARGS__);   \
    else if (lz_ == 16)                                                                        \
      KERNEL<T, PC, 16><<<grid_c(bu, xchunk, 16), dim3(64, TY), 0, (hipStream_t)s>>>(__VA_ARGS__); \
    else                                                                                       \
      KERNEL<T, PC, 64><<<grid_c(bu, xchunk, 64), dim3(64, TY), 0, (hipStream_t)s>>>(__VA_ARGS__); \
  } while (0)

template <typename T>
int launch_cpml_e(T* ex, T* ey, T* ez, const T* hx, const T* hy, const T* hz, const T* cbx, const T* cby,
                  const T* cbz, double cb, int nx, int ny, int nz, const int* boxes, int xchunk,
                  const void* const* cp, const int* ci, void* s) {
  if (nz % 4 != 0) return (int)hipErrorInvalidValue;
  Box3 bx = make_box(boxes), by = make_box(boxes + 6), bz = make_box(boxes + 12);
  Box3 bu = box_union(box_union(bx, by), bz);
  if (box_empty(bu)) return 0;
  {
    const dim3 g1 = grid_c(bu, 1, lanes_z(bu));
    xchunk = split_xchunk(bu.hi[0] - bu.lo[0], (long long)g1.x * g1.y, xchunk);
  }
  const CpmlK<T> K = make_cpml<T>(cp, ci);
  if (cbx)
    LAUNCH_LZ(k_update_e3d_cpml_v4, T, true, ex, ey, ez, hx, hy, hz, cbx, cby, cbz, (T)cb, nx, ny, nz, bx, by, bz, bu, xchunk, K);
  else
    LAUNCH_LZ(k_update_e3d_cpml_v4, T, false, ex, ey, ez, hx, hy, hz, cbx, cby, cbz, (T)cb, nx, ny, nz, bx, by, bz, bu, xchunk, K);
  FDTD_RETURN_LAUNCH_STATUS();
}

template <typename T>
int launch_cpml_h(T* hx, T* hy, T* hz, const T* ex, const T* ey, const T* ez, const T* dbx, const T* dby,
                  const T* dbz, double db, int nx, int ny, int nz, const int* boxes, int xchunk,
                  const void* const* cp, const int* ci, void* s) {
  if (nz % 4 != 0) return (int)hipErrorInvalidValue;
  Box3 bx = make_box(boxes), by = make_box(boxes + 6), bz = make_box(boxes + 12);
  Box3 bu = box_union(box_union(bx, by), bz);
  if (box_empty(bu)) return 0;
  {
    const dim3 g1 = grid_c(bu, 1, lanes_z(bu));
    xchunk = split_xchunk(bu.hi[0] - bu.lo[0], (long long)g1.x * g1.y, xchunk);
  }
  const CpmlK<T> K = make_cpml<T>(cp, ci);
  if (dbx)
    LAUNCH_LZ(k_update_h3d_cpml_v4, T, true, hx, hy, hz, ex, ey, ez, dbx, dby, dbz, (T)db, nx, ny, nz, bx, by, bz, bu, xchunk, K);
  else
    LAUNCH_LZ(k_update_h3d_cpml_v4, T, false, hx, hy, hz, ex, ey, ez, dbx, dby, dbz, (T)db, nx, ny, nz, bx, by, bz, bu, xchunk, K);
  FDTD_RETURN_LAUNCH_STATUS();
}

// the windows of one half step (boxes: 18 ints per window, the component
// boxes) grouped by row layout, up to MAXW3 per launch
template <typename T, bool KE>
int launch_cpml_multi(T* f0, T* f1, T* f2, const T* g0, const T* g1, const T* g2, const T* c0, const T* c1,
                      const T* c2, double cf, int nx, int ny, int nz, const int* boxes, int nwin,
                      const void* const* cp, const int* ci, void* s) {
  if (nz % 4 != 0 || nwin < 0) return (int)hipErrorInvalidValue;
  const CpmlK<T> K = make_cpml<T>(cp, ci);
  const bool pc = c0 != nullptr;
  const hipStream_t st = (hipStream_t)s;
  for (int lz : {64, 16, 8}) {
    Win3 W;
    W.n = 0;
    int total = 0;
    auto flush = [&]() {
      if (W.n == 0) return;
      W.start[W.n] = total;
      for (int q = W.n + 1; q <= MAXW3; ++q) W.start[q] = total;
      const dim3 g((unsigned)total), b(64, TY);
#define CPML_MULTI(LZ)                                                                                          \
  if (KE) {                                                                                                     \
    if (pc)                                                                                                     \
      k_update_e3d_cpml_multi<T, true, LZ><<<g, b, 0, st>>>(f0, f1, f2, g0, g1, g2, c0, c1, c2, (T)cf, nx, ny, nz, W, K); \
    else                                                                                                        \
      k_update_e3d_cpml_multi<T, false, LZ><<<g, b, 0, st>>>(f0, f1, f2, g0, g1, g2, c0, c1, c2, (T)cf, nx, ny, nz, W, K); \
  } else {                                                                                                      \
    if (pc)                                                                                                     \
      k_update_h3d_cpml_multi<T, true, LZ><<<g, b, 0, st>>>(f0, f1, f2, g0, g1, g2, c0, c1, c2, (T)cf, nx, ny, nz, W, K); \
    else                                                                                                        \
      k_update_h3d_cpml_multi<T, false, LZ><<<g, b, 0, st>>>(f0, f1, f2, g0, g1, g2, c0, c1, c2, (T)cf, nx, ny, nz, W, K); \
  }
      if (lz == 64) {
        CPML_MULTI(64)
      } else if (lz == 16) {
        CPML_MULTI(16)
      } else {
        CPML_MULTI(8)
      }
#undef CPML_MULTI
      W.n = 0;
      total = 0;
    };
    for (int q = 0; q < nwin; ++q) {
      const Box3 bx = make_box(boxes + 18 * q), by = make_box(boxes + 18 * q + 6), bz = make_box(boxes + 18 * q + 12);
      const Box3 bu = box_union(box_union(bx, by), bz);
      if (box_empty(bu) || lanes_z(bu) != lz) continue;
      const dim3 g1 = grid_c(bu, 1, lz);
      const int xc = split_xchunk(bu.hi[0] - bu.lo[0], (long long)g1.x * g1.y, 0);
      const dim3 g = grid_c(bu, xc, lz);
      const int n = W.n;
      W.bx[n] = bx;
      W.by[n] = by;
      W.bz[n] = bz;
      W.bu[n] = bu;
      W.xc[n] = xc;
      W.gx[n] = (int)g.x;
      W.gy[n] = (int)g.y;
      W.start[n] = total;
      total += (int)(g.x * g.y * g.z);
      W.n = n + 1;
      if (W.n == MAXW3) flush();
    }
    flush();
  }
  FDTD_RETURN_LAUNCH_STATUS();
}

}  // namespace

// Same arguments as fdtd_update_{e,h}3d_v4_f32 plus the CPML term table
// (9 entries, [component][axis]): cp = 5 pointers each, ci = 4 ints each.
// _f64: the same kernels on 4-cell double groups (32-byte lanes).
#define FDTD_CPML_V4_API(SUF, T)                                                                               \
  FDTD_API int fdtd_update_e3d_cpml_v4_##SUF(T* ex, T* ey, T* ez, const T* hx, const T* hy, const T* hz,       \
                                             const T* cbx, const T* cby, const T* cbz, double cb, int nx,      \
                                             int ny, int nz, const int* boxes, int xchunk,                     \
                                             const void* const* cp, const int* ci, void* s) {                  \
    return launch_cpml_e<T>(ex, ey, ez, hx, hy, hz, cbx, cby, cbz, cb, nx, ny, nz, boxes, xchunk, cp, ci, s); \
  }                                                                                                            \
  FDTD_API int fdtd_update_h3d_cpml_v4_##SUF(T* hx, T* hy, T* hz, const T* ex, const T* ey, const T* ez,       \
                                             const T* dbx, const T* dby, const T* dbz, double db, int nx,      \
                                             int ny, int nz, const int* boxes, int xchunk,                     \
                                             const void* const* cp, const int* ci, void* s) {                  \
    return launch_cpml_h<T>(hx, hy, hz, ex, ey, ez, dbx, dby, dbz, db, nx, ny, nz, boxes, xchunk, cp, ci, s); \
  }
FDTD_CPML_V4_API(f32, float)
FDTD_CPML_V4_API(f64, double)

// The split CPML updates of several disjoint windows in one launch per row
// layout (the hybrid shell's windows of a half step): ``boxes`` = 18 ints per
// window (the three component boxes), ``nwin`` windows; other arguments as
// fdtd_update_{e,h}3d_cpml_v4_*.
#define FDTD_CPML_MULTI_API(SUF, T)                                                                          \
  FDTD_API int fdtd_update_e3d_cpml_multi_##SUF(T* ex, T* ey, T* ez, const T* hx, const T* hy, const T* hz,  \
                                                const T* cbx, const T* cby, const T* cbz, double cb, int nx, \
                                                int ny, int nz, const int* boxes, int nwin,                  \
                                                const void* const* cp, const int* ci, void* s) {             \
    return launch_cpml_multi<T, true>(ex, ey, ez, hx, hy, hz, cbx, cby, cbz, cb, nx, ny, nz, boxes, nwin, cp,  \
                                      ci, s);                                                                \
  }                                                                                                          \
  FDTD_API int fdtd_update_h3d_cpml_multi_##SUF(T* hx, T* hy, T* hz, const T* ex, const T* ey, const T* ez,  \
                                                const T* dbx, const T* dby, const T* dbz, double db, int nx, \
                                                int ny, int nz, const int* boxes, int nwin,                  \
                                                const void* const* cp, const int* ci, void* s) {             \
    return launch_cpml_multi<T, false>(hx, hy, hz, ex, ey, ez, dbx, dby, dbz, db, nx, ny, nz, boxes, nwin, cp, \
                                       ci, s);                                                               \
  }
FDTD_CPML_MULTI_API(f32, float)
FDTD_CPML_MULTI_API(f64, double)
