// fp32 float4 3D Yee half-step kernels with the CPML folded in.
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

struct CpmlT {          // one curl term of one component
  float* psi[2];        // low / high slab (nullptr: no slab on that side)
  int lo[2], hi[2];     // slab range along the term axis (local index)
  const float* b;       // profiles along the axis (identity outside the slabs)
  const float* c;
  const float* k;       // 1/kappa - 1
};

struct CpmlK {
  CpmlT t[3][3];        // [component][term axis] (diagonal unused)
};

__device__ __forceinline__ float4 sub4(const float4& a, const float4& b) {
  return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
}

__device__ __forceinline__ float4 zm1(const float4& v, float s) { return make_float4(s, v.x, v.y, v.z); }
__device__ __forceinline__ float4 zp1(const float4& v, float s) { return make_float4(v.y, v.z, v.w, s); }

// CPML contribution of one term (without the term sign) for the lane's 4 cells
template <int AXIS>
__device__ __forceinline__ float4 cpml_term(const CpmlT& t, const float4& d, int i, int j, int kb, int ny, int nz,
                                            unsigned mask) {
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (AXIS < 2) {
    const int n = AXIS == 0 ? i : j;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (t.psi[s] && n >= t.lo[s] && n < t.hi[s]) {
        const int w = t.hi[s] - t.lo[s];
        const size_t po = AXIS == 0 ? ((size_t)(n - t.lo[s]) * ny + j) * nz + kb
                                    : ((size_t)i * w + (n - t.lo[s])) * nz + kb;
        const float bn = t.b[n], cn = t.c[n], kn = t.k[n];
        float4 p = ld4(t.psi[s], po);
        p = make_float4(bn * p.x + cn * d.x, bn * p.y + cn * d.y, bn * p.z + cn * d.z, bn * p.w + cn * d.w);
        if (mask == 0xFu) {
          st4(t.psi[s], po, p);
        } else {
          st4m(t.psi[s], po, p, mask);
        }
        r = make_float4(kn * d.x + p.x, kn * d.y + p.y, kn * d.z + p.z, kn * d.w + p.w);
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
        const float4 bn = ld4(t.b, kb), cn = ld4(t.c, kb), kn = ld4(t.k, kb);
        float4 p = ld4(t.psi[s], po);
        p = make_float4(bn.x * p.x + cn.x * d.x, bn.y * p.y + cn.y * d.y, bn.z * p.z + cn.z * d.z,
                        bn.w * p.w + cn.w * d.w);
        st4m(t.psi[s], po, p, mask);
        r = make_float4(kn.x * d.x + p.x, kn.y * d.y + p.y, kn.z * d.z + p.z, kn.w * d.w + p.w);
      }
    }
  }
  return r;
}

// F += c * (sa*da + sb*db + sa*corr_a + sb*corr_b) on the masked elements
__device__ __forceinline__ void apply4(float4& f, const float4& c, const float4& v, unsigned m) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (m & (1u << q)) f4set(f, q, f4(f, q) + f4(c, q) * f4(v, q));
}

__device__ __forceinline__ float4 comb(const float4& da, const float4& ca, const float4& db, const float4& cb_) {
  // (da + ca) - (db + cb): term a has sign +1, term b sign -1 (CURL_TERMS)
  return make_float4((da.x + ca.x) - (db.x + cb_.x), (da.y + ca.y) - (db.y + cb_.y), (da.z + ca.z) - (db.z + cb_.z),
                     (da.w + ca.w) - (db.w + cb_.w));
}

template <bool PERCELL, int LZ>
__global__ __launch_bounds__(64 * TY) void k_update_e3d_cpml_v4(
    float* __restrict__ ex, float* __restrict__ ey, float* __restrict__ ez, const float* __restrict__ hx,
    const float* __restrict__ hy, const float* __restrict__ hz, const float* __restrict__ cbx,
    const float* __restrict__ cby, const float* __restrict__ cbz, float cb, int nx, int ny, int nz, Box3 bx,
    Box3 by, Box3 bz, Box3 bu, int xchunk, CpmlK P) {
  // LZ lanes per z row, 64 / LZ rows per wave (LZ < 64 for z-thin boxes)
  const int zl = threadIdx.x % LZ;
  const int kb = (bu.lo[2] & ~3) + 4 * (blockIdx.x * LZ + zl);
  const int j = bu.lo[1] + (blockIdx.y * TY + threadIdx.y) * (64 / LZ) + threadIdx.x / LZ;
  const bool act = (kb < bu.hi[2]) && (j < bu.hi[1]);
  const int i0 = bu.lo[0] + blockIdx.z * xchunk;
  const int i1 = min(i0 + xchunk, bu.hi[0]);
  const size_t plane = (size_t)ny * nz;
  const size_t row = act ? (size_t)j * nz + kb : 0;
  const unsigned mx = act ? kmask(bx, j, kb) : 0u;
  const unsigned my = act ? kmask(by, j, kb) : 0u;
  const unsigned mz = act ? kmask(bz, j, kb) : 0u;
  float4 hz_m = make_float4(0, 0, 0, 0), hy_m = hz_m;
  if (act && i0 > 0 && (my | mz)) {
    hz_m = ld4(hz, (size_t)(i0 - 1) * plane + row);
    hy_m = ld4(hy, (size_t)(i0 - 1) * plane + row);
  }
  for (int i = i0; i < i1; ++i) {
    const size_t off = (size_t)i * plane + row;
    float4 hxc = make_float4(0, 0, 0, 0), hyc = hxc, hzc = hxc;
    if (act) {
      hxc = ld4(hx, off);
      hyc = ld4(hy, off);
      hzc = ld4(hz, off);
    }
    float hy_k0 = __shfl_up(hyc.w, 1, LZ);
    float hx_k0 = __shfl_up(hxc.w, 1, LZ);
    if (zl == 0 && act && kb > 0) {
      hy_k0 = hy[off - 1];
      hx_k0 = hx[off - 1];
    }
    const unsigned ux = (i >= bx.lo[0] && i < bx.hi[0]) ? mx : 0u;
    const unsigned uy = (i >= by.lo[0] && i < by.hi[0]) ? my : 0u;
    const unsigned uz = (i >= bz.lo[0] && i < bz.hi[0]) ? mz : 0u;
    if (ux) {  // Ex: (Hz, y, +) (Hy, z, -)
      float4 e = ld4(ex, off);
      const float4 da = sub4(hzc, ld4(hz, off - nz));
      const float4 db = sub4(hyc, zm1(hyc, hy_k0));
      const float4 ca = cpml_term<1>(P.t[0][1], da, i, j, kb, ny, nz, ux);
      const float4 cb2 = cpml_term<2>(P.t[0][2], db, i, j, kb, ny, nz, ux);
      const float4 c4 = PERCELL ? ld4(cbx, off) : make_float4(cb, cb, cb, cb);
      apply4(e, c4, comb(da, ca, db, cb2), ux);
      st4m(ex, off, e, ux);
    }
    if (uy) {  // Ey: (Hx, z, +) (Hz, x, -)
      float4 e = ld4(ey, off);
      const float4 da = sub4(hxc, zm1(hxc, hx_k0));
      const float4 db = sub4(hzc, hz_m);
      const float4 ca = cpml_term<2>(P.t[1][2], da, i, j, kb, ny, nz, uy);
      const float4 cb2 = cpml_term<0>(P.t[1][0], db, i, j, kb, ny, nz, uy);
      const float4 c4 = PERCELL ? ld4(cby, off) : make_float4(cb, cb, cb, cb);
      apply4(e, c4, comb(da, ca, db, cb2), uy);
      st4m(ey, off, e, uy);
    }
    if (uz) {  // Ez: (Hy, x, +) (Hx, y, -)
      float4 e = ld4(ez, off);
      const float4 da = sub4(hyc, hy_m);
      const float4 db = sub4(hxc, ld4(hx, off - nz));
      const float4 ca = cpml_term<0>(P.t[2][0], da, i, j, kb, ny, nz, uz);
      const float4 cb2 = cpml_term<1>(P.t[2][1], db, i, j, kb, ny, nz, uz);
      const float4 c4 = PERCELL ? ld4(cbz, off) : make_float4(cb, cb, cb, cb);
      apply4(e, c4, comb(da, ca, db, cb2), uz);
      st4m(ez, off, e, uz);
    }
    hz_m = hzc;
    hy_m = hyc;
  }
}

template <bool PERCELL, int LZ>
__global__ __launch_bounds__(64 * TY) void k_update_h3d_cpml_v4(
    float* __restrict__ hx, float* __restrict__ hy, float* __restrict__ hz, const float* __restrict__ ex,
    const float* __restrict__ ey, const float* __restrict__ ez, const float* __restrict__ dbx,
    const float* __restrict__ dby, const float* __restrict__ dbz, float db, int nx, int ny, int nz, Box3 bx,
    Box3 by, Box3 bz, Box3 bu, int xchunk, CpmlK P) {
  // LZ lanes per z row, 64 / LZ rows per wave (LZ < 64 for z-thin boxes)
  const int zl = threadIdx.x % LZ;
  const int kb = (bu.lo[2] & ~3) + 4 * (blockIdx.x * LZ + zl);
  const int j = bu.lo[1] + (blockIdx.y * TY + threadIdx.y) * (64 / LZ) + threadIdx.x / LZ;
  const bool act = (kb < bu.hi[2]) && (j < bu.hi[1]);
  const bool ld_ok = (kb < nz) && (j < ny);
  const int i0 = bu.lo[0] + blockIdx.z * xchunk;
  const int i1 = min(i0 + xchunk, bu.hi[0]);
  const size_t plane = (size_t)ny * nz;
  const size_t row = ld_ok ? (size_t)j * nz + kb : 0;
  const unsigned mx = act ? kmask(bx, j, kb) : 0u;
  const unsigned my = act ? kmask(by, j, kb) : 0u;
  const unsigned mz = act ? kmask(bz, j, kb) : 0u;
  float4 ey_c = make_float4(0, 0, 0, 0), ez_c = ey_c;
  if (ld_ok && i0 < i1) {
    ey_c = ld4(ey, (size_t)i0 * plane + row);
    ez_c = ld4(ez, (size_t)i0 * plane + row);
  }
  for (int i = i0; i < i1; ++i) {
    const size_t off = (size_t)i * plane + row;
    float4 exc = make_float4(0, 0, 0, 0), ey_n = exc, ez_n = exc;
    if (ld_ok) {
      exc = ld4(ex, off);
      if (i + 1 < nx) {
        ey_n = ld4(ey, off + plane);
        ez_n = ld4(ez, off + plane);
      }
    }
    float ey_k3 = __shfl_down(ey_c.x, 1, LZ);
    float ex_k3 = __shfl_down(exc.x, 1, LZ);
    if (zl == LZ - 1 && act && kb + 4 < nz) {
      ey_k3 = ey[off + 4];
      ex_k3 = ex[off + 4];
    }
    const unsigned ux = (i >= bx.lo[0] && i < bx.hi[0]) ? mx : 0u;
    const unsigned uy = (i >= by.lo[0] && i < by.hi[0]) ? my : 0u;
    const unsigned uz = (i >= bz.lo[0] && i < bz.hi[0]) ? mz : 0u;
    if (ux) {  // Hx: (Ey, z, +) (Ez, y, -)
      float4 h = ld4(hx, off);
      const float4 da = sub4(zp1(ey_c, ey_k3), ey_c);
      const float4 dd = sub4(ld4(ez, off + nz), ez_c);
      const float4 ca = cpml_term<2>(P.t[0][2], da, i, j, kb, ny, nz, ux);
      const float4 cb2 = cpml_term<1>(P.t[0][1], dd, i, j, kb, ny, nz, ux);
      const float4 c4 = PERCELL ? ld4(dbx, off) : make_float4(db, db, db, db);
      apply4(h, c4, comb(da, ca, dd, cb2), ux);
      st4m(hx, off, h, ux);
    }
    if (uy) {  // Hy: (Ez, x, +) (Ex, z, -)
      float4 h = ld4(hy, off);
      const float4 da = sub4(ez_n, ez_c);
      const float4 dd = sub4(zp1(exc, ex_k3), exc);
      const float4 ca = cpml_term<0>(P.t[1][0], da, i, j, kb, ny, nz, uy);
      const float4 cb2 = cpml_term<2>(P.t[1][2], dd, i, j, kb, ny, nz, uy);
      const float4 c4 = PERCELL ? ld4(dby, off) : make_float4(db, db, db, db);
      apply4(h, c4, comb(da, ca, dd, cb2), uy);
      st4m(hy, off, h, uy);
    }
    if (uz) {  // Hz: (Ex, y, +) (Ey, x, -)
      float4 h = ld4(hz, off);
      const float4 da = sub4(ld4(ex, off + nz), exc);
      const float4 dd = sub4(ey_n, ey_c);
      const float4 ca = cpml_term<1>(P.t[2][1], da, i, j, kb, ny, nz, uz);
      const float4 cb2 = cpml_term<0>(P.t[2][0], dd, i, j, kb, ny, nz, uz);
      const float4 c4 = PERCELL ? ld4(dbz, off) : make_float4(db, db, db, db);
      apply4(h, c4, comb(da, ca, dd, cb2), uz);
      st4m(hz, off, h, uz);
    }
    ey_c = ey_n;
    ez_c = ez_n;
  }
}

CpmlK make_cpml(const void* const* P, const int* I) {
  // per (component c, axis a): P[5 (3c + a) ..] = psi_lo psi_hi b c k; I[4 (3c + a) ..] = lo0 hi0 lo1 hi1
  CpmlK K;
  for (int c = 0; c < 3; ++c)
    for (int a = 0; a < 3; ++a) {
      const int n = 3 * c + a;
      CpmlT& t = K.t[c][a];
      t.psi[0] = (float*)P[5 * n];
      t.psi[1] = (float*)P[5 * n + 1];
      t.b = (const float*)P[5 * n + 2];
      t.c = (const float*)P[5 * n + 3];
      t.k = (const float*)P[5 * n + 4];
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
#define LAUNCH_LZ(KERNEL, PC, ...)                                                          \
  do {                                                                                      \
    const int lz_ = lanes_z(bu);                                                            \
    if (lz_ == 8)                                                                           \
      KERNEL<PC, 8><<<grid_c(bu, xchunk, 8), dim3(64, TY), 0, (hipStream_t)s>>>(__VA_ARGS__);   \
    else if (lz_ == 16)                                                                     \
      KERNEL<PC, 16><<<grid_c(bu, xchunk, 16), dim3(64, TY), 0, (hipStream_t)s>>>(__VA_ARGS__); \
    else                                                                                    \
      KERNEL<PC, 64><<<grid_c(bu, xchunk, 64), dim3(64, TY), 0, (hipStream_t)s>>>(__VA_ARGS__); \
  } while (0)

}  // namespace

// Same arguments as fdtd_update_{e,h}3d_v4_f32 plus the CPML term table
// (9 entries, [component][axis]): cp = 5 pointers each, ci = 4 ints each.
FDTD_API int fdtd_update_e3d_cpml_v4_f32(float* ex, float* ey, float* ez, const float* hx, const float* hy,
                                         const float* hz, const float* cbx, const float* cby, const float* cbz,
                                         double cb, int nx, int ny, int nz, const int* boxes, int xchunk,
                                         const void* const* cp, const int* ci, void* s) {
  if (nz % 4 != 0) return (int)hipErrorInvalidValue;
  Box3 bx = make_box(boxes), by = make_box(boxes + 6), bz = make_box(boxes + 12);
  Box3 bu = box_union(box_union(bx, by), bz);
  if (box_empty(bu)) return 0;
  {
    const dim3 g1 = grid_c(bu, 1, lanes_z(bu));
    xchunk = split_xchunk(bu.hi[0] - bu.lo[0], (long long)g1.x * g1.y, xchunk);
  }
  const CpmlK K = make_cpml(cp, ci);
  if (cbx)
    LAUNCH_LZ(k_update_e3d_cpml_v4, true, ex, ey, ez, hx, hy, hz, cbx, cby, cbz, (float)cb, nx, ny, nz, bx, by, bz, bu, xchunk, K);
  else
    LAUNCH_LZ(k_update_e3d_cpml_v4, false, ex, ey, ez, hx, hy, hz, cbx, cby, cbz, (float)cb, nx, ny, nz, bx, by, bz, bu, xchunk, K);
  FDTD_RETURN_LAUNCH_STATUS();
}

FDTD_API int fdtd_update_h3d_cpml_v4_f32(float* hx, float* hy, float* hz, const float* ex, const float* ey,
                                         const float* ez, const float* dbx, const float* dby, const float* dbz,
                                         double db, int nx, int ny, int nz, const int* boxes, int xchunk,
                                         const void* const* cp, const int* ci, void* s) {
  if (nz % 4 != 0) return (int)hipErrorInvalidValue;
  Box3 bx = make_box(boxes), by = make_box(boxes + 6), bz = make_box(boxes + 12);
  Box3 bu = box_union(box_union(bx, by), bz);
  if (box_empty(bu)) return 0;
  {
    const dim3 g1 = grid_c(bu, 1, lanes_z(bu));
    xchunk = split_xchunk(bu.hi[0] - bu.lo[0], (long long)g1.x * g1.y, xchunk);
  }
  const CpmlK K = make_cpml(cp, ci);
  if (dbx)
    LAUNCH_LZ(k_update_h3d_cpml_v4, true, hx, hy, hz, ex, ey, ez, dbx, dby, dbz, (float)db, nx, ny, nz, bx, by, bz, bu, xchunk, K);
  else
    LAUNCH_LZ(k_update_h3d_cpml_v4, false, hx, hy, hz, ex, ey, ez, dbx, dby, dbz, (float)db, nx, ny, nz, bx, by, bz, bu, xchunk, K);
  FDTD_RETURN_LAUNCH_STATUS();
}
