// fp32 3D Yee kernels with 16-byte (float4) lanes.
//
// Same arithmetic and boxes as yee3d.hip, but every lane owns four
// consecutive z cells: one global_load_dwordx4 per field per plane, so a wave
// moves 1 KiB per load instruction (cdna_hip_programming.md Guideline 13) and
// keeps 4x more bytes in flight per instruction -- the HBM3E stream needs
// ~50 KB in flight per CU.  The z-1 (E) / z+1 (H) neighbour of the edge
// element comes from the adjacent lane through a cross-lane shuffle; only the
// wave's first (last) lane issues one scalar load for the cell outside the
// 256-cell row.  Requires nz % 4 == 0 (host checks); rows are then 16-byte
// aligned because torch allocations are 256-byte aligned.

#include "common.h"

namespace {

constexpr int TY = 4;

struct KMask {
  // per-component bit e set when element e of the lane's 4-group is inside the box
  unsigned m[3];
};

__device__ __forceinline__ unsigned kmask(const Box3& b, int j, int kb) {
  if (j < b.lo[1] || j >= b.hi[1]) return 0u;
  unsigned m = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) m |= ((kb + e >= b.lo[2]) && (kb + e < b.hi[2])) ? (1u << e) : 0u;
  return m;
}

__device__ __forceinline__ float f4(const float4& v, int e) {
  return e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w));
}

__device__ __forceinline__ void f4set(float4& v, int e, float s) {
  if (e == 0) v.x = s;
  else if (e == 1) v.y = s;
  else if (e == 2) v.z = s;
  else v.w = s;
}

__device__ __forceinline__ float4 ld4(const float* p, size_t off) {
  return *reinterpret_cast<const float4*>(p + off);
}

__device__ __forceinline__ void st4(float* p, size_t off, const float4& v) {
  *reinterpret_cast<float4*>(p + off) = v;
}

template <bool PERCELL>
__global__ __launch_bounds__(64 * TY) void k_update_e3d_v4(
    float* __restrict__ ex, float* __restrict__ ey, float* __restrict__ ez,
    const float* __restrict__ hx, const float* __restrict__ hy, const float* __restrict__ hz,
    const float* __restrict__ cbx, const float* __restrict__ cby, const float* __restrict__ cbz,
    float cb, int nx, int ny, int nz, Box3 bx, Box3 by, Box3 bz, Box3 bu, int xchunk) {
  const int lane = threadIdx.x;
  const int kb = (bu.lo[2] & ~3) + 4 * (blockIdx.x * 64 + lane);
  const int j = bu.lo[1] + blockIdx.y * TY + threadIdx.y;
  const bool act = (kb < bu.hi[2]) && (j < bu.hi[1]);
  const int i0 = bu.lo[0] + blockIdx.z * xchunk;
  const int i1 = min(i0 + xchunk, bu.hi[0]);
  const size_t plane = (size_t)ny * nz;
  const size_t row = (size_t)j * nz + kb;
  const unsigned mx = act ? kmask(bx, j, kb) : 0u;
  const unsigned my = act ? kmask(by, j, kb) : 0u;
  const unsigned mz = act ? kmask(bz, j, kb) : 0u;
  float4 hz_m = make_float4(0, 0, 0, 0), hy_m = make_float4(0, 0, 0, 0);
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
    // z-1 neighbours of element 0 (previous lane's element 3)
    float hy_k0 = __shfl_up(hyc.w, 1, 64);
    float hx_k0 = __shfl_up(hxc.w, 1, 64);
    if (lane == 0 && act && kb > 0) {
      hy_k0 = hy[off - 1];
      hx_k0 = hx[off - 1];
    }
    const bool xin_x = i >= bx.lo[0] && i < bx.hi[0];
    const bool xin_y = i >= by.lo[0] && i < by.hi[0];
    const bool xin_z = i >= bz.lo[0] && i < bz.hi[0];
    if (xin_x && mx) {
      float4 e = ld4(ex, off);
      const float4 hz_j = ld4(hz, off - nz);
      const float4 c4 = PERCELL ? ld4(cbx, off) : make_float4(cb, cb, cb, cb);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (mx & (1u << q)) {
          const float hym = q == 0 ? hy_k0 : f4(hyc, q - 1);
          f4set(e, q, f4(e, q) + f4(c4, q) * ((f4(hzc, q) - f4(hz_j, q)) - (f4(hyc, q) - hym)));
        }
      }
      st4(ex, off, e);
    }
    if (xin_y && my) {
      float4 e = ld4(ey, off);
      const float4 c4 = PERCELL ? ld4(cby, off) : make_float4(cb, cb, cb, cb);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (my & (1u << q)) {
          const float hxm = q == 0 ? hx_k0 : f4(hxc, q - 1);
          f4set(e, q, f4(e, q) + f4(c4, q) * ((f4(hxc, q) - hxm) - (f4(hzc, q) - f4(hz_m, q))));
        }
      }
      st4(ey, off, e);
    }
    if (xin_z && mz) {
      float4 e = ld4(ez, off);
      const float4 hx_j = ld4(hx, off - nz);
      const float4 c4 = PERCELL ? ld4(cbz, off) : make_float4(cb, cb, cb, cb);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (mz & (1u << q)) {
          f4set(e, q, f4(e, q) + f4(c4, q) * ((f4(hyc, q) - f4(hy_m, q)) - (f4(hxc, q) - f4(hx_j, q))));
        }
      }
      st4(ez, off, e);
    }
    hz_m = hzc;
    hy_m = hyc;
  }
}

template <bool PERCELL>
__global__ __launch_bounds__(64 * TY) void k_update_h3d_v4(
    float* __restrict__ hx, float* __restrict__ hy, float* __restrict__ hz,
    const float* __restrict__ ex, const float* __restrict__ ey, const float* __restrict__ ez,
    const float* __restrict__ dbx, const float* __restrict__ dby, const float* __restrict__ dbz,
    float db, int nx, int ny, int nz, Box3 bx, Box3 by, Box3 bz, Box3 bu, int xchunk) {
  const int lane = threadIdx.x;
  const int kb = (bu.lo[2] & ~3) + 4 * (blockIdx.x * 64 + lane);
  const int j = bu.lo[1] + blockIdx.y * TY + threadIdx.y;
  const bool act = (kb < bu.hi[2]) && (j < bu.hi[1]);
  const bool ld_ok = (kb < nz) && (j < ny);  // lanes past the box still feed their z-1 neighbour
  const int i0 = bu.lo[0] + blockIdx.z * xchunk;
  const int i1 = min(i0 + xchunk, bu.hi[0]);
  const size_t plane = (size_t)ny * nz;
  const size_t row = (size_t)j * nz + kb;
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
    // z+1 neighbours of element 3 (next lane's element 0)
    float ey_k3 = __shfl_down(ey_c.x, 1, 64);
    float ex_k3 = __shfl_down(exc.x, 1, 64);
    if (lane == 63 && act && kb + 4 < nz) {
      ey_k3 = ey[off + 4];
      ex_k3 = ex[off + 4];
    }
    const bool xin_x = i >= bx.lo[0] && i < bx.hi[0];
    const bool xin_y = i >= by.lo[0] && i < by.hi[0];
    const bool xin_z = i >= bz.lo[0] && i < bz.hi[0];
    if (xin_x && mx) {
      float4 h = ld4(hx, off);
      const float4 ez_j = ld4(ez, off + nz);
      const float4 c4 = PERCELL ? ld4(dbx, off) : make_float4(db, db, db, db);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (mx & (1u << q)) {
          const float eyp = q == 3 ? ey_k3 : f4(ey_c, q + 1);
          f4set(h, q, f4(h, q) + f4(c4, q) * ((eyp - f4(ey_c, q)) - (f4(ez_j, q) - f4(ez_c, q))));
        }
      }
      st4(hx, off, h);
    }
    if (xin_y && my) {
      float4 h = ld4(hy, off);
      const float4 c4 = PERCELL ? ld4(dby, off) : make_float4(db, db, db, db);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (my & (1u << q)) {
          const float exp_ = q == 3 ? ex_k3 : f4(exc, q + 1);
          f4set(h, q, f4(h, q) + f4(c4, q) * ((f4(ez_n, q) - f4(ez_c, q)) - (exp_ - f4(exc, q))));
        }
      }
      st4(hy, off, h);
    }
    if (xin_z && mz) {
      float4 h = ld4(hz, off);
      const float4 ex_j = ld4(ex, off + nz);
      const float4 c4 = PERCELL ? ld4(dbz, off) : make_float4(db, db, db, db);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (mz & (1u << q)) {
          f4set(h, q, f4(h, q) + f4(c4, q) * ((f4(ex_j, q) - f4(exc, q)) - (f4(ey_n, q) - f4(ey_c, q))));
        }
      }
      st4(hz, off, h);
    }
    ey_c = ey_n;
    ez_c = ez_n;
  }
}

inline dim3 grid_v4(const Box3& bu, int xchunk) {
  const int kspan = bu.hi[2] - (bu.lo[2] & ~3);
  return dim3(cdiv(kspan, 256), cdiv(bu.hi[1] - bu.lo[1], TY), cdiv(bu.hi[0] - bu.lo[0], xchunk));
}

}  // namespace

FDTD_API int fdtd_update_e3d_v4_f32(float* ex, float* ey, float* ez, const float* hx, const float* hy,
                                    const float* hz, const float* cbx, const float* cby, const float* cbz,
                                    double cb, int nx, int ny, int nz, const int* boxes, int xchunk, void* s) {
  if (nz % 4 != 0) return (int)hipErrorInvalidValue;
  Box3 bx = make_box(boxes), by = make_box(boxes + 6), bz = make_box(boxes + 12);
  Box3 bu = box_union(box_union(bx, by), bz);
  if (box_empty(bu)) return 0;
  if (xchunk <= 0) xchunk = 16;
  if (cbx)
    k_update_e3d_v4<true><<<grid_v4(bu, xchunk), dim3(64, TY), 0, (hipStream_t)s>>>(
        ex, ey, ez, hx, hy, hz, cbx, cby, cbz, (float)cb, nx, ny, nz, bx, by, bz, bu, xchunk);
  else
    k_update_e3d_v4<false><<<grid_v4(bu, xchunk), dim3(64, TY), 0, (hipStream_t)s>>>(
        ex, ey, ez, hx, hy, hz, cbx, cby, cbz, (float)cb, nx, ny, nz, bx, by, bz, bu, xchunk);
  FDTD_RETURN_LAUNCH_STATUS();
}

FDTD_API int fdtd_update_h3d_v4_f32(float* hx, float* hy, float* hz, const float* ex, const float* ey,
                                    const float* ez, const float* dbx, const float* dby, const float* dbz,
                                    double db, int nx, int ny, int nz, const int* boxes, int xchunk, void* s) {
  if (nz % 4 != 0) return (int)hipErrorInvalidValue;
  Box3 bx = make_box(boxes), by = make_box(boxes + 6), bz = make_box(boxes + 12);
  Box3 bu = box_union(box_union(bx, by), bz);
  if (box_empty(bu)) return 0;
  if (xchunk <= 0) xchunk = 16;
  if (dbx)
    k_update_h3d_v4<true><<<grid_v4(bu, xchunk), dim3(64, TY), 0, (hipStream_t)s>>>(
        hx, hy, hz, ex, ey, ez, dbx, dby, dbz, (float)db, nx, ny, nz, bx, by, bz, bu, xchunk);
  else
    k_update_h3d_v4<false><<<grid_v4(bu, xchunk), dim3(64, TY), 0, (hipStream_t)s>>>(
        hx, hy, hz, ex, ey, ez, dbx, dby, dbz, (float)db, nx, ny, nz, bx, by, bz, bu, xchunk);
  FDTD_RETURN_LAUNCH_STATUS();
}
