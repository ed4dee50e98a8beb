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
#include "vec4.h"

namespace {

constexpr int TY = 4;

template <bool PERCELL, int LZ>
__global__ __launch_bounds__(64 * TY) void k_update_e3d_v4(
    float* __restrict__ ex, float* __restrict__ ey, float* __restrict__ ez,
    const float* __restrict__ hx, const float* __restrict__ hy, const float* __restrict__ hz,
    const float* __restrict__ cbx, const float* __restrict__ cby, const float* __restrict__ cbz,
    float cb, int nx, int ny, int nz, Box3 bx, Box3 by, Box3 bz, Box3 bu, int xchunk) {
  // LZ lanes per z row, 64 / LZ rows per wave (LZ < 64 for z-thin boxes)
  const int zl = threadIdx.x % LZ;
  const int kb = (bu.lo[2] & ~3) + 4 * (blockIdx.x * LZ + zl);
  const int j = bu.lo[1] + (blockIdx.y * TY + threadIdx.y) * (64 / LZ) + threadIdx.x / LZ;
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
    float hy_k0 = __shfl_up(hyc.w, 1, LZ);
    float hx_k0 = __shfl_up(hxc.w, 1, LZ);
    if (zl == 0 && act && kb > 0) {
      hy_k0 = hy[off - 1];
      hx_k0 = hx[off - 1];
    }
    const bool xin_x = i >= bx.lo[0] && i < bx.hi[0];
    const bool xin_y = i >= by.lo[0] && i < by.hi[0];
    const bool xin_z = i >= bz.lo[0] && i < bz.hi[0];
    if (xin_x && mx) {
      float4 e = ld4(ex, off);
      const float4 hz_j = ld4(hz, off - nz);
      const float4 c4 = (PERCELL && cbx) ? ld4(cbx, off) : make_float4(cb, cb, cb, cb);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (mx & (1u << q)) {
          const float hym = q == 0 ? hy_k0 : f4(hyc, q - 1);
          f4set(e, q, f4(e, q) + f4(c4, q) * ((f4(hzc, q) - f4(hz_j, q)) - (f4(hyc, q) - hym)));
        }
      }
      st4m(ex, off, e, mx);
    }
    if (xin_y && my) {
      float4 e = ld4(ey, off);
      const float4 c4 = (PERCELL && cby) ? ld4(cby, off) : make_float4(cb, cb, cb, cb);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (my & (1u << q)) {
          const float hxm = q == 0 ? hx_k0 : f4(hxc, q - 1);
          f4set(e, q, f4(e, q) + f4(c4, q) * ((f4(hxc, q) - hxm) - (f4(hzc, q) - f4(hz_m, q))));
        }
      }
      st4m(ey, off, e, my);
    }
    if (xin_z && mz) {
      float4 e = ld4(ez, off);
      const float4 hx_j = ld4(hx, off - nz);
      const float4 c4 = (PERCELL && cbz) ? ld4(cbz, off) : make_float4(cb, cb, cb, cb);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (mz & (1u << q)) {
          f4set(e, q, f4(e, q) + f4(c4, q) * ((f4(hyc, q) - f4(hy_m, q)) - (f4(hxc, q) - f4(hx_j, q))));
        }
      }
      st4m(ez, off, e, mz);
    }
    hz_m = hzc;
    hy_m = hyc;
  }
}

template <bool PERCELL, int LZ>
__global__ __launch_bounds__(64 * TY) void k_update_h3d_v4(
    float* __restrict__ hx, float* __restrict__ hy, float* __restrict__ hz,
    const float* __restrict__ ex, const float* __restrict__ ey, const float* __restrict__ ez,
    const float* __restrict__ dbx, const float* __restrict__ dby, const float* __restrict__ dbz,
    float db, int nx, int ny, int nz, Box3 bx, Box3 by, Box3 bz, Box3 bu, int xchunk) {
  // LZ lanes per z row, 64 / LZ rows per wave (LZ < 64 for z-thin boxes)
  const int zl = threadIdx.x % LZ;
  const int kb = (bu.lo[2] & ~3) + 4 * (blockIdx.x * LZ + zl);
  const int j = bu.lo[1] + (blockIdx.y * TY + threadIdx.y) * (64 / LZ) + threadIdx.x / LZ;
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
    float ey_k3 = __shfl_down(ey_c.x, 1, LZ);
    float ex_k3 = __shfl_down(exc.x, 1, LZ);
    if (zl == LZ - 1 && act && kb + 4 < nz) {
      ey_k3 = ey[off + 4];
      ex_k3 = ex[off + 4];
    }
    const bool xin_x = i >= bx.lo[0] && i < bx.hi[0];
    const bool xin_y = i >= by.lo[0] && i < by.hi[0];
    const bool xin_z = i >= bz.lo[0] && i < bz.hi[0];
    if (xin_x && mx) {
      float4 h = ld4(hx, off);
      const float4 ez_j = ld4(ez, off + nz);
      const float4 c4 = (PERCELL && dbx) ? ld4(dbx, off) : make_float4(db, db, db, db);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (mx & (1u << q)) {
          const float eyp = q == 3 ? ey_k3 : f4(ey_c, q + 1);
          f4set(h, q, f4(h, q) + f4(c4, q) * ((eyp - f4(ey_c, q)) - (f4(ez_j, q) - f4(ez_c, q))));
        }
      }
      st4m(hx, off, h, mx);
    }
    if (xin_y && my) {
      float4 h = ld4(hy, off);
      const float4 c4 = (PERCELL && dby) ? ld4(dby, off) : make_float4(db, db, db, db);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (my & (1u << q)) {
          const float exp_ = q == 3 ? ex_k3 : f4(exc, q + 1);
          f4set(h, q, f4(h, q) + f4(c4, q) * ((f4(ez_n, q) - f4(ez_c, q)) - (exp_ - f4(exc, q))));
        }
      }
      st4m(hy, off, h, my);
    }
    if (xin_z && mz) {
      float4 h = ld4(hz, off);
      const float4 ex_j = ld4(ex, off + nz);
      const float4 c4 = (PERCELL && dbz) ? ld4(dbz, off) : make_float4(db, db, db, db);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (mz & (1u << q)) {
          f4set(h, q, f4(h, q) + f4(c4, q) * ((f4(ex_j, q) - f4(exc, q)) - (f4(ey_n, q) - f4(ey_c, q))));
        }
      }
      st4m(hz, off, h, mz);
    }
    ey_c = ey_n;
    ez_c = ez_n;
  }
}

// ---------------------------------------------------------------------------
// Fused E+H step with float4 lanes (see k_fused3d in yee3d.hip for the
// algorithm).  Tile = 256 z (64 lanes x 4) x TY owned rows + 1 halo row.
// Per plane each thread computes E_new on its 4 cells, keeps its own E_new of
// the previous plane in registers (the H update's centre and z+1 terms come
// from registers / lane shuffles), and only the j+1 row (Ex, Ez) goes through
// LDS: 3 plane buffers, one barrier per plane.  Lane 63 additionally
// computes Ex, Ey at z = kb+4 (the tile's z halo).
// ---------------------------------------------------------------------------
template <bool PERCELL, int FTY>
__global__ __launch_bounds__(64 * (FTY + 1)) void k_fused3d_v4(
    const float* __restrict__ exi, const float* __restrict__ eyi, const float* __restrict__ ezi,
    const float* __restrict__ hxi, const float* __restrict__ hyi, const float* __restrict__ hzi,
    float* __restrict__ exo, float* __restrict__ eyo, float* __restrict__ ezo,
    float* __restrict__ hxo, float* __restrict__ hyo, float* __restrict__ hzo,
    const float* __restrict__ cbx, const float* __restrict__ cby, const float* __restrict__ cbz,
    const float* __restrict__ dbx, const float* __restrict__ dby, const float* __restrict__ dbz, float cb,
    float db, int nx, int ny, int nz, Box3 bex, Box3 bey, Box3 bez, Box3 bhx, Box3 bhy, Box3 bhz, Box3 R,
    int xchunk, long long src_off, int src_comp, float src_val) {
  __shared__ float4 sE[3][2][FTY + 1][64];  // [buffer][Ex, Ez][row][lane]
  const int lane = threadIdx.x;
  const int w = threadIdx.y;
  const int kb = (R.lo[2] & ~3) + 4 * (blockIdx.x * 64 + lane);
  const int j = R.lo[1] + blockIdx.y * FTY + w;
  const int i0 = R.lo[0] + blockIdx.z * xchunk;
  const int i1 = min(i0 + xchunk, R.hi[0]);
  const bool owned = (w < FTY) && (j < R.hi[1]) && (kb < R.hi[2]);
  const bool ld_ok = (j < ny) && (kb < nz);
  const bool extra = (lane == 63) && (w < FTY) && ld_ok && (kb + 4 < nz);
  const size_t plane = (size_t)ny * nz;
  const size_t row = (size_t)j * nz + kb;
  const unsigned mex = ld_ok ? kmask(bex, j, kb) : 0u;
  const unsigned mey = ld_ok ? kmask(bey, j, kb) : 0u;
  const unsigned mez = ld_ok ? kmask(bez, j, kb) : 0u;
  const unsigned mhx = owned ? kmask(bhx, j, kb) : 0u;
  const unsigned mhy = owned ? kmask(bhy, j, kb) : 0u;
  const unsigned mhz = owned ? kmask(bhz, j, kb) : 0u;
  const bool x1in = extra && j >= bex.lo[1] && j < bex.hi[1] && kb + 4 >= bex.lo[2] && kb + 4 < bex.hi[2];
  const bool y1in = extra && j >= bey.lo[1] && j < bey.hi[1] && kb + 4 >= bey.lo[2] && kb + 4 < bey.hi[2];
  const float4 z4 = make_float4(0, 0, 0, 0);

  float4 hxp = z4, hyp = z4, hzp = z4;       // H_old(x-1)
  float4 exp_ = z4, eyp = z4, ezp = z4;      // E_new(x-1), own cells
  float hz_p1 = 0, ex1p = 0, ey1p = 0;       // extra column: Hz_old(x-1), E_new(x-1)
  if (ld_ok && i0 > 0) {
    const size_t o = (size_t)(i0 - 1) * plane + row;
    hxp = ld4(hxi, o);
    hyp = ld4(hyi, o);
    hzp = ld4(hzi, o);
    if (extra) hz_p1 = hzi[o + 4];
  }
  for (int x = i0; x <= i1; ++x) {
    const int buf = (x - i0) % 3;
    float4 hxc = z4, hyc = z4, hzc = z4, exn = z4, eyn = z4, ezn = z4;
    const bool inx = ld_ok && x < nx;
    size_t off = (size_t)x * plane + row;
    if (inx) {
      hxc = ld4(hxi, off);
      hyc = ld4(hyi, off);
      hzc = ld4(hzi, off);
      exn = ld4(exi, off);
      eyn = ld4(eyi, off);
      ezn = ld4(ezi, off);
    }
    float hy_k0 = __shfl_up(hyc.w, 1, 64);
    float hx_k0 = __shfl_up(hxc.w, 1, 64);
    if (lane == 0 && inx && kb > 0) {
      hy_k0 = hyi[off - 1];
      hx_k0 = hxi[off - 1];
    }
    if (inx) {
      if (mex && x >= bex.lo[0] && x < bex.hi[0]) {
        const float4 hz_j = ld4(hzi, off - nz);
        const float4 c4 = (PERCELL && cbx) ? ld4(cbx, off) : make_float4(cb, cb, cb, cb);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (mex & (1u << q)) {
            const float hym = q == 0 ? hy_k0 : f4(hyc, q - 1);
            f4set(exn, q, f4(exn, q) + f4(c4, q) * ((f4(hzc, q) - f4(hz_j, q)) - (f4(hyc, q) - hym)));
          }
      }
      if (mey && x >= bey.lo[0] && x < bey.hi[0]) {
        const float4 c4 = (PERCELL && cby) ? ld4(cby, off) : make_float4(cb, cb, cb, cb);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (mey & (1u << q)) {
            const float hxm = q == 0 ? hx_k0 : f4(hxc, q - 1);
            f4set(eyn, q, f4(eyn, q) + f4(c4, q) * ((f4(hxc, q) - hxm) - (f4(hzc, q) - f4(hzp, q))));
          }
      }
      if (mez && x >= bez.lo[0] && x < bez.hi[0]) {
        const float4 hx_j = ld4(hxi, off - nz);
        const float4 c4 = (PERCELL && cbz) ? ld4(cbz, off) : make_float4(cb, cb, cb, cb);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (mez & (1u << q))
            f4set(ezn, q, f4(ezn, q) + f4(c4, q) * ((f4(hyc, q) - f4(hyp, q)) - (f4(hxc, q) - f4(hx_j, q))));
      }
      if (src_comp >= 0 && src_off >= (long long)off && src_off < (long long)off + 4) {
        const int q = (int)(src_off - (long long)off);
        if (src_comp == 0) f4set(exn, q, src_val);
        if (src_comp == 1) f4set(eyn, q, src_val);
        if (src_comp == 2) f4set(ezn, q, src_val);
      }
      // only cells inside a component's box are written: launches on
      // overlapping regions (interior / boundary shell) never clobber each other
      if (owned && x < i1) {
        st4m(exo, off, exn, (x >= bex.lo[0] && x < bex.hi[0]) ? mex : 0u);
        st4m(eyo, off, eyn, (x >= bey.lo[0] && x < bey.hi[0]) ? mey : 0u);
        st4m(ezo, off, ezn, (x >= bez.lo[0] && x < bez.hi[0]) ? mez : 0u);
      }
    }
    sE[buf][0][w][lane] = exn;
    sE[buf][1][w][lane] = ezn;
    float hz_c1 = 0, ex1 = 0, ey1 = 0;
    if (extra && x < nx) {
      // Ex, Ey at (x, j, kb+4): the z halo of this tile
      const size_t o1 = off + 4;
      ex1 = exi[o1];
      ey1 = eyi[o1];
      hz_c1 = hzi[o1];
      if (x1in && x >= bex.lo[0] && x < bex.hi[0]) {
        const float c = (PERCELL && cbx) ? cbx[o1] : cb;
        ex1 += c * ((hz_c1 - hzi[o1 - nz]) - (hyi[o1] - hyc.w));
      }
      if (y1in && x >= bey.lo[0] && x < bey.hi[0]) {
        const float c = (PERCELL && cby) ? cby[o1] : cb;
        ey1 += c * ((hxi[o1] - hxc.w) - (hz_c1 - hz_p1));
      }
      if (src_comp >= 0 && src_off == (long long)o1) {
        if (src_comp == 0) ex1 = src_val;
        if (src_comp == 1) ey1 = src_val;
      }
    }
    // z+1 neighbours of element 3 at plane x-1 (next lane's element 0)
    float ey_k3 = __shfl_down(eyp.x, 1, 64);
    float ex_k3 = __shfl_down(exp_.x, 1, 64);
    if (lane == 63) {
      ey_k3 = ey1p;
      ex_k3 = ex1p;
    }
    __syncthreads();
    if (x > i0 && (mhx | mhy | mhz)) {
      const int xm = x - 1;
      const int pb = (x - 1 - i0) % 3;
      const size_t o = (size_t)xm * plane + row;
      const float4 ex_jp = sE[pb][0][w + 1][lane];
      const float4 ez_jp = sE[pb][1][w + 1][lane];
      float4 hxn = hxp, hyn = hyp, hzn = hzp;
      if (mhx && xm >= bhx.lo[0] && xm < bhx.hi[0]) {
        const float4 c4 = (PERCELL && dbx) ? ld4(dbx, o) : make_float4(db, db, db, db);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (mhx & (1u << q)) {
            const float eyk = q == 3 ? ey_k3 : f4(eyp, q + 1);
            f4set(hxn, q, f4(hxn, q) + f4(c4, q) * ((eyk - f4(eyp, q)) - (f4(ez_jp, q) - f4(ezp, q))));
          }
      }
      if (mhy && xm >= bhy.lo[0] && xm < bhy.hi[0]) {
        const float4 c4 = (PERCELL && dby) ? ld4(dby, o) : make_float4(db, db, db, db);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (mhy & (1u << q)) {
            const float exk = q == 3 ? ex_k3 : f4(exp_, q + 1);
            f4set(hyn, q, f4(hyn, q) + f4(c4, q) * ((f4(ezn, q) - f4(ezp, q)) - (exk - f4(exp_, q))));
          }
      }
      if (mhz && xm >= bhz.lo[0] && xm < bhz.hi[0]) {
        const float4 c4 = (PERCELL && dbz) ? ld4(dbz, o) : make_float4(db, db, db, db);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (mhz & (1u << q))
            f4set(hzn, q, f4(hzn, q) + f4(c4, q) * ((f4(ex_jp, q) - f4(exp_, q)) - (f4(eyn, q) - f4(eyp, q))));
      }
      st4m(hxo, o, hxn, (xm >= bhx.lo[0] && xm < bhx.hi[0]) ? mhx : 0u);
      st4m(hyo, o, hyn, (xm >= bhy.lo[0] && xm < bhy.hi[0]) ? mhy : 0u);
      st4m(hzo, o, hzn, (xm >= bhz.lo[0] && xm < bhz.hi[0]) ? mhz : 0u);
    }
    hxp = hxc;
    hyp = hyc;
    hzp = hzc;
    exp_ = exn;
    eyp = eyn;
    ezp = ezn;
    hz_p1 = hz_c1;
    ex1p = ex1;
    ey1p = ey1;
  }
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

inline dim3 grid_v4(const Box3& bu, int xchunk, int lz) {
  const int kspan = bu.hi[2] - (bu.lo[2] & ~3);
  return dim3(cdiv(kspan, 4 * lz), cdiv(bu.hi[1] - bu.lo[1], TY * (64 / lz)), cdiv(bu.hi[0] - bu.lo[0], xchunk));
}

// launch one split-kernel instantiation with the box's lane layout
#define LAUNCH_LZ(KERNEL, PC, ...)                                                          \
  do {                                                                                      \
    const int lz_ = lanes_z(bu);                                                            \
    if (lz_ == 8)                                                                           \
      KERNEL<PC, 8><<<grid_v4(bu, xchunk, 8), dim3(64, TY), 0, (hipStream_t)s>>>(__VA_ARGS__);   \
    else if (lz_ == 16)                                                                     \
      KERNEL<PC, 16><<<grid_v4(bu, xchunk, 16), dim3(64, TY), 0, (hipStream_t)s>>>(__VA_ARGS__); \
    else                                                                                    \
      KERNEL<PC, 64><<<grid_v4(bu, xchunk, 64), dim3(64, TY), 0, (hipStream_t)s>>>(__VA_ARGS__); \
  } while (0)

}  // namespace

static int g_fused_rows = 7;  // owned rows per workgroup (3 or 7); tuning knob

FDTD_API void fdtd_set_fused_rows(int rows) { g_fused_rows = (rows == 3) ? 3 : 7; }

template <int FTY>
static int launch_fused_v4(const float* const* ein, const float* const* hin, float* const* eout,
                           float* const* hout, const float* const* cbs, const float* const* dbs, double cb,
                           double db, int nx, int ny, int nz, const int* boxes, int xchunk, long long src_off,
                           int src_comp, double src_val, void* s);

FDTD_API int fdtd_fused3d_v4_f32(const float* const* ein, const float* const* hin, float* const* eout,
                                 float* const* hout, const float* const* cbs, const float* const* dbs, double cb,
                                 double db, int nx, int ny, int nz, const int* boxes, int xchunk, long long src_off,
                                 int src_comp, double src_val, void* s) {
  if (g_fused_rows == 3)
    return launch_fused_v4<3>(ein, hin, eout, hout, cbs, dbs, cb, db, nx, ny, nz, boxes, xchunk, src_off, src_comp,
                              src_val, s);
  return launch_fused_v4<7>(ein, hin, eout, hout, cbs, dbs, cb, db, nx, ny, nz, boxes, xchunk, src_off, src_comp,
                            src_val, s);
}

template <int FTY>
static int launch_fused_v4(const float* const* ein, const float* const* hin, float* const* eout,
                           float* const* hout, const float* const* cbs, const float* const* dbs, double cb,
                           double db, int nx, int ny, int nz, const int* boxes, int xchunk, long long src_off,
                           int src_comp, double src_val, void* s) {
  if (nz % 4 != 0) return (int)hipErrorInvalidValue;
  Box3 b[6];
  for (int n = 0; n < 6; ++n) b[n] = make_box(boxes + 6 * n);
  Box3 R = b[0];
  for (int n = 1; n < 6; ++n) R = box_union(R, b[n]);
  if (box_empty(R)) return 0;
  if (xchunk <= 0) xchunk = 16;  // measured: 16 >= 64 >= 32 at 1024^3 (tools/kbench.py)
  const int kspan = R.hi[2] - (R.lo[2] & ~3);
  dim3 grid(cdiv(kspan, 256), cdiv(R.hi[1] - R.lo[1], FTY), cdiv(R.hi[0] - R.lo[0], xchunk));
  dim3 block(64, FTY + 1);
  if (cbs[0] || dbs[0])  // a null kind uses its scalar
    k_fused3d_v4<true, FTY><<<grid, block, 0, (hipStream_t)s>>>(
        ein[0], ein[1], ein[2], hin[0], hin[1], hin[2], eout[0], eout[1], eout[2], hout[0], hout[1], hout[2], cbs[0],
        cbs[1], cbs[2], dbs[0], dbs[1], dbs[2], (float)cb, (float)db, nx, ny, nz, b[0], b[1], b[2], b[3], b[4], b[5],
        R, xchunk, src_off, src_comp, (float)src_val);
  else
    k_fused3d_v4<false, FTY><<<grid, block, 0, (hipStream_t)s>>>(
        ein[0], ein[1], ein[2], hin[0], hin[1], hin[2], eout[0], eout[1], eout[2], hout[0], hout[1], hout[2], cbs[0],
        cbs[1], cbs[2], dbs[0], dbs[1], dbs[2], (float)cb, (float)db, nx, ny, nz, b[0], b[1], b[2], b[3], b[4], b[5],
        R, xchunk, src_off, src_comp, (float)src_val);
  FDTD_RETURN_LAUNCH_STATUS();
}

FDTD_API int fdtd_update_e3d_v4_f32(float* ex, float* ey, float* ez, const float* hx, const float* hy,
                                    const float* hz, const float* cbx, const float* cby, const float* cbz,
                                    double cb, int nx, int ny, int nz, const int* boxes, int xchunk, void* s) {
  if (nz % 4 != 0) return (int)hipErrorInvalidValue;
  Box3 bx = make_box(boxes), by = make_box(boxes + 6), bz = make_box(boxes + 12);
  Box3 bu = box_union(box_union(bx, by), bz);
  if (box_empty(bu)) return 0;
  {
    const dim3 g1 = grid_v4(bu, 1, lanes_z(bu));
    xchunk = split_xchunk(bu.hi[0] - bu.lo[0], (long long)g1.x * g1.y, xchunk);
  }
  if (cbx)
    LAUNCH_LZ(k_update_e3d_v4, true, ex, ey, ez, hx, hy, hz, cbx, cby, cbz, (float)cb, nx, ny, nz, bx, by, bz, bu, xchunk);
  else
    LAUNCH_LZ(k_update_e3d_v4, false, ex, ey, ez, hx, hy, hz, cbx, cby, cbz, (float)cb, nx, ny, nz, bx, by, bz, bu, xchunk);
  FDTD_RETURN_LAUNCH_STATUS();
}

FDTD_API int fdtd_update_h3d_v4_f32(float* hx, float* hy, float* hz, const float* ex, const float* ey,
                                    const float* ez, const float* dbx, const float* dby, const float* dbz,
                                    double db, int nx, int ny, int nz, const int* boxes, int xchunk, void* s) {
  if (nz % 4 != 0) return (int)hipErrorInvalidValue;
  Box3 bx = make_box(boxes), by = make_box(boxes + 6), bz = make_box(boxes + 12);
  Box3 bu = box_union(box_union(bx, by), bz);
  if (box_empty(bu)) return 0;
  {
    const dim3 g1 = grid_v4(bu, 1, lanes_z(bu));
    xchunk = split_xchunk(bu.hi[0] - bu.lo[0], (long long)g1.x * g1.y, xchunk);
  }
  if (dbx)
    LAUNCH_LZ(k_update_h3d_v4, true, hx, hy, hz, ex, ey, ez, dbx, dby, dbz, (float)db, nx, ny, nz, bx, by, bz, bu, xchunk);
  else
    LAUNCH_LZ(k_update_h3d_v4, false, hx, hy, hz, ex, ey, ez, dbx, dby, dbz, (float)db, nx, ny, nz, bx, by, bz, bu, xchunk);
  FDTD_RETURN_LAUNCH_STATUS();
}
