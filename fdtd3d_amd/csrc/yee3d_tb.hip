// Temporally blocked fp32 3D Yee kernel: T full leapfrog steps per HBM pass.
//
// The single-pass kernels (yee3d_v4.hip) move >= 48 B/cell/step, so one
// MI355X tops out near 6.3 TB/s / 48 B = 131 Gcells/s however well they are
// tiled.  This kernel reads E^n, H^n once and writes E^{n+T}, H^{n+T} once
// (reference has no counterpart: its CUDA path is one launch per component and
// step, Source/Cuda/CudaInterface.cu:583-812).
//
// Tile (one workgroup, 16 waves = 1024 threads, one workgroup per CU):
//   * z: a wave row of 64 lanes x V cells (V = 4: float4 lanes, 256 cells;
//     V = 2 for T >= 3, halving the registers every level carries); HL =
//     ceil(T / V) lanes at each end are halo, the rest are owned.
//   * y: 16 rows (one per wave); T rows at each side are halo, 16-2T owned.
//   * x: the workgroup streams planes X = i0-T .. i1+T-1 of its x chunk.
// Level l (1..T) of iteration X computes E_l on plane X-l+1 and H_l on plane
// X-l: a wavefront that lags one plane per level, so every x neighbour a
// level needs is either this iteration's result of the level below or a
// register carried from the previous iteration.  y neighbours (Hz, Hx at row
// j-1 for E; Ex, Ez at row j+1 for H) go through a double-buffered LDS slot
// (4 fields x 16 rows x 1 KiB, one barrier per level), z neighbours through
// lane shuffles.  Halo
// cells accumulate wrong values from the tile edge inward by one cell per
// half step; the T-deep halo keeps that cone away from every owned cell.
//
// Update boxes (where each component may change) and the output box (cells
// this launch stores) are separate: in a decomposed run the ghost layers are
// updated redundantly at the inner levels but never stored.

#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace {

constexpr int TBW = 16;  // waves (y rows) per workgroup

template <int V>
struct VT;
template <>
struct VT<1> {
  typedef float f __attribute__((ext_vector_type(1)));
  typedef unsigned u __attribute__((ext_vector_type(1)));
};
template <>
struct VT<2> {
  typedef float f __attribute__((ext_vector_type(2)));
  typedef unsigned u __attribute__((ext_vector_type(2)));
};
template <>
struct VT<4> {
  typedef float f __attribute__((ext_vector_type(4)));
  typedef unsigned u __attribute__((ext_vector_type(4)));
};

// neighbour lanes through DPP wave shifts (one VALU op, usually folded into
// the consuming v_sub as a _dpp modifier) instead of ds_bpermute round trips
// through the LDS pipe: lane_up(v) on lane i = v of lane i-1 (wave_shr:1),
// lane_dn(v) = v of lane i+1 (wave_shl:1); lanes shifted in from outside the
// wave read 0 -- they are halo lanes of every tile.
__device__ __forceinline__ float lane_up(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float lane_dn(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, false));
}

struct TbSrc {
  float v[8];  // hard-source value applied after E update of level l
};

// TF/SF plane-wave corrections folded into the blocked passes (fdtd3d_amd/
// models/tfsf.py TfsfSets).  A set is one (component, TF/SF face) pair of the
// reference's border tests (Scheme3D.cpp:138-208, YeeGridLayout.cpp:327-809):
// a box of target cells, one cell thick across the face.  For an incident
// direction along x or y the incident value a target sees depends on its
// index along that axis only (`va`), so each pass precomputes, per level,
// g = sign * projection * interpolated incident line at every index of a set
// (k_tfsf_pass below) and the kernels add g to the target's curl before the
// coefficient multiply -- from SCALAR loads (wave-uniform index), which do not
// queue behind the vector prefetch.
constexpr int TF_MAX_SETS = 24;
struct TfSet {
  int n;          // component 0..5 = Ex Ey Ez Hx Hy Hz
  int fa;         // axis the face is perpendicular to
  int lo[3], hi[3];
  int va;         // table axis (0 x, 1 y)
  int goff;       // first g entry of the set inside one level
};
// CPML convolution terms (fdtd3d_amd/models/cpml.py, layout of
// yee3d_cpml.hip): per (component, term axis) the low / high psi slabs, their
// ranges along the axis and the b / c / (1/kappa - 1) profiles (identity
// outside the slabs).  psi index of a slab along x: ((i-lo) ny + j) nz + k;
// along y: (i w + j-lo) nz + k; along z: (i ny + j) w + k-lo (w = hi - lo).
struct CpmlTerm {
  const float* psi[2];  // read (time n) ...
  float* out[2];        // ... and written (time n + 1): ping-pong, because the
                        // halo cells a tile recomputes belong to neighbour tiles
                        // that may already have advanced them
  int lo[2], hi[2];
  const float* b;
  const float* c;
  const float* k;
};
struct CpmlDev {
  CpmlTerm t[6][3];  // [Ex Ey Ez Hx Hy Hz][term axis]
};
// curl terms of each component: (axis, sign), Ex = +dHz/dy - dHy/dz etc.
__device__ constexpr int kTermAxis[6][2] = {{1, 2}, {2, 0}, {0, 1}, {2, 1}, {0, 2}, {1, 0}};

// the CPML table travels by value in the kernel arguments (CPML variants
// only): its pointers and profile reads are then wave-uniform scalar loads --
// SGPR descriptors, no waterfall loop, and profile loads that wait on the
// scalar counter instead of queueing behind the vector prefetch (a copy in
// LDS hands every field back in VGPRs)
template <bool ON>
struct CpArg {
  int unused;
};
template <>
struct CpArg<true> {
  CpmlDev d;
};

struct TfDev {
  int nsets;
  int ld;                   // g entries per level
  int xpl[2][2];            // [E / H][low / high] x-face planes (-1: none)
  TfSet s[TF_MAX_SETS];
};

// Memory access through buffer descriptors: one descriptor per (array, x
// plane) built in SGPRs from the wave-uniform plane index, plus ONE 32-bit
// per-lane byte offset shared by every array (buffer_load ... offen).  Flat
// 64-bit addressing would keep a per-lane pointer per array live across the
// x loop (24 VGPRs for 12 arrays) and spill.  Offsets past the descriptor's
// size read 0 / drop the store, which is how rows and planes outside the
// array are handled -- no per-lane load guards.
typedef __amdgpu_buffer_rsrc_t Rsrc;

__device__ __forceinline__ Rsrc plane_rsrc(const float* base, int x, int nx, size_t plane) {
  const bool in = x >= 0 && x < nx;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (size_t)(in ? x : 0) * plane), (short)0,
                                           in ? (int)(plane * 4) : 0, 0x00020000);
}

template <int V>
__device__ __forceinline__ typename VT<V>::f bld(Rsrc r, unsigned boff) {
  if constexpr (V == 1)
    return __builtin_bit_cast(typename VT<1>::f, __builtin_amdgcn_raw_buffer_load_b32(r, boff, 0, 0));
  else if constexpr (V == 4)
    return __builtin_bit_cast(typename VT<4>::f, __builtin_amdgcn_raw_buffer_load_b128(r, boff, 0, 0));
  else
    return __builtin_bit_cast(typename VT<2>::f, __builtin_amdgcn_raw_buffer_load_b64(r, boff, 0, 0));
}

template <int V>
__device__ __forceinline__ void bst(Rsrc r, unsigned boff, const typename VT<V>::f& v, unsigned mask) {
  if (mask == (1u << V) - 1u) {
    if constexpr (V == 1)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[0]), r, boff, 0, 0);
    else if constexpr (V == 4)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(typename VT<4>::u, v), r, boff, 0, 0);
    else
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(typename VT<2>::u, v), r, boff, 0, 0);
  } else if (V > 1 && mask) {
    // the b32 builtin takes the raw bits (an implicit float->uint would convert)
#pragma unroll
    for (int q = 0; q < V; ++q)
      if (mask & (1u << q)) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[q]), r, boff + 4 * q, 0, 0);
  }
}

// one unsigned compare (2 SALU) instead of two compares and an AND
__device__ __forceinline__ bool xin(const Box3& b, int x) {
  return (unsigned)(x - b.lo[0]) < (unsigned)(b.hi[0] - b.lo[0]);
}

// bit q set when element q of the lane's V-group (cells kb..kb+V-1) is in the box
template <int V>
__device__ __forceinline__ unsigned kmaskv(const Box3& b, int j, int kb) {
  if (j < b.lo[1] || j >= b.hi[1]) return 0u;
  unsigned m = 0;
#pragma unroll
  for (int e = 0; e < V; ++e) m |= ((kb + e >= b.lo[2]) && (kb + e < b.hi[2])) ? (1u << e) : 0u;
  return m;
}

// elements of c whose bit is set in m, zero elsewhere
template <int V>
__device__ __forceinline__ typename VT<V>::f cmask(typename VT<V>::f c, unsigned m) {
#pragma unroll
  for (int q = 0; q < V; ++q) c[q] = (m & (1u << q)) ? c[q] : 0.f;
  return c;
}

// z-1 / z+1 neighbours of a lane's V cells (s = the cell beyond the group)
template <int V>
__device__ __forceinline__ typename VT<V>::f zm1(const typename VT<V>::f& v, float s) {
  typename VT<V>::f r;
  r[0] = s;
#pragma unroll
  for (int q = 1; q < V; ++q) r[q] = v[q - 1];
  return r;
}
template <int V>
__device__ __forceinline__ typename VT<V>::f zp1(const typename VT<V>::f& v, float s) {
  typename VT<V>::f r;
#pragma unroll
  for (int q = 0; q < V - 1; ++q) r[q] = v[q + 1];
  r[V - 1] = s;
  return r;
}

template <int V>
struct F3 {
  typename VT<V>::f x, y, z;
};

template <int T, int V, int R, bool PERCELL>
__global__ __launch_bounds__(64 * TBW) void k_tb3d(
    const float* __restrict__ exi, const float* __restrict__ eyi, const float* __restrict__ ezi,
    const float* __restrict__ hxi, const float* __restrict__ hyi, const float* __restrict__ hzi,
    float* __restrict__ exo, float* __restrict__ eyo, float* __restrict__ ezo,
    float* __restrict__ hxo, float* __restrict__ hyo, float* __restrict__ hzo,
    const float* __restrict__ cbx, const float* __restrict__ cby, const float* __restrict__ cbz,
    const float* __restrict__ dbx, const float* __restrict__ dby, const float* __restrict__ dbz, float cb,
    float db, int nx, int ny, int nz, Box3 bex, Box3 bey, Box3 bez, Box3 bhx, Box3 bhy, Box3 bhz, Box3 O,
    int xchunk, int src_i, int src_j, int src_k, int src_comp, TbSrc sv, int xcd_swz) {
  typedef typename VT<V>::f vec;
  constexpr bool PF = V == 2;            // software prefetch of the next plane
  constexpr int LW = 64 / R;             // lanes per grid row (R rows per wave)
  constexpr int ROWS = TBW * R;          // y rows per workgroup
  constexpr int HL = (T + V - 1) / V;    // halo lanes per side
  constexpr int TBZ = (LW - 2 * HL) * V; // owned z cells per tile
  __shared__ vec sX[2][4][ROWS][LW];     // [buffer][field][row][lane]
  const int lane = threadIdx.x % LW;     // z position inside the row
  const int w = threadIdx.y * R + threadIdx.x / LW;  // row inside the workgroup
  // tile of this workgroup.  XCD-aware order (cdna_hip_programming.md 5.5 T1):
  // workgroups are dealt round-robin to the 8 XCDs, so remap the dispatch
  // index so that each XCD gets a contiguous run of tiles, y fastest -- tiles
  // adjacent in y then stream the same x planes at the same time on one L2
  // and the 2T halo rows they share are L2 hits instead of HBM re-reads.
  int tz = blockIdx.x, ty = blockIdx.y, tx = blockIdx.z;
  if (xcd_swz) {
    const int gx = gridDim.x, gy = gridDim.y;
    const int n = gx * gy * (int)gridDim.z;
    const int p = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int n8 = n & ~7;
    const int q = p < n8 ? (p & 7) * (n8 >> 3) + (p >> 3) : p;
    ty = q % gy;
    tz = (q / gy) % gx;
    tx = q / (gy * gx);
  }
  const int kb = (O.lo[2] & ~(V - 1)) - HL * V + TBZ * tz + V * lane;
  const int j = O.lo[1] - T + (ROWS - 2 * T) * ty + w;
  const int i0 = O.lo[0] + tx * xchunk;
  const int i1 = min(i0 + xchunk, O.hi[0]);
  const bool ld_ok = j >= 0 && j < ny && kb >= 0 && kb < nz;
  const bool own = ld_ok && lane >= HL && lane < LW - HL && w >= T && w < ROWS - T && j >= O.lo[1] && j < O.hi[1];
  const size_t plane = (size_t)ny * nz;
  // per-lane 32-bit offset inside a plane; plane bases are wave-uniform (SGPR)
  const unsigned row = ld_ok ? (unsigned)(j * nz + kb) * 4u : 0xF0000000u;  // byte offset (past end: reads 0)
  // element masks of the update boxes (all rows) and of the stored cells
  const unsigned mex = ld_ok ? kmaskv<V>(bex, j, kb) : 0u;
  const unsigned mey = ld_ok ? kmaskv<V>(bey, j, kb) : 0u;
  const unsigned mez = ld_ok ? kmaskv<V>(bez, j, kb) : 0u;
  const unsigned mhx = ld_ok ? kmaskv<V>(bhx, j, kb) : 0u;
  const unsigned mhy = ld_ok ? kmaskv<V>(bhy, j, kb) : 0u;
  const unsigned mhz = ld_ok ? kmaskv<V>(bhz, j, kb) : 0u;
  const unsigned mo = own ? kmaskv<V>(O, j, kb) : 0u;
  const bool src_here = src_comp >= 0 && j == src_j && src_k >= kb && src_k < kb + V;
  const int src_q = src_k - kb;
  const int rdn = w > 0 ? w - 1 : 0;
  const int rup = w < ROWS - 1 ? w + 1 : ROWS - 1;
  const vec zero = (vec)(0.f);
  const vec cbv = (vec)(cb), dbv = (vec)(db);
  // float2 lanes: scalar coefficients masked by the (loop-invariant) y/z box
  // masks once, per plane only the x-range test remains (a wave-uniform
  // select); float4 lanes have no registers to spare and mask per plane
  constexpr bool PREMASK = V == 2 && !PERCELL;
  const vec mcex = PREMASK ? cmask<V>(cbv, mex) : zero, mcey = PREMASK ? cmask<V>(cbv, mey) : zero;
  const vec mcez = PREMASK ? cmask<V>(cbv, mez) : zero, mchx = PREMASK ? cmask<V>(dbv, mhx) : zero;
  const vec mchy = PREMASK ? cmask<V>(dbv, mhy) : zero, mchz = PREMASK ? cmask<V>(dbv, mhz) : zero;
  // coefficient of one component on plane p: per-cell plane (PERCELL) or the
  // scalar, zeroed outside the component's update box
  auto coef = [&](const float* arr, const Box3& b, int p, unsigned m, const vec& pre, const vec& sc) -> vec {
    const bool in = xin(b, p);
    if (PERCELL && arr) return cmask<V>(bld<V>(plane_rsrc(arr, in ? p : -1, nx, plane), row), in ? m : 0u);
    if (PREMASK) return in ? pre : zero;
    return cmask<V>(sc, in ? m : 0u);
  };

  // carried state (see header): Hp[l] = H_l(X-1-l), Ep[l] = E_{l+1}(X-1-l)
  F3<V> Hp[T], Ep[T];
#pragma unroll
  for (int l = 0; l < T; ++l) {
    Hp[l].x = Hp[l].y = Hp[l].z = zero;
    Ep[l].x = Ep[l].y = Ep[l].z = zero;
  }
  int buf = 0;

  // plane X's six fields; with PF the next plane is loaded before this one's
  // levels run, so its HBM latency hides under the compute and barriers
  // (float2 lanes have the registers for it)
  auto load_plane = [&](int X, F3<V>& H, F3<V>& E) {
    H.x = bld<V>(plane_rsrc(hxi, X, nx, plane), row);
    H.y = bld<V>(plane_rsrc(hyi, X, nx, plane), row);
    H.z = bld<V>(plane_rsrc(hzi, X, nx, plane), row);
    E.x = bld<V>(plane_rsrc(exi, X, nx, plane), row);
    E.y = bld<V>(plane_rsrc(eyi, X, nx, plane), row);
    E.z = bld<V>(plane_rsrc(ezi, X, nx, plane), row);
  };
  F3<V> Hnx, Enx;
  if (PF) load_plane(i0 - T, Hnx, Enx);
  for (int X = i0 - T; X <= i1 + T - 1; ++X) {
    F3<V> Hc, Ec;
    if (PF) {
      Hc = Hnx;
      Ec = Enx;
      load_plane(X + 1, Hnx, Enx);
    } else {
      load_plane(X, Hc, Ec);
    }
    F3<V> En;
#pragma unroll
    for (int l = 0; l < T; ++l) {
      // ---- E_{l+1} on plane pe from H_l(pe) = Hc, H_l(pe-1) = Hp[l], E_l(pe) = Ec
      const int pe = X - l;
      // one LDS round per level: Hz, Hx of H_l(pe) for the row above (E needs
      // j-1) and Ex, Ez of E_{l+1}(pe-1) for the row below (H needs j+1)
      sX[buf][0][w][lane] = Hc.z;
      sX[buf][1][w][lane] = Hc.x;
      sX[buf][2][w][lane] = Ep[l].x;
      sX[buf][3][w][lane] = Ep[l].z;
      __syncthreads();
      const vec hz_j = sX[buf][0][rdn][lane];
      const vec hx_j = sX[buf][1][rdn][lane];
      const vec ex_jn = sX[buf][2][rup][lane];
      const vec ez_jn = sX[buf][3][rup][lane];
      buf ^= 1;
      const float hy_k0 = lane_up(Hc.y[V - 1]);
      const float hx_k0 = lane_up(Hc.x[V - 1]);
      // coefficients are zeroed outside each component's update box, so the
      // arithmetic is branch-free vector work and untouched cells keep E_l
      const vec cex = coef(cbx, bex, pe, mex, mcex, cbv);
      En.x = Ec.x + cex * ((Hc.z - hz_j) - (Hc.y - zm1<V>(Hc.y, hy_k0)));
      const vec cey = coef(cby, bey, pe, mey, mcey, cbv);
      En.y = Ec.y + cey * ((Hc.x - zm1<V>(Hc.x, hx_k0)) - (Hc.z - Hp[l].z));
      const vec cez = coef(cbz, bez, pe, mez, mcez, cbv);
      En.z = Ec.z + cez * ((Hc.y - Hp[l].y) - (Hc.x - hx_j));
      if (src_here && pe == src_i) {
        if (src_comp == 0) En.x[src_q] = sv.v[l];
        if (src_comp == 1) En.y[src_q] = sv.v[l];
        if (src_comp == 2) En.z[src_q] = sv.v[l];
      }
      // ---- H_{l+1} on plane ph = pe-1 from E_{l+1}(ph) = Ep[l], E_{l+1}(pe) = En,
      //      H_l(ph) = Hp[l]
      const int ph = pe - 1;
      const float ey_k3 = lane_dn(Ep[l].y[0]);
      const float ex_k3 = lane_dn(Ep[l].x[0]);
      F3<V> Hn;
      const vec chx = coef(dbx, bhx, ph, mhx, mchx, dbv);
      Hn.x = Hp[l].x + chx * ((zp1<V>(Ep[l].y, ey_k3) - Ep[l].y) - (ez_jn - Ep[l].z));
      const vec chy = coef(dby, bhy, ph, mhy, mchy, dbv);
      Hn.y = Hp[l].y + chy * ((En.z - Ep[l].z) - (zp1<V>(Ep[l].x, ex_k3) - Ep[l].x));
      const vec chz = coef(dbz, bhz, ph, mhz, mchz, dbv);
      Hn.z = Hp[l].z + chz * ((ex_jn - Ep[l].x) - (En.y - Ep[l].y));
      // ---- rotate: next level reads E_{l+1}(X-l-1) and H_{l+1}(X-l-1)
      Ec = Ep[l];
      Ep[l] = En;
      Hp[l] = Hc;
      Hc = Hn;
    }
    // outputs: E_T on plane X-T+1, H_T on plane X-T.  Cells of the output box
    // outside a component's update box are stored unchanged (PEC cells: equal
    // in both ping-pong buffers), so only the output box masks the store.
    if (mo) {
      const int pe = X - T + 1;
      if (pe >= i0 && pe < i1) {
        bst<V>(plane_rsrc(exo, pe, nx, plane), row, En.x, mo);
        bst<V>(plane_rsrc(eyo, pe, nx, plane), row, En.y, mo);
        bst<V>(plane_rsrc(ezo, pe, nx, plane), row, En.z, mo);
      }
      const int ph = X - T;
      if (ph >= i0 && ph < i1) {
        bst<V>(plane_rsrc(hxo, ph, nx, plane), row, Hc.x, mo);
        bst<V>(plane_rsrc(hyo, ph, nx, plane), row, Hc.y, mo);
        bst<V>(plane_rsrc(hzo, ph, nx, plane), row, Hc.z, mo);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Multi-row variant: every wave carries R ADJACENT y rows in registers (rows
// R*w .. R*w+R-1 of the tile), so one workgroup spans 16R rows and the 2T
// redundant halo rows are amortised over 16R instead of 16 (T=4: 8 of 16 rows
// owned by the single-row kernel, 24 of 32 at R=2).  y neighbours inside a
// wave's row group are registers; only the first / last row of the group goes
// through LDS (the same 4 fields x 16 slots as above, one barrier per level).
// Scalar lanes (V=1) keep the register footprint of the float2 single-row
// kernel; the extra z halo lanes (T per side) cost less than the y rows saved.
// Masks of the 7 boxes (6 update boxes + output box) for every row are packed
// into one bit field (R*V <= 4).
// PFD: planes loaded ahead (1 or 2).  DEFER: the results of plane X are
// stored after plane X+1's prefetch is issued -- vmcnt counts loads and
// stores together in issue order, so stores issued between two prefetches
// would otherwise be waited for with the older prefetch.
template <int T, int V, int R, int FX, int PFD, bool DEFER, int NW>
__global__ __launch_bounds__(64 * NW) void k_tb3d_mr(
    const float* __restrict__ exi, const float* __restrict__ eyi, const float* __restrict__ ezi,
    const float* __restrict__ hxi, const float* __restrict__ hyi, const float* __restrict__ hzi,
    float* __restrict__ exo, float* __restrict__ eyo, float* __restrict__ ezo,
    float* __restrict__ hxo, float* __restrict__ hyo, float* __restrict__ hzo,
    const float4* __restrict__ ce4, const float4* __restrict__ ch4, Box3 BE, Box3 BH, float cb,
    float db, int nx, int ny, int nz, Box3 bex, Box3 bey, Box3 bez, Box3 bhx, Box3 bhy, Box3 bhz, Box3 O,
    int xchunk, int src_i, int src_j, int src_k, int src_comp, TbSrc sv, int xcd_swz,
    const TfDev* __restrict__ tf, const float* __restrict__ gtab, const CpArg<(FX & 8) != 0> cpv,
    float* __restrict__ pscr) {
  // feature bits: 1 per-cell E, 2 per-cell H coefficients (sparse), 4 TF/SF,
  // 8 CPML.  A CPML pass of T > 1 steps hands each level's psi to the next
  // level through `pscr`, thread-private scratch (see the level loop)
  constexpr int PC = FX & 3;
  constexpr bool TFS = FX & 4;
  constexpr bool CPM = FX & 8;
  static_assert(V == 1 || !FX, "sparse coefficients / TF/SF: scalar lanes");
  constexpr bool PCE = PC & 1, PCH = PC & 2;  // per-cell E / H coefficients
  static_assert(R * V <= 4, "mask bit field holds 7 boxes x R rows x V cells");
  typedef typename VT<V>::f vec;
  constexpr int HL = (T + V - 1) / V;   // halo lanes per side
  constexpr int TBZ = (64 - 2 * HL) * V; // owned z cells per tile
  constexpr int ROWS = NW * R;         // y rows per workgroup
  constexpr unsigned VM = (1u << V) - 1u;
  __shared__ vec sX[2][4][NW][64];
  const int lane = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.y);  // one wave per y (SGPR)
  // the TF/SF table lives in LDS for the kernel's life: its fields are read in
  // many branches (with dynamic set indices)
  __shared__ unsigned sTFraw[TFS ? sizeof(TfDev) / 4 : 1];
  __shared__ unsigned long long sCPraw[1];  // stand-in table of the non-CPML variants (never read)
  if constexpr (TFS) {
    for (int q = threadIdx.x + 64 * threadIdx.y; q < (int)(sizeof(TfDev) / 4); q += 64 * NW)
      sTFraw[q] = ((const unsigned*)tf)[q];
  }
  if constexpr (TFS) __syncthreads();
  const TfDev& TF = *reinterpret_cast<const TfDev*>(sTFraw);
  auto cp_ref = [&]() -> const CpmlDev& {
    if constexpr (CPM)
      return cpv.d;
    else
      return *reinterpret_cast<const CpmlDev*>(sCPraw);
  };
  const CpmlDev& CP = cp_ref();
  // Tile of this workgroup.  A row of a tile starts at an arbitrary z (the
  // stride is the 64 - 2T owned cells), so its 64 cells straddle three
  // 128-B lines, one shared with each z neighbour tile.  Workgroups are dealt
  // round-robin to the 8 XCDs (own L2 each); with xcd_swz each XCD instead
  // gets a contiguous run of tiles, z fastest, so z neighbours run together
  // on one L2 and the shared lines are fetched from HBM once.
  int tz = blockIdx.x, ty = blockIdx.y, tx = blockIdx.z;
  if (xcd_swz & 1) {
    const int gx = gridDim.x, gy = gridDim.y;
    const int n = gx * gy * (int)gridDim.z;
    const int p = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int n8 = n & ~7;
    const int q = p < n8 ? (p & 7) * (n8 >> 3) + (p >> 3) : p;
    const int pz = (xcd_swz >> 8) & 0xff, py = (xcd_swz >> 16) & 0xff;
    if (pz > 0 && py > 0) {
      // patch order: an XCD's run of tiles is dealt in PZ x PY (z x y)
      // patches, so the ~32 workgroups one XCD holds at a time form a compact
      // block whose y AND z neighbours stream the same planes on the same L2
      // (a tile shares 2T of its rows with each y neighbour, 2T lanes with
      // each z neighbour).  Bands of PY tile rows; the last band and the last
      // patch of a band may be narrower.
      tx = q / (gx * gy);
      const int r = q - tx * gx * gy;
      const int band = r / (py * gx);
      const int h = min(py, gy - band * py);
      const int rb = r - band * py * gx;
      const int col = rb / (pz * h);
      const int wdt = min(pz, gx - col * pz);
      const int e = rb - col * pz * h;
      tz = col * pz + e % wdt;
      ty = band * py + e / wdt;
    } else {
      tz = q % gx;
      ty = (q / gx) % gy;
      tx = q / (gx * gy);
    }
  }
  const int kb = (O.lo[2] & ~(V - 1)) - HL * V + TBZ * tz + V * lane;
  const int jw = O.lo[1] - T + (ROWS - 2 * T) * ty + R * w;  // first row of this wave
  const int i0 = O.lo[0] + tx * xchunk;
  const int i1 = min(i0 + xchunk, O.hi[0]);
  const bool kin = kb >= 0 && kb < nz;
  const bool lane_own = lane >= HL && lane < 64 - HL;
  const size_t plane = (size_t)ny * nz;
  unsigned roff[R];
  unsigned mbits = 0;  // bit (r*7 + n)*V + q: cell q of row r inside box n
  const Box3* bx[7] = {&bex, &bey, &bez, &bhx, &bhy, &bhz, &O};
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int j = jw + r;
    const int t = R * w + r;
    const bool ld_ok = kin && j >= 0 && j < ny;
    roff[r] = ld_ok ? (unsigned)(j * nz + kb) * 4u : 0xF0000000u;
    const bool own = ld_ok && lane_own && t >= T && t < ROWS - T;
#pragma unroll
    for (int n = 0; n < 7; ++n) {
      const bool ok = n < 6 ? ld_ok : own;
      mbits |= (ok ? kmaskv<V>(*bx[n], j, kb) : 0u) << ((r * 7 + n) * V);
    }
  }
  const int rdn = w > 0 ? w - 1 : 0;
  const int rup = w < NW - 1 ? w + 1 : NW - 1;
  const vec zero = (vec)(0.f);
  const vec cbv = (vec)(cb), dbv = (vec)(db);
  // Tiles whose every lane and row lies inside all six update boxes in y / z
  // (all but the tiles on the domain's y / z border) run a copy of the whole
  // x loop in which a coefficient is just the x-range-selected scalar -- no
  // per-element mask extraction and select (3 VALU per coefficient, ~40% of
  // the kernel's VALU work).  The copy is of the OUTER loop, so the two
  // versions never hold registers at the same time.
  unsigned upd_bits = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) upd_bits |= ((1u << (6 * V)) - 1u) << (r * 7 * V);
  const bool tile_all = __all((mbits & upd_bits) == upd_bits);

  // Sparse per-cell coefficients (PC): the cells whose coefficient differs
  // from the kind's scalar lie in a box (BE for E, BH for H) and the three
  // components' values are one float4 per cell of that box (.w unused).  Each
  // trip loads, for every level, one 12-byte vector per kind and row -- only
  // on planes and waves that cross the box (wave-uniform tests), everything
  // else runs on the scalar -- and issues those loads BEFORE the next plane's
  // field prefetch: vmcnt retires loads in issue order, so a coefficient load
  // issued after the prefetch would make its level wait for the prefetch too.
  // Lanes outside the box in y / z read at an offset past the plane (0) and
  // select the scalar.
  unsigned eoff[R], hoff[R];
  unsigned inb = 0;  // bit r: row r of this lane inside BE (y, z); bit R + r: inside BH
  const int bez_n = BE.hi[2] - BE.lo[2], bhz_n = BH.hi[2] - BH.lo[2];
  const size_t eplane = (size_t)(BE.hi[1] - BE.lo[1]) * bez_n * 16u;
  const size_t hplane = (size_t)(BH.hi[1] - BH.lo[1]) * bhz_n * 16u;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int j = jw + r;
    const bool ie = PCE && kin && j >= BE.lo[1] && j < BE.hi[1] && kb >= BE.lo[2] && kb < BE.hi[2];
    const bool ih = PCH && kin && j >= BH.lo[1] && j < BH.hi[1] && kb >= BH.lo[2] && kb < BH.hi[2];
    eoff[r] = ie ? (unsigned)((j - BE.lo[1]) * bez_n + (kb - BE.lo[2])) * 16u : 0xF0000000u;
    hoff[r] = ih ? (unsigned)((j - BH.lo[1]) * bhz_n + (kb - BH.lo[2])) * 16u : 0xF0000000u;
    inb |= (ie ? 1u : 0u) << r;
    inb |= (ih ? 1u : 0u) << (R + r);
  }
  const bool wave_e = PCE && __any(inb & ((1u << R) - 1u));
  const bool wave_h = PCH && __any(inb >> R);
  // TF/SF.  x-face sets (one plane each, all rows / lanes of the TF box) are
  // rare per wave and go through scalar loads when a level hits their plane.
  // y / z-face sets (one row or one lane column) touch few waves but every
  // level of every trip of those waves, so each wave parks up to TF_SLOTS of
  // them per kind in slots: slot metadata in VGPR lanes (read back with
  // readlane at a compile-time lane), a per-lane bit per (slot, row) for the
  // cells it covers, and per trip ONE vector load of the g values of every
  // (slot, level, row) -- issued before the field prefetch, so the levels
  // never wait behind it.
  constexpr int TF_SLOTS = 6;                      // per kind
  constexpr int TF_ENT = 2 * TF_SLOTS * T * R;     // g entries per trip (<= 128 for T <= 5)
  static_assert(!TFS || TF_ENT <= 128, "TF/SF: at most 5 steps per pass");
  unsigned tf_wx[2] = {0u, 0u};
  unsigned tf_ov[2] = {0u, 0u};  // face sets beyond the slots: the scalar path every level
  int tf_xe0 = -1, tf_xe1 = -1, tf_xh0 = -1, tf_xh1 = -1;  // x-face planes (E / H sets)
  int tf_na0 = 0, tf_na1 = 0;                      // slots in use (E / H)
  unsigned tf_lbits = 0;                           // bit slot * R + r: this lane in the slot's set, row r
  int tf_mx = 0;                                   // lane s: x range of slot s (lo | hi << 16)
  int tf_mn = 0;                                   // lane s: component of slot s
  int tf_gb0 = 0, tf_gb1 = 0;                      // g index of entry lane / lane + 64 (plus X when va = 0)
  bool tf_ok0 = false, tf_ok1 = false;
  int tf_va = 0, tf_ld = 0;
  if constexpr (TFS) {
    const int ns = TF.nsets;
    const int ld = TF.ld;
    tf_ld = ld;
    tf_va = TF.s[0].va;
    int na[2] = {0, 0};
    for (int si = 0; si < ns; ++si) {
      const TfSet& S = TF.s[si];
      unsigned rb = 0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int j = jw + r;
        rb |= (kin && j >= S.lo[1] && j < S.hi[1] && kb >= S.lo[2] && kb < S.hi[2]) ? (1u << r) : 0u;
      }
      if (!__any(rb != 0u)) continue;
      const int k = S.n < 3 ? 0 : 1;
      if (S.fa == 0) {
        tf_wx[0] |= k == 0 ? (1u << si) : 0u;
        tf_wx[1] |= k == 1 ? (1u << si) : 0u;
        continue;
      }
      const int a = k == 0 ? na[0] : na[1];
      if (a >= TF_SLOTS) {
        tf_ov[0] |= k == 0 ? (1u << si) : 0u;
        tf_ov[1] |= k == 1 ? (1u << si) : 0u;
        continue;
      }
      const int slot = k * TF_SLOTS + a;
      if (k == 0) ++na[0]; else ++na[1];
      tf_lbits |= rb << (slot * R);
      if (lane == slot) {
        tf_mx = S.lo[0] | (S.hi[0] << 16);
        tf_mn = S.n;
      }
      // entries (slot, l, r) -> entry q = (slot * T + l) * R + r
#pragma unroll
      for (int l = 0; l < T; ++l)
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int q = (slot * T + l) * R + r;
          // level l: E sets on plane X - l, H sets on X - l - 1
          const int base = l * ld + S.goff + (S.va == 0 ? -S.lo[0] - l - k : (jw + r) - S.lo[1]);
          if (lane == q) { tf_gb0 = base; tf_ok0 = true; }
          if (lane + 64 == q) { tf_gb1 = base; tf_ok1 = true; }
        }
    }
    tf_na0 = na[0];
    tf_na1 = na[1];
    tf_xe0 = TF.xpl[0][0];
    tf_xe1 = TF.xpl[0][1];
    tf_xh0 = TF.xpl[1][0];
    tf_xh1 = TF.xpl[1][1];
  }
  const bool tf_slots = TFS && (tf_na0 + tf_na1) > 0;
  float tf_g0 = 0.f, tf_g1 = 0.f;  // this trip's g entries (lane q, q + 64)
  // add the TF/SF corrections of kind k at level l, plane p, row r to the curls
  auto tf_apply = [&](int k, int l, int p, int r, vec& c0, vec& c1, vec& c2) {
    if constexpr (TFS) {
      // y / z-face slots
      if (tf_slots) {
#pragma unroll
        for (int a = 0; a < TF_SLOTS; ++a) {
          if (a >= (k == 0 ? tf_na0 : tf_na1)) break;
          const int slot = k * TF_SLOTS + a;
          const int xr = __builtin_amdgcn_readlane(tf_mx, slot);
          if ((unsigned)(p - (xr & 0xffff)) >= (unsigned)((xr >> 16) - (xr & 0xffff))) continue;
          const int q = (slot * T + l) * R + r;
          const float g = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q < 64 ? tf_g0 : tf_g1), q & 63));
          const float gl = ((tf_lbits >> (slot * R + r)) & 1u) ? g : 0.f;
          const int c = __builtin_amdgcn_readlane(tf_mn, slot) - 3 * k;
          c0 = c0 + (vec)(c == 0 ? gl : 0.f);
          c1 = c1 + (vec)(c == 1 ? gl : 0.f);
          c2 = c2 + (vec)(c == 2 ? gl : 0.f);
        }
      }
      // x-face sets on their plane
      const bool xp = k == 0 ? (p == tf_xe0 || p == tf_xe1) : (p == tf_xh0 || p == tf_xh1);
      unsigned cand = (xp ? (k == 0 ? tf_wx[0] : tf_wx[1]) : 0u) | (k == 0 ? tf_ov[0] : tf_ov[1]);
      const int j = jw + r;
      while (cand) {
        const int si = __builtin_ctz(cand);
        cand &= cand - 1u;
        const TfSet& S = TF.s[si];
        if ((unsigned)(p - S.lo[0]) >= (unsigned)(S.hi[0] - S.lo[0]) || j < S.lo[1] || j >= S.hi[1]) continue;
        const float g = gtab[l * TF.ld + S.goff + (S.va == 0 ? p - S.lo[0] : j - S.lo[1])];
        // g on the set's lanes, 0 elsewhere, added to the set's component by
        // selects (conditional adds make the compiler index a scratch array)
        const float gl = (kb >= S.lo[2] && kb < S.hi[2]) ? g : 0.f;
        const int c = S.n - 3 * k;
        c0 = c0 + (vec)(c == 0 ? gl : 0.f);
        c1 = c1 + (vec)(c == 1 ? gl : 0.f);
        c2 = c2 + (vec)(c == 2 ? gl : 0.f);
      }
    }
  };
  typedef unsigned u3 __attribute__((ext_vector_type(3)));
  auto coef_ld = [&](const float4* arr, const Box3& B, unsigned off, size_t pl, int p) -> u3 {
    const Rsrc rs = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)arr + (size_t)(p - B.lo[0]) * pl),
                                                      (short)0, (int)pl, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b96(rs, off, 0, 0);
  };
  // RING: one per-cell kind; its coefficient planes X - l - RHS of the T
  // levels of trip X sit in T LDS slots (each wave reads and writes only its
  // own rows, so no barrier guards them)
  constexpr bool RING = PC == 1 || PC == 2;
  constexpr int NS = RING ? T : 1;
  constexpr int RHS = PC == 2 ? 1 : 0;  // H levels run one plane behind E
  __shared__ float sC[NS][3][RING ? ROWS : 1][64];
  const Box3& RB = PC == 2 ? BH : BE;
  const float4* rarr = PC == 2 ? ch4 : ce4;
  const size_t rpl = PC == 2 ? hplane : eplane;
  const unsigned* roffc = PC == 2 ? hoff : eoff;
  const bool wave_r = PC == 2 ? wave_h : wave_e;
  auto ring_slot = [&](int p) -> int { return (p + 64 * NS) % NS; };
  if (RING && wave_r && xin(RB, i0 - T - RHS)) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u3 v = coef_ld(rarr, RB, roffc[r], rpl, i0 - T - RHS);
      const int sl = ring_slot(i0 - T - RHS);
      sC[sl][0][R * w + r][lane] = __uint_as_float(v.x);
      sC[sl][1][R * w + r][lane] = __uint_as_float(v.y);
      sC[sl][2][R * w + r][lane] = __uint_as_float(v.z);
    }
  }

  // CPML helpers.  Terms are (component n, t):
  // axis kTermAxis[n][t].  y terms: Ex.0 Ez.1 Hx.1 Hz.0; z terms: Ex.1 Ey.0
  // Hx.0 Hy.1; x terms: the rest.
  auto ytm_index = [](int n) -> int { return n == 0 ? 0 : (n == 2 ? 1 : (n == 3 ? 2 : 3)); };
  auto ztm_index = [](int n) -> int { return n == 0 ? 0 : (n == 1 ? 1 : (n == 3 ? 2 : 3)); };
  // slab side holding index v along the term's axis (-1: none)
  auto side_of = [&](const CpmlTerm& tm, int v) -> int {
    return (tm.psi[0] && v >= tm.lo[0] && v < tm.hi[0]) ? 0 : ((tm.psi[1] && v >= tm.lo[1] && v < tm.hi[1]) ? 1 : -1);
  };
  auto psi_side_x = [&](int n, int t, int pl) -> int {
    return kTermAxis[n][t] == 0 ? side_of(CP.t[n][0], pl) : -1;
  };
  auto psi_side_y = [&](int n, int t, int j) -> int {
    return kTermAxis[n][t] == 1 ? side_of(CP.t[n][1], j) : -1;
  };
  // descriptor of plane pl of the side-sd slab of term (n, t), read or written copy
  auto psi_rsrc = [&](int n, int t, int sd, int pl, bool wr) -> Rsrc {
    const int a = kTermAxis[n][t];
    const CpmlTerm& tm = CP.t[n][a];
    const int wd = tm.hi[sd] - tm.lo[sd];
    const size_t pe_ = a == 0 ? (size_t)ny * nz : (a == 1 ? (size_t)wd * nz : (size_t)ny * wd);
    const size_t first = a == 0 ? (size_t)(pl - tm.lo[sd]) * pe_ : (size_t)pl * pe_;
    const float* base = wr ? tm.out[sd] : tm.psi[sd];
    return __builtin_amdgcn_make_buffer_rsrc((void*)(base + first), (short)0, (int)(pe_ * 4), 0x00020000);
  };
  // lane byte offset of row r in that plane (past the plane for lanes outside the slab)
  auto psi_off = [&](int n, int t, int sd, int r) -> unsigned {
    const int a = kTermAxis[n][t];
    const CpmlTerm& tm = CP.t[n][a];
    if (a == 0) return roff[r];
    if (a == 1) return roff[r] - (unsigned)(tm.lo[sd] * nz) * 4u;  // sentinel offsets stay past the plane
    const int j = jw + r;
    const bool in = kin && j >= 0 && j < ny && kb >= tm.lo[sd] && kb < tm.hi[sd];
    return in ? (unsigned)(j * (tm.hi[sd] - tm.lo[sd]) + (kb - tm.lo[sd])) * 4u : 0xF0000000u;
  };
  // wave-level activity of the 12 terms (bit 2n + t): x terms always (the
  // plane decides per trip), y terms when a row of the wave lies in a slab,
  // z terms when a lane does; z-term profiles per lane, y-term profiles of
  // the wave's rows in LDS (uniform reads)
  unsigned cpm_wave = 0;
  float ZB[CPM ? 4 : 1], ZC[CPM ? 4 : 1], ZK[CPM ? 4 : 1];
  __shared__ float sYP[CPM ? NW : 1][CPM ? 4 * R * 3 : 1];
  if constexpr (CPM) {
#pragma unroll
    for (int n = 0; n < 6; ++n)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int a = kTermAxis[n][t];
        const CpmlTerm& tm = CP.t[n][a];
        bool act = false;
        if (a == 0) {
          act = tm.psi[0] || tm.psi[1];
        } else if (a == 1) {
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int j = jw + r;
            const bool in = side_of(tm, j) >= 0;
            act |= in;
            const int q = (ytm_index(n) * R + r) * 3;
            if (lane == 0) {
              sYP[w][q] = in ? tm.b[j] : 1.f;
              sYP[w][q + 1] = in ? tm.c[j] : 0.f;
              sYP[w][q + 2] = in ? tm.k[j] : 0.f;
            }
          }
        } else {
          const bool in = kin && side_of(tm, kb) >= 0;
          act = __any(in);
          const int zi = ztm_index(n);
          ZB[zi] = in ? tm.b[kb] : 1.f;
          ZC[zi] = in ? tm.c[kb] : 0.f;
          ZK[zi] = in ? tm.k[kb] : 0.f;
        }
        cpm_wave |= act ? (1u << (2 * n + t)) : 0u;
      }
  }
  // Multi-step CPML: level l of trip X advances the psi of plane X - l (E
  // terms; H terms X - l - 1), and level l + 1 of trip X + 1 advances the same
  // cells again -- in the same lane of the same wave.  So the hand-off between
  // levels is thread-private: level l stores its psi in slot (X & 1, l) of
  // this thread's scratch column, the next trip's level l + 1 loads it back
  // (agent-scope loads: L1 bypassed, the thread's own store is in L2).  The
  // trip parity keeps this trip's level l from overwriting what its level
  // l + 1 has yet to read.  Level 0 reads
  // the slab arrays (psi at time n), level T - 1 writes the other copy (n + T)
  // for owned cells only.  Slots are slot-major across all threads of the
  // launch, so a wave's 64 lanes touch one contiguous 256-B run.
  const unsigned scr_nth = gridDim.x * gridDim.y * gridDim.z * NW * 64u;
  const unsigned scr_tid =
      ((blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * NW + w) * 64u + lane;
  const Rsrc scr_rs = __builtin_amdgcn_make_buffer_rsrc((void*)pscr, (short)0, CPM && T > 1 && pscr ? -1 : 0,
                                                        0x00020000);
  // (xcd_swz bit 24, tuning: plain loads that may hit L1 instead of agent-scope ones)
  const bool scr_l1 = (xcd_swz >> 24) & 1;
  // per-lane part of a slot address (one VGPR) + wave-uniform slot base (soffset)
  const unsigned scr_voff = scr_tid * 4u;
  auto scr_soff = [&](int par, int l, int n, int t, int r) -> int {
    return (int)((unsigned)((((par * (T - 1) + l) * 6 + n) * 2 + t) * R + r) * scr_nth * 4u);
  };

  auto run = [&](auto allin_tag) {
  constexpr bool ALLIN = decltype(allin_tag)::value;
  // coefficient of component n (box b) of row r on plane p: the lane's value
  // sc (scalar or per-cell) inside the update box, 0 outside
  auto coef = [&](const Box3& b, int p, int r, int n, float sc) -> vec {
    const bool in = xin(b, p);
    if constexpr (ALLIN) return in ? (vec)(sc) : zero;
    const unsigned m = in ? (mbits >> ((r * 7 + n) * V)) & VM : 0u;
    return cmask<V>((vec)(sc), m);
  };

  F3<V> Hp[T][R], Ep[T][R];
#pragma unroll
  for (int l = 0; l < T; ++l)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      Hp[l][r].x = Hp[l][r].y = Hp[l][r].z = zero;
      Ep[l][r].x = Ep[l][r].y = Ep[l][r].z = zero;
    }
  int buf = 0;
  auto load_plane = [&](int X, F3<V>* H, F3<V>* E) {
    const Rsrc rhx = plane_rsrc(hxi, X, nx, plane), rhy = plane_rsrc(hyi, X, nx, plane);
    const Rsrc rhz = plane_rsrc(hzi, X, nx, plane), rex = plane_rsrc(exi, X, nx, plane);
    const Rsrc rey = plane_rsrc(eyi, X, nx, plane), rez = plane_rsrc(ezi, X, nx, plane);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      H[r].x = bld<V>(rhx, roff[r]);
      H[r].y = bld<V>(rhy, roff[r]);
      H[r].z = bld<V>(rhz, roff[r]);
      E[r].x = bld<V>(rex, roff[r]);
      E[r].y = bld<V>(rey, roff[r]);
      E[r].z = bld<V>(rez, roff[r]);
    }
  };
  F3<V> Hnx[R], Enx[R], Hn2[R], En2[R];
  load_plane(i0 - T, Hnx, Enx);
  if (PFD == 2) load_plane(i0 - T + 1, Hn2, En2);
  F3<V> Hs[R];  // DEFER: H_T of the previous plane, stored next trip
#pragma unroll
  for (int r = 0; r < R; ++r) Hs[r] = F3<V>{};
  // stores of the results of trip X: E_T on plane X-T+1 (= Ep[T-1] until the
  // next trip's last level), H_T on plane X-T
  auto store_plane = [&](int X, const F3<V>* Es, const F3<V>* Hh) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const unsigned mo = (mbits >> ((r * 7 + 6) * V)) & VM;
      if constexpr (V == 1) {
        // unconditional stores masked by an out-of-range offset (dropped by
        // the descriptor): a fixed store count per trip keeps the compiler's
        // vmcnt bookkeeping exact, so the next prefetch wait does not drain
        // the stores (see DEFER)
        const int pe = X - T + 1, ph = X - T;
        const unsigned oe = mo && pe >= i0 && pe < i1 ? roff[r] : 0xF0000000u;
        const unsigned oh = mo && ph >= i0 && ph < i1 ? roff[r] : 0xF0000000u;
        bst<V>(plane_rsrc(exo, pe, nx, plane), oe, Es[r].x, 1u);
        bst<V>(plane_rsrc(eyo, pe, nx, plane), oe, Es[r].y, 1u);
        bst<V>(plane_rsrc(ezo, pe, nx, plane), oe, Es[r].z, 1u);
        bst<V>(plane_rsrc(hxo, ph, nx, plane), oh, Hh[r].x, 1u);
        bst<V>(plane_rsrc(hyo, ph, nx, plane), oh, Hh[r].y, 1u);
        bst<V>(plane_rsrc(hzo, ph, nx, plane), oh, Hh[r].z, 1u);
      } else if (mo) {
        const int pe = X - T + 1;
        if (pe >= i0 && pe < i1) {
          bst<V>(plane_rsrc(exo, pe, nx, plane), roff[r], Es[r].x, mo);
          bst<V>(plane_rsrc(eyo, pe, nx, plane), roff[r], Es[r].y, mo);
          bst<V>(plane_rsrc(ezo, pe, nx, plane), roff[r], Es[r].z, mo);
        }
        const int ph = X - T;
        if (ph >= i0 && ph < i1) {
          bst<V>(plane_rsrc(hxo, ph, nx, plane), roff[r], Hh[r].x, mo);
          bst<V>(plane_rsrc(hyo, ph, nx, plane), roff[r], Hh[r].y, mo);
          bst<V>(plane_rsrc(hzo, ph, nx, plane), roff[r], Hh[r].z, mo);
        }
      }
    }
  };
  for (int X = i0 - T; X <= i1 + T - 1; ++X) {
    F3<V> Hc[R], Ec[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      Hc[r] = Hnx[r];
      Ec[r] = Enx[r];
      if (PFD == 2) {
        Hnx[r] = Hn2[r];
        Enx[r] = En2[r];
      }
    }
    // this trip's coefficients.  One per-cell kind (RING): the next trip's
    // newest plane is loaded now and parked in the wave's own LDS ring slots
    // at the end of the trip.  Both kinds: every level's plane into registers.
    const int qn = X + 1 - RHS;  // ring: the plane the next trip's level 0 needs
    const bool ring_ld = RING && wave_r && xin(RB, qn);
    u3 RQ[R];
    if (ring_ld) {
#pragma unroll
      for (int r = 0; r < R; ++r) RQ[r] = coef_ld(rarr, RB, roffc[r], rpl, qn);
    }
    u3 CE[PC == 3 ? T : 1][R], CH[PC == 3 ? T : 1][R];
    if (PC == 3 && wave_e) {
#pragma unroll
      for (int l = 0; l < T; ++l)
        if (xin(BE, X - l))
#pragma unroll
          for (int r = 0; r < R; ++r) CE[PC == 3 ? l : 0][r] = coef_ld(ce4, BE, eoff[r], eplane, X - l);
    }
    if (PC == 3 && wave_h) {
#pragma unroll
      for (int l = 0; l < T; ++l)
        if (xin(BH, X - l - 1))
#pragma unroll
          for (int r = 0; r < R; ++r) CH[PC == 3 ? l : 0][r] = coef_ld(ch4, BH, hoff[r], hplane, X - l - 1);
    }
    // the lane's three coefficients of a kind at level l, plane p (scalar off the box)
    auto kcoef = [&](bool kind_e, int l, int p, int r) -> float3 {
      const float sc = kind_e ? cb : db;
      const bool wave = kind_e ? wave_e : wave_h;
      const bool lane_in = (inb >> (kind_e ? r : R + r)) & 1u;
      if constexpr (RING) {
        if (kind_e == (bool)PCE && wave && xin(RB, p) && lane_in) {
          const int sl = ring_slot(p);
          return make_float3(sC[sl][0][R * w + r][lane], sC[sl][1][R * w + r][lane], sC[sl][2][R * w + r][lane]);
        }
      } else if constexpr (PC == 3) {
        if (wave && xin(kind_e ? BE : BH, p) && lane_in) {
          const u3 raw = kind_e ? CE[PC == 3 ? l : 0][r] : CH[PC == 3 ? l : 0][r];
          return make_float3(__uint_as_float(raw.x), __uint_as_float(raw.y), __uint_as_float(raw.z));
        }
      }
      return make_float3(sc, sc, sc);
    };
    // CPML: this trip's psi (E terms on plane X, H terms on X - 1), loaded
    // before the prefetch (vmcnt order).  Slab membership is wave-uniform for
    // x (plane) and y (row) terms and per lane for z terms; every access goes
    // through a buffer descriptor of the slab plane with a 32-bit lane offset,
    // and lanes outside a slab get an offset past the descriptor (reads 0,
    // stores dropped) instead of a branch.
    float PS[CPM ? 6 : 1][2][R];
    if constexpr (CPM) {
#pragma unroll
      for (int n = 0; n < 6; ++n) {
        const int pl = n < 3 ? X : X - 1;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int a = kTermAxis[n][t];
#pragma unroll
          for (int r = 0; r < R; ++r) PS[n][t][r] = 0.f;
          if (!(cpm_wave >> (2 * n + t) & 1u) || pl < 0 || pl >= nx) continue;
#pragma unroll
          for (int sd = 0; sd < 2; ++sd) {
            const int side_pl = psi_side_x(n, t, pl);
            if (a == 0 && side_pl != sd) continue;
#pragma unroll
            for (int r = 0; r < R; ++r) {
              if (a == 1 && psi_side_y(n, t, jw + r) != sd) continue;
              const unsigned off = psi_off(n, t, sd, r);
              PS[n][t][r] +=
                  __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(psi_rsrc(n, t, sd, pl, false), off, 0, 0));
            }
          }
        }
      }
    }
    // psi update of term t of component n (plane pl, row r) from its raw
    // difference d; returns the curl correction sign * ((1/kappa - 1) d + psi)
    auto cpml = [&](int n, int t, int pl, int r, const vec& d) -> vec {
      if constexpr (CPM) {
        const int a = kTermAxis[n][t];
        const int sg = t == 0 ? 1 : -1;
        if (!(cpm_wave >> (2 * n + t) & 1u)) return zero;
        float bb, cc, kk;
        if (a == 0) {
          if (psi_side_x(n, t, pl) < 0) return zero;
          const CpmlTerm& tm = CP.t[n][0];
          bb = tm.b[pl];
          cc = tm.c[pl];
          kk = tm.k[pl];
        } else if (a == 1) {
          if (psi_side_y(n, t, jw + r) < 0) return zero;
          const int q = (ytm_index(n) * R + r) * 3;
          bb = sYP[w][q];
          cc = sYP[w][q + 1];
          kk = sYP[w][q + 2];
        } else {
          const int zi = ztm_index(n);
          bb = ZB[zi];
          cc = ZC[zi];
          kk = ZK[zi];
        }
        const float pn = bb * PS[n][t][r] + cc * d[0];
        PS[n][t][r] = pn;
        const float cr = kk * d[0] + pn;  // 0 off a z slab (identity profile, psi 0)
        return (vec)(sg > 0 ? cr : -cr);
      }
      return zero;
    };
    if (tf_slots) {
      // this trip's g entries of the face slots (va = 0: index moves with X)
      // (entries of planes outside a set's x range are never used; their
      // index is clamped into the table)
      const int dx = tf_va == 0 ? X : 0;
      const int last = T * tf_ld - 1;
      tf_g0 = tf_ok0 ? gtab[min(max(tf_gb0 + dx, 0), last)] : 0.f;
      if (TF_ENT > 64) tf_g1 = tf_ok1 ? gtab[min(max(tf_gb1 + dx, 0), last)] : 0.f;
    }
    // next plane(s) in flight under this plane's levels
    if (PFD == 2)
      load_plane(X + 2, Hn2, En2);
    else
      load_plane(X + 1, Hnx, Enx);
    if (DEFER && (V == 1 || X > i0 - T)) {  // V = 1: the first trip's stores are dropped
      F3<V> Es[R];
#pragma unroll
      for (int r = 0; r < R; ++r) Es[r] = Ep[T - 1][r];
      store_plane(X - 1, Es, Hs);
    }
    F3<V> En[R];
#pragma unroll
    for (int l = 0; l < T; ++l) {
      const int pe = X - l;
      if constexpr (CPM && T > 1) {
        if (l > 0) {
          // this level's psi: written by level l - 1 on the previous trip
#pragma unroll
          for (int n = 0; n < 6; ++n) {
            const int pl = n < 3 ? pe : pe - 1;
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              if (!(cpm_wave >> (2 * n + t) & 1u)) continue;
              if (kTermAxis[n][t] == 0 && psi_side_x(n, t, pl) < 0) continue;
#pragma unroll
              for (int r = 0; r < R; ++r) {
                const int so = scr_soff((X - 1) & 1, l - 1, n, t, r);
                PS[n][t][r] = __uint_as_float(scr_l1 ? __builtin_amdgcn_raw_buffer_load_b32(scr_rs, scr_voff, so, 0)
                                                     : __builtin_amdgcn_raw_buffer_load_b32(scr_rs, scr_voff, so, 16));
              }
            }
          }
        }
      }
      sX[buf][0][w][lane] = Hc[R - 1].z;
      sX[buf][1][w][lane] = Hc[R - 1].x;
      sX[buf][2][w][lane] = Ep[l][0].x;
      sX[buf][3][w][lane] = Ep[l][0].z;
      __syncthreads();
      const vec hz_dn = sX[buf][0][rdn][lane];
      const vec hx_dn = sX[buf][1][rdn][lane];
      const vec ex_up = sX[buf][2][rup][lane];
      const vec ez_up = sX[buf][3][rup][lane];
      buf ^= 1;
      const bool src_plane = src_comp >= 0 && pe == src_i;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const vec hz_j = r == 0 ? hz_dn : Hc[r > 0 ? r - 1 : 0].z;
        const vec hx_j = r == 0 ? hx_dn : Hc[r > 0 ? r - 1 : 0].x;
        const float hy_k0 = lane_up(Hc[r].y[V - 1]);
        const float hx_k0 = lane_up(Hc[r].x[V - 1]);
        const float3 ce = kcoef(true, l, pe, r);
        const vec dxy = Hc[r].z - hz_j, dxz = Hc[r].y - zm1<V>(Hc[r].y, hy_k0);
        const vec dyz = Hc[r].x - zm1<V>(Hc[r].x, hx_k0), dyx = Hc[r].z - Hp[l][r].z;
        const vec dzx = Hc[r].y - Hp[l][r].y, dzy = Hc[r].x - hx_j;
        vec cx = dxy - dxz;
        vec cy = dyz - dyx;
        vec cz = dzx - dzy;
        if constexpr (CPM) {
          cx += cpml(0, 0, pe, r, dxy) + cpml(0, 1, pe, r, dxz);
          cy += cpml(1, 0, pe, r, dyz) + cpml(1, 1, pe, r, dyx);
          cz += cpml(2, 0, pe, r, dzx) + cpml(2, 1, pe, r, dzy);
        }
        tf_apply(0, l, pe, r, cx, cy, cz);
        En[r].x = Ec[r].x + coef(bex, pe, r, 0, ce.x) * cx;
        En[r].y = Ec[r].y + coef(bey, pe, r, 1, ce.y) * cy;
        En[r].z = Ec[r].z + coef(bez, pe, r, 2, ce.z) * cz;
        if (src_plane && jw + r == src_j && src_k >= kb && src_k < kb + V) {
          const int q = src_k - kb;
          if (src_comp == 0) En[r].x[q] = sv.v[l];
          if (src_comp == 1) En[r].y[q] = sv.v[l];
          if (src_comp == 2) En[r].z[q] = sv.v[l];
        }
      }
      const int ph = pe - 1;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const vec ex_jn = r == R - 1 ? ex_up : Ep[l][r < R - 1 ? r + 1 : r].x;
        const vec ez_jn = r == R - 1 ? ez_up : Ep[l][r < R - 1 ? r + 1 : r].z;
        const float ey_k3 = lane_dn(Ep[l][r].y[0]);
        const float ex_k3 = lane_dn(Ep[l][r].x[0]);
        F3<V> Hn;
        const float3 ch = kcoef(false, l, ph, r);
        const vec gxz = zp1<V>(Ep[l][r].y, ey_k3) - Ep[l][r].y, gxy = ez_jn - Ep[l][r].z;
        const vec gyx = En[r].z - Ep[l][r].z, gyz = zp1<V>(Ep[l][r].x, ex_k3) - Ep[l][r].x;
        const vec gzy = ex_jn - Ep[l][r].x, gzx = En[r].y - Ep[l][r].y;
        vec dx = gxz - gxy;
        vec dy = gyx - gyz;
        vec dz = gzy - gzx;
        if constexpr (CPM) {
          dx += cpml(3, 0, ph, r, gxz) + cpml(3, 1, ph, r, gxy);
          dy += cpml(4, 0, ph, r, gyx) + cpml(4, 1, ph, r, gyz);
          dz += cpml(5, 0, ph, r, gzy) + cpml(5, 1, ph, r, gzx);
        }
        tf_apply(1, l, ph, r, dx, dy, dz);
        Hn.x = Hp[l][r].x + coef(bhx, ph, r, 3, ch.x) * dx;
        Hn.y = Hp[l][r].y + coef(bhy, ph, r, 4, ch.y) * dy;
        Hn.z = Hp[l][r].z + coef(bhz, ph, r, 5, ch.z) * dz;
        // later rows (r+1 ..) read only their own and higher rows' Ep, so
        // row r rotates as soon as its H is done
        Ec[r] = Ep[l][r];
        Ep[l][r] = En[r];
        Hp[l][r] = Hc[r];
        Hc[r] = Hn;
      }
      if constexpr (CPM && T > 1) {
        if (l < T - 1) {
#pragma unroll
          for (int n = 0; n < 6; ++n) {
            const int pl = n < 3 ? pe : pe - 1;
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              if (!(cpm_wave >> (2 * n + t) & 1u)) continue;
              if (kTermAxis[n][t] == 0 && psi_side_x(n, t, pl) < 0) continue;
#pragma unroll
              for (int r = 0; r < R; ++r)
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(PS[n][t][r]), scr_rs, scr_voff,
                                                      scr_soff(X & 1, l, n, t, r), 0);
            }
          }
        }
      }
    }
    if constexpr (CPM) {
      // psi of owned cells inside their component's update box (the last
      // level's planes)
#pragma unroll
      for (int n = 0; n < 6; ++n) {
        const int pl = n < 3 ? X - T + 1 : X - T;
        if (pl < i0 || pl >= i1 || !xin(*bx[n], pl)) continue;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int a = kTermAxis[n][t];
          if (!(cpm_wave >> (2 * n + t) & 1u)) continue;
#pragma unroll
          for (int sd = 0; sd < 2; ++sd) {
            if (a == 0 && psi_side_x(n, t, pl) != sd) continue;
#pragma unroll
            for (int r = 0; r < R; ++r) {
              if (a == 1 && psi_side_y(n, t, jw + r) != sd) continue;
              const bool st = ((mbits >> (r * 7 + 6)) & 1u) && ((mbits >> (r * 7 + n)) & 1u);
              const unsigned off = st ? psi_off(n, t, sd, r) : 0xF0000000u;
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(PS[n][t][r]), psi_rsrc(n, t, sd, pl, true), off,
                                                    0, 0);
            }
          }
        }
      }
    }
    if (ring_ld) {
      // slot of plane qn = that of plane qn - T, read at this trip's last level
      const int sl = ring_slot(qn);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        sC[sl][0][R * w + r][lane] = __uint_as_float(RQ[r].x);
        sC[sl][1][R * w + r][lane] = __uint_as_float(RQ[r].y);
        sC[sl][2][R * w + r][lane] = __uint_as_float(RQ[r].z);
      }
    }
    if (DEFER) {
#pragma unroll
      for (int r = 0; r < R; ++r) Hs[r] = Hc[r];
    } else {
      store_plane(X, En, Hc);
    }
  }
  if (DEFER) {
    F3<V> Es[R];
#pragma unroll
    for (int r = 0; r < R; ++r) Es[r] = Ep[T - 1][r];
    store_plane(i1 + T - 1, Es, Hs);
  }
  };
  if (tile_all && !(xcd_swz & 2))
    run(std::true_type{});
  else
    run(std::false_type{});
}


// x planes per workgroup.  A workgroup streams xchunk + 2T planes (T lead-in
// and T drain planes are re-read), and every variant holds ONE 16-wave
// workgroup per CU, so with uniform workgroups the pass takes
// ceil(G / CUs) rounds of (xchunk + 2T) plane steps, G = (y, z tiles) x
// ceil(nx / xchunk).  Pick the xchunk (nx split into k near-equal chunks)
// minimising that: long chunks for big grids, many short ones for the thin
// shells of a decomposed run (a 5-row y shell is 19 tiles: 13 chunks of 20
// planes fill the chip in one round instead of one 266-plane workgroup per
// tile).  Passes of several rounds then cap the chunk at 256 planes (see
// below).
int g_num_cus = 0;
int pick_xchunk(long long tiles_yz, int nxo, int T, int wg_per_cu = 1) {
  if (g_num_cus <= 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      g_num_cus = n;
    else
      g_num_cus = 256;
  }
  if (nxo <= 0) return 1;
  const long long slots = (long long)g_num_cus * wg_per_cu;
  // cap: the longest chunk considered (multi-round passes, below)
  auto search = [&](int cap, long long* rounds_out) {
    long long best_cost = -1, best_rounds = 1;
    int best = nxo;
    for (int k = 1; k <= 256; ++k) {
      const int xc = (nxo + k - 1) / k;
      if (xc > cap) continue;
      const long long chunks = (nxo + xc - 1) / xc;
      const long long rounds = (tiles_yz * chunks + slots - 1) / slots;
      const long long cost = rounds * (xc + 2LL * T);
      if (best_cost < 0 || cost < best_cost) {
        best_cost = cost;
        best = xc;
        best_rounds = rounds;
      }
      if (xc == 1) break;
    }
    *rounds_out = best_rounds;
    return best;
  };
  long long rounds = 1;
  const int best = search(nxo, &rounds);
  // A pass of several rounds balances better over the CUs with chunks of at
  // most 256 planes than the uniform-workgroup model predicts (measured T=5:
  // 1024^3 297k vs 288k Mcells/s at 256 vs 512 planes, 2048x1024x1024 293k vs
  // 263k at 256 vs 1024); a one-round pass keeps its long chunks (512^3:
  // 247k at 512 planes vs 236k at 256).
  if (rounds >= 2 && best > 256) return search(256, &rounds);
  return best;
}

int g_tb_vec = 0;   // 0: automatic (float4 lanes for T <= 2, float2 above), else 2 / 4
int g_tb_rows = 0;  // rows per wave: 0 automatic (1), 1 / 2
int g_tb_xcd = 0;   // XCD-aware tile order (measured: no gain, T=2 slower; off by default)

template <int T, int V, int R, bool PERCELL>
int launch_tb(const float* const* ein, const float* const* hin, float* const* eout, float* const* hout,
              const float* const* cbs, const float* const* dbs, float cb, float db, int nx, int ny, int nz,
              const Box3* b, const Box3& O, int xchunk, const int* src, const TbSrc& sv, hipStream_t s) {
  constexpr int HL = (T + V - 1) / V;
  constexpr int TBZ = (64 / R - 2 * HL) * V;
  dim3 grid(cdiv(O.hi[2] - (O.lo[2] & ~(V - 1)), TBZ), cdiv(O.hi[1] - O.lo[1], TBW * R - 2 * T),
            cdiv(O.hi[0] - O.lo[0], xchunk));
  k_tb3d<T, V, R, PERCELL><<<grid, dim3(64, TBW), 0, s>>>(
      ein[0], ein[1], ein[2], hin[0], hin[1], hin[2], eout[0], eout[1], eout[2], hout[0], hout[1], hout[2],
      cbs[0], cbs[1], cbs[2], dbs[0], dbs[1], dbs[2], cb, db, nx, ny, nz, b[0], b[1], b[2], b[3], b[4], b[5], O,
      xchunk, src[0], src[1], src[2], src[3], sv, g_tb_xcd);
  FDTD_RETURN_LAUNCH_STATUS();
}

template <int T, int V, int R>
int launch_tb_pc(bool pc, const float* const* ein, const float* const* hin, float* const* eout,
                 float* const* hout, const float* const* cbs, const float* const* dbs, float cb, float db, int nx,
                 int ny, int nz, const Box3* b, const Box3& O, int xchunk, const int* src, const TbSrc& sv,
                 hipStream_t s) {
  return pc ? launch_tb<T, V, R, true>(ein, hin, eout, hout, cbs, dbs, cb, db, nx, ny, nz, b, O, xchunk, src, sv, s)
            : launch_tb<T, V, R, false>(ein, hin, eout, hout, cbs, dbs, cb, db, nx, ny, nz, b, O, xchunk, src, sv,
                                        s);
}

// two rows per wave from 4 steps per pass on (T=4: 246-267k vs 247-260k
// Mcells/s single-row at 1024^3; T=3: 162k vs 207k, so single-row below)
constexpr int MR_AUTO_ROWS = 2;
int g_tb_mrows = 0;  // rows per wave of the multi-row kernel: 0 automatic, 1 = single-row kernel, 2 / 4

int g_tb_mr_noallin = 0;  // A/B knob: 1 = masked loop everywhere (no interior fast path)
int g_tb_mr_xcd = 1;   // multi-row kernel: XCD-contiguous tile order, z fastest (-16..20% HBM reads)
// patch order of the XCD-contiguous tile run (k_tb3d_mr): (pz << 8) | (py << 16),
// 0 = z fastest; FDTD3D_TB_PATCH="PZxPY" (e.g. 4x8) at first use
int g_tb_patch = -1;
int tb_patch_bits() {
  if (g_tb_patch < 0) {
    g_tb_patch = 0;
    const char* e = getenv("FDTD3D_TB_PATCH");
    int pz = 0, py = 0;
    if (e && sscanf(e, "%dx%d", &pz, &py) == 2 && pz > 0 && py > 0 && pz < 256 && py < 256)
      g_tb_patch = (pz << 8) | (py << 16);
  }
  return g_tb_patch;
}
int g_tb_variant = 0;  // multi-row kernel: bit 0 deferred stores, bit 1 two planes prefetched
// multi-step CPML scratch loads: 0 agent scope (default), 1 plain (FDTD3D_CPML_SCR_L1=1, tuning)
int cpml_scr_l1() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("FDTD3D_CPML_SCR_L1");
    v = (e && e[0] == '1') ? 1 : 0;
  }
  return v;
}
const int kNoBox[6] = {0, 0, 0, 0, 0, 0};
int g_tb_mr_shape = 0;  // plain multi-row kernel: 0 = 16 waves x 2 rows, 1 = 8 waves x 4 rows

template <int T, int V, int R, int FX, int NW = TBW>
int launch_tb_mr(const float* const* ein, const float* const* hin, float* const* eout, float* const* hout,
                 const float4* ce4, const float4* ch4, const Box3& BE, const Box3& BH, float cb, float db, int nx,
                 int ny, int nz, const Box3* b, const Box3& O, int xchunk, const int* src, const TbSrc& sv,
                 const TfDev* tf, const float* gtab, const CpmlDev* cp, float* pscr, hipStream_t s) {
  constexpr int HL = (T + V - 1) / V;
  constexpr int TBZ = (64 - 2 * HL) * V;
  dim3 grid(cdiv(O.hi[2] - (O.lo[2] & ~(V - 1)), TBZ), cdiv(O.hi[1] - O.lo[1], NW * R - 2 * T),
            cdiv(O.hi[0] - O.lo[0], xchunk));
  CpArg<(FX & 8) != 0> cpv{};
  if constexpr ((FX & 8) != 0) cpv.d = *cp;
#define MR_LAUNCH(PFD, DEFER)                                                                                 \
  k_tb3d_mr<T, V, R, FX, PFD, DEFER, NW><<<grid, dim3(64, NW), 0, s>>>(                                     \
      ein[0], ein[1], ein[2], hin[0], hin[1], hin[2], eout[0], eout[1], eout[2], hout[0], hout[1], hout[2], \
      ce4, ch4, BE, BH, cb, db, nx, ny, nz, b[0], b[1], b[2], b[3], b[4], b[5],                             \
      O, xchunk, src[0], src[1], src[2], src[3], sv,                                                       \
      (g_tb_mr_xcd ? (1 | (g_tb_mr_noallin << 1) | tb_patch_bits()) : (g_tb_mr_noallin << 1)) |          \
          (cpml_scr_l1() << 24),                                                                           \
      tf, gtab, cpv, pscr)
  if constexpr (FX != 0) {
    MR_LAUNCH(1, false);  // tuning variants: uniform media only
  } else {
    switch (g_tb_variant & 3) {
      case 0: MR_LAUNCH(1, false); break;
      case 1: MR_LAUNCH(1, true); break;
      case 2: MR_LAUNCH(2, false); break;
      default: MR_LAUNCH(2, true); break;
    }
  }
#undef MR_LAUNCH
  FDTD_RETURN_LAUNCH_STATUS();
}

// tile of the multi-step CPML passes: CPML_NW waves x CPML_R rows
constexpr int CPML_NW = 8, CPML_R = 2;

template <int T>
int launch_tb_mr_sel(int fx, const float* const* ein, const float* const* hin, float* const* eout,
                     float* const* hout, const float4* ce4, const float4* ch4, const Box3& BE, const Box3& BH,
                     float cb, float db, int nx, int ny, int nz, const Box3* b, const Box3& O, int xchunk,
                     const int* src, const TbSrc& sv, const TfDev* tf, const float* gtab, const CpmlDev* cp,
                     float* pscr, hipStream_t s) {
  // scalar lanes with 2 rows per wave: R = 4 or float2 lanes at R = 2
  // exceed 128 VGPRs and spill from T = 2 on
#define MR_ARGS ein, hin, eout, hout, ce4, ch4, BE, BH, cb, db, nx, ny, nz, b, O, xchunk, src, sv, tf, gtab, cp, pscr, s
  if constexpr (T == 1) {
    // CPML single-step passes (hybrid shells)
    switch (fx) {
      case 8: return launch_tb_mr<T, 1, 2, 8>(MR_ARGS);
      case 9: return launch_tb_mr<T, 1, 2, 9>(MR_ARGS);
      case 10: return launch_tb_mr<T, 1, 2, 10>(MR_ARGS);
      case 11: return launch_tb_mr<T, 1, 2, 11>(MR_ARGS);
      case 12: return launch_tb_mr<T, 1, 2, 12>(MR_ARGS);
      case 13: return launch_tb_mr<T, 1, 2, 13>(MR_ARGS);
      case 14: return launch_tb_mr<T, 1, 2, 14>(MR_ARGS);
      case 15: return launch_tb_mr<T, 1, 2, 15>(MR_ARGS);
    }
  } else if constexpr (T <= 5) {
    // multi-step CPML (+ TF/SF) passes over the shell boxes of a hybrid run
    switch (fx) {
      case 8: return launch_tb_mr<T, 1, CPML_R, 8, CPML_NW>(MR_ARGS);
      case 12: return launch_tb_mr<T, 1, CPML_R, 12, CPML_NW>(MR_ARGS);
    }
    if (fx & 8) return (int)hipErrorInvalidValue;
  } else {
    if (fx & 8) return (int)hipErrorInvalidValue;
  }
  // per-cell: one kind keeps T coefficient planes in LDS (24 KiB each, 160
  // KiB per CU: T <= 5); both kinds keep them in registers (spill-free to T = 2)
  if constexpr (T <= 5) {
    switch (fx) {
      case 1: return launch_tb_mr<T, 1, 2, 1>(MR_ARGS);
      case 2: return launch_tb_mr<T, 1, 2, 2>(MR_ARGS);
      case 3: return launch_tb_mr<T, 1, 2, 3>(MR_ARGS);
      case 4: return launch_tb_mr<T, 1, 2, 4>(MR_ARGS);
      case 5: return launch_tb_mr<T, 1, 2, 5>(MR_ARGS);
      case 6: return launch_tb_mr<T, 1, 2, 6>(MR_ARGS);
      case 7: return launch_tb_mr<T, 1, 2, 7>(MR_ARGS);
    }
  } else {
    if (fx) return (int)hipErrorInvalidValue;
  }
  // plain: 16 waves x 2 rows (4 waves / SIMD, <= 128 VGPRs) or 8 waves x 4
  // rows (2 waves / SIMD, <= 256 VGPRs: more rows of ILP per wave, half the
  // LDS row exchanges); both a 32-row tile
  if (g_tb_mr_shape == 1) return launch_tb_mr<T, 1, 4, 0, 8>(MR_ARGS);
  return launch_tb_mr<T, 1, 2, 0>(MR_ARGS);
#undef MR_ARGS
}

// automatic x chunk of a multi-row pass over output box O
int tb_mr_xchunk(int fx, const Box3& O, int steps) {
  const bool cpm = (fx & 8) && steps > 1;
  const int R = cpm ? CPML_R : 2, NW = cpm ? CPML_NW : TBW;
  const long long gz = cdiv(O.hi[2] - O.lo[2], 64 - 2 * steps);
  const long long gy = cdiv(O.hi[1] - O.lo[1], NW * R - 2 * steps);
  // the 8-wave shape fits two workgroups per CU
  return pick_xchunk(gz * gy, O.hi[0] - O.lo[0], steps, (fx == 0 && g_tb_mr_shape == 1) || cpm ? 2 : 1);
}

// bytes of thread-private psi scratch a multi-step CPML pass needs (0: none)
long long tb_mr_scratch_bytes(int fx, const Box3& O, int steps, int xchunk) {
  if (!(fx & 8) || steps <= 1 || box_empty(O)) return 0;
  if (xchunk <= 0) xchunk = tb_mr_xchunk(fx, O, steps);
  const long long gz = cdiv(O.hi[2] - O.lo[2], 64 - 2 * steps);
  const long long gy = cdiv(O.hi[1] - O.lo[1], CPML_NW * CPML_R - 2 * steps);
  const long long gx = cdiv(O.hi[0] - O.lo[0], xchunk);
  return 2LL * (steps - 1) * 12 * CPML_R * gz * gy * gx * CPML_NW * 64 * 4;
}

// multi-row pass (scalar lanes, 2 rows per wave): uniform media, sparse
// per-cell coefficients (fx bits 1 / 2), TF/SF corrections (fx bit 4)
int tb_mr_dispatch(int fx, const float* const* ein, const float* const* hin, float* const* eout,
                   float* const* hout, const float4* ce4, const float4* ch4, const Box3& BE, const Box3& BH,
                   float cb, float db, int nx, int ny, int nz, const Box3* b, const Box3& O, int xchunk, int steps,
                   const int* src, const TbSrc& sv, const TfDev* tf, const float* gtab, const CpmlDev* cp,
                   float* pscr, hipStream_t s) {
  if (xchunk <= 0) xchunk = tb_mr_xchunk(fx, O, steps);
#define MR_ARGS fx, ein, hin, eout, hout, ce4, ch4, BE, BH, cb, db, nx, ny, nz, b, O, xchunk, src, sv, tf, gtab, cp, pscr, s
  switch (steps) {
    case 1: return launch_tb_mr_sel<1>(MR_ARGS);
    case 2: return launch_tb_mr_sel<2>(MR_ARGS);
    case 3: return launch_tb_mr_sel<3>(MR_ARGS);
    case 4: return launch_tb_mr_sel<4>(MR_ARGS);
    case 5: return launch_tb_mr_sel<5>(MR_ARGS);
    case 6: return launch_tb_mr_sel<6>(MR_ARGS);
  }
#undef MR_ARGS
  return (int)hipErrorInvalidValue;
}

// Incident line + TF/SF g tables of one blocked pass (one workgroup): for
// each level l = 0..T-1 (step t + l) the E sets' values from the H line as
// it stands, the line's E half step (hard source at index 0), the H sets'
// values from the new E line, the line's H half step -- the order of the
// stepped scheme (models/scheme.py step).  Only the first `reach` cells of
// the line move: beyond the wave front every value is exactly 0.
__global__ __launch_bounds__(1024) void k_tfsf_pass(float* __restrict__ einc, float* __restrict__ hinc, int n,
                                                    float ce, float ch, TbSrc sv, int T, int reach, int nE, int nH,
                                                    const int* __restrict__ I0, const float* __restrict__ W0,
                                                    const float* __restrict__ W1, const float* __restrict__ C,
                                                    float* __restrict__ gtab) {
  const int tid = threadIdx.x;
  const int ld = nE + nH;
  const int m = min(n, reach);
  for (int l = 0; l < T; ++l) {
    for (int e = tid; e < nE; e += blockDim.x)
      gtab[l * ld + e] = C[e] * (W0[e] * hinc[I0[e]] + W1[e] * hinc[I0[e] + 1]);
    for (int i = tid; i < m; i += blockDim.x) einc[i] = i == 0 ? sv.v[l] : einc[i] + ce * (hinc[i - 1] - hinc[i]);
    __syncthreads();
    for (int e = nE + tid; e < ld; e += blockDim.x)
      gtab[l * ld + e] = C[e] * (W0[e] * einc[I0[e]] + W1[e] * einc[I0[e] + 1]);
    for (int i = tid; i < m && i < n - 1; i += blockDim.x) hinc[i] += ch * (einc[i] - einc[i + 1]);
    __syncthreads();
  }
}

}  // namespace

// lane width of the blocked kernel (tuning / tests): 0 = automatic, 2, 4
FDTD_API void fdtd_set_tb_vec(int v) { g_tb_vec = (v == 2 || v == 4) ? v : 0; }
// rows per wave of the blocked kernel: 0 = automatic, 1, 2 (2 rows of 32 lanes:
// a 32-row tile, halving the y-halo re-reads of float2 lanes)
FDTD_API void fdtd_set_tb_rows(int r) { g_tb_rows = (r == 1 || r == 2) ? r : 0; }
// XCD-aware tile order of the blocked kernel (1 = on, default)
FDTD_API void fdtd_set_tb_xcd(int on) { g_tb_xcd = on ? 1 : 0; }
// adjacent y rows carried per wave (k_tb3d_mr): 0 = automatic, 1 = the
// single-row kernel, 2
FDTD_API void fdtd_set_tb_mrows(int r) { g_tb_mrows = (r == 1 || r == 2) ? r : 0; }
// multi-row kernel variant (tuning): bit 0 deferred stores, bit 1 two planes
// prefetched, bit 2 XCD-contiguous tile order
FDTD_API void fdtd_set_tb_variant(int v) {
  g_tb_variant = v & 3;
  g_tb_mr_xcd = (v >> 2) & 1;      // bit 2: XCD-contiguous tile order
  g_tb_mr_noallin = (v >> 3) & 1;  // bit 3: no interior fast path (A/B)
}
// patch order of the multi-row kernel's XCD tile run: pz x py tiles (0: z fastest)
FDTD_API void fdtd_set_tb_patch(int pz, int py) {
  g_tb_patch = (pz > 0 && py > 0 && pz < 256 && py < 256) ? ((pz << 8) | (py << 16)) : 0;
}
// plain multi-row tile shape (tuning): 0 = 16 waves x 2 rows, 1 = 8 waves x 4 rows
FDTD_API void fdtd_set_tb_mr_shape(int v) { g_tb_mr_shape = v == 1 ? 1 : 0; }
// largest steps-per-pass the blocked kernels accept
FDTD_API int fdtd_tb_max_steps() { return 6; }

// T fused leapfrog steps: reads ein/hin, writes eout/hout (distinct buffers)
// on the output box `obox` (lo[3], hi[3]).  `boxes` = 6 update boxes
// (Ex Ey Ez Hx Hy Hz).  `src` = {i, j, k, comp} of a hard E point source (comp
// -1: none) with the value of each of the T E half steps in `src_vals`.
FDTD_API int fdtd_tb3d_v4_f32(const float* const* ein, const float* const* hin, float* const* eout,
                              float* const* hout, const float* const* cbs, const float* const* dbs, double cb,
                              double db, int nx, int ny, int nz, const int* boxes, const int* obox, int xchunk,
                              int steps, const int* src, const double* src_vals, void* stream) {
  if (nz % 4 != 0 || steps < 1 || steps > 6) return (int)hipErrorInvalidValue;
  Box3 b[6];
  for (int n = 0; n < 6; ++n) b[n] = make_box(boxes + 6 * n);
  const Box3 O = make_box(obox);
  if (box_empty(O)) return 0;
  TbSrc sv;
  for (int l = 0; l < 8; ++l) sv.v[l] = (src[3] >= 0 && l < steps) ? (float)src_vals[l] : 0.f;
  hipStream_t s = (hipStream_t)stream;
  // per-cell coefficients of either kind (a null kind uses its scalar)
  const bool pc = cbs[0] != nullptr || dbs[0] != nullptr;
  const float fcb = (float)cb, fdb = (float)db;
  // multi-row kernel for uniform media: automatic from 4 steps on, required
  // above 4 (full per-cell planes run on the single-row kernel; the sparse
  // per-cell form is fdtd_tb3d_sparse_f32)
  const int MR = g_tb_mrows ? g_tb_mrows : (steps >= 4 && !pc ? MR_AUTO_ROWS : 1);
  if (!pc && (MR > 1 || steps > 4)) {
    const Box3 nb = make_box(kNoBox);
    return tb_mr_dispatch(0, ein, hin, eout, hout, nullptr, nullptr, nb, nb, fcb, fdb, nx, ny, nz, b, O, xchunk,
                          steps, src, sv, nullptr, nullptr, nullptr, nullptr, s);
  }
  if (steps > 4) return (int)hipErrorInvalidValue;
  if (xchunk <= 0) {
    const int V = g_tb_vec ? g_tb_vec : (steps <= 2 ? 4 : 2);
    const int R = g_tb_rows ? g_tb_rows : 1;
    const int HL = (steps + V - 1) / V;
    const long long gz = cdiv(O.hi[2] - (O.lo[2] & ~(V - 1)), (64 / R - 2 * HL) * V);
    const long long gy = cdiv(O.hi[1] - O.lo[1], TBW * R - 2 * steps);
    xchunk = pick_xchunk(gz * gy, O.hi[0] - O.lo[0], steps);
  }
  const int V = g_tb_vec ? g_tb_vec : (steps <= 2 ? 4 : 2);
  const int R = g_tb_rows ? g_tb_rows : 1;  // 2 rows per wave measured slower (228k vs 245k, T=4)
#define TB_ARGS pc, ein, hin, eout, hout, cbs, dbs, fcb, fdb, nx, ny, nz, b, O, xchunk, src, sv, s
#define TB_CASE(TT)                                                                     \
  case TT:                                                                              \
    if (V == 4) return R == 2 ? launch_tb_pc<TT, 4, 2>(TB_ARGS) : launch_tb_pc<TT, 4, 1>(TB_ARGS); \
    return R == 2 ? launch_tb_pc<TT, 2, 2>(TB_ARGS) : launch_tb_pc<TT, 2, 1>(TB_ARGS);
  switch (steps) {
    TB_CASE(1)
    TB_CASE(2)
    TB_CASE(3)
    TB_CASE(4)
  }
#undef TB_CASE
#undef TB_ARGS
  return (int)hipErrorInvalidValue;
}

// T fused leapfrog steps on the multi-row kernel with its extensions:
// sparse per-cell coefficients -- ``ce4`` / ``ch4`` hold the E / H
// coefficients of the three components as one float4 per cell of the box
// ``ebox`` / ``hbox`` (x-major, z fastest, .w unused); every cell outside its
// kind's box, and either kind whose array is null, uses the scalar ``cb`` /
// ``db`` -- TF/SF corrections (``tf`` = device TfDev, ``gtab`` = the g
// table of this pass's first level, from fdtd_tfsf_pass_f32; null: none) and,
// CPML (``cpml`` = the CpmlDev block as HOST bytes, passed by value to the
// kernel; passes of more than one step need ``pscr``, ``pscr_bytes`` >=
// fdtd_tb3d_cpml_scratch_bytes; null: none).
// Other arguments as fdtd_tb3d_v4_f32.
FDTD_API int fdtd_tb3d_ext_f32(const float* const* ein, const float* const* hin, float* const* eout,
                               float* const* hout, const void* ce4, const int* ebox, const void* ch4,
                               const int* hbox, double cb, double db, int nx, int ny, int nz, const int* boxes,
                               const int* obox, int xchunk, int steps, const int* src, const double* src_vals,
                               const void* tf, const float* gtab, const void* cpml, void* pscr,
                               long long pscr_bytes, void* stream) {
  if (nz % 4 != 0 || steps < 1 || steps > 6) return (int)hipErrorInvalidValue;
  if (cpml && steps > 5) return (int)hipErrorInvalidValue;
  Box3 b[6];
  for (int n = 0; n < 6; ++n) b[n] = make_box(boxes + 6 * n);
  const Box3 O = make_box(obox);
  if (box_empty(O)) return 0;
  const Box3 BE = make_box(ce4 ? ebox : kNoBox), BH = make_box(ch4 ? hbox : kNoBox);
  TbSrc sv;
  for (int l = 0; l < 8; ++l) sv.v[l] = (src[3] >= 0 && l < steps) ? (float)src_vals[l] : 0.f;
  const int fx = (ce4 && !box_empty(BE) ? 1 : 0) | (ch4 && !box_empty(BH) ? 2 : 0) | (tf && gtab ? 4 : 0) |
                 (cpml ? 8 : 0);
  if ((fx & 8) && steps > 1) {
    // multi-step CPML: uniform media only; the caller's scratch must cover the launch
    if (fx & 3) return (int)hipErrorInvalidValue;
    if (xchunk <= 0) xchunk = tb_mr_xchunk(fx, O, steps);
    if (!pscr || pscr_bytes < tb_mr_scratch_bytes(fx, O, steps, xchunk) ||
        tb_mr_scratch_bytes(fx, O, steps, xchunk) > 0xFFFFFFFFLL)
      return (int)hipErrorInvalidValue;
  }
  return tb_mr_dispatch(fx, ein, hin, eout, hout, (const float4*)(box_empty(BE) ? nullptr : ce4),
                        (const float4*)(box_empty(BH) ? nullptr : ch4), BE, BH, (float)cb, (float)db, nx, ny, nz, b,
                        O, xchunk, steps, src, sv, (const TfDev*)tf, gtab, (const CpmlDev*)cpml, (float*)pscr,
                        (hipStream_t)stream);
}

// scratch bytes fdtd_tb3d_ext_f32 needs for a CPML pass of ``steps`` steps
// over output box ``obox`` (TF/SF on or off; 0 for single-step passes)
FDTD_API long long fdtd_tb3d_cpml_scratch_bytes(const int* obox, int xchunk, int steps, int tfsf) {
  return tb_mr_scratch_bytes(8 | (tfsf ? 4 : 0), make_box(obox), steps, xchunk);
}

// size of the CpmlDev block the host fills (ABI check)
FDTD_API int fdtd_cpmldev_size() { return (int)sizeof(CpmlDev); }

// size of the TfDev block the host fills (ABI check)
FDTD_API int fdtd_tfdev_size() { return (int)sizeof(TfDev); }

// incident line advanced ``steps`` steps from step t (source value per step
// in ``src_vals``) and the per-level g tables of the pass (k_tfsf_pass)
FDTD_API int fdtd_tfsf_pass_f32(float* einc, float* hinc, int n, double ce, double ch, const double* src_vals,
                                int steps, int reach, int nE, int nH, const int* I0, const float* W0,
                                const float* W1, const float* C, float* gtab, void* stream) {
  if (steps < 1 || steps > 8) return (int)hipErrorInvalidValue;
  TbSrc sv;
  for (int l = 0; l < 8; ++l) sv.v[l] = l < steps ? (float)src_vals[l] : 0.f;
  k_tfsf_pass<<<1, 1024, 0, (hipStream_t)stream>>>(einc, hinc, n, (float)ce, (float)ch, sv, steps, reach, nE, nH,
                                                   I0, W0, W1, C, gtab);
  FDTD_RETURN_LAUNCH_STATUS();
}
