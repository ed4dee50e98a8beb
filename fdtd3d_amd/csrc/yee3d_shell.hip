// Single-step fused E+H passes over the SHELL of a hybrid pass (fp32, 3D).
//
// A hybrid pass (models/blocking.py) advances the core of the grid -- every
// cell at least PML + T + 2 (TF/SF box + T + 3 with a plane wave) away from
// the faces -- T steps at a time through the temporally blocked kernel
// (yee3d_tb.hip), and the shell around it one step at a time over windows
// that shrink by one cell per step (the deep-halo rule of the reference's
// ParallelGrid.cpp:2365-2489, applied to the core boundary).  This kernel
// is that single step: E^{n+1} and H^{n+1} in ONE pass (read E^n, H^n once,
// write both once: 48 B/cell against 72 B for separate E and H kernels),
// over a work list of shell boxes in one launch, with the CPML convolution
// terms (models/cpml.py) of the absorbing layers folded in.  The reference
// updates its UPML cells with three sweeps per component
// (Scheme3D.cpp:266-416); its CUDA path has no absorbing layer at all.
//
// Tile: 16 waves x 64 lanes.  Lanes run along z: LW = 64 lanes per grid row,
// or LW = 32 (two grid rows per wave) for boxes at most 30 cells deep in z --
// the z shell slabs -- where 64-lane rows would leave half the lanes idle.
// Every lane group carries R = 2 adjacent y rows in registers; the first /
// last row of a group exchanges its y neighbours through a double-buffered
// LDS slot (one barrier per plane); z neighbours come through DPP lane
// shifts (lanes shifted in across a row-group boundary are halo lanes).  The
// workgroup streams x: trip X loads plane X, computes E^{n+1}(X) from H^n(X),
// H^n(X-1) (carried) and H^{n+1}(X-1) from E^{n+1}(X-1) (carried) and
// E^{n+1}(X).  One halo lane / row per side: halo cells are recomputed by the
// neighbour tile, so the CPML psi of a step is read from one copy and written
// to the other (models/cpml.py flip).
//
// CPML (models/cpml.py: psi = b psi + c d, curl += sign ((1/kappa - 1) d +
// psi)) is specialised per launch by the set AX of axes whose absorbing slab
// the launch's boxes touch (bit 0 x, 1 y, 2 z): a face slab carries 4 of the
// 12 terms, the interior band none; edges and corners take all axes.  A
// term's slab side is wave-uniform along x (plane) and, for 64-lane rows,
// along y (row); along z it is per lane.  Loads past a buffer descriptor read
// 0 and stores past it are dropped: lanes outside a slab use such offsets.
//
// TF/SF corrections are NOT in this kernel: they are additive, so the host
// adds Cb g to the E targets of the input buffer before the pass and Db g to
// the H targets of the output after it (models/blocking.py _hybrid2_step).

#include <cstring>
#include <cstdlib>
#include "common.h"

namespace {

typedef __amdgpu_buffer_rsrc_t Rsrc;

__device__ __forceinline__ float sh_up(float v) {  // lane i <- lane i-1
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float sh_dn(float v) {  // lane i <- lane i+1
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, false));
}

__device__ __forceinline__ Rsrc mk_rs(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ Rsrc plane_rs(const float* base, int x, int nx, size_t plane) {
  const bool in = x >= 0 && x < nx;
  return mk_rs(base + (size_t)(in ? x : 0) * plane, in ? (unsigned)(plane * 4) : 0u);
}
__device__ __forceinline__ float ldf(Rsrc r, unsigned off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ void stf(Rsrc r, unsigned off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}

constexpr unsigned kBad = 0xF0000000u;  // byte offset past every descriptor

// one (component, term axis) of the CPML: the layout of models/cpml.py
// device_table (and yee3d_tb.hip CpmlDev)
struct ShTerm {
  const float* psi[2];  // low / high slab, read (time n)
  float* out[2];        // written (time n + 1)
  int lo[2], hi[2];     // slab ranges along the axis (local; z padded to float4 groups)
  const float* b;
  const float* c;
  const float* k;       // 1 / kappa - 1
};
struct ShCpml {
  ShTerm t[6][3];  // [Ex Ey Ez Hx Hy Hz][axis]
};

// UPML in the reference's D/B form (Scheme3D.cpp:266-416, models/scheme.py
// _init_upml) over the shell, with the D (B) levels stored only where some
// sigma is non-zero: the 6 disjoint boxes of alloc minus the all-sigma-zero
// core I (x slabs over the whole y, z extent; y slabs over I's x range; z
// slabs over I's x, y ranges -- models/upml.py UPMLRegions).  Per component,
// with its profiles as (a, b) pairs per axis -- (caD, cbD) along aD, (caE,
// ica) along aCa, (cbEa, ccEa) along aCb:
//   Dn = caD D + cbD curl ;  E = caE E + s ica (cbEa Dn + ccEa D)
// D is read from one copy and written to the other (halo cells are
// recomputed by neighbour tiles); cells of no box run the same formula with
// D = 0, which is the plain update where every sigma vanishes.
struct ShUpml {
  int blo[6][3], bhi[6][3];   // D storage boxes (local): x-lo, x-hi, y-lo, y-hi, z-lo, z-hi
  const float* d[6][6];       // [component][box] D^n
  float* dn[6][6];            // [component][box] D^{n+1}
  const float2* pr[6][3];     // [component][axis] profile pairs over the local extent
  float s[6];                 // scalar of the E-from-D term
  int pad;
};
// Dispersive box (AX == 9): Drude / Lorentz media in the reference's chain
// form (Kernels.h:103-107, Scheme3D.cpp:326-364; models/scheme.py
// _init_upml) on the bounding box of the dispersive cells, where every sigma
// vanishes (caD = caE = 1 etc. as scalars).  Per component with dispersion:
// three D and D1 levels over the box (cur, prev, next -- the next level is
// the one no tile reads this step), a uint8 material index + 1 (0: the cell
// lies outside its row's material range and takes the plain update, exactly
// the row split of the stepped chain) and the (b0, b1, b2, ma1, ma2) table:
//   Dn = caD D + cbD curl ; D1n = b0 Dn + b1 D + b2 Dp + ma1 D1 + ma2 D1p
//   E  = caE E + sica (cbEa D1n + ccEa D1)
constexpr int SH_LUT = 16;  // coefficient tuples per component (more: stepped shell)
struct ShDrude {
  int lo[3], hi[3];
  const float* d[6][3];       // [component][cur, prev, next]
  const float* d1[6][3];
  const unsigned char* id[6]; // null: no dispersion in this component (plain update)
  const float* lut[6];        // (nlut, 5)
  float caD[6], cbD[6], caE[6], sica[6], cbEa[6], ccEa[6];
  int nlut[6];
};

// (aD, aCa, aCb) per component (layout/yee.py UPML_AXES)
__device__ constexpr int kUp[6][3] = {{1, 2, 0}, {2, 0, 1}, {0, 1, 2}, {1, 2, 0}, {2, 0, 1}, {0, 1, 2}};

// curl terms of each component: (axis of term 0, axis of term 1); the curl is
// +d0 - d1 (Ex = dHz/dy - dHy/dz, ..., Hx = dEy/dz - dEz/dy, ...)
__device__ constexpr int kAx[6][2] = {{1, 2}, {2, 0}, {0, 1}, {2, 1}, {0, 2}, {1, 0}};

constexpr int SH_MAX = 32;  // boxes per launch
struct ShList {
  int n;
  int first[SH_MAX + 1];  // first workgroup of each box; first[n] = grid size
  int tz[SH_MAX], ty[SH_MAX], xc[SH_MAX];
  Box3 box[SH_MAX];
};

// the CPML / UPML / dispersive block of a launch travels BY VALUE in the
// kernel arguments: kernarg loads are invariant, so the compiler keeps the
// psi / D descriptors in SGPRs (or re-reads them at will) instead of reloading
// them from global memory after every buffer store that might alias them --
// a dependent scalar-load chain per term and trip
union ShAux {
  ShCpml c;
  ShUpml u;
  ShDrude d;
};
constexpr int SR = 2;    // rows per lane group

template <int AX, bool KAP, int LW, int SNW>
__global__ __launch_bounds__(64 * SNW) void k_shell1(
    const float* __restrict__ exi, const float* __restrict__ eyi, const float* __restrict__ ezi,
    const float* __restrict__ hxi, const float* __restrict__ hyi, const float* __restrict__ hzi,
    float* __restrict__ exo, float* __restrict__ eyo, float* __restrict__ ezo, float* __restrict__ hxo,
    float* __restrict__ hyo, float* __restrict__ hzo, float cb, float db, int nx, int ny, int nz, Box3 bex,
    Box3 bey, Box3 bez, Box3 bhx, Box3 bhy, Box3 bhz, ShList L, int src_i, int src_j, int src_k, int src_comp,
    float src_v, const ShAux A) {
  constexpr int G = 64 / LW;         // lane groups (grid rows) per wave
  constexpr int NS = SNW * G;        // lane groups per workgroup
  constexpr int ROWS = NS * SR;      // y rows per tile
  constexpr bool UP = AX == 8;       // UPML launch (no CPML terms)
  constexpr bool DR = AX == 9;       // dispersive-box launch
  constexpr bool CPX = AX < 8 && (AX & 1), CPY = AX < 8 && (AX & 2), CPZ = AX < 8 && (AX & 4);
  constexpr bool CPM = AX < 8 && AX != 0;
  __shared__ float sX[2][4][NS][LW];
  // the CPML / UPML / dispersive blocks are read straight from (constant)
  // global memory with wave-uniform addresses: scalar loads into SGPRs, so
  // the psi / D descriptors built from them need no waterfall loop (an LDS
  // copy would hand the pointers back in VGPRs)
  const ShTerm* sT = &A.c.t[0][0];
  const int lane = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.y);
  const int g = LW == 64 ? 0 : lane / LW;
  const int li = LW == 64 ? lane : lane % LW;
  const int slot = w * G + g;
  const ShUpml& U = A.u;    // UPML launches only
  const ShDrude& DB = A.d;  // dispersive launches only
  __shared__ float sL[DR ? 6 : 1][DR ? SH_LUT * 5 : 1];
  if constexpr (DR) {
    // the coefficient tuples ARE indexed per lane (by material id): LDS
    for (int q = lane + 64 * w; q < 6 * SH_LUT * 5; q += 64 * SNW) {
      const int n = q / (SH_LUT * 5), e = q % (SH_LUT * 5);
      sL[n][e] = (DB.id[n] && e < 5 * DB.nlut[n]) ? DB.lut[n][e] : 0.f;
    }
    __syncthreads();
  }
  // ---- box and tile of this workgroup (wave-uniform)
  // (static indices only: a dynamic index into the by-value list would copy
  // it to scratch)
  const int bid = blockIdx.x;
  Box3 O = L.box[0];
  int first = 0, ntz = L.tz[0], nty = L.ty[0], xc = L.xc[0];
#pragma unroll
  for (int q = 1; q < SH_MAX; ++q)
    if (q < L.n && bid >= L.first[q]) {
      O = L.box[q];
      first = L.first[q];
      ntz = L.tz[q];
      nty = L.ty[q];
      xc = L.xc[q];
    }
  const int loc = bid - first;
  const int tz = loc % ntz, ty = (loc / ntz) % nty, tx = loc / (ntz * nty);
  const int i0 = O.lo[0] + tx * xc, i1 = min(i0 + xc, O.hi[0]);
  const int kb = O.lo[2] - 1 + (LW - 2) * tz + li;
  const int jr0 = O.lo[1] - 1 + (ROWS - 2) * ty + slot * SR;
  const bool kin = kb >= 0 && kb < nz;
  const size_t plane = (size_t)ny * nz;
  unsigned roff[SR];
  unsigned mbits = 0;  // bit r*7 + n: row r inside update box n (6 = stored)
  const Box3* bx[7] = {&bex, &bey, &bez, &bhx, &bhy, &bhz, &O};
#pragma unroll
  for (int r = 0; r < SR; ++r) {
    const int j = jr0 + r, t = slot * SR + r;
    const bool ok = kin && j >= 0 && j < ny;
    roff[r] = ok ? (unsigned)(j * nz + kb) * 4u : kBad;
    const bool own = ok && li >= 1 && li < LW - 1 && t >= 1 && t < ROWS - 1;
#pragma unroll
    for (int n = 0; n < 7; ++n) {
      const Box3& b = *bx[n];
      const bool in = (n < 6 ? ok : own) && j >= b.lo[1] && j < b.hi[1] && kb >= b.lo[2] && kb < b.hi[2];
      mbits |= (in ? 1u : 0u) << (r * 7 + n);
    }
  }
  const int rdn = slot > 0 ? slot - 1 : 0;
  const int rup = slot < NS - 1 ? slot + 1 : NS - 1;
  auto coef = [&](int n, int r, int p, float sc) -> float {
    const Box3& b = *bx[n];
    const bool in = (unsigned)(p - b.lo[0]) < (unsigned)(b.hi[0] - b.lo[0]) && ((mbits >> (r * 7 + n)) & 1u);
    return in ? sc : 0.f;
  };

  // ---- CPML: per-lane z offsets / profiles, per-row y offsets (tile constants)
  // E terms (n < 3) sit at plane X, H terms at X - 1.
  // y slab psi: ((i w + j - lo) nz + k); z slab psi: ((i ny + j) w + k - lo)
  unsigned yoff[2][2][SR], zoff[2][2][SR];  // [kind][side][row]
  bool yany[2][2] = {{false, false}, {false, false}}, zany[2][2] = {{false, false}, {false, false}};
  float zb[4], zc[4], zk[4];                // z terms Ex.1 Ey.0 Hx.0 Hy.1: profile at this lane
  if constexpr (CPY) {
#pragma unroll
    for (int kd = 0; kd < 2; ++kd) {
      const ShTerm& tm = sT[(kd == 0 ? 0 : 3) * 3 + 1];  // Ex / Hx y terms define the slab rows of the kind
#pragma unroll
      for (int sd = 0; sd < 2; ++sd) {
        bool any = false;
#pragma unroll
        for (int r = 0; r < SR; ++r) {
          const int j = jr0 + r;
          const bool in = tm.psi[sd] && kin && j >= tm.lo[sd] && j < tm.hi[sd];
          yoff[kd][sd][r] = in ? (unsigned)((j - tm.lo[sd]) * nz + kb) * 4u : kBad;
          any |= in;
        }
        yany[kd][sd] = __any(any);
      }
    }
  }
  if constexpr (CPZ) {
#pragma unroll
    for (int kd = 0; kd < 2; ++kd) {
      const ShTerm& tm = sT[(kd == 0 ? 0 : 3) * 3 + 2];  // Ex / Hx z terms
#pragma unroll
      for (int sd = 0; sd < 2; ++sd) {
        const bool in = tm.psi[sd] && kin && kb >= tm.lo[sd] && kb < tm.hi[sd];
        const int wd = tm.hi[sd] - tm.lo[sd];
#pragma unroll
        for (int r = 0; r < SR; ++r) {
          const int j = jr0 + r;
          zoff[kd][sd][r] = in && j >= 0 && j < ny ? (unsigned)(j * wd + kb - tm.lo[sd]) * 4u : kBad;
        }
        zany[kd][sd] = __any(in);
      }
    }
    const int zn[4] = {0, 1, 3, 4};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const ShTerm& tm = sT[zn[q] * 3 + 2];
      const bool in = kin && ((tm.psi[0] && kb >= tm.lo[0] && kb < tm.hi[0]) ||
                              (tm.psi[1] && kb >= tm.lo[1] && kb < tm.hi[1]));
      zb[q] = in ? tm.b[kb] : 1.f;
      zc[q] = in ? tm.c[kb] : 0.f;
      zk[q] = in && KAP ? tm.k[kb] : 0.f;
    }
  }

  // psi of term (n, t) on plane pl, row r: descriptor of the side that holds
  // this cell (x: by plane, y / z: both sides, offsets select) -- loaded into
  // ps[...] before the trip's field prefetch, updated and stored after use
  auto psi_load = [&](int n, int t, int pl, int r) -> float {
    const int a = kAx[n][t];
    const ShTerm& tm = sT[n * 3 + a];
    const int kd = n < 3 ? 0 : 1;
    float v = 0.f;
    if (pl < 0 || pl >= nx) return 0.f;
    if (a == 0) {
#pragma unroll
      for (int sd = 0; sd < 2; ++sd)
        if (tm.psi[sd] && pl >= tm.lo[sd] && pl < tm.hi[sd])
          v = ldf(mk_rs(tm.psi[sd] + (size_t)(pl - tm.lo[sd]) * plane, (unsigned)(plane * 4)), roff[r]);
    } else if (a == 1) {
#pragma unroll
      for (int sd = 0; sd < 2; ++sd)
        if (yany[kd][sd]) {
          const size_t pp = (size_t)(tm.hi[sd] - tm.lo[sd]) * nz;
          v += ldf(mk_rs(tm.psi[sd] + (size_t)pl * pp, (unsigned)(pp * 4)), yoff[kd][sd][r]);
        }
    } else {
#pragma unroll
      for (int sd = 0; sd < 2; ++sd)
        if (zany[kd][sd]) {
          const size_t pp = (size_t)ny * (tm.hi[sd] - tm.lo[sd]);
          v += ldf(mk_rs(tm.psi[sd] + (size_t)pl * pp, (unsigned)(pp * 4)), zoff[kd][sd][r]);
        }
    }
    return v;
  };
  // psi update of term (n, t) at plane pl, row r from the raw difference d:
  // returns the curl correction, stores the new psi for stored cells of the
  // component's update box
  auto psi_step = [&](int n, int t, int pl, int r, float ps, float d) -> float {
    const int a = kAx[n][t];
    const ShTerm& tm = sT[n * 3 + a];
    const int kd = n < 3 ? 0 : 1;
    // own cells only: halo planes / rows / lanes (recomputed here, owned by a
    // neighbour tile or chunk) must not write the psi copy
    const bool st = ((mbits >> (r * 7 + 6)) & 1u) && ((mbits >> (r * 7 + n)) & 1u) && pl >= i0 && pl < i1 &&
                    (unsigned)(pl - bx[n]->lo[0]) < (unsigned)(bx[n]->hi[0] - bx[n]->lo[0]);
    float b = 1.f, c = 0.f, k = 0.f;
    float r_ = 0.f;
    if (a == 0) {
      if (pl < 0 || pl >= nx) return 0.f;
#pragma unroll
      for (int sd = 0; sd < 2; ++sd)
        if (tm.psi[sd] && pl >= tm.lo[sd] && pl < tm.hi[sd]) {
          b = tm.b[pl];
          c = tm.c[pl];
          if (KAP) k = tm.k[pl];
          const float pn = b * ps + c * d;
          stf(mk_rs(tm.out[sd] + (size_t)(pl - tm.lo[sd]) * plane, (unsigned)(plane * 4)), st ? roff[r] : kBad, pn);
          r_ = k * d + pn;
        }
      return r_;
    } else if (a == 1) {
      const int j = jr0 + r;
      bool any = false;
#pragma unroll
      for (int sd = 0; sd < 2; ++sd) any |= yany[kd][sd];
      if (!any) return 0.f;
      const bool in = (tm.psi[0] && j >= tm.lo[0] && j < tm.hi[0]) || (tm.psi[1] && j >= tm.lo[1] && j < tm.hi[1]);
      if (in) {
        b = tm.b[j];
        c = tm.c[j];
        if (KAP) k = tm.k[j];
      }
      const float pn = b * ps + c * d;
#pragma unroll
      for (int sd = 0; sd < 2; ++sd)
        if (yany[kd][sd]) {
          const size_t pp = (size_t)(tm.hi[sd] - tm.lo[sd]) * nz;
          stf(mk_rs(tm.out[sd] + (size_t)pl * pp, (unsigned)(pp * 4)), st ? yoff[kd][sd][r] : kBad, pn);
        }
      return in ? k * d + pn : 0.f;
    } else {
      const int q = n == 0 ? 0 : (n == 1 ? 1 : (n == 3 ? 2 : 3));
      bool any = false;
#pragma unroll
      for (int sd = 0; sd < 2; ++sd) any |= zany[kd][sd];
      if (!any) return 0.f;
      const float pn = zb[q] * ps + zc[q] * d;
#pragma unroll
      for (int sd = 0; sd < 2; ++sd)
        if (zany[kd][sd]) {
          const size_t pp = (size_t)ny * (tm.hi[sd] - tm.lo[sd]);
          stf(mk_rs(tm.out[sd] + (size_t)pl * pp, (unsigned)(pp * 4)), st ? zoff[kd][sd][r] : kBad, pn);
        }
      return zk[q] * d + pn;  // 0 off the slab (b 1, c 0, k 0, psi 0)
    }
  };
  // which terms this launch carries: term (n, t) iff its axis is in AX
  auto term_on = [](int n, int t) -> bool { return CPM && ((AX >> kAx[n][t]) & 1); };

  // ---- UPML: D box offsets of the tile's rows / lanes (y and z boxes:
  // per-lane offsets, kBad off the box), z profile pairs of the lane
  unsigned uyo[2][SR], uzo[2][SR];  // [lo / hi box][row]
  bool uy_any[2] = {false, false}, uz_any[2] = {false, false};
  __shared__ float2 sUz[UP ? 6 : 1][UP ? LW : 1];  // z profile pairs of the tile's lanes
  if constexpr (UP) {
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      const int qy = 2 + sd, qz = 4 + sd;
      bool ay = false, az = false;
#pragma unroll
      for (int r = 0; r < SR; ++r) {
        const int j = jr0 + r;
        const bool iny = kin && j >= U.blo[qy][1] && j < U.bhi[qy][1] && kb >= U.blo[qy][2] && kb < U.bhi[qy][2];
        uyo[sd][r] = iny ? (unsigned)((j - U.blo[qy][1]) * (U.bhi[qy][2] - U.blo[qy][2]) + kb - U.blo[qy][2]) * 4u
                         : kBad;
        const bool inz = kin && j >= U.blo[qz][1] && j < U.bhi[qz][1] && kb >= U.blo[qz][2] && kb < U.bhi[qz][2];
        uzo[sd][r] = inz ? (unsigned)((j - U.blo[qz][1]) * (U.bhi[qz][2] - U.blo[qz][2]) + kb - U.blo[qz][2]) * 4u
                         : kBad;
        ay |= iny;
        az |= inz;
      }
      uy_any[sd] = __any(ay);
      uz_any[sd] = __any(az);
    }
    if (w == 0 && g == 0) {
#pragma unroll
      for (int n = 0; n < 6; ++n) sUz[n][li] = kin ? U.pr[n][2][kb] : make_float2(1.f, 0.f);
    }
    __syncthreads();
  }
  // descriptor of plane pl of D storage box q of component n (read / written copy)
  auto ud_rs = [&](int n, int q, int pl, bool wr) -> Rsrc {
    const size_t pp = (size_t)(U.bhi[q][1] - U.blo[q][1]) * (U.bhi[q][2] - U.blo[q][2]);
    const bool in = pl >= U.blo[q][0] && pl < U.bhi[q][0];
    const float* base = wr ? (const float*)U.dn[n][q] : U.d[n][q];
    return mk_rs(base + (size_t)(in ? pl - U.blo[q][0] : 0) * pp, in ? (unsigned)(pp * 4) : 0u);
  };
  // x box holding plane pl (-1: none); x boxes span the whole y / z extent
  auto ux_box = [&](int pl) -> int {
    return (pl >= U.blo[0][0] && pl < U.bhi[0][0]) ? 0 : ((pl >= U.blo[1][0] && pl < U.bhi[1][0]) ? 1 : -1);
  };
  // D of component n at plane pl, row r (0 outside every box)
  auto ud_load = [&](int n, int pl, int r) -> float {
    const int xb = ux_box(pl);
    if (xb >= 0) return ldf(ud_rs(n, xb, pl, false), roff[r]);
    float v = 0.f;
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      if (uy_any[sd]) v += ldf(ud_rs(n, 2 + sd, pl, false), uyo[sd][r]);
      if (uz_any[sd]) v += ldf(ud_rs(n, 4 + sd, pl, false), uzo[sd][r]);
    }
    return v;
  };
  auto ud_store = [&](int n, int pl, int r, float v, bool st) {
    const int xb = ux_box(pl);
    if (xb >= 0) {
      stf(ud_rs(n, xb, pl, true), st ? roff[r] : kBad, v);
      return;
    }
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      if (uy_any[sd]) stf(ud_rs(n, 2 + sd, pl, true), st ? uyo[sd][r] : kBad, v);
      if (uz_any[sd]) stf(ud_rs(n, 4 + sd, pl, true), st ? uzo[sd][r] : kBad, v);
    }
  };
  // profile pair of component n along axis a at plane pl / row r / this lane
  auto upair = [&](int n, int a, int pl, int r) -> float2 {
    if (a == 0) return U.pr[n][0][pl];
    if (a == 1) {
      const int j = jr0 + r;
      return (j >= 0 && j < ny) ? U.pr[n][1][j] : make_float2(1.f, 0.f);
    }
    return sUz[UP ? n : 0][UP ? li : 0];
  };
  // the UPML update of component n (E kind n < 3 on plane X, H on X - 1) from
  // its raw curl; returns the new field value
  auto upml = [&](int n, int pl, int r, float f, float curl, float Dv, bool upd, bool st) -> float {
    const float2 pD = upair(n, kUp[n][0], pl, r), pA = upair(n, kUp[n][1], pl, r);
    const float2 pB = upair(n, kUp[n][2], pl, r);
    const float Dn = pD.x * Dv + pD.y * curl;
    const float fn = pA.x * f + U.s[n] * pA.y * (pB.x * Dn + pB.y * Dv);
    ud_store(n, pl, r, Dn, upd && st);
    return upd ? fn : f;
  };

  // ---- dispersive box: element offset of each row's lane inside the box
  // (~0u off the box: byte / float loads past the descriptor read 0 = plain)
  unsigned dbo[SR];
  if constexpr (DR) {
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      const int j = jr0 + r;
      const bool in = kin && j >= DB.lo[1] && j < DB.hi[1] && kb >= DB.lo[2] && kb < DB.hi[2];
      dbo[r] = in ? (unsigned)((j - DB.lo[1]) * (DB.hi[2] - DB.lo[2]) + kb - DB.lo[2]) : 0x3C000000u;
    }
  }
  auto db_rs = [&](const void* base, int pl, unsigned esz) -> Rsrc {
    const size_t pp = (size_t)(DB.hi[1] - DB.lo[1]) * (DB.hi[2] - DB.lo[2]);
    const bool in = base && pl >= DB.lo[0] && pl < DB.hi[0];
    return mk_rs((const char*)base + (in ? (size_t)(pl - DB.lo[0]) * pp * esz : 0), in ? (unsigned)(pp * esz) : 0u);
  };
  // dispersive update of component n on plane pl, row r (plain where id = 0)
  auto drude = [&](int n, int pl, int r, float f, float curl, float pc, bool upd, bool st) -> float {
    const unsigned id = DB.id[n] ? __builtin_amdgcn_raw_buffer_load_b8(db_rs(DB.id[n], pl, 1), dbo[r], 0, 0) : 0u;
    if (id == 0u) return f + (upd ? pc : 0.f) * curl;
    const unsigned o = dbo[r] * 4u;
    const float D = ldf(db_rs(DB.d[n][0], pl, 4), o), Dp = ldf(db_rs(DB.d[n][1], pl, 4), o);
    const float D1 = ldf(db_rs(DB.d1[n][0], pl, 4), o), D1p = ldf(db_rs(DB.d1[n][1], pl, 4), o);
    const float* e = &sL[DR ? n : 0][DR ? 5 * (id - 1) : 0];
    const float Dn = DB.caD[n] * D + DB.cbD[n] * curl;
    const float D1n = e[0] * Dn + e[1] * D + e[2] * Dp + e[3] * D1 + e[4] * D1p;
    const float fn = DB.caE[n] * f + DB.sica[n] * (DB.cbEa[n] * D1n + DB.ccEa[n] * D1);
    const bool w_ = upd && st;
    stf(db_rs(DB.d[n][2], pl, 4), w_ ? o : kBad, Dn);
    stf(db_rs(DB.d1[n][2], pl, 4), w_ ? o : kBad, D1n);
    return upd ? fn : f;
  };

  float Hp[SR][3], Ep[SR][3];  // H^n(X-1) and E^{n+1}(X-1)
#pragma unroll
  for (int r = 0; r < SR; ++r)
#pragma unroll
    for (int q = 0; q < 3; ++q) Hp[r][q] = Ep[r][q] = 0.f;
  float Hn_[SR][3], En_[SR][3];  // next plane (prefetched)
  auto load_plane = [&](int X, float (*H)[3], float (*E)[3]) {
    const Rsrc a = plane_rs(hxi, X, nx, plane), b = plane_rs(hyi, X, nx, plane), c = plane_rs(hzi, X, nx, plane);
    const Rsrc d = plane_rs(exi, X, nx, plane), e = plane_rs(eyi, X, nx, plane), f = plane_rs(ezi, X, nx, plane);
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      H[r][0] = ldf(a, roff[r]);
      H[r][1] = ldf(b, roff[r]);
      H[r][2] = ldf(c, roff[r]);
      E[r][0] = ldf(d, roff[r]);
      E[r][1] = ldf(e, roff[r]);
      E[r][2] = ldf(f, roff[r]);
    }
  };
  load_plane(i0 - 1, Hn_, En_);
  int buf = 0;
  for (int X = i0 - 1; X <= i1; ++X) {
    float Hc[SR][3], Ec[SR][3];
#pragma unroll
    for (int r = 0; r < SR; ++r)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        Hc[r][q] = Hn_[r][q];
        Ec[r][q] = En_[r][q];
      }
    // this trip's psi (before the prefetch: vmcnt retires in issue order)
    float PS[6][2][SR];
#pragma unroll
    for (int n = 0; n < 6; ++n)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < SR; ++r) PS[n][t][r] = term_on(n, t) ? psi_load(n, t, n < 3 ? X : X - 1, r) : 0.f;
    float DV[UP ? 6 : 1][SR];
    if constexpr (UP) {
#pragma unroll
      for (int n = 0; n < 6; ++n)
#pragma unroll
        for (int r = 0; r < SR; ++r)
          DV[n][r] = (n < 3 ? (X >= 0 && X < nx) : (X - 1 >= 0 && X - 1 < nx)) ? ud_load(n, n < 3 ? X : X - 1, r)
                                                                             : 0.f;
    }
    load_plane(X + 1, Hn_, En_);
    // y neighbours: H(X) of the group's last row for the group above, E^{n+1}(X-1)
    // of its first row for the group below
    sX[buf][0][slot][li] = Hc[SR - 1][2];
    sX[buf][1][slot][li] = Hc[SR - 1][0];
    sX[buf][2][slot][li] = Ep[0][0];
    sX[buf][3][slot][li] = Ep[0][2];
    __syncthreads();
    const float hz_dn = sX[buf][0][rdn][li], hx_dn = sX[buf][1][rdn][li];
    const float ex_up = sX[buf][2][rup][li], ez_up = sX[buf][3][rup][li];
    buf ^= 1;
    float En[SR][3];
    // ---- E^{n+1} on plane X
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      const float hz_j = r == 0 ? hz_dn : Hc[r > 0 ? r - 1 : 0][2];
      const float hx_j = r == 0 ? hx_dn : Hc[r > 0 ? r - 1 : 0][0];
      const float hy_k = sh_up(Hc[r][1]), hx_k = sh_up(Hc[r][0]);
      const float dxy = Hc[r][2] - hz_j, dxz = Hc[r][1] - hy_k;
      const float dyz = Hc[r][0] - hx_k, dyx = Hc[r][2] - Hp[r][2];
      const float dzx = Hc[r][1] - Hp[r][1], dzy = Hc[r][0] - hx_j;
      float cx = dxy - dxz, cy = dyz - dyx, cz = dzx - dzy;
      if constexpr (CPM) {
        if (term_on(0, 0)) cx += psi_step(0, 0, X, r, PS[0][0][r], dxy);
        if (term_on(0, 1)) cx -= psi_step(0, 1, X, r, PS[0][1][r], dxz);
        if (term_on(1, 0)) cy += psi_step(1, 0, X, r, PS[1][0][r], dyz);
        if (term_on(1, 1)) cy -= psi_step(1, 1, X, r, PS[1][1][r], dyx);
        if (term_on(2, 0)) cz += psi_step(2, 0, X, r, PS[2][0][r], dzx);
        if (term_on(2, 1)) cz -= psi_step(2, 1, X, r, PS[2][1][r], dzy);
      }
      if constexpr (UP) {
        const bool se_ = (mbits >> (r * 7 + 6)) & 1u && X >= i0 && X < i1;
        En[r][0] = upml(0, X, r, Ec[r][0], cx, DV[0][r], coef(0, r, X, 1.f) != 0.f, se_);
        En[r][1] = upml(1, X, r, Ec[r][1], cy, DV[1][r], coef(1, r, X, 1.f) != 0.f, se_);
        En[r][2] = upml(2, X, r, Ec[r][2], cz, DV[2][r], coef(2, r, X, 1.f) != 0.f, se_);
      } else if constexpr (DR) {
        const bool se_ = (mbits >> (r * 7 + 6)) & 1u && X >= i0 && X < i1;
        En[r][0] = drude(0, X, r, Ec[r][0], cx, cb, coef(0, r, X, 1.f) != 0.f, se_);
        En[r][1] = drude(1, X, r, Ec[r][1], cy, cb, coef(1, r, X, 1.f) != 0.f, se_);
        En[r][2] = drude(2, X, r, Ec[r][2], cz, cb, coef(2, r, X, 1.f) != 0.f, se_);
      } else {
        En[r][0] = Ec[r][0] + coef(0, r, X, cb) * cx;
        En[r][1] = Ec[r][1] + coef(1, r, X, cb) * cy;
        En[r][2] = Ec[r][2] + coef(2, r, X, cb) * cz;
      }
      if (src_comp >= 0 && X == src_i && jr0 + r == src_j && kb == src_k) {
        if (src_comp == 0) En[r][0] = src_v;
        if (src_comp == 1) En[r][1] = src_v;
        if (src_comp == 2) En[r][2] = src_v;
      }
    }
    // ---- H^{n+1} on plane X - 1
    float Hn[SR][3];
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      const float ex_j = r == SR - 1 ? ex_up : Ep[r < SR - 1 ? r + 1 : r][0];
      const float ez_j = r == SR - 1 ? ez_up : Ep[r < SR - 1 ? r + 1 : r][2];
      const float ey_k = sh_dn(Ep[r][1]), ex_k = sh_dn(Ep[r][0]);
      const float gxz = ey_k - Ep[r][1], gxy = ez_j - Ep[r][2];
      const float gyx = En[r][2] - Ep[r][2], gyz = ex_k - Ep[r][0];
      const float gzy = ex_j - Ep[r][0], gzx = En[r][1] - Ep[r][1];
      float dx = gxz - gxy, dy = gyx - gyz, dz = gzy - gzx;
      if constexpr (CPM) {
        if (term_on(3, 0)) dx += psi_step(3, 0, X - 1, r, PS[3][0][r], gxz);
        if (term_on(3, 1)) dx -= psi_step(3, 1, X - 1, r, PS[3][1][r], gxy);
        if (term_on(4, 0)) dy += psi_step(4, 0, X - 1, r, PS[4][0][r], gyx);
        if (term_on(4, 1)) dy -= psi_step(4, 1, X - 1, r, PS[4][1][r], gyz);
        if (term_on(5, 0)) dz += psi_step(5, 0, X - 1, r, PS[5][0][r], gzy);
        if (term_on(5, 1)) dz -= psi_step(5, 1, X - 1, r, PS[5][1][r], gzx);
      }
      if constexpr (UP) {
        const bool sh_ = (mbits >> (r * 7 + 6)) & 1u && X - 1 >= i0 && X - 1 < i1;
        Hn[r][0] = upml(3, X - 1, r, Hp[r][0], dx, DV[3][r], coef(3, r, X - 1, 1.f) != 0.f, sh_);
        Hn[r][1] = upml(4, X - 1, r, Hp[r][1], dy, DV[4][r], coef(4, r, X - 1, 1.f) != 0.f, sh_);
        Hn[r][2] = upml(5, X - 1, r, Hp[r][2], dz, DV[5][r], coef(5, r, X - 1, 1.f) != 0.f, sh_);
      } else if constexpr (DR) {
        const bool sh_ = (mbits >> (r * 7 + 6)) & 1u && X - 1 >= i0 && X - 1 < i1;
        Hn[r][0] = drude(3, X - 1, r, Hp[r][0], dx, db, coef(3, r, X - 1, 1.f) != 0.f, sh_);
        Hn[r][1] = drude(4, X - 1, r, Hp[r][1], dy, db, coef(4, r, X - 1, 1.f) != 0.f, sh_);
        Hn[r][2] = drude(5, X - 1, r, Hp[r][2], dz, db, coef(5, r, X - 1, 1.f) != 0.f, sh_);
      } else {
        Hn[r][0] = Hp[r][0] + coef(3, r, X - 1, db) * dx;
        Hn[r][1] = Hp[r][1] + coef(4, r, X - 1, db) * dy;
        Hn[r][2] = Hp[r][2] + coef(5, r, X - 1, db) * dz;
      }
    }
    // ---- stores: E^{n+1}(X), H^{n+1}(X-1) of the tile's own cells
    const bool se = X >= i0 && X < i1, sh = X - 1 >= i0 && X - 1 < i1;
    const Rsrc rex = plane_rs(exo, X, nx, plane), rey = plane_rs(eyo, X, nx, plane), rez = plane_rs(ezo, X, nx, plane);
    const Rsrc rhx = plane_rs(hxo, X - 1, nx, plane), rhy = plane_rs(hyo, X - 1, nx, plane);
    const Rsrc rhz = plane_rs(hzo, X - 1, nx, plane);
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      const bool mo = (mbits >> (r * 7 + 6)) & 1u;
      const unsigned oe = mo && se ? roff[r] : kBad, oh = mo && sh ? roff[r] : kBad;
      stf(rex, oe, En[r][0]);
      stf(rey, oe, En[r][1]);
      stf(rez, oe, En[r][2]);
      stf(rhx, oh, Hn[r][0]);
      stf(rhy, oh, Hn[r][1]);
      stf(rhz, oh, Hn[r][2]);
    }
#pragma unroll
    for (int r = 0; r < SR; ++r)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        Hp[r][q] = Hc[r][q];
        Ep[r][q] = En[r][q];
      }
  }
}

template <int AX, bool KAP, int LW, int NW>
int launch_shell(const float* const* fi, float* const* fo, float cb, float db, int nx, int ny, int nz,
                 const Box3* b, const ShList& L, const int* src, float sv, const ShAux& A, hipStream_t s) {
  k_shell1<AX, KAP, LW, NW><<<L.first[L.n], dim3(64, NW), 0, s>>>(
      fi[0], fi[1], fi[2], fi[3], fi[4], fi[5], fo[0], fo[1], fo[2], fo[3], fo[4], fo[5], cb, db, nx, ny, nz, b[0],
      b[1], b[2], b[3], b[4], b[5], L, src[0], src[1], src[2], src[3], sv, A);
  FDTD_RETURN_LAUNCH_STATUS();
}

template <int AX, int NW>
int launch_shell_nw(bool kap, int lw, const float* const* fi, float* const* fo, float cb, float db, int nx, int ny,
                    int nz, const Box3* b, const ShList& L, const int* src, float sv, const ShAux& A, hipStream_t s) {
  if constexpr (AX == 8 || AX == 9 || AX == 0) {  // no kappa term: one variant
    if (lw == 32) return launch_shell<AX, false, 32, NW>(fi, fo, cb, db, nx, ny, nz, b, L, src, sv, A, s);
    return launch_shell<AX, false, 64, NW>(fi, fo, cb, db, nx, ny, nz, b, L, src, sv, A, s);
  } else {
    if (lw == 32)
      return kap ? launch_shell<AX, true, 32, NW>(fi, fo, cb, db, nx, ny, nz, b, L, src, sv, A, s)
                 : launch_shell<AX, false, 32, NW>(fi, fo, cb, db, nx, ny, nz, b, L, src, sv, A, s);
    return kap ? launch_shell<AX, true, 64, NW>(fi, fo, cb, db, nx, ny, nz, b, L, src, sv, A, s)
               : launch_shell<AX, false, 64, NW>(fi, fo, cb, db, nx, ny, nz, b, L, src, sv, A, s);
  }
}

// waves per workgroup (tuning): FDTD3D_SHELL_WAVES = 8 or 16 (default)
int shell_waves() {
  static int w = -1;
  if (w < 0) {
    const char* e = getenv("FDTD3D_SHELL_WAVES");
    w = (e && atoi(e) == 8) ? 8 : 16;
  }
  return w;
}

template <int AX>
int launch_shell_ax(bool kap, int lw, const float* const* fi, float* const* fo, float cb, float db, int nx, int ny,
                    int nz, const Box3* b, const ShList& L, const int* src, float sv, const ShAux& A, hipStream_t s) {
  if (shell_waves() == 8) return launch_shell_nw<AX, 8>(kap, lw, fi, fo, cb, db, nx, ny, nz, b, L, src, sv, A, s);
  return launch_shell_nw<AX, 16>(kap, lw, fi, fo, cb, db, nx, ny, nz, b, L, src, sv, A, s);
}

}  // namespace

// One step of the shell: reads fin (Ex Ey Ez Hx Hy Hz), writes fout on the
// `nwin` output boxes `wins` (6 ints each, local; disjoint) -- cells of a box
// outside a component's update box (`boxes`, 6 x 6 ints) are stored
// unchanged.  `ax[w]` = absorbing-layer axes of box w (bit 0 x, 1 y, 2 z: the
// slabs it may touch; 0 = none; any superset is correct).  CPML runs pass
// `cpml` = the CpmlDev block of models/cpml.py host_table, in HOST memory
// (psi read from psi[p], written to the alt copy) and `kap` = some
// 1/kappa - 1 is non-zero; UPML runs pass `upml` = the host ShUpml block of
// models/upml.py (every box with ax != 0 runs the D/B chain), dispersive
// boxes `drude` = the host ShDrude block.  `src` = {i, j, k, comp} of a hard E point
// source (comp -1: none), value `src_val`.  Boxes at most 30 cells deep in z
// run 32-lane rows.
FDTD_API int fdtd_shell1_f32(const float* const* fin, float* const* fout, double cb, double db, int nx, int ny,
                             int nz, const int* boxes, int nwin, const int* wins, const int* ax, const int* src,
                             double src_val, const void* cpml, int kap, const void* upml, const void* drude,
                             void* stream) {
  if (nwin < 0 || (cpml && upml)) return (int)hipErrorInvalidValue;
  for (int w = 0; w < nwin; ++w) {
    if ((ax[w] & 8) && !drude) return (int)hipErrorInvalidValue;
    if ((ax[w] & 7) && !cpml && !upml) return (int)hipErrorInvalidValue;
  }
  Box3 b[6];
  for (int n = 0; n < 6; ++n) b[n] = make_box(boxes + 6 * n);
  const hipStream_t s = (hipStream_t)stream;
  // the tables arrive as HOST bytes (models/cpml.py host_table, models/upml.py)
  ShAux aux;
  memset(&aux, 0, sizeof(aux));
  if (cpml) memcpy(&aux.c, cpml, sizeof(ShCpml));
  if (upml) memcpy(&aux.u, upml, sizeof(ShUpml));
  if (drude) memcpy(&aux.d, drude, sizeof(ShDrude));
  // group the boxes by (class, lane width); classes: none, CPML x, y, z,
  // the two-axis edges (xy, xz, yz), the corners (xyz), UPML, dispersive
  const int classes[10] = {0, 1, 2, 4, 3, 5, 6, 7, 8, 9};
  for (int ci = 0; ci < 10; ++ci) {
    for (int lw : {64, 32}) {
      ShList L;
      L.n = 0;
      long long work = 0;
      Box3 pend[256];
      int np = 0;
      for (int wi = 0; wi < nwin; ++wi) {
        const Box3 o = make_box(wins + 6 * wi);
        if (box_empty(o)) continue;
        const int a = ax[wi];
        const int cls = a == 0 ? 0 : ((a & 8) ? 9 : (upml ? 8 : (a & 7)));
        if (cls != classes[ci]) continue;
        const int zl = o.hi[2] - o.lo[2];
        if ((zl <= 30) != (lw == 32)) continue;
        if (np >= 256) return (int)hipErrorInvalidValue;
        pend[np++] = o;
      }
      if (np == 0) continue;
      const int ROWS = shell_waves() * (64 / lw) * SR;
      for (int q = 0; q < np; ++q) {
        const Box3& o = pend[q];
        work += (long long)cdiv(o.hi[2] - o.lo[2], lw - 2) * cdiv(o.hi[1] - o.lo[1], ROWS - 2) * (o.hi[0] - o.lo[0]);
      }
      // x chunk: about 1024 workgroups per launch, at least 16 planes (two
      // re-read lead-in / drain planes per chunk)
      int xc = (int)((work + 1023) / 1024);
      xc = xc < 16 ? 16 : (xc > 512 ? 512 : xc);
      int q = 0;
      while (q < np) {
        L.n = 0;
        int first = 0;
        while (q < np && L.n < SH_MAX) {
          const Box3& o = pend[q++];
          const int k = L.n++;
          L.box[k] = o;
          L.tz[k] = (int)cdiv(o.hi[2] - o.lo[2], lw - 2);
          L.ty[k] = (int)cdiv(o.hi[1] - o.lo[1], ROWS - 2);
          L.xc[k] = xc;
          L.first[k] = first;
          first += L.tz[k] * L.ty[k] * (int)cdiv(o.hi[0] - o.lo[0], xc);
        }
        L.first[L.n] = first;
        const float fc = (float)cb, fd = (float)db, sv = (float)src_val;
        int rc = 0;
#define SH_CASE(C) rc = launch_shell_ax<C>(kap != 0, lw, fin, fout, fc, fd, nx, ny, nz, b, L, src, sv, aux, s)
        switch (classes[ci]) {
          case 0: SH_CASE(0); break;
          case 1: SH_CASE(1); break;
          case 2: SH_CASE(2); break;
          case 4: SH_CASE(4); break;
          case 3: SH_CASE(3); break;
          case 5: SH_CASE(5); break;
          case 6: SH_CASE(6); break;
          case 7: SH_CASE(7); break;
          case 8: SH_CASE(8); break;
          default: SH_CASE(9); break;
        }
#undef SH_CASE
        if (rc) return rc;
      }
    }
  }
  return 0;
}

// size of the CPML block (ABI check against models/cpml.py device_table)
FDTD_API int fdtd_shell_cpml_size() { return (int)sizeof(ShCpml); }

// size of the UPML block (ABI check against models/upml.py)
FDTD_API int fdtd_shell_upml_size() { return (int)sizeof(ShUpml); }

// size of the dispersive-box block (ABI check against models/upml.py DrudeBox)
FDTD_API int fdtd_shell_drude_size() { return (int)sizeof(ShDrude); }
