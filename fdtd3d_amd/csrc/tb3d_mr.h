// Multi-row temporally blocked fp32 3D Yee kernel (k_tb3d_mr) and its
// launcher (yee3d_tb.hip holds the host API): plain, sparse per-cell
// coefficient and TF/SF variants.
#pragma once

#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "tfsf_dev.h"

namespace tb3d {

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

// Amplitude (steady-state) mode folded into the blocked passes (feature bit
// 8; reference Scheme3D.cpp:2945-3333, models/scheme.py
// perform_amplitude_steps): at every level each owned cell inside its
// component's amplitude box compares |f| with its running maximum a and, when
// |f| >= a and (|f| - a) / a > acc, sets a = |f| and counts one change for
// that level (step) -- the arithmetic of k_amplitude_many, level by level.  A
// cell's levels run in T consecutive trips of the same lane, so a hands from
// level to level through a per-thread LDS slot (T - 1 slots x 6 components x
// the 32 x 64 tile: 96 KiB at T = 3); level 0 reads it from memory (prefetched
// a trip ahead), the last level writes it back.  The changed counts of each
// level accumulate per lane and go to ``counts[l]`` with one atomic per wave
// and level at the end.  The amplitude mode's hard source is a z line
// (src_k .. k1 - 1).
struct AmpDev {
  float* a;          // running maxima of |Ex| .. |Hz|, [x][component][y][z]: ONE buffer descriptor
                     // per x plane covers all six (SGPRs are this kernel's scarce resource)
  Box3 b[6];         // amplitude boxes (computation box minus PML, local): y / z at setup
  int xr[6];         // their x ranges, lo | hi << 16 (the per-plane test)
  unsigned* counts;  // changed cells per level of the pass
  float acc;         // relative growth that counts as a change
  int k1;            // the source's z line: src_k .. k1 - 1
};

// Drude box folded into the blocked passes (feature bit 16, its own launch
// over the box grown by T: models/blocking.py _drude_blk_plan).  Reference
// Drude form Kernels.h:103-107 / Scheme3D.cpp:266-416, stepped here by the
// fused chain (chain_kernels.hip).  Inside the sigma = 0 region the chain
//   Dn = D + cbd curl,  D1n = b0 Dn + b1 D + b2 Dp + m1 D1 + m2 D1p,
//   E' = E + (cbEa D1n + ccEa D1) / (2 eps0) = E + (D1n - D1)
// keeps E - D1 invariant (0 from rest), and the Drude ADE has
// b1 = -(b0 + b2), so with D1 = E:
//   E' = (b0 cbd) curl - b2 (D - Dp) + m1 E + m2 Ep,   (D - Dp)' = cbd curl,  Ep' = E
// A cell's dispersive state is (delta = D - Dp, Ep) per E component -- six
// floats instead of the chain's four levels of D / D1 -- and the coefficient
// tuple (b0 cbd, b2, m1, m2) of each component comes from a per-component
// table indexed by the cell's material id (uint8; a Drude scene holds a
// handful of distinct tuples), parked in LDS.  The state of a cell moves
// from level to level in registers, like the fields: level l hands its
// output to level l + 1 of the next trip (the same plane), so a pass reads
// and writes it once.  Memory: per cell of B, two float4 per state set:
//   s[0] = (delta_x, delta_y, delta_z, id_x | id_y << 8 | id_z << 16 as bits)
//   s[1] = (Ep_x, Ep_y, Ep_z, 0)
constexpr int DR_MAX_IDS = 256;
struct DrDev {
  Box3 B;                  // dispersive box (local): the E components take the form above inside
  const float4* sin0;      // state in (delta + ids, Ep), x-major over B, z fastest
  const float4* sin1;
  float4* sout0;           // state out (distinct buffers: tiles re-read halo cells other tiles own)
  float4* sout1;
  const float4* lut;       // [3][nid]: (b0 cbd, b2, m1, m2) per component and id
  int nid;
  float cbd;               // D update coefficient dt / dx (the chain's cbD where sigma = 0)
};
struct DrS {
  float dx, dy, dz, px, py, pz;
  unsigned id;
};

// Memory access through buffer descriptors: one descriptor per (array, x
// plane) built in SGPRs from the wave-uniform plane index, plus ONE 32-bit
// per-lane byte offset shared by every array (buffer_load ... offen).  Flat
// 64-bit addressing would keep a per-lane pointer per array live across the
// x loop (24 VGPRs for 12 arrays) and spill.  Offsets past the descriptor's
// size read 0 / drop the store, which is how rows and planes outside the
// array are handled -- no per-lane load guards.
typedef __amdgpu_buffer_rsrc_t Rsrc;

// wave-uniform read of a table the kernel never writes, through the constant
// address space: a scalar load (s_load, lgkm counter) -- a plain global load
// of the same uniform address is a vector load that waits behind the plane
// prefetch
__device__ __forceinline__ float cload(const float* p, int i) {
  return ((const __attribute__((address_space(4))) float*)p)[i];
}

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
    const TfDev* __restrict__ tf, const float* __restrict__ gtab, AmpDev amp, DrDev dr) {
  // feature bits: 1 per-cell E, 2 per-cell H coefficients (sparse), 4 TF/SF,
  // 8 amplitude mode (alone; T <= 3: its LDS hand-off), 16 Drude box (alone)
  constexpr int PC = FX & 3;
  constexpr bool TFS = FX & 4;
  constexpr bool AMP = FX & 8;
  constexpr bool DRU = FX & 16;
  static_assert(!AMP || (FX == 8 && V == 1 && T <= 3), "amplitude mode: scalar lanes, alone, T <= 3");
  static_assert(!DRU || FX == 16, "Drude box: alone");
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
  // the TF/SF sets: scalar loads through the constant address space (every
  // index the kernel uses is wave-uniform)
  typedef const __attribute__((address_space(4))) TfDev* TfPtr;
  const TfPtr TFc = (TfPtr)tf;

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

  // amplitude mode: bit r * 6 + c -- row r of this lane is an owned cell of
  // the output box inside component c's amplitude box (y / z; x per plane)
  unsigned ambits = 0;
  constexpr int AS = AMP ? T - 1 : 1;
  __shared__ float sA[AS > 0 ? AS : 1][AMP ? 6 : 1][AMP ? ROWS : 1][AMP ? 64 : 1];
  float aPre[AMP ? 6 : 1][R], aPend[AMP ? 6 : 1][R];
  unsigned acnt[AMP ? T : 1];
  if constexpr (AMP) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int j = jw + r;
      const bool own = (mbits >> ((r * 7 + 6) * V)) & 1u;
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const Box3& ab = amp.b[c];
        const bool in = own && j >= ab.lo[1] && j < ab.hi[1] && kb >= ab.lo[2] && kb < ab.hi[2];
        ambits |= (in ? 1u : 0u) << (r * 6 + c);
        aPre[c][r] = aPend[c][r] = 0.f;
      }
    }
#pragma unroll
    for (int l = 0; l < T; ++l) acnt[l] = 0u;
  }
  // the six maxima of x plane p (offset c * plane * 4 + roff)
  auto amp_rsrc = [&](int p) -> Rsrc { return plane_rsrc(amp.a, p, nx, 6 * plane); };
  // level-0 maxima of the next trip (E on plane X + 1, H on plane X)
  auto amp_prefetch = [&](int X) {
    if constexpr (AMP) {
      const Rsrc re = amp_rsrc(X + 1), rh = amp_rsrc(X);
#pragma unroll
      for (int c = 0; c < 6; ++c) {
#pragma unroll
        for (int r = 0; r < R; ++r)
          // the component's plane offset rides in the instruction's SGPR offset
          aPre[c][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
              c < 3 ? re : rh, ((ambits >> (r * 6 + c)) & 1u) ? roff[r] : 0xF0000000u, c * 4 * (int)plane, 0));
      }
    }
  };
  // level l of kind k (0 E, 1 H) on plane p, row r: compare, count, hand on
  auto amp_level = [&](int k, int l, int p, int r, const F3<V>& f) {
    if constexpr (AMP) {
      const bool pin = p >= i0 && p < i1;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int c = 3 * k + q;
        const float fv = q == 0 ? f.x[0] : (q == 1 ? f.y[0] : f.z[0]);
        const float v = fabsf(fv);
        const int xr = amp.xr[c];
        const bool in = pin && ((ambits >> (r * 6 + c)) & 1u) &&
                        (unsigned)(p - (xr & 0xffff)) < (unsigned)((xr >> 16) - (xr & 0xffff));
        float& slot = sA[l > 0 ? l - 1 : 0][c][R * w + r][lane];
        // carried values hold a negated maximum once a level of this pass
        // changed it (maxima are >= 0): only those are written back
        const float raw = l == 0 ? aPre[c][r] : slot;
        const bool dirty = l > 0 && (__float_as_uint(raw) >> 31);
        const float old = fabsf(raw);
        const float den = old != 0.f ? old : (v != 0.f ? v : 1.f);
        // (v - old) / den > acc without the division (den > 0)
        const bool ch = in && v >= old && (v - old) > amp.acc * den;
        const float nv = ch ? v : old;
        acnt[l] += ch ? 1u : 0u;
        // the slot of level l - 1 now takes this trip's level l - 1 result
        // (plane p + 1), read by level l of the next trip
        if (l > 0) slot = aPend[c][r];
        if (l < T - 1) {
          aPend[c][r] = (dirty || ch) ? -nv : nv;
        } else {
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(nv), amp_rsrc(p),
                                                (in && (dirty || ch)) ? roff[r] : 0xF0000000u, c * 4 * (int)plane, 0);
        }
      }
    }
  };

  // Drude box: per row, the lane's byte offset in one x plane of the state
  // arrays (16 B per cell of B; past the plane outside B in y / z) and bit r
  // of dinb when row r of this lane lies in B (y / z; x per plane)
  unsigned doff[DRU ? R : 1];
  unsigned dinb = 0u;
  __shared__ float4 sL[DRU ? 3 * DR_MAX_IDS : 1];
  const int dbz = dr.B.hi[2] - dr.B.lo[2];
  const size_t dplane = DRU ? (size_t)(dr.B.hi[1] - dr.B.lo[1]) * dbz * 16u : 0;
  if constexpr (DRU) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int j = jw + r;
      const bool in = kin && j >= dr.B.lo[1] && j < dr.B.hi[1] && kb >= dr.B.lo[2] && kb < dr.B.hi[2];
      doff[r] = in ? (unsigned)((j - dr.B.lo[1]) * dbz + (kb - dr.B.lo[2])) * 16u : 0xF0000000u;
      dinb |= (in ? 1u : 0u) << r;
    }
    // the coefficient tables into LDS (read by lane id at every level)
    for (int i = lane + 64 * w; i < 3 * DR_MAX_IDS; i += 64 * NW) {
      const int c = i / DR_MAX_IDS, id = i - c * DR_MAX_IDS;
      sL[i] = id < dr.nid ? dr.lut[c * dr.nid + id] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
  }
  const bool wave_d = DRU && __any(dinb != 0u);
  auto dr_rsrc = [&](const void* base, int p) -> Rsrc {
    const bool in = xin(dr.B, p);
    return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + (in ? (size_t)(p - dr.B.lo[0]) * dplane : 0)),
                                             (short)0, in ? (int)dplane : 0, 0x00020000);
  };

  // TF/SF slots: the sets that touch this wave's rows / lanes, per kind k
  // (0 E, 1 H) numbered c * 4 + s (component c of the kind, its s-th set; a
  // component has at most 4 face sets: two curl axes x two faces).  Scalar
  // bit masks (bit c * 4 + s, E in the low half, H << 16) of the y / z-face
  // slots (looked at every level) and of the x-face slots (looked at on the
  // kind's x-face planes only); per-lane data in VGPR lanes, read back with
  // readlane -- no memory round trip inside the level loop:
  //   tf_xr    lane k * 12 + slot: x range (lo | hi << 16) of the slot's set
  //            cut to its component's update box;
  //   tf_lb[k] bit slot * R + r: this lane's cell of row r is a target of the
  //            slot (set box and update box in y / z);
  //   tf_off[k] lane e = slot * T + l (va = 0): g-table index of entry e less
  //            the plane, added per trip;
  //   tf_g[k][2] entries e (va = 0: slot * T + l; va = 1: (slot * T + l) * R
  //            + r), loaded once per trip (va = 1: once per kernel, the index
  //            does not move with the plane) before the field prefetch.
  unsigned tf_cm = 0u, tf_xm = 0u;
  int tf_xpl = -1, tf_xph = -1;  // x-face planes of the E / H sets: lo | hi << 16 (-1: none)
  int tf_xr = 0;
  // (separate scalars, not arrays: the set-up indexes them by a run-time
  // kind, which would put an array in scratch memory for the whole kernel)
  unsigned tf_lb0 = 0u, tf_lb1 = 0u;
  int tf_off0 = 0, tf_off1 = 0;
  float tf_g00 = 0.f, tf_g01 = 0.f, tf_g10 = 0.f, tf_g11 = 0.f;
  int tf_va = 0;
  const Rsrc tf_gr = __builtin_amdgcn_make_buffer_rsrc((void*)gtab, (short)0, TFS ? T * TFc->ld * 4 : 0, 0x00020000);
  if constexpr (TFS) {
    const int ns = TFc->nsets;
    const int ld = TFc->ld;
    tf_va = TFc->s[0].va;
    unsigned cnt = 0u;  // sets taken per component, 4 bits each
    for (int si = 0; si < ns; ++si) {
      const int lo1 = TFc->s[si].lo[1], hi1 = TFc->s[si].hi[1];
      const int lo2 = TFc->s[si].lo[2], hi2 = TFc->s[si].hi[2];
      const int n = TFc->s[si].n;
      const int k = n < 3 ? 0 : 1, c = n - 3 * k;
      // the component's update box, field by field (a Box3 picked among the
      // by-value box arguments would copy all six to scratch memory)
#define TF_UB(f, d) (n == 0 ? bex.f[d] : n == 1 ? bey.f[d] : n == 2 ? bez.f[d] : n == 3 ? bhx.f[d] : n == 4 ? bhy.f[d] : bhz.f[d])
      const int ul0 = TF_UB(lo, 0), uh0 = TF_UB(hi, 0), ul1 = TF_UB(lo, 1), uh1 = TF_UB(hi, 1);
      const int ul2 = TF_UB(lo, 2), uh2 = TF_UB(hi, 2);
#undef TF_UB
      unsigned rb = 0u;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int j = jw + r;
        const bool in = kin && j >= lo1 && j < hi1 && kb >= lo2 && kb < hi2 && j >= ul1 && j < uh1 && kb >= ul2 &&
                        kb < uh2;
        rb |= in ? (1u << r) : 0u;
      }
      if (!__any(rb != 0u)) continue;
      const int s = (cnt >> (4 * n)) & 0xf;
      cnt += 1u << (4 * n);
      if (s >= 4) continue;  // (cannot happen: a component has 4 face sets)
      const int slot = c * 4 + s;
      const unsigned bit = 1u << (slot + 16 * k);
      if (TFc->s[si].fa == 0) tf_xm |= bit; else tf_cm |= bit;
      const int xl = max(TFc->s[si].lo[0], ul0), xh = min(TFc->s[si].hi[0], uh0);
      if (lane == k * 12 + slot) tf_xr = xh > xl ? (xl | (xh << 16)) : 0;
      if (k == 0) tf_lb0 |= rb << (slot * R); else tf_lb1 |= rb << (slot * R);
      // va = 0: entry (slot, l) of plane p reads g[l * ld + goff + p - lo0]; the plane of level l at
      // trip X is X - l (E) or X - l - 1 (H), so the index less X is fixed per entry
#pragma unroll
      for (int l = 0; l < T; ++l)
        if (lane == slot * T + l) {
          const int o = l * ld + TFc->s[si].goff - TFc->s[si].lo[0] - l - k;
          if (k == 0) tf_off0 = o; else tf_off1 = o;
        }
      if (tf_va == 1) {
        // va = 1: the index moves with the row only -- load the pass's entries now
#pragma unroll
        for (int l = 0; l < T; ++l)
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int e = (slot * T + l) * R + r;
            const int gi = l * ld + TFc->s[si].goff + jw + r - lo1;
            const bool ok = jw + r >= lo1 && jw + r < hi1;
            const float v = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                tf_gr, (lane == (e & 63) && ok) ? (unsigned)gi * 4u : 0xF0000000u, 0, 0));
            if (lane == (e & 63)) {
              if (k == 0 && e < 64) tf_g00 = v;
              if (k == 0 && e >= 64) tf_g01 = v;
              if (k == 1 && e < 64) tf_g10 = v;
              if (k == 1 && e >= 64) tf_g11 = v;
            }
          }
      }
    }
    const int e0 = TFc->xpl[0][0], e1 = TFc->xpl[0][1], h0 = TFc->xpl[1][0], h1 = TFc->xpl[1][1];
    tf_xpl = (e0 & 0xffff) | (e1 << 16);
    tf_xph = (h0 & 0xffff) | (h1 << 16);
  }
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
  // Drude state (see DrDev): DS[l] = the output of level l in the previous
  // trip (plane X - 1 - l), which level l + 1 takes in this trip; Dc = the
  // input of the level running; Dnx = the next trip's level-0 input
  // (prefetched); DL = the last level's output, stored with the fields
  constexpr int NDS = DRU ? (T > 1 ? T - 1 : 1) : 1;
  constexpr int RD = DRU ? R : 1;
  DrS DS[NDS][RD], Dnx[RD], Dc[RD], DL[RD];
  typedef unsigned u4v __attribute__((ext_vector_type(4)));
  auto dr_load = [&](int X, DrS* S) {
    if constexpr (DRU) {
      const Rsrc r0 = dr_rsrc(dr.sin0, X), r1 = dr_rsrc(dr.sin1, X);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const u4v a = __builtin_amdgcn_raw_buffer_load_b128(r0, doff[r], 0, 0);
        const u3 b = __builtin_amdgcn_raw_buffer_load_b96(r1, doff[r], 0, 0);
        S[r].dx = __uint_as_float(a.x);
        S[r].dy = __uint_as_float(a.y);
        S[r].dz = __uint_as_float(a.z);
        S[r].id = a.w;
        S[r].px = __uint_as_float(b.x);
        S[r].py = __uint_as_float(b.y);
        S[r].pz = __uint_as_float(b.z);
      }
    }
  };
  if constexpr (DRU) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      DL[r] = Dc[r] = Dnx[r] = DrS{};
#pragma unroll
      for (int l = 0; l < NDS; ++l) DS[l][r] = DrS{};
    }
    if (wave_d) dr_load(i0 - T, Dnx);
  }
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
  // per trip, bit 2 l + k: level l has TF/SF fixes of kind k (0 E, 1 H) for
  // this wave
  unsigned tf_lv = 0u;
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
    // TF/SF corrections of kind k (0 E, 1 H) at level l on plane p, added to
    // the new values N of every row: N += c g, c the coefficient the update
    // multiplied the curl with (the slots' target bits already hold the
    // update box in y / z, their x ranges the box in x).  They run at the end
    // of the level, after the H update -- the level's barrier is a block
    // boundary anyway, while a branch between the E and H updates costs an
    // issue-bound level 16% even when idle (profiles/tfsf_cost_r5.md) -- so
    // an E correction of Ey / Ez also corrects the H update that read the
    // uncorrected value: Hadj (this level's new H on plane p - 1, same lanes
    // and rows) gets -/+ its coefficient times the correction.
    auto tf_fix = [&](int k, int l, int p, F3<V>* N, F3<V>* Hadj) {
      if constexpr (TFS) {
        const int xpp = k == 0 ? tf_xpl : tf_xph;
        const bool xp = p == (short)(xpp & 0xffff) || p == (xpp >> 16);
        const unsigned m0 = ((tf_cm | (xp ? tf_xm : 0u)) >> (16 * k)) & 0xfffu;
        if (m0 == 0u) return;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          unsigned m = (m0 >> (4 * c)) & 0xfu;
          while (m) {
            const int slot = c * 4 + __builtin_ctz(m);
            m &= m - 1u;
            const int xr = __builtin_amdgcn_readlane(tf_xr, k * 12 + slot);
            if ((unsigned)(p - (xr & 0xffff)) >= (unsigned)((xr >> 16) - (xr & 0xffff))) continue;
#pragma unroll
            for (int r = 0; r < R; ++r) {
              const int e = tf_va == 0 ? slot * T + l : (slot * T + l) * R + r;
              const float gv = k == 0 ? (e < 64 ? tf_g00 : tf_g01) : (e < 64 ? tf_g10 : tf_g11);
              const float g = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gv), e & 63));
              const float3 kc = kcoef(k == 0, l, p, r);
              const float sc = c == 0 ? kc.x : (c == 1 ? kc.y : kc.z);
              const bool t = ((k == 0 ? tf_lb0 : tf_lb1) >> (slot * R + r)) & 1u;
              const vec d = (vec)(t ? sc * g : 0.f);
              if (c == 0) N[r].x = N[r].x + d;
              if (c == 1) N[r].y = N[r].y + d;
              if (c == 2) N[r].z = N[r].z + d;
              if (k == 0 && c == 1) Hadj[r].z = Hadj[r].z - coef(bhz, p - 1, r, 5, kcoef(false, l, p - 1, r).z) * d;
              if (k == 0 && c == 2) Hadj[r].y = Hadj[r].y + coef(bhy, p - 1, r, 4, kcoef(false, l, p - 1, r).y) * d;
            }
          }
        }
      }
    };
    if constexpr (TFS) {
      // levels of this trip with fixes, bit 2 l + k (one scalar test per
      // level and kind); their g entries (va = 0) in one vector load per kind,
      // issued before the field prefetch so the levels never wait behind it
      unsigned lv = ((tf_cm & 0xfffu) ? 0x155u : 0u) | ((tf_cm >> 16) ? 0x2aau : 0u);
      if (tf_xm & 0xfffu) {
        const int q0 = (short)(tf_xpl & 0xffff), q1 = tf_xpl >> 16;
        if (q0 >= 0 && (unsigned)(X - q0) < (unsigned)T) lv |= 1u << (2 * (X - q0));
        if (q1 >= 0 && (unsigned)(X - q1) < (unsigned)T) lv |= 1u << (2 * (X - q1));
      }
      if (tf_xm >> 16) {
        const int q0 = (short)(tf_xph & 0xffff), q1 = tf_xph >> 16;
        if (q0 >= 0 && (unsigned)(X - 1 - q0) < (unsigned)T) lv |= 2u << (2 * (X - 1 - q0));
        if (q1 >= 0 && (unsigned)(X - 1 - q1) < (unsigned)T) lv |= 2u << (2 * (X - 1 - q1));
      }
      tf_lv = lv & ((1u << (2 * T)) - 1u);
      if (tf_va == 0 && tf_lv) {
        tf_g00 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            tf_gr, lane < 12 * T ? (unsigned)(tf_off0 + X) * 4u : 0xF0000000u, 0, 0));
        tf_g10 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            tf_gr, lane < 12 * T ? (unsigned)(tf_off1 + X) * 4u : 0xF0000000u, 0, 0));
      }
    }
    // Drude: this trip's level-0 state, the next one's in flight (issued
    // before the field prefetch: vmcnt retires in issue order)
    if constexpr (DRU) {
#pragma unroll
      for (int r = 0; r < R; ++r) Dc[r] = Dnx[r];
      if (wave_d) dr_load(X + 1, Dnx);
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
        En[r].x = Ec[r].x + coef(bex, pe, r, 0, ce.x) * cx;
        En[r].y = Ec[r].y + coef(bey, pe, r, 1, ce.y) * cy;
        En[r].z = Ec[r].z + coef(bez, pe, r, 2, ce.z) * cz;
        if constexpr (DRU) {
          // dispersive form inside B (see DrDev); the state moves on to level l + 1
          const DrS s = Dc[r];
          if (wave_d && xin(dr.B, pe)) {
            const float4 kx = sL[s.id & 0xffu];
            const float4 ky = sL[DR_MAX_IDS + ((s.id >> 8) & 0xffu)];
            const float4 kz = sL[2 * DR_MAX_IDS + ((s.id >> 16) & 0xffu)];
            const bool in = (dinb >> r) & 1u;
            const float nx_ = kx.x * cx[0] - kx.y * s.dx + kx.z * Ec[r].x[0] + kx.w * s.px;
            const float ny_ = ky.x * cy[0] - ky.y * s.dy + ky.z * Ec[r].y[0] + ky.w * s.py;
            const float nz_ = kz.x * cz[0] - kz.y * s.dz + kz.z * Ec[r].z[0] + kz.w * s.pz;
            if (in) {
              En[r].x[0] = nx_;
              En[r].y[0] = ny_;
              En[r].z[0] = nz_;
            }
          }
          DrS o;
          o.dx = dr.cbd * cx[0];
          o.dy = dr.cbd * cy[0];
          o.dz = dr.cbd * cz[0];
          o.px = Ec[r].x[0];
          o.py = Ec[r].y[0];
          o.pz = Ec[r].z[0];
          o.id = s.id;
          if (l < T - 1) {
            Dc[r] = DS[l < T - 1 ? l : 0][r];
            DS[l < T - 1 ? l : 0][r] = o;
          } else {
            DL[r] = o;
          }
        }
        if (src_plane && jw + r == src_j &&
            (AMP ? (kb >= src_k && kb < amp.k1) : (src_k >= kb && src_k < kb + V))) {
          const int q = AMP ? 0 : src_k - kb;
          if (src_comp == 0) En[r].x[q] = sv.v[l];
          if (src_comp == 1) En[r].y[q] = sv.v[l];
          if (src_comp == 2) En[r].z[q] = sv.v[l];
        }
        amp_level(0, l, pe, r, En[r]);
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
        Hn.x = Hp[l][r].x + coef(bhx, ph, r, 3, ch.x) * dx;
        Hn.y = Hp[l][r].y + coef(bhy, ph, r, 4, ch.y) * dy;
        Hn.z = Hp[l][r].z + coef(bhz, ph, r, 5, ch.z) * dz;
        amp_level(1, l, ph, r, Hn);
        // later rows (r+1 ..) read only their own and higher rows' Ep, so
        // row r rotates as soon as its H is done
        Ec[r] = Ep[l][r];
        Ep[l][r] = En[r];
        Hp[l][r] = Hc[r];
        Hc[r] = Hn;
      }
      // TF/SF fixes of the level (after the H update, see tf_fix): E on plane
      // pe (now Ep[l]), H on plane ph (now Hc)
      if constexpr (TFS) {
        if (tf_lv & (3u << (2 * l))) {
          tf_fix(0, l, pe, Ep[l], Hc);
          tf_fix(1, l, ph, Hc, Hc);
        }
      }
      // the next trip's level-0 maxima, in flight under the remaining levels
      if (AMP && l == 0) amp_prefetch(X);
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
    if constexpr (DRU) {
      // the last level's state (plane X - T + 1): owned cells of B
      const int pe = X - T + 1;
      const Rsrc r0 = dr_rsrc(dr.sout0, pe), r1 = dr_rsrc(dr.sout1, pe);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const unsigned mo = (mbits >> ((r * 7 + 6) * V)) & VM;
        const unsigned o = (wave_d && mo && ((dinb >> r) & 1u) && pe >= i0 && pe < i1) ? doff[r] : 0xF0000000u;
        u4v a;
        a.x = __float_as_uint(DL[r].dx);
        a.y = __float_as_uint(DL[r].dy);
        a.z = __float_as_uint(DL[r].dz);
        a.w = DL[r].id;
        u4v b;
        b.x = __float_as_uint(DL[r].px);
        b.y = __float_as_uint(DL[r].py);
        b.z = __float_as_uint(DL[r].pz);
        b.w = 0u;
        __builtin_amdgcn_raw_buffer_store_b128(a, r0, o, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(b, r1, o, 0, 0);
      }
    }
    if (DEFER) {
#pragma unroll
      for (int r = 0; r < R; ++r) Hs[r] = Hc[r];
    } else {
      if constexpr (TFS)
        store_plane(X, Ep[T - 1], Hc);  // (= En plus the last level's TF/SF fixes)
      else
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
  if constexpr (AMP) {
#pragma unroll
    for (int l = 0; l < T; ++l) {
      unsigned v = acnt[l];
#pragma unroll
      for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
      if (lane == 0 && v) atomicAdd(amp.counts + l, v);
    }
  }
}


// host-side knobs of the multi-row launches (defined in yee3d_tb.hip)
extern int g_tb_mr_noallin;
extern int g_tb_mr_xcd;
extern int g_tb_variant;
int tb_patch_bits();

template <int T, int V, int R, int FX, int NW = TBW>
int launch_tb_mr(const float* const* ein, const float* const* hin, float* const* eout, float* const* hout,
                 const float4* ce4, const float4* ch4, const Box3& BE, const Box3& BH, float cb, float db, int nx,
                 int ny, int nz, const Box3* b, const Box3& O, int xchunk, const int* src, const TbSrc& sv,
                 const TfDev* tf, const float* gtab, const AmpDev& amp, hipStream_t s, const DrDev& dr = DrDev{}) {
  constexpr int HL = (T + V - 1) / V;
  constexpr int TBZ = (64 - 2 * HL) * V;
  dim3 grid(cdiv(O.hi[2] - (O.lo[2] & ~(V - 1)), TBZ), cdiv(O.hi[1] - O.lo[1], NW * R - 2 * T),
            cdiv(O.hi[0] - O.lo[0], xchunk));
#define MR_LAUNCH(PFD, DEFER)                                                                                 \
  k_tb3d_mr<T, V, R, FX, PFD, DEFER, NW><<<grid, dim3(64, NW), 0, s>>>(                                     \
      ein[0], ein[1], ein[2], hin[0], hin[1], hin[2], eout[0], eout[1], eout[2], hout[0], hout[1], hout[2], \
      ce4, ch4, BE, BH, cb, db, nx, ny, nz, b[0], b[1], b[2], b[3], b[4], b[5],                             \
      O, xchunk, src[0], src[1], src[2], src[3], sv,                                                       \
      g_tb_mr_xcd ? (1 | (g_tb_mr_noallin << 1) | tb_patch_bits()) : (g_tb_mr_noallin << 1), tf, gtab, amp, dr)
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

}  // namespace tb3d
