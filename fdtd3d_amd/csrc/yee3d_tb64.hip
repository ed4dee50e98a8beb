// Temporally blocked fp64 3D Yee kernel (the reference's default value type
// is double, Source/Kernels/FieldValue.h:7-27).  Same wavefront as the fp32
// multi-row kernel in yee3d_tb.hip (a level lags one x plane; y neighbours
// between waves through a double-buffered LDS slot, one barrier per level; z
// neighbours by DPP wave shifts), with scalar fp64 lanes: every carried
// value takes two VGPRs, so one cell per lane (two cells spill from T = 2
// on).  Default tiles are 32 x 32 (each wave holds two y rows of 32 z lanes,
// HALF below); the 16-row x 64-lane shape stays selectable
// (fdtd_set_tb64_shape).  T halo rows / lanes on each side, 1..5 steps.
// 1024^3 vacuum, one MI355X (bench.py --dtype f64): 16 x 64 tiles T = 4
// 105-109k Mcells/s; 32 x 32 tiles T = 4 114k; + stores deferred one plane
// (no store-ack drain per plane) 120k; T = 5 116k.
// A single-pass fp64 step moves >= 96 B/cell; T steps per pass read and write
// the six fields once (plus the tile halos).

#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "tfsf_dev.h"

namespace {

constexpr int TBW = 16;  // waves per workgroup

typedef __amdgpu_buffer_rsrc_t Rsrc;

__device__ __forceinline__ Rsrc plane_rsrc64(const double* base, int x, int nx, size_t plane) {
  const bool in = x >= 0 && x < nx;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (size_t)(in ? x : 0) * plane), (short)0,
                                           in ? (int)(plane * 8) : 0, 0x00020000);
}

__device__ __forceinline__ double bld64(Rsrc r, unsigned boff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, boff, 0, 0));
}

typedef unsigned u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void bst64(Rsrc r, unsigned boff, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), r, boff, 0, 0);
}

// DPP wave shifts of a double (two 32-bit halves): lane i gets lane i-1 (up)
// or lane i+1 (dn); lanes shifted in from outside the wave read 0 (halo)
__device__ __forceinline__ double lane_up64(double v) {
  const u2 h = __builtin_bit_cast(u2, v);
  u2 r;
  r.x = (unsigned)__builtin_amdgcn_update_dpp(0, (int)h.x, 0x138, 0xf, 0xf, false);
  r.y = (unsigned)__builtin_amdgcn_update_dpp(0, (int)h.y, 0x138, 0xf, 0xf, false);
  return __builtin_bit_cast(double, r);
}
__device__ __forceinline__ double lane_dn64(double v) {
  const u2 h = __builtin_bit_cast(u2, v);
  u2 r;
  r.x = (unsigned)__builtin_amdgcn_update_dpp(0, (int)h.x, 0x130, 0xf, 0xf, false);
  r.y = (unsigned)__builtin_amdgcn_update_dpp(0, (int)h.y, 0x130, 0xf, 0xf, false);
  return __builtin_bit_cast(double, r);
}

__device__ __forceinline__ bool xin(const Box3& b, int x) { return x >= b.lo[0] && x < b.hi[0]; }
__device__ __forceinline__ bool yzin(const Box3& b, int j, int k) {
  return j >= b.lo[1] && j < b.hi[1] && k >= b.lo[2] && k < b.hi[2];
}

struct TbSrc64 {
  double v[8];
};

struct F3d {
  double x, y, z;
};

// Drude box of an fp64 pass (DRU; the fp32 form is tb3d_mr.h DrDev, whose
// comment derives the update): inside B the E components take
//   E' = (b0 cbd) curl - b2 delta + m1 E + m2 Ep,  delta' = cbd curl,  Ep' = E
// with (delta, Ep) carried level to level in registers and read / written
// once per pass: per cell of B two 32-byte records,
//   s0 = (delta_x, delta_y, delta_z, ids: id_x | id_y << 8 | id_z << 16 in the
//   low word of the fourth double), s1 = (Ep_x, Ep_y, Ep_z, 0);
// the (b0 cbd, b2, m1, m2) rows of each component's material ids in LDS.
constexpr int DR64_MAX_IDS = 256;
struct DrDev64 {
  Box3 B;
  const double* sin0;  // x-major over B, z fastest, 4 doubles per cell
  const double* sin1;
  double* sout0;       // distinct from sin: tiles re-read halo cells other tiles own
  double* sout1;
  const double* lut;   // [3][nid][4]
  int nid;
  double cbd;
};
struct DrS64 {
  double dx, dy, dz, px, py, pz;
  unsigned id;
};
typedef unsigned u4 __attribute__((ext_vector_type(4)));

int g_num_cus64 = 0;
bool g_tb64_half = true;

// x chunk minimising rounds x (chunk + 2T) (same model as yee3d_tb.hip)
int pick_xchunk64(long long tiles_yz, int nxo, int T) {
  if (g_num_cus64 <= 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      g_num_cus64 = n;
    else
      g_num_cus64 = 256;
  }
  if (nxo <= 0) return 1;
  long long best_cost = -1;
  int best = nxo;
  for (int k = 1; k <= 256; ++k) {
    const int xc = (nxo + k - 1) / k;
    const long long chunks = (nxo + xc - 1) / xc;
    const long long rounds = (tiles_yz * chunks + g_num_cus64 - 1) / g_num_cus64;
    const long long cost = rounds * (xc + 2LL * T);
    if (best_cost < 0 || cost < best_cost) {
      best_cost = cost;
      best = xc;
    }
    if (xc == 1) break;
  }
  return best;
}

// TFS: TF/SF corrections of the sets in ``tf`` (tfsf_dev.h; the fp64 g table
// ``gtab`` of the pass's levels, k_tfsf_pass<double>), added to a target's
// new value right after its kind's update -- E + c (curl + g) -- so the H
// update of the same level reads the corrected E, as the stepped scheme does.
// The kernel streams HBM at ~43 B per cell-step, so the corrections run from
// the set table directly: per wave, bit masks of the sets touching its lanes
// (y / z faces every level, x faces on their planes only), per lane the sets
// whose target it is; the set's fields and g come through scalar loads.
// HALF: each wave holds two y rows of 32 z lanes (lanes 0-31 row 2w, 32-63
// row 2w+1): 32 x 32 tiles instead of 16 x 64, so a larger share of the
// tile is owned (T = 4: 24 x 24 of 32 x 32 = 56% against 8 x 56 of 16 x 64 =
// 44%) for the same registers.  The z shift crosses the half boundary only
// into halo lanes; y neighbours are one flat LDS row (32 lanes) apart.
template <int T, int R, bool PERCELL, bool HALF, int NW, bool TFS, bool DRU>
__global__ __launch_bounds__(64 * NW) void k_tb3d_f64(
    const double* __restrict__ exi, const double* __restrict__ eyi, const double* __restrict__ ezi,
    const double* __restrict__ hxi, const double* __restrict__ hyi, const double* __restrict__ hzi,
    double* __restrict__ exo, double* __restrict__ eyo, double* __restrict__ ezo,
    double* __restrict__ hxo, double* __restrict__ hyo, double* __restrict__ hzo,
    const double* __restrict__ cbx, const double* __restrict__ cby, const double* __restrict__ cbz,
    const double* __restrict__ dbx, const double* __restrict__ dby, const double* __restrict__ dbz, double cb,
    double db, int nx, int ny, int nz, Box3 bex, Box3 bey, Box3 bez, Box3 bhx, Box3 bhy, Box3 bhz, Box3 O,
    int xchunk, int src_i, int src_j, int src_k, int src_comp, TbSrc64 sv, int patch,
    const tb3d::TfDev* __restrict__ tf, const double* __restrict__ gtab, DrDev64 dr) {
  static_assert(!DRU || (!PERCELL && !TFS && R == 1), "Drude box: uniform media, alone");
  constexpr int LW = HALF ? 32 : 64;  // z lanes per row
  constexpr int TBZ = LW - 2 * T;       // owned z cells per tile
  constexpr int ROWS = NW * R * (HALF ? 2 : 1);
  static_assert(!HALF || R == 1, "half-wave rows hold one row per half");
  __shared__ double sX[2][4][NW][64];
  const int lane = threadIdx.x;
  const int lz = HALF ? (lane & 31) : lane;
  const int hr = HALF ? (lane >> 5) : 0;
  const int w = threadIdx.y;
  // XCD-contiguous tile order, z fastest (see yee3d_tb.hip)
  int tz, ty, tx;
  {
    const int gx = gridDim.x, gy = gridDim.y;
    const int n = gx * gy * (int)gridDim.z;
    const int p = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int n8 = n & ~7;
    const int q = p < n8 ? (p & 7) * (n8 >> 3) + (p >> 3) : p;
    const int pz = patch & 0xff, py = (patch >> 8) & 0xff;
    if (pz > 0 && py > 0) {
      // patch order (yee3d_tb.hip k_tb3d_mr): an XCD's run of tiles in PZ x
      // PY blocks, so a tile's y neighbours -- 2T shared rows, a quarter of
      // a 32-row fp64 tile -- stream the same planes on the same L2
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
  const int k = O.lo[2] - T + TBZ * tz + lz;
  const int jw = O.lo[1] - T + (ROWS - 2 * T) * ty + (HALF ? 2 * w + hr : R * w);
  const int i0 = O.lo[0] + tx * xchunk;
  const int i1 = min(i0 + xchunk, O.hi[0]);
  const bool kin = k >= 0 && k < nz;
  const bool lane_own = lz >= T && lz < LW - T;
  const size_t plane = (size_t)ny * nz;
  unsigned roff[R];
  unsigned mbits = 0;  // bit r*7 + n: row r inside box n (n = 6: stored cells)
  const Box3* bx[7] = {&bex, &bey, &bez, &bhx, &bhy, &bhz, &O};
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int j = jw + r;
    const int t = HALF ? 2 * w + hr : R * w + r;
    const bool ld_ok = kin && j >= 0 && j < ny;
    roff[r] = ld_ok ? (unsigned)(j * nz + k) * 8u : 0xF0000000u;
    const bool own = ld_ok && lane_own && t >= T && t < ROWS - T;
#pragma unroll
    for (int n = 0; n < 7; ++n) {
      const bool ok = n < 6 ? ld_ok : own;
      mbits |= (ok && yzin(*bx[n], j, k) ? 1u : 0u) << (r * 7 + n);
    }
  }
  const int rdn = w > 0 ? w - 1 : 0;
  const int rup = w < NW - 1 ? w + 1 : NW - 1;
  auto coef = [&](const double* arr, const Box3& b, int p, int r, int n, double sc) -> double {
    const bool in = xin(b, p) && ((mbits >> (r * 7 + n)) & 1u);
    if (PERCELL && arr) return in ? bld64(plane_rsrc64(arr, p, nx, plane), roff[r]) : 0.0;
    return in ? sc : 0.0;
  };
  // TF/SF (TFS): wave masks of the E / H sets touching this wave's lanes
  // (y / z-face sets: tf_c*, x-face sets: tf_x*), bit si per set index;
  // tf_lm: this lane's cell is a target of set si (set box and its
  // component's update box, y / z)
  typedef const __attribute__((address_space(4))) tb3d::TfDev* TfPtr;
  const TfPtr TFc = (TfPtr)tf;
  unsigned tf_ce = 0u, tf_ch = 0u, tf_xe = 0u, tf_xh = 0u, tf_lm = 0u;
  int tf_pe = -1, tf_ph = -1;  // x-face planes of the E / H sets: lo | hi << 16
  if constexpr (TFS) {
    const int ns = TFc->nsets;
    for (int si = 0; si < ns; ++si) {
      const int n = TFc->s[si].n;
#define TF_UB(f, d) (n == 0 ? bex.f[d] : n == 1 ? bey.f[d] : n == 2 ? bez.f[d] : n == 3 ? bhx.f[d] : n == 4 ? bhy.f[d] : bhz.f[d])
      const int ul1 = TF_UB(lo, 1), uh1 = TF_UB(hi, 1), ul2 = TF_UB(lo, 2), uh2 = TF_UB(hi, 2);
#undef TF_UB
      const bool in = kin && jw >= TFc->s[si].lo[1] && jw < TFc->s[si].hi[1] && k >= TFc->s[si].lo[2] &&
                      k < TFc->s[si].hi[2] && jw >= ul1 && jw < uh1 && k >= ul2 && k < uh2;
      const unsigned bit = 1u << si;
      tf_lm |= in ? bit : 0u;
      if (__any(in)) {
        if (TFc->s[si].fa == 0)
          (n < 3 ? tf_xe : tf_xh) |= bit;
        else
          (n < 3 ? tf_ce : tf_ch) |= bit;
      }
    }
    tf_ce = __builtin_amdgcn_readfirstlane(tf_ce);
    tf_ch = __builtin_amdgcn_readfirstlane(tf_ch);
    tf_xe = __builtin_amdgcn_readfirstlane(tf_xe);
    tf_xh = __builtin_amdgcn_readfirstlane(tf_xh);
    tf_pe = (TFc->xpl[0][0] & 0xffff) | (TFc->xpl[0][1] << 16);
    tf_ph = (TFc->xpl[1][0] & 0xffff) | (TFc->xpl[1][1] << 16);
  }
  // the corrections of kind k (0 E, 1 H) at level l on plane p to the new
  // values f of row 0 (R == 1)
  auto tf_fix = [&](int kk, int l, int p, F3d& f) {
    const int xp = kk == 0 ? tf_pe : tf_ph;
    const bool xplane = p == (xp & 0xffff) || p == (xp >> 16);
    unsigned m = (kk == 0 ? tf_ce : tf_ch) | (xplane ? (kk == 0 ? tf_xe : tf_xh) : 0u);
    while (m) {
      const int si = __builtin_ctz(m);
      m &= m - 1u;
      const int lo0 = TFc->s[si].lo[0];
      if (p < lo0 || p >= TFc->s[si].hi[0]) continue;
      const int idx = TFc->s[si].va == 0 ? p - lo0 : jw - TFc->s[si].lo[1];
      const int gi = l * TFc->ld + TFc->s[si].goff + idx;
      if (!((tf_lm >> si) & 1u)) continue;
      const double g = gtab[gi];
      const int c = TFc->s[si].n - 3 * kk;
      if (kk == 0) {
        if (c == 0) f.x += coef(cbx, bex, p, 0, 0, cb) * g;
        else if (c == 1) f.y += coef(cby, bey, p, 0, 1, cb) * g;
        else f.z += coef(cbz, bez, p, 0, 2, cb) * g;
      } else {
        if (c == 0) f.x += coef(dbx, bhx, p, 0, 3, db) * g;
        else if (c == 1) f.y += coef(dby, bhy, p, 0, 4, db) * g;
        else f.z += coef(dbz, bhz, p, 0, 5, db) * g;
      }
    }
  };
  // Drude box (DRU): the lane's byte offset in one x plane of the state
  // records (past the plane outside B in y / z), the coefficient rows in LDS
  __shared__ double sL[DRU ? 3 * DR64_MAX_IDS * 4 : 1];
  const int drz = dr.B.hi[2] - dr.B.lo[2];
  const size_t dplane = DRU ? (size_t)(dr.B.hi[1] - dr.B.lo[1]) * drz * 32u : 0;
  unsigned doff = 0xF0000000u;
  bool din = false;
  if constexpr (DRU) {
    din = kin && jw >= dr.B.lo[1] && jw < dr.B.hi[1] && k >= dr.B.lo[2] && k < dr.B.hi[2];
    if (din) doff = (unsigned)((jw - dr.B.lo[1]) * drz + (k - dr.B.lo[2])) * 32u;
    for (int i = lane + 64 * w; i < 3 * DR64_MAX_IDS; i += 64 * NW) {
      const int c = i / DR64_MAX_IDS, id = i - c * DR64_MAX_IDS;
#pragma unroll
      for (int q = 0; q < 4; ++q) sL[4 * i + q] = id < dr.nid ? dr.lut[(c * dr.nid + id) * 4 + q] : 0.0;
    }
    __syncthreads();
  }
  const bool wave_d = DRU && __any(din);
  auto dr_rsrc = [&](const double* base, int p) -> Rsrc {
    const bool in = xin(dr.B, p);
    return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + (in ? (size_t)(p - dr.B.lo[0]) * dplane : 0)),
                                             (short)0, in ? (int)dplane : 0, 0x00020000);
  };
  auto dr_load = [&](int p, DrS64& S) {
    const Rsrc r0 = dr_rsrc(dr.sin0, p), r1 = dr_rsrc(dr.sin1, p);
    const u4 a = __builtin_amdgcn_raw_buffer_load_b128(r0, doff, 0, 0);
    const u4 b = __builtin_amdgcn_raw_buffer_load_b128(r0, doff, 16, 0);
    const u4 c = __builtin_amdgcn_raw_buffer_load_b128(r1, doff, 0, 0);
    const u2 d = __builtin_amdgcn_raw_buffer_load_b64(r1, doff, 16, 0);
    S.dx = __builtin_bit_cast(double, u2{a.x, a.y});
    S.dy = __builtin_bit_cast(double, u2{a.z, a.w});
    S.dz = __builtin_bit_cast(double, u2{b.x, b.y});
    S.id = b.z;
    S.px = __builtin_bit_cast(double, u2{c.x, c.y});
    S.py = __builtin_bit_cast(double, u2{c.z, c.w});
    S.pz = __builtin_bit_cast(double, d);
  };
  // DS[l]: the output of level l in the previous trip (plane X - 1 - l), the
  // input of level l + 1 in this one; Dc: the input of the level running;
  // Dnx: the next trip's level-0 input; DL: the last level's output
  constexpr int NDS = DRU ? (T > 1 ? T - 1 : 1) : 1;
  DrS64 DS[NDS], Dnx{}, Dc{}, DL{};
  if constexpr (DRU) {
#pragma unroll
    for (int l = 0; l < NDS; ++l) DS[l] = DrS64{};
    if (wave_d) dr_load(i0 - T, Dnx);
  }
  F3d Hp[T][R], Ep[T][R];
#pragma unroll
  for (int l = 0; l < T; ++l)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      Hp[l][r] = {0.0, 0.0, 0.0};
      Ep[l][r] = {0.0, 0.0, 0.0};
    }
  int buf = 0;
  auto load_plane = [&](int X, F3d* H, F3d* E) {
    const Rsrc rhx = plane_rsrc64(hxi, X, nx, plane), rhy = plane_rsrc64(hyi, X, nx, plane);
    const Rsrc rhz = plane_rsrc64(hzi, X, nx, plane), rex = plane_rsrc64(exi, X, nx, plane);
    const Rsrc rey = plane_rsrc64(eyi, X, nx, plane), rez = plane_rsrc64(ezi, X, nx, plane);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      H[r] = {bld64(rhx, roff[r]), bld64(rhy, roff[r]), bld64(rhz, roff[r])};
      E[r] = {bld64(rex, roff[r]), bld64(rey, roff[r]), bld64(rez, roff[r])};
    }
  };
  // outputs of plane X are stored one plane late, after the next prefetch:
  // the stores are issued unconditionally, masked by an out-of-range buffer
  // offset (dropped by the descriptor), so the wait at the top of a plane
  // covers loads and stores that were both issued a whole plane earlier
  // (with stores in flight the compiler drains vmcnt: storing right before
  // that wait stalled every plane on the write acknowledgements)
  F3d Ed[R], Hd[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    Ed[r] = {0.0, 0.0, 0.0};
    Hd[r] = {0.0, 0.0, 0.0};
  }
  auto store_out = [&](int Xs) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool own = (mbits >> (r * 7 + 6)) & 1u;
      const int pe = Xs - T + 1;
      const unsigned oe = own && pe >= i0 && pe < i1 ? roff[r] : 0xF0000000u;
      bst64(plane_rsrc64(exo, pe, nx, plane), oe, Ed[r].x);
      bst64(plane_rsrc64(eyo, pe, nx, plane), oe, Ed[r].y);
      bst64(plane_rsrc64(ezo, pe, nx, plane), oe, Ed[r].z);
      const int ph = Xs - T;
      const unsigned oh = own && ph >= i0 && ph < i1 ? roff[r] : 0xF0000000u;
      bst64(plane_rsrc64(hxo, ph, nx, plane), oh, Hd[r].x);
      bst64(plane_rsrc64(hyo, ph, nx, plane), oh, Hd[r].y);
      bst64(plane_rsrc64(hzo, ph, nx, plane), oh, Hd[r].z);
    }
  };
  F3d Hnx[R], Enx[R];
  load_plane(i0 - T, Hnx, Enx);
  for (int X = i0 - T; X <= i1 + T - 1; ++X) {
    F3d Hc[R], Ec[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      Hc[r] = Hnx[r];
      Ec[r] = Enx[r];
    }
    if constexpr (DRU) {
      // this trip's level-0 state; the next trip's in flight before the field prefetch
      Dc = Dnx;
      if (wave_d) dr_load(X + 1, Dnx);
    }
    load_plane(X + 1, Hnx, Enx);
    store_out(X - 1);  // the first plane's are out of [i0, i1): dropped
    F3d En[R];
#pragma unroll
    for (int l = 0; l < T; ++l) {
      const int pe = X - l;
      sX[buf][0][w][lane] = Hc[R - 1].z;
      sX[buf][1][w][lane] = Hc[R - 1].x;
      sX[buf][2][w][lane] = Ep[l][0].x;
      sX[buf][3][w][lane] = Ep[l][0].z;
      __syncthreads();
      double hz_dn, hx_dn, ex_up, ez_up;
      if constexpr (HALF) {
        // row j -/+ 1 is 32 lanes down / up in the flat [TBW * 64] slot
        const int fl = w * 64 + lane;
        const int fdn = fl >= 32 ? fl - 32 : fl;
        const int fup = fl < NW * 64 - 32 ? fl + 32 : fl;
        hz_dn = (&sX[buf][0][0][0])[fdn];
        hx_dn = (&sX[buf][1][0][0])[fdn];
        ex_up = (&sX[buf][2][0][0])[fup];
        ez_up = (&sX[buf][3][0][0])[fup];
      } else {
        hz_dn = sX[buf][0][rdn][lane];
        hx_dn = sX[buf][1][rdn][lane];
        ex_up = sX[buf][2][rup][lane];
        ez_up = sX[buf][3][rup][lane];
      }
      buf ^= 1;
      const bool src_plane = src_comp >= 0 && pe == src_i;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double hz_j = r == 0 ? hz_dn : Hc[r > 0 ? r - 1 : 0].z;
        const double hx_j = r == 0 ? hx_dn : Hc[r > 0 ? r - 1 : 0].x;
        const double hy_k = lane_up64(Hc[r].y);
        const double hx_k = lane_up64(Hc[r].x);
        const double cx = (Hc[r].z - hz_j) - (Hc[r].y - hy_k);
        const double cy = (Hc[r].x - hx_k) - (Hc[r].z - Hp[l][r].z);
        const double cz = (Hc[r].y - Hp[l][r].y) - (Hc[r].x - hx_j);
        En[r].x = Ec[r].x + coef(cbx, bex, pe, r, 0, cb) * cx;
        En[r].y = Ec[r].y + coef(cby, bey, pe, r, 1, cb) * cy;
        En[r].z = Ec[r].z + coef(cbz, bez, pe, r, 2, cb) * cz;
        if constexpr (DRU) {
          const DrS64 st = Dc;
          if (wave_d && xin(dr.B, pe)) {
            const double* kx = &sL[4 * (st.id & 0xffu)];
            const double* ky = &sL[4 * (DR64_MAX_IDS + ((st.id >> 8) & 0xffu))];
            const double* kz = &sL[4 * (2 * DR64_MAX_IDS + ((st.id >> 16) & 0xffu))];
            const double nx_ = kx[0] * cx - kx[1] * st.dx + kx[2] * Ec[r].x + kx[3] * st.px;
            const double ny_ = ky[0] * cy - ky[1] * st.dy + ky[2] * Ec[r].y + ky[3] * st.py;
            const double nz_ = kz[0] * cz - kz[1] * st.dz + kz[2] * Ec[r].z + kz[3] * st.pz;
            if (din) {
              En[r].x = nx_;
              En[r].y = ny_;
              En[r].z = nz_;
            }
          }
          DrS64 o;
          o.dx = dr.cbd * cx;
          o.dy = dr.cbd * cy;
          o.dz = dr.cbd * cz;
          o.px = Ec[r].x;
          o.py = Ec[r].y;
          o.pz = Ec[r].z;
          o.id = st.id;
          if (l < T - 1) {
            Dc = DS[l < T - 1 ? l : 0];
            DS[l < T - 1 ? l : 0] = o;
          } else {
            DL = o;
          }
        }
        if constexpr (TFS) tf_fix(0, l, pe, En[r]);
        if (src_plane && jw + r == src_j && src_k == k) {
          if (src_comp == 0) En[r].x = sv.v[l];
          if (src_comp == 1) En[r].y = sv.v[l];
          if (src_comp == 2) En[r].z = sv.v[l];
        }
      }
      const int ph = pe - 1;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double ex_jn = r == R - 1 ? ex_up : Ep[l][r < R - 1 ? r + 1 : r].x;
        const double ez_jn = r == R - 1 ? ez_up : Ep[l][r < R - 1 ? r + 1 : r].z;
        const double ey_k = lane_dn64(Ep[l][r].y);
        const double ex_k = lane_dn64(Ep[l][r].x);
        F3d Hn;
        Hn.x = Hp[l][r].x + coef(dbx, bhx, ph, r, 3, db) * ((ey_k - Ep[l][r].y) - (ez_jn - Ep[l][r].z));
        Hn.y = Hp[l][r].y + coef(dby, bhy, ph, r, 4, db) * ((En[r].z - Ep[l][r].z) - (ex_k - Ep[l][r].x));
        Hn.z = Hp[l][r].z + coef(dbz, bhz, ph, r, 5, db) * ((ex_jn - Ep[l][r].x) - (En[r].y - Ep[l][r].y));
        if constexpr (TFS) tf_fix(1, l, ph, Hn);
        Ec[r] = Ep[l][r];
        Ep[l][r] = En[r];
        Hp[l][r] = Hc[r];
        Hc[r] = Hn;
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      Ed[r] = En[r];
      Hd[r] = Hc[r];
    }
    if constexpr (DRU) {
      // the last level's state (plane X - T + 1): owned cells of B
      const int pe = X - T + 1;
      const Rsrc r0 = dr_rsrc(dr.sout0, pe), r1 = dr_rsrc(dr.sout1, pe);
      const bool own = (mbits >> 6) & 1u;
      const unsigned o = (wave_d && own && din && pe >= i0 && pe < i1) ? doff : 0xF0000000u;
      const u2 vx = __builtin_bit_cast(u2, DL.dx), vy = __builtin_bit_cast(u2, DL.dy), vz = __builtin_bit_cast(u2, DL.dz);
      const u2 px = __builtin_bit_cast(u2, DL.px), py = __builtin_bit_cast(u2, DL.py), pz = __builtin_bit_cast(u2, DL.pz);
      __builtin_amdgcn_raw_buffer_store_b128(u4{vx.x, vx.y, vy.x, vy.y}, r0, o, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(u4{vz.x, vz.y, DL.id, 0u}, r0, o, 16, 0);
      __builtin_amdgcn_raw_buffer_store_b128(u4{px.x, px.y, py.x, py.y}, r1, o, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(u4{pz.x, pz.y, 0u, 0u}, r1, o, 16, 0);
    }
  }
  store_out(i1 + T - 1);
}

// patch order of the XCD tile run: pz | (py << 8), 0 = z fastest.  Default
// 2 x 8 (z x y tiles): 1024^3 fp64 123.3k vs 118.3k Mcells/s z fastest, means
// of 3 / 4 alternating runs (profiles/fp64_patch_r5.md); FDTD3D_TB64_PATCH=
// "PZxPY" at first use ("0x0": z fastest), fdtd_set_tb64_patch
int g_tb64_patch = -1;
int tb64_patch() {
  if (g_tb64_patch < 0) {
    g_tb64_patch = 2 | (8 << 8);
    const char* e = getenv("FDTD3D_TB64_PATCH");
    int pz = 0, py = 0;
    if (e && sscanf(e, "%dx%d", &pz, &py) == 2 && pz >= 0 && py >= 0 && pz < 256 && py < 256)
      g_tb64_patch = (pz > 0 && py > 0) ? (pz | (py << 8)) : 0;
  }
  return g_tb64_patch;
}

template <int T, int R, bool HALF, int NW = TBW>
int launch_tb64(bool pc, const double* const* ein, const double* const* hin, double* const* eout,
                double* const* hout, const double* const* cbs, const double* const* dbs, double cb, double db,
                int nx, int ny, int nz, const Box3* b, const Box3& O, int xchunk, const int* src,
                const TbSrc64& sv, hipStream_t s, const tb3d::TfDev* tf = nullptr, const double* gtab = nullptr,
                const DrDev64* dr = nullptr) {
  constexpr int TBZ = (HALF ? 32 : 64) - 2 * T;
  const long long gz = cdiv(O.hi[2] - O.lo[2], TBZ);
  const long long gy = cdiv(O.hi[1] - O.lo[1], NW * R * (HALF ? 2 : 1) - 2 * T);
  if (xchunk <= 0) xchunk = pick_xchunk64(gz * gy, O.hi[0] - O.lo[0], T);
  dim3 grid((unsigned)gz, (unsigned)gy, cdiv(O.hi[0] - O.lo[0], xchunk));
#define TB64_ARGS                                                                                              \
  ein[0], ein[1], ein[2], hin[0], hin[1], hin[2], eout[0], eout[1], eout[2], hout[0], hout[1], hout[2],      \
      cbs[0], cbs[1], cbs[2], dbs[0], dbs[1], dbs[2], cb, db, nx, ny, nz, b[0], b[1], b[2], b[3], b[4], b[5], \
      O, xchunk, src[0], src[1], src[2], src[3], sv, tb64_patch(), tf, gtab, dr ? *dr : DrDev64{}
  if (dr) {
    if constexpr (NW == 8) {
      if (pc || tf) return (int)hipErrorInvalidValue;
      k_tb3d_f64<T, R, false, HALF, NW, false, true><<<grid, dim3(64, NW), 0, s>>>(TB64_ARGS);
    } else {
      return (int)hipErrorInvalidValue;
    }
  } else if (tf && gtab) {
    if (pc)
      k_tb3d_f64<T, R, true, HALF, NW, true, false><<<grid, dim3(64, NW), 0, s>>>(TB64_ARGS);
    else
      k_tb3d_f64<T, R, false, HALF, NW, true, false><<<grid, dim3(64, NW), 0, s>>>(TB64_ARGS);
  } else if (pc) {
    k_tb3d_f64<T, R, true, HALF, NW, false, false><<<grid, dim3(64, NW), 0, s>>>(TB64_ARGS);
  } else {
    k_tb3d_f64<T, R, false, HALF, NW, false, false><<<grid, dim3(64, NW), 0, s>>>(TB64_ARGS);
  }
#undef TB64_ARGS
  FDTD_RETURN_LAUNCH_STATUS();
}

}  // namespace

FDTD_API int fdtd_tb64_max_steps() { return 5; }

// 1: two rows of 32 lanes per wave (32 x 32 tiles, default); 0: one row of
// 64 lanes (16 x 64 tiles)
FDTD_API void fdtd_set_tb64_shape(int half) { g_tb64_half = half != 0; }

// patch order of the fp64 kernel's XCD tile run: pz x py tiles (0: z fastest)
FDTD_API void fdtd_set_tb64_patch(int pz, int py) {
  g_tb64_patch = (pz > 0 && py > 0 && pz < 256 && py < 256) ? (pz | (py << 8)) : 0;
}

namespace {
int tb64_run(const double* const* ein, const double* const* hin, double* const* eout, double* const* hout,
             const double* const* cbs, const double* const* dbs, double cb, double db, int nx, int ny, int nz,
             const int* boxes, const int* obox, int xchunk, int steps, const int* src, const double* src_vals,
             const tb3d::TfDev* tf, const double* gtab, void* stream) {
  if (steps < 1 || steps > 5) return (int)hipErrorInvalidValue;
  Box3 b[6];
  for (int n = 0; n < 6; ++n) b[n] = make_box(boxes + 6 * n);
  const Box3 O = make_box(obox);
  if (box_empty(O)) return 0;
  TbSrc64 sv;
  for (int l = 0; l < 8; ++l) sv.v[l] = (src[3] >= 0 && l < steps) ? src_vals[l] : 0.0;
  const bool pc = cbs[0] != nullptr || dbs[0] != nullptr;  // a null kind uses its scalar
  hipStream_t s = (hipStream_t)stream;
  // one row per wave: two rows of fp64 state spill from T = 2 on
#define TB64(TT, HF) \
  launch_tb64<TT, 1, HF>(pc, ein, hin, eout, hout, cbs, dbs, cb, db, nx, ny, nz, b, O, xchunk, src, sv, s, tf, gtab)
  if (g_tb64_half) {
    switch (steps) {
      case 1: return TB64(1, true);
      case 2: return TB64(2, true);
      case 3: return TB64(3, true);
      case 4: return TB64(4, true);
      case 5: return TB64(5, true);
    }
  } else {
    switch (steps) {
      case 1: return TB64(1, false);
      case 2: return TB64(2, false);
      case 3: return TB64(3, false);
      case 4: return TB64(4, false);
      case 5: return TB64(5, false);
    }
  }
#undef TB64
  return (int)hipErrorInvalidValue;
}
}  // namespace

// fp64 counterpart of fdtd_tb3d_v4_f32 (same arguments, double arrays), 1..5
// steps per pass, any nz.
FDTD_API int fdtd_tb3d_f64(const double* const* ein, const double* const* hin, double* const* eout,
                           double* const* hout, const double* const* cbs, const double* const* dbs, double cb,
                           double db, int nx, int ny, int nz, const int* boxes, const int* obox, int xchunk,
                           int steps, const int* src, const double* src_vals, void* stream) {
  return tb64_run(ein, hin, eout, hout, cbs, dbs, cb, db, nx, ny, nz, boxes, obox, xchunk, steps, src, src_vals,
                  nullptr, nullptr, stream);
}

// ... with the Drude box folded in (DrDev64; the fp64 counterpart of
// fdtd_tb3d_drude_f32): ``bbox`` = the box B (local, inside the E update
// boxes), ``sin`` / ``sout`` = the two 32-byte state records per cell of B in
// / out (distinct), ``lut`` = [3][nid][4] doubles (b0 cbd, b2, m1, m2),
// ``cbd`` the D coefficient; uniform media elsewhere.  Tiles of 8 waves x two
// 32-lane rows (the state of T - 1 levels rides in registers: <= 256 VGPRs).
FDTD_API int fdtd_tb3d_drude_f64(const double* const* ein, const double* const* hin, double* const* eout,
                                 double* const* hout, double cb, double db, int nx, int ny, int nz, const int* boxes,
                                 const int* obox, int xchunk, int steps, const int* src, const double* src_vals,
                                 const int* bbox, void* const* sin, void* const* sout, const double* lut, int nid,
                                 double cbd, void* stream) {
  if (steps < 1 || steps > 5 || !sin || !sout || !lut || nid < 1 || nid > DR64_MAX_IDS) return (int)hipErrorInvalidValue;
  Box3 b[6];
  for (int n = 0; n < 6; ++n) b[n] = make_box(boxes + 6 * n);
  const Box3 O = make_box(obox);
  if (box_empty(O)) return 0;
  DrDev64 D;
  D.B = make_box(bbox);
  if (box_empty(D.B)) return (int)hipErrorInvalidValue;
  for (int d = 0; d < 3; ++d) {
    if (D.B.lo[d] < 0 || D.B.hi[d] > (d == 0 ? nx : d == 1 ? ny : nz)) return (int)hipErrorInvalidValue;
    for (int n = 0; n < 3; ++n)
      if (D.B.lo[d] < b[n].lo[d] || D.B.hi[d] > b[n].hi[d]) return (int)hipErrorInvalidValue;
  }
  // one x plane of a state array is addressed by a 32-bit byte offset
  if ((long long)(D.B.hi[1] - D.B.lo[1]) * (D.B.hi[2] - D.B.lo[2]) * 32 >= (1ll << 31)) return (int)hipErrorInvalidValue;
  if (!sin[0] || !sin[1] || !sout[0] || !sout[1] || sin[0] == sout[0] || sin[1] == sout[1])
    return (int)hipErrorInvalidValue;
  D.sin0 = (const double*)sin[0];
  D.sin1 = (const double*)sin[1];
  D.sout0 = (double*)sout[0];
  D.sout1 = (double*)sout[1];
  D.lut = lut;
  D.nid = nid;
  D.cbd = cbd;
  TbSrc64 sv;
  for (int l = 0; l < 8; ++l) sv.v[l] = (src[3] >= 0 && l < steps) ? src_vals[l] : 0.0;
  const double* none[3] = {nullptr, nullptr, nullptr};
  hipStream_t s = (hipStream_t)stream;
#define TB64D(TT) \
  launch_tb64<TT, 1, true, 8>(false, ein, hin, eout, hout, none, none, cb, db, nx, ny, nz, b, O, xchunk, src, sv, s, \
                              nullptr, nullptr, &D)
  switch (steps) {
    case 1: return TB64D(1);
    case 2: return TB64D(2);
    case 3: return TB64D(3);
    case 4: return TB64D(4);
    case 5: return TB64D(5);
  }
#undef TB64D
  return (int)hipErrorInvalidValue;
}

// ... with the TF/SF corrections of the device set table ``tf`` (tfsf_dev.h
// TfDev, filled by models/tfsf.py TfsfSets) and the fp64 g table ``gtab`` of
// the pass's first level (fdtd_tfsf_pass_f64 / fdtd_tfsf_table_f64)
FDTD_API int fdtd_tb3d_tf_f64(const double* const* ein, const double* const* hin, double* const* eout,
                              double* const* hout, const double* const* cbs, const double* const* dbs, double cb,
                              double db, int nx, int ny, int nz, const int* boxes, const int* obox, int xchunk,
                              int steps, const int* src, const double* src_vals, const void* tf, const double* gtab,
                              void* stream) {
  if (!tf || !gtab) return (int)hipErrorInvalidValue;
  return tb64_run(ein, hin, eout, hout, cbs, dbs, cb, db, nx, ny, nz, boxes, obox, xchunk, steps, src, src_vals,
                  (const tb3d::TfDev*)tf, gtab, stream);
}
