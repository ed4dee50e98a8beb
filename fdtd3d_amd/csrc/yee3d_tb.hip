// Temporally blocked fp32 3D Yee kernel: T full leapfrog steps per HBM pass.
//
// The single-pass kernels (yee3d_v4.hip) move >= 48 B/cell/step, so one
// MI355X tops out near 6.3 TB/s / 48 B = 131 Gcells/s however well they are
// tiled.  This kernel reads E^n, H^n once and writes E^{n+T}, H^{n+T} once
// (reference has no counterpart: its CUDA path is one launch per component and
// step, Source/Cuda/CudaInterface.cu:583-812).
//
// Tile (one workgroup, 16 waves = 1024 threads, one workgroup per CU):
//   * z: a wave row of 64 lanes x float4 = 256 cells; lanes 0 and 63 are halo,
//     lanes 1..62 (248 cells) are owned -> tiles advance by 248 cells.
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

#include "common.h"
#include "vec4.h"

namespace {

constexpr int TBW = 16;  // waves (y rows) per workgroup
constexpr int TBZ = 248; // owned z cells per tile (lanes 1..62)

struct F3 {
  float4 x, y, z;
};

struct TbSrc {
  float v[8];  // hard-source value applied after E update of level l
};

// Memory access through buffer descriptors: one descriptor per (array, x
// plane) built in SGPRs from the wave-uniform plane index, plus ONE 32-bit
// per-lane byte offset shared by every array (buffer_load ... offen).  Flat
// 64-bit addressing would keep a per-lane pointer per array live across the
// x loop (24 VGPRs for 12 arrays) and spill.  Offsets past the descriptor's
// size read 0 / drop the store, which is how rows and planes outside the
// array are handled -- no per-lane load guards.
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t Rsrc;

__device__ __forceinline__ Rsrc plane_rsrc(const float* base, int x, int nx, size_t plane) {
  const bool in = x >= 0 && x < nx;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (size_t)(in ? x : 0) * plane), (short)0,
                                           in ? (int)(plane * 4) : 0, 0x00020000);
}

__device__ __forceinline__ float4 bld(Rsrc r, unsigned boff) {
  const v4f v = __builtin_amdgcn_raw_buffer_load_b128(r, boff, 0, 0);
  return make_float4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ void bst(Rsrc r, unsigned boff, const float4& v, unsigned mask) {
  if (mask == 0xFu) {
    v4f t = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(t, r, boff, 0, 0);
  } else if (mask) {
    // the b32 builtin takes the raw bits (an implicit float->uint would convert)
    if (mask & 1u) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v.x), r, boff, 0, 0);
    if (mask & 2u) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v.y), r, boff + 4, 0, 0);
    if (mask & 4u) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v.z), r, boff + 8, 0, 0);
    if (mask & 8u) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v.w), r, boff + 12, 0, 0);
  }
}

__device__ __forceinline__ bool xin(const Box3& b, int x) { return x >= b.lo[0] && x < b.hi[0]; }

// elements of c whose bit is set in m, zero elsewhere
__device__ __forceinline__ float4 cmask(const float4& c, unsigned m) {
  return make_float4((m & 1u) ? c.x : 0.f, (m & 2u) ? c.y : 0.f, (m & 4u) ? c.z : 0.f, (m & 8u) ? c.w : 0.f);
}

// v + c * ((a - b) - (d - e))
__device__ __forceinline__ float4 upd(const float4& v, const float4& c, const float4& a, const float4& b,
                                      const float4& d, const float4& e) {
  return make_float4(v.x + c.x * ((a.x - b.x) - (d.x - e.x)), v.y + c.y * ((a.y - b.y) - (d.y - e.y)),
                     v.z + c.z * ((a.z - b.z) - (d.z - e.z)), v.w + c.w * ((a.w - b.w) - (d.w - e.w)));
}

// z-1 / z+1 neighbours of a lane's 4 cells (s = the cell beyond the group)
__device__ __forceinline__ float4 zm1(const float4& v, float s) { return make_float4(s, v.x, v.y, v.z); }
__device__ __forceinline__ float4 zp1(const float4& v, float s) { return make_float4(v.y, v.z, v.w, s); }

template <int T, bool PERCELL>
__global__ __launch_bounds__(64 * TBW) void k_tb3d_v4(
    const float* __restrict__ exi, const float* __restrict__ eyi, const float* __restrict__ ezi,
    const float* __restrict__ hxi, const float* __restrict__ hyi, const float* __restrict__ hzi,
    float* __restrict__ exo, float* __restrict__ eyo, float* __restrict__ ezo,
    float* __restrict__ hxo, float* __restrict__ hyo, float* __restrict__ hzo,
    const float* __restrict__ cbx, const float* __restrict__ cby, const float* __restrict__ cbz,
    const float* __restrict__ dbx, const float* __restrict__ dby, const float* __restrict__ dbz, float cb,
    float db, int nx, int ny, int nz, Box3 bex, Box3 bey, Box3 bez, Box3 bhx, Box3 bhy, Box3 bhz, Box3 O,
    int xchunk, int src_i, int src_j, int src_k, int src_comp, TbSrc sv) {
  __shared__ float4 sX[2][4][TBW][64];  // [buffer][field][row][lane]: 128 KiB
  const int lane = threadIdx.x;
  const int w = threadIdx.y;
  const int kb = (O.lo[2] & ~3) - 4 + TBZ * (int)blockIdx.x + 4 * lane;
  const int j = O.lo[1] - T + (TBW - 2 * T) * (int)blockIdx.y + w;
  const int i0 = O.lo[0] + (int)blockIdx.z * xchunk;
  const int i1 = min(i0 + xchunk, O.hi[0]);
  const bool ld_ok = j >= 0 && j < ny && kb >= 0 && kb < nz;
  const bool own = ld_ok && lane >= 1 && lane <= 62 && w >= T && w < TBW - T && j >= O.lo[1] && j < O.hi[1];
  const size_t plane = (size_t)ny * nz;
  // per-lane 32-bit offset inside a plane; plane bases are wave-uniform (SGPR)
  const unsigned row = ld_ok ? (unsigned)(j * nz + kb) * 4u : 0xF0000000u;  // byte offset (past end: reads 0)
  // element masks of the update boxes (all rows) and of the stored cells
  const unsigned mex = ld_ok ? kmask(bex, j, kb) : 0u;
  const unsigned mey = ld_ok ? kmask(bey, j, kb) : 0u;
  const unsigned mez = ld_ok ? kmask(bez, j, kb) : 0u;
  const unsigned mhx = ld_ok ? kmask(bhx, j, kb) : 0u;
  const unsigned mhy = ld_ok ? kmask(bhy, j, kb) : 0u;
  const unsigned mhz = ld_ok ? kmask(bhz, j, kb) : 0u;
  const unsigned mo = own ? kmask(O, j, kb) : 0u;
  const bool src_here = src_comp >= 0 && j == src_j && src_k >= kb && src_k < kb + 4;
  const int src_q = src_k - kb;
  const int rdn = w > 0 ? w - 1 : 0;
  const int rup = w < TBW - 1 ? w + 1 : TBW - 1;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);

  // carried state (see header): Hp[l] = H_l(X-1-l), Ep[l] = E_{l+1}(X-1-l)
  F3 Hp[T], Ep[T];
#pragma unroll
  for (int l = 0; l < T; ++l) {
    Hp[l].x = Hp[l].y = Hp[l].z = z4;
    Ep[l].x = Ep[l].y = Ep[l].z = z4;
  }
  int buf = 0;

  for (int X = i0 - T; X <= i1 + T - 1; ++X) {
    F3 Hc, Ec;
    Hc.x = bld(plane_rsrc(hxi, X, nx, plane), row);
    Hc.y = bld(plane_rsrc(hyi, X, nx, plane), row);
    Hc.z = bld(plane_rsrc(hzi, X, nx, plane), row);
    Ec.x = bld(plane_rsrc(exi, X, nx, plane), row);
    Ec.y = bld(plane_rsrc(eyi, X, nx, plane), row);
    Ec.z = bld(plane_rsrc(ezi, X, nx, plane), row);
    F3 En;
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
      const float4 hz_j = sX[buf][0][rdn][lane];
      const float4 hx_j = sX[buf][1][rdn][lane];
      const float4 ex_jn = sX[buf][2][rup][lane];
      const float4 ez_jn = sX[buf][3][rup][lane];
      buf ^= 1;
      const float hy_k0 = __shfl_up(Hc.y.w, 1, 64);
      const float hx_k0 = __shfl_up(Hc.x.w, 1, 64);
      // coefficients are zeroed outside each component's update box, so the
      // arithmetic is branch-free float4 work and untouched cells keep E_l
      const float4 cex = cmask(PERCELL ? bld(plane_rsrc(cbx, xin(bex, pe) ? pe : -1, nx, plane), row) : make_float4(cb, cb, cb, cb),
                               xin(bex, pe) ? mex : 0u);
      En.x = upd(Ec.x, cex, Hc.z, hz_j, Hc.y, zm1(Hc.y, hy_k0));
      const float4 cey = cmask(PERCELL ? bld(plane_rsrc(cby, xin(bey, pe) ? pe : -1, nx, plane), row) : make_float4(cb, cb, cb, cb),
                               xin(bey, pe) ? mey : 0u);
      En.y = upd(Ec.y, cey, Hc.x, zm1(Hc.x, hx_k0), Hc.z, Hp[l].z);
      const float4 cez = cmask(PERCELL ? bld(plane_rsrc(cbz, xin(bez, pe) ? pe : -1, nx, plane), row) : make_float4(cb, cb, cb, cb),
                               xin(bez, pe) ? mez : 0u);
      En.z = upd(Ec.z, cez, Hc.y, Hp[l].y, Hc.x, hx_j);
      if (src_here && pe == src_i) {
        if (src_comp == 0) f4set(En.x, src_q, sv.v[l]);
        if (src_comp == 1) f4set(En.y, src_q, sv.v[l]);
        if (src_comp == 2) f4set(En.z, src_q, sv.v[l]);
      }
      // ---- H_{l+1} on plane ph = pe-1 from E_{l+1}(ph) = Ep[l], E_{l+1}(pe) = En,
      //      H_l(ph) = Hp[l]
      const int ph = pe - 1;
      const float ey_k3 = __shfl_down(Ep[l].y.x, 1, 64);
      const float ex_k3 = __shfl_down(Ep[l].x.x, 1, 64);
      F3 Hn;
      const float4 chx = cmask(PERCELL ? bld(plane_rsrc(dbx, xin(bhx, ph) ? ph : -1, nx, plane), row) : make_float4(db, db, db, db),
                               xin(bhx, ph) ? mhx : 0u);
      Hn.x = upd(Hp[l].x, chx, zp1(Ep[l].y, ey_k3), Ep[l].y, ez_jn, Ep[l].z);
      const float4 chy = cmask(PERCELL ? bld(plane_rsrc(dby, xin(bhy, ph) ? ph : -1, nx, plane), row) : make_float4(db, db, db, db),
                               xin(bhy, ph) ? mhy : 0u);
      Hn.y = upd(Hp[l].y, chy, En.z, Ep[l].z, zp1(Ep[l].x, ex_k3), Ep[l].x);
      const float4 chz = cmask(PERCELL ? bld(plane_rsrc(dbz, xin(bhz, ph) ? ph : -1, nx, plane), row) : make_float4(db, db, db, db),
                               xin(bhz, ph) ? mhz : 0u);
      Hn.z = upd(Hp[l].z, chz, ex_jn, Ep[l].x, En.y, Ep[l].y);
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
        bst(plane_rsrc(exo, pe, nx, plane), row, En.x, mo);
        bst(plane_rsrc(eyo, pe, nx, plane), row, En.y, mo);
        bst(plane_rsrc(ezo, pe, nx, plane), row, En.z, mo);
      }
      const int ph = X - T;
      if (ph >= i0 && ph < i1) {
        bst(plane_rsrc(hxo, ph, nx, plane), row, Hc.x, mo);
        bst(plane_rsrc(hyo, ph, nx, plane), row, Hc.y, mo);
        bst(plane_rsrc(hzo, ph, nx, plane), row, Hc.z, mo);
      }
    }
  }
}

template <int T, bool PERCELL>
int launch_tb(const float* const* ein, const float* const* hin, float* const* eout, float* const* hout,
              const float* const* cbs, const float* const* dbs, float cb, float db, int nx, int ny, int nz,
              const Box3* b, const Box3& O, int xchunk, const int* src, const TbSrc& sv, hipStream_t s) {
  dim3 grid(cdiv(O.hi[2] - (O.lo[2] & ~3), TBZ), cdiv(O.hi[1] - O.lo[1], TBW - 2 * T),
            cdiv(O.hi[0] - O.lo[0], xchunk));
  k_tb3d_v4<T, PERCELL><<<grid, dim3(64, TBW), 0, s>>>(
      ein[0], ein[1], ein[2], hin[0], hin[1], hin[2], eout[0], eout[1], eout[2], hout[0], hout[1], hout[2],
      cbs[0], cbs[1], cbs[2], dbs[0], dbs[1], dbs[2], cb, db, nx, ny, nz, b[0], b[1], b[2], b[3], b[4], b[5], O,
      xchunk, src[0], src[1], src[2], src[3], sv);
  FDTD_RETURN_LAUNCH_STATUS();
}

}  // namespace

// T fused leapfrog steps: reads ein/hin, writes eout/hout (distinct buffers)
// on the output box `obox` (lo[3], hi[3]).  `boxes` = 6 update boxes
// (Ex Ey Ez Hx Hy Hz).  `src` = {i, j, k, comp} of a hard E point source (comp
// -1: none) with the value of each of the T E half steps in `src_vals`.
FDTD_API int fdtd_tb3d_v4_f32(const float* const* ein, const float* const* hin, float* const* eout,
                              float* const* hout, const float* const* cbs, const float* const* dbs, double cb,
                              double db, int nx, int ny, int nz, const int* boxes, const int* obox, int xchunk,
                              int steps, const int* src, const double* src_vals, void* stream) {
  if (nz % 4 != 0 || steps < 1 || steps > 4) return (int)hipErrorInvalidValue;
  Box3 b[6];
  for (int n = 0; n < 6; ++n) b[n] = make_box(boxes + 6 * n);
  const Box3 O = make_box(obox);
  if (box_empty(O)) return 0;
  if (xchunk <= 0) xchunk = 64;
  TbSrc sv;
  for (int l = 0; l < 8; ++l) sv.v[l] = (src[3] >= 0 && l < steps) ? (float)src_vals[l] : 0.f;
  hipStream_t s = (hipStream_t)stream;
  const bool pc = cbs[0] != nullptr;
#define TB_CASE(TT)                                                                                              \
  case TT:                                                                                                       \
    return pc ? launch_tb<TT, true>(ein, hin, eout, hout, cbs, dbs, (float)cb, (float)db, nx, ny, nz, b, O,     \
                                    xchunk, src, sv, s)                                                          \
              : launch_tb<TT, false>(ein, hin, eout, hout, cbs, dbs, (float)cb, (float)db, nx, ny, nz, b, O,    \
                                     xchunk, src, sv, s);
  switch (steps) {
    TB_CASE(1)
    TB_CASE(2)
    TB_CASE(3)
    TB_CASE(4)
  }
#undef TB_CASE
  return (int)hipErrorInvalidValue;
}
