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

#include "tb3d_mr.h"

namespace tb3d {
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
}  // namespace tb3d

namespace {

using namespace tb3d;

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
  // A pass of several rounds balances better over the CUs with shorter
  // chunks than the uniform-workgroup model predicts (measured T=5: 1024^3
  // 297k vs 288k Mcells/s at 256 vs 512 planes, 2048x1024x1024 293k vs 263k
  // at 256 vs 1024; round 5: 1024^3 305.9k / 305.3k at 171 planes vs 302.4k /
  // 302.4k at 256, profiles/validation_r5.md); a one-round pass keeps its long
  // chunks (512^3: 247k at 512 planes vs 236k at 256).  FDTD3D_TB_XCAP: cap.
  static int cap = -1;
  if (cap < 0) {
    const char* e = getenv("FDTD3D_TB_XCAP");
    cap = (e && atoi(e) > 0) ? atoi(e) : 192;
  }
  if (rounds >= 2 && best > cap) return search(cap, &rounds);
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

const int kNoBox[6] = {0, 0, 0, 0, 0, 0};
// amplitude-mode tile shape (tuning): 0 = 16 waves x 2 rows, 2 = 8 waves x 2 rows
static int tb_amp_shape() {
  static const int v = [] {
    const char* e = getenv("FDTD3D_TB_AMP_SHAPE");
    return e ? atoi(e) : 0;
  }();
  return v;
}
int g_tb_mr_shape = 0;  // plain multi-row kernel: 0 = 16 waves x 2 rows, 1 = 8 waves x 4 rows, 2 = 8 x 2
int g_tb_dr_shape = 0;  // Drude variant: 0 = 8 waves x 2 rows, 1 = 16 waves x 1 row (both 16-row tiles)



template <int T>
int launch_tb_mr_sel(int fx, const float* const* ein, const float* const* hin, float* const* eout,
                     float* const* hout, const float4* ce4, const float4* ch4, const Box3& BE, const Box3& BH,
                     float cb, float db, int nx, int ny, int nz, const Box3* b, const Box3& O, int xchunk,
                     const int* src, const TbSrc& sv, const TfDev* tf, const float* gtab, const AmpDev& amp,
                     hipStream_t s, const DrDev& dr = DrDev{}) {
#define MR_ARGS ein, hin, eout, hout, ce4, ch4, BE, BH, cb, db, nx, ny, nz, b, O, xchunk, src, sv, tf, gtab, amp, s, dr
  // amplitude mode: uniform media, T <= 3 (tb3d_mr.h AmpDev)
  // Drude box (tb3d_mr.h DrDev): 8 waves x 2 rows (16-row tiles, <= 256
  // VGPRs: the dispersive state of T - 1 levels rides in registers)
  if (fx == 16) {
    if constexpr (T <= 5) {
      if (g_tb_dr_shape == 1) return launch_tb_mr<T, 1, 1, 16, 16>(MR_ARGS);
      return launch_tb_mr<T, 1, 2, 16, 8>(MR_ARGS);
    }
    return (int)hipErrorInvalidValue;
  }
  if (fx == 8) {
    if constexpr (T <= 3) {
      // 16 waves x 2 rows; the 8 x 4 shape (tuning knob 1) needs 200-256 VGPRs;
      // 8 waves x 2 rows (FDTD3D_TB_AMP_SHAPE=2: 16-row tiles, up to 256
      // VGPRs -- the 16 x 2 form caps at 128 and spills)
      if (g_tb_mr_shape == 1) return launch_tb_mr<T, 1, 4, 8, 8>(MR_ARGS);
      if (tb_amp_shape() == 2) return launch_tb_mr<T, 1, 2, 8, 8>(MR_ARGS);
      return launch_tb_mr<T, 1, 2, 8>(MR_ARGS);
    }
    return (int)hipErrorInvalidValue;
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
  // 8 waves x 2 rows (16-row tiles, two workgroups per CU): thin y boxes, the
  // y shells of decomposed passes
  if constexpr (T <= 5)
    if (g_tb_mr_shape == 2) return launch_tb_mr<T, 1, 2, 0, 8>(MR_ARGS);
  return launch_tb_mr<T, 1, 2, 0>(MR_ARGS);
#undef MR_ARGS
}

// automatic x chunk of a multi-row pass over output box O
int tb_mr_xchunk(int fx, const Box3& O, int steps) {
  const long long gz = cdiv(O.hi[2] - O.lo[2], 64 - 2 * steps);
  // (the Drude variant's tiles are 8 waves x 2 rows)
  const bool amp16 = fx == 8 && g_tb_mr_shape != 1 && tb_amp_shape() == 2;
  const bool rows16 = fx == 16 || amp16 || (fx == 0 && g_tb_mr_shape == 2 && steps <= 5);
  const long long gy = cdiv(O.hi[1] - O.lo[1], (rows16 ? 16 : TBW * 2) - 2 * steps);
  // the 8-wave shapes fit two workgroups per CU
  return pick_xchunk(gz * gy, O.hi[0] - O.lo[0], steps, ((fx == 0 && g_tb_mr_shape >= 1) || amp16) ? 2 : 1);
}

// multi-row pass (scalar lanes, 2 rows per wave): uniform media, sparse
// per-cell coefficients (fx bits 1 / 2), TF/SF corrections (fx bit 4)
int tb_mr_dispatch(int fx, const float* const* ein, const float* const* hin, float* const* eout,
                   float* const* hout, const float4* ce4, const float4* ch4, const Box3& BE, const Box3& BH,
                   float cb, float db, int nx, int ny, int nz, const Box3* b, const Box3& O, int xchunk, int steps,
                   const int* src, const TbSrc& sv, const TfDev* tf, const float* gtab, const AmpDev& amp,
                   hipStream_t s, const DrDev& dr = DrDev{}) {
  if (xchunk <= 0 && (fx & 4)) {
    // tuning: x chunk of the TF/SF variant's passes (FDTD3D_TF_XCHUNK, 0 automatic)
    static const int tfx = [] {
      const char* e = getenv("FDTD3D_TF_XCHUNK");
      return e ? atoi(e) : 0;
    }();
    if (tfx > 0) xchunk = tfx;
  }
  if (xchunk <= 0) xchunk = tb_mr_xchunk(fx, O, steps);
#define MR_ARGS fx, ein, hin, eout, hout, ce4, ch4, BE, BH, cb, db, nx, ny, nz, b, O, xchunk, src, sv, tf, gtab, amp, s, dr
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
//
// With ``esrc`` / ``hsrc`` set, the line is first copied from them into
// ``einc`` / ``hinc`` (scratch lines): the g tables of a pass whose real line
// is advanced elsewhere -- the hybrid's stepped shell steps it once per step
// while the blocked core applies the same pass's corrections in-kernel.
// (one template for the fp32 and fp64 blocked kernels' tables)
template <typename R>
struct LineSrc {
  R v[8];
};
template <typename R>
__global__ __launch_bounds__(1024) void k_tfsf_pass(R* __restrict__ einc, R* __restrict__ hinc, int n, R ce, R ch,
                                                    LineSrc<R> sv, int T, int reach, int nE, int nH,
                                                    const int* __restrict__ I0, const R* __restrict__ W0,
                                                    const R* __restrict__ W1, const R* __restrict__ C,
                                                    R* __restrict__ gtab, const R* __restrict__ esrc,
                                                    const R* __restrict__ hsrc) {
  const int tid = threadIdx.x;
  const int ld = nE + nH;
  const int m = min(n, reach);
  if (esrc) {
    // every cell a level reads: the moving part plus the interpolation's
    // upper neighbour of the farthest target (I0 + 1 < reach + 1)
    for (int i = tid; i < min(n, reach + 1); i += blockDim.x) {
      einc[i] = esrc[i];
      hinc[i] = hsrc[i];
    }
    __syncthreads();
  }
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
// Drude variant tile shape (tuning): 0 = 8 waves x 2 rows, 1 = 16 waves x 1 row
FDTD_API void fdtd_set_tb_dr_shape(int v) { g_tb_dr_shape = v == 1 ? 1 : 0; }
// plain multi-row tile shape (tuning): 0 = 16 waves x 2 rows, 1 = 8 waves x 4 rows
FDTD_API void fdtd_set_tb_mr_shape(int v) { g_tb_mr_shape = (v == 1 || v == 2) ? v : 0; }
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
                          steps, src, sv, nullptr, nullptr, AmpDev{}, s);
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

// Cost experiments of the in-kernel TF/SF (FDTD3D_TF_EXP, profiles/tfsf_cost_r5.md):
// 1 = no sets (the variant's structure alone), 2 = x-face sets only, 3 = y / z-face
// sets only.  The physics is then wrong; timing runs only.
static const void* tfsf_experiment(const void* tf, hipStream_t s) {
  static int mode = -1;
  static TfDev* scratch = nullptr;
  static const void* last = nullptr;  // the filtered copy is made once per set table (no sync per pass)
  if (mode < 0) {
    const char* e = getenv("FDTD3D_TF_EXP");
    mode = e ? atoi(e) : 0;
  }
  if (mode <= 0) return tf;
  if (tf == last && scratch) return scratch;
  last = tf;
  TfDev h;
  if (hipMemcpyAsync(&h, tf, sizeof(TfDev), hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return tf;
  TfDev o = h;
  o.nsets = 0;
  for (int i = 0; i < h.nsets; ++i) {
    const bool xf = h.s[i].fa == 0;
    if (mode == 1 || (mode == 2 && !xf) || (mode == 3 && xf)) continue;
    o.s[o.nsets++] = h.s[i];
  }
  if (mode != 2) o.xpl[0][0] = o.xpl[0][1] = o.xpl[1][0] = o.xpl[1][1] = -1;
  if (!scratch && hipMalloc(&scratch, sizeof(TfDev)) != hipSuccess) return tf;
  if (hipMemcpyAsync(scratch, &o, sizeof(TfDev), hipMemcpyHostToDevice, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return tf;
  return scratch;
}

// T fused leapfrog steps on the multi-row kernel with its extensions:
// sparse per-cell coefficients -- ``ce4`` / ``ch4`` hold the E / H
// coefficients of the three components as one float4 per cell of the box
// ``ebox`` / ``hbox`` (x-major, z fastest, .w unused); every cell outside its
// kind's box, and either kind whose array is null, uses the scalar ``cb`` /
// ``db`` -- and TF/SF corrections (``tf`` = device TfDev, ``gtab`` = the g
// table of this pass's first level, from fdtd_tfsf_pass_f32; null: none).
// Other arguments as fdtd_tb3d_v4_f32.
FDTD_API int fdtd_tb3d_ext_f32(const float* const* ein, const float* const* hin, float* const* eout,
                               float* const* hout, const void* ce4, const int* ebox, const void* ch4,
                               const int* hbox, double cb, double db, int nx, int ny, int nz, const int* boxes,
                               const int* obox, int xchunk, int steps, const int* src, const double* src_vals,
                               const void* tf, const float* gtab, void* stream) {
  if (nz % 4 != 0 || steps < 1 || steps > 6) return (int)hipErrorInvalidValue;
  Box3 b[6];
  for (int n = 0; n < 6; ++n) b[n] = make_box(boxes + 6 * n);
  const Box3 O = make_box(obox);
  if (box_empty(O)) return 0;
  const Box3 BE = make_box(ce4 ? ebox : kNoBox), BH = make_box(ch4 ? hbox : kNoBox);
  TbSrc sv;
  for (int l = 0; l < 8; ++l) sv.v[l] = (src[3] >= 0 && l < steps) ? (float)src_vals[l] : 0.f;
  const int fx = (ce4 && !box_empty(BE) ? 1 : 0) | (ch4 && !box_empty(BH) ? 2 : 0) | (tf && gtab ? 4 : 0);
  if (tf && gtab) tf = tfsf_experiment(tf, (hipStream_t)stream);
  return tb_mr_dispatch(fx, ein, hin, eout, hout, (const float4*)(box_empty(BE) ? nullptr : ce4),
                        (const float4*)(box_empty(BH) ? nullptr : ch4), BE, BH, (float)cb, (float)db, nx, ny, nz, b,
                        O, xchunk, steps, src, sv, (const TfDev*)tf, gtab, AmpDev{}, (hipStream_t)stream);
}

// T <= 3 fused leapfrog steps with the amplitude (steady-state) update of
// every level folded in (tb3d_mr.h AmpDev; uniform media, scalar
// coefficients): ``amp`` = the six running-maximum arrays (field shape, the
// planes of one [x][6][y][z] buffer: x stride 6 ny nz),
// ``aboxes`` = their six amplitude boxes, ``counts`` = T uint32 counters that
// receive the changed cells of each level (added to), ``accuracy`` the
// relative growth that counts.  ``src`` = {i, j, k0, comp, k1}: a hard E
// source on the z line k0 .. k1 - 1 (comp -1: none).  Other arguments as
// fdtd_tb3d_v4_f32.
FDTD_API int fdtd_tb3d_amp_f32(const float* const* ein, const float* const* hin, float* const* eout,
                               float* const* hout, double cb, double db, int nx, int ny, int nz, const int* boxes,
                               const int* obox, int xchunk, int steps, const int* src, const double* src_vals,
                               float* const* amp, const int* aboxes, double accuracy, unsigned* counts,
                               void* stream) {
  if (nz % 4 != 0 || steps < 1 || steps > 3 || !counts) return (int)hipErrorInvalidValue;
  Box3 b[6];
  for (int n = 0; n < 6; ++n) b[n] = make_box(boxes + 6 * n);
  const Box3 O = make_box(obox);
  if (box_empty(O)) return 0;
  TbSrc sv;
  for (int l = 0; l < 8; ++l) sv.v[l] = (src[3] >= 0 && l < steps) ? (float)src_vals[l] : 0.f;
  // the six arrays are the component planes of one [x][6][y][z] buffer
  const long long plane = (long long)ny * nz;
  // (the component offset rides in the instruction's SGPR offset: keep it
  // far below the 0xF0000000 "no access" lane offset)
  if (6 * plane * 4 >= (1ll << 28)) return (int)hipErrorInvalidValue;
  AmpDev A;
  A.a = amp[0];
  for (int c = 0; c < 6; ++c) {
    if (!amp[c] || amp[c] != amp[0] + c * plane) return (int)hipErrorInvalidValue;
    A.b[c] = make_box(aboxes + 6 * c);
    if (A.b[c].lo[0] < 0 || A.b[c].hi[0] >= 65536) return (int)hipErrorInvalidValue;
    A.xr[c] = A.b[c].lo[0] | (A.b[c].hi[0] << 16);
  }
  A.counts = counts;
  A.acc = (float)accuracy;
  A.k1 = src[4];
  const Box3 nb = make_box(kNoBox);
  return tb_mr_dispatch(8, ein, hin, eout, hout, nullptr, nullptr, nb, nb, (float)cb, (float)db, nx, ny, nz, b, O,
                        xchunk, steps, src, sv, nullptr, nullptr, A, (hipStream_t)stream);
}

// T <= 5 fused leapfrog steps over the output box with the Drude box B
// folded in (tb3d_mr.h DrDev; uniform media outside B, scalar coefficients):
// ``bbox`` = B (local lo[3], hi[3]), ``sin`` / ``sout`` = the two float4
// state arrays (delta + ids, Ep) over B before / after the pass (distinct),
// ``lut`` = 3 x ``nid`` float4 (b0 cbd, b2, m1, m2), ``cbd`` the D update
// coefficient.  B must lie inside the three E update boxes.  Other arguments
// as fdtd_tb3d_v4_f32.
FDTD_API int fdtd_tb3d_drude_f32(const float* const* ein, const float* const* hin, float* const* eout,
                                 float* const* hout, double cb, double db, int nx, int ny, int nz, const int* boxes,
                                 const int* obox, int xchunk, int steps, const int* src, const double* src_vals,
                                 const int* bbox, void* const* sin, void* const* sout, const void* lut, int nid,
                                 double cbd, void* stream) {
  if (nz % 4 != 0 || steps < 1 || steps > 5 || !sin || !sout || !lut || nid < 1 || nid > DR_MAX_IDS)
    return (int)hipErrorInvalidValue;
  Box3 b[6];
  for (int n = 0; n < 6; ++n) b[n] = make_box(boxes + 6 * n);
  const Box3 O = make_box(obox);
  if (box_empty(O)) return 0;
  DrDev D;
  D.B = make_box(bbox);
  if (box_empty(D.B)) return (int)hipErrorInvalidValue;
  for (int d = 0; d < 3; ++d) {
    if (D.B.lo[d] < 0 || D.B.hi[d] > (d == 0 ? nx : d == 1 ? ny : nz)) return (int)hipErrorInvalidValue;
    for (int n = 0; n < 3; ++n)
      if (D.B.lo[d] < b[n].lo[d] || D.B.hi[d] > b[n].hi[d]) return (int)hipErrorInvalidValue;
  }
  // one x plane of a state array is addressed by a 32-bit byte offset
  if ((long long)(D.B.hi[1] - D.B.lo[1]) * (D.B.hi[2] - D.B.lo[2]) * 16 >= (1ll << 31)) return (int)hipErrorInvalidValue;
  if (!sin[0] || !sin[1] || !sout[0] || !sout[1] || sin[0] == sout[0] || sin[1] == sout[1])
    return (int)hipErrorInvalidValue;
  D.sin0 = (const float4*)sin[0];
  D.sin1 = (const float4*)sin[1];
  D.sout0 = (float4*)sout[0];
  D.sout1 = (float4*)sout[1];
  D.lut = (const float4*)lut;
  D.nid = nid;
  D.cbd = (float)cbd;
  TbSrc sv;
  for (int l = 0; l < 8; ++l) sv.v[l] = (src[3] >= 0 && l < steps) ? (float)src_vals[l] : 0.f;
  const Box3 nb = make_box(kNoBox);
  return tb_mr_dispatch(16, ein, hin, eout, hout, nullptr, nullptr, nb, nb, (float)cb, (float)db, nx, ny, nz, b, O,
                        xchunk, steps, src, sv, nullptr, nullptr, AmpDev{}, (hipStream_t)stream, D);
}

// size of the TfDev block the host fills (ABI check)
FDTD_API int fdtd_tfdev_size() { return (int)sizeof(TfDev); }

// incident line advanced ``steps`` steps from step t (source value per step
// in ``src_vals``) and the per-level g tables of the pass (k_tfsf_pass)
namespace {
template <typename R>
int tfsf_pass(const R* esrc, const R* hsrc, R* einc, R* hinc, int n, double ce, double ch, const double* src_vals,
              int steps, int reach, int nE, int nH, const int* I0, const R* W0, const R* W1, const R* C, R* gtab,
              void* stream) {
  if (steps < 1 || steps > 8) return (int)hipErrorInvalidValue;
  if ((esrc || hsrc) && (!esrc || !hsrc || esrc == einc || hsrc == hinc)) return (int)hipErrorInvalidValue;
  LineSrc<R> sv;
  for (int l = 0; l < 8; ++l) sv.v[l] = l < steps ? (R)src_vals[l] : (R)0;
  k_tfsf_pass<R><<<1, 1024, 0, (hipStream_t)stream>>>(einc, hinc, n, (R)ce, (R)ch, sv, steps, reach, nE, nH, I0, W0,
                                                      W1, C, gtab, esrc, hsrc);
  FDTD_RETURN_LAUNCH_STATUS();
}
}  // namespace

FDTD_API int fdtd_tfsf_pass_f32(float* einc, float* hinc, int n, double ce, double ch, const double* src_vals,
                                int steps, int reach, int nE, int nH, const int* I0, const float* W0,
                                const float* W1, const float* C, float* gtab, void* stream) {
  return tfsf_pass<float>(nullptr, nullptr, einc, hinc, n, ce, ch, src_vals, steps, reach, nE, nH, I0, W0, W1, C,
                          gtab, stream);
}
FDTD_API int fdtd_tfsf_pass_f64(double* einc, double* hinc, int n, double ce, double ch, const double* src_vals,
                                int steps, int reach, int nE, int nH, const int* I0, const double* W0,
                                const double* W1, const double* C, double* gtab, void* stream) {
  return tfsf_pass<double>(nullptr, nullptr, einc, hinc, n, ce, ch, src_vals, steps, reach, nE, nH, I0, W0, W1, C,
                           gtab, stream);
}

// the g tables of a pass WITHOUT advancing the line: the line ``esrc`` /
// ``hsrc`` is copied into the scratch lines ``einc`` / ``hinc`` (length n
// each) and advanced there (hybrid passes, whose shell steps the real line)
FDTD_API int fdtd_tfsf_table_f32(const float* esrc, const float* hsrc, float* einc, float* hinc, int n, double ce,
                                 double ch, const double* src_vals, int steps, int reach, int nE, int nH,
                                 const int* I0, const float* W0, const float* W1, const float* C, float* gtab,
                                 void* stream) {
  if (!esrc || !hsrc) return (int)hipErrorInvalidValue;
  return tfsf_pass<float>(esrc, hsrc, einc, hinc, n, ce, ch, src_vals, steps, reach, nE, nH, I0, W0, W1, C, gtab,
                          stream);
}
FDTD_API int fdtd_tfsf_table_f64(const double* esrc, const double* hsrc, double* einc, double* hinc, int n,
                                 double ce, double ch, const double* src_vals, int steps, int reach, int nE, int nH,
                                 const int* I0, const double* W0, const double* W1, const double* C, double* gtab,
                                 void* stream) {
  if (!esrc || !hsrc) return (int)hipErrorInvalidValue;
  return tfsf_pass<double>(esrc, hsrc, einc, hinc, n, ce, ch, src_vals, steps, reach, nE, nH, I0, W0, W1, C, gtab,
                           stream);
}
