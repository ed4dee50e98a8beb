// Fused UPML / Drude chain for the PML slabs and dispersive regions.
//
// The reference updates every cell of every component through three sweeps
// (D from curl, Drude D1 from three D levels, E from D/D1: Scheme3D.cpp:266-416
// and 1158-1306 for H), each with per-cell virtual material lookups.  Outside
// the absorbing layers and the dispersive material the chain collapses
// algebraically to the plain Yee update (sigma = 0, omega = 0), so the scheme
// runs the plain float4 kernels there and this kernel only on the chain
// regions: one launch per region updates all three components of a kind, each
// cell going through D -> [D1] -> E in registers (one read of every operand,
// one write of every result).
//
// Per component (kind E; H is the mirror with forward differences), with the
// UPML coefficients in their factored form (profiles along the component's
// axes aD / aCa / aCb, models/scheme.py _init_upml):
//   curl = sg0 (s0[x] - s0[x - e_a0]) + sg1 (s1[x] - s1[x - e_a1])
//   Dn   = caD[nD] D + cbD[nD] curl
//   DRUDE: D1n = b0 Dn + b1 D + b2 Dp + ma1 D1 + ma2 D1p ; (new, old) = (D1n, D1)
//   else:                                                 (new, old) = (Dn, D)
//   E    = caE[nA] E + s cell ica[nA] (cbEa[nB] new + ccEa[nB] old)
// Every operand is loaded before the first store, so one cell keeps ~20 loads
// in flight (the generic Coef form, with a null check per factor, made the
// compiler wait on each load).

#include "common.h"
#include "vec4.h"

namespace {

template <typename T>
struct ChainComp {
  T* E;
  T* Dn;
  const T* D;
  const T* Dp;
  T* D1n;
  const T* D1;
  const T* D1p;
  const T* s0;
  const T* s1;
  const T* caD;
  const T* cbD;
  const T* caE;
  const T* ica;
  const T* cbEa;
  const T* ccEa;
  const T* cell;  // per-cell 1/(eps eps0) or nullptr
  const T* b0;
  const T* b1;
  const T* b2;
  const T* ma1;
  const T* ma2;
  const unsigned char* id;  // Drude material index per cell (null: the five per-cell arrays)
  const T* lut;             // id -> (b0, b1, b2, ma1, ma2)
  const T* pcell;           // plain part: per-cell (scaled) update coefficient, or null
  T s;
  T pcb;                    // plain part: scalar update coefficient
  int a0, a1, sg0, sg1, aD, aA, aB;
  Box3 box;
  Box3 pbox;                // plain Yee cells folded into this launch (empty: none)
  Box3 dbox;                // storage box of the D / D1 levels (empty: full-grid arrays)
};

// index of cell n in the D / D1 levels: region-local storage over the
// component's chain box (models/regions.py) or the full-grid offset
template <typename T>
__device__ __forceinline__ size_t aux_off(const ChainComp<T>& q, const int* n, size_t off) {
  if (q.dbox.hi[0] <= q.dbox.lo[0]) return off;
  return ((size_t)(n[0] - q.dbox.lo[0]) * (q.dbox.hi[1] - q.dbox.lo[1]) + (n[1] - q.dbox.lo[1])) *
             (q.dbox.hi[2] - q.dbox.lo[2]) +
         (n[2] - q.dbox.lo[2]);
}

// One component of one cell in one go (the dispersive form: see the kernel).
template <typename T, bool DRUDE, bool CELL>
__device__ __forceinline__ void chain_cell(const ChainComp<T>& q, bool kind_e, const long long* stride,
                                           const int* n, size_t off) {
  const long long s0 = stride[q.a0], s1 = stride[q.a1];
  if (!in_box(q.box, n[0], n[1], n[2])) {
    // plain Yee cells of a thin box folded into the launch (the rows a z PML
    // slab shares with the shell window next to it: one pass over whole
    // 128-byte row segments instead of two partial ones).  Same expression
    // as the float4 plain kernels: F + c * (d0 - d1).
    if (!in_box(q.pbox, n[0], n[1], n[2])) return;
    const T x0 = q.s0[off], x1 = q.s1[off];
    const T y0 = kind_e ? q.s0[off - s0] : q.s0[off + s0];
    const T y1 = kind_e ? q.s1[off - s1] : q.s1[off + s1];
    const T c = q.pcell ? q.pcell[off] : q.pcb;
    const T d0 = kind_e ? (x0 - y0) : (y0 - x0);
    const T d1 = kind_e ? (x1 - y1) : (y1 - x1);
    const T curl = (q.sg0 > 0 ? d0 : -d0) + (q.sg1 > 0 ? d1 : -d1);
    q.E[off] = q.E[off] + c * curl;
    return;
  }
  // ---- every load first
  const size_t da = aux_off(q, n, off);
  const T x0 = q.s0[off], x1 = q.s1[off];
  const T y0 = kind_e ? q.s0[off - s0] : q.s0[off + s0];
  const T y1 = kind_e ? q.s1[off - s1] : q.s1[off + s1];
  const T D = q.D[da];
  const T E = q.E[off];
  const T caD = q.caD[n[q.aD]], cbD = q.cbD[n[q.aD]];
  const T caE = q.caE[n[q.aA]], ica = q.ica[n[q.aA]];
  const T cbEa = q.cbEa[n[q.aB]], ccEa = q.ccEa[n[q.aB]];
  const T cell = CELL ? q.cell[off] : T(1);
  T Dp = 0, D1 = 0, D1p = 0, b0 = 0, b1 = 0, b2 = 0, m1 = 0, m2 = 0;
  if (DRUDE) {
    Dp = q.Dp[da];
    D1 = q.D1[da];
    D1p = q.D1p[da];
    if (q.id) {
      // material-ID + LUT: one byte per cell instead of 20 (a Drude scene
      // holds a handful of distinct coefficient tuples: vacuum, the
      // material and the averaged boundary cells)
      const T* e = q.lut + 5 * (int)q.id[off];
      b0 = e[0];
      b1 = e[1];
      b2 = e[2];
      m1 = e[3];
      m2 = e[4];
    } else {
      b0 = q.b0[off];
      b1 = q.b1[off];
      b2 = q.b2[off];
      m1 = q.ma1[off];
      m2 = q.ma2[off];
    }
  }
  // ---- compute
  const T d0 = kind_e ? (x0 - y0) : (y0 - x0);
  const T d1 = kind_e ? (x1 - y1) : (y1 - x1);
  const T curl = (q.sg0 > 0 ? d0 : -d0) + (q.sg1 > 0 ? d1 : -d1);
  const T Dn = caD * D + cbD * curl;
  T nw = Dn, old = D;
  if (DRUDE) {
    nw = b0 * Dn + b1 * D + b2 * Dp + m1 * D1 + m2 * D1p;
    old = D1;
  }
  const T En = caE * E + q.s * cell * ica * (cbEa * nw + ccEa * old);
  // ---- stores
  q.Dn[da] = Dn;
  if (DRUDE) q.D1n[da] = nw;
  q.E[off] = En;
}

// One cell of one component, split in two phases so the kernel issues the
// loads of all three components before the first store (stores through the
// component structs could alias later loads, which otherwise serialises the
// three memory round trips per cell).
// element a of a 3-vector held in registers (a runtime index into a local
// array would put the array in scratch)
template <typename V>
__device__ __forceinline__ V pick3(int a, V x, V y, V z) {
  return a == 0 ? x : (a == 1 ? y : z);
}

template <typename T>
struct ChainIn {
  int mode;  // 0 skip, 1 chain, 2 plain (folded box)
  size_t da; // index into the D / D1 levels
  T x0, x1, y0, y1, D, E, caD, cbD, caE, ica, cbEa, ccEa, cell, Dp, D1, D1p, b0, b1, b2, m1, m2;
};

template <typename T, bool DRUDE, bool CELL>
__device__ __forceinline__ ChainIn<T> chain_load(const ChainComp<T>& q, bool kind_e, const long long* stride,
                                                 const int* n, size_t off) {
  ChainIn<T> v;
  v.mode = in_box(q.box, n[0], n[1], n[2]) ? 1 : (in_box(q.pbox, n[0], n[1], n[2]) ? 2 : 0);
  if (v.mode == 0) return v;
  const long long s0 = pick3(q.a0, stride[0], stride[1], stride[2]);
  const long long s1 = pick3(q.a1, stride[0], stride[1], stride[2]);
  v.x0 = q.s0[off];
  v.x1 = q.s1[off];
  v.y0 = kind_e ? q.s0[off - s0] : q.s0[off + s0];
  v.y1 = kind_e ? q.s1[off - s1] : q.s1[off + s1];
  v.E = q.E[off];
  if (v.mode == 2) {
    // plain Yee cells of a thin box folded into the launch (the rows a z PML
    // slab shares with the shell window next to it: one pass over whole
    // 128-byte row segments instead of two partial ones)
    v.cell = q.pcell ? q.pcell[off] : q.pcb;
    return v;
  }
  v.da = aux_off(q, n, off);
  v.D = q.D[v.da];
  const int nD = pick3(q.aD, n[0], n[1], n[2]), nA = pick3(q.aA, n[0], n[1], n[2]);
  const int nB = pick3(q.aB, n[0], n[1], n[2]);
  v.caD = q.caD[nD];
  v.cbD = q.cbD[nD];
  v.caE = q.caE[nA];
  v.ica = q.ica[nA];
  v.cbEa = q.cbEa[nB];
  v.ccEa = q.ccEa[nB];
  v.cell = CELL ? q.cell[off] : T(1);
  if (DRUDE) {
    v.Dp = q.Dp[v.da];
    v.D1 = q.D1[v.da];
    v.D1p = q.D1p[v.da];
    if (q.id) {
      // material-ID + LUT: one byte per cell instead of 20 (a Drude scene
      // holds a handful of distinct coefficient tuples: vacuum, the
      // material and the averaged boundary cells)
      const T* e = q.lut + 5 * (int)q.id[off];
      v.b0 = e[0];
      v.b1 = e[1];
      v.b2 = e[2];
      v.m1 = e[3];
      v.m2 = e[4];
    } else {
      v.b0 = q.b0[off];
      v.b1 = q.b1[off];
      v.b2 = q.b2[off];
      v.m1 = q.ma1[off];
      v.m2 = q.ma2[off];
    }
  }
  return v;
}

template <typename T, bool DRUDE>
__device__ __forceinline__ void chain_finish(const ChainComp<T>& q, bool kind_e, const ChainIn<T>& v, size_t off) {
  if (v.mode == 0) return;
  const T d0 = kind_e ? (v.x0 - v.y0) : (v.y0 - v.x0);
  const T d1 = kind_e ? (v.x1 - v.y1) : (v.y1 - v.x1);
  const T curl = (q.sg0 > 0 ? d0 : -d0) + (q.sg1 > 0 ? d1 : -d1);
  if (v.mode == 2) {
    q.E[off] = v.E + v.cell * curl;  // the float4 plain kernels' F + c * (d0 - d1)
    return;
  }
  const T Dn = v.caD * v.D + v.cbD * curl;
  T nw = Dn, old = v.D;
  if (DRUDE) {
    nw = v.b0 * Dn + v.b1 * v.D + v.b2 * v.Dp + v.m1 * v.D1 + v.m2 * v.D1p;
    old = v.D1;
  }
  const T En = v.caE * v.E + q.s * v.cell * v.ica * (v.cbEa * nw + v.ccEa * old);
  q.Dn[v.da] = Dn;
  if (DRUDE) q.D1n[v.da] = nw;
  q.E[off] = En;
}

// Thread mapping: the (y, z) cells of the launch box are flattened (z
// fastest), so narrow boxes (a 10-cell z slab) still fill every lane and wide
// rows stay coalesced; each thread walks chain_chx() planes along x (default
// CHX; FDTD3D_CHAIN_CHX overrides it, read once per library).
constexpr int CHX = 8;
static inline int chain_chx() {
  static const int v = [] {
    const char* e = getenv("FDTD3D_CHAIN_CHX");
    return e && atoi(e) > 0 ? atoi(e) : CHX;
  }();
  return v;
}

// Plain Yee update of one component of one cell (mode 2 of chain_finish):
// the cells of a dispersive box outside the material's per-row z range.
template <typename T>
__device__ __forceinline__ ChainIn<T> plain_load(const ChainComp<T>& q, bool kind_e, const long long* stride,
                                                 const int* n, size_t off) {
  ChainIn<T> v;
  v.mode = in_box(q.box, n[0], n[1], n[2]) ? 2 : 0;
  if (v.mode == 0) return v;
  const long long s0 = pick3(q.a0, stride[0], stride[1], stride[2]);
  const long long s1 = pick3(q.a1, stride[0], stride[1], stride[2]);
  v.x0 = q.s0[off];
  v.x1 = q.s1[off];
  v.y0 = kind_e ? q.s0[off - s0] : q.s0[off + s0];
  v.y1 = kind_e ? q.s1[off - s1] : q.s1[off + s1];
  v.E = q.E[off];
  v.cell = q.pcell ? q.pcell[off] : q.pcb;
  return v;
}

// Per-row z range of the dispersive cells of a box (local indices): rows
// (x, y) of [lo0, lo0 + nx) x [lo1, lo1 + ny) hold int2 (z0, z1); cells of the
// launch outside their row's range run the plain update.  The split is a
// static property of the cell (the same in every window set), so a cell's D /
// D1 history is either always advanced or never read.
struct RowRanges {
  const int2* r;
  int lo0, lo1, nx, ny;
};

__device__ __forceinline__ int2 row_range(const RowRanges& rr, int x, int y) {
  const int tx = x - rr.lo0, ty = y - rr.lo1;
  if (tx < 0 || ty < 0 || tx >= rr.nx || ty >= rr.ny) return make_int2(0, 0);
  return rr.r[(size_t)tx * rr.ny + ty];
}

template <typename T, bool DRUDE, bool CELL>
__global__ __launch_bounds__(256) void k_chain3d(ChainComp<T> q0, ChainComp<T> q1, ChainComp<T> q2, int kind_e,
                                                 int ny, int nz, Box3 U, RowRanges rr, int chx) {
  const int W = U.hi[2] - U.lo[2];
  const int H = U.hi[1] - U.lo[1];
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)W * H) return;
  int n[3];
  n[1] = U.lo[1] + (int)(idx / W);
  n[2] = U.lo[2] + (int)(idx % W);
  const int i0 = U.lo[0] + (int)blockIdx.y * chx;
  const int i1 = min(i0 + chx, U.hi[0]);
  const long long stride[3] = {(long long)ny * nz, (long long)nz, 1};
  // dispersive launches with a row table: the next plane's range is loaded
  // one trip ahead, so the path decision never waits on its own load
  int2 nxt = make_int2(0, 0x7fffffff);
  if (DRUDE && rr.r && i0 < i1) nxt = row_range(rr, i0, n[1]);
#pragma unroll 1
  for (int i = i0; i < i1; ++i) {
    n[0] = i;
    const size_t off = ((size_t)i * ny + n[1]) * nz + n[2];
    if constexpr (DRUDE) {
      const int2 cur = nxt;
      if (rr.r && i + 1 < i1) nxt = row_range(rr, i + 1, n[1]);
      if (n[2] >= cur.x && n[2] < cur.y) {
        // the dispersive form holds twice the operands: one component at a
        // time (all three in flight spill: measured 47k vs 51k Mcells/s)
        chain_cell<T, DRUDE, CELL>(q0, kind_e != 0, stride, n, off);
        chain_cell<T, DRUDE, CELL>(q1, kind_e != 0, stride, n, off);
        chain_cell<T, DRUDE, CELL>(q2, kind_e != 0, stride, n, off);
      } else {
        const ChainIn<T> v0 = plain_load<T>(q0, kind_e != 0, stride, n, off);
        const ChainIn<T> v1 = plain_load<T>(q1, kind_e != 0, stride, n, off);
        const ChainIn<T> v2 = plain_load<T>(q2, kind_e != 0, stride, n, off);
        chain_finish<T, DRUDE>(q0, kind_e != 0, v0, off);
        chain_finish<T, DRUDE>(q1, kind_e != 0, v1, off);
        chain_finish<T, DRUDE>(q2, kind_e != 0, v2, off);
      }
    } else {
      // all three components' loads before the first store (UPML + TF/SF
      // 512^3: 69.6k vs 67.0k Mcells/s)
      const ChainIn<T> v0 = chain_load<T, DRUDE, CELL>(q0, kind_e != 0, stride, n, off);
      const ChainIn<T> v1 = chain_load<T, DRUDE, CELL>(q1, kind_e != 0, stride, n, off);
      const ChainIn<T> v2 = chain_load<T, DRUDE, CELL>(q2, kind_e != 0, stride, n, off);
      chain_finish<T, DRUDE>(q0, kind_e != 0, v0, off);
      chain_finish<T, DRUDE>(q1, kind_e != 0, v1, off);
      chain_finish<T, DRUDE>(q2, kind_e != 0, v2, off);
    }
  }
}

// Non-dispersive chain, one component per thread: blockIdx.z picks the
// component, whose struct is read through a uniform index into the kernel
// argument block (scalar loads of ONE component's pointers and boxes).  The
// three-components-per-thread kernel above keeps ~75 SGPRs of arguments per
// component live and spills 170-290 SGPRs into VGPR lanes (read back every
// plane); here a thread holds one component's operands, loads them all
// before its single store, and the arguments fit the SGPR file.
template <typename T>
struct ChainSet {
  ChainComp<T> q[3];
};

template <typename T, bool CELL>
__global__ __launch_bounds__(256) void k_chain3d_c(ChainSet<T> S, int kind_e, int ny, int nz, Box3 U, int chx) {
  const ChainComp<T>& q = S.q[blockIdx.z];
  const Box3 B = box_union(q.box, q.pbox);
  // the component's own boxes inside the launch's union box U
  const int W = U.hi[2] - U.lo[2];
  const int H = U.hi[1] - U.lo[1];
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)W * H) return;
  int n[3];
  n[1] = U.lo[1] + (int)(idx / W);
  n[2] = U.lo[2] + (int)(idx % W);
  if (n[1] < B.lo[1] || n[1] >= B.hi[1] || n[2] < B.lo[2] || n[2] >= B.hi[2]) return;
  const int i0 = max(U.lo[0] + (int)blockIdx.y * chx, B.lo[0]);
  const int i1 = min(min(U.lo[0] + ((int)blockIdx.y + 1) * chx, U.hi[0]), B.hi[0]);
  const long long stride[3] = {(long long)ny * nz, (long long)nz, 1};
#pragma unroll 1
  for (int i = i0; i < i1; ++i) {
    n[0] = i;
    const size_t off = ((size_t)i * ny + n[1]) * nz + n[2];
    const ChainIn<T> v = chain_load<T, false, CELL>(q, kind_e != 0, stride, n, off);
    chain_finish<T, false>(q, kind_e != 0, v, off);
  }
}

// ---------------------------------------------------------------------------
// float4 form of the non-dispersive chain (fp32, z rows of 4-cell groups):
// each thread owns 4 consecutive z cells of one (y, x-run), 16-byte loads and
// stores; per element the cell is a chain cell (its component's box), a
// folded plain cell (pbox) or skipped.  A z-derivative neighbour comes from
// the thread's own float4 plus one scalar load (guarded at the array ends).
__device__ __forceinline__ float4 bcast4(float v) { return make_float4(v, v, v, v); }

// a factored profile value along `axis` for the 4 cells (z: 4 values)
__device__ __forceinline__ float4 prof4(const float* p, int axis, int i, int j, int k) {
  if (axis == 2) return ld4(p, (size_t)k);
  return bcast4(p[axis == 0 ? i : j]);
}

__device__ __forceinline__ void chain_v4(const ChainComp<float>& q, bool kind_e, const long long* stride, int i, int j,
                                         int k, int nz, size_t off) {
  unsigned mc = kmask(q.box, j, k), mp = kmask(q.pbox, j, k);
  if (i < q.box.lo[0] || i >= q.box.hi[0]) mc = 0u;
  if (i < q.pbox.lo[0] || i >= q.pbox.hi[0]) mp = 0u;
  mp &= ~mc;
  if ((mc | mp) == 0u) return;
  const long long s0 = pick3(q.a0, stride[0], stride[1], stride[2]);
  const long long s1 = pick3(q.a1, stride[0], stride[1], stride[2]);
  const float4 x0 = ld4(q.s0, off), x1 = ld4(q.s1, off);
  float4 y0, y1;
  if (q.a0 != 2) {
    y0 = ld4(q.s0, kind_e ? off - s0 : off + s0);
  } else if (kind_e) {
    y0 = make_float4(k > 0 ? q.s0[off - 1] : 0.f, x0.x, x0.y, x0.z);
  } else {
    y0 = make_float4(x0.y, x0.z, x0.w, k + 4 < nz ? q.s0[off + 4] : 0.f);
  }
  if (q.a1 != 2) {
    y1 = ld4(q.s1, kind_e ? off - s1 : off + s1);
  } else if (kind_e) {
    y1 = make_float4(k > 0 ? q.s1[off - 1] : 0.f, x1.x, x1.y, x1.z);
  } else {
    y1 = make_float4(x1.y, x1.z, x1.w, k + 4 < nz ? q.s1[off + 4] : 0.f);
  }
  const float4 E = ld4(q.E, off);
  float4 D = bcast4(0.f), caD = D, cbD = D, caE = D, ica = D, cbEa = D, ccEa = D, cell = bcast4(1.f);
  if (mc) {
    D = ld4(q.D, off);
    caD = prof4(q.caD, q.aD, i, j, k);
    cbD = prof4(q.cbD, q.aD, i, j, k);
    caE = prof4(q.caE, q.aA, i, j, k);
    ica = prof4(q.ica, q.aA, i, j, k);
    cbEa = prof4(q.cbEa, q.aB, i, j, k);
    ccEa = prof4(q.ccEa, q.aB, i, j, k);
    if (q.cell) cell = ld4(q.cell, off);
  }
  const float4 pc = mp ? (q.pcell ? ld4(q.pcell, off) : bcast4(q.pcb)) : bcast4(0.f);
  float4 Dn = D, En = E;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float d0 = kind_e ? (f4(x0, e) - f4(y0, e)) : (f4(y0, e) - f4(x0, e));
    const float d1 = kind_e ? (f4(x1, e) - f4(y1, e)) : (f4(y1, e) - f4(x1, e));
    const float curl = (q.sg0 > 0 ? d0 : -d0) + (q.sg1 > 0 ? d1 : -d1);
    if (mc & (1u << e)) {
      const float dn = f4(caD, e) * f4(D, e) + f4(cbD, e) * curl;
      f4set(Dn, e, dn);
      f4set(En, e, f4(caE, e) * f4(E, e) +
                       q.s * f4(cell, e) * f4(ica, e) * (f4(cbEa, e) * dn + f4(ccEa, e) * f4(D, e)));
    } else if (mp & (1u << e)) {
      f4set(En, e, f4(E, e) + f4(pc, e) * curl);
    }
  }
  st4m(q.Dn, off, Dn, mc);
  st4m(q.E, off, En, mc | mp);
}

__global__ __launch_bounds__(256) void k_chain3d_v4(ChainComp<float> q0, ChainComp<float> q1, ChainComp<float> q2,
                                                    int kind_e, int ny, int nz, Box3 U) {
  const int W4 = (U.hi[2] - U.lo[2]) >> 2;
  const int H = U.hi[1] - U.lo[1];
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)W4 * H) return;
  const int j = U.lo[1] + (int)(idx / W4);
  const int k = U.lo[2] + 4 * (int)(idx % W4);
  const int i0 = U.lo[0] + (int)blockIdx.y * CHX;
  const int i1 = min(i0 + CHX, U.hi[0]);
  const long long stride[3] = {(long long)ny * nz, (long long)nz, 1};
#pragma unroll 1
  for (int i = i0; i < i1; ++i) {
    const size_t off = ((size_t)i * ny + j) * nz + k;
    chain_v4(q0, kind_e != 0, stride, i, j, k, nz, off);
    chain_v4(q1, kind_e != 0, stride, i, j, k, nz, off);
    chain_v4(q2, kind_e != 0, stride, i, j, k, nz, off);
  }
}

// off by default: measured slower than one cell per thread (512^3 UPML + TF/SF
// 58.1k vs 71.3k, Drude + UPML 46.2k vs 55.4k Mcells/s): A-B knob (fdtd_set_chain_v4)
static bool g_chain_v4 = false;

// non-dispersive chain launches: one component per thread (k_chain3d_c) or
// all three (k_chain3d); FDTD3D_CHAIN_SPLIT=0 / 1 overrides
static int g_chain_split = -1;
static bool chain_split() {
  if (g_chain_split < 0) {
    const char* e = getenv("FDTD3D_CHAIN_SPLIT");
    g_chain_split = (e && *e) ? (atoi(e) != 0) : 1;
  }
  return g_chain_split != 0;
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// every array the float4 chain touches 16-byte aligned (z rows of nz % 4 == 0)
template <typename T>
bool chain_v4_ok(const ChainComp<T>* q, int nz) {
  if (sizeof(T) != 4 || (nz & 3) != 0 || !g_chain_v4) return false;
  for (int c = 0; c < 3; ++c) {
    if (!box_empty(q[c].dbox)) return false;  // the float4 form indexes full-grid levels
    const void* ps[] = {q[c].E, q[c].Dn, q[c].D, q[c].s0, q[c].s1, q[c].caD, q[c].cbD, q[c].caE, q[c].ica,
                        q[c].cbEa, q[c].ccEa, q[c].cell, q[c].pcell};
    for (const void* p : ps)
      if (p && !al16(p)) return false;
  }
  return true;
}

constexpr int CP_PER = 24;  // pointers per component
constexpr int CI_PER = 25;  // ints per component

template <typename T>
ChainComp<T> make_comp(const void* const* P, double s, const int* I) {
  ChainComp<T> q;
  q.E = (T*)P[0];
  q.Dn = (T*)P[1];
  q.D = (const T*)P[2];
  q.Dp = (const T*)P[3];
  q.D1n = (T*)P[4];
  q.D1 = (const T*)P[5];
  q.D1p = (const T*)P[6];
  q.s0 = (const T*)P[7];
  q.s1 = (const T*)P[8];
  q.caD = (const T*)P[9];
  q.cbD = (const T*)P[10];
  q.caE = (const T*)P[11];
  q.ica = (const T*)P[12];
  q.cbEa = (const T*)P[13];
  q.ccEa = (const T*)P[14];
  q.cell = (const T*)P[15];
  q.b0 = (const T*)P[16];
  q.b1 = (const T*)P[17];
  q.b2 = (const T*)P[18];
  q.ma1 = (const T*)P[19];
  q.ma2 = (const T*)P[20];
  q.id = (const unsigned char*)P[21];
  q.lut = (const T*)P[22];
  q.pcell = (const T*)P[23];
  q.s = (T)s;
  q.a0 = I[0];
  q.a1 = I[1];
  q.sg0 = I[2];
  q.sg1 = I[3];
  q.aD = I[4];
  q.aA = I[5];
  q.aB = I[6];
  q.box = make_box(I + 7);
  q.pbox = make_box(I + 13);
  q.dbox = make_box(I + 19);
  return q;
}

template <typename T>
int launch_chain(const void* const* P, const double* S, const int* I, int drude, int kind_e, int ny, int nz,
                 RowRanges rr, hipStream_t s) {
  ChainComp<T> q[3];
  Box3 U = {{0, 0, 0}, {0, 0, 0}};
  bool cell = false;
  for (int c = 0; c < 3; ++c) {
    q[c] = make_comp<T>(P + CP_PER * c, S[2 * c], I + CI_PER * c);
    q[c].pcb = (T)S[2 * c + 1];
    if (!box_empty(q[c].box)) cell = cell || q[c].cell != nullptr;
    U = box_union(U, q[c].box);
    U = box_union(U, q[c].pbox);
  }
  if (box_empty(U)) return 0;
  for (int c = 0; c < 3; ++c) {
    if (!box_empty(q[c].box) && (q[c].cell != nullptr) != cell) return (int)hipErrorInvalidValue;
    // region-local levels: every chain cell inside the storage box
    if (!box_empty(q[c].box) && !box_empty(q[c].dbox))
      for (int d = 0; d < 3; ++d)
        if (q[c].box.lo[d] < q[c].dbox.lo[d] || q[c].box.hi[d] > q[c].dbox.hi[d]) return (int)hipErrorInvalidValue;
  }
  if constexpr (sizeof(T) == 4) {
    if (!drude && chain_v4_ok(q, nz)) {
      // 4-cell z groups: the union box widened to whole groups (per-element
      // box tests keep the cells outside every component's boxes untouched)
      Box3 U4 = U;
      U4.lo[2] &= ~3;
      U4.hi[2] = (U4.hi[2] + 3) & ~3;
      const long long groups = (long long)((U4.hi[2] - U4.lo[2]) >> 2) * (U4.hi[1] - U4.lo[1]);
      dim3 g4(cdiv(groups, 256), cdiv(U4.hi[0] - U4.lo[0], CHX));
      k_chain3d_v4<<<g4, 256, 0, s>>>(q[0], q[1], q[2], kind_e, ny, nz, U4);
      FDTD_RETURN_LAUNCH_STATUS();
    }
  }
  const long long cells = (long long)(U.hi[2] - U.lo[2]) * (U.hi[1] - U.lo[1]);
  const int chx = chain_chx();
  dim3 grid(cdiv(cells, 256), cdiv(U.hi[0] - U.lo[0], chx));
  if (!drude && chain_split()) {
    ChainSet<T> S;
    for (int c = 0; c < 3; ++c) S.q[c] = q[c];
    dim3 g3(grid.x, grid.y, 3);
    if (cell)
      k_chain3d_c<T, true><<<g3, 256, 0, s>>>(S, kind_e, ny, nz, U, chx);
    else
      k_chain3d_c<T, false><<<g3, 256, 0, s>>>(S, kind_e, ny, nz, U, chx);
    FDTD_RETURN_LAUNCH_STATUS();
  }
#define CH_LAUNCH(D, C) k_chain3d<T, D, C><<<grid, 256, 0, s>>>(q[0], q[1], q[2], kind_e, ny, nz, U, rr, chx)
  if (drude) {
    if (cell) CH_LAUNCH(true, true);
    else CH_LAUNCH(true, false);
  } else {
    if (cell) CH_LAUNCH(false, true);
    else CH_LAUNCH(false, false);
  }
#undef CH_LAUNCH
  FDTD_RETURN_LAUNCH_STATUS();
}

}  // namespace

// One chain launch for the three components of a kind.  Per component c:
// P[24c ..] = E Dn D Dp D1n D1 D1p s0 s1 caD cbD caE ica cbEa ccEa cell b0 b1 b2 ma1 ma2 id lut pcell
// (unused: nullptr; a non-null id replaces b0 .. ma2 by lut[5 id ..]), S[2c] = scalar of the
// E-from-D term, S[2c + 1] = plain-part coefficient, I[25c ..] = curl axes a0 a1, signs sg0
// sg1, UPML axes aD aCa aCb, chain box lo[3] hi[3], plain box lo[3] hi[3] (empty: skipped;
// the plain box holds cells updated F += c (curl) in the same launch), storage box of the D /
// D1 levels lo[3] hi[3] (empty: full-grid levels; else they hold that box only, x-major, z
// fastest, and the chain box must lie inside it).
FDTD_API int fdtd_chain3d_f32(const void* const* P, const double* S, const int* I, int drude, int kind_e, int ny,
                              int nz, void* s) {
  return launch_chain<float>(P, S, I, drude, kind_e, ny, nz, RowRanges{nullptr, 0, 0, 0, 0}, (hipStream_t)s);
}

FDTD_API int fdtd_chain3d_f64(const void* const* P, const double* S, const int* I, int drude, int kind_e, int ny,
                              int nz, void* s) {
  return launch_chain<double>(P, S, I, drude, kind_e, ny, nz, RowRanges{nullptr, 0, 0, 0, 0}, (hipStream_t)s);
}

FDTD_API void fdtd_set_chain_v4(int on) { g_chain_v4 = on != 0; }

// layout of the chain launch tables (checked by the callers that build them)
FDTD_API int fdtd_chain_ints_per_comp() { return CI_PER; }
FDTD_API int fdtd_chain_ptrs_per_comp() { return CP_PER; }

// Dispersive launch over a box with no PML (sigma = 0): rows = int2 (z0, z1)
// per (x, y) of [R[0], R[0] + R[2]) x [R[1], R[1] + R[3]); cells outside their
// row's range take the plain update with the per-component plain coefficient
// (P[24c + 23] per cell or S[2c + 1]).
FDTD_API int fdtd_chain3d_rows_f32(const void* const* P, const double* S, const int* I, int kind_e, int ny, int nz,
                                   const void* rows, const int* R, void* s) {
  return launch_chain<float>(P, S, I, 1, kind_e, ny, nz, RowRanges{(const int2*)rows, R[0], R[1], R[2], R[3]},
                             (hipStream_t)s);
}

FDTD_API int fdtd_chain3d_rows_f64(const void* const* P, const double* S, const int* I, int kind_e, int ny, int nz,
                                   const void* rows, const int* R, void* s) {
  return launch_chain<double>(P, S, I, 1, kind_e, ny, nz, RowRanges{(const int2*)rows, R[0], R[1], R[2], R[3]},
                              (hipStream_t)s);
}
