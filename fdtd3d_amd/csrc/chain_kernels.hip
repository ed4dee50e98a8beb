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
// one write of every result; the generic path of generic_kernels.hip needs 4
// launches and re-reads D / D1 / E between them).
//
// Per component c (kind E; H is the mirror with forward differences):
//   curl = sg0 (s0[x] - s0[x - e_a0]) + sg1 (s1[x] - s1[x - e_a1])
//   Dn   = caD D + cbD curl
//   DRUDE: D1n = b0 Dn + b1 D + b2 Dp + ma1 D1 + ma2 D1p ;  (new, old) = (D1n, D1)
//   else:                                                  (new, old) = (Dn, D)
//   E    = caE E + cbE new + ccE old
// Every coefficient is the factorised product of ops/coef.py (scalar x 1D
// profiles x optional per-cell array).

#include "common.h"

namespace {

template <typename T>
struct CCoef {
  T s;
  const T* px;
  const T* py;
  const T* pz;
  const T* cell;
};

template <typename T>
__device__ __forceinline__ T cc_at(const CCoef<T>& c, int i, int j, int k, size_t off) {
  T v = c.s;
  if (c.px) v *= c.px[i];
  if (c.py) v *= c.py[j];
  if (c.pz) v *= c.pz[k];
  if (c.cell) v *= c.cell[off];
  return v;
}

enum { C_CAD, C_CBD, C_CAE, C_CBE, C_CCE, C_B0, C_B1, C_B2, C_MA1, C_MA2, C_N };

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
  int a0, a1, sg0, sg1;
  CCoef<T> c[C_N];
  Box3 box;
};

template <typename T, bool DRUDE>
__device__ __forceinline__ void chain_cell(const ChainComp<T>& q, int kind_e, const long long* stride, int i, int j,
                                           int k, size_t off) {
  if (!in_box(q.box, i, j, k)) return;
  const long long s0 = stride[q.a0], s1 = stride[q.a1];
  const T d0 = kind_e ? (q.s0[off] - q.s0[off - s0]) : (q.s0[off + s0] - q.s0[off]);
  const T d1 = kind_e ? (q.s1[off] - q.s1[off - s1]) : (q.s1[off + s1] - q.s1[off]);
  const T curl = (q.sg0 > 0 ? d0 : -d0) + (q.sg1 > 0 ? d1 : -d1);
  const T D = q.D[off];
  const T Dn = cc_at(q.c[C_CAD], i, j, k, off) * D + cc_at(q.c[C_CBD], i, j, k, off) * curl;
  q.Dn[off] = Dn;
  T nw = Dn, old = D;
  if (DRUDE) {
    const T D1 = q.D1[off];
    const T D1n = cc_at(q.c[C_B0], i, j, k, off) * Dn + cc_at(q.c[C_B1], i, j, k, off) * D +
                  cc_at(q.c[C_B2], i, j, k, off) * q.Dp[off] + cc_at(q.c[C_MA1], i, j, k, off) * D1 +
                  cc_at(q.c[C_MA2], i, j, k, off) * q.D1p[off];
    q.D1n[off] = D1n;
    nw = D1n;
    old = D1;
  }
  q.E[off] = cc_at(q.c[C_CAE], i, j, k, off) * q.E[off] + cc_at(q.c[C_CBE], i, j, k, off) * nw +
             cc_at(q.c[C_CCE], i, j, k, off) * old;
}

template <typename T, bool DRUDE>
__global__ __launch_bounds__(256) void k_chain3d(ChainComp<T> q0, ChainComp<T> q1, ChainComp<T> q2, int kind_e,
                                                 int ny, int nz, Box3 U) {
  const int k = U.lo[2] + blockIdx.x * 64 + threadIdx.x;
  const int j = U.lo[1] + blockIdx.y * 4 + threadIdx.y;
  const int i = U.lo[0] + blockIdx.z;
  if (k >= U.hi[2] || j >= U.hi[1]) return;
  const long long stride[3] = {(long long)ny * nz, (long long)nz, 1};
  const size_t off = ((size_t)i * ny + j) * nz + k;
  chain_cell<T, DRUDE>(q0, kind_e, stride, i, j, k, off);
  chain_cell<T, DRUDE>(q1, kind_e, stride, i, j, k, off);
  chain_cell<T, DRUDE>(q2, kind_e, stride, i, j, k, off);
}

// pointer layout per component (see fdtd_chain3d_*)
constexpr int CP_FIELDS = 9;                    // E Dn D Dp D1n D1 D1p s0 s1
constexpr int CP_PER = CP_FIELDS + 4 * C_N;     // + (px py pz cell) per coefficient
constexpr int CI_PER = 10;                      // a0 a1 sg0 sg1 box[6]

template <typename T>
ChainComp<T> make_comp(const void* const* P, const double* S, const int* I) {
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
  for (int n = 0; n < C_N; ++n) {
    const void* const* p = P + CP_FIELDS + 4 * n;
    q.c[n] = CCoef<T>{(T)S[n], (const T*)p[0], (const T*)p[1], (const T*)p[2], (const T*)p[3]};
  }
  q.a0 = I[0];
  q.a1 = I[1];
  q.sg0 = I[2];
  q.sg1 = I[3];
  q.box = make_box(I + 4);
  return q;
}

template <typename T>
int launch_chain(const void* const* P, const double* S, const int* I, int drude, int kind_e, int ny, int nz,
                 hipStream_t s) {
  ChainComp<T> q[3];
  Box3 U = {{0, 0, 0}, {0, 0, 0}};
  for (int c = 0; c < 3; ++c) {
    q[c] = make_comp<T>(P + CP_PER * c, S + C_N * c, I + CI_PER * c);
    U = box_union(U, q[c].box);
  }
  if (box_empty(U)) return 0;
  dim3 grid(cdiv(U.hi[2] - U.lo[2], 64), cdiv(U.hi[1] - U.lo[1], 4), (unsigned)(U.hi[0] - U.lo[0]));
  if (drude)
    k_chain3d<T, true><<<grid, dim3(64, 4), 0, s>>>(q[0], q[1], q[2], kind_e, ny, nz, U);
  else
    k_chain3d<T, false><<<grid, dim3(64, 4), 0, s>>>(q[0], q[1], q[2], kind_e, ny, nz, U);
  FDTD_RETURN_LAUNCH_STATUS();
}

}  // namespace

// One chain launch for the three components of a kind.  Per component c:
// P[49c ..]: E Dn D Dp D1n D1 D1p s0 s1, then (px py pz cell) of caD cbD caE cbE
// ccE b0 b1 b2 ma1 ma2; S[10c ..]: the coefficient scalars; I[10c ..]: curl axes
// a0 a1, signs sg0 sg1, box lo[3] hi[3] (empty box: component skipped).
FDTD_API int fdtd_chain3d_f32(const void* const* P, const double* S, const int* I, int drude, int kind_e, int ny,
                              int nz, void* s) {
  return launch_chain<float>(P, S, I, drude, kind_e, ny, nz, (hipStream_t)s);
}

FDTD_API int fdtd_chain3d_f64(const void* const* P, const double* S, const int* I, int drude, int kind_e, int ny,
                              int nz, void* s) {
  return launch_chain<double>(P, S, I, drude, kind_e, ny, nz, (hipStream_t)s);
}
