// Temporally blocked 2D (TMz / TEz) Yee kernel: T leapfrog steps per HBM pass.
//
// The reference's 2D schemes update one component per sweep
// (Source/Scheme/SchemeTMz.cpp:162-1309, SchemeTEz.cpp:109-1025; CUDA TMz:
// Source/Cuda/CudaGlobalKernels.cu:5-153); a single-pass 2D step moves >= 24
// B/cell (3 fields read + written) and the split E / H kernels 36 B.  Here a
// wave owns a 256-cell run of one x row (64 lanes x float4 along the
// contiguous y axis) and streams x; level l of iteration X updates E on row
// X-l and H on row X-l-1 (the same one-row-per-level wavefront as the 3D
// kernels), so T steps cost one read and one write of the three fields.
// y neighbours come from the adjacent lane by DPP wave shifts; T halo cells
// at each end of the run are recomputed redundantly.  Waves never talk to
// each other: no LDS, no barriers.
//
//   TMz: Ez += cb ((Hy - Hy[x-1]) - (Hx - Hx[y-1])),  Hx += db (-(Ez[y+1] - Ez)),
//        Hy += db (Ez[x+1] - Ez)                                      (Kernels.h:64-74)
//   TEz: Ex += cb (Hz - Hz[y-1]),  Ey += cb (-(Hz - Hz[x-1])),
//        Hz += db ((Ex[y+1] - Ex) - (Ey[x+1] - Ey))
// Hard point source after the E half step on any of the three components
// (an H source -- TEz's reference source is Hz -- is set before the H update).

#include "common.h"

namespace {

constexpr int WPB = 4;  // independent waves per workgroup

typedef unsigned u4v __attribute__((ext_vector_type(4)));
typedef unsigned u2v __attribute__((ext_vector_type(2)));
typedef __amdgpu_buffer_rsrc_t Rsrc;

// 16 bytes per lane: float4 or double2 along y
template <typename F>
struct Vec;
template <>
struct Vec<float> {
  typedef float type __attribute__((ext_vector_type(4)));
  static constexpr int N = 4;
};
template <>
struct Vec<double> {
  typedef double type __attribute__((ext_vector_type(2)));
  static constexpr int N = 2;
};

template <typename F>
__device__ __forceinline__ Rsrc row_rsrc(const F* base, int x, int nx, int ny) {
  const bool in = x >= 0 && x < nx;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (size_t)(in ? x : 0) * ny), (short)0,
                                           in ? ny * (int)sizeof(F) : 0, 0x00020000);
}
template <typename F>
__device__ __forceinline__ typename Vec<F>::type ld(Rsrc r, unsigned off) {
  return __builtin_bit_cast(typename Vec<F>::type, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
template <typename F>
__device__ __forceinline__ void st(Rsrc r, unsigned off, const typename Vec<F>::type& v, unsigned m) {
  constexpr int N = Vec<F>::N;
  if (m == (1u << N) - 1u) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), r, off, 0, 0);
  } else if (m) {
#pragma unroll
    for (int q = 0; q < N; ++q) {
      if (!(m & (1u << q))) continue;
      if constexpr (sizeof(F) == 4)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, (float)v[q]), r, off + 4 * q, 0, 0);
      else
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, (double)v[q]), r, off + 8 * q,
                                              0, 0);
    }
  }
}
// value of lane - 1 (CTL 0x138 = wave_shr:1) / lane + 1 (0x130 = wave_shl:1)
template <int CTL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTL, 0xf, 0xf, false));
}
template <int CTL>
__device__ __forceinline__ double dpp(double v) {
  typedef int i2 __attribute__((ext_vector_type(2)));
  i2 w = __builtin_bit_cast(i2, v);
  w.x = __builtin_amdgcn_update_dpp(0, w.x, CTL, 0xf, 0xf, false);
  w.y = __builtin_amdgcn_update_dpp(0, w.y, CTL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, w);
}
template <typename V>
__device__ __forceinline__ V ym1(const V& v) {  // element y-1
  constexpr int N = sizeof(V) / sizeof(v[0]);
  V r;
  r[0] = dpp<0x138>(v[N - 1]);
#pragma unroll
  for (int q = 1; q < N; ++q) r[q] = v[q - 1];
  return r;
}
template <typename V>
__device__ __forceinline__ V yp1(const V& v) {  // element y+1
  constexpr int N = sizeof(V) / sizeof(v[0]);
  V r;
#pragma unroll
  for (int q = 0; q + 1 < N; ++q) r[q] = v[q + 1];
  r[N - 1] = dpp<0x130>(v[0]);
  return r;
}
template <int N>
__device__ __forceinline__ unsigned ymask(const Box3& b, int x, int jb) {
  if (x < b.lo[0] || x >= b.hi[0]) return 0u;
  unsigned m = 0;
#pragma unroll
  for (int e = 0; e < N; ++e) m |= (jb + e >= b.lo[1] && jb + e < b.hi[1]) ? (1u << e) : 0u;
  return m;
}
template <typename V>
__device__ __forceinline__ V sel(const V& c, unsigned m) {
  constexpr int N = sizeof(V) / sizeof(c[0]);
  V r;
#pragma unroll
  for (int q = 0; q < N; ++q) r[q] = (m & (1u << q)) ? c[q] : 0;
  return r;
}

template <typename F>
struct Src2 {
  F v[8];
};

// MODE 0 = TMz (E = {Ez}, H = {Hx, Hy}), 1 = TEz (E = {Ex, Ey}, H = {Hz}).
// Arrays: e0 e1 (e1 unused in TMz), h0 h1 (h1 unused in TEz); boxes b[3] in
// component order (TMz: Ez Hx Hy; TEz: Ex Ey Hz).
template <typename F, int T, int MODE, bool PERCELL>
__global__ __launch_bounds__(64 * WPB) void k_tb2d(const F* __restrict__ e0i, const F* __restrict__ e1i,
                                                   const F* __restrict__ h0i, const F* __restrict__ h1i,
                                                   F* __restrict__ e0o, F* __restrict__ e1o, F* __restrict__ h0o,
                                                   F* __restrict__ h1o, const F* __restrict__ c0,
                                                   const F* __restrict__ c1, const F* __restrict__ c2, F cb, F db,
                                                   int nx, int ny, Box3 b0, Box3 b1, Box3 b2, Box3 O, int xchunk,
                                                   int src_i, int src_j, int src_c, Src2<F> sv) {
  typedef typename Vec<F>::type V;
  constexpr int N = Vec<F>::N;
  constexpr int HL = (T + N - 1) / N;     // halo lanes per side
  constexpr int OWN = (64 - 2 * HL) * N;  // owned cells per wave run
  const int lane = threadIdx.x;
  const int tile = blockIdx.x * WPB + threadIdx.y;
  const int jb = (O.lo[1] & ~(N - 1)) - N * HL + OWN * tile + N * lane;
  if ((O.lo[1] & ~(N - 1)) - N * HL + OWN * tile >= O.hi[1]) return;  // whole wave past the box (uniform)
  const int i0 = O.lo[0] + (int)blockIdx.y * xchunk;
  const int i1 = min(i0 + xchunk, O.hi[0]);
  const bool ld_ok = jb >= 0 && jb < ny;
  const unsigned off = ld_ok ? (unsigned)jb * (unsigned)sizeof(F) : 0xF0000000u;
  const bool own = ld_ok && lane >= HL && lane < 64 - HL;
  const bool src_hit = src_c >= 0 && src_j >= jb && src_j < jb + N;
  const V zero = V(F(0));
  const V cbv = V(cb), dbv = V(db);
  // coefficient of component n (0..2) on row x
  auto coef = [&](const F* arr, const Box3& b, int x, const V& sc) -> V {
    const unsigned m = ld_ok ? ymask<N>(b, x, jb) : 0u;
    if (PERCELL && arr) return sel(ld<F>(row_rsrc(arr, x, nx, ny), off), m);  // null: the kind's scalar
    return sel(sc, m);
  };
  // carried per level l: Hp = H_l(row X-1-l), Ep = E_{l+1}(row X-1-l)
  V Hp0[T], Hp1[T], Ep0[T], Ep1[T];
#pragma unroll
  for (int l = 0; l < T; ++l) Hp0[l] = Hp1[l] = Ep0[l] = Ep1[l] = zero;
  V nh0, nh1, ne0, ne1;  // next row in flight
  auto load_row = [&](int X) {
    nh0 = ld<F>(row_rsrc(h0i, X, nx, ny), off);
    ne0 = ld<F>(row_rsrc(e0i, X, nx, ny), off);
    if (MODE == 0) nh1 = ld<F>(row_rsrc(h1i, X, nx, ny), off);
    else ne1 = ld<F>(row_rsrc(e1i, X, nx, ny), off);
  };
  load_row(i0 - T);
  for (int X = i0 - T; X <= i1 + T - 1; ++X) {
    V Hc0 = nh0, Hc1 = MODE == 0 ? nh1 : zero, Ec0 = ne0, Ec1 = MODE == 1 ? ne1 : zero;
    load_row(X + 1);
    V En0 = zero, En1 = zero;
#pragma unroll
    for (int l = 0; l < T; ++l) {
      const int pe = X - l, ph = pe - 1;
      if (MODE == 0) {
        // Ez on row pe: Hc0 = Hx_l(pe), Hc1 = Hy_l(pe), Hp1 = Hy_l(pe-1)
        En0 = Ec0 + coef(c0, b0, pe, cbv) * ((Hc1 - Hp1[l]) - (Hc0 - ym1(Hc0)));
        if (src_c == 0 && pe == src_i && src_hit) En0[src_j - jb] = sv.v[l];
        // hard Hx / Hy source on row ph before its H update (E of row pe above
        // read the pre-source values)
        V hx0 = Hp0[l], hy0 = Hp1[l];
        if (src_c == 1 && ph == src_i && src_hit) hx0[src_j - jb] = sv.v[l];
        if (src_c == 2 && ph == src_i && src_hit) hy0[src_j - jb] = sv.v[l];
        // Hx, Hy on row ph: Ep0 = Ez_{l+1}(ph), En0 = Ez_{l+1}(pe)
        const V hx = hx0 + coef(c1, b1, ph, dbv) * (-(yp1(Ep0[l]) - Ep0[l]));
        const V hy = hy0 + coef(c2, b2, ph, dbv) * (En0 - Ep0[l]);
        Ec0 = Ep0[l];
        Ep0[l] = En0;
        Hp0[l] = Hc0;
        Hp1[l] = Hc1;
        Hc0 = hx;
        Hc1 = hy;
      } else {
        // Ex, Ey on row pe: Hc0 = Hz_l(pe), Hp0 = Hz_l(pe-1)
        En0 = Ec0 + coef(c0, b0, pe, cbv) * (Hc0 - ym1(Hc0));
        En1 = Ec1 + coef(c1, b1, pe, cbv) * (-(Hc0 - Hp0[l]));
        // hard Hz source on row ph before its H update (the E update of row
        // pe above read the pre-source Hz_l(ph) through Hp0)
        V hz0 = Hp0[l];
        if (src_c == 2 && ph == src_i && src_hit) hz0[src_j - jb] = sv.v[l];
        if (src_c == 0 && pe == src_i && src_hit) En0[src_j - jb] = sv.v[l];
        if (src_c == 1 && pe == src_i && src_hit) En1[src_j - jb] = sv.v[l];
        // Hz on row ph: Ep0 = Ex_{l+1}(ph), Ep1 = Ey_{l+1}(ph), En1 = Ey_{l+1}(pe)
        const V hz = hz0 + coef(c2, b2, ph, dbv) * ((yp1(Ep0[l]) - Ep0[l]) - (En1 - Ep1[l]));
        Ec0 = Ep0[l];
        Ec1 = Ep1[l];
        Ep0[l] = En0;
        Ep1[l] = En1;
        Hp0[l] = Hc0;
        Hc0 = hz;
      }
    }
    // outputs: E_T on row X-T+1, H_T on row X-T
    const int pe = X - T + 1, ph = X - T;
    if (own) {
      if (pe >= i0 && pe < i1) {
        const unsigned m = ymask<N>(O, pe, jb);
        st<F>(row_rsrc(e0o, pe, nx, ny), off, En0, m);
        if (MODE == 1) st<F>(row_rsrc(e1o, pe, nx, ny), off, En1, m);
      }
      if (ph >= i0 && ph < i1) {
        const unsigned m = ymask<N>(O, ph, jb);
        st<F>(row_rsrc(h0o, ph, nx, ny), off, Hc0, m);
        if (MODE == 0) st<F>(row_rsrc(h1o, ph, nx, ny), off, Hc1, m);
      }
    }
  }
}

int g_num_cus2d = 0;

int pick_xchunk2d(long long tiles, int nxo, int T) {
  if (g_num_cus2d <= 0) {
    int dev = 0, n = 0;
    g_num_cus2d = (hipGetDevice(&dev) == hipSuccess &&
                   hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
                      ? n
                      : 256;
  }
  // 4-wave workgroups, several per CU: aim at >= 8 workgroups per CU, then
  // the longest chunk (fewest re-read lead-in rows)
  const long long slots = 8LL * g_num_cus2d;
  int best = nxo;
  long long best_cost = -1;
  for (int k = 1; k <= 512; ++k) {
    const int xc = (nxo + k - 1) / k;
    const long long chunks = (nxo + xc - 1) / xc;
    const long long rounds = (tiles * chunks + slots - 1) / slots;
    const long long cost = rounds * (xc + 2LL * T);
    if (best_cost < 0 || cost < best_cost) {
      best_cost = cost;
      best = xc;
    }
    if (xc == 1) break;
  }
  return best;
}

template <typename F, int T, int MODE>
int launch2d(bool pc, const F* const* ein, const F* const* hin, F* const* eout, F* const* hout, const F* const* cs,
             F cb, F db, int nx, int ny, const Box3* b, const Box3& O, int xchunk, const int* src, const Src2<F>& sv,
             hipStream_t s) {
  constexpr int N = Vec<F>::N;
  constexpr int HL = (T + N - 1) / N;
  constexpr int OWN = (64 - 2 * HL) * N;
  const long long tiles = cdiv(O.hi[1] - ((O.lo[1] & ~(N - 1)) - N * HL) - N * HL, OWN);
  if (xchunk <= 0) xchunk = pick_xchunk2d(cdiv(tiles, WPB), O.hi[0] - O.lo[0], T);
  dim3 grid(cdiv(tiles, WPB), cdiv(O.hi[0] - O.lo[0], xchunk));
#define K2D_ARGS                                                                                             \
  ein[0], ein[1], hin[0], hin[1], eout[0], eout[1], hout[0], hout[1], cs[0], cs[1], cs[2], cb, db, nx, ny, b[0], \
      b[1], b[2], O, xchunk, src[0], src[1], src[2], sv
  if (pc)
    k_tb2d<F, T, MODE, true><<<grid, dim3(64, WPB), 0, s>>>(K2D_ARGS);
  else
    k_tb2d<F, T, MODE, false><<<grid, dim3(64, WPB), 0, s>>>(K2D_ARGS);
#undef K2D_ARGS
  FDTD_RETURN_LAUNCH_STATUS();
}

template <typename F>
constexpr int max_steps2d() { return 8; }

template <typename F, int MODE>
int dispatch2d(int steps, bool pc, const F* const* ein, const F* const* hin, F* const* eout, F* const* hout,
               const F* const* cs, F cb, F db, int nx, int ny, const Box3* b, const Box3& O, int xchunk,
               const int* src, const Src2<F>& sv, hipStream_t s) {
#define C2D(TT)                                                                                                 \
  case TT:                                                                                                      \
    if constexpr (TT <= max_steps2d<F>())                                                                       \
      return launch2d<F, TT, MODE>(pc, ein, hin, eout, hout, cs, cb, db, nx, ny, b, O, xchunk, src, sv, s);     \
    break;
  switch (steps) {
    C2D(1) C2D(2) C2D(3) C2D(4) C2D(5) C2D(6) C2D(7) C2D(8)
  }
#undef C2D
  return (int)hipErrorInvalidValue;
}

template <typename F>
int tb2d(int mode, const F* const* ein, const F* const* hin, F* const* eout, F* const* hout, const F* const* cs,
         double cb, double db, int nx, int ny, const int* boxes, const int* obox, int xchunk, int steps,
         const int* src, const double* src_vals, void* stream) {
  if (ny % Vec<F>::N != 0 || steps < 1 || steps > max_steps2d<F>() || (mode != 0 && mode != 1))
    return (int)hipErrorInvalidValue;
  Box3 b[3];
  for (int n = 0; n < 3; ++n) b[n] = make_box(boxes + 6 * n);
  const Box3 O = make_box(obox);
  if (O.hi[0] <= O.lo[0] || O.hi[1] <= O.lo[1]) return 0;
  Src2<F> sv;
  for (int l = 0; l < 8; ++l) sv.v[l] = (src[2] >= 0 && l < steps) ? (F)src_vals[l] : F(0);
  const bool pc = cs[0] != nullptr || cs[1] != nullptr || cs[2] != nullptr;
  hipStream_t s = (hipStream_t)stream;
  if (mode == 0) return dispatch2d<F, 0>(steps, pc, ein, hin, eout, hout, cs, (F)cb, (F)db, nx, ny, b, O, xchunk, src, sv, s);
  return dispatch2d<F, 1>(steps, pc, ein, hin, eout, hout, cs, (F)cb, (F)db, nx, ny, b, O, xchunk, src, sv, s);
}

}  // namespace

FDTD_API int fdtd_tb2d_max_steps() { return max_steps2d<float>(); }
FDTD_API int fdtd_tb2d64_max_steps() { return max_steps2d<double>(); }

// T (1..8) 2D leapfrog steps in one pass: mode 0 TMz (e =
// {Ez}, h = {Hx, Hy}), 1 TEz (e = {Ex, Ey}, h = {Hz}); unused array slots may
// be null.  `cs` = 3 per-cell coefficient arrays in component order (all
// null: scalars cb / db), `boxes` = 3 update boxes (lo[3] hi[3]) in component
// order (a null array: that component uses its kind's scalar cb / db, so a
// uniform kind streams no constant plane), `obox` = cells stored; `src` = {x, y, component 0..2 | -1} with one
// value per step.  ny must be a multiple of 4 (fp32) / 2 (fp64): 16-byte rows.
FDTD_API int fdtd_tb2d_f32(int mode, const float* const* ein, const float* const* hin, float* const* eout,
                           float* const* hout, const float* const* cs, double cb, double db, int nx, int ny,
                           const int* boxes, const int* obox, int xchunk, int steps, const int* src,
                           const double* src_vals, void* stream) {
  return tb2d<float>(mode, ein, hin, eout, hout, cs, cb, db, nx, ny, boxes, obox, xchunk, steps, src, src_vals,
                     stream);
}
FDTD_API int fdtd_tb2d_f64(int mode, const double* const* ein, const double* const* hin, double* const* eout,
                           double* const* hout, const double* const* cs, double cb, double db, int nx, int ny,
                           const int* boxes, const int* obox, int xchunk, int steps, const int* src,
                           const double* src_vals, void* stream) {
  return tb2d<double>(mode, ein, hin, eout, hout, cs, cb, db, nx, ny, boxes, obox, xchunk, steps, src, src_vals,
                      stream);
}
