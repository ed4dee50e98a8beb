// Register-resident 1D Yee kernel: a whole run of N leapfrog steps in ONE
// launch of ONE workgroup.
//
// A 1D grid of the reference's sizes (BASELINE config 1: 10 000 cells) is far
// too small to fill 256 CUs, and one launch per half step makes the per-step
// path launch-bound (~1.3k Mcells/s even with HIP graphs).  Here 1024 threads
// (16 waves, one CU) hold the grid in registers -- CPL contiguous cells of Ez
// and Hy per thread -- and step it N times; the only traffic per half step is
// one boundary value per thread through LDS and one workgroup barrier.  The
// cell -> thread map is shifted so that the point source lands on element 0
// of its thread (one select per step, no dynamic register indexing).
//
//   Ez[i] += cb (Hy[i] - Hy[i-1]),   Hy[i] += db (Ez[i+1] - Ez[i])
// (reference 1D-form macros: Source/Kernels/Kernels.h; 1D driver semantics as
// the 2D/3D schemes: E half step, hard Ez source, H half step).

#include "common.h"

namespace {

constexpr int NT = 1024;

template <typename T, int CPL, bool PERCELL>
__global__ __launch_bounds__(NT) void k_res1d(T* __restrict__ ez, T* __restrict__ hy, const T* __restrict__ cbz,
                                              const T* __restrict__ dby, T cb, T db, int n, int elo, int ehi,
                                              int hlo, int hhi, int off, int nsteps, int src_t,
                                              const T* __restrict__ src_vals) {
  __shared__ T sH[NT], sE[NT];
  const int t = threadIdx.x;
  const int base = t * CPL - off;
  T e[CPL], h[CPL];
  T ce[PERCELL ? CPL : 1], ch[PERCELL ? CPL : 1];
  unsigned long long me = 0, mh = 0;  // box membership bits (scalar coefficients)
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int i = base + k;
    const bool in = i >= 0 && i < n;
    e[k] = in ? ez[i] : T(0);
    h[k] = in ? hy[i] : T(0);
    const bool ie = in && i >= elo && i < ehi, ih = in && i >= hlo && i < hhi;
    if (PERCELL) {
      ce[k] = ie ? cbz[i] : T(0);
      ch[k] = ih ? dby[i] : T(0);
    } else {
      me |= (unsigned long long)ie << k;
      mh |= (unsigned long long)ih << k;
    }
  }
  auto cE = [&](int k) -> T {
    if (PERCELL) return ce[k];
    return ((me >> k) & 1ull) ? cb : T(0);
  };
  auto cH = [&](int k) -> T {
    if (PERCELL) return ch[k];
    return ((mh >> k) & 1ull) ? db : T(0);
  };
  const bool src_here = src_vals != nullptr && t == src_t;
  T v = (src_vals != nullptr && nsteps > 0) ? src_vals[0] : T(0);
  for (int s = 0; s < nsteps; ++s) {
    const T vnext = (src_vals != nullptr && s + 1 < nsteps) ? src_vals[s + 1] : T(0);
    // E half step: Hy[i-1] of element 0 comes from the previous thread
    sH[t] = h[CPL - 1];
    __syncthreads();
    const T hm1 = t > 0 ? sH[t - 1] : T(0);
#pragma unroll
    for (int k = CPL - 1; k >= 1; --k) e[k] += cE(k) * (h[k] - h[k - 1]);
    e[0] += cE(0) * (h[0] - hm1);
    if (src_here) e[0] = v;
    // H half step: Ez[i+1] of the last element comes from the next thread
    sE[t] = e[0];
    __syncthreads();
    const T ep1 = t + 1 < NT ? sE[t + 1] : T(0);
#pragma unroll
    for (int k = 0; k < CPL - 1; ++k) h[k] += cH(k) * (e[k + 1] - e[k]);
    h[CPL - 1] += cH(CPL - 1) * (ep1 - e[CPL - 1]);
    v = vnext;
  }
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int i = base + k;
    if (i >= 0 && i < n) {
      ez[i] = e[k];
      hy[i] = h[k];
    }
  }
}

template <typename T, int CPL>
int launch(bool pc, T* ez, T* hy, const T* cbz, const T* dby, double cb, double db, int n, const int* b, int off,
           int nsteps, int src_t, const T* vals, hipStream_t s) {
  if (pc)
    k_res1d<T, CPL, true><<<1, NT, 0, s>>>(ez, hy, cbz, dby, (T)cb, (T)db, n, b[0], b[1], b[2], b[3], off, nsteps,
                                           src_t, vals);
  else
    k_res1d<T, CPL, false><<<1, NT, 0, s>>>(ez, hy, cbz, dby, (T)cb, (T)db, n, b[0], b[1], b[2], b[3], off, nsteps,
                                            src_t, vals);
  FDTD_RETURN_LAUNCH_STATUS();
}

// cells per thread instantiated (1024 threads leave 128 VGPRs per lane: fp32
// state fits up to 16 cells per thread, fp64 up to 12)
constexpr int CPLS[] = {1, 2, 4, 6, 8, 12, 16};
template <typename T>
constexpr int max_cpl() { return sizeof(T) == 8 ? 12 : 16; }

template <typename T>
int res1d(T* ez, T* hy, const T* cbz, const T* dby, double cb, double db, int n, const int* boxes, int nsteps,
          int src_i, const T* vals, hipStream_t s) {
  const bool pc = cbz != nullptr;
  if ((cbz == nullptr) != (dby == nullptr) || n <= 0 || nsteps < 0) return (int)hipErrorInvalidValue;
  for (int cpl : CPLS) {
    if (cpl > max_cpl<T>()) break;
    const int off = (vals != nullptr && src_i >= 0) ? (cpl - src_i % cpl) % cpl : 0;
    if ((long long)n + off > (long long)NT * cpl) continue;
    const int src_t = (vals != nullptr && src_i >= 0) ? (src_i + off) / cpl : -1;
    const T* v = src_t >= 0 ? vals : nullptr;
    switch (cpl) {
#define R1(C) \
  case C: return launch<T, C>(pc, ez, hy, cbz, dby, cb, db, n, boxes, off, nsteps, src_t, v, s);
      R1(1) R1(2) R1(4) R1(6) R1(8) R1(12)
#undef R1
      case 16:
        if constexpr (max_cpl<T>() >= 16) return launch<T, 16>(pc, ez, hy, cbz, dby, cb, db, n, boxes, off, nsteps, src_t, v, s);
        break;
    }
  }
  return (int)hipErrorInvalidValue;  // grid too long for one workgroup
}

}  // namespace

// Largest 1D grid one resident launch holds (cells) whatever the source cell
// (the source shift costs up to CPL - 1 cells), per element size.
FDTD_API int fdtd_res1d_max_cells(int elem_bytes) {
  const int c = elem_bytes == 8 ? max_cpl<double>() : max_cpl<float>();
  return NT * c - (c - 1);
}

// nsteps leapfrog steps of the 1D (Ez, Hy) grid of n cells in place; boxes =
// {E lo, E hi, H lo, H hi}; cbz / dby per-cell coefficients (both or neither);
// vals[nsteps] device array of hard Ez source values at cell src_i, or null.
FDTD_API int fdtd_res1d_f32(float* ez, float* hy, const float* cbz, const float* dby, double cb, double db, int n,
                            const int* boxes, int nsteps, int src_i, const float* vals, void* s) {
  return res1d<float>(ez, hy, cbz, dby, cb, db, n, boxes, nsteps, src_i, vals, (hipStream_t)s);
}
FDTD_API int fdtd_res1d_f64(double* ez, double* hy, const double* cbz, const double* dby, double cb, double db,
                            int n, const int* boxes, int nsteps, int src_i, const double* vals, void* s) {
  return res1d<double>(ez, hy, cbz, dby, cb, db, n, boxes, nsteps, src_i, vals, (hipStream_t)s);
}
