// Native CPU 1D leapfrog (Ez, Hy) of the torch/CPU backend -- the reference's
// plumbing configuration (BASELINE config 1: 10 000 cells, Gaussian pulse,
// CPU path).  Same arithmetic and order as the register-resident GPU kernel
// (yee1d_res.hip k_res1d): per step the E half step on [elo, ehi) from the
// old H, the hard Ez source, the H half step on [hlo, hhi) from the new E.
// A torch op per half step on 10 000 cells is launch-bound (~200 Mcells/s);
// this loop keeps both arrays in L1/L2 and vectorises.
#pragma GCC optimize("O3")
#include <cstddef>

namespace {

template <typename T>
__attribute__((always_inline)) inline void res1d_cpu(T* __restrict__ ez, T* __restrict__ hy, const T* __restrict__ cbz, const T* __restrict__ dby, T cb,
               T db, int n, const int* b, int nsteps, int src_i, const T* __restrict__ vals) {
  const int elo = b[0] < 1 ? 1 : b[0], ehi = b[1] > n ? n : b[1];
  const int hlo = b[2] < 0 ? 0 : b[2], hhi = b[3] > n - 1 ? n - 1 : b[3];
  for (int s = 0; s < nsteps; ++s) {
    // E from the old H (the loop writes only ez: no dependence between cells)
    if (cbz) {
#pragma GCC ivdep
      for (int i = elo; i < ehi; ++i) ez[i] += cbz[i] * (hy[i] - hy[i - 1]);
    } else {
#pragma GCC ivdep
      for (int i = elo; i < ehi; ++i) ez[i] += cb * (hy[i] - hy[i - 1]);
    }
    if (vals && src_i >= 0 && src_i < n) ez[src_i] = vals[s];
    if (dby) {
#pragma GCC ivdep
      for (int i = hlo; i < hhi; ++i) hy[i] += dby[i] * (ez[i + 1] - ez[i]);
    } else {
#pragma GCC ivdep
      for (int i = hlo; i < hhi; ++i) hy[i] += db * (ez[i + 1] - ez[i]);
    }
  }
}

}  // namespace

#define HOST_API extern "C" __attribute__((visibility("default")))
// one clone per vector ISA, picked when the library loads (the GPU box's host
// CPU may differ from the build machine's)
#define VEC_CLONES __attribute__((target_clones("avx512f", "avx2", "default")))

// nsteps steps in place; boxes = {E lo, E hi, H lo, H hi}; cbz / dby per-cell
// coefficients or null (scalars cb / db); vals[nsteps] source values at src_i
// or null.  Returns 0.
HOST_API VEC_CLONES int fdtd_res1d_cpu_f64(double* ez, double* hy, const double* cbz, const double* dby, double cb, double db,
                                int n, const int* boxes, int nsteps, int src_i, const double* vals) {
  res1d_cpu<double>(ez, hy, cbz, dby, cb, db, n, boxes, nsteps, src_i, vals);
  return 0;
}
HOST_API VEC_CLONES int fdtd_res1d_cpu_f32(float* ez, float* hy, const float* cbz, const float* dby, double cb, double db, int n,
                                const int* boxes, int nsteps, int src_i, const float* vals) {
  res1d_cpu<float>(ez, hy, cbz, dby, (float)cb, (float)db, n, boxes, nsteps, src_i, vals);
  return 0;
}
