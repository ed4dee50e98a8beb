// Auxiliary kernels: sources, halo pack/unpack, reductions, amplitude
// tracking.  All launch on the caller's stream and never synchronise, so they
// can be captured into HIP graphs together with the stencil kernels.

#include "common.h"
#include "vec4.h"

namespace {

// ---------------------------------------------------------------- sources
// Hard source: field[off] = value (Scheme3D.cpp:2011-2022).  The value is a
// host-computed double so the waveform (sin(2 pi f dt t), Gaussian, ...) is
// bit-identical between backends.
template <typename T>
__global__ void k_set_value(T* __restrict__ f, long long off, double v) {
  if (threadIdx.x == 0) f[off] = (T)v;
}

// Line/point list source: f[offs[n]] = v (amplitude-mode z-line source,
// Scheme3D.cpp:2995-3013).
template <typename T>
__global__ void k_set_values(T* __restrict__ f, const long long* __restrict__ offs, int n, double v) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) f[offs[t]] = (T)v;
}

// Graph-replayable source: the value comes from a device table indexed by a
// device step counter (+ the step's position inside the captured sequence),
// so one captured HIP graph of G steps can be replayed for any G steps.
template <typename T>
__global__ void k_set_value_tab(T* __restrict__ f, long long off, const double* __restrict__ tab,
                                const int* __restrict__ counter, int lag) {
  if (threadIdx.x == 0) f[off] = (T)tab[*counter + lag];
}

__global__ void k_counter_add(int* counter, int n) {
  if (threadIdx.x == 0) *counter += n;
}

// ---------------------------------------------------------------- halo boxes
// Copy a strided box of `ncomp` fields into a packed buffer (pack) or back
// (unpack).  One 16-byte vector (or one element on unaligned boxes) per
// thread and iteration; the z run of each box row is contiguous in both the
// field and the buffer, so rows are coalesced.
template <typename T>
struct FieldPtrs {
  T* p[8];
};

// Buffer layout [component][x][y][z].  grid.z walks (component, x plane) --
// wave-uniform, so the field pointer is a scalar load -- and grid.x threads
// walk the plane's (y, z) cells with ONE 32-bit divide each (the first
// version decoded a 64-bit linear index per element with three 64-bit
// divides, more instructions than the copy's memory time).
template <typename T, bool PACK, int V>
__global__ __launch_bounds__(256) void k_box_copy(FieldPtrs<T> fields, T* __restrict__ buf, int ny, int nz,
                                                  Box3 b) {
  // V elements (16 bytes when V > 1) per thread and iteration
  typedef T VT __attribute__((ext_vector_type(V)));
  const int bx = b.hi[0] - b.lo[0], by = b.hi[1] - b.lo[1], bz = b.hi[2] - b.lo[2];
  const int ci = blockIdx.z;  // component * bx + plane
  const int c = ci / bx, i = ci - c * bx;
  T* __restrict__ f = fields.p[c];
  const int bzv = bz / V, nyzv = by * bzv;
  const size_t fplane = (size_t)(b.lo[0] + i) * ny;
  const size_t bplane = (size_t)ci * by * bz;
  for (int jk = blockIdx.x * 256 + threadIdx.x; jk < nyzv; jk += gridDim.x * 256) {
    const int j = jk / bzv, kv = jk - j * bzv;
    const size_t off = (fplane + (b.lo[1] + j)) * nz + (b.lo[2] + kv * V);
    const size_t boff = bplane + (size_t)jk * V;
    if (V == 1) {
      if (PACK)
        buf[boff] = f[off];
      else
        f[off] = buf[boff];
    } else {
      if (PACK)
        *reinterpret_cast<VT*>(buf + boff) = *reinterpret_cast<const VT*>(f + off);
      else
        *reinterpret_cast<VT*>(f + off) = *reinterpret_cast<const VT*>(buf + boff);
    }
  }
}

// grid of a box copy with V elements per thread: up to 1024 blocks of 256
// threads per (component, plane)
inline dim3 box_copy_grid(const Box3& b, int ncomp, int V) {
  const long long nyz = (long long)(b.hi[1] - b.lo[1]) * (b.hi[2] - b.lo[2]) / V;
  const long long per = (nyz + 255) / 256;
  return dim3((unsigned)(per < 1024 ? per : 1024), 1, (unsigned)((b.hi[0] - b.lo[0]) * ncomp));
}

// 16-byte vectors when every row run, row start and the buffer are aligned
template <typename T>
inline int box_copy_vec(const Box3& b, int nz, const void* buf, T* const* fields, int ncomp) {
  constexpr int V = 16 / sizeof(T);
  bool ok = (b.hi[2] - b.lo[2]) % V == 0 && b.lo[2] % V == 0 && nz % V == 0 && ((uintptr_t)buf & 15) == 0;
  for (int c = 0; c < ncomp && ok; ++c) ok = ((uintptr_t)fields[c] & 15) == 0;
  return ok ? V : 1;
}

template <typename T, bool PACK>
int launch_box_copy(T* const* fields, T* buf, int ncomp, int ny, int nz, const Box3& b, hipStream_t s) {
  FieldPtrs<T> fp;
  for (int c = 0; c < ncomp; ++c) fp.p[c] = fields[c];
  if ((long long)(b.hi[0] - b.lo[0]) * ncomp > 65535) return (int)hipErrorInvalidValue;
  constexpr int VW = 16 / sizeof(T);
  if (box_copy_vec<T>(b, nz, buf, fields, ncomp) == VW)
    k_box_copy<T, PACK, VW><<<box_copy_grid(b, ncomp, VW), 256, 0, s>>>(fp, buf, ny, nz, b);
  else
    k_box_copy<T, PACK, 1><<<box_copy_grid(b, ncomp, 1), 256, 0, s>>>(fp, buf, ny, nz, b);
  FDTD_RETURN_LAUNCH_STATUS();
}

// Field-to-field copy of a box for `ncomp` component pairs (the hybrid
// pass's shell copy): same (component, plane) x (y, z) walk as k_box_copy.
template <typename T, int V>
__global__ __launch_bounds__(256) void k_box_xfer(FieldPtrs<T> src, FieldPtrs<T> dst, int ny, int nz, Box3 b) {
  typedef T VT __attribute__((ext_vector_type(V)));
  const int bx = b.hi[0] - b.lo[0], by = b.hi[1] - b.lo[1], bz = b.hi[2] - b.lo[2];
  const int ci = blockIdx.z;
  const int c = ci / bx, i = ci - c * bx;
  const T* __restrict__ f = src.p[c];
  T* __restrict__ g = dst.p[c];
  const int bzv = bz / V, nyzv = by * bzv;
  const size_t fplane = (size_t)(b.lo[0] + i) * ny;
  for (int jk = blockIdx.x * 256 + threadIdx.x; jk < nyzv; jk += gridDim.x * 256) {
    const int j = jk / bzv, kv = jk - j * bzv;
    const size_t off = (fplane + (b.lo[1] + j)) * nz + (b.lo[2] + kv * V);
    if (V == 1)
      g[off] = f[off];
    else
      *reinterpret_cast<VT*>(g + off) = *reinterpret_cast<const VT*>(f + off);
  }
}

// Unaligned z range on rows of whole 16-byte vectors: aligned vector loads
// over the covering groups, element stores only inside [lo, hi) (the cells
// next to the box belong to someone else's output).
template <typename T>
__global__ __launch_bounds__(256) void k_box_xfer_m(FieldPtrs<T> src, FieldPtrs<T> dst, int ny, int nz, Box3 b) {
  constexpr int V = 16 / sizeof(T);
  typedef T VT __attribute__((ext_vector_type(V)));
  const int bx = b.hi[0] - b.lo[0], by = b.hi[1] - b.lo[1];
  const int z0 = b.lo[2] & ~(V - 1);
  const int ng = (b.hi[2] - z0 + V - 1) / V;  // vector groups per row
  const int ci = blockIdx.z;
  const int c = ci / bx, i = ci - c * bx;
  const T* __restrict__ f = src.p[c];
  T* __restrict__ g = dst.p[c];
  const int nyzv = by * ng;
  const size_t fplane = (size_t)(b.lo[0] + i) * ny;
  for (int jk = blockIdx.x * 256 + threadIdx.x; jk < nyzv; jk += gridDim.x * 256) {
    const int j = jk / ng, q = jk - j * ng;
    const int k = z0 + q * V;
    const size_t off = (fplane + (b.lo[1] + j)) * nz + k;
    const VT v = *reinterpret_cast<const VT*>(f + off);
    if (k >= b.lo[2] && k + V <= b.hi[2]) {
      *reinterpret_cast<VT*>(g + off) = v;
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e)
        if (k + e >= b.lo[2] && k + e < b.hi[2]) g[off + e] = v[e];
    }
  }
}

template <typename T>
int launch_box_xfer(T* const* src, T* const* dst, int ncomp, int ny, int nz, const Box3& b, hipStream_t s) {
  FieldPtrs<T> fs, fd;
  constexpr int VW = 16 / sizeof(T);
  bool vec = (b.hi[2] - b.lo[2]) % VW == 0 && b.lo[2] % VW == 0 && nz % VW == 0;
  bool vrow = nz % VW == 0;  // rows of whole vectors: masked vector path for unaligned boxes
  for (int c = 0; c < ncomp; ++c) {
    fs.p[c] = src[c];
    fd.p[c] = dst[c];
    const bool al = ((uintptr_t)src[c] & 15) == 0 && ((uintptr_t)dst[c] & 15) == 0;
    vec = vec && al;
    vrow = vrow && al;
  }
  if ((long long)(b.hi[0] - b.lo[0]) * ncomp > 65535) return (int)hipErrorInvalidValue;
  if (vec)
    k_box_xfer<T, VW><<<box_copy_grid(b, ncomp, VW), 256, 0, s>>>(fs, fd, ny, nz, b);
  else if (vrow)
    k_box_xfer_m<T><<<box_copy_grid(b, ncomp, VW), 256, 0, s>>>(fs, fd, ny, nz, b);
  else
    k_box_xfer<T, 1><<<box_copy_grid(b, ncomp, 1), 256, 0, s>>>(fs, fd, ny, nz, b);
  FDTD_RETURN_LAUNCH_STATUS();
}

// ---------------------------------------------------------------- reductions
// max |f| over a box -> atomicMax on the float bit pattern (non-negative
// floats order like their integer bits).  Used by the amplitude mode and the
// non-finite watchdog (NaN is mapped to +inf so it is never lost).
template <typename T>
__device__ __forceinline__ float absf_sat(T v) {
  float a = fabsf((float)v);
  return (a != a) ? __builtin_huge_valf() : a;
}

template <typename T>
__global__ __launch_bounds__(256) void k_box_maxabs(const T* __restrict__ f, int ny, int nz, Box3 b,
                                                    unsigned int* __restrict__ out) {
  const int bx = b.hi[0] - b.lo[0], by = b.hi[1] - b.lo[1], bz = b.hi[2] - b.lo[2];
  const long long n = (long long)bx * by * bz;
  float m = 0.f;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(t % bz);
    const long long r = t / bz;
    const int j = (int)(r % by);
    const int i = (int)(r / by);
    const size_t off = ((size_t)(b.lo[0] + i) * ny + (b.lo[1] + j)) * nz + (b.lo[2] + k);
    m = fmaxf(m, absf_sat(f[off]));
  }
  // wave64 reduction
  for (int d = 32; d > 0; d >>= 1) m = fmaxf(m, __shfl_xor(m, d, 64));
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = red[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = fmaxf(r, red[w]);
    atomicMax(out, __float_as_uint(r));
  }
}

// Amplitude mode (Scheme3D.cpp:3294-3333): amp = max(amp, |f|) over a box and
// count the cells whose amplitude changed by more than `accuracy` relative.
template <typename T>
__global__ __launch_bounds__(256) void k_amplitude_update(const T* __restrict__ f, T* __restrict__ amp, int ny,
                                                          int nz, Box3 b, double accuracy,
                                                          unsigned int* __restrict__ changed) {
  const int bx = b.hi[0] - b.lo[0], by = b.hi[1] - b.lo[1], bz = b.hi[2] - b.lo[2];
  const long long n = (long long)bx * by * bz;
  unsigned int cnt = 0;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(t % bz);
    const long long r = t / bz;
    const int j = (int)(r % by);
    const int i = (int)(r / by);
    const size_t off = ((size_t)(b.lo[0] + i) * ny + (b.lo[1] + j)) * nz + (b.lo[2] + k);
    const T v = f[off] < T(0) ? -f[off] : f[off];
    const T a = amp[off];
    if (v >= a) {
      // relative growth, exactly Scheme3D::updateAmplitude (Scheme3D.cpp:3294-3333)
      T acc = v - a;
      if (a != T(0))
        acc /= a;
      else if (v != T(0))
        acc /= v;
      if (acc > (T)accuracy) {
        cnt++;
        amp[off] = v;
      }
    }
  }
  for (int d = 32; d > 0; d >>= 1) cnt += __shfl_xor(cnt, d, 64);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(changed, cnt);
}

// All components of a kind at once (blockIdx.y = component), accumulating
// into a device counter the host reads once per amplitude check period
// instead of once per component and step.
struct AmpSet {
  const void* f[6];
  void* amp[6];
  Box3 b[6];
  long long xs;  // x stride of the amp arrays (elements): the maxima of one x plane of all
                 // components are contiguous (models/scheme.py; tb3d_mr.h AmpDev)
};

// one cell of every component per thread: a 3D grid over the union of the
// component boxes (z lanes, 4 rows per workgroup, one x plane per grid
// slice), no index division; per-wave count reduction, one atomic per wave
template <typename T>
__global__ __launch_bounds__(256) void k_amplitude_many(AmpSet a, int ncomp, Box3 u, int ny, int nz,
                                                        double accuracy, unsigned int* __restrict__ changed) {
  const int k = u.lo[2] + blockIdx.x * 64 + threadIdx.x;
  const int j = u.lo[1] + blockIdx.y * 4 + threadIdx.y;
  const int i = u.lo[0] + blockIdx.z;
  unsigned int cnt = 0;
  if (k < u.hi[2] && j < u.hi[1]) {
    const size_t off = ((size_t)i * ny + j) * nz + k;
    const size_t aoff = (size_t)i * a.xs + (size_t)j * nz + k;
    const T acc_t = (T)accuracy;
    // every component's field and running maximum loaded before the first
    // store (a store through one amp pointer could alias the next loads, which
    // otherwise serialises six memory round trips per cell)
    T fv[6], am[6];
    bool in[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const Box3& b = a.b[c];
      in[c] = c < ncomp && i >= b.lo[0] && i < b.hi[0] && j >= b.lo[1] && j < b.hi[1] && k >= b.lo[2] &&
              k < b.hi[2];
      fv[c] = in[c] ? ((const T*)a.f[c])[off] : T(0);
      am[c] = in[c] ? ((const T*)a.amp[c])[aoff] : T(0);
    }
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const T v = fv[c] < T(0) ? -fv[c] : fv[c];
      if (in[c] && v >= am[c]) {
        const T den = am[c] != T(0) ? am[c] : (v != T(0) ? v : T(1));
        if ((v - am[c]) / den > acc_t) {
          cnt++;
          ((T*)a.amp[c])[aoff] = v;
        }
      }
    }
  }
  for (int d = 32; d > 0; d >>= 1) cnt += __shfl_xor(cnt, d, 64);
  if (threadIdx.x == 0 && cnt) atomicAdd(changed, cnt);
}

// fp32 float4 form (rows of whole 16-byte groups, nz % 4 == 0): four cells of
// every component per thread, 16-byte loads, masked stores of the changed
// maxima -- the amplitude update is a pure streaming pass (read f and amp,
// write the grown amp), so the vector width is its bandwidth
__global__ __launch_bounds__(256) void k_amplitude_many_v4(AmpSet a, int ncomp, Box3 u, int ny, int nz,
                                                           float accuracy, unsigned int* __restrict__ changed) {
  const int kb = (u.lo[2] & ~3) + 4 * (blockIdx.x * 64 + threadIdx.x);
  const int j = u.lo[1] + blockIdx.y * 4 + threadIdx.y;
  const int i = u.lo[0] + blockIdx.z;
  unsigned int cnt = 0;
  if (kb < u.hi[2] && j < u.hi[1]) {
    const size_t off = ((size_t)i * ny + j) * nz + kb;
    const size_t aoff = (size_t)i * a.xs + (size_t)j * nz + kb;
    float4 fv[6], am[6];
    unsigned m[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const Box3& b = a.b[c];
      m[c] = (c < ncomp && i >= b.lo[0] && i < b.hi[0]) ? kmask(b, j, kb) : 0u;
      fv[c] = m[c] ? ld4((const float*)a.f[c], off) : make_float4(0.f, 0.f, 0.f, 0.f);
      am[c] = m[c] ? ld4((const float*)a.amp[c], aoff) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      unsigned w = 0;
      float4 nv = am[c];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float f = f4(fv[c], e), v = f < 0.f ? -f : f, old = f4(am[c], e);
        const float den = old != 0.f ? old : (v != 0.f ? v : 1.f);
        if (((m[c] >> e) & 1u) && v >= old && (v - old) / den > accuracy) {
          w |= 1u << e;
          f4set(nv, e, v);
          cnt++;
        }
      }
      st4m((float*)a.amp[c], aoff, nv, w);
    }
  }
  for (int d = 32; d > 0; d >>= 1) cnt += __shfl_xor(cnt, d, 64);
  if (threadIdx.x == 0 && cnt) atomicAdd(changed, cnt);
}

inline unsigned reduce_grid(long long n) {
  long long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// Many boxes of many arrays to / from contiguous buffers in ONE launch (the
// halo exchange of a decomposed run: every message's fields and region-local
// auxiliary arrays, packed before the sends / unpacked after the receives).
// One table entry per (array, box, buffer part); the blocks of entry e are
// blk0[e] .. blk0[e + 1] - 1, 256 elements each, box cells z fastest.
struct BoxEnt {
  long long arr;  // array base (its dims: ny x nz per x plane)
  long long buf;  // this entry's first buffer element
  int ny, nz;
  int lo[3], hi[3];
  int blk0;       // first block of the entry
  int vec;        // elements per thread: 16-byte vectors (4 fp32 / 2 fp64) when every row run is aligned, else 1
  int pad[2];
};
static_assert(sizeof(BoxEnt) == 64, "BoxEnt layout (parallel/halo.py _BoxList)");

template <typename T, bool PACK, int V>
__device__ __forceinline__ void box_list_copy(const BoxEnt& e, int blk) {
  typedef T VT __attribute__((ext_vector_type(V)));
  const int by = e.hi[1] - e.lo[1], bzv = (e.hi[2] - e.lo[2]) / V;
  const int n = (e.hi[0] - e.lo[0]) * by * bzv;
  const int idx = blk * 256 + (int)threadIdx.x;  // in V-element groups
  if (idx >= n) return;
  const int kv = idx % bzv, jj = idx / bzv;
  const int j = jj % by, i = jj / by;
  T* a = (T*)e.arr;
  T* f = (T*)e.buf;
  const size_t off = ((size_t)(e.lo[0] + i) * e.ny + (e.lo[1] + j)) * e.nz + (e.lo[2] + kv * V);
  const size_t boff = (size_t)idx * V;
  if (V == 1) {
    if (PACK)
      f[boff] = a[off];
    else
      a[off] = f[boff];
  } else {
    if (PACK)
      *reinterpret_cast<VT*>(f + boff) = *reinterpret_cast<const VT*>(a + off);
    else
      *reinterpret_cast<VT*>(a + off) = *reinterpret_cast<const VT*>(f + boff);
  }
}

template <typename T, bool PACK>
__global__ __launch_bounds__(256) void k_box_list(const BoxEnt* __restrict__ tab, int n) {
  // the block's entry: binary search over blk0 (wave-uniform scalar loads)
  typedef const __attribute__((address_space(4))) BoxEnt* EntPtr;
  const EntPtr E = (EntPtr)tab;
  const int b = (int)blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (E[mid].blk0 <= b) lo = mid; else hi = mid - 1;
  }
  BoxEnt e;  // (field by field: the constant-address-space entry has no implicit copy)
  e.arr = E[lo].arr;
  e.buf = E[lo].buf;
  e.ny = E[lo].ny;
  e.nz = E[lo].nz;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    e.lo[d] = E[lo].lo[d];
    e.hi[d] = E[lo].hi[d];
  }
  e.blk0 = E[lo].blk0;
  e.vec = E[lo].vec;
  constexpr int VW = 16 / sizeof(T);
  if (e.vec == VW)
    box_list_copy<T, PACK, VW>(e, b - e.blk0);
  else
    box_list_copy<T, PACK, 1>(e, b - e.blk0);
}

}  // namespace

#define FDTD_AUX_API(SUF, T)                                                                                  \
  FDTD_API int fdtd_set_value_##SUF(T* f, long long off, double v, void* s) {                                 \
    k_set_value<T><<<1, 64, 0, (hipStream_t)s>>>(f, off, v);                                                   \
    FDTD_RETURN_LAUNCH_STATUS();                                                                              \
  }                                                                                                           \
  FDTD_API int fdtd_set_value_tab_##SUF(T* f, long long off, const double* tab, const int* counter, int lag,   \
                                       void* s) {                                                             \
    k_set_value_tab<T><<<1, 64, 0, (hipStream_t)s>>>(f, off, tab, counter, lag);                               \
    FDTD_RETURN_LAUNCH_STATUS();                                                                              \
  }                                                                                                           \
  FDTD_API int fdtd_set_values_##SUF(T* f, const long long* offs, int n, double v, void* s) {                 \
    if (n <= 0) return 0;                                                                                     \
    k_set_values<T><<<cdiv(n, 256), 256, 0, (hipStream_t)s>>>(f, offs, n, v);                                  \
    FDTD_RETURN_LAUNCH_STATUS();                                                                              \
  }                                                                                                           \
  FDTD_API int fdtd_box_pack_##SUF(T* const* fields, T* buf, int ncomp, int ny, int nz, const int* box,        \
                                   void* s) {                                                                 \
    Box3 b = make_box(box);                                                                                   \
    if (box_empty(b) || ncomp <= 0 || ncomp > 8) return ncomp > 8 ? (int)hipErrorInvalidValue : 0;             \
    return launch_box_copy<T, true>(fields, buf, ncomp, ny, nz, b, (hipStream_t)s);                          \
  }                                                                                                           \
  FDTD_API int fdtd_box_unpack_##SUF(T* const* fields, const T* buf, int ncomp, int ny, int nz,                \
                                     const int* box, void* s) {                                               \
    Box3 b = make_box(box);                                                                                   \
    if (box_empty(b) || ncomp <= 0 || ncomp > 8) return ncomp > 8 ? (int)hipErrorInvalidValue : 0;             \
    return launch_box_copy<T, false>(fields, (T*)buf, ncomp, ny, nz, b, (hipStream_t)s);                    \
  }                                                                                                           \
  FDTD_API int fdtd_box_xfer_##SUF(T* const* src, T* const* dst, int ncomp, int ny, int nz, const int* box,     \
                                   void* s) {                                                                 \
    Box3 b = make_box(box);                                                                                   \
    if (box_empty(b) || ncomp <= 0 || ncomp > 8) return ncomp > 8 ? (int)hipErrorInvalidValue : 0;             \
    return launch_box_xfer<T>(src, dst, ncomp, ny, nz, b, (hipStream_t)s);                                   \
  }                                                                                                           \
  FDTD_API int fdtd_box_maxabs_##SUF(const T* f, int ny, int nz, const int* box, unsigned int* out, void* s) { \
    Box3 b = make_box(box);                                                                                   \
    if (box_empty(b)) return 0;                                                                               \
    long long n = (long long)(b.hi[0] - b.lo[0]) * (b.hi[1] - b.lo[1]) * (b.hi[2] - b.lo[2]);                \
    k_box_maxabs<T><<<reduce_grid(n), 256, 0, (hipStream_t)s>>>(f, ny, nz, b, out);                            \
    FDTD_RETURN_LAUNCH_STATUS();                                                                              \
  }                                                                                                           \
  FDTD_API int fdtd_amplitude_update_##SUF(const T* f, T* amp, int ny, int nz, const int* box,                \
                                           double accuracy, unsigned int* changed, void* s) {                 \
    Box3 b = make_box(box);                                                                                   \
    if (box_empty(b)) return 0;                                                                               \
    long long n = (long long)(b.hi[0] - b.lo[0]) * (b.hi[1] - b.lo[1]) * (b.hi[2] - b.lo[2]);                \
    k_amplitude_update<T><<<reduce_grid(n), 256, 0, (hipStream_t)s>>>(f, amp, ny, nz, b, accuracy, changed);   \
    FDTD_RETURN_LAUNCH_STATUS();                                                                              \
  }

FDTD_AUX_API(f32, float)
FDTD_AUX_API(f64, double)

// k_box_list over a device table of n BoxEnt entries (nblocks = the last
// entry's blk0 + its blocks): pack (arrays -> buffers) or unpack
#define FDTD_BOX_LIST_API(SUF, T)                                                                            \
  FDTD_API int fdtd_box_list_##SUF(const void* tab, int n, int nblocks, int pack, void* s) {                  \
    if (n <= 0 || nblocks <= 0) return 0;                                                                     \
    if (pack)                                                                                                 \
      k_box_list<T, true><<<nblocks, 256, 0, (hipStream_t)s>>>((const BoxEnt*)tab, n);                       \
    else                                                                                                      \
      k_box_list<T, false><<<nblocks, 256, 0, (hipStream_t)s>>>((const BoxEnt*)tab, n);                      \
    FDTD_RETURN_LAUNCH_STATUS();                                                                              \
  }
FDTD_BOX_LIST_API(f32, float)
FDTD_BOX_LIST_API(f64, double)
FDTD_API int fdtd_box_ent_size() { return (int)sizeof(BoxEnt); }

template <typename T>
int amplitude_many(const void* const* f, void* const* amp, int ncomp, int ny, int nz, const int* boxes,
                   long long amp_xs, double accuracy, unsigned int* changed, hipStream_t s) {
  if (ncomp <= 0 || ncomp > 6) return (int)hipErrorInvalidValue;
  AmpSet a;
  a.xs = amp_xs > 0 ? amp_xs : (long long)ny * nz;
  long long nmax = 0;
  for (int c = 0; c < 6; ++c) {
    a.f[c] = c < ncomp ? f[c] : nullptr;
    a.amp[c] = c < ncomp ? amp[c] : nullptr;
    a.b[c] = c < ncomp ? make_box(boxes + 6 * c) : Box3{{0, 0, 0}, {0, 0, 0}};
    if (c < ncomp && !box_empty(a.b[c])) {
      const Box3& b = a.b[c];
      const long long n = (long long)(b.hi[0] - b.lo[0]) * (b.hi[1] - b.lo[1]) * (b.hi[2] - b.lo[2]);
      nmax = n > nmax ? n : nmax;
    }
  }
  if (nmax == 0) return 0;
  Box3 u = {{0, 0, 0}, {0, 0, 0}};
  bool first = true;
  for (int c = 0; c < ncomp; ++c) {
    if (box_empty(a.b[c])) continue;
    u = first ? a.b[c] : box_union(u, a.b[c]);
    first = false;
  }
  if (sizeof(T) == 4 && nz % 4 == 0) {
    bool al = true;
    for (int c = 0; c < ncomp; ++c) al = al && ((uintptr_t)a.f[c] % 16 == 0) && ((uintptr_t)a.amp[c] % 16 == 0);
    if (al) {
      const int kspan = u.hi[2] - (u.lo[2] & ~3);
      const dim3 g4((unsigned)cdiv(kspan, 256), (unsigned)cdiv(u.hi[1] - u.lo[1], 4), (unsigned)(u.hi[0] - u.lo[0]));
      k_amplitude_many_v4<<<g4, dim3(64, 4), 0, s>>>(a, ncomp, u, ny, nz, (float)accuracy, changed);
      FDTD_RETURN_LAUNCH_STATUS();
    }
  }
  const dim3 grid((unsigned)cdiv(u.hi[2] - u.lo[2], 64), (unsigned)cdiv(u.hi[1] - u.lo[1], 4),
                  (unsigned)(u.hi[0] - u.lo[0]));
  k_amplitude_many<T><<<grid, dim3(64, 4), 0, s>>>(a, ncomp, u, ny, nz, accuracy, changed);
  FDTD_RETURN_LAUNCH_STATUS();
}

// amplitude update of up to 6 components in one launch, the count of changed
// cells ADDED to *changed (no reset, no host read: models/scheme.py reads a
// whole check period's counters at once)
// ``amp_xs``: x stride of the amp arrays in elements (0: ny * nz, contiguous)
FDTD_API int fdtd_amplitude_many_f32(const void* const* f, void* const* amp, int ncomp, int ny, int nz,
                                     const int* boxes, long long amp_xs, double accuracy, unsigned int* changed,
                                     void* s) {
  return amplitude_many<float>(f, amp, ncomp, ny, nz, boxes, amp_xs, accuracy, changed, (hipStream_t)s);
}
FDTD_API int fdtd_amplitude_many_f64(const void* const* f, void* const* amp, int ncomp, int ny, int nz,
                                     const int* boxes, long long amp_xs, double accuracy, unsigned int* changed,
                                     void* s) {
  return amplitude_many<double>(f, amp, ncomp, ny, nz, boxes, amp_xs, accuracy, changed, (hipStream_t)s);
}

FDTD_API int fdtd_counter_add(int* counter, int n, void* s) {
  k_counter_add<<<1, 64, 0, (hipStream_t)s>>>(counter, n);
  FDTD_RETURN_LAUNCH_STATUS();
}

FDTD_API int fdtd_abi_version() { return 2; }
