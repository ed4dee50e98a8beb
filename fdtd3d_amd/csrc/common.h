// Shared definitions for the fdtd3d-amd HIP kernels (gfx950 / MI355X).
//
// Layout convention (same as the reference Grid, Source/Grid/Grid.cpp:127-139):
// a field of local shape (nx, ny, nz) is one contiguous array, z fastest,
// linear index  i*ny*nz + j*nz + k.  All kernels take boxes in LOCAL indices;
// the Python/C++ host code maps global computation ranges to local boxes.
#pragma once

#include <cstdlib>

#include <hip/hip_runtime.h>
#include <stdint.h>

#define FDTD_API extern "C" __attribute__((visibility("default")))

struct Box3 {
  int lo[3];
  int hi[3];
};

__device__ __forceinline__ bool in_box(const Box3& b, int i, int j, int k) {
  return i >= b.lo[0] && i < b.hi[0] && j >= b.lo[1] && j < b.hi[1] && k >= b.lo[2] && k < b.hi[2];
}

__host__ __device__ static inline bool box_empty(const Box3& b) {
  return b.hi[0] <= b.lo[0] || b.hi[1] <= b.lo[1] || b.hi[2] <= b.lo[2];
}

__host__ __device__ static inline Box3 box_union(const Box3& a, const Box3& b) {
  if (box_empty(a)) return b;
  if (box_empty(b)) return a;
  Box3 r;
  for (int d = 0; d < 3; ++d) {
    r.lo[d] = a.lo[d] < b.lo[d] ? a.lo[d] : b.lo[d];
    r.hi[d] = a.hi[d] > b.hi[d] ? a.hi[d] : b.hi[d];
  }
  return r;
}

static inline Box3 make_box(const int* lohi) {
  Box3 b;
  for (int d = 0; d < 3; ++d) {
    b.lo[d] = lohi[d];
    b.hi[d] = lohi[3 + d];
  }
  return b;
}

static inline unsigned cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }

// x planes per workgroup of the x-streaming split kernels: 16 (measured best
// on full grids), halved while the launch would hold fewer than 2048
// workgroups -- thin shell / slab windows (hybrid blocking, PML slabs) would
// otherwise leave most CUs idle.  `wg_per_chunk` = workgroups per x chunk.
// x planes per workgroup of the split (per-step) kernels: halve from `base`
// until the launch has FDTD3D_SPLIT_WGS workgroups (default 2048), not below
// FDTD3D_SPLIT_MINXC planes (default 2) -- read once per library at first use
static inline int split_param(int which) {
  static const int wgs = [] {
    const char* e = getenv("FDTD3D_SPLIT_WGS");
    return e && atoi(e) > 0 ? atoi(e) : 2048;
  }();
  static const int mxc = [] {
    const char* e = getenv("FDTD3D_SPLIT_MINXC");
    return e && atoi(e) > 0 ? atoi(e) : 2;
  }();
  return which ? mxc : wgs;
}

static inline int split_xchunk(int nxo, long long wg_per_chunk, int req, int base = 16, int min_xc = 0) {
  if (req > 0) return req;
  if (min_xc <= 0) min_xc = split_param(1);
  const long long target = split_param(0);
  int xc = base;
  while (xc > min_xc && wg_per_chunk * (long long)cdiv(nxo, xc) < target) xc /= 2;
  return xc;
}

#define FDTD_RETURN_LAUNCH_STATUS() return (int)hipGetLastError()
