// float4 (16-byte lane) helpers shared by the fp32 3D Yee kernels.
#pragma once

#include "common.h"

namespace {

__device__ __forceinline__ unsigned kmask(const Box3& b, int j, int kb) {
  if (j < b.lo[1] || j >= b.hi[1]) return 0u;
  unsigned m = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) m |= ((kb + e >= b.lo[2]) && (kb + e < b.hi[2])) ? (1u << e) : 0u;
  return m;
}

__device__ __forceinline__ float f4(const float4& v, int e) {
  return e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w));
}

__device__ __forceinline__ void f4set(float4& v, int e, float s) {
  if (e == 0) v.x = s;
  else if (e == 1) v.y = s;
  else if (e == 2) v.z = s;
  else v.w = s;
}

__device__ __forceinline__ float4 ld4(const float* p, size_t off) {
  return *reinterpret_cast<const float4*>(p + off);
}

__device__ __forceinline__ void st4(float* p, size_t off, const float4& v) {
  *reinterpret_cast<float4*>(p + off) = v;
}

// store the elements selected by `mask` (bit e = element e); one 16-byte
// store in the common all-inside case
__device__ __forceinline__ void st4m(float* p, size_t off, const float4& v, unsigned mask) {
  if (mask == 0xFu) {
    st4(p, off, v);
  } else if (mask) {
    if (mask & 1u) p[off] = v.x;
    if (mask & 2u) p[off + 1] = v.y;
    if (mask & 4u) p[off + 2] = v.z;
    if (mask & 8u) p[off + 3] = v.w;
  }
}

// fp64 twins: the same 4-cell z groups per lane, 32 bytes (two 16-byte
// accesses); offsets of whole groups are 32-byte aligned
__device__ __forceinline__ double f4(const double4& v, int e) {
  return e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w));
}

__device__ __forceinline__ void f4set(double4& v, int e, double s) {
  if (e == 0) v.x = s;
  else if (e == 1) v.y = s;
  else if (e == 2) v.z = s;
  else v.w = s;
}

__device__ __forceinline__ double4 ld4(const double* p, size_t off) {
  const double2 a = *reinterpret_cast<const double2*>(p + off);
  const double2 b = *reinterpret_cast<const double2*>(p + off + 2);
  return make_double4(a.x, a.y, b.x, b.y);
}

__device__ __forceinline__ void st4(double* p, size_t off, const double4& v) {
  *reinterpret_cast<double2*>(p + off) = make_double2(v.x, v.y);
  *reinterpret_cast<double2*>(p + off + 2) = make_double2(v.z, v.w);
}

__device__ __forceinline__ void st4m(double* p, size_t off, const double4& v, unsigned mask) {
  if (mask == 0xFu) {
    st4(p, off, v);
  } else if (mask) {
    if (mask & 1u) p[off] = v.x;
    if (mask & 2u) p[off + 1] = v.y;
    if (mask & 4u) p[off + 2] = v.z;
    if (mask & 8u) p[off + 3] = v.w;
  }
}

// the 4-lane vector of an element type
template <typename T>
struct Vec4;
template <>
struct Vec4<float> {
  using type = float4;
  static __device__ __forceinline__ float4 make(float a, float b, float c, float d) {
    return make_float4(a, b, c, d);
  }
};
template <>
struct Vec4<double> {
  using type = double4;
  static __device__ __forceinline__ double4 make(double a, double b, double c, double d) {
    return make_double4(a, b, c, d);
  }
};

}  // namespace
