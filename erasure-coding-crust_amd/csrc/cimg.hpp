// cimg.hpp — multiply tables from the element-indexed compact image
// (ec_kernels.hpp kCImg*, DevTables::cimg) resident at LDS address 0: the
// n = 1024 encode (enc_k256w.hip), its only user.  Kernels using it declare
// no static LDS (prepare_kernel checks), so the image starts at absolute LDS
// address 0.
#pragma once

#include "ec_device.hpp"
#include "ec_kernels.hpp"

namespace ecamd {
namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4u lds_r128(uint32_t a) {
  return *(const __attribute__((address_space(3))) v4u *)(uintptr_t(a));
}
__device__ __forceinline__ uint32_t lds_r32(uint32_t a) {
  return *(const __attribute__((address_space(3))) uint32_t *)(uintptr_t(a));
}

// Table of element x = (lane part) ^ (uniform part) from the compact image at
// LDS address 0 (the kernel has no static LDS): lt = cimg_lin(lane part),
// u = cimg_lin(uniform part).  The table type is the element's kind; the
// kind's bit (128 / 256) is folded into the uniform part here.  Planes are
// requested last-used first, so the first multiply waits once.
__device__ __forceinline__ void ctab(uint32_t lt, uint32_t u, SubTab &T) {
  const uint32_t a = lt ^ u;  // < 2048
  T.t[4] = lds_r32(a + kCImgSub1);
  const v4u v = lds_r128(a + kCImgSub0);
  T.t[0] = v.x;
  T.t[1] = v.y;
  T.t[2] = v.z;
  T.t[3] = v.w;
}
__device__ __forceinline__ void ctab(uint32_t lt, uint32_t u, F9Tab &T) {
  const uint32_t a = lt ^ u ^ cimg_lin(128);  // < 2048
#pragma unroll
  for (int q = 3; q >= 0; --q) {
    const v4u v = lds_r128(a + kCImgF9 + q * kCImgF9Plane);
    T.t[4 * q] = v.x;
    T.t[4 * q + 1] = v.y;
    T.t[4 * q + 2] = v.z;
    T.t[4 * q + 3] = v.w;
  }
}
__device__ __forceinline__ void ctab(uint32_t lt, uint32_t u, Tab &T) {
  const uint32_t a = lt ^ u ^ cimg_lin(256);  // < 4096
#pragma unroll
  for (int q = 4; q >= 0; --q) {
    const v4u v = lds_r128(a + kCImgGen + q * kCImgGenPlane);
    T.t[4 * q] = v.x;
    T.t[4 * q + 1] = v.y;
    T.t[4 * q + 2] = v.z;
    T.t[4 * q + 3] = v.w;
  }
}

}  // namespace
}  // namespace ecamd
