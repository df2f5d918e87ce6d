// Shared device/host helpers for librrin_hip (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rrin_hip.h"

namespace rrin {

constexpr int kPadRowsAlign = 16;  // hp = round_up(h,16) + 2
constexpr int kPadColsAlign = 32;  // wp = round_up(w,32) + 64
constexpr int kPadLeft = 32;       // pixel x at column x+32: every 32-px output row segment
                                   // is one whole 128-B line (full-line stores)

__host__ __device__ inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

inline rrin_geom make_geom(int h, int w) {
  rrin_geom g;
  g.h = h;
  g.w = w;
  g.hp = round_up(h, kPadRowsAlign) + 2;
  g.wp = round_up(w, kPadColsAlign) + 2 * kPadLeft;
  g.plane = (int64_t)g.hp * g.wp;
  return g;
}

// Offset (floats) of pixel (y,x) inside a plane.
__host__ __device__ inline int64_t pp_pix(const rrin_geom& g, int y, int x) {
  return (int64_t)(y + 1) * g.wp + (x + kPadLeft);
}

// Pointer to channel c (absolute, view offset applied) of image n.
__host__ __device__ inline float* pp_chan(const rrin_pp& v, int n, int c) {
  return v.base + n * v.img_stride + (int64_t)(v.ch_off + c) * v.g.plane;
}

inline int hip_code(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

}  // namespace rrin
