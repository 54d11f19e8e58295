// rt_types.h — the FP64 vector TYPES of the ray-trace path: storage only
// (x, y, z), no arithmetic.  Shared by the host loader's scene model
// (csrc/host/scene_model.h), the product's math (rt_math.h: glm 0.9.8.4
// operation order) and the CPU oracle, whose arithmetic is its own
// (oracle/glm_restated.h).
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline
#endif

namespace rtm {

struct dvec2 {
  double x, y;
};

struct dvec3 {
  double x, y, z;
  RT_HD double operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};

RT_HD dvec3 mk3(double x, double y, double z) { dvec3 r; r.x = x; r.y = y; r.z = z; return r; }
RT_HD dvec2 mk2(double x, double y) { dvec2 r; r.x = x; r.y = y; return r; }

}  // namespace rtm
