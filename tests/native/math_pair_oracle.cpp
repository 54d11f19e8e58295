// math_pair_oracle.cpp — TEST HARNESS: the ORACLE's vector math
// (oracle/glm_restated.h) behind the same flat entry point as
// math_pair_product.cpp; this file never sees rt_math.h.
#include <cstdint>

#include "../../oracle/glm_restated.h"

using rtm::dvec3;
using namespace glmr;

extern "C" int math_pair_oracle(int op, int n, const double* a, const double* b, const double* m, double* out) {
  for (int k = 0; k < n; ++k) {
    const dvec3 x = vec3(a[3 * k], a[3 * k + 1], a[3 * k + 2]);
    const dvec3 y = vec3(b[3 * k], b[3 * k + 1], b[3 * k + 2]);
    const double s = b[3 * k];
    const double* M = m + 16 * k;
    dvec3 r = vec3(0.0);
    switch (op) {
      case 0: r = x + y; break;
      case 1: r = x - y; break;
      case 2: r = x * y; break;
      case 3: r = x * s; break;
      case 4: r = s * x; break;
      case 5: r = x / s; break;
      case 6: r = -x; break;
      case 7: r.x = glmr::dot(x, y); break;
      case 8: r = glmr::cross(x, y); break;
      case 9: r.x = glmr::length(x); break;
      case 10: r = glmr::normalize(x); break;
      case 11: r.x = glmr::distance(x, y); break;
      case 12: r = glmr::clamp(x, 0.0, 1.0); break;
      case 13: r.x = glmr::clamp(x.x, 0.0, 1.0); break;
      case 14: r = glmr::pow(x, vec3(s)); break;
      case 15: r = glmr::mat4_mul_point(M, x); break;
      case 16: {
        double m9[9];
        for (int c = 0; c < 3; ++c)
          for (int q = 0; q < 3; ++q) m9[c * 3 + q] = M[c * 4 + q];
        r = glmr::mat3_mul(m9, x);
        break;
      }
      case 17: r.x = glmr::max(0.0, x.x); break;
      case 18: r.x = static_cast<double>(glmr::set_pixel_byte(x.x)); break;
      case 19: r = glmr::max(glmr::min(x, 1.0), 0.0); break;
      default: return 1;
    }
    out[3 * k] = r.x;
    out[3 * k + 1] = r.y;
    out[3 * k + 2] = r.z;
  }
  return 0;
}
