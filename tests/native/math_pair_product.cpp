// math_pair_product.cpp — TEST HARNESS: the PRODUCT's vector math
// (csrc/common/rt_math.h, glm 0.9.8.4 operation order) behind a flat C entry
// point, linked into one library with math_pair_oracle.cpp (the oracle's own
// restatement, oracle/glm_restated.h) so tests/test_oracle_math.py can
// compare the two bit for bit.  The two headers are never included in one
// translation unit (their operators would collide); this file sees only
// rt_math.h.
#include <cstdint>

#include "../../cs378hgraphics-raytracer_amd/csrc/common/rt_math.h"

using rtm::dvec3;
using rtm::mk3;

extern "C" int math_pair_product(int op, int n, const double* a, const double* b, const double* m, double* out) {
  for (int k = 0; k < n; ++k) {
    const dvec3 x = mk3(a[3 * k], a[3 * k + 1], a[3 * k + 2]);
    const dvec3 y = mk3(b[3 * k], b[3 * k + 1], b[3 * k + 2]);
    const double s = b[3 * k];
    const double* M = m + 16 * k;  // column-major c * 4 + r
    dvec3 r = mk3(0.0, 0.0, 0.0);
    switch (op) {
      case 0: r = x + y; break;
      case 1: r = x - y; break;
      case 2: r = x * y; break;
      case 3: r = x * s; break;
      case 4: r = s * x; break;
      case 5: r = x / s; break;
      case 6: r = -x; break;
      case 7: r.x = rtm::dot(x, y); break;
      case 8: r = rtm::cross(x, y); break;
      case 9: r.x = rtm::length(x); break;
      case 10: r = rtm::normalize(x); break;
      case 11: r.x = rtm::distance(x, y); break;
      case 12: r = rtm::gclamp3(x, 0.0, 1.0); break;
      case 13: r.x = rtm::gclamp(x.x, 0.0, 1.0); break;
      case 14: r = rtm::pow3(x, s); break;
      case 15: {  // the device layout: 12 doubles, m[c * 3 + r] (rows 0..2 of columns 0..3)
        double m12[12];
        for (int c = 0; c < 4; ++c)
          for (int q = 0; q < 3; ++q) m12[c * 3 + q] = M[c * 4 + q];
        r = rtm::xform_point(m12, x);
        break;
      }
      case 16: {
        double m9[9];
        for (int c = 0; c < 3; ++c)
          for (int q = 0; q < 3; ++q) m9[c * 3 + q] = M[c * 4 + q];
        r = rtm::mat3_mul(m9, x);
        break;
      }
      case 17: r.x = rtm::gmax(0.0, x.x); break;
      case 18: r.x = static_cast<double>(rtm::to_byte(x.x)); break;
      case 19: r = rtm::gmax3(rtm::gmin3(x, rtm::splat3(1.0)), rtm::splat3(0.0)); break;
      default: return 1;
    }
    out[3 * k] = r.x;
    out[3 * k + 1] = r.y;
    out[3 * k + 2] = r.z;
  }
  return 0;
}
