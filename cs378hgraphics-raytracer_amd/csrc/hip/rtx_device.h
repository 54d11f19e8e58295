// rtx_device.h — gfx950 device code for the ray-trace hot path.
//
// Per-lane FP64 arithmetic reproduces the reference operation for operation
// (see rt_math.h for the glm 0.9.8 order); the control structure is the
// GPU's own:
//   * iterative two-level BVH traversal with an explicit per-lane stack in
//     LDS (stack[depth*64 + lane]: conflict-free ds_read/ds_write_b32),
//   * closest-hit = lexicographic min of (t, DFS rank) — the winner the
//     reference's "first strict '<' in candidate order" produces
//     (scene.cpp:157-180, trimesh.cpp:79-95) — with conservative t-pruning,
//   * shadow rays walk the reference's sorted all-hits list one hit at a
//     time: next = min (t, object rank, sub-index) > previous key, which is
//     the order libstdc++ std::sort (insertion sort for <= 16 hits, stable)
//     gives the list built in candidate order (light.cpp:21-53),
//   * recursion (RayTracer.cpp:108-174) becomes a per-lane stack of pending
//     rays carrying their path weight.
#pragma once

#include <hip/hip_runtime.h>

#include "../common/rt_math.h"
#include "rtx.h"

// RtxObject.pad slots the device copy of an object carries:
//   WOPAQUE   the object is opaque to shadow walks (rtx_scene_create; walk_hit)
//   FACE_OFF, NODE_OFF, VERT_OFF, MFLAGS: a trimesh's RtxMesh fields
//             (face_off, node_off, vert_off; MFLAGS bit 0 node_count > 0,
//             bit 1 has_normals, bit 2 has_vmats), so the traversal's mesh
//             entry and resolve_hit read them with the object record instead
//             of a dependent load of the mesh record (augment_objects,
//             rtx_traverse.h)
#define RTX_OBJ_WOPAQUE 0
#define RTX_OBJ_FACE_OFF 1
#define RTX_OBJ_NODE_OFF 2
#define RTX_OBJ_VERT_OFF 3
#define RTX_OBJ_MFLAGS 4
#define RTX_MESH_TREE 1
#define RTX_MESH_NORMALS 2
#define RTX_MESH_VMATS 4

namespace rtxd {

// Materialise loaded values here (an empty asm that uses them): the loads
// of a record, box or face are issued as one burst and waited for once,
// instead of the compiler sinking each into the branch that first needs it
// (one dependent round trip per branch for a wave stepping alone).  Device
// code only; the host build of the traversal (tests/native) has no VGPRs.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void pin(double x) { asm volatile("" ::"v"(x)); }
__device__ __forceinline__ void pin(float x) { asm volatile("" ::"v"(x)); }
__device__ __forceinline__ void pin(int x) { asm volatile("" ::"v"(x)); }
// no instruction moves across this point (the AMDGPU scheduler): loads
// issued above stay issued before the arithmetic below, which then runs
// while they are in flight
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }
#else
inline void pin(double) {}
inline void pin(float) {}
inline void pin(int) {}
inline void sched_fence() {}
#endif

using rtm::dvec2;
using rtm::dvec3;
using rtm::mk3;

#define RTX_RAY_EPS 0.00000001           // scene/ray.h:136
#define RTX_EPS32 (0.00000001 / 32)      // util.h:7,9 ZCHK / BTTC
#define RTX_EPS_BACKUP 0.0000000001      // light.cpp:13
#define RTX_INF 1.0e308
#define RTX_MAX_LIGHTS 64

// Device BVH layout (built from the RtxNode arrays by rtx_scene_create): the
// reference's binary KdTree collapsed to 4-wide records.  A record stands
// for one internal node and holds the boxes of its children, where an
// internal child is replaced by ITS two children (so 2..4 entries): one
// 128-byte line tests up to four boxes and the walk needs half as many
// dependent fetches as on the binary tree.
//
// Exactness.  Node boxes are merges of their children's (kdTree.h:30-39) and
// the slab test (bbox.cc:33-70) is monotone under box containment in
// floating point too (per axis, (lo - o) / d rounds monotonically), so a box
// is only ever hit when its ancestors' are: the reference's candidates are
// exactly the faces whose LEAF box passes the exact slab test (and the
// objects whose world box does — Geometry::intersect re-tests it).  Internal
// boxes therefore only steer the walk, and any test that never rejects a
// box the exact one accepts is as good.  The records store them as floats
// rounded outward (a superset box) tested conservatively in float
// (box_cons32); the exact test runs where it decides a result: on each
// object's world box and on the leaf box of every face hit that would enter the answer (leaf_ok).
// child[k] >= 0: index of the child's record; child[k] < 0: the child is a
// leaf, ~child[k] = first_item << 2 | count (count 1..3, kdTree.h:6).  Item
// ranks (DFS-leaf order) are unchanged, so the winner of the lexicographic
// (t, rank) minimum does not depend on the visiting order.
struct DevNode4 {
  float lo[3][4];      // [axis][entry], rounded down
  float hi[3][4];      // [axis][entry], rounded up
  int32_t child[4];
  int32_t count;       // entries, 2..4
  int32_t pad[3];
};                     // 128 bytes

// Root of a BVH (scene or one mesh): its own box + the reference to descend.
struct DevRoot {
  double lo[3], hi[3];
  int32_t ref;         // >= 0: DevNode4 index; < 0: the root is a leaf (~code)
  int32_t pad[3];
};                     // 64 bytes

// Per face in traversal-tree leaf order (tfaces): its reference rank (index
// in faces / fids) and its reference leaf node (global index in mnodes) —
// loaded with the face, so leaf_ok needs one dependent load (the leaf box),
// not three (rank, face ids, leaf box).
struct TMeta {
  int32_t rank, leaf;
};

struct DevScene {
  const DevNode4* snode4;  // scene BVH records
  const DevNode4* mnode4;  // all mesh BVHs' records (global indices)
  const DevRoot* mroots;   // per mesh (valid when meshes[m].node_count > 0)
  DevRoot sroot;           // scene BVH root
  const RtxNode* snodes;
  const RtxObject* objs;
  const double* oprm;      // RTX_OBJ_PARAMS per object (cone shapes)
  const RtxMaterial* mats;
  const RtxMesh* meshes;
  const RtxNode* mnodes;
  const RtxFace* faces;
  const RtxFaceIds* fids;
  const RtxFace* tfaces;   // faces in traversal-tree leaf order (per mesh)
  const int32_t* trank;    // reference rank (index in faces) of each tfaces entry
  const TMeta* tmeta;      // rank + reference leaf node of each tfaces entry
  const double* vnormals;
  const RtxVertexMaterial* vmats;
  const RtxLight* lights;
  const RtxTexture* texs;
  const uint8_t* texels;
  const double* picks;   // area-light sample positions [light][ss_res][3]
  int32_t n_snodes, n_objs, n_lights, ss_res;
  int32_t n_srec;        // scene-tree records
  double margin;         // world-space pruning slack
  double lmargin;        // mesh-local pruning slack
  double cos45;          // glm::cos(PI / 4) computed on the host (light.cpp:145)
  double ambient[3];
  double air_index;      // intensityValue of air's index (material.cpp:17-21)
  int32_t skip_dark;     // shadow queries whose colour factor is exactly 0 may be skipped
  int32_t cube[6];       // cube-map face textures (+x,-x,+y,-y,+z,-z); cube[0] < 0: none
};

struct Counters {
  int64_t camera, secondary, shadow, nodes, objects, tris, shades, shadow_traced;
  int64_t queries;  // traversal queries started (trav_init): per-kernel work (rtx_last_work)
};

__host__ __device__ __forceinline__ dvec3 ld3(const double* p) { return mk3(p[0], p[1], p[2]); }

// Cone quadric in the object frame (Cone.cpp:19-37): coefficients and the
// two roots in the reference's names (nearRoot = (-b + sqrt) / 2a).
struct ConeRoots {
  double near_t, far_t;
  bool ok;  // a != 0 and discriminant > 0
};
__host__ __device__ __forceinline__ ConeRoots cone_roots(const double* prm, const dvec3& R0, const dvec3& Rd) {
  const double b2 = prm[RTX_CONE_B2], g = prm[RTX_CONE_G];
  ConeRoots cr;
  cr.near_t = cr.far_t = 0.0;
  cr.ok = false;
  const double a = Rd.x * Rd.x + Rd.y * Rd.y - b2 * Rd.z * Rd.z;
  if (a == 0.0) return cr;
  const double b = 2 * (R0.x * Rd.x + R0.y * Rd.y - b2 * ((R0.z + g) * Rd.z));
  const double c = -b2 * (g + R0.z) * (g + R0.z) + R0.x * R0.x + R0.y * R0.y;
  double disc = b * b - 4 * a * c;
  if (disc <= 0) return cr;
  disc = sqrt(disc);
  cr.near_t = (-b + disc) / (2 * a);
  cr.far_t = (-b - disc) / (2 * a);
  cr.ok = true;
  return cr;
}
// Cone::isGoodRoot (Cone.cpp:212-218)
__host__ __device__ __forceinline__ bool cone_good(const double* prm, const dvec3& P) {
  return !(P.z < 0 || P.z > prm[RTX_CONE_H]);
}

// Geometry::intersect's ray into the object frame (scene.cpp:17-19): pos =
// M^-1 (p, 1), dir = M^-1 (p + d, 1) - pos (not yet normalised).  (A
// shortcut for identity transforms measured slower: DESIGN.md §8, round 5.)
RT_HD void obj_local(const RtxObject& o, const dvec3& P, const dvec3& D, dvec3& pos, dvec3& dir) {
  pos = rtm::xform_point(o.inv, P);
  dir = rtm::xform_point(o.inv, P + D) - pos;
}

// ------------------------------------------------------------------ slab
// BoundingBox::intersect (bbox.cc:33-70), exact: same divisions, same
// vd == 0 skip, same per-axis early outs.  Also returns tMin/tMax.
// Branch-free form of bbox.cc's loop: the box is loaded whole before any
// test (per-axis branches made each axis's loads a dependent round trip),
// a d[a] == 0 axis is selected away instead of skipped, and the per-axis
// early outs are decided once at the end — tMin only grows and tMax only
// shrinks, so an early out taken at some axis holds at the end too, and the
// comparisons are bbox.cc's own (NaN behaves the same).
RT_HD bool slab(const double* bmin, const double* bmax, const dvec3& o, const dvec3& d,
                                     double& tMinOut, double& tMaxOut) {
  const double lo[3] = {bmin[0], bmin[1], bmin[2]}, hi[3] = {bmax[0], bmax[1], bmax[2]};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    pin(lo[a]);
    pin(hi[a]);
  }
  double tMin = -1.0e308, tMax = 1.0e308;
  bool out = false;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double vd = rtm::get(d, a);
    const double oa = rtm::get(o, a);
    const double u1 = (lo[a] - oa) / vd;
    const double u2 = (hi[a] - oa) / vd;
    const bool sw = u1 > u2;
    const double t1 = sw ? u2 : u1, t2 = sw ? u1 : u2;
    const bool on = !(vd == 0.0);
    tMin = on && t1 > tMin ? t1 : tMin;
    tMax = on && t2 < tMax ? t2 : tMax;
    out = out || (on && (tMin > tMax || tMax < RTX_RAY_EPS));
  }
  if (out) return false;
  tMinOut = tMin;
  tMaxOut = tMax;
  return true;
}

// Fast slab for traversal: multiplies by the ray's reciprocal direction
// (3 divisions per ray instead of 6 per box) and only falls back to the exact
// slab() when the rounded answer could differ from it.  (lo - o) is the same
// in both; x * fl(1/d) differs from fl(x / d) by <= 3 ulp relative, so a
// margin of 1e-15 relative on tMin/tMax separates certain hits and certain
// misses from the rare ambiguous case.  Per-axis early outs of bbox.cc are
// monotone (tMin only grows, tMax only shrinks), so deciding once at the end
// is the same test.  `fast` is false when a direction component is so small
// that 1/d overflows; then every box goes through slab().
struct RayInv {
  dvec3 inv;
  bool fast;
};

// ray_inv's fast flag: no component tiny but nonzero (1 / d past 1e290)
RT_HD bool ray_inv_fast(const dvec3& d) {
  bool f = true;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double v = rtm::get(d, a);
    if (v != 0.0 && fabs(v) < 1e-290) f = false;
  }
  return f;
}

RT_HD RayInv ray_inv(const dvec3& d) {
  RayInv r;
  r.fast = true;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double v = rtm::get(d, a);
    if (v != 0.0 && fabs(v) < 1e-290) r.fast = false;
    rtm::set(r.inv, a, v == 0.0 ? 0.0 : 1.0 / v);
  }
  return r;
}

RT_HD bool box_test(const double* lo, const double* hi, const dvec3& o, const dvec3& d,
                                         const RayInv& ri, double& a, double& b) {
  if (!ri.fast) return slab(lo, hi, o, d, a, b);
  // the box whole, then the axes branch-free (a d[k] == 0 axis selected away)
  const double l[3] = {lo[0], lo[1], lo[2]}, h[3] = {hi[0], hi[1], hi[2]};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    pin(l[k]);
    pin(h[k]);
  }
  double tmin = -1.0e308, tmax = 1.0e308;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double iv = rtm::get(ri.inv, k), oa = rtm::get(o, k);
    const double t1 = (l[k] - oa) * iv;
    const double t2 = (h[k] - oa) * iv;
    const bool on = !(rtm::get(d, k) == 0.0);
    tmin = on ? fmax(tmin, fmin(t1, t2)) : tmin;
    tmax = on ? fmin(tmax, fmax(t1, t2)) : tmax;
  }
  const double e1 = 1e-15 * fabs(tmin) + 1e-300, e2 = 1e-15 * fabs(tmax) + 1e-300;
  if (tmin - e1 > tmax + e2 || tmax + e2 < RTX_RAY_EPS) return false;  // certain miss
  if (tmin + e1 <= tmax - e2 && tmax - e2 >= RTX_RAY_EPS) {             // certain hit
    a = tmin;
    b = tmax;
    return true;
  }
  return slab(lo, hi, o, d, a, b);
}

// the next float toward +inf (finite f; nextafterf has no device version)
RT_HD float f_succ(float f) {
  if (f == 0.0f) return 0x1p-149f;
  const uint32_t u = __builtin_bit_cast(uint32_t, f);
  return __builtin_bit_cast(float, f > 0.0f ? u + 1u : u - 1u);
}
// a float >= x / <= x (x itself when representable)
RT_HD float f_up(double x) {
  float f = static_cast<float>(x);
  if (static_cast<double>(f) < x) f = f_succ(f);
  return f;
}
RT_HD float f_down(double x) {
  float f = static_cast<float>(x);
  if (static_cast<double>(f) > x) f = -f_succ(-f);
  return f;
}
// A float >= x / <= x in four instructions instead of f_up's nine (cvt, fma,
// max, add; the record walk widens its prune bounds with these on every record
// step): the nearest float h of x, moved out by |h| 2^-22 and the smallest
// normal float.  h is within |x| 2^-24 of x and the fma's rounding within
// |h| 2^-24 of its exact value, so the sum clears x by at least |h| 2^-23
// (h != 0), and by 2^-126 when h is 0 or flushed; +-inf stay +-inf.  At most
// a few ulps wider than f_up / f_down: the walk only visits slightly more
// (tests/test_record_test_host.py checks x <= up and dn <= x).
RT_HD float f_up_wide(double x) {
  const float h = static_cast<float>(x);
  // (x below -FLT_MAX: h = -inf and the fma NaN; fmax gives -FLT_MAX >= x)
  return fmaxf(fmaf(fabsf(h), 0x1p-22f, h), -3.40282347e38f) + 0x1p-126f;
}
RT_HD float f_down_wide(double x) {
  const float h = static_cast<float>(x);
  return fminf(fmaf(-fabsf(h), 0x1p-22f, h), 3.40282347e38f) - 0x1p-126f;
}

// Float copy of a ray for the record tests (box_cons32): origin and
// reciprocal direction rounded to float, and an absolute bound `err` of the
// error of every per-axis slab distance computed from them in float:
//   t = fl(fl(lo - fl(o)) * fl(1/d)) = (lo - o)/d + (o - fl(o))/d, times
//   (1 + eta) with |eta| <= 3.01 * 2^-24, so |t - t_exact| <= 1.01 |o / d|
//   2^-24 + 3.1 2^-24 |t|.  err = 2^-22 max_q |o_q / d_q| and the relative
//   2^-21 |t| applied to the result cover that with room (and the 2^-52
//   relative error of the double slab the exact test computes).
// An axis with d == 0 is an inside test instead: inv = +inf, the entry
// side's origin rounded up past o and the exit side's down (olo > o > ohi
// strictly), so its slab is (-inf, +inf) when lo <= o <= hi and empty
// otherwise.  That is NOT bbox.cc's rule (it skips the axis) but the
// conservative one for the device's own trees: their boxes only steer the
// walk and must contain every hit point, and a hit of such a ray has
// P.x == o.x exactly (DESIGN.md "Float record tests").  Skipping the axis
// made every such ray — the image column whose direction has x == 0 — visit
// thousands of records.  A nonzero d whose 1/d is past the float range
// (|d| < 3.4e-39) is skipped (olo = +inf, ohi = -inf: the slab is
// (-inf, +inf)): its hit points drift off o.x by t |d|, which an inside test
// would not cover at large t.
struct RayF {
  float olo[3], ohi[3], inv[3];
  float err;
};

RT_HD RayF ray_f(const dvec3& o, const dvec3& d, const RayInv& ri) {
  RayF r;
  double e = 0.0;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double da = rtm::get(d, a), oa = rtm::get(o, a);
    const double inv = rtm::get(ri.inv, a);  // 1 / da (ray_inv), 0 for da == 0
    if (da == 0.0) {
      const double dl = fabs(oa) * 0x1p-23 + 1e-30;
      r.olo[a] = f_up(oa + dl);
      r.ohi[a] = f_down(oa - dl);
      r.inv[a] = __builtin_inff();
      continue;
    }
    if (!(fabs(inv) < 3.0e38)) {  // tiny nonzero d: no slab on this axis
      r.olo[a] = __builtin_inff();
      r.ohi[a] = -__builtin_inff();
      r.inv[a] = __builtin_inff();
      continue;
    }
    r.olo[a] = r.ohi[a] = static_cast<float>(oa);
    r.inv[a] = static_cast<float>(inv);
    const double ea = fabs(oa * inv);
    e = ea > e ? ea : e;
  }
  r.err = f_up(e * 0x1p-22);
  return r;
}

// Conservative slab of a record entry in float (see RayF): never rejects a
// box containing a hit point of the ray; a <= the entry distance, b >= the
// exit distance.
// (the entry's six bounds as values: visit4 loads the whole record first)
RT_HD bool box_cons32v(float lox, float loy, float loz, float hix, float hiy, float hiz, const RayF& r, float& a,
                       float& b) {
  const float t1x = (lox - r.olo[0]) * r.inv[0], t2x = (hix - r.ohi[0]) * r.inv[0];
  const float t1y = (loy - r.olo[1]) * r.inv[1], t2y = (hiy - r.ohi[1]) * r.inv[1];
  const float t1z = (loz - r.olo[2]) * r.inv[2], t2z = (hiz - r.ohi[2]) * r.inv[2];
  const float tmin = fmaxf(fmaxf(fminf(t1x, t2x), fminf(t1y, t2y)), fminf(t1z, t2z));
  const float tmax = fminf(fminf(fmaxf(t1x, t2x), fmaxf(t1y, t2y)), fmaxf(t1z, t2z));
  // (err is finite; an infinite bound stays infinite)
  a = tmin - (r.err + fabsf(tmin) * 0x1p-21f);
  b = tmax + (r.err + fabsf(tmax) * 0x1p-21f);
  // tmin is finite or +inf and tmax finite or -inf (a ray has a nonzero
  // direction axis, whose slab is finite); the infinities come from
  // inside-test axes that miss, and give a = NaN (inf - inf) or b = NaN.
  // The ordered compares below are false on NaN: a miss, as it must be, with
  // no fix-up of a and b (a and b are used only on a hit).
  // (no 1e-8 cut on the exit, as the double slab had none here; leaf_ok
  // applies the reference's)
  return a <= b && b >= 0.0f;
}

RT_HD bool box_cons32(const DevNode4& nd, int k, const RayF& r, float& a, float& b) {
  return box_cons32v(nd.lo[0][k], nd.lo[1][k], nd.lo[2][k], nd.hi[0][k], nd.hi[1][k], nd.hi[2][k], r, a, b);
}


// ------------------------------------------------------------------ textures
// TextureMap::getMappedValue / getPixelAt (material.cpp:84-138)
__device__ __forceinline__ dvec3 tex_pixel(const DevScene& S, const RtxTexture& t, int x, int y) {
  if (0 <= x && x < t.width && 0 <= y && y < t.height) {
    const uint8_t* p = S.texels + t.offset + (size_t(x) + size_t(y) * t.width) * 3;
    return mk3(double(p[0]), double(p[1]), double(p[2]));
  }
  return mk3(0.0, 0.0, 0.0);
}

// noinline: one out-of-line copy instead of one inlined copy per material
// parameter (textures are rare; the register peak of the shading kernel
// must not carry eight bilinear lookups)
__device__ __noinline__ dvec3 tex_lookup(const DevScene& S, int tex, const dvec2& uv) {
  const RtxTexture t = S.texs[tex];
  double x = uv.x, y = uv.y;
  if (0.0 <= x && x <= 1.0 && 0.0 <= y && y <= 1.0) {
    x *= t.width - 1;
    y *= t.height - 1;
    int ix = (int)x, iy = (int)y;
    x -= ix;
    y -= iy;
    dvec3 prows[2];
#pragma unroll
    for (int i = 0; i < 2; i++) {
      dvec3 pl = tex_pixel(S, t, i + ix, 0 + iy);
      dvec3 pr = tex_pixel(S, t, i + ix, 1 + iy);
      prows[i] = y * (pr - pl) + pl;
    }
    return (x * (prows[1] - prows[0]) + prows[0]) / 255.0;
  }
  return mk3(0.0, 1.0, 0.0);
}

// CubeMap::getColor (cubeMap.cpp:12-44): the colour of a ray that hits
// nothing.  With |x| == |y| == |z| no face branch is taken; the reference then
// reads an uninitialised face index (decision U24: face 0, d = (0, 0)).
__device__ __noinline__ dvec3 cube_color(const DevScene& S, const dvec3 rd) {
  const double ax = fabs(rd.x), ay = fabs(rd.y), az = fabs(rd.z);
  const bool xy = ax >= ay, yz = ay >= az, zx = az >= ax;
  int map = 0;
  double scale = 0.5;
  dvec2 d = rtm::mk2(0.0, 0.0);
  if (xy && !zx) {  // x direction
    scale /= ax;
    d = rtm::mk2(rd.x > 0 ? rd.z : -rd.z, rd.y);
    map = rd.x > 0 ? 0 : 1;
  } else if (yz && !xy) {  // y direction
    scale /= ay;
    d = rtm::mk2(rd.x, rd.y > 0 ? rd.z : -rd.z);
    map = rd.y > 0 ? 2 : 3;
  } else if (zx && !yz) {  // z direction
    scale /= az;
    d = rtm::mk2(rd.z > 0 ? rd.x : -rd.x, rd.y);
    map = rd.z > 0 ? 4 : 5;
  }
  d = rtm::mk2(d.x * scale + 0.5, d.y * scale + 0.5);
  return tex_lookup(S, S.cube[map], d);
}

// MaterialParameter::value / intensityValue (material.cpp:140-158)
__device__ __forceinline__ dvec3 pval(const DevScene& S, const RtxParam& p, const dvec2& uv) {
  if (p.tex >= 0) return tex_lookup(S, p.tex, uv);
  return ld3(p.v);
}
__device__ __forceinline__ double intensity(const dvec3& v) { return (0.299 * v.x) + (0.587 * v.y) + (0.114 * v.z); }

// A material evaluated at one hit (all parameters looked up once).
struct EvalMat {
  dvec3 ke, ka, ks, kd, kr, kt;
  double sh, index;
  int flags;
};

__device__ EvalMat eval_material(const DevScene& S, const RtxMaterial& m, const dvec2& uv) {
  EvalMat e;
  e.ke = pval(S, m.p[RTX_P_KE], uv);
  e.ka = pval(S, m.p[RTX_P_KA], uv);
  e.ks = pval(S, m.p[RTX_P_KS], uv);
  e.kd = pval(S, m.p[RTX_P_KD], uv);
  e.kr = pval(S, m.p[RTX_P_KR], uv);
  e.kt = pval(S, m.p[RTX_P_KT], uv);
  const RtxParam& shp = m.p[RTX_P_SHININESS];
  e.sh = shp.tex >= 0 ? 128.0 * intensity(pval(S, shp, uv)) : intensity(ld3(shp.v));  // material.h:204-209
  e.index = intensity(pval(S, m.p[RTX_P_INDEX], uv));
  e.flags = m.flags;
  return e;
}

// Interpolated per-vertex material (trimesh.cpp:157-163): Material() +=
// b_k * M_k.  Decision U2: flags all false.
__device__ EvalMat eval_vertex_material(const DevScene& S, const RtxMesh& me, const RtxFaceIds& fi,
                                        const dvec3& bary) {
  EvalMat e;
  dvec3 z = mk3(0.0, 0.0, 0.0);
  e.ke = z; e.ka = z; e.ks = z; e.kd = z; e.kr = z; e.kt = z;
  dvec3 shv = z, idx = mk3(1.0, 1.0, 1.0);
  const double bw[3] = {bary.x, bary.y, bary.z};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const RtxVertexMaterial& vm = S.vmats[me.vert_off + fi.vi[k]];
    e.ke += ld3(vm.ke) * bw[k];
    e.ka += ld3(vm.ka) * bw[k];
    e.ks += ld3(vm.ks) * bw[k];
    e.kd += ld3(vm.kd) * bw[k];
    e.kr += ld3(vm.kr) * bw[k];
    e.kt += ld3(vm.kt) * bw[k];
    shv += ld3(vm.shininess) * bw[k];
    idx += ld3(vm.index) * bw[k];
  }
  e.sh = intensity(shv);
  e.index = intensity(idx);
  e.flags = 0;
  return e;
}

// ------------------------------------------------------------------ resolve helpers
// Box::computeNormal (Box.cpp:99-108)
__device__ dvec3 box_normal(const DevScene& S, const RtxMaterial& m, int bestIndex, const dvec2& uv) {
  dvec3 b = pval(S, m.p[RTX_P_BUMP], uv);
  if (rtm::length(b) > 0.0001) return rtm::normalize(b - mk3(0.5, 0.5, 0.5));
  if (bestIndex < 3) return mk3(-double(bestIndex == 0), -double(bestIndex == 1), -double(bestIndex == 2));
  return mk3(double(bestIndex == 3), double(bestIndex == 4), double(bestIndex == 5));
}

// ------------------------------------------------------------------ primitives, closest hit
// TrimeshFace::intersectLocal (trimesh.cpp:119-156) up to the barycentric
// denominators; the barycentrics are computed for the winner only.
// tcap: callers pass a bound past which the hit cannot matter (see
// traverse); rejecting there only skips work, never changes a result.
// One face's plane and vertices in registers (the leaf loop loads the next
// face's while it tests this one).
struct FaceV {
  dvec3 n, v0, v1, v2;
};
RT_HD FaceV face_ld(const RtxFace& F) { return FaceV{ld3(F.n), ld3(F.v0), ld3(F.v1), ld3(F.v2)}; }
RT_HD void face_pin(const FaceV& q) {
  pin(q.n.x), pin(q.n.y), pin(q.n.z), pin(q.v0.x), pin(q.v0.y), pin(q.v0.z);
  pin(q.v1.x), pin(q.v1.y), pin(q.v1.z), pin(q.v2.x), pin(q.v2.y), pin(q.v2.z);
}
RT_HD bool tri_test(const FaceV& q, const dvec3& p, const dvec3& d, double tcap, double& tOut) {
  const dvec3 n = q.n, v0 = q.v0, v1 = q.v1, v2 = q.v2;
  double t = rtm::dot(n, d);
  if (t < RTX_EPS32 && t > -RTX_EPS32) return false;
  t = rtm::dot(v0 - p, n) / t;
  if (t < RTX_EPS32 || t > tcap) return false;
  const dvec3 P = rtm::ray_at(p, d, t);
  if (rtm::dot(rtm::cross(v1 - v0, P - v0), n) < RTX_EPS32) return false;
  if (rtm::dot(rtm::cross(v2 - v1, P - v1), n) < RTX_EPS32) return false;
  if (rtm::dot(rtm::cross(v0 - v2, P - v2), n) < RTX_EPS32) return false;
  const double faceArea = rtm::dot(rtm::cross(v1 - v0, v2 - v0), n);
  if (faceArea < RTX_EPS32 && faceArea > -RTX_EPS32) return false;
  tOut = t;
  return true;
}
RT_HD bool tri_hit(const RtxFace& F, const dvec3& p, const dvec3& d, double tcap,
                                        double& tOut) {
  // the face whole before the plane test (its vertices used to be loaded
  // after it: a second dependent round trip per face)
  const FaceV q = face_ld(F);
  face_pin(q);
  return tri_test(q, p, d, tcap, tOut);
}

RT_HD dvec3 tri_bary(const RtxFace& F, const dvec3& p, const dvec3& d, double t) {
  const dvec3 n = ld3(F.n);
  const dvec3 v0 = ld3(F.v0), v1 = ld3(F.v1), v2 = ld3(F.v2);
  const dvec3 P = rtm::ray_at(p, d, t);
  const double faceArea = rtm::dot(rtm::cross(v1 - v0, v2 - v0), n);
  const double baryU = rtm::dot(rtm::cross(v1 - P, v2 - P), n);
  const double baryV = rtm::dot(rtm::cross(v2 - P, v0 - P), n);
  dvec3 b = mk3(baryU / faceArea, baryV / faceArea, 0);
  b.z = 1 - b.x - b.y;
  return b;
}

// Lexicographic key order used by both queries.
RT_HD bool key_less(double ta, int ra, int sa, double tb, int rb, int sb) {
  return ta < tb || (ta == tb && (ra < rb || (ra == rb && sa < sb)));
}

}  // namespace rtxd
