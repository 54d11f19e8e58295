// rtx_traverse.h — two-level BVH query of the ray-trace hot path (shared by
// every render kernel; also compiled for the host by the traversal unit test,
// tests/native/traverse_host.hip, so its logic can be checked against the CPU
// restatement without a GPU).
#pragma once

#include <climits>
#include <cstring>
#include <vector>

#include "rtx_device.h"

#define Q_NONE 0
#define Q_CLOSEST 1
#define Q_NEXT 2

namespace rtxd {

// Unified query over the two-level BVH.
//   Q_CLOSEST: Scene::intersect (scene.cpp:157-180): min over objects of
//     (t_world, object rank) where each object's t is its own closest hit
//     (Geometry::intersect + intersectLocal; a trimesh reduces its faces by
//     (t_local, face rank) first, trimesh.cpp:79-95).
//   Q_NEXT: the smallest (t_world, object rank, sub) list entry strictly
//     after (tp, rp, sq) with t_world <= tlimit (Scene::intersectList +
//     std::sort, light.cpp:25-26).
// Nodes are skipped only when the exact slab test (bbox.cc:33-70) rejects
// them or when their entry/exit distance proves that nothing inside can
// change the answer (margins in DESIGN.md).
template <bool STATS>
RT_HD bool traverse(const DevScene& S, const int qmode, const dvec3& P, const dvec3& D,
                                         const double tp, const int rp, const int sq, const double tlimit,
                                         double& bt, int& bobj, int& bsub, int* __restrict__ stk, const int lane,
                                         Counters& C) {
  const bool closest = qmode == Q_CLOSEST;
  bt = tlimit;
  bobj = INT_MAX;
  bsub = INT_MAX;
  bool have = false;
  if (S.n_snodes == 0) return false;
  const double tlo = closest ? -RTX_INF : tp - S.margin;
  const RayInv ri = ray_inv(D);
  {  // root box (KdTree::intersectList starts with the root's bbox test)
    if (STATS) C.nodes++;
    double a, b;
    if (!box_test(S.sroot.lo, S.sroot.hi, P, D, ri, a, b) || a > bt + S.margin || b < tlo) return false;
  }
  // ref >= 0: internal DevNode2; ref < 0: leaf ~(first << 2 | count)
  int sp = 0, ref = S.sroot.ref, mode = 0;  // mode: 0 scene BVH, 1 objects of a leaf, 2 mesh BVH
  int oc = 0, oe = 0;
  // mesh context (local frame of object moi)
  dvec3 lp = mk3(0, 0, 0), ld = mk3(0, 0, 0);
  RayInv lri;
  lri.inv = mk3(0, 0, 0);
  lri.fast = true;
  double len = 1.0, mbest = RTX_INF;
  int moi = 0, mbase = 0, mfoff = 0, mface = -1;
  bool mhave = false;
  for (;;) {
    if (mode == 0) {
      if (ref >= 0) {
        const DevNode2& nd = S.snode2[ref];
        if (STATS) C.nodes += 2;
        double a0, b0, a1, b1;
        const bool h0 = box_test(nd.box + 0, nd.box + 3, P, D, ri, a0, b0) && !(a0 > bt + S.margin) && !(b0 < tlo);
        const bool h1 = box_test(nd.box + 6, nd.box + 9, P, D, ri, a1, b1) && !(a1 > bt + S.margin) && !(b1 < tlo);
        const int c0 = nd.child[0], c1 = nd.child[1];
        if (h0 && h1) {  // nearer child first; the other waits on the stack
          const bool swap = a1 < a0;
          stk[sp * 64 + lane] = swap ? c0 : c1;
          ++sp;
          ref = swap ? c1 : c0;
          continue;
        }
        if (h0 || h1) {
          ref = h0 ? c0 : c1;
          continue;
        }
        if (sp == 0) break;
        --sp;
        ref = stk[sp * 64 + lane];
        continue;
      }
      const int code = ~ref;
      oc = code >> 2;
      oe = oc + (code & 3);
      mode = 1;
      continue;
    }
    if (mode == 1) {
      const int oi = oc++;
      const RtxObject& o = S.objs[oi];
      if (STATS) C.objects++;
      double a, b;
      // Geometry::intersect's world-box test (scene.cpp:15) + prune
      if (box_test(o.wmin, o.wmax, P, D, ri, a, b) && !(a > bt + S.margin) && !(b < tlo)) {
        const dvec3 pos = rtm::xform_point(o.inv, P);
        dvec3 dir = rtm::xform_point(o.inv, P + D) - pos;
        const double ln = rtm::length(dir);
        dir = rtm::normalize(dir);
        if (o.type == RTX_OBJ_TRIMESH) {
          if (S.meshes[o.mesh].node_count > 0) {
            const DevRoot& mr = S.mroots[o.mesh];
            const RayInv mri = ray_inv(dir);
            if (STATS) C.nodes++;
            double ma, mb;
            const double whi = (bt + S.margin) * ln * (1.0 + 1e-12);
            const double lo = closest ? -RTX_INF : tlo * ln * (1.0 - 1e-12) - S.lmargin;
            if (box_test(mr.lo, mr.hi, pos, dir, mri, ma, mb) && !(ma > whi) && !(mb < lo)) {
              lp = pos;
              ld = dir;
              lri = mri;
              len = ln;
              moi = oi;
              mbase = sp;
              mfoff = S.meshes[o.mesh].face_off;
              ref = mr.ref;
              mhave = false;
              mbest = RTX_INF;
              mface = -1;
              mode = 2;
              continue;
            }
          }
        } else {
          // the primitive's intersectLocalList entries, in list order.
          // Q_CLOSEST keeps the (t, sub)-smallest entry == intersectLocal
          // (DESIGN.md); Q_NEXT offers every entry to the key filter.
          double lt = RTX_INF;
          int ls = -1;
          auto entry = [&](double t, int sb) {
            if (closest) {
              if (ls < 0 || t < lt || (t == lt && sb < ls)) {
                lt = t;
                ls = sb;
              }
            } else {
              const double tw = t / ln;
              if (key_less(tp, rp, sq, tw, oi, sb) && tw <= tlimit && (!have || key_less(tw, oi, sb, bt, bobj, bsub))) {
                bt = tw;
                bobj = oi;
                bsub = sb;
                have = true;
              }
            }
          };
          if (o.type == RTX_OBJ_SPHERE) {  // Sphere.cpp:42-72
            const dvec3 d2 = rtm::normalize(dir);
            const dvec3 v = -pos;
            const double bb = rtm::dot(v, d2);
            double disc = bb * bb - rtm::dot(v, v) + 1;
            if (!(disc < 0.0)) {
              disc = sqrt(disc);
              const double t1 = bb - disc, t2 = bb + disc;
              if (t1 > RTX_RAY_EPS) entry(t1, 0);
              if (t2 > RTX_RAY_EPS) entry(t2, 1);
            }
          } else if (o.type == RTX_OBJ_BOX) {  // Box.cpp:65-97
            for (int it = 0; it < 6; it++) {
              const int mod0 = it % 3;
              const double dm = rtm::get(dir, mod0);
              if (dm == 0) continue;
              const double t = ((it / 3) - 0.5 - rtm::get(pos, mod0)) / dm;
              if (t < RTX_RAY_EPS) continue;
              const int mod1 = (it + 1) % 3, mod2 = (it + 2) % 3;
              const double x = rtm::get(pos, mod1) + t * rtm::get(dir, mod1);
              const double y = rtm::get(pos, mod2) + t * rtm::get(dir, mod2);
              if (x <= 0.5 && x >= -0.5 && y <= 0.5 && y >= -0.5) entry(t, it);
            }
          } else if (o.type == RTX_OBJ_CYLINDER) {  // Cylinder.cpp:155-263
            const double pz = pos.z, dz = dir.z;
            if (!(0.0 == dz)) {
              double t1, t2;
              if (dz > 0.0) {
                t1 = (-pz) / dz;
                t2 = (1.0 - pz) / dz;
              } else {
                t1 = (1.0 - pz) / dz;
                t2 = (-pz) / dz;
              }
              if (t1 >= RTX_RAY_EPS) {
                const dvec3 q = rtm::ray_at(pos, dir, t1);
                if ((q.x * q.x + q.y * q.y) <= 1.0) entry(t1, 0);
              }
              if (t2 >= RTX_RAY_EPS) {
                const dvec3 q = rtm::ray_at(pos, dir, t2);
                if ((q.x * q.x + q.y * q.y) <= 1.0) entry(t2, 1);
              }
            }
            const double x0 = pos.x, y0 = pos.y, x1 = dir.x, y1 = dir.y;
            const double aa = x1 * x1 + y1 * y1;
            const double bb = 2.0 * (x0 * x1 + y0 * y1);
            const double cc = x0 * x0 + y0 * y0 - 1.0;
            if (!(0.0 == aa)) {
              double disc = bb * bb - 4.0 * aa * cc;
              if (!(disc < 0.0)) {
                disc = sqrt(disc);
                const double t1 = (-bb - disc) / (2.0 * aa);
                const double t2 = (-bb + disc) / (2.0 * aa);
                if (t1 > RTX_RAY_EPS) {
                  const double z = rtm::ray_at(pos, dir, t1).z;
                  if (z >= 0.0 && z <= 1.0) entry(t1, 2);
                }
                if (t2 > RTX_RAY_EPS) {
                  const double z = rtm::ray_at(pos, dir, t2).z;
                  if (z >= 0.0 && z <= 1.0) entry(t2, 3);
                }
              }
            }
          } else if (o.type == RTX_OBJ_SQUARE) {  // Square.cpp:9-51
            if (!(dir.z == 0.0)) {
              const double t = -pos.z / dir.z;
              if (!(t <= RTX_RAY_EPS)) {
                const dvec3 Q = rtm::ray_at(pos, dir, t);
                if (!(Q.x < -0.5 || Q.x > 0.5) && !(Q.y < -0.5 || Q.y > 0.5)) entry(t, 0);
              }
            }
          }
          if (closest && ls >= 0) {
            const double tw = lt / ln;
            if (!have || tw < bt || (tw == bt && oi < bobj)) {
              bt = tw;
              bobj = oi;
              bsub = ls;
              have = true;
            }
          }
        }
      }
      if (oc == oe) {
        if (sp == 0) break;
        --sp;
        ref = stk[sp * 64 + lane];
        mode = 0;
      }
      continue;
    }
    // mode == 2: mesh BVH of object moi, local frame
    {
      const double whi = (bt + S.margin) * len * (1.0 + 1e-12);
      double hi = whi;
      if (closest && mhave) hi = rtm::gmin(hi, mbest + S.lmargin);
      const double lo = closest ? -RTX_INF : tlo * len * (1.0 - 1e-12) - S.lmargin;
      if (ref >= 0) {
        const DevNode2& nd = S.mnode2[ref];
        if (STATS) C.nodes += 2;
        double a0, b0, a1, b1;
        const bool h0 = box_test(nd.box + 0, nd.box + 3, lp, ld, lri, a0, b0) && !(a0 > hi) && !(b0 < lo);
        const bool h1 = box_test(nd.box + 6, nd.box + 9, lp, ld, lri, a1, b1) && !(a1 > hi) && !(b1 < lo);
        const int c0 = nd.child[0], c1 = nd.child[1];
        if (h0 && h1) {
          const bool swap = a1 < a0;
          stk[sp * 64 + lane] = swap ? c0 : c1;
          ++sp;
          ref = swap ? c1 : c0;
          continue;
        }
        if (h0 || h1) {
          ref = h0 ? c0 : c1;
          continue;
        }
      } else {
        const int code = ~ref;
        const int f0 = code >> 2, f1 = f0 + (code & 3);
        // a face whose plane hit lies beyond this bound cannot win (closest:
        // strictly farther than the mesh's best; next: farther than the
        // current best key) — tri_hit stops before the edge tests
        const double tcap = closest && mhave ? rtm::gmin(whi, mbest) : whi;
        for (int f = f0; f < f1; ++f) {
          if (STATS) C.tris++;
          double tf;
          if (tri_hit(S.faces[mfoff + f], lp, ld, tcap, tf)) {
            if (closest) {
              if (!mhave || tf < mbest || (tf == mbest && f < mface)) {
                mbest = tf;
                mface = f;
                mhave = true;
              }
            } else {
              const double tw = tf / len;
              if (key_less(tp, rp, sq, tw, moi, f) && tw <= tlimit &&
                  (!have || key_less(tw, moi, f, bt, bobj, bsub))) {
                bt = tw;
                bobj = moi;
                bsub = f;
                have = true;
              }
            }
          }
        }
      }
      if (sp > mbase) {
        --sp;
        ref = stk[sp * 64 + lane];
        continue;
      }
      // mesh finished: Trimesh::intersectLocal's result enters Scene::intersect
      if (closest && mhave) {
        const double tw = mbest / len;
        if (!have || tw < bt || (tw == bt && moi < bobj)) {
          bt = tw;
          bobj = moi;
          bsub = mface;
          have = true;
        }
      }
      if (oc < oe) {
        mode = 1;
      } else {
        if (sp == 0) break;
        --sp;
        ref = stk[sp * 64 + lane];
        mode = 0;
      }
    }
  }
  return have;
}


// Paired-child device layout (DevNode2) of one DFS-pre-order RtxNode tree
// nodes[0..n): child0 = i + 1, child1 = right (tree-relative), leaf items
// [first, first + count).  Internal node i becomes record base + k.
inline bool build_node2(const RtxNode* nodes, int n, std::vector<DevNode2>& out, DevRoot& root) {
  std::vector<int> idx(size_t(n), -1);
  const int base = static_cast<int>(out.size());
  int k = 0;
  for (int i = 0; i < n; ++i)
    if (nodes[i].count == 0) idx[size_t(i)] = base + k++;
  auto ref = [&](int c) -> int {
    const RtxNode& nd = nodes[c];
    if (nd.count == 0) return idx[size_t(c)];
    return ~((nd.first << 2) | nd.count);
  };
  for (int i = 0; i < n; ++i) {
    const RtxNode& nd = nodes[i];
    if (nd.count < 0 || nd.count > 3) return false;
    if (nd.count != 0) continue;
    const int c0 = i + 1, c1 = nd.right;
    if (c0 >= n || c1 <= i || c1 >= n) return false;
    DevNode2 r;
    std::memset(&r, 0, sizeof(r));
    for (int a = 0; a < 3; ++a) {
      r.box[0 + a] = nodes[c0].bmin[a];
      r.box[3 + a] = nodes[c0].bmax[a];
      r.box[6 + a] = nodes[c1].bmin[a];
      r.box[9 + a] = nodes[c1].bmax[a];
    }
    r.child[0] = ref(c0);
    r.child[1] = ref(c1);
    out.push_back(r);
  }
  std::memset(&root, 0, sizeof(root));
  for (int a = 0; a < 3; ++a) {
    root.lo[a] = nodes[0].bmin[a];
    root.hi[a] = nodes[0].bmax[a];
  }
  root.ref = ref(0);
  return true;
}

// pruning slack bases: largest coordinate magnitude in the
// scene / in any mesh-local box
inline double scene_extent(const RtxSceneDesc* d) {
  double e = 1.0;
  for (int i = 0; i < d->n_objects; ++i)
    for (int k = 0; k < 3; ++k) {
      e = fmax(e, fabs(d->objects[i].wmin[k]));
      e = fmax(e, fabs(d->objects[i].wmax[k]));
    }
  for (int k = 0; k < 3; ++k) e = fmax(e, fabs(d->camera.eye[k]));
  for (int i = 0; i < d->n_lights; ++i)
    for (int k = 0; k < 3; ++k) e = fmax(e, fabs(d->lights[i].pos[k]));
  return e;
}

inline double mesh_extent(const RtxSceneDesc* d) {
  double e = 1.0;
  for (int i = 0; i < d->n_mesh_nodes; ++i)
    for (int k = 0; k < 3; ++k) {
      e = fmax(e, fabs(d->mesh_nodes[i].bmin[k]));
      e = fmax(e, fabs(d->mesh_nodes[i].bmax[k]));
    }
  return e;
}

}  // namespace rtxd
