// rtx_traverse.h — two-level BVH query of the ray-trace hot path (shared by
// every render kernel; also compiled for the host by the traversal unit test,
// tests/native/traverse_host.hip, so its logic can be checked against the CPU
// restatement without a GPU).
#pragma once

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <functional>
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
//
// The loop is cut into units: trav_init, then trav_step until it returns
// true.  One step is one 4-wide BVH record, one object of a leaf, or
// one mesh leaf's faces.  The query's whole state lives in a Trav, so the
// persistent trace kernel can hand a lane a new query as soon as its own one
// ends while the other lanes of the wave keep stepping; traverse() runs one
// query to completion.
//
// Cold state.  The world ray (P, D) and its exact-fallback reciprocal (ri)
// are read only by the object steps (the world-box test, the transform into
// a mesh's frame) and when a mesh walk ends (the scene's float ray again) —
// not by the record steps that are most of the walk.  ColdRegs keeps them in
// registers; ColdLDS keeps them in a per-wave LDS block beside the stacks
// (field-major, [field][64 lanes], 8-byte accesses: conflict-free), which
// takes 19 VGPRs off the persistent traversal state of the trace kernels.
struct ColdRegs {
  dvec3 P, D;
  RayInv ri;
  dvec3 lp, ld;  // the mesh-local ray of a mesh walk
  RT_HD dvec3 getLP() const { return lp; }
  RT_HD dvec3 getLD() const { return ld; }
  RT_HD void setL(const dvec3& p, const dvec3& d) {
    lp = p;
    ld = d;
  }
  RT_HD dvec3 getP() const { return P; }
  RT_HD dvec3 getD() const { return D; }
  RT_HD RayInv getRI() const { return ri; }
  RT_HD void set(const dvec3& p, const dvec3& d, const RayInv& r) {
    P = p;
    D = d;
    ri = r;
  }
  RT_HD void reset() {
    P = D = lp = ld = mk3(0.0, 0.0, 0.0);
    ri.inv = mk3(0.0, 0.0, 0.0);
    ri.fast = true;
  }
};
#define RTX_COLD_FIELDS 9  // doubles per lane in a ColdLDS block (P, D, 1/D; fast is D's)
// (The mesh-local ray lp, ld — read by every leaf step — stays in registers:
// in LDS as well it measured no faster, 31.33 vs 31.32 ms with the short
// stack, and its 3 KB per wave do not fit beside a whole stack.)
struct ColdLDS {
  double* c;  // the lane's column of its wave's block: field k at c[k * 64]
  dvec3 lp, ld;
  RT_HD dvec3 getLP() const { return lp; }
  RT_HD dvec3 getLD() const { return ld; }
  RT_HD void setL(const dvec3& p, const dvec3& d) {
    lp = p;
    ld = d;
  }
  RT_HD dvec3 getP() const { return mk3(c[0 * 64], c[1 * 64], c[2 * 64]); }
  RT_HD dvec3 getD() const { return mk3(c[3 * 64], c[4 * 64], c[5 * 64]); }
  RT_HD RayInv getRI() const {
    RayInv r;
    r.inv = mk3(c[6 * 64], c[7 * 64], c[8 * 64]);
    r.fast = ray_inv_fast(getD());  // (ray_inv's flag, from D again)
    return r;
  }
  RT_HD void set(const dvec3& p, const dvec3& d, const RayInv& r) {
    c[0 * 64] = p.x;
    c[1 * 64] = p.y;
    c[2 * 64] = p.z;
    c[3 * 64] = d.x;
    c[4 * 64] = d.y;
    c[5 * 64] = d.z;
    c[6 * 64] = r.inv.x;
    c[7 * 64] = r.inv.y;
    c[8 * 64] = r.inv.z;
  }
  RT_HD void reset() { lp = ld = mk3(0.0, 0.0, 0.0); }
};

template <class Cold>
struct TravT {
  Cold cold;  // P, D, ri: the world ray and its exact-fallback reciprocal
  RayF rf;    // float tests of the records being walked: the scene's, or in
              // mode 2 the mesh's (local frame); reset when the mesh is done
  double tp, tlimit, tlo;
  int rp, sq;
  // answer so far
  double bt;
  int bobj, bsub;
  bool have;
  // walk: ref >= 0 DevNode4 record, ref < 0 leaf ~(first << 2 | count);
  // mode 0 scene BVH, 1 objects [oc, oe) of a scene leaf, 2 mesh BVH
  int sp, ref, mode, oc, oe;
  // mesh context (local frame of object moi; its ray in cold)
  double len, mbest;
  int moi, mbase, mfoff, mnoff, mface;
  bool mhave;
  bool closest;  // the query's mode (read by the Q_ANY instantiations)
};
using Trav = TravT<ColdRegs>;

// QMODE Q_ANY: one instantiation for both query kinds, the mode read from
// the Trav — for kernels whose lanes mix closest and next-hit queries (the
// tail), so a wave steps them together instead of running the two loops
// one after the other.
#define Q_ANY 0

// A face hit counts only if its mesh-BVH leaf box passes the exact slab test
// in the mesh's local frame (KdTree::intersectList collects the items of hit
// leaves, kdTree.h:100-117): the walk's internal tests are conservative.
// `leaf`: the face's reference leaf node (TMeta.leaf, a global mnodes index).
RT_HD bool leaf_ok(const dvec3& lp, const dvec3& ld, const DevScene& S, int leaf) {
  const RtxNode& lf = S.mnodes[leaf];
  double a, b;
  return slab(lf.bmin, lf.bmax, lp, ld, a, b);
}

// The walk's stack of pending entries (records or leaves), per lane.
// StackLDS: the whole stack in LDS, entry i of the lane at s[i * 64] (one
// column per lane of its wave's [entry][64] block: conflict-free).
// StackShort (the trace kernels of scenes whose whole stacks and cold state
// do not fit in LDS at 3 workgroups per CU, e.g. the 1M-face dragon): the
// first k entries in LDS (RTX_LDS_STACK; a test knob lowers it), the rest in
// a per-thread overflow column in HBM — walks rarely go that deep (the headline scene's deepest of
// 360 k sampled queries held 10 entries, the dragon's 13; the trees' worst
// cases are 31 / 41).  Where the whole stack fits it is faster (its put / get
// need no branch: headline 30.6-31.2 vs 31.3-31.4 ms).
#define RTX_LDS_STACK 16
struct StackLDS {
  int* s;
  RT_HD bool lds_only(int) const { return true; }
  RT_HD void put(int i, int v) const { s[i * 64] = v; }
  RT_HD void put_lds(int i, int v) const { s[i * 64] = v; }
  RT_HD int get(int i) const { return s[i * 64]; }
};
struct StackShort {
  int* s;       // the lane's LDS column (entry i at s[i * 64])
  int* sb;      // the workgroup's LDS stack block: s - sb = wave * k * 64 + lane
  int* ob;      // the workgroup's overflow columns (thread t's at ob[t])
  int ostride;  // threads of the launch
  int k;        // entries in LDS
  // the thread's overflow column, from its LDS column (no register of its
  // own for the rare deep walk)
  RT_HD int* col() const {
    const int q = static_cast<int>(s - sb);
    return ob + ((q / (k * 64)) * 64 + (q & 63));
  }
  // entries [0, n) all in LDS
  RT_HD bool lds_only(int n) const { return n <= k; }
  RT_HD void put(int i, int v) const {
    if (i < k) s[i * 64] = v;
    else col()[size_t(i - k) * ostride] = v;
  }
  RT_HD void put_lds(int i, int v) const { s[i * 64] = v; }
  // (the LDS read is unconditional, clamped; only an overflowed entry is
  // read again from HBM)
  RT_HD int get(int i) const {
    int v = s[(i < k ? i : k - 1) * 64];
    if (i >= k) v = col()[size_t(i - k) * ostride];
    return v;
  }
};

// Visit one 4-wide record: test its entries' boxes (conservatively, pruned
// to [lo, hi]), continue with the nearest entry hit and push the
// other hits farthest first, so the walk stays near-first.  False if no
// entry was hit (the caller pops).
// A record's 128 bytes as eight 16-byte loads (visit4's operand).
struct Rec4 {
  float4 lx, ly, lz, hx, hy, hz;
  int4 ch;
  int nrec;
};
RT_HD Rec4 load_rec4(const DevNode4& nd) {
  const float4* q4 = reinterpret_cast<const float4*>(&nd);
  Rec4 r;
  r.lx = q4[0];
  r.ly = q4[1];
  r.lz = q4[2];
  r.hx = q4[3];
  r.hy = q4[4];
  r.hz = q4[5];
  r.ch = reinterpret_cast<const int4*>(&nd)[6];
  r.nrec = reinterpret_cast<const int4*>(&nd)[7].x;
  return r;
}

template <bool STATS, class STK>
RT_HD bool visit4(const Rec4& R, const RayF& rf, const double hi, const double lo, const STK& stk, int& sp,
                  int& ref, Counters& C) {
  const float NOHIT = __builtin_inff();
  // prune bounds widened to floats (hi up, lo down): pruning stays safe
  const float hf = f_up_wide(hi), lf = f_down_wide(lo);
  float a0 = NOHIT, a1 = NOHIT, a2 = NOHIT, a3 = NOHIT;
  int r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  // the whole record in one burst of 16-byte loads before any test (the
  // caller issues them, load_rec4): the entries used to be loaded inside
  // their own `k < count` branches, up to nine dependent round trips per
  // record for a wave stepping alone.  Every entry is tested (empty ones are
  // masked by the count).
  const float4 lx = R.lx, ly = R.ly, lz = R.lz, hx = R.hx, hy = R.hy, hz = R.hz;
  const int4 ch = R.ch;
  const int nrec = R.nrec;
  auto test = [&](int k, float lox, float loy, float loz, float hix, float hiy, float hiz, int child, float& ak,
                  int& rk) {
    if (STATS && k < nrec) C.nodes++;
    float ta, tb;
    const bool hit = box_cons32v(lox, loy, loz, hix, hiy, hiz, rf, ta, tb) && ta <= hf && tb >= lf;
    if (k < nrec && hit) {
      ak = ta;
      rk = child;
    }
  };
  test(0, lx.x, ly.x, lz.x, hx.x, hy.x, hz.x, ch.x, a0, r0);
  test(1, lx.y, ly.y, lz.y, hx.y, hy.y, hz.y, ch.y, a1, r1);
  test(2, lx.z, ly.z, lz.z, hx.z, hy.z, hz.z, ch.z, a2, r2);
  test(3, lx.w, ly.w, lz.w, hx.w, hy.w, hz.w, ch.w, a3, r3);
  // sorting network on (entry distance, ref)
  auto cs = [](float& x, int& rx, float& y, int& ry) {
    const bool s = y < x;
    const float lo_ = s ? y : x, hi_ = s ? x : y;
    const int rlo = s ? ry : rx, rhi = s ? rx : ry;
    x = lo_;
    y = hi_;
    rx = rlo;
    ry = rhi;
  };
  cs(a0, r0, a1, r1);
  cs(a2, r2, a3, r3);
  cs(a0, r0, a2, r2);
  cs(a1, r1, a3, r3);
  cs(a1, r1, a2, r2);
  if (!(a0 < NOHIT)) return false;
  if (stk.lds_only(sp + 3)) {  // (every push of a shallow walk: LDS stores only)
    if (a3 < NOHIT) stk.put_lds(sp++, r3);
    if (a2 < NOHIT) stk.put_lds(sp++, r2);
    if (a1 < NOHIT) stk.put_lds(sp++, r1);
  } else {
    if (a3 < NOHIT) stk.put(sp++, r3);
    if (a2 < NOHIT) stk.put(sp++, r2);
    if (a1 < NOHIT) stk.put(sp++, r1);
  }
  ref = r0;
  return true;
}

// Start a query; false if it is already complete (empty scene or the root
// box is missed: KdTree::intersectList starts with the root's bbox test).
template <bool STATS, int QMODE, class TR>
RT_HD bool trav_init(TR& T, const DevScene& S, const dvec3& P, const dvec3& D, const double tp, const int rp,
                     const int sq, const double tlimit, Counters& C) {
  T.tp = tp;
  T.rp = rp;
  T.sq = sq;
  T.tlimit = tlimit;
  T.bt = tlimit;
  T.bobj = INT_MAX;
  T.bsub = INT_MAX;
  T.have = false;
  if (QMODE != Q_ANY) T.closest = QMODE == Q_CLOSEST;  // Q_ANY: set by the caller first
  if (S.n_snodes == 0) return false;
  T.tlo = QMODE == Q_CLOSEST ? -RTX_INF : tp - S.margin;  // Q_ANY: tp = -inf for a closest query
  const RayInv ri = ray_inv(D);
  T.cold.set(P, D, ri);
  T.rf = ray_f(P, D, ri);
  if (STATS) {
    C.nodes++;
    C.queries++;
  }
  double a, b;
  if (!box_test(S.sroot.lo, S.sroot.hi, P, D, ri, a, b) || a > T.bt + S.margin || b < T.tlo) return false;
  T.sp = 0;
  T.ref = S.sroot.ref;
  T.mode = 0;
  T.oc = 0;
  T.oe = 0;
  T.len = 1.0;
  T.mbest = RTX_INF;
  T.moi = 0;
  T.mbase = 0;
  T.mfoff = 0;
  T.mnoff = 0;
  T.mface = -1;
  T.mhave = false;
  return true;
}

// Every field a constant (a walk no lane continues): lets the compiler see
// the walk's registers as free between queries.
template <class TR>
RT_HD void trav_reset(TR& T) {
  T.cold.reset();
  T.rf = RayF{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  T.tp = T.tlimit = T.tlo = T.bt = T.len = T.mbest = 0.0;
  T.rp = T.sq = T.bobj = T.bsub = T.sp = T.ref = T.mode = T.oc = T.oe = 0;
  T.moi = T.mbase = T.mfoff = T.mnoff = T.mface = 0;
  T.have = T.mhave = T.closest = false;
}

// The lane's next unit is a 4-wide record (scene or mesh): the cheap step.
// Objects (mode 1: world-box test, transform to the mesh frame) and mesh
// leaves (exact face tests) are the costly ones.
template <class TR>
RT_HD bool trav_at_record(const TR& T) { return T.mode != 1 && T.ref >= 0; }

// One unit of the walk; true when the query is complete.
template <bool STATS, int QMODE, class TR, class STK>
RT_HD bool trav_step(TR& T, const DevScene& S, const STK& stk, Counters& C) {
  const bool closest = QMODE == Q_CLOSEST || (QMODE == Q_ANY && T.closest);
  const double tp = T.tp, tlimit = T.tlimit, tlo = T.tlo;
  const int rp = T.rp, sq = T.sq;
  double& bt = T.bt;
  int& bobj = T.bobj;
  int& bsub = T.bsub;
  bool& have = T.have;
  int& sp = T.sp;
  int& ref = T.ref;
  // a 4-wide record, scene (mode 0) or mesh (mode 2, local frame): one call
  // site for both, so a wave with lanes at both levels runs it once (and the
  // kernel carries one inlined copy)
  const bool mesh = T.mode == 2;
  if (T.mode != 1 && ref >= 0) {
    // the record's loads first, then the prune bounds (FP64) while they are
    // in flight (the scheduler used to place the loads after the bounds)
    const DevNode4* recs = !mesh ? S.snode4 : S.mnode4;
    const Rec4 rec = load_rec4(recs[ref]);
    double hi = bt + S.margin, lo = tlo;
    if (mesh) {
      const double len = T.len;
      hi = (bt + S.margin) * len * (1.0 + 1e-12);
      if (closest && T.mhave) hi = rtm::gmin(hi, T.mbest + S.lmargin);
      lo = closest ? -RTX_INF : tlo * len * (1.0 - 1e-12) - S.lmargin;
    }
    if (visit4<STATS>(rec, T.rf, hi, lo, stk, sp, ref, C)) return false;
    if (!mesh) {
      if (sp == 0) return true;
      --sp;
      ref = stk.get(sp);
      return false;
    }
  }
  if (T.mode == 0) {
    const int code = ~ref;
    T.oc = code >> 2;
    T.oe = T.oc + (code & 3);
    T.mode = 1;
    return false;
  }
  if (T.mode == 1) {
    const int oi = T.oc++;
    const RtxObject& o = S.objs[oi];
    if (STATS) C.objects++;
    double a, b;
    // Geometry::intersect's world-box test (scene.cpp:15) + prune
    const dvec3 wP = T.cold.getP(), wD = T.cold.getD();
    if (box_test(o.wmin, o.wmax, wP, wD, T.cold.getRI(), a, b) && !(a > bt + S.margin) && !(b < tlo)) {
      dvec3 pos, dir;
      obj_local(o, wP, wD, pos, dir);
      const double ln = rtm::length(dir);
      dir = rtm::normalize(dir);
      if (o.type == RTX_OBJ_TRIMESH) {
        if (o.pad[RTX_OBJ_MFLAGS] & RTX_MESH_TREE) {
          const DevRoot& mr = S.mroots[o.mesh];
          const RayInv mri = ray_inv(dir);
          if (STATS) C.nodes++;
          double ma, mb;
          const double whi = (bt + S.margin) * ln * (1.0 + 1e-12);
          const double lo = closest ? -RTX_INF : tlo * ln * (1.0 - 1e-12) - S.lmargin;
          if (box_test(mr.lo, mr.hi, pos, dir, mri, ma, mb) && !(ma > whi) && !(mb < lo)) {
            T.cold.setL(pos, dir);
            T.rf = ray_f(pos, dir, mri);
            T.len = ln;
            T.moi = oi;
            T.mbase = sp;
            T.mfoff = o.pad[RTX_OBJ_FACE_OFF];
            T.mnoff = o.pad[RTX_OBJ_NODE_OFF];
            ref = mr.ref;
            T.mhave = false;
            T.mbest = RTX_INF;
            T.mface = -1;
            T.mode = 2;
            return false;
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
            if (key_less(tp, rp, sq, tw, oi, sb) && tw <= tlimit) {
              if (!have || key_less(tw, oi, sb, bt, bobj, bsub)) {
                bt = tw;
                bobj = oi;
                bsub = sb;
                have = true;
              }
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
        } else if (o.type == RTX_OBJ_CONE) {
          // entries: 0 near body root, 1 far body root, 2 cap z=0, 3 cap z=h
          const double* prm = S.oprm + size_t(oi) * RTX_OBJ_PARAMS;
          const ConeRoots cr = cone_roots(prm, pos, dir);
          if (cr.ok) {
            const double pz = pos.z, dz = dir.z;
            const bool capped = prm[RTX_CONE_CAP] != 0.0;
            const double t1 = (-pz) / dz;
            const double t2 = (prm[RTX_CONE_H] - pz) / dz;
            const dvec3 p1 = rtm::ray_at(pos, dir, t1);
            const dvec3 p2 = rtm::ray_at(pos, dir, t2);
            const double br = prm[RTX_CONE_BR], tr = prm[RTX_CONE_TR];
            const bool in1 = capped && p1.x * p1.x + p1.y * p1.y <= br * br;
            const bool in2 = capped && p2.x * p2.x + p2.y * p2.y <= tr * tr;
            const bool near_good = cone_good(prm, rtm::ray_at(pos, dir, cr.near_t));
            const bool far_good = cone_good(prm, rtm::ray_at(pos, dir, cr.far_t));
            if (closest) {
              // intersectLocal's own root choice (Cone.cpp:41-98), not the
              // nearest list entry: a far root replaces the near one whenever
              // it is good and beyond RAY_EPSILON
              double root = RTX_RAY_EPS;
              int sb = -1;
              if (near_good && cr.near_t > root) {
                root = cr.near_t;
                sb = 0;
              }
              if (far_good && ((near_good && cr.far_t < root) || cr.far_t > RTX_RAY_EPS)) {
                root = cr.far_t;
                sb = 1;
              }
              if (in1 && t1 < root && t1 > RTX_RAY_EPS) {
                root = t1;
                sb = 2;
              }
              if (in2 && t2 < root && t2 > RTX_RAY_EPS) {
                root = t2;
                sb = 3;
              }
              if (!(root <= RTX_RAY_EPS)) entry(root, sb);
            } else {  // intersectLocalList (Cone.cpp:108-210)
              if (near_good && cr.near_t > RTX_RAY_EPS) entry(cr.near_t, 0);
              if (cr.far_t != cr.near_t && far_good && cr.far_t > RTX_RAY_EPS) entry(cr.far_t, 1);
              if (in1 && t1 > RTX_RAY_EPS) entry(t1, 2);
              if (in2 && t2 > RTX_RAY_EPS) entry(t2, 3);
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
    if (T.oc == T.oe) {
      if (sp == 0) return true;
      --sp;
      ref = stk.get(sp);
      T.mode = 0;
    }
    return false;
  }
  // mode == 2: mesh BVH of object moi, local frame (a record missed above,
  // or a leaf)
  const double len = T.len;
  const double whi = (bt + S.margin) * len * (1.0 + 1e-12);
  if (ref < 0) {
    const int code = ~ref;
    const int f0 = code >> 2, f1 = f0 + (code & 3);
    // a face whose plane hit lies beyond this bound cannot win (closest:
    // strictly farther than the mesh's best; next: farther than the
    // current best key) — tri_test stops before the edge tests
    const double tcap = closest && T.mhave ? rtm::gmin(whi, T.mbest) : whi;
    const dvec3 lp = T.cold.getLP(), ld = T.cold.getLD();
    // the next face's loads go out before this face's tests: one round trip
    // per leaf entry instead of one per face
    FaceV qn = face_ld(S.tfaces[T.mfoff + f0]);
    TMeta mn = S.tmeta[T.mfoff + f0];
    for (int f = f0; f < f1; ++f) {
      if (STATS) C.tris++;
      double tf;
      const FaceV q = qn;
      const TMeta meta = mn;
      if (f + 1 < f1) {
        qn = face_ld(S.tfaces[T.mfoff + f + 1]);
        mn = S.tmeta[T.mfoff + f + 1];
      }
      face_pin(q);
      const bool hit = tri_test(q, lp, ld, tcap, tf);
      pin(meta.rank);
      pin(meta.leaf);
      if (hit) {
        const int rk = meta.rank;
        if (closest) {
          if ((!T.mhave || tf < T.mbest || (tf == T.mbest && rk < T.mface)) && leaf_ok(lp, ld, S, meta.leaf)) {
            T.mbest = tf;
            T.mface = rk;
            T.mhave = true;
          }
        } else {
          const double tw = tf / len;
          if (key_less(tp, rp, sq, tw, T.moi, rk) && tw <= tlimit && leaf_ok(lp, ld, S, meta.leaf)) {
            if (!have || key_less(tw, T.moi, rk, bt, bobj, bsub)) {
              bt = tw;
              bobj = T.moi;
              bsub = rk;
              have = true;
            }
          }
        }
      }
    }
  }
  if (sp > T.mbase) {
    --sp;
    ref = stk.get(sp);
    return false;
  }
  // mesh finished: Trimesh::intersectLocal's result enters Scene::intersect
  T.rf = ray_f(T.cold.getP(), T.cold.getD(), T.cold.getRI());
  if (closest && T.mhave) {
    const double tw = T.mbest / len;
    if (!have || tw < bt || (tw == bt && T.moi < bobj)) {
      bt = tw;
      bobj = T.moi;
      bsub = T.mface;
      have = true;
    }
  }
  if (T.oc < T.oe) {
    T.mode = 1;
    return false;
  }
  if (sp == 0) return true;
  --sp;
  ref = stk.get(sp);
  T.mode = 0;
  return false;
}


// One query to completion (no shadow early-out).
template <bool STATS>
RT_HD bool traverse(const DevScene& S, const int qmode, const dvec3& P, const dvec3& D, const double tp, const int rp,
                    const int sq, const double tlimit, double& bt, int& bobj, int& bsub, int* __restrict__ stk,
                    const int lane, Counters& C) {
  Trav T;
  if (qmode == Q_CLOSEST) {
    if (trav_init<STATS, Q_CLOSEST>(T, S, P, D, tp, rp, sq, tlimit, C))
      while (!trav_step<STATS, Q_CLOSEST>(T, S, StackLDS{stk + lane}, C)) {
      }
  } else {
    if (trav_init<STATS, Q_NEXT>(T, S, P, D, tp, rp, sq, tlimit, C))
      while (!trav_step<STATS, Q_NEXT>(T, S, StackLDS{stk + lane}, C)) {
      }
  }
  bt = T.bt;
  bobj = T.bobj;
  bsub = T.bsub;
  return T.have;
}


// One query to completion, either kind, one traversal loop (Q_ANY).
template <bool STATS>
RT_HD bool traverse_any(const DevScene& S, const int qmode, const dvec3& P, const dvec3& D, const double tp,
                        const int rp, const int sq, const double tlimit, double& bt, int& bobj, int& bsub,
                        int* __restrict__ stk, const int lane, Counters& C) {
  Trav T;
  T.closest = qmode == Q_CLOSEST;
  if (trav_init<STATS, Q_ANY>(T, S, P, D, T.closest ? -RTX_INF : tp, rp, sq, tlimit, C))
    while (!trav_step<STATS, Q_ANY>(T, S, StackLDS{stk + lane}, C)) {
    }
  bt = T.bt;
  bobj = T.bobj;
  bsub = T.bsub;
  return T.have;
}

// float bounds of a double box rounded outward (the record holds a superset)
inline float round_down_f(double x) {
  float f = static_cast<float>(x);
  if (static_cast<double>(f) > x) f = std::nextafter(f, -HUGE_VALF);
  return f;
}
inline float round_up_f(double x) {
  float f = static_cast<float>(x);
  if (static_cast<double>(f) < x) f = std::nextafter(f, HUGE_VALF);
  return f;
}

// 4-wide records (DevNode4) of one DFS-pre-order RtxNode tree// 4-wide records (DevNode4) of one DFS-pre-order RtxNode tree nodes[0..n)
// (child0 = i + 1, child1 = right, tree-relative; leaf items [first,
// first + count)), emitted in DFS pre-order after the records already in
// `out`.  stack_need: the most stack entries a walk of this tree can hold
// (the sum of entries - 1 over the records of a root-to-leaf path).
inline bool build_node4(const RtxNode* nodes, int n, std::vector<DevNode4>& out, DevRoot& root, int& stack_need) {
  for (int i = 0; i < n; ++i) {
    const RtxNode& nd = nodes[i];
    if (nd.count < 0 || nd.count > 3) return false;
    if (nd.count == 0 && (i + 1 >= n || nd.right <= i || nd.right >= n)) return false;
  }
  auto leaf_code = [&](int c) { return ~((nodes[c].first << 2) | nodes[c].count); };
  std::function<int(int, int&)> emit = [&](int i, int& need) -> int {
    const int idx = static_cast<int>(out.size());
    out.emplace_back();
    DevNode4 r;
    std::memset(&r, 0, sizeof(r));
    // the node's children, then — while the record has room — the internal
    // entry of the largest surface area opened into its two children (a
    // node whose child is a leaf still fills four entries)
    int ents[4], ne = 0;
    ents[ne++] = i + 1;
    ents[ne++] = nodes[i].right;
    while (ne < 4) {
      int best = -1;
      double bsa = -1.0;
      for (int k = 0; k < ne; ++k) {
        const RtxNode& c = nodes[ents[k]];
        if (c.count != 0) continue;
        const double x = c.bmax[0] - c.bmin[0], y = c.bmax[1] - c.bmin[1], z = c.bmax[2] - c.bmin[2];
        const double sa = x * y + y * z + z * x;
        if (sa > bsa) {
          bsa = sa;
          best = k;
        }
      }
      if (best < 0) break;
      const int e = ents[best];
      ents[best] = e + 1;
      ents[ne++] = nodes[e].right;
    }
    r.count = ne;
    for (int k = ne; k < 4; ++k) {  // unused entries: empty boxes, never visited (k >= count)
      for (int a = 0; a < 3; ++a) {
        r.lo[a][k] = HUGE_VALF;
        r.hi[a][k] = -HUGE_VALF;
      }
      r.child[k] = 0;
    }
    int sub = 0;
    for (int k = 0; k < ne; ++k) {
      const int e = ents[k];
      for (int a = 0; a < 3; ++a) {
        r.lo[a][k] = round_down_f(nodes[e].bmin[a]);
        r.hi[a][k] = round_up_f(nodes[e].bmax[a]);
      }
      if (nodes[e].count == 0) {
        int below = 0;
        r.child[k] = emit(e, below);
        sub = below > sub ? below : sub;
      } else {
        r.child[k] = leaf_code(e);
      }
    }
    out[size_t(idx)] = r;
    need = (ne - 1) + sub;
    return idx;
  };
  std::memset(&root, 0, sizeof(root));
  for (int a = 0; a < 3; ++a) {
    root.lo[a] = nodes[0].bmin[a];
    root.hi[a] = nodes[0].bmax[a];
  }
  stack_need = 0;
  root.ref = nodes[0].count == 0 ? emit(0, stack_need) : leaf_code(0);
  return true;
}

// ------------------------------------------------------------------ traversal trees
// The device walks BVHs of its own, built here from the flat scene:
// binned-SAH trees over face boxes (leaves of <= 3 faces) per mesh, and a
// one-object-per-leaf tree over the objects' world boxes.  Results are the
// reference's all the same (DESIGN.md "Traversal trees"): an object is a
// candidate iff its exact world-box test passes (Geometry::intersect,
// scene.cpp:15, implies its leaf's), a face iff its REFERENCE leaf box
// passes the exact slab test (leaf_ok) — both are tested exactly where they
// decide — and every box of these trees contains its items, so the
// conservative walk reaches every object and every face a ray hits.  Ties
// keep the reference ranks (object index, face index in DFS-leaf order).
struct TBox {
  double lo[3], hi[3];
};

inline double tbox_area(const TBox& b) {
  const double x = b.hi[0] - b.lo[0], y = b.hi[1] - b.lo[1], z = b.hi[2] - b.lo[2];
  return x * y + y * z + z * x;
}
inline void tbox_grow(TBox& a, const TBox& b) {
  for (int k = 0; k < 3; ++k) {
    a.lo[k] = b.lo[k] < a.lo[k] ? b.lo[k] : a.lo[k];
    a.hi[k] = b.hi[k] > a.hi[k] ? b.hi[k] : a.hi[k];
  }
}
inline TBox tbox_empty() {
  TBox b;
  for (int k = 0; k < 3; ++k) {
    b.lo[k] = HUGE_VAL;
    b.hi[k] = -HUGE_VAL;
  }
  return b;
}

// Binned SAH over item boxes (defaults: 16 bins, traversal cost 1.2 per node
// against 1 per item, SahParams; other settings measured within noise,
// profiles/r04u_sah_sweep.txt).  Emits nodes in DFS
// pre-order (child0 = i + 1, right), leaves [first, first + count) into
// `order`, a permutation of the items.
struct SahParams {
  int bins = 16;
  double c_node = 1.2, c_item = 1.0;
};
inline void tree_build(const std::vector<TBox>& box, int max_leaf, std::vector<RtxNode>& nodes,
                       std::vector<int>& order, const SahParams& sp = SahParams()) {
  const int n = static_cast<int>(box.size());
  order.resize(size_t(n));
  for (int i = 0; i < n; ++i) order[size_t(i)] = i;
  nodes.clear();
  if (n == 0) return;
  std::vector<double> cen(size_t(n) * 3);
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) cen[size_t(i) * 3 + k] = 0.5 * (box[size_t(i)].lo[k] + box[size_t(i)].hi[k]);
  const int NBIN = sp.bins < 2 ? 2 : (sp.bins > 256 ? 256 : sp.bins);
  std::function<void(int, int, int)> rec = [&](int l, int r, int depth) {
    const int me = static_cast<int>(nodes.size());
    nodes.emplace_back();
    TBox b = tbox_empty(), cb = tbox_empty();
    for (int i = l; i < r; ++i) {
      const int it = order[size_t(i)];
      tbox_grow(b, box[size_t(it)]);
      TBox c;
      for (int k = 0; k < 3; ++k) c.lo[k] = c.hi[k] = cen[size_t(it) * 3 + k];
      tbox_grow(cb, c);
    }
    RtxNode nd;
    std::memset(&nd, 0, sizeof(nd));
    for (int k = 0; k < 3; ++k) {
      nd.bmin[k] = b.lo[k];
      nd.bmax[k] = b.hi[k];
    }
    nd.depth = depth;
    const int cnt = r - l;
    auto make_leaf = [&]() {
      nd.right = -1;
      nd.first = l;
      nd.count = cnt;
      nodes[size_t(me)] = nd;
    };
    if (cnt == 1) {
      make_leaf();
      return;
    }
    // best binned split over the three axes
    double best = HUGE_VAL;
    int bax = -1, bbin = -1;
    for (int k = 0; k < 3; ++k) {
      const double ext = cb.hi[k] - cb.lo[k];
      if (!(ext > 0.0)) continue;
      std::vector<int> bc(static_cast<size_t>(NBIN), 0);
      std::vector<TBox> bb(static_cast<size_t>(NBIN));
      for (int q = 0; q < NBIN; ++q) bb[q] = tbox_empty();
      for (int i = l; i < r; ++i) {
        const int it = order[size_t(i)];
        int q = static_cast<int>((cen[size_t(it) * 3 + k] - cb.lo[k]) / ext * NBIN);
        q = q < 0 ? 0 : (q >= NBIN ? NBIN - 1 : q);
        bc[q]++;
        tbox_grow(bb[q], box[size_t(it)]);
      }
      std::vector<double> ra(static_cast<size_t>(NBIN));
      std::vector<int> rc(static_cast<size_t>(NBIN));
      TBox acc = tbox_empty();
      int ac = 0;
      for (int q = NBIN - 1; q > 0; --q) {
        tbox_grow(acc, bb[q]);
        ac += bc[q];
        ra[q] = tbox_area(acc);
        rc[q] = ac;
      }
      acc = tbox_empty();
      ac = 0;
      for (int q = 0; q < NBIN - 1; ++q) {
        tbox_grow(acc, bb[q]);
        ac += bc[q];
        if (ac == 0 || rc[q + 1] == 0) continue;
        const double c = tbox_area(acc) * ac + ra[q + 1] * rc[q + 1];
        if (c < best) {
          best = c;
          bax = k;
          bbin = q;
        }
      }
    }
    const double area = tbox_area(b);
    const double split_cost = area > 0.0 && bax >= 0 ? sp.c_node + sp.c_item * best / area : HUGE_VAL;
    if (cnt <= max_leaf && sp.c_item * cnt <= split_cost) {
      make_leaf();
      return;
    }
    int m = l + cnt / 2;
    if (bax >= 0) {
      const double ext = cb.hi[bax] - cb.lo[bax];
      auto left = [&](int it) {
        int q = static_cast<int>((cen[size_t(it) * 3 + bax] - cb.lo[bax]) / ext * NBIN);
        q = q < 0 ? 0 : (q >= NBIN ? NBIN - 1 : q);
        return q <= bbin;
      };
      m = static_cast<int>(std::partition(order.begin() + l, order.begin() + r, left) - order.begin());
      if (m == l || m == r) m = l + cnt / 2;
    }
    rec(l, m, depth + 1);
    nd.right = static_cast<int>(nodes.size());
    nd.first = -1;
    nd.count = 0;
    nodes[size_t(me)] = nd;
    rec(m, r, depth + 1);
  };
  rec(0, n, 0);
}

// Everything rtx_scene_create uploads for the walk.
struct TravTrees {
  std::vector<DevNode4> sn4, mn4;
  std::vector<DevRoot> mroots;
  DevRoot sroot;
  std::vector<RtxFace> tfaces;
  std::vector<int32_t> trank;
  std::vector<TMeta> tmeta;
  std::vector<RtxObject> objs;  // the objects with their mesh fields in pad (augment_objects)
  int sneed = 0, mneed = 0;
};

// Renumber the mesh records so the hottest come first — every mesh's root
// record, then their children while `cap` allows — so every walk into a mesh
// starts on a few densely packed cache lines.
inline void hot_mesh_records(TravTrees& T, int cap) {
  const int n = static_cast<int>(T.mn4.size());
  std::vector<int> hot;
  std::vector<char> is_hot(size_t(n), 0);
  auto take = [&](int r) {
    if (r >= 0 && r < n && !is_hot[size_t(r)] && static_cast<int>(hot.size()) < cap) {
      is_hot[size_t(r)] = 1;
      hot.push_back(r);
    }
  };
  for (const DevRoot& mr : T.mroots) take(mr.ref);
  const size_t nroots = hot.size();
  for (size_t i = 0; i < nroots; ++i) {
    const DevNode4& nd = T.mn4[size_t(hot[i])];
    for (int k = 0; k < nd.count; ++k) take(nd.child[k]);
  }
  std::vector<int> remap(size_t(n), -1);
  int next = 0;
  for (int r : hot) remap[size_t(r)] = next++;
  for (int r = 0; r < n; ++r)
    if (!is_hot[size_t(r)]) remap[size_t(r)] = next++;
  std::vector<DevNode4> out(static_cast<size_t>(n));
  for (int r = 0; r < n; ++r) {
    DevNode4 nd = T.mn4[size_t(r)];
    for (int k = 0; k < nd.count; ++k)
      if (nd.child[k] >= 0) nd.child[k] = remap[size_t(nd.child[k])];
    out[size_t(remap[size_t(r)])] = nd;
  }
  T.mn4.swap(out);
  for (DevRoot& mr : T.mroots)
    if (mr.ref >= 0 && mr.ref < n) mr.ref = remap[size_t(mr.ref)];
}

// The device copy of the objects: a trimesh's mesh fields (face_off,
// node_off, vert_off, flags) in RtxObject.pad (RTX_OBJ_*), read with the
// object record.  pad[RTX_OBJ_WOPAQUE] is left 0 (rtx_scene_create sets it).
inline void augment_objects(const RtxSceneDesc* d, std::vector<RtxObject>& objs) {
  objs.assign(d->objects, d->objects + d->n_objects);
  for (RtxObject& o : objs) {
    for (int k = 0; k < 5; ++k) o.pad[k] = 0;
    if (o.type != RTX_OBJ_TRIMESH || o.mesh < 0 || o.mesh >= d->n_meshes) continue;
    const RtxMesh& me = d->meshes[o.mesh];
    o.pad[RTX_OBJ_FACE_OFF] = me.face_off;
    o.pad[RTX_OBJ_NODE_OFF] = me.node_off;
    o.pad[RTX_OBJ_VERT_OFF] = me.vert_off;
    o.pad[RTX_OBJ_MFLAGS] = (me.node_count > 0 ? RTX_MESH_TREE : 0) | (me.has_normals ? RTX_MESH_NORMALS : 0) |
                            (me.has_vmats ? RTX_MESH_VMATS : 0);
  }
}

inline bool build_trav_trees(const RtxSceneDesc* d, TravTrees& T) {
  std::memset(&T.sroot, 0, sizeof(T.sroot));
  augment_objects(d, T.objs);
  // mesh-tree SAH parameters (the walk's results do not depend on the tree,
  // DESIGN.md "Traversal trees")
  const SahParams sp;
  const int mesh_leaf = 3;  // leaf codes hold <= 3 faces
  std::vector<RtxNode> nodes;
  std::vector<int> order;
  std::vector<TBox> boxes;
  if (d->n_objects > 0 && d->n_scene_nodes > 0) {
    boxes.resize(size_t(d->n_objects));
    for (int i = 0; i < d->n_objects; ++i)
      for (int k = 0; k < 3; ++k) {
        boxes[size_t(i)].lo[k] = d->objects[i].wmin[k];
        boxes[size_t(i)].hi[k] = d->objects[i].wmax[k];
      }
    tree_build(boxes, 1, nodes, order);
    for (auto& nd : nodes)
      if (nd.count > 0) nd.first = order[size_t(nd.first)];  // one object per leaf: the leaf names it
    if (!build_node4(nodes.data(), static_cast<int>(nodes.size()), T.sn4, T.sroot, T.sneed)) return false;
    for (int k = 0; k < 3; ++k) {  // the root test is the reference's own (KdTree::intersectList)
      T.sroot.lo[k] = d->scene_nodes[0].bmin[k];
      T.sroot.hi[k] = d->scene_nodes[0].bmax[k];
    }
  }
  T.mroots.assign(size_t(d->n_meshes), DevRoot());
  T.tfaces.assign(size_t(d->n_faces), RtxFace());
  T.trank.assign(size_t(d->n_faces), 0);
  T.tmeta.assign(size_t(d->n_faces), TMeta{0, 0});
  for (int m = 0; m < d->n_meshes; ++m) {
    const RtxMesh& me = d->meshes[m];
    std::memset(&T.mroots[size_t(m)], 0, sizeof(DevRoot));
    if (me.node_count <= 0 || me.face_count <= 0) continue;
    boxes.resize(size_t(me.face_count));
    for (int f = 0; f < me.face_count; ++f) {
      const RtxFace& F = d->faces[me.face_off + f];
      for (int k = 0; k < 3; ++k) {
        boxes[size_t(f)].lo[k] = fmin(fmin(F.v0[k], F.v1[k]), F.v2[k]);
        boxes[size_t(f)].hi[k] = fmax(fmax(F.v0[k], F.v1[k]), F.v2[k]);
      }
    }
    tree_build(boxes, mesh_leaf, nodes, order, sp);
    for (int j = 0; j < me.face_count; ++j) {
      T.tfaces[size_t(me.face_off + j)] = d->faces[me.face_off + order[size_t(j)]];
      T.trank[size_t(me.face_off + j)] = order[size_t(j)];
      T.tmeta[size_t(me.face_off + j)] = TMeta{order[size_t(j)], me.node_off + d->face_ids[me.face_off + order[size_t(j)]].leaf};
    }
    int need = 0;
    if (!build_node4(nodes.data(), static_cast<int>(nodes.size()), T.mn4, T.mroots[size_t(m)], need)) return false;
    const RtxNode& rr = d->mesh_nodes[me.node_off];  // the reference's root test
    for (int k = 0; k < 3; ++k) {
      T.mroots[size_t(m)].lo[k] = rr.bmin[k];
      T.mroots[size_t(m)].hi[k] = rr.bmax[k];
    }
    T.mneed = need > T.mneed ? need : T.mneed;
  }
  hot_mesh_records(T, 64);
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
