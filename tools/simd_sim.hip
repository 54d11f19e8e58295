// simd_sim.hip — TOOL (not product, not a test): the device traversal
// (rtx_traverse.h) compiled for the host and stepped 64 lanes at a time the
// way trace_kernel's step loop steps a wave, to count how often each unit
// class (4-wide record / object / mesh leaf) is executed by a wave under a
// lane-selection policy.  A wave step runs the code of every class that has
// a stepping lane, so the wave-level cost of a policy is
//   sum over classes of (wave steps that ran the class) x (its code's cost).
// Used by tools/simd_sim.py to evaluate postponement policies on CPU.
#include <cstdint>
#include <cstring>
#include <vector>

#include "../cs378hgraphics-raytracer_amd/csrc/hip/rtx_traverse.h"

using namespace rtxd;

namespace {
struct HostScene {
  DevScene S;
  TravTrees T;
  int stack_cap = 0;
};

bool make_scene(const RtxSceneDesc* d, HostScene& H) {
  std::memset(&H.S, 0, sizeof(H.S));
  DevScene& S = H.S;
  if (!build_trav_trees(d, H.T)) return false;
  S.sroot = H.T.sroot;
  S.snode4 = H.T.sn4.data();
  S.mnode4 = H.T.mn4.data();
  S.mhot = S.mnode4;
  S.n_mhot = H.T.n_mhot;
  S.n_srec = static_cast<int32_t>(H.T.sn4.size());
  S.mroots = H.T.mroots.data();
  S.tfaces = H.T.tfaces.data();
  S.trank = H.T.trank.data();
  S.tmeta = H.T.tmeta.data();
  S.snodes = d->scene_nodes;
  S.objs = H.T.objs.data();
  S.oprm = d->obj_params;
  S.mats = d->materials;
  S.meshes = d->meshes;
  S.mnodes = d->mesh_nodes;
  S.faces = d->faces;
  S.fids = d->face_ids;
  S.n_snodes = d->n_scene_nodes;
  S.n_objs = d->n_objects;
  S.margin = 1e-9 * scene_extent(d);
  S.lmargin = 1e-9 * mesh_extent(d);
  H.stack_cap = H.T.sneed + H.T.mneed + 2;
  return true;
}

enum { C_REC = 0, C_OBJ = 1, C_LEAF = 2 };
int unit_class(const Trav& T) {
  if (T.mode != 1 && T.ref >= 0) return C_REC;
  if (T.mode == 1 || T.mode == 0) return C_OBJ;  // (mode 0 with a leaf ref: the leaf's objects are next)
  return C_LEAF;
}
}  // namespace

extern "C" {

// policy 0: trace_kernel's rule (records only while >= k1 lanes are at a
//           record, else every active lane);
// policy 1: one class per wave step: records while >= k1 lanes are at a
//           record; else the class with the most lanes if it has >= k2,
//           else every active lane;
// policy 2: like 0, but when the wave steps everything, lanes at a leaf
//           wait while fewer than k2 of them are (and some other lane can
//           step).
// qmode 1 closest (tlimit ignored), 2 next-hit from key (-inf, -1, -1)
// bounded by tlimit[k].
// out[0..2]: wave steps that ran records / objects / leaves; out[3..5]:
// lane steps of each class; out[6]: wave steps; out[7]: queries.
int simd_sim_run(const RtxSceneDesc* d, int32_t qmode, int32_t n, const double* P, const double* D,
                 const double* tlimit, int32_t policy, int32_t k1, int32_t k2, int64_t* out) {
  HostScene H;
  if (!make_scene(d, H)) return -1;
  const DevScene& S = H.S;
  std::vector<int> stk(size_t(H.stack_cap) * 64 + 64);
  for (int k = 0; k < 8; ++k) out[k] = 0;
  const NoBlocker nb;
  for (int base = 0; base < n; base += 64) {
    Trav T[64];
    bool act[64];
    Counters C = {};
    for (int l = 0; l < 64; ++l) {
      act[l] = false;
      const int q = base + l;
      if (q >= n) continue;
      const dvec3 p = mk3(P[q * 3], P[q * 3 + 1], P[q * 3 + 2]);
      const dvec3 dd = mk3(D[q * 3], D[q * 3 + 1], D[q * 3 + 2]);
      out[7]++;
      if (qmode == 1)
        act[l] = trav_init<false, Q_CLOSEST>(T[l], S, p, dd, -RTX_INF, -1, -1, RTX_INF, -RTX_INF, C);
      else
        act[l] = trav_init<false, Q_NEXT>(T[l], S, p, dd, -RTX_INF, -1, -1, tlimit[q], -RTX_INF, C);
    }
    for (;;) {
      int cnt[3] = {0, 0, 0}, nact = 0;
      int cls[64];
      for (int l = 0; l < 64; ++l) {
        if (!act[l]) continue;
        cls[l] = unit_class(T[l]);
        cnt[cls[l]]++;
        nact++;
      }
      if (nact == 0) break;
      bool go_cls[3] = {true, true, true};
      if (cnt[C_REC] >= k1) {
        go_cls[C_OBJ] = go_cls[C_LEAF] = false;
      } else if (policy == 1) {
        int best = C_OBJ;
        if (cnt[C_LEAF] > cnt[best]) best = C_LEAF;
        if (cnt[C_REC] > cnt[best]) best = C_REC;
        if (cnt[best] >= k2)
          for (int c = 0; c < 3; ++c) go_cls[c] = c == best;
      } else if (policy == 2) {
        if (cnt[C_LEAF] < k2 && cnt[C_REC] + cnt[C_OBJ] > 0) go_cls[C_LEAF] = false;
      }
      bool ran[3] = {false, false, false};
      for (int l = 0; l < 64; ++l) {
        if (!act[l] || !go_cls[cls[l]]) continue;
        ran[cls[l]] = true;
        out[3 + cls[l]]++;
        bool done;
        if (qmode == 1)
          done = trav_step<false, Q_CLOSEST>(T[l], S, stk.data(), l, nb, C);
        else
          done = trav_step<false, Q_NEXT>(T[l], S, stk.data(), l, nb, C);
        if (done) act[l] = false;
      }
      for (int c = 0; c < 3; ++c) out[c] += ran[c];
      out[6]++;
    }
  }
  return 0;
}
}
