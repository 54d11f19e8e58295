// traverse_host.hip — TEST HARNESS: the device traversal (rtx_traverse.h,
// the code every render kernel runs) compiled for the HOST so the unit test
// tests/test_traverse_host.py can compare it query by query with the CPU
// restatement's Scene::intersect / sorted intersectList on thousands of rays
// without a GPU.  Built with --offload-host-only; never shipped, never used
// by the product.
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../cs378hgraphics-raytracer_amd/csrc/hip/rtx_traverse.h"

using namespace rtxd;

namespace {
std::string g_err;

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
  S.n_srec = static_cast<int32_t>(H.T.sn4.size());
  S.mroots = H.T.mroots.data();
  S.tfaces = H.T.tfaces.data();
  S.trank = H.T.trank.data();
  S.snodes = d->scene_nodes;
  S.objs = H.T.objs.data();  // with the mesh fields in pad (augment_objects)
  S.tmeta = H.T.tmeta.data();
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
}  // namespace

extern "C" {

const char* trav_host_last_error(void) { return g_err.c_str(); }

// qmode 1: closest hit per ray -> t/object/face (orig ids), 1 entry.
// qmode 2: the shadow walk's successive next-hit queries, up to kmax entries
//          per ray, each query bounded by tlimit[k] (1e308 = unbounded).
// counters[3] += node box tests, object tests, triangle tests.
int trav_host_run(const RtxSceneDesc* d, int32_t qmode, int32_t n, const double* P, const double* D,
                  const double* tlimit, int32_t kmax, double* t, int32_t* object, int32_t* face, int32_t* nhits,
                  int64_t* counters) {
  HostScene H;
  if (!make_scene(d, H)) {
    g_err = "malformed BVH";
    return -1;
  }
  std::vector<int> stk(size_t(H.stack_cap + 4) * 64, 0);
  Counters C = {0, 0, 0, 0, 0, 0, 0};
  for (int32_t k = 0; k < n; ++k) {
    const dvec3 p = mk3(P[3 * k], P[3 * k + 1], P[3 * k + 2]);
    const dvec3 dd = mk3(D[3 * k], D[3 * k + 1], D[3 * k + 2]);
    double tp = -RTX_INF;
    int rp = -1, sq = -1, cnt = 0;
    const int kk = qmode == Q_CLOSEST ? 1 : kmax;
    for (int j = 0; j < kk; ++j) {
      t[size_t(k) * kk + j] = 0.0;
      object[size_t(k) * kk + j] = -1;
      face[size_t(k) * kk + j] = -1;
    }
    for (int j = 0; j < kk; ++j) {
      double bt;
      int bobj, bsub;
      const bool have = traverse<true>(H.S, qmode, p, dd, tp, rp, sq, qmode == Q_CLOSEST ? RTX_INF : tlimit[k], bt,
                                       bobj, bsub, stk.data(), 0, C);
      // the runtime-mode instantiation (tail kernels, megakernel) must agree
      // bit for bit; a disagreement poisons the answer (object -999)
      double bt2;
      int bobj2, bsub2;
      Counters C2 = C;
      const bool have2 = traverse_any<true>(H.S, qmode, p, dd, tp, rp, sq,
                                            qmode == Q_CLOSEST ? RTX_INF : tlimit[k], bt2, bobj2, bsub2, stk.data(), 0,
                                            C2);
      if (have2 != have || (have && (bt2 != bt || bobj2 != bobj || bsub2 != bsub))) {
        object[size_t(k) * kk + j] = -999;
        ++cnt;
        break;
      }
      if (!have) break;
      const RtxObject& o = d->objects[bobj];
      t[size_t(k) * kk + j] = bt;
      object[size_t(k) * kk + j] = o.orig_id;
      face[size_t(k) * kk + j] =
          o.type == RTX_OBJ_TRIMESH ? d->face_ids[d->meshes[o.mesh].face_off + bsub].orig_id : -1;
      ++cnt;
      tp = bt;
      rp = bobj;
      sq = bsub;
    }
    nhits[k] = cnt;
  }
  counters[0] += C.nodes;
  counters[1] += C.objects;
  counters[2] += C.tris;
  return 0;
}

// The float record test (box_cons32, as visit4 runs it) on n (ray, box)
// pairs: box k = (lo[6k..6k+3), hi[6k+3..6k+6)) in double, stored the way the
// records store it (rounded outward to float); ok[k] = 1 when the entry
// passes.  The test harness compares with an exact geometric slab.
int rec_test_host(int32_t n, const double* P, const double* D, const double* box, int32_t* ok, float* a_out) {
  for (int32_t k = 0; k < n; ++k) {
    const dvec3 p = mk3(P[3 * k], P[3 * k + 1], P[3 * k + 2]);
    const dvec3 d = mk3(D[3 * k], D[3 * k + 1], D[3 * k + 2]);
    const RayF rf = ray_f(p, d, ray_inv(d));
    DevNode4 nd;
    std::memset(&nd, 0, sizeof(nd));
    for (int q = 0; q < 3; ++q) {
      nd.lo[q][0] = round_down_f(box[6 * k + q]);
      nd.hi[q][0] = round_up_f(box[6 * k + 3 + q]);
    }
    nd.count = 1;
    float a, b;
    ok[k] = box_cons32(nd, 0, rf, a, b) ? 1 : 0;
    a_out[k] = a;
  }
  return 0;
}

// The record walk's prune bounds (f_up_wide / f_down_wide) for n doubles.
int prune_bounds_host(int32_t n, const double* x, float* up, float* dn) {
  for (int32_t k = 0; k < n; ++k) {
    up[k] = f_up_wide(x[k]);
    dn[k] = f_down_wide(x[k]);
  }
  return 0;
}

// Per-ray traversal cost of closest queries (record entries, object tests,
// face tests): which rays make the long queries (tools/ray_cost_probe.py).
int trav_host_cost(const RtxSceneDesc* d, int32_t n, const double* P, const double* D, int64_t* nodes,
                   int64_t* objs, int64_t* tris, int32_t* object) {
  HostScene H;
  if (!make_scene(d, H)) {
    g_err = "malformed BVH";
    return -1;
  }
  std::vector<int> stk(size_t(H.stack_cap + 4) * 64, 0);
  for (int32_t k = 0; k < n; ++k) {
    Counters C = {0, 0, 0, 0, 0, 0, 0};
    double bt;
    int bobj, bsub;
    const bool have = traverse<true>(H.S, Q_CLOSEST, mk3(P[3 * k], P[3 * k + 1], P[3 * k + 2]),
                                     mk3(D[3 * k], D[3 * k + 1], D[3 * k + 2]), -RTX_INF, -1, -1, RTX_INF, bt, bobj,
                                     bsub, stk.data(), 0, C);
    nodes[k] = C.nodes;
    objs[k] = C.objects;
    tris[k] = C.tris;
    object[k] = have ? d->objects[bobj].orig_id : -1;
  }
  return 0;
}

}  // extern "C"
