// bvh_flatten.cpp — BVH build + flattening of a SceneModel into the HBM
// layout of rtx.h, and the librtx_host.so C ABI.
//
// The BVH reproduces KdTree<T> (ray/src/scene/kdTree.h:27-78) node for node:
// node box = merge of item boxes (bbox.cc:107-119); split axis = longest
// extent, ties keep the lower axis (strict '<' at kdTree.h:53); items sorted
// by libstdc++ std::sort on (max+min)[axis] (kdTree.h:57-65, same comparator
// outcomes => same permutation); split at n/2; leaf when n <= 3 (LEAF_NUM,
// kdTree.h:6).  The reference captures the index vector by value in its
// comparator (an O(n^2) copy cost); this build sorts an index array against a
// precomputed key array, which yields the identical tree in O(n log n).
//
// Nodes are emitted in DFS pre-order (child0 = next node), and leaf items are
// stored contiguously in DFS-leaf order, so the traversal order of the GPU
// kernel is exactly the candidate order of KdTree::intersectList
// (kdTree.h:100-117).
#include <algorithm>
#include <cstring>
#include <fstream>
#include <memory>
#include <numeric>
#include <sstream>
#include <string>

#include "../../../include/rtx_host.h"
#include "raw_records.h"
#include "scene_model.h"
#include "../common/rt_math.h"

namespace rtxh {
namespace {

struct Box {
  bool empty = true;
  dvec3 bmin{0, 0, 0}, bmax{0, 0, 0};
  void merge(const Box& b) {  // bbox.cc:107-119
    if (b.empty) return;
    double mn[3] = {bmin.x, bmin.y, bmin.z}, mx[3] = {bmax.x, bmax.y, bmax.z};
    for (int a = 0; a < 3; ++a) {
      if (empty || rtm::get(b.bmin, a) < mn[a]) mn[a] = rtm::get(b.bmin, a);
      if (empty || rtm::get(b.bmax, a) > mx[a]) mx[a] = rtm::get(b.bmax, a);
    }
    bmin = rtm::mk3(mn[0], mn[1], mn[2]);
    bmax = rtm::mk3(mx[0], mx[1], mx[2]);
    empty = false;
  }
};

struct Builder {
  const std::vector<Box>* boxes;
  std::vector<RtxNode> nodes;
  std::vector<int> order;  // DFS-leaf order of item ids
  int max_depth = 0;

  int build(const std::vector<int>& indexes, int depth) {
    if (indexes.empty()) return -1;
    const std::vector<Box>& bx = *boxes;
    Box b = bx[indexes[0]];
    for (int ix : indexes) b.merge(bx[ix]);
    int me = static_cast<int>(nodes.size());
    nodes.emplace_back();
    RtxNode& n0 = nodes.back();
    n0.bmin[0] = b.bmin.x; n0.bmin[1] = b.bmin.y; n0.bmin[2] = b.bmin.z;
    n0.bmax[0] = b.bmax.x; n0.bmax[1] = b.bmax.y; n0.bmax[2] = b.bmax.z;
    n0.depth = depth;
    max_depth = std::max(max_depth, depth);
    if (indexes.size() <= 3) {
      n0.right = -1;
      n0.first = static_cast<int>(order.size());
      n0.count = static_cast<int>(indexes.size());
      for (int x : indexes) order.push_back(x);
      return me;
    }
    n0.first = -1;
    n0.count = 0;
    int mx = 0;
    for (int i = 1; i < 3; ++i)
      if (rtm::get(b.bmax, mx) - rtm::get(b.bmin, mx) < rtm::get(b.bmax, i) - rtm::get(b.bmin, i)) mx = i;
    std::vector<double> key(indexes.size());
    for (size_t k = 0; k < indexes.size(); ++k) {
      const Box& q = bx[indexes[k]];
      key[k] = rtm::get(q.bmax, mx) + rtm::get(q.bmin, mx);
    }
    std::vector<int> idxs(indexes.size());
    std::iota(idxs.begin(), idxs.end(), 0);
    std::sort(idxs.begin(), idxs.end(), [&key](const int a, const int c) { return key[a] < key[c]; });
    const size_t mid = indexes.size() / 2;
    std::vector<int> split[2];
    for (size_t i = 0; i < indexes.size(); ++i) split[i < mid ? 0 : 1].push_back(indexes[idxs[i]]);
    build(split[0], depth + 1);
    int r = build(split[1], depth + 1);
    nodes[me].right = r;
    return me;
  }
};

uint64_t fnv(uint64_t h, const void* p, size_t n) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  for (size_t i = 0; i < n; ++i) {
    h ^= b[i];
    h *= 1099511628211ull;
  }
  return h;
}

// Structural hash: DFS pre-order node boxes, leaf item original ids.
uint64_t hash_tree(uint64_t h, const RtxNode* nodes, int n, const int32_t* leaf_items_orig) {
  for (int i = 0; i < n; ++i) {
    h = fnv(h, nodes[i].bmin, sizeof(double) * 3);
    h = fnv(h, nodes[i].bmax, sizeof(double) * 3);
    int32_t c = nodes[i].count;
    h = fnv(h, &c, 4);
    for (int k = 0; k < nodes[i].count; ++k) h = fnv(h, &leaf_items_orig[nodes[i].first + k], 4);
  }
  return h;
}

void put3(double* d, const dvec3& v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; }

}  // namespace

struct HostScene {
  std::vector<RtxNode> scene_nodes;
  std::vector<RtxObject> objects;
  std::vector<double> obj_params;  // RTX_OBJ_PARAMS per object
  int32_t cubemap[6] = {-1, -1, -1, -1, -1, -1};
  std::vector<RtxMaterial> materials;
  std::vector<RtxMesh> meshes;
  std::vector<RtxNode> mesh_nodes;
  std::vector<RtxFace> faces;
  std::vector<RtxFaceIds> face_ids;
  std::vector<double> vnormals;
  std::vector<RtxVertexMaterial> vmats;
  std::vector<RtxLight> lights;
  std::vector<RtxTexture> textures;
  std::vector<uint8_t> texels;
  RtxCamera camera;
  double ambient[3];
  RtxHostInfo info;
};

static RtxParam to_param(const MatParam& p) {
  RtxParam r;
  std::memset(&r, 0, sizeof(r));
  put3(r.v, p.v);
  r.tex = p.tex;
  return r;
}

static RtxMaterial to_material(const Material& m) {
  RtxMaterial r;
  std::memset(&r, 0, sizeof(r));
  for (int k = 0; k < P_COUNT; ++k) r.p[k] = to_param(m.p[k]);
  r.flags = (m.refl ? RTX_MF_REFL : 0) | (m.trans ? RTX_MF_TRANS : 0) | (m.recur ? RTX_MF_RECUR : 0) |
            (m.spec ? RTX_MF_SPEC : 0) | (m.both ? RTX_MF_BOTH : 0);
  return r;
}

std::unique_ptr<HostScene> flatten(const SceneModel& sc) {
  std::unique_ptr<HostScene> hs(new HostScene());
  HostScene& H = *hs;
  std::memset(&H.info, 0, sizeof(H.info));

  // ---- scene BVH over objects (world boxes)
  std::vector<Box> oboxes(sc.objects.size());
  for (size_t i = 0; i < sc.objects.size(); ++i) {
    oboxes[i].empty = false;
    oboxes[i].bmin = sc.objects[i].wmin;
    oboxes[i].bmax = sc.objects[i].wmax;
  }
  Builder sb;
  sb.boxes = &oboxes;
  std::vector<int> all(sc.objects.size());
  std::iota(all.begin(), all.end(), 0);
  sb.build(all, 0);
  H.scene_nodes = sb.nodes;
  std::vector<int> obj_leaf(sc.objects.size(), -1);
  for (size_t n = 0; n < sb.nodes.size(); ++n)
    for (int k = 0; k < sb.nodes[n].count; ++k) obj_leaf[sb.order[sb.nodes[n].first + k]] = static_cast<int>(n);

  // ---- meshes: per-mesh BVH over local face boxes
  std::vector<int> mesh_vbase(sc.meshes.size(), 0);
  int nv_total = 0;
  for (size_t m = 0; m < sc.meshes.size(); ++m) {
    const Mesh& me = sc.meshes[m];
    RtxMesh rm;
    std::memset(&rm, 0, sizeof(rm));
    std::vector<Box> fboxes(me.faces.size());
    for (size_t f = 0; f < me.faces.size(); ++f) {
      fboxes[f].empty = false;
      fboxes[f].bmin = me.face_boxes[f][0];
      fboxes[f].bmax = me.face_boxes[f][1];
    }
    Builder mb;
    mb.boxes = &fboxes;
    std::vector<int> fi(me.faces.size());
    std::iota(fi.begin(), fi.end(), 0);
    mb.build(fi, 0);
    rm.node_off = static_cast<int>(H.mesh_nodes.size());
    rm.node_count = static_cast<int>(mb.nodes.size());
    rm.face_off = static_cast<int>(H.faces.size());
    rm.face_count = static_cast<int>(me.faces.size());
    H.mesh_nodes.insert(H.mesh_nodes.end(), mb.nodes.begin(), mb.nodes.end());
    H.info.mesh_depth = std::max(H.info.mesh_depth, mb.max_depth);
    std::vector<int> face_leaf(me.faces.size(), -1);
    for (size_t n = 0; n < mb.nodes.size(); ++n)
      for (int k = 0; k < mb.nodes[n].count; ++k) face_leaf[mb.order[mb.nodes[n].first + k]] = static_cast<int>(n);
    for (int f : mb.order) {
      RtxFace rf;
      const auto& tri = me.faces[f];
      put3(rf.v0, me.verts[tri[0]]);
      put3(rf.v1, me.verts[tri[1]]);
      put3(rf.v2, me.verts[tri[2]]);
      put3(rf.n, me.face_normals[f]);
      H.faces.push_back(rf);
      RtxFaceIds id;
      std::memset(&id, 0, sizeof(id));
      id.vi[0] = tri[0]; id.vi[1] = tri[1]; id.vi[2] = tri[2];
      id.orig_id = f;
      id.leaf = face_leaf[f];
      H.face_ids.push_back(id);
    }
    rm.has_normals = me.normals.empty() ? 0 : 1;
    rm.has_vmats = me.vmats.empty() ? 0 : 1;
    rm.vert_count = static_cast<int>(me.verts.size());
    rm.vert_off = nv_total;
    mesh_vbase[m] = nv_total;
    if (rm.has_normals || rm.has_vmats) nv_total += rm.vert_count;
    H.meshes.push_back(rm);
  }
  H.vnormals.assign(size_t(nv_total) * 3, 0.0);
  H.vmats.resize(nv_total);
  std::memset(H.vmats.data(), 0, sizeof(RtxVertexMaterial) * H.vmats.size());
  for (size_t m = 0; m < sc.meshes.size(); ++m) {
    const Mesh& me = sc.meshes[m];
    const RtxMesh& rm = H.meshes[m];
    if (!(rm.has_normals || rm.has_vmats)) continue;
    for (int v = 0; v < rm.vert_count; ++v) {
      if (rm.has_normals) put3(&H.vnormals[size_t(rm.vert_off + v) * 3], me.normals[v]);
      if (rm.has_vmats) {
        // operator*(double, Material) / operator+= touch only the constant
        // values; texture-mapped parameters contribute their _value (0).
        const Material& vm = me.vmats[v];
        RtxVertexMaterial& o = H.vmats[rm.vert_off + v];
        put3(o.ke, vm.p[P_KE].v); put3(o.ka, vm.p[P_KA].v); put3(o.ks, vm.p[P_KS].v);
        put3(o.kd, vm.p[P_KD].v); put3(o.kr, vm.p[P_KR].v); put3(o.kt, vm.p[P_KT].v);
        put3(o.shininess, vm.p[P_SHININESS].v); put3(o.index, vm.p[P_INDEX].v);
        put3(o.gloss, vm.p[P_GLOSS].v);
      }
    }
  }
  (void)mesh_vbase;

  // ---- objects in DFS-leaf order
  for (int rank = 0; rank < static_cast<int>(sb.order.size()); ++rank) {
    int oi = sb.order[rank];
    const Object& o = sc.objects[oi];
    RtxObject ro;
    std::memset(&ro, 0, sizeof(ro));
    put3(ro.wmin, o.wmin);
    put3(ro.wmax, o.wmax);
    for (int c = 0; c < 4; ++c)
      for (int r = 0; r < 3; ++r) ro.inv[c * 3 + r] = o.tf.inverse.m[c * 4 + r];
    for (int k = 0; k < 9; ++k) ro.normi[k] = o.tf.normi.m[k];
    ro.type = o.type;
    ro.material = o.material;
    ro.mesh = o.mesh;
    ro.orig_id = oi;
    ro.leaf = obj_leaf[oi];
    H.objects.push_back(ro);
    double prm[RTX_OBJ_PARAMS] = {0.0};
    if (o.type == OBJ_CONE) {
      prm[RTX_CONE_H] = o.cone_h;
      prm[RTX_CONE_BR] = o.cone_br;
      prm[RTX_CONE_TR] = o.cone_tr;
      prm[RTX_CONE_B2] = o.cone_b2;
      prm[RTX_CONE_G] = o.cone_g;
      prm[RTX_CONE_CAP] = o.cone_capped ? 1.0 : 0.0;
      H.info.n_cones++;
    }
    H.obj_params.insert(H.obj_params.end(), prm, prm + RTX_OBJ_PARAMS);
  }
  // rewrite scene-leaf item ranges: already DFS-leaf order == object rank
  for (const Material& m : sc.materials) H.materials.push_back(to_material(m));

  // ---- lights
  for (const Light& L : sc.lights) {
    RtxLight rl;
    std::memset(&rl, 0, sizeof(rl));
    rl.type = L.type;
    put3(rl.color, L.color);
    put3(rl.pos, L.pos);
    put3(rl.orient, L.orient);
    rl.atten[0] = static_cast<double>(L.c);
    rl.atten[1] = static_cast<double>(L.l);
    rl.atten[2] = static_cast<double>(L.q);
    rl.width = L.width; rl.height = L.height; rl.radius = L.radius; rl.angle = L.angle;
    rl.ang_tan = L.ang_tan; rl.offset = L.offset;
    put3(rl.u, L.u);
    put3(rl.v, L.v);
    H.lights.push_back(rl);
    if (L.type >= L_AREA_RECT) H.info.n_area_lights++;
  }

  // ---- textures
  for (const Texture& t : sc.textures) {
    RtxTexture rt;
    rt.width = t.width;
    rt.height = t.height;
    rt.offset = static_cast<int64_t>(H.texels.size());
    H.texels.insert(H.texels.end(), t.data.begin(), t.data.end());
    H.textures.push_back(rt);
  }

  put3(H.camera.eye, sc.camera.eye);
  put3(H.camera.look, sc.camera.look);
  put3(H.camera.u, sc.camera.u);
  put3(H.camera.v, sc.camera.v);
  H.camera.aspect = sc.camera.aspectRatio;
  put3(H.ambient, sc.ambient);

  RtxHostInfo& I = H.info;
  I.n_objects = static_cast<int>(H.objects.size());
  I.n_lights = static_cast<int>(H.lights.size());
  I.n_meshes = static_cast<int>(H.meshes.size());
  I.n_faces = static_cast<int>(H.faces.size());
  I.n_textures = static_cast<int>(H.textures.size());
  I.n_scene_nodes = static_cast<int>(H.scene_nodes.size());
  I.n_mesh_nodes = static_cast<int>(H.mesh_nodes.size());
  I.scene_depth = sb.max_depth;
  I.aspect = sc.camera.aspectRatio;
  std::vector<int32_t> orig(H.objects.size());
  for (size_t r = 0; r < H.objects.size(); ++r) orig[r] = H.objects[r].orig_id;
  I.scene_bvh_hash = hash_tree(1469598103934665603ull, H.scene_nodes.data(),
                               static_cast<int>(H.scene_nodes.size()), orig.data());
  uint64_t mh = 1469598103934665603ull;
  for (const Object& o : sc.objects) {
    if (o.type != OBJ_TRIMESH) continue;
    const RtxMesh& rm = H.meshes[o.mesh];
    std::vector<int32_t> forig(rm.face_count);
    for (int f = 0; f < rm.face_count; ++f) forig[f] = H.face_ids[rm.face_off + f].orig_id;
    mh = hash_tree(mh, H.mesh_nodes.data() + rm.node_off, rm.node_count, forig.data());
  }
  I.mesh_bvh_hash = mh;
  return hs;
}

}  // namespace rtxh

// ======================================================== C ABI
namespace {
thread_local std::string g_host_err;
}

extern "C" {

const char* rtx_host_last_error(void) { return g_host_err.c_str(); }

rtx_status rtx_host_load(const char* ray_path, void** handle) {
  if (!ray_path || !handle) {
    g_host_err = "rtx_host_load: null argument";
    return RTX_ERR_INVALID;
  }
  try {
    rtxh::SceneModel sc = rtxh::load_ray_file(ray_path);
    std::unique_ptr<rtxh::HostScene> hs = rtxh::flatten(sc);
    *handle = hs.release();
    return RTX_OK;
  } catch (const std::exception& e) {
    g_host_err = e.what();
    return RTX_ERR_INVALID;
  }
}

rtx_status rtx_host_cubemap(void* handle, const char* one_cubemap_file) {
  if (!handle || !one_cubemap_file) {
    g_host_err = "rtx_host_cubemap: null argument";
    return RTX_ERR_INVALID;
  }
  rtxh::HostScene& H = *static_cast<rtxh::HostScene*>(handle);
  rtxh::Texture faces[6];
  std::string err;
  if (!rtxh::load_cubemap(one_cubemap_file, faces, err)) {
    g_host_err = err;
    return RTX_ERR_INVALID;
  }
  for (int k = 0; k < 6; ++k) {
    RtxTexture rt;
    rt.width = faces[k].width;
    rt.height = faces[k].height;
    rt.offset = static_cast<int64_t>(H.texels.size());
    H.texels.insert(H.texels.end(), faces[k].data.begin(), faces[k].data.end());
    H.cubemap[k] = static_cast<int32_t>(H.textures.size());
    H.textures.push_back(rt);
  }
  H.info.n_textures = static_cast<int>(H.textures.size());
  return RTX_OK;
}

rtx_status rtx_host_desc(void* handle, RtxSceneDesc* d) {
  if (!handle || !d) return RTX_ERR_INVALID;
  rtxh::HostScene& H = *static_cast<rtxh::HostScene*>(handle);
  std::memset(d, 0, sizeof(*d));
  d->scene_nodes = H.scene_nodes.data(); d->n_scene_nodes = static_cast<int32_t>(H.scene_nodes.size());
  d->objects = H.objects.data();         d->n_objects = static_cast<int32_t>(H.objects.size());
  d->materials = H.materials.data();     d->n_materials = static_cast<int32_t>(H.materials.size());
  d->meshes = H.meshes.data();           d->n_meshes = static_cast<int32_t>(H.meshes.size());
  d->mesh_nodes = H.mesh_nodes.data();   d->n_mesh_nodes = static_cast<int32_t>(H.mesh_nodes.size());
  d->faces = H.faces.data();             d->n_faces = static_cast<int32_t>(H.faces.size());
  d->face_ids = H.face_ids.data();
  d->vnormals = H.vnormals.data();       d->n_vnormals = static_cast<int32_t>(H.vnormals.size() / 3);
  d->vmats = H.vmats.data();             d->n_vmats = static_cast<int32_t>(H.vmats.size());
  d->lights = H.lights.data();           d->n_lights = static_cast<int32_t>(H.lights.size());
  d->textures = H.textures.data();       d->n_textures = static_cast<int32_t>(H.textures.size());
  d->texels = H.texels.data();           d->n_texels = static_cast<int64_t>(H.texels.size());
  d->camera = H.camera;
  for (int k = 0; k < 3; ++k) d->ambient[k] = H.ambient[k];
  d->scene_depth = H.info.scene_depth;
  d->mesh_depth = H.info.mesh_depth;
  d->obj_params = H.obj_params.data();
  for (int k = 0; k < 6; ++k) d->cubemap[k] = H.cubemap[k];
  return RTX_OK;
}

rtx_status rtx_host_info(void* handle, RtxHostInfo* info) {
  if (!handle || !info) return RTX_ERR_INVALID;
  *info = static_cast<rtxh::HostScene*>(handle)->info;
  return RTX_OK;
}

rtx_status rtx_host_free(void* handle) {
  delete static_cast<rtxh::HostScene*>(handle);
  return RTX_OK;
}

rtx_status rtx_write_image(const char* path, int32_t w, int32_t h, const uint8_t* rgb) {
  std::string err;
  if (!rtxh::write_image(path, w, h, rgb, &err)) {
    g_host_err = err;
    return RTX_ERR_INVALID;
  }
  return RTX_OK;
}

rtx_status rtx_host_tokens(const char* ray_path, char* out, int64_t cap, int64_t* need) {
  if (!ray_path || !need) {
    g_host_err = "rtx_host_tokens: null argument";
    return RTX_ERR_INVALID;
  }
  std::ifstream ifs(ray_path, std::ios::binary);
  if (!ifs) {
    g_host_err = std::string("Error: couldn't read scene file ") + ray_path;
    return RTX_ERR_INVALID;
  }
  std::stringstream ss;
  ss << ifs.rdbuf();
  const std::string t = rtxh::dump_ray_tokens(ss.str());
  *need = static_cast<int64_t>(t.size()) + 1;
  if (out) {
    if (cap < *need) {
      g_host_err = "rtx_host_tokens: output buffer too small";
      return RTX_ERR_INVALID;
    }
    std::memcpy(out, t.c_str(), t.size() + 1);
  }
  return RTX_OK;
}

rtx_status rtx_host_raw_records(const char* ray_path, char* out, int64_t cap, int64_t* need) {
  if (!ray_path || !need) {
    g_host_err = "rtx_host_raw_records: null argument";
    return RTX_ERR_INVALID;
  }
  std::string t;
  try {
    t = rtxh::dump_raw_records(rtxh::parse_ray_file_raw(ray_path));
  } catch (const std::exception& e) {
    t = std::string("ERROR\t") + e.what() + "\n";
  }
  *need = static_cast<int64_t>(t.size()) + 1;
  if (out) {
    if (cap < *need) {
      g_host_err = "rtx_host_raw_records: output buffer too small";
      return RTX_ERR_INVALID;
    }
    std::memcpy(out, t.c_str(), t.size() + 1);
  }
  return RTX_OK;
}

int32_t rtx_image_height(int32_t width, double aspect) {
  return static_cast<int32_t>(width / aspect + 0.5);
}

rtx_status rtx_read_image(const char* path, int32_t* w, int32_t* h, int32_t* channels, uint8_t* out, int64_t cap) {
  if (!path || !w || !h || !channels) {
    g_host_err = "rtx_read_image: null argument";
    return RTX_ERR_INVALID;
  }
  int iw = 0, ih = 0;
  std::vector<uint8_t> d;
  try {
    d = rtxh::read_image(path, iw, ih);
  } catch (const std::exception& e) {  // (bad_alloc on a huge image: an error, not terminate)
    g_host_err = std::string("rtx_read_image: ") + e.what();
    return RTX_ERR_INVALID;
  }
  if (d.empty()) {
    g_host_err = std::string("Unable to load texture map '") + path + "'.";
    return RTX_ERR_INVALID;
  }
  *w = iw;
  *h = ih;
  *channels = static_cast<int32_t>(d.size() / (size_t(iw) * ih));
  if (out) {
    if (cap < static_cast<int64_t>(d.size())) {
      g_host_err = "rtx_read_image: output buffer too small";
      return RTX_ERR_INVALID;
    }
    std::memcpy(out, d.data(), d.size());
  }
  return RTX_OK;
}

// the deal of rtx_render.hip (deal_tile): deal index d = shard + k * nshards
// is tile row d / tiles_x, column (d % tiles_x + row) % tiles_x
rtx_status rtx_shard_tiles(int32_t width, int32_t height, int32_t tile, int32_t shard, int32_t nshards, int32_t* ids,
                           int32_t cap, int32_t* count) {
  if (width <= 0 || height <= 0 || tile <= 0 || nshards <= 0 || shard < 0 || shard >= nshards || !count) {
    g_host_err = "rtx_shard_tiles: bad arguments";
    return RTX_ERR_INVALID;
  }
  const int32_t tx = (width + tile - 1) / tile, ty = (height + tile - 1) / tile;
  int32_t n = 0;
  for (int64_t d = shard; d < int64_t(tx) * ty; d += nshards, ++n) {
    if (!ids) continue;
    if (n >= cap) {
      g_host_err = "rtx_shard_tiles: id buffer too small";
      return RTX_ERR_INVALID;
    }
    const int32_t row = static_cast<int32_t>(d / tx);
    ids[n] = row * tx + static_cast<int32_t>((d % tx + row) % tx);
  }
  *count = n;
  return RTX_OK;
}

rtx_status rtx_unpack_tiles(const void* packed, int32_t width, int32_t height, int32_t tile, int32_t shard,
                            int32_t nshards, int32_t elem, void* frame) {
  if (!packed || !frame || elem <= 0) {
    g_host_err = "rtx_unpack_tiles: bad arguments";
    return RTX_ERR_INVALID;
  }
  int32_t n = 0;
  if (rtx_shard_tiles(width, height, tile, shard, nshards, nullptr, 0, &n) != RTX_OK) return RTX_ERR_INVALID;
  std::vector<int32_t> ids(n);
  rtx_shard_tiles(width, height, tile, shard, nshards, ids.data(), n, &n);
  const int32_t tx = (width + tile - 1) / tile;
  const uint8_t* src = static_cast<const uint8_t*>(packed);
  uint8_t* dst = static_cast<uint8_t*>(frame);
  for (int32_t k = 0; k < n; ++k) {
    const int32_t x0 = (ids[k] % tx) * tile, y0 = (ids[k] / tx) * tile;
    const int32_t cw = std::min(tile, width - x0), chh = std::min(tile, height - y0);
    for (int32_t r = 0; r < chh; ++r)
      std::memcpy(dst + (size_t(y0 + r) * width + x0) * elem, src + ((size_t(k) * tile + r) * tile) * elem,
                  size_t(cw) * elem);
  }
  return RTX_OK;
}

}  // extern "C"
