// scene_build.cpp — the product's scene build: everything RayTracer::
// loadScene computes from the parsed attributes before the render starts.
//
//   TransformNode ctor          scene/scene.h:64-135 (xform = parent * local,
//                               inverse, normi = transpose(inverse(mat3)))
//   Geometry::ComputeBoundingBox scene/scene.cpp:78-116 (world box of the
//                               transformed local-box corners)
//   Camera                      scene/camera.cpp:39-111 (setLook, setFOV,
//                               setAspectRatio, quaternion, update)
//   Trimesh                     SceneObjects/trimesh.cpp:38-56 (addFace drops
//                               degenerate faces), :192-217 (generateNormals),
//                               trimesh.h:63-80, 100-161 (face normal, boxes)
//   light ctors                 scene/light.h:39-40, 102-104, 120-127, 153-155
//
// Matrix arithmetic is glm_compat.cpp's.  The CPU oracle does NOT link this
// file: it restates the same build on its own (oracle/scene_build_restated
// .cpp) from the parser's raw records, so an error here shows up as a parity
// failure instead of being shared by checker and product.
#include <cmath>
#include <fstream>

#include "scene_model.h"
#include "../common/rt_math.h"

namespace rtxh {

using rtm::mk3;

// ---------------------------------------------------------------- Camera
// camera.cpp:4 defines its own PI
static const double CAM_PI = 3.14159265359;

void Camera::update() {  // camera.cpp:94-99
  dvec3 ex = rtm::mat3_mul(m.m, mk3(1, 0, 0));
  dvec3 ey = rtm::mat3_mul(m.m, mk3(0, 1, 0));
  dvec3 ez = rtm::mat3_mul(m.m, mk3(0, 0, -1));
  u = (ex * normalizedHeight) * aspectRatio;
  v = ey * normalizedHeight;
  look = ez;
}

void Camera::setFOV(double fov) {  // camera.cpp:77-84
  fov /= (180.0 / CAM_PI);
  normalizedHeight = 2 * std::tan(fov / 2);
  update();
}

void Camera::setAspectRatio(double ar) {
  aspectRatio = ar;
  update();
}

void Camera::setLook(const dvec3& viewDir, const dvec3& upDir) {  // camera.cpp:64-74
  dvec3 z = -viewDir;
  const dvec3& y = upDir;
  dvec3 x = rtm::cross(y, z);
  // dmat3x3(x, y, z): columns
  m.m[0] = x.x; m.m[1] = x.y; m.m[2] = x.z;
  m.m[3] = y.x; m.m[4] = y.y; m.m[5] = y.z;
  m.m[6] = z.x; m.m[7] = z.y; m.m[8] = z.z;
  update();
}

void Camera::setLookQuat(double r, double i, double j, double k) {  // camera.cpp:39-62
  double a[3][3];  // a[c][r] as in the reference's m[c][r]
  a[0][0] = 1.0 - 2.0 * (i * i + j * j);
  a[0][1] = 2.0 * (r * i - j * k);
  a[0][2] = 2.0 * (j * r + i * k);
  a[1][0] = 2.0 * (r * i + j * k);
  a[1][1] = 1.0 - 2.0 * (j * j + r * r);
  a[1][2] = 2.0 * (i * j - r * k);
  a[2][0] = 2.0 * (j * r - i * k);
  a[2][1] = 2.0 * (i * j + r * k);
  a[2][2] = 1.0 - 2.0 * (i * i + r * r);
  Mat3 t;
  for (int c = 0; c < 3; ++c)
    for (int rr = 0; rr < 3; ++rr) t.m[c * 3 + rr] = a[c][rr];
  m = mat3_transpose(t);
  update();
}

namespace {

// the local matrix of one raw transform node (Parser.cpp:253-346)
Mat4 local_matrix(const XformOp& op) {
  switch (op.kind) {
    case XF_TRANSLATE: return mat4_translate(mk3(op.v[0], op.v[1], op.v[2]));
    case XF_ROTATE: return mat4_rotate(op.v[3], mk3(op.v[0], op.v[1], op.v[2]));
    case XF_SCALE: return mat4_scale(mk3(op.v[0], op.v[1], op.v[2]));
    default: {
      // glm::transpose(dmat4x4(row1..row4)): dmat4x4 takes the rows as columns
      Mat4 a;
      for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) a.m[c * 4 + r] = op.v[c * 4 + r];
      return mat4_transpose(a);
    }
  }
}

// TrimeshFace ctor + Trimesh::addFace (trimesh.h:100-130, trimesh.cpp:38-56)
void add_face(Mesh& me, int a, int b, int c) {
  const dvec3 A = me.verts[a], B = me.verts[b], C = me.verts[c];
  dvec3 vab = B - A, vac = C - A, vcb = B - C;
  if (rtm::length(vab) == 0.0 || rtm::length(vac) == 0.0 || rtm::length(vcb) == 0.0) return;  // degen
  dvec3 n = rtm::normalize(rtm::cross(B - A, C - A));
  // ComputeLocalBoundingBox (trimesh.h:149-161)
  dvec3 bmax = rtm::gmax3(A, B), bmin = rtm::gmin3(A, B);
  bmax = rtm::gmax3(C, bmax);
  bmin = rtm::gmin3(C, bmin);
  me.faces.push_back({a, b, c});
  me.face_normals.push_back(n);
  me.face_boxes.push_back({bmin, bmax});
}

void generate_normals(Mesh& me) {  // trimesh.cpp:192-217
  const size_t cnt = me.verts.size();
  me.normals.resize(cnt, dvec3{0, 0, 0});
  std::vector<int> numFaces(cnt, 0);
  for (size_t f = 0; f < me.faces.size(); ++f) {
    for (int i = 0; i < 3; ++i) {
      me.normals[me.faces[f][i]] += me.face_normals[f];
      ++numFaces[me.faces[f][i]];
    }
  }
  for (size_t i = 0; i < cnt; ++i)
    if (numFaces[i]) me.normals[i] = me.normals[i] / static_cast<double>(numFaces[i]);
}

void build_mesh(Mesh& me) {
  me.faces.clear();
  me.face_normals.clear();
  me.face_boxes.clear();
  for (const auto& f : me.raw_faces) add_face(me, f[0], f[1], f[2]);
  me.normals = me.raw_normals;
  if (me.gennormals) generate_normals(me);
  // ComputeLocalBoundingBox (trimesh.h:63-80)
  if (!me.verts.empty()) {
    me.lmax = me.verts[0];
    me.lmin = me.verts[0];
    for (const auto& v : me.verts) {
      me.lmax = rtm::gmax3(me.lmax, v);
      me.lmin = rtm::gmin3(me.lmin, v);
    }
    me.lbox_empty = false;
  }
}

// Geometry::ComputeBoundingBox (scene.cpp:78-116) over the local box
void world_box(const SceneModel& sc, Object& o) {
  dvec3 lmin, lmax;
  switch (o.type) {
    case OBJ_SPHERE: lmin = mk3(-1, -1, -1); lmax = mk3(1, 1, 1); break;
    case OBJ_BOX: lmin = mk3(-0.5, -0.5, -0.5); lmax = mk3(0.5, 0.5, 0.5); break;
    case OBJ_CYLINDER: lmin = mk3(-1, -1, 0); lmax = mk3(1, 1, 1); break;
    case OBJ_SQUARE: lmin = mk3(-0.5, -0.5, -0.00000001); lmax = mk3(0.5, 0.5, 0.00000001); break;
    case OBJ_CONE: {  // Cone::ComputeLocalBoundingBox (Cone.h:42-50)
      const double big = (o.cone_br > o.cone_tr) ? (o.cone_br) : (o.cone_tr);
      lmin = mk3(-big, -big, (o.cone_h < 0.0f) ? (o.cone_h) : (0.0f));
      lmax = mk3(big, big, (o.cone_h < 0.0f) ? (0.0f) : (o.cone_h));
      break;
    }
    case OBJ_TRIMESH: {  // an empty local box still yields corners at (0,0,0)
      const Mesh& me = sc.meshes[o.mesh];
      lmin = me.lmin;
      lmax = me.lmax;
      break;
    }
    default: lmin = lmax = mk3(0, 0, 0);
  }
  const dvec3 c[8] = {mk3(lmin.x, lmin.y, lmin.z), mk3(lmax.x, lmin.y, lmin.z), mk3(lmin.x, lmax.y, lmin.z),
                      mk3(lmax.x, lmax.y, lmin.z), mk3(lmin.x, lmin.y, lmax.z), mk3(lmax.x, lmin.y, lmax.z),
                      mk3(lmin.x, lmax.y, lmax.z), mk3(lmax.x, lmax.y, lmax.z)};
  double nmax[4], nmin[4];
  for (int k = 0; k < 8; ++k) {
    double in[4] = {c[k].x, c[k].y, c[k].z, 1.0}, v[4];
    mat4_mul_vec4(o.tf.xform, in, v);
    if (k == 0) {
      for (int a = 0; a < 4; ++a) nmax[a] = nmin[a] = v[a];
    } else {
      for (int a = 0; a < 4; ++a) {
        nmax[a] = rtm::gmax(nmax[a], v[a]);
        nmin[a] = rtm::gmin(nmin[a], v[a]);
      }
    }
  }
  o.wmax = mk3(nmax[0], nmax[1], nmax[2]);
  o.wmin = mk3(nmin[0], nmin[1], nmin[2]);
}

}  // namespace

void finalize_scene(SceneModel& sc) {
  if (sc.finalized) return;
  // camera attributes in file order
  for (const CamOp& op : sc.camera.ops) {
    switch (op.kind) {
      case CAM_FOV: sc.camera.setFOV(op.v[0]); break;
      case CAM_ASPECT: sc.camera.setAspectRatio(op.v[0]); break;
      case CAM_LOOK: sc.camera.setLook(mk3(op.v[0], op.v[1], op.v[2]), mk3(op.v[3], op.v[4], op.v[5])); break;
      case CAM_QUAT: sc.camera.setLookQuat(op.v[0], op.v[1], op.v[2], op.v[3]); break;
    }
  }
  for (Mesh& me : sc.meshes) build_mesh(me);
  // transform chains from the root node (make_transform(nullptr, I))
  const Transform root = make_transform(nullptr, mat4_identity());
  for (Object& o : sc.objects) {
    Transform t = root;
    for (const XformOp& op : o.chain) t = make_transform(&t, local_matrix(op));
    o.tf = t;
    world_box(sc, o);
  }
  for (Light& L : sc.lights) {
    if (L.type == L_POINT) continue;
    L.orient = rtm::normalize(L.raw_dir);  // DirectionalLight / AreaLight ctor (light.h:39-40, 102-104)
    if (L.type == L_AREA_RECT) {
      // AreaLightRect ctor (light.h:120-127): u(normalize(u)),
      // v(cross(ori, u)) where ori/u are the constructor PARAMETERS
      L.u = rtm::normalize(L.raw_up);
      L.v = rtm::cross(L.raw_dir, L.raw_up);
    }
    if (L.type == L_SPOT) {
      // SpotLight ctor (light.h:153-155), PI from util.h
      const double PI = 3.1415926535897932384626433832795028841971;
      L.ang_tan = std::tan(L.angle / 360 * PI);
      L.offset = L.ang_tan * L.radius;
    }
  }
  sc.finalized = true;
}

SceneModel load_ray_file(const std::string& path) {  // RayTracer::loadScene (RayTracer.cpp:196-240)
  SceneModel sc = parse_ray_file_raw(path);
  finalize_scene(sc);
  return sc;
}

}  // namespace rtxh
