// scene_model.h — host-side scene model produced by the .ray loader.
//
// Plain data mirroring what the reference's Parser builds into a Scene
// (ray/src/parser/Parser.cpp:26-95, scene/scene.h:224-302): objects with
// their TransformNode matrices, per-object Material copies, lights, camera,
// ambient, trimesh data and texture maps.  The product flattens this into
// RtxSceneDesc (rtx.h) with its own BVH builder; the CPU oracle consumes it
// directly.  No device code here.
#pragma once

#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "../common/rt_types.h"

namespace rtxh {

using rtm::dvec3;

// glm 0.9.8 dmat4, column-major m[c*4 + r]
struct Mat4 {
  double m[16];
};
struct Mat3 {
  double m[9];  // column-major m[c*3 + r]
};

enum ParamIdx { P_KE = 0, P_KA, P_KS, P_KD, P_KR, P_KT, P_BUMP, P_SHININESS, P_INDEX, P_GLOSS, P_COUNT };

// MaterialParameter (scene/material.h:78-146).  A texture-mapped parameter
// keeps _value = 0 (glm 0.9.8 default constructor zero-initialises).
struct MatParam {
  dvec3 v{0.0, 0.0, 0.0};
  int tex = -1;
};

// Material (scene/material.h:148-278).  Flags follow setBools
// (material.h:272-276).  Decision U1: the flags the
// default constructor leaves uninitialised (_recur, _spec, _both) are false.
struct Material {
  MatParam p[P_COUNT];
  bool refl = false, trans = false, recur = false, spec = false, both = false;
  Material() { p[P_INDEX].v = dvec3{1.0, 1.0, 1.0}; }
  void setBools();
};

enum ObjType { OBJ_SPHERE = 0, OBJ_BOX = 1, OBJ_CYLINDER = 2, OBJ_SQUARE = 3, OBJ_TRIMESH = 4, OBJ_CONE = 5 };

struct Transform {
  Mat4 xform, inverse;
  Mat3 normi;
};

// ---- raw parse records --------------------------------------------------
// What the .ray text says, before any scene-build arithmetic.  The parser
// fills only these (plus materials, textures, colours, attenuation
// coefficients and raw vertex / face lists); finalize_scene() (product,
// scene_build.cpp) derives every Transform, world box, camera basis, mesh
// face record and light axis from them, and the CPU oracle derives the same
// quantities with its own restatement (oracle/scene_build_restated.cpp).
enum XformKind { XF_TRANSLATE = 0, XF_ROTATE = 1, XF_SCALE = 2, XF_MATRIX = 3 };
struct XformOp {
  int kind = XF_TRANSLATE;
  double v[16] = {0};  // translate / scale: x y z; rotate: axis x y z, angle (rad); matrix: the 4 rows as written
};
enum CamOpKind { CAM_FOV = 0, CAM_ASPECT = 1, CAM_LOOK = 2, CAM_QUAT = 3 };
struct CamOp {
  int kind = CAM_FOV;
  double v[6] = {0};  // fov (deg); aspect; look: viewdir xyz, updir xyz; quat: r i j k
};

// Geometry (scene/scene.h:140-188) with its world bounding box.
struct Object {
  int type = OBJ_SPHERE;
  int material = -1;  // index into SceneModel::materials
  int mesh = -1;      // index into SceneModel::meshes
  std::vector<XformOp> chain;  // raw: transform nodes from the root down to the object
  Transform tf;                // derived (finalize): root * chain[0] * ... * chain[n-1]
  dvec3 wmin{0, 0, 0}, wmax{0, 0, 0};
  bool has_box = true;  // hasBoundingBoxCapability() (true for every supported primitive)
  // Cone (Cone.h:11-37): height, b_radius, t_radius, beta_squared, gamma
  double cone_h = 1.0, cone_br = 1.0, cone_tr = 0.0, cone_b2 = 0.0, cone_g = 0.0;
  bool cone_capped = true;
};

// Trimesh (SceneObjects/trimesh.h:18-91).  faces holds only the
// non-degenerate faces, in Trimesh::faces order (addFace, trimesh.cpp:38-56).
struct Mesh {
  std::vector<dvec3> verts;
  // raw: fan-triangulated faces as parsed (indices range-checked), the
  // parsed per-vertex normals, and the gennormals flag
  std::vector<std::array<int, 3>> raw_faces;
  std::vector<dvec3> raw_normals;
  bool gennormals = false;
  // derived (finalize):
  std::vector<std::array<int, 3>> faces;
  std::vector<dvec3> face_normals;            // TrimeshFace::normal
  std::vector<std::array<dvec3, 2>> face_boxes;  // local bounds (min, max)
  std::vector<dvec3> normals;                 // per-vertex (may be empty)
  std::vector<Material> vmats;                // per-vertex materials (may be empty)
  dvec3 lmin{0, 0, 0}, lmax{0, 0, 0};         // ComputeLocalBoundingBox
  bool lbox_empty = true;
};

enum LightType { L_DIRECTIONAL = 0, L_POINT = 1, L_AREA_RECT = 2, L_AREA_CIRC = 3, L_SPOT = 4 };

// Light family (scene/light.h:16-164).  Attenuation coefficients are stored
// as float, exactly like PointLight's members (light.h:86-88).
struct Light {
  int type = L_POINT;
  dvec3 color{0, 0, 0};
  dvec3 pos{0, 0, 0};
  dvec3 raw_dir{0, 0, 0}, raw_up{0, 0, 0};  // raw: direction / updir attributes
  dvec3 orient{0, 0, 0};  // derived: normalized (DirectionalLight / AreaLight ctor)
  float c = 0.0f, l = 0.0f, q = 1.0f;
  double width = 0, height = 0, radius = 0, angle = 0;  // raw
  double ang_tan = 0, offset = 0;                        // derived (SpotLight ctor)
  dvec3 u{0, 0, 0}, v{0, 0, 0};                          // derived: area-rect axes
};

struct Texture {
  std::string path;
  int width = 0, height = 0;
  std::vector<uint8_t> data;  // RGB8, row 0 = bottom row of the file
};

// Camera (scene/camera.cpp).  eye and ops are raw (the camera block's
// attributes in file order; viewdir + updir become one CAM_LOOK at the
// block's end, as Parser.cpp:97-154 applies them); m .. v are derived.
struct Camera {
  std::vector<CamOp> ops;
  Mat3 m{{1, 0, 0, 0, 1, 0, 0, 0, 1}};  // default identity (glm 0.9.8 default dmat3)
  double normalizedHeight = 1.0;
  double aspectRatio = 1.0;
  dvec3 eye{0, 0, 0};
  dvec3 look{0, 0, -1};
  dvec3 u{1, 0, 0};
  dvec3 v{0, 1, 0};
  void update();
  void setFOV(double fov);
  void setAspectRatio(double ar);
  void setLook(const dvec3& viewDir, const dvec3& upDir);
  void setLookQuat(double r, double i, double j, double k);
};

struct SceneModel {
  std::vector<Object> objects;      // Scene::objects, parse order
  std::vector<Material> materials;  // one per object (MaterialSceneObject owns a copy)
  std::vector<Mesh> meshes;
  std::vector<Light> lights;
  std::vector<Texture> textures;
  Camera camera;
  dvec3 ambient{0, 0, 0};
  std::string base_path;
  bool finalized = false;  // derived fields filled (finalize_scene)
};

struct ParseError : public std::runtime_error {
  explicit ParseError(const std::string& m) : std::runtime_error(m) {}
};

// Parse a .ray file (Parser::parseScene semantics) into the raw records.
// Throws ParseError with the reference's messages on malformed input.
SceneModel parse_ray_file_raw(const std::string& path);
SceneModel parse_ray_text(const std::string& text, const std::string& base_path);
// the tokenizer's output, one token per line (rtx_host_tokens)
std::string dump_ray_tokens(const std::string& text);
// Product scene build (scene_build.cpp): the derived fields from the raw
// records (TransformNode ctor, Geometry::ComputeBoundingBox, Camera,
// Trimesh::addFace / generateNormals / ComputeLocalBoundingBox, light ctors).
void finalize_scene(SceneModel& sc);
// parse_ray_file_raw + finalize_scene: RayTracer::loadScene's scene.
SceneModel load_ray_file(const std::string& path);

// glm 0.9.8 matrix helpers (glm_compat.cpp)
Mat4 mat4_identity();
Mat4 mat4_mul(const Mat4& a, const Mat4& b);
Mat4 mat4_translate(const dvec3& v);
Mat4 mat4_scale(const dvec3& v);
Mat4 mat4_rotate(double angle, const dvec3& axis);
Mat4 mat4_transpose(const Mat4& a);
Mat4 mat4_inverse(const Mat4& a);
Mat3 mat3_from4(const Mat4& a);
Mat3 mat3_inverse(const Mat3& a);
Mat3 mat3_transpose(const Mat3& a);
Mat3 mat3_identity();
dvec3 mat4_mul_point(const Mat4& m, const dvec3& v);  // scene.h:57-62
void mat4_mul_vec4(const Mat4& m, const double v[4], double out[4]);
Transform make_transform(const Transform* parent, const Mat4& local);

// Image I/O (image_io.cpp)
std::vector<uint8_t> read_image(const std::string& path, int& w, int& h);
// TraceUI::matchCubemapFiles + smartLoadCubemap's TextureMap loads
// (TraceUI.cc:87-167): fills faces[0..5] (+x,-x,+y,-y,+z,-z) or returns false
// with the message the reference prints.
bool load_cubemap(const std::string& one_cubemap_file, Texture faces[6], std::string& err);
bool write_image(const std::string& path, int w, int h, const uint8_t* rgb, std::string* err);

}  // namespace rtxh
