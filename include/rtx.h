/*
 * rtx.h — C ABI of librtx_hip.so, the MI355X (gfx950) ray-trace hot path.
 *
 * This is the drop-in boundary for the per-pixel path of the reference
 * (AlterionX/cs378hgraphics-raytracer).  The reference has no FFI: its
 * boundary is the C++ class API of RayTracer (ray/src/RayTracer.h:26-75),
 * called by CommandLineUI::run (ray/src/ui/CommandLineUI.cpp:149-190).
 * Each entry point below replaces one piece of that class:
 *
 *   rtx_scene_create   <- RayTracer::loadScene's result, uploaded once
 *                         (RayTracer.cpp:196-240; Scene::conclude,
 *                          scene/scene.cpp:145-153 builds the BVH on host)
 *   rtx_render         <- RayTracer::traceSetup + traceImage
 *                         (RayTracer.cpp:242-314), incl. tracePixel/trace/
 *                         traceRay/adaptaa (RayTracer.cpp:35-174,316-365)
 *   rtx_scene_destroy  <- ~RayTracer / Scene teardown
 *   rtx_last_error     <- traceUI->alert(msg) error reporting
 *
 * Plain pointers and sizes only.  Every function returns an rtx_status
 * (0 = ok, < 0 = error) and never throws across the ABI.  Host-side scene
 * loading (.ray parsing, BVH build, flattening into this layout) lives in
 * librtx_host.so, declared in rtx_host.h.
 *
 * Numerics: IEEE FP64 throughout, no FMA contraction, glm 0.9.8 operation
 * order (see cs378hgraphics-raytracer_amd/csrc/common/rt_math.h).
 */
#ifndef RTX_H_
#define RTX_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int rtx_status;
enum {
  RTX_OK = 0,
  RTX_ERR_INVALID = -1,   /* bad argument / unsupported option         */
  RTX_ERR_HIP = -2,       /* HIP runtime error (see rtx_last_error)     */
  RTX_ERR_NODEVICE = -3,  /* no gfx950 device visible                   */
  RTX_ERR_CAPACITY = -4,  /* scene exceeds a compiled limit             */
  RTX_ERR_FRAME = -5      /* a frame rendered into device buffers came
                             out wrong (rtx_frame_status names it)       */
};

/* ---- flat scene layout (host arrays; the library copies them to HBM) ---- */

/* BVH node, DFS pre-order.  Internal: child0 = this+1, child1 = `right`.
 * Leaf: items [first, first+count) of the owning item array (objects or
 * faces, stored in DFS-leaf order).  Mirrors KdTree<T> (scene/kdTree.h:19-130). */
typedef struct RtxNode {
  double bmin[3];
  double bmax[3];
  int32_t right;   /* internal: index of child1; leaf: -1            */
  int32_t first;   /* leaf: first item; internal: -1                 */
  int32_t count;   /* leaf: 1..3 (LEAF_NUM, kdTree.h:6); internal: 0 */
  int32_t depth;   /* depth of the node (root = 0)                   */
} RtxNode;         /* 64 bytes */

enum { RTX_OBJ_SPHERE = 0, RTX_OBJ_BOX = 1, RTX_OBJ_CYLINDER = 2,
       RTX_OBJ_SQUARE = 3, RTX_OBJ_TRIMESH = 4, RTX_OBJ_CONE = 5 };

/* Per-object shape parameters, RTX_OBJ_PARAMS doubles per object (parallel
 * to objects).  Cone (SceneObjects/Cone.h:11-37): height, b_radius,
 * t_radius, beta_squared, gamma, capped (0/1); unused otherwise. */
#define RTX_OBJ_PARAMS 8
enum { RTX_CONE_H = 0, RTX_CONE_BR, RTX_CONE_TR, RTX_CONE_B2, RTX_CONE_G, RTX_CONE_CAP };

/* Scene object (Geometry + TransformNode, scene/scene.h:64-188). */
typedef struct RtxObject {
  double wmin[3], wmax[3];  /* world box (Geometry::ComputeBoundingBox)       */
  double inv[12];           /* M^-1 columns 0..3, rows 0..2: inv[c*3+r]      */
  double normi[9];          /* transpose(inverse(mat3(M))): normi[c*3+r]      */
  int32_t type;             /* RTX_OBJ_*                                      */
  int32_t material;         /* index into materials                          */
  int32_t mesh;             /* index into meshes (trimesh) or -1              */
  int32_t orig_id;          /* index in Scene::objects (parse order)          */
  int32_t leaf;             /* scene-BVH leaf node holding this object        */
  int32_t pad[5];           /* to 256 bytes: two whole 128-byte lines         */
} RtxObject;                /* 256 bytes */

/* Material parameter: constant vec3 or texture (MaterialParameter,
 * scene/material.h:78-146).  tex < 0 means constant. */
typedef struct RtxParam {
  double v[3];
  int32_t tex;
  int32_t pad;
} RtxParam;

enum { RTX_P_KE = 0, RTX_P_KA, RTX_P_KS, RTX_P_KD, RTX_P_KR, RTX_P_KT,
       RTX_P_BUMP, RTX_P_SHININESS, RTX_P_INDEX, RTX_P_GLOSS, RTX_P_COUNT };

enum { RTX_MF_REFL = 1, RTX_MF_TRANS = 2, RTX_MF_RECUR = 4, RTX_MF_SPEC = 8,
       RTX_MF_BOTH = 16 };

typedef struct RtxMaterial {   /* Material, scene/material.h:148-278 */
  RtxParam p[RTX_P_COUNT];
  int32_t flags;               /* RTX_MF_* (setBools, material.h:272-276) */
  int32_t pad;
} RtxMaterial;

/* Triangle mesh (Trimesh, SceneObjects/trimesh.h:18-91). */
typedef struct RtxMesh {
  int32_t node_off, node_count;  /* mesh-local BVH nodes (local boxes)     */
  int32_t face_off, face_count;  /* faces in mesh-BVH DFS-leaf order       */
  int32_t vert_off, vert_count;  /* vertex normals / vertex materials base */
  int32_t has_normals;           /* per-vertex normals present             */
  int32_t has_vmats;             /* per-vertex materials present           */
} RtxMesh;

/* Face geometry (TrimeshFace, trimesh.h:93-164): vertices + unit normal. */
typedef struct RtxFace {
  double v0[3], v1[3], v2[3];
  double n[3];
} RtxFace;                       /* 96 bytes */

typedef struct RtxFaceIds {
  int32_t vi[3];                 /* mesh-local vertex indices              */
  int32_t orig_id;               /* index in Trimesh::faces                */
  int32_t leaf;                  /* mesh-BVH leaf node (mesh-relative)     */
  int32_t pad[3];
} RtxFaceIds;

/* Per-vertex material, already reduced to the parts Material::operator+=
 * and operator*(double, Material) touch (material.h:177-189, 281-293). */
typedef struct RtxVertexMaterial {
  double ke[3], ka[3], ks[3], kd[3], kr[3], kt[3];
  double shininess[3], index[3], gloss[3];
} RtxVertexMaterial;

enum { RTX_LIGHT_DIRECTIONAL = 0, RTX_LIGHT_POINT = 1, RTX_LIGHT_AREA_RECT = 2,
       RTX_LIGHT_AREA_CIRC = 3, RTX_LIGHT_SPOT = 4 };

typedef struct RtxLight {        /* Light family, scene/light.h:16-164 */
  int32_t type;
  int32_t pad;
  double color[3];
  double pos[3];                 /* point / area / spot position               */
  double orient[3];              /* normalized orientation (directional, area) */
  double atten[3];               /* float coefficients promoted to double      */
  double width, height, radius, angle, ang_tan, offset;  /* area / spot        */
  double u[3], v[3];             /* area-rect local axes                       */
} RtxLight;

typedef struct RtxTexture {
  int32_t width, height;
  int64_t offset;                /* byte offset into the texel pool (RGB8, row 0 = bottom) */
} RtxTexture;

typedef struct RtxCamera {       /* Camera, scene/camera.h:6-35 */
  double eye[3], look[3], u[3], v[3];
  double aspect;
} RtxCamera;

/* Whole scene, host-owned.  rtx_scene_create copies everything to HBM. */
typedef struct RtxSceneDesc {
  const RtxNode* scene_nodes;   int32_t n_scene_nodes;
  const RtxObject* objects;     int32_t n_objects;
  const RtxMaterial* materials; int32_t n_materials;
  const RtxMesh* meshes;        int32_t n_meshes;
  const RtxNode* mesh_nodes;    int32_t n_mesh_nodes;
  const RtxFace* faces;         int32_t n_faces;
  const RtxFaceIds* face_ids;
  const double* vnormals;       int32_t n_vnormals;    /* xyz triples           */
  const RtxVertexMaterial* vmats; int32_t n_vmats;
  const RtxLight* lights;       int32_t n_lights;
  const RtxTexture* textures;   int32_t n_textures;
  const uint8_t* texels;        int64_t n_texels;
  RtxCamera camera;
  double ambient[3];
  int32_t scene_depth;          /* max scene-BVH depth                         */
  int32_t mesh_depth;           /* max mesh-BVH depth over all meshes          */
  const double* obj_params;     /* RTX_OBJ_PARAMS per object (cone shapes)     */
  int32_t cubemap[6];           /* texture ids of the cube faces +x,-x,+y,-y,+z,-z
                                   (CubeMap::tMap, cubeMap.h); -1: no cube map   */
} RtxSceneDesc;

/* ---- render parameters (TraceUI flags, ui/TraceUI.h:34-129) ---- */
enum { RTX_AA_NONE = 0, RTX_AA_SUPERSAMPLE = 1, RTX_AA_ADAPTIVE = 2,
       RTX_AA_JITTERED = 3 };

typedef struct RtxRenderParams {
  int32_t width, height;        /* buffer size (CommandLineUI.cpp:155-156)     */
  int32_t depth;                /* -r                                          */
  int32_t aa_mode;              /* RTX_AA_*  (-O a/j/r)                        */
  int32_t aa_samples;           /* -A for a/j/r                                */
  int32_t dof;                  /* -O d                                        */
  int32_t dof_div;              /* -B for d                                    */
  int32_t anaglyph;             /* -O g                                        */
  int32_t ss_res;               /* -O s -A n (soft-shadow rays)                */
  int32_t overlapping;          /* -O o (Scene::discoverMat media)             */
  double aa_thresh;             /* -B for a                                    */
  double aterm_thresh;          /* -O c -A x                                   */
  double dof_fd;                /* -A for d                                    */
  double dof_apsz;              /* -C for d                                    */
  /* Tile sharding: the image is cut into tile x tile squares, numbered
   * row-major from the bottom-left, and dealt to shards diagonally: deal
   * index d is tile row d / tiles_x, column (d % tiles_x + row) % tiles_x,
   * and this call renders deal indices d with d % nshards == shard (packed
   * in increasing d).  tile == 0 renders the whole image. */
  int32_t tile;
  int32_t shard, nshards;
  int32_t packed;               /* 1: outputs packed per owned tile (tile*tile
                                   pixels each, in tile order); 0: full frame
                                   with the reference's (i + j*w) indexing   */
} RtxRenderParams;

/* Per-sample primary-ray hit record (first camera ray of each sample). */
typedef struct RtxHitRecord {
  int32_t object;      /* orig object id, -1 on miss                      */
  int32_t face;        /* orig face id within the mesh, -1 if not a mesh  */
  int32_t scene_leaf;  /* scene-BVH leaf node id, -1 on miss              */
  int32_t mesh_leaf;   /* mesh-BVH leaf node id, -1 if not a mesh hit     */
  int32_t nrays;       /* rays traced for this sample     */
  int32_t pad;
  double t;            /* world t of the primary hit (1000 on miss)       */
} RtxHitRecord;

typedef struct RtxStats {
  int64_t rays;          /* camera + reflect/refract traceRay calls + shadow queries */
  int64_t camera_rays;
  int64_t secondary_rays;
  int64_t shadow_rays;
  int64_t node_visits;   /* BVH node slab tests executed (scene + mesh) */
  int64_t object_tests;  /* Geometry::intersect calls                   */
  int64_t tri_tests;     /* TrimeshFace::intersectLocal calls           */
  int64_t shades;        /* Material::shade calls                       */
  double kernel_ms;      /* device time of the render kernel(s)         */
  int64_t shadow_traced; /* shadow queries actually traced: shadow_rays less the
                            dark lights counted but skipped */
} RtxStats;

/* ---- entry points ---- */
const char* rtx_last_error(void);                      /* thread-local message */
rtx_status rtx_device_count(int* n);
rtx_status rtx_scene_create(int device, const RtxSceneDesc* desc, void** scene);
rtx_status rtx_scene_destroy(void* scene);

/* Render.  Output pointers may be NULL.  When `device_ptrs` is nonzero the
 * outputs are device (HBM) pointers written asynchronously on `stream`
 * (a hipStream_t, NULL = default stream); otherwise they are host pointers
 * and the call is synchronous.
 * A synchronous render (host pointers, or `stats`) never returns RTX_OK with
 * a wrong image: when a frame sized from its own history (two-entry pending
 * stacks, a bucket-set pool of the last render's size) finds the history
 * short, the call renders the frame again with full-size buffers
 * (RTX_ERR_FRAME if that fails too).  An asynchronous render's outcome is
 * known only once its stream has run it: rtx_frame_status reports it.
 *   rgb8    : 3 bytes per pixel, (int)(255*c) truncation (RayTracer.cpp:388-394)
 *   rgb_f64 : 3 doubles per pixel, the value setPixel receives
 *   hits    : aa samples per pixel records (sample order si-major)
 * With `stats` non-NULL the call synchronizes and fills the counters
 * (the counting variant of the kernel is used: same results, slower). */
rtx_status rtx_render(void* scene, const RtxRenderParams* params,
                      uint8_t* rgb8, double* rgb_f64, RtxHitRecord* hits,
                      int device_ptrs, void* stream, RtxStats* stats);

/* Number of pixels this shard owns (size of packed outputs). */
rtx_status rtx_shard_pixels(const RtxRenderParams* params, int64_t* npixels);

/* Per-kernel work of the last render called with `stats` (the counting
 * variant of the kernels), RTX_WORK_COUNT int64 values, five per kernel
 * class — queries, BVH node visits, object tests, triangle tests, shades:
 *   [0..4]   batched closest-hit launches (trace_kernel<Q_CLOSEST>: camera,
 *            reflection and refraction rays; fused frames shade there too)
 *   [5..9]   batched next-hit launches (trace_kernel<Q_NEXT>: shadow walks)
 *   [10..14] tail launches (tail_kernel / tail_fused_kernel: both kinds)
 * A query is one traversal (a shadow walk is one query per hit it steps
 * through).  The megakernel path (RTX_MEGAKERNEL=1) leaves them 0.
 * `n` values are written (at most RTX_WORK_COUNT). */
#define RTX_WORK_COUNT 15
rtx_status rtx_last_work(void* scene, int64_t* out, int n);

/* Device time (ms) of the renders since the last call, read from hipEvents
 * recorded on the render stream (synchronizes those events), and the number
 * of kernels those renders launched (every launch of the render path). */
rtx_status rtx_kernel_time(void* scene, double* total_ms, int* launches);

/* Outcome of the asynchronous (device-buffer) renders issued so far on this
 * scene: waits for their device-side checks, then returns RTX_OK when every
 * one produced the image the reference would, or RTX_ERR_FRAME when one
 * did not (a history-sized buffer overflowed: the frame's later renders
 * already use full-size buffers).  *first_bad (may be NULL) receives the
 * 0-based sequence number of the first wrong frame among this scene's
 * rtx_render calls, -1 if none; *bad_frames (may be NULL) how many.  The
 * record is cleared by the call.  (Reference: traceImage always fills the
 * whole image, RayTracer.cpp:279-314 — a wrong frame is an error.) */
rtx_status rtx_frame_status(void* scene, int64_t* first_bad, int64_t* bad_frames);

/* How many rtx_render calls since the scene was created (or this counter
 * was last read) were pipelined — ran on the scene's alternating frame
 * contexts, free to overlap the frame before them (DESIGN.md "Frame
 * contexts") — out of *renders calls.  Either pointer may be NULL. */
rtx_status rtx_overlap_count(void* scene, int64_t* overlapped, int64_t* renders);

/* How many frame contexts the scene's last render rotated over (a
 * pipelined render waits only for the frame that last used its context:
 * with n contexts up to n frames are in flight; 1: the render was not
 * pipelined).  The library's choice: 3 for frames of at most 10 M work
 * units, 2 above (RTX_CONTEXTS caps it, 2..4).  No reference counterpart
 * (an extension of the pipelining above). */
rtx_status rtx_frame_contexts(void* scene, int32_t* n);

#ifdef __cplusplus
}
#endif
#endif /* RTX_H_ */
