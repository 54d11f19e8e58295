/*
 * rtx_host.h — C ABI of librtx_host.so: host-side scene loading for the
 * MI355X hot path.  Replaces RayTracer::loadScene (ray/src/RayTracer.cpp:
 * 196-240: Tokenizer + Parser::parseScene, Parser.cpp:26-95), the BVH
 * builds done at load time (Scene::conclude, scene/scene.cpp:145-153;
 * Trimesh::conclude, SceneObjects/trimesh.cpp:69-77) and the image writer
 * used by CommandLineUI::run (fileio/images.cc:59-68).
 *
 * rtx_host_load parses a .ray file, builds both BVH levels exactly like
 * KdTree<T> (scene/kdTree.h:27-78) and flattens the scene into the
 * RtxSceneDesc layout of rtx.h, ready for rtx_scene_create.
 */
#ifndef RTX_HOST_H_
#define RTX_HOST_H_

#include <stdint.h>
#include "rtx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct RtxHostInfo {
  int32_t n_objects, n_lights, n_meshes, n_faces, n_textures;
  int32_t n_scene_nodes, n_mesh_nodes;
  int32_t scene_depth, mesh_depth;
  int32_t n_cones, n_area_lights;
  double aspect;                  /* RayTracer::aspectRatio (RayTracer.cpp:191-194) */
  uint64_t scene_bvh_hash;        /* FNV-1a over DFS pre-order node boxes + leaf items */
  uint64_t mesh_bvh_hash;         /* same over every mesh BVH, in object order       */
} RtxHostInfo;

const char* rtx_host_last_error(void);
/* Parse + build + flatten.  On error returns RTX_ERR_INVALID and the
 * message RayTracer::loadScene would alert (rtx_host_last_error). */
rtx_status rtx_host_load(const char* ray_path, void** handle);
rtx_status rtx_host_desc(void* handle, RtxSceneDesc* desc);   /* pointers into handle */
rtx_status rtx_host_info(void* handle, RtxHostInfo* info);
rtx_status rtx_host_free(void* handle);
/* -c FILE: TraceUI::smartLoadCubemap (ui/TraceUI.cc:97-167): the six cube
 * faces are the files of FILE's directory matched by matchCubemapFiles;
 * they join the scene's textures and RtxSceneDesc.cubemap names them.  On
 * failure returns RTX_ERR_INVALID with the message the reference prints to
 * stderr and leaves the scene without a cube map (the reference renders
 * on without one). */
rtx_status rtx_host_cubemap(void* handle, const char* one_cubemap_file);
/* writeImage (fileio/images.cc:59-68): .png / .bmp by extension, RGB8 with
 * buffer row 0 at the bottom. */
rtx_status rtx_write_image(const char* path, int32_t w, int32_t h, const uint8_t* rgb);
/* readImage (fileio/images.cc:47-53; readBMP bitmap.cpp:17-93, readPNG
 * pngimage.cpp:195-216): decodes `path` (.bmp / .png by extension) into
 * `out` (capacity `cap` bytes; NULL to query the size), row 0 = bottom,
 * `*channels` bytes per pixel (3, or 4 for a PNG with alpha).  Returns
 * RTX_ERR_INVALID when the file cannot be read (the reference then throws
 * "Unable to load texture map"). */
rtx_status rtx_read_image(const char* path, int32_t* w, int32_t* h, int32_t* channels, uint8_t* out, int64_t cap);
/* Multi-GPU tile partition, the host side of the deal the
 * kernels use (rtx_render.hip deal_tile): the tiles shard `shard` of
 * `nshards` renders, as row-major tile ids from the bottom-left, in its
 * packed order.  `ids` may be NULL to query the count. */
rtx_status rtx_shard_tiles(int32_t width, int32_t height, int32_t tile, int32_t shard, int32_t nshards,
                           int32_t* ids, int32_t cap, int32_t* count);
/* Scatter one shard's packed tiles (tile*tile pixels per tile, `elem`
 * bytes per pixel, rows from the bottom) into a full width x height frame
 * (row 0 = bottom) — the reassembly after the gather. */
rtx_status rtx_unpack_tiles(const void* packed, int32_t width, int32_t height, int32_t tile, int32_t shard,
                            int32_t nshards, int32_t elem, void* frame);
/* The tokenizer's view of a .ray file (Tokenizer(fp, printTokens = true),
 * parser/Tokenizer.cpp:39-46,119-123; token names of Token::toString,
 * Token.cpp:27-107): one token per line — its name, then a tab and the
 * identifier or the scalar as %.17g — ending with "EOF", or with "ERROR"
 * after the tokens read before a syntax error.  `out` (capacity `cap`
 * bytes, NUL-terminated) may be NULL to query `*need`. */
rtx_status rtx_host_tokens(const char* ray_path, char* out, int64_t cap, int64_t* need);
/* The raw parse records of a .ray file (Parser::parseScene's output before
 * any scene-build arithmetic: transform chains, material copies, mesh
 * vertex / face / normal lists, light attributes, camera ops) as canonical
 * text (csrc/host/raw_records.h), or "ERROR\t<the loader's message>" when
 * the parse fails.  Diagnostic: tests compare it with the checker's own
 * restated parser.  `out` may be NULL to query `*need`. */
rtx_status rtx_host_raw_records(const char* ray_path, char* out, int64_t cap, int64_t* need);
/* height the CLI derives from -w (CommandLineUI.cpp:156) */
int32_t rtx_image_height(int32_t width, double aspect);

#ifdef __cplusplus
}
#endif
#endif /* RTX_HOST_H_ */
