/*
 * oracle.h — CPU restatement of the reference ray-trace path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle.so, and only as the checker
 * (or as the timed CPU baseline).  The product (librtx_hip.so, bin/ray) never
 * links or calls it.
 *
 * PARITY STATUS vs the original binary: UNPINNED.  The reference cannot be
 * built here (glm 0.9.8.4 is not vendored, <FL/gl.h> is absent, see
 * SURVEY.md 8(c)) and ships no golden vectors or known-answer tests for this
 * path; the only shipped renders are of scenes that are not in the repo.
 * This oracle is pinned instead by (a) line-by-line restatement of the
 * reference sources cited at every function, (b) analytic known-answer tests
 * (tests/test_oracle_kat.py) and (c) committed fixtures it generates
 * (tests/golden/).
 */
#ifndef RTX_ORACLE_H_
#define RTX_ORACLE_H_

#include <stdint.h>
#include "../include/rtx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct OracleRect {
  int32_t x0, y0, x1, y1;  /* pixel rectangle [x0,x1) x [y0,y1); x1 == 0 => full image */
  int32_t threads;         /* OpenMP threads, 0 = default                           */
} OracleRect;

const char* oracle_last_error(void);
/* RayTracer::aspectRatio (RayTracer.cpp:191-194) of the restated camera;
 * < 0 on a load error. */
double oracle_aspect(const char* ray_path);
/* Render `ray_path` with the reference algorithm.  Outputs are full-frame
 * (reference buffer indexing (i + j*w)*3); only pixels inside `rect` are
 * written.  hits: aa-samples-per-pixel records (NULL allowed).
 * cubemap_file: -c (NULL or "": none). */
int oracle_render(const char* ray_path, const char* cubemap_file, const RtxRenderParams* params,
                  const OracleRect* rect, uint8_t* rgb8, double* rgb_f64, RtxHitRecord* hits, RtxStats* stats);
/* The restated scene build (scene_build_restated.cpp) of `ray_path`: per
 * object (parse order) 27 doubles — world box min, max (6), inverse rows
 * 0..2 as inv[c*3+r] (12), normi[c*3+r] (9); and the camera's eye, look, u,
 * v (12).  *n = object count; objs may be NULL to query it. */
int oracle_scene_dump(const char* ray_path, double* objs, int32_t cap, int32_t* n, double* cam);
/* Structural hashes of the oracle's own KdTree builds (same definition as
 * RtxHostInfo.scene_bvh_hash / mesh_bvh_hash). */
int oracle_bvh_hash(const char* ray_path, uint64_t* scene_hash, uint64_t* mesh_hash);
/* Single-ray probe for known-answer tests: closest hit of the world ray
 * (p, d) against the scene.  Returns 1 on hit. */
int oracle_probe(const char* ray_path, const double p[3], const double d[3], double* t, double n[3],
                 int32_t* object, int32_t* face);

/* The raw parse records of the oracle's own loader (parse_restated.cpp) in
 * the canonical text of csrc/host/raw_records.h ("ERROR\t<message>" on a
 * parse error), and its tokenizer's stream in rtx_host_tokens' format.
 * `out` may be NULL to query `*need`. */
int oracle_raw_records(const char* ray_path, char* out, int64_t cap, int64_t* need);
int oracle_tokens(const char* ray_path, char* out, int64_t cap, int64_t* need);

/* Batched closest-hit (mode 0) or sorted all-hits (mode 1, kmax per ray)
 * queries for the traversal unit test. */
int oracle_query_batch(const char* ray_path, int32_t n, const double* P, const double* D, int32_t mode,
                       int32_t kmax, double* t, int32_t* object, int32_t* face, int32_t* nhits);

#ifdef __cplusplus
}
#endif
#endif
