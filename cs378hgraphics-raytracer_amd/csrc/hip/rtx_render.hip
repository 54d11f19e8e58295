// rtx_render.hip — gfx950 render kernels + the C ABI of include/rtx.h.
//
// Design:
//   * ONE traversal loop per wave, shared by every query a lane can have —
//     closest hit of a camera / reflection / refraction ray, or the next hit
//     of a shadow ray's ordered walk — so lanes that are at different points
//     of their sample still traverse together.  The loop is flattened over
//     the three levels (scene node / object / mesh node): each iteration
//     processes one unit, the per-lane stack lives in LDS.
//   * Around it, a per-lane state machine restates trace/traceRay/shade/
//     srsAttenuation (RayTracer.cpp:35-174, material.cpp:34-69,
//     light.cpp:16-53): camera ray -> pending-ray stack -> shade light by
//     light -> shadow walk hit by hit.
//   * Lanes refill with new samples as soon as they finish (ballot + popc
//     + mbcnt over a wave-local queue fed 256 samples per atomic), so the
//     wave stays full; sample colours go to an HBM sample buffer and a
//     second kernel sums each pixel's samples in the reference's si-major
//     order (RayTracer.cpp:288-298).
//   * Adaptive AA (RayTracer.cpp:316-365) runs one pixel per wave with the
//     region recursion kept wave-uniform.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <set>
#include <string>
#include <type_traits>
#include <map>
#include <vector>

#include "rtx_device.h"

using namespace rtxd;
using rtm::dvec2;
using rtm::dvec3;
using rtm::mk3;

#define WG 256  // threads per workgroup (64 / 128 measured within noise)
#define WAVES_PER_WG (WG / 64)
// -r limit: the pending-ray stack holds depth + 2 entries per slot in HBM
// and the slot pool shrinks to fit device memory, so this only bounds the
// stack's size (the reference's recursion is bounded by its C stack)
#define MAX_DEPTH 4096
#define QCHUNK 256                 // samples per queue atomic
// occupancy targets (waves per SIMD) of the wavefront kernels, measured on
// the headline frame: traversal at 3 waves (<= 168 VGPRs, no spills) beats 4
// (128 VGPRs + scratch spills) and 2; the state-machine kernel is left
// unconstrained
#ifndef RTX_TRACE_WAVES
#define RTX_TRACE_WAVES 3
#endif
#ifndef RTX_ADV_WAVES
#define RTX_ADV_WAVES 1
#endif


// ============================================================ frame parameters
// A region of adaptaa's recursion below the pixel (RayTracer.cpp:316-365):
// its rectangle in image coordinates, the region of the level above that
// subdivided (`parent`: a pixel's output slot at level 1) and which quarter
// it is (child = 2a + b of adaptaa's loops).
struct ARegion {
  double x1, x2, y1, y2;
  int parent, child;
};

struct FrameParams {
  RtxRenderParams P;
  RtxCamera cam;
  const double* offv;        // DoF eye offsets [divs][3] in HBM (RayTracer.cpp:64-69), host cos/sin
  int spp;                   // samples per pixel (1 or s^2)
  int s;                     // s (AA grid)
  int ppw;                   // pixels per work item
  int bw, bh;                // pixel block shape of one item
  int tw, th;                // tile size (whole image if no tiling)
  int tiles_x, tiles_y;
  int n_owned;               // owned tiles
  int items_per_tile;
  int bx_per_tile;           // blocks per tile row
  int64_t n_items;           // work items (pixel blocks)
  int64_t n_samples;         // n_items * ppw * spp  (sample ids)
  int qchunk;                // samples per queue atomic (multiple of 64)
  int wf_nslot;              // wavefront path: path slots (samples dealt slot + k * wf_nslot)
  int ncam;                  // camera rays per sample (1, or divs + 1 with DoF)
  int cam_split;             // 1: each DoF camera ray is its own work unit (wavefront path)
  // wavefront slot layout: G groups of wf_gs slots; the first wf_gsamp slots
  // of a group take samples (sample slot g * wf_gsamp + l, samples dealt
  // sample slot + k * wf_nslot), the rest are fork slots
  int wf_gs, wf_gsamp, wf_groups;
  // ray-tree buckets (wavefront path, no DoF / anaglyph; DESIGN.md "Ray-tree
  // forking"): the rays at heap positions 2 .. fork_npos + 1 of a sample's
  // ray tree (root 1, children 2p and 2p + 1, down to heap depth
  // fork_depth) are nodes; every other ray belongs to its nearest node
  // ancestor.  A ray's colour goes to its node's bucket — the root's to the
  // lane's acc, node p's to fbuf[sample][p - 2] (first write sets bit p - 2
  // of fmask[sample]) — and reduce_kernel adds the buckets in heap order
  // before the clamp.  A bucket's sum is the same whether its node ran on
  // the sample's own slot or was forked onto a spare slot, so the image does
  // not depend on which nodes won a fork slot.
  int fork_on, fork_npos;
  double* fbuf;
  unsigned int* fmask;
  // Bucket sets are pooled: only a unit whose root ray has a child (a node
  // at heap position 2 or 3) has buckets, and it takes set bidx[unit] from
  // the pool when its root is shaded (bucket_alloc: once per unit, by the
  // unit's own lane, before any child exists — so the count is the same on
  // every render of the same frame).  fbuf holds bcap sets; *bcnt counts
  // the sets taken; *bover is set if one is refused (the host sizes bcap
  // from the last render of the same frame, full size otherwise).
  int* bidx;
  unsigned int* bcnt;
  unsigned int* bover;
  int bcap;
  // fused shadow walks (rtx_fused.h): the finished terms of the walks,
  // wterm[(unit * nslot + slot) * 3 + c].  Light l's units start at
  // lunit[l]: a point or directional light has one (its term); an area or
  // spot light (area_mask bit l) has 2 + ss_res — its factors (dattn, d + s;
  // mode) and one attenuation per pick (rtx_fused.h "Area lights").  A slot's
  // walk records of light l start at record lrec[l] of its nrec (the tail
  // kernel's fixed positions).
  int fuse;
  double* wterm;
  int lunit[8], lrec[8];
  int nrec, area_mask;
  // adaptive AA on the wavefront path: a work unit is (region, Hammersley
  // index k) — level 0's regions are the pixels (item_pixel), a deeper
  // level's are aregs[0 .. n_samples / spp) (adapt_stats_kernel)
  int adapt;
  const ARegion* aregs;
  // bounds of the frame's device buffers (the bounds-check build's RTX_CHK,
  // DESIGN.md §5): bucket owners (bidx / fmask), wterm units, sample-buffer
  // entries, per-group live-list entries
  int64_t chk_units, chk_samples;
  int chk_wunits, chk_live;
};

// ---- bounds-check build (-DRTX_BOUNDS_CHECK, tools/build_variants.sh): every
// slot, query-record, live-list, bucket, pick, wterm and stack index the
// wavefront kernels compute is checked against its buffer's extent; the
// first violation (site, index, bound) and a count go to rtx_chk_state and
// the access is redirected to index 0 instead of faulting; rtx_render (host
// buffers) and rtx_frame_status (device buffers) report a violation as
// RTX_ERR_INVALID.  Without the flag RTX_CHK(site, i, n) is i.
#ifdef RTX_BOUNDS_CHECK
__device__ unsigned long long rtx_chk_state[3];  // count, first (site << 48 | index), its bound
__device__ __noinline__ long long rtx_chk_fail(int site, long long i, long long n) {
  const unsigned long long c = atomicAdd(&rtx_chk_state[0], 1ull);
  if (c == 0ull) {
    rtx_chk_state[1] = (static_cast<unsigned long long>(site) << 48) | (static_cast<unsigned long long>(i) & 0xffffffffffffull);
    rtx_chk_state[2] = static_cast<unsigned long long>(n);
  }
  return 0;
}
#define RTX_CHK(site, i, n) \
  ((static_cast<long long>(i) >= 0 && static_cast<long long>(i) < static_cast<long long>(n)) ? (i) \
                                                                                            : static_cast<std::remove_reference_t<decltype(i)>>(rtx_chk_fail(site, static_cast<long long>(i), static_cast<long long>(n))))
constexpr bool kBoundsCheck = true;
#else
#define RTX_CHK(site, i, n) (i)
constexpr bool kBoundsCheck = false;
#endif
// sites
enum { CHK_SLOT = 1, CHK_QREC, CHK_LIVE, CHK_FREE, CHK_BUNIT, CHK_BSET, CHK_BPOS, CHK_PEND, CHK_STACK, CHK_LIGHT,
       CHK_PICK, CHK_WUNIT, CHK_SAMPLE };

// Tile deal: deal index d = shard + k * nshards is tile row d / tiles_x,
// column (d % tiles_x + row) % tiles_x — row-major with each row rotated by
// its index, so shards own diagonal stripes of tiles rather than columns
// when nshards divides tiles_x (render cost is correlated along columns:
// 2-way shards of the headline frame 49.5 / 42.0 ms with column stripes).
// The same deal is restated by the host (rtx_shard_tiles, librtx_host) and
// by the Python mirror (owned_tiles); a test checks all three agree.
__host__ __device__ __forceinline__ void deal_tile(int d, int tiles_x, int& tx, int& ty) {
  ty = d / tiles_x;
  tx = (d % tiles_x + ty) % tiles_x;
}
__host__ __device__ __forceinline__ int tile_deal(int tx, int ty, int tiles_x) {
  return ty * tiles_x + ((tx - ty) % tiles_x + tiles_x) % tiles_x;
}

// Work item -> pixel; out_index is the output slot (packed tile order or
// (i + j*w) reference order).
__device__ __forceinline__ bool item_pixel(const FrameParams& F, int64_t item, int pix_in_item, int& i, int& j,
                                           int64_t& out_index) {
  const int k = static_cast<int>(item / F.items_per_tile);
  const int b = static_cast<int>(item % F.items_per_tile);
  int tx, ty;
  deal_tile(F.P.tile > 0 ? F.P.shard + k * F.P.nshards : 0, F.tiles_x, tx, ty);
  const int bx = b % F.bx_per_tile, by = b / F.bx_per_tile;
  const int lx = bx * F.bw + pix_in_item % F.bw;
  const int ly = by * F.bh + pix_in_item / F.bw;
  if (lx >= F.tw || ly >= F.th) return false;
  i = tx * F.tw + lx;
  j = ty * F.th + ly;
  if (i >= F.P.width || j >= F.P.height) return false;
  if (F.P.packed && F.P.tile > 0)
    out_index = static_cast<int64_t>(k) * F.tw * F.th + static_cast<int64_t>(ly) * F.tw + lx;
  else
    out_index = static_cast<int64_t>(i) + static_cast<int64_t>(j) * F.P.width;
  return true;
}

__device__ __forceinline__ double radinv2(int n) {  // hammersley x (util.cpp:3-11)
  double mul = 0.5, result = 0.0;
  while (n > 0) {
    result += (n % 2) ? mul : 0;
    n /= 2;
    mul /= 2.0;
  }
  return result;
}

#include "rtx_traverse.h"

// Recompute the winning entry's local quantities (deterministic: same
// operations as the traversal) and resolve the isect the reference returns:
// world normal (scene.cpp:31-33), uv, and where its material comes from.
// Material parameters are then evaluated one at a time where the state
// machine needs them (hit_param & co.), not all ten up front: the shading
// kernel's register peak is set by how much of a material is live at once.
struct HitRef {
  dvec3 N;
  dvec2 uv;
  dvec3 bary;
  int mat;          // material index (objects without per-vertex materials)
  int vm_off;       // >= 0: per-vertex materials of the mesh (vi valid)
  int vi0, vi1, vi2;
};

// Inlined by default: out of line (-DRTX_RESOLVE_NOINLINE) the shading
// kernel needs 4 fewer VGPRs but pays a 224-byte scratch frame per call, and
// the frame took 130.1 ms instead of 127.8.  The kernels pass S as *Sg (the
// device copy), so an out-of-line call never has to spill the by-value
// kernel-argument copy.
#define RTX_RESOLVE_ATTR __forceinline__
__device__ RTX_RESOLVE_ATTR HitRef resolve_hit(const DevScene& S, const dvec3& P, const dvec3& D, int oi, int sub,
                              int* rec_face, int* rec_mleaf) {
  HitRef r;
  const RtxObject& o = S.objs[oi];
  const RtxMaterial& mat = S.mats[o.material];
  dvec3 pos, dir;
  obj_local(o, P, D, pos, dir);
  dir = rtm::normalize(dir);
  dvec3 nl = mk3(0.0, 0.0, 1.0);
  dvec2 uv = rtm::mk2(0.0, 0.0);
  if (rec_face) {
    *rec_face = -1;
    *rec_mleaf = -1;
  }
  if (o.type == RTX_OBJ_TRIMESH) {
    // the mesh's fields ride in the object record (augment_objects)
    const int face_off = o.pad[RTX_OBJ_FACE_OFF], vert_off = o.pad[RTX_OBJ_VERT_OFF];
    const int mflags = o.pad[RTX_OBJ_MFLAGS];
    const RtxFace F = S.faces[face_off + sub];
    const RtxFaceIds fi = S.fids[face_off + sub];
    double tl = 0.0;
    tri_hit(F, pos, dir, RTX_INF, tl);
    const dvec3 bary = tri_bary(F, pos, dir, tl);
    if (mflags & RTX_MESH_NORMALS) {  // trimesh.cpp:166-172
      const dvec3 n0 = ld3(S.vnormals + size_t(vert_off + fi.vi[0]) * 3);
      const dvec3 n1 = ld3(S.vnormals + size_t(vert_off + fi.vi[1]) * 3);
      const dvec3 n2 = ld3(S.vnormals + size_t(vert_off + fi.vi[2]) * 3);
      const double mm[9] = {n0.x, n0.y, n0.z, n1.x, n1.y, n1.z, n2.x, n2.y, n2.z};
      nl = rtm::normalize(rtm::mat3_mul(mm, bary));
    } else {
      nl = ld3(F.n);
    }
    r.bary = bary;
    r.vm_off = (mflags & RTX_MESH_VMATS) ? vert_off : -1;
    r.vi0 = fi.vi[0];
    r.vi1 = fi.vi[1];
    r.vi2 = fi.vi[2];
    if (rec_face) {
      *rec_face = fi.orig_id;
      *rec_mleaf = fi.leaf;
    }
  } else {
    if (o.type == RTX_OBJ_SPHERE) {
      const dvec3 d2 = rtm::normalize(dir);
      const dvec3 v = -pos;
      const double bb = rtm::dot(v, d2);
      const double disc = sqrt(bb * bb - rtm::dot(v, v) + 1);
      const double t = sub == 0 ? bb - disc : bb + disc;
      nl = rtm::normalize(rtm::ray_at(pos, d2, t));
    } else if (o.type == RTX_OBJ_BOX) {
      const int it = sub, mod0 = it % 3;
      const double t = ((it / 3) - 0.5 - rtm::get(pos, mod0)) / rtm::get(dir, mod0);
      const dvec3 ip = rtm::ray_at(pos, dir, t);
      const int i1 = (it + 1) % 3, i2 = (it + 2) % 3;
      const int lo = i1 < i2 ? i1 : i2, hi = i1 < i2 ? i2 : i1;
      uv = (it < 3) ? rtm::mk2(0.5 - rtm::get(ip, lo), 0.5 + rtm::get(ip, hi))
                    : rtm::mk2(0.5 + rtm::get(ip, lo), 0.5 + rtm::get(ip, hi));
      nl = box_normal(S, mat, it, uv);
    } else if (o.type == RTX_OBJ_CYLINDER) {
      const double dz = dir.z;
      if (sub == 0) {
        nl = dz > 0.0 ? mk3(0.0, 0.0, -1.0) : mk3(0.0, 0.0, 1.0);
      } else if (sub == 1) {
        nl = dz > 0.0 ? mk3(0.0, 0.0, 1.0) : mk3(0.0, 0.0, -1.0);
      } else {
        const double x0 = pos.x, y0 = pos.y, x1 = dir.x, y1 = dir.y;
        const double aa = x1 * x1 + y1 * y1;
        const double bb = 2.0 * (x0 * x1 + y0 * y1);
        const double cc = x0 * x0 + y0 * y0 - 1.0;
        const double disc = sqrt(bb * bb - 4.0 * aa * cc);
        const double t = sub == 2 ? (-bb - disc) / (2.0 * aa) : (-bb + disc) / (2.0 * aa);
        const dvec3 Q = rtm::ray_at(pos, dir, t);
        nl = rtm::normalize(mk3(Q.x, Q.y, 0.0));
      }
    } else if (o.type == RTX_OBJ_CONE) {  // Cone.cpp:45-101 normals
      const double* prm = S.oprm + size_t(oi) * RTX_OBJ_PARAMS;
      const double dz = dir.z;
      if (sub == 2) {
        nl = dz > 0.0 ? mk3(0.0, 0.0, -1.0) : mk3(0.0, 0.0, 1.0);
      } else if (sub == 3) {
        nl = dz > 0.0 ? mk3(0.0, 0.0, 1.0) : mk3(0.0, 0.0, -1.0);
      } else {
        const ConeRoots cr = cone_roots(prm, pos, dir);
        const dvec3 Q = rtm::ray_at(pos, dir, sub == 0 ? cr.near_t : cr.far_t);
        dvec3 n = mk3(Q.x, Q.y, -2.0 * prm[RTX_CONE_B2] * (Q.z + prm[RTX_CONE_G]));
        if (!(prm[RTX_CONE_CAP] != 0.0) && rtm::dot(n, dir) > 0) n = -n;
        nl = rtm::normalize(n);
      }
    } else if (o.type == RTX_OBJ_SQUARE) {
      const double t = -pos.z / dir.z;
      const dvec3 Q = rtm::ray_at(pos, dir, t);
      nl = dir.z > 0.0 ? mk3(0.0, 0.0, -1.0) : mk3(0.0, 0.0, 1.0);
      uv = rtm::mk2(Q.x + 0.5, Q.y + 0.5);
    }
    r.bary = mk3(0.0, 0.0, 0.0);
    r.vm_off = -1;
    r.vi0 = r.vi1 = r.vi2 = 0;
  }
  r.mat = o.material;
  r.uv = uv;
  r.N = rtm::normalize(rtm::mat3_mul(o.normi, nl));
  return r;
}

// One material parameter at a hit: MaterialParameter::value
// (material.cpp:140-146), or the per-vertex interpolation
// Material() += b_k * M_k (trimesh.cpp:157-163, index starts at 1).
__device__ __forceinline__ dvec3 hit_param(const DevScene& S, const HitRef& h, int k) {
  if (h.vm_off >= 0) {
    const int f = k <= RTX_P_KT ? 3 * k : (k == RTX_P_SHININESS ? 18 : (k == RTX_P_INDEX ? 21 : 24));
    dvec3 e = k == RTX_P_INDEX ? mk3(1.0, 1.0, 1.0) : mk3(0.0, 0.0, 0.0);
    e += ld3(reinterpret_cast<const double*>(&S.vmats[h.vm_off + h.vi0]) + f) * h.bary.x;
    e += ld3(reinterpret_cast<const double*>(&S.vmats[h.vm_off + h.vi1]) + f) * h.bary.y;
    e += ld3(reinterpret_cast<const double*>(&S.vmats[h.vm_off + h.vi2]) + f) * h.bary.z;
    return e;
  }
  return pval(S, S.mats[h.mat].p[k], h.uv);
}
// shininess (material.h:204-209: a texture map is scaled by 128)
// A parameter's constant value at a hit, what Material::operator+= adds
// (textured parameters: their _value, 0); per-vertex materials: the
// interpolated value
__device__ __forceinline__ dvec3 hit_raw(const DevScene& S, const HitRef& h, int k) {
  if (h.vm_off >= 0) return hit_param(S, h, k);
  return ld3(S.mats[h.mat].p[k].v);
}
__device__ __forceinline__ double hit_shininess(const DevScene& S, const HitRef& h) {
  if (h.vm_off >= 0) return intensity(hit_param(S, h, RTX_P_SHININESS));
  const RtxParam& shp = S.mats[h.mat].p[RTX_P_SHININESS];
  return shp.tex >= 0 ? 128.0 * intensity(pval(S, shp, h.uv)) : intensity(ld3(shp.v));
}
__device__ __forceinline__ double hit_index(const DevScene& S, const HitRef& h) {
  return intensity(hit_param(S, h, RTX_P_INDEX));
}
// per-vertex materials never get setBools (decision U2: flags 0)
__device__ __forceinline__ int hit_flags(const DevScene& S, const HitRef& h) {
  return h.vm_off >= 0 ? 0 : S.mats[h.mat].flags;
}

// ============================================================ lights
__device__ __forceinline__ dvec3 light_dir(const RtxLight& L, const dvec3& P) {
  if (L.type == RTX_LIGHT_DIRECTIONAL) return -ld3(L.orient);  // light.cpp:59
  return rtm::normalize(ld3(L.pos) - P);                       // light.cpp:73
}

__device__ __forceinline__ double light_dist_atten(const RtxLight& L, const dvec3& P) {
  if (L.type == RTX_LIGHT_DIRECTIONAL) return 1.0;  // light.cpp:56
  const double d = rtm::distance(ld3(L.pos), P);    // light.cpp:61-64 (float terms promoted)
  return rtm::gclamp(1.0 / (L.atten[0] + L.atten[1] * d + L.atten[2] * d * d), 0.0, 1.0);
}

// Bounds of a shadow walk's next-hit query (DESIGN.md "Shadow walk"):
//   tlim: hits past it cannot change the walk's result.  For a point light
//     the U14 limit check trips past the light, and for the walk's FIRST hit
//     already past half the light distance (the double advance puts its
//     check point at twice the hit distance, light.cpp:38,66).
__device__ __forceinline__ double shadow_limit(const DevScene& S, const RtxLight& L, const dvec3& qP, bool first) {
  if (L.type != RTX_LIGHT_POINT) return RTX_INF;
  const double dl = rtm::distance(qP, ld3(L.pos));
  return (first ? 0.5 * dl : dl) * (1.0 + 1e-6) + S.margin;
}

// ============================================================ lane state machine
enum { ST_IDLE = 0, ST_CAM, ST_POP, ST_HIT, ST_LIGHT, ST_SRS, ST_WALK, ST_RECUR, ST_DISC, ST_WALK2 };
// discoverMat walks (-O o) return to: 1 ST_RECUR (traceRay), 2 ST_WALK2 (srsAttenuation)
enum { DISC_NONE = 0, DISC_RECUR = 1, DISC_WALK = 2 };

struct Pending {
  dvec3 p, d, W, ktf;
  int depth, kind;  // kind 0 camera, 1 reflection, 2 refraction
};

// Per-lane state of one sample's path (everything the state machine keeps
// between traversal queries, plus the last query's result).  It lives in HBM
// (L2 / Infinity-Cache resident), one array per field indexed by lane, so a
// wave's access to a field is one contiguous 64-lane line set, and no kernel
// has to hold the whole state in VGPRs: the state machine touches only the
// fields of its current step, and the traversal's registers are not shared
// with it.  LaneRef gives a lane's fields as accessors (LR.st(), LR.acc(), ...).
// The fields the fused machine (rtx_fused.h, claim_sample, lane_init) uses
// come first in each list: a fused frame allocates only those
// (LANE_*_FUSED of each type: 16 ints, 2 doubles, 3 vectors = 152 B per
// slot instead of 668), the others are the sequential machine's.
#define LANE_INT_FIELDS(X) X(st) X(sample_slot) X(rec_on) X(pass) X(camk) X(nrays) X(top) X(first_query) X(cam_end) \
  X(qmode) X(kdone) X(fpos) X(rpos) X(wmask) X(bunit) X(dret) \
  X(rdepth) X(rkind) X(sobj) X(ssub) X(m_flags) X(li) X(pick) X(qrp) X(qsq) X(bobj) X(bsub) X(bhave) \
  X(dpass) X(dpush) X(dhead) X(dtot) X(dlast) X(dopq) X(mo_trans) X(wobj) X(wsub)
#define LANE_DBL_FIELDS(X) X(sx) X(sy) X(st_t) X(m_sh) X(dattn) X(last_t) X(qtp) X(bt) X(mo_idx) X(wt) X(wtr)
#define LANE_VEC_FIELDS(X) X(acc) X(W) X(i_out) X(rp) X(rd) X(N) X(dscomp) X(m_kd) X(m_ks) X(area_sum) X(sdir) \
  X(wpos) X(sattn) X(dpos) X(ddir) X(dkt) X(didx) X(mo_kt)
#define LANE_INT_FUSED 16
#define LANE_DBL_FUSED 2
#define LANE_VEC_FUSED 3

enum {
#define E_(f) LI_##f,
  LANE_INT_FIELDS(E_)
#undef E_
  LI_COUNT
};
enum {
#define E_(f) LD_##f,
  LANE_DBL_FIELDS(E_)
#undef E_
  LD_COUNT
};
enum {
#define E_(f) LV_##f,
  LANE_VEC_FIELDS(E_)
#undef E_
  LV_COUNT
};

static_assert(LI_dret < LANE_INT_FUSED && LI_bunit < LANE_INT_FUSED && LI_qmode < LANE_INT_FUSED &&
                  LI_rdepth == LANE_INT_FUSED,
              "fused lane fields first");
static_assert(LD_sy < LANE_DBL_FUSED && LD_st_t == LANE_DBL_FUSED, "fused lane fields first");
static_assert(LV_i_out < LANE_VEC_FUSED && LV_rp == LANE_VEC_FUSED, "fused lane fields first");

struct LaneMem {
  int* i;     // [LI_COUNT][n]  (fused frames: [LANE_INT_FUSED][n])
  double* d;  // [LD_COUNT][n]  (LANE_DBL_FUSED)
  dvec3* v;   // [LV_COUNT][n]  (LANE_VEC_FUSED)
  size_t n;   // lanes
};

// fused: only the fused machine's fields (the leading ones of each list)
__host__ __device__ inline size_t lane_mem_bytes(size_t n, bool fused = false) {
  return n * ((fused ? LANE_INT_FUSED : LI_COUNT) * sizeof(int) + (fused ? LANE_DBL_FUSED : LD_COUNT) * sizeof(double) +
              (fused ? LANE_VEC_FUSED : LV_COUNT) * sizeof(dvec3)) +
         512;
}

// carve a LaneMem out of one allocation (256-byte aligned pieces)
inline LaneMem lane_mem_at(void* base, size_t n, bool fused = false) {
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  char* p = static_cast<char*>(base);
  LaneMem m;
  m.n = n;
  m.d = reinterpret_cast<double*>(p);
  p += al(n * (fused ? LANE_DBL_FUSED : LD_COUNT) * sizeof(double));
  m.v = reinterpret_cast<dvec3*>(p);
  p += al(n * (fused ? LANE_VEC_FUSED : LV_COUNT) * sizeof(dvec3));
  m.i = reinterpret_cast<int*>(p);
  return m;
}

struct LaneRef {
  LaneMem m;
  unsigned int g;  // lane
#define M_I(f) \
  __device__ __forceinline__ int& f() const { return m.i[size_t(LI_##f) * m.n + g]; }
#define M_D(f) \
  __device__ __forceinline__ double& f() const { return m.d[size_t(LD_##f) * m.n + g]; }
#define M_V(f) \
  __device__ __forceinline__ dvec3& f() const { return m.v[size_t(LV_##f) * m.n + g]; }
  LANE_INT_FIELDS(M_I)
  LANE_DBL_FIELDS(M_D)
  LANE_VEC_FIELDS(M_V)
#undef M_I
#undef M_D
#undef M_V
  __device__ __forceinline__ LaneRef(const LaneMem& mm, size_t gg)
      : m(mm), g(static_cast<unsigned int>(RTX_CHK(CHK_SLOT, gg, mm.n))) {}
  // Compiler barrier + opaque lane index: the state is memory, re-read per
  // step, and every field address is recomputed from (uniform base, g) where
  // it is used.  Without the opaque g, LLVM hoists the 43 per-lane 64-bit
  // field addresses out of the state loop and keeps them all in VGPRs.
  __device__ __forceinline__ void refresh() { asm volatile("" : "+v"(g)::"memory"); }
};

// the fields a slot's first advance reads: idle, nothing claimed, outside a
// discoverMat walk, no deferred colour
__device__ __forceinline__ void lane_init(LaneRef& L) {
  L.st() = ST_IDLE;
  L.kdone() = 0;
  L.dret() = DISC_NONE;
  L.wmask() = 0;
}

// zero one lane's state (kernel start)
__device__ __forceinline__ void lane_clear(const LaneMem& m, size_t g) {
  for (int k = 0; k < LI_COUNT; ++k) m.i[size_t(k) * m.n + g] = 0;
  for (int k = 0; k < LD_COUNT; ++k) m.d[size_t(k) * m.n + g] = 0.0;
  for (int k = 0; k < LV_COUNT; ++k) m.v[size_t(k) * m.n + g] = mk3(0.0, 0.0, 0.0);
}

// The ray of a lane's pending next-hit query: the shadow walk's (from the
// backed-up shading point toward the light, bounded by the light) or a
// discoverMat walk's (every hit of the ray, unbounded).
template <bool MEDIA>
__device__ __forceinline__ void next_query_ray(const DevScene& S, const LaneRef& L, dvec3& qP, dvec3& qD,
                                               double& qlim) {
  if (MEDIA && L.dret() != DISC_NONE) {
    qP = L.dpos();
    qD = L.ddir();
    qlim = RTX_INF;
    return;
  }
  qP = rtm::ray_at(L.rp(), L.rd(), L.st_t()) - L.rd() * RTX_EPS_BACKUP;
  qD = L.sdir();
  qlim = shadow_limit(S, S.lights[L.li()], qP, L.qrp() < 0);
}

// Scene::discoverMat (scene.cpp:212-237) over the ray (dpos, ddir): its
// sorted hits as successive next-hit queries from the list start
__device__ __forceinline__ void disc_query(LaneRef& LR, bool from_start) {
  LR.qmode() = Q_NEXT;
  LR.qtp() = from_start ? -RTX_INF : LR.bt();
  LR.qrp() = from_start ? -1 : LR.bobj();
  LR.qsq() = from_start ? -1 : LR.bsub();
}
__device__ __forceinline__ void disc_start(LaneRef& LR, int ret) {
  LR.dret() = ret;
  LR.dpass() = 0;
  LR.dpush() = 0;
  LR.dhead() = 0;
  LR.dlast() = -1;
  LR.dopq() = 0;
  LR.dkt() = mk3(1.0, 1.0, 1.0);  // Material(air): kt 1, index 1
  LR.didx() = mk3(1.0, 1.0, 1.0);
  LR.st() = ST_DISC;
  disc_query(LR, true);
}
// the shadow walk after a hit's limit check (light.cpp:47-49); m_out = (trans_o, kt_o)
__device__ __forceinline__ void walk_on(LaneRef& LR, const DevScene& S, double aterm, const HitRef& R, bool is_inside,
                                        double t, bool trans_o, const dvec3& kt_o, bool& done, dvec3& result) {
  const bool next_trans = is_inside ? trans_o : ((hit_flags(S, R) & RTX_MF_TRANS) != 0);
  if (!next_trans || (aterm > 0.0 && rtm::dot(LR.sattn(), LR.sattn()) < aterm * aterm)) {
    result = mk3(0.0, 0.0, 0.0);
    done = true;
  } else {
    const dvec3 kt = is_inside ? hit_param(S, R, RTX_P_KT) : kt_o;
    LR.sattn() *= rtm::pow3(kt, t);
    LR.qmode() = Q_NEXT;
    LR.qtp() = LR.bt();
    LR.qrp() = LR.bobj();
    LR.qsq() = LR.bsub();
  }
}
__device__ __forceinline__ void walk_done(LaneRef& LR, const RtxLight& L, const dvec3& result) {
  if (LR.pick() < 0) {
    LR.i_out() += LR.dattn() * result * ld3(L.color) * LR.dscomp();
    LR.li()++;
    LR.st() = ST_LIGHT;
  } else {
    LR.area_sum() += result;
    LR.st() = ST_SRS;
  }
}

// discoverMat walk steps and the shadow walk's resume after one (-O o).
// Inlined: an out-of-line call here (function-call ABI inside the state
// machine) measured 101 vs 91 ms on the headline frame.
__device__ __forceinline__ void media_step(LaneRef& LR, const DevScene& S, double aterm) {
  switch (LR.st()) {
      case ST_DISC: {
        // one hit of discoverMat's sorted list, or its end.  The object stack
        // only grows at the back (leaving hits) and loses its FRONT when an
        // entering hit matches the back's object (the erase(begin) of
        // scene.cpp:219-224; decision U4: checkObj returns check()), so the
        // stack is the pushes [dhead, dtot).  Pass 0 finds dhead and sums the
        // materials of all pushes; when dhead > 0 pass 1 sums again from
        // push dhead on (the sum is order dependent).
        if (LR.bhave()) {
          const HitRef R = resolve_hit(S, LR.dpos(), LR.ddir(), LR.bobj(), LR.bsub(), nullptr, nullptr);
          const bool leaving = rtm::dot(R.N, LR.ddir()) > 0;
          if (leaving && LR.dpush() >= LR.dhead()) {
            if (!(hit_flags(S, R) & RTX_MF_TRANS)) {
              LR.dopq() = 1;  // vantablack_mat
            } else {  // Material::operator+= adds the constant values (material.h:178-189)
              LR.dkt() += hit_raw(S, R, RTX_P_KT);
              LR.didx() += hit_raw(S, R, RTX_P_INDEX);
            }
          }
          if (LR.dpass() == 0) {
            if (leaving) {
              LR.dpush()++;
              LR.dlast() = LR.bobj();
            } else if (LR.dpush() > LR.dhead() && LR.bobj() == LR.dlast()) {
              LR.dhead()++;
            }
          } else if (leaving) {
            LR.dpush()++;
          }
          disc_query(LR, false);
          break;
        }
        if (LR.dpass() == 0) {
          LR.dtot() = LR.dpush();
          if (LR.dhead() > 0 && LR.dtot() > LR.dhead()) {  // sum again over the surviving pushes only
            LR.dpass() = 1;
            LR.dpush() = 0;
            LR.dopq() = 0;
            LR.dkt() = mk3(1.0, 1.0, 1.0);
            LR.didx() = mk3(1.0, 1.0, 1.0);
            disc_query(LR, true);
            break;
          }
          if (LR.dhead() > 0) {  // every push erased: the empty stack's average
            LR.dopq() = 0;
            LR.dkt() = mk3(1.0, 1.0, 1.0);
            LR.didx() = mk3(1.0, 1.0, 1.0);
          }
        }
        // blank = (1.0 / size) * blank (operator*(double, Material): each
        // constant value scaled); an empty stack divides by 0
        if (LR.dopq()) {
          LR.mo_trans() = 0;
          LR.mo_kt() = mk3(0.0, 0.0, 0.0);
          LR.mo_idx() = intensity(mk3(0.0, 0.0, 0.0));
        } else {
          const double s = 1.0 / static_cast<double>(LR.dtot() - LR.dhead());
          LR.mo_trans() = 1;
          LR.mo_kt() = LR.dkt() * s;
          LR.mo_idx() = intensity(LR.didx() * s);
        }
        LR.st() = LR.dret() == DISC_RECUR ? ST_RECUR : ST_WALK2;
        LR.dret() = DISC_NONE;
        break;
      }
      case ST_WALK2: {
        // the shadow walk's hit (wt, wobj, wsub) after its discoverMat
        const RtxLight& L = S.lights[LR.li()];
        LR.bt() = LR.wt();
        LR.bobj() = LR.wobj();
        LR.bsub() = LR.wsub();
        const dvec3 pb = rtm::ray_at(LR.rp(), LR.rd(), LR.st_t()) - LR.rd() * RTX_EPS_BACKUP;
        const HitRef R = resolve_hit(S, pb, LR.sdir(), LR.bobj(), LR.bsub(), nullptr, nullptr);
        const bool is_inside = rtm::dot(R.N, LR.sdir()) > 0;
        bool done = false;
        dvec3 result = LR.sattn();
        LR.st() = ST_WALK;  // the walk's next hit comes back to ST_WALK
        walk_on(LR, S, aterm, R, is_inside, LR.wtr(), LR.mo_trans() != 0, LR.mo_kt(), done, result);
        if (done) walk_done(LR, L, result);
        break;
      }
      default:
        break;
  }
}

// Fork slots of the calling kernel's group (FORK instantiations): a forked
// ray's sub-tree starts on a slot from the group's free list (fork slots
// whose sub-trees ended, pushed by advance_fused_kernel; free_ids null: no
// list) or else on spare_base + the next fresh spare while fewer than
// spare_n were handed out, and joins this iteration's live list.  fcnt
// (CNT_FORK) counts every request — the frame's fork history, which does
// not depend on how many were granted; fcnt[1] (CNT_FREE) is the free list's
// length, fcnt[2] (CNT_FRESH) the fresh spares taken.
struct ForkCtx {
  unsigned int* fcnt;
  int spare_base;
  unsigned int spare_n;
  int* live_out;
  unsigned int* live_cnt;
  const int* free_ids;
  int live_cap;  // entries of the group's live and free lists (the bounds check)
};

// lanes of the wave below the calling lane in `mask` (mbcnt)
__device__ __forceinline__ unsigned int lane_prefix(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<unsigned int>(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<unsigned int>(mask), 0u));
}

// A fork slot for each calling lane with `want`, or -1 (none left / not
// wanted).  Wave-aggregated — one atomic on the group's fork counter per call
// per wave, offsets by mbcnt — and called from divergent code: the ballot
// covers the lanes executing it.  (Per-lane atomics on the one counter
// serialised in L2: the shading step of a shard's first iteration forks
// hundreds of thousands of sub-trees.)
__device__ __forceinline__ int fork_claim(const ForkCtx* fk, bool want) {
  const unsigned long long m = __ballot(want);
  if (m == 0ull) return -1;
  const int leader = __builtin_ctzll(m);
  const int n = __popcll(m);
  // pops from the free list: no pushes run meanwhile (they are the advance
  // launch's), so concurrent pops take disjoint ranges below their old
  // lengths; a wave that finds fewer than it asked for gives the rest back
  int old = 0, avail = 0, fbase = 0;
  if (static_cast<int>(threadIdx.x & 63) == leader) {
    const int req = static_cast<int>(atomicAdd(fk->fcnt, static_cast<unsigned int>(n)));
    if (fk->free_ids) {
      old = static_cast<int>(atomicSub(fk->fcnt + 1, static_cast<unsigned int>(n)));
      avail = old < 0 ? 0 : (old < n ? old : n);
      if (avail < n) atomicAdd(fk->fcnt + 1, static_cast<unsigned int>(n - avail));
      if (avail < n) fbase = static_cast<int>(atomicAdd(fk->fcnt + 2, static_cast<unsigned int>(n - avail)));
    } else {
      fbase = req;  // no free list: the n-th request takes the n-th spare (CNT_FRESH unused)
    }
  }
  old = __shfl(old, leader);
  avail = __shfl(avail, leader);
  fbase = __shfl(fbase, leader);
  if (!want) return -1;
  const int r = static_cast<int>(lane_prefix(m));
  if (r < avail) return fk->free_ids[RTX_CHK(CHK_FREE, old - 1 - r, fk->live_cap)];
  const unsigned int idx = static_cast<unsigned int>(fbase + (r - avail));
  return idx < fk->spare_n ? fk->spare_base + static_cast<int>(idx) : -1;
}
// append fork slot T (lanes with T >= 0) to the iteration's live list,
// wave-aggregated like fork_claim
__device__ __forceinline__ void fork_join(const ForkCtx* fk, int T) {
  const unsigned long long m = __ballot(T >= 0);
  if (m == 0ull) return;
  const int leader = __builtin_ctzll(m);
  unsigned int base = 0;
  if (static_cast<int>(threadIdx.x & 63) == leader)
    base = atomicAdd(fk->live_cnt, static_cast<unsigned int>(__popcll(m)));
  base = __shfl(base, leader);
  if (T >= 0) fk->live_out[RTX_CHK(CHK_LIVE, base + lane_prefix(m), fk->live_cap)] = T;
}

// pending-ray entry field 12: bucket (the ray's heap position if it is a
// node, else its nearest node ancestor's; 0 without buckets), depth and kind
// (0 camera, 1 reflection, 2 refraction), exact in a double
__device__ __forceinline__ double pend_code(int pos, int depth, int kind) {
  return static_cast<double>((static_cast<int64_t>(pos) << 40) + (int64_t(1) << 39) + depth * 4 + kind);
}

// colour c of a ray in bucket b >= 2 of sample s: fbuf[s][b - 2] (written by
// one lane at a time, in that lane's ray order; the fmask bit says whether
// the bucket already holds a sum)
__device__ __forceinline__ void bucket_add(const FrameParams& F, int s, int b, const dvec3& c) {
  s = RTX_CHK(CHK_BUNIT, s, F.chk_units);
  b = RTX_CHK(CHK_BPOS, b - 2, F.fork_npos) + 2;
  const int set = F.bidx[s];
  if (set < 0) {  // (never: the root takes the set before its children exist)
    atomicOr(F.bover, 2u);
    return;
  }
  double* f = F.fbuf + (static_cast<int64_t>(RTX_CHK(CHK_BSET, set, F.bcap)) * F.fork_npos + (b - 2)) * 3;
  const unsigned int bit = 1u << (b - 2);
  const unsigned int old = atomicOr(&F.fmask[s], bit);
  if (old & bit) {
    f[0] += c.x;
    f[1] += c.y;
    f[2] += c.z;
  } else {
    f[0] = c.x;
    f[1] = c.y;
    f[2] = c.z;
  }
}

// A bucket set for unit s (lanes with `want`: a root ray about to push a
// node child), wave-aggregated like fork_claim.  Past the pool's capacity
// the unit gets none and *bover says so (bucket_add then drops its colours:
// collect_check reads the bit back per frame — a synchronous render is
// rendered again with a full-size pool, a device-buffer render reports
// RTX_ERR_FRAME).
__device__ __forceinline__ void bucket_alloc(const FrameParams& F, int s, bool want) {
  const unsigned long long m = __ballot(want);
  if (m == 0ull) return;
  const int leader = __builtin_ctzll(m);
  unsigned int base = 0;
  if (static_cast<int>(threadIdx.x & 63) == leader) base = atomicAdd(F.bcnt, static_cast<unsigned int>(__popcll(m)));
  base = __shfl(base, leader);
  if (!want) return;
  s = RTX_CHK(CHK_BUNIT, s, F.chk_units);
  const unsigned int idx = base + lane_prefix(m);
  if (idx < static_cast<unsigned int>(F.bcap)) {
    F.bidx[s] = static_cast<int>(idx);
  } else {
    F.bidx[s] = -1;
    atomicOr(F.bover, 1u);
  }
}

__host__ __device__ __forceinline__ int ilog2i(int v) { return 31 - __builtin_clz(static_cast<unsigned int>(v)); }

// Run one lane's state machine (trace / traceRay / shade / srsAttenuation,
// RayTracer.cpp:35-174, material.cpp:34-69, light.cpp:16-53) until it needs
// a traversal query (L.qmode != Q_NONE) or its sample is finished (ST_IDLE).
// The pending-ray stack lives in HBM: entry e, field f at
// pbuf[(e * 13 + f) * nlanes + glane].
// MEDIA: the -O o (overlapping media) states are compiled in; frames
// without -O o run the instantiation without them (smaller kernels).
template <bool STATS, bool ADAPTIVE, bool MEDIA, bool FORK = false>
__device__ __forceinline__ void advance_lane(LaneRef& LR, const DevScene& S, const FrameParams& F, Counters& C,
                                             double* __restrict__ sbuf, double* __restrict__ colbuf,
                                             RtxHitRecord* __restrict__ hits, int64_t apix_out, int an,
                                             double* __restrict__ pbuf, size_t nlanes, size_t glane, int pend_cap,
                                             const ForkCtx* fk = nullptr) {
  const RtxRenderParams& P = F.P;
  const double aterm = P.aterm_thresh;
  const int ncam = P.dof ? P.dof_div + 1 : 1;
  auto put_entry = [&](double* b, const dvec3& p, const dvec3& d, const dvec3& w, const dvec3& k, int depth, int kind,
                       int pos) {
    b[0 * nlanes] = p.x; b[1 * nlanes] = p.y; b[2 * nlanes] = p.z;
    b[3 * nlanes] = d.x; b[4 * nlanes] = d.y; b[5 * nlanes] = d.z;
    b[6 * nlanes] = w.x; b[7 * nlanes] = w.y; b[8 * nlanes] = w.z;
    b[9 * nlanes] = k.x; b[10 * nlanes] = k.y; b[11 * nlanes] = k.z;
    b[12 * nlanes] = pend_code(pos, depth, kind);
  };
  auto push = [&](int& tp, const dvec3& p, const dvec3& d, const dvec3& w, const dvec3& k, int depth, int kind,
                  int pos) {
    put_entry(pbuf + static_cast<size_t>(tp) * 13 * nlanes + LR.g, p, d, w, k, depth, kind, pos);
    ++tp;
  };
  // colour of the current ray (bucket LR.rpos()): the root's bucket is the
  // lane's acc, a node's bucket its fbuf entry
  auto contrib = [&](const dvec3& c) {
    if (F.fork_on && LR.rpos() >= 2) bucket_add(F, LR.bunit(), LR.rpos(), c);
    else LR.acc() += c;
  };
  // child node at heap position cpos: its sub-tree on a fork slot, if one is
  // free (same buckets, same sums as on the own stack); false leaves it to
  // the own stack
  auto fork_child = [&](const dvec3& p, const dvec3& d, const dvec3& w, const dvec3& k, int depth, int kind,
                        int cpos) -> bool {
    if (!FORK) return false;
    const int T = fork_claim(fk, cpos >= 2 && fk->spare_n != 0);
    if (T < 0) return false;
    LaneRef LT(LR.m, static_cast<size_t>(T));
    put_entry(pbuf + static_cast<size_t>(T), p, d, w, k, depth, kind, cpos);
    LT.top() = 1;
    LT.acc() = mk3(0.0, 0.0, 0.0);
    LT.nrays() = 0;
    LT.camk() = 1;
    LT.cam_end() = 1;
    LT.pass() = 0;
    LT.first_query() = 0;
    LT.rec_on() = LR.rec_on();
    LT.sample_slot() = LR.sample_slot();
    LT.bunit() = LR.bunit();
    LT.fpos() = cpos;
    LT.dret() = DISC_NONE;
    LT.st() = ST_POP;
    fork_join(fk, T);
    return true;
  };
  // traceRay's reflection / refraction (RayTracer.cpp:127-164); m_out =
  // (trans_o, idx_o, kt_o): air, or discoverMat's material under -O o
  auto recur = [&](bool trans_o, double idx_o, const dvec3& kt_o) {
    const int depth = LR.rdepth() - 1;
    const HitRef R = resolve_hit(S, LR.rp(), LR.rd(), LR.sobj(), LR.ssub(), nullptr, nullptr);
    const bool leaving = rtm::dot(LR.N(), LR.rd()) >= 0;
    const bool in_trans = (LR.m_flags() & RTX_MF_TRANS) != 0;
    const bool next_trans = leaving ? trans_o : in_trans;
    const dvec3 normal = (leaving ? -1.0 : 1.0) * LR.N();
    const double c = -1 * rtm::dot(normal, LR.rd());
    const double eta = next_trans ? (leaving ? hit_index(S, R) : idx_o) / (leaving ? idx_o : hit_index(S, R)) : 0;
    const double radicand = 1 - eta * eta * (1 - c * c);
    const bool tir = next_trans && radicand < 0;
    // buckets of the children: their own heap positions when they are nodes
    // (this ray is a node above the fork depth), else this ray's bucket
    const int pb = LR.rpos();
    const bool node = pb > 0 && P.depth - LR.rdepth() == ilog2i(pb);
    const int node_refl = node && 2 * pb < F.fork_npos + 2 ? 2 * pb : 0;
    const int node_refr = node && 2 * pb + 1 < F.fork_npos + 2 ? 2 * pb + 1 : 0;
    const int pos_refl = node_refl ? node_refl : pb;
    const int pos_refr = node_refr ? node_refr : pb;
    // the unit's bucket set, taken by its root before the first child exists
    if (F.fork_on && pb == 1)
      bucket_alloc(F, LR.bunit(),
                   (node_refl || node_refr) && ((next_trans && !tir) || (LR.m_flags() & RTX_MF_REFL) || tir));
    // push refraction first so that reflection is traced first
    if (next_trans && !tir && LR.top() < pend_cap) {
      const dvec3 tp = rtm::ray_at(LR.rp(), LR.rd(), LR.st_t() + RTX_RAY_EPS);
      const dvec3 td = eta * LR.rd() + (eta * c - sqrt(radicand)) * normal;
      const dvec3 kf = leaving ? kt_o : hit_param(S, R, RTX_P_KT);
      if (!fork_child(tp, td, LR.W(), kf, depth, 2, node_refr)) push(LR.top(), tp, td, LR.W(), kf, depth, 2, pos_refr);
      if (STATS) C.secondary++;
    }
    if (((LR.m_flags() & RTX_MF_REFL) || tir) && LR.top() < pend_cap) {
      const dvec3 rdir = LR.rd() + 2 * c * normal;
      const dvec3 rs = rtm::ray_at(LR.rp(), LR.rd(), LR.st_t() - RTX_RAY_EPS);
      const dvec3 wr = LR.W() * hit_param(S, R, RTX_P_KR);
      const dvec3 kf = leaving ? hit_param(S, R, RTX_P_KT) : kt_o;
      if (!fork_child(rs, rdir, wr, kf, depth, 1, node_refl)) push(LR.top(), rs, rdir, wr, kf, depth, 1, pos_refl);
      if (STATS) C.secondary++;
    }
  };
  LR.qmode() = Q_NONE;
  while (LR.st() != ST_IDLE && LR.qmode() == Q_NONE) {
    // the lane state is memory: each step re-reads the few fields it uses
    LR.refresh();
    switch (LR.st()) {
      case ST_CAM: {
        // next camera ray of trace(x, y) (RayTracer.cpp:35-79)
        if (LR.camk() == LR.cam_end()) {
          if (LR.fpos() != 0) {
            // a forked sub-tree: its colours are in its buckets already, its
            // rays join the sample's count
            if (LR.rec_on()) atomicAdd(&hits[LR.sample_slot()].nrays, LR.nrays());
            LR.fpos() = 0;
            LR.st() = ST_IDLE;
            break;
          }
          if (F.cam_split) {
            // one camera ray of a DoF sample (RayTracer.cpp:47-75): its own
            // sum; reduce_kernel adds the sample's rays in order, scales and
            // clamps
            const int64_t u = static_cast<int64_t>(LR.sample_slot()) * F.ncam + (LR.cam_end() - 1);
            (void)RTX_CHK(CHK_SAMPLE, u, F.chk_samples * F.ncam);
            sbuf[u * 3 + 0] = LR.acc().x;
            sbuf[u * 3 + 1] = LR.acc().y;
            sbuf[u * 3 + 2] = LR.acc().z;
            // per-sample ray count over the sample's units; the record starts
            // at -1 (0xff fill), the first ray's unit adds the 1 back
            if (LR.rec_on()) atomicAdd(&hits[LR.sample_slot()].nrays, LR.nrays() + (LR.cam_end() == 1 ? 1 : 0));
            LR.st() = ST_IDLE;
            break;
          }
          if (F.fork_on) {
            // the root's sum; reduce_kernel adds the forked sub-trees' sums,
            // then clamps (no anaglyph with forking; DoF splits above); the record's ray
            // count starts at -1 (0xff fill)
            double* out = sbuf + static_cast<int64_t>(LR.sample_slot()) * 3;
            out[0] = LR.acc().x;
            out[1] = LR.acc().y;
            out[2] = LR.acc().z;
            if (LR.rec_on()) atomicAdd(&hits[LR.sample_slot()].nrays, LR.nrays() + 1);
            LR.st() = ST_IDLE;
            break;
          }
          dvec3 ret = LR.acc();
          if (P.dof) ret *= (1.0 / (P.dof_div + 1.0));
          ret = rtm::gclamp3(ret, 0.0, 1.0);
          if (ADAPTIVE) {
            colbuf[LR.sample_slot() * 3 + 0] = ret.x;
            colbuf[LR.sample_slot() * 3 + 1] = ret.y;
            colbuf[LR.sample_slot() * 3 + 2] = ret.z;
            if (LR.rec_on()) hits[apix_out * an + LR.sample_slot()].nrays = LR.nrays();
            LR.st() = ST_IDLE;
            break;
          }
          double* out = sbuf + static_cast<int64_t>(LR.sample_slot()) * 3;
          if (P.anaglyph && LR.pass() == 0) {  // tracePixel (RayTracer.cpp:92-99): park pass 0 in the buffer
            out[0] = ret.x;
            out[1] = ret.y;
            out[2] = ret.z;
            LR.pass() = 1;
            LR.camk() = 0;
            LR.acc() = mk3(0, 0, 0);
            break;
          }
          if (P.anaglyph) {
            out[0] = ret.x;  // red from the shifted eye, green/blue from pass 0
          } else {
            out[0] = ret.x;
            out[1] = ret.y;
            out[2] = ret.z;
          }
          if (LR.rec_on()) hits[LR.sample_slot()].nrays = LR.nrays();
          LR.st() = ST_IDLE;
          break;
        }
        const RtxCamera& cam = F.cam;
        const dvec3 eye = LR.pass() ? ld3(cam.eye) + mk3(0.25, 0.0, 0.0) : ld3(cam.eye);
        const double x = LR.sx() - 0.5, y = LR.sy() - 0.5;
        const dvec3 cdir = rtm::normalize(ld3(cam.look) + x * ld3(cam.u) + y * ld3(cam.v));
        if (LR.camk() == 0) {
          LR.rp() = eye;
          LR.rd() = cdir;
          LR.first_query() = LR.rec_on() && LR.pass() == 0;
          if (LR.first_query()) {  // default record: miss (also what depth < 0 leaves)
            RtxHitRecord* hr = ADAPTIVE ? &hits[apix_out * an + LR.sample_slot()] : &hits[LR.sample_slot()];
            hr->object = hr->face = hr->scene_leaf = hr->mesh_leaf = -1;
            hr->t = 1000.0;
            hr->pad = 0;
          }
        } else {
          const double fd = rtm::gmax(P.dof_fd, 1.0);
          const dvec3 fp_n = -cdir;
          const dvec3 fp_pt = rtm::ray_at(eye, cdir, fd);
          double t = rtm::dot(fp_n, cdir);
          t = rtm::dot(fp_pt - eye, fp_n) / t;
          const dvec3 dest = rtm::ray_at(eye, cdir, t);
          LR.rp() = eye + ld3(&F.offv[(LR.camk() - 1) * 3]);
          LR.rd() = rtm::normalize(dest - LR.rp());
          LR.first_query() = false;
        }
        LR.camk()++;
        if (STATS) C.camera++;
        LR.top() = 0;
        push(LR.top(), LR.rp(), LR.rd(), mk3(1, 1, 1), mk3(1, 1, 1), P.depth, 0, F.fork_on ? 1 : 0);
        LR.st() = ST_POP;
        break;
      }
      case ST_POP: {
        if (LR.top() == 0) {
          LR.st() = ST_CAM;
          break;
        }
        --LR.top();
        const double* b = pbuf + static_cast<size_t>(LR.top()) * 13 * nlanes + LR.g;
        const int64_t code = static_cast<int64_t>(b[12 * nlanes]);
        const int dk = static_cast<int>((code & ((int64_t(1) << 40) - 1)) - (int64_t(1) << 39));
        LR.rpos() = static_cast<int>(code >> 40);
        LR.nrays()++;
        const int pdepth = dk >= 0 ? dk / 4 : -((-dk + 3) / 4);
        if (pdepth < 0) {  // `depth >= 0 &&` (RayTracer.cpp:116): no query, the miss colour
          if (S.cube[0] >= 0)
            contrib(mk3(b[6 * nlanes], b[7 * nlanes], b[8 * nlanes]) *
                    cube_color(S, mk3(b[3 * nlanes], b[4 * nlanes], b[5 * nlanes])));
          break;
        }
        LR.rp() = mk3(b[0 * nlanes], b[1 * nlanes], b[2 * nlanes]);
        LR.rd() = mk3(b[3 * nlanes], b[4 * nlanes], b[5 * nlanes]);
        LR.W() = mk3(b[6 * nlanes], b[7 * nlanes], b[8 * nlanes]);
        LR.area_sum() = mk3(b[9 * nlanes], b[10 * nlanes], b[11 * nlanes]);  // kt factor, parked until the hit
        LR.rdepth() = pdepth;
        LR.rkind() = dk - pdepth * 4;
        LR.qmode() = Q_CLOSEST;
        LR.qtp() = -RTX_INF;
        LR.qrp() = -1;
        LR.qsq() = -1;
        LR.st() = ST_HIT;
        break;
      }
      case ST_HIT: {
        // traceRay after scene->intersect (RayTracer.cpp:116-165)
        if (LR.first_query()) {
          LR.first_query() = false;
          if (LR.bhave()) {
            RtxHitRecord* hr = ADAPTIVE ? &hits[apix_out * an + LR.sample_slot()] : &hits[LR.sample_slot()];
            const RtxObject& o = S.objs[LR.bobj()];
            hr->object = o.orig_id;
            hr->scene_leaf = o.leaf;
            hr->t = LR.bt();
            if (o.type == RTX_OBJ_TRIMESH) {
              const RtxFaceIds fi = S.fids[o.pad[RTX_OBJ_FACE_OFF] + LR.bsub()];
              hr->face = fi.orig_id;
              hr->mesh_leaf = fi.leaf;
            }
          }
        }
        if (!LR.bhave()) {  // miss: the cube map's colour, else black (RayTracer.cpp:167-169)
          // a child's kt^t factor is kt^0 = 1 on a miss (decision U3)
          if (S.cube[0] >= 0) contrib(LR.W() * cube_color(S, LR.rd()));
          LR.st() = ST_POP;
          break;
        }
        if (LR.rkind() == 1)
          LR.W() = LR.W() * rtm::gmax3(rtm::gmin3(rtm::pow3(LR.area_sum(), LR.bt()), rtm::splat3(1.0)), rtm::splat3(0.0));
        else if (LR.rkind() == 2)
          LR.W() = LR.W() * rtm::pow3(LR.area_sum(), LR.bt());
        const HitRef R = resolve_hit(S, LR.rp(), LR.rd(), LR.bobj(), LR.bsub(), nullptr, nullptr);
        LR.N() = R.N;
        LR.m_kd() = hit_param(S, R, RTX_P_KD);
        LR.m_ks() = hit_param(S, R, RTX_P_KS);
        LR.m_sh() = hit_shininess(S, R);
        LR.m_flags() = hit_flags(S, R);
        LR.st_t() = LR.bt();
        LR.sobj() = LR.bobj();
        LR.ssub() = LR.bsub();
        if (STATS) C.shades++;
        // Material::shade (material.cpp:34-69)
        LR.i_out() = hit_param(S, R, RTX_P_KE) + hit_param(S, R, RTX_P_KA) * mk3(S.ambient[0], S.ambient[1], S.ambient[2]);
        LR.li() = 0;
        LR.st() = ST_LIGHT;
        break;
      }
      case ST_LIGHT: {
        if (LR.li() == S.n_lights) {
          // colorC = shade(...); adaptive termination; recursion
          const dvec3 col = LR.i_out();
          contrib(LR.W() * col);
          const int depth = LR.rdepth() - 1;
          LR.st() = ST_POP;
          if (aterm > 0.0 && rtm::dot(col, col) < aterm) break;
          if ((LR.m_flags() & RTX_MF_RECUR) && depth > 0) {
            if (MEDIA && P.overlapping) {
              // m_out = discoverMat(ray(r.at(t - RAY_EPSILON), d)) (RayTracer.cpp:128)
              LR.dpos() = rtm::ray_at(LR.rp(), LR.rd(), LR.st_t() - RTX_RAY_EPS);
              LR.ddir() = LR.rd();
              disc_start(LR, DISC_RECUR);
            } else {
              recur(true, S.air_index, mk3(1.0, 1.0, 1.0));  // m_out = air
            }
          }
          break;
        }
        const RtxLight& L = S.lights[LR.li()];
        const dvec3 X = rtm::ray_at(LR.rp(), LR.rd(), LR.st_t());
        const dvec3 l_i = light_dir(L, X);
        const dvec3 l_r = (l_i - 2 * (rtm::dot(l_i, LR.N())) * LR.N());
        double dt = rtm::dot(l_i, LR.N());
        if (LR.m_flags() & RTX_MF_TRANS) dt = fabs(dt);
        const dvec3 d_comp = LR.m_kd() * rtm::gmax(0.0, dt);
        // glm::pow(dvec3(x), dvec3(sh)): three identical std::pow calls, one here
        const dvec3 s_comp = LR.m_ks() * rtm::splat3(rtm::rpow(rtm::gmax(0.0, rtm::dot(l_r, LR.rd())), LR.m_sh()));
        LR.dscomp() = d_comp + s_comp;
        LR.dattn() = light_dist_atten(L, X);
        // shadowAttenuation (light.cpp:16-20) / AreaLight (light.cpp:76-87)
        if (L.type == RTX_LIGHT_DIRECTIONAL || L.type == RTX_LIGHT_POINT) {
          if (S.skip_dark && !P.overlapping && LR.dscomp().x == 0.0 && LR.dscomp().y == 0.0 && LR.dscomp().z == 0.0) {
            // the light's term is dattn * sattn * color * 0, and sattn is
            // finite in this scene (kt in [0,1]), so it adds +0: the shadow
            // ray still counts (the reference traces it) but is not traced
            if (STATS) C.shadow++;
            LR.nrays()++;
            LR.li()++;
            break;
          }
          LR.sdir() = light_dir(L, X - LR.rd() * RTX_EPS_BACKUP);
          LR.pick() = -1;
        } else {
          const dvec3 ori = ld3(L.orient), lpos = ld3(L.pos);
          if (L.type == RTX_LIGHT_SPOT &&
              !((rtm::dot(light_dir(L, X), ori) <= 0) &&
                (rtm::dot(rtm::normalize(X - (lpos - L.offset * ori)), ori) > S.cos45))) {
            LR.i_out() += LR.dattn() * mk3(0.0, 0.0, 0.0) * ld3(L.color) * LR.dscomp();
            LR.li()++;
            break;
          }
          LR.area_sum() = mk3(1.0, 1.0, 1.0);
          LR.pick() = 0;
        }
        LR.st() = ST_SRS;
        break;
      }
      case ST_SRS: {
        // start one srsAttenuation (light.cpp:21-53), or finish an area light
        const RtxLight& L = S.lights[LR.li()];
        const dvec3 pb = rtm::ray_at(LR.rp(), LR.rd(), LR.st_t()) - LR.rd() * RTX_EPS_BACKUP;
        if (LR.pick() >= 0) {
          bool started = false;
          while (LR.pick() < S.ss_res) {
            const dvec3 lp = ld3(S.picks + (size_t(LR.li()) * S.ss_res + LR.pick()) * 3);
            LR.pick()++;
            if (L.type == RTX_LIGHT_SPOT &&
                !((rtm::dot(light_dir(L, pb), ld3(L.orient)) <= 0) &&
                  (rtm::dot(rtm::normalize(pb - lp), ld3(L.orient)) > S.cos45)))
              continue;
            LR.sdir() = rtm::normalize(lp - pb);
            started = true;
            break;
          }
          if (!started) {
            dvec3 sa = LR.area_sum();
            sa *= (1.0 / (S.ss_res - 1));
            LR.i_out() += LR.dattn() * sa * ld3(L.color) * LR.dscomp();
            LR.li()++;
            LR.st() = ST_LIGHT;
            break;
          }
        }
        if (STATS) {
          C.shadow++;
          C.shadow_traced++;
        }
        LR.nrays()++;
        LR.sattn() = mk3(1.0, 1.0, 1.0);
        LR.wpos() = pb;
        LR.last_t() = 0.0;
        LR.qmode() = Q_NEXT;
        LR.qtp() = -RTX_INF;
        LR.qrp() = -1;
        LR.qsq() = -1;
        LR.st() = ST_WALK;
        break;
      }
      case ST_RECUR: {
        // after discoverMat (-O o): traceRay's recursion with its material
        LR.st() = ST_POP;
        if (MEDIA) recur(LR.mo_trans() != 0, LR.mo_idx(), LR.mo_kt());
        break;
      }
      case ST_DISC:
      case ST_WALK2:
        if (MEDIA) media_step(LR, S, aterm);  // -O o only
        else LR.st() = ST_IDLE;
        break;
      case ST_WALK: {
        const RtxLight& L = S.lights[LR.li()];
        bool done = false;
        dvec3 result = LR.sattn();
        if (!LR.bhave()) {
          done = true;
        } else {
          const double t = LR.bt() - LR.last_t();
          LR.last_t() = LR.bt();
          const dvec3 pb = rtm::ray_at(LR.rp(), LR.rd(), LR.st_t()) - LR.rd() * RTX_EPS_BACKUP;
          const HitRef R = resolve_hit(S, pb, LR.sdir(), LR.bobj(), LR.bsub(), nullptr, nullptr);
          const bool is_inside = rtm::dot(R.N, LR.sdir()) > 0;
          LR.wpos() = rtm::ray_at(LR.wpos(), LR.sdir(), t);
          bool limit = false;  // sattnLimitCheck with the relative t (U14)
          if (L.type == RTX_LIGHT_POINT) {
            limit = rtm::dot(ld3(L.pos) - rtm::ray_at(LR.wpos(), LR.sdir(), t), LR.sdir()) <= 0;
          } else if (L.type != RTX_LIGHT_DIRECTIONAL) {
            const dvec3 ori = ld3(L.orient), lpos = ld3(L.pos);
            double ti = rtm::dot(ori, LR.sdir());
            ti = rtm::dot(lpos - LR.wpos(), ori) / ti;
            dvec3 imp = rtm::ray_at(LR.wpos(), LR.sdir(), ti);
            if (L.type != RTX_LIGHT_AREA_RECT && !(rtm::dot(imp - lpos, imp - lpos) < (L.radius * L.radius)))
              imp = mk3(0.0, 0.0, 0.0);
            limit = rtm::dot(imp - rtm::ray_at(LR.wpos(), LR.sdir(), t), LR.sdir()) <= 0;
          }
          if (limit) {
            done = true;
          } else if (MEDIA && P.overlapping) {
            // m_out = discoverMat(ray(r2l)) from the moved origin (light.cpp:38-39)
            LR.wt() = LR.bt();
            LR.wtr() = t;
            LR.wobj() = LR.bobj();
            LR.wsub() = LR.bsub();
            LR.dpos() = LR.wpos();
            LR.ddir() = LR.sdir();
            disc_start(LR, DISC_WALK);
            break;
          } else {
            walk_on(LR, S, aterm, R, is_inside, t, true, mk3(1.0, 1.0, 1.0), done, result);  // m_out = air
          }
        }
        if (done) walk_done(LR, L, result);
        break;
      }
      default:
        LR.st() = ST_IDLE;
        break;
    }
  }

}

// per-wave sums of a kernel's counters into the frame's stats (indices 0-6:
// RtxStats rays..shades, 18: shadow rays traced)
__device__ __forceinline__ void stats_add(const Counters& C, unsigned long long* stats, int lane) {
  const int64_t v[8] = {C.camera, C.secondary, C.shadow, C.nodes, C.objects, C.tris, C.shades, C.shadow_traced};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    int64_t x = v[k];
    for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off);
    if (lane == 0 && x) atomicAdd(&stats[k < 7 ? k : 18], static_cast<unsigned long long>(x));
  }
}
// per-kernel work (rtx_last_work): queries, node visits, object and triangle
// tests, shades of one kernel class at stats[base .. base + 4] (20 batched
// closest-hit launches, 25 batched next-hit / walk launches, 30 tail launches)
// 35..38: the slowest wave of the last closest / next launch (RTX_DEBUG=2);
// 39 + 20 * (MODE - 1) ..: the trace kernels' cycle breakdown (STATS
// instantiations only): [c] core cycles of the wave steps whose stepping
// lanes were at the unit classes of bit mask c (1 record, 2 object or the
// step into a leaf's objects, 4 mesh leaf), [8 + c] their count, [16] / [17]
// cycles / runs of the per-query work between traversals (FUSED: shading,
// walk steps), [18] cycles the waves spent in all (RTX_DEBUG report)
#define RTX_STATS_PROF 39
#define RTX_STATS_N 79
__device__ __forceinline__ void stats_add_class(const Counters& C, unsigned long long* stats, int lane, int base) {
  const int64_t v[5] = {C.queries, C.nodes, C.objects, C.tris, C.shades};
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    int64_t x = v[k];
    for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off);
    if (lane == 0 && x) atomicAdd(&stats[base + k], static_cast<unsigned long long>(x));
  }
}

template <bool STATS, bool ADAPTIVE, bool MEDIA>
__global__ void __launch_bounds__(WG) render_kernel(DevScene S, const DevScene* __restrict__ Sg, const FrameParams* __restrict__ Fp,
                                                     unsigned long long* __restrict__ work,
                                                     double* __restrict__ sbuf, RtxHitRecord* __restrict__ hits,
                                                     uint8_t* __restrict__ rgb8, double* __restrict__ rgbf,
                                                     unsigned long long* __restrict__ stats, int stack_cap,
                                                     double* __restrict__ pbuf, int pend_cap, LaneMem lm) {
  extern __shared__ double smem[];
  const FrameParams& F = *Fp;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int cslots = ADAPTIVE ? (F.spp > 64 ? F.spp : 64) : 0;
  const int fslots = ADAPTIVE ? 16 * 8 : 0;  // adaptive region frames (8 doubles each)
  double* colbuf = smem + static_cast<size_t>(wave) * (cslots * 3 + fslots + stack_cap * 32);
  double* frbuf = colbuf + cslots * 3;
  int* stk = reinterpret_cast<int*>(frbuf + fslots);
  // per-lane pending-ray stack in HBM, field-major so a wave's accesses of
  // one field are contiguous: entry e, field f of lane g at
  // pbuf[(e * 13 + f) * nlanes + g]
  const size_t nlanes = static_cast<size_t>(gridDim.x) * WG;
  const size_t glane = static_cast<size_t>(blockIdx.x) * WG + threadIdx.x;
  Counters C = {0, 0, 0, 0, 0, 0, 0};
  const RtxRenderParams& P = F.P;
  const double aterm = P.aterm_thresh;
  const int ncam = P.dof ? P.dof_div + 1 : 1;

  // ---- lane state (HBM, see LaneRef)
  lane_clear(lm, glane);
  LaneRef LR(lm, glane);
  LR.st() = ST_IDLE;
  LR.sample_slot() = -1;

  // ---- wave-uniform scheduler state
  unsigned long long qnext = 0, qend = 0;
  bool exhausted = false;
  // adaptive
  // region frames live in LDS (wave-uniform): frbuf[f*8 + {x1,x2,y1,y2,ax,ay,az,child}]
  int fsp = 0, abase = 0;
  bool atop = false;
  int64_t apix_out = 0;
  const int an = F.spp;

  for (;;) {
    LR.refresh();
    // ------------------------------------------------ scheduling
    if (!ADAPTIVE) {
      unsigned long long idle = __ballot(LR.st() == ST_IDLE);
      while (idle != 0ull) {
        if (qnext >= qend) {
          if (exhausted) break;
          unsigned long long base = 0;
          if (lane == 0) base = atomicAdd(work, static_cast<unsigned long long>(F.qchunk));
          base = __shfl(base, 0);
          if (base >= static_cast<unsigned long long>(F.n_samples)) {
            exhausted = true;
            break;
          }
          qnext = base;
          qend = base + F.qchunk;
          if (qend > static_cast<unsigned long long>(F.n_samples)) qend = F.n_samples;
        }
        const unsigned int rank = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned int>(idle >> 32),
                                                            __builtin_amdgcn_mbcnt_lo(static_cast<unsigned int>(idle), 0u));
        const unsigned long long avail = qend - qnext;
        const unsigned int nidle = __popcll(idle);
        const unsigned int take = avail < nidle ? static_cast<unsigned int>(avail) : nidle;
        if (LR.st() == ST_IDLE && rank < take) {
          const int64_t sid = static_cast<int64_t>(qnext + rank);
          const int64_t item = sid / (F.ppw * F.spp);
          const int slot = static_cast<int>(sid % (F.ppw * F.spp));
          const int pix = slot / F.spp, smp = slot % F.spp;
          int i, j;
          int64_t oidx;
          if (item_pixel(F, item, pix, i, j, oidx)) {
            int pi = i, pj = j;
            double ssx = 1.0, ssy = 1.0;
            if (P.aa_mode != RTX_AA_NONE) {  // tracePixel(i*s + si, j*s + sj)
              pi = i * F.s + smp / F.s;
              pj = j * F.s + smp % F.s;
              ssx = F.s;
              ssy = F.s;
            }
            // tracePixel (RayTracer.cpp:87-88)
            LR.sx() = double(pi) / (double(P.width) * ssx);
            LR.sy() = double(pj) / (double(P.height) * ssy);
            LR.sample_slot() = static_cast<int>(oidx * F.spp + smp);
            LR.rec_on() = hits != nullptr;
            LR.pass() = 0;
            LR.camk() = 0;
            LR.cam_end() = ncam;
            LR.nrays() = 0;
            LR.acc() = mk3(0, 0, 0);
            LR.st() = ST_CAM;
          }
          // out-of-image slots stay idle and are simply consumed
        }
        qnext += take;
        idle = __ballot(LR.st() == ST_IDLE);
        if (take == 0) break;
        if (qnext < qend) break;  // every idle lane got work (or was consumed)
      }
    } else {
      // adaptive: one pixel per wave; all lanes idle => chunk finished.
      // Frames f: frbuf[f*8 + 0..3] = x1, x2, y1, y2; [4..6] = acc; [7] = child
      if (__ballot(LR.st() != ST_IDLE) == 0ull) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        auto facc = [&](int f) { return mk3(frbuf[f * 8 + 4], frbuf[f * 8 + 5], frbuf[f * 8 + 6]); };
        auto set_acc = [&](int f, const dvec3& a) {
          frbuf[f * 8 + 4] = a.x;
          frbuf[f * 8 + 5] = a.y;
          frbuf[f * 8 + 6] = a.z;
        };
        auto set_frame = [&](int f, double x1, double x2, double y1, double y2) {
          frbuf[f * 8 + 0] = x1;
          frbuf[f * 8 + 1] = x2;
          frbuf[f * 8 + 2] = y1;
          frbuf[f * 8 + 3] = y2;
          set_acc(f, mk3(0.0, 0.0, 0.0));
          frbuf[f * 8 + 7] = -1.0;
        };
        // pop frame fsp-1 with value mu into its parent (adaptaa's `mu += subval`)
        auto finish = [&](const dvec3& mu) {
          --fsp;
          if (fsp > 0) {
            set_acc(fsp - 1, facc(fsp - 1) + mu);
            frbuf[(fsp - 1) * 8 + 7] += 1.0;
          } else {
            LR.acc() = mu;  // pixel value
          }
        };
        bool need_new_pixel = fsp == 0;
        if (fsp > 0 && abase >= 0) {
          const int nxt = abase + 64;
          abase = nxt < an ? nxt : -1;  // -1: region samples complete
        }
        while (fsp > 0 && abase < 0) {
          const int f = fsp - 1;
          const int child = static_cast<int>(frbuf[f * 8 + 7]);
          if (child < 0) {
            // region statistics (RayTracer.cpp:337-347)
            dvec3 mu = mk3(0.0, 0.0, 0.0), sd = mk3(0.0, 0.0, 0.0);
            for (int k = 0; k < an; ++k) mu += mk3(colbuf[k * 3 + 0], colbuf[k * 3 + 1], colbuf[k * 3 + 2]);
            mu *= (1.0 / (an));
            for (int k = 0; k < an; ++k) {
              const dvec3 s_c = mk3(colbuf[k * 3 + 0], colbuf[k * 3 + 1], colbuf[k * 3 + 2]);
              sd += mk3(pow(fabs(s_c.x - mu.x), 2.0), pow(fabs(s_c.y - mu.y), 2.0), pow(fabs(s_c.z - mu.z), 2.0));
            }
            sd *= (1.0 / (an - 1));
            if (rtm::length(sd) > P.aa_thresh && fsp < 16) {
              set_acc(f, mk3(0.0, 0.0, 0.0));
              frbuf[f * 8 + 7] = 0.0;
            } else {
              finish(mu);
            }
            continue;
          }
          if (child < 4) {
            const double x1 = frbuf[f * 8 + 0], x2 = frbuf[f * 8 + 1], y1 = frbuf[f * 8 + 2], y2 = frbuf[f * 8 + 3];
            const double xs[3] = {x1, (x1 + x2) / 2.0, x2};
            const double ys[3] = {y1, (y1 + y2) / 2.0, y2};
            const int a = child / 2, b = child % 2;
            const double nx1 = a == 0 ? xs[0] : xs[1], nx2 = a == 0 ? xs[1] : xs[2];
            const double ny1 = b == 0 ? ys[0] : ys[1], ny2 = b == 0 ? ys[1] : ys[2];
            if (nx1 + 0.0001 >= nx2 || ny1 + 0.0001 >= ny2) {  // U8: the subregion contributes 0
              set_acc(f, facc(f) + mk3(0.0, 0.0, 0.0));
              frbuf[f * 8 + 7] += 1.0;
              continue;
            }
            set_frame(fsp, nx1, nx2, ny1, ny2);
            ++fsp;
            abase = 0;
            atop = false;
          } else {
            dvec3 mu = facc(f);
            mu *= (1.0 / 4.0);
            finish(mu);
          }
        }
        if (fsp == 0 && !need_new_pixel) {
          if (lane == 0) {  // setPixel (RayTracer.cpp:388-394)
            if (rgb8) {
              rgb8[apix_out * 3 + 0] = rtm::to_byte(LR.acc().x);
              rgb8[apix_out * 3 + 1] = rtm::to_byte(LR.acc().y);
              rgb8[apix_out * 3 + 2] = rtm::to_byte(LR.acc().z);
            }
            if (rgbf) {
              rgbf[apix_out * 3 + 0] = LR.acc().x;
              rgbf[apix_out * 3 + 1] = LR.acc().y;
              rgbf[apix_out * 3 + 2] = LR.acc().z;
            }
          }
          need_new_pixel = true;
        }
        while (need_new_pixel) {
          unsigned long long item = 0;
          if (lane == 0) item = atomicAdd(work, 1ull);
          item = __shfl(item, 0);
          if (item >= static_cast<unsigned long long>(F.n_items)) {
            exhausted = true;
            break;
          }
          int i, j;
          if (!item_pixel(F, static_cast<int64_t>(item), 0, i, j, apix_out)) continue;
          const double x1 = double(i) / double(P.width), x2 = double(i + 1) / double(P.width);
          const double y1 = double(j) / double(P.height), y2 = double(j + 1) / double(P.height);
          if (x1 + 0.0001 >= x2 || y1 + 0.0001 >= y2) {  // whole pixel under eps: black (U8)
            if (lane == 0) {
              if (rgb8) {
                rgb8[apix_out * 3 + 0] = 0;
                rgb8[apix_out * 3 + 1] = 0;
                rgb8[apix_out * 3 + 2] = 0;
              }
              if (rgbf) {
                rgbf[apix_out * 3 + 0] = 0.0;
                rgbf[apix_out * 3 + 1] = 0.0;
                rgbf[apix_out * 3 + 2] = 0.0;
              }
            }
            continue;
          }
          set_frame(0, x1, x2, y1, y2);
          fsp = 1;
          abase = 0;
          atop = true;
          need_new_pixel = false;
        }
        if (exhausted && fsp == 0) break;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // assign samples abase + lane of region fsp-1
        const int k = abase + lane;
        if (k < an) {
          const int f = fsp - 1;
          const double x1 = frbuf[f * 8 + 0], x2 = frbuf[f * 8 + 1], y1 = frbuf[f * 8 + 2], y2 = frbuf[f * 8 + 3];
          const double w = x2 - x1, h = y2 - y1;
          LR.sx() = radinv2(k) * w + x1;    // hammersley x
          LR.sy() = (0.0 / an) * h + y1;    // hammersley y is always 0 (U7)
          LR.sample_slot() = k;
          LR.rec_on() = hits != nullptr && atop;
          LR.pass() = 0;
          LR.camk() = 0;
          LR.cam_end() = ncam;
          LR.nrays() = 0;
          LR.acc() = mk3(0, 0, 0);
          LR.st() = ST_CAM;
        }
      }
    }

    // ------------------------------------------------ advance lanes to their next query
    advance_lane<STATS, ADAPTIVE, MEDIA>(LR, *Sg, F, C, sbuf, colbuf, hits, apix_out, an, pbuf, nlanes, glane, pend_cap);

    // ------------------------------------------------ exit / traversal
    const unsigned long long busy = __ballot(LR.qmode() != Q_NONE);
    if (busy == 0ull) {
      if (__ballot(LR.st() != ST_IDLE) == 0ull && exhausted) break;
      continue;
    }
    if (LR.qmode() != Q_NONE) {
      dvec3 qP = LR.rp(), qD = LR.rd();
      double qlim = RTX_INF;
      if (LR.qmode() == Q_NEXT) {
        next_query_ray<MEDIA>(S, LR, qP, qD, qlim);
      }
      LR.bhave() = traverse<STATS>(S, LR.qmode(), qP, qD, LR.qtp(), LR.qrp(), LR.qsq(), qlim, LR.bt(), LR.bobj(), LR.bsub(), stk, lane, C);
    }
  }
  if (STATS) {
    int64_t v[7] = {C.camera, C.secondary, C.shadow, C.nodes, C.objects, C.tris, C.shades};
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      int64_t x = v[k];
      for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off);
      if (lane == 0) atomicAdd(&stats[k], static_cast<unsigned long long>(x));
    }
  }
}

// ============================================================ wavefront path
// Path slots: NSLOT lanes whose LaneRef state lives in HBM.  Each iteration:
//   advance_kernel  — one thread per slot: take the last query's result, run
//                     the state machine to the next ray query, append it to
//                     the closest-hit or next-hit list (wave ballot + popc +
//                     one atomic per wave, mbcnt for the offset: compaction
//                     of the active-ray mask);
//   trace_kernel<Q> — persistent traversal of a compacted list, writing each
//                     result into its slot's state.
// Samples are dealt to slots statically (sample slot + k * NSLOT).
struct QList {
  int* slot;    // [cap]
  double* d;    // Px Py Pz Dx Dy Dz tp tlimit, field-major [QL_D][cap]
  int* iv;      // rp, sq  [2][cap]
  size_t cap;
};
#define QL_D 8
// per-group counters (unsigned ints), each on its own 128-byte line (the
// appends, claims and liveness atomics of three concurrent groups must not
// share lines: packed 4 bytes apart the frame took 5% longer):
// [CNT_Q + m * CNT_LINE] queries of mode m (0 closest, 1 next),
// [CNT_CLAIM + m * CNT_LINE] the trace claim cursors, and two live-slot
// counts used ping-pong: an even iteration appends its live slots to list A
// (count at line 0) and reads list B (line 5), an odd one the reverse, so
// one memset per iteration (lines 0-4 or 1-5) clears exactly the out-count
// and the query / claim counters
#define CNT_LINE 32
#define CNT_ALIVE_A 0
#define CNT_Q (1 * CNT_LINE)
#define CNT_CLAIM (3 * CNT_LINE)
#define CNT_ALIVE_B (5 * CNT_LINE)
#define CNT_FORK (6 * CNT_LINE)  // fork requests this frame, granted or not (not cleared per iteration)
#define CNT_FREE (CNT_FORK + 1)  // fork slots on the group's free list (same line: not cleared per iteration)
#define CNT_FRESH (CNT_FORK + 2) // spare slots handed out for the first time this frame
#define CNT_DONE (7 * CNT_LINE)  // workgroups of the iteration's last kernel that finished
#define CNT_PER_GROUP (8 * CNT_LINE)

// A slot's next statically dealt work unit, or -1: none left, or a fork
// slot.  Runs of 64 consecutive units (one wave's worth of neighbouring
// samples) are dealt to the groups round-robin, so every group gets a share
// of every image region: contiguous thirds left the bottom third's group
// idle after 3 iterations while the other two carried the costly rows.
__device__ __forceinline__ int64_t slot_unit(const FrameParams& F, int slot, int kdone) {
  const int g = slot / F.wf_gs, l = slot - g * F.wf_gs;
  if (l >= F.wf_gsamp) return -1;
  const int64_t unit = ((static_cast<int64_t>(l >> 6) * F.wf_groups + g) << 6) + (l & 63) +
                       static_cast<int64_t>(kdone) * F.wf_nslot;
  return unit < F.n_samples ? unit : -1;
}

// Claim the next statically dealt sample for an idle slot (what the
// scheduler of the megakernel does with its queue).
__device__ __forceinline__ void claim_sample(LaneRef& L, const FrameParams& F, RtxHitRecord* hits, int slot) {
  const RtxRenderParams& P = F.P;
  while (L.st() == ST_IDLE) {
    const int64_t unit = slot_unit(F, slot, L.kdone());
    if (unit < 0) return;
    L.kdone()++;
    // work unit -> sample (and, with cam_split, which of its camera rays)
    const int64_t sid = F.cam_split ? unit / F.ncam : unit;
    const int cam0 = F.cam_split ? static_cast<int>(unit - sid * F.ncam) : 0;
    const int64_t item = sid / (F.ppw * F.spp);
    const int sl = static_cast<int>(sid % (F.ppw * F.spp));
    const int pix = sl / F.spp, smp = sl % F.spp;
    int64_t oidx;
    bool rec = hits != nullptr;
    if (F.adapt) {
      // adaptaa's sample k of a region: trace(hammersley(k, s*s) * (w, h) +
      // (x1, y1)) (RayTracer.cpp:333-337; hammersley's y is 0, U7)
      double x1, x2, y1, y2;
      if (F.aregs) {
        const ARegion R = F.aregs[item];
        x1 = R.x1, x2 = R.x2, y1 = R.y1, y2 = R.y2;
        oidx = item;
        rec = false;  // hit records: the pixel's own samples only
      } else {
        int i, j;
        if (!item_pixel(F, item, 0, i, j, oidx)) continue;
        x1 = double(i) / double(P.width), x2 = double(i + 1) / double(P.width);
        y1 = double(j) / double(P.height), y2 = double(j + 1) / double(P.height);
        if (x1 + 0.0001 >= x2 || y1 + 0.0001 >= y2) continue;  // the whole pixel under eps: black (U8)
      }
      L.sx() = radinv2(smp) * (x2 - x1) + x1;
      L.sy() = (0.0 / F.spp) * (y2 - y1) + y1;
    } else {
      int i, j;
      if (!item_pixel(F, item, pix, i, j, oidx)) continue;
      int pi = i, pj = j;
      double ssx = 1.0, ssy = 1.0;
      if (P.aa_mode != RTX_AA_NONE) {  // tracePixel(i*s + si, j*s + sj)
        pi = i * F.s + smp / F.s;
        pj = j * F.s + smp % F.s;
        ssx = F.s;
        ssy = F.s;
      }
      L.sx() = double(pi) / (double(P.width) * ssx);  // tracePixel (RayTracer.cpp:87-88)
      L.sy() = double(pj) / (double(P.height) * ssy);
    }
    L.sample_slot() = static_cast<int>(RTX_CHK(CHK_SAMPLE, oidx * F.spp + smp, F.chk_samples));
    // the buckets' owner: the sample, or with the DoF split its camera ray
    L.bunit() = F.cam_split ? L.sample_slot() * F.ncam + cam0 : L.sample_slot();
    if (F.fork_on) L.bunit() = RTX_CHK(CHK_BUNIT, L.bunit(), F.chk_units);
    if (F.fork_on) {  // no bucket written yet (forks come later), no set taken
      F.fmask[L.bunit()] = 0u;
      F.bidx[L.bunit()] = -1;
    }
    L.rec_on() = rec;
    L.pass() = 0;
    L.camk() = cam0;
    L.cam_end() = F.cam_split ? cam0 + 1 : F.ncam;
    L.nrays() = 0;
    L.acc() = mk3(0, 0, 0);
    L.fpos() = 0;
    L.st() = ST_CAM;
  }
}

#include "rtx_fused.h"

template <bool STATS, bool MEDIA, bool FORK>
__global__ void __launch_bounds__(WG, RTX_ADV_WAVES) advance_kernel(DevScene S, const DevScene* __restrict__ Sg, const FrameParams* __restrict__ Fp, LaneMem lm,
                                                      double* __restrict__ sbuf, RtxHitRecord* __restrict__ hits,
                                                      double* __restrict__ pbuf, int pend_cap, QList q0, QList q1,
                                                      unsigned int* __restrict__ counters,
                                                      unsigned long long* __restrict__ stats, int slot_off,
                                                      const int* __restrict__ live_in, int* __restrict__ live_out,
                                                      int first, int in_cnt, int out_cnt) {
  const FrameParams& F = *Fp;
  // live slots only: the first iteration covers the group's slots, later
  // ones the slots the previous iteration left alive (its live_out list), so
  // the frame's tail iterations cost what their few live slots cost
  const int tid = blockIdx.x * WG + threadIdx.x;
  const bool valid = first || tid < static_cast<int>(counters[in_cnt]);
  const int slot = first ? slot_off + tid : (valid ? live_in[tid] : slot_off);
  Counters C = {0, 0, 0, 0, 0, 0, 0};
  LaneRef L(lm, static_cast<size_t>(slot));
  if (first) lane_init(L);
  int qm = Q_NONE;
  // fork slots: the group's slots past its sample slots (none in the
  // first iteration, which only starts camera rays)
  const ForkCtx fk = {counters + CNT_FORK, slot_off + F.wf_gsamp,
                      first ? 0u : static_cast<unsigned int>(F.wf_gs - F.wf_gsamp), live_out, counters + out_cnt,
                      nullptr, F.chk_live};
  if (valid && (L.st() != ST_IDLE || slot_unit(F, slot, L.kdone()) >= 0)) {
    // the previous iteration's query result is already in L.bt()/bobj/bsub/bhave
    L.qmode() = Q_NONE;
    for (;;) {
      claim_sample(L, F, hits, slot);
      if (L.st() == ST_IDLE) break;
      advance_lane<STATS, false, MEDIA, FORK>(L, *Sg, F, C, sbuf, nullptr, hits, 0, 0, pbuf, lm.n,
                                              static_cast<size_t>(slot), pend_cap, &fk);
      if (L.qmode() != Q_NONE) break;
    }
    qm = L.qmode();
  }
  // compaction: append queries to their list, one atomic per wave per list
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int m = Q_CLOSEST; m <= Q_NEXT; ++m) {
    const unsigned long long mask = __ballot(qm == m);
    if (mask == 0ull) continue;
    unsigned int base = 0;
    if (lane == 0)
      base = atomicAdd(&counters[CNT_Q + (m - 1) * CNT_LINE], static_cast<unsigned int>(__popcll(mask)));
    base = __shfl(base, 0);
    if (qm == m) {
      const QList& Q = m == Q_CLOSEST ? q0 : q1;
      const size_t cap = Q.cap;
      const size_t k = base + lane_prefix(mask);
      dvec3 qP = L.rp(), qD = L.rd();
      double qlim = RTX_INF;
      if (m == Q_NEXT) {
        next_query_ray<MEDIA>(S, L, qP, qD, qlim);
      }
      Q.slot[k] = slot;
      Q.d[0 * cap + k] = qP.x;
      Q.d[1 * cap + k] = qP.y;
      Q.d[2 * cap + k] = qP.z;
      Q.d[3 * cap + k] = qD.x;
      Q.d[4 * cap + k] = qD.y;
      Q.d[5 * cap + k] = qD.z;
      Q.d[6 * cap + k] = L.qtp();
      Q.d[7 * cap + k] = qlim;
      Q.iv[0 * cap + k] = L.qrp();
      Q.iv[1 * cap + k] = L.qsq();
    }
  }
  const bool live = valid && L.st() != ST_IDLE;  // a query pending: advance it again next iteration
  const unsigned long long alive = __ballot(live);
  if (alive) {
    unsigned int base = 0;
    if (lane == 0) base = atomicAdd(&counters[out_cnt], static_cast<unsigned int>(__popcll(alive)));
    base = __shfl(base, 0);
    if (live) live_out[RTX_CHK(CHK_LIVE, base + lane_prefix(alive), F.chk_live)] = slot;
  }
  if (STATS) {
    stats_add(C, stats, lane);
  }
}

// Tail of a slot group: once few slots are left, each remaining slot runs
// its own chain — state machine, query, state machine, ... — to the end in
// one persistent launch (the megakernel's inner loop over the wavefront's
// lane state).  In the batched iterations every launch waits for its slowest
// query (grazing rays take up to ~1700 steps), so a frame's tail costs
// (iterations) x (worst query); here each lane only waits for its own.
template <bool STATS, bool MEDIA>
__global__ void __launch_bounds__(WG) tail_kernel(DevScene S, const DevScene* __restrict__ Sg,
                                                   const FrameParams* __restrict__ Fp, LaneMem lm,
                                                   double* __restrict__ sbuf, RtxHitRecord* __restrict__ hits,
                                                   double* __restrict__ pbuf, int pend_cap,
                                                   const unsigned int* __restrict__ counters,
                                                   const int* __restrict__ live_in, int in_cnt, int stack_cap,
                                                   unsigned long long* __restrict__ stats) {
  extern __shared__ int lds_stack[];
  const FrameParams& F = *Fp;
  const int lane = threadIdx.x & 63;
  int* stk = lds_stack + (threadIdx.x >> 6) * stack_cap * 64;
  const int tid = blockIdx.x * WG + threadIdx.x;
  Counters C = {0, 0, 0, 0, 0, 0, 0};
  bool valid = tid < static_cast<int>(counters[in_cnt]);
  const int slot = valid ? live_in[tid] : 0;
  LaneRef L(lm, static_cast<size_t>(slot));
  const unsigned long long t_start = STATS ? __builtin_readcyclecounter() : 0ull;
  int64_t queries = 0;
  // one query at a time per wave (each lane waits for its wave's slowest);
  // the decoupled variant below measured slower (8-way shard 31.2 vs 25.8
  // ms, full frame 97 vs 90): its wave executes the state machine for a few
  // lanes in most rounds
  if (valid) {
    for (;;) {
      // the last query's result is in L.bt()/bobj/bsub/bhave
      L.qmode() = Q_NONE;
      claim_sample(L, F, hits, slot);
      if (L.st() == ST_IDLE) break;
      advance_lane<STATS, false, MEDIA>(L, *Sg, F, C, sbuf, nullptr, hits, 0, 0, pbuf, lm.n, static_cast<size_t>(slot),
                                 pend_cap);
      const int qm = L.qmode();
      if (qm == Q_NONE) continue;
      dvec3 qP = L.rp(), qD = L.rd();
      double qlim = RTX_INF;
      if (qm == Q_NEXT) {
        next_query_ray<MEDIA>(S, L, qP, qD, qlim);
      }
      double bt;
      int bobj, bsub;
      const bool have = traverse_any<STATS>(S, qm, qP, qD, L.qtp(), L.qrp(), L.qsq(), qlim, bt, bobj, bsub, stk, lane, C);
      L.bt() = bt;
      L.bobj() = bobj;
      L.bsub() = bsub;
      L.bhave() = have ? 1 : 0;
      if (STATS) queries++;
    }
  }
  if (STATS && tid < static_cast<int>(counters[in_cnt])) {  // the slowest chain of the tail (RTX_DEBUG report)
    atomicMax(&stats[6 + 10], static_cast<unsigned long long>(__builtin_readcyclecounter() - t_start));
    atomicMax(&stats[7 + 10], static_cast<unsigned long long>(queries));
  }
  if (STATS) {
    stats_add(C, stats, lane);
    stats_add_class(C, stats, lane, 30);
  }
}

// Persistent traversal of one group's compacted query list.  A wave claims
// 64 queries at a time (one atomic) and hands them to its idle lanes (ballot
// + mbcnt) once every lane's query is done.  Refilling idle lanes earlier
// (once fewer than 16 / 40 / 56 lanes were still stepping) measured slower
// (197 / 205 / 220 vs 182 ms/frame at the time): mixing a new query into a
// wave whose other lanes are deep in the tree costs more (divergent nodes
// and modes) than the idle lanes waste; the claims still balance waves
// against each other.  The fused machine relies on it (trav_reset below).
// FUSED (Q_NEXT on fused frames, rtx_fused.h): the list holds walk records;
// a lane whose query completes runs the walk's next step (walk_hit) and
// either queries again from the hit's key or writes the light's term to
// wterm[light][slot].
// FUSED Q_CLOSEST: a lane whose query completes shades the hit (shade_hit:
// colour, walk records, reflection / refraction pushes) before it claims
// the next query.
// CAM: the first iteration's instantiation (claims + first camera rays,
// SA.cam_n > 0); the others carry none of that code, so the later
// iterations' closest-hit launches keep their own register budget.
// LDS (trace_lds_bytes): per wave, the stack — [stack_cap][64] entries, or
// with SHORT [RTX_LDS_STACK][64] and the deeper entries in the group's
// overflow columns (StackShort) — then [RTX_COLD_FIELDS][64] doubles of the
// traversal's cold state (ColdLDS: the world ray and its reciprocal, 19
// VGPRs the persistent walk state no longer holds; spills of the fused
// kernels 48 / 64 B -> 0 / 16 B, headline 31.8-32.0 -> 30.6-31.2 ms).
template <bool STATS, int MODE, bool FUSED = false, bool FORK = false, bool CAM = false, bool SHORT = false>
__global__ void __launch_bounds__(WG, RTX_TRACE_WAVES)
    trace_kernel(DevScene S, const DevScene* __restrict__ Sg, QList Q, unsigned int* __restrict__ counters,
                 LaneMem lm, int stack_cap, unsigned long long* __restrict__ stats, double* __restrict__ wterm,
                 ShadeArgs SA, int clr) {
  extern __shared__ int lds_stack[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int scap = SHORT ? SA.lds_k : stack_cap;  // stack entries per lane in LDS
  using Stk = typename std::conditional<SHORT, StackShort, StackLDS>::type;
  Stk stk;
  if constexpr (SHORT)
    stk = StackShort{lds_stack + wave * scap * 64 + lane, lds_stack, SA.ovf + blockIdx.x * WG,
                     static_cast<int>(gridDim.x) * WG, scap};
  else
    stk = StackLDS{lds_stack + wave * stack_cap * 64 + lane};
  const size_t cap = Q.cap;
  const bool cam = CAM && FUSED && MODE == Q_CLOSEST && SA.cam_n > 0;  // first iteration: claims + camera rays here
  const unsigned int nq = cam ? static_cast<unsigned int>(SA.cam_n) : counters[CNT_Q + (MODE - 1) * CNT_LINE];
  unsigned int* claim = counters + CNT_CLAIM + (MODE - 1) * CNT_LINE;

  Counters C = {0, 0, 0, 0, 0, 0, 0};
  TravT<ColdLDS> T;
  T.cold.c = reinterpret_cast<double*>(lds_stack + WAVES_PER_WG * scap * 64) + wave * RTX_COLD_FIELDS * 64 + lane;
  bool active = false;
  size_t kq = 0;
  // wave-uniform claim state: [qnext, qend) of the list
  unsigned int qnext = 0, qend = 0;
  bool exhausted = false;
  int64_t wsteps = 0, lsteps = 0;
  int qsteps = 0;
  // (STATS) the wave's start, its claims and walk restarts: the slowest
  // wave of the launch is reported by RTX_DEBUG=2
  const uint64_t wt0 = STATS ? wall_clock64() : 0;
  // (STATS) cycle breakdown by unit class (RTX_STATS_PROF)
  uint64_t pcyc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pcnt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, xcyc = 0, xcnt = 0;
  const uint64_t pt0 = STATS ? clock64() : 0;
  unsigned int nclaims = 0, nrestart = 0;
  auto finish = [&]() {
    const size_t slot = static_cast<size_t>(Q.slot[kq]);
    lm.d[size_t(LD_bt) * lm.n + slot] = T.bt;
    lm.i[size_t(LI_bobj) * lm.n + slot] = T.bobj;
    lm.i[size_t(LI_bsub) * lm.n + slot] = T.bsub;
    lm.i[size_t(LI_bhave) * lm.n + slot] = T.have ? 1 : 0;
  };
  bool pend = false;  // FUSED: the lane's walk query completed, its walk step is due
  // FUSED: the walk step of a completed query — the next query of the walk
  // (its record keeps the walk's state and the new key) or the light's term
  auto walk_phase = [&](bool have_in, double bt_in, int bo_in, int bs_in) {
    bool w_have = have_in;
    double w_bt = bt_in;
    int w_bo = bo_in, w_bs = bs_in;
    while (pend) {
      // opaque record index: the record's field addresses are formed here
      // from (uniform base, k) each time, instead of being hoisted out of
      // the loop as a dozen 64-bit addresses that spill to scratch and come
      // back as dependent scratch loads (the LaneRef::refresh idea)
      size_t k = kq;
      asm volatile("" : "+v"(k));
      const int code = Q.iv[1 * cap + k];
      (void)RTX_CHK(CHK_LIGHT, walk_light(code), Sg->n_lights);
      (void)RTX_CHK(CHK_PICK, walk_pick(code) + 1, Sg->ss_res + 1);
      (void)RTX_CHK(CHK_WUNIT, SA.Fp->lunit[walk_light(code)] + (walk_pick(code) < 0 ? 0 : 2 + walk_pick(code)),
              SA.Fp->chk_wunits);
      const RtxLight& L = Sg->lights[walk_light(code)];
      const dvec3 pb = mk3(Q.d[QF_PX * cap + k], Q.d[QF_PY * cap + k], Q.d[QF_PZ * cap + k]);
      const dvec3 sdir = walk_dir(*Sg, code, pb);  // as the emitter computed it
      WalkState w;
      if (Q.iv[0 * cap + k] < 0) {  // the walk's first hit (light.cpp:28-29)
        w.wpos = pb;
        w.sattn = mk3(1.0, 1.0, 1.0);
        w.last_t = 0.0;
      } else {
        w.wpos = mk3(Q.d[QF_WPX * cap + k], Q.d[QF_WPY * cap + k], Q.d[QF_WPZ * cap + k]);
        w.sattn = mk3(Q.d[QF_SAX * cap + k], Q.d[QF_SAY * cap + k], Q.d[QF_SAZ * cap + k]);
        w.last_t = Q.d[QF_LAST * cap + k];
      }
      const double bt = w_bt;
      const int bo = w_bo, bs = w_bs;
      dvec3 res;
      if (walk_hit(*Sg, L, pb, sdir, w_have, bt, bo, bs, w, res)) {
        const size_t slot = static_cast<size_t>(Q.slot[k]);
        if (walk_pick(code) < 0) {
          const dvec3 dsc = mk3(Q.d[QF_SCX * cap + k], Q.d[QF_SCY * cap + k], Q.d[QF_SCZ * cap + k]);
          walk_store(wterm, SA.Fp->lunit, lm.n, slot, code, L, Q.d[QF_DATTN * cap + k], dsc, res);
        } else {
          walk_store(wterm, SA.Fp->lunit, lm.n, slot, code, L, 0.0, res, res);  // an area pick's attenuation
        }
        pend = false;
      } else {
        Q.d[QF_WPX * cap + k] = w.wpos.x;
        Q.d[QF_WPY * cap + k] = w.wpos.y;
        Q.d[QF_WPZ * cap + k] = w.wpos.z;
        Q.d[QF_SAX * cap + k] = w.sattn.x;
        Q.d[QF_SAY * cap + k] = w.sattn.y;
        Q.d[QF_SAZ * cap + k] = w.sattn.z;
        Q.d[QF_LAST * cap + k] = w.last_t;
        Q.iv[0 * cap + k] = bo;
        active = trav_init<STATS, MODE>(T, S, pb, sdir, bt, bo, bs, shadow_limit(*Sg, L, pb, false), C);
        pend = !active;  // answered by the root test: the walk's next step
        if (STATS) nrestart++;
        w_have = T.have;
        w_bt = T.bt;
        w_bo = T.bobj;
        w_bs = T.bsub;
      }
    }
  };
  for (;;) {
    const uint64_t xt0 = STATS ? clock64() : 0;
    if (FUSED) {
      // Every lane is idle here (the step loop below runs until
      // no lane is active), so the walk state is dead: resetting it to
      // constants tells the register allocator so, and the walk / shading
      // step's temporaries reuse its registers instead of spilling around it.
      const bool have = T.have;
      const double bt = T.bt;
      const int bo = T.bobj, bs = T.bsub;
      trav_reset(T);
      if (MODE == Q_NEXT) {
        walk_phase(have, bt, bo, bs);
      } else if (pend) {
        const FrameParams& F = *SA.Fp;
        const ForkCtx fk = {counters + CNT_FORK, SA.slot_off + F.wf_gsamp, static_cast<unsigned int>(F.wf_gs - F.wf_gsamp),
                            SA.live_out, counters + SA.out_cnt, SA.free_ids, F.chk_live};
        const WalkEmit we = {SA.qn, counters + CNT_Q + CNT_LINE, -1, 0};
        LaneRef LR(lm, static_cast<size_t>(cam ? SA.slot_off + static_cast<int>(kq) : Q.slot[kq]));
        const QRay qr = cam ? cam_first_ray(LR, F) : qray_at(LR, SA.pbuf, lm.n);
        // the scene through the device copy: indexing the by-value kernel
        // argument (cube-map faces) would copy all of it to scratch
        shade_hit<STATS, FORK>(LR, *Sg, F, C, SA.hits, SA.pbuf, lm.n, SA.pend_cap, &fk, &we, qr, have, bt, bo, bs);
        pend = false;
      }
    }
    unsigned long long idle = __ballot(!active);
    while (idle != 0ull && !exhausted) {
      if (qnext >= qend) {
        unsigned int base = nq;
        if (lane == 0) base = atomicAdd(claim, 64u);
        base = __shfl(base, 0);
        if (base >= nq) {
          exhausted = true;
        } else {
          if (STATS) nclaims++;
          qnext = base;
          qend = base + 64u < nq ? base + 64u : nq;
        }
        if (exhausted) break;
      }
      const unsigned int rank = lane_prefix(idle);
      const unsigned int avail = qend - qnext;
      const unsigned int nidle = __popcll(idle);
      const unsigned int take = avail < nidle ? avail : nidle;
      if (!active && !pend && rank < take) {
        kq = RTX_CHK(CHK_QREC, static_cast<size_t>(qnext) + rank, cap);
        bool noq = false;
        if (!FUSED) {
          const dvec3 P = mk3(Q.d[0 * cap + kq], Q.d[1 * cap + kq], Q.d[2 * cap + kq]);
          const dvec3 D = mk3(Q.d[3 * cap + kq], Q.d[4 * cap + kq], Q.d[5 * cap + kq]);
          active = trav_init<STATS, MODE>(T, S, P, D, Q.d[6 * cap + kq], Q.iv[0 * cap + kq], Q.iv[1 * cap + kq],
                                          Q.d[7 * cap + kq], C);
        } else if (MODE == Q_CLOSEST && cam) {  // claim the slot's first sample, its first camera ray
          const int slot = SA.slot_off + static_cast<int>(kq);
          LaneRef LR(lm, static_cast<size_t>(slot));
          // inlined (scratch 60-76 -> 16 B, headline -0.8 %); out of line in
          // the counting, short-stack and bounds-check instantiations, on which the backend
          // stops ("Subtarget requires even aligned vector registers": a
          // 64-bit scratch reload into an odd register pair)
          noq = STATS || SHORT || kBoundsCheck ? !cam_first_claim(lm, slot, *SA.Fp, SA.hits)
                                               : !cam_first_claim_inl(lm, slot, *SA.Fp, SA.hits);
          if (!noq) {
            if (STATS) C.camera++;
            // the ray from the claim's (sx, sy), here rather than through an
            // out-parameter of the out-of-line claim (a stack object: 80 B
            // of scratch written and read per camera ray)
            const QRay qr = cam_first_ray(LR, *SA.Fp);
            active = trav_init<STATS, MODE>(T, S, qr.p, qr.d, -RTX_INF, -1, -1, RTX_INF, C);
          }
        } else if (MODE == Q_CLOSEST) {  // fused closest record: the ray only
          const dvec3 P = mk3(Q.d[0 * cap + kq], Q.d[1 * cap + kq], Q.d[2 * cap + kq]);
          const dvec3 D = mk3(Q.d[3 * cap + kq], Q.d[4 * cap + kq], Q.d[5 * cap + kq]);
          active = trav_init<STATS, MODE>(T, S, P, D, -RTX_INF, -1, -1, RTX_INF, C);
        } else {  // a walk's first query (continuations restart in walk_phase)
          const int code = Q.iv[1 * cap + kq];
          const RtxLight& L = Sg->lights[walk_light(code)];
          const dvec3 pb = mk3(Q.d[QF_PX * cap + kq], Q.d[QF_PY * cap + kq], Q.d[QF_PZ * cap + kq]);
          active = trav_init<STATS, MODE>(T, S, pb, walk_dir(*Sg, code, pb), -RTX_INF, -1, -1,
                                          shadow_limit(*Sg, L, pb, true), C);
        }
        if (!active) {
          if (FUSED) pend = !noq;  // (a slot without a sample: nothing to shade)
          else finish();
        }
      }
      qnext += take;
      idle = __ballot(!active && !pend);
    }
    if (STATS) {
      xcyc += clock64() - xt0;
      xcnt++;
    }
    if (__ballot(active || pend) == 0ull) break;  // nothing claimed and nothing left
    do {
      // Postponed costly units (Aila & Laine's while-while, one call site):
      // while at least leaf_k lanes of the wave are at a 4-wide record, only
      // those lanes step, so most steps run the record test alone instead of
      // the record test AND the object / face tests of a mixed wave.  A
      // lane's own sequence of units is unchanged (results identical).
      const unsigned long long at_rec = __ballot(active && trav_at_record(T));
      const bool go = active && (static_cast<int>(__popcll(at_rec)) < SA.leaf_k || trav_at_record(T));
      uint64_t st0 = 0;
      int combo = 0;
      if (STATS) {  // SIMD efficiency of the walk (RTX_DEBUG report)
        wsteps++;
        lsteps += __popcll(__ballot(go));
        const int cls = !go ? 0 : (trav_at_record(T) ? 1 : (T.mode == 2 ? 4 : 2));
        combo = static_cast<int>((__ballot(cls == 1) ? 1 : 0) | (__ballot(cls == 2) ? 2 : 0) |
                                 (__ballot(cls == 4) ? 4 : 0));
        st0 = clock64();
      }
      if (go) {
        if (STATS) qsteps++;
        const bool qdone = trav_step<STATS, MODE>(T, S, stk, C);
        (void)RTX_CHK(CHK_STACK, T.sp, stack_cap + 1);  // (sp <= stack_cap: the LDS or overflow columns held every push)
        if (qdone) {
          if (FUSED) pend = true;
          else finish();
          active = false;
          if (STATS) {  // per-query step statistics (RTX_DEBUG report)
            atomicMax(&stats[12 + (MODE - 1)], static_cast<unsigned long long>(qsteps));
            if (qsteps > 100) atomicAdd(&stats[14 + (MODE - 1)], 1ull);
          }
          qsteps = 0;
        }
      }
      if (STATS) {
        const uint64_t dt = clock64() - st0;
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (c == combo) {
            pcyc[c] += dt;
            pcnt[c]++;
          }
      }
    } while (__ballot(active) != 0ull);
  }
  if (STATS && lane == 0) {
    unsigned long long* pr = stats + RTX_STATS_PROF + 20 * (MODE - 1);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      atomicAdd(&pr[c], static_cast<unsigned long long>(pcyc[c]));
      atomicAdd(&pr[8 + c], static_cast<unsigned long long>(pcnt[c]));
    }
    atomicAdd(&pr[16], static_cast<unsigned long long>(xcyc));
    atomicAdd(&pr[17], static_cast<unsigned long long>(xcnt));
    atomicAdd(&pr[18], static_cast<unsigned long long>(clock64() - pt0));
  }
  if (STATS) {
    stats_add(C, stats, lane);  // traversal counts (and the shading's, FUSED Q_CLOSEST)
    stats_add_class(C, stats, lane, MODE == Q_CLOSEST ? 20 : 25);
    if (lane == 0) {
      atomicAdd(&stats[8 + 2 * (MODE - 1)], static_cast<unsigned long long>(wsteps));
      atomicAdd(&stats[9 + 2 * (MODE - 1)], static_cast<unsigned long long>(lsteps));
      // the slowest wave (100 MHz wall clock ticks in the high word): its
      // wave steps; its claims and walk restarts
      const unsigned long long dur = static_cast<unsigned long long>(wall_clock64() - wt0) << 32;
      atomicMax(&stats[35 + 2 * (MODE - 1)], dur | static_cast<unsigned long long>(wsteps & 0xffffffffll));
      atomicMax(&stats[36 + 2 * (MODE - 1)],
                dur | (static_cast<unsigned long long>(nclaims & 0xffffu) << 16) | (nrestart & 0xffffu));
    }
  }
  // clr >= 0 (the iteration's last launch): the last workgroup to finish
  // clears the next iteration's counters (lines clr .. clr + 4: its live-slot
  // count, query counts and claim cursors), so no memset launch has to wait
  // for CU space between iterations
  if (clr >= 0) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      const unsigned int prev = atomicAdd(&counters[CNT_DONE], 1u);
      if (prev == gridDim.x - 1) {
        counters[CNT_DONE] = 0u;
        for (int l = clr; l < clr + 5; ++l) counters[l * CNT_LINE] = 0u;
        __threadfence();
      }
    }
  }
}

// Slots [first, first + n) start idle (lane_init): on a frame whose first
// closest-hit launch claims the samples (cam_first_claim), the slots it does
// not claim — spare (fork) slots and sample slots without a first sample.
__global__ void __launch_bounds__(WG) lane_init_kernel(LaneMem lm, int first, int n) {
  const int t = blockIdx.x * WG + threadIdx.x;
  if (t >= n) return;
  LaneRef L(lm, static_cast<size_t>(first + t));
  lane_init(L);
}

// trace()'s value of sample sid (RayTracer.cpp:35-79) from the sample buffer:
//   DoF split — the sample's camera rays' sums added in order, scaled and
//     clamped (RayTracer.cpp:73-77); a camera ray's sum is its root's plus,
//     with buckets, its buckets in heap order;
//   buckets — the root's sum plus the forked sub-trees' sums in heap order,
//     then the clamp (RayTracer.cpp:77);
//   otherwise the buffer holds the clamped value already.
__device__ __forceinline__ dvec3 sample_value(const FrameParams& F, const double* __restrict__ sbuf, int64_t sid) {
  auto unit_sum = [&](int64_t uid) {
    const double* r = sbuf + uid * 3;
    dvec3 u = mk3(r[0], r[1], r[2]);
    if (F.fork_on) {
      unsigned int m = F.fmask[uid];
      const int64_t set = m ? F.bidx[uid] : 0;
      while (m) {
        const int b = __builtin_ctz(m);
        m &= m - 1;
        const double* f = F.fbuf + (set * F.fork_npos + b) * 3;
        u += mk3(f[0], f[1], f[2]);
      }
    }
    return u;
  };
  if (F.cam_split) {
    dvec3 ret = unit_sum(sid * F.ncam);
    for (int k = 1; k < F.ncam; ++k) ret += unit_sum(sid * F.ncam + k);
    ret *= (1.0 / (F.P.dof_div + 1.0));
    return rtm::gclamp3(ret, 0.0, 1.0);
  }
  if (F.fork_on) return rtm::gclamp3(unit_sum(sid), 0.0, 1.0);
  return ld3(sbuf + sid * 3);
}

// The pixel (i, j) of output slot o, false for a slot this frame does not
// write: outside the image (packed tiles at the border) or, on a sharded
// full frame, another shard's tile.
__device__ __forceinline__ bool slot_pixel(const FrameParams& F, int64_t o, int& i, int& j) {
  if (F.P.packed && F.P.tile > 0) {
    const int64_t k = o / (int64_t(F.tw) * F.th);
    const int r = static_cast<int>(o % (int64_t(F.tw) * F.th));
    int tx, ty;
    deal_tile(F.P.shard + static_cast<int>(k) * F.P.nshards, F.tiles_x, tx, ty);
    i = tx * F.tw + r % F.tw;
    j = ty * F.th + r / F.tw;
    return i < F.P.width && j < F.P.height;
  }
  i = static_cast<int>(o % F.P.width);
  j = static_cast<int>(o / F.P.width);
  if (F.P.tile > 0) return tile_deal(i / F.tw, j / F.th, F.tiles_x) % F.P.nshards == F.P.shard;
  return true;
}

// Per-pixel ordered reduction of the sample buffer (RayTracer.cpp:288-298:
// col += tracePixel(...) in si-major order, col /= s*s; setPixel truncates).
// zeros into output slot o (packed padding)
__device__ __forceinline__ void pad_slot(int64_t o, uint8_t* __restrict__ rgb8, double* __restrict__ rgbf) {
  if (rgb8) rgb8[o * 3 + 0] = rgb8[o * 3 + 1] = rgb8[o * 3 + 2] = 0;
  if (rgbf) rgbf[o * 3 + 0] = rgbf[o * 3 + 1] = rgbf[o * 3 + 2] = 0.0;
}

__global__ void __launch_bounds__(WG) reduce_kernel(const FrameParams* __restrict__ Fp, const double* __restrict__ sbuf,
                                                     uint8_t* __restrict__ rgb8, double* __restrict__ rgbf,
                                                     int64_t npix_slots) {
  // one thread per sample, WG / spp pixels per workgroup: lane k reads sample
  // k's sums (neighbouring lanes neighbouring samples, coalesced), the
  // values meet in LDS and the pixel's first lane adds them in sample order
  // (with one thread per pixel, each load instruction touched 64 lines
  // spp * 24 B apart)
  __shared__ double sv[WG * 3];
  const FrameParams& F = *Fp;
  const int spp = F.spp;
  const int ppb = WG / spp;  // (spp <= 64: regular AA is capped at 8 x 8)
  const int t = threadIdx.x;
  const int pl = t / spp, q = t - pl * spp;
  const int64_t o = static_cast<int64_t>(blockIdx.x) * ppb + pl;
  int i, j;
  const bool in_slots = pl < ppb && o < npix_slots;
  const bool own = in_slots && slot_pixel(F, o, i, j);
  if (own) {
    const dvec3 v = sample_value(F, sbuf, o * spp + q);
    sv[t * 3 + 0] = v.x;
    sv[t * 3 + 1] = v.y;
    sv[t * 3 + 2] = v.z;
  }
  __syncthreads();
  if (!in_slots || q != 0) return;
  if (!own) {
    // a packed shard's slot past the image border (a partial tile): zeros,
    // as a host-mode render leaves it, not whatever the caller's buffer held
    // (a sharded full frame's other tiles are not ours to write)
    if (F.P.packed && F.P.tile > 0) pad_slot(o, rgb8, rgbf);
    return;
  }
  dvec3 acc = mk3(0.0, 0.0, 0.0);
  for (int k = 0; k < spp; ++k) acc += mk3(sv[(t + k) * 3 + 0], sv[(t + k) * 3 + 1], sv[(t + k) * 3 + 2]);
  if (F.P.aa_mode != RTX_AA_NONE) acc = acc / double(F.s * F.s);
  if (rgb8) {
    rgb8[o * 3 + 0] = rtm::to_byte(acc.x);
    rgb8[o * 3 + 1] = rtm::to_byte(acc.y);
    rgb8[o * 3 + 2] = rtm::to_byte(acc.z);
  }
  if (rgbf) {
    rgbf[o * 3 + 0] = acc.x;
    rgbf[o * 3 + 1] = acc.y;
    rgbf[o * 3 + 2] = acc.z;
  }
}

// ============================================================ adaptive AA, wavefront path
// adaptaa (RayTracer.cpp:316-365) level by level.  A level's regions run
// their s*s samples as ordinary work units of the wavefront machine
// (claim_sample); then
//   adapt_stats_kernel   — each region's mean and deviation in the
//                          reference's order; keeps mu, or marks the region
//                          for subdivision and counts its quarters above eps;
//   adapt_emit_kernel    — appends the marked regions' quarters to the next
//                          level (their order there does not matter: each
//                          keeps its parent and quarter);
//   adapt_combine_kernel — deepest level first: a subdivided region's value
//                          is (sum of its quarters' values, in adaptaa's loop
//                          order, 0 for a quarter under eps) * 1/4; level 0
//                          writes the pixel (setPixel).
// With the default threshold no region subdivides and a frame is one level:
// the samples, one stats launch, one combine launch.
struct ALevel {
  dvec3* val;          // [n] region value
  int* first;          // [n] -1 kept; -2 subdivided, quarters not yet emitted; >= 0 first quarter's index below
  int* mask;           // [n] quarters present below (bit 2a + b)
  const ARegion* reg;  // [n] the regions (level >= 1; level 0's are the output slots' pixels)
  int64_t n;
};

// The regions [r0, r0 + nr) of a level whose samples are sample ids
// (r - r0) * spp + k of the sample buffer.
__global__ void __launch_bounds__(WG) adapt_stats_kernel(const FrameParams* __restrict__ Fp,
                                                          const double* __restrict__ sbuf, ALevel lv, int64_t r0,
                                                          int64_t nr, unsigned int* __restrict__ nsub) {
  const FrameParams& F = *Fp;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * WG + threadIdx.x;
  if (t >= nr) return;
  const int64_t r = r0 + t;
  double x1, x2, y1, y2;
  if (lv.reg) {
    const ARegion R = lv.reg[r];
    x1 = R.x1, x2 = R.x2, y1 = R.y1, y2 = R.y2;
  } else {
    int i, j;
    if (!slot_pixel(F, r, i, j)) {
      lv.first[r] = -1;
      return;
    }
    x1 = double(i) / double(F.P.width), x2 = double(i + 1) / double(F.P.width);
    y1 = double(j) / double(F.P.height), y2 = double(j + 1) / double(F.P.height);
    if (x1 + 0.0001 >= x2 || y1 + 0.0001 >= y2) {  // no samples: black (U8)
      lv.val[r] = mk3(0.0, 0.0, 0.0);
      lv.first[r] = -1;
      return;
    }
  }
  const int an = F.spp;
  dvec3 mu = mk3(0.0, 0.0, 0.0), sd = mk3(0.0, 0.0, 0.0);
  for (int k = 0; k < an; ++k) mu += sample_value(F, sbuf, t * an + k);
  mu *= (1.0 / (an));
  for (int k = 0; k < an; ++k) {
    const dvec3 s_c = sample_value(F, sbuf, t * an + k);
    sd += mk3(pow(fabs(s_c.x - mu.x), 2.0), pow(fabs(s_c.y - mu.y), 2.0), pow(fabs(s_c.z - mu.z), 2.0));
  }
  sd *= (1.0 / (an - 1));
  lv.val[r] = mu;
  lv.first[r] = -1;
  if (!(rtm::length(sd) > F.P.aa_thresh)) return;
  const double xs[3] = {x1, (x1 + x2) / 2.0, x2};
  const double ys[3] = {y1, (y1 + y2) / 2.0, y2};
  int m = 0;
  for (int c = 0; c < 4; ++c) {
    const int a = c >> 1, b = c & 1;
    if (!(xs[a] + 0.0001 >= xs[a + 1] || ys[b] + 0.0001 >= ys[b + 1])) m |= 1 << c;
  }
  lv.first[r] = -2;
  lv.mask[r] = m;
  if (m) atomicAdd(nsub, static_cast<unsigned int>(__popc(m)));
}

__global__ void __launch_bounds__(WG) adapt_emit_kernel(const FrameParams* __restrict__ Fp, ALevel lv, ARegion* next,
                                                         unsigned int* __restrict__ cursor) {
  const FrameParams& F = *Fp;
  const int64_t r = static_cast<int64_t>(blockIdx.x) * WG + threadIdx.x;
  if (r >= lv.n || lv.first[r] != -2) return;
  double x1, x2, y1, y2;
  if (lv.reg) {
    const ARegion R = lv.reg[r];
    x1 = R.x1, x2 = R.x2, y1 = R.y1, y2 = R.y2;
  } else {
    int i, j;
    slot_pixel(F, r, i, j);
    x1 = double(i) / double(F.P.width), x2 = double(i + 1) / double(F.P.width);
    y1 = double(j) / double(F.P.height), y2 = double(j + 1) / double(F.P.height);
  }
  const double xs[3] = {x1, (x1 + x2) / 2.0, x2};
  const double ys[3] = {y1, (y1 + y2) / 2.0, y2};
  const int m = lv.mask[r];
  const unsigned int base = m ? atomicAdd(cursor, static_cast<unsigned int>(__popc(m))) : 0u;
  unsigned int k = base;
  for (int c = 0; c < 4; ++c) {
    if (!((m >> c) & 1)) continue;
    const int a = c >> 1, b = c & 1;
    ARegion q;
    q.x1 = xs[a];
    q.x2 = xs[a + 1];
    q.y1 = ys[b];
    q.y2 = ys[b + 1];
    q.parent = static_cast<int>(r);
    q.child = c;
    next[k++] = q;
  }
  lv.first[r] = static_cast<int>(base);
}

// fold level `below` into `lv` (below.n == 0: nothing subdivided), and at
// level 0 write the pixels
__global__ void __launch_bounds__(WG) adapt_combine_kernel(const FrameParams* __restrict__ Fp, ALevel lv, ALevel below,
                                                            uint8_t* __restrict__ rgb8, double* __restrict__ rgbf) {
  const FrameParams& F = *Fp;
  const int64_t r = static_cast<int64_t>(blockIdx.x) * WG + threadIdx.x;
  if (r >= lv.n) return;
  if (!lv.reg) {
    int i, j;
    if (!slot_pixel(F, r, i, j)) {
      if (F.P.packed && F.P.tile > 0) pad_slot(r, rgb8, rgbf);  // (as reduce_kernel)
      return;
    }
  }
  dvec3 v = lv.val[r];
  if (lv.first[r] != -1) {  // mu = 0; mu += subval (2 x 2, RayTracer.cpp:352-360); mu *= 1/4
    const int m = lv.mask[r];
    int k = lv.first[r];
    dvec3 mu = mk3(0.0, 0.0, 0.0);
    for (int c = 0; c < 4; ++c) mu += ((m >> c) & 1) ? below.val[k++] : mk3(0.0, 0.0, 0.0);
    mu *= (1.0 / 4.0);
    v = mu;
    lv.val[r] = v;
  }
  if (lv.reg) return;
  if (rgb8) {
    rgb8[r * 3 + 0] = rtm::to_byte(v.x);
    rgb8[r * 3 + 1] = rtm::to_byte(v.y);
    rgb8[r * 3 + 2] = rtm::to_byte(v.z);
  }
  if (rgbf) {
    rgbf[r * 3 + 0] = v.x;
    rgbf[r * 3 + 1] = v.y;
    rgbf[r * 3 + 2] = v.z;
  }
}

// ============================================================ host side / C ABI
namespace {

thread_local std::string g_err;

// every render-path kernel launch, counted for rtx_kernel_time (`st`: the
// SceneState of the render in progress)
#define RTX_LAUNCH(...)                \
  do {                                 \
    hipLaunchKernelGGL(__VA_ARGS__);   \
    ++st->n_launch;                    \
  } while (0)
#define HIP_TRY(expr)                                                            \
  do {                                                                           \
    hipError_t e_ = (expr);                                                      \
    if (e_ != hipSuccess) {                                                      \
      g_err = std::string(#expr) + ": " + hipGetErrorString(e_);                 \
      return RTX_ERR_HIP;                                                        \
    }                                                                            \
  } while (0)

// Everything one frame writes on the device, with the streams its slot
// groups run on.  A scene holds two: consecutive frames rendered into device
// buffers without hit records or counters (bench.py's loop, bin/ray --gpus)
// alternate between them, so frame k + 1's first, throughput-bound
// iterations run while frame k's last, latency-bound ones finish (DESIGN.md
// "Frame contexts"); every other render uses context 0 in caller-stream
// order, as before.
struct FrameCtx {
  FrameParams* d_frame = nullptr;
  double* d_offv = nullptr;     // DoF eye offsets
  size_t offv_bytes = 0;
  double* d_sbuf = nullptr;     // per-sample colours (HBM), grown on demand
  size_t sbuf_bytes = 0;
  double* d_pbuf = nullptr;     // per-lane pending-ray stacks (HBM)
  size_t pbuf_bytes = 0;
  double* d_fbuf = nullptr;     // forked sub-tree sums
  size_t fbuf_bytes = 0;
  unsigned int* d_fmask = nullptr;  // forked positions per sample
  size_t fmask_bytes = 0;
  double* d_wterm = nullptr;    // fused walks' terms [light][slot][3]
  size_t wterm_bytes = 0;
  // wavefront path: slot state, query lists, counters
  void* d_wf = nullptr;
  size_t wf_bytes = 0;
  void* d_lane = nullptr;       // LaneRef state of every lane / slot (HBM)
  size_t lane_bytes = 0;
  std::vector<hipStream_t> wf_streams;  // wavefront slot groups
  std::vector<hipEvent_t> wf_join, wf_check;
  hipEvent_t wf_fork = nullptr;
  unsigned int* d_counters = nullptr;
  unsigned int* h_counters = nullptr;  // pinned
  DevScene* d_scene = nullptr;         // device copy of S_launch (shadow early-out)
  unsigned int* d_acnt = nullptr;      // adaptive AA: regions to subdivide, emit cursor
  // pooled bucket sets (FrameParams.bidx): per unit its set index; pool
  // counters [taken, refused]; a first-time frame's count, read back later
  int* d_bidx = nullptr;
  size_t bidx_bytes = 0;
  int* d_free = nullptr;  // per slot group: its free fork slots (fork_claim / advance_fused_kernel)
  size_t free_bytes = 0;
  int* d_ovf = nullptr;  // per slot group: the trace kernels' stack overflow columns (StackShort)
  size_t ovf_bytes = 0;
  unsigned int* d_bstat = nullptr;
  unsigned int* h_bstat = nullptr;  // pinned: [taken, refused, -, -, fork requests of group g at 4 + g]
  hipEvent_t bstat_ev = nullptr;
  bool bstat_pending = false;
  uint64_t bstat_key = 0;
  int bstat_groups = 0;  // groups whose fork counts were read back (0: the frame did not fork)
  // the last history-sized frame's check: its *bover (bit 1 a bucket set
  // refused, bit 2 a push that fit neither a fork slot nor the two-entry
  // stack), read back into h_bstat[2]; chk_keys are the frame's history keys
  hipEvent_t chk_ev = nullptr;
  bool chk_pending = false;
  int64_t chk_seq = -1;
  std::vector<uint64_t> chk_keys;
  int wf_call = 0;  // run_wavefront calls of the current rtx_render
  bool bstat_clear = false;  // d_bstat (incl. *bover) cleared by this rtx_render's first forking run
  // adaptive AA: one buffer per level (values, first-quarter index, mask,
  // regions), grown on demand and reused by later frames (no hipMalloc /
  // hipFree, which synchronises the device, per level per frame)
  std::vector<void*> d_level;
  std::vector<size_t> level_bytes;
  hipEvent_t free_ev = nullptr;  // recorded on the caller's stream after the frame's last kernel
  bool used = false;
};

struct SceneState {
  int device = 0;
  DevScene S;
  DevScene S_launch;
  std::vector<void*> allocs;
  RtxSceneDesc desc;           // shallow copy (pointers valid only during create)
  RtxCamera cam;
  std::vector<RtxLight> lights;
  int stack_cap = 0;
  int n_cu = 256;
  unsigned long long* d_work = nullptr;
  unsigned long long* d_stats = nullptr;
  double* d_picks = nullptr;
  int picks_res = -1;
  FrameCtx cx[4];
  unsigned int next_cx = 0;
  // frame contexts pipelined renders rotate over (RTX_CONTEXTS 2..4): 3 on
  // frames of at most 10 M work units — a frame's latency-bound tail then
  // overlaps the next two frames' first iterations (8-way headline shard
  // 4.78-4.87 vs 5.08-5.09 ms with 2, C4's 6.12-6.17 vs 6.35-6.40; 4
  // contexts no better: profiles/r05v_ab_contexts.txt) — 2 on larger ones
  // (a 2-way shard's third set of buffers would take it from 31 to 47 GiB)
  unsigned int n_cx = 3;
  unsigned int last_ncx = 1;  // contexts the last render rotated over (1: not pipelined)
  bool any_recur = true;  // some material reflects or refracts (no: no ray tree, no buckets)
  // Pinned staging for the frame's host-to-device copies (frame record,
  // scene record, DoF offsets).  A hipMemcpyAsync from pageable memory may
  // read the host buffer only when its stream reaches the copy — after the
  // caller's locals are gone, or rewritten by the next frame's render, when
  // the stream waits for an earlier frame (a pipelined frame waits for its
  // context's previous one).  Entries are reused round-robin; an entry's
  // event says its last copy has run.
  struct Stage {
    void* h = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    bool used = false;
  };
  Stage stage[16];
  unsigned int next_stage = 0;
  // what each frame (key: its parameters and its place in the render) took
  // on its first render: bucket sets, and the most fork requests of one
  // slot group (-1: unknown, the frame did not fork)
  struct FrameHist {
    uint32_t sets;
    int64_t forks;
  };
  std::map<uint64_t, FrameHist> bucket_hist;
  // frames whose two-entry pending stacks overflowed once: full stacks from
  // then on
  std::set<uint64_t> full_stack_keys;
  // fork depth per whole frame (whole_frame_key: the parameters without the
  // tile deal), decided once by depth_probe (rtx_render) from a fixed subset
  // of the whole frame, so a frame and every shard of it use the same depth
  std::map<uint64_t, int> depth_rule;
  bool probe_mode = false;              // render_once is depth_probe's render
  int64_t probe_req = 0, probe_units = 0;  // its fork requests and work units
  // rtx_render calls so far (a frame's sequence number), the wrong frames
  // found since the last rtx_frame_status, pipelined renders counted for
  // rtx_overlap_count
  int64_t frame_seq = 0;
  int64_t bad_first = -1, bad_n = 0;
  int64_t n_renders = 0, n_pipelined = 0;
  int64_t last_work[RTX_STATS_N] = {};  // raw counters of the last counting render (rtx_last_work)
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  std::vector<hipEvent_t> ev_start, ev_stop;
  int64_t n_launch = 0;  // kernel launches since the last rtx_kernel_time
};

template <typename T>
rtx_status upload(SceneState& st, const T* src, size_t n, const T** dst) {
  if (n == 0 || !src) {
    *dst = nullptr;
    return RTX_OK;
  }
  void* p = nullptr;
  HIP_TRY(hipMalloc(&p, n * sizeof(T)));
  st.allocs.push_back(p);
  HIP_TRY(hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice));
  *dst = static_cast<const T*>(p);
  return RTX_OK;
}

// Area-light sample positions (AreaLightRect::pick / AreaLightCirc::pick,
// light.cpp:106-131): host glibc cos/sin, exactly as the CPU restatement.
std::vector<double> make_picks(const std::vector<RtxLight>& lights, int res) {
  const double PI = 3.1415926535897932384626433832795028841971;
  std::vector<double> out(lights.size() * size_t(res > 0 ? res : 0) * 3, 0.0);
  for (size_t li = 0; li < lights.size(); ++li) {
    const RtxLight& L = lights[li];
    for (int i = 0; i < res; ++i) {
      dvec3 p = mk3(0, 0, 0);
      if (L.type == RTX_LIGHT_AREA_RECT) {
        double mul = 0.5, result = 0.0;
        int n = i;
        while (n > 0) {
          result += (n % 2) ? mul : 0;
          n /= 2;
          mul /= 2.0;
        }
        double px = result, py = ((double)n) / res;
        double a = (px - 0.5) * L.width, b = (py - 0.5) * L.height;
        p = mk3(L.u[0] * a + L.v[0] * b, L.u[1] * a + L.v[1] * b, L.u[2] * a + L.v[2] * b);
      } else if (L.type == RTX_LIGHT_AREA_CIRC || L.type == RTX_LIGHT_SPOT) {
        double ang_rad = 2 * PI / res * i;
        double dist = 0.5 * L.radius;
        double x = std::cos(ang_rad) * dist;
        double y = std::sin(ang_rad) * dist;
        const dvec3 ori = ld3(L.orient);
        const dvec3 ab = mk3(std::fabs(ori.x), std::fabs(ori.y), std::fabs(ori.z));
        dvec3 u = mk3(0.0, 0.0, 0.0);
        if (ab.x < ab.y && ab.x < ab.z) u = mk3(0.0, -ori.z, ori.y);
        else if (ab.y < ab.z) u = mk3(-ori.z, 0.0, ori.x);
        else u = mk3(-ori.y, ori.x, 0.0);
        u = rtm::normalize(u);
        const dvec3 v = rtm::cross(ori, u);
        p = x * u + y * v + ld3(L.pos);
      }
      out[(li * res + i) * 3 + 0] = p.x;
      out[(li * res + i) * 3 + 1] = p.y;
      out[(li * res + i) * 3 + 2] = p.z;
    }
  }
  return out;
}

int isqrt_floor(int v) {
  int r = 0;
  while ((r + 1) * (r + 1) <= v) ++r;
  return r;
}

}  // namespace

// compile-time dispatch of runtime flags to kernel template arguments
template <class Fn>
void dispatch2(bool a, bool b, Fn&& f) {
  if (a) {
    if (b) f(std::true_type{}, std::true_type{});
    else f(std::true_type{}, std::false_type{});
  } else {
    if (b) f(std::false_type{}, std::true_type{});
    else f(std::false_type{}, std::false_type{});
  }
}

template <class Fn>
void dispatch3(bool a, bool b, bool c, Fn&& f) {
  dispatch2(a, b, [&](auto x, auto y) {
    if (c) f(x, y, std::true_type{});
    else f(x, y, std::false_type{});
  });
}

extern "C" {

const char* rtx_last_error(void) { return g_err.c_str(); }

rtx_status rtx_device_count(int* n) {
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) c = 0;
  *n = c;
  return RTX_OK;
}

rtx_status rtx_scene_create(int device, const RtxSceneDesc* d, void** out) {
  if (!d || !out) {
    g_err = "rtx_scene_create: null argument";
    return RTX_ERR_INVALID;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    g_err = "rtx_scene_create: no HIP device visible";
    return RTX_ERR_NODEVICE;
  }
  if (device < 0 || device >= ndev) {
    g_err = "rtx_scene_create: bad device index";
    return RTX_ERR_INVALID;
  }
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos) {
    g_err = std::string("rtx_scene_create: device is ") + prop.gcnArchName + ", this build targets gfx950";
    return RTX_ERR_NODEVICE;
  }
  SceneState* st = new SceneState();
  st->device = device;
  st->n_cu = prop.multiProcessorCount;
  std::memset(&st->S, 0, sizeof(st->S));
  DevScene& S = st->S;
  rtx_status rc = RTX_OK;
#define UP(src, n, dst) \
  if ((rc = upload(*st, src, size_t(n), &dst)) != RTX_OK) { rtx_scene_destroy(st); return rc; }
  UP(d->scene_nodes, d->n_scene_nodes, S.snodes);
  // objects as the loader flattened them, with their mesh fields in pad
  // (augment_objects) and pad[RTX_OBJ_WOPAQUE]: 1 when a shadow walk that
  // hits the object cannot carry light past it — its material is not
  // transmissive and its kt a constant (0, 0, 0), with no per-vertex
  // materials (walk_hit's shortcut, rtx_fused.h)
  std::vector<RtxObject> objs;
  augment_objects(d, objs);
  for (RtxObject& o : objs) {
    bool op = o.material >= 0 && o.material < d->n_materials;
    if (op) {
      const RtxMaterial& m = d->materials[o.material];
      const RtxParam& kt = m.p[RTX_P_KT];
      op = !(m.flags & RTX_MF_TRANS) && kt.tex < 0 && kt.v[0] == 0.0 && kt.v[1] == 0.0 && kt.v[2] == 0.0;
    }
    if (op && o.type == RTX_OBJ_TRIMESH)
      op = o.mesh >= 0 && o.mesh < d->n_meshes && !d->meshes[o.mesh].has_vmats;
    o.pad[RTX_OBJ_WOPAQUE] = op ? 1 : 0;
  }
  UP(objs.data(), d->n_objects, S.objs);
  UP(d->obj_params, size_t(d->n_objects) * RTX_OBJ_PARAMS, S.oprm);
  UP(d->materials, d->n_materials, S.mats);
  UP(d->meshes, d->n_meshes, S.meshes);
  UP(d->mesh_nodes, d->n_mesh_nodes, S.mnodes);
  UP(d->faces, d->n_faces, S.faces);
  UP(d->face_ids, d->n_faces, S.fids);
  UP(d->vnormals, size_t(d->n_vnormals) * 3, S.vnormals);
  UP(d->vmats, d->n_vmats, S.vmats);
  UP(d->lights, d->n_lights, S.lights);
  UP(d->textures, d->n_textures, S.texs);
  UP(d->texels, d->n_texels, S.texels);
#undef UP
  {
    TravTrees tt;
    if (!build_trav_trees(d, tt)) {
      g_err = "rtx_scene_create: malformed BVH (leaf with more than 3 items or bad child link)";
      rtx_scene_destroy(st);
      return RTX_ERR_INVALID;
    }
    S.sroot = tt.sroot;
    // per-lane LDS stack: scene-level entries stay below a mesh walk's
    st->stack_cap = tt.sneed + tt.mneed + 2;
#define UP(src, n, dst) \
  if ((rc = upload(*st, src, size_t(n), &dst)) != RTX_OK) { rtx_scene_destroy(st); return rc; }
    UP(tt.sn4.data(), tt.sn4.size(), S.snode4);
    UP(tt.mn4.data(), tt.mn4.size(), S.mnode4);
    S.n_srec = static_cast<int32_t>(tt.sn4.size());
    UP(tt.mroots.data(), tt.mroots.size(), S.mroots);
    UP(tt.tfaces.data(), tt.tfaces.size(), S.tfaces);
    UP(tt.trank.data(), tt.trank.size(), S.trank);
    UP(tt.tmeta.data(), tt.tmeta.size(), S.tmeta);
#undef UP
  }
  for (int k = 0; k < 6; ++k) {
    S.cube[k] = d->cubemap[0] >= 0 ? d->cubemap[k] : -1;
    if (S.cube[k] >= d->n_textures || (d->cubemap[0] >= 0 && S.cube[k] < 0)) {
      g_err = "rtx_scene_create: cube-map face names no texture";
      rtx_scene_destroy(st);
      return RTX_ERR_INVALID;
    }
  }
  S.n_snodes = d->n_scene_nodes;
  S.n_objs = d->n_objects;
  S.n_lights = d->n_lights;
  S.margin = 1e-9 * scene_extent(d);
  S.lmargin = 1e-9 * mesh_extent(d);
  S.cos45 = std::cos(3.1415926535897932384626433832795028841971 / 4);
  for (int k = 0; k < 3; ++k) S.ambient[k] = d->ambient[k];
  S.air_index = (0.299 * 1.0) + (0.587 * 1.0) + (0.114 * 1.0);
  {
    // skip_dark: every shadow attenuation is finite, i.e. every kt a walk
    // can multiply in lies in [0, 1] (textures: texel / 255) and colours are
    // finite, so a light term with a zero colour factor is exactly +0
    bool ok = true;
    auto in01 = [](const double* v) {
      for (int k = 0; k < 3; ++k)
        if (!(v[k] >= 0.0 && v[k] <= 1.0)) return false;
      return true;
    };
    for (int m = 0; m < d->n_materials; ++m)
      if (d->materials[m].p[RTX_P_KT].tex < 0 && !in01(d->materials[m].p[RTX_P_KT].v)) ok = false;
    for (int v = 0; v < d->n_vmats; ++v)
      if (!in01(d->vmats[v].kt)) ok = false;
    for (int l = 0; l < d->n_lights; ++l)
      for (int k = 0; k < 3; ++k)
        if (!std::isfinite(d->lights[l].color[k])) ok = false;
    S.skip_dark = ok ? 1 : 0;
  }
  st->cam = d->camera;
  st->lights.assign(d->lights, d->lights + d->n_lights);
  // can any hit spawn a reflection or refraction ray?  (per-vertex materials
  // never recurse: their flags are 0, hit_flags)
  st->any_recur = false;
  for (int m = 0; m < d->n_materials; ++m) st->any_recur |= (d->materials[m].flags & RTX_MF_RECUR) != 0;
  if (const char* e = getenv("RTX_CONTEXTS")) st->n_cx = static_cast<unsigned>(std::max(2, std::min(4, atoi(e))));
  if (hipMalloc(&st->cx[0].d_frame, sizeof(FrameParams)) != hipSuccess ||
      hipMalloc(&st->cx[1].d_frame, sizeof(FrameParams)) != hipSuccess ||
      hipMalloc(&st->cx[2].d_frame, sizeof(FrameParams)) != hipSuccess ||
      hipMalloc(&st->cx[3].d_frame, sizeof(FrameParams)) != hipSuccess ||
      hipMalloc(&st->d_work, sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc(&st->d_stats, RTX_STATS_N * sizeof(unsigned long long)) != hipSuccess) {
    g_err = "rtx_scene_create: hipMalloc failed";
    rtx_scene_destroy(st);
    return RTX_ERR_HIP;
  }
  *out = st;
  return RTX_OK;
}

// Context X's last history-sized frame: did its history fall short?  (wait:
// block until the check has run, else only take it if it has.)  A refused
// bucket set (bit 1) drops ray-tree colours and a push that fit neither a
// fork slot nor a two-entry stack (bit 2) drops a ray: either way the frame
// is wrong.  Its history is corrected — bucket pool back to a first render's
// size, full pending stacks — so the frame's later renders are right; the
// frame itself is recorded (rtx_frame_status) and reported.  Returns whether
// that frame was wrong.
static bool collect_check(SceneState* st, FrameCtx& X, bool wait) {
  if (!X.chk_pending) return false;
  if (wait) {
    if (hipEventSynchronize(X.chk_ev) != hipSuccess) return false;
  } else if (hipEventQuery(X.chk_ev) != hipSuccess) {
    return false;
  }
  X.chk_pending = false;
  const unsigned int bits = X.h_bstat[2];
  if (!(bits & 7u)) return false;
  for (uint64_t k : X.chk_keys) {
    if (bits & 3u) st->bucket_hist.erase(k);
    if (bits & 4u) st->full_stack_keys.insert(k);
  }
  if (st->bad_n++ == 0) st->bad_first = X.chk_seq;
  fprintf(stderr,
          "rtx_render: frame %lld (this scene's render %lld) is wrong: %s; its later renders use full-size "
          "buffers (rtx_frame_status reports it)\n",
          static_cast<long long>(X.chk_seq), static_cast<long long>(X.chk_seq),
          (bits & 4u) ? "a two-entry pending stack overflowed" : "the bucket-set pool refused a set");
  return true;
}

// The bounds-check build's record (RTX_CHK): a violation since the last
// read is an error, reported with its site, index and bound.  (Waits for
// the device.)
static rtx_status bounds_check_report() {
#ifdef RTX_BOUNDS_CHECK
  unsigned long long h[3] = {0, 0, 0};
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(h, HIP_SYMBOL(rtx_chk_state), sizeof(h)));
  if (h[0] != 0ull) {
    const unsigned long long z[3] = {0, 0, 0};
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(rtx_chk_state), z, sizeof(z)));
    g_err = "rtx bounds check: " + std::to_string(h[0]) + " out-of-range index(es); the first at site " +
            std::to_string(h[1] >> 48) + ", index " + std::to_string(static_cast<long long>(h[1] & 0xffffffffffffull)) +
            ", bound " + std::to_string(h[2]);
    fprintf(stderr, "%s\n", g_err.c_str());
    return RTX_ERR_INVALID;
  }
#endif
  return RTX_OK;
}

rtx_status rtx_frame_status(void* scene, int64_t* first_bad, int64_t* bad_frames) {
  if (!scene) return RTX_ERR_INVALID;
  SceneState* st = static_cast<SceneState*>(scene);
  HIP_TRY(hipSetDevice(st->device));
  {
    const rtx_status bc = bounds_check_report();
    if (bc != RTX_OK) return bc;
  }
  for (FrameCtx& X : st->cx) collect_check(st, X, true);
  const int64_t fb = st->bad_first, nb = st->bad_n;
  st->bad_first = -1;
  st->bad_n = 0;
  if (first_bad) *first_bad = fb;
  if (bad_frames) *bad_frames = nb;
  if (nb > 0) {
    g_err = "rtx_frame_status: " + std::to_string(nb) + " frame(s) came out wrong, the first is render " +
            std::to_string(fb) + " of this scene";
    return RTX_ERR_FRAME;
  }
  return RTX_OK;
}

rtx_status rtx_overlap_count(void* scene, int64_t* overlapped, int64_t* renders) {
  if (!scene) return RTX_ERR_INVALID;
  SceneState* st = static_cast<SceneState*>(scene);
  if (overlapped) *overlapped = st->n_pipelined;
  if (renders) *renders = st->n_renders;
  st->n_pipelined = 0;
  st->n_renders = 0;
  return RTX_OK;
}

rtx_status rtx_frame_contexts(void* scene, int32_t* n) {
  if (!scene || !n) return RTX_ERR_INVALID;
  *n = static_cast<int32_t>(static_cast<SceneState*>(scene)->last_ncx);
  return RTX_OK;
}

rtx_status rtx_scene_destroy(void* scene) {
  if (!scene) return RTX_OK;
  SceneState* st = static_cast<SceneState*>(scene);
  (void)hipSetDevice(st->device);
  (void)hipDeviceSynchronize();  // (pipelined frames may still be in flight)
  for (FrameCtx& X : st->cx) collect_check(st, X, true);  // (reported on stderr)
  for (void* p : st->allocs) (void)hipFree(p);
  if (st->d_work) (void)hipFree(st->d_work);
  if (st->d_stats) (void)hipFree(st->d_stats);
  if (st->d_picks) (void)hipFree(st->d_picks);
  for (FrameCtx& X : st->cx) {
    if (X.d_frame) (void)hipFree(X.d_frame);
    if (X.d_acnt) (void)hipFree(X.d_acnt);
    if (X.d_bidx) (void)hipFree(X.d_bidx);
    if (X.d_free) (void)hipFree(X.d_free);
    if (X.d_ovf) (void)hipFree(X.d_ovf);
    if (X.d_bstat) (void)hipFree(X.d_bstat);
    if (X.h_bstat) (void)hipHostFree(X.h_bstat);
    if (X.bstat_ev) (void)hipEventDestroy(X.bstat_ev);
    if (X.chk_ev) (void)hipEventDestroy(X.chk_ev);
    for (void* p : X.d_level)
      if (p) (void)hipFree(p);
    if (X.d_offv) (void)hipFree(X.d_offv);
    if (X.d_sbuf) (void)hipFree(X.d_sbuf);
    if (X.d_pbuf) (void)hipFree(X.d_pbuf);
    if (X.d_fbuf) (void)hipFree(X.d_fbuf);
    if (X.d_fmask) (void)hipFree(X.d_fmask);
    if (X.d_wterm) (void)hipFree(X.d_wterm);
    if (X.d_wf) (void)hipFree(X.d_wf);
    if (X.d_lane) (void)hipFree(X.d_lane);
    for (auto e : X.wf_join) (void)hipEventDestroy(e);
    for (auto e : X.wf_check) (void)hipEventDestroy(e);
    if (X.wf_fork) (void)hipEventDestroy(X.wf_fork);
    for (auto q : X.wf_streams) (void)hipStreamDestroy(q);
    if (X.d_counters) (void)hipFree(X.d_counters);
    if (X.h_counters) (void)hipHostFree(X.h_counters);
    if (X.d_scene) (void)hipFree(X.d_scene);
    if (X.free_ev) (void)hipEventDestroy(X.free_ev);
  }
  for (SceneState::Stage& E : st->stage) {
    if (E.ev) (void)hipEventSynchronize(E.ev);
    if (E.h) (void)hipHostFree(E.h);
    if (E.ev) (void)hipEventDestroy(E.ev);
  }
  for (auto e : st->ev_pool) (void)hipEventDestroy(e);
  for (auto e : st->ev_start) (void)hipEventDestroy(e);
  for (auto e : st->ev_stop) (void)hipEventDestroy(e);
  delete st;
  return RTX_OK;
}

// dst <- bytes at src on `stream`, through the next pinned staging entry (the
// source may change or go away as soon as this returns)
static rtx_status stage_copy(SceneState* st, void* dst, const void* src, size_t bytes, hipStream_t stream) {
  SceneState::Stage& E = st->stage[st->next_stage++ % 16u];
  if (E.used) HIP_TRY(hipEventSynchronize(E.ev));
  if (bytes > E.cap) {
    if (E.h) (void)hipHostFree(E.h);
    E.h = nullptr;
    E.cap = 0;
    HIP_TRY(hipHostMalloc(&E.h, bytes));
    E.cap = bytes;
  }
  if (!E.ev) HIP_TRY(hipEventCreateWithFlags(&E.ev, hipEventDisableTiming));
  std::memcpy(E.h, src, bytes);
  HIP_TRY(hipMemcpyAsync(dst, E.h, bytes, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipEventRecord(E.ev, stream));
  E.used = true;
  return RTX_OK;
}

static rtx_status build_frame(const SceneState* st, const RtxRenderParams* p, FrameParams& F,
                              std::vector<double>& offv) {
  std::memset(&F, 0, sizeof(F));
  F.P = *p;
  // adaptaa calls trace(), not tracePixel (RayTracer.cpp:305, :337): no
  // anaglyph eye on adaptive frames
  if (p->aa_mode == RTX_AA_ADAPTIVE) F.P.anaglyph = 0;
  F.cam = st->cam;
  if (p->width <= 0 || p->height <= 0) {
    g_err = "rtx_render: width/height must be positive";
    return RTX_ERR_INVALID;
  }
  if (p->depth > MAX_DEPTH) {
    g_err = "rtx_render: recursion depth above 4096 is not supported by this build";
    return RTX_ERR_CAPACITY;
  }
  if (p->dof && (p->dof_div < 0 || p->dof_div > (1 << 20))) {
    g_err = "rtx_render: DoF samples must be in [0, 2^20]";
    return RTX_ERR_CAPACITY;
  }
  if (p->aa_mode != RTX_AA_NONE && p->aa_samples <= 0) {
    g_err = "rtx_render: AA samples must be positive";
    return RTX_ERR_INVALID;
  }
  const int s = p->aa_mode == RTX_AA_NONE ? 1 : p->aa_samples;
  F.s = s;
  F.spp = s * s;
  if (p->aa_mode != RTX_AA_ADAPTIVE && F.spp > 64) {
    g_err = "rtx_render: regular AA with more than 8x8 samples is not supported";
    return RTX_ERR_CAPACITY;
  }
  if (p->aa_mode == RTX_AA_ADAPTIVE && F.spp > 1024) {
    g_err = "rtx_render: adaptive AA with more than 32x32 samples is not supported";
    return RTX_ERR_CAPACITY;
  }
  if (p->aa_mode == RTX_AA_ADAPTIVE) {
    F.ppw = 1;
  } else {
    F.ppw = 64 / F.spp;
  }
  const int r = isqrt_floor(F.ppw);
  if (r * r == F.ppw) {
    F.bw = r;
    F.bh = r;
  } else {
    F.bw = F.ppw;
    F.bh = 1;
  }
  if (p->tile > 0) {
    if (p->nshards <= 0 || p->shard < 0 || p->shard >= p->nshards) {
      g_err = "rtx_render: bad shard";
      return RTX_ERR_INVALID;
    }
    F.tw = p->tile;
    F.th = p->tile;
    F.tiles_x = (p->width + p->tile - 1) / p->tile;
    F.tiles_y = (p->height + p->tile - 1) / p->tile;
    const int nt = F.tiles_x * F.tiles_y;
    F.n_owned = nt > p->shard ? (nt - p->shard + p->nshards - 1) / p->nshards : 0;
  } else {
    F.tw = p->width;
    F.th = p->height;
    F.tiles_x = 1;
    F.tiles_y = 1;
    F.n_owned = 1;
  }
  F.bx_per_tile = (F.tw + F.bw - 1) / F.bw;
  F.items_per_tile = F.bx_per_tile * ((F.th + F.bh - 1) / F.bh);
  F.n_items = static_cast<int64_t>(F.items_per_tile) * F.n_owned;
  F.n_samples = F.n_items * F.ppw * F.spp;
  F.ncam = p->dof ? p->dof_div + 1 : 1;
  F.cam_split = 0;
  // DoF eye offsets: (cos(a) * V + sin(a) * U) * sz (RayTracer.cpp:62-67)
  if (p->dof) {
    const double PI = 3.1415926535897932384626433832795028841971;
    const double sz = p->dof_apsz / 2;
    const int divs = p->dof_div;
    const double baseAngle = PI / divs;
    const dvec3 V = ld3(st->cam.v), U = ld3(st->cam.u);
    offv.assign(size_t(divs) * 3, 0.0);
    for (int k = 0; k < divs; k++) {
      double offsetAngle = PI / 2;
      offsetAngle = offsetAngle / divs + (k - 1) * baseAngle;
      dvec3 o = (std::cos(offsetAngle) * V + std::sin(offsetAngle) * U) * sz;
      offv[k * 3 + 0] = o.x;
      offv[k * 3 + 1] = o.y;
      offv[k * 3 + 2] = o.z;
    }
  }
  return RTX_OK;
}

rtx_status rtx_shard_pixels(const RtxRenderParams* p, int64_t* npix) {
  if (!p || !npix) return RTX_ERR_INVALID;
  if (p->tile > 0 && p->packed) {
    const int tx = (p->width + p->tile - 1) / p->tile, ty = (p->height + p->tile - 1) / p->tile;
    const int nt = tx * ty;
    const int owned = nt > p->shard ? (nt - p->shard + p->nshards - 1) / p->nshards : 0;
    *npix = static_cast<int64_t>(owned) * p->tile * p->tile;
  } else {
    *npix = static_cast<int64_t>(p->width) * p->height;
  }
  return RTX_OK;
}

// A whole frame's identity for the fork-depth rule: the render parameters
// without the tile deal (tile, shard, nshards, packed), FNV-1a.
static uint64_t whole_frame_key(const RtxRenderParams& p) {
  RtxRenderParams q;
  std::memset(&q, 0, sizeof(q));
  q.width = p.width;
  q.height = p.height;
  q.depth = p.depth;
  q.aa_mode = p.aa_mode;
  q.aa_samples = p.aa_samples;
  q.dof = p.dof;
  q.dof_div = p.dof_div;
  q.anaglyph = p.anaglyph;
  q.ss_res = p.ss_res;
  q.overlapping = p.overlapping;
  q.aa_thresh = p.aa_thresh;
  q.aterm_thresh = p.aterm_thresh;
  q.dof_fd = p.dof_fd;
  q.dof_apsz = p.dof_apsz;
  uint64_t k = 1469598103934665603ull;
  const unsigned char* c = reinterpret_cast<const unsigned char*>(&q);
  for (size_t i = 0; i < sizeof(q); ++i) k = (k ^ c[i]) * 1099511628211ull;
  return k;
}

// One render of frame `seq` (rtx_render below).  *redo 1: this synchronous
// render found its history-sized buffers short (collect_check) — the image
// is wrong and the caller renders again, now with full-size buffers.
static rtx_status render_once(SceneState* st, const RtxRenderParams* params, uint8_t* rgb8, double* rgb_f64,
                              RtxHitRecord* hits, int device_ptrs, void* stream_v, RtxStats* stats, int64_t seq,
                              bool retry, int* redo) {
  HIP_TRY(hipSetDevice(st->device));
  hipStream_t stream = static_cast<hipStream_t>(stream_v);
  // Frame context (DESIGN.md "Frame contexts"): a render into device buffers
  // with no hit records, counters or adaptive levels alternates between the
  // scene's two contexts and runs on the context's own streams — after the
  // context's previous frame only, so it can overlap the frame before it —
  // and joins the caller's stream for its final reduce.  Every other render
  // uses context 0 on the caller's stream, after whatever was queued there
  // (RTX_PIPELINE=0: always that).
  FrameParams F;
  std::vector<double> offv;
  rtx_status rc = build_frame(st, params, F, offv);
  if (rc != RTX_OK) return rc;
  // Which frames overlap: at most RTX_PIPELINE_SAMPLES work units (samples x
  // DoF camera rays; default 20 M: the shards of a multi-GPU frame — a 4-way
  // shard gains 12 %, 8.8 vs 10.0 ms, an 8-way one 20 %, profiles/r04k_*).
  // A whole frame renders on one context, with one set of frame buffers: its
  // last iterations are a small share of it (the headline frame back to back
  // 32.5 vs 33.0 ms with two ~31-GiB sets, r04pipe1_*), not worth a second
  // set.  RTX_PIPELINE=0: never.
  const char* mk_env0 = getenv("RTX_MEGAKERNEL");
  const char* pipe_env = getenv("RTX_PIPELINE");
  int64_t pipe_max = 20000000;
  if (const char* e = getenv("RTX_PIPELINE_SAMPLES")) pipe_max = atoll(e);
  int64_t npix0 = 0;
  rtx_shard_pixels(params, &npix0);
  const int64_t units0 = npix0 * int64_t(F.spp) * int64_t(F.ncam);
  const bool pipelined = !(pipe_env && atoi(pipe_env) == 0) && device_ptrs && !hits && !stats &&
                         params->aa_mode != RTX_AA_ADAPTIVE && !(mk_env0 && atoi(mk_env0) != 0) &&
                         units0 <= pipe_max;
  const unsigned int ncx = units0 <= 10000000 ? st->n_cx : std::min(st->n_cx, 2u);
  FrameCtx* X = pipelined ? &st->cx[(st->next_cx++) % ncx] : &st->cx[0];
  st->last_ncx = pipelined ? ncx : 1u;
  if (!retry) {
    ++st->n_renders;
    if (pipelined) ++st->n_pipelined;
  }
  // the frame checks of earlier renders: this context's (its frame is long
  // done: the check is read before its buffers are reused), the other's if
  // it has run
  collect_check(st, *X, true);
  for (FrameCtx& C : st->cx)
    if (&C != X) collect_check(st, C, false);
  std::vector<uint64_t> chk_keys;  // this frame's history-sized runs (run_wavefront)
  if (!X->free_ev) HIP_TRY(hipEventCreateWithFlags(&X->free_ev, hipEventDisableTiming));
  if (X->wf_streams.empty()) {
    hipStream_t s0;
    HIP_TRY(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    X->wf_streams.push_back(s0);
    hipEvent_t ev;
    HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    X->wf_join.push_back(ev);
    HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    X->wf_check.push_back(ev);
  }
  // a buffer of this context may still be read by its previous frame (a
  // pipelined render returns before its frame ends): wait for that frame
  // before giving one back
  auto ctx_free = [&](void* p) {
    if (X->used) (void)hipEventSynchronize(X->free_ev);
    (void)hipFree(p);
  };
  hipStream_t ws = stream;  // the frame's work stream (slot group 0)
  if (pipelined) {
    ws = X->wf_streams[0];
    if (X->used) HIP_TRY(hipStreamWaitEvent(ws, X->free_ev, 0));
  } else {
    for (FrameCtx& C : st->cx)  // (a pipelined frame may still run on the other context)
      if (C.used) HIP_TRY(hipStreamWaitEvent(stream, C.free_ev, 0));
  }
  if (!offv.empty()) {
    const size_t need = offv.size() * sizeof(double);
    if (need > X->offv_bytes) {
      if (X->d_offv) ctx_free(X->d_offv);
      X->d_offv = nullptr;
      X->offv_bytes = 0;
      HIP_TRY(hipMalloc(&X->d_offv, need));
      X->offv_bytes = need;
    }
    if ((rc = stage_copy(st, X->d_offv, offv.data(), need, ws)) != RTX_OK) return rc;
    F.offv = X->d_offv;
  }
  // area-light pick tables depend on ss_res
  st->S_launch = st->S;
  DevScene& S = st->S_launch;
  S.ss_res = params->ss_res;
  bool need_picks = false;
  for (const auto& L : st->lights) need_picks |= L.type >= RTX_LIGHT_AREA_RECT;
  if (need_picks && st->picks_res != params->ss_res) {
    std::vector<double> pk = make_picks(st->lights, params->ss_res);
    if (st->d_picks) (void)hipFree(st->d_picks);
    st->d_picks = nullptr;
    if (!pk.empty()) {
      HIP_TRY(hipMalloc(&st->d_picks, pk.size() * sizeof(double)));
      HIP_TRY(hipMemcpy(st->d_picks, pk.data(), pk.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    st->picks_res = params->ss_res;
  }
  S.picks = st->d_picks;

  int64_t npix = 0;
  rtx_shard_pixels(params, &npix);
  uint8_t* d_rgb8 = rgb8;
  double* d_rgbf = rgb_f64;
  RtxHitRecord* d_hits = hits;
  // host-mode staging buffers: freed on every exit path (a failed call
  // must not leak them)
  struct TmpBufs {
    std::vector<void*> v;
    void push_back(void* p) { v.push_back(p); }
    ~TmpBufs() {
      for (void* p : v) (void)hipFree(p);
    }
  } tmp;
  if (!device_ptrs) {
    if (rgb8) { HIP_TRY(hipMalloc(&d_rgb8, npix * 3)); tmp.push_back(d_rgb8); HIP_TRY(hipMemsetAsync(d_rgb8, 0, npix * 3, ws)); }
    if (rgb_f64) { HIP_TRY(hipMalloc(&d_rgbf, npix * 3 * sizeof(double))); tmp.push_back(d_rgbf); HIP_TRY(hipMemsetAsync(d_rgbf, 0, npix * 3 * sizeof(double), ws)); }
    if (hits) {
      HIP_TRY(hipMalloc(&d_hits, npix * F.spp * sizeof(RtxHitRecord)));
      tmp.push_back(d_hits);
      HIP_TRY(hipMemsetAsync(d_hits, 0xff, npix * F.spp * sizeof(RtxHitRecord), ws));
    }
  }
  const bool adaptive = params->aa_mode == RTX_AA_ADAPTIVE;
  const bool media = params->overlapping != 0;  // -O o: the kernels with the discoverMat states
  // wavefront path by default (adaptive AA too: its levels run as work
  // units, adapt_*_kernel); RTX_MEGAKERNEL=1 uses the persistent megakernel
  // (kernels)
  const char* mk_env = getenv("RTX_MEGAKERNEL");
  const bool megakernel = mk_env && atoi(mk_env) != 0;
  // DoF on the wavefront path: each of a sample's divs + 1 camera rays is a
  // work unit of its own (17x the parallel units, paths 17x shorter)
  if (!megakernel && params->dof && !F.P.anaglyph) {
    F.cam_split = 1;
    F.n_samples *= F.ncam;
  }
  F.chk_samples = static_cast<int64_t>(npix) * F.spp;
  if (F.cam_split && hits) HIP_TRY(hipMemsetAsync(d_hits, 0xff, npix * F.spp * sizeof(RtxHitRecord), ws));
  if (!(adaptive && megakernel)) {
    const size_t need = size_t(npix) * F.spp * (F.cam_split ? F.ncam : 1) * 3 * sizeof(double);
    if (need > X->sbuf_bytes) {
      if (X->d_sbuf) ctx_free(X->d_sbuf);
      X->d_sbuf = nullptr;
      X->sbuf_bytes = 0;
      HIP_TRY(hipMalloc(&X->d_sbuf, need));
      X->sbuf_bytes = need;
    }
  }
  HIP_TRY(hipMemsetAsync(st->d_work, 0, sizeof(unsigned long long), ws));
  // device copy of the scene record: functions called out of line read it
  // through this pointer (a kernel-argument copy has no address)
  if (!X->d_scene) HIP_TRY(hipMalloc(&X->d_scene, sizeof(DevScene)));
  if ((rc = stage_copy(st, X->d_scene, &st->S_launch, sizeof(DevScene), ws)) != RTX_OK) return rc;
  if (stats) HIP_TRY(hipMemsetAsync(st->d_stats, 0, RTX_STATS_N * sizeof(unsigned long long), ws));
  const int pend_cap = (params->depth > 0 ? params->depth : 0) + 2;
  auto get_event = [&](hipEvent_t* e) -> rtx_status {
    if (!st->ev_pool.empty()) {
      *e = st->ev_pool.back();
      st->ev_pool.pop_back();
      return RTX_OK;
    }
    HIP_TRY(hipEventCreate(e));
    return RTX_OK;
  };
  static const bool dbg_alloc = getenv("RTX_DEBUG_ALLOC") && atoi(getenv("RTX_DEBUG_ALLOC")) != 0;
  auto ensure = [&](void** ptr, size_t* have, size_t need) -> rtx_status {
    if (need > *have) {
      if (dbg_alloc) fprintf(stderr, "rtx alloc ctx %d: %zu -> %zu B (call %d)\n", int(X - st->cx), *have, need, X->wf_call);
      if (*ptr) ctx_free(*ptr);
      *ptr = nullptr;
      *have = 0;
      HIP_TRY(hipMalloc(ptr, need));
      *have = need;
    }
    return RTX_OK;
  };
  double* sb = adaptive && megakernel ? nullptr : X->d_sbuf;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> frame_events;
  X->wf_call = 0;
  X->bstat_clear = false;

  if (megakernel) {
    const int cslots = adaptive ? (F.spp > 64 ? F.spp : 64) : 0;
    const int fslots = adaptive ? 16 * 8 : 0;
    const size_t lds_per_wave =
        size_t(cslots * 3 + fslots) * sizeof(double) + size_t(st->stack_cap) * 64 * sizeof(int);
    const size_t lds = lds_per_wave * WAVES_PER_WG;
    if (lds > 160 * 1024) {
      g_err = "rtx_render: LDS budget exceeded (BVH too deep or too many AA samples)";
      return RTX_ERR_CAPACITY;
    }
    // persistent grid: as many resident workgroups as the occupancy allows
    const void* kfn = nullptr;
    dispatch2(stats, adaptive, [&](auto st_, auto ad_) {
      kfn = media ? reinterpret_cast<const void*>(render_kernel<decltype(st_)::value, decltype(ad_)::value, true>)
                  : reinterpret_cast<const void*>(render_kernel<decltype(st_)::value, decltype(ad_)::value, false>);
    });
    int per_cu = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, WG, lds));
    if (per_cu < 1) per_cu = 1;
    int64_t grid = static_cast<int64_t>(st->n_cu) * per_cu;
    const int64_t waves_needed = adaptive ? F.n_items : (F.n_samples + 63) / 64;
    const int64_t grid_needed = (waves_needed + WAVES_PER_WG - 1) / WAVES_PER_WG;
    if (grid > grid_needed) grid = grid_needed;
    if (grid < 1) grid = 1;
    {
      // queue chunk: up to QCHUNK samples per atomic, but small frames must
      // still spread over every wave
      const int64_t waves = grid * WAVES_PER_WG;
      int64_t c = F.n_samples / (waves * 4);
      c = (c / 64) * 64;
      if (c < 64) c = 64;
      if (c > QCHUNK) c = QCHUNK;
      F.qchunk = static_cast<int>(c);
    }
    if ((rc = stage_copy(st, X->d_frame, &F, sizeof(FrameParams), ws)) != RTX_OK) return rc;
    if ((rc = ensure(reinterpret_cast<void**>(&X->d_pbuf), &X->pbuf_bytes,
                     size_t(grid) * WG * pend_cap * 13 * sizeof(double))) != RTX_OK)
      return rc;
    if ((rc = ensure(&X->d_lane, &X->lane_bytes, lane_mem_bytes(size_t(grid) * WG))) != RTX_OK) return rc;
    const LaneMem lm = lane_mem_at(X->d_lane, size_t(grid) * WG);
    hipEvent_t e0, e1;
    if ((rc = get_event(&e0)) != RTX_OK || (rc = get_event(&e1)) != RTX_OK) return rc;
    HIP_TRY(hipEventRecord(e0, ws));
    dispatch2(stats, adaptive, [&](auto st_, auto ad_) {
      constexpr bool ST_ = decltype(st_)::value, AD_ = decltype(ad_)::value;
      if (media)
        RTX_LAUNCH((render_kernel<ST_, AD_, true>), dim3(grid), dim3(WG), lds, ws, st->S_launch,
                           X->d_scene, X->d_frame, st->d_work, sb, d_hits, d_rgb8, d_rgbf, st->d_stats, st->stack_cap,
                           X->d_pbuf, pend_cap, lm);
      else
        RTX_LAUNCH((render_kernel<ST_, AD_, false>), dim3(grid), dim3(WG), lds, ws, st->S_launch,
                           X->d_scene, X->d_frame, st->d_work, sb, d_hits, d_rgb8, d_rgbf, st->d_stats, st->stack_cap,
                           X->d_pbuf, pend_cap, lm);
    });
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(e1, ws));
    frame_events.push_back({e0, e1});
  }
  // One run of the wavefront machine over F's work units (F.n_samples), whose
  // samples land in sample ids [0, nout * spp) of the sample buffer: the
  // whole frame, or one chunk of a deeper adaptive level (level0 false: the
  // hit records are not reset, the buckets are sized for the chunk).
  auto run_wavefront = [&](FrameParams& F, int64_t nout, bool level0) -> rtx_status {
    // ---------------- wavefront path
    // NSLOT path slots split into G groups, each iterating advance -> trace
    // (closest) -> trace (next) on its own ws, so one group's launch
    // tails overlap the other groups' work.
    int64_t nslot64 = static_cast<int64_t>(st->n_cu) * 49152;  // 12.6 M on 256 CUs (tools/gpu_exp*.sh sweeps)
    const char* ns_env = getenv("RTX_SLOTS");
    if (ns_env && atoll(ns_env) > 0) nslot64 = atoll(ns_env);
    int G = 3;
    const char* g_env = getenv("RTX_GROUPS");
    if (g_env && atoi(g_env) > 0) G = atoi(g_env);
    if (G > 16) G = 16;
    // Ray-tree buckets + forking (DESIGN.md "Ray-tree forking"; no DoF /
    // anaglyph): every frame of this kind accumulates per-node buckets; when
    // the frame has fewer samples than 3/4 of the slots, the spare slots run
    // forked reflection / refraction sub-trees, so a sample's critical path
    // is its deepest sub-tree instead of its whole tree (RTX_FORK=0: no
    // buckets, no forks; RTX_FORK_DEPTH: heap depth of the deepest node, 1..4)
    const char* fork_env = getenv("RTX_FORK");
    int fork_depth = 4;  // headline frame: 53.2 ms at 4 vs 54.2 at 3 (fused walks)
    const char* fd_env = getenv("RTX_FORK_DEPTH");
    if (fd_env && atoi(fd_env) > 0) fork_depth = std::min(4, atoi(fd_env));
    // (DoF: with the camera-ray split each camera ray owns its buckets)
    // (a scene whose materials never reflect or refract has no ray trees to
    // fork: the C5 dragon, whose 8 x 8 adaptive shards took 48 GB of
    // buckets for nothing)
    bool fork_ok = !(fork_env && atoi(fork_env) == 0) && !F.P.anaglyph && (!params->dof || F.cam_split) &&
                   st->any_recur && params->depth > 0;
    const size_t nunit_out = size_t(nout) * F.spp * (F.cam_split ? F.ncam : 1);  // bucket owners
    // fused shadow walks (rtx_fused.h): every light a point or directional
    // light, no overlapping media, no adaptive termination (RTX_FUSE=0: the
    // sequential machine)
    const char* fuse_env = getenv("RTX_FUSE");
    // (area and spot lights too: a walk per pick, rtx_fused.h "Area lights";
    // their term units and records per slot counted here)
    bool fuse = !(fuse_env && atoi(fuse_env) == 0) && !media && !(params->aterm_thresh > 0.0) &&
                st->lights.size() <= 8;
    int w_units = 0, w_recs = 0, w_amask = 0;
    {
      const int res = std::max(0, params->ss_res);
      for (size_t l = 0; l < st->lights.size() && l < 8; ++l) {
        F.lunit[l] = w_units;
        F.lrec[l] = w_recs;
        if (st->lights[l].type >= RTX_LIGHT_AREA_RECT) {
          w_units += 2 + res;
          w_recs += res;
          w_amask |= 1 << l;
        } else {
          w_units += 1;
          w_recs += 1;
        }
      }
      // (RTX_FUSE_AREA=0: area / spot light frames on the sequential machine)
      const char* fa_env = getenv("RTX_FUSE_AREA");
      if (w_amask && ((fa_env && atoi(fa_env) == 0) || w_recs > 64)) fuse = false;
    }
    F.nrec = fuse ? w_recs : 0;
    F.area_mask = fuse ? w_amask : 0;
    const size_t nl = fuse ? st->lights.size() : 0;
    const size_t n_units = fuse ? size_t(w_units) : 0;
    // pending-stack entries: a ray at entry i has depth <= P.depth - i (the
    // camera ray is entry 0, a forked sub-tree's root entry 0 with less; a
    // hit overwrites its own entry with one child and pushes the other), and
    // only rays of depth > 0 push, so the fused machine never writes past
    // entry P.depth - 1: P.depth entries (the sequential machine keeps
    // depth + 2 for its media walks)
    const int pcap = fuse ? std::max(1, params->depth) : pend_cap;
    // query records: closest (slot, 9 doubles, 2 ints); next: one per slot,
    // or one per light and slot with fused walks (slot, QF_D doubles, 3 ints)
    // (fused closest records hold the ray only: 6 doubles, no ints)
    const size_t qc_d = fuse ? 6 : QL_D, qc_i = fuse ? 0 : 2;
    const size_t rec_c = sizeof(int) + qc_d * sizeof(double) + qc_i * sizeof(int);
    const size_t rec_n = fuse ? sizeof(int) + QF_D * sizeof(double) + QF_I * sizeof(int) : rec_c;
    const size_t nrec_n = fuse ? std::max<size_t>(1, size_t(w_recs)) : 1;
    const size_t per_slot = lane_mem_bytes(1, fuse) - 512 + size_t(pcap) * 13 * sizeof(double) + rec_c +
                            nrec_n * rec_n + 2 * sizeof(int) + n_units * 3 * sizeof(double);
    // the bucket-set pool: as many sets as this frame took on its last
    // render (deterministic: one per unit whose root has a node child), the
    // full count (a set per unit) the first time.  Whether the frame has
    // buckets at all was decided above on the full count, so the image never
    // depends on the pool.
    size_t bcap = nunit_out;
    bool spares_enough = false;  // the spares cover every fork request (no free list needed)
    // spare slots per sample slot at most, in percent (RTX_SPARE): 50 on
    // whole frames, 100 on frames of at most 20 M units (the shards of a
    // multi-GPU frame, whose buffers are small: R1's 8-way shard 38.3 ->
    // 34.0 ms, the headline's and C4's unchanged, profiles/r04sp_*)
    int64_t spare_pct = F.n_samples <= 20000000 ? 100 : 50;
    if (const char* e = getenv("RTX_SPARE")) spare_pct = std::max<int64_t>(1, std::min<int64_t>(400, atoll(e)));
    // fork slots per group the frame needs: its largest per-group count of
    // fork requests on its first render (every node child asks for a fork
    // slot whether or not it gets one, so the count does not depend on the
    // spare slots; with at least that many spares every request is granted
    // as on the first render).  -1: unknown, half a slot per sample.
    int64_t fspare = -1;
    bool forks_outgrow = false;  // (the history shows more fork requests than spares: depth 3, the lower cap)
    // the frame's history key: its parameters, this run of the render and the
    // bucket layout (fork depth)
    auto frame_key = [&](int depth) {
      uint64_t k = 1469598103934665603ull;
      auto mix = [&](const void* p, size_t n) {
        const unsigned char* c = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < n; ++i) k = (k ^ c[i]) * 1099511628211ull;
      };
      mix(&F.P, sizeof(F.P));
      const int64_t npos = (int64_t(1) << (depth + 1)) - 2;
      const int64_t ks[6] = {F.n_samples, nout, level0 ? 1 : 0, X->wf_call, npos, int64_t(nunit_out)};
      mix(ks, sizeof(ks));
      return k;
    };
    uint64_t bkey = frame_key(fork_depth);
    {
      for (FrameCtx& C : st->cx)  // the first-time frames' counts (either context's; long done by now)
        if (C.bstat_pending) {
          HIP_TRY(hipEventSynchronize(C.bstat_ev));
          if ((C.h_bstat[1] & 3u) == 0u) {  // (bit 2, a two-entry stack's overflow: the frame check's)
            int64_t fm = C.bstat_groups > 0 ? 0 : -1;
            for (int g = 0; g < C.bstat_groups; ++g) fm = std::max<int64_t>(fm, C.h_bstat[4 + g]);
            st->bucket_hist[C.bstat_key] = {C.h_bstat[0], fm};
          } else {
            fprintf(stderr, "rtx_render: bucket pool refused a set (%u taken); frame pool reset\n", C.h_bstat[0]);
            st->bucket_hist.erase(C.bstat_key);
          }
          C.bstat_pending = false;
        }
      // A frame whose ray trees fork at many of their nodes (R1, the glass
      // frame: fork requests at nearly every hit) forks down to heap depth 3:
      // 14 bucket positions a set instead of 30, so the lower memory cap below
      // keeps more slots in flight — R1 at 252-254 ms in 38.7 GB against 255
      // ms in 55.9 GB at depth 4 (profiles/r05q_ab_r1_memory.txt).  The depth
      // moves the line between bucket sums and the running sum (f64 images
      // differ in the last bit), so every render of a frame — and every shard
      // of it on a multi-GPU job — uses the same one: depth_rule, decided once
      // per whole frame by depth_probe (rtx_render) from a fixed subset of the
      // whole frame, the same pixels whichever shard is being rendered.
      if (fork_ok && fork_depth == 4 && !fd_env && !adaptive && !st->probe_mode) {
        const auto dr = st->depth_rule.find(whole_frame_key(*params));
        if (dr != st->depth_rule.end() && dr->second == 3) {
          fork_depth = 3;
          bkey = frame_key(fork_depth);
          forks_outgrow = true;
          if (const char* e = getenv("RTX_DEBUG"))
            if (atoi(e) != 0) fprintf(stderr, "rtx: forks outgrow the spares: fork depth 3, 34-GiB cap\n");
        }
      }
      const auto it = st->bucket_hist.find(bkey);
      if (it != st->bucket_hist.end()) {
        bcap = std::min<size_t>(nunit_out, size_t(it->second.sets) + 64);
        // (test knob: a history that falls short, so the frame check and the
        // re-render can be exercised — tests/test_gpu_parity.py)
        if (const char* e = getenv("RTX_TEST_SHORT_POOL"))
          if (atoi(e) != 0) bcap = std::max<size_t>(1, size_t(it->second.sets) / 2);
        // (never more than the half slot per sample of the default pool)
        if (it->second.forks >= 0) {
          fspare = std::min<int64_t>(it->second.forks, (F.n_samples + G - 1) / G * spare_pct / 100);
          spares_enough = fspare == it->second.forks;
        }
      }
    }
    {
      // memory budget: what the device has free plus the frame buffers this
      // scene already holds (they are reused or replaced), less a reserve
      size_t freeb = 0, totb = 0;
      HIP_TRY(hipMemGetInfo(&freeb, &totb));
      const size_t held =
          X->lane_bytes + X->pbuf_bytes + X->wf_bytes + X->fbuf_bytes + X->fmask_bytes + X->wterm_bytes;
      const size_t sbuf_need = size_t(npix) * F.spp * 3 * sizeof(double);
      const size_t avail = freeb + held > sbuf_need ? (freeb + held - sbuf_need) / 10 * 8 : 0;
      const size_t npos = (size_t(1) << (fork_depth + 1)) - 2;
      const size_t bucket_need = fork_ok ? nunit_out * (npos * 3 * sizeof(double) + sizeof(unsigned)) : 0;
      if (bucket_need > avail / 2) fork_ok = false;  // buckets would crowd out the slots: plain accumulation
      // what the pooled sets take (bcap sets, a mask and a set index per unit)
      const size_t pool_need = fork_ok ? bcap * npos * 3 * sizeof(double) + nunit_out * 2 * sizeof(unsigned) : 0;
      // (unsigned: with less free memory than the pool needs the slots get
      // nothing — the pool is then floored below — never a wrapped-around
      // 96 GiB)
      size_t slot_budget = avail > pool_need ? std::min<size_t>(size_t(96) << 30, avail - pool_need) : 0;
      // Frame-memory cap (RTX_MEM_GB GiB, default 48, 34 for frames whose
      // forks outgrow their spares): the slot pool
      // gets what the cap leaves after the sample sums and the buckets.  The
      // buckets keep their size — whether a frame has buckets must not
      // depend on the cap, the image would change with it — so the cap only
      // sets how many samples are in flight at once (the rest are claimed
      // as slots free up, kdone).
      // 48 GiB: the headline, C3, C4, C5 and the shards stay under it (the
      // headline's buckets alone are 24 GB: at 34 GiB its pool falls below a
      // slot per sample, 34.4 vs 32.0 ms).  34 GiB where the forks outgrow
      // the spares: the knee of R1, the recursion-heavy glass frame, with its
      // buckets at fork depth 3 (above) — 36 / 38 / 42 / 50 GiB of frame
      // buffers at caps of 34 / 36 / 40 / 48 GiB, 254 / 251 / 252 / 251 ms,
      // 34 GiB at a cap of 32: 260 ms (profiles/r05q_ab_r1_memory.txt; at
      // depth 4: 71 GB uncapped, 255 ms, 44 GB at a 40-GiB cap, 270 ms,
      // r05a_r1_mem_knee.jsonl).  RTX_MEM_GB=0: no cap.
      size_t cap_gb = forks_outgrow ? 34 : 48;
      if (const char* e = getenv("RTX_MEM_GB")) cap_gb = static_cast<size_t>(atoll(e));
      if (cap_gb > 0) {
        const size_t cap_b = cap_gb << 30, fixed = sbuf_need + pool_need;
        const size_t min_slots = size_t(G) * 16 * WG;  // never below 16 workgroups per group
        slot_budget = std::min(slot_budget, std::max(cap_b > fixed ? cap_b - fixed : 0, min_slots * per_slot));
      }
      const int64_t cap = static_cast<int64_t>(slot_budget / per_slot);
      if (fork_ok && !(ns_env && atoll(ns_env) > 0)) {
        // one slot per sample plus half as many fork slots (headline frame:
        // 50 M slots, 89 -> 84 ms; 2-way shard 58 -> 50 ms)
        const int64_t spare_all = fspare >= 0 ? int64_t(G) * (fspare + WG) : F.n_samples * spare_pct / 100;
        const int64_t want = std::min<int64_t>(cap, F.n_samples + spare_all + int64_t(G) * 2 * WG);
        if (want > nslot64) nslot64 = want;
      }
      if (nslot64 > cap && !(ns_env && atoll(ns_env) > 0)) nslot64 = std::max<int64_t>(cap, int64_t(G) * 4 * WG);
    }
    // spare slots for forked sub-trees: a third of the pool when it cannot
    // give every sample a slot of its own plus half as many spares
    const bool fork = fork_ok && nslot64 >= int64_t(G) * 8 * WG;
    int64_t gsamp = (F.n_samples + G - 1) / G;  // sample slots per group
    // (a pool sized from the fork history holds every sample and the spares
    // its forks need: no third set aside)
    const bool spare_fit = fspare >= 0 && nslot64 >= F.n_samples + int64_t(G) * (fspare + WG);
    const int64_t gcap = fork && F.n_samples * 4 > nslot64 * 3 && !spare_fit ? nslot64 * 2 / 3 : nslot64;
    if (gsamp > (gcap + G - 1) / G) gsamp = (gcap + G - 1) / G;
    gsamp = (gsamp + 63) / 64 * 64;  // whole 64-unit runs (slot_unit)
    int64_t gspare = 0;
    if (fork) gspare = std::min<int64_t>(gsamp * spare_pct / 100 + WG, nslot64 / G - gsamp);
    const int64_t per = (gsamp + gspare + WG - 1) / WG;  // workgroups per group
    const int64_t gslots = per * WG;
    if (!fork) gsamp = gslots;
    nslot64 = gslots * G;
    // What the kernels assume of this geometry, checked before anything is
    // launched: slot ids, sample slots and bucket owners are int32 (LaneRef,
    // slot_unit, claim_sample's sample_slot / bunit), every group's sample
    // slots lie inside its slots (fork slots follow them), and the output
    // slots' samples fit the sample buffer.
    if (nslot64 > INT32_MAX || gsamp * G > INT32_MAX || gsamp > gslots || gslots < WG ||
        int64_t(nout) * F.spp * (F.cam_split ? F.ncam : 1) > INT32_MAX || F.n_samples > INT64_C(1) << 40) {
      g_err = "rtx_render: frame too large for this build (slot, sample or bucket index past int32)";
      return RTX_ERR_CAPACITY;
    }
    F.wf_nslot = static_cast<int>(gsamp * G);
    F.wf_gs = static_cast<int>(gslots);
    F.wf_gsamp = static_cast<int>(gsamp);
    F.wf_groups = G;
    F.fork_on = fork_ok ? 1 : 0;
    F.fork_npos = fork_ok ? (1 << (fork_depth + 1)) - 2 : 0;
    F.fbuf = nullptr;
    F.fmask = nullptr;
    F.bidx = nullptr;
    F.bcnt = F.bover = nullptr;
    F.bcap = 0;
    if (fork_ok) {
      const size_t nsamp_out = size_t(nout) * F.spp;
      const size_t fbuf_need = std::max<size_t>(1, bcap) * F.fork_npos * 3 * sizeof(double);
      // a smaller pool than the first render's: give it back (not on adaptive
      // frames, whose level chunks take smaller pools than their first pass)
      if (!adaptive && X->fbuf_bytes > 2 * fbuf_need + (size_t(64) << 20)) {
        ctx_free(X->d_fbuf);
        X->d_fbuf = nullptr;
        X->fbuf_bytes = 0;
      }
      if ((rc = ensure(reinterpret_cast<void**>(&X->d_fbuf), &X->fbuf_bytes, fbuf_need)) != RTX_OK) return rc;
      if ((rc = ensure(reinterpret_cast<void**>(&X->d_fmask), &X->fmask_bytes, nunit_out * sizeof(unsigned int))) !=
          RTX_OK)
        return rc;
      if ((rc = ensure(reinterpret_cast<void**>(&X->d_bidx), &X->bidx_bytes, nunit_out * sizeof(int))) != RTX_OK)
        return rc;
      if (!X->d_bstat) HIP_TRY(hipMalloc(&X->d_bstat, 4 * sizeof(unsigned int)));
      if (!X->h_bstat) HIP_TRY(hipHostMalloc(&X->h_bstat, (4 + 16) * sizeof(unsigned int)));
      if (!X->bstat_ev) HIP_TRY(hipEventCreateWithFlags(&X->bstat_ev, hipEventDisableTiming));
      // ([taken] per run; [bover] once per render, by its first forking run
      // whichever run that is: the frame check reads it after the frame's
      // last run)
      HIP_TRY(hipMemsetAsync(X->d_bstat, 0, (X->bstat_clear ? 1 : 4) * sizeof(unsigned int), ws));
      X->bstat_clear = true;
      F.fbuf = X->d_fbuf;
      F.fmask = X->d_fmask;
      F.bidx = X->d_bidx;
      F.bcnt = X->d_bstat;
      F.bover = X->d_bstat + 1;
      F.bcap = static_cast<int>(std::min<size_t>(bcap, size_t(INT32_MAX)));
      // fmask[sample] is cleared when the sample is claimed (claim_sample)
      if (hits && level0) HIP_TRY(hipMemsetAsync(d_hits, 0xff, nsamp_out * sizeof(RtxHitRecord), ws));
    }
    const size_t ns = static_cast<size_t>(nslot64);
    const size_t gs = static_cast<size_t>(gslots);
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    // per group: the closest and the next query list, then two live-slot
    // lists (ping-pong)
    const size_t capn = gs * nrec_n;
    const size_t bytes_qc = al(gs * sizeof(int)) + al(gs * qc_d * sizeof(double)) + al(gs * qc_i * sizeof(int));
    const size_t nd = fuse ? QF_D : QL_D, ni = fuse ? QF_I : 2;
    const size_t bytes_qn = al(capn * sizeof(int)) + al(capn * nd * sizeof(double)) + al(capn * ni * sizeof(int));
    // tail switch: a group whose live slots fall to this many finishes in
    // tail_kernel (RTX_TAIL; fused walks, headline frame: 64.0 / 62.4 / 62.0
    // ms at 200k / 400k / 1M; sequential machine: 92.6 / 91.0 / 99.5 ms at
    // 65k / 200k / 400k)
    int64_t tail_slots = 1000000;
    // (a capped pool, fewer slots than units: the same share of a group's
    // slots as 1 M is of the uncapped headline frame's 16.6 M)
    if (int64_t(F.wf_nslot) < F.n_samples) tail_slots = std::min<int64_t>(tail_slots, gslots * 6 / 100);
    const char* tail_env = getenv("RTX_TAIL");
    if (tail_env) tail_slots = atoll(tail_env);
    // RTX_TAIL_ITER=k: the tail kernel takes over at batched iteration k
    // whatever the live count (0: by the live count only).  Default 5: the
    // full frames have nothing left by then (46.4 vs 46.4 ms headline, 62.7
    // vs 63.4 C4) while a shard's stragglers finish without 1-2 more
    // launch pairs bounded by their slowest query (8-way shard 9.7 vs 10.4
    // ms, C4's 12.1 vs 12.4; iteration 4: full frames 0.5-1.5 ms slower)
    int tail_iter = 5;
    const char* ti_env = getenv("RTX_TAIL_ITER");
    if (ti_env) tail_iter = std::max(0, atoi(ti_env));
    // (only when every unit has its sample slot from the start: with fewer
    // slots than units, iteration 5 comes long before the units are all
    // claimed, and the switch waits for the live count instead)
    if (int64_t(F.wf_nslot) < F.n_samples && !ti_env) tail_iter = 0;
    // (nor when the frame's history shows more fork requests than spares:
    // its sub-trees then also run on their parents' stacks, one ray per
    // iteration, and much is left at iteration 5 — R1, the glass frame:
    // 394 -> 253 ms with the switch by live count only, profiles/r04w_*)
    if (fspare >= 0 && !spares_enough && !ti_env) tail_iter = 0;
    // Pending stacks of two entries, not P.depth, when every
    // ray that pushes children forks them all: the frame's history shows every
    // fork request granted (spares_enough — requests do not depend on the
    // grants, so a render with at least that many spares grants them all
    // again), every child is a node (P.depth <= fork depth + 1), and no such
    // ray reaches the tail kernel, which does not fork (rays with children
    // are shaded by iteration P.depth - 2; the tail starts at tail_iter, or
    // by the live count only once a check is read, iteration 7, unless the
    // group starts under tail_slots).  A slot then holds only its own ray.
    // A push that would not fit sets bit 2 of *bover, read back after the
    // frame: the host reports it and the frame's later renders use full
    // stacks (RTX_LOW_STACK=0: never two entries).
    // (RTX_LOW_STACK=2, a test knob: two entries whatever the history says,
    // so the overflow check and the re-render can be exercised)
    bool low_stack = false;
    {
      const char* e = getenv("RTX_LOW_STACK");
      const int ls_mode = e ? atoi(e) : 1;
      const bool proven = spares_enough && spare_fit && params->depth <= fork_depth + 1 && gslots > tail_slots &&
                          (tail_iter == 0 || tail_iter >= params->depth - 1) &&
                          st->bucket_hist.find(bkey) != st->bucket_hist.end();
      low_stack = fuse && fork && !adaptive && !st->full_stack_keys.count(bkey) &&
                  (ls_mode == 2 || (ls_mode == 1 && proven));
    }
    const int pcap_run = low_stack ? std::min(pcap, 2) : pcap;
    // the slot buffers follow the pool: a first render sizes them for the
    // default pool, later renders of the frame for its fork history, and a
    // buffer much larger than this frame needs is given back (once; hipFree
    // waits for the device) — on a render's first pass and not on adaptive
    // frames, whose level chunks would resize them back and forth
    auto fit = [&](void** ptr, size_t* have, size_t need) -> rtx_status {
      if (X->wf_call == 0 && !adaptive && *have > need + need / 8 + (size_t(64) << 20)) {
        ctx_free(*ptr);
        *ptr = nullptr;
        *have = 0;
      }
      return ensure(ptr, have, need);
    };
    if ((rc = fit(&X->d_wf, &X->wf_bytes, size_t(G) * (bytes_qc + bytes_qn + 2 * al(gs * sizeof(int))))) != RTX_OK)
      return rc;
    F.fuse = fuse ? 1 : 0;
    F.chk_units = fork_ok ? static_cast<int64_t>(nunit_out) : 0;
    F.chk_wunits = static_cast<int>(n_units);
    F.chk_live = static_cast<int>(gs);
#ifdef RTX_BOUNDS_CHECK
    // (the check's self-test: a live-list bound of 1, so the first group's
    // second live slot must be reported — profiles/r06i_bounds_check.txt)
    if (const char* e = getenv("RTX_TEST_CHK_SELFTEST"))
      if (atoi(e) != 0) F.chk_live = 1;
#endif
    F.wterm = nullptr;
    if (fuse && nl > 0) {
      if ((rc = fit(reinterpret_cast<void**>(&X->d_wterm), &X->wterm_bytes, n_units * ns * 3 * sizeof(double))) !=
          RTX_OK)
        return rc;
      F.wterm = X->d_wterm;
    }
    if ((rc = fit(&X->d_lane, &X->lane_bytes, lane_mem_bytes(ns, fuse))) != RTX_OK) return rc;
    const LaneMem A = lane_mem_at(X->d_lane, ns, fuse);
    if ((rc = fit(reinterpret_cast<void**>(&X->d_pbuf), &X->pbuf_bytes,
                     ns * pcap_run * 13 * sizeof(double))) != RTX_OK)
      return rc;
    // Fork slots go back on a free list when their sub-trees end, unless the
    // frame's history says the spares cover every request (the headline
    // frame: every fork is granted anyway).  R1 (glass): 447 -> 395 ms.
    const bool recycle = fuse && fork && !(spares_enough && spare_fit);
    if (recycle &&
        (rc = fit(reinterpret_cast<void**>(&X->d_free), &X->free_bytes, size_t(G) * gs * sizeof(int))) != RTX_OK)
      return rc;
    if (!X->d_counters) HIP_TRY(hipMalloc(&X->d_counters, 16 * CNT_PER_GROUP * sizeof(unsigned int)));
    if (!X->h_counters) HIP_TRY(hipHostMalloc(&X->h_counters, 16 * CNT_PER_GROUP * sizeof(unsigned int)));
    // group 0 runs on the caller's ws, groups 1.. on their own streams
    // (GPU_MAX_HW_QUEUES is 4 by default: more streams than queues would
    // serialize groups behind each other)
    while (static_cast<int>(X->wf_streams.size()) < G) {
      hipStream_t s2;
      HIP_TRY(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
      X->wf_streams.push_back(s2);
      hipEvent_t ev;
      HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      X->wf_join.push_back(ev);
      HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      X->wf_check.push_back(ev);
    }
    if (!X->wf_fork) HIP_TRY(hipEventCreateWithFlags(&X->wf_fork, hipEventDisableTiming));
    std::vector<QList> ql(size_t(G) * 2);
    {
      char* base = static_cast<char*>(X->d_wf);
      for (size_t m = 0; m < ql.size(); ++m) {
        const size_t cap = (m & 1) ? capn : gs, dn = (m & 1) ? nd : qc_d;
        ql[m].slot = reinterpret_cast<int*>(base);
        ql[m].d = reinterpret_cast<double*>(base + al(cap * sizeof(int)));
        ql[m].iv = reinterpret_cast<int*>(base + al(cap * sizeof(int)) + al(cap * dn * sizeof(double)));
        ql[m].cap = cap;
        base += (m & 1) ? bytes_qn : bytes_qc;
      }
    }
    std::vector<int*> live(size_t(G) * 2);  // [g * 2 + 0]: list A, [g * 2 + 1]: list B
    {
      char* base = static_cast<char*>(X->d_wf) + size_t(G) * (bytes_qc + bytes_qn);
      for (size_t k = 0; k < live.size(); ++k) {
        live[k] = reinterpret_cast<int*>(base);
        base += al(gs * sizeof(int));
      }
    }
    // upper bound of each group's live slots (counts only fall; read back by
    // the pipelined checks): sizes the tail iterations' grids
    std::vector<int64_t> live_bound(size_t(G), gslots);
    // upper bound of the live slots an iteration can see (live_bound plus
    // the forks that can still start): sizes the grids
    std::vector<int64_t> grid_bound(size_t(G), gslots);
    F.qchunk = 64;
    // First iteration without an advance launch (fused frames): the closest-
    // hit launch claims each sample slot's first sample and queries its first
    // camera ray itself (cam_first_claim).  cam_n[g]: the group's sample
    // slots with a first unit (slot_unit(kdone 0) is increasing in the slot,
    // so they are a prefix).  RTX_CAM_FIRST=0: the advance launch (A/B).
    bool cam_first = fuse && params->depth >= 0;
    {
      const char* e = getenv("RTX_CAM_FIRST");
      if (e && atoi(e) == 0) cam_first = false;
    }
    std::vector<int> cam_n(size_t(G), 0);
    for (int g = 0; g < G && cam_first; ++g) {
      int64_t c = 0;
      for (int64_t b = 0; b * 64 < gsamp; ++b) {
        const int64_t base = (b * G + g) * 64;
        if (base >= F.n_samples) break;
        c += std::min<int64_t>(std::min<int64_t>(64, gsamp - b * 64), F.n_samples - base);
      }
      cam_n[size_t(g)] = static_cast<int>(c);
      if (c > gsamp) {  // (never: the first units are a prefix of the sample slots)
        g_err = "rtx_render: internal error: first-launch claims exceed a group's sample slots";
        return RTX_ERR_INVALID;
      }
    }
    if ((rc = stage_copy(st, X->d_frame, &F, sizeof(FrameParams), ws)) != RTX_OK) return rc;
    // every slot starts ST_IDLE, kdone = 0, outside a discoverMat walk, no
    // deferred colour: set by the group's first advance_kernel, which visits
    // all of its slots (every other field is written before it is read)
    HIP_TRY(hipMemsetAsync(X->d_counters, 0, 16 * CNT_PER_GROUP * sizeof(unsigned int), ws));
    // LDS per workgroup: the tail kernels' whole stacks (cold state in
    // registers); the trace kernels' stacks and cold state (trace_kernel) —
    // whole stacks unless those would cost the trace kernels a resident
    // workgroup (RTX_TRACE_WAVES per SIMD: 3 of 160 KB), else SHORT stacks
    // (the 1M-face dragon: 41 entries)
    const size_t lds_stacks = size_t(st->stack_cap) * 64 * sizeof(int) * WAVES_PER_WG;
    const size_t lds = lds_stacks;
    const size_t lds_cold = size_t(RTX_COLD_FIELDS) * 64 * sizeof(double) * WAVES_PER_WG;
    const size_t lds_full = lds_stacks + lds_cold;
    int lds_k = RTX_LDS_STACK;
    bool short_stack = st->stack_cap > lds_k && lds_full * RTX_TRACE_WAVES > size_t(160) * 1024;
    // (test knob: short stacks of K entries on every frame, so the overflow
    // columns are exercised — tests/test_gpu_parity.py)
    if (const char* e = getenv("RTX_TEST_LDS_STACK"))
      if (atoi(e) > 0) {
        lds_k = std::min(atoi(e), 64);
        short_stack = st->stack_cap > lds_k;
      }
    const size_t lds_tr = short_stack ? size_t(lds_k) * 64 * sizeof(int) * WAVES_PER_WG + lds_cold : lds_full;
    const int ovf_entries = short_stack ? st->stack_cap - lds_k : 0;
    if (lds > 160 * 1024 || lds_tr > 160 * 1024) {
      g_err = "rtx_render: LDS budget exceeded (BVH too deep)";
      return RTX_ERR_CAPACITY;
    }
    const void* tfn =
        stats ? (short_stack ? reinterpret_cast<const void*>(trace_kernel<true, Q_CLOSEST, false, false, false, true>)
                             : reinterpret_cast<const void*>(trace_kernel<true, Q_CLOSEST>))
              : (short_stack ? reinterpret_cast<const void*>(trace_kernel<false, Q_CLOSEST, false, false, false, true>)
                             : reinterpret_cast<const void*>(trace_kernel<false, Q_CLOSEST>));
    int per_cu = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, tfn, WG, lds_tr));
    if (per_cu < 1) per_cu = 1;
    int64_t tgrid = static_cast<int64_t>(st->n_cu) * per_cu;
    const int64_t tgrid_full = std::min<int64_t>(per, tgrid);
    int64_t small_frame = 10000000;
    {
      // Persistent trace grids of 1/div of the resident workgroups, so the
      // groups' kernels share the GPU instead of each filling it: on small
      // frames (a shard of a multi-GPU frame: at most small_frame samples,
      // default 10 M), div = G — there the groups' launches are mostly
      // latency-bound and a group's advance launch otherwise waits for CU
      // space behind the other groups' persistent kernels (8-way headline
      // shard 7.85-8.08 -> 7.61 ms; the whole frame 36.9 -> 38.4 ms, so not
      // there).
      const int div = F.n_samples <= small_frame ? G : 1;
      if (div > 1) tgrid = std::max<int64_t>(1, tgrid / div);
    }
    if (tgrid > per) tgrid = per;
    // the fused kernels' own residency (their launch bounds differ:
    // as the plain ones, RTX_TRACE_WAVES, but different register counts)
    int64_t tgrid_c = tgrid, tgrid_n = tgrid;
    int64_t tfull_c = tgrid_full, tfull_n = tgrid_full;  // whole-GPU residency
    if (fuse) {
      int pc = 0, pn = 0;
      HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &pc,
          short_stack ? reinterpret_cast<const void*>(trace_kernel<false, Q_CLOSEST, true, true, false, true>)
                      : reinterpret_cast<const void*>(trace_kernel<false, Q_CLOSEST, true, true>),
          WG, lds_tr));
      HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &pn,
          short_stack ? reinterpret_cast<const void*>(trace_kernel<false, Q_NEXT, true, false, false, true>)
                      : reinterpret_cast<const void*>(trace_kernel<false, Q_NEXT, true>),
          WG, lds_tr));
      tgrid_c = std::min<int64_t>(per, std::max<int64_t>(1, tgrid * std::max(1, pc) / per_cu));
      tgrid_n = std::min<int64_t>(per, std::max<int64_t>(1, tgrid * std::max(1, pn) / per_cu));
      tfull_c = std::min<int64_t>(per, std::max<int64_t>(1, tgrid_full * std::max(1, pc) / per_cu));
      tfull_n = std::min<int64_t>(per, std::max<int64_t>(1, tgrid_full * std::max(1, pn) / per_cu));
    }
    // stack overflow columns (StackShort): per group, one column of
    // ovf_entries per thread of its largest trace launch
    const int64_t ovf_threads =
        std::max<int64_t>(std::max<int64_t>(std::max<int64_t>(tgrid, tgrid_c), std::max<int64_t>(tgrid_n, tfull_c)),
                          tfull_n) * WG;
    if (ovf_entries > 0 &&
        (rc = ensure(reinterpret_cast<void**>(&X->d_ovf), &X->ovf_bytes,
                     size_t(G) * size_t(ovf_entries) * size_t(ovf_threads) * sizeof(int))) != RTX_OK)
      return rc;
    // The first iteration's closest-hit / walk grids as a percentage of the
    // whole GPU's residency (tg0_c / tg0_n; 0 = the grids above).
    // On whole frames (div 1) the groups' first launches otherwise each take
    // the whole GPU in turn: group 0's camera rays first, then its walks
    // beside the others' camera rays, and its advance launch starved of CUs
    // until their walks end, so all three groups reach their advance launches
    // together and the GPU streams lane state with no traversal beside it.
    // Half-GPU first launches stagger the groups: headline 31.5-31.9 vs
    // 32.6-33.0 ms, C4 42.2-42.6 vs 43.9 (profiles/r05l_ab_first_grid.txt).
    // Shards keep their 1/G grids (no change measured there).
    const int tg0_c = F.n_samples > small_frame ? 50 : 0, tg0_n = F.n_samples > small_frame ? 50 : 0;
    const char* dbg_env = getenv("RTX_DEBUG");
    const bool dbg = dbg_env && atoi(dbg_env) != 0;
    const int dbg_level = dbg_env ? atoi(dbg_env) : 0;
    const int check_every = 4;
    // costly traversal units wait while this many lanes of a wave are at a
    // 4-wide record (trace_kernel; RTX_LEAF_K, 1..65, 65: never wait).  8
    // since round 6 (cold state in LDS): headline unchanged, R1 247 -> 243,
    // C4 40.9 -> 40.4 ms against 16 (profiles/r06n_ab_leaf_k.txt)
    int leaf_k = 8;
    {
      const char* e = getenv("RTX_LEAF_K");
      if (e && atoi(e) > 0) leaf_k = std::min(65, atoi(e));
    }
    hipEvent_t e0, e1;
    if ((rc = get_event(&e0)) != RTX_OK || (rc = get_event(&e1)) != RTX_OK) return rc;
    HIP_TRY(hipEventRecord(e0, ws));
    HIP_TRY(hipEventRecord(X->wf_fork, ws));
    for (int g = 1; g < G; ++g) HIP_TRY(hipStreamWaitEvent(X->wf_streams[size_t(g)], X->wf_fork, 0));
    std::vector<int> done(size_t(G), 0), pending_check(size_t(G), -1);
    int ndone = 0;
    for (int it = 0; ndone < G; ++it) {
      for (int g = 0; g < G; ++g) {
        if (done[size_t(g)]) continue;
        hipStream_t sg = g == 0 ? ws : X->wf_streams[size_t(g)];
        unsigned int* cnt = X->d_counters + CNT_PER_GROUP * g;
        const QList& q0 = ql[size_t(g) * 2];
        const QList& q1 = ql[size_t(g) * 2 + 1];
        // (after a claiming first launch, iteration 1 visits every slot by
        // index and writes the first live list: no tail before iteration 2)
        if (it > (cam_first ? 1 : 0) &&
            (live_bound[size_t(g)] <= tail_slots || (tail_iter > 0 && it >= tail_iter))) {
          // few slots left: finish them in one persistent launch
          const bool odd = (it & 1) != 0;  // this iteration would read the list the last one wrote
          const int in_cnt = odd ? CNT_ALIVE_A : CNT_ALIVE_B;
          const int* live_in = live[size_t(g) * 2 + (odd ? 0 : 1)];
          const int64_t lb = grid_bound[size_t(g)];
          const int64_t grid = std::max<int64_t>(1, (lb + WG - 1) / WG);
          if (fuse) {
            if (stats)
              RTX_LAUNCH((tail_fused_kernel<true>), dim3(grid), dim3(WG), lds, sg, S, X->d_scene, X->d_frame,
                                 A, sb, d_hits, X->d_pbuf, pcap_run, cnt, live_in, in_cnt, st->stack_cap, st->d_stats,
                                 ql[size_t(g) * 2 + 1], static_cast<int>(g * gslots));
            else
              RTX_LAUNCH((tail_fused_kernel<false>), dim3(grid), dim3(WG), lds, sg, S, X->d_scene, X->d_frame,
                                 A, sb, d_hits, X->d_pbuf, pcap_run, cnt, live_in, in_cnt, st->stack_cap, st->d_stats,
                                 ql[size_t(g) * 2 + 1], static_cast<int>(g * gslots));
          } else {
            dispatch2(stats, media, [&](auto st_, auto md_) {
              RTX_LAUNCH((tail_kernel<decltype(st_)::value, decltype(md_)::value>), dim3(grid), dim3(WG), lds,
                                 sg, S, X->d_scene, X->d_frame, A, sb, d_hits, X->d_pbuf, pcap_run, cnt, live_in,
                                 in_cnt, st->stack_cap, st->d_stats);
            });
          }
          HIP_TRY(hipGetLastError());
          done[size_t(g)] = 1;
          ++ndone;
          HIP_TRY(hipEventRecord(X->wf_join[size_t(g)], sg));
          continue;
        }
        // ping-pong live-slot lists: even iterations append to A, read B
        const bool odd = (it & 1) != 0;
        const int out_cnt = odd ? CNT_ALIVE_B : CNT_ALIVE_A, in_cnt = odd ? CNT_ALIVE_A : CNT_ALIVE_B;
        int* live_out = live[size_t(g) * 2 + (odd ? 1 : 0)];
        const int* live_in = live[size_t(g) * 2 + (odd ? 0 : 1)];
        // this iteration's counters were cleared by the last workgroup of the
        // previous iteration's next-hit kernel (the frame-start memset for
        // the first); this iteration's clears the next one's: even
        // iterations use lines 0-4 (out-count A), odd ones lines 1-5 (B)
        const int clr_next = odd ? 0 : 1;
        // advance mode: 1 init + every slot, 2 every slot (after a claiming
        // first launch), 0 the live list
        const int first = it == 0 ? 1 : (cam_first && it == 1 ? 2 : 0);
        const int64_t lb = grid_bound[size_t(g)];
        const int64_t agrid = first ? per : std::max<int64_t>(1, std::min<int64_t>(per, (lb + WG - 1) / WG));
        const int64_t tgc_it =
            fuse && it == 0 && tg0_c > 0 ? std::max<int64_t>(1, tfull_c * tg0_c / 100) : (fuse ? tgrid_c : tgrid);
        const int64_t tgn_it = fuse && it == 0 && tg0_n > 0 ? std::max<int64_t>(1, tfull_n * tg0_n / 100) : tgrid_n;
        const int64_t tg = std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(per, tgc_it), (lb + WG - 1) / WG));
        const bool cam_it = cam_first && it == 0;
        if (cam_it) {
          // the slots the first launch does not claim start idle
          const int n0 = static_cast<int>(gslots) - cam_n[size_t(g)];
          if (n0 > 0)
            RTX_LAUNCH(lane_init_kernel, dim3((n0 + WG - 1) / WG), dim3(WG), 0, sg, A,
                               static_cast<int>(g * gslots) + cam_n[size_t(g)], n0);
        } else if (fuse) {
          dispatch2(stats, fork, [&](auto st_, auto fk_) {
            RTX_LAUNCH((advance_fused_kernel<decltype(st_)::value, decltype(fk_)::value>), dim3(agrid),
                               dim3(WG), 0, sg, S, X->d_scene, X->d_frame, A, sb, d_hits, X->d_pbuf, pcap_run, q0,
                               q1, cnt, st->d_stats, static_cast<int>(g * gslots), live_in, live_out, first, in_cnt,
                               out_cnt, recycle ? X->d_free + size_t(g) * gs : nullptr);
          });
        } else {
          dispatch3(stats, media, fork, [&](auto st_, auto md_, auto fk_) {
            RTX_LAUNCH((advance_kernel<decltype(st_)::value, decltype(md_)::value, decltype(fk_)::value>),
                               dim3(agrid), dim3(WG), 0, sg,
                               S, X->d_scene, X->d_frame, A, sb, d_hits, X->d_pbuf, pcap_run, q0, q1, cnt,
                               st->d_stats, static_cast<int>(g * gslots), live_in, live_out, first, in_cnt, out_cnt);
          });
        }
        // the next-hit grid: fused walks can outnumber the live slots
        const int64_t tgn = fuse ? std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(per * nrec_n, tgn_it),
                                                                          (lb * int64_t(nrec_n) + WG - 1) / WG))
                                 : tg;
        ShadeArgs sa;
        std::memset(&sa, 0, sizeof(sa));
        sa.leaf_k = leaf_k;
        sa.free_ids = recycle ? X->d_free + size_t(g) * gs : nullptr;
        sa.ovf = ovf_entries > 0 ? X->d_ovf + size_t(g) * size_t(ovf_entries) * size_t(ovf_threads) : nullptr;
        sa.lds_k = lds_k;
        if (short_stack && std::max(tg, tgn) * WG > ovf_threads) {
          g_err = "rtx_render: internal error: a trace launch exceeds its stack overflow columns";
          return RTX_ERR_INVALID;
        }
        if (fuse) {
          sa.Fp = X->d_frame;
          sa.hits = d_hits;
          sa.pbuf = X->d_pbuf;
          sa.pend_cap = pcap_run;
          sa.qn = q1;
          sa.slot_off = static_cast<int>(g * gslots);
          sa.live_out = live_out;
          sa.out_cnt = out_cnt;
          sa.cam_n = cam_it ? cam_n[size_t(g)] : 0;
        }
        dispatch3(stats, fork, short_stack, [&](auto st_, auto fk_, auto sh_) {
          constexpr bool ST_ = decltype(st_)::value, FK_ = decltype(fk_)::value, SH_ = decltype(sh_)::value;
          if (fuse) {
            // (inside the dispatch lambda: no HIP_TRY returns here; debug only)
            hipEvent_t d0 = nullptr, d1 = nullptr;
            if (dbg_level >= 2) {  // RTX_DEBUG=2: every iteration's queries and closest-hit time (synchronous)
              (void)(hipStreamSynchronize(sg));
              if (stats) (void)(hipMemset(st->d_stats + 12, 0, 4 * sizeof(unsigned long long)));
              if (stats) (void)(hipMemset(st->d_stats + 35, 0, 4 * sizeof(unsigned long long)));
              (void)(hipEventCreate(&d0));
              (void)(hipEventCreate(&d1));
              (void)(hipEventRecord(d0, sg));
            }
            if (cam_it)
              RTX_LAUNCH((trace_kernel<ST_, Q_CLOSEST, true, FK_, true, SH_>), dim3(tg), dim3(WG), lds_tr, sg, S,
                                 X->d_scene, q0, cnt, A, st->stack_cap, st->d_stats, X->d_wterm, sa, -1);
            else
              RTX_LAUNCH((trace_kernel<ST_, Q_CLOSEST, true, FK_, false, SH_>), dim3(tg), dim3(WG), lds_tr, sg, S,
                                 X->d_scene, q0, cnt, A, st->stack_cap, st->d_stats, X->d_wterm, sa, -1);
            if (dbg_level >= 2) {
              unsigned int hc[CNT_PER_GROUP];
              unsigned long long hs[4] = {0, 0, 0, 0}, hw[4] = {0, 0, 0, 0};
              float ms = 0.f;
              (void)(hipEventRecord(d1, sg));
              (void)(hipStreamSynchronize(sg));
              (void)(hipEventElapsedTime(&ms, d0, d1));
              (void)(hipMemcpy(hc, cnt, sizeof(hc), hipMemcpyDeviceToHost));
              if (stats) (void)(hipMemcpy(hs, st->d_stats + 12, sizeof(hs), hipMemcpyDeviceToHost));
              if (stats) (void)(hipMemcpy(hw, st->d_stats + 35, sizeof(hw), hipMemcpyDeviceToHost));
              fprintf(stderr,
                      "rtx group %d iter %d: closest %u walks %u forks %u | closest-hit launch %.3f ms, max steps "
                      "%llu, queries over 100 steps %llu | slowest wave %.1f us, %llu wave steps, %llu claims\n",
                      g, it, cam_it ? static_cast<unsigned>(cam_n[size_t(g)]) : hc[CNT_Q], hc[CNT_Q + CNT_LINE],
                      hc[CNT_FORK], ms, hs[0], hs[2], (hw[0] >> 32) * 0.01, hw[0] & 0xffffffffull,
                      (hw[1] >> 16) & 0xffffull);
              (void)(hipEventDestroy(d0));
              (void)(hipEventDestroy(d1));
            }
            if (dbg_level >= 2) {
              (void)(hipEventCreate(&d0));
              (void)(hipEventCreate(&d1));
              (void)(hipEventRecord(d0, sg));
            }
            RTX_LAUNCH((trace_kernel<ST_, Q_NEXT, true, false, false, SH_>), dim3(tgn), dim3(WG), lds_tr, sg, S, X->d_scene, q1,
                               cnt, A, st->stack_cap, st->d_stats, X->d_wterm, sa, clr_next);
            if (dbg_level >= 2) {
              float ms = 0.f;
              unsigned long long hw[4] = {0, 0, 0, 0}, hs2[4] = {0, 0, 0, 0};
              (void)(hipEventRecord(d1, sg));
              (void)(hipStreamSynchronize(sg));
              (void)(hipEventElapsedTime(&ms, d0, d1));
              if (stats) (void)(hipMemcpy(hw, st->d_stats + 35, sizeof(hw), hipMemcpyDeviceToHost));
              if (stats) (void)(hipMemcpy(hs2, st->d_stats + 12, sizeof(hs2), hipMemcpyDeviceToHost));
              fprintf(stderr,
                      "rtx group %d iter %d: walk launch %.3f ms | max steps per query %llu | slowest wave %.1f us, "
                      "%llu wave steps, %llu claims, %llu walk restarts\n",
                      g, it, ms, hs2[1], (hw[2] >> 32) * 0.01, hw[2] & 0xffffffffull, (hw[3] >> 16) & 0xffffull,
                      hw[3] & 0xffffull);
              (void)(hipEventDestroy(d0));
              (void)(hipEventDestroy(d1));
            }
          } else if (!FK_) {
            RTX_LAUNCH((trace_kernel<ST_, Q_CLOSEST, false, false, false, SH_>), dim3(tg), dim3(WG), lds_tr, sg, S, X->d_scene, q0, cnt, A,
                               st->stack_cap, st->d_stats, nullptr, sa, -1);
            RTX_LAUNCH((trace_kernel<ST_, Q_NEXT, false, false, false, SH_>), dim3(tg), dim3(WG), lds_tr, sg, S, X->d_scene, q1, cnt, A,
                               st->stack_cap, st->d_stats, nullptr, sa, clr_next);
          }
        });
        if (!fuse && fork) {  // the sequential machine's trace kernels do not depend on forking
          dispatch2(stats, short_stack, [&](auto st_, auto sh_) {
            constexpr bool ST_ = decltype(st_)::value, SH_ = decltype(sh_)::value;
            RTX_LAUNCH((trace_kernel<ST_, Q_CLOSEST, false, false, false, SH_>), dim3(tg), dim3(WG), lds_tr, sg, S,
                       X->d_scene, q0, cnt, A, st->stack_cap, st->d_stats, nullptr, sa, -1);
            RTX_LAUNCH((trace_kernel<ST_, Q_NEXT, false, false, false, SH_>), dim3(tg), dim3(WG), lds_tr, sg, S,
                       X->d_scene, q1, cnt, A, st->stack_cap, st->d_stats, nullptr, sa, clr_next);
          });
        }
        HIP_TRY(hipGetLastError());
        if (it % check_every == check_every - 1) {
          // pipelined liveness check: read back the counters of the check
          // enqueued one round earlier (the GPU keeps ~check_every
          // iterations of this group queued meanwhile)
          if (pending_check[size_t(g)] >= 0) {
            HIP_TRY(hipEventSynchronize(X->wf_check[size_t(g)]));
            const unsigned int* hc = X->h_counters + CNT_PER_GROUP * g;
            const unsigned int alive = hc[(pending_check[size_t(g)] & 1) ? CNT_ALIVE_B : CNT_ALIVE_A];
            live_bound[size_t(g)] = alive;
            // forks add live slots: bound by the fork slots still free
            // (fresh spares only: a reused fork slot left the live count first)
            const int64_t forks_left =
                fork ? std::max<int64_t>(0, (gslots - gsamp) - static_cast<int64_t>(hc[recycle ? CNT_FRESH : CNT_FORK]))
                     : 0;
            grid_bound[size_t(g)] = std::min<int64_t>(gslots, alive + forks_left);
            if (dbg)
              // (the query counts of that iteration are already cleared by the
              // next one's last workgroup: RTX_DEBUG=2 prints them per launch)
              fprintf(stderr, "rtx group %d iter %d: alive %u\n", g, pending_check[size_t(g)], alive);
            if (alive == 0) {
              done[size_t(g)] = 1;
              ++ndone;
              HIP_TRY(hipEventRecord(X->wf_join[size_t(g)], sg));
              continue;
            }
          }
          HIP_TRY(hipMemcpyAsync(X->h_counters + CNT_PER_GROUP * g, cnt, CNT_PER_GROUP * sizeof(unsigned int),
                                 hipMemcpyDeviceToHost, sg));
          HIP_TRY(hipEventRecord(X->wf_check[size_t(g)], sg));
          pending_check[size_t(g)] = it;
        }
      }
      if (it > 1000000) {
        g_err = "rtx_render: wavefront loop did not terminate";
        return RTX_ERR_INVALID;
      }
    }
    for (int g = 1; g < G; ++g) HIP_TRY(hipStreamWaitEvent(ws, X->wf_join[size_t(g)], 0));
    HIP_TRY(hipEventRecord(e1, ws));
    frame_events.push_back({e0, e1});
    // a run sized from its history (two-entry stacks, a pool of the last
    // render's set count) is checked once the frame has run (rtx_render's end)
    if (low_stack || (fork_ok && bcap < nunit_out)) chk_keys.push_back(bkey);
    if (fork_ok && (st->probe_mode || st->bucket_hist.find(bkey) == st->bucket_hist.end()) && !X->bstat_pending) {
      // first render of this frame: its set count, read at the next call
      HIP_TRY(hipMemcpyAsync(X->h_bstat, X->d_bstat, 2 * sizeof(unsigned int), hipMemcpyDeviceToHost, ws));
      // (the fork counters are final: the other groups joined ws above)
      X->bstat_groups = fork ? G : 0;
      for (int g = 0; g < X->bstat_groups; ++g)
        HIP_TRY(hipMemcpyAsync(X->h_bstat + 4 + g, X->d_counters + CNT_PER_GROUP * g + CNT_FORK, sizeof(unsigned int),
                               hipMemcpyDeviceToHost, ws));
      HIP_TRY(hipEventRecord(X->bstat_ev, ws));
      X->bstat_pending = true;
      X->bstat_key = bkey;
    }
    X->wf_call++;
    return RTX_OK;
  };
  if (!adaptive) {
    if (!megakernel && (rc = run_wavefront(F, npix, true)) != RTX_OK) return rc;
    if (ws != stream) {  // the caller's stream waits for the frame (its group-0 stream, joined by the others)
      HIP_TRY(hipEventRecord(X->wf_join[0], ws));
      HIP_TRY(hipStreamWaitEvent(stream, X->wf_join[0], 0));
    }
    const int64_t ppb = WG / F.spp;
    const int64_t rblocks = (npix + ppb - 1) / ppb;
    RTX_LAUNCH(reduce_kernel, dim3(rblocks), dim3(WG), 0, stream, X->d_frame, sb, d_rgb8, d_rgbf, npix);
    HIP_TRY(hipGetLastError());
  } else if (!megakernel) {
    // adaptive AA, level by level (adapt_*_kernel): level 0's regions are the
    // output slots' pixels; a deeper level runs in chunks of at most npix
    // regions (the sample buffer and buckets are sized for npix * spp)
    F.adapt = 1;
    F.aregs = nullptr;
    if ((rc = run_wavefront(F, npix, true)) != RTX_OK) return rc;
    size_t nlevel = 0;  // level buffers handed out this frame
    auto level_alloc = [&](int64_t n, bool regs, ALevel& lv) -> rtx_status {
      auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
      const size_t bv = al(size_t(n) * sizeof(dvec3)), bi = al(size_t(n) * sizeof(int));
      const size_t br = regs ? al(size_t(n) * sizeof(ARegion)) : 0;
      if (X->d_level.size() <= nlevel) {
        X->d_level.push_back(nullptr);
        X->level_bytes.push_back(0);
      }
      if ((rc = ensure(&X->d_level[nlevel], &X->level_bytes[nlevel], bv + 2 * bi + br + 256)) != RTX_OK) return rc;
      char* b = static_cast<char*>(X->d_level[nlevel++]);
      lv.val = reinterpret_cast<dvec3*>(b);
      lv.first = reinterpret_cast<int*>(b + bv);
      lv.mask = reinterpret_cast<int*>(b + bv + bi);
      lv.reg = regs ? reinterpret_cast<const ARegion*>(b + bv + 2 * bi) : nullptr;
      lv.n = n;
      return RTX_OK;
    };
    std::vector<ALevel> levels(1);
    if ((rc = level_alloc(npix, false, levels[0])) != RTX_OK) return rc;
    if (!X->d_acnt) HIP_TRY(hipMalloc(&X->d_acnt, 2 * sizeof(unsigned int)));
    unsigned int hcnt[2] = {0u, 0u};
    HIP_TRY(hipMemsetAsync(X->d_acnt, 0, 2 * sizeof(unsigned int), ws));
    RTX_LAUNCH(adapt_stats_kernel, dim3((npix + WG - 1) / WG), dim3(WG), 0, ws, X->d_frame, sb,
                       levels[0], int64_t(0), int64_t(npix), X->d_acnt);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(hcnt, X->d_acnt, sizeof(hcnt), hipMemcpyDeviceToHost, ws));
    HIP_TRY(hipStreamSynchronize(ws));
    // (the recursion ends once a region is under eps: ~14 levels at most)
    while (hcnt[0] > 0 && levels.size() < 64) {
      const int64_t n = hcnt[0];
      ALevel nx;
      if ((rc = level_alloc(n, true, nx)) != RTX_OK) return rc;
      HIP_TRY(hipMemsetAsync(X->d_acnt, 0, 2 * sizeof(unsigned int), ws));
      const ALevel& up = levels.back();
      RTX_LAUNCH(adapt_emit_kernel, dim3((up.n + WG - 1) / WG), dim3(WG), 0, ws, X->d_frame, up,
                         const_cast<ARegion*>(nx.reg), X->d_acnt + 1);
      HIP_TRY(hipGetLastError());
      levels.push_back(nx);
      for (int64_t c0 = 0; c0 < n; c0 += npix) {
        const int64_t nc = std::min<int64_t>(npix, n - c0);
        FrameParams FL = F;
        FL.aregs = nx.reg + c0;
        FL.n_items = nc;
        FL.n_samples = nc * FL.spp * (FL.cam_split ? FL.ncam : 1);
        if ((rc = run_wavefront(FL, nc, false)) != RTX_OK) return rc;
        RTX_LAUNCH(adapt_stats_kernel, dim3((nc + WG - 1) / WG), dim3(WG), 0, ws, X->d_frame, sb, nx, c0,
                           nc, X->d_acnt);
        HIP_TRY(hipGetLastError());
        // (run_wavefront copies FL to the device before its first launch;
        // FL must outlive that copy)
        HIP_TRY(hipStreamSynchronize(ws));
      }
      HIP_TRY(hipMemcpyAsync(hcnt, X->d_acnt, sizeof(hcnt), hipMemcpyDeviceToHost, ws));
      HIP_TRY(hipStreamSynchronize(ws));
    }
    if (hcnt[0] > 0) {
      g_err = "rtx_render: adaptive AA recursion deeper than 64 levels";
      return RTX_ERR_CAPACITY;
    }
    for (size_t L = levels.size(); L-- > 0;) {
      ALevel below = L + 1 < levels.size() ? levels[L + 1] : ALevel{nullptr, nullptr, nullptr, nullptr, 0};
      RTX_LAUNCH(adapt_combine_kernel, dim3((levels[L].n + WG - 1) / WG), dim3(WG), 0, ws, X->d_frame,
                         levels[L], below, d_rgb8, d_rgbf);
      HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipStreamSynchronize(ws));  // the level buffers are freed on return
  }
  for (auto& pr : frame_events) {
    st->ev_start.push_back(pr.first);
    st->ev_stop.push_back(pr.second);
  }
  // the frame check (collect_check): the runs' *bover, once they have run
  if (!chk_keys.empty()) {
    if (!X->chk_ev) HIP_TRY(hipEventCreateWithFlags(&X->chk_ev, hipEventDisableTiming));
    HIP_TRY(hipMemcpyAsync(X->h_bstat + 2, X->d_bstat + 1, sizeof(unsigned int), hipMemcpyDeviceToHost, ws));
    HIP_TRY(hipEventRecord(X->chk_ev, ws));
    X->chk_pending = true;
    X->chk_seq = seq;
    X->chk_keys = chk_keys;
  }
  // the context is free again once the caller's stream has passed the frame
  // (its reduce on the caller's stream; ws == stream for the other renders)
  HIP_TRY(hipEventRecord(X->free_ev, stream));
  X->used = true;
  if (!device_ptrs) {
    if (rgb8) HIP_TRY(hipMemcpyAsync(rgb8, d_rgb8, npix * 3, hipMemcpyDeviceToHost, ws));
    if (rgb_f64) HIP_TRY(hipMemcpyAsync(rgb_f64, d_rgbf, npix * 3 * sizeof(double), hipMemcpyDeviceToHost, ws));
    if (hits) HIP_TRY(hipMemcpyAsync(hits, d_hits, npix * F.spp * sizeof(RtxHitRecord), hipMemcpyDeviceToHost, ws));
    HIP_TRY(hipStreamSynchronize(ws));
  }
  // a synchronous render (host buffers, counters, adaptive levels) knows its
  // outcome now: a wrong frame is rendered again (rtx_render), never returned
  if (X->chk_pending && (!device_ptrs || stats || adaptive)) {
    HIP_TRY(hipStreamSynchronize(ws));
    const int64_t nb = st->bad_n, fb = st->bad_first;
    if (collect_check(st, *X, true)) {
      st->bad_n = nb;  // (not recorded: the caller gets the re-rendered frame)
      st->bad_first = fb;
      *redo = 1;
      return RTX_OK;
    }
  }
  // depth_probe's render: its fork requests (every node child asks, granted
  // or not) and its work units, before it returns
  if (st->probe_mode && X->bstat_pending && X->bstat_groups > 0) {
    HIP_TRY(hipEventSynchronize(X->bstat_ev));
    st->probe_req = 0;
    for (int g = 0; g < X->bstat_groups; ++g) st->probe_req += X->h_bstat[4 + g];
    st->probe_units = F.n_samples;
  }
  if (stats) {
    unsigned long long c[RTX_STATS_N];
    HIP_TRY(hipMemcpyAsync(c, st->d_stats, sizeof(c), hipMemcpyDeviceToHost, ws));
    HIP_TRY(hipStreamSynchronize(ws));
    {
      const char* dbg = getenv("RTX_DEBUG");
      if (dbg && atoi(dbg) != 0)
      {
        fprintf(stderr, "rtx trace SIMD efficiency: closest %llu wave steps, %.3f active; next %llu, %.3f\n", c[8],
                c[8] ? double(c[9]) / (64.0 * c[8]) : 0.0, c[10], c[10] ? double(c[11]) / (64.0 * c[10]) : 0.0);
        fprintf(stderr, "rtx trace steps per query: max closest %llu next %llu; queries over 100 steps: %llu / %llu\n",
                c[12], c[13], c[14], c[15]);
        fprintf(stderr, "rtx tail: slowest chain %llu cycles, longest chain %llu queries\n", c[16], c[17]);
        for (int m = 0; m < 2; ++m) {  // cycle breakdown of the trace kernels by unit class
          const unsigned long long* pr = c + RTX_STATS_PROF + 20 * m;
          const double tot = pr[18] ? double(pr[18]) : 1.0;
          fprintf(stderr, "rtx %s kernel cycles %.4g: between traversals %.3f (%llu runs, %.0f cyc/run)",
                  m ? "next" : "closest", double(pr[18]), pr[16] / tot, pr[17], pr[17] ? double(pr[16]) / pr[17] : 0.0);
          static const char* nm[8] = {"idle", "R", "O", "RO", "L", "RL", "OL", "ROL"};
          for (int k = 1; k < 8; ++k)
            fprintf(stderr, "; %s %.3f (%llu steps, %.0f cyc)", nm[k], pr[k] / tot, pr[8 + k],
                    pr[8 + k] ? double(pr[k]) / pr[8 + k] : 0.0);
          fprintf(stderr, "\n");
        }
      }
    }
    std::memset(stats, 0, sizeof(*stats));
    stats->camera_rays = c[0];
    stats->secondary_rays = c[1];
    stats->shadow_rays = c[2];
    stats->rays = c[0] + c[1] + c[2];
    stats->node_visits = c[3];
    stats->object_tests = c[4];
    stats->tri_tests = c[5];
    stats->shades = c[6];
    stats->shadow_traced = c[18];
    double tot = 0.0;
    for (auto& pr : frame_events) {
      float ms = 0.0f;
      HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
      tot += ms;
    }
    stats->kernel_ms = tot;
    for (int k = 0; k < RTX_STATS_N; ++k) st->last_work[k] = static_cast<int64_t>(c[k]);
  }
  return RTX_OK;
}

// The fork-depth rule of a whole frame (run_wavefront, "forks at many of
// their nodes"), decided once per whole frame: a host-buffer render at the
// default depth of a FIXED subset of the whole frame — every 16 x 16 tile
// whose deal index is a multiple of tiles / 128 (about 128 tiles), or the
// whole frame when it has at most 256 such tiles — whose fork requests
// (every node child asks, granted or not) exceed half its work units: depth
// 3, else 4.  The subset depends on the frame's parameters only, not on the
// shard being rendered, so a single-GPU frame and every rank of a multi-GPU
// job decide alike and render the same bits.  The probe's kernels are not
// counted (rtx_kernel_time).
static rtx_status depth_probe(SceneState* st, const RtxRenderParams* params, void* stream_v, int64_t seq) {
  const char* fork_env = getenv("RTX_FORK");
  const char* fd_env = getenv("RTX_FORK_DEPTH");
  const char* mk_env = getenv("RTX_MEGAKERNEL");
  if ((fork_env && atoi(fork_env) == 0) || (fd_env && atoi(fd_env) > 0) || (mk_env && atoi(mk_env) != 0) ||
      params->anaglyph || !st->any_recur || params->depth <= 0 || params->aa_mode == RTX_AA_ADAPTIVE ||
      params->width <= 0 || params->height <= 0)
    return RTX_OK;  // (frames the rule does not apply to: run_wavefront never looks them up)
  const uint64_t key = whole_frame_key(*params);
  if (st->depth_rule.count(key)) return RTX_OK;
  RtxRenderParams q = *params;
  q.tile = 0;
  q.shard = 0;
  q.nshards = 1;
  q.packed = 0;
  const int64_t ntiles = int64_t((q.width + 15) / 16) * int64_t((q.height + 15) / 16);
  if (ntiles > 256) {
    q.tile = 16;
    q.nshards = static_cast<int32_t>(ntiles / 128);
    q.packed = 1;
  }
  int64_t npix = 0;
  rtx_status rc = rtx_shard_pixels(&q, &npix);
  if (rc != RTX_OK) return rc;
  std::vector<uint8_t> rgb(size_t(npix) * 3);
  const size_t ev0 = st->ev_start.size();
  const int64_t l0 = st->n_launch;
  st->probe_mode = true;
  st->probe_req = 0;
  st->probe_units = 0;
  int redo = 0;
  rc = render_once(st, &q, rgb.data(), nullptr, nullptr, 0, stream_v, nullptr, seq, true, &redo);
  st->probe_mode = false;
  for (size_t k = ev0; k < st->ev_start.size(); ++k) {  // (synchronous: its events are done)
    st->ev_pool.push_back(st->ev_start[k]);
    st->ev_pool.push_back(st->ev_stop[k]);
  }
  st->ev_start.resize(ev0);
  st->ev_stop.resize(ev0);
  st->n_launch = l0;
  if (rc != RTX_OK) return rc;
  st->depth_rule[key] = st->probe_units > 0 && 2 * st->probe_req > st->probe_units ? 3 : 4;
  if (const char* e = getenv("RTX_DEBUG"))
    if (atoi(e) != 0)
      fprintf(stderr, "rtx: fork-depth probe: %lld requests / %lld units -> depth %d\n",
              static_cast<long long>(st->probe_req), static_cast<long long>(st->probe_units), st->depth_rule[key]);
  return RTX_OK;
}

rtx_status rtx_render(void* scene, const RtxRenderParams* params, uint8_t* rgb8, double* rgb_f64,
                      RtxHitRecord* hits, int device_ptrs, void* stream_v, RtxStats* stats) {
  if (!scene || !params) {
    g_err = "rtx_render: null argument";
    return RTX_ERR_INVALID;
  }
  SceneState* st = static_cast<SceneState*>(scene);
  const int64_t seq = st->frame_seq++;
  rtx_status rc0 = depth_probe(st, params, stream_v, seq);
  if (rc0 != RTX_OK) return rc0;
  int redo = 0;
  const size_t ev0 = st->ev_start.size();
  const int64_t pip0 = st->n_pipelined;
  rtx_status rc = render_once(st, params, rgb8, rgb_f64, hits, device_ptrs, stream_v, stats, seq, false, &redo);
  if (rc == RTX_OK && redo) {
    if (redo == 1)
      fprintf(stderr, "rtx_render: rendering frame %lld again with full-size buffers\n", static_cast<long long>(seq));
    redo = 0;
    // the replaced attempt's kernel events and pipelining count go: the
    // counters (rtx_kernel_time, rtx_overlap_count) describe one frame
    for (size_t k = ev0; k < st->ev_start.size(); ++k) {
      HIP_TRY(hipEventSynchronize(st->ev_stop[k]));
      st->ev_pool.push_back(st->ev_start[k]);
      st->ev_pool.push_back(st->ev_stop[k]);
    }
    st->ev_start.resize(ev0);
    st->ev_stop.resize(ev0);
    st->n_pipelined = pip0;
    rc = render_once(st, params, rgb8, rgb_f64, hits, device_ptrs, stream_v, stats, seq, true, &redo);
    if (rc == RTX_OK && redo) {
      g_err = "rtx_render: the frame came out wrong twice (history-sized buffers short after a full-size re-render)";
      return RTX_ERR_FRAME;
    }
  }
#ifdef RTX_BOUNDS_CHECK
  if (rc == RTX_OK && (!device_ptrs || stats)) rc = bounds_check_report();
#endif
  return rc;
}

rtx_status rtx_last_work(void* scene, int64_t* out, int n) {
  if (!scene || !out || n < 0) return RTX_ERR_INVALID;
  const SceneState* st = static_cast<const SceneState*>(scene);
  const int m = n < RTX_WORK_COUNT ? n : RTX_WORK_COUNT;
  for (int k = 0; k < m; ++k) out[k] = st->last_work[20 + k];
  return RTX_OK;
}

rtx_status rtx_kernel_time(void* scene, double* total_ms, int* launches) {
  if (!scene) return RTX_ERR_INVALID;
  SceneState* st = static_cast<SceneState*>(scene);
  HIP_TRY(hipSetDevice(st->device));
  double tot = 0.0;
  for (size_t k = 0; k < st->ev_start.size(); ++k) {
    HIP_TRY(hipEventSynchronize(st->ev_stop[k]));
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, st->ev_start[k], st->ev_stop[k]));
    tot += ms;
    st->ev_pool.push_back(st->ev_start[k]);
    st->ev_pool.push_back(st->ev_stop[k]);
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = static_cast<int>(st->n_launch);
  st->n_launch = 0;
  st->ev_start.clear();
  st->ev_stop.clear();
  return RTX_OK;
}

}  // extern "C"
