// rtx_fused.h — fused shadow walks on the wavefront path (DESIGN.md §4
// "Fused shadow walks").  Included by rtx_render.hip after the lane state,
// the query lists and the sample claim.
//
// A frame whose lights are all point / directional lights (and that has no
// overlapping media and no adaptive termination) runs this state machine
// instead of advance_lane:
//   * at a closest hit the lane evaluates Material::shade's light loop
//     (material.cpp:34-69) for every light at once and appends one next-hit
//     record per light whose term can be non-zero — the shadow ray of
//     shadowAttenuation / srsAttenuation (light.cpp:16-53);
//   * trace_kernel<Q_NEXT, FUSED> runs each record's whole walk (hit after
//     hit, walk_hit below) in the same persistent launch and writes the
//     light's finished term dattn * sattn * color * (d + s) to a per-(light,
//     slot) buffer — no round trip through the lane state per hit;
//   * the lane does not wait for its terms: it pushes the hit's reflection /
//     refraction rays (with m_out = air and no adaptive termination they do
//     not depend on the colour), pops the next ray and issues its closest
//     query in the same step.  The hit's colour W * (i_out + terms) is added
//     at the start of the lane's next step, before anything else reaches the
//     sample's sum, so the sum's order — and every bit of it — is the
//     sequential machine's (the terms are added to i_out in light order).
// The tail kernel runs the same machine, each lane walking its own records
// (tail_fused_kernel).
#pragma once

#define Q_WAIT 3  // no query: the lane waits one iteration for its shadow terms

// next-hit record of a fused walk, field-major in the group's next list.
// The query ray is derived, not stored: the direction is light_dir(light,
// origin) and the bounds are shadow_bounds' (what the emitter computes).
enum {
  QF_PX = 0, QF_PY, QF_PZ,           // walk origin: the shading point backed up (light.cpp:13, 28)
  QF_DATTN, QF_SCX, QF_SCY, QF_SCZ,  // distanceAttenuation, d_comp + s_comp
  QF_WPX, QF_WPY, QF_WPZ,            // after a hit: the walk's moved origin (light.cpp:37)
  QF_SAX, QF_SAY, QF_SAZ,            //   sattn so far
  QF_LAST,                           //   t of the last hit
  QF_D
};
#define QF_I 2  // ints: 0 -1 before the walk's first hit (else the last hit's object), 1 the walk's code

// Area lights (AreaLight::shadowAttenuation, light.cpp:76-87): an area or spot
// light's shadow attenuation is (1 + the srsAttenuation walks toward its
// valid picks, in pick order) / (softShadowRes - 1), so each pick is a walk
// record of its own, and the light's term is formed when the hit's colour is
// flushed (flush_terms), from the picks' attenuations and the factors the
// shading left (dattn, d + s, and mode 1: a spot light whose cone misses the
// hit, term dattn * 0 * color * (d + s)).  A record's code is its light, with
// pick + 1 in bits 8 and up (0: a point or directional light's walk).
__device__ __forceinline__ int walk_code(int li, int pick) { return li | ((pick + 1) << 8); }
__device__ __forceinline__ int walk_light(int code) { return code & 255; }
__device__ __forceinline__ int walk_pick(int code) { return (code >> 8) - 1; }
// the walk's direction: toward the light (getDirection, light.cpp:59, :73),
// or toward the pick (glm::normalize(lpos - pb), light.cpp:84)
__device__ __forceinline__ dvec3 walk_dir(const DevScene& S, int code, const dvec3& pb) {
  const int li = walk_light(code), pick = walk_pick(code);
  if (pick < 0) return light_dir(S.lights[li], pb);
  return rtm::normalize(ld3(S.picks + (size_t(li) * S.ss_res + pick) * 3) - pb);
}

struct WalkState {
  dvec3 wpos, sattn;
  double last_t;
};

// One hit of srsAttenuation's sorted walk (light.cpp:30-50) toward a point
// or directional light with m_out = air (what ST_WALK + walk_on do on the
// sequential machine).  true: the walk is over and res is its attenuation.
__device__ __forceinline__ bool walk_hit(const DevScene& S, const RtxLight& L, const dvec3& pb, const dvec3& sdir,
                                         bool have, double bt, int bobj, int bsub, WalkState& w, dvec3& res) {
  if (!have) {
    res = w.sattn;
    return true;
  }
  const double t = bt - w.last_t;
  w.last_t = bt;
  w.wpos = rtm::ray_at(w.wpos, sdir, t);
  // sattnLimitCheck with the relative t (U14); directional lights never trip it
  if (L.type == RTX_LIGHT_POINT && rtm::dot(ld3(L.pos) - rtm::ray_at(w.wpos, sdir, t), sdir) <= 0) {
    res = w.sattn;
    return true;
  }
  if (L.type >= RTX_LIGHT_AREA_RECT) {
    // AreaLight::sattnLimitCheck (light.cpp:88-95): past the light's impact
    // point — the walk ray's crossing of the light's plane (impact,
    // light.cpp:101-105), for a disc or spot light (0, 0, 0) when it falls
    // outside the radius (light.cpp:133-141)
    const dvec3 ori = ld3(L.orient), lpos = ld3(L.pos);
    double ti = rtm::dot(ori, sdir);
    ti = rtm::dot(lpos - w.wpos, ori) / ti;
    dvec3 imp = rtm::ray_at(w.wpos, sdir, ti);
    if (L.type != RTX_LIGHT_AREA_RECT && !(rtm::dot(imp - lpos, imp - lpos) < (L.radius * L.radius)))
      imp = mk3(0.0, 0.0, 0.0);
    if (rtm::dot(imp - rtm::ray_at(w.wpos, sdir, t), sdir) <= 0) {
      res = w.sattn;
      return true;
    }
  }
  // An object opaque to walks (not transmissive, kt a constant 0, no
  // per-vertex materials): entered from outside the walk returns 0; left
  // from inside, sattn *= 0^t = +0 (t > 0) and, every kt in [0, 1]
  // (skip_dark), every later factor keeps it +0 — the walk's answer is +0
  // either way, so it ends here without the hit's normal (resolve_hit's
  // dependent loads) or its remaining queries.
  if (S.skip_dark && t > 0.0 && S.objs[bobj].pad[RTX_OBJ_WOPAQUE]) {
    res = mk3(0.0, 0.0, 0.0);
    return true;
  }
  const HitRef R = resolve_hit(S, pb, sdir, bobj, bsub, nullptr, nullptr);
  const bool is_inside = rtm::dot(R.N, sdir) > 0;
  const bool next_trans = is_inside ? true : ((hit_flags(S, R) & RTX_MF_TRANS) != 0);
  if (!next_trans) {
    res = mk3(0.0, 0.0, 0.0);
    return true;
  }
  const dvec3 kt = is_inside ? hit_param(S, R, RTX_P_KT) : mk3(1.0, 1.0, 1.0);
  w.sattn *= rtm::pow3(kt, t);
  return false;
}


// the group's next-hit list and its append counter
struct WalkEmit {
  QList q;
  unsigned int* cnt;
  int fixed_base;  // >= 0 (tail kernel): record (slot - fixed_base) * nrec + rec, no append
  int nrec;
};

// Append a walk record for the lanes with `on` (wave-aggregated: one atomic
// per call per wave, offsets by mbcnt).  Called from divergent code: the
// ballot covers the lanes executing it, the lowest of them claims.
// (rec: the record's index among the slot's nrec, for the tail's fixed
// positions; factors: a point or directional light's walk, whose record
// carries dattn and d + s — an area pick's walk needs neither)
__device__ __forceinline__ void emit_walk(const WalkEmit& E, bool on, int slot, int rec, int code, const dvec3& pb,
                                          double dattn, const dvec3& dscomp, bool factors = true) {
  size_t k;
  if (E.fixed_base >= 0) {
    if (!on) return;
    k = static_cast<size_t>(slot - E.fixed_base) * E.nrec + rec;
  } else {
    const unsigned long long m = __ballot(on);
    if (!on) return;
    const int leader = __builtin_ctzll(m);
    const int lane = threadIdx.x & 63;
    unsigned int base = 0;
    if (lane == leader) base = atomicAdd(E.cnt, static_cast<unsigned int>(__popcll(m)));
    base = __shfl(base, leader);
    k = base + lane_prefix(m);
  }
  const size_t cap = E.q.cap;
  k = RTX_CHK(CHK_QREC, k, cap);
  double* d = E.q.d;
  d[QF_PX * cap + k] = pb.x;
  d[QF_PY * cap + k] = pb.y;
  d[QF_PZ * cap + k] = pb.z;
  if (factors) {
    d[QF_DATTN * cap + k] = dattn;
    d[QF_SCX * cap + k] = dscomp.x;
    d[QF_SCY * cap + k] = dscomp.y;
    d[QF_SCZ * cap + k] = dscomp.z;
  }
  E.q.iv[0 * cap + k] = -1;
  E.q.iv[1 * cap + k] = code;
  E.q.slot[k] = slot;
}
// a walk that ended: a point or directional light's term dattn * sattn *
// color * (d + s) (material.cpp:62), or an area pick's attenuation
// (rtx_fused.h "Area lights"), into its wterm unit
__device__ __forceinline__ void walk_store(double* wterm, const int* lunit, size_t n, size_t slot, int code,
                                           const RtxLight& L, double dattn, const dvec3& dsc, const dvec3& res) {
  const int li = walk_light(code), pick = walk_pick(code);
  double* o = wterm + (static_cast<size_t>(lunit[li] + (pick < 0 ? 0 : 2 + pick)) * n + slot) * 3;
  const dvec3 v = pick < 0 ? dattn * res * ld3(L.color) * dsc : res;
  o[0] = v.x;
  o[1] = v.y;
  o[2] = v.z;
}

// colour c into bucket pos of the lane's sample (the root's bucket is acc)
__device__ __forceinline__ void contrib_at(LaneRef& LR, const FrameParams& F, int pos, const dvec3& c) {
  if (F.fork_on && pos >= 2) bucket_add(F, LR.bunit(), pos, c);
  else LR.acc() += c;
}

// The deferred colour of the lane's last hit: W * (i_out + its lights'
// terms in light order) (material.cpp:45-66, RayTracer.cpp:125).  An area or
// spot light's term is formed here from its picks' attenuations in pick
// order (AreaLight::shadowAttenuation, light.cpp:76-87, as ST_SRS sums them).
__device__ __forceinline__ void flush_terms(LaneRef& LR, const FrameParams& F, const DevScene& S) {
  unsigned int m = static_cast<unsigned int>(LR.wmask());
  if (!m) return;
  dvec3 col = LR.i_out();
  const size_t n = LR.m.n;
  while (m) {
    const int l = __builtin_ctz(m);
    m &= m - 1;
    const double* u = F.wterm + (size_t(F.lunit[l]) * n + LR.g) * 3;
    if (!((F.area_mask >> l) & 1)) {
      col += ld3(u);
      continue;
    }
    const double dattn = u[0];
    const dvec3 dsc = mk3(u[1], u[2], u[n * 3]);
    const RtxLight& L = S.lights[l];
    if (u[n * 3 + 1] != 0.0) {  // a spot light whose cone misses the hit (light.cpp:147-149)
      col += dattn * mk3(0.0, 0.0, 0.0) * ld3(L.color) * dsc;
      continue;
    }
    dvec3 sa = mk3(1.0, 1.0, 1.0);
    for (int i = 0; i < S.ss_res; ++i) sa += ld3(u + size_t(2 + i) * n * 3);  // (invalid picks hold +0)
    sa *= (1.0 / (S.ss_res - 1));
    col += dattn * sa * ld3(L.color) * dsc;
  }
  contrib_at(LR, F, LR.rpos(), LR.W() * col);
  LR.wmask() = 0;
}

// pending-ray entry of lane g: pbuf[(e * 13 + f) * nlanes + g] (advance_lane)
__device__ __forceinline__ void fused_put_entry(double* b, size_t nlanes, const dvec3& p, const dvec3& d, const dvec3& w,
                                                const dvec3& k, int depth, int kind, int pos) {
  b[0 * nlanes] = p.x; b[1 * nlanes] = p.y; b[2 * nlanes] = p.z;
  b[3 * nlanes] = d.x; b[4 * nlanes] = d.y; b[5 * nlanes] = d.z;
  b[6 * nlanes] = w.x; b[7 * nlanes] = w.y; b[8 * nlanes] = w.z;
  b[9 * nlanes] = k.x; b[10 * nlanes] = k.y; b[11 * nlanes] = k.z;
  b[12 * nlanes] = pend_code(pos, depth, kind);
}
__device__ __forceinline__ void fused_push(LaneRef& LR, double* pbuf, size_t nlanes, const dvec3& p, const dvec3& d,
                                           const dvec3& w, const dvec3& k, int depth, int kind, int pos) {
  fused_put_entry(pbuf + static_cast<size_t>(LR.top()) * 13 * nlanes + LR.g, nlanes, p, d, w, k, depth, kind, pos);
  ++LR.top();
}
// child node at heap position cpos: its sub-tree on a fork slot, if one is
// free (same buckets, same sums as on the own stack); false: the own stack
template <bool FORK>
__device__ __forceinline__ bool fused_fork_child(LaneRef& LR, const ForkCtx* fk, double* pbuf, size_t nlanes,
                                                 const dvec3& p, const dvec3& d, const dvec3& w, const dvec3& k,
                                                 int depth, int kind, int cpos) {
  if (!FORK) return false;
  const int T = fork_claim(fk, cpos >= 2 && fk->spare_n != 0);
  if (T < 0) return false;
  LaneRef LT(LR.m, static_cast<size_t>(T));
  fused_put_entry(pbuf + static_cast<size_t>(T), nlanes, p, d, w, k, depth, kind, cpos);
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
  LT.wmask() = 0;
  LT.st() = ST_POP;
  fork_join(fk, T);
  return true;
}

// traceRay after scene->intersect (RayTracer.cpp:116-165) and
// Material::shade (material.cpp:34-69) for the ray in pending entry `top`
// with the closest hit (have, bt, bobj, bsub): the hit record, the colour
// (now, or deferred until the walks' terms are in), the walk records, the
// reflection / refraction pushes.  Leaves the lane in ST_POP.  Run by
// trace_kernel<Q_CLOSEST, FUSED> right where a query completes (walks
// appended to the group's next list) and by the tail kernel (walks at the
// slot's own record positions, walked by the same lane).
// The ray of a closest query: pending-stack entry `top` (or, for a sample's
// first camera ray in the first iteration, regenerated: cam_first_ray).
struct QRay {
  dvec3 p, d, W;
  int64_t code;
};
__device__ __forceinline__ QRay qray_at(const LaneRef& LR, const double* __restrict__ pbuf, size_t nlanes) {
  const double* b = pbuf + static_cast<size_t>(LR.top()) * 13 * nlanes + LR.g;
  QRay r;
  r.p = mk3(b[0 * nlanes], b[1 * nlanes], b[2 * nlanes]);
  r.d = mk3(b[3 * nlanes], b[4 * nlanes], b[5 * nlanes]);
  r.W = mk3(b[6 * nlanes], b[7 * nlanes], b[8 * nlanes]);
  r.code = static_cast<int64_t>(b[12 * nlanes]);
  return r;
}

template <bool STATS, bool FORK>
__device__ __forceinline__ void shade_hit(LaneRef& LR, const DevScene& S, const FrameParams& F, Counters& C,
                                          RtxHitRecord* __restrict__ hits, double* __restrict__ pbuf, size_t nlanes,
                                          int pend_cap, const ForkCtx* fk, const WalkEmit* we, const QRay& qr,
                                          bool have, double bt, int bobj, int bsub) {
  const RtxRenderParams& P = F.P;
  const double* b = pbuf + static_cast<size_t>(LR.top()) * 13 * nlanes + LR.g;
  const dvec3 rp = qr.p;
  const dvec3 rd = qr.d;
  dvec3 W = qr.W;
  const int64_t code = qr.code;
  const int dk = static_cast<int>((code & ((int64_t(1) << 40) - 1)) - (int64_t(1) << 39));
  const int pos = static_cast<int>(code >> 40);
  const int rdepth = dk >= 0 ? dk / 4 : -((-dk + 3) / 4);
  const int rkind = dk - rdepth * 4;
  LR.st() = ST_POP;
  if (LR.first_query()) {
    LR.first_query() = false;
    if (have) {
      RtxHitRecord* hr = &hits[LR.sample_slot()];
      const RtxObject& o = S.objs[bobj];
      hr->object = o.orig_id;
      hr->scene_leaf = o.leaf;
      hr->t = bt;
      if (o.type == RTX_OBJ_TRIMESH) {
        const RtxFaceIds fi = S.fids[o.pad[RTX_OBJ_FACE_OFF] + bsub];
        hr->face = fi.orig_id;
        hr->mesh_leaf = fi.leaf;
      }
    }
  }
  if (!have) {  // miss: the cube map's colour, else black (RayTracer.cpp:167-169; U3)
    if (S.cube[0] >= 0) contrib_at(LR, F, pos, W * cube_color(S, rd));
    return;
  }
  if (rkind != 0) {  // the parked kt factor of a child ray (RayTracer.cpp:140-158)
    const dvec3 ktf = mk3(b[9 * nlanes], b[10 * nlanes], b[11 * nlanes]);
    if (rkind == 1)
      W = W * rtm::gmax3(rtm::gmin3(rtm::pow3(ktf, bt), rtm::splat3(1.0)), rtm::splat3(0.0));
    else
      W = W * rtm::pow3(ktf, bt);
  }
  const HitRef R = resolve_hit(S, rp, rd, bobj, bsub, nullptr, nullptr);
  const dvec3 N = R.N;
  const int flags = hit_flags(S, R);
  if (STATS) C.shades++;
  // Material::shade (material.cpp:34-69)
  dvec3 i_out = hit_param(S, R, RTX_P_KE) + hit_param(S, R, RTX_P_KA) * mk3(S.ambient[0], S.ambient[1], S.ambient[2]);
  {
    const dvec3 kd = hit_param(S, R, RTX_P_KD), ks = hit_param(S, R, RTX_P_KS);
    const double sh = hit_shininess(S, R);
    const dvec3 X = rtm::ray_at(rp, rd, bt);
    const dvec3 pb = X - rd * RTX_EPS_BACKUP;
    unsigned int wm = 0;
    int nr = 0;
    for (int li = 0; li < S.n_lights; ++li) {
      const RtxLight& L = S.lights[li];
      const dvec3 l_i = light_dir(L, X);
      const dvec3 l_r = (l_i - 2 * (rtm::dot(l_i, N)) * N);
      double dt = rtm::dot(l_i, N);
      if (flags & RTX_MF_TRANS) dt = fabs(dt);
      const dvec3 d_comp = kd * rtm::gmax(0.0, dt);
      const dvec3 s_comp = ks * rtm::splat3(rtm::rpow(rtm::gmax(0.0, rtm::dot(l_r, rd)), sh));
      const dvec3 dscomp = d_comp + s_comp;
      const double dattn = light_dist_atten(L, X);
      if (L.type >= RTX_LIGHT_AREA_RECT) {
        // AreaLight::shadowAttenuation (light.cpp:76-87): a walk per valid
        // pick; the term is formed in flush_terms from the factors here
        double* u = F.wterm + (size_t(F.lunit[li]) * nlanes + LR.g) * 3;
        u[0] = dattn;
        u[1] = dscomp.x;
        u[2] = dscomp.y;
        u[nlanes * 3] = dscomp.z;
        const dvec3 ori = ld3(L.orient), lpos = ld3(L.pos);
        // SpotLight::validImpact(r, p) at the hit (light.cpp:144-146)
        const bool cone = L.type != RTX_LIGHT_SPOT ||
                          ((rtm::dot(light_dir(L, X), ori) <= 0) &&
                           (rtm::dot(rtm::normalize(X - (lpos - L.offset * ori)), ori) > S.cos45));
        u[nlanes * 3 + 1] = cone ? 0.0 : 1.0;
        wm |= 1u << li;
        if (!cone) continue;
        for (int i = 0; i < S.ss_res; ++i) {
          const dvec3 lp = ld3(S.picks + (size_t(li) * S.ss_res + i) * 3);
          // validImpact(r, pb, lp) (light.cpp:147-149; always for rect / disc)
          const bool valid = L.type != RTX_LIGHT_SPOT ||
                             ((rtm::dot(light_dir(L, pb), ori) <= 0) && (rtm::dot(rtm::normalize(pb - lp), ori) > S.cos45));
          if (STATS && valid) {
            C.shadow++;
            C.shadow_traced++;
          }
          if (valid) ++nr;
          emit_walk(*we, valid, static_cast<int>(LR.g), F.lrec[li] + i, walk_code(li, i), pb, 0.0, dscomp, false);
          if (!valid) {  // no walk: the pick adds +0 (ST_SRS skips it)
            double* o = u + size_t(2 + i) * nlanes * 3;
            o[0] = o[1] = o[2] = 0.0;
            if (we->fixed_base >= 0)  // (the tail's fixed record: marked, not walked)
              we->q.iv[1 * we->q.cap + static_cast<size_t>(LR.g - we->fixed_base) * we->nrec + F.lrec[li] + i] = -1;
          }
        }
        continue;
      }
      if (STATS) C.shadow++;
      ++nr;
      // a zero colour factor with finite attenuations adds +0 (DESIGN.md:
      // dark lights are counted, not traced)
      const bool on = !(S.skip_dark && dscomp.x == 0.0 && dscomp.y == 0.0 && dscomp.z == 0.0);
      if (STATS && on) C.shadow_traced++;
      emit_walk(*we, on, static_cast<int>(LR.g), F.lrec[li], walk_code(li, -1), pb, dattn, dscomp);
      if (on) wm |= 1u << li;
    }
    LR.nrays() += nr;
    if (wm == 0) {
      contrib_at(LR, F, pos, W * i_out);
    } else {  // colorC = W * shade(...) once the terms are in (flush_terms)
      LR.W() = W;
      LR.i_out() = i_out;
      LR.wmask() = static_cast<int>(wm);
      LR.rpos() = pos;
    }
  }
  // recursion (RayTracer.cpp:127-164), m_out = air; no adaptive termination
  // on this path, so it does not wait for the colour
  const int depth = rdepth - 1;
  if (!((flags & RTX_MF_RECUR) && depth > 0)) return;
  const bool leaving = rtm::dot(N, rd) >= 0;
  const bool next_trans = leaving ? true : (flags & RTX_MF_TRANS) != 0;
  const dvec3 normal = (leaving ? -1.0 : 1.0) * N;
  const double c = -1 * rtm::dot(normal, rd);
  const double eta =
      next_trans ? (leaving ? hit_index(S, R) : S.air_index) / (leaving ? S.air_index : hit_index(S, R)) : 0;
  const double radicand = 1 - eta * eta * (1 - c * c);
  const bool tir = next_trans && radicand < 0;
  // buckets of the children: their own heap positions when they are nodes
  // (this ray is a node above the fork depth), else this ray's
  const bool node = pos > 0 && P.depth - rdepth == ilog2i(pos);
  const int node_refl = node && 2 * pos < F.fork_npos + 2 ? 2 * pos : 0;
  const int node_refr = node && 2 * pos + 1 < F.fork_npos + 2 ? 2 * pos + 1 : 0;
  // the unit's bucket set, taken by its root before the first child exists
  if (F.fork_on && pos == 1)
    bucket_alloc(F, LR.bunit(), (node_refl || node_refr) && ((next_trans && !tir) || (flags & RTX_MF_REFL) || tir));
  // push refraction first so that reflection is traced first (the entry at
  // `top` is this ray's own, read above: it is overwritten)
  // (a child that neither forks nor fits on the stack can only happen with
  // the two-entry stacks of rtx_render's low_stack rule: flagged, *bover bit 2)
  if (next_trans && !tir) {
    const dvec3 tp = rtm::ray_at(rp, rd, bt + RTX_RAY_EPS);
    const dvec3 td = eta * rd + (eta * c - sqrt(radicand)) * normal;
    const dvec3 kf = leaving ? mk3(1.0, 1.0, 1.0) : hit_param(S, R, RTX_P_KT);
    if (!fused_fork_child<FORK>(LR, fk, pbuf, nlanes, tp, td, W, kf, depth, 2, node_refr)) {
      if (LR.top() < pend_cap) fused_push(LR, pbuf, nlanes, tp, td, W, kf, depth, 2, node_refr ? node_refr : pos);
      else if (F.bover) atomicOr(F.bover, 4u);
    }
    if (STATS) C.secondary++;
  }
  if ((flags & RTX_MF_REFL) || tir) {
    const dvec3 rdir = rd + 2 * c * normal;
    const dvec3 rs = rtm::ray_at(rp, rd, bt - RTX_RAY_EPS);
    const dvec3 wr = W * hit_param(S, R, RTX_P_KR);
    const dvec3 kf = leaving ? hit_param(S, R, RTX_P_KT) : mk3(1.0, 1.0, 1.0);
    if (!fused_fork_child<FORK>(LR, fk, pbuf, nlanes, rs, rdir, wr, kf, depth, 1, node_refl)) {
      if (LR.top() < pend_cap) fused_push(LR, pbuf, nlanes, rs, rdir, wr, kf, depth, 1, node_refl ? node_refl : pos);
      else if (F.bover) atomicOr(F.bover, 4u);
    }
    if (STATS) C.secondary++;
  }
}

// What trace_kernel<Q_CLOSEST, FUSED> needs to shade a completed query.
struct ShadeArgs {
  const FrameParams* Fp;
  RtxHitRecord* hits;
  double* pbuf;
  int pend_cap;
  QList qn;        // the group's next list (walk records)
  int slot_off;    // the group's first slot
  int* live_out;   // this iteration's live list (forked slots join it)
  int out_cnt;     // its counter
  int cam_n;       // > 0: the first iteration — query k is the first camera
                   // ray of the group's slot k (cam_first_claim), k < cam_n
  int leaf_k;      // object / leaf units wait while >= leaf_k lanes are at a
                   // record (trace_kernel; 65: never)
  const int* free_ids;  // the group's free fork slots (advance_fused_kernel pushes them)
  int* ovf;        // the group's stack overflow columns (StackShort), one per thread of the launch
  int lds_k;       // StackShort: stack entries per lane in LDS
};

// Camera ray k of the sample at (sx, sy), eye pass `pass` (trace(),
// RayTracer.cpp:35-79: k = 0 the pinhole ray, k >= 1 the DoF lens rays).
__device__ __forceinline__ void camera_ray(const FrameParams& F, int pass, int k, double sx, double sy, dvec3& rp,
                                           dvec3& rd) {
  const RtxRenderParams& P = F.P;
  const RtxCamera& cam = F.cam;
  const dvec3 eye = pass ? ld3(cam.eye) + mk3(0.25, 0.0, 0.0) : ld3(cam.eye);
  const double x = sx - 0.5, y = sy - 0.5;
  const dvec3 cdir = rtm::normalize(ld3(cam.look) + x * ld3(cam.u) + y * ld3(cam.v));
  rp = eye;
  rd = cdir;
  if (k > 0) {
    const double fd = rtm::gmax(P.dof_fd, 1.0);
    const dvec3 fp_n = -cdir;
    const dvec3 fp_pt = rtm::ray_at(eye, cdir, fd);
    double t = rtm::dot(fp_n, cdir);
    t = rtm::dot(fp_pt - eye, fp_n) / t;
    const dvec3 dest = rtm::ray_at(eye, cdir, t);
    rp = eye + ld3(&F.offv[(k - 1) * 3]);
    rd = rtm::normalize(dest - rp);
  }
}
// ST_CAM's next camera ray: the ray, the hit-record default of a sample's
// first ray, camk advanced
__device__ __forceinline__ void cam_start(LaneRef& LR, const FrameParams& F, RtxHitRecord* __restrict__ hits,
                                          dvec3& rp, dvec3& rd) {
  const int k = LR.camk();
  camera_ray(F, LR.pass(), k, LR.sx(), LR.sy(), rp, rd);
  if (k == 0) {
    LR.first_query() = LR.rec_on() && LR.pass() == 0;
    if (LR.first_query()) {  // default record: miss (also what depth < 0 leaves)
      RtxHitRecord* hr = &hits[LR.sample_slot()];
      hr->object = hr->face = hr->scene_leaf = hr->mesh_leaf = -1;
      hr->t = 1000.0;
      hr->pad = 0;
    }
  } else {
    LR.first_query() = false;
  }
  LR.camk() = k + 1;
}

// First iteration of a fused frame (trace_kernel<Q_CLOSEST, FUSED> with
// cam_n > 0): the kernel claims the slot's first sample itself and queries
// its first camera ray straight away — what advance_fused (claim, ST_CAM,
// ST_POP) would have done, without the pending-stack entry and the query
// record round trip.  False: the slot has no sample (left idle).
// (only in the first iteration's instantiation of the closest-hit kernel,
// trace_kernel<..., CAM = true>; inlined there since the cold traversal state
// moved to LDS, out of line — cam_first_claim — in the instantiations the
// backend fails on inlined, "Subtarget requires even aligned vector
// registers")
// (the out-of-line version takes its arguments by value: a reference would
// put the caller's LaneRef and counters in scratch for the call)
__device__ __forceinline__ bool cam_first_claim_inl(const LaneMem lm, int slot, const FrameParams& F,
                                                   RtxHitRecord* __restrict__ hits) {
  LaneRef LR(lm, static_cast<size_t>(slot));
  lane_init(LR);
  claim_sample(LR, F, hits, slot);
  if (LR.st() == ST_IDLE) return false;
  // ST_CAM's bookkeeping (the hit record's default, camk); the caller forms
  // the ray itself (cam_first_ray)
  dvec3 rp, rd;
  cam_start(LR, F, hits, rp, rd);
  LR.top() = 0;     // the ray's own entry (never written: shading overwrites it with the children)
  LR.nrays()++;     // ST_POP
  LR.qmode() = Q_CLOSEST;
  LR.st() = ST_HIT;
  return true;
}
__device__ __noinline__ bool cam_first_claim(const LaneMem lm, int slot, const FrameParams& F,
                                             RtxHitRecord* __restrict__ hits) {
  return cam_first_claim_inl(lm, slot, F, hits);
}
// its ray again at shading time (the walk's registers are reused meanwhile)
__device__ __forceinline__ QRay cam_first_ray(const LaneRef& LR, const FrameParams& F) {
  QRay qr;
  camera_ray(F, LR.pass(), LR.camk() - 1, LR.sx(), LR.sy(), qr.p, qr.d);
  qr.W = mk3(1.0, 1.0, 1.0);
  qr.code = static_cast<int64_t>(pend_code(F.fork_on ? 1 : 0, F.P.depth, 0));
  return qr;
}

// The fused state machine (CAM -> POP): runs until the lane needs a
// closest-hit query (Q_CLOSEST: the ray is pending-stack entry `top`), has to
// wait for its terms (Q_WAIT) or its sample is finished (ST_IDLE).  The hit
// is shaded by whoever runs the query (trace_kernel<Q_CLOSEST, FUSED>, the
// tail kernel): the lane comes back in ST_POP.
template <bool STATS, bool FORK>
__device__ __forceinline__ void advance_fused(LaneRef& LR, const DevScene& S, const FrameParams& F, Counters& C,
                                              double* __restrict__ sbuf, RtxHitRecord* __restrict__ hits,
                                              double* __restrict__ pbuf, size_t nlanes, int pend_cap) {
  const RtxRenderParams& P = F.P;
  LR.qmode() = Q_NONE;
  while (LR.st() != ST_IDLE && LR.qmode() == Q_NONE) {
    LR.refresh();
    switch (LR.st()) {
      case ST_CAM: {
        // next camera ray of trace(x, y) (RayTracer.cpp:35-79)
        if (LR.camk() == LR.cam_end()) {
          if (LR.wmask()) {  // the last hit's colour belongs to this sum
            LR.qmode() = Q_WAIT;
            break;
          }
          if (LR.fpos() != 0) {  // a forked sub-tree: sums in its buckets, rays join the sample's count
            if (LR.rec_on()) atomicAdd(&hits[LR.sample_slot()].nrays, LR.nrays());
            LR.fpos() = 0;
            LR.st() = ST_IDLE;
            break;
          }
          if (F.cam_split) {  // one camera ray of a DoF sample: its own sum (reduce_kernel scales, clamps)
            const int64_t u = RTX_CHK(CHK_SAMPLE, static_cast<int64_t>(LR.sample_slot()) * F.ncam + (LR.cam_end() - 1),
                                      F.chk_samples * F.ncam);
            sbuf[u * 3 + 0] = LR.acc().x;
            sbuf[u * 3 + 1] = LR.acc().y;
            sbuf[u * 3 + 2] = LR.acc().z;
            if (LR.rec_on()) atomicAdd(&hits[LR.sample_slot()].nrays, LR.nrays() + (LR.cam_end() == 1 ? 1 : 0));
            LR.st() = ST_IDLE;
            break;
          }
          if (F.fork_on) {  // the root's sum; reduce_kernel adds the buckets, then clamps
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
          double* out = sbuf + static_cast<int64_t>(LR.sample_slot()) * 3;
          if (P.anaglyph && LR.pass() == 0) {  // tracePixel (RayTracer.cpp:92-99): park pass 0
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
        dvec3 rp, rd;
        cam_start(LR, F, hits, rp, rd);
        if (STATS) C.camera++;
        LR.top() = 0;
        fused_push(LR, pbuf, nlanes, rp, rd, mk3(1, 1, 1), mk3(1, 1, 1), P.depth, 0, F.fork_on ? 1 : 0);
        LR.st() = ST_POP;
        break;
      }
      case ST_POP: {
        if (LR.top() == 0) {
          LR.st() = ST_CAM;
          break;
        }
        const double* b = pbuf + static_cast<size_t>(LR.top() - 1) * 13 * nlanes + LR.g;
        const int64_t code = static_cast<int64_t>(b[12 * nlanes]);
        const int dk = static_cast<int>((code & ((int64_t(1) << 40) - 1)) - (int64_t(1) << 39));
        const int pdepth = dk >= 0 ? dk / 4 : -((-dk + 3) / 4);
        if (pdepth < 0) {  // `depth >= 0 &&` (RayTracer.cpp:116): no query, the miss colour
          if (S.cube[0] >= 0) {
            if (LR.wmask()) {
              LR.qmode() = Q_WAIT;
              break;
            }
            contrib_at(LR, F, static_cast<int>(code >> 40),
                       mk3(b[6 * nlanes], b[7 * nlanes], b[8 * nlanes]) *
                           cube_color(S, mk3(b[3 * nlanes], b[4 * nlanes], b[5 * nlanes])));
          }
          --LR.top();
          LR.nrays()++;
          break;
        }
        --LR.top();
        LR.nrays()++;
        LR.qmode() = Q_CLOSEST;  // the ray stays in entry `top` until its hit is shaded
        LR.st() = ST_HIT;
        break;
      }
      default:
        LR.st() = ST_IDLE;
        break;
    }
  }
}

// One step of every live slot of a group on a fused frame: add the last
// hit's colour, then run the machine to the next closest query (appended to
// q0 with ballot + popc + mbcnt, the ray read from the slot's pending stack)
// while walks go to q1 as they are found.
template <bool STATS, bool FORK>
__global__ void __launch_bounds__(WG, STATS ? 1 : RTX_ADV_WAVES)
    advance_fused_kernel(DevScene S, const DevScene* __restrict__ Sg, const FrameParams* __restrict__ Fp, LaneMem lm,
                         double* __restrict__ sbuf, RtxHitRecord* __restrict__ hits, double* __restrict__ pbuf,
                         int pend_cap, QList q0, QList q1, unsigned int* __restrict__ counters,
                         unsigned long long* __restrict__ stats, int slot_off, const int* __restrict__ live_in,
                         int* __restrict__ live_out, int first, int in_cnt, int out_cnt, int* __restrict__ free_ids) {
  const FrameParams& F = *Fp;
  const int tid = blockIdx.x * WG + threadIdx.x;
  // first: 1 every slot of the group, initialised here; 2 every slot (the
  // iteration after the first closest-hit launch claimed the samples, which
  // keeps no live list); 0 the live list
  const bool valid = first == 1 || (first == 2 ? tid < F.wf_gs : tid < static_cast<int>(counters[in_cnt]));
  const int slot = first ? slot_off + (valid ? tid : 0) : (valid ? live_in[tid] : slot_off);
  const int lane = threadIdx.x & 63;
  Counters C = {0, 0, 0, 0, 0, 0, 0};
  LaneRef L(lm, static_cast<size_t>(slot));
  if (first == 1) lane_init(L);
  int qm = Q_NONE;
  // a fork slot (past the group's sample slots) running a sub-tree
  const bool was_fork = FORK && valid && slot - slot_off >= F.wf_gsamp && L.st() != ST_IDLE;
  if (valid && (L.st() != ST_IDLE || slot_unit(F, slot, L.kdone()) >= 0)) {
    flush_terms(L, F, *Sg);
    L.qmode() = Q_NONE;
    for (;;) {
      claim_sample(L, F, hits, slot);
      if (L.st() == ST_IDLE) break;
      advance_fused<STATS, FORK>(L, *Sg, F, C, sbuf, hits, pbuf, lm.n, pend_cap);
      if (L.qmode() != Q_NONE) break;
    }
    qm = L.qmode();
  }
  const unsigned long long mask = __ballot(qm == Q_CLOSEST);
  if (mask) {
    unsigned int base = 0;
    if (lane == 0) base = atomicAdd(&counters[CNT_Q], static_cast<unsigned int>(__popcll(mask)));
    base = __shfl(base, 0);
    if (qm == Q_CLOSEST) {
      const size_t cap = q0.cap, n = lm.n;
      const size_t k = RTX_CHK(CHK_QREC, base + lane_prefix(mask), cap);
      const double* b = pbuf + static_cast<size_t>(RTX_CHK(CHK_PEND, L.top(), pend_cap)) * 13 * n + slot;
      q0.slot[k] = slot;
      q0.d[0 * cap + k] = b[0 * n];
      q0.d[1 * cap + k] = b[1 * n];
      q0.d[2 * cap + k] = b[2 * n];
      q0.d[3 * cap + k] = b[3 * n];
      q0.d[4 * cap + k] = b[4 * n];
      q0.d[5 * cap + k] = b[5 * n];
      // (key and bounds of a closest query are constants: not stored)
    }
  }
  const bool live = valid && L.st() != ST_IDLE;  // a query pending or waiting for terms
  const unsigned long long alive = __ballot(live);
  if (alive) {
    unsigned int base = 0;
    if (lane == 0) base = atomicAdd(&counters[out_cnt], static_cast<unsigned int>(__popcll(alive)));
    base = __shfl(base, 0);
    if (live) live_out[RTX_CHK(CHK_LIVE, base + lane_prefix(alive), F.chk_live)] = slot;
  }
  if (FORK && free_ids) {
    // a fork slot whose sub-tree ended here goes on the group's free list
    // (fork_claim in the closest-hit launch reuses it: the spare slots then
    // serve more forks than there are spares)
    const bool freed = was_fork && L.st() == ST_IDLE;
    const unsigned long long fm = __ballot(freed);
    if (fm) {
      unsigned int base = 0;
      if (lane == 0) base = atomicAdd(&counters[CNT_FREE], static_cast<unsigned int>(__popcll(fm)));
      base = __shfl(base, 0);
      if (freed) free_ids[RTX_CHK(CHK_FREE, base + lane_prefix(fm), F.chk_live)] = slot;
    }
  }
  if (STATS) {
    stats_add(C, stats, lane);
  }
}

// Tail of a fused frame (see tail_kernel): each slot runs its own chain —
// closest query, shading, its walks one after the other — with one
// traversal call site, so the kernel keeps the sequential tail's register
// budget.  The walk records go to the group's next list at the slot's own
// positions (the batched iterations are over, the list is free).
template <bool STATS>
__global__ void __launch_bounds__(WG) tail_fused_kernel(DevScene S, const DevScene* __restrict__ Sg,
                                                         const FrameParams* __restrict__ Fp, LaneMem lm,
                                                         double* __restrict__ sbuf, RtxHitRecord* __restrict__ hits,
                                                         double* __restrict__ pbuf, int pend_cap,
                                                         const unsigned int* __restrict__ counters,
                                                         const int* __restrict__ live_in, int in_cnt, int stack_cap,
                                                         unsigned long long* __restrict__ stats, QList qn,
                                                         int slot_off) {
  extern __shared__ int lds_stack[];
  const FrameParams& F = *Fp;
  const int lane = threadIdx.x & 63;
  int* stk = lds_stack + (threadIdx.x >> 6) * stack_cap * 64;
  const int tid = blockIdx.x * WG + threadIdx.x;
  Counters C = {0, 0, 0, 0, 0, 0, 0};
  const bool valid = tid < static_cast<int>(counters[in_cnt]);
  const int slot = valid ? live_in[tid] : 0;
  LaneRef L(lm, static_cast<size_t>(slot));
  const DevScene& SS = *Sg;
  const WalkEmit we = {qn, nullptr, slot_off, F.nrec};
  const size_t cap = qn.cap;
  unsigned int todo = 0;  // lights whose walks are still to run (records at the slot's positions)
  int wl = -1;            // the light being walked; w: its state
  int wp = 0;             // an area light's next pick
  int wcode = 0;          // the walk's code (walk_code)
  WalkState w = {mk3(0.0, 0.0, 0.0), mk3(0.0, 0.0, 0.0), 0.0};
  dvec3 pb = mk3(0.0, 0.0, 0.0), sdir = pb;
  double tp = -RTX_INF;
  int rp = -1, sq = -1;
  if (valid) flush_terms(L, F, SS);
  while (valid) {
    int qm;
    dvec3 qP, qD;
    double qlim = RTX_INF;
    if (todo) {
      if (wl < 0) {
        // the next walk: light order, an area light's picks in pick order
        // (records marked -1 — spot picks outside the cone — are skipped, and
        // a spot light whose cone misses the hit has none)
        bool found = false;
        while (todo && !found) {
          const int l = __builtin_ctz(todo);
          if (!((F.area_mask >> l) & 1)) {
            wl = l;
            wcode = walk_code(l, -1);
            found = true;
            break;
          }
          const double* u = F.wterm + (size_t(F.lunit[l]) * lm.n + slot) * 3;
          if (u[lm.n * 3 + 1] != 0.0 || wp >= SS.ss_res) {
            todo &= todo - 1;
            wp = 0;
            continue;
          }
          if (qn.iv[1 * cap + static_cast<size_t>(slot - slot_off) * F.nrec + F.lrec[l] + wp] < 0) {
            ++wp;
            continue;
          }
          wl = l;
          wcode = walk_code(l, wp);
          found = true;
        }
        if (!found) continue;  // every walk done: the lane's next closest query
        const size_t k = static_cast<size_t>(slot - slot_off) * F.nrec + F.lrec[wl] + (walk_pick(wcode) < 0 ? 0 : wp);
        pb = mk3(qn.d[QF_PX * cap + k], qn.d[QF_PY * cap + k], qn.d[QF_PZ * cap + k]);
        sdir = walk_dir(SS, wcode, pb);
        w.wpos = pb;
        w.sattn = mk3(1.0, 1.0, 1.0);
        w.last_t = 0.0;
        tp = -RTX_INF;
        rp = -1;
        sq = -1;
      }
      qlim = shadow_limit(SS, SS.lights[wl], pb, rp < 0);
      qm = Q_NEXT;
      qP = pb;
      qD = sdir;
    } else {
      flush_terms(L, F, SS);
      L.qmode() = Q_NONE;
      claim_sample(L, F, hits, slot);
      if (L.st() == ST_IDLE) break;
      advance_fused<STATS, false>(L, SS, F, C, sbuf, hits, pbuf, lm.n, pend_cap);
      if (L.qmode() != Q_CLOSEST) continue;  // the sample is done: claim the next one
      qm = Q_CLOSEST;
      const double* b = pbuf + static_cast<size_t>(L.top()) * 13 * lm.n + slot;
      qP = mk3(b[0 * lm.n], b[1 * lm.n], b[2 * lm.n]);
      qD = mk3(b[3 * lm.n], b[4 * lm.n], b[5 * lm.n]);
      tp = -RTX_INF;
      rp = -1;
      sq = -1;
    }
    double bt;
    int bobj, bsub;
    const bool have = traverse_any<STATS>(S, qm, qP, qD, tp, rp, sq, qlim, bt, bobj, bsub, stk, lane, C);
    if (qm == Q_NEXT) {
      dvec3 res;
      if (walk_hit(SS, SS.lights[wl], pb, sdir, have, bt, bobj, bsub, w, res)) {
        if (walk_pick(wcode) < 0) {
          const size_t k = static_cast<size_t>(slot - slot_off) * F.nrec + F.lrec[wl];
          const dvec3 dsc = mk3(qn.d[QF_SCX * cap + k], qn.d[QF_SCY * cap + k], qn.d[QF_SCZ * cap + k]);
          walk_store(F.wterm, F.lunit, lm.n, slot, wcode, SS.lights[wl], qn.d[QF_DATTN * cap + k], dsc, res);
          todo &= todo - 1;
        } else {
          walk_store(F.wterm, F.lunit, lm.n, slot, wcode, SS.lights[wl], 0.0, res, res);
          ++wp;
        }
        wl = -1;
      } else {
        tp = bt;
        rp = bobj;
        sq = bsub;
      }
    } else {
      shade_hit<STATS, false>(L, SS, F, C, hits, pbuf, lm.n, pend_cap, nullptr, &we, qray_at(L, pbuf, lm.n), have, bt,
                              bobj, bsub);
      todo = static_cast<unsigned int>(L.wmask());
    }
  }
  if (STATS) {
    stats_add(C, stats, lane);
    stats_add_class(C, stats, lane, 30);
  }
}
