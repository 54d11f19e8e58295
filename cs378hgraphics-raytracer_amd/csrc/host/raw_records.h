// raw_records.h — a canonical text form of a scene's RAW parse records
// (scene_model.h): objects with their transform chains and material copies,
// meshes, lights, camera attribute ops, ambient, textures.  Both the
// product's parser (rtx_host_raw_records) and the checker's own restated
// parser (oracle/parse_restated.cpp, oracle_raw_records) print through it, so
// tests/test_oracle_parser.py can compare the two loaders record for record.
// Only a printer: no parse semantics live here.
#pragma once

#include <cstdio>
#include <string>

#include "scene_model.h"

namespace rtxh {

inline std::string dump_raw_records(const SceneModel& s) {
  std::string o;
  char b[64];
  auto d = [&](double x) {
    std::snprintf(b, sizeof(b), " %.17g", x);
    o += b;
  };
  auto f = [&](float x) {
    std::snprintf(b, sizeof(b), " %.9g", static_cast<double>(x));
    o += b;
  };
  auto i = [&](long long x) {
    std::snprintf(b, sizeof(b), " %lld", x);
    o += b;
  };
  auto v3 = [&](const dvec3& v) {
    d(v.x);
    d(v.y);
    d(v.z);
  };
  auto mat = [&](const Material& m) {
    for (int k = 0; k < P_COUNT; ++k) {
      v3(m.p[k].v);
      i(m.p[k].tex);
    }
    i(m.refl);
    i(m.trans);
    i(m.recur);
    i(m.spec);
    i(m.both);
  };
  o += "camera";
  v3(s.camera.eye);
  o += "\n";
  for (const CamOp& op : s.camera.ops) {
    o += "camop";
    i(op.kind);
    for (double x : op.v) d(x);
    o += "\n";
  }
  o += "ambient";
  v3(s.ambient);
  o += "\n";
  for (size_t k = 0; k < s.objects.size(); ++k) {
    const Object& ob = s.objects[k];
    o += "object";
    i(ob.type);
    i(ob.material);
    i(ob.mesh);
    if (ob.type == OBJ_CONE) {
      d(ob.cone_h);
      d(ob.cone_br);
      d(ob.cone_tr);
      d(ob.cone_b2);
      d(ob.cone_g);
      i(ob.cone_capped);
    }
    o += "\n";
    for (const XformOp& x : ob.chain) {
      o += "  xform";
      i(x.kind);
      for (double y : x.v) d(y);
      o += "\n";
    }
  }
  for (const Material& m : s.materials) {
    o += "material";
    mat(m);
    o += "\n";
  }
  for (const Mesh& me : s.meshes) {
    o += "mesh";
    i(static_cast<long long>(me.verts.size()));
    i(static_cast<long long>(me.raw_faces.size()));
    i(static_cast<long long>(me.raw_normals.size()));
    i(static_cast<long long>(me.vmats.size()));
    i(me.gennormals);
    o += "\n";
    for (const dvec3& v : me.verts) {
      o += "  v";
      v3(v);
      o += "\n";
    }
    for (const auto& fc : me.raw_faces) {
      o += "  f";
      i(fc[0]);
      i(fc[1]);
      i(fc[2]);
      o += "\n";
    }
    for (const dvec3& n : me.raw_normals) {
      o += "  n";
      v3(n);
      o += "\n";
    }
    for (const Material& m : me.vmats) {
      o += "  vmat";
      mat(m);
      o += "\n";
    }
  }
  for (const Light& L : s.lights) {
    o += "light";
    i(L.type);
    v3(L.color);
    v3(L.pos);
    v3(L.raw_dir);
    v3(L.raw_up);
    f(L.c);
    f(L.l);
    f(L.q);
    d(L.width);
    d(L.height);
    d(L.radius);
    d(L.angle);
    o += "\n";
  }
  for (const Texture& t : s.textures) {
    o += "texture " + t.path;
    i(t.width);
    i(t.height);
    unsigned long long h = 1469598103934665603ull;  // FNV-1a of the texels
    for (uint8_t c : t.data) h = (h ^ c) * 1099511628211ull;
    std::snprintf(b, sizeof(b), " %016llx", h);
    o += b;
    o += "\n";
  }
  return o;
}

}  // namespace rtxh
