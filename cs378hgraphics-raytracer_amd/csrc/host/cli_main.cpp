// cli_main.cpp — `ray [options] in.ray out.png`, the drop-in for the
// reference CLI (ray/src/main.cpp:23-42, ui/CommandLineUI.cpp:23-190).
//
// Same getopt surface and exit codes; the render goes through the C ABI:
// rtx_host_load (RayTracer::loadScene) -> rtx_scene_create -> rtx_render
// (traceSetup + traceImage) -> rtx_write_image (writeImage).  There is no CPU
// fallback: without a gfx950 device the command fails loudly.
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "cli_opts.h"
#include "rtx.h"
#include "rtx_host.h"

int rtx_cli_multi_gpu(const rtxh::CliOptions& o, void* host_scene);  // multi_gpu.cpp

// raw dump of an extension output (--dump-f64 / --dump-hits); false after
// printing why it could not be written
static bool dump_raw(const std::string& path, const void* data, size_t elem, size_t n) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) {
    std::cerr << "cannot open '" << path << "' for writing: " << std::strerror(errno) << std::endl;
    return false;
  }
  const bool ok = std::fwrite(data, elem, n, f) == n;
  if (std::fclose(f) != 0 || !ok) {
    std::cerr << "write to '" << path << "' failed" << std::endl;
    return false;
  }
  return true;
}

int main(int argc, char** argv) {
  rtxh::CliOptions o;
  int rc = rtxh::cli_parse(argc, argv, o);
  if (rc) return rc;

  void* hs = nullptr;
  if (rtx_host_load(o.ray_name.c_str(), &hs) != RTX_OK) {
    std::cerr << rtx_host_last_error() << std::endl;
    std::cerr << "Unable to load ray file '" << o.ray_name << "'" << std::endl;
    return 1;
  }
  if (!o.cubemap.empty() && rtx_host_cubemap(hs, o.cubemap.c_str()) != RTX_OK)
    std::cerr << rtx_host_last_error() << std::endl;  // smartLoadCubemap: render on without one
  if (o.gpus > 0) {  // one process per GPU, RCCL gather (multi_gpu.cpp); no HIP call before the fork
    if (!o.dump_f64.empty() || !o.dump_hits.empty()) {
      std::cerr << "--dump-f64 / --dump-hits are single-GPU options" << std::endl;
      rtx_host_free(hs);
      return 1;
    }
    const int mrc = rtx_cli_multi_gpu(o, hs);
    rtx_host_free(hs);
    return mrc;
  }
  RtxHostInfo info;
  rtx_host_info(hs, &info);
  RtxSceneDesc desc;
  rtx_host_desc(hs, &desc);
  void* scene = nullptr;
  if (rtx_scene_create(o.device, &desc, &scene) != RTX_OK) {
    std::cerr << "rtx: " << rtx_last_error() << std::endl;
    rtx_host_free(hs);
    return 2;
  }
  const int width = o.size;
  const int height = rtx_image_height(width, info.aspect);  // CommandLineUI.cpp:156
  RtxRenderParams p = rtxh::cli_params(o, width, height);
  std::vector<uint8_t> rgb(size_t(width) * height * 3, 0);
  std::vector<double> f64;
  if (!o.dump_f64.empty()) f64.assign(size_t(width) * height * 3, 0.0);
  const int spp = o.aa_mode == RTX_AA_NONE ? 1 : o.aa_samples * o.aa_samples;
  std::vector<RtxHitRecord> hits;
  if (!o.dump_hits.empty()) hits.resize(size_t(width) * height * spp);
  RtxStats st;
  auto t0 = std::chrono::steady_clock::now();
  rtx_status r = rtx_render(scene, &p, rgb.data(), f64.empty() ? nullptr : f64.data(),
                            hits.empty() ? nullptr : hits.data(), 0, nullptr, o.stats ? &st : nullptr);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (r != RTX_OK) {
    std::cerr << "rtx: " << rtx_last_error() << std::endl;
    rtx_scene_destroy(scene);
    rtx_host_free(hs);
    return 2;
  }
  if (rtx_write_image(o.img_name.c_str(), width, height, rgb.data()) != RTX_OK) {
    std::cerr << rtx_host_last_error() << std::endl;
    return 1;
  }
  if (!o.dump_f64.empty() && !dump_raw(o.dump_f64, f64.data(), sizeof(double), f64.size())) rc = 1;
  if (!o.dump_hits.empty() && !dump_raw(o.dump_hits, hits.data(), sizeof(RtxHitRecord), hits.size())) rc = 1;
  if (o.stats)
    std::printf("{\"backend\": \"hip-gfx950\", \"ms\": %.3f, \"kernel_ms\": %.3f, \"rays\": %lld, "
                "\"mrays_per_s\": %.3f, \"node_visits\": %lld, \"object_tests\": %lld, \"tri_tests\": %lld, "
                "\"shades\": %lld}\n",
                ms, st.kernel_ms, (long long)st.rays, st.rays / st.kernel_ms / 1e3, (long long)st.node_visits,
                (long long)st.object_tests, (long long)st.tri_tests, (long long)st.shades);
  rtx_scene_destroy(scene);
  rtx_host_free(hs);
  return rc;
}
