// cli_opts.h — the reference command line, restated.
//
// getopt string "tr:w:hj:c:O:A:B:C:D" and the -O / -A / -B / -C state
// machine of CommandLineUI::CommandLineUI (ray/src/ui/CommandLineUI.cpp:
// 23-147), TraceUI defaults (ui/TraceUI.h:34-129) and the -j JSON keys of
// TraceUI::loadFromJson (ui/TraceUI.cc:42-84, incl. the "supersamples" ->
// m_aa_thresh quirk; decision U20: "kdtree" is ignored).  Long options that
// the reference lacks (--device, --stats, --dump-f64, --dump-hits) are
// accepted after the short ones.
#pragma once

#include <getopt.h>

#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>

#include "rtx.h"

namespace rtxh {

struct CliOptions {
  int size = 512;        // m_nSize
  int depth = 0;         // m_nDepth
  int block_size = 4;    // m_nBlockSize (read, unused: RayTracer.cpp:259)
  double aterm_thresh = 0;
  int aa_mode = RTX_AA_NONE;
  int aa_samples = 3;
  double aa_thresh = 1.0;
  bool overlapping = false;
  bool dof = false;
  double dof_apsz = 0.05;
  int dof_div = 5;
  double dof_fd = 3;
  bool anaglyph = false;
  int ss_res = 5;
  int threads = 0;
  std::string cubemap;
  std::string ray_name, img_name;
  // extensions
  int device = 0;      // first GPU (ranks use device + rank)
  int gpus = 0;        // > 0: tile-shard the frame over this many GPUs (multi_gpu.cpp)
  int tile = 16;       // shard tile size with --gpus (16: the 8-way headline's slowest shard 2-3 % faster than with 32, profiles/r05o_ab_tile.txt)
  bool stats = false;
  std::string dump_f64, dump_hits;
};

inline void cli_usage(const char* prog, const CliOptions& o) {
  std::cerr << "usage: " << prog << " [options] [input.ray output.png]\n"
            << "  -r <#>      set recursion level (default " << o.depth << ")\n"
            << "  -w <#>      set output image width (default " << o.size << ")\n"
            << "  -j <FILE>   set parameters from JSON file\n"
            << "  -c <FILE>   one Cubemap file, the remaining files will be detected automatically\n"
            << "  -O <char>   additional options: a adaptive AA, j jittered AA, r regular AA,\n"
            << "              o overlapping objects, d dof, g anaglyph, c adaptive termination,\n"
            << "              s stochastic lighting ray count\n"
            << "  -A <#>      value for the most recent -O (ajr: AA samples, c: termination\n"
            << "              threshold, s: soft-shadow rays, d: focal distance)\n"
            << "  -B <?>      a: adaptive AA threshold, d: DoF samples\n"
            << "  -C <?>      d: aperture size\n"
            << "  --device N  GPU index (extension)   --stats  print JSON stats (extension)\n"
            << "  --gpus N    one process per GPU, 16x16 tiles dealt over N GPUs, RCCL gather (extension)\n"
            << "  --tile T    tile size with --gpus (default 16)\n"
            << "  --dump-f64 FILE / --dump-hits FILE  raw float64 RGB / hit records (extension)\n";
}

// Minimal flat-object JSON reader for the keys loadFromJson uses.
inline std::map<std::string, std::string> cli_read_json(const std::string& path) {
  std::map<std::string, std::string> kv;
  std::ifstream f(path);
  std::stringstream ss;
  ss << f.rdbuf();
  std::string s = ss.str();
  size_t i = 0;
  auto skip = [&]() { while (i < s.size() && std::isspace(static_cast<unsigned char>(s[i]))) ++i; };
  skip();
  if (i >= s.size() || s[i] != '{') return kv;
  ++i;
  for (;;) {
    skip();
    if (i >= s.size() || s[i] == '}') break;
    if (s[i] == ',') { ++i; continue; }
    if (s[i] != '"') break;
    size_t e = s.find('"', i + 1);
    if (e == std::string::npos) break;
    std::string key = s.substr(i + 1, e - i - 1);
    i = e + 1;
    skip();
    if (i >= s.size() || s[i] != ':') break;
    ++i;
    skip();
    size_t st = i;
    if (i < s.size() && s[i] == '"') {
      size_t e2 = s.find('"', i + 1);
      kv[key] = s.substr(i + 1, e2 - i - 1);
      i = e2 + 1;
      continue;
    }
    while (i < s.size() && s[i] != ',' && s[i] != '}') ++i;
    std::string v = s.substr(st, i - st);
    while (!v.empty() && std::isspace(static_cast<unsigned char>(v.back()))) v.pop_back();
    kv[key] = v;
  }
  return kv;
}

inline void cli_load_json(CliOptions& o, const std::string& path) {  // TraceUI.cc:42-84
  auto kv = cli_read_json(path);
  auto num = [&](const char* k, double& dst) {
    auto it = kv.find(k);
    if (it != kv.end()) dst = std::atof(it->second.c_str());
  };
  auto inum = [&](const char* k, int& dst) {
    auto it = kv.find(k);
    if (it != kv.end()) dst = std::atoi(it->second.c_str());
  };
  inum("threads", o.threads);
  inum("size", o.size);
  inum("recursion_depth", o.depth);
  int aterm = static_cast<int>(o.aterm_thresh * 1000);
  inum("threshold", aterm);
  o.aterm_thresh = aterm / 1000.0;
  inum("blocksize", o.block_size);
  auto aa = kv.find("anti_alias");
  if (aa != kv.end()) o.aa_mode = (aa->second == "true" || std::atoi(aa->second.c_str()) != 0) ? 1 : 0;
  num("supersamples", o.aa_thresh);  // quirk: writes m_aa_thresh
  int aat = static_cast<int>(o.aa_thresh * 100);
  inum("aa_threshold", aat);
  o.aa_thresh = aat / 100.0;
}

// A whole decimal number in [lo, hi] for one of the long options the
// reference lacks (atoi would turn "abc" into 0 and "-3" into a silent
// fallback); false with a message otherwise.
inline bool cli_int_arg(const char* name, const char* s, int lo, int hi, int& out) {
  char* end = nullptr;
  errno = 0;
  const long v = std::strtol(s, &end, 10);
  if (s[0] == '\0' || *end != '\0' || errno == ERANGE || v < lo || v > hi) {
    std::cerr << "--" << name << " needs an integer in [" << lo << ", " << hi << "], got '" << s << "'" << std::endl;
    return false;
  }
  out = static_cast<int>(v);
  return true;
}

// Returns 0 on success, otherwise the exit code the reference would use.
inline int cli_parse(int argc, char** argv, CliOptions& o) {
  static struct option longopts[] = {{"device", required_argument, nullptr, 1000},
                                     {"stats", no_argument, nullptr, 1001},
                                     {"dump-f64", required_argument, nullptr, 1002},
                                     {"dump-hits", required_argument, nullptr, 1003},
                                     {"gpus", required_argument, nullptr, 1004},
                                     {"tile", required_argument, nullptr, 1005},
                                     {nullptr, 0, nullptr, 0}};
  const char* jsonfile = nullptr;
  char prev = 0;
  int i;
  optind = 1;
  while ((i = getopt_long(argc, argv, "tr:w:hj:c:O:A:B:C:D", longopts, nullptr)) != EOF) {
    switch (i) {
      case 'r': o.depth = std::atoi(optarg); break;
      case 'w': o.size = std::atoi(optarg); break;
      case 'j': jsonfile = optarg; break;
      case 'c': o.cubemap = optarg; break;
      case 'O':
        prev = *optarg;
        switch (prev) {
          case 'a': o.aa_mode = RTX_AA_ADAPTIVE; break;
          case 'j': o.aa_mode = RTX_AA_JITTERED; break;
          case 'r': o.aa_mode = RTX_AA_SUPERSAMPLE; break;
          case 'o': o.overlapping = true; break;
          case 'd': o.dof = true; break;
          case 'g': o.anaglyph = true; break;
          case 'c': case 's': break;
          default:
            std::cerr << "Invalid argument for O: '" << i << "'." << std::endl;
            cli_usage(argv[0], o);
            return 1;
        }
        break;
      case 'A':
        switch (prev) {
          case 'a': case 'j': case 'r': o.aa_samples = std::atoi(optarg); break;
          case 'c': o.aterm_thresh = std::atof(optarg); break;
          case 'd': o.dof_fd = std::atof(optarg); break;
          case 's': o.ss_res = std::atoi(optarg); break;
          default:
            std::cerr << "Invalid argument for A, with prequel " << prev << ": '" << i << "'." << std::endl;
            cli_usage(argv[0], o);
            return 1;
        }
        break;
      case 'B':
        switch (prev) {
          case 'a': o.aa_thresh = std::atof(optarg); break;
          case 'd': o.dof_div = std::atoi(optarg); break;
          default:
            std::cerr << "Invalid argument for B, with prequel " << (unsigned)prev << ": '" << i << "'." << std::endl;
            cli_usage(argv[0], o);
            return 1;
        }
        break;
      case 'C':
        switch (prev) {
          case 'd': o.dof_apsz = std::atof(optarg); break;
          default:
            std::cerr << "Invalid argument for C, with prequel " << (unsigned)prev << ": '" << i << "'." << std::endl;
            cli_usage(argv[0], o);
            return 1;
        }
        break;
      case 1000:
        if (!cli_int_arg("device", optarg, 0, 1023, o.device)) return 1;
        break;
      case 1001: o.stats = true; break;
      case 1002: o.dump_f64 = optarg; break;
      case 1003: o.dump_hits = optarg; break;
      case 1004:
        if (!cli_int_arg("gpus", optarg, 1, 64, o.gpus)) return 1;
        break;
      case 1005:
        if (!cli_int_arg("tile", optarg, 1, 4096, o.tile)) return 1;
        break;
      case 'h':
        cli_usage(argv[0], o);
        return 1;
      case 't': case 'D': break;  // accepted by the reference's getopt string, no case
      default:
        std::cerr << "Invalid argument: '" << i << "'." << std::endl;
        cli_usage(argv[0], o);
        return 1;
    }
  }
  if (jsonfile) cli_load_json(o, jsonfile);
  // -c: the cube map is loaded with the scene (rtx_host_cubemap), where a
  // failure is reported and the render goes on without one
  if (optind >= argc - 1) {
    std::cerr << "no input and/or output name." << std::endl;
    return 1;
  }
  o.ray_name = argv[optind];
  o.img_name = argv[optind + 1];
  return 0;
}

inline RtxRenderParams cli_params(const CliOptions& o, int width, int height) {
  RtxRenderParams p;
  std::memset(&p, 0, sizeof(p));
  p.width = width;
  p.height = height;
  p.depth = o.depth;
  p.aa_mode = o.aa_mode;
  p.aa_samples = o.aa_samples;
  p.aa_thresh = o.aa_thresh;
  p.aterm_thresh = o.aterm_thresh;
  p.dof = o.dof ? 1 : 0;
  p.dof_fd = o.dof_fd;
  p.dof_div = o.dof_div;
  p.dof_apsz = o.dof_apsz;
  p.anaglyph = o.anaglyph ? 1 : 0;
  p.ss_res = o.ss_res;
  p.overlapping = o.overlapping ? 1 : 0;
  p.tile = 0;
  p.shard = 0;
  p.nshards = 1;
  p.packed = 0;
  return p;
}

}  // namespace rtxh
