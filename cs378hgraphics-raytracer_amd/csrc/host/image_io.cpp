// image_io.cpp — image read/write for the loader and the CLI.
//
// Behaviour follows ray/src/fileio/images.cc:27-68 (extension dispatch,
// unknown extension -> BMP on write), bitmap.cpp:17-149 (24-bit BMP, rows
// stored bottom-up, BGR<->RGB swap, 4-byte row padding) and pngimage.cpp:
// 226-285 (RGB8 PNG whose first row is the LAST buffer row, i.e. buffer row
// 0 is the bottom of the picture).  The PNG encoder here uses stored
// (uncompressed) deflate blocks so it needs no libpng/zlib.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <strings.h>

#include "scene_model.h"

namespace rtxh {
namespace {

std::string ext_of(const std::string& fn) {
  size_t dot = fn.find_last_of('.');
  if (dot == std::string::npos || dot + 1 >= fn.size()) return "";
  return fn.substr(dot);
}

bool ieq(const std::string& a, const char* b) { return strcasecmp(a.c_str(), b) == 0; }

uint32_t rd32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | (uint32_t(p[3]) << 24); }
uint16_t rd16(const uint8_t* p) { return uint16_t(p[0] | (p[1] << 8)); }

std::vector<uint8_t> read_bmp(const std::string& fn, int& width, int& height) {
  std::ifstream f(fn, std::ios::binary);
  if (!f) return {};
  std::vector<uint8_t> file((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (file.size() < 54) return {};
  if (rd16(&file[0]) != 0x4d42) return {};
  uint32_t off = rd32(&file[10]);
  int32_t w = static_cast<int32_t>(rd32(&file[18]));
  int32_t h = static_cast<int32_t>(rd32(&file[22]));
  uint16_t bpp = rd16(&file[28]);
  if (bpp != 24) return {};
  if (w <= 0 || h <= 0) return {};
  int padWidth = w * 3;
  int pad = 0;
  if (padWidth % 4 != 0) {
    pad = 4 - (padWidth % 4);
    padWidth += pad;
  }
  size_t bytes = size_t(h) * padWidth;
  if (off + bytes > file.size()) return {};
  std::vector<uint8_t> image(file.begin() + off, file.begin() + off + bytes);
  uint8_t* in = image.data();
  uint8_t* out = image.data();
  for (int j = 0; j < h; ++j) {
    for (int i = 0; i < w; ++i) {
      out[1] = in[1];
      uint8_t t = in[2];
      out[2] = in[0];
      out[0] = t;
      in += 3;
      out += 3;
    }
    in += pad;
  }
  image.resize(size_t(w) * h * 3);
  width = w;
  height = h;
  return image;
}

bool write_bmp(const std::string& fn, int width, int height, const uint8_t* data, std::string* err) {
  FILE* f = std::fopen(fn.c_str(), "wb");
  if (!f) {
    if (err) *err = "could not open " + fn + " for writing";
    return false;
  }
  int bytes = width * 3;
  int pad = (bytes % 4) ? 4 - (bytes % 4) : 0;
  bytes += pad;
  uint8_t hdr[54] = {0};
  auto w32 = [&](int o, uint32_t v) { for (int k = 0; k < 4; ++k) hdr[o + k] = uint8_t(v >> (8 * k)); };
  hdr[0] = 'B'; hdr[1] = 'M';
  w32(2, 54 + bytes * height);
  w32(10, 54);
  w32(14, 40);
  w32(18, width);
  w32(22, height);
  hdr[26] = 1;
  hdr[28] = 24;
  w32(38, 2834);
  w32(42, 2834);
  std::fwrite(hdr, 1, 54, f);
  std::vector<uint8_t> line(bytes, 0);
  for (int j = 0; j < height; ++j) {
    std::memcpy(line.data(), data + size_t(j) * 3 * width, size_t(width) * 3);
    for (int i = 0; i < width; ++i) std::swap(line[i * 3], line[i * 3 + 2]);
    std::fwrite(line.data(), 1, bytes, f);
  }
  std::fclose(f);
  return true;
}

uint32_t crc_table[256];
bool crc_ready = false;
uint32_t crc32_update(uint32_t crc, const uint8_t* p, size_t n) {
  if (!crc_ready) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      crc_table[i] = c;
    }
    crc_ready = true;
  }
  for (size_t i = 0; i < n; ++i) crc = crc_table[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
  return crc;
}

void put_be32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back(uint8_t(x >> 24)); v.push_back(uint8_t(x >> 16));
  v.push_back(uint8_t(x >> 8)); v.push_back(uint8_t(x));
}

void png_chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
  put_be32(out, static_cast<uint32_t>(data.size()));
  size_t start = out.size();
  out.insert(out.end(), type, type + 4);
  out.insert(out.end(), data.begin(), data.end());
  uint32_t crc = crc32_update(0xffffffffu, &out[start], out.size() - start) ^ 0xffffffffu;
  put_be32(out, crc);
}

bool write_png(const std::string& fn, int width, int height, const uint8_t* data, std::string* err) {
  // raw scanlines: filter byte 0 + RGB; PNG row r = buffer row height-1-r
  const size_t stride = size_t(width) * 3 + 1;
  std::vector<uint8_t> raw(stride * height);
  for (int r = 0; r < height; ++r) {
    raw[r * stride] = 0;
    std::memcpy(&raw[r * stride + 1], data + size_t(height - 1 - r) * width * 3, size_t(width) * 3);
  }
  std::vector<uint8_t> z;
  z.push_back(0x78); z.push_back(0x01);
  size_t pos = 0;
  uint32_t a = 1, b = 0;
  for (uint8_t c : raw) { a = (a + c) % 65521u; b = (b + a) % 65521u; }
  do {
    size_t n = std::min<size_t>(65535, raw.size() - pos);
    bool last = pos + n == raw.size();
    z.push_back(last ? 1 : 0);
    z.push_back(uint8_t(n & 0xff)); z.push_back(uint8_t(n >> 8));
    z.push_back(uint8_t(~n & 0xff)); z.push_back(uint8_t((~n >> 8) & 0xff));
    z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + n);
    pos += n;
  } while (pos < raw.size());
  put_be32(z, (b << 16) | a);
  std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::vector<uint8_t> ihdr;
  put_be32(ihdr, width);
  put_be32(ihdr, height);
  ihdr.push_back(8); ihdr.push_back(2); ihdr.push_back(0); ihdr.push_back(0); ihdr.push_back(0);
  png_chunk(out, "IHDR", ihdr);
  png_chunk(out, "IDAT", z);
  png_chunk(out, "IEND", {});
  FILE* f = std::fopen(fn.c_str(), "wb");
  if (!f) {
    if (err) *err = "[write_png_file] File could not be opened for writing: " + fn;
    return false;
  }
  std::fwrite(out.data(), 1, out.size(), f);
  std::fclose(f);
  return true;
}

}  // namespace

std::vector<uint8_t> read_image(const std::string& path, int& w, int& h) {
  std::string e = ext_of(path);
  if (ieq(e, ".bmp")) return read_bmp(path, w, h);
  // PNG textures need libpng's gamma handling (pngimage.cpp:195-216);
  // not supported by this build: treated as unreadable.
  return {};
}

bool write_image(const std::string& path, int w, int h, const uint8_t* rgb, std::string* err) {
  std::string e = ext_of(path);
  if (ieq(e, ".png")) return write_png(path, w, h, rgb, err);
  if (!ieq(e, ".bmp"))
    std::fprintf(stderr, "Unrecognized extension for file %s, writing bmp format\n", path.c_str());
  return write_bmp(path, w, h, rgb, err);
}

}  // namespace rtxh
