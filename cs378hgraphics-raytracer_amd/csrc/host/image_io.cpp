// image_io.cpp — image read/write for the loader and the CLI.
//
// Behaviour follows ray/src/fileio/images.cc:27-68 (extension dispatch,
// unknown extension -> BMP on write), bitmap.cpp:17-149 (24-bit BMP, rows
// stored bottom-up, BGR<->RGB swap, 4-byte row padding) and pngimage.cpp:
// 226-285 (RGB8 PNG whose first row is the LAST buffer row, i.e. buffer row
// 0 is the bottom of the picture).  The PNG encoder here uses stored
// (uncompressed) deflate blocks; the PNG reader (textures) inflates with
// zlib and restates libpng's transforms (no libpng in this image).
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
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
  // bfSize counts sizeof(BMP_BITMAPFILEHEADER), which is 16 with the
  // struct's padding, not the 14 bytes written (bitmap.cpp:105)
  w32(2, 56 + bytes * height);
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
  // The reference copies the PADDED row length from the packed buffer
  // (bitmap.cpp:137), so a row's padding holds the first bytes of the next
  // row; for the last row it reads past the buffer (undefined: decision
  // U25, zeros here).
  const size_t total = size_t(width) * 3 * height;
  for (int j = 0; j < height; ++j) {
    const size_t at = size_t(j) * 3 * width;
    std::fill(line.begin(), line.end(), 0);
    std::memcpy(line.data(), data + at, std::min(size_t(bytes), total - at));
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

// ---------------------------------------------------------------- PNG read
// readPNG (pngimage.cpp:195-216) with the libpng transforms PNGReader::
// get_image registers (pngimage.cpp:140-170), restated over zlib's inflate:
//   palette -> RGB (png_set_expand), gray below 8 bits -> 8 bits, a tRNS
//   chunk -> an alpha channel, 16-bit samples -> their high byte
//   (png_set_strip_16), gray -> RGB (png_set_gray_to_rgb), and a gamma
//   correction only when the file has a gAMA chunk (display exponent 2.2;
//   libpng 1.6 skips corrections within 5% of 1 and maps an 8-bit sample v
//   in (0, 255) to floor(255 (v/255)^g + 0.5)).  Adam7 images are
//   de-interlaced (png_read_image turns interlace handling on).  The result
//   holds `channels` bytes per pixel (3, or 4 with alpha) with the rows
//   flipped, buffer row 0 = the picture's bottom row.  TextureMap indexes it
//   with a stride of 3 whatever the channel count (material.cpp:121-138),
//   and so does this build.  Any failure returns an empty buffer (the
//   reference's reader returns one too; TextureMap then throws).
uint32_t be32(const uint8_t* p) { return (uint32_t(p[0]) << 24) | (p[1] << 16) | (p[2] << 8) | p[3]; }

int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

// undo the filters of one (sub-)image of h rows of `rb` bytes, bpp bytes per
// complete pixel (>= 1); `in` holds the filter byte + row per row
bool unfilter(const uint8_t* in, size_t in_len, int h, size_t rb, int bpp, std::vector<uint8_t>& out) {
  if (in_len < size_t(h) * (rb + 1)) return false;
  out.assign(size_t(h) * rb, 0);
  for (int y = 0; y < h; ++y) {
    const uint8_t ft = in[size_t(y) * (rb + 1)];
    const uint8_t* src = in + size_t(y) * (rb + 1) + 1;
    uint8_t* row = out.data() + size_t(y) * rb;
    const uint8_t* up = y > 0 ? row - rb : nullptr;
    for (size_t x = 0; x < rb; ++x) {
      const int a = x >= size_t(bpp) ? row[x - bpp] : 0;
      const int b = up ? up[x] : 0;
      const int c = (up && x >= size_t(bpp)) ? up[x - bpp] : 0;
      int v = src[x];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) / 2; break;
        case 4: v += paeth(a, b, c); break;
        default: return false;
      }
      row[x] = static_cast<uint8_t>(v);
    }
  }
  return true;
}

std::vector<uint8_t> read_png(const std::string& fn, int& width, int& height) {
  std::ifstream f(fn, std::ios::binary);
  if (!f) return {};
  std::vector<uint8_t> file((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (file.size() < 8 || std::memcmp(file.data(), sig, 8) != 0) return {};
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = -1, interlace = 0;
  std::vector<uint8_t> idat, plte, trns;
  bool have_gama = false;
  uint32_t gama = 0;
  size_t pos = 8;
  while (pos + 12 <= file.size()) {
    const uint32_t len = be32(&file[pos]);
    if (pos + 12 + size_t(len) > file.size()) return {};
    const uint8_t* type = &file[pos + 4];
    const uint8_t* d = &file[pos + 8];
    if (!std::memcmp(type, "IHDR", 4)) {
      if (len < 13) return {};
      w = be32(d);
      h = be32(d + 4);
      depth = d[8];
      ctype = d[9];
      interlace = d[12];
    } else if (!std::memcmp(type, "PLTE", 4)) {
      plte.assign(d, d + len);
    } else if (!std::memcmp(type, "tRNS", 4)) {
      trns.assign(d, d + len);
    } else if (!std::memcmp(type, "gAMA", 4) && len >= 4) {
      have_gama = true;
      gama = be32(d);
    } else if (!std::memcmp(type, "IDAT", 4)) {
      idat.insert(idat.end(), d, d + len);
    } else if (!std::memcmp(type, "IEND", 4)) {
      break;
    }
    pos += 12 + size_t(len);
  }
  // at most 2^28 pixels (a 16k x 16k texture), so a few-byte header cannot
  // ask for a multi-terabyte allocation
  if (w == 0 || h == 0 || w > (1u << 24) || h > (1u << 24) || uint64_t(w) * h > (uint64_t(1) << 28) ||
      interlace > 1)
    return {};
  int spp_in;  // samples per pixel in the file
  switch (ctype) {
    case 0: spp_in = 1; break;
    case 2: spp_in = 3; break;
    case 3: spp_in = 1; break;
    case 4: spp_in = 2; break;
    case 6: spp_in = 4; break;
    default: return {};
  }
  if (depth != 1 && depth != 2 && depth != 4 && depth != 8 && depth != 16) return {};
  if (ctype == 3 && (depth > 8 || plte.size() < 3)) return {};
  if ((ctype == 2 || ctype == 4 || ctype == 6) && depth < 8) return {};
  const int bits_px = spp_in * depth;
  const int bpp = std::max(1, bits_px / 8);
  // Adam7 pass geometry (x0, y0, dx, dy); one pass covering all for none
  static const int A7[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                               {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
  const int npass = interlace ? 7 : 1;
  size_t raw_len = 0;
  for (int p = 0; p < npass; ++p) {
    const uint32_t pw = interlace ? (w + A7[p][2] - 1 - A7[p][0]) / A7[p][2] : w;
    const uint32_t ph = interlace ? (h + A7[p][3] - 1 - A7[p][1]) / A7[p][3] : h;
    if (pw && ph) raw_len += size_t(ph) * ((size_t(pw) * bits_px + 7) / 8 + 1);
  }
  // deflate expands at most ~1032:1: a stream too short for the header's
  // size is a truncated or forged file, rejected before allocating
  if (raw_len > idat.size() * 1032 + 4096) return {};
  std::vector<uint8_t> raw(raw_len);
  {
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (inflateInit(&zs) != Z_OK) return {};
    zs.next_in = idat.data();
    zs.avail_in = static_cast<uInt>(idat.size());
    zs.next_out = raw.data();
    zs.avail_out = static_cast<uInt>(raw.size());
    const int zr = inflate(&zs, Z_FINISH);
    const size_t got = raw.size() - zs.avail_out;
    inflateEnd(&zs);
    if ((zr != Z_STREAM_END && zr != Z_BUF_ERROR && zr != Z_OK) || got != raw.size()) return {};
  }
  // samples at full depth-resolution, per pixel, in picture order (top row first)
  const bool alpha_out = ctype == 4 || ctype == 6 || !trns.empty();
  const int ch = alpha_out ? 4 : 3;
  std::vector<uint8_t> img(size_t(w) * h * ch, 0);
  auto sample = [&](const uint8_t* row, uint32_t x, int k) -> int {  // k-th sample of pixel x, native depth
    if (depth == 16) return (row[(size_t(x) * spp_in + k) * 2] << 8) | row[(size_t(x) * spp_in + k) * 2 + 1];
    if (depth == 8) return row[size_t(x) * spp_in + k];
    const size_t bit = size_t(x) * depth;  // spp_in == 1 here
    return (row[bit / 8] >> (8 - depth - bit % 8)) & ((1 << depth) - 1);
  };
  const int maxv = (1 << depth) - 1;
  auto to8 = [&](int v) -> int { return depth == 16 ? v >> 8 : (depth == 8 ? v : v * 255 / maxv); };
  size_t off = 0;
  for (int p = 0; p < npass; ++p) {
    const uint32_t x0 = interlace ? A7[p][0] : 0, y0 = interlace ? A7[p][1] : 0;
    const uint32_t dx = interlace ? A7[p][2] : 1, dy = interlace ? A7[p][3] : 1;
    const uint32_t pw = interlace ? (w + dx - 1 - x0) / dx : w;
    const uint32_t ph = interlace ? (h + dy - 1 - y0) / dy : h;
    if (!pw || !ph) continue;
    const size_t rb = (size_t(pw) * bits_px + 7) / 8;
    std::vector<uint8_t> px;
    if (!unfilter(raw.data() + off, raw.size() - off, static_cast<int>(ph), rb, bpp, px)) return {};
    off += size_t(ph) * (rb + 1);
    for (uint32_t yy = 0; yy < ph; ++yy) {
      const uint8_t* row = px.data() + size_t(yy) * rb;
      for (uint32_t xx = 0; xx < pw; ++xx) {
        const uint32_t X = x0 + xx * dx, Y = y0 + yy * dy;
        uint8_t* o = &img[(size_t(Y) * w + X) * ch];
        int r, g, b, a = 255;
        if (ctype == 3) {
          const int idx = sample(row, xx, 0);
          if (size_t(idx) * 3 + 2 >= plte.size()) return {};
          r = plte[idx * 3];
          g = plte[idx * 3 + 1];
          b = plte[idx * 3 + 2];
          if (size_t(idx) < trns.size()) a = trns[idx];
        } else if (ctype == 0 || ctype == 4) {
          const int v = sample(row, xx, 0);
          r = g = b = to8(v);
          if (ctype == 4) a = to8(sample(row, xx, 1));
          else if (trns.size() >= 2 && v == ((trns[0] << 8) | trns[1])) a = 0;
        } else {
          const int R = sample(row, xx, 0), G = sample(row, xx, 1), B = sample(row, xx, 2);
          r = to8(R);
          g = to8(G);
          b = to8(B);
          if (ctype == 6) a = to8(sample(row, xx, 3));
          else if (trns.size() >= 6 && R == ((trns[0] << 8) | trns[1]) && G == ((trns[2] << 8) | trns[3]) &&
                   B == ((trns[4] << 8) | trns[5]))
            a = 0;
        }
        o[0] = static_cast<uint8_t>(r);
        o[1] = static_cast<uint8_t>(g);
        o[2] = static_cast<uint8_t>(b);
        if (alpha_out) o[3] = static_cast<uint8_t>(a);
      }
    }
  }
  if (have_gama && gama > 0) {
    // png_set_gamma(png, 2.2, file_gamma): correction 1 / (file_gamma * 2.2)
    // in libpng's 1e5 fixed point (png_reciprocal2), applied when it is off
    // 1 by more than PNG_GAMMA_THRESHOLD (0.05); alpha is not corrected
    const double corr = std::floor(1e15 / double(gama) / 220000.0 + 0.5);
    if (corr < 95000.0 || corr > 105000.0) {
      uint8_t table[256];
      for (int v = 0; v < 256; ++v)
        table[v] = (v > 0 && v < 255) ? static_cast<uint8_t>(std::floor(255 * std::pow(v / 255., corr * .00001) + .5))
                                      : static_cast<uint8_t>(v);
      for (size_t k = 0; k < img.size(); ++k)
        if (!(alpha_out && k % 4 == 3)) img[k] = table[img[k]];
    }
  }
  // flip rows: buffer row j = picture row h - 1 - j (pngimage.cpp:208-214)
  std::vector<uint8_t> data(img.size());
  const size_t rowbytes = size_t(w) * ch;
  for (uint32_t j = 0; j < h; ++j) std::memcpy(&data[size_t(j) * rowbytes], &img[size_t(h - 1 - j) * rowbytes], rowbytes);
  width = static_cast<int>(w);
  height = static_cast<int>(h);
  return data;
}

}  // namespace

// images.cc:27-58: dispatch on the extension (".bmp" / ".png", case
// insensitive); anything else is unreadable (an empty buffer)
std::vector<uint8_t> read_image(const std::string& path, int& w, int& h) {
  std::string e = ext_of(path);
  if (ieq(e, ".bmp")) return read_bmp(path, w, h);
  if (ieq(e, ".png")) return read_png(path, w, h);
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
