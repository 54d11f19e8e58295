// ref_harness.cpp — TEST INFRASTRUCTURE (build container only): extern "C"
// entry points over the reference's OWN tokenizer and image I/O, compiled
// unmodified from /root/reference/ray/src by oracle/Makefile's `ref` target
// into oracle/_ref/libref_io.so (git-ignored; nothing from the reference is
// committed, and nothing here runs on the GPU box).  tests/test_ref_pins.py
// compares the product's tokenizer and image reader / writer with these.
//
//   ref_tokens       Tokenizer(fp, ...) + Get() until EOFSYM
//                    (parser/Tokenizer.cpp:39-123), names by Token::toString
//                    (parser/Token.cpp:27-107)
//   ref_read_image   readImage (fileio/images.cc:47-53 -> readBMP
//                    bitmap.cpp:17-93 / readPNG pngimage.cpp:195-216)
//   ref_write_image  writeImage (fileio/images.cc:59-68 -> writeBMP /
//                    writePNG pngimage.cpp:226-285)
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "fileio/images.h"
#include "parser/ParserException.h"
#include "parser/Token.h"
#include "parser/Tokenizer.h"

namespace {
std::string g_err;

// Token::toString()'s name of a token kind; getNameForToken has no entry for
// fov and gennormals (it prints "Unknown token type"), so those print their
// reserved word, as the product's dump does.
std::string token_name(const Token& t) {
  if (t.kind() == FOV) return "fov";
  if (t.kind() == GENNORMALS) return "gennormals";
  return getNameForToken(t.kind());
}
}  // namespace

extern "C" {

const char* ref_last_error(void) { return g_err.c_str(); }

// One token per line: name, then a tab and the identifier / the scalar
// (%.17g); "ERROR" after the tokens read before a syntax error.
int ref_tokens(const char* path, char* out, int64_t cap, int64_t* need) {
  std::ifstream ifs(path);
  if (!ifs) {
    g_err = std::string("cannot open ") + path;
    return -1;
  }
  std::ostringstream o;
  try {
    Tokenizer tk(ifs, false);
    for (;;) {
      std::unique_ptr<Token> t = tk.Get();
      o << token_name(*t);
      if (t->kind() == IDENT) o << '\t' << t->ident();
      if (t->kind() == SCALAR) {
        char b[40];
        std::snprintf(b, sizeof(b), "%.17g", t->value());
        o << '\t' << b;
      }
      o << '\n';
      if (t->kind() == EOFSYM) break;
    }
  } catch (const ParserException&) {
    o << "ERROR\n";
  }
  const std::string s = o.str();
  *need = static_cast<int64_t>(s.size()) + 1;
  if (out) {
    if (cap < *need) return -1;
    std::memcpy(out, s.c_str(), s.size() + 1);
  }
  return 0;
}

// readImage: the returned vector as it is (row 0 = bottom) and its size.
// (readBMP returns height * padded-row bytes with the pixels packed at the
// front, bitmap.cpp:57-91; TextureMap reads (x + y * width) * 3 only,
// material.cpp:128-132.)
int ref_read_image(const char* path, int32_t* w, int32_t* h, int64_t* size, uint8_t* out, int64_t cap) {
  int iw = 0, ih = 0;
  std::vector<uint8_t> d = readImage(path, iw, ih);
  if (d.empty() || iw <= 0 || ih <= 0) {
    g_err = std::string("readImage failed: ") + path;
    return -1;
  }
  *w = iw;
  *h = ih;
  *size = static_cast<int64_t>(d.size());
  if (out) {
    if (cap < static_cast<int64_t>(d.size())) return -1;
    std::memcpy(out, d.data(), d.size());
  }
  return 0;
}

int ref_write_image(const char* path, int32_t w, int32_t h, const uint8_t* rgb) {
  try {
    writeImage(path, w, h, rgb);
  } catch (const std::string& e) {  // writePNG throws std::string (pngimage.cpp:237-279)
    g_err = e;
    return -1;
  }
  return 0;
}

}  // extern "C"
