// parser.cpp — .ray scene loader (host plumbing, not accelerated).
//
// Restates the grammar and the observable quirks of the reference parser:
//   tokenizer   ray/src/parser/Tokenizer.cpp:70-237, Token.cpp:121-196,
//               fileio/buffer.cpp (line-at-a-time reading, '\0' at EOF)
//   parser      ray/src/parser/Parser.cpp:26-1308
// It produces the RAW records of scene_model.h only (transform chains,
// camera attribute ops, raw faces / normals, light attributes): the scene
// build arithmetic (transforms, world boxes, camera basis, face records,
// light axes) is scene_build.cpp's, so the CPU oracle can link this parser
// and restate the build on its own.  Errors are reported as ParseError
// carrying the message RayTracer::loadScene would print
// (RayTracer.cpp:216-234).
#include <dirent.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <list>
#include <map>
#include <memory>
#include <sstream>

#include "scene_model.h"
#include "../common/rt_math.h"

namespace rtxh {

using rtm::mk3;

// ---------------------------------------------------------------- Material
void Material::setBools() {
  // isZero(): glm::length(_value) == 0.0 (material.h:129)
  auto isZero = [](const MatParam& q) { return rtm::length(q.v) == 0.0; };
  refl = !isZero(p[P_KR]);
  trans = !isZero(p[P_KT]);
  recur = refl || trans;
  spec = refl || !isZero(p[P_KS]);
  both = refl && trans;
}

// ---------------------------------------------------------------- Tokenizer
namespace {

enum Sym {
  EOFSYM, SBT_RAYTRACER, IDENT, SCALAR, SYMTRUE, SYMFALSE, LPAREN, RPAREN, LBRACE, RBRACE, COMMA,
  EQUALS, SEMICOLON, CAMERA, AMBIENT_LIGHT, POINT_LIGHT, DIRECTIONAL_LIGHT, AREA_LIGHT_RECT,
  AREA_LIGHT_CIRC, SPOT_LIGHT, CONSTANT_ATTENUATION_COEFF, LINEAR_ATTENUATION_COEFF,
  QUADRATIC_ATTENUATION_COEFF, SPHERE, BOX, SQUARE, CYLINDER, CONE, TRIMESH, POSITION, VIEWDIR,
  UPDIR, ASPECTRATIO, FOV, COLOR, DIRECTION, CAPPED, HEIGHT, WIDTH, ANGLE, BOTTOM_RADIUS,
  TOP_RADIUS, RADIUS, QUATERNIAN, POLYPOINTS, NORMALS, MATERIALS, FACES, GENNORMALS, TRANSLATE,
  SCALE, ROTATE, TRANSFORM, MATERIAL, EMISSIVE, AMBIENT, SPECULAR, REFLECTIVE, DIFFUSE,
  TRANSMISSIVE, SHININESS, INDEX, NAME, MAP, BUMP, GLOSS, UNKNOWN
};

const std::map<std::string, Sym>& reserved() {  // Token.cpp:121-196
  static const std::map<std::string, Sym> w = {
      {"ambient_light", AMBIENT_LIGHT}, {"ambient", AMBIENT}, {"aspectratio", ASPECTRATIO},
      {"bottom_radius", BOTTOM_RADIUS}, {"box", BOX}, {"camera", CAMERA}, {"capped", CAPPED},
      {"color", COLOR}, {"colour", COLOR}, {"cone", CONE},
      {"constant_attenuation_coeff", CONSTANT_ATTENUATION_COEFF}, {"cylinder", CYLINDER},
      {"diffuse", DIFFUSE}, {"direction", DIRECTION}, {"directional_light", DIRECTIONAL_LIGHT},
      {"emissive", EMISSIVE}, {"faces", FACES}, {"false", SYMFALSE}, {"fov", FOV},
      {"gennormals", GENNORMALS}, {"height", HEIGHT}, {"index", INDEX},
      {"linear_attenuation_coeff", LINEAR_ATTENUATION_COEFF}, {"material", MATERIAL},
      {"materials", MATERIALS}, {"map", MAP}, {"name", NAME}, {"normals", NORMALS},
      {"point_light", POINT_LIGHT}, {"points", POLYPOINTS}, {"polymesh", TRIMESH},
      {"position", POSITION}, {"quadratic_attenuation_coeff", QUADRATIC_ATTENUATION_COEFF},
      {"quaternian", QUATERNIAN}, {"reflective", REFLECTIVE}, {"rotate", ROTATE},
      {"SBT-raytracer", SBT_RAYTRACER}, {"scale", SCALE}, {"shininess", SHININESS},
      {"specular", SPECULAR}, {"sphere", SPHERE}, {"square", SQUARE}, {"top_radius", TOP_RADIUS},
      {"transform", TRANSFORM}, {"translate", TRANSLATE}, {"transmissive", TRANSMISSIVE},
      {"trimesh", TRIMESH}, {"true", SYMTRUE}, {"updir", UPDIR}, {"viewdir", VIEWDIR},
      {"bump", BUMP}, {"gloss", GLOSS}, {"angle", ANGLE}, {"width", WIDTH}, {"radius", RADIUS},
      {"area_light_rect", AREA_LIGHT_RECT}, {"area_light_circ", AREA_LIGHT_CIRC},
      {"spot_light", SPOT_LIGHT}};
  return w;
}

const char* sym_name(Sym s) {  // Token.cpp:9-92 (subset used in messages)
  switch (s) {
    case EOFSYM: return "EOF";
    case SBT_RAYTRACER: return "SBT-raytracer";
    case IDENT: return "Identifier";
    case SCALAR: return "Scalar";
    case LPAREN: return "Left paren";
    case RPAREN: return "Right paren";
    case LBRACE: return "Left brace";
    case RBRACE: return "Right brace";
    case COMMA: return "Comma";
    case EQUALS: return "Equals";
    case SEMICOLON: return "Semicolon";
    case MATERIAL: return "material";
    default: return "Unknown token type";
  }
}

struct Token {
  Sym kind = EOFSYM;
  double value = 0.0;
  std::string ident;
};

class Tokenizer {
 public:
  explicit Tokenizer(const std::string& text) {
    // Buffer reads line by line and re-appends '\n' to every line
    // (buffer.cpp GetLine); emulate by splitting on '\n'.
    size_t start = 0;
    while (start <= text.size()) {
      size_t nl = text.find('\n', start);
      if (nl == std::string::npos) {
        if (start < text.size()) lines_.push_back(text.substr(start) + "\n");
        break;
      }
      lines_.push_back(text.substr(start, nl - start) + "\n");
      start = nl + 1;
    }
    getCh();  // CurrentCh = ' ' then first GetCh happens in SkipWhiteSpace
  }

  Token get() {
    if (has_unget_) {
      has_unget_ = false;
      return unget_;
    }
    skipWhite();
    Token t;
    if (eof_) {
      t.kind = EOFSYM;
      return t;
    }
    unsigned char c = static_cast<unsigned char>(cur_);
    if (std::isalpha(c) || cur_ == '_') {
      std::string id;
      while (std::isalnum(static_cast<unsigned char>(cur_)) || cur_ == '_' || cur_ == '-') {
        id += cur_;
        getCh();
      }
      auto it = reserved().find(id);
      if (it == reserved().end()) {
        t.kind = IDENT;
        t.ident = id;
      } else {
        t.kind = it->second;
      }
    } else if (cur_ == '"') {
      getCh();
      std::string id;
      while (cur_ != '"') {
        if (cur_ == '\n') syntax("Unterminated string constant");
        if (eof_) syntax("Unterminated string constant");
        id += cur_;
        getCh();
      }
      getCh();
      t.kind = IDENT;
      t.ident = id;
    } else if (std::isdigit(c) || cur_ == '-' || cur_ == '.') {
      std::string s;
      while (std::isdigit(static_cast<unsigned char>(cur_)) || cur_ == '-' || cur_ == '.' || cur_ == 'e') {
        s += cur_;
        getCh();
      }
      t.kind = SCALAR;
      t.value = std::atof(s.c_str());
    } else {
      switch (cur_) {
        case '(': t.kind = LPAREN; break;
        case ')': t.kind = RPAREN; break;
        case '{': t.kind = LBRACE; break;
        case '}': t.kind = RBRACE; break;
        case ',': t.kind = COMMA; break;
        case '=': t.kind = EQUALS; break;
        case ';': t.kind = SEMICOLON; break;
        default: {
          std::ostringstream o;
          o << "unexpected character: '" << cur_ << "'";
          syntax(o.str());
        }
      }
      getCh();
    }
    return t;
  }

  const Token& peek() {
    Token t = get();
    unget_ = t;
    has_unget_ = true;
    return unget_;
  }

  Token read(Sym kind) {
    Token t = get();
    if (t.kind != kind) syntax(std::string(sym_name(kind)) + " expected");
    return t;
  }

  bool condRead(Sym kind) {
    if (peek().kind == kind) {
      get();
      return true;
    }
    return false;
  }

  [[noreturn]] void syntax(const std::string& msg) const {
    std::ostringstream o;
    o << "Line " << line_ << ": syntax error: " << msg;
    throw ParseError(o.str());
  }

 private:
  void getCh() {
    if (eof_) {
      cur_ = '\0';
      return;
    }
    if (li_ < lines_.size() && ci_ + 1 < lines_[li_].size() && started_) {
      ++ci_;
    } else if (!started_) {
      started_ = true;
      li_ = 0;
      ci_ = 0;
      if (lines_.empty()) {  // the first GetLine already fails: LineNumber 1
        eof_ = true;
        cur_ = '\0';
        line_ = 1;
        return;
      }
    } else {
      ++li_;
      ci_ = 0;
      if (li_ >= lines_.size()) {
        // Buffer::GetLine counts the failing read at EOF as a line too
        // (buffer.cpp:91-98: LineNumber++ before the stream is tested)
        eof_ = true;
        cur_ = '\0';
        line_ = static_cast<int>(li_) + 1;
        return;
      }
    }
    line_ = static_cast<int>(li_) + 1;
    cur_ = lines_[li_][ci_];
  }

  void skipWhite() {
    for (;;) {
      while (!eof_ && std::isspace(static_cast<unsigned char>(cur_))) getCh();
      if (cur_ != '/') return;
      int startLine = line_;
      getCh();
      if (cur_ == '/') {
        while (!eof_ && cur_ != '\n') getCh();
      } else if (cur_ == '*') {
        for (;;) {
          getCh();
          if (cur_ == '*') {
            getCh();
            if (cur_ == '/') {
              getCh();
              break;
            } else if (eof_) {
              std::ostringstream o;
              o << "Unterminated comment in line " << startLine;
              syntax(o.str());
            }
          } else if (eof_) {
            std::ostringstream o;
            o << "Unterminated comment in line " << startLine;
            syntax(o.str());
          }
        }
      } else {
        std::ostringstream o;
        o << "unexpected character: '" << cur_ << "'";
        syntax(o.str());
      }
    }
  }

  std::vector<std::string> lines_;
  size_t li_ = 0, ci_ = 0;
  bool started_ = false;
  bool eof_ = false;
  char cur_ = ' ';
  int line_ = 0;
  Token unget_;
  bool has_unget_ = false;
};

// ---------------------------------------------------------------- Parser
// a transform node of the parse: its raw operation and its parent (nullptr:
// the root node, identity)
struct TNode {
  const TNode* parent;
  XformOp op;
};

class Parser {
 public:
  Parser(Tokenizer& tk, const std::string& base) : tk_(tk), base_(base) {}

  SceneModel parseScene() {  // Parser.cpp:26-95
    sc_.base_path = base_;
    tk_.read(SBT_RAYTRACER);
    Token ver = tk_.read(SCALAR);
    if (ver.value > 1.1) {
      std::ostringstream o;
      o << "Parser: fatal exception SBT-raytracer version number " << ver.value
        << " too high; only able to parse v1.1 and below.";
      throw ParseError(o.str());
    }
    Material mat;  // root material: Material() (Parser.cpp:39)
    for (;;) {
      switch (tk_.peek().kind) {
        case SPHERE: case BOX: case SQUARE: case CYLINDER: case CONE: case TRIMESH:
        case TRANSLATE: case ROTATE: case SCALE: case TRANSFORM: case LBRACE:
          parseTransformableElement(nullptr, mat);
          break;
        case POINT_LIGHT: sc_.lights.push_back(parsePointLight()); break;
        case DIRECTIONAL_LIGHT: sc_.lights.push_back(parseDirectionalLight()); break;
        case AREA_LIGHT_RECT: sc_.lights.push_back(parseAreaLightRect()); break;
        case AREA_LIGHT_CIRC: sc_.lights.push_back(parseAreaLightCirc()); break;
        case SPOT_LIGHT: sc_.lights.push_back(parseSpotLight()); break;
        case AMBIENT_LIGHT: parseAmbientLight(); break;
        case CAMERA: parseCamera(); break;
        case MATERIAL: mat = parseMaterialExpression(mat); break;
        case SEMICOLON: tk_.read(SEMICOLON); break;
        case EOFSYM: return std::move(sc_);
        default: tk_.syntax("Expected: geometry, camera, or light information");
      }
    }
  }

 private:
  // ------------------------------------------------------------ camera
  void parseCamera() {  // Parser.cpp:97-154
    bool hasViewDir = false, hasUpDir = false;
    dvec3 viewDir{0, 0, 0}, upDir{0, 0, 0};
    tk_.read(CAMERA);
    tk_.read(LBRACE);
    for (;;) {
      switch (tk_.peek().kind) {
        case POSITION: sc_.camera.eye = parseVec3dExpression(); break;
        case FOV: {
          CamOp op;
          op.kind = CAM_FOV;
          op.v[0] = parseScalarExpression();
          sc_.camera.ops.push_back(op);
          break;
        }
        case QUATERNIAN: {
          double q[4];
          parseVec4dExpression(q);
          CamOp op;
          op.kind = CAM_QUAT;
          for (int k = 0; k < 4; ++k) op.v[k] = q[k];
          sc_.camera.ops.push_back(op);
          break;
        }
        case ASPECTRATIO: {
          CamOp op;
          op.kind = CAM_ASPECT;
          op.v[0] = parseScalarExpression();
          sc_.camera.ops.push_back(op);
          break;
        }
        case VIEWDIR: viewDir = parseVec3dExpression(); hasViewDir = true; break;
        case UPDIR: upDir = parseVec3dExpression(); hasUpDir = true; break;
        case RBRACE:
          if (hasViewDir) {
            if (!hasUpDir) tk_.syntax("Expected: 'updir'");
            CamOp op;  // setLook(viewDir, upDir) at the block's end
            op.kind = CAM_LOOK;
            op.v[0] = viewDir.x; op.v[1] = viewDir.y; op.v[2] = viewDir.z;
            op.v[3] = upDir.x; op.v[4] = upDir.y; op.v[5] = upDir.z;
            sc_.camera.ops.push_back(op);
          } else if (hasUpDir) {
            tk_.syntax("Expected: 'viewdir'");
          }
          tk_.read(RBRACE);
          return;
        default: tk_.syntax("Expected: camera attribute");
      }
    }
  }

  // ------------------------------------------------------------ geometry
  void parseTransformableElement(const TNode* tf, const Material& mat) {
    switch (tk_.peek().kind) {
      case SPHERE: case BOX: case SQUARE: case CYLINDER: case CONE: case TRIMESH:
      case TRANSLATE: case ROTATE: case SCALE: case TRANSFORM:
        parseGeometry(tf, mat);
        break;
      case LBRACE: parseGroup(tf, mat); break;
      default: tk_.syntax("Expected: transformable element");
    }
  }

  void parseGroup(const TNode* tf, const Material& mat) {  // Parser.cpp:180-211
    tk_.read(LBRACE);
    for (;;) {
      switch (tk_.peek().kind) {
        case SPHERE: case BOX: case SQUARE: case CYLINDER: case CONE: case TRIMESH:
        case TRANSLATE: case ROTATE: case SCALE: case TRANSFORM: case LBRACE:
          parseTransformableElement(tf, mat);
          break;
        case RBRACE: tk_.read(RBRACE); return;
        case MATERIAL:
          // U19: the reference parses the material, then falls through into
          // the default branch and throws (Parser.cpp:202-208).
          parseMaterialExpression(mat);
          tk_.syntax("Expected: '}' or geometry");
        default: tk_.syntax("Expected: '}' or geometry");
      }
    }
  }

  void parseGeometry(const TNode* tf, const Material& mat) {
    switch (tk_.peek().kind) {
      case SPHERE: parseSimple(tf, mat, SPHERE, OBJ_SPHERE, "sphere"); return;
      case BOX: parseSimple(tf, mat, BOX, OBJ_BOX, "box"); return;
      case SQUARE: parseSimple(tf, mat, SQUARE, OBJ_SQUARE, "square"); return;
      case CYLINDER: parseSimple(tf, mat, CYLINDER, OBJ_CYLINDER, "cylinder"); return;
      case CONE: parseCone(tf, mat); return;
      case TRIMESH: parseTrimesh(tf, mat); return;
      case TRANSLATE: parseTranslate(tf, mat); return;
      case ROTATE: parseRotate(tf, mat); return;
      case SCALE: parseScale(tf, mat); return;
      case TRANSFORM: parseTransform(tf, mat); return;
      default: throw ParseError("Parser: fatal exception Unrecognized geometry type.");
    }
  }

  // Each transform node is created before the child is parsed and lives for
  // the whole parse (TransformNode::createChild, scene.h:85-90); a node
  // records its raw operation, an object the chain of operations from the
  // root (identity) down to it.
  const TNode* child(const TNode* parent, const XformOp& op) {
    nodes_.emplace_back(new TNode{parent, op});
    return nodes_.back().get();
  }
  const TNode* rootOr(const TNode* tf) { return tf; }  // nullptr = the root node
  static std::vector<XformOp> chain_of(const TNode* n) {
    std::vector<XformOp> c;
    for (; n; n = n->parent) c.push_back(n->op);
    return std::vector<XformOp>(c.rbegin(), c.rend());
  }
  static XformOp xop(int kind, std::initializer_list<double> v) {
    XformOp op;
    op.kind = kind;
    int k = 0;
    for (double x : v) op.v[k++] = x;
    return op;
  }

  void parseTranslate(const TNode* tf, const Material& mat) {
    tk_.read(TRANSLATE);
    tk_.read(LPAREN);
    double x = parseScalar(); tk_.read(COMMA);
    double y = parseScalar(); tk_.read(COMMA);
    double z = parseScalar(); tk_.read(COMMA);
    parseTransformableElement(child(rootOr(tf), xop(XF_TRANSLATE, {x, y, z})), mat);
    tk_.read(RPAREN);
    tk_.condRead(SEMICOLON);
  }

  void parseRotate(const TNode* tf, const Material& mat) {
    tk_.read(ROTATE);
    tk_.read(LPAREN);
    double x = parseScalar(); tk_.read(COMMA);
    double y = parseScalar(); tk_.read(COMMA);
    double z = parseScalar(); tk_.read(COMMA);
    double w = parseScalar(); tk_.read(COMMA);
    parseTransformableElement(child(rootOr(tf), xop(XF_ROTATE, {x, y, z, w})), mat);
    tk_.read(RPAREN);
    tk_.condRead(SEMICOLON);
  }

  void parseScale(const TNode* tf, const Material& mat) {
    tk_.read(SCALE);
    tk_.read(LPAREN);
    double x = parseScalar(), y, z;
    tk_.read(COMMA);
    if (tk_.peek().kind == SCALAR) {
      y = parseScalar(); tk_.read(COMMA);
      z = parseScalar(); tk_.read(COMMA);
    } else {
      y = x;
      z = x;
    }
    parseTransformableElement(child(rootOr(tf), xop(XF_SCALE, {x, y, z})), mat);
    tk_.read(RPAREN);
    tk_.condRead(SEMICOLON);
  }

  void parseTransform(const TNode* tf, const Material& mat) {
    tk_.read(TRANSFORM);
    tk_.read(LPAREN);
    double rows[4][4];
    for (int r = 0; r < 4; ++r) {
      parseVec4d(rows[r]);
      tk_.read(COMMA);
    }
    // the scene build applies glm::transpose(dmat4x4(row1..row4))
    XformOp op;
    op.kind = XF_MATRIX;
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c) op.v[r * 4 + c] = rows[r][c];
    parseTransformableElement(child(rootOr(tf), op), mat);
    tk_.read(RPAREN);
    tk_.condRead(SEMICOLON);
  }

  // sphere / box / square / cylinder (Parser.cpp:348-470)
  void parseSimple(const TNode* tf, const Material& mat, Sym kw, int type, const char* what) {
    tk_.read(kw);
    tk_.read(LBRACE);
    bool haveMat = false;
    Material newMat;
    for (;;) {
      switch (tk_.peek().kind) {
        case MATERIAL: newMat = parseMaterialExpression(mat); haveMat = true; break;
        case NAME: parseIdentExpression(); break;
        case RBRACE: {
          tk_.read(RBRACE);
          Object o;
          o.type = type;
          o.chain = chain_of(tf);
          addObject(o, haveMat ? newMat : mat);
          return;
        }
        default: tk_.syntax(std::string("Expected: ") + what + " attributes");
      }
    }
  }

  void parseCone(const TNode* tf, const Material& mat) {  // Parser.cpp:472-518
    tk_.read(CONE);
    tk_.read(LBRACE);
    bool haveMat = false;
    Material newMat;
    double bottomRadius = 1.0, topRadius = 0.0, height = 1.0;
    bool capped = true;  // capped by default
    for (;;) {
      switch (tk_.peek().kind) {
        case MATERIAL: newMat = parseMaterialExpression(mat); haveMat = true; break;
        case NAME: parseIdentExpression(); break;
        case CAPPED: capped = parseBooleanExpression(); break;
        case BOTTOM_RADIUS: bottomRadius = parseScalarExpression(); break;
        case TOP_RADIUS: topRadius = parseScalarExpression(); break;
        case HEIGHT: height = parseScalarExpression(); break;
        case RBRACE: {
          tk_.read(RBRACE);
          Object o;
          o.type = OBJ_CONE;
          o.chain = chain_of(tf);
          // Cone::Cone (Cone.h:11-37), same operations in the same order
          o.cone_h = height;
          o.cone_br = (bottomRadius < 0.0f) ? (-bottomRadius) : (bottomRadius);
          o.cone_tr = (topRadius < 0.0f) ? (-topRadius) : (topRadius);
          o.cone_capped = capped;
          if (o.cone_br < 0.0001) o.cone_br = 0.0001;
          if (o.cone_tr < 0.0001) o.cone_tr = 0.0001;
          double beta = (o.cone_tr - o.cone_br) / o.cone_h;
          if (std::fabs(beta) < 0.001) beta = 0.001;
          double gamma = beta < 0.0 ? o.cone_tr / beta : o.cone_br / beta;
          o.cone_b2 = beta * beta;
          if (gamma < 0.0) gamma = gamma - o.cone_h;
          o.cone_g = gamma;
          addObject(o, haveMat ? newMat : mat);
          return;
        }
        default: tk_.syntax("Expected: cone attributes");
      }
    }
  }

  // Scene::add (scene.cpp:133-138): the object and its material copy; the
  // world box is the scene build's (scene_build.cpp)
  void addObject(Object& o, const Material& m) {
    o.material = static_cast<int>(sc_.materials.size());
    sc_.materials.push_back(m);
    sc_.objects.push_back(o);
  }

  void parseTrimesh(const TNode* tf, const Material& mat) {  // Parser.cpp:520-653
    Material meshMat = mat;
    tk_.read(TRIMESH);
    tk_.read(LBRACE);
    bool genNormals = false;
    std::list<std::array<double, 3>> faces;
    Mesh me;
    std::vector<Material> vmats;
    for (;;) {
      switch (tk_.peek().kind) {
        case GENNORMALS: tk_.read(GENNORMALS); tk_.read(SEMICOLON); genNormals = true; break;
        case MATERIAL: meshMat = parseMaterialExpression(mat); break;
        case NAME: parseIdentExpression(); break;
        case MATERIALS:
          tk_.read(MATERIALS); tk_.read(EQUALS); tk_.read(LPAREN);
          if (tk_.peek().kind != RPAREN) {
            vmats.push_back(parseMaterial(meshMat));
            for (;;) {
              if (tk_.peek().kind == RPAREN) break;
              tk_.read(COMMA);
              vmats.push_back(parseMaterial(meshMat));
            }
          }
          tk_.read(RPAREN); tk_.read(SEMICOLON);
          break;
        case NORMALS:
          tk_.read(NORMALS); tk_.read(EQUALS); tk_.read(LPAREN);
          if (tk_.peek().kind != RPAREN) {
            me.raw_normals.push_back(parseVec3d());
            for (;;) {
              if (tk_.peek().kind == RPAREN) break;
              tk_.read(COMMA);
              me.raw_normals.push_back(parseVec3d());
            }
          }
          tk_.read(RPAREN); tk_.read(SEMICOLON);
          break;
        case FACES:
          tk_.read(FACES); tk_.read(EQUALS); tk_.read(LPAREN);
          if (tk_.peek().kind != RPAREN) {
            parseFaces(faces);
            for (;;) {
              if (tk_.peek().kind == RPAREN) break;
              tk_.read(COMMA);
              parseFaces(faces);
            }
          }
          tk_.read(RPAREN); tk_.read(SEMICOLON);
          break;
        case POLYPOINTS:
          tk_.read(POLYPOINTS); tk_.read(EQUALS); tk_.read(LPAREN);
          if (tk_.peek().kind != RPAREN) {
            me.verts.push_back(parseVec3d());
            for (;;) {
              if (tk_.peek().kind == RPAREN) break;
              tk_.read(COMMA);
              me.verts.push_back(parseVec3d());
            }
          }
          tk_.read(RPAREN); tk_.read(SEMICOLON);
          break;
        case RBRACE: {
          tk_.read(RBRACE);
          const int vcnt = static_cast<int>(me.verts.size());
          for (const auto& f : faces) {
            int a = static_cast<int>(f[0]), b = static_cast<int>(f[1]), c = static_cast<int>(f[2]);
            if (a >= vcnt || b >= vcnt || c >= vcnt || a < 0 || b < 0 || c < 0) {
              std::ostringstream o;
              o << "Parser: fatal exception Bad face in trimesh: (" << f[0] << ", " << f[1] << ", " << f[2] << ")";
              throw ParseError(o.str());
            }
            me.raw_faces.push_back({a, b, c});  // Trimesh::addFace drops degenerate ones (scene build)
          }
          me.gennormals = genNormals;
          // generateNormals resizes the normals to the vertex count first
          // (trimesh.cpp:192-217), so only a mesh without gennormals can
          // have the wrong number (Parser.cpp:640-651)
          if (!vmats.empty() && vmats.size() != me.verts.size())
            throw ParseError("Parser: fatal exception Bad Trimesh: Wrong number of materials.");
          if (!genNormals && !me.raw_normals.empty() && me.raw_normals.size() != me.verts.size())
            throw ParseError("Parser: fatal exception Bad Trimesh: Wrong number of normals.");
          me.vmats = vmats;
          Object o;
          o.type = OBJ_TRIMESH;
          o.chain = chain_of(tf);
          o.mesh = static_cast<int>(sc_.meshes.size());
          sc_.meshes.push_back(std::move(me));
          addObject(o, meshMat);
          return;
        }
        default: tk_.syntax("Expected: trimesh attributes");
      }
    }
  }

  void parseFaces(std::list<std::array<double, 3>>& faces) {  // Parser.cpp:655-671
    std::list<double> pts = parseScalarList();
    if (pts.size() < 3) tk_.syntax("Faces must have at least 3 vertices.");
    auto it = pts.begin();
    double a = *it++;
    double b = *it++;
    while (it != pts.end()) {
      double c = *it++;
      faces.push_back({a, b, c});
      b = c;
    }
  }

  // ------------------------------------------------------------ lights
  void parseAmbientLight() {
    tk_.read(AMBIENT_LIGHT);
    tk_.read(LBRACE);
    if (tk_.peek().kind != COLOR) tk_.syntax("Expected color attribute");
    sc_.ambient += parseVec3dExpression();
    tk_.read(RBRACE);
  }

  Light parsePointLight() {  // Parser.cpp:688-746
    Light L;
    L.type = L_POINT;
    float c = 0.0f, l = 0.0f, q = 1.0f;
    bool hasPos = false, hasCol = false;
    tk_.read(POINT_LIGHT);
    tk_.read(LBRACE);
    for (;;) {
      switch (tk_.peek().kind) {
        case POSITION:
          if (hasPos) tk_.syntax("Repeated 'position' attribute");
          L.pos = parseVec3dExpression(); hasPos = true; break;
        case COLOR:
          if (hasCol) tk_.syntax("Repeated 'color' attribute");
          L.color = parseVec3dExpression(); hasCol = true; break;
        case CONSTANT_ATTENUATION_COEFF: c = static_cast<float>(parseScalarExpression()); break;
        case LINEAR_ATTENUATION_COEFF: l = static_cast<float>(parseScalarExpression()); break;
        case QUADRATIC_ATTENUATION_COEFF: q = static_cast<float>(parseScalarExpression()); break;
        case RBRACE:
          if (!hasCol) tk_.syntax("Expected: 'color'");
          if (!hasPos) tk_.syntax("Expected: 'position'");
          tk_.read(RBRACE);
          L.c = c; L.l = l; L.q = q;
          return L;
        default:
          tk_.syntax("expecting 'position' or 'color' attribute, or 'constant_attenuation_coeff', "
                     "'linear_attenuation_coeff', or 'quadratic_attenuation_coeff'");
      }
    }
  }

  Light parseDirectionalLight() {  // Parser.cpp:748-787
    Light L;
    L.type = L_DIRECTIONAL;
    bool hasDir = false, hasCol = false;
    dvec3 dir{0, 0, 0};
    tk_.read(DIRECTIONAL_LIGHT);
    tk_.read(LBRACE);
    for (;;) {
      switch (tk_.peek().kind) {
        case DIRECTION:
          if (hasDir) tk_.syntax("Repeated 'direction' attribute");
          dir = parseVec3dExpression(); hasDir = true; break;
        case COLOR:
          if (hasCol) tk_.syntax("Repeated 'color' attribute");
          L.color = parseVec3dExpression(); hasCol = true; break;
        case RBRACE:
          if (!hasCol) tk_.syntax("Expected: 'color'");
          if (!hasDir) tk_.syntax("Expected: 'position'");
          tk_.read(RBRACE);
          L.raw_dir = dir;  // DirectionalLight ctor normalizes it (scene build)
          return L;
        default: tk_.syntax("expecting 'position' or 'color' attribute");
      }
    }
  }

  // Shared attribute loop for the area / spot lights (Parser.cpp:790-1058).
  Light parseAreaLike(Sym kw, int type) {
    Light L;
    L.type = type;
    float c = 0.0f, l = 0.0f, q = 1.0f;
    bool hasPos = false, hasCol = false, hasDir = false, hasRadius = false, hasAngle = false,
         hasW = false, hasH = false, hasUp = false;
    dvec3 dir{0, 0, 0}, up{0, 0, 0};
    tk_.read(kw);
    tk_.read(LBRACE);
    for (;;) {
      Sym k = tk_.peek().kind;
      switch (k) {
        case DIRECTION:
          if (hasDir) tk_.syntax("Repeated 'direction' attribute");
          dir = parseVec3dExpression(); hasDir = true; break;
        case POSITION:
          if (hasPos) tk_.syntax("Repeated 'position' attribute");
          L.pos = parseVec3dExpression(); hasPos = true; break;
        case COLOR:
          if (hasCol) tk_.syntax("Repeated 'color' attribute");
          L.color = parseVec3dExpression(); hasCol = true; break;
        case CONSTANT_ATTENUATION_COEFF: c = static_cast<float>(parseScalarExpression()); break;
        case LINEAR_ATTENUATION_COEFF: l = static_cast<float>(parseScalarExpression()); break;
        case QUADRATIC_ATTENUATION_COEFF: q = static_cast<float>(parseScalarExpression()); break;
        case RADIUS:
          if (type == L_AREA_RECT) goto bad;
          if (hasRadius) tk_.syntax("Repeated 'radius' attribute");
          L.radius = parseScalarExpression(); hasRadius = true; break;
        case ANGLE:
          if (type != L_SPOT) goto bad;
          if (hasAngle) tk_.syntax("Repeated 'angle' attribute");
          L.angle = parseScalarExpression(); hasAngle = true; break;
        case WIDTH:
          if (type != L_AREA_RECT) goto bad;
          if (hasW) tk_.syntax("Repeated 'width' attribute");
          L.width = parseScalarExpression(); hasW = true; break;
        case HEIGHT:
          if (type != L_AREA_RECT) goto bad;
          if (hasH) tk_.syntax("Repeated 'height' attribute");
          L.height = parseScalarExpression(); hasH = true; break;
        case UPDIR:
          if (type != L_AREA_RECT) goto bad;
          if (hasUp) tk_.syntax("Repeated 'updir' attribute");
          up = parseVec3dExpression(); hasUp = true; break;
        case RBRACE: {
          if (type == L_AREA_RECT) {
            if (!hasW) tk_.syntax("Expected: 'width'");
            if (!hasH) tk_.syntax("Expected: 'height'");
            if (!hasUp) tk_.syntax("Expected: 'updir'");
          }
          if (type == L_SPOT && !hasAngle) tk_.syntax("Expected: 'angle'");
          if (type != L_AREA_RECT && !hasRadius) tk_.syntax("Expected: 'radius'");
          if (!hasCol) tk_.syntax("Expected: 'color'");
          if (!hasPos) tk_.syntax("Expected: 'position'");
          if (!hasDir) tk_.syntax("Expected: 'direction'");
          tk_.read(RBRACE);
          L.c = c; L.l = l; L.q = q;
          L.raw_dir = dir;  // the light ctors' axes are the scene build's
          L.raw_up = up;
          return L;
        }
        default:
        bad:
          tk_.syntax("expecting 'position' or 'color' attribute, or 'constant_attenuation_coeff', "
                     "'linear_attenuation_coeff', or 'quadratic_attenuation_coeff'");
      }
    }
  }
  Light parseAreaLightRect() { return parseAreaLike(AREA_LIGHT_RECT, L_AREA_RECT); }
  Light parseAreaLightCirc() { return parseAreaLike(AREA_LIGHT_CIRC, L_AREA_CIRC); }
  Light parseSpotLight() { return parseAreaLike(SPOT_LIGHT, L_SPOT); }

  // ------------------------------------------------------------ values
  double parseScalarExpression() {
    tk_.get();
    tk_.read(EQUALS);
    double v = parseScalar();
    tk_.condRead(SEMICOLON);
    return v;
  }
  bool parseBooleanExpression() {
    tk_.get();
    tk_.read(EQUALS);
    Sym k = tk_.peek().kind;
    bool v;
    if (k == SYMTRUE) { tk_.read(SYMTRUE); v = true; }
    else if (k == SYMFALSE) { tk_.read(SYMFALSE); v = false; }
    else tk_.syntax("Expected boolean");
    tk_.condRead(SEMICOLON);
    return v;
  }
  dvec3 parseVec3dExpression() {
    tk_.get();
    tk_.read(EQUALS);
    dvec3 v = parseVec3d();
    tk_.condRead(SEMICOLON);
    return v;
  }
  void parseVec4dExpression(double out[4]) {
    tk_.get();
    tk_.read(EQUALS);
    parseVec4d(out);
    tk_.condRead(SEMICOLON);
  }
  std::string parseIdentExpression() {
    tk_.get();
    tk_.read(EQUALS);
    std::string s = tk_.read(IDENT).ident;
    tk_.condRead(SEMICOLON);
    return s;
  }
  double parseScalar() { return tk_.read(SCALAR).value; }
  std::list<double> parseScalarList() {
    std::list<double> r;
    tk_.read(LPAREN);
    if (tk_.peek().kind != RPAREN) {
      r.push_back(parseScalar());
      for (;;) {
        if (tk_.peek().kind == RPAREN) break;
        tk_.read(COMMA);
        r.push_back(parseScalar());
      }
    }
    tk_.read(RPAREN);
    return r;
  }
  dvec3 parseVec3d() {
    tk_.read(LPAREN);
    double a = tk_.read(SCALAR).value; tk_.read(COMMA);
    double b = tk_.read(SCALAR).value; tk_.read(COMMA);
    double c = tk_.read(SCALAR).value;
    tk_.read(RPAREN);
    return mk3(a, b, c);
  }
  void parseVec4d(double out[4]) {
    tk_.read(LPAREN);
    for (int i = 0; i < 4; ++i) {
      out[i] = tk_.read(SCALAR).value;
      if (i < 3) tk_.read(COMMA);
    }
    tk_.read(RPAREN);
  }

  // ------------------------------------------------------------ materials
  Material parseMaterialExpression(const Material& parent) {  // Parser.cpp:1095-1101
    tk_.read(MATERIAL);
    tk_.read(EQUALS);
    Material m = parseMaterial(parent);
    tk_.condRead(SEMICOLON);
    return m;
  }

  Material parseMaterial(const Material& parent) {  // Parser.cpp:1188-1274
    if (tk_.peek().kind == IDENT) {
      // U19: returns a copy of the named material WITHOUT consuming the
      // identifier; the caller then trips over it.
      auto it = named_.find(tk_.peek().ident);
      return it == named_.end() ? Material() : it->second;
    }
    tk_.read(LBRACE);
    Material m = parent;
    std::string name;
    for (;;) {
      switch (tk_.peek().kind) {
        case EMISSIVE: m.p[P_KE] = parseVec3Param(); break;
        case AMBIENT: m.p[P_KA] = parseVec3Param(); break;
        case SPECULAR: m.p[P_KS] = parseVec3Param(); break;          // no setBools (material.h:233)
        case DIFFUSE: m.p[P_KD] = parseVec3Param(); break;
        case REFLECTIVE: m.p[P_KR] = parseVec3Param(); m.setBools(); break;
        case TRANSMISSIVE: m.p[P_KT] = parseVec3Param(); m.setBools(); break;
        case INDEX: m.p[P_INDEX] = parseScalarParam(); break;
        case SHININESS: m.p[P_SHININESS] = parseScalarParam(); break;
        case GLOSS: m.p[P_GLOSS] = parseScalarParam(); break;
        case BUMP: m.p[P_BUMP] = parseVec3Param(); break;
        case NAME:
          tk_.read(NAME);
          name = tk_.read(IDENT).ident;
          tk_.read(SEMICOLON);
          break;
        case RBRACE:
          tk_.read(RBRACE);
          if (!name.empty()) {
            if (named_.find(name) == named_.end()) {
              named_[name] = m;
            } else {
              tk_.syntax("Redefinition of material '" + name + "'.");
            }
          }
          return m;
        default: tk_.syntax("Expected: material attribute");
      }
    }
  }

  MatParam parseVec3Param() {  // Parser.cpp:1276-1292
    tk_.get();
    tk_.read(EQUALS);
    MatParam q;
    if (tk_.condRead(MAP)) {
      tk_.read(LPAREN);
      std::string fn = base_ + "/" + tk_.read(IDENT).ident;
      tk_.read(RPAREN);
      tk_.condRead(SEMICOLON);
      q.tex = texture(fn);
    } else {
      q.v = parseVec3d();
      tk_.condRead(SEMICOLON);
    }
    return q;
  }

  MatParam parseScalarParam() {  // Parser.cpp:1294-1308 (no base path for maps)
    tk_.get();
    tk_.read(EQUALS);
    MatParam q;
    if (tk_.condRead(MAP)) {
      tk_.read(LPAREN);
      std::string fn = tk_.read(IDENT).ident;
      tk_.read(RPAREN);
      tk_.condRead(SEMICOLON);
      q.tex = texture(fn);
    } else {
      double s = parseScalar();
      q.v = mk3(s, s, s);
      tk_.condRead(SEMICOLON);
    }
    return q;
  }

  // Scene::getTexture cache + TextureMap ctor (scene.cpp:199-206, material.cpp:70-81)
  int texture(const std::string& fn) {
    auto it = tex_cache_.find(fn);
    if (it != tex_cache_.end()) return it->second;
    Texture t;
    t.path = fn;
    t.data = read_image(fn, t.width, t.height);
    if (t.data.empty())
      throw ParseError("Texture mapping exception: Unable to load texture map '" + fn + "'.");
    int id = static_cast<int>(sc_.textures.size());
    sc_.textures.push_back(std::move(t));
    tex_cache_[fn] = id;
    return id;
  }

  Tokenizer& tk_;
  std::string base_;
  SceneModel sc_;
  std::map<std::string, Material> named_;
  std::map<std::string, int> tex_cache_;
  std::vector<std::unique_ptr<TNode>> nodes_;
};

}  // namespace

SceneModel parse_ray_text(const std::string& text, const std::string& base_path) {
  Tokenizer tk(text);
  Parser p(tk, base_path);
  return p.parseScene();
}

namespace {
// A token's name as the reference prints it (Token::toString: getNameForToken,
// Token.cpp:27-107, which has no entry for fov / gennormals — those print the
// reserved word itself here).
const char* token_text(Sym s) {
  switch (s) {
    case IDENT: return "Identifier";
    case SCALAR: return "Scalar";
    case SYMTRUE: return "true";
    case SYMFALSE: return "false";
    case EOFSYM: case SBT_RAYTRACER: case LPAREN: case RPAREN: case LBRACE: case RBRACE: case COMMA: case EQUALS:
    case SEMICOLON: case MATERIAL:
      return sym_name(s);
    default: break;
  }
  static const std::map<Sym, std::string> canon = [] {
    std::map<Sym, std::string> m;
    for (const auto& kv : reserved())  // the reference's name: the canonical spelling of aliases
      if (!m.count(kv.second) || kv.first == "trimesh" || kv.first == "color") m[kv.second] = kv.first;
    return m;
  }();
  auto it = canon.find(s);
  return it == canon.end() ? "Unknown token type" : it->second.c_str();
}
}  // namespace

// The token stream of a .ray text, one token per line: its name, then a
// tab and the identifier or the scalar (%.17g) — Tokenizer(fp, printTokens)
// (Tokenizer.cpp:39-46, 119-123) made comparable; "ERROR" after the tokens
// read before a syntax error.
std::string dump_ray_tokens(const std::string& text) {
  std::ostringstream o;
  try {
    Tokenizer tk(text);
    for (;;) {
      const Token t = tk.get();
      o << token_text(t.kind);
      if (t.kind == IDENT) o << '\t' << t.ident;
      if (t.kind == SCALAR) {
        char b[40];
        std::snprintf(b, sizeof(b), "%.17g", t.value);
        o << '\t' << b;
      }
      o << '\n';
      if (t.kind == EOFSYM) break;
    }
  } catch (const ParseError&) {
    o << "ERROR\n";
  }
  return o.str();
}

SceneModel parse_ray_file_raw(const std::string& path) {  // RayTracer::loadScene's parse (RayTracer.cpp:196-240)
  std::ifstream ifs(path, std::ios::binary);
  if (!ifs) throw ParseError("Error: couldn't read scene file " + path);
  std::stringstream ss;
  ss << ifs.rdbuf();
  std::string base;
  size_t slash = path.find_last_of("\\/");
  base = (slash == std::string::npos) ? std::string(".") : path.substr(0, slash);
  return parse_ray_text(ss.str(), base);
}

// ---------------------------------------------------------------- cube map (-c)
bool load_cubemap(const std::string& one_cubemap_file, Texture faces[6], std::string& err) {
  // TraceUI.cc:87-94; note find_first_of: ANY character of "pos" / "neg"
  static const char* const matcher[6][2] = {{"pos", "x"}, {"neg", "x"}, {"pos", "y"},
                                            {"neg", "y"}, {"pos", "z"}, {"neg", "z"}};
  const std::string fN = one_cubemap_file;
  const std::string pdir = fN.substr(0, fN.find_last_of("/"));
  DIR* dp = opendir(pdir.data());
  if (dp == nullptr) {
    err = "Couldn't open the directory " + pdir;
    return false;
  }
  std::string matched_fn[6];
  int matched = 0;
  while (struct dirent* ep = readdir(dp)) {  // directory order, as the reference
    const std::string fn(ep->d_name);
    for (int i = 0; i < 6; i++) {
      const auto pos0 = fn.find_first_of(matcher[i][0]);
      if (pos0 == std::string::npos) continue;
      const auto pos1 = fn.find_first_of(matcher[i][1], pos0);
      if (pos1 == std::string::npos) continue;
      if (!matched_fn[i].empty()) {
        closedir(dp);
        err = std::string(matcher[i][0]) + matcher[i][1] + " matches " + matched_fn[i] + " and " + fn +
              ", stop smartload to avoid confliction";
        return false;
      }
      matched_fn[i] = fn;
      matched++;
      break;
    }
    if (matched == 6) break;
  }
  closedir(dp);
  if (matched != 6) {
    err = "Cannot locate all six cubemap files";
    return false;
  }
  for (int i = 0; i < 6; i++) {  // TextureMap ctor (material.cpp:70-81)
    const std::string path = pdir + "/" + matched_fn[i];
    Texture t;
    t.path = path;
    t.data = read_image(path, t.width, t.height);
    if (t.data.empty()) {
      err = "Unable to load texture map '" + path + "'.";
      return false;
    }
    faces[i] = std::move(t);
  }
  return true;
}

}  // namespace rtxh
