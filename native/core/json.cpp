#include "json.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace kgwe {

namespace {

const Json& null_json() {
  static const Json n;
  return n;
}

struct Parser {
  const char* p;
  const char* end;

  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json parse error: ") + what);
  }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r')) ++p;
  }
  bool lit(const char* s) {
    size_t n = std::strlen(s);
    if (static_cast<size_t>(end - p) >= n && std::memcmp(p, s, n) == 0) {
      p += n;
      return true;
    }
    return false;
  }
  static void utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out.push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
      out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }
  uint32_t hex4() {
    if (end - p < 4) fail("short \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex");
    }
    return v;
  }
  std::string string() {
    if (p >= end || *p != '"') fail("expected string");
    ++p;
    std::string out;
    while (p < end && *p != '"') {
      char c = *p++;
      if (c != '\\') {
        out.push_back(c);
        continue;
      }
      if (p >= end) fail("bad escape");
      char e = *p++;
      switch (e) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            p += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    if (p >= end) fail("unterminated string");
    ++p;
    return out;
  }
  Json value(int depth) {
    if (depth > 256) fail("nesting too deep");
    ws();
    if (p >= end) fail("unexpected end");
    char c = *p;
    if (c == '{') {
      ++p;
      Json::Object o;
      ws();
      if (p < end && *p == '}') {
        ++p;
        return Json(std::move(o));
      }
      for (;;) {
        ws();
        std::string k = string();
        ws();
        if (p >= end || *p != ':') fail("expected ':'");
        ++p;
        o[k] = value(depth + 1);
        ws();
        if (p < end && *p == ',') { ++p; continue; }
        if (p < end && *p == '}') { ++p; break; }
        fail("expected ',' or '}'");
      }
      return Json(std::move(o));
    }
    if (c == '[') {
      ++p;
      Json::Array a;
      ws();
      if (p < end && *p == ']') {
        ++p;
        return Json(std::move(a));
      }
      for (;;) {
        a.push_back(value(depth + 1));
        ws();
        if (p < end && *p == ',') { ++p; continue; }
        if (p < end && *p == ']') { ++p; break; }
        fail("expected ',' or ']'");
      }
      return Json(std::move(a));
    }
    if (c == '"') return Json(string());
    if (lit("true")) return Json(true);
    if (lit("false")) return Json(false);
    if (lit("null")) return Json();
    char* e = nullptr;
    double v = std::strtod(p, &e);
    if (e == p) fail("bad token");
    p = e;
    return Json(v);
  }
};

}  // namespace

Json Json::parse(const std::string& text) {
  Parser ps{text.data(), text.data() + text.size()};
  Json v = ps.value(0);
  ps.ws();
  if (ps.p != ps.end) ps.fail("trailing characters");
  return v;
}

const std::string& Json::as_string() const {
  if (!is_string()) throw std::runtime_error("json: not a string");
  return *s_;
}

const Json::Array& Json::items() const {
  static const Array empty;
  return is_array() ? *a_ : empty;
}

Json::Array& Json::items() {
  if (is_null()) *this = Json(Array{});
  if (!is_array()) throw std::runtime_error("json: not an array");
  own();
  return *a_;
}

const Json::Object& Json::fields() const {
  static const Object empty;
  return is_object() ? *o_ : empty;
}

Json::Object& Json::fields() {
  if (is_null()) *this = Json(Object{});
  if (!is_object()) throw std::runtime_error("json: not an object");
  own();
  return *o_;
}

const Json& Json::get(const std::string& key) const {
  if (!is_object()) return null_json();
  auto it = o_->find(key);
  return it == o_->end() ? null_json() : it->second;
}

bool Json::has(const std::string& key) const {
  return is_object() && o_->count(key) > 0;
}

Json& Json::operator[](const std::string& key) { return fields()[key]; }

size_t Json::size() const {
  if (is_array()) return a_->size();
  if (is_object()) return o_->size();
  return 0;
}

void Json::push_back(Json v) { items().push_back(std::move(v)); }

void Json::own() {
  if (a_ && a_.use_count() > 1) a_ = std::make_shared<Array>(*a_);
  if (o_ && o_.use_count() > 1) o_ = std::make_shared<Object>(*o_);
}

std::string json_escape(const std::string& s) {
  std::string out;
  out.reserve(s.size() + 2);
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          std::snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out.push_back(static_cast<char>(c));
        }
    }
  }
  return out;
}

void Json::dump_to(std::string& out) const {
  switch (type_) {
    case Type::Null: out += "null"; break;
    case Type::Bool: out += b_ ? "true" : "false"; break;
    case Type::Number: {
      if (!std::isfinite(n_)) {
        out += "null";
      } else if (n_ == std::floor(n_) && std::fabs(n_) < 9e15) {
        char buf[32];
        std::snprintf(buf, sizeof buf, "%lld", static_cast<long long>(n_));
        out += buf;
      } else {
        char buf[32];
        std::snprintf(buf, sizeof buf, "%.10g", n_);
        out += buf;
      }
      break;
    }
    case Type::String:
      out.push_back('"');
      out += json_escape(*s_);
      out.push_back('"');
      break;
    case Type::Array: {
      out.push_back('[');
      bool first = true;
      for (const auto& v : *a_) {
        if (!first) out.push_back(',');
        first = false;
        v.dump_to(out);
      }
      out.push_back(']');
      break;
    }
    case Type::Object: {
      out.push_back('{');
      bool first = true;
      for (const auto& kv : *o_) {
        if (!first) out.push_back(',');
        first = false;
        out.push_back('"');
        out += json_escape(kv.first);
        out += "\":";
        kv.second.dump_to(out);
      }
      out.push_back('}');
      break;
    }
  }
}

std::string Json::dump() const {
  std::string s;
  dump_to(s);
  return s;
}

}  // namespace kgwe
