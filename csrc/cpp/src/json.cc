// JSON parse / serialise (see include/json.h).
#include "json.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace triton { namespace client { namespace json {

void
AppendEscapedString(std::string* out, const std::string& s)
{
  out->push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out->append("\\\""); break;
      case '\\': out->append("\\\\"); break;
      case '\n': out->append("\\n"); break;
      case '\r': out->append("\\r"); break;
      case '\t': out->append("\\t"); break;
      case '\b': out->append("\\b"); break;
      case '\f': out->append("\\f"); break;
      default:
        if (c < 0x20) {
          char b[8];
          std::snprintf(b, sizeof(b), "\\u%04x", c);
          out->append(b);
        } else {
          out->push_back(static_cast<char>(c));
        }
    }
  }
  out->push_back('"');
}

void
Value::Write(std::string* out) const
{
  char buf[64];
  switch (type_) {
    case Type::Null: out->append("null"); break;
    case Type::Bool: out->append(b_ ? "true" : "false"); break;
    case Type::Int: out->append(std::to_string(i_)); break;
    case Type::UInt: out->append(std::to_string(u_)); break;
    case Type::Double:
      if (std::isnan(d_)) {
        out->append("NaN");
      } else if (std::isinf(d_)) {
        out->append(d_ > 0 ? "Infinity" : "-Infinity");
      } else {
        std::snprintf(buf, sizeof(buf), "%.17g", d_);
        out->append(buf);
        // keep it a JSON number that re-parses as floating point
        if (!std::strpbrk(buf, ".eE")) out->append(".0");
      }
      break;
    case Type::String: AppendEscapedString(out, s_); break;
    case Type::Array:
      out->push_back('[');
      for (size_t i = 0; i < arr_.size(); ++i) {
        if (i) out->push_back(',');
        arr_[i].Write(out);
      }
      out->push_back(']');
      break;
    case Type::Object:
      out->push_back('{');
      for (size_t i = 0; i < obj_.size(); ++i) {
        if (i) out->push_back(',');
        AppendEscapedString(out, obj_[i].first);
        out->push_back(':');
        obj_[i].second.Write(out);
      }
      out->push_back('}');
      break;
  }
}

std::string
Value::Serialize() const
{
  std::string s;
  Write(&s);
  return s;
}

namespace {

struct Parser {
  const char* p;
  const char* end;
  std::string* err;
  int depth = 0;

  bool fail(const char* m)
  {
    if (err) *err = m;
    return false;
  }
  void ws()
  {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  bool lit(const char* s)
  {
    size_t n = std::strlen(s);
    if (static_cast<size_t>(end - p) < n || std::memcmp(p, s, n) != 0) return false;
    p += n;
    return true;
  }
  static void utf8(std::string* out, uint32_t cp)
  {
    if (cp < 0x80) {
      out->push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
      out->push_back(static_cast<char>(0xC0 | (cp >> 6)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out->push_back(static_cast<char>(0xE0 | (cp >> 12)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      out->push_back(static_cast<char>(0xF0 | (cp >> 18)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }
  bool hex4(uint32_t* v)
  {
    if (end - p < 4) return false;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p++;
      r <<= 4;
      if (c >= '0' && c <= '9') r |= c - '0';
      else if (c >= 'a' && c <= 'f') r |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') r |= c - 'A' + 10;
      else return false;
    }
    *v = r;
    return true;
  }
  bool str(std::string* out)
  {
    if (p >= end || *p != '"') return fail("expected string");
    ++p;
    while (p < end) {
      char c = *p++;
      if (c == '"') return true;
      if (c != '\\') {
        out->push_back(c);
        continue;
      }
      if (p >= end) break;
      char e = *p++;
      switch (e) {
        case '"': out->push_back('"'); break;
        case '\\': out->push_back('\\'); break;
        case '/': out->push_back('/'); break;
        case 'b': out->push_back('\b'); break;
        case 'f': out->push_back('\f'); break;
        case 'n': out->push_back('\n'); break;
        case 'r': out->push_back('\r'); break;
        case 't': out->push_back('\t'); break;
        case 'u': {
          uint32_t cp;
          if (!hex4(&cp)) return fail("bad \\u escape");
          if (cp >= 0xD800 && cp <= 0xDBFF && end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            p += 2;
            uint32_t lo;
            if (!hex4(&lo)) return fail("bad surrogate");
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(out, cp);
          break;
        }
        default: return fail("bad escape");
      }
    }
    return fail("unterminated string");
  }
  bool num(Value* v)
  {
    const char* s = p;
    bool neg = false;
    if (p < end && *p == '-') {
      neg = true;
      ++p;
    }
    if (lit("Infinity")) {
      *v = Value(neg ? -INFINITY : INFINITY);
      return true;
    }
    bool is_float = false;
    while (p < end && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' || *p == '+' || *p == '-')) {
      if (*p == '.' || *p == 'e' || *p == 'E') is_float = true;
      ++p;
    }
    std::string t(s, p - s);
    if (t.empty() || t == "-") return fail("bad number");
    if (!is_float) {
      errno = 0;
      if (neg) {
        long long x = std::strtoll(t.c_str(), nullptr, 10);
        if (errno == 0) { *v = Value(static_cast<int64_t>(x)); return true; }
      } else {
        unsigned long long x = std::strtoull(t.c_str(), nullptr, 10);
        if (errno == 0) {
          if (x <= static_cast<unsigned long long>(INT64_MAX)) *v = Value(static_cast<int64_t>(x));
          else *v = Value(static_cast<uint64_t>(x));
          return true;
        }
      }
    }
    *v = Value(std::strtod(t.c_str(), nullptr));
    return true;
  }
  bool value(Value* v)
  {
    if (++depth > 512) return fail("nesting too deep");
    ws();
    if (p >= end) return fail("unexpected end");
    bool ok = true;
    char c = *p;
    if (c == '{') {
      ++p;
      *v = Value::Object();
      ws();
      if (p < end && *p == '}') {
        ++p;
      } else {
        while (true) {
          ws();
          std::string k;
          if (!str(&k)) return false;
          ws();
          if (p >= end || *p != ':') return fail("expected ':'");
          ++p;
          Value m;
          if (!value(&m)) return false;
          v->Set(k, std::move(m));
          ws();
          if (p < end && *p == ',') { ++p; continue; }
          if (p < end && *p == '}') { ++p; break; }
          return fail("expected ',' or '}'");
        }
      }
    } else if (c == '[') {
      ++p;
      *v = Value::Array();
      ws();
      if (p < end && *p == ']') {
        ++p;
      } else {
        while (true) {
          Value m;
          if (!value(&m)) return false;
          v->Append(std::move(m));
          ws();
          if (p < end && *p == ',') { ++p; continue; }
          if (p < end && *p == ']') { ++p; break; }
          return fail("expected ',' or ']'");
        }
      }
    } else if (c == '"') {
      std::string s;
      ok = str(&s);
      *v = Value(s);
    } else if (lit("true")) {
      *v = Value(true);
    } else if (lit("false")) {
      *v = Value(false);
    } else if (lit("null")) {
      *v = Value();
    } else if (lit("NaN")) {
      *v = Value(NAN);
    } else {
      ok = num(v);
    }
    --depth;
    return ok;
  }
};

}  // namespace

bool
Parse(const char* data, size_t len, Value* out, std::string* err)
{
  Parser ps{data, data + len, err};
  if (!ps.value(out)) return false;
  ps.ws();
  if (ps.p != ps.end) {
    if (err) *err = "trailing characters after JSON value";
    return false;
  }
  return true;
}

}}}  // namespace triton::client::json
